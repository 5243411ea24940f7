// FP6 (e2m3) operands for the per_token GEMM: (1) the bit layout of
// v_cvt_scalef32_2xpk16_fp6_f32, (2) v_mfma_scale_f32_16x16x128_f8f6f4 on e2m3 int4 codes
// against the exact integer product and against the same codes in e4m3, (3) the MFMA issue
// rate of e2m3 vs e4m3 operands (independent accumulators, one workgroup per CU).
// hipcc --offload-arch=gfx950 -O3 tools/probes/fp6_mfma_probe.hip -o /tmp/fp6_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef int i6v __attribute__((ext_vector_type(6)));
typedef int i8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void pack_probe(const float* in, int* out) {
  f16v a, b;
  for (int i = 0; i < 16; ++i) { a[i] = in[i]; b[i] = in[16 + i]; }
  const i6v r = __builtin_amdgcn_cvt_scalef32_2xpk16_fp6_f32(a, b, 1.0f);
  if (threadIdx.x == 0)
    for (int i = 0; i < 6; ++i) out[i] = r[i];
}

// e4m3 bytes of 4 floats
__device__ inline int f8x4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}

// one wave: A [16][128], B [16][128] int codes; lane (r16, q) holds row r16, k 32q .. 32q + 31
__global__ void mfma_probe(const int* A, const int* B, float* d6, float* d8) {
  const int lane = threadIdx.x, r16 = lane & 15, q = lane >> 4;
  f16v a0, a1, b0, b1;
  for (int i = 0; i < 16; ++i) {
    a0[i] = (float)A[r16 * 128 + 32 * q + i];
    a1[i] = (float)A[r16 * 128 + 32 * q + 16 + i];
    b0[i] = (float)B[r16 * 128 + 32 * q + i];
    b1[i] = (float)B[r16 * 128 + 32 * q + 16 + i];
  }
  const i6v pa = __builtin_amdgcn_cvt_scalef32_2xpk16_fp6_f32(a0, a1, 1.0f);
  const i6v pb = __builtin_amdgcn_cvt_scalef32_2xpk16_fp6_f32(b0, b1, 1.0f);
  i8v xa = {pa[0], pa[1], pa[2], pa[3], pa[4], pa[5], 0, 0};
  i8v xb = {pb[0], pb[1], pb[2], pb[3], pb[4], pb[5], 0, 0};
  f4v z = {0.f, 0.f, 0.f, 0.f};
  f4v r6 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(xa, xb, z, 2, 2, 0, 127, 0, 127);
  i8v ya, yb;
  for (int d = 0; d < 4; ++d) {
    ya[d] = f8x4(a0[4 * d], a0[4 * d + 1], a0[4 * d + 2], a0[4 * d + 3]);
    ya[4 + d] = f8x4(a1[4 * d], a1[4 * d + 1], a1[4 * d + 2], a1[4 * d + 3]);
    yb[d] = f8x4(b0[4 * d], b0[4 * d + 1], b0[4 * d + 2], b0[4 * d + 3]);
    yb[4 + d] = f8x4(b1[4 * d], b1[4 * d + 1], b1[4 * d + 2], b1[4 * d + 3]);
  }
  f4v r8 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ya, yb, z, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) {
    d6[lane * 4 + r] = r6[r];
    d8[lane * 4 + r] = r8[r];
  }
}

// issue-rate loop: 8 independent accumulators, NIT iterations
template <int FMT>
__global__ __launch_bounds__(256) void rate_probe(float* out, int nit, int seed) {
  const int lane = threadIdx.x & 63;
  i8v a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (lane * 7 + i * 13 + seed) & 0x0F0F0F0F; b[i] = (lane * 5 + i * 11) & 0x0F0F0F0F; }
  f4v acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = f4v{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < nit; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], FMT, FMT, 0, 127, 0, 127);
  }
  float s = 0.f;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

static unsigned e2m3(int c) {  // host reference encoding of an integer |c| <= 7
  const unsigned s = c < 0 ? 0x20u : 0u;
  const int m = c < 0 ? -c : c;
  static const unsigned t[8] = {0x00, 0x08, 0x10, 0x14, 0x18, 0x1A, 0x1C, 0x1E};
  return s | t[m];
}

int main() {
  // (1) layout
  std::vector<float> in(32);
  for (int i = 0; i < 32; ++i) in[i] = (float)((i % 15) - 7);
  float* din; int* dout;
  CK(hipMalloc(&din, 32 * 4)); CK(hipMalloc(&dout, 6 * 4));
  CK(hipMemcpy(din, in.data(), 32 * 4, hipMemcpyHostToDevice));
  pack_probe<<<1, 64>>>(din, dout);
  CK(hipDeviceSynchronize());
  int w[6];
  CK(hipMemcpy(w, dout, 24, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 32; ++i) {
    const int bit = 6 * i;
    unsigned long long v = ((unsigned long long)(unsigned)w[bit / 32 + (bit / 32 < 5 ? 1 : 0)] << 32) | (unsigned)w[bit / 32];
    const unsigned got = (unsigned)(v >> (bit % 32)) & 0x3Fu;
    if (got != e2m3((i % 15) - 7)) ++bad;
  }
  printf("pack layout: element i at bits [6i, 6i+6), e2m3: %s (%d mismatches); words %08x %08x %08x %08x %08x %08x\n",
         bad ? "NO" : "yes", bad, w[0], w[1], w[2], w[3], w[4], w[5]);
  // (2) exactness
  std::vector<int> A(16 * 128), B(16 * 128);
  srand(5);
  for (auto& v : A) v = rand() % 15 - 7;
  for (auto& v : B) v = rand() % 15 - 7;
  int *dA, *dB; float *d6, *d8;
  CK(hipMalloc(&dA, A.size() * 4)); CK(hipMalloc(&dB, B.size() * 4));
  CK(hipMalloc(&d6, 256 * 4)); CK(hipMalloc(&d8, 256 * 4));
  CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  mfma_probe<<<1, 64>>>(dA, dB, d6, d8);
  CK(hipDeviceSynchronize());
  std::vector<float> h6(256), h8(256);
  CK(hipMemcpy(h6.data(), d6, 1024, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h8.data(), d8, 1024, hipMemcpyDeviceToHost));
  int same = 0, exact = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * (l >> 4) + r, col = l & 15;  // D[row][col]: A supplies row? check both
      long ref_ab = 0, ref_ba = 0;
      for (int k = 0; k < 128; ++k) { ref_ab += (long)A[col * 128 + k] * B[row * 128 + k]; ref_ba += (long)A[row * 128 + k] * B[col * 128 + k]; }
      same += h6[l * 4 + r] == h8[l * 4 + r];
      exact += (h6[l * 4 + r] == (float)ref_ab) || (h6[l * 4 + r] == (float)ref_ba);
    }
  printf("16x16x128 e2m3 vs e4m3 results equal: %d / 256; equal to the integer product: %d / 256\n", same, exact);
  // (3) rate
  int dev = 0, cu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev));
  float* dr;
  CK(hipMalloc(&dr, (size_t)cu * 4 * 256 * 4));
  const int nit = 4096;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int fmt : {0, 2, 0, 2}) {
    CK(hipEventRecord(e0));
    if (fmt == 0) rate_probe<0><<<cu * 4, 256>>>(dr, nit, 1); else rate_probe<2><<<cu * 4, 256>>>(dr, nit, 1);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double flop = 2.0 * 16 * 16 * 128 * 8.0 * nit * (cu * 4 * 4);
    printf("rate %s: %.3f ms, %.1f TFLOP/s (%d CUs, 16 waves per CU)\n", fmt ? "e2m3 (fp6)" : "e4m3 (fp8)", ms, flop / ms / 1e9, cu);
  }
  return 0;
}
