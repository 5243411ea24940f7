// FP6 (e2m3) operands for the per_token GEMM: (1) the bit layout of
// v_cvt_scalef32_2xpk16_fp6_f32, (2) v_mfma_scale_f32_16x16x128_f8f6f4 on e2m3 int4 codes
// against the exact integer product and against the same codes in e4m3, (3) the MFMA issue
// rate per operand format, measured by hand-written asm loops (rate_asm): fixed AGPR
// accumulators named literally, 16 independent-accumulator MFMAs per iteration and nothing
// else in the loop body but the scalar counter (no accumulator moves, no s_nop -- checked on
// the ISA by tests/test_probe_isa_cpu.py), one or two waves per SIMD (a dynamic LDS request
// keeps it to one workgroup per CU).
// hipcc --offload-arch=gfx950 -O3 tools/probes/fp6_mfma_probe.hip -o /tmp/fp6_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef int i4v __attribute__((ext_vector_type(4)));
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

// ---- issue-rate loops in asm.  16 MFMAs per iteration on the 8 accumulators a[0:3] ..
// a[28:31] (each written again 8 MFMAs later: no dependency stall at these latencies)
#define ACC_ZERO                                                                              \
  "v_accvgpr_write_b32 a0, 0\n v_accvgpr_write_b32 a1, 0\n v_accvgpr_write_b32 a2, 0\n"       \
  "v_accvgpr_write_b32 a3, 0\n v_accvgpr_write_b32 a4, 0\n v_accvgpr_write_b32 a5, 0\n"       \
  "v_accvgpr_write_b32 a6, 0\n v_accvgpr_write_b32 a7, 0\n v_accvgpr_write_b32 a8, 0\n"       \
  "v_accvgpr_write_b32 a9, 0\n v_accvgpr_write_b32 a10, 0\n v_accvgpr_write_b32 a11, 0\n"     \
  "v_accvgpr_write_b32 a12, 0\n v_accvgpr_write_b32 a13, 0\n v_accvgpr_write_b32 a14, 0\n"    \
  "v_accvgpr_write_b32 a15, 0\n v_accvgpr_write_b32 a16, 0\n v_accvgpr_write_b32 a17, 0\n"    \
  "v_accvgpr_write_b32 a18, 0\n v_accvgpr_write_b32 a19, 0\n v_accvgpr_write_b32 a20, 0\n"    \
  "v_accvgpr_write_b32 a21, 0\n v_accvgpr_write_b32 a22, 0\n v_accvgpr_write_b32 a23, 0\n"    \
  "v_accvgpr_write_b32 a24, 0\n v_accvgpr_write_b32 a25, 0\n v_accvgpr_write_b32 a26, 0\n"    \
  "v_accvgpr_write_b32 a27, 0\n v_accvgpr_write_b32 a28, 0\n v_accvgpr_write_b32 a29, 0\n"    \
  "v_accvgpr_write_b32 a30, 0\n v_accvgpr_write_b32 a31, 0\n"
#define SC_OP(ACC, F) "v_mfma_scale_f32_16x16x128_f8f6f4 " ACC ", %[a], %[b], " ACC ", %[s], %[s] op_sel_hi:[0,0,0]" F "\n"
#define SC8(F)                                                                                \
  SC_OP("a[0:3]", F) SC_OP("a[4:7]", F) SC_OP("a[8:11]", F) SC_OP("a[12:15]", F)              \
  SC_OP("a[16:19]", F) SC_OP("a[20:23]", F) SC_OP("a[24:27]", F) SC_OP("a[28:31]", F)
#define BF_OP(ACC) "v_mfma_f32_16x16x32_bf16 " ACC ", %[a], %[b], " ACC "\n"
#define BF8                                                                                   \
  BF_OP("a[0:3]") BF_OP("a[4:7]") BF_OP("a[8:11]") BF_OP("a[12:15]")                          \
  BF_OP("a[16:19]") BF_OP("a[20:23]") BF_OP("a[24:27]") BF_OP("a[28:31]")
#define LOOP_TAIL                                                                             \
  "s_sub_u32 %[n], %[n], 1\n s_cmp_lg_u32 %[n], 0\n s_cbranch_scc1 1b\n"                      \
  "s_nop 7\n s_nop 7\n v_accvgpr_read_b32 %[r], a0\n"
#define ACC_CLOBBERS                                                                          \
  "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13",     \
  "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26",  \
  "a27", "a28", "a29", "a30", "a31", "scc"

// FMT: 0 = e4m3 (8 operand dwords), 2 = e2m3 (6), 4 = e2m1 (4), -1 = bf16 16x16x32 (4)
template <int FMT>
__global__ __launch_bounds__(512) void rate_asm(float* out, int nit, int seed) {
  const int lane = threadIdx.x & 63;
  const int sc = 127;  // E8M0 scale 1.0
  float r = 0.f;
  int n = nit;
  if constexpr (FMT == 0) {
    i8v a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (lane * 7 + i * 13 + seed) & 0x0F0F0F0F; b[i] = (lane * 5 + i * 11) & 0x0F0F0F0F; }
    asm volatile(ACC_ZERO "1:\n" SC8("") SC8("") LOOP_TAIL
                 : [r] "=v"(r), [n] "+s"(n) : [a] "v"(a), [b] "v"(b), [s] "v"(sc) : ACC_CLOBBERS);
  } else if constexpr (FMT == 2) {
    i6v a, b;
    for (int i = 0; i < 6; ++i) { a[i] = (lane * 7 + i * 13 + seed) & 0x0F0F0F0F; b[i] = (lane * 5 + i * 11) & 0x0F0F0F0F; }
    asm volatile(ACC_ZERO "1:\n" SC8(" cbsz:2 blgp:2") SC8(" cbsz:2 blgp:2") LOOP_TAIL
                 : [r] "=v"(r), [n] "+s"(n) : [a] "v"(a), [b] "v"(b), [s] "v"(sc) : ACC_CLOBBERS);
  } else if constexpr (FMT == 4) {
    i4v a, b;
    for (int i = 0; i < 4; ++i) { a[i] = (lane * 7 + i * 13 + seed) & 0x07070707; b[i] = (lane * 5 + i * 11) & 0x07070707; }
    asm volatile(ACC_ZERO "1:\n" SC8(" cbsz:4 blgp:4") SC8(" cbsz:4 blgp:4") LOOP_TAIL
                 : [r] "=v"(r), [n] "+s"(n) : [a] "v"(a), [b] "v"(b), [s] "v"(sc) : ACC_CLOBBERS);
  } else {
    i4v a, b;
    for (int i = 0; i < 4; ++i) { a[i] = (lane * 7 + i * 13 + seed) & 0x3F003F00; b[i] = (lane * 5 + i * 11) & 0x3F003F00; }
    asm volatile(ACC_ZERO "1:\n" BF8 BF8 LOOP_TAIL
                 : [r] "=v"(r), [n] "+s"(n) : [a] "v"(a), [b] "v"(b) : ACC_CLOBBERS);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static unsigned e2m3(int c) {  // host reference encoding of an integer |c| <= 7
  const unsigned s = c < 0 ? 0x20u : 0u;
  const int m = c < 0 ? -c : c;
  static const unsigned t[8] = {0x00, 0x08, 0x10, 0x14, 0x18, 0x1A, 0x1C, 0x1E};
  return s | t[m];
}

template <int FMT>
static int time_rate(int cu, int threads, float* dr, const char* name, double flop_per_mfma) {
  const int nit = 8192;
  const size_t lds = 96 * 1024;  // one workgroup per CU (160 KiB of LDS)
  CK(hipFuncSetAttribute((const void*)rate_asm<FMT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  rate_asm<FMT><<<cu, threads, lds>>>(dr, 64, 1);  // warm-up (clocks, code)
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    rate_asm<FMT><<<cu, threads, lds>>>(dr, nit, 1);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double waves = (double)cu * threads / 64;
  const double flop = flop_per_mfma * 16.0 * nit * waves;
  printf("rate %-14s %d wave(s)/SIMD: %.3f ms, %7.1f TFLOP/s (%d CUs)\n", name, threads / 256, best,
         flop / best / 1e9, cu);
  return 0;
}

int main() {
  // (1) layout: the two 16-float sources interleave -- element 2i = a[i], 2i + 1 = b[i] --
  // each at bits [6 e, 6 e + 6) of the 192-bit result
  std::vector<float> in(32);
  for (int i = 0; i < 32; ++i) in[i] = (float)((i % 15) - 7);
  float* din; int* dout;
  CK(hipMalloc(&din, 32 * 4)); CK(hipMalloc(&dout, 6 * 4));
  CK(hipMemcpy(din, in.data(), 32 * 4, hipMemcpyHostToDevice));
  pack_probe<<<1, 64>>>(din, dout);
  CK(hipDeviceSynchronize());
  unsigned w[6];
  CK(hipMemcpy(w, dout, 24, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int e = 0; e < 32; ++e) {
    const int bit = 6 * e, wd = bit / 32, sh = bit % 32;
    unsigned long long v = w[wd];
    if (wd < 5) v |= (unsigned long long)w[wd + 1] << 32;
    const unsigned got = (unsigned)(v >> sh) & 0x3Fu;
    const int src = (e & 1) ? 16 + e / 2 : e / 2;  // a[e / 2] or b[e / 2]
    if (got != e2m3((src % 15) - 7)) ++bad;
  }
  printf("pack layout: element 2i = src0[i], 2i+1 = src1[i] at bits [6e, 6e+6): %s (%d mismatches); "
         "words %08x %08x %08x %08x %08x %08x\n", bad ? "NO" : "yes", bad, w[0], w[1], w[2], w[3], w[4], w[5]);
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
      const int row = 4 * (l >> 4) + r, col = l & 15;
      long ref_ab = 0, ref_ba = 0;
      for (int k = 0; k < 128; ++k) { ref_ab += (long)A[col * 128 + k] * B[row * 128 + k]; ref_ba += (long)A[row * 128 + k] * B[col * 128 + k]; }
      same += h6[l * 4 + r] == h8[l * 4 + r];
      exact += (h6[l * 4 + r] == (float)ref_ab) || (h6[l * 4 + r] == (float)ref_ba);
    }
  printf("16x16x128 e2m3 vs e4m3 results equal: %d / 256; equal to the integer product: %d / 256\n", same, exact);
  // (3) rates
  int dev = 0, cu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev));
  float* dr;
  CK(hipMalloc(&dr, (size_t)cu * 512 * 4));
  const double sc = 2.0 * 16 * 16 * 128, bf = 2.0 * 16 * 16 * 32;
  for (int threads : {256, 512}) {
    if (time_rate<-1>(cu, threads, dr, "bf16 16x16x32", bf)) return 1;
    if (time_rate<0>(cu, threads, dr, "e4m3 (fp8)", sc)) return 1;
    if (time_rate<2>(cu, threads, dr, "e2m3 (fp6)", sc)) return 1;
    if (time_rate<4>(cu, threads, dr, "e2m1 (fp4)", sc)) return 1;
  }
  return 0;
}
