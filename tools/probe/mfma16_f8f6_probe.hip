// Probe: operand lane maps of v_mfma_scale_f32_16x16x128_f8f6f4 on gfx950 (fp8 e4m3 and
// fp6 e2m3), checked on the host against candidate maps with exact integer data.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/mfma16_f8f6_probe.hip -o /tmp/mfma16_probe
// Candidate A map: lane l (r = l & 15, q = l >> 4) holds A[row r][k = kmap(q, e)], e = 0..31;
// B likewise with column r; D: col = l & 15, row = 4 q + i.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void probe(const int* a, const int* b, float* c, int fmt) {
  const int l = threadIdx.x;
  v8i av, bv;
  for (int i = 0; i < 8; ++i) { av[i] = a[l * 8 + i]; bv[i] = b[l * 8 + i]; }
  v4f acc = {};
  if (fmt == 0)
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, 127, 0, 127);
  else
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 2, 2, 0, 127, 0, 127);
  for (int i = 0; i < 4; ++i) c[l * 4 + i] = acc[i];
}

static unsigned char enc8(int v) {
  if (v == 0) return 0;
  unsigned char s = v < 0 ? 0x80 : 0; int a = v < 0 ? -v : v;
  int e = 0; while ((a >> (e + 1)) > 0) ++e;
  int m = ((a << 3) >> e) & 7;
  return s | ((e + 7) << 3) | m;
}
static unsigned enc6(int v) {
  static const unsigned t[8] = {0, 8, 16, 20, 24, 26, 28, 30};
  return (v < 0 ? 32u : 0u) | t[v < 0 ? -v : v];
}
static int kmap(int hyp, int q, int e) {
  switch (hyp) {
    case 0: return 32 * q + e;                               // contiguous 32 per lane group
    case 1: return (e < 16) ? 16 * q + e : 64 + 16 * q + e - 16;  // two 16-runs
    case 2: return 8 * q + (e & 7) + 32 * (e >> 3);           // 8-runs interleaved
    default: return (e < 8) ? 8 * q + e : 32 + (((e - 8) / 8) * 32) + 8 * q + (e & 7);
  }
}

int main() {
  int A[16][128], B[128][16];
  srand(3);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 128; ++k) A[i][k] = rand() % 15 - 7;
  for (int k = 0; k < 128; ++k) for (int j = 0; j < 16; ++j) B[k][j] = rand() % 15 - 7;
  double ref[16][16];
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    double s = 0; for (int k = 0; k < 128; ++k) s += A[i][k] * B[k][j]; ref[i][j] = s;
  }
  int *da, *db; float* dc;
  hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dc, 64 * 16);
  for (int fmt = 0; fmt < 2; ++fmt)
    for (int hyp = 0; hyp < 4; ++hyp) {
      unsigned ha[64 * 8], hb[64 * 8];
      memset(ha, 0, sizeof(ha)); memset(hb, 0, sizeof(hb));
      for (int l = 0; l < 64; ++l) {
        const int r = l & 15, q = l >> 4;
        for (int e = 0; e < 32; ++e) {
          const int k = kmap(hyp, q, e);
          if (fmt == 0) {
            ((unsigned char*)ha)[l * 32 + e] = enc8(A[r][k]);
            ((unsigned char*)hb)[l * 32 + e] = enc8(B[k][r]);
          } else {
            const int bit = 6 * e;
            const unsigned xa = enc6(A[r][k]), xb = enc6(B[k][r]);
            ha[l * 8 + bit / 32] |= xa << (bit % 32);
            hb[l * 8 + bit / 32] |= xb << (bit % 32);
            if (bit % 32 > 26) { ha[l * 8 + bit / 32 + 1] |= xa >> (32 - bit % 32); hb[l * 8 + bit / 32 + 1] |= xb >> (32 - bit % 32); }
          }
        }
      }
      hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
      hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
      probe<<<1, 64>>>(da, db, dc, fmt);
      float hc[64 * 4];
      hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
      int bad = 0;
      for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) bad += hc[l * 4 + i] != (float)ref[4 * (l >> 4) + i][l & 15];
      printf("fmt %s hyp %d: %d of 256 outputs differ\n", fmt ? "fp6" : "fp8", hyp, bad);
    }
  return 0;
}
