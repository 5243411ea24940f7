#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
// A/B: per lane 32 bytes (fp8 e4m3); out: per lane 16 floats
__global__ void probe(const int* a, const int* b, float* c, const int* a6, const int* b6, float* c6) {
  const int l = threadIdx.x;
  v8i av, bv, av6, bv6;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[l * 8 + i]; bv[i] = b[l * 8 + i]; av6[i] = a6[l * 8 + i]; bv6[i] = b6[l * 8 + i];
  }
  v16f acc = {}, acc6 = {};
  // fmt 0 = fp8 e4m3, 2 = fp6 e2m3 for A and B; scale = 127 (E8M0 1.0)
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 0, 0, 0, 127, 0, 127);
  acc6 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av6, bv6, acc6, 2, 2, 0, 127, 0, 127);
  for (int i = 0; i < 16; ++i) { c[l * 16 + i] = acc[i]; c6[l * 16 + i] = acc6[i]; }
}
int main() {
  // e4m3 encoding of small ints
  auto enc = [](int v) -> unsigned char {
    if (v == 0) return 0;
    unsigned char s = v < 0 ? 0x80 : 0; int a = v < 0 ? -v : v;
    int e = 0; while ((a >> (e + 1)) > 0) ++e;   // 2^e <= a
    int m = ((a << 3) >> e) & 7;                  // 3 mantissa bits (exact for a < 16)
    return s | ((e + 7) << 3) | m;
  };
  const int n = 64 * 32;
  unsigned char ha[n], hb[n];
  int va[n], vb[n];
  srand(1);
  for (int i = 0; i < n; ++i) { va[i] = rand() % 15 - 7; vb[i] = rand() % 15 - 7; ha[i] = enc(va[i]); hb[i] = enc(vb[i]); }
  // fp6 e2m3, 32 values per lane packed as contiguous 6-bit fields (hypothesis), 8 dwords
  auto enc6 = [](int v) -> unsigned {
    static const unsigned t[8] = {0, 8, 16, 20, 24, 26, 28, 30};
    return (v < 0 ? 32u : 0u) | t[v < 0 ? -v : v];
  };
  static unsigned a6[64 * 8], b6[64 * 8];
  for (int l = 0; l < 64; ++l)
    for (int e = 0; e < 32; ++e) {
      const int bit = 6 * e;
      const unsigned xa = enc6(va[l * 32 + e]), xb = enc6(vb[l * 32 + e]);
      a6[l * 8 + bit / 32] |= xa << (bit % 32);
      b6[l * 8 + bit / 32] |= xb << (bit % 32);
      if (bit % 32 > 26) { a6[l * 8 + bit / 32 + 1] |= xa >> (32 - bit % 32); b6[l * 8 + bit / 32 + 1] |= xb >> (32 - bit % 32); }
    }
  int *da, *db, *da6, *db6; float *dc, *dc6;
  hipMalloc(&da, n); hipMalloc(&db, n); hipMalloc(&dc, 64 * 16 * 4);
  hipMalloc(&da6, sizeof(a6)); hipMalloc(&db6, sizeof(b6)); hipMalloc(&dc6, 64 * 16 * 4);
  hipMemcpy(da, ha, n, hipMemcpyHostToDevice); hipMemcpy(db, hb, n, hipMemcpyHostToDevice);
  hipMemcpy(da6, a6, sizeof(a6), hipMemcpyHostToDevice); hipMemcpy(db6, b6, sizeof(b6), hipMemcpyHostToDevice);
  probe<<<1, 64>>>(da, db, dc, da6, db6, dc6);
  float hc[64 * 16], hc6[64 * 16];
  hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  hipMemcpy(hc6, dc6, sizeof(hc6), hipMemcpyDeviceToHost);
  FILE* f = fopen("gpurun_out/probe.txt", "w");
  for (int i = 0; i < n; ++i) fprintf(f, "%d ", va[i]); fprintf(f, "\n");
  for (int i = 0; i < n; ++i) fprintf(f, "%d ", vb[i]); fprintf(f, "\n");
  for (int i = 0; i < 64 * 16; ++i) fprintf(f, "%g ", hc[i]); fprintf(f, "\n");
  for (int i = 0; i < 64 * 16; ++i) fprintf(f, "%g ", hc6[i]); fprintf(f, "\n");
  fclose(f);
  printf("done\n");
  return 0;
}
