// Probe: the two rates gemm_f6_kernel overlaps, at BASELINE config 2 (M = 16384,
// K = N = 4096, S_pad = 256, G = 128): the full kernel, DMA + barriers only (PROBE 1) and
// compute + barriers only (PROBE 2).  Operand bytes are arbitrary (timing only).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I smoothquant-mixedprecision_amd/csrc \
//     tools/probe/f6_rate_probe.hip -o tools/probe/f6_rate_probe
#include "../../smoothquant-mixedprecision_amd/csrc/sqmp_gemm_f8.hip"

#include <stdio.h>

template <int P>
static float time_it(int iters, const unsigned char* a6, const float* sa, const _Float16* xs,
                     const unsigned char* w6, const float* ws, const _Float16* wsal,
                     _Float16* y, int M, int N, int Kp, int S_pad) {
  const int tm = cdiv(M, 256), tn = cdiv(N, 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w)
    gemm_f6_kernel<F16, P><<<tm * tn, 512>>>(a6, sa, xs, w6, ws, wsal, nullptr, y, M, N, Kp,
                                             S_pad, 128, Kp / 128, tm, tn, 4);
  hipEventRecord(e0);
  for (int i = 0; i < iters; ++i)
    gemm_f6_kernel<F16, P><<<tm * tn, 512>>>(a6, sa, xs, w6, ws, wsal, nullptr, y, M, N, Kp,
                                             S_pad, 128, Kp / 128, tm, tn, 4);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / iters;
}

int main(int argc, char** argv) {
  const int M = 16384, N = 4096, Kp = 4096;
  const int S_pad = argc > 1 ? atoi(argv[1]) : 256;
  unsigned char *a6, *w6;
  float *sa, *ws;
  _Float16 *xs, *wsal, *y;
  hipMalloc(&a6, (size_t)M * Kp * 3 / 4);
  hipMalloc(&w6, (size_t)N * Kp * 3 / 4);
  hipMalloc(&sa, (size_t)M * 4);
  hipMalloc(&ws, (size_t)(Kp / 128) * N * 4);
  hipMalloc(&xs, (size_t)M * (S_pad > 8 ? S_pad : 8) * 2);
  hipMalloc(&wsal, (size_t)N * (S_pad > 8 ? S_pad : 8) * 2);
  hipMalloc(&y, (size_t)M * N * 2);
  hipMemset(a6, 0x11, (size_t)M * Kp * 3 / 4);
  hipMemset(w6, 0x11, (size_t)N * Kp * 3 / 4);
  hipMemset(sa, 0, (size_t)M * 4);
  hipMemset(ws, 0, (size_t)(Kp / 128) * N * 4);
  hipMemset(xs, 0, (size_t)M * (S_pad > 8 ? S_pad : 8) * 2);
  hipMemset(wsal, 0, (size_t)N * (S_pad > 8 ? S_pad : 8) * 2);
  const double flop = 2.0 * M * N * (double)(Kp + S_pad);
  const float t0 = time_it<0>(200, a6, sa, xs, w6, ws, wsal, y, M, N, Kp, S_pad);
  const float t1 = time_it<1>(200, a6, sa, xs, w6, ws, wsal, y, M, N, Kp, S_pad);
  const float t2 = time_it<2>(200, a6, sa, xs, w6, ws, wsal, y, M, N, Kp, S_pad);
  printf("S_pad %d  full %.4f ms (%.0f TFLOP/s)  dma-only %.4f ms  compute-only %.4f ms\n",
         S_pad, t0, flop / t0 / 1e9, t1, t2);
  return hipDeviceSynchronize() != hipSuccess;
}
