// Sibling operand reuse: the faithful GEMM operand of one layer rebuilt from a sibling's.
//
// Layers that quantize the SAME input with the same salient set and the same act mode (q/k/v,
// gate/up: their importance vectors come from the same calibration input, fake_quant.py
// :464-560) get identical x_hat values (fake_quant.py:291-304 depends only on x, the salient
// set and the act mode); only the packed K order differs, because every weight is packed in
// its own weight-sorted order (:157-207).  So the second sibling's operand
//   A_dst[m][p] = x_hat[m][perm_dst[p]]  (0 at its salient / padding positions), then the tail
// is the first one's with its positions permuted: A_dst[m][p] = A_src[m][map[p]] (map[p] < 0:
// 0) for p < P, and the exact salient tail A_src[m][P + j] unchanged (same salient order) --
// a pure data movement, bit-exact, instead of a second table build + quantizer pass.
//
// One workgroup = 256 threads, a run of row pairs.  Per pair: both rows into LDS INTERLEAVED
// (word k = (src[m][k], src[m+1][k]), the quantizer's layout), one barrier, then each thread
// assembles 16-B output chunks from its cached map entries (one ds_read_b32 carries both
// rows' values of a position) and stores both rows.
#include "sqmp_internal.h"

namespace sqmp {

namespace {

constexpr int PR_CH = 4;  // output chunks of 8 positions per thread: P + S_pad <= 8192

template <class T>
__global__ __launch_bounds__(256) void permute_rows_kernel(const T* __restrict__ src,
                                                           T* __restrict__ dst,
                                                           const int32_t* __restrict__ map,
                                                           int M, int P, int S_pad, int ppw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t pr_buf[];  // [W] position pairs
  const int tid = threadIdx.x;
  const int W = P + S_pad;  // row length (a multiple of 8)
  const int nch = W / 8;    // 16-B chunks per row
  const int npair = (M + 1) / 2;
  const int p0 = blockIdx.x * ppw, p1 = min(npair, p0 + ppw);
  // the first pair's rows are requested before the map (both latencies overlap)
  u32x4 ra[PR_CH], rb[PR_CH];
  auto load_pair = [&](int rp) {
    const int m0 = 2 * rp;
    const u32x4* s0 = (const u32x4*)(src + (size_t)m0 * W);
    const u32x4* s1 = (const u32x4*)(src + (size_t)(m0 + 1 < M ? m0 + 1 : m0) * W);
#pragma unroll
    for (int c = 0; c < PR_CH; ++c) {
      const int ch = tid + 256 * c;
      if (ch < nch) {
        ra[c] = s0[ch];
        rb[c] = s1[ch];
      }
    }
  };
  if (p0 < p1) load_pair(p0);
  // this thread's output chunks' source positions (16-B map loads, cached for every pair;
  // the tail chunks copy their own positions)
  int src_pos[PR_CH][8];
#pragma unroll
  for (int c = 0; c < PR_CH; ++c) {
    const int ch = tid + 256 * c;
    if (8 * ch + 8 <= P) {
      const i32x4 m0 = ((const i32x4*)map)[2 * ch], m1 = ((const i32x4*)map)[2 * ch + 1];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        src_pos[c][e] = m0[e];
        src_pos[c][4 + e] = m1[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) src_pos[c][e] = ch >= nch ? -1 : 8 * ch + e;  // the tail
    }
  }
  for (int rp = p0; rp < p1; ++rp) {
    const int m0 = 2 * rp;
    const bool has1 = m0 + 1 < M;
#pragma unroll
    for (int c = 0; c < PR_CH; ++c) {
      const int ch = tid + 256 * c;
      if (ch < nch) {
        const u32x4 a = ra[c], b = rb[c];
        u32x4 w0, w1;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          w0[2 * k] = __builtin_amdgcn_perm(b[k], a[k], 0x05040100u);
          w0[2 * k + 1] = __builtin_amdgcn_perm(b[k], a[k], 0x07060302u);
          w1[2 * k] = __builtin_amdgcn_perm(b[k + 2], a[k + 2], 0x05040100u);
          w1[2 * k + 1] = __builtin_amdgcn_perm(b[k + 2], a[k + 2], 0x07060302u);
        }
        ((u32x4*)pr_buf)[2 * ch] = w0;
        ((u32x4*)pr_buf)[2 * ch + 1] = w1;
      }
    }
    if (rp + 1 < p1) load_pair(rp + 1);  // the next pair's loads overlap this pair's work
    __syncthreads();
    T* d0 = dst + (size_t)m0 * W;
    T* d1 = dst + (size_t)(m0 + 1) * W;
#pragma unroll
    for (int c = 0; c < PR_CH; ++c) {
      const int ch = tid + 256 * c;
      if (ch < nch) {
        uint32_t v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = src_pos[c][e] >= 0 ? pr_buf[src_pos[c][e]] : 0u;
        u32x4 y0, y1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          y0[k] = __builtin_amdgcn_perm(v[2 * k + 1], v[2 * k], 0x05040100u);
          y1[k] = __builtin_amdgcn_perm(v[2 * k + 1], v[2 * k], 0x07060302u);
        }
        ((u32x4*)d0)[ch] = y0;
        if (has1) ((u32x4*)d1)[ch] = y1;
      }
    }
    __syncthreads();  // the buffer is rewritten by the next pair
  }
}

}  // namespace

}  // namespace sqmp

using namespace sqmp;

extern "C" int sqmp_permute_act(const void* src, void* dst, const int32_t* map, int dtype, int M,
                                int P, int S_pad, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!src || !dst || !map || M < 0 || P <= 0 || P % 8 || S_pad < 0 || S_pad % 8)
    return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if ((P + S_pad) / 8 > 256 * PR_CH) return SQMP_EUNSUPPORTED;
  if (((uintptr_t)src) % 16 || ((uintptr_t)dst) % 16) return SQMP_EUNSUPPORTED;
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
  const int npair = (M + 1) / 2;
  // one pair per workgroup up to 4096 pairs (latency-bound at 2048-token prefill), then
  // runs of pairs with the next pair prefetched
  const int ppw = npair > 4096 ? cdiv(npair, 4096) : 1;
  const dim3 grid((unsigned)cdiv(npair, ppw));
  const size_t lds = sizeof(uint32_t) * (size_t)(P + S_pad);
  // the dynamic-LDS limit raised once to the largest row this entry accepts (256 PR_CH chunks
  // of 8 positions), not per launch
  constexpr int kMaxLds = (int)sizeof(uint32_t) * 8 * 256 * PR_CH;
  static uint64_t attr_h = 0, attr_b = 0;  // (per device)
  if (dtype == SQMP_F16) {
    if (first_on_device(attr_h))
      SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)permute_rows_kernel<_Float16>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds));
    permute_rows_kernel<_Float16><<<grid, dim3(256), lds, s>>>(
        (const _Float16*)src, (_Float16*)dst, map, M, P, S_pad, ppw);
  } else {
    if (first_on_device(attr_b))
      SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)permute_rows_kernel<__bf16>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds));
    permute_rows_kernel<__bf16><<<grid, dim3(256), lds, s>>>(
        (const __bf16*)src, (__bf16*)dst, map, M, P, S_pad, ppw);
  }
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}
