// Column statistics shared by the weight packer and the activation quantizer:
//   * column absmax over all rows   (fake_quant.py:113 `t.abs().max(dim=0)`, :164 for W)
//   * stable ascending column rank  (fake_quant.py:116 / :167 `torch.argsort(col_max)`,
//                                    pinned to stable=True; ties -> lower index first)
//   * index maps of the packed K axis (salient split of fake_quant.py:291-301, :347-365)
#include "sqmp_internal.h"

namespace sqmp {

// ------------------------------------------------------------------ column absmax
// Block = 4 waves; a lane owns VEC consecutive columns (one 16-B load per row), the four
// waves split the block's row chunk, partial maxima meet in LDS, then one global
// atomicMax per column per block.  1-D grid of cblocks x row-block tiles, row-block major,
// dealt to the XCDs in contiguous eighths (blocks go round-robin over the 8 XCDs): XCD x
// reads the rows the lane-contiguous quantizer's workgroups on XCD x read next (its row pairs
// also come in contiguous eighths), so an input of up to 8 x 4 MiB is still in that XCD's L2
// when the quantizer loads it.
template <class DT, int VEC>
__global__ __launch_bounds__(256) void colmax_kernel(const typename DT::T* __restrict__ x,
                                                     int R, int C, int rows_per_block,
                                                     int cblocks, uint32_t* __restrict__ cmax) {
  typedef typename DT::T T;
  __shared__ float red[4][64 * VEC];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nb = gridDim.x, xcd = blockIdx.x & 7, per = nb >> 3, rem = nb & 7;
  const int t = (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + (blockIdx.x >> 3);
  const int bx = t % cblocks, by = t / cblocks;
  const int c0 = (bx * 64 + lane) * VEC;
  const int r0 = by * rows_per_block;
  const int r1 = min(R, r0 + rows_per_block);
  float m[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) m[i] = 0.f;
  if (c0 + VEC <= C && VEC > 1) {
    // explicit batches of 8 rows: 8 loads in flight per lane (an unrolled loop over a
    // pointer chain was compiled to one load + vmcnt(0) per row)
    int r = r0 + wid;
    for (; r + 28 < r1; r += 32) {
      u32x4 raw[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) raw[u] = *(const u32x4*)(x + (size_t)(r + 4 * u) * C + c0);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const T* v = (const T*)&raw[u];
#pragma unroll
        for (int i = 0; i < VEC; ++i) m[i] = fmaxf(m[i], fabsf(DT::to_f(v[i])));
      }
    }
    for (; r < r1; r += 4) {
      const u32x4 raw = *(const u32x4*)(x + (size_t)r * C + c0);
      const T* v = (const T*)&raw;
#pragma unroll
      for (int i = 0; i < VEC; ++i) m[i] = fmaxf(m[i], fabsf(DT::to_f(v[i])));
    }
  } else if (c0 < C) {
    for (int r = r0 + wid; r < r1; r += 4)
#pragma unroll
      for (int i = 0; i < VEC; ++i)
        if (c0 + i < C) m[i] = fmaxf(m[i], fabsf(DT::to_f(x[(size_t)r * C + c0 + i])));
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) red[wid][lane * VEC + i] = m[i];
  __syncthreads();
  for (int u = threadIdx.x; u < 64 * VEC; u += 256) {
    const float v = fmaxf(fmaxf(red[0][u], red[1][u]), fmaxf(red[2][u], red[3][u]));
    const int c = bx * 64 * VEC + u;
    if (c < C && v > 0.f) atomicMax(&cmax[c], __float_as_uint(v));
  }
}

template <class DT>
static void colmax_launch(const void* x, int R, int C, uint32_t* cmax, hipStream_t s) {
  typedef typename DT::T T;
  constexpr int VEC = 16 / sizeof(T);
  const bool vec_ok = ((C * sizeof(T)) % 16 == 0) && (((uintptr_t)x) % 16 == 0);
  int rows_per_block = 128;
  const int cblocks_v = cdiv(C, 64 * VEC);
  // keep >= ~1024 blocks in flight when R is large, fewer row passes when R is small (at
  // least 32 rows per block: 2048-row Llama inputs 25.7 -> 24.1 us for the whole prepass,
  // fewer atomics per column; profiles/r03_prepass_sweep.txt)
  while (rows_per_block > 32 && (long)cblocks_v * cdiv(R, rows_per_block) < 1024)
    rows_per_block >>= 1;
  if (const char* e = knob("SQMP_COLMAX_RPB")) rows_per_block = atoi(e);
  dim3 block(256);
  const int rblocks = cdiv(R, rows_per_block);
  if (vec_ok) {
    colmax_kernel<DT, VEC><<<dim3(cblocks_v * rblocks), block, 0, s>>>(
        (const T*)x, R, C, rows_per_block, cblocks_v, cmax);
  } else {
    const int cb = cdiv(C, 64);
    colmax_kernel<DT, 1><<<dim3(cb * rblocks), block, 0, s>>>((const T*)x, R, C, rows_per_block,
                                                             cb, cmax);
  }
}

int launch_colmax(const void* x, int dtype, int R, int C, uint32_t* cmax, hipStream_t s,
                  bool zero) {
  if (zero) SQMP_HIP_CHECK(hipMemsetAsync(cmax, 0, sizeof(uint32_t) * (size_t)C, s));
  if (R <= 0 || C <= 0) return SQMP_OK;
  switch (dtype) {
    case SQMP_F32: colmax_launch<F32>(x, R, C, cmax, s); break;
    case SQMP_F16: colmax_launch<F16>(x, R, C, cmax, s); break;
    case SQMP_BF16: colmax_launch<BF16>(x, R, C, cmax, s); break;
    default: return SQMP_EINVAL;
  }
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

// ------------------------------------------------------------------ mean + 3 sigma key
// The "statistical sorting (mean + 3*STD)" strategy of the reference's README (README.md:36;
// absent from its code, so this key is defined here -- parity unpinned): per column,
// key = mean|x| + 3 * std|x| over the R rows (population std), computed from fp64 sums of
// |x| and x^2 and rounded once to fp32.  Stored as fp32 bits in the same slot as the
// absmax key, so the stable rank kernels order both the same way.
template <class DT, int VEC>
__global__ __launch_bounds__(256) void colsum_kernel(const typename DT::T* __restrict__ x,
                                                     int R, int C, int rows_per_block,
                                                     double* __restrict__ s1,
                                                     double* __restrict__ s2) {
  typedef typename DT::T T;
  __shared__ double red[2][4][64 * VEC];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c0 = (blockIdx.x * 64 + lane) * VEC;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(R, r0 + rows_per_block);
  double a[VEC], q[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) a[i] = q[i] = 0.0;
  if (c0 + VEC <= C && VEC > 1) {
    for (int r = r0 + wid; r < r1; r += 4) {
      const u32x4 raw = *(const u32x4*)(x + (size_t)r * C + c0);
      const T* v = (const T*)&raw;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const double d = fabs((double)DT::to_f(v[i]));
        a[i] = __dadd_rn(a[i], d);
        q[i] = __dadd_rn(q[i], __dmul_rn(d, d));
      }
    }
  } else if (c0 < C) {
    for (int r = r0 + wid; r < r1; r += 4)
#pragma unroll
      for (int i = 0; i < VEC; ++i)
        if (c0 + i < C) {
          const double d = fabs((double)DT::to_f(x[(size_t)r * C + c0 + i]));
          a[i] = __dadd_rn(a[i], d);
          q[i] = __dadd_rn(q[i], __dmul_rn(d, d));
        }
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    red[0][wid][lane * VEC + i] = a[i];
    red[1][wid][lane * VEC + i] = q[i];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 64 * VEC; t += 256) {
    const int c = blockIdx.x * 64 * VEC + t;
    if (c >= C) continue;
    const double va = (red[0][0][t] + red[0][1][t]) + (red[0][2][t] + red[0][3][t]);
    const double vq = (red[1][0][t] + red[1][1][t]) + (red[1][2][t] + red[1][3][t]);
    if (va != 0.0) atomicAdd(&s1[c], va);
    if (vq != 0.0) atomicAdd(&s2[c], vq);
  }
}

__global__ __launch_bounds__(256) void mean3std_key_kernel(double* __restrict__ s1,
                                                           double* __restrict__ s2,
                                                           int R, int C,
                                                           uint32_t* __restrict__ key,
                                                           int clear) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const double a1 = s1[c], a2 = s2[c];
  if (clear) s1[c] = s2[c] = 0.0;  // leave the sums zero for the next call
  const double mean = __ddiv_rn(a1, (double)R);
  double var = __dsub_rn(__ddiv_rn(a2, (double)R), __dmul_rn(mean, mean));
  var = var > 0.0 ? var : 0.0;
  const double k = __dadd_rn(mean, __dmul_rn(3.0, __dsqrt_rn(var)));
  key[c] = __float_as_uint(__double2float_rn(k));
}

template <class DT>
static void colsum_launch(const void* x, int R, int C, double* s1, double* s2, hipStream_t s) {
  typedef typename DT::T T;
  constexpr int VEC = 16 / sizeof(T);
  const bool vec_ok = ((C * sizeof(T)) % 16 == 0) && (((uintptr_t)x) % 16 == 0);
  int rows_per_block = 128;
  const int cblocks_v = cdiv(C, 64 * VEC);
  while (rows_per_block > 16 && (long)cblocks_v * cdiv(R, rows_per_block) < 1024)
    rows_per_block >>= 1;
  if (vec_ok) {
    colsum_kernel<DT, VEC><<<dim3(cblocks_v, cdiv(R, rows_per_block)), dim3(256), 0, s>>>(
        (const T*)x, R, C, rows_per_block, s1, s2);
  } else {
    colsum_kernel<DT, 1><<<dim3(cdiv(C, 64), cdiv(R, rows_per_block)), dim3(256), 0, s>>>(
        (const T*)x, R, C, rows_per_block, s1, s2);
  }
}

int launch_colkey_mean3std(const void* x, int dtype, int R, int C, double* sums,
                           uint32_t* key, hipStream_t s, bool clean) {
  if (!clean) SQMP_HIP_CHECK(hipMemsetAsync(sums, 0, 2 * sizeof(double) * (size_t)C, s));
  if (R <= 0 || C <= 0) return SQMP_OK;
  double* s1 = sums;
  double* s2 = sums + C;
  switch (dtype) {
    case SQMP_F32: colsum_launch<F32>(x, R, C, s1, s2, s); break;
    case SQMP_F16: colsum_launch<F16>(x, R, C, s1, s2, s); break;
    case SQMP_BF16: colsum_launch<BF16>(x, R, C, s1, s2, s); break;
    default: return SQMP_EINVAL;
  }
  SQMP_LAUNCH_CHECK();
  mean3std_key_kernel<<<dim3(cdiv(C, 256)), dim3(256), 0, s>>>(s1, s2, R, C, key, clean ? 1 : 0);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

// ------------------------------------------------------------------ stable rank
// 2-D grid of (256 owners) x (RANK_TILE competitors); each owner counts competitors that
// order before it -- (value, list index) lexicographically, i.e. a stable ascending sort
// -- and adds its partial count.  O(L^2) 32-bit compares over broadcast LDS reads,
// fully parallel, deterministic and stable by construction.
constexpr int RANK_TILE = 256;

__global__ __launch_bounds__(256) void rank_kernel(const uint32_t* __restrict__ cmax,
                                                   const int32_t* __restrict__ cols, int L,
                                                   int32_t* __restrict__ rank_by_col) {
  __shared__ uint32_t kv[RANK_TILE];
  const int j0 = blockIdx.y * RANK_TILE;
  const int jn = min(RANK_TILE, L - j0);
  {
    const int t = threadIdx.x;
    // sentinel above every non-negative float's bits: never orders first
    kv[t] = t < jn ? cmax[cols ? cols[j0 + t] : j0 + t] : 0xFFFFFFFFu;
  }
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const int ci = cols ? cols[i] : i;
  const uint32_t mine = cmax[ci];
  const int lim = i - j0;  // competitors t < lim have a lower list index
  int cnt = 0;
#pragma unroll 16
  for (int t = 0; t < RANK_TILE; ++t) {
    const uint32_t k = kv[t];
    cnt += (k < mine || (k == mine && t < lim)) ? 1 : 0;
  }
  if (cnt) atomicAdd(&rank_by_col[ci], cnt);
}

// Counting rank with 128-competitor tiles (more, shorter blocks than rank_kernel): adds
// into counts[cols[i]], which the caller guarantees to be zero (clean workspace).
__global__ __launch_bounds__(256) void rank_count_kernel(const uint32_t* __restrict__ cmax,
                                                         const int32_t* __restrict__ cols, int L,
                                                         int32_t* __restrict__ counts) {
  __shared__ uint32_t kv[128];
  const int j0 = blockIdx.y * 128;
  const int jn = min(128, L - j0);
  if (threadIdx.x < 128)
    kv[threadIdx.x] = (int)threadIdx.x < jn ? cmax[cols[j0 + threadIdx.x]] : 0xFFFFFFFFu;
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const int ci = cols[i];
  const uint32_t mine = cmax[ci];
  const int lim = i - j0;
  int c0 = 0, c1 = 0;
#pragma unroll 16
  for (int t = 0; t < 128; t += 2) {
    c0 += (kv[t] < mine || (kv[t] == mine && t < lim)) ? 1 : 0;
    c1 += (kv[t + 1] < mine || (kv[t + 1] == mine && t + 1 < lim)) ? 1 : 0;
  }
  if (c0 + c1) atomicAdd(&counts[ci], c0 + c1);
}

int launch_rank_count(const uint32_t* cmax, const int32_t* cols, int L, int32_t* counts,
                      hipStream_t s) {
  if (L <= 0) return SQMP_OK;
  rank_count_kernel<<<dim3(cdiv(L, 256), cdiv(L, 128)), dim3(256), 0, s>>>(cmax, cols, L, counts);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

int launch_rank(const uint32_t* cmax, const int32_t* cols, int L, int C,
                int32_t* rank_by_col, hipStream_t s, bool zero) {
  // rank_by_col is indexed by column: clear the whole column range the list can touch.
  if (zero) SQMP_HIP_CHECK(hipMemsetAsync(rank_by_col, 0, sizeof(int32_t) * (size_t)C, s));
  if (L <= 0) return SQMP_OK;
  dim3 grid(cdiv(L, 256), cdiv(L, RANK_TILE));
  rank_kernel<<<grid, dim3(256), 0, s>>>(cmax, cols, L, rank_by_col);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

// Same counts without atomics: block (bx, by) writes the count of competitor tile by for
// its 256 owners to part[by][owner]; the consumer sums the cdiv(L, RANK_TILE) partials.
// Every (tile, owner) slot is written, so the buffer needs no clearing.
__global__ __launch_bounds__(256) void rank_partial_kernel(const uint32_t* __restrict__ cmax,
                                                           const int32_t* __restrict__ cols, int L,
                                                           int ld, int32_t* __restrict__ part) {
  __shared__ uint32_t kv[RANK_TILE];
  const int j0 = blockIdx.y * RANK_TILE;
  const int jn = min(RANK_TILE, L - j0);
  {
    const int t = threadIdx.x;
    kv[t] = t < jn ? cmax[cols ? cols[j0 + t] : j0 + t] : 0xFFFFFFFFu;
  }
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const uint32_t mine = cmax[cols ? cols[i] : i];
  const int lim = i - j0;
  int cnt = 0;
#pragma unroll 16
  for (int t = 0; t < RANK_TILE; ++t) {
    const uint32_t k = kv[t];
    cnt += (k < mine || (k == mine && t < lim)) ? 1 : 0;
  }
  part[(size_t)blockIdx.y * ld + i] = cnt;
}

int rank_tiles(int L) { return L > 0 ? cdiv(L, RANK_TILE) : 0; }

int launch_rank_partial(const uint32_t* cmax, const int32_t* cols, int L, int ld,
                        int32_t* part, hipStream_t s) {
  if (L <= 0) return SQMP_OK;
  dim3 grid(cdiv(L, 256), cdiv(L, RANK_TILE));
  rank_partial_kernel<<<grid, dim3(256), 0, s>>>(cmax, cols, L, ld, part);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

// ------------------------------------------------------------------ index maps
// One workgroup.  flag[k] marks salient columns; the non-salient list is an ordered
// compaction (block-wide exclusive scan over per-thread chunk counts).
__global__ __launch_bounds__(1024) void build_maps_kernel(
    int K, int Kp, const int32_t* __restrict__ rank_by_col, const int32_t* __restrict__ sal,
    int S, int32_t* __restrict__ perm, int32_t* __restrict__ amap,
    int32_t* __restrict__ amap_fq, int32_t* __restrict__ nonsal) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_maps[];
  int* scan = (int*)smem_maps;                      // 1024 ints
  unsigned char* flag = smem_maps + 1024 * sizeof(int);  // K bytes
  const int t = threadIdx.x;
  for (int k = t; k < K; k += 1024) flag[k] = 0;
  __syncthreads();
  for (int j = t; j < S; j += 1024) flag[sal[j]] = 1;
  __syncthreads();
  for (int k = t; k < K; k += 1024) {
    const int p = rank_by_col ? rank_by_col[k] : k;
    perm[p] = k;
    amap[p] = flag[k] ? -1 : k;
    amap_fq[k] = flag[k] ? -2 : k;
  }
  for (int p = K + t; p < Kp; p += 1024) {
    perm[p] = -1;
    amap[p] = -1;
  }
  // ordered compaction of the non-salient columns
  const int chunk = (K + 1023) / 1024;
  const int kb = t * chunk, ke = min(K, kb + chunk);
  int cnt = 0;
  for (int k = kb; k < ke; ++k) cnt += flag[k] ? 0 : 1;
  scan[t] = cnt;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = t >= off ? scan[t - off] : 0;
    __syncthreads();
    scan[t] += v;
    __syncthreads();
  }
  int pos = scan[t] - cnt;
  for (int k = kb; k < ke; ++k)
    if (!flag[k]) nonsal[pos++] = k;
}

int launch_build_maps(int K, int Kp, const int32_t* rank_by_col, const int32_t* salient,
                      int S, int32_t* perm, int32_t* amap, int32_t* amap_fq,
                      int32_t* nonsal, hipStream_t s) {
  const size_t lds = 1024 * sizeof(int) + (size_t)round_up(K, 16);
  if (lds > 160 * 1024) return SQMP_EUNSUPPORTED;
  SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)build_maps_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  build_maps_kernel<<<dim3(1), dim3(1024), lds, s>>>(K, Kp, rank_by_col, salient, S, perm,
                                                      amap, amap_fq, nonsal);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace sqmp
