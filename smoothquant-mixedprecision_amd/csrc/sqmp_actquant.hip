// Runtime activation quantization: the pre-GEMM half of W4A4Linear.forward
// (/root/reference/smoothquant/fake_quant.py:291-304) and the output quantizer (:308-316).
//
// Reference semantics restated (x is [M][K] in D, S = salient columns, A = x[:, ~S]):
//   per_token  (:56-64)   s[m]    = D(D(clamp(max_k |A[m,k]|, 1e-5)) / q_max)
//   per_tensor (:67-75)   s       = same over the whole of A
//   per_group  (:104-154) columns of A sorted ascending (stable) by their batch absmax
//                         max_m |A[m,k]|; groups of G consecutive sorted columns;
//                         s[m,g] per row and group.  (:77-101 unsorted variant: groups
//                         of G consecutive non-salient columns.)
//   x_hat = D(rne(D(x / s)) * s); salient columns pass through exactly (:297-301).
//
// Pipeline (per_group): colmax over M (1 kernel) -> stable rank of the K' non-salient
// columns (1 kernel) -> this row kernel.  per_tensor: colmax -> row kernel.
// per_token: row kernel only.
//
// Row kernel: persistent workgroups (grid-stride over rows).  Each workgroup builds its
// LDS tables once (column -> group, output position -> (group, column)), then per row:
// stage the row in LDS, per-(row, group) absmax with LDS atomics, scales, and writes the
// output row in OUTPUT order with 16-B coalesced stores (gathering from the LDS row).
#include <stdlib.h>

#include "sqmp_internal.h"

namespace sqmp {

__device__ inline int fdiv_floor_a(int r, int G, float invG) {
  int q = (int)((float)r * invG);
  if ((q + 1) * G <= r) ++q;
  if (q * G > r) --q;
  return q;
}

constexpr uint32_t G_ZERO = 0xFFFFu;  // output position holds 0 (salient / padding)
constexpr uint32_t G_PASS = 0xFFFEu;  // output position passes the input through

enum { MODE_TOKEN = 0, MODE_TENSOR = 1, MODE_GROUP = 2 };
constexpr int PFC_FP = 6;  // 16-B row chunks per thread held for the next row (K*esize <= 24 KiB)

template <class DT, int MODE, int OUT>
__global__ __launch_bounds__(256) void quant_act_kernel(
    typename DT::T* __restrict__ x, int M, int K, int q_max, int G, int nga,
    const int32_t* __restrict__ amap, int P, const int32_t* __restrict__ nonsal, int Kn,
    const int32_t* __restrict__ sal, int S, int S_pad,
    const int32_t* __restrict__ rank_by_col, const uint32_t* __restrict__ cmax,
    void* __restrict__ out, float* __restrict__ out_scale,
    typename DT::T* __restrict__ out_xs) {
  typedef typename DT::T T;
  constexpr int VEC = 16 / sizeof(T);  // D elements per 16-B store
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_q[];
  // LDS carve (all offsets 16-B aligned)
  const int rowb = (int)round_up_dev(K * (int)sizeof(T), 16);
  T* row = (T*)smem_q;                                        // K
  uint32_t* ent = (uint32_t*)(smem_q + rowb);                 // P: (group << 16) | column
  uint16_t* grp = (uint16_t*)(ent + P);                       // K: group of column
  const int grpb = (int)round_up_dev(K * 2, 16);
  uint32_t* gmax = (uint32_t*)((unsigned char*)grp + grpb);   // nga
  float* sc = (float*)(gmax + nga);                           // nga
  float* red = sc + nga;                                      // 16
  const int tid = threadIdx.x;
  const float invG = 1.0f / (float)G;

  // ---- tables (once per workgroup)
  for (int k = tid; k < K; k += 256) grp[k] = (uint16_t)G_ZERO;
  __syncthreads();
  for (int i = tid; i < Kn; i += 256) {
    const int k = nonsal[i];
    int g = 0;
    if (MODE == MODE_GROUP) g = fdiv_floor_a(rank_by_col ? rank_by_col[k] : i, G, invG);
    grp[k] = (uint16_t)g;
  }
  __syncthreads();
  for (int p = tid; p < P; p += 256) {
    const int k = amap[p];
    uint32_t e;
    if (k >= 0) e = ((uint32_t)grp[k] << 16) | (uint32_t)k;
    else if (k == -2) e = (G_PASS << 16) | (uint32_t)p;
    else e = G_ZERO << 16;
    ent[p] = e;
  }
  float s_all = 0.f;
  if (MODE == MODE_TENSOR) {
    float m = 0.f;
    for (int i = tid; i < Kn; i += 256) m = fmaxf(m, __uint_as_float(cmax[nonsal[i]]));
    m = block_max(m, red);
    s_all = group_scale<DT>(m, q_max);
  }
  __syncthreads();

  const bool xvec = ((K * (int)sizeof(T)) % 16 == 0) && (((uintptr_t)x) % 16 == 0);
  // Rows of at most PFC 16-B chunks per thread are software-pipelined: the next row's
  // chunks are loaded into registers while this row is quantized (hides HBM latency).
  constexpr int PFC = 4;
  const int nch = xvec ? K / VEC : 0;
  const bool pipe = xvec && nch <= PFC * 256;
  u32x4 nxt[PFC];
  auto load_row = [&](int mm) {
    const u32x4* src = (const u32x4*)(x + (size_t)mm * K);
#pragma unroll
    for (int i = 0; i < PFC; ++i) {
      const int c = tid + 256 * i;
      if (c < nch) nxt[i] = src[c];
    }
  };
  if (pipe && (int)blockIdx.x < M) load_row(blockIdx.x);
  for (int m = blockIdx.x; m < M; m += gridDim.x) {
    T* xr = x + (size_t)m * K;
    // ---- stage the row
    if (pipe) {
#pragma unroll
      for (int i = 0; i < PFC; ++i) {
        const int c = tid + 256 * i;
        if (c < nch) ((u32x4*)row)[c] = nxt[i];
      }
      if (m + (int)gridDim.x < M) load_row(m + gridDim.x);
    } else if (xvec) {
      for (int c = tid; c < K / VEC; c += 256) ((u32x4*)row)[c] = ((const u32x4*)xr)[c];
    } else {
      for (int k = tid; k < K; k += 256) row[k] = xr[k];
    }
    if (MODE == MODE_GROUP)
      for (int g = tid; g < nga; g += 256) gmax[g] = 0u;
    __syncthreads();
    // ---- statistics
    float s_row = s_all;
    if (MODE == MODE_TOKEN) {
      float mx = 0.f;
      for (int k = tid; k < K; k += 256)
        if (grp[k] != G_ZERO) mx = fmaxf(mx, fabsf(DT::to_f(row[k])));
      mx = block_max(mx, red);
      s_row = group_scale<DT>(mx, q_max);
    } else if (MODE == MODE_GROUP) {
      for (int k = tid; k < K; k += 256) {
        const uint32_t g = grp[k];
        if (g != G_ZERO) {
          const float v = fabsf(DT::to_f(row[k]));
          if (v > 0.f) atomicMax(&gmax[g], __float_as_uint(v));
        }
      }
      __syncthreads();
      for (int g = tid; g < nga; g += 256) sc[g] = group_scale<DT>(__uint_as_float(gmax[g]), q_max);
      __syncthreads();
    }
    // ---- outputs, in output order
    if (OUT == SQMP_OUT_FP) {
      const int W = P + S_pad;
      T* o = (T*)out + (size_t)m * W;
      for (int c = tid; c < W / VEC; c += 256) {
        T v[VEC];
#pragma unroll
        for (int e8 = 0; e8 < VEC; ++e8) {
          const int p = c * VEC + e8;
          float r = 0.f;
          if (p < P) {
            const uint32_t e = ent[p];
            const uint32_t g = e >> 16;
            if (g != G_ZERO) {
              const float s = MODE == MODE_GROUP ? sc[g] : s_row;
              const float t = DT::to_f(row[e & 0xFFFFu]);
              // x_hat, rounded to D below; the sign of x is kept on zero codes (the
              // reference's -0.0, fake_quant.py:142)
              r = __builtin_copysignf(__builtin_rintf(rd<DT>(t / s)) * s, t);
            }
          } else if (p - P < S) {
            r = DT::to_f(row[sal[p - P]]);
          }
          v[e8] = DT::from_f(r);
        }
        ((u32x4*)o)[c] = *(const u32x4*)v;
      }
    } else {  // SQMP_OUT_INPLACE: P == K, write back through amap_fq
      if (xvec) {
        for (int c = tid; c < K / VEC; c += 256) {
          T v[VEC];
#pragma unroll
          for (int e8 = 0; e8 < VEC; ++e8) {
            const int p = c * VEC + e8;
            const uint32_t e = ent[p];
            const uint32_t g = e >> 16;
            if (g == G_PASS || g == G_ZERO) {
              v[e8] = row[p];
            } else {
              const float s = MODE == MODE_GROUP ? sc[g] : s_row;
              const float t = DT::to_f(row[e & 0xFFFFu]);
              v[e8] = DT::from_f(__builtin_copysignf(__builtin_rintf(rd<DT>(t / s)) * s, t));
            }
          }
          ((u32x4*)xr)[c] = *(const u32x4*)v;
        }
      } else {
        for (int p = tid; p < K; p += 256) {
          const uint32_t e = ent[p];
          const uint32_t g = e >> 16;
          if (g == G_PASS || g == G_ZERO) continue;
          const float s = MODE == MODE_GROUP ? sc[g] : s_row;
          const float t = DT::to_f(row[e & 0xFFFFu]);
          xr[p] = DT::from_f(__builtin_copysignf(__builtin_rintf(rd<DT>(t / s)) * s, t));
        }
      }
    }
    __syncthreads();  // row / gmax reuse
  }
}

// ---------------------------------------------------------------- OUT_FP fast kernel
// x_hat code of one element: rne(D(t / s)).  q = t * r with r = RN(1/s) is within ~1 fp32
// ulp of the correctly rounded quotient, so D(q) == D(t / s) unless q lies within a few
// ulps of a D rounding midpoint (low 13 / 16 dropped bits == half) -- then the exact
// division decides.  |q| < 0.25 always yields a (signed) zero code.
template <class DT>
__device__ inline float fast_code(float t, float s, float r) {
  if (DT::id == SQMP_F32) {
    // RN(t / s) from r = RN(1 / s): q0 = t r, e = t - q0 s exactly (fma), RN(q0 + e r) is
    // the correctly rounded quotient (Markstein); the code is its rint
    const float q0 = t * r;
    const float e = __builtin_fmaf(-q0, s, t);
    return __builtin_rintf(__builtin_fmaf(e, r, q0));
  }
  const float q = t * r;
  const uint32_t b = __float_as_uint(q);
  constexpr int DROP = DT::id == SQMP_F16 ? 13 : 16;
  constexpr uint32_t MASK = (1u << DROP) - 1, HALF = 1u << (DROP - 1);
  const uint32_t lo = b & MASK;
  const uint32_t d = lo > HALF ? lo - HALF : HALF - lo;
  if (d <= 3u && fabsf(q) >= 0.25f) return __builtin_rintf(rd<DT>(t / s));
  return __builtin_rintf(rd<DT>(q));
}

// Per row: stage the row in LDS (software-pipelined through registers), ONE gather pass
// over the output positions (values kept in registers; per-group absmax by LDS atomics),
// the group scales and reciprocals, then quantize from registers and write 16-B chunks.
// The entry table is chunk-major (two planes of 4 entries) so lanes read consecutive
// 16-B words.  Rows up to FCH*2048 packed positions; longer rows use quant_act_kernel.
constexpr int FCH = 6;  // output chunks (8 positions) per thread
template <class DT, int MODE>
__global__ __launch_bounds__(256) void quant_fp_kernel(
    const typename DT::T* __restrict__ x, int M, int K, int q_max, int G, int nga,
    const int32_t* __restrict__ amap, int P, const int32_t* __restrict__ nonsal, int Kn,
    const int32_t* __restrict__ sal, int S, int S_pad,
    const int32_t* __restrict__ rank_by_col, const uint32_t* __restrict__ cmax,
    typename DT::T* __restrict__ out) {
  typedef typename DT::T T;
  constexpr int VEC = 16 / sizeof(T);
  static_assert(VEC == 8, "fp16 / bf16 only");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_f[];
  const int NCH = P / 8;                       // main chunks (P % 128 == 0)
  const int W = P + S_pad, WCH = W / 8;        // all output chunks
  const int rowb = (int)round_up_dev(K * (int)sizeof(T), 16);
  T* row = (T*)smem_f;
  u32x4* ent = (u32x4*)(smem_f + rowb);        // [2][NCH]
  uint16_t* grp = (uint16_t*)(ent + 2 * NCH);  // K
  const int grpb = (int)round_up_dev(K * 2, 16);
  float2* scr = (float2*)((unsigned char*)grp + grpb);      // nga: (scale, 1/scale)
  uint32_t* gmax = (uint32_t*)(scr + nga);                   // nga
  uint16_t* salc = (uint16_t*)(gmax + nga);                  // S_pad: salient column or 0xFFFF
  float* red = (float*)(salc + round_up_dev(S_pad, 8));      // 16
  const int tid = threadIdx.x;
  const float invG = 1.0f / (float)G;

  for (int k = tid; k < K; k += 256) grp[k] = (uint16_t)G_ZERO;
  for (int j = tid; j < S_pad; j += 256) salc[j] = j < S ? (uint16_t)sal[j] : (uint16_t)0xFFFFu;
  __syncthreads();
  for (int i = tid; i < Kn; i += 256) {
    const int k = nonsal[i];
    int g = 0;
    if (MODE == MODE_GROUP) g = fdiv_floor_a(rank_by_col ? rank_by_col[k] : i, G, invG);
    grp[k] = (uint16_t)g;
  }
  __syncthreads();
  for (int c = tid; c < NCH; c += 256) {
    uint32_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = amap[c * 8 + j];
      e[j] = k >= 0 ? (((uint32_t)grp[k] << 16) | (uint32_t)k) : (G_ZERO << 16);
    }
    ent[c] = u32x4{e[0], e[1], e[2], e[3]};
    ent[NCH + c] = u32x4{e[4], e[5], e[6], e[7]};
  }
  float s_all = 0.f, r_all = 0.f;
  if (MODE == MODE_TENSOR) {
    float m = 0.f;
    for (int i = tid; i < Kn; i += 256) m = fmaxf(m, __uint_as_float(cmax[nonsal[i]]));
    m = block_max(m, red);
    s_all = group_scale<DT>(m, q_max);
    r_all = 1.0f / s_all;
  }
  __syncthreads();

  const int nch = K / VEC;
  u32x4 nxt[PFC_FP];
  auto load_row = [&](int mm) {
    const u32x4* src = (const u32x4*)(x + (size_t)mm * K);
#pragma unroll
    for (int i = 0; i < PFC_FP; ++i) {
      const int c = tid + 256 * i;
      if (c < nch) nxt[i] = src[c];
    }
  };
  if ((int)blockIdx.x < M) load_row(blockIdx.x);
  for (int m = blockIdx.x; m < M; m += gridDim.x) {
#pragma unroll
    for (int i = 0; i < PFC_FP; ++i) {
      const int c = tid + 256 * i;
      if (c < nch) ((u32x4*)row)[c] = nxt[i];
    }
    if (m + (int)gridDim.x < M) load_row(m + gridDim.x);
    if (MODE == MODE_GROUP)
      for (int g = tid; g < nga; g += 256) gmax[g] = 0u;
    __syncthreads();
    // ---- gather pass: values of this thread's chunks into registers + group absmax
    uint32_t vals[FCH][4];
    float lmax = 0.f;
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const int c = tid + 256 * i;
      if (c < NCH) {
        const u32x4 e0 = ent[c], e1 = ent[NCH + c];
        const uint32_t e[8] = {e0[0], e0[1], e0[2], e0[3], e1[0], e1[1], e1[2], e1[3]};
        T v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t g = e[j] >> 16;
          v[j] = g != G_ZERO ? row[e[j] & 0xFFFFu] : DT::from_f(0.f);
          const float a = fabsf(DT::to_f(v[j]));
          if (MODE == MODE_GROUP) {
            if (g != G_ZERO && a > 0.f) atomicMax(&gmax[g], __float_as_uint(a));
          } else {
            lmax = fmaxf(lmax, a);
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[i][j] = v[j];
      }
    }
    float s_row = s_all, r_row = r_all;
    if (MODE == MODE_TOKEN) {
      const float mx = block_max(lmax, red);
      s_row = group_scale<DT>(mx, q_max);
      r_row = 1.0f / s_row;
    } else if (MODE == MODE_GROUP) {
      __syncthreads();
      for (int g = tid; g < nga; g += 256) {
        const float sg = group_scale<DT>(__uint_as_float(gmax[g]), q_max);
        scr[g] = make_float2(sg, 1.0f / sg);
      }
      __syncthreads();
    }
    // ---- quantize from registers, 16-B stores in output order
    T* o = out + (size_t)m * W;
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const int c = tid + 256 * i;
      if (c < NCH) {
        const u32x4 e0 = ent[c], e1 = ent[NCH + c];
        const uint32_t e[8] = {e0[0], e0[1], e0[2], e0[3], e1[0], e1[1], e1[2], e1[3]};
        const T* v = (const T*)vals[i];
        T r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t g = e[j] >> 16;
          float y = 0.f;
          if (g != G_ZERO) {
            const float2 sr = MODE == MODE_GROUP ? scr[g] : make_float2(s_row, r_row);
            const float t = DT::to_f(v[j]);
            y = __builtin_copysignf(fast_code<DT>(t, sr.x, sr.y) * sr.x, t);  // -0.0 as the reference
          }
          r[j] = DT::from_f(y);
        }
        ((u32x4*)o)[c] = *(const u32x4*)r;
      }
    }
    // ---- exact salient tail
    for (int c = NCH + tid; c < WCH; c += 256) {
      T r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t k = salc[(c - NCH) * 8 + j];
        r[j] = k != 0xFFFFu ? row[k] : DT::from_f(0.f);
      }
      ((u32x4*)o)[c] = *(const u32x4*)r;
    }
    __syncthreads();  // row / gmax reuse
  }
}

// ---------------------------------------------------------------- entry table
// Once per call: for every packed position p, ent = (group << 16) | column (G_ZERO for
// salient / padding positions), written in the wave kernel's LDS image order (two planes
// of 4 entries per 8-position chunk), and rank_by_col[column] for the block kernels.
// The list index of column k is found by binary search in the ascending `nonsal`; its
// rank is the sum of the rank_partial tiles (per_group), the list index itself otherwise.
__global__ __launch_bounds__(256) void build_ent_kernel(
    const int32_t* __restrict__ amap, int P, const int32_t* __restrict__ nonsal, int Kn,
    const int32_t* __restrict__ part, int ntile, int ld, int mode, int G,
    uint32_t* __restrict__ ent, int32_t* __restrict__ rank_by_col, uint32_t* __restrict__ lctab,
    int lc_len, uint32_t lc_none, int32_t* __restrict__ colsorted) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  // ranks [Kn, lc_len) of the lane-contiguous table: (zero word, sink word) entries
  if (lctab)
    for (int r = Kn + p; r < lc_len; r += P) lctab[r] = lc_none;
  if (p >= P) return;
  const int k = amap[p];
  uint32_t e = G_ZERO << 16;
  if (k >= 0 && Kn > 0) {
    int lo = 0, hi = Kn - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (nonsal[mid] < k) lo = mid + 1; else hi = mid;
    }
    int r = lo;
    if (part) {
      r = 0;
      for (int t = 0; t < ntile; ++t) r += part[(size_t)t * ld + lo];
      if (rank_by_col) rank_by_col[k] = r;
      if (colsorted) colsorted[r] = k;  // the sorted order, for SQMP_QA_REUSE_STATS
    }
    const int g = mode == MODE_GROUP ? r / G : 0;
    e = ((uint32_t)g << 16) | (uint32_t)k;
    // rank-ordered (column, packed position) table of the lane-contiguous quantizer
    if (lctab) lctab[r] = (uint32_t)k | ((uint32_t)p << 16);
  }
  if (ent) {
    const int c = p >> 3, j = p & 7;
    ent[(size_t)(j >> 2) * (P / 2) + c * 4 + (j & 3)] = e;
  }
}


// ---------------------------------------------------------------- entry table from lctab
// The wave quantizers' chunk-major entry table built from the lane-contiguous table of the
// same call (lctab[r] = column | packed position << 16 for rank r < Kn): rank threads
// scatter (group << 16) | column to their position, position threads mark the positions
// amap leaves empty (salient / padding: -1; in-place salient pass-through: -2) G_ZERO --
// disjoint sets.  Also clears the column keys the rank table read (clean workspace).
__global__ __launch_bounds__(256) void ent_from_lctab_kernel(
    const uint32_t* __restrict__ lctab, int Kn, const int32_t* __restrict__ amap, int P,
    int G, uint32_t* __restrict__ ent, uint32_t* __restrict__ key_clear, int clear_words) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  auto put = [&](int p, uint32_t e) {
    const int c = p >> 3, j = p & 7;
    ent[(size_t)(j >> 2) * (P / 2) + c * 4 + (j & 3)] = e;
  };
  if (t < Kn) {
    const uint32_t e = lctab[t];
    put((int)(e >> 16), ((uint32_t)(t / G) << 16) | (e & 0xFFFFu));
  }
  if (t < P && amap[t] < 0) put(t, G_ZERO << 16);
  if (key_clear && t < clear_words) key_clear[t] = 0u;
}

// ---------------------------------------------------------------- table padding
// Ranks [Kn, lc_len) of the lane-contiguous table.  With the salient list and a per-weight
// posmap, the first S of them are (zero word, packed position of salient column j) entries:
// the quantizer gathers the zero word and scatters it to the salient positions itself, so it
// needs no salient-position mask (the amap loads and ballots it used to make per workgroup).
// The rest, and every pad rank without a posmap (in-place output quantization: salient
// columns pass through), are the (zero word, sink word) entry lc_none.
__device__ inline uint32_t pad_entry(int r, int Kn, uint32_t lc_none,
                                     const int32_t* __restrict__ sal, int S,
                                     const int32_t* __restrict__ posmap) {
  const int j = r - Kn;
  return (posmap && j < S) ? (lc_none & 0xFFFFu) | ((uint32_t)posmap[sal[j]] << 16) : lc_none;
}

// ---------------------------------------------------------------- lane-contiguous table
// Per call, one thread per non-salient list entry i (column nonsal[i]):
//   TAB_COUNTS  r = counts[col] (the stable rank), counts[col] = 0 afterwards, and the
//               sorted column list colsorted[r] = col is kept for sibling layers;
//   TAB_SORTED  col = colsorted[i], r = i (statistics reused from a previous call);
//   TAB_LIST    r = i (unsorted groups / per_token / per_tensor).
// lctab[r] = col | posmap[col] << 16, ranks [Kn, lc_len) the padding entries (pad_entry),
// and key[0..K) is cleared when given (clean-workspace protocol).
enum { TAB_COUNTS = 0, TAB_SORTED = 1, TAB_LIST = 2 };
__global__ __launch_bounds__(256) void lc_table_kernel(
    int mode, const int32_t* __restrict__ nonsal, int Kn, int K,
    const int32_t* __restrict__ posmap, int32_t* __restrict__ counts,
    int32_t* __restrict__ colsorted, uint32_t* __restrict__ key, uint32_t* __restrict__ lctab,
    int lc_len, uint32_t lc_none, const int32_t* __restrict__ sal, int S) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int nt = gridDim.x * 256;
  if (t < Kn) {
    int col, r;
    if (mode == TAB_SORTED) {
      col = colsorted[t];
      r = t;
    } else {
      col = nonsal[t];
      r = t;
      if (mode == TAB_COUNTS) {
        r = counts[col];
        counts[col] = 0;
        colsorted[r] = col;
      }
    }
    lctab[r] = (uint32_t)col | ((uint32_t)(posmap ? posmap[col] : col) << 16);
  }
  if (key && t < K) key[t] = 0u;
  for (int r = Kn + t; r < lc_len; r += nt) lctab[r] = pad_entry(r, Kn, lc_none, sal, S, posmap);
}

// The F8 quantizer's table in packed-POSITION order: lctab[p] = amap[p] | p << 16 for the
// positions of a non-salient column, the (zero word, sink word) entry for salient / padding
// positions and for p in [P, lc_len): a thread's entries are then consecutive output positions.
__global__ __launch_bounds__(256) void pos_table_kernel(const int32_t* __restrict__ amap, int P,
                                                        uint32_t* __restrict__ lctab, int lc_len,
                                                        uint32_t lc_none) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= lc_len) return;
  const int c = p < P ? amap[p] : -1;
  lctab[p] = c >= 0 ? (uint32_t)c | ((uint32_t)p << 16) : lc_none;
}

// ---------------------------------------------------------------- rank + table, one launch
// For lists up to RT_MAX entries: every workgroup stages all L keys key[nonsal[j]] in LDS
// and ranks R * 256 / TPO owners, TPO lanes per group of R owners splitting the competitors
// (16-B LDS reads, interleaved so the TPO lanes hit consecutive chunks; each chunk read is
// compared against all R owners), then reduces the TPO partial counts by lane shuffles.  The
// stable rank of owner i is
//   #{j : key_j < key_i} + #{j < i : key_j == key_i}
// (the reference's stable argsort, fake_quant.py:113), counted as key_j < thr with
// thr = key_i + 1 on 4-entry chunks wholly below i, key_i elsewhere, plus the equal keys
// of i's own chunk below i.  Writes colsorted[r] and lctab[r] = col | posmap[col] << 16,
// and the (zero, sink) entries of ranks [L, lc_len).  The keys are NOT cleared here (other
// workgroups may still read them): the quantizer launched next clears them.
// The staging gathers up to SB entries per thread in one batch (all index loads, then
// all key loads: two dependent round trips for the whole list up to 256 * SB entries):
// SB = 24 (SQMP_RT_SB = 8 / 16 / 24 A/B; 64 -- one batch up to RT_MAX -- measured 2.4-3.2x
// slower at 4096 / 11008 columns: the registers cost occupancy, profiles/r04_rank_sb.txt).
constexpr int RT_MAX = 16384;  // 64 KiB of keys in LDS

// stage the L keys key[nonsal[j]] (padded with 0xFFFFFFFF to 4 L4 entries) into LDS
template <int RT_SB>
__device__ inline void rank_stage_keys(const uint32_t* key, const int32_t* __restrict__ nonsal,
                                       int L, int L4, uint32_t* rt_kv) {
  for (int j0 = threadIdx.x; j0 < 4 * L4; j0 += 256 * RT_SB) {
    int idx[RT_SB];
    uint32_t kv[RT_SB];
#pragma unroll
    for (int u = 0; u < RT_SB; ++u) {
      const int j = j0 + 256 * u;
      idx[u] = j < L ? nonsal[j] : -1;
    }
#pragma unroll
    for (int u = 0; u < RT_SB; ++u) kv[u] = idx[u] >= 0 ? key[idx[u]] : 0xFFFFFFFFu;
#pragma unroll
    for (int u = 0; u < RT_SB; ++u) {
      const int j = j0 + 256 * u;
      if (j < 4 * L4) rt_kv[j] = kv[u];
    }
  }
}

// DENSE staging (SQMP_RT_DENSE): every column's key key[0 .. K) by coalesced 16-B loads in ONE
// batch (no nonsal -> key gather: one round trip instead of two dependent ones per batch),
// padded to 4 K4 entries, then the salient columns' keys (loaded alongside) set to 0xFFFFFFFF,
// above every real key: an owner then ranks against the non-salient columns in COLUMN order,
// which is the list order (nonsal ascending), so its ties still break by list index.
template <int CB>
__device__ inline void rank_stage_dense(const uint32_t* __restrict__ key, int K, int K4,
                                        const int32_t* __restrict__ sal, int S, uint32_t* rt_kv) {
  const u32x4* k4 = (const u32x4*)key;
  const u32x4 none = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  const int Kq = K >> 2;  // K % 4 == 0 (quant_lc_supported: K % 8 == 0)
  const int tid = threadIdx.x;
  // the first CB salient indices of this thread ride along with the first key batch
  int sv[CB];
  const int nb = (K4 + 256 * CB - 1) / (256 * CB);  // batches (uniform: barriers follow)
  for (int b = 0; b < nb; ++b) {
    const int c0 = tid + 256 * CB * b;
    u32x4 v[CB];
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const int c = c0 + 256 * u;
      v[u] = c < Kq ? k4[c] : none;
      if (b == 0) sv[u] = c < S ? sal[c] : -1;
    }
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const int c = c0 + 256 * u;
      if (c < K4) ((u32x4*)rt_kv)[c] = v[u];
    }
  }
  __syncthreads();  // every key is staged before a salient column's key is overwritten
#pragma unroll
  for (int u = 0; u < CB; ++u)
    if (sv[u] >= 0) rt_kv[sv[u]] = 0xFFFFFFFFu;
  for (int c = tid + 256 * CB; c < S; c += 256) rt_kv[sal[c]] = 0xFFFFFFFFu;
}

// Rank the R owners g0 .. g0 + R - 1 of this lane group (TPO lanes, `sub` = this lane's index
// in it) against the L staged keys, then write their table entries (see rank_table_kernel).
// An owner's table entries: its column and packed positions (this layer's and the
// siblings'), loaded at kernel start so that their round trips overlap the key staging.
template <int R>
struct RankOwnerEnt {
  uint32_t ent[R][3];  // col | pos << 16 for the table and up to two sibling tables
  int col[R];
};

// BYCOL (the dense stagings): owner g is COLUMN g (< n = K) -- no list lookup in front of the
// posmap load; a salient column's staged key is the sentinel, and it ranks nothing.  Else
// owner g is list entry g (< n = L), column nonsal[g].
template <int R, bool BYCOL = false>
__device__ inline RankOwnerEnt<R> rank_owner_ents(int g0, int sub, int n,
                                                  const int32_t* __restrict__ nonsal,
                                                  const int32_t* __restrict__ posmap,
                                                  const SibTables& sib) {
  RankOwnerEnt<R> e;
  int pm[R][3];
#pragma unroll
  for (int o = 0; o < R; ++o)
    e.col[o] = sub == 0 && g0 + o < n ? (BYCOL ? g0 + o : nonsal[g0 + o]) : -1;
#pragma unroll
  for (int o = 0; o < R; ++o) {
    const int c = e.col[o] < 0 ? 0 : e.col[o];
    pm[o][0] = e.col[o] >= 0 && posmap ? posmap[c] : c;
    pm[o][1] = e.col[o] >= 0 && sib.n > 0 ? sib.posmap[0][c] : 0;
    pm[o][2] = e.col[o] >= 0 && sib.n > 1 ? sib.posmap[1][c] : 0;
  }
#pragma unroll
  for (int o = 0; o < R; ++o)
#pragma unroll
    for (int t = 0; t < 3; ++t) e.ent[o][t] = (uint32_t)e.col[o] | ((uint32_t)pm[o][t] << 16);
  return e;
}

template <int TPO, int R, bool DENSE = false>
__device__ inline void rank_owner_group(const uint32_t* rt_kv, int L, int L4, int g0, int sub,
                                        const RankOwnerEnt<R>& oe,
                                        int32_t* __restrict__ colsorted,
                                        uint32_t* __restrict__ lctab, const SibTables& sib) {
  uint32_t mine[R], cnt[R];
  int ochunk[R], oidx[R];
#pragma unroll
  for (int o = 0; o < R; ++o) {
    const int li = g0 + o < L ? g0 + o : L - 1;
    // (DENSE: the staged array is column-indexed -- the owner sits at its column, which the
    // group's sub 0 lane loaded; owners past the list rank column 0 and discard)
    int oi = li;
    if constexpr (DENSE) {  // (owner = column: rank_owner_ents<R, true>)
      const int c = __shfl(oe.col[o], (int)(threadIdx.x & 63) & ~(TPO - 1), 64);
      oi = c >= 0 ? c : 0;
    }
    oidx[o] = oi;
    mine[o] = rt_kv[oi];
    ochunk[o] = oi >> 2;
    cnt[o] = 0u;
  }
  const u32x4* kv4 = (const u32x4*)rt_kv;
#pragma unroll 2
  for (int j4 = sub; j4 < L4; j4 += TPO) {
    const u32x4 k = kv4[j4];
#pragma unroll
    for (int o = 0; o < R; ++o) {
      const uint32_t thr = j4 < ochunk[o] ? mine[o] + 1u : mine[o];  // keys never reach 0xFFFFFFFF
      cnt[o] += (k[0] < thr ? 1u : 0u) + (k[1] < thr ? 1u : 0u) + (k[2] < thr ? 1u : 0u) +
                (k[3] < thr ? 1u : 0u);
    }
  }
#pragma unroll
  for (int o = 0; o < R; ++o) {
    const int oi = oidx[o];
    if (sub == (ochunk[o] % TPO))
      for (int e = 0; e < (oi & 3); ++e) cnt[o] += rt_kv[4 * ochunk[o] + e] == mine[o] ? 1u : 0u;
#pragma unroll
    for (int w = 1; w < TPO; w <<= 1) cnt[o] += (uint32_t)__shfl_xor((int)cnt[o], w, 64);
    // (DENSE: a salient column's owner -- sentinel key -- writes nothing)
    if (sub == 0 && (DENSE ? (oe.col[o] >= 0 && mine[o] != 0xFFFFFFFFu) : g0 + o < L)) {
      colsorted[cnt[o]] = oe.col[o];
      lctab[cnt[o]] = oe.ent[o][0];
      if (sib.n > 0) sib.lctab[0][cnt[o]] = oe.ent[o][1];
      if (sib.n > 1) sib.lctab[1][cnt[o]] = oe.ent[o][2];
    }
  }
}

// ---- 16-bit dense ranking (KW = 1 / 2: column maxima of f16 / bf16 data, whose keys are
// the values' 15-bit f16 / bf16 patterns -- monotone for non-negative values): half the LDS
// bytes, and two keys per packed u16 compare: [key < thr] = min(sat(thr - key), 1) with
// v_pk_sub_u16 clamp / v_pk_min_u16 / v_pk_add_u16 (three packed ops per two compares, no
// VCC round trip); the salient / padding sentinel 0xFFFF never counts (thr <= 0x8000).
typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2r __attribute__((ext_vector_type(2)));
template <int KW, int CB>
__device__ inline void rank_stage_dense16(const uint32_t* __restrict__ key, int K, int K8,
                                          const int32_t* __restrict__ sal, int S, uint16_t* kv) {
  const u32x4* k4 = (const u32x4*)key;
  const int Kq = K >> 2, Q = 2 * K8;  // u32x4 key chunks: real, staged (4 keys each)
  const int tid = threadIdx.x;
  int sv[CB];
  const int nb = (Q + 256 * CB - 1) / (256 * CB);
  for (int b = 0; b < nb; ++b) {
    const int c0 = tid + 256 * CB * b;
    u32x4 v[CB];
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const int c = c0 + 256 * u;
      v[u] = c < Kq ? k4[c] : u32x4{0u, 0u, 0u, 0u};
      if (b == 0) sv[u] = c < S ? sal[c] : -1;
    }
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const int c = c0 + 256 * u;
      if (c < Q) {
        uint32_t h[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          h[e] = c < Kq ? (KW == 2 ? v[u][e] >> 16
                                   : (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)__uint_as_float(v[u][e])))
                        : 0xFFFFu;
        ((u32x2r*)kv)[c] = u32x2r{h[0] | h[1] << 16, h[2] | h[3] << 16};
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < CB; ++u)
    if (sv[u] >= 0) kv[sv[u]] = 0xFFFFu;
  for (int c = tid + 256 * CB; c < S; c += 256) kv[sal[c]] = 0xFFFFu;
}

template <int TPO, int R>
__device__ inline void rank_owner_group16(const uint16_t* kv, int L, int K8, int g0, int sub,
                                          const RankOwnerEnt<R>& oe,
                                          int32_t* __restrict__ colsorted,
                                          uint32_t* __restrict__ lctab, const SibTables& sib) {
  uint32_t mine[R], cnt[R];
  int ochunk[R], oidx[R];
#pragma unroll
  for (int o = 0; o < R; ++o) {
    const int c = __shfl(oe.col[o], (int)(threadIdx.x & 63) & ~(TPO - 1), 64);
    oidx[o] = c >= 0 ? c : 0;
    mine[o] = kv[oidx[o]];
    ochunk[o] = oidx[o] >> 3;
  }
  const u32x4* kv8 = (const u32x4*)kv;
  const uint32_t one = 0x00010001u;
  uint32_t pk[R];
#pragma unroll
  for (int o = 0; o < R; ++o) pk[o] = 0u;
#pragma unroll 2
  for (int j8 = sub; j8 < K8; j8 += TPO) {
    const u32x4 k = kv8[j8];
#pragma unroll
    for (int o = 0; o < R; ++o) {
      const uint32_t t = j8 < ochunk[o] ? mine[o] + 1u : mine[o];
      const uint32_t thr = t | t << 16;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        // (asm: the compiler turns the builtin form back into compares + selects)
        uint32_t x;
        asm("v_pk_sub_u16 %0, %1, %2 clamp\n\tv_pk_min_u16 %0, %0, %3" : "=&v"(x) : "v"(thr), "v"(k[d]), "v"(one));
        asm("v_pk_add_u16 %0, %0, %1" : "+v"(pk[o]) : "v"(x));
      }
    }
  }
#pragma unroll
  for (int o = 0; o < R; ++o) {
    cnt[o] = (pk[o] & 0xFFFFu) + (pk[o] >> 16);
    const int oi = oidx[o];
    if (sub == (ochunk[o] % TPO))
      for (int e = 0; e < (oi & 7); ++e) cnt[o] += kv[8 * ochunk[o] + e] == mine[o] ? 1u : 0u;
#pragma unroll
    for (int w = 1; w < TPO; w <<= 1) cnt[o] += (uint32_t)__shfl_xor((int)cnt[o], w, 64);
    // (owner = column; a salient column's sentinel key writes nothing)
    if (sub == 0 && oe.col[o] >= 0 && mine[o] != 0xFFFFu) {
      colsorted[cnt[o]] = oe.col[o];
      lctab[cnt[o]] = oe.ent[o][0];
      if (sib.n > 0) sib.lctab[0][cnt[o]] = oe.ent[o][1];
      if (sib.n > 1) sib.lctab[1][cnt[o]] = oe.ent[o][2];
    }
  }
}

template <int TPO, int R, int SB, bool DENSE = false, int KW = 0>
__global__ __launch_bounds__(256) void rank_table_kernel(
    const uint32_t* __restrict__ key, const int32_t* __restrict__ nonsal, int L,
    const int32_t* __restrict__ posmap, int32_t* __restrict__ colsorted,
    uint32_t* __restrict__ lctab, int lc_len, uint32_t lc_none, SibTables sib,
    int K = 0, const int32_t* __restrict__ sal = nullptr, int S = 0) {
  extern __shared__ __attribute__((aligned(16))) uint32_t rt_kv[];  // roundup(L or K, 4 TPO)
  const int tid = threadIdx.x;
  const int L4 = (int)round_up_dev(DENSE ? K : L, (KW ? 8 : 4) * TPO) >> 2;  // u32x4 words: L4 / (KW ? 2 : 1) chunks
  const int g0 = (blockIdx.x * (256 / TPO) + tid / TPO) * R;  // this lane group's first owner
  // (DENSE: owners are the K columns, else the L list entries)
  const RankOwnerEnt<R> oe = rank_owner_ents<R, DENSE>(g0, tid % TPO, DENSE ? K : L, nonsal, posmap, sib);
  if constexpr (KW != 0)
    rank_stage_dense16<KW, 12>(key, K, L4 >> 1, sal, S, (uint16_t*)rt_kv);
  else if constexpr (DENSE)
    rank_stage_dense<12>(key, K, L4, sal, S, rt_kv);
  else
    rank_stage_keys<SB>(key, nonsal, L, L4, rt_kv);
  const int nt = gridDim.x * 256;
  for (int r = L + blockIdx.x * 256 + tid; r < lc_len; r += nt) {
    lctab[r] = pad_entry(r, L, lc_none, sal, S, posmap);
    for (int o = 0; o < sib.n; ++o) sib.lctab[o][r] = pad_entry(r, L, lc_none, sal, S, sib.posmap[o]);
  }
  __syncthreads();
  if constexpr (KW != 0)
    rank_owner_group16<TPO, R>((const uint16_t*)rt_kv, L, L4 >> 1, g0, tid % TPO, oe, colsorted, lctab, sib);
  else
    rank_owner_group<TPO, R, DENSE>(rt_kv, L, L4, g0, tid % TPO, oe, colsorted, lctab, sib);
}

// ---------------------------------------------------------------- 16-bit histogram rank
// The same stable ranks and table as rank_table_kernel's 16-bit dense path, from a histogram
// of the 15-bit f16 / bf16 key patterns instead of all-pairs compares.  Every workgroup (1024
// threads) stages all K keys (salient and padding: the 0xFFFF sentinel, never counted), counts
// them into 32768 bins (two u16 counts per LDS word, atomic adds that cannot carry across the
// halves: counts <= K <= 16384), turns the counts into exclusive bin starts (one block scan),
// scatters the columns into bin order (the same atomics return each column's slot, leaving
// every bin's END behind, so bin k starts where bin k - 1 ends), and ranks its owners:
//   rank(c) = start(key_c) + #{j in bin(key_c) : j < c}
// -- #{j : key_j < key_c} + #{j < c : key_j == key_c}, the reference's stable argsort
// (fake_quant.py:113, ties by list index = column order).  An owner's bin is scanned by TPO
// lanes; a bin holding many equal keys costs compares, never correctness.
constexpr int RH_BINS = 32768, RH_THREADS = 1024, RH_TPO = 4, RH_OWNERS = RH_THREADS / RH_TPO;

template <int KW>
__global__ __launch_bounds__(RH_THREADS) void rank_hist16_kernel(
    const uint32_t* __restrict__ key, int K, int L, const int32_t* __restrict__ posmap,
    int32_t* __restrict__ colsorted, uint32_t* __restrict__ lctab, int lc_len,
    uint32_t lc_none, SibTables sib, const int32_t* __restrict__ sal, int S) {
  extern __shared__ __attribute__((aligned(16))) uint32_t rh_lds[];
  uint32_t* hist = rh_lds;                                  // [RH_BINS / 2] u16 pairs
  uint16_t* kv = (uint16_t*)(hist + RH_BINS / 2);           // [K8] 16-bit keys
  const int K8 = (int)round_up_dev(K, 8);
  uint16_t* order = kv + K8;                                // [K8] columns in bin order
  __shared__ uint32_t wsum[RH_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = tid % RH_TPO;
  const int owner = blockIdx.x * RH_OWNERS + tid / RH_TPO;  // a column
  const RankOwnerEnt<1> oe = rank_owner_ents<1, true>(owner, sub, K, nullptr, posmap, sib);
  // ---- bins zeroed, keys staged (coalesced 16-B loads: 4 keys per load)
  for (int i = tid; i < RH_BINS / 8; i += RH_THREADS) ((u32x4*)hist)[i] = u32x4{0u, 0u, 0u, 0u};
  const int Kq = K >> 2;  // K % 4 == 0 (the launcher)
  for (int c = tid; c < K8 / 4; c += RH_THREADS) {
    const u32x4 v = c < Kq ? ((const u32x4*)key)[c] : u32x4{0u, 0u, 0u, 0u};
    uint32_t h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      h[e] = c < Kq ? (KW == 2 ? v[e] >> 16
                               : (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)__uint_as_float(v[e])))
                    : 0xFFFFu;
    ((uint2*)kv)[c] = uint2{h[0] | h[1] << 16, h[2] | h[3] << 16};
  }
  for (int r = L + blockIdx.x * RH_THREADS + tid; r < lc_len; r += gridDim.x * RH_THREADS) {
    lctab[r] = pad_entry(r, L, lc_none, sal, S, posmap);
    for (int o = 0; o < sib.n; ++o) sib.lctab[o][r] = pad_entry(r, L, lc_none, sal, S, sib.posmap[o]);
  }
  __syncthreads();
  for (int j = tid; j < S; j += RH_THREADS) kv[sal[j]] = 0xFFFFu;  // salient: never counted
  __syncthreads();
  // ---- counts
  for (int c = tid; c < K; c += RH_THREADS) {
    const uint32_t k = kv[c];
    if (k < (uint32_t)RH_BINS) atomicAdd(&hist[k >> 1], 1u << ((k & 1u) * 16u));
  }
  __syncthreads();
  // ---- exclusive bin starts: 32 bins (16 words) per thread, then across the block
  constexpr int PW = RH_BINS / 2 / RH_THREADS;  // words per thread
  uint32_t w[PW], run = 0u;
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    w[i] = hist[PW * tid + i];
    run += (w[i] & 0xFFFFu) + (w[i] >> 16);
  }
  uint32_t inc = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint32_t base = inc - run;
  for (int i = 0; i < wave; ++i) base += wsum[i];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const uint32_t lo = base, hi = base + (w[i] & 0xFFFFu);
    hist[PW * tid + i] = lo | (hi << 16);
    base = hi + (w[i] >> 16);
  }
  __syncthreads();
  // ---- columns into bin order; each bin's word half ends at the bin's end
  for (int c = tid; c < K; c += RH_THREADS) {
    const uint32_t k = kv[c];
    if (k < (uint32_t)RH_BINS) {
      const uint32_t sh = (k & 1u) * 16u;
      const uint32_t old = atomicAdd(&hist[k >> 1], 1u << sh);
      order[(old >> sh) & 0xFFFFu] = (uint16_t)c;
    }
  }
  __syncthreads();
  // ---- ranks of this workgroup's owners (TPO lanes each)
  const int c = owner < K ? owner : K - 1;
  const uint32_t mine = kv[c];
  const bool real = owner < K && mine < (uint32_t)RH_BINS;
  uint32_t cnt = 0u, lo = 0u;
  if (real) {
    auto end_of = [&](uint32_t k) { return (hist[k >> 1] >> ((k & 1u) * 16u)) & 0xFFFFu; };
    lo = mine > 0u ? end_of(mine - 1u) : 0u;
    const uint32_t hi = end_of(mine);
    for (uint32_t e = lo + sub; e < hi; e += RH_TPO) cnt += order[e] < c ? 1u : 0u;
  }
#pragma unroll
  for (int o = 1; o < RH_TPO; o <<= 1) cnt += (uint32_t)__shfl_xor((int)cnt, o, 64);
  if (sub == 0 && real) {
    const uint32_t rk = lo + cnt;
    colsorted[rk] = oe.col[0];
    lctab[rk] = oe.ent[0][0];
    if (sib.n > 0) sib.lctab[0][rk] = oe.ent[0][1];
    if (sib.n > 1) sib.lctab[1][rk] = oe.ent[0][2];
  }
}

// ---------------------------------------------------------------- bucketed rank + table
// The same stable ranks and table as rank_table_kernel with O(L * bucket) compares instead of
// O(L^2): every workgroup stages the L keys (as above), counts them into 4096 buckets by the
// key's position in the list's [min, max] key range (a monotone map, so every key of a lower
// bucket is smaller), scans the counts and scatters the list
// indices bucket by bucket (any order inside a bucket); an owner's rank is then the count of
// the lower buckets plus, inside its own bucket,
//   #{j : key_j < key_i} + #{j < i : key_j == key_i}
// (the reference's stable argsort, fake_quant.py:113), split over TPO lanes.  A skewed key
// distribution costs compares (a bucket holding every key degenerates to rank_table_kernel's
// work per owner over TPO lanes), never correctness.
constexpr int RB_BUCKETS = 4096;

template <int TPO, int SB>
__global__ __launch_bounds__(256) void rank_bucket_kernel(
    const uint32_t* __restrict__ key, const int32_t* __restrict__ nonsal, int L,
    const int32_t* __restrict__ posmap, int32_t* __restrict__ colsorted,
    uint32_t* __restrict__ lctab, int lc_len, uint32_t lc_none, SibTables sib,
    const int32_t* __restrict__ sal, int S) {
  extern __shared__ __attribute__((aligned(16))) uint32_t rb_lds[];
  const int tid = threadIdx.x;
  const int L4 = (int)round_up_dev(L, 4) >> 2;
  uint32_t* keys = rb_lds;                        // [4 L4]
  uint32_t* start = keys + 4 * L4;                // [RB_BUCKETS + 1] bucket starts
  uint32_t* fill = start + RB_BUCKETS + 4;        // [RB_BUCKETS] scatter cursors
  uint16_t* bj = (uint16_t*)(fill + RB_BUCKETS);  // [L] list indices in bucket order
  const int g0 = blockIdx.x * (256 / TPO) + tid / TPO;  // this lane group's owner
  const RankOwnerEnt<1> oe = rank_owner_ents<1>(g0, tid % TPO, L, nonsal, posmap, sib);
  for (int b = tid; b < RB_BUCKETS; b += 256) fill[b] = 0u;
  rank_stage_keys<SB>(key, nonsal, L, L4, keys);
  const int nt = gridDim.x * 256;
  for (int r = L + blockIdx.x * 256 + tid; r < lc_len; r += nt) {
    lctab[r] = pad_entry(r, L, lc_none, sal, S, posmap);
    for (int o = 0; o < sib.n; ++o) sib.lctab[o][r] = pad_entry(r, L, lc_none, sal, S, sib.posmap[o]);
  }
  __syncthreads();
  // ---- the key range (bucket = its position in [kmin, kmax], monotone in the key: column
  // maxima cluster, so fixed exponent buckets would hold most keys in a few)
  __shared__ uint32_t kmm[2][4];
  uint32_t kmn = 0xFFFFFFFFu, kmx = 0u;
  for (int j = tid; j < L; j += 256) {
    const uint32_t k = keys[j];
    kmn = k < kmn ? k : kmn;
    kmx = k > kmx ? k : kmx;
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a = (uint32_t)__shfl_xor((int)kmn, o, 64);
    const uint32_t b = (uint32_t)__shfl_xor((int)kmx, o, 64);
    kmn = a < kmn ? a : kmn;
    kmx = b > kmx ? b : kmx;
  }
  if ((tid & 63) == 0) {
    kmm[0][tid >> 6] = kmn;
    kmm[1][tid >> 6] = kmx;
  }
  __syncthreads();
  kmn = kmm[0][0];
  kmx = kmm[1][0];
#pragma unroll
  for (int w = 1; w < 4; ++w) {
    kmn = kmm[0][w] < kmn ? kmm[0][w] : kmn;
    kmx = kmm[1][w] > kmx ? kmm[1][w] : kmx;
  }
  const float bscale = (float)RB_BUCKETS / ((float)(kmx - kmn) + 1.0f);
  auto bucket = [&](uint32_t k) {
    const int b = (int)((float)(k - kmn) * bscale);
    return b < RB_BUCKETS - 1 ? b : RB_BUCKETS - 1;
  };
  // ---- bucket counts
  for (int j = tid; j < L; j += 256) atomicAdd(&fill[bucket(keys[j])], 1u);
  __syncthreads();
  // ---- exclusive scan of the counts: 16 buckets per thread, then across the 256 threads
  constexpr int PER = RB_BUCKETS / 256;
  uint32_t c[PER], run = 0u;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    c[i] = fill[PER * tid + i];
    run += c[i];
  }
  const int lane = tid & 63, wave = tid >> 6;
  uint32_t inc = run;  // inclusive scan of the per-thread totals over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)inc, o, 64);
    if (lane >= o) inc += v;
  }
  __shared__ uint32_t wtot[4];
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  uint32_t base = inc - run;
  for (int w = 0; w < wave; ++w) base += wtot[w];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    start[PER * tid + i] = base;
    fill[PER * tid + i] = base;
    base += c[i];
  }
  if (tid == 0) start[RB_BUCKETS] = (uint32_t)L;
  __syncthreads();
  // ---- list indices in bucket order
  for (int j = tid; j < L; j += 256) bj[atomicAdd(&fill[bucket(keys[j])], 1u)] = (uint16_t)j;
  __syncthreads();
  // ---- ranks: the lower buckets, then the owner's own bucket over TPO lanes
  {
    const int oi = g0 < L ? g0 : L - 1;  // whole lane groups past the list compute and discard
    const uint32_t mine = keys[oi];
    const int b = bucket(mine);
    const int lo = (int)start[b], hi = (int)start[b + 1];
    uint32_t cnt = 0u;
    for (int e = lo + tid % TPO; e < hi; e += TPO) {
      const int jj = bj[e];
      const uint32_t k = keys[jj];
      cnt += (k < mine || (k == mine && jj < oi)) ? 1u : 0u;
    }
#pragma unroll
    for (int w = 1; w < TPO; w <<= 1) cnt += (uint32_t)__shfl_xor((int)cnt, w, 64);
    cnt += (uint32_t)lo;
    if (tid % TPO == 0 && g0 < L) {
      colsorted[cnt] = oe.col[0];
      lctab[cnt] = oe.ent[0][0];
      if (sib.n > 0) sib.lctab[0][cnt] = oe.ent[0][1];
      if (sib.n > 1) sib.lctab[1][cnt] = oe.ent[0][2];
    }
  }
}

// SQMP_RANK_TABLE_OFF=1 keeps rank_count + lc_table (A/B diagnostics).
static bool rank_table_fits(int L) {
  const bool off = knob("SQMP_RANK_TABLE_OFF") != nullptr;
  return !off && L > 0 && L <= RT_MAX;
}

template <int SBV, bool DN = false, int KWV = 0>
static void rank_table_go(int tpo, int r, int grid, size_t lds, hipStream_t s,
                          const uint32_t* key, const int32_t* nonsal, int L,
                          const int32_t* posmap, int32_t* colsorted, uint32_t* lctab,
                          int lc_len, uint32_t lc_none, const SibTables& sib, int K = 0,
                          const int32_t* sal = nullptr, int S = 0) {
#define SQMP_RT(T, RR)                                                                       \
  do {                                                                                      \
    static uint64_t attr = 0; /* up to 64 KiB of keys: the dynamic-LDS limit, per device */ \
    if (first_on_device(attr))                                                              \
      (void)hipFuncSetAttribute((const void*)rank_table_kernel<T, RR, SBV, DN, KWV>,        \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 4 * RT_MAX);    \
    rank_table_kernel<T, RR, SBV, DN, KWV><<<dim3(grid), dim3(256), lds, s>>>(              \
        key, nonsal, L, posmap, colsorted, lctab, lc_len, lc_none, sib, K, sal, S);         \
  } while (0)
#define SQMP_RT_T(T)            \
  switch (r) {                  \
    case 2: SQMP_RT(T, 2); break; \
    case 4: SQMP_RT(T, 4); break; \
    default: SQMP_RT(T, 1); break; \
  }
  switch (tpo) {
    case 8: SQMP_RT_T(8); break;
    case 16: SQMP_RT_T(16); break;
    default: SQMP_RT_T(32); break;
  }
#undef SQMP_RT_T
#undef SQMP_RT
}

// the 16-bit dense rank's key kind: column maxima of f16 / bf16 data (the per_group sort
// key), else 0 (fp32 data, mean3std keys: 32-bit keys)
static int rank_key_kind(int amode, int dtype) {
  if (amode != SQMP_ACT_PER_GROUP) return 0;
  return dtype == SQMP_F16 ? 1 : dtype == SQMP_BF16 ? 2 : 0;
}

// K / sal / S (K > 0): the column count and salient list, for the dense key staging; kw: the
// key kind (rank_key_kind)
static int launch_rank_table(const uint32_t* key, const int32_t* nonsal, int L,
                             const int32_t* posmap, int32_t* colsorted, uint32_t* lctab,
                             int lc_len, uint32_t lc_none, hipStream_t s,
                             const SibTables& sib = SibTables{}, int K = 0,
                             const int32_t* sal = nullptr, int S = 0, int kw = 0) {
  // TPO lanes per group of R owners (SQMP_RT_TPO = 8 / 16 / 32 and SQMP_RT_R = 1 / 2 / 4
  // override, tuning only, read per launch)
  const char* te = knob("SQMP_RT_TPO");
  const char* re = knob("SQMP_RT_R");
  const char* be = knob("SQMP_RT_SB");
  // two owners per lane group above 8192 entries (half the workgroups staging the whole key
  // list: Llama down_proj's 10458-column prepass 61 -> 55.6 us; profiles/r03_prepass_sweep.txt)
  int tpo = L <= 2048 ? 16 : 32, r = L > 8192 ? 2 : 1, sb = 24;
  if (te && (atoi(te) == 8 || atoi(te) == 16 || atoi(te) == 32)) tpo = atoi(te);
  if (re && (atoi(re) == 1 || atoi(re) == 2 || atoi(re) == 4)) r = atoi(re);
  if (be && (atoi(be) == 8 || atoi(be) == 16 || atoi(be) == 24)) sb = atoi(be);
  // SQMP_RT_BUCKET=1: the bucketed kernel (A/B), TPO lanes per owner (SQMP_RT_BTPO, 4)
  const char* bk = knob("SQMP_RT_BUCKET");
  if (bk && atoi(bk) == 1 && L <= 65535) {
    const char* bt = knob("SQMP_RT_BTPO");
    int btpo = bt ? atoi(bt) : 4;
    if (btpo != 1 && btpo != 2 && btpo != 4 && btpo != 8 && btpo != 16) btpo = 4;
    const int bgrid = cdiv((long)L * btpo, 256L);
    const size_t blds = sizeof(uint32_t) * ((size_t)round_up(L, 4) + 2 * RB_BUCKETS + 4) +
                        sizeof(uint16_t) * (size_t)round_up(L, 2);
#define SQMP_RB(T)                                                                            \
  do {                                                                                       \
    static uint64_t battr = 0;                                                               \
    if (first_on_device(battr))                                                              \
      (void)hipFuncSetAttribute((const void*)rank_bucket_kernel<T, 24>,                      \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);     \
    rank_bucket_kernel<T, 24><<<dim3(bgrid), dim3(256), blds, s>>>(key, nonsal, L, posmap,   \
                                                                  colsorted, lctab, lc_len,  \
                                                                  lc_none, sib, sal, S);     \
  } while (0)
    switch (btpo) {
      case 1: SQMP_RB(1); break;
      case 2: SQMP_RB(2); break;
      case 8: SQMP_RB(8); break;
      case 16: SQMP_RB(16); break;
      default: SQMP_RB(4); break;
    }
#undef SQMP_RB
    SQMP_LAUNCH_CHECK();
    return SQMP_OK;
  }
  const int grid = cdiv((long)L * tpo, 256L * r);
  // every column's key staged by coalesced loads, the salient ones masked (rank_stage_dense;
  // default: down_proj's packed-order prepass 49.9 -> 47.7 us, config-2 C4 prepass 73.0 ->
  // 72.0 us, profiles/r06_ab_rank_dense.txt); SQMP_RT_DENSE=0: the list gather (A/B)
  const char* de = knob("SQMP_RT_DENSE");
  if (!(de && atoi(de) == 0) && K > 0 && K <= RT_MAX && K % 4 == 0 && (S == 0 || sal)) {
    // owners are the K columns (rank_owner_ents<R, true>)
    const int grid = cdiv((long)K * tpo, 256L * r);
    // 16-bit keys (f16 / bf16 column maxima; down_proj prepass 47.5 -> 45.2 us,
    // profiles/r05_ab_rank_k16.txt) unless SQMP_RT_K16=0 (A/B)
    const char* k16 = knob("SQMP_RT_K16");
    // the histogram rank (rank_hist16_kernel) above 8192 columns: Llama down_proj's 10458-rank
    // table 14.8 -> 10.2 us, while at 4096 columns its fixed chain (32768 bins zeroed and
    // scanned per workgroup) is slower than the all-pairs compares, 5.2-7.8 -> 7.6-9.2 us
    // (profiles/r06_ab_rank_hist.txt).  SQMP_RT_HIST=0 / 1 forces it off / on (A/B).
    const char* he = knob("SQMP_RT_HIST");
    const bool hist = he ? atoi(he) != 0 : K > 8192;
    if (kw != 0 && !(k16 && atoi(k16) == 0) && hist && K <= 16384) {
      const size_t hl = sizeof(uint32_t) * (RH_BINS / 2) + 2 * sizeof(uint16_t) * (size_t)round_up(K, 8);
      const int hgrid = cdiv(K, RH_OWNERS);
#define SQMP_RH(KWV)                                                                            \
  do {                                                                                         \
    static uint64_t hattr = 0;                                                                 \
    if (first_on_device(hattr))                                                                \
      (void)hipFuncSetAttribute((const void*)rank_hist16_kernel<KWV>,                          \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);       \
    rank_hist16_kernel<KWV><<<dim3(hgrid), dim3(RH_THREADS), hl, s>>>(                         \
        key, K, L, posmap, colsorted, lctab, lc_len, lc_none, sib, sal, S);                    \
  } while (0)
      if (kw == 2) SQMP_RH(2); else SQMP_RH(1);
#undef SQMP_RH
      SQMP_LAUNCH_CHECK();
      return SQMP_OK;
    }
    if (kw != 0 && !(k16 && atoi(k16) == 0)) {
      const size_t hlds = sizeof(uint16_t) * (size_t)round_up(K, 8 * tpo);
      if (kw == 2)
        rank_table_go<24, true, 2>(tpo, r, grid, hlds, s, key, nonsal, L, posmap, colsorted,
                                   lctab, lc_len, lc_none, sib, K, sal, S);
      else
        rank_table_go<24, true, 1>(tpo, r, grid, hlds, s, key, nonsal, L, posmap, colsorted,
                                   lctab, lc_len, lc_none, sib, K, sal, S);
      SQMP_LAUNCH_CHECK();
      return SQMP_OK;
    }
    const size_t dlds = sizeof(uint32_t) * (size_t)round_up(K, 4 * tpo);
    rank_table_go<24, true>(tpo, r, grid, dlds, s, key, nonsal, L, posmap, colsorted, lctab,
                            lc_len, lc_none, sib, K, sal, S);
    SQMP_LAUNCH_CHECK();
    return SQMP_OK;
  }
  const size_t lds = sizeof(uint32_t) * (size_t)round_up(L, 4 * tpo);
  if (sb == 8)
    rank_table_go<8>(tpo, r, grid, lds, s, key, nonsal, L, posmap, colsorted, lctab, lc_len,
                     lc_none, sib, 0, sal, S);
  else if (sb == 16)
    rank_table_go<16>(tpo, r, grid, lds, s, key, nonsal, L, posmap, colsorted, lctab, lc_len,
                     lc_none, sib, 0, sal, S);
  else
    rank_table_go<24>(tpo, r, grid, lds, s, key, nonsal, L, posmap, colsorted, lctab, lc_len,
                     lc_none, sib, 0, sal, S);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

// ---------------------------------------------------------------- wave-per-row variant
// Same arithmetic as quant_fp_kernel, but each wave owns whole rows: no block barrier on
// the per-row path, so every wave of the CU streams its own rows (next row prefetched
// into registers while this one is quantized).  RCH = 16-B row chunks per lane
// (K * esize <= RCH * 1 KiB), VCH = 8-position output chunks per lane (P <= VCH * 512).
// The block (4 waves) shares the entry table and the salient column list.
// H2 (fp32, SQMP_OUT_H2): the row is written as the two f16 planes of sqmp_gemm_h2d's
// operand (out: planes [2][ldr][P + S_pad], hplane = ldr (P + S_pad) halves) with its exponent
// in aexp[m]; the exponent needs max |x_hat| of the row before any value is stored, and that
// is known from the statistics: |code * s| is monotone in |t| within a scale group, so the
// group's largest output is fast_code(gmax, s) * s (the row's: that of the row maximum), and
// the salient tail adds its own maximum.
template <class DT, int MODE, int RCH, int VCH, bool H2 = false>
__global__ __launch_bounds__(256) void quant_fp_wave_kernel(
    const typename DT::T* __restrict__ x, int M, int K, int q_max, int nga,
    const u32x4* __restrict__ ent_g, int P, const int32_t* __restrict__ nonsal, int Kn,
    const int32_t* __restrict__ sal, int S, int S_pad, const uint32_t* __restrict__ cmax,
    typename DT::T* __restrict__ out, int* __restrict__ aexp = nullptr, size_t hplane = 0) {
  static_assert(!H2 || DT::id == SQMP_F32, "the two-plane output is of fp32 rows");
  typedef typename DT::T T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_w[];
  const int NCH = P / 8;
  const int W = P + S_pad, WCH = W / 8;
  const int rowb = (int)round_up_dev(K * (int)sizeof(T), 16);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  u32x4* ent = (u32x4*)smem_w;                                   // [2][NCH]
  uint16_t* salc = (uint16_t*)(ent + 2 * NCH);                   // S_pad
  unsigned char* wbase = (unsigned char*)(salc + round_up_dev(S_pad, 8));
  const int wbytes = rowb + (int)round_up_dev(12 * nga, 16);
  T* row = (T*)(wbase + wave * wbytes);                          // this wave's row
  float2* scr = (float2*)((unsigned char*)row + rowb);           // nga
  uint32_t* gmax = (uint32_t*)(scr + nga);                       // nga

  // ---- the call's entry table (build_ent_kernel): one coalesced copy
  for (int c = tid; c < 2 * NCH; c += 256) ent[c] = ent_g[c];
  for (int j = tid; j < S_pad; j += 256) salc[j] = j < S ? (uint16_t)sal[j] : (uint16_t)0xFFFFu;
  float s_all = 0.f, r_all = 0.f;
  if (MODE == MODE_TENSOR) {
    float m = 0.f;
    for (int i = lane; i < Kn; i += 64) m = fmaxf(m, __uint_as_float(cmax[nonsal[i]]));
    m = wave_max(m);
    s_all = group_scale<DT>(m, q_max);
    r_all = 1.0f / s_all;
  }
  __syncthreads();  // tables complete; row buffers are the waves' own

  constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-B row chunk
  const int nch = K / EPC;
  const int wstride = gridDim.x * 4;
  u32x4 nxt[RCH];
  auto load_row = [&](int mm) {
    const u32x4* src = (const u32x4*)(x + (size_t)mm * K);
#pragma unroll
    for (int i = 0; i < RCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) nxt[i] = src[c];
    }
  };
  int m = blockIdx.x * 4 + wave;
  if (m < M) load_row(m);
  for (; m < M; m += wstride) {
#pragma unroll
    for (int i = 0; i < RCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) ((u32x4*)row)[c] = nxt[i];
    }
    if (m + wstride < M) load_row(m + wstride);
    if (MODE == MODE_GROUP)
      for (int g = lane; g < nga; g += 64) gmax[g] = 0u;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // ---- gather pass
    T vals[VCH][8];
    float lmax = 0.f;
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = lane + 64 * i;
      if (c < NCH) {
        const u32x4 e0 = ent[c], e1 = ent[NCH + c];
        const uint32_t e[8] = {e0[0], e0[1], e0[2], e0[3], e1[0], e1[1], e1[2], e1[3]};
        T v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t g = e[j] >> 16;
          v[j] = g != G_ZERO ? row[e[j] & 0xFFFFu] : DT::from_f(0.f);
          const float a = fabsf(DT::to_f(v[j]));
          if (MODE == MODE_GROUP) {
            if (g != G_ZERO && a > 0.f) atomicMax(&gmax[g], __float_as_uint(a));
          } else {
            lmax = fmaxf(lmax, a);
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[i][j] = v[j];
      }
    }
    float s_row = s_all, r_row = r_all;
    float ym = 0.f;  // H2: max |x_hat| of the row
    if (MODE == MODE_TOKEN) {
      const float rm = wave_max(lmax);
      s_row = group_scale<DT>(rm, q_max);
      r_row = 1.0f / s_row;
      if (H2) ym = fast_code<DT>(rm, s_row, r_row) * s_row;
    } else if (MODE == MODE_GROUP) {
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      for (int g = lane; g < nga; g += 64) {
        const float gm = __uint_as_float(gmax[g]);
        const float sg = group_scale<DT>(gm, q_max);
        scr[g] = make_float2(sg, 1.0f / sg);
        if (H2) ym = fmaxf(ym, fast_code<DT>(gm, sg, 1.0f / sg) * sg);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    } else if (H2) {
      ym = fast_code<DT>(wave_max(lmax), s_row, r_row) * s_row;
    }
    int eh = 0;
    if constexpr (H2) {
      for (int j = lane; j < S; j += 64) ym = fmaxf(ym, fabsf(DT::to_f(row[salc[j]])));
      eh = row_exp_of(wave_max(ym));
      if (lane == 0) aexp[m] = eh;
    }
    // ---- quantize from registers, 16-B stores
    T* o = out + (size_t)m * W;
    uint16_t* oh = (uint16_t*)out + (size_t)m * W;
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = lane + 64 * i;
      if (c < NCH) {
        const u32x4 e0 = ent[c], e1 = ent[NCH + c];
        const uint32_t e[8] = {e0[0], e0[1], e0[2], e0[3], e1[0], e1[1], e1[2], e1[3]};
        const T* v = vals[i];
        T r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t g = e[j] >> 16;
          float y = 0.f;
          if (g != G_ZERO) {
            const float2 sr = MODE == MODE_GROUP ? scr[g] : make_float2(s_row, r_row);
            const float t = DT::to_f(v[j]);
            y = __builtin_copysignf(fast_code<DT>(t, sr.x, sr.y) * sr.x, t);  // -0.0 as the reference
          }
          r[j] = DT::from_f(y);
        }
        if constexpr (H2) {
          store_h2x8(oh + 8 * c, hplane, (const float*)r, eh);
        } else {
#pragma unroll
          for (int h = 0; h < 8 / EPC; ++h) ((u32x4*)o)[(8 / EPC) * c + h] = ((const u32x4*)r)[h];
        }
      }
    }
    for (int c = NCH + lane; c < WCH; c += 64) {
      T r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t k = salc[(c - NCH) * 8 + j];
        r[j] = k != 0xFFFFu ? row[k] : DT::from_f(0.f);
      }
      if constexpr (H2) {
        store_h2x8(oh + 8 * c, hplane, (const float*)r, eh);
      } else {
#pragma unroll
        for (int h = 0; h < 8 / EPC; ++h) ((u32x4*)o)[(8 / EPC) * c + h] = ((const u32x4*)r)[h];
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // row / gmax reuse
  }
}


// ---------------------------------------------------------------- fp32 rows, any length
// One wave per row, the row staged in LDS (K * 4 bytes per wave), the call's entry table
// read from global memory (chunk-major planes of build_ent_kernel, L2-resident), two
// gathers from LDS (statistics, then quantize) instead of values held in registers, so
// rows of any length that fits LDS run at full occupancy of what fits.  OUT_FP writes the
// packed-order x_hat + exact salient tail; INPLACE (the output quantizer, P == K) writes
// the row back over itself, G_ZERO positions (salient columns) passing through.
// H2: the two f16 planes + row exponent of quant_fp_wave_kernel<..., H2>
template <int MODE, bool INPLACE, bool H2 = false>
__global__ __launch_bounds__(256) void quant_f32w_kernel(
    float* __restrict__ x, int M, int K, int q_max, int nga, const u32x4* __restrict__ ent,
    int P, const int32_t* __restrict__ nonsal, int Kn, const int32_t* __restrict__ sal,
    int S, int S_pad, const uint32_t* __restrict__ cmax, float* __restrict__ out,
    int* __restrict__ aexp = nullptr, size_t hplane = 0) {
  static_assert(!(H2 && INPLACE), "the two-plane output is the GEMM operand");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_f32w[];
  const int NCH = P / 8;
  const int W = INPLACE ? K : P + S_pad, WCH = W / 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  const int wbytes = (int)round_up_dev(4 * K, 16) + (int)round_up_dev(12 * nga, 16);
  float* row = (float*)(smem_f32w + wave * wbytes);
  float2* scr = (float2*)(row + round_up_dev(K, 4));
  uint32_t* gmax = (uint32_t*)(scr + nga);
  float s_all = 0.f, r_all = 0.f;
  if (MODE == MODE_TENSOR) {
    float m = 0.f;
    for (int i = lane; i < Kn; i += 64) m = fmaxf(m, __uint_as_float(cmax[nonsal[i]]));
    m = wave_max(m);
    s_all = group_scale<F32>(m, q_max);
    r_all = 1.0f / s_all;
  }
  const int nch4 = K / 4;
  for (int m = blockIdx.x * nwave + wave; m < M; m += gridDim.x * nwave) {
    // the whole row by LDS-DMA (1 KiB per wave instruction, all in flight at once: one
    // memory latency per row instead of one per register batch); the tail chunks (K % 256)
    // through registers
    const u32x4* src = (const u32x4*)(x + (size_t)m * K);
    const int nfull = nch4 & ~63;
    for (int c = 0; c < nfull; c += 64)
      __builtin_amdgcn_global_load_lds((const void*)(src + c + lane),
                                       (__attribute__((address_space(3))) void*)(row + 4 * c),
                                       16, 0, 0);
    if (nfull + lane < nch4) ((u32x4*)row)[nfull + lane] = src[nfull + lane];
    if (MODE == MODE_GROUP)
      for (int g = lane; g < nga; g += 64) gmax[g] = 0u;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // entry-table chunks are loaded EB per lane at once (global / L2 latency once per
    // batch, not once per chunk)
    constexpr int EB = 8;
    u32x4 ea[EB], eb[EB];
    auto load_ent = [&](int c0) {
#pragma unroll
      for (int b = 0; b < EB; ++b) {
        const int c = c0 + 64 * b;
        if (c < NCH) {
          ea[b] = ent[c];
          eb[b] = ent[NCH + c];
        }
      }
    };
    float lmax = 0.f;
    for (int c0 = lane; c0 < NCH; c0 += 64 * EB) {
      load_ent(c0);
#pragma unroll
      for (int b = 0; b < EB; ++b) {
        if (c0 + 64 * b >= NCH) break;
        const uint32_t e[8] = {ea[b][0], ea[b][1], ea[b][2], ea[b][3],
                               eb[b][0], eb[b][1], eb[b][2], eb[b][3]};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t g = e[j] >> 16;
          if (g == G_ZERO) continue;
          const float a = fabsf(row[e[j] & 0xFFFFu]);
          if (MODE == MODE_GROUP) {
            if (a > 0.f) atomicMax(&gmax[g], __float_as_uint(a));
          } else {
            lmax = fmaxf(lmax, a);
          }
        }
      }
    }
    float s_row = s_all, r_row = r_all;
    float ym = 0.f;  // H2: max |x_hat| of the row (see quant_fp_wave_kernel)
    if (MODE == MODE_TOKEN) {
      const float rm = wave_max(lmax);
      s_row = group_scale<F32>(rm, q_max);
      r_row = 1.0f / s_row;
      if (H2) ym = fast_code<F32>(rm, s_row, r_row) * s_row;
    } else if (MODE == MODE_GROUP) {
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      for (int g = lane; g < nga; g += 64) {
        const float gm = __uint_as_float(gmax[g]);
        const float sg = group_scale<F32>(gm, q_max);
        scr[g] = make_float2(sg, 1.0f / sg);
        if (H2) ym = fmaxf(ym, fast_code<F32>(gm, sg, 1.0f / sg) * sg);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    } else if (H2) {
      ym = fast_code<F32>(wave_max(lmax), s_row, r_row) * s_row;
    }
    int eh = 0;
    if constexpr (H2) {
      for (int j = lane; j < S; j += 64) ym = fmaxf(ym, fabsf(row[sal[j]]));
      eh = row_exp_of(wave_max(ym));
      if (lane == 0) aexp[m] = eh;
    }
    float* o = (INPLACE ? x : out) + (size_t)m * W;
    uint16_t* oh = (uint16_t*)out + (size_t)m * W;
    for (int c0 = lane; c0 < NCH; c0 += 64 * EB) {
      load_ent(c0);
#pragma unroll
      for (int b = 0; b < EB; ++b) {
        const int c = c0 + 64 * b;
        if (c >= NCH) break;
        const uint32_t e[8] = {ea[b][0], ea[b][1], ea[b][2], ea[b][3],
                               eb[b][0], eb[b][1], eb[b][2], eb[b][3]};
        float r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t g = e[j] >> 16;
          if (g == G_ZERO) {
            r[j] = INPLACE ? row[8 * c + j] : 0.f;
          } else {
            const float2 sr = MODE == MODE_GROUP ? scr[g] : make_float2(s_row, r_row);
            const float t = row[e[j] & 0xFFFFu];
            r[j] = __builtin_copysignf(fast_code<F32>(t, sr.x, sr.y) * sr.x, t);
          }
        }
        if constexpr (H2) {
          store_h2x8(oh + 8 * c, hplane, r, eh);
        } else {
          ((u32x4*)o)[2 * c] = ((const u32x4*)r)[0];
          ((u32x4*)o)[2 * c + 1] = ((const u32x4*)r)[1];
        }
      }
    }
    if (!INPLACE) {
      for (int c = NCH + lane; c < WCH; c += 64) {
        float r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = (c - NCH) * 8 + j;
          r[j] = i < S ? row[sal[i]] : 0.f;
        }
        if constexpr (H2) {
          store_h2x8(oh + 8 * c, hplane, r, eh);
        } else {
          ((u32x4*)o)[2 * c] = ((const u32x4*)r)[0];
          ((u32x4*)o)[2 * c + 1] = ((const u32x4*)r)[1];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // row / gmax reuse
  }
}

template <int MODE, bool INPLACE, bool H2 = false>
static int quant_f32w_launch(void* x, int M, int K, int q_max, int nga, const uint32_t* ent,
                             int P, const int32_t* nonsal, int Kn, const int32_t* sal, int S,
                             int S_pad, const uint32_t* cmax, void* out, hipStream_t s,
                             int* aexp = nullptr, size_t hplane = 0) {
  const size_t wb = (size_t)round_up(4L * K, 16) + (size_t)round_up(12L * nga, 16);
  int nw = (int)((160 * 1024) / wb);
  if (nw < 1) return SQMP_EUNSUPPORTED;
  nw = nw > 4 ? 4 : nw;
  const size_t lds = nw * wb;
  SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)quant_f32w_kernel<MODE, INPLACE, H2>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int per_cu = (int)((160 * 1024) / lds);
  int grid = 256 * (per_cu < 1 ? 1 : per_cu);
  if (grid > cdiv(M, nw)) grid = cdiv(M, nw);
  quant_f32w_kernel<MODE, INPLACE, H2><<<dim3(grid), dim3(64 * nw), lds, s>>>(
      (float*)x, M, K, q_max, nga, (const u32x4*)ent, P, nonsal, Kn, sal, S, S_pad, cmax,
      (float*)out, aexp, hplane);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

static size_t quant_fp_wave_lds_bytes(int K, int P, int nga, int S_pad, int esize) {
  // entry table + salient list + 4 per-wave (row, scales, group max) regions
  const size_t wb = (size_t)round_up((long)K * esize, 16) + (size_t)round_up(12L * nga, 16);
  return 4 * (size_t)P + 2 * (size_t)round_up(S_pad, 8) + 4 * wb;
}

static size_t quant_fp_lds_bytes(int K, int P, int nga, int S_pad, int esize) {
  return (size_t)round_up((long)K * esize, 16) + 4 * (size_t)P + (size_t)round_up(2L * K, 16) +
         12 * (size_t)nga + 2 * (size_t)round_up(S_pad, 8) + 64;
}

static size_t quant_lds_bytes(int K, int P, int nga, int esize) {
  return (size_t)round_up((long)K * esize, 16) + 4 * (size_t)P + (size_t)round_up(2L * K, 16) +
         8 * (size_t)nga + 64;
}

template <class DT, int MODE, int OUT>
static int quant_launch(void* x, int M, int K, int q_max, int G, int nga, const int32_t* amap,
                        int P, const int32_t* nonsal, int Kn, const int32_t* sal, int S,
                        int S_pad, const int32_t* rank, const uint32_t* cmax, void* out,
                        void* out_scale, void* out_xs, hipStream_t s) {
  typedef typename DT::T T;
  const size_t lds = quant_lds_bytes(K, P, nga, sizeof(T));
  if (lds > 160 * 1024) return SQMP_EUNSUPPORTED;
  SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)quant_act_kernel<DT, MODE, OUT>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  per_cu = per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu);
  int grid = 256 * per_cu;
  if (grid > M) grid = M;
  quant_act_kernel<DT, MODE, OUT><<<dim3(grid), dim3(256), lds, s>>>(
      (T*)x, M, K, q_max, G, nga, amap, P, nonsal, Kn, sal, S, S_pad, rank, cmax, out,
      (float*)out_scale, (T*)out_xs);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT, int MODE, int RCH, int VCH, bool H2 = false>
static int quant_fpw_launch(void* x, int M, int K, int q_max, int nga, const uint32_t* ent, int P,
                            const int32_t* nonsal, int Kn, const int32_t* sal, int S, int S_pad,
                            const uint32_t* cmax, void* out, size_t lds, hipStream_t s,
                            int* aexp = nullptr, size_t hplane = 0) {
  typedef typename DT::T T;
  SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)quant_fp_wave_kernel<DT, MODE, RCH, VCH, H2>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  per_cu = per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu);
  int grid = 256 * per_cu;
  if (grid > cdiv(M, 4)) grid = cdiv(M, 4);
  quant_fp_wave_kernel<DT, MODE, RCH, VCH, H2><<<dim3(grid), dim3(256), lds, s>>>(
      (const T*)x, M, K, q_max, nga, (const u32x4*)ent, P, nonsal, Kn, sal, S, S_pad, cmax,
      (T*)out, aexp, hplane);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT, int MODE>
static int quant_fp_launch(void* x, int M, int K, int q_max, int G, int nga, const int32_t* amap,
                           int P, const int32_t* nonsal, int Kn, const int32_t* sal, int S,
                           int S_pad, const int32_t* rank, const uint32_t* cmax, void* out,
                           size_t lds, hipStream_t s) {
  typedef typename DT::T T;
  SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)quant_fp_kernel<DT, MODE>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  per_cu = per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu);
  int grid = 256 * per_cu;
  if (grid > M) grid = M;
  quant_fp_kernel<DT, MODE><<<dim3(grid), dim3(256), lds, s>>>(
      (const T*)x, M, K, q_max, G, nga, amap, P, nonsal, Kn, sal, S, S_pad, rank, cmax, (T*)out);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT>
static int quant_dispatch(void* x, int M, int K, int amode, int q_max, int G, int nga,
                          const int32_t* amap, int P, const int32_t* nonsal, int Kn,
                          const int32_t* sal, int S, int S_pad, const int32_t* rank,
                          const uint32_t* cmax, const uint32_t* ent, int out_kind, void* out,
                          void* out_scale, void* out_xs, hipStream_t s) {
#define SQMP_Q(MODE, OUTK)                                                                  \
  quant_launch<DT, MODE, OUTK>(x, M, K, q_max, G, nga, amap, P, nonsal, Kn, sal, S, S_pad, \
                               rank, cmax, out, out_scale, out_xs, s)
  const int mode = amode == SQMP_ACT_PER_TOKEN    ? MODE_TOKEN
                   : amode == SQMP_ACT_PER_TENSOR ? MODE_TENSOR
                                                  : MODE_GROUP;
  if constexpr (DT::id == SQMP_F32) {
    // the two-plane operand of sqmp_gemm_h2d (planes [2][roundup(M, 128)][P + S_pad], row
    // exponents in out_scale): the wave kernel up to 4096 columns, else quant_f32w_kernel
    if (out_kind == SQMP_OUT_H2) {
      if (!ent || K % 8 != 0 || P % 8 != 0 || ((uintptr_t)x) % 16 != 0 || ((uintptr_t)out) % 16 != 0)
        return SQMP_EUNSUPPORTED;
      const size_t hplane = (size_t)round_up(M, 128) * (P + S_pad);
      int* aexp = (int*)out_scale;
      if (K <= 4096 && P <= 4096) {
        const size_t lds = quant_fp_wave_lds_bytes(K, P, nga, S_pad, sizeof(float));
        if (lds <= 160 * 1024) {
          const bool sm = K <= 2048 && P <= 2048;
#define SQMP_QH(MODE)                                                                          \
  (sm ? quant_fpw_launch<DT, MODE, 8, 4, true>(x, M, K, q_max, nga, ent, P, nonsal, Kn, sal, S,  \
                                               S_pad, cmax, out, lds, s, aexp, hplane)        \
      : quant_fpw_launch<DT, MODE, 16, 8, true>(x, M, K, q_max, nga, ent, P, nonsal, Kn, sal, S, \
                                                S_pad, cmax, out, lds, s, aexp, hplane))
          if (mode == MODE_TOKEN) return SQMP_QH(MODE_TOKEN);
          if (mode == MODE_TENSOR) return SQMP_QH(MODE_TENSOR);
          return SQMP_QH(MODE_GROUP);
#undef SQMP_QH
        }
      }
#define SQMP_QH(MODE)                                                                           \
  quant_f32w_launch<MODE, false, true>(x, M, K, q_max, nga, ent, P, nonsal, Kn, sal, S, S_pad, cmax, \
                                       out, s, aexp, hplane)
      return mode == MODE_TOKEN ? SQMP_QH(MODE_TOKEN)
           : mode == MODE_TENSOR ? SQMP_QH(MODE_TENSOR) : SQMP_QH(MODE_GROUP);
#undef SQMP_QH
    }
    // fp32 rows longer than the register-staged wave kernel holds, and the in-place output
    // quantizer: one wave per row from LDS (quant_f32w_kernel)
    if (ent && K % 8 == 0 && P % 8 == 0 && (((uintptr_t)x) % 16 == 0) &&
        ((out_kind == SQMP_OUT_FP && (K > 4096 || P > 4096) && ((uintptr_t)out) % 16 == 0) ||
         out_kind == SQMP_OUT_INPLACE)) {
#define SQMP_QF32(MODE, INP)                                                                  \
  quant_f32w_launch<MODE, INP>(x, M, K, q_max, nga, ent, P, nonsal, Kn, sal, S, S_pad, cmax, out, s)
      int st32;
      if (out_kind == SQMP_OUT_INPLACE)
        st32 = mode == MODE_TOKEN ? SQMP_QF32(MODE_TOKEN, true)
             : mode == MODE_TENSOR ? SQMP_QF32(MODE_TENSOR, true) : SQMP_QF32(MODE_GROUP, true);
      else
        st32 = mode == MODE_TOKEN ? SQMP_QF32(MODE_TOKEN, false)
             : mode == MODE_TENSOR ? SQMP_QF32(MODE_TENSOR, false) : SQMP_QF32(MODE_GROUP, false);
#undef SQMP_QF32
      if (st32 != SQMP_EUNSUPPORTED) return st32;
    }
    // fp32 rows on the wave kernel (RCH = 16-B row chunks = 2 VCH): K, P <= 4096
    if (ent && out_kind == SQMP_OUT_FP && K % 8 == 0 && K <= 4096 && P <= 4096 &&
        (((uintptr_t)x) % 16 == 0)) {
      const size_t lds = quant_fp_wave_lds_bytes(K, P, nga, S_pad, sizeof(typename DT::T));
      if (lds <= 160 * 1024) {
        const bool sm = K <= 2048 && P <= 2048;
#define SQMP_QW32(MODE)                                                                        \
  (sm ? quant_fpw_launch<DT, MODE, 8, 4>(x, M, K, q_max, nga, ent, P, nonsal, Kn, sal, S, S_pad, \
                                         cmax, out, lds, s)                                   \
      : quant_fpw_launch<DT, MODE, 16, 8>(x, M, K, q_max, nga, ent, P, nonsal, Kn, sal, S,     \
                                          S_pad, cmax, out, lds, s))
        if (mode == MODE_TOKEN) return SQMP_QW32(MODE_TOKEN);
        if (mode == MODE_TENSOR) return SQMP_QW32(MODE_TENSOR);
        return SQMP_QW32(MODE_GROUP);
#undef SQMP_QW32
      }
    }
  }
  if constexpr (DT::id != SQMP_F32) {
  if (ent && out_kind == SQMP_OUT_FP && K % 8 == 0 && K <= 12288 && P <= 12288 &&
      (((uintptr_t)x) % 16 == 0)) {
    const size_t lds = quant_fp_wave_lds_bytes(K, P, nga, S_pad, sizeof(typename DT::T));
    if (lds <= 160 * 1024) {
      const int sz = (K <= 4096 && P <= 4096) ? 0 : (K <= 8192 && P <= 8192) ? 1 : 2;
#define SQMP_QW1(MODE, R)                                                                   \
  quant_fpw_launch<DT, MODE, R, R>(x, M, K, q_max, nga, ent, P, nonsal, Kn, sal, S, S_pad, cmax, \
                                   out, lds, s)
#define SQMP_QW(MODE) \
  (sz == 0 ? SQMP_QW1(MODE, 8) : sz == 1 ? SQMP_QW1(MODE, 16) : SQMP_QW1(MODE, 24))
      if (mode == MODE_TOKEN) return SQMP_QW(MODE_TOKEN);
      if (mode == MODE_TENSOR) return SQMP_QW(MODE_TENSOR);
      return SQMP_QW(MODE_GROUP);
#undef SQMP_QW
#undef SQMP_QW1
    }
  }
  if (out_kind == SQMP_OUT_FP && K % 8 == 0 && K * 2 <= PFC_FP * 256 * 16 &&
      P <= FCH * 256 * 8 && (((uintptr_t)x) % 16 == 0)) {
    const size_t lds = quant_fp_lds_bytes(K, P, nga, S_pad, sizeof(typename DT::T));
    if (lds <= 160 * 1024) {
#define SQMP_QF(MODE)                                                                         \
  quant_fp_launch<DT, MODE>(x, M, K, q_max, G, nga, amap, P, nonsal, Kn, sal, S, S_pad, rank, \
                            cmax, out, lds, s)
      if (mode == MODE_TOKEN) return SQMP_QF(MODE_TOKEN);
      if (mode == MODE_TENSOR) return SQMP_QF(MODE_TENSOR);
      return SQMP_QF(MODE_GROUP);
#undef SQMP_QF
    }
  }
  }
  if (out_kind == SQMP_OUT_FP) {
    if (mode == MODE_TOKEN) return SQMP_Q(MODE_TOKEN, SQMP_OUT_FP);
    if (mode == MODE_TENSOR) return SQMP_Q(MODE_TENSOR, SQMP_OUT_FP);
    return SQMP_Q(MODE_GROUP, SQMP_OUT_FP);
  }
  if (mode == MODE_TOKEN) return SQMP_Q(MODE_TOKEN, SQMP_OUT_INPLACE);
  if (mode == MODE_TENSOR) return SQMP_Q(MODE_TENSOR, SQMP_OUT_INPLACE);
  return SQMP_Q(MODE_GROUP, SQMP_OUT_INPLACE);
#undef SQMP_Q
}

}  // namespace sqmp

using namespace sqmp;

// Workspace: cmax u32 [K64] | rank_by_col i32 [K64] | rank partials i32 [tiles][K64] |
// entry table u32 [Kp64] | lane-contiguous table u32 [roundup(K, 4096)] | rank counts
// i32 [K64] | sorted column list i32 [K64] | fp64 column sums [2][K64] (mean + 3 sigma).
// Without SQMP_QA_CLEAN_WS only what a call reads before writing is cleared per call.
static size_t ws_k64(int K) { return (size_t)round_up(K > 0 ? K : 1, 64); }
static size_t ws_u32_words(int K, int Kp) {
  const size_t k64 = ws_k64(K);
  return k64 * (4 + (size_t)rank_tiles(K)) + (size_t)round_up(Kp > K ? Kp : K, 64) +
         (size_t)round_up(K > 0 ? K : 1, 4096);
}
// + the two sibling tables of sqmp_quant_act_group (round_up(K, 4096) words each) at the end
static size_t ws_sib_offset(int K, int Kp) {
  return sizeof(uint32_t) * ws_u32_words(K, Kp) + 2 * sizeof(double) * ws_k64(K);
}
extern "C" size_t sqmp_act_workspace_bytes(int M, int K, int Kp) {
  (void)M;
  return ws_sib_offset(K, Kp) + 2 * sizeof(uint32_t) * (size_t)round_up(K > 0 ? K : 1, 4096);
}

static int quant_act_impl(void* x, int dtype, int M, int K, int amode, int n_bits,
                          int group_size, const int32_t* amap, int Kp, const int32_t* nonsal,
                          const int32_t* salient, int S, int S_pad, const int32_t* posmap,
                          int flags, int out_kind, void* out, void* out_scale, void* out_xs,
                          void* workspace, size_t ws_bytes, void* stream, const C4Weight* cw);

extern "C" int sqmp_quant_act_v2(void* x, int dtype, int M, int K, int amode, int n_bits,
                                 int group_size, const int32_t* amap, int Kp,
                                 const int32_t* nonsal, const int32_t* salient, int S,
                                 int S_pad, const int32_t* posmap, int flags, int out_kind,
                                 void* out, void* out_scale, void* out_xs, void* workspace,
                                 size_t ws_bytes, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  return quant_act_impl(x, dtype, M, K, amode, n_bits, group_size, amap, Kp, nonsal, salient, S,
                        S_pad, posmap, flags, out_kind, out, out_scale, out_xs, workspace,
                        ws_bytes, stream, nullptr);
}

static int quant_act_impl(void* x, int dtype, int M, int K, int amode, int n_bits,
                          int group_size, const int32_t* amap, int Kp, const int32_t* nonsal,
                          const int32_t* salient, int S, int S_pad, const int32_t* posmap,
                          int flags, int out_kind, void* out, void* out_scale, void* out_xs,
                          void* workspace, size_t ws_bytes, void* stream, const C4Weight* cw) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype < SQMP_F32 || dtype > SQMP_BF16 || M < 0 || K <= 0 || K > 65000) return SQMP_EINVAL;
  if (amode < SQMP_ACT_PER_TOKEN || amode > SQMP_ACT_PER_GROUP_MEAN3STD) return SQMP_EINVAL;
  if (n_bits < 2 || n_bits > 8) return SQMP_EUNSUPPORTED;
  if (S < 0 || S > K || !x || !amap || (K - S > 0 && !nonsal)) return SQMP_EINVAL;
  if (flags & ~(SQMP_QA_CLEAN_WS | SQMP_QA_REUSE_STATS | SQMP_QA_STATS_GIVEN | SQMP_QA_TILED |
                SQMP_QA_TILED4 | SQMP_QA_TABLE_READY | SQMP_QA_WRITE_X))
    return SQMP_EINVAL;
  if ((flags & SQMP_QA_WRITE_X) && out_kind != SQMP_OUT_F8) return SQMP_EINVAL;
  if ((flags & (SQMP_QA_TILED | SQMP_QA_TILED4)) && out_kind != SQMP_OUT_C4)
    return SQMP_EINVAL;
  // column maxima already in the workspace (written by sqmp_gemm_fq_colmax's epilogue)
  const bool stats_given = (flags & SQMP_QA_STATS_GIVEN) != 0;
  if (stats_given && (out_kind != SQMP_OUT_INPLACE ||
                      (amode != SQMP_ACT_PER_GROUP && amode != SQMP_ACT_PER_TENSOR)))
    return SQMP_EINVAL;
  if (out_kind == SQMP_OUT_INPLACE) {
    if (Kp != K) return SQMP_EINVAL;
  } else if (out_kind == SQMP_OUT_C4) {
    if (Kp < K || Kp % 128 != 0 || S_pad < S || S_pad % 64 != 0 || !out || !out_scale) return SQMP_EINVAL;
    if ((S > 0 && (!salient || !out_xs)) || !posmap) return SQMP_EINVAL;
    if (n_bits > 4 || (amode != SQMP_ACT_PER_GROUP && amode != SQMP_ACT_PER_GROUP_UNSORTED &&
                       amode != SQMP_ACT_PER_GROUP_MEAN3STD) ||
        group_size % 64 != 0)
      return SQMP_EUNSUPPORTED;
  } else if (out_kind == SQMP_OUT_FP || out_kind == SQMP_OUT_F8 ||
             out_kind == SQMP_OUT_H2) {
    if (Kp < K || Kp % 128 != 0 || S_pad < S || S_pad % 64 != 0 || !out) return SQMP_EINVAL;
    if (out_kind == SQMP_OUT_H2 && (dtype != SQMP_F32 || !out_scale)) return SQMP_EINVAL;
    if (out_kind == SQMP_OUT_F8) {
      if (!out_scale || (S_pad > 0 && !out_xs)) return SQMP_EINVAL;
      // e4m3 holds every integer code up to 16 exactly, e2m3 up to 7; one scale per row
      if (n_bits > 4 || (amode != SQMP_ACT_PER_TOKEN && amode != SQMP_ACT_PER_TENSOR))
        return SQMP_EUNSUPPORTED;
    }
    if (S > 0 && !salient) return SQMP_EINVAL;
  } else {
    return SQMP_EINVAL;
  }
  const bool group = amode == SQMP_ACT_PER_GROUP || amode == SQMP_ACT_PER_GROUP_UNSORTED ||
                     amode == SQMP_ACT_PER_GROUP_MEAN3STD;
  if (group && (group_size <= 0 || group_size > 65000)) return SQMP_EINVAL;
  if (M == 0) return SQMP_OK;
  if (ws_bytes < sqmp_act_workspace_bytes(M, K, Kp) || !workspace) return SQMP_EWORKSPACE;
  const bool clean = (flags & SQMP_QA_CLEAN_WS) != 0;
  const size_t k64 = ws_k64(K);
  uint32_t* cmax = (uint32_t*)workspace;
  int32_t* rank = (int32_t*)(cmax + k64);
  int32_t* part = rank + k64;
  uint32_t* ent = (uint32_t*)(part + k64 * (size_t)rank_tiles(K));
  uint32_t* lctab = ent + round_up(Kp > K ? Kp : K, 64);
  int32_t* counts = (int32_t*)(lctab + round_up(K, 4096));
  int32_t* colsorted = counts + k64;
  double* sums = (double*)((uint32_t*)workspace + ws_u32_words(K, Kp));
  const int Kn = K - S;
  if (Kn == 0) {
    // every channel salient: the reference skips quantization entirely (:299)
    if (out_kind == SQMP_OUT_INPLACE) return SQMP_OK;
  }
  int st;
  const bool sorted = amode == SQMP_ACT_PER_GROUP || amode == SQMP_ACT_PER_GROUP_MEAN3STD;
  const int q_max = (1 << (n_bits - 1)) - 1;
  // SQMP_DISABLE_LC=1 selects the previous row kernels (A/B timing diagnostics only)
  const bool lc_off = knob("SQMP_DISABLE_LC") != nullptr;
  const bool use_lc = out_kind == SQMP_OUT_FP && !lc_off &&
                      quant_lc_supported(dtype, M, K, group, group_size, Kn, Kp, S_pad, x, out);
  const int lmode = group ? 2 : amode == SQMP_ACT_PER_TENSOR ? 1 : 0;
  const uint32_t lc_none = (uint32_t)(Kp + S_pad) | ((uint32_t)(Kp + S_pad + 1) << 16);
  const int lc_len = (int)round_up(K, 4096);

  // ---- lane-contiguous quantizer: statistics, then the rank-ordered (column, position)
  // table -- one rank_table launch for lists up to RT_MAX, else rank_count + lc_table; no
  // memsets in the clean-workspace protocol, only the table when statistics are reused.
  auto lc_prepare = [&](const int32_t* pm, uint32_t none, bool reuse,
                        uint32_t*& key_clear) -> int {
    key_clear = nullptr;
    int tmode = TAB_LIST;
    if (sorted) {
      if (reuse) {
        tmode = TAB_SORTED;
      } else {
        tmode = TAB_COUNTS;
        int st2;
        if (amode == SQMP_ACT_PER_GROUP) {
          if (stats_given) {
            st2 = SQMP_OK;
          } else {
            if (!clean) SQMP_HIP_CHECK(hipMemsetAsync(cmax, 0, sizeof(uint32_t) * k64, s));
            st2 = launch_colmax(x, dtype, M, K, cmax, s, false);
          }
        } else {
          st2 = launch_colkey_mean3std(x, dtype, M, K, sums, cmax, s, clean);
        }
        if (st2) return st2;
        if (rank_table_fits(Kn)) {
          key_clear = cmax;  // cleared by the quantizer, after every rank_table read
          return launch_rank_table(cmax, nonsal, Kn, pm, colsorted, lctab, lc_len, none, s,
                                   SibTables{}, K, salient, S, rank_key_kind(amode, dtype));
        }
        if (!clean) SQMP_HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int32_t) * k64, s));
        st2 = launch_rank_count(cmax, nonsal, Kn, counts, s);
        if (st2) return st2;
      }
    }
    // (SQMP_QA_TABLE_READY: the list table of a previous call is still in place)
    if (tmode == TAB_LIST && (flags & SQMP_QA_TABLE_READY)) return SQMP_OK;
    const int nthr = K > Kn ? K : (Kn > 0 ? Kn : 1);
    lc_table_kernel<<<dim3(cdiv(nthr, 256)), dim3(256), 0, s>>>(
        tmode, nonsal, Kn, K, pm, counts, colsorted, tmode == TAB_COUNTS ? cmax : nullptr,
        lctab, lc_len, none, salient, S);
    SQMP_LAUNCH_CHECK();
    return SQMP_OK;
  };

  // e4m3 codes for the f8 GEMM and x_hat over x in one pass (SQMP_QA_WRITE_X: per_token, no
  // salient column, identity packed order)
  if (out_kind == SQMP_OUT_F8 && (flags & SQMP_QA_WRITE_X)) {
    if (amode != SQMP_ACT_PER_TOKEN || S != 0 || Kp != K || lc_off) return SQMP_EUNSUPPORTED;
    return launch_token_rows(dtype, x, M, K, q_max, s, (unsigned char*)out, (float*)out_scale);
  }
  // e4m3 codes for the f8 GEMM (token / tensor scales): list-order table, lc
  // quantizer
  if (out_kind == SQMP_OUT_F8) {
    if (!posmap || lc_off || !quant_lc_supported(dtype, M, K, false, 0, Kn, Kp, S_pad, x, out) ||
        ((uintptr_t)out_xs) % 16 != 0)
      return SQMP_EUNSUPPORTED;
    if (amode == SQMP_ACT_PER_TENSOR) {
      if (!clean) SQMP_HIP_CHECK(hipMemsetAsync(cmax, 0, sizeof(uint32_t) * k64, s));
      st = launch_colmax(x, dtype, M, K, cmax, s, false);
      if (st) return st;
    }
    pos_table_kernel<<<dim3(cdiv(lc_len, 256)), dim3(256), 0, s>>>(amap, Kp, lctab, lc_len, lc_none);
    SQMP_LAUNCH_CHECK();
    st = launch_quant_lc(dtype, amode == SQMP_ACT_PER_TENSOR ? 1 : 0, x, M, K, q_max, 1, lctab,
                         Kn, amap, Kp, salient, S, S_pad, cmax, nonsal, out, nullptr, 0, s,
                         (float*)out_scale, out_xs);
    if (st) return st;
    // the per-tensor maximum was read by every workgroup: clear it after the launch
    if (clean && amode == SQMP_ACT_PER_TENSOR)
      SQMP_HIP_CHECK(hipMemsetAsync(cmax, 0, sizeof(uint32_t) * k64, s));
    return SQMP_OK;
  }

  // act-order int4 codes (the sqmp_gemm_fqt operand): the OUT_FP fast path's table, codes
  // written straight from the quantizing lanes
  if (out_kind == SQMP_OUT_C4) {
    if (Kn == 0 || lc_off || !quant_lc_supported(dtype, M, K, true, group_size, Kn, Kp, S_pad, x, out) ||
        ((uintptr_t)out_xs) % 16 != 0)
      return SQMP_EUNSUPPORTED;
    uint32_t* kc;
    st = lc_prepare(posmap, lc_none, (flags & SQMP_QA_REUSE_STATS) != 0, kc);
    if (st) return st;
    return launch_quant_lc_c4(dtype, x, M, K, q_max, group_size, lctab, Kn, Kp, salient, S,
                              S_pad, cmax, nonsal, out, out_scale,
                              (flags & SQMP_QA_TILED4) ? -(int)(cdiv(Kn, group_size) * 8 + 4)
                              : (flags & SQMP_QA_TILED) ? -(int)(cdiv(Kn, group_size) * 8 + 2)
                                                        : (int)round_up(M, 256),
                              out_xs, kc, (int)k64, s, cw);
  }

  // fast path: the table maps ranks straight to packed positions (per-weight posmap)
  if (use_lc && posmap && amode != SQMP_ACT_PER_TENSOR) {
    uint32_t* kc;
    st = lc_prepare(posmap, lc_none, (flags & SQMP_QA_REUSE_STATS) != 0, kc);
    if (st) return st;
    // (amap NULL: the table's pad entries zero the salient positions, pad_entry)
    return launch_quant_lc(dtype, lmode, x, M, K, q_max, group_size, lctab, Kn, nullptr, Kp,
                           salient, S, S_pad, cmax, nonsal, out, kc, (int)k64, s);
  }

  // ---- in-place per-token quantization without salient columns: one row-pair pass, no
  // table (launch_token_rows).  The list table is still left in the workspace (unless it is
  // there already: SQMP_QA_TABLE_READY), so that a later unsorted in-place call may skip it.
  if (out_kind == SQMP_OUT_INPLACE && amode == SQMP_ACT_PER_TOKEN && S == 0 && !lc_off &&
      (dtype == SQMP_F16 || dtype == SQMP_BF16) && K % 8 == 0 && ((uintptr_t)x) % 16 == 0) {
    if (!(flags & SQMP_QA_TABLE_READY)) {
      lc_table_kernel<<<dim3(cdiv(K, 256)), dim3(256), 0, s>>>(
          TAB_LIST, nonsal, Kn, K, nullptr, counts, colsorted, nullptr, lctab, lc_len,
          (uint32_t)K | ((uint32_t)(K + 1) << 16), salient, S);
      SQMP_LAUNCH_CHECK();
    }
    return launch_token_rows(dtype, x, M, K, q_max, s);
  }

  // ---- in-place output quantization (fake_quant.py:308-316) on the same kernels: the
  // "packed" order is the identity, salient columns keep their values (no zeroing, no
  // tail), and the row is written back over itself.
  if (out_kind == SQMP_OUT_INPLACE && !lc_off && amode != SQMP_ACT_PER_TENSOR &&
      quant_lc_supported(dtype, M, K, group, group_size, Kn, K, 0, x, x)) {
    uint32_t* kc;
    st = lc_prepare(nullptr, (uint32_t)K | ((uint32_t)(K + 1) << 16), false, kc);
    if (st) return st;
    return launch_quant_lc(dtype, lmode, x, M, K, q_max, group_size, lctab, Kn, nullptr, K,
                           salient, 0, 0, cmax, nonsal, x, kc, (int)k64, s);
  }

  // ---- fp32 rows (OUT_FP, and the in-place output quantizer): the lane-contiguous
  // pipeline's statistics and rank table (clean workspace, no memsets), the entry table
  // scattered from it in one launch, the fp32 wave quantizers
  const bool h2 = out_kind == SQMP_OUT_H2;
  if (dtype == SQMP_F32 && !lc_off && Kn > 0 && amode != SQMP_ACT_PER_TENSOR && K % 8 == 0 &&
      (((uintptr_t)x) % 16 == 0) &&
      (((out_kind == SQMP_OUT_FP || h2) && posmap && Kp % 8 == 0 && ((uintptr_t)out) % 16 == 0) ||
       out_kind == SQMP_OUT_INPLACE) &&
      (out_kind == SQMP_OUT_FP || h2 || clean)) {
    const bool inplace = out_kind == SQMP_OUT_INPLACE;
    const int P = inplace ? K : Kp;
    const size_t wb = (size_t)round_up(4L * K, 16) + (size_t)round_up(12L * (group ? cdiv(Kn, group_size) : 1), 16);
    if (wb <= 160 * 1024) {
      uint32_t* kc;
      const uint32_t none = inplace ? (uint32_t)K | ((uint32_t)(K + 1) << 16) : lc_none;
      st = lc_prepare(inplace ? nullptr : posmap, none,
                      !inplace && (flags & SQMP_QA_REUSE_STATS) != 0, kc);
      if (st) return st;
      const int nthr = P > Kn ? P : Kn;
      const int cw = kc ? (int)k64 : 0;
      ent_from_lctab_kernel<<<dim3(cdiv(nthr > cw ? nthr : cw, 256)), dim3(256), 0, s>>>(
          lctab, Kn, amap, P, group ? group_size : (1 << 30), ent, kc, cw);
      SQMP_LAUNCH_CHECK();
      const int nga = group ? cdiv(Kn, group_size) : 1;
      return quant_dispatch<F32>(x, M, K, amode, q_max, group_size, nga, amap, P, nonsal, Kn,
                                 salient, S, S_pad, nullptr, cmax, ent, out_kind, out,
                                 out_scale, out_xs, s);
    }
  }

  if (h2) return SQMP_EUNSUPPORTED;  // the two-plane output: the fp32 wave kernels only

  // (the in-place list table is left in the workspace by every in-place call of an unsorted
  // per-row / per-group mode, whichever path quantizes, so that a caller's
  // SQMP_QA_TABLE_READY on the next such call never finds a stale table)
  if (out_kind == SQMP_OUT_INPLACE && !sorted && amode != SQMP_ACT_PER_TENSOR &&
      !(flags & SQMP_QA_TABLE_READY)) {
    const int nthr = K > Kn ? K : (Kn > 0 ? Kn : 1);
    lc_table_kernel<<<dim3(cdiv(nthr, 256)), dim3(256), 0, s>>>(
        TAB_LIST, nonsal, Kn, K, nullptr, counts, colsorted, nullptr, lctab, lc_len,
        (uint32_t)K | ((uint32_t)(K + 1) << 16), salient, S);
    SQMP_LAUNCH_CHECK();
  }

  // ---- general path (fp32, 8-bit int output, large rows, other group sizes)
  // SQMP_QA_REUSE_STATS: the rank partials of the previous call on this workspace (a
  // sibling layer on the same input, same K / Kp / salient set) are still in place
  const bool reuse_part = sorted && (flags & SQMP_QA_REUSE_STATS) != 0;
  if ((amode == SQMP_ACT_PER_TENSOR || amode == SQMP_ACT_PER_GROUP) && !stats_given && !reuse_part) {
    SQMP_HIP_CHECK(hipMemsetAsync(cmax, 0, sizeof(uint32_t) * k64, s));
    st = launch_colmax(x, dtype, M, K, cmax, s, false);
    if (st) return st;
  } else if (amode == SQMP_ACT_PER_GROUP_MEAN3STD && !reuse_part) {
    st = launch_colkey_mean3std(x, dtype, M, K, sums, cmax, s, clean);
    if (st) return st;
  }
  if (sorted && !reuse_part) {
    st = launch_rank_partial(cmax, nonsal, Kn, (int)k64, part, s);
    if (st) return st;
  }
  // entry table (read by the wave kernel) and rank_by_col (read by the block kernels)
  const int mode_e = group ? MODE_GROUP : MODE_TOKEN;
  const int Pe = out_kind == SQMP_OUT_INPLACE ? K : Kp;
  const bool need_ent = (out_kind == SQMP_OUT_FP || (out_kind == SQMP_OUT_INPLACE && dtype == SQMP_F32)) &&
                        Pe % 8 == 0;
  if (need_ent || sorted || use_lc) {
    build_ent_kernel<<<dim3(cdiv(Pe, 256)), dim3(256), 0, s>>>(
        amap, Pe, nonsal, Kn, sorted ? part : nullptr, rank_tiles(Kn), (int)k64, mode_e,
        group ? group_size : 1, need_ent && !use_lc ? ent : nullptr, sorted ? rank : nullptr,
        use_lc ? lctab : nullptr, lc_len, lc_none, sorted ? colsorted : nullptr);
    SQMP_LAUNCH_CHECK();
  }
  if (use_lc) {
    st = launch_quant_lc(dtype, lmode, x, M, K, q_max, group_size, lctab, Kn, amap, Kp,
                         salient, S, S_pad, cmax, nonsal, out, nullptr, 0, s);
  } else {
    const int nga = group ? (Kn > 0 ? cdiv(Kn, group_size) : 1) : 1;
    const int32_t* rk = sorted ? rank : nullptr;
    const uint32_t* entp = need_ent ? ent : nullptr;
    switch (dtype) {
      case SQMP_F32:
        st = quant_dispatch<F32>(x, M, K, amode, q_max, group_size, nga, amap, Kp, nonsal, Kn,
                                 salient, S, S_pad, rk, cmax, entp, out_kind, out, out_scale,
                                 out_xs, s);
        break;
      case SQMP_F16:
        st = quant_dispatch<F16>(x, M, K, amode, q_max, group_size, nga, amap, Kp, nonsal, Kn,
                                 salient, S, S_pad, rk, cmax, entp, out_kind, out, out_scale,
                                 out_xs, s);
        break;
      default:
        st = quant_dispatch<BF16>(x, M, K, amode, q_max, group_size, nga, amap, Kp, nonsal, Kn,
                                  salient, S, S_pad, rk, cmax, entp, out_kind, out, out_scale,
                                  out_xs, s);
    }
  }
  if (st) return st;
  // the general path leaves the column keys behind: restore the clean-workspace invariant
  if (clean && (amode == SQMP_ACT_PER_TENSOR || sorted))
    SQMP_HIP_CHECK(hipMemsetAsync(cmax, 0, sizeof(uint32_t) * k64, s));
  return SQMP_OK;
}

extern "C" int sqmp_quant_act(void* x, int dtype, int M, int K, int amode, int n_bits,
                              int group_size, const int32_t* amap, int Kp,
                              const int32_t* nonsal, const int32_t* salient, int S, int S_pad,
                              int out_kind, void* out, void* out_scale, void* out_xs,
                              void* workspace, size_t ws_bytes, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  return sqmp_quant_act_v2(x, dtype, M, K, amode, n_bits, group_size, amap, Kp, nonsal,
                           salient, S, S_pad, nullptr, 0, out_kind, out, out_scale, out_xs,
                           workspace, ws_bytes, stream);
}

// ---------------------------------------------------------------- act-order weight (C4)
static const uint32_t* ws_lctab(const void* workspace, int K, int Kp) {
  const size_t k64 = ws_k64(K);
  return (const uint32_t*)workspace + k64 * (2 + (size_t)rank_tiles(K)) +
         (size_t)round_up(Kp > K ? Kp : K, 64);
}

extern "C" int sqmp_perm_weight_c4(const void* workspace, int K, int Kp, int S, int S_pad,
                                   const void* codes, const void* wscale, const void* wsal,
                                   int dtype, int N, int Gw, int ngw, void* wp, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!workspace || !codes || !wscale || !wp || (S > 0 && !wsal)) return SQMP_EINVAL;
  if (K <= 0 || S < 0 || S >= K || Kp < K || Kp % 128 || S_pad < S || S_pad % 64 || N <= 0 ||
      Gw <= 0 || ngw <= 0)
    return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (Gw % 8 || Kp > 32768) return SQMP_EUNSUPPORTED;
  return launch_perm_weight_c4(dtype, ws_lctab(workspace, K, Kp), codes, wscale, wsal, N, Kp,
                               Gw, ngw, K - S, S_pad, wp, (hipStream_t)stream);
}

extern "C" int sqmp_quant_act_c4(void* x, int dtype, int M, int K, int amode, int n_bits,
                                 int group_size, const int32_t* amap, int Kp,
                                 const int32_t* nonsal, const int32_t* salient, int S,
                                 int S_pad, const int32_t* posmap, int flags, void* acodes,
                                 void* ascale, void* xs, const void* codes, const void* wscale,
                                 const void* wsal, int N, int Gw, int ngw, void* wp,
                                 void* workspace, size_t ws_bytes, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!codes || !wscale || !wp || (S > 0 && !wsal) || N <= 0 || Gw <= 0 || ngw <= 0)
    return SQMP_EINVAL;
  if (Gw % 8 || Kp > 32768) return SQMP_EUNSUPPORTED;
  const C4Weight cw{codes, wscale, wsal, wp, N, Kp, Gw, ngw};
  return quant_act_impl(x, dtype, M, K, amode, n_bits, group_size, amap, Kp, nonsal, salient, S,
                        S_pad, posmap, flags, SQMP_OUT_C4, acodes, ascale, xs, workspace,
                        ws_bytes, stream, &cw);
}

// ---------------------------------------------------------------- sibling layers (group)
// One quantizer pass for a layer and up to two siblings that quantize the same input with the
// same salient set and sorted per_group mode (q/k/v, gate/up): the statistics and the rank
// once, the rank tables of every sibling from the same launch, and every sibling's OUT_FP
// operand written from the same quantized values (each in its own packed order).  Every
// output equals what sqmp_quant_act_v2(SQMP_OUT_FP) writes for that sibling, bit for bit.
extern "C" int sqmp_quant_act_group(void* x, int dtype, int M, int K, int amode, int n_bits,
                                    int group_size, int nout, const int32_t* const* amaps,
                                    const int32_t* const* posmaps, int Kp, const int32_t* nonsal,
                                    const int32_t* salient, int S, int S_pad, int flags,
                                    void* const* outs, void* workspace, size_t ws_bytes,
                                    void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (nout < 1 || nout > 3 || !amaps || !posmaps || !outs) return SQMP_EINVAL;
  for (int o = 0; o < nout; ++o)
    if (!amaps[o] || !posmaps[o] || !outs[o]) return SQMP_EINVAL;
  if (nout == 1)
    return sqmp_quant_act_v2(x, dtype, M, K, amode, n_bits, group_size, amaps[0], Kp, nonsal,
                             salient, S, S_pad, posmaps[0], flags, SQMP_OUT_FP, outs[0], nullptr,
                             nullptr, workspace, ws_bytes, stream);
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (amode != SQMP_ACT_PER_GROUP && amode != SQMP_ACT_PER_GROUP_MEAN3STD) return SQMP_EUNSUPPORTED;
  if (flags != SQMP_QA_CLEAN_WS) return SQMP_EUNSUPPORTED;
  if (M < 0 || K <= 0 || K > 65000 || S < 0 || S >= K || !x || !nonsal || (S > 0 && !salient))
    return SQMP_EINVAL;
  if (n_bits < 2 || n_bits > 8) return SQMP_EUNSUPPORTED;
  if (Kp < K || Kp % 128 != 0 || S_pad < S || S_pad % 64 != 0) return SQMP_EINVAL;
  const int Kn = K - S;
  if (!rank_table_fits(Kn)) return SQMP_EUNSUPPORTED;
  for (int o = 0; o < nout; ++o)
    if (!quant_lc_supported(dtype, M, K, true, group_size, Kn, Kp, S_pad, x, outs[o]))
      return SQMP_EUNSUPPORTED;
  if (group_size < 16) return SQMP_EUNSUPPORTED;
  // the quantizer's LDS: one region of Kp + S_pad + 8 words per output, at most two (a third
  // output reuses the second) + the salient list and masks (checked before any launch: a
  // refusal after the statistics pass would leave the workspace dirty)
  if ((size_t)4 * ((Kp + S_pad + 8) * (nout < 2 ? nout : 2) + S_pad + 2 * ((Kp + 63) / 64)) > 150 * 1024)
    return SQMP_EUNSUPPORTED;
  if (M == 0) return SQMP_OK;
  if (ws_bytes < sqmp_act_workspace_bytes(M, K, Kp) || !workspace) return SQMP_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const size_t k64 = ws_k64(K);
  uint32_t* cmax = (uint32_t*)workspace;
  int32_t* rank = (int32_t*)(cmax + k64);
  int32_t* part = rank + k64;
  uint32_t* ent = (uint32_t*)(part + k64 * (size_t)rank_tiles(K));
  uint32_t* lctab = ent + round_up(Kp > K ? Kp : K, 64);
  int32_t* counts = (int32_t*)(lctab + round_up(K, 4096));
  int32_t* colsorted = counts + k64;
  double* sums = (double*)((uint32_t*)workspace + ws_u32_words(K, Kp));
  uint32_t* sibtab = (uint32_t*)((unsigned char*)workspace + ws_sib_offset(K, Kp));
  const int lc_len = (int)round_up(K, 4096);
  const uint32_t lc_none = (uint32_t)(Kp + S_pad) | ((uint32_t)(Kp + S_pad + 1) << 16);
  SibTables st;
  LcSib ls;
  st.n = ls.n = nout - 1;
  for (int o = 0; o + 1 < nout; ++o) {
    st.posmap[o] = posmaps[o + 1];
    st.lctab[o] = sibtab + (size_t)o * lc_len;
    ls.tab[o] = st.lctab[o];
    ls.amap[o] = amaps[o + 1];
    ls.out[o] = outs[o + 1];
  }
  int r = amode == SQMP_ACT_PER_GROUP ? launch_colmax(x, dtype, M, K, cmax, s, false)
                                      : launch_colkey_mean3std(x, dtype, M, K, sums, cmax, s, true);
  if (r) return r;
  r = launch_rank_table(cmax, nonsal, Kn, posmaps[0], colsorted, lctab, lc_len, lc_none, s, st, K,
                        salient, S, rank_key_kind(amode, dtype));
  if (r) return r;
  // (amap NULL: the tables' pad entries zero the salient positions, pad_entry)
  return launch_quant_lc_group(dtype, x, M, K, (1 << (n_bits - 1)) - 1, group_size, lctab, Kn,
                               nullptr, Kp, salient, S, S_pad, cmax, nonsal, outs[0], cmax,
                               (int)k64, ls, s);
}
