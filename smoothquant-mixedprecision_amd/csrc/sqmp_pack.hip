// Offline weight quantization + packing: W4A4Linear.from_float
// (/root/reference/smoothquant/fake_quant.py:324-371).
//
//   column absmax over all N rows (salient columns included, as the reference quantizes
//   module.weight before restoring them, :347-365)  -> stable rank (:164-173)
//   -> index maps -> one workgroup per output row: per-(row, group) absmax over the packed
//   (sorted) K axis, scale D(D(clamp(max,1e-5))/q_max), code rne(D(w/s)) (:188-193), nibble
//   packing, and the exact salient columns (:347, :363-365) in a dense side slice.
#include "sqmp_internal.h"

namespace sqmp {

// float-reciprocal floor division, exact for 0 <= r < 2^24, 0 < G < 2^16 after the fixup
__device__ inline int fdiv_floor(int r, int G, float invG) {
  int q = (int)((float)r * invG);
  if ((q + 1) * G <= r) ++q;
  if (q * G > r) --q;
  return q;
}

template <class DT, int WBITS>
__global__ __launch_bounds__(256) void pack_rows_kernel(
    const typename DT::T* __restrict__ w, int N, int K, int Kp, int Gw, int ngw, int q_max,
    int per_tensor, const int32_t* __restrict__ perm, const int32_t* __restrict__ amap,
    const uint32_t* __restrict__ cmax, const int32_t* __restrict__ sal, int S, int S_pad,
    uint32_t* __restrict__ codes, typename DT::T* __restrict__ wscale,
    typename DT::T* __restrict__ wsal) {
  extern __shared__ __attribute__((aligned(16))) float smem_pack[];
  float* row = smem_pack;                       // K values of this row (as fp32, exact)
  uint32_t* gmax = (uint32_t*)(row + K);        // ngw group absmax (float bits)
  float* sc = (float*)(gmax + ngw);             // ngw scales
  float* red = sc + ngw;                        // 16 floats for block reductions
  const int n = blockIdx.x, tid = threadIdx.x;
  const typename DT::T* wr = w + (size_t)n * K;
  for (int k = tid; k < K; k += 256) row[k] = DT::to_f(wr[k]);
  for (int g = tid; g < ngw; g += 256) gmax[g] = 0u;
  __syncthreads();
  if (per_tensor) {
    // fake_quant.py:22 `w.abs().max()` -- global, from the column maxima
    float m = 0.f;
    for (int k = tid; k < K; k += 256) m = fmaxf(m, __uint_as_float(cmax[k]));
    m = block_max(m, red);
    if (tid == 0) gmax[0] = __float_as_uint(m);
  } else {
    const int Ptot = ngw * Gw;  // positions covered by groups (zero padding included)
    const bool wave_groups = (Gw % 64) == 0;
    for (int base = 0; base < Ptot; base += 256) {
      const int p = base + tid;
      float v = 0.f;
      if (p < Ptot && p < Kp) {
        const int k = perm[p];
        if (k >= 0) v = fabsf(row[k]);
      }
      if (wave_groups) {
        v = wave_max(v);
        const int pw = base + (tid & ~63);
        if ((tid & 63) == 0 && pw < Ptot && v > 0.f) atomicMax(&gmax[pw / Gw], __float_as_uint(v));
      } else if (p < Ptot && v > 0.f) {
        atomicMax(&gmax[p / Gw], __float_as_uint(v));
      }
    }
  }
  __syncthreads();
  for (int g = tid; g < ngw; g += 256) {
    const float s = WBITS == 0 ? 1.f : group_scale<DT>(__uint_as_float(gmax[per_tensor ? 0 : g]), q_max);
    sc[g] = s;
    wscale[(size_t)g * pad_n(N) + n] = DT::from_f(s);  // [ngw][Np]
  }
  __syncthreads();
  const float invG = 1.0f / (float)Gw;
  if (WBITS == 0) {
    // no weight quantization: dense D values in packed order (salient / pad -> 0)
    typename DT::T* dense = (typename DT::T*)codes + (size_t)n * Kp;
    for (int p = tid; p < Kp; p += 256) {
      const int k = amap[p];
      dense[p] = DT::from_f(k >= 0 ? row[k] : 0.f);
    }
  } else if (WBITS == 4) {
    const int nw = Kp / 8;  // 8 nibbles per 32-bit word, bpack order (sqmp_common.h)
    for (int wi = tid; wi < nw; wi += 256) {
      uint32_t word = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int p = bpack_pos(wi, e);
        const int k = amap[p];
        int c = 0;
        if (k >= 0) c = (int)quant_code<DT>(row[k], sc[fdiv_floor(p, Gw, invG)]);
        word |= (uint32_t)(c + 8) << bpack_shift(p);
      }
      codes[(size_t)n * nw + wi] = word;
    }
  } else {
    const int nw = Kp / 4;  // 4 int8 codes per word
    for (int wi = tid; wi < nw; wi += 256) {
      uint32_t word = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int p = wi * 4 + e;
        const int k = amap[p];
        int c = 0;
        if (k >= 0) c = (int)quant_code<DT>(row[k], sc[fdiv_floor(p, Gw, invG)]);
        word |= ((uint32_t)c & 0xFFu) << (8 * e);
      }
      codes[(size_t)n * nw + wi] = word;
    }
  }
  for (int j = tid; j < S_pad; j += 256)
    wsal[(size_t)n * S_pad + j] = DT::from_f(j < S ? row[sal[j]] : 0.f);
}

template <class DT, int WBITS>
static int pack_rows_launch(const void* w, int N, int K, int Kp, int Gw, int ngw, int q_max,
                            int per_tensor, const int32_t* perm, const int32_t* amap,
                            const uint32_t* cmax, const int32_t* sal, int S, int S_pad,
                            void* codes, void* wscale, void* wsal, hipStream_t s) {
  typedef typename DT::T T;
  const size_t lds = sizeof(float) * ((size_t)K + 2 * (size_t)ngw + 16);
  if (lds > 160 * 1024) return SQMP_EUNSUPPORTED;
  SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)pack_rows_kernel<DT, WBITS>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  pack_rows_kernel<DT, WBITS><<<dim3(N), dim3(256), lds, s>>>(
      (const T*)w, N, K, Kp, Gw, ngw, q_max, per_tensor, perm, amap, cmax, sal, S, S_pad,
      (uint32_t*)codes, (T*)wscale, (T*)wsal);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

// ------------------------------------------------------------------ dequant (W_hat)
template <class DT, int WBITS>
__global__ __launch_bounds__(256) void dequant_kernel(
    const uint8_t* __restrict__ codes, const typename DT::T* __restrict__ wscale,
    const typename DT::T* __restrict__ wsal, const int32_t* __restrict__ amap,
    const int32_t* __restrict__ sal, int N, int K, int S, int Kp, int Gw, int ngw, int S_pad,
    typename DT::T* __restrict__ w_hat) {
  const long total = (long)N * Kp;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int n = (int)(idx / Kp), p = (int)(idx % Kp);
    const int k = amap[p];
    if (k < 0) continue;
    if (WBITS == 0) {
      w_hat[(size_t)n * K + k] = ((const typename DT::T*)codes)[(size_t)n * Kp + p];
      continue;
    }
    int c;
    if (WBITS == 4) {
      const uint32_t wd = ((const uint32_t*)codes)[(size_t)n * (Kp / 8) + bpack_dword(p)];
      c = (int)((wd >> bpack_shift(p)) & 0xFu) - 8;
    } else {
      c = (int)(int8_t)codes[(size_t)n * Kp + p];
    }
    const float s = DT::to_f(wscale[(size_t)(p / Gw) * pad_n(N) + n]);
    w_hat[(size_t)n * K + k] = DT::from_f((float)c * s);  // fake_quant.py:193 mul_ in D
  }
  const long tsal = (long)N * S;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < tsal; idx += (long)gridDim.x * 256) {
    const int n = (int)(idx / S), j = (int)(idx % S);
    w_hat[(size_t)n * K + sal[j]] = wsal[(size_t)n * S_pad + j];  // :363-365
  }
}

// W_hat in PACKED order [N][Kp] (salient / padding positions 0): the dense B operand of
// sqmp_gemm_fq when groups are finer than one 16-B chunk (e.g. group_size 4).
template <class DT, int WBITS>
__global__ __launch_bounds__(256) void dequant_packed_kernel(
    const uint8_t* __restrict__ codes, const typename DT::T* __restrict__ wscale, int N,
    int Kp, int Gw, int ngw, typename DT::T* __restrict__ out) {
  const long total = (long)N * Kp;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int n = (int)(idx / Kp), p = (int)(idx % Kp);
    int c;
    if (WBITS == 4) {
      const uint32_t wd = ((const uint32_t*)codes)[(size_t)n * (Kp / 8) + bpack_dword(p)];
      c = (int)((wd >> bpack_shift(p)) & 0xFu) - 8;
    } else {
      c = (int)(int8_t)codes[(size_t)n * Kp + p];
    }
    const int g = min(p / Gw, ngw - 1);
    out[idx] = DT::from_f((float)c * DT::to_f(wscale[(size_t)g * pad_n(N) + n]));
  }
}

template <class DT, int WBITS>
static int dequant_packed_launch(const void* codes, const void* wscale, int N, int Kp, int Gw,
                                 int ngw, void* out, hipStream_t s) {
  typedef typename DT::T T;
  const long total = (long)N * Kp;
  const int grid = (int)std::min<long>(4096, (total + 255) / 256);
  dequant_packed_kernel<DT, WBITS><<<dim3(grid > 0 ? grid : 1), dim3(256), 0, s>>>(
      (const uint8_t*)codes, (const T*)wscale, N, Kp, Gw, ngw, (T*)out);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT, int WBITS>
static int dequant_launch(const void* codes, const void* wscale, const void* wsal,
                          const int32_t* amap, const int32_t* sal, int N, int K, int S,
                          int Kp, int Gw, int ngw, int S_pad, void* w_hat, hipStream_t s) {
  typedef typename DT::T T;
  const long total = (long)N * Kp;
  const int grid = (int)std::min<long>(4096, (total + 255) / 256);
  dequant_kernel<DT, WBITS><<<dim3(grid > 0 ? grid : 1), dim3(256), 0, s>>>(
      (const uint8_t*)codes, (const T*)wscale, (const T*)wsal, amap, sal, N, K, S, Kp, Gw,
      ngw, S_pad, (T*)w_hat);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace sqmp

using namespace sqmp;

extern "C" int sqmp_weight_geometry(int K, int S, int wmode, int group_size, int* Kp,
                                    int* Gw, int* ngw, int* S_pad) {
  if (K <= 0 || K > 65000 || S < 0 || S > K) return SQMP_EINVAL;
  int kp, gw, ng;
  if (wmode == SQMP_W_PER_GROUP || wmode == SQMP_W_PER_GROUP_UNSORTED ||
      wmode == SQMP_W_PER_GROUP_MEAN3STD) {
    if (group_size <= 0 || group_size > 65000) return SQMP_EINVAL;
    ng = cdiv(K, group_size);
    gw = group_size;
    kp = (int)round_up((long)ng * group_size, 128);
  } else if (wmode == SQMP_W_PER_CHANNEL || wmode == SQMP_W_PER_TENSOR ||
             wmode == SQMP_W_NONE) {
    kp = (int)round_up(K, 128);
    gw = kp;
    ng = 1;
  } else {
    return SQMP_EINVAL;
  }
  if (kp > 65000) return SQMP_EUNSUPPORTED;
  if (Kp) *Kp = kp;
  if (Gw) *Gw = gw;
  if (ngw) *ngw = ng;
  if (S_pad) *S_pad = (int)round_up(S, 64);  // the GEMMs' dense stages are 32 / 64 wide
  return SQMP_OK;
}

// Workspace: key u32 [K64] | rank i32 [K64] | fp64 column sums [2][K64] (mean + 3 sigma).
extern "C" size_t sqmp_pack_workspace_bytes(int N, int K) {
  (void)N;
  return (2 * sizeof(uint32_t) + 2 * sizeof(double)) * (size_t)round_up(K > 0 ? K : 1, 64);
}

extern "C" int sqmp_pack_weight(const void* w, int dtype, int N, int K, int wmode,
                                int n_bits, int group_size, const int32_t* salient, int S,
                                void* codes, void* wscale, void* wsal, int32_t* perm,
                                int32_t* amap, int32_t* amap_fq, int32_t* nonsal,
                                void* workspace, size_t ws_bytes, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  hipStream_t s = (hipStream_t)stream;
  if (dtype < SQMP_F32 || dtype > SQMP_BF16 || N <= 0) return SQMP_EINVAL;
  if (wmode == SQMP_W_NONE) n_bits = 0;
  else if (n_bits != 4 && n_bits != 8) return SQMP_EUNSUPPORTED;
  int Kp, Gw, ngw, S_pad;
  int st = sqmp_weight_geometry(K, S, wmode, group_size, &Kp, &Gw, &ngw, &S_pad);
  if (st != SQMP_OK) return st;
  if (!w || !codes || !wscale || !perm || !amap || !amap_fq || !nonsal) return SQMP_EINVAL;
  if (S > 0 && (!salient || !wsal)) return SQMP_EINVAL;
  if (ws_bytes < sqmp_pack_workspace_bytes(N, K) || !workspace) return SQMP_EWORKSPACE;
  uint32_t* cmax = (uint32_t*)workspace;
  int32_t* rank = (int32_t*)((char*)workspace + sizeof(uint32_t) * round_up(K, 64));
  double* sums = (double*)((char*)workspace + 2 * sizeof(uint32_t) * round_up(K, 64));
  const bool mean3std = wmode == SQMP_W_PER_GROUP_MEAN3STD;
  const bool sorted = wmode == SQMP_W_PER_GROUP || mean3std;
  const bool per_tensor = wmode == SQMP_W_PER_TENSOR;
  if (mean3std) {
    st = launch_colkey_mean3std(w, dtype, N, K, sums, cmax, s);
    if (st) return st;
  } else if (sorted || per_tensor) {
    st = launch_colmax(w, dtype, N, K, cmax, s);
    if (st) return st;
  }
  if (sorted) {
    st = launch_rank(cmax, nullptr, K, K, rank, s);
    if (st) return st;
  }
  st = launch_build_maps(K, Kp, sorted ? rank : nullptr, salient, S, perm, amap, amap_fq,
                         nonsal, s);
  if (st) return st;
  const int q_max = n_bits ? (1 << (n_bits - 1)) - 1 : 1;
#define SQMP_PACK(DTT, WB)                                                                 \
  pack_rows_launch<DTT, WB>(w, N, K, Kp, Gw, ngw, q_max, per_tensor, perm, amap, cmax,   \
                            salient, S, S_pad, codes, wscale, wsal, s)
  switch (dtype) {
    case SQMP_F32: return n_bits == 4 ? SQMP_PACK(F32, 4) : n_bits == 8 ? SQMP_PACK(F32, 8) : SQMP_PACK(F32, 0);
    case SQMP_F16: return n_bits == 4 ? SQMP_PACK(F16, 4) : n_bits == 8 ? SQMP_PACK(F16, 8) : SQMP_PACK(F16, 0);
    default: return n_bits == 4 ? SQMP_PACK(BF16, 4) : n_bits == 8 ? SQMP_PACK(BF16, 8) : SQMP_PACK(BF16, 0);
  }
#undef SQMP_PACK
}

extern "C" int sqmp_dequant_weight(const void* codes, const void* wscale, const void* wsal,
                                   const int32_t* amap, const int32_t* salient, int dtype,
                                   int N, int K, int S, int n_bits, int Kp, int Gw, int ngw,
                                   int S_pad, void* w_hat, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  hipStream_t s = (hipStream_t)stream;
  if (dtype < SQMP_F32 || dtype > SQMP_BF16 || N <= 0 || K <= 0 || Kp < K || Gw <= 0)
    return SQMP_EINVAL;
  if (n_bits != 0 && n_bits != 4 && n_bits != 8) return SQMP_EUNSUPPORTED;
  if (!codes || !wscale || !amap || !w_hat || (S > 0 && (!wsal || !salient)))
    return SQMP_EINVAL;
#define SQMP_DQ(DTT, WB) \
  dequant_launch<DTT, WB>(codes, wscale, wsal, amap, salient, N, K, S, Kp, Gw, ngw, S_pad, w_hat, s)
  switch (dtype) {
    case SQMP_F32: return n_bits == 4 ? SQMP_DQ(F32, 4) : n_bits == 8 ? SQMP_DQ(F32, 8) : SQMP_DQ(F32, 0);
    case SQMP_F16: return n_bits == 4 ? SQMP_DQ(F16, 4) : n_bits == 8 ? SQMP_DQ(F16, 8) : SQMP_DQ(F16, 0);
    default: return n_bits == 4 ? SQMP_DQ(BF16, 4) : n_bits == 8 ? SQMP_DQ(BF16, 8) : SQMP_DQ(BF16, 0);
  }
#undef SQMP_DQ
}

extern "C" int sqmp_dequant_weight_packed(const void* codes, const void* wscale, int dtype,
                                          int N, int Kp, int Gw, int ngw, int n_bits,
                                          void* out, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  hipStream_t s = (hipStream_t)stream;
  if (dtype < SQMP_F32 || dtype > SQMP_BF16 || N <= 0 || Kp <= 0 || Gw <= 0 || ngw <= 0)
    return SQMP_EINVAL;
  if (n_bits != 4 && n_bits != 8) return SQMP_EUNSUPPORTED;
  if (!codes || !wscale || !out) return SQMP_EINVAL;
#define SQMP_DP(DTT, WB) dequant_packed_launch<DTT, WB>(codes, wscale, N, Kp, Gw, ngw, out, s)
  switch (dtype) {
    case SQMP_F32: return n_bits == 4 ? SQMP_DP(F32, 4) : SQMP_DP(F32, 8);
    case SQMP_F16: return n_bits == 4 ? SQMP_DP(F16, 4) : SQMP_DP(F16, 8);
    default: return n_bits == 4 ? SQMP_DP(BF16, 4) : SQMP_DP(BF16, 8);
  }
#undef SQMP_DP
}

extern "C" int sqmp_build_maps(int K, const int32_t* salient, int S, int32_t* perm,
                               int32_t* amap, int32_t* amap_fq, int32_t* nonsal, int Kp,
                               void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (K <= 0 || K > 65000 || S < 0 || S > K || Kp < K) return SQMP_EINVAL;
  if (!perm || !amap || !amap_fq || (K - S > 0 && !nonsal) || (S > 0 && !salient))
    return SQMP_EINVAL;
  return launch_build_maps(K, Kp, nullptr, salient, S, perm, amap, amap_fq, nonsal,
                           (hipStream_t)stream);
}
