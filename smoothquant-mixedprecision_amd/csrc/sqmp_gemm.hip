// GEMM entry points of the C ABI + the generic fallback kernel.
//
//   sqmp_gemm_fq -> gemm_fq3 (sqmp_gemm_fast.hip) for fp16 / bf16 with int4 codes at
//                   group sizes that are a multiple of 32, or dense weights;
//                   gemm_generic below for everything else (fp32, 8-bit codes, groups
//                   of 8 / 16 elements): the round-1 register-staged 128 x 128 kernel.
#include <stdlib.h>

#include <type_traits>

#include "sqmp_mfma.h"

namespace sqmp {

constexpr int BM = 128, BN = 128;
constexpr int ROWB = 128;
constexpr int TILE_BYTES = BM * ROWB;

__device__ inline int lds_off(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 7)) << 4); }

// Decode one thread's share of a weight row for one K-tile: BKE/2 consecutive positions
// -> 64 bytes of D values (4 LDS chunks).  WBITS 4 = bpack, 8 = row-major int8,
// 0 = dense D.  Value = D((float)code * s), the reference's D(code * s) (fake_quant.py:193).
template <class DT, int WBITS>
struct BDecode {
  typedef typename DT::T T;
  static constexpr int BKE = ROWB / sizeof(T);
  static constexpr int NCODE = BKE / 2;
  static constexpr int RAWW = WBITS == 4 ? NCODE / 8 : WBITS == 8 ? NCODE / 4 : NCODE * (int)sizeof(T) / 4;
  static constexpr int EPC = 16 / sizeof(T);

  __device__ static inline void load(const uint8_t* codes, int n, int Kp, int p0, uint32_t* raw) {
    if (WBITS == 4) {
      const uint32_t* row = (const uint32_t*)codes + (size_t)n * (Kp / 8);
#pragma unroll
      for (int w = 0; w < RAWW; ++w) raw[w] = row[bpack_dword(p0 + 8 * w)];
    } else if (WBITS == 8) {
      const uint32_t* src = (const uint32_t*)(codes + (size_t)n * Kp + p0);
#pragma unroll
      for (int w = 0; w < RAWW; ++w) raw[w] = src[w];
    } else {
      const uint32_t* src = (const uint32_t*)((const T*)codes + (size_t)n * Kp + p0);
#pragma unroll
      for (int w = 0; w < RAWW; ++w) raw[w] = src[w];
    }
  }
  __device__ static inline int code_at(const uint32_t* raw, int e) {
    if (WBITS == 4) return (int)((raw[e >> 3] >> bpack_shift(e & 7)) & 0xFu) - 8;
    return (int)(int8_t)((raw[e >> 2] >> (8 * (e & 3))) & 0xFFu);
  }
  __device__ static inline void run(const uint32_t* raw, const float* s, u32x4* out) {
    if (WBITS == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) out[c] = u32x4{raw[4 * c], raw[4 * c + 1], raw[4 * c + 2], raw[4 * c + 3]};
      return;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      T v[EPC];
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] = DT::from_f((float)code_at(raw, c * EPC + e) * s[c]);
      out[c] = *(const u32x4*)v;
    }
  }
};

// WN = waves along N (2: 4 waves of 64 x 64, the 16-bit default; 4: 8 waves of 64 x 32, the
// fp32 build -- two waves per SIMD at one 128 x 128 tile per CU, so one wave's MFMAs cover
// the other's barrier and staging; f32 MFMAs leave VALU and LDS idle otherwise)
template <class DT, int WBITS, int WN = 2>
__global__ __launch_bounds__(128 * WN, 2) void gemm_generic_kernel(
    const typename DT::T* __restrict__ A, const uint8_t* __restrict__ codes,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n, uint32_t* __restrict__ colmax) {
  typedef typename DT::T T;
  typedef BDecode<DT, WBITS> Dec;
  constexpr int BKE = ROWB / sizeof(T);
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * 2 * TILE_BYTES];

  constexpr int NT = 128 * WN;          // threads
  constexpr int LI = 1024 / NT;          // 16-B A / dense-B chunks per thread per stage
  constexpr int CW = BN / WN, J = CW / 16;  // columns per wave, 16-wide tiles
  int tm, tn;
  tile_coords(tiles_m, tiles_n, 8, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int Ktot = Kp + S_pad;
  const int nkt_main = Kp / BKE, nkt = Ktot / BKE;
  const int Np = pad_n(N);

  f32x4 acc[4][J];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[LI], rb[LI];
  uint32_t rc[Dec::RAWW];
  float rs[4];
  // weight decode: thread (bn, bh) decodes half bh of weight row bn (256 threads)
  const bool dec_thr = tid < 256;
  const int bn = (tid & 255) >> 1, bh = tid & 1;
  const int gbn = n0 + bn;

  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < LI; ++i) {
      const int q = tid + NT * i, row = q >> 3, c = q & 7;
      const int gm = min(m0 + row, M - 1);
      ra[i] = *(const u32x4*)(A + (size_t)gm * Ktot + (size_t)kt * BKE + c * (16 / sizeof(T)));
    }
    if (kt < nkt_main) {
      if (!dec_thr) return;
      const int p0 = kt * BKE + bh * (BKE / 2);
      const int n = min(gbn, N - 1);
      Dec::load(codes, n, Kp, p0, rc);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int p = p0 + c * (BKE / 8);
        rs[c] = WBITS ? DT::to_f(wscale[(size_t)min(p / Gw, ngw - 1) * Np + n]) : 1.f;
      }
    } else {
      const int ks = (kt - nkt_main) * BKE;
#pragma unroll
      for (int i = 0; i < LI; ++i) {
        const int q = tid + NT * i, row = q >> 3, c = q & 7;
        const int gn = min(n0 + row, N - 1);
        rb[i] = *(const u32x4*)(wsal + (size_t)gn * S_pad + ks + c * (16 / sizeof(T)));
      }
    }
  };
  auto store = [&](int kt, int buf) {
    unsigned char* la = lds + buf * 2 * TILE_BYTES;
    unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < LI; ++i) {
      const int q = tid + NT * i, row = q >> 3, c = q & 7;
      *(u32x4*)(la + lds_off(row, c)) = ra[i];
    }
    if (kt < nkt_main) {
      if (!dec_thr) return;
      u32x4 dec[4];
      Dec::run(rc, rs, dec);
#pragma unroll
      for (int c = 0; c < 4; ++c) *(u32x4*)(lb + lds_off(bn, bh * 4 + c)) = dec[c];
    } else {
#pragma unroll
      for (int i = 0; i < LI; ++i) {
        const int q = tid + NT * i, row = q >> 3, c = q & 7;
        *(u32x4*)(lb + lds_off(row, c)) = rb[i];
      }
    }
  };
  auto compute = [&](int buf) {
    const unsigned char* la = lds + buf * 2 * TILE_BYTES;
    const unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 af[4], bf[J];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(la + lds_off(wm * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < J; ++j) bf[j] = *(const u32x4*)(lb + lds_off(wn * CW + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) Mfma<DT>::run(acc[i][j], af[i], bf[j]);
    }
  };

  load(0);
  store(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) load(kt + 1);
    compute(cur);
    if (kt + 1 < nkt) store(kt + 1, cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int gn = n0 + wn * CW + j * 16 + (lane & 15);
    const float bv = bias && gn < N ? DT::to_f(bias[gn]) : 0.f;
    float cm = 0.f;  // max |y| of this lane's rows in column gn (the stored D values)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const T v = DT::from_f(acc[i][j][r] + bv);
        if (gm < M && gn < N) {
          Y[(size_t)gm * N + gn] = v;
          cm = fmaxf(cm, fabsf(DT::to_f(v)));
        }
      }
    if (colmax) {  // lanes l, l + 16, l + 32, l + 48 hold the same column
      cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
      cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
      if (lane < 16 && gn < N) atomicMax(colmax + gn, __float_as_uint(cm));
    }
  }
}

template <class DT, int WBITS>
static int generic_launch(const void* a, const void* codes, const void* wscale,
                          const void* wsal, const void* bias, void* y, int M, int N, int Kp,
                          int S_pad, int Gw, int ngw, uint32_t* colmax, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  const char* wn2 = knob("SQMP_F32_WN2");  // A/B knob: the 4-wave build for fp32 too
  const bool f32_4w = wn2 && atoi(wn2) == 1;
  if constexpr (std::is_same<DT, F32>::value) if (!f32_4w) {
    gemm_generic_kernel<DT, WBITS, 4><<<dim3(tiles_m * tiles_n), dim3(512), 0, s>>>(
        (const T*)a, (const uint8_t*)codes, (const T*)wscale, (const T*)wsal, (const T*)bias,
        (T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, tiles_n, colmax);
    SQMP_LAUNCH_CHECK();
    return SQMP_OK;
  }
  gemm_generic_kernel<DT, WBITS><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
      (const T*)a, (const uint8_t*)codes, (const T*)wscale, (const T*)wsal, (const T*)bias,
      (T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, tiles_n, colmax);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace sqmp

using namespace sqmp;

static int check_gemm_geometry(int dtype, int M, int N, int Kp, int S_pad, int Gw, int ngw,
                               int n_bits) {
  if (dtype < SQMP_F32 || dtype > SQMP_BF16 || M < 0 || N <= 0) return SQMP_EINVAL;
  if (Kp <= 0 || Kp % 128 != 0 || S_pad < 0 || S_pad % 64 != 0) return SQMP_EINVAL;
  if (n_bits == 0) return SQMP_OK;  // dense operand: no groups
  if (Gw <= 0 || ngw <= 0 || (long)(ngw - 1) * Gw >= Kp) return SQMP_EINVAL;
  if (n_bits != 4 && n_bits != 8) return SQMP_EUNSUPPORTED;
  // one scale per 16-B chunk of decoded B: groups must not split a chunk
  const int epc = dtype == SQMP_F32 ? 4 : 8;
  if (Gw % epc != 0) return SQMP_EUNSUPPORTED;
  return SQMP_OK;
}

extern "C" int sqmp_gemm_fq(const void* a, const void* codes, const void* wscale,
                            const void* wsal, const void* bias, void* y, int dtype, int M,
                            int N, int Kp, int S_pad, int Gw, int ngw, int n_bits,
                            void* stream) {
  SQMP_DEVICE_GUARD(stream);
  return sqmp_gemm_fq_colmax(a, codes, wscale, wsal, bias, y, dtype, M, N, Kp, S_pad, Gw, ngw,
                             n_bits, nullptr, stream);
}

extern "C" int sqmp_gemm_fq_colmax(const void* a, const void* codes, const void* wscale,
                                   const void* wsal, const void* bias, void* y, int dtype,
                                   int M, int N, int Kp, int S_pad, int Gw, int ngw,
                                   int n_bits, uint32_t* colmax, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  int st = check_gemm_geometry(dtype, M, N, Kp, S_pad, Gw, ngw, n_bits);
  if (st) return st;
  if (!a || !codes || (n_bits && !wscale) || !y || (S_pad > 0 && !wsal)) return SQMP_EINVAL;
  if (M == 0) return SQMP_OK;
  if (n_bits == 0) { Gw = Kp; ngw = 1; }
  hipStream_t s = (hipStream_t)stream;
  const bool fast = dtype != SQMP_F32 && (n_bits == 0 || (n_bits == 4 && (Gw % 64 == 0 || Gw == 32)));
  if (fast)
    return launch_gemm_fq_fast(dtype, a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw,
                               n_bits, colmax, s);
#define SQMP_G(DTT, WB) generic_launch<DTT, WB>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, colmax, s)
  switch (dtype) {
    case SQMP_F32: return n_bits == 4 ? SQMP_G(F32, 4) : n_bits == 8 ? SQMP_G(F32, 8) : SQMP_G(F32, 0);
    case SQMP_F16: return n_bits == 4 ? SQMP_G(F16, 4) : n_bits == 8 ? SQMP_G(F16, 8) : SQMP_G(F16, 0);
    default: return n_bits == 4 ? SQMP_G(BF16, 4) : n_bits == 8 ? SQMP_G(BF16, 8) : SQMP_G(BF16, 0);
  }
#undef SQMP_G
}

extern "C" int sqmp_gemm_fqt(const void* acodes, const void* ascale, const void* xs,
                             const void* wp, const void* bias, void* y, int dtype, int M, int N,
                             int Kq, int S_pad, int G, int ngq, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  using namespace sqmp;
  if (!acodes || !ascale || !wp || !y || (S_pad > 0 && !xs)) return SQMP_EINVAL;
  if (M < 0 || N <= 0 || Kq <= 0 || Kq % 64 || S_pad < 0 || S_pad % 64 || G <= 0 || ngq <= 0)
    return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (G % 64 || N % 8) return SQMP_EUNSUPPORTED;
  if (M == 0) return SQMP_OK;
  return launch_gemm_fqt(dtype, acodes, ascale, xs, wp, bias, y, M, N, Kq, S_pad, G, ngq,
                         (hipStream_t)stream);
}
