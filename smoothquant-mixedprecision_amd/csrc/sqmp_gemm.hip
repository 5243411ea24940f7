// W4A4 mixed-precision GEMMs for gfx950 (the F.linear of fake_quant.py:306).
//
// Both kernels compute y[M][N] = A . B^T over the packed K axis of a packed weight
// (include/sqmp_w4a4.h): Kp positions of the quantized operand in weight-sorted group
// order, then S_pad positions of the exact salient slice, in one K loop and one
// workgroup, with fp32 accumulation and a single rounding to D in the epilogue.
//
//   sqmp_gemm_fq  "faithful": A = x_hat in D (the reference's dequantized activations,
//                 bit-exact); B decoded in registers from int4/int8 codes as
//                 D(code * wscale) == the reference's W_hat bit for bit, written to LDS;
//                 MFMA in D (f16 / bf16 16x16x32, f32 16x16x4).  Exact up to fp32
//                 accumulation order for every act mode, including per_group.
//   sqmp_gemm_i8  integer: A = int8 act codes (per_token / per_tensor), B = int4 codes
//                 unpacked to int8, v_mfma_i32_16x16x64_i8, per-weight-group fold
//                 acc_f32 += float(acc_i32) * wscale, per-row act scale, then the salient
//                 tail on the D MFMA into the same accumulators.
//
// Tiling: 128x128 output tile per 256-thread workgroup (2x2 waves of 64x64 = 4x4 MFMA
// 16x16 tiles), K-tile = 128 bytes per row for both operands (64 D elements / 128 int8
// codes), double-buffered LDS with one barrier per K-tile: global loads for tile t+1 are
// issued before the MFMAs of tile t and written (decoded) to the other buffer after.
// LDS rows are 128 B with a 16-B-chunk XOR swizzle (chunk ^ (row & 7)) for the
// ds_read_b128 fragment reads.  Workgroup ids are remapped XCD-aware (contiguous chunks
// of the tile sequence per XCD) and grouped along M for L2 reuse of the weight tiles.
#include "sqmp_internal.h"

namespace sqmp {

constexpr int BM = 128, BN = 128;
constexpr int ROWB = 128;                 // bytes per LDS row per K-tile
constexpr int TILE_BYTES = BM * ROWB;     // 16 KiB per operand per buffer
constexpr int GROUP_M = 8;

__device__ inline int lds_off(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 7)) << 4); }

__device__ inline void tile_coords(int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD; give each XCD a
  // contiguous range of the logical tile sequence.
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // grouped ordering along M
  const int per_group = GROUP_M * tiles_n;
  const int gid = wg / per_group;
  const int first_m = gid * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_g = wg - gid * per_group;
  tm = first_m + in_g % gsz;
  tn = in_g / gsz;
}

// ---------------------------------------------------------------- MFMA wrappers
template <class DT> struct Mfma;
template <> struct Mfma<F16> {
  __device__ static inline void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(*(const f16x8*)&a, *(const f16x8*)&b, acc, 0, 0, 0);
  }
};
template <> struct Mfma<BF16> {
  __device__ static inline void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)&a, *(const bf16x8*)&b, acc, 0, 0, 0);
  }
};
template <> struct Mfma<F32> {
  // 16x16x4 f32: lane group q supplies k = q; element e of the 16-B chunk is a separate
  // k-slice, so four MFMAs consume the chunk (A and B use the same k assignment).
  __device__ static inline void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    const float* af = (const float*)&a;
    const float* bf = (const float*)&b;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e], bf[e], acc, 0, 0, 0);
  }
};

// ---------------------------------------------------------------- B decode
// Decode one thread's share of a weight row for one K-tile: BKE/2 consecutive codes
// -> 64 bytes of D values (4 LDS chunks).  Value = D((float)code * s) which equals the
// reference's D(code * s) rounding (fake_quant.py:193).
// WBITS == 0: the operand is already dense D (W4A4Linear built without weight
// quantization, fake_quant.py:227-235, or a group size finer than one 16-B chunk).
template <class DT, int WBITS>
struct BDecode {
  typedef typename DT::T T;
  static constexpr int BKE = ROWB / sizeof(T);   // D elements per K-tile
  static constexpr int NCODE = BKE / 2;          // codes per thread
  static constexpr int RAWB = WBITS ? NCODE * WBITS / 8 : NCODE * (int)sizeof(T);
  static constexpr int RAWW = RAWB / 4;
  static constexpr int EPC = 16 / sizeof(T);     // elements per 16-B chunk

  __device__ static inline int code_at(const uint32_t* raw, int e) {
    if (WBITS == 4) return (int)((raw[e >> 3] >> (4 * (e & 7))) & 0xFu) - 8;
    return (int)(int8_t)((raw[e >> 2] >> (8 * (e & 3))) & 0xFFu);
  }
  // out: 4 chunks of 16 B; s[c] = scale (fp32 value of the D scale) of chunk c
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

// fp16 fast path: 0x6400|n is the half 1024+n; minus 1032 gives the code exactly, and the
// packed half multiply by the scale rounds once (RNE) -- identical to D(code*s).
template <>
struct BDecode<F16, 4> {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  static constexpr int BKE = 64, NCODE = 32, RAWB = 16, RAWW = 4, EPC = 8;
  __device__ static inline void run(const uint32_t* raw, const float* s, u32x4* out) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t w = raw[c];
      const uint32_t t = w & 0x0F0F0F0Fu;          // codes 0,2,4,6 (+8)
      const uint32_t u = (w >> 4) & 0x0F0F0F0Fu;   // codes 1,3,5,7 (+8)
      const _Float16 sh = (_Float16)s[c];
      const h2 s2 = {sh, sh};
      const h2 off = {(_Float16)1032.0f, (_Float16)1032.0f};
      uint32_t o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t bits = ((t >> (8 * i)) & 0xFu) | (((u >> (8 * i)) & 0xFu) << 16) | 0x64006400u;
        h2 h = *(const h2*)&bits;
        h = (h - off) * s2;
        o[i] = *(const uint32_t*)&h;
      }
      out[c] = u32x4{o[0], o[1], o[2], o[3]};
    }
  }
};

// ---------------------------------------------------------------- faithful kernel
template <class DT, int WBITS>
__global__ __launch_bounds__(256, 2) void gemm_fq_kernel(
    const typename DT::T* __restrict__ A, const uint8_t* __restrict__ codes,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  typedef BDecode<DT, WBITS> Dec;
  constexpr int BKE = ROWB / sizeof(T);  // D elements per K-tile
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * 2 * TILE_BYTES];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int Ktot = Kp + S_pad;
  const int nkt_main = Kp / BKE, nkt = Ktot / BKE;
  constexpr int EB = WBITS ? 0 : (int)sizeof(T);  // dense element bytes
  const size_t codes_row = WBITS ? (size_t)Kp * WBITS / 8 : (size_t)Kp * EB;
  const float invG = 1.0f / (float)Gw;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4];             // A staging: 4 x 16 B
  u32x4 rb[4];             // B staging: salient 4 x 16 B, or raw codes
  uint32_t rc[Dec::RAWW];  // raw codes
  float rs[4];             // chunk scales

  // B-thread mapping for the code path: row bn, half bh of the K-tile
  const int bn = tid >> 1, bh = tid & 1;
  const int gbn = n0 + bn;

  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      const int gm = m0 + row;
      ra[i] = gm < M ? *(const u32x4*)(A + (size_t)gm * Ktot + (size_t)kt * BKE + c * (16 / sizeof(T)))
                     : u32x4{0u, 0u, 0u, 0u};
    }
    if (kt < nkt_main) {
      const int p0 = kt * BKE + bh * (BKE / 2);
      if (gbn < N) {
        const uint32_t* src = (const uint32_t*)(codes + (size_t)gbn * codes_row +
                                                (WBITS ? (size_t)p0 * WBITS / 8 : (size_t)p0 * EB));
#pragma unroll
        for (int w = 0; w < Dec::RAWW; ++w) rc[w] = src[w];
#pragma unroll
        for (int c = 0; c < 4 && WBITS != 0; ++c) {
          const int p = p0 + c * (BKE / 8);
          int g = (int)((float)p * invG);
          if ((g + 1) * Gw <= p) ++g;
          if (g * Gw > p) --g;
          rs[c] = DT::to_f(wscale[(size_t)gbn * ngw + g]);
        }
      } else {
#pragma unroll
        for (int w = 0; w < Dec::RAWW; ++w) rc[w] = WBITS == 4 ? 0x88888888u : 0u;
#pragma unroll
        for (int c = 0; c < 4; ++c) rs[c] = 0.f;
      }
    } else {
      const int ks = (kt - nkt_main) * BKE;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = tid + 256 * i, row = q >> 3, c = q & 7;
        const int gn = n0 + row;
        rb[i] = gn < N ? *(const u32x4*)(wsal + (size_t)gn * S_pad + ks + c * (16 / sizeof(T)))
                       : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  auto store = [&](int kt, int buf) {
    unsigned char* la = lds + buf * 2 * TILE_BYTES;
    unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      *(u32x4*)(la + lds_off(row, c)) = ra[i];
    }
    if (kt < nkt_main) {
      u32x4 dec[4];
      Dec::run(rc, rs, dec);
#pragma unroll
      for (int c = 0; c < 4; ++c) *(u32x4*)(lb + lds_off(bn, bh * 4 + c)) = dec[c];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = tid + 256 * i, row = q >> 3, c = q & 7;
        *(u32x4*)(lb + lds_off(row, c)) = rb[i];
      }
    }
  };
  auto compute = [&](int buf) {
    const unsigned char* la = lds + buf * 2 * TILE_BYTES;
    const unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 af[4], bf[4];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(la + lds_off(wm * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *(const u32x4*)(lb + lds_off(wn * 64 + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Mfma<DT>::run(acc[i][j], af[i], bf[j]);
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

  // epilogue: + bias, one rounding to D
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int gn = n0 + wn * 64 + j * 16 + (lane & 15);
    if (gn >= N) continue;
    const float bv = bias ? DT::to_f(bias[gn]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (gm < M) Y[(size_t)gm * N + gn] = DT::from_f(acc[i][j][r] + bv);
      }
  }
}

// ---------------------------------------------------------------- integer kernel
template <class DT, int WBITS>
__global__ __launch_bounds__(256, 2) void gemm_i8_kernel(
    const int8_t* __restrict__ A8, const float* __restrict__ ascale,
    const typename DT::T* __restrict__ XS, const uint8_t* __restrict__ codes,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  constexpr int BKC = 128;                         // int8 codes per K-tile (main loop)
  constexpr int BKE = ROWB / sizeof(T);            // D elements per K-tile (salient loop)
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * 2 * TILE_BYTES];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nkt_main = Kp / BKC, nkt_sal = S_pad / BKE;
  const size_t codes_row = (size_t)Kp * WBITS / 8;
  const int bn = tid >> 1, bh = tid & 1;
  const int gbn = n0 + bn;

  f32x4 tot[4][4];
  i32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[i][j] = i32x4{0, 0, 0, 0};
    }

  u32x4 ra[4], rb[4];
  constexpr int RAWW = 64 * WBITS / 8 / 4;  // 64 codes per thread per K-tile
  uint32_t rc[RAWW];

  auto load_main = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      const int gm = m0 + row;
      ra[i] = gm < M ? *(const u32x4*)(A8 + (size_t)gm * Kp + (size_t)kt * BKC + c * 16) : u32x4{0u, 0u, 0u, 0u};
    }
    if (gbn < N) {
      const uint32_t* src = (const uint32_t*)(codes + (size_t)gbn * codes_row + ((size_t)kt * BKC + bh * 64) * WBITS / 8);
#pragma unroll
      for (int w = 0; w < RAWW; ++w) rc[w] = src[w];
    } else {
#pragma unroll
      for (int w = 0; w < RAWW; ++w) rc[w] = WBITS == 4 ? 0x88888888u : 0u;
    }
  };
  auto store_main = [&](int buf) {
    unsigned char* la = lds + buf * 2 * TILE_BYTES;
    unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      *(u32x4*)(la + lds_off(row, c)) = ra[i];
    }
    if (WBITS == 4) {
      // 8 nibbles (code+8) per word -> 8 int8 codes
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t o[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t w = rc[c * 2 + h];
          const uint32_t t = w & 0x0F0F0F0Fu, u = (w >> 4) & 0x0F0F0F0Fu;
          // bytes (c0,c1,c2,c3) and (c4,c5,c6,c7), still offset by 8
          const uint32_t lo = (t & 0xFFu) | ((u & 0xFFu) << 8) | ((t & 0xFF00u) << 8) | ((u & 0xFF00u) << 16);
          const uint32_t hi = ((t >> 16) & 0xFFu) | (((u >> 16) & 0xFFu) << 8) | ((t >> 24) << 16) | ((u >> 24) << 24);
          o[h * 2 + 0] = (lo + 0x78787878u) ^ 0x80808080u;
          o[h * 2 + 1] = (hi + 0x78787878u) ^ 0x80808080u;
        }
        *(u32x4*)(lb + lds_off(bn, bh * 4 + c)) = u32x4{o[0], o[1], o[2], o[3]};
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        *(u32x4*)(lb + lds_off(bn, bh * 4 + c)) = u32x4{rc[c * 4], rc[c * 4 + 1], rc[c * 4 + 2], rc[c * 4 + 3]};
    }
  };
  auto compute_main = [&](int kt, int buf) {
    const unsigned char* la = lds + buf * 2 * TILE_BYTES;
    const unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 af[4], bf[4];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(la + lds_off(wm * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *(const u32x4*)(lb + lds_off(wn * 64 + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(*(const i32x4*)&af[i], *(const i32x4*)&bf[j], acc[i][j], 0, 0, 0);
      const int p_end = kt * BKC + (kk + 1) * 64;
      if (p_end % Gw == 0) {
        const int g = p_end / Gw - 1;
        if (g < ngw) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int gn = n0 + wn * 64 + j * 16 + (lane & 15);
            const float s = gn < N ? DT::to_f(wscale[(size_t)gn * ngw + g]) : 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
              for (int r = 0; r < 4; ++r) tot[i][j][r] += (float)acc[i][j][r] * s;
              acc[i][j] = i32x4{0, 0, 0, 0};
            }
          }
        }
      }
    }
  };

  if (nkt_main > 0) {
    load_main(0);
    store_main(0);
    __syncthreads();
    for (int kt = 0; kt < nkt_main; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nkt_main) load_main(kt + 1);
      compute_main(kt, cur);
      if (kt + 1 < nkt_main) store_main(cur ^ 1);
      __syncthreads();
    }
  }
  // per-row activation scale (fake_quant.py:56-75 scale, factored out of the sum)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gm = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
      const float sa = gm < M ? ascale[gm] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) tot[i][j][r] *= sa;
    }

  // salient tail: exact D operands on the D MFMA
  auto load_sal = [&](int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      const int gm = m0 + row, gn = n0 + row;
      ra[i] = gm < M ? *(const u32x4*)(XS + (size_t)gm * S_pad + (size_t)ks * BKE + c * (16 / sizeof(T))) : u32x4{0u, 0u, 0u, 0u};
      rb[i] = gn < N ? *(const u32x4*)(wsal + (size_t)gn * S_pad + (size_t)ks * BKE + c * (16 / sizeof(T))) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store_sal = [&](int buf) {
    unsigned char* la = lds + buf * 2 * TILE_BYTES;
    unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      *(u32x4*)(la + lds_off(row, c)) = ra[i];
      *(u32x4*)(lb + lds_off(row, c)) = rb[i];
    }
  };
  auto compute_sal = [&](int buf) {
    const unsigned char* la = lds + buf * 2 * TILE_BYTES;
    const unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 af[4], bf[4];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(la + lds_off(wm * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *(const u32x4*)(lb + lds_off(wn * 64 + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Mfma<DT>::run(tot[i][j], af[i], bf[j]);
    }
  };
  if (nkt_sal > 0) {
    load_sal(0);
    store_sal(0);
    __syncthreads();
    for (int ks = 0; ks < nkt_sal; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nkt_sal) load_sal(ks + 1);
      compute_sal(cur);
      if (ks + 1 < nkt_sal) store_sal(cur ^ 1);
      __syncthreads();
    }
  }

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int gn = n0 + wn * 64 + j * 16 + (lane & 15);
    if (gn >= N) continue;
    const float bv = bias ? DT::to_f(bias[gn]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (gm < M) Y[(size_t)gm * N + gn] = DT::from_f(tot[i][j][r] + bv);
      }
  }
}

template <class DT, int WBITS>
static int gemm_fq_launch(const void* a, const void* codes, const void* wscale,
                          const void* wsal, const void* bias, void* y, int M, int N, int Kp,
                          int S_pad, int Gw, int ngw, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  gemm_fq_kernel<DT, WBITS><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
      (const T*)a, (const uint8_t*)codes, (const T*)wscale, (const T*)wsal, (const T*)bias,
      (T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, tiles_n);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT, int WBITS>
static int gemm_i8_launch(const int8_t* a8, const float* ascale, const void* xs,
                          const void* codes, const void* wscale, const void* wsal,
                          const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                          int ngw, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  gemm_i8_kernel<DT, WBITS><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
      a8, ascale, (const T*)xs, (const uint8_t*)codes, (const T*)wscale, (const T*)wsal,
      (const T*)bias, (T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, tiles_n);
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
  int st = check_gemm_geometry(dtype, M, N, Kp, S_pad, Gw, ngw, n_bits);
  if (st) return st;
  if (!a || !codes || (n_bits && !wscale) || !y || (S_pad > 0 && !wsal)) return SQMP_EINVAL;
  if (M == 0) return SQMP_OK;
  if (n_bits == 0) { Gw = Kp; ngw = 1; }
  hipStream_t s = (hipStream_t)stream;
#define SQMP_G(DTT, WB) gemm_fq_launch<DTT, WB>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s)
  switch (dtype) {
    case SQMP_F32: return n_bits == 4 ? SQMP_G(F32, 4) : n_bits == 8 ? SQMP_G(F32, 8) : SQMP_G(F32, 0);
    case SQMP_F16: return n_bits == 4 ? SQMP_G(F16, 4) : n_bits == 8 ? SQMP_G(F16, 8) : SQMP_G(F16, 0);
    default: return n_bits == 4 ? SQMP_G(BF16, 4) : n_bits == 8 ? SQMP_G(BF16, 8) : SQMP_G(BF16, 0);
  }
#undef SQMP_G
}

extern "C" int sqmp_gemm_i8(const int8_t* a8, const float* ascale, const void* xs,
                            const void* codes, const void* wscale, const void* wsal,
                            const void* bias, void* y, int dtype, int M, int N, int Kp,
                            int S_pad, int Gw, int ngw, int n_bits, void* stream) {
  int st = check_gemm_geometry(dtype, M, N, Kp, S_pad, Gw, ngw, n_bits);
  if (st) return st;
  if (dtype == SQMP_F32 || n_bits == 0 || Gw % 64 != 0) return SQMP_EUNSUPPORTED;
  if (!a8 || !ascale || !codes || !wscale || !y || (S_pad > 0 && (!wsal || !xs)))
    return SQMP_EINVAL;
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
#define SQMP_G(DTT, WB) gemm_i8_launch<DTT, WB>(a8, ascale, xs, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s)
  switch (dtype) {
    case SQMP_F16: return n_bits == 4 ? SQMP_G(F16, 4) : SQMP_G(F16, 8);
    default: return n_bits == 4 ? SQMP_G(BF16, 4) : SQMP_G(BF16, 8);
  }
#undef SQMP_G
}
