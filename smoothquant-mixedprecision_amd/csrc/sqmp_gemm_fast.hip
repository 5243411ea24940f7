// Fast W4A4 GEMMs for gfx950 (fp16 / bf16): the F.linear of fake_quant.py:306.
//
// gemm_fq4 -- the faithful mixed-precision GEMM
//   y[M][N] = D( A[M][Kp + S_pad] . B^T + bias ):  A = dequantized activations x_hat in
//   packed K order + the exact salient columns (bit-exact with the reference's q_x);
//   B = int4 codes decoded in registers to D(code * scale) (bit-exact with the
//   reference's W_hat), then the exact salient weight slice; MFMA 16x16x32 in D, fp32
//   accumulation, one rounding to D.
//
//   Tile 256 (M) x 256 (N) per 512-thread workgroup: 8 waves as 2 (M) x 4 (N), each
//   128 x 64 = 8 x 4 MFMA tiles (128 fp32 accumulators per lane), two waves per SIMD so
//   one wave's MFMAs cover the other's LDS reads and decode.  Every main-loop global byte
//   moves by LDS-DMA (global_load_lds_dwordx4) into a 3-slot LDS ring, two 64-element
//   K-stages ahead of the MFMAs:
//     A  256 rows x 128 B, 16-B chunks XOR-swizzled by (row >> 1) & 7
//     B  256 weight rows x one 32-B bpack block; each lane reads its 8 bytes (its two B
//        fragments) with ds_read_b64, 8-B pieces swizzled by (row >> 2) & 2
//     S  the block's group scales, 1 KiB per wave (its 64 columns).
//   Waits are hand-counted (`s_waitcnt vmcnt(N)` keeps the next stage in flight) and the
//   workgroup syncs once per stage with a raw s_barrier; no ordinary global load runs in
//   the main loop, so the compiler never drains the ring.  The salient tail streams its
//   exact B fragments through registers.
//   The MFMA takes the weight fragment in its A slot, so each lane holds 4 consecutive
//   output columns of one row: 8-byte stores in the epilogue.
//
// gemm_i8v2 -- per_token / per_tensor activations on the integer MFMA (see below).
#include "sqmp_mfma.h"

namespace sqmp {

template <int N>
__device__ inline void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ inline void raw_barrier() {
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// ----------------------------------------------------------------- LDS ring geometry
constexpr int F4_A = 32768;                      // 256 rows x 128 B
constexpr int F4_B = 8192;                       // 256 rows x 32 B
constexpr int F4_S = 8192;                       // 8 waves x 1 KiB
constexpr int F4_SLOT = F4_A + F4_B + F4_S;      // 49152
constexpr int F4_NSLOT = 3;                      // 147456 B of 160 KiB
constexpr int F4_VM_CODES = 4 + 1 + 1;           // DMA ops per wave per codes stage
constexpr int F4_VM_DENSE = 4;                   // ... per dense (A-only) stage

// A stage image: row r, 16-B chunk c at r*128 + ((c ^ ((r >> 1) & 7)) << 4)
__device__ inline const u32x4* a4_frag(const unsigned char* st, int row, int chunk) {
  return (const u32x4*)(st + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
}

// GB = weight groups per 64-position block (1: Gw % 64 == 0, 2: Gw == 32);
// GB = 0: dense D weights (no codes) in every main stage.
template <class DT, int GB>
__global__ __launch_bounds__(512, 1) void gemm_fq4_kernel(
    const typename DT::T* __restrict__ A, const void* __restrict__ Bw,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  __shared__ __attribute__((aligned(16))) unsigned char lds[F4_NSLOT * F4_SLOT];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, 4, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int r16 = lane & 15, q = lane >> 4;
  const int lda = Kp + S_pad;
  const int nkt = lda / 64;
  const int nkd = Kp / 64;                // main (non-salient) stages
  const int nkm = GB ? nkd : 0;           // main stages that carry int4 codes
  const int Np = pad_n(N);

  // ---- per-lane DMA source offsets (bytes); per-instruction steps are scalar
  const int arow = 8 * wave + (lane >> 3);
  const uint32_t a_off = (uint32_t)((size_t)(m0 + arow) * lda * sizeof(T) +
                                    (((lane & 7) ^ ((arow >> 1) & 7)) << 4));
  const uint32_t a_str = (uint32_t)(64 * (size_t)lda * sizeof(T));
  const uint32_t b_off = (uint32_t)((size_t)(n0 + 32 * wave + (lane >> 1)) * (Kp / 2) +
                                    (((lane & 1) ^ ((lane >> 4) & 1)) << 4));
  const int s_u = min(lane >> 3, GB > 0 ? GB - 1 : 0);
  const uint32_t s_off = (uint32_t)((n0 + 64 * wn + (lane & 7) * 8) * sizeof(T));

  auto issue = [&](int kt) {
    unsigned char* slot = lds + (kt % F4_NSLOT) * F4_SLOT;
    const unsigned char* ab = (const unsigned char*)A + (size_t)kt * 64 * sizeof(T);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(ab + (size_t)i * a_str + a_off, slot + (i * 8 + wave) * 1024);
    if (GB > 0 && kt < nkm) {
      glds16((const unsigned char*)Bw + (size_t)kt * 32 + b_off, slot + F4_A + wave * 1024);
      const int g0 = GB == 1 ? (kt * 64) / Gw : kt * 2;
      const int g = min(g0 + s_u, ngw - 1);  // zero-code padding past the last group
      glds16((const unsigned char*)wscale + (size_t)g * Np * sizeof(T) + s_off,
             slot + F4_A + F4_B + wave * 1024);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A fragment t = 8 s + i (sub-step s, M tile i) of the current slot; rows of one wave
  // share the swizzle (r16 >> 1) & 7, so consecutive i differ by an immediate 2 KiB.
  const int a_row0 = (wm * 128 + r16) * 128;
  const int a_sw = (r16 >> 1) & 7;
  auto ald = [&](const unsigned char* __restrict__ slot, int t) {
    return *(const u32x4*)(slot + a_row0 + (t & 7) * 2048 + (((4 * (t >> 3) + q) ^ a_sw) << 4));
  };
  // 16 blocks of 4 MFMAs; the A fragment of block t+3 is read during block t and one
  // sched_barrier per block keeps the compiler from hoisting every read (register budget:
  // 2 waves per SIMD, 256 registers, 128 of them accumulators).
#define SQMP_FQ4_BLOCKS(BF, HOOK)                                              \
  {                                                                            \
    u32x4 a[4];                                                                \
    a[0] = ald(slot, 0);                                                       \
    a[1] = ald(slot, 1);                                                       \
    a[2] = ald(slot, 2);                                                       \
    _Pragma("unroll") for (int t = 0; t < 16; ++t) {                           \
      if (t + 3 < 16) a[(t + 3) & 3] = ald(slot, t + 3);                       \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                            \
          Mfma<DT>::run(acc[t & 7][j], BF[t >> 3][j], a[t & 3]);               \
      HOOK;                                                                    \
      __builtin_amdgcn_sched_barrier(0);                                       \
    }                                                                          \
  }

  auto compute_codes = [&](const unsigned char* __restrict__ slot) {
    const unsigned char* sb = slot + F4_A;
    const unsigned char* ss = slot + F4_A + F4_B + wave * 1024;
    uint2 bw[4];
    uint32_t sc[4][GB > 0 ? GB : 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + 16 * j + r16;
      bw[j] = *(const uint2*)(sb + row * 32 + ((q ^ ((r16 >> 2) & 2)) << 3));
#pragma unroll
      for (int u = 0; u < (GB > 0 ? GB : 1); ++u) sc[j][u] = *(const uint16_t*)(ss + u * 128 + (16 * j + r16) * 2);
    }
    u32x4 bf[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[0][j] = Dec8<DT>::run(bw[j].x, sc[j][0]);
    // sub-step 1's fragments are decoded under the MFMAs of blocks 1..4
    SQMP_FQ4_BLOCKS(bf, if (t >= 1 && t <= 4) bf[1][t - 1] = Dec8<DT>::run(bw[t - 1].y, sc[t - 1][GB == 2 ? 1 : 0]));
  };

  // dense B through registers (salient tail; every stage when GB == 0); 32-bit row offsets
  uint32_t brow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) brow[j] = (uint32_t)min(n0 + wn * 64 + j * 16 + r16, N - 1);
  auto compute_dense = [&](const unsigned char* __restrict__ slot, const T* __restrict__ Bd, uint32_t ldb, int kofs) {
    u32x4 bf[2][4];
    const unsigned char* bb = (const unsigned char*)(Bd + kofs + 8 * q);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[s][j] = *(const u32x4*)(bb + (brow[j] * ldb + 32 * s) * sizeof(T));
    SQMP_FQ4_BLOCKS(bf, (void)0);
  };
#undef SQMP_FQ4_BLOCKS

  // ---- the ring: stage kt lives in slot kt % 3, issued two stages ahead.  Three loops,
  // one compute body each, so the accumulators keep their registers across iterations.
  auto enter = [&](int kt) {
    // retire stage kt; the DMA of stage kt+1 (issued after it) may stay in flight
    if (kt + 1 < nkt) {
      if (kt + 1 < nkm) vm_wait<F4_VM_CODES>();
      else vm_wait<F4_VM_DENSE>();
    } else {
      vm_wait<0>();
    }
    raw_barrier();  // every wave's DMA for stage kt has landed; slot (kt+2)%3 is free
    if (kt + 2 < nkt) issue(kt + 2);
    return (const unsigned char*)lds + (kt % F4_NSLOT) * F4_SLOT;
  };
  issue(0);
  if (nkt > 1) issue(1);
  int kt = 0;
  for (; kt < nkm; ++kt) compute_codes(enter(kt));
  for (; kt < nkd; ++kt) compute_dense(enter(kt), (const T*)Bw, (uint32_t)Kp, kt * 64);
  for (; kt < nkt; ++kt) compute_dense(enter(kt), wsal, (uint32_t)S_pad, (kt - nkd) * 64);

  // ---- epilogue: acc[i][j][r] = C[n = n0 + 64 wn + 16 j + 4 q + r][m = m0 + 128 wm + 16 i + r16]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nb = n0 + wn * 64 + j * 16 + q * 4;
    if (nb >= N) continue;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = (bias && nb + r < N) ? DT::to_f(bias[nb + r]) : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int gm = m0 + wm * 128 + i * 16 + r16;
      if (gm >= M) continue;
      T v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = DT::from_f(acc[i][j][r] + bv[r]);
      T* dst = Y + (size_t)gm * N + nb;
      if (nb + 4 <= N && (N & 3) == 0) {
        *(uint2*)dst = *(const uint2*)v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (nb + r < N) dst[r] = v[r];
      }
    }
  }
}

// ================================================================= gemm_i8v2
// per_token / per_tensor activations: int8 act codes x int4 weight codes on
// v_mfma_i32_16x16x64_i8, per-weight-group fp32 fold, per-row act scale, salient tail on
// the D MFMA into the same accumulators.  128 x 128 tile, 4 waves as 2 (M) x 2 (N), each
// 64 x 64.  A stages hold 256 int8 codes (4 bpack blocks) per row: i8 sub-step t (one
// 64-code block) reads chunk 4 t + q; the activation codes were written in the K order
// that matches unpack_i8 of the bpack dword pair of lane group q.
struct StageA256 {
  uint32_t off, stride16;
  __device__ inline void init(int m0, size_t lda_b, int wave, int lane) {
    const int rin = 4 * wave + (lane >> 4);
    off = (uint32_t)((size_t)(m0 + rin) * lda_b + (((lane & 15) ^ (rin & 15)) << 4));
    stride16 = (uint32_t)(16 * lda_b);
  }
  __device__ inline void issue(const unsigned char* base, unsigned char* st, int wave) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) glds16(base + (size_t)i * stride16 + off, st + (i * 4 + wave) * 1024);
  }
};

__device__ inline const u32x4* a256_frag(const unsigned char* st, int row, int chunk) {
  return (const u32x4*)(st + row * 256 + ((chunk ^ (row & 15)) << 4));
}

template <class DT>
__global__ __launch_bounds__(256, 1) void gemm_i8v2_kernel(
    const int8_t* __restrict__ A8, const float* __restrict__ ascale,
    const typename DT::T* __restrict__ XS, const uint32_t* __restrict__ B4,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  constexpr int ST = 32768;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * ST];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, 8, tm, tn);
  const int m0 = tm * 128, n0 = tn * 128;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, q = lane >> 4;
  const int nkm = (Kp + 255) / 256;    // 256-code stages (the last may be partial)
  const int nks = S_pad / 128;         // 128-element salient stages
  const int nblk = Kp / 64;
  const int Np = pad_n(N);

  int nrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) nrow[j] = min(n0 + wn * 64 + j * 16 + r16, N - 1);

  f32x4 tot[4][4];
  i32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[i][j] = i32x4{0, 0, 0, 0};
    }

  const size_t brow_dw = (size_t)Kp / 8;
  uint2 bc[4][4], bn[4][4];
  auto load_codes = [&](int ks, uint2 (&b)[4][4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int blk = min(ks * 4 + t, nblk - 1);
        b[j][t] = *(const uint2*)(B4 + (size_t)nrow[j] * brow_dw + (size_t)blk * 8 + q * 2);
      }
  };
  auto fold = [&](int g) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wn * 64 + j * 16 + q * 4;
      float s[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) s[r] = DT::to_f(wscale[(size_t)g * Np + min(nb + r, N - 1)]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) tot[i][j][r] += (float)acc[i][j][r] * s[r];
        acc[i][j] = i32x4{0, 0, 0, 0};
      }
    }
  };
  auto compute_codes = [&](int ks, const unsigned char* st, const uint2 (&b)[4][4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int p_end = ks * 256 + (t + 1) * 64;
      if (p_end > Kp) break;  // partial last stage
      u32x4 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t l0, h0, l1, h1;
        unpack_i8(b[j][t].x, l0, h0);
        unpack_i8(b[j][t].y, l1, h1);
        bf[j] = u32x4{l0, h0, l1, h1};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x4 af = *a256_frag(st, wm * 64 + i * 16 + r16, 4 * t + q);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(*(const i32x4*)&bf[j], *(const i32x4*)&af, acc[i][j], 0, 0, 0);
      }
      if (p_end % Gw == 0 && p_end / Gw <= ngw) fold(p_end / Gw - 1);
    }
  };

  const int lda8 = nkm * 256;
  StageA256 sa;
  sa.init(m0, (size_t)lda8, wave, lane);
  const unsigned char* Ab = (const unsigned char*)A8;
  if (nkm > 0) {
    sa.issue(Ab, lds, wave);
    load_codes(0, bc);
    __syncthreads();
    for (int ks = 0; ks < nkm; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nkm) {
        sa.issue(Ab + (size_t)(ks + 1) * 256, lds + (cur ^ 1) * ST, wave);
        load_codes(ks + 1, bn);
      }
      compute_codes(ks, lds + cur * ST, bc);
      if (ks + 1 < nkm) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) bc[j][t] = bn[j][t];
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = min(m0 + wm * 64 + i * 16 + r16, M - 1);
    const float s = ascale[gm];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[i][j][r] *= s;
  }
  if (nks > 0) {
    StageA256 sx;
    sx.init(m0, (size_t)S_pad * sizeof(T), wave, lane);
    const unsigned char* Xb = (const unsigned char*)XS;
    sx.issue(Xb, lds, wave);
    __syncthreads();
    for (int ks = 0; ks < nks; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nks) sx.issue(Xb + (size_t)(ks + 1) * 128 * sizeof(T), lds + (cur ^ 1) * ST, wave);
      const unsigned char* st = lds + cur * ST;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        u32x4 bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bf[j] = *(const u32x4*)(wsal + (size_t)nrow[j] * S_pad + ks * 128 + 32 * s + 8 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u32x4 af = *a256_frag(st, wm * 64 + i * 16 + r16, 4 * s + q);
#pragma unroll
          for (int j = 0; j < 4; ++j) Mfma<DT>::run(tot[i][j], bf[j], af);
        }
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nb = n0 + wn * 64 + j * 16 + q * 4;
    if (nb >= N) continue;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = (bias && nb + r < N) ? DT::to_f(bias[nb + r]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gm = m0 + wm * 64 + i * 16 + r16;
      if (gm >= M) continue;
      T v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = DT::from_f(tot[i][j][r] + bv[r]);
      T* dst = Y + (size_t)gm * N + nb;
      if (nb + 4 <= N && (N & 3) == 0) {
        *(uint2*)dst = *(const uint2*)v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (nb + r < N) dst[r] = v[r];
      }
    }
  }
}

// ================================================================= launchers
template <class DT, int GB>
static int fq4_launch(const void* a, const void* codes, const void* wscale, const void* wsal,
                      const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                      int ngw, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, 256), tiles_n = cdiv(N, 256);
  gemm_fq4_kernel<DT, GB><<<dim3(tiles_m * tiles_n), dim3(512), 0, s>>>(
      (const T*)a, codes, (const T*)wscale, (const T*)wsal, (const T*)bias, (T*)y, M, N, Kp,
      S_pad, Gw, ngw, tiles_m, tiles_n);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT>
static int fq4_dispatch(const void* a, const void* codes, const void* wscale, const void* wsal,
                        const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                        int ngw, int n_bits, hipStream_t s) {
  if (n_bits == 0) return fq4_launch<DT, 0>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, 1, 1, s);
  if (n_bits != 4) return SQMP_EUNSUPPORTED;
  if (Gw % 64 == 0) return fq4_launch<DT, 1>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s);
  if (Gw == 32) return fq4_launch<DT, 2>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s);
  return SQMP_EUNSUPPORTED;
}

int launch_gemm_fq_fast(int dtype, const void* a, const void* codes, const void* wscale,
                        const void* wsal, const void* bias, void* y, int M, int N, int Kp,
                        int S_pad, int Gw, int ngw, int n_bits, hipStream_t s) {
  if (dtype == SQMP_F16)
    return fq4_dispatch<F16>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s);
  if (dtype == SQMP_BF16)
    return fq4_dispatch<BF16>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s);
  return SQMP_EUNSUPPORTED;
}

int launch_gemm_i8_fast(int dtype, const int8_t* a8, const float* ascale, const void* xs,
                        const void* codes, const void* wscale, const void* wsal,
                        const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                        int ngw, hipStream_t s) {
  const int tiles_m = cdiv(M, 128), tiles_n = cdiv(N, 128);
  if (dtype == SQMP_F16) {
    gemm_i8v2_kernel<F16><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
        a8, ascale, (const _Float16*)xs, (const uint32_t*)codes, (const _Float16*)wscale,
        (const _Float16*)wsal, (const _Float16*)bias, (_Float16*)y, M, N, Kp, S_pad, Gw, ngw,
        tiles_m, tiles_n);
  } else if (dtype == SQMP_BF16) {
    gemm_i8v2_kernel<BF16><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
        a8, ascale, (const __bf16*)xs, (const uint32_t*)codes, (const __bf16*)wscale,
        (const __bf16*)wsal, (const __bf16*)bias, (__bf16*)y, M, N, Kp, S_pad, Gw, ngw,
        tiles_m, tiles_n);
  } else {
    return SQMP_EUNSUPPORTED;
  }
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace sqmp
