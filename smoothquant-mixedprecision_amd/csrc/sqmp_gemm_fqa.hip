// gemm_fqa -- the activation-order faithful W4A4 GEMM (fake_quant.py:306 F.linear on q_x and
// W_hat, the non-salient K - S columns in the batch's activation order plus the exact salient
// tail) with the roles of gemm_fqt7's operands swapped:
//
//   * the int4 act codes are decoded ONCE per workgroup: every lane of the 512-thread
//     workgroup decodes 16 codes of the 128-token x 64-position stage to D(code * scale) (the
//     reference's x_hat bit for bit) and writes them to an LDS f16 tile (3-slot ring);
//   * the permuted weight wp (D values, sqmp_quant_act_c4 + SQMP_QA_WPT writes it tile-major,
//     one 1-KiB piece per wave instruction) is the register operand: each wave owns 64 weight
//     rows and loads its 8 fragments per stage straight into VGPRs, one stage ahead;
//   * 128 tokens x 512 weight rows per workgroup, 8 waves of 128 tokens x 64 rows on
//     v_mfma_f32_16x16x32 (A = wp rows, B = the LDS act tile), 128 fp32 accumulators per lane.
//
// Against gemm_fqt7 (256 wp rows by LDS-DMA, each wave decoding its own 32 tokens): per MFMA
// half the LDS fragment reads (each act fragment feeds 4 MFMAs, each wp fragment in registers
// 8), half the int4 decode (a decoded value feeds 512 weight rows), no LDS-DMA in the codes
// stages (the salient tail's f16 x moves by LDS-DMA).  The cost is the register operand's
// L2 traffic: wp is fetched once per 128 tokens.
//
// Fragment geometry: sub-step h (32 of a 64-position stage) covers positions 32 h .. 32 h + 31;
// lane (r16, q) holds positions 32 h + 8 q .. + 7 of both operands, so
//   acc[i][j][r] = y[m0 + 16 i + r16][n0 + 64 wave + 16 j + 4 q + r].
// wpt layout (elements): [Nt / 64][nkt][4 row blocks rb][2 sub-steps h][64 lanes][8], lane
// (q, r16) of fragment (rb, h) = wp[64 nb + 16 rb + r16][64 kt + 32 h + 8 q .. + 7],
// nkt = (Kq + S_pad) / 64, Nt = roundup(N, 512).
// LDS act tile (per slot, 16 KiB): token t at byte 128 t, 16-B chunk c (positions 8 c .. + 7)
// at chunk c ^ ((t >> 1) & 7) -- conflict-free for the ds_read_b128 fragment reads.
#include <stdlib.h>

#include <type_traits>

#include "sqmp_mfma.h"

namespace sqmp {
namespace fqa {

typedef int rsrc_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// raw buffer resource, no range check (every offset stays inside its operand)
__device__ inline rsrc_t make_rsrc(const void* base) {
  const uint64_t a = (uint64_t)(size_t)base;
  rsrc_t r;
  r[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = (int)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xFFFFu);
  r[2] = -1;
  r[3] = 0x00020000;
  return r;
}
template <int N>
__device__ inline void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ inline void lgkwait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ inline void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // no LDS access moves across the barrier
  __builtin_amdgcn_sched_barrier(0);
}
// LDS-DMA of 16 B per lane to the wave-uniform LDS base + 16 * lane (s_nop 0: the M0 write ->
// LDS-DMA wait state; hipcc pads nothing inside an asm string)
__device__ inline void dma16(const rsrc_t& r, uint32_t voff, uint32_t soff, unsigned char* lds_dst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(
      (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m0v),
               "v"(voff), "s"(r), "s"(soff)
               : "memory", "m0");
}
// register loads, counted in vmcnt together with the DMA (waited for by hand)
template <int OFF>
__device__ inline void ld16(u32x4& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
               : "=v"(d)
               : "v"(voff), "s"(r), "s"(soff), "n"(OFF));
}
__device__ inline void ld8(u32x2& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(r), "s"(soff));
}
__device__ inline void ldu16(uint32_t& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_ushort %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(r), "s"(soff));
}
template <class V>
__device__ inline void fence(V& v) {
  asm volatile("" : "+v"(v));
}
// the lane index computed again where it is used (volatile: not kept live from kernel entry)
__device__ inline int lane_now() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return (int)l;
}

constexpr int NS = 3;   // act tile ring slots
constexpr int PF = 2;   // act fragment read-ahead (blocks)
constexpr int WSTG = 16384;  // per-wave epilogue staging: 128 accumulators x 64 lanes x 2 B

// chunk (8 positions) of bpack dword d of a 64-position block (sqmp_common.h bpack_pos)
__device__ inline int chunk_of(int d) { return 2 * (d & 3) + (d >> 2); }

// RB = 16-row weight blocks per wave (4: 128 tokens x 512 weight rows per workgroup, 8 waves of
// 128 tokens x 64 rows; 2: 256 tokens x 256 weight rows, 8 waves of 256 x 32).  TB = 32 / RB
// token blocks of 16 per wave keep 128 fp32 accumulators per lane either way: RB = 2 fetches
// the register operand half as often per FLOP (wp once per 256 tokens) but reads twice the LDS
// act tile per MFMA and decodes twice the codes per lane.
// OPT bit 0: waves 4-7 at s_setprio 1 through the K loop (MI355X_MICROARCH.md "Two waves per
// SIMD" item 4).
// DIAG (timing diagnostics, wrong results by design, SQMP_DIAG_BUILD only; 0 = the product
// kernel): 1 no wp register loads after the prologue, 2 no act decode / LDS writes after the
// prologue, 3 the decode without its LDS writes, 4 half the act fragment LDS reads (each used
// for two blocks), 5 no per-stage barrier
template <class DT, int RB, int OPT, int DIAG = 0>
__global__ __launch_bounds__(512, 1) void gemm_fqa_kernel(
    const unsigned char* __restrict__ codes, const typename DT::T* __restrict__ ascale,
    const typename DT::T* __restrict__ xs, const typename DT::T* __restrict__ wpt,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N, int Kq,
    int S_pad, int gsh, int ldsc, int tiles_t, int tiles_w, int group_m,
    uint32_t* __restrict__ colmax, int nt) {
  typedef typename DT::T T;
  constexpr int TB = 32 / RB, TT = 16 * TB, WR = 16 * RB, TW = 8 * WR;
  constexpr int SLOT = TT * 128;        // TT tokens x 64 positions x 2 B
  constexpr int LDS_BYTES = 8 * WSTG > NS * SLOT ? 8 * WSTG : NS * SLOT;
  constexpr int CPL = TT / 64;          // bpack dwords (8 codes) a decode lane takes per stage
  constexpr int LPT = 8 / CPL;          // decode lanes per token
  constexpr int XP = SLOT / 8192;       // salient-tail DMA pieces per wave and stage
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

  int tt, tw;
  tile_coords(tiles_t, tiles_w, group_m, tt, tw);
  const int m0 = tt * TT, n0 = tw * TW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int nkm = Kq / 64, nks = S_pad / 64, nkt = nkm + nks;
  const int nw0 = n0 + WR * wave;        // this wave's first weight row
  const int nb = nw0 >> 6, rb0 = (nw0 >> 4) & 3;  // its 64-row block of wpt, first row block

  // ---- wp: the register operand, 2 RB x 1 KiB per wave and stage (fragments (rb, h) of the
  // wave's rows: consecutive 1-KiB pieces from rb0)
  const rsrc_t rW = make_rsrc(wpt + (size_t)nb * nkt * 4096 + rb0 * 1024);
  const uint32_t vW = (uint32_t)lane * 16u;
  auto issue_w = [&](int kt, u32x4(&w)[2 * RB]) {
    if (DIAG == 1 && kt > 0) return;
    const uint32_t so = (uint32_t)kt * 8192u, so1 = so + 4096u;  // (12-bit instruction offsets)
    ld16<0>(w[0], rW, vW, so);
    ld16<1024>(w[1], rW, vW, so);
    ld16<2048>(w[2], rW, vW, so);
    ld16<3072>(w[3], rW, vW, so);
    if constexpr (RB == 4) {
      ld16<0>(w[4], rW, vW, so1);
      ld16<1024>(w[5], rW, vW, so1);
      ld16<2048>(w[6], rW, vW, so1);
      ld16<3072>(w[7], rW, vW, so1);
    }
  };

  // ---- act codes (row-major bpack rows of Kq / 2 bytes) + group scales [ngq][ldsc]: decode
  // lane (dt = token, dh) takes bpack dwords CPL dh .. CPL dh + CPL - 1 of its token's 64-block
  const int dt = tid / LPT, dh = tid % LPT, todd = dt & 1;
  const rsrc_t rC = make_rsrc(codes + (size_t)m0 * (Kq / 2));
  const rsrc_t rS = make_rsrc(ascale + m0);
  const uint32_t vC = (uint32_t)dt * (uint32_t)(Kq / 2) + (uint32_t)dh * (4u * CPL);
  const uint32_t vS = (uint32_t)dt * 2u;
  typedef typename std::conditional<CPL == 2, u32x2, u32x4>::type CRegs;
  struct Cd {
    CRegs c;
    uint32_t s;
  };
  auto issue_c = [&](int kt, Cd& d) {
    if (DIAG == 2 && kt > 1) return;
    if constexpr (CPL == 2)
      ld8(d.c, rC, vC, (uint32_t)kt * 32u);
    else
      ld16<0>(d.c, rC, vC, (uint32_t)kt * 32u);
    ldu16(d.s, rS, vS, (uint32_t)(((kt * 64) >> gsh) * ldsc) * (uint32_t)sizeof(T));
  };
  // write offset of this lane's e-th decoded dword (CPL = 2: odd tokens write their second
  // dword first, so the 8 lanes of a ds_write_b128 bank group cover 8 chunks)
  const int swz = (dt >> 1) & 7;
  const uint32_t wrow = (uint32_t)(dt * 128);
  auto wr_off = [&](int e) -> uint32_t {
    const int d = CPL * dh + (CPL == 2 ? (e ^ todd) : e);
    return wrow + (uint32_t)((chunk_of(d) ^ swz) << 4);
  };
  const DecK dk = make_deck();
  auto decode_one = [&](const Cd& d, int e) -> u32x4 {
    uint32_t w;
    if constexpr (CPL == 2)
      w = (e ^ todd) ? d.c.y : d.c.x;  // (a select: no run-time vector index)
    else
      w = d.c[e];
    return Dec<DT>::run(w, Dec<DT>::prep(d.s & 0xFFFFu), dk);
  };

  // ---- the salient tail's exact x by LDS-DMA: piece p = XP wave + i covers tokens 8 p .. 8 p +
  // 7, lane l moving logical chunk (l & 7) ^ swz(token) of token 8 p + (l >> 3) into physical
  // chunk l & 7
  const rsrc_t rX = make_rsrc(xs + (size_t)m0 * (S_pad > 0 ? S_pad : 1));
  auto issue_x = [&](int kd, unsigned char* slot) {
    const int l = lane_now();  // (recomputed: not live through the codes stages)
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int row = 8 * (XP * wave + i) + (l >> 3);
      const uint32_t xo = (uint32_t)((row * S_pad + 8 * ((l & 7) ^ ((row >> 1) & 7))) * (int)sizeof(T));
      dma16(rX, xo, (uint32_t)kd * 64u * (uint32_t)sizeof(T), slot + (XP * wave + i) * 1024);
    }
  };

  f32x4 acc[TB][RB];
#pragma unroll
  for (int i = 0; i < TB; ++i)
#pragma unroll
    for (int j = 0; j < RB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // act fragment t = TB h + i: token block i, sub-step h
  const int rsw = (r16 >> 1) & 7;
  const uint32_t ro0 = (uint32_t)(r16 * 128 + ((q ^ rsw) << 4));
  const uint32_t ro1 = (uint32_t)(r16 * 128 + (((4 + q) ^ rsw) << 4));
  auto bld = [&](const unsigned char* __restrict__ slot, int t) {
    if (DIAG == 4) t &= ~1;
    return *(const u32x4*)(slot + (t % TB) * 2048 + ((t / TB) ? ro1 : ro0));
  };

  u32x4 W[2][2 * RB];
  Cd cd[2];

  // prologue: codes(0) -> decode -> slot 0 (Kq = 0, a dense GEMM: x(0) by DMA); wp(0); codes(1)
  if (nkm > 0)
    issue_c(0, cd[0]);
  else
    issue_x(0, lds);
  issue_w(0, W[0]);
  issue_c(nkm > 1 ? 1 : 0, cd[1]);
  vmwait<2 * RB + 2>();
  if (nkm > 0) {
    fence(cd[0].c);
    fence(cd[0].s);
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      const u32x4 v = decode_one(cd[0], e);
      *(u32x4*)(lds + wr_off(e)) = v;
    }
  }
  if ((OPT & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);

  // stage kt on register sets P (wp) / P ^ 1 (the codes of stage kt + 1).  Every stage in the
  // loop issues the same register loads (addresses clamped past the end: those values are
  // live around the back edge, so their registers stay reserved while the loads fly); the
  // stage after the loop (LAST, nkt odd) issues none -- a dead asm output's register could be
  // reused while its load is still in flight.
  int sc = 0;  // kt % NS
  constexpr int NBLK = 2 * TB;  // MFMA blocks per stage (RB MFMAs each)
  auto stage = [&](int kt, auto pc, auto lastc) {
    constexpr int P = decltype(pc)::value;
    constexpr bool LAST = decltype(lastc)::value;
    vmwait<0>();
    lgkwait0();
#pragma unroll
    for (int f = 0; f < 2 * RB; ++f) fence(W[P][f]);
    fence(cd[P ^ 1].c);
    fence(cd[P ^ 1].s);
    if (DIAG != 5) barrier();  // slot sc complete (decode writes / DMA of the previous stage)
    const int sn = sc == NS - 1 ? 0 : sc + 1;
    const unsigned char* __restrict__ slot = lds + sc * SLOT;
    unsigned char* nslot = lds + sn * SLOT;
    const bool dec = kt + 1 < nkm && (DIAG != 2 || kt < 1);
    const bool dma = kt + 1 >= nkm && kt + 1 < nkt;
    if constexpr (!LAST) {
      if (dma) issue_x(kt + 1 - nkm, nslot);
      issue_w(kt + 1 < nkt ? kt + 1 : kt, W[P ^ 1]);
      issue_c(kt + 2 < nkm ? kt + 2 : (nkm > 0 ? nkm - 1 : 0), cd[P]);
    }
    u32x4 b[PF + 1];
    u32x4 dv;
#pragma unroll
    for (int t = 0; t < PF; ++t) b[t] = bld(slot, t);
#pragma unroll
    for (int t = 0; t < NBLK; ++t) {
      if (t + PF < NBLK) b[(t + PF) % (PF + 1)] = bld(slot, t + PF);
#pragma unroll
      for (int j = 0; j < RB; ++j)
        Mfma<DT>::run(acc[t % TB][j], W[P][2 * j + t / TB], b[t % (PF + 1)]);
      if (dec) {
        // decode dword e at block 4 e + 1, its LDS write at block 4 e + 3
#pragma unroll
        for (int e = 0; e < CPL; ++e) {
          if (t == 4 * e + 1) dv = decode_one(cd[P ^ 1], e);
          if (t == 4 * e + 3 && DIAG != 3) *(u32x4*)(nslot + wr_off(e)) = dv;
          if (t == 4 * e + 3 && DIAG == 3) fence(dv);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    sc = sn;
  };
  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;
  using NL = std::integral_constant<bool, false>;
  using L1 = std::integral_constant<bool, true>;
  int kt = 0;
  for (; kt + 1 < nkt; kt += 2) {
    stage(kt, Z(), NL());
    stage(kt + 1, O(), NL());
  }
  if (kt < nkt) stage(kt, Z(), L1());

  // ---- epilogue: each wave stages its TT x WR tile in its own 16-KiB region (token row of 2 WR
  // bytes, 8-B unit u = 4 j + q at u ^ (token % (4 RB))), then stores whole row pieces, one 16-B
  // chunk per lane
  vmwait<0>();
  lgkwait0();
  barrier();  // every wave is past its last read of the ring
  if ((OPT & 1) && wave >= 4) __builtin_amdgcn_s_setprio(0);
  constexpr int RS = 2 * WR, UM = 4 * RB - 1;  // staged row bytes, unit swizzle mask
  unsigned char* st = lds + wave * WSTG;
  float cm[RB][4];
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nw0 + 16 * j + 4 * q + r;
      bv[r] = bias && n < N ? DT::to_f(bias[n]) : 0.f;
      cm[j][r] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      const int tl = 16 * i + r16;
      T v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = DT::from_f(acc[i][j][r] + bv[r]);
      if (colmax && m0 + tl < M) {
#pragma unroll
        for (int r = 0; r < 4; ++r) cm[j][r] = fmaxf(cm[j][r], fabsf(DT::to_f(v[r])));
      }
      *(u32x2*)(st + tl * RS + (((4 * j + q) ^ (tl & UM)) << 3)) = *(const u32x2*)v;
    }
  }
  if (colmax) {
    // fused output-quant statistics (as sqmp_gemm_fq_colmax): max over the lane's tokens, then
    // the 16 token lanes, one atomic per column and wave (bits of |y| order like unsigned ints)
#pragma unroll
    for (int j = 0; j < RB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = cm[j][r];
        v = fmaxf(v, __shfl_xor(v, 1, 64));
        v = fmaxf(v, __shfl_xor(v, 2, 64));
        v = fmaxf(v, __shfl_xor(v, 4, 64));
        v = fmaxf(v, __shfl_xor(v, 8, 64));
        const int n = nw0 + 16 * j + 4 * q + r;
        if (r16 == 0 && n < N) atomicMax(colmax + n, __float_as_uint(v));
      }
  }
  lgkwait0();  // the wave's own staging writes (no other wave reads this region)
  constexpr int CPR = RS / 16, RPI = 64 / CPR;  // 16-B chunks per staged row, rows per pass
  const int v8 = lane % CPR;
  const bool nok = nw0 + 8 * v8 < N;  // N % 8 == 0 (launcher)
#pragma unroll 4
  for (int it = 0; it < TT / RPI; ++it) {
    const int row = RPI * it + lane / CPR, s = row & UM;
    const u32x4 a = *(const u32x4*)(st + row * RS + ((v8 ^ (s >> 1)) << 4));
    const u32x4 val = (s & 1) ? u32x4{a[2], a[3], a[0], a[1]} : a;
    if (m0 + row < M && nok) {
      T* dst = Y + (size_t)(m0 + row) * N + nw0 + 8 * v8;
      if (nt)  // streaming stores of a large output (nt_output)
        store16_nt(dst, val);
      else
        *(u32x4*)dst = val;
    }
  }
}

// ---- tile-major wp for a dense f16 operand (the dense-core A/B: `tools/dense_core.py`)
// wpt[nb][kt][rb][h][lane][8] = w[64 nb + 16 rb + r16][64 kt + 32 h + 8 q .. + 7]
template <class T>
__global__ void pack_wpt_kernel(const T* __restrict__ w, T* __restrict__ wpt, int N, int L,
                                long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one 16-B chunk
  if (idx >= total) return;
  const int lane = (int)(idx & 63), h = (int)((idx >> 6) & 1), rb = (int)((idx >> 7) & 3);
  const long rest = idx >> 9;
  const int nkt = L / 64;
  const int kt = (int)(rest % nkt);
  const long nbk = rest / nkt;
  const long n = nbk * 64 + 16 * rb + (lane & 15);
  const int k = 64 * kt + 32 * h + 8 * (lane >> 4);
  u32x4 v = u32x4{0u, 0u, 0u, 0u};
  if (n < N) v = *(const u32x4*)(w + n * L + k);
  *(u32x4*)(wpt + idx * 8) = v;
}

// SQMP_FQA_RB = 2 / 4 (A/B knob): 16-row weight blocks per wave, default 4
static int rb_knob() {
  const char* e = knob("SQMP_FQA_RB");
  return e && atoi(e) == 2 ? 2 : 4;
}
#ifdef SQMP_DIAG_BUILD
static int diag_knob() {
  const char* e = knob("SQMP_FQA_DIAG");
  return e ? atoi(e) : 0;
}
#endif

// the launch: XCD x runs all token tiles of a weight-row tile (group_m = every token tile): the
// 32 concurrent workgroups of an XCD stream the same wp rows through its L2
template <class DT, int RB>
static int launch(const void* codes, const void* ascale, const void* xs, const void* wpt,
                  const void* bias, void* y, int M, int N, int Kq, int S_pad, int gsh, int ldsc,
                  uint32_t* colmax, hipStream_t s) {
  typedef typename DT::T T;
  constexpr int TT = 16 * (32 / RB), TW = 128 * RB;
  const int tiles_t = cdiv(M, TT), tiles_w = cdiv(N, TW);
  const int nt = nt_output((size_t)M * N * sizeof(T)) ? 1 : 0;
#define SQMP_FQA_L(D)                                                                           \
  gemm_fqa_kernel<DT, RB, 1, D><<<dim3(tiles_t * tiles_w), dim3(512), 0, s>>>(                  \
      (const unsigned char*)codes, (const T*)ascale, (const T*)xs, (const T*)wpt, (const T*)bias, \
      (T*)y, M, N, Kq, S_pad, gsh, ldsc, tiles_t, tiles_w, tiles_t, colmax, nt)
#ifdef SQMP_DIAG_BUILD
  if (std::is_same<DT, F16>::value) {
    switch (diag_knob()) {
      case 1: SQMP_FQA_L(1); SQMP_LAUNCH_CHECK(); return SQMP_OK;
      case 2: SQMP_FQA_L(2); SQMP_LAUNCH_CHECK(); return SQMP_OK;
      case 3: SQMP_FQA_L(3); SQMP_LAUNCH_CHECK(); return SQMP_OK;
      case 4: SQMP_FQA_L(4); SQMP_LAUNCH_CHECK(); return SQMP_OK;
      case 5: SQMP_FQA_L(5); SQMP_LAUNCH_CHECK(); return SQMP_OK;
      default: break;
    }
  }
#endif
  SQMP_FQA_L(0);
#undef SQMP_FQA_L
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT>
static int dispatch(const void* codes, const void* ascale, const void* xs, const void* wpt,
                    const void* bias, void* y, int M, int N, int Kq, int S_pad, int gsh, int ldsc,
                    uint32_t* colmax, hipStream_t s) {
  if (rb_knob() == 2)
    return launch<DT, 2>(codes, ascale, xs, wpt, bias, y, M, N, Kq, S_pad, gsh, ldsc, colmax, s);
  return launch<DT, 4>(codes, ascale, xs, wpt, bias, y, M, N, Kq, S_pad, gsh, ldsc, colmax, s);
}

}  // namespace fqa

extern "C" size_t sqmp_fqa_wpt_elems(int N, int Kq, int S_pad) {
  if (N <= 0 || Kq < 0 || S_pad < 0) return 0;
  return (size_t)((N + 511) / 512 * 512) * (size_t)(Kq + S_pad);
}

extern "C" int sqmp_gemm_fqa(const void* acodes, const void* ascale, const void* xs,
                             const void* wpt, const void* bias, void* y, int dtype, int M, int N,
                             int Kq, int S_pad, int G, int ldsc, uint32_t* colmax, void* stream) {
  // Kq = 0: a dense GEMM y = xs . wpt^T (the dense-core measurement; acodes / ascale unused)
  if (Kq == 0) acodes = ascale = xs;
  if (!acodes || !ascale || !wpt || !y || (S_pad > 0 && !xs)) return SQMP_EINVAL;
  if (M < 0 || N <= 0 || Kq < 0 || Kq % 64 || S_pad < 0 || S_pad % 64 || G <= 0) return SQMP_EINVAL;
  if (Kq + S_pad == 0) return SQMP_EINVAL;
  if (ldsc < (M + 255) / 256 * 256) return SQMP_EINVAL;  // (256-token tiles at RB = 2)
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (G % 64 || (G & (G - 1)) || N % 8) return SQMP_EUNSUPPORTED;
  // 32-bit buffer offsets: the codes / xs rows of one tile and a wave's wp block
  if ((long)(Kq + S_pad) * 64 * 2 * 2 >= (1L << 31)) return SQMP_EUNSUPPORTED;
  if (M == 0) return SQMP_OK;
  int gsh = 0;
  while ((1 << gsh) < G) ++gsh;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SQMP_F16)
    return fqa::dispatch<F16>(acodes, ascale, xs, wpt, bias, y, M, N, Kq, S_pad, gsh, ldsc, colmax, s);
  return fqa::dispatch<BF16>(acodes, ascale, xs, wpt, bias, y, M, N, Kq, S_pad, gsh, ldsc, colmax, s);
}

// dense W [N][L] (L % 64 == 0) -> the wpt layout (rows roundup(N, 512), zeros past N)
extern "C" int sqmp_pack_wpt(const void* w, int dtype, int N, int L, void* wpt, void* stream) {
  if (!w || !wpt || N <= 0 || L <= 0 || L % 64) return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  const long total = (long)((N + 511) / 512 * 512) * L / 8;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SQMP_F16)
    fqa::pack_wpt_kernel<_Float16><<<dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s>>>(
        (const _Float16*)w, (_Float16*)wpt, N, L, total);
  else
    fqa::pack_wpt_kernel<__bf16><<<dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s>>>(
        (const __bf16*)w, (__bf16*)wpt, N, L, total);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace sqmp
