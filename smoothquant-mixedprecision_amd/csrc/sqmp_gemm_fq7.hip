// gemm_fq7 -- the faithful W4A4 GEMM (fake_quant.py:306 F.linear on q_x and W_hat) with
// the int4 weight operand held in registers.
//
//   y[M][N] = D( A[M][Kp + S_pad] . W_hat^T + bias ),  A = x_hat in packed K order + the
//   exact salient columns (sqmp_quant_act_v2 OUT_FP), W_hat = D(code * scale) decoded in
//   registers (bit-exact with the reference's W_hat), then the exact salient weights.
//
// Why a second faithful kernel (gemm_fq6 stages A, the codes and the scales by LDS-DMA,
// 48 one-KiB pieces per 256 x 256 x 64 stage, and an LDS-DMA piece holds its wave's
// instruction stream for 60-185 cycles, MI355X_MICROARCH.md cycle table):
//   * TM x 512 output tile (TM = 128 or 64) per 512-thread workgroup, 8 waves as 1 x 8,
//     each TM x 64 on v_mfma_f32_16x16x32 -- half the A bytes per FLOP of a 256 x 256 tile;
//   * only A moves through LDS (16 pieces per stage at TM = 128, 4-slot ring, 3 stages in
//     flight).  Each wave's weight rows are private to it, so their codes, scales and
//     salient slice are loaded straight into VGPRs from a tile-major copy of the packed
//     weight (sqmp_pack_fq7): per stage a lane loads exactly its fragment bytes, 32 B of
//     codes + 8 B of scales (codes stages) or 128 B of salient weights (tail stages), one
//     stage ahead, with buffer loads whose per-stage offset is a scalar;
//   * every vector-memory op of the loop (the DMA and the register loads) is issued from
//     inline asm and waited for by hand-counted s_waitcnt vmcnt(N) (see gemm_fq6 for why
//     the compiler must not see the LDS-DMA), with an empty asm "fence" that ties each
//     loaded register to the wait before its first use.
// Fragment geometry (as gemm_fq6): lane (r16, q) of sub-step s (32 of a 64-position stage)
// takes bpack dword 2q + s of its weight row and A chunk c = 4 (q & 1) + 2 s + (q >> 1) --
// the positions 8c .. 8c + 7 of that dword.  The weight fragment goes in the MFMA's A
// slot, so acc[i][j][r] = C[n = n0 + 64 wave + 16 j + 4 q + r][m = m0 + 16 i + r16].
#include <stdlib.h>

#include <type_traits>

#include "sqmp_mfma.h"

namespace sqmp {
namespace fq7 {

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
// wave-uniform count -> immediate (waiting for more than needed is always safe)
__device__ inline void vmwait_dyn(int n) {
  switch (n) {
    case 1: vmwait<1>(); break;
    case 2: vmwait<2>(); break;
    case 3: vmwait<3>(); break;
    case 4: vmwait<4>(); break;
    case 5: vmwait<5>(); break;
    case 6: vmwait<6>(); break;
    case 7: vmwait<7>(); break;
    case 8: vmwait<8>(); break;
    case 9: vmwait<9>(); break;
    case 10: vmwait<10>(); break;
    case 11: vmwait<11>(); break;
    case 12: vmwait<12>(); break;
    case 16: vmwait<16>(); break;
    default: vmwait<0>(); break;
  }
}
__device__ inline void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // no LDS read moves above the barrier
  __builtin_amdgcn_sched_barrier(0);
}

// LDS-DMA of 16 B per lane to the wave-uniform LDS base + 16 * lane.  s_nop 0: the M0
// write -> LDS-DMA wait state (hipcc pads nothing inside an asm string).
__device__ inline void dma16(const rsrc_t& r, uint32_t voff, uint32_t soff, unsigned char* lds_dst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(
      (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m0v),
               "v"(voff), "s"(r), "s"(soff)
               : "memory", "m0");
}
// register loads, counted in vmcnt together with the DMA
template <int OFF>
__device__ inline void ld16(u32x4& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
               : "=v"(d)
               : "v"(voff), "s"(r), "s"(soff), "n"(OFF));
}
__device__ inline void ld8(u32x2& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(r), "s"(soff));
}
__device__ inline void ld4(uint32_t& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(r), "s"(soff));
}
__device__ inline void ld_s(u32x2& d, const rsrc_t& r, uint32_t voff, uint32_t soff) { ld8(d, r, voff, soff); }
__device__ inline void ld_s(uint32_t& d, const rsrc_t& r, uint32_t voff, uint32_t soff) { ld4(d, r, voff, soff); }
template <class V>
__device__ inline void fence(V& v) {
  asm volatile("" : "+v"(v));
}

// the lane index computed again where it is used (volatile: never merged with the kernel-entry
// value), so that lane-derived offsets of the salient tail and the epilogue are not live
// through the codes loop (OPT bit 3, 128 VGPRs)
__device__ inline int lane_now() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return (int)l;
}

__host__ __device__ inline int brev3(int c) { return ((c & 1) << 2) | (c & 2) | ((c >> 2) & 1); }

// Sibling problems of one grouped launch (sqmp_gemm_fq7_group): problem p owns the global
// tiles [tile_end[p - 1], tile_end[p]) and its own operands; M, Kp, S_pad, Gw, ngw are shared.
constexpr int FQ7_GRP_MAX = 4;
struct Fq7Grp {
  const void* A[FQ7_GRP_MAX];
  const uint32_t* Bt[FQ7_GRP_MAX];
  const void* St[FQ7_GRP_MAX];
  const void* Salt[FQ7_GRP_MAX];
  const void* bias[FQ7_GRP_MAX];
  void* Y[FQ7_GRP_MAX];
  uint32_t* colmax[FQ7_GRP_MAX];
  int N[FQ7_GRP_MAX], tiles_n[FQ7_GRP_MAX], tile_end[FQ7_GRP_MAX];
  int n;
};

// DIAG (timing diagnostics, wrong results by design, instantiated only in a SQMP_DIAG_BUILD;
// 0 = the product kernel): 1 no weight
// register loads after the prologue, 2 no A DMA after the prologue, 3 no int4 decode, 4 no
// per-stage barrier, 5 half the A fragment LDS reads (each fragment used for two blocks), 6 the
// A pieces written by ds_write_b128 from registers instead of LDS-DMA, 7 the A DMA from two
// L2-hot stages only, 8 the A loads into a scratch register (VMEM issue without the LDS write);
// activation-order (TR) epilogue: 9 none (the accumulators kept live, nothing staged or
// stored), 10 staged in LDS but not stored, 11 stored without the LDS staging writes
// J = 16-row weight tiles per wave: tile TM x TN with TN = 8 * 16 J (J = 4: 128 x 512;
// J = 2: 256 x 256, fq6's decode-optimal shape -- a decoded fragment feeds TM / 16 MFMAs)
// TR (sqmp_gemm_fqt on the tile-major activation operands): A = the permuted weight wp,
// the register operand = the activation codes / group scales / salient x in this kernel's
// tile-major layouts (sqmp_quant_act_c4 writes them so with ldsc < 0); kernel M = weight
// rows, kernel N = tokens, Y[n][m] stored transposed with the bias per kernel row.
// OPT (the activation-order launch, A/B knob SQMP_FQT7_OPT): bit 0 -- waves 4-7 run at
// s_setprio 1 through the K loop (MI355X_MICROARCH.md "Two waves per SIMD" item 4); bit 1 --
// loader split: waves 0-3 issue every LDS-DMA piece of a stage (their own and those of
// waves 4-7), waves 4-7 only wait, read and multiply (gemm_fq6's split); bit 2 -- A fragments
// read 3 blocks ahead instead of 2; bit 3 -- two workgroups per CU (128 VGPRs: DMA pieces
// i > 0 addressed through the scalar offset, the two fragment offsets kept instead of the lane
// index, which the salient tail and the epilogue compute again; spill-free at TM = 128 only,
// checked by tests/test_fq7_build_cpu.py)
// bit 4 -- K split inside the workgroup (packed order, TM = 128, J = 2, with bit 3's register
// budget): 1024 threads as two 8-wave halves on the same tile, half 0 the stages [0, h), half 1
// [h, nkt) with the salient tail, each on its own 4-slot ring (2 x 64 KiB); half 1 hands its
// fp32 accumulators to half 0 through LDS, half 0 adds them and runs the epilogue.  Sixteen
// waves per CU on one tile instead of eight: a one-tile-per-CU grid (2048-token Llama
// o_proj / down_proj) gets two waves per SIMD more, without a second tile's A and W traffic.
// The partial sums are added in a different order than in one pass (y within fp32 rounding
// of the unsplit kernel's, not bit-identical).
// GRP: a grouped launch over the problems of `grp` (A, Bt, St, Salt, bias, Y, colmax, N and
// tiles_n are taken from the block's problem; the other arguments are shared)
template <class DT, int GB, int TM, int J, int DIAG = 0, bool TR = false, int OPT = 0,
          bool GRP = false>
__global__ __launch_bounds__((OPT & 16) ? 1024 : 512, ((OPT & 8) && !(OPT & 16)) ? 4 : 1) void gemm_fq7_kernel(
    const typename DT::T* __restrict__ A, const uint32_t* __restrict__ Bt,
    const typename DT::T* __restrict__ St, const typename DT::T* __restrict__ Salt,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n, int group_m,
    uint32_t* __restrict__ colmax, int nt, const Fq7Grp grp) {
  typedef typename DT::T T;
  constexpr int I = TM / 16;            // 16 x 16 tiles per wave: TM rows x 16 J weight rows
  constexpr int TN = 128 * J, WR = 16 * J;  // tile width, weight rows per wave
  constexpr int PA = 3, NS = PA + 1;    // A stages in flight, ring slots
  constexpr int SLOT = TM * 128;        // TM rows x 64 positions x 2 B
  constexpr int NA = TM / 64;           // A pieces per wave per stage
  // A fragment read-ahead (blocks; 2 keeps the packed-order TM = 256 kernel spill-free;
  // OPT bit 2: 3 on the activation-order kernel)
  constexpr int PF = (TM == 256 && !(OPT & 4)) ? 2 : 3;
  constexpr int EPI = TR ? TN * (2 * TM + 16) : TM * TN * 2;  // epilogue staging bytes
  constexpr bool KS2 = (OPT & 16) != 0;  // K split over two 8-wave halves (bit 4)
  static_assert(!KS2 || (!TR && TM == 128 && J == 2 && (OPT & 8)), "bit 4: packed order, TM 128, J 2, bit 3");
  constexpr int NH = KS2 ? 2 : 1;                 // rings (halves)
  constexpr int PART = KS2 ? TM * TN * 4 : 0;     // half 1's fp32 accumulators
  constexpr int LDS0 = NH * NS * SLOT > EPI ? NH * NS * SLOT : EPI;
  constexpr int LDS_BYTES = LDS0 > PART ? LDS0 : PART;
  static_assert(J <= I, "sub-step 1 decode must finish before block I");
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

  int tm, tn;
  if constexpr (GRP) {
    // XCD-aware bijective remap over every problem's tiles, then the problem and its own
    // grouped raster (as tile_coords)
    const int nwg = grp.tile_end[grp.n - 1];
    const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    int p = 0;
#pragma unroll
    for (int i = 1; i < FQ7_GRP_MAX; ++i)
      if (i < grp.n && wg >= grp.tile_end[i - 1]) p = i;
    wg -= p > 0 ? grp.tile_end[p - 1] : 0;
    A = (const T*)grp.A[p];
    Bt = grp.Bt[p];
    St = (const T*)grp.St[p];
    Salt = (const T*)grp.Salt[p];
    bias = (const T*)grp.bias[p];
    Y = (T*)grp.Y[p];
    colmax = grp.colmax[p];
    N = grp.N[p];
    tiles_n = grp.tiles_n[p];
    const int per_group = group_m * tiles_n, gid = wg / per_group, first_m = gid * group_m;
    const int gsz = min(tiles_m - first_m, group_m), in_g = wg - gid * per_group;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
  } else {
    tile_coords(tiles_m, tiles_n, group_m, tm, tn);
  }
  const int m0 = tm * TM, n0 = tn * TN;
  const int lane = threadIdx.x & 63;
  const int wave_wg = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int half = KS2 ? wave_wg >> 3 : 0;        // (bit 4) this wave's K half
  const int wave = KS2 ? wave_wg & 7 : wave_wg;   // wave within its half
  const int tid = KS2 ? wave * 64 + lane : (int)threadIdx.x;  // thread within its half
  const int r16 = lane & 15, q = lane >> 4;
  const int lda = Kp + S_pad;
  const int nkm = Kp / 64, nks = S_pad / 64, nkt = nkm + nks;
  // this half's stages [k_lo, k_hi): bit 4 splits at an even h <= nkm - 2 near nkt / 2 (both
  // halves' codes stage counts stay even); the salient tail is half 1's
  const int hsplit = KS2 ? min(nkm - 2, (nkt / 2 + 1) & ~1) : nkt;
  const int k_lo = half == 1 ? hsplit : 0, k_hi = (KS2 && half == 0) ? hsplit : nkt;
  const int kc_hi = KS2 ? min(k_hi, nkm) : nkm;   // end of this half's codes stages
  const bool has_tail = KS2 ? k_hi > nkm : nks > 0;
  unsigned char* const ring = lds + half * (NS * SLOT);
  const int nb = tn * 8 + wave;  // this wave's WR-row weight block

  // ---- A (x_hat) by LDS-DMA: piece i of wave w = rows 64 i + 8 w + (lane >> 3), the lane
  // moving logical chunk brev3(p ^ ((row >> 1) & 7)) into physical chunk p = lane & 7
  constexpr bool SPLIT = (OPT & 2) != 0;
  constexpr int NO = SPLIT ? 2 : 1;       // waves whose pieces this wave issues
  const rsrc_t rA = make_rsrc(A + (size_t)m0 * lda);
  // (OPT bit 3: piece i > 0 is piece 0 moved by 64 i rows, through the scalar offset)
  constexpr int NAV = (OPT & 8) ? 1 : NA;
  uint32_t a_off[NO][NAV];
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    const int arow = 8 * (wave + 4 * o) + (lane >> 3);
#pragma unroll
    for (int i = 0; i < NAV; ++i)
      a_off[o][i] = (uint32_t)((size_t)(arow + 64 * i) * lda * sizeof(T)) +
                    (uint32_t)(brev3((lane & 7) ^ ((arow >> 1) & 7)) << 4);
  }
  // A pieces this wave issues per stage (the vmcnt of one stage's DMA)
  const int na_w = SPLIT ? (wave < 4 ? 2 * NA : 0) : NA;
  auto issue_a = [&](int kt) {
    if (kt < k_hi && (DIAG != 2 || kt < PA) && (!SPLIT || wave < 4)) {
      unsigned char* slot = ring + (kt % NS) * SLOT;
      const uint32_t so = (uint32_t)(DIAG == 7 ? (kt & 1) : kt) * 64 * sizeof(T);
#pragma unroll
      for (int o = 0; o < NO; ++o)
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          unsigned char* dst = slot + (i * 8 + wave + 4 * o) * 1024;
          if (DIAG == 8 && kt >= PA) {  // the same VMEM loads into a scratch register, no LDS write
            u32x4 sink;
            asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(sink)
                         : "v"(a_off[o][i]), "s"(rA), "s"(so));
            asm volatile("" ::"v"(sink));
          } else if (DIAG == 6 && kt >= PA) {  // the same LDS bytes written by ds_write_b128, no VMEM
            const u32x4 v = {a_off[o][i], so, 0u, 0u};
            const uint32_t la = (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)dst + lane * 16;
            asm volatile("ds_write_b128 %0, %1" ::"v"(la), "v"(v) : "memory");
          } else {
            if constexpr ((OPT & 8) != 0)
              dma16(rA, a_off[o][0], so + (uint32_t)(i * 64 * lda * (int)sizeof(T)), dst);
            else
              dma16(rA, a_off[o][i], so, dst);
          }
        }
    }
  };

  // ---- weight operand straight to registers (tile-major copies, sqmp_pack_fq7)
  // per wave block and stage: codes 512 J B, scales (per group) 32 J B, salient 2048 J B
  const rsrc_t rB = make_rsrc(Bt + (size_t)nb * nkm * (128 * J));
  const rsrc_t rS = make_rsrc(St + (size_t)nb * ngw * (16 * J));
  const rsrc_t rD = make_rsrc(Salt + (size_t)nb * (nks > 0 ? nks : 1) * (1024 * J));
  const uint32_t vB = (uint32_t)lane * (8u * J), vD = (uint32_t)lane * (32u * J);
  const uint32_t vS = (uint32_t)r16 * (2u * J);
  // one stage ahead: stage kt computes on register set kt & 1 (codes) / kd & 1 (salient
  // tail) while the next stage's loads land in the other set.  No value in flight is ever
  // copied (a copy the compiler placed before the wait would read the registers before
  // the load lands), so the loops are unrolled by two with compile-time set indices: Kp %
  // 128 == 0 makes the codes stage count even and the last codes stage odd.
  typedef typename std::conditional<J == 4, u32x2, uint32_t>::type SRegs;
  struct Codes {
    u32x4 w[J / 2];  // dwords [j][s] of rows 16 j + r16
    SRegs s;         // scales of rows 16 j + r16 (J x D)
  };
  struct Dense {
    u32x4 w[2 * J];  // chunk c(q, s) of rows 16 j + r16, [j][s]
  };

  auto issue_codes = [&](int kt, Codes& d) {
    if (DIAG == 1 && kt > 1) return;
    ld16<0>(d.w[0], rB, vB, (uint32_t)kt * (512u * J));
    if (J == 4) ld16<16>(d.w[J / 2 - 1], rB, vB, (uint32_t)kt * (512u * J));
    // Gw = 32: the lane's dwords lie in group 2 kt + (q & 1) (clamped: padding)
    const int g = GB == 1 ? min((kt * 64) / Gw, ngw - 1) : min(2 * kt + (q & 1), ngw - 1);
    const uint32_t vo = GB == 1 ? vS : (uint32_t)g * (32u * J) + vS;
    const uint32_t so = GB == 1 ? (uint32_t)g * (32u * J) : 0u;
    ld_s(d.s, rS, vo, so);
  };
  // salient stage kd, sub-step s: the fragments [j][s] (4 x 16 B per lane)
  auto issue_dense = [&](int kd, Dense& d, auto sc) {
    constexpr int S = decltype(sc)::value;
    const uint32_t so = (uint32_t)kd * (2048u * J);
    const uint32_t v = (OPT & 8) ? (uint32_t)lane_now() * (32u * J) : vD;
    ld16<16 * S>(d.w[S], rD, v, so);
    ld16<32 + 16 * S>(d.w[2 + S], rD, v, so);
    if (J == 4) {
      ld16<64 + 16 * S>(d.w[(4 + S) % (2 * J)], rD, v, so);
      ld16<96 + 16 * S>(d.w[(6 + S) % (2 * J)], rD, v, so);
    }
  };
  auto fence_codes = [&](Codes& d) {
#pragma unroll
    for (int u = 0; u < J / 2; ++u) fence(d.w[u]);
    fence(d.s);
  };

  f32x4 acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const DecK dk = make_deck();
  const int a_sw = (r16 >> 1) & 7;
  // A fragment of block t (sub-step s = t / I, row tile i = t % I)
  // (OPT bit 3: the lane's two sub-step offsets kept instead of the lane index)
  uint32_t a_lo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    a_lo[s] = (uint32_t)(r16 * 128 + ((brev3(4 * (q & 1) + 2 * s + (q >> 1)) ^ a_sw) << 4));
  auto ald = [&](const unsigned char* __restrict__ slot, int t) {
    if (DIAG == 5) t &= ~1;  // timing diagnostic: half the A fragment reads
    if constexpr ((OPT & 8) != 0) return *(const u32x4*)(slot + 16 * (t % I) * 128 + a_lo[t / I]);
    const int c = 4 * (q & 1) + 2 * (t / I) + (q >> 1);
    return *(const u32x4*)(slot + (16 * (t % I) + r16) * 128 + ((brev3(c) ^ a_sw) << 4));
  };
#define SQMP_FQ7_BLOCKS(BF, LD, ...)                                           \
  {                                                                            \
    u32x4 a[PF + 1];                                                           \
    _Pragma("unroll") for (int t = 0; t < PF; ++t) a[t] = LD(slot, t);         \
    _Pragma("unroll") for (int t = 0; t < 2 * I; ++t) {                        \
      if (t + PF < 2 * I) a[(t + PF) % (PF + 1)] = LD(slot, t + PF);           \
      _Pragma("unroll") for (int j = 0; j < J; ++j)                            \
          Mfma<DT>::run(acc[t % I][j], BF(t / I, j), a[t % (PF + 1)]);         \
      __VA_ARGS__;                                                             \
      __builtin_amdgcn_sched_barrier(0);                                       \
    }                                                                          \
  }

  auto compute_codes = [&](const unsigned char* __restrict__ slot, const Codes& cd) {
    uint32_t sb[4];
    if constexpr (J == 4) {
      sb[0] = cd.s.x & 0xFFFFu, sb[1] = cd.s.x >> 16, sb[2] = cd.s.y & 0xFFFFu, sb[3] = cd.s.y >> 16;
    } else {
      sb[0] = cd.s & 0xFFFFu, sb[1] = cd.s >> 16, sb[2] = 0u, sb[3] = 0u;
    }
    uint32_t sp[J];
#pragma unroll
    for (int j = 0; j < J; ++j) sp[j] = Dec<DT>::prep(sb[j]);
    u32x4 bf[2][J];
#pragma unroll
    for (int j = 0; j < J; ++j)
      bf[0][j] = DIAG == 3 ? u32x4{cd.w[j >> 1][(j & 1) * 2], sp[j], sp[j], sp[j]}
                           : (J == 4 ? Dec<DT>::run_lean(cd.w[j >> 1][(j & 1) * 2], sp[j], dk)
                                     : Dec<DT>::run(cd.w[j >> 1][(j & 1) * 2], sp[j], dk));
#define SQMP_BF7(s, j) bf[s][j]
    SQMP_FQ7_BLOCKS(SQMP_BF7, ald,
                    if (t < J) bf[1][t] = DIAG == 3 ? u32x4{cd.w[t >> 1][(t & 1) * 2 + 1], sp[t], sp[t], sp[t]}
                                                    : (J == 4 ? Dec<DT>::run_lean(cd.w[t >> 1][(t & 1) * 2 + 1], sp[t], dk)
                                                              : Dec<DT>::run(cd.w[t >> 1][(t & 1) * 2 + 1], sp[t], dk)));
#undef SQMP_BF7
  };
  // hook(t) runs after the MFMAs of block t (the mid-stage wait / issue at t = I - 1)
  auto compute_dense = [&](const unsigned char* __restrict__ slot, Dense& dd, auto hook) {
#define SQMP_BD7(s, j) dd.w[2 * (j) + (s)]
    SQMP_FQ7_BLOCKS(SQMP_BD7, ald, hook(t));
#undef SQMP_BD7
  };
#undef SQMP_FQ7_BLOCKS

  // ops issued after B(kt) when stage kt starts: A(kt - 1 + PA) (or, at kt = 0, the
  // prologue's A(1 .. PA-1)); A(kt) is older than B(kt) and so covered by the same wait
  auto wait_stage = [&](int kt) {
    const int n = kt == k_lo ? na_w * min(PA - 1, k_hi - k_lo - 1) : (kt - 1 + PA < k_hi ? na_w : 0);
    vmwait_dyn(n);
  };

  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;
  Codes cs[2];
  Dense dd;  // one set: sub-step 0 of stage kd + 1 lands while sub-step 1 of kd computes

  // prologue: A(k_lo), B(k_lo), A(k_lo + 1 .. k_lo + PA - 1)
  issue_a(k_lo);
  issue_codes(k_lo, cs[0]);
#pragma unroll
  for (int p = 1; p < PA; ++p) issue_a(k_lo + p);

  // codes stage kt on set P; the next codes stage's loads go to the other set, and after
  // the last codes stage the first salient stage's two sub-steps
  auto codes_step = [&](int kt, auto pc, bool last) {
    constexpr int P = decltype(pc)::value;
    wait_stage(kt);
    fence_codes(cs[P]);
    if (DIAG != 4) barrier();
    if (!last) issue_codes(kt + 1, cs[P ^ 1]);
    issue_a(kt + PA);
    compute_codes(ring + (kt % NS) * SLOT, cs[P]);
    if (last && has_tail) {
      issue_dense(0, dd, Z());
      issue_dense(0, dd, O());
    }
  };
  if ((OPT & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  int kt = k_lo;  // (even)
  for (; kt + 2 < kc_hi; kt += 2) {
    codes_step(kt, Z(), false);
    codes_step(kt + 1, O(), false);
  }
  codes_step(kt, Z(), false);
  codes_step(kt + 1, O(), true);
  kt += 2;
  // salient tail.  Issue order per stage kd: A(k + PA) at the top, sub-step 0 of kd + 1
  // after block I - 1, sub-step 1 of kd + 1 at the end; so at the top of stage kd the ops
  // younger than its sub-step 0 are its sub-step 1 (4), and at block I those younger
  // than its sub-step 1 are A(k + PA).
  for (int kd = 0; kd < (KS2 ? (has_tail ? nks : 0) : nks); ++kd) {
    const int k = nkm + kd;
    vmwait<J>();
#pragma unroll
    for (int j = 0; j < J; ++j) fence(dd.w[2 * j]);
    barrier();
    issue_a(k + PA);
    const bool more = kd + 1 < nks;
    compute_dense(ring + (k % NS) * SLOT, dd, [&](int t) {
      if (t == I - 1) {
        if (k + PA < nkt)
          vmwait_dyn(na_w);
        else
          vmwait<0>();
#pragma unroll
        for (int j = 0; j < J; ++j) fence(dd.w[2 * j + 1]);
        if (more) issue_dense(kd + 1, dd, Z());
      }
    });
    if (more) issue_dense(kd + 1, dd, O());
  }

  if constexpr (KS2) {
    // the two halves ran k_hi - k_lo per-stage barriers each: the shorter half adds the
    // difference, so that every s_barrier below pairs the same arrivals
    const int extra = (nkt - hsplit) - hsplit;
    for (int e = 0; e < (half == 0 ? extra : -extra); ++e) barrier();
  }
  // ---- epilogue: the TM x TN tile staged in LDS (row m: 2 TN bytes, 16-B chunk c at
  // c ^ (m & 15)), stored as whole rows, one 16-B chunk per lane
  if constexpr (TR && DIAG == 9) {
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < J; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  barrier();  // every wave is past its last read of the ring
  if constexpr (KS2) {
    // half 1's accumulators to half 0 through LDS (lane-contiguous f32x4: conflict-free)
    f32x4* part = (f32x4*)lds;
    if (half == 1) {
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) part[((wave * I + i) * J + j) * 64 + lane] = acc[i][j];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
    if (half == 0) {
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] += part[((wave * I + i) * J + j) * 64 + lane];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();  // the partials are read before the staging below overwrites them
  }
  if constexpr (TR) {
    // y^T staged [nl TN][ml TM] at a row stride of 2 TM + 16 bytes (the four q groups of a
    // write land 16 banks apart), stored as TM-wide row pieces of Y[n][m]
    constexpr int RS = 2 * TM + 16;
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int ml = 16 * i + r16;
      const float bv = bias && m0 + ml < M ? DT::to_f(bias[m0 + ml]) : 0.f;
      float cm = 0.f;  // |y| max of output column m0 + ml over this lane's tokens
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const T v = DT::from_f(acc[i][j][r] + bv);
          if (DIAG == 11)
            asm volatile("" ::"v"(v));
          else
            *(T*)(lds + (WR * wave + 16 * j + 4 * q + r) * RS + ml * 2) = v;
          if (colmax && n0 + WR * wave + 16 * j + 4 * q + r < N) cm = fmaxf(cm, fabsf(DT::to_f(v)));
        }
      if (colmax) {
        // fused output-quant statistics (sqmp_gemm_fqt7_colmax): max over the lane's tokens,
        // the four q lane groups, then one atomic per column and wave (bits of |y| order
        // like unsigned integers)
        cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
        if (q == 0 && m0 + ml < M) atomicMax(colmax + m0 + ml, __float_as_uint(cm));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
    constexpr int CPR = TM / 8;  // 16-B chunks per staged row
#pragma unroll 4
    for (int k = tid; k < TN * CPR; k += 512) {
      const int nl = k / CPR, c = k % CPR;
      const int gn = n0 + nl, gm = m0 + c * 8;
      if (gn < N && gm < M && DIAG != 10)  // M % 8 == 0 (launcher)
      {
        const u32x4 v = *(const u32x4*)(lds + nl * RS + c * 16);
        if (nt)  // streaming stores of a large output (nt_output)
          store16_nt(Y + (size_t)gn * M + gm, v);
        else
          *(u32x4*)(Y + (size_t)gn * M + gm) = v;
      }
    }
    return;
  }
  // (OPT bit 3: the lane index computed again here rather than kept live from the entry)
  const int el = (OPT & 8) ? lane_now() : lane;
  const int etid = wave * 64 + el, er16 = el & 15, eq = el >> 4;
  float cmx[J][4] = {};
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int nl = WR * wave + 16 * j + 4 * eq;  // first of the lane's 4 columns
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bv[r] = bias && n0 + nl + r < N ? DT::to_f(bias[n0 + nl + r]) : 0.f;
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int ml = 16 * i + er16;
      T v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = DT::from_f(acc[i][j][r] + bv[r]);
      if (colmax && m0 + ml < M) {
#pragma unroll
        for (int r = 0; r < 4; ++r) cmx[j][r] = fmaxf(cmx[j][r], fabsf(DT::to_f(v[r])));
      }
      const int c = nl >> 3;
      if (!KS2 || half == 0)
        *(u32x2*)(lds + ml * (TN * 2) + ((c ^ (ml & 15)) << 4) + (nl & 4) * 2) = *(const u32x2*)v;
    }
  }
  if (colmax && (!KS2 || half == 0)) {
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = cmx[j][r];
        v = fmaxf(v, __shfl_xor(v, 1, 64));
        v = fmaxf(v, __shfl_xor(v, 2, 64));
        v = fmaxf(v, __shfl_xor(v, 4, 64));
        v = fmaxf(v, __shfl_xor(v, 8, 64));
        const int n = n0 + WR * wave + 16 * j + 4 * eq + r;
        if (er16 == 0 && n < N) atomicMax(colmax + n, __float_as_uint(v));
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  barrier();
  constexpr int CPR = TN / 8, RPP = 512 / CPR;  // 16-B chunks per row, rows per pass
  const int c = etid % CPR;
  const bool cok = n0 + c * 8 < N;  // N % 8 == 0 (launcher)
#pragma unroll
  for (int k = 0; k < TM / RPP; ++k) {
    const int ml = RPP * k + etid / CPR;
    const int gm = m0 + ml;
    const u32x4 val = *(const u32x4*)(lds + ml * (TN * 2) + ((c ^ (ml & 15)) << 4));
    if (gm < M && cok && (!KS2 || half == 0)) {
      u32x4* dst = (u32x4*)(Y + (size_t)gm * N + n0 + c * 8);
      if (nt)  // streaming stores of a large output (nt_output)
        store16_nt(dst, val);
      else
        *dst = val;
    }
  }
}

// ---- tile-major copies of the packed weight (once per layer), blocks of WR = 16 J rows
// Bt[nb][kb][lane][j][s] (dwords) = bpack dword 2q + s of block kb of row WR nb + 16 j + r16
__global__ void pack_codes_kernel(const uint32_t* __restrict__ codes, uint32_t* __restrict__ Bt,
                                  int Np, int KB, int J, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int d = (int)(idx % (2 * J)), lane = (int)((idx / (2 * J)) & 63);
  const long rest = idx / (128 * J);
  const int kb = (int)(rest % KB);
  const long nbk = rest / KB;
  const int j = d >> 1, s = d & 1, q = lane >> 4, r16 = lane & 15;
  const long n = nbk * 16 * J + 16 * j + r16;
  Bt[idx] = n < Np ? codes[n * (KB * 8) + kb * 8 + 2 * q + s] : 0u;
}
// St[nb][g][r16][j] = wscale[g][WR nb + 16 j + r16]
template <class T>
__global__ void pack_scales_kernel(const T* __restrict__ wscale, T* __restrict__ St, int Np,
                                   int ngw, int J, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int j = (int)(idx % J), r16 = (int)((idx / J) & 15);
  const long rest = idx / (16 * J);
  const int g = (int)(rest % ngw);
  const long nbk = rest / ngw;
  const long n = nbk * 16 * J + 16 * j + r16;
  St[idx] = n < Np ? wscale[(long)g * Np + n] : (T)0.f;
}
// Salt[nb][kd][lane][j][s][e] = wsal[WR nb + 16 j + r16][64 kd + 8 c(q, s) + e]
template <class T>
__global__ void pack_sal_kernel(const T* __restrict__ wsal, T* __restrict__ Salt, int N,
                                int S_pad, int J, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int e = (int)(idx & 7), s = (int)((idx >> 3) & 1), j = (int)((idx >> 4) % J);
  const int lane = (int)((idx / (16 * J)) & 63);
  const int KS = S_pad / 64;
  const long rest = idx / (1024 * J);
  const int kd = (int)(rest % KS);
  const long nbk = rest / KS;
  const int q = lane >> 4, r16 = lane & 15;
  const int c = 4 * (q & 1) + 2 * s + (q >> 1);
  const long n = nbk * 16 * J + 16 * j + r16;
  Salt[idx] = n < N ? wsal[n * S_pad + kd * 64 + 8 * c + e] : (T)0.f;
}

// the packed-order launch: 4 row tiles per raster group (same box, 8 / 2 / 4 / 16 at
// 2048 x 4096 -> 4096 69.9 / 68.7 / 68.2 / 69.1 us, -> 11008 170.8 / 171.6 / 169.8 / 172.1,
// 2048 x 11008 -> 4096 173.3 / 172.8 / 171.6 / 176.7, config 2 in packed order 467.3 / 463.1
// / 459.6 / 473.6; profiles/r03_ab_group_m.txt); SQMP_FQ7_GROUP_M overrides
static int group_m_env() {  // (A/B knob; sqmp_knobs.hip)
  const char* e = knob("SQMP_FQ7_GROUP_M");
  return e && atoi(e) > 0 ? atoi(e) : 4;
}

// the activation-order (TR) launch: 4 weight-row tiles per raster group (same box, config 2:
// GEMM 422.5 vs 429.8 us at 8, alternating runs); SQMP_FQT7_GROUP_M overrides
static int group_m_tr_env() {  // (A/B knob; sqmp_knobs.hip)
  const char* e = knob("SQMP_FQT7_GROUP_M");
  return e && atoi(e) > 0 ? atoi(e) : 4;
}

// K split inside the workgroup (OPT bit 4) for the fp16 packed-order 128-row tiles, only where
// Kp >= 256 (each half at least two codes stages).  Default (1): grids of at most one 128-row
// tile per CU, i.e. where the unsplit kernel runs eight waves per CU -- same box, Llama-2-7B at
// 2048 tokens: o_proj 93.4 -> 89.8 us, down_proj 222.7 -> 211.6 us (profiles/r05_ab_fq7_ksplit.txt).
// 0 off; 2 every 128-row grid (q/k/v 214 -> 225 us: two unsplit workgroups per CU hide more);
// 3 as 2 and 128-row tiles for the grouped launches that take 256 (gate/up 338 -> 380 us).
// (A/B knob SQMP_FQ7_KS)
static int ks_env() {  // (A/B knob; sqmp_knobs.hip)
  const char* e = knob("SQMP_FQ7_KS");
  return e ? atoi(e) : 1;
}

// the packed-order launch's OPT variant (A/B knob, see gemm_fq7_kernel): default 3, same box
// (profiles/r03_ab_fq7_opt.txt): 2048 x 4096 -> 4096 67.2 -> 65.6 us, -> 11008 182.4 -> 181.9,
// 11008 -> 4096 164.5 -> 163.9, config 2 in packed order 461.2 -> 448.3
// 128-row tiles with more than one tile per CU: 8 (two workgroups per CU, 128 VGPRs), same
// box (profiles/r03_ab_fq7_two_wg_per_cu.txt): 2048 x 4096 -> 11008 179.5 -> 159.6 us; at one
// tile per CU (2048 x 4096 -> 4096, 2048 x 11008 -> 4096) within +-1 % of 3
static int opt_pk_env(int tm, long tiles, int kp) {  // (A/B knob; sqmp_knobs.hip)
  const char* e = knob("SQMP_FQ7_OPT");
  if (e) return atoi(e);
  const int ks = ks_env();
  if (tm == 128 && kp >= 256 && (ks >= 2 || (ks == 1 && tiles <= 256))) return 24;
  return tm == 128 && tiles > 256 ? 8 : 3;
}

// The OPT variant a packed-order launch of TM-row tiles actually instantiates (launch_k's
// switch: 8 / 9 need 128-row tiles, 24 also Kp >= 256; F16, J = 2, GB = 1 only -- else 0)
static int eff_opt_pk(bool f16_j2_gb1, int tm, long tiles, int kp) {
  if (!f16_j2_gb1) return 0;
  const int o = opt_pk_env(tm, tiles, kp);
  switch (o) {
    case 1: case 2: case 3: return o;
    case 8: return tm == 128 ? 8 : 0;
    case 9: return tm == 128 ? 9 : 3;
    case 24: return tm == 128 ? (kp >= 256 ? 24 : 8) : 3;
    default: return 0;
  }
}

// the activation-order launch's OPT variant (A/B knob, see gemm_fq7_kernel)
// default 3 (setprio + loader split): same box, interleaved rounds at config 2, 421.6 us
// against 431.4 us for 0 (either bit alone +-0.3 %, PF = 3 +-0.1 %; tools/ab_fqt7.py,
// profiles/r03_ab_fqt7.txt)
static int opt_tr_env() {  // (A/B knob; sqmp_knobs.hip)
  const char* e = knob("SQMP_FQT7_OPT");
  return e ? atoi(e) : 3;
}

#ifdef SQMP_DIAG_BUILD
// timing-diagnostic variants (wrong results by design) only in a diagnostics build:
// SQMP_DIAG=1 python smoothquant-mixedprecision_amd/build_ext.py --force
static int diag_env() {  // (A/B knob; sqmp_knobs.hip)
  const char* e = knob("SQMP_FQ7_DIAG");
  return e ? atoi(e) : 0;
}
#endif

template <class DT, int GB, int TM, int J, int DIAG = 0>
static int launch_k(const void* a, const void* bt, const void* st, const void* salt,
                  const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw, int ngw,
                  uint32_t* colmax, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, TM), tiles_n = cdiv(N, 128 * J);
  const int nt = nt_output((size_t)M * N * sizeof(T)) ? 1 : 0;
#define SQMP_PK(O)                                                                              \
  gemm_fq7_kernel<DT, GB, TM, J, DIAG, false, O><<<dim3(tiles_m * tiles_n), dim3((O) & 16 ? 1024 : 512), 0, s>>>( \
      (const T*)a, (const uint32_t*)bt, (const T*)st, (const T*)salt, (const T*)bias, (T*)y, M,  \
      N, Kp, S_pad, Gw, ngw, tiles_m, tiles_n, group_m_env(), colmax, nt, Fq7Grp{})
  // OPT variants (setprio for waves 4-7, loader split, two workgroups per CU, K split) for the
  // fp16 and bf16 J = 2 kernels, the 2048-token Llama GEMMs (A/B knob SQMP_FQ7_OPT, read per
  // launch)
  if constexpr ((std::is_same<DT, F16>::value || std::is_same<DT, BF16>::value) && J == 2 &&
                GB == 1 && DIAG == 0) {
    switch (eff_opt_pk(true, TM, (long)tiles_m * tiles_n, Kp)) {
      case 1: SQMP_PK(1); break;
      case 2: SQMP_PK(2); break;
      case 3: SQMP_PK(3); break;
      case 8: if constexpr (TM == 128) { SQMP_PK(8); } else { SQMP_PK(0); } break;
      case 9: if constexpr (TM == 128) { SQMP_PK(9); } else { SQMP_PK(3); } break;
      case 24:  // (the K split needs two codes stages per half: Kp >= 256)
        if constexpr (TM == 128) { if (Kp >= 256) { SQMP_PK(24); } else { SQMP_PK(8); } } else { SQMP_PK(3); }
        break;
      default: SQMP_PK(0); break;
    }
  } else {
    SQMP_PK(0);
  }
#undef SQMP_PK
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT, int GB, int TM, int J>
static int launch(const void* a, const void* bt, const void* st, const void* salt,
                  const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw, int ngw,
                  uint32_t* colmax, hipStream_t s) {
#define SQMP_L(D) launch_k<DT, GB, TM, J, D>(a, bt, st, salt, bias, y, M, N, Kp, S_pad, Gw, ngw, colmax, s)
#ifdef SQMP_DIAG_BUILD
  if (std::is_same<DT, F16>::value && GB == 1 && TM == 128 * 4 / J) {
    switch (diag_env()) {
      case 1: return SQMP_L(1);
      case 2: return SQMP_L(2);
      case 3: return SQMP_L(3);
      case 4: return SQMP_L(4);
      default: break;
    }
  }
#endif
  return SQMP_L(0);
#undef SQMP_L
}

// The row-tile height of a standalone packed-order launch (dispatch): J = 4: 128 x 512 tiles
// (64-row tiles when those leave CUs idle); J = 2: 256 x 256 (128 x 256 when those leave CUs
// idle; always 128 in bf16)
static int tm_standalone(bool bf16, int M, int N, int J) {
  if (J == 4) return (long)cdiv(M, 128) * cdiv(N, 512) >= 256 ? 128 : 64;
  return (!bf16 && (long)cdiv(M, 256) * cdiv(N, 256) >= 512) ? 256 : 128;
}

template <class DT>
static int dispatch(const void* a, const void* bt, const void* st, const void* salt,
                    const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                    int ngw, int J, uint32_t* colmax, hipStream_t s) {
  const int tm = J == 4 ? tm_standalone(false, M, N, J)
                        : ((long)cdiv(M, 256) * cdiv(N, 256) >= 512 ? 256 : 128);
  // (bf16 at 256 x 256 puts an array in scratch: 128-row tiles there)
  constexpr int TM2 = std::is_same<DT, BF16>::value ? 128 : 256;
#define SQMP_FQ7(GB)                                                                              \
  (J == 4 ? (tm == 128 ? launch<DT, GB, 128, 4>(a, bt, st, salt, bias, y, M, N, Kp, S_pad, Gw, ngw, colmax, s) \
                       : launch<DT, GB, 64, 4>(a, bt, st, salt, bias, y, M, N, Kp, S_pad, Gw, ngw, colmax, s))  \
          : (tm == 256 ? launch<DT, GB, TM2, 2>(a, bt, st, salt, bias, y, M, N, Kp, S_pad, Gw, ngw, colmax, s) \
                       : launch<DT, GB, 128, 2>(a, bt, st, salt, bias, y, M, N, Kp, S_pad, Gw, ngw, colmax, s)))
  if (Gw % 64 == 0) return SQMP_FQ7(1);
  if (Gw == 32) return SQMP_FQ7(2);
  return SQMP_EUNSUPPORTED;
#undef SQMP_FQ7
}

// The grouped packed-order launch (sqmp_gemm_fq7_group): J = 2, whole 64-blocks per weight
// group.  Row tiles of 256 where the problems' 256 x 256 tiles fill two rounds of the CUs, else
// of 128 (two workgroups per CU where that gives more than one tile per CU), as dispatch();
// SQMP_FQ7G_TM = 128 / 256 overrides (A/B, read per launch).
static int tm_group(bool bf16, int M, const int* Ns, int n) {
  long t256 = 0;
  for (int p = 0; p < n; ++p) t256 += (long)cdiv(M, 256) * cdiv(Ns[p], 256);
  int tm = t256 >= 512 && ks_env() < 3 ? 256 : 128;
  if (const char* e = knob("SQMP_FQ7G_TM")) tm = atoi(e) == 256 ? 256 : 128;
  return bf16 ? 128 : tm;  // (bf16 at 256 x 256 puts an array in scratch)
}
// the OPT variant dispatch_group launches
// (fp16 and bf16 alike; bf16 groups always take 128-row tiles, tm_group)
static int group_opt(int tm, long tiles, int kp) {
  if (tm == 256) return 3;
  const int o = opt_pk_env(128, tiles, kp);
  if (o == 24) return 24;
  return o == 8 ? 8 : 3;
}

template <class DT>
static int dispatch_group(Fq7Grp& g, int M, int Kp, int S_pad, int Gw, int ngw, int nt,
                          hipStream_t s) {
  typedef typename DT::T T;
  const int tm = tm_group(std::is_same<DT, BF16>::value, M, g.N, g.n);
  const int tiles_m = cdiv(M, tm);
  int end = 0;
  for (int p = 0; p < g.n; ++p) {
    g.tiles_n[p] = cdiv(g.N[p], 256);
    end += tiles_m * g.tiles_n[p];
    g.tile_end[p] = end;
  }
#define SQMP_G(TMV, O)                                                                          \
  gemm_fq7_kernel<DT, 1, TMV, 2, 0, false, O, true><<<dim3(end), dim3((O) & 16 ? 1024 : 512), 0, s>>>( \
      (const T*)nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, M, 0, Kp, S_pad, Gw, ngw, \
      tiles_m, 0, group_m_env(), nullptr, nt, g)
  switch (group_opt(tm, end, Kp)) {
    case 3:
      if (tm == 256) {
        if constexpr (std::is_same<DT, F16>::value) SQMP_G(256, 3);
      } else {
        SQMP_G(128, 3);
      }
      break;
    case 24: SQMP_G(128, 24); break;
    case 8: SQMP_G(128, 8); break;
    default: break;
  }
#undef SQMP_G
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

// the activation-order GEMM (TR): kernel M = weight rows N (wp rows), kernel N = tokens M
// J = 2: 256 weight rows x 256 tokens (8 waves of 32 tokens); J = 4: 128 weight rows x 512
// tokens (8 waves of 64 tokens: half the wp LDS-DMA and LDS fragment reads per MFMA, twice the
// act-code decode per MFMA)
template <class DT, int J>
static int dispatch_tr(const void* wp, const void* codes_t, const void* scale_t, const void* sal_t,
                       const void* bias, void* y, int M, int N, int Kq, int S_pad, int G, int ngq,
                       uint32_t* colmax, hipStream_t s) {
  typedef typename DT::T T;
  constexpr int TM = (J == 4 || std::is_same<DT, BF16>::value) ? 128 : 256;
  const int tiles_m = cdiv(N, TM), tiles_n = cdiv(M, 128 * J);
#define SQMP_TR(O)                                                                              \
  gemm_fq7_kernel<DT, 1, TM, J, 0, true, O><<<dim3(tiles_m * tiles_n), dim3(512), 0, s>>>(      \
      (const T*)wp, (const uint32_t*)codes_t, (const T*)scale_t, (const T*)sal_t, (const T*)bias, \
      (T*)y, N, M, Kq, S_pad, G, ngq, tiles_m, tiles_n, group_m_tr_env(), colmax, nt, Fq7Grp{})
  const int nt = nt_output((size_t)M * N * sizeof(T)) ? 1 : 0;
#ifdef SQMP_DIAG_BUILD
#define SQMP_TRD(D)                                                                             \
  gemm_fq7_kernel<DT, 1, TM, 2, D, true, 3><<<dim3(tiles_m * tiles_n), dim3(512), 0, s>>>(      \
      (const T*)wp, (const uint32_t*)codes_t, (const T*)scale_t, (const T*)sal_t, (const T*)bias, \
      (T*)y, N, M, Kq, S_pad, G, ngq, tiles_m, tiles_n, group_m_tr_env(), colmax, nt, Fq7Grp{})
  if (std::is_same<DT, F16>::value && J == 2 && diag_env() > 0) {
    switch (diag_env()) {
      case 1: SQMP_TRD(1); break;
      case 2: SQMP_TRD(2); break;
      case 3: SQMP_TRD(3); break;
      case 4: SQMP_TRD(4); break;
      case 5: SQMP_TRD(5); break;
      case 6: SQMP_TRD(6); break;
      case 7: SQMP_TRD(7); break;
      case 9: SQMP_TRD(9); break;
      case 10: SQMP_TRD(10); break;
      case 11: SQMP_TRD(11); break;
      default: SQMP_TRD(8); break;
    }
    SQMP_LAUNCH_CHECK();
    return SQMP_OK;
  }
#undef SQMP_TRD
#endif
  if constexpr (J == 4) {
    // setprio only (the loader split spills a VGPR at J = 4; OPT 0 / 4 / 5 measured within
    // 0.3 % of 1 at config 2, all 7 % slower than J = 2: profiles/r03_ab_fqt7_j4.txt)
    SQMP_TR(1);
  } else {
    switch (opt_tr_env()) {
      case 1: SQMP_TR(1); break;
      case 2: SQMP_TR(2); break;
      case 3: SQMP_TR(3); break;
      case 4: SQMP_TR(4); break;
      case 5: SQMP_TR(5); break;
#define SQMP_TR128(O)                                                                           \
  gemm_fq7_kernel<DT, 1, 128, 2, 0, true, O><<<dim3(cdiv(N, 128) * tiles_n), dim3(512), 0, s>>>( \
      (const T*)wp, (const uint32_t*)codes_t, (const T*)scale_t, (const T*)sal_t, (const T*)bias, \
      (T*)y, N, M, Kq, S_pad, G, ngq, cdiv(N, 128), tiles_n, group_m_tr_env(), colmax, nt, Fq7Grp{})
      // 128-row tiles at two workgroups per CU (OPT bit 3; 8, 9 spill at 128 VGPRs)
      case 10: if constexpr (TM == 256) { SQMP_TR128(10); } else { SQMP_TR(0); } break;
      case 11: if constexpr (TM == 256) { SQMP_TR128(11); } else { SQMP_TR(0); } break;
#undef SQMP_TR128
      default: SQMP_TR(0); break;  // 6, 7 (split + PF = 3) spill with the colmax epilogue
    }
  }
#undef SQMP_TR
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace fq7

// rows of the tile-major copies: N rounded up to the 128 J-row tile
static inline long fq7_rows(int N, int J) { return (N + 128L * J - 1) / (128L * J) * (128L * J); }

extern "C" int sqmp_fq7_sizes(int N, int Kp, int S_pad, int ngw, int J, size_t* codes_bytes,
                              size_t* scale_elems, size_t* sal_elems) {
  if (N <= 0 || Kp <= 0 || Kp % 64 || S_pad < 0 || S_pad % 64 || ngw <= 0) return SQMP_EINVAL;
  if (J != 2 && J != 4) return SQMP_EINVAL;
  const long R = fq7_rows(N, J);
  if (codes_bytes) *codes_bytes = (size_t)R * Kp / 2;
  if (scale_elems) *scale_elems = (size_t)R * ngw;
  if (sal_elems) *sal_elems = (size_t)R * (S_pad > 0 ? S_pad : 64);
  return SQMP_OK;
}

extern "C" int sqmp_pack_fq7(const void* codes, const void* wscale, const void* wsal, int dtype,
                             int N, int Kp, int S_pad, int ngw, int J, void* codes_t,
                             void* scale_t, void* sal_t, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!codes || !wscale || !codes_t || !scale_t || !sal_t || (S_pad > 0 && !wsal))
    return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (N <= 0 || Kp <= 0 || Kp % 64 || S_pad < 0 || S_pad % 64 || ngw <= 0) return SQMP_EINVAL;
  if (J != 2 && J != 4) return SQMP_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const long R = fq7_rows(N, J);
  const int Np = pad_n(N), KB = Kp / 64;
  const long tc = R * Kp / 8, ts = R * ngw;
  fq7::pack_codes_kernel<<<dim3((unsigned)cdiv(tc, 256)), dim3(256), 0, s>>>(
      (const uint32_t*)codes, (uint32_t*)codes_t, Np, KB, J, tc);
  SQMP_LAUNCH_CHECK();
  if (dtype == SQMP_F16)
    fq7::pack_scales_kernel<_Float16><<<dim3((unsigned)cdiv(ts, 256)), dim3(256), 0, s>>>(
        (const _Float16*)wscale, (_Float16*)scale_t, Np, ngw, J, ts);
  else
    fq7::pack_scales_kernel<__bf16><<<dim3((unsigned)cdiv(ts, 256)), dim3(256), 0, s>>>(
        (const __bf16*)wscale, (__bf16*)scale_t, Np, ngw, J, ts);
  SQMP_LAUNCH_CHECK();
  if (S_pad > 0) {
    const long tsl = R * S_pad;
    if (dtype == SQMP_F16)
      fq7::pack_sal_kernel<_Float16><<<dim3((unsigned)cdiv(tsl, 256)), dim3(256), 0, s>>>(
          (const _Float16*)wsal, (_Float16*)sal_t, N, S_pad, J, tsl);
    else
      fq7::pack_sal_kernel<__bf16><<<dim3((unsigned)cdiv(tsl, 256)), dim3(256), 0, s>>>(
          (const __bf16*)wsal, (__bf16*)sal_t, N, S_pad, J, tsl);
    SQMP_LAUNCH_CHECK();
  }
  return SQMP_OK;
}

extern "C" int sqmp_gemm_fq7(const void* a, const void* codes_t, const void* scale_t,
                             const void* sal_t, const void* bias, void* y, int dtype, int M,
                             int N, int Kp, int S_pad, int Gw, int ngw, int J, uint32_t* colmax,
                             void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!a || !codes_t || !scale_t || !sal_t || !y) return SQMP_EINVAL;
  if (M < 0 || N <= 0 || Kp <= 0 || Kp % 128 || S_pad < 0 || S_pad % 64 || Gw <= 0 || ngw <= 0)
    return SQMP_EINVAL;
  if (J != 2 && J != 4) return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (N % 8) return SQMP_EUNSUPPORTED;  // whole 16-B output chunks
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SQMP_F16)
    return fq7::dispatch<F16>(a, codes_t, scale_t, sal_t, bias, y, M, N, Kp, S_pad, Gw, ngw, J, colmax, s);
  return fq7::dispatch<BF16>(a, codes_t, scale_t, sal_t, bias, y, M, N, Kp, S_pad, Gw, ngw, J, colmax, s);
}

extern "C" int sqmp_gemm_fq7_group(const sqmp_fq7_problem* probs, int nprob, int dtype, int M,
                                   int Kp, int S_pad, int Gw, int ngw, int J, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!probs || nprob < 1 || nprob > fq7::FQ7_GRP_MAX) return SQMP_EINVAL;
  if (M < 0 || Kp <= 0 || Kp % 128 || S_pad < 0 || S_pad % 64 || Gw <= 0 || ngw <= 0)
    return SQMP_EINVAL;
  if (J != 2 || Gw % 64) return SQMP_EUNSUPPORTED;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  fq7::Fq7Grp g{};
  g.n = nprob;
  size_t ybytes = 0;
  for (int p = 0; p < nprob; ++p) {
    const sqmp_fq7_problem& q = probs[p];
    if (!q.a || !q.codes_t || !q.scale_t || !q.sal_t || !q.y || q.N <= 0) return SQMP_EINVAL;
    if (q.N % 8) return SQMP_EUNSUPPORTED;  // whole 16-B output chunks
    g.A[p] = q.a;
    g.Bt[p] = (const uint32_t*)q.codes_t;
    g.St[p] = q.scale_t;
    g.Salt[p] = q.sal_t;
    g.bias[p] = q.bias;
    g.Y[p] = q.y;
    g.colmax[p] = q.colmax;
    g.N[p] = q.N;
    const size_t yb = (size_t)M * q.N * 2;
    ybytes = yb > ybytes ? yb : ybytes;
  }
  if (M == 0) return SQMP_OK;
  const int nt = nt_output(ybytes) ? 1 : 0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SQMP_F16) return fq7::dispatch_group<F16>(g, M, Kp, S_pad, Gw, ngw, nt, s);
  return fq7::dispatch_group<BF16>(g, M, Kp, S_pad, Gw, ngw, nt, s);
}

// Which kernel variant sqmp_gemm_fq7 (nprob = 0: N[0] alone) or sqmp_gemm_fq7_group (nprob
// problems of N[0 .. nprob)) launches for these shapes: row-tile height and the OPT bits of
// gemm_fq7_kernel (bit 4 = the K split inside the workgroup, whose fp32 partial sums add in
// another order).  Test and tool use: which launches must agree bit for bit.
extern "C" int sqmp_fq7_plan(int dtype, int M, const int* N, int nprob, int Kp, int Gw, int J,
                             int* tm, int* opt) {
  if (!N || !tm || !opt || M <= 0 || Kp <= 0 || nprob < 0 || nprob > fq7::FQ7_GRP_MAX)
    return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  const bool bf16 = dtype == SQMP_BF16;
  if (nprob == 0) {
    const int t = fq7::tm_standalone(bf16, M, N[0], J);
    *tm = t;
    *opt = fq7::eff_opt_pk(J == 2 && Gw % 64 == 0, t, (long)cdiv(M, t) * cdiv(N[0], 128 * J), Kp);
    return SQMP_OK;
  }
  if (J != 2 || Gw % 64) return SQMP_EUNSUPPORTED;
  const int t = fq7::tm_group(bf16, M, N, nprob);
  long tiles = 0;
  for (int p = 0; p < nprob; ++p) tiles += (long)cdiv(M, t) * cdiv(N[p], 256);
  *tm = t;
  *opt = fq7::group_opt(t, tiles, Kp);
  return SQMP_OK;
}

// sqmp_gemm_fqt7: the activation-order GEMM (sqmp_gemm_fqt) on fq7's register-operand
// structure, its activation operands in the tile-major layout (J = 2) that sqmp_quant_act_c4
// writes when called with the SQMP_QA_TILED flag
static int gemm_fqt7_impl(const void* codes_t, const void* scale_t, const void* sal_t,
                          const void* wp, const void* bias, void* y, int dtype, int M, int N,
                          int Kq, int S_pad, int G, int ngq, int J, uint32_t* colmax,
                          void* stream) {
  if (!codes_t || !scale_t || !sal_t || !wp || !y) return SQMP_EINVAL;
  if (J != 2 && J != 4) return SQMP_EINVAL;
  if (M < 0 || N <= 0 || Kq <= 0 || Kq % 128 || S_pad < 0 || S_pad % 64 || G <= 0 || ngq <= 0)
    return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (G % 64 || N % 8) return SQMP_EUNSUPPORTED;
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
#define SQMP_DTR(DTT, JJ) \
  fq7::dispatch_tr<DTT, JJ>(wp, codes_t, scale_t, sal_t, bias, y, M, N, Kq, S_pad, G, ngq, colmax, s)
  if (dtype == SQMP_F16) return J == 4 ? SQMP_DTR(F16, 4) : SQMP_DTR(F16, 2);
  return J == 4 ? SQMP_DTR(BF16, 4) : SQMP_DTR(BF16, 2);
#undef SQMP_DTR
}

extern "C" int sqmp_gemm_fqt7(const void* codes_t, const void* scale_t, const void* sal_t,
                              const void* wp, const void* bias, void* y, int dtype, int M, int N,
                              int Kq, int S_pad, int G, int ngq, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  return gemm_fqt7_impl(codes_t, scale_t, sal_t, wp, bias, y, dtype, M, N, Kq, S_pad, G, ngq,
                        2, nullptr, stream);
}

// the same with the fused output-quant statistics (as sqmp_gemm_fq_colmax): colmax[n] =
// max(colmax[n], bits(|y[m][n]|)) over every row m
extern "C" int sqmp_gemm_fqt7_colmax(const void* codes_t, const void* scale_t, const void* sal_t,
                                     const void* wp, const void* bias, void* y, int dtype, int M,
                                     int N, int Kq, int S_pad, int G, int ngq, uint32_t* colmax,
                                     void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!colmax) return SQMP_EINVAL;
  return gemm_fqt7_impl(codes_t, scale_t, sal_t, wp, bias, y, dtype, M, N, Kq, S_pad, G, ngq,
                        2, colmax, stream);
}

// the general entry: J = 2 (SQMP_QA_TILED operands) or 4 (SQMP_QA_TILED4); colmax may be NULL
extern "C" int sqmp_gemm_fqt7j(const void* codes_t, const void* scale_t, const void* sal_t,
                               const void* wp, const void* bias, void* y, int dtype, int M, int N,
                               int Kq, int S_pad, int G, int ngq, int J, uint32_t* colmax,
                               void* stream) {
  SQMP_DEVICE_GUARD(stream);
  return gemm_fqt7_impl(codes_t, scale_t, sal_t, wp, bias, y, dtype, M, N, Kq, S_pad, G, ngq, J,
                        colmax, stream);
}

}  // namespace sqmp
