// gemm_fqt8 -- the activation-order faithful GEMM (sqmp_gemm_fqt7's operands and numerics:
// y = D(x_hat . W_hat^T + bias), fake_quant.py:306, computed as y^T = wp . codes^T with the
// act codes decoded in registers to D(code * scale) = the reference's x_hat bit for bit) at ONE
// wave per SIMD.
//
// Why ("What bounds the activation-order GEMM"): fqt7 runs 8 waves of 256 wp
// rows x 32 tokens (two waves per SIMD, 128 fp32 accumulators each), so every wave reads the
// whole 256-row wp tile from LDS per stage: 256 KiB of LDS reads per CU per 64-position stage,
// and 0.8 decode VALU per MFMA.  Here 4 waves own 256 wp rows x 64 tokens each (the whole
// 512-entry register file: 256 accumulators in AGPRs, the operands in VGPRs): the same 256 x
// 256 tile per CU, half the LDS reads per MFMA (128 KiB per stage) and half the decode per
// MFMA, the same wp DMA (32 one-KiB pieces per stage, 8 per wave).
//
// With no partner wave on the SIMD, nothing hides a stall but the schedule itself, so it is
// written out: per stage 32 blocks (block t = wp row tile t % 16 of sub-step t / 16), each one
// LDS fragment read PF = 3 blocks ahead and 4 MFMAs (one per 16-token tile);
//   blocks 4-7     decode the stage's sub-step-1 act fragments (4 x bpack dword -> 8 halves)
//   block 8        issues stage kt + 2's act operand into the registers just decoded
//   blocks 1..15   (odd) the 8 LDS-DMA pieces of stage kt + 2 (3-slot ring)
//   block 19       the counted vmcnt that retires stage kt + 1's act operand and DMA pieces,
//                  then its scales prepared
//   blocks 20-23   decode the NEXT stage's sub-step-0 fragments (so a stage opens on MFMAs)
// and one s_barrier per stage.  The code stages whose next two are code stages run with every
// kind known at compile time (no branches in that loop); the last code stages and the salient
// ones run the same stage with the kinds tested at run time.  The 256 accumulators are literal
// AGPRs (below); hipcc pads no hazard inside an asm statement: the fragments an MFMA reads are
// written >= 12 blocks earlier (decode) or waited for by hipcc's own lgkmcnt (LDS reads, which
// it sees as operands), accumulators chain MFMA -> MFMA only (0 states), and the epilogue reads
// them after an explicit s_nop pad.
//
// Measured (config 2): 443 us vs sqmp_gemm_fqt7's 417 us on the same
// box -- bit-identical results, opt-in (SQMP_FQT8=1).  Its timing diagnostics put the MFMA-only
// floor of this tiling at 292 us; the wp DMA (+47 us), the act decode (+58 us) and the LDS
// fragment reads (+34 us) each overflow the 8 free issue cycles of a 16-cycle 16x16x32 MFMA gap
// at one wave per SIMD, where fqt7's partner wave hides them.
//
// Operands: wp [roundup(N, 256)][Kq + S_pad] (sqmp_quant_act_c4's permuted weight) by
// LDS-DMA; the act codes / group scales / salient x in the SQMP_QA_TILED4 tile-major layouts
// (64-token blocks, sqmp_pack_fq7's J = 4 order) straight to VGPRs.  Kq % 128 == 0,
// S_pad % 64 == 0, G % 64 == 0, N % 8 == 0, fp16 / bf16.
#include <stdlib.h>

#include <type_traits>

#include "sqmp_mfma.h"

namespace sqmp {
namespace fqt8 {

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
__device__ inline void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // no LDS read moves above the barrier
  __builtin_amdgcn_sched_barrier(0);
}

// LDS-DMA of 16 B per lane to the wave-uniform LDS base + 16 * lane (s_nop 0: M0 write ->
// LDS-DMA wait state; hipcc pads nothing inside an asm string)
__device__ inline void dma16(const rsrc_t& r, uint32_t voff, uint32_t soff, uint32_t lds_addr) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m0v),
               "v"(voff), "s"(r), "s"(soff)
               : "memory", "m0");
}
// register loads, counted in vmcnt together with the DMA (hipcc does not see them)
template <int OFF>
__device__ inline void ld16(u32x4& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
               : "=v"(d)
               : "v"(voff), "s"(r), "s"(soff), "n"(OFF));
}
__device__ inline void ld8(u32x2& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(r), "s"(soff));
}
// ties a loaded register to the wait before its first use (no copy of it above the wait)
template <class V>
__device__ inline void fence(V& v) {
  asm volatile("" : "+v"(v));
}
// wave-uniform count -> immediate (waiting for more than needed is always safe)
__device__ inline void vmwait_dyn(int n) {
  switch (n) {
    case 16: vmwait<16>(); break;
    case 11: vmwait<11>(); break;
    default: vmwait<0>(); break;
  }
}

__host__ __device__ inline int brev3(int c) { return ((c & 1) << 2) | (c & 2) | ((c >> 2) & 1); }

// The 256 accumulators live in FIXED accumulator registers a[0:255], named literally in the
// MFMA statements: hipcc never sees them as values, so it cannot move them (with "+a" operands
// it homed the loop-carried accumulators in VGPRs and copied them to AGPRs around every use).
// acc_init() claims all 256 (its clobber list makes the kernel descriptor allocate them) and
// zeroes them; hipcc's own values then fit in the 256 VGPRs, so it never touches an AGPR --
// tests/test_fq7_build_cpu.py checks the ISA: no spills, no compiler v_accvgpr_* outside the
// asm statements.  Accumulator (i, j) (wp row tile i, token tile j) = a[4 (J i + j) .. +3].
#define SQMP_AGPR_ALL "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127", "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143", "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159", "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191", "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207", "a208", "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223", "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239", "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255"
__device__ inline void acc_init() {
  asm volatile(".irp r, 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15\n\t.irp s, 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15\n\t"
               "v_accvgpr_write_b32 a[\\r*16+\\s], 0\n\t.endr\n\t.endr\n\ts_nop 1" ::
                   : SQMP_AGPR_ALL);
}
// compile-time loop: f(integral_constant<int, B>), ..., f(integral_constant<int, E - 1>)
template <int B, int E, class F>
__device__ inline void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>());
    sfor<B + 1, E>(f);
  }
}
template <class DT, int A0> struct MfmaA;
template <int A0> struct MfmaA<F16, A0> {
  __device__ static inline void run(const u32x4& a, const u32x4& b) {
    asm volatile("v_mfma_f32_16x16x32_f16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(a), "v"(b),
                 "n"(A0), "n"(A0 + 3));
  }
};
template <int A0> struct MfmaA<BF16, A0> {
  __device__ static inline void run(const u32x4& a, const u32x4& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(a), "v"(b),
                 "n"(A0), "n"(A0 + 3));
  }
};
template <int R>
__device__ inline float acc_read() {
  float v;
  asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(v) : "n"(R));
  return v;
}

constexpr int NW = 4;              // waves per workgroup: one per SIMD
constexpr int J = 4;               // 16-token tiles per wave (64 tokens)
constexpr int TM = 256;            // wp rows per tile (kernel M)
constexpr int I = TM / 16;         // 16-row wp tiles per wave
constexpr int WR = 16 * J;         // tokens per wave
constexpr int TN = NW * WR;        // tokens per tile (kernel N)
constexpr int NS = 3;              // ring slots: stage kt + 2 lands while kt is computed
constexpr int SLOT = TM * 128;     // 256 rows x 64 positions x 2 B
constexpr int PF = 3;              // LDS fragment read-ahead (blocks)
constexpr int RS = 2 * TM + 16;    // epilogue: y^T row stride (bytes)
constexpr int EPI = TN * RS;
constexpr int LDS_BYTES = NS * SLOT > EPI ? NS * SLOT : EPI;

// DIAG (timing diagnostics, wrong results by design, instantiated only in a SQMP_DIAG_BUILD,
// selected by SQMP_FQT8_DIAG): 1 no wp DMA in the K loop, 2 no LDS fragment reads in it, 4 no
// act decode / copy, 8 no barrier, 16 no act operand loads in it.
template <class DT, int DIAG = 0>
__global__ __launch_bounds__(256, 1) void gemm_kernel(
    const typename DT::T* __restrict__ A, const uint32_t* __restrict__ Ct,
    const typename DT::T* __restrict__ St, const typename DT::T* __restrict__ Xt,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kq, int S_pad, int G, int ngq, int tiles_m, int tiles_n, int group_m,
    uint32_t* __restrict__ colmax, int nt) {
  typedef typename DT::T T;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

  // the ring's LDS byte address (the DMA's M0 base) once, as an integer
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(
      (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)lds);
  int tm, tn;
  tile_coords(tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int lda = Kq + S_pad;
  const int nkm = Kq / 64, nks = S_pad / 64, nkt = nkm + nks;
  const int nb = tn * NW + wave;  // this wave's 64-token block of the tile-major operands

  // ---- wp by LDS-DMA: piece i (0..7) of this wave = tile rows 32 i + 8 wave + (lane >> 3),
  // the lane moving logical chunk brev3(p ^ ((row >> 1) & 7)) into physical chunk p = lane & 7
  // ((row >> 1) & 7 does not depend on i: piece i is piece 0 moved by 32 i rows)
  const rsrc_t rA = make_rsrc(A + (size_t)m0 * lda);
  const int arow = 8 * wave + (lane >> 3);
  const uint32_t a_off = (uint32_t)((size_t)arow * lda * sizeof(T)) +
                         (uint32_t)(brev3((lane & 7) ^ ((arow >> 1) & 7)) << 4);
  const uint32_t a_piece = 32u * (uint32_t)lda * (uint32_t)sizeof(T);

  // ---- act operands straight to registers (SQMP_QA_TILED4 layouts, J = 4): per stage a lane
  // loads 32 B of codes + 8 B of group scales, per salient stage 128 B of exact x
  const rsrc_t rC = make_rsrc(Ct + (size_t)nb * nkm * (128 * J));
  const rsrc_t rS = make_rsrc(St + (size_t)nb * ngq * (16 * J));
  const rsrc_t rX = make_rsrc(Xt + (size_t)nb * (nks > 0 ? nks : 1) * (1024 * J));
  const uint32_t vC = (uint32_t)lane * (8u * J), vX = (uint32_t)lane * (32u * J);
  const uint32_t vS = (uint32_t)r16 * (2u * J);
  struct Codes {
    u32x4 w[2];  // dwords [j][s] of token rows 16 j + r16
    u32x2 s;     // the 4 rows' group scales
  };
  struct Dense {
    u32x4 w[2 * J];  // fragment [j][s] of token rows 16 j + r16
  };
  auto issue_codes = [&](int kt, Codes& d) {
    ld16<0>(d.w[0], rC, vC, (uint32_t)kt * (512u * J));
    ld16<16>(d.w[1], rC, vC, (uint32_t)kt * (512u * J));
    const int g = min((kt * 64) / G, ngq - 1);
    ld8(d.s, rS, vS, (uint32_t)g * (32u * J));
  };
  auto issue_dense = [&](int kd, Dense& d) {
    const uint32_t so = (uint32_t)kd * (2048u * J);
    ld16<0>(d.w[0], rX, vX, so);
    ld16<16>(d.w[1], rX, vX, so);
    ld16<32>(d.w[2], rX, vX, so);
    ld16<48>(d.w[3], rX, vX, so);
    ld16<64>(d.w[4], rX, vX, so);
    ld16<80>(d.w[5], rX, vX, so);
    ld16<96>(d.w[6], rX, vX, so);
    ld16<112>(d.w[7], rX, vX, so);
  };

  acc_init();

  const DecK dk = make_deck();
  const int a_sw = (r16 >> 1) & 7;
  uint32_t a_lo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    a_lo[s] = (uint32_t)(r16 * 128 + ((brev3(4 * (q & 1) + 2 * s + (q >> 1)) ^ a_sw) << 4));

  Codes cs[2];
  Dense dd[2];
  uint32_t sp[2][J];  // prepared scales of cs[P]
  u32x4 bf[2][J];     // decoded act fragments [sub-step][token tile] of the current stage

  auto prep = [&](const Codes& c, uint32_t* out) {
    const uint32_t sb[4] = {c.s.x & 0xFFFFu, c.s.x >> 16, c.s.y & 0xFFFFu, c.s.y >> 16};
#pragma unroll
    for (int j = 0; j < J; ++j) out[j] = Dec<DT>::prep(sb[j]);
  };
  // fragment of token tile j, sub-step s: dword [j][s] = component (j & 1) * 2 + s of w[j >> 1]
  auto dec = [&](const Codes& c, const uint32_t* spj, int j, int s) {
    return Dec<DT>::run(c.w[j >> 1][(j & 1) * 2 + s], spj[j], dk);
  };

  // one stage on register parity P = k & 1 (compile time), its kinds at run time (uniform
  // branches): act fragments decoded from cs[P] (k < nkm) or taken from the exact salient x in
  // dd[P]; the next stage's operand loaded into cs[P ^ 1] / dd[P ^ 1] (or none after the last).
  // 32 blocks (sub-step t / 16, wp row tile t % 16), 4 MFMAs each, MFMAs always on bf.
  auto stage = [&](int k, int slot_c, int slot_d, auto pp, auto steady) {
    constexpr int P = decltype(pp)::value, PN = P ^ 1;
    // steady: k, k + 1 and k + 2 all code stages (known at compile time: no branches)
    constexpr bool ST = decltype(steady)::value;
    const bool cur_codes = ST || k < nkm;
    const int nk = ST ? 0 : (k + 1 < nkm ? 0 : (k + 1 < nkt ? 1 : 2));  // next: codes / salient / none
    const int n2 = ST ? 0 : (k + 2 < nkm ? 0 : (k + 2 < nkt ? 1 : 2));  // the one after
    if constexpr (!(DIAG & 8))
      barrier();  // every wave's pieces of stage k landed (their vmcnt ran a stage earlier);
                  // every wave is done with slot_d (read in stage k - 1)
    const bool dma = !(DIAG & 1) && (ST || k + 2 < nkt);
    const unsigned char* __restrict__ slot = lds + slot_c * SLOT;
    const uint32_t dlds = lds_base + (uint32_t)slot_d * SLOT + (uint32_t)wave * 1024u;
    const uint32_t dso = (uint32_t)(k + 2) * 128u;
    u32x4 a[PF + 1];
#pragma unroll
    for (int t = 0; t < PF; ++t)
      a[t] = *(const u32x4*)(slot + 16 * (t % I) * 128 + a_lo[t / I]);
    sfor<0, 2 * I>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t + PF < 2 * I && !(DIAG & 2))
        a[(t + PF) % (PF + 1)] =
            *(const u32x4*)(slot + 16 * ((t + PF) % I) * 128 + a_lo[(t + PF) / I]);
      constexpr int s = t / I, i = t % I;
      sfor<0, J>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        MfmaA<DT, 4 * (J * i + j)>::run(bf[s][j], a[t % (PF + 1)]);
      });
      // this stage's sub-step-1 fragments (blocks 4-7: >= 8 MFMAs after their last read)
      if constexpr (t >= 4 && t < 4 + J && !(DIAG & 4)) {
        if (cur_codes)
          bf[1][t - 4] = dec(cs[P], sp[P], t - 4, 1);
        else
          bf[1][t - 4] = dd[P].w[2 * (t - 4) + 1];
      }
      if constexpr ((t & 1) && t < 16) {  // piece t / 2 of stage k + 2
        if (dma) dma16(rA, a_off, dso + (uint32_t)(t >> 1) * a_piece, dlds + (uint32_t)(t >> 1) * 4096u);
      }
      // stage k + 2's act operand into the registers this stage finished decoding at block 7
      // (two stages of latency: with one wave per SIMD nothing else hides it)
      if constexpr (t == 8 && !(DIAG & 16)) {
        if (n2 == 0)
          issue_codes(k + 2, cs[P]);
        else if (n2 == 1)
          issue_dense(k + 2 - nkm, dd[P]);
      }
      if constexpr (t == 19) {
        if (nk != 2) {
          // in flight after the wait: this stage's DMA pieces and operand (both for k + 2)
          if constexpr ((DIAG & 17) != 0)
            vmwait<0>();
          else
            vmwait_dyn(dma ? (n2 == 0 ? 11 : 16) : 0);
          if (nk == 0) {
            fence(cs[PN].w[0]);
            fence(cs[PN].w[1]);
            fence(cs[PN].s);
            prep(cs[PN], sp[PN]);
          } else {
#pragma unroll
            for (int u = 0; u < 2 * J; ++u) fence(dd[PN].w[u]);
          }
        }
      }
      // the next stage's sub-step-0 fragments (its first MFMAs then wait on nothing)
      if constexpr (t >= 20 && t < 20 + J && !(DIAG & 4)) {
        if (nk == 0)
          bf[0][t - 20] = dec(cs[PN], sp[PN], t - 20, 0);
        else if (nk == 1)
          bf[0][t - 20] = dd[PN].w[2 * (t - 20)];
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;

  // ---- prologue: DMA(0), codes(0), codes(1), DMA(1); wait for DMA(0) and codes(0) (nkm >= 2)
#pragma unroll
  for (int p = 0; p < 8; ++p)
    dma16(rA, a_off, (uint32_t)p * a_piece, lds_base + (uint32_t)(4 * p + wave) * 1024u);
  issue_codes(0, cs[0]);
  issue_codes(1, cs[1]);
#pragma unroll
  for (int p = 0; p < 8; ++p)
    dma16(rA, a_off, 128u + (uint32_t)p * a_piece,
          lds_base + (uint32_t)SLOT + (uint32_t)(4 * p + wave) * 1024u);
  vmwait<11>();
  fence(cs[0].w[0]);
  fence(cs[0].w[1]);
  fence(cs[0].s);
  prep(cs[0], sp[0]);
#pragma unroll
  for (int j = 0; j < J; ++j) bf[0][j] = dec(cs[0], sp[0], j, 0);

  // ---- every stage in ONE loop (one register allocation for all of them): pairs of stages
  // with compile-time register parity
  using Yes = std::true_type;
  using No = std::false_type;
  int sc = 0, k = 0;
  // the code stages whose next two are code stages too: every kind known at compile time
  for (; k + 3 < nkm; k += 2) {
    stage(k, sc, sc == 0 ? 2 : sc - 1, Z(), Yes());
    sc = sc == 2 ? 0 : sc + 1;
    stage(k + 1, sc, sc == 0 ? 2 : sc - 1, O(), Yes());
    sc = sc == 2 ? 0 : sc + 1;
  }
  // the rest (the last code stages and the salient ones): kinds at run time
  for (; k < nkt; k += 2) {
    stage(k, sc, sc == 0 ? 2 : sc - 1, Z(), No());
    sc = sc == 2 ? 0 : sc + 1;
    if (k + 1 < nkt) {
      stage(k + 1, sc, sc == 0 ? 2 : sc - 1, O(), No());
      sc = sc == 2 ? 0 : sc + 1;
    }
  }

  // ---- epilogue: y^T staged [token][wp row] at a row stride of 2 TM + 16 bytes, stored as
  // TM-wide row pieces of Y[token][wp row]
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  barrier();  // every wave is past its last read of the ring
  // the last asm MFMA's results -> hipcc's accumulator reads below (8-pass XDL: 12 states)
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  sfor<0, I>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    const int ml = 16 * i + r16;
    const float bv = bias && m0 + ml < M ? DT::to_f(bias[m0 + ml]) : 0.f;
    float cm = 0.f;  // |y| max of output column m0 + ml over this lane's tokens
    sfor<0, 4 * J>([&](auto jr) {
      constexpr int j = decltype(jr)::value / 4, r = decltype(jr)::value % 4;
      const T v = DT::from_f(acc_read<4 * (J * i + j) + r>() + bv);
      *(T*)(lds + (WR * wave + 16 * j + 4 * q + r) * RS + ml * 2) = v;
      if (colmax && n0 + WR * wave + 16 * j + 4 * q + r < N) cm = fmaxf(cm, fabsf(DT::to_f(v)));
    });
    if (colmax) {
      cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
      cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
      if (q == 0 && m0 + ml < M) atomicMax(colmax + m0 + ml, __float_as_uint(cm));
    }
  });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  barrier();
  constexpr int CPR = TM / 8;  // 16-B chunks per staged row
#pragma unroll 4
  for (int c2 = tid; c2 < TN * CPR; c2 += 256) {
    const int nl = c2 / CPR, c = c2 % CPR;
    const int gn = n0 + nl, gm = m0 + c * 8;
    if (gn < N && gm < M) {  // M % 8 == 0 (launcher)
      const u32x4 v = *(const u32x4*)(lds + nl * RS + c * 16);
      if (nt)  // streaming stores of a large output (nt_output)
        store16_nt(Y + (size_t)gn * M + gm, v);
      else
        *(u32x4*)(Y + (size_t)gn * M + gm) = v;
    }
  }
}

// raster groups of 4 wp-row tiles (as sqmp_gemm_fqt7); SQMP_FQT8_GROUP_M overrides (A/B)
static int group_m_env() {
  const char* e = getenv("SQMP_FQT8_GROUP_M");
  return e && atoi(e) > 0 ? atoi(e) : 4;
}

template <class DT>
static int launch(const void* wp, const void* codes_t, const void* scale_t, const void* sal_t,
                  const void* bias, void* y, int M, int N, int Kq, int S_pad, int G, int ngq,
                  uint32_t* colmax, hipStream_t s) {
  typedef typename DT::T T;
  // kernel M = weight rows (wp rows, N of the layer), kernel N = tokens (M of the layer)
  const int tiles_m = cdiv(N, TM), tiles_n = cdiv(M, TN);
  const int nt = nt_output((size_t)M * N * sizeof(T)) ? 1 : 0;
  auto go = [&](auto kern) {
    kern<<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
        (const T*)wp, (const uint32_t*)codes_t, (const T*)scale_t, (const T*)sal_t,
        (const T*)bias, (T*)y, N, M, Kq, S_pad, G, ngq, tiles_m, tiles_n, group_m_env(), colmax,
        nt);
  };
#ifdef SQMP_DIAG_BUILD
  const char* de = getenv("SQMP_FQT8_DIAG");
  const int diag = de ? atoi(de) : 0;
  if (std::is_same<DT, F16>::value && diag) {
    switch (diag) {
      case 1: go(gemm_kernel<DT, 1>); break;
      case 2: go(gemm_kernel<DT, 2>); break;
      case 4: go(gemm_kernel<DT, 4>); break;
      case 8: go(gemm_kernel<DT, 8>); break;
      case 16: go(gemm_kernel<DT, 16>); break;
      case 7: go(gemm_kernel<DT, 7>); break;
      case 20: go(gemm_kernel<DT, 20>); break;
      case 31: go(gemm_kernel<DT, 31>); break;
      default: return SQMP_EINVAL;
    }
    SQMP_LAUNCH_CHECK();
    return SQMP_OK;
  }
#endif
  go(gemm_kernel<DT>);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace fqt8

// sqmp_gemm_fqt8: sqmp_gemm_fqt7j(J = 4)'s operands (SQMP_QA_TILED4) and results at one wave
// per SIMD.  colmax may be NULL.
extern "C" int sqmp_gemm_fqt8(const void* codes_t, const void* scale_t, const void* sal_t,
                              const void* wp, const void* bias, void* y, int dtype, int M, int N,
                              int Kq, int S_pad, int G, int ngq, uint32_t* colmax, void* stream) {
  if (!codes_t || !scale_t || !sal_t || !wp || !y) return SQMP_EINVAL;
  if (M < 0 || N <= 0 || Kq <= 0 || Kq % 128 || S_pad < 0 || S_pad % 64 || G <= 0 || ngq <= 0)
    return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (G % 64 || N % 8) return SQMP_EUNSUPPORTED;
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SQMP_F16)
    return fqt8::launch<F16>(wp, codes_t, scale_t, sal_t, bias, y, M, N, Kq, S_pad, G, ngq, colmax, s);
  return fqt8::launch<BF16>(wp, codes_t, scale_t, sal_t, bias, y, M, N, Kq, S_pad, G, ngq, colmax, s);
}

}  // namespace sqmp
