// gemm_fqt9 -- the activation-order faithful GEMM at ONE wave per SIMD on the 32x32x16 MFMA
// (sqmp_gemm_fqt7's numerics: y = D(x_hat . W_hat^T + bias), fake_quant.py:306, computed as
// y^T = wp . codes^T with the act codes decoded in registers to D(code * scale) = the
// reference's x_hat bit for bit).
//
// Why: sqmp_gemm_fqt8 (the same one-wave-per-SIMD tiling on the
// 16x16x32 MFMA) measured 443 us against fqt7's 417 because at one wave per SIMD a 16-cycle
// MFMA leaves 8 cycles of vector issue and the tile needs about 11 per MFMA (wp DMA issue, the
// exact act decode, the fragment reads).  v_mfma_f32_32x32x16_f16 does twice the work in 32
// cycles and holds issue for 8 of them (MI355X_MICROARCH.md "vector-instruction ISSUE cost"):
// 24 free cycles per MFMA, 1.5x the issue headroom per FLOP for the same fillers per FLOP.
//
// 4 waves of 256 wp rows x 64 tokens (8 x 2 tiles of 32 x 32, 256 fp32 accumulators in the
// accumulator registers, named literally as in fqt8); per 64-position stage 4 k-steps x 8 row
// tiles = 32 blocks of one LDS wp-fragment read (3 blocks ahead) + 2 MFMAs:
//   blocks 8s+2, 8s+4  decode k-step s+1's act fragments (s = 3: the next stage's k-step 0)
//   blocks 1..15 odd   the 8 LDS-DMA pieces of stage k + 2 (3-slot ring)
//   block 21           stage k + 2's act operand (codes + scales, or the exact salient x)
//   block 23           the counted vmcnt retiring stage k + 1's operand and DMA pieces
// Operands: wp [roundup(N, 256)][Kq + S_pad] (sqmp_quant_act_c4's permuted weight) by LDS-DMA,
// 128-B rows with chunk c at c ^ ((row >> 1) & 7) (conflict-free for the ds_read_b128 lane
// groups); the act codes / scales / salient x in the SQMP_QA_TILED32 layouts (64-token blocks;
// lane 32 h + r holds token 32 j + r, positions 16 s + 8 h .. + 7 of k-step s).  Kq % 128 == 0,
// S_pad % 64 == 0, G % 64 == 0, N % 8 == 0, fp16 / bf16, no fused column statistics.
#include <stdlib.h>

#include <type_traits>

#include "sqmp_mfma.h"

namespace sqmp {
namespace fqt9 {

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
__device__ inline void ld4(uint32_t& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(r), "s"(soff));
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


// The 256 accumulators live in FIXED accumulator registers a[0:255], named literally in the
// MFMA statements: hipcc never sees them as values, so it cannot move them (with "+a" operands
// it homed the loop-carried accumulators in VGPRs and copied them to AGPRs around every use).
// acc_init() claims all 256 (its clobber list makes the kernel descriptor allocate them) and
// zeroes them; hipcc's own values then fit in the 256 VGPRs, so it never touches an AGPR --
// tests/test_fq7_build_cpu.py checks the ISA: no spills, no compiler v_accvgpr_* outside the
// asm statements.  Accumulator (i, j) (wp row tile i, token tile j) = a[16 (J i + j) .. +15].
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
    asm volatile("v_mfma_f32_32x32x16_f16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(a), "v"(b),
                 "n"(A0), "n"(A0 + 15));
  }
};
template <int A0> struct MfmaA<BF16, A0> {
  __device__ static inline void run(const u32x4& a, const u32x4& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(a), "v"(b),
                 "n"(A0), "n"(A0 + 15));
  }
};
template <int R>
__device__ inline float acc_read() {
  float v;
  asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(v) : "n"(R));
  return v;
}


constexpr int NW = 4;              // waves per workgroup: one per SIMD
constexpr int J = 2;               // 32-token tiles per wave (64 tokens)
constexpr int TM = 256;            // wp rows per tile (kernel M)
constexpr int I = TM / 32;         // 32-row wp tiles per wave
constexpr int KS = 4;              // 16-position k-steps per 64-position stage
constexpr int NB = KS * I;         // blocks per stage
constexpr int WR = 32 * J;         // tokens per wave
constexpr int TN = NW * WR;        // tokens per tile (kernel N)
constexpr int NS = 3;              // ring slots: stage kt + 2 lands while kt is computed
constexpr int SLOT = TM * 128;     // 256 rows x 64 positions x 2 B
constexpr int PF = 3;              // LDS fragment read-ahead (blocks)
constexpr int RS = 2 * TM + 16;    // epilogue: y^T row stride (bytes)
constexpr int EPI = TN * RS;
constexpr int LDS_BYTES = NS * SLOT > EPI ? NS * SLOT : EPI;

template <class DT>
__global__ __launch_bounds__(256, 1) void gemm_kernel(
    const typename DT::T* __restrict__ A, const uint32_t* __restrict__ Ct,
    const typename DT::T* __restrict__ St, const typename DT::T* __restrict__ Xt,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kq, int S_pad, int G, int ngq, int tiles_m, int tiles_n, int group_m, int nt) {
  typedef typename DT::T T;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(
      (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)lds);
  int tm, tn;
  tile_coords(tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  const int lda = Kq + S_pad;
  const int nkm = Kq / 64, nks = S_pad / 64, nkt = nkm + nks;
  const int nb = tn * NW + wave;  // this wave's 64-token block of the tile-major operands

  // ---- wp by LDS-DMA: piece p (0..7) of this wave = tile rows 32 p + 8 wave + (lane >> 3),
  // the lane moving logical chunk (lane & 7) ^ ((row >> 1) & 7) into physical chunk lane & 7
  const rsrc_t rA = make_rsrc(A + (size_t)m0 * lda);
  const int arow = 8 * wave + (lane >> 3);
  const uint32_t a_off = (uint32_t)((size_t)arow * lda * sizeof(T)) +
                         (uint32_t)((((lane & 7) ^ ((arow >> 1) & 7))) << 4);
  const uint32_t a_piece = 32u * (uint32_t)lda * (uint32_t)sizeof(T);

  // ---- act operands straight to registers (SQMP_QA_TILED32): per stage a lane loads 32 B of
  // codes (dword [s][j]) + one dword of group scales (tokens 32 j + r32, j = 0, 1), per
  // salient stage 128 B of exact x (fragment [s][j])
  const rsrc_t rC = make_rsrc(Ct + (size_t)nb * nkm * 512);
  const rsrc_t rS = make_rsrc(St + (size_t)nb * ngq * 64);
  const rsrc_t rX = make_rsrc(Xt + (size_t)nb * (nks > 0 ? nks : 1) * 4096);
  const uint32_t vC = (uint32_t)lane * 32u, vX = (uint32_t)lane * 128u;
  const uint32_t vS = (uint32_t)r32 * 4u;
  struct Codes {
    u32x4 w[2];  // dwords [s][j]
    uint32_t s;  // the two token tiles' group scales
  };
  struct Dense {
    u32x4 w[KS * J];  // fragment [s][j]
  };
  auto issue_codes = [&](int kt, Codes& d) {
    ld16<0>(d.w[0], rC, vC, (uint32_t)kt * 2048u);
    ld16<16>(d.w[1], rC, vC, (uint32_t)kt * 2048u);
    const int g = min((kt * 64) / G, ngq - 1);
    ld4(d.s, rS, vS, (uint32_t)g * 128u);
  };
  auto issue_dense = [&](int kd, Dense& d) {
    const uint32_t so = (uint32_t)kd * 8192u;
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
  const int a_sw = (r32 >> 1) & 7;
  uint32_t a_lo[KS];  // byte offset of this lane's fragment (row r32, chunk 2 s + h) in a row tile
#pragma unroll
  for (int s = 0; s < KS; ++s) a_lo[s] = (uint32_t)(r32 * 128 + (((2 * s + h) ^ a_sw) << 4));

  Codes cs[2];
  Dense dd[2];
  uint32_t sp[2][J];  // prepared scales of cs[P]
  u32x4 bf[2][J];     // decoded act fragments [k-step parity][token tile]

  auto prep = [&](const Codes& c, uint32_t* out) {
    out[0] = Dec<DT>::prep(c.s & 0xFFFFu);
    out[1] = Dec<DT>::prep(c.s >> 16);
  };
  // fragment of token tile j, k-step s: dword [s][j] = component (s & 1) * 2 + j of w[s >> 1]
  auto dec = [&](const Codes& c, const uint32_t* spj, int s, int j) {
    return Dec<DT>::run(c.w[s >> 1][(s & 1) * 2 + j], spj[j], dk);
  };

  // one stage on register parity P = k & 1 (compile time); ST: k, k + 1 and k + 2 are code
  // stages (every kind known at compile time), else the kinds are tested at run time
  auto stage = [&](int k, int slot_c, int slot_d, auto pp, auto steady) {
    constexpr int P = decltype(pp)::value, PN = P ^ 1;
    constexpr bool ST = decltype(steady)::value;
    const bool cur_codes = ST || k < nkm;
    const int nk = ST ? 0 : (k + 1 < nkm ? 0 : (k + 1 < nkt ? 1 : 2));  // next: codes / salient / none
    const int n2 = ST ? 0 : (k + 2 < nkm ? 0 : (k + 2 < nkt ? 1 : 2));  // the one after
    barrier();  // every wave's pieces of stage k landed; every wave is done with slot_d
    const bool dma = ST || k + 2 < nkt;
    const unsigned char* __restrict__ slot = lds + slot_c * SLOT;
    const uint32_t dlds = lds_base + (uint32_t)slot_d * SLOT + (uint32_t)wave * 1024u;
    const uint32_t dso = (uint32_t)(k + 2) * 128u;
    u32x4 a[PF + 1];
#pragma unroll
    for (int t = 0; t < PF; ++t) a[t] = *(const u32x4*)(slot + (t % I) * 4096 + a_lo[t / I]);
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t + PF < NB)
        a[(t + PF) % (PF + 1)] =
            *(const u32x4*)(slot + ((t + PF) % I) * 4096 + a_lo[(t + PF) / I]);
      constexpr int s = t / I, i = t % I;
      sfor<0, J>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        MfmaA<DT, 16 * (J * i + j)>::run(bf[s & 1][j], a[t % (PF + 1)]);
      });
      // k-step s + 1's fragments of this stage (blocks 8 s + 2 and 8 s + 4, s < 3)
      if constexpr (s < KS - 1 && (i == 2 || i == 4)) {
        constexpr int j = (i - 2) / 2;
        if (cur_codes)
          bf[(s + 1) & 1][j] = dec(cs[P], sp[P], s + 1, j);
        else
          bf[(s + 1) & 1][j] = dd[P].w[(s + 1) * J + j];
      }
      if constexpr ((t & 1) && t < 16) {  // piece t / 2 of stage k + 2
        if (dma) dma16(rA, a_off, dso + (uint32_t)(t >> 1) * a_piece, dlds + (uint32_t)(t >> 1) * 4096u);
      }
      // stage k + 2's act operand into the registers this stage finished decoding at block 20
      if constexpr (t == 21) {
        if (n2 == 0)
          issue_codes(k + 2, cs[P]);
        else if (n2 == 1)
          issue_dense(k + 2 - nkm, dd[P]);
      }
      if constexpr (t == 23) {
        if (nk != 2) {
          // in flight after the wait: this stage's DMA pieces and operand (both for k + 2)
          vmwait_dyn(dma ? (n2 == 0 ? 11 : 16) : 0);
          if (nk == 0) {
            fence(cs[PN].w[0]);
            fence(cs[PN].w[1]);
            fence(cs[PN].s);
            prep(cs[PN], sp[PN]);
          } else {
#pragma unroll
            for (int u = 0; u < KS * J; ++u) fence(dd[PN].w[u]);
          }
        }
      }
      // the next stage's k-step-0 fragments (blocks 26 and 28)
      if constexpr (s == KS - 1 && (i == 2 || i == 4)) {
        constexpr int j = (i - 2) / 2;
        if (nk == 0)
          bf[0][j] = dec(cs[PN], sp[PN], 0, j);
        else if (nk == 1)
          bf[0][j] = dd[PN].w[j];
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
  for (int j = 0; j < J; ++j) bf[0][j] = dec(cs[0], sp[0], 0, j);

  using Yes = std::true_type;
  using No = std::false_type;
  int sc = 0, k = 0;
  for (; k + 3 < nkm; k += 2) {
    stage(k, sc, sc == 0 ? 2 : sc - 1, Z(), Yes());
    sc = sc == 2 ? 0 : sc + 1;
    stage(k + 1, sc, sc == 0 ? 2 : sc - 1, O(), Yes());
    sc = sc == 2 ? 0 : sc + 1;
  }
  for (; k < nkt; k += 2) {
    stage(k, sc, sc == 0 ? 2 : sc - 1, Z(), No());
    sc = sc == 2 ? 0 : sc + 1;
    if (k + 1 < nkt) {
      stage(k + 1, sc, sc == 0 ? 2 : sc - 1, O(), No());
      sc = sc == 2 ? 0 : sc + 1;
    }
  }

  // ---- epilogue: accumulator (i, j) register g = token 32 j + (g & 3) + 8 (g >> 2) + 4 h of
  // this wave, wp row 32 i + r32; y^T staged [token][wp row] at a row stride of 2 TM + 16 B
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  barrier();  // every wave is past its last read of the ring
  // the last MFMA's results -> the accumulator reads below (16-pass XDL: 18 states)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  sfor<0, I>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    const int ml = 32 * i + r32;
    const float bv = bias && m0 + ml < M ? DT::to_f(bias[m0 + ml]) : 0.f;
    sfor<0, 16 * J>([&](auto jg) {
      constexpr int j = decltype(jg)::value / 16, g = decltype(jg)::value % 16;
      const T v = DT::from_f(acc_read<16 * (J * i + j) + g>() + bv);
      const int tok = WR * wave + 32 * j + (g & 3) + 8 * (g >> 2) + 4 * h;
      *(T*)(lds + tok * RS + ml * 2) = v;
    });
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
      if (nt)
        store16_nt(Y + (size_t)gn * M + gm, v);
      else
        *(u32x4*)(Y + (size_t)gn * M + gm) = v;
    }
  }
}

static int group_m_env() {
  const char* e = getenv("SQMP_FQT9_GROUP_M");
  return e && atoi(e) > 0 ? atoi(e) : 4;
}

template <class DT>
static int launch(const void* wp, const void* codes_t, const void* scale_t, const void* sal_t,
                  const void* bias, void* y, int M, int N, int Kq, int S_pad, int G, int ngq,
                  hipStream_t s) {
  typedef typename DT::T T;
  // kernel M = weight rows (wp rows, N of the layer), kernel N = tokens (M of the layer)
  const int tiles_m = cdiv(N, TM), tiles_n = cdiv(M, TN);
  const int nt = nt_output((size_t)M * N * sizeof(T)) ? 1 : 0;
  gemm_kernel<DT><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
      (const T*)wp, (const uint32_t*)codes_t, (const T*)scale_t, (const T*)sal_t,
      (const T*)bias, (T*)y, N, M, Kq, S_pad, G, ngq, tiles_m, tiles_n, group_m_env(), nt);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace fqt9

// sqmp_gemm_fqt9: the activation-order GEMM on SQMP_QA_TILED32 operands at one wave per SIMD
// on the 32x32x16 MFMA (same results as sqmp_gemm_fqt7 up to the accumulation order).
extern "C" int sqmp_gemm_fqt9(const void* codes_t, const void* scale_t, const void* sal_t,
                              const void* wp, const void* bias, void* y, int dtype, int M, int N,
                              int Kq, int S_pad, int G, int ngq, void* stream) {
  if (!codes_t || !scale_t || !sal_t || !wp || !y) return SQMP_EINVAL;
  if (M < 0 || N <= 0 || Kq <= 0 || Kq % 128 || S_pad < 0 || S_pad % 64 || G <= 0 || ngq <= 0)
    return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (G % 64 || N % 8) return SQMP_EUNSUPPORTED;
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SQMP_F16)
    return fqt9::launch<F16>(wp, codes_t, scale_t, sal_t, bias, y, M, N, Kq, S_pad, G, ngq, s);
  return fqt9::launch<BF16>(wp, codes_t, scale_t, sal_t, bias, y, M, N, Kq, S_pad, G, ngq, s);
}

}  // namespace sqmp
