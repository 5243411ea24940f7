// Fast W4A4 GEMMs for gfx950 (fp16 / bf16): the F.linear of fake_quant.py:306.
//
// gemm_fq6 -- the faithful mixed-precision GEMM
//   y[M][N] = D( A[M][Kp + S_pad] . B^T + bias ):  A = dequantized activations x_hat in
//   packed K order + the exact salient columns (bit-exact with the reference's q_x);
//   B = int4 codes decoded in registers to D(code * scale) (bit-exact with the
//   reference's W_hat), then the exact salient weight slice; v_mfma_f32_16x16x32 in D,
//   fp32 accumulation, one rounding to D.  Layout and schedule: the comment above the
//   kernel; measurements: DESIGN.md §4.
//
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "sqmp_mfma.h"

namespace sqmp {

template <int N>
__device__ inline void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ inline void raw_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // no LDS read moves above the barrier
  __builtin_amdgcn_sched_barrier(0);
}

// LDS-DMA of 16 B per lane (LDS destination = wave-uniform base + 16 * lane) issued from
// inline asm.  Through the builtin, hipcc (ROCm 7.2) models the pending DMA as an LDS
// write and then waits lgkmcnt(0) before EVERY ds_read that follows in the k-loop instead
// of the counted lgkmcnt(N) of the A-fragment read-ahead (measured: 14 full drains per
// 64 MFMAs).  The asm form is invisible to that analysis, so every kernel using it waits
// for its DMAs itself (vm_wait) and never relies on __syncthreads() to drain them.
__device__ inline void glds16a(const void* src, unsigned char* lds_dst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(
      (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_dst);
  // s_nop 0: M0 write -> LDS-DMA wait state (MI355X asm guide §4.1)
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0v),
               "v"(src)
               : "memory", "m0");
}

// The same LDS-DMA through a buffer resource: 32-bit per-lane offset (constant across the
// k-loop) + a scalar offset per stage, so issuing a piece costs no vector address math
// and moves 4 address bytes per lane instead of 8.  num_records = 0xFFFFFFFF (no range
// check; every offset stays inside the operand).
typedef int i32x4r __attribute__((ext_vector_type(4)));
__device__ inline i32x4r buf_rsrc(const void* base) {
  const uint64_t a = (uint64_t)(size_t)base;
  i32x4r r;
  r[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = (int)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xFFFFu);
  r[2] = -1;
  r[3] = 0x00020000;
  return r;
}
__device__ inline void blds16(const i32x4r& rsrc, uint32_t voff, uint32_t soff,
                              unsigned char* lds_dst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(
      (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_dst);
  // s_nop 0: M0 write -> LDS-DMA wait state (hazard table of the MI355X asm guide, §4.1;
  // hipcc pads nothing inside an asm string).  soff is wave-uniform SALU arithmetic (the
  // "s" constraint rejects anything else at compile time), so no v_readfirstlane ->
  // soffset hazard arises; the descriptor is built once, long before.
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               ::"s"(m0v), "v"(voff), "s"(rsrc), "s"(soff)
               : "memory", "m0");
}

// ----------------------------------------------------------------- LDS ring geometry
constexpr int F5_A = 32768;                      // 256 rows x 128 B
constexpr int F5_B = 8192;                       // 256 rows x 32 B
constexpr int F5_S = 8192;                       // 8 waves x 1 KiB
constexpr int F5_SLOT = F5_A + F5_B + F5_S;      // 49152
constexpr int F5_NSLOT = 3;                      // 147456 B of 160 KiB
constexpr int F5_VM_CODES = 4 + 1 + 1;           // DMA ops per wave per codes stage
constexpr int F5_VM_DENSE = 2 + 2;              // ... per 32-column dense stage
constexpr int F5_DB = 16384;                     // dense stage: B image after 256 x 64 B of A
constexpr int F5_DN = 16384;                     // fq6 dense stage: B after 128 x 128 B of A

// LDS images of the ring:
//   codes-stage A: 256 rows x 128 B, logical 16-B chunk c of row r at physical chunk
//     a_pchunk(c, r) = bitrev3(c) ^ ((r >> 1) & 7) -- conflict-free for both fragment
//     read patterns (32x32: chunk 2u+h; 16x16: chunk 4(q&1)+2s+(q>>1));
//   dense-stage A and B: 256 rows x 64 B, chunk c of row r at c ^ d_f((r >> 2) & 3).
__host__ __device__ inline int bitrev3(int c) { return ((c & 1) << 2) | (c & 2) | ((c >> 2) & 1); }
__device__ inline int a_pchunk(int c, int r) { return bitrev3(c) ^ ((r >> 1) & 7); }
__device__ inline int d_f(int g) { return (-g) & 3; }

// ================================================================= gemm_fq6
// Tile TM x 256 per 512-thread workgroup, 1 x 8 waves (TM x 32 per wave) on v_mfma_f32_16x16x32:
// 16 x 2 tiles of 16 x 16 per wave (128 fp32 accumulators), two 32-element sub-steps per
// 64-element stage.  Lane (r16, q) of sub-step s takes bpack dword 2q + s of its weight
// row (one ds_read_b64 per tile column carries both sub-steps) and A chunk
// 4 (q & 1) + 2 s + (q >> 1) -- the positions of that dword.  Every main-loop byte moves by
// LDS-DMA (buffer_load ... lds) into a 3-slot ring two 64-element K-stages ahead, waits
// hand-counted (s_waitcnt vmcnt(N)), one raw s_barrier per stage.  Dense stages (the exact salient slice; every stage for dense weights) are 64
// columns wide over 128 rows of the tile (two half-height stages per 64-column block when
// TM = 256): A 128 rows x 128 B + B 256 weight rows x 128 B fill one 48 KiB slot, every
// DMA moves whole 128-B lines, both images use the codes-stage A swizzle, and lane
// (r16, q) of sub-step s reads chunk 4 (q & 1) + 2 s + (q >> 1) of A and B alike.
// (Measured alternatives, DESIGN.md §4: s_setprio schemes, a 2 x 4 wave layout, a
// 5-block A read-ahead, the scale / B pieces issued by their own waves -- none faster.)
// colmax != NULL: the epilogue also atomic-maxes bits(max |y|) of each output column into
// colmax (the statistics of the fused output quantizer, SQMP_QA_STATS_GIVEN).
// TR (sqmp_gemm_fqt, activation order): A = the permuted weight wp, Bw / wscale / wsal = the
// act codes / group scales / exact salient x, so the tile is y^T: the epilogue adds bias[m]
// per A row and stores Y[n][m] (ld = M); colmax must be NULL.
template <class DT, int GB, int TM, bool TR = false>
__global__ __launch_bounds__(512, 1) void gemm_fq6_kernel(
    const typename DT::T* __restrict__ A, const void* __restrict__ Bw,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n, int group_m,
    uint32_t* __restrict__ colmax) {
  typedef typename DT::T T;
  constexpr int WM = 1, PF = 3;         // 1 x 8 waves of TM x 32; A read-ahead (blocks)
  constexpr int NWN = 8 / WM;           // waves along N
  constexpr int CW = 256 / NWN;         // weight rows (output columns) per wave
  constexpr int MW = TM / WM;           // rows per wave
  constexpr int I = MW / 16, J = CW / 16;  // 16 x 16 tiles per wave
  constexpr int NA = TM / 64;           // codes-stage A DMA ops per wave (64 rows each)
  // dense stages: TM = 128 -> 64 columns x 128 rows (A 16 KiB + B 32 KiB, 128-B lines);
  // TM = 256 -> 32 columns x 256 rows (A 16 KiB + B 16 KiB, 64-B row pieces: measured
  // faster there than 64-column half-height stages, which move B twice)
  constexpr int DW = TM == 128 ? 64 : 32;
  // dense A ops per wave: 2 (64-col or TM = 256), 1 (TM = 64: one 128-row op, upper half unused)
  constexpr int NAD = DW == 64 ? 2 : (TM == 256 ? 2 : 1);
  constexpr int VM_CODES = NA + 1 + 1, VM_DENSE = DW == 64 ? 2 + 4 : NAD + 2;
  constexpr int GBn = GB > 0 ? GB : 1;
  // Loader split (codes stages): waves 0-3 issue the DMA pieces of all 8 waves, waves 4-7
  // (one per SIMD, beside a loader) issue none.  An LDS-DMA piece holds up its wave's
  // instruction stream for ≈60-185 cycles (MI355X_MICROARCH.md cycle table), so a wave
  // that issues none keeps its SIMD's MFMA pipe fed meanwhile (config-2 GEMM +3-4 %;
  // handing the scale piece, or the B and scale pieces, back to their own wave: -7 / -9 %).
  constexpr bool LSPLIT = true, LB = true, LS = true;
  constexpr int VM_LOAD = 2 * NA + (LB ? 2 : 1) + (LS ? 2 : 1);  // loader ops per codes stage
  constexpr int VM_COMP = (LB ? 0 : 1) + (LS ? 0 : 1);            // ... of waves 4-7
  __shared__ __attribute__((aligned(16))) unsigned char lds[F5_NSLOT * F5_SLOT];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * TM, n0 = tn * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  const int r16 = lane & 15, q = lane >> 4;
  const int lda = Kp + S_pad;
  const int nkm = GB ? Kp / 64 : 0;
  const int nkt = nkm + (lda - nkm * 64) / DW;
  const int Np = pad_n(N);

  const int arow = 8 * wave + (lane >> 3);
  const uint32_t lchunk = (uint32_t)(bitrev3((lane & 7) ^ ((arow >> 1) & 7)) << 4);
  // buffer resources: A at the tile's first row, B codes at the tile's first weight row,
  // scales at the tile's first column; dense-stage B by absolute (clamped) row
  const i32x4r rA = buf_rsrc(A + (size_t)m0 * lda);
  const i32x4r rB = buf_rsrc((const unsigned char*)Bw + (size_t)n0 * (Kp / 2));
  const i32x4r rS = buf_rsrc(wscale + n0);
  const i32x4r rBd = buf_rsrc(Bw);
  const i32x4r rSal = buf_rsrc(wsal);
  const uint32_t a_off = (uint32_t)((size_t)arow * lda * sizeof(T)) + lchunk;
  const uint32_t a_str = (uint32_t)(64 * (size_t)lda * sizeof(T));
  // 64-column dense-stage B rows of this lane (clamped: wsal has N rows), for the salient
  // tail (ldb = S_pad) and, dense weights only, the main stages (ldb = Kp)
  uint32_t bd_tail[4], bd_main[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t r = (uint32_t)min(n0 + arow + 64 * i, N - 1);
    bd_tail[i] = r * (uint32_t)S_pad * sizeof(T) + lchunk;
    bd_main[i] = GB == 0 ? r * (uint32_t)Kp * sizeof(T) + lchunk : 0u;
  }
  // 32-column dense stages: 4 lanes per 64-B row piece, chunks swizzled by (row >> 2) & 3
  const int drow = 16 * wave + (lane >> 2);
  const int dchunk = (lane & 3) ^ d_f((lane >> 4) & 3);
  // TM = 64: the op's upper 64 rows repeat the tile's (unused there) -- never past the
  // tile, whose rows the operand's roundup(M, 256) allocation covers
  const int darow = TM == 64 ? (drow & 63) : drow;
  const uint32_t ad_off = (uint32_t)((size_t)darow * lda * sizeof(T) + dchunk * 16);
  const uint32_t ad_str = (uint32_t)(128 * (size_t)lda * sizeof(T));
  const uint32_t bd_r0 = (uint32_t)min(n0 + drow, N - 1), bd_r1 = (uint32_t)min(n0 + drow + 128, N - 1);
  const uint32_t b32_tail0 = bd_r0 * (uint32_t)S_pad * sizeof(T) + dchunk * 16;
  const uint32_t b32_tail1 = bd_r1 * (uint32_t)S_pad * sizeof(T) + dchunk * 16;
  const uint32_t b32_main0 = GB == 0 ? bd_r0 * (uint32_t)Kp * sizeof(T) + dchunk * 16 : 0u;
  const uint32_t b32_main1 = GB == 0 ? bd_r1 * (uint32_t)Kp * sizeof(T) + dchunk * 16 : 0u;
  const uint32_t b_off = (uint32_t)((32 * wave + (lane >> 1)) * (Kp / 2) +
                                    (((lane & 1) ^ ((lane >> 4) & 1)) << 4));
  constexpr int LPG = CW / 8;  // scale-DMA lanes per group (8 scales per lane)
  // lane's group within the block (GB = 2: groups 2 kt, 2 kt + 1) goes in the per-lane
  // offset; the block's first group in the scalar one
  const int s_u = min(lane / LPG, GBn - 1);
  const uint32_t s_off0 = (uint32_t)((CW * wn + (lane % LPG) * 8) * sizeof(T));
  const uint32_t s_off1 = s_off0 + (uint32_t)(s_u * Np * sizeof(T));

  auto issue = [&](int kt) {
    unsigned char* slot = lds + (kt % F5_NSLOT) * F5_SLOT;
    if (kt < nkm) {
      const int ks = kt;
      const uint32_t sa = (uint32_t)ks * 64 * sizeof(T);
#pragma unroll
      for (int i = 0; i < NA; ++i)
        if (!LSPLIT || wave < 4) {
          blds16(rA, a_off, sa + i * a_str, slot + (i * 8 + wave) * 1024);
          // loader split: waves 0-3 also move waves 4-7's pieces (rows + 32)
          if (LSPLIT) blds16(rA, a_off + 32u * lda * sizeof(T), sa + i * a_str, slot + (i * 8 + wave + 4) * 1024);
        }
      if (!LB || wave < 4) {
        blds16(rB, b_off, (uint32_t)ks * 32, slot + F5_A + wave * 1024);
        if (LB) blds16(rB, b_off + 128u * (Kp / 2), (uint32_t)ks * 32, slot + F5_A + (wave + 4) * 1024);
      }
      // GB = 2 blocks hold groups 2 kt and 2 kt + 1; past the last group (the zero codes
      // of the padding to Kp) the scales are clamped to group ngw - 1 -- never read past
      // the [ngw][Np] array (a NaN there would turn 0 * s into NaN)
      const int g0 = GB == 1 ? min((kt * 64) / Gw, ngw - 1) : min(kt * 2, ngw - 1);
      const uint32_t s_off = g0 + 1 <= ngw - 1 ? s_off1 : s_off0;
      // GBn groups x CW columns of scales (the other lanes repeat them: same lines; one
      // wave moving all 256 columns instead measured no faster)
      if (!LS || wave < 4) {
        blds16(rS, s_off, (uint32_t)g0 * Np * sizeof(T), slot + F5_A + F5_B + wave * 1024);
        if (LS)
          // (WM = 2: wave + 4 has the same column block, hence the same scales)
          blds16(rS, s_off + (WM == 1 ? 4u * CW * sizeof(T) : 0u), (uint32_t)g0 * Np * sizeof(T),
                 slot + F5_A + F5_B + (wave + 4) * 1024);
      }
    } else if (DW == 64) {
      const int col = nkm * 64 + (kt - nkm) * 64;
      const uint32_t sa = (uint32_t)col * sizeof(T);
      blds16(rA, a_off, sa, slot + wave * 1024);
      blds16(rA, a_off, sa + a_str, slot + (8 + wave) * 1024);
      const bool main = GB == 0 && col < Kp;
      const uint32_t sb = (uint32_t)(main ? col : col - Kp) * sizeof(T);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        blds16(main ? rBd : rSal, main ? bd_main[i] : bd_tail[i], sb,
               slot + F5_DN + (i * 8 + wave) * 1024);
    } else {
      const int col = nkm * 64 + (kt - nkm) * 32;
      const uint32_t sa = (uint32_t)col * sizeof(T);
      blds16(rA, ad_off, sa, slot + wave * 1024);
      if (NAD == 2) blds16(rA, ad_off, sa + ad_str, slot + (8 + wave) * 1024);
      const bool main = GB == 0 && col < Kp;
      const uint32_t sb = (uint32_t)(main ? col : col - Kp) * sizeof(T);
      blds16(main ? rBd : rSal, main ? b32_main0 : b32_tail0, sb, slot + F5_DB + wave * 1024);
      blds16(main ? rBd : rSal, main ? b32_main1 : b32_tail1, sb, slot + F5_DB + (8 + wave) * 1024);
    }
  };

  f32x4 acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const DecK dk = make_deck();
  const int a_row0 = (wm * MW + r16) * 128;
  const int a_sw = (r16 >> 1) & 7;
  // A fragment of block t = I*s + i: row 16 i + r16, chunk 4 (q&1) + 2 s + (q>>1)
  auto ald = [&](const unsigned char* __restrict__ slot, int t) {
    const int c = 4 * (q & 1) + 2 * (t / I) + (q >> 1);
    return *(const u32x4*)(slot + a_row0 + (t % I) * 2048 + ((bitrev3(c) ^ a_sw) << 4));
  };
#define SQMP_FQ6_BLOCKS(BF, ...)                                               \
  {                                                                            \
    u32x4 a[PF + 1];                                                           \
    _Pragma("unroll") for (int t = 0; t < PF; ++t) a[t] = ald(slot, t);        \
    _Pragma("unroll") for (int t = 0; t < 2 * I; ++t) {                        \
      if (t + PF < 2 * I) a[(t + PF) % (PF + 1)] = ald(slot, t + PF);          \
      _Pragma("unroll") for (int j = 0; j < J; ++j)                            \
          Mfma<DT>::run(acc[t % I][j], BF(t / I, j), a[t % (PF + 1)]);         \
      __VA_ARGS__;                                                             \
      __builtin_amdgcn_sched_barrier(0);                                       \
    }                                                                          \
  }

  auto compute_codes = [&](const unsigned char* __restrict__ slot) {
    const unsigned char* sb = slot + F5_A;
    const unsigned char* ss = slot + F5_A + F5_B + wave * 1024;
    uint2 bw[J];
    uint32_t sp[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int row = wn * CW + 16 * j + r16;
      bw[j] = *(const uint2*)(sb + row * 32 + (((q >> 1) ^ ((r16 >> 3) & 1)) << 4) + (q & 1) * 8);
      // group of this lane's dwords: 0 for GB == 1; q & 1 for Gw == 32 (positions 32(q&1)..)
      const int g = GB == 2 ? (q & 1) : 0;
      sp[j] = Dec<DT>::prep(*(const uint16_t*)(ss + g * CW * 2 + (16 * j + r16) * 2));
    }
    u32x4 bf[2][J];
#pragma unroll
    for (int j = 0; j < J; ++j) bf[0][j] = Dec<DT>::run(bw[j].x, sp[j], dk);
#define SQMP_BF6(s, j) bf[s][j]
    // sub-step 1 fragments decoded under the first J blocks (used from block I on)
    static_assert(J <= I, "sub-step 1 decode must finish before block I");
    SQMP_FQ6_BLOCKS(SQMP_BF6,
                    if (t < J) bf[1][t] = Dec<DT>::run(bw[t].y, sp[t], dk));
#undef SQMP_BF6
  };
#undef SQMP_FQ6_BLOCKS

  // 32-column dense stage over all TM rows
  const int d_sw = d_f((r16 >> 2) & 3);
  auto compute_dense32 = [&](const unsigned char* __restrict__ slot) {
    const int co = (q ^ d_sw) << 4;
    u32x4 bf[J];
#pragma unroll
    for (int j = 0; j < J; ++j) bf[j] = *(const u32x4*)(slot + F5_DB + (wn * CW + 16 * j + r16) * 64 + co);
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const u32x4 af = *(const u32x4*)(slot + (wm * MW + 16 * i + r16) * 64 + co);
#pragma unroll
      for (int j = 0; j < J; ++j) Mfma<DT>::run(acc[i][j], bf[j], af);
    }
  };
  // 64-column dense stage over 128 rows (TM = 128)
  auto compute_dense = [&](const unsigned char* __restrict__ slot, auto hc) {
    constexpr int H = decltype(hc)::value;
    constexpr int I2 = I;
    u32x4 bf[2][J];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = 4 * (q & 1) + 2 * s2 + (q >> 1);
        bf[s2][j] = *(const u32x4*)(slot + F5_DN + (wn * CW + 16 * j + r16) * 128 +
                                    ((bitrev3(c) ^ a_sw) << 4));
      }
    // A fragments read PF blocks ahead, one sched_barrier per block (as the codes loop)
    auto ald2 = [&](int t) {
      const int c = 4 * (q & 1) + 2 * (t / I2) + (q >> 1);
      return *(const u32x4*)(slot + a_row0 + (t % I2) * 2048 + ((bitrev3(c) ^ a_sw) << 4));
    };
    u32x4 a[PF + 1];
#pragma unroll
    for (int t = 0; t < PF; ++t) a[t] = ald2(t);
#pragma unroll
    for (int t = 0; t < 2 * I2; ++t) {
      if (t + PF < 2 * I2) a[(t + PF) % (PF + 1)] = ald2(t + PF);
#pragma unroll
      for (int j = 0; j < J; ++j)
        Mfma<DT>::run(acc[H * I2 + t % I2][j], bf[t / I2][j], a[t % (PF + 1)]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  issue(0);
  if (nkt > 1) issue(1);
  int kt = 0;
  for (; kt < nkm; ++kt) {
    if (kt + 1 < nkt) {
      if (kt + 1 < nkm) {
        if (!LSPLIT) vm_wait<VM_CODES>();
        else if (wave < 4) vm_wait<VM_LOAD>();
        else vm_wait<VM_COMP>();
      } else {
        vm_wait<VM_DENSE>();
      }
    } else {
      vm_wait<0>();
    }
    raw_barrier();
    if (kt + 2 < nkt) issue(kt + 2);
    compute_codes(lds + (kt % F5_NSLOT) * F5_SLOT);
  }
  for (; kt < nkt; ++kt) {
    if (kt + 1 < nkt) {
      vm_wait<VM_DENSE>();
    } else {
      vm_wait<0>();
    }
    raw_barrier();
    if (kt + 2 < nkt) issue(kt + 2);
    unsigned char* slot = lds + (kt % F5_NSLOT) * F5_SLOT;
    if constexpr (DW == 64)
      compute_dense(slot, std::integral_constant<int, 0>());
    else
      compute_dense32(slot);
  }

  if constexpr (TR) {
    // y^T tile staged [nl 256][ml TM] at a row stride of 2 TM + 16 bytes (the four q-groups
    // of a write land 16 banks apart), then stored as TM-wide row pieces of Y[n][m]
    constexpr int RS = 2 * TM + 16;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();  // every wave is past its last read of the ring
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int ml = wm * MW + 16 * i + r16;
      const float bv = bias && m0 + ml < M ? DT::to_f(bias[m0 + ml]) : 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *(T*)(lds + (wn * CW + 16 * j + 4 * q + r) * RS + ml * 2) = DT::from_f(acc[i][j][r] + bv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    constexpr int CPR = TM / 8;  // 16-B chunks per staged row
#pragma unroll 4
    for (int k = tid; k < 256 * CPR; k += 512) {
      const int nl = k / CPR, c = k % CPR;
      const int gn = n0 + nl, gm = m0 + c * 8;
      if (gn < N && gm < M)  // M % 8 == 0 (launcher)
        *(u32x4*)(Y + (size_t)gn * M + gm) = *(const u32x4*)(lds + nl * RS + c * 16);
    }
    return;
  }

  // ---- epilogue: acc[i][j][r] = C[n = n0 + CW wn + 16 j + 4 q + r][m = m0 + MW wm + 16 i + r16]
  // fused output-quant statistics: the lane's per-column maxima over its rows, reduced
  // over the 16 lanes of its q group (the tile's rows of this wave), one atomic max per
  // column from lane r16 == 0 (each wave holds all TM rows of its 32 columns)
  auto flush_colmax = [&](float (&cmx)[J][4]) {
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = cmx[j][r];
        v = fmaxf(v, __shfl_xor(v, 1, 64));
        v = fmaxf(v, __shfl_xor(v, 2, 64));
        v = fmaxf(v, __shfl_xor(v, 4, 64));
        v = fmaxf(v, __shfl_xor(v, 8, 64));
        const int n = n0 + wn * CW + 16 * j + 4 * q + r;
        if (r16 == 0 && n < N) atomicMax(colmax + n, __float_as_uint(v));
      }
  };
  {
    // Full-width tiles: the TM x 256 output tile is staged in LDS (row m: 512 B, 16-B
    // chunk c at c ^ (m & 15), conflict-free both ways) and stored as whole rows, one 16-B
    // chunk per lane (two rows per wave instruction, 4 full 128-B lines each) instead of
    // 8-B pieces of 16 rows (config-2 GEMM +2.8 %).
    if (n0 + 256 <= N && (N & 7) == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();  // every wave is past its last read of the ring
      float cmx[J][4] = {};
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int nl = wn * CW + 16 * j + 4 * q;  // first of the lane's 4 columns
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = bias ? DT::to_f(bias[n0 + nl + r]) : 0.f;
#pragma unroll
        for (int i = 0; i < I; ++i) {
          const int ml = wm * MW + 16 * i + r16;
          T v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = DT::from_f(acc[i][j][r] + bv[r]);
          if (colmax && m0 + ml < M) {
#pragma unroll
            for (int r = 0; r < 4; ++r) cmx[j][r] = fmaxf(cmx[j][r], fabsf(DT::to_f(v[r])));
          }
          const int c = nl >> 3;
          *(uint2*)(lds + ml * 512 + ((c ^ (ml & 15)) << 4) + (nl & 4) * 2) = *(const uint2*)v;
        }
      }
      if (colmax) flush_colmax(cmx);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's tile writes landed
      raw_barrier();
      const int c = tid & 31;
#pragma unroll
      for (int k = 0; k < TM / 16; ++k) {
        const int ml = 16 * k + (tid >> 5);
        const int gm = m0 + ml;
        const u32x4 val = *(const u32x4*)(lds + ml * 512 + ((c ^ (ml & 15)) << 4));
        if (gm < M) *(u32x4*)(Y + (size_t)gm * N + n0 + c * 8) = val;
      }
      return;
    }
  }
  float bvs[J][4];
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bvs[j][r] = bias ? DT::to_f(bias[min(n0 + wn * CW + 16 * j + 4 * q + r, N - 1)]) : 0.f;
  if (colmax) {  // column statistics first: the shuffles need every lane (no early exits)
    float cmx[J][4] = {};
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int i = 0; i < I; ++i)
        if (m0 + wm * MW + 16 * i + r16 < M) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            cmx[j][r] = fmaxf(cmx[j][r], fabsf(DT::to_f(DT::from_f(acc[i][j][r] + bvs[j][r]))));
        }
    flush_colmax(cmx);
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int nb = n0 + wn * CW + 16 * j + 4 * q;
    if (nb >= N) continue;
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int gm = m0 + wm * MW + 16 * i + r16;
      if (gm >= M) continue;
      T v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = DT::from_f(acc[i][j][r] + bvs[j][r]);
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
// M-tiles per raster group (tile_coords): SQMP_GROUP_M overrides (A/B tuning knob; 4 and
// 8 measured equal at config 2, 1 and 2 0.5-1 % slower)
static int fq6_group_m() {
  const char* e = knob("SQMP_GROUP_M");
  return e && atoi(e) > 0 ? atoi(e) : 4;
}

template <class DT, int GB, int TM, bool TR = false>
static int fq6_launch(const void* a, const void* codes, const void* wscale, const void* wsal,
                      const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                      int ngw, uint32_t* colmax, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, TM), tiles_n = cdiv(N, 256);
  gemm_fq6_kernel<DT, GB, TM, TR><<<dim3(tiles_m * tiles_n), dim3(512), 0, s>>>(
      (const T*)a, codes, (const T*)wscale, (const T*)wsal, (const T*)bias, (T*)y, M, N, Kp,
      S_pad, Gw, ngw, tiles_m, tiles_n, fq6_group_m(), colmax);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT>
static int fq6_dispatch(const void* a, const void* codes, const void* wscale, const void* wsal,
                        const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                        int ngw, int n_bits, uint32_t* colmax, hipStream_t s) {
  // 128-row tiles when 256-row tiles would leave the chip under two workgroups per CU;
  // 64-row tiles when even 128-row tiles would leave CUs idle (e.g. OPT-1.3B's 2048-wide
  // layers at 2048 tokens: 128 tiles of 128 x 256)
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256), t128 = (long)cdiv(M, 128) * cdiv(N, 256);
  const int tm = t256 >= 2L * 256 ? 256 : (t128 >= 256 || M <= 64 ? 128 : 64);
#define SQMP_FQ6(GB, GW, NGW)                                                                          \
  (tm == 256 ? fq6_launch<DT, GB, 256>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, GW, NGW, colmax, s) \
   : tm == 128 ? fq6_launch<DT, GB, 128>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, GW, NGW, colmax, s) \
               : fq6_launch<DT, GB, 64>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, GW, NGW, colmax, s))
  if (n_bits == 0) return SQMP_FQ6(0, 1, 1);
  if (n_bits != 4) return SQMP_EUNSUPPORTED;
  if (Gw % 64 == 0) return SQMP_FQ6(1, Gw, ngw);
  if (Gw == 32) return SQMP_FQ6(2, Gw, ngw);
  return SQMP_EUNSUPPORTED;
#undef SQMP_FQ6
}

int launch_gemm_fq_fast(int dtype, const void* a, const void* codes, const void* wscale,
                        const void* wsal, const void* bias, void* y, int M, int N, int Kp,
                        int S_pad, int Gw, int ngw, int n_bits, uint32_t* colmax,
                        hipStream_t s) {
  if (dtype == SQMP_F16)
    return fq6_dispatch<F16>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, colmax, s);
  if (dtype == SQMP_BF16)
    return fq6_dispatch<BF16>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, colmax, s);
  return SQMP_EUNSUPPORTED;
}

// sqmp_gemm_fqt: the activation-order GEMM on gemm_fq6<TR> (kernel M = weight rows N, kernel
// N = activation rows M)
template <class DT>
static int fqt_dispatch(const void* acodes, const void* ascale, const void* xs, const void* wp,
                        const void* bias, void* y, int M, int N, int Kq, int S_pad, int G,
                        int ngq, hipStream_t s) {
  const long t256 = (long)cdiv(N, 256) * cdiv(M, 256);
  if (t256 >= 2L * 256)
    return fq6_launch<DT, 1, 256, true>(wp, acodes, ascale, xs, bias, y, N, M, Kq, S_pad, G, ngq,
                                        nullptr, s);
  return fq6_launch<DT, 1, 128, true>(wp, acodes, ascale, xs, bias, y, N, M, Kq, S_pad, G, ngq,
                                      nullptr, s);
}

int launch_gemm_fqt(int dtype, const void* acodes, const void* ascale, const void* xs,
                    const void* wp, const void* bias, void* y, int M, int N, int Kq, int S_pad,
                    int G, int ngq, hipStream_t s) {
  if (dtype == SQMP_F16)
    return fqt_dispatch<F16>(acodes, ascale, xs, wp, bias, y, M, N, Kq, S_pad, G, ngq, s);
  if (dtype == SQMP_BF16)
    return fqt_dispatch<BF16>(acodes, ascale, xs, wp, bias, y, M, N, Kq, S_pad, G, ngq, s);
  return SQMP_EUNSUPPORTED;
}

}  // namespace sqmp
