// W4A4 GEMM for per_token / per_tensor activations on the block-scaled FP8 MFMA
// (v_mfma_scale_f32_32x32x64_f8f6f4, e4m3 operands, unit block scales): the integer
// contraction of fake_quant.py:306 for the activation modes whose scale is one per row
// (:56-75), where x_hat[m,k] * W_hat[n,k] = sa[m] * ws[n,g(k)] * ca[m,k] * cw[n,k].
//
//   y[m][n] = D( sa[m] * sum_g ws[n][g] * (sum_{k in g} ca[m][k] cw[n][k])
//               + sum_j xs[m][j] wsal[n][j] + bias[n] )
//
// Both code operands are small integers (|c| <= 7), exact in e4m3; each 64-position block
// lies in one weight group (Gw % 64 == 0), so one MFMA per 32 x 32 tile and block gives
// the exact integer block sum in fp32 and the fold tot += tmp * ws[n][g] is one fp32 FMA
// per element (versus a convert + FMA per element on the i8 MFMA).  The e4m3 instruction
// runs at twice the f16 MFMA rate.  The numerics differ from the reference's
// F.linear(D(ca sa), D(cw ws)) only by the D() roundings of the two dequantized operands
// (relative 2^-11 per element), as the i8 path.
//
// Tile 256 (m) x 256 (n) per 512-thread workgroup; 8 waves, wave w owns columns
// [32 w, 32 w + 32) over all 256 rows (8 tiles of 32 x 32).  MFMA A = activation rows,
// B = weight columns, so a lane's 16 results share one weight column (one scale per
// fold).  K-stages: 64-position code blocks (A and B 256 rows x 64 B of e4m3), then the
// exact salient tail in 32-column f16 stages (v_mfma_f32_32x32x16_f16, same 256 x 64 B
// images) after the accumulators are scaled by sa.  Every stage moves 2 A + 2 B 1-KiB
// LDS-DMA pieces per wave through buffer resources into a 4-slot ring (3 stages ahead);
// wave 0 also moves the stage's 256 fp32 weight scales (code stages) or the tile's 256
// row scales (first tail stage).  LDS rows are 64 B with 16-B chunk c of row r at
// c ^ ((r >> 2) & 3): conflict-free for the ds_read_b128 lane groups.
#include <stdlib.h>

#include "sqmp_mfma.h"

namespace sqmp {

namespace {

typedef int i32x4b __attribute__((ext_vector_type(4)));
typedef int i32x8b __attribute__((ext_vector_type(8)));

constexpr int F8_A = 0, F8_B = 16384, F8_S = 32768;
constexpr int F8_SLOT = 33792;  // A 16 KiB + B 16 KiB + S 1 KiB
constexpr int F8_NSLOT = 4;     // 135168 B of LDS

__device__ inline i32x4b rsrc_of(const void* base, uint32_t nrec) {
  const uint64_t a = (uint64_t)(size_t)base;
  i32x4b r;
  r[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = (int)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xFFFFu);
  r[2] = (int)nrec;
  r[3] = 0x00020000;
  return r;
}

// 16 B per lane to LDS (wave-uniform destination + 16 * lane), issued from asm so the
// compiler's LDS wait analysis does not see a pending DMA (see sqmp_gemm_fast.hip).
__device__ inline void dma16(const i32x4b& rsrc, uint32_t voff, uint32_t soff,
                             unsigned char* lds_dst) {
  // the low half of an LDS pointer's generic address is its LDS address (the aperture
  // is the high half): no generic -> local cast, whose null check costs 4 SALU per piece
  const uint32_t m0v = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)lds_dst);
  // s_nop 0: M0 write -> LDS-DMA (hazard table, MI355X asm guide §4.1); soff is SALU
  // arithmetic ("s" rejects a VGPR value at compile time), the descriptor built long before
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               ::"s"(m0v), "v"(voff), "s"(rsrc), "s"(soff)
               : "memory", "m0");
}

template <int N>
__device__ inline void vmw() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ inline int sw64(int r, int c) { return (r << 6) + (((c ^ (r >> 2)) & 3) << 4); }

}  // namespace

template <class DT>
__global__ __launch_bounds__(512, 1) void gemm_f8_kernel(
    const unsigned char* __restrict__ A8, const float* __restrict__ ascale,
    const typename DT::T* __restrict__ XS, const unsigned char* __restrict__ W8,
    const float* __restrict__ ws32, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  __shared__ __attribute__((aligned(16))) unsigned char lds[F8_NSLOT * F8_SLOT];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, 4, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int nk8 = Kp / 64, nkt = nk8 + S_pad / 32;
  const int Np = pad_n(N);

  // ---- DMA geometry: piece j of a wave covers rows 16 (2 wave + j) + (lane >> 2), the
  // lane's physical chunk lane & 3 holds logical chunk (lane & 3) ^ ((row >> 2) & 3)
  uint32_t va8[2], vw8[2], vxs[2], vsal[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 16 * (2 * wave + j) + (lane >> 2);
    const int c = ((lane & 3) ^ (r >> 2)) & 3;
    va8[j] = (uint32_t)r * Kp + c * 16;
    vw8[j] = (uint32_t)r * Kp + c * 16;
    vxs[j] = (uint32_t)r * S_pad * sizeof(T) + c * 16;
    vsal[j] = (uint32_t)min(n0 + r, N - 1) * S_pad * sizeof(T) + c * 16;
  }
  const i32x4b rA = rsrc_of(A8 + (size_t)m0 * Kp, 0xFFFFFFFFu);
  const i32x4b rW = rsrc_of(W8 + (size_t)n0 * Kp, 0xFFFFFFFFu);
  const i32x4b rX = rsrc_of(XS + (size_t)m0 * S_pad, 0xFFFFFFFFu);
  const i32x4b rL = rsrc_of(wsal, 0xFFFFFFFFu);
  const i32x4b rS = rsrc_of(ws32 + n0, 0xFFFFFFFFu);
  // row scales of rows m0 .. m0 + 255 (range-checked: rows >= M read 0)
  const i32x4b rR = rsrc_of(ascale + m0, (uint32_t)(M - m0) * 4u);

  auto issue = [&](int kt) {
    unsigned char* slot = lds + (kt % F8_NSLOT) * F8_SLOT;
    if (kt < nk8) {
      const uint32_t so = (uint32_t)kt * 64;
#pragma unroll
      for (int j = 0; j < 2; ++j) dma16(rA, va8[j], so, slot + F8_A + (2 * wave + j) * 1024);
#pragma unroll
      for (int j = 0; j < 2; ++j) dma16(rW, vw8[j], so, slot + F8_B + (2 * wave + j) * 1024);
      if (wave == 0) {
        const int g = min((kt * 64) / Gw, ngw - 1);
        dma16(rS, (uint32_t)lane * 16, (uint32_t)g * Np * 4, slot + F8_S);
      }
    } else {
      const uint32_t so = (uint32_t)(kt - nk8) * 32 * sizeof(T);
#pragma unroll
      for (int j = 0; j < 2; ++j) dma16(rX, vxs[j], so, slot + F8_A + (2 * wave + j) * 1024);
#pragma unroll
      for (int j = 0; j < 2; ++j) dma16(rL, vsal[j], so, slot + F8_B + (2 * wave + j) * 1024);
      if (wave == 0) dma16(rR, (uint32_t)lane * 16, 0u, slot + F8_S);
    }
  };

  f32x16 tot[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) tot[i][r] = 0.f;

  const int brow = 32 * wave + l32;
  // code stage: e4m3 A (rows 32 i + l32) x e4m3 B (column brow), k half h of the block
  auto compute_f8 = [&](const unsigned char* __restrict__ slot) {
    const float s = *(const float*)(slot + F8_S + brow * 4);
    i32x8b b;
    {
      const u32x4 b0 = *(const u32x4*)(slot + F8_B + sw64(brow, 2 * h));
      const u32x4 b1 = *(const u32x4*)(slot + F8_B + sw64(brow, 2 * h + 1));
      b = i32x8b{(int)b0[0], (int)b0[1], (int)b0[2], (int)b0[3],
                 (int)b1[0], (int)b1[1], (int)b1[2], (int)b1[3]};
    }
    const f32x16 zero = {};
    auto ald = [&](int i) {
      const int ar = 32 * i + l32;
      const u32x4 a0 = *(const u32x4*)(slot + F8_A + sw64(ar, 2 * h));
      const u32x4 a1 = *(const u32x4*)(slot + F8_A + sw64(ar, 2 * h + 1));
      return i32x8b{(int)a0[0], (int)a0[1], (int)a0[2], (int)a0[3],
                    (int)a1[0], (int)a1[1], (int)a1[2], (int)a1[3]};
    };
    // software pipeline: A fragments read two tiles ahead, the MFMA of tile i + 1 issued
    // before the fold of tile i (which waits for its own MFMA's result); sched barriers
    // keep that order (left alone, hipcc folds each tile right after its MFMA)
    i32x8b a[2];
    a[0] = ald(0);
    a[1] = ald(1);
    f32x16 t[2];
    t[0] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[0], b, zero, 0, 0, 0, 127, 0, 127);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i + 1 < 8) {
        const i32x8b an = a[(i + 1) & 1];
        if (i + 2 < 8) a[i & 1] = ald(i + 2);
        t[(i + 1) & 1] =
            __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(an, b, zero, 0, 0, 0, 127, 0, 127);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 16; ++r) tot[i][r] = __builtin_fmaf(t[i & 1][r], s, tot[i][r]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // first tail stage: scale the integer part by the row scales (rows 32 i + (r & 3) +
  // 8 (r >> 2) + 4 h of the tile, from the stage's S image)
  auto apply_row_scales = [&](const unsigned char* __restrict__ slot) {
    const float* rs = (const float*)(slot + F8_S);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const f32x4 v = *(const f32x4*)(rs + 32 * i + 8 * r4 + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) tot[i][4 * r4 + e] *= v[e];
      }
  };
  // tail stage: exact D salient columns, 32 per stage, on the 32x32x16 D MFMA
  auto compute_tail = [&](const unsigned char* __restrict__ slot) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const u32x4 b = *(const u32x4*)(slot + F8_B + sw64(brow, 2 * st + h));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const u32x4 a = *(const u32x4*)(slot + F8_A + sw64(32 * i + l32, 2 * st + h));
        Mfma32<DT>::run(tot[i], a, b);
      }
    }
  };

  // ---- 4-slot ring, 3 stages in flight; per stage and wave 4 DMA ops (+1 on wave 0)
  const int npre = nkt < 3 ? nkt : 3;
  for (int k = 0; k < npre; ++k) issue(k);
  auto stage_top = [&](int kt) {
    const int ahead = nkt - 1 - kt;  // stages issued after kt that may stay in flight
    if (wave == 0) {
      if (ahead >= 2) vmw<10>();
      else if (ahead == 1) vmw<5>();
      else vmw<0>();
    } else {
      if (ahead >= 2) vmw<8>();
      else if (ahead == 1) vmw<4>();
      else vmw<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 3 < nkt) issue(kt + 3);
    return (const unsigned char*)(lds + (kt % F8_NSLOT) * F8_SLOT);
  };
  int kt = 0;
  for (; kt < nk8; ++kt) compute_f8(stage_top(kt));
  for (; kt < nkt; ++kt) {
    const unsigned char* slot = stage_top(kt);
    if (kt == nk8) apply_row_scales(slot);
    compute_tail(slot);
  }
  if (nkt == nk8) {  // no salient tail: row scales straight from global memory
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        tot[i][r] *= gm < M ? ascale[gm] : 0.f;
      }
  }

  // ---- epilogue: lane = column n0 + brow, rows 32 i + (r & 3) + 8 (r >> 2) + 4 h
  const int gn = n0 + brow;
  if (gn >= N) return;
  const float bv = bias ? DT::to_f(bias[gn]) : 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int gm = m0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (gm < M) Y[(size_t)gm * N + gn] = DT::from_f(tot[i][r] + bv);
    }
}

// ================================================================= gemm_f8v2
// Weight groups of whole 128-position blocks (Gw % 128 == 0): the same contraction on
// v_mfma_scale_f32_16x16x128_f8f6f4.  One MFMA covers a whole 128-position block, which
// lies in one weight group, so each 16 x 16 tile folds its exact integer block sum once per
// 128 positions: 4 fp32 FMAs per lane per MFMA, against 16 per 64 positions on the 32x32x64
// kernel above (whose fold kept the VALU, not the matrix pipe, busy: DESIGN.md §4).
//
// Tile 256 (m) x 256 (n) per 512-thread workgroup, 8 waves as 2 (m) x 4 (n), each wave
// 128 rows x 64 weight columns = 8 x 4 tiles of 16 x 16 (128 fp32 accumulators).  The
// weight fragment goes in the MFMA's A slot (D row = weight column), so a lane holds 4
// consecutive output columns of one activation row: one float4 of weight scales per tile
// column for the fold, one activation-row scale per tile row, 8-byte output stores.
// K-stages: 128-position code blocks (A and B images 256 rows x 128 B of e4m3 + the
// block's 256 fp32 weight scales), then the exact salient tail as 64-column D stages (the
// same 256 x 128 B images; 16x16x32 D MFMA into the same accumulators after the row
// scales are applied).  Two ring slots of 65 KiB; the DMA of stage k+1 (8 1-KiB pieces per
// wave through buffer resources, +1 scale piece on wave 0) runs under the compute of
// stage k.  LDS rows are 128 B with 16-B chunk c of row r at c ^ v2_sw(r), conflict-free
// for the ds_read_b128 lane groups of both the e4m3 fragment reads (chunks 2q, 2q + 1)
// and the D tail reads (chunk 4u + q).
namespace {
constexpr int V2_A = 0, V2_B = 32768, V2_S = 65536;
constexpr int V2_SLOT = 66560;  // A 32 KiB + B 32 KiB + S 1 KiB
constexpr int V2_NSLOT = 2;     // 133120 B

__device__ inline int v2_sw(int r) {
  return ((r >> 1) & 1) ^ (((r >> 2) & 1) << 2) ^ (((r >> 3) & 1) * 6);
}
__device__ inline int v2_off(int r, int c) { return (r << 7) + ((c ^ v2_sw(r)) << 4); }
__device__ inline i32x8b cat8(const u32x4& a, const u32x4& b) {
  return i32x8b{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}
}  // namespace

// OPT (A/B knob SQMP_F8_OPT, read per launch): bit 0 -- waves 4-7 at s_setprio 1 through the
// K loop; bit 1 -- loader split: waves 0-3 issue every DMA piece of a stage (their own and
// those of waves 4-7), waves 4-7 only wait, read and multiply
// DIAG (timing diagnostics, wrong results by design, only in a SQMP_DIAG_BUILD): 1 the code
// stages' DMA from two L2-hot stages, 2 no code-stage DMA after the first two stages, 3 no
// per-group fold (the MFMA accumulates straight into the totals)
// TMR (round 6): 256-row tiles, or 128-row tiles (8 waves as 2 x 4 of 64 rows x 64 columns)
// where the 256-row grid would leave CUs idle (2048-token Llama shapes: 128 tiles for
// N = 4096); the K order of every output is the same, so both are bit-identical.
template <class DT, int OPT = 0, int DIAG = 0, int TMR = 256>
__global__ __launch_bounds__(512, 1) void gemm_f8v2_kernel(
    const unsigned char* __restrict__ A8, const float* __restrict__ ascale,
    const typename DT::T* __restrict__ XS, const unsigned char* __restrict__ W8,
    const float* __restrict__ ws32, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n, int group_m,
    uint32_t* __restrict__ colmax, int nt) {
  typedef typename DT::T T;
  __shared__ __attribute__((aligned(16))) unsigned char lds[V2_NSLOT * V2_SLOT];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, group_m, tm, tn);
  constexpr int I = TMR / 32;       // 16-row activation tiles per wave
  constexpr int APW = TMR / 64;     // A pieces (8 rows x 128 B) per virtual wave per stage
  const int m0 = tm * TMR, n0 = tn * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int r16 = lane & 15, q = lane >> 4;
  const int nk8 = Kp / 128, nkt = nk8 + S_pad / 64;
  const int Np = pad_n(N);

  // ---- DMA geometry: piece p = 4 w + j moves rows 8p .. 8p + 7 of a 256 x 128 B image;
  // lane L writes row 8p + (L >> 3), physical chunk L & 7 = logical chunk (L & 7) ^ v2_sw
  // (offsets recomputed per stage: a few VALU ops instead of 12 live VGPRs)
  const i32x4b rA = rsrc_of(A8 + (size_t)m0 * Kp, 0xFFFFFFFFu);
  const i32x4b rW = rsrc_of(W8 + (size_t)n0 * Kp, 0xFFFFFFFFu);
  const i32x4b rX = rsrc_of(XS + (size_t)m0 * S_pad, 0xFFFFFFFFu);
  const i32x4b rL = rsrc_of(wsal, 0xFFFFFFFFu);
  const i32x4b rS = rsrc_of(ws32 + n0, 0xFFFFFFFFu);
  const i32x4b rR = rsrc_of(ascale + m0, (uint32_t)(M - m0) * 4u);  // rows >= M read 0

  constexpr bool SPLIT = (OPT & 2) != 0;
  auto issue = [&](int kt) {
    if (SPLIT && wave >= 4) return;
    unsigned char* slot = lds + (kt & 1) * V2_SLOT;
#pragma unroll
    for (int o = 0; o < (SPLIT ? 2 : 1); ++o) {
      const int w = wave + 4 * o;  // the (virtual) wave whose pieces these are
      const int r0 = 32 * w + (lane >> 3);          // weight rows (256 per tile)
      const int a0 = 8 * APW * w + (lane >> 3);     // activation rows (TMR per tile)
      auto row = [&](int j) { return r0 + 8 * j; };
      auto arow = [&](int j) { return a0 + 8 * j; };
      auto ch = [&](int r) { return (uint32_t)(((lane & 7) ^ v2_sw(r)) << 4); };
      if (kt < nk8) {
        if (DIAG == 2 && kt >= 2) continue;
        const uint32_t so = (uint32_t)(DIAG == 1 && kt >= 2 ? (kt & 1) : kt) * 128;
#pragma unroll
        for (int j = 0; j < APW; ++j)
          dma16(rA, (uint32_t)arow(j) * Kp + ch(arow(j)), so, slot + V2_A + (APW * w + j) * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          dma16(rW, (uint32_t)row(j) * Kp + ch(row(j)), so, slot + V2_B + (4 * w + j) * 1024);
      } else {
        const uint32_t so = (uint32_t)(kt - nk8) * 64 * sizeof(T);
#pragma unroll
        for (int j = 0; j < APW; ++j)
          dma16(rX, (uint32_t)arow(j) * S_pad * sizeof(T) + ch(arow(j)), so,
                slot + V2_A + (APW * w + j) * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          dma16(rL, (uint32_t)min(n0 + row(j), N - 1) * S_pad * sizeof(T) + ch(row(j)), so,
                slot + V2_B + (4 * w + j) * 1024);
      }
    }
    if (wave == 0) {
      if (kt < nk8) {
        const int g = min((kt * 128) / Gw, ngw - 1);
        dma16(rS, (uint32_t)lane * 16, (uint32_t)g * Np * 4, slot + V2_S);
      } else if (kt == nk8) {
        dma16(rR, (uint32_t)lane * 16, 0u, slot + V2_S);
      }
    }
  };

  f32x4 tot[I][4];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wcol0 = wn * 64 + r16;          // + 16 j: the lane's weight row in the B image
  const int xrow0 = wm * (TMR / 2) + r16;   // + 16 i: the lane's activation row in the A image
  auto compute_f8 = [&](const unsigned char* __restrict__ slot) {
    i32x8b bw[4];
    f32x4 sv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = wcol0 + 16 * j;
      bw[j] = cat8(*(const u32x4*)(slot + V2_B + v2_off(c, 2 * q)),
                   *(const u32x4*)(slot + V2_B + v2_off(c, 2 * q + 1)));
      sv[j] = *(const f32x4*)(slot + V2_S + (wn * 64 + 16 * j + 4 * q) * 4);
    }
    auto ald = [&](int i) {
      const int r = xrow0 + 16 * i;
      return cat8(*(const u32x4*)(slot + V2_A + v2_off(r, 2 * q)),
                  *(const u32x4*)(slot + V2_A + v2_off(r, 2 * q + 1)));
    };
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    // the 32 MFMAs u = 4 i + j (activation tile i, weight tile j) in order, the fold of MFMA
    // u - 2 issued behind MFMA u: two MFMAs (64 cycles) cover the result latency, so the
    // folds need no s_nop padding (one MFMA between them did: 14-18 nop cycles per tile);
    // tile i + 1's fragment read goes out with MFMA 4 i.  One sched barrier per MFMA keeps
    // that order (and the fragment reads from being hoisted: register pressure).
    i32x8b ax[2];
    ax[0] = ald(0);
    if constexpr (DIAG == 3) {
#pragma unroll
      for (int i = 0; i < I; ++i) {
        if (i + 1 < I) ax[(i + 1) & 1] = ald(i + 1);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          tot[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bw[j], ax[i & 1], tot[i][j], 0, 0, 0, 127, 0, 127);
        __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
    f32x4 t[3];
#pragma unroll
    for (int u = 0; u < 4 * I + 2; ++u) {
      const int i = u >> 2, j = u & 3;
      if (u < 4 * I) {
        if (j == 0 && i + 1 < I) ax[(i + 1) & 1] = ald(i + 1);
        t[u % 3] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bw[j], ax[i & 1], zero, 0, 0, 0, 127, 0, 127);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (u >= 2) {
        const int v = u - 2, vi = v >> 2, vj = v & 3;
#pragma unroll
        for (int r = 0; r < 4; ++r) tot[vi][vj][r] = __builtin_fmaf(t[v % 3][r], sv[vj][r], tot[vi][vj][r]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // first tail stage (or the end, without a tail): scale row 16 i + r16 by its act scale
  auto apply_row_scales = [&](const float* rs) {
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const float s = rs[xrow0 + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) tot[i][j] *= s;
    }
  };
  auto compute_tail = [&](const unsigned char* __restrict__ slot) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      u32x4 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *(const u32x4*)(slot + V2_B + v2_off(wcol0 + 16 * j, 4 * u + q));
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const u32x4 af = *(const u32x4*)(slot + V2_A + v2_off(xrow0 + 16 * i, 4 * u + q));
#pragma unroll
        for (int j = 0; j < 4; ++j) Mfma<DT>::run(tot[i][j], bf[j], af);
      }
    }
  };

  // ---- two-slot ring: stage k's DMA is the only one in flight when stage k starts.  One
  // loop per compute body (no branch between bodies inside a loop: the accumulators keep
  // their registers); the last code stage issues the first tail stage.
  auto top = [&](int kt) {
    vmw<0>();
    __builtin_amdgcn_s_barrier();  // every wave's pieces of stage kt have landed; every
    asm volatile("" ::: "memory");  // wave is past its reads of slot (kt + 1) & 1
    __builtin_amdgcn_sched_barrier(0);
    return (const unsigned char*)(lds + (kt & 1) * V2_SLOT);
  };
  issue(0);
  if ((OPT & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  int kt = 0;
  for (; kt + 1 < nk8; ++kt) {
    const unsigned char* slot = top(kt);
    issue(kt + 1);
    compute_f8(slot);
  }
  if (kt < nk8) {  // last code stage
    const unsigned char* slot = top(kt);
    if (kt + 1 < nkt) issue(kt + 1);
    compute_f8(slot);
    ++kt;
  }
  for (; kt < nkt; ++kt) {
    const unsigned char* slot = top(kt);
    if (kt + 1 < nkt) issue(kt + 1);
    if (kt == nk8) apply_row_scales((const float*)(slot + V2_S));
    compute_tail(slot);
  }
  if (nkt == nk8) {  // no salient tail: row scales straight from global memory
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int gm = m0 + xrow0 + 16 * i;
      const float s = gm < M ? ascale[gm] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) tot[i][j] *= s;
    }
  }

  // fused output-quant statistics (sqmp_gemm_f8_colmax): per output column the max of
  // |D(y)| over the lane's rows, the 16 r16 lanes, then one atomic per column and wave
  if (colmax) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nl = wn * 64 + 16 * j + 4 * q;
      float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float bv = (bias && n0 + nl + r < N) ? DT::to_f(bias[n0 + nl + r]) : 0.f;
#pragma unroll
        for (int i = 0; i < I; ++i)
          if (m0 + xrow0 + 16 * i < M)
            cm[r] = fmaxf(cm[r], fabsf(DT::to_f(DT::from_f(tot[i][j][r] + bv))));
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = cm[r];
        v = fmaxf(v, __shfl_xor(v, 1, 64));
        v = fmaxf(v, __shfl_xor(v, 2, 64));
        v = fmaxf(v, __shfl_xor(v, 4, 64));
        v = fmaxf(v, __shfl_xor(v, 8, 64));
        if (r16 == 0 && n0 + nl + r < N) atomicMax(colmax + n0 + nl + r, __float_as_uint(v));
      }
    }
  }

  // ---- epilogue, full-width tiles: the TMR x 256 output tile is staged in LDS (row m:
  // 512 B, 16-B chunk c at physical chunk c ^ (m & 31)), then each row leaves as one
  // 512-B run (32 lanes x 16 B) instead of 16 rows x 32 B per store instruction
  if (n0 + 256 <= N && (N & 7) == 0) {
    __builtin_amdgcn_s_barrier();  // every wave is past its last fragment read
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nl = wn * 64 + 16 * j + 4 * q;
      float bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = bias ? DT::to_f(bias[n0 + nl + r]) : 0.f;
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const int ml = xrow0 + 16 * i;
        T v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = DT::from_f(tot[i][j][r] + bv[r]);
        *(uint2*)(lds + ml * 512 + (((nl >> 3) ^ (ml & 31)) << 4) + (nl & 4) * 2) =
            *(const uint2*)v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's tile writes landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int c = tid & 31;
#pragma unroll
    for (int k = 0; k < TMR / 16; ++k) {
      const int ml = 16 * k + (tid >> 5);
      const u32x4 val = *(const u32x4*)(lds + ml * 512 + ((c ^ (ml & 31)) << 4));
      if (m0 + ml < M) {
        u32x4* dst = (u32x4*)(Y + (size_t)(m0 + ml) * N + n0 + c * 8);
        if (nt)  // streaming stores of a large output (nt_output)
          store16_nt(dst, val);
        else
          *dst = val;
      }
    }
    return;
  }

  // ---- epilogue: lane = row m0 + xrow0 + 16 i, columns n0 + wn 64 + 16 j + 4 q + r
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nb = n0 + wn * 64 + 16 * j + 4 * q;
    if (nb >= N) continue;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = (bias && nb + r < N) ? DT::to_f(bias[nb + r]) : 0.f;
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int gm = m0 + xrow0 + 16 * i;
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

// bpack int4 codes -> e4m3 bytes [Np][Kp] (natural packed order), D scales -> fp32.
template <class DT>
__global__ __launch_bounds__(256) void pack_f8_kernel(const uint32_t* __restrict__ codes,
                                                      const typename DT::T* __restrict__ wscale,
                                                      int Np, int Kp, int ngw,
                                                      uint32_t* __restrict__ w8,
                                                      float* __restrict__ ws32) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t words = (size_t)Np * (Kp / 4);  // 4 output bytes per thread
  if (w8 && t < words) {
    const int n = (int)(t / (Kp / 4));
    const int p0 = (int)(t % (Kp / 4)) * 4;
    uint32_t out = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int p = p0 + e;
      const uint32_t wd = codes[(size_t)n * (Kp / 8) + bpack_dword(p)];
      const int c = (int)((wd >> bpack_shift(p)) & 0xFu) - 8;
      const uint32_t b = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32((float)c, 0.f, 0, false) & 0xFFu;
      out |= b << (8 * e);
    }
    w8[t] = out;
  }
  if (t < (size_t)ngw * Np) ws32[t] = DT::to_f(wscale[t]);
}

}  // namespace sqmp

using namespace sqmp;

extern "C" int sqmp_pack_f8(const void* codes, const void* wscale, int dtype, int N, int Kp,
                            int ngw, void* w8, float* ws32, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!codes || !wscale || !ws32 || N <= 0 || Kp <= 0 || Kp % 128 != 0 || ngw <= 0)
    return SQMP_EINVAL;  // w8 = NULL: the scales only
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int Np = pad_n(N);
  const size_t words = (size_t)Np * (Kp / 4);
  const size_t n = words > (size_t)ngw * Np ? words : (size_t)ngw * Np;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == SQMP_F16)
    pack_f8_kernel<F16><<<grid, dim3(256), 0, s>>>((const uint32_t*)codes,
                                                    (const F16::T*)wscale, Np, Kp, ngw,
                                                    (uint32_t*)w8, ws32);
  else
    pack_f8_kernel<BF16><<<grid, dim3(256), 0, s>>>((const uint32_t*)codes,
                                                     (const BF16::T*)wscale, Np, Kp, ngw,
                                                     (uint32_t*)w8, ws32);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

static int gemm_f8_impl(const void* a8, const float* ascale, const void* xs, const void* w8,
                        const float* ws32, const void* wsal, const void* bias, void* y,
                        int dtype, int M, int N, int Kp, int S_pad, int Gw, int ngw,
                        uint32_t* colmax, void* stream) {
  if (M < 0 || N <= 0 || Kp <= 0 || Kp % 128 != 0 || S_pad < 0 || S_pad % 64 != 0)
    return SQMP_EINVAL;
  if (!a8 || !ascale || !w8 || !ws32 || !y || (S_pad > 0 && (!xs || !wsal))) return SQMP_EINVAL;
  if (Gw <= 0 || Gw % 64 != 0 || ngw <= 0) return SQMP_EUNSUPPORTED;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
  // Gw % 128 == 0 runs the 16x16x128 kernel (SQMP_F8_V1=1 keeps the 32x32x64 one, A/B)
  const char* v1e = knob("SQMP_F8_V1");
  const bool v1_only = v1e && atoi(v1e) != 0;
  const bool v2 = Gw % 128 == 0 && !v1_only;
  // v2 row tiles: 128 where the 256-row grid does not fill one round of the CUs (2048 x 4096
  // -> 4096: 128 tiles of 256 rows leave half the chip idle; 256 of 128 rows fill it: q/k/v/o
  // 54.0 -> 44.5 us, down_proj 146.5 -> 118 us).  Past one round the 256-row tiles stay (gate /
  // up, 344 tiles: 112 us, 129.5 on 688 of 128 rows; profiles/r06_token_fp16_layer_trace.txt).
  // SQMP_F8_TM = 128 / 256 overrides (A/B, read per launch)
  int tmr = 256;
  if (v2) {
    if ((long)cdiv(M, 256) * cdiv(N, 256) < 256) tmr = 128;
    if (const char* te = knob("SQMP_F8_TM")) tmr = atoi(te) == 128 ? 128 : 256;
  }
  const int tiles_m = cdiv(M, tmr), tiles_n = cdiv(N, 256);
  const dim3 grid(tiles_m * tiles_n), block(512);
  if (colmax && !v2) return SQMP_EUNSUPPORTED;  // fused statistics: the 16x16x128 kernel only
  // M-tiles per raster group (SQMP_GROUP_M: A/B knob, read per launch)
  const char* ge = knob("SQMP_GROUP_M");
  const int group_m = ge && atoi(ge) > 0 ? atoi(ge) : 4;
  const bool nt = nt_output((size_t)M * N * (dtype == SQMP_F32 ? 4 : 2));
  // default 2 (loader split): same-box config-2 per_token step 334.5 -> 324.0 us; setprio for
  // waves 4-7 +-0 (profiles/r03_ab_f8_opt.txt).  SQMP_F8_OPT: A/B knob, read per launch
  const char* oe = knob("SQMP_F8_OPT");
  const int opt = oe ? atoi(oe) & 3 : 2;
#define SQMP_F8V2T(DTT, O, TR)                                                               \
  gemm_f8v2_kernel<DTT, O, 0, TR><<<grid, block, 0, s>>>(                                    \
      (const unsigned char*)a8, ascale, (const DTT::T*)xs, (const unsigned char*)w8, ws32,   \
      (const DTT::T*)wsal, (const DTT::T*)bias, (DTT::T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, \
      tiles_n, group_m, colmax, nt ? 1 : 0)
#define SQMP_F8V2(DTT, O) \
  if (tmr == 128) { SQMP_F8V2T(DTT, O, 128); } else { SQMP_F8V2T(DTT, O, 256); }
#ifdef SQMP_DIAG_BUILD
  const char* de = knob("SQMP_F8_DIAG");  // (sqmp_knobs.hip)
  const int diag = de ? atoi(de) : 0;
#define SQMP_F8D(DTT, D)                                                                     \
  gemm_f8v2_kernel<DTT, 2, D><<<grid, block, 0, s>>>(                                        \
      (const unsigned char*)a8, ascale, (const DTT::T*)xs, (const unsigned char*)w8, ws32,   \
      (const DTT::T*)wsal, (const DTT::T*)bias, (DTT::T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, \
      tiles_n, group_m, colmax, nt ? 1 : 0)
  if (v2 && dtype == SQMP_F16 && diag > 0 && tmr == 256) {
    if (diag == 1) SQMP_F8D(F16, 1); else if (diag == 2) SQMP_F8D(F16, 2); else SQMP_F8D(F16, 3);
    SQMP_LAUNCH_CHECK();
    return SQMP_OK;
  }
#undef SQMP_F8D
#endif
#define SQMP_F8L(DTT)                                                                        \
  if (v2) {                                                                                  \
    switch (opt) {                                                                           \
      case 1: SQMP_F8V2(DTT, 1); break;                                                      \
      case 2: SQMP_F8V2(DTT, 2); break;                                                      \
      case 3: SQMP_F8V2(DTT, 3); break;                                                      \
      default: SQMP_F8V2(DTT, 0); break;                                                     \
    }                                                                                        \
  }                                                                                          \
  else gemm_f8_kernel<DTT><<<grid, block, 0, s>>>(                                           \
      (const unsigned char*)a8, ascale, (const DTT::T*)xs, (const unsigned char*)w8, ws32,   \
      (const DTT::T*)wsal, (const DTT::T*)bias, (DTT::T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, \
      tiles_n)
  if (dtype == SQMP_F16) {
    SQMP_F8L(F16);
  } else {
    SQMP_F8L(BF16);
  }
#undef SQMP_F8L
#undef SQMP_F8V2
#undef SQMP_F8V2T
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

extern "C" int sqmp_gemm_f8(const void* a8, const float* ascale, const void* xs, const void* w8,
                            const float* ws32, const void* wsal, const void* bias, void* y,
                            int dtype, int M, int N, int Kp, int S_pad, int Gw, int ngw,
                            void* stream) {
  SQMP_DEVICE_GUARD(stream);
  return gemm_f8_impl(a8, ascale, xs, w8, ws32, wsal, bias, y, dtype, M, N, Kp, S_pad, Gw, ngw,
                      nullptr, stream);
}

// sqmp_gemm_f8 with the fused output-quant statistics (as sqmp_gemm_fq_colmax); Gw % 128 == 0
extern "C" int sqmp_gemm_f8_colmax(const void* a8, const float* ascale, const void* xs,
                                   const void* w8, const float* ws32, const void* wsal,
                                   const void* bias, void* y, int dtype, int M, int N, int Kp,
                                   int S_pad, int Gw, int ngw, uint32_t* colmax, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!colmax) return SQMP_EINVAL;
  return gemm_f8_impl(a8, ascale, xs, w8, ws32, wsal, bias, y, dtype, M, N, Kp, S_pad, Gw, ngw,
                      colmax, stream);
}
