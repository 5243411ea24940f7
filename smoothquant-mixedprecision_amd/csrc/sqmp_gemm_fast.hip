// Fast W4A4 GEMMs for gfx950 (fp16 / bf16): the F.linear of fake_quant.py:306.
//
// gemm_fq5 -- the faithful mixed-precision GEMM
//   y[M][N] = D( A[M][Kp + S_pad] . B^T + bias ):  A = dequantized activations x_hat in
//   packed K order + the exact salient columns (bit-exact with the reference's q_x);
//   B = int4 codes decoded in registers to D(code * scale) (bit-exact with the
//   reference's W_hat), then the exact salient weight slice; v_mfma_f32_32x32x16 in D,
//   fp32 accumulation, one rounding to D.
//
//   Tile 256 (M) x 256 (N) per 512-thread workgroup: 8 waves as WMW (M) x 8/WMW (N), two
//   waves per SIMD, 128 fp32 accumulators per lane.  The 32x32x16 MFMA holds the SIMD's
//   vector issue for 8 of its 32 cycles (16x16x32: 8 of 16), which leaves the issue
//   slots the int4 decode needs.  Every main-loop global byte moves by LDS-DMA
//   (global_load_lds_dwordx4) into a 3-slot LDS ring, two 64-element K-stages ahead:
//     A  256 rows x 128 B, 16-B chunks permuted (bitrev3) and XOR-swizzled by (row >> 1) & 7
//     B  256 weight rows x one 32-B bpack block; lane half h reads its 16-B half (its four
//        sub-step fragments) with one ds_read_b128, halves swizzled by (row >> 3) & 1
//     S  the block's group scales, 1 KiB per wave (its columns).
//   Waits are hand-counted (`s_waitcnt vmcnt(N)` keeps the next stage in flight), the
//   workgroup syncs once per stage with a raw s_barrier, and the LDS reads carry
//   restrict-scoped alias info, so the compiler adds no drain of the ring.  Dense stages
//   (the exact salient slice; every stage for dense weights) are 32 columns wide: A and
//   B both 256 rows x 64 B in the slot, chunks swizzled by (row >> 2) & 3.
//   The MFMA takes the weight fragment in its A slot, so each lane holds 4 consecutive
//   output columns of one row: 8-byte stores in the epilogue.
//
// gemm_i8v2 -- per_token / per_tensor activations on the integer MFMA (see below).
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

// LDS images of the ring, shared by the 32x32x16 (fq5) and 16x16x32 (fq6) kernels:
//   codes-stage A: 256 rows x 128 B, logical 16-B chunk c of row r at physical chunk
//     a_pchunk(c, r) = bitrev3(c) ^ ((r >> 1) & 7) -- conflict-free for both fragment
//     read patterns (32x32: chunk 2u+h; 16x16: chunk 4(q&1)+2s+(q>>1));
//   dense-stage A and B: 256 rows x 64 B, chunk c of row r at c ^ d_f((r >> 2) & 3).
__host__ __device__ inline int bitrev3(int c) { return ((c & 1) << 2) | (c & 2) | ((c >> 2) & 1); }
__device__ inline int a_pchunk(int c, int r) { return bitrev3(c) ^ ((r >> 1) & 7); }
__device__ inline int d_f(int g) { return (-g) & 3; }

// GB = weight groups per 64-position block (1: Gw % 64 == 0, 2: Gw == 32);
// GB = 0: dense D weights (no codes) in every main stage.  WMW = waves along M (1 or 2);
// PF = A-fragment read-ahead (blocks); NOWAIT = 1 is a timing diagnostic only (skips the
// DMA waits, so results are garbage; every address stays in bounds).
template <class DT, int GB, int WMW, int PF = 3, int NOWAIT = 0>
__global__ __launch_bounds__(512, 1) void gemm_fq5_kernel(
    const typename DT::T* __restrict__ A, const void* __restrict__ Bw,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  constexpr int NWV = 8 / WMW;        // waves along N
  constexpr int MW = 256 / WMW;       // rows per wave
  constexpr int CW = 256 / NWV;       // weight rows (output columns) per wave
  constexpr int I = MW / 32, J = CW / 32;
  constexpr int GBn = GB > 0 ? GB : 1;
  constexpr int LPG = CW / 8;         // scale-DMA lanes per group (8 scales per lane)
  __shared__ __attribute__((aligned(16))) unsigned char lds[F5_NSLOT * F5_SLOT];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, 4, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWV, wn = wave % NWV;
  const int r32 = lane & 31, h = lane >> 5;
  const int lda = Kp + S_pad;
  const int nkm = GB ? Kp / 64 : 0;       // 64-column stages that carry int4 codes
  const int nkt = nkm + (lda - nkm * 64) / 32;  // + 32-column dense stages
  const int Np = pad_n(N);

  // ---- per-lane DMA source offsets (bytes); per-instruction steps are scalar
  // dense stage: A and B as 256 rows x 64 B, chunk c of row r at ((c ^ ((r >> 2) & 3)) << 4)
  const int drow = 16 * wave + (lane >> 2);
  const int dchunk = (lane & 3) ^ d_f((lane >> 4) & 3);
  const uint32_t ad_off = (uint32_t)((size_t)(m0 + drow) * lda * sizeof(T) + dchunk * 16);
  const uint32_t ad_str = (uint32_t)(128 * (size_t)lda * sizeof(T));
  const uint32_t bd_row0 = (uint32_t)min(n0 + drow, N - 1);
  const uint32_t bd_row1 = (uint32_t)min(n0 + drow + 128, N - 1);
  const int arow = 8 * wave + (lane >> 3);
  const uint32_t a_off = (uint32_t)((size_t)(m0 + arow) * lda * sizeof(T) +
                                    (bitrev3((lane & 7) ^ ((arow >> 1) & 7)) << 4));
  const uint32_t a_str = (uint32_t)(64 * (size_t)lda * sizeof(T));
  const uint32_t b_off = (uint32_t)((size_t)(n0 + 32 * wave + (lane >> 1)) * (Kp / 2) +
                                    (((lane & 1) ^ ((lane >> 4) & 1)) << 4));
  const int s_u = min(lane / LPG, GBn - 1);
  const uint32_t s_off = (uint32_t)((n0 + CW * wn + (lane % LPG) * 8) * sizeof(T));

  // DMA of stage kt into its ring slot: codes stages (kt < nkm) 4 A + 1 B + 1 S ops,
  // dense stages 2 A + 2 B ops per wave.
  auto issue = [&](int kt) {
    unsigned char* slot = lds + (kt % F5_NSLOT) * F5_SLOT;
    if (kt < nkm) {
      const unsigned char* ab = (const unsigned char*)A + (size_t)kt * 64 * sizeof(T);
#pragma unroll
      for (int i = 0; i < 4; ++i) glds16(ab + (size_t)i * a_str + a_off, slot + (i * 8 + wave) * 1024);
      glds16((const unsigned char*)Bw + (size_t)kt * 32 + b_off, slot + F5_A + wave * 1024);
      const int g0 = GB == 1 ? (kt * 64) / Gw : kt * 2;
      const int g = min(g0 + s_u, ngw - 1);  // zero-code padding past the last group
      glds16((const unsigned char*)wscale + (size_t)g * Np * sizeof(T) + s_off,
             slot + F5_A + F5_B + wave * 1024);
    } else {
      const int col = nkm * 64 + (kt - nkm) * 32;
      const unsigned char* ab = (const unsigned char*)A + (size_t)col * sizeof(T);
      glds16(ab + ad_off, slot + wave * 1024);
      glds16(ab + ad_str + ad_off, slot + (8 + wave) * 1024);
      const bool main = col < Kp;  // dense main weights (GB == 0) or the salient slice
      const unsigned char* bb = main ? (const unsigned char*)Bw : (const unsigned char*)wsal;
      const uint32_t ldb = main ? (uint32_t)Kp : (uint32_t)S_pad;
      const uint32_t c0 = (uint32_t)(main ? col : col - Kp) * sizeof(T) + dchunk * 16;
      glds16(bb + bd_row0 * ldb * sizeof(T) + c0, slot + F5_DB + wave * 1024);
      glds16(bb + bd_row1 * ldb * sizeof(T) + c0, slot + F5_DB + (8 + wave) * 1024);
    }
  };

  f32x16 acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const DecK dk = make_deck();

  // A fragment t = I*u + i (sub-step u, M tile i) of a slot: rows of one wave share the
  // swizzle (r32 >> 1) & 7, so tiles differ by an immediate 4 KiB.
  const int a_row0 = (wm * MW + r32) * 128;
  const int a_sw = (r32 >> 1) & 7;
  auto ald = [&](const unsigned char* __restrict__ slot, int t) {
    return *(const u32x4*)(slot + a_row0 + (t % I) * 4096 + ((bitrev3(2 * (t / I) + h) ^ a_sw) << 4));
  };
  // 4*I blocks of J MFMAs; the A fragment of block t+3 is read during block t, one
  // sched_barrier per block keeps the compiler from hoisting every read, and HOOK runs
  // the decode of the next sub-step under the MFMAs.
#define SQMP_FQ5_BLOCKS(BF, ...)                                               \
  {                                                                            \
    u32x4 a[PF + 1];                                                           \
    _Pragma("unroll") for (int t = 0; t < PF; ++t) a[t] = ald(slot, t);        \
    _Pragma("unroll") for (int t = 0; t < 4 * I; ++t) {                        \
      if (t + PF < 4 * I) a[(t + PF) % (PF + 1)] = ald(slot, t + PF);          \
      _Pragma("unroll") for (int j = 0; j < J; ++j)                            \
          Mfma32<DT>::run(acc[t % I][j], BF(t / I, j), a[t % (PF + 1)]);       \
      __VA_ARGS__;                                                             \
      __builtin_amdgcn_sched_barrier(0);                                       \
    }                                                                          \
  }

  auto compute_codes = [&](const unsigned char* __restrict__ slot) {
    const unsigned char* sb = slot + F5_A;
    const unsigned char* ss = slot + F5_A + F5_B + wave * 1024;
    u32x4 bw[J];
    uint32_t sp[J][GBn];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int row = wn * CW + 32 * j + r32;
      bw[j] = *(const u32x4*)(sb + row * 32 + ((h ^ ((r32 >> 3) & 1)) << 4));
#pragma unroll
      for (int g = 0; g < GBn; ++g)
        sp[j][g] = Dec<DT>::prep(*(const uint16_t*)(ss + g * CW * 2 + (32 * j + r32) * 2));
    }
    u32x4 bf[2][J];
#pragma unroll
    for (int j = 0; j < J; ++j) bf[0][j] = Dec<DT>::run(bw[j][0], sp[j][0], dk);
#define SQMP_BF_CODES(u, j) bf[(u) & 1][j]
    SQMP_FQ5_BLOCKS(SQMP_BF_CODES,
                    if (t / I < 3 && t % I >= 1 && t % I <= J) {
                      const int un = t / I + 1, jj = t % I - 1;
                      bf[un & 1][jj] = Dec<DT>::run(bw[jj][un], sp[jj][GB == 2 ? (un >> 1) : 0], dk);
                    });
#undef SQMP_BF_CODES
  };

  // dense stage: two 16-element sub-steps, A and B fragments both from the slot
  const int d_sw = d_f((r32 >> 2) & 3);
  auto compute_dense = [&](const unsigned char* __restrict__ slot) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int co = ((2 * u + h) ^ d_sw) << 4;
      u32x4 bf[J];
#pragma unroll
      for (int j = 0; j < J; ++j) bf[j] = *(const u32x4*)(slot + F5_DB + (wn * CW + 32 * j + r32) * 64 + co);
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const u32x4 af = *(const u32x4*)(slot + (wm * MW + 32 * i + r32) * 64 + co);
#pragma unroll
        for (int j = 0; j < J; ++j) Mfma32<DT>::run(acc[i][j], bf[j], af);
      }
    }
  };
#undef SQMP_FQ5_BLOCKS

  // ---- the ring: stage kt lives in slot kt % 3, issued two stages ahead.  One loop per
  // compute body, so the accumulators keep their registers across iterations.
  issue(0);
  if (nkt > 1) issue(1);
  int kt = 0;
  for (; kt < nkm; ++kt) {
    // retire stage kt; the DMA of stage kt+1 (issued after it) may stay in flight
    if (kt + 1 < nkt) {
      if (NOWAIT) {
      } else if (kt + 1 < nkm) vm_wait<F5_VM_CODES>();
      else vm_wait<F5_VM_DENSE>();
    } else {
      vm_wait<0>();
    }
    if (NOWAIT < 2) raw_barrier();  // every wave's DMA for stage kt has landed; slot (kt+2)%3 is free
    if (kt + 2 < nkt) issue(kt + 2);
    compute_codes(lds + (kt % F5_NSLOT) * F5_SLOT);
  }
  for (; kt < nkt; ++kt) {
    if (kt + 1 < nkt) {
      if (!NOWAIT) vm_wait<F5_VM_DENSE>();
    } else {
      vm_wait<0>();
    }
    raw_barrier();
    if (kt + 2 < nkt) issue(kt + 2);
    compute_dense(lds + (kt % F5_NSLOT) * F5_SLOT);
  }

  // ---- epilogue: acc[i][j][4 rr + r] = C[n = n0 + CW wn + 32 j + 8 rr + 4 h + r]
  //                                        [m = m0 + MW wm + 32 i + r32]
  // bias: every load issued before the first use (clamped columns, one wait)
  float bvs[J][4][4];
  if (bias) {
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          bvs[j][rr][r] = DT::to_f(bias[min(n0 + wn * CW + 32 * j + 8 * rr + 4 * h + r, N - 1)]);
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int r = 0; r < 4; ++r) bvs[j][rr][r] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int nb = n0 + wn * CW + 32 * j + 8 * rr + 4 * h;
      if (nb >= N) continue;
      const float* bv = bvs[j][rr];
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const int gm = m0 + wm * MW + 32 * i + r32;
        if (gm >= M) continue;
        T v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = DT::from_f(acc[i][j][4 * rr + r] + bv[r]);
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
}

// ================================================================= gemm_fq6
// The fq5 ring and wave layout (1 x 8 waves, 256 x 32 per wave) on v_mfma_f32_16x16x32:
// 16 x 2 tiles of 16 x 16 per wave (128 fp32 accumulators), two 32-element sub-steps per
// 64-element stage.  Lane (r16, q) of sub-step s takes bpack dword 2q + s of its weight
// row (one ds_read_b64 per tile column carries both sub-steps) and A chunk
// 4 (q & 1) + 2 s + (q >> 1) -- the positions of that dword.  Same DMA ring and waits as
// fq5.  Dense stages (the exact salient slice; every stage for dense weights) are 64
// columns wide over 128 rows of the tile (two half-height stages per 64-column block when
// TM = 256): A 128 rows x 128 B + B 256 weight rows x 128 B fill one 48 KiB slot, every
// DMA moves whole 128-B lines, both images use the codes-stage A swizzle, and lane
// (r16, q) of sub-step s reads chunk 4 (q & 1) + 2 s + (q >> 1) of A and B alike.
// PRIO (tuning knob): 0 none; 1 = one s_setprio 1 for the younger half (waves 4-7) before
// the main loop; 2 = s_setprio 1 / 0 around each stage's compute (MI355X guide T5).
// WM = waves along M (1: 1 x 8 waves of TM x 32; 2: 2 x 4 waves of TM/2 x 64).
template <class DT, int GB, int TM, int PRIO = 0, int WM = 1, int PF = 3>
__global__ __launch_bounds__(512, 1) void gemm_fq6_kernel(
    const typename DT::T* __restrict__ A, const void* __restrict__ Bw,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
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
  // Loader split (default, codes stages): waves 0-3 issue the DMA pieces of all 8 waves,
  // waves 4-7 (one per SIMD, beside a loader) issue none.  An LDS-DMA piece holds up its
  // wave's instruction stream for ≈60-185 cycles (MI355X_MICROARCH.md cycle table), so a
  // wave that issues none keeps its SIMD's MFMA pipe fed meanwhile (config-2 GEMM +3-4 %;
  // handing the scale piece, or the B and scale pieces, back to their own wave: -7 / -9 %).
  // PRIO 24 = every wave issues its own pieces (the previous scheme, A/B only); LB / LS
  // (variants 22 / 23) = B / scale pieces by the owning wave.
  constexpr bool LSPLIT = PRIO == 0 || PRIO == 19 || PRIO == 20 || PRIO == 22 || PRIO == 23;
  constexpr bool LB = LSPLIT && PRIO != 23, LS = LSPLIT && PRIO != 22 && PRIO != 23;
  constexpr int VM_LOAD = 2 * NA + (LB ? 2 : 1) + (LS ? 2 : 1);  // loader ops per codes stage
  constexpr int VM_COMP = (LB ? 0 : 1) + (LS ? 0 : 1);            // ... of waves 4-7
  __shared__ __attribute__((aligned(16))) unsigned char lds[F5_NSLOT * F5_SLOT];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, 4, tm, tn);
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
      // PRIO 6 (diagnostic): every codes stage re-reads stage 0's bytes (L2-resident)
      const int ks = PRIO == 6 ? 0 : kt;
      const uint32_t sa = (uint32_t)ks * 64 * sizeof(T);
#pragma unroll
      for (int i = 0; i < NA; ++i)
        if ((PRIO != 8 || kt < 2) && (!LSPLIT || wave < 4)) {
          blds16(rA, a_off, sa + i * a_str, slot + (i * 8 + wave) * 1024);
          // PRIO 18: waves 0-3 also move waves 4-7's pieces (rows + 32, columns + 128)
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
      // PRIO 15 (diagnostic): no scale pieces after the first two stages
      if ((PRIO != 15 || kt < 2) && (!LS || wave < 4)) {
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

  // PRIO 4 / 5 are timing diagnostics (garbage results, in-bounds addresses): 4 keeps
  // the DMA but skips every wait on it, 5 moves no bytes after the first two stages.
  constexpr bool DIAG_NOWAIT = PRIO == 4 || PRIO == 5 || PRIO == 8 || PRIO == 12 || PRIO == 15;  // 8: no A DMA in the loop
  constexpr bool DIAG_NOBAR = PRIO == 12;  // 12: no waits and no barriers in the codes loop
  issue(0);
  if (nkt > 1) issue(1);
  if ((PRIO == 1 || PRIO == 19) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  if (PRIO == 20 && wave < 4) __builtin_amdgcn_s_setprio(1);
  int kt = 0;
  for (; kt < nkm; ++kt) {
    if (DIAG_NOWAIT && kt >= 2) {
    } else if (kt + 1 < nkt) {
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
    if (!DIAG_NOBAR || kt < 2) raw_barrier();
    if (kt + 2 < nkt && PRIO != 5) issue(kt + 2);
    if (PRIO == 2) __builtin_amdgcn_s_setprio(1);
    compute_codes(lds + (kt % F5_NSLOT) * F5_SLOT);
    if (PRIO == 2) __builtin_amdgcn_s_setprio(0);
  }
  for (; kt < nkt; ++kt) {
    if (DIAG_NOWAIT && kt + 1 < nkt) {
    } else if (kt + 1 < nkt) {
      vm_wait<VM_DENSE>();
    } else {
      vm_wait<0>();
    }
    raw_barrier();
    if (kt + 2 < nkt && PRIO != 5) issue(kt + 2);
    unsigned char* slot = lds + (kt % F5_NSLOT) * F5_SLOT;
    if (PRIO == 2) __builtin_amdgcn_s_setprio(1);
    if constexpr (DW == 64)
      compute_dense(slot, std::integral_constant<int, 0>());
    else
      compute_dense32(slot);
    if (PRIO == 2) __builtin_amdgcn_s_setprio(0);
  }
  if (PRIO == 1 || PRIO == 19 || PRIO == 20) __builtin_amdgcn_s_setprio(0);

  // ---- epilogue: acc[i][j][r] = C[n = n0 + CW wn + 16 j + 4 q + r][m = m0 + MW wm + 16 i + r16]
  {
    // Full-width tiles: the TM x 256 output tile is staged in LDS (row m: 512 B, 16-B
    // chunk c at c ^ (m & 15), conflict-free both ways) and stored as whole rows, one 16-B
    // chunk per lane (two rows per wave instruction, 4 full 128-B lines each) instead of
    // 8-B pieces of 16 rows (config-2 GEMM +2.8 %).
    if (n0 + 256 <= N && (N & 7) == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();  // every wave is past its last read of the ring
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
          const int c = nl >> 3;
          *(uint2*)(lds + ml * 512 + ((c ^ (ml & 15)) << 4) + (nl & 4) * 2) = *(const uint2*)v;
        }
      }
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

// ================================================================= gemm_i8v2
// per_token / per_tensor activations: int8 act codes x int4 weight codes on
// v_mfma_i32_16x16x64_i8, per-weight-group fp32 fold, per-row act scale, salient tail on
// the D MFMA into the same accumulators.  128 x 128 tile, 4 waves as 2 (M) x 2 (N), each
// 64 x 64.  A stages hold 256 int8 codes (4 bpack blocks) per row: i8 sub-step t (one
// 64-code block) reads chunk 4 t + q; the activation codes were written in the K order
// that matches unpack_i8 of the bpack dword pair of lane group q.
struct StageA256 {
  uint32_t off, off_half, stride16;
  __device__ inline void init(int m0, size_t lda_b, int wave, int lane) {
    const int rin = 4 * wave + (lane >> 4);
    const int c = (lane & 15) ^ (rin & 15);
    off = (uint32_t)((size_t)(m0 + rin) * lda_b + (c << 4));
    // a half stage (the last 64 salient columns when S_pad % 128 == 64): the upper 8
    // chunks re-read the lower ones (in bounds; those sub-steps are skipped)
    off_half = (uint32_t)((size_t)(m0 + rin) * lda_b + ((c & 7) << 4));
    stride16 = (uint32_t)(16 * lda_b);
  }
  __device__ inline void issue(const unsigned char* base, unsigned char* st, int wave,
                               bool half = false) const {
    const uint32_t o = half ? off_half : off;
#pragma unroll
    for (int i = 0; i < 8; ++i) glds16(base + (size_t)i * stride16 + o, st + (i * 4 + wave) * 1024);
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
  const int nks = (S_pad + 127) / 128;  // 128-element salient stages (the last may be 64)
  const bool tail_half = (S_pad & 127) != 0;
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
        b[j][t] = *(const uint2*)(B4 + (size_t)nrow[j] * brow_dw + (size_t)blk * 8 + 4 * (q & 1) + 2 * (q >> 1));
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
    sx.issue(Xb, lds, wave, tail_half && nks == 1);
    __syncthreads();
    for (int ks = 0; ks < nks; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nks)
        sx.issue(Xb + (size_t)(ks + 1) * 128 * sizeof(T), lds + (cur ^ 1) * ST, wave,
                 tail_half && ks + 2 == nks);
      const unsigned char* st = lds + cur * ST;
      const int nsub = tail_half && ks + 1 == nks ? 2 : 4;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (s >= nsub) break;
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
template <class DT, int GB, int WMW, int PF = 3, int NOWAIT = 0>
static int fq5_launch(const void* a, const void* codes, const void* wscale, const void* wsal,
                      const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                      int ngw, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, 256), tiles_n = cdiv(N, 256);
  gemm_fq5_kernel<DT, GB, WMW, PF, NOWAIT><<<dim3(tiles_m * tiles_n), dim3(512), 0, s>>>(
      (const T*)a, codes, (const T*)wscale, (const T*)wsal, (const T*)bias, (T*)y, M, N, Kp,
      S_pad, Gw, ngw, tiles_m, tiles_n);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT, int WMW>
static int fq5_dispatch(const void* a, const void* codes, const void* wscale, const void* wsal,
                        const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                        int ngw, int n_bits, hipStream_t s) {
  if (n_bits == 0) return fq5_launch<DT, 0, WMW>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, 1, 1, s);
  if (n_bits != 4) return SQMP_EUNSUPPORTED;
  if (Gw % 64 == 0) return fq5_launch<DT, 1, WMW>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s);
  if (Gw == 32) return fq5_launch<DT, 2, WMW>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s);
  return SQMP_EUNSUPPORTED;
}

static int fq6_prio() {
  static int v = [] {
    const char* e = getenv("SQMP_FQ6_PRIO");
    return e ? atoi(e) : 0;
  }();
  return v;
}
static int fq6_wm() {
  static int v = [] {
    const char* e = getenv("SQMP_FQ6_WM");
    return e ? atoi(e) : 1;
  }();
  return v;
}

template <class DT, int GB, int TM>
static int fq6_launch(const void* a, const void* codes, const void* wscale, const void* wsal,
                      const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                      int ngw, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, TM), tiles_n = cdiv(N, 256);
#define SQMP_FQ6_L(PR, WMV)                                                                   \
  gemm_fq6_kernel<DT, GB, TM, PR, WMV><<<dim3(tiles_m * tiles_n), dim3(512), 0, s>>>(         \
      (const T*)a, codes, (const T*)wscale, (const T*)wsal, (const T*)bias, (T*)y, M, N, Kp, \
      S_pad, Gw, ngw, tiles_m, tiles_n)
  const int pr = fq6_prio();
  bool done = false;
  if constexpr (TM >= 128) {
    if (fq6_wm() == 2) {
      SQMP_FQ6_L(0, 2);
      done = true;
    }
  }
  if (done) {
  } else if (pr == 1) SQMP_FQ6_L(1, 1);
  else if (pr == 2) SQMP_FQ6_L(2, 1);
  else if (pr == 4) SQMP_FQ6_L(4, 1);  // diagnostics (wrong results): no DMA waits
  else if (pr == 5) SQMP_FQ6_L(5, 1);  // ... no DMA after the first two stages
  else if (pr == 6) SQMP_FQ6_L(6, 1);  // ... codes stages re-read stage 0 (L2 hits)
  else if (pr == 8) SQMP_FQ6_L(8, 1);  // ... codes stages move B and S only
  else if (pr == 12) SQMP_FQ6_L(12, 1);  // ... no waits, no barriers in the codes loop
  else if (pr == 15) SQMP_FQ6_L(15, 1);  // diagnostic: no scale pieces in the loop
  else if (pr == 19) SQMP_FQ6_L(19, 1);  // loader split + compute waves 4-7 at priority 1
  else if (pr == 20) SQMP_FQ6_L(20, 1);  // loader split + loader waves 0-3 at priority 1
  else if (pr == 22) SQMP_FQ6_L(22, 1);  // loader split, scale pieces by their own wave
  else if (pr == 23) SQMP_FQ6_L(23, 1);  // loader split, B and scale pieces by their own wave
  else if (pr == 24) SQMP_FQ6_L(24, 1);  // every wave issues its own pieces (pre-split)
  else if (pr == 3)  // A-fragment read-ahead of 5 blocks (tuning)
    gemm_fq6_kernel<DT, GB, TM, 0, 1, 5><<<dim3(tiles_m * tiles_n), dim3(512), 0, s>>>(
        (const T*)a, codes, (const T*)wscale, (const T*)wsal, (const T*)bias, (T*)y, M, N, Kp,
        S_pad, Gw, ngw, tiles_m, tiles_n);
  else SQMP_FQ6_L(0, 1);
#undef SQMP_FQ6_L
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT>
static int fq6_dispatch(const void* a, const void* codes, const void* wscale, const void* wsal,
                        const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                        int ngw, int n_bits, hipStream_t s) {
  // 128-row tiles when 256-row tiles would leave the chip under two workgroups per CU;
  // 64-row tiles when even 128-row tiles would leave CUs idle (e.g. OPT-1.3B's 2048-wide
  // layers at 2048 tokens: 128 tiles of 128 x 256)
  const long t256 = (long)cdiv(M, 256) * cdiv(N, 256), t128 = (long)cdiv(M, 128) * cdiv(N, 256);
  const int tm = t256 >= 2L * 256 ? 256 : (t128 >= 256 || M <= 64 ? 128 : 64);
#define SQMP_FQ6(GB, GW, NGW)                                                                     \
  (tm == 256 ? fq6_launch<DT, GB, 256>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, GW, NGW, s) \
   : tm == 128 ? fq6_launch<DT, GB, 128>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, GW, NGW, s) \
               : fq6_launch<DT, GB, 64>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, GW, NGW, s))
  if (n_bits == 0) return SQMP_FQ6(0, 1, 1);
  if (n_bits != 4) return SQMP_EUNSUPPORTED;
  if (Gw % 64 == 0) return SQMP_FQ6(1, Gw, ngw);
  if (Gw == 32) return SQMP_FQ6(2, Gw, ngw);
  return SQMP_EUNSUPPORTED;
#undef SQMP_FQ6
}

// GEMM variant (tuning knob SQMP_FQ_VARIANT): default "fq6" (16x16x32, 1 x 8 waves);
// "wm1" = fq5 (32x32x16, 1 x 8), "wm2" = fq5 (2 x 4), "pf6" = fq5 with a 6-block A
// read-ahead, "nowait" / "nobar" = fq5 timing diagnostics that skip the DMA waits / also
// the stage barrier of the codes loop (wrong results, in-bounds addresses).
static int fq_variant() {
  static int v = [] {
    const char* e = getenv("SQMP_FQ_VARIANT");
    if (!e || !strcmp(e, "fq6")) return 5;
    if (!strcmp(e, "wm1") || !strcmp(e, "fq5")) return 0;
    if (!strcmp(e, "wm2")) return 1;
    if (!strcmp(e, "pf6")) return 2;
    if (!strcmp(e, "nowait")) return 3;
    if (!strcmp(e, "nobar")) return 4;
    return 5;
  }();
  return v;
}

int launch_gemm_fq_fast(int dtype, const void* a, const void* codes, const void* wscale,
                        const void* wsal, const void* bias, void* y, int M, int N, int Kp,
                        int S_pad, int Gw, int ngw, int n_bits, hipStream_t s) {
  const int v = fq_variant();
  if (v == 5) {
    if (dtype == SQMP_F16)
      return fq6_dispatch<F16>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s);
    if (dtype == SQMP_BF16)
      return fq6_dispatch<BF16>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s);
    return SQMP_EUNSUPPORTED;
  }
  if (dtype == SQMP_F16) {
    if (v == 2 && n_bits == 4 && Gw % 64 == 0)
      return fq5_launch<F16, 1, 1, 6>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s);
    if (v == 3 && n_bits == 4 && Gw % 64 == 0)
      return fq5_launch<F16, 1, 1, 3, 1>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s);
    if (v == 4 && n_bits == 4 && Gw % 64 == 0)
      return fq5_launch<F16, 1, 1, 3, 2>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s);
    return v == 1 ? fq5_dispatch<F16, 2>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s)
                  : fq5_dispatch<F16, 1>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s);
  }
  if (dtype == SQMP_BF16)
    return v == 1 ? fq5_dispatch<BF16, 2>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s)
                  : fq5_dispatch<BF16, 1>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s);
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
