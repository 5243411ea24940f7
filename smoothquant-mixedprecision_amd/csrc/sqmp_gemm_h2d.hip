// fp32 W4A4 GEMM (the F.linear of fake_quant.py:306 for fp32 models; OPT runs in fp32 in the
// reference, run_experiments.py:146-156) on the two-piece fp16 form of sqmp_gemm_h2, with
// the activation planes moved by LDS-DMA through a 4-slot ring and the weight planes held in
// registers (the structure of gemm_fq7's salient tail, applied to the whole K range).
//
//   y[m][n] = 2^-(ea[m] + eb[n]) sum_k (al.bh + ah.bl + ah.bh)[m][n][k] + bias[n]
//
// where a' = 2^ea[m] a and b' = 2^eb[n] b are row-scaled so that each row's maximum lies in
// [2^13, 2^14), a' = ah + al and b' = bh + bl with ah = f16(a'), al = f16(a' - ah) (exact
// fp16 splits: |a' - ah - al| <= 2^-22 |a'|), every product exact in the fp32 accumulator of
// v_mfma_f32_16x16x32_f16 -- the numerics of sqmp_gemm_h2 (sqmp_gemm_x3.hip), with the same
// k order within each 32-position MFMA and the same term order per accumulator, so the two
// kernels agree bit for bit.
//
// Why a second kernel: gemm_x3_kernel<H> stages both operands through registers into a
// single-buffered LDS tile with two barriers per 64-position stage, and splits A while
// staging (1.8 ms at config 2 in fp32, MFMA busy 44 %, 5.1x its algorithmic HBM bytes).  Here
//   * the activation planes [2][Mp][L] come pre-split -- written by the fp32 quantizer itself
//     (sqmp_quant_act_v2 SQMP_OUT_H2) or by sqmp_split2_f16 -- and move by LDS-DMA:
//     TM = 128 rows x 64 positions x 2 planes = 32 KiB per stage, 4 slots, 3 stages in flight,
//     all pieces issued by waves 0-3 (the loader split of gemm_fq6/fq7);
//   * the weight planes live in a tile-major copy (sqmp_pack_h2d, once per layer) from which a
//     lane loads exactly its fragments, 8 x 16 B per stage, one stage ahead, into registers;
//   * tile 128 tokens x 256 weight rows, 8 waves each 128 x 32 (8 x 2 tiles of 16 x 16), 96
//     MFMAs per wave per stage against 4 fragment reads per 6 MFMAs.
// Fragment geometry: sub-step s of a stage covers positions 32 s .. 32 s + 31; lane (r16, q)
// holds positions 32 s + 8 q .. + 7 of its row.  The weight fragment goes in the MFMA's A
// slot, so acc[i][j][r] = C[n = n0 + 32 wave + 16 j + 4 q + r][m = m0 + 16 i + r16].
#include <stdlib.h>

#include "sqmp_mfma.h"

namespace sqmp {
namespace h2d {

typedef int rsrc_t __attribute__((ext_vector_type(4)));

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
__device__ inline void vmwait_dyn(int n) {
  switch (n) {
    case 8: vmwait<8>(); break;
    case 16: vmwait<16>(); break;
    default: vmwait<0>(); break;
  }
}
__device__ inline void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// LDS-DMA of 16 B per lane to the wave-uniform LDS address + 16 * lane (s_nop 0: the M0
// write -> LDS-DMA wait state)
__device__ inline void dma16(const rsrc_t& r, uint32_t voff, uint32_t soff, uint32_t lds_addr) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m0v),
               "v"(voff), "s"(r), "s"(soff)
               : "memory", "m0");
}
template <int OFF>
__device__ inline void ld16(u32x4& d, const rsrc_t& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
               : "=v"(d)
               : "v"(voff), "s"(r), "s"(soff), "n"(OFF));
}
template <class V>
__device__ inline void fence(V& v) {
  asm volatile("" : "+v"(v));
}

// TM = 128 token rows per tile, or 64 where 128-row tiles leave CUs idle (OPT-1.3B's N = 2048
// layers at 2048 tokens: 128 tiles of 128 x 256, 256 of 64 x 256)
constexpr int TN = 256, J = 2, WR = 16 * J;
constexpr int PA = 3, NS = PA + 1;     // A stages in flight, ring slots
constexpr int PF = 2;                  // A fragment read-ahead (blocks)

// 128-B LDS rows: 16-B chunk c of row r at c ^ (r & 7) (conflict-free for the ds_read_b128
// lane groups, as gemm_x3's K-64 layout)
__device__ inline uint32_t a_off(int row, int chunk) {
  return (uint32_t)(row * 128 + ((chunk ^ (row & 7)) << 4));
}

// W registers of one stage: [plane][j][s]
struct Wreg {
  u32x4 w[2][J][2];
};

template <bool COLMAX, int TM>
__global__ __launch_bounds__(512, 1) void gemm_h2d_kernel(
    const uint16_t* __restrict__ A2, size_t a_plane, const int* __restrict__ aexp,
    const uint16_t* __restrict__ Wt, const int* __restrict__ bexp, const float* __restrict__ bias,
    float* __restrict__ Y, int M, int N, int L, int tiles_m, int tiles_n, int group_m,
    uint32_t* __restrict__ colmax, int nt) {
  constexpr int I = TM / 16;
  constexpr int PLANE = TM * 128;   // one activation plane of a stage: TM rows x 128 B
  constexpr int SLOT = 2 * PLANE;   // 32 KiB at TM = 128
  constexpr int NA = TM / 64;       // DMA pieces per wave per plane and stage
  constexpr int EPI = TM * TN * 4;  // fp32 output tile staged in LDS: 128 KiB at TM = 128
  constexpr int LDS_BYTES = NS * SLOT > EPI ? NS * SLOT : EPI;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  const uint32_t lds32 = (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)lds;

  int tm, tn;
  tile_coords(tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int nkt = L / 64;
  const int nb = tn * 8 + wave;  // this wave's 32-row weight block

  // ---- A planes by LDS-DMA (waves 0-3 issue every piece): piece i of virtual wave w and
  // plane p = rows 64 i + 8 w + (lane >> 3); the lane moves logical chunk (lane & 7) ^ (row
  // & 7) into physical chunk lane & 7
  const rsrc_t rA = make_rsrc(A2 + (size_t)m0 * L);
  uint32_t av[2][NA];  // [o][i]: per-lane offsets of virtual wave wave + 4 o
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = 64 * i + 8 * (wave + 4 * o) + (lane >> 3);
      av[o][i] = (uint32_t)row * (uint32_t)L * 2u + (uint32_t)(((lane & 7) ^ (row & 7)) << 4);
    }
  const int na_w = wave < 4 ? 2 * 2 * NA : 0;  // DMA ops of one stage issued by this wave
  const uint32_t pl_bytes = (uint32_t)(a_plane * 2);
  auto issue_a = [&](int kt) {
    if (kt < nkt && wave < 4) {
      const uint32_t slot = lds32 + (uint32_t)((kt % NS) * SLOT);
      const uint32_t so = (uint32_t)kt * 128u;
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int o = 0; o < 2; ++o)
#pragma unroll
          for (int i = 0; i < NA; ++i)
            dma16(rA, av[o][i], so + (p ? pl_bytes : 0u),
                  slot + (uint32_t)(p * PLANE + (i * 8 + wave + 4 * o) * 1024));
    }
  };

  // ---- W planes straight to registers from Wt[p][nb][kt][lane][j][s][8]
  const size_t wplane = (size_t)tiles_n * 8 * nkt * 64 * J * 2 * 8;  // halves per plane
  const rsrc_t rW = make_rsrc(Wt + (size_t)nb * nkt * (64 * J * 2 * 8));
  const uint32_t vW = (uint32_t)lane * (J * 2 * 16);  // 64 B per lane and stage
  const uint32_t wpl = (uint32_t)(wplane * 2);
  auto issue_w = [&](int kt, Wreg& d) {
    const uint32_t so = (uint32_t)kt * (64u * J * 2 * 16);
    ld16<0>(d.w[0][0][0], rW, vW, so);
    ld16<16>(d.w[0][0][1], rW, vW, so);
    ld16<32>(d.w[0][1][0], rW, vW, so);
    ld16<48>(d.w[0][1][1], rW, vW, so);
    ld16<0>(d.w[1][0][0], rW, vW, so + wpl);
    ld16<16>(d.w[1][0][1], rW, vW, so + wpl);
    ld16<32>(d.w[1][1][0], rW, vW, so + wpl);
    ld16<48>(d.w[1][1][1], rW, vW, so + wpl);
  };
  auto fence_w = [&](Wreg& d) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) fence(d.w[p][j][s]);
  };

  f32x4 acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // block t = 16-row tile t % I of sub-step t / I: its two plane fragments
  struct Af {
    u32x4 h, l;
  };
  auto ald = [&](const unsigned char* __restrict__ slot, int t) {
    const uint32_t o = a_off(16 * (t % I) + r16, 4 * (t / I) + q);
    return Af{*(const u32x4*)(slot + o), *(const u32x4*)(slot + PLANE + o)};
  };
  auto compute = [&](const unsigned char* __restrict__ slot, const Wreg& w) {
    Af a[PF + 1];
#pragma unroll
    for (int t = 0; t < PF; ++t) a[t] = ald(slot, t);
#pragma unroll
    for (int t = 0; t < 2 * I; ++t) {
      if (t + PF < 2 * I) a[(t + PF) % (PF + 1)] = ald(slot, t + PF);
      const Af& f = a[t % (PF + 1)];
      const int s = t / I, i = t % I;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        // smallest terms first, the order of gemm_x3_kernel<H>
        Mfma<F16>::run(acc[i][j], w.w[0][j][s], f.l);
        Mfma<F16>::run(acc[i][j], w.w[1][j][s], f.h);
        Mfma<F16>::run(acc[i][j], w.w[0][j][s], f.h);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- K loop: stage kt computes on W set kt & 1 while stage kt + 1's W loads land in the
  // other set (unrolled by two: compile-time set indices, no register copies)
  Wreg ws[2];
  issue_a(0);
  issue_w(0, ws[0]);
#pragma unroll
  for (int p = 1; p < PA; ++p) issue_a(p);
  // ops issued after W(kt) when stage kt starts: A(kt - 1 + PA) (or, at kt = 0, A(1 .. PA-1))
  auto step = [&](int kt, auto pc) {
    constexpr int P = decltype(pc)::value;
    const int n = kt == 0 ? na_w * min(PA - 1, nkt - 1) : (kt - 1 + PA < nkt ? na_w : 0);
    vmwait_dyn(n);
    fence_w(ws[P]);
    barrier();  // every wave's pieces of stage kt landed; every wave is past stage kt - 1
    if (kt + 1 < nkt) issue_w(kt + 1, ws[P ^ 1]);
    issue_a(kt + PA);
    compute(lds + (kt % NS) * SLOT, ws[P]);
  };
  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  int kt = 0;
  for (; kt + 1 < nkt; kt += 2) {
    step(kt, Z());
    step(kt + 1, O());
  }
  if (kt < nkt) step(kt, Z());
  if (wave >= 4) __builtin_amdgcn_s_setprio(0);

  // ---- epilogue: scales undone, bias, staged in LDS as fp32 rows (row m: 1 KiB, 16-B chunk
  // c at c ^ (m & 15)), stored as whole 1-KiB rows
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  barrier();  // every wave is past its last read of the ring
  float cmx[J][4] = {};
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int nl = WR * wave + 16 * j + 4 * q;  // first of the lane's 4 columns
    float bv[4];
    int be[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + nl + r;
      bv[r] = bias && n < N ? bias[n] : 0.f;
      be[r] = bexp[n];  // [Np]
    }
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int ml = 16 * i + r16;
      const int ae = aexp[min(m0 + ml, M - 1)];
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = __builtin_ldexpf(acc[i][j][r], -(ae + be[r])) + bv[r];
      if (COLMAX && m0 + ml < M) {
#pragma unroll
        for (int r = 0; r < 4; ++r) cmx[j][r] = fmaxf(cmx[j][r], fabsf(v[r]));
      }
      const int c = nl >> 2;
      *(f32x4*)(lds + ml * (TN * 4) + ((c ^ (ml & 15)) << 4)) = v;
    }
  }
  if (COLMAX) {
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = cmx[j][r];
        v = fmaxf(v, __shfl_xor(v, 1, 64));
        v = fmaxf(v, __shfl_xor(v, 2, 64));
        v = fmaxf(v, __shfl_xor(v, 4, 64));
        v = fmaxf(v, __shfl_xor(v, 8, 64));
        const int n = n0 + WR * wave + 16 * j + 4 * q + r;
        if (r16 == 0 && n < N) atomicMax(colmax + n, __float_as_uint(v));
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  barrier();
  constexpr int CPR = TN / 4, RPP = 512 / CPR;  // 16-B chunks per row, rows per pass
  const int c = tid % CPR;
  const bool cok = n0 + c * 4 < N;  // N % 4 == 0 (launcher)
#pragma unroll 4
  for (int k = 0; k < TM / RPP; ++k) {
    const int ml = RPP * k + tid / CPR;
    const int gm = m0 + ml;
    const u32x4 val = *(const u32x4*)(lds + ml * (TN * 4) + ((c ^ (ml & 15)) << 4));
    if (gm < M && cok) {
      u32x4* dst = (u32x4*)(Y + (size_t)gm * N + n0 + c * 4);
      if (nt)  // streaming stores of a large output (nt_output)
        store16_nt(dst, val);
      else
        *dst = val;
    }
  }
}

// Wt[p][nb][kt][lane][j][s][e] = planes[p][32 nb + 16 j + r16][64 kt + 32 s + 8 q + e]
__global__ __launch_bounds__(256) void pack_h2d_kernel(const uint16_t* __restrict__ planes, int Np,
                                                       int L, uint16_t* __restrict__ Wt) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;  // one 16-B chunk (8 halves)
  const long per_plane = (long)Np * L / 8;
  if (idx >= 2 * per_plane) return;
  const int p = (int)(idx / per_plane);
  long r = idx % per_plane;
  const int s = (int)(r & 1), j = (int)((r >> 1) & 1), lane = (int)((r >> 2) & 63);
  r >>= 8;
  const int nkt = L / 64;
  const int kt = (int)(r % nkt);
  const long nbk = r / nkt;
  const int q = lane >> 4, r16 = lane & 15;
  const long n = nbk * 32 + 16 * j + r16;
  const u32x4 v = *(const u32x4*)(planes + ((size_t)p * Np + n) * L + 64 * kt + 32 * s + 8 * q);
  *(u32x4*)(Wt + (size_t)idx * 8) = v;
}

}  // namespace h2d
}  // namespace sqmp

using namespace sqmp;

extern "C" int sqmp_pack_h2d(const void* planes, int Np, int L, void* wt, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!planes || !wt || Np <= 0 || Np % 256 != 0 || L <= 0 || L % 64 != 0) return SQMP_EINVAL;
  const long chunks = 2L * Np * L / 8;
  h2d::pack_h2d_kernel<<<cdiv(chunks, 256), 256, 0, (hipStream_t)stream>>>(
      (const uint16_t*)planes, Np, L, (uint16_t*)wt);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

extern "C" int sqmp_gemm_h2d(const void* a2, int ldr, const int* aexp, const void* wt,
                             const int* bexp, const float* bias, float* y, int M, int N, int L,
                             uint32_t* colmax, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!a2 || !aexp || !wt || !bexp || !y || M < 0 || N <= 0 || L <= 0) return SQMP_EINVAL;
  if (L % 64 != 0 || N % 4 != 0 || ldr < 128 * cdiv(M, 128)) return SQMP_EINVAL;
  if (M == 0) return SQMP_OK;
  const int tiles_n = cdiv(N, h2d::TN);
  const int tm = (long)cdiv(M, 128) * tiles_n >= 256 ? 128 : 64;
  const int tiles_m = cdiv(M, tm);
  const int nt = nt_output((size_t)M * N * sizeof(float)) ? 1 : 0;
  const char* ge = knob("SQMP_H2D_GROUP_M");  // A/B knob (sqmp_knobs.hip)
  const int gm = ge && atoi(ge) > 0 ? atoi(ge) : 4;
  const size_t a_plane = (size_t)ldr * L;
  // (32-bit buffer offsets: both planes of the tile rows within 4 GiB)
  if ((size_t)2 * a_plane * 2 >= (1ull << 32)) return SQMP_EINVAL;
  // ... and the weight planes (sqmp_pack_h2d: 2 planes of roundup(N, 256) rows x L halves)
  if ((size_t)4 * (size_t)round_up(N, 256) * (size_t)L >= (1ull << 32)) return SQMP_EUNSUPPORTED;
#define SQMP_H2D(CM)                                                                            \
  if (tm == 128) SQMP_H2D_TM(CM, 128); else SQMP_H2D_TM(CM, 64)
#define SQMP_H2D_TM(CM, TMV)                                                                    \
  h2d::gemm_h2d_kernel<CM, TMV><<<dim3(tiles_m * tiles_n), dim3(512), 0, (hipStream_t)stream>>>(      \
      (const uint16_t*)a2, a_plane, aexp, (const uint16_t*)wt, bexp, bias, y, M, N, L, tiles_m, \
      tiles_n, gm, colmax, nt)
  if (colmax) {
    SQMP_H2D(true);
  } else {
    SQMP_H2D(false);
  }
#undef SQMP_H2D
#undef SQMP_H2D_TM
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}
