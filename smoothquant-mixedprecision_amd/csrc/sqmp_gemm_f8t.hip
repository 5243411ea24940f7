// gemm_f8t -- the FP8 W4A4 GEMM for per_token / per_tensor activations (fake_quant.py:306 on
// the activation modes with one scale per row, :56-75) with the weight operand in registers.
//
//   y[m][n] = D( sa[m] * sum_g ws[n][g] * (sum_{k in g} ca[m][k] cw[n][k])
//               + sum_j xs[m][j] wsal[n][j] + bias[n] )
//
// Same contraction and numerics as gemm_f8v2 (sqmp_gemm_f8.hip): e4m3 act and weight codes
// (|c| <= 7, exact) on v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales, one
// 128-position block per MFMA inside one weight group (Gw % 128 == 0), the exact integer block
// sum folded by one fp32 FMA per element, the row scales applied before the exact salient
// tail (f16 / bf16 MFMA into the same accumulators).  y is bit-identical to gemm_f8v2's.
//
// What changes (gemm_f8v2 moves both 32-KiB code images of a stage through LDS by LDS-DMA,
// 9 pieces per wave, two 65-KiB slots, one stage in flight):
//   * 8 waves as 1 (m) x 8 (n): wave w owns the 32 weight columns n0 + 32 w .. + 31 over all
//     256 activation rows (16 x 2 tiles of 16 x 16, 128 accumulators).  Its weight codes are
//     private, so they are loaded straight into VGPRs from a tile-major copy of the weight
//     (sqmp_pack_f8t: per 32-column block and 128-position stage, [j][half][lane][16 B], one
//     contiguous KiB per load instruction), one stage ahead in two register sets;
//   * only the activation codes (256 rows x 128 B per stage) move through LDS: 4 LDS-DMA
//     pieces per wave per stage, a 4-slot ring of 32-KiB slots, three stages in flight;
//   * every vector-memory op of the loop is issued from inline asm and waited for by
//     hand-counted s_waitcnt vmcnt(N) (gemm_fq7's discipline: the compiler never sees a
//     pending LDS-DMA; an empty asm "fence" ties each loaded register to its wait).
// The salient tail: 64-position stages, xs through the same ring, wsal tile-major in the same
// register sets ([u][j][lane][16 B] per 32-column block and stage).
#include <stdlib.h>

#include <type_traits>

#include "sqmp_mfma.h"

namespace sqmp {
namespace f8t {

typedef int i32x4b __attribute__((ext_vector_type(4)));
typedef int i32x8b __attribute__((ext_vector_type(8)));

constexpr int IMG = 32768;         // one stage's activation image: 256 rows x 128 B
constexpr int SLOT = IMG + 1024;   // + the stage's 256 fp32 weight scales (code stages)
constexpr int NS = 4, PA = 3;      // ring slots, stages in flight
constexpr int SA_OFF = NS * SLOT;  // the tile's 256 row scales (fp32), DMA'd in the prologue
constexpr int LDS_BYTES = SA_OFF + 1024;

__device__ inline i32x4b rsrc_of(const void* base, uint32_t nrec) {
  const uint64_t a = (uint64_t)(size_t)base;
  i32x4b r;
  r[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = (int)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xFFFFu);
  r[2] = (int)nrec;
  r[3] = 0x00020000;
  return r;
}

// 16 B per lane to LDS (wave-uniform destination + 16 * lane); s_nop 0: the M0 write ->
// LDS-DMA wait state
__device__ inline void dma16(const i32x4b& r, uint32_t voff, uint32_t soff, unsigned char* lds_dst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(
      (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m0v),
               "v"(voff), "s"(r), "s"(soff)
               : "memory", "m0");
}
template <int OFF>
__device__ inline void ld16(u32x4& d, const i32x4b& r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
               : "=v"(d)
               : "v"(voff), "s"(r), "s"(soff), "n"(OFF));
}
template <class V>
__device__ inline void fence(V& v) {
  asm volatile("" : "+v"(v));
}
template <int N>
__device__ inline void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ inline void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// LDS image rows are 128 B; 16-B chunk c of row r at c ^ sw(r): conflict-free for the
// ds_read_b128 lane groups of the e4m3 fragment reads (chunks 2q, 2q + 1) and the D tail
// reads (chunk 4u + q) -- gemm_f8v2's swizzle
__device__ inline int sw(int r) { return ((r >> 1) & 1) ^ (((r >> 2) & 1) << 2) ^ (((r >> 3) & 1) * 6); }
__device__ inline int img_off(int r, int c) { return (r << 7) + ((c ^ sw(r)) << 4); }
__device__ inline i32x8b cat8(const u32x4& a, const u32x4& b) {
  return i32x8b{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}

template <class DT>
__global__ __launch_bounds__(512, 1) void gemm_f8t_kernel(
    const unsigned char* __restrict__ A8, const float* __restrict__ ascale,
    const typename DT::T* __restrict__ XS, const unsigned char* __restrict__ W8t,
    const float* __restrict__ ws32, const typename DT::T* __restrict__ Salt,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n, int group_m,
    uint32_t* __restrict__ colmax) {
  typedef typename DT::T T;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int nk8 = Kp / 128, nks = S_pad / 64, nkt = nk8 + nks;
  const int Np = pad_n(N);
  const int nb = tn * 8 + wave;  // this wave's 32-column weight block
  // fragment chunk offsets inside an image row: sw(16 i + r16) == sw(r16)
  const int oq0 = ((2 * q) ^ sw(r16)) << 4, oq1 = ((2 * q + 1) ^ sw(r16)) << 4;
  const int ot0 = (q ^ sw(r16)) << 4, ot1 = ((4 + q) ^ sw(r16)) << 4;

  // ---- A (act codes, then xs) by LDS-DMA: piece j of wave w = rows 32 w + 8 j + (lane >> 3)
  const int drow0 = 32 * wave + (lane >> 3);
  const i32x4b rA = rsrc_of(A8 + (size_t)m0 * Kp, 0xFFFFFFFFu);
  const i32x4b rX = rsrc_of(XS + (size_t)m0 * (S_pad > 0 ? S_pad : 0), 0xFFFFFFFFu);
  const i32x4b rS = rsrc_of(ws32 + n0, 0xFFFFFFFFu);
  // A pieces this wave issues for stage kt (wave 0 also moves a code stage's weight scales)
  auto na = [&](int kt) __attribute__((always_inline)) {
    return kt >= nkt ? 0 : 4 + (wave == 0 && kt < nk8 ? 1 : 0);
  };
  auto issue_a = [&](int kt) __attribute__((always_inline)) {
    if (kt >= nkt) return;
    unsigned char* slot = lds + (kt % NS) * SLOT;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = drow0 + 8 * j;
      const uint32_t c16 = (uint32_t)(((lane & 7) ^ sw(row)) << 4);
      if (kt < nk8)
        dma16(rA, (uint32_t)row * Kp + c16, (uint32_t)kt * 128, slot + (4 * wave + j) * 1024);
      else
        dma16(rX, (uint32_t)row * S_pad * sizeof(T) + c16, (uint32_t)(kt - nk8) * 128,
              slot + (4 * wave + j) * 1024);
    }
    if (wave == 0 && kt < nk8) {
      const int g = min((kt * 128) / Gw, ngw - 1);
      dma16(rS, (uint32_t)lane * 16, (uint32_t)g * Np * 4, slot + IMG);
    }
  };

  // ---- weight operand straight to registers
  // codes: W8t[nb][kb][j][h][lane][16 B]; tail: Salt[nb][kd][u][j][lane][8 D] (the weight
  // scales of a code stage ride with its activation image: ws32[g][n0 .. n0 + 255])
  const i32x4b rB = rsrc_of(W8t + (size_t)nb * nk8 * 4096, 0xFFFFFFFFu);
  const i32x4b rD = rsrc_of(Salt + (size_t)nb * (nks > 0 ? nks : 1) * 2048, 0xFFFFFFFFu);
  const uint32_t vB = (uint32_t)lane * 16;
  struct Regs {
    u32x4 w[4];  // codes: [j][h]; tail: [u][j]
  };
  auto issue_b = [&](int kt, Regs& d) __attribute__((always_inline)) {
    if (kt >= nkt) return;
    if (kt < nk8) {
      const uint32_t so = (uint32_t)kt * 4096;
      ld16<0>(d.w[0], rB, vB, so);
      ld16<1024>(d.w[1], rB, vB, so);
      ld16<2048>(d.w[2], rB, vB, so);
      ld16<3072>(d.w[3], rB, vB, so);
    } else {
      const uint32_t so = (uint32_t)(kt - nk8) * 4096;
      ld16<0>(d.w[0], rD, vB, so);
      ld16<1024>(d.w[1], rD, vB, so);
      ld16<2048>(d.w[2], rD, vB, so);
      ld16<3072>(d.w[3], rD, vB, so);
    }
  };
  auto fence_b = [&](int kt, Regs& d) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) fence(d.w[u]);
  };

  f32x4 tot[16][2];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  // one code stage: per act tile i two MFMAs (j = 0, 1); the fold of j = 1 issued behind
  // the next tile's first MFMA (its result latency), act fragments read one tile ahead
  auto compute_f8 = [&](const unsigned char* __restrict__ slot, const Regs& d) __attribute__((always_inline)) {
    const i32x8b bw0 = cat8(d.w[0], d.w[1]), bw1 = cat8(d.w[2], d.w[3]);
    const float* sp = (const float*)(slot + IMG) + 32 * wave + 4 * q;  // columns 16 j + 4 q + r
    const f32x4 s0 = *(const f32x4*)sp, s1 = *(const f32x4*)(sp + 16);
    auto ald = [&](int i) __attribute__((always_inline)) {
      const unsigned char* rp = slot + (16 * i + r16) * 128;
      return cat8(*(const u32x4*)(rp + oq0), *(const u32x4*)(rp + oq1));
    };
    i32x8b a[2];
    a[0] = ald(0);
    f32x4 p1 = zero;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i + 1 < 16) a[(i + 1) & 1] = ald(i + 1);
      const f32x4 t0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bw0, a[i & 1], zero, 0, 0, 0, 127, 0, 127);
      if (i > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) tot[i - 1][1][r] = __builtin_fmaf(p1[r], s1[r], tot[i - 1][1][r]);
      }
      p1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bw1, a[i & 1], zero, 0, 0, 0, 127, 0, 127);
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[i][0][r] = __builtin_fmaf(t0[r], s0[r], tot[i][0][r]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) tot[15][1][r] = __builtin_fmaf(p1[r], s1[r], tot[15][1][r]);
  };
  // one salient stage (64 positions, two 32-wide sub-steps u)
  auto compute_tail = [&](const unsigned char* __restrict__ slot, const Regs& d) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const u32x4 af = *(const u32x4*)(slot + (16 * i + r16) * 128 + (u ? ot1 : ot0));
        Mfma<DT>::run(tot[i][0], d.w[2 * u], af);
        Mfma<DT>::run(tot[i][1], d.w[2 * u + 1], af);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto apply_row_scales = [&]() __attribute__((always_inline)) {
    const float* rs = (const float*)(lds + SA_OFF);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float sv = rs[16 * i + r16];
      tot[i][0] *= sv;
      tot[i][1] *= sv;
    }
  };

  // ---- prologue: the row scales (wave 0, oldest op), A(0), B(0), A(1 .. PA-1)
  if (wave == 0) {
    const i32x4b rR = rsrc_of(ascale + m0, (uint32_t)(M - m0) * 4u);  // rows >= M read 0
    dma16(rR, (uint32_t)lane * 16, 0u, lds + SA_OFF);
  }
  Regs rg[2];
  issue_a(0);
  issue_b(0, rg[0]);
#pragma unroll
  for (int p = 1; p < PA; ++p) issue_a(p);

  // stage kt on register set P: at its top, the ops younger than B(kt) are A(kt + PA - 1)
  // (na pieces, or none past the last stage; at kt = 0 the prologue's A(1 .. PA - 1)).  One
  // loop per compute body (code stages, then the salient tail), each unrolled by two for
  // compile-time register sets: no branch between bodies inside a loop, so the accumulators
  // keep their registers (gemm_f8v2's rule)
  auto top = [&](int kt, Regs& d) __attribute__((always_inline)) {
    const int younger = kt == 0 ? na(1) + na(2) : na(kt - 1 + PA);
    switch (younger) {
      case 10: vmwait<10>(); break;
      case 9: vmwait<9>(); break;
      case 8: vmwait<8>(); break;
      case 5: vmwait<5>(); break;
      case 4: vmwait<4>(); break;
      default: vmwait<0>(); break;
    }
    fence_b(kt, d);
    barrier();  // every wave's pieces of stage kt landed; every wave is past slot kt - 1
  };
  auto code_step = [&](int kt, auto pc) __attribute__((always_inline)) {
    constexpr int P = decltype(pc)::value;
    top(kt, rg[P]);
    issue_b(kt + 1, rg[P ^ 1]);
    issue_a(kt + PA);
    compute_f8(lds + (kt % NS) * SLOT, rg[P]);
  };
  auto tail_step = [&](int kt, auto pc) __attribute__((always_inline)) {
    constexpr int P = decltype(pc)::value;
    top(kt, rg[P]);
    issue_b(kt + 1, rg[P ^ 1]);
    issue_a(kt + PA);
    if (kt == nk8) apply_row_scales();
    compute_tail(lds + (kt % NS) * SLOT, rg[P]);
  };
  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;
  int kt = 0;
  for (; kt + 1 < nk8; kt += 2) {
    code_step(kt, Z());
    code_step(kt + 1, O());
  }
  if (kt < nk8) {
    code_step(kt, Z());
    ++kt;
  }
  // the tail's first stage uses register set nk8 & 1
  auto tail_loop = [&](auto first) __attribute__((always_inline)) {
    using F = decltype(first);
    using G = std::integral_constant<int, F::value ^ 1>;
    int k = nk8;
    for (; k + 1 < nkt; k += 2) {
      tail_step(k, F());
      tail_step(k + 1, G());
    }
    if (k < nkt) tail_step(k, F());
  };
  if (nks > 0) {
    if (nk8 & 1)
      tail_loop(O());
    else
      tail_loop(Z());
  } else {
    barrier();
    apply_row_scales();
  }

  // ---- fused output-quant statistics (sqmp_gemm_f8t with colmax): per output column the
  // max of |D(y)| over the lane's rows, the 16 r16 lanes, one atomic per column and wave
  if (colmax) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nl = 32 * wave + 16 * j + 4 * q;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float bv = (bias && n0 + nl + r < N) ? DT::to_f(bias[n0 + nl + r]) : 0.f;
        float c = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (m0 + 16 * i + r16 < M) c = fmaxf(c, fabsf(DT::to_f(DT::from_f(tot[i][j][r] + bv))));
        c = fmaxf(c, __shfl_xor(c, 1, 64));
        c = fmaxf(c, __shfl_xor(c, 2, 64));
        c = fmaxf(c, __shfl_xor(c, 4, 64));
        c = fmaxf(c, __shfl_xor(c, 8, 64));
        if (r16 == 0 && n0 + nl + r < N) atomicMax(colmax + n0 + nl + r, __float_as_uint(c));
      }
    }
  }

  // ---- epilogue: the 256 x 256 tile staged in LDS (row m: 512 B, 16-B chunk c at c ^ (m &
  // 31)), each row stored as one 512-B run (32 lanes x 16 B) -- gemm_f8v2's
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  barrier();  // every wave is past its last fragment read of the ring
  if (n0 + 256 <= N) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nl = 32 * wave + 16 * j + 4 * q;
      float bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = bias ? DT::to_f(bias[n0 + nl + r]) : 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ml = 16 * i + r16;
        T v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = DT::from_f(tot[i][j][r] + bv[r]);
        *(uint2*)(lds + ml * 512 + (((nl >> 3) ^ (ml & 31)) << 4) + (nl & 4) * 2) = *(const uint2*)v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
    const int c = tid & 31;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int ml = 16 * k + (tid >> 5);
      const u32x4 val = *(const u32x4*)(lds + ml * 512 + ((c ^ (ml & 31)) << 4));
      if (m0 + ml < M) *(u32x4*)(Y + (size_t)(m0 + ml) * N + n0 + c * 8) = val;
    }
    return;
  }
  // partial column tile: per lane, 8-byte stores of 4 consecutive columns (N % 8 == 0)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int gn = n0 + 32 * wave + 16 * j + 4 * q;
    if (gn >= N) continue;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = bias ? DT::to_f(bias[gn + r]) : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int gm = m0 + 16 * i + r16;
      if (gm >= M) continue;
      T v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = DT::from_f(tot[i][j][r] + bv[r]);
      *(uint2*)(Y + (size_t)gm * N + gn) = *(const uint2*)v;
    }
  }
}

// ---- tile-major weight copies (once per layer)
// W8t[nb][kb][j][h][lane][16 B] = w8[32 nb + 16 j + r16][128 kb + 32 q + 16 h .. + 16]
__global__ void pack_codes_t_kernel(const u32x4* __restrict__ w8, u32x4* __restrict__ w8t, int Np,
                                    int Kp, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int lane = (int)(idx & 63), h = (int)((idx >> 6) & 1), j = (int)((idx >> 7) & 1);
  const long rest = idx >> 8;
  const int KB = Kp / 128;
  const int kb = (int)(rest % KB);
  const long nb = rest / KB;
  const int q = lane >> 4, r16 = lane & 15;
  const long n = nb * 32 + 16 * j + r16;
  w8t[idx] = n < Np ? w8[(n * Kp + 128L * kb + 32 * q + 16 * h) / 16] : u32x4{0u, 0u, 0u, 0u};
}
// Salt[nb][kd][u][j][lane][8 D] = wsal[32 nb + 16 j + r16][64 kd + 32 u + 8 q .. + 8]
__global__ void pack_sal_t_kernel(const u32x4* __restrict__ wsal, u32x4* __restrict__ salt, int N,
                                  int S_pad, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int lane = (int)(idx & 63), j = (int)((idx >> 6) & 1), u = (int)((idx >> 7) & 1);
  const long rest = idx >> 8;
  const int KS = S_pad / 64;
  const int kd = (int)(rest % KS);
  const long nb = rest / KS;
  const int q = lane >> 4, r16 = lane & 15;
  const long n = nb * 32 + 16 * j + r16;
  salt[idx] = n < N ? wsal[(n * S_pad + 64L * kd + 32 * u + 8 * q) / 8] : u32x4{0u, 0u, 0u, 0u};
}

}  // namespace f8t

extern "C" int sqmp_pack_f8t(const void* w8, const void* wsal, int dtype, int N, int Kp, int S_pad,
                             void* w8t, void* salt, void* stream) {
  if (!w8 || !w8t || N <= 0 || Kp <= 0 || Kp % 128 || S_pad < 0 || S_pad % 64) return SQMP_EINVAL;
  if (S_pad > 0 && (!wsal || !salt)) return SQMP_EINVAL;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int Np = pad_n(N);
  const long tc = (long)Np * Kp / 16;
  f8t::pack_codes_t_kernel<<<dim3((unsigned)cdiv(tc, 256)), dim3(256), 0, s>>>(
      (const u32x4*)w8, (u32x4*)w8t, Np, Kp, tc);
  SQMP_LAUNCH_CHECK();
  if (S_pad > 0) {
    const long ts = (long)Np * S_pad / 8;
    f8t::pack_sal_t_kernel<<<dim3((unsigned)cdiv(ts, 256)), dim3(256), 0, s>>>(
        (const u32x4*)wsal, (u32x4*)salt, N, S_pad, ts);
    SQMP_LAUNCH_CHECK();
  }
  return SQMP_OK;
}

extern "C" int sqmp_gemm_f8t(const void* a8, const float* ascale, const void* xs, const void* w8t,
                             const float* ws32, const void* salt, const void* bias, void* y,
                             int dtype, int M, int N, int Kp, int S_pad, int Gw, int ngw,
                             uint32_t* colmax, void* stream) {
  if (M < 0 || N <= 0 || Kp <= 0 || Kp % 128 != 0 || S_pad < 0 || S_pad % 64 != 0)
    return SQMP_EINVAL;
  if (!a8 || !ascale || !w8t || !ws32 || !y || (S_pad > 0 && (!xs || !salt))) return SQMP_EINVAL;
  if (Gw <= 0 || Gw % 128 != 0 || ngw <= 0) return SQMP_EUNSUPPORTED;
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return SQMP_EUNSUPPORTED;
  if (N % 8) return SQMP_EUNSUPPORTED;  // 8-byte / 16-byte output stores
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
  const int tiles_m = cdiv(M, 256), tiles_n = cdiv(N, 256);
  static const int group_m = [] {
    const char* e = getenv("SQMP_GROUP_M");
    return e && atoi(e) > 0 ? atoi(e) : 4;
  }();
  const dim3 grid(tiles_m * tiles_n), block(512);
  if (dtype == SQMP_F16)
    f8t::gemm_f8t_kernel<F16><<<grid, block, 0, s>>>(
        (const unsigned char*)a8, ascale, (const F16::T*)xs, (const unsigned char*)w8t, ws32,
        (const F16::T*)salt, (const F16::T*)bias, (F16::T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m,
        tiles_n, group_m, colmax);
  else
    f8t::gemm_f8t_kernel<BF16><<<grid, block, 0, s>>>(
        (const unsigned char*)a8, ascale, (const BF16::T*)xs, (const unsigned char*)w8t, ws32,
        (const BF16::T*)salt, (const BF16::T*)bias, (BF16::T*)y, M, N, Kp, S_pad, Gw, ngw,
        tiles_m, tiles_n, group_m, colmax);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace sqmp
