// fp32 W4A4 GEMM on the bf16 MFMA (sqmp_gemm_x3): the F.linear of fake_quant.py:306 for
// fp32 models (OPT runs in fp32 in the reference, run_experiments.py:146-156).
//
// Every fp32 value v is split exactly into three bf16 pieces v = h + m + l (h = bf16(v),
// m = bf16(v - h), l = v - h - m; bf16 has the exponent range of fp32 and 8-bit
// significands, so the third residual is representable).  A product a.b is then the sum
// of the nine piece products, each exact in fp32; the three of order 2^-24 and below
// (m.l, l.m, l.l) are dropped, so
//     acc += ah.bh + ah.bm + am.bh + ah.bl + al.bh + am.bm
// on v_mfma_f32_16x16x32_bf16 (fp32 accumulation): a relative error per product of a few
// units of 2^-24 -- the rounding an fp32 FMA makes -- at 6/16 of the f32-MFMA cost (the
// f32 MFMA runs at 1/16 of the bf16 rate on gfx950, MI355X_MICROARCH.md).
//
// A: x_hat in packed K order + the exact salient columns, fp32 [>= 128-row pad][L], split
//    in registers while it is staged into LDS (one HBM/L2 read of 4 B per element).
// B: the packed-order W_hat + salient slice, split once per layer (sqmp_split3_bf16) into
//    three bf16 planes [3][Np][L].
// Tile 128 x 128, K stage 32, 4 waves (2 x 2, 64 x 64 each, 16 x 16 output tiles),
// 96 MFMAs per wave per stage; single-buffered LDS (48 KiB) with the next stage's global
// loads in flight over the MFMAs, two workgroups per CU (8 waves of 64 x 32 in one
// workgroup when the grid has fewer than two tiles per CU).
#include <stdlib.h>

#include "sqmp_mfma.h"

namespace sqmp {

namespace {

constexpr int X3_BM = 128, X3_BN = 128, X3_BK = 32;
constexpr int X3_PLANE = X3_BM * X3_BK * 2;  // one bf16 plane of a 128-row tile: 8 KiB

// 64-B rows (four 16-B chunks).  ds_read_b128 serves lanes in groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): lane (r16, q) reads chunk q of row r16; the
// physical chunk q ^ H[(row >> 2) & 3] with H = {0, 2, 3, 1} puts the 16 lanes of every
// group on 16 distinct (row & 3, chunk) bank quarters -- conflict-free.
__device__ inline int x3_off(int row, int chunk) {
  const int h = (0x1320 >> (4 * ((row >> 2) & 3))) & 3;  // H = {0, 2, 3, 1}

  return row * 64 + ((chunk ^ h) << 4);
}

// 128-B rows (K stage 64): chunk c of row r at c ^ (r & 7) -- conflict-free for the same
// lane groups (fragment chunk 4 s + q of sub-step s)
template <int BK>
__device__ inline int xk_off(int row, int chunk) {
  if (BK == 64) return row * 128 + ((chunk ^ (row & 7)) << 4);
  return x3_off(row, chunk);
}

__device__ inline uint32_t bf16_bits(float v) {
  const __bf16 b = (__bf16)v;  // RNE
  return (uint32_t)(*(const uint16_t*)&b);
}
__device__ inline float bf16_val(uint32_t bits) { return __uint_as_float(bits << 16); }

// v -> (h, m, l) bf16 bit patterns with v == h + m + l exactly
__device__ inline void split3(float v, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = bf16_bits(v);
  const float r = v - bf16_val(h);  // exact
  m = bf16_bits(r);
  l = bf16_bits(r - bf16_val(m));   // exact, and exact in bf16
}

// WN = waves along N: 2 -> 4 waves of 64 x 64 (two workgroups per CU), 4 -> 8 waves of
// 64 x 32 (grids of fewer than two tiles per CU: two waves per SIMD from one workgroup)
// H: the two-piece fp16 form (see sqmp_gemm_h2 below): A rows and B rows scaled by 2^aexp[m]
// / 2^bexp[n] into [2^13, 2^14) at their maximum, v' = h + l with h = f16(v'),
// l = f16(v' - h), three products (al.bh + ah.bl + ah.bh) on v_mfma_f32_16x16x32_f16, the
// scales undone in the epilogue.
template <bool COLMAX, int WN, bool H = false, int BN = 128, int BK = 32>
__global__ __launch_bounds__(128 * WN, 4 / WN) void gemm_x3_kernel(
    const float* __restrict__ A, const uint16_t* __restrict__ B3, const float* __restrict__ bias,
    float* __restrict__ Y, int M, int N, int L, int Np, int tiles_m, int tiles_n,
    uint32_t* __restrict__ colmax, const int* __restrict__ aexp, const int* __restrict__ bexp,
    int nt, int group_m) {
  constexpr int NPL = H ? 2 : 3;  // pieces per operand
  // A planes (NPL x 128 rows) then B planes (NPL x BN rows), rows of BK 16-bit values
  constexpr int APL = X3_BM * BK * 2;  // one A plane
  constexpr int BPL = APL * BN / X3_BM;  // one B plane
  constexpr int CPR = BK / 8;          // 16-B chunks per 16-bit row
  constexpr int CSH = BK == 64 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) unsigned char lds[NPL * (APL + BPL)];
  unsigned char* const ldsb = lds + NPL * APL;
  int tm, tn;
  tile_coords(tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * X3_BM, n0 = tn * BN;
  constexpr int NT = 128 * WN, CW = BN / WN, J = CW / 16;
  constexpr int BSH = (BN == 256 ? 8 : 7) + CSH;  // log2(16-B chunks per B plane)
  constexpr int LA = 2 * CPR * X3_BM / NT, LB = CPR * BN * NPL / NT;  // 16-B staging chunks per thread
  constexpr int ASH = CSH + 1;  // log2(16-B fp32 chunks per A row)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r16 = lane & 15, q = lane >> 4;
  const int nkt = L / BK;
  const size_t plane = (size_t)Np * L;

  // staging: A 128 rows x 8 chunks of 4 fp32; B NPL planes x 128 rows x 4 chunks of 8 x 16 bit
  u32x4 ra[LA], rb[LB];
  int ae[LA];  // H: the row exponents of this thread's A chunks (fixed over the K loop)
  if (H) {
#pragma unroll
    for (int i = 0; i < LA; ++i) ae[i] = aexp[min(m0 + ((tid + NT * i) >> ASH), M - 1)];
  }
  auto load = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + NT * i, row = idx >> ASH, c = idx & (2 * CPR - 1);
      ra[i] = *(const u32x4*)(A + (size_t)(m0 + row) * L + k0 + 4 * c);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + NT * i, p = idx >> BSH, row = (idx >> CSH) & (BN - 1), c = idx & (CPR - 1);
      rb[i] = *(const u32x4*)(B3 + p * plane + (size_t)(n0 + row) * L + k0 + 8 * c);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + NT * i, row = idx >> ASH, c = idx & (2 * CPR - 1);
      const int off = xk_off<BK>(row, c >> 1) + (c & 1) * 8;
      if (H) {
        uint32_t h[4], l[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) split2h(__builtin_ldexpf(__uint_as_float(ra[i][e]), ae[i]), h[e], l[e]);
        *(uint2*)(lds + off) = uint2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
        *(uint2*)(lds + APL + off) = uint2{l[0] | (l[1] << 16), l[2] | (l[3] << 16)};
      } else {
        uint32_t h[4], m[4], l[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) split3(__uint_as_float(ra[i][e]), h[e], m[e], l[e]);
        *(uint2*)(lds + off) = uint2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
        *(uint2*)(lds + APL + off) = uint2{m[0] | (m[1] << 16), m[2] | (m[3] << 16)};
        *(uint2*)(lds + 2 * APL + off) = uint2{l[0] | (l[1] << 16), l[2] | (l[3] << 16)};
      }
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + NT * i, p = idx >> BSH, row = (idx >> CSH) & (BN - 1), c = idx & (CPR - 1);
      *(u32x4*)(ldsb + p * BPL + xk_off<BK>(row, c)) = rb[i];
    }
  };

  f32x4 acc[4][J];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&]() {
#pragma unroll
   for (int sst = 0; sst < BK / 32; ++sst) {
    // B fragments (output columns) in the MFMA's A slot: the lane's 4 results are 4
    // consecutive columns of one row (16-B stores)
    u32x4 bf[NPL][J];
#pragma unroll
    for (int p = 0; p < NPL; ++p)
#pragma unroll
      for (int j = 0; j < J; ++j)
        bf[p][j] = *(const u32x4*)(ldsb + p * BPL + xk_off<BK>(wn * CW + 16 * j + r16, 4 * sst + q));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      u32x4 af[NPL];
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        af[p] = *(const u32x4*)(lds + p * APL + xk_off<BK>(wm * 64 + 16 * i + r16, 4 * sst + q));
#pragma unroll
      for (int j = 0; j < J; ++j) {
        // smallest terms first (one accumulator per chain: measured faster than term-major
        // order over the accumulators)
        if (H) {
          Mfma<F16>::run(acc[i][j], bf[0][j], af[1]);
          Mfma<F16>::run(acc[i][j], bf[1][j], af[0]);
          Mfma<F16>::run(acc[i][j], bf[0][j], af[0]);
        } else {
          Mfma<BF16>::run(acc[i][j], bf[1][j], af[1]);
          Mfma<BF16>::run(acc[i][j], bf[2][j], af[0]);
          Mfma<BF16>::run(acc[i][j], bf[0][j], af[2]);
          Mfma<BF16>::run(acc[i][j], bf[1][j], af[0]);
          Mfma<BF16>::run(acc[i][j], bf[0][j], af[1]);
          Mfma<BF16>::run(acc[i][j], bf[0][j], af[0]);
        }
      }
    }
   }
  };

  load(0);
  for (int kt = 0; kt < nkt; ++kt) {
    store();
    __syncthreads();
    if (kt + 1 < nkt) load(kt + 1);
    compute();
    __syncthreads();
  }

  // epilogue: acc[i][j][r] = C[m = m0 + 64 wm + 16 i + r16][n = n0 + CW wn + 16 j + 4 q + r]
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int nb = n0 + wn * CW + 16 * j + 4 * q;
    float bv[4];
    int be[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bv[r] = bias && nb + r < N ? bias[nb + r] : 0.f;
      if (H) be[r] = bexp[nb + r];  // [Np]
    }
    float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gm = m0 + wm * 64 + 16 * i + r16;
      const int aei = H ? aexp[min(gm, M - 1)] : 0;
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] = (H ? __builtin_ldexpf(acc[i][j][r], -(aei + be[r])) : acc[i][j][r]) + bv[r];
      if (gm < M) {
        if (nb + 4 <= N && (N & 3) == 0) {
          if (nt)  // streaming stores of a large output (nt_output)
            store16_nt(Y + (size_t)gm * N + nb, __builtin_bit_cast(u32x4, v));
          else
            *(f32x4*)(Y + (size_t)gm * N + nb) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (nb + r < N) Y[(size_t)gm * N + nb + r] = v[r];
        }
        if (COLMAX) {
#pragma unroll
          for (int r = 0; r < 4; ++r) cm[r] = fmaxf(cm[r], fabsf(v[r]));
        }
      }
    }
    if (COLMAX) {  // the 16 lanes of a q group hold the tile's 16 rows of these columns
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float c = cm[r];
        c = fmaxf(c, __shfl_xor(c, 1, 64));
        c = fmaxf(c, __shfl_xor(c, 2, 64));
        c = fmaxf(c, __shfl_xor(c, 4, 64));
        c = fmaxf(c, __shfl_xor(c, 8, 64));
        if (r16 == 0 && nb + r < N) atomicMax(colmax + nb + r, __float_as_uint(c));
      }
    }
  }
}

// one wave per row: exp[r] = row_exp_of(max_c |src[r][c]|)
__global__ __launch_bounds__(256) void row_exp_kernel(const float* __restrict__ src, int R, int L,
                                                      int* __restrict__ exp_out) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* row = src + (size_t)r * L;
  float mx = 0.f;
  if ((L & 3) == 0) {
    for (int c = lane; c < L / 4; c += 64) {
      const f32x4 v = ((const f32x4*)row)[c];
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
  } else {
    for (int c = lane; c < L; c += 64) mx = fmaxf(mx, fabsf(row[c]));
  }
  mx = wave_max(mx);
  if (lane == 0) exp_out[r] = row_exp_of(mx);
}

// [R][L] fp32 -> two f16 planes [2][ldr][L] of the row-scaled values + exp[ldr] (rows >= R
// zero, exponent 0).  One wave per row: the row maximum from 16-B loads, then a second pass
// over the (L2-resident) row writing 16 B per plane per 8 values (L % 8 == 0; a scalar tail
// otherwise)
__global__ __launch_bounds__(256) void split2h_kernel(const float* __restrict__ src, int R, int L,
                                                      int ldr, uint16_t* __restrict__ dst,
                                                      int* __restrict__ exp_out) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= ldr) return;
  const float* row = src + (size_t)r * L;
  const bool vec = (L & 7) == 0;
  float mx = 0.f;
  if (r < R) {
    if (vec) {
      for (int c = lane; c < L / 4; c += 64) {
        const f32x4 v = ((const f32x4*)row)[c];
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      }
    } else {
      for (int c = lane; c < L; c += 64) mx = fmaxf(mx, fabsf(row[c]));
    }
  }
  mx = wave_max(mx);
  const int e = row_exp_of(mx);
  if (lane == 0) exp_out[r] = e;
  uint16_t* dh = dst + (size_t)r * L;
  uint16_t* dl = dst + (size_t)ldr * L + (size_t)r * L;
  if (vec) {
    for (int c = lane; c < L / 8; c += 64) {
      f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
      if (r < R) {
        v0 = ((const f32x4*)row)[2 * c];
        v1 = ((const f32x4*)row)[2 * c + 1];
      }
      uint32_t h[8], l[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        split2h(__builtin_ldexpf(v0[k], e), h[k], l[k]);
        split2h(__builtin_ldexpf(v1[k], e), h[4 + k], l[4 + k]);
      }
      ((u32x4*)dh)[c] = u32x4{h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16)};
      ((u32x4*)dl)[c] = u32x4{l[0] | (l[1] << 16), l[2] | (l[3] << 16), l[4] | (l[5] << 16), l[6] | (l[7] << 16)};
    }
  } else {
    for (int c = lane; c < L; c += 64) {
      uint32_t h, l;
      split2h(r < R ? __builtin_ldexpf(row[c], e) : 0.f, h, l);
      dh[c] = (uint16_t)h;
      dl[c] = (uint16_t)l;
    }
  }
}

}  // namespace

}  // namespace sqmp

using namespace sqmp;

extern "C" int sqmp_split2_f16(const float* src, int R, int L, int ldr, void* dst, int* rexp,
                               void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!src || !dst || !rexp || R <= 0 || L <= 0 || ldr < R) return SQMP_EINVAL;
  split2h_kernel<<<cdiv(ldr, 4), 256, 0, (hipStream_t)stream>>>(src, R, L, ldr, (uint16_t*)dst, rexp);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

extern "C" int sqmp_row_exp(const float* src, int R, int L, int* rexp, void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!src || !rexp || R < 0 || L <= 0) return SQMP_EINVAL;
  if (R == 0) return SQMP_OK;
  row_exp_kernel<<<cdiv(R, 4), 256, 0, (hipStream_t)stream>>>(src, R, L, rexp);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

extern "C" int sqmp_gemm_h2(const float* a, const int* aexp, const void* b2, const int* bexp,
                            const float* bias, float* y, int M, int N, int L, uint32_t* colmax,
                            void* stream) {
  SQMP_DEVICE_GUARD(stream);
  if (!a || !aexp || !b2 || !bexp || !y || M < 0 || N <= 0 || L <= 0) return SQMP_EINVAL;
  if (L % X3_BK != 0) return SQMP_EINVAL;
  if (M == 0) return SQMP_OK;
  const int Np = pad_n(N);
  const int tiles_m = cdiv(M, X3_BM), tiles_n = cdiv(N, X3_BN);
  const bool small = (long)tiles_m * tiles_n < 2L * 256;
  // 128 x 256 tiles (8 waves of 64 x 64: half the A re-fetch and A split work per MFMA of
  // 128 x 128 tiles) wherever they still give every CU a workgroup
  const int tiles_n2 = cdiv(N, 256);
  const char* we = knob("SQMP_H2_WIDE");  // SQMP_H2_WIDE=0: 128 x 128 tiles only (A/B knob)
  const bool wide_ok = !we || atoi(we) != 0;
  const bool wide = wide_ok && (long)tiles_m * tiles_n2 >= 256;
  const char* be = knob("SQMP_H2_BK64");  // SQMP_H2_BK64=0: K stages of 32 (A/B knob)
  const bool bk64 = !be || atoi(be) != 0;
  const bool k64 = bk64 && L % 64 == 0;
  const int nt = nt_output((size_t)M * N * sizeof(float)) ? 1 : 0;
  // row tiles per raster group: 4 (same box, config-2 fp32 step: 1 / 2 / 4 / 8 / 16 / 32 ->
  // 2078.7 / 2074.1 / 2002.3 / 2037.9 / 2146.8 / 2178.6 us, profiles/r03_ab_h2_group_m.txt);
  // SQMP_H2_GROUP_M: A/B knob, read per launch
  const char* ge = knob("SQMP_H2_GROUP_M");
  const int gm = ge && atoi(ge) > 0 ? atoi(ge) : 4;
#define SQMP_H2(CM, WN, BNV, TN)                                                                 \
  (k64 ? gemm_x3_kernel<CM, WN, true, BNV, 64><<<tiles_m * TN, 128 * WN, 0, (hipStream_t)stream>>>( \
             a, (const uint16_t*)b2, bias, y, M, N, L, Np, tiles_m, TN, colmax, aexp, bexp, nt, gm) \
       : gemm_x3_kernel<CM, WN, true, BNV, 32><<<tiles_m * TN, 128 * WN, 0, (hipStream_t)stream>>>( \
             a, (const uint16_t*)b2, bias, y, M, N, L, Np, tiles_m, TN, colmax, aexp, bexp, nt, gm))
  if (colmax) {
    if (wide) SQMP_H2(true, 4, 256, tiles_n2); else if (small) SQMP_H2(true, 4, 128, tiles_n); else SQMP_H2(true, 2, 128, tiles_n);
  } else {
    if (wide) SQMP_H2(false, 4, 256, tiles_n2); else if (small) SQMP_H2(false, 4, 128, tiles_n); else SQMP_H2(false, 2, 128, tiles_n);
  }
#undef SQMP_H2
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}
