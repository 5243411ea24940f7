// Lane-contiguous activation quantizer (OUT_FP, fp16 / bf16): the pre-GEMM half of
// W4A4Linear.forward (/root/reference/smoothquant/fake_quant.py:291-304) with the bound
// act quantizer (:56-75 per_token / per_tensor, :77-101 unsorted and :104-154 sorted
// per_group), producing the faithful GEMM's A operand [M][P + S_pad]:
//   positions p < P (packed weight order): x_hat of column amap[p], 0 at salient/padding;
//   positions P + j: the exact salient column sal[j], 0 beyond S.
//
// Layout of the work (one workgroup = NW waves, two rows at a time):
//   * LDS holds the two rows INTERLEAVED: word k = (x[m][k], x[m+1][k]) as two D halves,
//     so every 32-bit LDS access moves both rows' values of one column.
//   * Thread t owns the RPL consecutive activation ranks [RPL t, RPL (t+1)) (its entries
//     of the per-call table: column | packed position << 16 in rank order, built by
//     build_ent_kernel).  A per_group group is G consecutive ranks, so for G >= RPL a
//     thread's values lie in one group (G / RPL lanes per group, combined by lane
//     shuffles; groups never straddle waves) and for G < RPL a thread holds RPL / G whole
//     groups: the group absmax needs no LDS atomics.
//   * Per row pair: 16-B global loads (the next pair's issued after the interleave) -> interleave into
//     LDS -> gather the thread's RPL column pairs (ds_read_b32) -> group absmax on the
//     packed magnitudes (v_pk_max_u16) -> scales -> quantize both rows at once with packed
//     math -> scatter to the packed positions in the same LDS buffer (ds_write_b32) ->
//     de-interleave 16-B chunks -> 16-B global stores of both rows.
// Numerics (bit-exact with the reference, signed zeros included):
//   scale s = D(D(clamp(absmax, 1e-5)) / q_max), r = fp32(1 / s) correctly rounded;
//   q = fl32(x / s) by Markstein's correction (q0 = x r, e = fma(-q0, s, x) exact,
//   q = fma(e, r, q0) is the correctly rounded quotient); code = rne(D(q)) (fp16: the
//   1536 magic add, exact for |q| < 512); x_hat = D(code * s) (one correctly rounded D
//   product) with the sign of x (the reference's -0.0 for small negative values).
#include <stdlib.h>

#include "sqmp_internal.h"

namespace sqmp {

namespace {

constexpr int LC_MODE_TOKEN = 0, LC_MODE_TENSOR = 1, LC_MODE_GROUP = 2;
constexpr int LC_CH = 2;    // 16-B input chunks per thread per row
constexpr int LC_MAXW = 16;  // waves per workgroup (1024 threads)

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 b16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

__device__ inline uint32_t pk_absmax(uint32_t a, uint32_t b) {
  // both halves are D values; their magnitudes order like unsigned 16-bit integers
  const u16x2 x = __builtin_bit_cast(u16x2, a & 0x7FFF7FFFu);
  const u16x2 y = __builtin_bit_cast(u16x2, b & 0x7FFF7FFFu);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
}

template <class DT>
__device__ inline float half_lo(uint32_t w) {
  return DT::to_f(__builtin_bit_cast(typename DT::T, (uint16_t)(w & 0xFFFFu)));
}
template <class DT>
__device__ inline float half_hi(uint32_t w) {
  return DT::to_f(__builtin_bit_cast(typename DT::T, (uint16_t)(w >> 16)));
}

// lane-xor max of both halves over `width` lanes (width a power of two <= 64)
__device__ inline uint32_t xor_max(uint32_t v, int width) {
  for (int o = 1; o < width; o <<= 1) v = pk_absmax(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// the two rows' scales of one group
struct PairScale {
  f32x2 s, r;     // D scale (as fp32) and its correctly rounded reciprocal
  uint32_t sd;    // both scales as D bit patterns
};

// s = D(fl32(D(clamp(absmax, 1e-5)) / q_max)) and r = fl32(1 / s) without IEEE divisions:
// the quotient by Markstein's correction with rq = fl32(1 / q_max) and the reciprocal by
// one Newton step from v_rcp_f32 -- both equal to the correctly rounded results for every
// D operand (exhaustive proof: tests/test_lc_arith_cpu.py)
template <class DT>
__device__ inline PairScale pair_scale(uint32_t mx, float qm, float rq) {
  PairScale c;
  const float lo = rd<DT>(1e-5f);
  f32x2 a = {half_lo<DT>(mx), half_hi<DT>(mx)};
  a[0] = a[0] < lo ? lo : a[0];
  a[1] = a[1] < lo ? lo : a[1];
  const f32x2 q0 = a * rq;
  const f32x2 e = __builtin_elementwise_fma(-q0, (f32x2){qm, qm}, a);
  const f32x2 s = __builtin_elementwise_fma(e, (f32x2){rq, rq}, q0);
  c.s[0] = rd<DT>(s[0]);
  c.s[1] = rd<DT>(s[1]);
  const f32x2 y = {__builtin_amdgcn_rcpf(c.s[0]), __builtin_amdgcn_rcpf(c.s[1])};
  const f32x2 ey = __builtin_elementwise_fma(-c.s, y, (f32x2){1.f, 1.f});
  c.r = __builtin_elementwise_fma(ey, y, y);
  c.sd = (uint32_t)__builtin_bit_cast(uint16_t, DT::from_f(c.s[0])) |
         ((uint32_t)__builtin_bit_cast(uint16_t, DT::from_f(c.s[1])) << 16);
  return c;
}

template <class DT>
__device__ inline uint32_t quant_pair(uint32_t v, const PairScale& c);

template <>
__device__ inline uint32_t quant_pair<F16>(uint32_t v, const PairScale& c) {
  const f32x2 t = __builtin_convertvector(__builtin_bit_cast(h16x2, v), f32x2);
  const f32x2 q0 = t * c.r;
  const f32x2 e = __builtin_elementwise_fma(-q0, c.s, t);
  const f32x2 q = __builtin_elementwise_fma(e, c.r, q0);
  const h16x2 d = __builtin_convertvector(q, h16x2);
  const h16x2 magic = {(_Float16)1536.0f, (_Float16)1536.0f};
  const h16x2 code = (d + magic) - magic;
  const h16x2 y = code * __builtin_bit_cast(h16x2, c.sd);
  return __builtin_bit_cast(uint32_t, y) | (v & 0x80008000u);
}

template <>
__device__ inline uint32_t quant_pair<BF16>(uint32_t v, const PairScale& c) {
  f32x2 t;
  t[0] = __uint_as_float(v << 16);
  t[1] = __uint_as_float(v & 0xFFFF0000u);
  const f32x2 q0 = t * c.r;
  const f32x2 e = __builtin_elementwise_fma(-q0, c.s, t);
  const f32x2 q = __builtin_elementwise_fma(e, c.r, q0);
  const uint32_t db = __builtin_bit_cast(uint32_t, __builtin_convertvector(q, b16x2));
  f32x2 d;
  d[0] = __uint_as_float(db << 16);
  d[1] = __uint_as_float(db & 0xFFFF0000u);
  const f32x2 y = __builtin_elementwise_roundeven(d) * c.s;  // code * s: exact in fp32
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(y, b16x2)) | (v & 0x80008000u);
}

// The two rows' integer codes (the same D(x/s) and round-half-even as quant_pair) as fp32.
template <class DT>
__device__ inline f32x2 code_pair(uint32_t v, const PairScale& c);

template <>
__device__ inline f32x2 code_pair<F16>(uint32_t v, const PairScale& c) {
  const f32x2 t = __builtin_convertvector(__builtin_bit_cast(h16x2, v), f32x2);
  const f32x2 q0 = t * c.r;
  const f32x2 e = __builtin_elementwise_fma(-q0, c.s, t);
  const f32x2 q = __builtin_elementwise_fma(e, c.r, q0);
  const h16x2 d = __builtin_convertvector(q, h16x2);
  const h16x2 magic = {(_Float16)1536.0f, (_Float16)1536.0f};
  return __builtin_convertvector((d + magic) - magic, f32x2);
}

template <>
__device__ inline f32x2 code_pair<BF16>(uint32_t v, const PairScale& c) {
  f32x2 t;
  t[0] = __uint_as_float(v << 16);
  t[1] = __uint_as_float(v & 0xFFFF0000u);
  const f32x2 q0 = t * c.r;
  const f32x2 e = __builtin_elementwise_fma(-q0, c.s, t);
  const f32x2 q = __builtin_elementwise_fma(e, c.r, q0);
  const uint32_t db = __builtin_bit_cast(uint32_t, __builtin_convertvector(q, b16x2));
  f32x2 d;
  d[0] = __uint_as_float(db << 16);
  d[1] = __uint_as_float(db & 0xFFFF0000u);
  return __builtin_elementwise_roundeven(d);
}

// The two rows' 4-bit codes + 8 (the same D(x/s) and round-half-even as code_pair) in
// bytes 0 (row m0) and 2 (row m0 + 1), the other bytes unspecified: the low byte of D(q) + 1544
// (fp16, one ulp = 1 from 1024) / fl32(D(q) + 2^23 + 8) (bf16) is code + 8 (exhaustive
// check: tests/test_lc_arith_cpu.py)
template <class DT>
__device__ inline uint32_t nib_pair(uint32_t v, const PairScale& c);

template <>
__device__ inline uint32_t nib_pair<F16>(uint32_t v, const PairScale& c) {
  const f32x2 t = __builtin_convertvector(__builtin_bit_cast(h16x2, v), f32x2);
  const f32x2 q0 = t * c.r;
  const f32x2 e = __builtin_elementwise_fma(-q0, c.s, t);
  const f32x2 q = __builtin_elementwise_fma(e, c.r, q0);
  const h16x2 magic = {(_Float16)1544.0f, (_Float16)1544.0f};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(q, h16x2) + magic);
}

template <>
__device__ inline uint32_t nib_pair<BF16>(uint32_t v, const PairScale& c) {
  f32x2 t;
  t[0] = __uint_as_float(v << 16);
  t[1] = __uint_as_float(v & 0xFFFF0000u);
  const f32x2 q0 = t * c.r;
  const f32x2 e = __builtin_elementwise_fma(-q0, c.s, t);
  const f32x2 q = __builtin_elementwise_fma(e, c.r, q0);
  const uint32_t db = __builtin_bit_cast(uint32_t, __builtin_convertvector(q, b16x2));
  f32x2 dq;
  dq[0] = __uint_as_float(db << 16);
  dq[1] = __uint_as_float(db & 0xFFFF0000u);
  const f32x2 m = dq + (f32x2){8388616.0f, 8388616.0f};
  return __builtin_amdgcn_perm(__float_as_uint(m[1]), __float_as_uint(m[0]), 0x0c040c00u);
}

// F8 output: the codes as OCP e4m3 bytes, row m0 in byte 0, row m0 + 1 in byte 2 -- exact
// for |code| <= 15, so every 4-bit code.
template <class DT>
__device__ inline uint32_t f8_pair(uint32_t v, const PairScale& c) {
  const f32x2 code = code_pair<DT>(v, c);
  const int w = __builtin_amdgcn_cvt_pk_fp8_f32(code[0], 0.f, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(code[1], 0.f, w, true);
}

}  // namespace

// Timing stamps (SQMP_DIAG_BUILD only): thread 0 of quantizer workgroup b records the 100-MHz
// real-time counter at kernel entry (0), after the prologue (1) and, for its first row pair,
// after the interleave (2), the gather + statistics (3) and the quantize / scatter (4)
// barriers and at the pair's end (5), and when it leaves (6); (7) once the salient mask's
// loads (issued after the first pair's) have landed: tools/lc_stamps.py
#ifdef SQMP_DIAG_BUILD
__device__ unsigned long long sqmp_lc_stamps[8192][8];
#define LC_STAMP(k)                                                   \
  do {                                                                \
    if (threadIdx.x == 0 && bid < 8192)                               \
      sqmp_lc_stamps[bid][k] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
#else
#define LC_STAMP(k) \
  do {              \
  } while (0)
#endif

// RPL = ranks per thread; GS = the group size when it is below RPL (RPL / GS groups per
// thread), else 0.  blockDim = 64 * NW.  F8 = 1 (token / tensor modes): out is e4m3 codes
// [M][P] (bytes), out_scale the fp32 row scales, out_xs the exact salient columns [M][S_pad].
// F8 = 3 (SQMP_OUT_C4, group mode, G >= RPL): out is the int4 codes in ACTIVATION-RANK
// order as bpack rows of Kq positions (Kq / 2 bytes per row; the act-order GEMM operand),
// out_scale (as D) the group scales [Kq / G][ldsc], out_xs the exact salient columns.
// ldsc < 0 (SQMP_QA_TILED): the three in sqmp_gemm_fqt7's tile-major layouts (fq7 with TJ =
// 2 or 4 row tiles: 16 TJ-row blocks nb = m / (16 TJ), row tile j = m / 16 % TJ, r16 = m % 16);
// -ldsc = ngq * 8 + TJ.
// (the body of quant_lc_kernel: workgroup `bid` of `nblk` quantizer workgroups)
template <class DT, int MODE, int RPL, int GS, int F8 = 0, int NOUT = 1>
__device__ __forceinline__ void quant_lc_body(
    const typename DT::T* x, int M, int K, int q_max, int G,
    const uint32_t* __restrict__ lctab, int Kn, const int32_t* __restrict__ amap, int P,
    const int32_t* __restrict__ sal, int S, int S_pad, const uint32_t* __restrict__ cmax,
    const int32_t* __restrict__ nonsal, typename DT::T* out, uint32_t* __restrict__ key_clear,
    int clear_words, float* __restrict__ out_scale, typename DT::T* __restrict__ out_xs,
    int Kq, int ldsc, const int bid, const int nblk, const LcSib& sib = LcSib{}) {
  static_assert(!F8 || F8 == 3 || MODE != LC_MODE_GROUP, "F8 codes need one scale per row");
  static_assert(NOUT == 1 || (F8 == 0 && GS == 0), "sibling outputs: OUT_FP, groups >= RPL");
  static_assert(F8 != 3 || (MODE == LC_MODE_GROUP && GS == 0), "C4: groups of >= RPL ranks");
  // x and out alias for in-place output quantization (every row is read before it is
  // written: a workgroup stores a pair only after loading it)
  typedef typename DT::T T;
  // [NR][W + 8] column pairs: region 0 = the interleaved input, then output 0; region 1 =
  // the sibling outputs, one after another (NOUT = 3: output 1, stored, then output 2 over
  // it -- every position < P of a sibling output is rewritten by its scatter, the values at
  // its non-salient positions and zeros at its salient ones from the table's pad entries,
  // pad_entry in sqmp_actquant.hip; padding positions >= K are never written and stay zero).
  // Two regions instead of three keep the q/k/v quantizer at four workgroups per CU.
  constexpr int NR = NOUT < 2 ? NOUT : 2;
  extern __shared__ __attribute__((aligned(16))) uint32_t lc_buf[];
  __shared__ float lc_red[2][LC_MAXW];
  const int nthr = blockDim.x;
  const int NW = nthr >> 6;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = P + S_pad;          // output row length (multiple of 8)
  const int nchk = K / 8;           // 16-B input chunks per row
  const int ochk = W / 8;           // 16-B output chunks per row
  const int rb = RPL * tid;         // this thread's first rank
  const float qmf = (float)q_max, rqf = 1.0f / qmf;  // pair_scale's divisor, reciprocal

  // the first row pair's loads go out before the prologue (their latency covers it)
  const int npair = (M + 1) / 2;
  u32x4 nx0[LC_CH], nx1[LC_CH];
  // Every call issues exactly 2 LC_CH loads (pair index and chunk clamped, never
  // conditional): the compiler's vmcnt waits count them, so waiting for an older load (the
  // table entries of the current pair) does not wait for the prefetched pair as well
  auto load_pair = [&](int rp) {
    rp = rp < npair - 1 ? rp : npair - 1;
    const int m0 = 2 * rp;
    const bool has1 = m0 + 1 < M;
    const u32x4* s0 = (const u32x4*)(x + (size_t)m0 * K);
    const u32x4* s1 = (const u32x4*)(x + (size_t)(has1 ? m0 + 1 : m0) * K);
#pragma unroll
    for (int i = 0; i < LC_CH; ++i) {
      // (chunks past the row reload its last one, rows past M row m0: those lanes are never
      // written to LDS or stored)
      const int c = min(tid + nthr * i, nchk - 1);
      nx0[i] = s0[c];
      nx1[i] = s1[c];
    }
  };

  // Row pairs in contiguous runs per workgroup, consecutive runs on one XCD (blocks are dealt
  // round-robin over the 8 XCDs): the workgroups that write one 32-row block of the
  // tile-major outputs (and neighbouring rows of the row-major ones) share an L2, so its
  // partial-line writes merge there instead of leaving eight XCDs as masked writes.
  const int xcd = bid & 7, per = nblk >> 3, rem = nblk & 7;
  const int wg = (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + (bid >> 3);
  // (runs of floor or ceil(npair / nblk) pairs: every XCD gets an eighth of the rows)
  LC_STAMP(0);
  const int rp_end = (int)((long)(wg + 1) * npair / nblk);
  int rp = (int)((long)wg * npair / nblk);

  // ---- this thread's RPL table entries (L1/L2-resident, padded to whole rounds with pad
  // entries), the same for every row pair: for the OUT_FP outputs the first pair's are loaded
  // here, first, so that their round trip overlaps x's instead of following the prologue
  // (the F8 / C4 outputs load them per pair: held through the prologue they cost those
  // kernels 16 VGPRs and a wave per SIMD)
  uint32_t tab[RPL];
  uint32_t tabs[NOUT > 1 ? NOUT - 1 : 1][RPL];  // the siblings' tables (same ranks, their positions)
  auto load_tab = [&]() {
    int toff = rb;
    asm volatile("" : "+v"(toff));  // re-read per pair (no loop-invariant hoisting)
#pragma unroll
    for (int i = 0; i < RPL / 4; ++i) {
      const u32x4 e = ((const u32x4*)(lctab + toff))[i];
      tab[4 * i] = e[0]; tab[4 * i + 1] = e[1]; tab[4 * i + 2] = e[2]; tab[4 * i + 3] = e[3];
    }
#pragma unroll
    for (int o = 0; o + 1 < NOUT; ++o)
#pragma unroll
      for (int i = 0; i < RPL / 4; ++i) {
        const u32x4 e = ((const u32x4*)(sib.tab[o] + toff))[i];
        tabs[o][4 * i] = e[0]; tabs[o][4 * i + 1] = e[1];
        tabs[o][4 * i + 2] = e[2]; tabs[o][4 * i + 3] = e[3];
      }
  };
  if (F8 == 0) load_tab();

  // ---- once per workgroup: zeroed buffer (+ two spare words: W = a zero read by padding
  // table entries, W + 1 = a write-only sink for their scatter).  The salient positions of
  // the output are zeroed by the table itself where its producer wrote (zero word, salient
  // position) pad entries (pad_entry, sqmp_actquant.hip; amap NULL here); with amap, by a
  // mask built here.  Issue order: the mask's and the salient list's loads, then the first
  // row pair's x, so that the mask's wait (vmcnt counts in issue order) does not wait for x
  // and the prologue runs under x's latency.
  const int zp0 = 64 * tid;
  // the salient mask of 64-position chunk c (bit i: amap[64 c + i] < 0, positions < K) is one
  // wave ballot over a coalesced dword per lane; wave w takes chunks w, w + NW, ... (at most
  // 16: K <= 16384, NW >= K / 1024) and parks the masks in LDS for their owner, thread c
  const int nzc = F8 == 0 && amap ? (K + 63) >> 6 : 0;
  uint32_t zraw[F8 == 0 ? 16 : 1];
  if (F8 == 0 && amap) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = 64 * (wave + NW * i) + lane;  // (clamped: an unconditional load)
      zraw[i] = (uint32_t)amap[min(p, K - 1)];
    }
  }
  // the salient list in two registers per thread (unconditional loads from a clamped index --
  // lctab stands in for an empty list -- so no select waits for them)
  const bool sal_reg = S <= 2 * nthr;
  const int32_t* const salp = S > 0 ? sal : (const int32_t*)lctab;
  uint32_t salr[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) salr[k] = (uint32_t)salp[min(tid + k * nthr, S > 0 ? S - 1 : 0)];
  __builtin_amdgcn_sched_barrier(0);
  load_pair(rp);
  __builtin_amdgcn_sched_barrier(0);
  // (amap NULL: in-place output quantization, salient columns pass through: no mask)
  uint32_t* const zm_l = lc_buf + NR * (W + 8) + S_pad;  // [nzc] u64 masks
  if (F8 == 0 && amap) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = wave + NW * i;
      const int p = 64 * c + lane;
      const uint64_t b = __ballot(p < K && (int)zraw[i] < 0);
      if (c < nzc && lane == 0) {
        zm_l[2 * c] = (uint32_t)b;
        zm_l[2 * c + 1] = (uint32_t)(b >> 32);
      }
    }
  }
#ifdef SQMP_DIAG_BUILD
  if (F8 == 0 && amap && zraw[0] == 0x5A5A5A5Au) lc_buf[0] = 1u;  // (keeps the stamp behind the mask's loads)
#endif
  LC_STAMP(7);
  const int RW = W + 8;  // LDS region stride (words; a multiple of 8)
  for (int c = tid; c < (NOUT > 1 ? NR * RW : W + 2); c += nthr) lc_buf[c] = 0u;
  // the salient columns' input positions, once per workgroup (every row pair gathers them:
  // an LDS read instead of a dependent global load per pair)
  uint32_t* const sal_l = lc_buf + NR * RW;
  if (sal_reg) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (tid + k * nthr < S) sal_l[tid + k * nthr] = salr[k];
  } else {
    for (int j = tid; j < S; j += nthr) sal_l[j] = (uint32_t)sal[j];
  }
  // the column statistics of this call, read by the (completed) table kernel: restore the
  // clean-workspace zeros
  if (key_clear)
    for (int c = bid * nthr + tid; c < (clear_words >> 2); c += nblk * nthr)
      ((u32x4*)key_clear)[c] = u32x4{0u, 0u, 0u, 0u};
  PairScale tens;
  if (MODE == LC_MODE_TENSOR) {
    float m = 0.f;
    for (int i = tid; i < Kn; i += nthr) m = fmaxf(m, __uint_as_float(cmax[nonsal[i]]));
    m = wave_max(m);
    if (lane == 0) lc_red[0][wave] = m;
    __syncthreads();
    m = 0.f;
    for (int w = 0; w < NW; ++w) m = fmaxf(m, lc_red[0][w]);
    const uint32_t mb = (uint32_t)__builtin_bit_cast(uint16_t, DT::from_f(m));
    tens = pair_scale<DT>(mb | (mb << 16), qmf, rqf);
  }
  __syncthreads();
  LC_STAMP(1);
  const int rp0 = rp;
  const uint64_t zmask = F8 == 0 && tid < nzc
                             ? (uint64_t)zm_l[2 * tid] | ((uint64_t)zm_l[2 * tid + 1] << 32)
                             : 0ull;

  for (; rp < rp_end; ++rp) {
    const int m0 = 2 * rp;
    const bool has1 = m0 + 1 < M;
    // the table entries again for every later pair (the registers are not kept across
    // pairs), issued first so their latency overlaps the interleave
    if (F8 != 0 || rp != rp0) load_tab();
    // ---- interleave the two rows into LDS: word k = (x[m0][k], x[m0+1][k])
#pragma unroll
    for (int i = 0; i < LC_CH; ++i) {
      const int c = tid + nthr * i;
      if (c < nchk) {
        u32x4 w0, w1;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          w0[2 * k] = __builtin_amdgcn_perm(nx1[i][k], nx0[i][k], 0x05040100u);
          w0[2 * k + 1] = __builtin_amdgcn_perm(nx1[i][k], nx0[i][k], 0x07060302u);
          w1[2 * k] = __builtin_amdgcn_perm(nx1[i][k + 2], nx0[i][k + 2], 0x05040100u);
          w1[2 * k + 1] = __builtin_amdgcn_perm(nx1[i][k + 2], nx0[i][k + 2], 0x07060302u);
        }
        // lanes 4-7 of every 8 write their second half first: ds_write_b128 banks (a/4) mod 32
        // over groups of 8 contiguous lanes (MI355X_MICROARCH.md §LDS), where in order lanes
        // i and i + 4 of a 32-B-stride write meet in one bank
        const bool sw = (c >> 2) & 1;
        ((u32x4*)lc_buf)[2 * c + (sw ? 1 : 0)] = sw ? w1 : w0;
        ((u32x4*)lc_buf)[2 * c + (sw ? 0 : 1)] = sw ? w0 : w1;
      }
    }
    // prefetch the next pair: its registers are free once interleaved, and its latency now
    // overlaps this pair's gather, quantization and stores (same VGPR count)
    load_pair(rp + 1 < rp_end ? rp + 1 : rp);  // (the last pair reloads itself, unused)
    __syncthreads();
    if (rp == rp0) LC_STAMP(2);

    // ---- gather; exact salient columns into the tail (>= K)
    uint32_t v[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) v[i] = lc_buf[tab[i] & 0xFFFFu];
    for (int j = tid; j < S; j += nthr) {
      const uint32_t xs = lc_buf[sal_l[j]];
      lc_buf[P + j] = xs;
      if (NOUT > 1) lc_buf[RW + P + j] = xs;  // the siblings' shared salient tail
    }

    // ---- scales, then quantize + scatter
    if (MODE == LC_MODE_GROUP && GS > 0) {
      __syncthreads();  // every gather done before the scatter below
      if (rp == rp0) LC_STAMP(3);
#pragma unroll
      for (int g = 0; g < RPL / (GS > 0 ? GS : RPL); ++g) {
        uint32_t mx = 0u;
#pragma unroll
        for (int i = g * GS; i < (g + 1) * GS; ++i) mx = pk_absmax(mx, v[i]);
        const PairScale c = pair_scale<DT>(mx, qmf, rqf);
#pragma unroll
        for (int i = g * GS; i < (g + 1) * GS; ++i) lc_buf[tab[i] >> 16] = quant_pair<DT>(v[i], c);
      }
    } else {
      PairScale c = tens;
      if (MODE != LC_MODE_TENSOR) {
        uint32_t mx = 0u;
#pragma unroll
        for (int i = 0; i < RPL; ++i) mx = pk_absmax(mx, v[i]);
        if (MODE == LC_MODE_GROUP) {
          mx = xor_max(mx, G / RPL);
        } else {
          mx = xor_max(mx, 64);
          if (lane == 0) {
            lc_red[0][wave] = half_lo<DT>(mx);
            lc_red[1][wave] = half_hi<DT>(mx);
          }
        }
        __syncthreads();  // every gather done before the scatter below (+ token maxima)
        if (rp == rp0) LC_STAMP(3);
        if (MODE == LC_MODE_TOKEN) {
          float m0f = 0.f, m1f = 0.f;
          for (int w = 0; w < NW; ++w) {
            m0f = fmaxf(m0f, lc_red[0][w]);
            m1f = fmaxf(m1f, lc_red[1][w]);
          }
          mx = (uint32_t)__builtin_bit_cast(uint16_t, DT::from_f(m0f)) |
               ((uint32_t)__builtin_bit_cast(uint16_t, DT::from_f(m1f)) << 16);
        }
        c = pair_scale<DT>(mx, qmf, rqf);
      } else {
        __syncthreads();
        if (rp == rp0) LC_STAMP(3);
      }
      if (F8 == 3) {
        // ranks rb .. rb + 15 = positions 16 u .. 16 u + 15 of bpack block rb / 64: dwords u
        // (elements 0-7) and 4 + u (8-15); element e at nibble e / 2 (even e) or 4 + e / 2
        if (rb < Kq) {
          // elements 2p, 2p + 1 of a dword: one v_perm_b32 per row puts their code bytes at
          // bits 0 and 16, shifted to nibbles p and 4 + p
          uint32_t d0[2] = {0u, 0u}, d1[2] = {0u, 0u};
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int p = 0; p < 4; ++p) {
              const uint32_t lo = nib_pair<DT>(v[8 * h + 2 * p], c);
              const uint32_t hi = nib_pair<DT>(v[8 * h + 2 * p + 1], c);
              d0[h] |= __builtin_amdgcn_perm(hi, lo, 0x0c040c00u) << (4 * p);
              d1[h] |= __builtin_amdgcn_perm(hi, lo, 0x0c060c02u) << (4 * p);
            }
          const int u = (rb >> 4) & 3;
          if (ldsc < 0) {
            // Bt[nb][kb][lane][j][s] (TJ = 2 or 4 row tiles of 16 per 16 TJ-row block nb):
            // dword d of the row's block kb at lane 16 (d / 2) + r16, slot 2 j + d % 2 (m0
            // even: both rows share nb and j).  Lanes u and u ^ 1 hold the two slots of a
            // lane: the even one stores row m0's pair, the odd one row m0 + 1's, 8 B each
            // (Kq % 128 == 0: both lanes of a pair are active)
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            const int TJ = (-ldsc) & 7, ngq = (-ldsc) >> 3;
            const int nb = m0 / (16 * TJ), j = (m0 >> 4) & (TJ - 1), r = m0 & 15, od = u & 1;
            const uint32_t x0 = __shfl_xor(od ? d0[0] : d1[0], 1, 64);
            const uint32_t x1 = __shfl_xor(od ? d0[1] : d1[1], 1, 64);
            u32x2* t = (u32x2*)out + ((size_t)nb * (Kq / 64) + (rb >> 6)) * (64 * TJ) + j;
            const int rr = r + od;
            if (!od || has1) {
              const u32x2 va = od ? u32x2{x0, d1[0]} : u32x2{d0[0], x0};
              const u32x2 vb = od ? u32x2{x1, d1[1]} : u32x2{d0[1], x1};
              t[(16 * (u >> 1) + rr) * TJ] = va;
              t[(16 * (2 + (u >> 1)) + rr) * TJ] = vb;
            }
            if (rb % G == 0) {
              // St[nb][g][r16][j]
              uint16_t* sc = (uint16_t*)out_scale + ((size_t)(nb * ngq + rb / G) * 16 + r) * TJ + j;
              sc[0] = (uint16_t)(c.sd & 0xFFFFu);
              if (has1) sc[TJ] = (uint16_t)(c.sd >> 16);
            }
          } else {
            uint32_t* r0 = (uint32_t*)((unsigned char*)out + (size_t)m0 * (Kq / 2)) + (rb >> 6) * 8;
            uint32_t* r1 = (uint32_t*)((unsigned char*)out + (size_t)(m0 + 1) * (Kq / 2)) + (rb >> 6) * 8;
            r0[u] = d0[0];
            r0[4 + u] = d0[1];
            if (has1) {
              r1[u] = d1[0];
              r1[4 + u] = d1[1];
            }
            if (rb % G == 0) {
              uint16_t* sc = (uint16_t*)out_scale + (size_t)(rb / G) * ldsc + m0;
              sc[0] = (uint16_t)(c.sd & 0xFFFFu);
              if (has1) sc[1] = (uint16_t)(c.sd >> 16);
            }
          }
        }
      } else if (F8) {
        // F8 = 1: the table is in packed-POSITION order (pos_table_kernel), so this thread's
        // RPL codes are positions rb .. rb + RPL - 1 of both rows: packed in registers and
        // stored straight to global memory (no LDS scatter, no second pass)
        if (rb < P) {
          uint32_t w0[RPL / 4], w1[RPL / 4];
#pragma unroll
          for (int d = 0; d < RPL / 4; ++d) {
            const uint32_t b0 = f8_pair<DT>(v[4 * d], c), b1 = f8_pair<DT>(v[4 * d + 1], c);
            const uint32_t b2 = f8_pair<DT>(v[4 * d + 2], c), b3 = f8_pair<DT>(v[4 * d + 3], c);
            // v_perm_b32 selector bytes: 0-3 = lo operand, 4-7 = hi operand
            const uint32_t lo0 = __builtin_amdgcn_perm(b1, b0, 0x0c0c0400u);
            const uint32_t hi0 = __builtin_amdgcn_perm(b3, b2, 0x04000c0cu);
            const uint32_t lo1 = __builtin_amdgcn_perm(b1, b0, 0x0c0c0602u);
            const uint32_t hi1 = __builtin_amdgcn_perm(b3, b2, 0x06020c0cu);
            w0[d] = lo0 | hi0;
            w1[d] = lo1 | hi1;
          }
          unsigned char* b0p = (unsigned char*)out + (size_t)m0 * P + rb;
#pragma unroll
          for (int d = 0; d < RPL / 16; ++d)
            ((u32x4*)b0p)[d] = u32x4{w0[4 * d], w0[4 * d + 1], w0[4 * d + 2], w0[4 * d + 3]};
          if (has1) {
            unsigned char* b1p = (unsigned char*)out + (size_t)(m0 + 1) * P + rb;
#pragma unroll
            for (int d = 0; d < RPL / 16; ++d)
              ((u32x4*)b1p)[d] = u32x4{w1[4 * d], w1[4 * d + 1], w1[4 * d + 2], w1[4 * d + 3]};
          }
        }
        if (tid == 0) {
          out_scale[m0] = c.s[0];
          if (has1) out_scale[m0 + 1] = c.s[1];
        }
      } else {
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
          const uint32_t y = quant_pair<DT>(v[i], c);
          lc_buf[tab[i] >> 16] = y;
          if (NOUT > 1) lc_buf[RW + (tabs[0][i] >> 16)] = y;
          if (NOUT > 2) v[i] = y;  // (kept for output 2's scatter)
        }
      }
    }
    // salient columns' own packed positions hold 0 (their weight codes are 0 too; the F8
    // position-order table gathers the zero word for them)
    if (F8 == 0 && amap)
      for (uint64_t zm = zmask; zm; zm &= zm - 1) lc_buf[zp0 + __builtin_ctzll(zm)] = 0u;
    __syncthreads();
    if (rp == rp0) LC_STAMP(4);

    if (F8) {
      // exact salient columns -> out_xs [M][S_pad]
      T* x0 = out_xs + (size_t)m0 * S_pad;
      T* x1 = out_xs + (size_t)(m0 + 1) * S_pad;
      for (int c = tid; c < S_pad / 8; c += nthr) {
        const u32x4 a = ((const u32x4*)lc_buf)[2 * (P / 8 + c)];
        const u32x4 b = ((const u32x4*)lc_buf)[2 * (P / 8 + c) + 1];
        u32x4 z0, z1;
        z0[0] = __builtin_amdgcn_perm(a[1], a[0], 0x05040100u);
        z0[1] = __builtin_amdgcn_perm(a[3], a[2], 0x05040100u);
        z0[2] = __builtin_amdgcn_perm(b[1], b[0], 0x05040100u);
        z0[3] = __builtin_amdgcn_perm(b[3], b[2], 0x05040100u);
        z1[0] = __builtin_amdgcn_perm(a[1], a[0], 0x07060302u);
        z1[1] = __builtin_amdgcn_perm(a[3], a[2], 0x07060302u);
        z1[2] = __builtin_amdgcn_perm(b[1], b[0], 0x07060302u);
        z1[3] = __builtin_amdgcn_perm(b[3], b[2], 0x07060302u);
        if (F8 == 3 && ldsc < 0) {
          // Salt[nb][kd][lane][j][s][8]: chunk cc of block kd = c(q, s) = 4 (q & 1) + 2 s + q / 2
          const int TJ = (-ldsc) & 7;
          const int nb = m0 / (16 * TJ), j = (m0 >> 4) & (TJ - 1), r = m0 & 15, kd = c >> 3, cc = c & 7;
          const int lq = 16 * ((cc >> 2) | ((cc & 1) << 1)), sl = (cc >> 1) & 1;
          u32x4* t = (u32x4*)out_xs + ((size_t)nb * (S_pad / 64) + kd) * (128 * TJ) + 2 * j + sl;
          t[(lq + r) * 2 * TJ] = z0;
          if (has1) t[(lq + r + 1) * 2 * TJ] = z1;
        } else {
          ((u32x4*)x0)[c] = z0;
          if (has1) ((u32x4*)x1)[c] = z1;
        }
      }
      __syncthreads();  // the buffer is rewritten by the next pair
      if (rp == rp0) LC_STAMP(5);
      continue;
    }
    // ---- de-interleave 16-B chunks and store both rows of every output
    // (region r of the LDS as output ob)
    auto store_region = [&](int r, T* ob) {
      for (int c = tid; c < ochk; c += nthr) {
        // ds_read_b128 groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32), banks (a/4) mod 64:
        // at a 32-B stride lanes l and l ^ 24 (l ^ 8 ...) collide; reading the second half first
        // where lane bit 3 is set separates every such pair
        const bool sw = (c >> 3) & 1;
        const u32x4 f = ((const u32x4*)(lc_buf + r * RW))[2 * c + (sw ? 1 : 0)];
        const u32x4 g = ((const u32x4*)(lc_buf + r * RW))[2 * c + (sw ? 0 : 1)];
        const u32x4 a = sw ? g : f, b = sw ? f : g;
        u32x4 y0, y1;
        y0[0] = __builtin_amdgcn_perm(a[1], a[0], 0x05040100u);
        y0[1] = __builtin_amdgcn_perm(a[3], a[2], 0x05040100u);
        y0[2] = __builtin_amdgcn_perm(b[1], b[0], 0x05040100u);
        y0[3] = __builtin_amdgcn_perm(b[3], b[2], 0x05040100u);
        y1[0] = __builtin_amdgcn_perm(a[1], a[0], 0x07060302u);
        y1[1] = __builtin_amdgcn_perm(a[3], a[2], 0x07060302u);
        y1[2] = __builtin_amdgcn_perm(b[1], b[0], 0x07060302u);
        y1[3] = __builtin_amdgcn_perm(b[3], b[2], 0x07060302u);
        ((u32x4*)(ob + (size_t)m0 * W))[c] = y0;
        if (has1) ((u32x4*)(ob + (size_t)(m0 + 1) * W))[c] = y1;
      }
    };
    if constexpr (NR == 2) {
      // both regions in one pass (their loads interleave)
      for (int c = tid; c < ochk; c += nthr) {
        const bool sw = (c >> 3) & 1;
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          const u32x4 f = ((const u32x4*)(lc_buf + o * RW))[2 * c + (sw ? 1 : 0)];
          const u32x4 g = ((const u32x4*)(lc_buf + o * RW))[2 * c + (sw ? 0 : 1)];
          const u32x4 a = sw ? g : f, b = sw ? f : g;
          u32x4 y0, y1;
          y0[0] = __builtin_amdgcn_perm(a[1], a[0], 0x05040100u);
          y0[1] = __builtin_amdgcn_perm(a[3], a[2], 0x05040100u);
          y0[2] = __builtin_amdgcn_perm(b[1], b[0], 0x05040100u);
          y0[3] = __builtin_amdgcn_perm(b[3], b[2], 0x05040100u);
          y1[0] = __builtin_amdgcn_perm(a[1], a[0], 0x07060302u);
          y1[1] = __builtin_amdgcn_perm(a[3], a[2], 0x07060302u);
          y1[2] = __builtin_amdgcn_perm(b[1], b[0], 0x07060302u);
          y1[3] = __builtin_amdgcn_perm(b[3], b[2], 0x07060302u);
          T* ob = o == 0 ? out : (T*)sib.out[0];
          ((u32x4*)(ob + (size_t)m0 * W))[c] = y0;
          if (has1) ((u32x4*)(ob + (size_t)(m0 + 1) * W))[c] = y1;
        }
      }
    } else {
      store_region(0, out);
    }
    if constexpr (NOUT > 2) {
      // output 2 over region 1 (every position < P rewritten: its values and its pad
      // entries' zeros), then stored
      __syncthreads();  // region 1 is read before it is rewritten
#pragma unroll
      for (int i = 0; i < RPL; ++i) lc_buf[RW + (tabs[1][i] >> 16)] = v[i];
      __syncthreads();
      store_region(1, (T*)sib.out[1]);
    }
    __syncthreads();  // the buffer is rewritten by the next pair
    if (rp == rp0) LC_STAMP(5);
  }
  LC_STAMP(6);
}


// The packed-order group quantizer (one output) is held to 80 VGPRs (six waves per SIMD, no
// spills): Llama down_proj's 11-wave workgroups then run two per CU instead of one, its 1024
// row pairs in two rounds instead of four sequential pairs per workgroup.
template <int MODE, int F8, int NOUT>
constexpr int lc_waves_per_eu() { return MODE == LC_MODE_GROUP && F8 == 0 && NOUT == 1 ? 6 : 1; }

template <class DT, int MODE, int RPL, int GS, int F8 = 0, int NOUT = 1>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(lc_waves_per_eu<MODE, F8, NOUT>())))
void quant_lc_kernel(
    const typename DT::T* x, int M, int K, int q_max, int G,
    const uint32_t* __restrict__ lctab, int Kn, const int32_t* __restrict__ amap, int P,
    const int32_t* __restrict__ sal, int S, int S_pad, const uint32_t* __restrict__ cmax,
    const int32_t* __restrict__ nonsal, typename DT::T* out, uint32_t* __restrict__ key_clear,
    int clear_words, float* __restrict__ out_scale, typename DT::T* __restrict__ out_xs,
    int Kq, int ldsc, LcSib sib) {
  quant_lc_body<DT, MODE, RPL, GS, F8, NOUT>(x, M, K, q_max, G, lctab, Kn, amap, P, sal, S,
                                             S_pad, cmax, nonsal, out, key_clear, clear_words,
                                             out_scale, out_xs, Kq, ldsc, blockIdx.x, gridDim.x,
                                             sib);
}

// ---- the activation-order weight operand (sqmp_gemm_fqt): wp[n][j] = W_hat[n][pos_j],
// pos_j = lctab[j] >> 16 (the weight-packed position of the column of activation rank j),
// 0 past Kn, then wsal[n][:].  Workgroup `bid` dequantizes its RB codes rows into LDS in
// packed order (one bpack dword -> 8 D values D(code * scale), one 16-B LDS write), then
// gathers them in rank order (an output chunk's table entries are read once for all RB
// rows) and stores 16-B chunks.  Latency-bound rather than byte-bound, so it runs in the
// same launch as the C4 quantizer (quant_c4_fused_kernel), on workgroups of its own.
struct PermArgs {
  const uint32_t* codes;  // bpack [Np][Kp/2]
  const void* wscale;     // D [ngw][Np]
  const void* wsal;       // D [N][S_pad]
  void* wp;               // D [Np][Kq + S_pad]
  int N, Np, Kp, Gw, ngw, Kn, Kq, S_pad, RB;
};

// the 16-B chunk of wp row n at position j0 (j0 % 8 == 0)
template <class T>
__device__ __forceinline__ T* wp_chunk(const PermArgs& a, T* wp, int n, int j0) {
  return wp + (size_t)n * (a.Kq + a.S_pad) + j0;
}

// Even RB: rows in PAIRS interleaved in LDS (word k of pair r2 = (W_hat[n0 + 2 r2][k],
// W_hat[n0 + 2 r2 + 1][k])), so one random-position ds_read_b32 of the rank-order gather
// serves two rows -- half the gather instructions and their bank conflicts of the 16-bit
// reads (4.35 conflict cycles per LDS instruction, profiles/r04_pmc_c4_conflict_split.txt).
template <class DT>
__device__ __forceinline__ void perm_weight_pairs(const PermArgs& a, const uint32_t* __restrict__ lctab,
                                                  const int bid) {
  typedef typename DT::T T;
  extern __shared__ __attribute__((aligned(16))) uint32_t pw_lds[];  // [RB / 2][Kp] row pairs
  const T* wscale = (const T*)a.wscale;
  const T* wsal = (const T*)a.wsal;
  T* wp = (T*)a.wp;
  const int RB = a.RB, Kp = a.Kp, n0 = bid * RB, tid = threadIdx.x;
  const int dw = Kp / 8;  // bpack dwords per codes row
#pragma unroll 2
  for (int i = tid; i < (RB / 2) * dw; i += blockDim.x) {
    const int r2 = i / dw, d = i - r2 * dw, na = n0 + 2 * r2;
    const int p0 = bpack_pos(d, 0);  // its 8 positions p0 .. p0 + 7 (one group: Gw % 8 == 0)
    const int g = min(p0 / a.Gw, a.ngw - 1);
    uint32_t w[8];
    if constexpr (std::is_same<DT, F16>::value) {
      // fp16: the GEMM's decode -- nibbles of elements 2k, 2k + 1 at bits 0 and 16 (bpack_shift),
      // | 0x6400 = 1024 + nibble, - 1032 = code, * scale = D(code * scale) in one rounding (the
      // product is exact before it), two rows per pk op; rows >= N stay +0
      uint32_t pr[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int n = na + h;
        const bool in = n < a.N;
        const uint32_t c = in ? a.codes[(size_t)n * dw + d] : 0u;
        const _Float16 s1 = in ? wscale[(size_t)g * a.Np + n] : (_Float16)0.f;
        const h16x2 sc = {s1, s1};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const h16x2 f = __builtin_bit_cast(h16x2, ((c >> (4 * k)) & 0x000F000Fu) | 0x64006400u);
          const h16x2 y = (f + (h16x2){(_Float16)-1032.f, (_Float16)-1032.f}) * sc;
          pr[h][k] = in ? __builtin_bit_cast(uint32_t, y) : 0u;
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        w[2 * k] = __builtin_amdgcn_perm(pr[1][k], pr[0][k], 0x05040100u);
        w[2 * k + 1] = __builtin_amdgcn_perm(pr[1][k], pr[0][k], 0x07060302u);
      }
    } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = na + h;
      uint32_t c = 0u;
      float sc = 0.f;
      if (n < a.N) {
        c = a.codes[(size_t)n * dw + d];
        sc = DT::to_f(wscale[(size_t)g * a.Np + n]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const T v = n < a.N ? DT::from_f((float)((int)((c >> bpack_shift(e)) & 0xFu) - 8) * sc)
                            : DT::from_f(0.f);
        const uint32_t b = (uint32_t)__builtin_bit_cast(uint16_t, v);
        w[e] = h ? (w[e] | (b << 16)) : b;
      }
    }
    }
    u32x4* dst = (u32x4*)(pw_lds + (size_t)r2 * Kp + p0);
    dst[0] = u32x4{w[0], w[1], w[2], w[3]};
    dst[1] = u32x4{w[4], w[5], w[6], w[7]};
  }
  __syncthreads();
  const int W = a.Kq + a.S_pad, nch = W / 8;
  for (int c = tid; c < nch; c += blockDim.x) {
    const int j0 = 8 * c;
    if (j0 < a.Kq) {
      int pos[8];
      const u32x4 t0 = ((const u32x4*)(lctab + j0))[0], t1 = ((const u32x4*)(lctab + j0))[1];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        pos[e] = j0 + e < a.Kn ? (int)((e < 4 ? t0[e] : t1[e - 4]) >> 16) : -1;
      for (int r2 = 0; r2 < RB / 2; ++r2) {
        uint32_t v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = pos[e] >= 0 ? pw_lds[(size_t)r2 * Kp + pos[e]] : 0u;
        u32x4 lo, hi;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          lo[k] = __builtin_amdgcn_perm(v[2 * k + 1], v[2 * k], 0x05040100u);
          hi[k] = __builtin_amdgcn_perm(v[2 * k + 1], v[2 * k], 0x07060302u);
        }
        *(u32x4*)wp_chunk(a, wp, n0 + 2 * r2, j0) = lo;
        *(u32x4*)wp_chunk(a, wp, n0 + 2 * r2 + 1, j0) = hi;
      }
    } else {
      for (int r = 0; r < RB; ++r) {
        const int n = n0 + r;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        if (n < a.N) v = *(const u32x4*)(wsal + (size_t)n * a.S_pad + (j0 - a.Kq));
        *(u32x4*)wp_chunk(a, wp, n, j0) = v;
      }
    }
  }
}

template <class DT>
__device__ __forceinline__ void perm_weight_body(const PermArgs& a, const uint32_t* __restrict__ lctab,
                                                 const int bid) {
  if (a.RB % 2 == 0) {
    perm_weight_pairs<DT>(a, lctab, bid);
    return;
  }
  typedef typename DT::T T;
  extern __shared__ __attribute__((aligned(16))) uint32_t pw_lds[];  // [RB][Kp] D values
  T* wl = (T*)pw_lds;
  const T* wscale = (const T*)a.wscale;
  const T* wsal = (const T*)a.wsal;
  T* wp = (T*)a.wp;
  const int RB = a.RB, Kp = a.Kp, n0 = bid * RB, tid = threadIdx.x;
  const int dw = Kp / 8;  // bpack dwords per codes row
#pragma unroll 4
  for (int i = tid; i < RB * dw; i += blockDim.x) {
    const int r = i / dw, d = i - r * dw, n = n0 + r;
    const int p0 = bpack_pos(d, 0);  // its 8 positions p0 .. p0 + 7 (one group: Gw % 8 == 0)
    T v[8];
    if (n < a.N) {
      const uint32_t w = a.codes[(size_t)n * dw + d];
      const float sc = DT::to_f(wscale[(size_t)min(p0 / a.Gw, a.ngw - 1) * a.Np + n]);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[e] = DT::from_f((float)((int)((w >> bpack_shift(e)) & 0xFu) - 8) * sc);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = DT::from_f(0.f);
    }
    *(u32x4*)(wl + (size_t)r * Kp + p0) = *(const u32x4*)v;
  }
  __syncthreads();
  const int W = a.Kq + a.S_pad, nch = W / 8;
  for (int c = tid; c < nch; c += blockDim.x) {
    const int j0 = 8 * c;
    if (j0 < a.Kq) {
      // the 8 table entries as two 16-B loads (lctab is padded with (zero, sink) entries to
      // whole rounds of the quantizer, >= Kq)
      int pos[8];
      const u32x4 t0 = ((const u32x4*)(lctab + j0))[0], t1 = ((const u32x4*)(lctab + j0))[1];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        pos[e] = j0 + e < a.Kn ? (int)((e < 4 ? t0[e] : t1[e - 4]) >> 16) : -1;
      for (int r = 0; r < RB; ++r) {
        T v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = pos[e] >= 0 ? wl[(size_t)r * Kp + pos[e]] : DT::from_f(0.f);
        *(u32x4*)wp_chunk(a, wp, n0 + r, j0) = *(const u32x4*)v;
      }
    } else {
      for (int r = 0; r < RB; ++r) {
        const int n = n0 + r;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        if (n < a.N) v = *(const u32x4*)(wsal + (size_t)n * a.S_pad + (j0 - a.Kq));
        *(u32x4*)wp_chunk(a, wp, n, j0) = v;
      }
    }
  }
}

template <class DT>
__global__ __launch_bounds__(1024) void perm_weight_kernel(PermArgs a, const uint32_t* __restrict__ lctab) {
  perm_weight_body<DT>(a, lctab, blockIdx.x);
}

// The C4 quantizer (workgroups 0 .. nq-1) and the weight permutation (the rest) in one
// launch: the two are independent given the table and overlap on the chip.
template <class DT>
__global__ __launch_bounds__(1024) void quant_c4_fused_kernel(
    const typename DT::T* x, int M, int K, int q_max, int G, const uint32_t* __restrict__ lctab,
    int Kn, int P, const int32_t* __restrict__ sal, int S, int S_pad,
    const uint32_t* __restrict__ cmax, const int32_t* __restrict__ nonsal, void* codes,
    uint32_t* __restrict__ key_clear, int clear_words, void* scales, typename DT::T* xs,
    int Kq, int ldsc, int nq, PermArgs pa) {
  if ((int)blockIdx.x < nq)
    quant_lc_body<DT, LC_MODE_GROUP, 16, 0, 3>(x, M, K, q_max, G, lctab, Kn, nullptr, P, sal, S,
                                               S_pad, cmax, nonsal, (typename DT::T*)codes,
                                               key_clear, clear_words, (float*)scales, xs, Kq,
                                               ldsc, blockIdx.x, nq);
  else
    perm_weight_body<DT>(pa, lctab, blockIdx.x - nq);
}

constexpr int LC_RPL = 16;

// dynamic LDS words of quant_lc_body: min(NOUT, 2) regions of P + S_pad + 8 words, the salient list
// and the salient masks of the 64-position chunks (2 words each, K <= P)
static size_t lc_lds_words(int P, int S_pad, int nout) {
  const int nr = nout < 2 ? nout : 2;  // (a third output reuses region 1)
  return (size_t)(P + S_pad + 8) * nr + S_pad + 2 * (size_t)((P + 63) / 64);
}

// Workgroups of `block` threads and `lds` dynamic LDS bytes a CU holds at once for kernel f
// (registers included: the C4 quantizer's 70 VGPRs allow 7 four-wave workgroups, not the 8
// its LDS would), cached per (kernel, block, lds)
static int occ_per_cu(const void* f, int block, size_t lds) {
  struct E { const void* f; int block; size_t lds; int n; };
  static thread_local E cache[16];
  static thread_local int next = 0;
  for (const E& e : cache)
    if (e.f == f && e.block == block && e.lds == lds) return e.n;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, block, lds) != hipSuccess || n < 1) n = 1;
  cache[next] = E{f, block, lds, n};
  next = (next + 1) % 16;
  return n;
}

static int lc_waves(int K, int Kn) {
  const int a = Kn > 0 ? cdiv(Kn, 64 * LC_RPL) : 1;
  const int b = cdiv(K / 8, 64 * LC_CH);
  return a > b ? a : b;
}

// Quantizer workgroups for npair row pairs with `slots` workgroups per CU: runs of a power
// of two pairs (config 2, 8192 pairs at 7 slots: 1024 workgroups of 8 pairs 71 us, 2048 of 4
// 70.5 us, 1792 of 4-5 pairs 76.6 us; tools/prepass_split.py)
static int lc_grid(int npair, int slots) {
  int ppw = 1;
  while (ppw < cdiv(npair, 256L * slots)) ppw <<= 1;
  return cdiv(npair, ppw);
}

template <class DT, int MODE, int GS, int F8, int NOUT = 1>
static int quant_lc_launch(const void* x, int M, int K, int q_max, int G, const uint32_t* lctab,
                           int Kn, const int32_t* amap, int P, const int32_t* sal, int S,
                           int S_pad, const uint32_t* cmax, const int32_t* nonsal, void* out,
                           uint32_t* key_clear, int clear_words, float* out_scale,
                           void* out_xs, hipStream_t s, int Kq = 0, int ldsc = 0,
                           const LcSib& sib = LcSib{}) {
  typedef typename DT::T T;
  const void* kf = (const void*)quant_lc_kernel<DT, MODE, LC_RPL, GS, F8, NOUT>;
  int nw = lc_waves(K, Kn);
  // F8: every packed position is some thread's (position-order table)
  if (F8 == 1 && cdiv(P, 64 * LC_RPL) > nw) nw = cdiv(P, 64 * LC_RPL);
  if (nw > LC_MAXW) return SQMP_EUNSUPPORTED;
  const size_t lds = sizeof(uint32_t) * lc_lds_words(P, S_pad, NOUT);
  SQMP_HIP_CHECK(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = occ_per_cu(kf, 64 * nw, lds);
  if (const char* e = knob("SQMP_LC_PERCU"))  // tuning only (0 / unparsable: the default)
    if (atoi(e) > 0) per_cu = atoi(e);
  const int npair = (M + 1) / 2;
  int grid = lc_grid(npair, per_cu);
  // the e4m3 output (row-major, no 32-row blocks to keep together): runs of 3 pairs where the
  // pairs exceed one round of slots -- config 2 per_token 46.4 -> 43.3 us against runs of 8
  // (1 / 2 / 4 / 5 / 6 pairs: 46.5 / 47.5 / 43.9 / 44.3 / 45.7 us; profiles/r05_ab_lc_ppw.txt)
  if (F8 == 1 && npair > 256 * per_cu) grid = cdiv(npair, 3);
  if (const char* e = knob("SQMP_LC_PPW"))  // (A/B: exact row pairs per workgroup)
    if (atoi(e) > 0) grid = cdiv(npair, atoi(e));
  quant_lc_kernel<DT, MODE, LC_RPL, GS, F8, NOUT><<<dim3(grid), dim3(64 * nw), lds, s>>>(
      (const T*)x, M, K, q_max, G, lctab, Kn, amap, P, sal, S, S_pad, cmax, nonsal, (T*)out,
      key_clear, clear_words, out_scale, (T*)out_xs, Kq, ldsc, sib);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

bool quant_lc_supported(int dtype, int M, int K, int amode_group, int G, int Kn, int P,
                        int S_pad, const void* x, const void* out) {
  if (dtype != SQMP_F16 && dtype != SQMP_BF16) return false;
  if (M <= 0 || K % 8 != 0 || K > 16384 || Kn > 16384 || P + S_pad >= 65536) return false;
  if (((uintptr_t)x) % 16 != 0 || ((uintptr_t)out) % 16 != 0) return false;
  if ((size_t)4 * lc_lds_words(P, S_pad, 1) > 150 * 1024) return false;
  if (lc_waves(K, Kn) > LC_MAXW) return false;
  if (amode_group) {
    // power-of-two groups that never straddle a wave's 64 * RPL ranks; below RPL only 8
    if (G < 8 || G > 64 * LC_RPL || (G & (G - 1)) != 0) return false;
  }
  return true;
}

int launch_quant_lc(int dtype, int mode, const void* x, int M, int K, int q_max, int G,
                    const uint32_t* lctab, int Kn, const int32_t* amap, int P,
                    const int32_t* sal, int S, int S_pad, const uint32_t* cmax,
                    const int32_t* nonsal, void* out, uint32_t* key_clear, int clear_words,
                    hipStream_t s, float* out_scale, void* out_xs) {
#define SQMP_LC(DTT, MD, GSV, F8V)                                                           \
  quant_lc_launch<DTT, MD, GSV, F8V>(x, M, K, q_max, G, lctab, Kn, amap, P, sal, S, S_pad,   \
                                     cmax, nonsal, out, key_clear, clear_words, out_scale,  \
                                     out_xs, s)
#define SQMP_LC_MODE(DTT)                                                                  \
  (out_scale ? (mode == LC_MODE_TOKEN    ? SQMP_LC(DTT, LC_MODE_TOKEN, 0, 1)               \
                : mode == LC_MODE_TENSOR ? SQMP_LC(DTT, LC_MODE_TENSOR, 0, 1)              \
                                         : SQMP_EUNSUPPORTED)                              \
   : mode == LC_MODE_TOKEN ? SQMP_LC(DTT, LC_MODE_TOKEN, 0, 0)                             \
   : mode == LC_MODE_TENSOR ? SQMP_LC(DTT, LC_MODE_TENSOR, 0, 0)                           \
   : G < LC_RPL ? SQMP_LC(DTT, LC_MODE_GROUP, 8, 0) : SQMP_LC(DTT, LC_MODE_GROUP, 0, 0))
  if (dtype == SQMP_F16) return SQMP_LC_MODE(F16);
  if (dtype == SQMP_BF16) return SQMP_LC_MODE(BF16);
  return SQMP_EUNSUPPORTED;
#undef SQMP_LC_MODE
#undef SQMP_LC
}

// ---- in-place per-token quantization without salient columns (fake_quant.py:56-64 on the
// caller's x: the reference's ppl_eval flow quantizes every linear's input and the q/k/v
// outputs this way): no table, no gather, no LDS row -- a workgroup takes two rows, each thread
// CH 16-B chunks of both, interleaved in registers into (row m0, row m0 + 1) pairs, one
// workgroup-wide packed absmax, then pair_scale / quant_pair (the lane-contiguous quantizer's
// arithmetic, so bit for bit its values) and the chunks stored back over the rows.
// (rows longer than CH chunks per thread: the chunks are streamed twice, max then quantize)
// F8OUT (the FP8 GEMM's operand in the same pass, identity packed order): the e4m3 codes
// [M][K] (bytes, row-major, the OUT_F8 layout) and the fp32 row scales as well.
template <class DT, int CH, bool F8OUT = false>
__global__ __launch_bounds__(1024) void token_rows_kernel(typename DT::T* __restrict__ x, int M,
                                                          int K, float qmf, float rqf,
                                                          unsigned char* __restrict__ codes = nullptr,
                                                          float* __restrict__ oscale = nullptr) {
  __shared__ uint32_t red[LC_MAXW];
  const int nthr = blockDim.x, tid = threadIdx.x, lane = tid & 63, NW = nthr >> 6;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nchk = K >> 3, npair = (M + 1) >> 1;
  const bool cached = nchk <= CH * nthr;
  auto pk_lo = [](uint32_t b, uint32_t a) { return __builtin_amdgcn_perm(b, a, 0x05040100u); };
  auto pk_hi = [](uint32_t b, uint32_t a) { return __builtin_amdgcn_perm(b, a, 0x07060302u); };
  for (int rp = blockIdx.x; rp < npair; rp += gridDim.x) {
    const int m0 = 2 * rp;
    const bool has1 = m0 + 1 < M;
    u32x4* r0 = (u32x4*)(x + (size_t)m0 * K);
    u32x4* r1 = (u32x4*)(x + (size_t)(has1 ? m0 + 1 : m0) * K);
    u32x4 a[CH], b[CH];
    uint32_t mx = 0u;
    for (int c0 = 0; c0 < nchk; c0 += CH * nthr) {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int c = min(c0 + tid + nthr * i, nchk - 1);  // (clamped: unconditional loads)
        a[i] = r0[c];
        b[i] = r1[c];
      }
#pragma unroll
      for (int i = 0; i < CH; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          mx = pk_absmax(pk_absmax(mx, pk_lo(b[i][k], a[i][k])), pk_hi(b[i][k], a[i][k]));
    }
    mx = xor_max(mx, 64);
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    mx = 0u;
    for (int w = 0; w < NW; ++w) mx = pk_absmax(mx, red[w]);
    __syncthreads();  // (red is rewritten by the next pair)
    const PairScale sc = pair_scale<DT>(mx, qmf, rqf);
    if (F8OUT && tid == 0) {
      oscale[m0] = sc.s[0];
      if (has1) oscale[m0 + 1] = sc.s[1];
    }
    for (int c0 = 0; c0 < nchk; c0 += CH * nthr) {
      if (!cached) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int c = min(c0 + tid + nthr * i, nchk - 1);
          a[i] = r0[c];
          b[i] = r1[c];
        }
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int c = c0 + tid + nthr * i;
        if (c >= nchk) continue;
        u32x4 o0, o1;
        uint32_t f[8];  // (F8OUT) the e4m3 code pairs of columns 8c .. 8c + 7
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t wl = pk_lo(b[i][k], a[i][k]), wh = pk_hi(b[i][k], a[i][k]);
          const uint32_t lo = quant_pair<DT>(wl, sc);
          const uint32_t hi = quant_pair<DT>(wh, sc);
          o0[k] = pk_lo(hi, lo);
          o1[k] = pk_hi(hi, lo);
          if (F8OUT) {
            f[2 * k] = f8_pair<DT>(wl, sc);
            f[2 * k + 1] = f8_pair<DT>(wh, sc);
          }
        }
        r0[c] = o0;
        if (has1) r1[c] = o1;
        if (F8OUT) {
          // row m0's codes are byte 0 of each pair word, row m0 + 1's byte 2 (f8_pair)
          u32x2v c0w, c1w;
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            c0w[d] = __builtin_amdgcn_perm(f[4 * d + 1], f[4 * d], 0x0c0c0400u) |
                     __builtin_amdgcn_perm(f[4 * d + 3], f[4 * d + 2], 0x04000c0cu);
            c1w[d] = __builtin_amdgcn_perm(f[4 * d + 1], f[4 * d], 0x0c0c0602u) |
                     __builtin_amdgcn_perm(f[4 * d + 3], f[4 * d + 2], 0x06020c0cu);
          }
          *(u32x2v*)(codes + (size_t)m0 * K + 8 * c) = c0w;
          if (has1) *(u32x2v*)(codes + (size_t)(m0 + 1) * K + 8 * c) = c1w;
        }
      }
    }
  }
}

template <class DT>
static int token_rows_launch(void* x, int M, int K, int q_max, hipStream_t s,
                             unsigned char* codes = nullptr, float* oscale = nullptr) {
  const int nchk = K / 8;
  const int ch = nchk <= 2048 ? 2 : 4;
  const int nthr = (int)min(1024L, round_up(cdiv(nchk, ch), 64));
  const int npair = (M + 1) / 2;
  const dim3 grid(npair < 65536 ? npair : 65536), block(nthr < 64 ? 64 : nthr);
  const float qmf = (float)q_max, rqf = 1.0f / qmf;
  typedef typename DT::T T;
  if (codes) {
    if (ch == 2)
      token_rows_kernel<DT, 2, true><<<grid, block, 0, s>>>((T*)x, M, K, qmf, rqf, codes, oscale);
    else
      token_rows_kernel<DT, 4, true><<<grid, block, 0, s>>>((T*)x, M, K, qmf, rqf, codes, oscale);
  } else if (ch == 2) {
    token_rows_kernel<DT, 2><<<grid, block, 0, s>>>((T*)x, M, K, qmf, rqf);
  } else {
    token_rows_kernel<DT, 4><<<grid, block, 0, s>>>((T*)x, M, K, qmf, rqf);
  }
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

int launch_token_rows(int dtype, void* x, int M, int K, int q_max, hipStream_t s,
                      unsigned char* codes, float* oscale) {
  if (M <= 0 || K <= 0 || K % 8 != 0 || ((uintptr_t)x) % 16 != 0) return SQMP_EUNSUPPORTED;
  if (codes && (!oscale || ((uintptr_t)codes) % 8 != 0 || q_max > 7)) return SQMP_EUNSUPPORTED;
  if (dtype == SQMP_F16) return token_rows_launch<F16>(x, M, K, q_max, s, codes, oscale);
  if (dtype == SQMP_BF16) return token_rows_launch<BF16>(x, M, K, q_max, s, codes, oscale);
  return SQMP_EUNSUPPORTED;
}

// The OUT_FP quantizer for a layer and up to two siblings (sqmp_quant_act_group): group mode,
// groups of >= LC_RPL ranks; out[0] in the packed order of lctab, sib.out[o] in sib.tab[o]'s.
int launch_quant_lc_group(int dtype, const void* x, int M, int K, int q_max, int G,
                          const uint32_t* lctab, int Kn, const int32_t* amap, int P,
                          const int32_t* sal, int S, int S_pad, const uint32_t* cmax,
                          const int32_t* nonsal, void* out, uint32_t* key_clear, int clear_words,
                          const LcSib& sib, hipStream_t s) {
  if (G < LC_RPL || sib.n < 0 || sib.n > 2) return SQMP_EUNSUPPORTED;
  // one LDS region of P + S_pad + 8 words per output (+ the salient list)
  if ((size_t)4 * lc_lds_words(P, S_pad, sib.n + 1) > 150 * 1024) return SQMP_EUNSUPPORTED;
#define SQMP_LCG(DTT, NO)                                                                     \
  quant_lc_launch<DTT, LC_MODE_GROUP, 0, 0, NO>(x, M, K, q_max, G, lctab, Kn, amap, P, sal, S, \
                                               S_pad, cmax, nonsal, out, key_clear,            \
                                               clear_words, nullptr, nullptr, s, 0, 0, sib)
#define SQMP_LCG_N(DTT) (sib.n == 0 ? SQMP_LCG(DTT, 1) : sib.n == 1 ? SQMP_LCG(DTT, 2) : SQMP_LCG(DTT, 3))
  if (dtype == SQMP_F16) return SQMP_LCG_N(F16);
  if (dtype == SQMP_BF16) return SQMP_LCG_N(BF16);
  return SQMP_EUNSUPPORTED;
#undef SQMP_LCG_N
#undef SQMP_LCG
}

static int pw_rows(int Kp) {
  // rows per permutation batch: 16 KiB of dequantized rows; Np % 256 == 0, so RB | Np
  const char* e = knob("SQMP_PW_RB");  // tuning only (sqmp_knobs.hip)
  const int env = e ? atoi(e) : 0;
  int rb = env > 0 ? env : 16384 / (Kp * 2);
  return rb >= 8 ? 8 : rb >= 4 ? 4 : rb >= 2 ? 2 : 1;
}

int launch_perm_weight_c4(int dtype, const uint32_t* lctab, const void* codes,
                          const void* wscale, const void* wsal, int N, int Kp, int Gw, int ngw,
                          int Kn, int S_pad, void* wp, hipStream_t s) {
  const int Np = pad_n(N), RB = pw_rows(Kp);
  const int Kq = (int)round_up(Kn, 64);
  PermArgs pa{(const uint32_t*)codes, wscale, wsal, wp, N, Np, Kp, Gw, ngw, Kn, Kq, S_pad, RB};
  const size_t lds = (size_t)RB * Kp * 2;
  const dim3 grid((unsigned)(Np / RB));
  if (dtype == SQMP_F16) {
    SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)perm_weight_kernel<F16>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    perm_weight_kernel<F16><<<grid, dim3(256), lds, s>>>(pa, lctab);
  } else if (dtype == SQMP_BF16) {
    SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)perm_weight_kernel<BF16>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    perm_weight_kernel<BF16><<<grid, dim3(256), lds, s>>>(pa, lctab);
  } else {
    return SQMP_EUNSUPPORTED;
  }
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

int launch_quant_lc_c4(int dtype, const void* x, int M, int K, int q_max, int G,
                       const uint32_t* lctab, int Kn, int P, const int32_t* sal, int S,
                       int S_pad, const uint32_t* cmax, const int32_t* nonsal, void* codes,
                       void* scales, int ldsc, void* xs, uint32_t* key_clear, int clear_words,
                       hipStream_t s, const C4Weight* cw) {
  const int Kq = (int)round_up(Kn, 64);
  if (G < LC_RPL) return SQMP_EUNSUPPORTED;
  if (!cw) {
    if (dtype == SQMP_F16)
      return quant_lc_launch<F16, LC_MODE_GROUP, 0, 3>(x, M, K, q_max, G, lctab, Kn, nullptr, P,
                                                       sal, S, S_pad, cmax, nonsal, codes,
                                                       key_clear, clear_words, (float*)scales, xs,
                                                       s, Kq, ldsc);
    if (dtype == SQMP_BF16)
      return quant_lc_launch<BF16, LC_MODE_GROUP, 0, 3>(x, M, K, q_max, G, lctab, Kn, nullptr, P,
                                                        sal, S, S_pad, cmax, nonsal, codes,
                                                        key_clear, clear_words, (float*)scales,
                                                        xs, s, Kq, ldsc);
    return SQMP_EUNSUPPORTED;
  }
  // fused: the quantizer's grid (as quant_lc_launch) + Np / RB permutation workgroups
  const int nw = lc_waves(K, Kn);
  const int Np = pad_n(cw->N), RB = pw_rows(cw->Kp);
  PermArgs pa{(const uint32_t*)cw->codes, cw->wscale, cw->wsal, cw->wp, cw->N, Np, cw->Kp,
              cw->Gw, cw->ngw, Kn, Kq, S_pad, RB};
  const int Nrows = Np;  // the permutation's rows
  const size_t lq = sizeof(uint32_t) * lc_lds_words(P, S_pad, 1), lp = (size_t)RB * cw->Kp * 2;
  const size_t lds = lq > lp ? lq : lp;
  const void* kf = dtype == SQMP_BF16 ? (const void*)quant_c4_fused_kernel<BF16>
                                       : (const void*)quant_c4_fused_kernel<F16>;
  const int per_cu = occ_per_cu(kf, 64 * nw, lds);
  // quantizer workgroups per CU: the rest of every CU's slots go to the permutation
  // workgroups (issued after them), so the two run side by side
  const char* qe = knob("SQMP_C4_QPERCU");  // tuning only (sqmp_knobs.hip)
  const int q_env = qe ? atoi(qe) : 0;
  const int qpc = q_env > 0 ? q_env : (per_cu > 2 ? per_cu - 2 : 1);
  int nq = lc_grid((M + 1) / 2, qpc < per_cu ? qpc : per_cu);
  if (const char* e = knob("SQMP_LC_PPW"))  // (A/B: exact row pairs per quantizer workgroup)
    if (atoi(e) > 0) nq = cdiv((M + 1) / 2, atoi(e));
  const dim3 grid(nq + Nrows / RB), block(64 * nw);
  if (dtype == SQMP_F16) {
    SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)quant_c4_fused_kernel<F16>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    quant_c4_fused_kernel<F16><<<grid, block, lds, s>>>(
        (const _Float16*)x, M, K, q_max, G, lctab, Kn, P, sal, S, S_pad, cmax, nonsal, codes,
        key_clear, clear_words, scales, (_Float16*)xs, Kq, ldsc, nq, pa);
  } else if (dtype == SQMP_BF16) {
    SQMP_HIP_CHECK(hipFuncSetAttribute((const void*)quant_c4_fused_kernel<BF16>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    quant_c4_fused_kernel<BF16><<<grid, block, lds, s>>>(
        (const __bf16*)x, M, K, q_max, G, lctab, Kn, P, sal, S, S_pad, cmax, nonsal, codes,
        key_clear, clear_words, scales, (__bf16*)xs, Kq, ldsc, nq, pa);
  } else {
    return SQMP_EUNSUPPORTED;
  }
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace sqmp

#ifdef SQMP_DIAG_BUILD
// the quantizer's timing stamps of the last launch (diagnostics build only)
// (host == NULL: clear them)
extern "C" int sqmp_diag_lc_stamps(unsigned long long* host, int nblk) {
  if (nblk > 8192) nblk = 8192;
  if (!host) {
    void* d = nullptr;
    if (hipGetSymbolAddress(&d, HIP_SYMBOL(sqmp::sqmp_lc_stamps)) != hipSuccess) return -3;
    return hipMemset(d, 0, sizeof(unsigned long long) * 8 * 8192) == hipSuccess ? 0 : -3;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(sqmp::sqmp_lc_stamps), sizeof(unsigned long long) * 8 * nblk, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
#endif
