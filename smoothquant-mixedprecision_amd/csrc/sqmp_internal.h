// Internal (non-ABI) launchers shared between the translation units of libsqmp_w4a4.so.
#pragma once
#include <stdlib.h>

#include "sqmp_common.h"

namespace sqmp {

// The value of launch knob `name` (an SQMP_* environment variable, read once at library load
// and again by sqmp_reload_knobs; sqmp_knobs.hip), or NULL when unset.
const char* knob(const char* name);

// Whether a GEMM stores its output with non-temporal (streaming) stores.  An output larger
// than a quarter of the 256-MiB Infinity Cache left dirty there is written back to HBM during
// the kernels that follow -- at config 2 the next forward's prepass, which then shares HBM
// with 134 MB of write-back.  Same-box step A/B (GEMM time unchanged;
// profiles/r03_step_ab_nt.txt): per_group 523.1 -> 502.3 us, per_token 359.9 -> 351.2 us,
// fp32 2068 -> 2044 us.  Smaller outputs stay cached for their consumer.
// SQMP_NT_STORES = 0 / 1 forces it off / on.
inline bool nt_output(size_t bytes) {
  if (const char* e = knob("SQMP_NT_STORES")) return atoi(e) != 0;
  return bytes >= ((size_t)64 << 20);
}

// The two-piece fp16 form of fp32 values (sqmp_gemm_h2 / _h2d, the fp32 quantizer's
// SQMP_OUT_H2 mode): rows scaled by 2^e so that their maximum lies in [2^13, 2^14), then
// v (|v| < 2^14) -> (h, l) f16 bit patterns, h = f16(v), l = f16(v - h): v - h is exact in
// fp32 and l keeps its 11 leading bits, so |v - h - l| <= 2^-22 |v| (+ the f16 subnormal
// floor 2^-25)
__device__ inline void split2h(float v, uint32_t& h, uint32_t& l) {
  const _Float16 hh = (_Float16)v;
  const _Float16 ll = (_Float16)(v - (float)hh);
  h = (uint32_t)(*(const uint16_t*)&hh);
  l = (uint32_t)(*(const uint16_t*)&ll);
}

// the exponent e with max |row| * 2^e in [2^13, 2^14) (0 for an all-zero row)
__device__ inline int row_exp_of(float mx) {
  // floor(log2 mx) from the exponent field (a subnormal mx counts as 2^-127: the scaled
  // maximum then stays below 2^14 all the same)
  return mx > 0.f ? 13 - ((int)((__float_as_uint(mx) >> 23) & 0xFFu) - 127) : 0;
}

// 8 consecutive fp32 values of a row with exponent e -> 16 B of each plane at p (the l plane
// `hplane` halves further)
__device__ inline void store_h2x8(uint16_t* p, size_t hplane, const float* r, int e) {
  uint32_t h[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) split2h(__builtin_ldexpf(r[j], e), h[j], l[j]);
  *(u32x4*)p = u32x4{h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16)};
  *(u32x4*)(p + hplane) =
      u32x4{l[0] | (l[1] << 16), l[2] | (l[3] << 16), l[4] | (l[5] << 16), l[6] | (l[7] << 16)};
}

// cmax[c] = bits(max_r |x[r][c]|) over a contiguous D matrix [R][C] (fp32 bits of the
// D value; non-negative floats order like their bit patterns).  Zeroes cmax first.
int launch_colmax(const void* x, int dtype, int R, int C, uint32_t* cmax, hipStream_t s,
                  bool zero = true);  // zero: clear cmax first (else the caller did)

// key[c] = bits(fp32(mean|x| + 3 std|x|)) over the R rows (the mean + 3 sigma sort key);
// `sums` is a 2*C fp64 scratch (cleared here).
// clean: `sums` is zero on entry (no memset) and is left zero.
int launch_colkey_mean3std(const void* x, int dtype, int R, int C, double* sums,
                           uint32_t* key, hipStream_t s, bool clean = false);
// counts[cols[i]] += stable rank of list entry i (counts zero on entry).
int launch_rank_count(const uint32_t* cmax, const int32_t* cols, int L, int32_t* counts,
                      hipStream_t s);

// Stable ascending rank of the list cols[0..L) (NULL = identity) keyed by cmax[col]:
// rank_by_col[cols[i]] = #{j : (cmax[cols[j]], j) < (cmax[cols[i]], i)}.  Zeroes the
// C-entry rank_by_col first.
int launch_rank(const uint32_t* cmax, const int32_t* cols, int L, int C,
                int32_t* rank_by_col, hipStream_t s, bool zero = true);
// Atomic-free variant: part[tile][i] = competitors of tile `tile` ordered before list
// entry i (tiles of 256); rank(i) = sum over the rank_tiles(L) tiles.  ld = row stride.
int rank_tiles(int L);
int launch_rank_partial(const uint32_t* cmax, const int32_t* cols, int L, int ld,
                        int32_t* part, hipStream_t s);

// Index maps of a packed weight (see include/sqmp_w4a4.h).  rank_by_col == NULL keeps the
// original column order (per_channel / per_tensor / unsorted per_group).
int launch_build_maps(int K, int Kp, const int32_t* rank_by_col, const int32_t* salient,
                      int S, int32_t* perm, int32_t* amap, int32_t* amap_fq,
                      int32_t* nonsal, hipStream_t s);

// Sibling layers of one input (q/k/v, gate/up: same K, salient set and act mode, each in its
// own packed order): the rank-table kernel also writes their rank-ordered tables
// lctab[o][r] = column | posmap[o][column] << 16 (padding ranks: the (zero, sink) entry).
struct SibTables {
  int n = 0;
  const int32_t* posmap[2] = {nullptr, nullptr};
  uint32_t* lctab[2] = {nullptr, nullptr};
};
// ... and the lane-contiguous quantizer writes their OUT_FP operands from the same pass:
// out[o] in the packed order of table tab[o], zeros at the positions amap[o] marks < 0.
struct LcSib {
  int n = 0;
  const uint32_t* tab[2] = {nullptr, nullptr};
  const int32_t* amap[2] = {nullptr, nullptr};
  void* out[2] = {nullptr, nullptr};
};

// Lane-contiguous OUT_FP quantizer (sqmp_actquant_lc.hip).  mode: 0 token, 1 tensor,
// 2 group (any rank order: sorted / unsorted / mean3std -- lctab carries it).
bool quant_lc_supported(int dtype, int M, int K, int amode_group, int G, int Kn, int P,
                        int S_pad, const void* x, const void* out);
// in-place per-token quantization of [M][K] rows without salient columns (f16 / bf16, K % 8 == 0,
// 16-B aligned; else SQMP_EUNSUPPORTED)
// codes / oscale (optional): also the e4m3 codes [M][K] and fp32 row scales of SQMP_OUT_F8
int launch_token_rows(int dtype, void* x, int M, int K, int q_max, hipStream_t s,
                      unsigned char* codes = nullptr, float* oscale = nullptr);
int launch_quant_lc(int dtype, int mode, const void* x, int M, int K, int q_max, int G,
                    const uint32_t* lctab, int Kn, const int32_t* amap, int P,
                    const int32_t* sal, int S, int S_pad, const uint32_t* cmax,
                    const int32_t* nonsal, void* out, uint32_t* key_clear, int clear_words,
                    hipStream_t s, float* out_scale = nullptr, void* out_xs = nullptr);
// key_clear: zeroed (clear_words % 4 == 0), may be NULL.  out_scale != NULL selects the
// e4m3 code output (token / tensor modes): out = codes [M][P], out_xs = D [M][S_pad].
// group mode with up to two sibling outputs (sib.n), fp16 / bf16, G >= 16
int launch_quant_lc_group(int dtype, const void* x, int M, int K, int q_max, int G,
                          const uint32_t* lctab, int Kn, const int32_t* amap, int P,
                          const int32_t* sal, int S, int S_pad, const uint32_t* cmax,
                          const int32_t* nonsal, void* out, uint32_t* key_clear, int clear_words,
                          const LcSib& sib, hipStream_t s);

// SQMP_OUT_C4 lane-contiguous quantizer (act-order int4 codes, group scales [Kq/G][ldsc],
// exact salient columns); P = the table's packed length (Kp).  cw != NULL: the same launch
// also builds the activation-order weight operand (sqmp_quant_act_c4).
struct C4Weight {
  const void* codes;   // bpack [pad_n(N)][Kp/2]
  const void* wscale;  // D [ngw][pad_n(N)]
  const void* wsal;    // D [N][S_pad]
  void* wp;            // D [pad_n(N)][Kq + S_pad]
  int N, Kp, Gw, ngw;
};
int launch_quant_lc_c4(int dtype, const void* x, int M, int K, int q_max, int G,
                       const uint32_t* lctab, int Kn, int P, const int32_t* sal, int S,
                       int S_pad, const uint32_t* cmax, const int32_t* nonsal, void* codes,
                       void* scales, int ldsc, void* xs, uint32_t* key_clear, int clear_words,
                       hipStream_t s, const C4Weight* cw = nullptr);
int launch_perm_weight_c4(int dtype, const uint32_t* lctab, const void* codes,
                          const void* wscale, const void* wsal, int N, int Kp, int Gw, int ngw,
                          int Kn, int S_pad, void* wp, hipStream_t s);

// Fast GEMMs (sqmp_gemm_fast.hip); SQMP_EUNSUPPORTED when the shape has no fast kernel.
// colmax != NULL: the epilogue also atomic-maxes bits(max |y|) per output column into it
int launch_gemm_fq_fast(int dtype, const void* a, const void* codes, const void* wscale,
                        const void* wsal, const void* bias, void* y, int M, int N, int Kp,
                        int S_pad, int Gw, int ngw, int n_bits, uint32_t* colmax,
                        hipStream_t s);
// activation-order GEMM (sqmp_gemm_fqt): y^T = wp . codes^T on gemm_fq6<TR>
int launch_gemm_fqt(int dtype, const void* acodes, const void* ascale, const void* xs,
                    const void* wp, const void* bias, void* y, int M, int N, int Kq, int S_pad,
                    int G, int ngq, hipStream_t s);

}  // namespace sqmp
