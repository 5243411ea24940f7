/*
 * sqmp_w4a4.h -- C ABI of the MI355X-native W4A4 mixed-precision linear operator.
 *
 * Drop-in boundary for the hot path of adithyab100/smoothquant-mixedprecision:
 *   W4A4Linear.from_float  (/root/reference/smoothquant/fake_quant.py:324-371)
 *   W4A4Linear.forward     (/root/reference/smoothquant/fake_quant.py:279-322)
 * The reference is pure Python (no FFI); these entry points replace the ATen calls that
 * its forward and from_float make, and are bound from Python with ctypes by
 * smoothquant-mixedprecision_amd/smoothquant/_lib.py.
 *
 * Conventions
 *   - Plain C: device pointers, sizes, and a hipStream_t passed as `void*` (NULL = the
 *     default stream).  Nothing is allocated; the caller owns every buffer, including the
 *     workspace (size from the *_workspace_bytes queries).  No host synchronisation, so
 *     every launch function may be captured into a hipGraph.
 *   - Return value: SQMP_OK (0) or a negative status.  The Python layer maps
 *     SQMP_EINVAL/SQMP_EUNSUPPORTED to ValueError (the reference's error type for bad
 *     modes, fake_quant.py:256, :287, :361) and SQMP_EHIP/SQMP_EWORKSPACE to RuntimeError.
 *   - dtype codes: model dtype D of x, W, bias, y (fp32 / fp16 / bf16).  All scale and
 *     dequantized values are exact D values (rounded at the same points as the reference).
 *
 * Packed weight layout (produced by sqmp_pack_weight, consumed by the GEMMs)
 *   Kp        packed K length: weight groups in weight-sorted column order, zero padded
 *             (multiple of 128).  Position p < K holds original column perm[p].
 *   Np        = roundup(N, 256): codes are allocated with Np rows (rows >= N are never
 *             stored to y) and wscale rows have stride Np.
 *   codes     4-bit weights: "bpack", uint8 [Np][Kp/2].  Per row, per 64-position block,
 *             8 dwords; dword (h*4 + u) holds the 8 codes of positions 16u + 8h + e
 *             (e = 0..7): even e in nibble e/2 of the low half-word, odd e in nibble e/2
 *             of the high half-word; nibble = code + 8 (code in [-7, 7]).  A 16-byte half
 *             h is one 32x32x16 lane half's four sub-step fragments; dwords 2q, 2q+1 are
 *             one 16x16x32 lane group's two sub-steps (and its 16x16x64 i8 fragment).
 *             8-bit weights: int8 [N][Kp] row-major.  Salient columns and padding hold 0.
 *   wscale    D [ngw][Np]: per-(group, row) scale; group of position p is p / Gw.
 *   wsal      D [N][S_pad]: the salient weight columns, exact (fake_quant.py:363-365),
 *             in salient_indices order, zero padded to S_pad (multiple of 64).
 *   perm      int32 [Kp]: original column at packed position p, -1 for padding.
 *   amap      int32 [Kp]: perm with salient columns replaced by -1 (GEMM A-operand map).
 *   amap_fq   int32 [K]:  k, or -2 for salient k (in-place output-quant map).
 *   nonsal    int32 [K-S]: non-salient columns, ascending (the x[:, mask] order).
 */
#ifndef SQMP_W4A4_H
#define SQMP_W4A4_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SQMP_OK 0
#define SQMP_EINVAL (-1)
#define SQMP_EUNSUPPORTED (-2)
#define SQMP_EHIP (-3)
#define SQMP_EWORKSPACE (-4)

enum sqmp_dtype { SQMP_F32 = 0, SQMP_F16 = 1, SQMP_BF16 = 2 };

/* act_quant (fake_quant.py:246-256); PER_GROUP is the sorted variant the reference
 * binds (:104-154); PER_GROUP_UNSORTED is the unwired :77-101 variant;
 * PER_GROUP_MEAN3STD sorts the columns by mean|x| + 3 std|x| over the batch instead of
 * the column absmax (the README.md:36 "statistical sorting", absent from the reference's
 * code -- defined by this library, parity unpinned). */
enum sqmp_act_mode {
  SQMP_ACT_PER_TOKEN = 0,
  SQMP_ACT_PER_TENSOR = 1,
  SQMP_ACT_PER_GROUP = 2,
  SQMP_ACT_PER_GROUP_UNSORTED = 3,
  SQMP_ACT_PER_GROUP_MEAN3STD = 4
};

/* weight_quant (fake_quant.py:348-361); PER_GROUP = sorted (:156-207). */
enum sqmp_weight_mode {
  SQMP_W_PER_CHANNEL = 0,
  SQMP_W_PER_TENSOR = 1,
  SQMP_W_PER_GROUP = 2,
  SQMP_W_PER_GROUP_UNSORTED = 3,
  SQMP_W_NONE = 4,  /* no weight quantization: `codes` holds dense D [N][Kp] (a directly
                       constructed W4A4Linear, fake_quant.py:227-235); GEMM n_bits = 0 */
  SQMP_W_PER_GROUP_MEAN3STD = 5  /* groups over columns sorted by mean|W| + 3 std|W| over
                                    the N rows (see SQMP_ACT_PER_GROUP_MEAN3STD) */
};

/* Output of sqmp_quant_act. */
enum sqmp_act_out {
  SQMP_OUT_FP = 0,      /* out: D [M][Kp + S_pad]: x_hat at packed positions, exact
                           salient x in the tail (operand of sqmp_gemm_fq) */
  /* 1: reserved (the int8-code output of the removed integer GEMM, ABI < 0.6) */
  SQMP_OUT_INPLACE = 2, /* fake-quantize `x` in place through amap_fq (output quant,
                           fake_quant.py:308-316) */
  SQMP_OUT_F8 = 3,      /* per_token / per_tensor, n_bits <= 4, sqmp_quant_act_v2 with
                           posmap only: out = OCP e4m3 integer codes [M][Kp] (bytes) in
                           packed order (0 at salient / padding positions); out_scale: fp32
                           [M] (the D scale); out_xs: D [M][S_pad] exact salient x
                           (operands of sqmp_gemm_f8) */
  /* 4: reserved (the removed FP6 code output) */
  SQMP_OUT_C4 = 5,      /* per_group activations in ACTIVATION order (operands of
                           sqmp_gemm_fqt): out = int4 codes [roundup(M, 256)][Kq / 2] bytes,
                           Kq = roundup(K - S, 64), bpack rows whose position j is the
                           column of activation rank j (zeros past K - S); out_scale = the D
                           group scales [Kq / group_size][roundup(M, 256)]; out_xs = the
                           exact salient columns [M][S_pad].  4-bit, group_size % 64 == 0,
                           fp16/bf16, posmap required. */
  SQMP_OUT_H2 = 6       /* fp32 layers: the SQMP_OUT_FP values as the two f16 planes of
                           sqmp_gemm_h2d -- out = f16 [2][roundup(M, 128)][Kp + S_pad] (rows
                           scaled by 2^aexp[m], split h + l), out_scale = int32 aexp [M];
                           bit-identical to SQMP_OUT_FP + sqmp_split2_f16.  The fp32 wave
                           quantizers only (act per_token / per_group, K % 8 == 0, posmap):
                           SQMP_EUNSUPPORTED elsewhere. */
};

/* Library identity. */
const char* sqmp_version(void);
const char* sqmp_status_string(int status);

/* Host-only geometry of a packed weight (no GPU work).
 * Replaces the implicit shapes of fake_quant.py:156-207 / :347-365. */
int sqmp_weight_geometry(int K, int S, int wmode, int group_size, int* Kp, int* Gw,
                         int* ngw, int* S_pad);

size_t sqmp_pack_workspace_bytes(int N, int K);
size_t sqmp_act_workspace_bytes(int M, int K, int Kp);  /* Kp: packed length (K for INPLACE) */

/* Offline weight quantization + packing: W4A4Linear.from_float (fake_quant.py:324-371)
 * with quantize_weight_per_{channel,tensor}_absmax (:9-26), quantize_weight_per_group_
 * absmax[_sort] (:29-53, :156-207) and the salient-column restore (:347, :363-365).
 * `salient` (device int32 [S]) may be NULL when S == 0. */
int sqmp_pack_weight(const void* w, int dtype, int N, int K, int wmode, int n_bits,
                     int group_size, const int32_t* salient, int S, void* codes,
                     void* wscale, void* wsal, int32_t* perm, int32_t* amap,
                     int32_t* amap_fq, int32_t* nonsal, void* workspace, size_t ws_bytes,
                     void* stream);

/* The reference's dequantized `weight` buffer W_hat [N][K] in D (fake_quant.py:357-365). */
int sqmp_dequant_weight(const void* codes, const void* wscale, const void* wsal,
                        const int32_t* amap, const int32_t* salient, int dtype, int N,
                        int K, int S, int n_bits, int Kp, int Gw, int ngw, int S_pad,
                        void* w_hat, void* stream);

/* W_hat in PACKED order, D [N][Kp] (salient and padding positions 0): the dense B operand
 * (GEMM n_bits = 0) for group sizes finer than one 16-byte chunk of D (e.g. 4). */
int sqmp_dequant_weight_packed(const void* codes, const void* wscale, int dtype, int N,
                               int Kp, int Gw, int ngw, int n_bits, void* out, void* stream);

/* Index maps for the identity column order (activation-only quantizers: the reference's
 * quantize_activation_* primitives called directly, fake_quant.py:56-154). */
int sqmp_build_maps(int K, const int32_t* salient, int S, int32_t* perm, int32_t* amap,
                    int32_t* amap_fq, int32_t* nonsal, int Kp, void* stream);

/* Runtime activation quantization: the pre-GEMM half of W4A4Linear.forward
 * (fake_quant.py:291-304) with the bound act quantizer (:56-75, :77-101, :104-154).
 * x: D [M][K] contiguous.  `amap` is the packed map (SQMP_OUT_FP / _I8, length Kp) or
 * amap_fq (SQMP_OUT_INPLACE, length K).  `nonsal` lists the K-S columns the batch
 * statistics run over. */
int sqmp_quant_act(void* x, int dtype, int M, int K, int amode, int n_bits,
                   int group_size, const int32_t* amap, int Kp, const int32_t* nonsal,
                   const int32_t* salient, int S, int S_pad, int out_kind, void* out,
                   void* out_scale, void* out_xs, void* workspace, size_t ws_bytes,
                   void* stream);

/* sqmp_quant_act_v2 flags. */
#define SQMP_QA_CLEAN_WS 1    /* the workspace's statistics regions are zero on entry (a
                                 persistent workspace, first allocated zeroed); the call
                                 leaves them zero again, so no per-call memset is needed */
#define SQMP_QA_REUSE_STATS 2 /* the workspace still holds the sorted column order of THIS
                                 batch x and non-salient list (a previous call on the same
                                 input, e.g. q/k/v or gate/up sharing x): skip the column
                                 statistics and the rank (sorted per_group modes only) */
#define SQMP_QA_STATS_GIVEN 4 /* SQMP_OUT_INPLACE, act per_group (sorted) or per_tensor:
                                 the workspace's column-maximum region (its first K words:
                                 fp32 bits of max_m |x[m][k]|) was filled by the producer of
                                 x -- sqmp_gemm_fq_colmax's epilogue -- so the column
                                 statistics pass is skipped (output quantization fused into
                                 the GEMM epilogue, fake_quant.py:308-316) */
#define SQMP_QA_TILED 8       /* SQMP_OUT_C4: codes, group scales and salient x written in the
                                 tile-major layouts of sqmp_gemm_fqt7 (sqmp_fq7_sizes with
                                 J = 2 and N = M gives their sizes) instead of row-major */
#define SQMP_QA_TILED4 16     /* as SQMP_QA_TILED with 64-row blocks (J = 4), the operands of
                                 sqmp_gemm_fqt7j with J = 4 */
#define SQMP_QA_TABLE_READY 32 /* unsorted act modes (per_token, per_group_unsorted) on the
                                 lane-contiguous quantizer: the workspace's rank table already
                                 holds exactly the list table this call would build (a previous
                                 call on this workspace with the same K, non-salient list,
                                 salient set and position map, e.g. the in-place quantizers of
                                 consecutive layers without salient channels): its build launch
                                 is skipped.  Ignored by the sorted modes. */
#define SQMP_QA_WRITE_X 64    /* SQMP_OUT_F8, per_token, no salient column, identity packed
                                 order (Kp == K), f16 / bf16 rows with K % 8 == 0 and 16-B
                                 alignment: x_hat is also written over x in the same pass (the
                                 reference's in-place act quantization of the caller's input,
                                 fake_quant.py:56-64 via :304); else SQMP_EUNSUPPORTED */

/* sqmp_quant_act with the per-weight map posmap (int32 [K]: packed position of column k,
 * the inverse of perm; NULL = derive it per call) and flags.  With posmap, OUT_FP on
 * fp16/bf16 runs column statistics -> rank -> table -> the lane-contiguous quantizer. */
int sqmp_quant_act_v2(void* x, int dtype, int M, int K, int amode, int n_bits,
                      int group_size, const int32_t* amap, int Kp, const int32_t* nonsal,
                      const int32_t* salient, int S, int S_pad, const int32_t* posmap,
                      int flags, int out_kind, void* out, void* out_scale, void* out_xs,
                      void* workspace, size_t ws_bytes, void* stream);

/* GEMM operand allocation rule: the activation operands (a / a8 / xs) are read in whole
 * 256-row tiles by LDS-DMA, so their allocations must hold roundup(M, 256) rows (rows
 * >= M may hold anything; they never reach y).  a8 rows are roundup(Kp, 256) bytes.
 *
 * Faithful GEMM: y[M][N] = D( A[M][Kp+S_pad] . B^T + bias ), B decoded in-kernel from
 * the int4/int8 codes as D(code * wscale) (bit-exact W_hat) for p < Kp and taken from
 * wsal for the salient tail; D-MFMA with fp32 accumulation (fake_quant.py:306).
 * n_bits = 4 / 8: codes are packed codes (group size a multiple of 8 elements, 4 for
 * fp32); n_bits = 0: `codes` is a dense D [N][Kp] operand (SQMP_W_NONE or the output of
 * sqmp_dequant_weight_packed), wscale unused. */
int sqmp_gemm_fq(const void* a, const void* codes, const void* wscale, const void* wsal,
                 const void* bias, void* y, int dtype, int M, int N, int Kp, int S_pad,
                 int Gw, int ngw, int n_bits, void* stream);

/* sqmp_gemm_fq whose epilogue also folds the column maxima of the stored output into
 * colmax[N]: colmax[n] = max(colmax[n], bits(fp32 max_m |y[m][n]|)) by atomic max (the
 * values are those of y after the rounding to D).  colmax = NULL is sqmp_gemm_fq.  Feeds
 * the in-place output quantizer (sqmp_quant_act_v2 + SQMP_QA_STATS_GIVEN): the reference's
 * output quantization (fake_quant.py:308-316) without a statistics pass over y. */
int sqmp_gemm_fq_colmax(const void* a, const void* codes, const void* wscale,
                        const void* wsal, const void* bias, void* y, int dtype, int M, int N,
                        int Kp, int S_pad, int Gw, int ngw, int n_bits, uint32_t* colmax,
                        void* stream);

/* e4m3 operands of sqmp_gemm_f8 from a packed 4-bit weight: w8 = the int4 codes as OCP
 * e4m3 bytes [Np][Kp] in packed order, ws32 = the D group scales as fp32 [ngw][Np]
 * (Np = roundup(N, 256)).  Once per layer.  w8 = NULL builds the scales only. */
int sqmp_pack_f8(const void* codes, const void* wscale, int dtype, int N, int Kp, int ngw,
                 void* w8, float* ws32, void* stream);

/* Low-precision GEMM for per_token / per_tensor activations with 4-bit codes (operands of
 * SQMP_OUT_F8 and sqmp_pack_f8): e4m3 codes x e4m3 codes on the block-scaled FP8 MFMA
 * (exact integer block sums in fp32), per-weight-group fold, per-row act scale, exact
 * salient tail on the D MFMA, bias, one rounding to D.  Gw % 64 == 0, fp16/bf16.
 * a8 and xs: roundup(M, 256) rows allocated (operand allocation rule above). */
int sqmp_gemm_f8(const void* a8, const float* ascale, const void* xs, const void* w8,
                 const float* ws32, const void* wsal, const void* bias, void* y, int dtype,
                 int M, int N, int Kp, int S_pad, int Gw, int ngw, void* stream);

/* sqmp_gemm_f8 with the output quantizer's column statistics fused into its epilogue, as
 * sqmp_gemm_fq_colmax: colmax[n] = max(colmax[n], bits(|y[m][n]|)) over every row m
 * (fake_quant.py:308-316 then skips its statistics pass: SQMP_QA_STATS_GIVEN).
 * Gw % 128 == 0 (the 16x16x128 kernel). */
int sqmp_gemm_f8_colmax(const void* a8, const float* ascale, const void* xs, const void* w8,
                        const float* ws32, const void* wsal, const void* bias, void* y,
                        int dtype, int M, int N, int Kp, int S_pad, int Gw, int ngw,
                        uint32_t* colmax, void* stream);

/* Register-operand copy of a packed 4-bit weight for sqmp_gemm_fq7 (same values, tile-major
 * order; once per layer), for J (2 or 4) 16-row weight tiles per wave (WR = 16 J rows per
 * block).  Sizes from sqmp_fq7_sizes: codes_t bytes = R * Kp / 2, scale_t elements (D) =
 * R * ngw, sal_t elements (D) = R * max(S_pad, 64), R = roundup(N, 128 J).
 *   codes_t[n/WR][Kp/64][lane][j][s] dwords = bpack dword 2q + s (q = lane >> 4) of the
 *     64-position block of row WR (n/WR) + 16 j + (lane & 15);
 *   scale_t[n/WR][g][r][j] = wscale[g][WR (n/WR) + 16 j + r];
 *   sal_t[n/WR][S_pad/64][lane][j][s][e] = wsal[WR (n/WR) + 16 j + (lane & 15)]
 *     [64 kd + 8 (4 (q & 1) + 2 s + (q >> 1)) + e]  (the GEMM's fragment chunk order).
 * Rows >= N are zero. */
int sqmp_fq7_sizes(int N, int Kp, int S_pad, int ngw, int J, size_t* codes_bytes,
                   size_t* scale_elems, size_t* sal_elems);
int sqmp_pack_fq7(const void* codes, const void* wscale, const void* wsal, int dtype, int N,
                  int Kp, int S_pad, int ngw, int J, void* codes_t, void* scale_t, void* sal_t,
                  void* stream);

/* sqmp_gemm_fq_colmax (4-bit codes, Gw % 64 == 0 or Gw == 32, fp16/bf16, N % 8 == 0) on
 * the sqmp_pack_fq7 operands: the same operands and numerics (x_hat . W_hat with W_hat =
 * D(code * scale) decoded in registers, fp32 accumulation, bias, one rounding to D), the
 * codes, scales and salient weights loaded straight into registers; 128 x 512 tiles (J = 4)
 * or 256 x 256 (J = 2), the operands packed with the same J.
 * a: roundup(M, 256) rows allocated.  colmax may be NULL. */
int sqmp_gemm_fq7(const void* a, const void* codes_t, const void* scale_t, const void* sal_t,
                  const void* bias, void* y, int dtype, int M, int N, int Kp, int S_pad,
                  int Gw, int ngw, int J, uint32_t* colmax, void* stream);

/* The weight operand of sqmp_gemm_fqt for the activation order of the LAST
 * sqmp_quant_act_v2(SQMP_OUT_C4) call on `workspace` (same K, Kp, S, S_pad): wp
 * [roundup(N, 256)][Kq + S_pad] in D, wp[n][j] = W_hat[n][column of activation rank j]
 * (= D(code * scale), bit-exact with the reference's W_hat) for j < K - S, 0 for
 * K - S <= j < Kq, then the exact salient weights wsal[n][:]; rows >= N are 0.
 * codes / wscale / wsal: a packed 4-bit weight (sqmp_pack_weight). */
int sqmp_perm_weight_c4(const void* workspace, int K, int Kp, int S, int S_pad,
                        const void* codes, const void* wscale, const void* wsal, int dtype,
                        int N, int Gw, int ngw, void* wp, void* stream);

/* sqmp_quant_act_v2(SQMP_OUT_C4) + sqmp_perm_weight_c4 in one call: the quantizer and the
 * weight permutation run in the same launch (independent given the rank table).  The
 * whole per-forward prepass of sqmp_gemm_fqt. */
int sqmp_quant_act_c4(void* x, int dtype, int M, int K, int amode, int n_bits, int group_size,
                      const int32_t* amap, int Kp, const int32_t* nonsal,
                      const int32_t* salient, int S, int S_pad, const int32_t* posmap,
                      int flags, void* acodes, void* ascale, void* xs, const void* codes,
                      const void* wscale, const void* wsal, int N, int Gw, int ngw, void* wp,
                      void* workspace, size_t ws_bytes, void* stream);

/* The faithful GEMM in activation order: y[M][N] = D(x_hat . W_hat^T + bias) computed as
 * y^T = wp . codes^T with the act codes decoded in registers to D(code * scale) (= the
 * reference's x_hat bit for bit) and the exact salient tail (xs x wsal): the same products
 * as sqmp_gemm_fq minus the zero salient positions of the packed-order stream.  Operands
 * of SQMP_OUT_C4 + sqmp_perm_weight_c4; G % 64 == 0, N % 8 == 0, fp16/bf16. */
int sqmp_gemm_fqt(const void* acodes, const void* ascale, const void* xs, const void* wp,
                  const void* bias, void* y, int dtype, int M, int N, int Kq, int S_pad,
                  int G, int ngq, void* stream);

/* sqmp_gemm_fqt on the tile-major activation operands that sqmp_quant_act_c4 writes with
 * SQMP_QA_TILED (codes [R][Kq/2], scales [R/32][ngq][32], xs [R][S_pad] in the layouts of
 * sqmp_pack_fq7 with J = 2, R = roundup(M, 256)): the act codes ride in registers like
 * sqmp_gemm_fq7's weight codes; the same values as sqmp_gemm_fqt.  Kq % 128 == 0. */
int sqmp_gemm_fqt7(const void* codes_t, const void* scale_t, const void* sal_t, const void* wp,
                   const void* bias, void* y, int dtype, int M, int N, int Kq, int S_pad,
                   int G, int ngq, void* stream);

/* sqmp_gemm_fqt7 with the fused output-quant column statistics (as sqmp_gemm_fq_colmax). */
int sqmp_gemm_fqt7_colmax(const void* codes_t, const void* scale_t, const void* sal_t,
                          const void* wp, const void* bias, void* y, int dtype, int M, int N,
                          int Kq, int S_pad, int G, int ngq, uint32_t* colmax, void* stream);

/* sqmp_gemm_fqt7 / _colmax for either tile-major operand layout: J = 2 (SQMP_QA_TILED, 32-row
 * blocks; 256 x 256 output tiles) or J = 4 (SQMP_QA_TILED4, 64-row blocks; 128 weight rows x
 * 512 tokens per tile).  colmax NULL: no statistics. */
int sqmp_gemm_fqt7j(const void* codes_t, const void* scale_t, const void* sal_t, const void* wp,
                    const void* bias, void* y, int dtype, int M, int N, int Kq, int S_pad, int G,
                    int ngq, int J, uint32_t* colmax, void* stream);

/* Re-read the launch-variant knobs (the SQMP_* A/B and tuning variables of DESIGN.md §7), which
 * the library otherwise reads once, at load: for tools that switch a variant in-process. */
int sqmp_reload_knobs(void);

/* Sibling operand reuse: dst = the SQMP_OUT_FP operand of a layer whose weight shares the
 * quantized input, the salient set and the act mode with the layer that produced src (q/k/v,
 * gate/up), rebuilt by moving positions instead of quantizing again: dst[m][p] =
 * map[p] >= 0 ? src[m][map[p]] : 0 for p < P, dst[m][P + j] = src[m][P + j] (the salient tail)
 * -- bit-exact.  map[p] = the source layer's packed position of the destination layer's
 * column at p (-1 at its salient / padding positions).  fp16 / bf16; P + S_pad <= 8192; src,
 * dst 16-B aligned with rows of P + S_pad elements. */
int sqmp_permute_act(const void* src, void* dst, const int32_t* map, int dtype, int M, int P,
                     int S_pad, void* stream);

/* Sibling layers (q/k/v, gate/up: W4A4Linear modules that the model calls on the SAME input
 * with the same salient set and sorted per_group act mode; fake_quant.py:479-561 swaps them
 * one by one and each forward repeats :291-304 on that input).  One call quantizes x once for
 * `nout` (1..3) packed weights: amaps[o] / posmaps[o] are weight o's amap and posmap (its
 * packed order), outs[o] its SQMP_OUT_FP operand D [roundup(M, 256) rows][Kp + S_pad].  Every
 * outs[o] equals what sqmp_quant_act_v2(..., SQMP_OUT_FP, ...) writes for weight o, bit for
 * bit.  The weights share K, Kp, S_pad and the salient set.  fp16 / bf16, act mode PER_GROUP
 * or PER_GROUP_MEAN3STD, group_size a power of two in [16, 1024], K - S <= 16384,
 * 4 (Kp + S_pad + 8) nout <= 150 KiB (one LDS region per output), flags == SQMP_QA_CLEAN_WS
 * (else SQMP_EUNSUPPORTED before anything is launched).  amaps, posmaps and outs are HOST
 * arrays of device pointers. */
int sqmp_quant_act_group(void* x, int dtype, int M, int K, int amode, int n_bits,
                         int group_size, int nout, const int32_t* const* amaps,
                         const int32_t* const* posmaps, int Kp, const int32_t* nonsal,
                         const int32_t* salient, int S, int S_pad, int flags, void* const* outs,
                         void* workspace, size_t ws_bytes, void* stream);

/* One launch of sqmp_gemm_fq7 over `nprob` (1..4) problems that share M, Kp, S_pad, Gw, ngw
 * and J (the sibling layers above: each problem its own A operand, packed weight, bias,
 * output and colmax); problem p computes exactly what sqmp_gemm_fq7 computes for it, bit for
 * bit.  The tiles of all problems are scheduled together (no launch gap between siblings, and
 * the last partial round of one problem's tiles is filled by the next problem's).  `probs`
 * is a HOST array. */
typedef struct sqmp_fq7_problem {
  const void* a;        /* SQMP_OUT_FP operand, roundup(M, 256) rows allocated */
  const void* codes_t;  /* sqmp_pack_fq7 operands of the problem's weight */
  const void* scale_t;
  const void* sal_t;
  const void* bias;     /* D [N] or NULL */
  void* y;              /* D [M][N] */
  uint32_t* colmax;     /* NULL or as sqmp_gemm_fq_colmax */
  int N;                /* output features, N % 8 == 0 */
} sqmp_fq7_problem;
int sqmp_gemm_fq7_group(const sqmp_fq7_problem* probs, int nprob, int dtype, int M, int Kp,
                        int S_pad, int Gw, int ngw, int J, void* stream);

/* The kernel variant sqmp_gemm_fq7 (nprob = 0: the problem N[0] alone) or sqmp_gemm_fq7_group
 * (nprob problems of N[0 .. nprob)) launches for these shapes: *tm = the row-tile height, *opt =
 * the OPT bits of the packed-order kernel (bit 16 = the K split inside the workgroup: its fp32
 * partial sums add in another order, so its y equals the unsplit kernel's only within fp32
 * rounding; every other bit gives bit-identical y).  Tests and tools use it to know which
 * launches must agree bit for bit. */
int sqmp_fq7_plan(int dtype, int M, const int* N, int nprob, int Kp, int Gw, int J, int* tm,
                  int* opt);

/* The fp32 faithful GEMM on the f16 MFMA (the default for fp32 layers): every row of A and
 * of W is scaled by a power of two (exact) so that its maximum lies in [2^13, 2^14), each
 * scaled value v is split as v = h + l + r with h = f16(v), l = f16(v - h) (|r| <= 2^-22 |v|,
 * plus the f16 subnormal floor 2^-25), and y[m][n] = 2^-(aexp[m] + bexp[n]) (al.wh + ah.wl +
 * ah.wh) + bias with fp32 accumulation: an error below 2^-21 of sum_k |a_k w_k| per output,
 * under the fp32 accumulation error of the GEMM itself, at 3 f16 MFMAs per product.
 * sqmp_split2_f16: src fp32 [R][L] -> dst f16 [2][ldr][L] (h, l of the scaled rows) and
 * rexp int32 [ldr] (rows >= R: zero, exponent 0); once per layer (ldr = Np).
 * sqmp_row_exp: rexp[r] = the scaling exponent of row r of src fp32 [R][L] (per forward, A).
 * sqmp_gemm_h2: a / aexp: the SQMP_OUT_FP operand (fp32, roundup(M, 256) rows allocated) and
 * its row exponents; b2 / bexp: sqmp_split2_f16 of the packed-order W_hat + salient slice.
 * L % 32 == 0; colmax as sqmp_gemm_fq_colmax. */
int sqmp_split2_f16(const float* src, int R, int L, int ldr, void* dst, int* rexp,
                    void* stream);
int sqmp_row_exp(const float* src, int R, int L, int* rexp, void* stream);
int sqmp_gemm_h2(const float* a, const int* aexp, const void* b2, const int* bexp,
                 const float* bias, float* y, int M, int N, int L, uint32_t* colmax,
                 void* stream);

/* The same product on the LDS-DMA ring (the default where L % 64 == 0 and N % 4 == 0; bit-
 * identical to sqmp_gemm_h2): a2 / aexp = sqmp_split2_f16 of the SQMP_OUT_FP operand with ldr
 * >= roundup(M, 128) rows (the two activation planes [2][ldr][L]), wt = sqmp_pack_h2d of the
 * sqmp_split2_f16 weight planes [2][Np][L] (once per layer: Wt[p][Np / 32][L / 64][64][2][2][8],
 * the register fragments of 32-row weight blocks), bexp as for sqmp_gemm_h2.  Replaces the
 * F.linear of fake_quant.py:306 for fp32 layers (run_experiments.py:146-156). */
int sqmp_pack_h2d(const void* planes, int Np, int L, void* wt, void* stream);
int sqmp_gemm_h2d(const void* a2, int ldr, const int* aexp, const void* wt, const int* bexp,
                  const float* bias, float* y, int M, int N, int L, uint32_t* colmax,
                  void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SQMP_W4A4_H */
