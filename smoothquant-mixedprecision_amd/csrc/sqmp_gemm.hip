// W4A4 mixed-precision GEMMs for gfx950 (the F.linear of fake_quant.py:306).
//
// All kernels compute y[M][N] = A . B^T over the packed K axis of a packed weight
// (include/sqmp_w4a4.h): Kp positions of the quantized operand in weight-sorted group
// order, then S_pad positions of the exact salient slice, in one K loop and one
// workgroup, with fp32 accumulation and a single rounding to D in the epilogue.
//
//   gemm_fq2   (fp16 / bf16, int4 or dense B)  "faithful": A = x_hat in D, bit-exact;
//              B decoded in registers from the bpack int4 layout as D(code * scale)
//              (the reference's W_hat bit for bit); D MFMA 16x16x32.
//   gemm_i8v2  (fp16 / bf16 out, int4 B)  per_token / per_tensor activations: int8 act
//              codes x int4 weight codes (unpacked to int8 in registers) on
//              v_mfma_i32_16x16x64_i8, per-weight-group fp32 fold, per-row act scale,
//              salient tail on the D MFMA into the same accumulators.
//   gemm_generic  any dtype (fp32 included), 4-bit / 8-bit / dense B: the round-1
//              register-staged kernel, kept as the fallback path.
//
// Fast-kernel structure (gemm_fq2): 128 x 256 output tile per 256-thread workgroup, the
// four waves side by side along N (each 128 x 64 = 8 x 4 MFMA tiles).  The activation
// tile (the shared operand) is staged by LDS-DMA (global_load_lds_dwordx4) into a
// double-buffered LDS ring of 128-element K stages (256-B rows, 16-B chunks XOR-swizzled
// by row & 15 on the source side, conflict-free ds_read_b128 fragment reads).  The
// weight operand never touches LDS: each lane loads its own 16 bytes of int4 codes per
// K stage straight into VGPRs (the bpack layout makes them exactly its four B fragments),
// double-buffered one stage ahead, and decodes them next to the MFMAs.  The MFMA takes
// the weight fragment in the A slot, so each lane ends up holding 4 consecutive output
// columns of one row: 8-byte stores in the epilogue.
#include "sqmp_internal.h"

namespace sqmp {

// ================================================================= shared helpers
__device__ inline void tile_coords(int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD; give each XCD a
  // contiguous range of the logical tile sequence.
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // grouped ordering along M: tiles sharing a weight column block run together
  const int per_group = group_m * tiles_n;
  const int gid = wg / per_group;
  const int first_m = gid * group_m;
  const int gsz = min(tiles_m - first_m, group_m);
  const int in_g = wg - gid * per_group;
  tm = first_m + in_g % gsz;
  tn = in_g / gsz;
}

template <class DT> struct Mfma;
template <> struct Mfma<F16> {
  __device__ static inline void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(*(const f16x8*)&a, *(const f16x8*)&b, acc, 0, 0, 0);
  }
};
template <> struct Mfma<BF16> {
  __device__ static inline void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)&a, *(const bf16x8*)&b, acc, 0, 0, 0);
  }
};
template <> struct Mfma<F32> {
  // 16x16x4 f32: lane group q supplies k = q; element e of the 16-B chunk is a separate
  // k-slice, so four MFMAs consume the chunk (A and B use the same k assignment).
  __device__ static inline void run(f32x4& acc, const u32x4& a, const u32x4& b) {
    const float* af = (const float*)&a;
    const float* bf = (const float*)&b;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e], bf[e], acc, 0, 0, 0);
  }
};

// One bpack dword (8 codes) -> the 8 D values D(code * s) of one B fragment.
template <class DT> struct Dec8;
template <> struct Dec8<F16> {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  // (0x6400 | nibble) is the half 1024 + nibble; minus 1032 gives the code exactly; the
  // packed half multiply rounds code * s once (RNE) == the reference's D(code * s).
  __device__ static inline u32x4 run(uint32_t w, float s) {
    const _Float16 sh = (_Float16)s;
    const h2 s2 = {sh, sh};
    const h2 off = {(_Float16)1032.0f, (_Float16)1032.0f};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t bits = ((w >> (4 * i)) & 0x000F000Fu) | 0x64006400u;
      h2 h = *(const h2*)&bits;
      h = (h - off) * s2;
      o[i] = *(const uint32_t*)&h;
    }
    return u32x4{o[0], o[1], o[2], o[3]};
  }
};
template <> struct Dec8<BF16> {
  // code * s is exact in fp32 (3-bit code x 8-bit bf16 mantissa); one RNE cast to bf16.
  __device__ static inline u32x4 run(uint32_t w, float s) {
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float lo = (float)((int)((w >> (4 * i)) & 0xFu) - 8) * s;
      const float hi = (float)((int)((w >> (16 + 4 * i)) & 0xFu) - 8) * s;
      const __bf16 bl = (__bf16)lo, bh = (__bf16)hi;
      o[i] = (uint32_t)(*(const uint16_t*)&bl) | ((uint32_t)(*(const uint16_t*)&bh) << 16);
    }
    return u32x4{o[0], o[1], o[2], o[3]};
  }
};

// int4 bpack dword -> two int8 dwords, byte order (e0,e4,e1,e5) and (e2,e6,e3,e7); the
// i8 activation operand is written in the matching K order (sqmp_actquant.hip).
__device__ inline void unpack_i8(uint32_t w, uint32_t& lo, uint32_t& hi) {
  lo = ((w & 0x0F0F0F0Fu) + 0x78787878u) ^ 0x80808080u;
  hi = (((w >> 4) & 0x0F0F0F0Fu) + 0x78787878u) ^ 0x80808080u;
}

// LDS image of a 128-row x 256-byte stage: 16-B chunk c of row r at r*256 + (c^(r&15))*16.
constexpr int ST_ROWB = 256;
constexpr int ST_BYTES = 128 * ST_ROWB;  // 32 KiB

typedef __attribute__((address_space(3))) void* lds_void_ptr;

// Issue one stage of LDS-DMA: 128 rows x 256 B of the row-major A (row stride lda_b
// bytes) starting at byte column col_b.  Eight global_load_lds_dwordx4 per lane; wave w
// writes rows 16 i + 4 w .. +3 of each 16-row group i, lane L the source chunk
// (L & 15) ^ (row & 15) so that the plain ds_read of chunk c at c ^ (row & 15) is right.
// The operand's rows are allocated padded to a multiple of 128 (sqmp_quant_act callers),
// so a tile never clamps: one VGPR offset per lane, the 16-row step is a scalar.
struct StageA {
  uint32_t off;       // this lane's byte offset: row m0 + rin, its swizzled source chunk
  uint32_t stride16;  // 16 rows, bytes (wave-uniform)
  __device__ inline void init(int m0, size_t lda_b, int wave, int lane) {
    const int rin = 4 * wave + (lane >> 4);
    const int chunk = (lane & 15) ^ (rin & 15);
    off = (uint32_t)((size_t)(m0 + rin) * lda_b + chunk * 16);
    stride16 = (uint32_t)(16 * lda_b);
  }
  __device__ inline void issue(const unsigned char* base, unsigned char* lds_stage, int wave) const {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(base + (size_t)i * stride16 + off),
                                       (lds_void_ptr)(lds_stage + (i * 4 + wave) * 1024), 16, 0, 0);
  }
};

__device__ inline const u32x4* lds_frag(const unsigned char* stage, int row, int chunk) {
  return (const u32x4*)(stage + row * ST_ROWB + ((chunk ^ (row & 15)) << 4));
}

// ================================================================= gemm_fq2
// NSC = scales per weight group per 128-position block seen by one lane:
//   1: Gw % 128 == 0 (one group per block), 2: Gw == 64, 4: Gw in {8, 16, 32}.
template <class DT, int WB, int NSC>
__global__ __launch_bounds__(256, 1) void gemm_fq2_kernel(
    const typename DT::T* __restrict__ A, const void* __restrict__ Bw,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int lgG, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * ST_BYTES];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, 4, tm, tn);
  const int m0 = tm * 128, n0 = tn * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int lda = Kp + S_pad;
  const int nkt = lda / 128, nkm = Kp / 128;

  StageA sa;
  sa.init(m0, (size_t)lda * sizeof(T), wave, lane);
  const unsigned char* Ab = (const unsigned char*)A;

  // this lane's 4 weight rows (one per 16-column sub-tile j), clamped for the loads
  int nrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) nrow[j] = min(n0 + wave * 64 + j * 16 + r16, N - 1);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---------------------------------------------------------------- B register stage
  u32x4 bc[4], bn[4];
  float scc[4][NSC], scn[4][NSC];
  const uint32_t* B4 = (const uint32_t*)Bw;
  const size_t brow_dw = (size_t)Kp / 8;  // dwords per bpack row
  auto load_codes = [&](int kt, u32x4 (&b)[4], float (&sc)[4][NSC]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b[j] = *(const u32x4*)(B4 + (size_t)nrow[j] * brow_dw + (size_t)kt * 16 + q * 4);
#pragma unroll
    for (int u = 0; u < NSC; ++u) {
      int g;
      if (NSC == 1) g = (kt * 128) / Gw;
      else if (NSC == 2) g = kt * 2 + u;
      else g = (kt * 128 + 32 * u + 8 * q) >> lgG;
      g = min(g, ngw - 1);  // zero-code padding past the last group
#pragma unroll
      for (int j = 0; j < 4; ++j) sc[j][u] = DT::to_f(wscale[(size_t)g * N + nrow[j]]);
    }
  };

  auto compute_codes = [&](const unsigned char* st, const u32x4 (&b)[4], const float (&sc)[4][NSC]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u32x4 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float scale = NSC == 1 ? sc[j][0] : NSC == 2 ? sc[j][s >> 1] : sc[j][s];
        bf[j] = Dec8<DT>::run(b[j][s], scale);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const u32x4 af = *lds_frag(st, i * 16 + r16, 4 * s + q);
#pragma unroll
        for (int j = 0; j < 4; ++j) Mfma<DT>::run(acc[i][j], bf[j], af);
      }
    }
  };

  // dense B (salient tail, or an unquantized / finely grouped weight): per sub-step each
  // lane loads its 16-B fragment per sub-tile, one sub-step ahead
  auto compute_dense = [&](const unsigned char* st, const T* Bd, size_t ldb, int kofs) {
    u32x4 cur[4], nxt[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) cur[j] = *(const u32x4*)(Bd + (size_t)nrow[j] * ldb + kofs + 8 * q);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s < 3) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          nxt[j] = *(const u32x4*)(Bd + (size_t)nrow[j] * ldb + kofs + 32 * (s + 1) + 8 * q);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const u32x4 af = *lds_frag(st, i * 16 + r16, 4 * s + q);
#pragma unroll
        for (int j = 0; j < 4; ++j) Mfma<DT>::run(acc[i][j], cur[j], af);
      }
      if (s < 3) {
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
      }
    }
  };

  // ---------------------------------------------------------------- main loop
  // stage kt lives in LDS buffer kt & 1; its LDS-DMA is issued one stage ahead.
  auto issue_stage = [&](int kt) {
    sa.issue(Ab + (size_t)kt * 128 * sizeof(T), lds + (kt & 1) * ST_BYTES, wave);
  };
  issue_stage(0);
  if (WB == 4 && nkm > 0) load_codes(0, bc, scc);
  __syncthreads();
  int kt = 0;
  if (WB == 4) {
    // two stages per iteration: the B register sets alternate without copies
    for (; kt + 1 < nkm; kt += 2) {
      issue_stage(kt + 1);
      load_codes(kt + 1, bn, scn);
      compute_codes(lds, bc, scc);
      __syncthreads();
      if (kt + 2 < nkt) issue_stage(kt + 2);
      if (kt + 2 < nkm) load_codes(kt + 2, bc, scc);
      compute_codes(lds + ST_BYTES, bn, scn);
      __syncthreads();
    }
    if (kt < nkm) {  // odd number of main stages: the last one (even kt, buffer 0)
      if (kt + 1 < nkt) issue_stage(kt + 1);
      compute_codes(lds, bc, scc);
      __syncthreads();
      ++kt;
    }
  } else {
    for (; kt < nkm; ++kt) {
      if (kt + 1 < nkt) issue_stage(kt + 1);
      compute_dense(lds + (kt & 1) * ST_BYTES, (const T*)Bw, (size_t)Kp, kt * 128);
      __syncthreads();
    }
  }
  // salient tail: exact weight columns, dense D
  for (; kt < nkt; ++kt) {
    if (kt + 1 < nkt) issue_stage(kt + 1);
    compute_dense(lds + (kt & 1) * ST_BYTES, wsal, (size_t)S_pad, (kt - nkm) * 128);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][r] = C[n = n0 + 64 wave + 16 j + 4 q + r][m = m0 + 16 i + r16]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nb = n0 + wave * 64 + j * 16 + q * 4;
    if (nb >= N) continue;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = (bias && nb + r < N) ? DT::to_f(bias[nb + r]) : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int gm = m0 + i * 16 + r16;
      if (gm >= M) continue;
      T v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = DT::from_f(acc[i][j][r] + bv[r]);
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
// 128 x 128 tile, 4 waves as 2 (M) x 2 (N), each 64 x 64.  A stages hold 256 int8
// codes (2 bpack blocks) per row: i8 sub-step t (64 codes) reads chunk 4 t + q; the
// activation codes were written in the K order that matches unpack_i8 of the bpack
// dwords (2t, 2t+1) of lane group q.
template <class DT>
__global__ __launch_bounds__(256, 1) void gemm_i8v2_kernel(
    const int8_t* __restrict__ A8, const float* __restrict__ ascale,
    const typename DT::T* __restrict__ XS, const uint32_t* __restrict__ B4,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * ST_BYTES];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, 8, tm, tn);
  const int m0 = tm * 128, n0 = tn * 128;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, q = lane >> 4;
  const int nkm = Kp / 256 + ((Kp % 256) ? 1 : 0);  // 256-code stages (last may be half)
  const int nks = S_pad / 128;                        // 128-element salient stages

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
  // B registers for one 256-code stage: 2 blocks x 4 dwords per sub-tile j
  u32x4 bc[4][2], bn[4][2];
  auto load_codes = [&](int ks, u32x4 (&b)[4][2]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int blk = min(ks * 2 + h, Kp / 128 - 1);
        b[j][h] = *(const u32x4*)(B4 + (size_t)nrow[j] * brow_dw + (size_t)blk * 16 + q * 4);
      }
  };
  // fold the int32 group partials: acc holds C[n = ... + 4q + r][m = ... + r16]
  auto fold = [&](int g) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wn * 64 + j * 16 + q * 4;
      float s[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) s[r] = DT::to_f(wscale[(size_t)g * N + min(nb + r, N - 1)]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) tot[i][j][r] += (float)acc[i][j][r] * s[r];
        acc[i][j] = i32x4{0, 0, 0, 0};
      }
    }
  };
  auto compute_codes = [&](int ks, const unsigned char* st, const u32x4 (&b)[4][2]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int p_end = ks * 256 + (t + 1) * 64;
      if (p_end > Kp) break;  // half stage at the end of an odd number of blocks
      u32x4 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u32x4 w = b[j][t >> 1];
        uint32_t l0, h0, l1, h1;
        unpack_i8(w[(t & 1) * 2], l0, h0);
        unpack_i8(w[(t & 1) * 2 + 1], l1, h1);
        bf[j] = u32x4{l0, h0, l1, h1};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x4 af = *lds_frag(st, wm * 64 + i * 16 + r16, 4 * t + q);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(*(const i32x4*)&bf[j], *(const i32x4*)&af, acc[i][j], 0, 0, 0);
      }
      if (p_end % Gw == 0 && p_end / Gw <= ngw) fold(p_end / Gw - 1);
    }
  };

  // ---- main (int) stages: rows of 256 B (Kp may end in a half stage: the quantizer pads
  // A8 rows to a multiple of 256 codes)
  const int lda8 = nkm * 256;
  StageA sa;
  sa.init(m0, (size_t)lda8, wave, lane);
  const unsigned char* Ab = (const unsigned char*)A8;
  if (nkm > 0) {
    sa.issue(Ab, lds, wave);
    load_codes(0, bc);
    __syncthreads();
    for (int ks = 0; ks < nkm; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nkm) {
        sa.issue(Ab + (size_t)(ks + 1) * 256, lds + (cur ^ 1) * ST_BYTES, wave);
        load_codes(ks + 1, bn);
      }
      compute_codes(ks, lds + cur * ST_BYTES, bc);
      if (ks + 1 < nkm) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { bc[j][0] = bn[j][0]; bc[j][1] = bn[j][1]; }
      }
      __syncthreads();
    }
  }
  // per-row activation scale (fake_quant.py:56-75, factored out of the sum)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = min(m0 + wm * 64 + i * 16 + r16, M - 1);
    const float s = ascale[gm];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[i][j][r] *= s;
  }
  // ---- salient tail on the D MFMA (exact operands)
  if (nks > 0) {
    StageA sx;
    sx.init(m0, (size_t)S_pad * sizeof(T), wave, lane);
    const unsigned char* Xb = (const unsigned char*)XS;
    sx.issue(Xb, lds, wave);
    __syncthreads();
    for (int ks = 0; ks < nks; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nks) sx.issue(Xb + (size_t)(ks + 1) * 128 * sizeof(T), lds + (cur ^ 1) * ST_BYTES, wave);
      const unsigned char* st = lds + cur * ST_BYTES;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        u32x4 bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bf[j] = *(const u32x4*)(wsal + (size_t)nrow[j] * S_pad + ks * 128 + 32 * s + 8 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u32x4 af = *lds_frag(st, wm * 64 + i * 16 + r16, 4 * s + q);
#pragma unroll
          for (int j = 0; j < 4; ++j) Mfma<DT>::run(tot[i][j], bf[j], af);
        }
      }
      __syncthreads();
    }
  }
  // ---- epilogue: 4 consecutive columns per lane -> 8-byte stores
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

// ================================================================= generic fallback
constexpr int BM = 128, BN = 128;
constexpr int ROWB = 128;
constexpr int TILE_BYTES = BM * ROWB;

__device__ inline int lds_off(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 7)) << 4); }

// Decode one thread's share of a weight row for one K-tile: BKE/2 consecutive positions
// -> 64 bytes of D values (4 LDS chunks).  WBITS 4 = bpack, 8 = row-major int8,
// 0 = dense D.
template <class DT, int WBITS>
struct BDecode {
  typedef typename DT::T T;
  static constexpr int BKE = ROWB / sizeof(T);
  static constexpr int NCODE = BKE / 2;
  static constexpr int RAWW = WBITS == 4 ? NCODE / 8 : WBITS == 8 ? NCODE / 4 : NCODE * (int)sizeof(T) / 4;
  static constexpr int EPC = 16 / sizeof(T);

  __device__ static inline void load(const uint8_t* codes, int n, int Kp, int p0, uint32_t* raw) {
    if (WBITS == 4) {
      const uint32_t* row = (const uint32_t*)codes + (size_t)n * (Kp / 8);
#pragma unroll
      for (int w = 0; w < RAWW; ++w) raw[w] = row[bpack_dword(p0 + 8 * w)];
    } else if (WBITS == 8) {
      const uint32_t* src = (const uint32_t*)(codes + (size_t)n * Kp + p0);
#pragma unroll
      for (int w = 0; w < RAWW; ++w) raw[w] = src[w];
    } else {
      const uint32_t* src = (const uint32_t*)((const T*)codes + (size_t)n * Kp + p0);
#pragma unroll
      for (int w = 0; w < RAWW; ++w) raw[w] = src[w];
    }
  }
  __device__ static inline int code_at(const uint32_t* raw, int e) {
    if (WBITS == 4) return (int)((raw[e >> 3] >> bpack_shift(e & 7)) & 0xFu) - 8;
    return (int)(int8_t)((raw[e >> 2] >> (8 * (e & 3))) & 0xFFu);
  }
  __device__ static inline void run(const uint32_t* raw, const float* s, u32x4* out) {
    if (WBITS == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) out[c] = u32x4{raw[4 * c], raw[4 * c + 1], raw[4 * c + 2], raw[4 * c + 3]};
      return;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      T v[EPC];
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] = DT::from_f((float)code_at(raw, c * EPC + e) * s[c]);
      out[c] = *(const u32x4*)v;
    }
  }
};

template <class DT, int WBITS>
__global__ __launch_bounds__(256, 2) void gemm_generic_kernel(
    const typename DT::T* __restrict__ A, const uint8_t* __restrict__ codes,
    const typename DT::T* __restrict__ wscale, const typename DT::T* __restrict__ wsal,
    const typename DT::T* __restrict__ bias, typename DT::T* __restrict__ Y, int M, int N,
    int Kp, int S_pad, int Gw, int ngw, int tiles_m, int tiles_n) {
  typedef typename DT::T T;
  typedef BDecode<DT, WBITS> Dec;
  constexpr int BKE = ROWB / sizeof(T);
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * 2 * TILE_BYTES];

  int tm, tn;
  tile_coords(tiles_m, tiles_n, 8, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int Ktot = Kp + S_pad;
  const int nkt_main = Kp / BKE, nkt = Ktot / BKE;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4], rb[4];
  uint32_t rc[Dec::RAWW];
  float rs[4];
  const int bn = tid >> 1, bh = tid & 1;
  const int gbn = n0 + bn;

  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      const int gm = min(m0 + row, M - 1);
      ra[i] = *(const u32x4*)(A + (size_t)gm * Ktot + (size_t)kt * BKE + c * (16 / sizeof(T)));
    }
    if (kt < nkt_main) {
      const int p0 = kt * BKE + bh * (BKE / 2);
      const int n = min(gbn, N - 1);
      Dec::load(codes, n, Kp, p0, rc);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int p = p0 + c * (BKE / 8);
        rs[c] = WBITS ? DT::to_f(wscale[(size_t)min(p / Gw, ngw - 1) * N + n]) : 1.f;
      }
    } else {
      const int ks = (kt - nkt_main) * BKE;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = tid + 256 * i, row = q >> 3, c = q & 7;
        const int gn = min(n0 + row, N - 1);
        rb[i] = *(const u32x4*)(wsal + (size_t)gn * S_pad + ks + c * (16 / sizeof(T)));
      }
    }
  };
  auto store = [&](int kt, int buf) {
    unsigned char* la = lds + buf * 2 * TILE_BYTES;
    unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      *(u32x4*)(la + lds_off(row, c)) = ra[i];
    }
    if (kt < nkt_main) {
      u32x4 dec[4];
      Dec::run(rc, rs, dec);
#pragma unroll
      for (int c = 0; c < 4; ++c) *(u32x4*)(lb + lds_off(bn, bh * 4 + c)) = dec[c];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = tid + 256 * i, row = q >> 3, c = q & 7;
        *(u32x4*)(lb + lds_off(row, c)) = rb[i];
      }
    }
  };
  auto compute = [&](int buf) {
    const unsigned char* la = lds + buf * 2 * TILE_BYTES;
    const unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 af[4], bf[4];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(la + lds_off(wm * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *(const u32x4*)(lb + lds_off(wn * 64 + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Mfma<DT>::run(acc[i][j], af[i], bf[j]);
    }
  };

  load(0);
  store(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) load(kt + 1);
    compute(cur);
    if (kt + 1 < nkt) store(kt + 1, cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int gn = n0 + wn * 64 + j * 16 + (lane & 15);
    if (gn >= N) continue;
    const float bv = bias ? DT::to_f(bias[gn]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (gm < M) Y[(size_t)gm * N + gn] = DT::from_f(acc[i][j][r] + bv);
      }
  }
}

// ================================================================= launchers
template <class DT, int WB, int NSC>
static int fq2_launch(const void* a, const void* codes, const void* wscale, const void* wsal,
                      const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                      int lgG, int ngw, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, 128), tiles_n = cdiv(N, 256);
  gemm_fq2_kernel<DT, WB, NSC><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
      (const T*)a, codes, (const T*)wscale, (const T*)wsal, (const T*)bias, (T*)y, M, N, Kp,
      S_pad, Gw, lgG, ngw, tiles_m, tiles_n);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT>
static int fq2_dispatch(const void* a, const void* codes, const void* wscale, const void* wsal,
                        const void* bias, void* y, int M, int N, int Kp, int S_pad, int Gw,
                        int ngw, int n_bits, hipStream_t s) {
  if (n_bits == 0) return fq2_launch<DT, 0, 1>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, 1, 0, 1, s);
  if (Gw % 128 == 0) return fq2_launch<DT, 4, 1>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, 0, ngw, s);
  if (Gw == 64) return fq2_launch<DT, 4, 2>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, 6, ngw, s);
  const int lg = Gw == 32 ? 5 : Gw == 16 ? 4 : 3;
  return fq2_launch<DT, 4, 4>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, lg, ngw, s);
}

template <class DT, int WBITS>
static int generic_launch(const void* a, const void* codes, const void* wscale,
                          const void* wsal, const void* bias, void* y, int M, int N, int Kp,
                          int S_pad, int Gw, int ngw, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  gemm_generic_kernel<DT, WBITS><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
      (const T*)a, (const uint8_t*)codes, (const T*)wscale, (const T*)wsal, (const T*)bias,
      (T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, tiles_n);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

template <class DT>
static int i8_launch(const int8_t* a8, const float* ascale, const void* xs, const void* codes,
                     const void* wscale, const void* wsal, const void* bias, void* y, int M,
                     int N, int Kp, int S_pad, int Gw, int ngw, hipStream_t s) {
  typedef typename DT::T T;
  const int tiles_m = cdiv(M, 128), tiles_n = cdiv(N, 128);
  gemm_i8v2_kernel<DT><<<dim3(tiles_m * tiles_n), dim3(256), 0, s>>>(
      a8, ascale, (const T*)xs, (const uint32_t*)codes, (const T*)wscale, (const T*)wsal,
      (const T*)bias, (T*)y, M, N, Kp, S_pad, Gw, ngw, tiles_m, tiles_n);
  SQMP_LAUNCH_CHECK();
  return SQMP_OK;
}

}  // namespace sqmp

using namespace sqmp;

static int check_gemm_geometry(int dtype, int M, int N, int Kp, int S_pad, int Gw, int ngw,
                               int n_bits) {
  if (dtype < SQMP_F32 || dtype > SQMP_BF16 || M < 0 || N <= 0) return SQMP_EINVAL;
  if (Kp <= 0 || Kp % 128 != 0 || S_pad < 0 || S_pad % 128 != 0) return SQMP_EINVAL;
  if (n_bits == 0) return SQMP_OK;  // dense operand: no groups
  if (Gw <= 0 || ngw <= 0 || (long)(ngw - 1) * Gw >= Kp) return SQMP_EINVAL;
  if (n_bits != 4 && n_bits != 8) return SQMP_EUNSUPPORTED;
  // one scale per 16-B chunk of decoded B: groups must not split a chunk
  const int epc = dtype == SQMP_F32 ? 4 : 8;
  if (Gw % epc != 0) return SQMP_EUNSUPPORTED;
  return SQMP_OK;
}

extern "C" int sqmp_gemm_fq(const void* a, const void* codes, const void* wscale,
                            const void* wsal, const void* bias, void* y, int dtype, int M,
                            int N, int Kp, int S_pad, int Gw, int ngw, int n_bits,
                            void* stream) {
  int st = check_gemm_geometry(dtype, M, N, Kp, S_pad, Gw, ngw, n_bits);
  if (st) return st;
  if (!a || !codes || (n_bits && !wscale) || !y || (S_pad > 0 && !wsal)) return SQMP_EINVAL;
  if (M == 0) return SQMP_OK;
  if (n_bits == 0) { Gw = Kp; ngw = 1; }
  hipStream_t s = (hipStream_t)stream;
  // fast kernel: fp16 / bf16 with int4 (Gw a multiple of 128 or a power of two >= 8) or
  // dense weights; everything else (fp32, 8-bit codes, odd group sizes) -> generic
  const bool pow2 = (Gw & (Gw - 1)) == 0;
  const bool fast_g = n_bits == 0 || (n_bits == 4 && (Gw % 128 == 0 || (pow2 && Gw >= 8)));
  if (dtype != SQMP_F32 && fast_g) {
    return dtype == SQMP_F16 ? fq2_dispatch<F16>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s)
                             : fq2_dispatch<BF16>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, n_bits, s);
  }
#define SQMP_G(DTT, WB) generic_launch<DTT, WB>(a, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s)
  switch (dtype) {
    case SQMP_F32: return n_bits == 4 ? SQMP_G(F32, 4) : n_bits == 8 ? SQMP_G(F32, 8) : SQMP_G(F32, 0);
    case SQMP_F16: return n_bits == 4 ? SQMP_G(F16, 4) : n_bits == 8 ? SQMP_G(F16, 8) : SQMP_G(F16, 0);
    default: return n_bits == 4 ? SQMP_G(BF16, 4) : n_bits == 8 ? SQMP_G(BF16, 8) : SQMP_G(BF16, 0);
  }
#undef SQMP_G
}

extern "C" int sqmp_gemm_i8(const int8_t* a8, const float* ascale, const void* xs,
                            const void* codes, const void* wscale, const void* wsal,
                            const void* bias, void* y, int dtype, int M, int N, int Kp,
                            int S_pad, int Gw, int ngw, int n_bits, void* stream) {
  int st = check_gemm_geometry(dtype, M, N, Kp, S_pad, Gw, ngw, n_bits);
  if (st) return st;
  if (dtype == SQMP_F32 || n_bits != 4 || Gw % 64 != 0) return SQMP_EUNSUPPORTED;
  if (!a8 || !ascale || !codes || !wscale || !y || (S_pad > 0 && (!wsal || !xs)))
    return SQMP_EINVAL;
  if (M == 0) return SQMP_OK;
  hipStream_t s = (hipStream_t)stream;
  return dtype == SQMP_F16 ? i8_launch<F16>(a8, ascale, xs, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s)
                           : i8_launch<BF16>(a8, ascale, xs, codes, wscale, wsal, bias, y, M, N, Kp, S_pad, Gw, ngw, s);
}
