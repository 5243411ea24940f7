// MFMA wrappers, in-register weight decoders and LDS-DMA helpers shared by the GEMMs.
#pragma once
#include "sqmp_internal.h"

namespace sqmp {

typedef __attribute__((address_space(3))) void* lds_void_ptr;

// XCD-aware bijective block remap + grouped ordering along M (tiles that share a weight
// column block run together on one XCD).
__device__ inline void tile_coords(int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
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

typedef float f32x16 __attribute__((ext_vector_type(16)));

// 32x32x16 MFMA: lane (r = l & 31, h = l >> 5) holds row r, k = 8h + e of each operand;
// D register g holds row (g & 3) + 8 (g >> 2) + 4h, column r.
template <class DT> struct Mfma32;
template <> struct Mfma32<F16> {
  __device__ static inline void run(f32x16& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const f16x8*)&a, *(const f16x8*)&b, acc, 0, 0, 0);
  }
};
template <> struct Mfma32<BF16> {
  __device__ static inline void run(f32x16& acc, const u32x4& a, const u32x4& b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)&a, *(const bf16x8*)&b, acc, 0, 0, 0);
  }
};

// Decode constants held in VGPRs (gfx950 VOP3 takes no literal), so (x & m) | c is one
// v_and_or_b32.  make_deck() runs once per kernel; the empty asm hides the values.
struct DecK {
  uint32_t m0, m1, c0, c1;
};
__device__ inline DecK make_deck() {
  DecK k{0x000F000Fu, 0x00F000F0u, 0x64006400u, 0x54005400u};
  asm volatile("" : "+v"(k.m0), "+v"(k.m1), "+v"(k.c0), "+v"(k.c1));
  return k;
}
__device__ inline uint32_t and_or(uint32_t x, uint32_t m, uint32_t c) { return (x & m) | c; }

// One bpack dword (8 codes of one lane's fragment) + its prepared scale -> the 8 D values
// D(code * s) (exactly the reference's W_hat, fake_quant.py:193).
template <class DT> struct Dec;
template <> struct Dec<F16> {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  __device__ static inline u32x4 run_lean(uint32_t w, uint32_t s2b, const DecK& k) { return run(w, s2b, k); }
  __device__ static inline uint32_t prep(uint32_t sbits) { return sbits | (sbits << 16); }
  // Nibble slot 0 of a half-word under 0x6400 is the half 1024 + n; slot 1 (bits 4..7)
  // under 0x5400 is 64 + n (ulp 1/16); minus 1032 / 72 gives the code exactly, and the
  // packed half multiply rounds code * s once (RNE).
  __device__ static inline u32x4 run(uint32_t w, uint32_t s2b, const DecK& k) {
    const h2 s2 = *(const h2*)&s2b;
    const h2 o0 = {(_Float16)1032.0f, (_Float16)1032.0f};
    const h2 o1 = {(_Float16)72.0f, (_Float16)72.0f};
    const uint32_t t = w >> 8;
    const uint32_t b[4] = {and_or(w, k.m0, k.c0), and_or(w, k.m1, k.c1), and_or(t, k.m0, k.c0),
                           and_or(t, k.m1, k.c1)};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      h2 hv = *(const h2*)&b[i];
      hv = (hv - ((i & 1) ? o1 : o0)) * s2;
      o[i] = *(const uint32_t*)&hv;
    }
    return u32x4{o[0], o[1], o[2], o[3]};
  }
};
template <> struct Dec<BF16> {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  __device__ static inline uint32_t prep(uint32_t sbits) { return sbits << 16; }
  // The nibbles as bytes (b: nibbles 0, 2, 4, 6; c: 1, 3, 5, 7), each to fp32 by one
  // v_cvt_f32_ubyteN, then (n - 8) * s = fma(n, s, -8 s) on v_pk_fma_f32 -- n * s (4 x 8
  // significant bits) and -8 s are exact, so is their sum (code * s, <= 12 bits: no rounding,
  // and +0 for code 0 as the reference's 0 * s with s > 0) -- and one RNE cast per pair to bf16
  // (v_cvt_pk_bf16_f32): D(code * s) as before, in 20 VALU per 8 values instead of 46.
  __device__ static inline u32x4 run(uint32_t w, uint32_t sf, const DecK&) {
    const float s = __uint_as_float(sf);
    const f2 s2 = {s, s}, m2 = {-8.0f * s, -8.0f * s};
    uint32_t b = w & 0x0F0F0F0Fu, c = (w >> 4) & 0x0F0F0F0Fu;
    asm volatile("" : "+v"(b), "+v"(c));  // (keeps the byte form: v_cvt_f32_ubyte0..3)
    const f2 p0 = {(float)(b & 0xFFu), (float)((b >> 16) & 0xFFu)};  // nibbles 0, 4
    const f2 p1 = {(float)(c & 0xFFu), (float)((c >> 16) & 0xFFu)};  // 1, 5
    const f2 p2 = {(float)((b >> 8) & 0xFFu), (float)(b >> 24)};     // 2, 6
    const f2 p3 = {(float)((c >> 8) & 0xFFu), (float)(c >> 24)};     // 3, 7
    const bf2 r0 = __builtin_convertvector(__builtin_elementwise_fma(p0, s2, m2), bf2);
    const bf2 r1 = __builtin_convertvector(__builtin_elementwise_fma(p1, s2, m2), bf2);
    const bf2 r2 = __builtin_convertvector(__builtin_elementwise_fma(p2, s2, m2), bf2);
    const bf2 r3 = __builtin_convertvector(__builtin_elementwise_fma(p3, s2, m2), bf2);
    return u32x4{__builtin_bit_cast(uint32_t, r0), __builtin_bit_cast(uint32_t, r1),
                 __builtin_bit_cast(uint32_t, r2), __builtin_bit_cast(uint32_t, r3)};
  }
  // the same values with scalar fp32 math, fewer live registers (the J = 4 fq7 tiles, which
  // sit at 256 VGPRs: the packed form's register pairs there spill)
  __device__ static inline u32x4 run_lean(uint32_t w, uint32_t sf, const DecK&) {
    const float s = __uint_as_float(sf);
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

// 16-B non-temporal (streaming) global store.  From inline asm: hipcc merges the two arms of
// `if (nt) __builtin_nontemporal_store(v, p); else *p = v;` into one plain store.
__device__ inline void store16_nt(void* p, const u32x4& v) {
  asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
}

__device__ inline void glds16(const void* src, unsigned char* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)lds_dst, 16, 0, 0);
}

}  // namespace sqmp
