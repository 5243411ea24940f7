// Shared device helpers for the W4A4 mixed-precision linear on MI355X (gfx950 / CDNA4).
//
// Numerics contract (mirrors /root/reference/smoothquant/fake_quant.py):
//   * D is the model dtype (fp32 / fp16 / bf16).  Every elementwise quantizer op is
//     computed in fp32 and rounded to D (PyTorch's opmath rule), round() is
//     round-half-to-even, scales are `D(D(clamp(absmax, 1e-5)) / q_max)`.
//   * Column sorts are stable ascending (ties -> lower column index first).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sqmp_w4a4.h"  // include/ (build_ext.py passes -I include)

namespace sqmp {

// Every C entry that launches work runs it on its STREAM's device: the reference's callers
// place layers on several GPUs (accelerate device_map="auto", run_experiments.py:146-148,
// examples/ppl_eval.sh:17-18), so the caller's current device need not be the tensors'.  The
// guard makes the stream's device current for the call and restores the caller's on return
// (one hipGetDevice when they already agree; the null stream means the current device).
class DeviceGuard {
 public:
  explicit DeviceGuard(void* stream) {
    if (!stream) return;
    int dev = -1, cur = -1;
    if (hipStreamGetDevice((hipStream_t)stream, &dev) != hipSuccess) return;
    if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess)
      prev_ = cur;
  }
  ~DeviceGuard() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

 private:
  int prev_ = -1;
};
#define SQMP_DEVICE_GUARD(stream) ::sqmp::DeviceGuard sqmp_device_guard_((void*)(stream))

// A launch attribute (hipFuncSetAttribute) belongs to the CURRENT device: a call site that
// sets one once keeps a bit per device in `seen` (true the first time on this device).
inline bool first_on_device(uint64_t& seen) {
  int d = 0;
  (void)hipGetDevice(&d);
  const uint64_t bit = 1ull << (d & 63);
  return (__atomic_fetch_or(&seen, bit, __ATOMIC_RELAXED) & bit) == 0;
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- dtype traits
struct F32 {
  typedef float T;
  static constexpr int id = SQMP_F32;
  __device__ static inline float to_f(T v) { return v; }
  __device__ static inline T from_f(float v) { return v; }
};
struct F16 {
  typedef _Float16 T;
  static constexpr int id = SQMP_F16;
  __device__ static inline float to_f(T v) { return (float)v; }
  __device__ static inline T from_f(float v) { return (T)v; }  // RNE (v_cvt_f16_f32)
};
struct BF16 {
  typedef __bf16 T;
  static constexpr int id = SQMP_BF16;
  __device__ static inline float to_f(T v) { return (float)v; }
  __device__ static inline T from_f(float v) { return (T)v; }  // RNE (v_cvt_pk_bf16_f32)
};

// Round an fp32 value to D and widen it back (the "rounded to D" step).
template <class DT>
__device__ inline float rd(float v) {
  return DT::to_f(DT::from_f(v));
}

// clamp(min=1e-5) then div by q_max, both rounded to D (fake_quant.py:14, 62, 139, 190).
template <class DT>
__device__ inline float group_scale(float absmax_d, int q_max) {
  const float lo = rd<DT>(1e-5f);
  float c = absmax_d < lo ? lo : absmax_d;
  return rd<DT>(c / (float)q_max);
}

// code = round_half_even(D(t / s)) (fake_quant.py:15, 63, 142, 193).
template <class DT>
__device__ inline float quant_code(float t, float s) {
  return __builtin_rintf(rd<DT>(t / s));
}

// ---------------------------------------------------------------- small utils
__device__ inline float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ inline float block_max(float v, float* red /* >= 16 floats of LDS */) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, red[i]);
  return r;
}

__host__ __device__ inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------- packed int4 layout
// "bpack": per weight row, per 64-position block, 32 bytes = 8 dwords.  Dword (h * 4 + u)
// holds the 8 codes of positions 16*u + 8*h + e (e = 0..7): the two 16-byte halves of a
// block are exactly what lane half h of a 32x32x16 MFMA B operand needs for the block's
// four K sub-steps u (one ds_read_b128).  Inside a dword, even e sit in the low half-word
// (nibble e/2), odd e in the high half-word (nibble 4 + e/2), so (w & 0x000F000F) and
// (w & 0x00F000F0) hold the pairs (e=0,1) and (e=2,3) in two 16-bit lanes without a
// shift.  Nibble = code + 8 (offset binary, code in [-7, 7]).
__host__ __device__ inline int bpack_dword(int p) {
  const int kin = p & 63;
  return (p >> 6) * 8 + ((kin >> 3) & 1) * 4 + (kin >> 4);
}
__host__ __device__ inline int bpack_shift(int p) {
  const int e = p & 7;
  return (e & 1) ? 16 + 4 * (e >> 1) : 4 * (e >> 1);
}
// Weight rows are allocated padded to Np = roundup(N, 256) (one fast-GEMM N tile): the
// codes buffer holds Np rows and wscale rows have stride Np, so whole tiles are staged by
// LDS-DMA without per-lane clamps.  Rows >= N never reach y.
__host__ __device__ inline int pad_n(int N) { return (N + 255) / 256 * 256; }

// packed position of element e of dword d
__host__ __device__ inline int bpack_pos(int d, int e) {
  return (d >> 3) * 64 + (d & 3) * 16 + ((d >> 2) & 1) * 8 + e;
}
__host__ __device__ inline int bpack_elem_of_shift(int sh) {  // inverse of bpack_shift
  return sh >= 16 ? 2 * ((sh - 16) >> 2) + 1 : 2 * (sh >> 2);
}
__host__ __device__ inline long round_up(long a, long b) { return (a + b - 1) / b * b; }
__device__ inline long round_up_dev(long a, long b) { return (a + b - 1) / b * b; }

}  // namespace sqmp

#define SQMP_HIP_CHECK(expr)                        \
  do {                                              \
    hipError_t _e = (expr);                         \
    if (_e != hipSuccess) return SQMP_EHIP;         \
  } while (0)

#define SQMP_LAUNCH_CHECK()                         \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return SQMP_EHIP;         \
  } while (0)
