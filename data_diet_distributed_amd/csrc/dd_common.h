// Shared helpers for libdd.so (gfx950 only): error reporting, launch checks, wave reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/dd_capi.h"

namespace dd {

// thread-local "last error" text returned by dd_last_error()
void set_error(const char* fmt, ...);
void clear_error();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

#define DD_REQUIRE(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      ::dd::set_error(__VA_ARGS__);           \
      return DD_EINVAL;                       \
    }                                         \
  } while (0)

#define DD_CHECK_LAUNCH(what)                                                    \
  do {                                                                           \
    hipError_t _e = hipGetLastError();                                           \
    if (_e != hipSuccess) {                                                      \
      ::dd::set_error("%s: %s", what, hipGetErrorString(_e));                    \
      return DD_ELAUNCH;                                                         \
    }                                                                            \
  } while (0)

#define DD_CHECK_HIP(call, what)                                                 \
  do {                                                                           \
    hipError_t _e = (call);                                                      \
    if (_e != hipSuccess) {                                                      \
      ::dd::set_error("%s: %s", what, hipGetErrorString(_e));                    \
      return DD_ELAUNCH;                                                         \
    }                                                                            \
  } while (0)

constexpr int kWave = 64;  // CDNA wavefront width

// butterfly sum over `width` consecutive lanes (width a power of two <= 64)
template <int WIDTH>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, WIDTH);
  return v;
}

template <int WIDTH>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WIDTH));
  return v;
}

// max(v, f) that propagates NaN (IEEE 754-2019 maximum: v_maximum3_f32, one instruction like
// v_max_f32).  Every ReLU / max-pool of the scoring passes uses it: fmaxf returns the non-NaN
// operand, so a value that left the fp16 operand range (inf, then inf - inf = NaN in the split)
// would be turned back into a finite 0 by the next ReLU and reach the scores as silent garbage;
// with nmax it reaches them as NaN, which the engine detects (ScoringEngine._validate).
__device__ __forceinline__ float nmax(float v, float f) {
  return __builtin_elementwise_maximum(v, f);
}
__device__ __forceinline__ float wave_sum(float v) { return group_sum<kWave>(v); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// the weight scale of a split-MFMA pack and the matching accumulator scale of its forward:
// powers of two (exact to apply and undo); bf16 packs are unscaled
inline bool operand_scale_ok(int32_t operands, float s) {
  if (operands == DD_OPERANDS_BF16X3) return s == 1.f;
  int e = 0;
  return operands == DD_OPERANDS_F16X3 && s > 0.f && __builtin_isfinite(s) &&
         __builtin_frexpf(s, &e) == 0.5f;
}

// compute units of the current device (cached per process; 256 on MI355X)
inline int device_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

}  // namespace dd
