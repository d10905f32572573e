// Shared pieces of the split-bf16 MFMA kernels (dd_conv.hip, dd_down.hip): fragment types,
// the hardware-transposed LDS read of B fragments, the butterfly transpose-reduce used by the
// BN statistics epilogues, the bf16 hi/lo split.
#pragma once
#include "dd_common.h"

#include <type_traits>
#include <utility>

namespace dd {
namespace conv {

// one butterfly step of the transpose-reduce: 2M values -> M values per lane
template <int M>
__device__ __forceinline__ void xreduce_step(float (&v)[32], int lane) {
  const bool hi = (lane & M) != 0;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const float keep = hi ? v[j + M] : v[j];
    const float send = hi ? v[j] : v[j + M];
    v[j] = keep + __shfl_xor(send, M, 64);
  }
}

// sum over each aligned group of 8 lanes, every lane of the group receiving it: DPP
// quad_perm [1,0,3,2], [2,3,0,1], then row_half_mirror (lane i <-> 7 - i) adds the other quad
// (every lane reads a valid source, so the DPP old value is never used: mov_dpp leaves it
// undefined, and the move folds into the add as one v_add_f32_dpp instead of a zeroing move, a
// DPP move and an add)
__device__ __forceinline__ float sum8(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xf,
                                                          0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xf,
                                                          0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xf,
                                                          0xf, false));
  return v;
}

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) shortx4 lds_shortx4;

constexpr int CC = 16;  // input channels per K chunk

// compile-time loop: f(std::integral_constant<int, 0>) ... f(<N - 1>), so register-array
// indices derived from the counter are constants whatever the unroller decides
template <typename F, int... Ts>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Ts...>) {
  (f(std::integral_constant<int, Ts>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}


__host__ __device__ constexpr int pad_to(int v, int m) { return (v + m - 1) / m * m; }

__device__ __forceinline__ bf16x8 tr_read8(const char* lds_generic_a, const char* lds_generic_b) {
  // two transposed 4-row reads -> 8 consecutive k elements (rows) of this lane's column
  const lds_shortx4* pa = (const lds_shortx4*)(__attribute__((address_space(3))) const char*)
      (lds_generic_a);
  const lds_shortx4* pb = (const lds_shortx4*)(__attribute__((address_space(3))) const char*)
      (lds_generic_b);
  const shortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4*)pa);
  const shortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4*)pb);
  const shortx8 v = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return __builtin_bit_cast(bf16x8, v);
}

// epilogue output store of 4 consecutive fp32 values: a non-temporal vector store (the conv
// outputs are streams far larger than an XCD's L2).  Whole-job A/B (tools/ab_bench.sh,
// alternated on one box, profiles/r05_s7/ab_nt_*): config 2 +0.45 %, config 4 (N = 10 240)
// +1.0 %; per kernel (tools/ab_conv.py) up to 1.27x on the 1x1 expansions and 1.05-1.09x on
// the stem, 0.98-1.0x on the 64-channel 32x32 conv.  DD_NT_STORE=0 builds plain stores.
#ifndef DD_NT_STORE
#define DD_NT_STORE 1
#endif
__device__ __forceinline__ void store_out4(float* p, float a, float b, float c, float d) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v v = {a, b, c, d};
  if constexpr (DD_NT_STORE != 0)
    __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
  else
    *reinterpret_cast<f4v*>(p) = v;
}

// XCD-aware workgroup order: blocks are dealt round-robin over the 8 XCDs, so physical block p
// runs on XCD p % 8; returning a logical id that is contiguous per XCD keeps runs of
// neighbouring tiles (same example, adjacent rows / channel blocks: shared input rows and
// weights) in one XCD's L2.  Bijective for any grid size.
__device__ __forceinline__ unsigned xcd_order(unsigned p, unsigned n) {
  const unsigned q = n / 8, r = n % 8, x = p % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + p / 8;
}

// two floats -> packed bf16x2 (round to nearest even: v_cvt_pk_bf16_f32), a in the low half
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// v = hi + lo with both halves bf16 (lo = bf16(v - hi)): ~2^-16 relative per split product
__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}

// ---- operand halves: bf16 (default) or fp16 (F16) ------------------------------------------
// The split products hi*hi + hi*lo + lo*hi keep 2 x 8 significant bits per operand in bf16
// (~2^-17 relative per product: the dropped lo*lo and each operand's residual) but 2 x 11 in
// fp16 (~2^-22), at the same MFMA rate on gfx950 (v_mfma_f32_32x32x16_f16).  fp16's range
// (|v| < 65504, subnormal below 6.1e-5, whose halves then carry an absolute error of at most
// 2^-25) suits bounded operands: the EL2N forward, whose inputs are batch-normalised
// activations and raw conv weights (tools/emulate_split.py: ResNet-50 EL2N 9.1e-4 -> 3.3e-5
// max relative error).  The GraNd backward keeps bf16: its gradients span many octaves and
// fall into fp16's subnormal range.  Halves are carried as 16-bit patterns in the bf16x8
// fragment registers either way; only the split and the MFMA opcode differ.
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

// two floats -> packed halves (round to nearest even), a in the low half
template <bool F16>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  if constexpr (F16) {
    typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
    const halfx2 v = {(_Float16)a, (_Float16)b};  // v_cvt_pk_f16_f32
    return __builtin_bit_cast(uint32_t, v);
  } else {
    return pack_bf16x2(a, b);
  }
}
// the float value of the low / high half of a packed pair
template <bool F16>
__device__ __forceinline__ float half_lo(uint32_t v) {
  if constexpr (F16)
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(v & 0xffffu));
  else
    return __uint_as_float(v << 16);
}
template <bool F16>
__device__ __forceinline__ float half_hi(uint32_t v) {
  if constexpr (F16)
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(v >> 16));
  else
    return __uint_as_float(v & 0xffff0000u);
}
// v = hi + lo in the operand type (stored as 16-bit patterns in __bf16 slots)
template <bool F16>
__device__ __forceinline__ void split16(float v, __bf16& hi, __bf16& lo) {
  if constexpr (F16) {
    const _Float16 h = (_Float16)v;
    hi = __builtin_bit_cast(__bf16, h);
    lo = __builtin_bit_cast(__bf16, (_Float16)(v - (float)h));
  } else {
    split_bf16(v, hi, lo);
  }
}
// one 32x32x16 MFMA on operand halves of the given type
template <bool F16>
__device__ __forceinline__ floatx16 mfma16(bf16x8 a, bf16x8 b, floatx16 d) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, a),
                                                  __builtin_bit_cast(halfx8, b), d, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, d, 0, 0, 0);
}

// Staging of one lane's 4 consecutive positions of a channel row (v) for the three kx shifts of
// a 3-wide window: hi[kx] / lo[kx] = bf16 hi / lo of positions x - 1 + kx .. x + 2 + kx as
// bf16x4 (two dwords), x the lane's first position.  The split works on packed pairs
// (v_cvt_pk_bf16_f32: the same RNE values as split_bf16 per element) and the halo columns
// come from the neighbouring lanes' packed halves by DPP row shifts; `first` / `last` (the
// row's first / last lane) take the zero padding instead.
template <bool F16 = false>
__device__ __forceinline__ void split_shift3(float4 v, bool first, bool last, uint2 (&hi)[3],
                                             uint2 (&lo)[3]) {
  uint32_t h01 = pack2<F16>(v.x, v.y), h23 = pack2<F16>(v.z, v.w);
  // fp16: the packed halves are opaque to the compiler, which otherwise re-converts every
  // element on its own (v_cvt_f16_f32) for the residuals and the shifted pairs beside the
  // packed v_cvt_pk_f16_f32 (6 extra conversions per float4); same values either way
  if constexpr (F16) asm("" : "+v"(h01), "+v"(h23));
  uint32_t l01 = pack2<F16>(v.x - half_lo<F16>(h01), v.y - half_hi<F16>(h01));
  uint32_t l23 = pack2<F16>(v.z - half_lo<F16>(h23), v.w - half_hi<F16>(h23));
  if constexpr (F16) asm("" : "+v"(l01), "+v"(l23));
  auto shifts = [&](uint32_t a01, uint32_t a23, uint2(&o)[3]) {
    uint32_t nl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a23, 0x111, 0xf, 0xf, true);
    uint32_t nr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a01, 0x101, 0xf, 0xf, true);
    nl = first ? 0u : nl;  // left neighbour's (z, w): w is this lane's x - 1
    nr = last ? 0u : nr;   // right neighbour's (x, y): x is this lane's x + 4
    const uint32_t yz = __builtin_amdgcn_alignbit(a23, a01, 16);
    o[0] = make_uint2(__builtin_amdgcn_alignbit(a01, nl, 16), yz);  // (x - 1, x), (y, z)
    o[1] = make_uint2(a01, a23);
    o[2] = make_uint2(yz, __builtin_amdgcn_alignbit(nr, a23, 16));  // (y, z), (w, x + 4)
  };
  shifts(h01, h23, hi);
  shifts(l01, l23, lo);
}

// v where ok, else +0.0 (a bitwise AND: a select on a loaded value compiles into a branch
// around the wait for the load, which splits the scheduling region it sits in)
__device__ __forceinline__ float4 keep_if(float4 v, bool ok) {
  const uint32_t m = ok ? 0xffffffffu : 0u;
  return make_float4(__uint_as_float(__float_as_uint(v.x) & m),
                     __uint_as_float(__float_as_uint(v.y) & m),
                     __uint_as_float(__float_as_uint(v.z) & m),
                     __uint_as_float(__float_as_uint(v.w) & m));
}

// v with its elements j >= n zeroed (the columns of a quad past the image row), by masks as
// keep_if
__device__ __forceinline__ float4 keep_cols(float4 v, int n) {
  return make_float4(__uint_as_float(__float_as_uint(v.x) & (n > 0 ? 0xffffffffu : 0u)),
                     __uint_as_float(__float_as_uint(v.y) & (n > 1 ? 0xffffffffu : 0u)),
                     __uint_as_float(__float_as_uint(v.z) & (n > 2 ? 0xffffffffu : 0u)),
                     __uint_as_float(__float_as_uint(v.w) & (n > 3 ? 0xffffffffu : 0u)));
}

// the previous / next lane's value within rows of ROW consecutive lanes: a DPP row shift (a
// VALU op) where ROW divides the 16-lane DPP row, else a lane shuffle (an LDS permute and its
// wait); a row's first / last lane gets an unspecified value (callers substitute the padding)
template <int ROW>
__device__ __forceinline__ float lane_prev(float v) {
  if constexpr (ROW <= 16 && 16 % ROW == 0)
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));  // row_shr:1
  else
    return __shfl_up(v, 1, ROW);
}
template <int ROW>
__device__ __forceinline__ float lane_next(float v) {
  if constexpr (ROW <= 16 && 16 % ROW == 0)
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        0, __builtin_bit_cast(int, v), 0x101, 0xf, 0xf, true));  // row_shl:1
  else
    return __shfl_down(v, 1, ROW);
}

// a buffer resource over `bytes` bytes at `base` (wave-uniform inputs), for
// __builtin_amdgcn_raw_buffer_load_*: loads past the range return zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

}  // namespace conv
}  // namespace dd
