// GraNd per-example weight-gradient squared norms for Conv2d layers, on fp32 MFMA.
//
// For one example b, with U = im2col(act[b]) (T x d_a, t = output position, m = (c, ky, kx))
// and Gt = gout[b] viewed as T x d_g, the weight gradient is G = U^T Gt and we need ||G||_F^2.
//
//   DIRECT : G is computed tile by tile on MFMA (v_mfma_f32_32x32x2_f32), squared and summed
//            in registers; never written out.  2 T d_a d_g flop.
//   GHOST  : ||U^T Gt||^2 = sum_{t,t'} (U U^T)_{tt'} (Gt Gt^T)_{tt'}: both T x T Grams are
//            built on MFMA in accumulator registers and contracted elementwise.
//            2 T^2 (d_a + d_g) flop — the cheaper method once T^2 < T d_a d_g/(d_a+d_g).
//
// m is enumerated as (ky, kx, c) rather than (c, ky, kx): the norm is a sum over m, so any
// order is valid, and a fixed spatial shift per tile keeps activation reads contiguous in x.
// Each workgroup writes one partial sum; a reduce kernel adds them to sq_accum in a fixed
// order (deterministic, no float atomics).
#include "dd_common.h"
#include "dd_mfma.h"
#include "dd_pgram.h"
#include "dd_stem.h"

namespace dd {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct Geom {
  int cin, h, w, cout, ho, wo, kh, kw, stride, pad;
};

// XCD-aware remap (MI355X: blocks are dealt round-robin over 8 XCDs; keep runs of logical
// ids — the tiles of one example — on one XCD so its activation is fetched into one L2).
// Bijective for any grid size (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
__device__ __forceinline__ unsigned xcd_remap(unsigned orig, unsigned nwg) {
  const unsigned q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// ------------------------------------------------------------------------------------------
// DIRECT: workgroup = (example b, shift (ky,kx), 64 input channels, 64 output channels);
// K loop over output positions t in steps of 32 staged through LDS (register prefetch of the
// next step overlaps the 16 MFMAs of the current one).  4 waves in a 2x2 grid of 32x32 tiles.
// ------------------------------------------------------------------------------------------
constexpr int DBM = 64, DBN = 64, DBK = 32;

__global__ __launch_bounds__(256) void pegrad_direct_kernel(const float* __restrict__ act,
                                                            const float* __restrict__ gout,
                                                            Geom g, int n_cblk, int n_oblk,
                                                            const float* __restrict__ col_scale,
                                                            float* __restrict__ partial) {
  __shared__ float As[DBK][DBM + 1];
  __shared__ float Bs[DBK][DBN + 1];
  __shared__ float red[4];

  const int ntiles = g.kh * g.kw * n_cblk * n_oblk;
  const unsigned lid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = lid / ntiles;
  int tile = lid - b * ntiles;
  const int ob = tile % n_oblk;
  tile /= n_oblk;
  const int cb = tile % n_cblk;
  const int shift = tile / n_cblk;
  const int ky = shift / g.kw, kx = shift - (shift / g.kw) * g.kw;
  const int c0 = cb * DBM, o0 = ob * DBN;
  const int T = g.ho * g.wo, HW = g.h * g.w;
  const float* a_b = act + (size_t)b * g.cin * HW;
  const float* g_b = gout + (size_t)b * g.cout * T;

  const int tid = threadIdx.x, tl = tid & 31, rg = tid >> 5;
  float ra[8], rb[8];
  auto load = [&](int t0) {
    const int t = t0 + tl;
    const bool vt = t < T;
    const int oy = vt ? t / g.wo : 0;
    const int ox = vt ? t - oy * g.wo : 0;
    const int iy = oy * g.stride + ky - g.pad, ix = ox * g.stride + kx - g.pad;
    const bool va = vt && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
    const int off = iy * g.w + ix;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + rg + 8 * j;
      ra[j] = (va && c < g.cin) ? a_b[(size_t)c * HW + off] : 0.f;
      const int o = o0 + rg + 8 * j;
      rb[j] = (vt && o < g.cout) ? g_b[(size_t)o * T + t] : 0.f;
    }
  };

  const int lane = tid & 63, wv = tid >> 6, wm = wv & 1, wn = wv >> 1;
  const int kr = lane >> 5, col = lane & 31;
  floatx16 acc = {0};
  const int nk = (T + DBK - 1) / DBK;
  load(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      As[tl][rg + 8 * j] = ra[j];
      Bs[tl][rg + 8 * j] = rb[j];
    }
    __syncthreads();
    if (kt + 1 < nk) load((kt + 1) * DBK);
#pragma unroll
    for (int kk = 0; kk < DBK / 2; ++kk) {
      const float av = As[2 * kk + kr][wm * 32 + col];
      const float bv = Bs[2 * kk + kr][wn * 32 + col];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
  }
  // C/D layout: column = lane & 31 -> output channel o; all 16 registers share it
  const int o = o0 + wn * 32 + col;
  float s2 = 1.f;
  if (col_scale) {
    const float s = (o < g.cout) ? col_scale[o] : 0.f;
    s2 = s * s;
  }
  float v = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) v += acc[r] * acc[r];
  v = wave_sum(v * s2);
  if (lane == 0) red[wv] = v;
  __syncthreads();
  if (tid == 0) partial[lid] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ------------------------------------------------------------------------------------------
// DIRECT 1x1, split-bf16 (the Bottleneck conv1 / conv3 and projection norms of ResNet-50, the
// ResNet-18 shortcut): G = U^T g is a [cin x cout] GEMM over the T output positions (K =
// positions).  Workgroup = (example b, 64 LC input channels, 64 (4 / LC) output channels),
// LC = waves along c (1, 2 or 4: the layout the channel counts fill); each wave 64 c x 64 o
// (2 x 2 accumulators of v_mfma_f32_32x32x16_bf16).  K steps of 32 positions: the step's
// act and g rows are loaded coalesced (float4 along positions; register prefetch of the next
// step under the current MFMAs), split into bf16 hi / lo and staged as [hi|lo][row][t]; an
// MFMA operand (8 consecutive positions of one row) is then one ds_read_b128 per plane.
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

template <int S, int LC>
__global__ __launch_bounds__(256) void pegrad_direct1x1_kernel(const float* __restrict__ act,
                                                               const float* __restrict__ gout,
                                                               Geom g, int n_cblk, int n_oblk,
                                                               const float* __restrict__ col_scale,
                                                               float* __restrict__ partial) {
  constexpr int LO = 4 / LC;
  constexpr int MC = 64 * LC, MO = 64 * LO, R = MC + MO;  // staged rows: act, then g
  constexpr int KT = 32;                                   // positions per K step
  constexpr int RS = KT * 2 + 16;  // bytes per staged bf16 row (+16: conflict-free b128 reads)
  constexpr int PL = R * RS;       // one plane
  constexpr int NL = R * (KT / 4) / 256;  // float4 loads per thread per step
  static_assert(R * (KT / 4) % 256 == 0, "whole float4 loads per thread");
  __shared__ __attribute__((aligned(16))) char lds[2 * PL];
  __shared__ float red[4];
  const int ntiles = n_cblk * n_oblk;
  const unsigned lid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = lid / ntiles;
  const int tile = lid - b * ntiles;
  const int ob = tile % n_oblk, cb = tile / n_oblk;
  const int c0 = cb * MC, o0 = ob * MO;
  const int T = g.ho * g.wo, HW = g.h * g.w;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* __restrict__ a_b = act + (size_t)b * g.cin * HW;
  const float* __restrict__ g_b = gout + (size_t)b * g.cout * T;
  // float4 path: 4 consecutive positions share an output row (and, at stride 2, read input
  // columns 2 ox .. 2 ox + 6 of one row: two aligned float4)
  const bool vec = T % 4 == 0 && (S == 1 || g.wo % 4 == 0) && HW % 4 == 0;

  float4 rv[NL];
  auto load = [&](int t0) {
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int q = tid + 256 * k, row = q / (KT / 4), x4 = q % (KT / 4);
      const int t = t0 + 4 * x4;
      const bool isa = row < MC;
      const int ch = isa ? c0 + row : o0 + row - MC;
      const bool rok = ch < (isa ? g.cin : g.cout);
      const float* base = isa ? a_b + (size_t)(rok ? ch : 0) * HW
                              : g_b + (size_t)(rok ? ch : 0) * T;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (vec) {
        if (rok && t < T) {
          if (!isa || S == 1) {
            const float4 u = *reinterpret_cast<const float4*>(base + t);
            v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
          } else {
            const int oy = t / g.wo, ox = t - oy * g.wo;
            const float* src = base + (size_t)oy * S * g.w + ox * S;
            const float4 u0 = *reinterpret_cast<const float4*>(src);
            const float4 u1 = *reinterpret_cast<const float4*>(src + 4);
            v[0] = u0.x; v[1] = u0.z; v[2] = u1.x; v[3] = u1.z;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int tj = t + j;
          if (rok && tj < T) {
            int ia = tj;
            if (isa && S != 1) {
              const int oy = tj / g.wo, ox = tj - oy * g.wo;
              ia = oy * S * g.w + ox * S;
            }
            v[j] = base[ia];
          }
        }
      }
      rv[k] = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int q = tid + 256 * k, row = q / (KT / 4), x4 = q % (KT / 4);
      const float f[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
      bf16x4_t hv, lv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const __bf16 x = (__bf16)f[j];
        hv[j] = x;
        lv[j] = (__bf16)(f[j] - (float)x);
      }
      char* p = lds + row * RS + x4 * 8;
      *reinterpret_cast<bf16x4_t*>(p) = hv;
      *reinterpret_cast<bf16x4_t*>(p + PL) = lv;
    }
  };

  const int r = lane & 31, h = lane >> 5;
  const int wc = wv % LC, wo_ = wv / LC;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx16{0};
  load(0);
  for (int t0 = 0; t0 < T; t0 += KT) {
    __syncthreads();  // the previous step's fragment reads are done
    stage();
    __syncthreads();
    if (t0 + KT < T) load(t0 + KT);  // the next step's rows load under these MFMAs
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t ah[2], al[2], gh[2], gl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const char* pa = lds + (wc * 64 + 32 * i + r) * RS + (16 * s + 8 * h) * 2;
        const char* pg = lds + (MC + wo_ * 64 + 32 * i + r) * RS + (16 * s + 8 * h) * 2;
        ah[i] = *reinterpret_cast<const bf16x8_t*>(pa);
        al[i] = *reinterpret_cast<const bf16x8_t*>(pa + PL);
        gh[i] = *reinterpret_cast<const bf16x8_t*>(pg);
        gl[i] = *reinterpret_cast<const bf16x8_t*>(pg + PL);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          floatx16 d = acc[i][j];
          d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], gh[j], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], gl[j], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], gh[j], d, 0, 0, 0);
          acc[i][j] = d;
        }
    }
  }
  // D[c][o]: column o = lane & 31 of block j, the 16 registers run over c
  float v = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int o = o0 + wo_ * 64 + 32 * j + r;
    float s2 = 1.f;
    if (col_scale) {
      const float sc = o < g.cout ? col_scale[o] : 0.f;
      s2 = sc * sc;
    }
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) q += acc[i][j][k] * acc[i][j][k];
    v += q * s2;
  }
  v = wave_sum(v);
  if (lane == 0) red[wv] = v;
  __syncthreads();
  if (tid == 0) partial[lid] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ------------------------------------------------------------------------------------------
// GHOST, general T: workgroup = (example b, 64x64 tile (bi, bj) of the T x T Grams); 4 waves
// in a 2x2 grid of 32x32 tiles.  Operands come straight from global memory (lanes run along
// t, so each load is contiguous in x; both operands share the cache lines).  The A and B
// fragments of U U^T are the same im2col column read at two row blocks.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pegrad_ghost64_kernel(const float* __restrict__ act,
                                                             const float* __restrict__ gout,
                                                             Geom g, int nT,
                                                             const float* __restrict__ col_scale,
                                                             float* __restrict__ partial) {
  __shared__ float red[4];
  const int ntiles = nT * nT;
  const unsigned lid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = lid / ntiles;
  const int tile = lid - b * ntiles;
  const int bi = tile / nT, bj = tile - (tile / nT) * nT;
  const int T = g.ho * g.wo, HW = g.h * g.w;
  const float* a_b = act + (size_t)b * g.cin * HW;
  const float* g_b = gout + (size_t)b * g.cout * T;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int ti = bi * 64 + (wv & 1) * 32 + r;
  const int tj = bj * 64 + (wv >> 1) * 32 + r;
  const bool vti = ti < T, vtj = tj < T;
  const int oyi = vti ? ti / g.wo : 0, oxi = vti ? ti - oyi * g.wo : 0;
  const int oyj = vtj ? tj / g.wo : 0, oxj = vtj ? tj - oyj * g.wo : 0;

  floatx16 accA = {0}, accG = {0};
  const int npair = (g.cin + 1) / 2;
  for (int ky = 0; ky < g.kh; ++ky) {
    for (int kx = 0; kx < g.kw; ++kx) {
      const int iyi = oyi * g.stride + ky - g.pad, ixi = oxi * g.stride + kx - g.pad;
      const int iyj = oyj * g.stride + ky - g.pad, ixj = oxj * g.stride + kx - g.pad;
      const bool vi = vti && iyi >= 0 && iyi < g.h && ixi >= 0 && ixi < g.w;
      const bool vj = vtj && iyj >= 0 && iyj < g.h && ixj >= 0 && ixj < g.w;
      const float* pi = a_b + (vi ? iyi * g.w + ixi : 0);
      const float* pj = a_b + (vj ? iyj * g.w + ixj : 0);
      int p = 0;
      for (; p + 4 <= npair; p += 4) {
        float ai[4], aj[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = 2 * (p + u) + h;
          ai[u] = (vi && c < g.cin) ? pi[(size_t)c * HW] : 0.f;
          aj[u] = (vj && c < g.cin) ? pj[(size_t)c * HW] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          accA = __builtin_amdgcn_mfma_f32_32x32x2f32(ai[u], aj[u], accA, 0, 0, 0);
      }
      for (; p < npair; ++p) {
        const int c = 2 * p + h;
        const float ai = (vi && c < g.cin) ? pi[(size_t)c * HW] : 0.f;
        const float aj = (vj && c < g.cin) ? pj[(size_t)c * HW] : 0.f;
        accA = __builtin_amdgcn_mfma_f32_32x32x2f32(ai, aj, accA, 0, 0, 0);
      }
    }
  }
  const int opair = (g.cout + 1) / 2;
  for (int p = 0; p < opair; ++p) {
    const int o = 2 * p + h;
    const bool vo = o < g.cout;
    const float s = (col_scale && vo) ? col_scale[o] : 1.f;
    const float gi = (vti && vo) ? g_b[(size_t)o * T + ti] * s : 0.f;
    const float gj = (vtj && vo) ? g_b[(size_t)o * T + tj] * s : 0.f;
    accG = __builtin_amdgcn_mfma_f32_32x32x2f32(gi, gj, accG, 0, 0, 0);
  }
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) v += accA[k] * accG[k];
  v = wave_sum(v);
  if (lane == 0) red[wv] = v;
  __syncthreads();
  if (tid == 0) partial[lid] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ------------------------------------------------------------------------------------------
// GHOST, T <= 16: one wave per example, v_mfma_f32_16x16x4_f32 (lane: t = lane & 15,
// k-slot = lane >> 4).  A and B fragments of both Grams are the same register.  Two
// accumulators alternate to cover the 40-cycle dependent latency of the 16x16x4 form.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pegrad_ghost16_kernel(const float* __restrict__ act,
                                                             const float* __restrict__ gout,
                                                             int64_t B, Geom g,
                                                             const float* __restrict__ col_scale,
                                                             float* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // uniform per wave
  const int T = g.ho * g.wo, HW = g.h * g.w;
  const float* a_b = act + (size_t)b * g.cin * HW;
  const float* g_b = gout + (size_t)b * g.cout * T;
  const int t = lane & 15, kq = lane >> 4;
  const bool vt = t < T;
  const int oy = vt ? t / g.wo : 0, ox = vt ? t - oy * g.wo : 0;

  floatx4 a0 = {0}, a1 = {0}, gA = {0}, gB = {0};
  const int nq = (g.cin + 3) / 4;
  for (int ky = 0; ky < g.kh; ++ky) {
    for (int kx = 0; kx < g.kw; ++kx) {
      const int iy = oy * g.stride + ky - g.pad, ix = ox * g.stride + kx - g.pad;
      const bool v = vt && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
      const float* p = a_b + (v ? iy * g.w + ix : 0);
      int q = 0;
      for (; q + 4 <= nq; q += 4) {
        float x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = 4 * (q + u) + kq;
          x[u] = (v && c < g.cin) ? p[(size_t)c * HW] : 0.f;
        }
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[0], x[0], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[1], x[1], a1, 0, 0, 0);
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[2], x[2], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[3], x[3], a1, 0, 0, 0);
      }
      for (; q < nq; ++q) {
        const int c = 4 * q + kq;
        const float x = (v && c < g.cin) ? p[(size_t)c * HW] : 0.f;
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, a0, 0, 0, 0);
      }
    }
  }
  const int no = (g.cout + 3) / 4;
  int q = 0;
  for (; q + 2 <= no; q += 2) {
    float x[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int o = 4 * (q + u) + kq;
      const bool vo = o < g.cout;
      const float s = (col_scale && vo) ? col_scale[o] : 1.f;
      x[u] = (vt && vo) ? g_b[(size_t)o * T + t] * s : 0.f;
    }
    gA = __builtin_amdgcn_mfma_f32_16x16x4f32(x[0], x[0], gA, 0, 0, 0);
    gB = __builtin_amdgcn_mfma_f32_16x16x4f32(x[1], x[1], gB, 0, 0, 0);
  }
  for (; q < no; ++q) {
    const int o = 4 * q + kq;
    const bool vo = o < g.cout;
    const float s = (col_scale && vo) ? col_scale[o] : 1.f;
    const float x = (vt && vo) ? g_b[(size_t)o * T + t] * s : 0.f;
    gA = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, gA, 0, 0, 0);
  }
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) v += (a0[k] + a1[k]) * (gA[k] + gB[k]);
  v = wave_sum(v);
  if (lane == 0) partial[b] = v;
}

// ------------------------------------------------------------------------------------------
// DIRECT 3x3 / stride 1 / pad 1, split-bf16 ("bf16x3") MFMA, all nine taps per workgroup.
//
// workgroup = (example b, 64 input channels, 64 output channels, all 9 taps); 4 waves in a
// 2x2 grid, each owning 32 c x 32 o x 9 taps = 9 accumulators of v_mfma_f32_32x32x16_bf16.
// The K loop walks output rows: each step covers R = 32/W rows (32 output positions = two
// k16 sub-steps).  Input rows live in an LDS ring of S = 2R+2 slots (window of R+2 rows plus
// R prefetched rows), so every activation and output-gradient byte is read from HBM once.
// Each input row is stored three times, pre-shifted by kx-1, so every A fragment is an
// aligned 16-byte ds_read_b128; rows are padded to an odd number of 16-byte units, which
// makes the ds_read_b128 lane groups conflict-free.  Operands are split v = hi + lo (both
// bf16, lo = bf16(v - hi)) and each product is hi*hi + hi*lo + lo*hi: ~2^-16 relative per
// product, fp32 accumulation (the norm tolerance is 1e-3).  Global loads for step k+1 are
// issued before step k's MFMAs and written to LDS after them: one barrier per step.
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// STR = 2 (a stage's downsampling head, 3x3 / stride 2 / pad 1): W is the output width; the
// input rows (width 2W) are staged decimated, image kx holding a[.., 2 xo + kx - 1], so the
// A fragments keep the stride-1 addressing; a step's R output rows read 2R + 1 input rows.
template <int W, int STR>
struct D3Cfg {
  static constexpr int R = 32 / W;            // output rows per step
  static constexpr int NEW = STR * R;         // input rows entering the window per step
  static constexpr int WIN = STR == 1 ? R + 2 : 2 * R + 1;  // input rows a step reads
  static constexpr int S = WIN + NEW;         // ring slots (window + prefetched rows)
  static constexpr int WI = STR * W;          // input row width
  // channel row pitch: an odd number of 16-B units (conflict-free b128 reads); unpadded at
  // stride 2, where the 9-slot ring of padded rows would exceed the 160 KB of LDS (2-way
  // conflicts on the A reads, small beside the MFMA time)
  static constexpr int CS = ((W * 2 / 16) % 2 == 1 || STR == 2) ? W * 2 : W * 2 + 16;
  static constexpr int PLANE = 64 * CS;       // one (slot, kx, hi|lo) plane, bytes
  static constexpr int ACT_BYTES = S * 3 * 2 * PLANE;
  static constexpr int GCS = 80;              // g stage: 32 t bf16 = 64 B + 16 pad
  static constexpr int GPLANE = 64 * GCS;
  static constexpr int G_BYTES = 2 * 2 * GPLANE;  // [buf][hi|lo][o][t]
  static constexpr int LDS = ACT_BYTES + G_BYTES;
  static constexpr int TPR = WI / 4;          // threads per input row of one channel
  static constexpr int NA = NEW * 64 * WI / 4 / 256;  // activation float4 per thread per step
  static_assert(NEW * 64 * WI / 4 % 256 == 0, "whole float4 rounds");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ void split4(float4 v, bf16x4& hi, bf16x4& lo) {
  const __bf16 h0 = (__bf16)v.x, h1 = (__bf16)v.y, h2 = (__bf16)v.z, h3 = (__bf16)v.w;
  hi = bf16x4{h0, h1, h2, h3};
  lo = bf16x4{(__bf16)(v.x - (float)h0), (__bf16)(v.y - (float)h1), (__bf16)(v.z - (float)h2),
              (__bf16)(v.w - (float)h3)};
}

// TG = 2: two tap groups of 4 waves (taps 0-4 and 5-8), 512 threads: each wave holds 5 (4)
// tap accumulators instead of 9, so two waves fit per SIMD and each hides the other's LDS
// latency and barrier waits (at TG = 1 the kernel runs one wave per SIMD with 9 accumulators).
// ||G||^2 is a sum over taps, so the groups' squared sums add with no exchange of G.
template <int W, int STR, int TG>
__global__ __launch_bounds__(256 * TG, 1) void pegrad_direct3x3_kernel(
    const float* __restrict__ act, const float* __restrict__ gout, int cin, int cout, int H,
    int n_cblk, int n_oblk, const float* __restrict__ col_scale, float* __restrict__ partial) {
  using C = D3Cfg<W, STR>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* act_lds = smem;
  char* g_lds = smem + C::ACT_BYTES;

  const unsigned lid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_ex = n_cblk * n_oblk;
  const int b = lid / per_ex;
  const int rem = lid - b * per_ex;
  const int c0 = (rem / n_oblk) * 64, o0 = (rem % n_oblk) * 64;
  const int HW = H * W;                       // output positions
  const int HI = STR * H, HWI = HI * C::WI;    // input rows, positions
  const float* a_b = act + (size_t)b * cin * HWI;
  const float* g_b = gout + (size_t)b * cout * HW;

  constexpr int NTH = 256 * TG;
  static_assert(C::NA % TG == 0, "whole staging rounds per tap group");
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wq = wv & 3, tg = __builtin_amdgcn_readfirstlane(wv >> 2);
  const int wc = wq & 1, wo = wq >> 1, r = lane & 31, h = lane >> 5;

  // ---- staging: 2 float4 of activations (one input row slice) + 2 float4 of gradients.
  // Loads are unconditional from clamped addresses and out-of-range values are zeroed when
  // they are converted: a predicated `v = cond ? load : 0` makes hipcc branch around the load
  // and wait vmcnt(0) right behind it, which would serialise the prefetch.
  constexpr int NAT = C::NA / TG, NGT = 2 / TG;  // float4 per thread: activations, gradients
  float4 ra[NAT], rg[NGT];
  bool va[NAT], vg[NGT];
  auto load_rows = [&](int ir0, int nrows, int tstep) {
#pragma unroll
    for (int k = 0; k < NAT; ++k) {
      const int idx = tid + NTH * k;
      const int x4 = idx % C::TPR, c = (idx / C::TPR) % 64, rr = idx / (C::TPR * 64);
      const int ir = ir0 + rr;
      const int cg = c0 + c;
      va[k] = rr < nrows && ir >= 0 && ir < HI && cg < cin;
      const int irc = ir < 0 ? 0 : (ir >= HI ? HI - 1 : ir);
      const int cgc = cg < cin ? cg : cin - 1;
      ra[k] = *reinterpret_cast<const float4*>(a_b + (size_t)cgc * HWI + irc * C::WI + x4 * 4);
    }
    if (tstep >= 0) {
      const int ts = tstep < HW / 32 ? tstep : HW / 32 - 1;  // last step prefetches a dummy
#pragma unroll
      for (int k = 0; k < NGT; ++k) {
        const int idx = tid + NTH * k;
        const int o = idx >> 3, t4 = idx & 7;
        const int og = o0 + o;
        vg[k] = og < cout;
        const int ogc = og < cout ? og : cout - 1;
        rg[k] = *reinterpret_cast<const float4*>(g_b + (size_t)ogc * HW + ts * 32 + t4 * 4);
      }
    }
  };
  // (a bitwise AND: a select on a loaded value compiles into a branch around the wait for the
  // load, which would split the scheduling region the staging interleaves with)
  auto zero_if = [](float4 v, bool ok) { return conv::keep_if(v, ok); };
  // nrows < R only in the prologue (rows beyond it are skipped); in the main loop every
  // store is unconditional so the staging interleaves with the MFMAs in one basic block
  auto store_rows = [&](int ir0, int nrows, int gbuf) {
#pragma unroll
    for (int k = 0; k < NAT; ++k) {
      const int idx = tid + NTH * k;
      const int x4 = idx % C::TPR, c = (idx / C::TPR) % 64, rr = idx / (C::TPR * 64);
      if (nrows < C::NEW && rr >= nrows) continue;  // prologue only; uniform per row group
      const int slot = (ir0 + rr + 1) % C::S;
      const float4 v = zero_if(ra[k], va[k]);
      if constexpr (STR == 1) {
        // the three shifted copies from one packed split; halo columns from the neighbouring
        // lanes of the row (DPP row shifts: TPR <= 16 lanes per row)
        static_assert(C::TPR <= 16 && 16 % C::TPR == 0, "row of lanes inside a DPP row");
        uint2 hs[3], ls[3];
        conv::split_shift3(v, x4 == 0, x4 == C::TPR - 1, hs, ls);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          char* base = act_lds + ((slot * 3 + kx) * 2) * C::PLANE + c * C::CS + x4 * 8;
          *reinterpret_cast<uint2*>(base) = hs[kx];
          *reinterpret_cast<uint2*>(base + C::PLANE) = ls[kx];
        }
      } else {
        float left = conv::lane_prev<C::TPR>(v.w);
        if (x4 == 0) left = 0.f;
        // input columns 4 x4 - 1 .. 4 x4 + 3 -> decimated columns 2 x4, 2 x4 + 1 of image kx
        // (input column 2 xo + kx - 1)
        const float f[5] = {left, v.x, v.y, v.z, v.w};
        __bf16 hv[5], lv[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          hv[i] = (__bf16)f[i];
          lv[i] = (__bf16)(f[i] - (float)hv[i]);
        }
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          char* base = act_lds + ((slot * 3 + kx) * 2) * C::PLANE + c * C::CS + x4 * 4;
          *reinterpret_cast<bf16x2*>(base) = bf16x2{hv[kx], hv[kx + 2]};
          *reinterpret_cast<bf16x2*>(base + C::PLANE) = bf16x2{lv[kx], lv[kx + 2]};
        }
      }
    }
    if (gbuf >= 0) {
#pragma unroll
      for (int k = 0; k < NGT; ++k) {
        const int idx = tid + NTH * k;
        const int o = idx >> 3, t4 = idx & 7;
        bf16x4 hi, lo;
        split4(zero_if(rg[k], vg[k]), hi, lo);
        char* base = g_lds + ((gbuf * 2) * 64 + o) * C::GCS + t4 * 8;
        *reinterpret_cast<bf16x4*>(base) = hi;
        *reinterpret_cast<bf16x4*>(base + C::GPLANE) = lo;
      }
    }
  };

  constexpr int NACC = TG == 1 ? 9 : 5;  // accumulators per wave: its tap group's taps
  floatx16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = floatx16{0};

  const int nsteps = H / C::R;
  // prologue: input rows -1 .. WIN - 2 (the first window) and the gradients of step 0
  for (int ir0 = -1; ir0 < C::WIN - 1; ir0 += C::NEW) {
    const int n = C::NEW < C::WIN - 1 - ir0 ? C::NEW : C::WIN - 1 - ir0;
    load_rows(ir0, n, ir0 == -1 ? 0 : -1);
    store_rows(ir0, n, ir0 == -1 ? 0 : -1);
  }
  __syncthreads();

  // one fragment: B hi / lo (T < 0) or tap T's A hi / lo, of sub-step s
  auto frag = [&](int y0, int gbuf, int s, int t, int lo) -> bf16x8 {
    const int tl = 16 * s + 8 * h;
    const int ro = tl / W, x = tl % W;
    if (t < 0) {
      const char* gb = g_lds + ((gbuf * 2) * 64 + wo * 32 + r) * C::GCS + tl * 2;
      return *reinterpret_cast<const bf16x8*>(gb + lo * C::GPLANE);
    }
    const int ky = t / 3, kx = t % 3;
    const int slot = (STR * (y0 + ro) + ky) % C::S;
    const char* ab = act_lds + ((slot * 3 + kx) * 2) * C::PLANE + (wc * 32 + r) * C::CS + x * 2;
    return *reinterpret_cast<const bf16x8*>(ab + lo * C::PLANE);
  };
  // one step of tap group (T0, NTAP): NTAP taps from T0 (compile-time, so every fragment
  // address and accumulator index folds)
  auto group_step = [&](int y0, int gbuf, int inext, auto T0c, auto NTc) {
    constexpr int T0 = decltype(T0c)::value, NTAP = decltype(NTc)::value;
    bf16x8 bh0, bl0, ah0[NTAP], al0[NTAP], bh1, bl1, ah1[NTAP], al1[NTAP];
    // only B and the first tap of sub-step 0 before its first MFMA; its other reads and
    // sub-step 1's B go two per MFMA gap behind the first NTAP MFMAs, then sub-step 1's A
    // reads one per gap, in this fixed order
    bh0 = frag(y0, gbuf, 0, -1, 0);
    bl0 = frag(y0, gbuf, 0, -1, 1);
    ah0[0] = frag(y0, gbuf, 0, T0, 0);
    al0[0] = frag(y0, gbuf, 0, T0, 1);
    auto rd = [&](int j) {  // the j-th read behind the MFMAs
      constexpr int J0 = 2 * (NTAP - 1), J1 = J0 + 2, J2 = J1 + 2 * NTAP;
      if (j < J0) {
        if (j & 1) al0[1 + j / 2] = frag(y0, gbuf, 0, T0 + 1 + j / 2, 1);
        else ah0[1 + j / 2] = frag(y0, gbuf, 0, T0 + 1 + j / 2, 0);
      } else if (j < J1) {
        (j == J0 ? bh1 : bl1) = frag(y0, gbuf, 1, -1, j - J0);
      } else if (j < J2) {
        if ((j - J1) & 1) al1[(j - J1) / 2] = frag(y0, gbuf, 1, T0 + (j - J1) / 2, 1);
        else ah1[(j - J1) / 2] = frag(y0, gbuf, 1, T0 + (j - J1) / 2, 0);
      }
    };
#pragma unroll
    for (int i = 0; i < NTAP; ++i) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        __builtin_amdgcn_sched_barrier(0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q == 2 ? al0[i] : ah0[i],
                                                         q == 1 ? bl0 : bh0, acc[i], 0, 0, 0);
        const int g = 3 * i + q;  // gap g: reads j0 .. j0 + nr - 1
        const int j0 = g < NTAP ? 2 * g : NTAP + g, nr = g < NTAP ? 2 : 1;
        rd(j0);
        if (nr == 2) rd(j0 + 1);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // sub-step 1 MFMAs; the next step's rows are converted and staged behind them (those
    // slots / the other gradient buffer are not read in this step)
#pragma unroll
    for (int i = 0; i < NTAP; ++i) {
      floatx16 a = acc[i];
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1[i], bh1, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1[i], bl1, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al1[i], bh1, a, 0, 0, 0);
      acc[i] = a;
    }
    store_rows(inext, C::NEW, gbuf ^ 1);
#pragma unroll
    for (int i = 0; i < 3 * NTAP - 1; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 1);  // 4 VALU
      __builtin_amdgcn_sched_group_barrier(0x080, 1, 1);  // 1 LDS op
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I5 = std::integral_constant<int, 5>;
  for (int st = 0; st < nsteps; ++st) {
    const int y0 = st * C::R;
    // prefetch the next step's rows (on the last step: clamped, harmless, never read)
    const int inext = STR * y0 + C::WIN - 1;  // first input row past this step's window
    load_rows(inext, C::NEW, st + 1);
    const int gbuf = st & 1;
    if constexpr (TG == 1) {
      group_step(y0, gbuf, inext, I0{}, std::integral_constant<int, 9>{});
    } else if (tg == 0) {
      group_step(y0, gbuf, inext, I0{}, I5{});
    } else {
      group_step(y0, gbuf, inext, I5{}, std::integral_constant<int, 4>{});
    }
    __syncthreads();
  }

  const int o = o0 + wo * 32 + r;  // C/D column = lane & 31
  float s2 = (o < cout) ? 1.f : 0.f;
  if (col_scale && o < cout) {
    const float sc = col_scale[o];
    s2 = sc * sc;
  }
  float v = 0.f;
  const int ntap = TG == 1 ? 9 : (tg == 0 ? 5 : 4);
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int k = 0; k < 16; ++k) v += i < ntap ? acc[i][k] * acc[i][k] : 0.f;
  v = wave_sum(v * s2);
  float* red = reinterpret_cast<float*>(smem);
  if (lane == 0) red[wv] = v;
  __syncthreads();
  if (tid == 0) {
    float sum = (red[0] + red[1]) + (red[2] + red[3]);
    if constexpr (TG == 2) sum += (red[4] + red[5]) + (red[6] + red[7]);
    partial[lid] = sum;
  }
}

// tap groups of the direct3x3 kernels: one group of 4 waves (9 accumulators, one wave per
// SIMD) by default; DD_D3_TG=2 takes the two-group form (5 / 4 accumulators, two waves per
// SIMD), measured 0.76x at 32x32 and 0.90x on the persistent 16x16 kernel (in-process A/B,
// profiles/r04_conv/ab_pegrad_tg2_rejected.txt): the second wave re-reads the B fragments and
// the LDS traffic per MFMA rises, which costs more than the hidden latency gains
static int d3_tap_groups() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DD_D3_TG");
    v = (e && e[0] == '2') ? 2 : 1;
  }
  return v;
}

template <int W, int STR, int TG>
static void launch_direct3x3_tg(const float* act, const float* gout, int64_t B, int cin,
                                int cout, int H, const float* col_scale, float* partial,
                                hipStream_t st) {
  using C = D3Cfg<W, STR>;
  const int ncb = (int)ceil_div(cin, 64), nob = (int)ceil_div(cout, 64);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pegrad_direct3x3_kernel<W, STR, TG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr_set = true;
  }
  pegrad_direct3x3_kernel<W, STR, TG><<<(unsigned)(B * ncb * nob), 256 * TG, C::LDS, st>>>(
      act, gout, cin, cout, H, ncb, nob, col_scale, partial);
}

template <int W, int STR>
static void launch_direct3x3(const float* act, const float* gout, int64_t B, int cin, int cout,
                             int H, const float* col_scale, float* partial, hipStream_t st) {
  if (d3_tap_groups() == 1)
    launch_direct3x3_tg<W, STR, 1>(act, gout, B, cin, cout, H, col_scale, partial, st);
  else
    launch_direct3x3_tg<W, STR, 2>(act, gout, B, cin, cout, H, col_scale, partial, st);
}

// Persistent where it pays (16-wide output maps: 8 steps per tile): one workgroup per CU walks
// the tiles t = blockIdx.x, + gridDim.x, ... (logical tile xcd_remap(t, total): a run of an
// example's tiles per XCD).  A tile's last step loads the next tile's first window and step-0
// gradients into registers, so the next prologue's HBM latency hides under those MFMAs; only
// its conversion into LDS is exposed.  (The prologue was 9-15 % of a one-tile workgroup;
// measured 1.04x at 16x16 and 1.06x on the 32 -> 16 head, 0.95x at 32x32 — 32 steps per
// tile, where pegrad_direct3x3_kernel stays: one tile per workgroup.)
template <int W, int STR, int TG>
__global__ __launch_bounds__(256 * TG, 1) void pegrad_direct3x3p_kernel(
    const float* __restrict__ act, const float* __restrict__ gout, int cin, int cout, int H,
    int n_cblk, int n_oblk, const float* __restrict__ col_scale, float* __restrict__ partial,
    int total) {
  using C = D3Cfg<W, STR>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* act_lds = smem;
  char* g_lds = smem + C::ACT_BYTES;
  float* red = reinterpret_cast<float*>(smem + C::LDS);  // 4 TG floats past the staging

  const int per_ex = n_cblk * n_oblk;
  const int HW = H * W;                       // output positions
  const int HI = STR * H, HWI = HI * C::WI;    // input rows, positions
  int lid, c0, o0;
  const float *a_b, *g_b;
  auto set_tile = [&](int t) {
    lid = (int)xcd_remap((unsigned)t, (unsigned)total);
    const int b = lid / per_ex;
    const int rem = lid - b * per_ex;
    c0 = (rem / n_oblk) * 64;
    o0 = (rem % n_oblk) * 64;
    a_b = act + (size_t)b * cin * HWI;
    g_b = gout + (size_t)b * cout * HW;
  };

  constexpr int NTH = 256 * TG;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wq = wv & 3, tg = __builtin_amdgcn_readfirstlane(wv >> 2);
  const int wc = wq & 1, wo = wq >> 1, r = lane & 31, h = lane >> 5;

  // ---- staging: 2 float4 of activations (one input row slice) + 2 float4 of gradients.
  // Loads are unconditional from clamped addresses and out-of-range values are zeroed when
  // they are converted: a predicated `v = cond ? load : 0` makes hipcc branch around the load
  // and wait vmcnt(0) right behind it, which would serialise the prefetch.
  // NK float4 of activation rows per thread: C::NA (NEW rows, a step's prefetch) or NAW (the
  // WIN rows of a tile's first window)
  constexpr int NAW = C::WIN * 64 * C::WI / 4 / NTH;
  static_assert(C::WIN * 64 * C::WI / 4 % NTH == 0, "whole float4 rounds");
  static_assert(C::NA % TG == 0, "whole staging rounds per tap group");
  constexpr int NGT = 2 / TG;  // gradient float4 per thread
  float4 ra[NAW], rg[NGT];
  bool va[NAW], vg[NGT];
  auto load_rows = [&](auto NKc, int ir0, int nrows, int tstep) {
    constexpr int NK = decltype(NKc)::value;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int idx = tid + NTH * k;
      const int x4 = idx % C::TPR, c = (idx / C::TPR) % 64, rr = idx / (C::TPR * 64);
      const int ir = ir0 + rr;
      const int cg = c0 + c;
      va[k] = rr < nrows && ir >= 0 && ir < HI && cg < cin;
      const int irc = ir < 0 ? 0 : (ir >= HI ? HI - 1 : ir);
      const int cgc = cg < cin ? cg : cin - 1;
      ra[k] = *reinterpret_cast<const float4*>(a_b + (size_t)cgc * HWI + irc * C::WI + x4 * 4);
    }
    if (tstep >= 0) {
      const int ts = tstep < HW / 32 ? tstep : HW / 32 - 1;  // last step prefetches a dummy
#pragma unroll
      for (int k = 0; k < NGT; ++k) {
        const int idx = tid + NTH * k;
        const int o = idx >> 3, t4 = idx & 7;
        const int og = o0 + o;
        vg[k] = og < cout;
        const int ogc = og < cout ? og : cout - 1;
        rg[k] = *reinterpret_cast<const float4*>(g_b + (size_t)ogc * HW + ts * 32 + t4 * 4);
      }
    }
  };
  // (a bitwise AND: a select on a loaded value compiles into a branch around the wait for the
  // load, which would split the scheduling region the staging interleaves with)
  auto zero_if = [](float4 v, bool ok) { return conv::keep_if(v, ok); };
  // nrows < R only in the prologue (rows beyond it are skipped); in the main loop every
  // store is unconditional so the staging interleaves with the MFMAs in one basic block
  auto store_rows = [&](auto NKc, int ir0, int gbuf) {
    constexpr int NK = decltype(NKc)::value;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int idx = tid + NTH * k;
      const int x4 = idx % C::TPR, c = (idx / C::TPR) % 64, rr = idx / (C::TPR * 64);
      const int slot = (ir0 + rr + 1) % C::S;
      const float4 v = zero_if(ra[k], va[k]);
      if constexpr (STR == 1) {
        // the three shifted copies from one packed split; halo columns from the neighbouring
        // lanes of the row (DPP row shifts: TPR <= 16 lanes per row)
        static_assert(C::TPR <= 16 && 16 % C::TPR == 0, "row of lanes inside a DPP row");
        uint2 hs[3], ls[3];
        conv::split_shift3(v, x4 == 0, x4 == C::TPR - 1, hs, ls);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          char* base = act_lds + ((slot * 3 + kx) * 2) * C::PLANE + c * C::CS + x4 * 8;
          *reinterpret_cast<uint2*>(base) = hs[kx];
          *reinterpret_cast<uint2*>(base + C::PLANE) = ls[kx];
        }
      } else {
        float left = conv::lane_prev<C::TPR>(v.w);
        if (x4 == 0) left = 0.f;
        // input columns 4 x4 - 1 .. 4 x4 + 3 -> decimated columns 2 x4, 2 x4 + 1 of image kx
        // (input column 2 xo + kx - 1)
        const float f[5] = {left, v.x, v.y, v.z, v.w};
        __bf16 hv[5], lv[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          hv[i] = (__bf16)f[i];
          lv[i] = (__bf16)(f[i] - (float)hv[i]);
        }
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          char* base = act_lds + ((slot * 3 + kx) * 2) * C::PLANE + c * C::CS + x4 * 4;
          *reinterpret_cast<bf16x2*>(base) = bf16x2{hv[kx], hv[kx + 2]};
          *reinterpret_cast<bf16x2*>(base + C::PLANE) = bf16x2{lv[kx], lv[kx + 2]};
        }
      }
    }
    if (gbuf >= 0) {
#pragma unroll
      for (int k = 0; k < NGT; ++k) {
        const int idx = tid + NTH * k;
        const int o = idx >> 3, t4 = idx & 7;
        bf16x4 hi, lo;
        split4(zero_if(rg[k], vg[k]), hi, lo);
        char* base = g_lds + ((gbuf * 2) * 64 + o) * C::GCS + t4 * 8;
        *reinterpret_cast<bf16x4*>(base) = hi;
        *reinterpret_cast<bf16x4*>(base + C::GPLANE) = lo;
      }
    }
  };

  constexpr int NACC = TG == 1 ? 9 : 5;  // accumulators per wave: its tap group's taps
  floatx16 acc[NACC];
  const std::integral_constant<int, C::NA / TG> KN;
  const std::integral_constant<int, NAW> KW;

  const int nsteps = H / C::R;
  // prologue of the first tile: input rows -1 .. WIN - 2 (the first window) and the gradients
  // of step 0
  int t = blockIdx.x;
  set_tile(t);
  load_rows(KW, -1, C::WIN, 0);
  store_rows(KW, -1, 0);
  __syncthreads();

  // one fragment: B hi / lo (T < 0) or tap T's A hi / lo, of sub-step s
  auto frag = [&](int y0, int gbuf, int s, int t, int lo) -> bf16x8 {
    const int tl = 16 * s + 8 * h;
    const int ro = tl / W, x = tl % W;
    if (t < 0) {
      const char* gb = g_lds + ((gbuf * 2) * 64 + wo * 32 + r) * C::GCS + tl * 2;
      return *reinterpret_cast<const bf16x8*>(gb + lo * C::GPLANE);
    }
    const int ky = t / 3, kx = t % 3;
    const int slot = (STR * (y0 + ro) + ky) % C::S;
    const char* ab = act_lds + ((slot * 3 + kx) * 2) * C::PLANE + (wc * 32 + r) * C::CS + x * 2;
    return *reinterpret_cast<const bf16x8*>(ab + lo * C::PLANE);
  };
  // one step; LAST: the tile's last step, which prefetches the next tile's first window
  // (when there is one) instead of this tile's next rows, and stages nothing
  auto step = [&](int st, auto LASTc, bool has_next) {
    constexpr bool LAST = decltype(LASTc)::value;
    const int y0 = st * C::R;
    const int inext = STR * y0 + C::WIN - 1;  // first input row past this step's window
    if constexpr (!LAST) {
      load_rows(KN, inext, C::NEW, st + 1);
    } else {
      if (has_next) load_rows(KW, -1, C::WIN, 0);  // the tile vars already name the next tile
    }
    const int gbuf = st & 1;
    auto group = [&](auto T0c, auto NTc) {
      constexpr int T0 = decltype(T0c)::value, NTAP = decltype(NTc)::value;
      bf16x8 bh0, bl0, ah0[NTAP], al0[NTAP], bh1, bl1, ah1[NTAP], al1[NTAP];
      // only B and the first tap of sub-step 0 before its first MFMA; its other reads and
      // sub-step 1's B go two per MFMA gap behind the first NTAP MFMAs, then sub-step 1's A
      // reads one per gap, in this fixed order
      bh0 = frag(y0, gbuf, 0, -1, 0);
      bl0 = frag(y0, gbuf, 0, -1, 1);
      ah0[0] = frag(y0, gbuf, 0, T0, 0);
      al0[0] = frag(y0, gbuf, 0, T0, 1);
      auto rd = [&](int j) {  // the j-th read behind the MFMAs
        constexpr int J0 = 2 * (NTAP - 1), J1 = J0 + 2, J2 = J1 + 2 * NTAP;
        if (j < J0) {
          if (j & 1) al0[1 + j / 2] = frag(y0, gbuf, 0, T0 + 1 + j / 2, 1);
          else ah0[1 + j / 2] = frag(y0, gbuf, 0, T0 + 1 + j / 2, 0);
        } else if (j < J1) {
          (j == J0 ? bh1 : bl1) = frag(y0, gbuf, 1, -1, j - J0);
        } else if (j < J2) {
          if ((j - J1) & 1) al1[(j - J1) / 2] = frag(y0, gbuf, 1, T0 + (j - J1) / 2, 1);
          else ah1[(j - J1) / 2] = frag(y0, gbuf, 1, T0 + (j - J1) / 2, 0);
        }
      };
#pragma unroll
      for (int i = 0; i < NTAP; ++i) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          __builtin_amdgcn_sched_barrier(0);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q == 2 ? al0[i] : ah0[i],
                                                           q == 1 ? bl0 : bh0, acc[i], 0, 0, 0);
          const int g = 3 * i + q;  // gap g: reads j0 .. j0 + nr - 1
          const int j0 = g < NTAP ? 2 * g : NTAP + g, nr = g < NTAP ? 2 : 1;
          rd(j0);
          if (nr == 2) rd(j0 + 1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // sub-step 1 MFMAs; the next step's rows are converted and staged behind them (those
      // slots / the other gradient buffer are not read in this step)
#pragma unroll
      for (int i = 0; i < NTAP; ++i) {
        floatx16 a = acc[i];
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1[i], bh1, a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1[i], bl1, a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al1[i], bh1, a, 0, 0, 0);
        acc[i] = a;
      }
      if constexpr (!LAST) {
        store_rows(KN, inext, gbuf ^ 1);
#pragma unroll
        for (int i = 0; i < 3 * NTAP - 1; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 1);  // 4 VALU
          __builtin_amdgcn_sched_group_barrier(0x080, 1, 1);  // 1 LDS op
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I5 = std::integral_constant<int, 5>;
    if constexpr (TG == 1) {
      group(I0{}, std::integral_constant<int, 9>{});
    } else if (tg == 0) {
      group(I0{}, I5{});
    } else {
      group(I5{}, std::integral_constant<int, 4>{});
    }
    __syncthreads();
  };

  const int ntap = TG == 1 ? 9 : (tg == 0 ? 5 : 4);
  for (;;) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = floatx16{0};
    for (int st = 0; st + 1 < nsteps; ++st) step(st, std::false_type{}, false);
    // the last step: switch the tile variables to the next tile first (its window loads
    // issue under this step's MFMAs); this tile's output index and column scales are kept
    const int lid_c = lid, o0_c = o0;
    const int tn = t + (int)gridDim.x;
    const bool has_next = tn < total;
    if (has_next) set_tile(tn);
    step(nsteps - 1, std::true_type{}, has_next);

    const int o = o0_c + wo * 32 + r;  // C/D column = lane & 31
    float s2 = (o < cout) ? 1.f : 0.f;
    if (col_scale && o < cout) {
      const float sc = col_scale[o];
      s2 = sc * sc;
    }
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NACC; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) v += i < ntap ? acc[i][k] * acc[i][k] : 0.f;
    v = wave_sum(v * s2);
    if (lane == 0) red[wv] = v;
    // the next tile's window and step-0 gradients into LDS (every wave passed the last
    // step's barrier, so no slot is being read)
    if (has_next) store_rows(KW, -1, 0);
    __syncthreads();
    if (tid == 0) {
      float sum = (red[0] + red[1]) + (red[2] + red[3]);
      if constexpr (TG == 2) sum += (red[4] + red[5]) + (red[6] + red[7]);
      partial[lid_c] = sum;
    }
    if (!has_next) break;
    __syncthreads();  // red is rewritten by the next tile
    t = tn;
  }
}

template <int W, int STR, int TG>
static void launch_direct3x3p_tg(const float* act, const float* gout, int64_t B, int cin,
                                 int cout, int H, const float* col_scale, float* partial,
                                 hipStream_t st) {
  using C = D3Cfg<W, STR>;
  const int ncb = (int)ceil_div(cin, 64), nob = (int)ceil_div(cout, 64);
  constexpr int LDS = C::LDS + 16 * TG;  // + the 4 TG partial sums
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pegrad_direct3x3p_kernel<W, STR, TG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  const int64_t total = B * ncb * nob;
  const int64_t grid = std::min<int64_t>(total, device_cus());
  pegrad_direct3x3p_kernel<W, STR, TG><<<(unsigned)grid, 256 * TG, LDS, st>>>(
      act, gout, cin, cout, H, ncb, nob, col_scale, partial, (int)total);
}

template <int W, int STR>
static void launch_direct3x3p(const float* act, const float* gout, int64_t B, int cin, int cout,
                              int H, const float* col_scale, float* partial, hipStream_t st) {
  // (the stride-2 head keeps one tap group: its 5-row next-tile window held in registers
  // across the last step does not fit the 256 registers of two waves per SIMD -- 49 spilled)
  if (d3_tap_groups() == 1 || STR == 2)
    launch_direct3x3p_tg<W, STR, 1>(act, gout, B, cin, cout, H, col_scale, partial, st);
  else
    launch_direct3x3p_tg<W, STR, 2>(act, gout, B, cin, cout, H, col_scale, partial, st);
}

static bool direct3x3_ok(const dd_conv_geom* g) {
  if (g->kh != 3 || g->kw != 3 || g->pad != 1) return false;
  if (g->stride == 1)
    return g->ho == g->h && g->wo == g->w && (g->w == 8 || g->w == 16 || g->w == 32) &&
           (g->h % (32 / g->w)) == 0;
  // stride 2 over an even map: output width 16 (a 32-wide head input)
  return g->stride == 2 && g->h == 2 * g->ho && g->w == 2 * g->wo && g->wo == 16 &&
         (g->ho % 2) == 0;
}

// sq[b] += sum_i partial[b * ntiles + i], fixed order
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ partial,
                                                              int64_t B, int ntiles,
                                                              float* __restrict__ sq) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* p = partial + b * ntiles;
  float s = 0.f;
  for (int i = 0; i < ntiles; ++i) s += p[i];
  sq[b] += s;
}

// ---- host-side planning -------------------------------------------------------------------
struct Plan {
  int method;  // DD_PEGRAD_DIRECT / DD_PEGRAD_GHOST
  int ghost16; // ghost with the T <= 16 kernel
  int d3x3;    // direct with the split-bf16 all-taps 3x3 kernel
  int d1x1;    // direct with the split-bf16 1x1 kernel: its waves along c (1, 2 or 4)
  int pgram;   // ghost by shifted Grams of input positions (dd_pgram.hip)
  int pgq;     // the same, tiled by quarters of the output positions (16 x 16 maps)
  int stem;    // direct over the <= 32 im2col rows of a few-channel input (dd_stem.hip)
  int ntiles;  // partials per example
  int n_cblk, n_oblk, nT;
};

static bool geom_ok(const dd_conv_geom* gm) {
  if (!gm) return false;
  if (gm->batch < 0 || gm->cin <= 0 || gm->cout <= 0 || gm->h <= 0 || gm->w <= 0) return false;
  if (gm->kh <= 0 || gm->kw <= 0 || gm->stride <= 0 || gm->pad < 0) return false;
  const int ho = (gm->h + 2 * gm->pad - gm->kh) / gm->stride + 1;
  const int wo = (gm->w + 2 * gm->pad - gm->kw) / gm->stride + 1;
  return ho == gm->ho && wo == gm->wo && ho > 0 && wo > 0;
}

static double direct_cost(const dd_conv_geom* gm) {
  const double T = (double)ceil_div((int64_t)gm->ho * gm->wo, DBK) * DBK;
  const double da = (double)gm->kh * gm->kw * ceil_div(gm->cin, DBM) * DBM;
  const double dg = (double)ceil_div(gm->cout, DBN) * DBN;
  return 2.0 * T * da * dg;
}

static double ghost_cost(const dd_conv_geom* gm) {
  const int64_t T = (int64_t)gm->ho * gm->wo;
  if (T <= 16) {
    const double da = (double)gm->kh * gm->kw * ceil_div(gm->cin, 4) * 4;
    const double dg = (double)ceil_div(gm->cout, 4) * 4;
    return 2.0 * 256.0 * (da + dg);
  }
  const double Tp = (double)ceil_div(T, 64) * 64;
  const double da = (double)gm->kh * gm->kw * ceil_div(gm->cin, 2) * 2;
  const double dg = (double)ceil_div(gm->cout, 2) * 2;
  // operands are read without LDS staging: weight the ghost flops by its lower efficiency
  return 2.0 * Tp * Tp * (da + dg) * 1.5;
}

// split-bf16 MFMA runs 16x the fp32 MFMA rate at 3 MFMAs per product (~5x), and the 3x3
// kernel reads every byte once; weight its flops accordingly in the AUTO choice
static constexpr double kD3x3Weight = 0.25;

// split-bf16 1x1 workgroup layout: waves along c (1, 2 or 4) with the least padding of the
// 64 LC x 64 (4 / LC) tile; 0 when even that pads more than a quarter of the tile (the
// ResNet-18 64 -> 128 shortcut), where the fp32 direct kernel is as fast.  Both kernels read
// act and g once per tile and are bound by it (measured 94-97 TFLOP/s on ResNet-50 1x1s)
static int d1x1_layout(const dd_conv_geom* gm) {
  int best = 0;
  double best_eff = 0.0;
  for (int lc = 1; lc <= 4; lc *= 2) {
    const double pc = (double)ceil_div(gm->cin, 64 * lc) * 64 * lc;
    const double po = (double)ceil_div(gm->cout, 64 * (4 / lc)) * 64 * (4 / lc);
    const double eff = (double)gm->cin * gm->cout / (pc * po);
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = lc;
    }
  }
  return best_eff >= 0.75 ? best : 0;
}

static Plan make_plan(const dd_conv_geom* gm, int method, int precision) {
  Plan p{};
  const bool d3 = precision == DD_PREC_BF16X3 && direct3x3_ok(gm);
  // 1x1, pad 0, stride 1 or 2: the split-bf16 GEMM-form kernel
  const bool d1 = precision == DD_PREC_BF16X3 && gm->kh == 1 && gm->kw == 1 && gm->pad == 0 &&
                  (gm->stride == 1 || gm->stride == 2) &&
                  gm->ho == (gm->h - 1) / gm->stride + 1 &&
                  gm->wo == (gm->w - 1) / gm->stride + 1 && d1x1_layout(gm) > 0;
  // small maps: the shifted-Gram ghost reads a and g once and needs ~2 (Ti^2 cin + To^2 cout)
  // flop, far below either alternative — always the choice where it applies
  // the network's input conv (cin * 9 <= 32): one 32-row block of G, bound by reading g once
  if (precision == DD_PREC_BF16X3 && method != DD_PEGRAD_GHOST && stem_ok(gm)) {
    p.method = DD_PEGRAD_DIRECT;
    p.stem = 1;
    p.ntiles = 1;  // no partials: the kernel adds to sq_accum itself
    return p;
  }
  if (precision == DD_PREC_BF16X3 && method != DD_PEGRAD_DIRECT && pgram_ok(gm)) {
    p.method = DD_PEGRAD_GHOST;
    p.pgram = 1;
    p.ntiles = 1;  // no partials: the kernel adds to sq_accum itself
    return p;
  }
  // 16 x 16 maps at stride 1 (ResNet-18 layer2): the quarter-tiled shifted-Gram ghost, 33.5
  // (42 with P's halo rows) against the direct form's 75.5 MFLOP per example at 128 channels --
  // but measured 394 us against direct3x3's 202 us per 1024 examples (one workgroup per CU:
  // its 135 KB P image, staging latency and the LDS gather are not hidden), so AUTO keeps the
  // direct kernel and the quarter-tiled ghost runs when GHOST is asked for (DD_PGQ=1: AUTO too)
  if (precision == DD_PREC_BF16X3 && method != DD_PEGRAD_DIRECT && pgram_q_ok(gm) &&
      (method == DD_PEGRAD_GHOST || pgram_q_auto())) {
    p.method = DD_PEGRAD_GHOST;
    p.pgq = 1;
    p.ntiles = 4;  // one partial per quarter
    return p;
  }
  if (method == DD_PEGRAD_AUTO) {
    const double dc = direct_cost(gm) * (d3 ? kD3x3Weight : 1.0);
    method = ghost_cost(gm) < dc ? DD_PEGRAD_GHOST : DD_PEGRAD_DIRECT;
  }
  p.method = method;
  const int64_t T = (int64_t)gm->ho * gm->wo;
  if (method == DD_PEGRAD_DIRECT && d1) {
    p.d1x1 = d1x1_layout(gm);
    p.n_cblk = (int)ceil_div(gm->cin, 64 * p.d1x1);
    p.n_oblk = (int)ceil_div(gm->cout, 64 * (4 / p.d1x1));
    p.ntiles = p.n_cblk * p.n_oblk;
  } else if (method == DD_PEGRAD_DIRECT && d3) {
    p.d3x3 = 1;
    p.n_cblk = (int)ceil_div(gm->cin, 64);
    p.n_oblk = (int)ceil_div(gm->cout, 64);
    p.ntiles = p.n_cblk * p.n_oblk;
  } else if (method == DD_PEGRAD_DIRECT) {
    p.n_cblk = (int)ceil_div(gm->cin, DBM);
    p.n_oblk = (int)ceil_div(gm->cout, DBN);
    p.ntiles = gm->kh * gm->kw * p.n_cblk * p.n_oblk;
  } else {
    p.ghost16 = T <= 16;
    p.nT = (int)ceil_div(T, 64);
    p.ntiles = p.ghost16 ? 1 : p.nT * p.nT;
  }
  return p;
}

}  // namespace dd

using namespace dd;

extern "C" {

static bool prec_ok(int precision) {
  return precision == DD_PREC_FP32 || precision == DD_PREC_BF16X3;
}

int dd_conv_pegrad_method(const dd_conv_geom* geom, int method, int precision) {
  clear_error();
  DD_REQUIRE(geom_ok(geom), "dd_conv_pegrad_method: inconsistent conv geometry");
  DD_REQUIRE(method >= DD_PEGRAD_AUTO && method <= DD_PEGRAD_GHOST, "bad method %d", method);
  DD_REQUIRE(prec_ok(precision), "bad precision %d", precision);
  const Plan p = make_plan(geom, method, precision);
  return p.d3x3 ? DD_PEGRAD_DIRECT3X3 : p.d1x1 ? DD_PEGRAD_DIRECT1X1 : p.pgram ? DD_PEGRAD_PGRAM
         : p.pgq ? DD_PEGRAD_PGRAM_Q : p.stem ? DD_PEGRAD_STEM : p.method;
}

size_t dd_conv_pegrad_workspace_bytes(const dd_conv_geom* geom, int method, int precision) {
  if (!geom_ok(geom) || method < DD_PEGRAD_AUTO || method > DD_PEGRAD_GHOST ||
      !prec_ok(precision))
    return 0;
  const Plan p = make_plan(geom, method, precision);
  return (size_t)geom->batch * p.ntiles * sizeof(float);
}

int dd_conv_pegrad_sqnorm(const float* act, const float* gout, const dd_conv_geom* geom,
                          const float* col_scale, int method, int precision, float* sq_accum,
                          void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  DD_REQUIRE(geom_ok(geom), "dd_conv_pegrad_sqnorm: inconsistent conv geometry");
  DD_REQUIRE(method >= DD_PEGRAD_AUTO && method <= DD_PEGRAD_GHOST, "bad method %d", method);
  DD_REQUIRE(prec_ok(precision), "bad precision %d", precision);
  const int64_t B = geom->batch;
  if (B == 0) return DD_OK;
  DD_REQUIRE(act && gout && sq_accum, "dd_conv_pegrad_sqnorm: null buffer");
  DD_REQUIRE((int64_t)geom->cin * geom->h * geom->w < (1ll << 31) &&
                 (int64_t)geom->cout * geom->ho * geom->wo < (1ll << 31),
             "dd_conv_pegrad_sqnorm: per-example tensor too large");
  const Plan p = make_plan(geom, method, precision);
  const size_t need = (size_t)B * p.ntiles * sizeof(float);
  if (workspace_bytes < need || !workspace) {
    set_error("dd_conv_pegrad_sqnorm: workspace %zu < %zu bytes", workspace_bytes, need);
    return DD_EWORKSPACE;
  }
  float* partial = static_cast<float*>(workspace);
  Geom g{geom->cin, geom->h, geom->w, geom->cout, geom->ho, geom->wo,
         geom->kh, geom->kw, geom->stride, geom->pad};
  hipStream_t st = as_stream(stream);
  if (p.pgram) return pgram_launch(act, gout, geom, col_scale, sq_accum, st);
  if (p.stem) return stem_launch(act, gout, geom, col_scale, sq_accum, st);
  const int64_t nblk = B * p.ntiles;
  DD_REQUIRE(nblk < (1ll << 31), "dd_conv_pegrad_sqnorm: grid too large");
  if (p.pgq) {
    pgram_q_launch(act, gout, geom, col_scale, partial, st);
  } else if (p.d3x3) {
    // the kernel's H is the output height (= the input height at stride 1)
    if (geom->stride == 2)
      launch_direct3x3p<16, 2>(act, gout, B, geom->cin, geom->cout, geom->ho, col_scale, partial,
                               st);
    else if (geom->w == 32)
      launch_direct3x3<32, 1>(act, gout, B, geom->cin, geom->cout, geom->h, col_scale, partial,
                              st);
    else if (geom->w == 16)
      launch_direct3x3p<16, 1>(act, gout, B, geom->cin, geom->cout, geom->h, col_scale, partial,
                               st);
    else
      launch_direct3x3<8, 1>(act, gout, B, geom->cin, geom->cout, geom->h, col_scale, partial,
                             st);
  } else if (p.d1x1) {
#define DD_D1(S_, LC_)                                                                   \
  pegrad_direct1x1_kernel<S_, LC_><<<(unsigned)nblk, 256, 0, st>>>(act, gout, g, p.n_cblk, \
                                                                   p.n_oblk, col_scale, partial)
    if (geom->stride == 1) {
      if (p.d1x1 == 1) DD_D1(1, 1); else if (p.d1x1 == 2) DD_D1(1, 2); else DD_D1(1, 4);
    } else {
      if (p.d1x1 == 1) DD_D1(2, 1); else if (p.d1x1 == 2) DD_D1(2, 2); else DD_D1(2, 4);
    }
#undef DD_D1
  } else if (p.method == DD_PEGRAD_DIRECT) {
    pegrad_direct_kernel<<<(unsigned)nblk, 256, 0, st>>>(act, gout, g, p.n_cblk, p.n_oblk,
                                                         col_scale, partial);
  } else if (p.ghost16) {
    pegrad_ghost16_kernel<<<(unsigned)ceil_div(B, 4), 256, 0, st>>>(act, gout, B, g,
                                                                   col_scale, partial);
  } else {
    pegrad_ghost64_kernel<<<(unsigned)nblk, 256, 0, st>>>(act, gout, g, p.nT, col_scale,
                                                          partial);
  }
  DD_CHECK_LAUNCH("dd_conv_pegrad_sqnorm");
  reduce_partials_kernel<<<(unsigned)ceil_div(B, 256), 256, 0, st>>>(partial, B, p.ntiles,
                                                                     sq_accum);
  DD_CHECK_LAUNCH("dd_conv_pegrad_sqnorm(reduce)");
  return DD_OK;
}

}  // extern "C"
