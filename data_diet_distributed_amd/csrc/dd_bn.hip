// Train-mode BatchNorm of the EL2N pass, grouped: the reference scores with the network in
// train mode (train.py:59-63 never calls .eval()), so every BatchNorm2d normalises with the
// statistics of its batch (models/resnet.py:13-16, 89).  Here one launch carries G batches
// ("BN groups" of group_size examples, the pinned partition of SURVEY §8.0) and each group
// keeps its own statistics.
//
//   partial statistics  [G][C][tiles][2] (sum, sum of squares) — written by the conv epilogue
//                       (dd_conv3x3_forward) or by dd_channel_stats for any other producer
//   dd_bn_finalize      partials -> per (group, channel) affine: scale = gamma / sqrt(var+eps),
//                       shift = beta - mean * scale (biased variance, as F.batch_norm in
//                       training); the partials are summed in double in a fixed order
//   dd_bn_apply         out = relu?(y * scale + shift + R), R = the residual branch (raw, or
//                       its own affine / ReLU); optionally the 4x4 average pool of the CIFAR
//                       head (models/resnet.py:94) instead of the full output
// All are HBM/latency-bound elementwise or reduction kernels: float4 accesses, wave64
// reductions, no atomics (deterministic).
#include "dd_common.h"

#include <math.h>

namespace dd {
namespace bn {

// the ImageNet stem's BN + ReLU + max_pool2d(3, stride 2, padding 1) in one pass (reference
// torchvision-style ResNet stem): out = max over the in-image 3x3 window of
// relu(y * scale[g][c] + shift[g][c]); the window always holds its centre, so it is never empty
__global__ __launch_bounds__(256) void apply_maxpool_kernel(
    const float* __restrict__ y, int64_t B, int C, int h, int w, int ho, int wo, int gsize,
    const float* __restrict__ scale, const float* __restrict__ shift, float* __restrict__ out) {
  const int64_t n = B * C * ho * wo;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int xo = (int)(i % wo);
    int64_t r = i / wo;
    const int yo = (int)(r % ho);
    r /= ho;  // b * C + c
    const int c = (int)(r % C);
    const int64_t b = r / C;
    const int64_t gc = (b / gsize) * C + c;
    const float sc = scale[gc], sh = shift[gc];
    const float* p = y + r * h * w;
    float m = 0.f;  // relu outputs are >= 0 and the centre is always in the window
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int iy = 2 * yo + dy;
      if (iy < 0 || iy >= h) continue;
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int ix = 2 * xo + dx;
        if (ix < 0 || ix >= w) continue;
        m = nmax(m, fmaf(p[iy * w + ix], sc, sh));
      }
    }
    out[i] = m;
  }
}

// the same pass, one thread per 4 consecutive outputs of an output row (w = 2 wo, w % 8 == 0:
// the ImageNet stem's 112 -> 56): the 3 input rows' 9 columns 8 q - 1 .. 8 q + 7 as two float4
// and the left column, 32-bit index math, one float4 store.  The same fmaf / nmax per window
// element as apply_maxpool_kernel (max is exact and order-free), so bitwise its output.
// (The scalar kernel ran config 5's stem tail at 2.1 TB/s, 0.26 of HBM, with five 64-bit
// divisions per output: profiles/r06_c5/bench_c5.json, bn_apply:maxpool.)
__global__ __launch_bounds__(256) void apply_maxpool4_kernel(
    const float* __restrict__ y, uint32_t n, int C, int h, int w, int ho, int wo, int gsize,
    const float* __restrict__ scale, const float* __restrict__ shift, float* __restrict__ out) {
  const int nq = wo >> 2;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const uint32_t row = i / (uint32_t)nq, q = i - row * (uint32_t)nq;
    const uint32_t plane = row / (uint32_t)ho, yo = row - plane * (uint32_t)ho;
    const uint32_t b = plane / (uint32_t)C, c = plane - b * (uint32_t)C;
    const uint32_t gc = (b / (uint32_t)gsize) * (uint32_t)C + c;
    const float sc = scale[gc], sh = shift[gc];
    const float* p = y + (size_t)plane * h * w + 8 * q;
    float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;  // relu outputs are >= 0 (see above)
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int iy = 2 * (int)yo + dy;
      if (iy < 0 || iy >= h) continue;
      const float* r = p + (size_t)iy * w;
      const float4 a = *reinterpret_cast<const float4*>(r);
      const float4 bb = *reinterpret_cast<const float4*>(r + 4);
      const float ax = fmaf(a.x, sc, sh), ay = fmaf(a.y, sc, sh), az = fmaf(a.z, sc, sh),
                  aw = fmaf(a.w, sc, sh), bx = fmaf(bb.x, sc, sh), by = fmaf(bb.y, sc, sh),
                  bz = fmaf(bb.z, sc, sh), bw = fmaf(bb.w, sc, sh);
      if (q > 0) m0 = nmax(m0, fmaf(r[-1], sc, sh));
      m0 = nmax(nmax(m0, ax), ay);
      m1 = nmax(nmax(nmax(m1, ay), az), aw);
      m2 = nmax(nmax(nmax(m2, aw), bx), by);
      m3 = nmax(nmax(nmax(m3, by), bz), bw);
    }
    *reinterpret_cast<float4*>(out + (size_t)row * wo + 4 * q) = make_float4(m0, m1, m2, m3);
  }
}

// one workgroup per (group, channel): sum the valid tiles' partials in double.  A conv
// producer leaves one partial per 32 positions (4096 per channel for a 128-example group at
// 32x32), so the 256 threads stride the list with 16-B loads (two partials each).
__global__ __launch_bounds__(256) void finalize_kernel(
    const float* __restrict__ part, int64_t G, int gsize, int64_t n_valid, int tiles_per_group,
    int images_per_tile, int row_tiles, int C, int64_t hw, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ scale,
    float* __restrict__ shift) {
  const int64_t wid = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t g = wid / C;
  const int c = (int)(wid - g * C);
  int64_t count = n_valid - g * gsize;
  count = count < 0 ? 0 : (count > gsize ? gsize : count);
  // images_per_tile < 0: tiles are runs of -images_per_tile consecutive positions of the
  // group's flattened (example, position) space (producers whose tiles straddle examples)
  const int ntiles =
      images_per_tile > 0
          ? (int)((count + images_per_tile - 1) / images_per_tile) * row_tiles
          : (int)((count * hw + (-images_per_tile) - 1) / (-images_per_tile));
  const float* p = part + (size_t)wid * tiles_per_group * 2;
  double s = 0.0, q = 0.0;
  if (((uintptr_t)p & 15) == 0) {
    const int npair = ntiles >> 1;
    for (int i = tid; i < npair; i += 256) {
      const float4 v = *reinterpret_cast<const float4*>(p + 4 * i);
      s += (double)v.x + (double)v.z;
      q += (double)v.y + (double)v.w;
    }
    if ((ntiles & 1) && tid == 0) {
      s += p[2 * (ntiles - 1)];
      q += p[2 * (ntiles - 1) + 1];
    }
  } else {
    for (int i = tid; i < ntiles; i += 256) {
      const float2 v = *reinterpret_cast<const float2*>(p + 2 * i);
      s += v.x;
      q += v.y;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  __shared__ double red[2][4];
  if (lane == 0) {
    red[0][wv] = s;
    red[1][wv] = q;
  }
  __syncthreads();
  if (tid == 0) {
    s = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    q = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    float sc = 0.f, sh = 0.f;
    if (count > 0) {
      const double n = (double)count * (double)hw;
      const double mean = s / n;
      double var = q / n - mean * mean;
      var = var < 0.0 ? 0.0 : var;
      const double k = (double)gamma[c] / sqrt(var + (double)eps);
      sc = (float)k;
      sh = (float)((double)beta[c] - mean * k);
    }
    scale[wid] = sc;
    shift[wid] = sh;
  }
}

// partials of an arbitrary NCHW producer: one wave per (example, channel), tile = example
__global__ __launch_bounds__(256) void channel_stats_kernel(const float* __restrict__ y,
                                                            int64_t B, int C, int64_t hw,
                                                            int gsize, int64_t n_stat,
                                                            float* __restrict__ part) {
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wid >= B * C) return;
  const int64_t b = wid / C;
  const int c = (int)(wid - b * C);
  const float* row = y + (size_t)wid * hw;
  float s = 0.f, q = 0.f;
  if (b < n_stat) {
    if (hw % 4 == 0) {
      for (int64_t i = lane; i < hw / 4; i += 64) {
        const float4 v = reinterpret_cast<const float4*>(row)[i];
        s += (v.x + v.y) + (v.z + v.w);
        q += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
      }
    } else {
      for (int64_t i = lane; i < hw; i += 64) {
        const float v = row[i];
        s += v;
        q += v * v;
      }
    }
  }
  s = wave_sum(s);
  q = wave_sum(q);
  if (lane == 0) {
    const int64_t g = b / gsize;
    const int64_t tile = b - g * gsize;
    float* dst = part + (((size_t)g * C + c) * gsize + tile) * 2;
    dst[0] = s;
    dst[1] = q;
  }
}

struct ApplyArgs {
  const float* y;
  const float* scale;
  const float* shift;
  const float* r;        // residual source or NULL
  const float* r_scale;  // NULL: R = r raw
  const float* r_shift;
  float* out;            // NULL when only pooling
  float* pool;           // NULL or [B][C]
  int64_t B;
  int C;
  int64_t hw;
  int gsize;
  int relu, r_relu;
};

__device__ __forceinline__ float4 affine4(float4 v, float s, float t) {
  return make_float4(fmaf(v.x, s, t), fmaf(v.y, s, t), fmaf(v.z, s, t), fmaf(v.w, s, t));
}
__device__ __forceinline__ float4 relu4(float4 v) {
  return make_float4(nmax(v.x, 0.f), nmax(v.y, 0.f), nmax(v.z, 0.f), nmax(v.w, 0.f));
}

__device__ __forceinline__ float4 apply_one(const ApplyArgs& a, int64_t i4, int64_t* bc_out) {
  const int64_t e = i4 * 4;
  const int64_t bc = e / a.hw;  // b * C + c
  const int64_t b = bc / a.C;
  const int c = (int)(bc - b * a.C);
  const int64_t gi = (b / a.gsize) * a.C + c;
  float4 v = affine4(reinterpret_cast<const float4*>(a.y)[i4], a.scale[gi], a.shift[gi]);
  if (a.r) {
    float4 r = reinterpret_cast<const float4*>(a.r)[i4];
    if (a.r_scale) r = affine4(r, a.r_scale[gi], a.r_shift[gi]);
    if (a.r_relu) r = relu4(r);
    v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
  }
  if (a.relu) v = relu4(v);
  *bc_out = bc;
  return v;
}

__global__ __launch_bounds__(256) void apply_kernel(const ApplyArgs a) {
  const int64_t n4 = a.B * a.C * a.hw / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * 256) {
    int64_t bc;
    const float4 v = apply_one(a, i, &bc);
    reinterpret_cast<float4*>(a.out)[i] = v;
  }
}

// any hw (e.g. the 7x7 maps of the ImageNet stem): one element per thread
__global__ __launch_bounds__(256) void apply_scalar_kernel(const ApplyArgs a) {
  const int64_t n = a.B * a.C * a.hw;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bc = i / a.hw;
    const int64_t b = bc / a.C;
    const int c = (int)(bc - b * a.C);
    const int64_t gi = (b / a.gsize) * a.C + c;
    float v = fmaf(a.y[i], a.scale[gi], a.shift[gi]);
    if (a.r) {
      float r = a.r[i];
      if (a.r_scale) r = fmaf(r, a.r_scale[gi], a.r_shift[gi]);
      if (a.r_relu) r = nmax(r, 0.f);
      v += r;
    }
    if (a.relu) v = nmax(v, 0.f);
    a.out[i] = v;
  }
}

// hw % 4 != 0 with the flat tensor a multiple of 4 and 16-B aligned (the ImageNet network's 7x7
// unit tails): 4 consecutive flat elements per thread as float4, 32-bit index math (one division
// chain per quad; a quad spans at most two (b, c) rows since hw >= 4); per element the
// arithmetic of apply_scalar_kernel, so bitwise its output
__global__ __launch_bounds__(256) void apply_quad_kernel(const ApplyArgs a, uint32_t n4) {
  const uint32_t hw = (uint32_t)a.hw, C = (uint32_t)a.C;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n4; i += gridDim.x * 256u) {
    const uint32_t e0 = 4 * i, bc0 = e0 / hw, rem0 = e0 - bc0 * hw;
    const float4 y4 = reinterpret_cast<const float4*>(a.y)[i];
    float4 r4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.r) r4 = reinterpret_cast<const float4*>(a.r)[i];
    const float yv[4] = {y4.x, y4.y, y4.z, y4.w}, rv[4] = {r4.x, r4.y, r4.z, r4.w};
    float ov[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t bc = bc0 + (rem0 + j >= hw ? 1u : 0u);
      const uint32_t b = bc / C, c = bc - b * C;
      const uint32_t gi = (b / (uint32_t)a.gsize) * C + c;
      float v = fmaf(yv[j], a.scale[gi], a.shift[gi]);
      if (a.r) {
        float r = rv[j];
        if (a.r_scale) r = fmaf(r, a.r_scale[gi], a.r_shift[gi]);
        if (a.r_relu) r = nmax(r, 0.f);
        v += r;
      }
      if (a.relu) v = nmax(v, 0.f);
      ov[j] = v;
    }
    reinterpret_cast<float4*>(a.out)[i] = make_float4(ov[0], ov[1], ov[2], ov[3]);
  }
}

// L = hw / 4 lanes per (b, c) row: the row's mean is reduced across them
template <int L>
__global__ __launch_bounds__(256) void apply_pool_kernel(const ApplyArgs a) {
  const int64_t n4 = a.B * a.C * a.hw / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = i < n4;  // rows never straddle blocks (256 % L == 0)
  int64_t bc = 0;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    v = apply_one(a, i, &bc);
    if (a.out) reinterpret_cast<float4*>(a.out)[i] = v;
  }
  float s = group_sum<L>((v.x + v.y) + (v.z + v.w));
  if (live && (threadIdx.x % L) == 0) a.pool[bc] = s / (float)a.hw;
}

// ---- per-example gradient norm of an eval-mode BN's affine parameters (grand_params: all) --
// With the BN output v = gamma * xhat + beta (+ r, a residual added after it) and g the
// gradient w.r.t. that output: d/dgamma_c = sum_t g xhat = sum_t g (v - r - beta_c) / gamma_c,
// d/dbeta_c = sum_t g.  One workgroup per example walks its channels: L lanes per channel row
// (float4 each), R = 256 / L rows at a time; each row's two sums by a width-L butterfly, the
// squares accumulated per thread, one fixed-order block reduction, one add per example (no
// float atomics: deterministic).
template <int L, bool VEC>
__global__ __launch_bounds__(256) void bn_pegrad_kernel(const float* __restrict__ v,
                                                        const float* __restrict__ r,
                                                        const float* __restrict__ g, int C,
                                                        int64_t hw,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        float* __restrict__ sq) {
  constexpr int R = 256 / L;
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid % L, row = tid / L;
  float acc = 0.f;
  for (int c0 = 0; c0 < C; c0 += R) {
    const int c = c0 + row;
    const bool live = c < C;
    const int cc = live ? c : C - 1;
    const int64_t base = (b * C + cc) * hw;
    const float bt = beta[cc];
    float dg = 0.f, db = 0.f;
    if (VEC) {
      for (int64_t i = 4 * lane; i < hw; i += 4 * L) {
        const float4 gv = *reinterpret_cast<const float4*>(g + base + i);
        float4 vv = *reinterpret_cast<const float4*>(v + base + i);
        if (r) {
          const float4 rv = *reinterpret_cast<const float4*>(r + base + i);
          vv.x -= rv.x;
          vv.y -= rv.y;
          vv.z -= rv.z;
          vv.w -= rv.w;
        }
        dg += gv.x * (vv.x - bt) + gv.y * (vv.y - bt) + gv.z * (vv.z - bt) + gv.w * (vv.w - bt);
        db += gv.x + gv.y + gv.z + gv.w;
      }
    } else {
      for (int64_t i = lane; i < hw; i += L) {
        const float gi = g[base + i];
        const float vi = v[base + i] - (r ? r[base + i] : 0.f);
        dg += gi * (vi - bt);
        db += gi;
      }
    }
    dg = group_sum<L>(dg);
    db = group_sum<L>(db);
    if (live && lane == 0) {
      const float d = dg / gamma[cc];
      acc += d * d + db * db;
    }
  }
  acc = wave_sum(acc);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) sq[b] += (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace bn
}  // namespace dd

using namespace dd;

extern "C" {

int dd_channel_stats(const float* y, int64_t B, int32_t C, int64_t hw, int32_t group_size,
                     int64_t n_stat, float* stats, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && C > 0 && hw > 0 && group_size > 0, "dd_channel_stats: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(y && stats, "dd_channel_stats: null buffer");
  DD_REQUIRE(hw % 4 != 0 || (uintptr_t)y % 16 == 0, "dd_channel_stats: y must be 16-B aligned");
  bn::channel_stats_kernel<<<(unsigned)ceil_div(B * C, 4), 256, 0, as_stream(stream)>>>(
      y, B, C, hw, group_size, n_stat, stats);
  DD_CHECK_LAUNCH("dd_channel_stats");
  return DD_OK;
}

int dd_bn_finalize(const float* stats, int64_t n_groups, int32_t group_size, int64_t n_valid,
                   int32_t tiles_per_group, int32_t images_per_tile, int32_t row_tiles,
                   int32_t C, int64_t hw, const float* gamma, const float* beta, float eps,
                   float* scale, float* shift, void* stream) {
  clear_error();
  DD_REQUIRE(n_groups >= 0 && group_size > 0 && C > 0 && hw > 0 && tiles_per_group > 0 &&
                 images_per_tile != 0 && row_tiles > 0,
             "dd_bn_finalize: bad sizes");
  DD_REQUIRE(images_per_tile > 0
                 ? tiles_per_group ==
                       (group_size + images_per_tile - 1) / images_per_tile * row_tiles
                 : tiles_per_group == ((int64_t)group_size * hw + (-images_per_tile) - 1) /
                                          (-images_per_tile),
             "dd_bn_finalize: tiles_per_group inconsistent with the tile geometry");
  if (n_groups == 0) return DD_OK;
  DD_REQUIRE(stats && gamma && beta && scale && shift, "dd_bn_finalize: null buffer");
  DD_REQUIRE(eps >= 0.f, "dd_bn_finalize: eps < 0");
  bn::finalize_kernel<<<(unsigned)(n_groups * C), 256, 0, as_stream(stream)>>>(
      stats, n_groups, group_size, n_valid, tiles_per_group, images_per_tile, row_tiles, C, hw,
      gamma, beta, eps, scale, shift);
  DD_CHECK_LAUNCH("dd_bn_finalize");
  return DD_OK;
}

int dd_bn_apply_maxpool(const float* y, int64_t B, int32_t C, int32_t h, int32_t w,
                        int32_t group_size, const float* scale, const float* shift,
                        float* out, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && C > 0 && h > 0 && w > 0 && group_size > 0,
             "dd_bn_apply_maxpool: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(y && scale && shift && out, "dd_bn_apply_maxpool: null buffer");
  const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const int64_t n = B * C * ho * wo;
  const int64_t n4 = n / 4;
  if (w == 2 * wo && w % 8 == 0 && ((uintptr_t)y | (uintptr_t)out) % 16 == 0 && n4 < (1ll << 32)) {
    bn::apply_maxpool4_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n4, 256), 1 << 20), 256, 0,
                                as_stream(stream)>>>(y, (uint32_t)n4, C, h, w, ho, wo,
                                                     group_size, scale, shift, out);
  } else {
    bn::apply_maxpool_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 1 << 20), 256, 0,
                               as_stream(stream)>>>(y, B, C, h, w, ho, wo, group_size, scale,
                                                    shift, out);
  }
  DD_CHECK_LAUNCH("dd_bn_apply_maxpool");
  return DD_OK;
}

// DD_BN_QUAD=0: the scalar kernel at every width that is not a multiple of 4 (A/B, tests; read
// per call)
static bool quad_on() {
  const char* e = getenv("DD_BN_QUAD");
  return !e || atoi(e) != 0;
}

int dd_bn_apply(const float* y, int64_t B, int32_t C, int64_t hw, int32_t group_size,
                const float* scale, const float* shift, const float* residual,
                const float* res_scale, const float* res_shift, int32_t res_relu, int32_t relu,
                float* out, float* pool_out, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && C > 0 && hw > 0 && group_size > 0, "dd_bn_apply: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(y && scale && shift, "dd_bn_apply: null buffer");
  DD_REQUIRE(out || pool_out, "dd_bn_apply: nothing to write");
  DD_REQUIRE(!res_scale == !res_shift, "dd_bn_apply: res_scale and res_shift go together");
  DD_REQUIRE(residual || !res_scale, "dd_bn_apply: residual affine without a residual");
  bn::ApplyArgs a{y, scale, shift, residual, res_scale, res_shift, out, pool_out,
                  B, C, hw, group_size, relu, res_relu};
  hipStream_t st = as_stream(stream);
  bool vec = hw % 4 == 0, al = true;
  for (const void* p : {(const void*)y, (const void*)residual, (const void*)out})
    al = al && (uintptr_t)p % 16 == 0;
  vec = vec && al;
  const int64_t n = B * C * hw;
  if (!vec && !pool_out && al && hw >= 4 && n % 4 == 0 && n < (1ll << 32) && quad_on()) {
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n / 4, 256), 16384);
    bn::apply_quad_kernel<<<grid, 256, 0, st>>>(a, (uint32_t)(n / 4));
    DD_CHECK_LAUNCH("dd_bn_apply");
    return DD_OK;
  }
  if (!vec) {
    DD_REQUIRE(!pool_out, "dd_bn_apply: pooling needs hw % 4 == 0 and 16-B aligned tensors");
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(B * C * hw, 256), 16384);
    bn::apply_scalar_kernel<<<grid, 256, 0, st>>>(a);
    DD_CHECK_LAUNCH("dd_bn_apply");
    return DD_OK;
  }
  const int64_t n4 = B * C * hw / 4;
  if (pool_out) {
    const int64_t L = hw / 4;
    const unsigned grid = (unsigned)ceil_div(n4, 256);
    switch (L) {
      case 1: bn::apply_pool_kernel<1><<<grid, 256, 0, st>>>(a); break;
      case 2: bn::apply_pool_kernel<2><<<grid, 256, 0, st>>>(a); break;
      case 4: bn::apply_pool_kernel<4><<<grid, 256, 0, st>>>(a); break;
      case 8: bn::apply_pool_kernel<8><<<grid, 256, 0, st>>>(a); break;
      case 16: bn::apply_pool_kernel<16><<<grid, 256, 0, st>>>(a); break;
      case 32: bn::apply_pool_kernel<32><<<grid, 256, 0, st>>>(a); break;
      case 64: bn::apply_pool_kernel<64><<<grid, 256, 0, st>>>(a); break;
      default:
        set_error("dd_bn_apply: pooling needs hw / 4 a power of two <= 64 (hw = %lld)",
                  (long long)hw);
        return DD_EINVAL;
    }
  } else {
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n4, 256), 16384);
    bn::apply_kernel<<<grid, 256, 0, st>>>(a);
  }
  DD_CHECK_LAUNCH("dd_bn_apply");
  return DD_OK;
}

int dd_bn_pegrad_sqnorm(const float* v, const float* r, const float* g, int64_t B, int32_t C,
                        int64_t hw, const float* gamma, const float* beta, float* sq_accum,
                        void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && C > 0 && hw > 0, "dd_bn_pegrad_sqnorm: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(v && g && gamma && beta && sq_accum, "dd_bn_pegrad_sqnorm: null buffer");
  DD_REQUIRE(B < (1ll << 31), "dd_bn_pegrad_sqnorm: B too large");
  hipStream_t st = as_stream(stream);
  const bool vec = hw % 4 == 0 && (uintptr_t)v % 16 == 0 && (uintptr_t)g % 16 == 0 &&
                   (!r || (uintptr_t)r % 16 == 0);
  const dim3 grid((unsigned)B);
  if (vec && hw <= 16)
    bn::bn_pegrad_kernel<4, true><<<grid, 256, 0, st>>>(v, r, g, C, hw, gamma, beta, sq_accum);
  else if (vec && hw <= 64)
    bn::bn_pegrad_kernel<16, true><<<grid, 256, 0, st>>>(v, r, g, C, hw, gamma, beta, sq_accum);
  else if (vec)
    bn::bn_pegrad_kernel<64, true><<<grid, 256, 0, st>>>(v, r, g, C, hw, gamma, beta, sq_accum);
  else
    bn::bn_pegrad_kernel<64, false><<<grid, 256, 0, st>>>(v, r, g, C, hw, gamma, beta,
                                                          sq_accum);
  DD_CHECK_LAUNCH("dd_bn_pegrad_sqnorm");
  return DD_OK;
}

}  // extern "C"
