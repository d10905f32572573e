// EL2N, input normalisation, linear-layer GraNd term and ensemble elementwise kernels.
//
// All of these are HBM/latency-bound row or element kernels: one pass over their inputs,
// 16-B-per-lane accesses where the layout allows, rows reduced with wave64 shuffles.
#include "dd_common.h"

#include <math.h>

#include <algorithm>
#include <string.h>

namespace dd {

static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
void clear_error() { g_err[0] = 0; }

// ------------------------------------------------------------------------------------------
// EL2N rows: LPR lanes per row (16/32/64), each lane keeps up to EPL logits in registers.
// reference get_scores_and_prune.py:16-18 (softmax, minus one_hot, L2 over classes).
// ------------------------------------------------------------------------------------------
template <int LPR, int EPL>
__global__ __launch_bounds__(256) void el2n_rows_kernel(const float* __restrict__ logits,
                                                        const int64_t* __restrict__ labels,
                                                        int64_t B, int C,
                                                        float* __restrict__ score,
                                                        float* __restrict__ e_out,
                                                        float* __restrict__ accum,
                                                        int* __restrict__ bad_labels) {
  constexpr int ROWS = 256 / LPR;
  const int lane = threadIdx.x % LPR;
  const int64_t row = (int64_t)blockIdx.x * ROWS + threadIdx.x / LPR;
  const bool live = row < B;  // keep every lane in the shuffles
  const float* x = logits + (live ? row : 0) * (int64_t)C;

  float v[EPL];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int j = lane + i * LPR;
    v[i] = (live && j < C) ? x[j] : -INFINITY;
    m = fmaxf(m, v[i]);
  }
  m = group_max<LPR>(m);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int j = lane + i * LPR;
    v[i] = (j < C) ? expf(v[i] - m) : 0.f;
    s += v[i];
  }
  s = group_sum<LPR>(s);
  const int64_t y = live ? labels[row] : -1;
  const bool bad = live && (y < 0 || y >= C);  // one_hot would raise (reference :17)
  // e for the GraNd seed without the cancellation of p_y - 1: e_y = -sum_{j != y} p_j
  float so = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int j = lane + i * LPR;
    so += (j < C && j != y) ? v[i] : 0.f;
  }
  if (e_out) so = group_sum<LPR>(so);
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int j = lane + i * LPR;
    if (j < C) {
      const float p = v[i] / s;
      const float e = p - (j == y ? 1.f : 0.f);  // the reference's arithmetic (score)
      sq += e * e;
      if (live && e_out)
        e_out[row * (int64_t)C + j] = bad ? __builtin_nanf("") : (j == y) ? -so / s : p;
    }
  }
  sq = group_sum<LPR>(sq);
  if (live && lane == 0) {
    const float sc = bad ? __builtin_nanf("") : sqrtf(sq);
    if (score) score[row] = sc;
    if (accum) accum[row] += sc;
    if (bad && bad_labels) atomicAdd(bad_labels, 1);
  }
}

// very wide rows (C > 64*32): one 256-thread block per row, logits re-read from cache
__global__ __launch_bounds__(256) void el2n_wide_kernel(const float* __restrict__ logits,
                                                        const int64_t* __restrict__ labels,
                                                        int64_t B, int C,
                                                        float* __restrict__ score,
                                                        float* __restrict__ e_out,
                                                        float* __restrict__ accum,
                                                        int* __restrict__ bad_labels) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const float* x = logits + row * (int64_t)C;
  const int t = threadIdx.x, w = t / kWave, l = t % kWave;
  auto block_reduce = [&](float v, bool is_max) -> float {
    v = is_max ? group_max<kWave>(v) : group_sum<kWave>(v);
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < 4; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
    return r;
  };
  float m = -INFINITY;
  for (int j = t; j < C; j += 256) m = fmaxf(m, x[j]);
  m = block_reduce(m, true);
  float s = 0.f;
  for (int j = t; j < C; j += 256) s += expf(x[j] - m);
  s = block_reduce(s, false);
  const int64_t y = labels[row];
  const bool bad = y < 0 || y >= C;
  float so = 0.f;
  for (int j = t; j < C; j += 256) so += (j != y) ? expf(x[j] - m) : 0.f;
  so = block_reduce(so, false);
  float sq = 0.f;
  for (int j = t; j < C; j += 256) {
    const float p = expf(x[j] - m) / s;
    const float e = p - (j == y ? 1.f : 0.f);
    sq += e * e;
    if (e_out)
      e_out[row * (int64_t)C + j] = bad ? __builtin_nanf("") : (j == y) ? -so / s : p;
  }
  sq = block_reduce(sq, false);
  if (t == 0) {
    const float sc = bad ? __builtin_nanf("") : sqrtf(sq);
    if (score) score[row] = sc;
    if (accum) accum[row] += sc;
    if (bad && bad_labels) atomicAdd(bad_labels, 1);
  }
}

// Narrow rows (C <= 128): a one-wave block owns R = 64 / LPR consecutive rows, ONE
// contiguous span of logits, streamed into LDS with 16-byte loads (coalesced, all of a lane's
// loads in flight at once) and scattered to rows of odd stride CP = C | 1; then LPR lanes
// reduce a row from LDS in registers (lane part p takes classes p, p + LPR, ...; one
// shuffle step per reduction when LPR = 2..4), write its e row back in place, and the wave
// streams e out with 16-byte stores.  Small blocks (<= 8.3 KB of LDS at C = 128) keep many
// waves per CU so one block's load phase overlaps others' reductions.  Per row: 4C + 8 bytes
// in, 4 (+ 4C e, + 8 accum RMW) out, nothing re-read from HBM.  (The lanes-per-row kernel
// above moved 0.85-1.2 TB/s at C = 10-100.)
template <int EPL, int LPR>
__global__ __launch_bounds__(64) void el2n_lds_kernel(const float* __restrict__ logits,
                                                      const int64_t* __restrict__ labels,
                                                      int64_t B, int C, uint32_t cmag,
                                                      float* __restrict__ score,
                                                      float* __restrict__ e_out,
                                                      float* __restrict__ accum,
                                                      int* __restrict__ bad_labels, int vec) {
  constexpr int R = 64 / LPR;
  extern __shared__ __attribute__((aligned(16))) float sl[];  // R rows x CP floats
  const int tid = threadIdx.x, CP = C | 1;
  const int lr = tid / LPR, part = tid % LPR;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int rows = (int)(B - row0 < R ? B - row0 : R);
  const int cnt = rows * C;
  // flat index i of the span -> LDS slot (i / C) * CP + i % C; i < 64 * 128, so the
  // multiply-high by cmag = ceil(2^32 / C) is exact (cmag = 0: C = 1)
  auto slot = [&](uint32_t i) {
    const uint32_t r = cmag ? __umulhi(i, cmag) : i;
    return r * CP + (i - r * C);
  };
  const float* __restrict__ src = logits + row0 * C;
  int tail = 0;
  if (vec) {  // vec: the span starts 16-byte aligned
    const int n4 = cnt >> 2;
    for (int i = tid; i < n4; i += 64) {
      const float4 t = reinterpret_cast<const float4*>(src)[i];
      sl[slot(4 * i)] = t.x;
      sl[slot(4 * i + 1)] = t.y;
      sl[slot(4 * i + 2)] = t.z;
      sl[slot(4 * i + 3)] = t.w;
    }
    tail = n4 << 2;
  }
  for (int i = tail + tid; i < cnt; i += 64) sl[slot(i)] = src[i];
  const bool live = lr < rows;
  const int64_t y = live ? labels[row0 + lr] : -1;
  const bool bad = live && (y < 0 || y >= C);  // one_hot would raise (reference :17)
  const float acc0 = (live && accum && part == 0) ? accum[row0 + lr] : 0.f;
  __syncthreads();
  float* r = sl + lr * CP;  // rows >= `rows` read stale LDS: their results are dropped
  float v[EPL];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int j = part + LPR * i;
    v[i] = j < C ? r[j] : -INFINITY;
    m = fmaxf(m, v[i]);
  }
  m = group_max<LPR>(m);
  float s = 0.f, so = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int j = part + LPR * i;
    const float ev = j < C ? __expf(v[i] - m) : 0.f;
    v[i] = ev;
    s += ev;
    so += (j != y) ? ev : 0.f;
  }
  s = group_sum<LPR>(s);
  if (e_out) so = group_sum<LPR>(so);
  const float inv = 1.f / s;
  // sum of e_j^2 over j != y, the label term e_y = p_y - 1 (the reference's arithmetic)
  // added last: rows that differ only in which class is the label (all-tie rows) score
  // bit-identically, so ties keep loader order exactly as the reference's sort does
  float sq = 0.f, ey = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int j = part + LPR * i;
    if (j < C) {
      const float p = v[i] * inv;
      if (j == y)
        ey = p - 1.f;
      else
        sq += p * p;
      // e for the GraNd seed without the cancellation of p_y - 1: e_y = -sum_{j != y} p_j
      if (e_out) r[j] = bad ? __builtin_nanf("") : (j == y) ? -so * inv : p;
    }
  }
  sq = group_sum<LPR>(sq);
  ey = group_sum<LPR>(ey);  // one lane holds the label term, the others 0
  sq += ey * ey;
  if (live && part == 0) {
    const float sc = bad ? __builtin_nanf("") : sqrtf(sq);
    if (score) score[row0 + lr] = sc;
    if (accum) accum[row0 + lr] = acc0 + sc;
    if (bad && bad_labels) atomicAdd(bad_labels, 1);
  }
  if (e_out) {
    __syncthreads();
    float* __restrict__ dst = e_out + row0 * C;
    tail = 0;
    if (vec) {
      const int n4 = cnt >> 2;
      for (int i = tid; i < n4; i += 64)
        reinterpret_cast<float4*>(dst)[i] = make_float4(sl[slot(4 * i)], sl[slot(4 * i + 1)],
                                                        sl[slot(4 * i + 2)], sl[slot(4 * i + 3)]);
      tail = n4 << 2;
    }
    for (int i = tail + tid; i < cnt; i += 64) dst[i] = sl[slot(i)];
  }
}

template <int EPL, int LPR>
static void launch_el2n_lds(const float* logits, const int64_t* labels, int64_t B, int C,
                            float* score, float* e, float* accum, int* bad, hipStream_t st) {
  constexpr int R = 64 / LPR;
  // 16-B staging: block spans start at R C floats from the base (16-B aligned when R C is a
  // multiple of 4, always for R >= 16)
  const int vec = ((uintptr_t)logits % 16 == 0) && (!e || (uintptr_t)e % 16 == 0) &&
                  (R * C) % 4 == 0;
  const uint32_t cmag = C == 1 ? 0u : (uint32_t)((((uint64_t)1 << 32) + C - 1) / C);
  el2n_lds_kernel<EPL, LPR><<<(unsigned)ceil_div(B, R), 64, (size_t)R * (C | 1) * 4, st>>>(
      logits, labels, B, C, cmag, score, e, accum, bad, vec);
}

template <int LPR, int EPL>
static void launch_el2n(const float* logits, const int64_t* labels, int64_t B, int C,
                        float* score, float* e, float* accum, int* bad, hipStream_t st) {
  constexpr int ROWS = 256 / LPR;
  const unsigned grid = (unsigned)ceil_div(B, ROWS);
  el2n_rows_kernel<LPR, EPL><<<grid, 256, 0, st>>>(logits, labels, B, C, score, e, accum,
                                                   bad);
}

// ------------------------------------------------------------------------------------------
// ToTensor + Normalize (reference data/loader.py:8-11): (u8 / 255 - mean[c]) / std[c]
// ------------------------------------------------------------------------------------------
struct NormParams {
  float mean[4];
  float std[4];
};

__device__ __forceinline__ float norm_px(unsigned v, float mean, float sd) {
  return ((float)v / 255.0f - mean) / sd;
}

// 16 pixels per thread; requires hw % 16 == 0 (image rows never straddle a channel)
__global__ __launch_bounds__(256) void normalize_vec16_kernel(const uint8_t* __restrict__ img,
                                                              const int64_t* __restrict__ index,
                                                              int64_t n, int C, int64_t hw,
                                                              NormParams prm,
                                                              float* __restrict__ out) {
  const int64_t per_img = (int64_t)C * hw / 16;
  const int64_t total = n * per_img;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = q / per_img;
    const int64_t r = (q - i * per_img) * 16;
    const int c = (int)(r / hw);
    const int64_t src = index ? index[i] : i;
    const uint4 raw = *reinterpret_cast<const uint4*>(img + src * C * hw + r);
    const float mu = prm.mean[c], sd = prm.std[c];
    float4* o = reinterpret_cast<float4*>(out + i * C * hw + r);
    const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float4 f;
      f.x = norm_px(w[k] & 0xff, mu, sd);
      f.y = norm_px((w[k] >> 8) & 0xff, mu, sd);
      f.z = norm_px((w[k] >> 16) & 0xff, mu, sd);
      f.w = norm_px(w[k] >> 24, mu, sd);
      o[k] = f;
    }
  }
}

__global__ __launch_bounds__(256) void normalize_scalar_kernel(const uint8_t* __restrict__ img,
                                                               const int64_t* __restrict__ index,
                                                               int64_t n, int C, int64_t hw,
                                                               NormParams prm,
                                                               float* __restrict__ out) {
  const int64_t per_img = (int64_t)C * hw;
  const int64_t total = n * per_img;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = q / per_img;
    const int64_t r = q - i * per_img;
    const int c = (int)(r / hw);
    const int64_t src = index ? index[i] : i;
    out[q] = norm_px(img[src * per_img + r], prm.mean[c], prm.std[c]);
  }
}

static int launch_normalize(const uint8_t* img, const int64_t* index, int64_t n, int C,
                            int64_t hw, const float* mean, const float* sd, float* out,
                            hipStream_t st) {
  DD_REQUIRE(n >= 0 && hw > 0, "dd_normalize_u8: bad sizes n=%lld hw=%lld", (long long)n,
             (long long)hw);
  DD_REQUIRE(C >= 1 && C <= 4, "dd_normalize_u8: channels must be 1..4 (got %d)", C);
  DD_REQUIRE(mean && sd, "dd_normalize_u8: mean/std are required");
  if (n == 0) return DD_OK;
  DD_REQUIRE(img && out, "dd_normalize_u8: null buffer");
  NormParams p{};
  for (int c = 0; c < C; ++c) {
    DD_REQUIRE(sd[c] != 0.f, "dd_normalize_u8: std[%d] == 0", c);
    p.mean[c] = mean[c];
    p.std[c] = sd[c];
  }
  const bool vec = (hw % 16 == 0) && ((uintptr_t)img % 16 == 0) && ((uintptr_t)out % 16 == 0);
  const int64_t work = vec ? n * C * hw / 16 : n * C * hw;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(work, 256), 8192);
  if (vec)
    normalize_vec16_kernel<<<grid, 256, 0, st>>>(img, index, n, C, hw, p, out);
  else
    normalize_scalar_kernel<<<grid, 256, 0, st>>>(img, index, n, C, hw, p, out);
  DD_CHECK_LAUNCH("dd_normalize_u8");
  return DD_OK;
}

// ------------------------------------------------------------------------------------------
// Linear-layer per-example gradient norm: ||a g^T||_F^2 = ||a||^2 ||g||^2 (+ ||g||^2 bias).
// One wave per row.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void linear_pegrad_kernel(const float* __restrict__ act,
                                                            const float* __restrict__ gout,
                                                            int64_t B, int din, int dout,
                                                            int has_bias,
                                                            float* __restrict__ sq) {
  const int64_t row = (int64_t)blockIdx.x * 4 + threadIdx.x / kWave;
  const int l = threadIdx.x % kWave;
  if (row >= B) return;  // whole wave exits together
  float aa = 0.f, gg = 0.f;
  for (int j = l; j < din; j += kWave) {
    const float v = act[row * din + j];
    aa += v * v;
  }
  for (int j = l; j < dout; j += kWave) {
    const float v = gout[row * dout + j];
    gg += v * v;
  }
  aa = wave_sum(aa);
  gg = wave_sum(gg);
  if (l == 0) sq[row] += aa * gg + (has_bias ? gg : 0.f);
}

__global__ __launch_bounds__(256) void sqrt_accumulate_kernel(const float* __restrict__ sq,
                                                              int64_t B,
                                                              float* __restrict__ accum) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) accum[i] += sqrtf(sq[i]);
}

__global__ __launch_bounds__(256) void finalize_kernel(const float* __restrict__ accum,
                                                       int64_t n, int K,
                                                       float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // K == 1 must reproduce the single-checkpoint score bit for bit: divide, don't scale
  if (i < n) out[i] = (K == 1) ? accum[i] : accum[i] / (float)K;
}

}  // namespace dd

using namespace dd;

// ------------------------------------------------------------------------------------------
// CIFAR head of the GraNd forward/backward (reference models/resnet.py:94-96: avg_pool2d(out,
// 4) -> view -> linear): the pooled features, and the gradient w.r.t. the last block's
// pre-ReLU output d[b][c][p] = scale * (e_b . W[:, c]) * (a[b][c][p] > 0), one pass each.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void head_pool_kernel(const float* __restrict__ a, int64_t BC,
                                                        int hw, float inv, float* __restrict__ feat) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < BC;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float* r = a + i * hw;
    float s = 0.f;
    if (hw % 4 == 0 && ((uintptr_t)a & 15) == 0) {
      for (int p = 0; p < hw; p += 4) {
        const float4 v = *reinterpret_cast<const float4*>(r + p);
        s += (v.x + v.y) + (v.z + v.w);
      }
    } else {
      for (int p = 0; p < hw; ++p) s += r[p];
    }
    feat[i] = s * inv;
  }
}

// one thread per 4 consecutive positions (float4) of one (example, channel) row when hw % 4 == 0,
// so consecutive lanes stream consecutive 16-byte pieces of a and d; the (e_b . W[:, c]) dot
// product (ncls FMAs, operands L2-resident) is recomputed by the hw / 4 lanes of a row
__global__ __launch_bounds__(256) void head_backward_kernel(
    const float* __restrict__ a, const float* __restrict__ e, const float* __restrict__ w,
    int64_t B, int C, int hw, int ncls, float scale, float* __restrict__ d) {
  const int per = hw % 4 == 0 ? hw / 4 : hw;  // work items per (b, c) row
  const int64_t n = B * C * per;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / per;
    const int k = (int)(i - row * per);
    const int c = (int)(row % C);
    const int64_t b = row / C;
    const float* eb = e + b * ncls;
    float g = 0.f;
    for (int j = 0; j < ncls; ++j) g = fmaf(eb[j], w[(size_t)j * C + c], g);
    g *= scale;
    if (hw % 4 == 0) {
      const size_t off = (size_t)row * hw + 4 * k;
      const float4 v = *reinterpret_cast<const float4*>(a + off);
      *reinterpret_cast<float4*>(d + off) =
          make_float4(v.x > 0.f ? g : 0.f, v.y > 0.f ? g : 0.f, v.z > 0.f ? g : 0.f,
                      v.w > 0.f ? g : 0.f);
    } else {
      const size_t off = (size_t)row * hw + k;
      d[off] = a[off] > 0.f ? g : 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Classifier y = feat W^T + bias (reference models/resnet.py:96 `self.linear(out)`), per
// (example row, class): lane l accumulates k = l, l + 64, ... in order and the 64 partials meet
// in a fixed butterfly, so a row's logits depend on that row alone -- bitwise the same whatever the
// chunk / shard size (a library GEMM picks its kernel, and its rounding, per batch size).
// The rows' features sit in registers; W rows stream from L2 / the Infinity Cache, each W
// element feeding the wave's rows.
// ------------------------------------------------------------------------------------------
template <int KPL, int R>  // features per lane (d <= 64 * KPL), rows per wave
__global__ __launch_bounds__(256) void linear_rows_kernel(const float* __restrict__ feat,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          int64_t B, int d, int C, int cslice,
                                                          float* __restrict__ out) {
  // a wave owns R rows x one slice of cslice classes (a multiple of 64): each W element it
  // loads feeds R rows (the ImageNet head's W is 8 MB; streamed once per row it was ~8 GB of
  // L2 / Infinity-Cache reads per 1024 rows), and the class slices spread a small batch over
  // more waves.  Per (row, class) the arithmetic is the one-row form's: fmaf over the row's
  // features in lane / register order, then the 64-lane butterfly -- bitwise the same.
  const int lane = threadIdx.x & 63;
  const int nslice = (C + cslice - 1) / cslice;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t items = (B + R - 1) / R * nslice;
  for (int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); it < items; it += nw) {
    const int64_t b0 = it / nslice * R;
    const int cs = (int)(it % nslice) * cslice;
    const int ce = min(C, cs + cslice);
    float f[R][KPL];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool vr = b0 + r < B;
      const float* fr = feat + (vr ? b0 + r : B - 1) * d;
#pragma unroll
      for (int i = 0; i < KPL; ++i) {
        const int k = lane + 64 * i;
        f[r][i] = (vr && k < d) ? fr[k] : 0.f;
      }
    }
    float mine[R];  // lane c % 64 keeps class c's logit; one coalesced store per 64 classes
#pragma unroll
    for (int r = 0; r < R; ++r) mine[r] = 0.f;
    for (int c = cs; c < ce; ++c) {
      const float* wr = w + (size_t)c * d;
      float wv[KPL];
#pragma unroll
      for (int i = 0; i < KPL; ++i) {
        const int k = lane + 64 * i;
        wv[i] = k < d ? wr[k] : 0.f;
      }
      const float bc = bias ? bias[c] : 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < KPL; ++i) acc = fmaf(f[r][i], wv[i], acc);
        acc = group_sum<64>(acc);
        if (lane == (c & 63)) mine[r] = acc + bc;
      }
      if ((c & 63) == 63 || c == ce - 1) {
        const int c0 = c & ~63;
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (b0 + r < B && c0 + lane <= c) out[(b0 + r) * C + c0 + lane] = mine[r];
      }
    }
  }
}

static inline int64_t conv_pad64(int64_t v) { return (v + 63) / 64 * 64; }

extern "C" {

int dd_linear_forward(const float* feat, const float* w, const float* bias, int64_t B,
                      int32_t d_in, int32_t d_out, float* out, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && d_in > 0 && d_out > 0, "dd_linear_forward: bad sizes");
  DD_REQUIRE(d_in <= 64 * 64, "dd_linear_forward: d_in %d > 4096", d_in);
  if (B == 0) return DD_OK;
  DD_REQUIRE(feat && w && out, "dd_linear_forward: null buffer");
  hipStream_t st = as_stream(stream);
  // rows per wave: 4 (each W element feeds four rows) where the features fit the registers;
  // class slices of 256 for wide heads (C = 1000: four waves share a row group)
  const int cslice = d_out > 256 ? 256 : (int)(conv_pad64(d_out));
  const int nslice = (int)ceil_div(d_out, cslice);
  auto grid = [&](int rows) {
    return (unsigned)std::min<int64_t>(ceil_div(ceil_div(B, rows) * nslice, 4), 8192);
  };
  if (d_in <= 512)
    linear_rows_kernel<8, 4><<<grid(4), 256, 0, st>>>(feat, w, bias, B, d_in, d_out, cslice, out);
  else if (d_in <= 2048)
    linear_rows_kernel<32, 4><<<grid(4), 256, 0, st>>>(feat, w, bias, B, d_in, d_out, cslice,
                                                       out);
  else
    linear_rows_kernel<64, 2><<<grid(2), 256, 0, st>>>(feat, w, bias, B, d_in, d_out, cslice,
                                                       out);
  DD_CHECK_LAUNCH("dd_linear_forward");
  return DD_OK;
}

int dd_head_pool(const float* a, int64_t B, int32_t C, int32_t hw, float* feat, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && C > 0 && hw > 0, "dd_head_pool: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(a && feat, "dd_head_pool: null buffer");
  const int64_t BC = B * C;
  head_pool_kernel<<<(unsigned)std::min<int64_t>(ceil_div(BC, 256), 65536), 256, 0,
                     as_stream(stream)>>>(a, BC, hw, 1.f / (float)hw, feat);
  DD_CHECK_LAUNCH("dd_head_pool");
  return DD_OK;
}

int dd_head_backward(const float* a, const float* e, const float* w, int64_t B, int32_t C,
                     int32_t hw, int32_t ncls, float scale, float* d, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && C > 0 && hw > 0 && ncls > 0, "dd_head_backward: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(a && e && w && d, "dd_head_backward: null buffer");
  DD_REQUIRE(hw % 4 != 0 || ((uintptr_t)a % 16 == 0 && (uintptr_t)d % 16 == 0),
             "dd_head_backward: a and d must be 16-byte aligned");
  const int64_t items = B * C * (hw % 4 == 0 ? hw / 4 : hw);
  head_backward_kernel<<<(unsigned)std::min<int64_t>(ceil_div(items, 256), 1 << 20), 256, 0,
                         as_stream(stream)>>>(a, e, w, B, C, hw, ncls, scale, d);
  DD_CHECK_LAUNCH("dd_head_backward");
  return DD_OK;
}


int dd_abi_version(void) { return 10; }

const char* dd_last_error(void) { return dd::g_err; }

int dd_normalize_u8(const uint8_t* img, int64_t n, int32_t channels, int64_t hw,
                    const float* mean_host, const float* std_host, float* out, void* stream) {
  clear_error();
  return launch_normalize(img, nullptr, n, channels, hw, mean_host, std_host, out,
                          as_stream(stream));
}

int dd_normalize_u8_gather(const uint8_t* img, const int64_t* index, int64_t n,
                           int32_t channels, int64_t hw, const float* mean_host,
                           const float* std_host, float* out, void* stream) {
  clear_error();
  DD_REQUIRE(index || n == 0, "dd_normalize_u8_gather: null index");
  return launch_normalize(img, index, n, channels, hw, mean_host, std_host, out,
                          as_stream(stream));
}

int dd_el2n(const float* logits, const int64_t* labels, int64_t B, int32_t C, float* score,
            float* e, float* accum, int32_t* bad_labels, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0, "dd_el2n: B < 0");
  DD_REQUIRE(C > 0, "dd_el2n: C must be positive (got %d)", C);
  if (B == 0) return DD_OK;
  DD_REQUIRE(logits && labels, "dd_el2n: null logits/labels");
  hipStream_t st = as_stream(stream);
  if (C <= 16)
    launch_el2n_lds<16, 1>(logits, labels, B, C, score, e, accum, bad_labels, st);
  else if (C <= 32)
    launch_el2n_lds<32, 1>(logits, labels, B, C, score, e, accum, bad_labels, st);
  else if (C <= 64)
    launch_el2n_lds<32, 2>(logits, labels, B, C, score, e, accum, bad_labels, st);
  else if (C <= 128)
    launch_el2n_lds<32, 4>(logits, labels, B, C, score, e, accum, bad_labels, st);
  else if (C <= 256)
    launch_el2n<64, 4>(logits, labels, B, C, score, e, accum, bad_labels, st);
  else if (C <= 1024)
    launch_el2n<64, 16>(logits, labels, B, C, score, e, accum, bad_labels, st);
  else if (C <= 2048)
    launch_el2n<64, 32>(logits, labels, B, C, score, e, accum, bad_labels, st);
  else
    el2n_wide_kernel<<<(unsigned)B, 256, 0, st>>>(logits, labels, B, C, score, e, accum,
                                                  bad_labels);
  DD_CHECK_LAUNCH("dd_el2n");
  return DD_OK;
}

int dd_linear_pegrad_sqnorm(const float* act, const float* gout, int64_t B, int32_t d_in,
                            int32_t d_out, int32_t has_bias, float* sq_accum, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && d_in > 0 && d_out > 0, "dd_linear_pegrad_sqnorm: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(act && gout && sq_accum, "dd_linear_pegrad_sqnorm: null buffer");
  linear_pegrad_kernel<<<(unsigned)ceil_div(B, 4), 256, 0, as_stream(stream)>>>(
      act, gout, B, d_in, d_out, has_bias, sq_accum);
  DD_CHECK_LAUNCH("dd_linear_pegrad_sqnorm");
  return DD_OK;
}

int dd_sqrt_accumulate(const float* sq, int64_t B, float* accum, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0, "dd_sqrt_accumulate: B < 0");
  if (B == 0) return DD_OK;
  DD_REQUIRE(sq && accum, "dd_sqrt_accumulate: null buffer");
  sqrt_accumulate_kernel<<<(unsigned)ceil_div(B, 256), 256, 0, as_stream(stream)>>>(sq, B,
                                                                                    accum);
  DD_CHECK_LAUNCH("dd_sqrt_accumulate");
  return DD_OK;
}

int dd_ensemble_finalize(const float* accum, int64_t n, int32_t K, float* out, void* stream) {
  clear_error();
  DD_REQUIRE(n >= 0 && K >= 1, "dd_ensemble_finalize: bad n/K");
  if (n == 0) return DD_OK;
  DD_REQUIRE(accum && out, "dd_ensemble_finalize: null buffer");
  finalize_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, as_stream(stream)>>>(
      accum, n, K, out);
  DD_CHECK_LAUNCH("dd_ensemble_finalize");
  return DD_OK;
}

int64_t dd_keep_count(int64_t train_samples, double sparsity) {
  // reference get_scores_and_prune.py:22: int((1 - sparsity) * train_samples), IEEE double,
  // truncation toward zero (Python int() of a float)
  const double v = (1.0 - sparsity) * (double)train_samples;
  return (int64_t)v;
}

}  // extern "C"
