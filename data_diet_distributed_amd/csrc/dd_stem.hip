// GraNd per-example weight-gradient norm of the network's input conv (reference
// models/resnet.py:71, conv1 3 -> 64, 3x3 / stride 1 / pad 1 on 32x32 CIFAR images) on
// split-bf16 MFMA.  The reference has no GraNd.
//
// With only cin = 3 input channels the im2col has d_a = 27 rows, so the weight gradient
// G = U^T g (27 x cout per example) is one 32-row MFMA block: the generic all-taps kernel,
// which pads cin to a 64-channel block, would multiply 21x zeros.  Here the GEMM is
//   D[m][o] = sum_t U[t][m] g[o][t],   m = (c, ky, kx) < cin * 9 padded to 32,
// over all T = H*W output positions, K = t: the A fragment of lane (m, k-half) is 8
// consecutive positions of one (c, tap) — 8 floats of one row of the zero-padded image staged
// in LDS, shifted by the tap — and the B fragment is 8 consecutive positions of one output
// channel, two float4 straight from HBM (g is read exactly once and never staged).  Each of
// the 4 waves runs a quarter of the positions for all output channels; the partial D's are
// summed across the waves in LDS and squared.  The kernel is bound by reading g once
// (4 cout T bytes per example); the MFMA work is 2 T 32 cout flop.
#include "dd_mfma.h"
#include "dd_stem.h"

namespace dd {
namespace stem {

using namespace conv;

constexpr int MAXC = 3;   // input channels (cin * 9 <= 32)
constexpr int NOB = 2;    // 32-channel output blocks (cout <= 64)

template <int W>
__global__ __launch_bounds__(256, 2) void stem_kernel(const float* __restrict__ act,
                                                      const float* __restrict__ gout, int cin,
                                                      int H, int cout,
                                                      const float* __restrict__ col_scale,
                                                      float* __restrict__ sq) {
  constexpr int PW = W + 2;  // padded row pitch (floats)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int PLANE = (H + 2) * PW;
  float* img = sm;                   // [cin][H + 2][PW], zero border
  float* red = sm + MAXC * PLANE;    // [4 waves][NOB][16][64] partial D's
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int T = H * W;

  // ---- the zero-padded image
  for (int i = tid; i < MAXC * PLANE; i += 256) img[i] = 0.f;
  __syncthreads();
  const float* __restrict__ xa = act + (size_t)b * cin * T;
  for (int i = tid; i < cin * T / 4; i += 256) {
    const float4 v = *reinterpret_cast<const float4*>(xa + 4 * i);
    const int c = (4 * i) / T, r = 4 * i - c * T, y = r / W, x = r - y * W;
    float* d = img + c * PLANE + (y + 1) * PW + x + 1;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
  __syncthreads();

  // ---- lane roles: A row m = (c, ky, kx), B column o, k half hk (positions 8 hk .. 8 hk + 7
  // of each 16-position step)
  const int m = lane & 31, hk = lane >> 5;
  const bool vm = m < cin * 9;
  const int c = m / 9, tap = m - 9 * (m / 9);
  const int aoff = vm ? c * PLANE + (tap / 3) * PW + tap % 3 : 0;
  const float am = vm ? 1.f : 0.f;
  const float* __restrict__ gb = gout + (size_t)b * cout * T;
  const float* gp[NOB];
  float so[NOB];
#pragma unroll
  for (int j = 0; j < NOB; ++j) {
    const int o = j * 32 + m;
    const int oc = o < cout ? o : cout - 1;
    gp[j] = gb + (size_t)oc * T + 8 * hk;
    so[j] = o < cout ? (col_scale ? col_scale[oc] : 1.f) : 0.f;
  }

  floatx16 acc[NOB];
#pragma unroll
  for (int j = 0; j < NOB; ++j) acc[j] = floatx16{0};
  const int nks = T / 16 / 4;  // 16-position steps per wave
  const int ks0 = wv * nks;
  float4 gr[2][NOB][2];
  auto load_g = [&](float4 (&r)[NOB][2], int ks) {
#pragma unroll
    for (int j = 0; j < NOB; ++j) {
      const float* p = gp[j] + ks * 16;
      r[j][0] = *reinterpret_cast<const float4*>(p);
      r[j][1] = *reinterpret_cast<const float4*>(p + 4);
    }
  };
  auto step = [&](const float4 (&r)[NOB][2], int ks) {
    const int t0 = ks * 16 + 8 * hk;
    const int y = t0 / W, x0 = t0 - y * W;
    const float* ap = img + aoff + y * PW + x0;
    bf16x8 ah, al;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __bf16 hi, lo;
      split_bf16(ap[i] * am, hi, lo);
      ah[i] = hi;
      al[i] = lo;
    }
#pragma unroll
    for (int j = 0; j < NOB; ++j) {
      const float f[8] = {r[j][0].x, r[j][0].y, r[j][0].z, r[j][0].w,
                          r[j][1].x, r[j][1].y, r[j][1].z, r[j][1].w};
      bf16x8 bh, bl;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        __bf16 hi, lo;
        split_bf16(f[i] * so[j], hi, lo);
        bh[i] = hi;
        bl[i] = lo;
      }
      floatx16 d = acc[j];
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, d, 0, 0, 0);
      acc[j] = d;
    }
  };
  // two register sets: step k + 1's loads are in flight while step k multiplies
  load_g(gr[0], ks0);
  for (int k = 0; k < nks; k += 2) {
    load_g(gr[1], ks0 + (k + 1 < nks ? k + 1 : k));
    step(gr[0], ks0 + k);
    if (k + 1 >= nks) break;
    load_g(gr[0], ks0 + (k + 2 < nks ? k + 2 : k + 1));
    step(gr[1], ks0 + k + 1);
  }

  // ---- sum the 4 waves' partial D's, square, reduce
#pragma unroll
  for (int j = 0; j < NOB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((wv * NOB + j) * 16 + r) * 64 + lane] = acc[j][r];
  __syncthreads();
  constexpr int NE = NOB * 16 * 64;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < NE / 256; ++i) {
    const int e = tid + 256 * i;
    const float s = (red[e] + red[NE + e]) + (red[2 * NE + e] + red[3 * NE + e]);
    v += s * s;
  }
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  if (tid == 0) sq[b] += (red[0] + red[1]) + (red[2] + red[3]);
}

static size_t lds_bytes(int h, int w) {
  return ((size_t)MAXC * (h + 2) * (w + 2) + 4 * NOB * 16 * 64) * sizeof(float);
}

}  // namespace stem

bool stem_ok(const dd_conv_geom* g) {
  return g->kh == 3 && g->kw == 3 && g->pad == 1 && g->stride == 1 && g->cin * 9 <= 32 &&
         g->cin <= stem::MAXC && g->cout <= 32 * stem::NOB && g->ho == g->h && g->wo == g->w &&
         (g->w == 8 || g->w == 16 || g->w == 32) && (g->h * g->w) % 64 == 0 && g->h <= 64;
}

int stem_launch(const float* act, const float* gout, const dd_conv_geom* g,
                const float* col_scale, float* sq, hipStream_t st) {
  const size_t lds = stem::lds_bytes(g->h, g->w);
  const unsigned grid = (unsigned)g->batch;
#define DD_STEM(W_)                                                                           \
  {                                                                                           \
    static bool attr = false;                                                                 \
    if (!attr) {                                                                              \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem::stem_kernel<W_>),        \
                                hipFuncAttributeMaxDynamicSharedMemorySize,                   \
                                (int)stem::lds_bytes(64, W_));                                \
      attr = true;                                                                            \
    }                                                                                         \
    stem::stem_kernel<W_><<<grid, 256, lds, st>>>(act, gout, g->cin, g->h, g->cout,           \
                                                  col_scale, sq);                             \
  }
  if (g->w == 32) DD_STEM(32)
  else if (g->w == 16) DD_STEM(16)
  else DD_STEM(8)
#undef DD_STEM
  DD_CHECK_LAUNCH("dd_conv_pegrad_sqnorm(stem)");
  return DD_OK;
}

}  // namespace dd
