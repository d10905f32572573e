// Split-bf16 1x1 convolution (a batched GEMM over positions), NCHW fp32 in and out: the
// Bottleneck convs of ResNet-50 (reference models/resnet.py:40, 44: conv1, conv3) and the 1x1
// projection shortcuts (:49-54, stride 1 or 2), forward and backward-data.
//
//   y[b][o][p] = epi( sum_c W[o][c] * xf(x[b][c][s p]) )     p an output position, s = stride
//
// GEMM: M = output channels, K = input channels, N = the flattened (example, position) space
// (P = b * HWo + p).  A workgroup owns 128 consecutive P (one example's run of positions, or
// several whole examples when HWo < 128) x OB output channels; 4 waves as 2 (o) x 2 (P).  K loop
// over chunks of 32 input channels: the chunk is converted to bf16 hi/lo while staged in LDS
// channel-major ([hi|lo][c][P], rows padded so the transposed reads are conflict-free), double
// buffered; B fragments (8 consecutive channels at one position) are ds_read_b64_tr_b16 pairs
// as in dd_conv.hip.  A fragments are the dd_conv1x1_pack layout (pre-split, from L2).
// Products hi*hi + hi*lo + lo*hi, fp32 accumulation (~2^-16 relative per product).
//
// Epilogue (same operations and BN-statistics layout as dd_conv3x3_forward):
//   v = acc + bias[o] + residual + up2(residual_up2) -> ReLU? -> * (mask_src > 0)
// where up2(r)[y][x] = r[y/2][x/2] at even (y, x) and 0 elsewhere: the backward of a 1x1
// stride-2 projection (its transposed conv scatters to even positions), added to the
// backward of the block's conv1 in the same pass.  xf = the producer's grouped train-mode BN
// + ReLU applied while staging (EL2N pass).
#include "dd_mfma.h"

namespace dd {
namespace c1 {

using namespace conv;

constexpr int KC = 32;          // input channels per K chunk (two MFMA K steps)
constexpr int TB = 128;         // flattened positions per workgroup
constexpr int XS = TB * 2 + 64; // bytes of one staged channel row (bf16), padded for banks
constexpr int PLANE = KC * XS;  // one hi or lo plane
constexpr int BUF = 2 * PLANE;
constexpr int LDS = 2 * BUF + 16384;  // two K buffers + 4 x 4 KB epilogue transpose blocks

struct Args {
  const float* x;
  const __bf16* wpack;
  const float* bias;
  const float* residual;
  const float* res_up2;  // [B][cout][HWo/4] at (y/2, x/2), or NULL
  const float* mask_src;
  const float* in_scale;
  const float* in_shift;
  float* y;
  float* stats;
  int64_t B, n_stat;
  int cin, cout, op, H, W, Ho, Wo, stride;
  int relu, gsize, tiles_per_group;
  float in_floor;
  int n_ob, n_tiles;
};

// NA: 32-row output blocks per wave (wave = NA*32 o x 64 P); VEC: HWo % 4 == 0 and stride 1
// (float4 staging and stores); S2: stride-2 input gather; XF: staging transform
template <int NA, bool VEC, bool XF>
__global__ __launch_bounds__(256, NA == 1 ? 2 : 1) void conv1x1_kernel(const Args A) {
  constexpr int NT = 2;            // 32-wide P tiles per wave (64 P)
  constexpr int OB = 2 * NA * 32;  // output channels per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wo = wv & 1, wt = wv >> 1, h = lane >> 5;
  const int cin = A.cin, cout = A.cout;
  const int HWo = A.Ho * A.Wo, HWi = A.H * A.W;
  const int64_t Ptot = A.B * HWo;
  const float* __restrict__ x = A.x;

  struct Tile {
    int64_t P0, b0, grp;
    int o0, ob32, xf_base;
  };
  auto decode = [&](int tile) {
    Tile T;
    T.o0 = (tile % A.n_ob) * OB;
    T.P0 = (int64_t)(tile / A.n_ob) * TB;
    T.b0 = T.P0 / HWo;
    // a tile never straddles a BN group (group_size * HWo is a multiple of TB, or the tile
    // lies in one example)
    T.grp = T.b0 / A.gsize;
    T.xf_base = (int)(T.grp * cin);
    T.ob32 = (T.o0 >> 5) + wo * NA;
    return T;
  };

  // source element (channel c, flattened output position P) -> input offset
  auto src_off = [&](int64_t P, int c) -> int64_t {
    const int64_t b = P / HWo;
    const int p = (int)(P - b * HWo);
    int pi = p;
    if (A.stride == 2) {
      const int yo = p / A.Wo, xo = p - yo * A.Wo;
      pi = 2 * yo * A.W + 2 * xo;
    }
    return (b * cin + c) * (int64_t)HWi + pi;
  };

  // ---- staging: 32 channels x 128 positions = 1024 quads of 4 positions, 4 per thread
  constexpr int NQ = KC * TB / 4 / 256;
  float4 ra[NQ];
  float xs[NQ], xt[NQ];
  auto load_chunk = [&](const Tile& T, int c0) {
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int q = tid + 256 * k;
      const int i4 = q % (TB / 4), c = q / (TB / 4);
      const int cg = c0 + c, cgc = cg < cin ? cg : cin - 1;
      const int64_t P = T.P0 + 4 * i4;
      if constexpr (VEC) {
        const int64_t Pc = P < Ptot ? P : Ptot - 4;
        ra[k] = *reinterpret_cast<const float4*>(x + src_off(Pc, cgc));
      } else {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t Pj = P + j < Ptot ? P + j : Ptot - 1;
          v[j] = x[src_off(Pj, cgc)];
        }
        ra[k] = make_float4(v[0], v[1], v[2], v[3]);
      }
      if constexpr (XF) {
        xs[k] = A.in_scale[T.xf_base + cgc];
        xt[k] = A.in_shift[T.xf_base + cgc];
      }
    }
  };
  auto store_chunk = [&](const Tile& T, int c0, int buf) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int q = tid + 256 * k;
      const int i4 = q % (TB / 4), c = q / (TB / 4);
      float v[4] = {ra[k].x, ra[k].y, ra[k].z, ra[k].w};
      const bool cok = c0 + c < cin;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float u = v[j];
        if constexpr (XF) u = fmaxf(fmaf(u, xs[k], xt[k]), A.in_floor);
        v[j] = (cok && T.P0 + 4 * i4 + j < Ptot) ? u : 0.f;
      }
      const uint32_t h01 = pack_bf16x2(v[0], v[1]), h23 = pack_bf16x2(v[2], v[3]);
      const uint32_t l01 = pack_bf16x2(v[0] - __uint_as_float(h01 << 16),
                                       v[1] - __uint_as_float(h01 & 0xffff0000u));
      const uint32_t l23 = pack_bf16x2(v[2] - __uint_as_float(h23 << 16),
                                       v[3] - __uint_as_float(h23 & 0xffff0000u));
      char* p = base + c * XS + i4 * 8;
      *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
      *reinterpret_cast<uint2*>(p + PLANE) = make_uint2(l01, l23);
    }
  };

  // ---- weights: per chunk 2 K steps x NA blocks x hi|lo fragments (16 B per lane)
  bf16x8 wa[2][NA][2];
  const int nob32 = A.op >> 5;
  auto load_w = [&](int ob32, int c0) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        const __bf16* p = A.wpack + ((size_t)((c0 / CC + s) * nob32 + ob32 + a) * 2) * 512 +
                          lane * 8;
        wa[s][a][0] = *reinterpret_cast<const bf16x8*>(p);
        wa[s][a][1] = *reinterpret_cast<const bf16x8*>(p + 512);
      }
  };

  // transposed-read geometry (dd_conv.hip): lane 4q+p of each 16-lane group supplies channel
  // row q, positions 4p..4p+3 of the group's 16 positions
  const int q = (lane >> 2) & 3, pp = lane & 3, g1 = (lane >> 4) & 1;
  int rd[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) rd[n] = (wt * 64 + n * 32 + 16 * g1 + 4 * pp) * 2;

  floatx16 acc[NA][NT];

  auto compute = [&](const char* base) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 bf[NT][2];
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const char* a = base + (16 * s + 8 * h + q) * XS + rd[n];
        bf[n][0] = tr_read8(a, a + 4 * XS);
        bf[n][1] = tr_read8(a + PLANE, a + PLANE + 4 * XS);
      }
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          floatx16 d = acc[a][n];
          d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s][a][0], bf[n][0], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s][a][0], bf[n][1], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s][a][1], bf[n][0], d, 0, 0, 0);
          acc[a][n] = d;
        }
    }
  };

  // ---- epilogue: each 32x32 fragment transposed through a wave-private 4 KB LDS block so a
  // lane owns 4 consecutive positions of one channel (float4 loads / stores when VEC)
  auto epilogue = [&](const Tile& T) {
    float* ep = reinterpret_cast<float*>(smem + 2 * BUF) + wv * 1024;
    const int tl = lane & 7, ol = lane >> 3;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ep[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + (lane & 31)] = acc[a][n][r];
        asm volatile("" ::: "memory");
        float4 vv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          vv[k] = *reinterpret_cast<const float4*>(ep + (8 * k + ol) * 32 + 4 * tl);
        asm volatile("" ::: "memory");
        const int64_t Pf = T.P0 + wt * 64 + n * 32;  // the fragment's first position
        const int64_t P = Pf + 4 * tl;
        const int ob = T.o0 + (wo * NA + a) * 32 + ol;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int o = ob + 8 * k;
          const int oc = o < cout ? o : cout - 1;
          float f[4] = {vv[k].x, vv[k].y, vv[k].z, vv[k].w};
          float s_ = 0.f, q_ = 0.f;
          const float bia = A.bias ? A.bias[oc] : 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t Pj = P + j;
            const bool live = Pj < Ptot;
            const int64_t Pc = live ? Pj : Ptot - 1;
            const int64_t b = Pc / HWo;
            const int p = (int)(Pc - b * HWo);
            const int64_t oi = (b * cout + oc) * (int64_t)HWo + p;
            float u = f[j] + bia;
            if (A.residual) u += A.residual[oi];
            if (A.res_up2) {
              const int yo = p / A.Wo, xo = p - yo * A.Wo;
              if (!(yo & 1) && !(xo & 1))
                u += A.res_up2[(b * cout + oc) * (int64_t)(HWo / 4) + (yo >> 1) * (A.Wo >> 1) +
                               (xo >> 1)];
            }
            if (A.relu) u = fmaxf(u, 0.f);
            if (A.mask_src && !(A.mask_src[oi] > 0.f)) u = 0.f;
            f[j] = u;
            const float us = (live && b < A.n_stat) ? u : 0.f;
            s_ += us;
            q_ += us * us;
            if (!VEC && live && o < cout) A.y[oi] = u;
          }
          if constexpr (VEC) {
            const int64_t b = (P < Ptot ? P : Ptot - 1) / HWo;
            const int p = (int)(P - b * HWo);
            if (P < Ptot && o < cout)
              *reinterpret_cast<float4*>(A.y + (b * cout + o) * (int64_t)HWo + p) =
                  make_float4(f[0], f[1], f[2], f[3]);
          }
          if (A.stats) {
            // the 8 lanes of one channel hold its 32 positions of this fragment
            s_ = sum8(s_);
            q_ = sum8(q_);
            const int64_t pi = (Pf - T.grp * A.gsize * (int64_t)HWo) >> 5;
            if (tl == 0 && o < cout)
              *reinterpret_cast<float2*>(
                  A.stats + (((size_t)T.grp * cout + o) * A.tiles_per_group + pi) * 2) =
                  make_float2(s_, q_);
          }
        }
      }
  };

  const int nchunks = (cin + KC - 1) / KC;
  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    const Tile T = decode(tile);
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[a][n] = floatx16{0};
    load_chunk(T, 0);
    load_w(T.ob32, 0);
    store_chunk(T, 0, 0);
    __syncthreads();
    for (int kc = 0; kc < nchunks; ++kc) {
      const int cur = kc & 1;
      const bool more = kc + 1 < nchunks;
      if (more) load_chunk(T, (kc + 1) * KC);
      compute(smem + cur * BUF);
      if (more) {
        load_w(T.ob32, (kc + 1) * KC);
        store_chunk(T, (kc + 1) * KC, cur ^ 1);
      }
      __syncthreads();
    }
    epilogue(T);
  }
}

// the pack's K is padded to 32 (two 16-channel pack chunks per K chunk)
static int launch_any(const Args& a0, int na, hipStream_t st) {
  Args a = a0;
  const bool vec = (a.stride == 1) && (a.Ho * a.Wo) % 4 == 0 &&
                   (uintptr_t)a.x % 16 == 0 && (uintptr_t)a.y % 16 == 0;
  const int OB = 2 * na * 32;
  a.n_ob = (a.op + OB - 1) / OB;
  const int64_t ntiles = ceil_div(a.B * a.Ho * a.Wo, TB) * a.n_ob;
  DD_REQUIRE(ntiles < (1ll << 31), "dd_conv1x1_forward: too many tiles");
  a.n_tiles = (int)ntiles;
  const int64_t cap = (na == 2 ? 1 : 2) * (int64_t)device_cus();
  const dim3 g((unsigned)std::min<int64_t>(ntiles, cap));
  const bool xf = a.in_scale != nullptr;
  static bool attr = false;
  if (!attr) {
    for (const void* f : {reinterpret_cast<const void*>(&conv1x1_kernel<1, true, false>),
                          reinterpret_cast<const void*>(&conv1x1_kernel<1, true, true>),
                          reinterpret_cast<const void*>(&conv1x1_kernel<1, false, false>),
                          reinterpret_cast<const void*>(&conv1x1_kernel<1, false, true>),
                          reinterpret_cast<const void*>(&conv1x1_kernel<2, true, false>),
                          reinterpret_cast<const void*>(&conv1x1_kernel<2, true, true>),
                          reinterpret_cast<const void*>(&conv1x1_kernel<2, false, false>),
                          reinterpret_cast<const void*>(&conv1x1_kernel<2, false, true>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
#define DD_C1(NA_, V_, X_) conv1x1_kernel<NA_, V_, X_><<<g, 256, LDS, st>>>(a)
  if (na == 2) {
    if (vec) xf ? DD_C1(2, true, true) : DD_C1(2, true, false);
    else xf ? DD_C1(2, false, true) : DD_C1(2, false, false);
  } else {
    if (vec) xf ? DD_C1(1, true, true) : DD_C1(1, true, false);
    else xf ? DD_C1(1, false, true) : DD_C1(1, false, false);
  }
#undef DD_C1
  DD_CHECK_LAUNCH("dd_conv1x1_forward");
  return DD_OK;
}

}  // namespace c1
}  // namespace dd

using namespace dd;

extern "C" {

int dd_conv1x1_tiles_per_group(int32_t ho, int32_t wo, int32_t group_size) {
  const int64_t hw = (int64_t)ho * wo;
  if (group_size <= 0 || hw <= 0) return -1;
  // every 32-position fragment and every 128-position tile inside one BN group
  if ((group_size * hw) % c1::TB != 0) return -1;
  if (hw % 32 != 0 && 32 % hw != 0) return -1;
  return (int)(group_size * hw / 32);
}

int dd_conv1x1_forward(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                       int32_t stride, const void* packed, int32_t cout, const float* bias,
                       const float* residual, const float* res_up2, const float* mask_src,
                       int32_t relu, const float* in_scale, const float* in_shift,
                       int32_t in_relu, int32_t group_size, int64_t n_stat, float* stats,
                       float* y, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && cin > 0 && cout > 0 && h > 0 && w > 0, "dd_conv1x1_forward: bad sizes");
  DD_REQUIRE(stride == 1 || stride == 2, "dd_conv1x1_forward: stride must be 1 or 2");
  DD_REQUIRE(stride == 1 || (h % 2 == 0 && w % 2 == 0),
             "dd_conv1x1_forward: stride 2 needs an even input");
  if (B == 0) return DD_OK;
  DD_REQUIRE(x && packed && y, "dd_conv1x1_forward: null buffer");
  DD_REQUIRE(!in_scale == !in_shift, "dd_conv1x1_forward: in_scale and in_shift go together");
  const int ho = h / stride, wo = w / stride;
  DD_REQUIRE(!res_up2 || (ho % 2 == 0 && wo % 2 == 0),
             "dd_conv1x1_forward: res_up2 needs an even output");
  DD_REQUIRE((int64_t)cin * h * w < (1ll << 31) && (int64_t)cout * ho * wo < (1ll << 31),
             "dd_conv1x1_forward: per-example tensor too large");
  c1::Args a{};
  a.x = x;
  a.wpack = static_cast<const __bf16*>(packed);
  a.bias = bias;
  a.residual = residual;
  a.res_up2 = res_up2;
  a.mask_src = mask_src;
  a.y = y;
  a.stats = stats;
  a.B = B;
  a.cin = cin;
  a.cout = cout;
  a.op = conv::pad_to(cout, 64);
  a.H = h;
  a.W = w;
  a.Ho = ho;
  a.Wo = wo;
  a.stride = stride;
  a.relu = relu;
  const bool grouped = in_scale || stats;
  DD_REQUIRE(!grouped || group_size > 0, "dd_conv1x1_forward: group_size must be positive");
  a.gsize = grouped ? group_size : (int)std::min<int64_t>(B + c1::TB, 1 << 30);
  if (grouped) {
    const int tpg = dd_conv1x1_tiles_per_group(ho, wo, group_size);
    DD_REQUIRE(tpg > 0, "dd_conv1x1_forward: no grouped layout for %dx%d with group_size %d",
               ho, wo, group_size);
    a.tiles_per_group = tpg;
  }
  a.n_stat = stats ? std::min<int64_t>(std::max<int64_t>(n_stat, 0), B) : 0;
  a.in_scale = in_scale;
  a.in_shift = in_shift;
  a.in_floor = in_relu ? 0.f : -INFINITY;
  // wide tiles (64 o per wave, 128 per workgroup) where the padded outputs are a multiple
  // of 128 (every ResNet width above 64); narrow (64 per workgroup) otherwise
  return c1::launch_any(a, a.op % 128 == 0 ? 2 : 1, as_stream(stream));
}

}  // extern "C"
