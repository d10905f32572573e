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

#include <stdlib.h>

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
  int kh, kw, pad, nkc;  // taps (1x1: 1, 1, 0) and K chunks (per tap unless dense)
  int dense;             // K = (channel, tap) dense (MODE 3)
  int relu, gsize, tiles_per_group;
  float in_floor;
  int n_ob, n_tiles;
  int xcd;               // XCD-contiguous persistent tile order (DD_C1_XCD)
  int f16;               // fp16 operand halves (DD_OPERANDS_F16X3)
  float acc_scale;       // fp16 packs hold W * 2^s: accumulators times 2^-s (exact)
  // fused residual-unit input (XU > 0, dd_conv1x1_forward_unit_input): the staged value is
  // relu(x * in_scale + in_shift [+ xres (* xres_scale + xres_shift)]), in dd_bn_apply's order,
  // and the output-block-0 tiles write it to xout once
  float* xout;
  const float* xres;
  const float* xres_scale;
  const float* xres_shift;
};

// Tile families (4 waves as WO along o x 4/WO along P; a wave owns NA 32-row output blocks x
// NT 32-position tiles): WO = 2 (NA = 1: 64 o per workgroup), WO = 4 (NA = 1 / 2: 128 / 256 o
// per workgroup, every wave over all 128 positions).  The widest family the padded outputs
// fill stages each input element once for up to 256 outputs: at short K (64-256 input
// channels) the tile's input staging, not the MFMAs, is the cost.
// Staging MODE 0: 1x1 with HWo % 4 == 0 (and Wo % 4 == 0 at stride 2), float4 loads;
// 1: 1x1, scalar; 2: any kh x kw / stride / pad as an implicit GEMM with K = (tap, channel)
// tap-major, each K chunk gathering one tap's shifted window of 32 channels (zero outside
// the image); 3: the same with K = (channel, tap) dense (PyTorch's weight order), for inputs
// with few channels (the 7x7 ImageNet stem: K = 147 in 5 chunks instead of 49).
// 4: MODE 2's 3x3 / stride 1 / pad 1 special case when the width is a multiple of 4 (the
// ImageNet-stem network's 56x56 and 28x28 maps): a thread's 4 positions are one aligned quad of
// an output row, so a tap's shifted window is ONE float4 buffer load of the input row (the kx = 1
// tap) plus, for kx = 0 / 2, the one column left / right of it (a dword load), instead of four
// dword gathers; staged values, K order and MFMAs are MODE 2's, so results are bitwise equal.
// VE: float4 epilogue (HWo % 4 == 0, 16-B aligned).  XF: staging transform.  F16: fp16 operand
// halves (DD_OPERANDS_F16X3: the EL2N forward), else bf16.
// EPI: 0 = the epilogue's operations read at run time from Args (any combination); otherwise
// kC1Spec | the operations present, each compiled to exactly its own epilogue (the launch
// shapes of the scoring passes: EL2N statistics; GraNd forward bias + ReLU, + residual, bias;
// GraNd backward mask, + residual, + up2 residual, plain)
constexpr int kC1Bias = 1, kC1Res = 2, kC1Msk = 4, kC1Up2 = 8, kC1Relu = 16, kC1Stats = 32,
              kC1Spec = 64;
// XU: the fused residual-unit input (0 none; 1 relu(bn(x)); 2 + identity residual; 3 +
// residual with its own BN affine) -- MODE 0, stride 1, with the staging transform
template <int NA, int WO, int MODE, bool VE, bool XF, bool F16 = false, int EPI = 0, int XU = 0>
__global__ __launch_bounds__(256, (NA == 1 && (WO == 2 || MODE != 3)) ? 2 : 1) void conv1x1_kernel(
    const Args A) {
  constexpr int WT = 4 / WO;       // waves along P
  constexpr int TW = TB / WT;      // positions per wave
  constexpr int NT = TW / 32;      // 32-wide P tiles per wave
  constexpr int OB = WO * NA * 32; // output channels per workgroup
  constexpr bool VEC = MODE == 0;  // float4 staging
  constexpr bool TAPS = MODE >= 2;
  constexpr bool ROWQ = MODE == 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wo = wv % WO, wt = wv / WO, h = lane >> 5;
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

  // ---- staging: 32 channels x 128 positions = 1024 quads of 4 positions, 4 per thread.  A
  // thread always stages the same position quad (i4 = tid % 32) for channels tid / 32 + 8 k,
  // so the quad's input offsets are computed once per tile (32-bit divisions: P < 2^31)
  constexpr int NQ = KC * TB / 4 / 256;
  const int i4 = tid % (TB / 4), cq0 = tid / (TB / 4);
  int64_t poff[4];  // input offset of position j of the quad (channel 0); VEC uses [0]
  bool pval[4];
  int pyi[4], pxi[4];  // MODE 2: top-left input coordinate of position j's window
  // MODE 4: a buffer resource over the tile's first example and the next (a 128-position tile
  // spans at most two, HWo >= 128), poff[0] = the quad's example offset relative to it
  __amdgpu_buffer_rsrc_t xq_rsrc;
  auto pos_offsets = [&](const Tile& T) {
    if constexpr (ROWQ) {
      const int64_t nb = A.B - T.b0 < 2 ? A.B - T.b0 : 2;
      xq_rsrc = buffer_rsrc(x + T.b0 * cin * (int64_t)HWi, (uint32_t)(nb * cin * HWi * 4));
    }
#pragma unroll
    for (int j = 0; j < (VEC || ROWQ ? 1 : 4); ++j) {
      const int64_t P = T.P0 + 4 * i4 + j;
      pval[j] = P < Ptot;
      const unsigned Pc = (unsigned)(P < Ptot ? P : Ptot - 1);
      const unsigned b = Pc / (unsigned)HWo, p = Pc - b * (unsigned)HWo;
      const unsigned yo = p / (unsigned)A.Wo, xo = p - yo * (unsigned)A.Wo;
      unsigned pi = p;
      if (A.stride == 2) pi = 2 * yo * A.W + 2 * xo;
      if (ROWQ) {
        pyi[j] = (int)yo - 1;  // the quad's row above (tap row ky = 0)
        pxi[j] = (int)xo;      // the quad's first column
        poff[j] = (int64_t)(b - (unsigned)T.b0) * cin * HWi;
      } else if (TAPS) {
        pyi[j] = (int)yo * A.stride - A.pad;
        pxi[j] = (int)xo * A.stride - A.pad;
        poff[j] = (int64_t)b * cin * HWi;
      } else {
        poff[j] = (int64_t)b * cin * HWi + pi;
      }
    }
    if (VEC || ROWQ) pval[1] = pval[2] = pval[3] = pval[0];
    if constexpr (VEC) {
      // stride 2: the quad's second pair (positions 2, 3), which starts the next output row
      // when the width is even but not a multiple of 4 (a pair never straddles one)
      if (A.stride == 2) {
        const int64_t P = T.P0 + 4 * i4 + 2;
        const unsigned Pc = (unsigned)(P < Ptot ? P : Ptot - 1);
        const unsigned b = Pc / (unsigned)HWo, p = Pc - b * (unsigned)HWo;
        const unsigned yo = p / (unsigned)A.Wo, xo = p - yo * (unsigned)A.Wo;
        poff[2] = (int64_t)b * cin * HWi + 2 * yo * A.W + 2 * xo;
      }
    }
  };
  // validity of element (channel row k, position j) of the staged chunk, bit 4 k + j: the
  // channel exists, the position exists, and (TAPS) its tap lies inside the image
  uint32_t vm = 0;
  static_assert(XU == 0 || (MODE == 0 && XF), "the unit input is a float4 1x1 staging mode");
  float4 ra[NQ];
  float4 rv[XU >= 2 ? NQ : 1];
  float rs[XU == 3 ? NQ : 1], rt[XU == 3 ? NQ : 1];
  float xs[NQ], xt[NQ];
  auto load_chunk = [&](const Tile& T, int kc) {
    const int tap = MODE == 2 || ROWQ ? kc / A.nkc : 0;
    const int c0 = (MODE == 2 || ROWQ ? kc - tap * A.nkc : kc) * KC;
    int64_t toff[4];
    bool tin[4];
    if constexpr (MODE == 2) {
      const int ky = tap / A.kw, kx = tap - ky * A.kw;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int yi = pyi[j] + ky, xi = pxi[j] + kx;
        tin[j] = yi >= 0 && yi < A.H && xi >= 0 && xi < A.W;
        toff[j] = poff[j] + (tin[j] ? (int64_t)yi * A.W + xi : 0);
      }
    }
    vm = 0;
    const int taps = A.kh * A.kw;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int cg = c0 + cq0 + 8 * k;
      int cgc = cg < cin ? cg : cin - 1;
      if constexpr (ROWQ) {
        // one float4 of the tap's input row at the quad's columns (rows outside the image
        // re-read the nearest image row, masked), and for kx = 0 / 2 the column left / right of
        // it (clamped to the quad at the image edge, masked): the window of kx is
        // (left, q.x, q.y, q.z) / q / (q.y, q.z, q.w, right)
        const int ky = tap / 3, kx = tap - 3 * ky;
        const int yi = pyi[0] + ky;
        const bool rok = pval[0] && yi >= 0 && yi < A.H;
        const int yc = yi < 0 ? 0 : (yi >= A.H ? A.H - 1 : yi);
        const uint32_t ro = (uint32_t)(poff[0] + (int64_t)cgc * HWi + yc * A.W + pxi[0]);
        const float4 qv = __builtin_bit_cast(
            float4, __builtin_amdgcn_raw_buffer_load_b128(xq_rsrc, ro * 4, 0, 0));
        const bool cok = cg < cin && rok;
        uint32_t bits = cok ? 0xfu : 0u;
        if (kx == 0) {  // uniform
          const bool eok = pxi[0] > 0;
          const float l = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                         xq_rsrc, (ro - (eok ? 1 : 0)) * 4, 0, 0));
          ra[k] = make_float4(l, qv.x, qv.y, qv.z);
          bits &= eok ? 0xfu : 0xeu;
        } else if (kx == 2) {
          const bool eok = pxi[0] + 4 < A.W;
          const float r = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                         xq_rsrc, (ro + (eok ? 4 : 3)) * 4, 0, 0));
          ra[k] = make_float4(qv.y, qv.z, qv.w, r);
          bits &= eok ? 0xfu : 0x7u;
        } else {
          ra[k] = qv;
        }
        vm |= bits << (4 * k);
      } else if constexpr (MODE == 3) {
        // K row m = c * taps + tap (dense)
        const int m = cg, mc = m < cin * taps ? m : cin * taps - 1;
        cgc = mc / taps;
        const int tp = mc - cgc * taps, ky = tp / A.kw, kx = tp - ky * A.kw;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int yi = pyi[j] + ky, xi = pxi[j] + kx;
          const bool in = m < cin * taps && pval[j] && yi >= 0 && yi < A.H && xi >= 0 && xi < A.W;
          v[j] = x[poff[j] + (in ? (int64_t)cgc * HWi + (int64_t)yi * A.W + xi : 0)];
          vm |= (in ? 1u : 0u) << (4 * k + j);
        }
        ra[k] = make_float4(v[0], v[1], v[2], v[3]);
      } else if constexpr (MODE == 2) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = x[toff[j] + (int64_t)cgc * HWi];
          vm |= ((cg < cin && pval[j] && tin[j]) ? 1u : 0u) << (4 * k + j);
        }
        ra[k] = make_float4(v[0], v[1], v[2], v[3]);
      } else if constexpr (VEC) {
        const float* src = x + poff[0] + (int64_t)cgc * HWi;
        if constexpr (XU >= 2)
          rv[k] = *reinterpret_cast<const float4*>(A.xres + poff[0] + (int64_t)cgc * HWi);
        if (XU > 0 || A.stride == 1) {  // (the unit input runs at stride 1 only)
          ra[k] = *reinterpret_cast<const float4*>(src);
        } else {
          // stride 2: each pair of the quad's outputs reads input columns 2xo, 2xo + 2 of one
          // row (both pairs in one row: columns 2xo .. 2xo + 6)
          const float4 u0 = *reinterpret_cast<const float4*>(src);
          const float4 u1 =
              *reinterpret_cast<const float4*>(x + poff[2] + (int64_t)cgc * HWi);
          ra[k] = make_float4(u0.x, u0.z, u1.x, u1.z);
        }
      } else {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = x[poff[j] + (int64_t)cgc * HWi];
        ra[k] = make_float4(v[0], v[1], v[2], v[3]);
      }
      if constexpr (MODE < 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) vm |= ((cg < cin && pval[j]) ? 1u : 0u) << (4 * k + j);
      }
      if constexpr (XF) {
        xs[k] = A.in_scale[T.xf_base + cgc];
        xt[k] = A.in_shift[T.xf_base + cgc];
      }
      if constexpr (XU == 3) {
        rs[k] = A.xres_scale[T.xf_base + cgc];
        rt[k] = A.xres_shift[T.xf_base + cgc];
      }
    }
  };
  auto store_chunk = [&](const Tile& T, int kc, int buf) {
    char* base = smem + buf * BUF;
    const int c0s = kc * KC;  // (MODE 0: the chunk's first channel; used by XU)
    (void)c0s;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int c = cq0 + 8 * k;
      float v[4] = {ra[k].x, ra[k].y, ra[k].z, ra[k].w};
      float r4[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (XU >= 2) {
        r4[0] = rv[k].x;
        r4[1] = rv[k].y;
        r4[2] = rv[k].z;
        r4[3] = rv[k].w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float u = v[j];
        if constexpr (XU > 0) {
          // dd_bn_apply's order: affine, (+ the residual after its own affine), ReLU
          u = fmaf(u, xs[k], xt[k]);
          if constexpr (XU == 3) u = u + fmaf(r4[j], rs[k], rt[k]);
          if constexpr (XU == 2) u = u + r4[j];
          u = nmax(u, 0.f);
          r4[j] = u;
        } else if constexpr (XF) {
          u = nmax(fmaf(u, xs[k], xt[k]), A.in_floor);
        }
        v[j] = ((vm >> (4 * k + j)) & 1u) ? u : 0.f;
      }
      if constexpr (XU > 0) {
        // the unit output, once: the output-block-0 tiles, whole valid quads
        if (T.o0 == 0 && (vm >> (4 * k) & 0xfu) == 0xfu)
          *reinterpret_cast<float4*>(A.xout + poff[0] + (int64_t)(c0s + c) * HWi) =
              make_float4(r4[0], r4[1], r4[2], r4[3]);
      }
      const uint32_t h01 = pack2<F16>(v[0], v[1]), h23 = pack2<F16>(v[2], v[3]);
      const uint32_t l01 = pack2<F16>(v[0] - half_lo<F16>(h01), v[1] - half_hi<F16>(h01));
      const uint32_t l23 = pack2<F16>(v[2] - half_lo<F16>(h23), v[3] - half_hi<F16>(h23));
      char* p = base + c * XS + i4 * 8;
      *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
      *reinterpret_cast<uint2*>(p + PLANE) = make_uint2(l01, l23);
    }
  };

  // ---- weights: per chunk 2 K steps x NA blocks x hi|lo fragments (16 B per lane)
  bf16x8 wa[2][NA][2];
  const int nob32 = A.op >> 5;
  // pack chunks of 16 input channels, tap-major: K chunk kc (32 channels) = pack chunks
  // 2 kc, 2 kc + 1 (each tap's channels padded to 32)
  auto load_w = [&](int ob32, int kc) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        const __bf16* p = A.wpack + ((size_t)((2 * kc + s) * nob32 + ob32 + a) * 2) * 512 +
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
  for (int n = 0; n < NT; ++n) rd[n] = (wt * TW + n * 32 + 16 * g1 + 4 * pp) * 2;

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
          d = mfma16<F16>(wa[s][a][0], bf[n][0], d);
          d = mfma16<F16>(wa[s][a][0], bf[n][1], d);
          d = mfma16<F16>(wa[s][a][1], bf[n][0], d);
          acc[a][n] = d;
        }
    }
  };

  // ---- epilogue: each 32x32 fragment transposed through a wave-private 4 KB LDS block so a
  // lane owns 4 consecutive positions of one channel (float4 operands and stores when VEC:
  // the 4 positions then share one example; one 32-bit division per fragment)
  auto epilogue = [&](const Tile& T) {
    float* ep = reinterpret_cast<float*>(smem + 2 * BUF) + wv * 1024;
    const int tl = lane & 7, ol = lane >> 3;
    // HOIST (float4 operands of the 1x1 modes): every operand load of a fragment issued before
    // any is used; the other modes keep per-element loads (their registers are spent)
    constexpr bool HOIST = VE && MODE < 2;
    constexpr bool ES = (EPI & kC1Spec) != 0;
    static_assert(!ES || HOIST, "specialised epilogues exist for the float4 1x1 modes only");
    const bool has_res = ES ? (EPI & kC1Res) != 0 : A.residual != nullptr,
               has_msk = ES ? (EPI & kC1Msk) != 0 : A.mask_src != nullptr,
               has_up2 = ES ? (EPI & kC1Up2) != 0 : A.res_up2 != nullptr,
               has_bias = ES ? (EPI & kC1Bias) != 0 : A.bias != nullptr,
               do_relu = ES ? (EPI & kC1Relu) != 0 : A.relu != 0,
               do_stats = ES ? (EPI & kC1Stats) != 0 : A.stats != nullptr;
    // BN partials per 64 positions (a pair of fragments; NT is even): half the partial
    // stores, whose issue slots the store tail of the wide outputs is bound by
    float sacc[4], qacc[4];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ep[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + (lane & 31)] =
              F16 ? acc[a][n][r] * A.acc_scale : acc[a][n][r];
        asm volatile("" ::: "memory");
        float4 vv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          vv[k] = *reinterpret_cast<const float4*>(ep + (8 * k + ol) * 32 + 4 * tl);
        asm volatile("" ::: "memory");
        const int64_t Pf = T.P0 + wt * TW + n * 32;  // the fragment's first position
        const int64_t P = Pf + 4 * tl;
        const int ob = T.o0 + (wo * NA + a) * 32 + ol;
        // per position j: example / position -> output offset at channel 0, validity
        int64_t qoff[4], qb[4];
        int qp[4];
        bool qv[4];
#pragma unroll
        for (int j = 0; j < (VE ? 1 : 4); ++j) {
          const int64_t Pj = P + j;
          qv[j] = Pj < Ptot;
          const unsigned Pc = (unsigned)(qv[j] ? Pj : Ptot - 1);
          const unsigned b = Pc / (unsigned)HWo;
          qp[j] = (int)(Pc - b * (unsigned)HWo);
          qb[j] = b;
          qoff[j] = (int64_t)b * cout * HWo + qp[j];
        }
        if (VE) {
#pragma unroll
          for (int j = 1; j < 4; ++j) {
            qv[j] = qv[0];
            qp[j] = qp[0] + j;
            qb[j] = qb[0];
            qoff[j] = qoff[0] + j;
          }
        }
        if constexpr (HOIST) {
        // operand loads of the whole fragment issued before any is used, each pointer test
        // hoisted out of the element loops (a test inside them makes hipcc branch around every
        // load and wait for it alone: one memory round trip per load)
        int oc4[4];
        int64_t co4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int o = ob + 8 * k;
          oc4[k] = o < cout ? o : cout - 1;
          co4[k] = (int64_t)oc4[k] * HWo;
        }
        // one output row group k's operands: residual, mask, upsampled residual (at even
        // (y, x) only: clamped addresses elsewhere, zeroed), each under a test outside its loads
        float rsv[4][4], msv[4][4], upv[4][4], biav[4];
        auto load_k = [&](int k) {
          if (has_res) {
            if (VE) {
              const float4 t = *reinterpret_cast<const float4*>(A.residual + qoff[0] + co4[k]);
              rsv[k][0] = t.x; rsv[k][1] = t.y; rsv[k][2] = t.z; rsv[k][3] = t.w;
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) rsv[k][j] = A.residual[qoff[j] + co4[k]];
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) rsv[k][j] = 0.f;
          }
          if (has_msk) {
            if (VE) {
              const float4 t = *reinterpret_cast<const float4*>(A.mask_src + qoff[0] + co4[k]);
              msv[k][0] = t.x; msv[k][1] = t.y; msv[k][2] = t.z; msv[k][3] = t.w;
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) msv[k][j] = A.mask_src[qoff[j] + co4[k]];
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) msv[k][j] = 1.f;
          }
          if (has_up2) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int yo = qp[j] / A.Wo, xo = qp[j] - yo * A.Wo;
              const bool even = !(yo & 1) && !(xo & 1);
              const float t = A.res_up2[(qb[j] * cout + oc4[k]) * (int64_t)(HWo / 4) +
                                        (yo >> 1) * (A.Wo >> 1) + (xo >> 1)];
              upv[k][j] = even ? t : 0.f;
            }
          }
          biav[k] = has_bias ? A.bias[oc4[k]] : 0.f;
        };
        // float4 operands: the whole fragment's loads issued before any is used (scalar
        // operands: one row group at a time, within the register budget)
        if (VE) {
#pragma unroll
          for (int k = 0; k < 4; ++k) load_k(k);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!VE) load_k(k);
          const int o = ob + 8 * k;
          const int64_t co = co4[k];
          float f[4] = {vv[k].x, vv[k].y, vv[k].z, vv[k].w};
          float s_ = 0.f, q_ = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float u = f[j] + biav[k] + rsv[k][j];
            if (has_up2) u += upv[k][j];
            if (do_relu) u = nmax(u, 0.f);
            if (!(msv[k][j] > 0.f)) u = 0.f;
            f[j] = u;
            if (do_stats) {
              const float us = (qv[j] && qb[j] < A.n_stat) ? u : 0.f;
              s_ += us;
              q_ += us * us;
            }
            if (!VE && qv[j] && o < cout) A.y[qoff[j] + co] = u;
          }
          if (VE && qv[0] && o < cout)
            store_out4(A.y + qoff[0] + co, f[0], f[1], f[2], f[3]);
          if (do_stats) {
            if ((n & 1) == 0) {
              sacc[k] = s_;
              qacc[k] = q_;
            } else {
              // the 8 lanes of one channel hold its 64 positions of this fragment pair
              const float st = sum8(sacc[k] + s_), qt = sum8(qacc[k] + q_);
              const int64_t pi = (Pf - 32 - T.grp * A.gsize * (int64_t)HWo) >> 6;
              if (tl == 0 && o < cout)
                *reinterpret_cast<float2*>(
                    A.stats + (((size_t)T.grp * cout + o) * A.tiles_per_group + pi) * 2) =
                    make_float2(st, qt);
            }
          }
        }
        } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int o = ob + 8 * k;
          const int oc = o < cout ? o : cout - 1;
          const int64_t co = (int64_t)oc * HWo;
          float f[4] = {vv[k].x, vv[k].y, vv[k].z, vv[k].w};
          const float bia = A.bias ? A.bias[oc] : 0.f;
          float rs[4] = {0.f, 0.f, 0.f, 0.f}, ms[4] = {1.f, 1.f, 1.f, 1.f};
          if (VE) {
            if (A.residual) {
              const float4 t = *reinterpret_cast<const float4*>(A.residual + qoff[0] + co);
              rs[0] = t.x; rs[1] = t.y; rs[2] = t.z; rs[3] = t.w;
            }
            if (A.mask_src) {
              const float4 t = *reinterpret_cast<const float4*>(A.mask_src + qoff[0] + co);
              ms[0] = t.x; ms[1] = t.y; ms[2] = t.z; ms[3] = t.w;
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (A.residual) rs[j] = A.residual[qoff[j] + co];
              if (A.mask_src) ms[j] = A.mask_src[qoff[j] + co];
            }
          }
          float s_ = 0.f, q_ = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float u = f[j] + bia + rs[j];
            if (A.res_up2) {
              const int yo = qp[j] / A.Wo, xo = qp[j] - yo * A.Wo;
              if (!(yo & 1) && !(xo & 1)) {
                u += A.res_up2[(qb[j] * cout + oc) * (int64_t)(HWo / 4) + (yo >> 1) * (A.Wo >> 1) +
                               (xo >> 1)];
              }
            }
            if (A.relu) u = nmax(u, 0.f);
            if (!(ms[j] > 0.f)) u = 0.f;
            f[j] = u;
            if (A.stats) {
              const float us = (qv[j] && qb[j] < A.n_stat) ? u : 0.f;
              s_ += us;
              q_ += us * us;
            }
            if (!VE && qv[j] && o < cout) A.y[qoff[j] + co] = u;
          }
          if (VE && qv[0] && o < cout)
            store_out4(A.y + qoff[0] + co, f[0], f[1], f[2], f[3]);
          if (A.stats) {
            if ((n & 1) == 0) {
              sacc[k] = s_;
              qacc[k] = q_;
            } else {
              // the 8 lanes of one channel hold its 64 positions of this fragment pair
              const float st = sum8(sacc[k] + s_), qt = sum8(qacc[k] + q_);
              const int64_t pi = (Pf - 32 - T.grp * A.gsize * (int64_t)HWo) >> 6;
              if (tl == 0 && o < cout)
                *reinterpret_cast<float2*>(
                    A.stats + (((size_t)T.grp * cout + o) * A.tiles_per_group + pi) * 2) =
                    make_float2(st, qt);
            }
          }
        }
        }
      }
  };

  // persistent: a workgroup walks tiles blockIdx.x, +gridDim.x, ...; a tile's last K chunk
  // stages the NEXT tile's first chunk (global loads issued before this tile's last MFMAs),
  // so the next tile starts computing as soon as this tile's epilogue is done
  const int nchunks = MODE == 3 ? A.nkc : A.nkc * A.kh * A.kw;  // (MODE 4: 9 taps)
  // (XCD-contiguous start: the n_ob output blocks of a position block, which stage the same
  // input, run on one XCD's L2 -- as dd_conv3x3_forward's conv_xcd)
  int tile = A.xcd ? (int)xcd_order(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  if (tile >= A.n_tiles) return;
  Tile T = decode(tile);
  pos_offsets(T);
  load_chunk(T, 0);
  load_w(T.ob32, 0);
  store_chunk(T, 0, 0);
  __syncthreads();
  int g = 0;  // chunks consumed by this workgroup: the LDS buffer parity
  for (;;) {
    const int tile_n = tile + (int)gridDim.x;
    const bool has_next = tile_n < A.n_tiles;
    const Tile Tn = has_next ? decode(tile_n) : T;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[a][n] = floatx16{0};
    for (int kc = 0; kc < nchunks; ++kc) {
      const int cur = g & 1;
      const bool last = kc + 1 == nchunks;
      if (!last) {
        load_chunk(T, kc + 1);
      } else if (has_next) {
        pos_offsets(Tn);  // this tile's staging offsets are no longer needed
        load_chunk(Tn, 0);
      }
      compute(smem + cur * BUF);
      if (!last) {
        load_w(T.ob32, kc + 1);
        store_chunk(T, kc + 1, cur ^ 1);
      } else if (has_next) {
        load_w(Tn.ob32, 0);
        store_chunk(Tn, 0, cur ^ 1);
      }
      __syncthreads();
      ++g;
    }
    epilogue(T);
    if (!has_next) break;
    tile = tile_n;
    T = Tn;
  }
}

// the pack's K is padded to 32 (two 16-channel pack chunks per K chunk).  Instantiated
// (MODE, VE, XF): 1x1 vec (0, 1, *), 1x1 scalar (1, 0, *), tap-major (2, 0|1, *), dense-K
// (3, 0|1, false: the stem reads the network input); each with bf16 and fp16 operands
#define DD_C1_LIST1(F_, NA_, WO_, H_)                                                           \
  F_(NA_, WO_, 0, true, false, H_) F_(NA_, WO_, 0, true, true, H_)                              \
  F_(NA_, WO_, 1, false, false, H_) F_(NA_, WO_, 1, false, true, H_)                            \
  F_(NA_, WO_, 2, false, false, H_) F_(NA_, WO_, 2, false, true, H_)                            \
  F_(NA_, WO_, 2, true, false, H_) F_(NA_, WO_, 2, true, true, H_)                              \
  F_(NA_, WO_, 3, false, false, H_) F_(NA_, WO_, 3, true, false, H_)                            \
  F_(NA_, WO_, 4, true, false, H_) F_(NA_, WO_, 4, true, true, H_)
#define DD_C1_LIST(F_, NA_, WO_) DD_C1_LIST1(F_, NA_, WO_, false) DD_C1_LIST1(F_, NA_, WO_, true)
// the specialised epilogues (MODE 0, float4): (XF, F16, EPI).  Both operand types: the EL2N
// statistics (with and without the producer's BN + ReLU staged; the fused unit-input kernels
// use this epilogue, and the separate pass they replace must round its sums alike).  fp16:
// the GraNd forward's conv1 (folded BN: bias + ReLU) and projection (bias); bf16: the GraNd backward (conv3^T mask, conv1^T residual +
// mask or up2 residual + mask, the projection's plain ^T).  Measured (tools/ab_conv.py --kernel
// c1x1, profiles/r05_s7/c1x1_epi/): 1.04-1.31x with statistics, up to 1.34x on the plain 64 ->
// 256 expansion, 1.0-1.14x on the backward; the GraNd conv3 epilogue (bias + residual + ReLU)
// measured 0.93-1.03x specialised and keeps the run-time flags
#define DD_C1_SPEC_LIST(F_, NA_, WO_)                                                    \
  F_(NA_, WO_, true, true, kC1Spec | kC1Stats)                                           \
  F_(NA_, WO_, false, true, kC1Spec | kC1Stats)                                          \
  F_(NA_, WO_, true, false, kC1Spec | kC1Stats)                                          \
  F_(NA_, WO_, false, false, kC1Spec | kC1Stats)                                         \
  F_(NA_, WO_, false, true, kC1Spec | kC1Bias | kC1Relu)                                 \
  F_(NA_, WO_, false, true, kC1Spec | kC1Bias)                                           \
  F_(NA_, WO_, false, false, kC1Spec | kC1Msk)                                           \
  F_(NA_, WO_, false, false, kC1Spec | kC1Res | kC1Msk)                                  \
  F_(NA_, WO_, false, false, kC1Spec | kC1Up2 | kC1Msk)                                  \
  F_(NA_, WO_, false, false, kC1Spec)

// the fused residual-unit input launches (the EL2N statistics epilogue): (F16, XU)
#define DD_C1_UNIT_LIST(F_, NA_, WO_)                                                    \
  F_(NA_, WO_, true, 1) F_(NA_, WO_, true, 2) F_(NA_, WO_, true, 3)                      \
  F_(NA_, WO_, false, 1) F_(NA_, WO_, false, 2) F_(NA_, WO_, false, 3)

// the epilogue of a launch as an EPI code (kC1Spec | operations)
inline int c1_epi_code(const Args& a) {
  return kC1Spec | (a.bias ? kC1Bias : 0) | (a.residual ? kC1Res : 0) |
         (a.mask_src ? kC1Msk : 0) | (a.res_up2 ? kC1Up2 : 0) | (a.relu ? kC1Relu : 0) |
         (a.stats ? kC1Stats : 0);
}
// DD_C1_ROWQ=0: MODE 2 for the 3x3 / stride-1 shapes MODE 4 takes (A/B; read per launch, so a
// test can compare the two modes in one process)
static bool c1_rowq() {
  const char* e = getenv("DD_C1_ROWQ");
  return !e || atoi(e) != 0;
}
// DD_C1_EPI=0: the run-time-flag epilogue everywhere (A/B)
static bool c1_epi_specialised() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DD_C1_EPI");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}

template <int NA, int WO>
static void set_attrs() {
  static bool attr = false;
  if (attr) return;
#define DD_C1_ATTR(NA_, WO_, M_, VE_, XF_, H_)                                            \
  (void)hipFuncSetAttribute(                                                              \
      reinterpret_cast<const void*>(&conv1x1_kernel<NA_, WO_, M_, VE_, XF_, H_>),         \
      hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
  DD_C1_LIST(DD_C1_ATTR, NA, WO)
#undef DD_C1_ATTR
#define DD_C1_SATTR(NA_, WO_, XF_, H_, E_)                                                \
  (void)hipFuncSetAttribute(                                                              \
      reinterpret_cast<const void*>(&conv1x1_kernel<NA_, WO_, 0, true, XF_, H_, E_>),     \
      hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
  DD_C1_SPEC_LIST(DD_C1_SATTR, NA, WO)
#undef DD_C1_SATTR
#define DD_C1_UATTR(NA_, WO_, H_, U_)                                                     \
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(                                \
                                &conv1x1_kernel<NA_, WO_, 0, true, true, H_,              \
                                                kC1Spec | kC1Stats, U_>),                 \
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
  DD_C1_UNIT_LIST(DD_C1_UATTR, NA, WO)
#undef DD_C1_UATTR
  attr = true;
}

template <int NA, int WO>
static int launch_cfg(Args a, hipStream_t st) {
  constexpr int OB = WO * NA * 32;
  set_attrs<NA, WO>();
  DD_REQUIRE(a.op % OB == 0, "dd_conv_gemm: padded outputs %d not a multiple of %d", a.op, OB);
  const int taps = a.kh * a.kw;
  const bool k1 = taps == 1 && a.pad == 0 && !a.dense;
  const bool al = (uintptr_t)a.x % 16 == 0 && (uintptr_t)a.y % 16 == 0;
  // MODE 0: quads of 4 outputs share an example (at stride 2 with Wo even, each pair of a quad
  // shares a row, and the 4 input columns a pair reads are one aligned float4: the ImageNet
  // network's 28 -> 14 projection as well as the multiple-of-4 widths; measured
  // (tools/c1_micro.py, B = 512) 512 -> 1024 at 28 / 2 1133 us in the scalar mode 1)
  const bool vec = k1 && (a.Ho * a.Wo) % 4 == 0 && (a.stride == 1 || a.Wo % 2 == 0) && al;
  const bool ve = (a.Ho * a.Wo) % 4 == 0 && (uintptr_t)a.y % 16 == 0 &&
                  (!a.residual || (uintptr_t)a.residual % 16 == 0) &&
                  (!a.mask_src || (uintptr_t)a.mask_src % 16 == 0);
  // MODE 4: 3x3 / stride 1 / pad 1 at a width that is a multiple of 4, at least 128 output
  // positions per example (a tile spans at most two examples), 16-byte aligned input.  Taken
  // at widths >= 56 only: measured (tools/gemm_micro.py, B = 512, f16 halves, BN staged) at
  // 56x56 64 -> 64 1257 -> 1203 us, at 28x28 128 -> 128 656 -> 819 us (slower)
  const bool rowq = !a.dense && a.kh == 3 && a.kw == 3 && a.stride == 1 && a.pad == 1 &&
                    a.W % 4 == 0 && a.W >= 56 && a.Ho == a.H && a.Wo == a.W &&
                    a.Ho * a.Wo >= TB &&
                    (uintptr_t)a.x % 16 == 0 && ve && 2ll * a.cin * a.H * a.W * 4 < (1ll << 31) &&
                    c1_rowq();
  const int mode = a.dense ? 3 : vec ? 0 : k1 ? 1 : rowq ? 4 : 2;
  a.n_ob = a.op / OB;
  const int64_t ntiles = ceil_div(a.B * a.Ho * a.Wo, TB) * a.n_ob;
  DD_REQUIRE(ntiles < (1ll << 31) && a.B * a.Ho * a.Wo < (1ll << 31) &&
                 a.B * a.H * a.W < (1ll << 31),
             "dd_conv_gemm: more than 2^31 positions");
  a.n_tiles = (int)ntiles;
  // resident workgroups per CU: two where the register budget allows (the 64-o and 128-o
  // tiles, except the 128-o dense-K mode, which would spill), so one's epilogue store tail
  // overlaps the other's MFMAs
  const int per_cu = (NA == 1 && (WO == 2 || mode != 3)) ? 2 : 1;
  const dim3 g((unsigned)std::min<int64_t>(ntiles, (int64_t)per_cu * device_cus()));
  const bool xf = a.in_scale != nullptr;
  DD_REQUIRE(!(xf && mode == 3), "dd_conv_gemm: no input transform with a dense-K pack");
  const bool h16 = a.f16 != 0;
  if (a.xout) {
    DD_REQUIRE(mode == 0 && ve && a.stride == 1 && xf && a.stats && !a.bias && !a.residual &&
                   !a.res_up2 && !a.mask_src && !a.relu,
               "dd_conv1x1_forward_unit_input: needs the float4 1x1 layout at stride 1 "
               "(h * w %% 4 == 0, 16-byte aligned tensors) and the statistics epilogue alone");
    const int xu = !a.xres ? 1 : !a.xres_scale ? 2 : 3;
#define DD_C1_UGO(NA_, WO_, H_, U_)                                                     \
    if (h16 == H_ && xu == U_) {                                                        \
      conv1x1_kernel<NA_, WO_, 0, true, true, H_, kC1Spec | kC1Stats, U_>               \
          <<<g, 256, LDS, st>>>(a);                                                     \
      DD_CHECK_LAUNCH("dd_conv1x1_forward_unit_input");                                 \
      return DD_OK;                                                                     \
    }
    DD_C1_UNIT_LIST(DD_C1_UGO, NA, WO)
#undef DD_C1_UGO
  }
  if (mode == 0 && ve && c1_epi_specialised()) {
    const int code = c1_epi_code(a);
#define DD_C1_SGO(NA_, WO_, XF_, H_, E_)                                             \
    if (xf == XF_ && h16 == H_ && code == (E_)) {                                    \
      conv1x1_kernel<NA_, WO_, 0, true, XF_, H_, E_><<<g, 256, LDS, st>>>(a);        \
      DD_CHECK_LAUNCH("dd_conv_gemm");                                               \
      return DD_OK;                                                                  \
    }
    DD_C1_SPEC_LIST(DD_C1_SGO, NA, WO)
#undef DD_C1_SGO
  }
#define DD_C1_GO(NA_, WO_, M_, VE_, XF_, H_)                                        \
  if (mode == M_ && (mode == 0 || mode == 1 || ve == VE_) && xf == XF_ && h16 == H_) { \
    conv1x1_kernel<NA_, WO_, M_, VE_, XF_, H_><<<g, 256, LDS, st>>>(a);             \
    DD_CHECK_LAUNCH("dd_conv_gemm");                                                \
    return DD_OK;                                                                   \
  }
  DD_C1_LIST(DD_C1_GO, NA, WO)
#undef DD_C1_GO
  DD_REQUIRE(false, "dd_conv_gemm: no kernel for mode %d", mode);
}

// family: 0 = auto, 1 = 64 o (WO 2), 2 = 128 o (WO 4, NA 1), 3 = 256 o (WO 4, NA 2)
static int launch_any(const Args& a, int fam, hipStream_t st) {
  // measured (tools/conv_micro.py --only c1x1, every ResNet-50 1x1 shape, profiles/r02_v2/
  // experiments/c1x1_family_*): the 128-o tile at two workgroups per CU is fastest or within
  // 5 % everywhere (1.3-1.7x over the one-per-CU 256-o tile at 64->256, 512->128, 2048->512:
  // the second workgroup's MFMAs cover one's epilogue store tail); the 256-o tile keeps a
  // 10 % edge only on the deep expansion (cin >= 512, cout >= 4 cin)
  // Round 6, the EL2N statistics launches (not the fused unit input) re-measured on both
  // networks' shapes (tools/c1_micro.py, B = 512, alternated, profiles/r06_c5/c1_knobs/): the
  // 256-o tile is now 0.75-0.84x the time on every stride-2 projection and 0.91-0.93x on the
  // expansions from 256 channels and on the 56x56 one, 1.08-1.2x on the 32x32 expansion from
  // 64 and the 2048 -> 512 reductions, which keep the 128-o tile
  // The GraNd forward's projections (bias epilogue, fp16) likewise, 0.66-0.73x at stride 2
  // (`--epi grandf`); its expansions (1.1-1.35x) and the backward-data GEMMs (mixed,
  // `--epi grandb`) keep the old rule.
  // The fused unit-input launches (reductions into 64-512 outputs, `--epi unit`): the 256-o
  // tile wherever the padded outputs fill it, 0.67-0.93x with the XCD order (cout >= 256)
  // The GraNd backward-data GEMMs (`--epi bwd`, config 4's launches): the projections' plain
  // W^T 0.67-0.92x, the conv3^T mask reductions at 16x16 / 8x8 0.92x (1.09x at 4x4); the
  // conv1^T residual + mask expansions keep the 128-o tile (1.08-1.1x).
  const bool k1 = a.kh * a.kw == 1;
  const bool el2n = a.stats && !a.xout && k1;
  const bool expand = a.cout >= 4 * a.cin;
  const bool plain = !a.stats && !a.bias && !a.residual && !a.res_up2 && !a.mask_src && !a.relu;
  const bool mask_red = !a.stats && !a.bias && !a.residual && !a.res_up2 && a.mask_src &&
                        !a.relu && a.cout < a.cin && a.Ho * a.Wo >= 64;
  if (fam == 0)
    fam = (a.op % 256 == 0 &&
           ((a.cin >= 512 && expand) || (k1 && a.stride == 2) || (a.xout && k1) ||
            (el2n && expand && (a.cin >= 256 || a.Ho * a.Wo >= 2048)) ||
            (k1 && a.stride == 1 && (plain || mask_red))))
              ? 3
          : a.op % 128 == 0 ? 2
                            : 1;
  if (fam == 3 && a.op % 256 == 0) return launch_cfg<2, 4>(a, st);
  if (fam >= 2 && a.op % 128 == 0) return launch_cfg<1, 4>(a, st);
  return launch_cfg<1, 2>(a, st);
}

// W [cout][cin][taps] -> [tap][16-channel chunk over cp][32-o block][hi|lo][lane][8] (the
// A-operand map of v_mfma_f32_32x32x16_bf16, one 1x1 pack per tap, channels padded to cp)
__global__ void pack_taps_kernel(const float* __restrict__ w, int cout, int cin, int taps,
                                 int op, int cp, int f16, float scale,
                                 __bf16* __restrict__ out) {
  const int nob32 = op / 32, nk16 = cp / 16;
  const int64_t total = (int64_t)taps * nk16 * nob32 * 1024;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i & 7), lane = (int)((i >> 3) & 63);
    int64_t r = i >> 9;
    const int pr = (int)(r & 1);
    r >>= 1;
    const int blk = (int)(r % nob32);
    const int64_t kk = r / nob32;
    const int tap = (int)(kk / nk16), k16 = (int)(kk - (int64_t)tap * nk16);
    const int o = blk * 32 + (lane & 31), c = k16 * 16 + 8 * (lane >> 5) + j;
    float v = 0.f;
    if (o < cout && c < cin) v = w[((size_t)o * cin + c) * taps + tap];
    v *= scale;  // a power of two (1 for bf16 packs): exact
    __bf16 hi, lo;
    if (f16)
      split16<true>(v, hi, lo);
    else
      split16<false>(v, hi, lo);
    out[i] = pr == 0 ? hi : lo;
  }
}

}  // namespace c1
}  // namespace dd

using namespace dd;

extern "C" {

int dd_conv1x1_tiles_per_group(int32_t ho, int32_t wo, int32_t group_size) {
  const int64_t hw = (int64_t)ho * wo;
  if (group_size <= 0 || hw <= 0) return -1;
  // every 128-position tile inside one BN group; one partial per 64 consecutive positions
  // of the group's flattened (example, position) space (dd_bn_finalize images_per_tile = -64)
  if ((group_size * hw) % c1::TB != 0) return -1;
  if (group_size * hw / 64 >= (1ll << 31)) return -1;
  return (int)(group_size * hw / 64);
}

}  // extern "C"

namespace {

// shared by dd_conv1x1_forward and dd_conv_gemm_forward
int gemm_forward(const char* fn, const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                 int32_t kh, int32_t kw, int32_t stride, int32_t pad, const void* packed,
                 int32_t cout, const float* bias, const float* residual, const float* res_up2,
                 const float* mask_src, int32_t relu, const float* in_scale,
                 const float* in_shift, int32_t in_relu, int32_t group_size, int64_t n_stat,
                 float* stats, float* y, int32_t operands, float acc_scale, void* stream,
                 float* xout = nullptr, const float* xres = nullptr,
                 const float* xres_scale = nullptr, const float* xres_shift = nullptr) {
  DD_REQUIRE(B >= 0 && cin > 0 && cout > 0 && h > 0 && w > 0 && kh > 0 && kw > 0 && pad >= 0,
             "%s: bad sizes", fn);
  DD_REQUIRE(operands == DD_OPERANDS_BF16X3 || operands == DD_OPERANDS_F16X3,
             "%s: operands must be DD_OPERANDS_BF16X3 or DD_OPERANDS_F16X3", fn);
  DD_REQUIRE(operand_scale_ok(operands, acc_scale),
             "%s: acc_scale must be 1 (bf16 operands) or a power of two (fp16)", fn);
  DD_REQUIRE(stride == 1 || stride == 2, "%s: stride must be 1 or 2", fn);
  const int ho = (h + 2 * pad - kh) / stride + 1, wo = (w + 2 * pad - kw) / stride + 1;
  DD_REQUIRE(h + 2 * pad >= kh && w + 2 * pad >= kw && ho > 0 && wo > 0, "%s: empty output",
             fn);
  if (B == 0) return DD_OK;
  DD_REQUIRE(x && packed && y, "%s: null buffer", fn);
  DD_REQUIRE(!in_scale == !in_shift, "%s: in_scale and in_shift go together", fn);
  DD_REQUIRE(!res_up2 || (ho % 2 == 0 && wo % 2 == 0), "%s: res_up2 needs an even output", fn);
  DD_REQUIRE((int64_t)cin * h * w < (1ll << 31) && (int64_t)cout * ho * wo < (1ll << 31),
             "%s: per-example tensor too large", fn);
  const int taps = kh * kw;
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
  a.kh = kh;
  a.kw = kw;
  a.pad = pad;
  a.dense = dd_conv_gemm_dense(cin, kh, kw);
  a.nkc = a.dense ? (int)ceil_div((int64_t)cin * taps, c1::KC) : (int)ceil_div(cin, c1::KC);
  a.relu = relu;
  const bool grouped = in_scale || stats;
  DD_REQUIRE(!grouped || group_size > 0, "%s: group_size must be positive", fn);
  a.gsize = grouped ? group_size : (int)std::min<int64_t>(B + c1::TB, 1 << 30);
  if (grouped) {
    const int tpg = dd_conv1x1_tiles_per_group(ho, wo, group_size);
    DD_REQUIRE(tpg > 0, "%s: no grouped layout for %dx%d with group_size %d", fn, ho, wo,
               group_size);
    a.tiles_per_group = tpg;
  }
  a.n_stat = stats ? std::min<int64_t>(std::max<int64_t>(n_stat, 0), B) : 0;
  a.in_scale = in_scale;
  a.in_shift = in_shift;
  a.in_floor = in_relu ? 0.f : -INFINITY;
  a.f16 = operands == DD_OPERANDS_F16X3;
  a.acc_scale = acc_scale;
  {
    // read per launch (A/B in one process).  Off by default on the GraNd launches, the
    // unit-input launches into fewer than 256 outputs (1-4 % slower with it) and the kh x kw
    // modes: measured neutral on the ResNet-50 1x1 shapes (0.98-1.02x, alternated twice) and
    // on config 4 at N = 10 240 (1926 / 1928 vs 1939 / 1927 ex/s), profiles/r06_s3/c1_xcd/.  On
    // the EL2N statistics launches (no fused unit input) on since round 6: with the 256-o tile
    // rule in launch_any, 0.89x the summed time of config 5's and 0.91x of config 4's shapes
    // (profiles/r06_c5/c1_knobs/); on the unit-input launches into 256 or more outputs too
    // (profiles/r06_c5/c1_knobs_unit/)
    const char* e = getenv("DD_C1_XCD");
    const bool plain = !stats && !bias && !residual && !res_up2 && !mask_src && !relu;
    a.xcd = e ? atoi(e)
              : (taps == 1 && ((stats && (!xout || conv::pad_to(cout, 64) % 256 == 0)) ||
                               (plain && conv::pad_to(cout, 64) % 256 == 0))
                     ? 1
                     : 0);
  }
  DD_REQUIRE(!xres || xout, "%s: a unit residual needs the unit output", fn);
  DD_REQUIRE(!xres_scale == !xres_shift && (!xres_scale || xres),
             "%s: xres_scale and xres_shift go together, with xres", fn);
  DD_REQUIRE(!xout || (in_scale && in_relu), "%s: the unit input needs its BN affine + ReLU", fn);
  a.xout = xout;
  a.xres = xres;
  a.xres_scale = xres_scale;
  a.xres_shift = xres_shift;
  // tile family: DD_C1_FAMILY=1|2|3 forces one for A/B runs (falls back to a narrower one
  // the padded outputs fit); default: the widest that fits
  static int force = -1;
  if (force < 0) {
    const char* e = getenv("DD_C1_FAMILY");
    force = e ? atoi(e) : 0;
  }
  return c1::launch_any(a, force, as_stream(stream));
}

}  // namespace

extern "C" {

int dd_conv1x1_forward(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                       int32_t stride, const void* packed, int32_t cout, const float* bias,
                       const float* residual, const float* res_up2, const float* mask_src,
                       int32_t relu, const float* in_scale, const float* in_shift,
                       int32_t in_relu, int32_t group_size, int64_t n_stat, float* stats,
                       float* y, int32_t operands, float acc_scale, void* stream) {
  clear_error();
  DD_REQUIRE(stride == 1 || stride == 2, "dd_conv1x1_forward: stride must be 1 or 2");
  DD_REQUIRE(stride == 1 || (h % 2 == 0 && w % 2 == 0),
             "dd_conv1x1_forward: stride 2 needs an even input");
  return gemm_forward("dd_conv1x1_forward", x, B, cin, h, w, 1, 1, stride, 0, packed, cout,
                      bias, residual, res_up2, mask_src, relu, in_scale, in_shift, in_relu,
                      group_size, n_stat, stats, y, operands, acc_scale, stream);
}

int dd_conv1x1_forward_unit_input(const float* y_prev, const float* scale, const float* shift,
                                  const float* xres, const float* xres_scale,
                                  const float* xres_shift, float* xout, int64_t B, int32_t cin,
                                  int32_t h, int32_t w, const void* packed, int32_t cout,
                                  int32_t group_size, int64_t n_stat, float* stats, float* y,
                                  int32_t operands, float acc_scale, void* stream) {
  clear_error();
  DD_REQUIRE(y_prev && scale && shift && xout && stats,
             "dd_conv1x1_forward_unit_input: null buffer");
  return gemm_forward("dd_conv1x1_forward_unit_input", y_prev, B, cin, h, w, 1, 1, 1, 0, packed,
                      cout, nullptr, nullptr, nullptr, nullptr, 0, scale, shift, 1, group_size,
                      n_stat, stats, y, operands, acc_scale, stream, xout, xres, xres_scale,
                      xres_shift);
}

int dd_conv_gemm_dense(int32_t cin, int32_t kh, int32_t kw) {
  // dense K (channel, tap) when a 32-channel chunk per tap would be mostly padding
  return (kh * kw > 1 && cin < c1::KC) ? 1 : 0;
}

size_t dd_conv_gemm_pack_bytes(int32_t out_channels, int32_t in_channels, int32_t kh,
                               int32_t kw) {
  if (out_channels <= 0 || in_channels <= 0 || kh <= 0 || kw <= 0) return 0;
  const int64_t taps = (int64_t)kh * kw;
  const int64_t k = dd_conv_gemm_dense(in_channels, kh, kw)
                        ? conv::pad_to((int)(in_channels * taps), c1::KC)
                        : taps * conv::pad_to(in_channels, c1::KC);
  return (size_t)conv::pad_to(out_channels, 64) * k * 2 * sizeof(__bf16);
}

int dd_conv_gemm_pack(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw,
                      int32_t operands, float scale, void* packed, void* stream) {
  clear_error();
  DD_REQUIRE(w && packed && cout > 0 && cin > 0 && kh > 0 && kw > 0,
             "dd_conv_gemm_pack: bad arguments");
  DD_REQUIRE(operands == DD_OPERANDS_BF16X3 || operands == DD_OPERANDS_F16X3,
             "dd_conv_gemm_pack: operands must be DD_OPERANDS_BF16X3 or DD_OPERANDS_F16X3");
  DD_REQUIRE(operand_scale_ok(operands, scale),
             "dd_conv_gemm_pack: scale must be 1 (bf16 operands) or a power of two (fp16)");
  // dense K: W [cout][cin * taps] is the 1x1 pack of a (cin * taps)-channel input
  if (dd_conv_gemm_dense(cin, kh, kw))
    return dd_conv1x1_pack(w, cout, cin * kh * kw, 0, operands, scale, packed, stream);
  const int op = conv::pad_to(cout, 64), cp = conv::pad_to(cin, c1::KC);
  const int64_t total = (int64_t)kh * kw * cp * op * 2;
  c1::pack_taps_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 8192), 256, 0,
                         as_stream(stream)>>>(w, cout, cin, kh * kw, op, cp,
                                              operands == DD_OPERANDS_F16X3, scale,
                                              static_cast<__bf16*>(packed));
  DD_CHECK_LAUNCH("dd_conv_gemm_pack");
  return DD_OK;
}

int dd_conv_gemm_forward(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                         int32_t kh, int32_t kw, int32_t stride, int32_t pad,
                         const void* packed, int32_t cout, const float* bias,
                         const float* residual, int32_t relu, const float* in_scale,
                         const float* in_shift, int32_t in_relu, int32_t group_size,
                         int64_t n_stat, float* stats, float* y, int32_t operands,
                         float acc_scale, void* stream) {
  clear_error();
  return gemm_forward("dd_conv_gemm_forward", x, B, cin, h, w, kh, kw, stride, pad, packed,
                      cout, bias, residual, nullptr, nullptr, relu, in_scale, in_shift, in_relu,
                      group_size, n_stat, stats, y, operands, acc_scale, stream);
}

}  // extern "C"
