// ResNet downsampling head on split-bf16 MFMA: the stride-2 3x3 conv of a stage's first block
// and, fused with it, the block's 1x1 stride-2 projection shortcut (reference
// models/resnet.py:12 conv1 at stride 2 and :20-23 shortcut), NCHW fp32 in and out.
//
//   y  = epi(conv3x3_s2_p1(x, W))        [B][cout][HO][WO]
//   ys = epi_s(conv1x1_s2(x, Ws))        [B][cout][HO][WO]   (optional)
// The 1x1 stride-2 conv reads exactly the centre tap (ky, kx) = (1, 1) of the 3x3 stride-2
// window, so both GEMMs share every staged input byte and every B fragment of that tap: the
// shortcut costs 3 more MFMAs per 27 and no extra HBM or LDS traffic.
//
// GEMM per example: D[o][t] = sum_{tap, c} W[o][c][tap] * x[c][2 yo + ky - 1][2 xo + kx - 1].
// workgroup = (E images, RB output rows = TB = 64 positions, 64 output channels); 4 waves as
// 2 (o) x 2 (t), each one 32 x 32 tile of v_mfma_f32_32x32x16_bf16 per output.  K loop over
// chunks of 16 input channels: the 2 RB + 1 input rows a tile reads are staged in LDS as
// [row][kx][hi|lo][c][xo] images already decimated by the stride (image kx holds
// x[.., 2 xo + kx - 1]), double-buffered; B fragments come from them with the transposed
// read ds_read_b64_tr_b16 exactly as in dd_conv.hip.  Epilogues as there: folded-BN bias and
// ReLU, or the grouped train-mode BN statistics (dd_bn_finalize).
#include "dd_mfma.h"

#include <stdlib.h>

namespace dd {
namespace down {

using namespace conv;

template <int WO, int RB, int E>
struct DCfg {
  static constexpr int SR = 2 * RB + 1;        // input rows staged per image
  static constexpr int NR = E * SR;
  static constexpr int WI = 2 * WO;            // input row width
  static constexpr int XS = WO * 2;            // bytes of one decimated channel row (bf16)
  static constexpr int PLANE = CC * XS;
  // padded row / image pitches: the transposed B reads of a 32-lane group step by 2 staged
  // rows (stride 2), so 2 * ROWP must land on distinct 256-byte bank offsets (dd_conv.hip)
  static constexpr int ROWP = 3 * 2 * PLANE + (WO == 16 ? 64 : WO == 8 ? 32 : WO == 4 ? 16 : 0);
  static constexpr int IMGP = SR * ROWP + (WO == 4 ? 240 : 0);
  static constexpr int BUF = E * IMGP;
  static constexpr int TB = E * RB * WO;       // output positions per workgroup
  static constexpr int TPR = WI / 8;           // threads per input channel row (8 columns each)
  static constexpr int NF8 = NR * CC * WI / 8;
  static constexpr int NST = (NF8 + 255) / 256;
  static constexpr int TPR4 = WI / 4;          // the float4 form: 4 columns per thread
  static constexpr int NF4 = NR * CC * WI / 4;
  static constexpr int NST4 = (NF4 + 255) / 256;
  // the lanes past the last staging round store into a scratch region behind the two buffers
  // instead of branching around their stores: behind such a branch the compiler sinks the
  // round's global load to its use and waits for it on the spot
  static constexpr int TAILB = (NF8 % 256 != 0 || NF4 % 256 != 0) ? 6 * PLANE + 512 : 0;
  static constexpr int LDS = 2 * BUF + TAILB;
  static_assert(TB == 64, "two 32-position t tiles per workgroup");
  static_assert(WO % 4 == 0, "transposed reads take 4 consecutive columns");
  static_assert(BUF >= 4 * 4096, "the epilogue's four 4 KB transpose blocks live in a buffer");
};

struct Out {
  float* y;
  const float* bias;
  float* stats;
  int relu;
  float scale;  // fp16 packs hold W * 2^s: the accumulator times 2^-s (exact); 1 for bf16
};

struct FwdArgs {
  const float* x;
  const __bf16* w3;  // dd_conv3x3_pack layout
  const __bf16* ws;  // dd_conv1x1_pack layout (NULL: no shortcut)
  Out main, sc;
  int64_t B, n_stat;
  int cin, HO, cout, nob32;
  int gsize, tiles_per_group, n_tb, n_ob, n_tiles;
  // XCD-contiguous tile order of the one-tile-per-workgroup grid (default; DD_DOWN_XCD=0 turns
  // it off): the n_ob output-channel tiles of a position block (consecutive tile ids) run on
  // one XCD, so the input they all stage is fetched into that XCD's L2 once instead of into
  // n_ob of them.  1.015-1.024x on the layer3 / layer4 heads' forward and backward, neutral
  // on the layer2 head (profiles/r05_s4/ab_down_xcd_summary.txt).  DD_DOWN_XCD=2 (the forward
  // default since round 6) also orders the persistent layer2-head grid (xcd_order(p) + k grid:
  // neighbouring row blocks, which share halo rows, on one L2): the bench's PMC fetch per
  // down_fwd launch 534 -> 472 MB, the head 0.95-1.0x in time (profiles/r06_s3/down_xcd/)
  int xcd;
  int wog;  // the output width in memory of a padded-width launch (PW, see down_fwd_kernel)
  // staging transform (XM, see down_fwd_kernel): x' = relu(x * in_scale[g][c] + in_shift[g][c]
  // (+ xres)), the producer's BN + ReLU (+ the unit's identity shortcut)
  const float* in_scale;
  const float* in_shift;
  const float* xres;
};

// staging modes of down_fwd_kernel (template parameter XM): none; the producer's train-mode BN
// + ReLU (a Bottleneck's stride-2 conv2); BN + the identity shortcut + ReLU (a BasicBlock unit's
// output, reference models/resnet.py:31-32, consumed by the next stage's head: nothing else
// reads it, so it is never written)
constexpr int kXmNone = 0, kXmAffine = 1, kXmUnit = 3;

// NA = output-channel blocks of 32 per wave: 1 (workgroup 64 o x 64 t, two per CU) or 2
// (128 o x 64 t, one per CU with the 512-register budget: every staged B fragment feeds
// twice the MFMAs).
// Persistent, as dd_conv.hip's conv3x3_kernel: each workgroup walks tiles blockIdx.x,
// +gridDim.x, ...; a tile's last K chunk stages the next tile's first chunk, whose weights load
// after the epilogue, so a tile's prologue (a quarter of the layer2 head's 4-chunk K loop)
// hides under the previous tile's MFMAs.
// PT = false: one tile per workgroup (the grid covers every tile; has_next folds to false)
// WA = waves along o: 2 (2 x 2 waves, each 32 NA o x 32 t) or 4 (4 x 1 waves, each 32 o x 64 t,
// NA = 1: a workgroup covers 128 outputs of the same staged chunk, so the staging and every
// weight fragment feed twice the MFMAs; B fragments are then read one tap ahead, column tile
// by column tile, to stay within the two-workgroups-per-CU register budget)
// EPI = the epilogue, fixed at compile time for the two launch shapes of the scoring passes
// (a runtime test per flag had split the epilogue into ~60 basic blocks): 1 = train-mode BN
// statistics of both outputs, no bias or ReLU (EL2N); 2 = bias + ReLU on the main output,
// bias on the shortcut, no statistics (GraNd, folded eval BN); 0 = any combination, read from
// the Out flags at run time
// F16: fp16 operand halves (DD_OPERANDS_F16X3, the EL2N launch shapes), else bf16
// PW (padded width, as conv3x3's): the EL2N statistics launch of a Bottleneck's stride-2 conv2
// at an output width that is not a tile width (the ImageNet-stem network's 56 -> 28, 28 -> 14,
// 14 -> 7 heads).  The tile keeps its WO-wide LDS images; the map in memory is WOG = A.wog
// wide (input 2 WOG), its columns and rows past the map are staged as zeros and never stored or
// counted.  PW = 1: WOG % 4 == 0 (float4 loads and stores); 2: WOG even (float4 loads, dword
// stores); 3: any WOG (dword loads and stores).
template <int WO, int RB, int E, bool SC, int NA, bool PT, int WA, int EPI = 0, int XM = 0,
          bool F16 = false, int PW = 0>
__global__ __launch_bounds__(256, NA == 1 ? 2 : 1) void down_fwd_kernel(const FwdArgs A) {
  using C = DCfg<WO, RB, E>;
  constexpr int NT = WA == 4 ? 2 : 1;  // 32-position column tiles per wave
  static_assert(WA == 2 || NA == 1, "four waves along o take one 32-o block each");
  constexpr bool S8 = WO >= 8;
  static_assert(!PW || (!SC && S8 && E == 1 && XM != kXmUnit && EPI == 0),
                "padded-width heads: the plain EL2N statistics launch");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int HO = A.HO, HI = 2 * HO, cin = A.cin, cout = A.cout;
  const int64_t B = A.B;
  const int WOG = PW ? A.wog : WO, WIG = 2 * WOG;
  const int HWI = HI * WIG, HWO = HO * WOG;
  const int ntiles = A.n_tiles;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = WA == 4 ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  const int wo = WA == 4 ? wv : wv & 1, wt = WA == 4 ? 0 : wv >> 1, h = lane >> 5;

  struct Tile {
    int64_t b, grp;
    int tb, y0, o_w, ob32;
  };
  auto decode = [&](int tile) {
    Tile T;
    int bid = tile;
    const int ob = bid % A.n_ob;
    bid /= A.n_ob;
    T.tb = bid % A.n_tb;
    T.b = (int64_t)(bid / A.n_tb) * E;
    T.y0 = T.tb * RB;
    T.grp = T.b / A.gsize;
    T.o_w = ob * 32 * WA * NA + wo * 32 * NA;  // this wave's first of NA x 32 channels
    T.ob32 = T.o_w >> 5;
    return T;
  };

  // ---- staging: 16 input channels x NR input rows, decimated into 3 kx images
  const float* __restrict__ x = A.x;
  // staging, two forms: S8 (a thread takes 8 input columns: one 8-byte LDS store per kx
  // image and plane; measured +9-11 % at 32->16) and the float4 form (4 columns, 4-byte
  // stores; faster at 8->4, where a thread's 8 columns are the whole row)
  float4 ra4[S8 ? 1 : C::NST4];
  bool va4[S8 ? 1 : C::NST4];
  // the staging transform (XM): one channel per thread in every round (256 threads cover whole
  // channel-row groups), so its affine is two scalars; the shortcut values of XM = kXmUnit
  static_assert(256 % (C::TPR4 * CC) == 0 && 256 % (C::TPR * CC) == 0,
                "a thread's staged channel must not depend on the round");
  float xs = 1.f, xt = 0.f;
  float4 rr4[(S8 || XM != kXmUnit) ? 1 : C::NST4];
  float4 rr8[(S8 && XM == kXmUnit) ? C::NST : 1][2];
  auto load_affine = [&](const Tile& T, int c0, int tpr) {
    if constexpr (XM != kXmNone) {
      const int cg = c0 + (tid / tpr) % CC;
      const int xi = (int)(T.grp * cin) + (cg < cin ? cg : cin - 1);
      xs = A.in_scale[xi];
      xt = A.in_shift[xi];
    }
  };
  // (dd_bn_apply's arithmetic, in its order)
  auto xform = [&](float4 v, float4 r) {
    if constexpr (XM == kXmNone) {
      return v;
    } else {
      v = make_float4(fmaf(v.x, xs, xt), fmaf(v.y, xs, xt), fmaf(v.z, xs, xt), fmaf(v.w, xs, xt));
      if constexpr (XM == kXmUnit) v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
      return make_float4(nmax(v.x, 0.f), nmax(v.y, 0.f), nmax(v.z, 0.f), nmax(v.w, 0.f));
    }
  };
  auto load_chunk4 = [&](const Tile& T, int c0) {
#pragma unroll
    for (int k = 0; k < C::NST4; ++k) {
      const int q = tid + 256 * k;
      const int x4 = q % C::TPR4, c = (q / C::TPR4) % CC, sr = q / (C::TPR4 * CC);
      const int e = sr / C::SR, rr = sr - e * C::SR;
      const int ir = 2 * T.y0 - 1 + rr, cg = c0 + c;
      const bool ve = T.b + e < B;
      va4[k] = q < C::NF4 && ir >= 0 && ir < HI && cg < cin && ve;
      const int irc = ir < 0 ? 0 : (ir >= HI ? HI - 1 : ir);
      const int cgc = cg < cin ? cg : cin - 1;
      const int64_t bc = ve ? T.b + e : B - 1;
      const size_t ofs = ((size_t)bc * cin + cgc) * HWI + irc * C::WI + x4 * 4;
      ra4[k] = *reinterpret_cast<const float4*>(x + ofs);
      if constexpr (!S8 && XM == kXmUnit) rr4[k] = *reinterpret_cast<const float4*>(A.xres + ofs);
    }
    load_affine(T, c0, C::TPR4);
  };
  auto store_chunk4 = [&](int buf) {
    char* base0 = smem + buf * C::BUF;
#pragma unroll
    for (int k = 0; k < C::NST4; ++k) {
      const int q = tid + 256 * k;
      const bool tail = C::NF4 % 256 != 0 && k == C::NST4 - 1 && q >= C::NF4;  // see TAILB
      const int x4 = q % C::TPR4, c = (q / C::TPR4) % CC, sr = q / (C::TPR4 * CC);
      float4 rk = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (!S8 && XM == kXmUnit) rk = rr4[k];
      const float4 v = keep_if(xform(ra4[k], rk), va4[k]);
      float left = lane_prev<C::TPR4>(v.w);  // input column 4 x4 - 1
      if (x4 == 0) left = 0.f;
      // image kx, output columns 2 x4 and 2 x4 + 1 read input columns 4 x4 + kx - 1 (+2)
      const float f[3][2] = {{left, v.y}, {v.x, v.z}, {v.y, v.w}};
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        __bf16 h0, l0, h1, l1;
        split16<F16>(f[kx][0], h0, l0);
        split16<F16>(f[kx][1], h1, l1);
        const int se = sr / C::SR, rr = sr - se * C::SR;
        char* p = tail ? smem + 2 * C::BUF + (kx * 2) * C::PLANE + lane * 4
                       : base0 + se * C::IMGP + rr * C::ROWP + (kx * 2) * C::PLANE + c * C::XS +
                             x4 * 4;
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<bf16x2*>(p) = bf16x2{h0, h1};
        *reinterpret_cast<bf16x2*>(p + C::PLANE) = bf16x2{l0, l1};
      }
    }
  };

  // a thread stages 8 consecutive input columns (two float4) of one channel row: each kx
  // image gets 4 decimated columns = one 8-byte LDS store per plane
  float4 ra[S8 ? C::NST : 1][2];
  bool va[S8 ? C::NST : 1];
  auto load_chunk8 = [&](const Tile& T, int c0) {
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {
      const int q = tid + 256 * k;
      const int x8 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const int e = sr / C::SR, rr = sr - e * C::SR;
      const int ir = 2 * T.y0 - 1 + rr, cg = c0 + c;
      const bool ve = T.b + e < B;
      va[k] = q < C::NF8 && ir >= 0 && ir < HI && cg < cin && ve && (!PW || x8 * 8 < WIG);
      const int irc = ir < 0 ? 0 : (ir >= HI ? HI - 1 : ir);
      const int cgc = cg < cin ? cg : cin - 1;
      const int64_t bc = ve ? T.b + e : B - 1;
      // (PW: columns past the row re-read its first column, masked at staging: never a read
      // past the tensor)
      const int col = PW && x8 * 8 >= WIG ? 0 : x8 * 8;
      const size_t ofs = ((size_t)bc * cin + cgc) * HWI + irc * WIG + col;
      if constexpr (PW == 3) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = x[ofs + (col + j < WIG ? j : 0)];
        ra[k][0] = make_float4(v[0], v[1], v[2], v[3]);
        ra[k][1] = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        ra[k][0] = *reinterpret_cast<const float4*>(x + ofs);
        ra[k][1] = *reinterpret_cast<const float4*>(x + ofs + (!PW || col + 4 < WIG ? 4 : 0));
      }
      if constexpr (S8 && XM == kXmUnit) {
        rr8[k][0] = *reinterpret_cast<const float4*>(A.xres + ofs);
        rr8[k][1] = *reinterpret_cast<const float4*>(A.xres + ofs + 4);
      }
    }
    load_affine(T, c0, C::TPR);
  };
  auto store_chunk8 = [&](int buf) {
    char* base0 = smem + buf * C::BUF;
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {
      const int q = tid + 256 * k;
      const bool tail = C::NF8 % 256 != 0 && k == C::NST - 1 && q >= C::NF8;  // see TAILB
      const int x8 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0;
      if constexpr (S8 && XM == kXmUnit) {
        r0 = rr8[k][0];
        r1 = rr8[k][1];
      }
      float4 v0 = keep_if(xform(ra[k][0], r0), va[k]), v1 = keep_if(xform(ra[k][1], r1), va[k]);
      if constexpr (PW != 0) {
        v0 = keep_cols(v0, WIG - x8 * 8);
        v1 = keep_cols(v1, WIG - x8 * 8 - 4);
      }
      float left = C::TPR > 1 ? lane_prev<C::TPR>(v1.w) : 0.f;  // input column 8 x8 - 1
      if (x8 == 0) left = 0.f;
      // value i = input column 8 x8 + i - 1; image kx, decimated column 4 x8 + m reads input
      // column 8 x8 + 2 m + kx - 1 = value 2 m + kx
      const float f[9] = {left, v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      __bf16 hv[9], lv[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) split16<F16>(f[i], hv[i], lv[i]);
      const int se = sr / C::SR, rr = sr - se * C::SR;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        char* p = tail ? smem + 2 * C::BUF + (kx * 2) * C::PLANE + lane * 8
                       : base0 + se * C::IMGP + rr * C::ROWP + (kx * 2) * C::PLANE + c * C::XS +
                             x8 * 8;
        *reinterpret_cast<bf16x4*>(p) = bf16x4{hv[kx], hv[kx + 2], hv[kx + 4], hv[kx + 6]};
        *reinterpret_cast<bf16x4*>(p + C::PLANE) = bf16x4{lv[kx], lv[kx + 2], lv[kx + 4], lv[kx + 6]};
      }
    }
  };

  auto load_chunk = [&](const Tile& T, int c0) {
    if constexpr (S8) load_chunk8(T, c0); else load_chunk4(T, c0);
  };
  auto store_chunk = [&](int buf) {
    if constexpr (S8) store_chunk8(buf); else store_chunk4(buf);
  };

  // ---- weights: 9 taps (hi|lo) of the 3x3 pack, 1 tap of the 1x1 pack, 16 B per lane
  bf16x8 wa[NA][18], wsc[NA][2];
  const __bf16* __restrict__ w3 = A.w3;
  const __bf16* __restrict__ wsp = A.ws;
  auto load_w_taps = [&](int ob32, int kc, int tap0, int ntap) {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      // blocks past the padded outputs (cout % (64 NA) != 0) re-read the last one; their
      // outputs are never stored
      const int blk = min(ob32 + a, A.nob32 - 1);
      const __bf16* base = w3 + ((size_t)(kc * A.nob32 + blk) * 18) * 512 + lane * 8;
      // constant trip count (the tap range folds at every call site), so wa stays in VGPRs
#pragma unroll
      for (int i = 0; i < 18; ++i)
        if (i >= 2 * tap0 && i < 2 * (tap0 + ntap))
          wa[a][i] = *reinterpret_cast<const bf16x8*>(base + i * 512);
    }
  };
  auto load_w_sc = [&](int ob32, int kc) {
    if constexpr (SC) {
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        const int blk = min(ob32 + a, A.nob32 - 1);
        const __bf16* base = wsp + ((size_t)(kc * A.nob32 + blk) * 2) * 512 + lane * 8;
        wsc[a][0] = *reinterpret_cast<const bf16x8*>(base);
        wsc[a][1] = *reinterpret_cast<const bf16x8*>(base + 512);
      }
    }
  };
  // all 9 taps (+ the shortcut) of chunk kc in tap order, each tap fenced: the waitcnt pass
  // merges the paths into the chunk loop, and with the scheduler free to issue tap 0 late on
  // one of them, every chunk's first MFMA waited for the back edge's newest weight loads
  auto load_w_ordered = [&](int ob32, int kc) {
    static_for<9>([&](auto Tc) {
      load_w_taps(ob32, kc, decltype(Tc)::value, 1);
      if constexpr (decltype(Tc)::value == 4) load_w_sc(ob32, kc);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // transposed-read geometry of this lane's 4 columns in each of the wave's NT column tiles
  const int q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
  int tr_off[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int t = (wt + n) * 32 + 16 * g1 + 4 * p;
    const int e = t / (RB * WO);
    tr_off[n] = e * C::IMGP + 2 * ((t / WO) % RB) * C::ROWP + (8 * h + q) * C::XS + (t % WO) * 2;
  }

  floatx16 acc[NA][NT], acc_s[NA][NT];
  auto read_b = [&](const char* base, int ky, bf16x8 (&bf)[3][2]) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const char* a = base + tr_off[0] + ky * C::ROWP + (kx * 2) * C::PLANE;
      bf[kx][0] = tr_read8(a, a + 4 * C::XS);
      bf[kx][1] = tr_read8(a + C::PLANE, a + C::PLANE + 4 * C::XS);
    }
  };
  auto mfma_row = [&](int ky, const bf16x8 (&bf)[3][2]) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        const int tap = ky * 3 + kx;
        floatx16 d = acc[a][0];
        d = mfma16<F16>(wa[a][tap * 2], bf[kx][0], d);
        d = mfma16<F16>(wa[a][tap * 2], bf[kx][1], d);
        d = mfma16<F16>(wa[a][tap * 2 + 1], bf[kx][0], d);
        acc[a][0] = d;
        if constexpr (SC) {
          if (ky == 1 && kx == 1) {
            floatx16 s = acc_s[a][0];
            s = mfma16<F16>(wsc[a][0], bf[1][0], s);
            s = mfma16<F16>(wsc[a][0], bf[1][1], s);
            s = mfma16<F16>(wsc[a][1], bf[1][0], s);
            acc_s[a][0] = s;
          }
        }
      }
  };

  // ---- epilogues: each 32 x 32 fragment (column t = lane & 31 of this wave's 32 positions,
  // row o = (r&3) + 8(r>>2) + 4h) is transposed through a wave-private 4 KB LDS block in the
  // staging buffer the tile's last chunk consumed, so a lane then owns 4 consecutive positions
  // (one output row, one image) of 4 channels: float4 stores, a quarter of the store
  // instructions.  BN partials: one per (channel, 32-position fragment), summed over the 8
  // lanes of a channel by DPP (the stats layout of dd_conv3x3_forward: 2 partials per tile).
  auto epilogue = [&](const Tile& T, const floatx16& a, const Out& out, const int o_w,
                      char* ep_buf, const int tc, auto MAINc) {
    constexpr bool MAIN = decltype(MAINc)::value;
    const bool has_bias = EPI == 0 ? out.bias != nullptr : EPI == 2;
    const bool relu = EPI == 0 ? out.relu != 0 : (EPI == 2 && MAIN);
    const bool has_stats = EPI == 0 ? out.stats != nullptr : EPI == 1;
    float* ep = reinterpret_cast<float*>(ep_buf) + wv * 1024;
    const int tl = lane & 7, ol = lane >> 3;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      ep[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + (lane & 31)] = F16 ? a[r] * out.scale : a[r];
    asm volatile("" ::: "memory");
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      v[k] = *reinterpret_cast<const float4*>(ep + (8 * k + ol) * 32 + 4 * tl);
    asm volatile("" ::: "memory");
    const int tt = tc * 32 + 4 * tl;  // this lane's first position in the tile
    const int e = tt / (RB * WO);
    int t = T.y0 * WO + tt % (RB * WO);
    bool in_map = true;
    int ncol = 4;  // PW >= 2: columns of the lane's quad inside the map
    if constexpr (PW != 0) {
      const int rem = tt % (RB * WO), row = T.y0 + rem / WO, col = rem % WO;
      in_map = row < HO && col < WOG;
      ncol = WOG - col;
      t = in_map ? row * WOG + col : 0;
    }
    const bool ve = T.b + e < B && in_map;
    const float in_stat = (T.b + e < A.n_stat && in_map) ? 1.f : 0.f;
    const int64_t be = T.b + e < B ? T.b + e : B - 1;
    const int frag = ((int)((T.b - T.grp * A.gsize) / E) * A.n_tb + T.tb) * 2 + tc;
    // BN partials of channels o_w + ol + 8 k: one base, a constant stride
    float* const sp = has_stats ? out.stats + (((size_t)T.grp * cout + o_w + ol) *
                                               A.tiles_per_group + frag) * 2 : nullptr;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int o = o_w + 8 * k + ol;
      const float bia = has_bias ? out.bias[o < cout ? o : cout - 1] : 0.f;
      float f[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
      float s_ = 0.f, q_ = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float u = f[j] + bia;
        if (relu) u = nmax(u, 0.f);
        f[j] = u;
        const float us = (PW >= 2 && j >= ncol) ? 0.f : u * in_stat;
        s_ += us;
        q_ += us * us;
      }
      if constexpr (PW >= 2) {
        if (ve && o < cout) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < ncol) out.y[((size_t)be * cout + o) * HWO + t + j] = f[j];
        }
      } else if (ve && o < cout) {
        store_out4(out.y + ((size_t)be * cout + o) * HWO + t, f[0], f[1], f[2], f[3]);
      }
      if (has_stats) {
        s_ = sum8(s_);
        q_ = sum8(q_);
        if (tl == 0 && o < cout)
          *reinterpret_cast<float2*>(sp + k * 16 * A.tiles_per_group) = make_float2(s_, q_);
      }
    }
    asm volatile("" ::: "memory");  // the next fragment reuses the block (in order per wave)
  };

  const int nchunks = (cin + CC - 1) / CC;
  // (the persistent grid walks xcd_order(p) + k grid, as conv3x3's, with DD_DOWN_XCD=2)
  int tile = A.xcd >= (PT ? 2 : 1) ? (int)xcd_order(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  Tile T = decode(tile);
  load_chunk(T, 0);
  __builtin_amdgcn_sched_barrier(0);
  load_w_ordered(T.ob32, 0);
  store_chunk(0);
  __syncthreads();
  int g = 0;  // chunks processed by this workgroup: LDS buffer parity
  for (;;) {
    const int tile_n = tile + (int)gridDim.x;
    const bool has_next = PT && tile_n < ntiles;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[a][n] = acc_s[a][n] = floatx16{0};
    // one K chunk; wload = false on a tile's last chunk, whose prefetch target is the next
    // tile's first chunk (its weights load after the epilogue)
    // WA = 4: tap by tap; after a tap's MFMAs the next tap's B fragments of that column tile
    // are read and (wload) the next chunk's weights of that tap are loaded into its registers
    auto chunk4 = [&](const Tile& Tp, int kn, bool wload) {
      const int cur = g & 1;
      load_chunk(Tp, kn * CC);
      // fences keep every global load where it is written (the scheduler otherwise sinks the
      // staging and weight loads next to their uses, and the next chunk's first MFMA waits for
      // the weights loaded just before the barrier)
      __builtin_amdgcn_sched_barrier(0);
      const char* base = smem + cur * C::BUF;
      bf16x8 bb[NT][2];
      auto rb = [&](int tap, int n) {
        const char* a = base + tr_off[n] + (tap / 3) * C::ROWP + ((tap % 3) * 2) * C::PLANE;
        bb[n][0] = tr_read8(a, a + 4 * C::XS);
        bb[n][1] = tr_read8(a + C::PLANE, a + C::PLANE + 4 * C::XS);
      };
#pragma unroll
      for (int n = 0; n < NT; ++n) rb(0, n);
      static_for<9>([&](auto Tc) {
        constexpr int t = decltype(Tc)::value;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          floatx16 d = acc[0][n];
          d = mfma16<F16>(wa[0][t * 2], bb[n][0], d);
          d = mfma16<F16>(wa[0][t * 2], bb[n][1], d);
          d = mfma16<F16>(wa[0][t * 2 + 1], bb[n][0], d);
          acc[0][n] = d;
          if constexpr (SC && t == 4) {
            floatx16 s_ = acc_s[0][n];
            s_ = mfma16<F16>(wsc[0][0], bb[n][0], s_);
            s_ = mfma16<F16>(wsc[0][0], bb[n][1], s_);
            s_ = mfma16<F16>(wsc[0][1], bb[n][0], s_);
            acc_s[0][n] = s_;
          }
          if constexpr (t + 1 < 9) rb(t + 1, n);
        }
        if (wload) {
          load_w_taps(Tp.ob32, kn, t, 1);
          if constexpr (t == 4) load_w_sc(Tp.ob32, kn);
        }
        if constexpr (t == 6) store_chunk(cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      });
      __syncthreads();
      ++g;
    };
    auto chunk = [&](const Tile& Tp, int kn, bool wload) {
      if constexpr (WA == 4) {
        chunk4(Tp, kn, wload);
        return;
      }
      const int cur = g & 1;
      load_chunk(Tp, kn * CC);
      const char* base = smem + cur * C::BUF;
      bf16x8 b0[3][2], b1[3][2];
      read_b(base, 0, b0);
      __builtin_amdgcn_sched_barrier(0);
      read_b(base, 1, b1);
      mfma_row(0, b0);
      if (wload) load_w_taps(Tp.ob32, kn, 0, 3);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if constexpr (NA == 2) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      read_b(base, 2, b0);
      mfma_row(1, b1);
      if (wload) {
        load_w_taps(Tp.ob32, kn, 3, 3);
        load_w_sc(Tp.ob32, kn);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 1);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        if constexpr (NA == 2) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x020, 2, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_row(2, b0);
      store_chunk(cur ^ 1);
      if (wload) load_w_taps(Tp.ob32, kn, 6, 3);
#pragma unroll
      for (int i = 0; i < 9 * NA; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
        __builtin_amdgcn_sched_group_barrier(0x002, NA == 1 ? 5 : 3, 2);
        __builtin_amdgcn_sched_group_barrier(0x080, 1, 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      ++g;
    };
    for (int kc = 0; kc + 1 < nchunks; ++kc) chunk(T, kc + 1, true);
    // last chunk: stage the next tile's first chunk (or, on the last tile, a clamped re-load
    // into the idle buffer that is never read)
    {
      const Tile Tn = has_next ? decode(tile_n) : T;
      chunk(Tn, has_next ? 0 : nchunks - 1, false);
    }
    // the last chunk read buffer (g - 1) & 1; the next tile's first chunk sits in g & 1
    char* ep_buf = smem + ((g - 1) & 1) * C::BUF;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        epilogue(T, acc[a][n], A.main, T.o_w + 32 * a, ep_buf, wt + n, std::true_type{});
        if constexpr (SC)
          epilogue(T, acc_s[a][n], A.sc, T.o_w + 32 * a, ep_buf, wt + n, std::false_type{});
      }
    if constexpr (!PT) break;  // one tile per workgroup: nothing follows
    __syncthreads();  // the next tile's first staging store overwrites the transpose blocks
    // the next tile's weights (re-loading this tile's on the last one) BEFORE the exit test: the
    // CFG structurizer routes a `break` through the loop latch, and a path reaching it without
    // these loads made the waitcnt pass treat the back edge's weight loads as the newest
    const int tile_w = has_next ? tile_n : tile;
    T = decode(tile_w);  // re-derived rather than held across the epilogue (register pressure)
    load_w_ordered(T.ob32, 0);
    if (!has_next) break;
    tile = tile_n;
  }
}

// ------------------------------------------------------------------------------------------
// Backward-data of the downsampling head (the GraNd backward, grand_fast.py):
//   dx = (conv3x3_s2^T(dh, W) + conv1x1_s2^T(dz, Ws)) * (mask > 0)      [B][cin][2HO][2WO]
// The transposed stride-2 conv splits into 4 sub-pixel classes (py, px) of dx positions
// (2i + py, 2j + px), each a stride-1 GEMM over dh with its own taps: ky = 1 feeds py = 0 at
// row offset 0; ky = 0 / 2 feed py = 1 at row offsets +1 / 0 (likewise kx, px).  All 9 taps
// are used once and no zero is ever multiplied (a zero-inserted upsampling would waste 3/4 of
// the MFMAs).  The 1x1 shortcut adds Ws^T dz to class (0, 0) only.
// workgroup = (E images, RB rows of (i, j), 64 input channels c); 4 waves as 2 (c) x 2 (t),
// each with 4 class accumulators of v_mfma_f32_32x32x16_bf16.  K loop over chunks of 16
// output channels o: dh rows i0 .. i0+RB are staged in LDS as [row][shift 0|1][hi|lo][o][j]
// (shift 1 holds dh[.., j + 1]), dz rows as [row][hi|lo][o][j].  The epilogue writes the px = 0
// and px = 1 classes of a position as one float2 (dx columns 2j, 2j + 1).
// ------------------------------------------------------------------------------------------
template <int WO, int RB, int E, bool SC>
struct UCfg {
  static constexpr int NRH = E * (RB + 1);
  static constexpr int NRZ = E * RB;
  static constexpr int XS = WO * 2;
  static constexpr int PLANE = CC * XS;
  // padded pitches (see DCfg): the reads of a 32-lane group step by one staged row
  static constexpr int PADR = WO == 16 ? 128 : WO == 8 ? 64 : WO == 4 ? 32 : 0;
  static constexpr int ROWP = 2 * 2 * PLANE + PADR;
  static constexpr int IMGP = (RB + 1) * ROWP + (WO == 4 ? 224 : 0);
  static constexpr int ROWPZ = 2 * PLANE + PADR;
  static constexpr int IMGPZ = RB * ROWPZ;
  static constexpr int HBUF = E * IMGP;
  static constexpr int ZBUF = SC ? E * IMGPZ : 0;
  static constexpr int BUF = HBUF + ZBUF;
  static constexpr int TB = E * RB * WO;
  static constexpr int TPR = WO / 4;
  static constexpr int NF4H = NRH * CC * WO / 4;
  static constexpr int NF4Z = NRZ * CC * WO / 4;
  static constexpr int NSTH = (NF4H + 255) / 256;
  static constexpr int NSTZ = (NF4Z + 255) / 256;
  // scratch region for the lanes past the last staging round (see DCfg::TAILB)
  static constexpr int TAILB = (NF4H % 256 != 0 || NF4Z % 256 != 0) ? 4 * PLANE + 512 : 0;
  static constexpr int LDS = 2 * BUF + TAILB;
};

struct BwdArgs {
  const float* dh;
  const float* dz;
  const __bf16* w3t;  // dd_conv3x3_pack(W, transpose_flip = 1)
  const __bf16* w1t;  // dd_conv1x1_pack(Ws, transpose = 1)
  const float* mask;
  // or the mask as plane bits: bit p & 31 of word ((b * cin + c) * 4 HO WO + p) >> 5 =
  // (mask[b][c][p] > 0) (dd_conv3x3_mask_plane_bits of the producer's fragment masks)
  const uint32_t* mask_bits;
  float* dx;
  int64_t B;
  int cin, cout, HO, nob32;
  int n_tb, n_ob;
  int xcd;  // XCD-contiguous tile order (DD_DOWN_XCD=1, as FwdArgs::xcd)
};

template <int WO, int RB, int E, bool SC>
__global__ __launch_bounds__(256, 2) void down_bwd_kernel(const BwdArgs A) {
  using C = UCfg<WO, RB, E, SC>;
  static_assert(C::TB == 64, "two 32-position t tiles per workgroup");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int HO = A.HO, HI = 2 * HO, WI = 2 * WO, cin = A.cin, cout = A.cout;
  const int64_t B = A.B;
  const int HWO = HO * WO;
  int bid = blockIdx.x;
  const int ob = bid % A.n_ob;
  bid /= A.n_ob;
  const int tb = bid % A.n_tb;
  const int64_t b = (int64_t)(bid / A.n_tb) * E;
  const int i0 = tb * RB;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wc = wv & 1, wt = wv >> 1, h = lane >> 5;
  const int c_w = ob * 64 + wc * 32;  // this wave's 32 dx channels
  const int ob32 = min(c_w >> 5, A.nob32 - 1);

  float4 rh[C::NSTH], rz[C::NSTZ];
  bool vh[C::NSTH], vz[C::NSTZ];
  auto load_chunk = [&](int o0) {
#pragma unroll
    for (int k = 0; k < C::NSTH; ++k) {
      const int q = tid + 256 * k;
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const int e = sr / (RB + 1), rr = sr - e * (RB + 1);
      const int ir = i0 + rr, og = o0 + c;
      const bool ve = b + e < B;
      vh[k] = q < C::NF4H && ir < HO && og < cout && ve;
      const int irc = ir < HO ? ir : HO - 1;
      const int ogc = og < cout ? og : cout - 1;
      const int64_t bc = ve ? b + e : B - 1;
      rh[k] = *reinterpret_cast<const float4*>(A.dh + ((size_t)bc * cout + ogc) * HWO +
                                               irc * WO + x4 * 4);
    }
    if constexpr (SC) {
#pragma unroll
      for (int k = 0; k < C::NSTZ; ++k) {
        const int q = tid + 256 * k;
        const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
        const int e = sr / RB, rr = sr - e * RB;
        const int og = o0 + c;
        const bool ve = b + e < B;
        vz[k] = q < C::NF4Z && og < cout && ve;
        const int ogc = og < cout ? og : cout - 1;
        const int64_t bc = ve ? b + e : B - 1;
        rz[k] = *reinterpret_cast<const float4*>(A.dz + ((size_t)bc * cout + ogc) * HWO +
                                                 (i0 + rr) * WO + x4 * 4);
      }
    }
  };
  auto store4 = [&](char* pl, const float* f) {  // hi plane at pl, lo plane at pl + PLANE
    __bf16 hi[4], lo[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) split_bf16(f[i], hi[i], lo[i]);
    *reinterpret_cast<bf16x4*>(pl) = bf16x4{hi[0], hi[1], hi[2], hi[3]};
    *reinterpret_cast<bf16x4*>(pl + C::PLANE) = bf16x4{lo[0], lo[1], lo[2], lo[3]};
  };
  auto store_chunk = [&](int buf) {
    char* base0 = smem + buf * C::BUF;
#pragma unroll
    for (int k = 0; k < C::NSTH; ++k) {
      const int q = tid + 256 * k;
      const bool tail = C::NF4H % 256 != 0 && k == C::NSTH - 1 && q >= C::NF4H;  // TAILB
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const float4 v = keep_if(rh[k], vh[k]);
      float right = lane_next<C::TPR>(v.x);  // dh column 4 x4 + 4
      if (x4 == C::TPR - 1) right = 0.f;
      const float f0[4] = {v.x, v.y, v.z, v.w};
      const float f1[4] = {v.y, v.z, v.w, right};
      const int se = sr / (RB + 1), rr = sr - se * (RB + 1);
      char* p = tail ? smem + 2 * C::BUF + lane * 8
                     : base0 + se * C::IMGP + rr * C::ROWP + c * C::XS + x4 * 8;
      store4(p, f0);
      store4(p + 2 * C::PLANE, f1);
    }
    if constexpr (SC) {
#pragma unroll
      for (int k = 0; k < C::NSTZ; ++k) {
        const int q = tid + 256 * k;
        const bool tail = C::NF4Z % 256 != 0 && k == C::NSTZ - 1 && q >= C::NF4Z;  // TAILB
        const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
        const float4 v = keep_if(rz[k], vz[k]);
        const float f0[4] = {v.x, v.y, v.z, v.w};
        const int se = sr / RB, rr = sr - se * RB;
        store4(tail ? smem + 2 * C::BUF + lane * 8
                    : base0 + C::HBUF + se * C::IMGPZ + rr * C::ROWPZ + c * C::XS + x4 * 8,
               f0);
      }
    }
  };

  bf16x8 wa[18], wsc[2];
  auto load_w = [&](int kc) {
    const __bf16* base = A.w3t + ((size_t)(kc * A.nob32 + ob32) * 18) * 512 + lane * 8;
#pragma unroll
    for (int f = 0; f < 18; ++f) wa[f] = *reinterpret_cast<const bf16x8*>(base + f * 512);
    if constexpr (SC) {
      const __bf16* bs = A.w1t + ((size_t)(kc * A.nob32 + ob32) * 2) * 512 + lane * 8;
      wsc[0] = *reinterpret_cast<const bf16x8*>(bs);
      wsc[1] = *reinterpret_cast<const bf16x8*>(bs + 512);
    }
  };

  const int q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
  int tr_h, tr_z, tr_j;
  {
    const int t = wt * 32 + 16 * g1 + 4 * p;
    const int e = t / (RB * WO), il = (t / WO) % RB;
    tr_h = e * C::IMGP + il * C::ROWP;
    tr_z = e * C::IMGPZ + il * C::ROWPZ;
    tr_j = t % WO;
  }

  floatx16 acc[4];  // class py * 2 + px
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = floatx16{0};

  const int nchunks = (cout + CC - 1) / CC;
  load_chunk(0);
  load_w(0);
  store_chunk(0);
  __syncthreads();
  for (int kc = 0; kc < nchunks; ++kc) {
    const int cur = kc & 1;
    const int kn = kc + 1 < nchunks ? kc + 1 : kc;
    load_chunk(kn * CC);
    const char* base = smem + cur * C::BUF;
    bf16x8 bh[2][2][2], bz[2];  // [row offset][column shift][hi|lo]
#pragma unroll
    for (int oy = 0; oy < 2; ++oy)
#pragma unroll
      for (int ox = 0; ox < 2; ++ox) {
        const char* a = base + tr_h + oy * C::ROWP + (ox * 2) * C::PLANE + (8 * h + q) * C::XS +
                        tr_j * 2;
        bh[oy][ox][0] = tr_read8(a, a + 4 * C::XS);
        bh[oy][ox][1] = tr_read8(a + C::PLANE, a + C::PLANE + 4 * C::XS);
      }
    if constexpr (SC) {
      const char* a = base + C::HBUF + tr_z + (8 * h + q) * C::XS + tr_j * 2;
      bz[0] = tr_read8(a, a + 4 * C::XS);
      bz[1] = tr_read8(a + C::PLANE, a + C::PLANE + 4 * C::XS);
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int oy = ky == 0, ox = kx == 0;
        const int cls = (ky != 1) * 2 + (kx != 1);
        const int f = (8 - (ky * 3 + kx)) * 2;  // the pack is spatially flipped
        floatx16 d = acc[cls];
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[f], bh[oy][ox][0], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[f], bh[oy][ox][1], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[f + 1], bh[oy][ox][0], d, 0, 0, 0);
        acc[cls] = d;
      }
    if constexpr (SC) {
      floatx16 d = acc[0];
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wsc[0], bz[0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wsc[0], bz[1], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wsc[1], bz[0], d, 0, 0, 0);
      acc[0] = d;
    }
    load_w(kn);
    store_chunk(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane column t -> position (i, j); classes px = 0 / 1 -> one float2
  const int tt = wt * 32 + (lane & 31);
  const int e = tt / (RB * WO), rem = tt % (RB * WO);
  const int i = i0 + rem / WO, j = rem % WO;
  const bool ve = b + e < B;
  const int64_t be = ve ? b + e : B - 1;
#pragma unroll
  for (int py = 0; py < 2; ++py) {
    float2 mk[16];
    if (A.mask) {  // hoisted pointer test: the 16 loads issue back to back
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = c_w + (r & 3) + 8 * (r >> 2) + 4 * h;
        const size_t off = (((size_t)be * cin + (c < cin ? c : cin - 1)) * HI + 2 * i + py) *
                               WI + 2 * j;
        mk[r] = *reinterpret_cast<const float2*>(A.mask + off);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) mk[r] = make_float2(1.f, 1.f);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = c_w + (r & 3) + 8 * (r >> 2) + 4 * h;
      const size_t off = (((size_t)be * cin + (c < cin ? c : cin - 1)) * HI + 2 * i + py) * WI +
                         2 * j;
      float2 v = make_float2(acc[py * 2][r], acc[py * 2 + 1][r]);
      if (!(mk[r].x > 0.f)) v.x = 0.f;
      if (!(mk[r].y > 0.f)) v.y = 0.f;
      if (ve && c < cin) *reinterpret_cast<float2*>(A.dx + off) = v;
    }
  }
}

// The same backward with 128-position workgroups ("bwd2"): 2 (c) x 2 (t) waves, each 32 c x
// 64 t = two column tiles x 4 classes (8 accumulators), so each weight fragment loaded from L2
// feeds twice the MFMAs.  To fit two workgroups per CU, weights rotate through a few register
// slots instead of holding a chunk's 9 taps, and B fragments are read one step ahead per column
// tile (the shortcut's dz fragments as a tenth step).
template <int WO, int RB, int E, bool SC>
__global__ __launch_bounds__(256, 2) void down_bwd2_kernel(const BwdArgs A) {
  using C = UCfg<WO, RB, E, SC>;
  constexpr int NT = 2;
  static_assert(C::TB == 128, "two 64-position wave halves per workgroup");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int HO = A.HO, HI = 2 * HO, WI = 2 * WO, cin = A.cin, cout = A.cout;
  const int64_t B = A.B;
  const int HWO = HO * WO;
  int bid = A.xcd ? (int)xcd_order(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int ob = bid % A.n_ob;
  bid /= A.n_ob;
  const int tb = bid % A.n_tb;
  const int64_t b = (int64_t)(bid / A.n_tb) * E;
  const int i0 = tb * RB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wv & 1, wt = wv >> 1, h = lane >> 5;
  const int c_w = ob * 64 + wc * 32;  // this wave's 32 dx channels
  const int ob32 = min(c_w >> 5, A.nob32 - 1);

  float4 rh[C::NSTH], rz[C::NSTZ];
  bool vh[C::NSTH], vz[C::NSTZ];
  auto load_chunk = [&](int o0) {
#pragma unroll
    for (int k = 0; k < C::NSTH; ++k) {
      const int q = tid + 256 * k;
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const int e = sr / (RB + 1), rr = sr - e * (RB + 1);
      const int ir = i0 + rr, og = o0 + c;
      const bool ve = b + e < B;
      vh[k] = q < C::NF4H && ir < HO && og < cout && ve;
      const int irc = ir < HO ? ir : HO - 1;
      const int ogc = og < cout ? og : cout - 1;
      const int64_t bc = ve ? b + e : B - 1;
      rh[k] = *reinterpret_cast<const float4*>(A.dh + ((size_t)bc * cout + ogc) * HWO +
                                               irc * WO + x4 * 4);
    }
    if constexpr (SC) {
#pragma unroll
      for (int k = 0; k < C::NSTZ; ++k) {
        const int q = tid + 256 * k;
        const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
        const int e = sr / RB, rr = sr - e * RB;
        const int og = o0 + c;
        const bool ve = b + e < B;
        vz[k] = q < C::NF4Z && og < cout && ve;
        const int ogc = og < cout ? og : cout - 1;
        const int64_t bc = ve ? b + e : B - 1;
        rz[k] = *reinterpret_cast<const float4*>(A.dz + ((size_t)bc * cout + ogc) * HWO +
                                                 (i0 + rr) * WO + x4 * 4);
      }
    }
  };
  auto store4 = [&](char* pl, const float* f) {
    __bf16 hi[4], lo[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) split_bf16(f[i], hi[i], lo[i]);
    *reinterpret_cast<bf16x4*>(pl) = bf16x4{hi[0], hi[1], hi[2], hi[3]};
    *reinterpret_cast<bf16x4*>(pl + C::PLANE) = bf16x4{lo[0], lo[1], lo[2], lo[3]};
  };
  auto store_chunk = [&](int buf) {
    char* base0 = smem + buf * C::BUF;
#pragma unroll
    for (int k = 0; k < C::NSTH; ++k) {
      const int q = tid + 256 * k;
      const bool tail = C::NF4H % 256 != 0 && k == C::NSTH - 1 && q >= C::NF4H;  // TAILB
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const float4 v = keep_if(rh[k], vh[k]);
      float right = lane_next<C::TPR>(v.x);  // dh column 4 x4 + 4
      if (x4 == C::TPR - 1) right = 0.f;
      const float f0[4] = {v.x, v.y, v.z, v.w};
      const float f1[4] = {v.y, v.z, v.w, right};
      const int se = sr / (RB + 1), rr = sr - se * (RB + 1);
      char* p = tail ? smem + 2 * C::BUF + lane * 8
                     : base0 + se * C::IMGP + rr * C::ROWP + c * C::XS + x4 * 8;
      store4(p, f0);
      store4(p + 2 * C::PLANE, f1);
    }
    if constexpr (SC) {
#pragma unroll
      for (int k = 0; k < C::NSTZ; ++k) {
        const int q = tid + 256 * k;
        const bool tail = C::NF4Z % 256 != 0 && k == C::NSTZ - 1 && q >= C::NF4Z;  // TAILB
        const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
        const float4 v = keep_if(rz[k], vz[k]);
        const float f0[4] = {v.x, v.y, v.z, v.w};
        const int se = sr / RB, rr = sr - se * RB;
        store4(tail ? smem + 2 * C::BUF + lane * 8
                    : base0 + C::HBUF + se * C::IMGPZ + rr * C::ROWPZ + c * C::XS + x4 * 8,
               f0);
      }
    }
  };

  // weights: the steps of a chunk (9 taps, then the shortcut) rotate through NW register
  // slots; after step s's MFMAs its slot is refilled with step s + NW (this chunk's or the
  // next one's), NW - 1 steps of prefetch distance.  NW divides the step count, so the slot of
  // a step is the same in every chunk.  Tap (ky, kx) of the forward conv is tap 8 - (3 ky + kx)
  // of the flipped pack.
  const int nkc = (cout + CC - 1) / CC;
  constexpr int NS = SC ? 10 : 9;
  constexpr int NW = SC ? 5 : 3;
  bf16x8 wsl[NW][2];
  auto load_step = [&](int kc, int s) {  // s compile-time at every call
    const int k = kc < nkc ? kc : nkc - 1;
    const __bf16* base =
        s < 9 ? A.w3t + ((size_t)(k * A.nob32 + ob32) * 18 + (8 - s) * 2) * 512 + lane * 8
              : A.w1t + ((size_t)(k * A.nob32 + ob32) * 2) * 512 + lane * 8;
    wsl[s % NW][0] = *reinterpret_cast<const bf16x8*>(base);
    wsl[s % NW][1] = *reinterpret_cast<const bf16x8*>(base + 512);
  };

  const int q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
  int tr_h[NT], tr_z[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int t = wt * 64 + n * 32 + 16 * g1 + 4 * p;
    const int e = t / (RB * WO), il = (t / WO) % RB;
    tr_h[n] = e * C::IMGP + il * C::ROWP + (8 * h + q) * C::XS + (t % WO) * 2;
    tr_z[n] = C::HBUF + e * C::IMGPZ + il * C::ROWPZ + (8 * h + q) * C::XS + (t % WO) * 2;
  }

  floatx16 acc[4][NT];  // [class py * 2 + px][column tile]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[i][n] = floatx16{0};

  bf16x8 bb[NT][2];
  // step s < 9: forward tap (ky, kx) = (s / 3, s % 3) reads dh fragment (oy, ox) = (ky == 0,
  // kx == 0); step 9: the shortcut's dz fragment
  auto read_step = [&](int buf, int s, int n) {
    const char* base = smem + buf * C::BUF;
    const char* a = s < 9 ? base + tr_h[n] + (s / 3 == 0) * C::ROWP + ((s % 3 == 0) * 2) * C::PLANE
                          : base + tr_z[n];
    bb[n][0] = tr_read8(a, a + 4 * C::XS);
    bb[n][1] = tr_read8(a + C::PLANE, a + C::PLANE + 4 * C::XS);
  };
  auto chunk = [&](int buf, int c) {
    load_chunk((c + 1) * CC);
#pragma unroll
    for (int n = 0; n < NT; ++n) read_step(buf, 0, n);
    static_for<NS>([&](auto Sc) {
      constexpr int s = decltype(Sc)::value;
      constexpr int ky = s / 3, kx = s % 3;
      constexpr int cls = s < 9 ? (ky != 1) * 2 + (kx != 1) : 0;
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        floatx16 d = acc[cls][n];
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wsl[s % NW][0], bb[n][0], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wsl[s % NW][0], bb[n][1], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wsl[s % NW][1], bb[n][0], d, 0, 0, 0);
        acc[cls][n] = d;
        if constexpr (s + 1 < NS) read_step(buf, s + 1, n);
      }
      if constexpr (s + NW < NS) load_step(c, s + NW);
      else load_step(c + 1, s + NW - NS);
      if constexpr (s == 6) store_chunk(buf ^ 1);
    });
    __syncthreads();
  };

  load_chunk(0);
  static_for<NW>([&](auto Sc) { load_step(0, decltype(Sc)::value); });
  store_chunk(0);
  __syncthreads();
  for (int c = 0; c < nkc; ++c) chunk(c & 1, c);

  // ---- epilogue: lane column t -> position (i, j); classes px = 0 / 1 -> one float2
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int tt = wt * 64 + n * 32 + (lane & 31);
    const int e = tt / (RB * WO), rem = tt % (RB * WO);
    const int i = i0 + rem / WO, j = rem % WO;
    const bool ve = b + e < B;
    const int64_t be = ve ? b + e : B - 1;
#pragma unroll
    for (int py = 0; py < 2; ++py) {
      // the mask of each row's two dx columns as bits 0 (px = 0) and 1 (px = 1): from the
      // plane bits (1 bit per element; a 32-bit word covers 32 consecutive positions of a
      // channel plane, so the lanes of a row share one word) or the fp32 mask (> 0)
      unsigned mk[16];
      if (A.mask_bits) {
        const int pos = (2 * i + py) * WI + 2 * j;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = c_w + (r & 3) + 8 * (r >> 2) + 4 * h;
          const size_t pl = ((size_t)be * cin + (c < cin ? c : cin - 1)) * HI * WI + pos;
          mk[r] = (A.mask_bits[pl >> 5] >> (pl & 31)) & 3u;
        }
      } else if (A.mask) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = c_w + (r & 3) + 8 * (r >> 2) + 4 * h;
          const size_t off =
              (((size_t)be * cin + (c < cin ? c : cin - 1)) * HI + 2 * i + py) * WI + 2 * j;
          const float2 m2 = *reinterpret_cast<const float2*>(A.mask + off);
          mk[r] = (m2.x > 0.f ? 1u : 0u) | (m2.y > 0.f ? 2u : 0u);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) mk[r] = 3u;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = c_w + (r & 3) + 8 * (r >> 2) + 4 * h;
        const size_t off =
            (((size_t)be * cin + (c < cin ? c : cin - 1)) * HI + 2 * i + py) * WI + 2 * j;
        float2 v = make_float2(acc[py * 2][n][r], acc[py * 2 + 1][n][r]);
        if (!(mk[r] & 1u)) v.x = 0.f;
        if (!(mk[r] & 2u)) v.y = 0.f;
        if (ve && c < cin) *reinterpret_cast<float2*>(A.dx + off) = v;
      }
    }
  }
}

// 1x1 weights [cout][cin] -> fragment-major bf16 hi/lo [chunk][32-o block][hi|lo][lane][8]
// (the A-operand map of v_mfma_f32_32x32x16_bf16, as the 3x3 pack with one tap); tflip
// packs the transposed matrix (the backward-data conv: out = cin, in = cout)
__global__ void pack1x1_kernel(const float* __restrict__ w, int cout, int cin, int tflip, int op,
                               int cp, int f16, float scale, __bf16* __restrict__ out) {
  const int nob32 = op / 32, nkc = cp / CC;
  const int total = nkc * nob32 * 2 * 512;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int j = i & 7, lane = (i >> 3) & 63;
    int r = i >> 9;
    const int pr = r & 1;
    r >>= 1;
    const int blk = r % nob32, kc = r / nob32;
    const int o = blk * 32 + (lane & 31), c = kc * CC + 8 * (lane >> 5) + j;
    const int no = tflip ? cin : cout, nc = tflip ? cout : cin;
    float v = 0.f;
    if (o < no && c < nc) v = tflip ? w[(size_t)c * cin + o] : w[(size_t)o * cin + c];
    v *= scale;  // a power of two (1 for bf16 packs): exact
    __bf16 hi, lo;
    if (f16)
      split16<true>(v, hi, lo);
    else
      split16<false>(v, hi, lo);
    out[i] = pr == 0 ? hi : lo;
  }
}

template <int WO, int RB, int E, bool SC, int NA, int WA, int EPI = 0, int XM = 0,
          bool F16 = false>
static int launch_fwd(FwdArgs a, hipStream_t st) {
  using C = DCfg<WO, RB, E>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(
        reinterpret_cast<const void*>(&down_fwd_kernel<WO, RB, E, SC, NA, false, WA, EPI, XM, F16>),
        hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    (void)hipFuncSetAttribute(
        reinterpret_cast<const void*>(&down_fwd_kernel<WO, RB, E, SC, NA, true, WA, EPI, XM, F16>),
        hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  DD_REQUIRE(a.HO % RB == 0, "dd_down_forward: HO must be a multiple of the row block");
  DD_REQUIRE(a.gsize % E == 0, "dd_down_forward: group_size %d must be a multiple of %d",
             a.gsize, E);
  a.n_tb = a.HO / RB;
  a.n_ob = (int)ceil_div(a.cout, 32 * WA * NA);
  a.tiles_per_group = (a.gsize / E) * a.n_tb * 2;  // two 32-position partials per tile
  const int64_t ntiles = ceil_div(a.B, E) * a.n_tb * a.n_ob;
  DD_REQUIRE(ntiles < (1ll << 31), "dd_down_forward: too many tiles");
  a.n_tiles = (int)ntiles;
  // persistent (as dd_conv.hip) where the K loop is short and a tile's prologue shows: two
  // resident workgroups per CU walk the tiles.  Measured (1024 examples, shortcut fused):
  // +5-9 % at cin = 64 (4 K chunks, the layer2 head), -2.5-4 % at cin = 128 / 256 (the
  // persistent loop costs ~30 VGPRs there), which keep one tile per workgroup.
  const bool pt = a.cin <= 64;
  const int64_t cap = pt ? (NA == 2 ? 1ll : 2ll) * device_cus() : ntiles;
  const int64_t grid = ntiles < cap ? ntiles : cap;
  if (pt)
    down_fwd_kernel<WO, RB, E, SC, NA, true, WA, EPI, XM, F16>
        <<<(unsigned)grid, 256, C::LDS, st>>>(a);
  else
    down_fwd_kernel<WO, RB, E, SC, NA, false, WA, EPI, XM, F16>
        <<<(unsigned)grid, 256, C::LDS, st>>>(a);
  DD_CHECK_LAUNCH("dd_down_forward");
  return DD_OK;
}

// the padded-width heads (down_fwd_kernel PW): 128-output workgroups (four waves along o), one
// tile per workgroup, the EL2N statistics launch with the producer's BN + ReLU staged or raw
template <int WO, int RB, int PW, int XM, bool F16>
static int launch_fwd_pw(FwdArgs a, hipStream_t st) {
  using C = DCfg<WO, RB, 1>;
  constexpr auto K = &down_fwd_kernel<WO, RB, 1, false, 1, false, 4, 0, XM, F16, PW>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(K),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  a.n_tb = (a.HO + RB - 1) / RB;
  a.n_ob = (int)ceil_div(a.cout, 128);
  a.tiles_per_group = a.gsize * a.n_tb * 2;  // two 32-position partials per tile
  const int64_t ntiles = a.B * a.n_tb * a.n_ob;
  DD_REQUIRE(ntiles < (1ll << 31), "dd_down_forward: too many tiles");
  a.n_tiles = (int)ntiles;
  K<<<(unsigned)ntiles, 256, C::LDS, st>>>(a);
  DD_CHECK_LAUNCH("dd_down_forward");
  return DD_OK;
}

// channel blocks per wave: 1 by default.  NA = 2 (DD_DOWN_NA=2, where the padded outputs fill
// 128-channel workgroups) needs 336-344 registers, so one workgroup per CU: measured 3-5 %
// slower on all three ResNet-18 heads (profiles/r01_v18/experiments/down_na2_ab.txt)
static int fwd_na(int cout) {
  static int f = -1;
  if (f < 0) {
    const char* e = getenv("DD_DOWN_NA");
    f = e ? atoi(e) : 0;
  }
  return f == 2 && conv::pad_to(cout, 64) % 128 == 0 ? 2 : 1;
}
// four waves along o (128-output workgroups) where the padded outputs fill them: 1.13-1.26x
// the 2 x 2 layout on the three ResNet-18 heads, bit-identical (tools/ab_conv.py --kernel down,
// B = 1024, profiles/r02_s2/ab_down_fwd_wa4.txt); DD_DOWN_WA=2 keeps the 2 x 2 layout
// the compile-time epilogue of a launch with the shortcut fused (down_fwd_kernel EPI): 1 / 2
// for the EL2N / GraNd flag sets, 0 otherwise or with DD_DOWN_EPI=0 (the runtime-flag kernel)
static int fwd_epi(const Out& m, const Out& s) {
  static int f = -1;
  if (f < 0) {
    const char* e = getenv("DD_DOWN_EPI");
    f = e ? atoi(e) : 1;
  }
  if (f == 0 || !s.y) return 0;
  if (!m.bias && !m.relu && m.stats && !s.bias && !s.relu && s.stats) return 1;
  if (m.bias && m.relu && !m.stats && s.bias && !s.relu && !s.stats) return 2;
  return 0;
}
static int fwd_wa(int cout) {
  static int f = -1;
  if (f < 0) {
    const char* e = getenv("DD_DOWN_WA");
    f = e ? atoi(e) : 4;
  }
  return f == 4 && conv::pad_to(cout, 64) % 128 == 0 ? 4 : 2;
}

template <int WO, int RB, int E, bool SC>
static int launch_bwd(BwdArgs a, hipStream_t st) {
  using C = UCfg<WO, RB, E, SC>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&down_bwd_kernel<WO, RB, E, SC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  DD_REQUIRE(a.HO % RB == 0, "dd_down_backward: HO must be a multiple of the row block");
  a.n_tb = a.HO / RB;
  a.n_ob = (int)ceil_div(a.cin, 64);
  const int64_t grid = ceil_div(a.B, E) * a.n_tb * a.n_ob;
  DD_REQUIRE(grid < (1ll << 31), "dd_down_backward: grid too large");
  down_bwd_kernel<WO, RB, E, SC><<<(unsigned)grid, 256, C::LDS, st>>>(a);
  DD_CHECK_LAUNCH("dd_down_backward");
  return DD_OK;
}

template <int WO, int RB, int E, bool SC>
static int launch_bwd2(BwdArgs a, hipStream_t st) {
  using C = UCfg<WO, RB, E, SC>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&down_bwd2_kernel<WO, RB, E, SC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  static_assert(2 * C::LDS <= 160 * 1024, "two workgroups per CU");
  DD_REQUIRE(a.HO % RB == 0, "dd_down_backward: HO must be a multiple of the row block");
  a.n_tb = a.HO / RB;
  a.n_ob = (int)ceil_div(a.cin, 64);
  const int64_t grid = ceil_div(a.B, E) * a.n_tb * a.n_ob;
  DD_REQUIRE(grid < (1ll << 31), "dd_down_backward: grid too large");
  down_bwd2_kernel<WO, RB, E, SC><<<(unsigned)grid, 256, C::LDS, st>>>(a);
  DD_CHECK_LAUNCH("dd_down_backward");
  return DD_OK;
}

// backward workgroups of 128 positions (down_bwd2_kernel) unless DD_DOWN_BWD=1: 1.21-1.38x the
// 64-position kernel on the three ResNet-18 heads, bit-identical (tools/ab_conv.py --kernel bwd,
// B = 1024, profiles/r02_s2/ab_down_bwd2.txt)
static bool bwd2() {
  static int f = -1;
  if (f < 0) {
    const char* e = getenv("DD_DOWN_BWD");
    f = e ? atoi(e) : 2;
  }
  return f == 2;
}

// padded-width geometry (down_fwd_kernel PW): tile width, row block and PW mode of an output
// width that is not a tile width, or 0 (DD_DOWN_PW=0 turns them off; read per call)
static int pw_geometry(int ho, int wo, int* rb, int* pw) {
  const char* env = getenv("DD_DOWN_PW");
  if ((env && atoi(env) == 0) || ho <= 0) return 0;
  if (wo > 16 && wo <= 32 && wo % 4 == 0) { *rb = 2; *pw = 1; return 32; }
  if (wo > 8 && wo <= 16 && wo % 2 == 0) { *rb = 4; *pw = 2; return 16; }
  if (wo > 4 && wo <= 8) { *rb = 8; *pw = 3; return 8; }
  return 0;
}

static bool geometry(int ho, int wo, int* rb, int* e) {
  if (wo == 32 && ho % 2 == 0) { *rb = 2; *e = 1; return true; }
  if (wo == 16 && ho % 4 == 0) { *rb = 4; *e = 1; return true; }
  if (wo == 8 && ho == 8) { *rb = 8; *e = 1; return true; }
  if (wo == 4 && ho == 4) { *rb = 4; *e = 4; return true; }
  return false;
}

}  // namespace down
}  // namespace dd

using namespace dd;

extern "C" {

size_t dd_conv1x1_pack_bytes(int32_t out_channels, int32_t in_channels) {
  if (out_channels <= 0 || in_channels <= 0) return 0;
  // K padded to 32: dd_conv1x1_forward reads 32-channel chunks (the zero tail is never read
  // by the down kernels' 16-channel K loop)
  return (size_t)2 * conv::pad_to(out_channels, 64) * conv::pad_to(in_channels, 2 * conv::CC) *
         sizeof(__bf16);
}

int dd_conv1x1_pack(const float* w, int32_t cout, int32_t cin, int32_t transpose,
                    int32_t operands, float scale, void* packed, void* stream) {
  clear_error();
  DD_REQUIRE(w && packed && cout > 0 && cin > 0, "dd_conv1x1_pack: bad arguments");
  DD_REQUIRE(operands == DD_OPERANDS_BF16X3 || operands == DD_OPERANDS_F16X3,
             "dd_conv1x1_pack: operands must be DD_OPERANDS_BF16X3 or DD_OPERANDS_F16X3");
  DD_REQUIRE(operand_scale_ok(operands, scale),
             "dd_conv1x1_pack: scale must be 1 (bf16 operands) or a power of two (fp16)");
  const int no = transpose ? cin : cout, nc = transpose ? cout : cin;
  const int op = conv::pad_to(no, 64), cp = conv::pad_to(nc, 2 * conv::CC);
  const int total = 2 * op * cp;
  down::pack1x1_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 4096), 256, 0,
                         as_stream(stream)>>>(w, cout, cin, transpose, op, cp,
                                              operands == DD_OPERANDS_F16X3, scale,
                                              static_cast<__bf16*>(packed));
  DD_CHECK_LAUNCH("dd_conv1x1_pack");
  return DD_OK;
}

int dd_down_tiles_per_group(int32_t ho, int32_t wo, int32_t group_size) {
  int rb, e, pw;
  if (group_size <= 0) return -1;
  if (!down::geometry(ho, wo, &rb, &e)) {
    // a padded-width head: the same layout on the padded grid
    if (!down::pw_geometry(ho, wo, &rb, &pw)) return -1;
    return group_size * ((ho + rb - 1) / rb) * 2;
  }
  if (group_size % e) return -1;
  return (group_size / e) * (ho / rb) * 2;  // one BN partial per 32-position fragment
}

int dd_down_padded_supported(int32_t ho, int32_t wo, int32_t cin, int32_t cout,
                             int32_t group_size) {
  int rb, e, pw;
  if (ho <= 0 || wo <= 0 || cin <= 64 || cout <= 0 || group_size <= 0 ||
      down::geometry(ho, wo, &rb, &e) || !down::pw_geometry(ho, wo, &rb, &pw))
    return 0;
  return down::fwd_wa(cout) == 4 && (int64_t)cin * 4 * ho * wo < (1ll << 31) ? 1 : 0;
}

static int down_forward_impl(const float* x, int64_t B, int32_t cin, int32_t ho, int32_t wo,
                             const void* packed3x3, const void* packed1x1, int32_t cout,
                             const float* bias, int32_t relu, float* stats, float* y,
                             const float* bias_sc, int32_t relu_sc, float* stats_sc,
                             float* y_sc, int32_t group_size, int64_t n_stat,
                             const float* in_scale, const float* in_shift, const float* xres,
                             int32_t operands, float acc_scale, float acc_scale_sc,
                             void* stream) {
  DD_REQUIRE(B >= 0 && cin > 0 && cout > 0 && ho > 0, "dd_down_forward: bad sizes");
  DD_REQUIRE(operands == DD_OPERANDS_BF16X3 || operands == DD_OPERANDS_F16X3,
             "dd_down_forward: operands must be DD_OPERANDS_BF16X3 or DD_OPERANDS_F16X3");
  DD_REQUIRE(operand_scale_ok(operands, acc_scale) && operand_scale_ok(operands, acc_scale_sc),
             "dd_down_forward: acc_scale must be 1 (bf16 operands) or a power of two (fp16)");
  if (B == 0) return DD_OK;
  DD_REQUIRE(x && packed3x3 && y, "dd_down_forward: null buffer");
  DD_REQUIRE(!packed1x1 == !y_sc, "dd_down_forward: shortcut pack and output go together");
  // dd_conv3x3_pack writes the stride-1 stem layout for cin <= CC / 3 (dd_conv.hip)
  DD_REQUIRE(cin > conv::CC / 3, "dd_down_forward: cin %d <= %d is packed in the stem layout",
             cin, conv::CC / 3);
  DD_REQUIRE((int64_t)cin * 4 * ho * wo < (1ll << 31), "dd_down_forward: tensor too large");
  const bool grouped = stats || stats_sc;
  DD_REQUIRE(!grouped || group_size > 0, "dd_down_forward: group_size must be positive");
  int rb, e, pw = 0, pw_w = 0;
  if (!down::geometry(ho, wo, &rb, &e)) {
    // the padded-width heads: the EL2N statistics launch of a Bottleneck's conv2 alone
    if (stats && !packed1x1 && !bias && !relu && !xres &&
        dd_down_padded_supported(ho, wo, cin, cout, group_size))
      pw_w = down::pw_geometry(ho, wo, &rb, &pw);
    if (!pw_w) {
      set_error("dd_down_forward: unsupported output shape %dx%d (32 wide with even HO, 16 wide "
                "with HO %% 4 == 0, 8x8 or 4x4; other widths up to 32 for the statistics "
                "launch without a shortcut, cin > 64, cout padded to 128)", ho, wo);
      return DD_EINVAL;
    }
    e = 1;
  }
  down::FwdArgs a{};
  a.x = x;
  a.w3 = static_cast<const __bf16*>(packed3x3);
  a.ws = static_cast<const __bf16*>(packed1x1);
  a.main = down::Out{y, bias, stats, relu, acc_scale};
  a.sc = down::Out{y_sc, bias_sc, stats_sc, relu_sc, acc_scale_sc};
  a.B = B;
  a.n_stat = grouped ? std::min<int64_t>(std::max<int64_t>(n_stat, 0), B) : 0;
  a.cin = cin;
  a.HO = ho;
  a.cout = cout;
  a.nob32 = conv::pad_to(cout, 64) / 32;
  a.gsize = grouped ? group_size : (int)(std::min<int64_t>(B + e, 1 << 30) / e * e);
  static int xcd = -1;
  if (xcd < 0) {
    const char* ev = getenv("DD_DOWN_XCD");
    xcd = ev ? atoi(ev) : 2;
  }
  a.xcd = xcd;
  hipStream_t st = as_stream(stream);
  const bool sc = packed1x1 != nullptr;
  a.in_scale = in_scale;
  a.in_shift = in_shift;
  a.xres = xres;
  a.wog = wo;
  if (pw_w) {
    const bool f16 = operands == DD_OPERANDS_F16X3, xf = in_scale != nullptr;
#define DD_DOWN_PWL(WO_, RB_, PW_)                                                              \
    if (pw_w == WO_ && pw == PW_)                                                               \
      return f16 ? (xf ? down::launch_fwd_pw<WO_, RB_, PW_, down::kXmAffine, true>(a, st)       \
                       : down::launch_fwd_pw<WO_, RB_, PW_, down::kXmNone, true>(a, st))        \
                 : (xf ? down::launch_fwd_pw<WO_, RB_, PW_, down::kXmAffine, false>(a, st)      \
                       : down::launch_fwd_pw<WO_, RB_, PW_, down::kXmNone, false>(a, st));
    DD_DOWN_PWL(32, 2, 1)
    DD_DOWN_PWL(16, 4, 2)
    DD_DOWN_PWL(8, 8, 3)
#undef DD_DOWN_PWL
    set_error("dd_down_forward: no padded-width head for width %d", wo);
    return DD_EINVAL;
  }
  if (operands == DD_OPERANDS_F16X3) {
    // fp16 operand halves: the EL2N launch shapes (statistics epilogue; the staging transform
    // or none) and the GraNd forward's (bias + ReLU) at the default wave layout, and the
    // run-time epilogue for anything else
    const int wa = down::fwd_wa(cout);
    const int epi = down::fwd_epi(a.main, a.sc);  // 1: EL2N statistics, 2: GraNd bias + ReLU
    DD_REQUIRE(!xres || (sc && epi == 1),
               "dd_down_forward_unit_input: the unit form needs the fused shortcut and "
               "statistics on both outputs");
    DD_REQUIRE(!in_scale || xres || !sc,
               "dd_down_forward_unit_input: BN + ReLU staging without a shortcut only");
#define DD_DOWN_F(WO_, RB_, E_, WA_)                                                          \
    if (xres) return down::launch_fwd<WO_, RB_, E_, true, 1, WA_, 1, down::kXmUnit, true>(a, st); \
    if (in_scale) return down::launch_fwd<WO_, RB_, E_, false, 1, WA_, 0, down::kXmAffine, true>(a, st); \
    if (sc && epi == 1) return down::launch_fwd<WO_, RB_, E_, true, 1, WA_, 1, 0, true>(a, st); \
    if (sc && epi == 2) return down::launch_fwd<WO_, RB_, E_, true, 1, WA_, 2, 0, true>(a, st); \
    if (sc) return down::launch_fwd<WO_, RB_, E_, true, 1, WA_, 0, 0, true>(a, st);           \
    return down::launch_fwd<WO_, RB_, E_, false, 1, WA_, 0, 0, true>(a, st);
#define DD_DOWN_FW(WO_, RB_, E_) \
    if (wa == 4) { DD_DOWN_F(WO_, RB_, E_, 4) } else { DD_DOWN_F(WO_, RB_, E_, 2) }
    if (wo == 32) { DD_DOWN_FW(32, 2, 1) }
    if (wo == 16) { DD_DOWN_FW(16, 4, 1) }
    if (wo == 8) { DD_DOWN_FW(8, 8, 1) }
    DD_DOWN_FW(4, 4, 4)
#undef DD_DOWN_FW
#undef DD_DOWN_F
  }
  if (in_scale) {
    // the staging transform: BN + ReLU (+ the unit's identity shortcut), on the EL2N launch
    // shapes only (statistics epilogue; 64-output-wave tiles)
    // (the unit form of the persistent cin <= 64 head spills 7 registers at four waves along
    // o, and is still faster there than two along o: EL2N forward 3.625-3.639 vs 3.681-3.682
    // ms, profiles/r04_fuse/ab_head_wa.txt; DD_DOWN_XWA=2 takes two, for A/B runs)
    static int xwa = -1;
    if (xwa < 0) {
      const char* e = getenv("DD_DOWN_XWA");
      xwa = e ? atoi(e) : 4;
    }
    const int wa = xres && cin <= 64 && xwa == 2 ? 2 : down::fwd_wa(cout);
#define DD_DOWN_X(WO_, RB_, E_)                                                          \
    if (xres) {                                                                          \
      DD_REQUIRE(sc && down::fwd_epi(a.main, a.sc) == 1,                                 \
                 "dd_down_forward_unit_input: the unit form needs the fused shortcut and " \
                 "statistics on both outputs");                                          \
      return wa == 4 ? down::launch_fwd<WO_, RB_, E_, true, 1, 4, 1, down::kXmUnit>(a, st) \
                     : down::launch_fwd<WO_, RB_, E_, true, 1, 2, 1, down::kXmUnit>(a, st); \
    }                                                                                    \
    DD_REQUIRE(!sc, "dd_down_forward_unit_input: BN + ReLU staging without a shortcut only"); \
    return wa == 4 ? down::launch_fwd<WO_, RB_, E_, false, 1, 4, 0, down::kXmAffine>(a, st) \
                   : down::launch_fwd<WO_, RB_, E_, false, 1, 2, 0, down::kXmAffine>(a, st);
    if (wo == 32) { DD_DOWN_X(32, 2, 1) }
    if (wo == 16) { DD_DOWN_X(16, 4, 1) }
    if (wo == 8) { DD_DOWN_X(8, 8, 1) }
    DD_DOWN_X(4, 4, 4)
#undef DD_DOWN_X
  }
  const int na = down::fwd_na(cout), wa = na == 2 ? 2 : down::fwd_wa(cout);
  const int epi = na == 2 ? 0 : down::fwd_epi(a.main, a.sc);
#define DD_DOWN_SC(WO_, RB_, E_, WA_)                                                  \
  (epi == 1   ? down::launch_fwd<WO_, RB_, E_, true, 1, WA_, 1>(a, st)                \
   : epi == 2 ? down::launch_fwd<WO_, RB_, E_, true, 1, WA_, 2>(a, st)                \
              : down::launch_fwd<WO_, RB_, E_, true, 1, WA_, 0>(a, st))
#define DD_DOWN(WO_, RB_, E_)                                                    \
  return na == 2 ? (sc ? down::launch_fwd<WO_, RB_, E_, true, 2, 2>(a, st)       \
                       : down::launch_fwd<WO_, RB_, E_, false, 2, 2>(a, st))     \
         : wa == 4 ? (sc ? DD_DOWN_SC(WO_, RB_, E_, 4)                           \
                         : down::launch_fwd<WO_, RB_, E_, false, 1, 4>(a, st))   \
                 : (sc ? DD_DOWN_SC(WO_, RB_, E_, 2)                             \
                       : down::launch_fwd<WO_, RB_, E_, false, 1, 2>(a, st))
  if (wo == 32) DD_DOWN(32, 2, 1);
  if (wo == 16) DD_DOWN(16, 4, 1);
  if (wo == 8) DD_DOWN(8, 8, 1);
  DD_DOWN(4, 4, 4);
#undef DD_DOWN
#undef DD_DOWN_SC
}

int dd_down_forward(const float* x, int64_t B, int32_t cin, int32_t ho, int32_t wo,
                    const void* packed3x3, const void* packed1x1, int32_t cout,
                    const float* bias, int32_t relu, float* stats, float* y,
                    const float* bias_sc, int32_t relu_sc, float* stats_sc, float* y_sc,
                    int32_t group_size, int64_t n_stat, int32_t operands, float acc_scale,
                    float acc_scale_sc, void* stream) {
  clear_error();
  return down_forward_impl(x, B, cin, ho, wo, packed3x3, packed1x1, cout, bias, relu, stats, y,
                           bias_sc, relu_sc, stats_sc, y_sc, group_size, n_stat, nullptr,
                           nullptr, nullptr, operands, acc_scale, acc_scale_sc, stream);
}

int dd_down_forward_unit_input(const float* y_prev, const float* in_scale,
                               const float* in_shift, const float* res, int64_t B, int32_t cin,
                               int32_t ho, int32_t wo, const void* packed3x3,
                               const void* packed1x1, int32_t cout, float* stats, float* y,
                               float* stats_sc, float* y_sc, int32_t group_size,
                               int64_t n_stat, int32_t operands, float acc_scale,
                               float acc_scale_sc, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0, "dd_down_forward_unit_input: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(y_prev && in_scale && in_shift && stats && y && group_size > 0,
             "dd_down_forward_unit_input: null buffer or group");
  DD_REQUIRE(!res == !packed1x1 && !packed1x1 == !y_sc && !y_sc == !stats_sc,
             "dd_down_forward_unit_input: the shortcut (res, its pack, y_sc, stats_sc) goes "
             "together");
  return down_forward_impl(y_prev, B, cin, ho, wo, packed3x3, packed1x1, cout, nullptr, 0,
                           stats, y, nullptr, 0, stats_sc, y_sc, group_size, n_stat, in_scale,
                           in_shift, res, operands, acc_scale, acc_scale_sc, stream);
}

int dd_down_backward(const float* dh, const float* dz, int64_t B, int32_t cout, int32_t ho,
                     int32_t wo, const void* packed3x3_t, const void* packed1x1_t, int32_t cin,
                     const float* mask_src, const uint32_t* mask_bits, float* dx,
                     void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && cin > 0 && cout > 0 && ho > 0, "dd_down_backward: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(dh && packed3x3_t && dx, "dd_down_backward: null buffer");
  DD_REQUIRE(!dz == !packed1x1_t, "dd_down_backward: dz and the shortcut pack go together");
  DD_REQUIRE((int64_t)cin * 4 * ho * wo < (1ll << 31), "dd_down_backward: tensor too large");
  int rb, e;
  if (!down::geometry(ho, wo, &rb, &e)) {
    set_error("dd_down_backward: unsupported output shape %dx%d", ho, wo);
    return DD_EINVAL;
  }
  down::BwdArgs a{};
  a.dh = dh;
  a.dz = dz;
  a.w3t = static_cast<const __bf16*>(packed3x3_t);
  a.w1t = static_cast<const __bf16*>(packed1x1_t);
  DD_REQUIRE(!(mask_src && mask_bits), "dd_down_backward: mask_src and mask_bits are exclusive");
  a.mask = mask_src;
  a.mask_bits = mask_bits;
  a.dx = dx;
  a.B = B;
  a.cin = cin;
  a.cout = cout;
  a.HO = ho;
  a.nob32 = conv::pad_to(cin, 64) / 32;
  static int xcd = -1;
  if (xcd < 0) {
    const char* ev = getenv("DD_DOWN_XCD");
    xcd = ev ? atoi(ev) : 1;
  }
  a.xcd = xcd;
  hipStream_t st = as_stream(stream);
  const bool sc = dz != nullptr;
#define DD_UP2(WO_, RB_, E_)                                      \
  return sc ? down::launch_bwd2<WO_, RB_, E_, true>(a, st)        \
            : down::launch_bwd2<WO_, RB_, E_, false>(a, st)
  // mask_bits is read only by the 128-position kernel: exactly its three dispatch cases below
  // (a 16-wide map with ho % 8 != 0 falls through to launch_bwd, which reads A.mask only)
  DD_REQUIRE(!mask_bits || (down::bwd2() && ((wo == 16 && ho % 8 == 0) || (wo == 8 && ho == 8) ||
                                             (wo == 4 && ho == 4))),
             "dd_down_backward: mask_bits needs the 128-position kernel (16-wide maps with "
             "ho %% 8 == 0, 8x8, 4x4)");
  if (down::bwd2()) {
    if (wo == 16 && ho % 8 == 0) DD_UP2(16, 8, 1);
    if (wo == 8 && ho == 8) DD_UP2(8, 8, 2);
    if (wo == 4 && ho == 4) DD_UP2(4, 4, 8);
  }
#undef DD_UP2
#define DD_UP(WO_, RB_, E_)                                       \
  return sc ? down::launch_bwd<WO_, RB_, E_, true>(a, st)         \
            : down::launch_bwd<WO_, RB_, E_, false>(a, st)
  if (wo == 32) DD_UP(32, 2, 1);
  if (wo == 16) DD_UP(16, 4, 1);
  if (wo == 8) DD_UP(8, 8, 1);
  DD_UP(4, 4, 4);
#undef DD_UP
}

}  // extern "C"
