// Split-bf16 implicit-GEMM 3x3 / stride-1 / pad-1 convolution, NCHW fp32 in and out.
//
// Serves the backbone's 3x3 stride-1 convs (88% of ResNet-18 flops) in both directions of the
// GraNd pass and the forward of the EL2N pass:
//   forward    y = epilogue(conv(x, W))                      W packed as-is
//   bwd-data   dx = epilogue(conv(dy, flip(W)^T))            same kernel, weights repacked
// epilogue(v) = ((v + bias[o]) + residual) -> ReLU? -> * (mask_src > 0)?  (each optional), so
// the folded-BN bias, the residual add, the ReLU and the ReLU-backward mask never take an
// extra pass over HBM.
//
// GEMM per example: D[o][t] = sum_{tap, c} W[o][c][tap] * x[c][t + shift(tap)].
// workgroup = (example, 64 output channels, RB output rows = TB positions); 4 waves as 2 (o) x
// 2 (t), each 32 o x TB/2 t = NT tiles of v_mfma_f32_32x32x16_bf16.  K loop over chunks of 16
// input channels: the chunk's RB+2 input rows are staged in LDS as [row][kx][hi|lo][c][x]
// images pre-shifted by kx-1 (double-buffered), and the B operand (8 consecutive channels at one
// position) is read with ds_read_b64_tr_b16, the hardware-transposed read, from the same
// channel-major image the GraNd norm kernel uses.  A fragments (weights, 16 B per lane) come
// from a pre-split bf16 hi/lo pack [hi|lo][tap][o][c] in global memory (L2-resident).
// Products are hi*hi + hi*lo + lo*hi with fp32 accumulation (~2^-16 relative per product).
//
// Train-mode BatchNorm (the EL2N pass, reference semantics: batch statistics over each pinned
// batch) is fused around the kernel instead of taking passes of its own:
//   * input transform at staging: x' = max(x * in_scale[g][c] + in_shift[g][c], in_floor), so
//     the previous conv's BN + ReLU is applied while its raw output is staged (g = the BN group
//     of the example = b / group_size; the identity when no transform is given);
//   * statistics epilogue: per workgroup and output channel, the sum and the sum of squares of
//     the written values over the tile's valid positions (rows b < n_stat), reduced across the
//     wave by a butterfly transpose-reduce (31 shuffles for 32 values), one partial per
//     (group, channel, tile); dd_bn_finalize turns them into the next consumer's affine.
//
// (This header holds the kernel templates and their launchers; dd_conv.hip (host entry points,
// packing, tile selection, the narrow 32x32 tile), dd_conv_nw.hip (the other narrow / wide
// tiles) and dd_conv_r2.hip (the r2 tiles) instantiate them, so the three compile in
// parallel.)
// Two kernels share the argument block, staging, fragment order, masks and statistics
// layouts: conv3x3_kernel (the narrow / wide tiles; the 32x32 layers and the stem) and
// conv3x3_r2_kernel (16x16 and smaller maps with 128-output workgroups of 4 waves along o);
// select() picks per shape from measured A/B runs.
#pragma once

#ifndef DD_R2_FENCE
#define DD_R2_FENCE 2
#endif
#include "dd_mfma.h"

#include <stdlib.h>
#include <string.h>

namespace dd {
namespace conv {

struct Args {
  const float* x;
  const __bf16* wpack;
  const float* bias;
  const float* residual;
  const float* mask_src;
  const float* in_scale;  // [G][cin], or g_unit_affine with xf_mask = 0
  const float* in_shift;  // [G][cin], or g_unit_affine + 1
  float* y;
  float* stats;           // NULL or partials [G][cout][tiles_per_group][2]
  // ReLU masks in fragment order (one 16-bit word per lane per 32-position tile: bit r =
  // (output of row r > 0)).  A producer writes mask_out; a later launch with the same
  // geometry (B, h, w and output channels) reads mask_in in place of mask_src.
  uint16_t* mask_out;
  const uint16_t* mask_in;
  int64_t B, n_stat;
  int cin, H, cout, op, cp;
  int relu, xf_mask, gsize, tiles_per_group;
  float in_floor;         // 0 (ReLU after the affine) or -inf
  int n_tb, n_ob, n_tiles;
  int kx1;                // the stem layout (cin <= kStemCin; see conv3x3_kernel)
  int f16;                // fp16 operand halves (pack and staging; DD_OPERANDS_F16X3)
  float acc_scale;        // fp16 packs hold W * 2^s: accumulators are multiplied by 2^-s (exact)
  int xcd;                // XCD-contiguous persistent tile order (DD_CONV_XCD, see conv_xcd)
  int wg;                 // the image width in memory of a padded-width launch (PW tiles)
  int stagger;            // shader cycles the upper half of the grid waits before its first
                          // tile (DD_CONV_STAGGER; 0 = off): desynchronises the two resident
                          // workgroups of a CU so their epilogues do not coincide
  // the fused residual-unit input (staging modes XF >= 2, see kXfOut): the staged value is
  // max(x * in_scale + in_shift + R, in_floor) with R = xres (XF = 3) or xres * xres_scale +
  // xres_shift (XF = 4), and the output-channel block 0 tiles write it to xout once
  const float* xres;
  const float* xres_scale;  // [G][cin]
  const float* xres_shift;
  float* xout;
};

// staging modes (template parameter XF): none, the producer's BN affine (+ ReLU), and the
// fused residual-unit input -- the affine plus the write-out, with an identity or BN'd
// residual added before the ReLU (reference models/resnet.py:31-32, out += shortcut(x);
// relu(out), computed while the next unit's first conv stages it)
constexpr int kXfNone = 0, kXfAffine = 1, kXfOut = 2, kXfOutRes = 3, kXfOutResAff = 4;

// the upper half of a persistent grid starts `cycles` later (see Args::stagger)
__device__ __forceinline__ void stagger_start(int cycles) {
  if (cycles > 0 && blockIdx.x >= (gridDim.x >> 1)) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < (uint64_t)cycles) __builtin_amdgcn_s_sleep(8);
  }
}

// XCD-contiguous tile order of the persistent grids (default; DD_CONV_XCD=0 turns it off):
// workgroup p starts at logical tile xcd_order(p, grid) and walks +grid, so at any moment each
// XCD works on one contiguous run of tiles -- the output-channel blocks of a position block
// (which stage the same input rows) and neighbouring row blocks (which share halo rows) meet
// in one L2.  The tiles and their numbering (the fragment-order masks are indexed by tile) are
// unchanged, so results are bitwise equal either way.  Measured (tools/xcd_ab.sh, B = 1024,
// profiles/r06_s3/xcd_ab/): PMC fetch per dispatch 1.22 -> 1.00x algorithmic at 32x32, 1.36 ->
// 1.04x at 16x16, 1.94 -> 1.34x at 8x8 (4x4 and the stem unchanged); time 0.98-0.99x per shape
// (alternated twice), whole job within 0.4 %.
inline int conv_xcd() {
  const char* e = getenv("DD_CONV_XCD");
  return e ? atoi(e) : 1;
}

inline int stagger_cycles() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DD_CONV_STAGGER");
    v = e ? atoi(e) : 0;
    if (v < 0) v = 0;
  }
  return v;
}

// input channels up to which dd_conv3x3_pack writes the stem layout (3 cin <= CC)
constexpr int kStemCin = CC / 3;

// Compile-time epilogue variants (template parameter EPI).  0: every operation is decided at
// run time from Args (any combination).  Otherwise kEpiSpec | the operations present: the
// launch shapes of the scoring passes each compile to exactly their own epilogue, with no run
// time tests and no dead operand paths (epilogue_code() picks one at launch).
constexpr int kEpiBias = 1, kEpiRes = 2, kEpiRelu = 4, kEpiMsrc = 8, kEpiMin = 16,
              kEpiMout = 32, kEpiStats = 64, kEpiSpec = 128;
// operand halves of the launch (dd_mfma.h): fp16 with this bit set, else bf16 (not an epilogue
// operation: carried in EPI so one template parameter selects the compiled variant)
constexpr int kEpiF16 = 256;

// the epilogue flags of one launch
struct EpiFlags {
  bool bias, res, relu, msrc, min, mout, stats;
};
template <int EPI>
__device__ __forceinline__ EpiFlags epi_flags(const Args& A) {
  if constexpr ((EPI & ~kEpiF16) == 0) {
    return {A.bias != nullptr, A.residual != nullptr, A.relu != 0, A.mask_src != nullptr,
            A.mask_in != nullptr, A.mask_out != nullptr, A.stats != nullptr};
  } else {
    return {(EPI & kEpiBias) != 0, (EPI & kEpiRes) != 0, (EPI & kEpiRelu) != 0,
            (EPI & kEpiMsrc) != 0, (EPI & kEpiMin) != 0, (EPI & kEpiMout) != 0,
            (EPI & kEpiStats) != 0};
  }
}

typedef unsigned uint4v __attribute__((ext_vector_type(4)));

// the staged value of one input element under staging mode XF (the arithmetic of
// dd_bn_apply's apply_one, in its order, so the fused and the separate passes agree bitwise)
template <int XF>
__device__ __forceinline__ float4 stage_transform(float4 v, float s, float t, float4 r, float rs,
                                                  float rt, float floor_) {
  v = make_float4(fmaf(v.x, s, t), fmaf(v.y, s, t), fmaf(v.z, s, t), fmaf(v.w, s, t));
  if constexpr (XF >= kXfOutRes) {
    if constexpr (XF == kXfOutResAff)
      r = make_float4(fmaf(r.x, rs, rt), fmaf(r.y, rs, rt), fmaf(r.z, rs, rt), fmaf(r.w, rs, rt));
    v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
  }
  return make_float4(nmax(v.x, floor_), nmax(v.y, floor_), nmax(v.z, floor_),
                     nmax(v.w, floor_));
}

// Tile configuration.  A workgroup = 4 waves as WO (along o) x WT = 4 / WO (along t); a wave
// owns NA 32-row A blocks (output channels) x NT 32-column t tiles, NA * NT accumulators of
// v_mfma_f32_32x32x16_bf16.
//   NA = 1, WO = 2 ("narrow"): 32 o x TB/2 t per wave, two workgroups per CU;
//   NA = 2 ("wide"): 64 o x 64 t per wave, one workgroup per CU with the 512-register budget.
// Each B fragment read from LDS and each staged input element then serves twice the MFMAs:
// the narrow tile spends ~5.8 non-MFMA instructions per MFMA, past what the SIMD can issue
// beside the matrix pipe at two waves per SIMD.
template <int W, int RB, int E, int NA, int WO>
struct Cfg {
  static constexpr int WT = 4 / WO;            // waves along t
  static constexpr int NR = E * (RB + 2);      // input rows staged per chunk (E images)
  static constexpr int XS = W * 2;             // bytes of one channel row (bf16)
  static constexpr int PLANE = CC * XS;        // one (row, kx, hi|lo) image
  // staged row pitch / image pitch, padded so that the transposed B reads of one 32-lane
  // group (4 channels x 32 consecutive positions, spanning 1, 2, 4 or 8 staged rows) hit
  // distinct LDS banks: rows step by 128 / 64 / 32 bytes mod 256 at W = 16 / 8 / 4, and at 4x4
  // the second image of a group starts 128 bytes further (measured 38-76 % of LDS cycles lost
  // to conflicts without the padding)
  static constexpr int ROWP = 3 * 2 * PLANE + (W == 16 ? 128 : W == 8 ? 64 : W == 4 ? 32 : 0);
  static constexpr int IMGP = (RB + 2) * ROWP + (W == 4 ? 192 : 0);
  static constexpr int BUF = E * IMGP;
  // double-buffered over K chunks; the epilogue's 4 x 4 KB transpose blocks live in the
  // buffer the last chunk consumed (buffer 1 at the latest)
  static constexpr int LDS = 2 * BUF > BUF + 16384 ? 2 * BUF : BUF + 16384;
  static constexpr int TB = E * RB * W;        // output positions per workgroup
  static constexpr int TW = TB / WT;           // output positions per wave
  static constexpr int NT = TW / 32;           // 32-wide t tiles per wave
  static constexpr int OB = WO * NA * 32;      // output channels per workgroup
  static constexpr int TPR = W / 4;            // threads per staged channel row (float4 each)
  static constexpr int NF4 = NR * CC * W / 4;  // float4 per chunk
  static constexpr int NST = (NF4 + 255) / 256;
  static_assert(TW % 32 == 0 && NT >= 1, "a wave must own whole 32-position tiles");
  static_assert(WO * WT == 4, "four waves per workgroup");
};

// E > 1: the tile stacks E whole images (H == RB), each staged with its own halo rows.
// Persistent: each workgroup walks tiles blockIdx.x, +gridDim.x, ...; the last K chunk of a
// tile stages the next tile's first chunk, so a tile's prologue latency hides under the
// previous tile's MFMAs.
// XF: the input transform is present (without it, staging skips the affine + clamp: the
// GraNd launches, two thirds of the conv time, have none)
// KX1: the stem layout (cin <= kStemCin, dd_conv3x3_pack): the three kx shifts of the cin
// input channels are staged as 3 cin pseudo-channels k = kx cin + c of the kx = 1 image, so a
// tap row is one K step of 16 (k, c) pairs instead of three mostly-zero ones: a third of the
// MFMAs, B-fragment reads and staging stores.
// PW: the padded-width form of conv3x3_r2_kernel (see there), here for the 64-wide tile of the
// ImageNet-stem network's 56x56 maps (64 outputs: the narrow 64-output workgroup)
template <int W, int RB, int E, int NA, int WO, int XF, bool KX1, int EPI = 0, int PW = 0>
__global__ __launch_bounds__(256, NA == 1 ? 2 : 1) void conv3x3_kernel(const Args A) {
  using C = Cfg<W, RB, E, NA, WO>;
  constexpr int NT = C::NT;
  constexpr bool F16 = (EPI & kEpiF16) != 0;
  static_assert(!PW || (XF <= kXfAffine && !KX1 && (EPI & ~kEpiF16) == (kEpiSpec | kEpiStats)),
                "padded-width tiles: the statistics epilogue with an optional BN staging only");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = A.H, cin = A.cin, cout = A.cout;
  const int64_t B = A.B;
  const float* __restrict__ x = A.x;
  const int WG = PW ? A.wg : W;
  const int HW = H * WG;
  const int HWP = PW ? A.n_tb * RB * W : HW;  // the padded plane (BN-partial layout)
  const int ntiles = A.n_tiles;
  stagger_start(A.stagger);

  // wave-uniform indices in SGPRs (weight addresses are then a scalar base + lane offset)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wo = wv % WO, wt = wv / WO, h = lane >> 5;

  struct Tile {
    int64_t b, grp;
    int ob, tb, o0, y0, xf_base, ob32;
  };
  auto decode = [&](int tile) {
    Tile T;
    int bid = tile;
    T.ob = bid % A.n_ob;
    bid /= A.n_ob;
    T.tb = bid % A.n_tb;
    T.b = (int64_t)(bid / A.n_tb) * E;
    T.o0 = T.ob * C::OB;
    T.y0 = T.tb * RB;
    // BN group of the tile (group_size % E == 0, so the E images share it)
    T.grp = T.b / A.gsize;
    T.xf_base = (int)(T.grp * cin);
    T.ob32 = (T.o0 >> 5) + wo * NA;  // the wave's first 32-o block
    return T;
  };

  // ---- staging of one K chunk (16 input channels x NR rows) into buffer `buf`
  float4 ra[C::NST];
  // a thread stages the same channel in every round k (256 threads cover whole channel-row
  // groups), so the per-channel affine is one value per thread
  static_assert(256 % (C::TPR * CC) == 0, "a thread's staged channel must not depend on k");
  float xs = 1.f, xt = 0.f;
  bool va[C::NST];
  // the fused residual-unit input (XF >= kXfOut): residual values and affine, and where the
  // staged values of this chunk go (buffer offsets past the range are dropped)
  float4 rv[C::NST];
  float rs = 1.f, rt = 0.f;
  __amdgpu_buffer_rsrc_t xo_rsrc;
  int xo_base = 0;
  bool xo_tile = false;
  auto load_chunk = [&](const Tile& T, int c0) {
    // buffer loads over the tile's images: a 32-bit lane offset, no clamping (an offset outside
    // the range reads zeros; lanes outside the image rows or channels are masked by va)
    const int64_t left = (B - T.b) * cin * HW * 4;
    const uint32_t range = (uint32_t)(left < 0x7fffffff ? left : 0x7fffffff);
    const __amdgpu_buffer_rsrc_t xr = buffer_rsrc(x + (size_t)T.b * cin * HW, range);
    const int ubase = c0 * HW * 4;
    __amdgpu_buffer_rsrc_t rr_rsrc;
    if constexpr (XF >= kXfOut) {
      xo_rsrc = buffer_rsrc(A.xout + (size_t)T.b * cin * HW, range);
      xo_base = ubase + (T.y0 - 1) * W * 4;
      xo_tile = T.o0 == 0;  // the output-channel block 0 tiles write the unit output once
      if constexpr (XF >= kXfOutRes) rr_rsrc = buffer_rsrc(A.xres + (size_t)T.b * cin * HW, range);
    }
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {
      const int q = tid + 256 * k;
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const int e = sr / (RB + 2), rr = sr - e * (RB + 2);
      const int ir = T.y0 - 1 + rr, cg = c0 + c;
      va[k] = q < C::NF4 && ir >= 0 && ir < H && cg < cin && T.b + e < B &&
              (!PW || x4 * 4 < WG);
      // the halo rows outside the image re-read the nearest image row (masked; already in
      // cache) instead of a neighbouring channel's row
      const int irc = ir < 0 ? 0 : (ir >= H ? H - 1 : ir);
      const int xoff = ubase + ((e * cin + c) * HW + irc * WG + x4 * 4) * 4;
      if constexpr (PW == 2) {
        ra[k] = make_float4(
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, xoff, 0, 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, xoff + 4, 0, 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, xoff + 8, 0, 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, xoff + 12, 0, 0)));
      } else {
        ra[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff, 0, 0));
      }
      if constexpr (XF >= kXfOutRes)
        rv[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                               rr_rsrc, ubase + ((e * cin + c) * HW + irc * W + x4 * 4) * 4,
                                               0, 0));
    }
    if constexpr (XF != kXfNone) {
      const int cg = c0 + (tid / C::TPR) % CC;
      const int xi = T.xf_base + (cg < cin ? cg : cin - 1);
      xs = A.in_scale[xi];
      xt = A.in_shift[xi];
      if constexpr (XF == kXfOutResAff) {
        rs = A.xres_scale[xi];
        rt = A.xres_shift[xi];
      }
    }
  };
  auto store_chunk = [&](int buf) {
    char* base0 = smem + buf * C::BUF;
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {
      const int q = tid + 256 * k;
      if (C::NF4 % 256 != 0 && k == C::NST - 1 && q >= C::NF4) continue;  // wave-uniform
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);  // staged row
      const int se = sr / (RB + 2), rr = sr - se * (RB + 2);
      float4 v = ra[k];
      // input transform (BN affine + ReLU of the producer; identity by default); padding and
      // out-of-range rows stay exact zeros
      if constexpr (XF != kXfNone) v = stage_transform<XF>(v, xs, xt, rv[k], rs, rt, A.in_floor);
      v = keep_if(v, va[k]);
      if constexpr (PW == 2) v = keep_cols(v, WG - x4 * 4);
      if constexpr (XF >= kXfOut) {
        // the unit output, once: interior rows (not the halo) of valid lanes of block-0 tiles
        const bool wr = xo_tile && va[k] && rr >= 1 && rr <= RB;
        const int off = xo_base + ((se * cin + c) * HW + rr * W + x4 * 4) * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), xo_rsrc,
                                               wr ? off : (int)0x80000000, 0, 0);
      }
      // bf16 hi / lo of the three kx shifts; the halo columns come from the neighbouring lanes
      // of the row (DPP row shifts), a row's first / last lane takes the zero padding
      uint2 hs[3], ls[3];
      split_shift3<F16>(v, x4 == 0, x4 == C::TPR - 1, hs, ls);
      if constexpr (KX1) {
        // channel c < cin fills pseudo-channels kx cin + c of image 1; channels c >= 3 cin
        // write their zeros (padding); the rest are filled by the first cin channels
        const int cin = A.cin;
        if (c < cin) {
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            char* p = base0 + se * C::IMGP + rr * C::ROWP + 2 * C::PLANE +
                      (kx * cin + c) * C::XS + x4 * 8;
            *reinterpret_cast<uint2*>(p) = hs[kx];
            *reinterpret_cast<uint2*>(p + C::PLANE) = ls[kx];
          }
        } else if (c >= 3 * cin) {
          char* p = base0 + se * C::IMGP + rr * C::ROWP + 2 * C::PLANE + c * C::XS + x4 * 8;
          *reinterpret_cast<uint2*>(p) = hs[1];
          *reinterpret_cast<uint2*>(p + C::PLANE) = ls[1];
        }
      } else {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          char* p = base0 + se * C::IMGP + rr * C::ROWP + (kx * 2) * C::PLANE + c * C::XS +
                    x4 * 8;
          *reinterpret_cast<uint2*>(p) = hs[kx];
          *reinterpret_cast<uint2*>(p + C::PLANE) = ls[kx];
        }
      }
    }
  };

  // ---- weights of one chunk: NA blocks x 9 taps x hi|lo fragments, 16 B per lane.  The pack
  // is fragment-major ([chunk][32-o block][tap][hi|lo][lane][8]), so each fragment load is one
  // contiguous 1 KB wave access.
  bf16x8 wa[NA][18];
  const int nob32 = A.op >> 5;
  const __bf16* __restrict__ wpack = A.wpack;
  auto load_w_taps = [&](int ob32, int kc, int tap0, int ntap) {
    // constant trip counts, so the loops always unroll and wa stays in registers (the tap
    // range folds at every call site)
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const __bf16* base = wpack + ((size_t)(kc * nob32 + ob32 + a) * 18) * 512 + lane * 8;
#pragma unroll
      for (int i = 0; i < 18; ++i)
        if (i >= 2 * tap0 && i < 2 * (tap0 + ntap) && (!KX1 || (i >> 1) % 3 == 1))
          wa[a][i] = *reinterpret_cast<const bf16x8*>(base + i * 512);
    }
  };

  // per-lane transposed-read geometry: lane 4q+p of each 16-lane group supplies row q,
  // columns 4p..4p+3 of a 4 x 16 block; the group's 16 columns are t = 16*(g&1) + 0..15
  const int q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
  int tr_yo[NT], tr_xo[NT];  // LDS offset of the tap-(0,*) input row, x offset
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int t = wt * C::TW + n * 32 + 16 * g1 + 4 * p;
    const int e = t / (RB * W);
    tr_yo[n] = e * C::IMGP + ((t / W) % RB) * C::ROWP;
    tr_xo[n] = t % W;
  }

  floatx16 acc[NA][NT];

  // B fragments of one tap row ky: [kx][n][hi|lo]
  auto read_b = [&](const char* base, int ky, bf16x8 (&bf)[3][NT][2], int kxa = KX1 ? 1 : 0,
                    int kxb = KX1 ? 2 : 3) {
#pragma unroll
    for (int kx = KX1 ? 1 : 0; kx < (KX1 ? 2 : 3); ++kx)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        if (kx < kxa || kx >= kxb) continue;  // (constant after unrolling)
        const char* a = base + tr_yo[n] + ky * C::ROWP + (kx * 2) * C::PLANE +
                        (8 * h + q) * C::XS + tr_xo[n] * 2;
        bf[kx][n][0] = tr_read8(a, a + 4 * C::XS);
        bf[kx][n][1] = tr_read8(a + C::PLANE, a + C::PLANE + 4 * C::XS);
      }
  };
  auto mfma_row = [&](int ky, const bf16x8 (&bf)[3][NT][2]) {
#pragma unroll
    for (int kx = KX1 ? 1 : 0; kx < (KX1 ? 2 : 3); ++kx)
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          const int tap = ky * 3 + kx;
          floatx16 d = acc[a][n];
          d = mfma16<F16>(wa[a][tap * 2], bf[kx][n][0], d);
          d = mfma16<F16>(wa[a][tap * 2], bf[kx][n][1], d);
          d = mfma16<F16>(wa[a][tap * 2 + 1], bf[kx][n][0], d);
          acc[a][n] = d;
        }
  };

  // ---- epilogue, per 32 x 32 fragment D[o][t] (lane holds column t = lane & 31, rows
  // o = (r&3) + 8(r>>2) + 4h): transposed through a wave-private 4 KB LDS block in the staging
  // buffer the last chunk consumed, so that each lane then owns 4 consecutive positions of
  // one channel (o = 8k + lane/8, t = 4(lane%8) + 0..3, k = 0..3) and the residual / mask
  // loads and the output stores are float4 (a quarter of the dword instructions, whose issue
  // rate bounds the epilogue).  Loads come from clamped addresses and only the stores are
  // predicated.  BN partials go per 32-position fragment column (the same stats layout for
  // every tile config); ReLU mask bits in this transposed order: bit 4k + j.
  auto epilogue = [&](const Tile& T, int tile, int free_buf) {
    const EpiFlags F = epi_flags<EPI>(A);
    const float* __restrict__ bias = A.bias;
    const float* __restrict__ residual = A.residual;
    const float* __restrict__ mask_src = A.mask_src;
    float* __restrict__ y = A.y;
    float* ep = reinterpret_cast<float*>(smem + free_buf * C::BUF) + wv * 1024;
    const int tl = lane & 7, ol = lane >> 3;
    // phase 1: every operand load of every fragment is issued before any is used (the main
    // loop's registers are free here), so the tile pays one memory round trip, not one per
    // fragment.  Each pointer test is hoisted out of the element loops (a select between a
    // load and a constant inside one makes hipcc branch around every load and wait for it).
    size_t ibase[NT];
    bool vlan[NT];
    float in_stat[NT];
    int ncol[NT];  // PW = 2: columns of the lane's quad inside the image (>= 4: all)
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int tt = wt * C::TW + n * 32 + 4 * tl;
      const int e = tt / (RB * W);
      int t = T.y0 * W + tt % (RB * W);
      bool in_img = true;
      if constexpr (PW) {
        const int rem = tt % (RB * W), row = T.y0 + rem / W, col = rem % W;
        in_img = row < H && col < WG;
        ncol[n] = WG - col;
        t = in_img ? row * WG + col : 0;
      }
      vlan[n] = T.b + e < B && in_img;
      in_stat[n] = (T.b + e < A.n_stat && in_img) ? 1.f : 0.f;
      const int64_t be = T.b + e < B ? T.b + e : B - 1;
      ibase[n] = (size_t)be * cout * HW + t;
    }
    int off[NA][4];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int o = T.o0 + (wo * NA + a) * 32 + ol + 8 * k;
        off[a][k] = (o < cout ? o : cout - 1) * HW;
      }
    float4 res[NA][NT][4];
    // ReLU-backward mask as bits (bit 4 k + j: element j of row group k passes): from the
    // fragment-order words directly, or from the float mask (mask_src > 0) when loaded
    unsigned mbits[NA][NT];
    float bia[NA][4];
    if (F.res) {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            res[a][n][k] = *reinterpret_cast<const float4*>(residual + ibase[n] + off[a][k]);
    } else {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int k = 0; k < 4; ++k) res[a][n][k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (F.msrc) {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          unsigned mb = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float4 mk = *reinterpret_cast<const float4*>(mask_src + ibase[n] + off[a][k]);
            mb |= ((mk.x > 0.f ? 1u : 0u) | (mk.y > 0.f ? 2u : 0u) | (mk.z > 0.f ? 4u : 0u) |
                   (mk.w > 0.f ? 8u : 0u)) << (4 * k);
          }
          mbits[a][n] = mb;
        }
    } else {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const size_t fidx = ((((size_t)tile * 4 + wv) * NA + a) * NT + n) * 64 + lane;
          mbits[a][n] = F.min ? A.mask_in[fidx] : 0xffffu;
        }
    }
    if (F.bias) {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int o = T.o0 + (wo * NA + a) * 32 + ol + 8 * k;
          bia[a][k] = bias[o < cout ? o : cout - 1];
        }
    } else {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int k = 0; k < 4; ++k) bia[a][k] = 0.f;
    }
    // phase 2, per fragment: transpose through LDS, combine, store
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        // fragment -> LDS [o][t] (two 32-lane halves write rows 4 apart: a 2-way conflict
        // that a ds_write_b32 absorbs), then rows back as float4
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ep[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + (lane & 31)] =
              F16 ? acc[a][n][r] * A.acc_scale : acc[a][n][r];
        asm volatile("" ::: "memory");  // LDS is in order within a wave; keep the compiler so
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] = *reinterpret_cast<const float4*>(ep + (8 * k + ol) * 32 + 4 * tl);
        asm volatile("" ::: "memory");
        const int tt0 = wt * C::TW + n * 32;  // the fragment's first position in the tile
        const int ob = T.o0 + (wo * NA + a) * 32 + ol;
        unsigned obits = 0;
        // BN partials of this fragment's channels ob + 8 k: one base, a constant stride
        float* sp = nullptr;
        if (F.stats) {
          const int pi = (int)(((T.b + tt0 / (RB * W) - T.grp * A.gsize) * HWP + T.y0 * W +
                                tt0 % (RB * W)) >> 5);
          sp = A.stats + (((size_t)T.grp * cout + ob) * A.tiles_per_group + pi) * 2;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float f[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
          const float4 rk = res[a][n][k];
          const float rs[4] = {rk.x, rk.y, rk.z, rk.w};
          float s_ = 0.f, q_ = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float u = f[j] + bia[a][k];
            if (F.res) u += rs[j];
            if (F.relu) u = nmax(u, 0.f);
            if ((F.msrc || F.min) && !((mbits[a][n] >> (4 * k + j)) & 1u)) u = 0.f;
            f[j] = u;
            obits |= (u > 0.f ? 1u : 0u) << (4 * k + j);
            const float us = (PW == 2 && j >= ncol[n]) ? 0.f : u * in_stat[n];
            s_ += us;
            q_ += us * us;
          }
          const int o = ob + 8 * k;
          if constexpr (PW == 2) {
            if (vlan[n] && o < cout) {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (j < ncol[n]) y[ibase[n] + off[a][k] + j] = f[j];
            }
          } else if (vlan[n] && o < cout) {
            store_out4(y + ibase[n] + off[a][k], f[0], f[1], f[2], f[3]);
          }
          if (F.stats) {
            // the 8 lanes of one channel hold its 32 positions of this fragment
            s_ = sum8(s_);
            q_ = sum8(q_);
            if (tl == 0 && o < cout)
              *reinterpret_cast<float2*>(sp + k * 16 * A.tiles_per_group) = make_float2(s_, q_);
          }
        }
        if (F.mout) {
          const size_t fidx = ((((size_t)tile * 4 + wv) * NA + a) * NT + n) * 64 + lane;
          A.mask_out[fidx] = (uint16_t)obits;
        }
      }
  };

  const int nchunks = (cin + CC - 1) / CC;
  int tile = A.xcd ? (int)xcd_order(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  Tile T = decode(tile);
  load_chunk(T, 0);
  // the first tile's weights in tap-row order, fenced: the waitcnt pass merges this entry
  // path with the loop's back edge, where row 0's weights are the oldest loads in flight; with
  // the scheduler free to issue row 0 last here, every chunk's first MFMA waited for the
  // previous chunk's row-2 weights (vmcnt(8) instead of vmcnt(22) in the EL2N-stats variant)
  load_w_taps(T.ob32, 0, 0, 3);
  __builtin_amdgcn_sched_barrier(0);
  load_w_taps(T.ob32, 0, 3, 3);
  __builtin_amdgcn_sched_barrier(0);
  load_w_taps(T.ob32, 0, 6, 3);
  __builtin_amdgcn_sched_barrier(0);
  store_chunk(0);
  __syncthreads();
  int g = 0;  // chunks processed by this workgroup: LDS buffer parity
  for (;;) {
    const int tile_n = tile + (int)gridDim.x;
    const bool has_next = tile_n < ntiles;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[a][n] = floatx16{0};
    // one K chunk; wload = false on a tile's last chunk, whose prefetch target is the next
    // tile's first chunk: its activations are staged now, its weights are loaded after the
    // epilogue (held in VGPRs across the epilogue they would spill)
    auto chunk = [&](const Tile& Tp, int kn, bool wload) {
      const int cur = g & 1;
      load_chunk(Tp, kn * CC);
      const char* base = smem + cur * C::BUF;
      bf16x8 b0[3][NT][2], b1[3][NT][2];
      // ROW0 (narrow tiles): only tap (0, 0)'s fragments are read before the first MFMA; the
      // row's other two taps are read between its first MFMAs, ahead of row 1's reads (with
      // all 24 row-0 reads outstanding the first MFMA waited for every one of them: the
      // LDS counter holds 15)
      constexpr bool ROW0 = NA == 1 && !KX1;
      read_b(base, 0, b0, KX1 ? 1 : 0, ROW0 ? 1 : (KX1 ? 2 : 3));
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (ROW0) read_b(base, 0, b0, 1, 3);
      // tap row 0 MFMAs | row 1 reads | next chunk's row-0 weights
      read_b(base, 1, b1);
      mfma_row(0, b0);
      if (wload) load_w_taps(Tp.ob32, kn, 0, 3);
#pragma unroll
      for (int i = 0; i < (KX1 ? 1 : 3) * NT; ++i) {
        if constexpr (ROW0) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        } else if constexpr (NA == 1) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // tap row 1 MFMAs | row 2 reads | next chunk's row-1 weights
      read_b(base, 2, b0);
      mfma_row(1, b1);
      if (wload) load_w_taps(Tp.ob32, kn, 3, 3);
#pragma unroll
      for (int i = 0; i < (KX1 ? 1 : 3) * NT; ++i) {
        if constexpr (NA == 1) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
          __builtin_amdgcn_sched_group_barrier(0x020, 2, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // tap row 2 MFMAs | next chunk staged into the idle buffer | next chunk's row-2 weights
      mfma_row(2, b0);
      store_chunk(cur ^ 1);
      if (wload) load_w_taps(Tp.ob32, kn, 6, 3);
#pragma unroll
      for (int i = 0; i < (KX1 ? 3 : 9) * NT * NA; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
        __builtin_amdgcn_sched_group_barrier(0x002, NA == 1 ? 5 : 3, 2);
        __builtin_amdgcn_sched_group_barrier(0x080, 1, 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      ++g;
    };
    // wide tiles: two chunks per iteration.  The waitcnt pass loses the order of loads
    // carried around the loop back-edge and then waits for the previous chunk's row-2 weight
    // loads in the middle of row 0; inside one iteration its counts are exact (+1-2 % at 4x4;
    // the narrow tiles spill and lose 2-25 % this way, profiles/r01_v17/experiments)
    int kc = 0;
    if constexpr (NA == 2) {
      for (; kc + 2 < nchunks; kc += 2) {
        chunk(T, kc + 1, true);
        chunk(T, kc + 2, true);
      }
    }
    for (; kc + 1 < nchunks; ++kc) chunk(T, kc + 1, true);
    // last chunk: stage the next tile's first chunk (or, on the last tile, a clamped re-load
    // into the idle buffer that is never read)
    const Tile Tn = has_next ? decode(tile_n) : T;
    chunk(Tn, has_next ? 0 : nchunks - 1, false);
    // the next tile's tap-row-0 weights load under the epilogue (its first MFMAs need them
    // right after it); the other 6 taps after it, under those MFMAs (held across the
    // epilogue they would spill).  Both loads, and the barrier, run on the last tile too (a
    // harmless re-load of its own weights), and the exit test comes after them: the CFG
    // structurizer routes a `break` through the loop latch, and a path that loaded row 0 but
    // skipped rows 1-2 made the waitcnt pass assume row 0's weights were the newest loads in
    // flight at every chunk's first MFMA (vmcnt(10) where vmcnt(22) is exact)
    load_w_taps(Tn.ob32, 0, 0, 3);
    // the last chunk read buffer (g - 1) & 1; the next tile's first chunk sits in g & 1
    epilogue(T, tile, (g - 1) & 1);
    __syncthreads();  // the next tile's first staging store overwrites the epilogue's block
    load_w_taps(Tn.ob32, 0, 3, 6);
    if (!has_next) break;
    tile = tile_n;
    T = Tn;
  }
}

// Tiles at two workgroups per CU with whole-row register blocking ("r2"): a wave owns NA 32-o
// blocks x NT 32-position tiles (the default form: NA = 1, NT = 4, four waves along o), so each
// weight fragment loaded from L2 feeds NT column tiles.  What keeps it within the 256-register
// budget with a long weight prefetch:
//   * weights are held one tap row at a time in two register sets instead of a chunk's 9 taps:
//     after a tap's MFMAs its slot is refilled with the same kx two tap rows ahead (5 taps of
//     MFMAs of prefetch distance; row r + 2 of a chunk is row r - 1 of the next);
//   * B fragments are read one tap ahead, column tile by column tile;
//   * the epilogue takes the fragments two at a time.
// Row r of chunk c uses set (c + r) & 1 and chunk c stages into LDS buffer c & 1, so two chunks
// are one loop body with every index compile-time; a tile's chunk count is made even (a zero
// chunk when cin / 16 is odd: its staged rows are zeros, its weight loads clamped).  Staging
// (the stem layout included: its chunks run the kx = 1 taps only), fragment order, mask and
// statistics layouts are those of conv3x3_kernel.
// SB: one LDS staging buffer (for tiles whose double buffer would not fit two per CU): a
// chunk's prefetched rows are stored between two barriers after its MFMAs, so the staging
// overlaps the other workgroup's MFMAs instead of its own; the epilogue blocks sit past it.
// PW (padded width): the EL2N statistics launches at a width that is not a tile width (the
// ImageNet-stem network's 28 / 14 / 7 maps).  The tile keeps its W-wide LDS image; the image in
// memory is WG = A.wg <= W wide, and its columns >= WG and rows >= H (the last row block may
// overhang) are staged as zeros and never stored or counted.  PW = 1: WG % 4 == 0 (float4 loads
// and stores, as the native tiles); PW = 2: any WG (rows are not 16-byte aligned: dword loads
// and stores).  BN partials keep the native layout on the padded grid (32 positions each).
template <int W, int RB, int E, int NA, int WO, int XF, bool KX1, bool SB, int EPI = 0, int PW = 0>
__global__ __launch_bounds__(256, 2) void conv3x3_r2_kernel(const Args A) {
  using C = Cfg<W, RB, E, NA, WO>;
  constexpr int NT = C::NT;
  constexpr bool F16 = (EPI & kEpiF16) != 0;
  static_assert(!PW || (XF <= kXfAffine && !KX1 && !SB &&
                        (EPI & ~kEpiF16) == (kEpiSpec | kEpiStats)),
                "padded-width tiles: the statistics epilogue with an optional BN staging only");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = A.H, cin = A.cin, cout = A.cout;
  const int64_t B = A.B;
  const float* __restrict__ x = A.x;
  const int WG = PW ? A.wg : W;
  const int HW = H * WG;
  const int HWP = PW ? A.n_tb * RB * W : HW;  // the padded plane (BN-partial layout)
  const int ntiles = A.n_tiles;
  stagger_start(A.stagger);

  // wave-uniform indices in SGPRs (weight addresses are then a scalar base + lane offset)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wo = wv % WO, wt = wv / WO, h = lane >> 5;

  struct Tile {
    int64_t b, grp;
    int tb, o0, y0, xf_base, ob32;
  };
  auto decode = [&](int tile) {
    Tile T;
    int bid = tile;
    const int ob = bid % A.n_ob;
    bid /= A.n_ob;
    T.tb = bid % A.n_tb;
    T.b = (int64_t)(bid / A.n_tb) * E;
    T.o0 = ob * C::OB;
    T.y0 = T.tb * RB;
    T.grp = T.b / A.gsize;
    T.xf_base = (int)(T.grp * cin);
    T.ob32 = (T.o0 >> 5) + wo * NA;
    return T;
  };

  // ---- staging (as conv3x3_kernel)
  float4 ra[C::NST];
  // a thread stages the same channel in every round k (256 threads cover whole channel-row
  // groups), so the per-channel affine is one value per thread
  static_assert(256 % (C::TPR * CC) == 0, "a thread's staged channel must not depend on k");
  float xs = 1.f, xt = 0.f;
  bool va[C::NST];
  // the fused residual-unit input (XF >= kXfOut): residual values and affine, and where the
  // staged values of this chunk go (buffer offsets past the range are dropped)
  float4 rv[C::NST];
  float rs = 1.f, rt = 0.f;
  __amdgpu_buffer_rsrc_t xo_rsrc;
  int xo_base = 0;
  bool xo_tile = false;
  auto load_chunk = [&](const Tile& T, int c0) {
    // buffer loads over the tile's images: a 32-bit lane offset, no clamping (an offset outside
    // the range reads zeros; lanes outside the image rows or channels are masked by va)
    const int64_t left = (B - T.b) * cin * HW * 4;
    const uint32_t range = (uint32_t)(left < 0x7fffffff ? left : 0x7fffffff);
    const __amdgpu_buffer_rsrc_t xr = buffer_rsrc(x + (size_t)T.b * cin * HW, range);
    const int ubase = c0 * HW * 4;
    __amdgpu_buffer_rsrc_t rr_rsrc;
    if constexpr (XF >= kXfOut) {
      xo_rsrc = buffer_rsrc(A.xout + (size_t)T.b * cin * HW, range);
      xo_base = ubase + (T.y0 - 1) * W * 4;
      xo_tile = T.o0 == 0;  // the output-channel block 0 tiles write the unit output once
      if constexpr (XF >= kXfOutRes) rr_rsrc = buffer_rsrc(A.xres + (size_t)T.b * cin * HW, range);
    }
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {
      const int q = tid + 256 * k;
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const int e = sr / (RB + 2), rr = sr - e * (RB + 2);
      const int ir = T.y0 - 1 + rr, cg = c0 + c;
      va[k] = q < C::NF4 && ir >= 0 && ir < H && cg < cin && T.b + e < B &&
              (!PW || x4 * 4 < WG);
      // the halo rows outside the image re-read the nearest image row (masked; already in
      // cache) instead of a neighbouring channel's row
      const int irc = ir < 0 ? 0 : (ir >= H ? H - 1 : ir);
      const int xoff = ubase + ((e * cin + c) * HW + irc * WG + x4 * 4) * 4;
      if constexpr (PW == 2) {
        // (columns past the row read the next row, or zeros past the range: zeroed at staging)
        ra[k] = make_float4(
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, xoff, 0, 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, xoff + 4, 0, 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, xoff + 8, 0, 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, xoff + 12, 0, 0)));
      } else {
        ra[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff, 0, 0));
      }
      if constexpr (XF >= kXfOutRes)
        rv[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                               rr_rsrc, ubase + ((e * cin + c) * HW + irc * W + x4 * 4) * 4,
                                               0, 0));
    }
    if constexpr (XF != kXfNone) {
      const int cg = c0 + (tid / C::TPR) % CC;
      const int xi = T.xf_base + (cg < cin ? cg : cin - 1);
      xs = A.in_scale[xi];
      xt = A.in_shift[xi];
      if constexpr (XF == kXfOutResAff) {
        rs = A.xres_scale[xi];
        rt = A.xres_shift[xi];
      }
    }
  };
  auto store_chunk = [&](int buf) {
    char* base0 = smem + (SB ? 0 : buf) * C::BUF;
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {
      const int q = tid + 256 * k;
      if (C::NF4 % 256 != 0 && k == C::NST - 1 && q >= C::NF4) continue;  // wave-uniform
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const int se = sr / (RB + 2), rr = sr - se * (RB + 2);
      float4 v = ra[k];
      // input transform (BN affine + ReLU of the producer; identity by default); padding and
      // out-of-range rows stay exact zeros
      if constexpr (XF != kXfNone) v = stage_transform<XF>(v, xs, xt, rv[k], rs, rt, A.in_floor);
      v = keep_if(v, va[k]);
      if constexpr (PW == 2) v = keep_cols(v, WG - x4 * 4);
      if constexpr (XF >= kXfOut) {
        // the unit output, once: interior rows (not the halo) of valid lanes of block-0 tiles
        const bool wr = xo_tile && va[k] && rr >= 1 && rr <= RB;
        const int off = xo_base + ((se * cin + c) * HW + rr * W + x4 * 4) * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), xo_rsrc,
                                               wr ? off : (int)0x80000000, 0, 0);
      }
      // bf16 hi / lo of the three kx shifts; the halo columns come from the neighbouring lanes
      // of the row (DPP row shifts), a row's first / last lane takes the zero padding
      uint2 hs[3], ls[3];
      split_shift3<F16>(v, x4 == 0, x4 == C::TPR - 1, hs, ls);
      if constexpr (KX1) {
        // the stem layout: channel c < cin fills pseudo-channels kx cin + c of image 1,
        // channels c >= 3 cin write their zeros
        const int cin = A.cin;
        if (c < cin) {
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            char* p = base0 + se * C::IMGP + rr * C::ROWP + 2 * C::PLANE +
                      (kx * cin + c) * C::XS + x4 * 8;
            *reinterpret_cast<uint2*>(p) = hs[kx];
            *reinterpret_cast<uint2*>(p + C::PLANE) = ls[kx];
          }
        } else if (c >= 3 * cin) {
          char* p = base0 + se * C::IMGP + rr * C::ROWP + 2 * C::PLANE + c * C::XS + x4 * 8;
          *reinterpret_cast<uint2*>(p) = hs[1];
          *reinterpret_cast<uint2*>(p + C::PLANE) = ls[1];
        }
      } else {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          char* p = base0 + se * C::IMGP + rr * C::ROWP + (kx * 2) * C::PLANE + c * C::XS +
                    x4 * 8;
          *reinterpret_cast<uint2*>(p) = hs[kx];
          *reinterpret_cast<uint2*>(p + C::PLANE) = ls[kx];
        }
      }
    }
  };

  // ---- weights: two sets of one tap row each, [set][a][kx][hi|lo]
  const int nkc = (cin + CC - 1) / CC;
  const int nk2 = (nkc + 1) & ~1;
  bf16x8 ws[2][NA][3][2];
  const int nob32 = A.op >> 5;
  const __bf16* __restrict__ wpack = A.wpack;
  // (the stem layout uses the kx = 1 taps only)
  auto load_tap = [&](int set, int ob32, int kc, int ky, int kx) {
    if (KX1 && kx != 1) return;
    const int k = kc < nkc ? kc : nkc - 1;  // the zero chunk's weights: any finite values
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const __bf16* base =
          wpack + ((size_t)(k * nob32 + ob32 + a) * 18 + (ky * 3 + kx) * 2) * 512 + lane * 8;
      ws[set][a][kx][0] = *reinterpret_cast<const bf16x8*>(base);
      ws[set][a][kx][1] = *reinterpret_cast<const bf16x8*>(base + 512);
    }
  };

  const int q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
  int tr_off[NT];  // LDS offset of this lane's tap-(0, 0) B read, hi plane
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int t = wt * C::TW + n * 32 + 16 * g1 + 4 * p;
    const int e = t / (RB * W);
    tr_off[n] = e * C::IMGP + ((t / W) % RB) * C::ROWP + (8 * h + q) * C::XS + (t % W) * 2;
  }

  floatx16 acc[NA][NT];
  // B fragments [n][hi|lo], one tap at a time: column tile n of the next tap is read as soon as
  // this tap's MFMAs on column tile n have issued (NA x 3 MFMAs of distance)
  bf16x8 bb[NT][2];
  auto read_b = [&](int buf, int ky, int kx, int n) {
    const char* a = smem + (SB ? 0 : buf) * C::BUF + ky * C::ROWP + (kx * 2) * C::PLANE + tr_off[n];
    bb[n][0] = tr_read8(a, a + 4 * C::XS);
    bb[n][1] = tr_read8(a + C::PLANE, a + C::PLANE + 4 * C::XS);
  };
  auto mfma_b = [&](int set, int kx, int n) {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      floatx16 d = acc[a][n];
      d = mfma16<F16>(ws[set][a][kx][0], bb[n][0], d);
      d = mfma16<F16>(ws[set][a][kx][0], bb[n][1], d);
      d = mfma16<F16>(ws[set][a][kx][1], bb[n][0], d);
      acc[a][n] = d;
    }
  };

  // ---- epilogue (conv3x3_kernel's, one A block at a time: the operands of one block are
  // loaded, then combined and stored, so the live registers stay within the budget)
  auto epilogue = [&](const Tile& T, int tile, int free_buf) {
    const EpiFlags F = epi_flags<EPI>(A);
    const float* __restrict__ bias = A.bias;
    const float* __restrict__ residual = A.residual;
    const float* __restrict__ mask_src = A.mask_src;
    float* __restrict__ y = A.y;
    float* ep = reinterpret_cast<float*>(smem + (SB ? 1 : free_buf) * C::BUF) + wv * 1024;
    const int tl = lane & 7, ol = lane >> 3;
    size_t ibase[NT];
    bool vlan[NT];
    float in_stat[NT];
    int ncol[NT];  // PW = 2: columns of the lane's quad inside the image (>= 4: all)
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int tt = wt * C::TW + n * 32 + 4 * tl;
      const int e = tt / (RB * W);
      int t = T.y0 * W + tt % (RB * W);
      bool in_img = true;
      if constexpr (PW) {
        const int rem = tt % (RB * W), row = T.y0 + rem / W, col = rem % W;
        in_img = row < H && col < WG;
        ncol[n] = WG - col;
        t = in_img ? row * WG + col : 0;
      }
      vlan[n] = T.b + e < B && in_img;
      in_stat[n] = (T.b + e < A.n_stat && in_img) ? 1.f : 0.f;
      const int64_t be = T.b + e < B ? T.b + e : B - 1;
      ibase[n] = (size_t)be * cout * HW + t;
    }
    // fragments in groups of NG along n: one group's operands are loaded, then combined and
    // stored, so the live registers stay within the budget
    constexpr int NG = NT < 2 ? NT : 2;
    static_for<NA * (NT / NG)>([&](auto Gc) {
      constexpr int a = decltype(Gc)::value / (NT / NG);
      constexpr int n0 = (decltype(Gc)::value % (NT / NG)) * NG;
      int off[4];
      float bia[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int o = T.o0 + (wo * NA + a) * 32 + ol + 8 * k;
        const int oc = o < cout ? o : cout - 1;
        off[k] = oc * HW;
        bia[k] = F.bias ? bias[oc] : 0.f;
      }
      float4 res[NG][4];
      unsigned mbits[NG];  // ReLU-backward mask bits, as in conv3x3_kernel
      if (F.res) {
#pragma unroll
        for (int m = 0; m < NG; ++m)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            res[m][k] = *reinterpret_cast<const float4*>(residual + ibase[n0 + m] + off[k]);
      } else {
#pragma unroll
        for (int m = 0; m < NG; ++m)
#pragma unroll
          for (int k = 0; k < 4; ++k) res[m][k] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (F.msrc) {
#pragma unroll
        for (int m = 0; m < NG; ++m) {
          unsigned mb = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float4 mk = *reinterpret_cast<const float4*>(mask_src + ibase[n0 + m] + off[k]);
            mb |= ((mk.x > 0.f ? 1u : 0u) | (mk.y > 0.f ? 2u : 0u) | (mk.z > 0.f ? 4u : 0u) |
                   (mk.w > 0.f ? 8u : 0u)) << (4 * k);
          }
          mbits[m] = mb;
        }
      } else {
#pragma unroll
        for (int m = 0; m < NG; ++m) {
          const size_t fidx = ((((size_t)tile * 4 + wv) * NA + a) * NT + n0 + m) * 64 + lane;
          mbits[m] = F.min ? A.mask_in[fidx] : 0xffffu;
        }
      }
#pragma unroll
      for (int m = 0; m < NG; ++m) {
        const int n = n0 + m;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ep[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + (lane & 31)] =
              F16 ? acc[a][n][r] * A.acc_scale : acc[a][n][r];
        asm volatile("" ::: "memory");
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] = *reinterpret_cast<const float4*>(ep + (8 * k + ol) * 32 + 4 * tl);
        asm volatile("" ::: "memory");
        const int tt0 = wt * C::TW + n * 32;
        const int ob = T.o0 + (wo * NA + a) * 32 + ol;
        unsigned obits = 0;
        float* sp = nullptr;  // BN partials of channels ob + 8 k: one base, a constant stride
        if (F.stats) {
          const int pi = (int)(((T.b + tt0 / (RB * W) - T.grp * A.gsize) * HWP + T.y0 * W +
                                tt0 % (RB * W)) >> 5);
          sp = A.stats + (((size_t)T.grp * cout + ob) * A.tiles_per_group + pi) * 2;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float f[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
          const float4 rk = res[m][k];
          const float rs[4] = {rk.x, rk.y, rk.z, rk.w};
          float s_ = 0.f, q_ = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float u = f[j] + bia[k];
            if (F.res) u += rs[j];
            if (F.relu) u = nmax(u, 0.f);
            if ((F.msrc || F.min) && !((mbits[m] >> (4 * k + j)) & 1u)) u = 0.f;
            f[j] = u;
            obits |= (u > 0.f ? 1u : 0u) << (4 * k + j);
            const float us = (PW == 2 && j >= ncol[n]) ? 0.f : u * in_stat[n];
            s_ += us;
            q_ += us * us;
          }
          const int o = ob + 8 * k;
          if constexpr (PW == 2) {
            if (vlan[n] && o < cout) {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (j < ncol[n]) y[ibase[n] + off[k] + j] = f[j];
            }
          } else if (vlan[n] && o < cout) {
            store_out4(y + ibase[n] + off[k], f[0], f[1], f[2], f[3]);
          }
          if (F.stats) {
            s_ = sum8(s_);
            q_ = sum8(q_);
            if (tl == 0 && o < cout)
              *reinterpret_cast<float2*>(sp + k * 16 * A.tiles_per_group) = make_float2(s_, q_);
          }
        }
        if (F.mout) {
          const size_t fidx = ((((size_t)tile * 4 + wv) * NA + a) * NT + n) * 64 + lane;
          A.mask_out[fidx] = (uint16_t)obits;
        }
      }
    });
  };

// ---- one K chunk c of tile T (LDS buffer P = c & 1, weight sets (P + r) & 1): stages
  // (Ts, chunk ks) into the other buffer; tap row 0 refills its slots with row 2 of chunk c,
  // row 1 with row 0 of (Tw, chunk kw), row 2 (when w2) with row 1 of (Tw, kw)
  auto chunk = [&](auto Pc, auto W2c, const Tile& T, int c, const Tile& Ts, int ks,
                   const Tile& Tw, int kw) {
    constexpr int P = decltype(Pc)::value;
    load_chunk(Ts, ks * CC);
#if DD_R2_FENCE >= 1
    // fences keep the staging loads at the chunk start and each tap's weight loads behind
    // its MFMAs: unfenced, the scheduler sank a staging load next to its masking and waited
    // for it on the spot, and bunched the weight loads before the barrier
    __builtin_amdgcn_sched_barrier(0);
#endif
    // taps in order (the stem layout: the kx = 1 taps only, each one K step of 3 cin
    // pseudo-channels)
    constexpr int T0 = KX1 ? 1 : 0, TS = KX1 ? 3 : 1;
#pragma unroll
    for (int n = 0; n < NT; ++n) read_b(P, 0, T0, n);
    static_for<9>([&](auto Tc) {
      constexpr int t = decltype(Tc)::value;
      constexpr int ky = t / 3, kx = t % 3, set = (P + ky) & 1;
      if constexpr (!KX1 || kx == 1) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          mfma_b(set, kx, n);
          if constexpr (t + TS < 9) read_b(P, (t + TS) / 3, (t + TS) % 3, n);
        }
        if constexpr (ky == 0)
          load_tap(set, T.ob32, c, 2, kx);
        else if constexpr (ky == 1)
          load_tap(set, Tw.ob32, kw, 0, kx);
        else if constexpr (decltype(W2c)::value)
          load_tap(set, Tw.ob32, kw, 1, kx);
      }
      if constexpr (t == 6 && !SB) store_chunk(P ^ 1);
#if DD_R2_FENCE >= 2
      __builtin_amdgcn_sched_barrier(0);
#endif
    });
    if constexpr (SB) {
      __syncthreads();  // every wave is done reading the buffer
      store_chunk(0);
    }
    __syncthreads();
  };
  const std::integral_constant<int, 0> I0;
  const std::integral_constant<int, 1> I1;
  const std::true_type Y;
  const std::false_type N;

  int tile = A.xcd ? (int)xcd_order(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  Tile T = decode(tile);
  load_chunk(T, 0);
  static_for<3>([&](auto Kc) {
    load_tap(0, T.ob32, 0, 0, decltype(Kc)::value);
    load_tap(1, T.ob32, 0, 1, decltype(Kc)::value);
  });
  store_chunk(0);
  __syncthreads();
  for (;;) {
    const int tile_n = tile + (int)gridDim.x;
    const bool has_next = tile_n < ntiles;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[a][n] = floatx16{0};
    int c = 0;
    for (; c + 2 < nk2; c += 2) {
      chunk(I0, Y, T, c, T, c + 1, T, c + 1);
      chunk(I1, Y, T, c + 1, T, c + 2, T, c + 2);
    }
    // the last two chunks: the final one stages the next tile's first chunk (a clamped
    // re-load never read on the last tile) and loads its tap-row-0 weights; its row-1 weights
    // are loaded after the epilogue (held across it they would not fit)
    const Tile Tn = has_next ? decode(tile_n) : T;
    chunk(I0, Y, T, c, T, c + 1, T, c + 1);
    chunk(I1, N, T, c + 1, Tn, has_next ? 0 : nkc - 1, Tn, 0);
    epilogue(T, tile, 1);
    __syncthreads();  // the next tile's first staging store overwrites the epilogue's block
    // (on the last tile too, with the exit test after the loads: see conv3x3_kernel -- a
    // `break` before them reaches the latch with row 0 loaded and row 1 not, and the waitcnt
    // pass then waits for the newest weight loads at the start of every chunk)
    load_tap(1, Tn.ob32, 0, 1, 0);
    load_tap(1, Tn.ob32, 0, 1, 1);
    load_tap(1, Tn.ob32, 0, 1, 2);
    if (!has_next) break;
    tile = tile_n;
    T = Tn;
  }
}

// the dynamic-LDS attribute of one kernel instantiation, set once
template <auto K>
static void lds_attr(int bytes) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(K),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    done = true;
  }
}

// the epilogue of a launch as an EPI code (kEpiSpec | operations)
inline int epilogue_code(const Args& a) {
  return kEpiSpec | (a.bias ? kEpiBias : 0) | (a.residual ? kEpiRes : 0) |
         (a.relu ? kEpiRelu : 0) | (a.mask_src ? kEpiMsrc : 0) | (a.mask_in ? kEpiMin : 0) |
         (a.mask_out ? kEpiMout : 0) | (a.stats ? kEpiStats : 0);
}
// the launch shapes of the scoring passes, each compiled with its own epilogue:
//   EL2N forward        stats                         (staging transform or not; the stem)
//   GraNd forward       bias + ReLU + fragment mask   (+ residual: a block's second conv)
//   GraNd backward-data fragment mask in (+ residual) or fp32 mask (a head block's conv2^T)
constexpr int kE_Stats = kEpiSpec | kEpiStats;
constexpr int kE_Fwd = kEpiSpec | kEpiBias | kEpiRelu | kEpiMout;
constexpr int kE_FwdRes = kE_Fwd | kEpiRes;
constexpr int kE_Bwd = kEpiSpec | kEpiMin;
constexpr int kE_BwdRes = kE_Bwd | kEpiRes;
constexpr int kE_BwdSrc = kEpiSpec | kEpiMsrc;
// DD_CONV_EPI=0: every launch on the generic (run-time) epilogue, for A/B runs
inline bool epi_specialised() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DD_CONV_EPI");
    v = e ? atoi(e) != 0 : 1;
  }
  return v != 0;
}

// the staging mode of a launch (kXf*)
inline int xf_mode(const Args& a) {
  return !a.xf_mask ? kXfNone : !a.xout ? kXfAffine : !a.xres ? kXfOut
         : !a.xres_scale ? kXfOutRes : kXfOutResAff;
}

// go.template run<XF, KX1, EPI>() for the launch's (staging mode, stem layout, epilogue); the
// fused residual-unit input (EL2N forward, a unit's first conv) exists on the specialised
// statistics epilogue only
// FB: kEpiF16 for the fp16-operand launches, which exist for the EL2N statistics epilogue
// (every staging mode), the GraNd forward epilogues and the generic epilogue
template <bool SPEC, typename Go, bool FUSE, int FB>
static int dispatch_epi_t(const Args& a, Go& go) {
  const int code = epilogue_code(a);
  const int xm = xf_mode(a);
  if constexpr (FUSE) {
    if (xm >= kXfOut && code == kE_Stats && !a.kx1) {
      if (xm == kXfOut) return go.template run<kXfOut, false, kE_Stats | FB>();
      if (xm == kXfOutRes) return go.template run<kXfOutRes, false, kE_Stats | FB>();
      return go.template run<kXfOutResAff, false, kE_Stats | FB>();
    }
  }
  if (xm >= kXfOut) {
    set_error("dd_conv3x3_forward_unit_input: no fused-input kernel for this launch (stats "
              "epilogue on the scoring tiles only; see dd_conv3x3_unit_input_supported)");
    return DD_EINVAL;
  }
  if (SPEC && epi_specialised()) {
    const bool xf = a.xf_mask != 0, k1 = a.kx1 != 0;
    if (code == kE_Stats) {
      if (xf && !k1) return go.template run<true, false, kE_Stats | FB>();
      if (!xf && !k1) return go.template run<false, false, kE_Stats | FB>();
      if (!xf && k1) return go.template run<false, true, kE_Stats | FB>();
    }
    // the GraNd forward (folded BN: bias + ReLU + fragment mask, + residual) in either
    // operand type; the GraNd backward shapes in bf16 only (gradients leave fp16's range)
    if (!xf && code == kE_Fwd) {
      if (k1) return go.template run<false, true, kE_Fwd | FB>();
      return go.template run<false, false, kE_Fwd | FB>();
    }
    if (!xf && !k1 && code == kE_FwdRes) return go.template run<false, false, kE_FwdRes | FB>();
    if constexpr (FB == 0) {
      if (!xf && !k1) {
        if (code == kE_Bwd) return go.template run<false, false, kE_Bwd>();
        if (code == kE_BwdRes) return go.template run<false, false, kE_BwdRes>();
        if (code == kE_BwdSrc) return go.template run<false, false, kE_BwdSrc>();
      }
    }
  }
  if (a.kx1)
    return a.xf_mask ? go.template run<true, true, FB>() : go.template run<false, true, FB>();
  return a.xf_mask ? go.template run<true, false, FB>() : go.template run<false, false, FB>();
}
template <bool SPEC, typename Go, bool FUSE = SPEC>
static int dispatch_epi(const Args& a, Go& go) {
  return a.f16 ? dispatch_epi_t<SPEC, Go, FUSE, kEpiF16>(a, go)
               : dispatch_epi_t<SPEC, Go, FUSE, 0>(a, go);
}

// epilogue specialisation where the scoring passes run (the 32x32 narrow tile and the r2
// tiles); other tile configs (A/B families, odd channel counts) use the generic epilogue
template <int W, int RB, int E, int NA, int WO>
constexpr bool kSpecNarrow = W == 32 && RB == 4 && E == 1 && NA == 1 && WO == 2;

// launchers of one tile config for dispatch_epi
template <int W, int RB, int E, int NA, int WO>
struct GoNarrow {
  const Args& a;
  dim3 g;
  hipStream_t st;
  template <int XF, bool KX1, int EPI>
  int run() {
    constexpr auto K = &conv3x3_kernel<W, RB, E, NA, WO, XF, KX1, EPI>;
    lds_attr<K>(Cfg<W, RB, E, NA, WO>::LDS);
    K<<<g, 256, Cfg<W, RB, E, NA, WO>::LDS, st>>>(a);
    DD_CHECK_LAUNCH("dd_conv3x3_forward");
    return DD_OK;
  }
};
template <int W, int RB, int E, int NA, int WO, bool SB>
struct GoR2 {
  static constexpr int LDS = SB ? Cfg<W, RB, E, NA, WO>::BUF + 16384 : Cfg<W, RB, E, NA, WO>::LDS;
  const Args& a;
  dim3 g;
  hipStream_t st;
  template <int XF, bool KX1, int EPI>
  int run() {
    constexpr auto K = &conv3x3_r2_kernel<W, RB, E, NA, WO, XF, KX1, SB, EPI>;
    lds_attr<K>(LDS);
    K<<<g, 256, LDS, st>>>(a);
    DD_CHECK_LAUNCH("dd_conv3x3_forward");
    return DD_OK;
  }
};

template <int W, int RB, int E, int NA, int WO>
static int launch(Args a, hipStream_t st) {
  using C = Cfg<W, RB, E, NA, WO>;
  DD_REQUIRE(a.H % RB == 0, "dd_conv3x3_forward: H must be a multiple of the row block");
  DD_REQUIRE(a.gsize % E == 0, "dd_conv3x3_forward: group_size %d must be a multiple of %d "
             "(images per tile at %dx%d)", a.gsize, E, a.H, W);
  DD_REQUIRE(a.op % C::OB == 0, "dd_conv3x3_forward: padded outputs %d not a multiple of %d",
             a.op, C::OB);
  a.n_tb = a.H / RB;
  a.n_ob = a.op / C::OB;
  const int64_t ntiles = ceil_div(a.B, E) * a.n_tb * a.n_ob;
  DD_REQUIRE(ntiles < (1ll << 31), "dd_conv3x3_forward: too many tiles");
  a.n_tiles = (int)ntiles;
  // persistent: each resident workgroup walks tiles.  Wide tiles: one workgroup per CU.
  // Narrow tiles: two per CU where the K loop is short and a tile's prologue latency shows
  // (measured +5-10 % at the stem, +3 % at 64 channels, -4 % at 512: one tile per workgroup)
  const int64_t cap = NA == 2 ? device_cus() : a.cin <= 256 ? 2ll * device_cus() : ntiles;
  const int64_t grid = ntiles < cap ? ntiles : cap;
  GoNarrow<W, RB, E, NA, WO> go{a, dim3((unsigned)grid), st};
  return dispatch_epi<kSpecNarrow<W, RB, E, NA, WO>>(a, go);
}

template <int W, int RB, int E, int NA, int WO, bool SB = false>
static int launch_r2(Args a, hipStream_t st) {
  using C = Cfg<W, RB, E, NA, WO>;
  constexpr int LDS = SB ? C::BUF + 16384 : C::LDS;
  static_assert(2 * LDS <= 160 * 1024, "r2 tiles run two workgroups per CU");
  DD_REQUIRE(a.H % RB == 0, "dd_conv3x3_forward: H must be a multiple of the row block");
  DD_REQUIRE(a.gsize % E == 0, "dd_conv3x3_forward: group_size %d must be a multiple of %d "
             "(images per tile at %dx%d)", a.gsize, E, a.H, W);
  DD_REQUIRE(a.op % C::OB == 0, "dd_conv3x3_forward: padded outputs %d not a multiple of %d",
             a.op, C::OB);
  a.n_tb = a.H / RB;
  a.n_ob = a.op / C::OB;
  const int64_t ntiles = ceil_div(a.B, E) * a.n_tb * a.n_ob;
  DD_REQUIRE(ntiles < (1ll << 31), "dd_conv3x3_forward: too many tiles");
  a.n_tiles = (int)ntiles;
  // persistent, two workgroups per CU
  const int64_t cap = 2ll * device_cus();
  GoR2<W, RB, E, NA, WO, SB> go{a, dim3((unsigned)(ntiles < cap ? ntiles : cap)), st};
  // the default r2 tiles (cout a multiple of 128, one image row block per workgroup at 16x16,
  // 2 images at 8x8, 8 at 4x4) get the specialised epilogues; the A/B-only 32x32 forms do not
  constexpr bool spec = NA == 1 && WO == 4 && !SB;
  // the fused unit input at 16x16 and 8x8 (at 4x4 its residual registers spill)
  return dispatch_epi<spec, decltype(go), spec && W >= 8>(a, go);
}

// the padded-width r2 tiles (conv3x3_r2_kernel PW): the EL2N statistics launch, staged with the
// producer's BN (+ ReLU) or raw, fp16 or bf16 operand halves; 128-output workgroups, two per CU
template <int W, int RB, int E, int PW, int XF, int EPI>
static int run_pw(const Args& a, dim3 g, hipStream_t st) {
  constexpr auto K = &conv3x3_r2_kernel<W, RB, E, 1, 4, XF, false, false, EPI, PW>;
  lds_attr<K>(Cfg<W, RB, E, 1, 4>::LDS);
  K<<<g, 256, Cfg<W, RB, E, 1, 4>::LDS, st>>>(a);
  DD_CHECK_LAUNCH("dd_conv3x3_forward");
  return DD_OK;
}
template <int W, int RB, int E, int PW>
static int launch_r2_pw(Args a, hipStream_t st) {
  using C = Cfg<W, RB, E, 1, 4>;
  static_assert(2 * C::LDS <= 160 * 1024, "r2 tiles run two workgroups per CU");
  DD_REQUIRE(a.gsize % E == 0, "dd_conv3x3_forward: group_size %d must be a multiple of %d "
             "(images per tile at %dx%d)", a.gsize, E, a.H, a.wg);
  DD_REQUIRE(a.op % C::OB == 0, "dd_conv3x3_forward: padded outputs %d not a multiple of %d",
             a.op, C::OB);
  DD_REQUIRE(a.wg > 0 && a.wg <= W && (PW == 2 || a.wg % 4 == 0) && (E == 1 || a.H <= RB),
             "dd_conv3x3_forward: no padded-width tile for %dx%d", a.H, a.wg);
  DD_REQUIRE(epilogue_code(a) == kE_Stats && xf_mode(a) <= kXfAffine && !a.kx1,
             "dd_conv3x3_forward: the padded-width tiles take the statistics epilogue only");
  a.n_tb = (a.H + RB - 1) / RB;
  a.n_ob = a.op / C::OB;
  const int64_t ntiles = ceil_div(a.B, E) * a.n_tb * a.n_ob;
  DD_REQUIRE(ntiles < (1ll << 31), "dd_conv3x3_forward: too many tiles");
  a.n_tiles = (int)ntiles;
  const int64_t cap = 2ll * device_cus();
  const dim3 g((unsigned)(ntiles < cap ? ntiles : cap));
  const bool xf = a.xf_mask != 0;
  if (a.f16)
    return xf ? run_pw<W, RB, E, PW, kXfAffine, kE_Stats | kEpiF16>(a, g, st)
              : run_pw<W, RB, E, PW, kXfNone, kE_Stats | kEpiF16>(a, g, st);
  return xf ? run_pw<W, RB, E, PW, kXfAffine, kE_Stats>(a, g, st)
            : run_pw<W, RB, E, PW, kXfNone, kE_Stats>(a, g, st);
}

// the padded-width narrow tile (conv3x3_kernel PW: 64-output workgroups, the EL2N statistics
// launch); its LDS image takes one workgroup per CU at W = 64
template <int W, int RB, int E, int PW, int XF, int EPI>
static int run_pw_narrow(const Args& a, dim3 g, hipStream_t st) {
  constexpr auto K = &conv3x3_kernel<W, RB, E, 1, 2, XF, false, EPI, PW>;
  lds_attr<K>(Cfg<W, RB, E, 1, 2>::LDS);
  K<<<g, 256, Cfg<W, RB, E, 1, 2>::LDS, st>>>(a);
  DD_CHECK_LAUNCH("dd_conv3x3_forward");
  return DD_OK;
}
template <int W, int RB, int E, int PW>
static int launch_narrow_pw(Args a, hipStream_t st) {
  using C = Cfg<W, RB, E, 1, 2>;
  static_assert(C::LDS <= 160 * 1024, "LDS");
  DD_REQUIRE(a.gsize % E == 0, "dd_conv3x3_forward: group_size %d must be a multiple of %d "
             "(images per tile at %dx%d)", a.gsize, E, a.H, a.wg);
  DD_REQUIRE(a.op % C::OB == 0, "dd_conv3x3_forward: padded outputs %d not a multiple of %d",
             a.op, C::OB);
  DD_REQUIRE(a.wg > 0 && a.wg <= W && (PW == 2 || a.wg % 4 == 0) && (E == 1 || a.H <= RB),
             "dd_conv3x3_forward: no padded-width tile for %dx%d", a.H, a.wg);
  DD_REQUIRE(epilogue_code(a) == kE_Stats && xf_mode(a) <= kXfAffine && !a.kx1,
             "dd_conv3x3_forward: the padded-width tiles take the statistics epilogue only");
  a.n_tb = (a.H + RB - 1) / RB;
  a.n_ob = a.op / C::OB;
  const int64_t ntiles = ceil_div(a.B, E) * a.n_tb * a.n_ob;
  DD_REQUIRE(ntiles < (1ll << 31), "dd_conv3x3_forward: too many tiles");
  a.n_tiles = (int)ntiles;
  const int64_t cap = (int64_t)(160 * 1024 / C::LDS) * device_cus();
  const dim3 g((unsigned)(ntiles < cap ? ntiles : cap));
  const bool xf = a.xf_mask != 0;
  if (a.f16)
    return xf ? run_pw_narrow<W, RB, E, PW, kXfAffine, kE_Stats | kEpiF16>(a, g, st)
              : run_pw_narrow<W, RB, E, PW, kXfNone, kE_Stats | kEpiF16>(a, g, st);
  return xf ? run_pw_narrow<W, RB, E, PW, kXfAffine, kE_Stats>(a, g, st)
            : run_pw_narrow<W, RB, E, PW, kXfNone, kE_Stats>(a, g, st);
}

// tile-config dispatchers of the other translation units (key = rb*1000 + e*100 + na*10 + wo)
int dispatch_r2(int w, int key, const Args& a, hipStream_t st);       // dd_conv_r2.hip
int dispatch_small(int w, int key, const Args& a, hipStream_t st);    // dd_conv_nw.hip
int dispatch_pw(int w, int pw, const Args& a, hipStream_t st);        // dd_conv_pw.hip

}  // namespace conv
}  // namespace dd
