// Host entry points of the split-bf16 3x3 convolution (see dd_conv_kern.h for the kernels):
// weight packing, tile selection, and the narrow 32x32 tile of the scoring passes.
#include "dd_conv_kern.h"

#include <stdlib.h>
#include <string.h>

namespace dd {

// identity affine for the staging transform (scale 1 at [0], shift 0 at [1]; index mask 0)
__device__ float g_unit_affine[2] = {1.f, 0.f};

namespace conv {

// pack fp32 weights [cout][cin][3][3] into fragment-major hi/lo halves (bf16, or fp16 with
// f16: DD_OPERANDS_F16X3):
// [chunk kc][32-o block][tap][hi|lo][lane 0..63][8], where lane (r, h) of a fragment holds
// W[o = 32*blk + r][c = 16*kc + 8*h + j][tap], j = 0..7 (the A-operand map of
// v_mfma_f32_32x32x16_bf16).  Zero padded to op outputs / cp inputs.  With tflip the packed
// conv is the backward-data conv: out channels = cin, in channels = cout,
// W'[c][o][tap] = W[o][c][8 - tap].
__global__ void pack_kernel(const float* __restrict__ w, int cout, int cin, int tflip, int op,
                            int cp, int f16, float scale, __bf16* __restrict__ out) {
  const int nob32 = op / 32, nkc = cp / CC;
  const int total = nkc * nob32 * 18 * 512;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int j = i & 7, lane = (i >> 3) & 63;
    int r = i >> 9;
    const int f = r % 18;
    r /= 18;
    const int blk = r % nob32, kc = r / nob32;
    const int tap = f >> 1, pr = f & 1;
    const int o = blk * 32 + (lane & 31), c = kc * CC + 8 * (lane >> 5) + j;
    // packed conv: no outputs, nc inputs, W'(o, c, tap) (= W[c][o][8 - tap] with tflip)
    const int no = tflip ? cin : cout, nc = tflip ? cout : cin;
    auto wp = [&](int oo, int ci, int t) {
      return tflip ? w[((size_t)ci * cin + oo) * 9 + (8 - t)] : w[((size_t)oo * cin + ci) * 9 + t];
    };
    float v = 0.f;
    if (nc <= kStemCin) {
      // stem layout, decided by the PACKED conv's input channels exactly as the kernel
      // decides it (a.kx1 = cin <= kStemCin): tap (ky, 1) of pseudo-channel k = kx nc + c'
      // holds W'(o, c', (ky, kx)).  A backward-data pack of a conv with cout <= 5 is one.
      const int ky = tap / 3, kx = c / nc, cc = c - kx * nc;
      if (o < no && tap % 3 == 1 && c < 3 * nc) v = wp(o, cc, ky * 3 + kx);
    } else if (o < no && c < nc) {
      v = wp(o, c, tap);
    }
    v *= scale;  // a power of two (1 for bf16 packs): exact
    __bf16 hi, lo;
    if (f16)
      split16<true>(v, hi, lo);
    else
      split16<false>(v, hi, lo);
    out[i] = pr == 0 ? hi : lo;
  }
}

// tile configuration for an h x w image with `cout` outputs and BN groups of `gsize` examples
// (tiles of several images only when they always share a group)
struct Sel {
  int rb, e, na, wo;
  int r2;  // conv3x3_r2_kernel (two workgroups per CU, whole-row register blocking)
};
// tuning knob for A/B runs: DD_CONV_TILE=narrow | wide | r2 forces one family where it applies
static int tile_family() {
  static int f = -1;
  if (f < 0) {
    const char* e = getenv("DD_CONV_TILE");
    f = !e ? 0 : !strcmp(e, "narrow") ? 1 : !strcmp(e, "wide") ? 2 : !strcmp(e, "r2") ? 3
        : !strcmp(e, "r2w32") ? 5 : !strcmp(e, "r2sb") ? 6 : 0;
  }
  return f;
}

static bool select(int h, int w, int cout, int gsize, Sel* s) {
  // wide: 64 o x 64 t per wave; 2 x 2 waves (128 o x 128 t) when the padded outputs allow,
  // else 1 x 4 (64 o x 256 t)
  const int wo = pad_to(cout, 64) % 128 == 0 ? 2 : 1;
  const int tb = (4 / wo) * 64;
  // measured (tools/ab_conv.py, B = 512): wide wins at 4x4 (512 channels, +16-21 %), narrow
  // at 8x8 and above (+6-10 % at 256 down to 128 channels, more at 64)
  const int fam = tile_family();
  // r2: 128 o x 128 t workgroups (2 x 2 waves of 64 o x 64 t) with cout a multiple of 128.
  // Measured against the other families (tools/ab_conv.py, B = 1024, profiles/r02_s2): +3-5 %
  // at 8x8 (256 channels), 0.98x at 4x4 (vs wide), 0.83-0.92x at 16x16 (vs narrow), so by
  // default at 8x8 only; DD_CONV_TILE=r2 takes it wherever it applies.  (Not at 32x32: the
  // stem's layout shares that geometry's masks.)
  // r2: 128 o x 128 t workgroups of 4 waves along o, each 32 o x 128 t (NA = 1, NT = 4), two
  // workgroups per CU, at 16x16, 8x8 and 4x4 with cout a multiple of 128.  A weight fragment
  // feeds 4 column tiles (twice the narrow tile's), so the weight stream from L2 per MFMA
  // halves.  Measured (tools/ab_conv.py, B = 1024, profiles/r02_s2/ab_conv_r2t.txt): 1.06-1.09x
  // the narrow tile at 16x16, 1.06x the NA = 2 r2 form at 8x8 (itself 1.03-1.05x narrow),
  // 1.01-1.03x the wide tile at 4x4; bit-identical.  (Not at 32x32: the stem's layout shares
  // that geometry's masks, and a 256-position tile there would not fit two per CU.)
  // DD_CONV_TILE=r2w32: at 32x32 with 64 outputs, 4 waves along t, each 64 o x 32 t (NA = 2,
  // NT = 1: a B fragment feeds both 32-o blocks, a weight fragment one column tile).  Measured
  // 0.75-0.91x the narrow tile (profiles/r02_s2/ab_conv_r2_w32_rejected.txt): the weight stream
  // per MFMA, not the B reads, is what costs there, so it is not the default.
  if (fam == 5 && wo == 1 && w == 32 && h % 4 == 0 && cout <= 64) {
    *s = {4, 1, 2, 1, 1};
    return true;
  }
  // DD_CONV_TILE=r2sb: at 32x32 with 64 outputs, 2 x 2 waves of 32 o x 128 t (NA = 1, NT = 4:
  // a weight fragment feeds 4 column tiles), 8-row tiles (1.25x input rows staged instead of
  // 1.5x), one staging buffer so that two fit per CU.  Measured 0.98-1.01x the narrow tile on
  // 64 channels and 0.76-0.87x on the stem (profiles/r02_s2/ab_conv_r2sb_rejected.txt): the
  // 32x32 layers are bound neither by the weight stream nor by the halo re-reads.
  if (fam == 6 && wo == 1 && w == 32 && h % 8 == 0 && cout <= 64) {
    *s = {8, 1, 1, 2, 1};
    return true;
  }
  if (wo == 2 && (fam == 3 || fam == 0) && w <= 16) {
    if (w == 16 && h % 8 == 0) { *s = {8, 1, 1, 4, 1}; return true; }
    if (w == 8 && h == 8 && gsize % 2 == 0) { *s = {8, 2, 1, 4, 1}; return true; }
    if (w == 4 && h == 4 && gsize % 8 == 0) { *s = {4, 8, 1, 4, 1}; return true; }
  }
  if (fam == 2 || (fam == 0 && w == 4)) {
    if ((w == 32 || w == 16) && h % (tb / w) == 0) { *s = {tb / w, 1, 2, wo}; return true; }
    if (w == 8 && h == 8 && gsize % (tb / 64) == 0) { *s = {8, tb / 64, 2, wo}; return true; }
    if (w == 4 && h == 4 && gsize % (tb / 16) == 0) { *s = {4, tb / 16, 2, wo}; return true; }
  }
  // narrow fallbacks
  if (w == 32 && h % 4 == 0) { *s = {4, 1, 1, 2}; return true; }
  if (w == 16 && h % 8 == 0) { *s = {8, 1, 1, 2}; return true; }
  if (w == 8 && h == 8 && gsize % 2 == 0) { *s = {8, 2, 1, 2}; return true; }
  if (w == 8 && h % 8 == 0) { *s = {8, 1, 1, 2}; return true; }
  if (w == 4 && h == 4 && gsize % 4 == 0) { *s = {4, 4, 1, 2}; return true; }
  return false;
}

// padded-width geometry (conv3x3_r2_kernel PW) for an image width that is not a tile width:
// the tile width (0: none), its row block, images per tile and PW mode.  The 128-output r2
// workgroups of the EL2N statistics launch (the 64-output narrow one at widths past 32); DD_CONV_PW=0 turns it off (read per call, for A/B
// runs in one process: the caller then takes the implicit GEMM)
static int pw_tile(int h, int w, int gsize, int* rb, int* e, int* pw) {
  const char* env = getenv("DD_CONV_PW");
  if ((env && atoi(env) == 0) || h <= 0 || gsize <= 0) return 0;
  if (w > 32 && w <= 64 && w % 4 == 0) { *rb = 2; *e = 1; *pw = 1; return 64; }
  if (w > 16 && w <= 32 && w % 4 == 0) { *rb = 4; *e = 1; *pw = 1; return 32; }
  if (w > 8 && w <= 16) { *rb = 8; *e = 1; *pw = 2; return 16; }
  if (w > 4 && w <= 8 && h <= 8 && gsize % 2 == 0) { *rb = 8; *e = 2; *pw = 2; return 8; }
  return 0;
}

// group size of an ungrouped launch: every tile height divides it
constexpr int kFreeGroup = 16;

// Fragment-order ReLU mask words of a dd_conv3x3_forward launch (mask_out: one 16-bit word per
// lane per 32 x 32 accumulator fragment, bit 4 k + j = output (o0 + 8 k + lane / 8, position
// t0 + 4 (lane % 8) + j) > 0) -> plane bits: bit p & 31 of word ((b cout + o) h w + p) >> 5.
// One thread per plane word; the word's 32 positions are one fragment's (the tile's rows are
// contiguous plane positions and a fragment covers 32 of them), gathered from 8 lanes' words.
__global__ __launch_bounds__(256) void mask_plane_bits_kernel(
    const uint16_t* __restrict__ mf, int64_t nwords, int cout, int H, int W, int rb, int e,
    int na, int wo, int n_ob, uint32_t* __restrict__ bits) {
  const int HW = H * W, wpp = HW / 32;
  const int OB = wo * na * 32, TW = e * rb * W / (4 / wo), NT = TW / 32, n_tb = H / rb;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nwords;
       i += (int64_t)gridDim.x * 256) {
    const int64_t plane = i / wpp;
    const int p0 = (int)(i - plane * wpp) * 32;
    const int64_t b = plane / cout;
    const int o = (int)(plane - b * cout);
    const int y = p0 / W, tb = y / rb;
    const int tt0 = (int)(b % e) * rb * W + (y - tb * rb) * W + p0 % W;  // in the tile
    const int ob = o / OB, oo = o - ob * OB;
    const int wo_ = oo / (na * 32), a = (oo / 32) % na, oin = oo & 31;
    const int wt = tt0 / TW, n = (tt0 % TW) / 32;
    const int64_t tile = ((b / e) * n_tb + tb) * n_ob + ob;
    const int wv = wo_ + wo * wt;
    const uint16_t* w8 = mf + ((((tile * 4 + wv) * na + a) * NT + n) * 64 + (oin & 7) * 8);
    const int sh = 4 * (oin >> 3);
    uint32_t v = 0;
#pragma unroll
    for (int tl = 0; tl < 8; ++tl) v |= (uint32_t)((w8[tl] >> sh) & 0xFu) << (4 * tl);
    bits[i] = v;
  }
}

static int dispatch(const Sel& s, int w, const Args& a, hipStream_t st) {
  const int k = s.rb * 1000 + s.e * 100 + s.na * 10 + s.wo;
  if (s.r2) return dispatch_r2(w, k, a, st);
  if (w == 32 && k == 4000 + 100 + 10 + 2) return launch<32, 4, 1, 1, 2>(a, st);
  return dispatch_small(w, k, a, st);
}

}  // namespace conv
}  // namespace dd

using namespace dd;

extern "C" {

size_t dd_conv3x3_pack_bytes(int32_t out_channels, int32_t in_channels) {
  if (out_channels <= 0 || in_channels <= 0) return 0;
  const int op = conv::pad_to(out_channels, 64), cp = conv::pad_to(in_channels, conv::CC);
  return (size_t)2 * 9 * op * cp * sizeof(__bf16);
}

int dd_conv3x3_pack(const float* w, int32_t cout, int32_t cin, int32_t transpose_flip,
                    int32_t operands, float scale, void* packed, void* stream) {
  clear_error();
  DD_REQUIRE(w && packed && cout > 0 && cin > 0, "dd_conv3x3_pack: bad arguments");
  DD_REQUIRE(operands == DD_OPERANDS_BF16X3 || operands == DD_OPERANDS_F16X3,
             "dd_conv3x3_pack: operands must be DD_OPERANDS_BF16X3 or DD_OPERANDS_F16X3");
  DD_REQUIRE(operand_scale_ok(operands, scale),
             "dd_conv3x3_pack: scale must be 1 (bf16 operands) or a power of two (fp16)");
  const int no = transpose_flip ? cin : cout, nc = transpose_flip ? cout : cin;
  const int op = conv::pad_to(no, 64), cp = conv::pad_to(nc, conv::CC);
  const int total = 2 * 9 * op * cp;
  conv::pack_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 4096), 256, 0,
                      as_stream(stream)>>>(w, cout, cin, transpose_flip, op, cp,
                                           operands == DD_OPERANDS_F16X3, scale,
                                           static_cast<__bf16*>(packed));
  DD_CHECK_LAUNCH("dd_conv3x3_pack");
  return DD_OK;
}

size_t dd_conv3x3_mask_bytes(int64_t B, int32_t cout, int32_t h, int32_t w) {
  conv::Sel sl;
  if (B <= 0 || cout <= 0 || !conv::select(h, w, cout, conv::kFreeGroup, &sl)) return 0;
  const int ob = sl.wo * sl.na * 32;
  const int64_t tiles = ceil_div(B, sl.e) * (h / sl.rb) * (conv::pad_to(cout, 64) / ob);
  // per tile: 4 waves x (positions x channels per wave / 32 / 32) fragments x 64 lanes
  const int64_t frags = (int64_t)sl.e * sl.rb * w * ob / 1024 / 4;
  return (size_t)tiles * 4 * frags * 64 * sizeof(uint16_t);
}

int dd_conv3x3_mask_plane_bits(const uint16_t* mask, int64_t B, int32_t cout, int32_t h,
                               int32_t w, uint32_t* bits, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && cout > 0 && h > 0 && w > 0, "dd_conv3x3_mask_plane_bits: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(mask && bits, "dd_conv3x3_mask_plane_bits: null buffer");
  conv::Sel sl;
  DD_REQUIRE(conv::select(h, w, cout, conv::kFreeGroup, &sl),
             "dd_conv3x3_mask_plane_bits: unsupported shape %dx%d", h, w);
  DD_REQUIRE((h * w) % 32 == 0 && (sl.rb * w) % 32 == 0,
             "dd_conv3x3_mask_plane_bits: a %dx%d map's fragments are not whole plane words",
             h, w);
  const int ob = sl.wo * sl.na * 32;
  const int64_t nwords = B * cout * (int64_t)h * w / 32;
  conv::mask_plane_bits_kernel<<<(unsigned)std::min<int64_t>(ceil_div(nwords, 256), 1 << 16),
                                 256, 0, as_stream(stream)>>>(
      mask, nwords, cout, h, w, sl.rb, sl.e, sl.na, sl.wo, conv::pad_to(cout, 64) / ob, bits);
  DD_CHECK_LAUNCH("dd_conv3x3_mask_plane_bits");
  return DD_OK;
}

// BN partial layout: one partial per (group, channel, 32 consecutive positions of the group's
// examples), whatever the tile config
int dd_conv3x3_tiles_per_group(int32_t h, int32_t w, int32_t group_size) {
  conv::Sel sl;
  if (group_size <= 0 || h <= 0 || w <= 0) return -1;
  if (!conv::select(h, w, 64, group_size, &sl)) {
    // a padded-width launch: the native layout on the padded grid
    int rb = 0, e = 0, pw = 0;
    const int wt = conv::pw_tile(h, w, group_size, &rb, &e, &pw);
    if (!wt || group_size % e) return -1;
    return (int)((int64_t)group_size * ((h + rb - 1) / rb) * rb * wt / 32);
  }
  if (group_size % sl.e) return -1;
  const int64_t pos = (int64_t)group_size * h * w;
  if ((h * w) % 32 != 0 && !(h * w == 16 && group_size % 2 == 0)) return -1;
  return (int)(pos / 32);
}

static int forward_impl(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                        const void* packed, int32_t cout, const float* bias,
                        const float* residual, const float* mask_src, int32_t relu,
                        const float* in_scale, const float* in_shift, int32_t in_relu,
                        int32_t group_size, int64_t n_stat, float* stats, uint16_t* mask_out,
                        const uint16_t* mask_in, float* y, const float* xres,
                        const float* xres_scale, const float* xres_shift, float* xout,
                        int32_t operands, float acc_scale, void* stream) {
  DD_REQUIRE(B >= 0 && cin > 0 && cout > 0 && h > 0, "dd_conv3x3_forward: bad sizes");
  DD_REQUIRE(operands == DD_OPERANDS_BF16X3 || operands == DD_OPERANDS_F16X3,
             "dd_conv3x3_forward: operands must be DD_OPERANDS_BF16X3 or DD_OPERANDS_F16X3");
  DD_REQUIRE(operand_scale_ok(operands, acc_scale),
             "dd_conv3x3_forward: acc_scale must be 1 (bf16 operands) or a power of two (fp16)");
  if (B == 0) return DD_OK;
  DD_REQUIRE(x && packed && y, "dd_conv3x3_forward: null buffer");
  DD_REQUIRE((int64_t)cin * h * w < (1ll << 31) && (int64_t)cout * h * w < (1ll << 31),
             "dd_conv3x3_forward: per-example tensor too large");
  DD_REQUIRE(!in_scale == !in_shift, "dd_conv3x3_forward: in_scale and in_shift go together");
  const bool grouped = in_scale || stats;
  DD_REQUIRE(!grouped || group_size > 0, "dd_conv3x3_forward: group_size must be positive");
  conv::Sel sl;
  int pw_w = 0, pw_mode = 0;
  if (!conv::select(h, w, cout, grouped ? group_size : conv::kFreeGroup, &sl)) {
    // the padded-width tiles: the EL2N statistics launch only
    const bool stats_only = stats && !bias && !residual && !mask_src && !relu && !mask_out &&
                            !mask_in && !xout && cin > conv::kStemCin;
    if (stats_only) pw_w = conv::pw_tile(h, w, group_size, &sl.rb, &sl.e, &pw_mode);
    if (!pw_w) {
      set_error("dd_conv3x3_forward: unsupported spatial shape %dx%d (W in {8,16,32} with H a "
                "multiple of the row block, or 8x8 / 4x4; other widths up to 32 with the "
                "statistics epilogue alone)", h, w);
      return DD_EINVAL;
    }
  }
  conv::Args a{};
  a.x = x;
  a.wpack = static_cast<const __bf16*>(packed);
  a.bias = bias;
  a.residual = residual;
  a.mask_src = mask_src;
  a.y = y;
  a.stats = stats;
  a.mask_out = mask_out;
  a.mask_in = mask_in;
  DD_REQUIRE(!(mask_in && mask_src), "dd_conv3x3_forward: mask_in and mask_src are exclusive");
  a.B = B;
  a.n_stat = stats ? std::min<int64_t>(std::max<int64_t>(n_stat, 0), B) : 0;
  a.cin = cin;
  a.H = h;
  a.cout = cout;
  a.op = conv::pad_to(cout, 64);
  a.cp = conv::pad_to(cin, conv::CC);
  a.kx1 = cin <= conv::kStemCin;  // dd_conv3x3_pack wrote the stem layout
  a.f16 = operands == DD_OPERANDS_F16X3;
  a.acc_scale = acc_scale;
  a.stagger = conv::stagger_cycles();
  a.xcd = conv::conv_xcd();
  a.relu = relu;
  // ungrouped: one group spanning the batch, a multiple of every tile height
  a.gsize = grouped ? group_size
                    : (int)(std::min<int64_t>(B + conv::kFreeGroup, 1 << 30) / conv::kFreeGroup *
                            conv::kFreeGroup);
  if (stats) {
    const int tpg = dd_conv3x3_tiles_per_group(h, w, a.gsize);
    DD_REQUIRE(tpg > 0, "dd_conv3x3_forward: no stats layout for %dx%d with group_size %d", h,
               w, a.gsize);
    a.tiles_per_group = tpg;
  }
  if (in_scale) {
    a.in_scale = in_scale;
    a.in_shift = in_shift;
    a.xf_mask = -1;
    a.in_floor = in_relu ? 0.f : -INFINITY;
  } else {
    static float* unit = nullptr;
    if (!unit) DD_CHECK_HIP(hipGetSymbolAddress(reinterpret_cast<void**>(&unit),
                                                HIP_SYMBOL(g_unit_affine)),
                            "dd_conv3x3_forward: unit affine");
    a.in_scale = unit;
    a.in_shift = unit + 1;
    a.xf_mask = 0;
    a.in_floor = -INFINITY;
  }
  a.xres = xres;
  a.xres_scale = xres_scale;
  a.xres_shift = xres_shift;
  a.xout = xout;
  a.wg = w;
  if (pw_w) return conv::dispatch_pw(pw_w, pw_mode, a, as_stream(stream));
  return conv::dispatch(sl, w, a, as_stream(stream));
}

int dd_conv3x3_padded_supported(int32_t h, int32_t w, int32_t cin, int32_t cout,
                                int32_t group_size) {
  conv::Sel sl;
  int rb = 0, e = 0, pw = 0;
  if (h <= 0 || w <= 0 || cin <= conv::kStemCin || cout <= 0 || group_size <= 0 ||
      conv::select(h, w, cout, group_size, &sl))
    return 0;
  const int wt = conv::pw_tile(h, w, group_size, &rb, &e, &pw);
  // (the 64-wide tile has 64-output workgroups, the others 128-output ones)
  return wt && group_size % e == 0 && (wt == 64 || conv::pad_to(cout, 64) % 128 == 0) &&
                 (int64_t)cin * h * w < (1ll << 31) && (int64_t)cout * h * w < (1ll << 31)
             ? 1
             : 0;
}

int dd_conv3x3_forward(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                       const void* packed, int32_t cout, const float* bias,
                       const float* residual, const float* mask_src, int32_t relu,
                       const float* in_scale, const float* in_shift, int32_t in_relu,
                       int32_t group_size, int64_t n_stat, float* stats, uint16_t* mask_out,
                       const uint16_t* mask_in, float* y, int32_t operands, float acc_scale,
                       void* stream) {
  clear_error();
  return forward_impl(x, B, cin, h, w, packed, cout, bias, residual, mask_src, relu, in_scale,
                      in_shift, in_relu, group_size, n_stat, stats, mask_out, mask_in, y,
                      nullptr, nullptr, nullptr, nullptr, operands, acc_scale, stream);
}

int dd_conv3x3_unit_input_supported(int32_t h, int32_t w, int32_t cin, int32_t cout,
                                    int32_t group_size) {
  conv::Sel sl;
  if (h <= 0 || w <= 0 || cin <= conv::kStemCin || cout <= 0 || group_size <= 0 ||
      !conv::select(h, w, cout, group_size, &sl) || group_size % sl.e)
    return 0;
  // the tiles with the specialised statistics epilogue (conv::launch / launch_r2)
  const bool narrow = !sl.r2 && w == 32 && sl.rb == 4 && sl.e == 1 && sl.na == 1 && sl.wo == 2;
  const bool r2 = sl.r2 && sl.na == 1 && sl.wo == 4 && w >= 8;
  return (narrow || r2) && dd_conv3x3_tiles_per_group(h, w, group_size) > 0 ? 1 : 0;
}

int dd_conv3x3_forward_unit_input(const float* y_prev, const float* in_scale,
                                  const float* in_shift, const float* res,
                                  const float* res_scale, const float* res_shift, float* x_out,
                                  int64_t B, int32_t cin, int32_t h, int32_t w,
                                  const void* packed, int32_t cout, int32_t group_size,
                                  int64_t n_stat, float* stats, float* y, int32_t operands,
                                  float acc_scale, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0, "dd_conv3x3_forward_unit_input: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(y_prev && in_scale && in_shift && x_out && stats && y,
             "dd_conv3x3_forward_unit_input: null buffer");
  DD_REQUIRE(!res_scale == !res_shift && (res || !res_scale),
             "dd_conv3x3_forward_unit_input: res_scale and res_shift go with res");
  DD_REQUIRE(dd_conv3x3_unit_input_supported(h, w, cin, cout, group_size),
             "dd_conv3x3_forward_unit_input: unsupported shape (%d -> %d at %dx%d, group %d)",
             cin, cout, h, w, group_size);
  return forward_impl(y_prev, B, cin, h, w, packed, cout, nullptr, nullptr, nullptr, 0,
                      in_scale, in_shift, 1, group_size, n_stat, stats, nullptr, nullptr, y, res,
                      res_scale, res_shift, x_out, operands, acc_scale, stream);
}

}  // extern "C"
