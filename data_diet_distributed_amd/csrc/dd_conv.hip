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
#include "dd_mfma.h"

namespace dd {

// identity affine for the staging transform (scale 1 at [0], shift 0 at [1]; index mask 0)
__device__ float g_unit_affine[2] = {1.f, 0.f};

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
  int n_tb, n_ob;
};

template <int W, int RB, int E>
struct Cfg {
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
  static constexpr int LDS = 2 * BUF;          // double-buffered over K chunks
  static constexpr int TB = E * RB * W;        // output positions per workgroup
  static constexpr int NT = TB / 64;           // 32-wide t tiles per wave (2 waves along t)
  static constexpr int TPR = W / 4;            // threads per staged channel row (float4 each)
  static constexpr int NF4 = NR * CC * W / 4;  // float4 per chunk
  static constexpr int NST = (NF4 + 255) / 256;
  static_assert(TB % 64 == 0, "tile must hold a multiple of 64 positions");
};

// E > 1: the tile stacks E whole images (H == RB), each staged with its own halo rows
template <int W, int RB, int E>
__global__ __launch_bounds__(256, 2) void conv3x3_kernel(const Args A) {
  using C = Cfg<W, RB, E>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = A.H, cin = A.cin, cout = A.cout;
  const int64_t B = A.B;
  const float* __restrict__ x = A.x;
  const int HW = H * W;
  int bid = blockIdx.x;
  const int ob = bid % A.n_ob;
  bid /= A.n_ob;
  const int tb = bid % A.n_tb;
  const int64_t b = (int64_t)(bid / A.n_tb) * E;
  const int o0 = ob * 64, y0 = tb * RB;
  // BN group of the tile (group_size % E == 0, so the E images share it)
  const int64_t grp = b / A.gsize;
  const int xf_base = (int)(grp * cin);

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wo = wv & 1, wt = wv >> 1, h = lane >> 5;

  // ---- staging of one K chunk (16 input channels x NR rows) into buffer `buf`
  float4 ra[C::NST];
  float xs[C::NST], xt[C::NST];
  bool va[C::NST];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int k = 0; k < C::NST; ++k) {
      const int q = tid + 256 * k;
      const int x4 = q % C::TPR, c = (q / C::TPR) % CC, sr = q / (C::TPR * CC);
      const int e = sr / (RB + 2), rr = sr - e * (RB + 2);
      const int ir = y0 - 1 + rr, cg = c0 + c;
      const bool ve = b + e < B;
      va[k] = q < C::NF4 && ir >= 0 && ir < H && cg < cin && ve;
      const int irc = ir < 0 ? 0 : (ir >= H ? H - 1 : ir);
      const int cgc = cg < cin ? cg : cin - 1;
      const int64_t bc = ve ? b + e : B - 1;
      ra[k] = *reinterpret_cast<const float4*>(x + ((size_t)bc * cin + cgc) * HW + irc * W +
                                               x4 * 4);
      const int xi = (xf_base + cgc) & A.xf_mask;
      xs[k] = A.in_scale[xi];
      xt[k] = A.in_shift[xi];
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
      v.x = fmaxf(fmaf(v.x, xs[k], xt[k]), A.in_floor);
      v.y = fmaxf(fmaf(v.y, xs[k], xt[k]), A.in_floor);
      v.z = fmaxf(fmaf(v.z, xs[k], xt[k]), A.in_floor);
      v.w = fmaxf(fmaf(v.w, xs[k], xt[k]), A.in_floor);
      v = va[k] ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      // halo columns from the neighbouring lanes of the row: DPP row shifts (a VALU op, where
      // a width-limited shuffle is an LDS ds_bpermute with its lgkmcnt wait); a row's first /
      // last lane takes the zero padding instead
      float left = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
          0, __builtin_bit_cast(int, v.w), 0x111, 0xf, 0xf, true));  // row_shr:1
      float right = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
          0, __builtin_bit_cast(int, v.x), 0x101, 0xf, 0xf, true));  // row_shl:1
      if (x4 == 0) left = 0.f;
      if (x4 == C::TPR - 1) right = 0.f;
      const float f[6] = {left, v.x, v.y, v.z, v.w, right};
      __bf16 hv[6], lv[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        hv[i] = (__bf16)f[i];
        lv[i] = (__bf16)(f[i] - (float)hv[i]);
      }
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        char* p = base0 + se * C::IMGP + rr * C::ROWP + (kx * 2) * C::PLANE + c * C::XS +
                  x4 * 8;
        *reinterpret_cast<bf16x4*>(p) = bf16x4{hv[kx], hv[kx + 1], hv[kx + 2], hv[kx + 3]};
        *reinterpret_cast<bf16x4*>(p + C::PLANE) =
            bf16x4{lv[kx], lv[kx + 1], lv[kx + 2], lv[kx + 3]};
      }
    }
  };

  // ---- weights of one chunk: 9 taps x hi|lo fragments, 16 B per lane.  The pack is
  // fragment-major ([chunk][32-o block][tap][hi|lo][lane][8]), so each fragment load is one
  // contiguous 1 KB wave access.
  bf16x8 wa[18];
  const int ob32 = (o0 >> 5) + wo, nob32 = A.op >> 5;
  const __bf16* __restrict__ wpack = A.wpack;
  auto load_w_taps = [&](int kc, int tap0, int ntap) {
    const __bf16* base = wpack + ((size_t)(kc * nob32 + ob32) * 18) * 512 + lane * 8;
#pragma unroll
    for (int tap = tap0; tap < tap0 + ntap; ++tap)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
        wa[tap * 2 + pr] = *reinterpret_cast<const bf16x8*>(base + (tap * 2 + pr) * 512);
  };

  // per-lane transposed-read geometry: lane 4q+p of each 16-lane group supplies row q,
  // columns 4p..4p+3 of a 4 x 16 block; the group's 16 columns are t = 16*(g&1) + 0..15
  const int q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
  int tr_yo[C::NT], tr_xo[C::NT];  // LDS offset of the tap-(0,*) input row, x offset
#pragma unroll
  for (int n = 0; n < C::NT; ++n) {
    const int t = wt * (C::TB / 2) + n * 32 + 16 * g1 + 4 * p;
    const int e = t / (RB * W);
    tr_yo[n] = e * C::IMGP + ((t / W) % RB) * C::ROWP;
    tr_xo[n] = t % W;
  }

  floatx16 acc[C::NT];
#pragma unroll
  for (int n = 0; n < C::NT; ++n) acc[n] = floatx16{0};

  // B fragments of one tap row ky: [kx][n][hi|lo]
  auto read_b = [&](const char* base, int ky, bf16x8 (&bf)[3][C::NT][2]) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int n = 0; n < C::NT; ++n) {
        const char* a = base + tr_yo[n] + ky * C::ROWP + (kx * 2) * C::PLANE +
                        (8 * h + q) * C::XS + tr_xo[n] * 2;
        bf[kx][n][0] = tr_read8(a, a + 4 * C::XS);
        bf[kx][n][1] = tr_read8(a + C::PLANE, a + C::PLANE + 4 * C::XS);
      }
  };
  auto mfma_row = [&](int ky, const bf16x8 (&bf)[3][C::NT][2]) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int n = 0; n < C::NT; ++n) {
        const int tap = ky * 3 + kx;
        floatx16 d = acc[n];
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[tap * 2], bf[kx][n][0], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[tap * 2], bf[kx][n][1], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[tap * 2 + 1], bf[kx][n][0], d, 0, 0, 0);
        acc[n] = d;
      }
  };

  const int nchunks = (cin + CC - 1) / CC;
  load_chunk(0);
  load_w_taps(0, 0, 9);
  store_chunk(0);
  __syncthreads();
  for (int kc = 0; kc < nchunks; ++kc) {
    const int cur = kc & 1;
    // next chunk (on the last chunk: clamped re-loads, stored to the idle buffer, never read)
    const int kn = kc + 1 < nchunks ? kc + 1 : kc;
    load_chunk(kn * CC);
    const char* base = smem + cur * C::BUF;
    bf16x8 b0[3][C::NT][2], b1[3][C::NT][2];
    read_b(base, 0, b0);
    __builtin_amdgcn_sched_barrier(0);
    // tap row 0 MFMAs | row 1 reads | next chunk's row-0 weights
    read_b(base, 1, b1);
    mfma_row(0, b0);
    load_w_taps(kn, 0, 3);
#pragma unroll
    for (int i = 0; i < 3 * C::NT; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    // tap row 1 MFMAs | row 2 reads | next chunk's row-1 weights
    read_b(base, 2, b0);
    mfma_row(1, b1);
    load_w_taps(kn, 3, 3);
#pragma unroll
    for (int i = 0; i < 3 * C::NT; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 1);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    // tap row 2 MFMAs | next chunk staged into the idle buffer | next chunk's row-2 weights
    mfma_row(2, b0);
    store_chunk(cur ^ 1);
    load_w_taps(kn, 6, 3);
#pragma unroll
    for (int i = 0; i < 9 * C::NT; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 2);
      __builtin_amdgcn_sched_group_barrier(0x080, 1, 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  }

  // ---- epilogue: D[o][t], column t = lane & 31, row o = (r&3) + 8(r>>2) + 4h.  Loads of
  // the residual / mask come from clamped addresses and only the stores are predicated: a
  // load under a per-lane branch would be waited for one element at a time.
  const float* __restrict__ bias = A.bias;
  const float* __restrict__ residual = A.residual;
  const float* __restrict__ mask_src = A.mask_src;
  float* __restrict__ y = A.y;
  const bool want_stats = A.stats != nullptr;
  float st_s[16], st_q[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) st_s[r] = st_q[r] = 0.f;
#pragma unroll
  for (int n = 0; n < C::NT; ++n) {
    const int tt = wt * (C::TB / 2) + n * 32 + (lane & 31);
    const int e = tt / (RB * W);
    const int t = y0 * W + tt % (RB * W);
    const bool ve = b + e < B;
    const float in_stat = (b + e < A.n_stat) ? 1.f : 0.f;
    const int64_t be = ve ? b + e : B - 1;
    const size_t fidx = (((size_t)blockIdx.x * 4 + wv) * C::NT + n) * 64 + lane;
    unsigned obits = 0;
    // epilogue operands: each pointer test is hoisted out of the element loop (a select
    // between a load and a constant inside it makes hipcc branch around every load and wait
    // for it alone: 16 serialised round trips per tile)
    float res[16], msk[16], bia[16];
    size_t off[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      off[r] = ((size_t)be * cout + (o < cout ? o : cout - 1)) * HW + t;
    }
    if (residual) {
#pragma unroll
      for (int r = 0; r < 16; ++r) res[r] = residual[off[r]];
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) res[r] = 0.f;
    }
    if (mask_src) {
#pragma unroll
      for (int r = 0; r < 16; ++r) msk[r] = mask_src[off[r]];
    } else {
      const unsigned mbits = A.mask_in ? A.mask_in[fidx] : 0xffffu;
#pragma unroll
      for (int r = 0; r < 16; ++r) msk[r] = (float)((mbits >> r) & 1u);
    }
    if (bias) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        bia[r] = bias[o < cout ? o : cout - 1];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) bia[r] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      float v = acc[n][r] + bia[r];
      v += res[r];
      if (A.relu) v = fmaxf(v, 0.f);
      if (!(msk[r] > 0.f)) v = 0.f;
      if (ve && o < cout) y[off[r]] = v;
      obits |= (v > 0.f ? 1u : 0u) << r;
      const float vs = v * in_stat;
      st_s[r] += vs;
      st_q[r] += vs * vs;
    }
    if (A.mask_out) A.mask_out[fidx] = (uint16_t)obits;
  }
  if (want_stats) {
    // transpose-reduce the 16 sums + 16 sums of squares over the 32 lanes of this half-wave:
    // afterwards lane J = lane & 31 holds value J (J < 16: sum of row r = J, else sum of
    // squares of row J - 16), summed over the wave's positions
    float v32[32];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      v32[r] = st_s[r];
      v32[16 + r] = st_q[r];
    }
    xreduce_step<16>(v32, lane);
    xreduce_step<8>(v32, lane);
    xreduce_step<4>(v32, lane);
    xreduce_step<2>(v32, lane);
    xreduce_step<1>(v32, lane);
    // the two t-waves of each o half combine through LDS (free after the loop's barrier)
    float* red = reinterpret_cast<float*>(smem);
    if (wt == 1) red[wo * 64 + lane] = v32[0];
    __syncthreads();
    if (wt == 0) {
      const float tot = v32[0] + red[wo * 64 + lane];
      const int J = lane & 31, r = J & 15;
      const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int tile = (int)((b - grp * A.gsize) / E) * A.n_tb + tb;
      if (o < cout)
        A.stats[(((size_t)grp * cout + o) * A.tiles_per_group + tile) * 2 + (J >> 4)] = tot;
    }
  }
}

// pack fp32 weights [cout][cin][3][3] into fragment-major bf16 hi/lo:
// [chunk kc][32-o block][tap][hi|lo][lane 0..63][8], where lane (r, h) of a fragment holds
// W[o = 32*blk + r][c = 16*kc + 8*h + j][tap], j = 0..7 (the A-operand map of
// v_mfma_f32_32x32x16_bf16).  Zero padded to op outputs / cp inputs.  With tflip the packed
// conv is the backward-data conv: out channels = cin, in channels = cout,
// W'[c][o][tap] = W[o][c][8 - tap].
__global__ void pack_kernel(const float* __restrict__ w, int cout, int cin, int tflip, int op,
                            int cp, __bf16* __restrict__ out) {
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
    const int no = tflip ? cin : cout, nc = tflip ? cout : cin;
    float v = 0.f;
    if (o < no && c < nc)
      v = tflip ? w[((size_t)c * cin + o) * 9 + (8 - tap)] : w[((size_t)o * cin + c) * 9 + tap];
    const __bf16 hi = (__bf16)v;
    out[i] = pr == 0 ? hi : (__bf16)(v - (float)hi);
  }
}

template <int W, int RB, int E>
static int launch(Args a, hipStream_t st) {
  using C = Cfg<W, RB, E>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_kernel<W, RB, E>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  DD_REQUIRE(a.H % RB == 0, "dd_conv3x3_forward: H must be a multiple of the row block");
  DD_REQUIRE(a.gsize % E == 0, "dd_conv3x3_forward: group_size %d must be a multiple of %d "
             "(images per tile at %dx%d)", a.gsize, E, a.H, W);
  a.n_tb = a.H / RB;
  a.n_ob = a.op / 64;
  a.tiles_per_group = (a.gsize / E) * a.n_tb;
  const int64_t grid = ceil_div(a.B, E) * a.n_tb * a.n_ob;
  DD_REQUIRE(grid < (1ll << 31), "dd_conv3x3_forward: grid too large");
  conv3x3_kernel<W, RB, E><<<(unsigned)grid, 256, C::LDS, st>>>(a);
  DD_CHECK_LAUNCH("dd_conv3x3_forward");
  return DD_OK;
}

// tile geometry the kernel uses for an h x w image: rows per tile, images per tile (two 8x8
// images per tile only when they always share a BN group)
static bool tile_geometry(int h, int w, int gsize, int* rb, int* e) {
  if (w == 32 && h % 4 == 0) { *rb = 4; *e = 1; return true; }
  if (w == 16 && h % 8 == 0) { *rb = 8; *e = 1; return true; }
  if (w == 8 && h == 8 && gsize % 2 == 0) { *rb = 8; *e = 2; return true; }
  if (w == 8 && h % 8 == 0) { *rb = 8; *e = 1; return true; }
  if (w == 4 && h == 4) { *rb = 4; *e = 4; return true; }
  return false;
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
                    void* packed, void* stream) {
  clear_error();
  DD_REQUIRE(w && packed && cout > 0 && cin > 0, "dd_conv3x3_pack: bad arguments");
  const int no = transpose_flip ? cin : cout, nc = transpose_flip ? cout : cin;
  const int op = conv::pad_to(no, 64), cp = conv::pad_to(nc, conv::CC);
  const int total = 2 * 9 * op * cp;
  conv::pack_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 4096), 256, 0,
                      as_stream(stream)>>>(w, cout, cin, transpose_flip, op, cp,
                                           static_cast<__bf16*>(packed));
  DD_CHECK_LAUNCH("dd_conv3x3_pack");
  return DD_OK;
}

size_t dd_conv3x3_mask_bytes(int64_t B, int32_t cout, int32_t h, int32_t w) {
  int rb, e;
  if (B <= 0 || cout <= 0 || !conv::tile_geometry(h, w, 2, &rb, &e)) return 0;
  const int64_t blocks = ceil_div(B, e) * (h / rb) * (conv::pad_to(cout, 64) / 64);
  return (size_t)blocks * 4 * (e * rb * w / 64) * 64 * sizeof(uint16_t);
}

int dd_conv3x3_tiles_per_group(int32_t h, int32_t w, int32_t group_size) {
  int rb, e;
  if (group_size <= 0 || !conv::tile_geometry(h, w, group_size, &rb, &e) || group_size % e)
    return -1;
  return (group_size / e) * (h / rb);
}

int dd_conv3x3_forward(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                       const void* packed, int32_t cout, const float* bias,
                       const float* residual, const float* mask_src, int32_t relu,
                       const float* in_scale, const float* in_shift, int32_t in_relu,
                       int32_t group_size, int64_t n_stat, float* stats, uint16_t* mask_out,
                       const uint16_t* mask_in, float* y, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && cin > 0 && cout > 0 && h > 0, "dd_conv3x3_forward: bad sizes");
  if (B == 0) return DD_OK;
  DD_REQUIRE(x && packed && y, "dd_conv3x3_forward: null buffer");
  DD_REQUIRE((int64_t)cin * h * w < (1ll << 31) && (int64_t)cout * h * w < (1ll << 31),
             "dd_conv3x3_forward: per-example tensor too large");
  DD_REQUIRE(!in_scale == !in_shift, "dd_conv3x3_forward: in_scale and in_shift go together");
  const bool grouped = in_scale || stats;
  DD_REQUIRE(!grouped || group_size > 0, "dd_conv3x3_forward: group_size must be positive");
  int rb, e;
  if (!conv::tile_geometry(h, w, grouped ? group_size : 2, &rb, &e)) {
    set_error("dd_conv3x3_forward: unsupported spatial shape %dx%d (W in {8,16,32} with H a "
              "multiple of the row block, or 8x8 / 4x4)", h, w);
    return DD_EINVAL;
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
  a.relu = relu;
  a.gsize = grouped ? group_size : (int)std::min<int64_t>(B + e, 1 << 30) / e * e;
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
  hipStream_t st = as_stream(stream);
  if (w == 32) return conv::launch<32, 4, 1>(a, st);
  if (w == 16) return conv::launch<16, 8, 1>(a, st);
  if (w == 8 && h == 8 && a.gsize % 2 == 0) return conv::launch<8, 8, 2>(a, st);
  if (w == 8) return conv::launch<8, 8, 1>(a, st);
  return conv::launch<4, 4, 4>(a, st);
}

}  // extern "C"
