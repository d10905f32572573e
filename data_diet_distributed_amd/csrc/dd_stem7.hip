// The ImageNet stem's 7x7 / stride 2 / pad 3 conv (3 -> 64 channels; reference
// models/resnet.py:35-63 with the ImageNet stem) on split MFMA, EL2N launch
// shape only: y raw, grouped train-mode BN partial statistics out.
//
//   y[b][o][yo][xo] = sum_{c, ky, kx} W[o][c][ky][kx] x[b][c][2 yo + ky - 3][2 xo + kx - 3]
//
// The implicit GEMM (dd_conv1x1.hip mode 3) gathers the 147-row K of every 128-position tile
// from global memory, chunk after chunk: 0.06 of the split peak.  Here a workgroup owns one
// image's pair of output rows: the 9 input rows they read (3 channels, zero-padded) are staged
// once in LDS as fp32, and K is ordered (c, ky, kx8) with kx8 = 0..7 (kx = 7 a zero weight), so
// a B fragment -- 8 consecutive K values of one output position -- is 8 consecutive columns of
// one staged row: four 8-byte LDS reads, split into hi / lo halves in registers.  21 (c, ky)
// rows = 11 K steps of 16 (the last half zero).  4 waves: output row (wave / 2) of the pair x
// two 32-position column tiles, each against both 32-output blocks (64 outputs); the padded
// columns past the map (a 112-wide map on 128 tile columns) are never stored or counted.
// Epilogue as the conv kernels': transpose through a wave-private LDS block, float4 stores,
// one BN partial per (channel, 32-position fragment).
#include "dd_mfma.h"

namespace dd {
namespace stem7 {

using namespace conv;

constexpr int KS = 11;    // K steps of 16: 21 (c, ky) rows of 8 kx values, padded to 22
constexpr int NOB = 2;    // 32-output blocks (cout <= 64)
constexpr int LP = 264;   // staged row pitch (floats): columns -3 .. 260 of the input
constexpr int NR = 9;     // input rows per output-row pair
constexpr int PLANE = NR * LP;
constexpr int NFRAG = 8;  // 32-position fragments per output-row pair (2 rows x 4)

struct Args {
  const float* x;        // [B][3][H][W]
  const __bf16* wpack;   // dd_stem7_pack
  float* y;              // [B][cout][Ho][Wo]
  float* stats;          // [G][cout][tiles_per_group][2]
  int64_t B, n_stat;
  int H, W, Ho, Wo, cout, gsize, n_rp, tiles_per_group;
  float acc_scale;
};

template <bool F16>
__global__ __launch_bounds__(256, 2) void stem7_kernel(const Args A) {
  __shared__ __attribute__((aligned(16))) float img[3 * PLANE];
  __shared__ __attribute__((aligned(16))) float ep_all[4 * 1024];
  const int64_t b = blockIdx.x / A.n_rp;
  const int rp = (int)(blockIdx.x - b * A.n_rp);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5;
  const int H = A.H, W = A.W;

  // ---- stage the 9 input rows 4 rp - 3 .. 4 rp + 5 of the 3 channels, zero-padded: a wave per
  // staged row, every LDS slot written once (the image value or the padding's zero)
  // (all of a lane's loads are issued before the first LDS store: one memory round trip per
  // workgroup instead of one per staged row)
  const float* __restrict__ xb = A.x + b * 3 * (int64_t)H * W;
  constexpr int RPW = (3 * NR + 3) / 4, CPL = (LP + 63) / 64;  // rows per wave, slots per lane
  float sv[RPW][CPL];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int cr = wv + 4 * k;
    const int c = cr / NR, r = cr - c * NR, ir = 4 * rp - 3 + r;
    const bool rok = cr < 3 * NR && ir >= 0 && ir < H;
    const float* __restrict__ src = xb + ((int64_t)(rok ? c : 0) * H + (rok ? ir : 0)) * W;
#pragma unroll
    for (int m = 0; m < CPL; ++m) {
      const int col = lane + 64 * m - 3;
      const bool ok = rok && col >= 0 && col < W;
      sv[k][m] = src[ok ? col : 0];
      sv[k][m] = ok ? sv[k][m] : 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int cr = wv + 4 * k;
    if (cr >= 3 * NR) continue;
    const int c = cr / NR, r = cr - c * NR;
    float* dst = img + c * PLANE + r * LP;
#pragma unroll
    for (int m = 0; m < CPL; ++m)
      if (lane + 64 * m < LP) dst[lane + 64 * m] = sv[k][m];
  }
  __syncthreads();

  // ---- K loop: this wave's output row (of the pair) and column tiles
  const int row = wv >> 1, tc0 = (wv & 1) * 2;
  floatx16 acc[NOB][2];
#pragma unroll
  for (int a = 0; a < NOB; ++a)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[a][n] = floatx16{0};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    bf16x8 ah[NOB], al[NOB];
#pragma unroll
    for (int a = 0; a < NOB; ++a) {
      const __bf16* p = A.wpack + ((size_t)(s * NOB + a) * 2) * 512 + lane * 8;
      ah[a] = *reinterpret_cast<const bf16x8*>(p);
      al[a] = *reinterpret_cast<const bf16x8*>(p + 512);
    }
    // this half-wave's (c, ky) row (the padded 22nd reads a real row against zero weights)
    const int q = min(2 * s + h, 20), c = q / 7, ky = q - 7 * c;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int xo = (tc0 + n) * 32 + (lane & 31);
      // input columns 2 xo - 3 + kx8 = staged columns 2 xo + kx8 (8-byte aligned)
      const float* src = img + c * PLANE + (2 * row + ky) * LP + 2 * xo;
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 t = *reinterpret_cast<const float2*>(src + 2 * j);
        v[2 * j] = t.x;
        v[2 * j + 1] = t.y;
      }
      uint32_t hv[4], lv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hv[j] = pack2<F16>(v[2 * j], v[2 * j + 1]);
        lv[j] = pack2<F16>(v[2 * j] - half_lo<F16>(hv[j]), v[2 * j + 1] - half_hi<F16>(hv[j]));
      }
      const bf16x8 bh = __builtin_bit_cast(bf16x8, make_uint4(hv[0], hv[1], hv[2], hv[3]));
      const bf16x8 bl = __builtin_bit_cast(bf16x8, make_uint4(lv[0], lv[1], lv[2], lv[3]));
#pragma unroll
      for (int a = 0; a < NOB; ++a) {
        floatx16 d = acc[a][n];
        d = mfma16<F16>(ah[a], bh, d);
        d = mfma16<F16>(ah[a], bl, d);
        d = mfma16<F16>(al[a], bh, d);
        acc[a][n] = d;
      }
    }
  }

  // ---- epilogue: per 32 x 32 fragment, transposed through this wave's 4 KB block so a lane
  // owns 4 consecutive positions of one channel; BN partials summed over a channel's 8 lanes
  float* ep = ep_all + wv * 1024;
  const int tl = lane & 7, ol = lane >> 3;
  const int yo = 2 * rp + row;
  const int64_t grp = b / A.gsize;
  const float in_stat = (b < A.n_stat && yo < A.Ho) ? 1.f : 0.f;
#pragma unroll
  for (int a = 0; a < NOB; ++a)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ep[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + (lane & 31)] =
            F16 ? acc[a][n][r] * A.acc_scale : acc[a][n][r];
      asm volatile("" ::: "memory");
      float4 vv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) vv[k] = *reinterpret_cast<const float4*>(ep + (8 * k + ol) * 32 + 4 * tl);
      asm volatile("" ::: "memory");
      const int xo = (tc0 + n) * 32 + 4 * tl;
      const bool ok = xo < A.Wo && yo < A.Ho;  // (Wo % 4 == 0: whole quads)
      const float st = ok ? in_stat : 0.f;
      const int pi = (int)((b - grp * A.gsize) * A.n_rp * NFRAG) + rp * NFRAG + row * 4 + tc0 + n;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int o = a * 32 + ol + 8 * k;
        const float4 u = vv[k];
        if (ok && o < A.cout)
          store_out4(A.y + ((b * A.cout + o) * (int64_t)A.Ho + yo) * A.Wo + xo, u.x, u.y, u.z, u.w);
        float s_ = (u.x + u.y + u.z + u.w) * st;
        float q_ = (u.x * u.x + u.y * u.y + u.z * u.z + u.w * u.w) * st;
        s_ = sum8(s_);
        q_ = sum8(q_);
        if (tl == 0 && o < A.cout)
          *reinterpret_cast<float2*>(A.stats + (((size_t)grp * A.cout + o) * A.tiles_per_group + pi) * 2) =
              make_float2(s_, q_);
      }
      asm volatile("" ::: "memory");  // the next fragment reuses the block (in order per wave)
    }
}

// W [cout][3][7][7] -> [s][ob][hi|lo][lane][8]: lane (o = 32 ob + lane % 32, h = lane / 32),
// element j = W[o][c][ky][j] for (c, ky) = row 2 s + h (j = 7 and rows >= 21: zero)
__global__ void pack_kernel(const float* __restrict__ w, int cout, int f16, float scale,
                            __bf16* __restrict__ out) {
  const int total = KS * NOB * 2 * 512;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int j = i & 7, lane = (i >> 3) & 63, rest = i >> 9;
    const int pr = rest & 1, ob = (rest >> 1) % NOB, s = (rest >> 1) / NOB;
    const int o = ob * 32 + (lane & 31), q = 2 * s + (lane >> 5);
    float v = 0.f;
    if (o < cout && q < 21 && j < 7) v = w[((size_t)o * 3 + q / 7) * 49 + (q % 7) * 7 + j] * scale;
    __bf16 hi, lo;
    if (f16)
      split16<true>(v, hi, lo);
    else
      split16<false>(v, hi, lo);
    out[i] = pr == 0 ? hi : lo;
  }
}

}  // namespace stem7
}  // namespace dd

using namespace dd;

extern "C" {

size_t dd_stem7_pack_bytes(void) { return (size_t)stem7::KS * stem7::NOB * 2 * 512 * sizeof(__bf16); }

int dd_stem7_pack(const float* w, int32_t cout, int32_t operands, float scale, void* packed,
                  void* stream) {
  clear_error();
  DD_REQUIRE(w && packed && cout > 0 && cout <= 32 * stem7::NOB, "dd_stem7_pack: bad arguments");
  DD_REQUIRE(operands == DD_OPERANDS_BF16X3 || operands == DD_OPERANDS_F16X3,
             "dd_stem7_pack: operands must be DD_OPERANDS_BF16X3 or DD_OPERANDS_F16X3");
  DD_REQUIRE(operand_scale_ok(operands, scale),
             "dd_stem7_pack: scale must be 1 (bf16 operands) or a power of two (fp16)");
  stem7::pack_kernel<<<64, 256, 0, as_stream(stream)>>>(w, cout, operands == DD_OPERANDS_F16X3,
                                                        scale, static_cast<__bf16*>(packed));
  DD_CHECK_LAUNCH("dd_stem7_pack");
  return DD_OK;
}

int dd_stem7_supported(int32_t h, int32_t w, int32_t cin, int32_t cout, int32_t group_size) {
  const int wo = w / 2;
  return cin == 3 && cout > 0 && cout <= 32 * stem7::NOB && h > 0 && h % 2 == 0 && w % 2 == 0 &&
                 wo % 4 == 0 && wo <= 128 && group_size > 0
             ? 1
             : 0;
}

int dd_stem7_tiles_per_group(int32_t h, int32_t w, int32_t group_size) {
  if (!dd_stem7_supported(h, w, 3, 64, group_size)) return -1;
  return group_size * ((h / 2 + 1) / 2) * stem7::NFRAG;
}

int dd_stem7_forward(const float* x, int64_t B, int32_t h, int32_t w, const void* packed,
                     int32_t cout, int32_t group_size, int64_t n_stat, float* stats, float* y,
                     int32_t operands, float acc_scale, void* stream) {
  clear_error();
  DD_REQUIRE(B >= 0 && dd_stem7_supported(h, w, 3, cout, group_size),
             "dd_stem7_forward: unsupported shape (3 -> %d at %dx%d, group %d)", cout, h, w,
             group_size);
  DD_REQUIRE(operands == DD_OPERANDS_BF16X3 || operands == DD_OPERANDS_F16X3,
             "dd_stem7_forward: operands must be DD_OPERANDS_BF16X3 or DD_OPERANDS_F16X3");
  DD_REQUIRE(operand_scale_ok(operands, acc_scale),
             "dd_stem7_forward: acc_scale must be 1 (bf16 operands) or a power of two (fp16)");
  if (B == 0) return DD_OK;
  DD_REQUIRE(x && packed && stats && y, "dd_stem7_forward: null buffer");
  stem7::Args a{};
  a.x = x;
  a.wpack = static_cast<const __bf16*>(packed);
  a.y = y;
  a.stats = stats;
  a.B = B;
  a.n_stat = std::min<int64_t>(std::max<int64_t>(n_stat, 0), B);
  a.H = h;
  a.W = w;
  a.Ho = h / 2;
  a.Wo = w / 2;
  a.cout = cout;
  a.gsize = group_size;
  a.n_rp = (a.Ho + 1) / 2;
  a.tiles_per_group = group_size * a.n_rp * stem7::NFRAG;
  a.acc_scale = acc_scale;
  const int64_t grid = B * a.n_rp;
  DD_REQUIRE(grid < (1ll << 31), "dd_stem7_forward: too many workgroups");
  if (operands == DD_OPERANDS_F16X3)
    stem7::stem7_kernel<true><<<(unsigned)grid, 256, 0, as_stream(stream)>>>(a);
  else
    stem7::stem7_kernel<false><<<(unsigned)grid, 256, 0, as_stream(stream)>>>(a);
  DD_CHECK_LAUNCH("dd_stem7_forward");
  return DD_OK;
}

}  // extern "C"
