// GraNd per-example conv weight-gradient norms for small feature maps by the shifted-Gram
// ghost identity (split-bf16 MFMA).  The reference has no GraNd; the layers are
// the Conv2d of models/resnet.py:12-23 at 8x8 and 4x4 (ResNet-18 layer3 / layer4, their
// stride-2 heads and 1x1 projections).
//
// With U the im2col of one example's input a [cin][Ti] (t = output position, m = (c, tap)) and
// g [cout][To] its output gradient:
//   ||U^T g^T||_F^2 = sum_{t,t'} K_a[t][t'] K_g[t][t'],   K_g = g^T g   (over cout),
//   K_a[t][t'] = sum_{c,tap} a[c][p(t,tap)] a[c][p(t',tap)] = sum_tap P[p(t,tap)][p(t',tap)]
// where P = a^T a is the Ti x Ti Gram of input positions over channels and p(t, tap) the input
// position a tap reads (a zero-padding tap contributes nothing).  The usual ghost norm builds
// K_a over d_a = 9 cin (2 To^2 9 cin flop); here P costs 2 Ti^2 cin and the 9-tap sum is a
// gather from LDS, so a layer4 conv needs ~1 MFLOP per example instead of the 75 MFLOP of the
// direct weight gradient, and the kernel is bound by reading a and g once from HBM.
//
// One workgroup per example, 4 waves.  Channel chunks of 64 are staged into LDS as bf16 hi|lo
// [c][position] images (one float4 per lane per 16 positions, register prefetch of the next
// chunk); 32x32 Gram tiles come from v_mfma_f32_32x32x16_bf16 with both operands read by the
// transposed LDS read (a Gram's A and B fragments of a position block are the same register).
// 64 positions = 2x2 tiles (one per wave); 32 positions = one tile, K split over the 4 waves.
// P goes to LDS in fp32; each lane then forms K_a for its K_g accumulator entries with 9 LDS
// gathers and accumulates K_a * K_g.  The per-example total is added to sq_accum[b] by that
// example's only workgroup (deterministic, no atomics).
#include "dd_mfma.h"
#include "dd_pgram.h"

#include <stdlib.h>

namespace dd {
namespace pgram {

using namespace conv;

constexpr int CH = 64;  // channels per staged chunk

struct Args {
  const float* act;
  const float* gout;
  const float* col_scale;
  float* sq;
  int cin, cout, hi, wi, ho, wo, k, stride, pad;
};

template <int TP>
struct Stage {
  static constexpr int ROWB = TP == 64 ? 192 : 64;  // bf16 row pitch, bank-conflict-free reads
  static constexpr int BYTES = 2 * CH * ROWB;       // [hi|lo][c][pos]
  static constexpr int NF4 = CH * TP / 4;
  static constexpr int NST = NF4 / 256;
  static_assert(NF4 % 256 == 0, "whole float4 per thread");
};

// Position map of a Gram: plain (u is the position in a plane of `plane` elements) or one
// parity class (py, px) of a 2x-decimated plane of width wi: u = i * (wi / 2) + j reads
// element (2i + py) * wi + 2j + px.
struct PosMap {
  int plane;     // elements per channel plane
  int cls;       // -1: plain; else py * 2 + px
  int wi;        // plane width (parity mode)
  __device__ __forceinline__ int at(int u) const {
    if (cls < 0) return u;
    const int wc = wi >> 1;
    return (2 * (u / wc) + (cls >> 1)) * wi + 2 * (u % wc) + (cls & 1);
  }
};

// Pieces of a Gram over channels of x [nch][plane] at the npos positions of `pm` (the rest
// zero), scaled per channel by scale[c]^2 when given.  A wave's accumulator is one 32x32 tile
// (64 positions: 2x2 tiles, one per wave) or one K slice of the single tile (32 positions: K
// split over the 4 waves, the caller sums the four partials).  buf: two Stage<TP>::BYTES
// buffers.
template <int TP>
struct Gram {
  using S = Stage<TP>;
  const float* __restrict__ x;
  const float* __restrict__ scale;
  int nch, npos;
  PosMap pm;

  __device__ __forceinline__ int nchunks() const { return (nch + CH - 1) / CH; }

  // one chunk's float4s of this thread (clamped addresses, zeros outside)
  __device__ __forceinline__ void load(float4 (&r)[S::NST], int c0) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < S::NST; ++k) {
      const int i = tid + 256 * k;
      const int c = i / (TP / 4), u4 = i % (TP / 4);
      const int cg = c0 + c;
      const bool ok = cg < nch && u4 * 4 < npos;
      const float* src = x + (size_t)(cg < nch ? cg : nch - 1) * pm.plane;
      float4 v;
      if (pm.cls < 0) {  // wave-uniform
        v = *reinterpret_cast<const float4*>(src + (ok ? u4 * 4 : 0));
      } else {           // strided class positions: four scalar loads
        const int u0 = ok ? u4 * 4 : 0;
        v = make_float4(src[pm.at(u0)], src[pm.at(u0 + 1)], src[pm.at(u0 + 2)],
                        src[pm.at(u0 + 3)]);
      }
      const float s = scale ? scale[cg < nch ? cg : nch - 1] : 1.f;
      v = make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
      r[k] = keep_if(v, ok);
    }
  }

  __device__ __forceinline__ static void store(const float4 (&r)[S::NST], char* dst) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < S::NST; ++k) {
      const int i = tid + 256 * k;
      const int c = i / (TP / 4), u4 = i % (TP / 4);
      const float f[4] = {r[k].x, r[k].y, r[k].z, r[k].w};
      __bf16 hv[4], lv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) split_bf16(f[j], hv[j], lv[j]);
      char* pp = dst + c * S::ROWB + u4 * 8;
      *reinterpret_cast<bf16x4*>(pp) = bf16x4{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<bf16x4*>(pp + CH * S::ROWB) = bf16x4{lv[0], lv[1], lv[2], lv[3]};
    }
  }

  __device__ __forceinline__ static void multiply(floatx16& acc, const char* cur) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, h = lane >> 5;
    const int q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
    const int U = TP == 64 ? (wv >> 1) : 0, V = TP == 64 ? (wv & 1) : 0;
    const int ks0 = TP == 64 ? 0 : wv, ks1 = TP == 64 ? 4 : wv + 1;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks < ks0 || ks >= ks1) continue;  // wave-uniform
      const char* rowp = cur + (ks * 16 + 8 * h + q) * S::ROWB;
      const char* au = rowp + (U * 32 + 16 * g1 + 4 * p) * 2;
      const char* av = rowp + (V * 32 + 16 * g1 + 4 * p) * 2;
      const bf16x8 uh = tr_read8(au, au + 4 * S::ROWB);
      const bf16x8 ul = tr_read8(au + CH * S::ROWB, au + CH * S::ROWB + 4 * S::ROWB);
      const bf16x8 vh = tr_read8(av, av + 4 * S::ROWB);
      const bf16x8 vl = tr_read8(av + CH * S::ROWB, av + CH * S::ROWB + 4 * S::ROWB);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uh, vh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uh, vl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ul, vh, acc, 0, 0, 0);
    }
  }

  // streaming: two register sets, chunk k + 2's loads in flight while chunk k is multiplied
  // and chunk k + 1 is staged (any channel count)
  __device__ floatx16 run(char* buf) const {
    float4 r0[S::NST], r1[S::NST];
    floatx16 acc = floatx16{0};
    const int n = nchunks();
    char* buf0 = buf;
    char* buf1 = buf + S::BYTES;
    load(r0, 0);
    if (n > 1) load(r1, CH);
    store(r0, buf0);
    __syncthreads();
    for (int kc = 0; kc < n; kc += 2) {
      if (kc + 2 < n) load(r0, (kc + 2) * CH);
      multiply(acc, buf0);
      if (kc + 1 < n) store(r1, buf1);
      __syncthreads();
      if (kc + 1 >= n) break;
      if (kc + 3 < n) load(r1, (kc + 3) * CH);
      multiply(acc, buf1);
      if (kc + 2 < n) store(r0, buf0);
      __syncthreads();
    }
    return acc;
  }

  // preloaded: up to MAXC chunks (16 float4 per thread) issued at once, so a whole example
  // costs one global-load round trip instead of one per chunk; every slot is loaded (slots
  // past the channel count read clamped addresses and stay zero), which keeps the waitcnt
  // counts exact
  static constexpr int MAXC = 16 / S::NST;
  __device__ __forceinline__ bool fits() const { return nch <= MAXC * CH; }
  __device__ __forceinline__ void preload(float4 (&r)[MAXC][S::NST]) const {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) load(r[c], c * CH);
  }
  __device__ floatx16 run_pre(const float4 (&r)[MAXC][S::NST], char* buf) const {
    floatx16 acc = floatx16{0};
    const int n = nchunks();
    store(r[0], buf);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < n) {  // uniform
        if (c + 1 < n && c + 1 < MAXC) store(r[c + 1 < MAXC ? c + 1 : c], buf + ((c + 1) & 1) * S::BYTES);
        multiply(acc, buf + (c & 1) * S::BYTES);
        __syncthreads();
      }
    }
    return acc;
  }
};

// padded input positions (hi + 2 pad) x (wi + 2 pad) a P_pad region holds per TPI class
template <int TPI>
struct PadCap {
  static constexpr int NPP = TPI == 64 ? 112 : 48;
  static constexpr int BYTES = NPP * (NPP + 1) * 4;
};

// q = n / d for 0 <= n < 2^12, d >= 1 (exact: (n + 0.5) / d is never within 0.5/d of an integer)
__device__ __forceinline__ int small_div(int n, float inv_d) {
  return (int)(((float)n + 0.5f) * inv_d);
}

// K_g first (it stays in registers), then P = a^T a, written into a zero-padded P_pad over
// the (hi + 2 pad) x (wi + 2 pad) padded input grid in the staging region the Grams are done
// with.  A padding position's row and column are zero, so K_a[t][t'] = sum_tap
// P_pad[pp(t) + d_tap][pp(t') + d_tap] (pp = the padded position of output t's window origin,
// d_tap = ky * PW + kx) needs no bounds test: one add and one LDS read per (entry, tap).
// Entries past To carry K_g = 0 (the Gram of zero-padded rows), their indices are clamped.
template <int TPI, int TPO>
__global__ __launch_bounds__(256) void pgram_kernel(const Args A) {
  constexpr int SB = 2 * (Stage<TPI>::BYTES > Stage<TPO>::BYTES ? Stage<TPI>::BYTES
                                                                : Stage<TPO>::BYTES);
  constexpr int PARTB = TPI == 64 ? 0 : 4 * 32 * 32 * 4;  // K-slice partials (32 positions)
  constexpr int PR = PadCap<TPI>::BYTES + PARTB;
  constexpr int LDSB = SB > PR ? SB : PR;
  __shared__ __attribute__((aligned(16))) char smem[LDSB + 64];
  char* sbuf = smem;
  float* Pp = reinterpret_cast<float*>(smem);
  float* part = reinterpret_cast<float*>(smem + PadCap<TPI>::BYTES);
  float* red = reinterpret_cast<float*>(smem + LDSB);

  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5;
  const int Ti = A.hi * A.wi, To = A.ho * A.wo;
  const int PW = A.wi + 2 * A.pad, NPP = (A.hi + 2 * A.pad) * PW, PPP = NPP + 1;
  const float inv_wi = 1.f / (float)A.wi, inv_wo = 1.f / (float)A.wo;

  const Gram<TPI> ga{A.act + (size_t)b * A.cin * Ti, nullptr, A.cin, Ti, PosMap{Ti, -1, A.wi}};
  const Gram<TPO> gg{A.gout + (size_t)b * A.cout * To, A.col_scale, A.cout, To,
                     PosMap{To, -1, A.wo}};
  // ---- K_g = g^T g over output channels (BN-folded scale s_o^2 applied as g * s_o), then
  // P = a^T a over input channels; both operands in flight at once when they fit the
  // registers (the ResNet-18 layer3 / layer4 shapes)
  floatx16 kg, pa;
  if (ga.fits() && gg.fits()) {  // uniform
    float4 ra[Gram<TPI>::MAXC][Stage<TPI>::NST], rg[Gram<TPO>::MAXC][Stage<TPO>::NST];
    gg.preload(rg);
    ga.preload(ra);
    kg = gg.run_pre(rg, sbuf);
    pa = ga.run_pre(ra, sbuf);
  } else {
    kg = gg.run(sbuf);
    pa = ga.run(sbuf);
  }
  // ---- P_pad: zero, then the interior (run_pre / run end with a barrier)
  for (int i = tid; i < NPP * PPP; i += 256) Pp[i] = 0.f;
  auto pad_of = [&](int u) {
    const int y = small_div(u, inv_wi);
    return (y + A.pad) * PW + (u - y * A.wi) + A.pad;
  };
  if (TPI == 64) {
    __syncthreads();
    const int U = wv >> 1, V = wv & 1;
    const int v = V * 32 + (lane & 31);
    const int pv = pad_of(v < Ti ? v : 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int u = U * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (u < Ti && v < Ti) Pp[pad_of(u) * PPP + pv] = pa[r];
    }
  } else {
    // four K-slice partials, summed in a fixed order
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int u = (r & 3) + 8 * (r >> 2) + 4 * h;
      part[(wv * 32 + u) * 32 + (lane & 31)] = pa[r];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = tid + 256 * j, u = e >> 5, v = e & 31;
      const float s4 = (part[e] + part[1024 + e]) + (part[2048 + e] + part[3072 + e]);
      if (u < Ti && v < Ti) Pp[pad_of(u) * PPP + pad_of(v)] = s4;
    }
  }
  __syncthreads();

  // ---- sum_{t,t'} K_a[t][t'] K_g[t][t'] over this wave's K_g entries
  const int T1 = TPO == 64 ? (wv >> 1) : 0, T2 = TPO == 64 ? (wv & 1) : 0;
  auto origin = [&](int t) {  // padded position of output t's window origin (tap 0, 0)
    t = t < To ? t : 0;
    const int yo = small_div(t, inv_wo);
    return A.stride * yo * PW + A.stride * (t - yo * A.wo);
  };
  const int p2 = origin(T2 * 32 + (lane & 31));
  const int ntap = A.k * A.k;
  int dt[9];  // d_tap * (PPP + 1): the same tap shift on both sides
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
    dt[tap] = ((A.k == 3 ? tap / 3 : 0) * PW + (A.k == 3 ? tap % 3 : 0)) * (PPP + 1);
  float tot = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int t1 = T1 * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    const float* base = Pp + origin(t1) * PPP + p2;
    float ka = base[dt[0]];
    if (ntap == 9) {  // uniform
#pragma unroll
      for (int tap = 1; tap < 9; ++tap) ka += base[dt[tap]];
    }
    tot += ka * kg[r];
  }
  tot = wave_sum(tot);
  if (lane == 0) red[wv] = tot;
  __syncthreads();
  if (tid == 0) A.sq[b] += (red[0] + red[1]) + (red[2] + red[3]);
}

// Stride 2 over a 16 x 16 input: tap (ky, kx) reads input parity class ((ky - 1) & 1,
// (kx - 1) & 1) only, so K_a = sum over the 4 classes of class-Gram gathers.  K_g first (kept
// in registers); then chunks of 16 channels x 256 positions are loaded as contiguous float4
// rows and de-interleaved while staged into four 8 x 8 class images [cls][hi|lo][c][64]; each
// wave accumulates its 32 x 32 tile of all four class Grams.  Class by class, P_c goes into a
// zero-padded 9 x 9 grid (class row/column -1 is the padding), where the class position a tap
// reads for output (yo, xo) is (yo + (ky > 0), xo + (kx > 0)): no bounds tests in the gather.
// A 1x1 / pad 0 conv is tap (1, 1) of the same scheme.
__global__ __launch_bounds__(256, 2) void pgram_par_kernel(const Args A) {
  constexpr int ROWB = 192;             // bf16 class-image row pitch (64 positions, padded)
  constexpr int CC16 = 16;              // channels per chunk
  constexpr int IMG = 2 * CC16 * ROWB;  // one class: [hi|lo][c][pos]
  constexpr int BUFB = 4 * IMG;
  constexpr int GP = 9, NPP = GP * GP, PPP = NPP + 1;
  constexpr int SB = 2 * (BUFB > Stage<64>::BYTES ? BUFB : Stage<64>::BYTES);
  constexpr int PB = NPP * PPP * 4;
  static_assert(PB <= SB, "P_pad aliases the staging buffers");
  __shared__ __attribute__((aligned(16))) char smem[SB + 64];
  float* Pp = reinterpret_cast<float*>(smem);
  float* red = reinterpret_cast<float*>(smem + SB);

  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5;
  const int To = A.ho * A.wo;  // 64
  const int cin = A.cin;

  // ---- K_g (TPO = 64)
  floatx16 kg;
  {
    const Gram<64> gg{A.gout + (size_t)b * A.cout * To, A.col_scale, A.cout, To,
                      PosMap{To, -1, A.wo}};
    if (gg.fits()) {
      float4 rg[Gram<64>::MAXC][Stage<64>::NST];
      gg.preload(rg);
      kg = gg.run_pre(rg, smem);
    } else {
      kg = gg.run(smem);
    }
  }

  // ---- the four class Grams, 16-channel chunks of the whole 16 x 16 plane
  const float* __restrict__ xa = A.act + (size_t)b * cin * 256;
  auto load = [&](float4 (&r)[4], int c0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int qd = tid + 256 * k, c = qd >> 6, cg = c0 + c;
      const float4 v = *reinterpret_cast<const float4*>(
          xa + (size_t)(cg < cin ? cg : cin - 1) * 256 + (qd & 63) * 4);
      r[k] = keep_if(v, cg < cin);
    }
  };
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  auto store = [&](const float4 (&r)[4], char* dst) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int qd = tid + 256 * k, c = qd >> 6, p4 = qd & 63;
      const int y = p4 >> 2, x0 = (p4 & 3) * 4;           // row, first column
      const int u = (y >> 1) * 8 + (x0 >> 1);             // class position of x0 (and x0 + 1)
      char* e = dst + ((y & 1) * 2) * IMG + c * ROWB + u * 2;  // class (py, 0)
      char* o = e + IMG;                                       // class (py, 1)
      __bf16 h0, l0, h1, l1, h2, l2, h3, l3;
      split_bf16(r[k].x, h0, l0);
      split_bf16(r[k].y, h1, l1);
      split_bf16(r[k].z, h2, l2);
      split_bf16(r[k].w, h3, l3);
      *reinterpret_cast<bf16x2*>(e) = bf16x2{h0, h2};
      *reinterpret_cast<bf16x2*>(e + CC16 * ROWB) = bf16x2{l0, l2};
      *reinterpret_cast<bf16x2*>(o) = bf16x2{h1, h3};
      *reinterpret_cast<bf16x2*>(o + CC16 * ROWB) = bf16x2{l1, l3};
    }
  };
  const int q = (lane >> 2) & 3, pl = lane & 3, g1 = (lane >> 4) & 1;
  const int U = wv >> 1, V = wv & 1;
  floatx16 pc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) pc[c] = floatx16{0};
  auto multiply = [&](const char* cur) {
#pragma unroll
    for (int cls = 0; cls < 4; ++cls) {
      const char* rowp = cur + cls * IMG + (8 * h + q) * ROWB;
      const char* au = rowp + (U * 32 + 16 * g1 + 4 * pl) * 2;
      const char* av = rowp + (V * 32 + 16 * g1 + 4 * pl) * 2;
      const bf16x8 uh = tr_read8(au, au + 4 * ROWB);
      const bf16x8 ul = tr_read8(au + CC16 * ROWB, au + CC16 * ROWB + 4 * ROWB);
      const bf16x8 vh = tr_read8(av, av + 4 * ROWB);
      const bf16x8 vl = tr_read8(av + CC16 * ROWB, av + CC16 * ROWB + 4 * ROWB);
      floatx16 d = pc[cls];
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uh, vh, d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uh, vl, d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ul, vh, d, 0, 0, 0);
      pc[cls] = d;
    }
  };
  {
    const int n = (cin + CC16 - 1) / CC16;
    float4 r0[4], r1[4];
    char* buf0 = smem;
    char* buf1 = smem + BUFB;
    load(r0, 0);
    load(r1, n > 1 ? CC16 : 0);
    store(r0, buf0);
    __syncthreads();
    for (int kc = 0; kc < n; kc += 2) {
      load(r0, kc + 2 < n ? (kc + 2) * CC16 : 0);
      multiply(buf0);
      if (kc + 1 < n) store(r1, buf1);
      __syncthreads();
      if (kc + 1 >= n) break;
      load(r1, kc + 3 < n ? (kc + 3) * CC16 : 0);
      multiply(buf1);
      if (kc + 2 < n) store(r0, buf0);
      __syncthreads();
    }
  }

  // ---- per class: P_pad, then the taps that read it
  const int t2 = V * 32 + (lane & 31);
  const int yo2 = t2 >> 3, xo2 = t2 & 7;
  const int ntap = A.k * A.k;
  float tot = 0.f;
#pragma unroll
  for (int cls = 0; cls < 4; ++cls) {
    bool used = false;  // uniform; 1x1 / pad 0 is tap (1, 1): class (0, 0)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = A.k == 3 ? tap / 3 : 1, kx = A.k == 3 ? tap % 3 : 1;
      used |= tap < ntap && (((ky - 1) & 1) * 2 + ((kx - 1) & 1)) == cls;
    }
    if (!used) continue;
    for (int i = tid; i < NPP * PPP; i += 256) Pp[i] = 0.f;
    __syncthreads();
    {
      const int v = V * 32 + (lane & 31);
      const int pv = ((v >> 3) + 1) * GP + (v & 7) + 1;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int u = U * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        Pp[(((u >> 3) + 1) * GP + (u & 7) + 1) * PPP + pv] = pc[cls][r];
      }
    }
    __syncthreads();
    const int p2 = yo2 * GP + xo2;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap >= ntap) continue;  // uniform
      const int ky = A.k == 3 ? tap / 3 : 1, kx = A.k == 3 ? tap % 3 : 1;
      if ((((ky - 1) & 1) * 2 + ((kx - 1) & 1)) != cls) continue;  // uniform
      const int d = ((ky > 0) * GP + (kx > 0)) * (PPP + 1);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t1 = U * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        tot += Pp[((t1 >> 3) * GP + (t1 & 7)) * PPP + p2 + d] * kg[r];
      }
    }
    __syncthreads();  // P_pad is rewritten by the next class
  }
  tot = wave_sum(tot);
  if (lane == 0) red[wv] = tot;
  __syncthreads();
  if (tid == 0) A.sq[b] += (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace pgram

// ---- 16 x 16 maps at stride 1 (ResNet-18 layer2: 128 -> 128, T = 256) -----------------------
// The same identity at T = 256, where the input-position Gram P (256 x 256 fp32, 256 KB) does
// not fit LDS: the output-position sum is split by quarters J of t' (4 image rows, 64
// positions).  A workgroup takes one (example, quarter):
//   K_g[:, J] = g^T g[:, J]            256 x 64  over cout  (2 x 2 tiles per wave, registers)
//   P[:, J+]  = a^T a[:, J+]           256 x 96  over cin   (J+ = the 6 rows J's taps read;
//                                                            2 x 3 tiles per wave)
//   S_J = sum_{t, t' in J} K_g[t][t'] sum_tap P[t + d_tap][t' + d_tap]
// with one 16-channel K step of both Grams per staged chunk (split-bf16 MFMA, the operands by
// transposed LDS reads as above).  P goes to a zero-padded [18 x 18 padded positions][LD] LDS
// image (the s side padded, so a tap that leaves the image reads a zero row; the t' side masked
// per tap), and each lane gathers its 16 K_g entries' 9 taps at one base register plus
// compile-time offsets.  2 (Ti^2 cin + To^2 cout) = 33.5 MFLOP per example at 128 channels is
// the algorithmic work (the quarters compute 42: P's halo rows), against 75.5 for the direct
// weight gradient.  The 4 quarter sums of an example go to partial[b][4] (a fixed-order reduce
// follows: deterministic); the 4 workgroups of an example run on one XCD (its L2 holds the
// example's 256 KB of operands).
namespace pgq {
using namespace conv;
constexpr int HW = 16, T = 256;
constexpr int ROWB = T * 2 + 64;             // bf16 row pitch of a staged channel (576 B)
constexpr int PLANE = 2 * CC * ROWB;         // one hi or lo plane: [a | g][16 channels][pos]
constexpr int BUF = 2 * PLANE;               // one staged chunk: [hi | lo] planes
constexpr int LD = 104;                      // P row pitch in floats (4 LD = 32 mod 64 banks)
constexpr int NPP = (HW + 2) * (HW + 2);     // padded positions (324)
constexpr int GLO = 20 * LD;                 // guard before P (masked taps read below row 0)
constexpr int PBYTES = (GLO + NPP * LD + 32) * 4;
constexpr int LDSB = PBYTES > 2 * BUF ? PBYTES : 2 * BUF;
static_assert(LDSB + 64 <= 160 * 1024, "one workgroup per CU");

// ABL (ablation builds for tools/bench_pegrad.py, DD_PGQ_ABL; 0 in production): bit 0 skips
// the LDS gather, bit 1 the MFMAs, bit 2 the P write-out, bit 3 the staging's global loads
template <int ABL = 0>
__global__ __launch_bounds__(256, 1) void pgram_q_kernel(const float* __restrict__ act,
                                                         const float* __restrict__ gout,
                                                         int64_t B, int cin, int cout,
                                                         const float* __restrict__ col_scale,
                                                         float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // (example, quarter) of this workgroup: the 4 quarters of an example are blocks
  // 32 i + r + 8 j (r < 8): same XCD (block p runs on XCD p % 8)
  const unsigned p = blockIdx.x;
  const int j = (int)((p >> 3) & 3);
  const int64_t b = (int64_t)(p >> 5) * 8 + (p & 7);
  if (b >= B) return;  // (whole workgroup)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5;
  const int q = (lane >> 2) & 3, pl = lane & 3, g1 = (lane >> 4) & 1;
  const int y0e = j == 0 ? 0 : (j == 3 ? 10 : 4 * j - 1);  // first of the 6 rows J's taps read
  const int u0 = y0e * HW;
  const float* __restrict__ xa = act + (size_t)b * cin * T;
  const float* __restrict__ xg = gout + (size_t)b * cout * T;
  const int nchunk = ((cin > cout ? cin : cout) + CC - 1) / CC;

  // ---- staging: per chunk 16 channels x 256 positions of a and of g (8 float4 per thread)
  float4 r[8];
  auto load = [&](int c0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = tid + 256 * (k & 3), c = c0 + i / 64, u4 = i % 64;
      const bool isg = k >= 4;
      const int nc = isg ? cout : cin;
      const float* src = (isg ? xg : xa) + (size_t)(c < nc ? c : nc - 1) * T + u4 * 4;
      float4 v = (ABL & 8) ? make_float4(1.f, 2.f, 3.f, (float)c)
                           : *reinterpret_cast<const float4*>(src);
      if (isg && col_scale) {  // the BN-folded scale s_o of g (K_g then carries s_o^2)
        const float sc = col_scale[c < nc ? c : nc - 1];
        v = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
      }
      r[k] = keep_if(v, c < nc);
    }
  };
  auto store = [&](char* dst) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = tid + 256 * (k & 3), c = i / 64, u4 = i % 64;
      const int ag = k >= 4;
      const uint32_t h01 = pack_bf16x2(r[k].x, r[k].y), h23 = pack_bf16x2(r[k].z, r[k].w);
      const uint32_t l01 = pack_bf16x2(r[k].x - __uint_as_float(h01 << 16),
                                       r[k].y - __uint_as_float(h01 & 0xffff0000u));
      const uint32_t l23 = pack_bf16x2(r[k].z - __uint_as_float(h23 << 16),
                                       r[k].w - __uint_as_float(h23 & 0xffff0000u));
      char* pp = dst + (ag * CC + c) * ROWB + u4 * 8;
      *reinterpret_cast<uint2*>(pp) = make_uint2(h01, h23);
      *reinterpret_cast<uint2*>(pp + PLANE) = make_uint2(l01, l23);
    }
  };

  // ---- the two Grams: this wave's rows are positions 64 wv .. 64 wv + 63 (t and s blocks
  // 2 wv, 2 wv + 1); K_g's columns are J, P's the 96 positions of J's 6 tap rows
  floatx16 kg[2][2], pa[2][3];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
#pragma unroll
    for (int y = 0; y < 2; ++y) kg[x][y] = floatx16{0};
#pragma unroll
    for (int y = 0; y < 3; ++y) pa[x][y] = floatx16{0};
  }
  auto frag = [&](const char* buf, int ag, int pos0, bf16x8& hi, bf16x8& lo) {
    const char* a = buf + (ag * CC + 8 * h + q) * ROWB + (pos0 + 16 * g1 + 4 * pl) * 2;
    hi = tr_read8(a, a + 4 * ROWB);
    lo = tr_read8(a + PLANE, a + PLANE + 4 * ROWB);
  };
  auto multiply = [&](const char* buf) {
    if constexpr ((ABL & 2) != 0) return;
    bf16x8 th[2], tl[2], jh[2], jl[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      frag(buf, 1, 64 * wv + 32 * x, th[x], tl[x]);
      frag(buf, 1, 64 * j + 32 * x, jh[x], jl[x]);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        floatx16 d = kg[x][y];
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th[x], jh[y], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th[x], jl[y], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tl[x], jh[y], d, 0, 0, 0);
        kg[x][y] = d;
      }
    bf16x8 sh[2], sl[2], uh[3], ul[3];
#pragma unroll
    for (int x = 0; x < 2; ++x) frag(buf, 0, 64 * wv + 32 * x, sh[x], sl[x]);
#pragma unroll
    for (int y = 0; y < 3; ++y) frag(buf, 0, u0 + 32 * y, uh[y], ul[y]);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 3; ++y) {
        floatx16 d = pa[x][y];
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sh[x], uh[y], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sh[x], ul[y], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sl[x], uh[y], d, 0, 0, 0);
        pa[x][y] = d;
      }
  };
  {
    char* buf0 = smem;
    char* buf1 = smem + BUF;
    load(0);
    store(buf0);
    __syncthreads();
    for (int kc = 0; kc < nchunk; kc += 2) {
      if (kc + 1 < nchunk) load((kc + 1) * CC);
      multiply(buf0);
      if (kc + 1 < nchunk) store(buf1);
      __syncthreads();
      if (kc + 1 >= nchunk) break;
      if (kc + 2 < nchunk) load((kc + 2) * CC);
      multiply(buf1);
      if (kc + 2 < nchunk) store(buf0);
      __syncthreads();
    }
  }

  // ---- P into the padded image: Pp[spad(s) * LD + (u - u0)], spad(s) = (y + 1) 18 + x + 1;
  // the padding rows are zeroed (the staging buffers are done with: the loop ended on a
  // barrier)
  float* Pp = reinterpret_cast<float*>(smem) + GLO;
  if constexpr ((ABL & 4) == 0) {
  for (int i = tid; i < NPP * (96 / 4); i += 256) {
    const int row = i / 24, py = row / 18, px = row - 18 * py;
    if (py == 0 || py == 17 || px == 0 || px == 17)
      *reinterpret_cast<float4*>(Pp + row * LD + (i - row * 24) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    // s = 64 wv + 32 x + (r & 3) + 8 (r >> 2) + 4 h: image row 4 wv + 2 x + (r >> 3)
    const int sb = (4 * wv + 2 * x + 1) * 18 + 1 + 4 * h;  // spad of r = 0
#pragma unroll
    for (int y = 0; y < 3; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int sp = sb + (e & 3) + 8 * ((e >> 2) & 1) + 18 * (e >> 3);
        Pp[sp * LD + 32 * y + (lane & 31)] = pa[x][y][e];
      }
  }
  }
  __syncthreads();

  // ---- S_J: per K_g entry, the 9 taps of P at one base address + compile-time offsets
  float tot = 0.f;
  if constexpr ((ABL & 1) != 0) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) tot += kg[x][y][e] + pa[x][y][e] + pa[x][2][e];
  } else
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int tq = 64 * j + 32 * y + (lane & 31);  // this lane's t'
    const int yq = tq >> 4, xq = tq & 15;
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      // t_r = 64 wv + 32 x + (r & 3) + 8 (r >> 2) + 4 h; base at tap (-1, -1)
      const int sb = (4 * wv + 2 * x + 1) * 18 + 1 + 4 * h;
      const float* base = Pp + (sb - 19) * LD + (tq - u0 - 17);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        float ts = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int off = ((e & 3) + 8 * ((e >> 2) & 1) + 18 * (e >> 3) + (dy + 1) * 18 + dx + 1) *
                              LD + (dy + 1) * 16 + dx + 1;
          ts += base[off] * kg[x][y][e];
        }
        const bool ok = yq + dy >= 0 && yq + dy < HW && xq + dx >= 0 && xq + dx < HW;
        tot += ok ? ts : 0.f;  // a select: masked taps may read garbage
      }
    }
  }
  tot = wave_sum(tot);
  float* red = reinterpret_cast<float*>(smem + LDSB);
  __syncthreads();  // (red aliases nothing, but keep the reads of P ordered before exit)
  if (lane == 0) red[wv] = tot;
  __syncthreads();
  if (tid == 0) partial[b * 4 + j] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace pgq

// stride 2 over a 16 x 16 input: four 8 x 8 parity classes of input positions
static bool pgram_par_ok(const dd_conv_geom* g) {
  const bool k3 = g->kh == 3 && g->kw == 3 && g->pad == 1;
  const bool k1 = g->kh == 1 && g->kw == 1 && g->pad == 0;
  return (k3 || k1) && g->stride == 2 && g->h == 16 && g->w == 16 && g->ho == 8 &&
         g->wo == 8;
}

bool pgram_ok(const dd_conv_geom* g) {
  const int ti = g->h * g->w, to = g->ho * g->wo;
  const bool k3 = g->kh == 3 && g->kw == 3 && g->pad == 1;
  const bool k1 = g->kh == 1 && g->kw == 1 && g->pad == 0;
  // the zero-padded input-position Gram must fit its LDS region
  const int npp = (g->h + 2 * g->pad) * (g->w + 2 * g->pad);
  const bool fits = npp <= (ti > 32 ? pgram::PadCap<64>::NPP : pgram::PadCap<32>::NPP);
  return ((k3 || k1) && ti <= 64 && to <= 64 && ti % 4 == 0 && to % 4 == 0 && fits &&
          (g->stride == 1 || g->stride == 2)) || pgram_par_ok(g);
}

int pgram_launch(const float* act, const float* gout, const dd_conv_geom* g,
                 const float* col_scale, float* sq, hipStream_t st) {
  pgram::Args a{act, gout, col_scale, sq, g->cin, g->cout, g->h, g->w, g->ho, g->wo, g->kh,
                g->stride, g->pad};
  const int ti = g->h * g->w, to = g->ho * g->wo;
  const unsigned grid = (unsigned)g->batch;
  if (ti > 64) {
    pgram::pgram_par_kernel<<<grid, 256, 0, st>>>(a);
    DD_CHECK_LAUNCH("dd_conv_pegrad_sqnorm(pgram_par)");
    return DD_OK;
  }
  if (ti > 32 && to > 32)
    pgram::pgram_kernel<64, 64><<<grid, 256, 0, st>>>(a);
  else if (ti > 32)
    pgram::pgram_kernel<64, 32><<<grid, 256, 0, st>>>(a);
  else if (to > 32)
    pgram::pgram_kernel<32, 64><<<grid, 256, 0, st>>>(a);
  else
    pgram::pgram_kernel<32, 32><<<grid, 256, 0, st>>>(a);
  DD_CHECK_LAUNCH("dd_conv_pegrad_sqnorm(pgram)");
  return DD_OK;
}

// the quarter-tiled kernel: 3x3 / pad 1 / stride 1 on a 16 x 16 map
bool pgram_q_ok(const dd_conv_geom* g) {
  return g->kh == 3 && g->kw == 3 && g->pad == 1 && g->stride == 1 && g->h == 16 &&
         g->w == 16 && g->ho == 16 && g->wo == 16;
}

// whether AUTO takes it (DD_PGQ=1; read per call, for A/B runs in one process)
bool pgram_q_auto() {
  const char* e = getenv("DD_PGQ");
  return e && atoi(e) != 0;
}

int pgram_q_launch(const float* act, const float* gout, const dd_conv_geom* g,
                   const float* col_scale, float* partial, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
#define DD_PGQ_ATTR(A_)                                                                  \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pgq::pgram_q_kernel<A_>),   \
                              hipFuncAttributeMaxDynamicSharedMemorySize, pgq::LDSB + 64);
    DD_PGQ_ATTR(0) DD_PGQ_ATTR(1) DD_PGQ_ATTR(2) DD_PGQ_ATTR(4) DD_PGQ_ATTR(8) DD_PGQ_ATTR(15)
#undef DD_PGQ_ATTR
    attr = true;
  }
  const unsigned grid = (unsigned)(ceil_div(g->batch, 8) * 32);
  const char* e = getenv("DD_PGQ_ABL");
  const int abl = e ? atoi(e) : 0;
#define DD_PGQ_GO(A_)                                                                      \
  if (abl == A_) {                                                                         \
    pgq::pgram_q_kernel<A_><<<grid, 256, pgq::LDSB + 64, st>>>(act, gout, g->batch, g->cin, \
                                                               g->cout, col_scale, partial); \
    DD_CHECK_LAUNCH("dd_conv_pegrad_sqnorm(pgram_q)");                                     \
    return DD_OK;                                                                          \
  }
  DD_PGQ_GO(1) DD_PGQ_GO(2) DD_PGQ_GO(4) DD_PGQ_GO(8) DD_PGQ_GO(15)
#undef DD_PGQ_GO
  pgq::pgram_q_kernel<0><<<grid, 256, pgq::LDSB + 64, st>>>(act, gout, g->batch, g->cin, g->cout,
                                                            col_scale, partial);
  DD_CHECK_LAUNCH("dd_conv_pegrad_sqnorm(pgram_q)");
  return DD_OK;
}

}  // namespace dd
