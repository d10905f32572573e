// On-device synthetic training sets (BASELINE config 5).
//
// The reference reads CIFAR-10 through torchvision with a download (data/loader.py:27-33),
// impossible offline, and at ImageNet shape (1.28M x 3 x 224 x 224 = 193 GB of uint8) a host
// generator plus H2D copy would dominate the job.  Here every pixel and label is a pure
// function of (seed, global example index, channel, y, x) — a counter-based 32-bit hash — so a
// rank materialises exactly its shard in HBM, any sub-range reproduces the same bytes, and
// oracle/synth.py restates it bit for bit in NumPy.
//
// Definition (all arithmetic on uint32 with wrap-around; mix = the murmur3 finaliser):
//   key    = mix(mix(i0 ^ mix(s0 + 0x9E3779B9)) ^ (i1 * 0x85EBCA77 + s1))
//            (i0/i1 = low/high words of the index, s0/s1 of the seed)
//   label  = mix(key ^ 0xA511E9B3) % num_classes
//   hc     = mix(label * 0x9E3779B1 + 0x6A09E667)             (class pattern)
//   fx, fy = 1 + (hc & 7), 1 + ((hc >> 3) & 7)
//   base   = 32 + ((mix(hc + ch) >> 25) & 127)
//   stripe = (((x * fx + y * fy) * 16) / W) & 1
//   noise  = mix(key ^ ((ch * H * W + y * W + x) * 0x27D4EB2F)) & 63
//   pixel  = min(base + 48 * stripe + ((key >> 8) & 31) + noise, 255)
// HBM-write bound: C*H*W bytes per image (+ 8 for the label); 16 pixels (one 16-byte store)
// per thread when W % 16 == 0.
#include "dd_common.h"

namespace dd {
namespace synth {

__device__ __forceinline__ uint32_t mix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t example_key(uint64_t seed, uint64_t i) {
  const uint32_t s0 = (uint32_t)seed, s1 = (uint32_t)(seed >> 32);
  const uint32_t i0 = (uint32_t)i, i1 = (uint32_t)(i >> 32);
  return mix(mix(i0 ^ mix(s0 + 0x9E3779B9u)) ^ (i1 * 0x85EBCA77u + s1));
}

struct Geo {
  uint64_t seed;
  int64_t idx0, n;
  int C, H, W, num_classes;
};

// VEC: 16 consecutive pixels of one row per thread (W % 16 == 0); else one pixel per thread
template <bool VEC>
__global__ __launch_bounds__(256) void synth_kernel(const Geo g, uint8_t* __restrict__ img,
                                                    int64_t* __restrict__ labels) {
  constexpr int PX = VEC ? 16 : 1;
  const int64_t hw = (int64_t)g.H * g.W;
  const int64_t per_img = g.C * hw / PX;
  const int64_t total = g.n * per_img;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = q / per_img;
    const uint32_t r = (uint32_t)((q - i * per_img) * PX);  // offset inside the image
    const uint32_t key = example_key(g.seed, (uint64_t)(g.idx0 + i));
    const uint32_t label = mix(key ^ 0xA511E9B3u) % (uint32_t)g.num_classes;
    if (r == 0 && labels) labels[i] = (int64_t)label;
    const uint32_t ch = r / (uint32_t)hw;
    const uint32_t p = r - ch * (uint32_t)hw;
    const uint32_t y = p / (uint32_t)g.W, x0 = p - y * (uint32_t)g.W;
    const uint32_t hc = mix(label * 0x9E3779B1u + 0x6A09E667u);
    const uint32_t fx = 1u + (hc & 7u), fy = 1u + ((hc >> 3) & 7u);
    const uint32_t base = 32u + ((mix(hc + ch) >> 25) & 127u) + ((key >> 8) & 31u);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const uint32_t x = x0 + j;
      const uint32_t stripe = (((x * fx + y * fy) * 16u) / (uint32_t)g.W) & 1u;
      const uint32_t noise = mix(key ^ ((r + j) * 0x27D4EB2Fu)) & 63u;
      const uint32_t v = base + 48u * stripe + noise;
      w[j >> 2] |= (v < 255u ? v : 255u) << (8 * (j & 3));
    }
    if constexpr (VEC)
      *reinterpret_cast<uint4*>(img + i * g.C * hw + r) = make_uint4(w[0], w[1], w[2], w[3]);
    else
      img[i * g.C * hw + r] = (uint8_t)w[0];
  }
}

}  // namespace synth
}  // namespace dd

using namespace dd;

extern "C" int dd_synth_images_u8(uint64_t seed, int64_t idx0, int64_t n, int32_t channels,
                                  int32_t h, int32_t w, int32_t num_classes, uint8_t* img,
                                  int64_t* labels, void* stream) {
  clear_error();
  DD_REQUIRE(n >= 0 && idx0 >= 0 && channels > 0 && h > 0 && w > 0 && num_classes > 0,
             "dd_synth_images_u8: bad sizes");
  DD_REQUIRE((int64_t)channels * h * w < (1ll << 32),
             "dd_synth_images_u8: image too large for 32-bit pixel offsets");
  if (n == 0) return DD_OK;
  DD_REQUIRE(img, "dd_synth_images_u8: null image buffer");
  synth::Geo g{seed, idx0, n, channels, h, w, num_classes};
  const bool vec = w % 16 == 0 && reinterpret_cast<uintptr_t>(img) % 16 == 0;
  const int64_t work = n * channels * h * w / (vec ? 16 : 1);
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(work, 256), 16 * device_cus());
  if (vec)
    synth::synth_kernel<true><<<grid, 256, 0, as_stream(stream)>>>(g, img, labels);
  else
    synth::synth_kernel<false><<<grid, 256, 0, as_stream(stream)>>>(g, img, labels);
  DD_CHECK_LAUNCH("dd_synth_images_u8");
  return DD_OK;
}
