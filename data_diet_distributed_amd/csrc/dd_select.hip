// Global keep-set selection: float-key radix select + stable radix sort of the survivors.
//
// Replaces reference get_scores_and_prune.py:22-24 (stable `sorted(..., reverse=True)[:k]`).
// Scores map to order-preserving u32 keys (+0 == -0, NaN below everything).
//
//   hist_top    one read of the n keys (float4), each block over a contiguous chunk: the
//               histogram of the top 11 key bits (2048 bins) per block (kept for the split's
//               offsets) and summed over blocks, plus the NaN count
//   pick        (one block) the top digit d* holding the k-th largest key: gt1 keys lie above
//               its bin, c keys in it; m = gt1 + c >= k
//   blockcounts per block, its keys above / in bin d* (from the block histograms)
//   split       second and last read of the n keys: keys above bin d* and keys in it (with
//               their indices) are compacted, each class in index order, into one buffer
//               [above | in bin] of m entries
//   4 x (count, offsets, scatter)   stable LSD radix passes over the m entries, 8 bits each,
//               descending: per block a digit histogram of its contiguous chunk, a per-digit
//               scan over blocks, then a scatter in which each 4096-entry tile is ranked with
//               8-ballot digit matching and wave-private running counts (one barrier round per
//               tile); the last pass writes the first k indices as int64 and the k-th key as
//               the threshold
// Because the above-bin keys are all larger than the in-bin ones and each class enters the
// sort in index order, the stable sort of the m entries by key puts the k kept indices first,
// ordered by key descending and ties by ascending index (the reference's visit order).
//
// HBM traffic per call: 8n (two reads of the keys) + 8m (split write) + 4 x 20m (each pass
// reads the keys for its counts, then keys + indices, and writes both) against the
// algorithmic minimum 4n + 8k; nothing waits on another workgroup (no look-back chains), and
// the host learns no intermediate count (no syncs).
#include "dd_common.h"

namespace dd {
namespace sel {

constexpr int kThreads = 256;
constexpr int kRounds = 16;                      // rounds of 64 entries per wave per tile
constexpr int kTile = 4 * kRounds * 64;          // 4096 entries per tile
constexpr int kTopBins = 2048;                   // top 11 key bits
constexpr int kTopShift = 21;
constexpr int kMaxBlocks = 512;                  // blocks of the chunked kernels

struct State {
  uint32_t dstar, gt1, c, m, k;
  uint32_t nan_count;
  uint32_t pad[10];
};

__device__ __forceinline__ uint32_t order_key(float f, bool& is_nan) {
  uint32_t u = __float_as_uint(f);
  const uint32_t a = u & 0x7fffffffu;
  if (a > 0x7f800000u) {
    is_nan = true;
    return 0u;
  }
  if (a == 0) u = 0;  // -0.0 ties with +0.0 (Python float comparison)
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float key_to_float(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// lanes of the wave holding the same BITS-bit digit d (restricted to `live`)
template <int BITS = 8>
__device__ __forceinline__ uint64_t match8(uint32_t d, uint64_t live) {
  uint64_t peers = live;
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bb = __ballot(bit);
    peers &= bit ? bb : ~bb;
  }
  return peers;
}

// [lo, hi) of block `b` of `nb` over `len` entries, in whole tiles
__device__ __forceinline__ void chunk_of(int64_t len, int b, int nb, int64_t& lo, int64_t& hi) {
  const int64_t tiles = (len + kTile - 1) / kTile;
  const int64_t per = (tiles + nb - 1) / nb;
  lo = (int64_t)b * per * kTile;
  hi = lo + per * kTile;
  if (lo > len) lo = len;
  if (hi > len) hi = len;
}

// exclusive prefix over blocks < b of v[] (len nb), by the whole workgroup
__device__ uint32_t block_prefix(const uint32_t* __restrict__ v, int b, uint32_t* red) {
  uint32_t s = 0;
  for (int i = threadIdx.x; i < b; i += kThreads) s += v[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const uint32_t t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

// ---- threshold digit -------------------------------------------------------------------------
// per block over its chunk: bh[b][2048] histogram of the top 11 bits; hist[] += it; NaNs
__global__ __launch_bounds__(kThreads) void hist_top_kernel(const float* __restrict__ keys,
                                                            int64_t n, int vec, State* st,
                                                            uint32_t* __restrict__ hist,
                                                            uint32_t* __restrict__ bh) {
  __shared__ uint32_t h[kTopBins];
  __shared__ uint32_t s_nan[4];
  for (int i = threadIdx.x; i < kTopBins; i += kThreads) h[i] = 0;
  __syncthreads();
  int64_t lo, hi;
  chunk_of(n, blockIdx.x, gridDim.x, lo, hi);
  uint32_t nans = 0;
  // the lanes of one digit add once (scores crowd into a few exponent bins: plain per-lane
  // LDS atomics would serialise on them)
  const int lane = threadIdx.x & 63;
  auto add = [&](float f, bool valid) {
    bool isn = false;
    const uint32_t u = order_key(f, isn);
    nans += valid && isn;
    const uint32_t d = u >> kTopShift;
    const uint64_t peers = match8<11>(d, __ballot(valid));
    if (valid && __popcll(peers & lanemask_lt(lane)) == 0)
      atomicAdd(&h[d], (uint32_t)__popcll(peers));
  };
  int64_t i = lo + threadIdx.x;
  if (vec) {  // lo is a multiple of 4096 and keys 16-B aligned
    const float4* __restrict__ k4 = reinterpret_cast<const float4*>(keys);
    const int64_t j1 = hi >> 2;
    for (int64_t j0 = lo >> 2; j0 < j1; j0 += kThreads) {  // workgroup-uniform trip count
      const int64_t j = j0 + threadIdx.x;
      const bool valid = j < j1;
      const float4 v = k4[valid ? j : j1 - 1];
      add(v.x, valid);
      add(v.y, valid);
      add(v.z, valid);
      add(v.w, valid);
    }
    i = ((hi >> 2) << 2) + threadIdx.x;
  }
  for (int64_t i0 = i - threadIdx.x; i0 < hi; i0 += kThreads) {
    const int64_t j = i0 + threadIdx.x;
    add(keys[j < hi ? j : hi - 1], j < hi);
  }
  for (int o = 32; o > 0; o >>= 1) nans += __shfl_xor(nans, o);
  if ((threadIdx.x & 63) == 0) s_nan[threadIdx.x >> 6] = nans;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = s_nan[0] + s_nan[1] + s_nan[2] + s_nan[3];
    if (t) atomicAdd(&st->nan_count, t);
  }
  uint32_t* row = bh + (size_t)blockIdx.x * kTopBins;
  for (int j = threadIdx.x; j < kTopBins; j += kThreads) {
    const uint32_t c = h[j];
    row[j] = c;
    if (c) atomicAdd(&hist[j], c);
  }
}

// one block of 1024: thread t owns digits 2047 - 2t and 2046 - 2t (descending positions 2t,
// 2t + 1); an inclusive scan over the pairs finds the bin holding the k-th largest key
__global__ __launch_bounds__(1024) void pick_kernel(State* st, const uint32_t* __restrict__ hist,
                                                    uint32_t k, int32_t* nan_out) {
  __shared__ uint32_t s[1024];
  const int t = threadIdx.x;
  const uint32_t a = hist[2047 - 2 * t], b = hist[2046 - 2 * t];
  s[t] = a + b;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t v = t >= o ? s[t - o] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  const uint32_t incl = s[t], excl = incl - (a + b);
  if (excl < k && k <= excl + a) {
    st->dstar = 2047 - 2 * t;
    st->gt1 = excl;
    st->c = a;
    st->m = excl + a;
  } else if (excl + a < k && k <= incl) {
    st->dstar = 2046 - 2 * t;
    st->gt1 = excl + a;
    st->c = b;
    st->m = incl;
  }
  if (t == 0) {
    st->k = k;
    if (nan_out) *nan_out = (int32_t)st->nan_count;
  }
}

// NaN count only (k == 0)
__global__ void nan_out_kernel(const State* st, int32_t* nan_out) {
  if (threadIdx.x == 0 && nan_out) *nan_out = (int32_t)st->nan_count;
}

// one wave per block row of bh: its keys above bin d* and in it
__global__ __launch_bounds__(kThreads) void blockcount_kernel(const uint32_t* __restrict__ bh,
                                                              int nb, const State* st,
                                                              uint32_t* __restrict__ cnt_gt,
                                                              uint32_t* __restrict__ cnt_eq) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= nb) return;
  const uint32_t dstar = st->dstar;
  const uint32_t* row = bh + (size_t)b * kTopBins;
  uint32_t g = 0;
  for (int d = (int)dstar + 1 + lane; d < kTopBins; d += 64) g += row[d];
  for (int o = 32; o > 0; o >>= 1) g += __shfl_xor(g, o);
  if (lane == 0) {
    cnt_gt[b] = g;
    cnt_eq[b] = row[dstar];
  }
}

// ---- stable split of the n keys into [above d* | in d*] ---------------------------------------
__global__ __launch_bounds__(kThreads) void split_kernel(const float* __restrict__ keys,
                                                         int64_t n, const State* st,
                                                         const uint32_t* __restrict__ cnt_gt,
                                                         const uint32_t* __restrict__ cnt_eq,
                                                         uint32_t* __restrict__ okey,
                                                         uint32_t* __restrict__ oidx) {
  __shared__ uint32_t red[4];
  __shared__ uint32_t wg[4], we[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int64_t lo, hi;
  chunk_of(n, blockIdx.x, gridDim.x, lo, hi);
  const uint32_t dstar = st->dstar, gt1 = st->gt1;
  uint32_t base_g = block_prefix(cnt_gt, blockIdx.x, red);
  uint32_t base_e = gt1 + block_prefix(cnt_eq, blockIdx.x, red);
  for (int64_t t0 = lo; t0 < hi; t0 += kTile) {
    uint32_t u[kRounds], pos[kRounds];
    uint32_t cls = 0;  // 2 bits per round: 1 above, 2 in-bin
    uint32_t run_g = 0, run_e = 0;
    const int64_t wbase = t0 + wv * (kRounds * 64);
    // every load first, from clamped addresses (a load under the validity test is compiled
    // into a branch that waits for it alone)
    float kf[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int64_t i = wbase + r * 64 + lane;
      kf[r] = keys[i < hi ? i : hi - 1];
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int64_t i = wbase + r * 64 + lane;
      const bool valid = i < hi;
      bool isn = false;
      const uint32_t key = valid ? order_key(kf[r], isn) : 0u;
      const uint32_t d = key >> kTopShift;
      const bool g = valid && d > dstar, e = valid && d == dstar;
      const uint64_t bg = __ballot(g), be = __ballot(e);
      pos[r] = g ? run_g + __popcll(bg & lanemask_lt(lane))
                 : run_e + __popcll(be & lanemask_lt(lane));
      run_g += __popcll(bg);
      run_e += __popcll(be);
      u[r] = key;
      cls |= (g ? 1u : e ? 2u : 0u) << (2 * r);
    }
    if (lane == 0) {
      wg[wv] = run_g;
      we[wv] = run_e;
    }
    __syncthreads();
    uint32_t pg = base_g, pe = base_e, tg = 0, te = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (w < wv) {
        pg += wg[w];
        pe += we[w];
      }
      tg += wg[w];
      te += we[w];
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const uint32_t cl = (cls >> (2 * r)) & 3u;
      if (cl) {
        const uint32_t p = (cl == 1 ? pg : pe) + pos[r];
        okey[p] = u[r];
        oidx[p] = (uint32_t)(wbase + r * 64 + lane);
      }
    }
    base_g += tg;
    base_e += te;
    __syncthreads();  // wg / we are rewritten by the next tile
  }
}

// ---- LSD radix pass: 8 bits, descending, stable ----------------------------------------------
__device__ __forceinline__ uint32_t digit_of(uint32_t u, int shift) {
  return 255u - ((u >> shift) & 255u);
}

// per block over its chunk of the m entries: hist[d * nb + b].  Each wave takes 16 x 64
// entries at a time (all loads issued first); the lanes of one digit add once (no-return LDS
// atomic by the group's first lane)
__global__ __launch_bounds__(kThreads) void count_kernel(const uint32_t* __restrict__ key,
                                                         const State* st, int shift,
                                                         uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int w = 0; w < 4; ++w) h[w][tid] = 0;
  __syncthreads();
  int64_t lo, hi;
  chunk_of(st->m, blockIdx.x, gridDim.x, lo, hi);
  for (int64_t t0 = lo + wv * (kRounds * 64); t0 < hi; t0 += kTile) {
    uint32_t kk[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int64_t i = t0 + r * 64 + lane;
      kk[r] = key[i < hi ? i : hi - 1];
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const bool valid = t0 + r * 64 + lane < hi;
      const uint32_t d = digit_of(kk[r], shift);
      const uint64_t peers = match8(d, __ballot(valid));
      if (valid && __popcll(peers & lanemask_lt(lane)) == 0) atomicAdd(&h[wv][d], (uint32_t)__popcll(peers));
    }
  }
  __syncthreads();
  hist[(size_t)tid * gridDim.x + blockIdx.x] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

// one block per digit: offs[d * nb + b] = sum_{b' < b} hist[d * nb + b'], tot[d] = the digit's
// total (nb <= 1024)
__global__ __launch_bounds__(1024) void offsets_kernel(const uint32_t* __restrict__ hist,
                                                       int nb, uint32_t* __restrict__ offs,
                                                       uint32_t* __restrict__ tot) {
  __shared__ uint32_t s[1024];
  const int t = threadIdx.x, d = blockIdx.x;
  const uint32_t v = t < nb ? hist[(size_t)d * nb + t] : 0u;
  s[t] = v;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t a = t >= o ? s[t - o] : 0u;
    __syncthreads();
    s[t] += a;
    __syncthreads();
  }
  if (t < nb) offs[(size_t)d * nb + t] = s[t] - v;
  if (t == 1023) tot[d] = s[t];
}

// per block, tile by tile in order: ranks within the tile (wave-private running counts over
// 16 rounds of 8-ballot matching), then positions = the block's running digit base + the
// waves' exclusive prefix + the rank
template <bool LAST>
__global__ __launch_bounds__(kThreads) void scatter_kernel(
    const uint32_t* __restrict__ ikey, const uint32_t* __restrict__ iidx, const State* st,
    int shift, const uint32_t* __restrict__ offs, const uint32_t* __restrict__ tot,
    uint32_t* __restrict__ okey, uint32_t* __restrict__ oidx, int64_t* __restrict__ out,
    float* thr_out) {
  __shared__ uint32_t run[4][256];
  __shared__ uint32_t base[256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // digit bases: exclusive scan of the digit totals + this block's offset within the digit
  {
    const uint32_t c = tot[tid];
    base[tid] = c;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const uint32_t a = tid >= o ? base[tid - o] : 0u;
      __syncthreads();
      base[tid] += a;
      __syncthreads();
    }
    base[tid] = base[tid] - c + offs[(size_t)tid * gridDim.x + blockIdx.x];
  }
  int64_t lo, hi;
  chunk_of(st->m, blockIdx.x, gridDim.x, lo, hi);
  const uint32_t k = st->k;
  for (int64_t t0 = lo; t0 < hi; t0 += kTile) {
#pragma unroll
    for (int w = 0; w < 4; ++w) run[w][tid] = 0;
    __syncthreads();
    uint32_t u[kRounds], id[kRounds], pos[kRounds], dg[kRounds / 4];
#pragma unroll
    for (int q = 0; q < kRounds / 4; ++q) dg[q] = 0;
    uint32_t vmask = 0;
    const int64_t wbase = t0 + wv * (kRounds * 64);
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int64_t i = wbase + r * 64 + lane;
      const int64_t ic = i < hi ? i : hi - 1;
      u[r] = ikey[ic];
      id[r] = iidx[ic];
    }
    // ranks: the first lane of each digit group adds the group's size to the wave's running
    // count (LDS atomics of one wave complete in order, so rounds stay ordered) and the old
    // count goes to the group's lanes by a lane permute: no LDS round trip per round
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const bool valid = wbase + r * 64 + lane < hi;
      const uint32_t d = digit_of(u[r], shift);
      const uint64_t peers = match8(d, __ballot(valid));
      const uint32_t rnk = __popcll(peers & lanemask_lt(lane));
      uint32_t prev = 0;
      if (valid && rnk == 0) prev = atomicAdd(&run[wv][d], (uint32_t)__popcll(peers));
      const int leader = peers ? __builtin_ctzll(peers) : lane;
      prev = (uint32_t)__builtin_amdgcn_ds_bpermute(leader << 2, (int)prev);
      pos[r] = prev + rnk;
      dg[r >> 2] |= d << (8 * (r & 3));
      vmask |= (uint32_t)valid << r;
    }
    __syncthreads();
    // per digit: the waves' counts -> exclusive prefixes (+ the running base); tile total
    const uint32_t c0 = run[0][tid], c1 = run[1][tid], c2 = run[2][tid], c3 = run[3][tid];
    const uint32_t b0 = base[tid];
    run[0][tid] = b0;
    run[1][tid] = b0 + c0;
    run[2][tid] = b0 + c0 + c1;
    run[3][tid] = b0 + c0 + c1 + c2;
    base[tid] = b0 + c0 + c1 + c2 + c3;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      if (!((vmask >> r) & 1u)) continue;
      const uint32_t d = (dg[r >> 2] >> (8 * (r & 3))) & 255u;
      const uint32_t p = run[wv][d] + pos[r];
      if constexpr (LAST) {
        if (p < k) {
          out[p] = (int64_t)id[r];
          if (p == k - 1 && thr_out) *thr_out = key_to_float(u[r]);
        }
      } else {
        okey[p] = u[r];
        oidx[p] = id[r];
      }
    }
    __syncthreads();  // run[] is reset by the next tile
  }
}

struct Layout {
  size_t state, hist, bh, cnt_gt, cnt_eq, shist, soff, stot, k0, i0, k1, i1, total;
  int nb1, nb2;
};

static Layout layout(int64_t n) {
  Layout L{};
  const int64_t tiles = std::max<int64_t>(1, ceil_div(n, kTile));
  L.nb1 = (int)std::min<int64_t>(tiles, kMaxBlocks);
  L.nb2 = L.nb1;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  L.state = take(sizeof(State));   // [state, hist] zeroed per call
  L.hist = take(kTopBins * 4);
  L.bh = take((size_t)L.nb1 * kTopBins * 4);
  L.cnt_gt = take((size_t)L.nb1 * 4);
  L.cnt_eq = take((size_t)L.nb1 * 4);
  L.shist = take((size_t)256 * L.nb2 * 4);
  L.soff = take((size_t)256 * L.nb2 * 4);
  L.stot = take(256 * 4);
  const size_t nn = (size_t)std::max<int64_t>(n, 1) * 4;
  L.k0 = take(nn);
  L.i0 = take(nn);
  L.k1 = take(nn);
  L.i1 = take(nn);
  L.total = o;
  return L;
}

}  // namespace sel
}  // namespace dd

using namespace dd;
using namespace dd::sel;

extern "C" {

size_t dd_select_workspace_bytes(int64_t n) {
  if (n < 0) return 0;
  return sel::layout(n).total;
}

int dd_select_topk(const float* keys, int64_t n, int64_t k, int64_t* idx_out, float* thr_out,
                   int32_t* nan_count_out, void* workspace, size_t workspace_bytes,
                   void* stream) {
  clear_error();
  DD_REQUIRE(n >= 0 && k >= 0 && k <= n, "dd_select_topk: need 0 <= k <= n (k=%lld n=%lld)",
             (long long)k, (long long)n);
  DD_REQUIRE(n < (1ll << 31), "dd_select_topk: n >= 2^31 unsupported");
  hipStream_t s = as_stream(stream);
  const sel::Layout L = sel::layout(n);
  if (!workspace || workspace_bytes < L.total) {
    set_error("dd_select_topk: workspace %zu < %zu bytes", workspace_bytes, L.total);
    return DD_EWORKSPACE;
  }
  char* ws = static_cast<char*>(workspace);
  auto* st = reinterpret_cast<State*>(ws + L.state);
  auto* hist = reinterpret_cast<uint32_t*>(ws + L.hist);
  auto* bh = reinterpret_cast<uint32_t*>(ws + L.bh);
  auto* cnt_gt = reinterpret_cast<uint32_t*>(ws + L.cnt_gt);
  auto* cnt_eq = reinterpret_cast<uint32_t*>(ws + L.cnt_eq);
  auto* shist = reinterpret_cast<uint32_t*>(ws + L.shist);
  auto* soff = reinterpret_cast<uint32_t*>(ws + L.soff);
  auto* stot = reinterpret_cast<uint32_t*>(ws + L.stot);
  auto* k0 = reinterpret_cast<uint32_t*>(ws + L.k0);
  auto* i0 = reinterpret_cast<uint32_t*>(ws + L.i0);
  auto* k1 = reinterpret_cast<uint32_t*>(ws + L.k1);
  auto* i1 = reinterpret_cast<uint32_t*>(ws + L.i1);
  DD_CHECK_HIP(hipMemsetAsync(ws + L.state, 0, L.bh - L.state, s), "dd_select_topk(clear)");
  if (n == 0) {
    if (nan_count_out) nan_out_kernel<<<1, 64, 0, s>>>(st, nan_count_out);
    DD_CHECK_LAUNCH("dd_select_topk(empty)");
    return DD_OK;
  }
  DD_REQUIRE(keys != nullptr, "dd_select_topk: null keys");
  const int vec = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
  hist_top_kernel<<<L.nb1, kThreads, 0, s>>>(keys, n, vec, st, hist, bh);
  DD_CHECK_LAUNCH("dd_select_topk(hist)");
  if (k == 0) {
    if (nan_count_out) nan_out_kernel<<<1, 64, 0, s>>>(st, nan_count_out);
    DD_CHECK_LAUNCH("dd_select_topk(nan)");
    return DD_OK;
  }
  DD_REQUIRE(idx_out != nullptr, "dd_select_topk: null idx_out");
  pick_kernel<<<1, 1024, 0, s>>>(st, hist, (uint32_t)k, nan_count_out);
  blockcount_kernel<<<(unsigned)ceil_div(L.nb1, 4), kThreads, 0, s>>>(bh, L.nb1, st, cnt_gt,
                                                                      cnt_eq);
  split_kernel<<<L.nb1, kThreads, 0, s>>>(keys, n, st, cnt_gt, cnt_eq, k0, i0);
  DD_CHECK_LAUNCH("dd_select_topk(split)");
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    const uint32_t* sk = (pass & 1) ? k1 : k0;
    const uint32_t* si = (pass & 1) ? i1 : i0;
    uint32_t* dk = (pass & 1) ? k0 : k1;
    uint32_t* di = (pass & 1) ? i0 : i1;
    count_kernel<<<L.nb2, kThreads, 0, s>>>(sk, st, shift, shist);
    offsets_kernel<<<256, 1024, 0, s>>>(shist, L.nb2, soff, stot);
    if (pass == 3)
      scatter_kernel<true><<<L.nb2, kThreads, 0, s>>>(sk, si, st, shift, soff, stot, dk, di,
                                                      idx_out, thr_out);
    else
      scatter_kernel<false><<<L.nb2, kThreads, 0, s>>>(sk, si, st, shift, soff, stot, dk, di,
                                                       idx_out, thr_out);
  }
  DD_CHECK_LAUNCH("dd_select_topk(sort)");
  return DD_OK;
}

}  // extern "C"
