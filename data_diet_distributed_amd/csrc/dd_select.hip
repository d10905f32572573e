// Global keep-set selection: float-key radix select + stable radix sort of the survivors.
//
// Replaces reference get_scores_and_prune.py:22-24 (stable `sorted(..., reverse=True)[:k]`).
// Scores map to order-preserving u32 keys (+0 == -0, NaN below everything).
//
//   hist_top    one read of the n keys (float4, 1024-thread blocks over contiguous chunks):
//               the histogram of the top 11 key bits (2048 bins) summed over blocks, per block
//               as suffix sums (keys at or above each bin), plus the NaN count
//   split       second and last read of the n keys.  Each block finds the top digit d*
//               holding the k-th largest key from the summed histogram (m >= k keys lie in or
//               above its bin) and compacts its survivors, in index order, after those of the
//               blocks before it (one suffix-row load per earlier block).  Every survivor's key
//               is >= base = d* << 21 and below (D + 1) << 21 (D the highest non-empty bin), so
//               the sort needs only the R = 21 + bitlen(D - d*) low bits of key - base: three
//               LSD passes of ceil(R / 3) bits (7-8 when the survivors span fewer than 8 top
//               bins = two octaves, at most 11), decided on the device
//   3 x (count, offsets, scatter)  stable LSD radix passes over the m survivors, descending:
//               per block a digit histogram of its contiguous chunk, a per-digit scan over
//               blocks, then a scatter in which each 4096-entry tile is ranked (ballot digit
//               matching, wave-private running counts), reordered by digit in LDS, and written
//               back as contiguous runs (consecutive lanes -> consecutive addresses); the last
//               pass writes the first k indices as int64 and the k-th key as the threshold
// Each block-serial kernel loads its next tile before working on the current one.  Because
// the survivors enter the sort in index order and every pass is stable, the sort by key puts
// the k kept indices first, ordered by key descending and ties by ascending index (the
// reference's visit order).
//
// HBM traffic per call: 8n (two reads of the keys) + 8m (split write) + 3 x 20m (each pass
// reads the keys for its counts, then keys + indices, and writes both; the last writes k int64
// indices instead) ~ 8n + 68m, against the algorithmic minimum 4n + 8k; 12 launches (13 on a
// process's first call on a device: a 32-workgroup probe of LDS atomic return order whose
// verdict the scatters read; a graph captured from that call replays the probe too); nothing
// waits on another workgroup (no look-back chains), and the host learns no intermediate count
// (no syncs).
#include "dd_common.h"

#include <algorithm>
#include <atomic>
#include <stdlib.h>

namespace dd {
namespace sel {

constexpr int kThreads = 256;
#ifndef DD_SEL_ROUNDS
#define DD_SEL_ROUNDS 16
#endif
#ifndef DD_SEL_BLOCKS
#define DD_SEL_BLOCKS 512
#endif
#ifndef DD_SEL_PREFETCH
#define DD_SEL_PREFETCH 1
#endif
constexpr int kRounds = DD_SEL_ROUNDS;           // rounds of 64 entries per wave per tile
constexpr int kTile = 4 * kRounds * 64;          // 4096 entries per tile
constexpr int kTopBins = 2048;                   // top 11 key bits
constexpr int kTopShift = 21;
constexpr int kHistThreads = 1024;               // hist_top
constexpr int kMaxTopBlocks = 256;               // hist_top / split blocks
constexpr int kMaxSortBlocks = DD_SEL_BLOCKS;    // count / scatter blocks
constexpr int kPasses = 3;                       // LSD passes of <= 11 bits
constexpr int kProbeBlocks = 32, kProbeIters = 16;  // lds_order_probe_kernel
constexpr int kMaxBins = 2048;

struct State {
  uint32_t dstar, m, k, nan_count, base, bits, top;
  uint32_t unused;
  uint32_t pad[8];
};

// The lane-order probe's verdict, per device (module globals are per device): mismatches seen
// and probe workgroups finished.  The probe runs once per process and device (the first
// dd_select_topk call enqueues it on its stream); a scatter takes the atomic rank only once
// every probe workgroup has reported and none saw a lane out of order, and the ballot-match
// rank otherwise (e.g. a call on another stream that overtakes the probe).
__device__ uint32_t g_lane_order_bad = 0;
__device__ uint32_t g_lane_order_done = 0;

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

// [lo, hi) of block `b` of `nb` over `len` entries, in whole tiles
__device__ __forceinline__ void chunk_of(int64_t len, int b, int nb, int64_t& lo, int64_t& hi) {
  const int64_t tiles = (len + kTile - 1) / kTile;
  const int64_t per = (tiles + nb - 1) / nb;
  lo = (int64_t)b * per * kTile;
  hi = lo + per * kTile;
  if (lo > len) lo = len;
  if (hi > len) hi = len;
}

// inclusive scan of one value per thread over an NT-thread workgroup (thread order); `red`
// holds NT / 64 words; one barrier (callers separate reuses of `red` by a barrier)
template <int NT>
__device__ __forceinline__ uint32_t block_incl_scan(uint32_t v, uint32_t* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t s = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(s, o);
    if (lane >= o) s += t;
  }
  if (lane == 63) red[wv] = s;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w)
    if (w < wv) before += red[w];
  return before + s;
}

// descending digit of a pass over the key relative to the survivors' base
__device__ __forceinline__ uint32_t digit_of(uint32_t u, uint32_t base, int shift, uint32_t mask) {
  return mask - (((u - base) >> shift) & mask);
}

// lanes of the wave holding the same `bits`-bit digit d (restricted to `live`)
__device__ __forceinline__ uint64_t match_bits(uint32_t d, uint64_t live, int bits) {
  uint64_t peers = live;
  for (int b = 0; b < bits; ++b) {  // wave-uniform trip count
    const bool bit = (d >> b) & 1u;
    const uint64_t bb = __ballot(bit);
    peers &= bit ? bb : ~bb;
  }
  return peers;
}

// ---- threshold digit -------------------------------------------------------------------------
// per block over its chunk: the histogram of the top 11 bits, written as suffix sums
// (bh[b][d] = the block's keys whose top bits are >= d, so a later kernel reads any block's
// count above a threshold digit with one load); hist[] += the plain histogram; NaNs.
// Scores crowd into a few bins: the lanes sharing the wave's first digit add once, the others
// add one each (an 11-ballot match per element costs more than the LDS atomics it saves).
__global__ __launch_bounds__(kHistThreads) void hist_top_kernel(const float* __restrict__ keys,
                                                                int64_t n, int vec, State* st,
                                                                uint32_t* __restrict__ hist,
                                                                uint32_t* __restrict__ bh) {
  // four copies, by wave % 4 (0.93x the time of one; plain per-lane atomics without the match
  // took 0.87x on uniform keys but serialise 64-way when the scores share one bin)
  constexpr int NH = 4;
  __shared__ uint32_t h[NH][kTopBins];
  __shared__ uint32_t red[kHistThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63;
  uint32_t* hw = h[(tid >> 6) % NH];
  for (int i = tid; i < NH * kTopBins; i += kHistThreads) (&h[0][0])[i] = 0;
  __syncthreads();
  int64_t lo, hi;
  chunk_of(n, blockIdx.x, gridDim.x, lo, hi);
  uint32_t nans = 0;
  auto add = [&](float f, bool valid) {
    bool isn = false;
    const uint32_t u = order_key(f, isn);
    nans += valid && isn;
    const uint32_t d = u >> kTopShift;
    const uint64_t live = __ballot(valid);
    if (!live) return;  // wave-uniform
    const int first = __builtin_ctzll(live);
    const uint32_t d0 = __builtin_amdgcn_readlane(d, first);
    const uint64_t same = __ballot(valid && d == d0);
    if (lane == first) atomicAdd(&hw[d0], (uint32_t)__popcll(same));
    if (valid && d != d0) atomicAdd(&hw[d], 1u);
  };
  int64_t i0 = lo;
  if (vec) {  // lo is a multiple of 4096 and the keys 16-B aligned: 4 float4 per thread in flight
    const float4* __restrict__ k4 = reinterpret_cast<const float4*>(keys);
    const int64_t j1 = hi >> 2;
    constexpr int U = 4;
    for (int64_t j0 = lo >> 2; j0 < j1; j0 += U * kHistThreads) {  // workgroup-uniform
      float4 v[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = j0 + u * kHistThreads + tid;
        ok[u] = j < j1;
        v[u] = k4[ok[u] ? j : j1 - 1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        add(v[u].x, ok[u]);
        add(v[u].y, ok[u]);
        add(v[u].z, ok[u]);
        add(v[u].w, ok[u]);
      }
    }
    // the scalar tail starts after the vector part; an empty block (lo == hi == n, once the
    // tiles do not fill every block) has no tail: (hi >> 2) << 2 would lie below its lo
    i0 = (hi >> 2) << 2;
    if (i0 < lo) i0 = lo;
  }
  for (int64_t b0 = i0; b0 < hi; b0 += kHistThreads) {
    const int64_t j = b0 + tid;
    add(keys[j < hi ? j : hi - 1], j < hi);
  }
  for (int o = 32; o > 0; o >>= 1) nans += __shfl_xor(nans, o);
  if (lane == 0) red[tid >> 6] = nans;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kHistThreads / 64; ++w) t += red[w];
    if (t) atomicAdd(&st->nan_count, t);
  }
  // thread t owns bins 2047 - 2t and 2046 - 2t: a scan in thread order is a suffix sum
  uint32_t a = 0, b = 0;
#pragma unroll
  for (int c = 0; c < NH; ++c) {
    a += h[c][2047 - 2 * tid];
    b += h[c][2046 - 2 * tid];
  }
  if (a) atomicAdd(&hist[2047 - 2 * tid], a);
  if (b) atomicAdd(&hist[2046 - 2 * tid], b);
  __syncthreads();  // red is reused
  const uint32_t incl = block_incl_scan<kHistThreads>(a + b, red);
  uint32_t* row = bh + (size_t)blockIdx.x * kTopBins;
  row[2047 - 2 * tid] = incl - b;
  row[2046 - 2 * tid] = incl;
}

// zero the per-call state and histogram (a kernel rather than hipMemsetAsync: one node type
// under stream capture, replayed like every other launch of the call)
__global__ __launch_bounds__(256) void clear_kernel(uint4* __restrict__ p, int n16) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256)
    p[i] = make_uint4(0u, 0u, 0u, 0u);
}

// NaN count only (k == 0)
__global__ void nan_out_kernel(const State* st, int32_t* nan_out) {
  if (threadIdx.x == 0 && nan_out) *nan_out = (int32_t)st->nan_count;
}

// ---- stable compaction of the survivors (top digit >= d*), in index order ---------------------
// Every block first finds d* itself from the global histogram (thread t owns bins 2047 - 2t and
// 2046 - 2t; a scan in thread order counts the keys at or above each bin): d* is the bin
// holding the k-th largest key, m the keys at or above it, D the highest non-empty bin; the
// survivors' keys lie in [base, (D + 1) << 21) with base = d* << 21, so the sort needs the
// R = 21 + bitlen(D - d*) low bits of key - base: three LSD passes of ceil(R / 3) <= 11 bits.
// Block 0 publishes them in State for the sort kernels.  The block's output offset is the
// survivors of the blocks before it (one suffix-row load each).  1024-thread blocks over
// hist_top's chunks, 16 waves x 16 rounds of 64 keys per tile; the next tile's keys load while
// the current one is compacted.
constexpr int kSplitThreads = 1024;
constexpr int kSplitWaves = kSplitThreads / 64;
constexpr int kSplitTile = kSplitWaves * kRounds * 64;
__global__ __launch_bounds__(kSplitThreads) void split_kernel(
    const float* __restrict__ keys, int64_t n, uint32_t k, State* st,
    const uint32_t* __restrict__ hist, const uint32_t* __restrict__ bh,
    uint32_t* __restrict__ okey, uint32_t* __restrict__ oidx, int32_t* nan_out) {
  __shared__ uint32_t red[kSplitWaves];
  __shared__ uint32_t wc[2][kSplitWaves];
  __shared__ uint32_t s_dstar, s_top, s_base;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_top = 0;
  {
    const uint32_t a = hist[2047 - 2 * tid], b = hist[2046 - 2 * tid];
    __syncthreads();
    if (a | b) atomicMax(&s_top, a ? 2047u - 2 * tid : 2046u - 2 * tid);
    const uint32_t incl = block_incl_scan<kSplitThreads>(a + b, red);
    const uint32_t excl = incl - (a + b);
    if (excl < k && k <= excl + a) {
      s_dstar = 2047 - 2 * tid;
      if (blockIdx.x == 0) st->m = excl + a;
    } else if (excl + a < k && k <= incl) {
      s_dstar = 2046 - 2 * tid;
      if (blockIdx.x == 0) st->m = incl;
    }
  }
  __syncthreads();
  const uint32_t dstar = s_dstar;
  if (blockIdx.x == 0 && tid == 0) {
    const uint32_t span = s_top - dstar;
    const uint32_t R = kTopShift + (span ? 32 - __clz(span) : 0);
    st->dstar = dstar;
    st->base = dstar << kTopShift;
    st->top = s_top;
    st->bits = (R + kPasses - 1) / kPasses;
    st->k = k;
    if (nan_out) *nan_out = (int32_t)st->nan_count;
  }
  if (wv == 0) {
    uint32_t s = 0;
    for (int i = lane; i < (int)blockIdx.x; i += 64) s += bh[(size_t)i * kTopBins + dstar];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) s_base = s;
  }
  int64_t lo, hi;
  // hist_top's chunks (its grid is this kernel's grid)
  chunk_of(n, blockIdx.x, gridDim.x, lo, hi);
  float kf[kRounds];
  auto load = [&](int64_t t0, float (&dst)[kRounds]) {
    const int64_t wbase = t0 + wv * (kRounds * 64);
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int64_t i = wbase + r * 64 + lane;
      dst[r] = keys[i < hi ? i : hi - 1];
    }
  };
  if (lo < hi) load(lo, kf);
  __syncthreads();
  uint32_t run = s_base;
  int par = 0;
  for (int64_t t0 = lo; t0 < hi; t0 += kSplitTile, par ^= 1) {
    float nk[kRounds];
    if (t0 + kSplitTile < hi) load(t0 + kSplitTile, nk);  // workgroup-uniform
    uint32_t u[kRounds], pos[kRounds];
    uint32_t keep = 0, rw = 0;
    const int64_t wbase = t0 + wv * (kRounds * 64);
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int64_t i = wbase + r * 64 + lane;
      bool isn = false;
      const uint32_t key = order_key(kf[r], isn);
      const bool s = i < hi && (key >> kTopShift) >= dstar;
      const uint64_t bs = __ballot(s);
      pos[r] = rw + __popcll(bs & lanemask_lt(lane));
      rw += __popcll(bs);
      u[r] = key;
      keep |= (uint32_t)s << r;
    }
    if (lane == 0) wc[par][wv] = rw;
    __syncthreads();  // (double-buffered counts: one barrier per tile)
    uint32_t pw = run, tt = 0;
#pragma unroll
    for (int w = 0; w < kSplitWaves; ++w) {
      const uint32_t c = wc[par][w];
      if (w < wv) pw += c;
      tt += c;
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      if ((keep >> r) & 1u) {
        const uint32_t p = pw + pos[r];
        okey[p] = u[r];
        oidx[p] = (uint32_t)(wbase + r * 64 + lane);
      }
    }
    run += tt;
#pragma unroll
    for (int r = 0; r < kRounds; ++r) kf[r] = nk[r];
  }
}

// ---- LSD radix pass: `bits` (<= 11) bits of key - base, descending, stable --------------------
// per block over its chunk of the m entries: hist[d * nb + b] (wave-private LDS histograms,
// 4 keys per 16-B load, 4 loads per thread in flight)
__global__ __launch_bounds__(kThreads) void count_kernel(const uint32_t* __restrict__ key,
                                                         const State* st, int pass,
                                                         uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[4][kMaxBins];
  const int tid = threadIdx.x, wv = tid >> 6;
  const int bits = (int)st->bits, nbins = 1 << bits;
  const uint32_t mask = (uint32_t)nbins - 1, base = st->base;
  const int shift = bits * pass;
  for (int i = tid; i < nbins; i += kThreads)
#pragma unroll
    for (int w = 0; w < 4; ++w) h[w][i] = 0;
  __syncthreads();
  int64_t lo, hi;
  chunk_of(st->m, blockIdx.x, gridDim.x, lo, hi);
  const uint4* __restrict__ k4 = reinterpret_cast<const uint4*>(key);
  // lo is a multiple of 4096; the buffers are padded to whole tiles, so a partial last uint4
  // is in bounds (its entries past hi are masked)
  for (int64_t t0 = lo; t0 < hi; t0 += kTile) {
    constexpr int NU = kTile / (4 * kThreads);
    uint4 v[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) v[u] = k4[(t0 >> 2) + u * kThreads + tid];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int64_t e = t0 + 4 * ((int64_t)u * kThreads + tid);
      const uint32_t kk[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (e + j < hi) atomicAdd(&h[wv][digit_of(kk[j], base, shift, mask)], 1u);
    }
  }
  __syncthreads();
  for (int i = tid; i < nbins; i += kThreads)
    hist[(size_t)i * gridDim.x + blockIdx.x] = h[0][i] + h[1][i] + h[2][i] + h[3][i];
}

// one block per digit: offs[d * nb + b] = sum_{b' < b} hist[d * nb + b'], tot[d] = the digit's
// total (nb <= 1024: 4 consecutive blocks per thread, one workgroup scan)
__global__ __launch_bounds__(kThreads) void offsets_kernel(const State* st,
                                                           const uint32_t* __restrict__ hist,
                                                           int nb, uint32_t* __restrict__ offs,
                                                           uint32_t* __restrict__ tot) {
  const int d = blockIdx.x;
  if (d >= (1 << st->bits)) return;
  __shared__ uint32_t red[4];
  const int t = threadIdx.x;
  const uint32_t* row = hist + (size_t)d * nb;
  uint32_t v[4], s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = 4 * t + j;
    v[j] = b < nb ? row[b] : 0u;
    s += v[j];
  }
  uint32_t e = block_incl_scan<kThreads>(s, red) - s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = 4 * t + j;
    if (b < nb) offs[(size_t)d * nb + b] = e;
    e += v[j];
  }
  if (t == kThreads - 1) tot[d] = e;
}

// per block, tile by tile in order: ranks within the tile (wave-private running counts over 16
// rounds of ballot digit matching: every round's LDS atomic is issued before the first lane
// permute waits on one), the tile reordered by digit in LDS, then written back as contiguous
// digit runs at the block's running digit base.  Thread t owns digits [t D, t D + D), D =
// max(1, bins / 256), in the per-digit steps.
__global__ __launch_bounds__(kThreads, 2) void scatter_kernel(
    const uint32_t* __restrict__ ikey, const uint32_t* __restrict__ iidx, const State* st,
    int pass, const uint32_t* __restrict__ offs, const uint32_t* __restrict__ tot,
    uint32_t* __restrict__ okey, uint32_t* __restrict__ oidx, int64_t* __restrict__ out,
    float* thr_out, int force_match) {
  const bool last = pass == kPasses - 1;
  // the rank from lane-ordered LDS atomic returns only when the process's probe has finished
  // and saw them in lane order (lds_order_probe_kernel, enqueued before the first call's
  // scatters on that call's stream)
  const bool ord = !force_match &&
                   __hip_atomic_load(&g_lane_order_done, __ATOMIC_ACQUIRE,
                                     __HIP_MEMORY_SCOPE_AGENT) >= (uint32_t)kProbeBlocks &&
                   __hip_atomic_load(&g_lane_order_bad, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) == 0;
  // per-wave running digit counts, two waves per word (16 bits each: a wave ranks at most
  // 1024 entries per tile, and the digit-ordered starts stay below 4096)
  __shared__ uint32_t run2[2][kMaxBins];
  __shared__ uint32_t gbase[kMaxBins], gofs[kMaxBins];
  __shared__ uint32_t red[4];
  __shared__ uint2 lkv[kTile];  // the tile in digit order: (key, index) pairs
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int bits = (int)st->bits, nbins = 1 << bits;
  const uint32_t mask = (uint32_t)nbins - 1, base = st->base;
  const int shift = bits * pass;
  const int D = nbins > kThreads ? nbins / kThreads : 1;
  const int d0 = tid * D;  // this thread's first digit (>= nbins: none)
  const int wpair = wv >> 1, whalf = 16 * (wv & 1);
  // digit bases: exclusive scan of the digit totals + this block's offset within the digit
  {
    uint32_t s = 0;
    for (int j = 0; j < D; ++j)
      if (d0 + j < nbins) s += tot[d0 + j];
    uint32_t e = block_incl_scan<kThreads>(s, red) - s;
    for (int j = 0; j < D; ++j)
      if (d0 + j < nbins) {
        const int d = d0 + j;
        gbase[d] = e + offs[(size_t)d * gridDim.x + blockIdx.x];
        e += tot[d];
      }
  }
  int64_t lo, hi;
  chunk_of(st->m, blockIdx.x, gridDim.x, lo, hi);
  const uint32_t k = st->k;
  uint32_t u[kRounds], id[kRounds];
  auto load = [&](int64_t t0, uint32_t (&ku)[kRounds], uint32_t (&ki)[kRounds]) {
    const int64_t wbase = t0 + wv * (kRounds * 64);
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int64_t i = wbase + r * 64 + lane;
      const int64_t ic = i < hi ? i : hi - 1;
      ku[r] = ikey[ic];
      ki[r] = iidx[ic];
    }
  };
  if (DD_SEL_PREFETCH && lo < hi) load(lo, u, id);
  for (int64_t t0 = lo; t0 < hi; t0 += kTile) {
    uint32_t nu[kRounds], nid[kRounds];
    if (!DD_SEL_PREFETCH) load(t0, u, id);
    else if (t0 + kTile < hi) load(t0 + kTile, nu, nid);  // workgroup-uniform
    for (int j = 0; j < D; ++j) {  // (d0 + j < kMaxBins always)
      run2[0][d0 + j] = 0;
      run2[1][d0 + j] = 0;
    }
    __syncthreads();
    // ranks.  ord: each lane adds 1 to its digit's running count of the wave and the old
    // value is its rank: the returns of one LDS atomic instruction come back in lane order
    // (checked once per process by lds_order_probe_kernel) and the instructions of one
    // wave complete in order.  Otherwise the first lane of each ballot-matched digit group
    // adds the group's size and the old count goes to the group's lanes by a lane permute.
    uint32_t pos[kRounds];
    const int64_t wbase = t0 + wv * (kRounds * 64);
    if (ord) {  // uniform over the grid
#pragma unroll
      for (int r = 0; r < kRounds; ++r) {
        uint32_t prev = 0;
        if (wbase + r * 64 + lane < hi)
          prev = atomicAdd(&run2[wpair][digit_of(u[r], base, shift, mask)], 1u << whalf);
        pos[r] = (prev >> whalf) & 0xffffu;
      }
    } else {
      uint32_t prev[kRounds], rl[kRounds];  // rl: rank | leader << 16
#pragma unroll
      for (int r = 0; r < kRounds; ++r) {
        const bool valid = wbase + r * 64 + lane < hi;
        const uint32_t d = digit_of(u[r], base, shift, mask);
        const uint64_t peers = match_bits(d, __ballot(valid), bits);
        const uint32_t rnk = __popcll(peers & lanemask_lt(lane));
        prev[r] = 0;
        if (valid && rnk == 0)
          prev[r] = atomicAdd(&run2[wpair][d], (uint32_t)__popcll(peers) << whalf);
        const uint32_t leader = peers ? (uint32_t)__builtin_ctzll(peers) : (uint32_t)lane;
        rl[r] = rnk | (leader << 16);
      }
#pragma unroll
      for (int r = 0; r < kRounds; ++r)
        pos[r] = ((uint32_t)__builtin_amdgcn_ds_bpermute((int)(rl[r] >> 16) << 2,
                                                          (int)(prev[r] >> whalf)) & 0xffffu) +
                 (rl[r] & 0xffffu);
    }
    __syncthreads();
    // per digit: the tile's count, its start in the digit-ordered tile and the waves' starts;
    // global position of tile entry e of digit d = gofs[d] + e
    {
      uint32_t cs = 0;
      for (int j = 0; j < D; ++j)
        if (d0 + j < nbins) {
          const int d = d0 + j;
          const uint32_t a = run2[0][d], b = run2[1][d];
          cs += (a & 0xffffu) + (a >> 16) + (b & 0xffffu) + (b >> 16);
        }
      uint32_t ls = block_incl_scan<kThreads>(cs, red) - cs;
      for (int j = 0; j < D; ++j)
        if (d0 + j < nbins) {
          const int d = d0 + j;
          const uint32_t a = run2[0][d], b = run2[1][d];
          const uint32_t c0 = a & 0xffffu, c1 = a >> 16, c2 = b & 0xffffu, c3 = b >> 16;
          run2[0][d] = ls | ((ls + c0) << 16);
          run2[1][d] = (ls + c0 + c1) | ((ls + c0 + c1 + c2) << 16);
          gofs[d] = gbase[d] - ls;
          const uint32_t c = c0 + c1 + c2 + c3;
          gbase[d] += c;
          ls += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      if (wbase + r * 64 + lane < hi) {
        const uint32_t l =
            ((run2[wpair][digit_of(u[r], base, shift, mask)] >> whalf) & 0xffffu) + pos[r];
        lkv[l] = make_uint2(u[r], id[r]);
      }
    }
    __syncthreads();
    const int cnt = (int)(hi - t0 < kTile ? hi - t0 : kTile);
#pragma unroll 4
    for (int j = 0; j < kTile / kThreads; ++j) {
      const int e = j * kThreads + tid;
      if (e < cnt) {
        const uint2 kv = lkv[e];
        const uint32_t p = gofs[digit_of(kv.x, base, shift, mask)] + (uint32_t)e;
        if (last) {
          if (p < k) {
            out[p] = (int64_t)kv.y;
            if (p == k - 1 && thr_out) *thr_out = key_to_float(kv.x);
          }
        } else {
          okey[p] = kv.x;
          oidx[p] = kv.y;
        }
      }
    }
    __syncthreads();  // lkv / run2 are rewritten by the next tile
    if (DD_SEL_PREFETCH) {
#pragma unroll
      for (int r = 0; r < kRounds; ++r) {
        u[r] = nu[r];
        id[r] = nid[r];
      }
    }
  }
}

// ---- lane order of returning LDS atomics (checked once per process and device) ----------------
// Each wave adds 1 from every active lane to pseudo-random counters (1..256 distinct per
// instruction, partial exec masks) and compares each return with the count a ballot match
// predicts for lane order; g_lane_order_bad counts mismatches, g_lane_order_done the
// workgroups finished.  The scatter passes read the verdict, so a device whose LDS returns were
// ever out of order takes the ballot-match rank.  Nothing is allocated and the host never
// waits for it (the ABI's graph-capture contract).
__global__ __launch_bounds__(kThreads) void lds_order_probe_kernel() {
  __shared__ uint32_t c[4][256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t nbad = 0;
  for (int t = 0; t < kProbeIters; ++t) {
    for (int i = threadIdx.x; i < 1024; i += kThreads) (&c[0][0])[i] = (uint32_t)(i * 7 + t);
    __syncthreads();
    uint32_t h = (uint32_t)t * 2654435761u ^ (uint32_t)(blockIdx.x * 4 + wv) * 40503u ^
                 (uint32_t)lane * 2246822519u;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    const uint32_t K = 1u + ((uint32_t)t * 37u + blockIdx.x) % ((t & 1) ? 8u : 256u);
    const uint32_t d = h % K;
    const bool act = (t & 2) ? ((h >> 20) & 3u) != 0 : true;
    const uint32_t before = c[wv][d];
    __syncthreads();
    uint32_t prev = 0;
    if (act) prev = atomicAdd(&c[wv][d], 1u);
    const uint64_t peers = match_bits(d, __ballot(act), 8);
    if (act && prev != before + __popcll(peers & lanemask_lt(lane))) ++nbad;
    __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) nbad += __shfl_xor(nbad, o);
  if (lane == 0 && nbad) atomicAdd(&g_lane_order_bad, nbad);
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(&g_lane_order_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// whether this process has enqueued the probe on device `dev` (host side, once per device)
static bool probe_once(int dev) {
  static std::atomic<uint8_t> done[64];
  if (dev < 0 || dev >= 64) return true;  // (no probe: the scatters take the match rank)
  uint8_t expect = 0;
  return !done[dev].compare_exchange_strong(expect, 1);
}

// "match" in $DD_SELECT_RANK forces the ballot-match rank (read once; no device work)
static int force_match_rank() {
  static const int v = [] {
    const char* e = getenv("DD_SELECT_RANK");
    return (e && e[0] == 'm') ? 1 : 0;
  }();
  return v;
}

struct Layout {
  size_t state, hist, bh, shist, soff, stot, k0, i0, k1, i1, total;
  int nb1, nb2;
};

static Layout layout(int64_t n) {
  Layout L{};
  const int64_t tiles = std::max<int64_t>(1, ceil_div(n, kTile));
  L.nb1 = (int)std::min<int64_t>(tiles, kMaxTopBlocks);
  L.nb2 = (int)std::min<int64_t>(tiles, kMaxSortBlocks);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  L.state = take(sizeof(State));   // [state, hist] zeroed per call
  L.hist = take(kTopBins * 4);
  L.bh = take((size_t)L.nb1 * kTopBins * 4);
  L.shist = take((size_t)kMaxBins * L.nb2 * 4);
  L.soff = take((size_t)kMaxBins * L.nb2 * 4);
  L.stot = take(kMaxBins * 4);
  // whole tiles, so the count kernel's 16-B loads of a partial last group stay in bounds
  const size_t nn = (size_t)tiles * kTile * 4;
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
  const int force_match = force_match_rank();
  if (!workspace || workspace_bytes < L.total) {
    set_error("dd_select_topk: workspace %zu < %zu bytes", workspace_bytes, L.total);
    return DD_EWORKSPACE;
  }
  DD_REQUIRE(reinterpret_cast<uintptr_t>(workspace) % 16 == 0,
             "dd_select_topk: workspace must be 16-byte aligned");
  char* ws = static_cast<char*>(workspace);
  auto* st = reinterpret_cast<State*>(ws + L.state);
  auto* hist = reinterpret_cast<uint32_t*>(ws + L.hist);
  auto* bh = reinterpret_cast<uint32_t*>(ws + L.bh);
  auto* shist = reinterpret_cast<uint32_t*>(ws + L.shist);
  auto* soff = reinterpret_cast<uint32_t*>(ws + L.soff);
  auto* stot = reinterpret_cast<uint32_t*>(ws + L.stot);
  auto* k0 = reinterpret_cast<uint32_t*>(ws + L.k0);
  auto* i0 = reinterpret_cast<uint32_t*>(ws + L.i0);
  auto* k1 = reinterpret_cast<uint32_t*>(ws + L.k1);
  auto* i1 = reinterpret_cast<uint32_t*>(ws + L.i1);
  clear_kernel<<<(unsigned)ceil_div((int64_t)((L.bh - L.state) / 16), 256), 256, 0, s>>>(
      reinterpret_cast<uint4*>(ws + L.state), (int)((L.bh - L.state) / 16));
  DD_CHECK_LAUNCH("dd_select_topk(clear)");
  if (n == 0) {
    if (nan_count_out) nan_out_kernel<<<1, 64, 0, s>>>(st, nan_count_out);
    DD_CHECK_LAUNCH("dd_select_topk(empty)");
    return DD_OK;
  }
  DD_REQUIRE(keys != nullptr, "dd_select_topk: null keys");
  const int vec = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
  hist_top_kernel<<<L.nb1, kHistThreads, 0, s>>>(keys, n, vec, st, hist, bh);
  DD_CHECK_LAUNCH("dd_select_topk(hist)");
  if (k == 0) {
    if (nan_count_out) nan_out_kernel<<<1, 64, 0, s>>>(st, nan_count_out);
    DD_CHECK_LAUNCH("dd_select_topk(nan)");
    return DD_OK;
  }
  DD_REQUIRE(idx_out != nullptr, "dd_select_topk: null idx_out");
  split_kernel<<<L.nb1, kSplitThreads, 0, s>>>(keys, n, (uint32_t)k, st, hist, bh, k0, i0,
                                                nan_count_out);
  DD_CHECK_LAUNCH("dd_select_topk(split)");
  if (!force_match) {
    int dev = -1;
    DD_CHECK_HIP(hipGetDevice(&dev), "dd_select_topk: device");
    if (!probe_once(dev)) lds_order_probe_kernel<<<kProbeBlocks, kThreads, 0, s>>>();
  }
  for (int pass = 0; pass < kPasses; ++pass) {
    const uint32_t* sk = (pass & 1) ? k1 : k0;
    const uint32_t* si = (pass & 1) ? i1 : i0;
    uint32_t* dk = (pass & 1) ? k0 : k1;
    uint32_t* di = (pass & 1) ? i0 : i1;
    count_kernel<<<L.nb2, kThreads, 0, s>>>(sk, st, pass, shist);
    offsets_kernel<<<kMaxBins, kThreads, 0, s>>>(st, shist, L.nb2, soff, stot);
    scatter_kernel<<<L.nb2, kThreads, 0, s>>>(sk, si, st, pass, soff, stot, dk, di, idx_out,
                                              thr_out, force_match);
  }
  DD_CHECK_LAUNCH("dd_select_topk(sort)");
  return DD_OK;
}

}  // extern "C"
