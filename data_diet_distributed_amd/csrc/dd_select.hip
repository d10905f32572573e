// Global keep-set selection: float-key radix select + stable compaction + LSD sort.
//
// Replaces reference get_scores_and_prune.py:22-24 (stable `sorted(..., reverse=True)[:k]`).
// Scores map to order-preserving u32 keys (+0 == -0, NaN below everything).  The k-th key T is
// found by four MSD 8-bit digit passes (LDS-privatised histograms, one global 256-bin
// histogram per pass, a one-block pick kernel that narrows the prefix on device).  A stable
// compaction then writes the keys > T (with their indices, in index order) to a survivor
// buffer and the first r = k - #(> T) indices with key == T straight to their final slots at
// the tail of the output (ties keep ascending index = the reference's loader-visit order under
// the unshuffled protocol).  Four stable LSD passes sort the survivors by key descending.
// Everything stays on device; the host never learns intermediate counts (no syncs).
#include "dd_common.h"

namespace dd {

struct SelState {
  uint32_t prefix, mask, krem, gt;  // after the 4 passes: T, all-ones, r, #(> T)
  uint32_t nan_count;
  uint32_t pad[11];
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

__global__ void sel_init_kernel(SelState* st, uint32_t* hist, uint32_t k) {
  const int t = threadIdx.x;
  if (t == 0) {
    st->prefix = 0;
    st->mask = 0;
    st->krem = k;
    st->gt = 0;
    st->nan_count = 0;
  }
  hist[t] = 0;  // 256 threads
}

// MSD digit histogram over the keys that still match the prefix
__global__ __launch_bounds__(256) void sel_hist_kernel(const float* __restrict__ keys, int64_t n,
                                                       SelState* st, uint32_t* hist, int shift,
                                                       int count_nan) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t prefix = st->prefix, mask = st->mask;
  uint32_t nans = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    bool isn = false;
    const uint32_t u = order_key(keys[i], isn);
    nans += isn;
    if ((u & mask) == prefix) atomicAdd(&h[(u >> shift) & 255u], 1u);
  }
  if (count_nan) {
    // nans are few; one atomic per lane that saw any
    if (nans) atomicAdd(&st->nan_count, nans);
  }
  __syncthreads();
  const uint32_t c = h[threadIdx.x];
  if (c) atomicAdd(&hist[threadIdx.x], c);
}

// one block of 256: digit d = 255 - t (descending); find the bin holding the krem-th key
__global__ __launch_bounds__(256) void sel_pick_kernel(SelState* st, uint32_t* hist, int shift) {
  __shared__ uint32_t s[256];
  const int t = threadIdx.x;
  const uint32_t c = hist[255 - t];
  s[t] = c;
  __syncthreads();
  // inclusive Hillis-Steele scan (256 entries)
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t v = t >= o ? s[t - o] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  const uint32_t incl = s[t], excl = incl - c;
  const uint32_t krem = st->krem;
  __syncthreads();
  if (excl < krem && krem <= incl) {
    const uint32_t d = 255u - (uint32_t)t;
    st->gt += excl;
    st->krem = krem - excl;
    st->prefix |= d << shift;
    st->mask |= 255u << shift;
  }
  hist[t] = 0;  // ready for the next pass
}

// ---- stable compaction ----------------------------------------------------------------------
__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// counts of (> T) and (== T) per contiguous chunk
__global__ __launch_bounds__(256) void sel_count_kernel(const float* __restrict__ keys, int64_t n,
                                                        int64_t chunk, const SelState* st,
                                                        uint32_t* cnt_gt, uint32_t* cnt_eq) {
  __shared__ uint32_t sg[4], se[4];
  const uint32_t T = st->prefix;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  uint32_t g = 0, e = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
    bool isn = false;
    const uint32_t u = order_key(keys[i], isn);
    g += u > T;
    e += u == T;
  }
  // block reduce
  for (int o = 32; o > 0; o >>= 1) {
    g += __shfl_xor(g, o);
    e += __shfl_xor(e, o);
  }
  if ((threadIdx.x & 63) == 0) {
    sg[threadIdx.x >> 6] = g;
    se[threadIdx.x >> 6] = e;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    cnt_gt[blockIdx.x] = sg[0] + sg[1] + sg[2] + sg[3];
    cnt_eq[blockIdx.x] = se[0] + se[1] + se[2] + se[3];
  }
}

// single-block exclusive scan of len u32 values (len <= 1024 * 1024)
__global__ __launch_bounds__(1024) void exclusive_scan_kernel(const uint32_t* __restrict__ in,
                                                              uint32_t* __restrict__ out,
                                                              int64_t len) {
  __shared__ uint32_t s[1024];
  const int t = threadIdx.x;
  const int64_t per = (len + 1023) / 1024;
  const int64_t lo = t * per, hi = (lo + per < len) ? lo + per : len;
  uint32_t sum = 0;
  for (int64_t i = lo; i < hi; ++i) sum += in[i];
  s[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t v = t >= o ? s[t - o] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  uint32_t run = s[t] - sum;
  for (int64_t i = lo; i < hi; ++i) {
    const uint32_t v = in[i];
    out[i] = run;
    run += v;
  }
}

// per chunk, in order: keys > T -> survivors (stable), first r keys == T -> out[gt + rank]
__global__ __launch_bounds__(256) void sel_write_kernel(const float* __restrict__ keys, int64_t n,
                                                        int64_t chunk, const SelState* st,
                                                        const uint32_t* off_gt,
                                                        const uint32_t* off_eq,
                                                        uint32_t* surv_key, uint32_t* surv_idx,
                                                        int64_t* out_idx) {
  __shared__ uint32_t wg[4], we[4];
  const uint32_t T = st->prefix, r = st->krem, gt_total = st->gt;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  uint32_t base_g = off_gt[blockIdx.x], base_e = off_eq[blockIdx.x];
  for (int64_t t0 = lo; t0 < hi; t0 += 256) {
    const int64_t i = t0 + threadIdx.x;
    uint32_t u = 0;
    bool valid = i < hi;
    if (valid) {
      bool isn = false;
      u = order_key(keys[i], isn);
    }
    const bool pg = valid && u > T, pe = valid && u == T;
    const uint64_t bg = __ballot(pg), be = __ballot(pe);
    if (lane == 0) {
      wg[wv] = __popcll(bg);
      we[wv] = __popcll(be);
    }
    __syncthreads();
    uint32_t pre_g = 0, pre_e = 0, tot_g = 0, tot_e = 0;
    for (int w = 0; w < 4; ++w) {
      if (w < wv) {
        pre_g += wg[w];
        pre_e += we[w];
      }
      tot_g += wg[w];
      tot_e += we[w];
    }
    if (pg) {
      const uint32_t pos = base_g + pre_g + __popcll(bg & lanemask_lt(lane));
      surv_key[pos] = u;
      surv_idx[pos] = (uint32_t)i;
    }
    if (pe) {
      const uint32_t er = base_e + pre_e + __popcll(be & lanemask_lt(lane));
      if (er < r) out_idx[gt_total + er] = i;
    }
    base_g += tot_g;
    base_e += tot_e;
    __syncthreads();
  }
}

// ---- LSD radix sort of the survivors (key descending, stable) ------------------------------
__device__ __forceinline__ int64_t sort_chunk(uint32_t m, int nb) {
  int64_t c = ((int64_t)m + nb - 1) / nb;
  return (c + 255) / 256 * 256;
}

__device__ __forceinline__ uint32_t desc_digit(uint32_t u, int shift) {
  return 255u - ((u >> shift) & 255u);
}

// hist[d * nb + blk]
__global__ __launch_bounds__(256) void sort_hist_kernel(const uint32_t* __restrict__ key,
                                                        const SelState* st, int shift,
                                                        uint32_t* hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t m = st->gt;
  const int nb = gridDim.x;
  const int64_t chunk = sort_chunk(m, nb);
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < (int64_t)m ? lo + chunk : (int64_t)m;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256)
    atomicAdd(&h[desc_digit(key[i], shift)], 1u);
  __syncthreads();
  hist[(int64_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// per-digit exclusive scan of the block histograms hist[d * nb + b] over b (one block per
// digit, nb <= 1024): offs[d * nb + b] = sum_{b' < b} hist[d][b'], tot[d] = the digit's total.
// The digit bases (a 256-entry scan of tot) are added by the scatter blocks themselves.
__global__ __launch_bounds__(1024) void sort_offsets_kernel(const uint32_t* __restrict__ hist,
                                                            int nb, uint32_t* __restrict__ offs,
                                                            uint32_t* __restrict__ tot) {
  __shared__ uint32_t s[1024];
  const int t = threadIdx.x, d = blockIdx.x;
  const uint32_t v = t < nb ? hist[(int64_t)d * nb + t] : 0u;
  s[t] = v;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t a = t >= o ? s[t - o] : 0u;
    __syncthreads();
    s[t] += a;
    __syncthreads();
  }
  if (t < nb) offs[(int64_t)d * nb + t] = s[t] - v;
  if (t == 1023) tot[d] = s[t];
}

// stable scatter: tiles of 256 in order; rank inside a wave by 8-ballot match, across waves
// through LDS counts
template <bool LAST>
__global__ __launch_bounds__(256) void sort_scatter_kernel(const uint32_t* __restrict__ key,
                                                           const uint32_t* __restrict__ idx,
                                                           const SelState* st, int shift,
                                                           const uint32_t* __restrict__ offs,
                                                           const uint32_t* __restrict__ tot,
                                                           uint32_t* __restrict__ okey,
                                                           uint32_t* __restrict__ oidx,
                                                           int64_t* __restrict__ out_final) {
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[4][256];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t m = st->gt;
  const int nb = gridDim.x;
  const int64_t chunk = sort_chunk(m, nb);
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < (int64_t)m ? lo + chunk : (int64_t)m;
  // digit base = exclusive scan of the digit totals (descending digits already), in LDS
  {
    const uint32_t c = tot[t];
    base[t] = c;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const uint32_t a = t >= o ? base[t - o] : 0u;
      __syncthreads();
      base[t] += a;
      __syncthreads();
    }
    base[t] = base[t] - c + offs[(int64_t)t * nb + blockIdx.x];
    __syncthreads();
  }
  for (int64_t t0 = lo; t0 < hi; t0 += 256) {
    for (int w = 0; w < 4; ++w) wcnt[w][t] = 0;
    __syncthreads();
    const int64_t i = t0 + t;
    const bool valid = i < hi;
    const uint32_t u = valid ? key[i] : 0u;
    const uint32_t d = valid ? desc_digit(u, shift) : 0u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const uint64_t b = __ballot((d >> bit) & 1u);
      peers &= ((d >> bit) & 1u) ? b : ~b;
    }
    const uint32_t rank = __popcll(peers & lanemask_lt(lane));
    if (valid && rank == 0) wcnt[wv][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pre = 0;
      for (int w = 0; w < wv; ++w) pre += wcnt[w][d];
      const uint32_t pos = base[d] + pre + rank;
      if (LAST) {
        out_final[pos] = (int64_t)idx[i];
      } else {
        okey[pos] = u;
        oidx[pos] = idx[i];
      }
    }
    __syncthreads();
    base[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
    __syncthreads();
  }
}

__global__ void sel_finish_kernel(const SelState* st, float* thr_out, int32_t* nan_out) {
  if (threadIdx.x == 0) {
    if (thr_out) *thr_out = key_to_float(st->prefix);
    if (nan_out) *nan_out = (int32_t)st->nan_count;
  }
}

struct WsLayout {
  size_t state, hist, cnt_gt, cnt_eq, off_gt, off_eq, shist, soff, stot, k0, i0, k1, i1, total;
  int nb_c, nb_s;
  int64_t chunk_c;
};

static WsLayout layout(int64_t n) {
  WsLayout L{};
  const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(1024, ceil_div(n, 2048)));
  L.nb_c = (int)nb;
  L.chunk_c = ceil_div(ceil_div(std::max<int64_t>(n, 1), nb), 256) * 256;
  L.nb_s = (int)nb;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  L.state = take(sizeof(SelState));
  L.hist = take(256 * 4);
  L.cnt_gt = take(nb * 4);
  L.cnt_eq = take(nb * 4);
  L.off_gt = take(nb * 4);
  L.off_eq = take(nb * 4);
  L.shist = take(256 * nb * 4);
  L.soff = take(256 * nb * 4);
  L.stot = take(256 * 4);
  const size_t nn = (size_t)std::max<int64_t>(n, 1) * 4;
  L.k0 = take(nn);
  L.i0 = take(nn);
  L.k1 = take(nn);
  L.i1 = take(nn);
  L.total = o;
  return L;
}

}  // namespace dd

using namespace dd;

extern "C" {

size_t dd_select_workspace_bytes(int64_t n) {
  if (n < 0) return 0;
  return layout(n).total;
}

int dd_select_topk(const float* keys, int64_t n, int64_t k, int64_t* idx_out, float* thr_out,
                   int32_t* nan_count_out, void* workspace, size_t workspace_bytes,
                   void* stream) {
  clear_error();
  DD_REQUIRE(n >= 0 && k >= 0 && k <= n, "dd_select_topk: need 0 <= k <= n (k=%lld n=%lld)",
             (long long)k, (long long)n);
  DD_REQUIRE(n < (1ll << 31), "dd_select_topk: n >= 2^31 unsupported");
  hipStream_t s = as_stream(stream);
  const WsLayout L = layout(n);
  if (!workspace || workspace_bytes < L.total) {
    set_error("dd_select_topk: workspace %zu < %zu bytes", workspace_bytes, L.total);
    return DD_EWORKSPACE;
  }
  char* ws = static_cast<char*>(workspace);
  SelState* st = reinterpret_cast<SelState*>(ws + L.state);
  uint32_t* hist = reinterpret_cast<uint32_t*>(ws + L.hist);
  sel_init_kernel<<<1, 256, 0, s>>>(st, hist, (uint32_t)k);
  DD_CHECK_LAUNCH("dd_select_topk(init)");
  if (n == 0 || k == 0) {
    // still report NaNs for k == 0
    if (n > 0 && nan_count_out) {
      sel_hist_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256 * 8), 2048), 256, 0, s>>>(
          keys, n, st, hist, 24, 1);
      DD_CHECK_LAUNCH("dd_select_topk(nan)");
    }
    sel_finish_kernel<<<1, 64, 0, s>>>(st, nullptr, nan_count_out);
    DD_CHECK_LAUNCH("dd_select_topk(finish)");
    return DD_OK;
  }
  DD_REQUIRE(keys && idx_out, "dd_select_topk: null keys/idx_out");
  const unsigned hgrid = (unsigned)std::min<int64_t>(ceil_div(n, 256 * 8), 2048);
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    sel_hist_kernel<<<hgrid, 256, 0, s>>>(keys, n, st, hist, shift, pass == 0);
    sel_pick_kernel<<<1, 256, 0, s>>>(st, hist, shift);
  }
  DD_CHECK_LAUNCH("dd_select_topk(select)");
  uint32_t* cnt_gt = reinterpret_cast<uint32_t*>(ws + L.cnt_gt);
  uint32_t* cnt_eq = reinterpret_cast<uint32_t*>(ws + L.cnt_eq);
  uint32_t* off_gt = reinterpret_cast<uint32_t*>(ws + L.off_gt);
  uint32_t* off_eq = reinterpret_cast<uint32_t*>(ws + L.off_eq);
  uint32_t* k0 = reinterpret_cast<uint32_t*>(ws + L.k0);
  uint32_t* i0 = reinterpret_cast<uint32_t*>(ws + L.i0);
  uint32_t* k1 = reinterpret_cast<uint32_t*>(ws + L.k1);
  uint32_t* i1 = reinterpret_cast<uint32_t*>(ws + L.i1);
  sel_count_kernel<<<L.nb_c, 256, 0, s>>>(keys, n, L.chunk_c, st, cnt_gt, cnt_eq);
  exclusive_scan_kernel<<<1, 1024, 0, s>>>(cnt_gt, off_gt, L.nb_c);
  exclusive_scan_kernel<<<1, 1024, 0, s>>>(cnt_eq, off_eq, L.nb_c);
  sel_write_kernel<<<L.nb_c, 256, 0, s>>>(keys, n, L.chunk_c, st, off_gt, off_eq, k0, i0,
                                          idx_out);
  DD_CHECK_LAUNCH("dd_select_topk(compact)");
  uint32_t* shist = reinterpret_cast<uint32_t*>(ws + L.shist);
  uint32_t* soff = reinterpret_cast<uint32_t*>(ws + L.soff);
  uint32_t* stot = reinterpret_cast<uint32_t*>(ws + L.stot);
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    const uint32_t* sk = (pass & 1) ? k1 : k0;
    const uint32_t* si = (pass & 1) ? i1 : i0;
    uint32_t* dk = (pass & 1) ? k0 : k1;
    uint32_t* di = (pass & 1) ? i0 : i1;
    sort_hist_kernel<<<L.nb_s, 256, 0, s>>>(sk, st, shift, shist);
    sort_offsets_kernel<<<256, 1024, 0, s>>>(shist, L.nb_s, soff, stot);
    if (pass == 3)
      sort_scatter_kernel<true><<<L.nb_s, 256, 0, s>>>(sk, si, st, shift, soff, stot, dk, di,
                                                       idx_out);
    else
      sort_scatter_kernel<false><<<L.nb_s, 256, 0, s>>>(sk, si, st, shift, soff, stot, dk, di,
                                                        idx_out);
  }
  DD_CHECK_LAUNCH("dd_select_topk(sort)");
  sel_finish_kernel<<<1, 64, 0, s>>>(st, thr_out, nan_count_out);
  DD_CHECK_LAUNCH("dd_select_topk(finish)");
  return DD_OK;
}

}  // extern "C"
