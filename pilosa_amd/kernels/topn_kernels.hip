// Device TopN with a src filter: TopN(f, <src>, n) without counting
// src ∩ row for every cached row one pair at a time.
//
// Reference semantics (fragment.go:1568-1700 `top`, executor.go:863-930):
// per shard the ranked cache (rows by count desc, id asc) is walked; the
// first n rows with count = |src ∩ row| >= max(1, threshold) fill a heap,
// T = the heap minimum; later rows are pushed while their cached count is
// >= T and their src count is >= T, and the walk stops at the first cached
// count < T.  Phase 1 sums the pushed (row, count) pairs over shards, phase 2
// (ids=) re-counts exactly those ids on every shard.
//
// MI355X design.  The pair-per-candidate formulation costs |cache| row
// intersections per (query, shard) (~10k in the Zipf headline index).  We
// invert it: a column-major *slot index* of the cached rows is kept in HBM
// next to the arena (per shard: colptr[2^20+1] + u16 cache slots, 2 B per
// set bit of a cached row), so the src counts of ALL cached rows of a shard
// are one histogram over src's columns: |src_s| x (bits per column) LDS
// increments.  One 1024-thread workgroup owns one (query, shard):
//   1. zero an LDS histogram over the K cache slots (u32 / u16 / u8 counters
//      by the slot's cached-count bound: K = 50,000 Zipf slots fit in ~52 KB,
//      two 1024-thread workgroups per CU);
//   2. stream src's materialised columns and, per column, its slot list;
//   3. mode 1: run the reference heap walk with block scans over the slots
//      (fill = first n qualifying slots, T = their min, then the sorted cache
//      counts bound the tail) and add pushed counts into acc[q][row];
//      mode 2: gather the counts of the phase-1 ids (slot map, with an exact
//      probe for ids outside this shard's cache).
// Rows are addressed in an "acc space" (sorted row ids shared by every rank of
// a multi-GPU node) so acc / out reduce with one all-reduce.
// The index is built on the device by two passes over the cached rows'
// containers (count per column, then scatter slots behind an exclusive scan).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "kernels.h"

// Cost-isolation bits of the src-TopN kernels (PILOSA_TOPN_DBG): read only
// in the kbench module (pilosa_amd/native/build.py --kbench); the shipped
// kernels compile every such branch out.
#ifdef PK_KBENCH
#define PK_DBG(p) ((p).dbg)
#else
#define PK_DBG(p) 0
#endif

namespace pk {
namespace {

constexpr int TN_THREADS = 1024;
constexpr int TN_WAVES = TN_THREADS / 64;
constexpr int64_t SW = int64_t(1) << 20;  // columns per shard
constexpr int64_t CP_STRIDE = SW + 1;      // colptr entries per shard

__device__ __forceinline__ uint32_t tn_xcd_remap(uint32_t bid, uint32_t nblk) {
  // consecutive units (same shard, different queries) land on one XCD so the
  // shard's colptr / slot lists are shared through that XCD's L2
  const uint32_t nx = 8;
  const uint32_t xcd = bid % nx, loc = bid / nx;
  const uint32_t q = nblk / nx, r = nblk % nx;
  const uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + loc;
}

#if defined(__HIP_DEVICE_COMPILE__)
#define TN_GLOBAL __attribute__((address_space(1)))
#else
#define TN_GLOBAL
#endif
template <class T>
__device__ __forceinline__ const TN_GLOBAL T* gp(const T* ptr) {
  return (const TN_GLOBAL T*)(ptr);
}

// f(x) for every value x of the container described by meta word m; the
// threads tid, tid + nthr, ... of a group split the work.
template <class F>
__device__ __forceinline__ void container_values(const uint16_t* payload, int64_t m, int tid, int nthr, F&& f) {
  const uint16_t* p = payload + meta_off16(m) * 8;
  const int t = meta_type(m);
  if (t == CT_ARRAY) {
    const int n = meta_n(m);
    for (int i = tid; i < n; i += nthr) f(int(p[i]));
  } else if (t == CT_BITMAP) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(p);
    for (int i = tid; i < 1024; i += nthr)
      for (uint64_t b = w[i]; b; b &= b - 1) f(i * 64 + __builtin_ctzll(b));
  } else {
    const int nr = p[0];
    const uint16_t* r = p + 8;
    for (int k = 0; k < nr; k++) {
      const int a = r[2 * k], b = r[2 * k + 1];
      for (int x = a + tid; x <= b; x += nthr) f(x);
    }
  }
}

// Pass 1 (FILL=false): colcnt[s][col] = number of cached rows of shard s
// ranked k >= k0 (the tail; ranks below k0 are counted by topn_hot_kernel)
// with a bit at col.  Pass 2 (FILL=true): scatter the tail slot k - k0 of
// each such (row, col) to slots[entbase[s] + colptr[s][col] + cursor].  One
// wave per cache entry (s, k); grid-stride.
template <bool FILL>
__global__ __launch_bounds__(256) void topn_index_kernel(ViewDev v, int S, int K, int k0,
                                                         const int32_t* __restrict__ cache_dense,
                                                         uint32_t* __restrict__ colcnt,
                                                         const uint32_t* __restrict__ colptr,
                                                         const int64_t* __restrict__ entbase,
                                                         uint16_t* __restrict__ slots) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = int64_t(gridDim.x) * 4;
  const int Kt = K - k0;
  const int64_t total = int64_t(S) * Kt;
  for (int64_t e = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); e < total; e += nw) {
    const int s = int(e / Kt);
    const int kt = int(e - int64_t(s) * Kt);
    const int d = cache_dense[int64_t(s) * K + k0 + kt];
    if (d < 0) continue;
    const uint16_t k = uint16_t(kt);
    const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
    const int64_t sb = v.shard_base[s];
    const int64_t c0 = sb + rp[d], c1 = sb + rp[d + 1];
    for (int64_t c = c0; c < c1; c++) {
      const int64_t m = v.meta[c];
      const int64_t colbase = int64_t(meta_j(m)) << 16;
      uint32_t* cc = colcnt + int64_t(s) * SW + colbase;
      if constexpr (!FILL) {
        container_values(v.payload, m, lane, 64, [&](int x) { atomicAdd(cc + x, 1u); });
      } else {
        const uint32_t* cp = colptr + int64_t(s) * CP_STRIDE + colbase;
        uint16_t* sl = slots + entbase[s];
        container_values(v.payload, m, lane, 64, [&](int x) {
          const uint32_t pos = atomicAdd(cc + x, 1u);
          sl[cp[x] + pos] = k;
        });
      }
    }
  }
}

// ---------------------------------------------------------------- src TopN

// Slot histogram layout, three counter widths chosen from the cached counts
// (a slot's src count never exceeds its row's count in the shard):
//   [0, H32)   u32   slots whose cached count can reach 2^16
//   [H32, H16) u16   two per word (cached counts < 2^16 in every shard)
//   [H16, K)   u8    four per word (cached counts < 2^8)
// Packed fields are bumped with a shifted 32-bit LDS atomic add; they never
// carry into their neighbour because the count bound holds.
struct HistLayout {
  int H32, H16, W16, words;
  __device__ __forceinline__ HistLayout(int K, int h32, int h16) : H32(h32), H16(h16) {
    W16 = H32 + ((H16 - H32 + 1) >> 1);
    words = W16 + ((K - H16 + 3) >> 2);
  }
};

// Counter word and increment of slot k, branch-free (one ds_add per slot
// whatever the tier mix of a wave).
__device__ __forceinline__ void hist_inc(uint32_t* h, const HistLayout& L, int k) {
  const int r16 = k - L.H32, r8 = k - L.H16;
  const bool t32 = k < L.H32, t16 = k < L.H16;
  const int w = t32 ? k : (t16 ? L.H32 + (r16 >> 1) : L.W16 + (r8 >> 2));
  const int sh = t32 ? 0 : (t16 ? (r16 & 1) << 4 : (r8 & 3) << 3);
  atomicAdd(h + w, 1u << sh);
}

template <class P>
__device__ __forceinline__ uint32_t hist_get(P h, const HistLayout& L, int k) {
  if (k < L.H32) return h[k];
  if (k < L.H16) {
    const int r = k - L.H32;
    return (h[L.H32 + (r >> 1)] >> ((r & 1) * 16)) & 0xffffu;
  }
  const int r = k - L.H16;
  return (h[L.W16 + (r >> 2)] >> ((r & 3) * 8)) & 0xffu;
}

// src count of cache slot k of unit (q, s): the hot-rank count matrix below
// R, the tail histogram (tail-relative slot) above.
template <class P>
__device__ __forceinline__ uint32_t slot_count(const TopNLaunch& p, P h, const HistLayout& L, int q, int s, int k) {
  if (k < p.R) return p.hot_cnt[(int64_t(s) * p.Q + q) * p.R + k];
  return hist_get(h, L, k - p.R);
}

struct BlockScratch {
  int wsum[TN_WAVES];
  uint32_t wmin[TN_WAVES];
  int wmax[TN_WAVES];
};

// Exclusive rank of `flag` among the block's threads (thread order) and the
// block total.  Contains two barriers.
__device__ __forceinline__ int block_rank(bool flag, BlockScratch& bs, int& total) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t m = __ballot(flag);
  const int below = __popcll(m & ((uint64_t(1) << lane) - 1));
  if (lane == 0) bs.wsum[wave] = __popcll(m);
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < TN_WAVES; w++) {
    const int c = bs.wsum[w];
    pre += w < wave ? c : 0;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return pre + below;
}

__device__ __forceinline__ void block_minmax(uint32_t vmin, int vmax, BlockScratch& bs, uint32_t& omin, int& omax) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    vmin = min(vmin, uint32_t(__shfl_xor(int(vmin), o, 64)));
    vmax = max(vmax, __shfl_xor(vmax, o, 64));
  }
  if (lane == 0) {
    bs.wmin[wave] = vmin;
    bs.wmax[wave] = vmax;
  }
  __syncthreads();
  uint32_t a = 0xffffffffu;
  int b = -1;
#pragma unroll
  for (int w = 0; w < TN_WAVES; w++) {
    a = min(a, bs.wmin[w]);
    b = max(b, bs.wmax[w]);
  }
  __syncthreads();
  omin = a;
  omax = b;
}

// |src(q, s) ∩ row d of shard s| by probing the (sorted) materialised src
// containers with the row's values: ids outside this shard's cache (rare, cold).
__device__ uint32_t src_row_count(const ViewDev& v, int s, int d, const int32_t* scnt, const int64_t* soff,
                                  const uint16_t* svals) {
  const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
  const int64_t sb = v.shard_base[s];
  uint32_t total = 0;
  for (int64_t c = sb + rp[d]; c < sb + rp[d + 1]; c++) {
    const int64_t m = v.meta[c];
    const int j = meta_j(m);
    const int n = scnt[j];
    if (n <= 0) continue;
    const uint16_t* a = svals + soff[j];
    if (n > ARRAY_MAX) {
      const uint64_t* w = reinterpret_cast<const uint64_t*>(a);
      container_values(v.payload, m, 0, 1, [&](int x) { total += uint32_t(w[x >> 6] >> (x & 63)) & 1u; });
    } else {
      container_values(v.payload, m, 0, 1, [&](int x) {
        int lo = 0, hi = n;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (int(a[mid]) < x) lo = mid + 1; else hi = mid;
        }
        total += (lo < n && int(a[lo]) == x) ? 1u : 0u;
      });
    }
  }
  return total;
}

// the same over the p.M arena sub-shards of fragment s (query q's src)
__device__ uint32_t src_row_count_frag(const TopNLaunch& p, int q, int s, int d) {
  uint32_t total = 0;
  for (int m = 0; m < p.M; m++) {
    const int ds = s * p.M + m;
    const int64_t kb = (int64_t(q) * p.S * p.M + ds) * 16;
    total += src_row_count(p.v, ds, d, p.src_counts + kb, p.src_offs + kb, p.src_vals);
  }
  return total;
}

__device__ __forceinline__ int64_t unit_index(const TopNLaunch& p, int q, int s) { return int64_t(q) * p.S + s; }

__device__ __forceinline__ int64_t unit_hist_base(const TopNLaunch& p, int q, int s, int words) {
  return (int64_t(q) * p.S + s) * int64_t(words);
}

template <int MODE>
__global__ __launch_bounds__(TN_THREADS, 8) void topn_src_kernel(TopNLaunch p) {
  extern __shared__ uint32_t hist[];
  __shared__ BlockScratch bs;
  const uint32_t unit = tn_xcd_remap(blockIdx.x, gridDim.x);
  const int q = int(unit % p.Q), s = int(unit / p.Q);
  const int tid = threadIdx.x;
  const int K = p.K;
  const HistLayout L(K - p.R, p.H32, p.H16);
  const int words = L.words;
  const uint32_t mt = uint32_t(max(1, p.min_threshold[q]));
  const int32_t* cc = p.cache_cnt + int64_t(s) * K;
  // Mode 1 with hot ranks: replay the fill over the hot counts first.  When
  // the walk provably ends inside the hot ranks (n rows found and the first
  // tail rank's cached count below their minimum, or cached counts below the
  // threshold), the tail histogram is never read: skip building it.  Dense
  // srcs -- the ones whose histograms are expensive -- end here.
  bool need_tail = p.R < K && !(PK_DBG(p) & 1);
  if (MODE == 1 && need_tail && p.R > 0) {
    const int nmax = p.ns[q];
    int found = 0;
    uint32_t T = 0xffffffffu;
    bool filled = false;
    for (int base = 0; base < p.R; base += TN_THREADS) {
      const int k = base + tid;
      const uint32_t cnt = k < p.R ? uint32_t(cc[k]) : 0u;
      const uint32_t cv = cnt >= mt ? p.hot_cnt[(int64_t(s) * p.Q + q) * p.R + k] : 0u;
      const bool ok = cnt >= mt && cv >= mt;
      int tot;
      const int rank = block_rank(ok, bs, tot);
      const bool take = ok && (nmax == 0 || found + rank < nmax);
      uint32_t tmin;
      int pmax;
      block_minmax(take ? cv : 0xffffffffu, -1, bs, tmin, pmax);
      T = min(T, uint32_t(__builtin_amdgcn_readfirstlane(int(tmin))));
      found += __builtin_amdgcn_readfirstlane(tot);
      if (nmax > 0 && found >= nmax) {
        filled = true;
        break;
      }
    }
    const uint32_t c_r = uint32_t(cc[p.R]);
    if (c_r < mt || (filled && c_r < T)) need_tail = false;
  }
  if (MODE == 1 && p.tail_built) {
    if (tid == 0) p.tail_built[unit_index(p, q, s)] = need_tail ? 1 : 0;
  }
  if (need_tail) {
    for (int i = tid; i < words; i += TN_THREADS) hist[i] = 0;
  }
  __syncthreads();

  // histogram of cache slots over src's columns, 4 columns per thread in
  // flight.  A column's slot run (~bits-per-column u16 entries) is read as
  // the two aligned 16-byte words starting at or below it -- 8 independent
  // vector loads for the 4 columns, issued before any is consumed, one or
  // two cache lines per column -- and counted with predicated LDS adds;
  // longer runs finish in a short tail loop.  (The previous shape, a per-lane
  // loop of u16 loads per column, serialised ~15 dependent round trips per 4
  // columns: 54 ms for 16 hot-src queries over 954 shards.)
  // a fragment wider than 2^20 columns is p.M consecutive arena sub-shards:
  // its histogram sums the slot runs of all of them (the slot index and the
  // materialised src are per sub-shard, the cache and the walk per fragment)
  const int64_t amax = ((p.slots_n - 16) & ~int64_t(7));
  const auto sl4 = gp(reinterpret_cast<const uint4*>(p.slots));
  // the array containers of src's 16 keys (of one arena sub-shard) as ONE
  // flat value stream: fl_pre = exclusive prefix of their sizes, fl_off =
  // their payload offsets.  Every thread takes values of any key, so a
  // sparse src (a few hundred values per shard) is one round of run4 instead
  // of one per key -- 16 serial slot-run round trips (cold srcs: 2.6 of 3.6 ms
  // of the phase, call U).  Bitmap containers keep the per-key loop.
  __shared__ int fl_pre[17];
  __shared__ int64_t fl_off[16];
  for (int m = 0; m < (need_tail ? p.M : 0); m++) {
    const int ds = s * p.M + m;
    const int64_t kb = (int64_t(q) * p.S * p.M + ds) * 16;
    const int64_t eb = p.entbase[ds];
    // colptr of the sub-shard, indexed by the column (key << 16 | value)
    const auto cp = gp(p.colptr + int64_t(ds) * CP_STRIDE);
    auto run4 = [&](const int (&x)[4]) {
      uint32_t e0[4], e1[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int xx = x[r] >= 0 ? x[r] : 0;
        e0[r] = cp[xx];
        e1[r] = x[r] >= 0 ? cp[xx + 1] : e0[r];
      }
      int64_t a[4];
      uint4 w0[4], w1[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        // exec-masked: columns without (tail) slots fetch nothing
        a[r] = min((eb + int64_t(e0[r])) & ~int64_t(7), amax);
        const int64_t hi = eb + int64_t(e1[r]) - a[r];
        w0[r] = make_uint4(0, 0, 0, 0);
        w1[r] = make_uint4(0, 0, 0, 0);
        if (e1[r] > e0[r]) w0[r] = sl4[a[r] >> 3];
        if (hi > 8) w1[r] = sl4[(a[r] >> 3) + 1];
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int lo = int(eb + int64_t(e0[r]) - a[r]), hi = int(eb + int64_t(e1[r]) - a[r]);
        const uint32_t wd[8] = {w0[r].x, w0[r].y, w0[r].z, w0[r].w, w1[r].x, w1[r].y, w1[r].z, w1[r].w};
#pragma unroll
        for (int t = 0; t < 16; t++)
          if (t >= lo && t < hi) hist_inc(hist, L, int((wd[t >> 1] >> ((t & 1) << 4)) & 0xffffu));
        for (int b = 16; b < hi; b += 8) {
          const uint4 w = sl4[(a[r] + b) >> 3];
          const uint32_t wt[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int t = 0; t < 8; t++)
            if (b + t < hi) hist_inc(hist, L, int((wt[t >> 1] >> ((t & 1) << 4)) & 0xffffu));
        }
      }
    };
    if (tid == 0) {
      int acc = 0;
      for (int j = 0; j < 16; j++) {
        const int n = p.src_counts[kb + j];
        fl_pre[j] = acc;
        fl_off[j] = p.src_offs[kb + j];
        acc += (n > 0 && n <= ARRAY_MAX) ? n : 0;
      }
      fl_pre[16] = acc;
    }
    __syncthreads();
    const int N = fl_pre[16];
    for (int i = tid; i < N; i += 4 * TN_THREADS) {
      int x[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int idx = i + r * TN_THREADS;
        x[r] = -1;
        if (idx < N) {
          int j = 0;   // the key holding value idx: the largest j with fl_pre[j] <= idx
#pragma unroll
          for (int st = 8; st > 0; st >>= 1)
            if (fl_pre[j + st] <= idx) j += st;
          x[r] = (j << 16) | int(p.src_vals[fl_off[j] + (idx - fl_pre[j])]);
        }
      }
      run4(x);
    }
    __syncthreads();   // fl_pre / fl_off are rewritten for the next sub-shard
    for (int j = 0; j < 16; j++) {
      const int n = p.src_counts[kb + j];
      if (n <= ARRAY_MAX) continue;
      const auto w = gp(reinterpret_cast<const uint64_t*>(p.src_vals + p.src_offs[kb + j]));
      for (int i = tid; i < 1024; i += TN_THREADS) {
        uint64_t b = w[i];
        while (b) {
          int x[4];
#pragma unroll
          for (int r = 0; r < 4; r++) {
            x[r] = b ? (j << 16) | (i * 64 + __builtin_ctzll(b)) : -1;
            b &= b ? b - 1 : 0;
          }
          run4(x);
        }
      }
    }
  }
  __syncthreads();
  if (MODE == 1 && p.hist_out && need_tail) {
    // keep the histogram for the ids= re-count (topn_gather_kernel)
    uint32_t* ho = p.hist_out + unit_hist_base(p, q, s, words);
    for (int i = tid; i < words; i += TN_THREADS) ho[i] = hist[i];
  }

  if (MODE == 1 && (PK_DBG(p) & 2)) return;
  if constexpr (MODE == 1) {
    const int32_t* ca = p.cache_acc + int64_t(s) * K;
    int32_t* acc = p.acc + int64_t(q) * p.A;
    const int nmax = p.ns[q];
    int found = 0, P = -1;
    uint32_t T = 0xffffffffu;
    bool filled = false;
    // fill phase: the first nmax slots with cached count and src count >= mt
    for (int base = 0; base < K; base += TN_THREADS) {
      const int k = base + tid;
      const uint32_t cnt = k < K ? uint32_t(cc[k]) : 0u;
      const uint32_t cv = cnt >= mt ? slot_count(p, hist, L, q, s, k) : 0u;
      const bool ok = cnt >= mt && cv >= mt;
      int tot;
      const int rank = block_rank(ok, bs, tot);
      const bool take = ok && (nmax == 0 || found + rank < nmax);
      if (take && !(PK_DBG(p) & 8192)) atomicAdd(acc + ca[k], int32_t(cv));
      uint32_t tmin;
      int pmax;
      block_minmax(take ? cv : 0xffffffffu, take ? k : -1, bs, tmin, pmax);
      // block-uniform: keep them in SGPRs
      T = min(T, uint32_t(__builtin_amdgcn_readfirstlane(int(tmin))));
      P = max(P, __builtin_amdgcn_readfirstlane(pmax));
      found += __builtin_amdgcn_readfirstlane(tot);
      if (nmax > 0 && found >= nmax) {
        filled = true;
        break;
      }
      // cached counts are sorted desc: nothing after a chunk ending below mt qualifies
      if (uint32_t(cc[min(base + TN_THREADS, K) - 1]) < mt) break;
    }
    if (filled) {
      // tail: rows whose cached count can still reach the heap minimum T
      for (int base = P + 1; base < K; base += TN_THREADS) {
        const int k = base + tid;
        if (k < K && uint32_t(cc[k]) >= T) {
          const uint32_t cv = slot_count(p, hist, L, q, s, k);
          if (cv >= T && !(PK_DBG(p) & 8192)) atomicAdd(acc + ca[k], int32_t(cv));
        }
        if (uint32_t(cc[min(base + TN_THREADS, K) - 1]) < T) break;
      }
    }
  } else {
    const int32_t* sm = p.slotmap + int64_t(s) * p.A;
    const int64_t p0 = p.pair_off[q], p1 = p.pair_off[q + 1];
    for (int64_t i = p0 + tid; i < p1; i += TN_THREADS) {
      const int a = p.pair_idx[i];
      const int k = sm[a];
      uint32_t c = 0;
      if (k >= 0) {
        c = slot_count(p, hist, L, q, s, k);
      } else {
        const int d = p.a2dense[a];
        if (d >= 0) c = src_row_count_frag(p, q, s, d);
      }
      if (c >= mt) atomicAdd(p.out + i, (unsigned long long)c);
    }
  }
}

// ids= re-count from the histograms phase 1 kept (hist_in): one 256-thread
// block per (query, shard) gathers the slot counts of that query's ids.
__global__ __launch_bounds__(256) void topn_gather_kernel(TopNLaunch p) {
  const uint32_t unit = tn_xcd_remap(blockIdx.x, gridDim.x);
  const int q = int(unit % p.Q), s = int(unit / p.Q);
  const HistLayout L(p.K - p.R, p.H32, p.H16);
  const auto h = gp(p.hist_in + unit_hist_base(p, q, s, L.words));
  const uint32_t mt = uint32_t(max(1, p.min_threshold[q]));
  const int32_t* sm = p.slotmap + int64_t(s) * p.A;
  const int64_t p0 = p.pair_off[q], p1 = p.pair_off[q + 1];
  for (int64_t i = p0 + threadIdx.x; i < p1; i += blockDim.x) {
    const int a = p.pair_idx[i];
    const int k = sm[a];
    uint32_t c = 0;
    if (k >= 0 && (k < p.R || !p.tail_built || p.tail_built[unit_index(p, q, s)])) {
      c = slot_count(p, h, L, q, s, k);
    } else if (k >= 0) {
      // phase 1 skipped this unit's tail histogram: count the row exactly
      c = src_row_count_frag(p, q, s, int(p.cache_dense[int64_t(s) * p.K + k]));
    } else {
      const int d = p.a2dense[a];
      if (d >= 0) c = src_row_count_frag(p, q, s, d);
    }
    if (c >= mt) atomicAdd(p.out + i, (unsigned long long)c);
  }
}


// ---------------------------------------------------------------- hot ranks
// The first R cache ranks of every shard hold most of the cached rows' bits
// (Zipf: ranks < 2048 carry ~90% of them), and every query of a batch needs
// their src counts before its heap walk can stop.  Counting them through the
// column-major slot histogram costs |src| x (bits per column) scattered
// slot-run reads PER QUERY; here they are counted row-major ONCE for the
// whole batch (Q <= 16):
//   one 1024-thread workgroup per shard; for each container key j
//     1. an LDS table of 65536 u16 query masks (128 KB): bit q of entry x
//        is set when src(q) has column j*2^16 + x;
//     2. each wave streams its hot rows' key-j containers (coalesced reads
//        of the arena payload) and sums, per query, the mask bits of the
//        row's values: 16 per-lane counters, reduced over the wave by a
//        17-shuffle transpose (lane l ends with query (l >> 2) & 15);
//     3. the wave adds them into hot_cnt[s][q][k] (it owns row k for every j,
//        so the read-modify-write needs no atomics).
// hot_meta[s][j][k] is the row's key-j container (meta index relative to the
// shard, -1 = none), built once with the index.
constexpr int HOT_THREADS = 1024;
constexpr int HOT_TAB_WORDS = 32768;
// Lane-owned (small) containers: at most SMALLN values (PILOSA_TOPN_SMALL_N
// = 63, 255, 1023 or 4096 = every array).  Counts are carry-save planes that a
// lane turns into per-query totals every 240 values, so bigger rows lane-owned
// skip the wave-cooperative path's per-row transpose-reduce.
constexpr int HOT_SMALL_N = 255;
// largest array of the quarter-wave (mid) path: a lane of a 16-lane quarter
// then holds <= 128 of a row's values (7 carry-save planes per packed half
// for NQ 16, 8 per query for NQ 32); the default bound is HOT_MID_N
constexpr int HOT_MID_MAX = 2048, HOT_MID_N = 2048;

// Bit-sliced (carry-save) counting.  A "word" is a query mask: for NQ = 16
// the masks of two values packed as lo | hi << 16 (bit q and bit 16 + q both
// count query q), for NQ = 32 one value's u32 mask.  pl[k] holds bit k of 32
// per-bit counters; adding W words is a Harley-Seal tree of carry-save
// adders (3 ops each: xor3, xor, bfi) whose last carry ripples up to plane
// MAXP - 1 (2 ops a plane).  That is ~2.5 ops per value against the 12-14 of
// spreading every mask into byte counters (a nibble times 0x00204081, the
// round-4 kernel: profiles/r05_hotcsa/); the planes are turned into counts
// once per row (hs_counts).
__device__ __forceinline__ void csa(uint32_t& s, uint32_t& c, uint32_t a, uint32_t b) {
  // s + a + b = (s ^ a ^ b) + 2 * maj(s, a, b)
  const uint32_t u = s ^ a;
  c = (u & b) | (~u & s);
  s = u ^ b;
}
template <int K0, int MAXP>
__device__ __forceinline__ void hs_ripple(uint32_t (&pl)[8], uint32_t c) {
#pragma unroll
  for (int k = K0; k < MAXP; k++) {
    const uint32_t t = pl[k] & c;
    pl[k] ^= c;
    c = t;
  }
}
template <int W, int MAXP>
__device__ __forceinline__ void hs_add(uint32_t (&pl)[8], const uint32_t* w) {
  uint32_t a, b, c2a, c2b;
  if constexpr (W == 2) {
    csa(pl[0], a, w[0], w[1]);
    hs_ripple<1, MAXP>(pl, a);
  } else if constexpr (W == 4) {
    csa(pl[0], a, w[0], w[1]);
    csa(pl[0], b, w[2], w[3]);
    csa(pl[1], c2a, a, b);
    hs_ripple<2, MAXP>(pl, c2a);
  } else {
    static_assert(W == 8 || W == 16, "hs_add: W in {2, 4, 8, 16}");
    uint32_t c3a, c3b, c4;
#pragma unroll
    for (int h = 0; h < W / 8; h++) {
      const uint32_t* v = w + 8 * h;
      csa(pl[0], a, v[0], v[1]);
      csa(pl[0], b, v[2], v[3]);
      csa(pl[1], c2a, a, b);
      csa(pl[0], a, v[4], v[5]);
      csa(pl[0], b, v[6], v[7]);
      csa(pl[1], c2b, a, b);
      csa(pl[2], h ? c3b : c3a, c2a, c2b);
    }
    if constexpr (W == 8) {
      hs_ripple<3, MAXP>(pl, c3a);
    } else {
      csa(pl[3], c4, c3a, c3b);
      hs_ripple<4, MAXP>(pl, c4);
    }
  }
}
// Add the counters held in planes pl[0..NP) to acc[NQ] and clear the planes.
// An 8x8 bit transpose inside every byte (3 delta-swap rounds over the 8
// plane words) leaves in byte b of word c the 8-bit count of bit 8b + c; a
// v_dot4 then sums the bytes that belong to one query into acc.
template <int NQ, int NP>
__device__ __forceinline__ void hs_counts(uint32_t (&pl)[8], uint32_t (&acc)[NQ]) {
#pragma unroll
  for (int k = NP; k < 8; k++) pl[k] = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t t = ((pl[k] >> 4) ^ pl[k + 4]) & 0x0f0f0f0fu;
    pl[k + 4] ^= t;
    pl[k] ^= t << 4;
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (k & 2) continue;
    const uint32_t t = ((pl[k] >> 2) ^ pl[k + 2]) & 0x33333333u;
    pl[k + 2] ^= t;
    pl[k] ^= t << 2;
  }
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    const uint32_t t = ((pl[k] >> 1) ^ pl[k + 1]) & 0x55555555u;
    pl[k + 1] ^= t;
    pl[k] ^= t << 1;
  }
  // word c: bytes = counts of bits c, 8 + c, 16 + c, 24 + c
#pragma unroll
  for (int c = 0; c < 8; c++) {
    if (NQ == 16) {
      // bits q and 16 + q are both query q
      acc[c] = __builtin_amdgcn_udot4(pl[c], 0x00010001u, acc[c], false);
      acc[8 + c] = __builtin_amdgcn_udot4(pl[c], 0x01000100u, acc[8 + c], false);
    } else {
#pragma unroll
      for (int b = 0; b < 4; b++) acc[(8 * b + c) % NQ] = __builtin_amdgcn_udot4(pl[c], 1u << (8 * b), acc[(8 * b + c) % NQ], false);
    }
    pl[c] = 0;
  }
}

// NQ = 16: one workgroup per (shard, key j), a u16 query mask per value of
// the key (64K x 2 B).  NQ = 32 (17..32 queries per launch): one workgroup
// per (shard, key, half h) with u32 masks for the key's values
// [h*32768, h*32768 + 32768) -- the same 128 KB of LDS -- so a launch counts
// twice the queries for the same streamed bytes (the two halves' workgroups
// are consecutive, on one XCD: the second read of a container hits L2).
template <int NQ, int SMALLN = HOT_SMALL_N>
__global__ __launch_bounds__(HOT_THREADS, 1) void topn_hot_kernel(TopNLaunch p) {
  extern __shared__ uint32_t tab[];
  __shared__ int grab[2];
  // one workgroup per (shard, key j[, half]); consecutive blocks share a shard (XCD L2)
  const int unit = int(tn_xcd_remap(blockIdx.x, gridDim.x));
  constexpr int HB = NQ == 32 ? 1 : 0;  // half bit
  const int s = unit >> (4 + HB), j = (unit >> HB) & 15;
  const int lo = HB ? (unit & 1) * 32768 : 0;
  constexpr int NLO = HB ? 32768 : 65536;  // values per workgroup
  const int tid = threadIdx.x, lane = tid & 63;
  const int Q = p.Q, R = p.R;
  const int64_t sb = p.v.shard_base[s];
  uint32_t* out = p.hot_cnt + int64_t(s) * Q * R;
  // 1. query-mask table of key j: bitmap srcs as a transpose of their bits
  //    (every table word written once), then array srcs OR'd in with LDS
  //    atomics, one wave per query (wave w takes queries w, w + 16), 16
  //    value loads per lane in flight.  (Spreading every query's values over
  //    the whole workgroup instead measured slower: mix 7.6 vs 6.9 ms,
  //    profiles/r05_hotcsa/.)
  const int wave = tid >> 6;
  // bit q: src q's key-j container is a bitmap (the same mask in every wave)
  uint32_t bmq;
  {
    const int nq = lane < Q ? p.src_counts[(int64_t(lane) * p.S + s) * 16 + j] : 0;
    bmq = uint32_t(__ballot(nq > ARRAY_MAX && nq >= p.tbuild_min));
    if (!__syncthreads_or(tid < Q && nq > 0)) return;  // block-uniform: no src has key j in this shard
  }
  if (tid == 0) grab[0] = grab[1] = 0;
  if (bmq && !(PK_DBG(p) & 1024)) {
    // bitmap srcs: every table word is written once as the transpose of the
    // bitmaps' bits (thread-owned words, 32 loads in flight per query)
    // instead of one LDS atomic per set bit -- a dense src row is 30-50k bits
    // per key, which serialised ~500 atomics per lane.  Array srcs OR in below.
    constexpr int PER = HOT_TAB_WORDS / HOT_THREADS;  // 32 table words per thread
    const int sh = HB ? (tid & 31) : ((2 * tid) & 31);
    uint32_t e[PER];
#pragma unroll
    for (int t = 0; t < PER; t++) e[t] = 0u;
    for (uint32_t m = bmq; m; m &= m - 1) {
      const int q = __builtin_ctz(m);
      const int64_t kk = (int64_t(q) * p.S + s) * 16 + j;
      const auto w32 = reinterpret_cast<const TN_GLOBAL uint32_t*>(gp(p.src_vals + p.src_offs[kk]));
      uint32_t v[PER];
#pragma unroll
      for (int t = 0; t < PER; t++)
        v[t] = HB ? w32[((lo + tid) >> 5) + 32 * t] : w32[(tid >> 4) + 64 * t];
#pragma unroll
      for (int t = 0; t < PER; t++) {
        if (HB) {
          e[t] |= ((v[t] >> sh) & 1u) << q;           // entry x = lo + tid + 1024 t
        } else {
          const uint32_t b2 = (v[t] >> sh) & 3u;      // entries x = 2 (tid + 1024 t) + {0, 1}
          e[t] |= ((b2 & 1u) << q) | ((b2 >> 1) << (16 + q));
        }
      }
    }
#pragma unroll
    for (int t = 0; t < PER; t++) tab[tid + HOT_THREADS * t] = e[t];
  } else {
    uint4* t4 = reinterpret_cast<uint4*>(tab);
    for (int i = tid; i < HOT_TAB_WORDS / 4; i += HOT_THREADS) t4[i] = make_uint4(0, 0, 0, 0);
    bmq = 0;
  }
  __syncthreads();
  for (int q = wave; q < Q; q += HOT_THREADS / 64) {
    const int64_t kk = (int64_t(q) * p.S + s) * 16 + j;
    const int n = p.src_counts[kk];
    if (n <= 0) continue;
    const auto vals = gp(p.src_vals + p.src_offs[kk]);
    if (n <= ARRAY_MAX) {
      // 16 value loads per lane in flight (a 4096-value array in 4 round trips)
      for (int i0 = 0; i0 < n; i0 += 64 * 16) {
        int xv[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int i = i0 + 64 * u + lane;
          xv[u] = i < n ? int(vals[i]) : -1;
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int x = xv[u];
          if (x < 0) continue;
          if (HB) {
            if (unsigned(x - lo) < unsigned(NLO)) atomicOr(&tab[x - lo], 1u << q);
          } else {
            atomicOr(&tab[x >> 1], 1u << (q + ((x & 1) << 4)));
          }
        }
      }
    } else if (!((bmq >> q) & 1u) && !(PK_DBG(p) & 512)) {
      const auto w = reinterpret_cast<const TN_GLOBAL uint64_t*>(vals);
      for (int i = lane + (lo >> 6); i < (lo + NLO) >> 6; i += 64)
        for (uint64_t bb = w[i]; bb; bb &= bb - 1) {
          const int x = i * 64 + __builtin_ctzll(bb);
          if (HB) atomicOr(&tab[x - lo], 1u << q);
          else atomicOr(&tab[x >> 1], 1u << (q + ((x & 1) << 4)));
        }
    }
  }
  __syncthreads();
  // NQ 16: entry x is the u16 half x of the table (one ds_read_u16, no
  // shift/select); NQ 32: u32 entry x - lo, 0 outside the workgroup's half
  const uint16_t* tab16 = reinterpret_cast<const uint16_t*>(tab);
  auto mask_of = [&](int x) -> uint32_t {
    if (HB) return unsigned(x - lo) < unsigned(NLO) ? tab[x - lo] : 0u;
    return tab16[x];
  };
  const int32_t* hm = p.hot_meta + (int64_t(s) * 16 + j) * R;
  const int B = min(R, p.hot_split[(int64_t(s) * 16 + j) * 2]);
  const int B1 = min(B, p.hot_split[(int64_t(s) * 16 + j) * 2 + 1]);

  // 2. big containers, ranks [0, B1): wave w takes ranks w + 16 i (sizes fall
  //    with rank, so every wave gets a similar mix).  Per group of 64 of its
  //    ranks, lane l loads rank l's container index and meta word (2 vector
  //    loads per 64 rows); then rows stream as 512-value chunks (8 rounds of
  //    64 consecutive values) with the NEXT chunk's loads -- possibly the next
  //    row's first chunk -- in flight while the current one is counted.
  //    Carry-save planes per lane, counted at the row's end, then a
  //    17-shuffle transpose-reduce per row, totals in lanes (l >> 2) & 15.
  for (int gb = wave; gb < ((PK_DBG(p) & 16) ? 0 : B1); gb += 64 * (HOT_THREADS / 64)) {
    const int kl = gb + (HOT_THREADS / 64) * lane;
    const int cl = kl < B1 ? hm[kl] : -1;
    const int64_t ml = cl >= 0 ? p.v.meta[sb + cl] : 0;
    uint64_t live = __ballot(cl >= 0);
    if (!live) continue;
    auto row_meta = [&](int r) -> int64_t {
      const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(ml)), r));
      const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(ml) >> 32)), r));
      return int64_t((uint64_t(hi) << 32) | lo);
    };
    // lane l takes values base + 8l .. +7 with ONE 16-byte load (the payload
    // is 16-byte aligned and padded to 8 values).  16 values per lane per
    // step (two loads, 124 VGPRs) measured 10.7 vs 10.4 ms (profiles/r03_ch16)
    // Branch-free: every lane always loads a valid chunk (its own, or the
    // container's last / the payload's first when it has none) and zeroes
    // it after, so the load is never behind a branch and the compiler can
    // count the loads in flight instead of draining them all (vmcnt(0)).
    // m == 0 (no container to prefetch) reads the payload's first chunk.
    auto load_chunk = [&](int64_t m, int base, uint4& x, int& nv) {
      const uint4* pp4 = reinterpret_cast<const uint4*>(p.v.payload + meta_off16(m) * 8);
      const int i0 = base + 8 * lane;
      const int n = meta_n(m);
      nv = min(max(n - i0, 0), 8);
      x = pp4[min(i0, max(n - 1, 0)) >> 3];
      if (nv <= 0) x = make_uint4(0, 0, 0, 0);
    };
    int r = __builtin_ctzll(live);
    live &= live - 1;
    int64_t m = row_meta(r);
    int base = 0;
    // Three chunk buffers rotate through the unrolled loop below: a load
    // cursor runs two (row, chunk) steps ahead of the count cursor and each
    // step loads into the buffer the step before last consumed.  No buffer is
    // ever copied into another, so the wait before a chunk is counted is for
    // THAT chunk's load only (a rotating copy of in-flight registers made the
    // compiler wait for the newest prefetch before every chunk).
    uint4 b0 = make_uint4(0, 0, 0, 0), b1 = make_uint4(0, 0, 0, 0), b2 = make_uint4(0, 0, 0, 0);
    int v0 = 0, v1 = 0, v2 = 0;
    load_chunk(meta_type(m) == CT_ARRAY ? m : 0, 0, b0, v0);
    int lr = r, lbase = 0;
    int64_t lm = m;
    uint64_t llive = live;
    auto adv = [&]() {
      if (lr < 0) return;
      if (meta_type(lm) == CT_ARRAY && lbase + 512 < meta_n(lm)) {
        lbase += 512;
        return;
      }
      lr = llive ? __builtin_ctzll(llive) : -1;
      llive &= llive - 1;
      lbase = 0;
      lm = lr >= 0 ? row_meta(lr) : 0;
    };
    adv();
    load_chunk(lr >= 0 && meta_type(lm) == CT_ARRAY ? lm : 0, lbase, b1, v1);
    adv();
    uint32_t acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) acc[q] = 0;
    // carry-save planes: an array row gives a lane <= 64 values (6 planes
    // hold 32 per packed half, 7 hold 64); bitmap rows use all 8 (<= 192
    // bits between counts), runs too (<= 240 values)
    constexpr int HW = NQ == 16 ? 4 : 8, COOP_P = NQ == 16 ? 6 : 7;
    uint32_t pl[8];
#pragma unroll
    for (int k = 0; k < 8; k++) pl[k] = 0;
    // one (row, chunk) step: count `cur`, load two steps ahead into `ldb`;
    // false once the wave's last row is done
    auto step = [&](const uint4& cur, const int curv, uint4& ldb, int& ldv) -> bool {
      const int ty = meta_type(m);
      const int n = meta_n(m);
      const bool more = ty == CT_ARRAY && base + 512 < n;
      int rn = r, bn = base + 512;
      int64_t mn = m;
      const bool row_end = !more;
      if (row_end) {
        rn = live ? __builtin_ctzll(live) : -1;
        bn = 0;
        mn = rn >= 0 ? row_meta(rn) : 0;
      }
      load_chunk(lr >= 0 && meta_type(lm) == CT_ARRAY ? lm : 0, lbase, ldb, ldv);
      adv();
      const uint16_t* pp = p.v.payload + meta_off16(m) * 8;
      if (ty == CT_ARRAY && !(PK_DBG(p) & 64)) {
        // an array gives a lane at most 64 values (6-7 carry-save planes).
        // All 8 table reads issue before any is consumed (one LDS wait per
        // chunk); values past the array read entry 0 and count nothing.
        const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
        uint32_t mk[8];
#pragma unroll
        for (int t = 0; t < 8; t++) mk[t] = mask_of(int((wd[t >> 1] >> ((t & 1) << 4)) & 0xffffu));
        // carry-save planes, counted once at the row's end; when every
        // lane holds 8 values (the inner chunks of a big array, which carry
        // most of the values) no per-value pad select
        uint32_t hw[HW];
        if (__ballot(curv < 8) == 0) {
#pragma unroll
          for (int k = 0; k < HW; k++) hw[k] = NQ == 16 ? mk[2 * k] | (mk[2 * k + 1] << 16) : mk[k];
        } else {
#pragma unroll
          for (int k = 0; k < HW; k++)
            hw[k] = NQ == 16 ? (2 * k < curv ? mk[2 * k] : 0u) | (2 * k + 1 < curv ? mk[2 * k + 1] << 16 : 0u)
                             : (k < curv ? mk[k] : 0u);
        }
        hs_add<HW, COOP_P>(pl, hw);
      } else if (ty == CT_BITMAP && !(PK_DBG(p) & 32)) {
        // the lane's words load a quarter at a time (register budget); set
        // bits are taken four at a time (four table reads in flight)
        constexpr int NIT = NLO / 4096;  // 64-word rounds of the workgroup's values
        constexpr int HALF = NIT / 4;     // words loaded per batch
        const uint64_t* w = reinterpret_cast<const uint64_t*>(pp) + (lo >> 6);
        uint64_t wv[HALF];
#pragma unroll
        for (int it = 0; it < NIT; it++) {
          if (it % HALF == 0) {
#pragma unroll
            for (int h = 0; h < HALF; h++) wv[h] = w[lane + 64 * (it + h)];
          }
          const int i = (lo >> 6) + lane + 64 * it;
          for (uint64_t bb = wv[it % HALF]; bb;) {
            uint32_t mk[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const bool v = bb != 0;
              mk[k] = v ? mask_of(i * 64 + __builtin_ctzll(bb)) : 0u;
              bb &= bb - 1;
            }
            if (NQ == 16) {
              const uint32_t hw[2] = {mk[0] | (mk[1] << 16), mk[2] | (mk[3] << 16)};
              hs_add<2, 8>(pl, hw);
            } else {
              hs_add<4, 8>(pl, mk);
            }
          }
          if (it % 3 == 2) hs_counts<NQ, 8>(pl, acc);  // <= 192 bits per lane between counts
        }
      } else if (ty == CT_RUN) {
        const int nr = pp[0];
        const uint16_t* rr = pp + 8;
        int since = 0;
        for (int t = 0; t < nr; t++) {
          const int a0 = max(int(rr[2 * t]), lo), b0_ = min(int(rr[2 * t + 1]), lo + NLO - 1);
          // one value at a time (runs are rare among hot rows): a half-adder
          // ripple; a lane counts its planes every 240 values
          for (int xx = a0 + lane; xx <= b0_; xx += 64) {
            hs_ripple<0, 8>(pl, mask_of(xx));
            if (++since == 240) {
              hs_counts<NQ, 8>(pl, acc);
              since = 0;
            }
          }
        }
      }
      if (row_end) {
        hs_counts<NQ, 8>(pl, acc);
        // transpose-reduce: NQ counters x 64 lanes -> one total per 64/NQ
        // lanes: each level halves the counters a lane holds and sums the
        // exchanged half with lane ^ step (query bit = lane bit)
        uint32_t t16[16], t8[8], t4[4], t2[2];
        if (NQ == 32) {
          const bool h5 = lane & 32;
#pragma unroll
          for (int i = 0; i < 16; i++) {
            const uint32_t mine = h5 ? acc[(16 + i) % NQ] : acc[i], other = h5 ? acc[i] : acc[(16 + i) % NQ];
            t16[i] = mine + uint32_t(__shfl_xor(int(other), 32, 64));
          }
        } else {
#pragma unroll
          for (int i = 0; i < 16; i++) t16[i] = acc[i];
        }
        {
          const int st = NQ == 32 ? 16 : 32;
          const bool hb = lane & st;
#pragma unroll
          for (int i = 0; i < 8; i++) {
            const uint32_t mine = hb ? t16[8 + i] : t16[i], other = hb ? t16[i] : t16[8 + i];
            t8[i] = mine + uint32_t(__shfl_xor(int(other), st, 64));
          }
        }
        {
          const int st = NQ == 32 ? 8 : 16;
          const bool hb = lane & st;
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const uint32_t mine = hb ? t8[4 + i] : t8[i], other = hb ? t8[i] : t8[4 + i];
            t4[i] = mine + uint32_t(__shfl_xor(int(other), st, 64));
          }
        }
        {
          const int st = NQ == 32 ? 4 : 8;
          const bool hb = lane & st;
#pragma unroll
          for (int i = 0; i < 2; i++) {
            const uint32_t mine = hb ? t4[2 + i] : t4[i], other = hb ? t4[i] : t4[2 + i];
            t2[i] = mine + uint32_t(__shfl_xor(int(other), st, 64));
          }
        }
        const int st1 = NQ == 32 ? 2 : 4;
        const bool h1 = lane & st1;
        uint32_t d = (h1 ? t2[1] : t2[0]) + uint32_t(__shfl_xor(int(h1 ? t2[0] : t2[1]), st1, 64));
        if (NQ == 16) d += uint32_t(__shfl_xor(int(d), 2, 64));
        d += uint32_t(__shfl_xor(int(d), 1, 64));
        // the query of this lane's total: bits (lane >> log2(64/NQ)) in the
        // order the levels consumed them
        const int q = NQ == 32 ? (lane >> 1) & 31 : (lane >> 2) & 15;
        const int k = gb + (HOT_THREADS / 64) * r;
        if ((lane & (64 / NQ - 1)) == 0 && q < Q && d) atomicAdd(out + int64_t(q) * R + k, d);
#pragma unroll
        for (int qq = 0; qq < NQ; qq++) acc[qq] = 0;
        if (rn < 0) return false;
        live &= live - 1;
      }
      r = rn;
      base = bn;
      m = mn;
      return true;
    };
    for (;;) {
      if (!step(b0, v0, b2, v2)) break;
      if (!step(b1, v1, b0, v0)) break;
      if (!step(b2, v2, b1, v1)) break;
    }
  }


  // 2b. mid-size arrays (lane-owned bound < n <= PILOSA_TOPN_MID_N), ranks [B1, B):
  //     a 16-lane quarter wave per row, 4 rows per wave (wave w takes the
  //     rank quads B1 + 4 (w + 16 i)).  Lane l of a quarter counts values
  //     8l..8l+7 of every 128-value round (one 16-byte load, the next round's
  //     in flight) into carry-save planes; at the row's end the planes become
  //     counts and a 4-level transpose-reduce over the quarter leaves query l
  //     (NQ 16; 2l and 2l + 1 for NQ 32) in lane l.  The cooperative path
  //     spends a 6-level reduction of every row over the whole wave, which
  //     rows of a few hundred values cannot amortise.
  if (!(PK_DBG(p) & 2048)) {
    constexpr int MW = NQ == 16 ? 4 : 8, MID_P = NQ == 16 ? 7 : 8;
    const int sl = lane & 15;
    // the rank -> container -> meta -> payload chain runs ahead: a quad's
    // first chunk loads with the quad before, its meta word two quads
    // ahead, its container index three ahead
    constexpr int QSTEP = 4 * (HOT_THREADS / 64);
    auto quad_c = [&](int g4) -> int {
      const int kq = g4 + (lane >> 4);
      return kq < B ? hm[kq] : -1;
    };
    int cq = quad_c(B1 + 4 * wave);
    int64_t mq = cq >= 0 ? p.v.meta[sb + cq] : 0;
    int cq1 = quad_c(B1 + 4 * wave + QSTEP);
    int64_t mq1 = cq1 >= 0 ? p.v.meta[sb + cq1] : 0;
    int cq2 = quad_c(B1 + 4 * wave + 2 * QSTEP);
    // a quad's first chunk loads with the quad before it
    auto first_chunk = [&](int c, int64_t m) -> uint4 {
      const int nn = c >= 0 ? meta_n(m) : 0;
      return reinterpret_cast<const uint4*>(p.v.payload + meta_off16(m) * 8)[min(sl, max(nn - 1, 0) >> 3)];
    };
    uint4 px0 = first_chunk(cq, mq);
    // a quad's totals are added after the next quad's first round is counted
    // (see the lane-owned path: atomics ahead of loads delay them)
    uint32_t mpend[NQ / 16];
    int mpk = -1;  // rank of the pending totals' quarter (-1 = none; wave-uniform validity)
    auto mflush = [&]() {
      if (mpk < 0) return;
#pragma unroll
      for (int e = 0; e < NQ / 16; e++) {
        const int q = NQ == 16 ? sl : 2 * sl + e;
        if (q < Q && mpend[e] && !(PK_DBG(p) & 256)) atomicAdd(out + int64_t(q) * R + mpk, mpend[e]);
      }
      mpk = -1;
    };
    for (int g4 = B1 + 4 * wave; g4 < B; g4 += QSTEP) {
      const int k = g4 + (lane >> 4);
      const int64_t m = mq;
      const int n = cq >= 0 ? meta_n(m) : 0;  // arrays only in this rank range
      const uint4* pp = reinterpret_cast<const uint4*>(p.v.payload + meta_off16(m) * 8);
      const int lastc = max(n - 1, 0) >> 3;
      uint4 x0 = px0, x1;
      px0 = first_chunk(cq1, mq1);
      const int64_t mq2 = cq2 >= 0 ? p.v.meta[sb + cq2] : 0;
      cq = cq1;
      mq = mq1;
      cq1 = cq2;
      mq1 = mq2;
      cq2 = quad_c(g4 + 3 * QSTEP);
      uint32_t mpl[8];
#pragma unroll
      for (int t = 0; t < 8; t++) mpl[t] = 0u;
      auto count8 = [&](const uint4& x, const int i0) {
        const int nv = n - i0;  // values of this lane's chunk in the row (<= 0: none)
        const uint32_t wd[4] = {x.x, x.y, x.z, x.w};
        uint32_t mk[8];
#pragma unroll
        for (int t = 0; t < 8; t++) mk[t] = mask_of(int((wd[t >> 1] >> ((t & 1) << 4)) & 0xffffu));
        uint32_t hw[MW];
        if (__ballot(nv < 8) == 0) {
#pragma unroll
          for (int w = 0; w < MW; w++) hw[w] = NQ == 16 ? mk[2 * w] | (mk[2 * w + 1] << 16) : mk[w];
        } else {
#pragma unroll
          for (int w = 0; w < MW; w++)
            hw[w] = NQ == 16 ? (2 * w < nv ? mk[2 * w] : 0u) | (2 * w + 1 < nv ? mk[2 * w + 1] << 16 : 0u)
                             : (w < nv ? mk[w] : 0u);
        }
        hs_add<MW, MID_P>(mpl, hw);
      };
      for (int r = 0;;) {
        if (!__ballot(128 * r < n)) break;
        x1 = pp[min(16 * (r + 1) + sl, lastc)];
        count8(x0, 128 * r + 8 * sl);
        mflush();
        r++;
        if (!__ballot(128 * r < n)) break;
        x0 = pp[min(16 * (r + 1) + sl, lastc)];
        count8(x1, 128 * r + 8 * sl);
        r++;
      }
      uint32_t a[NQ];
#pragma unroll
      for (int q = 0; q < NQ; q++) a[q] = 0u;
      hs_counts<NQ, MID_P>(mpl, a);
      // level st: lanes with bit st keep the upper half of the counters and
      // add their partner's copy of it (the query index takes the lane bit)
#pragma unroll
      for (int st = 8, sz = NQ; st >= 1; st >>= 1, sz >>= 1) {
        const bool hb = lane & st;
#pragma unroll
        for (int i = 0; i < NQ / 2; i++) {
          if (i >= sz / 2) break;
          const uint32_t mine = hb ? a[sz / 2 + i] : a[i], other = hb ? a[i] : a[sz / 2 + i];
          a[i] = mine + uint32_t(__shfl_xor(int(other), st, 64));
        }
      }
      mflush();  // (a quad without values)
#pragma unroll
      for (int e = 0; e < NQ / 16; e++) mpend[e] = a[e];
      mpk = k;
    }
    mflush();
  }


  // 3. small array containers (<= HOT_SMALL_N values), ranks [B, R): waves
  //    grab groups of 64 consecutive ranks, each lane counts its own row
  //    (8 values per 16-byte load), no reduction; atomics are coalesced
  //    (consecutive ranks per query).  A row here has a handful of values, so
  //    the rank -> meta -> payload chain of loads is the cost: groups are
  //    claimed two ahead and the next group's meta word and the one after's
  //    meta index are loaded with the current group's payload (one round trip
  //    per group instead of three).
  if (!(PK_DBG(p) & 8)) {
    auto claim = [&]() -> int {
      int g = 0;
      if (lane == 0) g = atomicAdd(&grab[1], 1);
      return __builtin_amdgcn_readfirstlane(g);
    };
    auto rank_meta = [&](int g) -> int {
      const int kl = B + 64 * g + lane;
      return kl < R ? hm[kl] : -1;
    };
    int g = claim();
    int cl = rank_meta(g);
    int64_t ml = cl >= 0 ? p.v.meta[sb + cl] : 0;
    int gn = claim();
    int cln = rank_meta(gn);
    // a group's counts are added one group later, after the next group's
    // first loads have been consumed: vmcnt counts atomics with loads, so
    // atomics issued just before a group's loads made those loads wait out
    // the atomics' round trip too
    uint32_t pend[NQ];
    int pk = -1;  // rank of the pending counts (wave-uniform: -1 = none)
    auto flush_pend = [&]() {
      if (pk < 0) return;
#pragma unroll
      for (int q = 0; q < NQ; q++)
        if (q < Q && pend[q] && !(PK_DBG(p) & 256)) atomicAdd(out + int64_t(q) * R + pk + lane, pend[q]);
      pk = -1;
    };
    while (B + 64 * g < R) {
      const int kl = B + 64 * g + lane;
      const int nl = cl >= 0 ? meta_n(ml) : 0;
      const auto pp = gp(reinterpret_cast<const uint4*>(p.v.payload + meta_off16(ml) * 8));
      // every lane loads (clamped to its row's last chunk; values past the
      // row are masked when counted), so no load sits behind a branch
      const int lastc = max(nl - 1, 0) >> 3;
      uint4 w0 = pp[0], w1 = pp[min(1, lastc)];
      const int64_t mln = cln >= 0 ? p.v.meta[sb + cln] : 0;
      const int gnn = claim();
      const int clnn = rank_meta(gnn);
      uint32_t lpl[8], lcnt[NQ];
#pragma unroll
      for (int k = 0; k < 8; k++) lpl[k] = 0u;
#pragma unroll
      for (int q = 0; q < NQ; q++) lcnt[q] = 0u;
      int since = 0;
      // 16 values per lane per step; two buffers alternate so the next
      // step's loads are in flight while this one is counted
      auto body = [&](const uint4& x0, const uint4& x1, const int i) {
        if (PK_DBG(p) & 4096) {  // cost isolation: loads only (keep them live)
          lpl[0] ^= x0.x ^ x1.y;
          return;
        }
        const uint32_t wd[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        uint32_t mk[16];
#pragma unroll
        for (int t = 0; t < 16; t++) mk[t] = mask_of(int((wd[t >> 1] >> ((t & 1) << 4)) & 0xffffu));
        // carry-save planes (<= 240 values per lane between counts: 8
        // planes hold them), counted at the row's end
        constexpr int LW = NQ == 16 ? 8 : 16;
        uint32_t hw[LW];
        if (__ballot(i + 16 > nl) == 0) {
#pragma unroll
          for (int k = 0; k < LW; k++) hw[k] = NQ == 16 ? mk[2 * k] | (mk[2 * k + 1] << 16) : mk[k];
        } else {
#pragma unroll
          for (int k = 0; k < LW; k++)
            hw[k] = NQ == 16 ? (i + 2 * k < nl ? mk[2 * k] : 0u) | (i + 2 * k + 1 < nl ? mk[2 * k + 1] << 16 : 0u)
                             : (i + k < nl ? mk[k] : 0u);
        }
        hs_add<LW, 8>(lpl, hw);
        if (SMALLN > 255 && ++since == 15) {  // wave-uniform
          since = 0;
          hs_counts<NQ, 8>(lpl, lcnt);
        }
      };
      uint4 n0, n1;
      for (int i = 0;;) {
        if (!__ballot(i < nl)) break;
        n0 = pp[min((i >> 3) + 2, lastc)];
        n1 = pp[min((i >> 3) + 3, lastc)];
        body(w0, w1, i);
        flush_pend();
        i += 16;
        if (!__ballot(i < nl)) break;
        w0 = pp[min((i >> 3) + 2, lastc)];
        w1 = pp[min((i >> 3) + 3, lastc)];
        body(n0, n1, i);
        i += 16;
      }
      hs_counts<NQ, 8>(lpl, lcnt);
      flush_pend();  // (a group without values)
#pragma unroll
      for (int q = 0; q < NQ; q++) pend[q] = lcnt[q];
      pk = B + 64 * g;
      g = gn;
      cl = cln;
      ml = mln;
      gn = gnn;
      cln = clnn;
    }
    flush_pend();
  }
}

// hot_meta[s][j][k] = meta index (relative to the shard) of the key-j
// container of the row at cache rank k < R, -1 when absent.  Thread per (s, k).
template <int SMALLN>
__global__ __launch_bounds__(256) void topn_hot_meta_kernel(ViewDev v, int S, int K, int R,
                                                            const int32_t* __restrict__ cache_dense,
                                                            int32_t* __restrict__ hot_meta,
                                                            int32_t* __restrict__ hot_split, int midn) {
  const int64_t total = int64_t(S) * R;
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < total;
       e += int64_t(gridDim.x) * blockDim.x) {
    const int s = int(e / R), k = int(e - int64_t(s) * R);
    const int d = cache_dense[int64_t(s) * K + k];
    if (d < 0) continue;
    const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
    const int64_t sb = v.shard_base[s];
    for (uint32_t c = rp[d]; c < rp[d + 1]; c++) {
      const int64_t m = v.meta[sb + c];
      hot_meta[(int64_t(s) * 16 + meta_j(m)) * R + k] = int32_t(c);
      // ranks before the split take the cooperative path (see topn_hot_kernel)
      int32_t* hs = hot_split + (int64_t(s) * 16 + meta_j(m)) * 2;
      if (meta_type(m) != CT_ARRAY || meta_n(m) > SMALLN) atomicMax(hs, k + 1);
      // ranks before hs[1] take the wave-cooperative path; [hs[1], hs[0]) the
      // quarter-wave path of mid-size arrays
      if (meta_type(m) != CT_ARRAY || meta_n(m) > midn) atomicMax(hs + 1, k + 1);
    }
  }
}

// Src containers of plain-row srcs straight from the arena (no copy):
// counts[(q*S + s)*16 + j] = n, offs = the container's u16 payload offset;
// run containers set *has_run (the caller then materialises instead).
__global__ __launch_bounds__(256) void leaf_src_kernel(ViewDev v, const int64_t* __restrict__ rows, int Q, int S,
                                                       int32_t* __restrict__ counts, int64_t* __restrict__ offs,
                                                       int32_t* __restrict__ has_run) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= int64_t(Q) * S) return;
  const int q = int(e / S), s = int(e - int64_t(q) * S);
  const int64_t d = rows[q];
  if (d < 0) return;
  const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
  const int64_t sb = v.shard_base[s];
  for (uint32_t c = rp[d]; c < rp[d + 1]; c++) {
    const int64_t m = v.meta[sb + c];
    const int64_t o = (int64_t(q) * S + s) * 16 + meta_j(m);
    counts[o] = meta_n(m);
    offs[o] = meta_off16(m) * 8;
    if (meta_type(m) == CT_RUN) atomicOr(has_run, 1);
  }
}


// Row cardinality of dense row d in local shard s: the metadata counts of its
// (at most 16) containers, no payload read (fragment.go:459 CountRange).
__device__ __forceinline__ int32_t row_card(const ViewDev& v, int s, int64_t d) {
  if (d < 0 || d >= v.D) return 0;
  const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
  const int64_t sb = v.shard_base[s];
  int32_t n = 0;
  for (uint32_t c = rp[d]; c < rp[d + 1]; c++) n += meta_n(v.meta[sb + c]);
  return n;
}

// Rank-cache entries (shard, dense row) -> row counts (device rank caches of
// cold fragments: the .cache file's ids with the arena's counts).
__global__ __launch_bounds__(256) void row_counts_kernel(ViewDev v, const int32_t* __restrict__ shard_of,
                                                         const int32_t* __restrict__ dense, int64_t N,
                                                         int32_t* __restrict__ out) {
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < N; e += int64_t(gridDim.x) * blockDim.x)
    out[e] = row_card(v, shard_of[e], dense[e]);
}

// ids= re-count without a src row (fragment.top with RowIDs, cache-only):
// out[p] = sum over the local shards of row p's count where it reaches
// threshold[p].  One 256-thread workgroup per id walks the shards; wave64
// shuffle reduction, one store per id.
__global__ __launch_bounds__(256) void row_counts_sum_kernel(ViewDev v, int S, const int32_t* __restrict__ dense,
                                                             const int32_t* __restrict__ threshold, int P,
                                                             unsigned long long* __restrict__ out) {
  __shared__ unsigned long long part[4];
  const int p = blockIdx.x;
  if (p >= P) return;
  const int64_t d = dense[p];
  const int32_t th = threshold[p] > 1 ? threshold[p] : 1;
  unsigned long long acc = 0;
  if (d >= 0)
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      const int32_t n = row_card(v, s, d);
      if (n >= th) acc += unsigned(n);
    }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[p] = part[0] + part[1] + part[2] + part[3];
}

}  // namespace

void launch_leaf_src(const ViewDev& v, const int64_t* rows, int Q, int S, int32_t* counts, int64_t* offs,
                     int32_t* has_run, hipStream_t st) {
  const int64_t total = int64_t(Q) * S;
  if (total <= 0) return;
  hipLaunchKernelGGL(leaf_src_kernel, dim3(unsigned((total + 255) / 256)), dim3(256), 0, st, v, rows, Q, S, counts,
                     offs, has_run);
}

// lane-owned container bound of the hot-rank kernels (63, 255, 1023 or 4096
// = every array), fixed per process: the split the meta kernel records must
// match the counting kernel's
static int hot_small_n() {
  static const int n = [] {
    const char* e = getenv("PILOSA_TOPN_SMALL_N");
    const int v = e ? atoi(e) : 0;
    return v > 1023 ? 4096 : v > 255 ? 1023 : (v > 0 && v < 255) ? 63 : 255;
  }();
  return n;
}

// mid-size arrays (lane-owned bound < n <= this) are counted by 16-lane
// quarter waves, 4 rows per wave (PILOSA_TOPN_MID_N; 0 = none: the
// cooperative path takes them)
static int hot_mid_n() {
  static const int n = [] {
    const char* e = getenv("PILOSA_TOPN_MID_N");
    return e ? std::max(0, std::min(atoi(e), HOT_MID_MAX)) : HOT_MID_N;
  }();
  return n;
}

template <int SMALLN>
static void launch_hot_meta_t(const ViewDev& v, int S, int K, int R, const int32_t* cache_dense, int32_t* hot_meta,
                              int32_t* hot_split, int blocks, hipStream_t st) {
  hipLaunchKernelGGL(topn_hot_meta_kernel<SMALLN>, dim3(blocks), dim3(256), 0, st, v, S, K, R, cache_dense, hot_meta,
                     hot_split, std::max(hot_mid_n(), SMALLN));
}

void launch_topn_hot_meta(const ViewDev& v, int S, int K, int R, const int32_t* cache_dense, int32_t* hot_meta,
                          int32_t* hot_split, hipStream_t st) {
  const int64_t total = int64_t(S) * R;
  if (total <= 0) return;
  const int64_t want = (total + 255) / 256;
  const int blocks = int(want < 65536 ? want : 65536);
  switch (hot_small_n()) {
    case 4096: launch_hot_meta_t<4096>(v, S, K, R, cache_dense, hot_meta, hot_split, blocks, st); break;
    case 63: launch_hot_meta_t<63>(v, S, K, R, cache_dense, hot_meta, hot_split, blocks, st); break;
    case 1023: launch_hot_meta_t<1023>(v, S, K, R, cache_dense, hot_meta, hot_split, blocks, st); break;
    default: launch_hot_meta_t<255>(v, S, K, R, cache_dense, hot_meta, hot_split, blocks, st);
  }
}

template <int NQ, int SMALLN>
static void launch_hot_t(const TopNLaunch& a, hipStream_t st) {
  const int tab = HOT_TAB_WORDS * 4;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(topn_hot_kernel<NQ, SMALLN>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, tab);
  hipLaunchKernelGGL((topn_hot_kernel<NQ, SMALLN>), dim3(unsigned(a.S) * unsigned(NQ)), dim3(HOT_THREADS), tab, st,
                     a);
}

void launch_topn_index(const ViewDev& v, int S, int K, int k0, const int32_t* cache_dense, uint32_t* colcnt,
                       const uint32_t* colptr, const int64_t* entbase, uint16_t* slots, bool fill, hipStream_t st) {
  const int64_t waves = int64_t(S) * (K - k0);
  const int64_t want = (waves + 3) / 4;
  const int blocks = int(want < 256 * 64 ? want : 256 * 64);
  if (blocks <= 0) return;
  if (fill)
    hipLaunchKernelGGL(topn_index_kernel<true>, dim3(blocks), dim3(256), 0, st, v, S, K, k0, cache_dense, colcnt,
                       colptr, entbase, slots);
  else
    hipLaunchKernelGGL(topn_index_kernel<false>, dim3(blocks), dim3(256), 0, st, v, S, K, k0, cache_dense, colcnt,
                       colptr, entbase, slots);
}

int topn_lds_bytes(int K, int H32, int H16) {
  return (H32 + ((H16 - H32 + 1) >> 1) + ((K - H16 + 3) >> 2)) * 4;
}

void launch_topn_src(const TopNLaunch& a0, int mode, hipStream_t st) {
  TopNLaunch a = a0;
#ifdef PK_KBENCH
  static const int dbg = [] {
    const char* e = getenv("PILOSA_TOPN_DBG");
    return e ? atoi(e) : 0;
  }();
  a.dbg = dbg;
#else
  a.dbg = 0;
#endif
  // bitmap srcs at least this dense take the transposed table build, the
  // rest one LDS atomic per set bit
  static const int tbuild_min = [] {
    const char* e = getenv("PILOSA_TOPN_TBUILD_MIN");
    return e ? atoi(e) : 4097;
  }();
  a.tbuild_min = tbuild_min;
  const int lds = topn_lds_bytes(a.K - a.R, a.H32, a.H16);
  const int64_t units = int64_t(a.Q) * a.S;
  if (units <= 0) return;
  if (mode == 4) {
    // hot-rank count matrix (before mode 1/2 of the same batch)
    if (a.R <= 0) return;
    // the split must match the meta kernel's bound (hot_small_n)
    const bool q32 = a.Q > 16;
    switch (hot_small_n()) {
      case 4096: q32 ? launch_hot_t<32, 4096>(a, st) : launch_hot_t<16, 4096>(a, st); break;
      case 63: q32 ? launch_hot_t<32, 63>(a, st) : launch_hot_t<16, 63>(a, st); break;
      case 1023: q32 ? launch_hot_t<32, 1023>(a, st) : launch_hot_t<16, 1023>(a, st); break;
      default: q32 ? launch_hot_t<32, 255>(a, st) : launch_hot_t<16, 255>(a, st);
    }
  } else if (mode == 3) {
    hipLaunchKernelGGL(topn_gather_kernel, dim3(unsigned(units)), dim3(256), 0, st, a);
  } else if (mode == 1) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(topn_src_kernel<1>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(topn_src_kernel<1>, dim3(unsigned(units)), dim3(TN_THREADS), lds, st, a);
  } else {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(topn_src_kernel<2>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(topn_src_kernel<2>, dim3(unsigned(units)), dim3(TN_THREADS), lds, st, a);
  }
}


void launch_row_counts(const ViewDev& v, const int32_t* shard_of, const int32_t* dense, int64_t N, int32_t* out,
                       hipStream_t st) {
  if (N <= 0) return;
  const int64_t want = (N + 255) / 256;
  const int blocks = int(want < 256 * 64 ? want : 256 * 64);
  hipLaunchKernelGGL(row_counts_kernel, dim3(blocks), dim3(256), 0, st, v, shard_of, dense, N, out);
}

void launch_row_counts_sum(const ViewDev& v, int S, const int32_t* dense, const int32_t* threshold, int P,
                           unsigned long long* out, hipStream_t st) {
  if (P <= 0) return;
  hipLaunchKernelGGL(row_counts_sum_kernel, dim3(unsigned(P)), dim3(256), 0, st, v, S, dense, threshold, P, out);
}

// ---------------------------------------------------------------------------
// Cache-only TopN batch (TopN(field, n) without a src row): the reference
// runs, per shard, fragment.top's fill phase over the rank cache
// (fragment.go:1436-1530 with src == nil) and then re-counts the union of
// the candidates with ids= (executor.go executeTopN phase 2).  On the device
// the whole batch is three kernels over the rank caches already resident in
// HBM: a per-query membership bitmap over the candidate rows, one total per
// (distinct threshold, candidate) from the memoised [candidate x shard]
// count matrix, and one workgroup per query that compacts its members into
// LDS, bitonic-sorts the composite key (count desc, row asc) and writes the
// first n.  No data-dependent host round trips between them.
namespace {

constexpr int TC_CAP = 8192;   // members per query sorted in LDS (64 KB of keys)
// threads of the per-query select: 16 waves on the query's CU -- the bitonic
// stages loop over up to TC_CAP keys, 4x fewer iterations per thread than 256
// (the select was ~half of a wide cache-only batch's GPU time)
constexpr int TC_THREADS = 1024;

__global__ __launch_bounds__(256) void topn_cache_counts_kernel(ViewDev v, int S, const int32_t* __restrict__ u,
                                                                int64_t N, int32_t* __restrict__ cm) {
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < N; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t j = e / S;
    cm[e] = row_card(v, int(e - j * S), u[j]);
  }
}

// member[q, inv[s*nmax + k]] = 1 for the first lim[q] ranks of shard s whose
// cached count reaches mt[q]
// nmax = the memoised prefix (inv's row stride); nlim <= nmax = the ranks this
// batch can take (its largest n): a batch reuses a longer prefix's memo
// without walking the ranks beyond its own n
__global__ __launch_bounds__(256) void topn_cache_member_kernel(const int32_t* __restrict__ cnt, int K, int S, int nmax,
                                                                const int32_t* __restrict__ inv,
                                                                const int32_t* __restrict__ prm, int Q, int U,
                                                                uint8_t* __restrict__ member, int nlim) {
  const int q = blockIdx.y;
  const int L = min(prm[q], nlim);
  const int32_t m = prm[Q + q];
  const int64_t N = int64_t(S) * nlim;
  uint8_t* mq = member + int64_t(q) * U;
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < N; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t s = e / nlim;
    const int k = int(e - s * nlim);
    if (k < L && cnt[s * K + k] >= m) mq[inv[s * nmax + k]] = 1;
  }
}

// The same membership with one thread per (shard, rank) for every query of
// the batch (Q <= 256): the rank's count and candidate index are read once
// instead of once per query (the per-query grid re-read them Q times).
// ``mark``: the byte a member gets (1 after a clear; a cycling epoch when the
// buffer is reused uncleared, CacheTopN); block b of nb blocks.
__device__ __forceinline__ void cache_member_q_body(const int32_t* __restrict__ cnt, int K, int S, int nmax,
                                                    const int32_t* __restrict__ inv, const int32_t* __restrict__ prm,
                                                    int Q, int U, uint8_t* __restrict__ member, int nlim, uint8_t mark,
                                                    int b, int nb) {
  __shared__ int32_t lim[256], thr[256];
  for (int q = threadIdx.x; q < Q; q += blockDim.x) {
    lim[q] = min(prm[q], nlim);
    thr[q] = prm[Q + q];
  }
  __syncthreads();
  const int64_t N = int64_t(S) * nlim;
  for (int64_t e = int64_t(b) * blockDim.x + threadIdx.x; e < N; e += int64_t(nb) * blockDim.x) {
    const int64_t s = e / nlim;
    const int k = int(e - s * nlim);
    const int32_t c = cnt[s * K + k];
    if (c <= 0) continue;
    const int j = inv[s * nmax + k];
    for (int q = 0; q < Q; q++)
      if (k < lim[q] && c >= thr[q]) member[int64_t(q) * U + j] = mark;
  }
}

__global__ __launch_bounds__(256) void topn_cache_member_q_kernel(const int32_t* __restrict__ cnt, int K, int S,
                                                                  int nmax, const int32_t* __restrict__ inv,
                                                                  const int32_t* __restrict__ prm, int Q, int U,
                                                                  uint8_t* __restrict__ member, int nlim) {
  cache_member_q_body(cnt, K, S, nmax, inv, prm, Q, U, member, nlim, 1, int(blockIdx.x), int(gridDim.x));
}

// tot[t*U + j] = sum over shards of cm[j*S + s] where it reaches th[t]; one
// wave per (threshold, candidate), coalesced over the shard axis.  TT = long
// long on one rank; int on a mesh rank, whose partial totals travel in the
// batch's one int32 all-reduce (parallel/mesh.py OP_TOPN)
template <class TT>
__global__ __launch_bounds__(256) void topn_cache_totals_kernel(const int32_t* __restrict__ cm, int S, int U,
                                                                const int32_t* __restrict__ th, int T,
                                                                TT* __restrict__ tot) {
  const int w = int(blockIdx.x) * 4 + int(threadIdx.x >> 6);
  const int lane = int(threadIdx.x & 63);
  if (w >= T * U) return;
  const int t = w / U;
  const int j = w - t * U;
  const int32_t m = th[t];
  const int32_t* row = cm + int64_t(j) * S;
  int acc = 0;
  for (int s = lane; s < S; s += 64) {
    const int32_t n = row[s];
    acc += n >= m ? n : 0;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) tot[w] = TT(acc);
}

// The same totals for up to 16 thresholds in ONE pass over the count matrix:
// one wave per candidate, every count compared against all thresholds in
// registers (the per-threshold kernel re-read the [U x S] matrix T times:
// ~1.2 GB for 16 distinct thresholds over a 20k-candidate prefix).
template <class TT>
__device__ __forceinline__ void cache_totals16_body(const int32_t* __restrict__ cm, int S, int U,
                                                    const int32_t* __restrict__ th, int T, TT* __restrict__ tot,
                                                    int b);

template <class TT>
__global__ __launch_bounds__(256) void topn_cache_totals16_kernel(const int32_t* __restrict__ cm, int S, int U,
                                                                  const int32_t* __restrict__ th, int T,
                                                                  TT* __restrict__ tot) {
  cache_totals16_body<TT>(cm, S, U, th, T, tot, int(blockIdx.x));
}

template <class TT>
__device__ __forceinline__ void cache_totals16_body(const int32_t* __restrict__ cm, int S, int U,
                                                    const int32_t* __restrict__ th, int T, TT* __restrict__ tot,
                                                    int b) {
  const int j = b * 4 + int(threadIdx.x >> 6);
  const int lane = int(threadIdx.x & 63);
  if (j >= U) return;
  int32_t thr[16];
#pragma unroll
  for (int t = 0; t < 16; t++) thr[t] = t < T ? th[t] : 0x7fffffff;
  int acc[16];
#pragma unroll
  for (int t = 0; t < 16; t++) acc[t] = 0;
  const int32_t* row = cm + int64_t(j) * S;
  for (int s = lane; s < S; s += 64) {
    const int32_t n = row[s];
#pragma unroll
    for (int t = 0; t < 16; t++) acc[t] += n >= thr[t] ? n : 0;
  }
#pragma unroll
  for (int t = 0; t < 16; t++) {
    if (t >= T) break;
    int v = acc[t];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) tot[int64_t(t) * U + j] = TT(v);
  }
}

// Membership and the 16-threshold totals in ONE launch (Q <= 256, T <= 16):
// blocks [0, nbm) run the membership, the rest the totals -- independent
// work, one launch latency less per cache-only request.
template <class TT>
__global__ __launch_bounds__(256) void topn_cache_member_totals16_kernel(
    const int32_t* __restrict__ cnt, int K, int S, int nmax, const int32_t* __restrict__ inv,
    const int32_t* __restrict__ prm, int Q, int U, uint8_t* __restrict__ member, int nlim, uint8_t mark, int nbm,
    const int32_t* __restrict__ cm, int T, TT* __restrict__ tot) {
  if (int(blockIdx.x) < nbm)
    cache_member_q_body(cnt, K, S, nmax, inv, prm, Q, U, member, nlim, mark, int(blockIdx.x), nbm);
  else
    cache_totals16_body<TT>(cm, S, U, prm + 4 * Q, T, tot, int(blockIdx.x) - nbm);
}

template <class TT>
__global__ __launch_bounds__(TC_THREADS) void topn_cache_select_kernel(const uint8_t* __restrict__ member,
                                                                const TT* __restrict__ tot,
                                                                const int32_t* __restrict__ u,
                                                                const int32_t* __restrict__ prm, int Q, int U, int KK,
                                                                long long* __restrict__ out,
                                                                const int32_t* __restrict__ flags, int mark) {
  __shared__ long long keys[TC_CAP];
  __shared__ int nmem;
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  if (flags != nullptr && (flags[0] | flags[1])) {
    // a mesh batch some rank could not take part in (all-reduced flag words:
    // [stale candidate space, declined]): no answer, the front end re-plans
    if (tid == 0) out[int64_t(q) * (KK + 1)] = flags[1] ? -4 : -3;
    return;
  }
  if (tid == 0) nmem = 0;
  __syncthreads();
  const uint8_t* mq = member + int64_t(q) * U;
  const TT* tq = tot + int64_t(prm[2 * Q + q]) * U;
  // compaction with one LDS atomic per wave (ballot + prefix popcount), not
  // one per member: every member of a wave used to serialise on nmem
  const int lane = tid & 63;
  for (int j0 = 0; j0 < U; j0 += TC_THREADS) {   // block-uniform trip count
    const int j = j0 + tid;
    bool keep = false;
    long long key = 0;
    // a member: byte == mark (an epoch-marked reused buffer), or nonzero
    // (mark 0: a cleared buffer, or the mesh's all-reduced byte sums)
    if (j < U && (mark ? mq[j] == mark : mq[j] != 0)) {
      const int32_t d = u[j];
      const long long sc = (long long)tq[j];
      if (d >= 0 && sc > 0) {
        keep = true;
        key = (sc << 32) | (0xFFFFFFFFll - d);
      }
    }
    const uint64_t m = __ballot(keep);
    int base = 0;
    if (lane == 0 && m) base = atomicAdd(&nmem, __popcll(m));
    base = __shfl(base, 0, 64);
    if (keep) {
      const int p = base + __popcll(m & ((uint64_t(1) << lane) - 1));
      if (p < TC_CAP) keys[p] = key;
    }
  }
  __syncthreads();
  const int M = nmem;
  long long* o = out + int64_t(q) * (KK + 1);
  if (M > TC_CAP) {   // uniform over the workgroup: the host redoes this batch
    if (tid == 0) o[0] = -2;
    return;
  }
  int P = 1;
  while (P < M) P <<= 1;
  for (int i = M + tid; i < P; i += TC_THREADS) keys[i] = -1;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1)
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      for (int i = tid; i < P; i += TC_THREADS) {
        const int ixj = i ^ jj;
        if (ixj > i) {
          const long long a = keys[i], b = keys[ixj];
          if (((i & k) == 0) ? (a < b) : (a > b)) {
            keys[i] = b;
            keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  const int lim = min(min(M, prm[3 * Q + q]), KK);
  if (tid == 0) o[0] = lim;
  for (int i = tid; i < lim; i += TC_THREADS) o[1 + i] = keys[i];
}

}  // namespace

void launch_topn_cache_counts(const ViewDev& v, int S, const int32_t* u, int U, int32_t* cm, hipStream_t st) {
  const int64_t N = int64_t(U) * S;
  if (N <= 0) return;
  const int64_t want = (N + 255) / 256;
  const int blocks = int(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(topn_cache_counts_kernel, dim3(blocks), dim3(256), 0, st, v, S, u, N, cm);
}

void launch_topn_cache_batch(const int32_t* cnt, int K, int S, int nmax, const int32_t* inv, const int32_t* u,
                             const int32_t* cm, const int32_t* prm, int Q, int T, int U, int KK, uint8_t* member,
                             long long* tot, long long* out, hipStream_t st, int nlim, int mark) {
  if (Q <= 0 || U <= 0) return;
  if (nlim <= 0 || nlim > nmax) nlim = nmax;
  // mark 0: the membership bytes are cleared here and members get 1; mark
  // 1..255: the caller's buffer holds earlier batches' (smaller) marks and
  // is cleared only when the epoch wraps to 1 -- no clear per batch
  if (mark <= 1) (void)hipMemsetAsync(member, 0, size_t(Q) * size_t(U), st);
  const uint8_t mk = uint8_t(mark <= 0 ? 1 : mark);
  const int64_t N = int64_t(S) * nlim;
  const int64_t want = N > 0 ? (N + 255) / 256 : 0;
  if (Q <= 256 && T <= 16) {
    // membership and totals in one launch
    const int nbm = int(want < 8192 ? want : 8192);
    const int nbt = (U + 3) / 4;
    hipLaunchKernelGGL(topn_cache_member_totals16_kernel<long long>, dim3(unsigned(nbm + nbt)), dim3(256), 0, st, cnt,
                       K, S, nmax, inv, prm, Q, U, member, nlim, mk, nbm, cm, T, tot);
  } else {
    if (N > 0) {
      const int bx = int(want < 1024 ? want : 1024);
      if (Q <= 256)
        hipLaunchKernelGGL(topn_cache_member_q_kernel, dim3(unsigned(want < 8192 ? want : 8192)), dim3(256), 0, st,
                           cnt, K, S, nmax, inv, prm, Q, U, member, nlim);
      else
        hipLaunchKernelGGL(topn_cache_member_kernel, dim3(bx, Q), dim3(256), 0, st, cnt, K, S, nmax, inv, prm, Q, U,
                           member, nlim);
    }
    const int64_t waves = int64_t(T) * U;
    if (T <= 16)
      hipLaunchKernelGGL(topn_cache_totals16_kernel<long long>, dim3(unsigned((U + 3) / 4)), dim3(256), 0, st, cm, S,
                         U, prm + 4 * Q, T, tot);
    else
      hipLaunchKernelGGL(topn_cache_totals_kernel<long long>, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, st, cm,
                         S, U, prm + 4 * Q, T, tot);
  }
  // the separate member kernels write 1 (a cleared buffer): test nonzero
  const int smark = (Q <= 256 && T <= 16) ? int(mk) : 0;
  hipLaunchKernelGGL(topn_cache_select_kernel<long long>, dim3(Q), dim3(TC_THREADS), 0, st, member, tot, u, prm, Q, U,
                     KK, out, (const int32_t*)nullptr, smark);
}

// A mesh rank's share of a cache-only batch over the NODE candidate space:
// membership bytes and int32 partial totals, side by side in the buffer the
// ranks all-reduce (member as bytes: a sum over < 256 ranks cannot carry into
// the next byte), then the two flag words [stale, declined] this rank votes
// with -- the readiness vote rides in the data all-reduce, so a batch is ONE
// collective with no host read before it.  The whole buffer is cleared here.
// The select runs after the all-reduce, on the front end.
void launch_topn_cache_partial(const int32_t* cnt, int K, int S, int nmax, int nlim, const int32_t* inv,
                               const int32_t* cm, const int32_t* prm, int Q, int T, int U, uint8_t* member,
                               int32_t* tot, int32_t* flags, int stale, int declined, hipStream_t st) {
  const int64_t mw = (int64_t(Q) * U + 3) / 4;
  (void)hipMemsetAsync(member, 0, size_t(mw + int64_t(T) * U + 2) * 4, st);
  if (stale) (void)hipMemsetD32Async(flags, stale, 1, st);
  if (declined) (void)hipMemsetD32Async(flags + 1, declined, 1, st);
  if (Q <= 0 || U <= 0 || stale || declined || cnt == nullptr) return;
  if (nlim <= 0 || nlim > nmax) nlim = nmax;
  const int64_t N = int64_t(S) * nlim;
  if (Q <= 256 && T <= 16 && S > 0) {   // membership + totals in one launch
    const int64_t want = N > 0 ? (N + 255) / 256 : 0;
    const int nbm = int(want < 8192 ? want : 8192);
    hipLaunchKernelGGL(topn_cache_member_totals16_kernel<int>, dim3(unsigned(nbm + (U + 3) / 4)), dim3(256), 0, st,
                       cnt, K, S, nmax, inv, prm, Q, U, member, nlim, uint8_t(1), nbm, cm, T, tot);
    return;
  }
  if (N > 0) {
    const int64_t want = (N + 255) / 256;
    if (Q <= 256)
      hipLaunchKernelGGL(topn_cache_member_q_kernel, dim3(unsigned(want < 8192 ? want : 8192)), dim3(256), 0, st, cnt,
                         K, S, nmax, inv, prm, Q, U, member, nlim);
    else
      hipLaunchKernelGGL(topn_cache_member_kernel, dim3(int(want < 1024 ? want : 1024), Q), dim3(256), 0, st, cnt, K,
                         S, nmax, inv, prm, Q, U, member, nlim);
  }
  const int64_t waves = int64_t(T) * U;
  if (S > 0 && T <= 16)
    hipLaunchKernelGGL(topn_cache_totals16_kernel<int>, dim3(unsigned((U + 3) / 4)), dim3(256), 0, st, cm, S, U,
                       prm + 4 * Q, T, tot);
  else if (S > 0)
    hipLaunchKernelGGL(topn_cache_totals_kernel<int>, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, st, cm, S, U,
                       prm + 4 * Q, T, tot);
}

void launch_topn_cache_select32(const uint8_t* member, const int32_t* tot, const int32_t* ids, const int32_t* prm,
                                int Q, int U, int KK, long long* out, const int32_t* flags, hipStream_t st) {
  if (Q <= 0 || U <= 0) return;
  hipLaunchKernelGGL(topn_cache_select_kernel<int>, dim3(Q), dim3(TC_THREADS), 0, st, member, tot, ids, prm, Q, U, KK,
                     out, flags, 0);
}

}  // namespace pk
