// Count(Intersect(Row(a), Row(b))) for a batch of queries, organised around
// container keys instead of (query, shard) work items.
//
// Why a separate path: in the headline workload ~70 % of container pairs are
// array&array (~1.1k values each), 26 % array&bitmap.  The generic kernel
// walks the <=16 keys of one (query, shard) sequentially, so every container
// costs two dependent global round trips (meta -> payload) and a wave never
// has more than one container in flight; it also streams each row once per
// query, although in a Zipf batch every hot row is read by many queries.
//
// Here the work is split in two launches:
//   K1 pair_build   one thread per (shard, query): resolves both rows' CSR
//                   ranges, derives the key-presence masks (no meta loads for
//                   full rows) and writes the matching container index pair
//                   for every key j to pairs[(s*16 + j) * Q + q].
//   K2 and2_pairs   one wave per (shard, key, chunk of CQ queries).  The
//                   batch is sorted on the host by (hot row, other row), so
//                   consecutive queries in a chunk usually share row a: the
//                   wave stages a's container ONCE into its 8 KiB LDS bitmap
//                   and only streams b's container per query.  Waves of one
//                   (shard, key) unit are consecutive and XCD-remapped onto
//                   one XCD, so the unit's containers (~1.3 MB) live in that
//                   XCD's 4 MB L2 while all its chunks run.
// Per-(unit, query) counts go to an int32 partial buffer that torch reduces
// (deterministic, no contended atomics).
//
// Reference hot loops replaced: roaring/roaring.go:3078-3215 intersectionCount*
// and executor.go:1230-1290 (executeCount over executeIntersect).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace pk {
namespace {

constexpr uint32_t NONE = 0xffffffffu;
constexpr int PAIR_WAVES = 4;
#ifndef PAIR_SMALL
#define PAIR_SMALL 1
#endif

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Wave-wide sum through DPP row ops (ockl), not __shfl_xor: the latter is six
// dependent ds_bpermute round trips through the LDS pipe per call.
extern "C" __device__ int __ockl_wfred_add_i32(int);
__device__ __forceinline__ int wave_sum(int v) { return __ockl_wfred_add_i32(v); }

__device__ __forceinline__ uint32_t xcd_remap_blocks(uint32_t bid, uint32_t nblk) {
  const uint32_t nx = 8;
  const uint32_t xcd = bid % nx, loc = bid / nx;
  const uint32_t q = nblk / nx, r = nblk % nx;
  const uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + loc;
}

// Payload/meta pointers live in ViewDev as generic pointers; casting them to
// the global address space gives global_load (vmcnt only) instead of
// flat_load, which also counts against lgkmcnt and so serialises with LDS.
// (The host compilation pass parses these bodies too, without address spaces.)
#if defined(__HIP_DEVICE_COMPILE__)
#define PK_GLOBAL __attribute__((address_space(1)))
#else
#define PK_GLOBAL
#endif
template <class T>
__device__ __forceinline__ const PK_GLOBAL T* gp(const T* p) {
  return (const PK_GLOBAL T*)(p);
}

__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Key-presence mask and absolute first-container index of dense row d in shard s.
__device__ __forceinline__ uint32_t row_keys(const ViewDev& v, int s, int64_t d, int64_t& lo) {
  lo = 0;
  if (d < 0) return 0;
  const auto rp = gp(v.rowptr + int64_t(s) * (v.D + 1));
  const uint32_t r0 = rp[d], r1 = rp[d + 1];
  lo = gp(v.shard_base)[s] + r0;
  const int n = int(r1 - r0);
  if (n == 16) return 0xffffu;
  uint32_t pres = 0;
#pragma unroll
  for (int k = 0; k < 16; k++)
    if (k < n) pres |= 1u << meta_j(gp(v.meta)[lo + k]);
  return pres;
}

__global__ __launch_bounds__(256) void pair_build_kernel(const QueryProg* __restrict__ progs, int Q,
                                                         const ViewDev* __restrict__ views, int S,
                                                         uint2* __restrict__ pairs) {
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= int64_t(Q) * S) return;
  const int s = int(t / Q), q = int(t % Q);
  const QueryProg& qp = progs[q];
  int64_t loa, lob;
  const uint32_t pa = row_keys(views[qp.leaf_view[0]], s, qp.leaf_row[0], loa);
  const uint32_t pb = row_keys(views[qp.leaf_view[1]], s, qp.leaf_row[1], lob);
  const uint32_t both = pa & pb;
  uint2* dst = pairs + int64_t(s) * 16 * Q + q;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    uint2 e = make_uint2(NONE, NONE);
    if ((both >> j) & 1) {
      const uint32_t below = (1u << j) - 1;
      e.x = uint32_t(loa + __popc(pa & below));
      e.y = uint32_t(lob + __popc(pb & below));
    }
    dst[int64_t(j) * Q] = e;
  }
}

// ---- container primitives (wave-cooperative, lb = wave-private 1024-word LDS bitmap)

__device__ __forceinline__ const uint16_t* payload_of(const ViewDev& v, int64_t m) {
  return v.payload + meta_off16(m) * 8;
}

__device__ __forceinline__ void lds_clear(uint64_t* lb) {
  ulong2* l2 = reinterpret_cast<ulong2*>(lb);
  const int lane = lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) l2[i * 64 + lane] = make_ulong2(0, 0);
}

// Stage a container of any type into lb as a bitmap.
__device__ __forceinline__ void stage(uint64_t* lb, const uint16_t* p, int64_t m) {
  const int lane = lane_id();
  const int type = meta_type(m);
  ulong2* l2 = reinterpret_cast<ulong2*>(lb);
  if (type == CT_BITMAP) {
    const auto g = gp(reinterpret_cast<const ulong2*>(p));
    const ulong2 t0 = g[lane], t1 = g[64 + lane], t2 = g[128 + lane], t3 = g[192 + lane];
    const ulong2 t4 = g[256 + lane], t5 = g[320 + lane], t6 = g[384 + lane], t7 = g[448 + lane];
    l2[lane] = t0; l2[64 + lane] = t1; l2[128 + lane] = t2; l2[192 + lane] = t3;
    l2[256 + lane] = t4; l2[320 + lane] = t5; l2[384 + lane] = t6; l2[448 + lane] = t7;
    lds_wait();
    return;
  }
  lds_clear(lb);
  lds_wait();
  if (type == CT_ARRAY) {
    const int n = meta_n(m);
    const auto p4 = gp(reinterpret_cast<const uint4*>(p));
    const int n8 = (n + 7) >> 3;
    for (int e8 = lane; e8 < n8; e8 += 64) {
      const uint4 v4 = p4[e8];
      const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
      const int rem = n - e8 * 8;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t v = (w[k >> 1] >> ((k & 1) * 16)) & 0xffff;
        atomicOr(reinterpret_cast<uint32_t*>(lb) + (v >> 5), k < rem ? (1u << (v & 31)) : 0u);
      }
    }
  } else {
    const auto pr = gp(p);
    const int nr = pr[0];
    for (int r = lane; r < nr; r += 64) {
      const uint32_t s = pr[8 + 2 * r], e = uint32_t(pr[9 + 2 * r]) + 1;
      const uint32_t ws = s >> 6, we = (e - 1) >> 6;
      if (ws == we) {
        const uint64_t mk = (e - s == 64) ? ~0ull : (((1ull << (e - s)) - 1) << (s & 63));
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[ws]), mk);
      } else {
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[ws]), ~0ull << (s & 63));
        for (uint32_t w = ws + 1; w < we; w++) lb[w] = ~0ull;
        const uint32_t hb = e & 63;
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[we]), hb ? ((1ull << hb) - 1) : ~0ull);
      }
    }
  }
  lds_wait();
}

// Count array values present in a 1024-word bitmap (LDS or global).
// DBG (cost isolation, scripts/kbench.py variants 14/15; results wrong):
// bit 2 = synthetic array values instead of loading B, bit 3 = load B but
// skip the LDS probes.
template <int DBG = 0, class BM>
__device__ __forceinline__ int probe(BM bm, const uint16_t* arr, int n) {
  const int lane = lane_id();
  const auto p4 = gp(reinterpret_cast<const uint4*>(arr));
  const int n8 = (n + 7) >> 3;
  int c = 0;
  for (int e8 = lane; e8 < n8; e8 += 64) {
    uint4 v4;
    if (DBG & 4) {
      const uint32_t h = uint32_t(e8) * 2654435761u;
      v4 = make_uint4(h, h * 7u + 1u, h * 13u + 5u, h * 31u + 9u);
    } else {
      v4 = p4[e8];
    }
    const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
    const int rem = n - e8 * 8;
    if (DBG & 8) {
      c += int((w[0] ^ w[1] ^ w[2] ^ w[3]) & 1) + (rem > 0);
      continue;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (w[k >> 1] >> ((k & 1) * 16)) & 0xffff;
      c += k < rem ? int((bm[v >> 5] >> (v & 31)) & 1) : 0;
    }
  }
  return c;
}

// probe() with the next chunk's load issued before the current chunk's LDS
// probes (2-deep register pipeline inside one array; the later load is issued
// after the one being waited for, so the in-order vmcnt wait does not cover it).
template <class BM>
__device__ __forceinline__ int probe_pipe(BM bm, const uint16_t* arr, int n) {
  const int lane = lane_id();
  const auto p4 = gp(reinterpret_cast<const uint4*>(arr));
  const int n8 = (n + 7) >> 3;
  const int iters = (n8 + 63) >> 6;
  int c = 0;
  int e8 = lane;
  uint4 cur = make_uint4(0, 0, 0, 0);
  if (e8 < n8) cur = p4[e8];
#pragma unroll 2
  for (int it = 0; it < iters; it++) {
    const int ne8 = e8 + 64;
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (it + 1 < iters && ne8 < n8) nxt = p4[ne8];
    const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
    const int rem = n - e8 * 8;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (w[k >> 1] >> ((k & 1) * 16)) & 0xffff;
      c += k < rem ? int((bm[v >> 5] >> (v & 31)) & 1) : 0;
    }
    cur = nxt;
    e8 = ne8;
  }
  return c;
}

// probe_pipe() that also carries the first chunk across pairs: `pre` holds
// this array's first chunk when have_pre (loaded during the previous pair's
// last iteration), and the last iteration here loads the next pair's first
// chunk (next != nullptr) into `pre` -- issued after every load of this
// array, so the in-order vmcnt waits of this pair never cover it.
template <class BM>
__device__ __forceinline__ int probe_pipe_x(BM bm, const uint16_t* arr, int n, uint4& pre, bool have_pre,
                                            const uint16_t* next, int next_n) {
  const int lane = lane_id();
  const auto p4 = gp(reinterpret_cast<const uint4*>(arr));
  const int n8 = (n + 7) >> 3;
  const int iters = (n8 + 63) >> 6;
  const int nn8 = (next_n + 7) >> 3;
  int c = 0;
  int e8 = lane;
  uint4 cur = pre;
  if (!have_pre) {
    cur = make_uint4(0, 0, 0, 0);
    if (e8 < n8) cur = p4[e8];
  }
#pragma unroll 2
  for (int it = 0; it < iters; it++) {
    const int ne8 = e8 + 64;
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (it + 1 < iters) {
      if (ne8 < n8) nxt = p4[ne8];
    } else if (next != nullptr && lane < nn8) {
      nxt = gp(reinterpret_cast<const uint4*>(next))[lane];
    }
    const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
    const int rem = n - e8 * 8;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (w[k >> 1] >> ((k & 1) * 16)) & 0xffff;
      c += k < rem ? int((bm[v >> 5] >> (v & 31)) & 1) : 0;
    }
    cur = nxt;
    e8 = ne8;
  }
  pre = cur;
  return c;
}

template <class PX>
__device__ __forceinline__ int and_bitmaps(PX a, const uint64_t* y) {
  const int lane = lane_id();
  const auto b = gp(reinterpret_cast<const ulong2*>(y));
  ulong2 u[8], v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) u[i] = a[i * 64 + lane];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = b[i * 64 + lane];
  int c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) c += __popcll(u[i].x & v[i].x) + __popcll(u[i].y & v[i].y);
  return c;
}

// Count bits of a run container inside the LDS bitmap.
__device__ __forceinline__ int runs_in_lds(const uint64_t* lb, const uint16_t* p) {
  const int lane = lane_id();
  const auto pr = gp(p);
  const int nr = pr[0];
  int c = 0;
  for (int r = lane; r < nr; r += 64) {
    const uint32_t s = pr[8 + 2 * r], e = uint32_t(pr[9 + 2 * r]) + 1;
    const uint32_t ws = s >> 6, we = (e - 1) >> 6;
    for (uint32_t w = ws; w <= we; w++) {
      uint64_t mk = ~0ull;
      if (w == ws) mk &= ~0ull << (s & 63);
      if (w == we && (e & 63)) mk &= (1ull << (e & 63)) - 1;
      c += __popcll(lb[w] & mk);
    }
  }
  return c;
}

// |B ∩ staged| where staged lives in lb.  Arrays use the pipelined probe
// (34.7 -> 33.2 ms per 4096-query batch, profiles/r01_and2/kbench_b4096_pipe.log);
// the cost-isolation builds (DBG 4 / 8) use the plain loop they modify.
// Small arrays (n <= SMALL_ARRAY_N, the Zipf tail rows): one value per lane
// and iteration.  probe_pipe() gives each lane 8 values of one 16-byte chunk,
// so a 20-value array would run 8 LDS probe instructions on 3 lanes; here it
// is one 2-byte load and one probe per lane, all loads issued before the
// probes.  Per 4096-query batch: 31.7 ms without, 29.8 (n <= 128),
// 29.5 (256), 29.55 (192, with the one-off gather; 256: 29.40), 30.6 (512)
// (profiles/r01_small_probe/kbench_*.log).
#ifndef SMALL_ARRAY_N
#define SMALL_ARRAY_N 256
#endif
constexpr int SMALL_ITERS = SMALL_ARRAY_N / 64;
template <class BM>
__device__ __forceinline__ int probe_small(BM bm, const uint16_t* arr, int n) {
  const int lane = lane_id();
  const auto p = gp(arr);
  uint32_t v[SMALL_ITERS];
#pragma unroll
  for (int k = 0; k < SMALL_ITERS; k++) v[k] = lane + 64 * k < n ? p[lane + 64 * k] : 0u;
  int c = 0;
#pragma unroll
  for (int k = 0; k < SMALL_ITERS; k++) c += lane + 64 * k < n ? int((bm[v[k] >> 5] >> (v[k] & 31)) & 1) : 0;
  return c;
}

template <int DBG = 0>
__device__ __forceinline__ int count_vs_lds(const uint64_t* lb, const uint16_t* p, int64_t m) {
  const int type = meta_type(m);
  if (type == CT_BITMAP) return and_bitmaps(reinterpret_cast<const ulong2*>(lb), reinterpret_cast<const uint64_t*>(p));
  if (type == CT_ARRAY) {
    if (DBG & 12) return probe<DBG>(reinterpret_cast<const uint32_t*>(lb), p, meta_n(m));
    if (PAIR_SMALL && meta_n(m) <= SMALL_ARRAY_N)
      return probe_small(reinterpret_cast<const uint32_t*>(lb), p, meta_n(m));
    return probe_pipe(reinterpret_cast<const uint32_t*>(lb), p, meta_n(m));
  }
  return runs_in_lds(lb, p);
}

// Cross-pair prefetch of the next B array's first chunk: measured slower
// (37.0 vs 32.0 ms per 4096-query batch, profiles/r01_and2/kbench_b4096_xpf*.log),
// kept selectable.
constexpr bool PAIR_XPF = false;

// B payload of pair i + 1 when it is an array (the only case probed by
// probe_pipe_x); wave-uniform.
__device__ __forceinline__ uint64_t rl_u64(uint64_t v, int i) {
  return (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(v >> 32), i))) << 32) |
         uint32_t(__builtin_amdgcn_readlane(int(v), i));
}

__device__ __forceinline__ void next_b_array(int i, int nq, uint32_t ea, int64_t mb, uint64_t pbl,
                                             const uint16_t*& nB, int& nBn) {
  if (i + 1 >= nq || __builtin_amdgcn_readlane(ea, i + 1) == NONE) return;
  const int64_t m1 = int64_t(rl_u64(uint64_t(mb), i + 1));
  if (meta_type(m1) != CT_ARRAY) return;
  nB = reinterpret_cast<const uint16_t*>(rl_u64(pbl, i + 1));
  nBn = meta_n(m1);
}

// count_vs_lds() for DBG == 0 with the cross-pair first-chunk prefetch;
// have_pre is updated to whether `pre` now holds the next array's chunk.
__device__ __forceinline__ int count_vs_lds_x(const uint64_t* lb, const uint16_t* p, int64_t m, uint4& pre,
                                              bool& have_pre, const uint16_t* next, int next_n) {
  const int type = meta_type(m);
  if (type == CT_ARRAY) {
    const int c = probe_pipe_x(reinterpret_cast<const uint32_t*>(lb), p, meta_n(m), pre, have_pre, next, next_n);
    have_pre = next != nullptr;
    return c;
  }
  have_pre = false;
  if (type == CT_BITMAP) return and_bitmaps(reinterpret_cast<const ulong2*>(lb), reinterpret_cast<const uint64_t*>(p));
  return runs_in_lds(lb, p);
}

// DBG (profiling builds only): bit 0 = never stage (probe the stale LDS
// bitmap), bit 1 = skip counting; results are wrong, timings isolate costs.
template <int CQ, int DBG = 0>
__global__ __launch_bounds__(64 * PAIR_WAVES) void and2_pairs_kernel(const QueryProg* __restrict__ progs, int Q,
                                                                    const ViewDev* __restrict__ views, int S,
                                                                    const uint2* __restrict__ pairs,
                                                                    int32_t* __restrict__ partial) {
  __shared__ uint64_t lbs[PAIR_WAVES][1024];
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t gw = int64_t(xcd_remap_blocks(blockIdx.x, gridDim.x)) * PAIR_WAVES + wave;
  const int nch = (Q + CQ - 1) / CQ;
  const int64_t u = gw / nch;
  if (u >= int64_t(S) * 16) return;
  const int q0 = int(gw % nch) * CQ;
  uint64_t* lb = lbs[wave];

  // lane i < CQ prefetches query q0+i's pair, views and both metas
  uint32_t ea = NONE, eb = NONE;
  int vai = 0, vbi = 0;
  int64_t ma = 0, mb = 0;
  uint64_t pal = 0, pbl = 0;  // per-lane payload addresses: no scalar loads in the pair loop
  if (lane < CQ && q0 + lane < Q) {
    const uint2 e = pairs[u * Q + q0 + lane];
    ea = e.x;
    eb = e.y;
    if (ea != NONE) {
      vai = progs[q0 + lane].leaf_view[0];
      vbi = progs[q0 + lane].leaf_view[1];
      ma = gp(views[vai].meta)[ea];
      mb = gp(views[vbi].meta)[eb];
      pal = reinterpret_cast<uint64_t>(payload_of(views[vai], ma));
      pbl = reinterpret_cast<uint64_t>(payload_of(views[vbi], mb));
    }
  }
  int mine = 0;
  uint32_t cached = NONE;
  int cached_v = -1;
  const int nq = min(CQ, Q - q0);
  uint4 pre = make_uint4(0, 0, 0, 0);  // first chunk of this pair's B array (cross-pair prefetch)
  bool have_pre = false;
  for (int i = 0; i < nq; i++) {
    const uint32_t a = __builtin_amdgcn_readlane(ea, i);
    if (a == NONE) {
      have_pre = false;
      continue;
    }
    const int va = __builtin_amdgcn_readlane(vai, i);
    const int vb = __builtin_amdgcn_readlane(vbi, i);
    const int64_t mA = int64_t((uint64_t(uint32_t(__builtin_amdgcn_readlane(int(ma >> 32), i))) << 32) |
                               uint32_t(__builtin_amdgcn_readlane(int(ma), i)));
    const int64_t mB = int64_t((uint64_t(uint32_t(__builtin_amdgcn_readlane(int(mb >> 32), i))) << 32) |
                               uint32_t(__builtin_amdgcn_readlane(int(mb), i)));
    const uint16_t* pA = reinterpret_cast<const uint16_t*>(rl_u64(pal, i));
    const uint16_t* pB = reinterpret_cast<const uint16_t*>(rl_u64(pbl, i));
    const int tA = meta_type(mA), tB = meta_type(mB);
    int c;
    if (DBG & 3) {
      c = 0;
      if (!(DBG & 1) && !(a == cached && va == cached_v)) {
        lds_wait();
        stage(lb, pA, mA);
        cached = a;
        cached_v = va;
      }
      if (!(DBG & 2)) c = count_vs_lds(lb, pB, mB);
    } else if (a == cached && va == cached_v) {
      if (DBG || !PAIR_XPF) {
        c = count_vs_lds<DBG>(lb, pB, mB);
      } else {
        const uint16_t* nB = nullptr;
        int nBn = 0;
        next_b_array(i, nq, ea, mb, pbl, nB, nBn);
        c = count_vs_lds_x(lb, pB, mB, pre, have_pre, nB, nBn);
      }
    } else {
      const bool next_same = i + 1 < nq && __builtin_amdgcn_readlane(ea, i + 1) == a &&
                             __builtin_amdgcn_readlane(vai, i + 1) == va;
      if (!next_same && tA == CT_BITMAP && tB == CT_BITMAP) {
        // one-off bitmap pair: two coalesced 8 KiB streams, no LDS
        c = and_bitmaps(gp(reinterpret_cast<const ulong2*>(pA)), reinterpret_cast<const uint64_t*>(pB));
        have_pre = false;
      } else if (!next_same && tA == CT_ARRAY && tB == CT_BITMAP && PAIR_SMALL && meta_n(mA) <= SMALL_ARRAY_N) {
        // one-off small array & bitmap: gather the array's bits straight from
        // the global bitmap instead of copying it into LDS (29.47 -> 29.40 ms);
        // doing the same when A is the staged, reused row is slower (30.1 ms,
        // profiles/r01_small_probe/kbench_gather2.log)
        c = probe_small(gp(reinterpret_cast<const uint32_t*>(pB)), pA, meta_n(mA));
        have_pre = false;
      } else if (!next_same && tA == CT_ARRAY && tB == CT_BITMAP) {
        // one-off array & bitmap: copy the bitmap into LDS (64 coalesced lines)
        // and probe the array there; probing the bitmap in global memory
        // instead costs one cache-line request per value (measured 3x slower)
        lds_wait();
        stage(lb, pB, mB);
        cached = NONE;
        cached_v = -1;
        c = count_vs_lds(lb, pA, mA);
        have_pre = false;
      } else {
        lds_wait();  // previous readers of lb are done before it is rewritten
        stage(lb, pA, mA);
        cached = a;
        cached_v = va;
        if (DBG || !PAIR_XPF) {
          c = count_vs_lds<DBG>(lb, pB, mB);
        } else {
          const uint16_t* nB = nullptr;
          int nBn = 0;
          next_b_array(i, nq, ea, mb, pbl, nB, nBn);
          c = count_vs_lds_x(lb, pB, mB, pre, have_pre, nB, nBn);
        }
      }
    }
    c = wave_sum(c);
    if (lane == i) mine = c;
  }
  if (lane < nq) partial[u * Q + q0 + lane] = mine;
}


// ---- v2: register-resident operands, software-pipelined over the chunk.
//
// v1 is latency-bound (PMC: SQ_WAIT_ANY ~63 % of wave cycles, ~1 VMEM load in
// flight per wave): every pair waited for A's payload, then for B's.  v2
// loads any container payload as exactly 8 lane-strided 16 B chunks (bitmap:
// the whole 8 KiB; array: n <= 4096 values = <= 512 chunks, index clamped so
// nothing is read past the container), issues query i+1's B while query i is
// staged and counted, and issues A before B so one vmcnt wait covers A while
// B(i+1) stays in flight.  Bitmap&bitmap pairs never touch LDS.

struct R8 {
  uint4 r[8];
};

__device__ __forceinline__ int chunks_of(int64_t m) {
  const int t = meta_type(m);
  return t == CT_BITMAP ? 512 : (t == CT_ARRAY ? (meta_n(m) + 7) >> 3 : 1);
}

__device__ __forceinline__ void issue8(const uint16_t* p, int64_t m, R8& x) {
  const int lane = lane_id();
  const auto g = gp(reinterpret_cast<const uint4*>(p));
  const int nc = chunks_of(m);
#pragma unroll
  for (int k = 0; k < 8; k++)
    if (k * 64 < nc) x.r[k] = g[min(k * 64 + lane, nc - 1)];  // wave-uniform skip of absent chunks
}

// scatter an array held in registers into the (cleared) LDS bitmap.
// Per-element bounds use rem = n - 8*chunk (one VGPR per chunk) rather than
// 64 distinct "8*chunk+e < n" compares, which LICM hoisted into 64 live VGPRs;
// masked elements OR in 0 instead of branching around the atomic.
__device__ __forceinline__ void scatter_regs(uint64_t* lb, int n, const R8& x) {
  const int lane = lane_id();
  uint32_t* l32 = reinterpret_cast<uint32_t*>(lb);
  const int n8 = (n + 7) >> 3;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (k * 64 >= n8) break;  // wave-uniform
    const int rem = n - (k * 64 + lane) * 8;
    const uint32_t w[4] = {x.r[k].x, x.r[k].y, x.r[k].z, x.r[k].w};
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const uint32_t v = (w[e >> 1] >> ((e & 1) * 16)) & 0xffff;
      atomicOr(l32 + (v >> 5), e < rem ? (1u << (v & 31)) : 0u);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ void copy_regs(uint64_t* lb, const R8& x) {
  const int lane = lane_id();
  uint4* l4 = reinterpret_cast<uint4*>(lb);
#pragma unroll
  for (int k = 0; k < 8; k++) l4[k * 64 + lane] = x.r[k];
}

__device__ __forceinline__ int probe_regs(const uint64_t* lb, int n, const R8& x) {
  const int lane = lane_id();
  const uint32_t* l32 = reinterpret_cast<const uint32_t*>(lb);
  const int n8 = (n + 7) >> 3;
  int c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (k * 64 >= n8) break;  // wave-uniform
    const int rem = n - (k * 64 + lane) * 8;
    const uint32_t w[4] = {x.r[k].x, x.r[k].y, x.r[k].z, x.r[k].w};
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const uint32_t v = (w[e >> 1] >> ((e & 1) * 16)) & 0xffff;
      c += e < rem ? int((l32[v >> 5] >> (v & 31)) & 1) : 0;
    }
    // keep at most one chunk of LDS reads in flight (VGPR pressure)
    __builtin_amdgcn_sched_barrier(0);
  }
  return c;
}

__device__ __forceinline__ int and_regs_lds(const uint64_t* lb, const R8& x) {
  const int lane = lane_id();
  const uint4* l4 = reinterpret_cast<const uint4*>(lb);
  int c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint4 y = l4[k * 64 + lane];
    c += __popc(y.x & x.r[k].x) + __popc(y.y & x.r[k].y) + __popc(y.z & x.r[k].z) + __popc(y.w & x.r[k].w);
  }
  return c;
}

__device__ __forceinline__ int and_regs(const R8& a, const R8& b) {
  int c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++)
    c += __popc(a.r[k].x & b.r[k].x) + __popc(a.r[k].y & b.r[k].y) + __popc(a.r[k].z & b.r[k].z) +
         __popc(a.r[k].w & b.r[k].w);
  return c;
}

// |B ∩ staged-in-LDS| with B in registers (runs read from memory)
__device__ __forceinline__ int count_b(const uint64_t* lb, const uint16_t* pB, int64_t mB, const R8& b) {
  const int t = meta_type(mB);
  if (t == CT_BITMAP) return and_regs_lds(lb, b);
  if (t == CT_ARRAY) return probe_regs(lb, meta_n(mB), b);
  return runs_in_lds(lb, pB);
}

__device__ __forceinline__ int64_t rl64(int64_t v, int i) {
  return int64_t((uint64_t(uint32_t(__builtin_amdgcn_readlane(int(v >> 32), i))) << 32) |
                 uint32_t(__builtin_amdgcn_readlane(int(v), i)));
}

template <int CQ>
__global__ __launch_bounds__(64 * PAIR_WAVES, 3) void and2_pairs_v2_kernel(const QueryProg* __restrict__ progs, int Q,
                                                                       const ViewDev* __restrict__ views, int S,
                                                                       const uint2* __restrict__ pairs,
                                                                       int32_t* __restrict__ partial) {
  __shared__ uint64_t lbs[PAIR_WAVES][1024];
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t gw = int64_t(xcd_remap_blocks(blockIdx.x, gridDim.x)) * PAIR_WAVES + wave;
  const int nch = (Q + CQ - 1) / CQ;
  const int64_t u = gw / nch;
  if (u >= int64_t(S) * 16) return;
  const int q0 = int(gw % nch) * CQ;
  uint64_t* lb = lbs[wave];

  uint32_t ea = NONE;
  int vai = 0, vbi = 0;
  int64_t ma = 0, mb = 0;
  if (lane < CQ && q0 + lane < Q) {
    const uint2 e = pairs[u * Q + q0 + lane];
    if (e.x != NONE) {
      ea = e.x;
      vai = progs[q0 + lane].leaf_view[0];
      vbi = progs[q0 + lane].leaf_view[1];
      ma = gp(views[vai].meta)[e.x];
      mb = gp(views[vbi].meta)[e.y];
    }
  }
  const int nq = min(CQ, Q - q0);
  int mine = 0;
  uint32_t cached = NONE;
  int cached_v = -1;
  R8 ra, rb, rn;
  // prologue: B of the first valid query
  int i = 0;
  while (i < nq && __builtin_amdgcn_readlane(ea, i) == NONE) i++;
  if (i < nq) {
    const int64_t m = rl64(mb, i);
    issue8(payload_of(views[__builtin_amdgcn_readlane(vbi, i)], m), m, rb);
  }
  while (i < nq) {
    const uint32_t a = __builtin_amdgcn_readlane(ea, i);
    const int va = __builtin_amdgcn_readlane(vai, i);
    const int64_t mA = rl64(ma, i), mB = rl64(mb, i);
    const uint16_t* pA = payload_of(views[va], mA);
    const uint16_t* pB = payload_of(views[__builtin_amdgcn_readlane(vbi, i)], mB);
    const int tA = meta_type(mA), tB = meta_type(mB);
    // next valid query
    int j = i + 1;
    while (j < nq && __builtin_amdgcn_readlane(ea, j) == NONE) j++;
    const bool hit = a == cached && va == cached_v;
    if (!hit) issue8(pA, mA, ra);  // A first: its wait leaves B(j) in flight
    if (j < nq) {
      const int64_t m = rl64(mb, j);
      issue8(payload_of(views[__builtin_amdgcn_readlane(vbi, j)], m), m, rn);
    }
    const bool next_same = j < nq && __builtin_amdgcn_readlane(ea, j) == a && __builtin_amdgcn_readlane(vai, j) == va;
    // one code site per primitive (inlining each per branch tripled VGPRs)
    const bool bb = tA == CT_BITMAP && tB == CT_BITMAP;
    if (!hit) {
      if (tA == CT_RUN || tB == CT_RUN) {
        lds_wait();
        stage(lb, pA, mA);
      } else if (tA == CT_BITMAP) {
        if (!bb || next_same) copy_regs(lb, ra);
      } else {
        lds_clear(lb);
        scatter_regs(lb, meta_n(mA), ra);
      }
      if (!bb || next_same) {
        cached = a;
        cached_v = va;
      }
    }
    int c;
    if (!hit && bb) c = and_regs(ra, rb);
    else c = count_b(lb, pB, mB, rb);
    c = wave_sum(c);
    if (lane == i) mine = c;
    rb = rn;
    i = j;
  }
  if (lane < nq) partial[u * Q + q0 + lane] = mine;
}

}  // namespace

void launch_and2_pairs(const QueryProg* progs, int Q, const ViewDev* views, int S, uint2* pairs, int32_t* partial,
                       int cq, int variant, hipStream_t st) {
  const int64_t items = int64_t(Q) * S;
  if (items == 0) return;
  hipLaunchKernelGGL(pair_build_kernel, dim3(unsigned((items + 255) / 256)), dim3(256), 0, st, progs, Q, views, S,
                     pairs);
  const int64_t units = int64_t(S) * 16;
#define PK_LAUNCH(KERNEL, CQV)                                                                                \
  {                                                                                                           \
    const int64_t waves = units * ((Q + CQV - 1) / CQV);                                                      \
    hipLaunchKernelGGL(KERNEL<CQV>, dim3(unsigned((waves + PAIR_WAVES - 1) / PAIR_WAVES)),                    \
                       dim3(64 * PAIR_WAVES), 0, st, progs, Q, views, S, pairs, partial);                     \
  }
  // variant 1 (default): stage-on-demand kernel; variant 2: register-pipelined
  // kernel (fewer waits, but 168 VGPRs -> 3 waves/SIMD; slower on the Zipf
  // benchmark, kept for batches of dense rows).  cq <= 0 picks by batch size:
  // bigger chunks amortise more leaf-0 stagings (measured: 32 for Q <= 2048,
  // 64 above).
  if (cq <= 0) cq = Q <= 2048 ? 32 : 64;
  if (variant == 14 || variant == 15) {  // cost isolation: no B loads (14) / no LDS probes (15)
    const int64_t waves = units * ((Q + 63) / 64);
    const dim3 g(unsigned((waves + PAIR_WAVES - 1) / PAIR_WAVES)), b(64 * PAIR_WAVES);
    if (variant == 14) hipLaunchKernelGGL((and2_pairs_kernel<64, 4>), g, b, 0, st, progs, Q, views, S, pairs, partial);
    else hipLaunchKernelGGL((and2_pairs_kernel<64, 8>), g, b, 0, st, progs, Q, views, S, pairs, partial);
    return;
  }
  if (variant >= 11 && variant <= 13) {  // cost-isolation builds (scripts/kbench.py --cq2 / variant)
    const int64_t waves = units * ((Q + 31) / 32);
    const dim3 g(unsigned((waves + PAIR_WAVES - 1) / PAIR_WAVES)), b(64 * PAIR_WAVES);
    if (variant == 11) hipLaunchKernelGGL((and2_pairs_kernel<32, 1>), g, b, 0, st, progs, Q, views, S, pairs, partial);
    else if (variant == 12) hipLaunchKernelGGL((and2_pairs_kernel<32, 2>), g, b, 0, st, progs, Q, views, S, pairs, partial);
    else hipLaunchKernelGGL((and2_pairs_kernel<32, 3>), g, b, 0, st, progs, Q, views, S, pairs, partial);
    return;
  }
  if (variant == 2) {
    switch (cq) {
      case 4: PK_LAUNCH(and2_pairs_v2_kernel, 4) break;
      case 8: PK_LAUNCH(and2_pairs_v2_kernel, 8) break;
      case 16: PK_LAUNCH(and2_pairs_v2_kernel, 16) break;
      case 32: PK_LAUNCH(and2_pairs_v2_kernel, 32) break;
      default: PK_LAUNCH(and2_pairs_v2_kernel, 64) break;
    }
  } else {
    switch (cq) {
      case 4: PK_LAUNCH(and2_pairs_kernel, 4) break;
      case 8: PK_LAUNCH(and2_pairs_kernel, 8) break;
      case 16: PK_LAUNCH(and2_pairs_kernel, 16) break;
      case 32: PK_LAUNCH(and2_pairs_kernel, 32) break;
      default: PK_LAUNCH(and2_pairs_kernel, 64) break;
    }
  }
#undef PK_LAUNCH
}

}  // namespace pk
