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
// Variants (launch_and2_pairs `variant`): 1 = the round-1 kernel (4 waves per
// workgroup), 4/5 = the same with 1/2 waves per workgroup, 6 (default) = one
// wave per workgroup + next-pair B prefetch, 2/3 = register-pipelined
// experiments.  Per 4096-query batch on the 954-shard index
// (profiles/r02_pairs/): round 1 29.4 ms; branch-free 8-probe chunks 21.7 ms
// (variant 1); 1 wave per workgroup 18.1 ms (4); + B-head prefetch 16.9 ms (6).
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
  const uint32_t r0 = rp[d];
  lo = gp(v.shard_base)[s] + r0;
  // the view's mask table: one 2-byte load instead of the row's metas
  if (v.keymask) return gp(v.keymask)[int64_t(s) * v.D + d];
  const uint32_t r1 = rp[d + 1];
  const int n = int(r1 - r0);
  if (n == 16) return 0xffffu;
  uint32_t pres = 0;
#pragma unroll
  for (int k = 0; k < 16; k++)
    if (k < n) pres |= 1u << meta_j(gp(v.meta)[lo + k]);
  return pres;
}

// keymask[s][d] = row_keys() of every (shard, dense row): built once per view
// generation (DeviceView.ensure_keymask), it turns pair_build's up-to-16
// scattered meta loads per row into one 2-byte load (1.4 ms of a 4096-query
// Count(Intersect) batch on the headline index was pair_build).
__global__ __launch_bounds__(256) void keymask_build_kernel(ViewDev v, int S, uint16_t* __restrict__ out) {
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= int64_t(S) * v.D) return;
  const int s = int(t / v.D);
  const int64_t d = t - int64_t(s) * v.D;
  v.keymask = nullptr;
  int64_t lo;
  out[t] = uint16_t(row_keys(v, s, d, lo));
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

// Cost-isolation probe (profiling builds only, scripts/kbench.py variants
// 14/15; results wrong): DBG bit 2 = synthetic array values instead of
// loading B, bit 3 = load B but skip the LDS probes.  Same shape as
// probe_pipe() otherwise.
template <int DBG, class BM>
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
    if (DBG & 8) {
      c += int((v4.x ^ v4.y ^ v4.z ^ v4.w) & 1);
      continue;
    }
    const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      x[2 * k] = bm[(w[k] & 0xffffu) >> 5];
      x[2 * k + 1] = bm[w[k] >> 21];
    }
#pragma unroll
    for (int k = 0; k < 4; k++)
      c += int(__builtin_amdgcn_ubfe(x[2 * k], w[k], 1u)) + int(__builtin_amdgcn_ubfe(x[2 * k + 1], w[k] >> 16, 1u));
  }
  return c;
}

// Probe the 8 values packed in one 16-byte chunk against a 1024-word bitmap.
// Branch-free: all 8 word reads are issued before any is consumed (one
// lgkmcnt wait per chunk instead of one per value; a per-value `k < rem ?`
// select compiled to exec-masked branches with an lgkmcnt(0) wait inside each
// and serialised every LDS round trip).  Pad values are 0 and are probed too;
// the caller subtracts their hits once per array (pad_hits()).  The bit is
// extracted with v_bfe_u32, whose offset operand only uses bits 4:0, so the
// value itself is the offset (no `& 31`).
template <class BM>
__device__ __forceinline__ int probe8(BM bm, const uint4 v4) {
  const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    x[2 * k] = bm[(w[k] & 0xffffu) >> 5];
    x[2 * k + 1] = bm[w[k] >> 21];
  }
  int c = 0;
#pragma unroll
  for (int k = 0; k < 4; k++)
    c += int(__builtin_amdgcn_ubfe(x[2 * k], w[k], 1u)) + int(__builtin_amdgcn_ubfe(x[2 * k + 1], w[k] >> 16, 1u));
  return c;
}

// Hits of `slots - n` zero-valued pad probes: bit 0 of the bitmap times the
// number of probed slots that were not array values (counted on lane 0 only,
// so the wave sum subtracts it once).
template <class BM>
__device__ __forceinline__ int pad_hits(BM bm, int slots, int n) {
  return lane_id() == 0 ? int(bm[0] & 1u) * (slots - n) : 0;
}

// probe() with the next chunk's load issued before the current chunk's LDS
// probes (2-deep register pipeline inside one array).  Lanes past the array
// hold zero chunks; every lane probes 8 slots per iteration.
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
    if (ne8 < n8) nxt = p4[ne8];
    c += probe8(bm, cur);
    cur = nxt;
    e8 = ne8;
  }
  return c - pad_hits(bm, iters * 512, n);
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
static_assert(SMALL_ARRAY_N % 64 == 0 && SMALL_ARRAY_N > 0, "SMALL_ARRAY_N must be a positive multiple of 64");
constexpr int SMALL_ITERS = SMALL_ARRAY_N / 64;
template <class BM>
__device__ __forceinline__ int probe_small(BM bm, const uint16_t* arr, int n) {
  const int lane = lane_id();
  const auto p = gp(arr);
  if (n <= 64) {  // one value per lane, one probe (wave-uniform branch)
    const uint32_t v = lane < n ? uint32_t(p[lane]) : 0u;
    return int(__builtin_amdgcn_ubfe(bm[v >> 5], v, 1u)) - pad_hits(bm, 64, n);
  }
  uint32_t v[SMALL_ITERS];
#pragma unroll
  for (int k = 0; k < SMALL_ITERS; k++) v[k] = lane + 64 * k < n ? uint32_t(p[lane + 64 * k]) : 0u;
  uint32_t x[SMALL_ITERS];
#pragma unroll
  for (int k = 0; k < SMALL_ITERS; k++) x[k] = bm[v[k] >> 5];
  int c = 0;
#pragma unroll
  for (int k = 0; k < SMALL_ITERS; k++) c += int(__builtin_amdgcn_ubfe(x[k], v[k], 1u));
  return c - pad_hits(bm, 64 * SMALL_ITERS, n);
}

template <class PX>
__device__ __forceinline__ int and_bitmaps_halves(PX a, const uint64_t* y) {
  const int lane = lane_id();
  const auto b = gp(reinterpret_cast<const ulong2*>(y));
  int c = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    ulong2 u[4], v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) u[i] = a[(h * 4 + i) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = b[(h * 4 + i) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 4; i++) c += __popcll(u[i].x & v[i].x) + __popcll(u[i].y & v[i].y);
  }
  return c;
}

template <int DBG = 0, bool HALF = false>
__device__ __forceinline__ int count_vs_lds(const uint64_t* lb, const uint16_t* p, int64_t m) {
  const int type = meta_type(m);
  if (type == CT_BITMAP) {
    if (HALF) return and_bitmaps_halves(reinterpret_cast<const ulong2*>(lb), reinterpret_cast<const uint64_t*>(p));
    return and_bitmaps(reinterpret_cast<const ulong2*>(lb), reinterpret_cast<const uint64_t*>(p));
  }
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
// W = waves per workgroup; W = 1 puts the wave's LDS bitmap at address 0, so
// probe addresses need no per-wave base add.
template <int CQ, int DBG = 0, int W = PAIR_WAVES>
__global__ __launch_bounds__(64 * W, W == 1 ? 5 : 1) void and2_pairs_kernel(const QueryProg* __restrict__ progs, int Q,
                                                           const ViewDev* __restrict__ views, int S,
                                                           const uint2* __restrict__ pairs,
                                                           int32_t* __restrict__ partial) {
  __shared__ uint64_t lbs[W][1024];
  const int wave = W == 1 ? 0 : int(threadIdx.x >> 6);
  const int lane = lane_id();
  const int64_t gw = int64_t(xcd_remap_blocks(blockIdx.x, gridDim.x)) * W + wave;
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
        c = count_vs_lds<DBG, W == 1>(lb, pB, mB);
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
        c = W == 1 ? and_bitmaps_halves(gp(reinterpret_cast<const ulong2*>(pA)), reinterpret_cast<const uint64_t*>(pB))
                   : and_bitmaps(gp(reinterpret_cast<const ulong2*>(pA)), reinterpret_cast<const uint64_t*>(pB));
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
        c = count_vs_lds<0, W == 1>(lb, pA, mA);
        have_pre = false;
      } else {
        lds_wait();  // previous readers of lb are done before it is rewritten
        stage(lb, pA, mA);
        cached = a;
        cached_v = va;
        if (DBG || !PAIR_XPF) {
          c = count_vs_lds<DBG, W == 1>(lb, pB, mB);
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


// ---- v3: groups of equal A, A's head prefetched one group ahead.
//
// Cost isolation of v1 (profiles/r02_pairs/kbench_dbg.log): B loads + probes
// alone 3.5 ms, A loads + staging alone 8.1 ms, both 21.6 ms per 4096-query
// batch: the wave serialised two global round trips per group (A, then the
// first B).  Here a wave walks its chunk group by group (all lanes whose pair
// has the same A container, in lane order):
//   * the first PF x 16 B per lane of A's payload (a whole array of up to
//     PF*512 values, the head of a bitmap / bigger array) is loaded for the
//     NEXT group right after the current group is staged and before its first
//     B load, so the two round trips overlap instead of adding up (chunk index
//     clamped to the container: the loads are unconditional, vmcnt is counted
//     statically); the rest of a big A is loaded when it is staged;
//   * the LDS bitmap stays all-zero between groups: an array A of at most 512
//     values is unstaged by zeroing just its words (its values are the first
//     prefetched register), anything bigger by a full 8 KiB clear -- staging a
//     tail row costs its size, not 8 KiB of clearing;
//   * one-off groups skip LDS: bitmap & bitmap ANDs A with B from memory, a
//     small array A & bitmap B gathers A's values from B.
constexpr int PF = 2;

__device__ __forceinline__ int chunks16(int64_t m) {
  const int t = meta_type(m);
  return t == CT_BITMAP ? 512 : (t == CT_ARRAY ? (meta_n(m) + 7) >> 3 : 1);
}

struct RegP {
  uint4 r[PF];
};

__device__ __forceinline__ void load_head(const uint16_t* p, int64_t m, RegP& x) {
  const int lane = lane_id();
  const int last = chunks16(m) - 1;
  const auto g = gp(reinterpret_cast<const uint4*>(p));
#pragma unroll
  for (int k = 0; k < PF; k++) x.r[k] = g[min(k * 64 + lane, last)];
}

__device__ __forceinline__ int popc_and4(const uint4 a, const uint4 b) {
  return __popc(a.x & b.x) + __popc(a.y & b.y) + __popc(a.z & b.z) + __popc(a.w & b.w);
}

// set the bits of the values in one 16 B chunk (rem = values left from it)
__device__ __forceinline__ void scatter_chunk(uint32_t* l32, const uint4 c, int rem) {
  const uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const uint32_t v = (w[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
    atomicOr(l32 + (v >> 5), e < rem ? (1u << (v & 31)) : 0u);
  }
}

// Stage A into the clean LDS bitmap: the head from registers, the rest of a
// bitmap / big array from memory.
__device__ __forceinline__ void stage_head(uint64_t* lb, const uint16_t* p, int64_t m, const RegP& x) {
  const int lane = lane_id();
  const int t = meta_type(m);
  const auto g = gp(reinterpret_cast<const uint4*>(p));
  if (t == CT_BITMAP) {
    uint4* l4 = reinterpret_cast<uint4*>(lb);
    uint4 y[8 - PF];
#pragma unroll
    for (int k = 0; k < 8 - PF; k++) y[k] = g[(PF + k) * 64 + lane];
#pragma unroll
    for (int k = 0; k < PF; k++) l4[k * 64 + lane] = x.r[k];
#pragma unroll
    for (int k = 0; k < 8 - PF; k++) l4[(PF + k) * 64 + lane] = y[k];
    return;
  }
  if (t != CT_ARRAY) {
    stage(lb, p, m);  // runs (clears first)
    return;
  }
  uint32_t* l32 = reinterpret_cast<uint32_t*>(lb);
  const int n = meta_n(m), n8 = (n + 7) >> 3;
#pragma unroll
  for (int k = 0; k < PF; k++)
    if (k * 64 < n8) scatter_chunk(l32, x.r[k], n - (k * 64 + lane) * 8);
  for (int e8 = PF * 64 + lane; e8 < n8; e8 += 64) scatter_chunk(l32, g[e8], n - e8 * 8);
}

// zero the words an array of n <= 512 values touched (its chunk in `keep`)
__device__ __forceinline__ void unstage_small(uint64_t* lb, const uint4 keep) {
  uint32_t* l32 = reinterpret_cast<uint32_t*>(lb);
  const uint32_t w[4] = {keep.x, keep.y, keep.z, keep.w};
#pragma unroll
  for (int e = 0; e < 4; e++) {
    l32[(w[e] & 0xffffu) >> 5] = 0u;
    l32[w[e] >> 21] = 0u;
  }
}

// bitmap A (head in registers) & bitmap B, both from memory otherwise
__device__ __forceinline__ int and_head_global(const uint16_t* pA, const RegP& x, const uint16_t* pB) {
  const int lane = lane_id();
  const auto ga = gp(reinterpret_cast<const uint4*>(pA));
  const auto gb = gp(reinterpret_cast<const uint4*>(pB));
  int c = 0;
#pragma unroll
  for (int k = 0; k < PF; k++) c += popc_and4(x.r[k], gb[k * 64 + lane]);
#pragma unroll
  for (int h = PF; h < 8; h += 2) {
    const uint4 a0 = ga[h * 64 + lane], a1 = ga[(h + 1) * 64 + lane];
    const uint4 b0 = gb[h * 64 + lane], b1 = gb[(h + 1) * 64 + lane];
    c += popc_and4(a0, b0) + popc_and4(a1, b1);
  }
  return c;
}

// staged LDS bitmap & a global bitmap, in halves (fewer live VGPRs)
__device__ __forceinline__ int and_lds_global(const uint64_t* lb, const uint16_t* pB) {
  const int lane = lane_id();
  const auto g = gp(reinterpret_cast<const uint4*>(pB));
  const uint4* l4 = reinterpret_cast<const uint4*>(lb);
  int c = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint4 b[4], x[4];
#pragma unroll
    for (int k = 0; k < 4; k++) b[k] = g[(h * 4 + k) * 64 + lane];
#pragma unroll
    for (int k = 0; k < 4; k++) x[k] = l4[(h * 4 + k) * 64 + lane];
#pragma unroll
    for (int k = 0; k < 4; k++) c += popc_and4(x[k], b[k]);
  }
  return c;
}

// count_vs_lds() for v3 (bitmap B in halves)
__device__ __forceinline__ int count_vs_lds3(const uint64_t* lb, const uint16_t* p, int64_t m) {
  const int type = meta_type(m);
  if (type == CT_BITMAP) return and_lds_global(lb, p);
  if (type == CT_ARRAY) {
    if (PAIR_SMALL && meta_n(m) <= SMALL_ARRAY_N) return probe_small(reinterpret_cast<const uint32_t*>(lb), p, meta_n(m));
    return probe_pipe(reinterpret_cast<const uint32_t*>(lb), p, meta_n(m));
  }
  return runs_in_lds(lb, p);
}

template <int CQ>
__global__ __launch_bounds__(64 * PAIR_WAVES) void and2_pairs_v3_kernel(const QueryProg* __restrict__ progs, int Q,
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
  const int nq = min(CQ, Q - q0);

  uint32_t ea = NONE;
  int vai = -1;
  int64_t ma = 0, mb = 0;
  uint64_t pal = 0, pbl = 0;
  if (lane < nq) {
    const uint2 e = pairs[u * Q + q0 + lane];
    if (e.x != NONE) {
      ea = e.x;
      vai = progs[q0 + lane].leaf_view[0];
      const int vbi = progs[q0 + lane].leaf_view[1];
      ma = gp(views[vai].meta)[e.x];
      mb = gp(views[vbi].meta)[e.y];
      pal = reinterpret_cast<uint64_t>(payload_of(views[vai], ma));
      pbl = reinterpret_cast<uint64_t>(payload_of(views[vbi], mb));
    }
  }
  const uint64_t valid = __ballot(ea != NONE);
  int mine = 0;
  if (valid) {
    lds_clear(lb);  // clean invariant: all-zero between groups
    uint64_t todo = valid;
    int i = __builtin_ctzll(todo);
    int64_t mA = rl64(ma, i);
    const uint16_t* pA = reinterpret_cast<const uint16_t*>(rl_u64(pal, i));
    RegP ra;
    load_head(pA, mA, ra);
    for (;;) {
      const uint32_t a = __builtin_amdgcn_readlane(ea, i);
      const int va = __builtin_amdgcn_readlane(vai, i);
      const uint64_t group = __ballot(ea == a && vai == va) & todo;
      todo &= ~group;
      const int jn = todo ? __builtin_ctzll(todo) : -1;
      const int tA = meta_type(mA), nA = meta_n(mA);
      int64_t mA2 = 0;
      const uint16_t* pA2 = nullptr;
      if (jn >= 0) {
        mA2 = rl64(ma, jn);
        pA2 = reinterpret_cast<const uint16_t*>(rl_u64(pal, jn));
      }
      bool staged = false;
      if (__popcll(group) == 1) {
        const int64_t mB = rl64(mb, i);
        const uint16_t* pB = reinterpret_cast<const uint16_t*>(rl_u64(pbl, i));
        const int tB = meta_type(mB);
        int c = 0;
        if (tA == CT_BITMAP && tB == CT_BITMAP) {
          c = and_head_global(pA, ra, pB);
        } else if (tA == CT_ARRAY && tB == CT_BITMAP && nA <= 512) {
          const auto bm = gp(reinterpret_cast<const uint32_t*>(pB));
          const uint4 v = lane < ((nA + 7) >> 3) ? ra.r[0] : make_uint4(0, 0, 0, 0);
          c = probe8(bm, v) - pad_hits(bm, 512, nA);
        } else {
          staged = true;
        }
        if (!staged) {
          c = wave_sum(c);
          if (lane == i) mine = c;
          if (jn < 0) break;
          load_head(pA2, mA2, ra);
          i = jn;
          mA = mA2;
          pA = pA2;
          continue;
        }
      }
      uint4 keep = ra.r[0];
      stage_head(lb, pA, mA, ra);
      // next group's A head: issued before this group's B loads (overlapping
      // round trips); kept below the staging (no second register copy)
      __builtin_amdgcn_sched_barrier(0);
      if (jn >= 0) load_head(pA2, mA2, ra);
      __builtin_amdgcn_sched_barrier(0);
      for (uint64_t g = group; g; g &= g - 1) {
        const int k = __builtin_ctzll(g);
        const int64_t mB = rl64(mb, k);
        const uint16_t* pB = reinterpret_cast<const uint16_t*>(rl_u64(pbl, k));
        int c = count_vs_lds3(lb, pB, mB);
        c = wave_sum(c);
        if (lane == k) mine = c;
      }
      // back to all-zero
      if (tA == CT_ARRAY && nA <= 512) {
        if (lane >= ((nA + 7) >> 3)) keep = make_uint4(0, 0, 0, 0);
        unstage_small(lb, keep);
      } else {
        lds_clear(lb);
      }
      if (jn < 0) break;
      i = jn;
      mA = mA2;
      pA = pA2;
    }
  }
  if (lane < nq) partial[u * Q + q0 + lane] = mine;
}


// ---- v6: one wave per workgroup (LDS bitmap at address 0) + the next pair's
// B head prefetched while the current pair is counted.
//
// Per pair, before anything of the current pair waits, ONE load is issued for
// the next valid pair's B: its whole array when n <= 64 (one value per lane),
// else its first 16 B per lane (all of an array of <= 512 values, chunk 0 of a
// bitmap / bigger array).  The current pair's head arrived during the previous
// pair, so a tail pair (most pairs) waits for nothing; the in-order vmcnt wait
// for anything loaded later also covers the prefetch, which by then has had
// the previous pair's work to arrive.
__device__ __forceinline__ uint4 load_bhead(const uint16_t* p, int64_t m) {
  const int lane = lane_id();
  const int t = meta_type(m);
  if (t == CT_ARRAY && meta_n(m) <= 64) {
    const uint32_t v = uint32_t(gp(p)[min(lane, meta_n(m) - 1)]);
    return make_uint4(v, 0, 0, 0);
  }
  const int last = t == CT_BITMAP ? 511 : (t == CT_ARRAY ? ((meta_n(m) + 7) >> 3) - 1 : 0);
  return gp(reinterpret_cast<const uint4*>(p))[min(lane, last)];
}

// |B & staged| with B's head (load_bhead) already in registers
__device__ __forceinline__ int count_vs_head(const uint64_t* lb, const uint16_t* p, int64_t m, const uint4 head) {
  const int lane = lane_id();
  const int t = meta_type(m);
  const uint32_t* bm = reinterpret_cast<const uint32_t*>(lb);
  if (t == CT_ARRAY) {
    const int n = meta_n(m);
    if (n <= 64) {
      const uint32_t v = lane < n ? head.x : 0u;
      return int(__builtin_amdgcn_ubfe(bm[v >> 5], v, 1u)) - pad_hits(bm, 64, n);
    }
    const int n8 = (n + 7) >> 3;
    if (n <= 512) return probe8(bm, lane < n8 ? head : make_uint4(0, 0, 0, 0)) - pad_hits(bm, 512, n);
    // bigger arrays: chunk `lane` is the head, the rest pipelined as probe_pipe
    const auto p4 = gp(reinterpret_cast<const uint4*>(p));
    const int iters = (n8 + 63) >> 6;
    int c = 0;
    int e8 = lane;
    uint4 cur = head;  // n8 > 64: every lane's head chunk is real
#pragma unroll 2
    for (int it = 0; it < iters; it++) {
      const int ne8 = e8 + 64;
      uint4 nxt = make_uint4(0, 0, 0, 0);
      if (ne8 < n8) nxt = p4[ne8];
      c += probe8(bm, cur);
      cur = nxt;
      e8 = ne8;
    }
    return c - pad_hits(bm, iters * 512, n);
  }
  if (t == CT_BITMAP) {
    const auto g = gp(reinterpret_cast<const uint4*>(p));
    const uint4* l4 = reinterpret_cast<const uint4*>(lb);
    int c = popc_and4(l4[lane], head);
    {
      uint4 b[4], x[4];
#pragma unroll
      for (int k = 0; k < 4; k++) b[k] = g[(1 + k) * 64 + lane];
#pragma unroll
      for (int k = 0; k < 4; k++) x[k] = l4[(1 + k) * 64 + lane];
#pragma unroll
      for (int k = 0; k < 4; k++) c += popc_and4(x[k], b[k]);
    }
    {
      uint4 b[3], x[3];
#pragma unroll
      for (int k = 0; k < 3; k++) b[k] = g[(5 + k) * 64 + lane];
#pragma unroll
      for (int k = 0; k < 3; k++) x[k] = l4[(5 + k) * 64 + lane];
#pragma unroll
      for (int k = 0; k < 3; k++) c += popc_and4(x[k], b[k]);
    }
    return c;
  }
  return runs_in_lds(lb, p);
}

template <int CQ>
__global__ __launch_bounds__(64, 5) void and2_pairs_v6_kernel(const QueryProg* __restrict__ progs, int Q,
                                                             const ViewDev* __restrict__ views, int S,
                                                             const uint2* __restrict__ pairs,
                                                             int32_t* __restrict__ partial) {
  __shared__ uint64_t lb[1024];
  const int lane = lane_id();
  const int64_t gw = int64_t(xcd_remap_blocks(blockIdx.x, gridDim.x));
  const int nch = (Q + CQ - 1) / CQ;
  const int64_t u = gw / nch;
  if (u >= int64_t(S) * 16) return;
  const int q0 = int(gw % nch) * CQ;
  const int nq = min(CQ, Q - q0);

  uint32_t ea = NONE;
  int vai = -1;
  int64_t ma = 0, mb = 0;
  uint64_t pal = 0, pbl = 0;
  if (lane < nq) {
    const uint2 e = pairs[u * Q + q0 + lane];
    if (e.x != NONE) {
      ea = e.x;
      vai = progs[q0 + lane].leaf_view[0];
      const int vbi = progs[q0 + lane].leaf_view[1];
      ma = gp(views[vai].meta)[e.x];
      mb = gp(views[vbi].meta)[e.y];
      pal = reinterpret_cast<uint64_t>(payload_of(views[vai], ma));
      pbl = reinterpret_cast<uint64_t>(payload_of(views[vbi], mb));
    }
  }
  uint64_t todo = __ballot(ea != NONE);
  int mine = 0;
  if (todo) {
    uint32_t cached = NONE;
    int cached_v = -1;
    int i = __builtin_ctzll(todo);
    todo &= todo - 1;
    uint4 pre = load_bhead(reinterpret_cast<const uint16_t*>(rl_u64(pbl, i)), rl64(mb, i));
    for (;;) {
      const uint32_t a = __builtin_amdgcn_readlane(ea, i);
      const int va = __builtin_amdgcn_readlane(vai, i);
      const int64_t mA = rl64(ma, i), mB = rl64(mb, i);
      const uint16_t* pA = reinterpret_cast<const uint16_t*>(rl_u64(pal, i));
      const uint16_t* pB = reinterpret_cast<const uint16_t*>(rl_u64(pbl, i));
      const int tA = meta_type(mA), tB = meta_type(mB);
      const int j = todo ? __builtin_ctzll(todo) : -1;
      const uint4 head = pre;
      if (j >= 0) pre = load_bhead(reinterpret_cast<const uint16_t*>(rl_u64(pbl, j)), rl64(mb, j));
      int c;
      if (a == cached && va == cached_v) {
        c = count_vs_head(lb, pB, mB, head);
      } else {
        const bool next_same = j >= 0 && __builtin_amdgcn_readlane(ea, j) == a &&
                               __builtin_amdgcn_readlane(vai, j) == va;
        if (!next_same && tA == CT_BITMAP && tB == CT_BITMAP) {
          c = and_bitmaps_halves(gp(reinterpret_cast<const ulong2*>(pA)), reinterpret_cast<const uint64_t*>(pB));
        } else if (!next_same && tA == CT_ARRAY && tB == CT_BITMAP && PAIR_SMALL && meta_n(mA) <= SMALL_ARRAY_N) {
          c = probe_small(gp(reinterpret_cast<const uint32_t*>(pB)), pA, meta_n(mA));
        } else if (!next_same && tA == CT_ARRAY && tB == CT_BITMAP) {
          lds_wait();
          stage(lb, pB, mB);
          cached = NONE;
          cached_v = -1;
          c = count_vs_lds<0, true>(lb, pA, mA);
        } else {
          lds_wait();  // previous readers of lb are done before it is rewritten
          stage(lb, pA, mA);
          cached = a;
          cached_v = va;
          c = count_vs_head(lb, pB, mB, head);
        }
      }
      c = wave_sum(c);
      if (lane == i) mine = c;
      if (j < 0) break;
      i = j;
      todo &= todo - 1;
    }
  }
  if (lane < nq) partial[u * Q + q0 + lane] = mine;
}
}  // namespace

void launch_keymask_build(const ViewDev& v, int S, uint16_t* out, hipStream_t st) {
  const int64_t n = int64_t(S) * v.D;
  if (n == 0) return;
  hipLaunchKernelGGL(keymask_build_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, v, S, out);
}

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
  if (variant == 6) {
    switch (cq) {
      case 16: { const int64_t wv = units * ((Q + 15) / 16);
        hipLaunchKernelGGL(and2_pairs_v6_kernel<16>, dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); } break;
      case 32: { const int64_t wv = units * ((Q + 31) / 32);
        hipLaunchKernelGGL(and2_pairs_v6_kernel<32>, dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); } break;
      default: { const int64_t wv = units * ((Q + 63) / 64);
        hipLaunchKernelGGL(and2_pairs_v6_kernel<64>, dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); } break;
    }
    return;
  }
  if (variant == 4 || variant == 5) {  // stage-on-demand kernel with 1 / 2 waves per workgroup
    const int W = variant == 4 ? 1 : 2;
    const int64_t waves = units * ((Q + cq - 1) / cq);
    const dim3 g(unsigned((waves + W - 1) / W)), b(64 * W);
#define PK_LAUNCH_W(CQV)                                                                                       \
  {                                                                                                            \
    const int64_t wv = units * ((Q + CQV - 1) / CQV);                                                          \
    if (W == 1) hipLaunchKernelGGL((and2_pairs_kernel<CQV, 0, 1>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q,\
                                   views, S, pairs, partial);                                                  \
    else hipLaunchKernelGGL((and2_pairs_kernel<CQV, 0, 2>), dim3(unsigned((wv + 1) / 2)), dim3(128), 0, st,    \
                            progs, Q, views, S, pairs, partial);                                               \
  }
    (void)g;
    (void)b;
    switch (cq) {
      case 16: PK_LAUNCH_W(16) break;
      case 32: PK_LAUNCH_W(32) break;
      default: PK_LAUNCH_W(64) break;
    }
#undef PK_LAUNCH_W
    return;
  }
  if (variant == 3) {
    switch (cq) {
      case 4: PK_LAUNCH(and2_pairs_v3_kernel, 4) break;
      case 8: PK_LAUNCH(and2_pairs_v3_kernel, 8) break;
      case 16: PK_LAUNCH(and2_pairs_v3_kernel, 16) break;
      case 32: PK_LAUNCH(and2_pairs_v3_kernel, 32) break;
      default: PK_LAUNCH(and2_pairs_v3_kernel, 64) break;
    }
  } else if (variant == 2) {
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
