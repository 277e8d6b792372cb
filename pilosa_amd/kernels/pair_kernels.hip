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
// The shipped kernel is v6: one wave per workgroup, the next pair's B head
// prefetched while the current pair is counted.  Per 4096-query batch on the 954-shard index
// (profiles/r02_pairs/, r03_pairs/): round 1 29.4 ms; branch-free 8-probe
// chunks 21.7 ms; 1 wave per workgroup 18.1 ms; + B-head prefetch 16.9 ms.
// Rejected experiments (git history): register-pipelined operands (v2/v3),
// multi-wave workgroups (v1/v4/v5), size-class lane groups with per-run
// staging (v7, 18.5 ms: lower occupancy, probes unchanged) and lane-interleaved
// u16 probes (v8, 24.0 ms: 5x the load instructions although LDS conflicts
// fell from 0.52 to 0.33 of the LDS cycles) and an XOR-swizzled LDS bitmap
// (18.8 ms, see lds_swz); one-op LDS word addressing per probe half through
// an inline-asm mask (28 instead of 32 VALU per 8 probes, but 17.2 ms: the asm
// stopped the probe loop's unroll; 32 / 16 queries per wave 17.5 / 19.9 ms,
// profiles/r04_l/); non-temporal loads for B containers whose row occurs once
// in the batch (host-marked, so they would not evict reused containers from
// L2: 17.4 vs 16.7 ms, profiles/r04_o/); every load of a container issued before any of it
// is consumed (v9, 20.9 ms: one round trip per array instead of one per
// 512 values, but slower -- the chunked walk is not latency-bound,
// profiles/r03_v9/).  Occupancy: the kernel holds 20 waves/CU (8 KiB LDS and
// 84 VGPRs per wave); padding LDS to 16 / 12 waves/CU measured 17.9 / 23.3 ms
// against 16.7 (profiles/r03_occ/), so sharing one bitmap between two waves
// to reach 32 waves/CU would buy well under the 12->16 step.  One-ahead
// prefetch in the multi-chunk array walks (two rotating register buffers,
// branch-free clamped loads, the stage's first load before the LDS clear)
// measured 23.5 vs 16.7 ms (profiles/r03_pf/): like v9, issuing the array
// loads earlier made the kernel slower, not faster.
//
// Reference hot loops replaced: roaring/roaring.go:3078-3215 intersectionCount*
// and executor.go:1230-1290 (executeCount over executeIntersect).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace pk {
namespace {

constexpr uint32_t NONE = 0xffffffffu;

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
//
// LDS layout: the staged container is a plain 1024-word bitmap.  lds_swz*()
// map a dword / 64-bit word / 16-byte chunk index to its LDS slot; an XOR
// swizzle there (dword w at w ^ (((w >> 5) & 7) << 2), spreading the banks of
// lanes that probe values a fixed stride apart) measured SLOWER on the Zipf
// batch: 18.8 vs 16.8 ms per 4096 queries (profiles/r03_pairs/): the extra
// address VALU per probe costs more than the conflicts it removes, whose
// pattern on real data is already close to random.  Kept as identity hooks.
__device__ __forceinline__ uint32_t lds_swz(uint32_t w) { return w; }
__device__ __forceinline__ uint32_t lds_swz64(uint32_t W) { return W; }
__device__ __forceinline__ uint32_t lds_swzc(uint32_t c) { return c; }

__device__ __forceinline__ const uint16_t* payload_of(const ViewDev& v, int64_t m) {
  return v.payload + meta_off16(m) * 8;
}

__device__ __forceinline__ void lds_clear(uint64_t* lb) {
  ulong2* l2 = reinterpret_cast<ulong2*>(lb);
  const int lane = lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) l2[i * 64 + lane] = make_ulong2(0, 0);
}

// ---- lane-rotated chunks (ROT): bank conflicts of the array probes.
// A lane holds a 16-byte chunk of 8 sorted values and probe8 issues one LDS
// read per value slot k.  With one chunk per lane the k-th values of the 32
// lanes of a ds_read_b32 group lie one chunk apart, i.e. at a near-constant
// stride through the bitmap: for a 512-value array lane l's slot-k value is
// ~1024 l + 128 k, its dword ~32 l + 4 k, so all 32 lanes land on the few
// banks around 4 k ((a/4) mod 32) and each read replays ~5-8 times
// (SQ_LDS_BANK_CONFLICT = 52 % of the LDS-active cycles, profiles/r05_pairs/).
// Rotating each lane's chunk by (lane & 3) dwords before the probes puts
// lane l's slot k on value 2 ((k/2 + l) & 3) + (k & 1): four lanes in a row
// now read values 256 apart (8 dwords, 8 banks), spreading every group over 4x
// the banks.  The count is a sum, so the order is free; 8 v_cndmask per
// chunk (1 VALU per probe).  Staging (ds_or scatter) gets the same rotation,
// with its tail mask rotated alike.
__device__ __forceinline__ uint4 rot4(const uint4 v) {
  const int l = lane_id();
  const uint4 a = (l & 1) ? make_uint4(v.y, v.z, v.w, v.x) : v;
  return (l & 2) ? make_uint4(a.z, a.w, a.x, a.y) : a;
}

// valid-slot mask of a lane's chunk holding `rem` (> 0) of an array's values,
// rotated as rot4 rotates the chunk (bit k = new slot k holds a value)
__device__ __forceinline__ uint32_t rot_mask(int rem) {
  const uint32_t vm = rem >= 8 ? 0xffu : ((1u << rem) - 1u);
  const uint32_t r2 = uint32_t(lane_id() & 3) * 2u;
  return ((vm | (vm << 8)) >> r2) & 0xffu;
}

// Stage a container of any type into lb as a (swizzled) bitmap.  BST
// (batched staging): an array's chunks are all loaded (4 per lane per round
// trip) before the LDS clear and the scatter, instead of one dependent load
// per 512 values -- a 4096-value array was 8 serial round trips, and staging
// was ~60 % of a 32-query batch's pair-kernel time (profiles/r05_serve/).
template <bool BST = false, bool ROT = false>
__device__ __forceinline__ void stage(uint64_t* lb, const uint16_t* p, int64_t m) {
  const int lane = lane_id();
  const int type = meta_type(m);
  ulong2* l2 = reinterpret_cast<ulong2*>(lb);
  if (type == CT_BITMAP) {
    const auto g = gp(reinterpret_cast<const ulong2*>(p));
    ulong2 t[8];
#pragma unroll
    for (int i = 0; i < 8; i++) t[i] = g[i * 64 + lane];
#pragma unroll
    for (int i = 0; i < 8; i++) l2[lds_swzc(uint32_t(i * 64 + lane))] = t[i];
    lds_wait();
    return;
  }
  uint32_t* l32 = reinterpret_cast<uint32_t*>(lb);
  if (BST && type == CT_ARRAY) {
    const int n = meta_n(m);
    const auto p4 = gp(reinterpret_cast<const uint4*>(p));
    const int n8 = (n + 7) >> 3;
    bool cleared = false;
    for (int b = 0; b < n8; b += 4 * 64) {
      uint4 v[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int e8 = b + k * 64 + lane;
        v[k] = make_uint4(0, 0, 0, 0);
        if (e8 < n8) v[k] = p4[e8];
      }
      if (!cleared) {   // the clear overlaps the first round of loads
        lds_clear(lb);
        lds_wait();
        cleared = true;
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int e8 = b + k * 64 + lane;
        const uint4 vk = ROT ? rot4(v[k]) : v[k];
        const uint32_t w[4] = {vk.x, vk.y, vk.z, vk.w};
        const int rem = n - e8 * 8;
        const uint32_t vm = ROT ? rot_mask(rem) : 0u;
#pragma unroll
        for (int t = 0; t < 8; t++) {
          const uint32_t x = (w[t >> 1] >> ((t & 1) * 16)) & 0xffff;
          const bool ok = ROT ? ((vm >> t) & 1u) != 0u : t < rem;
          if (e8 < n8) atomicOr(l32 + lds_swz(x >> 5), ok ? (1u << (x & 31)) : 0u);
        }
      }
    }
    if (!cleared) {
      lds_clear(lb);
    }
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
      const uint4 raw = p4[e8];
      const uint4 v4 = ROT ? rot4(raw) : raw;
      const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
      const int rem = n - e8 * 8;
      const uint32_t vm = ROT ? rot_mask(rem) : 0u;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t v = (w[k >> 1] >> ((k & 1) * 16)) & 0xffff;
        const bool ok = ROT ? ((vm >> k) & 1u) != 0u : k < rem;
        atomicOr(l32 + lds_swz(v >> 5), ok ? (1u << (v & 31)) : 0u);
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
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[lds_swz64(ws)]), mk);
      } else {
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[lds_swz64(ws)]), ~0ull << (s & 63));
        for (uint32_t w = ws + 1; w < we; w++) lb[lds_swz64(w)] = ~0ull;
        const uint32_t hb = e & 63;
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[lds_swz64(we)]), hb ? ((1ull << hb) - 1) : ~0ull);
      }
    }
  }
  lds_wait();
}

// Bit of value v in a 1024-word bitmap: SWZ = the swizzled LDS layout, else a
// plain bitmap (a container in global memory).
template <bool SWZ, class BM>
__device__ __forceinline__ uint32_t bm_word(BM bm, uint32_t v) {
  return bm[SWZ ? lds_swz(v >> 5) : (v >> 5)];
}

// Probe the 8 values packed in one 16-byte chunk against a 1024-word bitmap.
// Branch-free: all 8 word reads are issued before any is consumed (one
// lgkmcnt wait per chunk instead of one per value).  Pad values are 0 and are
// probed too; the caller subtracts their hits once per array (pad_hits()).
// v_bfe_u32 only uses bits 4:0 of its offset operand, so the value itself is
// the offset (no `& 31`).
template <bool SWZ, class BM>
__device__ __forceinline__ int probe8(BM bm, const uint4 v4) {
  const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    x[2 * k] = bm_word<SWZ>(bm, w[k] & 0xffffu);
    x[2 * k + 1] = bm_word<SWZ>(bm, w[k] >> 16);
  }
  int c = 0;
#pragma unroll
  for (int k = 0; k < 4; k++)
    c += int(__builtin_amdgcn_ubfe(x[2 * k], w[k], 1u)) + int(__builtin_amdgcn_ubfe(x[2 * k + 1], w[k] >> 16, 1u));
  return c;
}

// Hits of `slots - n` zero-valued pad probes: bit 0 of the bitmap times the
// number of probed slots that were not array values (counted on lane 0 only,
// so the wave sum subtracts it once).  Dword 0 is not moved by the swizzle.
template <class BM>
__device__ __forceinline__ int pad_hits(BM bm, int slots, int n) {
  return lane_id() == 0 ? int(bm[0] & 1u) * (slots - n) : 0;
}

// Whole-array probe with the next chunk's load issued before the current
// chunk's LDS probes (2-deep register pipeline); lanes past the array hold zero
// chunks; every lane probes 8 slots per iteration.
template <bool SWZ, class BM, bool ROT = false>
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
    c += probe8<SWZ>(bm, ROT ? rot4(cur) : cur);
    cur = nxt;
    e8 = ne8;
  }
  return c - pad_hits(bm, iters * 512, n);
}

// |staged ∩ B| for a bitmap B in global memory (staged chunk c at lds_swzc(c))
__device__ __forceinline__ int and_lds_bitmap(const uint64_t* lb, const uint64_t* y) {
  const int lane = lane_id();
  const ulong2* a = reinterpret_cast<const ulong2*>(lb);
  const auto b = gp(reinterpret_cast<const ulong2*>(y));
  int c = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    ulong2 u[4], v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = b[(h * 4 + i) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 4; i++) u[i] = a[lds_swzc(uint32_t((h * 4 + i) * 64 + lane))];
#pragma unroll
    for (int i = 0; i < 4; i++) c += __popcll(u[i].x & v[i].x) + __popcll(u[i].y & v[i].y);
  }
  return c;
}

// |A ∩ B| of two bitmaps in global memory
__device__ __forceinline__ int and_global_bitmaps(const uint64_t* x, const uint64_t* y) {
  const int lane = lane_id();
  const auto a = gp(reinterpret_cast<const ulong2*>(x));
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

// Count bits of a run container inside the staged bitmap.
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
      c += __popcll(lb[lds_swz64(w)] & mk);
    }
  }
  return c;
}

// Small arrays (n <= SMALL_ARRAY_N, the Zipf tail rows): one value per lane
// and iteration, all loads issued before the probes (probe8 would run 8 LDS
// probe instructions on a few lanes for a 20-value array).
#ifndef SMALL_ARRAY_N
#define SMALL_ARRAY_N 256
#endif
static_assert(SMALL_ARRAY_N % 64 == 0 && SMALL_ARRAY_N > 0, "SMALL_ARRAY_N must be a positive multiple of 64");
constexpr int SMALL_ITERS = SMALL_ARRAY_N / 64;
template <bool SWZ, class BM>
__device__ __forceinline__ int probe_small(BM bm, const uint16_t* arr, int n) {
  const int lane = lane_id();
  const auto p = gp(arr);
  if (n <= 64) {  // one value per lane, one probe (wave-uniform branch)
    const uint32_t v = lane < n ? uint32_t(p[lane]) : 0u;
    return int(__builtin_amdgcn_ubfe(bm_word<SWZ>(bm, v), v, 1u)) - pad_hits(bm, 64, n);
  }
  uint32_t v[SMALL_ITERS];
#pragma unroll
  for (int k = 0; k < SMALL_ITERS; k++) v[k] = lane + 64 * k < n ? uint32_t(p[lane + 64 * k]) : 0u;
  uint32_t x[SMALL_ITERS];
#pragma unroll
  for (int k = 0; k < SMALL_ITERS; k++) x[k] = bm_word<SWZ>(bm, v[k]);
  int c = 0;
#pragma unroll
  for (int k = 0; k < SMALL_ITERS; k++) c += int(__builtin_amdgcn_ubfe(x[k], v[k], 1u));
  return c - pad_hits(bm, 64 * SMALL_ITERS, n);
}

// |B ∩ staged| for any B container type (staged in lb)
template <bool ROT = false>
__device__ __forceinline__ int count_vs_lds(const uint64_t* lb, const uint16_t* p, int64_t m) {
  const int type = meta_type(m);
  if (type == CT_BITMAP) return and_lds_bitmap(lb, reinterpret_cast<const uint64_t*>(p));
  if (type == CT_ARRAY) {
    const uint32_t* bm = reinterpret_cast<const uint32_t*>(lb);
    if (meta_n(m) <= SMALL_ARRAY_N) return probe_small<true>(bm, p, meta_n(m));
    return probe_pipe<true, const uint32_t*, ROT>(bm, p, meta_n(m));
  }
  return runs_in_lds(lb, p);
}

__device__ __forceinline__ uint64_t rl_u64(uint64_t v, int i) {
  return (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(v >> 32), i))) << 32) |
         uint32_t(__builtin_amdgcn_readlane(int(v), i));
}

__device__ __forceinline__ int64_t rl64(int64_t v, int i) { return int64_t(rl_u64(uint64_t(v), i)); }

__device__ __forceinline__ int popc_and4(const uint4 a, const uint4 b) {
  return __popc(a.x & b.x) + __popc(a.y & b.y) + __popc(a.z & b.z) + __popc(a.w & b.w);
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
template <bool SWZ, bool ROT = false>
__device__ __forceinline__ int count_vs_head(const uint64_t* lb, const uint16_t* p, int64_t m, const uint4 head) {
  const int lane = lane_id();
  const int t = meta_type(m);
  const uint32_t* bm = reinterpret_cast<const uint32_t*>(lb);
  if (t == CT_ARRAY) {
    const int n = meta_n(m);
    if (n <= 64) {
      const uint32_t v = lane < n ? head.x : 0u;
      return int(__builtin_amdgcn_ubfe(bm_word<SWZ>(bm, v), v, 1u)) - pad_hits(bm, 64, n);
    }
    const int n8 = (n + 7) >> 3;
    if (n <= 512) {
      const uint4 h = lane < n8 ? head : make_uint4(0, 0, 0, 0);
      return probe8<SWZ>(bm, ROT ? rot4(h) : h) - pad_hits(bm, 512, n);
    }
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
      c += probe8<SWZ>(bm, ROT ? rot4(cur) : cur);
      cur = nxt;
      e8 = ne8;
    }
    return c - pad_hits(bm, iters * 512, n);
  }
  if (t == CT_BITMAP) {
    const auto g = gp(reinterpret_cast<const uint4*>(p));
    const uint4* l4 = reinterpret_cast<const uint4*>(lb);
    auto li = [&](int k) { return SWZ ? lds_swzc(uint32_t(k * 64 + lane)) : uint32_t(k * 64 + lane); };
    int c = popc_and4(l4[li(0)], head);
    {
      uint4 b[4], x[4];
#pragma unroll
      for (int k = 0; k < 4; k++) b[k] = g[(1 + k) * 64 + lane];
#pragma unroll
      for (int k = 0; k < 4; k++) x[k] = l4[li(1 + k)];
#pragma unroll
      for (int k = 0; k < 4; k++) c += popc_and4(x[k], b[k]);
    }
    {
      uint4 b[3], x[3];
#pragma unroll
      for (int k = 0; k < 3; k++) b[k] = g[(5 + k) * 64 + lane];
#pragma unroll
      for (int k = 0; k < 3; k++) x[k] = l4[li(5 + k)];
#pragma unroll
      for (int k = 0; k < 3; k++) c += popc_and4(x[k], b[k]);
    }
    return c;
  }
  return runs_in_lds(lb, p);
}

// ---- dense shadows (SHD): a hot row's container as a 1024-word bitmap in
// HBM (DeviceView.ensure_shadow, shadow_build_kernel), so staging it is one
// coalesced 8 KiB copy and a one-off pair reads it in place.

// copy a global bitmap into the LDS bitmap (one round trip: all 8 loads first)
__device__ __forceinline__ void stage_bitmap(uint64_t* lb, const uint64_t* g) {
  const int lane = lane_id();
  const auto g2 = gp(reinterpret_cast<const ulong2*>(g));
  ulong2* l2 = reinterpret_cast<ulong2*>(lb);
  ulong2 t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = g2[i * 64 + lane];
#pragma unroll
  for (int i = 0; i < 8; i++) l2[lds_swzc(uint32_t(i * 64 + lane))] = t[i];
  lds_wait();
}

// |B & A| for A a bitmap in global memory (a shadow), B any container with
// its head already in registers; a run B goes through the LDS bitmap
__device__ __forceinline__ int count_global_vs_head(uint64_t* lb, const uint64_t* gA, const uint16_t* pB, int64_t mB,
                                                    const uint4 head) {
  const int lane = lane_id();
  const int t = meta_type(mB);
  if (t == CT_ARRAY) {
    const auto g32 = gp(reinterpret_cast<const uint32_t*>(gA));
    const int nb = meta_n(mB);
    if (nb <= 64) {
      const uint32_t v = lane < nb ? head.x : 0u;
      return int(__builtin_amdgcn_ubfe(g32[v >> 5], v, 1u)) - pad_hits(g32, 64, nb);
    }
    if (nb <= 512) return probe8<false>(g32, lane < ((nb + 7) >> 3) ? head : make_uint4(0, 0, 0, 0)) - pad_hits(g32, 512, nb);
    return probe_pipe<false>(g32, pB, nb);
  }
  if (t == CT_BITMAP) {
    const auto a4 = gp(reinterpret_cast<const uint4*>(gA));
    const auto b4 = gp(reinterpret_cast<const uint4*>(pB));
    int c;
    {   // two halves keep the kernel inside its 96-VGPR budget (5 waves/SIMD)
      uint4 x[4], y[3];
#pragma unroll
      for (int k = 0; k < 4; k++) x[k] = a4[k * 64 + lane];
#pragma unroll
      for (int k = 0; k < 3; k++) y[k] = b4[(k + 1) * 64 + lane];
      c = popc_and4(x[0], head);
#pragma unroll
      for (int k = 0; k < 3; k++) c += popc_and4(x[k + 1], y[k]);
    }
    {
      uint4 x[4], y[4];
#pragma unroll
      for (int k = 0; k < 4; k++) x[k] = a4[(k + 4) * 64 + lane];
#pragma unroll
      for (int k = 0; k < 4; k++) y[k] = b4[(k + 4) * 64 + lane];
#pragma unroll
      for (int k = 0; k < 4; k++) c += popc_and4(x[k], y[k]);
    }
    return c;
  }
  lds_wait();
  stage_bitmap(lb, gA);
  return runs_in_lds(lb, pB);
}

#ifdef PK_KBENCH
// shadow[r][s][j]: row rows[r]'s key-j container of shard s as a bitmap (zeros
// where absent).  One wave per (r, s, j): built in LDS by stage(), copied out.
__global__ __launch_bounds__(64) void shadow_build_kernel(ViewDev v, int S, const int32_t* __restrict__ rows, int R,
                                                          uint64_t* __restrict__ shadow) {
  __shared__ uint64_t lb[1024];
  const int64_t w = int64_t(blockIdx.x) + int64_t(blockIdx.y) * 65535;
  if (w >= int64_t(R) * S * 16) return;
  const int j = int(w & 15);
  const int64_t rs = w >> 4;
  const int s = int(rs % S);
  const int r = int(rs / S);
  const int lane = lane_id();
  ulong2* dst = reinterpret_cast<ulong2*>(shadow + w * 1024);
  const int64_t d = rows[r];
  int64_t c = -1;
  if (d >= 0) {
    int64_t lo;
    const uint32_t pres = row_keys(v, s, d, lo);
    if ((pres >> j) & 1) c = lo + __popc(pres & ((1u << j) - 1));
  }
  if (c < 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) dst[i * 64 + lane] = make_ulong2(0, 0);
    return;
  }
  const int64_t m = gp(v.meta)[c];
  stage<true>(lb, payload_of(v, m), m);
  const ulong2* l2 = reinterpret_cast<const ulong2*>(lb);
#pragma unroll
  for (int i = 0; i < 8; i++) dst[i * 64 + lane] = l2[lds_swzc(uint32_t(i * 64 + lane))];
}

#endif  // PK_KBENCH

// Array A of <= 512 values staged from its chunk already in registers (one
// 16-byte chunk per lane, loaded while the previous pair was counted).
template <bool ROT = false>
__device__ __forceinline__ void stage_array_head(uint64_t* lb, int64_t m, const uint4 v4in) {
  const int lane = lane_id();
  lds_clear(lb);
  lds_wait();
  uint32_t* l32 = reinterpret_cast<uint32_t*>(lb);
  const int n = meta_n(m);
  if (lane < ((n + 7) >> 3)) {
    const uint4 v4 = ROT ? rot4(v4in) : v4in;
    const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
    const int rem = n - lane * 8;
    const uint32_t vm = ROT ? rot_mask(rem) : 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (w[k >> 1] >> ((k & 1) * 16)) & 0xffff;
      const bool ok = ROT ? ((vm >> k) & 1u) != 0u : k < rem;
      atomicOr(l32 + lds_swz(v >> 5), ok ? (1u << (v & 31)) : 0u);
    }
  }
  lds_wait();
}

// APF (variant 13): the next pair's A chunk is prefetched too when that pair
// switches to a new A that is an array of <= 512 values (41.6M of the 58.6M
// pairs of the headline batch are array x array), so staging it waits on no
// global load.  Measured 17.7 vs 16.7 ms (profiles/r04_f/): not the default.
// DBG (cost attribution only, wrong answers): 1 = control
// skeleton (pair table, metas, B-head prefetch, readlanes, wave_sum; no
// staging, no counting), 2 = no wave_sum, 3 = no staging, 4 = no counting,
// 5 = skeleton without the B-head loads
//
// SB > 0 (v16): right after A is staged, every pair of A's run whose B is an
// array of <= SB values is counted LANE-parallel in one pass -- each such
// lane walks its own B (16-byte chunks) against the staged bitmap -- instead
// of one wave-cooperative iteration per pair (readlanes, type dispatch, a
// probe pass with most lanes idle, a wave_sum).  27 % of the headline batch's
// pairs have B <= 64 values (scripts/pair_stats.py).
//
// PD = B-head prefetch depth: the heads of the next PD pairs are in flight
// while the current pair is counted (PD = 1: the shipped v6).  The control
// skeleton (DBG 1) with v6's occupancy spends 4.6 of its 7.5 ms waiting on
// these heads (profiles/r05_pairs/).
//
// ONE (v38): pairs whose A is not reused by the next pair ("one-off": nearly
// every pair of a small serving batch) skip staging A when it costs more than
// it saves: a bitmap A is probed in place by B's values (its prefetched head,
// global gathers, no 8 KiB LDS copy), and of two arrays the smaller one is
// staged and the larger probes it.
template <int CQ, bool APF = false, int DBG = 0, int SB = 0, int PD = 1, bool ONE = false, bool BST = false,
          bool SHD = false, bool ROT = false>
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
  uint64_t sha = 0;   // SHD: A's bitmap shadow for this unit (0 = none)
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
      if (SHD && views[vai].shadow_slot != nullptr && meta_type(ma) != CT_BITMAP) {
        const int sl = gp(views[vai].shadow_slot)[progs[q0 + lane].leaf_row[0]];
        if (sl >= 0) sha = reinterpret_cast<uint64_t>(views[vai].shadow + ((int64_t(sl) * S + (u >> 4)) * 16 + (u & 15)) * 1024);
      }
    }
  }
  uint64_t todo = __ballot(ea != NONE);
  int mine = 0;
  if (DBG) lb[lane] = 0;   // cost-attribution variants keep v6's 8 KiB LDS (and occupancy)
  if (todo) {
    uint32_t cached = NONE;
    int cached_v = -1;
    int i = __builtin_ctzll(todo);
    todo &= todo - 1;
    // pf[k]: head of the k-th pair from the current one (k = 0: pair i)
    uint4 pf[PD];
    pf[0] = load_bhead(reinterpret_cast<const uint16_t*>(rl_u64(pbl, i)), rl64(mb, i));
    {
      uint64_t t = todo;
#pragma unroll
      for (int k = 1; k < PD; k++) {
        pf[k] = make_uint4(0, 0, 0, 0);
        if (t) {
          const int jk = __builtin_ctzll(t);
          t &= t - 1;
          pf[k] = load_bhead(reinterpret_cast<const uint16_t*>(rl_u64(pbl, jk)), rl64(mb, jk));
        }
      }
    }
    // A chunk of the pair about to run (APF), valid when apre_ok
    auto small_array = [](int64_t m) { return meta_type(m) == CT_ARRAY && meta_n(m) <= 512; };
    auto load_ahead = [&](int k) {
      const int64_t m = rl64(ma, k);
      const int last = ((meta_n(m) + 7) >> 3) - 1;
      return gp(reinterpret_cast<const uint4*>(rl_u64(pal, k)))[min(lane_id(), last)];
    };
    uint4 apre = make_uint4(0, 0, 0, 0);
    bool apre_ok = false;
    if (APF && small_array(rl64(ma, i))) {
      apre = load_ahead(i);
      apre_ok = true;
    }
    for (;;) {
      const uint32_t a = __builtin_amdgcn_readlane(ea, i);
      const int va = __builtin_amdgcn_readlane(vai, i);
      const int64_t mA = rl64(ma, i), mB = rl64(mb, i);
      const uint16_t* pA = reinterpret_cast<const uint16_t*>(rl_u64(pal, i));
      const uint16_t* pB = reinterpret_cast<const uint16_t*>(rl_u64(pbl, i));
      const int tA = meta_type(mA), tB = meta_type(mB);
      int j = todo ? __builtin_ctzll(todo) : -1;
      const uint4 head = pf[0];
      const uint4 ahead = apre;
      const bool aok = apre_ok;
#pragma unroll
      for (int k = 0; k + 1 < PD; k++) pf[k] = pf[k + 1];
      {
        // the pair PD - 1 places after j enters the ring
        uint64_t t = todo;
#pragma unroll
        for (int k = 1; k < PD; k++) t &= t - 1;
        const int jn = t ? __builtin_ctzll(t) : -1;
        if (DBG == 5)
          pf[PD - 1] = make_uint4(uint32_t(jn), 0, 0, 0);
        else if (jn >= 0)
          pf[PD - 1] = load_bhead(reinterpret_cast<const uint16_t*>(rl_u64(pbl, jn)), rl64(mb, jn));
      }
      if (APF) {
        apre_ok = false;
        if (j >= 0 && !(__builtin_amdgcn_readlane(ea, j) == a && __builtin_amdgcn_readlane(vai, j) == va) &&
            small_array(rl64(ma, j))) {
          apre = load_ahead(j);
          apre_ok = true;
        }
      }
      int c = 0;
      bool done_i = false;   // pair i answered by the lane-parallel small-B pass
      if (DBG == 1 || DBG == 5) {
        c = int(head.x & 1u) + int(tA == tB);
      } else if (a == cached && va == cached_v) {
        c = DBG == 4 ? int(head.x & 1u) : count_vs_head<true, ROT>(lb, pB, mB, head);
      } else if (DBG == 3 || DBG == 4) {
        // staging skipped (3: count against whatever lb holds) or counting
        // skipped (4: stage only), with v6's branch structure
        const bool next_same = j >= 0 && __builtin_amdgcn_readlane(ea, j) == a &&
                               __builtin_amdgcn_readlane(vai, j) == va;
        if (DBG == 4 && !(!next_same && tA == CT_BITMAP && tB == CT_BITMAP) &&
            !(!next_same && tA == CT_ARRAY && tB == CT_BITMAP && meta_n(mA) <= SMALL_ARRAY_N)) {
          lds_wait();
          if (!next_same && tA == CT_ARRAY && tB == CT_BITMAP) {
            stage<BST, ROT>(lb, pB, mB);
            cached = NONE;
            cached_v = -1;
          } else {
            stage<BST, ROT>(lb, pA, mA);
            cached = a;
            cached_v = va;
          }
          c = int(head.x & 1u);
        } else if (DBG == 4) {
          c = int(head.x & 1u);
        } else {
          cached = a;
          cached_v = va;
          c = count_vs_head<true, ROT>(lb, pB, mB, head);
        }
      } else {
        const bool next_same = j >= 0 && __builtin_amdgcn_readlane(ea, j) == a &&
                               __builtin_amdgcn_readlane(vai, j) == va;
        if (!next_same && tA == CT_BITMAP && tB == CT_BITMAP) {
          c = and_global_bitmaps(reinterpret_cast<const uint64_t*>(pA), reinterpret_cast<const uint64_t*>(pB));
        } else if (!next_same && tA == CT_ARRAY && tB == CT_BITMAP && meta_n(mA) <= SMALL_ARRAY_N) {
          c = probe_small<false>(gp(reinterpret_cast<const uint32_t*>(pB)), pA, meta_n(mA));
        } else if (SHD && rl_u64(sha, i) != 0) {
          // A has a dense shadow: a run of pairs copies it into LDS in one
          // round trip; a one-off pair reads it in place
          const uint64_t* gA = reinterpret_cast<const uint64_t*>(rl_u64(sha, i));
          if (next_same) {
            lds_wait();
            stage_bitmap(lb, gA);
            cached = a;
            cached_v = va;
            c = count_vs_head<true, ROT>(lb, pB, mB, head);
          } else {
            c = count_global_vs_head(lb, gA, pB, mB, head);
            if (tB == CT_RUN) {
              cached = NONE;
              cached_v = -1;
            }
          }
        } else if (!next_same && tA == CT_ARRAY && tB == CT_BITMAP) {
          lds_wait();
          stage<BST, ROT>(lb, pB, mB);
          cached = NONE;
          cached_v = -1;
          c = count_vs_lds<ROT>(lb, pA, mA);
        } else if (ONE && !next_same && tA == CT_BITMAP && tB == CT_ARRAY) {
          // B's values probe A where it lies (B's head chunk is in registers)
          const auto gA = gp(reinterpret_cast<const uint32_t*>(pA));
          const int nb = meta_n(mB);
          if (nb <= 64) {
            const uint32_t v = lane < nb ? head.x : 0u;
            c = int(__builtin_amdgcn_ubfe(gA[v >> 5], v, 1u)) - pad_hits(gA, 64, nb);
          } else if (nb <= 512) {
            c = probe8<false>(gA, lane < ((nb + 7) >> 3) ? head : make_uint4(0, 0, 0, 0)) - pad_hits(gA, 512, nb);
          } else {
            c = probe_pipe<false>(gA, pB, nb);
          }
        } else if (ONE && !next_same && tA == CT_ARRAY && tB == CT_ARRAY && meta_n(mB) < meta_n(mA)) {
          // the smaller array is staged, the larger one probes it
          lds_wait();
          stage<BST, ROT>(lb, pB, mB);
          cached = NONE;
          cached_v = -1;
          c = count_vs_lds<ROT>(lb, pA, mA);
        } else {
          lds_wait();  // previous readers of lb are done before it is rewritten
          if (APF && aok && small_array(mA))
            stage_array_head<ROT>(lb, mA, ahead);
          else
            stage<BST, ROT>(lb, pA, mA);
          cached = a;
          cached_v = va;
          if constexpr (SB > 0) {
            const uint64_t runm = __ballot(ea == a && vai == va) & (todo | (1ull << i));
            const uint64_t sm = runm & __ballot(meta_type(mb) == CT_ARRAY && meta_n(mb) <= SB);
            if (PD == 1 && (sm & (sm - 1))) {   // two or more: one lane-parallel pass
              const uint32_t* bm32 = reinterpret_cast<const uint32_t*>(lb);
              if ((sm >> lane) & 1) {
                const int nb = meta_n(mb);
                const int n8 = (nb + 7) >> 3;
                const auto p4 = gp(reinterpret_cast<const uint4*>(pbl));
                // every chunk's load in flight before the first probe (one round trip)
                uint4 v[SB > 0 ? SB / 8 : 1];
#pragma unroll
                for (int k = 0; k < SB / 8; k++) {
                  v[k] = make_uint4(0, 0, 0, 0);
                  if (k < n8) v[k] = p4[k];
                }
                int cnt = 0;
#pragma unroll
                for (int k = 0; k < SB / 8; k++) cnt += probe8<true>(bm32, v[k]);
                mine = cnt - int(bm32[0] & 1u) * ((SB / 8) * 8 - nb);   // zero pad slots
              }
              todo &= ~sm;
              done_i = (sm >> i) & 1;
              if (j >= 0 && ((sm >> j) & 1)) {
                // the prefetched next pair was answered here: prefetch the new next
                j = todo ? __builtin_ctzll(todo) : -1;
                if (j >= 0) pf[0] = load_bhead(reinterpret_cast<const uint16_t*>(rl_u64(pbl, j)), rl64(mb, j));
              }
            }
          }
          if (!done_i) c = count_vs_head<true, ROT>(lb, pB, mB, head);
        }
      }
      if (done_i) {
      } else if (DBG == 2) {
        mine += c;
      } else {
        c = wave_sum(c);
        if (lane == i) mine = c;
      }
      if (j < 0) break;
      i = j;
      todo &= todo - 1;
    }
  }
  if (DBG) {
    lds_wait();
    mine += int(lb[lane] & 1u);
  }
  if (lane < nq) partial[u * Q + q0 + lane] = mine;
}
#ifdef PK_KBENCH
// ---- v10: one wave per (unit, chunk of CQ queries) as v6, but a run of
// queries that share the staged row A is counted as ONE flat stream.
//
// v6 handles one pair at a time: readlanes, a type dispatch, one probe pass
// with most lanes idle for the typical 30-300-value partner, and a wave_sum,
// for each of the 58.6M pairs of a 4096-query batch.  Here, after A is
// staged, the run's array partners are laid end to end as 16-byte chunks
// (8 values): an inclusive wave scan of their chunk counts gives each pair's
// first chunk, and every iteration gives each lane the next chunk of the
// stream, whatever pair it belongs to.  The lane->pair map of an iteration
// is a popcount: the pairs' first chunks are bits of a boundary bitmap in
// LDS, so pair(lane) = pairs started before the window + mbcnt of the
// window's 64 boundary bits up to the lane.  Per-pair sums are kept in a
// register while a lane stays on one pair and flushed with a non-returning
// LDS add when it moves on; each pair's lane reads its total at the end.
// Bitmap / run partners (rare) keep v6's per-pair wave-cooperative count.
extern "C" __device__ int __ockl_wfscan_add_i32(int, bool);

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}

constexpr int V10_WIN = 2048;  // chunks per boundary window: 64 dwords, one per lane

// DBG (cost isolation only, wrong answers): 1 = no probes, 2 = no staging,
// 3 = no chunk loads, 4 = singletons skipped
template <int CQ, int PF, int DBG = 0>
__global__ __launch_bounds__(64, 4) void and2_pairs_v10_kernel(const QueryProg* __restrict__ progs, int Q,
                                                              const ViewDev* __restrict__ views, int S,
                                                              const uint2* __restrict__ pairs,
                                                              int32_t* __restrict__ partial) {
  __shared__ uint64_t lb[1024];          // the staged container, as a bitmap
  __shared__ uint4 tbl[64];              // per array partner: payload pointer, first chunk, n
  __shared__ uint32_t bnd[V10_WIN / 32];  // first-chunk bits of the current window
  __shared__ int32_t cnt[64];            // per array partner: its count
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
  const bool valid = ea != NONE;
  const int tB = meta_type(mb);
  const int nB = meta_n(mb);
  const uint32_t* bm32 = reinterpret_cast<const uint32_t*>(lb);
  uint64_t todo = __ballot(valid);
  int mine = 0;
  while (todo) {
    const int i = __builtin_ctzll(todo);
    const uint32_t a = __builtin_amdgcn_readlane(ea, i);
    const int va = __builtin_amdgcn_readlane(vai, i);
    // the batch is sorted by (A, B): a run's lanes are consecutive among the valid ones
    const uint64_t run = __ballot(valid && ea == a && vai == va) & todo;
    todo &= ~run;
    const int64_t mA = rl64(ma, i);
    const uint16_t* pA = reinterpret_cast<const uint16_t*>(rl_u64(pal, i));
    const int tA = meta_type(mA);
    if (DBG == 4 && (run & (run - 1)) == 0) continue;
    if ((run & (run - 1)) == 0) {
      // a pair of its own: v6's shortcuts that need no staging, else stage the smaller array
      const int64_t mB = rl64(mb, i);
      const uint16_t* pB = reinterpret_cast<const uint16_t*>(rl_u64(pbl, i));
      const int tb = meta_type(mB);
      int c;
      if (tA == CT_BITMAP && tb == CT_BITMAP) {
        c = and_global_bitmaps(reinterpret_cast<const uint64_t*>(pA), reinterpret_cast<const uint64_t*>(pB));
      } else if (tA == CT_ARRAY && tb == CT_BITMAP && meta_n(mA) <= SMALL_ARRAY_N) {
        c = probe_small<false>(gp(reinterpret_cast<const uint32_t*>(pB)), pA, meta_n(mA));
      } else if (tA == CT_ARRAY && (tb == CT_BITMAP || (tb == CT_ARRAY && meta_n(mB) < meta_n(mA)))) {
        lds_wait();
        stage(lb, pB, mB);
        c = count_vs_lds(lb, pA, mA);
      } else {
        lds_wait();
        stage(lb, pA, mA);
        c = count_vs_lds(lb, pB, mB);
      }
      c = wave_sum(c);
      if (lane == i) mine = c;
      continue;
    }
    lds_wait();  // previous readers of lb / tbl / cnt are done before they are rewritten
    if (DBG != 2) stage(lb, pA, mA);
    const bool inrun = (run >> lane) & 1;
    const uint64_t am = __ballot(inrun && tB == CT_ARRAY);
    // bitmap / run partners: one at a time, wave-cooperative
    for (uint64_t other = run & ~am; other; other &= other - 1) {
      const int j = __builtin_ctzll(other);
      int c = count_vs_lds(lb, reinterpret_cast<const uint16_t*>(rl_u64(pbl, j)), rl64(mb, j));
      c = wave_sum(c);
      if (lane == j) mine = c;
    }
    if (!am) continue;
    // array partners: one flat stream of 16-byte chunks
    const bool isArr = (am >> lane) & 1;
    const int n8 = isArr ? (nB + 7) >> 3 : 0;
    const int incl = __ockl_wfscan_add_i32(n8, true);
    const int start = incl - n8;
    const int T = __builtin_amdgcn_readlane(incl, 63);
    const int ord = int(mbcnt64(am));
    if (isArr) {
      tbl[ord] = make_uint4(uint32_t(pbl), uint32_t(pbl >> 32), uint32_t(start), uint32_t(nB));
      cnt[ord] = 0;
    }
    const int bit0 = int(bm32[0] & 1u);  // hits of a zero-valued pad probe
    int kb = -1, curk = -1, acc = 0;
#pragma unroll 1
    for (int w0 = 0; w0 < T; w0 += V10_WIN) {
      bnd[lane] = 0u;
      lds_wait();
      if (isArr && start >= w0 && start < w0 + V10_WIN)
        atomicOr(&bnd[(start - w0) >> 5], 1u << (start & 31));
      lds_wait();
      // the window's boundary words live in a VGPR (lane w = word w): each
      // iteration takes its 64 bits with two readlanes, no LDS round trip
      const uint32_t bw = bnd[lane];
      const int wend = min(T, w0 + V10_WIN);
      const int iters = (wend - w0 + 63) >> 6;
      // software pipeline: the mapping and chunk load of iteration it+PF are
      // issued before iteration it's chunk is probed (PF register slots,
      // statically indexed by unrolling the slot loop)
      auto fetch = [&](int it, uint4& v, int& k, int& rem) {
        const uint64_t M = (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(bw), 2 * it + 1))) << 32) |
                           uint32_t(__builtin_amdgcn_readlane(int(bw), 2 * it));
        k = kb + int(mbcnt64(M)) + int((M >> lane) & 1u);
        kb += __popcll(M);
        const int t = w0 + it * 64 + lane;
        v = make_uint4(0, 0, 0, 0);
        rem = -1;
        if (t < wend) {
          const uint4 e = tbl[k];
          const int c = t - int(e.z);
          if (DBG == 3)
            v = make_uint4(uint32_t(c) * 0x10001u, e.x, e.y, uint32_t(t));
          else
            v = gp(reinterpret_cast<const uint4*>((uint64_t(e.y) << 32) | e.x))[c];
          rem = int(e.w) - c * 8;
        }
      };
      uint4 bv[PF];
      int bk[PF], brem[PF];
#pragma unroll
      for (int sl = 0; sl < PF; sl++) {
        bk[sl] = -1;
        brem[sl] = -1;
        bv[sl] = make_uint4(0, 0, 0, 0);
        if (sl < iters) fetch(sl, bv[sl], bk[sl], brem[sl]);
      }
#pragma unroll 1
      for (int it0 = 0; it0 < iters; it0 += PF) {
#pragma unroll
        for (int sl = 0; sl < PF; sl++) {
          const int it = it0 + sl;
          if (it >= iters) break;
          const uint4 cv = bv[sl];
          const int ck = bk[sl], crem = brem[sl];
          brem[sl] = -1;
          if (it + PF < iters) fetch(it + PF, bv[sl], bk[sl], brem[sl]);
          if (crem >= 0) {
            int cc = DBG == 1 ? int(cv.x ^ cv.y ^ cv.z ^ cv.w) & 7 : probe8<true>(bm32, cv);
            if (crem < 8) cc -= bit0 * (8 - crem);
            if (ck != curk) {
              if (curk >= 0) atomicAdd(&cnt[curk], acc);
              curk = ck;
              acc = cc;
            } else {
              acc += cc;
            }
          }
        }
      }
    }
    if (curk >= 0) atomicAdd(&cnt[curk], acc);
    lds_wait();
    if (isArr) mine = cnt[ord];
  }
  if (lane < nq) partial[u * Q + q0 + lane] = mine;
}
#endif  // PK_KBENCH
}  // namespace

#ifdef PK_KBENCH
template <int CQ>
void launch_v10_dbg(int dbg, int64_t wv, const QueryProg* progs, int Q, const ViewDev* views, int S, uint2* pairs,
                    int32_t* partial, hipStream_t st) {
  switch (dbg) {
    case 1: hipLaunchKernelGGL((and2_pairs_v10_kernel<CQ, 2, 1>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    case 2: hipLaunchKernelGGL((and2_pairs_v10_kernel<CQ, 2, 2>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    case 3: hipLaunchKernelGGL((and2_pairs_v10_kernel<CQ, 2, 3>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    default: hipLaunchKernelGGL((and2_pairs_v10_kernel<CQ, 2, 4>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
  }
}

template <int CQ>
void launch_v6_dbg(int dbg, int64_t wv, const QueryProg* progs, int Q, const ViewDev* views, int S, uint2* pairs,
                   int32_t* partial, hipStream_t st) {
  switch (dbg) {
    case 1: hipLaunchKernelGGL((and2_pairs_v6_kernel<CQ, false, 1>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    case 2: hipLaunchKernelGGL((and2_pairs_v6_kernel<CQ, false, 2>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    case 3: hipLaunchKernelGGL((and2_pairs_v6_kernel<CQ, false, 3>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    case 4: hipLaunchKernelGGL((and2_pairs_v6_kernel<CQ, false, 4>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    case 5: hipLaunchKernelGGL((and2_pairs_v6_kernel<CQ, false, 5>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    case 6: hipLaunchKernelGGL((and2_pairs_v6_kernel<CQ, false, 1, 0, 2>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
    default: hipLaunchKernelGGL((and2_pairs_v6_kernel<CQ, false, 1, 0, 3>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial); break;
  }
}

void launch_shadow_build(const ViewDev& v, int S, const int32_t* rows, int R, uint64_t* shadow, hipStream_t st) {
  const int64_t w = int64_t(R) * S * 16;
  if (w <= 0) return;
  const dim3 grid(unsigned(w < 65535 ? w : 65535), unsigned((w + 65534) / 65535));
  hipLaunchKernelGGL(shadow_build_kernel, grid, dim3(64), 0, st, v, S, rows, R, shadow);
}

#endif  // PK_KBENCH

void launch_keymask_build(const ViewDev& v, int S, uint16_t* out, hipStream_t st) {
  const int64_t n = int64_t(S) * v.D;
  if (n == 0) return;
  hipLaunchKernelGGL(keymask_build_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, v, S, out);
}

// pair_build then the pair kernel; `cq` = queries per wave (16 / 32 / 64; <= 0
// picks by batch size: 32 for Q <= 2048, 64 above).  `variant` 10 runs the
// flat-stream kernel (and2_pairs_v10) with 1 chunk prefetched, 11 / 12 with 2
// / 3, anything else v6.
void launch_and2_pairs(const QueryProg* progs, int Q, const ViewDev* views, int S, uint2* pairs, int32_t* partial,
                       int cq, int variant, hipStream_t st) {
  const int64_t items = int64_t(Q) * S;
  if (items == 0) return;
  hipLaunchKernelGGL(pair_build_kernel, dim3(unsigned((items + 255) / 256)), dim3(256), 0, st, progs, Q, views, S,
                     pairs);
  const int64_t units = int64_t(S) * 16;
  // serving-size batches (<= 128 queries: almost every pair is one-off):
  // batched array staging (variant 39: an array's chunk loads all in flight
  // before the LDS scatter) at 4 queries per wave up to 32 queries, 32 up to
  // 64, 16 up to 128.  Round 6 sweeps (profiles/r06_serve/kbench_b*.log):
  // 0.437 / 0.794 / 1.225 ms at 32 / 64 / 128 queries against 0.554 / 1.019 /
  // 1.353 ms for round 5's variant 40 at 8 per wave (whose one-off in-place
  // probes cost more than they save).  Bigger batches keep v6.
  if (variant == 6 && cq <= 0 && Q <= 128) {
    variant = 39;
    cq = Q <= 32 ? 4 : (Q <= 64 ? 32 : 16);
  }
#ifdef PK_KBENCH
  if (variant == 50 && cq <= 0 && Q <= 128) variant = 51;   // the serving variant, lane-rotated
#endif
  if (variant == 41 && cq <= 0 && Q <= 128) variant = 42;   // the same with dense shadows
  if (cq <= 0) cq = Q <= 128 ? 8 : (Q <= 2048 ? 32 : 64);
// The shipped build instantiates v6 and its serving variant 39 only; every
// measured-and-rejected variant and cost-isolation skeleton (v10-v13,
// 16-24, 31-38, 40-42, 50/51) is built into the kbench module alone
// (pilosa_amd/native/build.py --kbench, scripts/kbench.py).
#ifdef PK_KBENCH
#define PK_LAUNCH(CQV)                                                                                       \
  {                                                                                                          \
    const int64_t wv = units * ((Q + CQV - 1) / CQV);                                                        \
    if (variant == 10)                                                                                       \
      hipLaunchKernelGGL((and2_pairs_v10_kernel<CQV, 1>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, \
                         S, pairs, partial);                                                                 \
    else if (variant == 11)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v10_kernel<CQV, 2>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, \
                         S, pairs, partial);                                                                 \
    else if (variant == 12)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v10_kernel<CQV, 3>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, \
                         S, pairs, partial);                                                                 \
    else if (variant >= 21 && variant <= 24)                                                                 \
      launch_v10_dbg<CQV>(variant - 20, wv, progs, Q, views, S, pairs, partial, st);                         \
    else if (variant == 16)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 32>), dim3(unsigned(wv)), dim3(64), 0, st, progs, \
                         Q, views, S, pairs, partial);                                                       \
    else if (variant == 17)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 16>), dim3(unsigned(wv)), dim3(64), 0, st, progs, \
                         Q, views, S, pairs, partial);                                                       \
    else if (variant == 18)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 2>), dim3(unsigned(wv)), dim3(64), 0, st,     \
                         progs, Q, views, S, pairs, partial);                                                \
    else if (variant == 19)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 3>), dim3(unsigned(wv)), dim3(64), 0, st,     \
                         progs, Q, views, S, pairs, partial);                                                \
    else if (variant == 20)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 4>), dim3(unsigned(wv)), dim3(64), 0, st,     \
                         progs, Q, views, S, pairs, partial);                                                \
    else if (variant >= 31 && variant <= 37)                                                                 \
      launch_v6_dbg<CQV>(variant - 30, wv, progs, Q, views, S, pairs, partial, st);                          \
    else if (variant == 41)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 1, false, false, true>), dim3(unsigned(wv)),  \
                         dim3(64), 0, st, progs, Q, views, S, pairs, partial);                               \
    else if (variant == 42)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 1, true, true, true>), dim3(unsigned(wv)),    \
                         dim3(64), 0, st, progs, Q, views, S, pairs, partial);                               \
    else if (variant == 39)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 1, false, true>), dim3(unsigned(wv)), dim3(64), 0, \
                         st, progs, Q, views, S, pairs, partial);                                            \
    else if (variant == 40)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 1, true, true>), dim3(unsigned(wv)), dim3(64), 0, \
                         st, progs, Q, views, S, pairs, partial);                                            \
    else if (variant == 38)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 1, true>), dim3(unsigned(wv)), dim3(64), 0, st, \
                         progs, Q, views, S, pairs, partial);                                                \
    else if (variant == 50)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 1, false, false, false, true>),               \
                         dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial);           \
    else if (variant == 51)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 1, true, true, false, true>),                 \
                         dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S, pairs, partial);           \
    else if (variant == 13)                                                                                  \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, true>), dim3(unsigned(wv)), dim3(64), 0, st, progs, Q,    \
                         views, S, pairs, partial);                                                          \
    else                                                                                                     \
      hipLaunchKernelGGL(and2_pairs_v6_kernel<CQV>, dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S,  \
                         pairs, partial);                                                                    \
  }
#else
#define PK_LAUNCH(CQV)                                                                                       \
  {                                                                                                          \
    const int64_t wv = units * ((Q + CQV - 1) / CQV);                                                        \
    if (variant == 39)                                                                                       \
      hipLaunchKernelGGL((and2_pairs_v6_kernel<CQV, false, 0, 0, 1, false, true>), dim3(unsigned(wv)), dim3(64), 0, \
                         st, progs, Q, views, S, pairs, partial);                                            \
    else                                                                                                     \
      hipLaunchKernelGGL(and2_pairs_v6_kernel<CQV>, dim3(unsigned(wv)), dim3(64), 0, st, progs, Q, views, S,  \
                         pairs, partial);                                                                    \
  }
#endif  // PK_KBENCH
  switch (cq) {
    case 4: PK_LAUNCH(4) break;
    case 8: PK_LAUNCH(8) break;
    case 16: PK_LAUNCH(16) break;
    case 32: PK_LAUNCH(32) break;
    default: PK_LAUNCH(64) break;
  }
#undef PK_LAUNCH
}

// Column sums of the pair kernel's per-(unit, query) partials (int32[U][n])
// scattered straight into the batch result: out[ti[q]] += sum_u partial[u][q].
// Replaces a strided torch reduction (~67 us for a 36-query serving batch,
// profiles/r05_serve/) plus an index_copy.  Block = 64 columns x 4 row lanes
// over a 128-row chunk; one int64 atomic per (block, column).
__global__ __launch_bounds__(256) void partial_sum_scatter_kernel(const int32_t* __restrict__ partial, int64_t U,
                                                                  int n, const int64_t* __restrict__ ti,
                                                                  unsigned long long* __restrict__ out,
                                                                  int64_t nout) {
  __shared__ long long acc[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int q = int(blockIdx.x) * 64 + tx;
  const int64_t r0 = int64_t(blockIdx.y) * 128;
  const int64_t r1 = r0 + 128 < U ? r0 + 128 : U;
  long long a = 0;
  if (q < n) {
#pragma unroll 8
    for (int64_t r = r0 + ty; r < r1; r += 4) a += partial[r * n + q];
  }
  acc[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && q < n) {
    const long long t = acc[0][tx] + acc[1][tx] + acc[2][tx] + acc[3][tx];
    const int64_t o = ti[q];
    if (t && o >= 0 && o < nout) atomicAdd(out + o, (unsigned long long)t);
  }
}

void launch_partial_sum_scatter(const int32_t* partial, int64_t U, int n, const int64_t* ti, int64_t* out,
                                int64_t nout, hipStream_t st) {
  if (U <= 0 || n <= 0) return;
  const dim3 grid(unsigned((n + 63) / 64), unsigned((U + 127) / 128));
  hipLaunchKernelGGL(partial_sum_scatter_kernel, grid, dim3(256), 0, st, partial, U, n, ti,
                     reinterpret_cast<unsigned long long*>(out), nout);
}

}  // namespace pk
