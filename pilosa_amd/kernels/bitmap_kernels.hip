// CDNA4 (gfx950) kernels for the bitmap index hot path.
//
// Reference hot loops replaced here:
//   K1/K2 popcountAndSlice / intersectionCount  roaring/roaring.go:3078-3215,5061-5072
//   K3-K6 intersect/union/difference/xor        roaring/roaring.go:3217-4344
//   K8    count/countRange                      roaring/roaring.go:2000-2110
//   K10   OffsetRange row extraction             roaring/roaring.go:535-558
//   K13   BSI sum                                fragment.go:1109-1141
//   K17/K21 TopN / GroupBy intersection counts  fragment.go:1568-1700, executor.go:3060-3230
//
// Execution model (ours): a whole batch of queries is evaluated over ALL local
// shards in one launch.  One 64-lane wave owns one (query, shard) work item
// and walks the <=16 container keys of the row in that shard.  A container is
// held as a register "tile": 1024 u64 words spread over the wave, lane l owns
// words {128*i + 2*l + h | i<8, h<2} so every tile load is eight fully
// coalesced 1 KiB global_load_dwordx4 wave-instructions.  Array and run
// containers are expanded into a wave-private 8 KiB LDS bitmap (ds_or_b64
// scatter) and read back in the same layout.  Boolean query trees are compiled
// on the host to a tiny postfix program (<=32 ops, <=16 leaves) that the wave
// interprets with a 4-deep register stack (static register moves, no scratch).
// Fast paths: Count(Row) sums container cardinalities from the metadata only;
// Count(Intersect(a,b)) dispatches on the container type pair
// (bitmap&bitmap popcount, array->bitmap probe, array->LDS-bitmap probe).
//
// Workgroups are remapped XCD-aware: consecutive logical blocks (same shard,
// different queries -> the same hot containers) are kept on one XCD so they
// share its L2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.h"

namespace pk {

__device__ __forceinline__ int wave_lane() { return threadIdx.x & 63; }

// Wave-wide sum through DPP row ops (ockl) instead of six dependent
// ds_bpermute round trips (__shfl_xor).
extern "C" __device__ long __ockl_wfred_add_i64(long);
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) { return int64_t(__ockl_wfred_add_i64(long(v))); }

// broadcast lane `src` (wave-uniform) with scalar readlanes, no LDS pipe
__device__ __forceinline__ int64_t rl_i64(int64_t v, int src) {
  return int64_t((uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint64_t(v) >> 32), src))) << 32) |
                 uint32_t(__builtin_amdgcn_readlane(int(v), src)));
}

__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nblk) {
  // bijective remap: blocks b, b+8, b+16 ... (same XCD) get consecutive ids
  const uint32_t nx = 8;
  uint32_t xcd = bid % nx, loc = bid / nx;
  uint32_t q = nblk / nx, r = nblk % nx;
  uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + loc;
}

struct Tile {
  ulong2 w[8];
};

__device__ __forceinline__ void tile_zero(Tile& t) {
#pragma unroll
  for (int i = 0; i < 8; i++) t.w[i] = make_ulong2(0, 0);
}

__device__ __forceinline__ int tile_popc(const Tile& t) {
  int c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) c += __popcll(t.w[i].x) + __popcll(t.w[i].y);
  return c;
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Expand an array / run container into the wave-private LDS bitmap `lb`
// (1024 u64).  Caller reads it back.
__device__ __forceinline__ void lds_expand(uint64_t* lb, const uint16_t* payload, int64_t m) {
  const int lane = wave_lane();
  ulong2* l2 = reinterpret_cast<ulong2*>(lb);
#pragma unroll
  for (int i = 0; i < 8; i++) l2[i * 64 + lane] = make_ulong2(0, 0);
  lds_fence();
  const int type = meta_type(m);
  const uint16_t* p = payload + meta_off16(m) * 8;
  if (type == CT_ARRAY) {
    // 16-byte loads: 8 values per lane per instruction (payload is 16B aligned,
    // padded to a multiple of 8 values; the tail is masked by index).
    const int n = meta_n(m);
    const uint4* p4 = reinterpret_cast<const uint4*>(p);
    const int n8 = (n + 7) >> 3;
    for (int e8 = lane; e8 < n8; e8 += 64) {
      const uint4 v4 = p4[e8];
      const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t v = (w[k >> 1] >> ((k & 1) * 16)) & 0xffff;
        if (e8 * 8 + k < n) atomicOr(reinterpret_cast<unsigned long long*>(&lb[v >> 6]), 1ull << (v & 63));
      }
    }
  } else {  // run
    const int nr = p[0];
    for (int r = lane; r < nr; r += 64) {
      uint32_t s = p[8 + 2 * r], e = uint32_t(p[9 + 2 * r]) + 1;  // [s,e)
      uint32_t ws = s >> 6, we = (e - 1) >> 6;
      if (ws == we) {
        uint64_t mk = (e - s == 64) ? ~0ull : (((1ull << (e - s)) - 1) << (s & 63));
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[ws]), mk);
      } else {
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[ws]), ~0ull << (s & 63));
        for (uint32_t w = ws + 1; w < we; w++) lb[w] = ~0ull;
        uint32_t hb = e & 63;
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[we]), hb ? ((1ull << hb) - 1) : ~0ull);
      }
    }
  }
  lds_fence();
}

__device__ __forceinline__ void tile_load(Tile& t, const uint16_t* payload, int64_t m, uint64_t* lb) {
  const int lane = wave_lane();
  if (meta_type(m) == CT_BITMAP) {
    const ulong2* p = reinterpret_cast<const ulong2*>(payload + meta_off16(m) * 8);
#pragma unroll
    for (int i = 0; i < 8; i++) t.w[i] = p[i * 64 + lane];
  } else {
    lds_expand(lb, payload, m);
    const ulong2* l2 = reinterpret_cast<const ulong2*>(lb);
#pragma unroll
    for (int i = 0; i < 8; i++) t.w[i] = l2[i * 64 + lane];
    lds_fence();
  }
}

template <int OP>
__device__ __forceinline__ void tile_op(Tile& a, const Tile& b) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (OP == OP_AND) { a.w[i].x &= b.w[i].x; a.w[i].y &= b.w[i].y; }
    if (OP == OP_OR) { a.w[i].x |= b.w[i].x; a.w[i].y |= b.w[i].y; }
    if (OP == OP_XOR) { a.w[i].x ^= b.w[i].x; a.w[i].y ^= b.w[i].y; }
    if (OP == OP_ANDNOT) { a.w[i].x &= ~b.w[i].x; a.w[i].y &= ~b.w[i].y; }
  }
}

// Per-wave scratch in LDS.
struct WaveScratch {
  uint64_t lb[1024];          // 8 KiB expansion bitmap
  int64_t meta[MAXLEAF][16];  // container meta word per (leaf, j), -1 absent
};

// Build the (leaf, key) meta table for query `qp` in shard `s`; returns the
// presence mask of each leaf in `mask[]` (wave-uniform).  Lanes take
// (leaf, container) pairs -- 4 leaves per pass, passes unrolled -- so the
// rowptr and meta loads of all leaves are in flight together instead of one
// leaf's dependent chain after the other's; the key loops then read metas
// from LDS, not global memory.
__device__ __forceinline__ void build_slots(const QueryProg& qp, const ViewDev* views, int s, WaveScratch& ws,
                                            uint32_t* mask) {
  const int lane = wave_lane();
  for (int t = lane; t < MAXLEAF * 16; t += 64) (&ws.meta[0][0])[t] = -1;
  lds_fence();
  const int nleaf = qp.nleaf;
#pragma unroll
  for (int k0 = 0; k0 < MAXLEAF; k0 += 4) {
    const int k = k0 + (lane >> 4), idx = lane & 15;
    if (k0 < nleaf && k < nleaf) {
      const int64_t d = qp.leaf_row[k];
      if (d >= 0) {
        const ViewDev& v = views[qp.leaf_view[k]];
        const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
        const int64_t base = v.shard_base[s];
        const int64_t lo = base + rp[d], hi = base + rp[d + 1];
        if (idx < hi - lo) {
          const int64_t m = v.meta[lo + idx];
          ws.meta[k][meta_j(m)] = m;
        }
      }
    }
  }
  lds_fence();
  for (int k0 = 0; k0 < MAXLEAF; k0 += 4) {
    const int k = k0 + (lane >> 4);
    const bool has = ws.meta[k][lane & 15] >= 0;
    const uint64_t b = __ballot(has);
#pragma unroll
    for (int i = 0; i < 4; i++) mask[k0 + i] = uint32_t((b >> (16 * i)) & 0xffff);
  }
}

// Candidate keys: evaluate the program over presence masks.
__device__ __forceinline__ uint32_t candidate_mask(const QueryProg& qp, const uint32_t* mask) {
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;  // s0 = top
  for (int pc = 0; pc < qp.nprog; pc++) {
    const int op = qp.prog[pc];
    if (op < OP_AND) {
      s3 = s2; s2 = s1; s1 = s0; s0 = mask[op];
    } else {
      uint32_t r;
      if (op == OP_AND) r = s1 & s0;
      else if (op == OP_ANDNOT) r = s1;
      else r = s1 | s0;  // OR, XOR
      s0 = r; s1 = s2; s2 = s3; s3 = 0;
    }
  }
  return s0;
}

// Evaluate the program for key j into `acc`.
__device__ __forceinline__ void eval_tile(const QueryProg& qp, const ViewDev* views, int s, int j, WaveScratch& ws,
                                          Tile& acc) {
  Tile t1, t2, t3;
  tile_zero(acc);
  tile_zero(t1);
  tile_zero(t2);
  tile_zero(t3);
  for (int pc = 0; pc < qp.nprog; pc++) {
    const int op = qp.prog[pc];
    if (op < OP_AND) {
      t3 = t2; t2 = t1; t1 = acc;
      const int64_t m = ws.meta[op][j];
      if (m < 0) tile_zero(acc);
      else tile_load(acc, views[qp.leaf_view[op]].payload, m, ws.lb);
    } else {
      // acc = t1 OP acc
      if (op == OP_AND) { tile_op<OP_AND>(t1, acc); }
      else if (op == OP_OR) { tile_op<OP_OR>(t1, acc); }
      else if (op == OP_XOR) { tile_op<OP_XOR>(t1, acc); }
      else { tile_op<OP_ANDNOT>(t1, acc); }
      acc = t1; t1 = t2; t2 = t3; tile_zero(t3);
    }
  }
}

// Count array values whose bit is set in the 1024-word bitmap `bm` (global or
// LDS); 16-byte loads of 8 values per lane.
__device__ __forceinline__ int probe_array(const uint64_t* bm, const uint16_t* arr, int n) {
  const int lane = wave_lane();
  const uint4* p4 = reinterpret_cast<const uint4*>(arr);
  const int n8 = (n + 7) >> 3;
  int c = 0;
  for (int e8 = lane; e8 < n8; e8 += 64) {
    const uint4 v4 = p4[e8];
    const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (w[k >> 1] >> ((k & 1) * 16)) & 0xffff;
      const int hit = int((bm[v >> 6] >> (v & 63)) & 1);
      c += (e8 * 8 + k < n) ? hit : 0;
    }
  }
  return c;
}

// |A ∩ B| for two containers with a type-pair dispatch (no full tiles for arrays).
__device__ __forceinline__ int and2_count(const ViewDev& va, int64_t ma, const ViewDev& vb, int64_t mb,
                                          uint64_t* lb) {
  const int lane = wave_lane();
  const int ta = meta_type(ma), tb = meta_type(mb);
  int c = 0;
  if (ta == CT_BITMAP && tb == CT_BITMAP) {
    const ulong2* pa = reinterpret_cast<const ulong2*>(va.payload + meta_off16(ma) * 8);
    const ulong2* pb = reinterpret_cast<const ulong2*>(vb.payload + meta_off16(mb) * 8);
    ulong2 x[8], y[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = pa[i * 64 + lane];
#pragma unroll
    for (int i = 0; i < 8; i++) y[i] = pb[i * 64 + lane];
#pragma unroll
    for (int i = 0; i < 8; i++) c += __popcll(x[i].x & y[i].x) + __popcll(x[i].y & y[i].y);
    return c;
  }
  if (ta == CT_RUN || tb == CT_RUN) {
    Tile a, b;
    tile_load(a, va.payload, ma, lb);
    tile_load(b, vb.payload, mb, lb);
    tile_op<OP_AND>(a, b);
    return tile_popc(a);
  }
  if (ta == CT_BITMAP || tb == CT_BITMAP) {
    // probe the bitmap with the array values; large arrays first stage the
    // 8 KiB bitmap into LDS with coalesced 16 B loads (random 8 B global
    // probes would touch every line anyway).
    const bool abit = ta == CT_BITMAP;
    const uint64_t* bw = reinterpret_cast<const uint64_t*>((abit ? va.payload : vb.payload) +
                                                           meta_off16(abit ? ma : mb) * 8);
    const int64_t am = abit ? mb : ma;
    const uint16_t* arr = (abit ? vb.payload : va.payload) + meta_off16(am) * 8;
    const int n = meta_n(am);
    const uint64_t* probe = bw;
    if (n >= 256) {
      const ulong2* src = reinterpret_cast<const ulong2*>(bw);
      ulong2* l2 = reinterpret_cast<ulong2*>(lb);
      ulong2 t[8];
#pragma unroll
      for (int i = 0; i < 8; i++) t[i] = src[i * 64 + lane];
#pragma unroll
      for (int i = 0; i < 8; i++) l2[i * 64 + lane] = t[i];
      lds_fence();
      probe = lb;
    }
    c = probe_array(probe, arr, n);
    if (n >= 256) lds_fence();
    return c;
  }
  // array & array: scatter the larger into LDS, probe with the smaller
  const bool abig = meta_n(ma) >= meta_n(mb);
  const int64_t mbig = abig ? ma : mb, msmall = abig ? mb : ma;
  const ViewDev& vbig = abig ? va : vb;
  const ViewDev& vsmall = abig ? vb : va;
  lds_expand(lb, vbig.payload, mbig);
  c = probe_array(lb, vsmall.payload + meta_off16(msmall) * 8, meta_n(msmall));
  lds_fence();
  return c;
}

constexpr int WAVES_PER_BLOCK = 4;

// Count kernel: out[q] += |program(q)| over all local shards.
// MODE 1 (fast) handles only Count(Row) and Count(Intersect(a,b)) programs
// (no register tile stack -> far fewer VGPRs, higher occupancy); MODE 2
// (flat) handles left folds "l0 l1 op l2 op ..." (Union/Intersect/Difference/
// Xor of leaves, time-range view unions, Not) with one accumulator tile and
// one load tile; MODE 0 interprets any program with the 4-deep tile stack.

// Flat fold: acc = l0; acc = acc op_i l_i.
__device__ __forceinline__ void load_leaf(const QueryProg& qp, const ViewDev* views, int s, int j, WaveScratch& ws,
                                          int k, Tile& t) {
  const int64_t m = ws.meta[k][j];
  if (m < 0) tile_zero(t);
  else tile_load(t, views[qp.leaf_view[k]].payload, m, ws.lb);
}

__device__ __forceinline__ void eval_flat(const QueryProg& qp, const ViewDev* views, int s, int j, WaveScratch& ws,
                                          Tile& acc) {
  load_leaf(qp, views, s, j, ws, qp.prog[0], acc);
  for (int pc = 1; pc + 1 < qp.nprog; pc += 2) {
    Tile t;
    load_leaf(qp, views, s, j, ws, qp.prog[pc], t);
    const int op = qp.prog[pc + 1];
    if (op == OP_AND) tile_op<OP_AND>(acc, t);
    else if (op == OP_OR) tile_op<OP_OR>(acc, t);
    else if (op == OP_XOR) tile_op<OP_XOR>(acc, t);
    else tile_op<OP_ANDNOT>(acc, t);
  }
}

template <int MODE>
__global__ __launch_bounds__(256, MODE == 0 ? 1 : 4) void expr_count_kernel(const QueryProg* __restrict__ progs, int Q,
                                                         const ViewDev* __restrict__ views, int S,
                                                         unsigned long long* __restrict__ out,
                                                         int32_t* __restrict__ per_key,
                                                         int64_t* __restrict__ per_shard) {
  __shared__ WaveScratch scratch[WAVES_PER_BLOCK];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  if (item >= int64_t(Q) * S) return;
  const int q = int(item % Q);
  const int s = int(item / Q);
  const QueryProg& qp = progs[q];
  WaveScratch& ws = scratch[wave];
  uint32_t mask[MAXLEAF];
  build_slots(qp, views, s, ws, mask);
  const uint32_t cand = candidate_mask(qp, mask);
  int64_t total = 0;
  if (cand) {
    if (qp.nprog == 1) {
      // Count(Row): metadata only
      if (lane < 16 && ((cand >> lane) & 1)) {
        const int n = meta_n(ws.meta[0][lane]);
        total = n;
        if (per_key) per_key[(int64_t(q) * S + s) * 16 + lane] = n;
      }
    } else if (MODE == 1) {
      // Count(Intersect(leaf0, leaf1)) with a container type-pair dispatch
      const ViewDev& va = views[qp.leaf_view[0]];
      const ViewDev& vb = views[qp.leaf_view[1]];
      for (uint32_t cm = cand; cm; cm &= cm - 1) {
        const int j = __builtin_ctz(cm);
        const int64_t ma = ws.meta[0][j];
        const int64_t mb = ws.meta[1][j];
        total += and2_count(va, ma, vb, mb, ws.lb);
      }
    } else {
      for (uint32_t cm = cand; cm; cm &= cm - 1) {
        const int j = __builtin_ctz(cm);
        Tile acc;
        if (MODE == 2) eval_flat(qp, views, s, j, ws, acc);
        else eval_tile(qp, views, s, j, ws, acc);
        int c = tile_popc(acc);
        if (per_key) {
          const int64_t cj = wave_sum_i64(c);
          if (lane == 0) per_key[(int64_t(q) * S + s) * 16 + j] = int32_t(cj);
        }
        total += c;
      }
    }
  }
  total = wave_sum_i64(total);
  if (lane == 0 && total && out) atomicAdd(out + q, (unsigned long long)total);
  if (lane == 0 && per_shard) per_shard[int64_t(q) * S + s] = total;
}

// Union count (MODE 3 of launch_expr_count): Count(Union(l0, l1, ...)) of
// plain leaves, e.g. the covering time views of Row(t=r, from, to)
// (reference executeRowShard unions the views, executor.go:1444-1533).  Per
// key the wave clears one LDS bitmap and ORs every leaf container into it
// with returning LDS atomics; a bit counts when its OR flips it
// (popcount(mask & ~old)), so no tile is expanded, combined or read back --
// for the small arrays of time views that is most of the work.
__global__ __launch_bounds__(256) void union_count_kernel(const QueryProg* __restrict__ progs, int Q,
                                                          const ViewDev* __restrict__ views, int S,
                                                          unsigned long long* __restrict__ out) {
  __shared__ WaveScratch scratch[WAVES_PER_BLOCK];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  if (item >= int64_t(Q) * S) return;
  const int q = int(item % Q);
  const int s = int(item / Q);
  const QueryProg& qp = progs[q];
  WaveScratch& ws = scratch[wave];
  uint32_t mask[MAXLEAF];
  build_slots(qp, views, s, ws, mask);
  uint32_t cand = 0;
  for (int k = 0; k < qp.nleaf; k++) cand |= mask[k];
  unsigned long long* lb64 = reinterpret_cast<unsigned long long*>(ws.lb);
  uint32_t* lb32 = reinterpret_cast<uint32_t*>(ws.lb);
  int64_t total = 0;
  for (uint32_t cm = cand; cm; cm &= cm - 1) {
    const int j = __builtin_ctz(cm);
    ulong2* l2 = reinterpret_cast<ulong2*>(ws.lb);
#pragma unroll
    for (int i = 0; i < 8; i++) l2[i * 64 + lane] = make_ulong2(0, 0);
    lds_fence();
    for (int k = 0; k < qp.nleaf; k++) {
      const int64_t m = ws.meta[k][j];
      if (m < 0) continue;
      const ViewDev& v = views[qp.leaf_view[k]];
      const uint16_t* p = v.payload + meta_off16(m) * 8;
      const int type = meta_type(m);
      if (type == CT_BITMAP) {
        const ulong2* g = reinterpret_cast<const ulong2*>(p);
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const ulong2 w = g[i * 64 + lane];
          const int wi = 2 * (i * 64 + lane);
          const unsigned long long ox = atomicOr(lb64 + wi, (unsigned long long)w.x);
          const unsigned long long oy = atomicOr(lb64 + wi + 1, (unsigned long long)w.y);
          total += __popcll(w.x & ~ox) + __popcll(w.y & ~oy);
        }
      } else if (type == CT_ARRAY) {
        const int n = meta_n(m);
        const uint4* p4 = reinterpret_cast<const uint4*>(p);
        for (int e8 = lane; e8 < ((n + 7) >> 3); e8 += 64) {
          const uint4 v4 = p4[e8];
          const uint32_t w4[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
          for (int t = 0; t < 8; t++) {
            if (e8 * 8 + t < n) {
              const uint32_t x = (w4[t >> 1] >> ((t & 1) * 16)) & 0xffff;
              const uint32_t bit = 1u << (x & 31);
              total += (atomicOr(lb32 + (x >> 5), bit) & bit) ? 0 : 1;
            }
          }
        }
      } else {
        const int nr = p[0];
        for (int r = lane; r < nr; r += 64) {
          const uint32_t st = p[8 + 2 * r], e = uint32_t(p[9 + 2 * r]) + 1;
          for (uint32_t w = st >> 6; w <= (e - 1) >> 6; w++) {
            uint64_t mk = ~0ull;
            if (w == (st >> 6)) mk &= ~0ull << (st & 63);
            if (w == ((e - 1) >> 6) && (e & 63)) mk &= (1ull << (e & 63)) - 1;
            total += __popcll(mk & ~atomicOr(lb64 + w, (unsigned long long)mk));
          }
        }
      }
    }
    lds_fence();
  }
  total = wave_sum_i64(total);
  if (lane == 0 && total) atomicAdd(out + q, (unsigned long long)total);
}

// Union count v2 (MODE 4, the default for Count(Union(leaves))).  v1 above
// walks the leaves of a key one after the other: slot (LDS) -> meta (global)
// -> payload (global) -> returning LDS atomics, i.e. two dependent global
// round trips per (leaf, key), ~7x16 of them in series per (query, shard) for
// a YMDH time range.  Here
//   * the metas of every (leaf, key) are fetched in one parallel round trip
//     (lane = (leaf, container) pair) into a wave-private LDS table;
//   * per key, the present leaves' payloads are walked as ONE flat list of
//     16-byte chunks (array: 8 values, bitmap: 2 words), so the loads of all
//     leaves are in flight together (4 per lane per step); a lane finds its
//     chunk's leaf by comparing with the leaves' chunk prefix (scalar
//     readlanes) and fetches the leaf's meta / payload pointer with bpermutes;
//   * values are OR-ed into the LDS bitmap with NON-returning ds_or, and the
//     key's union is counted by one popcount pass that also re-zeroes it;
//   * a key present in one leaf only is counted from its metadata.
// Run containers (rare in time views) are OR-ed in a second, per-run loop.
__device__ __forceinline__ int shfl_i32(int v, int src) { return __shfl(v, src); }
__device__ __forceinline__ int64_t shfl_i64(int64_t v, int src) {
  const int lo = __shfl(int(uint64_t(v)), src), hi = __shfl(int(uint64_t(v) >> 32), src);
  return int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
}

__global__ __launch_bounds__(256) void union_count2_kernel(const QueryProg* __restrict__ progs, int Q,
                                                           const ViewDev* __restrict__ views, int S,
                                                           unsigned long long* __restrict__ out) {
  __shared__ uint32_t lbits[WAVES_PER_BLOCK][2048];
  __shared__ int64_t lmeta[WAVES_PER_BLOCK][MAXLEAF * 16];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  if (item >= int64_t(Q) * S) return;
  const int q = int(item % Q);
  const int s = int(item / Q);
  const QueryProg& qp = progs[q];
  const int nleaf = qp.nleaf;
  uint32_t* lb = lbits[wave];
  int64_t* mt = lmeta[wave];
  for (int t = lane; t < MAXLEAF * 16; t += 64) mt[t] = -1;
  {
    uint4* lb4 = reinterpret_cast<uint4*>(lb);
#pragma unroll
    for (int i = 0; i < 8; i++) lb4[i * 64 + lane] = make_uint4(0, 0, 0, 0);
  }
  lds_fence();
  // (leaf, container) metas: lane -> leaf k0 + lane/16, container lane%16
#pragma unroll
  for (int k0 = 0; k0 < MAXLEAF; k0 += 4) {
    const int k = k0 + (lane >> 4), idx = lane & 15;
    if (k0 < nleaf && k < nleaf) {
      const int64_t d = qp.leaf_row[k];
      if (d >= 0) {
        const ViewDev& v = views[qp.leaf_view[k]];
        const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
        const int64_t base = v.shard_base[s];
        const int64_t lo = base + rp[d], hi = base + rp[d + 1];
        if (idx < hi - lo) {
          const int64_t m = v.meta[lo + idx];
          mt[k * 16 + meta_j(m)] = m;
        }
      }
    }
  }
  lds_fence();
  bool has = false;
  if (lane < 16)
    for (int k = 0; k < nleaf; k++) has |= mt[k * 16 + lane] >= 0;
  const uint32_t cand = uint32_t(__ballot(has) & 0xffff);
  // per-leaf payload base pointer (lane k < nleaf)
  const uint16_t* lpay = lane < nleaf ? views[qp.leaf_view[lane]].payload : nullptr;
  int64_t total = 0;
  unsigned long long* lb64 = reinterpret_cast<unsigned long long*>(lb);
  for (uint32_t cm = cand; cm; cm &= cm - 1) {
    const int j = __builtin_ctz(cm);
    const int64_t m = lane < nleaf ? mt[lane * 16 + j] : -1;
    const uint64_t pres = __ballot(m >= 0);
    if (__popcll(pres) == 1) {  // one leaf holds this key: its cardinality
      if (lane == __builtin_ctzll(pres)) total += meta_n(m);
      continue;
    }
    const int type = m >= 0 ? meta_type(m) : -1;
    const int cnt = type == CT_ARRAY ? (meta_n(m) + 7) >> 3 : (type == CT_BITMAP ? 512 : 0);
    // inclusive scan of chunk counts over lanes 0..15
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const int t = __shfl_up(incl, d);
      if ((lane & 15) >= d) incl += t;
    }
    const int pre = incl - cnt;
    const int tot = __builtin_amdgcn_readlane(incl, 15);
    const uint16_t* lptr = (m >= 0) ? lpay + meta_off16(m) * 8 : nullptr;
    for (int c0 = 0; c0 < tot; c0 += 256) {
      int c[4], leaf[4];
#pragma unroll
      for (int u = 0; u < 4; u++) { c[u] = c0 + u * 64 + lane; leaf[u] = 0; }
      for (int k = 1; k < nleaf; k++) {
        const int pk = __builtin_amdgcn_readlane(pre, k);
#pragma unroll
        for (int u = 0; u < 4; u++) leaf[u] += c[u] >= pk;
      }
      uint4 v[4];
      int64_t mm[4];
      int loc[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        mm[u] = shfl_i64(m, leaf[u]);
        loc[u] = c[u] - shfl_i32(pre, leaf[u]);
        const uint4* p = reinterpret_cast<const uint4*>(shfl_i64(int64_t(lptr), leaf[u]));
        if (c[u] < tot) v[u] = p[loc[u]];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (c[u] >= tot) continue;
        if (meta_type(mm[u]) == CT_BITMAP) {
          atomicOr(lb64 + 2 * loc[u], (unsigned long long)(uint64_t(v[u].y) << 32 | v[u].x));
          atomicOr(lb64 + 2 * loc[u] + 1, (unsigned long long)(uint64_t(v[u].w) << 32 | v[u].z));
        } else {
          const int n = meta_n(mm[u]);
          const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int t = 0; t < 8; t++) {
            const uint32_t x = (w4[t >> 1] >> ((t & 1) * 16)) & 0xffff;
            if (loc[u] * 8 + t < n) atomicOr(lb + (x >> 5), 1u << (x & 31));
          }
        }
      }
    }
    // run containers of this key
    uint64_t runs = __ballot(type == CT_RUN);
    for (; runs; runs &= runs - 1) {
      const int k = __builtin_ctzll(runs);
      const uint16_t* p = reinterpret_cast<const uint16_t*>(shfl_i64(int64_t(lptr), k));
      const int nr = p[0];
      for (int r = lane; r < nr; r += 64) {
        const uint32_t st = p[8 + 2 * r], e = uint32_t(p[9 + 2 * r]) + 1;
        for (uint32_t w = st >> 6; w <= (e - 1) >> 6; w++) {
          uint64_t mk = ~0ull;
          if (w == (st >> 6)) mk &= ~0ull << (st & 63);
          if (w == ((e - 1) >> 6) && (e & 63)) mk &= (1ull << (e & 63)) - 1;
          atomicOr(lb64 + w, (unsigned long long)mk);
        }
      }
    }
    lds_fence();
    uint4* lb4 = reinterpret_cast<uint4*>(lb);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint4 w = lb4[i * 64 + lane];
      total += __popc(w.x) + __popc(w.y) + __popc(w.z) + __popc(w.w);
      lb4[i * 64 + lane] = make_uint4(0, 0, 0, 0);
    }
    lds_fence();
  }
  total = wave_sum_i64(total);
  if (lane == 0 && total) atomicAdd(out + q, (unsigned long long)total);
}

// Materialize kernel: writes result containers for every (q, s, j) with
// counts[q,s,j] > 0 at u16 offset offs[q,s,j]; array if n <= 4096 else bitmap.
__global__ __launch_bounds__(256) void expr_materialize_kernel(const QueryProg* __restrict__ progs, int Q,
                                                               const ViewDev* __restrict__ views, int S,
                                                               const int32_t* __restrict__ counts,
                                                               const int64_t* __restrict__ offs,
                                                               uint16_t* __restrict__ outp) {
  __shared__ WaveScratch scratch[WAVES_PER_BLOCK];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  if (item >= int64_t(Q) * S) return;
  const int q = int(item % Q);
  const int s = int(item / Q);
  const QueryProg& qp = progs[q];
  WaveScratch& ws = scratch[wave];
  uint32_t mask[MAXLEAF];
  build_slots(qp, views, s, ws, mask);
  const uint32_t cand = candidate_mask(qp, mask);
  for (uint32_t cm = cand; cm; cm &= cm - 1) {
    const int j = __builtin_ctz(cm);
    const int64_t key = (int64_t(q) * S + s) * 16 + j;
    const int n = counts[key];
    if (n <= 0) continue;
    Tile acc;
    eval_tile(qp, views, s, j, ws, acc);
    uint16_t* dst = outp + offs[key];
    if (n > ARRAY_MAX) {
      ulong2* d2 = reinterpret_cast<ulong2*>(dst);
#pragma unroll
      for (int i = 0; i < 8; i++) d2[i * 64 + lane] = acc.w[i];
    } else {
      // ordered compaction: chunk i covers words [128i, 128i+128), lane l owns
      // words 128i+2l, 128i+2l+1 -> exclusive wave scan of per-lane popcounts.
      int base = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint64_t x = acc.w[i].x, y = acc.w[i].y;
        const int c = __popcll(x) + __popcll(y);
        int incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        int pos = base + incl - c;
        const int wbase = 128 * i + 2 * lane;
        for (uint64_t b = x; b; b &= b - 1) dst[pos++] = uint16_t(wbase * 64 + __builtin_ctzll(b));
        for (uint64_t b = y; b; b &= b - 1) dst[pos++] = uint16_t((wbase + 1) * 64 + __builtin_ctzll(b));
        base += __shfl(incl, 63, 64);
      }
    }
  }
}

// Dense evaluation: every (q, s, j) result tile is written as a bitmap
// container at the fixed u16 offset ((q*S + s)*16 + j) * 4096 of `outp`, with
// its metadata word (key j, bitmap, n, offset) in out_meta.  The result is a
// one-row device view per query whose shard layout matches the inputs; Shift
// (row_kernels.hip) reads it back word-addressed.
__global__ __launch_bounds__(256) void expr_dense_kernel(const QueryProg* __restrict__ progs, int Q,
                                                         const ViewDev* __restrict__ views, int S,
                                                         uint16_t* __restrict__ outp, int64_t* __restrict__ out_meta) {
  __shared__ WaveScratch scratch[WAVES_PER_BLOCK];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  if (item >= int64_t(Q) * S) return;
  const int q = int(item % Q);
  const int s = int(item / Q);
  const QueryProg& qp = progs[q];
  WaveScratch& ws = scratch[wave];
  uint32_t mask[MAXLEAF];
  build_slots(qp, views, s, ws, mask);
  const uint32_t cand = candidate_mask(qp, mask);
  for (int j = 0; j < 16; j++) {
    const int64_t key = (int64_t(q) * S + s) * 16 + j;
    Tile acc;
    if ((cand >> j) & 1) eval_tile(qp, views, s, j, ws, acc);
    else tile_zero(acc);
    ulong2* d2 = reinterpret_cast<ulong2*>(outp + key * 4096);
#pragma unroll
    for (int i = 0; i < 8; i++) d2[i * 64 + lane] = acc.w[i];
    const int64_t n = wave_sum_i64(tile_popc(acc));
    if (lane == 0) out_meta[key] = int64_t(j) | (int64_t(CT_BITMAP) << 4) | (n << 6) | ((key * 512) << 23);
  }
}

// BSI sum over bit-sliced rows (fragment.go:1109-1141):
//   consider = exists & filter ; count = |consider|
//   sum = Σ_i 2^i (|B_i & consider & ~sign| - |B_i & consider & sign|)
// The host resolves the BSI view's rows 0 (exists), 1 (sign) and 2+i (bit i)
// to dense row indices (bsi.row_exists / row_sign / bit_row[i], -1 = absent).
__global__ __launch_bounds__(256) void bsi_sum_kernel(const QueryProg* __restrict__ progs, int Q,
                                                      const ViewDev* __restrict__ views, int S, BsiArgs bsi,
                                                      unsigned long long* __restrict__ out_sum,
                                                      unsigned long long* __restrict__ out_cnt) {
  __shared__ WaveScratch scratch[WAVES_PER_BLOCK];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  if (item >= int64_t(Q) * S) return;
  const int q = int(item % Q);
  const int s = int(item / Q);
  const QueryProg& qp = progs[q];  // filter program (nprog == 0: no filter)
  WaveScratch& ws = scratch[wave];
  const ViewDev& bv = views[bsi.view];
  uint32_t mask[MAXLEAF];
  build_slots(qp, views, s, ws, mask);
  uint32_t cand = qp.nprog ? candidate_mask(qp, mask) : 0xffffu;
  // exists row presence
  const uint32_t* rp = bv.rowptr + int64_t(s) * (bv.D + 1);
  const int64_t base = bv.shard_base[s];
  auto row_range = [&](int64_t d, int64_t& lo, int64_t& hi) {
    if (d < 0) { lo = hi = 0; return; }
    lo = rp[d]; hi = rp[d + 1];
  };
  auto find_j = [&](int64_t d, int j) -> int64_t {
    // container of dense row d at key j in this shard (or -1); wave-uniform
    int64_t lo, hi;
    row_range(d, lo, hi);
    int64_t found = -1;
    if (lane < hi - lo) {
      if (meta_j(bv.meta[base + lo + lane]) == j) found = base + lo + lane;
    }
    const uint64_t b = __ballot(found >= 0);
    if (!b) return -1;
    return rl_i64(found, int(__builtin_ctzll(b)));
  };
  int64_t lo_e, hi_e;
  row_range(bsi.row_exists, lo_e, hi_e);
  uint32_t emask = 0;
  {
    int64_t j = -1;
    if (lane < hi_e - lo_e) j = meta_j(bv.meta[base + lo_e + lane]);
    for (int t = 0; t < 16; t++) emask |= (__ballot(j == t) ? 1u : 0u) << t;
  }
  cand &= emask;
  int64_t acc_sum = 0, acc_cnt = 0;
  for (uint32_t cm = cand; cm; cm &= cm - 1) {
    const int j = __builtin_ctz(cm);
    Tile consider, sign, bits;
    tile_load(consider, bv.payload, bv.meta[find_j(bsi.row_exists, j)], ws.lb);
    if (qp.nprog) {
      Tile f;
      eval_tile(qp, views, s, j, ws, f);
      tile_op<OP_AND>(consider, f);
    }
    acc_cnt += tile_popc(consider);
    const int64_t cs = find_j(bsi.row_sign, j);
    if (cs >= 0) tile_load(sign, bv.payload, bv.meta[cs], ws.lb);
    else tile_zero(sign);
    for (int i = 0; i < bsi.depth; i++) {
      const int64_t cb = find_j(bsi.bit_row[i], j);
      if (cb < 0) continue;
      tile_load(bits, bv.payload, bv.meta[cb], ws.lb);
      int pc = 0, nc = 0;
#pragma unroll
      for (int w = 0; w < 8; w++) {
        const uint64_t bx = bits.w[w].x & consider.w[w].x, by = bits.w[w].y & consider.w[w].y;
        pc += __popcll(bx & ~sign.w[w].x) + __popcll(by & ~sign.w[w].y);
        nc += __popcll(bx & sign.w[w].x) + __popcll(by & sign.w[w].y);
      }
      acc_sum += int64_t(uint64_t(int64_t(pc - nc)) << i);
    }
  }
  acc_sum = wave_sum_i64(acc_sum);
  acc_cnt = wave_sum_i64(acc_cnt);
  if (lane == 0) {
    if (acc_sum) atomicAdd(out_sum + q, (unsigned long long)acc_sum);
    if (acc_cnt) atomicAdd(out_cnt + q, (unsigned long long)acc_cnt);
  }
}

// BSI sum, key-parallel (default): one wave per (shard, key, query), the
// queries of one (shard, key) on consecutive waves of one XCD so the bit
// planes they all read are shared through its L2.  Lanes first resolve the
// container of every bit plane at this key in parallel (lane i: plane i), so
// the plane loop issues its tile loads without a dependent metadata walk.
// FMODE: 0 no filter, 1 flat-fold filter (two tiles), 2 any program (tile stack).
template <int FMODE>
__global__ __launch_bounds__(256) void bsi_sum_keys_kernel(const QueryProg* __restrict__ progs, int Q,
                                                           const ViewDev* __restrict__ views, int S, BsiArgs bsi,
                                                           unsigned long long* __restrict__ out_sum,
                                                           unsigned long long* __restrict__ out_cnt) {
  __shared__ WaveScratch scratch[WAVES_PER_BLOCK];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  const bool live = item < int64_t(Q) * S * 16;
  const int q = live ? int(item % Q) : -1;
  // the wave's (sum, count); the block folds its waves' results into one
  // atomic pair per query: 15k waves hitting the same two words serialise
  // at one L2 channel
  int64_t tsum = 0, tcnt = 0;
  auto work = [&]() {
    const int j = int((item / Q) & 15);
    const int s = int(item / (int64_t(Q) * 16));
    const QueryProg& qp = progs[q];
    WaveScratch& ws = scratch[wave];
    const ViewDev& bv = views[bsi.view];
    const uint32_t* rp = bv.rowptr + int64_t(s) * (bv.D + 1);
    const int64_t base = bv.shard_base[s];
    // container index of dense row d at key j (or -1), evaluated per lane
    auto lane_find = [&](int64_t d) -> int64_t {
      if (d < 0) return -1;
      const int64_t lo = base + rp[d], hi = base + rp[d + 1];
      if (hi - lo == 16) return lo + j;   // every key present (dense planes): no meta walk
      for (int64_t c = lo; c < hi; c++)
        if (meta_j(bv.meta[c]) == j) return c;
      return -1;
    };
    // lane i < depth (<= 63): bit plane i; lanes 0 / 1 then resolve exists /
    // sign in a second parallel lookup
    const int64_t mine = lane < bsi.depth ? lane_find(bsi.bit_row[lane]) : -1;
    const int64_t extra = lane == 0 ? lane_find(bsi.row_exists) : (lane == 1 ? lane_find(bsi.row_sign) : -1);
    const int64_t ce = rl_i64(extra, 0);
    if (ce < 0) return;
    Tile consider, sign, bits;
    tile_load(consider, bv.payload, bv.meta[ce], ws.lb);
    if (FMODE != 0 && qp.nprog) {
      uint32_t mask[MAXLEAF];
      build_slots(qp, views, s, ws, mask);
      if (!((candidate_mask(qp, mask) >> j) & 1)) return;
      Tile f;
      if (FMODE == 1) eval_flat(qp, views, s, j, ws, f);
      else eval_tile(qp, views, s, j, ws, f);
      tile_op<OP_AND>(consider, f);
    }
    const int64_t acc_cnt = tile_popc(consider);
    const int64_t cs = rl_i64(extra, 1);
    if (cs >= 0) tile_load(sign, bv.payload, bv.meta[cs], ws.lb);
    else tile_zero(sign);
    // consider splits into its non-negative and negative columns once per key
    // (consider <- consider & ~sign, sign <- consider & sign); a key with no
    // negative column (the usual case: the sign row is sparse) then counts one
    // AND + popcount per plane word instead of two
    uint64_t anyneg = 0;
  #pragma unroll
    for (int w = 0; w < 8; w++) {
      const ulong2 c = consider.w[w], g = sign.w[w];
      consider.w[w] = make_ulong2(c.x & ~g.x, c.y & ~g.y);
      sign.w[w] = make_ulong2(c.x & g.x, c.y & g.y);
      anyneg |= sign.w[w].x | sign.w[w].y;
    }
    const bool neg = __ballot(anyneg != 0) != 0;
    int64_t acc_sum = 0;
    // planes double-buffered: the next present plane's tile is in flight
    // while the current one is counted (one load round trip per plane, not
    // a wait before every plane)
    const uint64_t present = __ballot(mine >= 0) & (bsi.depth >= 64 ? ~0ull : ((1ull << bsi.depth) - 1));
    auto count_plane = [&](const Tile& t, int i) {
      int pc = 0, nc = 0;
  #pragma unroll
      for (int w = 0; w < 8; w++) pc += __popcll(t.w[w].x & consider.w[w].x) + __popcll(t.w[w].y & consider.w[w].y);
      if (neg) {
  #pragma unroll
        for (int w = 0; w < 8; w++) nc += __popcll(t.w[w].x & sign.w[w].x) + __popcll(t.w[w].y & sign.w[w].y);
      }
      acc_sum += int64_t(uint64_t(int64_t(pc - nc)) << i);
    };
    Tile bits2;
    uint64_t left = present;
    int cur = left ? __builtin_ctzll(left) : -1;
    if (cur >= 0) {
      left &= left - 1;
      tile_load(bits, bv.payload, bv.meta[rl_i64(mine, cur)], ws.lb);
    }
    while (cur >= 0) {
      int nxt = left ? __builtin_ctzll(left) : -1;
      if (nxt >= 0) {
        left &= left - 1;
        tile_load(bits2, bv.payload, bv.meta[rl_i64(mine, nxt)], ws.lb);
      }
      count_plane(bits, cur);
      cur = nxt;
      if (cur < 0) break;
      nxt = left ? __builtin_ctzll(left) : -1;
      if (nxt >= 0) {
        left &= left - 1;
        tile_load(bits, bv.payload, bv.meta[rl_i64(mine, nxt)], ws.lb);
      }
      count_plane(bits2, cur);
      cur = nxt;
    }
    tsum = wave_sum_i64(acc_sum);
    tcnt = wave_sum_i64(acc_cnt);
  };
  if (live) work();
  __shared__ long long red_s[WAVES_PER_BLOCK], red_c[WAVES_PER_BLOCK];
  __shared__ int red_q[WAVES_PER_BLOCK];
  if (lane == 0) {
    red_s[wave] = tsum;
    red_c[wave] = tcnt;
    red_q[wave] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 0; w < WAVES_PER_BLOCK; w++) {
      const int qw = red_q[w];
      if (qw < 0) continue;
      long long ss = red_s[w], cc = red_c[w];
      for (int w2 = w + 1; w2 < WAVES_PER_BLOCK; w2++)
        if (red_q[w2] == qw) {
          ss += red_s[w2];
          cc += red_c[w2];
          red_q[w2] = -1;
        }
      if (ss) atomicAdd(out_sum + qw, (unsigned long long)ss);
      if (cc) atomicAdd(out_cnt + qw, (unsigned long long)cc);
    }
  }
}

// ---------------------------------------------------------------- BSI range
// Bit-sliced comparators (O'Neil), reference fragment.go:1271-1534, with the
// exact control flow of pilosa_amd/models/fragment.py (_range_eq/_lt/_gt/
// _between).  One wave per (shard, key): the predicate result of that
// container is built in registers from the exists/sign/bit-slice tiles and
// written as a bitmap container of a temporary device view, which ordinary
// expression programs then consume as a leaf (Count(Intersect(Row(f=1),
// Row(v > 10))) = one range launch + one count launch).

struct BsiCtx {
  const BsiArgs& bsi;
  const ViewDev& bv;
  int s;
  int j;
  int64_t base;
  const uint32_t* rp;
  uint64_t* lb;
  // lane i < depth (<= 63): container of bit plane i at key j (-1 = absent),
  // resolved once, in parallel, by plane_index().
  int64_t planes = -1;
};

// Every lane resolves one BSI row's container at (s, j): the plane loops then
// broadcast it with readlanes instead of a dependent ballot walk per plane.
__device__ __forceinline__ void plane_index(BsiCtx& c) {
  const int lane = wave_lane();
  const int64_t d = lane < c.bsi.depth ? c.bsi.bit_row[lane] : -1;
  int64_t found = -1;
  if (d >= 0) {
    const int64_t lo = c.base + c.rp[d], hi = c.base + c.rp[d + 1];
    if (hi - lo == 16) {   // every key present (dense planes): no meta walk
      c.planes = lo + c.j;
      return;
    }
    for (int64_t ci = lo; ci < hi; ci++)
      if (meta_j(c.bv.meta[ci]) == c.j) {
        found = ci;
        break;
      }
  }
  c.planes = found;
}

// container index of dense row d at key j in shard s (wave-uniform, -1 absent)
__device__ __forceinline__ int64_t bsi_find(const BsiCtx& c, int64_t d) {
  if (d < 0) return -1;
  const int lane = wave_lane();
  const int64_t lo = c.rp[d], hi = c.rp[d + 1];
  int64_t found = -1;
  if (lane < hi - lo && meta_j(c.bv.meta[c.base + lo + lane]) == c.j) found = c.base + lo + lane;
  const uint64_t b = __ballot(found >= 0);
  if (!b) return -1;
  return rl_i64(found, int(__builtin_ctzll(b)));
}

__device__ __forceinline__ void bsi_row(const BsiCtx& c, int64_t d, Tile& t) {
  const int64_t ci = bsi_find(c, d);
  if (ci < 0) tile_zero(t);
  else tile_load(t, c.bv.payload, c.bv.meta[ci], c.lb);
}

__device__ __forceinline__ void bsi_plane(const BsiCtx& c, int lane_slot, Tile& t) {
  const int64_t ci = rl_i64(c.planes, lane_slot);
  if (ci < 0) tile_zero(t);
  else tile_load(t, c.bv.payload, c.bv.meta[ci], c.lb);
}

__device__ __forceinline__ void bsi_bit(const BsiCtx& c, int i, Tile& t) {
  if (i < 0 || i >= c.bsi.depth) tile_zero(t);
  else bsi_plane(c, i, t);
}

// filt = filt & ~(filt & ~r & ~keep)   (reference: filt.Difference(filt.Difference(row).Difference(keep)))
__device__ __forceinline__ void keep_set_bits(Tile& f, const Tile& r, const Tile& k) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    f.w[i].x &= ~(f.w[i].x & ~r.w[i].x & ~k.w[i].x);
    f.w[i].y &= ~(f.w[i].y & ~r.w[i].y & ~k.w[i].y);
  }
}

// filt = filt & ~(r & ~keep)
__device__ __forceinline__ void drop_set_bits(Tile& f, const Tile& r, const Tile& k) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    f.w[i].x &= ~(r.w[i].x & ~k.w[i].x);
    f.w[i].y &= ~(r.w[i].y & ~k.w[i].y);
  }
}

__device__ void bsi_lt_unsigned(const BsiCtx& c, Tile& filt, int depth, uint64_t pred, bool allow_eq) {
  Tile keep, r;
  tile_zero(keep);
  bool leading = true;
  for (int i = depth - 1; i >= 0; i--) {
    bsi_bit(c, i, r);
    const int bit = int((pred >> i) & 1);
    if (leading) {
      if (bit == 0) {
        tile_op<OP_ANDNOT>(filt, r);
        continue;
      }
      leading = false;
    }
    if (i == 0 && !allow_eq) {
      if (bit == 0) {
        filt = keep;
        return;
      }
      drop_set_bits(filt, r, keep);
      return;
    }
    if (bit == 0) {
      drop_set_bits(filt, r, keep);
      continue;
    }
    if (i > 0) {
#pragma unroll
      for (int w = 0; w < 8; w++) {
        keep.w[w].x |= filt.w[w].x & ~r.w[w].x;
        keep.w[w].y |= filt.w[w].y & ~r.w[w].y;
      }
    }
  }
}

__device__ void bsi_gt_unsigned(const BsiCtx& c, Tile& filt, int depth, uint64_t pred, bool allow_eq) {
  Tile keep, r;
  tile_zero(keep);
  for (int i = depth - 1; i >= 0; i--) {
    bsi_bit(c, i, r);
    const int bit = int((pred >> i) & 1);
    if (i == 0 && !allow_eq) {
      if (bit == 1) {
        filt = keep;
        return;
      }
      keep_set_bits(filt, r, keep);
      return;
    }
    if (bit == 1) {
      keep_set_bits(filt, r, keep);
      continue;
    }
    if (i > 0) {
#pragma unroll
      for (int w = 0; w < 8; w++) {
        keep.w[w].x |= filt.w[w].x & r.w[w].x;
        keep.w[w].y |= filt.w[w].y & r.w[w].y;
      }
    }
  }
}

__device__ void bsi_between_unsigned(const BsiCtx& c, Tile& filt, int depth, uint64_t pmin, uint64_t pmax) {
  Tile keep1, keep2, r;
  tile_zero(keep1);
  tile_zero(keep2);
  for (int i = depth - 1; i >= 0; i--) {
    bsi_bit(c, i, r);
    const int b1 = int((pmin >> i) & 1), b2 = int((pmax >> i) & 1);
    if (b1 == 1) {
      keep_set_bits(filt, r, keep1);
    } else if (i > 0) {
#pragma unroll
      for (int w = 0; w < 8; w++) {
        keep1.w[w].x |= filt.w[w].x & r.w[w].x;
        keep1.w[w].y |= filt.w[w].y & r.w[w].y;
      }
    }
    if (b2 == 0) {
      drop_set_bits(filt, r, keep2);
    } else if (i > 0) {
#pragma unroll
      for (int w = 0; w < 8; w++) {
        keep2.w[w].x |= filt.w[w].x & ~r.w[w].x;
        keep2.w[w].y |= filt.w[w].y & ~r.w[w].y;
      }
    }
  }
}

__device__ __forceinline__ void tile_or(Tile& a, const Tile& b) { tile_op<OP_OR>(a, b); }

// op: 0 EQ, 1 NEQ, 2 LT, 3 LTE, 4 GT, 5 GTE, 6 BETWEEN(p1..p2), 7 NOT NULL
// OPC: the comparison as a template constant, so each instantiation keeps only
// its own path's tiles live (the runtime switch over every op held 256 VGPRs,
// one wave per SIMD).  ``op_rt`` is unused (kept for the launcher's signature).
template <int OPC>
__global__ __launch_bounds__(256, 2) void bsi_range_kernel(const ViewDev* __restrict__ views, int S, BsiArgs bsi,
                                                        int op_rt, int64_t p1, int64_t p2,
                                                        uint16_t* __restrict__ out_payload,
                                                        int64_t* __restrict__ out_meta,
                                                        unsigned long long* __restrict__ out_count) {
  __shared__ WaveScratch scratch[WAVES_PER_BLOCK];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  const bool live = item < int64_t(S) * 16;
  if (!live && !out_count) return;  // (the count path's block barrier needs every wave)
  const int64_t it = live ? item : 0;
  const int s = int(it >> 4), j = int(it & 15);
  const ViewDev& bv = views[bsi.view];
  BsiCtx c{bsi, bv, s, j, bv.shard_base[s], bv.rowptr + int64_t(s) * (bv.D + 1), scratch[wave].lb};
  plane_index(c);
  const int depth = bsi.depth;
  constexpr int op = OPC;
  (void)op_rt;
  Tile b, sign, res;
  bsi_row(c, bsi.row_exists, b);
  bsi_row(c, bsi.row_sign, sign);
  if (op == 7) {
    res = b;
  } else if (op == 0 || op == 1) {
    Tile eq = b, r;
    const uint64_t up = uint64_t(p1 < 0 ? -p1 : p1);
    if (p1 < 0) tile_op<OP_AND>(eq, sign);
    else tile_op<OP_ANDNOT>(eq, sign);
    for (int i = depth - 1; i >= 0; i--) {
      bsi_bit(c, i, r);
      if ((up >> i) & 1) tile_op<OP_AND>(eq, r);
      else tile_op<OP_ANDNOT>(eq, r);
    }
    res = b;
    if (op == 1) tile_op<OP_ANDNOT>(res, eq);
    else res = eq;
  } else if (op == 2 || op == 3) {
    const bool allow = op == 3;
    const uint64_t up = uint64_t(p1 < 0 ? -p1 : p1);
    if ((p1 >= 0 && allow) || (p1 >= -1 && !allow)) {
      Tile pos = b;
      tile_op<OP_ANDNOT>(pos, sign);
      bsi_lt_unsigned(c, pos, depth, up, allow);
      res = sign;
      tile_or(res, pos);
    } else {
      res = b;
      tile_op<OP_AND>(res, sign);
      bsi_gt_unsigned(c, res, depth, up, allow);
    }
  } else if (op == 4 || op == 5) {
    const bool allow = op == 5;
    const uint64_t up = uint64_t(p1 < 0 ? -p1 : p1);
    if ((p1 >= 0 && allow) || (p1 >= -1 && !allow)) {
      res = b;
      tile_op<OP_ANDNOT>(res, sign);
      bsi_gt_unsigned(c, res, depth, up, allow);
    } else {
      Tile neg = b;
      tile_op<OP_AND>(neg, sign);
      res = b;   // the positives, taken before the descent so b and sign are dead during it
      tile_op<OP_ANDNOT>(res, sign);
      bsi_lt_unsigned(c, neg, depth, up, allow);
      tile_or(res, neg);
    }
  } else {  // between
    const uint64_t umin = uint64_t(p1 < 0 ? -p1 : p1), umax = uint64_t(p2 < 0 ? -p2 : p2);
    if (p1 >= 0) {
      res = b;
      tile_op<OP_ANDNOT>(res, sign);
      bsi_between_unsigned(c, res, depth, umin, umax);
    } else if (p2 < 0) {
      res = b;
      tile_op<OP_AND>(res, sign);
      bsi_between_unsigned(c, res, depth, umax, umin);
    } else {
      Tile pos = b, neg = b;
      tile_op<OP_ANDNOT>(pos, sign);
      tile_op<OP_AND>(neg, sign);
      bsi_lt_unsigned(c, pos, depth, umax, true);
      bsi_lt_unsigned(c, neg, depth, umin, true);
      res = pos;
      tile_or(res, neg);
    }
  }
  const int64_t n = wave_sum_i64(tile_popc(res));
  if (out_count) {  // Count(Row(v <op> x)): no predicate view is written
    // the block's waves fold into one atomic: every wave of the launch
    // adding to the same word serialises at one L2 channel
    // (through each wave's own scratch word 0, free by now: no extra LDS)
    if (lane == 0) scratch[wave].lb[0] = live ? uint64_t(n) : 0ull;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long t = 0;
      for (int w = 0; w < WAVES_PER_BLOCK; w++) t += scratch[w].lb[0];
      if (t) atomicAdd(out_count, t);
    }
    return;
  }
  ulong2* dst = reinterpret_cast<ulong2*>(out_payload + item * 4096);
#pragma unroll
  for (int i = 0; i < 8; i++) dst[i * 64 + lane] = res.w[i];
  if (lane == 0) out_meta[item] = int64_t(j) | (int64_t(CT_BITMAP) << 4) | (n << 6) | ((item * 512) << 23);
}

// ---------------------------------------------------------------- BSI min/max
// Per (shard, key) MSB-first descents (reference fragment.go:1145-1225):
// consider = exists & filter; for Min the max-magnitude negative and the
// unsigned minimum of the positives, for Max the unsigned maximum of the
// positives and the minimum magnitude of the negatives.  out[item] = 4 x
// (value, count); the host folds keys into shard results exactly as one
// shard-wide descent would (the key sets partition the shard).  WHICH = 1
// (Min) runs only maxU(neg) / minU(pos), 2 (Max) only maxU(pos) / minU(neg):
// half the tiles, popcounts and wave reductions per bit (0 = all four).
template <int WHICH, int MINW = 2>
__global__ __launch_bounds__(256, MINW) void bsi_minmax_kernel(const QueryProg* __restrict__ progs,
                                                         const ViewDev* __restrict__ views, int S, BsiArgs bsi,
                                                         int64_t* __restrict__ out) {
  __shared__ WaveScratch scratch[WAVES_PER_BLOCK];
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x >> 6;
  const int lane = wave_lane();
  const int64_t item = int64_t(blk) * WAVES_PER_BLOCK + wave;
  if (item >= int64_t(S) * 16) return;
  const int s = int(item >> 4), j = int(item & 15);
  const ViewDev& bv = views[bsi.view];
  WaveScratch& ws = scratch[wave];
  BsiCtx c{bsi, bv, s, j, bv.shard_base[s], bv.rowptr + int64_t(s) * (bv.D + 1), ws.lb};
  plane_index(c);
  const int depth = bsi.depth;
  const QueryProg& qp = progs[0];
  Tile pos, neg;
  bsi_row(c, bsi.row_exists, pos);
  if (qp.nprog) {
    uint32_t mask[MAXLEAF];
    build_slots(qp, views, s, ws, mask);
    Tile f;
    if ((candidate_mask(qp, mask) >> j) & 1) eval_tile(qp, views, s, j, ws, f);
    else tile_zero(f);
    tile_op<OP_AND>(pos, f);
  }
  {
    Tile sign;
    bsi_row(c, bsi.row_sign, sign);
    neg = pos;
    tile_op<OP_AND>(neg, sign);
    tile_op<OP_ANDNOT>(pos, sign);
  }
  // counted first, so pos / neg are dead once the descents' tiles take them
  const int64_t npos = wave_sum_i64(tile_popc(pos)), nneg = wave_sum_i64(tile_popc(neg));
  // four descents share each bit-slice load: maxU(neg), minU(pos), maxU(pos), minU(neg)
  Tile fmaxn = neg, fminp = pos, fmaxp = pos, fminn = neg, r;
  int64_t vmaxn = 0, vminp = 0, vmaxp = 0, vminn = 0;
  int64_t cmaxn = 0, cminp = 0, cmaxp = 0, cminn = 0;
  for (int i = depth - 1; i >= 0; i--) {
    bsi_bit(c, i, r);
    Tile t;
    int64_t k;
    if (WHICH != 2) {  // maxU(neg)
      t = fmaxn;
      tile_op<OP_AND>(t, r);
      k = wave_sum_i64(tile_popc(t));
      if (k > 0) { vmaxn |= int64_t(1) << i; fmaxn = t; cmaxn = k; }
      else if (i == 0) cmaxn = wave_sum_i64(tile_popc(fmaxn));
    }
    if (WHICH != 1) {  // maxU(pos)
      t = fmaxp;
      tile_op<OP_AND>(t, r);
      k = wave_sum_i64(tile_popc(t));
      if (k > 0) { vmaxp |= int64_t(1) << i; fmaxp = t; cmaxp = k; }
      else if (i == 0) cmaxp = wave_sum_i64(tile_popc(fmaxp));
    }
    if (WHICH != 2) {  // minU(pos)
      t = fminp;
      tile_op<OP_ANDNOT>(t, r);
      k = wave_sum_i64(tile_popc(t));
      if (k > 0) { fminp = t; cminp = k; }
      else { vminp += int64_t(1) << i; if (i == 0) cminp = wave_sum_i64(tile_popc(fminp)); }
    }
    if (WHICH != 1) {  // minU(neg)
      t = fminn;
      tile_op<OP_ANDNOT>(t, r);
      k = wave_sum_i64(tile_popc(t));
      if (k > 0) { fminn = t; cminn = k; }
      else { vminn += int64_t(1) << i; if (i == 0) cminn = wave_sum_i64(tile_popc(fminn)); }
    }
  }
  if (lane == 0) {
    int64_t* o = out + item * 10;
    o[0] = vmaxn; o[1] = cmaxn; o[2] = vminp; o[3] = cminp;
    o[4] = vmaxp; o[5] = cmaxp; o[6] = vminn; o[7] = cminn;
    o[8] = npos; o[9] = nneg;
  }
}

// Fold of the per-key descents into the call's ONE (value, count), on the
// device (one small D2H instead of the [S, 16, 10] table): per fragment (its
// G = 16 * sub-shards keys) fragment.min/max's sign rules -- Min: the largest
// |negative| if any negative, else the smallest positive; Max: the largest
// positive if any, else the smallest |negative| (fragment.go:1145-1225) --
// with the counts of every key holding that value summed; across fragments
// the extreme, counted in the FIRST fragment holding it (executor.go
// ValCount.Smaller / Larger keep the earlier shard's).  One 1024-thread block;
// out = {value, count, found}.
constexpr int FOLD_THREADS = 1024;
// GT: the keys per fragment as a compile-time constant (16: every key's
// loads issue together -- the runtime-G loop serialised them, 44 us per call)
// or 0 (runtime G, wide shards)
template <int GT>
__global__ __launch_bounds__(FOLD_THREADS) void bsi_minmax_fold_kernel(const int64_t* __restrict__ o, int F, int Grt,
                                                                      int is_min, int64_t* __restrict__ out) {
  const int G = GT > 0 ? GT : Grt;
  __shared__ int64_t sv[FOLD_THREADS / 64];
  __shared__ int sf[FOLD_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t BIG = 0x7fffffffffffffffLL;
  // this thread's best (value, fragment) over its fragments; key = value
  // for Min, -value for Max (smaller key wins; ties: lower fragment)
  int64_t bkey = BIG, bval = 0, bcnt = 0;
  int bfrag = 0x7fffffff;
  if (GT == 16) {
    // 16 lanes per fragment, lane g on key g: its 10 words are 5 coalesced
    // 16-byte loads (a thread per fragment striding 80 bytes per key touched
    // 64 cache lines per load instruction: 47 us per call), two fragments
    // per group in flight; the group's extreme and count by shuffles
    const int g = tid & 15;
    auto fold = [&](const longlong2 w0, const longlong2 w1, const longlong2 w2, const longlong2 w3,
                    const longlong2 w4, const int f) {
      const bool live = f < F;
      const bool anyp = (uint64_t(__ballot(live && w4.x > 0)) >> (lane & 48)) & 0xFFFFu;
      const bool anyn = (uint64_t(__ballot(live && w4.y > 0)) >> (lane & 48)) & 0xFFFFu;
      if (!anyp && !anyn) return;  // group-uniform
      const bool use_neg = is_min ? anyn : !anyp;
      const int vc = is_min ? (anyn ? 0 : 2) : (anyp ? 4 : 6);
      const bool largest = vc == 0 || vc == 4;
      const bool valid = (use_neg ? w4.y : w4.x) > 0;
      const longlong2 xc = vc == 0 ? w0 : vc == 2 ? w1 : vc == 4 ? w2 : w3;  // (value, count)
      int64_t best = valid ? int64_t(xc.x) : (largest ? int64_t(-1) : BIG);
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) {
        const int64_t b2 = __shfl_xor(best, off, 64);
        best = largest ? (b2 > best ? b2 : best) : (b2 < best ? b2 : best);
      }
      int64_t cnt = valid && int64_t(xc.x) == best ? int64_t(xc.y) : 0;
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
      const int64_t val = use_neg ? -best : best;
      const int64_t key = is_min ? val : -val;
      if (g == 0 && (key < bkey || (key == bkey && f < bfrag))) { bkey = key; bval = val; bcnt = cnt; bfrag = f; }
    };
    const int grp = tid >> 4;  // 64 groups
    for (int f0 = grp; f0 < F; f0 += 2 * (FOLD_THREADS / 16)) {
      const int f1 = f0 + FOLD_THREADS / 16;
      const longlong2* e0 = reinterpret_cast<const longlong2*>(o + (int64_t(f0) * 16 + g) * 10);
      const longlong2* e1 = reinterpret_cast<const longlong2*>(o + (int64_t(f1 < F ? f1 : f0) * 16 + g) * 10);
      const longlong2 a0 = e0[0], a1 = e0[1], a2 = e0[2], a3 = e0[3], a4 = e0[4];
      const longlong2 b0 = e1[0], b1 = e1[1], b2 = e1[2], b3 = e1[3], b4 = e1[4];
      fold(a0, a1, a2, a3, a4, f0);
      fold(b0, b1, b2, b3, b4, f1);
    }
  } else
  for (int f = tid; f < F; f += FOLD_THREADS) {
    const int64_t* e = o + int64_t(f) * G * 10;
    bool anyp = false, anyn = false;
#pragma unroll
    for (int g = 0; g < G; g++) {
      anyp |= e[g * 10 + 8] > 0;
      anyn |= e[g * 10 + 9] > 0;
    }
    if (!anyp && !anyn) continue;
    // column pair and sign of the fragment's candidate: Min: neg -> max |neg| (0/1),
    // else min pos (2/3); Max: pos -> max pos (4/5), else min |neg| (6/7)
    const bool use_neg = is_min ? anyn : !anyp;
    const int vc = is_min ? (anyn ? 0 : 2) : (anyp ? 4 : 6);
    const bool largest = vc == 0 || vc == 4;
    const int mcol = use_neg ? 9 : 8;
    int64_t best = largest ? -1 : BIG, cnt = 0;
#pragma unroll
    for (int g = 0; g < G; g++) {
      if (e[g * 10 + mcol] <= 0) continue;
      const int64_t v = e[g * 10 + vc];
      if (largest ? v > best : v < best) { best = v; cnt = 0; }
      if (v == best) cnt += e[g * 10 + vc + 1];
    }
    const int64_t val = use_neg ? -best : best;
    const int64_t key = is_min ? val : -val;
    if (key < bkey || (key == bkey && f < bfrag)) { bkey = key; bval = val; bcnt = cnt; bfrag = f; }
  }
  // block argmin of (key, fragment): wave shuffles, then LDS across waves
  int64_t k = bkey;
  int fr = bfrag;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t k2 = __shfl_xor(k, off, 64);
    const int f2 = __shfl_xor(fr, off, 64);
    if (k2 < k || (k2 == k && f2 < fr)) { k = k2; fr = f2; }
  }
  if (lane == 0) { sv[wave] = k; sf[wave] = fr; }
  __syncthreads();
  if (wave == 0) {
    k = lane < FOLD_THREADS / 64 ? sv[lane] : BIG;
    fr = lane < FOLD_THREADS / 64 ? sf[lane] : 0x7fffffff;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const int64_t k2 = __shfl_xor(k, off, 64);
      const int f2 = __shfl_xor(fr, off, 64);
      if (k2 < k || (k2 == k && f2 < fr)) { k = k2; fr = f2; }
    }
    if (lane == 0) { sv[0] = k; sf[0] = fr; }
  }
  __syncthreads();
  // the owner of the winning fragment writes it (vector stores)
  if (sf[0] == bfrag && bfrag != 0x7fffffff && sv[0] == bkey) {
    out[0] = bval;
    out[1] = bcnt;
    out[2] = 1;
  } else if (tid == 0 && sf[0] == 0x7fffffff) {
    out[0] = 0;
    out[1] = 0;
    out[2] = 0;
  }
}

// Multi-block fold (16 keys per fragment): block b takes fragments
// 64 b .. 64 b + 63, one per 16-lane group (the same per-fragment rules as
// bsi_minmax_fold_kernel), and writes its winner as part[4 b ..] = {key,
// value, count, fragment} (key = value for Min, -value for Max; BIG = none).
__global__ __launch_bounds__(FOLD_THREADS) void bsi_minmax_fold_part_kernel(const int64_t* __restrict__ o, int F,
                                                                           int is_min, int64_t* __restrict__ part) {
  __shared__ int64_t sv[FOLD_THREADS / 64];
  __shared__ int sf[FOLD_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = tid & 15;
  const int64_t BIG = 0x7fffffffffffffffLL;
  const int f = int(blockIdx.x) * (FOLD_THREADS / 16) + (tid >> 4);
  const longlong2* e = reinterpret_cast<const longlong2*>(o + (int64_t(f < F ? f : 0) * 16 + g) * 10);
  const longlong2 w0 = e[0], w1 = e[1], w2 = e[2], w3 = e[3], w4 = e[4];
  const bool live = f < F;
  const bool anyp = (uint64_t(__ballot(live && w4.x > 0)) >> (lane & 48)) & 0xFFFFu;
  const bool anyn = (uint64_t(__ballot(live && w4.y > 0)) >> (lane & 48)) & 0xFFFFu;
  int64_t key = BIG, val = 0, cnt = 0;
  if (anyp || anyn) {  // group-uniform
    const bool use_neg = is_min ? anyn : !anyp;
    const int vc = is_min ? (anyn ? 0 : 2) : (anyp ? 4 : 6);
    const bool largest = vc == 0 || vc == 4;
    const bool valid = (use_neg ? w4.y : w4.x) > 0;
    const longlong2 xc = vc == 0 ? w0 : vc == 2 ? w1 : vc == 4 ? w2 : w3;
    int64_t best = valid ? int64_t(xc.x) : (largest ? int64_t(-1) : BIG);
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
      const int64_t b2 = __shfl_xor(best, off, 64);
      best = largest ? (b2 > best ? b2 : best) : (b2 < best ? b2 : best);
    }
    int64_t c = valid && int64_t(xc.x) == best ? int64_t(xc.y) : 0;
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    val = use_neg ? -best : best;
    key = is_min ? val : -val;
    cnt = c;
  }
  // block argmin of (key, fragment) over the groups' lane 0
  int64_t k = g == 0 ? key : BIG;
  int fr = g == 0 && key != BIG ? f : 0x7fffffff;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t k2 = __shfl_xor(k, off, 64);
    const int f2 = __shfl_xor(fr, off, 64);
    if (k2 < k || (k2 == k && f2 < fr)) { k = k2; fr = f2; }
  }
  if (lane == 0) { sv[wave] = k; sf[wave] = fr; }
  __syncthreads();
  if (wave == 0) {
    k = lane < FOLD_THREADS / 64 ? sv[lane] : BIG;
    fr = lane < FOLD_THREADS / 64 ? sf[lane] : 0x7fffffff;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const int64_t k2 = __shfl_xor(k, off, 64);
      const int f2 = __shfl_xor(fr, off, 64);
      if (k2 < k || (k2 == k && f2 < fr)) { k = k2; fr = f2; }
    }
    if (lane == 0) { sv[0] = k; sf[0] = fr; }
  }
  __syncthreads();
  int64_t* pb = part + int64_t(blockIdx.x) * 4;
  if (sf[0] == 0x7fffffff) {
    if (tid == 0) { pb[0] = BIG; pb[1] = 0; pb[2] = 0; pb[3] = 0x7fffffff; }
  } else if (g == 0 && f == sf[0] && key == sv[0]) {
    pb[0] = key; pb[1] = val; pb[2] = cnt; pb[3] = f;
  }
}

// The blocks' winners -> out = {value, count, found}: smallest key, ties to
// the lower fragment (the first shard holding the extreme).
__global__ __launch_bounds__(256) void bsi_minmax_fold_final_kernel(const int64_t* __restrict__ part, int nb,
                                                                   int64_t* __restrict__ out) {
  __shared__ int64_t sk[4], sv[4], sc[4];
  __shared__ int sfr[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t BIG = 0x7fffffffffffffffLL;
  int64_t k = BIG, v = 0, c = 0;
  int fr = 0x7fffffff;
  for (int b = tid; b < nb; b += 256) {
    const int64_t k2 = part[int64_t(b) * 4], f2 = part[int64_t(b) * 4 + 3];
    if (k2 < k || (k2 == k && int(f2) < fr)) {
      k = k2; fr = int(f2); v = part[int64_t(b) * 4 + 1]; c = part[int64_t(b) * 4 + 2];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t k2 = __shfl_xor(k, off, 64), v2 = __shfl_xor(v, off, 64), c2 = __shfl_xor(c, off, 64);
    const int f2 = __shfl_xor(fr, off, 64);
    if (k2 < k || (k2 == k && f2 < fr)) { k = k2; fr = f2; v = v2; c = c2; }
  }
  if (lane == 0) { sk[wave] = k; sv[wave] = v; sc[wave] = c; sfr[wave] = fr; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; w++)
      if (sk[w] < k || (sk[w] == k && sfr[w] < fr)) { k = sk[w]; fr = sfr[w]; v = sv[w]; c = sc[w]; }
    const bool found = fr != 0x7fffffff;
    out[0] = found ? v : 0;
    out[1] = found ? c : 0;
    out[2] = found ? 1 : 0;
  }
}

}  // namespace pk

// ------------------------------------------------------------ launchers
namespace pk {

static inline unsigned grid_for(int64_t items) {
  return unsigned((items + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
}

void launch_expr_count(const QueryProg* progs, int Q, const ViewDev* views, int S, unsigned long long* out,
                       int32_t* per_key, int64_t* per_shard, int mode, hipStream_t st) {
  const int64_t items = int64_t(Q) * S;
  if (items == 0) return;
  const dim3 grid(grid_for(items)), block(64 * WAVES_PER_BLOCK);
  if (mode == 4 && per_key == nullptr && per_shard == nullptr)
    hipLaunchKernelGGL(union_count2_kernel, grid, block, 0, st, progs, Q, views, S, out);
  else if (mode == 3 && per_key == nullptr && per_shard == nullptr)
    hipLaunchKernelGGL(union_count_kernel, grid, block, 0, st, progs, Q, views, S, out);
  else if (mode == 1 && per_key == nullptr)
    hipLaunchKernelGGL(expr_count_kernel<1>, grid, block, 0, st, progs, Q, views, S, out, per_key, per_shard);
  else if (mode == 2 || mode == 3 || mode == 4)
    hipLaunchKernelGGL(expr_count_kernel<2>, grid, block, 0, st, progs, Q, views, S, out, per_key, per_shard);
  else
    hipLaunchKernelGGL(expr_count_kernel<0>, grid, block, 0, st, progs, Q, views, S, out, per_key, per_shard);
}

void launch_expr_materialize(const QueryProg* progs, int Q, const ViewDev* views, int S, const int32_t* counts,
                             const int64_t* offs, uint16_t* outp, hipStream_t st) {
  const int64_t items = int64_t(Q) * S;
  if (items == 0) return;
  hipLaunchKernelGGL(expr_materialize_kernel, dim3(grid_for(items)), dim3(64 * WAVES_PER_BLOCK), 0, st, progs,
                     Q, views, S, counts, offs, outp);
}

void launch_expr_dense(const QueryProg* progs, int Q, const ViewDev* views, int S, uint16_t* outp, int64_t* out_meta,
                       hipStream_t st) {
  const int64_t items = int64_t(Q) * S;
  if (items == 0) return;
  hipLaunchKernelGGL(expr_dense_kernel, dim3(grid_for(items)), dim3(64 * WAVES_PER_BLOCK), 0, st, progs, Q, views, S,
                     outp, out_meta);
}

void launch_bsi_range(const ViewDev* views, int S, BsiArgs bsi, int op, int64_t p1, int64_t p2, uint16_t* out_payload,
                      int64_t* out_meta, unsigned long long* out_count, hipStream_t st) {
  const int64_t items = int64_t(S) * 16;
  if (items == 0) return;
  const dim3 grid(grid_for(items)), block(64 * WAVES_PER_BLOCK);
#define PK_RANGE(OPV)                                                                                       \
  case OPV:                                                                                                 \
    hipLaunchKernelGGL(bsi_range_kernel<OPV>, grid, block, 0, st, views, S, bsi, op, p1, p2, out_payload,  \
                       out_meta, out_count);                                                                \
    break;
  switch (op) {
    PK_RANGE(0) PK_RANGE(1) PK_RANGE(2) PK_RANGE(3) PK_RANGE(4) PK_RANGE(5) PK_RANGE(6) PK_RANGE(7)
    default: break;
  }
#undef PK_RANGE
}

void launch_bsi_minmax(const QueryProg* progs, const ViewDev* views, int S, BsiArgs bsi, int64_t* out,
                       hipStream_t st, int which) {
  const int64_t items = int64_t(S) * 16;
  if (items == 0) return;
  const dim3 grid(grid_for(items)), block(64 * WAVES_PER_BLOCK);
  // 2 waves per SIMD; 3 (168 VGPRs, 224 B of spills) measured the same
  // (1.29 vs 1.31 ms per Min, profiles/r04_u/)
  if (which == 1)
    hipLaunchKernelGGL((bsi_minmax_kernel<1, 2>), grid, block, 0, st, progs, views, S, bsi, out);
  else if (which == 2)
    hipLaunchKernelGGL((bsi_minmax_kernel<2, 2>), grid, block, 0, st, progs, views, S, bsi, out);
  else
    hipLaunchKernelGGL((bsi_minmax_kernel<0, 2>), grid, block, 0, st, progs, views, S, bsi, out);
}

void launch_bsi_minmax_fold(const int64_t* o, int F, int G, int is_min, int64_t* out, int64_t* part,
                            hipStream_t st) {
  if (G == 16 && part && F > FOLD_THREADS / 16) {
    // one fragment per 16-lane group over ceil(F / 64) blocks, then the
    // blocks' winners (one load round trip each instead of ~8 in one block)
    const int nb = (F + FOLD_THREADS / 16 - 1) / (FOLD_THREADS / 16);
    hipLaunchKernelGGL(bsi_minmax_fold_part_kernel, dim3(nb), dim3(FOLD_THREADS), 0, st, o, F, is_min, part);
    hipLaunchKernelGGL(bsi_minmax_fold_final_kernel, dim3(1), dim3(256), 0, st, part, nb, out);
  } else if (G == 16) {
    hipLaunchKernelGGL(bsi_minmax_fold_kernel<16>, dim3(1), dim3(FOLD_THREADS), 0, st, o, F, G, is_min, out);
  } else {
    hipLaunchKernelGGL(bsi_minmax_fold_kernel<0>, dim3(1), dim3(FOLD_THREADS), 0, st, o, F, G, is_min, out);
  }
}

void launch_bsi_sum(const QueryProg* progs, int Q, const ViewDev* views, int S, BsiArgs bsi,
                    unsigned long long* out_sum, unsigned long long* out_cnt, int fmode, hipStream_t st) {
  static const int variant = [] {
    const char* e = getenv("PILOSA_BSI_SUM_VARIANT");
    return e ? atoi(e) : 1;
  }();
  if (variant == 0) {  // one wave per (query, shard), keys walked in sequence
    const int64_t items = int64_t(Q) * S;
    if (items == 0) return;
    hipLaunchKernelGGL(bsi_sum_kernel, dim3(grid_for(items)), dim3(64 * WAVES_PER_BLOCK), 0, st, progs, Q, views,
                       S, bsi, out_sum, out_cnt);
    return;
  }
  const int64_t items = int64_t(Q) * S * 16;
  if (items == 0) return;
  const dim3 grid(grid_for(items)), block(64 * WAVES_PER_BLOCK);
  if (fmode == 0)
    hipLaunchKernelGGL(bsi_sum_keys_kernel<0>, grid, block, 0, st, progs, Q, views, S, bsi, out_sum, out_cnt);
  else if (fmode == 1)
    hipLaunchKernelGGL(bsi_sum_keys_kernel<1>, grid, block, 0, st, progs, Q, views, S, bsi, out_sum, out_cnt);
  else
    hipLaunchKernelGGL(bsi_sum_keys_kernel<2>, grid, block, 0, st, progs, Q, views, S, bsi, out_sum, out_cnt);
}

}  // namespace pk
