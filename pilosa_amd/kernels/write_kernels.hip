// Device write path (gfx950): bulk set/clear of bits straight into an HBM
// arena, instead of rebuilding the touched containers on the host.
//
//   K11  AddN / RemoveN          roaring/roaring.go:277-310 (directOpN)
//   K12  ImportRoaringBits       roaring/roaring.go:1463-1558
//
// The host groups a write batch by container (row*16 + key) and finds each
// container's current metadata word in the shard's segment (-1 = new).  Then
//
//   merge: one 256-thread workgroup per touched container expands the old
//          container (array / bitmap / run) into an 8 KiB LDS bitmap,
//          applies the delta -- sorted u16 lows (positions mode) or a whole
//          delta container (roaring mode) -- with OR or AND-NOT, and writes
//          the bitmap plus its cardinality to scratch;
//   emit:  the container's encoding follows the reference's Optimize rule
//          (roaring.go:2289-2338): run when runs <= 2048 and runs <= n/2,
//          else array when n < 4096, else bitmap.  After an exclusive scan of
//          the output sizes (run: 8-u16 header + (start, last) pairs; array:
//          n values; both padded to 8; bitmap 4096 u16; empty containers
//          vanish), one workgroup per container writes it at the tail of the
//          arena payload -- bitmap words copied, the array's values or the
//          runs' starts and lasts placed by workgroup prefix sums over
//          per-thread popcounts -- and its new metadata word.
//
// The host then splices the new metadata words into the shard's segment.  Only
// the write batch (8 B per position) crosses PCIe, never container payloads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kernels.h"

namespace pk {

namespace {

constexpr int WG = 256;               // 4 waves of 64
constexpr int WORDS_PER_THREAD = 1024 / WG;

// OR (set) a container of the arena into the LDS bitmap, or AND-NOT (clear) it.
template <bool CLEAR>
__device__ __forceinline__ void apply_container(uint64_t* bm, const uint16_t* payload, int64_t m) {
  const int tid = threadIdx.x;
  const int type = meta_type(m);
  const uint16_t* p = payload + meta_off16(m) * 8;
  if (type == CT_BITMAP) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(p);
    for (int i = tid; i < 1024; i += WG) bm[i] = CLEAR ? (bm[i] & ~w[i]) : (bm[i] | w[i]);
  } else if (type == CT_ARRAY) {
    const int n = meta_n(m);
    for (int i = tid; i < n; i += WG) {
      const uint32_t v = p[i];
      if (CLEAR)
        atomicAnd(reinterpret_cast<unsigned long long*>(&bm[v >> 6]), ~(1ull << (v & 63)));
      else
        atomicOr(reinterpret_cast<unsigned long long*>(&bm[v >> 6]), 1ull << (v & 63));
    }
  } else {  // run: p[0] runs, (start, last) pairs from p[8]
    const int nr = p[0];
    for (int r = tid; r < nr; r += WG) {
      const uint32_t s = p[8 + 2 * r], e = uint32_t(p[9 + 2 * r]) + 1;  // [s, e)
      const uint32_t ws = s >> 6, we = (e - 1) >> 6;
      for (uint32_t w = ws; w <= we; w++) {
        const uint32_t lo = w == ws ? (s & 63) : 0, hi = w == we ? ((e - 1) & 63) + 1 : 64;
        const uint64_t mk = (hi - lo == 64) ? ~0ull : (((1ull << (hi - lo)) - 1) << lo);
        if (CLEAR)
          atomicAnd(reinterpret_cast<unsigned long long*>(&bm[w]), ~mk);
        else
          atomicOr(reinterpret_cast<unsigned long long*>(&bm[w]), mk);
      }
    }
  }
}

// mode 0: positions (dstart/dlows), mode 1: delta containers (dmeta/dpayload).
template <bool CLEAR, int MODE>
__global__ __launch_bounds__(WG) void container_merge_kernel(const int64_t* __restrict__ old_meta,
                                                             const uint16_t* __restrict__ payload,
                                                             const int32_t* __restrict__ dstart,
                                                             const uint16_t* __restrict__ dlows,
                                                             const int64_t* __restrict__ dmeta,
                                                             const uint16_t* __restrict__ dpayload,
                                                             uint64_t* __restrict__ scratch,
                                                             int32_t* __restrict__ card,
                                                             int32_t* __restrict__ nruns) {
  __shared__ uint64_t bm[1024];
  __shared__ int32_t red[WG / 64], redr[WG / 64];
  const int tid = threadIdx.x;
  const int64_t u = blockIdx.x;
  for (int i = tid; i < 1024; i += WG) bm[i] = 0;
  __syncthreads();
  const int64_t om = old_meta[u];
  if (om >= 0) apply_container<false>(bm, payload, om);
  __syncthreads();
  if (MODE == 0) {
    const int32_t b = dstart[u], e = dstart[u + 1];
    for (int32_t i = b + tid; i < e; i += WG) {
      const uint32_t v = dlows[i];
      if (CLEAR)
        atomicAnd(reinterpret_cast<unsigned long long*>(&bm[v >> 6]), ~(1ull << (v & 63)));
      else
        atomicOr(reinterpret_cast<unsigned long long*>(&bm[v >> 6]), 1ull << (v & 63));
    }
  } else {
    const int64_t dm = dmeta[u];
    if (dm >= 0) apply_container<CLEAR>(bm, dpayload, dm);
  }
  __syncthreads();
  int c = 0, r = 0;
  uint64_t* out = scratch + u * 1024;
#pragma unroll
  for (int k = 0; k < WORDS_PER_THREAD; k++) {
    const int i = k * WG + tid;  // coalesced
    const uint64_t w = bm[i];
    const uint64_t prev_top = i ? (bm[i - 1] >> 63) : 0ull;
    out[i] = w;
    c += __popcll(w);
    r += __popcll(w & ~((w << 1) | prev_top));   // run starts: set bits whose predecessor is clear
  }
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_down(c, o, 64);
    r += __shfl_down(r, o, 64);
  }
  if ((tid & 63) == 0) red[tid >> 6] = c, redr[tid >> 6] = r;
  __syncthreads();
  if (tid == 0) {
    card[u] = red[0] + red[1] + red[2] + red[3];
    nruns[u] = redr[0] + redr[1] + redr[2] + redr[3];
  }
}

// The reference's Optimize choice for a container of n bits in `runs` runs.
__device__ __forceinline__ int emit_type(int n, int runs) {
  if (runs <= RUN_MAX && runs <= n / 2) return CT_RUN;
  return n < ARRAY_MAX ? CT_ARRAY : CT_BITMAP;
}

// Exclusive workgroup scan of one int per thread (Hillis-Steele in LDS).
__device__ __forceinline__ int wg_exclusive_scan(int32_t* scan, int v) {
  const int tid = threadIdx.x;
  scan[tid] = v;
  __syncthreads();
  for (int o = 1; o < WG; o <<= 1) {
    const int x = tid >= o ? scan[tid - o] : 0;
    __syncthreads();
    scan[tid] += x;
    __syncthreads();
  }
  const int at = scan[tid] - v;
  __syncthreads();
  return at;
}

__global__ __launch_bounds__(WG) void container_emit_kernel(const uint64_t* __restrict__ scratch,
                                                            const int32_t* __restrict__ card,
                                                            const int32_t* __restrict__ nruns,
                                                            const int64_t* __restrict__ off16,
                                                            const int32_t* __restrict__ jkey,
                                                            uint16_t* __restrict__ payload,
                                                            int64_t* __restrict__ meta_out) {
  __shared__ int32_t scan[WG];
  const int tid = threadIdx.x;
  const int64_t u = blockIdx.x;
  const int n = card[u];
  const uint64_t* src = scratch + u * 1024;
  if (n == 0) {
    if (tid == 0) meta_out[u] = -1;
    return;
  }
  const int64_t o16 = off16[u];
  const int type = emit_type(n, nruns[u]);
  if (type == CT_RUN) {
    // thread t owns words [4t, 4t+4): run starts (bit set, predecessor clear)
    // and lasts (bit set, successor clear) are numbered by two prefix sums;
    // the k-th start and the k-th last form run k
    uint64_t w[WORDS_PER_THREAD];
#pragma unroll
    for (int k = 0; k < WORDS_PER_THREAD; k++) w[k] = src[tid * WORDS_PER_THREAD + k];
    const uint64_t before = tid ? src[tid * WORDS_PER_THREAD - 1] : 0ull;
    const uint64_t after = tid + 1 < WG ? src[(tid + 1) * WORDS_PER_THREAD] : 0ull;
    uint64_t st[WORDS_PER_THREAD], la[WORDS_PER_THREAD];
    int cs = 0, cl = 0;
#pragma unroll
    for (int k = 0; k < WORDS_PER_THREAD; k++) {
      const uint64_t prev_top = (k ? w[k - 1] : before) >> 63;
      const uint64_t next_low = (k + 1 < WORDS_PER_THREAD ? w[k + 1] : after) & 1ull;
      st[k] = w[k] & ~((w[k] << 1) | prev_top);
      la[k] = w[k] & ~((w[k] >> 1) | (next_low << 63));
      cs += __popcll(st[k]);
      cl += __popcll(la[k]);
    }
    int as = wg_exclusive_scan(scan, cs);
    int al = wg_exclusive_scan(scan, cl);
    uint16_t* dst = payload + o16 * 8;
#pragma unroll
    for (int k = 0; k < WORDS_PER_THREAD; k++) {
      const int base = (tid * WORDS_PER_THREAD + k) * 64;
      for (uint64_t x = st[k]; x; x &= x - 1) dst[8 + 2 * (as++)] = uint16_t(base + __ffsll((long long)x) - 1);
      for (uint64_t x = la[k]; x; x &= x - 1) dst[9 + 2 * (al++)] = uint16_t(base + __ffsll((long long)x) - 1);
    }
    const int nr = nruns[u];
    const int used = 8 + 2 * nr, padded = (used + 7) & ~7;
    if (tid < 8) dst[tid] = tid == 0 ? uint16_t(nr) : uint16_t(0);
    if (tid < padded - used) dst[used + tid] = 0;
    if (tid == 0) meta_out[u] = int64_t(jkey[u]) | (int64_t(CT_RUN) << 4) | (int64_t(n) << 6) | (o16 << 23);
    return;
  }
  if (type == CT_BITMAP) {
    uint64_t* dst = reinterpret_cast<uint64_t*>(payload + o16 * 8);
    for (int i = tid; i < 1024; i += WG) dst[i] = src[i];
    if (tid == 0) meta_out[u] = int64_t(jkey[u]) | (int64_t(CT_BITMAP) << 4) | (int64_t(n) << 6) | (o16 << 23);
    return;
  }
  // array: thread t owns words [4t, 4t+4); exclusive scan of their popcounts
  uint64_t w[WORDS_PER_THREAD];
  int c = 0;
#pragma unroll
  for (int k = 0; k < WORDS_PER_THREAD; k++) {
    w[k] = src[tid * WORDS_PER_THREAD + k];
    c += __popcll(w[k]);
  }
  scan[tid] = c;
  __syncthreads();
  for (int o = 1; o < WG; o <<= 1) {  // Hillis-Steele inclusive scan
    const int x = tid >= o ? scan[tid - o] : 0;
    __syncthreads();
    scan[tid] += x;
    __syncthreads();
  }
  int at = scan[tid] - c;
  uint16_t* dst = payload + o16 * 8;
#pragma unroll
  for (int k = 0; k < WORDS_PER_THREAD; k++) {
    uint64_t x = w[k];
    const int base = (tid * WORDS_PER_THREAD + k) * 64;
    while (x) {
      const int b = __ffsll(static_cast<long long>(x)) - 1;
      dst[at++] = uint16_t(base + b);
      x &= x - 1;
    }
  }
  const int padded = (n + 7) & ~7;
  if (tid < padded - n) dst[n + tid] = 0;
  if (tid == 0) meta_out[u] = int64_t(jkey[u]) | (int64_t(CT_ARRAY) << 4) | (int64_t(n) << 6) | (o16 << 23);
}

// Payload compaction: container c (metadata word meta[c], type 0 = unused
// slot) is copied from its old payload offset to new_off16[c]*8 of dst; one
// wave per container, grid-stride, 16-byte loads and stores.
__global__ __launch_bounds__(WG) void payload_compact_kernel(const int64_t* __restrict__ meta, int64_t C,
                                                             const int64_t* __restrict__ new_off16,
                                                             const int64_t* __restrict__ size16,
                                                             const uint16_t* __restrict__ src,
                                                             uint16_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = int64_t(gridDim.x) * (WG / 64);
  for (int64_t c = int64_t(blockIdx.x) * (WG / 64) + (threadIdx.x >> 6); c < C; c += waves) {
    const int64_t m = meta[c];
    const int64_t n16 = size16[c];
    if (meta_type(m) == 0 || n16 == 0) continue;
    const uint4* sp = reinterpret_cast<const uint4*>(src + meta_off16(m) * 8);
    uint4* dp = reinterpret_cast<uint4*>(dst + new_off16[c] * 8);
    for (int64_t i = lane; i < n16; i += 64) dp[i] = sp[i];
  }
}

}  // namespace

void launch_payload_compact(const int64_t* meta, int64_t C, const int64_t* new_off16, const int64_t* size16,
                            const uint16_t* src, uint16_t* dst, hipStream_t st) {
  if (C <= 0) return;
  const int64_t blocks = std::min<int64_t>((C + 3) / 4, 256 * 64);   // 64 waves per CU worth of work in flight
  hipLaunchKernelGGL(payload_compact_kernel, dim3(unsigned(blocks)), dim3(WG), 0, st, meta, C, new_off16, size16,
                     src, dst);
}

void launch_container_merge(const int64_t* old_meta, const uint16_t* payload, int64_t U, const int32_t* dstart,
                            const uint16_t* dlows, const int64_t* dmeta, const uint16_t* dpayload, int mode,
                            bool clear, uint64_t* scratch, int32_t* card, int32_t* nruns, hipStream_t st) {
  if (U <= 0) return;
  const dim3 g{unsigned(U)}, b{unsigned(WG)};
  if (mode == 0) {
    if (clear)
      hipLaunchKernelGGL((container_merge_kernel<true, 0>), g, b, 0, st, old_meta, payload, dstart, dlows, dmeta,
                         dpayload, scratch, card, nruns);
    else
      hipLaunchKernelGGL((container_merge_kernel<false, 0>), g, b, 0, st, old_meta, payload, dstart, dlows, dmeta,
                         dpayload, scratch, card, nruns);
  } else {
    if (clear)
      hipLaunchKernelGGL((container_merge_kernel<true, 1>), g, b, 0, st, old_meta, payload, dstart, dlows, dmeta,
                         dpayload, scratch, card, nruns);
    else
      hipLaunchKernelGGL((container_merge_kernel<false, 1>), g, b, 0, st, old_meta, payload, dstart, dlows, dmeta,
                         dpayload, scratch, card, nruns);
  }
}

void launch_container_emit(const uint64_t* scratch, const int32_t* card, const int32_t* nruns, const int64_t* off16,
                           const int32_t* jkey, int64_t U, uint16_t* payload, int64_t* meta_out, hipStream_t st) {
  if (U <= 0) return;
  hipLaunchKernelGGL(container_emit_kernel, dim3(unsigned(U)), dim3(WG), 0, st, scratch, card, nruns, off16, jkey,
                     payload, meta_out);
}

}  // namespace pk
