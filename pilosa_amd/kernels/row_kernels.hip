// Row-level device kernels (gfx950): Shift and the Rows listing.
//
//   K7  Shift(row, n)   roaring/roaring.go:944-977 (Bitmap.Shift), row.go:217-239
//   K20 Rows listing    fragment.go:2601-2712 (rows / rowsForColumn)
//
// Shift.  The reference shifts a row segment by one bit n times, container by
// container with a carry.  Here the child expression is first evaluated into
// a dense one-row view (expr_dense_kernel: one 8 KiB bitmap per (shard, key),
// i.e. 16384 words per shard), then one pass moves every word: target word T
// takes source words T - n/64 and T - n/64 - 1, funnel-shifted by n % 64.
// A shard wider than 2^20 columns is M consecutive device sub-shards whose
// words form one row, so carries cross sub-shard boundaries in that pass.
// Targets past the shard's last column form the "spill" view: the bits a
// per-shard evaluation carries into the next shard's segment (row.go keeps
// them in the shard's segment; Row.Merge folds them into shard s + 1).  One
// wave per (shard, half, key), 16 words per lane, fully coalesced.
//
// Rows.  One thread per dense row walks the shards: the row is listed at its
// first non-empty container (with column=: the first key-j container holding
// that column's bit -- bitmap word test, binary search over array values or
// run starts).  Flags are a byte per dense row.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

extern "C" __device__ long __ockl_wfred_add_i64(long);

namespace pk {

namespace {

constexpr int SHARD_WORDS = 16 * 1024;

// M = device sub-shards per shard (shards wider than 2^20 columns,
// pilosa_amd/shardwidth.py): the M sub-shards of a shard are consecutive in
// the view and form one M * 16384-word row, so a word carried past a
// sub-shard's end lands in the next sub-shard of the same shard; only words
// carried past the SHARD's end form the spill, whose sub-shard m part
// belongs to sub-shard m of the next shard.  M = 1 at widths <= 2^20.
// row_words = the host shard's width in words: M * 16384 from 2^20 columns
// up, 2^e / 64 for a narrower 2^e-column shard, which fills only the first
// 2^(e-16) containers of its device shard -- words carried past 2^e columns
// form its spill, and the device containers past it stay empty.
__global__ __launch_bounds__(256) void shift_dense_kernel(const uint64_t* __restrict__ src, int S, int M, int64_t n,
                                                          int64_t row_words,
                                                          uint64_t* __restrict__ main_out,
                                                          int64_t* __restrict__ main_meta,
                                                          uint64_t* __restrict__ spill_out,
                                                          int64_t* __restrict__ spill_meta) {
  const int lane = threadIdx.x & 63;
  const int64_t item = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (item >= int64_t(S) * 32) return;
  const int s = int(item >> 5);
  const int half = int(item >> 4) & 1;
  const int k = int(item & 15);
  const int64_t nw = n >> 6;
  const int sh = int(n & 63);
  const int m = s % M;
  const uint64_t* sp = src + int64_t(s - m) * SHARD_WORDS;        // its first sub-shard
  uint64_t* dst = (half ? spill_out : main_out) + int64_t(s) * SHARD_WORDS + k * 1024;
  // word of this wave within the shard's row, and the target word counted
  // from the shard's first word (the spill continues past the shard's end)
  const int64_t l0 = int64_t(m) * SHARD_WORDS + k * 1024;
  const int64_t t0 = int64_t(half) * row_words + l0;
  int c = 0;
#pragma unroll 4
  for (int i = 0; i < 16; i++) {
    const int w = i * 64 + lane;
    const int64_t a = t0 + w - nw;
    const bool in = l0 + w < row_words;                           // inside a narrow shard's width
    const uint64_t x = (in && a >= 0 && a < row_words) ? sp[a] : 0ull;
    uint64_t r = x;
    if (sh) {
      const uint64_t y = (in && a - 1 >= 0 && a - 1 < row_words) ? sp[a - 1] : 0ull;
      r = (x << sh) | (y >> (64 - sh));
    }
    dst[w] = r;
    c += __popcll(r);
  }
  const int64_t tot = int64_t(__ockl_wfred_add_i64(long(c)));
  if (lane == 0) {
    const int64_t key = int64_t(s) * 16 + k;
    (half ? spill_meta : main_meta)[key] =
        int64_t(k) | (int64_t(CT_BITMAP) << 4) | (tot << 6) | ((key * 512) << 23);
  }
}

__device__ __forceinline__ bool container_has(const uint16_t* payload, int64_t m, uint32_t v) {
  const int type = meta_type(m);
  const uint16_t* p = payload + meta_off16(m) * 8;
  if (type == CT_BITMAP) return (reinterpret_cast<const uint64_t*>(p)[v >> 6] >> (v & 63)) & 1;
  if (type == CT_ARRAY) {
    int lo = 0, hi = meta_n(m);  // first index with p[i] >= v
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (p[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    return lo < meta_n(m) && p[lo] == v;
  }
  const int nr = p[0];  // runs [start, last] at p[8 + 2r], p[9 + 2r]
  int lo = 0, hi = nr;  // last run with start <= v
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (p[8 + 2 * mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo > 0 && v <= p[9 + 2 * (lo - 1)];
}

__global__ __launch_bounds__(256) void rows_kernel(ViewDev v, int s0, int ns, int j, uint32_t col16,
                                                   uint8_t* __restrict__ flags) {
  // one thread per dense row, walking the shards until the row shows up
  // (hot rows stop at the first shard; rowptr reads are coalesced across d)
  const int64_t d = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (d >= v.D) return;
  for (int s = s0; s < s0 + ns; s++) {
    const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
    const int64_t base = v.shard_base[s];
    const int64_t lo = base + rp[d], hi = base + rp[d + 1];
    for (int64_t ci = lo; ci < hi; ci++) {
      const int64_t m = v.meta[ci];
      if (meta_n(m) == 0) continue;
      if (j < 0) {
        flags[d] = 1;
        return;
      }
      if (meta_j(m) == j) {
        if (container_has(v.payload, m, col16)) {
          flags[d] = 1;
          return;
        }
        break;
      }
    }
  }
}

}  // namespace

void launch_shift_dense(const uint64_t* src, int S, int M, int64_t n, int64_t row_words, uint64_t* main_out,
                        int64_t* main_meta, uint64_t* spill_out, int64_t* spill_meta, hipStream_t st) {
  const int64_t waves = int64_t(S) * 32;
  if (waves == 0 || M <= 0 || S % M || row_words <= 0 || row_words > int64_t(M) * SHARD_WORDS) return;
  hipLaunchKernelGGL(shift_dense_kernel, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, st, src, S, M, n, row_words,
                     main_out, main_meta, spill_out, spill_meta);
}

void launch_rows(const ViewDev& v, int s0, int ns, int j, uint32_t col16, uint8_t* flags, hipStream_t st) {
  if (ns == 0 || v.D == 0) return;
  hipLaunchKernelGGL(rows_kernel, dim3(unsigned((v.D + 255) / 256)), dim3(256), 0, st, v, s0, ns, j, col16, flags);
}

}  // namespace pk
