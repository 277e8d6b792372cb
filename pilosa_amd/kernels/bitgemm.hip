// Pairwise row-intersection count matrices on the matrix cores.
//
//   C[m][n] = sum over bit positions k of A[m][k] * B[n][k]
//
// for two sets of dense rows A (M rows) and B (N rows) over K bits: the
// count matrix of GroupBy(Rows(a), Rows(b)) (reference groupByIterator,
// executor.go:3060-3230, which intersects row pairs one at a time) and the
// bit-plane products behind batched BSI aggregates.
//
// MODE 1 (MFMA): every 32-bit k-step of a 32x32 output tile is one
// v_mfma_i32_32x32x32_i8.  Lane (r, h) of a wave feeds 16 k-bits of row r
// (bits 16h..16h+15 of the step) as 16 bytes of 0/1; both operands use the
// same lane->k map, so the MFMA sums A[r][k] * B[c][k] over exactly those k.
// Bits become bytes through a 256-entry LDS table (8 bits -> 8 bytes, one
// ds_read_b64 per byte of input) instead of VALU shifts.
// MODE 0 (VALU): the same tiles with 64-bit AND + popcount, as the
// reference implementation of this kernel and the A/B baseline: each lane
// owns the 16 outputs the MFMA accumulator layout gives it.
//
// A workgroup (4 waves, 2x2 wave tiles) owns a 64x64 output tile and one
// K-split; A/B chunks of 512 bits per row are staged in LDS with coalesced
// 16-byte loads.  Splits add into C with int32 atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace pk {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int BT = 64;            // output tile (rows of A and of B) per workgroup

// 16 k-bits -> 16 bytes of 0/1: per nibble one 24-bit multiply spreads
// bits 0..3 to bits 0, 8, 16, 24 (x * 0x204081, no carries) and a mask keeps
// them: 3 full-rate VALU ops per 4 bits, no LDS traffic.
__device__ __forceinline__ v4i unpack16(uint32_t x) {
  v4i r;
#pragma unroll
  for (int i = 0; i < 4; i++) r[i] = int(__umul24((x >> (4 * i)) & 0xfu, 0x204081u) & 0x01010101u);
  return r;
}
constexpr int KC_WORDS = 8;       // 512 bits per row per LDS chunk
constexpr int KC_BYTES = KC_WORDS * 8;

template <int MODE>
__global__ __launch_bounds__(256) void bitgemm_kernel(const uint64_t* __restrict__ A, const uint64_t* __restrict__ B,
                                                      int M, int N, int64_t KW, int64_t kw_per_split,
                                                      int32_t* __restrict__ C) {
  __shared__ uint64_t sa[BT][KC_WORDS];
  __shared__ uint64_t sb[BT][KC_WORDS];
  __shared__ uint64_t tab[256];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tiles_n = (N + BT - 1) / BT;
  const int tile = blockIdx.x;
  const int m0 = (tile / tiles_n) * BT, n0 = (tile % tiles_n) * BT;
  const int64_t k0 = int64_t(blockIdx.y) * kw_per_split;
  const int64_t k1 = k0 + kw_per_split < KW ? k0 + kw_per_split : KW;
  if (MODE == 1) {
    uint64_t v = 0;
    for (int b = 0; b < 8; b++) v |= uint64_t((tid >> b) & 1) << (8 * b);
    tab[tid] = v;  // 256 threads = 256 entries
  }
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;  // this wave's 32x32 sub-tile
  v16i acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int cnt[16];
#pragma unroll
  for (int i = 0; i < 16; i++) cnt[i] = 0;
  // staging map: thread t loads 16 B of row (t >> 2), words 2*(t&3) .. +1
  const int srow = tid >> 2, sw = (tid & 3) * 2;
  for (int64_t kc = k0; kc < k1; kc += KC_WORDS) {
    __syncthreads();
    {
      const int64_t kw = kc + sw;
      ulong2 va = make_ulong2(0, 0), vb = make_ulong2(0, 0);
      if (m0 + srow < M && kw < k1) {
        const uint64_t* p = A + int64_t(m0 + srow) * KW + kw;
        va.x = kw < k1 ? p[0] : 0;
        va.y = kw + 1 < k1 ? p[1] : 0;
      }
      if (n0 + srow < N && kw < k1) {
        const uint64_t* p = B + int64_t(n0 + srow) * KW + kw;
        vb.x = kw < k1 ? p[0] : 0;
        vb.y = kw + 1 < k1 ? p[1] : 0;
      }
      sa[srow][sw] = va.x;
      sa[srow][sw + 1] = va.y;
      sb[srow][sw] = vb.x;
      sb[srow][sw + 1] = vb.y;
    }
    __syncthreads();
    if (MODE == 3) {
      // 64x64 workgroup tile, one 32x32 accumulator per wave, operands
      // unpacked with 24-bit multiplies (unpack16); a wave whose rows or
      // columns lie past M / N skips its MFMAs (skinny shapes, e.g. the
      // Q filters x (2 depth + 1) planes of a batched BSI Sum)
      if (m0 + wm < M && n0 + wn < N) {
        const int r = lane & 31, h = lane >> 5;
        const uint64_t* ar = &sa[wm + r][0];
        const uint64_t* br = &sb[wn + r][0];
#pragma unroll 4
        for (int ks = 0; ks < KC_WORDS * 2; ks++) {
          const uint32_t xa = uint32_t(ar[ks >> 1] >> (32 * (ks & 1))) >> (16 * h);
          const uint32_t xb = uint32_t(br[ks >> 1] >> (32 * (ks & 1))) >> (16 * h);
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(unpack16(xa), unpack16(xb), acc, 0, 0, 0);
        }
      }
    } else if (MODE == 1) {
      const int r = lane & 31, h = lane >> 5;
      const uint8_t* ar = reinterpret_cast<const uint8_t*>(&sa[wm + r][0]);
      const uint8_t* br = reinterpret_cast<const uint8_t*>(&sb[wn + r][0]);
#pragma unroll 4
      for (int ks = 0; ks < KC_BYTES / 4; ks++) {
        // k-step ks covers bytes 4ks..4ks+3 of the chunk; half h takes 2 bytes
        const int byte = 4 * ks + 2 * h;
        const uint64_t a0 = tab[ar[byte]], a1 = tab[ar[byte + 1]];
        const uint64_t b0 = tab[br[byte]], b1 = tab[br[byte + 1]];
        const v4i av = {int(uint32_t(a0)), int(uint32_t(a0 >> 32)), int(uint32_t(a1)), int(uint32_t(a1 >> 32))};
        const v4i bv = {int(uint32_t(b0)), int(uint32_t(b0 >> 32)), int(uint32_t(b1)), int(uint32_t(b1 >> 32))};
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
      }
    } else {
      // lane (c, h): output column c, rows (i&3) + 8(i>>2) + 4h of the wave tile
      const int c = lane & 31, h = lane >> 5;
#pragma unroll
      for (int w = 0; w < KC_WORDS; w++) {
        const uint64_t bw = sb[wn + c][w];
#pragma unroll
        for (int i = 0; i < 16; i++) cnt[i] += __popcll(sa[wm + (i & 3) + 8 * (i >> 2) + 4 * h][w] & bw);
      }
    }
  }
  // accumulator layout (dtype-independent on gfx950): col = lane & 31,
  // row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5)
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int m = m0 + wm + (i & 3) + 8 * (i >> 2) + 4 * h, n = n0 + wn + c;
    const int v = MODE >= 1 ? acc[i] : cnt[i];
    if (m < M && n < N && v) atomicAdd(C + int64_t(m) * N + n, v);
  }
}

// MODE 2 (MFMA, default): each wave owns a 64x64 output tile (2x2 MFMA
// accumulators), so every unpacked operand feeds two MFMAs; workgroup tile
// 128x128.
constexpr int BT2 = 128;

__global__ __launch_bounds__(256) void bitgemm_mfma64_kernel(const uint64_t* __restrict__ A,
                                                             const uint64_t* __restrict__ B, int M, int N,
                                                             int64_t KW, int64_t kw_per_split,
                                                             int32_t* __restrict__ C) {
  __shared__ uint32_t sa[BT2][KC_WORDS * 2 + 1];  // +1 dword: rows on different banks
  __shared__ uint32_t sb[BT2][KC_WORDS * 2 + 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tiles_n = (N + BT2 - 1) / BT2;
  const int m0 = (blockIdx.x / tiles_n) * BT2, n0 = (blockIdx.x % tiles_n) * BT2;
  const int64_t k0 = int64_t(blockIdx.y) * kw_per_split;
  const int64_t k1 = k0 + kw_per_split < KW ? k0 + kw_per_split : KW;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  v16i acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int i = 0; i < 16; i++) acc[a][b][i] = 0;
  const int r = lane & 31, h = lane >> 5;
  for (int64_t kc = k0; kc < k1; kc += KC_WORDS) {
    __syncthreads();
    // 128 rows x 8 words per operand: thread t stages row t>>1, words 4*(t&1)..+3
    {
      const int row = tid >> 1, w0 = (tid & 1) * 4;
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const int64_t kw = kc + w0 + w;
        const uint64_t va = (m0 + row < M && kw < k1) ? A[int64_t(m0 + row) * KW + kw] : 0ull;
        const uint64_t vb = (n0 + row < N && kw < k1) ? B[int64_t(n0 + row) * KW + kw] : 0ull;
        sa[row][2 * (w0 + w)] = uint32_t(va);
        sa[row][2 * (w0 + w) + 1] = uint32_t(va >> 32);
        sb[row][2 * (w0 + w)] = uint32_t(vb);
        sb[row][2 * (w0 + w) + 1] = uint32_t(vb >> 32);
      }
    }
    __syncthreads();
#pragma unroll 2
    for (int ks = 0; ks < KC_WORDS * 2; ks++) {
      v4i av[2], bv[2];
#pragma unroll
      for (int g = 0; g < 2; g++) {
        av[g] = unpack16(sa[wm + 32 * g + r][ks] >> (16 * h));
        bv[g] = unpack16(sb[wn + 32 * g + r][ks] >> (16 * h));
      }
#pragma unroll
      for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const int m = m0 + wm + 32 * a + (i & 3) + 8 * (i >> 2) + 4 * h, n = n0 + wn + 32 * b + r;
        const int v = acc[a][b][i];
        if (m < M && n < N && v) atomicAdd(C + int64_t(m) * N + n, v);
      }
}

// MODE 4 (MFMA, K-sliced skinny): workgroup tile 32 x 64 (rows of A x rows
// of B, e.g. the Q <= 32 filters x 2*depth+1 planes of a batched BSI Sum).
// The 4 waves do not split the tile but the k-steps of each staged chunk
// (wave w takes steps w, w+4, ...), so no wave idles on a skinny shape and
// every unpacked A operand feeds two MFMAs (both 32-column halves of B).
// The waves' accumulators are summed in LDS before one set of atomics per
// workgroup.
constexpr int K4_WORDS = 32;  // 2048 bits per row per staged chunk

__global__ __launch_bounds__(256) void bitgemm_kslice_kernel(const uint64_t* __restrict__ A,
                                                             const uint64_t* __restrict__ B, int M, int N,
                                                             int64_t KW, int64_t kw_per_split,
                                                             int32_t* __restrict__ C) {
  __shared__ uint64_t sa[32][K4_WORDS + 1];
  __shared__ uint64_t sb[64][K4_WORDS + 1];
  __shared__ int red[2][16][64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tiles_n = (N + 63) / 64;
  const int m0 = (blockIdx.x / tiles_n) * 32, n0 = (blockIdx.x % tiles_n) * 64;
  const int64_t k0 = int64_t(blockIdx.y) * kw_per_split;
  const int64_t k1 = k0 + kw_per_split < KW ? k0 + kw_per_split : KW;
  v16i acc[2];
#pragma unroll
  for (int b = 0; b < 2; b++)
#pragma unroll
    for (int i = 0; i < 16; i++) acc[b][i] = 0;
  for (int e = tid; e < 2 * 16 * 64; e += 256) (&red[0][0][0])[e] = 0;
  const int r = lane & 31, h = lane >> 5;
  for (int64_t kc = k0; kc < k1; kc += K4_WORDS) {
    __syncthreads();
    // 96 rows x 32 words: thread t stages 12 words
#pragma unroll
    for (int e = 0; e < 12; e++) {
      const int idx = e * 256 + tid;  // 0 .. 3071
      const int row = idx >> 5, w = idx & 31;
      const int64_t kw = kc + w;
      if (row < 32) {
        sa[row][w] = (m0 + row < M && kw < k1) ? A[int64_t(m0 + row) * KW + kw] : 0ull;
      } else {
        const int rb = row - 32;
        sb[rb][w] = (n0 + rb < N && kw < k1) ? B[int64_t(n0 + rb) * KW + kw] : 0ull;
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int ks = wave; ks < K4_WORDS * 2; ks += 4) {
      const int sh = 32 * (ks & 1) + 16 * h;
      const v4i av = unpack16(uint32_t(sa[r][ks >> 1] >> sh));
      const v4i b0 = unpack16(uint32_t(sb[r][ks >> 1] >> sh));
      const v4i b1 = unpack16(uint32_t(sb[32 + r][ks >> 1] >> sh));
      acc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, b1, acc[1], 0, 0, 0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 2; b++)
#pragma unroll
    for (int i = 0; i < 16; i++) atomicAdd(&red[b][i][lane], acc[b][i]);
  __syncthreads();
  // 2 x 16 x 64 = 2048 outputs, 8 per thread
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const int o = e * 256 + tid;
    const int b = o >> 10, i = (o >> 6) & 15, l = o & 63;
    const int v = red[b][i][l];
    const int m = m0 + (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), n = n0 + 32 * b + (l & 31);
    if (m < M && n < N && v) atomicAdd(C + int64_t(m) * N + n, v);
  }
}

// Dense bit rows from an arena: out[r][(s - s0) * 16384 + j * 1024 + w] for
// dense row rows[r] of view v, shards [s0, s1); absent containers are zero.
// One wave per (row, shard, key).
__global__ __launch_bounds__(256) void densify_kernel(ViewDev v, const int64_t* __restrict__ rows, int R, int s0,
                                                      int s1, uint64_t* __restrict__ out) {
  __shared__ uint64_t lbs[4][1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t item = int64_t(blockIdx.x) * 4 + wave;
  const int ns = s1 - s0;
  if (item >= int64_t(R) * ns * 16) return;
  const int j = int(item & 15);
  const int s = s0 + int((item >> 4) % ns);
  const int r = int((item >> 4) / ns);
  ulong2* dst = reinterpret_cast<ulong2*>(out + (int64_t(r) * ns + (s - s0)) * 16384 + j * 1024);
  const int64_t d = rows[r];
  int64_t m = -1;
  if (d >= 0) {
    const uint32_t* rp = v.rowptr + int64_t(s) * (v.D + 1);
    const int64_t lo = v.shard_base[s] + rp[d], hi = v.shard_base[s] + rp[d + 1];
    int64_t found = -1;
    if (lane < hi - lo && meta_j(v.meta[lo + lane]) == j) found = lo + lane;
    const uint64_t bal = __ballot(found >= 0);
    if (bal) m = v.meta[__shfl(found, int(__builtin_ctzll(bal)), 64)];
  }
  if (m < 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) dst[i * 64 + lane] = make_ulong2(0, 0);
    return;
  }
  const uint16_t* p = v.payload + meta_off16(m) * 8;
  if (meta_type(m) == CT_BITMAP) {
    const ulong2* src = reinterpret_cast<const ulong2*>(p);
#pragma unroll
    for (int i = 0; i < 8; i++) dst[i * 64 + lane] = src[i * 64 + lane];
    return;
  }
  uint64_t* lb = lbs[wave];
  for (int i = lane; i < 1024; i += 64) lb[i] = 0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (meta_type(m) == CT_ARRAY) {
    const int n = meta_n(m);
    for (int i = lane; i < n; i += 64) {
      const uint32_t x = p[i];
      atomicOr(reinterpret_cast<unsigned long long*>(&lb[x >> 6]), 1ull << (x & 63));
    }
  } else {
    const int nr = p[0];
    for (int k = 0; k < nr; k++) {
      const int a = p[8 + 2 * k], b = p[9 + 2 * k];
      for (int x = a + lane; x <= b; x += 64)
        atomicOr(reinterpret_cast<unsigned long long*>(&lb[x >> 6]), 1ull << (x & 63));
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const ulong2* l2 = reinterpret_cast<const ulong2*>(lb);
#pragma unroll
  for (int i = 0; i < 8; i++) dst[i * 64 + lane] = l2[i * 64 + lane];
}

}  // namespace

void launch_bitgemm(const uint64_t* A, const uint64_t* B, int M, int N, int64_t KW, int splits, int mode,
                    int32_t* C, hipStream_t st) {
  if (M <= 0 || N <= 0 || KW <= 0) return;
  const int bt = mode == 2 ? BT2 : BT;
  const int tiles = mode == 4 ? ((M + 31) / 32) * ((N + 63) / 64) : ((M + bt - 1) / bt) * ((N + bt - 1) / bt);
  if (splits < 1) splits = 1;
  int64_t per = (KW + splits - 1) / splits;
  const int chunk = mode == 4 ? K4_WORDS : KC_WORDS;
  per = (per + chunk - 1) / chunk * chunk;
  const int ns = int((KW + per - 1) / per);
  const dim3 grid(tiles, ns);
  if (mode == 2)
    hipLaunchKernelGGL(bitgemm_mfma64_kernel, grid, dim3(256), 0, st, A, B, M, N, KW, per, C);
  else if (mode == 3)
    hipLaunchKernelGGL(bitgemm_kernel<3>, grid, dim3(256), 0, st, A, B, M, N, KW, per, C);
  else if (mode == 4)
    hipLaunchKernelGGL(bitgemm_kslice_kernel, grid, dim3(256), 0, st, A, B, M, N, KW, per, C);
  else if (mode == 1)
    hipLaunchKernelGGL(bitgemm_kernel<1>, grid, dim3(256), 0, st, A, B, M, N, KW, per, C);
  else
    hipLaunchKernelGGL(bitgemm_kernel<0>, grid, dim3(256), 0, st, A, B, M, N, KW, per, C);
}

void launch_densify(const ViewDev& v, const int64_t* rows, int R, int s0, int s1, uint64_t* out, hipStream_t st) {
  const int64_t items = int64_t(R) * (s1 - s0) * 16;
  if (items <= 0) return;
  hipLaunchKernelGGL(densify_kernel, dim3(unsigned((items + 3) / 4)), dim3(256), 0, st, v, rows, R, s0, s1, out);
}

}  // namespace pk
