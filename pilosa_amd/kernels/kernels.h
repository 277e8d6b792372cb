// Shared host/device declarations for the gfx950 bitmap kernels.
// The byte layouts of QueryProg / ViewDev / BsiArgs are mirrored by numpy
// structured dtypes in pilosa_amd/ops/device.py (static_asserts below pin them).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pk {

constexpr int MAXLEAF = 16;
constexpr int MAXPROG = 32;
constexpr int ARRAY_MAX = 4096;
constexpr int RUN_MAX = 2048;
constexpr int CT_ARRAY = 1, CT_BITMAP = 2, CT_RUN = 3;
// opcodes: 0..MAXLEAF-1 push leaf k; then binary ops
constexpr int OP_AND = 32, OP_OR = 33, OP_XOR = 34, OP_ANDNOT = 35;

// container metadata word (see pilosa_amd/native/pyroaring.cpp)
__host__ __device__ __forceinline__ int meta_j(int64_t m) { return int(m & 15); }
__host__ __device__ __forceinline__ int meta_type(int64_t m) { return int((m >> 4) & 3); }
__host__ __device__ __forceinline__ int meta_n(int64_t m) { return int((m >> 6) & 0x1ffff); }
__host__ __device__ __forceinline__ int64_t meta_off16(int64_t m) { return int64_t(uint64_t(m) >> 23); }

struct QueryProg {
  int32_t nleaf;
  int32_t nprog;
  int32_t leaf_view[MAXLEAF];
  int64_t leaf_row[MAXLEAF];  // dense row index in the view, -1 = empty row
  uint8_t prog[MAXPROG];
  int64_t pad[3];
};
static_assert(sizeof(QueryProg) == 256, "QueryProg layout");

struct ViewDev {
  const uint32_t* rowptr;      // [S][D+1]
  const int64_t* shard_base;   // [S+1]
  const int64_t* meta;         // [C]
  const uint16_t* payload;     // [P]
  int64_t D;
  const uint16_t* keymask;     // [S][D] key-presence mask per (shard, row); nullptr = derive from meta
  // dense bitmap shadows of the view's hottest rows (pair kernels): row d's
  // key-j container in shard s as a 1024-word bitmap at
  // shadow + ((shadow_slot[d] * S + s) * 16 + j) * 1024; nullptr / -1 = none
  const uint64_t* shadow;
  const int32_t* shadow_slot;  // [D]
};
static_assert(sizeof(ViewDev) == 64, "ViewDev layout");

struct BsiArgs {
  int32_t view;
  int32_t depth;
  int64_t row_exists;
  int64_t row_sign;
  int64_t bit_row[64];
};

void launch_expr_count(const QueryProg* progs, int Q, const ViewDev* views, int S, unsigned long long* out,
                       int32_t* per_key, int64_t* per_shard, int mode, hipStream_t st);
void launch_expr_materialize(const QueryProg* progs, int Q, const ViewDev* views, int S, const int32_t* counts,
                             const int64_t* offs, uint16_t* outp, hipStream_t st);
// Count(Intersect(a, b)) via key-major pair kernels (pair_kernels.hip):
// pairs = uint2[S*16*Q] scratch, partial = int32[S*16*Q] per-(shard,key,query) counts.
// out[ti[q]] += sum over the U rows of partial[U][n] (pair-kernel partials)
void launch_partial_sum_scatter(const int32_t* partial, int64_t U, int n, const int64_t* ti, int64_t* out,
                                int64_t nout, hipStream_t st);
void launch_and2_pairs(const QueryProg* progs, int Q, const ViewDev* views, int S, uint2* pairs, int32_t* partial,
                       int cq, int variant, hipStream_t st);
// BSI predicate -> one bitmap container per (shard, key): payload u16[S*16*4096], meta int64[S*16].
// op: 0 EQ, 1 NEQ, 2 LT, 3 LTE, 4 GT, 5 GTE, 6 BETWEEN, 7 NOT NULL (values are base-relative).
// out_count != nullptr: only add the matching column count (no view is written).
void launch_bsi_range(const ViewDev* views, int S, BsiArgs bsi, int op, int64_t p1, int64_t p2, uint16_t* out_payload,
                      int64_t* out_meta, unsigned long long* out_count, hipStream_t st);
// BSI min/max descents per (shard, key): out int64[S*16*10] (see bitmap_kernels.hip).
// the [F fragments x G keys x 10] descents -> out int64[3] {value, count, found}
// part: int64[4 * ceil(F / 64)] scratch of the multi-block fold (G == 16), or nullptr
void launch_bsi_minmax_fold(const int64_t* o, int F, int G, int is_min, int64_t* out, int64_t* part,
                            hipStream_t st);
void launch_bsi_minmax(const QueryProg* progs, const ViewDev* views, int S, BsiArgs bsi, int64_t* out,
                       hipStream_t st, int which = 0);
// fmode: 0 no filters, 1 flat-fold filter programs, 2 any program.
void launch_bsi_sum(const QueryProg* progs, int Q, const ViewDev* views, int S, BsiArgs bsi,
                    unsigned long long* out_sum, unsigned long long* out_cnt, int fmode, hipStream_t st);

// Device TopN slot index (topn_kernels.hip): pass 1 counts cached-row bits per
// column into colcnt[S*2^20]; pass 2 (fill) scatters cache slots behind the
// per-shard exclusive scan colptr[S][2^20+1] (colcnt reused as cursors).
void launch_topn_index(const ViewDev& v, int S, int K, int k0, const int32_t* cache_dense, uint32_t* colcnt,
                       const uint32_t* colptr, const int64_t* entbase, uint16_t* slots, bool fill, hipStream_t st);
// Arguments of the src-TopN kernel.  Rows are addressed in an "acc space" of
// A sorted row ids (identical on every rank of a node).
struct TopNLaunch {
  ViewDev v;                      // the TopN field's view (fallback probes)
  int Q, S, K;                     // queries, shards (fragments), cache slots
  int H32, H16;                   // counter tiers: u32 < H32 <= u16 < H16 <= u8
  int64_t A;                      // acc-space size
  const int32_t* src_counts;      // [Q*S*16] materialised src containers
  const int64_t* src_offs;        // [Q*S*16] u16 offsets into src_vals
  const uint16_t* src_vals;       // array (n <= 4096) or bitmap (4096 u16)
  const uint32_t* colptr;         // [S][2^20+1] per-shard entry offsets
  const int64_t* entbase;         // [S] first slot entry of each shard
  const uint16_t* slots;          // cache slot per (column, cached row)
  int64_t slots_n;                // entries allocated (>= used + 16, multiple of 8)
  const int32_t* cache_cnt;       // [S][K] cached counts (desc), 0 = empty
  const int32_t* cache_acc;       // [S][K] acc index of each slot's row
  const int32_t* slotmap;         // [S][A] cache slot of each acc row, -1
  const int32_t* a2dense;         // [A] dense row in v, -1 = absent here
  const int32_t* ns;              // [Q] n (0 = unlimited)
  const int32_t* min_threshold;   // [Q]
  int32_t* acc;                   // mode 1: [Q][A] summed pushed counts
  const int64_t* pair_off;        // mode 2: [Q+1]
  const int32_t* pair_idx;        // mode 2: [P] acc index of each id
  unsigned long long* out;        // mode 2/3: [P] summed counts >= threshold
  uint32_t* hist_out;             // mode 1 (optional): [Q*S][words] kept histograms
  const uint32_t* hist_in;        // mode 3: histograms kept by mode 1
  int R;                          // hot ranks [0, R) counted by mode 4; slot index / histogram cover [R, K)
  const int32_t* hot_meta;        // [S][16][R] key-j container of each hot row (meta index in shard), -1
  const int32_t* hot_split;       // [S][16][2] ranks before [0] hold containers over the lane-owned bound,
                                  // before [1] the cooperative ones (bitmaps, runs, arrays > HOT_MID_N)
  uint32_t* hot_cnt;              // [S][Q][R] src counts of the hot ranks (mode 4 writes, 1-3 read)
  int32_t* tail_built;            // [Q*S] mode 1: 1 = unit's tail histogram built (kept), 0 = skipped
  const int32_t* cache_dense;     // [S][K] dense row of each cache slot (mode 3 exact probes)
  int M;                          // arena sub-shards per fragment (S fragments, S*M device shards: src, colptr,
                                  // entbase, slots, hot_meta/split are per sub-shard; mode 4 runs with S*M, M=1)
  int tbuild_min;                 // mode 4: bitmap srcs of >= this many bits build the table by transpose
  int dbg;                        // PILOSA_TOPN_DBG cost isolation: 1 skip histogram, 2 skip walk, 8 skip small hot rows,
                                  // 16 skip big hot rows, 32 skip their bitmaps, 64 skip their arrays,
                                  // 256 no lane-owned / mid atomics, 512 table skips bitmap srcs, 1024
                                  // bitmap srcs by LDS atomics (not the transposed build), 2048 skip mid-size rows, 4096
                                  // lane-owned rows load but do not count, 8192 phase 1 adds nothing to acc
                                  // (answers then wrong, except 1024)
};
// LDS bytes of the (query, shard) slot histogram (u32 / u16 / u8 tiers).
int topn_lds_bytes(int K, int H32, int H16);
// mode 1: phase-1 heap walk -> acc[Q][A] (+ hist_out); mode 2: ids= re-count
// -> out[P] (rebuilds the histograms); mode 3: ids= re-count from hist_in.
// mode 4: hot-rank count matrix hot_cnt (row-major over the batch).
void launch_topn_src(const TopNLaunch& a, int mode, hipStream_t st);
// Src containers (counts / u16 offsets into the arena payload) of plain
// rows; *has_run set when a run container needs materialising.
void launch_leaf_src(const ViewDev& v, const int64_t* rows, int Q, int S, int32_t* counts, int64_t* offs,
                     int32_t* has_run, hipStream_t st);
// shadow[r][s][j] = row rows[r]'s key-j container of shard s as a bitmap
void launch_shadow_build(const ViewDev& v, int S, const int32_t* rows, int R, uint64_t* shadow, hipStream_t st);
void launch_keymask_build(const ViewDev& v, int S, uint16_t* out, hipStream_t st);
// Row counts of (shard, dense row) entries -> out[N] (device rank caches).
void launch_row_counts(const ViewDev& v, const int32_t* shard_of, const int32_t* dense, int64_t N, int32_t* out,
                       hipStream_t st);
// out[p] = sum over shards of row dense[p]'s count where >= threshold[p] (ids= re-count, no src).
void launch_row_counts_sum(const ViewDev& v, int S, const int32_t* dense, const int32_t* threshold, int P,
                           unsigned long long* out, hipStream_t st);
// Cache-only TopN: cm[j*S + s] = candidate u[j]'s count in shard s (memoised per rank-cache prefix).
void launch_topn_cache_counts(const ViewDev& v, int S, const int32_t* u, int U, int32_t* cm, hipStream_t st);
// Cache-only TopN batch: membership, per-threshold totals and per-query top-n
// (prm = lim[Q] | mt[Q] | tsel[Q] | nq[Q] | th[T]; out[Q, KK+1], column 0 = rows kept or -2 on overflow).
void launch_topn_cache_batch(const int32_t* cnt, int K, int S, int nmax, const int32_t* inv, const int32_t* u,
                             const int32_t* cm, const int32_t* prm, int Q, int T, int U, int KK, uint8_t* member,
                             long long* tot, long long* out, hipStream_t st, int nlim = 0, int mark = 0);
// Mesh cache-only TopN: one rank's buffer [member bytes | int32 totals[T, U] | flags[2]] (cleared here;
// flags = this rank's [stale, declined] vote, which rides in the batch's one all-reduce) and the front
// end's select over the reduced buffer (out[q, 0] = -3 / -4 when some rank was stale / declined).
void launch_topn_cache_partial(const int32_t* cnt, int K, int S, int nmax, int nlim, const int32_t* inv,
                               const int32_t* cm, const int32_t* prm, int Q, int T, int U, uint8_t* member,
                               int32_t* tot, int32_t* flags, int stale, int declined, hipStream_t st);
void launch_topn_cache_select32(const uint8_t* member, const int32_t* tot, const int32_t* ids, const int32_t* prm,
                                int Q, int U, int KK, long long* out, const int32_t* flags, hipStream_t st);
void launch_topn_hot_meta(const ViewDev& v, int S, int K, int R, const int32_t* cache_dense, int32_t* hot_meta,
                          int32_t* hot_split, hipStream_t st);

// Row-pair intersection count matrix C[M][N] (int32, atomically accumulated)
// of dense bit rows A[M][KW] and B[N][KW] (u64 words), bitgemm.hip.
// mode 1: i8 MFMA (v_mfma_i32_32x32x32_i8), mode 0: VALU popcount.
void launch_bitgemm(const uint64_t* A, const uint64_t* B, int M, int N, int64_t KW, int splits, int mode,
                    int32_t* C, hipStream_t st);
// Dense bit rows of an arena: out[R][(s1-s0) * 16384] u64 for dense rows `rows`.
void launch_densify(const ViewDev& v, const int64_t* rows, int R, int s0, int s1, uint64_t* out, hipStream_t st);

// Dense one-row result views: container (q, s, j) is a bitmap at u16 offset
// ((q*S + s)*16 + j) * 4096 of outp; out_meta[(q*S + s)*16 + j] its metadata.
void launch_expr_dense(const QueryProg* progs, int Q, const ViewDev* views, int S, uint16_t* outp, int64_t* out_meta,
                       hipStream_t st);
// Shift a dense view (u64[S][16384]) up by n (0 < n < 2^20) columns per shard:
// main_out = bits that stay in the shard, spill_out = bits carried into the
// next shard (both dense, with metadata like launch_expr_dense).
void launch_shift_dense(const uint64_t* src, int S, int M, int64_t n, int64_t row_words, uint64_t* main_out,
                        int64_t* main_meta, uint64_t* spill_out, int64_t* spill_meta, hipStream_t st);
// Rows listing: flags[d] = 1 for dense rows with a non-empty container in
// shards [s0, s0 + ns) (j >= 0: only rows whose key-j container holds col16).
void launch_rows(const ViewDev& v, int s0, int ns, int j, uint32_t col16, uint8_t* flags, hipStream_t st);

// Device write path (write_kernels.hip).  merge: one workgroup per touched
// container u -> scratch[u][1024] u64 bitmap + card[u]; mode 0 applies sorted
// u16 lows dlows[dstart[u], dstart[u+1]), mode 1 the delta container dmeta[u]
// (arena metadata into dpayload, -1 none); old_meta[u] = -1 for a new
// container; nruns[u] = its number of runs.  emit: final container u at u16
// offset off16[u]*8 of payload, encoded by the reference's Optimize rule
// (run / array / bitmap), and its metadata word (-1 if empty).
void launch_container_merge(const int64_t* old_meta, const uint16_t* payload, int64_t U, const int32_t* dstart,
                            const uint16_t* dlows, const int64_t* dmeta, const uint16_t* dpayload, int mode,
                            bool clear, uint64_t* scratch, int32_t* card, int32_t* nruns, hipStream_t st);
// Copy every live container (meta type != 0) of size size16[c] 16-byte units
// from src to new_off16[c] of dst (payload compaction).
void launch_payload_compact(const int64_t* meta, int64_t C, const int64_t* new_off16, const int64_t* size16,
                            const uint16_t* src, uint16_t* dst, hipStream_t st);
void launch_container_emit(const uint64_t* scratch, const int32_t* card, const int32_t* nruns, const int64_t* off16,
                           const int32_t* jkey, int64_t U, uint16_t* payload, int64_t* meta_out, hipStream_t st);

}  // namespace pk
