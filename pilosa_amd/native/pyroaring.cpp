// pybind11 bindings for the host roaring core (module pilosa_amd._roaring).
//
// Besides the Bitmap API used by the fragment layer, this module builds the
// per-device container arena (build_arena) that the HIP kernels consume and
// converts device result containers back into host bitmaps
// (bitmap_from_containers).  Arena layout (one per field-view per GPU):
//
//   rows      u64[D]        sorted distinct row ids present in any local shard
//   rowptr    u32[S*(D+1)]  per shard, CSR offsets (relative to shard_base[s])
//                           of the first container of each row
//   shard_base i64[S+1]     first container index of each shard
//   meta      i64[C]        packed container descriptor:
//                             bits 0-3   j    = key % 16 (container within row)
//                             bits 4-5   type (1 array, 2 bitmap, 3 run)
//                             bits 6-22  n    = cardinality (1..65536)
//                             bits 23-63 payload offset in 16-byte units
//   payload   u16[P]        array: n values (padded to 8); bitmap: 4096 u16
//                           (1024 little-endian u64 words); run: 8-u16 header
//                           (nruns at [0]) then (start,last) pairs, padded.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <structmember.h>  // PyMemberDef (T_OBJECT_EX): make_pairs

#include <algorithm>
#include <queue>
#include <atomic>
#include <cmath>
#include <thread>

#include "roaring.hpp"
#include "synth.hpp"

namespace py = pybind11;

#ifndef PILOSA_ROARING_MODULE
#define PILOSA_ROARING_MODULE _roaring
#endif
using pr::Bitmap;
using pr::Container;

using u64arr = py::array_t<uint64_t, py::array::c_style | py::array::forcecast>;

static u64arr to_np(const std::vector<uint64_t>& v) {
  u64arr out(v.size());
  if (!v.empty()) memcpy(out.mutable_data(), v.data(), v.size() * 8);
  return out;
}

static size_t payload_u16(const Container& c) {
  switch (c.type) {
    case pr::CT_ARRAY: return (c.a.size() + 7) & ~size_t(7);
    case pr::CT_BITMAP: return 4096;
    case pr::CT_RUN: return 8 + ((c.r.size() * 2 + 7) & ~size_t(7));
  }
  return 0;
}

static void write_payload(const Container& c, uint16_t* dst) {
  switch (c.type) {
    case pr::CT_ARRAY:
      memcpy(dst, c.a.data(), c.a.size() * 2);
      break;
    case pr::CT_BITMAP:
      memcpy(dst, c.b.data(), 8192);
      break;
    case pr::CT_RUN:
      dst[0] = uint16_t(c.r.size());
      for (size_t i = 0; i < c.r.size(); i++) {
        dst[8 + 2 * i] = c.r[i].start;
        dst[9 + 2 * i] = c.r[i].last;
      }
      break;
  }
}

static py::tuple build_arena(std::vector<py::object> shards, uint64_t cpr, int nthreads) {
  // cpr = containers per row of the source bitmaps (ShardWidth / 2^16): 16
  // for 2^20-column shards, 1..8 for narrower ones (their rows use the first
  // cpr of the arena's 16 container slots)
  if (cpr == 0 || cpr > 16 || (cpr & (cpr - 1)))
    throw std::invalid_argument("build_arena: containers per row must be a power of two <= 16");
  size_t S = shards.size();
  std::vector<const Bitmap*> bms(S, nullptr);
  for (size_t s = 0; s < S; s++)
    if (!shards[s].is_none()) bms[s] = shards[s].cast<const Bitmap*>();

  // distinct rows
  std::vector<uint64_t> rows;
  for (size_t s = 0; s < S; s++) {
    if (!bms[s]) continue;
    uint64_t last = ~0ull;
    for (auto& kv : bms[s]->cs) {
      if (!kv.second.n) continue;
      uint64_t r = kv.first / cpr;
      if (r != last) rows.push_back(r), last = r;
    }
  }
  std::sort(rows.begin(), rows.end());
  rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
  size_t D = rows.size();

  // container counts per shard + payload sizes
  std::vector<int64_t> shard_base(S + 1, 0), pay_base(S + 1, 0);
  for (size_t s = 0; s < S; s++) {
    int64_t nc = 0, np = 0;
    if (bms[s])
      for (auto& kv : bms[s]->cs)
        if (kv.second.n) nc++, np += int64_t(payload_u16(kv.second));
    shard_base[s + 1] = shard_base[s] + nc;
    pay_base[s + 1] = pay_base[s] + np;
  }
  int64_t C = shard_base[S], P = pay_base[S];
  py::array_t<uint64_t> rows_np(D);
  if (D) memcpy(rows_np.mutable_data(), rows.data(), D * 8);
  py::array_t<uint32_t> rowptr({(py::ssize_t)S, (py::ssize_t)(D + 1)});
  py::array_t<int64_t> sb(S + 1);
  memcpy(sb.mutable_data(), shard_base.data(), (S + 1) * 8);
  py::array_t<int64_t> meta(std::max<int64_t>(C, 1));
  py::array_t<uint16_t> payload(std::max<int64_t>(P, 8));
  uint32_t* rp = rowptr.mutable_data();
  int64_t* mp = meta.mutable_data();
  uint16_t* pp = payload.mutable_data();
  memset(pp, 0, size_t(std::max<int64_t>(P, 8)) * 2);
  if (C == 0) mp[0] = 0;

  auto work = [&](size_t s0, size_t s1) {
    for (size_t s = s0; s < s1; s++) {
      uint32_t* rps = rp + s * (D + 1);
      int64_t ci = 0, pi = pay_base[s];
      size_t d = 0;
      if (bms[s]) {
        for (auto& kv : bms[s]->cs) {
          const Container& c = kv.second;
          if (!c.n) continue;
          uint64_t r = kv.first / cpr;
          while (d < D && rows[d] < r) rps[d++] = uint32_t(ci);
          if (d < D && rows[d] == r) rps[d++] = uint32_t(ci);  // first container of row r
          // (subsequent containers of the same row do not advance d)
          uint64_t j = kv.first % cpr;
          uint64_t m = j | (uint64_t(c.type) << 4) | (uint64_t(c.n) << 6) | (uint64_t(pi / 8) << 23);
          mp[shard_base[s] + ci] = int64_t(m);
          write_payload(c, pp + pi);
          pi += int64_t(payload_u16(c));
          ci++;
        }
      }
      while (d <= D) rps[d++] = uint32_t(ci);
    }
  };
  {
    py::gil_scoped_release nogil;
    int nt = std::max(1, std::min<int>(nthreads, int(S)));
    std::vector<std::thread> th;
    size_t per = (S + nt - 1) / std::max(nt, 1);
    for (int t = 0; t < nt; t++) {
      size_t a = t * per, b = std::min(S, a + per);
      if (a < b) th.emplace_back(work, a, b);
    }
    for (auto& t : th) t.join();
  }
  return py::make_tuple(rows_np, rowptr, sb, meta, payload);
}

// Device results → host bitmap.  keys u64[K], types u8[K], ns i32[K],
// offs i64[K] (u16 units into payload), payload u16[].
static Bitmap bitmap_from_containers(py::array_t<uint64_t> keys, py::array_t<uint8_t> types,
                                     py::array_t<int32_t> ns, py::array_t<int64_t> offs,
                                     py::array_t<uint16_t> payload) {
  Bitmap out;
  auto K = keys.size();
  const uint64_t* kp = keys.data();
  const uint8_t* tp = types.data();
  const int32_t* np_ = ns.data();
  const int64_t* op = offs.data();
  const uint16_t* pp = payload.data();
  for (py::ssize_t i = 0; i < K; i++) {
    if (np_[i] <= 0) continue;
    Container c;
    c.type = tp[i];
    c.n = np_[i];
    const uint16_t* src = pp + op[i];
    if (c.type == pr::CT_ARRAY) {
      c.a.assign(src, src + c.n);
    } else if (c.type == pr::CT_BITMAP) {
      c.b.resize(pr::BITMAP_N);
      memcpy(c.b.data(), src, 8192);
      c.recount();
      if (c.n == 0) continue;
    } else {
      throw std::invalid_argument("bitmap_from_containers: unsupported type");
    }
    out.cs[kp[i]] = std::move(c);
  }
  return out;
}


// ------------------------------------------------------------------ synthetic data
// Generator and per-shard arena builder: synth.hpp.
using synth::Rng;
using synth::ShardOut;
using synth::mix3;

// Concatenate per-shard outputs into (rows, rowptr[S][R+1], shard_base, meta, payload).
static py::tuple concat_arena(std::vector<ShardOut>& outs, const std::vector<uint64_t>& rows, int nthreads) {
  const int64_t S = int64_t(outs.size());
  const int64_t R = int64_t(rows.size());
  // concatenate
  std::vector<int64_t> sb(S + 1, 0), pb(S + 1, 0);
  for (int64_t s = 0; s < S; s++) {
    sb[s + 1] = sb[s] + int64_t(outs[s].meta.size());
    pb[s + 1] = pb[s] + int64_t(outs[s].payload.size());
  }
  py::array_t<uint64_t> rows_np(R);
  for (int64_t r = 0; r < R; r++) rows_np.mutable_data()[r] = rows[r];
  py::array_t<uint32_t> rowptr({(py::ssize_t)S, (py::ssize_t)(R + 1)});
  py::array_t<int64_t> sbn(S + 1);
  memcpy(sbn.mutable_data(), sb.data(), (S + 1) * 8);
  py::array_t<int64_t> meta(std::max<int64_t>(sb[S], 1));
  py::array_t<uint16_t> payload(std::max<int64_t>(pb[S], 8));
  {
    py::gil_scoped_release nogil;
    uint32_t* rp = rowptr.mutable_data();
    int64_t* mp = meta.mutable_data();
    uint16_t* pp = payload.mutable_data();
    if (sb[S] == 0) mp[0] = 0;
    if (pb[S] == 0) memset(pp, 0, 16);
    std::vector<std::thread> th;
    std::atomic<int64_t> next{0};
    int nt = std::max<int>(1, std::min<int64_t>(nthreads, S));
    for (int t = 0; t < nt; t++)
      th.emplace_back([&]() {
        for (;;) {
          int64_t s = next.fetch_add(1);
          if (s >= S) break;
          ShardOut& o = outs[s];
          memcpy(rp + s * (R + 1), o.rowptr.data(), (R + 1) * 4);
          const int64_t poff16 = pb[s] / 8;
          for (size_t i = 0; i < o.meta.size(); i++) {
            uint64_t m = uint64_t(o.meta[i]);
            uint64_t off = (m >> 23) + uint64_t(poff16);
            mp[sb[s] + int64_t(i)] = int64_t((m & ((1ull << 23) - 1)) | (off << 23));
          }
          if (!o.payload.empty()) memcpy(pp + pb[s], o.payload.data(), o.payload.size() * 2);
          ShardOut().rowptr.swap(o.rowptr);
          std::vector<int64_t>().swap(o.meta);
          std::vector<uint16_t>().swap(o.payload);
        }
      });
    for (auto& t : th) t.join();
  }
  return py::make_tuple(rows_np, rowptr, sbn, meta, payload);
}

static py::tuple gen_zipf_arena(int64_t shard_lo, int64_t shard_hi, int64_t total_cols, int64_t nrows,
                                double bits_per_col, double zs, double zv, uint64_t seed, int nthreads) {
  const int64_t S = shard_hi - shard_lo;
  const int64_t R = nrows;
  const std::vector<double> dens = synth::zipf_densities(R, bits_per_col, zs, zv);
  std::vector<ShardOut> outs(S);
  {
    py::gil_scoped_release nogil;
    int nt = std::max<int>(1, std::min<int64_t>(nthreads, S));
    std::vector<std::thread> th;
    std::atomic<int64_t> next{0};
    for (int t = 0; t < nt; t++)
      th.emplace_back([&]() {
        for (;;) {
          int64_t s = next.fetch_add(1);
          if (s >= S) break;
          synth::gen_zipf_shard(outs[s], shard_lo + s, total_cols, dens, seed);
        }
      });
    for (auto& t : th) t.join();
  }
  std::vector<uint64_t> rows(R);
  for (int64_t r = 0; r < R; r++) rows[r] = uint64_t(r);
  return concat_arena(outs, rows, nthreads);
}

// Synthetic BSI arena (BASELINE config 4): a fraction `fill` of the columns
// hold a value uniform in [vmin, vmax]; rows 0 = exists, 1 = sign, 2+i = bit i
// of |value| (reference bsiExistsBit / bsiSignBit / bsiOffsetBit layout).
static py::tuple gen_bsi_arena(int64_t shard_lo, int64_t shard_hi, int64_t total_cols, int depth, double fill,
                               int64_t vmin, int64_t vmax, uint64_t seed, int nthreads) {
  if (depth < 1 || depth > 62) throw std::invalid_argument("depth must be in 1..62");
  const int64_t S = shard_hi - shard_lo;
  const int64_t R = depth + 2;
  std::vector<ShardOut> outs(S);
  auto work = [&](int64_t si) {
    synth::gen_bsi_shard(outs[si], shard_lo + si, total_cols, depth, fill, vmin, vmax, seed);
  };
  {
    py::gil_scoped_release nogil;
    int nt = std::max<int>(1, std::min<int64_t>(nthreads, S));
    std::vector<std::thread> th;
    std::atomic<int64_t> next{0};
    for (int t = 0; t < nt; t++)
      th.emplace_back([&]() {
        for (;;) {
          int64_t s = next.fetch_add(1);
          if (s >= S) break;
          work(s);
        }
      });
    for (auto& t : th) t.join();
  }
  std::vector<uint64_t> rows(R);
  for (int64_t r = 0; r < R; r++) rows[r] = uint64_t(r);
  return concat_arena(outs, rows, nthreads);
}

// Rebuild a host Bitmap for one local shard of an arena (CPU oracle / baseline).
static Bitmap arena_shard_bitmap(py::array_t<uint64_t> rows, py::array_t<uint32_t> rowptr,
                                 py::array_t<int64_t> shard_base, py::array_t<int64_t> meta,
                                 py::array_t<uint16_t> payload, int64_t s) {
  Bitmap out;
  const int64_t D = rows.size();
  const uint32_t* rp = rowptr.data() + s * (D + 1);
  const int64_t base = shard_base.data()[s];
  const int64_t* mp = meta.data();
  const uint16_t* pp = payload.data();
  for (int64_t d = 0; d < D; d++) {
    for (uint32_t c = rp[d]; c < rp[d + 1]; c++) {
      uint64_t m = uint64_t(mp[base + c]);
      int j = int(m & 15), type = int((m >> 4) & 3), n = int((m >> 6) & 0x1ffff);
      const uint16_t* src = pp + (m >> 23) * 8;
      Container ct;
      ct.type = uint8_t(type);
      ct.n = n;
      if (type == pr::CT_ARRAY) ct.a.assign(src, src + n);
      else if (type == pr::CT_BITMAP) { ct.b.resize(1024); memcpy(ct.b.data(), src, 8192); }
      else {
        int nr = src[0];
        ct.r.resize(nr);
        for (int i = 0; i < nr; i++) ct.r[i] = {src[8 + 2 * i], src[9 + 2 * i]};
      }
      out.cs.emplace_hint(out.cs.end(), rows.data()[d] * 16 + uint64_t(j), std::move(ct));
    }
  }
  return out;
}


// TopN per-shard heap replay (reference fragment.go:1568-1700 top(); same
// control flow as pilosa_amd/models/fragment.py Fragment.top with a src row):
// cache candidates in rank order, the first n counted unconditionally, then
// stop at the first candidate whose cached count is below the heap minimum.
// Intersection counts come from the device (counted[R, S] for the sorted row
// ids in counted_rows); a shard whose walk reaches an uncounted row is
// reported in need_more and contributes nothing yet.
using I64Arr = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;

static py::tuple topn_replay(I64Arr cand_rows, I64Arr cand_cnts,
                             py::array_t<int32_t, py::array::c_style | py::array::forcecast> shards, int64_t n,
                             int64_t min_threshold,
                             std::vector<std::pair<I64Arr, py::array_t<int32_t, py::array::c_style | py::array::forcecast>>> blocks,
                             int nthreads) {
  if (cand_rows.ndim() != 2 || cand_cnts.ndim() != 2)
    throw std::invalid_argument("topn_replay: 2-d candidate arrays expected");
  const int64_t S = cand_rows.shape(0), K = cand_rows.shape(1);
  if (cand_cnts.shape(0) != S || cand_cnts.shape(1) != K) throw std::invalid_argument("topn_replay: shape mismatch");
  // counted blocks: rows[r_b] with shard-major counts[S, r_b]
  struct Blk { const int64_t* rows; const int32_t* cnt; int64_t r; };
  std::vector<Blk> bl;
  int64_t maxid = -1, R = 0;
  for (auto& b : blocks) {
    if (b.second.ndim() != 2 || b.second.shape(0) != S || b.second.shape(1) != b.first.shape(0))
      throw std::invalid_argument("topn_replay: block must be (rows[r], counts[S, r])");
    Blk x{b.first.data(), b.second.data(), b.first.shape(0)};
    for (int64_t i = 0; i < x.r; i++) maxid = std::max(maxid, x.rows[i]);
    R += x.r;
    bl.push_back(x);
  }
  const int64_t* cr = cand_rows.data();
  const int64_t* cc = cand_cnts.data();
  const int32_t* sh = shards.data();
  const int64_t M = shards.shape(0);
  for (int64_t m = 0; m < M; m++)
    if (sh[m] < 0 || sh[m] >= S) throw std::out_of_range("topn_replay: shard index");
  py::array_t<bool> need(M);
  bool* needp = need.mutable_data();
  std::vector<std::vector<std::pair<int64_t, int64_t>>> res(M);
  {
    py::gil_scoped_release nogil;
    // row id -> (block, column): dense table for small ids, sorted index otherwise
    std::vector<int64_t> dense;                       // (block << 32) | col, -1 = absent
    std::vector<std::pair<int64_t, int64_t>> sorted;  // (row id, (block << 32) | col)
    if (maxid >= 0 && maxid < (int64_t(1) << 26)) {
      dense.assign(size_t(maxid + 1), -1);
      for (size_t b = 0; b < bl.size(); b++)
        for (int64_t i = 0; i < bl[b].r; i++)
          if (bl[b].rows[i] >= 0) dense[size_t(bl[b].rows[i])] = (int64_t(b) << 32) | i;
    } else {
      for (size_t b = 0; b < bl.size(); b++)
        for (int64_t i = 0; i < bl[b].r; i++) sorted.emplace_back(bl[b].rows[i], (int64_t(b) << 32) | i);
      std::sort(sorted.begin(), sorted.end());
    }
    auto loc = [&](int64_t rid) -> int64_t {
      if (!dense.empty() || sorted.empty()) return (rid >= 0 && rid <= maxid && !dense.empty()) ? dense[size_t(rid)] : -1;
      auto it = std::lower_bound(sorted.begin(), sorted.end(), std::make_pair(rid, int64_t(-1)));
      return (it == sorted.end() || it->first != rid) ? -1 : it->second;
    };
    using E = std::pair<int64_t, int64_t>;  // (count, -id): min-heap top = smallest count, then largest id
    auto walk = [&](int64_t m) {
      const int64_t s = sh[m];
      auto count_of = [&](int64_t rid, int64_t& v) -> bool {
        const int64_t l = loc(rid);
        if (l < 0) return false;
        const Blk& b = bl[size_t(l >> 32)];
        v = b.cnt[s * b.r + (l & 0xffffffff)];
        return true;
      };
      std::priority_queue<E, std::vector<E>, std::greater<E>> heap;
      bool more = false;
      for (int64_t k = 0; k < K; k++) {
        const int64_t rid = cr[s * K + k], c = cc[s * K + k];
        if (c == 0 || c < min_threshold) continue;
        int64_t v;
        if (n == 0 || int64_t(heap.size()) < n) {
          if (!count_of(rid, v)) { more = true; break; }
          if (v == 0 || v < min_threshold) continue;
          heap.emplace(v, -rid);
          continue;
        }
        const int64_t thr = heap.top().first;
        if (thr < min_threshold || c < thr) break;
        if (!count_of(rid, v)) { more = true; break; }
        if (v < thr) continue;
        heap.emplace(v, -rid);
      }
      needp[m] = more;
      if (more) return;
      auto& out = res[m];
      out.reserve(heap.size());
      while (!heap.empty()) {
        out.emplace_back(-heap.top().second, heap.top().first);
        heap.pop();
      }
    };
    const int nt = std::max<int>(1, std::min<int64_t>(nthreads, M));
    std::vector<std::thread> th;
    std::atomic<int64_t> next{0};
    for (int t = 0; t < nt; t++)
      th.emplace_back([&]() {
        for (;;) {
          const int64_t m = next.fetch_add(1);
          if (m >= M) break;
          walk(m);
        }
      });
    for (auto& t : th) t.join();
    (void)R;
  }
  size_t tot = 0;
  for (auto& r : res) tot += r.size();
  py::array_t<int64_t> ids(tot), cnts(tot);
  int64_t* ip = ids.mutable_data();
  int64_t* cp = cnts.mutable_data();
  for (auto& r : res)
    for (auto& e : r) *ip++ = e.first, *cp++ = e.second;
  return py::make_tuple(need, ids, cnts);
}

void register_arena_io(py::module_& m);  // arena_io.cpp
void register_wire_decode(py::module_& m);  // wire_decode.cpp

// Bulk construction of pilosa_amd.models.cache.Pair objects (a __slots__
// class: id, key, count) from id / count arrays.  A TopN request of 16 calls
// returns a few thousand pairs; building them through Pair.__init__ costs
// ~0.5 us each under the GIL (about 2 ms per request, more than its GPU
// work).  Here each object is allocated by the type and its three slots are
// filled directly (the member descriptors' offsets), so the objects are the
// same as __init__ would build.  Returns None when the type does not have the
// expected slot layout (the caller then builds them in Python).
// A TopN result's JSON array, [{"id":1,"count":2},...], written straight
// from the id / count arrays (Go's encoding/json layout: compact, field order
// id, count), so a columnar result never becomes Python objects on the way
// out of the HTTP handler.
static py::bytes pairs_json(u64arr ids, I64Arr counts) {
  const ssize_t n = ids.size();
  if (counts.size() != n) throw std::invalid_argument("pairs_json: ids and counts differ in length");
  const uint64_t* pi = ids.data();
  const int64_t* pc = counts.data();
  std::string out;
  out.reserve(size_t(n) * 32 + 2);
  out.push_back('[');
  char buf[64];
  for (ssize_t i = 0; i < n; i++) {
    const int k = snprintf(buf, sizeof buf, "%s{\"id\":%llu,\"count\":%lld}", i ? "," : "",
                           (unsigned long long)pi[i], (long long)pc[i]);
    out.append(buf, size_t(k));
  }
  out.push_back(']');
  return py::bytes(out);
}

static py::object make_pairs(py::object type, u64arr ids, I64Arr counts) {
  if (!PyType_Check(type.ptr())) throw std::invalid_argument("make_pairs: not a type");
  PyTypeObject* tp = reinterpret_cast<PyTypeObject*>(type.ptr());
  Py_ssize_t off[3];
  const char* names[3] = {"id", "count", "key"};
  for (int i = 0; i < 3; i++) {
    PyObject* d = PyDict_GetItemString(tp->tp_dict, names[i]);  // borrowed
    if (!d || Py_TYPE(d) != &PyMemberDescr_Type) return py::none();
    const PyMemberDef* md = reinterpret_cast<PyMemberDescrObject*>(d)->d_member;
    if (md->type != T_OBJECT_EX || md->offset <= 0 || size_t(md->offset) + sizeof(PyObject*) > size_t(tp->tp_basicsize))
      return py::none();
    off[i] = md->offset;
  }
  const ssize_t n = ids.size();
  if (counts.size() != n) throw std::invalid_argument("make_pairs: ids and counts differ in length");
  const uint64_t* pi = ids.data();
  const int64_t* pc = counts.data();
  py::list out(n);
  PyObject* empty = PyUnicode_FromString("");
  if (!empty) throw py::error_already_set();
  for (ssize_t i = 0; i < n; i++) {
    PyObject* o = tp->tp_alloc(tp, 0);
    PyObject* vid = PyLong_FromUnsignedLongLong(pi[i]);
    PyObject* vc = PyLong_FromLongLong(pc[i]);
    if (!o || !vid || !vc) {
      Py_XDECREF(o);
      Py_XDECREF(vid);
      Py_XDECREF(vc);
      Py_DECREF(empty);
      throw py::error_already_set();
    }
    *reinterpret_cast<PyObject**>(reinterpret_cast<char*>(o) + off[0]) = vid;
    *reinterpret_cast<PyObject**>(reinterpret_cast<char*>(o) + off[1]) = vc;
    Py_INCREF(empty);
    *reinterpret_cast<PyObject**>(reinterpret_cast<char*>(o) + off[2]) = empty;
    PyList_SET_ITEM(out.ptr(), i, o);
  }
  Py_DECREF(empty);
  return std::move(out);
}

PYBIND11_MODULE(PILOSA_ROARING_MODULE, m) {
  m.attr("ROARING_STATS") = pr::STATS_ENABLED;
  m.def("roaring_stats", [](bool reset) {
    py::dict d;
    for (int k = 0; k < pr::ST_COUNT; k++) d[pr::STAT_NAMES[k]] = pr::stats_get(pr::StatId(k));
    if (reset) pr::stats_reset();
    return d;
  }, py::arg("reset") = false, "container event counters (built with PILOSA_ROARING_STATS)");

  m.doc() = "Host roaring core (containers, pilosa file format, op log, device arena builder)";
  m.attr("ARRAY_MAX") = pr::ARRAY_MAX;
  m.attr("RUN_MAX") = pr::RUN_MAX;
  m.attr("MAGIC") = pr::MAGIC;

  // value iterator with Seek (reference roaring.go:1767-1982); next() returns
  // (value, eof) like the reference, and the object is a Python iterator too
  py::class_<pr::Iterator>(m, "Iterator")
      .def("seek", &pr::Iterator::seek)
      .def("next", [](pr::Iterator& it) {
        uint64_t v = 0;
        bool ok = it.next(&v);
        return py::make_tuple(v, !ok);
      })
      .def("__iter__", [](pr::Iterator& it) -> pr::Iterator& { return it; })
      .def("__next__", [](pr::Iterator& it) {
        uint64_t v = 0;
        if (!it.next(&v)) throw py::stop_iteration();
        return v;
      });

  py::class_<Bitmap>(m, "Bitmap")
      .def(py::init<>())
      .def(py::init([](u64arr vals) {
        Bitmap b;
        std::vector<uint64_t> v(vals.data(), vals.data() + vals.size());
        std::sort(v.begin(), v.end());
        b.add_many(v.data(), v.size());
        return b;
      }))
      .def("add", &Bitmap::add)
      .def("remove", &Bitmap::remove)
      .def("contains", &Bitmap::contains)
      .def("__contains__", &Bitmap::contains)
      .def("add_many", [](Bitmap& b, u64arr vals, bool sorted) {
        std::vector<uint64_t> v(vals.data(), vals.data() + vals.size());
        if (!sorted) std::sort(v.begin(), v.end());
        py::gil_scoped_release nogil;
        return b.add_many(v.data(), v.size());
      }, py::arg("values"), py::arg("sorted") = false)
      .def("remove_many", [](Bitmap& b, u64arr vals) {
        const uint64_t* p = vals.data();
        const size_t n = size_t(vals.size());
        py::gil_scoped_release nogil;
        return b.remove_many(p, n);
      })
      .def("count", &Bitmap::count)
      .def("__len__", &Bitmap::count)
      .def("count_range", &Bitmap::count_range)
      .def("any", &Bitmap::any)
      .def("max", &Bitmap::max)
      .def("min", &Bitmap::min)
      .def("iterator", [](const Bitmap& b) { return pr::Iterator(&b); }, py::keep_alive<0, 1>())
      .def("slice", [](const Bitmap& b) { return to_np(b.slice()); })
      .def("slice_range", [](const Bitmap& b, uint64_t s, uint64_t e) { return to_np(b.slice_range(s, e)); })
      .def("offset_range", &Bitmap::offset_range)
      .def("sub_shard", &Bitmap::sub_shard, py::arg("key_shift"), py::arg("sub"))
      .def("intersect", &Bitmap::intersect, py::call_guard<py::gil_scoped_release>())
      .def("union", &Bitmap::unite, py::call_guard<py::gil_scoped_release>())
      .def("difference", &Bitmap::difference, py::call_guard<py::gil_scoped_release>())
      .def("xor", &Bitmap::xor_, py::call_guard<py::gil_scoped_release>())
      .def("intersection_count", &Bitmap::intersection_count, py::call_guard<py::gil_scoped_release>())
      .def("range_intersection_count", &Bitmap::range_intersection_count, py::arg("a_start"), py::arg("other"),
           py::arg("b_start"), py::arg("length"), py::call_guard<py::gil_scoped_release>())
      .def_static("range_union_count", [](std::vector<std::pair<const Bitmap*, uint64_t>> srcs, uint64_t len) {
        py::gil_scoped_release nogil;
        return Bitmap::range_union_count(srcs, len);
      }, py::arg("sources"), py::arg("length"))
      .def("union_in_place", [](Bitmap& b, std::vector<const Bitmap*> others) {
        py::gil_scoped_release nogil;
        b.union_in_place(others);
      })
      .def("shift", &Bitmap::shift)
      .def("flip", &Bitmap::flip)
      .def("optimize", &Bitmap::optimize)
      .def("clone", [](const Bitmap& b) { return Bitmap(b); })
      .def("equals", &Bitmap::equals)
      .def("__eq__", &Bitmap::equals)
      .def("check", &Bitmap::check)
      .def_readwrite("flags", &Bitmap::flags)
      .def_readwrite("ops", &Bitmap::ops)
      .def_readwrite("opn", &Bitmap::opn)
      .def("container_count", [](const Bitmap& b) { return b.cs.size(); })
      .def("keys", [](const Bitmap& b) {
        std::vector<uint64_t> k;
        for (auto& kv : b.cs)
          if (kv.second.n) k.push_back(kv.first);
        return to_np(k);
      })
      .def("container_info", [](const Bitmap& b) {
        py::list out;
        for (auto& kv : b.cs) {
          static const char* names[] = {"nil", "array", "bitmap", "run"};
          out.append(py::make_tuple(kv.first, names[kv.second.type & 3], kv.second.n));
        }
        return out;
      })
      .def("container_runs", [](const Bitmap& b, uint64_t key) {
        // (start, last) intervals of a run container; count_runs() of any other
        // type is reported through container_run_count (debug / tests)
        std::vector<std::pair<int, int>> out;
        auto it = b.cs.find(key);
        if (it == b.cs.end() || it->second.type != pr::CT_RUN) throw std::invalid_argument("no run container at key");
        for (const auto& iv : it->second.r) out.emplace_back(iv.start, iv.last);
        return out;
      })
      .def("container_run_count", [](const Bitmap& b, uint64_t key) {
        auto it = b.cs.find(key);
        return it == b.cs.end() ? 0 : it->second.count_runs();
      })
      .def("convert_container", [](Bitmap& b, uint64_t key, const std::string& to) {
        // force the encoding of one container (the reference's arrayToRun,
        // runToBitmap, ... conversions; debug / tests)
        auto it = b.cs.find(key);
        if (it == b.cs.end()) throw std::invalid_argument("no container at key");
        if (to == "array") it->second.to_array();
        else if (to == "bitmap") it->second.to_bitmap();
        else if (to == "run") it->second.to_run();
        else throw std::invalid_argument("type must be array, bitmap or run");
      })
      .def("to_bytes", [](Bitmap& b) {
        std::string s = b.to_bytes();
        return py::bytes(s);
      })
      .def_static("from_bytes", [](py::bytes data) {
        std::string s = data;
        Bitmap b;
        b.from_bytes(reinterpret_cast<const uint8_t*>(s.data()), s.size());
        return b;
      })
      .def("load_bytes", [](Bitmap& b, py::buffer data) {
        py::buffer_info info = data.request();
        b.from_bytes(reinterpret_cast<const uint8_t*>(info.ptr), size_t(info.size * info.itemsize));
      })
      .def("import_roaring", [](Bitmap& b, py::bytes data, bool clear, uint64_t cpr) {
        std::string s = data;
        std::map<uint64_t, int64_t> rd;
        int64_t ch = b.import_roaring(reinterpret_cast<const uint8_t*>(s.data()), s.size(), clear, cpr, &rd);
        py::dict d;
        for (auto& kv : rd) d[py::int_(kv.first)] = kv.second;
        return py::make_tuple(ch, d);
      }, py::arg("data"), py::arg("clear") = false, py::arg("containers_per_row") = 16)
      .def("row_counts", [](const Bitmap& b, uint64_t cpr) {
        // count per row (row = key / cpr), used by rank-cache rebuilds
        py::dict d;
        uint64_t cur = ~0ull;
        int64_t acc = 0;
        for (auto& kv : b.cs) {
          if (!kv.second.n) continue;
          uint64_t r = kv.first / cpr;
          if (r != cur) {
            if (cur != ~0ull) d[py::int_(cur)] = acc;
            cur = r;
            acc = 0;
          }
          acc += kv.second.n;
        }
        if (cur != ~0ull) d[py::int_(cur)] = acc;
        return d;
      }, py::arg("containers_per_row") = 16)
      .def("count_rows", [](const Bitmap& b, u64arr rows, uint64_t cpr) {
        // cardinality of each given row (rows*cpr .. +cpr container keys), one
        // map lookup per row: bulk imports refresh caches without per-row calls
        const uint64_t* r = rows.data();
        const py::ssize_t n = rows.size();
        py::array_t<int64_t> out(n);
        int64_t* o = out.mutable_data();
        {
          py::gil_scoped_release nogil;
          for (py::ssize_t i = 0; i < n; i++) {
            int64_t acc = 0;
            const uint64_t k0 = r[i] * cpr;
            for (auto it = b.cs.lower_bound(k0); it != b.cs.end() && it->first < k0 + cpr; ++it) acc += it->second.n;
            o[i] = acc;
          }
        }
        return out;
      }, py::arg("rows"), py::arg("containers_per_row") = 16)
      .def("rows_with_column", [](const Bitmap& b, uint64_t col, uint64_t cpr) {
        // rows whose container at key (row*cpr + col>>16) holds col (mutex/bool vectors)
        std::vector<uint64_t> rows;
        const uint64_t j = (col >> 16) % cpr;
        const uint16_t lo = uint16_t(col & 0xffff);
        for (auto& kv : b.cs)
          if (kv.first % cpr == j && kv.second.n && kv.second.contains(lo)) rows.push_back(kv.first / cpr);
        return to_np(rows);
      }, py::arg("col"), py::arg("containers_per_row") = 16)
      .def("clear_row", [](Bitmap& b, uint64_t row, uint64_t cpr) {
        bool changed = false;
        for (uint64_t k = row * cpr; k < (row + 1) * cpr; k++) {
          auto it = b.cs.find(k);
          if (it != b.cs.end()) { changed = changed || it->second.n > 0; b.cs.erase(it); }
        }
        return changed;
      }, py::arg("row"), py::arg("containers_per_row") = 16)
      .def("set_row_from", [](Bitmap& b, uint64_t row, const Bitmap& src, uint64_t src_key0, uint64_t cpr) {
        // replace row with the containers of src keys [src_key0, src_key0+cpr)
        for (uint64_t k = row * cpr; k < (row + 1) * cpr; k++) b.cs.erase(k);
        for (auto it = src.cs.lower_bound(src_key0); it != src.cs.end() && it->first < src_key0 + cpr; ++it)
          if (it->second.n) b.cs[row * cpr + (it->first - src_key0)] = it->second;
      }, py::arg("row"), py::arg("src"), py::arg("src_key0"), py::arg("containers_per_row") = 16)
      .def("row_ids", [](const Bitmap& b, uint64_t cpr) {
        std::vector<uint64_t> rows;
        uint64_t cur = ~0ull;
        for (auto& kv : b.cs) {
          if (!kv.second.n) continue;
          uint64_t r = kv.first / cpr;
          if (r != cur) rows.push_back(r), cur = r;
        }
        return to_np(rows);
      }, py::arg("containers_per_row") = 16);

  py::class_<pr::MappedBitmap>(m, "MappedBitmap",
                               "Copy-on-write mmap view of a Pilosa fragment file (see roaring.hpp)")
      .def(py::init<const std::string&>(), py::arg("path"))
      .def("contains", &pr::MappedBitmap::contains)
      .def("__contains__", &pr::MappedBitmap::contains)
      .def("add", &pr::MappedBitmap::add)
      .def("remove", &pr::MappedBitmap::remove)
      .def("count", &pr::MappedBitmap::count)
      .def("count_range", &pr::MappedBitmap::count_range)
      .def("any", &pr::MappedBitmap::any)
      .def("max", &pr::MappedBitmap::max)
      .def("offset_range", &pr::MappedBitmap::offset_range)
      .def("sub_shard", &pr::MappedBitmap::sub_shard, py::arg("key_shift"), py::arg("sub"))
      .def("rows_with_column", [](const pr::MappedBitmap& b, uint64_t col, uint64_t cpr) {
        return to_np(b.rows_with_column(col, cpr));
      }, py::arg("col"), py::arg("containers_per_row") = 16)
      .def("count_rows", [](const pr::MappedBitmap& b, u64arr rows, uint64_t cpr) {
        const uint64_t* r = rows.data();
        const py::ssize_t n = rows.size();
        py::array_t<int64_t> out(n);
        int64_t* o = out.mutable_data();
        for (py::ssize_t i = 0; i < n; i++) o[i] = b.count_range((r[i] * cpr) << 16, ((r[i] + 1) * cpr) << 16);
        return out;
      }, py::arg("rows"), py::arg("containers_per_row") = 16)
      .def("add_many", [](pr::MappedBitmap& b, u64arr vals, bool sorted) {
        std::vector<uint64_t> v(vals.data(), vals.data() + vals.size());
        if (!sorted) std::sort(v.begin(), v.end());
        return b.add_many(v.data(), v.size());
      }, py::arg("values"), py::arg("sorted") = false)
      .def("remove_many", [](pr::MappedBitmap& b, u64arr vals) {
        std::vector<uint64_t> v(vals.data(), vals.data() + vals.size());
        std::sort(v.begin(), v.end());
        return b.remove_many(v.data(), v.size());
      })
      .def("import_roaring", [](pr::MappedBitmap& b, py::bytes data, bool clear, uint64_t cpr) {
        std::string s = data;
        std::map<uint64_t, int64_t> rd;
        int64_t ch = b.import_roaring(reinterpret_cast<const uint8_t*>(s.data()), s.size(), clear, cpr, &rd);
        py::dict d;
        for (auto& kv : rd) d[py::int_(kv.first)] = kv.second;
        return py::make_tuple(ch, d);
      }, py::arg("data"), py::arg("clear") = false, py::arg("containers_per_row") = 16)
      .def("write_snapshot", &pr::MappedBitmap::write_snapshot, py::arg("path"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("mapped_containers", &pr::MappedBitmap::mapped_containers)
      .def_property_readonly("overlay_containers", &pr::MappedBitmap::overlay_containers)
      .def_property_readonly("mapped_bytes", &pr::MappedBitmap::mapped_bytes)
      .def_readonly("flags", &pr::MappedBitmap::flags)
      .def_readonly("ops", &pr::MappedBitmap::ops)
      .def_readonly("opn", &pr::MappedBitmap::opn);

  m.def("encode_op", [](uint8_t typ, uint64_t value, u64arr values, py::bytes roaring, uint32_t opn) {
    std::string r = roaring;
    const uint64_t* p = values.data();
    const size_t n = size_t(values.size());
    std::string enc;
    {
      py::gil_scoped_release nogil;
      enc = pr::encode_op(typ, value, p, n, r, opn);
    }
    return py::bytes(enc);
  }, py::arg("typ"), py::arg("value") = 0, py::arg("values") = u64arr(0), py::arg("roaring") = py::bytes(""),
     py::arg("opn") = 0);
  m.def("make_pairs", &make_pairs, py::arg("type"), py::arg("ids"), py::arg("counts"));
  m.def("pairs_json", &pairs_json, py::arg("ids"), py::arg("counts"));
  m.def("fnv32a", [](py::bytes data) {
    std::string s = data;
    return pr::fnv32a(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  m.def("build_arena", &build_arena, py::arg("shards"), py::arg("containers_per_row") = 16,
        py::arg("nthreads") = 8);
  m.def("bitmap_from_containers", &bitmap_from_containers);
  m.def("topn_replay", &topn_replay, py::arg("cand_rows"), py::arg("cand_cnts"), py::arg("shards"), py::arg("n"),
        py::arg("min_threshold"), py::arg("blocks"), py::arg("nthreads") = 8,
        "Per-shard TopN heap replay over device-counted candidates -> (need_more, ids, counts)");
  m.def("gen_bsi_arena", &gen_bsi_arena, py::arg("shard_lo"), py::arg("shard_hi"), py::arg("total_cols"),
        py::arg("depth"), py::arg("fill"), py::arg("vmin"), py::arg("vmax"), py::arg("seed") = 1,
        py::arg("nthreads") = 8, "synthetic BSI field arena (exists, sign, bit planes)");
  m.def("gen_zipf_arena", &gen_zipf_arena, py::arg("shard_lo"), py::arg("shard_hi"), py::arg("total_cols"),
        py::arg("nrows"), py::arg("bits_per_col") = 8.0, py::arg("zipf_s") = 1.6, py::arg("zipf_v") = 50.0,
        py::arg("seed") = 1, py::arg("nthreads") = 8);
  m.def("arena_shard_bitmap", &arena_shard_bitmap);
  register_arena_io(m);
  register_wire_decode(m);
}
