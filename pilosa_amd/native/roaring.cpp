// Implementation of the host roaring core.  See roaring.hpp for the design.
// Reference behaviour: roaring/roaring.go (container kernels :2000-4963,
// file format :1052-1653, op log :4416-4559, official format :5081-5139).
#include "roaring.hpp"
#include <map>

#include <algorithm>
#include <atomic>
#include <cstdio>

namespace pr {

static inline int popc(uint64_t x) { return __builtin_popcountll(x); }

static inline uint16_t rd16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline void put16(std::string& s, uint16_t v) { s.append(reinterpret_cast<const char*>(&v), 2); }
static inline void put32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
static inline void put64(std::string& s, uint64_t v) { s.append(reinterpret_cast<const char*>(&v), 8); }

const char* const STAT_NAMES[ST_COUNT] = {
    "NewContainer",        "arrayAdd/append",          "arrayAdd/insert", "arrayAdd/arrayToBitmap",
    "bitmapRemove/bitmapToArray", "runAdd/convert",    "runRemove/convert", "optimize/toRun",
    "optimize/toArray",    "optimize/toBitmap",        "optimize/unchanged", "unionInPlace",
    "sliceContainers/Remove"};
#ifdef PILOSA_ROARING_STATS
static std::atomic<int64_t> g_stats[ST_COUNT];
void stats_hit(StatId s) { g_stats[s].fetch_add(1, std::memory_order_relaxed); }
int64_t stats_get(StatId s) { return g_stats[s].load(std::memory_order_relaxed); }
void stats_reset() {
  for (auto& x : g_stats) x.store(0, std::memory_order_relaxed);
}
#else
int64_t stats_get(StatId) { return 0; }
void stats_reset() {}
#endif

// ---------------------------------------------------------------- container

bool Container::contains(uint16_t v) const {
  switch (type) {
    case CT_ARRAY: return std::binary_search(a.begin(), a.end(), v);
    case CT_BITMAP: return (b[v >> 6] >> (v & 63)) & 1;
    case CT_RUN: {
      // first run with last >= v
      auto it = std::lower_bound(r.begin(), r.end(), v,
                                 [](const Iv& iv, uint16_t x) { return iv.last < x; });
      return it != r.end() && it->start <= v;
    }
  }
  return false;
}

void Container::to_words(uint64_t* w) const {
  switch (type) {
    case CT_ARRAY:
      for (uint16_t v : a) w[v >> 6] |= 1ull << (v & 63);
      break;
    case CT_BITMAP:
      for (int i = 0; i < BITMAP_N; i++) w[i] |= b[i];
      break;
    case CT_RUN:
      for (const Iv& iv : r) {
        uint32_t s = iv.start, e = uint32_t(iv.last) + 1;  // [s,e)
        uint32_t ws = s >> 6, we = (e - 1) >> 6;
        if (ws == we) {
          uint64_t m = (e - s == 64) ? ~0ull : (((1ull << (e - s)) - 1) << (s & 63));
          w[ws] |= m;
        } else {
          w[ws] |= ~0ull << (s & 63);
          for (uint32_t i = ws + 1; i < we; i++) w[i] = ~0ull;
          uint32_t hb = e & 63;
          w[we] |= hb ? ((1ull << hb) - 1) : ~0ull;
        }
      }
      break;
  }
}

void Container::recount() {
  switch (type) {
    case CT_ARRAY: n = int32_t(a.size()); break;
    case CT_BITMAP: {
      int32_t c = 0;
      for (int i = 0; i < BITMAP_N; i++) c += popc(b[i]);
      n = c;
      break;
    }
    case CT_RUN: {
      int32_t c = 0;
      for (const Iv& iv : r) c += int32_t(iv.last) - iv.start + 1;
      n = c;
      break;
    }
  }
}

void Container::set_words(const uint64_t* w) {
  int32_t c = 0;
  for (int i = 0; i < BITMAP_N; i++) c += popc(w[i]);
  r.clear();
  if (c <= ARRAY_MAX) {
    type = CT_ARRAY;
    b.clear();
    a.clear();
    a.reserve(c);
    for (int i = 0; i < BITMAP_N; i++) {
      uint64_t x = w[i];
      while (x) {
        int t = __builtin_ctzll(x);
        a.push_back(uint16_t(i * 64 + t));
        x &= x - 1;
      }
    }
  } else {
    type = CT_BITMAP;
    a.clear();
    b.assign(w, w + BITMAP_N);
  }
  n = c;
}

void Container::to_bitmap() {
  if (type == CT_BITMAP) return;
  std::vector<uint64_t> w(BITMAP_N, 0);
  to_words(w.data());
  a.clear();
  a.shrink_to_fit();
  r.clear();
  r.shrink_to_fit();
  b.swap(w);
  type = CT_BITMAP;
}

void Container::to_array() {
  if (type == CT_ARRAY) return;
  std::vector<uint16_t> out;
  out.reserve(n);
  if (type == CT_BITMAP) {
    for (int i = 0; i < BITMAP_N; i++) {
      uint64_t x = b[i];
      while (x) {
        out.push_back(uint16_t(i * 64 + __builtin_ctzll(x)));
        x &= x - 1;
      }
    }
  } else {
    for (const Iv& iv : r)
      for (uint32_t v = iv.start; v <= iv.last; v++) out.push_back(uint16_t(v));
  }
  b.clear();
  b.shrink_to_fit();
  r.clear();
  r.shrink_to_fit();
  a.swap(out);
  type = CT_ARRAY;
}

void Container::to_run() {
  if (type == CT_RUN) return;
  std::vector<Iv> out;
  if (type == CT_ARRAY) {
    size_t i = 0;
    while (i < a.size()) {
      uint16_t s = a[i];
      size_t j = i;
      while (j + 1 < a.size() && a[j + 1] == uint16_t(a[j] + 1)) j++;
      out.push_back({s, a[j]});
      i = j + 1;
    }
  } else {
    int v = 0;
    while (v < 65536) {
      // find next set bit
      int wi = v >> 6;
      uint64_t x = b[wi] & (~0ull << (v & 63));
      while (!x && ++wi < BITMAP_N) x = b[wi];
      if (wi >= BITMAP_N) break;
      int s = wi * 64 + __builtin_ctzll(x);
      // find next clear bit after s
      wi = s >> 6;
      uint64_t y = ~b[wi] & (~0ull << (s & 63));
      while (!y && ++wi < BITMAP_N) y = ~b[wi];
      int e = (wi >= BITMAP_N) ? 65536 : wi * 64 + __builtin_ctzll(y);
      out.push_back({uint16_t(s), uint16_t(e - 1)});
      v = e;
    }
  }
  a.clear();
  a.shrink_to_fit();
  b.clear();
  b.shrink_to_fit();
  r.swap(out);
  type = CT_RUN;
}

int Container::count_runs() const {
  switch (type) {
    case CT_RUN: return int(r.size());
    case CT_ARRAY: {
      int c = 0;
      for (size_t i = 0; i < a.size(); i++)
        if (i == 0 || a[i] != uint16_t(a[i - 1] + 1)) c++;
      return c;
    }
    case CT_BITMAP: {
      // runs = number of 0->1 transitions
      int c = 0;
      uint64_t prev_top = 0;
      for (int i = 0; i < BITMAP_N; i++) {
        uint64_t x = b[i];
        uint64_t starts = x & ~((x << 1) | prev_top);
        c += popc(starts);
        prev_top = x >> 63;
      }
      return c;
    }
  }
  return 0;
}

void Container::optimize() {
  if (n == 0) return;
  int runs = count_runs();
  uint8_t nt;
  if (runs <= RUN_MAX && runs <= n / 2) nt = CT_RUN;
  else if (n < ARRAY_MAX) nt = CT_ARRAY;
  else nt = CT_BITMAP;
  if (nt == type) {
    stats_hit(ST_OPT_UNCHANGED);
    return;
  }
  if (nt == CT_RUN) { stats_hit(ST_OPT_TO_RUN); to_run(); }
  else if (nt == CT_ARRAY) { stats_hit(ST_OPT_TO_ARRAY); to_array(); }
  else { stats_hit(ST_OPT_TO_BITMAP); to_bitmap(); }
}

bool Container::add(uint16_t v) {
  switch (type) {
    case CT_ARRAY: {
      auto it = std::lower_bound(a.begin(), a.end(), v);
      if (it != a.end() && *it == v) return false;
      if (int(a.size()) >= ARRAY_MAX) {
        stats_hit(ST_ARRAY_ADD_TO_BITMAP);
        to_bitmap();
        b[v >> 6] |= 1ull << (v & 63);
        n++;
        return true;
      }
      stats_hit(it == a.end() ? ST_ARRAY_ADD_APPEND : ST_ARRAY_ADD_INSERT);
      a.insert(it, v);
      n++;
      return true;
    }
    case CT_BITMAP: {
      uint64_t m = 1ull << (v & 63);
      if (b[v >> 6] & m) return false;
      b[v >> 6] |= m;
      n++;
      return true;
    }
    case CT_RUN: {
      if (contains(v)) return false;
      stats_hit(ST_RUN_ADD_CONVERT);
      if (n + 1 > ARRAY_MAX) to_bitmap(); else to_array();
      return add(v);
    }
  }
  return false;
}

bool Container::remove(uint16_t v) {
  switch (type) {
    case CT_ARRAY: {
      auto it = std::lower_bound(a.begin(), a.end(), v);
      if (it == a.end() || *it != v) return false;
      a.erase(it);
      n--;
      return true;
    }
    case CT_BITMAP: {
      uint64_t m = 1ull << (v & 63);
      if (!(b[v >> 6] & m)) return false;
      b[v >> 6] &= ~m;
      n--;
      if (n <= ARRAY_MAX / 2) {
        stats_hit(ST_BITMAP_REMOVE_TO_ARRAY);
        to_array();
      }
      return true;
    }
    case CT_RUN: {
      if (!contains(v)) return false;
      stats_hit(ST_RUN_REMOVE_CONVERT);
      if (n - 1 > ARRAY_MAX) to_bitmap(); else to_array();
      return remove(v);
    }
  }
  return false;
}

int32_t Container::count_range(int start, int end) const {
  if (start >= end) return 0;
  switch (type) {
    case CT_ARRAY: {
      auto lo = std::lower_bound(a.begin(), a.end(), uint32_t(start),
                                 [](uint16_t x, uint32_t y) { return uint32_t(x) < y; });
      auto hi = std::lower_bound(a.begin(), a.end(), uint32_t(end),
                                 [](uint16_t x, uint32_t y) { return uint32_t(x) < y; });
      return int32_t(hi - lo);
    }
    case CT_BITMAP: {
      int32_t c = 0;
      int ws = start >> 6, we = (end - 1) >> 6;
      if (ws == we) {
        uint64_t m = (end - start == 64) ? ~0ull : (((1ull << (end - start)) - 1) << (start & 63));
        return popc(b[ws] & m);
      }
      c += popc(b[ws] & (~0ull << (start & 63)));
      for (int i = ws + 1; i < we; i++) c += popc(b[i]);
      int hb = end & 63;
      c += popc(b[we] & (hb ? ((1ull << hb) - 1) : ~0ull));
      return c;
    }
    case CT_RUN: {
      int32_t c = 0;
      for (const Iv& iv : r) {
        int s = std::max<int>(iv.start, start), e = std::min<int>(int(iv.last) + 1, end);
        if (e > s) c += e - s;
      }
      return c;
    }
  }
  return 0;
}

int Container::max() const {
  switch (type) {
    case CT_ARRAY: return a.empty() ? -1 : a.back();
    case CT_BITMAP:
      for (int i = BITMAP_N - 1; i >= 0; i--)
        if (b[i]) return i * 64 + 63 - __builtin_clzll(b[i]);
      return -1;
    case CT_RUN: return r.empty() ? -1 : r.back().last;
  }
  return -1;
}

int Container::min() const {
  switch (type) {
    case CT_ARRAY: return a.empty() ? -1 : a.front();
    case CT_BITMAP:
      for (int i = 0; i < BITMAP_N; i++)
        if (b[i]) return i * 64 + __builtin_ctzll(b[i]);
      return -1;
    case CT_RUN: return r.empty() ? -1 : r.front().start;
  }
  return -1;
}

int Container::next_from(int v) const {
  if (v > 65535) return -1;
  switch (type) {
    case CT_ARRAY: {
      auto p = std::lower_bound(a.begin(), a.end(), uint16_t(v));
      return p == a.end() ? -1 : int(*p);
    }
    case CT_BITMAP: {
      int i = v >> 6;
      uint64_t w = b[i] & (~0ull << (v & 63));
      while (true) {
        if (w) return i * 64 + __builtin_ctzll(w);
        if (++i >= BITMAP_N) return -1;
        w = b[i];
      }
    }
    case CT_RUN:
      for (const Iv& iv : r) {  // runs are few (<= 2048); linear is fine
        if (iv.last < v) continue;
        return iv.start > v ? int(iv.start) : v;
      }
      return -1;
  }
  return -1;
}

void Iterator::seek(uint64_t v) {
  it_ = bm_->cs.lower_bound(v >> 16);
  low_ = (it_ != bm_->cs.end() && it_->first == (v >> 16)) ? int(v & 0xffff) : 0;
}

bool Iterator::next(uint64_t* v) {
  while (it_ != bm_->cs.end()) {
    int x = it_->second.n ? it_->second.next_from(low_) : -1;
    if (x >= 0) {
      *v = (it_->first << 16) | uint64_t(x);
      low_ = x + 1;
      return true;
    }
    ++it_;
    low_ = 0;
  }
  return false;
}

size_t Container::encoded_size() const {
  switch (type) {
    case CT_ARRAY: return a.size() * 2;
    case CT_BITMAP: return BITMAP_N * 8;
    case CT_RUN: return 2 + r.size() * 4;
  }
  return 0;
}

std::string Container::check() const {
  char buf[160];
  switch (type) {
    case CT_ARRAY:
      if (int(a.size()) != n) {
        snprintf(buf, sizeof buf, "array count mismatch: count=%zu, n=%d", a.size(), n);
        return buf;
      }
      for (size_t i = 1; i < a.size(); i++)
        if (a[i - 1] >= a[i]) return "array not sorted/unique";
      break;
    case CT_BITMAP: {
      if (b.size() != BITMAP_N) return "bitmap wrong length";
      int32_t c = 0;
      for (uint64_t w : b) c += popc(w);
      if (c != n) {
        snprintf(buf, sizeof buf, "bitmap count mismatch: count=%d, n=%d", c, n);
        return buf;
      }
      break;
    }
    case CT_RUN: {
      int32_t c = 0;
      for (size_t i = 0; i < r.size(); i++) {
        if (r[i].start > r[i].last) return "run start > last";
        if (i && uint32_t(r[i].start) <= uint32_t(r[i - 1].last) + 1) return "runs overlap or adjacent";
        c += int32_t(r[i].last) - r[i].start + 1;
      }
      if (c != n) {
        snprintf(buf, sizeof buf, "run count mismatch: count=%d, n=%d", c, n);
        return buf;
      }
      break;
    }
    default:
      return "invalid container type";
  }
  return "";
}

// ---------------------------------------------------------------- pairwise

// word buffers of the pairwise ops live on the stack (8 KiB each): no heap
// allocation per container pair
static Container from_words_vec(const uint64_t* w) {
  Container c;
  c.set_words(w);
  return c;
}

Container c_intersect(const Container& x, const Container& y) {
  Container out;
  if (x.n == 0 || y.n == 0) return out;
  if (x.type == CT_ARRAY && y.type == CT_ARRAY) {
    out.a.reserve(std::min(x.a.size(), y.a.size()));
    std::set_intersection(x.a.begin(), x.a.end(), y.a.begin(), y.a.end(), std::back_inserter(out.a));
    out.n = int32_t(out.a.size());
    return out;
  }
  if (x.type == CT_ARRAY || y.type == CT_ARRAY) {
    const Container& arr = x.type == CT_ARRAY ? x : y;
    const Container& oth = x.type == CT_ARRAY ? y : x;
    for (uint16_t v : arr.a)
      if (oth.contains(v)) out.a.push_back(v);
    out.n = int32_t(out.a.size());
    return out;
  }
  uint64_t wx[BITMAP_N] = {0}, wy[BITMAP_N] = {0};
  x.to_words(wx);
  y.to_words(wy);
  for (int i = 0; i < BITMAP_N; i++) wx[i] &= wy[i];
  return from_words_vec(wx);
}

Container c_union(const Container& x, const Container& y) {
  if (x.n == 0) return y;
  if (y.n == 0) return x;
  if (x.type == CT_ARRAY && y.type == CT_ARRAY && x.n + y.n <= ARRAY_MAX) {
    Container out;
    out.a.reserve(x.a.size() + y.a.size());
    std::set_union(x.a.begin(), x.a.end(), y.a.begin(), y.a.end(), std::back_inserter(out.a));
    out.n = int32_t(out.a.size());
    return out;
  }
  uint64_t w[BITMAP_N] = {0};
  x.to_words(w);
  y.to_words(w);
  return from_words_vec(w);
}

Container c_difference(const Container& x, const Container& y) {
  if (x.n == 0) return Container();
  if (y.n == 0) return x;
  if (x.type == CT_ARRAY) {
    Container out;
    for (uint16_t v : x.a)
      if (!y.contains(v)) out.a.push_back(v);
    out.n = int32_t(out.a.size());
    return out;
  }
  uint64_t wx[BITMAP_N] = {0}, wy[BITMAP_N] = {0};
  x.to_words(wx);
  y.to_words(wy);
  for (int i = 0; i < BITMAP_N; i++) wx[i] &= ~wy[i];
  return from_words_vec(wx);
}

Container c_xor(const Container& x, const Container& y) {
  if (x.n == 0) return y;
  if (y.n == 0) return x;
  if (x.type == CT_ARRAY && y.type == CT_ARRAY && x.n + y.n <= ARRAY_MAX) {
    Container out;
    std::set_symmetric_difference(x.a.begin(), x.a.end(), y.a.begin(), y.a.end(), std::back_inserter(out.a));
    out.n = int32_t(out.a.size());
    return out;
  }
  uint64_t wx[BITMAP_N] = {0}, wy[BITMAP_N] = {0};
  x.to_words(wx);
  y.to_words(wy);
  for (int i = 0; i < BITMAP_N; i++) wx[i] ^= wy[i];
  return from_words_vec(wx);
}

int64_t c_intersection_count(const Container& x, const Container& y) {
  if (x.n == 0 || y.n == 0) return 0;
  if (x.type == CT_ARRAY && y.type == CT_ARRAY) {
    // merge, galloping when sizes are very different
    const auto& s = x.a.size() <= y.a.size() ? x.a : y.a;
    const auto& l = x.a.size() <= y.a.size() ? y.a : x.a;
    int64_t c = 0;
    if (s.size() * 32 < l.size()) {
      auto it = l.begin();
      for (uint16_t v : s) {
        it = std::lower_bound(it, l.end(), v);
        if (it == l.end()) break;
        if (*it == v) c++;
      }
      return c;
    }
    if (s.size() >= 64) {
      // scatter the larger array into a stack bitmap and probe it with the
      // smaller one: no data-dependent branches (a merge mispredicts about
      // every other step on random arrays)
      uint64_t w[BITMAP_N];
      memset(w, 0, sizeof w);
      for (uint16_t v : l) w[v >> 6] |= 1ull << (v & 63);
      int64_t c0 = 0, c1 = 0;
      size_t i = 0;
      for (; i + 2 <= s.size(); i += 2) {
        c0 += (w[s[i] >> 6] >> (s[i] & 63)) & 1;
        c1 += (w[s[i + 1] >> 6] >> (s[i + 1] & 63)) & 1;
      }
      if (i < s.size()) c0 += (w[s[i] >> 6] >> (s[i] & 63)) & 1;
      return c0 + c1;
    }
    size_t i = 0, j = 0;
    while (i < s.size() && j < l.size()) {
      if (s[i] < l[j]) i++;
      else if (s[i] > l[j]) j++;
      else { c++; i++; j++; }
    }
    return c;
  }
  if (x.type == CT_BITMAP && y.type == CT_BITMAP) {
    int64_t c = 0;
    for (int i = 0; i < BITMAP_N; i++) c += popc(x.b[i] & y.b[i]);
    return c;
  }
  if (x.type == CT_ARRAY || y.type == CT_ARRAY) {
    const Container& arr = x.type == CT_ARRAY ? x : y;
    const Container& oth = x.type == CT_ARRAY ? y : x;
    int64_t c = 0;
    if (oth.type == CT_BITMAP) {
      // branch-free bit probes, 4 independent accumulators
      const uint64_t* w = oth.b.data();
      const uint16_t* a = arr.a.data();
      const size_t n = arr.a.size();
      int64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
      size_t i = 0;
      for (; i + 4 <= n; i += 4) {
        c0 += (w[a[i] >> 6] >> (a[i] & 63)) & 1;
        c1 += (w[a[i + 1] >> 6] >> (a[i + 1] & 63)) & 1;
        c2 += (w[a[i + 2] >> 6] >> (a[i + 2] & 63)) & 1;
        c3 += (w[a[i + 3] >> 6] >> (a[i + 3] & 63)) & 1;
      }
      for (; i < n; i++) c0 += (w[a[i] >> 6] >> (a[i] & 63)) & 1;
      return c0 + c1 + c2 + c3;
    }
    // array & run: one merge walk over the sorted values and runs
    size_t r = 0;
    for (uint16_t v : arr.a) {
      while (r < oth.r.size() && oth.r[r].last < v) r++;
      if (r == oth.r.size()) break;
      c += oth.r[r].start <= v;
    }
    return c;
  }
  // run with bitmap or run with run
  if (x.type == CT_RUN && y.type == CT_RUN) {
    int64_t c = 0;
    size_t i = 0, j = 0;
    while (i < x.r.size() && j < y.r.size()) {
      int s = std::max(x.r[i].start, y.r[j].start), e = std::min(x.r[i].last, y.r[j].last);
      if (e >= s) c += e - s + 1;
      if (x.r[i].last < y.r[j].last) i++; else j++;
    }
    return c;
  }
  const Container& run = x.type == CT_RUN ? x : y;
  const Container& bm = x.type == CT_RUN ? y : x;
  int64_t c = 0;
  for (const Iv& iv : run.r) c += bm.count_range(iv.start, int(iv.last) + 1);
  return c;
}

// ---------------------------------------------------------------- bitmap

Container& get_or_create(Bitmap& b, uint64_t key) { return b.cs[key]; }

bool Bitmap::add(uint64_t v) {
  auto it = cs.find(v >> 16);
  if (it == cs.end()) {
    stats_hit(ST_NEW_CONTAINER);
    it = cs.emplace(v >> 16, Container()).first;
  }
  return it->second.add(uint16_t(v & 0xffff));
}

bool Bitmap::remove(uint64_t v) {
  auto it = cs.find(v >> 16);
  if (it == cs.end()) return false;
  bool ch = it->second.remove(uint16_t(v & 0xffff));
  if (it->second.n == 0) {
    stats_hit(ST_CONTAINER_REMOVED);
    cs.erase(it);
  }
  return ch;
}

bool Bitmap::contains(uint64_t v) const {
  auto it = cs.find(v >> 16);
  return it != cs.end() && it->second.contains(uint16_t(v & 0xffff));
}

int64_t Bitmap::add_many(const uint64_t* v, size_t n) {
  int64_t changed = 0;
  size_t i = 0;
  while (i < n) {
    uint64_t key = v[i] >> 16;
    size_t j = i;
    while (j < n && (v[j] >> 16) == key) j++;
    Container& c = cs[key];
    if (j - i > 64 && c.type != CT_BITMAP) {
      // bulk: materialize, set, canonicalize
      std::vector<uint64_t> w(BITMAP_N, 0);
      c.to_words(w.data());
      int32_t before = c.n;
      for (size_t k = i; k < j; k++) w[(v[k] & 0xffff) >> 6] |= 1ull << (v[k] & 63);
      c.set_words(w.data());
      changed += c.n - before;
    } else {
      for (size_t k = i; k < j; k++) changed += c.add(uint16_t(v[k] & 0xffff));
    }
    i = j;
  }
  return changed;
}

int64_t Bitmap::remove_many(const uint64_t* v, size_t n) {
  int64_t changed = 0;
  for (size_t i = 0; i < n; i++) changed += remove(v[i]);
  return changed;
}

int64_t Bitmap::count() const {
  int64_t c = 0;
  for (auto& kv : cs) c += kv.second.n;
  return c;
}

int64_t Bitmap::count_range(uint64_t start, uint64_t end) const {
  if (start >= end) return 0;
  uint64_t sk = start >> 16, ek = end >> 16;
  int64_t c = 0;
  for (auto it = cs.lower_bound(sk); it != cs.end() && it->first <= ek; ++it) {
    int s = it->first == sk ? int(start & 0xffff) : 0;
    int e = it->first == ek ? int(end & 0xffff) : 65536;
    c += it->second.count_range(s, e);
  }
  return c;
}

bool Bitmap::any() const {
  for (auto& kv : cs)
    if (kv.second.n) return true;
  return false;
}

uint64_t Bitmap::max() const {
  for (auto it = cs.rbegin(); it != cs.rend(); ++it)
    if (it->second.n) return (it->first << 16) | uint64_t(it->second.max());
  return 0;
}

uint64_t Bitmap::min() const {
  for (auto& kv : cs)
    if (kv.second.n) return (kv.first << 16) | uint64_t(kv.second.min());
  return 0;
}

static void append_values(std::vector<uint64_t>& out, uint64_t key, const Container& c, int s, int e) {
  uint64_t base = key << 16;
  switch (c.type) {
    case CT_ARRAY:
      for (uint16_t v : c.a)
        if (v >= s && v < e) out.push_back(base | v);
      break;
    case CT_BITMAP:
      for (int i = s >> 6; i < BITMAP_N && i * 64 < e; i++) {
        uint64_t x = c.b[i];
        while (x) {
          int v = i * 64 + __builtin_ctzll(x);
          x &= x - 1;
          if (v >= s && v < e) out.push_back(base | uint64_t(v));
        }
      }
      break;
    case CT_RUN:
      for (const Iv& iv : c.r)
        for (int v = std::max<int>(iv.start, s); v <= iv.last && v < e; v++) out.push_back(base | uint64_t(v));
      break;
  }
}

std::vector<uint64_t> Bitmap::slice() const {
  std::vector<uint64_t> out;
  out.reserve(size_t(count()));
  for (auto& kv : cs) append_values(out, kv.first, kv.second, 0, 65536);
  return out;
}

std::vector<uint64_t> Bitmap::slice_range(uint64_t start, uint64_t end) const {
  std::vector<uint64_t> out;
  if (start >= end) return out;
  uint64_t sk = start >> 16, ek = end >> 16;
  for (auto it = cs.lower_bound(sk); it != cs.end() && it->first <= ek; ++it) {
    int s = it->first == sk ? int(start & 0xffff) : 0;
    int e = it->first == ek ? int(end & 0xffff) : 65536;
    append_values(out, it->first, it->second, s, e);
  }
  return out;
}

Bitmap Bitmap::offset_range(uint64_t offset, uint64_t start, uint64_t end) const {
  // reference: roaring.go:535-558 (all three must be container aligned)
  if ((offset & 0xffff) || (start & 0xffff) || (end & 0xffff))
    throw std::invalid_argument("offset_range: offset/start/end must be multiples of 65536");
  Bitmap out;
  uint64_t off = offset >> 16, sk = start >> 16, ek = end >> 16;
  for (auto it = cs.lower_bound(sk); it != cs.end() && it->first < ek; ++it)
    if (it->second.n) out.cs.emplace_hint(out.cs.end(), off + (it->first - sk), it->second);
  return out;
}

Bitmap Bitmap::sub_shard(int key_shift, uint64_t sub) const {
  if (key_shift < 4 || key_shift > 16) throw std::invalid_argument("sub_shard: key_shift must be in [4, 16]");
  const uint64_t mask = (uint64_t(1) << (key_shift - 4)) - 1;
  if (sub > mask) throw std::invalid_argument("sub_shard: sub-shard out of range");
  Bitmap out;
  for (auto& kv : cs)
    if (kv.second.n && ((kv.first >> 4) & mask) == sub)
      out.cs.emplace_hint(out.cs.end(), ((kv.first >> key_shift) << 4) | (kv.first & 15), kv.second);
  return out;
}

Bitmap Bitmap::intersect(const Bitmap& o) const {
  Bitmap out;
  auto i = cs.begin();
  auto j = o.cs.begin();
  while (i != cs.end() && j != o.cs.end()) {
    if (i->first < j->first) ++i;
    else if (i->first > j->first) ++j;
    else {
      Container c = c_intersect(i->second, j->second);
      if (c.n) out.cs.emplace_hint(out.cs.end(), i->first, std::move(c));
      ++i;
      ++j;
    }
  }
  return out;
}

Bitmap Bitmap::unite(const Bitmap& o) const {
  Bitmap out;
  auto i = cs.begin();
  auto j = o.cs.begin();
  while (i != cs.end() || j != o.cs.end()) {
    if (j == o.cs.end() || (i != cs.end() && i->first < j->first)) {
      if (i->second.n) out.cs.emplace_hint(out.cs.end(), i->first, i->second);
      ++i;
    } else if (i == cs.end() || j->first < i->first) {
      if (j->second.n) out.cs.emplace_hint(out.cs.end(), j->first, j->second);
      ++j;
    } else {
      Container c = c_union(i->second, j->second);
      if (c.n) out.cs.emplace_hint(out.cs.end(), i->first, std::move(c));
      ++i;
      ++j;
    }
  }
  return out;
}

Bitmap Bitmap::difference(const Bitmap& o) const {
  Bitmap out;
  auto j = o.cs.begin();
  for (auto i = cs.begin(); i != cs.end(); ++i) {
    while (j != o.cs.end() && j->first < i->first) ++j;
    if (j != o.cs.end() && j->first == i->first) {
      Container c = c_difference(i->second, j->second);
      if (c.n) out.cs.emplace_hint(out.cs.end(), i->first, std::move(c));
    } else if (i->second.n) {
      out.cs.emplace_hint(out.cs.end(), i->first, i->second);
    }
  }
  return out;
}

Bitmap Bitmap::xor_(const Bitmap& o) const {
  Bitmap out;
  auto i = cs.begin();
  auto j = o.cs.begin();
  while (i != cs.end() || j != o.cs.end()) {
    if (j == o.cs.end() || (i != cs.end() && i->first < j->first)) {
      if (i->second.n) out.cs.emplace_hint(out.cs.end(), i->first, i->second);
      ++i;
    } else if (i == cs.end() || j->first < i->first) {
      if (j->second.n) out.cs.emplace_hint(out.cs.end(), j->first, j->second);
      ++j;
    } else {
      Container c = c_xor(i->second, j->second);
      if (c.n) out.cs.emplace_hint(out.cs.end(), i->first, std::move(c));
      ++i;
      ++j;
    }
  }
  return out;
}

int64_t Bitmap::intersection_count(const Bitmap& o) const {
  int64_t c = 0;
  auto i = cs.begin();
  auto j = o.cs.begin();
  while (i != cs.end() && j != o.cs.end()) {
    if (i->first < j->first) ++i;
    else if (i->first > j->first) ++j;
    else {
      c += c_intersection_count(i->second, j->second);
      ++i;
      ++j;
    }
  }
  return c;
}

int64_t Bitmap::range_intersection_count(uint64_t a_start, const Bitmap& o, uint64_t b_start, uint64_t len) const {
  // |rows a ∩ b| read in place: the same container walk as intersection_count,
  // but over key windows [a_start, a_start+len) of this bitmap and
  // [b_start, b_start+len) of `o`, so no row is extracted (the reference
  // executor pays OffsetRange copies per row, fragment.go:559-580).
  if ((a_start & 0xffff) || (b_start & 0xffff) || (len & 0xffff))
    throw std::invalid_argument("range_intersection_count: starts/len must be multiples of 65536");
  const uint64_t ak = a_start >> 16, bk = b_start >> 16, nk = len >> 16;
  int64_t c = 0;
  auto i = cs.lower_bound(ak);
  auto j = o.cs.lower_bound(bk);
  while (i != cs.end() && j != o.cs.end() && i->first - ak < nk && j->first - bk < nk) {
    const uint64_t ri = i->first - ak, rj = j->first - bk;
    if (ri < rj) ++i;
    else if (ri > rj) ++j;
    else {
      c += c_intersection_count(i->second, j->second);
      ++i;
      ++j;
    }
  }
  return c;
}

int64_t Bitmap::range_union_count(const std::vector<std::pair<const Bitmap*, uint64_t>>& srcs, uint64_t len) {
  // |∪ rows| over key windows of several bitmaps (a time Row's covering views,
  // executor.go:1444-1533) without building the union: per relative key the
  // containers are OR-ed into one word buffer, a lone container is counted
  // from its cardinality.
  if (len & 0xffff) throw std::invalid_argument("range_union_count: len must be a multiple of 65536");
  const uint64_t nk = len >> 16;
  std::map<uint64_t, std::vector<const Container*>> bykey;
  for (auto& s : srcs) {
    if (s.second & 0xffff) throw std::invalid_argument("range_union_count: starts must be multiples of 65536");
    const uint64_t sk = s.second >> 16;
    for (auto it = s.first->cs.lower_bound(sk); it != s.first->cs.end() && it->first - sk < nk; ++it)
      if (it->second.n) bykey[it->first - sk].push_back(&it->second);
  }
  int64_t c = 0;
  std::vector<uint64_t> w(BITMAP_N);
  for (auto& kv : bykey) {
    if (kv.second.size() == 1) {
      c += kv.second[0]->n;
      continue;
    }
    std::fill(w.begin(), w.end(), 0);
    for (const Container* x : kv.second) x->to_words(w.data());
    for (int i = 0; i < BITMAP_N; i++) c += popc(w[i]);
  }
  return c;
}

void Bitmap::union_in_place(const std::vector<const Bitmap*>& others) {
  // N-way union: materialize per key once (reference: roaring.go:737-886)
  std::map<uint64_t, std::vector<const Container*>> bykey;
  for (const Bitmap* o : others)
    for (auto& kv : o->cs)
      if (kv.second.n) bykey[kv.first].push_back(&kv.second);
  std::vector<uint64_t> w(BITMAP_N);
  stats_hit(ST_UNION_IN_PLACE);
  for (auto& kv : bykey) {
    Container& dst = cs[kv.first];
    if (kv.second.size() == 1 && dst.n == 0) {
      dst = *kv.second[0];
      continue;
    }
    std::fill(w.begin(), w.end(), 0);
    dst.to_words(w.data());
    for (const Container* c : kv.second) c->to_words(w.data());
    dst.set_words(w.data());
  }
}

static Bitmap shift1(const Bitmap& in) {
  // shift every value up by one with carry across containers (roaring.go:944-977)
  Bitmap out;
  bool last_carry = false;
  uint64_t last_key = 0;
  std::vector<uint64_t> w(BITMAP_N);
  for (auto& kv : in.cs) {
    if (!kv.second.n) continue;
    if (last_carry && kv.first > last_key + 1) {
      Container extra;
      extra.add(0);
      out.cs.emplace_hint(out.cs.end(), last_key + 1, std::move(extra));
      last_carry = false;
    }
    std::fill(w.begin(), w.end(), 0);
    kv.second.to_words(w.data());
    bool carry = (w[BITMAP_N - 1] >> 63) & 1;
    for (int i = BITMAP_N - 1; i > 0; i--) w[i] = (w[i] << 1) | (w[i - 1] >> 63);
    w[0] = (w[0] << 1) | (last_carry ? 1ull : 0ull);
    Container c;
    c.set_words(w.data());
    if (c.n) out.cs.emplace_hint(out.cs.end(), kv.first, std::move(c));
    last_carry = carry;
    last_key = kv.first;
  }
  if (last_carry && last_key != ((1ull << 48) - 1)) {
    Container extra;
    extra.add(0);
    out.cs.emplace_hint(out.cs.end(), last_key + 1, std::move(extra));
  }
  return out;
}

Bitmap Bitmap::shift(int n) const {
  // Equivalent to n rounds of shift1 (the reference's Shift(1) loop,
  // row.go:217-239): every value moves up by n, bits past the largest
  // container key are dropped.  One pass: container k lands in keys k + n/2^16
  // and the next one, funnel-shifted by n % 2^16.
  if (n < 0) throw std::invalid_argument("shift: negative shift");
  if (n == 0) return *this;
  if (n == 1) return shift1(*this);
  constexpr uint64_t MAXKEY = (1ull << 48) - 1;
  const uint64_t nk = uint64_t(n) >> 16;
  const int rw = (n & 0xffff) >> 6, rb = n & 63;
  std::map<uint64_t, std::vector<uint64_t>> acc;
  std::vector<uint64_t> w(BITMAP_N);
  for (auto& kv : cs) {
    if (!kv.second.n) continue;
    std::fill(w.begin(), w.end(), 0);
    kv.second.to_words(w.data());
    const uint64_t k0 = kv.first + nk;
    if (k0 < kv.first || k0 > MAXKEY) continue;  // moved past the last key
    auto& lo = acc[k0];
    lo.resize(BITMAP_N, 0);
    std::vector<uint64_t>* hi = nullptr;
    if (k0 < MAXKEY) {
      hi = &acc[k0 + 1];
      hi->resize(BITMAP_N, 0);
    }
    for (int j = 0; j < BITMAP_N; j++) {
      if (!w[j]) continue;
      const int t = j + rw;
      const uint64_t a = w[j] << rb, b = rb ? (w[j] >> (64 - rb)) : 0;
      if (t < BITMAP_N) lo[t] |= a;
      else if (hi) (*hi)[t - BITMAP_N] |= a;
      if (b) {
        if (t + 1 < BITMAP_N) lo[t + 1] |= b;
        else if (hi) (*hi)[t + 1 - BITMAP_N] |= b;
      }
    }
  }
  Bitmap out;
  for (auto& kv : acc) {
    Container c;
    c.set_words(kv.second.data());
    if (c.n) out.cs.emplace_hint(out.cs.end(), kv.first, std::move(c));
  }
  return out;
}

Bitmap Bitmap::flip(uint64_t start, uint64_t end) const {
  // flip bits in [start, end] inclusive, keep everything else (roaring.go:1727)
  Bitmap out;
  if (end < start) return *this;
  uint64_t sk = start >> 16, ek = end >> 16;
  for (auto it = cs.begin(); it != cs.end() && it->first < sk; ++it)
    if (it->second.n) out.cs.emplace_hint(out.cs.end(), it->first, it->second);
  std::vector<uint64_t> w(BITMAP_N);
  for (uint64_t k = sk;; k++) {
    std::fill(w.begin(), w.end(), 0);
    auto it = cs.find(k);
    if (it != cs.end()) it->second.to_words(w.data());
    int s = k == sk ? int(start & 0xffff) : 0;
    int e = k == ek ? int(end & 0xffff) : 65535;
    for (int v = s; v <= e;) {
      if ((v & 63) == 0 && v + 63 <= e) { w[v >> 6] = ~w[v >> 6]; v += 64; }
      else { w[v >> 6] ^= 1ull << (v & 63); v++; }
    }
    Container c;
    c.set_words(w.data());
    if (c.n) out.cs.emplace_hint(out.cs.end(), k, std::move(c));
    if (k == ek) break;
  }
  for (auto it = cs.upper_bound(ek); it != cs.end(); ++it)
    if (it->second.n) out.cs.emplace_hint(out.cs.end(), it->first, it->second);
  return out;
}

void Bitmap::optimize() {
  for (auto it = cs.begin(); it != cs.end();) {
    if (it->second.n == 0) it = cs.erase(it);
    else {
      it->second.optimize();
      ++it;
    }
  }
}

void Bitmap::remove_empty() {
  for (auto it = cs.begin(); it != cs.end();) {
    if (it->second.n == 0) it = cs.erase(it);
    else ++it;
  }
}

bool Bitmap::equals(const Bitmap& o) const {
  auto i = cs.begin();
  auto j = o.cs.begin();
  std::vector<uint64_t> wx(BITMAP_N), wy(BITMAP_N);
  while (true) {
    while (i != cs.end() && i->second.n == 0) ++i;
    while (j != o.cs.end() && j->second.n == 0) ++j;
    if (i == cs.end() || j == o.cs.end()) return i == cs.end() && j == o.cs.end();
    if (i->first != j->first || i->second.n != j->second.n) return false;
    std::fill(wx.begin(), wx.end(), 0);
    std::fill(wy.begin(), wy.end(), 0);
    i->second.to_words(wx.data());
    j->second.to_words(wy.data());
    if (wx != wy) return false;
    ++i;
    ++j;
  }
}

std::string Bitmap::check() const {
  std::string errs;
  for (auto& kv : cs) {
    std::string e = kv.second.check();
    if (!e.empty()) {
      errs += std::to_string(kv.first) + "/" + e + "\n";
    }
  }
  return errs;
}

// ---------------------------------------------------------------- format

std::string Bitmap::to_bytes() {
  optimize();
  uint32_t count = 0;
  for (auto& kv : cs)
    if (kv.second.n) count++;
  std::string s;
  s.reserve(HEADER_BASE + count * 16);
  put32(s, MAGIC | (STORAGE_VERSION << 16) | (uint32_t(flags) << 24));
  put32(s, count);
  for (auto& kv : cs) {
    if (!kv.second.n) continue;
    put64(s, kv.first);
    put16(s, uint16_t(kv.second.type));
    put16(s, uint16_t(kv.second.n - 1));
  }
  uint32_t offset = HEADER_BASE + count * 16;
  for (auto& kv : cs) {
    if (!kv.second.n) continue;
    put32(s, offset);
    offset += uint32_t(kv.second.encoded_size());
  }
  for (auto& kv : cs) {
    const Container& c = kv.second;
    if (!c.n) continue;
    switch (c.type) {
      case CT_ARRAY: s.append(reinterpret_cast<const char*>(c.a.data()), c.a.size() * 2); break;
      case CT_BITMAP: s.append(reinterpret_cast<const char*>(c.b.data()), BITMAP_N * 8); break;
      case CT_RUN:
        put16(s, uint16_t(c.r.size()));
        for (const Iv& iv : c.r) {
          put16(s, iv.start);
          put16(s, iv.last);
        }
        break;
    }
  }
  return s;
}

void Bitmap::parse_pilosa(const uint8_t* data, size_t n, size_t* ops_offset) {
  if (n < HEADER_BASE) throw std::runtime_error("data too small");
  uint32_t magic = rd16(data);
  if (magic != MAGIC) throw std::runtime_error("invalid roaring file, magic number " + std::to_string(magic) + " is incorrect");
  if (data[2] != STORAGE_VERSION)
    throw std::runtime_error("wrong roaring version, file is v" + std::to_string(data[2]) + ", server requires v0");
  flags = data[3];
  uint32_t keyn = rd32(data + 4);
  // the reference's wording (roaring.go:1581-1583), its count included (keyN / 12)
  if (size_t(HEADER_BASE) + size_t(keyn) * 12 > n)
    throw std::runtime_error("malformed bitmap, key-cardinality not provided for " + std::to_string(keyn / 12) +
                             " containers");
  if (size_t(HEADER_BASE) + size_t(keyn) * 16 > n)
    throw std::runtime_error("malformed bitmap, offsets not provided for " + std::to_string(keyn) + " containers");
  cs.clear();
  const uint8_t* hdr = data + HEADER_BASE;
  const uint8_t* offs = hdr + size_t(keyn) * 12;
  size_t end = HEADER_BASE + size_t(keyn) * 16;
  for (uint32_t i = 0; i < keyn; i++) {
    uint64_t key = rd64(hdr + i * 12);
    uint8_t typ = uint8_t(rd16(hdr + i * 12 + 8));
    int32_t cn = int32_t(rd16(hdr + i * 12 + 10)) + 1;
    uint32_t off = rd32(offs + i * 4);
    if (off >= n) throw std::runtime_error("offset out of bounds: off=" + std::to_string(off) + ", len=" + std::to_string(n));
    Container c;
    c.type = typ;
    c.n = cn;
    switch (typ) {
      case CT_ARRAY:
        if (off + size_t(cn) * 2 > n) throw std::runtime_error("array container overruns data");
        c.a.resize(cn);
        memcpy(c.a.data(), data + off, size_t(cn) * 2);
        end = off + size_t(cn) * 2;
        break;
      case CT_BITMAP:
        if (off + BITMAP_N * 8 > n) throw std::runtime_error("bitmap container overruns data");
        c.b.resize(BITMAP_N);
        memcpy(c.b.data(), data + off, BITMAP_N * 8);
        end = off + BITMAP_N * 8;
        break;
      case CT_RUN: {
        if (off + 2 > n) throw std::runtime_error("run container overruns data");
        uint16_t nr = rd16(data + off);
        if (off + 2 + size_t(nr) * 4 > n) throw std::runtime_error("run container overruns data");
        c.r.resize(nr);
        for (uint16_t k = 0; k < nr; k++) {
          c.r[k].start = rd16(data + off + 2 + k * 4);
          c.r[k].last = rd16(data + off + 4 + k * 4);
        }
        end = off + 2 + size_t(nr) * 4;
        break;
      }
      default:
        throw std::runtime_error("unknown container type " + std::to_string(typ));
    }
    cs.emplace_hint(cs.end(), key, std::move(c));
  }
  *ops_offset = end;
}

void Bitmap::parse_official(const uint8_t* data, size_t n) {
  // errors in the header read "reading roaring header: ...", errors past it
  // "reading offsets from official roaring format: ..." (roaring.go:5141-5245)
  auto header_err = [](const std::string& m) { return std::runtime_error("reading roaring header: " + m); };
  auto offset_err = [](const std::string& m) {
    return std::runtime_error("reading offsets from official roaring format: " + m);
  };
  if (n < 8) throw header_err("buffer too small, expecting at least 8 bytes, was " + std::to_string(n));
  uint32_t cookie = rd32(data);
  size_t pos = 4;
  uint32_t size;
  bool have_runs = false;
  const uint8_t* isrun = nullptr;
  if (cookie == OFFICIAL_NORUN) {
    size = rd32(data + pos);
    pos += 4;
  } else if ((cookie & 0xffff) == OFFICIAL_RUN) {
    have_runs = true;
    size = (cookie >> 16) + 1;
    size_t rb = (size + 7) / 8;
    if (pos + rb > n) throw header_err("malformed bitmap, is-run bitmap overruns buffer at " + std::to_string(pos + rb));
    isrun = data + pos;
    pos += rb;
  } else {
    throw header_err("did not find expected serialCookie in header");
  }
  if (size > 65536) throw header_err("it is logically impossible to have more than (1<<16) containers");
  if (pos + size_t(size) * 4 >= n)
    throw header_err("malformed bitmap, key-cardinality slice overruns buffer at " + std::to_string(pos + size_t(size) * 4));
  const uint8_t* hdr = data + pos;
  pos += size_t(size) * 4;
  const uint8_t* offs = nullptr;
  if (!have_runs || size >= 4) {
    if (pos + size_t(size) * 4 > n) throw offset_err("offset incomplete: len=" + std::to_string((n - pos) % 4));
    offs = data + pos;
    pos += size_t(size) * 4;
  } else if (pos + 2 > n) {
    throw offset_err("offset incomplete: len=" + std::to_string(n));
  }
  cs.clear();
  size_t cur = pos;
  for (uint32_t i = 0; i < size; i++) {
    uint16_t key = rd16(hdr + i * 4);
    int32_t card = int32_t(rd16(hdr + i * 4 + 2)) + 1;
    bool run = have_runs && (isrun[i / 8] >> (i % 8)) & 1;
    if (offs) {
      cur = rd32(offs + i * 4);
      if (cur >= n)
        throw offset_err("offset out of bounds: off=" + std::to_string(cur) + ", len=" + std::to_string(n));
    }
    Container c;
    c.n = card;
    if (run) {
      if (cur + 2 > n) throw offset_err("run container overruns buffer");
      uint16_t nr = rd16(data + cur);
      cur += 2;
      if (cur + size_t(nr) * 4 > n) throw offset_err("run container overruns buffer");
      c.type = CT_RUN;
      c.r.resize(nr);
      for (uint16_t k = 0; k < nr; k++) {
        uint16_t s = rd16(data + cur + k * 4), len = rd16(data + cur + k * 4 + 2);
        c.r[k].start = s;
        c.r[k].last = uint16_t(s + len);
      }
      cur += size_t(nr) * 4;
    } else if (card <= ARRAY_MAX) {
      if (cur + size_t(card) * 2 > n) throw offset_err("array container overruns buffer");
      c.type = CT_ARRAY;
      c.a.resize(card);
      memcpy(c.a.data(), data + cur, size_t(card) * 2);
      cur += size_t(card) * 2;
    } else {
      if (cur + BITMAP_N * 8 > n) throw offset_err("bitmap container overruns buffer");
      c.type = CT_BITMAP;
      c.b.resize(BITMAP_N);
      memcpy(c.b.data(), data + cur, BITMAP_N * 8);
      cur += BITMAP_N * 8;
    }
    c.recount();
    cs.emplace_hint(cs.end(), uint64_t(key), std::move(c));
  }
}

uint32_t fnv32a(const uint8_t* p, size_t n, uint32_t h) {
  for (size_t i = 0; i < n; i++) {
    h ^= p[i];
    h *= 16777619u;
  }
  return h;
}

std::string encode_op(uint8_t typ, uint64_t value, const uint64_t* values, size_t nvalues,
                      const std::string& roaring, uint32_t opn) {
  std::string buf;
  buf.push_back(char(typ));
  switch (typ) {
    case OP_ADD:
    case OP_REMOVE:
      put64(buf, value);
      put32(buf, 0);
      break;
    case OP_ADD_BATCH:
    case OP_REMOVE_BATCH:
      put64(buf, uint64_t(nvalues));
      put32(buf, 0);
      buf.append(reinterpret_cast<const char*>(values), nvalues * 8);
      break;
    case OP_ADD_ROARING:
    case OP_REMOVE_ROARING:
      put64(buf, uint64_t(roaring.size()));
      put32(buf, 0);
      put32(buf, opn);
      break;
    default:
      throw std::invalid_argument("can't marshal unknown op type");
  }
  const uint8_t* p = reinterpret_cast<const uint8_t*>(buf.data());
  uint32_t h = fnv32a(p, 9);
  h = fnv32a(p + 13, buf.size() - 13, h);
  if (typ == OP_ADD_ROARING || typ == OP_REMOVE_ROARING)
    h = fnv32a(reinterpret_cast<const uint8_t*>(roaring.data()), roaring.size(), h);
  memcpy(&buf[9], &h, 4);
  if (typ == OP_ADD_ROARING || typ == OP_REMOVE_ROARING) buf += roaring;
  return buf;
}

void Bitmap::replay_ops(const uint8_t* data, size_t n) {
  size_t pos = 0;
  while (pos < n) {
    const uint8_t* p = data + pos;
    size_t rem = n - pos;
    if (rem < 13) throw std::runtime_error("op data out of bounds: len=" + std::to_string(rem));
    uint8_t typ = p[0];
    uint64_t value = rd64(p + 1);
    uint32_t h = fnv32a(p, 9);
    size_t sz = 13;
    switch (typ) {
      case OP_ADD:
      case OP_REMOVE:
        break;
      case OP_ADD_BATCH:
      case OP_REMOVE_BATCH:
        if (value > (1ull << 59)) throw std::runtime_error("maximum operation size exceeded");
        if (rem < 13 + value * 8) throw std::runtime_error("op data truncated");
        h = fnv32a(p + 13, value * 8, h);
        sz = 13 + value * 8;
        break;
      case OP_ADD_ROARING:
      case OP_REMOVE_ROARING:
        if (rem < 17 + value) throw std::runtime_error("op data truncated");
        h = fnv32a(p + 13, 4 + value, h);
        sz = 17 + value;
        break;
      default:
        throw std::runtime_error("unknown op type: " + std::to_string(typ));
    }
    if (rd32(p + 9) != h) {
      char b[96];
      snprintf(b, sizeof b, "checksum mismatch: type %d, exp=%08x, got=%08x", typ, h, rd32(p + 9));
      throw std::runtime_error(b);
    }
    switch (typ) {
      case OP_ADD: add(value); opn += 1; break;
      case OP_REMOVE: remove(value); opn += 1; break;
      case OP_ADD_BATCH:
      case OP_REMOVE_BATCH: {
        std::vector<uint64_t> vals(value);
        memcpy(vals.data(), p + 13, value * 8);
        if (typ == OP_ADD_BATCH) {
          std::vector<uint64_t> sorted(vals);
          std::sort(sorted.begin(), sorted.end());
          add_many(sorted.data(), sorted.size());
        } else {
          remove_many(vals.data(), vals.size());
        }
        opn += int64_t(value);
        break;
      }
      case OP_ADD_ROARING:
      case OP_REMOVE_ROARING:
        import_roaring(p + 17, value, typ == OP_REMOVE_ROARING, 16, nullptr);
        opn += rd32(p + 13);
        break;
    }
    ops++;
    pos += sz;
  }
}

void Bitmap::from_bytes(const uint8_t* data, size_t n) {
  ops = 0;
  opn = 0;
  if (n == 0) {
    cs.clear();
    return;
  }
  if (n >= 2 && rd16(data) == MAGIC) {
    try {
      size_t off = 0;
      parse_pilosa(data, n, &off);
      replay_ops(data + off, n - off);
    } catch (const std::runtime_error& e) {
      throw std::runtime_error(std::string("unmarshaling as pilosa roaring: ") + e.what());
    }
  } else {
    parse_official(data, n);   // anything else is read as the official format
  }
}

int64_t Bitmap::import_roaring(const uint8_t* data, size_t n, bool clear, uint64_t cpr,
                               std::map<uint64_t, int64_t>* rowdelta) {
  // reference: roaring.go:1463-1558 (ImportRoaringBits)
  Bitmap src;
  uint32_t magic = n >= 2 ? rd16(data) : 0;
  if (magic == MAGIC) {
    size_t off = 0;
    src.parse_pilosa(data, n, &off);
  } else {
    src.parse_official(data, n);
  }
  int64_t changed = 0;
  if (cpr == 0) cpr = 1;
  for (auto& kv : src.cs) {
    if (!kv.second.n) continue;
    int64_t delta;
    if (clear) {
      auto it = cs.find(kv.first);
      if (it == cs.end()) continue;
      int32_t before = it->second.n;
      Container c = c_difference(it->second, kv.second);
      delta = int64_t(c.n) - before;
      if (c.n) it->second = std::move(c);
      else cs.erase(it);
    } else {
      Container& dst = cs[kv.first];
      int32_t before = dst.n;
      dst = c_union(dst, kv.second);
      delta = int64_t(dst.n) - before;
    }
    if (delta) {
      changed += delta < 0 ? -delta : delta;
      if (rowdelta) (*rowdelta)[kv.first / cpr] += delta;
    }
  }
  return changed;
}

}  // namespace pr
