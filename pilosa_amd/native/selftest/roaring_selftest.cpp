// Randomised self-test of the C++ roaring core against std::set, meant to be
// built with -fsanitize=address,undefined (the reference runs
// its suite under `go test -race` and ships a roaring fuzzer; this is the
// native-code analogue for our host core).  Exit status 0 = pass.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../roaring.hpp"

using pr::Bitmap;

static int fails = 0;
#define EXPECT(c)                                                        \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);  \
      fails++;                                                           \
    }                                                                    \
  } while (0)

static std::vector<uint64_t> to_vec(const std::set<uint64_t>& s) { return {s.begin(), s.end()}; }

static Bitmap from_set(const std::set<uint64_t>& s) {
  Bitmap b;
  std::vector<uint64_t> v = to_vec(s);
  b.add_many(v.data(), v.size());
  return b;
}

static std::set<uint64_t> gen(std::mt19937_64& rng, int kind) {
  std::set<uint64_t> s;
  const uint64_t base = (rng() % 8) << 16;
  if (kind == 0) {  // sparse
    for (int i = 0, n = int(rng() % 3000); i < n; i++) s.insert(base + rng() % (1 << 20));
  } else if (kind == 1) {  // dense
    for (int i = 0, n = 20000 + int(rng() % 40000); i < n; i++) s.insert(base + rng() % 65536);
  } else {  // runs
    for (int r = 0; r < 30; r++) {
      const uint64_t st = base + rng() % 200000, len = 1 + rng() % 3000;
      for (uint64_t x = st; x < st + len; x++) s.insert(x);
    }
  }
  return s;
}

// Concurrent readers (the executor's host pool runs roaring ops with the GIL
// released, several threads reading the same fragment bitmaps) plus
// per-thread writers; built with -fsanitize=thread by
// tests/test_native_sanitizers.py.  Any shared mutable state in the core
// (e.g. the roaringstats counters) shows up as a data race.
static int run_threads(int nthreads) {
  std::mt19937_64 rng(777);
  auto sa = gen(rng, 0), sb = gen(rng, 1), sc = gen(rng, 2);
  sa.insert(sc.begin(), sc.end());
  const Bitmap a = from_set(sa), b = from_set(sb);
  const int64_t want = a.intersection_count(b);
  const int64_t want_u = a.unite(b).count();
  const Bitmap a0 = a.offset_range(0, 0, 1 << 20), b0 = b.offset_range(0, 0, 1 << 20);
  const int64_t want_r = a0.intersection_count(b0), want_ru = a0.unite(b0).count();
  std::vector<int> bad(nthreads, 0);
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; t++) {
    ts.emplace_back([&, t] {
      std::mt19937_64 r(t);
      Bitmap own;
      for (int k = 0; k < 200; k++) {
        if (a.intersection_count(b) != want) bad[t]++;
        if (a.range_intersection_count(0, b, 0, 1 << 20) != want_r) bad[t]++;
        if (Bitmap::range_union_count({{&a, 0}, {&b, 0}}, 1 << 20) != want_ru) bad[t]++;
        if (a.unite(b).count() != want_u) bad[t]++;
        own.add(r() % (1 << 20));
        own.remove(r() % (1 << 20));
        Bitmap o = own.intersect(a);
        o.optimize();
      }
    });
  }
  for (auto& th : ts) th.join();
  int n = 0;
  for (int x : bad) n += x;
  std::fprintf(stderr, "threads: %d failures\n", n);
  return n ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && std::strcmp(argv[2], "threads") == 0) return run_threads(std::atoi(argv[1]));
  const int iters = argc > 1 ? std::atoi(argv[1]) : 60;
  std::mt19937_64 rng(12345);
  for (int it = 0; it < iters; it++) {
    auto sa = gen(rng, it % 3), sb = gen(rng, (it / 3) % 3);
    Bitmap a = from_set(sa), b = from_set(sb);
    if (it & 1) {
      a.optimize();
      b.optimize();
    }
    EXPECT(a.check().empty());
    EXPECT(a.count() == int64_t(sa.size()));
    std::set<uint64_t> inter, uni, diff, x;
    for (auto v : sa) (sb.count(v) ? inter : diff).insert(v);
    uni = sa;
    uni.insert(sb.begin(), sb.end());
    for (auto v : uni)
      if (sa.count(v) != sb.count(v)) x.insert(v);
    EXPECT(a.intersection_count(b) == int64_t(inter.size()));
    EXPECT(a.intersect(b).slice() == to_vec(inter));
    EXPECT(a.unite(b).slice() == to_vec(uni));
    EXPECT(a.difference(b).slice() == to_vec(diff));
    EXPECT(a.xor_(b).slice() == to_vec(x));
    // in-place row counts over 2^20-wide windows (rows 0 and 1 of a shard)
    for (uint64_t ra : {0ull, 1ull})
      for (uint64_t rb : {0ull, 1ull}) {
        int64_t ic = 0, uc = 0;
        std::set<uint64_t> u;
        for (auto v : sa)
          if (v >> 20 == ra) u.insert(v & ((1 << 20) - 1));
        for (auto v : sb)
          if (v >> 20 == rb) {
            ic += u.count(v & ((1 << 20) - 1));
          }
        for (auto v : sb)
          if (v >> 20 == rb) u.insert(v & ((1 << 20) - 1));
        uc = int64_t(u.size());
        EXPECT(a.range_intersection_count(ra << 20, b, rb << 20, 1 << 20) == ic);
        EXPECT(Bitmap::range_union_count({{&a, ra << 20}, {&b, rb << 20}}, 1 << 20) == uc);
      }
    // serialisation round trip (pilosa format) and op-log-free reload
    std::string bytes = a.to_bytes();
    Bitmap c;
    c.from_bytes(reinterpret_cast<const uint8_t*>(bytes.data()), bytes.size());
    EXPECT(c.slice() == to_vec(sa));
    EXPECT(c.check().empty());
    // point mutations against the oracle
    for (int k = 0; k < 2000; k++) {
      const uint64_t v = rng() % (1 << 21);
      if (rng() & 1) {
        EXPECT(c.add(v) == (sa.insert(v).second));
      } else {
        EXPECT(c.remove(v) == (sa.erase(v) == 1));
      }
    }
    EXPECT(c.slice() == to_vec(sa));
    // ranges, shift, flip, offset_range
    const uint64_t lo = rng() % (1 << 20), hi = lo + rng() % (1 << 20);
    int64_t cr = 0;
    for (auto v : sa) cr += (v >= lo && v < hi);
    EXPECT(c.count_range(lo, hi) == cr);
    std::set<uint64_t> sh;
    for (auto v : sa) sh.insert(v + 1);
    EXPECT(c.shift(1).slice() == to_vec(sh));
    std::set<uint64_t> fl = sa;
    for (uint64_t v = lo; v <= lo + 5000; v++)
      if (!fl.erase(v)) fl.insert(v);
    EXPECT(c.flip(lo, lo + 5000).slice() == to_vec(fl));
    // truncated / corrupted input must be rejected without UB
    for (size_t cut : {size_t(0), size_t(3), bytes.size() / 2}) {
      Bitmap d;
      try {
        d.from_bytes(reinterpret_cast<const uint8_t*>(bytes.data()), cut);
      } catch (const std::exception&) {
      }
    }
  }
  std::fprintf(stderr, "%s: %d failures\n", argv[0], fails);
  return fails ? 1 : 0;
}
