// Native PQL -> device program compiler for count batches (part of module
// pilosa_amd._pql).
//
// The serving hot path receives many `Count(<bitmap expr>)` queries whose
// leaves are plain `Row(field=<id>)` calls.  Going through the general parser
// (Python AST objects), the planner and the Python program compiler costs
// ~12 us/query on the host, which is more than the GPU needs per query.  This
// compiler scans the PQL text directly into the 256-byte QueryProg records of
// pilosa_amd/kernels/kernels.h (same postfix encoding as
// pilosa_amd/ops/device.py:compile_expr) without creating Python objects.
//
// Accepted subset (everything else is flagged for the general path, so
// semantics are never approximated here):
//   query := ws 'Count' ws '(' ws expr ws ')' ws EOF
//   expr  := ('Row'|'Bitmap') ws '(' ws field ws '=' ws uint [range] ws ')'
//          | ('Intersect'|'Union'|'Difference'|'Xor') ws '(' ws expr (ws ',' ws expr)* ws ')'
//   range := (ws ',' ws ('from'|'to') ws '=' ws time)+      each key at most once
// A Row with a time range is the union of the row over the range's covering
// views (executor.go:1444-1533 with time.go:104-181 viewsByTimeRange): the
// caller resolves each distinct (field, from, to) to those views' slots
// (count_text_ranges), and the leaf compiles to leaf0 leaf1 OR leaf2 OR ...
// Reference semantics: executor.go:585-680 (bitmap call tree), 1668-1790
// (Intersect/Union/Difference/Xor folding left to right).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cctype>
#include <thread>
#include <tuple>
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int MAXLEAF = 16, MAXPROG = 32, MAXDEPTH = 4;
constexpr uint8_t OP_AND = 32, OP_OR = 33, OP_XOR = 34, OP_ANDNOT = 35;

#pragma pack(push, 1)
struct QueryProg {
  int32_t nleaf;
  int32_t nprog;
  int32_t leaf_view[MAXLEAF];
  int64_t leaf_row[MAXLEAF];
  uint8_t prog[MAXPROG];
  int64_t pad[3];
};
#pragma pack(pop)
static_assert(sizeof(QueryProg) == 256, "QueryProg layout");

struct View {
  const uint64_t* rows;
  int64_t D;
  bool identity;
  int64_t dense(uint64_t r) const {
    if (identity) return r < uint64_t(D) ? int64_t(r) : -1;
    int64_t lo = 0, hi = D;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (rows[mid] < r) lo = mid + 1;
      else hi = mid;
    }
    return (lo < D && rows[lo] == r) ? lo : -1;
  }
};

struct Unsupported {};

// (field, from, to) of a time-range Row -> slots of its covering views
using RangeMap = std::unordered_map<std::string, std::vector<int>>;
static const RangeMap kNoRanges;
constexpr char kAbsent = '\x01';  // from/to not given

static std::string range_key(const std::string& field, const std::string& from, const std::string& to) {
  return field + '\x1f' + from + '\x1f' + to;
}

// A time value: a quoted string ('...' or "...", no escapes) or a bare
// timestamp token; the text between the quotes is returned.
static bool scan_time(std::string_view s, size_t& i, std::string& out) {
  if (i >= s.size()) return false;
  const char q = s[i];
  if (q == '\'' || q == '"') {
    const size_t e = s.find(q, i + 1);
    if (e == std::string_view::npos) return false;
    out.assign(s.substr(i + 1, e - i - 1));
    i = e + 1;
    return true;
  }
  const size_t b = i;
  while (i < s.size() && (std::isalnum(static_cast<unsigned char>(s[i])) || s[i] == ':' || s[i] == '-' || s[i] == '.'))
    i++;
  if (i == b) return false;
  out.assign(s.substr(b, i - b));
  return true;
}

static void skip_ws(std::string_view s, size_t& i) {
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
}

static bool key_word(std::string_view s, size_t& i, const char* w) {
  const size_t n = std::strlen(w);
  if (s.compare(i, n, w) != 0) return false;
  if (i + n < s.size() && (std::isalnum(static_cast<unsigned char>(s[i + n])) || s[i + n] == '_')) return false;
  i += n;
  return true;
}

// `, from=<t>, to=<t>` after a Row's row id, up to and including the
// closing ')'.  false = not this shape (the caller takes the general path).
static bool scan_range(std::string_view s, size_t& i, std::string& from, std::string& to) {
  bool hf = false, ht = false;
  from.assign(1, kAbsent);
  to.assign(1, kAbsent);
  for (;;) {
    skip_ws(s, i);
    if (key_word(s, i, "from")) {
      if (hf) return false;
      hf = true;
      skip_ws(s, i);
      if (i >= s.size() || s[i++] != '=') return false;
      skip_ws(s, i);
      if (!scan_time(s, i, from)) return false;
    } else if (key_word(s, i, "to")) {
      if (ht) return false;
      ht = true;
      skip_ws(s, i);
      if (i >= s.size() || s[i++] != '=') return false;
      skip_ws(s, i);
      if (!scan_time(s, i, to)) return false;
    } else {
      return false;
    }
    skip_ws(s, i);
    if (i < s.size() && s[i] == ')') {
      i++;
      return true;
    }
    if (i >= s.size() || s[i++] != ',') return false;
  }
}

class Compiler {
 public:
  Compiler(std::string_view s, const std::unordered_map<std::string, int>& fields, const std::vector<View>& views,
           QueryProg& out, const RangeMap& ranges = kNoRanges)
      : s_(s), fields_(fields), views_(views), outp_(&out), ranges_(ranges) {}

  bool run() {
    if (!call()) return false;
    ws();
    return i_ == s_.size();
  }

  // One `Count(<expr>)` call starting at pos(); leaves the cursor after it.
  bool call() {
    std::memset(outp_, 0, sizeof(QueryProg));
    nleaf_ = nprog_ = depth_ = 0;
    ws();
    if (!word("Count")) return false;
    ws();
    if (!ch('(')) return false;
    ws();
    if (!expr()) return false;
    ws();
    if (!ch(')')) return false;
    outp_->nleaf = nleaf_;
    outp_->nprog = nprog_;
    return true;
  }

  size_t pos() const { return i_; }
  void seek(size_t i) { i_ = i; }
  void retarget(QueryProg* out) { outp_ = out; }
  bool at_end() {
    ws();
    return i_ >= s_.size();
  }

 private:
  std::string_view s_;
  size_t i_ = 0;
  const std::unordered_map<std::string, int>& fields_;
  const std::vector<View>& views_;
  QueryProg* outp_;
  const RangeMap& ranges_;
  int nleaf_ = 0, nprog_ = 0, depth_ = 0;

  // leaf index of (view slot, dense row), added if new
  int leaf_of(int slot, int64_t d) {
    for (int x = 0; x < nleaf_; x++)
      if (outp_->leaf_view[x] == slot && outp_->leaf_row[x] == d) return x;
    if (nleaf_ >= MAXLEAF) return -1;
    outp_->leaf_view[nleaf_] = slot;
    outp_->leaf_row[nleaf_] = d;
    return nleaf_++;
  }

  void ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) i_++;
  }
  bool ch(char c) {
    if (i_ < s_.size() && s_[i_] == c) {
      i_++;
      return true;
    }
    return false;
  }
  static bool is_ident(char c) { return std::isalnum(static_cast<unsigned char>(c)) || c == '_' || c == '-'; }
  bool word(const char* w) {
    const size_t n = std::strlen(w);
    if (s_.compare(i_, n, w) != 0) return false;
    if (i_ + n < s_.size() && is_ident(s_[i_ + n])) return false;
    i_ += n;
    return true;
  }
  bool emit(uint8_t code) {
    if (nprog_ >= MAXPROG) return false;
    outp_->prog[nprog_++] = code;
    return true;
  }

  bool leaf() {
    ws();
    if (!ch('(')) return false;
    ws();
    const size_t f0 = i_;
    if (i_ >= s_.size() || !std::isalpha(static_cast<unsigned char>(s_[i_]))) return false;
    while (i_ < s_.size() && is_ident(s_[i_])) i_++;
    const std::string field(s_.substr(f0, i_ - f0));
    ws();
    if (!ch('=')) return false;
    ws();
    // a bare '=' followed by '=' is a condition (BSI) -> general path
    if (i_ < s_.size() && !std::isdigit(static_cast<unsigned char>(s_[i_]))) return false;
    uint64_t row = 0;
    int nd = 0;
    while (i_ < s_.size() && std::isdigit(static_cast<unsigned char>(s_[i_]))) {
      if (++nd > 18) return false;  // keep well inside int64
      row = row * 10 + uint64_t(s_[i_++] - '0');
    }
    if (i_ < s_.size() && s_[i_] == '.') return false;  // float
    ws();
    if (ch(',')) {
      // time range: the row over the covering views, OR-folded
      std::string from, to;
      if (!scan_range(s_, i_, from, to)) return false;
      auto rt = ranges_.find(range_key(field, from, to));
      if (rt == ranges_.end() || rt->second.empty()) return false;
      bool first = true;
      for (int slot : rt->second) {
        if (slot < 0 || slot >= int(views_.size())) return false;
        const int k = leaf_of(slot, views_[slot].dense(row));
        if (k < 0 || ++depth_ > MAXDEPTH) return false;
        if (!emit(uint8_t(k))) return false;
        if (!first) {
          if (!emit(OP_OR)) return false;
          depth_--;
        }
        first = false;
      }
      return true;
    }
    if (!ch(')')) return false;
    auto it = fields_.find(field);
    if (it == fields_.end()) return false;
    const int slot = it->second;
    const int k = leaf_of(slot, views_[slot].dense(row));
    if (k < 0 || ++depth_ > MAXDEPTH) return false;
    return emit(uint8_t(k));
  }

  bool expr() {
    uint8_t code;
    if (word("Row") || word("Bitmap")) return leaf();
    if (word("Intersect")) code = OP_AND;
    else if (word("Union")) code = OP_OR;
    else if (word("Difference")) code = OP_ANDNOT;
    else if (word("Xor")) code = OP_XOR;
    else return false;
    ws();
    if (!ch('(')) return false;
    ws();
    if (!expr()) return false;
    for (;;) {
      ws();
      if (ch(')')) return true;
      if (!ch(',')) return false;
      ws();
      if (!expr()) return false;
      if (!emit(code)) return false;
      depth_--;
    }
  }
};

// compile_counts(queries, fields, dirs) -> (progs uint8[Q*256], ok bool[Q])
py::tuple compile_counts(const std::vector<std::string>& queries, const std::unordered_map<std::string, int>& fields,
                         const std::vector<py::array_t<uint64_t, py::array::c_style | py::array::forcecast>>& dirs) {
  std::vector<View> views;
  views.reserve(dirs.size());
  for (const auto& d : dirs) {
    View v;
    v.rows = d.data();
    v.D = d.size();
    v.identity = v.D > 0 && v.rows[v.D - 1] == uint64_t(v.D - 1);
    views.push_back(v);
  }
  for (const auto& kv : fields)
    if (kv.second < 0 || kv.second >= int(views.size())) throw std::out_of_range("field slot out of range");
  const size_t Q = queries.size();
  py::array_t<uint8_t> progs(Q * sizeof(QueryProg));
  py::array_t<bool> ok(Q);
  auto* pp = reinterpret_cast<QueryProg*>(progs.mutable_data());
  bool* okp = ok.mutable_data();
  {
    py::gil_scoped_release nogil;
    for (size_t q = 0; q < Q; q++) {
      Compiler c(queries[q], fields, views, pp[q]);
      okp[q] = c.run();
      if (!okp[q]) std::memset(&pp[q], 0, sizeof(QueryProg));
    }
  }
  return py::make_tuple(progs, ok);
}

// compile_count_text(text, fields, dirs) -> (progs uint8[Q*256], Q) or None.
// `text` is a whole request of top-level Count() calls ("Count(..) Count(..)");
// None when any call is outside the subset (the caller parses generally).
py::object compile_count_text(const std::string& text, const std::unordered_map<std::string, int>& fields,
                              const std::vector<py::array_t<uint64_t, py::array::c_style | py::array::forcecast>>& dirs) {
  std::vector<View> views;
  views.reserve(dirs.size());
  for (const auto& d : dirs) {
    View v;
    v.rows = d.data();
    v.D = d.size();
    v.identity = v.D > 0 && v.rows[v.D - 1] == uint64_t(v.D - 1);
    views.push_back(v);
  }
  for (const auto& kv : fields)
    if (kv.second < 0 || kv.second >= int(views.size())) throw std::out_of_range("field slot out of range");
  std::vector<QueryProg> out;
  bool ok = true;
  {
    py::gil_scoped_release nogil;
    out.reserve(text.size() / 40 + 1);
    QueryProg tmp;
    Compiler c(text, fields, views, tmp);
    while (!c.at_end()) {
      out.emplace_back();
      c.retarget(&out.back());
      if (!c.call()) {
        ok = false;
        break;
      }
    }
    ok = ok && !out.empty();
  }
  if (!ok) return py::none();
  const size_t Q = out.size();
  py::array_t<uint8_t> progs(Q * sizeof(QueryProg));
  std::memcpy(progs.mutable_data(), out.data(), Q * sizeof(QueryProg));
  return py::make_tuple(progs, Q);
}

// ---------------------------------------------------------------- batch planner
// plan_count_text(text, fields, dirs, use_and2, use_union, nthreads): the host
// half of a count batch in one native call (the numpy version is
// ops/device.py GpuEngine.prepare_progs): compile every Count() call of the
// request, canonicalise Intersect(a, a), classify each program by kernel
// route, put the batch's more frequent row first in Count(Intersect(a, b))
// (the pair kernel stages leaf 0 once per run of equal rows), sort each
// route's programs by (leaf row 0, leaf row 1) and lay them out with their
// submission indices in one buffer ready for a single H2D copy.
// -> (Q, [(kind, n, progs_off, order_off)], buf uint8[]) or None.
enum Kind { K_AND2 = 0, K_ROW = 1, K_GENERIC = 2, K_FLAT = 3, K_UNION = 4, K_ALIAS = 5 };

static bool is_flat(const QueryProg& p) {
  const int n = p.nprog;
  if (n < 3 || (n % 2) == 0) return false;
  for (int i = 0; i < n; i++) {
    const bool want_leaf = i == 0 || (i % 2 == 1);
    if ((p.prog[i] < OP_AND) != want_leaf) return false;
  }
  return true;
}

py::object plan_count_text(const std::string& text, const std::unordered_map<std::string, int>& fields,
                           const std::vector<py::array_t<uint64_t, py::array::c_style | py::array::forcecast>>& dirs,
                           bool use_and2, bool use_union, int nthreads, const RangeMap& ranges) {
  std::vector<View> views;
  views.reserve(dirs.size());
  for (const auto& d : dirs) {
    View v;
    v.rows = d.data();
    v.D = d.size();
    v.identity = v.D > 0 && v.rows[v.D - 1] == uint64_t(v.D - 1);
    views.push_back(v);
  }
  for (const auto& kv : fields)
    if (kv.second < 0 || kv.second >= int(views.size())) throw std::out_of_range("field slot out of range");
  for (const auto& kv : ranges)
    for (int slot : kv.second)
      if (slot < 0 || slot >= int(views.size())) throw std::out_of_range("range view slot out of range");
  std::vector<QueryProg> progs;
  std::vector<int> kind;
  bool ok = true;
  std::vector<uint8_t> buf;
  std::vector<std::tuple<int, size_t, size_t, size_t>> segs;
  {
    py::gil_scoped_release nogil;
    // 1. call boundaries (top-level parentheses), then compile in parallel
    std::vector<std::pair<size_t, size_t>> calls;
    {
      size_t i = 0, n = text.size();
      while (i < n) {
        while (i < n && (text[i] == ' ' || text[i] == '\t' || text[i] == '\n' || text[i] == '\r')) i++;
        if (i >= n) break;
        const size_t b = i;
        int depth = 0;
        bool seen = false;
        for (; i < n; i++) {
          const char c = text[i];
          if (c == '"' || c == '\'') {  // quoted (time values): parentheses inside do not count
            const size_t e = text.find(c, i + 1);
            if (e == std::string::npos) {
              ok = false;
              break;
            }
            i = e;
            continue;
          }
          if (c == '(') depth++, seen = true;
          else if (c == ')' && --depth == 0) {
            i++;
            break;
          }
          if (depth < 0) {
            ok = false;
            break;
          }
        }
        if (!ok || !seen || depth != 0) {
          ok = false;
          break;
        }
        calls.emplace_back(b, i);
      }
    }
    const size_t Q = calls.size();
    ok = ok && Q > 0;
    if (ok) {
      progs.resize(Q);
      std::vector<char> good(Q, 0);
      auto work = [&](size_t lo, size_t hi) {
        for (size_t q = lo; q < hi; q++) {
          Compiler c(std::string_view(text).substr(calls[q].first, calls[q].second - calls[q].first), fields, views,
                     progs[q], ranges);
          good[q] = c.run() ? 1 : 0;
        }
      };
      const int nt = Q >= 1024 ? std::max(1, std::min(nthreads, 8)) : 1;
      if (nt == 1) {
        work(0, Q);
      } else {
        std::vector<std::thread> th;
        const size_t per = (Q + nt - 1) / nt;
        for (int t = 0; t < nt; t++) {
          const size_t lo = std::min(Q, t * per), hi = std::min(Q, lo + per);
          if (lo < hi) th.emplace_back(work, lo, hi);
        }
        for (auto& t : th) t.join();
      }
      for (size_t q = 0; q < Q && ok; q++) ok = good[q] != 0;
    }
    if (ok) {
      // 2. canonicalise + classify
      kind.resize(Q);
      for (size_t q = 0; q < Q; q++) {
        QueryProg& p = progs[q];
        if (p.nprog == 3 && p.nleaf == 1 && p.prog[0] == 0 && p.prog[1] == 0 && p.prog[2] == OP_AND) {
          p.nleaf = 2;
          p.leaf_row[1] = p.leaf_row[0];
          p.leaf_view[1] = p.leaf_view[0];
          p.prog[1] = 1;
        }
        const bool and2 = p.nprog == 3 && p.prog[0] == 0 && p.prog[1] == 1 && p.prog[2] == OP_AND;
        int k;
        if (p.nprog == 1 || (and2 && !use_and2)) {
          k = K_ROW;
        } else if (and2) {
          k = K_AND2;
        } else if (is_flat(p)) {
          bool all_or = true;
          for (int i = 2; i < p.nprog; i += 2) all_or = all_or && p.prog[i] == OP_OR;
          k = (all_or && use_union) ? K_UNION : K_FLAT;
        } else {
          k = K_GENERIC;
        }
        kind[q] = k;
      }
      // 3. hot leaf first for Count(Intersect(a, b)): frequency of every
      // (view, row) leaf over the pair programs (open-addressing hash count)
      size_t cap = 16;
      while (cap < Q * 4) cap <<= 1;
      std::vector<uint64_t> hk(cap, ~0ull);
      std::vector<uint32_t> hc(cap, 0);
      auto slot = [&](uint64_t k) {
        size_t h = size_t((k * 0x9E3779B97F4A7C15ull) >> 20) & (cap - 1);
        while (hk[h] != ~0ull && hk[h] != k) h = (h + 1) & (cap - 1);
        return h;
      };
      auto key_of = [](const QueryProg& p, int l) {
        return ((uint64_t(uint32_t(p.leaf_view[l])) << 40) ^ uint64_t(p.leaf_row[l])) & ~(1ull << 63);
      };
      for (size_t q = 0; q < Q; q++)
        if (kind[q] == K_AND2)
          for (int l = 0; l < 2; l++) {
            const uint64_t k = key_of(progs[q], l);
            const size_t h = slot(k);
            hk[h] = k;
            hc[h]++;
          }
      std::vector<uint32_t> cnt(Q * 2, 0);
      for (size_t q = 0; q < Q; q++)
        if (kind[q] == K_AND2)
          for (int l = 0; l < 2; l++) cnt[q * 2 + size_t(l)] = hc[slot(key_of(progs[q], l))];
      for (size_t q = 0; q < Q; q++) {
        if (kind[q] != K_AND2) continue;
        QueryProg& p = progs[q];
        const uint64_t ka = (uint64_t(uint32_t(p.leaf_view[0])) << 40) ^ uint64_t(p.leaf_row[0]);
        const uint64_t kb = (uint64_t(uint32_t(p.leaf_view[1])) << 40) ^ uint64_t(p.leaf_row[1]);
        const uint32_t ca = cnt[q * 2], cb = cnt[q * 2 + 1];
        if (cb > ca || (cb == ca && kb < ka)) {
          std::swap(p.leaf_row[0], p.leaf_row[1]);
          std::swap(p.leaf_view[0], p.leaf_view[1]);
        }
      }
      // 4. per route: sort by (leaf views, leaf row 0, leaf row 1, submission), lay out
      const int route_order[5] = {K_AND2, K_ROW, K_FLAT, K_UNION, K_GENERIC};
      struct SortKey {
        int64_t v, r0, r1;
        int64_t q;
        bool operator<(const SortKey& o) const {
          return r0 != o.r0 ? r0 < o.r0 : (r1 != o.r1 ? r1 < o.r1 : (v != o.v ? v < o.v : q < o.q));
        }
      };
      std::vector<std::vector<SortKey>> sel(5);
      for (size_t q = 0; q < Q; q++)
        sel[size_t(kind[q])].push_back({(int64_t(progs[q].leaf_view[0]) << 32) | uint32_t(progs[q].leaf_view[1]),
                                        progs[q].leaf_row[0], progs[q].leaf_row[1], int64_t(q)});
      // 4b. a Count(Intersect(a, b)) asked more than once in the batch (the
      // hot-leaf order above makes (a, b) and (b, a) one key) runs once: the
      // repeats become (copy from, copy to) submission pairs, a K_ALIAS
      // segment applied after the kernels (~4 % of a 4096-query Zipf batch)
      std::vector<std::pair<int64_t, int64_t>> alias;
      {
        auto& v = sel[size_t(K_AND2)];
        std::sort(v.begin(), v.end());
        size_t w = 0;
        for (size_t i = 0; i < v.size(); i++) {
          if (w > 0 && v[i].v == v[w - 1].v && v[i].r0 == v[w - 1].r0 && v[i].r1 == v[w - 1].r1) {
            alias.emplace_back(v[w - 1].q, v[i].q);
            continue;
          }
          v[w++] = v[i];
        }
        v.resize(w);
      }
      size_t total = 0;
      auto align = [](size_t x) { return (x + 255) & ~size_t(255); };
      for (int r : route_order) {
        auto& v = sel[size_t(r)];
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        const size_t po = total;
        total = align(total + v.size() * sizeof(QueryProg));
        const size_t oo = total;
        total = align(total + v.size() * 8);
        segs.emplace_back(r, v.size(), po, oo);
      }
      if (!alias.empty()) {   // (from, to) int64 pairs: the last segment
        const size_t po = total;
        total = align(total + alias.size() * 8);
        const size_t oo = total;
        total = align(total + alias.size() * 8);
        segs.emplace_back(K_ALIAS, alias.size(), po, oo);
      }
      buf.resize(std::max<size_t>(total, 256));
      for (auto& sg : segs) {
        if (std::get<0>(sg) == K_ALIAS) {
          int64_t* from = reinterpret_cast<int64_t*>(buf.data() + std::get<2>(sg));
          int64_t* to = reinterpret_cast<int64_t*>(buf.data() + std::get<3>(sg));
          for (size_t i = 0; i < alias.size(); i++) {
            from[i] = alias[i].first;
            to[i] = alias[i].second;
          }
          continue;
        }
        const auto& v = sel[size_t(std::get<0>(sg))];
        QueryProg* dst = reinterpret_cast<QueryProg*>(buf.data() + std::get<2>(sg));
        int64_t* ord = reinterpret_cast<int64_t*>(buf.data() + std::get<3>(sg));
        for (size_t i = 0; i < v.size(); i++) {
          dst[i] = progs[size_t(v[i].q)];
          ord[i] = v[i].q;
        }
      }
    }
  }
  if (!ok) return py::none();
  py::array_t<uint8_t> out(buf.size());
  std::memcpy(out.mutable_data(), buf.data(), buf.size());
  py::list sl;
  for (auto& sg : segs)
    sl.append(py::make_tuple(std::get<0>(sg), std::get<1>(sg), std::get<2>(sg), std::get<3>(sg)));
  return py::make_tuple(progs.size(), sl, out);
}

// Field names of the Row(field=...) leaves of a request (distinct, first-seen
// order); views for them are resolved before compile_count_text.
std::vector<std::string> count_text_fields(const std::string& text) {
  std::vector<std::string> out;
  const size_t n = text.size();
  for (size_t i = 0; i + 4 < n; i++) {
    if (text[i] != 'R' || text.compare(i, 3, "Row") != 0) continue;
    if (i > 0 && (std::isalnum(static_cast<unsigned char>(text[i - 1])) || text[i - 1] == '_')) continue;
    size_t j = i + 3;
    while (j < n && (text[j] == ' ' || text[j] == '\t' || text[j] == '\n' || text[j] == '\r')) j++;
    if (j >= n || text[j] != '(') continue;
    j++;
    while (j < n && (text[j] == ' ' || text[j] == '\t' || text[j] == '\n' || text[j] == '\r')) j++;
    const size_t f0 = j;
    while (j < n && (std::isalnum(static_cast<unsigned char>(text[j])) || text[j] == '_' || text[j] == '-')) j++;
    if (j == f0) continue;
    std::string f = text.substr(f0, j - f0);
    // a time-range Row (`f=<id>, from=..`) needs its covering views, not the
    // standard view: count_text_ranges lists it
    size_t k = j;
    skip_ws(text, k);
    if (k < n && text[k] == '=') {
      k++;
      skip_ws(text, k);
      while (k < n && std::isdigit(static_cast<unsigned char>(text[k]))) k++;
      skip_ws(text, k);
      if (k < n && text[k] == ',') {
        i = j;
        continue;
      }
    }
    bool seen = false;
    for (const auto& x : out) seen = seen || x == f;
    if (!seen) out.push_back(std::move(f));
    i = j;
  }
  return out;
}

// A request made only of plain cache-only TopN calls -- TopN(<field>
// [, n=<uint>] [, threshold=<uint>]) in any argument order, separated by
// whitespace -- as (field per call, n per call, threshold per call; 0 =
// absent), or None for anything else (the general parser then runs).  The
// serving fast path for cache-only TopN requests needs no Call objects.
py::object topn_plain(const std::string& text) {
  std::vector<std::string> fields;
  std::vector<int64_t> ns, ths;
  const size_t n = text.size();
  size_t i = 0;
  auto ident = [&](size_t& k) -> std::string {
    const size_t f0 = k;
    while (k < n && (std::isalnum(static_cast<unsigned char>(text[k])) || text[k] == '_' || text[k] == '-')) k++;
    return text.substr(f0, k - f0);
  };
  auto uint = [&](size_t& k, int64_t& v) -> bool {
    const size_t d0 = k;
    v = 0;
    while (k < n && std::isdigit(static_cast<unsigned char>(text[k]))) {
      if (v > (INT64_MAX - 9) / 10) return false;
      v = v * 10 + (text[k] - '0');
      k++;
    }
    return k > d0;
  };
  for (;;) {
    skip_ws(text, i);
    if (i >= n) break;
    if (text.compare(i, 5, "TopN(") != 0) return py::none();
    i += 5;
    skip_ws(text, i);
    std::string f = ident(i);
    if (f.empty() || !(std::isalpha(static_cast<unsigned char>(f[0])))) return py::none();
    skip_ws(text, i);
    int64_t nv = 0, tv = 0;
    bool has_n = false, has_t = false;
    while (i < n && text[i] == ',') {
      i++;
      skip_ws(text, i);
      const std::string key = ident(i);
      skip_ws(text, i);
      if (i >= n || text[i] != '=') return py::none();
      i++;
      skip_ws(text, i);
      int64_t v;
      if (!uint(i, v)) return py::none();
      if (key == "n" && !has_n) {
        nv = v;
        has_n = true;
      } else if (key == "threshold" && !has_t) {
        tv = v;
        has_t = true;
      } else {
        return py::none();
      }
      skip_ws(text, i);
    }
    if (i >= n || text[i] != ')') return py::none();
    i++;
    fields.push_back(std::move(f));
    ns.push_back(nv);
    ths.push_back(tv);
  }
  if (fields.empty()) return py::none();
  return py::make_tuple(fields, ns, ths);
}

// Distinct (field, from, to) of the time-range Row leaves of a request, in
// first-seen order; from / to are None when not given.  The caller maps
// each to its covering views (plan_count_text's `ranges`, keyed by
// range_key with "\x01" for an absent bound).
py::list count_text_ranges(const std::string& text) {
  py::list out;
  std::vector<std::string> seen;
  const std::string_view s(text);
  const size_t n = s.size();
  for (size_t i = 0; i + 4 < n; i++) {
    if (s[i] != 'R' || s.compare(i, 3, "Row") != 0) continue;
    if (i > 0 && (std::isalnum(static_cast<unsigned char>(s[i - 1])) || s[i - 1] == '_')) continue;
    size_t j = i + 3;
    skip_ws(s, j);
    if (j >= n || s[j] != '(') continue;
    j++;
    skip_ws(s, j);
    const size_t f0 = j;
    while (j < n && (std::isalnum(static_cast<unsigned char>(s[j])) || s[j] == '_' || s[j] == '-')) j++;
    if (j == f0) continue;
    const std::string field(s.substr(f0, j - f0));
    size_t k = j;
    skip_ws(s, k);
    if (k >= n || s[k] != '=') continue;
    k++;
    skip_ws(s, k);
    const size_t d0 = k;
    while (k < n && std::isdigit(static_cast<unsigned char>(s[k]))) k++;
    if (k == d0) continue;
    skip_ws(s, k);
    if (k >= n || s[k] != ',') continue;
    k++;
    std::string from, to;
    if (!scan_range(s, k, from, to)) continue;
    const std::string key = range_key(field, from, to);
    bool dup = false;
    for (const auto& x : seen) dup = dup || x == key;
    if (!dup) {
      seen.push_back(key);
      py::object pf = from == std::string(1, kAbsent) ? py::object(py::none()) : py::object(py::str(from));
      py::object pt = to == std::string(1, kAbsent) ? py::object(py::none()) : py::object(py::str(to));
      out.append(py::make_tuple(field, pf, pt));
    }
    i = k - 1;
  }
  return out;
}

}  // namespace

void register_compile(py::module_& m) {
  m.def("compile_count_text", &compile_count_text, py::arg("text"), py::arg("fields"), py::arg("dirs"),
        "Compile a request of top-level Count(<Row/Intersect/Union/Difference/Xor tree>) calls straight to "
        "QueryProg records; (progs uint8[Q*256], Q), or None when a call needs the general path");
  m.def("count_text_fields", &count_text_fields, py::arg("text"));
  m.def("topn_plain", &topn_plain, py::arg("text"),
        "(fields, n, threshold) per call of a request of plain TopN(<field>[, n=][, threshold=]) calls, or None");
  m.def("count_text_ranges", &count_text_ranges, py::arg("text"),
        "Distinct (field, from, to) of the time-range Row(f=<id>, from=, to=) leaves of a request");
  m.def("plan_count_text", &plan_count_text, py::arg("text"), py::arg("fields"), py::arg("dirs"),
        py::arg("use_and2") = true, py::arg("use_union") = true, py::arg("nthreads") = 4,
        py::arg("ranges") = RangeMap{},
        "Compile + classify + order a request of Count() calls into one H2D-ready buffer; "
        "(Q, [(kind, n, progs_off, order_off)], buf) or None");
  m.def("compile_counts", &compile_counts, py::arg("queries"), py::arg("fields"), py::arg("dirs"),
        "Compile Count(<Row/Intersect/Union/Difference/Xor tree>) PQL strings straight to QueryProg records; "
        "returns (progs uint8[Q*256], ok bool[Q]) -- rows with ok=False need the general path");
}
