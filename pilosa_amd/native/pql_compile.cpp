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
//   expr  := ('Row'|'Bitmap') ws '(' ws field ws '=' ws uint ws ')'
//          | ('Intersect'|'Union'|'Difference'|'Xor') ws '(' ws expr (ws ',' ws expr)* ws ')'
// Reference semantics: executor.go:585-680 (bitmap call tree), 1668-1790
// (Intersect/Union/Difference/Xor folding left to right).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

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

class Compiler {
 public:
  Compiler(std::string_view s, const std::unordered_map<std::string, int>& fields, const std::vector<View>& views,
           QueryProg& out)
      : s_(s), fields_(fields), views_(views), out_(out) {}

  bool run() {
    std::memset(&out_, 0, sizeof(out_));
    ws();
    if (!word("Count")) return false;
    ws();
    if (!ch('(')) return false;
    ws();
    if (!expr()) return false;
    ws();
    if (!ch(')')) return false;
    ws();
    if (i_ != s_.size()) return false;
    out_.nleaf = nleaf_;
    out_.nprog = nprog_;
    return true;
  }

 private:
  std::string_view s_;
  size_t i_ = 0;
  const std::unordered_map<std::string, int>& fields_;
  const std::vector<View>& views_;
  QueryProg& out_;
  int nleaf_ = 0, nprog_ = 0, depth_ = 0;

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
    out_.prog[nprog_++] = code;
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
    if (!ch(')')) return false;
    auto it = fields_.find(field);
    if (it == fields_.end()) return false;
    const int slot = it->second;
    const int64_t d = views_[slot].dense(row);
    int k = -1;
    for (int x = 0; x < nleaf_; x++)
      if (out_.leaf_view[x] == slot && out_.leaf_row[x] == d) k = x;
    if (k < 0) {
      if (nleaf_ >= MAXLEAF) return false;
      k = nleaf_++;
      out_.leaf_view[k] = slot;
      out_.leaf_row[k] = d;
    }
    if (++depth_ > MAXDEPTH) return false;
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

}  // namespace

void register_compile(py::module_& m) {
  m.def("compile_counts", &compile_counts, py::arg("queries"), py::arg("fields"), py::arg("dirs"),
        "Compile Count(<Row/Intersect/Union/Difference/Xor tree>) PQL strings straight to QueryProg records; "
        "returns (progs uint8[Q*256], ok bool[Q]) -- rows with ok=False need the general path");
}
