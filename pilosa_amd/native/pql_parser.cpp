// Native PQL parser (module pilosa_amd._pql).
//
// Recursive descent with PEG semantics (ordered choice, backtracking only at
// alternatives) for the grammar in reference pql/pql.peg:8-83; it builds the
// same pilosa_amd.pql.ast objects as the pure-Python parser
// (pilosa_amd/pql/parser.py), which stays as the executable specification and
// fallback.  The reference parser is generated Go code; this one is compiled
// C++ so that PQL parsing is not the QPS bottleneck in front of the GPU.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct Fail {};

struct Ctx {
  py::object Call, Condition, ParseError;
};

Ctx* g_ctx = nullptr;

Ctx& ctx() {
  if (!g_ctx) {
    g_ctx = new Ctx();
    py::module_ ast = py::module_::import("pilosa_amd.pql.ast");
    py::module_ prs = py::module_::import("pilosa_amd.pql.parser");
    g_ctx->Call = ast.attr("Call");
    g_ctx->Condition = ast.attr("Condition");
    g_ctx->ParseError = prs.attr("ParseError");
  }
  return *g_ctx;
}

[[noreturn]] void parse_error(const std::string& msg) {
  PyErr_SetString(ctx().ParseError.ptr(), msg.c_str());
  throw py::error_already_set();
}

inline bool is_alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_alnum(char c) { return is_alpha(c) || is_digit(c); }

struct Args {
  py::dict d;
  void put(const std::string& k, py::object v) {
    py::str key(k);
    if (d.contains(key)) parse_error("duplicate argument provided: " + k);
    d[key] = v;
  }
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s), n_(s.size()) {}

  py::list parse() {
    py::list calls;
    size_t i = sp(0);
    while (i < n_) {
      try {
        py::object c;
        i = call(i, c);
        calls.append(c);
      } catch (Fail&) {
        err(i);
      }
      i = sp(i);
    }
    return calls;
  }

 private:
  const std::string& s_;
  size_t n_;

  [[noreturn]] void err(size_t i) {
    size_t line = 1, col = 1;
    for (size_t k = 0; k < i && k < n_; k++) {
      if (s_[k] == '\n') line++, col = 1;
      else col++;
    }
    std::string near = s_.substr(i, 20);
    parse_error("parse error at line " + std::to_string(line) + ", column " + std::to_string(col) +
                ": unexpected '" + near + "'");
  }

  bool starts(size_t i, const char* t) const {
    size_t l = strlen(t);
    return i + l <= n_ && memcmp(s_.data() + i, t, l) == 0;
  }
  size_t sp(size_t i) const {
    while (i < n_ && (s_[i] == ' ' || s_[i] == '\t' || s_[i] == '\n')) i++;
    return i;
  }
  size_t lit(size_t i, const char* t) const {
    if (!starts(i, t)) throw Fail();
    return i + strlen(t);
  }
  size_t open(size_t i) const { return sp(lit(i, "(")); }
  size_t close(size_t i) const { return sp(lit(i, ")")); }
  size_t comma(size_t i) const { return sp(lit(sp(i), ",")); }
  bool at_comma(size_t i) const {
    size_t j = sp(i);
    return j < n_ && s_[j] == ',';
  }
  bool ts_ahead(size_t i) const {
    if (i < n_ && (s_[i] == '"' || s_[i] == '\'')) return ts_at(i + 1);
    return ts_at(i);
  }

  size_t ident(size_t i, std::string& out) const {  // [A-Za-z][A-Za-z0-9]*
    if (i >= n_ || !is_alpha(s_[i])) throw Fail();
    size_t j = i + 1;
    while (j < n_ && is_alnum(s_[j])) j++;
    out.assign(s_, i, j - i);
    return j;
  }
  size_t field_expr(size_t i, std::string& out) const {  // [A-Za-z][A-Za-z0-9_-]*
    if (i >= n_ || !is_alpha(s_[i])) throw Fail();
    size_t j = i + 1;
    while (j < n_ && (is_alnum(s_[j]) || s_[j] == '_' || s_[j] == '-')) j++;
    out.assign(s_, i, j - i);
    return j;
  }
  size_t field(size_t i, std::string& out) const {
    static const char* reserved[] = {"_row", "_col", "_start", "_end", "_timestamp", "_field"};
    for (const char* r : reserved)
      if (starts(i, r)) {
        out = r;
        return i + strlen(r);
      }
    return field_expr(i, out);
  }
  bool call_ahead(size_t i) const {
    if (i >= n_ || !is_alpha(s_[i])) return false;
    size_t j = i + 1;
    while (j < n_ && is_alnum(s_[j])) j++;
    return j < n_ && s_[j] == '(';
  }

  static py::object make_int(const std::string& t) {
    errno = 0;
    char* end = nullptr;
    long long v = strtoll(t.c_str(), &end, 10);
    if (errno == ERANGE)
      parse_error("integer value out of range: strconv.ParseInt: parsing \"" + t + "\": value out of range");
    return py::int_(v);
  }
  static py::object make_num(const std::string& t) {
    if (t.find('.') != std::string::npos) return py::float_(strtod(t.c_str(), nullptr));
    return make_int(t);
  }

  // ------------------------------------------------------------ calls
  // Nesting guard: the reference's PEG runs on growable goroutine stacks; a
  // fixed native stack needs a bound (pql/parser.py MAX_NESTING, same value).
  static constexpr int MAX_NESTING = 1000;
  int depth_ = 0;
  struct Nest {
    int& d;
    explicit Nest(int& d_) : d(d_) { ++d; }
    ~Nest() { --d; }
  };

  size_t call(size_t i, py::object& out) {
    Nest guard(depth_);
    if (depth_ > MAX_NESTING) parse_error("query nesting exceeds " + std::to_string(MAX_NESTING) + " levels");
    std::string name;
    size_t j = ident(i, name);
    static const char* lits[] = {"Set", "SetRowAttrs", "SetColumnAttrs", "Clear", "ClearRow",
                                 "Store", "TopN", "Rows", "Range"};
    for (int k = 0; k < 9; k++) {
      if (!starts(i, lits[k])) continue;
      size_t p = i + strlen(lits[k]);
      try {
        switch (k) {
          case 0: return set_call(p, lits[k], out);
          case 1: return set_row_attrs(p, lits[k], out);
          case 2: case 3: return col_args_call(p, lits[k], out);
          case 4: return clear_row(p, lits[k], out);
          case 5: return store(p, lits[k], out);
          case 6: case 7: return posfield_call(p, lits[k], out);
          case 8: return range_call(p, lits[k], out);
        }
      } catch (Fail&) {
        continue;
      }
    }
    return generic(j, name, out);
  }

  py::object mk(const std::string& name, Args& a, py::list kids) {
    return ctx().Call(py::str(name), a.d, kids);
  }

  size_t set_call(size_t i, const char* name, py::object& out) {
    Args a;
    i = open(i);
    i = posval(i, a, "_col");
    i = comma(i);
    i = args(i, a);
    try {
      size_t k = comma(i);
      std::string ts;
      k = timestampfmt(k, ts);
      a.put("_timestamp", py::str(ts));
      i = k;
    } catch (Fail&) {
    }
    i = close(i);
    out = mk(name, a, py::list());
    return i;
  }
  size_t set_row_attrs(size_t i, const char* name, py::object& out) {
    Args a;
    i = open(i);
    std::string f;
    i = field_expr(i, f);
    a.put("_field", py::str(f));
    i = comma(i);
    i = posval(i, a, "_row");
    i = comma(i);
    i = args(i, a);
    i = close(i);
    out = mk(name, a, py::list());
    return i;
  }
  size_t col_args_call(size_t i, const char* name, py::object& out) {
    Args a;
    i = open(i);
    i = posval(i, a, "_col");
    i = comma(i);
    i = args(i, a);
    i = close(i);
    out = mk(name, a, py::list());
    return i;
  }
  size_t clear_row(size_t i, const char* name, py::object& out) {
    Args a;
    i = open(i);
    i = arg(i, a);
    i = close(i);
    out = mk(name, a, py::list());
    return i;
  }
  size_t store(size_t i, const char* name, py::object& out) {
    Args a;
    i = open(i);
    py::object child;
    i = call(i, child);
    i = comma(i);
    i = arg(i, a);
    i = close(i);
    py::list kids;
    kids.append(child);
    out = mk(name, a, kids);
    return i;
  }
  size_t posfield_call(size_t i, const char* name, py::object& out) {
    Args a;
    py::list kids;
    i = open(i);
    std::string f;
    i = field_expr(i, f);
    a.put("_field", py::str(f));
    try {
      size_t k = comma(i);
      k = allargs(k, a, kids);
      i = k;
    } catch (Fail&) {
    }
    i = close(i);
    out = mk(name, a, kids);
    return i;
  }
  size_t range_call(size_t i, const char* name, py::object& out) {
    Args a;
    i = open(i);
    std::string f;
    i = field(i, f);
    i = sp(i);
    i = lit(i, "=");
    i = sp(i);
    py::object v;
    i = value(i, v);
    a.put(f, v);
    i = comma(i);
    if (starts(i, "from=")) i += 5;
    std::string ts;
    i = timestampfmt(i, ts);
    a.put("from", py::str(ts));
    i = comma(i);
    if (starts(i, "to=")) i += 3;
    i = sp(i);
    i = timestampfmt(i, ts);
    a.put("to", py::str(ts));
    i = close(i);
    out = mk(name, a, py::list());
    return i;
  }
  size_t generic(size_t i, const std::string& name, py::object& out) {
    Args a;
    py::list kids;
    i = open(i);
    i = allargs(i, a, kids);
    if (at_comma(i)) i = comma(i);
    i = close(i);
    out = mk(name, a, kids);
    return i;
  }

  // ------------------------------------------------------------ args
  size_t allargs(size_t i, Args& a, py::list& kids) {
    if (call_ahead(i)) {
      try {
        py::object c;
        size_t k = call(i, c);
        std::vector<py::object> cs{c};
        while (at_comma(k) && call_ahead(sp(sp(k) + 1))) {
          try {
            size_t k2 = comma(k);
            py::object c2;
            k2 = call(k2, c2);
            cs.push_back(c2);
            k = k2;
          } catch (Fail&) {
            break;
          }
        }
        if (at_comma(k)) try {
          size_t k2 = comma(k);
          Args sub;
          k2 = args(k2, sub);
          for (auto item : sub.d) a.put(item.first.cast<std::string>(), py::reinterpret_borrow<py::object>(item.second));
          k = k2;
        } catch (Fail&) {
        }
        for (auto& c3 : cs) kids.append(c3);
        return k;
      } catch (Fail&) {
      }
    }
    try {
      Args sub;
      size_t k = args(i, sub);
      for (auto item : sub.d) a.put(item.first.cast<std::string>(), py::reinterpret_borrow<py::object>(item.second));
      return k;
    } catch (Fail&) {
    }
    return sp(i);
  }

  size_t args(size_t i, Args& a) {
    i = arg(i, a);
    while (at_comma(i)) {
      try {
        size_t k = comma(i);
        k = arg(k, a);
        i = k;
      } catch (Fail&) {
        break;
      }
    }
    return sp(i);
  }

  size_t arg(size_t i, Args& a) {
    // field sp '=' sp value
    bool fld = i < n_ && (is_alpha(s_[i]) || s_[i] == '_');
    if (fld) try {
      std::string f;
      size_t k = field(i, f);
      k = sp(k);
      k = lit(k, "=");
      if (starts(k, "=")) throw Fail();
      k = sp(k);
      py::object v;
      k = value(k, v);
      a.put(f, v);
      return k;
    } catch (Fail&) {
    }
    // field sp COND sp value
    if (fld) try {
      std::string f;
      size_t k = field(i, f);
      k = sp(k);
      static const char* ops[] = {"><", "<=", ">=", "==", "!=", "<", ">"};
      const char* op = nullptr;
      for (const char* o : ops)
        if (starts(k, o)) {
          op = o;
          k += strlen(o);
          break;
        }
      if (!op) throw Fail();
      k = sp(k);
      py::object v;
      k = value(k, v);
      a.put(f, ctx().Condition(py::str(op), v));
      return k;
    } catch (Fail&) {
    }
    // conditional: int < field <= int
    std::string lo, hi, f, op1, op2;
    size_t k = condint(i, lo);
    k = sp(k);
    k = condlt(k, op1);
    k = field_expr(k, f);
    k = sp(k);
    k = condlt(k, op2);
    k = condint(k, hi);
    k = sp(k);
    long long low = make_int(lo).cast<long long>(), high = make_int(hi).cast<long long>();
    if (op1 == "<") low++;
    if (op2 == "<") high--;
    py::list bounds;
    bounds.append(py::int_(low));
    bounds.append(py::int_(high));
    a.put(f, ctx().Condition(py::str("><"), bounds));
    return k;
  }

  size_t condint(size_t i, std::string& out) const {  // '-'? [1-9][0-9]* / '0'
    size_t j = i;
    if (j < n_ && s_[j] == '0') {
      out = "0";
      return j + 1;
    }
    if (j < n_ && s_[j] == '-') j++;
    if (j >= n_ || s_[j] < '1' || s_[j] > '9') throw Fail();
    while (j < n_ && is_digit(s_[j])) j++;
    out.assign(s_, i, j - i);
    return j;
  }
  size_t condlt(size_t i, std::string& op) const {
    if (starts(i, "<=")) {
      op = "<=";
      return sp(i + 2);
    }
    if (starts(i, "<")) {
      op = "<";
      return sp(i + 1);
    }
    throw Fail();
  }

  size_t posval(size_t i, Args& a, const char* key) {
    if (i < n_ && is_digit(s_[i])) {  // [1-9][0-9]* / '0'
      size_t j = i;
      if (s_[j] == '0') j++;
      else
        while (j < n_ && is_digit(s_[j])) j++;
      a.put(key, make_int(s_.substr(i, j - i)));
      return j;
    }
    if (i < n_ && (s_[i] == '\'' || s_[i] == '"')) {
      char q = s_[i];
      size_t j = quoted_end(i + 1, q);
      a.put(key, py::str(s_.substr(i + 1, j - i - 1)));
      return lit(j, q == '"' ? "\"" : "'");
    }
    throw Fail();
  }

  size_t quoted_end(size_t i, char q) const {
    size_t j = i;
    while (j < n_) {
      if (s_[j] == '\\' && j + 1 < n_ && (s_[j + 1] == q || s_[j + 1] == '\\')) {
        j += 2;
        continue;
      }
      if (s_[j] == q) break;
      j++;
    }
    return j;
  }

  bool ts_at(size_t i) const {  // [0-9]{4}-[01][0-9]-[0-3][0-9]T[0-9]{2}:[0-9]{2}
    if (i + 16 > n_) return false;
    const char* p = s_.data() + i;
    return is_digit(p[0]) && is_digit(p[1]) && is_digit(p[2]) && is_digit(p[3]) && p[4] == '-' &&
           (p[5] == '0' || p[5] == '1') && is_digit(p[6]) && p[7] == '-' && p[8] >= '0' && p[8] <= '3' &&
           is_digit(p[9]) && p[10] == 'T' && is_digit(p[11]) && is_digit(p[12]) && p[13] == ':' &&
           is_digit(p[14]) && is_digit(p[15]);
  }
  size_t timestampfmt(size_t i, std::string& out) const {
    if (i < n_ && (s_[i] == '"' || s_[i] == '\'')) {
      if (!ts_at(i + 1)) throw Fail();
      out.assign(s_, i + 1, 16);
      return lit(i + 17, s_[i] == '"' ? "\"" : "'");
    }
    if (!ts_at(i)) throw Fail();
    out.assign(s_, i, 16);
    return i + 16;
  }

  // ------------------------------------------------------------ values
  size_t value(size_t i, py::object& out) {
    if (starts(i, "[")) {
      size_t k = sp(i + 1);
      py::list vals;
      py::object v;
      k = item(k, v);
      vals.append(v);
      while (at_comma(k)) {
        try {
          size_t k2 = comma(k);
          k2 = item(k2, v);
          vals.append(v);
          k = k2;
        } catch (Fail&) {
          break;
        }
      }
      k = sp(k);
      k = lit(k, "]");
      out = vals;
      return sp(k);
    }
    return item(i, out);
  }

  bool peek_end(size_t i) const {
    size_t j = sp(i);
    return j < n_ && (s_[j] == ',' || s_[j] == ')');
  }

  size_t item(size_t i, py::object& out) {
    if (starts(i, "null") && peek_end(i + 4)) {
      out = py::none();
      return i + 4;
    }
    if (starts(i, "true") && peek_end(i + 4)) {
      out = py::bool_(true);
      return i + 4;
    }
    if (starts(i, "false") && peek_end(i + 5)) {
      out = py::bool_(false);
      return i + 5;
    }
    if (ts_ahead(i)) try {
      std::string ts;
      size_t k = timestampfmt(i, ts);
      out = py::str(ts);
      return k;
    } catch (Fail&) {
    }
    {  // '-'? [0-9]+ ('.' [0-9]*)?   /   '-'? '.' [0-9]+
      size_t j = i;
      if (j < n_ && s_[j] == '-') j++;
      if (j < n_ && is_digit(s_[j])) {
        while (j < n_ && is_digit(s_[j])) j++;
        if (j < n_ && s_[j] == '.') {
          j++;
          while (j < n_ && is_digit(s_[j])) j++;
        }
        out = make_num(s_.substr(i, j - i));
        return j;
      }
      if (j + 1 < n_ && s_[j] == '.' && is_digit(s_[j + 1])) {
        j++;
        while (j < n_ && is_digit(s_[j])) j++;
        out = make_num(s_.substr(i, j - i));
        return j;
      }
    }
    if (call_ahead(i)) {
      std::string name;
      size_t j = ident(i, name);
      try {
        size_t k = open(j);
        Args a;
        py::list kids;
        k = allargs(k, a, kids);
        try {
          k = comma(k);
        } catch (Fail&) {
        }
        k = close(k);
        out = mk(name, a, kids);
        return k;
      } catch (Fail&) {
      }
    }
    {  // bare word ([A-Za-z0-9-_:])+
      size_t j = i;
      while (j < n_ && (is_alnum(s_[j]) || s_[j] == '-' || s_[j] == '_' || s_[j] == ':')) j++;
      if (j > i) {
        out = py::str(s_.substr(i, j - i));
        return j;
      }
    }
    if (i < n_ && s_[i] == '"') {
      size_t j = quoted_end(i + 1, '"');
      size_t k = lit(j, "\"");
      out = unquote(s_.substr(i + 1, j - i - 1));
      return k;
    }
    if (i < n_ && s_[i] == '\'') {
      size_t j = quoted_end(i + 1, '\'');
      size_t k = lit(j, "'");
      out = py::str(s_.substr(i + 1, j - i - 1));
      return k;
    }
    throw Fail();
  }

  static py::object unquote(const std::string& raw) {
    std::string o;
    o.reserve(raw.size());
    for (size_t i = 0; i < raw.size(); i++) {
      char c = raw[i];
      if (c == '\\' && i + 1 < raw.size()) {
        char nx = raw[i + 1];
        switch (nx) {
          case 'n': o += '\n'; i++; continue;
          case 't': o += '\t'; i++; continue;
          case 'r': o += '\r'; i++; continue;
          case '"': o += '"'; i++; continue;
          case '\\': o += '\\'; i++; continue;
          case '\'': o += '\''; i++; continue;
          case '0': o += '\0'; i++; continue;
          default: break;
        }
      }
      o += c;
    }
    return py::str(o);
  }
};

}  // namespace

void register_compile(py::module_& m);  // pql_compile.cpp

PYBIND11_MODULE(_pql, m) {
  m.doc() = "Native PQL parser (grammar: reference pql/pql.peg)";
  m.def("parse_calls", [](const std::string& s) { return Parser(s).parse(); },
        "Parse PQL text into a list of pilosa_amd.pql.ast.Call objects");
  register_compile(m);
}
