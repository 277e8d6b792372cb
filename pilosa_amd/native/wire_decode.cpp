// Native decode of the bulk-import request bodies (part of module
// pilosa_amd._roaring).
//
// POST /index/{i}/field/{f}/import carries an ImportRequest or
// ImportValueRequest (internal/public.proto; wire/pilosa.proto here) whose
// id / value / timestamp lists are packed varints.  The Python protobuf
// runtime decodes them into repeated-field containers that then have to be
// walked element by element to reach numpy, ~45 ms per 200k-bit request;
// this decoder writes the varints straight into numpy arrays (~2 ms).
// Unknown fields are skipped as protobuf requires; a malformed body raises.
// Reference: http/handler.go:1054 handlePostImport, encoding/proto/proto.go
// (ImportRequest decode).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= e) throw std::runtime_error("proto: truncated varint");
      const uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("proto: varint overflow");
  }
  std::pair<const uint8_t*, size_t> bytes() {
    const uint64_t n = varint();
    if (n > uint64_t(e - p)) throw std::runtime_error("proto: truncated length-delimited field");
    const uint8_t* b = p;
    p += n;
    return {b, size_t(n)};
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1:
        if (e - p < 8) throw std::runtime_error("proto: truncated fixed64");
        p += 8;
        break;
      case 2: bytes(); break;
      case 5:
        if (e - p < 4) throw std::runtime_error("proto: truncated fixed32");
        p += 4;
        break;
      default: throw std::runtime_error("proto: bad wire type " + std::to_string(wt));
    }
  }
};

// one repeated integer field: packed (wire type 2) or not (wire type 0)
void take_ints(Reader& r, int wt, std::vector<uint64_t>& out) {
  if (wt == 0) {
    out.push_back(r.varint());
    return;
  }
  if (wt != 2) throw std::runtime_error("proto: bad wire type for a repeated integer");
  auto [b, n] = r.bytes();
  Reader sub{b, b + n};
  while (sub.p < sub.e) out.push_back(sub.varint());
}

template <class T>
py::array_t<T> to_array(const std::vector<uint64_t>& v) {
  py::array_t<T> a(v.size());
  T* d = a.mutable_data();
  for (size_t i = 0; i < v.size(); i++) d[i] = T(v[i]);
  return a;
}

// decode_import_request(body, values=False) -> dict with Index, Field, Shard,
// and numpy arrays (RowIDs, ColumnIDs, Timestamps | ColumnIDs, Values) plus
// the key lists.  Field numbers: ImportRequest 1 Index, 2 Field, 3 Shard,
// 4 RowIDs, 5 ColumnIDs, 6 Timestamps, 7 RowKeys, 8 ColumnKeys;
// ImportValueRequest 1, 2, 3, 5 ColumnIDs, 6 Values, 7 ColumnKeys.
py::dict decode_import_request(py::bytes body, bool values) {
  std::string buf = body;
  std::string index, field;
  uint64_t shard = 0;
  std::vector<uint64_t> rows, cols, vals, ts;
  std::vector<std::string> rkeys, ckeys;
  {
    py::gil_scoped_release nogil;
    Reader r{reinterpret_cast<const uint8_t*>(buf.data()), reinterpret_cast<const uint8_t*>(buf.data()) + buf.size()};
    while (r.p < r.e) {
      const uint64_t tag = r.varint();
      const int fn = int(tag >> 3), wt = int(tag & 7);
      if (fn == 1 && wt == 2) {
        auto [b, n] = r.bytes();
        index.assign(reinterpret_cast<const char*>(b), n);
      } else if (fn == 2 && wt == 2) {
        auto [b, n] = r.bytes();
        field.assign(reinterpret_cast<const char*>(b), n);
      } else if (fn == 3 && wt == 0) {
        shard = r.varint();
      } else if (!values && fn == 4 && (wt == 0 || wt == 2)) {
        take_ints(r, wt, rows);
      } else if (fn == 5 && (wt == 0 || wt == 2)) {
        take_ints(r, wt, cols);
      } else if (fn == 6 && (wt == 0 || wt == 2)) {
        take_ints(r, wt, values ? vals : ts);
      } else if (!values && fn == 7 && wt == 2) {
        auto [b, n] = r.bytes();
        rkeys.emplace_back(reinterpret_cast<const char*>(b), n);
      } else if ((values ? fn == 7 : fn == 8) && wt == 2) {
        auto [b, n] = r.bytes();
        ckeys.emplace_back(reinterpret_cast<const char*>(b), n);
      } else {
        r.skip(wt);
      }
    }
  }
  py::dict d;
  d["Index"] = index;
  d["Field"] = field;
  d["Shard"] = shard;
  d["ColumnIDs"] = to_array<uint64_t>(cols);
  d["ColumnKeys"] = ckeys;
  if (values) {
    d["Values"] = to_array<int64_t>(vals);  // int64 varints: two's complement in 64 bits
  } else {
    d["RowIDs"] = to_array<uint64_t>(rows);
    d["RowKeys"] = rkeys;
    d["Timestamps"] = to_array<int64_t>(ts);
  }
  return d;
}

}  // namespace

void register_wire_decode(py::module_& m) {
  m.def("decode_import_request", &decode_import_request, py::arg("body"), py::arg("values") = false,
        "ImportRequest / ImportValueRequest protobuf body -> dict with numpy id/value arrays");
}
