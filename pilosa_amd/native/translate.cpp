// Key <-> id translation store on the reference's log format
// (translate.go:716-866 LogEntry, :880-1037 RHH index), pybind11 module
// ``_translate``.
//
// File: a sequence of entries
//   uvarint len | u8 type (1 column, 2 row) | uvarint len(index) index |
//   uvarint len(field) field | uvarint n | n x (uvarint id, uvarint len(key) key)
// where ``len`` counts the bytes after itself.  The file is mapped read-only
// (MAP_SHARED, a large reservation that grows by remapping) and appended
// with write(2) + fdatasync, so the page cache keeps the mapping coherent.
//
// Per (type, index, field) a Robin-Hood hash table maps key -> (id, offset
// of the key's uvarint length in the file) without copying key bytes onto
// the heap; ids are dense from 1, so id -> offset is a flat vector.  Lookups
// take a shared lock and run without the GIL.
#include <fcntl.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

constexpr uint8_t T_COLUMN = 1, T_ROW = 2;

inline void put_uvarint(std::string& b, uint64_t v) {
  while (v >= 0x80) {
    b.push_back(char(uint8_t(v) | 0x80));
    v >>= 7;
  }
  b.push_back(char(uint8_t(v)));
}

// Returns bytes consumed, 0 on truncation/overflow.
inline size_t get_uvarint(const uint8_t* p, size_t avail, uint64_t* out) {
  uint64_t v = 0;
  for (size_t i = 0; i < avail && i < 10; i++) {
    v |= uint64_t(p[i] & 0x7f) << (7 * i);
    if (!(p[i] & 0x80)) {
      *out = v;
      return i + 1;
    }
  }
  return 0;
}

inline size_t uvarint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}

// MurmurHash64A; 0 is reserved for "empty slot".
inline uint64_t hash_key(const uint8_t* k, size_t len) {
  const uint64_t m = 0xc6a4a7935bd1e995ULL;
  const int r = 47;
  uint64_t h = 0x9747b28c0ddc0ffeULL ^ (len * m);
  size_t n8 = len / 8;
  for (size_t i = 0; i < n8; i++) {
    uint64_t w;
    memcpy(&w, k + 8 * i, 8);
    w *= m;
    w ^= w >> r;
    w *= m;
    h ^= w;
    h *= m;
  }
  const uint8_t* t = k + 8 * n8;
  switch (len & 7) {
    case 7: h ^= uint64_t(t[6]) << 48; [[fallthrough]];
    case 6: h ^= uint64_t(t[5]) << 40; [[fallthrough]];
    case 5: h ^= uint64_t(t[4]) << 32; [[fallthrough]];
    case 4: h ^= uint64_t(t[3]) << 24; [[fallthrough]];
    case 3: h ^= uint64_t(t[2]) << 16; [[fallthrough]];
    case 2: h ^= uint64_t(t[1]) << 8; [[fallthrough]];
    case 1: h ^= uint64_t(t[0]); h *= m;
  }
  h ^= h >> r;
  h *= m;
  h ^= h >> r;
  return h ? h : 1;
}

struct Elem {
  uint64_t hash = 0;
  int64_t offset = 0;  // file offset of the key's uvarint length
  uint64_t id = 0;
};

struct Parsed {
  uint8_t type = 0;
  std::string index, field;
  size_t pairs_at = 0;  // file offset of the first (id, key) pair
  uint64_t n = 0;
  size_t end = 0;       // file offset just past the entry
};

class Store;

// Robin-Hood key -> (id, offset) map plus dense id -> offset.
struct KeyIndex {
  uint64_t seq = 0;
  std::vector<Elem> elems;
  uint64_t mask = 0, threshold = 0, n = 0;
  std::vector<int64_t> off_by_id;                  // id -> offset, -1 = none
  std::unordered_map<uint64_t, int64_t> sparse;    // ids far past the dense range

  KeyIndex() { alloc(256); }

  void alloc(uint64_t cap) {
    elems.assign(cap, Elem{});
    mask = cap - 1;
    threshold = cap * 90 / 100;  // load factor 90 (translate.go defaultLoadFactor)
  }
  uint64_t dist(uint64_t hash, uint64_t i) const { return (i + elems.size() - (hash & mask)) & mask; }

  void set_offset(uint64_t id, int64_t off) {
    if (id < off_by_id.size()) {
      off_by_id[id] = off;
    } else if (id < 2 * off_by_id.size() + (1u << 20)) {
      off_by_id.resize(std::max<size_t>(id + 1, off_by_id.size() * 3 / 2 + 1024), -1);
      off_by_id[id] = off;
    } else {
      sparse[id] = off;
    }
  }
  int64_t offset_of(uint64_t id) const {
    if (id < off_by_id.size()) return off_by_id[id];
    auto it = sparse.find(id);
    return it == sparse.end() ? -1 : it->second;
  }
};

inline bool key_at(const uint8_t* data, size_t size, int64_t off, const uint8_t** k, size_t* len) {
  uint64_t l;
  size_t s = get_uvarint(data + off, size - size_t(off), &l);
  if (!s || size_t(off) + s + l > size) return false;
  *k = data + off + s;
  *len = size_t(l);
  return true;
}

class Store {
 public:
  Store(std::string path, bool read_only, uint64_t map_size)
      : path_(std::move(path)), read_only_(read_only), map_size_(map_size ? map_size : (10ULL << 30)) {}
  ~Store() { close(); }

  // Open + replay; returns the number of bytes of valid entries (a torn
  // tail is truncated away).
  int64_t open() {
    std::unique_lock<std::shared_mutex> g(mu_);
    closed_ = false;
    if (!path_.empty()) {
      fd_ = ::open(path_.c_str(), O_RDWR | O_CREAT | O_APPEND | O_CLOEXEC, 0666);
      if (fd_ < 0) throw std::runtime_error("open " + path_ + ": " + strerror(errno));
      struct stat st;
      fstat(fd_, &st);
      size_ = size_t(st.st_size);
      remap(size_);
    }
    idx_.clear();
    size_t end = replay(0, size_);
    if (end != size_) {
      if (!path_.empty() && ftruncate(fd_, off_t(end)) != 0)
        throw std::runtime_error("truncate " + path_ + ": " + strerror(errno));
      if (path_.empty()) mem_.resize(end);
      size_ = end;
    }
    return int64_t(end);
  }

  void close() {
    std::unique_lock<std::shared_mutex> g(mu_);
    if (map_) munmap(map_, map_len_);
    map_ = nullptr;
    map_len_ = 0;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    // a closed store answers nothing: callers racing a close()/reopen get an
    // error instead of reading key offsets through an unmapped log
    idx_.clear();
    size_ = 0;
    mem_.clear();
    closed_ = true;
  }

  int64_t size() {
    std::shared_lock<std::shared_mutex> g(mu_);
    return int64_t(size_);
  }
  bool read_only() const { return read_only_; }
  void set_read_only(bool v) { read_only_ = v; }

  // keys -> ids; with create (and a writable store) missing keys get the
  // next ids in one appended entry.  Missing keys map to 0 otherwise.
  std::vector<uint64_t> translate(uint8_t type, const std::string& index, const std::string& field,
                                  const std::vector<std::string>& keys, bool create) {
    std::vector<uint64_t> ids(keys.size(), 0);
    bool missing = false;
    {
      std::shared_lock<std::shared_mutex> g(mu_);
      check_open();
      const KeyIndex* ki = find_index(type, index, field);
      for (size_t i = 0; i < keys.size(); i++) {
        ids[i] = ki ? lookup(*ki, keys[i]) : 0;
        missing |= ids[i] == 0;
      }
    }
    if (!missing || !create || read_only_) return ids;
    std::unique_lock<std::shared_mutex> g(mu_);
    check_open();
    KeyIndex& ki = index_for(type, index, field);
    std::unordered_map<std::string, uint64_t> fresh;
    std::vector<size_t> new_pos;
    std::vector<uint64_t> new_ids;
    for (size_t i = 0; i < keys.size(); i++) {
      if (ids[i]) continue;
      if ((ids[i] = lookup(ki, keys[i]))) continue;  // created between the locks
      auto it = fresh.find(keys[i]);
      if (it != fresh.end()) {
        ids[i] = it->second;
        continue;
      }
      ids[i] = ++ki.seq;
      fresh.emplace(keys[i], ids[i]);
      new_pos.push_back(i);
      new_ids.push_back(ids[i]);
    }
    if (new_pos.empty()) return ids;
    std::string body;
    body.push_back(char(type));
    put_uvarint(body, index.size());
    body += index;
    put_uvarint(body, type == T_ROW ? field.size() : 0);
    if (type == T_ROW) body += field;
    put_uvarint(body, new_pos.size());
    for (size_t j = 0; j < new_pos.size(); j++) {
      put_uvarint(body, new_ids[j]);
      put_uvarint(body, keys[new_pos[j]].size());
      body += keys[new_pos[j]];
    }
    std::string rec;
    put_uvarint(rec, body.size());
    rec += body;
    const size_t at = size_;
    append(rec);
    size_t end = replay(at, size_);  // index the entry from its bytes in the file
    if (end != size_) throw std::runtime_error("translate: appended entry failed to parse");
    return ids;
  }

  // ids -> keys ("" when unknown, like TranslateColumnToString).
  std::vector<std::string> keys_of(uint8_t type, const std::string& index, const std::string& field,
                                   const std::vector<uint64_t>& ids) {
    std::shared_lock<std::shared_mutex> g(mu_);
    check_open();
    std::vector<std::string> out(ids.size());
    const KeyIndex* ki = find_index(type, index, field);
    if (!ki) return out;
    const uint8_t* d = data();
    for (size_t i = 0; i < ids.size(); i++) {
      int64_t off = ki->offset_of(ids[i]);
      const uint8_t* k;
      size_t len;
      if (off >= 0 && key_at(d, size_, off, &k, &len)) out[i].assign(reinterpret_cast<const char*>(k), len);
    }
    return out;
  }

  // Replica tailing: validate whole entries, append them verbatim, index
  // them.  Returns the bytes consumed (a partial trailing entry is left).
  int64_t apply_log(const std::string& chunk) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(chunk.data());
    size_t used = 0;
    while (used < chunk.size()) {
      Parsed e;
      if (!parse(p + used, chunk.size() - used, 0, &e)) break;
      used = used + e.end;
    }
    if (!used) return 0;
    std::unique_lock<std::shared_mutex> g(mu_);
    check_open();
    const size_t at = size_;
    append(chunk.substr(0, used));
    replay(at, size_);
    return int64_t(used);
  }

  py::bytes read_from(int64_t offset) {
    std::string out;
    {
      std::shared_lock<std::shared_mutex> g(mu_);
      check_open();
      if (offset < 0) offset = 0;
      if (size_t(offset) < size_) out.assign(reinterpret_cast<const char*>(data()) + offset, size_ - size_t(offset));
    }
    return py::bytes(out);
  }

  uint64_t seq(uint8_t type, const std::string& index, const std::string& field) {
    std::shared_lock<std::shared_mutex> g(mu_);
    const KeyIndex* ki = find_index(type, index, field);
    return ki ? ki->seq : 0;
  }

  // [(type, index, field, ids, keys)] of every entry from ``offset`` (tests,
  // the inspect command).
  py::list entries(int64_t offset) {
    std::shared_lock<std::shared_mutex> g(mu_);
    check_open();
    py::list out;
    size_t at = size_t(std::max<int64_t>(offset, 0));
    const uint8_t* d = data();
    while (at < size_) {
      Parsed e;
      if (!parse(d + at, size_ - at, at, &e)) break;
      py::list ids, keys;
      size_t q = e.pairs_at;
      for (uint64_t i = 0; i < e.n; i++) {
        uint64_t id, kl;
        q += get_uvarint(d + q, size_ - q, &id);
        q += get_uvarint(d + q, size_ - q, &kl);
        ids.append(id);
        keys.append(py::bytes(reinterpret_cast<const char*>(d + q), kl));
        q += kl;
      }
      // names come from the file: decode lossily so a damaged log can still be inspected
      out.append(py::make_tuple(int(e.type), lossy(e.index), lossy(e.field), ids, keys, e.end - at));
      at = e.end;
    }
    return out;
  }

 private:
  static py::str lossy(const std::string& s) {
    PyObject* o = PyUnicode_DecodeUTF8(s.data(), Py_ssize_t(s.size()), "replace");
    if (!o) throw py::error_already_set();
    return py::reinterpret_steal<py::str>(o);
  }
  void check_open() const {
    if (closed_) throw std::runtime_error("translate store " + path_ + " is closed");
  }

  const uint8_t* data() const {
    return path_.empty() ? reinterpret_cast<const uint8_t*>(mem_.data()) : reinterpret_cast<const uint8_t*>(map_);
  }

  void remap(size_t need) {
    if (path_.empty()) return;
    if (map_ && need <= map_len_) return;
    size_t len = map_len_ ? map_len_ : size_t(map_size_);
    while (len < need) len *= 2;
    if (map_) munmap(map_, map_len_);
    map_ = mmap(nullptr, len, PROT_READ, MAP_SHARED, fd_, 0);
    if (map_ == MAP_FAILED) {
      map_ = nullptr;
      map_len_ = 0;
      throw std::runtime_error("mmap " + path_ + ": " + strerror(errno));
    }
    map_len_ = len;
  }

  void append(const std::string& rec) {
    if (path_.empty()) {
      mem_ += rec;
    } else {
      size_t done = 0;
      while (done < rec.size()) {
        ssize_t w = ::write(fd_, rec.data() + done, rec.size() - done);
        if (w < 0) {
          if (errno == EINTR) continue;
          throw std::runtime_error("write " + path_ + ": " + strerror(errno));
        }
        done += size_t(w);
      }
      if (fdatasync(fd_) != 0) throw std::runtime_error("sync " + path_ + ": " + strerror(errno));
      remap(size_ + rec.size());
    }
    size_ += rec.size();
  }

  // Parse the entry at p (``base`` = its file offset); false if torn.
  static bool parse(const uint8_t* p, size_t avail, size_t base, Parsed* e) {
    uint64_t len;
    size_t s = get_uvarint(p, avail, &len);
    if (!s || s + len > avail || len < 1) return false;
    const uint8_t* q = p + s;
    const uint8_t* end = q + len;
    e->type = *q++;
    uint64_t il, fl, n;
    size_t t = get_uvarint(q, size_t(end - q), &il);
    if (!t || il > uint64_t(end - q - t)) return false;
    q += t;
    e->index.assign(reinterpret_cast<const char*>(q), il);
    q += il;
    t = get_uvarint(q, size_t(end - q), &fl);
    if (!t || fl > uint64_t(end - q - t)) return false;
    q += t;
    e->field.assign(reinterpret_cast<const char*>(q), fl);
    q += fl;
    t = get_uvarint(q, size_t(end - q), &n);
    if (!t) return false;
    q += t;
    e->pairs_at = base + size_t(q - p);
    e->n = n;
    for (uint64_t i = 0; i < n; i++) {
      uint64_t id, kl;
      t = get_uvarint(q, size_t(end - q), &id);
      if (!t) return false;
      q += t;
      t = get_uvarint(q, size_t(end - q), &kl);
      if (!t || kl > uint64_t(end - q - t)) return false;
      q += t + kl;
    }
    if (q != end || (e->type != T_COLUMN && e->type != T_ROW)) return false;
    e->end = base + s + size_t(len);
    return true;
  }

  // Index every whole entry in [from, to); returns where parsing stopped.
  size_t replay(size_t from, size_t to) {
    const uint8_t* d = data();
    size_t at = from;
    while (at < to) {
      Parsed e;
      if (!parse(d + at, to - at, at, &e)) break;
      KeyIndex& ki = index_for(e.type, e.index, e.field);
      size_t q = e.pairs_at;
      for (uint64_t i = 0; i < e.n; i++) {
        uint64_t id, kl;
        q += get_uvarint(d + q, to - q, &id);
        insert(ki, id, int64_t(q));
        get_uvarint(d + q, to - q, &kl);
        q += uvarint_size(kl) + kl;
        if (id > ki.seq) ki.seq = id;
      }
      at = e.end;
    }
    return at;
  }

  static std::string ikey(uint8_t type, const std::string& index, const std::string& field) {
    std::string k(1, char(type));
    k += index;
    k.push_back('\0');
    if (type == T_ROW) k += field;
    return k;
  }
  const KeyIndex* find_index(uint8_t type, const std::string& index, const std::string& field) const {
    auto it = idx_.find(ikey(type, index, field));
    return it == idx_.end() ? nullptr : &it->second;
  }
  KeyIndex& index_for(uint8_t type, const std::string& index, const std::string& field) {
    return idx_[ikey(type, index, field)];
  }

  uint64_t lookup(const KeyIndex& ki, const std::string& key) const {
    const uint8_t* kb = reinterpret_cast<const uint8_t*>(key.data());
    const uint64_t h = hash_key(kb, key.size());
    const uint8_t* d = data();
    uint64_t pos = h & ki.mask, dist = 0;
    for (;;) {
      const Elem& e = ki.elems[pos];
      if (e.hash == 0 || dist > ki.dist(e.hash, pos)) return 0;
      if (e.hash == h) {
        const uint8_t* k;
        size_t len;
        if (key_at(d, size_, e.offset, &k, &len) && len == key.size() && memcmp(k, kb, len) == 0) return e.id;
      }
      pos = (pos + 1) & ki.mask;
      dist++;
    }
  }

  void insert(KeyIndex& ki, uint64_t id, int64_t off) {
    ki.set_offset(id, off);
    if (++ki.n > ki.threshold) {
      std::vector<Elem> old;
      old.swap(ki.elems);
      ki.alloc(old.size() * 2);
      for (const Elem& e : old)
        if (e.hash) place(ki, e);
    }
    const uint8_t* k;
    size_t len;
    if (!key_at(data(), size_, off, &k, &len)) return;
    if (place(ki, Elem{hash_key(k, len), off, id})) ki.n--;  // key re-mapped: no new slot
  }

  // Robin-Hood placement; true if an equal key was overwritten.
  bool place(KeyIndex& ki, Elem cur) {
    const uint8_t* d = data();
    const uint8_t *ck, *ek;
    size_t cl, el;
    key_at(d, size_, cur.offset, &ck, &cl);
    uint64_t pos = cur.hash & ki.mask, dist = 0;
    bool carrying_original = true;
    for (;;) {
      Elem& e = ki.elems[pos];
      if (e.hash == 0) {
        e = cur;
        return false;
      }
      if (carrying_original && e.hash == cur.hash && key_at(d, size_, e.offset, &ek, &el) && el == cl &&
          memcmp(ek, ck, cl) == 0) {
        e = cur;
        return true;
      }
      const uint64_t ed = ki.dist(e.hash, pos);
      if (ed < dist) {
        std::swap(e, cur);
        dist = ed;
        carrying_original = false;  // displaced entries are already unique
      }
      pos = (pos + 1) & ki.mask;
      dist++;
    }
  }

  std::string path_;
  bool read_only_;
  uint64_t map_size_;
  int fd_ = -1;
  void* map_ = nullptr;
  size_t map_len_ = 0;
  size_t size_ = 0;
  std::string mem_;
  bool closed_ = false;
  std::unordered_map<std::string, KeyIndex> idx_;
  mutable std::shared_mutex mu_;
};

}  // namespace

PYBIND11_MODULE(_translate, m) {
  m.doc() = "Key translation store on the reference LogEntry log with a Robin-Hood key index";
  m.attr("T_COLUMN") = int(T_COLUMN);
  m.attr("T_ROW") = int(T_ROW);
  py::class_<Store>(m, "Store")
      .def(py::init<std::string, bool, uint64_t>(), py::arg("path"), py::arg("read_only") = false,
           py::arg("map_size") = 0)
      .def("open", &Store::open, py::call_guard<py::gil_scoped_release>())
      .def("close", &Store::close, py::call_guard<py::gil_scoped_release>())
      .def("size", &Store::size)
      .def_property("read_only", &Store::read_only, &Store::set_read_only)
      .def("translate", &Store::translate, py::arg("type"), py::arg("index"), py::arg("field"), py::arg("keys"),
           py::arg("create") = true, py::call_guard<py::gil_scoped_release>())
      .def("keys_of", &Store::keys_of, py::call_guard<py::gil_scoped_release>())
      .def("apply_log", [](Store& s, py::bytes b) {
        std::string c = b;
        py::gil_scoped_release nogil;
        return s.apply_log(c);
      })
      .def("read_from", &Store::read_from)
      .def("seq", &Store::seq)
      .def("entries", &Store::entries, py::arg("offset") = 0);
}
