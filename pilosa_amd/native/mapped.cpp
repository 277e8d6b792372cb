// MappedBitmap: copy-on-write view of a Pilosa fragment file through mmap
// (declaration and contract in roaring.hpp).  Reference behaviour being
// matched: roaring/container_stash.go:262-346 (frozen containers that point
// into the mapped file, unfrozen on write), roaring.go:1616-1622 (mapped
// unmarshal), fragment.go:311-456 (fragment open maps the file and replays
// the op log).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <set>
#include <stdexcept>

#include "roaring.hpp"

namespace pr {

namespace {
inline uint16_t r16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
inline uint32_t r32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint64_t r64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

// Keys the op log at ``data`` touches (checksums are verified by the replay
// that follows; a torn tail is reported there, as Bitmap::from_bytes does).
void op_keys(const uint8_t* data, size_t n, std::set<uint64_t>& keys) {
  size_t pos = 0;
  while (pos + 13 <= n) {
    const uint8_t* p = data + pos;
    const uint8_t typ = p[0];
    const uint64_t value = r64(p + 1);
    size_t sz = 13;
    switch (typ) {
      case OP_ADD:
      case OP_REMOVE:
        keys.insert(value >> 16);
        break;
      case OP_ADD_BATCH:
      case OP_REMOVE_BATCH:
        if (value > (1ull << 59) || n - pos < 13 + value * 8) return;
        for (uint64_t k = 0; k < value; k++) keys.insert(r64(p + 13 + k * 8) >> 16);
        sz = 13 + value * 8;
        break;
      case OP_ADD_ROARING:
      case OP_REMOVE_ROARING: {
        if (n - pos < 17 + value) return;
        Bitmap blob;
        blob.from_bytes(p + 17, value);
        for (auto& kv : blob.cs) keys.insert(kv.first);
        sz = 17 + value;
        break;
      }
      default:
        return;
    }
    pos += sz;
  }
}
}  // namespace

MappedBitmap::MappedBitmap(const std::string& path) {
  fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd_ < 0) throw std::runtime_error("open " + path + ": " + strerror(errno));
  struct stat st;
  if (fstat(fd_, &st) != 0) {
    ::close(fd_);
    throw std::runtime_error("stat " + path + ": " + strerror(errno));
  }
  len_ = size_t(st.st_size);
  void* p = len_ ? mmap(nullptr, len_, PROT_READ, MAP_SHARED, fd_, 0) : nullptr;
  const int err = errno;
  // the mapping stays valid without the descriptor: one fd per fragment
  // (Fragment's own append handle), as the reference keeps
  ::close(fd_);
  fd_ = -1;
  if (len_ == 0) return;  // empty fragment
  if (p == MAP_FAILED) throw std::runtime_error("mmap " + path + ": " + strerror(err));
  base_ = static_cast<const uint8_t*>(p);
  madvise(p, len_, MADV_RANDOM);
  auto fail = [&](const std::string& msg) {
    munmap(const_cast<uint8_t*>(base_), len_);
    base_ = nullptr;
    throw std::runtime_error(msg);
  };
  if (len_ < size_t(HEADER_BASE)) fail("data too small");
  if (r16(base_) != MAGIC) fail("not a Pilosa-format roaring file (mapped access needs one)");
  if (base_[2] != STORAGE_VERSION) fail("wrong roaring version");
  flags = base_[3];
  keyn_ = r32(base_ + 4);
  if (size_t(HEADER_BASE) + size_t(keyn_) * 16 > len_) fail("malformed bitmap, header overruns data");
  hdr_ = base_ + HEADER_BASE;
  offs_ = hdr_ + size_t(keyn_) * 12;
  // Only the LAST container is checked here (the op log follows it): the
  // header is not walked at open, so opening touches a few pages however
  // many containers the file holds.  Every access bounds-checks the
  // container it reads instead (span()).
  size_t end = HEADER_BASE + size_t(keyn_) * 16;
  if (keyn_) {
    size_t off, sz;
    if (!span(keyn_ - 1, &off, &sz)) fail("container overruns data");
    end = off + sz;
  }
  if (end < len_) {
    std::set<uint64_t> keys;
    try {
      op_keys(base_ + end, len_ - end, keys);
      for (uint64_t k : keys) cow(k);
      over_.replay_ops(base_ + end, len_ - end);
    } catch (const std::exception& e) {
      fail(std::string("op log: ") + e.what());
    }
    ops = over_.ops;
    opn = over_.opn;
  }
}

MappedBitmap::~MappedBitmap() {
  if (base_) munmap(const_cast<uint8_t*>(base_), len_);
  if (fd_ >= 0) ::close(fd_);
}

uint64_t MappedBitmap::key_at(size_t i) const { return r64(hdr_ + i * 12); }

size_t MappedBitmap::lower(uint64_t key) const {
  size_t lo = 0, hi = keyn_;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (key_at(mid) < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

int64_t MappedBitmap::find(uint64_t key) const {
  const size_t i = lower(key);
  return i < keyn_ && key_at(i) == key ? int64_t(i) : -1;
}

bool MappedBitmap::span(size_t i, size_t* off, size_t* sz) const {
  *off = r32(offs_ + i * 4);
  const uint16_t typ = r16(hdr_ + i * 12 + 8);
  if (typ == CT_ARRAY) *sz = size_t(mapped_n(i)) * 2;
  else if (typ == CT_BITMAP) *sz = size_t(BITMAP_N) * 8;
  else if (typ == CT_RUN) {
    if (*off + 2 > len_) return false;
    *sz = 2 + size_t(r16(base_ + *off)) * 4;
  } else {
    return false;
  }
  return *off + *sz <= len_;
}

const uint8_t* MappedBitmap::payload(size_t i) const {
  size_t off, sz;
  if (!span(i, &off, &sz))
    throw std::runtime_error("mapped container " + std::to_string(key_at(i)) + " overruns the file or has an unknown type");
  return base_ + off;
}

int32_t MappedBitmap::mapped_n(size_t i) const { return int32_t(r16(hdr_ + i * 12 + 10)) + 1; }

Container MappedBitmap::load(size_t i) const {
  Container c;
  c.type = uint8_t(r16(hdr_ + i * 12 + 8));
  c.n = mapped_n(i);
  const uint8_t* d = payload(i);
  switch (c.type) {
    case CT_ARRAY:
      c.a.resize(size_t(c.n));
      memcpy(c.a.data(), d, size_t(c.n) * 2);
      break;
    case CT_BITMAP:
      c.b.resize(BITMAP_N);
      memcpy(c.b.data(), d, size_t(BITMAP_N) * 8);
      break;
    default: {
      const uint16_t nr = r16(d);
      c.r.resize(nr);
      for (uint16_t k = 0; k < nr; k++) {
        c.r[k].start = r16(d + 2 + size_t(k) * 4);
        c.r[k].last = r16(d + 4 + size_t(k) * 4);
      }
    }
  }
  return c;
}

bool MappedBitmap::mapped_contains(size_t i, uint16_t low) const {
  const uint8_t* d = payload(i);
  switch (r16(hdr_ + i * 12 + 8)) {
    case CT_ARRAY: {
      size_t lo = 0, hi = size_t(mapped_n(i));
      while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        const uint16_t v = r16(d + mid * 2);
        if (v == low) return true;
        if (v < low) lo = mid + 1;
        else hi = mid;
      }
      return false;
    }
    case CT_BITMAP:
      return (r64(d + size_t(low >> 6) * 8) >> (low & 63)) & 1;
    default: {
      size_t lo = 0, hi = r16(d);
      while (lo < hi) {  // first run with last >= low
        const size_t mid = (lo + hi) / 2;
        if (r16(d + 4 + mid * 4) < low) lo = mid + 1;
        else hi = mid;
      }
      return lo < r16(d) && r16(d + 2 + lo * 4) <= low;
    }
  }
}

Container& MappedBitmap::cow(uint64_t key) {
  if (!touched_.count(key)) {
    touched_.emplace(key, true);
    const int64_t i = find(key);
    if (i >= 0) over_.cs[key] = load(size_t(i));
  }
  return get_or_create(over_, key);
}

bool MappedBitmap::contains(uint64_t v) const {
  const uint64_t key = v >> 16;
  if (touched_.count(key)) return over_.contains(v);
  const int64_t i = find(key);
  return i >= 0 && mapped_contains(size_t(i), uint16_t(v & 0xffff));
}

bool MappedBitmap::add(uint64_t v) {
  if (contains(v)) return false;
  cow(v >> 16);
  return over_.add(v);
}

bool MappedBitmap::remove(uint64_t v) {
  if (!contains(v)) return false;
  cow(v >> 16);
  return over_.remove(v);
}

int64_t MappedBitmap::count_range(uint64_t start, uint64_t end) const {
  if (end <= start) return 0;
  const uint64_t sk = start >> 16, ek = (end - 1) >> 16;  // inclusive key span
  int64_t n = 0;
  for (size_t i = lower(sk); i < keyn_ && key_at(i) <= ek; i++) {
    const uint64_t key = key_at(i);
    if (touched_.count(key)) continue;
    const uint64_t k0 = key << 16;
    if (k0 >= start && k0 + 65536 <= end) {
      n += mapped_n(i);  // whole container: the header's cardinality, payload untouched
    } else {
      const int s = int(std::max(start, k0) - k0), e = int(std::min(end, k0 + 65536) - k0);
      n += load(i).count_range(s, e);
    }
  }
  for (auto it = touched_.lower_bound(sk); it != touched_.end() && it->first <= ek; ++it) {
    auto c = over_.cs.find(it->first);
    if (c == over_.cs.end()) continue;
    const uint64_t k0 = it->first << 16;
    const int s = int(std::max(start, k0) - k0), e = int(std::min(end, k0 + 65536) - k0);
    n += (s == 0 && e == 65536) ? c->second.n : c->second.count_range(s, e);
  }
  return n;
}

int64_t MappedBitmap::count() const { return count_range(0, ~0ull); }

bool MappedBitmap::any() const {
  for (size_t i = 0; i < keyn_; i++)
    if (!touched_.count(key_at(i))) return true;  // mapped containers are never empty (n-1 encoding)
  for (auto& kv : over_.cs)
    if (kv.second.n) return true;
  return false;
}

uint64_t MappedBitmap::max() const {
  uint64_t best = 0;
  bool have = false;
  for (size_t i = keyn_; i-- > 0;) {
    if (touched_.count(key_at(i))) continue;
    best = (key_at(i) << 16) | uint64_t(load(i).max());
    have = true;
    break;
  }
  for (auto it = over_.cs.rbegin(); it != over_.cs.rend(); ++it) {
    if (!it->second.n) continue;
    const uint64_t v = (it->first << 16) | uint64_t(it->second.max());
    if (!have || v > best) best = v;
    break;
  }
  return best;
}

Bitmap MappedBitmap::offset_range(uint64_t offset, uint64_t start, uint64_t end) const {
  if ((offset & 0xffff) || (start & 0xffff) || (end & 0xffff))
    throw std::invalid_argument("offset_range: offset/start/end must be multiples of 65536");
  Bitmap out;
  const uint64_t off = offset >> 16, sk = start >> 16, ek = end >> 16;
  for (size_t i = lower(sk); i < keyn_ && key_at(i) < ek; i++)
    if (!touched_.count(key_at(i))) out.cs.emplace(off + (key_at(i) - sk), load(i));
  for (auto it = over_.cs.lower_bound(sk); it != over_.cs.end() && it->first < ek; ++it)
    if (it->second.n) out.cs[off + (it->first - sk)] = it->second;
  return out;
}

Bitmap MappedBitmap::sub_shard(int key_shift, uint64_t sub) const {
  if (key_shift < 4 || key_shift > 16) throw std::invalid_argument("sub_shard: key_shift must be in [4, 16]");
  const uint64_t mask = (uint64_t(1) << (key_shift - 4)) - 1;
  if (sub > mask) throw std::invalid_argument("sub_shard: sub-shard out of range");
  Bitmap out;
  auto rekey = [&](uint64_t k) { return ((k >> key_shift) << 4) | (k & 15); };
  for (size_t i = 0; i < keyn_; i++) {
    const uint64_t k = key_at(i);
    if (((k >> 4) & mask) == sub && !touched_.count(k)) out.cs.emplace(rekey(k), load(i));
  }
  for (auto& kv : over_.cs)
    if (kv.second.n && ((kv.first >> 4) & mask) == sub) out.cs[rekey(kv.first)] = kv.second;
  return out;
}

std::vector<uint64_t> MappedBitmap::rows_with_column(uint64_t col, uint64_t cpr) const {
  const uint64_t ck = col >> 16;
  const uint16_t low = uint16_t(col & 0xffff);
  std::set<uint64_t> rows;
  for (size_t i = 0; i < keyn_; i++) {
    const uint64_t key = key_at(i);
    if (key % cpr != ck || touched_.count(key)) continue;
    if (mapped_contains(i, low)) rows.insert(key / cpr);
  }
  for (auto& kv : over_.cs)
    if (kv.first % cpr == ck && kv.second.n && kv.second.contains(low)) rows.insert(kv.first / cpr);
  return std::vector<uint64_t>(rows.begin(), rows.end());
}

int64_t MappedBitmap::add_many(const uint64_t* v, size_t n) {
  int64_t changed = 0;
  for (size_t i = 0; i < n;) {
    const uint64_t key = v[i] >> 16;
    size_t j = i;
    while (j < n && (v[j] >> 16) == key) j++;
    cow(key);
    changed += over_.add_many(v + i, j - i);
    i = j;
  }
  return changed;
}

int64_t MappedBitmap::remove_many(const uint64_t* v, size_t n) {
  int64_t changed = 0;
  for (size_t i = 0; i < n;) {
    const uint64_t key = v[i] >> 16;
    size_t j = i;
    while (j < n && (v[j] >> 16) == key) j++;
    if (touched_.count(key) || find(key) >= 0) {  // nothing to clear in an absent container
      cow(key);
      changed += over_.remove_many(v + i, j - i);
    }
    i = j;
  }
  return changed;
}

int64_t MappedBitmap::import_roaring(const uint8_t* data, size_t n, bool clear, uint64_t cpr,
                                     std::map<uint64_t, int64_t>* rowdelta) {
  Bitmap blob;
  blob.from_bytes(data, n);
  for (auto& kv : blob.cs)
    if (kv.second.n && (!clear || touched_.count(kv.first) || find(kv.first) >= 0)) cow(kv.first);
  // over_ now owns every container the blob can change
  return over_.import_roaring(data, n, clear, cpr, rowdelta);
}

namespace {
void put_le(std::string& s, uint64_t v, int bytes) {
  for (int k = 0; k < bytes; k++) s.push_back(char((v >> (8 * k)) & 0xff));
}
}  // namespace

size_t MappedBitmap::write_snapshot(const std::string& path) {
  for (auto& kv : touched_) {
    auto it = over_.cs.find(kv.first);
    if (it != over_.cs.end() && it->second.n) it->second.optimize();
  }
  // merged key order: (key, mapped index or -1 for the overlay copy)
  std::vector<std::pair<uint64_t, int64_t>> order;
  order.reserve(keyn_ + touched_.size());
  size_t i = 0;
  auto ot = touched_.begin();
  while (i < keyn_ || ot != touched_.end()) {
    const uint64_t mk = i < keyn_ ? key_at(i) : ~0ull;
    const uint64_t tk = ot != touched_.end() ? ot->first : ~0ull;
    if (tk <= mk) {
      auto c = over_.cs.find(tk);
      if (c != over_.cs.end() && c->second.n) order.emplace_back(tk, -1);
      ++ot;
      if (tk == mk) i++;  // the overlay copy replaces the mapped container
    } else {
      order.emplace_back(mk, int64_t(i));
      i++;
    }
  }
  std::string head;
  head.reserve(HEADER_BASE + order.size() * 16);
  put_le(head, MAGIC | (STORAGE_VERSION << 16) | (uint32_t(flags) << 24), 4);
  put_le(head, order.size(), 4);
  std::vector<size_t> sizes(order.size());
  for (size_t k = 0; k < order.size(); k++) {
    uint16_t typ;
    int32_t cn;
    if (order[k].second >= 0) {
      const size_t mi = size_t(order[k].second);
      size_t off;
      if (!span(mi, &off, &sizes[k])) throw std::runtime_error("write_snapshot: corrupt mapped container");
      typ = r16(hdr_ + mi * 12 + 8);
      cn = mapped_n(mi);
    } else {
      const Container& c = over_.cs.at(order[k].first);
      typ = c.type;
      cn = c.n;
      sizes[k] = c.encoded_size();
    }
    put_le(head, order[k].first, 8);
    put_le(head, typ, 2);
    put_le(head, uint16_t(cn - 1), 2);
  }
  size_t off = HEADER_BASE + order.size() * 16;
  for (size_t k = 0; k < order.size(); k++) {
    if (off + sizes[k] > 0xFFFFFFFFull) throw std::runtime_error("write_snapshot: file exceeds 4 GiB offsets");
    put_le(head, off, 4);
    off += sizes[k];
  }
  FILE* fh = fopen(path.c_str(), "wb");
  if (!fh) throw std::runtime_error("write_snapshot: open " + path + ": " + strerror(errno));
  bool ok = fwrite(head.data(), 1, head.size(), fh) == head.size();
  std::string buf;
  for (size_t k = 0; k < order.size() && ok; k++) {
    if (order[k].second >= 0) {
      ok = fwrite(payload(size_t(order[k].second)), 1, sizes[k], fh) == sizes[k];
      continue;
    }
    const Container& c = over_.cs.at(order[k].first);
    buf.clear();
    switch (c.type) {
      case CT_ARRAY: buf.append(reinterpret_cast<const char*>(c.a.data()), c.a.size() * 2); break;
      case CT_BITMAP: buf.append(reinterpret_cast<const char*>(c.b.data()), size_t(BITMAP_N) * 8); break;
      default:
        put_le(buf, c.r.size(), 2);
        for (const Iv& iv : c.r) {
          put_le(buf, iv.start, 2);
          put_le(buf, iv.last, 2);
        }
    }
    ok = fwrite(buf.data(), 1, buf.size(), fh) == buf.size();
  }
  if (fclose(fh) != 0) ok = false;
  if (!ok) throw std::runtime_error("write_snapshot: short write to " + path);
  return off;
}

}  // namespace pr
