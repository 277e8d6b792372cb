// Fragment files <-> device container arena, without host Bitmaps (part of
// module pilosa_amd._roaring).
//
// Reference: a node opens every fragment by mmap + header walk + op-log replay
// (fragment.go:311-456 openStorage, roaring/roaring.go:1562-1653
// unmarshalPilosaRoaring) and keeps "mapped" containers that alias the file
// (roaring/container_stash.go:262-346).  Here the HBM arena is the read
// replica, so the loader goes straight from the mapped files to the arena
// layout of pyroaring.cpp: no per-container heap objects are ever created.
//
//   FragmentLoader(paths, nthreads)
//     scan()        mmap + validate every file's header; a file with an op log
//                   after its snapshot (or in the official roaring format) is
//                   materialised once through Bitmap::from_bytes (replay) and
//                   re-encoded, so every shard then reads as a plain snapshot
//     rows()        sorted distinct row ids over all shards (the directory)
//     fill_index()  rowptr / shard_base / meta (+ per-shard slack for in-place
//                   patches) with global payload offsets
//     fill_payload(s0, s1, out)  the payload of shards [s0, s1) into a caller
//                   buffer (pinned staging for the chunked H2D); the shards'
//                   mappings are released afterwards
//
//   write_zipf_fragments(dir, ...)  the bench's 1M-row x 1B-column Zipf set
//                   field written as one Pilosa-format fragment file per shard
//                   (writeToUnoptimized layout, roaring.go:1052-1122), plus
//                   the shard's `<shard>.cache` TopN rank-cache file (protobuf
//                   Cache{IDs}, fragment.go:2397-2421): the ids of its
//                   cache_size most populated rows, as a bulk import followed
//                   by a cache flush leaves it.
//
//   read_cache_files(paths)  the ids of every `<shard>.cache` file (packed or
//                   unpacked protobuf varints) for the device rank caches:
//                   a cold fragment's cache is these ids with the arena's row
//                   counts (fragment.go:459 openCache's CountRange per id),
//                   without materialising the fragment on the host.
#include <fcntl.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "roaring.hpp"
#include "synth.hpp"

namespace py = pybind11;

namespace {

inline uint16_t rd16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

template <class F>
void parallel_for(int64_t n, int nthreads, F&& fn) {
  const int nt = std::max<int>(1, std::min<int64_t>(nthreads, n));
  std::vector<std::thread> th;
  std::atomic<int64_t> next{0};
  std::exception_ptr err;
  std::atomic<bool> failed{false};
  for (int t = 0; t < nt; t++)
    th.emplace_back([&]() {
      for (;;) {
        const int64_t i = next.fetch_add(1);
        if (i >= n || failed.load()) break;
        try {
          fn(i);
        } catch (...) {
          if (!failed.exchange(true)) err = std::current_exception();
        }
      }
    });
  for (auto& t : th) t.join();
  if (err) std::rethrow_exception(err);
}

// Arena payload size (u16 units) of one container, as pyroaring.cpp payload_u16.
inline int64_t arena_u16(int type, int64_t n, int64_t nruns) {
  if (type == pr::CT_ARRAY) return (n + 7) & ~int64_t(7);
  if (type == pr::CT_BITMAP) return 4096;
  return 8 + ((nruns * 2 + 7) & ~int64_t(7));
}

struct Shard {
  std::string path;
  int fd = -1;
  const uint8_t* map = nullptr;  // mmap of the file, or owned.data()
  size_t len = 0;
  std::string owned;             // re-encoded snapshot of a replayed file
  uint32_t keyn = 0;
  const uint8_t* hdr = nullptr;  // keyn x (u64 key, u16 type, u16 n-1)
  const uint8_t* offs = nullptr; // keyn x u32
  int64_t containers = 0;        // with n > 0
  int64_t payload = 0;           // arena u16
  uint64_t last_key = 0;         // highest container key (row << key_shift | j)
  bool replayed = false;
  // shards wider than 2^20 columns: this entry is device sub-shard `sub` of
  // the file (its containers c with (c >> 4) & sub_mask == sub), -1 = all
  int64_t sub = -1;
  uint64_t sub_mask = 0;

  bool keep(uint64_t key) const { return sub < 0 || ((key >> 4) & sub_mask) == uint64_t(sub); }

  void release() {
    if (map && owned.empty()) munmap(const_cast<uint8_t*>(map), len);
    if (fd >= 0) ::close(fd);
    map = nullptr;
    fd = -1;
    std::string().swap(owned);
  }
  ~Shard() { release(); }
};

class FragmentLoader {
 public:
  // key_shift = log2(containers per row) = shard-width exponent - 16: 4 for
  // 2^20-column shards; 0..3 for narrower shards, whose rows then fill only
  // the first 2^key_shift of the arena's 16 container slots per row; 5..16
  // for wider shards, whose files each serve 2^(key_shift-4) device
  // sub-shards of 2^20 columns: ``subs[i]`` names the sub-shard entry i loads
  // (container c of a row goes to sub-shard c >> 4, arena slot c & 15).
  FragmentLoader(std::vector<std::string> paths, int nthreads, int key_shift = 4, std::vector<int64_t> subs = {})
      : nthreads_(std::max(1, nthreads)), ks_(key_shift), jm_((uint64_t(1) << std::min(key_shift, 4)) - 1) {
    if (key_shift < 0 || key_shift > 16) throw std::invalid_argument("FragmentLoader: key_shift must be in [0, 16]");
    if (key_shift > 4 && subs.size() != paths.size())
      throw std::invalid_argument("FragmentLoader: key_shift > 4 needs one sub-shard index per path");
    if (key_shift <= 4 && !subs.empty()) throw std::invalid_argument("FragmentLoader: subs only for key_shift > 4");
    const uint64_t mask = key_shift > 4 ? (uint64_t(1) << (key_shift - 4)) - 1 : 0;
    shards_.resize(paths.size());
    for (size_t i = 0; i < paths.size(); i++) {
      shards_[i] = std::make_unique<Shard>();
      shards_[i]->path = paths[i];
      if (key_shift > 4) {
        if (subs[i] < 0 || uint64_t(subs[i]) > mask) throw std::invalid_argument("FragmentLoader: sub-shard out of range");
        shards_[i]->sub = subs[i];
        shards_[i]->sub_mask = mask;
      }
    }
  }

  py::dict scan() {
    {
      py::gil_scoped_release nogil;
      parallel_for(int64_t(shards_.size()), nthreads_, [&](int64_t s) { scan_one(*shards_[size_t(s)]); });
    }
    int64_t C = 0, P = 0, replayed = 0, bytes = 0;
    for (auto& sp : shards_) {
      C += sp->containers;
      P += sp->payload;
      replayed += sp->replayed;
      bytes += int64_t(sp->len);
    }
    scanned_ = true;
    py::dict d;
    d["containers"] = C;
    d["payload_u16"] = P;
    d["replayed"] = replayed;
    d["file_bytes"] = bytes;
    return d;
  }

  py::array_t<uint64_t> rows() {
    need_scan();
    std::vector<uint64_t> out;
    {
      py::gil_scoped_release nogil;
      uint64_t maxrow = 0;
      bool any = false;
      for (auto& sp : shards_)
        if (sp->containers) any = true, maxrow = std::max(maxrow, sp->last_key >> ks_);
      if (any && maxrow < (uint64_t(1) << 31)) {
        // presence bits, set in parallel (fetch_or), then compacted in order
        const size_t W = size_t(maxrow / 64 + 1);
        std::vector<std::atomic<uint64_t>> bits(W);
        for (auto& b : bits) b.store(0, std::memory_order_relaxed);
        parallel_for(int64_t(shards_.size()), nthreads_, [&](int64_t s) {
          const Shard& sh = *shards_[size_t(s)];
          uint64_t prev = ~0ull;
          for (uint32_t i = 0; i < sh.keyn; i++) {
            const uint64_t key = rd64(sh.hdr + size_t(i) * 12);
            if (!sh.keep(key)) continue;
            const uint64_t r = key >> ks_;
            if (r == prev) continue;
            prev = r;
            bits[r >> 6].fetch_or(1ull << (r & 63), std::memory_order_relaxed);
          }
        });
        for (size_t w = 0; w < W; w++)
          for (uint64_t b = bits[w].load(std::memory_order_relaxed); b; b &= b - 1)
            out.push_back(uint64_t(w) * 64 + uint64_t(__builtin_ctzll(b)));
      } else if (any) {
        for (auto& sp : shards_) {
          uint64_t prev = ~0ull;
          for (uint32_t i = 0; i < sp->keyn; i++) {
            const uint64_t key = rd64(sp->hdr + size_t(i) * 12);
            if (!sp->keep(key)) continue;
            const uint64_t r = key >> ks_;
            if (r != prev) out.push_back(r), prev = r;
          }
        }
        std::sort(out.begin(), out.end());
        out.erase(std::unique(out.begin(), out.end()), out.end());
      }
    }
    rows_ = out;
    have_rows_ = true;
    py::array_t<uint64_t> a(out.size());
    if (!out.empty()) memcpy(a.mutable_data(), out.data(), out.size() * 8);
    return a;
  }

  // -> (rowptr u32[S, D+1], shard_base i64[S+1], meta i64[max(cap,1)], cap i64[S], pay_base i64[S+1])
  py::tuple fill_index(double slack, int64_t min_slack) {
    need_scan();
    if (!have_rows_) throw std::runtime_error("FragmentLoader: rows() first");
    const int64_t S = int64_t(shards_.size()), D = int64_t(rows_.size());
    std::vector<int64_t> cap(static_cast<size_t>(S), 0), sb(static_cast<size_t>(S + 1), 0), pb(static_cast<size_t>(S + 1), 0);
    for (int64_t s = 0; s < S; s++) {
      const int64_t n = shards_[size_t(s)]->containers;
      cap[size_t(s)] = slack > 0 || min_slack > 0 ? n + std::max<int64_t>(min_slack, int64_t(double(n) * slack)) : n;
      sb[size_t(s + 1)] = sb[size_t(s)] + cap[size_t(s)];
      pb[size_t(s + 1)] = pb[size_t(s)] + shards_[size_t(s)]->payload;
    }
    py::array_t<uint32_t> rowptr({(py::ssize_t)S, (py::ssize_t)(D + 1)});
    py::array_t<int64_t> meta(std::max<int64_t>(sb[size_t(S)], 1));
    py::array_t<int64_t> sbn(S + 1), capn(std::max<int64_t>(S, 0)), pbn(S + 1);
    memcpy(sbn.mutable_data(), sb.data(), size_t(S + 1) * 8);
    memcpy(pbn.mutable_data(), pb.data(), size_t(S + 1) * 8);
    if (S) memcpy(capn.mutable_data(), cap.data(), size_t(S) * 8);
    uint32_t* rp = rowptr.mutable_data();
    int64_t* mp = meta.mutable_data();
    {
      py::gil_scoped_release nogil;
      const bool identity = D > 0 && rows_[size_t(D - 1)] == uint64_t(D - 1);
      parallel_for(S, nthreads_, [&](int64_t s) {
        const Shard& sh = *shards_[size_t(s)];
        uint32_t* rps = rp + size_t(s) * size_t(D + 1);
        int64_t* ms = mp + sb[size_t(s)];
        int64_t ci = 0, pi = pb[size_t(s)];
        int64_t d = 0;
        for (uint32_t i = 0; i < sh.keyn; i++) {
          const uint8_t* h = sh.hdr + size_t(i) * 12;
          const uint64_t key = rd64(h);
          if (!sh.keep(key)) continue;
          const int type = rd16(h + 8);
          const int64_t n = int64_t(rd16(h + 10)) + 1;
          const uint64_t r = key >> ks_;
          if (identity) {
            while (d <= int64_t(r) && d < D) rps[d++] = uint32_t(ci);
          } else {
            while (d < D && rows_[size_t(d)] < r) rps[d++] = uint32_t(ci);
            if (d < D && rows_[size_t(d)] == r) rps[d++] = uint32_t(ci);
          }
          const int64_t nr = type == pr::CT_RUN ? int64_t(rd16(sh.map + rd32(sh.offs + size_t(i) * 4))) : 0;
          ms[ci++] = int64_t((key & jm_) | (uint64_t(type) << 4) | (uint64_t(n) << 6) | (uint64_t(pi / 8) << 23));
          pi += arena_u16(type, n, nr);
        }
        while (d <= D) rps[d++] = uint32_t(ci);
        for (int64_t k = ci; k < cap[size_t(s)]; k++) ms[k] = 0;
      });
      if (sb[size_t(S)] == 0) mp[0] = 0;
    }
    return py::make_tuple(rowptr, sbn, meta, capn, pbn);
  }

  // payload of shards [s0, s1) into out (u16, >= pay_base[s1]-pay_base[s0]); releases their mappings
  int64_t fill_payload(int64_t s0, int64_t s1, py::array_t<uint16_t, py::array::c_style> out) {
    need_scan();
    const int64_t S = int64_t(shards_.size());
    if (s0 < 0 || s1 > S || s0 > s1) throw std::out_of_range("fill_payload: shard range");
    std::vector<int64_t> base(size_t(s1 - s0 + 1), 0);
    for (int64_t s = s0; s < s1; s++) base[size_t(s - s0 + 1)] = base[size_t(s - s0)] + shards_[size_t(s)]->payload;
    const int64_t need = base.back();
    if (int64_t(out.size()) < need) throw std::out_of_range("fill_payload: output buffer too small");
    uint16_t* op = out.mutable_data();
    {
      py::gil_scoped_release nogil;
      parallel_for(s1 - s0, nthreads_, [&](int64_t k) {
        Shard& sh = *shards_[size_t(s0 + k)];
        uint16_t* dst = op + base[size_t(k)];
        for (uint32_t i = 0; i < sh.keyn; i++) {
          const uint8_t* h = sh.hdr + size_t(i) * 12;
          if (!sh.keep(rd64(h))) continue;
          const int type = rd16(h + 8);
          const int64_t n = int64_t(rd16(h + 10)) + 1;
          const uint8_t* src = sh.map + rd32(sh.offs + size_t(i) * 4);
          if (type == pr::CT_ARRAY) {
            memcpy(dst, src, size_t(n) * 2);
            const int64_t pad = arena_u16(type, n, 0);
            for (int64_t x = n; x < pad; x++) dst[x] = 0;
            dst += pad;
          } else if (type == pr::CT_BITMAP) {
            memcpy(dst, src, 8192);
            dst += 4096;
          } else {
            const int64_t nr = rd16(src);
            const int64_t sz = arena_u16(type, n, nr);
            memset(dst, 0, size_t(sz) * 2);
            dst[0] = uint16_t(nr);
            memcpy(dst + 8, src + 2, size_t(nr) * 4);  // (start, last) pairs, as in the file
            dst += sz;
          }
        }
        sh.release();
      });
    }
    return need;
  }

  int64_t size() const { return int64_t(shards_.size()); }

 private:
  std::vector<std::unique_ptr<Shard>> shards_;
  std::vector<uint64_t> rows_;
  bool scanned_ = false, have_rows_ = false;
  int nthreads_;
  int ks_;
  uint64_t jm_;

  void need_scan() const {
    if (!scanned_) throw std::runtime_error("FragmentLoader: scan() first");
  }

  static void fail(const Shard& sh, const std::string& what) {
    throw std::runtime_error("fragment " + sh.path + ": " + what);
  }

  void scan_one(Shard& sh) {
    if (sh.path.empty()) return;
    sh.fd = ::open(sh.path.c_str(), O_RDONLY | O_CLOEXEC);
    if (sh.fd < 0) {
      if (errno == ENOENT) return;
      fail(sh, std::string("open: ") + strerror(errno));
    }
    struct stat st;
    if (fstat(sh.fd, &st) != 0) fail(sh, std::string("stat: ") + strerror(errno));
    sh.len = size_t(st.st_size);
    if (sh.len == 0) {
      sh.release();
      return;
    }
    void* m = mmap(nullptr, sh.len, PROT_READ, MAP_SHARED, sh.fd, 0);
    if (m == MAP_FAILED) fail(sh, std::string("mmap: ") + strerror(errno));
    sh.map = static_cast<const uint8_t*>(m);
    madvise(m, sh.len, MADV_SEQUENTIAL);
    bool plain = sh.len >= size_t(pr::HEADER_BASE) && rd16(sh.map) == pr::MAGIC && sh.map[2] == pr::STORAGE_VERSION;
    if (plain && !walk(sh)) plain = false;
    if (!plain) {
      // op log after the snapshot, official format, unsorted keys: replay once
      // through the host core and re-encode (Bitmap::from_bytes validates)
      pr::Bitmap bm;
      bm.from_bytes(sh.map, sh.len);
      const uint8_t flags = bm.flags;
      std::string enc = bm.to_bytes();
      enc[3] = char(flags);
      munmap(const_cast<uint8_t*>(sh.map), sh.len);
      ::close(sh.fd);
      sh.fd = -1;
      sh.owned = std::move(enc);
      sh.map = reinterpret_cast<const uint8_t*>(sh.owned.data());
      sh.len = sh.owned.size();
      sh.replayed = true;
      if (!walk(sh)) fail(sh, "re-encoded snapshot does not parse");
    }
  }

  // Validate a plain snapshot: bounds, sorted keys, no trailing op log.
  static bool walk(Shard& sh) {
    const size_t n = sh.len;
    if (n < size_t(pr::HEADER_BASE)) return false;
    const uint32_t keyn = rd32(sh.map + 4);
    if (size_t(pr::HEADER_BASE) + size_t(keyn) * 16 > n) fail(sh, "malformed bitmap, key-cardinality overruns file");
    sh.keyn = keyn;
    sh.hdr = sh.map + pr::HEADER_BASE;
    sh.offs = sh.hdr + size_t(keyn) * 12;
    size_t end = size_t(pr::HEADER_BASE) + size_t(keyn) * 16;
    int64_t P = 0, kept = 0;
    uint64_t prev = 0, last = 0;
    for (uint32_t i = 0; i < keyn; i++) {
      const uint8_t* h = sh.hdr + size_t(i) * 12;
      const uint64_t key = rd64(h);
      const int type = rd16(h + 8);
      const int64_t cn = int64_t(rd16(h + 10)) + 1;
      const size_t off = rd32(sh.offs + size_t(i) * 4);
      if (i && key <= prev) return false;
      prev = key;
      size_t sz;
      int64_t nr = 0;
      if (type == pr::CT_ARRAY) {
        sz = size_t(cn) * 2;
      } else if (type == pr::CT_BITMAP) {
        sz = 8192;
      } else if (type == pr::CT_RUN) {
        if (off + 2 > n) fail(sh, "run container overruns data");
        nr = rd16(sh.map + off);
        sz = 2 + size_t(nr) * 4;
      } else {
        fail(sh, "unknown container type " + std::to_string(type));
        return false;
      }
      if (off + sz > n) fail(sh, "container overruns data");
      end = off + sz;
      if (!sh.keep(key)) continue;
      P += arena_u16(type, cn, nr);
      kept++;
      last = key;
    }
    if (end != n) return false;  // op log follows: replay path
    sh.containers = kept;
    sh.payload = P;
    sh.last_key = last;
    return true;
  }
};

// Encode one synthetic shard (rows 0..R-1) as a Pilosa-format file.
void write_shard_file(const std::string& path, const synth::ShardOut& o, uint8_t flags) {
  const size_t C = o.meta.size();
  const int64_t R = int64_t(o.rowptr.size()) - 1;
  std::string hdr;
  hdr.resize(size_t(pr::HEADER_BASE) + C * 16);
  uint8_t* h = reinterpret_cast<uint8_t*>(&hdr[0]);
  const uint32_t cookie = pr::MAGIC | (pr::STORAGE_VERSION << 16) | (uint32_t(flags) << 24);
  memcpy(h, &cookie, 4);
  const uint32_t cn = uint32_t(C);
  memcpy(h + 4, &cn, 4);
  uint64_t off = uint64_t(pr::HEADER_BASE) + C * 16;
  size_t i = 0;
  for (int64_t r = 0; r < R; r++) {
    for (uint32_t c = o.rowptr[size_t(r)]; c < o.rowptr[size_t(r + 1)]; c++, i++) {
      const uint64_t m = uint64_t(o.meta[c]);
      const uint64_t key = uint64_t(r) * 16 + (m & 15);
      const uint16_t type = uint16_t((m >> 4) & 3);
      const uint32_t n = uint32_t((m >> 6) & 0x1ffff);
      const uint16_t nm1 = uint16_t(n - 1);
      uint8_t* e = h + pr::HEADER_BASE + i * 12;
      memcpy(e, &key, 8);
      memcpy(e + 8, &type, 2);
      memcpy(e + 10, &nm1, 2);
      if (off > 0xffffffffull) throw std::runtime_error("fragment file exceeds 4 GiB offsets");
      const uint32_t o32 = uint32_t(off);
      memcpy(h + pr::HEADER_BASE + C * 12 + i * 4, &o32, 4);
      off += type == pr::CT_ARRAY ? uint64_t(n) * 2 : 8192;
    }
  }
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("open " + tmp + ": " + strerror(errno));
  std::vector<char> buf(1 << 22);
  setvbuf(f, buf.data(), _IOFBF, buf.size());
  bool ok = fwrite(hdr.data(), 1, hdr.size(), f) == hdr.size();
  for (size_t c = 0; ok && c < C; c++) {
    const uint64_t m = uint64_t(o.meta[c]);
    const int type = int((m >> 4) & 3);
    const size_t n = size_t((m >> 6) & 0x1ffff);
    const uint16_t* src = o.payload.data() + (m >> 23) * 8;
    const size_t bytes = type == pr::CT_ARRAY ? n * 2 : 8192;
    ok = fwrite(src, 1, bytes, f) == bytes;
  }
  ok = (fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error("write " + tmp + " failed");
  if (rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename " + tmp + ": " + strerror(errno));
}

inline void put_uvarint(std::string& out, uint64_t v) {
  while (v >= 0x80) {
    out.push_back(char(uint8_t(v) | 0x80));
    v >>= 7;
  }
  out.push_back(char(v));
}

// <shard>.cache of a synthetic shard: protobuf Cache{repeated uint64 IDs = 1}
// (packed) with the ids of the `cache_size` rows of largest count (count desc,
// id asc on ties), in ascending id order (rankCache.IDs, cache.go).
void write_cache_file(const std::string& path, const synth::ShardOut& o, int64_t cache_size) {
  const int64_t R = int64_t(o.rowptr.size()) - 1;
  std::vector<std::pair<int64_t, int64_t>> rc;  // (-count, row)
  for (int64_t r = 0; r < R; r++) {
    int64_t n = 0;
    for (uint32_t c = o.rowptr[size_t(r)]; c < o.rowptr[size_t(r + 1)]; c++) n += int64_t((uint64_t(o.meta[c]) >> 6) & 0x1ffff);
    if (n > 0) rc.emplace_back(-n, r);
  }
  if (int64_t(rc.size()) > cache_size) {
    std::nth_element(rc.begin(), rc.begin() + cache_size, rc.end());
    rc.resize(size_t(cache_size));
  }
  std::vector<uint64_t> ids;
  ids.reserve(rc.size());
  for (auto& x : rc) ids.push_back(uint64_t(x.second));
  std::sort(ids.begin(), ids.end());
  std::string body;
  for (uint64_t id : ids) put_uvarint(body, id);
  std::string msg;
  if (!body.empty()) {
    msg.push_back(char(0x0A));  // field 1, wire type 2 (packed)
    put_uvarint(msg, body.size());
    msg += body;
  }
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("open " + tmp + ": " + strerror(errno));
  bool ok = msg.empty() || fwrite(msg.data(), 1, msg.size(), f) == msg.size();
  ok = (fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error("write " + tmp + " failed");
  if (rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename " + tmp + ": " + strerror(errno));
}

// Ids of a protobuf Cache message (field 1: packed or one varint per entry;
// unknown fields skipped).  false on a malformed message.
bool parse_cache_ids(const uint8_t* p, size_t n, std::vector<uint64_t>& out) {
  size_t i = 0;
  auto uv = [&](uint64_t* v) -> bool {
    uint64_t x = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (i >= n) return false;
      const uint8_t b = p[i++];
      x |= uint64_t(b & 0x7f) << sh;
      if (!(b & 0x80)) {
        *v = x;
        return true;
      }
    }
    return false;
  };
  while (i < n) {
    uint64_t tag;
    if (!uv(&tag)) return false;
    const uint64_t field = tag >> 3, wt = tag & 7;
    if (wt == 0) {
      uint64_t v;
      if (!uv(&v)) return false;
      if (field == 1) out.push_back(v);
    } else if (wt == 2) {
      uint64_t len;
      if (!uv(&len) || len > n - i) return false;
      const size_t end = i + size_t(len);
      if (field == 1) {
        while (i < end) {
          uint64_t v;
          if (!uv(&v) || i > end) return false;
          out.push_back(v);
        }
      }
      i = end;
    } else if (wt == 1) {
      if (n - i < 8) return false;
      i += 8;
    } else if (wt == 5) {
      if (n - i < 4) return false;
      i += 4;
    } else {
      return false;
    }
  }
  return true;
}

// -> (offsets int64[S+1], ids uint64[N], ok bool[S]); a missing file is an
// empty cache, a corrupt one ok=False (the caller rebuilds, as openCache does).
py::tuple read_cache_files(const std::vector<std::string>& paths, int nthreads) {
  const int64_t S = int64_t(paths.size());
  std::vector<std::vector<uint64_t>> per(static_cast<size_t>(S));
  std::vector<char> good(static_cast<size_t>(S), 1);
  {
    py::gil_scoped_release nogil;
    parallel_for(S, nthreads, [&](int64_t s) {
      const std::string& path = paths[size_t(s)];
      if (path.empty()) return;
      FILE* f = fopen(path.c_str(), "rb");
      if (!f) return;  // no cache file: empty rank cache
      std::string data;
      char buf[1 << 16];
      size_t r;
      while ((r = fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, r);
      fclose(f);
      if (!parse_cache_ids(reinterpret_cast<const uint8_t*>(data.data()), data.size(), per[size_t(s)])) {
        per[size_t(s)].clear();
        good[size_t(s)] = 0;
      }
    });
  }
  py::array_t<int64_t> offs(S + 1);
  int64_t* op = offs.mutable_data();
  op[0] = 0;
  for (int64_t s = 0; s < S; s++) op[s + 1] = op[s] + int64_t(per[size_t(s)].size());
  py::array_t<uint64_t> ids(std::max<int64_t>(op[S], 0));
  py::array_t<bool> ok(S);
  uint64_t* ip = ids.mutable_data();
  for (int64_t s = 0; s < S; s++) {
    if (!per[size_t(s)].empty()) memcpy(ip + op[s], per[size_t(s)].data(), per[size_t(s)].size() * 8);
    ok.mutable_data()[s] = good[size_t(s)] != 0;
  }
  return py::make_tuple(offs, ids, ok);
}

py::dict write_zipf_fragments(const std::string& dir, int64_t shard_lo, int64_t shard_hi, int64_t total_cols,
                              int64_t nrows, double bits_per_col, double zs, double zv, uint64_t seed, int nthreads,
                              uint8_t flags, int64_t cache_size) {
  const int64_t S = std::max<int64_t>(0, shard_hi - shard_lo);
  std::atomic<int64_t> bytes{0}, containers{0};
  {
    py::gil_scoped_release nogil;
    const std::vector<double> dens = synth::zipf_densities(nrows, bits_per_col, zs, zv);
    parallel_for(S, nthreads, [&](int64_t k) {
      synth::ShardOut o;
      const int64_t shard = shard_lo + k;
      synth::gen_zipf_shard(o, shard, total_cols, dens, seed);
      if (o.meta.empty()) return;
      write_shard_file(dir + "/" + std::to_string(shard), o, flags);
      if (cache_size > 0) write_cache_file(dir + "/" + std::to_string(shard) + ".cache", o, cache_size);
      containers += int64_t(o.meta.size());
      int64_t b = int64_t(pr::HEADER_BASE) + int64_t(o.meta.size()) * 16;
      for (int64_t m : o.meta) {
        const uint64_t u = uint64_t(m);
        b += ((u >> 4) & 3) == pr::CT_ARRAY ? int64_t((u >> 6) & 0x1ffff) * 2 : 8192;
      }
      bytes += b;
    });
  }
  py::dict d;
  d["shards"] = S;
  d["containers"] = containers.load();
  d["bytes"] = bytes.load();
  return d;
}

// The synthetic BSI int field of BASELINE config 4 as Pilosa-format fragment
// files of its bsig_<field> view (one per shard).
py::dict write_bsi_fragments(const std::string& dir, int64_t shard_lo, int64_t shard_hi, int64_t total_cols, int depth,
                             double fill, int64_t vmin, int64_t vmax, uint64_t seed, int nthreads, uint8_t flags) {
  if (depth < 1 || depth > 62) throw std::invalid_argument("depth must be in 1..62");
  const int64_t S = std::max<int64_t>(0, shard_hi - shard_lo);
  std::atomic<int64_t> containers{0};
  {
    py::gil_scoped_release nogil;
    parallel_for(S, nthreads, [&](int64_t k) {
      synth::ShardOut o;
      const int64_t shard = shard_lo + k;
      synth::gen_bsi_shard(o, shard, total_cols, depth, fill, vmin, vmax, seed);
      if (o.meta.empty()) return;
      write_shard_file(dir + "/" + std::to_string(shard), o, flags);
      containers += int64_t(o.meta.size());
    });
  }
  py::dict d;
  d["shards"] = S;
  d["containers"] = containers.load();
  return d;
}

}  // namespace

void register_arena_io(py::module_& m) {
  py::class_<FragmentLoader>(m, "FragmentLoader")
      .def(py::init<std::vector<std::string>, int, int, std::vector<int64_t>>(), py::arg("paths"),
           py::arg("nthreads") = 16, py::arg("key_shift") = 4, py::arg("subs") = std::vector<int64_t>{})
      .def("scan", &FragmentLoader::scan)
      .def("rows", &FragmentLoader::rows)
      .def("fill_index", &FragmentLoader::fill_index, py::arg("slack") = 0.0, py::arg("min_slack") = 0)
      .def("fill_payload", &FragmentLoader::fill_payload, py::arg("s0"), py::arg("s1"), py::arg("out"))
      .def("__len__", &FragmentLoader::size);
  m.def("write_zipf_fragments", &write_zipf_fragments, py::arg("dir"), py::arg("shard_lo"), py::arg("shard_hi"),
        py::arg("total_cols"), py::arg("nrows"), py::arg("bits_per_col") = 8.0, py::arg("zipf_s") = 1.6,
        py::arg("zipf_v") = 50.0, py::arg("seed") = 1, py::arg("nthreads") = 16, py::arg("flags") = 1,
        py::arg("cache_size") = 50000,
        "Write the synthetic Zipf set field as one Pilosa-format fragment file per shard (<dir>/<shard>) "
        "and its rank-cache file (<dir>/<shard>.cache, cache_size most populated rows; 0 = none)");
  m.def("write_bsi_fragments", &write_bsi_fragments, py::arg("dir"), py::arg("shard_lo"), py::arg("shard_hi"),
        py::arg("total_cols"), py::arg("depth"), py::arg("fill"), py::arg("vmin"), py::arg("vmax"), py::arg("seed") = 1,
        py::arg("nthreads") = 16, py::arg("flags") = 1,
        "Write a synthetic BSI int field (exists, sign, magnitude planes) as Pilosa-format fragment files");
  m.def("read_cache_files", &read_cache_files, py::arg("paths"), py::arg("nthreads") = 16,
        "Ids of <shard>.cache rank-cache files -> (offsets int64[S+1], ids uint64[N], ok bool[S])");
}
