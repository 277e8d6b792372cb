// Host roaring core for the MI355X bitmap index.
//
// 64-bit roaring bitmap: key = value >> 16 selects a container holding the low
// 16 bits.  Three container encodings (array / bitmap / run) as in the
// reference (roaring/roaring.go:46-51, ArrayMaxSize=4096 :1984, runMaxSize=2048
// :1987).  This is the authoritative host copy of every fragment and the CPU
// oracle the HIP kernels are tested against.  It also owns the bit-exact
// Pilosa file format (roaring.go:1052-1122 writer, :1562-1653 reader), the
// official-roaring reader (:5081-5139) and the op-log WAL codec
// (:4416-4559, fnv32a checksums).
//
// Design notes (ours, not the reference's):
//  * containers live in a std::map keyed by the 48-bit high key; payloads are
//    plain vectors (no mmap aliasing / frozen copy-on-write: the GPU arena is
//    the read-mostly replica, the host copy is mutable);
//  * pairwise ops have merge fast paths for array/array and word-parallel
//    paths for everything else; results are canonicalised (array if n<=4096,
//    else bitmap); runs only appear through optimize() or file loads;
//  * export_containers()/build_arena() flatten a set of shard bitmaps into the
//    device arena layout consumed by pilosa_amd/kernels/bitmap_kernels.hip.
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <vector>
#include <utility>
#include <stdexcept>

namespace pr {

constexpr int ARRAY_MAX = 4096;
constexpr int RUN_MAX = 2048;
constexpr int BITMAP_N = 1024;
constexpr uint32_t MAGIC = 12348;
constexpr uint32_t STORAGE_VERSION = 0;
constexpr int HEADER_BASE = 8;
constexpr uint32_t OFFICIAL_NORUN = 12346;
constexpr uint32_t OFFICIAL_RUN = 12347;

enum : uint8_t { CT_NIL = 0, CT_ARRAY = 1, CT_BITMAP = 2, CT_RUN = 3 };

// Container event counters: the reference's ``roaringstats`` build tag
// (roaring/roaring_stats.go, statsHit call sites across roaring.go).  Built in
// with -DPILOSA_ROARING_STATS (native/build.py ``PILOSA_ROARING_STATS=1``),
// read and reset through _roaring.roaring_stats(); otherwise a no-op.
enum StatId : int {
  ST_NEW_CONTAINER,
  ST_ARRAY_ADD_APPEND,
  ST_ARRAY_ADD_INSERT,
  ST_ARRAY_ADD_TO_BITMAP,
  ST_BITMAP_REMOVE_TO_ARRAY,
  ST_RUN_ADD_CONVERT,
  ST_RUN_REMOVE_CONVERT,
  ST_OPT_TO_RUN,
  ST_OPT_TO_ARRAY,
  ST_OPT_TO_BITMAP,
  ST_OPT_UNCHANGED,
  ST_UNION_IN_PLACE,
  ST_CONTAINER_REMOVED,
  ST_COUNT
};
extern const char* const STAT_NAMES[ST_COUNT];
#ifdef PILOSA_ROARING_STATS
void stats_hit(StatId s);
constexpr bool STATS_ENABLED = true;
#else
inline void stats_hit(StatId) {}
constexpr bool STATS_ENABLED = false;
#endif
int64_t stats_get(StatId s);
void stats_reset();

struct Iv {
  uint16_t start, last;
};

struct Container {
  uint8_t type = CT_ARRAY;
  int32_t n = 0;
  std::vector<uint16_t> a;   // sorted values (array)
  std::vector<uint64_t> b;   // 1024 words (bitmap)
  std::vector<Iv> r;         // sorted disjoint runs (run)

  bool empty() const { return n == 0; }
  bool contains(uint16_t v) const;
  bool add(uint16_t v);
  bool remove(uint16_t v);
  void to_words(uint64_t* w) const;          // OR-materialise into w (w must be zeroed)
  void set_words(const uint64_t* w);         // canonical array/bitmap from words
  int count_runs() const;
  int32_t count_range(int start, int end) const;  // [start,end) in 0..65536
  int max() const;
  int min() const;
  int next_from(int v) const;               // smallest value >= v, or -1
  void optimize();
  void to_bitmap();
  void to_array();
  void to_run();
  size_t encoded_size() const;               // bytes in pilosa file
  std::string check() const;
  void recount();
};

Container c_intersect(const Container& x, const Container& y);
Container c_union(const Container& x, const Container& y);
Container c_difference(const Container& x, const Container& y);
Container c_xor(const Container& x, const Container& y);
int64_t c_intersection_count(const Container& x, const Container& y);

// op log
enum OpType : uint8_t {
  OP_ADD = 0, OP_REMOVE = 1, OP_ADD_BATCH = 2, OP_REMOVE_BATCH = 3,
  OP_ADD_ROARING = 4, OP_REMOVE_ROARING = 5
};

uint32_t fnv32a(const uint8_t* p, size_t n, uint32_t h = 2166136261u);
std::string encode_op(uint8_t typ, uint64_t value, const uint64_t* values, size_t nvalues,
                      const std::string& roaring, uint32_t opn);

class Bitmap {
 public:
  std::map<uint64_t, Container> cs;
  uint8_t flags = 0;
  int64_t ops = 0;   // number of ops replayed/logged
  int64_t opn = 0;   // number of bits touched by ops

  Bitmap() = default;

  bool add(uint64_t v);
  bool remove(uint64_t v);
  bool contains(uint64_t v) const;
  int64_t add_many(const uint64_t* v, size_t n);
  int64_t remove_many(const uint64_t* v, size_t n);
  int64_t count() const;
  int64_t count_range(uint64_t start, uint64_t end) const;
  bool any() const;
  uint64_t max() const;
  uint64_t min() const;
  std::vector<uint64_t> slice() const;
  std::vector<uint64_t> slice_range(uint64_t start, uint64_t end) const;
  Bitmap offset_range(uint64_t offset, uint64_t start, uint64_t end) const;
  // device sub-shard `sub` of a shard wider than 2^20 columns (key = row <<
  // key_shift | c): containers with c >> 4 == sub, re-keyed row * 16 + (c & 15)
  Bitmap sub_shard(int key_shift, uint64_t sub) const;
  Bitmap intersect(const Bitmap& o) const;
  Bitmap unite(const Bitmap& o) const;
  Bitmap difference(const Bitmap& o) const;
  Bitmap xor_(const Bitmap& o) const;
  int64_t intersection_count(const Bitmap& o) const;
  // zero-copy row counts: key windows [start, start+len) (65536-aligned)
  int64_t range_intersection_count(uint64_t a_start, const Bitmap& o, uint64_t b_start, uint64_t len) const;
  static int64_t range_union_count(const std::vector<std::pair<const Bitmap*, uint64_t>>& srcs, uint64_t len);
  void union_in_place(const std::vector<const Bitmap*>& others);
  Bitmap shift(int n) const;
  Bitmap flip(uint64_t start, uint64_t end) const;
  void optimize();
  void remove_empty();
  bool equals(const Bitmap& o) const;
  std::string check() const;

  // serialization
  std::string to_bytes();                           // pilosa format (optimizes)
  void from_bytes(const uint8_t* data, size_t n);   // pilosa or official; replays op log
  // merge a serialized roaring blob without keeping it; returns changed bits and
  // per-row deltas (row = key / containers_per_row)
  int64_t import_roaring(const uint8_t* data, size_t n, bool clear, uint64_t containers_per_row,
                         std::map<uint64_t, int64_t>* rowdelta);
  // apply a Pilosa op log (13-byte ops + batches / roaring blobs) in order
  void replay_ops(const uint8_t* data, size_t n);

 private:
  void parse_pilosa(const uint8_t* data, size_t n, size_t* ops_offset);
  void parse_official(const uint8_t* data, size_t n);
};

// Read-mostly view of a Pilosa fragment file through mmap (the reference's
// frozen, mapped containers: roaring/container_stash.go:262-346,
// roaring.go:1616-1622).  Lookups binary-search the mapped header and read
// container payloads in place; the first write to a container copies it into
// an owned overlay (copy-on-write), so a cold fragment that takes a few
// writes holds only the containers those writes touched.  The file's own op
// log is replayed into that overlay at open.  Only the operations a cold
// fragment needs are offered (membership, counts, row extraction, single-bit
// writes); anything else loads the whole file into a Bitmap.
class MappedBitmap {
 public:
  explicit MappedBitmap(const std::string& path);
  ~MappedBitmap();
  MappedBitmap(const MappedBitmap&) = delete;
  MappedBitmap& operator=(const MappedBitmap&) = delete;

  bool contains(uint64_t v) const;
  bool add(uint64_t v);
  bool remove(uint64_t v);
  int64_t count() const;
  int64_t count_range(uint64_t start, uint64_t end) const;
  bool any() const;
  uint64_t max() const;
  Bitmap offset_range(uint64_t offset, uint64_t start, uint64_t end) const;
  Bitmap sub_shard(int key_shift, uint64_t sub) const;
  std::vector<uint64_t> rows_with_column(uint64_t col, uint64_t cpr) const;
  int64_t add_many(const uint64_t* v, size_t n);     // v sorted ascending
  int64_t remove_many(const uint64_t* v, size_t n);  // v sorted ascending
  int64_t import_roaring(const uint8_t* data, size_t n, bool clear, uint64_t cpr,
                         std::map<uint64_t, int64_t>* rowdelta);
  // Pilosa-format snapshot of the current state streamed to ``path``:
  // untouched containers are copied from the map byte for byte, overlay
  // containers are optimised and encoded (Bitmap::to_bytes layout).  Returns
  // the bytes written.
  size_t write_snapshot(const std::string& path);
  size_t mapped_containers() const { return keyn_; }
  size_t overlay_containers() const { return touched_.size(); }
  size_t mapped_bytes() const { return len_; }

  uint8_t flags = 0;
  int64_t ops = 0, opn = 0;

 private:
  int fd_ = -1;
  const uint8_t* base_ = nullptr;
  size_t len_ = 0;
  uint32_t keyn_ = 0;
  const uint8_t* hdr_ = nullptr;   // keyn x (key u64, type u16, n-1 u16)
  const uint8_t* offs_ = nullptr;  // keyn x u32
  Bitmap over_;                    // owned copies of touched containers
  std::map<uint64_t, bool> touched_;  // keys whose authoritative copy is in over_ (absent there = empty)

  uint64_t key_at(size_t i) const;
  size_t lower(uint64_t key) const;                 // first header index with key >= key
  int64_t find(uint64_t key) const;                 // header index of key, or -1
  Container load(size_t i) const;                   // copy of mapped container i
  int32_t mapped_n(size_t i) const;
  bool span(size_t i, size_t* off, size_t* sz) const;  // payload extent of container i, false if corrupt
  const uint8_t* payload(size_t i) const;              // checked payload pointer (throws if corrupt)
  bool mapped_contains(size_t i, uint16_t low) const;
  Container& cow(uint64_t key);
};

Container& get_or_create(Bitmap& b, uint64_t key);

// Value iterator with Seek (reference roaring.go:1767-1982 Iterator).  Holds
// the container map position between calls, so a forward walk costs one map
// step per container; Seek re-positions with one lower_bound.  The bitmap must
// not be mutated while an iterator is live (same contract as the reference).
class Iterator {
 public:
  explicit Iterator(const Bitmap* b) : bm_(b) { seek(0); }
  void seek(uint64_t v);
  // next value, or eof=true when exhausted
  bool next(uint64_t* v);
 private:
  const Bitmap* bm_;
  std::map<uint64_t, Container>::const_iterator it_;
  int low_ = 0;  // next low-16 candidate inside *it_ (65536 = past the end)
};

}  // namespace pr
