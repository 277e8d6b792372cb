// Single-producer / multi-consumer command ring in POSIX shared memory: the
// command channel of a node's GPU mesh (parallel/mesh.py).
//
// Every request on a multi-GPU node starts with rank 0 sending its command
// (op + a few hundred bytes) to every other rank.  Over a gloo broadcast that
// is a TCP round trip per request, paid before any GPU work starts, and the
// receiving ranks block inside a collective whose timeout also fires when the
// node is merely idle.  All ranks of a mesh live on one host, so the command
// travels through shared memory instead: the producer writes the slot and
// bumps a sequence word; each consumer spins briefly on it, then sleeps on a
// futex the producer wakes.  Consumers wait indefinitely while the producer
// process is alive (an idle node is not a failure) and raise once it is gone.
//
// Layout: Header | reader cursors | slots[nslots] of {u64 seq, i64 op, u64 len,
// u8 data[slot_bytes]}.  The producer may reuse slot (s % nslots) once every
// reader's cursor is past s - nslots.  Reference analog: the coordinator's
// per-query fan-out of QueryRequests (executor.go:2458-2555), which a node's
// ranks replace with this ring plus RCCL collectives.
#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <pybind11/pybind11.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace {

constexpr uint64_t MAGIC = 0x50494c4f53524e47ull;  // "PILOSRNG"
constexpr int MAX_READERS = 64;

struct alignas(64) Cursor {
  std::atomic<uint64_t> seq;   // next sequence number this reader will read
  std::atomic<int32_t> pid;
  char pad[64 - sizeof(std::atomic<uint64_t>) - sizeof(std::atomic<int32_t>)];
};

struct alignas(64) Header {
  uint64_t magic;
  uint32_t nslots, nreaders;
  uint64_t slot_bytes;
  std::atomic<int32_t> producer_pid;
  std::atomic<uint32_t> closed;
  char pad0[64 - 32];
  std::atomic<uint64_t> head;          // sequence number of the next message to write
  std::atomic<uint32_t> data_futex;    // bumped on every publish (readers sleep on it)
  std::atomic<uint32_t> sleepers;      // readers asleep on data_futex
  std::atomic<uint32_t> space_futex;   // bumped on every read (a blocked producer sleeps on it)
  char pad1[64 - 20];
  uint64_t board_bytes;                // per-rank result bytes of a board entry (0: no board)
  uint32_t board_ranks;                // ranks posting results (readers + the producer)
  std::atomic<uint32_t> board_futex;   // bumped on every post (a collecting front end sleeps on it)
  std::atomic<uint32_t> board_sleepers;
  char pad2[64 - 20];
  Cursor cur[MAX_READERS];
};

// One rank's result for command `seq` on the results board: the one-shot
// gather of small partials (a few bytes to a few KB: Sum/Min/Max/Rows/...)
// that needs no collective and no device copy.  len < 0: it did not fit
// (-len bytes would have).
struct BoardEntry {
  std::atomic<uint64_t> seq;   // command sequence number + 1 once posted
  int64_t len;
};

struct Slot {
  std::atomic<uint64_t> seq;   // sequence number + 1 once written
  int64_t op;
  uint64_t len;
};

long futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const struct timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

bool alive(int32_t pid) { return pid <= 0 || kill(pid, 0) == 0 || errno == EPERM; }

class Ring {
 public:
  Ring(const std::string& name, bool create, uint32_t nslots, uint64_t slot_bytes, uint32_t nreaders,
       uint64_t board_bytes)
      : name_(name), owner_(create) {
    if (create) {
      if (nslots < 2 || nreaders > MAX_READERS || slot_bytes < 64) throw std::invalid_argument("ring geometry");
      size_ = sizeof(Header) + size_t(nslots) * slot_stride(slot_bytes) +
              size_t(nslots) * (nreaders + 1) * board_stride(board_bytes);
      shm_unlink(name.c_str());
      int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
      if (ftruncate(fd, off_t(size_)) != 0) {
        close(fd);
        throw std::runtime_error("ftruncate: " + std::string(std::strerror(errno)));
      }
      map(fd);
      std::memset(static_cast<void*>(h_), 0, sizeof(Header));
      h_->nslots = nslots;
      h_->nreaders = nreaders;
      h_->slot_bytes = slot_bytes;
      h_->board_bytes = board_bytes;
      h_->board_ranks = nreaders + 1;
      h_->producer_pid.store(int32_t(getpid()));
      for (uint32_t i = 0; i < nslots; i++) slot(i)->seq.store(0);
      if (board_bytes)
        for (uint32_t i = 0; i < nslots; i++)
          for (uint32_t r = 0; r <= nreaders; r++) entry(i, r)->seq.store(0);
      std::atomic_thread_fence(std::memory_order_seq_cst);
      h_->magic = MAGIC;
    } else {
      int fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
      struct stat st;
      if (fstat(fd, &st) != 0 || size_t(st.st_size) < sizeof(Header)) {
        close(fd);
        throw std::runtime_error("ring " + name + " too small");
      }
      size_ = size_t(st.st_size);
      map(fd);
      if (h_->magic != MAGIC) throw std::runtime_error("ring " + name + " not initialised");
      if (size_ < sizeof(Header) + size_t(h_->nslots) * slot_stride(h_->slot_bytes) +
                      size_t(h_->nslots) * h_->board_ranks * board_stride(h_->board_bytes))
        throw std::runtime_error("ring " + name + " truncated");
    }
  }
  ~Ring() {
    if (base_ != nullptr) munmap(base_, size_);
    if (owner_) shm_unlink(name_.c_str());
  }

  uint64_t slot_bytes() const { return h_->slot_bytes; }
  uint64_t board_bytes() const { return h_->board_bytes; }
  uint32_t nreaders() const { return h_->nreaders; }
  uint64_t head() const { return h_->head.load(); }

  // reader `r` attaches: its cursor starts at the current head
  void attach(uint32_t r) {
    check_reader(r);
    h_->cur[r].seq.store(h_->head.load());
    h_->cur[r].pid.store(int32_t(getpid()));
  }

  // producer: one message; waits (GIL released) while the slowest reader is a
  // whole ring behind, up to timeout_s (then TimeoutError)
  uint64_t publish(int64_t op, py::bytes payload, double timeout_s) {
    std::string_view data = payload;
    if (data.size() > h_->slot_bytes) throw std::length_error("payload larger than a ring slot");
    const uint64_t s = h_->head.load(std::memory_order_relaxed);
    int fail = 0, dead = -1;
    {
      py::gil_scoped_release nogil;
      const auto t0 = std::chrono::steady_clock::now();
      int spins = 0;
      for (;;) {
        const uint64_t low = min_cursor();
        if (s - low < h_->nslots) break;
        const uint32_t f = h_->space_futex.load();
        if (s - min_cursor() < h_->nslots) break;
        if (++spins < 2000) {
          std::this_thread::yield();
          continue;
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > timeout_s) {
          fail = 1;
          break;
        }
        for (uint32_t r = 0; r < h_->nreaders && dead < 0; r++)
          if (!alive(h_->cur[r].pid.load())) dead = int(r);
        if (dead >= 0) {
          fail = 2;
          break;
        }
        struct timespec ts = {0, 10 * 1000 * 1000};
        futex(&h_->space_futex, FUTEX_WAIT, f, &ts);
      }
    }
    if (fail == 1) throw py::value_error("command ring full: a reader is more than a ring behind");
    if (fail == 2) throw std::runtime_error("ring reader " + std::to_string(dead) + " is gone");
    Slot* sl = slot(uint32_t(s % h_->nslots));
    sl->op = op;
    sl->len = data.size();
    std::memcpy(reinterpret_cast<char*>(sl) + sizeof(Slot), data.data(), data.size());
    sl->seq.store(s + 1, std::memory_order_release);
    h_->head.store(s + 1, std::memory_order_release);
    h_->data_futex.fetch_add(1, std::memory_order_acq_rel);
    if (h_->sleepers.load() != 0) futex(&h_->data_futex, FUTEX_WAKE, INT32_MAX, nullptr);
    return s;
  }

  // reader `r`: the next message (op, payload); waits without limit while the
  // producer lives (spin ~spin_us, then futex sleeps), raises once it is gone
  // or the ring is closed
  py::tuple read(uint32_t r, double spin_us) {
    check_reader(r);
    const uint64_t s = h_->cur[r].seq.load(std::memory_order_relaxed);
    Slot* sl = slot(uint32_t(s % h_->nslots));
    int why = 0;
    {
      py::gil_scoped_release nogil;
      const auto t0 = std::chrono::steady_clock::now();
      auto last_check = t0;
      for (;;) {
        if (sl->seq.load(std::memory_order_acquire) == s + 1) break;
        if (h_->closed.load()) {
          why = 1;
          break;
        }
        const auto now = std::chrono::steady_clock::now();
        if (std::chrono::duration<double, std::micro>(now - t0).count() < spin_us) {
#if defined(__x86_64__)
          __builtin_ia32_pause();
#endif
          continue;
        }
        if (std::chrono::duration<double>(now - last_check).count() > 1.0) {
          last_check = now;
          if (!alive(h_->producer_pid.load())) {
            why = 2;
            break;
          }
        }
        const uint32_t f = h_->data_futex.load();
        h_->sleepers.fetch_add(1);
        if (sl->seq.load(std::memory_order_acquire) != s + 1) {
          struct timespec ts = {0, 200 * 1000 * 1000};
          futex(&h_->data_futex, FUTEX_WAIT, f, &ts);
        }
        h_->sleepers.fetch_sub(1);
      }
    }
    if (why == 1) throw std::runtime_error("command ring closed");
    if (why == 2) throw std::runtime_error("command ring producer is gone");
    const int64_t op = sl->op;
    py::bytes data(reinterpret_cast<const char*>(sl) + sizeof(Slot), sl->len);
    h_->cur[r].seq.store(s + 1, std::memory_order_release);
    h_->space_futex.fetch_add(1, std::memory_order_acq_rel);
    futex(&h_->space_futex, FUTEX_WAKE, 1, nullptr);
    return py::make_tuple(op, data, s);
  }

  // any rank: its result of command `seq` (rank 0 = the producer, reader r =
  // rank r + 1); a payload larger than board_bytes posts its size only
  void post(uint32_t rank, uint64_t seq, py::bytes payload) {
    if (!h_->board_bytes) throw std::runtime_error("ring has no results board");
    if (rank >= h_->board_ranks) throw std::out_of_range("board rank");
    std::string_view data = payload;
    BoardEntry* e = entry(uint32_t(seq % h_->nslots), rank);
    if (data.size() > h_->board_bytes) {
      e->len = -int64_t(data.size());
    } else {
      e->len = int64_t(data.size());
      std::memcpy(reinterpret_cast<char*>(e) + sizeof(BoardEntry), data.data(), data.size());
    }
    e->seq.store(seq + 1, std::memory_order_release);
    h_->board_futex.fetch_add(1, std::memory_order_acq_rel);
    if (h_->board_sleepers.load() != 0) futex(&h_->board_futex, FUTEX_WAKE, INT32_MAX, nullptr);
  }

  // producer: every rank's posted result of command `seq` (bytes, or the int
  // -size of one that did not fit), waiting up to timeout_s; raises when a
  // reader process is gone, the ring is closed or the wait times out
  py::list collect(uint64_t seq, double timeout_s, double spin_us) {
    if (!h_->board_bytes) throw std::runtime_error("ring has no results board");
    const uint32_t R = h_->board_ranks;
    const uint32_t k = uint32_t(seq % h_->nslots);
    int why = 0, dead = -1;
    {
      py::gil_scoped_release nogil;
      const auto t0 = std::chrono::steady_clock::now();
      auto last_check = t0;
      for (;;) {
        bool all = true;
        for (uint32_t r = 0; r < R && all; r++) {
          const uint64_t v = entry(k, r)->seq.load(std::memory_order_acquire);
          if (v > seq + 1) {   // overwritten by a later command: this result is lost
            why = 3;
            break;
          }
          all = v == seq + 1;
        }
        if (why || all) break;
        const auto now = std::chrono::steady_clock::now();
        const double el = std::chrono::duration<double>(now - t0).count();
        if (el * 1e6 < spin_us) {
#if defined(__x86_64__)
          __builtin_ia32_pause();
#endif
          continue;
        }
        if (el > timeout_s) {
          why = 1;
          break;
        }
        if (std::chrono::duration<double>(now - last_check).count() > 1.0) {
          last_check = now;
          for (uint32_t r = 0; r < h_->nreaders && dead < 0; r++)
            if (!alive(h_->cur[r].pid.load())) dead = int(r);
          if (dead >= 0) {
            why = 2;
            break;
          }
        }
        const uint32_t f = h_->board_futex.load();
        h_->board_sleepers.fetch_add(1);
        bool ready = true;
        for (uint32_t r = 0; r < R && ready; r++) ready = entry(k, r)->seq.load(std::memory_order_acquire) == seq + 1;
        if (!ready) {
          struct timespec ts = {0, 50 * 1000 * 1000};
          futex(&h_->board_futex, FUTEX_WAIT, f, &ts);
        }
        h_->board_sleepers.fetch_sub(1);
      }
    }
    if (why == 1) throw std::runtime_error("results board: timed out waiting for the ranks");
    if (why == 2) throw std::runtime_error("results board: rank " + std::to_string(dead + 1) + " is gone");
    if (why == 3) throw std::runtime_error("results board: entry overwritten");
    py::list out;
    for (uint32_t r = 0; r < R; r++) {
      BoardEntry* e = entry(k, r);
      if (e->len < 0)
        out.append(py::int_(e->len));
      else
        out.append(py::bytes(reinterpret_cast<const char*>(e) + sizeof(BoardEntry), size_t(e->len)));
    }
    return out;
  }

  // producer: readers blocked in read() raise (orderly shutdown / failover)
  void close_ring() {
    h_->closed.store(1);
    h_->data_futex.fetch_add(1);
    futex(&h_->data_futex, FUTEX_WAKE, INT32_MAX, nullptr);
  }

 private:
  static size_t slot_stride(uint64_t slot_bytes) { return (sizeof(Slot) + size_t(slot_bytes) + 63) & ~size_t(63); }
  void map(int fd) {
    void* p = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap: " + std::string(std::strerror(errno)));
    base_ = static_cast<char*>(p);
    h_ = reinterpret_cast<Header*>(base_);
  }
  static size_t board_stride(uint64_t board_bytes) {
    return board_bytes ? (sizeof(BoardEntry) + size_t(board_bytes) + 63) & ~size_t(63) : 0;
  }
  Slot* slot(uint32_t i) { return reinterpret_cast<Slot*>(base_ + sizeof(Header) + size_t(i) * slot_stride(h_->slot_bytes)); }
  BoardEntry* entry(uint32_t i, uint32_t r) {
    char* b = base_ + sizeof(Header) + size_t(h_->nslots) * slot_stride(h_->slot_bytes);
    return reinterpret_cast<BoardEntry*>(b + (size_t(i) * h_->board_ranks + r) * board_stride(h_->board_bytes));
  }
  uint64_t min_cursor() const {
    uint64_t m = h_->head.load();
    for (uint32_t r = 0; r < h_->nreaders; r++) m = std::min(m, h_->cur[r].seq.load(std::memory_order_acquire));
    return m;
  }
  void check_reader(uint32_t r) const {
    if (r >= h_->nreaders) throw std::out_of_range("reader index");
  }

  std::string name_;
  bool owner_;
  size_t size_ = 0;
  char* base_ = nullptr;
  Header* h_ = nullptr;
};

}  // namespace

PYBIND11_MODULE(_shmring, m) {
  m.doc() = "single-producer / multi-consumer command ring in POSIX shared memory (parallel/mesh.py)";
  py::class_<Ring>(m, "Ring")
      .def(py::init<const std::string&, bool, uint32_t, uint64_t, uint32_t, uint64_t>(), py::arg("name"),
           py::arg("create"), py::arg("nslots") = 64, py::arg("slot_bytes") = 1 << 16, py::arg("nreaders") = 1,
           py::arg("board_bytes") = 0)
      .def("post", &Ring::post, py::arg("rank"), py::arg("seq"), py::arg("payload"))
      .def("collect", &Ring::collect, py::arg("seq"), py::arg("timeout_s") = 120.0, py::arg("spin_us") = 200.0)
      .def("attach", &Ring::attach)
      .def("publish", &Ring::publish, py::arg("op"), py::arg("payload"), py::arg("timeout_s") = 120.0)
      .def("read", &Ring::read, py::arg("reader"), py::arg("spin_us") = 200.0)
      .def("close", &Ring::close_ring)
      .def_property_readonly("slot_bytes", &Ring::slot_bytes)
      .def_property_readonly("board_bytes", &Ring::board_bytes)
      .def_property_readonly("nreaders", &Ring::nreaders)
      .def_property_readonly("head", &Ring::head);
}
