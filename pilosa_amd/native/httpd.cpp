// Native HTTP/1.1 front end: epoll workers, keep-alive, pipelining, chunked
// request bodies.  Reference: the Go net/http server behind http/handler.go
// (routes :276-314, query route :293 -> handlePostQuery :495, content
// negotiation :977-1052).
//
// Parsing, connection handling and response writing run on native threads
// without the GIL.  Requests reach Python through three queues:
//
//   * kind 1 -- "count batchable": POST /index/{i}/query with a JSON-acceptable
//     Accept header, no query arguments, a non-protobuf body made only of
//     top-level Count(...) calls.  take_counts() hands Python every queued
//     request of this kind grouped by index as ONE concatenated PQL text plus
//     the (request id, calls) list, so a whole group commit is one native
//     compile + one device launch (executor._count_text_fast); the counts go
//     back in one respond_counts() call that formats {"results": [...]} here.
//     A group Python cannot answer that way is requeue()d as kind 0.
//   * kind 2 -- "topn batchable" (when enabled): the same shape made only of
//     flat TopN(...) calls (no nested call: cache-only TopN).  take_topn()
//     groups them like take_counts(), so the concurrent TopN requests of a
//     serving mix become one device batch (executor._topn_text_fast).
//   * kind 0 -- everything else: take() returns (id, method, path, query,
//     headers, body) and Python's route table answers with respond().
//
// Responses on a connection are written in request order (a per-connection
// sequence number), from whichever thread produces them; a short write
// leaves the rest to the connection's epoll worker (EPOLLOUT).
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace httpd {

constexpr size_t MAX_HEADER = 1 << 20;

struct Conn;

struct Req {
  uint64_t id = 0;
  std::shared_ptr<Conn> conn;
  uint64_t seq = 0;
  bool close_after = false;
  int kind = 0;
  int ncalls = 0;
  std::string method, path, query, index, body;
  std::vector<std::pair<std::string, std::string>> headers;
  std::string cors;   // CORS response headers when the Origin is allowed (else empty)
};

struct Conn : std::enable_shared_from_this<Conn> {
  int fd = -1;
  int epfd = -1;
  std::mutex mu;
  std::string in;
  uint64_t next_seq = 0;  // next request sequence number to assign
  uint64_t send_seq = 0;  // next response sequence number to write
  std::map<uint64_t, std::pair<std::string, bool>> ready;  // seq -> (bytes, close after)
  std::string out;
  size_t out_off = 0;
  bool closing = false;   // shut down once `out` drains
  bool closed = false;
  bool want_out = false;  // EPOLLOUT armed
  bool peer_eof = false;  // the client shut its side: answer what is queued, read no more
  bool sent_continue = false;
  // HTTP/1.1 pipelining: a connection's requests execute one at a time, in
  // order (as Go's net/http serves a connection); later ones wait here
  bool busy = false;
  std::deque<std::shared_ptr<Req>> waiting;
};

// epoll interest of a connection (conn lock held)
static void rearm(Conn& c) {
  epoll_event ev{};
  ev.events = (c.peer_eof ? 0u : uint32_t(EPOLLIN | EPOLLRDHUP)) | (c.want_out ? uint32_t(EPOLLOUT) : 0u);
  ev.data.ptr = &c;
  epoll_ctl(c.epfd, EPOLL_CTL_MOD, c.fd, &ev);
}

static bool ieq(const std::string& a, const char* b) {
  const size_t n = strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; i++)
    if (tolower(static_cast<unsigned char>(a[i])) != tolower(static_cast<unsigned char>(b[i]))) return false;
  return true;
}

static std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t')) a++;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) b--;
  return s.substr(a, b - a);
}

static const char* reason(int st) {
  switch (st) {
    case 100: return "Continue";
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 406: return "Not Acceptable";
    case 409: return "Conflict";
    case 411: return "Length Required";
    case 413: return "Request Entity Too Large";
    case 415: return "Unsupported Media Type";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

static std::string make_response(int status, const std::string& ctype, const char* body, size_t n, bool close,
                                 const char* extra = nullptr) {
  std::string r;
  r.reserve(160 + n);
  r += "HTTP/1.1 ";
  r += std::to_string(status);
  r += ' ';
  r += reason(status);
  r += "\r\n";
  if (!ctype.empty()) {
    r += "Content-Type: ";
    r += ctype;
    r += "\r\n";
  }
  r += "Content-Length: ";
  r += std::to_string(n);
  r += "\r\n";
  if (extra) r += extra;
  if (close) r += "Connection: close\r\n";
  r += "\r\n";
  r.append(body, n);
  return r;
}

// Top-level calls of a PQL text (the planner's split, native/pql_compile.cpp
// plan_count_text): -1 when quoted strings or unbalanced parentheses appear,
// else the number of calls; *all_count = every call starts with "Count(";
// *all_topn = every call is a flat "TopN(...)" (no nested call: the cache-only
// shape the TopN group commit answers).
static int split_calls(const std::string& t, bool* all_count, bool* all_topn = nullptr) {
  size_t i = 0, n = t.size();
  int calls = 0;
  *all_count = true;
  if (all_topn) *all_topn = true;
  while (i < n) {
    while (i < n && (t[i] == ' ' || t[i] == '\t' || t[i] == '\n' || t[i] == '\r')) i++;
    if (i >= n) break;
    if (t.compare(i, 6, "Count(") != 0) *all_count = false;
    if (all_topn && t.compare(i, 5, "TopN(") != 0) *all_topn = false;
    int depth = 0;
    bool seen = false;
    for (; i < n; i++) {
      const char c = t[i];
      if (c == '"' || c == '\'') return -1;
      if (c == '(') {
        depth++;
        if (depth > 1 && all_topn) *all_topn = false;
        seen = true;
      } else if (c == ')' && --depth == 0) {
        i++;
        break;
      }
      if (depth < 0) return -1;
    }
    if (!seen || depth != 0) return -1;
    calls++;
  }
  return calls;
}

// Strict UTF-8 (no overlongs, surrogates or code points past U+10FFFF): the
// request head reaches Python as str, so anything else is refused with 400.
static bool valid_utf8(const char* s, size_t n) {
  const auto* p = reinterpret_cast<const unsigned char*>(s);
  size_t i = 0;
  while (i < n) {
    const unsigned c = p[i];
    if (c < 0x80) {
      i++;
      continue;
    }
    size_t len;
    unsigned cp;
    if ((c & 0xE0) == 0xC0) len = 2, cp = c & 0x1F;
    else if ((c & 0xF0) == 0xE0) len = 3, cp = c & 0x0F;
    else if ((c & 0xF8) == 0xF0) len = 4, cp = c & 0x07;
    else return false;
    if (i + len > n) return false;
    for (size_t k = 1; k < len; k++) {
      if ((p[i + k] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (p[i + k] & 0x3F);
    }
    if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000) || cp > 0x10FFFF ||
        (cp >= 0xD800 && cp <= 0xDFFF))
      return false;
    i += len;
  }
  return true;
}

static py::str str_lossy(const std::string& s) {
  PyObject* o = PyUnicode_DecodeUTF8(s.data(), Py_ssize_t(s.size()), "replace");
  if (!o) throw py::error_already_set();
  return py::reinterpret_steal<py::str>(o);
}

static bool accept_json(const std::string& acc) {
  if (acc.empty()) return true;
  size_t p = 0;
  while (p <= acc.size()) {
    size_t e = acc.find(',', p);
    if (e == std::string::npos) e = acc.size();
    std::string v = acc.substr(p, e - p);
    const size_t semi = v.find(';');
    if (semi != std::string::npos) v = v.substr(0, semi);
    v = trim(v);
    if (v == "application/json" || v == "*/*" || v == "*/json" || v == "application/*") return true;
    p = e + 1;
  }
  return false;
}

class Server {
 public:
  Server(const std::string& host, int port, int nthreads, int64_t max_body)
      : nthreads_(std::max(1, nthreads)), max_body_(size_t(max_body)) {
    lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (lfd_ < 0) throw std::runtime_error("socket: " + std::string(strerror(errno)));
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(uint16_t(port));
    const std::string h = host.empty() ? "0.0.0.0" : host;
    if (inet_pton(AF_INET, h.c_str(), &a.sin_addr) != 1) {
      ::close(lfd_);
      throw std::runtime_error("bad bind host: " + h);
    }
    if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(lfd_, 4096) != 0) {
      const std::string err = strerror(errno);
      ::close(lfd_);
      throw std::runtime_error("bind/listen " + h + ":" + std::to_string(port) + ": " + err);
    }
    socklen_t len = sizeof(a);
    getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &len);
    port_ = ntohs(a.sin_port);
  }

  ~Server() {
    stop();
    if (lfd_ >= 0) ::close(lfd_);
  }

  int port() const { return port_; }

  void start() {
    if (running_.exchange(true)) return;
    for (int t = 0; t < nthreads_; t++) {
      const int ep = epoll_create1(EPOLL_CLOEXEC);
      const int wk = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLEXCLUSIVE;
      ev.data.u64 = LISTEN_TAG;
      epoll_ctl(ep, EPOLL_CTL_ADD, lfd_, &ev);
      ev.events = EPOLLIN;
      ev.data.u64 = WAKE_TAG;
      epoll_ctl(ep, EPOLL_CTL_ADD, wk, &ev);
      epfds_.push_back(ep);
      wakefds_.push_back(wk);
    }
    for (int t = 0; t < nthreads_; t++) workers_.emplace_back([this, t] { loop(t); });
  }

  void stop() {
    if (!running_.exchange(false)) return;
    stopping_ = true;
    for (int w : wakefds_) {
      uint64_t one = 1;
      (void)!::write(w, &one, 8);
    }
    for (auto& th : workers_) th.join();
    workers_.clear();
    // a stopped server refuses new connections (workers closed the open ones)
    if (lfd_ >= 0) ::close(lfd_);
    lfd_ = -1;
    for (int e : epfds_) ::close(e);
    for (int w : wakefds_) ::close(w);
    epfds_.clear();
    wakefds_.clear();
    {
      std::lock_guard<std::mutex> g(qmu_);
      for (auto& q : q_) q.clear();
    }
    qcv_.notify_all();
    std::lock_guard<std::mutex> g(pmu_);
    pending_.clear();
  }

  // kind-0 requests: [(id, method, path, query, [(name, value)], body)]
  py::list take(int max_n, int timeout_ms) {
    std::vector<std::shared_ptr<Req>> got;
    {
      py::gil_scoped_release nogil;
      pop(0, size_t(std::max(1, max_n)), timeout_ms, got);
    }
    py::list out;
    for (auto& r : got) {
      py::list hs;
      for (auto& kv : r->headers) hs.append(py::make_tuple(str_lossy(kv.first), str_lossy(kv.second)));
      out.append(py::make_tuple(r->id, str_lossy(r->method), str_lossy(r->path), str_lossy(r->query), hs,
                                py::bytes(r->body)));
    }
    return out;
  }

  // kind-1 requests grouped by index: [(index, [ids], [ncalls], text)]
  // min_n / hold_us: once a request is queued, wait up to hold_us more for
  // min_n of them (adaptive group commit: the batcher asks for a fuller batch
  // only while another batch keeps the device busy)
  py::list take_counts(int max_n, int timeout_ms, int min_n, int hold_us) {
    return take_grouped(1, max_n, timeout_ms, min_n, hold_us);
  }

  py::list take_grouped(int kind, int max_n, int timeout_ms, int min_n = 1, int hold_us = 0) {
    std::vector<std::shared_ptr<Req>> got;
    std::vector<std::pair<std::string, std::vector<size_t>>> groups;
    std::vector<std::string> texts;
    {
      py::gil_scoped_release nogil;
      pop(kind, size_t(std::max(1, max_n)), timeout_ms, got, size_t(std::max(1, min_n)), hold_us);
      for (size_t i = 0; i < got.size(); i++) {
        size_t g = 0;
        while (g < groups.size() && groups[g].first != got[i]->index) g++;
        if (g == groups.size()) groups.emplace_back(got[i]->index, std::vector<size_t>());
        groups[g].second.push_back(i);
      }
      texts.resize(groups.size());
      for (size_t g = 0; g < groups.size(); g++) {
        size_t n = 0;
        for (size_t i : groups[g].second) n += got[i]->body.size() + 1;
        texts[g].reserve(n);
        for (size_t i : groups[g].second) {
          texts[g] += got[i]->body;
          texts[g] += '\n';
        }
      }
    }
    py::list out;
    for (size_t g = 0; g < groups.size(); g++) {
      py::list ids, nc;
      for (size_t i : groups[g].second) {
        ids.append(got[i]->id);
        nc.append(got[i]->ncalls);
      }
      out.append(py::make_tuple(str_lossy(groups[g].first), ids, nc, str_lossy(texts[g])));
    }
    return out;
  }

  // kind-2 requests (flat TopN calls), grouped by index like take_counts
  py::list take_topn(int max_n, int timeout_ms) { return take_grouped(2, max_n, timeout_ms); }

  // Give count requests back to the general path (kind 0).
  void requeue(const std::vector<uint64_t>& ids) {
    std::vector<std::shared_ptr<Req>> rs;
    {
      std::lock_guard<std::mutex> g(pmu_);
      for (uint64_t id : ids) {
        auto it = pending_.find(id);
        if (it != pending_.end()) rs.push_back(it->second);
      }
    }
    {
      std::lock_guard<std::mutex> g(qmu_);
      for (auto& r : rs) {
        r->kind = 0;
        q_[0].push_back(r);
      }
    }
    qcv_.notify_all();
  }

  void respond(uint64_t id, int status, const std::string& ctype, py::bytes body) {
    char* p = nullptr;
    Py_ssize_t n = 0;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    std::string bytes(p, size_t(n));
    py::gil_scoped_release nogil;
    finish(id, status, ctype, bytes);
  }

  // {"results": [c, ...]} per request, counts in call order over the group
  void respond_counts(const std::vector<uint64_t>& ids, const std::vector<int>& ncalls,
                      const std::vector<int64_t>& counts) {
    if (ids.size() != ncalls.size()) throw std::invalid_argument("ids / ncalls length mismatch");
    size_t total = 0;
    for (int c : ncalls) total += size_t(std::max(0, c));
    if (total != counts.size()) throw std::invalid_argument("counts do not match the calls");
    py::gil_scoped_release nogil;
    size_t k = 0;
    std::string body;
    for (size_t i = 0; i < ids.size(); i++) {
      body.assign("{\"results\":[");   // Go's encoding/json: no spaces
      for (int c = 0; c < ncalls[i]; c++, k++) {
        if (c) body += ",";
        body += std::to_string(counts[k]);
      }
      body += "]}\n";
      finish(ids[i], 200, "application/json", body);
    }
  }

  void set_count_batching(bool on) { count_batching_ = on; }
  void set_topn_batching(bool on) { topn_batching_ = on; }

  // origins allowed by CORS (set before start())
  void set_cors(const std::vector<std::string>& origins) { cors_origins_ = origins; }

  // A fixed 200 response for (method, path) with no query string, served by
  // the epoll workers without a round trip through Python.
  void set_static(const std::string& method, const std::string& path, const std::string& ctype, py::bytes body) {
    std::string b = body;
    std::lock_guard<std::mutex> g(smu_);
    statics_[method + " " + path] = std::make_pair(ctype, std::move(b));
    statics_empty_ = false;
  }

  py::dict stats() {
    py::dict d;
    d["requests"] = requests_.load();
    d["count_requests"] = count_requests_.load();
    d["topn_requests"] = topn_requests_.load();
    d["connections"] = connections_.load();
    d["responses"] = responses_.load();
    std::lock_guard<std::mutex> g(qmu_);
    d["queued_generic"] = q_[0].size();
    d["queued_counts"] = q_[1].size();
    d["queued_topn"] = q_[2].size();
    return d;
  }

 private:
  static constexpr uint64_t LISTEN_TAG = 1, WAKE_TAG = 2;

  void pop(int kind, size_t max_n, int timeout_ms, std::vector<std::shared_ptr<Req>>& got, size_t min_n = 1,
           int hold_us = 0) {
    std::unique_lock<std::mutex> g(qmu_);
    auto& q = q_[kind];
    // system_clock deadline: its wait maps to pthread_cond_timedwait, which
    // ThreadSanitizer intercepts (a steady_clock wait_for goes through
    // pthread_cond_clockwait, which gcc-11's TSan does not, and then reports a
    // false double lock); the wait is a short poll, so clock jumps only end it
    // early or late by that much
    if (q.empty())
      qcv_.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(std::max(0, timeout_ms)),
                      [&] { return !q.empty() || stopping_; });
    if (!q.empty() && q.size() < std::min(min_n, max_n) && hold_us > 0)
      qcv_.wait_until(g, std::chrono::system_clock::now() + std::chrono::microseconds(hold_us),
                      [&] { return q.size() >= std::min(min_n, max_n) || stopping_; });
    while (!q.empty() && got.size() < max_n) {
      got.push_back(std::move(q.front()));
      q.pop_front();
    }
  }

  void finish(uint64_t id, int status, const std::string& ctype, const std::string& body) {
    std::shared_ptr<Req> r;
    {
      std::lock_guard<std::mutex> g(pmu_);
      auto it = pending_.find(id);
      if (it == pending_.end()) return;
      r = std::move(it->second);
      pending_.erase(it);
    }
    responses_++;
    auto c = r->conn;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->closed) {
      std::lock_guard<std::mutex> pg(pmu_);
      for (auto& w : c->waiting) pending_.erase(w->id);
      c->waiting.clear();
      c->busy = false;
      return;
    }
    c->ready.emplace(r->seq, std::make_pair(make_response(status, ctype, body.data(), body.size(), r->close_after,
                                                          r->cors.empty() ? nullptr : r->cors.c_str()),
                                            r->close_after));
    drain_ready(*c);
    flush(*c);
    if (!c->waiting.empty()) {
      auto nx = std::move(c->waiting.front());
      c->waiting.pop_front();
      enqueue(nx);
    } else {
      c->busy = false;
    }
  }

  void enqueue(const std::shared_ptr<Req>& r) {
    {
      std::lock_guard<std::mutex> g(qmu_);
      q_[r->kind].push_back(r);
    }
    qcv_.notify_all();
  }

  // move in-order ready responses into the output buffer (conn lock held)
  static void drain_ready(Conn& c) {
    while (!c.ready.empty() && c.ready.begin()->first == c.send_seq) {
      auto it = c.ready.begin();
      if (c.out_off == c.out.size()) {
        c.out.clear();
        c.out_off = 0;
      }
      c.out += it->second.first;
      if (it->second.second) c.closing = true;
      c.ready.erase(it);
      c.send_seq++;
    }
  }

  // write what we can (conn lock held); arm EPOLLOUT on a short write
  void flush(Conn& c) {
    while (c.out_off < c.out.size()) {
      const ssize_t w = ::send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (w > 0) {
        c.out_off += size_t(w);
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (!c.want_out) {
          c.want_out = true;
          rearm(c);
        }
        return;
      }
      // peer gone: drop the output, the worker closes on the hangup
      c.out.clear();
      c.out_off = 0;
      ::shutdown(c.fd, SHUT_RDWR);
      return;
    }
    c.out.clear();
    c.out_off = 0;
    if (c.want_out) {
      c.want_out = false;
      rearm(c);
    }
    // everything answered on a closing connection: hang up (the worker sees
    // EPOLLHUP and closes the descriptor)
    if (c.closing && c.ready.empty() && c.send_seq == c.next_seq) ::shutdown(c.fd, SHUT_RDWR);
  }

  void loop(int t) {
    const int ep = epfds_[t];
    std::unordered_map<Conn*, std::shared_ptr<Conn>> conns;
    std::vector<epoll_event> evs(256);
    std::vector<char> buf(1 << 16);
    while (!stopping_) {
      const int n = epoll_wait(ep, evs.data(), int(evs.size()), 200);
      for (int i = 0; i < n; i++) {
        const uint64_t tag = evs[i].data.u64;
        if (tag == WAKE_TAG) continue;
        if (tag == LISTEN_TAG) {
          for (;;) {
            const int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
            if (fd < 0) break;
            int one = 1;
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            auto c = std::make_shared<Conn>();
            c->fd = fd;
            c->epfd = ep;
            epoll_event ev{};
            ev.events = EPOLLIN | EPOLLRDHUP;
            ev.data.ptr = c.get();
            conns.emplace(c.get(), c);
            connections_++;
            epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
          }
          continue;
        }
        Conn* cp = static_cast<Conn*>(evs[i].data.ptr);
        auto it = conns.find(cp);
        if (it == conns.end()) continue;
        std::shared_ptr<Conn> c = it->second;
        bool dead = false;
        {
          std::lock_guard<std::mutex> g(c->mu);
          if (evs[i].events & EPOLLOUT) flush(*c);
          if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
            for (;;) {
              const ssize_t r = ::recv(c->fd, buf.data(), buf.size(), 0);
              if (r > 0) {
                c->in.append(buf.data(), size_t(r));
                continue;
              }
              if (r < 0 && errno == EINTR) continue;
              if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
              if (r == 0) c->peer_eof = true;
              else dead = true;  // error
              break;
            }
            if (!dead && !parse(*c)) dead = true;
            if (!dead && c->peer_eof) {
              if (c->send_seq == c->next_seq && c->ready.empty()) {
                dead = true;  // nothing outstanding
              } else {
                c->closing = true;  // answer the queued requests first
                rearm(*c);
              }
            }
            if (evs[i].events & (EPOLLHUP | EPOLLERR)) dead = true;
          }
          if (dead) {
            c->closed = true;
            epoll_ctl(ep, EPOLL_CTL_DEL, c->fd, nullptr);
            ::close(c->fd);
            c->fd = -1;
          }
        }
        if (dead) conns.erase(it);
      }
    }
    for (auto& kv : conns) {
      std::lock_guard<std::mutex> g(kv.second->mu);
      if (!kv.second->closed) {
        kv.second->closed = true;
        ::close(kv.second->fd);
      }
    }
  }

  // queue an immediate native response (errors, OPTIONS) in sequence order
  void native_reply(Conn& c, uint64_t seq, int status, const std::string& body, bool close,
                    const char* extra = nullptr) {
    c.ready.emplace(seq, std::make_pair(make_response(status, body.empty() ? "" : "text/plain; charset=utf-8",
                                                      body.data(), body.size(), close, extra),
                                        close));
    drain_ready(c);
    flush(c);
  }

  // Parse every complete request in c.in (conn lock held); false = protocol
  // error after which the connection is closed.
  bool parse(Conn& c) {
    size_t off = 0;
    bool ok = true;
    while (!c.closing) {
      const size_t he = c.in.find("\r\n\r\n", off);
      if (he == std::string::npos) {
        if (c.in.size() - off > MAX_HEADER) {
          native_reply(c, c.next_seq++, 431, "request header too large\n", true);
          ok = false;
        }
        break;
      }
      if (!valid_utf8(c.in.data() + off, he - off)) {
        native_reply(c, c.next_seq++, 400, "request head is not valid UTF-8\n", true);
        ok = false;
        break;
      }
      // request line
      const size_t le = c.in.find("\r\n", off);
      const std::string line = c.in.substr(off, le - off);
      const size_t s1 = line.find(' '), s2 = line.rfind(' ');
      if (s1 == std::string::npos || s2 == s1) {
        native_reply(c, c.next_seq++, 400, "malformed request line\n", true);
        ok = false;
        break;
      }
      auto r = std::make_shared<Req>();
      r->method = line.substr(0, s1);
      const std::string target = line.substr(s1 + 1, s2 - s1 - 1);
      const std::string version = line.substr(s2 + 1);
      const size_t qm = target.find('?');
      r->path = target.substr(0, qm);
      r->query = qm == std::string::npos ? "" : target.substr(qm + 1);
      bool keep = version == "HTTP/1.1";
      bool chunked = false, expect100 = false;
      size_t clen = 0;
      bool has_len = false, bad_len = false;
      std::string ctype, accept, origin, preflight;
      for (size_t p = le + 2; p < he;) {
        size_t e = c.in.find("\r\n", p);
        if (e == std::string::npos || e > he) e = he;
        const size_t colon = c.in.find(':', p);
        if (colon != std::string::npos && colon < e) {
          std::string k = c.in.substr(p, colon - p), v = trim(c.in.substr(colon + 1, e - colon - 1));
          if (ieq(k, "content-length")) {
            bool digits = !v.empty() && v.size() <= 18;
            for (char ch : v) digits = digits && ch >= '0' && ch <= '9';
            if (!digits || (has_len && clen != size_t(strtoull(v.c_str(), nullptr, 10)))) bad_len = true;
            has_len = true;
            clen = digits ? size_t(strtoull(v.c_str(), nullptr, 10)) : 0;
          } else if (ieq(k, "transfer-encoding")) {
            chunked = v.find("chunked") != std::string::npos;
          } else if (ieq(k, "connection")) {
            if (ieq(v, "close")) keep = false;
            else if (ieq(v, "keep-alive")) keep = true;
          } else if (ieq(k, "expect")) {
            expect100 = ieq(v, "100-continue");
          } else if (ieq(k, "content-type")) {
            ctype = v;
          } else if (ieq(k, "accept")) {
            accept = v;
          } else if (ieq(k, "origin")) {
            origin = v;
          } else if (ieq(k, "access-control-request-method")) {
            preflight = v;
          }
          r->headers.emplace_back(std::move(k), std::move(v));
        }
        p = e + 2;
      }
      // a malformed Content-Length, or both framings at once (request smuggling)
      if (bad_len || (chunked && has_len)) {
        native_reply(c, c.next_seq++, 400, "bad request framing\n", true);
        ok = false;
        break;
      }
      // body
      size_t end = he + 4;
      if (chunked) {
        std::string body;
        size_t p = end;
        bool complete = false, bad = false, malformed = false;
        for (;;) {
          const size_t e = c.in.find("\r\n", p);
          if (e == std::string::npos) break;
          // chunk-size line: 1..15 hex digits, optional ";ext"
          size_t sz = 0, nd = 0, q = p;
          for (; q < e && nd < 16; q++, nd++) {
            const int ch = static_cast<unsigned char>(c.in[q]);
            int v;
            if (ch >= '0' && ch <= '9') v = ch - '0';
            else if (ch >= 'a' && ch <= 'f') v = ch - 'a' + 10;
            else if (ch >= 'A' && ch <= 'F') v = ch - 'A' + 10;
            else break;
            sz = (sz << 4) | size_t(v);
          }
          if (nd == 0 || nd > 15 || (q < e && c.in[q] != ';' && c.in[q] != ' ' && c.in[q] != '\t')) {
            malformed = true;
            break;
          }
          if (sz > max_body_ || body.size() > max_body_ - sz) {
            bad = true;
            break;
          }
          if (sz == 0) {
            // optional trailer lines, then an empty line
            if (c.in.size() >= e + 4 && c.in.compare(e + 2, 2, "\r\n") == 0) {
              end = e + 4;
              complete = true;
            } else {
              const size_t t = c.in.find("\r\n\r\n", e + 2);
              if (t != std::string::npos) {
                end = t + 4;
                complete = true;
              }
            }
            break;
          }
          if (c.in.size() - (e + 2) < sz + 2) break;
          if (c.in.compare(e + 2 + sz, 2, "\r\n") != 0) {
            malformed = true;
            break;
          }
          body.append(c.in, e + 2, sz);
          p = e + 2 + sz + 2;   // strictly increases (sz + 4 >= 4 bytes per chunk)
        }
        if (malformed) {
          native_reply(c, c.next_seq++, 400, "malformed chunked body\n", true);
          ok = false;
          break;
        }
        if (bad) {
          native_reply(c, c.next_seq++, 413, "request body too large\n", true);
          ok = false;
          break;
        }
        if (!complete) {
          if (expect100 && !c.sent_continue) {
            c.sent_continue = true;
            c.out += "HTTP/1.1 100 Continue\r\n\r\n";
            flush(c);
          }
          break;
        }
        r->body = std::move(body);
      } else {
        if (has_len && clen > max_body_) {
          native_reply(c, c.next_seq++, 413, "request body too large\n", true);
          ok = false;
          break;
        }
        if (c.in.size() < end + clen) {
          if (expect100 && !c.sent_continue) {
            c.sent_continue = true;
            c.out += "HTTP/1.1 100 Continue\r\n\r\n";
            flush(c);
          }
          break;
        }
        r->body.assign(c.in, end, clen);
        end += clen;
      }
      off = end;
      c.sent_continue = false;
      r->seq = c.next_seq++;
      r->close_after = !keep;
      requests_++;
      // CORS (http/handler.go OptHandlerAllowedOrigins): only for configured
      // origins; a preflight from one is answered here, any other OPTIONS goes
      // to the route table (405 / 404, as without CORS)
      if (!origin.empty() && !cors_origins_.empty() &&
          std::find(cors_origins_.begin(), cors_origins_.end(), origin) != cors_origins_.end())
        r->cors = "Access-Control-Allow-Origin: " + origin + "\r\nVary: Origin\r\n";
      if (r->method == "OPTIONS" && !r->cors.empty() && !preflight.empty()) {
        const std::string extra = r->cors + "Access-Control-Allow-Methods: " + preflight +
                                  "\r\nAccess-Control-Allow-Headers: Content-Type\r\n";
        native_reply(c, r->seq, 200, "", r->close_after, extra.c_str());
        continue;
      }
      if (r->query.empty() && !statics_empty_.load()) {
        // fixed responses answered on the I/O thread (liveness probes: a
        // busy Python worker pool must not make a node look dead)
        std::string hit_ct, hit_body;
        bool hit = false;
        {
          std::lock_guard<std::mutex> g(smu_);
          auto it = statics_.find(r->method + " " + r->path);
          if (it != statics_.end()) hit = true, hit_ct = it->second.first, hit_body = it->second.second;
        }
        if (hit) {
          c.ready.emplace(r->seq, std::make_pair(make_response(200, hit_ct, hit_body.data(), hit_body.size(),
                                                               r->close_after,
                                                               r->cors.empty() ? nullptr : r->cors.c_str()),
                                                 r->close_after));
          drain_ready(c);
          flush(c);
          if (r->close_after) {
            c.closing = true;
            break;
          }
          continue;
        }
      }
      classify(*r, ctype, accept);
      r->conn = c.shared_from_this();
      r->id = next_id_++;
      {
        std::lock_guard<std::mutex> g(pmu_);
        pending_.emplace(r->id, r);
      }
      if (c.busy) {
        c.waiting.push_back(r);   // runs once the earlier requests are answered
      } else {
        c.busy = true;
        enqueue(r);
      }
      if (r->close_after) {
        c.closing = true;  // answer what we have, read nothing more
        break;
      }
    }
    if (off) c.in.erase(0, off);
    return ok;
  }

  // kind 1 when the request is a JSON Count-only query with no arguments,
  // kind 2 when it is only flat TopN(...) calls (cache-only TopN batching)
  void classify(Req& r, const std::string& ctype, const std::string& accept) {
    r.kind = 0;
    if ((!count_batching_ && !topn_batching_) || r.method != "POST" || !r.query.empty() ||
        ctype == "application/x-protobuf" || !accept_json(accept))
      return;
    std::string p = r.path;
    while (p.size() > 1 && p.back() == '/') p.pop_back();
    static const std::string pre = "/index/", suf = "/query";
    if (p.size() <= pre.size() + suf.size() || p.compare(0, pre.size(), pre) != 0 ||
        p.compare(p.size() - suf.size(), suf.size(), suf) != 0)
      return;
    std::string name = p.substr(pre.size(), p.size() - pre.size() - suf.size());
    if (name.empty() || name.find('/') != std::string::npos) return;
    bool all_count = false, all_topn = false;
    const int n = split_calls(r.body, &all_count, &all_topn);
    if (n <= 0) return;
    if (all_count && count_batching_) {
      r.kind = 1;
      count_requests_++;
    } else if (all_topn && topn_batching_) {
      r.kind = 2;
      topn_requests_++;
    } else {
      return;
    }
    r.ncalls = n;
    r.index = std::move(name);
  }

 private:
  int lfd_ = -1, port_ = 0, nthreads_;
  size_t max_body_;
  std::atomic<bool> running_{false}, stopping_{false}, count_batching_{true}, topn_batching_{false},
      statics_empty_{true};
  std::vector<std::string> cors_origins_;
  std::mutex smu_;
  std::unordered_map<std::string, std::pair<std::string, std::string>> statics_;
  std::vector<std::thread> workers_;
  std::vector<int> epfds_, wakefds_;
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<std::shared_ptr<Req>> q_[3];
  std::mutex pmu_;
  std::unordered_map<uint64_t, std::shared_ptr<Req>> pending_;
  std::atomic<uint64_t> next_id_{1};
  std::atomic<uint64_t> requests_{0}, count_requests_{0}, topn_requests_{0}, connections_{0}, responses_{0};
};


// ---------------------------------------------------------------- load client
// Closed-loop HTTP/1.1 load generator for the serving benchmark (the role
// wrk plays for the reference's Go server): `conns` keep-alive connections
// spread over `threads` epoll threads; each connection POSTs bodies[k] (k
// round-robin from a per-connection offset) and sends the next request when
// the response is complete.  Runs without the GIL.
struct LoadConn {
  int fd = -1;
  size_t k = 0;
  std::string in;
  std::chrono::steady_clock::time_point t0;
};

static bool send_all(int fd, const std::string& s) {
  size_t o = 0;
  while (o < s.size()) {
    const ssize_t w = ::send(fd, s.data() + o, s.size() - o, MSG_NOSIGNAL);
    if (w > 0) {
      o += size_t(w);
    } else if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) {
      std::this_thread::yield();
    } else {
      return false;
    }
  }
  return true;
}

py::dict load(const std::string& host, int port, const std::string& path, const std::vector<std::string>& bodies,
              int conns, int threads, double seconds, int samples) {
  if (bodies.empty() || conns <= 0) throw std::invalid_argument("load: bodies and conns required");
  threads = std::max(1, std::min(threads, conns));
  std::vector<std::string> reqs;
  reqs.reserve(bodies.size());
  for (auto& b : bodies)
    reqs.push_back("POST " + path + " HTTP/1.1\r\nHost: " + host + "\r\nContent-Length: " +
                   std::to_string(b.size()) + "\r\n\r\n" + b);
  std::atomic<uint64_t> total{0}, errors{0};
  std::mutex smu;
  std::vector<std::pair<size_t, std::string>> sample;
  std::string first_error;
  std::vector<std::vector<double>> lats(static_cast<size_t>(threads));
  std::atomic<int> failed_connect{0};
  double elapsed = 0;
  {
    py::gil_scoped_release nogil;
    // the clock starts once every connection is up (a slow accept backlog
    // must not eat the measurement window)
    std::mutex lmu;
    std::condition_variable lcv;
    int connected = 0;
    std::chrono::steady_clock::time_point deadline, start;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
      th.emplace_back([&, t] {
        const int ep = epoll_create1(EPOLL_CLOEXEC);
        std::vector<LoadConn> cs;
        for (int c = t; c < conns; c += threads) {
          LoadConn lc;
          lc.fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
          sockaddr_in a{};
          a.sin_family = AF_INET;
          a.sin_port = htons(uint16_t(port));
          inet_pton(AF_INET, host.c_str(), &a.sin_addr);
          if (::connect(lc.fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
            failed_connect++;
            ::close(lc.fd);
            continue;
          }
          int one = 1;
          setsockopt(lc.fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          fcntl(lc.fd, F_SETFL, fcntl(lc.fd, F_GETFL) | O_NONBLOCK);
          lc.k = size_t(c) * 7919 % reqs.size();
          cs.push_back(std::move(lc));
        }
        {
          std::unique_lock<std::mutex> g(lmu);
          if (++connected == threads) {
            start = std::chrono::steady_clock::now();
            deadline = start + std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::duration<double>(seconds));
            lcv.notify_all();
          } else {
            lcv.wait(g, [&] { return connected == threads; });
          }
        }
        for (size_t i = 0; i < cs.size(); i++) {
          epoll_event ev{};
          ev.events = EPOLLIN;
          ev.data.u64 = i;
          epoll_ctl(ep, EPOLL_CTL_ADD, cs[i].fd, &ev);
          cs[i].t0 = std::chrono::steady_clock::now();
          send_all(cs[i].fd, reqs[cs[i].k]);
        }
        std::vector<epoll_event> evs(256);
        std::vector<char> buf(1 << 16);
        auto& lat = lats[size_t(t)];
        size_t live = cs.size();
        while (live && std::chrono::steady_clock::now() < deadline) {
          const int n = epoll_wait(ep, evs.data(), int(evs.size()), 20);
          for (int e = 0; e < n; e++) {
            LoadConn& c = cs[evs[e].data.u64];
            if (c.fd < 0) continue;
            bool dead = false;
            for (;;) {
              const ssize_t r = ::recv(c.fd, buf.data(), buf.size(), 0);
              if (r > 0) {
                c.in.append(buf.data(), size_t(r));
                continue;
              }
              if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) break;
              dead = true;
              break;
            }
            for (;;) {
              const size_t he = c.in.find("\r\n\r\n");
              if (he == std::string::npos) break;
              size_t clen = 0;
              const size_t cl = c.in.find("Content-Length: ");
              if (cl != std::string::npos && cl < he) clen = size_t(strtoull(c.in.c_str() + cl + 16, nullptr, 10));
              if (c.in.size() < he + 4 + clen) break;
              const bool ok = c.in.compare(0, 12, "HTTP/1.1 200") == 0;
              const auto now = std::chrono::steady_clock::now();
              lat.push_back(std::chrono::duration<double>(now - c.t0).count());
              total++;
              if (!ok) {
                errors++;
                std::lock_guard<std::mutex> g(smu);
                if (first_error.empty()) first_error = c.in.substr(0, he + 4 + std::min<size_t>(clen, 300));
              } else if (samples > 0) {
                std::lock_guard<std::mutex> g(smu);
                if (int(sample.size()) < samples) sample.emplace_back(c.k, c.in.substr(he + 4, clen));
              }
              c.in.erase(0, he + 4 + clen);
              c.k = (c.k + 1) % reqs.size();
              c.t0 = now;
              if (now < deadline && !send_all(c.fd, reqs[c.k])) dead = true;
            }
            if (dead) {
              ::close(c.fd);
              c.fd = -1;
              live--;
            }
          }
        }
        for (auto& c : cs)
          if (c.fd >= 0) ::close(c.fd);
        ::close(ep);
      });
    }
    for (auto& x : th) x.join();
    elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
  }
  std::vector<double> all;
  for (auto& v : lats) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, size_t(p * double(all.size())))]; };
  double sum = 0;
  for (double x : all) sum += x;
  py::dict d;
  d["requests"] = total.load();
  d["elapsed_s"] = elapsed;
  d["errors"] = errors.load();
  d["failed_connect"] = failed_connect.load();
  d["first_error"] = py::bytes(first_error);
  d["mean_ms"] = all.empty() ? 0.0 : sum / double(all.size()) * 1e3;
  d["p50_ms"] = pct(0.5) * 1e3;
  d["p99_ms"] = pct(0.99) * 1e3;
  py::list sm;
  for (auto& kv : sample) sm.append(py::make_tuple(kv.first, py::bytes(kv.second)));
  d["samples"] = sm;
  return d;
}

}  // namespace httpd

PYBIND11_MODULE(_httpd, m) {
  m.doc() = "Native HTTP/1.1 front end (epoll) for the pilosa_amd server";
  py::class_<httpd::Server>(m, "Server")
      .def(py::init<const std::string&, int, int, int64_t>(), py::arg("host"), py::arg("port"),
           py::arg("threads") = 4, py::arg("max_body") = int64_t(1) << 31)
      .def("port", &httpd::Server::port)
      .def("start", &httpd::Server::start)
      .def("stop", &httpd::Server::stop, py::call_guard<py::gil_scoped_release>())
      .def("take", &httpd::Server::take, py::arg("max_n") = 1, py::arg("timeout_ms") = 100)
      .def("take_counts", &httpd::Server::take_counts, py::arg("max_n") = 1 << 16, py::arg("timeout_ms") = 100,
           py::arg("min_n") = 1, py::arg("hold_us") = 0)
      .def("take_topn", &httpd::Server::take_topn, py::arg("max_n") = 1 << 16, py::arg("timeout_ms") = 100)
      .def("set_topn_batching", &httpd::Server::set_topn_batching)
      .def("requeue", &httpd::Server::requeue)
      .def("respond", &httpd::Server::respond)
      .def("respond_counts", &httpd::Server::respond_counts)
      .def("set_count_batching", &httpd::Server::set_count_batching)
      .def("set_cors", &httpd::Server::set_cors, py::arg("origins"))
      .def("set_static", &httpd::Server::set_static, py::arg("method"), py::arg("path"), py::arg("content_type"),
           py::arg("body"))
      .def("stats", &httpd::Server::stats);
  m.def("load", &httpd::load, py::arg("host"), py::arg("port"), py::arg("path"), py::arg("bodies"),
        py::arg("conns") = 128, py::arg("threads") = 4, py::arg("seconds") = 10.0, py::arg("samples") = 0,
        "closed-loop keep-alive HTTP load generator (serving benchmark client)");
}
