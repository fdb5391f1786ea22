// Native gRPC load generator (HTTP/2 client on libnghttp2), GIL-free.
//
// The benchmark client of the serving stack: pre-serialised
// request bodies (e.g. the exact PredictRequest the reference client builds,
// src/lib.rs:244-263) are fired over `connections` HTTP/2 connections with
// `concurrency` unary calls in flight; per-call latency is recorded from
// submit to end-of-stream (trailers) on the client clock.
#include <pthread.h>
#include <time.h>
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <sys/uio.h>

#include <algorithm>
#include <deque>
#include <cstring>
#include <stdexcept>

#include "http2.h"
#include "nghttp2_min.h"
#include "wire.h"

namespace tfs {

namespace {

struct Shared {
  std::vector<std::string> framed;
  std::string path, authority;
  std::atomic<uint64_t> total{0};
  std::atomic<uint64_t> issued{0};
  std::atomic<uint64_t> finished{0};
  // continuous mode (LoadGen::start): no request budget and no deadline; the
  // workers run until stop(), every completion gets a global sequence number
  // so a timed window can pick out exactly its completions
  std::atomic<bool> continuous{false};
  std::atomic<bool> stopping{false};
  Clock::time_point deadline;
  // a window() waiting for completion number `target`: the worker that
  // completes it wakes the waiter (no polling thread burning a core of the
  // CPU share the server and the generator run in)
  std::atomic<uint64_t> target{~uint64_t(0)};
  std::mutex wmu;
  std::condition_variable wcv;
};

// One completion in continuous mode: (sequence number, latency, ok, when)
struct Done {
  uint64_t seq;
  double us;
  bool ok;
  Clock::time_point at;
};

struct Req {
  const std::string* body;
  size_t off = 0;        // bytes handed to nghttp2 (read callback)
  size_t sent = 0;       // bytes queued for the socket (send_data callback)
  Clock::time_point t0;
  int http_status = 0;
  int grpc_status = -1;
  std::string grpc_message;
  size_t bytes = 0;
};

struct ClientConn {
  int fd = -1;
  nghttp2_session* sess = nullptr;
  Shared* sh = nullptr;
  int inflight = 0;
  int target = 0;
  bool dead = false;
  // Outgoing byte queue: small frames are copied (owned), DATA payloads are
  // borrowed straight from the pre-framed request bodies (zero-copy: the
  // only copy of a 602 KB request is the kernel's in writev()).
  struct Chunk {
    std::string own;
    const uint8_t* p = nullptr;   // borrowed when non-null
    size_t len = 0;
  };
  std::deque<Chunk> outq;
  size_t out_off = 0;             // progress within outq.front()
  bool want_out = false;
  uint64_t next_body = 0;
  // results
  std::vector<double>* lat;
  uint64_t* ok;
  uint64_t* err;
  std::string* first_error;
  uint64_t* bytes_sent;
  uint64_t* bytes_recv;
  // continuous mode: completions are logged here (under done_mu) instead
  std::mutex* done_mu = nullptr;
  std::vector<Done>* done = nullptr;
};

ssize_t read_body(nghttp2_session*, int32_t, uint8_t*, size_t length, uint32_t* flags, nghttp2_data_source* src,
                  void*) {
  Req* r = static_cast<Req*>(src->ptr);
  const size_t n = std::min(length, r->body->size() - r->off);
  r->off += n;
  *flags |= NGHTTP2_DATA_FLAG_NO_COPY;     // payload goes out through send_data()
  if (r->off == r->body->size()) *flags |= NGHTTP2_DATA_FLAG_EOF;
  return ssize_t(n);
}

void queue_copy(ClientConn* c, const uint8_t* data, size_t len) {
  if (c->outq.empty() || c->outq.back().p != nullptr || c->outq.back().own.size() > (64u << 10))
    c->outq.emplace_back();
  c->outq.back().own.append(reinterpret_cast<const char*>(data), len);
  c->outq.back().len = c->outq.back().own.size();
}

ssize_t on_send(nghttp2_session*, const uint8_t* data, size_t len, int, void* ud) {
  queue_copy(static_cast<ClientConn*>(ud), data, len);
  return ssize_t(len);
}

int on_send_data(nghttp2_session*, nghttp2_frame*, const uint8_t* framehd, size_t length, nghttp2_data_source* src,
                 void* ud) {
  ClientConn* c = static_cast<ClientConn*>(ud);
  Req* r = static_cast<Req*>(src->ptr);
  queue_copy(c, framehd, 9);
  ClientConn::Chunk ch;
  ch.p = reinterpret_cast<const uint8_t*>(r->body->data()) + r->sent;
  ch.len = length;
  c->outq.push_back(std::move(ch));
  r->sent += length;
  return 0;
}

int on_header(nghttp2_session* s, const nghttp2_frame* f, const uint8_t* name, size_t nl, const uint8_t* value,
              size_t vl, uint8_t, void*) {
  Req* r = static_cast<Req*>(nghttp2_session_get_stream_user_data(s, f->hd.stream_id));
  if (!r) return 0;
  std::string n((const char*)name, nl);
  if (n == ":status") r->http_status = atoi(std::string((const char*)value, vl).c_str());
  else if (n == "grpc-status") r->grpc_status = atoi(std::string((const char*)value, vl).c_str());
  else if (n == "grpc-message") r->grpc_message.assign((const char*)value, vl);
  return 0;
}

int on_data(nghttp2_session* s, uint8_t, int32_t sid, const uint8_t*, size_t len, void*) {
  Req* r = static_cast<Req*>(nghttp2_session_get_stream_user_data(s, sid));
  if (r) r->bytes += len;
  return 0;
}

bool submit_one(ClientConn* c);

// Emit DATA frames as large as the peer allows (its SETTINGS_MAX_FRAME_SIZE and
// the flow-control windows) instead of nghttp2's 16 KB default: a 602 KB
// request becomes 1 frame + 1 copy instead of 38 frames and 38 send() calls.
ssize_t read_length(nghttp2_session*, uint8_t, int32_t, int32_t session_window, int32_t stream_window,
                    uint32_t max_frame, void*) {
  int64_t n = std::min<int64_t>(std::min<int64_t>(session_window, stream_window), max_frame);
  return ssize_t(std::max<int64_t>(n, 1));
}

int on_close(nghttp2_session* s, int32_t sid, uint32_t err, void* ud) {
  ClientConn* c = static_cast<ClientConn*>(ud);
  Req* r = static_cast<Req*>(nghttp2_session_get_stream_user_data(s, sid));
  if (!r) return 0;
  const auto now = Clock::now();
  const double us = std::chrono::duration<double, std::micro>(now - r->t0).count();
  *c->bytes_recv += r->bytes;
  const bool good = err == 0 && r->http_status == 200 && r->grpc_status == 0;
  if (c->sh->continuous.load(std::memory_order_relaxed)) {
    uint64_t seq;
    {
      std::lock_guard<std::mutex> g(*c->done_mu);
      seq = c->sh->finished.fetch_add(1);
      c->done->push_back(Done{seq, us, good, now});
    }
    if (seq + 1 == c->sh->target.load(std::memory_order_acquire)) {
      std::lock_guard<std::mutex> g(c->sh->wmu);
      c->sh->wcv.notify_all();
    }
  }
  if (good) {
    (*c->ok)++;
    if (!c->sh->continuous.load(std::memory_order_relaxed)) c->lat->push_back(us);
  } else {
    (*c->err)++;
    if (c->first_error->empty())
      *c->first_error = "http " + std::to_string(r->http_status) + " grpc-status " + std::to_string(r->grpc_status) +
                        " " + r->grpc_message + (err ? " rst " + std::to_string(err) : "");
  }
  delete r;
  c->inflight--;
  if (!c->sh->continuous.load(std::memory_order_relaxed)) c->sh->finished++;
  submit_one(c);
  return 0;
}

bool submit_one(ClientConn* c) {
  Shared* sh = c->sh;
  if (c->inflight >= c->target) return false;
  if (sh->continuous.load(std::memory_order_relaxed)) {
    if (sh->stopping.load(std::memory_order_relaxed)) return false;
  }
  const uint64_t k = sh->issued.fetch_add(1);
  if (!sh->continuous.load(std::memory_order_relaxed) && k >= sh->total) {
    sh->issued.fetch_sub(1);
    return false;
  }
  Req* r = new Req();
  r->body = &sh->framed[(c->next_body++) % sh->framed.size()];
  r->t0 = Clock::now();
  static const std::string m = ":method", post = "POST", sc = ":scheme", http = "http", pa = ":path",
                           au = ":authority", ct = "content-type", grpc = "application/grpc", te = "te",
                           tr = "trailers";
  nghttp2_nv nv[] = {
      {(uint8_t*)m.data(), (uint8_t*)post.data(), m.size(), post.size(), 0},
      {(uint8_t*)sc.data(), (uint8_t*)http.data(), sc.size(), http.size(), 0},
      {(uint8_t*)pa.data(), (uint8_t*)sh->path.data(), pa.size(), sh->path.size(), 0},
      {(uint8_t*)au.data(), (uint8_t*)sh->authority.data(), au.size(), sh->authority.size(), 0},
      {(uint8_t*)ct.data(), (uint8_t*)grpc.data(), ct.size(), grpc.size(), 0},
      {(uint8_t*)te.data(), (uint8_t*)tr.data(), te.size(), tr.size(), 0},
  };
  nghttp2_data_provider prd;
  prd.source.ptr = r;
  prd.read_callback = read_body;
  int32_t sid = nghttp2_submit_request(c->sess, nullptr, nv, 6, &prd, r);
  if (sid < 0) {
    delete r;
    sh->issued.fetch_sub(1);
    c->dead = true;
    return false;
  }
  *c->bytes_sent += r->body->size();
  c->inflight++;
  return true;
}

int connect_to(const std::string& host, int port) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("cannot resolve " + host);
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
    int e = errno;
    freeaddrinfo(res);
    ::close(fd);
    throw std::runtime_error(std::string("connect failed: ") + strerror(e));
  }
  freeaddrinfo(res);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int sz = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK);
  return fd;
}

bool cflush(ClientConn* c, int ep, uint64_t tag) {
  for (;;) {
    if (c->outq.empty()) {
      if (nghttp2_session_send(c->sess) != 0) return false;   // serialises into outq
      if (c->outq.empty()) break;
    }
    iovec iov[64];
    int cnt = 0;
    size_t off = c->out_off;
    for (auto it = c->outq.begin(); it != c->outq.end() && cnt < 64; ++it, ++cnt) {
      const uint8_t* base = it->p ? it->p : reinterpret_cast<const uint8_t*>(it->own.data());
      iov[cnt].iov_base = const_cast<uint8_t*>(base + off);
      iov[cnt].iov_len = it->len - off;
      off = 0;
    }
    msghdr mh{};
    mh.msg_iov = iov;
    mh.msg_iovlen = size_t(cnt);
    ssize_t n = sendmsg(c->fd, &mh, MSG_NOSIGNAL);
    if (n < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      return false;
    }
    size_t left = size_t(n);
    while (left > 0 && !c->outq.empty()) {
      const size_t avail = c->outq.front().len - c->out_off;
      if (left >= avail) {
        left -= avail;
        c->outq.pop_front();
        c->out_off = 0;
      } else {
        c->out_off += left;
        left = 0;
      }
    }
  }
  const bool pending = !c->outq.empty();
  if (pending != c->want_out) {
    epoll_event ev{};
    ev.events = EPOLLIN | (pending ? EPOLLOUT : 0);
    ev.data.u64 = tag;
    epoll_ctl(ep, EPOLL_CTL_MOD, c->fd, &ev);
    c->want_out = pending;
  }
  return true;
}

nghttp2_session_callbacks* make_callbacks() {
  nghttp2_session_callbacks* cbs;
  nghttp2_session_callbacks_new(&cbs);
  nghttp2_session_callbacks_set_on_header_callback(cbs, on_header);
  nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs, on_data);
  nghttp2_session_callbacks_set_on_stream_close_callback(cbs, on_close);
  nghttp2_session_callbacks_set_data_source_read_length_callback(cbs, read_length);
  nghttp2_session_callbacks_set_send_callback(cbs, on_send);
  nghttp2_session_callbacks_set_send_data_callback(cbs, on_send_data);
  return cbs;
}

}  // namespace

// One client thread's connections (HTTP/2 sessions + epoll set); they persist
// across LoadGen::run() calls like a real client's channel does.
struct LoadGen::Worker {
  int ep = -1;
  std::vector<std::unique_ptr<ClientConn>> conns;
  LoadGenResult part;
  std::string connect_error;
  std::mutex done_mu;
  std::vector<Done> done;   // continuous mode completions not yet consumed by a window
  ~Worker() {
    for (auto& c : conns) {
      if (c->sess) nghttp2_session_del(c->sess);
      if (c->fd >= 0) ::close(c->fd);
    }
    if (ep >= 0) ::close(ep);
  }
};

LoadGen::LoadGen(const std::string& host, int port, const std::string& method,
                 const std::vector<std::string>& bodies, int concurrency, int connections, int threads) {
  if (bodies.empty()) throw std::invalid_argument("no request bodies");
  auto shp = std::make_shared<Shared>();
  sh_ = shp;
  Shared* sh = shp.get();
  sh->path = method;
  sh->authority = host + ":" + std::to_string(port);
  for (auto& b : bodies) {
    std::string f(5 + b.size(), '\0');
    grpc_frame_header(reinterpret_cast<uint8_t*>(&f[0]), uint32_t(b.size()));
    memcpy(&f[5], b.data(), b.size());
    sh->framed.push_back(std::move(f));
  }
  cbs_ = make_callbacks();
  threads = std::max(1, std::min(threads, connections));
  connections = std::max(connections, threads);
  const int per_conn = std::max(1, concurrency / connections);
  for (int t = 0; t < threads; ++t) {
    auto w = std::make_unique<Worker>();
    w->ep = epoll_create1(0);
    const int nconn = connections / threads + (t < connections % threads ? 1 : 0);
    for (int i = 0; i < nconn; ++i) {
      auto c = std::make_unique<ClientConn>();
      try {
        c->fd = connect_to(host, port);
      } catch (const std::exception& e) {
        if (w->connect_error.empty()) w->connect_error = e.what();
        continue;
      }
      c->sh = sh;
      c->target = per_conn;
      c->next_body = uint64_t(t * 131 + i) * 7919;
      nghttp2_session_client_new(&c->sess, static_cast<nghttp2_session_callbacks*>(cbs_), c.get());
      nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS, 4096},
                                     {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 16u << 20}};
      nghttp2_submit_settings(c->sess, NGHTTP2_FLAG_NONE, iv, 2);
      nghttp2_session_set_local_window_size(c->sess, NGHTTP2_FLAG_NONE, 0, 1 << 30);
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.u64 = w->conns.size();
      epoll_ctl(w->ep, EPOLL_CTL_ADD, c->fd, &ev);
      w->conns.push_back(std::move(c));
    }
    workers_.push_back(std::move(w));
  }
}

LoadGen::~LoadGen() {
  if (!threads_.empty()) stop(10.0);
  workers_.clear();
  if (cbs_) nghttp2_session_callbacks_del(static_cast<nghttp2_session_callbacks*>(cbs_));
}

namespace {

void worker_loop(LoadGen::Worker* w, Shared* sh) {
  LoadGenResult* out = &w->part;
  if (!w->connect_error.empty()) {
    out->first_error = w->connect_error;
    out->errors++;
  }
  auto& conns = w->conns;
  for (auto& c : conns) {
    c->lat = &out->latency_us;
    c->ok = &out->ok;
    c->err = &out->errors;
    c->first_error = &out->first_error;
    c->bytes_sent = &out->bytes_sent;
    c->bytes_recv = &out->bytes_recv;
    c->done_mu = &w->done_mu;
    c->done = &w->done;
  }
  for (size_t i = 0; i < conns.size(); ++i) {
    if (conns[i]->dead) continue;
    while (submit_one(conns[i].get())) {}
    if (!cflush(conns[i].get(), w->ep, i)) conns[i]->dead = true;
  }
  std::vector<uint8_t> rbuf(1 << 20);
  std::vector<epoll_event> evs(64);
  for (;;) {
    bool any_live = false;
    for (auto& c : conns)
      if (!c->dead && (c->inflight > 0)) any_live = true;
    if (!any_live) break;
    if ((!sh->continuous.load(std::memory_order_relaxed) || sh->stopping.load(std::memory_order_acquire)) &&
        Clock::now() > sh->deadline) {
      if (out->first_error.empty()) out->first_error = "load generator timed out";
      break;
    }
    int n = epoll_wait(w->ep, evs.data(), int(evs.size()), 100);
    for (int i = 0; i < n; ++i) {
      const uint64_t idx = evs[i].data.u64;
      ClientConn* c = conns[idx].get();
      if (c->dead) continue;
      if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
        for (;;) {
          ssize_t r = recv(c->fd, rbuf.data(), rbuf.size(), 0);
          if (r > 0) {
            if (nghttp2_session_mem_recv(c->sess, rbuf.data(), size_t(r)) < 0) { c->dead = true; break; }
            if (size_t(r) < rbuf.size()) break;
            continue;
          }
          if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) c->dead = true;
          break;
        }
      }
      if (!c->dead && !cflush(c, w->ep, idx)) c->dead = true;
      if (c->dead && out->first_error.empty()) out->first_error = "connection lost";
    }
  }
  for (auto& c : conns) {
    if (c->dead && c->inflight > 0) {   // requests lost with a dead connection
      out->errors += uint64_t(c->inflight);
      c->inflight = 0;
    }
  }
}

}  // namespace

LoadGenResult LoadGen::run(uint64_t total, double timeout_s) {
  Shared* sh = static_cast<Shared*>(sh_.get());
  if (!threads_.empty()) throw std::logic_error("LoadGen::run while a continuous run is active (stop() first)");
  sh->continuous = false;
  sh->total = total;
  sh->issued = 0;
  sh->finished = 0;
  sh->deadline = Clock::now() + std::chrono::microseconds(int64_t(timeout_s * 1e6));
  std::vector<std::thread> ts;
  const auto t0 = Clock::now();
  for (auto& wp : workers_) {
    wp->part = LoadGenResult();
    LoadGen::Worker* w = wp.get();
    ts.emplace_back([w, sh] {
      pthread_setname_np(pthread_self(), "tfs-loadgen");
      timespec a{}, b{};
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &a);
      worker_loop(w, sh);
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &b);
      w->part.cpu_s = double(b.tv_sec - a.tv_sec) + 1e-9 * double(b.tv_nsec - a.tv_nsec);
    });
  }
  for (auto& t : ts) t.join();
  LoadGenResult res;
  res.elapsed_s = std::chrono::duration<double>(Clock::now() - t0).count();
  for (auto& w : workers_) {
    const LoadGenResult& p = w->part;
    res.ok += p.ok;
    res.errors += p.errors;
    res.bytes_sent += p.bytes_sent;
    res.bytes_recv += p.bytes_recv;
    res.cpu_s += p.cpu_s;
    res.latency_us.insert(res.latency_us.end(), p.latency_us.begin(), p.latency_us.end());
    if (res.first_error.empty()) res.first_error = p.first_error;
  }
  return res;
}

void LoadGen::start() {
  Shared* sh = static_cast<Shared*>(sh_.get());
  if (!threads_.empty()) return;
  sh->continuous = true;
  sh->stopping = false;
  sh->issued = 0;
  sh->finished = 0;
  for (auto& wp : workers_) {
    wp->part = LoadGenResult();
    {
      std::lock_guard<std::mutex> g(wp->done_mu);
      wp->done.clear();
    }
    LoadGen::Worker* w = wp.get();
    threads_.emplace_back([w, sh] {
      pthread_setname_np(pthread_self(), "tfs-loadgen");
      timespec a{}, b{};
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &a);
      worker_loop(w, sh);
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &b);
      w->part.cpu_s = double(b.tv_sec - a.tv_sec) + 1e-9 * double(b.tv_nsec - a.tv_nsec);
    });
  }
}

uint64_t LoadGen::completed() const {
  return static_cast<Shared*>(sh_.get())->finished.load();
}

LoadGenResult LoadGen::window(uint64_t n, double timeout_s) {
  Shared* sh = static_cast<Shared*>(sh_.get());
  if (threads_.empty()) throw std::logic_error("LoadGen::window needs start()");
  LoadGenResult res;
  const uint64_t s0 = sh->finished.load();
  const auto t0 = Clock::now();
  const auto deadline = t0 + std::chrono::microseconds(int64_t(timeout_s * 1e6));
  // drop completions older than the window so the logs stay bounded
  for (auto& w : workers_) {
    std::lock_guard<std::mutex> g(w->done_mu);
    w->done.erase(std::remove_if(w->done.begin(), w->done.end(), [&](const Done& d) { return d.seq < s0; }),
                  w->done.end());
  }
  // the window ends at the completion with sequence number s0 + n - 1
  sh->target.store(s0 + n, std::memory_order_release);
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(sh->wmu);
      sh->wcv.wait_for(lk, std::chrono::milliseconds(2), [&] { return sh->finished.load() >= s0 + n; });
    }
    if (sh->finished.load() >= s0 + n) break;
    if (Clock::now() > deadline) {
      res.first_error = "load generator window timed out";
      break;
    }
    bool alive = false;
    for (auto& w : workers_)
      for (auto& c : w->conns)
        if (!c->dead) alive = true;
    if (!alive) {
      res.first_error = "every connection was lost";
      break;
    }
  }
  sh->target.store(~uint64_t(0), std::memory_order_release);
  res.elapsed_s = std::chrono::duration<double>(Clock::now() - t0).count();
  for (auto& w : workers_) {
    std::lock_guard<std::mutex> g(w->done_mu);
    for (auto& d : w->done) {
      if (d.seq < s0 || d.seq >= s0 + n) continue;
      res.done_s.push_back(std::chrono::duration<double>(d.at - t0).count());
      if (d.ok) {
        res.ok++;
        res.latency_us.push_back(d.us);
      } else {
        res.errors++;
      }
    }
  }
  if (res.first_error.empty() && res.errors)
    for (auto& w : workers_)
      if (!w->part.first_error.empty()) {
        res.first_error = w->part.first_error;
        break;
      }
  return res;
}

LoadGenResult LoadGen::stop(double timeout_s) {
  Shared* sh = static_cast<Shared*>(sh_.get());
  LoadGenResult res;
  if (threads_.empty()) return res;
  sh->deadline = Clock::now() + std::chrono::microseconds(int64_t(timeout_s * 1e6));
  sh->stopping.store(true, std::memory_order_release);   // no new submissions; workers drain and exit
  for (auto& t : threads_) t.join();
  threads_.clear();
  sh->continuous = false;
  for (auto& w : workers_) {
    const LoadGenResult& p = w->part;
    res.ok += p.ok;
    res.errors += p.errors;
    res.bytes_sent += p.bytes_sent;
    res.bytes_recv += p.bytes_recv;
    res.cpu_s += p.cpu_s;
    if (res.first_error.empty()) res.first_error = p.first_error;
  }
  return res;
}

LoadGenResult run_loadgen(const std::string& host, int port, const std::string& method,
                          const std::vector<std::string>& bodies, uint64_t total, int concurrency, int connections,
                          int threads, double timeout_s) {
  LoadGen lg(host, port, method, bodies, concurrency, connections, threads);
  return lg.run(total, timeout_s);
}

}  // namespace tfs
