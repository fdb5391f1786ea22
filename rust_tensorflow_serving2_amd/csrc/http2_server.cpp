// gRPC/HTTP2 server: epoll IO threads + libnghttp2 sessions (see http2.h).
#include <pthread.h>
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

#include "http2.h"
#include "nghttp2_min.h"
#include "router.h"

namespace tfs {

namespace {

constexpr size_t kReadBuf = 1 << 20;
constexpr uint64_t kListenTag = 0;
constexpr uint64_t kWakeTag = 1;

void set_nonblock(int fd) {
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
}

nghttp2_nv make_nv(const std::string& n, const std::string& v) {
  return nghttp2_nv{(uint8_t*)n.data(), (uint8_t*)v.data(), n.size(), v.size(), NGHTTP2_NV_FLAG_NONE};
}

// grpc-message percent encoding (gRPC HTTP/2 spec)
std::string pct_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  out.reserve(s.size());
  for (unsigned char c : s) {
    if (c >= 0x20 && c <= 0x7e && c != '%') {
      out.push_back(char(c));
    } else {
      out.push_back('%');
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 15]);
    }
  }
  return out;
}

int64_t parse_grpc_timeout(const std::string& v) {
  if (v.size() < 2) return 0;
  int64_t n = 0;
  for (size_t i = 0; i + 1 < v.size(); ++i) {
    if (v[i] < '0' || v[i] > '9') return 0;
    n = n * 10 + (v[i] - '0');
  }
  switch (v.back()) {
    case 'H': return n * 3600LL * 1000000;
    case 'M': return n * 60LL * 1000000;
    case 'S': return n * 1000000;
    case 'm': return n * 1000;
    case 'u': return n;
    case 'n': return n / 1000;
    default: return 0;
  }
}

enum StreamMode : int { kProbeMode = 0, kBufferMode = 1, kStreamMode = 2 };
constexpr size_t kProbeMax = 4096;          // header bytes inspected before giving up on streaming
constexpr size_t kStreamMin = 64 << 10;     // payloads smaller than this are simply buffered
static const char* const kPredictMethod = "/tensorflow.serving.PredictionService/Predict";

struct Stream {
  int32_t id = 0;
  std::string path;
  std::string body;          // raw DATA (with gRPC prefix); in stream mode only the header
  int64_t timeout_us = 0;
  bool bad_content_type = false;
  // streaming decode (Predict payload copied straight into a batch slot)
  int mode = kProbeMode;
  std::shared_ptr<StreamRes> sres;
  bool committed = false;
  bool overflow = false;     // bytes beyond the gRPC message
  // response
  std::string resp;          // gRPC-framed message
  size_t resp_off = 0;
  bool responding = false;
  ~Stream() {
    if (sres && !committed) sres->abandon();   // reset / connection lost mid-payload
  }
};

struct Outgoing {
  uint64_t conn_id;
  int32_t stream_id;
  int status;
  std::string message;
  std::string body;
};

}  // namespace

// Frame boundaries of the inbound byte stream, tracked alongside nghttp2 so a
// recv() can stop exactly where a DATA payload starts: the payload of a
// streaming Predict then goes from the socket straight into its pinned batch
// row (one kernel->user copy, no pass through the read buffer).
struct FrameTrack {
  size_t preface = 24;      // client connection preface still to pass
  uint8_t hdr[9];
  int hlen = 0;             // bytes of a partial frame header seen
  bool in_payload = false;
  size_t remain = 0;        // payload bytes left in the current frame
  uint8_t type = 0, flags = 0;
  int32_t sid = 0;
  void advance(const uint8_t* p, size_t n) {
    while (n) {
      size_t k;
      if (preface) {
        k = std::min(preface, n);
        preface -= k;
      } else if (in_payload) {
        k = std::min(remain, n);
        remain -= k;
        in_payload = remain != 0;
      } else {
        k = std::min<size_t>(size_t(9 - hlen), n);
        memcpy(hdr + hlen, p, k);
        hlen += int(k);
        if (hlen == 9) {
          hlen = 0;
          remain = (size_t(hdr[0]) << 16) | (size_t(hdr[1]) << 8) | hdr[2];
          type = hdr[3];
          flags = hdr[4];
          sid = int32_t(((uint32_t(hdr[5]) << 24) | (uint32_t(hdr[6]) << 16) | (uint32_t(hdr[7]) << 8) | hdr[8]) &
                        0x7fffffffu);
          in_payload = remain != 0;
        }
      }
      p += k;
      n -= k;
    }
  }
  // bytes up to the end of the next frame header
  size_t to_next_payload() const {
    if (preface) return preface + 9;
    if (in_payload) return remain + 9;
    return size_t(9 - hlen);
  }
};

struct Conn {
  FrameTrack ft;
  int fd = -1;
  uint64_t id = 0;
  nghttp2_session* sess = nullptr;
  std::unordered_map<int32_t, std::unique_ptr<Stream>> streams;
  std::string wbuf;
  size_t wpos = 0;
  bool want_out = false;
  bool dead = false;
};

class IoThread {
 public:
  IoThread(Server* srv, int index, const std::string& host, int port, bool listener)
      : srv_(srv), index_(index), port_(port) {
    if (listener) open_listener(host, port);   // may throw: nothing else is allocated yet
    ep_ = epoll_create1(0);
    wake_ = eventfd(0, EFD_NONBLOCK);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = kWakeTag;
    epoll_ctl(ep_, EPOLL_CTL_ADD, wake_, &ev);
    if (lfd_ >= 0) {
      ev.data.u64 = kListenTag;
      epoll_ctl(ep_, EPOLL_CTL_ADD, lfd_, &ev);
    }
    rbuf_.resize(kReadBuf);
    init_callbacks();
  }

  // The process's one listening socket (IO thread 0): SO_REUSEPORT so GPU
  // replicas (processes) share the port; other IO threads get connections
  // from it through adopt().
  void open_listener(const std::string& host, int port) {
    lfd_ = socket(AF_INET, SOCK_STREAM, 0);
    if (lfd_ < 0) throw std::runtime_error("socket() failed");
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_port = htons(uint16_t(port));
    if (host.empty() || host == "0.0.0.0" || host == "[::]" || host == "::") {
      addr.sin_addr.s_addr = htonl(INADDR_ANY);
    } else if (host == "localhost") {
      addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    } else if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) {
      ::close(lfd_);
      throw std::runtime_error("bad IPv4 host " + host);
    }
    if (bind(lfd_, (sockaddr*)&addr, sizeof(addr)) != 0) {
      int e = errno;
      ::close(lfd_);
      throw std::runtime_error(std::string("bind failed: ") + strerror(e));
    }
    if (listen(lfd_, 1024) != 0) {
      ::close(lfd_);
      throw std::runtime_error("listen failed");
    }
    socklen_t len = sizeof(addr);
    getsockname(lfd_, (sockaddr*)&addr, &len);
    port_ = ntohs(addr.sin_port);
    set_nonblock(lfd_);
  }

  void init_callbacks() {
    nghttp2_session_callbacks_new(&cbs_);
    nghttp2_session_callbacks_set_on_begin_headers_callback(cbs_, &IoThread::on_begin_headers);
    nghttp2_session_callbacks_set_on_header_callback(cbs_, &IoThread::on_header);
    nghttp2_session_callbacks_set_on_frame_recv_callback(cbs_, &IoThread::on_frame_recv);
    nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs_, &IoThread::on_data_chunk);
    nghttp2_session_callbacks_set_on_stream_close_callback(cbs_, &IoThread::on_stream_close);
    nghttp2_session_callbacks_set_data_source_read_length_callback(cbs_, &IoThread::read_length);
  }

  ~IoThread() {
    stop();
    for (auto& kv : conns_) close_conn(kv.second.get(), false);
    conns_.clear();
    for (int fd : adopt_) ::close(fd);
    if (cbs_) nghttp2_session_callbacks_del(cbs_);
    if (lfd_ >= 0) ::close(lfd_);
    if (ep_ >= 0) ::close(ep_);
    if (wake_ >= 0) ::close(wake_);
  }

  int port() const { return port_; }
  int live_connections() const { return nconns_.load(std::memory_order_relaxed); }

  // A connection accepted by the acceptor thread, registered on this thread's
  // epoll set by this thread (its loop's wake-up adopts it).
  void adopt(int fd) {
    nconns_.fetch_add(1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(amu_);
      adopt_.push_back(fd);
    }
    uint64_t one = 1;
    (void)!write(wake_, &one, sizeof(one));
  }

  void start() {
    running_ = true;
    th_ = std::thread([this] {
      pthread_setname_np(pthread_self(), "tfs-h2io");
      loop();
    });
  }

  void stop() {
    if (!running_.exchange(false)) return;
    uint64_t one = 1;
    (void)!write(wake_, &one, sizeof(one));
    if (th_.joinable()) th_.join();
  }

  void post(Outgoing&& o) {
    {
      std::lock_guard<std::mutex> g(omu_);
      outbox_.push_back(std::move(o));
    }
    uint64_t one = 1;
    (void)!write(wake_, &one, sizeof(one));
  }

 private:
  // ------------------------------------------------------------ nghttp2 callbacks
  static int on_begin_headers(nghttp2_session* s, const nghttp2_frame* f, void* ud) {
    Conn* c = static_cast<Conn*>(ud);
    if (f->hd.type != NGHTTP2_HEADERS) return 0;
    if (c->streams.count(f->hd.stream_id)) return 0;   // trailers
    auto st = std::make_unique<Stream>();
    st->id = f->hd.stream_id;
    nghttp2_session_set_stream_user_data(s, f->hd.stream_id, st.get());
    c->streams.emplace(f->hd.stream_id, std::move(st));
    return 0;
  }

  static int on_header(nghttp2_session* s, const nghttp2_frame* f, const uint8_t* name, size_t namelen,
                       const uint8_t* value, size_t valuelen, uint8_t, void*) {
    Stream* st = static_cast<Stream*>(nghttp2_session_get_stream_user_data(s, f->hd.stream_id));
    if (!st) return 0;
    std::string n((const char*)name, namelen);
    if (n == ":path") {
      st->path.assign((const char*)value, valuelen);
    } else if (n == "grpc-timeout") {
      st->timeout_us = parse_grpc_timeout(std::string((const char*)value, valuelen));
    } else if (n == "content-type") {
      std::string v((const char*)value, valuelen);
      st->bad_content_type = v.rfind("application/grpc", 0) != 0;
    }
    return 0;
  }

  // large responses go out in frames as big as the peer allows (not 16 KB)
  static ssize_t read_length(nghttp2_session*, uint8_t, int32_t, int32_t session_window, int32_t stream_window,
                             uint32_t max_frame, void*) {
    int64_t n = std::min<int64_t>(std::min<int64_t>(session_window, stream_window), max_frame);
    return ssize_t(std::max<int64_t>(n, 1));
  }

  static int on_data_chunk(nghttp2_session* s, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud) {
    Conn* c = static_cast<Conn*>(ud);
    Stream* st = static_cast<Stream*>(nghttp2_session_get_stream_user_data(s, sid));
    if (!st) return 0;
    IoThread* self = tls_self_;
    if (st->mode == kStreamMode) {
      StreamRes* r = st->sres.get();
      const size_t n = std::min(len, r->len - r->got);
      if (n) r->write(data, n);
      if (len > n) st->overflow = true;
      return 0;
    }
    if (st->mode == kProbeMode) {
      if (st->path != kPredictMethod || !(self->srv_->stream_reserve() || self->srv_->router())) {
        st->mode = kBufferMode;
      } else {
        const size_t before = st->body.size();
        const size_t take = std::min(len, kProbeMax - before);
        st->body.append((const char*)data, take);
        ProbeInfo pi;
        Probe pr = probe_predict_header((const uint8_t*)st->body.data(), st->body.size(), kStreamMin, pi);
        if (pr == Probe::kFound) {
          std::shared_ptr<StreamRes> res =
              self->srv_->reserve_stream(pi, (const uint8_t*)st->body.data(), st->body.size(), st->path);
          if (res) {
            // payload = framed-message bytes [payload_off, payload_off + len): part may sit in
            // the header buffer, the rest in this chunk (data[take..] is message offset before+take..)
            size_t pos = pi.payload_off;
            const size_t body_end = before + take;
            if (pos < body_end) {
              res->write((const uint8_t*)st->body.data() + pos, body_end - pos);
              pos = body_end;
            }
            const size_t seen = before + len;
            if (pos < seen) {
              const size_t n = std::min(seen - pos, res->len - res->got);
              res->write(data + (pos - before), n);
              if (seen - pos > n) st->overflow = true;
            }
            st->body.resize(pi.payload_off);
            st->sres = std::move(res);
            st->mode = kStreamMode;
            return 0;
          }
          pr = Probe::kNoStream;
        }
        if (pr == Probe::kNeedMore && take == len && st->body.size() < kProbeMax) return 0;
        st->mode = kBufferMode;     // not streamable: buffer the rest as usual
        data += take;
        len -= take;
      }
    }
    if (st->body.size() < 5 && st->body.size() + len >= 5) {
      std::string hdr = st->body;
      hdr.append((const char*)data, 5 - st->body.size());
      const uint8_t* h = (const uint8_t*)hdr.data();
      const uint32_t msg = (uint32_t(h[1]) << 24) | (uint32_t(h[2]) << 16) | (uint32_t(h[3]) << 8) | h[4];
      if (msg <= self->srv_->max_message()) st->body.reserve(size_t(msg) + 5);
    } else if (st->body.size() >= 5 && st->body.capacity() < 4096 + kProbeMax) {
      const uint8_t* h = (const uint8_t*)st->body.data();
      const uint32_t msg = (uint32_t(h[1]) << 24) | (uint32_t(h[2]) << 16) | (uint32_t(h[3]) << 8) | h[4];
      if (msg <= self->srv_->max_message()) st->body.reserve(size_t(msg) + 5);
    }
    if (st->body.size() + len > self->srv_->max_message() + 5) {
      nghttp2_submit_rst_stream(s, NGHTTP2_FLAG_NONE, sid, NGHTTP2_CANCEL);
      return 0;
    }
    st->body.append((const char*)data, len);
    (void)c;
    return 0;
  }

  static int on_frame_recv(nghttp2_session* s, const nghttp2_frame* f, void* ud) {
    Conn* c = static_cast<Conn*>(ud);
    if ((f->hd.type == NGHTTP2_DATA || f->hd.type == NGHTTP2_HEADERS) && (f->hd.flags & NGHTTP2_FLAG_END_STREAM)) {
      auto it = c->streams.find(f->hd.stream_id);
      if (it == c->streams.end()) return 0;
      tls_self_->request_done(c, it->second.get());
    }
    (void)s;
    return 0;
  }

  static int on_stream_close(nghttp2_session*, int32_t sid, uint32_t, void* ud) {
    Conn* c = static_cast<Conn*>(ud);
    c->streams.erase(sid);
    return 0;
  }

  static ssize_t read_resp(nghttp2_session* s, int32_t sid, uint8_t* buf, size_t length, uint32_t* flags,
                           nghttp2_data_source* src, void*) {
    Stream* st = static_cast<Stream*>(src->ptr);
    const size_t n = std::min(length, st->resp.size() - st->resp_off);
    memcpy(buf, st->resp.data() + st->resp_off, n);
    st->resp_off += n;
    if (st->resp_off == st->resp.size()) {
      *flags |= NGHTTP2_DATA_FLAG_EOF | NGHTTP2_DATA_FLAG_NO_END_STREAM;
      static const std::string k_status = "grpc-status", k_zero = "0";
      nghttp2_nv tr[] = {make_nv(k_status, k_zero)};
      nghttp2_submit_trailer(s, sid, tr, 1);
      std::string().swap(st->resp);
      st->resp_off = 0;
    }
    return ssize_t(n);
  }

  // ------------------------------------------------------------ request / response
  void request_done(Conn* c, Stream* st) {
    if (st->mode == kStreamMode) {
      StreamRes* r = st->sres.get();
      if (st->bad_content_type || r->got != r->len || st->overflow) {
        r->abandon();
        st->committed = true;   // nothing left to abandon
        answer(c, st, 13 /*INTERNAL*/,
               st->bad_content_type ? "unsupported content-type (expected application/grpc)"
                                    : "gRPC message length mismatch (streaming calls are not supported)",
               std::string());
        return;
      }
      auto call = std::make_unique<Call>();
      call->conn_id = c->id;
      call->io_index = index_;
      call->stream_id = st->id;
      call->method = st->path;
      call->arrival = Clock::now();
      call->timeout_us = st->timeout_us;
      if (!r->remote()) srv_->count(*call);   // a remote row counts in its replica's load
      srv_->stats.requests++;
      srv_->stats.fast_path++;
      srv_->stats.streamed++;
      srv_->stats.bytes_in += st->body.size() - 5 + r->len;
      st->committed = true;
      if (r->keep_header()) call->head = std::move(st->body);
      std::string().swap(st->body);
      r->commit(std::move(call));
      return;
    }
    if (st->bad_content_type) {
      answer(c, st, 13 /*INTERNAL*/, "unsupported content-type (expected application/grpc)", std::string());
      return;
    }
    if (st->body.size() < 5) {
      answer(c, st, 13, "missing gRPC message", std::string());
      return;
    }
    const uint8_t* d = (const uint8_t*)st->body.data();
    if (d[0] != 0) {
      answer(c, st, 12 /*UNIMPLEMENTED*/, "compressed gRPC messages are not supported", std::string());
      return;
    }
    const uint32_t len = (uint32_t(d[1]) << 24) | (uint32_t(d[2]) << 16) | (uint32_t(d[3]) << 8) | d[4];
    if (size_t(len) + 5 != st->body.size()) {
      answer(c, st, 13, "gRPC message length mismatch (streaming calls are not supported)", std::string());
      return;
    }
    auto call = std::make_unique<Call>();
    call->conn_id = c->id;
    call->io_index = index_;
    call->stream_id = st->id;
    call->method = st->path;
    call->body = std::move(st->body);   // no copy: the prefix is skipped via `off`
    call->off = 5;
    std::string().swap(st->body);
    call->arrival = Clock::now();
    call->timeout_us = st->timeout_us;
    srv_->stats.requests++;
    srv_->stats.bytes_in += call->size();
    srv_->dispatch(std::move(call));
  }

  void answer(Conn* c, Stream* st, int status, const std::string& msg, std::string body) {
    static const std::string k_st = ":status", k_200 = "200", k_ct = "content-type", k_grpc = "application/grpc",
                             k_gs = "grpc-status", k_gm = "grpc-message";
    if (st->responding) return;
    st->responding = true;
    srv_->stats.responses++;
    if (status == 0) {
      st->resp.resize(5 + body.size());
      const uint32_t n = uint32_t(body.size());
      st->resp[0] = 0;
      st->resp[1] = char(n >> 24); st->resp[2] = char(n >> 16); st->resp[3] = char(n >> 8); st->resp[4] = char(n);
      memcpy(&st->resp[5], body.data(), body.size());
      srv_->stats.bytes_out += body.size();
      st->resp_off = 0;
      nghttp2_nv hdr[] = {make_nv(k_st, k_200), make_nv(k_ct, k_grpc)};
      nghttp2_data_provider prd;
      prd.source.ptr = st;
      prd.read_callback = &IoThread::read_resp;
      nghttp2_submit_response(c->sess, st->id, hdr, 2, &prd);
    } else {
      srv_->stats.errors++;
      const std::string code = std::to_string(status);
      const std::string m = pct_encode(msg);
      nghttp2_nv hdr[] = {make_nv(k_st, k_200), make_nv(k_ct, k_grpc), make_nv(k_gs, code), make_nv(k_gm, m)};
      nghttp2_submit_response(c->sess, st->id, hdr, 4, nullptr);   // trailers-only
    }
  }

  // ------------------------------------------------------------ loop
  void accept_all() {
    for (;;) {
      int fd = accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      IoThread* t = srv_->pick_io();
      if (t != this) {
        t->adopt(fd);
        continue;
      }
      nconns_.fetch_add(1, std::memory_order_relaxed);
      add_conn(fd);
    }
  }

  void adopt_pending() {
    std::vector<int> fds;
    {
      std::lock_guard<std::mutex> g(amu_);
      fds.swap(adopt_);
    }
    for (int fd : fds) add_conn(fd);
  }

  void add_conn(int fd) {
    {
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      int sz = 4 << 20;
      setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
      setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->id = (uint64_t(index_) << 48) | (++next_id_);
      nghttp2_session_server_new(&c->sess, cbs_, c.get());
      nghttp2_settings_entry iv[] = {
          {NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS, 4096},
          {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 16u << 20},
          {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1u << 20},
      };
      nghttp2_submit_settings(c->sess, NGHTTP2_FLAG_NONE, iv, 3);
      nghttp2_session_set_local_window_size(c->sess, NGHTTP2_FLAG_NONE, 0, 1 << 30);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c->id;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
      srv_->stats.connections++;
      Conn* raw = c.get();
      conns_.emplace(c->id, std::move(c));
      flush(raw);
    }
  }

  void close_conn(Conn* c, bool erase) {
    if (c->fd >= 0) {
      epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
      ::close(c->fd);
      c->fd = -1;
      nconns_.fetch_sub(1, std::memory_order_relaxed);
    }
    if (c->sess) {
      nghttp2_session_del(c->sess);
      c->sess = nullptr;
    }
    c->streams.clear();
    if (erase) conns_.erase(c->id);
  }

  bool flush(Conn* c) {
    for (;;) {
      if (c->wpos < c->wbuf.size()) {
        ssize_t n = send(c->fd, c->wbuf.data() + c->wpos, c->wbuf.size() - c->wpos, MSG_NOSIGNAL);
        if (n < 0) {
          if (errno == EAGAIN || errno == EWOULDBLOCK) break;
          return false;
        }
        c->wpos += size_t(n);
        continue;
      }
      c->wbuf.clear();
      c->wpos = 0;
      const uint8_t* data;
      ssize_t n = nghttp2_session_mem_send(c->sess, &data);
      if (n < 0) return false;
      if (n == 0) break;
      // try a direct send first to avoid a copy
      ssize_t w = send(c->fd, data, size_t(n), MSG_NOSIGNAL);
      if (w < 0) {
        if (errno != EAGAIN && errno != EWOULDBLOCK) return false;
        w = 0;
      }
      if (w < n) c->wbuf.assign((const char*)data + w, size_t(n - w));
    }
    const bool pending = c->wpos < c->wbuf.size();
    if (pending != c->want_out) {
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP | (pending ? EPOLLOUT : 0);
      ev.data.u64 = c->id;
      epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &ev);
      c->want_out = pending;
    }
    if (!pending && !nghttp2_session_want_read(c->sess) && !nghttp2_session_want_write(c->sess)) return false;
    return true;
  }

  // Where the next recv() lands: normally the read buffer, but only up to the
  // end of the next frame header; inside the DATA payload of a streaming
  // Predict, straight into the request's batch row (the row's `writers` count
  // is held across the syscall so the batcher cannot hand the row to another
  // request meanwhile).
  uint8_t* recv_target(Conn* c, size_t& want, StreamRes*& held) {
    FrameTrack& ft = c->ft;
    held = nullptr;
    if (ft.in_payload && ft.type == 0 /*DATA*/ && !(ft.flags & 0x8 /*PADDED*/)) {
      auto it = c->streams.find(ft.sid);
      Stream* st = it == c->streams.end() ? nullptr : it->second.get();
      if (st && st->mode == kStreamMode && !st->overflow && st->sres) {
        StreamRes* r = st->sres.get();
        const size_t room = r->len - r->got;
        if (room && !r->conv) {   // (a converting row takes its bytes through write())
          r->writers.fetch_add(1);
          if (r->state.load() == 0) {
            held = r;
            want = std::min(ft.remain, room);
            srv_->stats.direct_bytes += want;
            return r->dst + r->got;
          }
          r->writers.fetch_sub(1);
        }
      }
      if (st && st->mode == kProbeMode) {   // the Predict header: probe, then stream the rest
        want = std::min(ft.remain, kProbeMax);
        return rbuf_.data();
      }
    }
    want = std::min(rbuf_.size(), ft.to_next_payload());
    return rbuf_.data();
  }

  void on_readable(Conn* c) {
    for (;;) {
      const auto t0 = Clock::now();
      size_t want = 0;
      StreamRes* held = nullptr;
      uint8_t* buf = recv_target(c, want, held);
      ssize_t n = recv(c->fd, buf, want, 0);
      if (held) held->writers.fetch_sub(1);
      const auto t1 = Clock::now();
      srv_->stats.ns_recv += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
      if (n > 0) {
        srv_->stats.recv_calls.fetch_add(1, std::memory_order_relaxed);
        srv_->stats.recv_bytes.fetch_add(uint64_t(n), std::memory_order_relaxed);
        c->ft.advance(buf, size_t(n));
        ssize_t r = nghttp2_session_mem_recv(c->sess, buf, size_t(n));
        srv_->stats.ns_h2 +=
            uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t1).count());
        if (r < 0) {
          c->dead = true;
          return;
        }
        if (size_t(n) < want) break;   // socket drained
        continue;
      }
      if (n == 0) {
        c->dead = true;
        return;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        srv_->stats.recv_empty.fetch_add(1, std::memory_order_relaxed);
        break;
      }
      c->dead = true;
      return;
    }
  }

  void drain_outbox() {
    std::vector<Outgoing> items;
    {
      std::lock_guard<std::mutex> g(omu_);
      items.swap(outbox_);
    }
    std::vector<Conn*> touched;
    for (auto& o : items) {
      auto it = conns_.find(o.conn_id);
      if (it == conns_.end()) continue;
      Conn* c = it->second.get();
      auto st = c->streams.find(o.stream_id);
      if (st == c->streams.end()) continue;     // client went away
      answer(c, st->second.get(), o.status, o.message, std::move(o.body));
      touched.push_back(c);
    }
    for (Conn* c : touched)
      if (c->fd >= 0 && !flush(c)) c->dead = true;
  }

  void loop() {
    tls_self_ = this;
    std::vector<epoll_event> evs(256);
    while (running_) {
      int n = epoll_wait(ep_, evs.data(), int(evs.size()), 100);
      for (int i = 0; i < n; ++i) {
        const uint64_t tag = evs[i].data.u64;
        if (tag == kListenTag) {
          accept_all();
          continue;
        }
        if (tag == kWakeTag) {
          uint64_t v;
          while (read(wake_, &v, sizeof(v)) > 0) {}
          adopt_pending();
          continue;
        }
        auto it = conns_.find(tag);
        if (it == conns_.end()) continue;
        Conn* c = it->second.get();
        if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) on_readable(c);
        const auto tf = Clock::now();
        if (!c->dead && !flush(c)) c->dead = true;
        srv_->stats.ns_send += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - tf).count());
      }
      const auto td = Clock::now();
      drain_outbox();
      srv_->stats.ns_send += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - td).count());
      for (auto it = conns_.begin(); it != conns_.end();) {
        if (it->second->dead) {
          Conn* c = it->second.get();
          ++it;
          close_conn(c, true);
        } else {
          ++it;
        }
      }
    }
    tls_self_ = nullptr;
  }

  Server* srv_;
  int index_;
  int lfd_ = -1, ep_ = -1, wake_ = -1, port_ = 0;
  std::thread th_;
  std::atomic<bool> running_{false};
  nghttp2_session_callbacks* cbs_ = nullptr;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns_;
  uint64_t next_id_ = 1;
  std::vector<uint8_t> rbuf_;
  std::mutex omu_;
  std::vector<Outgoing> outbox_;
  std::atomic<int> nconns_{0};       // live + handed-over connections
  std::mutex amu_;
  std::vector<int> adopt_;           // accepted by the acceptor, not yet registered
  static thread_local IoThread* tls_self_;
};

thread_local IoThread* IoThread::tls_self_ = nullptr;

// ---------------------------------------------------------------- Server
Server::Server(const std::string& host, int port, int io_threads, size_t max_message)
    : host_(host), port_(port), max_message_(max_message) {
  if (io_threads < 1) io_threads = 1;
  io_.emplace_back(std::make_unique<IoThread>(this, 0, host, port, true));
  port_ = io_[0]->port();
  for (int i = 1; i < io_threads; ++i) io_.emplace_back(std::make_unique<IoThread>(this, i, host, port_, false));
}

std::vector<int> Server::io_connections() const {
  std::vector<int> v;
  for (const auto& t : io_) v.push_back(t->live_connections());
  return v;
}

IoThread* Server::pick_io() {
  const unsigned n = unsigned(io_.size());
  const unsigned start = next_io_.fetch_add(1, std::memory_order_relaxed) % n;
  IoThread* best = io_[start].get();
  for (unsigned k = 1; k < n; ++k) {
    IoThread* t = io_[(start + k) % n].get();
    if (t->live_connections() < best->live_connections()) best = t;
  }
  return best;
}

Server::~Server() { stop(); }

void Server::start() {
  if (running_.exchange(true)) return;
  for (auto& t : io_) t->start();
}

void Server::stop() {
  if (!running_.exchange(false)) return;
  for (auto& t : io_) t->stop();
  qcv_.notify_all();
}

void Server::respond(uint64_t conn_id, int io_index, int32_t stream_id, int status, std::string message,
                     std::string body) {
  if (io_index < 0 || io_index >= int(io_.size())) return;
  io_[io_index]->post(Outgoing{conn_id, stream_id, status, std::move(message), std::move(body)});
}

void Server::set_router(Router* r) {
  router_ = r;
  load_ = r ? r->load_word() : &own_load_;
}

std::shared_ptr<StreamRes> Server::reserve_stream(const ProbeInfo& pi, const uint8_t* head, size_t head_len,
                                                  const std::string& method) {
  if (router_) {
    auto r = router_->reserve_stream(pi, head, head_len, method);
    if (r) return r;
  }
  return reserve_ ? reserve_(pi) : nullptr;
}

void Server::dispatch(std::unique_ptr<Call> c) {
  if (router_ && !c->routed && c->method == kPredictMethod && router_->forward(c)) return;
  count(*c);
  if (fast_) {
    const auto t0 = Clock::now();
    const bool taken = fast_(c);
    stats.ns_dispatch += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count());
    if (taken) {
      stats.fast_path++;
      return;
    }
  }
  stats.slow_path++;
  push_call(std::move(c));
}

void Server::push_call(std::unique_ptr<Call> c) {
  {
    std::lock_guard<std::mutex> g(qmu_);
    queue_.push_back(std::move(c));
  }
  qcv_.notify_one();
}

std::unique_ptr<Call> Server::next_call(int timeout_ms) {
  std::unique_lock<std::mutex> lk(qmu_);
  qcv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return !queue_.empty() || !running_; });
  if (queue_.empty()) return nullptr;
  auto c = std::move(queue_.front());
  queue_.pop_front();
  return c;
}

}  // namespace tfs
