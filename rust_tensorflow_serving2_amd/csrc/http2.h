// Native gRPC-over-HTTP/2 front end (server) and load generator (client).
//
// Replaces the transport layer the reference leaves to tonic/hyper/h2 on the
// client side (src/lib.rs:132-138; Cargo.lock tonic 0.1 / h2 0.2) and to the
// external TF-Serving container on the server side (serving/rundocker.sh:15).
// Design: N epoll IO threads; IO thread 0 owns the one SO_REUSEPORT listening
// socket of this process (the kernel spreads connections across server
// processes, one per GPU) and hands each accepted connection to the IO thread
// with the fewest live connections (the kernel's per-thread reuseport hash put
// the reference client's two connections on ONE thread in about one run in
// six, halving that run); libnghttp2 for framing/HPACK/flow control; request
// bodies assembled per stream and dispatched either to the C++ Predict fast
// path (batcher.h) or to a queue drained by Python control-plane threads.
// Responses from any thread are posted to the owning IO thread (eventfd).
#pragma once
#include "ingest.h"
#include <atomic>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "wire.h"

namespace tfs {

using Clock = std::chrono::steady_clock;

struct Call;

// Answers calls that another replica placed in this replica's shared-memory
// ring (router.h): the answer goes back through the ring, not a socket.
class RemoteSink {
 public:
  virtual ~RemoteSink() = default;
  virtual void respond_remote(const Call& c, int status, const std::string& msg, const std::string& body) = 0;
};

// One completed unary request waiting for its answer.
struct Call {
  uint64_t conn_id = 0;
  int io_index = 0;
  int32_t stream_id = 0;
  std::string method;      // ":path", e.g. /tensorflow.serving.PredictionService/Predict
  // gRPC message as received: the 5-byte length prefix is kept (skipped via
  // `off`) so the 602 KB request buffer moves into the Call without a copy
  std::string body;
  size_t off = 0;
  // a message held outside `body`: the cell of a cross-replica call (router.h)
  const uint8_t* ext = nullptr;
  size_t ext_len = 0;
  // a streamed request's header bytes (length prefix + everything before the
  // payload), kept only when its endpoint logs requests (request_log.h)
  std::string head;
  RemoteSink* remote = nullptr;   // answer through this sink (cell index below)
  uint32_t cell = 0;
  bool routed = false;            // placed by the router already: never forwarded again
  // outstanding-call counter this call was counted in (decremented when answered)
  std::atomic<int64_t>* load = nullptr;
  const uint8_t* data() const { return ext ? ext : reinterpret_cast<const uint8_t*>(body.data()) + off; }
  size_t size() const { return ext ? ext_len : body.size() - off; }
  Clock::time_point arrival;
  int64_t timeout_us = 0;  // grpc-timeout, 0 = none
  // the client's deadline (grpc-timeout) has passed: answer DEADLINE_EXCEEDED, skip the work
  bool expired(Clock::time_point now = Clock::now()) const {
    return timeout_us > 0 && now - arrival > std::chrono::microseconds(timeout_us);
  }
};

class Server;

// Fast-path hook: return true when the call was taken (it will be answered
// later through Server::respond).
using FastDispatch = std::function<bool(std::unique_ptr<Call>&)>;

// A batch-slot row reserved for a request that is still arriving: the IO
// thread copies the tensor payload straight from its socket read buffer into
// `dst` (pinned memory the GPU reads), so a 602 KB image is copied once in
// user space instead of being assembled into a body first.
struct StreamRes {
  std::atomic<int> state{0};     // 0 streaming, 1 committed, 2 abandoned (by either side)
  std::atomic<int> writers{0};   // IO thread inside write(); the batcher waits for 0 before reusing the row
  uint8_t* dst = nullptr;
  size_t len = 0, got = 0;       // payload (wire) bytes expected / arrived
  // ingest conversion: 1 = the wire's fp32 values land in the row as bf16
  // (csrc/ingest.h), so the row holds len / 2 bytes and a float split across
  // two chunks waits in `carry`
  int conv = 0;
  int ncarry = 0;
  uint8_t carry[4] = {0, 0, 0, 0};
  virtual ~StreamRes() = default;
  // Every payload byte arrived and the message ended: hand over the call.
  virtual void commit(std::unique_ptr<Call> call) = 0;
  // The IO side gives up (stream reset, protocol error).
  virtual void abandon() = 0;
  // The row lives in another replica's ring (router.h), not a local batch slot.
  virtual bool remote() const { return false; }
  // The committed Call should keep the request's header bytes (Call::head).
  virtual bool keep_header() const { return false; }
  // Copy the next chunk; false once the batcher has abandoned the row (too slow).
  bool write(const uint8_t* p, size_t n) {
    writers.fetch_add(1);
    const bool live = state.load() == 0;
    if (live) {
      if (conv) {
        write_converted(p, n);
      } else if (p != dst + got) {   // p == dst + got: recv()'d straight into the row
        std::memcpy(dst + got, p, n);
      }
    }
    writers.fetch_sub(1);
    got += n;
    return live;
  }

 private:
  void write_converted(const uint8_t* p, size_t n) {
    uint16_t* out = reinterpret_cast<uint16_t*>(dst) + (got - size_t(ncarry)) / 4;   // values completed so far
    size_t i = 0;
    if (ncarry) {
      while (ncarry < 4 && i < n) carry[ncarry++] = p[i++];
      if (ncarry < 4) return;
      ingest_f32_to_bf16(out++, carry, 1);
      ncarry = 0;
    }
    const size_t nv = (n - i) / 4;
    ingest_f32_to_bf16(out, p + i, nv);
    i += nv * 4;
    while (i < n) carry[ncarry++] = p[i++];
  }
};

// Reserve a row for a probed request header; nullptr = not streamable here.
using StreamReserve = std::function<std::shared_ptr<StreamRes>(const ProbeInfo&)>;

struct ServerStats {
  std::atomic<uint64_t> connections{0}, requests{0}, fast_path{0}, slow_path{0}, responses{0}, errors{0};
  std::atomic<uint64_t> streamed{0};   // fast-path requests whose payload went socket -> slot directly
  std::atomic<uint64_t> expired{0};    // answered DEADLINE_EXCEEDED (client grpc-timeout passed)
  std::atomic<uint64_t> bytes_in{0}, bytes_out{0};
  std::atomic<uint64_t> direct_bytes{0};   // payload bytes recv()'d straight into batch rows
  // IO-thread time split (ns): recv() syscalls, nghttp2 frame processing incl.
  // body assembly, fast-path dispatch (decode + batch-slot copy), send()
  std::atomic<uint64_t> ns_recv{0}, ns_h2{0}, ns_dispatch{0}, ns_send{0};
  // recv() shape (the reference-client slow-mode diagnostic, round-5 VERDICT
  // item 6): calls that returned data, calls that found the socket empty
  // (EAGAIN: one per epoll wake-up that drained it), bytes returned
  std::atomic<uint64_t> recv_calls{0}, recv_empty{0}, recv_bytes{0};
};

class IoThread;
class Router;

class Server {
 public:
  Server(const std::string& host, int port, int io_threads, size_t max_message);
  ~Server();
  void start();
  void stop();
  int port() const { return port_; }

  void set_fast_dispatch(FastDispatch fn) { fast_ = std::move(fn); }
  void set_stream_reserve(StreamReserve fn) { reserve_ = std::move(fn); }
  const StreamReserve& stream_reserve() const { return reserve_; }
  // Answer a call (thread-safe).  status = grpc code; body ignored unless OK.
  void respond(uint64_t conn_id, int io_index, int32_t stream_id, int status, std::string message,
               std::string body);
  void respond(const Call& c, int status, std::string message, std::string body) {
    if (c.load) c.load->fetch_sub(1, std::memory_order_relaxed);
    if (c.remote) {
      c.remote->respond_remote(c, status, message, body);
      return;
    }
    respond(c.conn_id, c.io_index, c.stream_id, status, std::move(message), std::move(body));
  }
  // Cross-replica routing (router.h); null = every call stays local.  Set
  // before start().
  void set_router(Router* r);
  Router* router() const { return router_; }
  // A streamed Predict's row: on a peer (router) or in a local batch slot.
  std::shared_ptr<StreamRes> reserve_stream(const ProbeInfo& pi, const uint8_t* head, size_t head_len,
                                            const std::string& method);
  // Count a call in this replica's load (answered calls uncount themselves).
  void count(Call& c) {
    if (c.load) return;
    c.load = load_;
    c.load->fetch_add(1, std::memory_order_relaxed);
  }
  int64_t load() const { return load_->load(std::memory_order_relaxed); }
  // Slow path queue for the Python control plane.
  std::unique_ptr<Call> next_call(int timeout_ms);
  void push_call(std::unique_ptr<Call> c);

  // Called by IO threads when a request is complete.
  void dispatch(std::unique_ptr<Call> c);
  // IO thread with the fewest live connections (ties: round-robin), the
  // acceptor's target for a new connection.
  IoThread* pick_io();
  // live connections per IO thread (diagnostics / tests)
  std::vector<int> io_connections() const;
  size_t max_message() const { return max_message_; }
  ServerStats stats;

 private:
  std::string host_;
  int port_;
  size_t max_message_;
  std::vector<std::unique_ptr<IoThread>> io_;
  FastDispatch fast_;
  StreamReserve reserve_;
  Router* router_ = nullptr;
  std::atomic<int64_t> own_load_{0};
  std::atomic<int64_t>* load_ = &own_load_;
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<std::unique_ptr<Call>> queue_;
  std::atomic<bool> running_{false};
  std::atomic<unsigned> next_io_{0};
};

// ---------------------------------------------------------------- load generator
struct LoadGenResult {
  uint64_t ok = 0, errors = 0;
  double elapsed_s = 0;
  std::vector<double> latency_us;   // per successful request
  std::string first_error;
  uint64_t bytes_sent = 0, bytes_recv = 0;
  double cpu_s = 0;                 // CPU time of the client threads
  // window(): seconds from the window's start to each of its completions
  // (every completion, in no particular order)
  std::vector<double> done_s;
};

// Persistent load generator: `threads` client threads each own a share of
// `connections` HTTP/2 connections, opened once in the constructor (like a
// real client's channel) and reused by every run(); `concurrency` unary calls
// of `method` stay in flight, bodies used round-robin (pre-serialised).
class LoadGen {
 public:
  LoadGen(const std::string& host, int port, const std::string& method, const std::vector<std::string>& bodies,
          int concurrency, int connections, int threads);
  ~LoadGen();
  LoadGenResult run(uint64_t total, double timeout_s);
  // Continuous mode: keep `concurrency` calls in flight until stop(), so a
  // benchmark's warmup and timed windows see a pipeline that never drains.
  void start();
  // Block until the next `n` completions (counted from the call) have
  // arrived; their latencies / errors and the wall time of the window.
  LoadGenResult window(uint64_t n, double timeout_s);
  uint64_t completed() const;
  // Stop submitting, drain in-flight calls, join; totals since start().
  LoadGenResult stop(double timeout_s);
  struct Worker;

 private:
  std::vector<std::thread> threads_;
  std::shared_ptr<void> sh_;       // shared request state (type private to the .cpp)
  void* cbs_ = nullptr;            // nghttp2_session_callbacks*
  std::vector<std::unique_ptr<Worker>> workers_;
};

// Drive `total` unary calls of `method` against host:port with `concurrency`
// streams in flight spread over `connections` HTTP/2 connections served by
// `threads` client threads.  Bodies are used round-robin (pre-serialised).
LoadGenResult run_loadgen(const std::string& host, int port, const std::string& method,
                          const std::vector<std::string>& bodies, uint64_t total, int concurrency,
                          int connections, int threads, double timeout_s);

}  // namespace tfs
