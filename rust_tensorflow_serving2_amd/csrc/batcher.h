// Predict fast path + dynamic batching into pinned GPU staging slots.
//
// Python registers an *endpoint* per (model, version, signature) whose inputs
// all have a leading batch dimension and static per-row shapes.  For each
// Predict call the IO thread: decodes the request with the native codec (no
// Python, no GIL), validates it against the endpoint, reserves rows in the
// currently open batch *slot* and memcpy's the tensor bytes straight into
// that slot's pinned host buffer (parallel across IO threads).  A GPU worker
// (one per slot/lane) waits until its slot is full or the batch timeout
// expires, runs the device program on the rows, and calls complete(): the
// per-request PredictResponses are encoded from the pinned output buffers and
// posted back to the IO threads.  Anything the fast path does not handle
// (labels, fill-rule tensors, mismatched aliases/shapes, output filters with
// unknown aliases, ...) falls through to the Python core, which produces the
// exact TF-Serving error or result.
#pragma once
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "http2.h"
#include "request_log.h"
#include "wire.h"

namespace tfs {

struct TensorSpecC {
  std::string alias;
  int dtype = 0;
  std::vector<int64_t> row_shape;
  size_t row_elems = 1;
  size_t row_bytes = 0;    // one row on the wire
  // the row in a batch slot: the wire bytes (conv 0) or, for an fp32 input the
  // device program takes as bf16, the values converted while they are copied
  // in (conv 1, csrc/ingest.h: half the bytes)
  int conv = 0;
  size_t slot_bytes() const { return conv == 1 ? row_elems * 2 : row_bytes; }
};

class Endpoint;

// A row reserved for a request whose payload is still streaming in (http2.h
// StreamRes); committed by the IO thread when the message is complete.
struct SlotStream final : StreamRes {
  std::shared_ptr<Endpoint> ep;
  int slot = -1, idx = -1, n = 0;
  void commit(std::unique_ptr<Call> call) override;
  void abandon() override;
  bool keep_header() const override;
};

struct Pending {
  std::unique_ptr<Call> call;   // null: abandoned streaming row (padding, no answer)
  int row0 = 0, n = 0;
  std::vector<int> outs;   // output indices to encode (empty = all)
  std::shared_ptr<SlotStream> sres;
  bool failed = false;     // its rows could not be copied in: answered INTERNAL
};

// A validated request waiting for a batch slot (every slot busy on the GPU).
// IO threads never block: they park the request here and move on; the lane
// worker that frees a slot moves queued requests into it.
struct Queued {
  std::unique_ptr<Call> call;
  int n = 0;
  std::vector<int> outs;
  std::vector<const uint8_t*> src;     // per input: row data (views into call->body or `owned`)
  std::vector<std::string> owned;      // kOwned tensors (non-packed encodings)
};

// kDead: the lane gave the slot's batch up (device hang); the GPU may still
// write its pinned output rows, so the slot is never handed out again.
enum SlotState : int { kFree = 0, kOpen = 1, kReady = 2, kRunning = 3, kDead = 4 };

struct Slot {
  std::vector<uint8_t*> in_base;     // per input: pinned [max_rows][row]
  std::vector<const uint8_t*> out_base;
  int reserved = 0;
  int copied = 0;
  int state = kFree;
  Clock::time_point first;
  std::vector<Pending> reqs;
  // row ranges (row0, n) whose bytes are complete in the pinned buffer and not
  // yet handed to the lane (eager H2D: the lane copies rows to the device
  // while the batch is still filling, off the batch's critical path)
  std::vector<std::pair<int, int>> ready;
  // per-slot wakeups: only the lane that owns the slot is woken (a shared
  // condition variable woke every lane on every request)
  std::shared_ptr<std::condition_variable> cv = std::make_shared<std::condition_variable>();
};

struct EndpointStats {
  uint64_t requests = 0, batches = 0, rows = 0, rejected = 0;
  // failed batches in total and since the last completed one (the replica
  // health monitor reloads a servable whose device keeps failing)
  uint64_t failed = 0, consecutive_failed = 0;
  // drains of the FIFO queue spread over the drain pool (>= kDrainMinJobs
  // requests moved into slots at once), and row copies that threw
  uint64_t pooled_drains = 0, copy_errors = 0;
};

class Endpoint {
 public:
  Endpoint(int id, std::string model, int64_t version, std::string signature, std::vector<TensorSpecC> inputs,
           std::vector<TensorSpecC> outputs, int max_rows, int64_t timeout_us, int max_wait_ms);
  void set_slot_buffers(int slot, std::vector<uint8_t*> in_base, std::vector<const uint8_t*> out_base);
  // IO thread, never blocks.  Returns 0 if accepted (batched or queued), 1 if
  // not applicable (slow path), 2 if rejected (queue full).
  int offer(std::unique_ptr<Call>& call, PredictRequestView& req);
  // IO thread: reserve a row for a streaming request (nullptr = use the buffered path).
  std::shared_ptr<StreamRes> reserve_stream(const std::shared_ptr<Endpoint>& self, const ProbeInfo& pi);
  void commit_stream(SlotStream& r, std::unique_ptr<Call> call);
  void abandon_stream(SlotStream& r);
  void set_server(Server* srv) { srv_ = srv; }
  // Idle dispatch: a partly filled batch runs right away when no batch of
  // this endpoint is executing (the device would otherwise idle for the
  // batch timeout); under load some batch is always running, so batches
  // still fill up to max_rows / the timeout.
  void set_idle_dispatch(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    idle_dispatch_ = on;
  }
  // GPU worker side.  With `ranges`, rows that completed since the last call
  // are appended to it (the worker copies them to the device right away) and
  // the call also returns 0 early whenever new rows are available.
  int acquire(int slot, int timeout_ms, std::vector<std::pair<int, int>>* ranges = nullptr);
  // when the slot's current batch opened (first row reserved); for tracing
  Clock::time_point slot_opened(int slot) {
    std::lock_guard<std::mutex> g(mu_);
    return slots_[slot].first;
  }
  void complete(int slot, Server& srv);
  void fail(int slot, Server& srv, int code, const std::string& msg);
  // Like fail(), but the slot is retired (kDead) instead of freed: its batch
  // timed out on the device, whose late writes must not land in a reused slot.
  void fail_dead(int slot, Server& srv, int code, const std::string& msg);
  // Closes the endpoint.  With `srv`, every request that has not started on
  // the device (queued, or in an open / ready slot) is answered UNAVAILABLE;
  // running batches are left to their lanes.  Returns after every in-flight
  // row copy into the slots' pinned buffers has finished, so the caller may
  // release those buffers once the lanes are joined.
  void close(Server* srv = nullptr);

  const int id;
  const std::string model;
  const int64_t version;
  const std::string signature;
  std::vector<TensorSpecC> inputs, outputs;
  const int max_rows;
  const int64_t timeout_us;
  const int max_wait_ms;
  EndpointStats stats();
  // Request logging (null: off).  Sampled pairs go to the log's writer thread.
  void set_log(std::shared_ptr<RequestLog> log) {
    std::lock_guard<std::mutex> g(mu_);
    log_ = std::move(log);
    logging_.store(log_ != nullptr);
  }
  bool logging() const { return logging_.load(std::memory_order_relaxed); }
  bool busy() {
    std::lock_guard<std::mutex> g(mu_);
    return running_ > 0;
  }

 private:
  int open_slot_locked(int n);
  // one look at a slot for acquire (caller holds mu_): > 0 the
  // slot's batch was taken (rows), 0 not ready (wake <- when to look again),
  // -1 its state just changed (look again now)
  int poll_slot_locked(int slot, Clock::time_point now, Clock::time_point& wake);
  // Move queued requests into open slots; copies run outside the lock.
  void drain_queue();
  struct CopyJob {
    uint8_t* dst;
    const uint8_t* src;
    size_t bytes;
  };
  void copy_rows(int slot, int r0, int n, const std::vector<const uint8_t*>& src) noexcept;
  // batcher-side abandonment of rows whose payload stalls (caller holds mu_)
  void abandon_stalled_locked(Slot& s);
  Server* srv_ = nullptr;
  std::mutex mu_;
  std::deque<Queued> queue_;
  size_t max_queue_ = 0;
  std::condition_variable cv_ready_, cv_free_;
  std::vector<Slot> slots_;
  int open_ = -1;
  int next_ = 0;
  int running_ = 0;          // slots in kRunning
  int copying_ = 0;          // copy_rows() calls writing into slot buffers outside mu_
  bool idle_dispatch_ = true;
  bool closed_ = false;
  EndpointStats st_;
  std::shared_ptr<RequestLog> log_;
  std::atomic<bool> logging_{false};
};

class FastPath {
 public:
  explicit FastPath(Server* srv) : srv_(srv) {}
  bool try_dispatch(std::unique_ptr<Call>& call);
  std::shared_ptr<Endpoint> route(const ModelSpecView& spec);
  std::shared_ptr<StreamRes> reserve_stream(const ProbeInfo& pi);
  int add_endpoint(std::shared_ptr<Endpoint> ep);
  // `retired`: also endpoints already removed — a lane that finishes a batch
  // after its endpoint closed must still reach it to answer that batch
  std::shared_ptr<Endpoint> endpoint(int id, bool retired = false);
  void remove_endpoint(int id);
  // route (model, signature) [+version] to an endpoint; version < 0 = "latest"
  void set_route(const std::string& model, const std::string& signature, int64_t version, int ep_id);
  void clear_routes(const std::string& model);
  int next_id() { return ++ids_; }
  Server* server() { return srv_; }

 private:
  Server* srv_;
  std::shared_mutex mu_;
  std::map<int, std::shared_ptr<Endpoint>> eps_;
  // removed endpoints, kept until no batch of theirs is running (pruned on
  // the next removal): they own no buffers, only their bookkeeping
  std::map<int, std::shared_ptr<Endpoint>> retired_;
  std::map<std::string, int> routes_;   // key = model \0 signature \0 version|"L"
  int ids_ = 0;
};

}  // namespace tfs
