// pybind11 registration of the HTTP/2 front end, Predict fast path and load generator.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <dlfcn.h>
#include <cstdio>
#include <cstdlib>
#include <pthread.h>
#include <sys/prctl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <thread>

#include "batcher.h"
#include "http2.h"
#include "router.h"

namespace py = pybind11;
using namespace tfs;

namespace {

// ---------------------------------------------------------------- native GPU lanes
// The HIP runtime is resolved at run time (dlopen of the libamdhip64 that torch
// already loaded), so this CPU extension builds without HIP and costs nothing
// on machines without a GPU.
struct HipRt {
  using launch_t = int (*)(void*, void*);
  using setdev_t = int (*)(int);
  using errstr_t = const char* (*)(int);
  using memcpy_t = int (*)(void*, const void*, size_t, int, void*);
  using evcreate_t = int (*)(void**, unsigned);
  using evrecord_t = int (*)(void*, void*);
  using evsync_t = int (*)(void*);
  using evquery_t = int (*)(void*);
  using evdestroy_t = int (*)(void*);
  using screate_t = int (*)(void**, unsigned);
  using sdestroy_t = int (*)(void*);
  using swait_t = int (*)(void*, void*, unsigned);
  launch_t launch = nullptr;
  setdev_t set_device = nullptr;
  errstr_t err = nullptr;
  memcpy_t memcpy_async = nullptr;
  evcreate_t event_create = nullptr;
  evrecord_t event_record = nullptr;
  evsync_t event_sync = nullptr;
  evquery_t event_query = nullptr;
  evdestroy_t event_destroy = nullptr;
  screate_t stream_create = nullptr;
  sdestroy_t stream_destroy = nullptr;
  swait_t stream_wait_event = nullptr;
  bool load() {
    if (launch) return true;
    void* h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("libamdhip64.so", RTLD_NOW);
    if (!h) return false;
    auto sym = [&](const char* n) { return dlsym(h, n); };
    set_device = reinterpret_cast<setdev_t>(sym("hipSetDevice"));
    err = reinterpret_cast<errstr_t>(sym("hipGetErrorString"));
    memcpy_async = reinterpret_cast<memcpy_t>(sym("hipMemcpyAsync"));
    event_create = reinterpret_cast<evcreate_t>(sym("hipEventCreateWithFlags"));
    event_record = reinterpret_cast<evrecord_t>(sym("hipEventRecord"));
    event_sync = reinterpret_cast<evsync_t>(sym("hipEventSynchronize"));
    event_query = reinterpret_cast<evquery_t>(sym("hipEventQuery"));
    event_destroy = reinterpret_cast<evdestroy_t>(sym("hipEventDestroy"));
    launch = reinterpret_cast<launch_t>(sym("hipGraphLaunch"));
    stream_create = reinterpret_cast<screate_t>(sym("hipStreamCreateWithFlags"));
    stream_destroy = reinterpret_cast<sdestroy_t>(sym("hipStreamDestroy"));
    stream_wait_event = reinterpret_cast<swait_t>(sym("hipStreamWaitEvent"));
    return launch && set_device && memcpy_async && event_create && event_record && event_sync && event_query &&
           event_destroy;
  }
};
constexpr int kHipMemcpyHostToDevice = 1, kHipMemcpyDeviceToHost = 2;
constexpr unsigned kHipEventDisableTiming = 0x2;
constexpr unsigned kHipStreamNonBlocking = 0x1;
constexpr int kHipErrorNotReady = 600;
constexpr int kLaneHung = -2;   // NativeLane::wait gave up (not a hipError_t)

HipRt& hip_rt() {
  static HipRt rt;
  return rt;
}

// ---------------------------------------------------------------- roctx
// Opt-in (TFSERVE_ROCTX=1) roctx ranges around each native-lane batch and its
// phases, so `rocprofv3 --marker-trace` lines host-side batch phases up with
// the kernels they launched.  The rocprofiler-sdk roctx library is dlopen'ed
// (no link dependency); without it, or unset, the calls are no-ops.
struct Roctx {
  using push_t = int (*)(const char*);
  using pop_t = int (*)();
  push_t push_ = nullptr;
  pop_t pop_ = nullptr;
  Roctx() {
    const char* on = getenv("TFSERVE_ROCTX");
    if (!on || std::atoi(on) == 0) return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    push_ = reinterpret_cast<push_t>(dlsym(h, "roctxRangePushA"));
    pop_ = reinterpret_cast<pop_t>(dlsym(h, "roctxRangePop"));
    if (!push_ || !pop_) push_ = nullptr, pop_ = nullptr;
  }
  bool on() const { return push_ != nullptr; }
  void push(const char* m) const {
    if (push_) push_(m);
  }
  void pop() const {
    if (pop_) pop_();
  }
};
const Roctx& roctx() {
  static Roctx r;
  return r;
}

// ---------------------------------------------------------------- batch trace
// One record per GPU batch served by a native lane (--trace_dir): times are
// microseconds on the steady clock: batch opened (first row reserved),
// acquired by the lane (batch closed), H2D+graph+D2H issued, GPU done, responses posted.
struct BatchTrace {
  int endpoint, slot, rows;
  double opened_us, acquired_us, issued_us, done_us, posted_us;
};
struct TraceBuf {
  std::mutex mu;
  std::vector<BatchTrace> recs;
  std::atomic<bool> on{false};
  void add(const BatchTrace& t) {
    std::lock_guard<std::mutex> g(mu);
    if (recs.size() < 1000000) recs.push_back(t);
  }
  std::vector<BatchTrace> drain() {
    std::lock_guard<std::mutex> g(mu);
    std::vector<BatchTrace> out;
    out.swap(recs);
    return out;
  }
};
TraceBuf& trace_buf() {
  static TraceBuf t;
  return t;
}
double us_of(Clock::time_point t) {
  return std::chrono::duration<double, std::micro>(t.time_since_epoch()).count();
}

// Compute gate (TFSERVE_GPU_CONCURRENCY=K, 0 = off): at most K bucket graphs
// of the lanes on one device run at once, while every lane's H2D copy still
// goes out as soon as its batch closes.  Graph launch s makes its stream wait
// (GPU side, hipStreamWaitEvent) for the event recorded right after graph
// launch s - K, so no host thread blocks.  Why: ResNet-50 b32 computes a batch
// in 0.536 ms with 3 replays in flight but 0.583 ms with 4
// (scripts/probe_concurrency.py, profiles/round6/r6k/conc.log), while the
// serving lanes need a fourth batch in flight to hide each batch's 175-us
// input copy (3 lanes: 37k vs 53k RPC/s, round 5).  Launch order is a global
// sequence taken under the gate's mutex together with the launch and the
// record, so every wait names an event recorded by an earlier launch and the
// dependencies are acyclic.  Measured neutral, so off by default: 2000-step
// headline 54.1k (K = 3, 4 lanes) vs 53.0-53.8k (off) on one box; K = 2 50.1k;
// K = 3 with 5 / 6 lanes 45.1k / 50.0k (profiles/round6/r6p/).
struct ComputeGate {
  std::mutex mu;
  int cap = 0;
  uint64_t seq = 0;
  std::vector<void*> ring;    // cap + 16 events, reused round robin
};
ComputeGate* compute_gate(HipRt& rt, int device) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<ComputeGate>> gates;
  static const int cap = [] {
    const char* e = getenv("TFSERVE_GPU_CONCURRENCY");
    return e ? std::max(0, std::atoi(e)) : 0;
  }();
  if (cap <= 0 || !rt.stream_wait_event) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  auto& slot = gates[device];
  if (!slot) {
    auto gate = std::make_unique<ComputeGate>();
    gate->cap = cap;
    gate->ring.assign(size_t(cap) + 16, nullptr);
    for (auto& ev : gate->ring)
      if (rt.event_create(&ev, kHipEventDisableTiming) != 0) return nullptr;
    slot = std::move(gate);
  }
  return slot.get();
}

struct LaneCopy {
  uintptr_t dst, src;
  size_t row_bytes;
};
struct LaneBucket {
  int rows = 0;
  void* exec = nullptr;
  std::vector<LaneCopy> in, out;   // per batch: n rows each way (live rows only)
};

// One GPU lane served entirely in C++: wait for the slot's batch, H2D the n
// live rows (SDMA), launch the bucket's HIP graph, D2H the n result rows, and
// wait for the completion event (polled with naps, not spun); then encode and
// post the responses.  No Python and no GIL per batch.
class NativeLane {
 public:
  NativeLane(Server* srv, std::shared_ptr<Endpoint> ep, int slot, int device, void* stream,
             std::vector<LaneBucket> buckets)
      : srv_(srv), ep_(std::move(ep)), slot_(slot), device_(device), stream_(stream), buckets_(std::move(buckets)) {
    // fault injection for tests (same spec as utils/faults.py):
    // TFSERVE_FAULT=lane_every=N fails every Nth batch, lane_after=N every
    // batch after the first N of this lane (a device that went bad)
    if (const char* f = getenv("TFSERVE_FAULT")) {
      const std::string spec(f);
      auto k = spec.find("lane_every=");
      if (k != std::string::npos) fault_every_ = std::atoi(spec.c_str() + k + 11);
      k = spec.find("lane_after=");
      if (k != std::string::npos) fault_after_ = std::atoi(spec.c_str() + k + 11);
      k = spec.find("lane_hang=");
      if (k != std::string::npos) fault_hang_ = std::atoi(spec.c_str() + k + 10);
    }
    std::sort(buckets_.begin(), buckets_.end(), [](auto& a, auto& b) { return a.rows < b.rows; });
    // eager H2D (rows copied to the device while the batch fills) needs every
    // bucket graph to read the same device input rows (GpuRunner shares one
    // max-bucket buffer per lane).  Opt-in (TFSERVE_EAGER_H2D=1): measured on
    // ResNet-50 b32 it LOSES (29-33k vs 39-41k RPC/s) — one hipMemcpyAsync per
    // 602 KB row costs more lane-thread time and SDMA setup than the single
    // batched copy it takes off the critical path.
    eager_ = !buckets_.empty();
    for (auto& b : buckets_) {
      if (b.in.size() != buckets_.back().in.size()) eager_ = false;
      for (size_t i = 0; eager_ && i < b.in.size(); ++i)
        if (b.in[i].dst != buckets_.back().in[i].dst || b.in[i].src != buckets_.back().in[i].src) eager_ = false;
    }
    if (const char* t = getenv("TFSERVE_LANE_TIMEOUT_MS")) timeout_floor_ms_ = std::max(1, std::atoi(t));
    const char* eager_env = getenv("TFSERVE_EAGER_H2D");
    eager_ = eager_ && eager_env && std::atoi(eager_env) != 0;
    th_ = std::thread([this] { run(); });
  }
  ~NativeLane() { join(); }
  void join() {
    if (th_.joinable()) th_.join();
  }
  int endpoint_id() const { return ep_->id; }
  std::atomic<uint64_t> batches{0}, errors{0};
  std::atomic<bool> dead{false};   // gave up on a hung batch and exited

 private:
  int batch(HipRt& rt, void* done, int n) {
    const LaneBucket* b = nullptr;
    for (auto& x : buckets_)
      if (x.rows >= n) {
        b = &x;
        break;
      }
    if (!b) return -1;
    const Roctx& rx = roctx();
    char label[64];
    if (rx.on()) {
      snprintf(label, sizeof label, "tfs.batch ep=%d slot=%d rows=%d", ep_->id, slot_, n);
      rx.push(label);
      rx.push("tfs.issue");   // H2D + graph launch + D2H enqueued on the lane stream
    }
    int e = 0;
    const auto t_issue = Clock::now();
    if (eager_) {
      // every row was already queued on the copy stream as it arrived
      e = rt.event_record(copied_, copy_stream_);
      if (!e) e = rt.stream_wait_event(stream_, copied_, 0);
    } else {
      if (rx.on()) rx.push("tfs.h2d");
      for (auto& c : b->in)
        if (!e) e = rt.memcpy_async(reinterpret_cast<void*>(c.dst), reinterpret_cast<const void*>(c.src),
                                    c.row_bytes * size_t(n), kHipMemcpyHostToDevice, stream_);
      if (rx.on()) rx.pop();
    }
    if (rx.on()) rx.push("tfs.graph_launch");
    if (gate_ && !e) {
      std::lock_guard<std::mutex> g(gate_->mu);
      const uint64_t sq = gate_->seq++;
      const size_t R = gate_->ring.size();
      if (sq >= uint64_t(gate_->cap)) e = rt.stream_wait_event(stream_, gate_->ring[(sq - gate_->cap) % R], 0);
      if (!e) e = rt.launch(b->exec, stream_);
      if (!e) e = rt.event_record(gate_->ring[sq % R], stream_);
    } else if (!e) {
      e = rt.launch(b->exec, stream_);
    }
    if (rx.on()) rx.pop();
    for (auto& c : b->out)
      if (!e) e = rt.memcpy_async(reinterpret_cast<void*>(c.dst), reinterpret_cast<const void*>(c.src),
                                  c.row_bytes * size_t(n), kHipMemcpyDeviceToHost, stream_);
    if (!e) e = rt.event_record(done, stream_);
    if (rx.on()) {
      rx.pop();
      rx.push("tfs.gpu_wait");
    }
    const size_t bi = size_t(b - buckets_.data());
    if (!e) e = wait(rt, done, t_issue, deadline_from(Clock::now()), ema_us_[bi], b->rows <= kSpinTailRows);
    if (!e) {
      const double us = std::chrono::duration<double, std::micro>(Clock::now() - t_issue).count();
      ema_us_[bi] = ema_us_[bi] <= 0 ? us : 0.8 * ema_us_[bi] + 0.2 * us;
    }
    if (rx.on()) {
      rx.pop();
      rx.pop();
    }
    return e;
  }
  // Wait for the batch's completion event without burning a core (a
  // hipEventSynchronize spin would take one per lane from the IO threads):
  // ONE nap for most of this bucket's expected issue->done time (a running
  // average), then polls every ~8 us.  The lane thread runs with 1-us timer
  // slack, so a nap ends when asked (the default 50-us slack made each 40-us
  // nap ~90 us, which a batch-1 request paid in full).  Small buckets
  // (`spin_tail`: the latency-bound, low-load regime -- a batch-1 request
  // waits on nothing else) poll the last quarter with yields only, so the
  // completion is seen within ~1 us instead of up to one 8-us nap; the large
  // buckets of the throughput regime keep napping.  Gives up after
  // `deadline` (a hung kernel or wedged stream): returns kLaneHung.
  static constexpr int kSpinTailRows = 4;
  static int wait(HipRt& rt, void* ev, Clock::time_point t_issue, Clock::time_point deadline, double expect_us,
                  bool spin_tail) {
    if (expect_us > 60.0) {
      const auto wake = t_issue + std::chrono::microseconds(int64_t(0.75 * expect_us));
      if (Clock::now() < wake && rt.event_query(ev) == kHipErrorNotReady) std::this_thread::sleep_until(wake);
    }
    for (int i = 0;; ++i) {
      const int e = rt.event_query(ev);
      if (e != kHipErrorNotReady) return e;
      if (i < 8 || (spin_tail && i < (1 << 20))) {
        if (spin_tail && (i & 1023) == 1023 && Clock::now() > deadline) return kLaneHung;
        std::this_thread::yield();
      } else {
        if ((i & 63) == 0 && Clock::now() > deadline) return kLaneHung;
        std::this_thread::sleep_for(std::chrono::microseconds(8));
      }
    }
  }
  // Batch deadline: 50x the lane's running mean batch time, never under the
  // floor (first batches include lazy device init; TFSERVE_LANE_TIMEOUT_MS).
  Clock::time_point deadline_from(Clock::time_point t0) const {
    const double ms = std::max(double(timeout_floor_ms_), 50.0 * mean_ms_);
    return t0 + std::chrono::microseconds(int64_t(ms * 1e3));
  }
  // H2D of rows that just completed in the pinned slot (row ranges from acquire)
  int copy_rows(HipRt& rt, const std::vector<std::pair<int, int>>& ranges) {
    const LaneBucket& b = buckets_.back();
    int e = 0;
    for (auto& r : ranges)
      for (auto& c : b.in)
        if (!e) e = rt.memcpy_async(reinterpret_cast<void*>(c.dst + size_t(r.first) * c.row_bytes),
                                    reinterpret_cast<const void*>(c.src + size_t(r.first) * c.row_bytes),
                                    c.row_bytes * size_t(r.second), kHipMemcpyHostToDevice, copy_stream_);
    return e;
  }
  void run() {
    pthread_setname_np(pthread_self(), "tfs-nlane");
    prctl(PR_SET_TIMERSLACK, 1000UL);     // 1-us timer slack for the completion naps (wait())
    ema_us_.assign(buckets_.size(), 0.0);
    HipRt& rt = hip_rt();
    rt.set_device(device_);
    gate_ = compute_gate(rt, device_);
    void* done = nullptr;
    if (rt.event_create(&done, kHipEventDisableTiming) != 0) done = nullptr;
    if (eager_ && (!rt.stream_create || !rt.stream_wait_event ||
                   rt.stream_create(&copy_stream_, kHipStreamNonBlocking) != 0 ||
                   rt.event_create(&copied_, kHipEventDisableTiming) != 0))
      eager_ = false;
    std::vector<std::pair<int, int>> ranges;
    int copy_err = 0;
    bool hung = false;
    for (;;) {
      ranges.clear();
      const int n = ep_->acquire(slot_, 100, eager_ ? &ranges : nullptr);
      if (!ranges.empty() && !copy_err) copy_err = copy_rows(rt, ranges);
      if (n < 0) break;   // endpoint closed
      if (n == 0) continue;
      if (copy_err) {
        errors++;
        ep_->fail(slot_, *srv_, 13 /*INTERNAL*/, std::string("GPU row copy failed: ") + (rt.err ? rt.err(copy_err) : ""));
        copy_err = 0;
        continue;
      }
      ++seen_;
      if (fault_hang_ >= 0 && seen_ > uint64_t(fault_hang_)) {
        // simulated wedged device: the batch never completes within the deadline
        std::this_thread::sleep_for(std::chrono::milliseconds(timeout_floor_ms_));
        errors++;
        hung = true;
        ep_->fail_dead(slot_, *srv_, 14 /*UNAVAILABLE*/, "GPU batch timed out (device not responding)");
        break;
      }
      if ((fault_every_ > 0 && seen_ % uint64_t(fault_every_) == 0) ||
          (fault_after_ >= 0 && seen_ > uint64_t(fault_after_))) {
        errors++;
        ep_->fail(slot_, *srv_, 13 /*INTERNAL*/, "injected fault (TFSERVE_FAULT)");
        continue;
      }
      const bool tracing = trace_buf().on.load(std::memory_order_relaxed);
      const auto t_acq = Clock::now();
      const int e = done ? batch(rt, done, n) : -1;
      if (e == kLaneHung) {
        // the device stopped making progress: answer the batch, retire the
        // slot (late GPU writes may still land in it) and end this lane so an
        // unload can join it; the health monitor sees the failure counters
        errors++;
        hung = true;
        ep_->fail_dead(slot_, *srv_, 14 /*UNAVAILABLE*/, "GPU batch timed out (device not responding)");
        break;
      }
      if (e != 0) {
        errors++;
        std::string why = e > 0 && rt.err ? std::string(rt.err(e)) : std::string("no graph for this batch");
        ep_->fail(slot_, *srv_, 13 /*INTERNAL*/, "GPU batch failed: " + why);
        continue;
      }
      batches++;
      const auto t_done = Clock::now();
      const double ms = std::chrono::duration<double, std::milli>(t_done - t_acq).count();
      mean_ms_ = batches == 1 ? ms : 0.9 * mean_ms_ + 0.1 * ms;
      const auto t_open = tracing ? ep_->slot_opened(slot_) : t_done;
      ep_->complete(slot_, *srv_);
      if (tracing)
        trace_buf().add({ep_->id, slot_, n, us_of(t_open), us_of(t_acq), us_of(t_acq), us_of(t_done),
                         us_of(Clock::now())});
    }
    dead = hung;
    if (hung) return;   // the wedged stream still references these: leak them rather than block
    if (done) rt.event_destroy(done);
    if (copied_) rt.event_destroy(copied_);
    if (copy_stream_ && rt.stream_destroy) rt.stream_destroy(copy_stream_);
  }
  Server* srv_;
  std::shared_ptr<Endpoint> ep_;
  int slot_, device_;
  void* stream_;
  std::vector<LaneBucket> buckets_;
  bool eager_ = false;
  ComputeGate* gate_ = nullptr;   // shared by the device's lanes (TFSERVE_GPU_CONCURRENCY)
  void* copy_stream_ = nullptr;
  void* copied_ = nullptr;
  int fault_every_ = 0;
  int fault_after_ = -1;
  int fault_hang_ = -1;
  int timeout_floor_ms_ = 10000;
  double mean_ms_ = 0.0;
  std::vector<double> ema_us_;     // per bucket: running issue -> done time (wait()'s first nap)
  uint64_t seen_ = 0;
  std::thread th_;
};

struct PyServer {
  // declared first: destroyed last, after every lane / endpoint that may
  // still answer a call another replica placed in its ring
  std::unique_ptr<Router> router;
  std::unique_ptr<Server> srv;
  std::unique_ptr<FastPath> fast;
  std::mutex lmu;
  std::vector<std::unique_ptr<NativeLane>> lanes;
  // Explicit teardown (also when stop_router()/stop() were never called, e.g.
  // an exception during start-up): the router's thread dispatches into srv
  // and answers its pending calls through srv, so it stops while srv is alive;
  // member order alone would destroy srv first.
  ~PyServer() {
    if (router) router->stop();
    if (srv) srv->stop();
  }
  // join (and drop) the lanes of an endpoint that has been closed
  void join_lanes(int ep_id) {
    std::vector<std::unique_ptr<NativeLane>> done;
    {
      std::lock_guard<std::mutex> g(lmu);
      for (auto it = lanes.begin(); it != lanes.end();) {
        if (ep_id < 0 || (*it)->endpoint_id() == ep_id) {
          done.push_back(std::move(*it));
          it = lanes.erase(it);
        } else {
          ++it;
        }
      }
    }
    for (auto& l : done) l->join();
  }
};

// A slow-path call handed to Python.
struct PyCall {
  std::unique_ptr<Call> call;
};

std::vector<TensorSpecC> specs_from(const py::list& l) {
  std::vector<TensorSpecC> out;
  for (auto it : l) {
    auto t = it.cast<py::tuple>();
    TensorSpecC s;
    s.alias = t[0].cast<std::string>();
    s.dtype = t[1].cast<int>();
    s.row_shape = t[2].cast<std::vector<int64_t>>();
    s.row_elems = 1;
    for (auto d : s.row_shape) s.row_elems *= size_t(d);
    const int esz = dtype_size(s.dtype);
    if (esz == 0) throw std::invalid_argument("fast path: unsupported dtype for " + s.alias);
    s.row_bytes = s.row_elems * size_t(esz);
    // optional 4th field: the dtype of the batch-slot rows (DT_BFLOAT16 for an
    // fp32 input converted on ingest)
    if (t.size() > 3 && !t[3].is_none()) {
      const int slot_dt = t[3].cast<int>();
      if (slot_dt == DT_BFLOAT16 && s.dtype == DT_FLOAT) {
        s.conv = 1;
      } else if (slot_dt != s.dtype) {
        throw std::invalid_argument("fast path: unsupported slot dtype for " + s.alias);
      }
    }
    out.push_back(std::move(s));
  }
  std::sort(out.begin(), out.end(), [](const TensorSpecC& a, const TensorSpecC& b) { return a.alias < b.alias; });
  return out;
}

}  // namespace

void register_server(py::module_& m) {
  py::class_<PyCall>(m, "Call")
      .def_property_readonly("method", [](const PyCall& c) { return c.call->method; })
      .def_property_readonly("body", [](const PyCall& c) {
        return py::bytes(reinterpret_cast<const char*>(c.call->data()), c.call->size());
      })
      .def_property_readonly("timeout_us", [](const PyCall& c) { return c.call->timeout_us; })
      .def_property_readonly("expired", [](const PyCall& c) { return c.call->expired(); });

  py::class_<RequestLog, std::shared_ptr<RequestLog>>(m, "RequestLog")
      .def(py::init([](const std::string& path, double rate, size_t max_pending) {
             return std::make_shared<RequestLog>(path, rate, max_pending);
           }),
           py::arg("path"), py::arg("sampling_rate"), py::arg("max_pending") = size_t(256) << 20)
      .def_readonly("path", &RequestLog::path)
      .def_readonly("sampling_rate", &RequestLog::rate)
      .def("sample", &RequestLog::sample)
      .def("submit_record", [](RequestLog& l, const py::bytes& rec) { return l.submit_record(std::string(rec)); })
      .def("flush", [](RequestLog& l) {
        py::gil_scoped_release nogil;
        l.flush();
      })
      .def("close", [](RequestLog& l) {
        py::gil_scoped_release nogil;
        l.close();
      })
      .def("stats", [](RequestLog& l) {
        py::dict d;
        d["written"] = l.written.load(); d["dropped"] = l.dropped.load(); d["bytes"] = l.bytes.load();
        return d;
      });

  py::class_<PyServer>(m, "Http2Server")
      .def(py::init([](const std::string& host, int port, int io_threads, size_t max_message) {
             auto p = std::make_unique<PyServer>();
             p->srv = std::make_unique<Server>(host, port, io_threads, max_message);
             p->fast = std::make_unique<FastPath>(p->srv.get());
             FastPath* fp = p->fast.get();
             p->srv->set_fast_dispatch([fp](std::unique_ptr<Call>& c) { return fp->try_dispatch(c); });
             p->srv->set_stream_reserve([fp](const ProbeInfo& pi) { return fp->reserve_stream(pi); });
             return p;
           }),
           py::arg("host"), py::arg("port"), py::arg("io_threads") = 4, py::arg("max_message") = size_t(2147483647))
      .def_property_readonly("port", [](const PyServer& s) { return s.srv->port(); })
      .def("start", [](PyServer& s) { s.srv->start(); })
      .def("stop", [](PyServer& s) {
        py::gil_scoped_release nogil;
        s.srv->stop();
      })
      .def("next_call", [](PyServer& s, int timeout_ms) -> py::object {
        std::unique_ptr<Call> c;
        {
          py::gil_scoped_release nogil;
          c = s.srv->next_call(timeout_ms);
        }
        if (!c) return py::none();
        auto pc = std::make_unique<PyCall>();
        pc->call = std::move(c);
        return py::cast(std::move(pc));
      }, py::arg("timeout_ms") = 100)
      .def("respond", [](PyServer& s, PyCall& c, int status, const std::string& message, const py::bytes& body) {
        if (!c.call) throw std::runtime_error("call already answered");
        std::string b = body;
        if (status == 4 && c.call->expired()) s.srv->stats.expired++;
        s.srv->respond(*c.call, status, message, std::move(b));
        c.call.reset();
      }, py::arg("call"), py::arg("status"), py::arg("message"), py::arg("body"))
      .def("stats", [](PyServer& s) {
        auto& st = s.srv->stats;
        py::dict d;
        d["connections"] = st.connections.load(); d["requests"] = st.requests.load();
        d["fast_path"] = st.fast_path.load(); d["slow_path"] = st.slow_path.load();
        d["streamed"] = st.streamed.load(); d["expired"] = st.expired.load(); d["direct_bytes"] = st.direct_bytes.load();
        d["responses"] = st.responses.load(); d["errors"] = st.errors.load();
        d["bytes_in"] = st.bytes_in.load(); d["bytes_out"] = st.bytes_out.load();
        d["io_s_recv"] = st.ns_recv.load() * 1e-9; d["io_s_h2"] = st.ns_h2.load() * 1e-9;
        d["io_s_dispatch"] = st.ns_dispatch.load() * 1e-9; d["io_s_send"] = st.ns_send.load() * 1e-9;
        d["recv_calls"] = st.recv_calls.load(); d["recv_empty"] = st.recv_empty.load();
        d["recv_bytes"] = st.recv_bytes.load();
        d["io_connections"] = s.srv->io_connections();
        return d;
      })
      // ---- fast path endpoints
      .def("add_endpoint", [](PyServer& s, const std::string& model, int64_t version, const std::string& sig,
                              const py::list& inputs, const py::list& outputs, int max_rows, int64_t timeout_us,
                              int max_wait_ms) {
        const int id = s.fast->next_id();
        auto ep = std::make_shared<Endpoint>(id, model, version, sig, specs_from(inputs), specs_from(outputs),
                                             max_rows, timeout_us, max_wait_ms);
        return s.fast->add_endpoint(ep);
      }, py::arg("model"), py::arg("version"), py::arg("signature"), py::arg("inputs"), py::arg("outputs"),
         py::arg("max_rows"), py::arg("timeout_us"), py::arg("max_wait_ms") = 200)
      .def("set_idle_dispatch", [](PyServer& s, int id, bool on) {
        auto ep = s.fast->endpoint(id);
        if (!ep) throw std::invalid_argument("no such endpoint");
        ep->set_idle_dispatch(on);
      })
      .def("set_endpoint_log", [](PyServer& s, int id, std::shared_ptr<RequestLog> log) {
        auto ep = s.fast->endpoint(id);
        if (!ep) throw std::invalid_argument("no such endpoint");
        ep->set_log(std::move(log));
      }, py::arg("endpoint"), py::arg("log").none(true))
      .def("endpoint_io_order", [](PyServer& s, int id) {
        auto ep = s.fast->endpoint(id);
        if (!ep) throw std::invalid_argument("no such endpoint");
        py::list ins, outs;
        for (auto& t : ep->inputs) ins.append(t.alias);
        for (auto& t : ep->outputs) outs.append(t.alias);
        return py::make_tuple(ins, outs);
      })
      .def("set_slot_buffers", [](PyServer& s, int id, int slot, const std::vector<uintptr_t>& in_ptrs,
                                  const std::vector<uintptr_t>& out_ptrs) {
        auto ep = s.fast->endpoint(id);
        if (!ep) throw std::invalid_argument("no such endpoint");
        // (empty lists: the slot has no buffers and is never opened again)
        if ((in_ptrs.size() != ep->inputs.size() || out_ptrs.size() != ep->outputs.size()) &&
            !(in_ptrs.empty() && out_ptrs.empty()))
          throw std::invalid_argument("buffer count mismatch");
        std::vector<uint8_t*> in;
        std::vector<const uint8_t*> out;
        for (auto p : in_ptrs) in.push_back(reinterpret_cast<uint8_t*>(p));
        for (auto p : out_ptrs) out.push_back(reinterpret_cast<const uint8_t*>(p));
        ep->set_slot_buffers(slot, in, out);
      })
      .def("set_route", [](PyServer& s, const std::string& model, const std::string& sig, int64_t version, int id) {
        s.fast->set_route(model, sig, version, id);
      })
      .def("clear_routes", [](PyServer& s, const std::string& model) { s.fast->clear_routes(model); })
      .def("remove_endpoint", [](PyServer& s, int id) {
        py::gil_scoped_release nogil;
        s.fast->remove_endpoint(id);   // closes the endpoint: its native lanes see acquire() < 0
        s.join_lanes(id);
      })
      .def("start_native_lane", [](PyServer& s, int id, int slot, int device, uintptr_t stream,
                                   const py::list& buckets) {
        auto ep = s.fast->endpoint(id);
        if (!ep || buckets.empty() || !hip_rt().load()) return false;
        auto parse = [](const py::list& l) {
          std::vector<LaneBucket> bs;
          for (auto item : l) {
            auto t = item.cast<py::tuple>();
            LaneBucket b;
            b.rows = t[0].cast<int>();
            b.exec = reinterpret_cast<void*>(t[1].cast<uintptr_t>());
            for (auto c : t[2].cast<py::list>()) {
              auto ct = c.cast<py::tuple>();
              b.in.push_back({ct[0].cast<uintptr_t>(), ct[1].cast<uintptr_t>(), ct[2].cast<size_t>()});
            }
            for (auto c : t[3].cast<py::list>()) {
              auto ct = c.cast<py::tuple>();
              b.out.push_back({ct[0].cast<uintptr_t>(), ct[1].cast<uintptr_t>(), ct[2].cast<size_t>()});
            }
            bs.push_back(std::move(b));
          }
          return bs;
        };
        std::lock_guard<std::mutex> g(s.lmu);
        s.lanes.push_back(std::make_unique<NativeLane>(s.srv.get(), ep, slot, device, reinterpret_cast<void*>(stream),
                                                       parse(buckets)));
        return true;
      }, py::arg("endpoint"), py::arg("slot"), py::arg("device"), py::arg("stream"), py::arg("buckets"))
      .def("enable_router", [](PyServer& s, const std::string& group, int rank, int world, int ncells,
                               size_t req_cap, size_t resp_cap, int margin) {
        if (s.router) throw std::runtime_error("router already enabled");
        s.router = std::make_unique<Router>(s.srv.get(), group, rank, world, ncells, req_cap, resp_cap, margin);
        s.srv->set_router(s.router.get());
        s.router->start();
      }, py::arg("group"), py::arg("rank"), py::arg("world"), py::arg("ncells") = 64,
         py::arg("req_cap") = size_t(1) << 20, py::arg("resp_cap") = size_t(64) << 10, py::arg("margin") = 8)
      .def("set_router_local_cap", [](PyServer& s, int64_t cap) {
        if (s.router) s.router->set_local_cap(cap);
      })
      .def("stop_router", [](PyServer& s) {
        py::gil_scoped_release nogil;
        if (s.router) s.router->stop();
      })
      .def("router_stats", [](PyServer& s) {
        py::dict d;
        if (!s.router) return d;
        auto& st = s.router->stats;
        d["forwarded"] = st.forwarded.load(); d["streamed"] = st.streamed.load();
        d["ingested"] = st.ingested.load(); d["returned"] = st.returned.load();
        d["reclaimed"] = st.reclaimed.load(); d["lost"] = st.lost.load(); d["no_cell"] = st.no_cell.load();
        d["rerun"] = st.rerun.load(); d["too_large"] = st.too_large.load(); d["tomb_freed"] = st.tomb_freed.load(); d["unseen_origin"] = st.unseen_origin.load();
        d["orphaned"] = st.orphaned.load();
        d["local_cap"] = s.router->local_cap();
        d["peers_alive"] = s.router->peers_alive();
        d["loads"] = s.router->loads();
        d["rank"] = s.router->rank();
        return d;
      })
      .def("load", [](PyServer& s) { return s.srv->load(); })
      .def("set_tracing", [](PyServer&, bool on) { trace_buf().on = on; })
      .def("drain_trace", [](PyServer&) {
        py::list out;
        for (auto& t : trace_buf().drain())
          out.append(py::make_tuple(t.endpoint, t.slot, t.rows, t.opened_us, t.acquired_us, t.issued_us,
                                    t.done_us, t.posted_us));
        return out;
      })
      .def_static("now_us", []() { return us_of(Clock::now()); })
      .def("native_lane_stats", [](PyServer& s) {
        std::lock_guard<std::mutex> g(s.lmu);
        py::list out;
        for (auto& l : s.lanes)
          out.append(py::make_tuple(l->endpoint_id(), l->batches.load(), l->errors.load(), l->dead.load()));
        return out;
      })
      .def("acquire", [](PyServer& s, int id, int slot, int timeout_ms) {
        auto ep = s.fast->endpoint(id, true);
        if (!ep) return -1;
        py::gil_scoped_release nogil;
        return ep->acquire(slot, timeout_ms);
      })
      .def("complete", [](PyServer& s, int id, int slot) {
        auto ep = s.fast->endpoint(id, true);
        if (!ep) return;
        py::gil_scoped_release nogil;
        ep->complete(slot, *s.srv);
      })
      .def("fail", [](PyServer& s, int id, int slot, int code, const std::string& msg) {
        auto ep = s.fast->endpoint(id, true);
        if (!ep) return;
        py::gil_scoped_release nogil;
        ep->fail(slot, *s.srv, code, msg);
      })
      .def("endpoint_stats", [](PyServer& s, int id) {
        auto ep = s.fast->endpoint(id);
        py::dict d;
        if (!ep) return d;
        auto st = ep->stats();
        d["requests"] = st.requests; d["batches"] = st.batches; d["rows"] = st.rows; d["rejected"] = st.rejected;
        d["failed"] = st.failed; d["consecutive_failed"] = st.consecutive_failed;
        d["pooled_drains"] = st.pooled_drains; d["copy_errors"] = st.copy_errors;
        return d;
      });

  py::class_<LoadGen>(m, "LoadGen")
      .def(py::init([](const std::string& host, int port, const std::string& method, const py::list& bodies,
                       int concurrency, int connections, int threads) {
             std::vector<std::string> b;
             for (auto x : bodies) b.push_back(x.cast<std::string>());
             py::gil_scoped_release nogil;
             return std::make_unique<LoadGen>(host, port, method, b, concurrency, connections, threads);
           }),
           py::arg("host"), py::arg("port"), py::arg("method"), py::arg("bodies"), py::arg("concurrency") = 64,
           py::arg("connections") = 8, py::arg("threads") = 4)
      .def("run", [](LoadGen& lg, uint64_t total, double timeout_s) {
        LoadGenResult r;
        {
          py::gil_scoped_release nogil;
          r = lg.run(total, timeout_s);
        }
        py::dict d;
        d["ok"] = r.ok; d["errors"] = r.errors; d["elapsed_s"] = r.elapsed_s;
        d["latency_us"] = r.latency_us; d["first_error"] = r.first_error;
        d["bytes_sent"] = r.bytes_sent; d["bytes_recv"] = r.bytes_recv; d["cpu_s"] = r.cpu_s;
        return d;
      }, py::arg("total"), py::arg("timeout_s") = 120.0)
      .def("start", [](LoadGen& lg) {
        py::gil_scoped_release nogil;
        lg.start();
      })
      .def("completed", [](LoadGen& lg) { return lg.completed(); })
      .def("window", [](LoadGen& lg, uint64_t n, double timeout_s) {
        LoadGenResult r;
        {
          py::gil_scoped_release nogil;
          r = lg.window(n, timeout_s);
        }
        py::dict d;
        d["ok"] = r.ok; d["errors"] = r.errors; d["elapsed_s"] = r.elapsed_s;
        d["latency_us"] = r.latency_us; d["first_error"] = r.first_error;
        d["done_s"] = r.done_s;
        return d;
      }, py::arg("n"), py::arg("timeout_s") = 120.0)
      .def("stop", [](LoadGen& lg, double timeout_s) {
        LoadGenResult r;
        {
          py::gil_scoped_release nogil;
          r = lg.stop(timeout_s);
        }
        py::dict d;
        d["ok"] = r.ok; d["errors"] = r.errors; d["first_error"] = r.first_error;
        d["bytes_sent"] = r.bytes_sent; d["bytes_recv"] = r.bytes_recv; d["cpu_s"] = r.cpu_s;
        return d;
      }, py::arg("timeout_s") = 30.0);

  m.def("run_loadgen", [](const std::string& host, int port, const std::string& method, const py::list& bodies,
                          uint64_t total, int concurrency, int connections, int threads, double timeout_s) {
    std::vector<std::string> b;
    for (auto x : bodies) b.push_back(x.cast<std::string>());
    LoadGenResult r;
    {
      py::gil_scoped_release nogil;
      r = run_loadgen(host, port, method, b, total, concurrency, connections, threads, timeout_s);
    }
    py::dict d;
    d["ok"] = r.ok; d["errors"] = r.errors; d["elapsed_s"] = r.elapsed_s;
    d["latency_us"] = r.latency_us; d["first_error"] = r.first_error;
    d["bytes_sent"] = r.bytes_sent; d["bytes_recv"] = r.bytes_recv; d["cpu_s"] = r.cpu_s;
    return d;
  }, py::arg("host"), py::arg("port"), py::arg("method"), py::arg("bodies"), py::arg("total"),
     py::arg("concurrency") = 64, py::arg("connections") = 8, py::arg("threads") = 4, py::arg("timeout_s") = 120.0);
}
