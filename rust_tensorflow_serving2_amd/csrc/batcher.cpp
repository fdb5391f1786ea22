// Predict fast path + dynamic batching into pinned slots (see batcher.h).
#include "batcher.h"

#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <condition_variable>
#include <cstring>
#include <functional>
#include <thread>

namespace tfs {

namespace {

// Helpers for drain_queue(): when a slot frees up with requests parked in the
// queue, their rows (602 KB fp32 -> 301 KB bf16 each for ResNet-50) used to
// be converted one after another on the lane thread that freed the slot -- a
// full batch of them took ~2 ms on that one thread, and a server with more
// requests in flight than its lanes hold ran 43.5k instead of 53.0k RPC/s
// (profiles/round5/s35).  The process-wide pool spreads a drain's copies over
// a few threads.  It is created when the first endpoint is (before any
// serving thread is pinned), and each pool thread sets its own CPU mask to
// the process-wide one (the main thread's): a pool first used from a lane
// thread pinned to one core would otherwise have inherited that single core
// and serialised the "parallel" copies behind the lane (round-5 ADVICE).
// Jobs run inside a try block and always count down their latch (a throwing
// job neither ends the process nor leaves the lane waiting).  Detached and
// leaked on purpose: no joinable std::thread is left for static destruction.
class DrainPool {
 public:
  explicit DrainPool(int n) {
    cpu_set_t mask;
    CPU_ZERO(&mask);
    const bool have_mask = sched_getaffinity(getpid(), sizeof(mask), &mask) == 0;   // the main thread's
    for (int i = 0; i < n; ++i) {
      std::thread([this, mask, have_mask] {
        pthread_setname_np(pthread_self(), "tfs-drain");
        if (have_mask) pthread_setaffinity_np(pthread_self(), sizeof(mask), &mask);
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [this] { return !jobs_.empty(); });
            job = std::move(jobs_.front());
            jobs_.pop_front();
          }
          try {
            job();
          } catch (...) {
            // the job's own guard has already counted its latch down
          }
        }
      }).detach();
    }
  }
  void post(std::function<void()> job) {
    {
      std::lock_guard<std::mutex> g(mu_);
      jobs_.push_back(std::move(job));
    }
    cv_.notify_one();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> jobs_;
};

constexpr int kDrainThreads = 3;      // + the calling lane thread
constexpr int kDrainMinJobs = 4;      // below this a drain stays on the caller

DrainPool& drain_pool() {
  static DrainPool* pool = new DrainPool(kDrainThreads);
  return *pool;
}

// count-down latch shared by a drain's caller and its pool jobs (shared-owned:
// a pool thread may still be leaving its notify when the caller, woken, returns)
struct Latch {
  std::mutex m;
  std::condition_variable cv;
  int left = 0;
  void done() {
    std::lock_guard<std::mutex> g(m);
    if (--left == 0) cv.notify_all();
  }
};

}  // namespace

static const char* kPredictPath = "/tensorflow.serving.PredictionService/Predict";
// how long a ready batch waits for a row whose payload is still arriving
static constexpr std::chrono::milliseconds kStreamStall(200);

Endpoint::Endpoint(int id_, std::string model_, int64_t version_, std::string signature_,
                   std::vector<TensorSpecC> inputs_, std::vector<TensorSpecC> outputs_, int max_rows_,
                   int64_t timeout_us_, int max_wait_ms_)
    : id(id_), model(std::move(model_)), version(version_), signature(std::move(signature_)),
      inputs(std::move(inputs_)), outputs(std::move(outputs_)), max_rows(max_rows_), timeout_us(timeout_us_),
      max_wait_ms(max_wait_ms_) {
  drain_pool();   // created before any serving thread is pinned (see DrainPool)
}

void Endpoint::set_slot_buffers(int slot, std::vector<uint8_t*> in_base, std::vector<const uint8_t*> out_base) {
  std::lock_guard<std::mutex> g(mu_);
  if (slot >= int(slots_.size())) slots_.resize(slot + 1);
  slots_[slot].in_base = std::move(in_base);
  slots_[slot].out_base = std::move(out_base);
}

int Endpoint::open_slot_locked(int n) {
  if (open_ >= 0) {
    Slot& s = slots_[open_];
    if (s.reserved + n <= max_rows) return open_;
    s.state = kReady;
    open_ = -1;
    s.cv->notify_all();
  }
  const int N = int(slots_.size());
  for (int k = 0; k < N; ++k) {
    const int idx = (next_ + k) % N;
    if (slots_[idx].state == kFree && !slots_[idx].in_base.empty()) {
      Slot& s = slots_[idx];
      s.state = kOpen;
      s.first = Clock::now();
      s.reserved = s.copied = 0;
      open_ = idx;
      next_ = (idx + 1) % N;
      s.cv->notify_all();   // the lane starts its batch-timeout clock
      return idx;
    }
  }
  return -1;
}

int Endpoint::offer(std::unique_ptr<Call>& call, PredictRequestView& req) {
  if (req.inputs.size() != inputs.size()) return 1;
  if (call->expired()) {
    if (srv_) {
      srv_->stats.expired++;
      srv_->respond(*call, 4 /*DEADLINE_EXCEEDED*/, "Deadline Exceeded", std::string());
      return 0;
    }
  }
  // match aliases (inputs sorted by alias on registration)
  std::vector<TensorView*> tv(inputs.size(), nullptr);
  for (auto& kv : req.inputs) {
    bool found = false;
    for (size_t i = 0; i < inputs.size(); ++i) {
      if (inputs[i].alias == kv.first) {
        tv[i] = &kv.second;
        found = true;
        break;
      }
    }
    if (!found) return 1;
  }
  int n = -1;
  for (size_t i = 0; i < inputs.size(); ++i) {
    const TensorView& t = *tv[i];
    const TensorSpecC& s = inputs[i];
    if (t.dtype != s.dtype || t.shape.size() != s.row_shape.size() + 1) return 1;
    if (t.storage != Storage::kView && t.storage != Storage::kOwned) return 1;
    for (size_t d = 0; d < s.row_shape.size(); ++d)
      if (t.shape[d + 1] != s.row_shape[d]) return 1;
    const int64_t rows = t.shape[0];
    if (rows < 1 || rows > max_rows) return 1;
    if (n < 0) n = int(rows);
    if (rows != n) return 1;
    if (t.count != size_t(rows) * s.row_elems) return 1;
    if (t.nbytes != size_t(rows) * s.row_bytes) return 1;
  }
  std::vector<int> outs;
  for (auto& a : req.output_filter) {
    int found = -1;
    for (size_t j = 0; j < outputs.size(); ++j)
      if (outputs[j].alias == a) found = int(j);
    if (found < 0) return 1;
    for (int o : outs)
      if (o == found) return 1;   // duplicate alias -> python reports it
    outs.push_back(found);
  }

  // the Call is heap-allocated and its body is never modified again, so these
  // pointers stay valid after the unique_ptr moves into a slot or the queue
  const uint8_t* body = call->data();
  std::vector<const uint8_t*> src(inputs.size());
  std::vector<std::string> owned;
  owned.reserve(inputs.size());   // no reallocation: src may point into (SSO) strings
  for (size_t i = 0; i < inputs.size(); ++i) {
    TensorView& t = *tv[i];
    if (t.storage == Storage::kView) {
      src[i] = body + t.offset;
    } else {
      owned.push_back(std::move(t.owned));
      src[i] = reinterpret_cast<const uint8_t*>(owned.back().data());
    }
  }
  int slot = -1, r0 = 0;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_) return 1;
    // FIFO: once anything is queued, later requests queue behind it
    if (!queue_.empty() || (slot = open_slot_locked(n)) < 0) {
      const size_t cap = max_queue_ ? max_queue_ : size_t(max_rows) * 64;
      if (queue_.size() >= cap) {
        st_.rejected++;
        return 2;
      }
      Queued q;
      q.call = std::move(call);
      q.n = n;
      q.outs = std::move(outs);
      q.owned = std::move(owned);   // vector move steals the element buffer: src stays valid
      q.src = std::move(src);
      queue_.push_back(std::move(q));
      st_.requests++;
      return 0;
    }
    Slot& s = slots_[slot];
    r0 = s.reserved;
    s.reserved += n;
    Pending p;
    p.row0 = r0;
    p.n = n;
    p.outs = std::move(outs);
    p.call = std::move(call);
    s.reqs.push_back(std::move(p));
    st_.requests++;
    if (s.reserved == max_rows) {
      s.state = kReady;
      open_ = -1;
    }
    ++copying_;
  }
  // copy outside the lock: IO threads fill different rows of a slot in parallel
  copy_rows(slot, r0, n, src);
  return 0;
}

// Caller incremented copying_ under mu_ when it reserved the rows.  Never
// throws: a copy that fails still completes the slot's bookkeeping (the lane
// is not left waiting for rows that will not come) and marks the request
// that owns rows r0.. failed, so it is answered INTERNAL instead of with the
// batch's output.
void Endpoint::copy_rows(int slot, int r0, int n, const std::vector<const uint8_t*>& src) noexcept {
  Slot& s = slots_[slot];
  bool ok = true;
  try {
    for (size_t i = 0; i < inputs.size(); ++i)
      ingest_rows(s.in_base[i] + size_t(r0) * inputs[i].slot_bytes(), src[i], size_t(n) * inputs[i].row_bytes,
                  inputs[i].conv);
  } catch (...) {
    ok = false;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (!ok) {
    st_.copy_errors++;
    for (auto& p : s.reqs)
      if (p.row0 == r0) p.failed = true;
  }
  s.copied += n;
  try {
    s.ready.emplace_back(r0, n);
  } catch (...) {
    // (only streamed rows consult `ready`; the batch still completes on `copied`)
  }
  s.cv->notify_all();
  if (--copying_ == 0 && closed_) cv_free_.notify_all();
}

void Endpoint::drain_queue() {
  struct Job {
    int slot, r0, n;
    std::vector<const uint8_t*> src;
    std::vector<std::string> owned;
  };
  std::vector<Job> jobs;
  {
    std::lock_guard<std::mutex> lk(mu_);
    while (!queue_.empty() && !closed_) {
      Queued& q = queue_.front();
      const int slot = open_slot_locked(q.n);
      if (slot < 0) break;
      Slot& s = slots_[slot];
      Job j{slot, s.reserved, q.n, std::move(q.src), std::move(q.owned)};
      s.reserved += q.n;
      Pending p;
      p.row0 = j.r0;
      p.n = q.n;
      p.outs = std::move(q.outs);
      p.call = std::move(q.call);
      s.reqs.push_back(std::move(p));
      if (s.reserved == max_rows) {
        s.state = kReady;
        open_ = -1;
      }
      queue_.pop_front();
      jobs.push_back(std::move(j));
      ++copying_;
    }
  }
  if (int(jobs.size()) < kDrainMinJobs) {
    for (auto& j : jobs) copy_rows(j.slot, j.r0, j.n, j.src);
    return;
  }
  // contiguous shares: the caller takes the first, the pool the rest; the
  // caller waits for all of them (the jobs' sources live in `jobs`).
  // copy_rows never throws, and a job's latch count-down runs from a guard,
  // so the wait below always ends.
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.pooled_drains++;
  }
  const auto latch = std::make_shared<Latch>();
  const Job* js = jobs.data();
  const int parts = kDrainThreads + 1;
  const int per = (int(jobs.size()) + parts - 1) / parts;
  for (int b = per; b < int(jobs.size()); b += per) {
    const int e = std::min(int(jobs.size()), b + per);
    {
      std::lock_guard<std::mutex> g(latch->m);
      ++latch->left;
    }
    try {
      drain_pool().post([this, js, b, e, latch] {
        struct Done {
          Latch& l;
          ~Done() { l.done(); }
        } done{*latch};
        for (int i = b; i < e; ++i) copy_rows(js[i].slot, js[i].r0, js[i].n, js[i].src);
      });
    } catch (...) {
      // could not queue the share: copy it here
      for (int i = b; i < e; ++i) copy_rows(js[i].slot, js[i].r0, js[i].n, js[i].src);
      latch->done();
    }
  }
  for (int i = 0; i < std::min(per, int(jobs.size())); ++i) copy_rows(js[i].slot, js[i].r0, js[i].n, js[i].src);
  std::unique_lock<std::mutex> g(latch->m);
  latch->cv.wait(g, [&latch] { return latch->left == 0; });
}

// ---------------------------------------------------------------- streaming rows
void SlotStream::commit(std::unique_ptr<Call> call) { ep->commit_stream(*this, std::move(call)); }
void SlotStream::abandon() { ep->abandon_stream(*this); }
bool SlotStream::keep_header() const { return ep->logging(); }

std::shared_ptr<StreamRes> Endpoint::reserve_stream(const std::shared_ptr<Endpoint>& self, const ProbeInfo& pi) {
  // the same acceptance rules as offer(), on the header alone
  if (inputs.size() != 1) return nullptr;
  const TensorSpecC& in = inputs[0];
  // a logged request is recorded from its bytes as received: with a converting
  // row those are gone, so logged endpoints buffer such requests instead
  if (in.conv && logging()) return nullptr;
  if (pi.alias != in.alias || pi.dtype != in.dtype || pi.shape.size() != in.row_shape.size() + 1) return nullptr;
  for (size_t d = 0; d < in.row_shape.size(); ++d)
    if (pi.shape[d + 1] != in.row_shape[d]) return nullptr;
  const int64_t rows = pi.shape[0];
  if (rows < 1 || rows > max_rows || pi.payload_len != size_t(rows) * in.row_bytes) return nullptr;
  auto r = std::make_shared<SlotStream>();
  std::lock_guard<std::mutex> lk(mu_);
  if (closed_ || !queue_.empty()) return nullptr;   // keep FIFO order behind queued requests
  const int n = int(rows);
  const int slot = open_slot_locked(n);
  if (slot < 0) return nullptr;
  Slot& s = slots_[slot];
  const int r0 = s.reserved;
  s.reserved += n;
  Pending p;
  p.row0 = r0;
  p.n = n;
  p.sres = r;
  s.reqs.push_back(std::move(p));
  st_.requests++;
  if (s.reserved == max_rows) {
    s.state = kReady;
    open_ = -1;
  }
  r->ep = self;
  r->slot = slot;
  r->idx = int(s.reqs.size()) - 1;
  r->n = n;
  r->dst = s.in_base[0] + size_t(r0) * in.slot_bytes();
  r->len = pi.payload_len;
  r->conv = in.conv;
  return r;
}

void Endpoint::commit_stream(SlotStream& r, std::unique_ptr<Call> call) {
  int expect = 0;
  if (!r.state.compare_exchange_strong(expect, 1)) {
    // the batcher gave the row up (payload stalled): the rows ran as padding
    if (srv_) srv_->respond(*call, 14 /*UNAVAILABLE*/, "request payload arrived too slowly for its batch",
                            std::string());
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  Slot& s = slots_[r.slot];
  s.reqs[r.idx].call = std::move(call);
  s.copied += r.n;
  s.ready.emplace_back(s.reqs[r.idx].row0, r.n);
  s.cv->notify_all();
}

void Endpoint::abandon_stream(SlotStream& r) {
  int expect = 0;
  if (!r.state.compare_exchange_strong(expect, 2)) return;
  std::lock_guard<std::mutex> g(mu_);
  Slot& s = slots_[r.slot];
  s.copied += r.n;   // the row runs as padding; complete() skips it (no call)
  if (s.copied == s.reserved) s.cv->notify_all();
}

void Endpoint::abandon_stalled_locked(Slot& s) {
  for (auto& p : s.reqs) {
    if (!p.sres) continue;
    int expect = 0;
    if (!p.sres->state.compare_exchange_strong(expect, 2)) continue;
    s.copied += p.n;
    while (p.sres->writers.load() != 0) {}   // an in-flight chunk copy finishes in microseconds
  }
}

int Endpoint::poll_slot_locked(int slot, Clock::time_point now, Clock::time_point& wake) {
  Slot& s = slots_[slot];
  if (s.state == kReady && s.reserved > 0 && s.copied == s.reserved) {
    s.state = kRunning;
    ++running_;
    st_.batches++;
    st_.rows += s.reserved;
    return s.reserved;
  }
  if (s.state == kReady && s.reserved > 0) {
    // rows still streaming in: give a stalled sender kStreamStall, then run without it
    const auto stall = s.first + std::chrono::microseconds(timeout_us) + kStreamStall;
    if (now >= stall) {
      abandon_stalled_locked(s);
      return -1;
    }
    wake = std::min(wake, stall);
    return 0;
  }
  if (s.state == kOpen && s.reserved > 0) {
    const auto due = s.first + std::chrono::microseconds(timeout_us);
    if (now >= due || (idle_dispatch_ && running_ == 0 && s.copied == s.reserved)) {
      s.state = kReady;
      if (open_ == slot) open_ = -1;
      return -1;
    }
    wake = std::min(wake, due);
  }
  return 0;
}

int Endpoint::acquire(int slot, int timeout_ms, std::vector<std::pair<int, int>>* ranges) {
  std::unique_lock<std::mutex> lk(mu_);
  if (slot < 0 || slot >= int(slots_.size())) return -1;
  const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
  while (!closed_) {
    Slot& s = slots_[slot];
    const auto now = Clock::now();
    if (ranges && !s.ready.empty()) {
      ranges->insert(ranges->end(), s.ready.begin(), s.ready.end());
      s.ready.clear();
      // hand the rows over now unless this already completes the batch
      if (!(s.state == kReady && s.reserved > 0 && s.copied == s.reserved)) return 0;
    }
    auto wake = deadline;
    const int r = poll_slot_locked(slot, now, wake);
    if (r > 0) return r;
    if (r < 0) continue;
    if (now >= deadline) return 0;
    s.cv->wait_until(lk, wake);
  }
  return -1;
}

void Endpoint::complete(int slot, Server& srv) {
  Slot& s = slots_[slot];
  ModelSpecView spec;
  spec.name = model;
  spec.has_version = true;
  spec.version = version;
  spec.signature_name = signature;
  std::vector<OutTensor> outs;
  const auto now = Clock::now();
  std::shared_ptr<RequestLog> log;
  if (logging()) {
    std::lock_guard<std::mutex> g(mu_);
    log = log_;
  }
  for (auto& p : s.reqs) {
    if (!p.call) continue;   // abandoned streaming row
    if (p.failed) {
      srv.respond(*p.call, 13 /*INTERNAL*/, "request rows could not be copied into the batch", std::string());
      continue;
    }
    if (p.call->expired(now)) {
      srv.stats.expired++;
      srv.respond(*p.call, 4 /*DEADLINE_EXCEEDED*/, "Deadline Exceeded", std::string());
      continue;
    }
    outs.clear();
    const size_t nout = p.outs.empty() ? outputs.size() : p.outs.size();
    for (size_t k = 0; k < nout; ++k) {
      const int j = p.outs.empty() ? int(k) : p.outs[k];
      const TensorSpecC& o = outputs[j];
      OutTensor t;
      t.alias = o.alias;
      t.dtype = o.dtype;
      t.shape.push_back(p.n);
      t.shape.insert(t.shape.end(), o.row_shape.begin(), o.row_shape.end());
      t.data = s.out_base[j] + size_t(p.row0) * o.row_bytes;
      t.count = size_t(p.n) * o.row_elems;
      outs.push_back(std::move(t));
    }
    std::string body = encode_predict_response(&spec, outs, false);
    if (log && log->sample()) {
      // the request message as received: a streamed one is its header bytes +
      // the payload sitting in this slot's row (not yet reused)
      if (p.sres) {
        // (a converted row no longer holds the request's fp32 bytes: such a
        // stream is not reserved while logging is on, see reserve_stream)
        if (p.call->head.size() > 5 && !p.sres->conv)
          log->submit_predict(spec, p.call->head.substr(5),
                              std::string(reinterpret_cast<const char*>(p.sres->dst), p.sres->len), body);
      } else {
        log->submit_predict(spec, std::string(reinterpret_cast<const char*>(p.call->data()), p.call->size()),
                            std::string(), body);
      }
    }
    srv.respond(*p.call, 0, std::string(), std::move(body));
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    s.reqs.clear();
    s.ready.clear();
    s.reserved = s.copied = 0;
    if (s.state == kRunning) --running_;
    s.state = kFree;
    st_.consecutive_failed = 0;
    if (running_ == 0 && open_ >= 0) slots_[open_].cv->notify_all();   // idle dispatch
    cv_free_.notify_all();
  }
  drain_queue();
}

void Endpoint::fail(int slot, Server& srv, int code, const std::string& msg) {
  Slot& s = slots_[slot];
  for (auto& p : s.reqs)
    if (p.call) srv.respond(*p.call, code, msg, std::string());
  {
    std::lock_guard<std::mutex> g(mu_);
    s.reqs.clear();
    s.ready.clear();
    s.reserved = s.copied = 0;
    if (s.state == kRunning) --running_;
    s.state = kFree;
    st_.failed++;
    st_.consecutive_failed++;
    if (running_ == 0 && open_ >= 0) slots_[open_].cv->notify_all();
    cv_free_.notify_all();
  }
  drain_queue();
}

void Endpoint::fail_dead(int slot, Server& srv, int code, const std::string& msg) {
  Slot& s = slots_[slot];
  for (auto& p : s.reqs)
    if (p.call) srv.respond(*p.call, code, msg, std::string());
  std::lock_guard<std::mutex> g(mu_);
  s.reqs.clear();
  s.ready.clear();
  if (s.state == kRunning) --running_;
  s.state = kDead;
  st_.failed++;
  st_.consecutive_failed++;
  cv_free_.notify_all();
}

void Endpoint::close(Server* srv) {
  std::deque<Queued> left;
  std::vector<std::unique_ptr<Call>> unstarted;
  {
    std::unique_lock<std::mutex> g(mu_);
    closed_ = true;
    for (auto& s : slots_) abandon_stalled_locked(s);
    left.swap(queue_);
    // requests sitting in slots no lane has started: their lanes see
    // acquire() < 0 and exit, so nobody else would ever answer them
    for (auto& s : slots_) {
      if (s.state != kOpen && s.state != kReady) continue;
      for (auto& p : s.reqs)
        if (p.call) unstarted.push_back(std::move(p.call));
      s.reqs.clear();
      s.ready.clear();
      s.reserved = s.copied = 0;
      s.state = kFree;
    }
    open_ = -1;
    for (auto& sl : slots_) sl.cv->notify_all();
    cv_free_.notify_all();
    // IO threads may still be copying rows (reserved before closed_ was set)
    // into the pinned buffers: the caller frees those once this returns
    cv_free_.wait(g, [this] { return copying_ == 0; });
  }
  if (srv) {
    for (auto& q : left) srv->respond(*q.call, 14 /*UNAVAILABLE*/, "Servable is being unloaded", std::string());
    for (auto& c : unstarted) srv->respond(*c, 14 /*UNAVAILABLE*/, "Servable is being unloaded", std::string());
  }
}

EndpointStats Endpoint::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return st_;
}

// ---------------------------------------------------------------- FastPath
static std::string route_key(const std::string& m, const std::string& s, int64_t v) {
  std::string k = m;
  k.push_back('\0');
  k += s;
  k.push_back('\0');
  k += v < 0 ? std::string("L") : std::to_string(v);
  return k;
}

std::shared_ptr<Endpoint> FastPath::route(const ModelSpecView& spec) {
  if (spec.has_label) return nullptr;
  const std::string sig = spec.signature_name.empty() ? "serving_default" : spec.signature_name;
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = routes_.find(route_key(spec.name, sig, spec.has_version ? spec.version : -1));
  if (it == routes_.end()) return nullptr;
  auto e = eps_.find(it->second);
  return e == eps_.end() ? nullptr : e->second;
}

std::shared_ptr<StreamRes> FastPath::reserve_stream(const ProbeInfo& pi) {
  auto ep = route(pi.spec);
  return ep ? ep->reserve_stream(ep, pi) : nullptr;
}

bool FastPath::try_dispatch(std::unique_ptr<Call>& call) {
  if (call->method != kPredictPath) return false;
  PredictRequestView req;
  try {
    parse_predict_request(call->data(), call->size(), req);
  } catch (const std::exception&) {
    return false;   // python path reports the precise error
  }
  if (!req.has_spec || req.spec.has_label) return false;
  const std::string sig = req.spec.signature_name.empty() ? "serving_default" : req.spec.signature_name;
  std::shared_ptr<Endpoint> ep;
  {
    std::shared_lock<std::shared_mutex> g(mu_);
    auto it = routes_.find(route_key(req.spec.name, sig, req.spec.has_version ? req.spec.version : -1));
    if (it == routes_.end()) return false;
    auto e = eps_.find(it->second);
    if (e == eps_.end()) return false;
    ep = e->second;
  }
  const int r = ep->offer(call, req);
  if (r == 0) return true;
  if (r == 2) {
    srv_->respond(*call, 14 /*UNAVAILABLE*/, "The batch scheduling queue is full", std::string());
    return true;
  }
  return false;
}

int FastPath::add_endpoint(std::shared_ptr<Endpoint> ep) {
  ep->set_server(srv_);
  std::unique_lock<std::shared_mutex> g(mu_);
  eps_[ep->id] = ep;
  return ep->id;
}

std::shared_ptr<Endpoint> FastPath::endpoint(int id, bool retired) {
  std::shared_lock<std::shared_mutex> g(mu_);
  auto it = eps_.find(id);
  if (it != eps_.end()) return it->second;
  if (!retired) return nullptr;
  auto r = retired_.find(id);
  return r == retired_.end() ? nullptr : r->second;
}

void FastPath::remove_endpoint(int id) {
  std::shared_ptr<Endpoint> ep;
  {
    std::unique_lock<std::shared_mutex> g(mu_);
    for (auto it = routes_.begin(); it != routes_.end();) {
      if (it->second == id) it = routes_.erase(it);
      else ++it;
    }
    auto it = eps_.find(id);
    if (it != eps_.end()) {
      ep = it->second;
      eps_.erase(it);
      for (auto r = retired_.begin(); r != retired_.end();) {   // drop the ones nobody holds any more
        if (!r->second->busy()) r = retired_.erase(r);
        else ++r;
      }
      retired_[id] = ep;
    }
  }
  if (ep) ep->close(srv_);
}

void FastPath::set_route(const std::string& model, const std::string& signature, int64_t version, int ep_id) {
  std::unique_lock<std::shared_mutex> g(mu_);
  const std::string k = route_key(model, signature, version);
  if (ep_id < 0) routes_.erase(k);
  else routes_[k] = ep_id;
}

void FastPath::clear_routes(const std::string& model) {
  std::unique_lock<std::shared_mutex> g(mu_);
  const std::string prefix = model + std::string(1, '\0');
  for (auto it = routes_.begin(); it != routes_.end();) {
    if (it->first.compare(0, prefix.size(), prefix) == 0) it = routes_.erase(it);
    else ++it;
  }
}

}  // namespace tfs
