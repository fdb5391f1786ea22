// Cross-replica request routing over POSIX shared memory (see router.h).
#include "router.h"

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <pthread.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace tfs {

namespace {

constexpr uint64_t kMagic = 0x7466735f726f7574ULL;   // "tfs_rout"
constexpr int kMaxRanks = 64;
constexpr size_t kMethodCap = 256, kErrCap = 256;
enum CellState : uint32_t { kFree = 0, kWriting = 1, kReady = 2, kTaken = 3, kDone = 4 };
// CellHdr::status of a DONE cell whose answer did not fit the cell's response
// area: the origin runs the call itself (its message is still in the cell)
constexpr int32_t kRerunLocally = -1;

struct alignas(64) SegHdr {
  uint64_t magic;
  uint32_t rank, gen;
  int32_t pid;
  uint32_t ncells;
  uint64_t req_cap, resp_cap, stride;
  alignas(64) std::atomic<uint64_t> heartbeat;
  alignas(64) std::atomic<int64_t> load;
  alignas(64) std::atomic<uint32_t> doorbell;    // futex word: a cell became READY here, or an answer DONE for us
  alignas(64) std::atomic<uint32_t> hint;        // where origins start looking for a free cell
};

struct alignas(64) CellHdr {
  std::atomic<uint32_t> state;
  uint32_t origin, origin_gen;
  uint32_t method_len;
  uint64_t token;
  uint64_t msg_len;
  int64_t timeout_us, arrival_ns;
  int32_t status;
  uint32_t err_len;
  uint64_t resp_len;
};

// directory: rank -> current generation / pid (gen 0 = never started)
struct Dir {
  std::atomic<uint32_t> gen[kMaxRanks];
  std::atomic<int32_t> pid[kMaxRanks];
};

static_assert(std::atomic<uint32_t>::is_always_lock_free && std::atomic<int64_t>::is_always_lock_free,
              "shared-memory atomics must be address-free");

long futex(std::atomic<uint32_t>* w, int op, uint32_t val, const timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), op, val, ts, nullptr, 0);
}

std::string seg_name(const std::string& group, int rank, uint32_t gen) {
  return "/tfs_" + group + "_r" + std::to_string(rank) + "_g" + std::to_string(gen);
}

bool pid_alive(int32_t pid) { return pid > 0 && (kill(pid, 0) == 0 || errno == EPERM); }

}  // namespace

struct RouterSeg {
  std::string name;
  void* base = nullptr;
  size_t len = 0;
  bool owner = false;
  SegHdr* hdr() const { return static_cast<SegHdr*>(base); }
  uint8_t* cell_base(int i) const {
    return static_cast<uint8_t*>(base) + sizeof(SegHdr) + size_t(i) * hdr()->stride;
  }
  CellHdr* cell(int i) const { return reinterpret_cast<CellHdr*>(cell_base(i)); }
  char* method(int i) const { return reinterpret_cast<char*>(cell_base(i) + sizeof(CellHdr)); }
  uint8_t* msg(int i) const { return cell_base(i) + sizeof(CellHdr) + kMethodCap; }
  char* err(int i) const { return reinterpret_cast<char*>(msg(i) + hdr()->req_cap); }
  uint8_t* resp(int i) const { return reinterpret_cast<uint8_t*>(err(i)) + kErrCap; }
  ~RouterSeg() {
    if (base) munmap(base, len);
    if (owner) shm_unlink(name.c_str());
  }
};

struct RouterDir {
  Dir* d = nullptr;
};

struct Router::Peer {
  uint32_t gen = 0;
  std::shared_ptr<RouterSeg> seg;
  bool alive = false;
  uint64_t last_hb = 0;
  Clock::time_point hb_at;
};

struct Router::Pending {
  int peer;
  std::shared_ptr<RouterSeg> seg;   // keeps the mapping while the call is out
  int cell;
  std::unique_ptr<Call> call;
};

// A call given up on (its peer looked dead while running it) whose cell the
// peer may still mark DONE later -- a stalled heartbeat, not a dead process.
// Nobody else frees such a cell, so the origin keeps the token and frees it.
struct Router::Tomb {
  int peer;
  std::shared_ptr<RouterSeg> seg;
  int cell;
  uint64_t token;
};

namespace {
// The message of a forwarded call, rebuilt as a local call (gRPC frame prefix + message)
void take_message(Call& c, const RouterSeg& s, int cell) {
  c.body.assign(5, '\0');
  c.body.append(reinterpret_cast<const char*>(s.msg(cell)), s.cell(cell)->msg_len);
  c.off = 5;
  c.routed = true;
}
}  // namespace

// A streamed Predict whose payload goes from the socket into a peer's cell.
struct RemoteStream final : StreamRes {
  Router* r = nullptr;
  int peer = -1, cell = -1;
  std::shared_ptr<RouterSeg> seg;
  bool remote() const override { return true; }
  void commit(std::unique_ptr<Call> call) override {
    int expect = 0;
    if (!state.compare_exchange_strong(expect, 1)) return;
    r->stats.streamed++;
    r->publish(peer, seg, cell, std::move(call));
  }
  void abandon() override {
    int expect = 0;
    if (!state.compare_exchange_strong(expect, 2)) return;
    while (writers.load() != 0) {}
    seg->cell(cell)->state.store(kFree, std::memory_order_release);
  }
};

Router::Router(Server* srv, const std::string& group, int rank, int world, int ncells, size_t req_cap,
               size_t resp_cap, int margin)
    : srv_(srv), group_(group), rank_(rank), world_(world), ncells_(ncells), margin_(margin),
      req_cap_((req_cap + 63) & ~size_t(63)), resp_cap_((resp_cap + 63) & ~size_t(63)) {
  if (rank < 0 || rank >= world || world > kMaxRanks || ncells < 1)
    throw std::invalid_argument("router: bad rank / world / ncells");
  for (char ch : group)
    if (!(isalnum(static_cast<unsigned char>(ch)) || ch == '_' || ch == '-'))
      throw std::invalid_argument("router: group name must be [A-Za-z0-9_-]");
  // directory (created by whichever replica comes first; zero-filled by ftruncate)
  dir_name_ = "/tfs_" + group + "_dir";
  int fd = shm_open(dir_name_.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("router: shm_open(dir) failed: " + std::string(strerror(errno)));
  struct stat sb {};
  fstat(fd, &sb);
  if (size_t(sb.st_size) < sizeof(Dir) && ftruncate(fd, sizeof(Dir)) != 0) {
    close(fd);
    throw std::runtime_error("router: ftruncate(dir) failed");
  }
  void* d = mmap(nullptr, sizeof(Dir), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (d == MAP_FAILED) throw std::runtime_error("router: mmap(dir) failed");
  dir_ = new RouterDir{static_cast<Dir*>(d)};
  // own segment, a new generation (a restarted replica never reuses a name peers may still map)
  const uint32_t gen = dir_->d->gen[rank].load() + 1;
  auto seg = std::make_shared<RouterSeg>();
  seg->name = seg_name(group, rank, gen);
  const size_t stride = sizeof(CellHdr) + kMethodCap + req_cap_ + kErrCap + resp_cap_;
  seg->len = sizeof(SegHdr) + size_t(ncells) * stride;
  shm_unlink(seg->name.c_str());
  fd = shm_open(seg->name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("router: shm_open(" + seg->name + ") failed: " + strerror(errno));
  if (ftruncate(fd, off_t(seg->len)) != 0) {
    close(fd);
    shm_unlink(seg->name.c_str());
    throw std::runtime_error("router: ftruncate(segment) failed (is /dev/shm large enough?)");
  }
  seg->base = mmap(nullptr, seg->len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (seg->base == MAP_FAILED) {
    seg->base = nullptr;
    shm_unlink(seg->name.c_str());
    throw std::runtime_error("router: mmap(segment) failed");
  }
  seg->owner = true;
  SegHdr* h = seg->hdr();
  new (h) SegHdr();
  h->rank = uint32_t(rank);
  h->gen = gen;
  h->pid = int32_t(getpid());
  h->ncells = uint32_t(ncells);
  h->req_cap = req_cap_;
  h->resp_cap = resp_cap_;
  h->stride = stride;
  for (int i = 0; i < ncells; ++i) new (seg->cell(i)) CellHdr();
  std::atomic_thread_fence(std::memory_order_release);
  h->magic = kMagic;
  self_ = seg;
  if (gen > 1) shm_unlink(seg_name(group, rank, gen - 1).c_str());   // the previous incarnation's ring
  dir_->d->pid[rank].store(int32_t(getpid()));
  dir_->d->gen[rank].store(gen, std::memory_order_release);
  peers_.resize(size_t(world));
  for (auto& p : peers_) p = std::make_unique<Peer>();
}

Router::~Router() {
  stop();
  if (dir_) {
    munmap(dir_->d, sizeof(Dir));
    delete dir_;
  }
}

std::atomic<int64_t>* Router::load_word() { return &self_->hdr()->load; }

void Router::start() {
  if (running_.exchange(true)) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    rescan();
  }
  th_ = std::thread([this] { run(); });
}

void Router::stop() {
  if (!running_.exchange(false)) return;
  SegHdr* h = self_->hdr();
  h->doorbell.fetch_add(1);
  futex(&h->doorbell, FUTEX_WAKE, INT32_MAX, nullptr);
  if (th_.joinable()) th_.join();
  // calls still out on peers: their clients get an answer now
  std::map<uint64_t, std::unique_ptr<Pending>> left;
  {
    std::lock_guard<std::mutex> g(mu_);
    left.swap(pending_);
  }
  for (auto& kv : left) srv_->respond(*kv.second->call, 14 /*UNAVAILABLE*/, "server shutting down", std::string());
  dir_->d->pid[rank_].store(0);
}

// ---------------------------------------------------------------- routing
int Router::pick(size_t msg_len) {
  if (msg_len > req_cap_ || world_ < 2) return -1;
  const int64_t mine = self_->hdr()->load.load(std::memory_order_relaxed);
  if (mine < local_cap_.load(std::memory_order_relaxed)) return -1;
  int best = -1;
  int64_t best_load = mine - margin_;
  std::lock_guard<std::mutex> g(mu_);
  for (int p = 0; p < world_; ++p) {
    if (p == rank_ || !peers_[p]->alive || !peers_[p]->seg) continue;
    const int64_t l = peers_[p]->seg->hdr()->load.load(std::memory_order_relaxed);
    if (l < best_load) {
      best_load = l;
      best = p;
    }
  }
  return best;
}

int Router::claim(RouterSeg& seg) {
  SegHdr* h = seg.hdr();
  const uint32_t n = h->ncells;
  const uint32_t start = h->hint.fetch_add(1, std::memory_order_relaxed);
  for (uint32_t k = 0; k < n; ++k) {
    const int i = int((start + k) % n);
    uint32_t expect = kFree;
    if (seg.cell(i)->state.compare_exchange_strong(expect, kWriting, std::memory_order_acq_rel)) return i;
  }
  return -1;
}

void Router::ring(RouterSeg& seg) {
  SegHdr* h = seg.hdr();
  h->doorbell.fetch_add(1, std::memory_order_release);
  futex(&h->doorbell, FUTEX_WAKE, INT32_MAX, nullptr);
}

// The cell's message bytes are in place: fill in the header, remember the
// client call and hand the cell to the peer.
void Router::publish(int p, const std::shared_ptr<RouterSeg>& seg, int cell, std::unique_ptr<Call> call) {
  CellHdr* ch = seg->cell(cell);
  const size_t ml = std::min(call->method.size(), kMethodCap);
  memcpy(seg->method(cell), call->method.data(), ml);
  ch->method_len = uint32_t(ml);
  ch->origin = uint32_t(rank_);
  ch->origin_gen = self_->hdr()->gen;
  ch->timeout_us = call->timeout_us;
  ch->arrival_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(call->arrival.time_since_epoch()).count();
  ch->status = 0;
  ch->err_len = 0;
  ch->resp_len = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    // tokens are unique across origins and incarnations (rank, generation,
    // sequence): an origin only ever collects a DONE cell that carries its own
    // token, so a cell freed and reused under a stale pending entry cannot
    // hand that entry another origin's answer
    const uint64_t tok = (uint64_t(rank_) << 56) | (uint64_t(self_->hdr()->gen & 0xffffff) << 32) |
                         (next_token_++ & 0xffffffffULL);
    ch->token = tok;
    auto pend = std::make_unique<Pending>();
    pend->peer = p;
    pend->seg = seg;
    pend->cell = cell;
    pend->call = std::move(call);
    pending_[tok] = std::move(pend);
  }
  seg->hdr()->load.fetch_add(1, std::memory_order_relaxed);   // outstanding on the peer from now on
  ch->state.store(kReady, std::memory_order_release);
  stats.forwarded++;
  ring(*seg);
}

bool Router::forward(std::unique_ptr<Call>& c) {
  const int p = pick(c->size());
  if (p < 0) return false;
  std::shared_ptr<RouterSeg> seg;
  {
    std::lock_guard<std::mutex> g(mu_);
    seg = peers_[p]->seg;
  }
  if (!seg) return false;
  const int cell = claim(*seg);
  if (cell < 0) {
    stats.no_cell++;
    return false;
  }
  seg->cell(cell)->msg_len = c->size();
  memcpy(seg->msg(cell), c->data(), c->size());
  publish(p, seg, cell, std::move(c));
  return true;
}

std::shared_ptr<StreamRes> Router::reserve_stream(const ProbeInfo& pi, const uint8_t* head, size_t head_len,
                                                  const std::string& method) {
  if (pi.payload_off < 5 || head_len < pi.payload_off || method.size() > kMethodCap) return nullptr;
  const size_t msg_len = pi.payload_off - 5 + pi.payload_len;   // the payload ends the message (wire.cpp probe)
  const int p = pick(msg_len);
  if (p < 0) return nullptr;
  std::shared_ptr<RouterSeg> seg;
  {
    std::lock_guard<std::mutex> g(mu_);
    seg = peers_[p]->seg;
  }
  if (!seg) return nullptr;
  const int cell = claim(*seg);
  if (cell < 0) {
    stats.no_cell++;
    return nullptr;
  }
  seg->cell(cell)->msg_len = msg_len;
  memcpy(seg->msg(cell), head + 5, pi.payload_off - 5);
  auto r = std::make_shared<RemoteStream>();
  r->r = this;
  r->peer = p;
  r->cell = cell;
  r->seg = seg;
  r->dst = seg->msg(cell) + (pi.payload_off - 5);
  r->len = pi.payload_len;
  return r;
}

// ---------------------------------------------------------------- serving peers' calls
void Router::respond_remote(const Call& c, int status, const std::string& msg, const std::string& body) {
  RouterSeg& s = *self_;
  CellHdr* ch = s.cell(int(c.cell));
  if (status == 0 && body.size() > s.hdr()->resp_cap) {
    // the answer does not fit the cell: the origin runs the call itself, so a
    // routed call succeeds exactly when the same call served locally would
    status = kRerunLocally;
    ch->err_len = 0;
    ch->resp_len = 0;
    stats.too_large++;
  } else {
    ch->err_len = uint32_t(std::min(msg.size(), kErrCap));
    memcpy(s.err(int(c.cell)), msg.data(), ch->err_len);
    ch->resp_len = status == 0 ? body.size() : 0;
    if (ch->resp_len) memcpy(s.resp(int(c.cell)), body.data(), body.size());
  }
  ch->status = status;
  const uint32_t origin = ch->origin;
  ch->state.store(kDone, std::memory_order_release);
  std::shared_ptr<RouterSeg> oseg;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (origin < peers_.size() && peers_[origin]->gen == ch->origin_gen) oseg = peers_[origin]->seg;
  }
  if (oseg) {
    ring(*oseg);
    return;
  }
  // this replica's view of the origin is stale (not re-scanned yet) or the
  // origin is gone.  Freeing the cell here (round 5) leaked the origin's call
  // whenever the view was merely stale: the origin waited forever, and once
  // another replica reused the cell, the stale entry took that replica's
  // answer (found by the 8-rank CPU rehearsal).  The cell stays DONE: a live
  // origin collects it on its next reap (its doorbell rings on other traffic
  // and every 20 ms wait times out); a dead origin's ring is reclaimed with
  // its generation.
  stats.unseen_origin++;
  std::shared_ptr<RouterSeg> any;
  {
    std::lock_guard<std::mutex> g(mu_);
    rescan();
    if (origin < peers_.size() && peers_[origin]->gen == ch->origin_gen) any = peers_[origin]->seg;
  }
  if (any) ring(*any);
}

void Router::ingest() {
  RouterSeg& s = *self_;
  const int n = int(s.hdr()->ncells);
  for (int i = 0; i < n; ++i) {
    CellHdr* ch = s.cell(i);
    if (ch->state.load(std::memory_order_acquire) != kReady) continue;
    uint32_t expect = kReady;
    if (!ch->state.compare_exchange_strong(expect, kTaken, std::memory_order_acq_rel)) continue;
    auto call = std::make_unique<Call>();
    call->method.assign(s.method(i), ch->method_len);
    call->ext = s.msg(i);
    call->ext_len = ch->msg_len;
    call->remote = this;
    call->cell = uint32_t(i);
    call->routed = true;
    call->load = &s.hdr()->load;   // the origin counted it in our load when it published
    call->timeout_us = ch->timeout_us;
    call->arrival = Clock::time_point(std::chrono::duration_cast<Clock::duration>(
        std::chrono::nanoseconds(ch->arrival_ns)));
    stats.ingested++;
    srv_->stats.requests++;
    srv_->dispatch(std::move(call));
  }
}

// ---------------------------------------------------------------- our forwarded calls
void Router::reap(bool check_peers) {
  struct Ans {
    std::unique_ptr<Call> call;
    int status;
    std::string msg, body;
  };
  std::vector<Ans> answers;
  std::vector<std::unique_ptr<Call>> rerun;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = pending_.begin(); it != pending_.end();) {
      Pending& pd = *it->second;
      RouterSeg& s = *pd.seg;
      CellHdr* ch = s.cell(pd.cell);
      const uint32_t st = ch->state.load(std::memory_order_acquire);
      if (ch->token != it->first && st != kWriting) {
        // the cell was freed and reused under this call (it cannot be ours
        // any more): answer it rather than wait forever or take another
        // origin's answer
        Ans a;
        a.call = std::move(pd.call);
        a.status = 14;   // UNAVAILABLE
        a.msg = "replica " + std::to_string(pd.peer) + " lost the forwarded request";
        answers.push_back(std::move(a));
        stats.orphaned++;
        it = pending_.erase(it);
        continue;
      }
      if (st == kDone) {
        if (ch->status == kRerunLocally) {
          std::unique_ptr<Call> c = std::move(pd.call);
          take_message(*c, s, pd.cell);
          ch->state.store(kFree, std::memory_order_release);
          rerun.push_back(std::move(c));
          stats.rerun++;
          it = pending_.erase(it);
          continue;
        }
        Ans a;
        a.call = std::move(pd.call);
        a.status = ch->status;
        a.msg.assign(s.err(pd.cell), ch->err_len);
        if (ch->status == 0) a.body.assign(reinterpret_cast<const char*>(s.resp(pd.cell)), ch->resp_len);
        ch->state.store(kFree, std::memory_order_release);
        answers.push_back(std::move(a));
        it = pending_.erase(it);
        continue;
      }
      const bool dead = check_peers && (!peers_[pd.peer]->alive || peers_[pd.peer]->seg != pd.seg);
      if (dead) {
        uint32_t expect = kReady;
        // READY -> TAKEN (not FREE) while the message is copied out: a replica
        // that still thinks the peer alive must not claim the cell meanwhile
        if (ch->state.compare_exchange_strong(expect, kTaken)) {
          std::unique_ptr<Call> c = std::move(pd.call);
          take_message(*c, s, pd.cell);
          ch->state.store(kFree, std::memory_order_release);
          rerun.push_back(std::move(c));
          stats.reclaimed++;
        } else {
          Ans a;
          a.call = std::move(pd.call);
          a.status = 14;   // UNAVAILABLE
          a.msg = "replica " + std::to_string(pd.peer) + " failed while serving the request";
          answers.push_back(std::move(a));
          stats.lost++;
          tombs_.push_back(Tomb{pd.peer, pd.seg, pd.cell, ch->token});
        }
        it = pending_.erase(it);
        continue;
      }
      ++it;
    }
    // abandoned calls: free the cell if the peer finishes after all; forget it
    // once the peer's process is gone or replaced (its ring goes with it)
    for (auto it = tombs_.begin(); it != tombs_.end();) {
      CellHdr* ch = it->seg->cell(it->cell);
      if (ch->token != it->token) {
        it = tombs_.erase(it);
        continue;
      }
      if (ch->state.load(std::memory_order_acquire) == kDone) {
        ch->state.store(kFree, std::memory_order_release);
        stats.tomb_freed++;
        it = tombs_.erase(it);
        continue;
      }
      if (check_peers && (peers_[it->peer]->seg != it->seg || !pid_alive(it->seg->hdr()->pid))) {
        it = tombs_.erase(it);
        continue;
      }
      ++it;
    }
  }
  for (auto& a : answers) {
    stats.returned++;
    srv_->respond(*a.call, a.status, std::move(a.msg), std::move(a.body));
  }
  for (auto& c : rerun) srv_->dispatch(std::move(c));
}

// (mu_ held) map peers' current generations, refresh liveness
void Router::rescan() {
  const auto now = Clock::now();
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    Peer& pr = *peers_[p];
    const uint32_t gen = dir_->d->gen[p].load(std::memory_order_acquire);
    if (gen != pr.gen && gen != 0) {
      auto seg = std::make_shared<RouterSeg>();
      seg->name = seg_name(group_, p, gen);
      const int fd = shm_open(seg->name.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat sb {};
        if (fstat(fd, &sb) == 0 && size_t(sb.st_size) >= sizeof(SegHdr)) {
          void* b = mmap(nullptr, size_t(sb.st_size), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
          if (b != MAP_FAILED) {
            seg->base = b;
            seg->len = size_t(sb.st_size);
          }
        }
        close(fd);
      }
      if (seg->base && seg->hdr()->magic == kMagic && seg->hdr()->gen == gen) {
        pr.seg = seg;
        pr.gen = gen;
        pr.last_hb = seg->hdr()->heartbeat.load();
        pr.hb_at = now;
      }
    }
    if (!pr.seg) {
      pr.alive = false;
      continue;
    }
    const uint64_t hb = pr.seg->hdr()->heartbeat.load(std::memory_order_relaxed);
    if (hb != pr.last_hb) {
      pr.last_hb = hb;
      pr.hb_at = now;
    }
    pr.alive = pid_alive(pr.seg->hdr()->pid) && now - pr.hb_at < std::chrono::seconds(2);
  }
}

// (mu_ held) answers in our ring that no origin will collect: the origin's
// process is gone or was replaced by a new generation.  Only those are freed
// (a live origin collects its own cells, however stale our view of it was).
void Router::collect_orphans() {
  RouterSeg& s = *self_;
  const int n = int(s.hdr()->ncells);
  for (int i = 0; i < n; ++i) {
    CellHdr* ch = s.cell(i);
    if (ch->state.load(std::memory_order_acquire) != kDone) continue;
    const uint32_t o = ch->origin;
    if (o >= uint32_t(world_) || o >= uint32_t(kMaxRanks)) continue;
    const bool replaced = dir_->d->gen[o].load(std::memory_order_acquire) != ch->origin_gen;
    if (replaced || !pid_alive(dir_->d->pid[o].load(std::memory_order_acquire))) {
      uint32_t expect = kDone;
      ch->state.compare_exchange_strong(expect, kFree, std::memory_order_acq_rel);
    }
  }
}

void Router::run() {
  pthread_setname_np(pthread_self(), "tfs-router");
  SegHdr* h = self_->hdr();
  auto last_scan = Clock::now();
  while (running_.load()) {
    const uint32_t seen = h->doorbell.load(std::memory_order_acquire);
    ingest();
    const auto now = Clock::now();
    const bool scan = now - last_scan > std::chrono::milliseconds(100);
    if (scan) {
      std::lock_guard<std::mutex> g(mu_);
      rescan();
      last_scan = now;
      collect_orphans();
    }
    reap(scan);
    h->heartbeat.fetch_add(1, std::memory_order_relaxed);
    if (h->doorbell.load(std::memory_order_acquire) != seen) continue;   // rung meanwhile
    timespec ts{0, 20 * 1000 * 1000};
    futex(&h->doorbell, FUTEX_WAIT, seen, &ts);
  }
}

int Router::peers_alive() {
  std::lock_guard<std::mutex> g(mu_);
  int n = 0;
  for (int p = 0; p < world_; ++p)
    if (p != rank_ && peers_[p]->alive) ++n;
  return n;
}

std::vector<int64_t> Router::loads() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<int64_t> out(size_t(world_), -1);
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) out[p] = self_->hdr()->load.load();
    else if (peers_[p]->alive && peers_[p]->seg) out[p] = peers_[p]->seg->hdr()->load.load();
  }
  return out;
}

}  // namespace tfs
