// Cross-replica request routing over POSIX shared memory.
//
// One server process per GPU (parallel/replicas.py).  The kernel's
// SO_REUSEPORT hash spreads *connections* over the replicas, but the
// reference client multiplexes every call of a program over one or two
// HTTP/2 connections (src/lib.rs:132-138, 148-156; examples/async.rs:29-46),
// so connection-level balancing pins all of its traffic on one GPU.  The
// router balances per *stream*: every replica's front end may place a
// Predict on the least-loaded replica of the node.
//
//   * Each replica owns a ring of `ncells` cells in a shared-memory segment
//     (/dev/shm/tfs_<group>_r<rank>_g<generation>).  A cell holds one request
//     message (up to `req_cap` bytes) and, later, its response.
//   * A front end that routes a call to replica p claims a FREE cell of p's
//     ring (CAS), writes the message there — for a streamed Predict the
//     tensor payload goes from the socket straight into the cell, so a remote
//     request costs no more copies than a local one — marks it READY and
//     rings p's doorbell (a futex word in p's segment header).
//   * p's router thread takes READY cells and dispatches them as local calls
//     (fast path or Python) whose body is the cell itself; the answer is
//     written back into the cell (DONE) and the origin's doorbell rung; the
//     origin's router thread answers the original HTTP/2 stream.  An answer
//     larger than the cell's response area is sent back as "run it yourself"
//     and the origin serves the call locally from the message still in the cell.
//   * Load = calls a replica has accepted and not answered yet (an atomic in
//     its header).  A call goes remote only when the local load has reached
//     `local_cap` (the local GPU's batch pipeline is full: lanes x max batch)
//     and a live peer's load is lower than the local one by more than
//     `margin`: balanced replicas (many connections, the benchmark) keep their
//     own traffic, and a client with fewer calls in flight than one GPU can
//     batch is served at full batch size instead of in fragments on every GPU.
//   * Liveness: the owner's pid and a heartbeat its router thread advances.
//     A peer that dies leaves its calls: cells it had not taken yet are
//     re-dispatched locally, taken ones are answered UNAVAILABLE (and their
//     cells freed should the peer, only stalled, finish them later); a restarted
//     replica gets a new generation (a directory segment maps rank ->
//     generation) and peers re-map it.
#pragma once
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "http2.h"

namespace tfs {

struct RouterSeg;       // one mapped segment (private to router.cpp)
struct RouterDir;

struct RouterStats {
  std::atomic<uint64_t> forwarded{0};   // calls this front end placed on a peer
  std::atomic<uint64_t> streamed{0};    // ... of which the payload was received straight into the peer's cell
  std::atomic<uint64_t> ingested{0};    // calls peers placed here
  std::atomic<uint64_t> returned{0};    // answers of forwarded calls relayed back to their clients
  std::atomic<uint64_t> reclaimed{0};   // forwarded calls re-run locally (the peer died before taking them)
  std::atomic<uint64_t> lost{0};        // forwarded calls answered UNAVAILABLE (the peer died while running them)
  std::atomic<uint64_t> no_cell{0};     // routing wanted a peer whose ring was full
  std::atomic<uint64_t> rerun{0};       // forwarded calls re-run here: the answer did not fit the cell
  std::atomic<uint64_t> too_large{0};   // peers' calls whose answer did not fit their cell (sent back)
  std::atomic<uint64_t> tomb_freed{0};  // cells of given-up calls freed when the peer finished late
  // answers written into a cell whose origin this replica could not see (its
  // view of the origin's generation stale): the cell is left DONE for the
  // origin to collect, never freed here
  std::atomic<uint64_t> unseen_origin{0};
  // forwarded calls whose cell no longer carries their token (it was freed
  // and reused under them): answered UNAVAILABLE instead of waiting forever
  std::atomic<uint64_t> orphaned{0};
};

class Router : public RemoteSink {
 public:
  Router(Server* srv, const std::string& group, int rank, int world, int ncells, size_t req_cap, size_t resp_cap,
         int margin);
  ~Router() override;
  void start();
  void stop();
  // Place a complete call on a peer (true: taken, the call is answered later).
  bool forward(std::unique_ptr<Call>& c);
  // A streamed Predict: a row in a peer's cell, or nullptr to keep it local.
  std::shared_ptr<StreamRes> reserve_stream(const ProbeInfo& pi, const uint8_t* head, size_t head_len,
                                            const std::string& method);
  // this replica's outstanding-call counter (lives in its shared segment)
  std::atomic<int64_t>* load_word();
  void respond_remote(const Call& c, int status, const std::string& msg, const std::string& body) override;
  int rank() const { return rank_; }
  // Keep calls local while this replica has fewer than `cap` outstanding: a
  // GPU replica's batches fill (and its HIP graphs run at full batch size)
  // before any call spills to a peer; 0 = route on load difference alone.
  void set_local_cap(int64_t cap) { local_cap_.store(cap, std::memory_order_relaxed); }
  int64_t local_cap() const { return local_cap_.load(std::memory_order_relaxed); }
  int peers_alive();
  std::vector<int64_t> loads();
  RouterStats stats;

  struct Pending;
  struct Peer;
  struct Tomb;

 private:
  friend struct RemoteStream;
  int pick(size_t msg_len);
  // claim a FREE cell of peer p's ring; -1 if none
  int claim(RouterSeg& seg);
  void publish(int p, const std::shared_ptr<RouterSeg>& seg, int cell, std::unique_ptr<Call> call);
  void run();
  void ingest();
  void reap(bool check_peers);
  void rescan();
  void collect_orphans();
  void ring(RouterSeg& seg);

  Server* srv_;
  std::string group_;
  int rank_, world_, ncells_, margin_;
  size_t req_cap_, resp_cap_;
  std::shared_ptr<RouterSeg> self_;
  RouterDir* dir_ = nullptr;
  std::string dir_name_;
  std::mutex mu_;                                 // peers_ + pending_
  std::vector<std::unique_ptr<Peer>> peers_;
  std::map<uint64_t, std::unique_ptr<Pending>> pending_;
  std::vector<Tomb> tombs_;
  uint64_t next_token_ = 1;
  std::atomic<bool> running_{false};
  std::atomic<int64_t> local_cap_{0};
  std::thread th_;
};

}  // namespace tfs
