// Host-side stress / fuzz driver for the native data plane, built with
// -fsanitize=address,undefined (tests/test_sanitizers.py).  Exercises:
//   * the wire codec: encode -> parse round trips, every truncation and random
//     byte flips of valid requests (must throw or parse, never crash or read OOB),
//     the streaming header probe on every prefix;
//   * the SSTable writer/reader with corruption;
//   * the batcher: concurrent offers + streamed rows (commit / abandon) against
//     a lane thread acquiring and completing, through a real Server instance;
//   * the cross-replica router: two front ends in one process sharing a
//     routing group (shared-memory rings), buffered and streamed calls routed
//     both ways while responders answer them, then one router stops.
// Built twice: ASan + UBSan, and TSan (the IO / lane / router threads).
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include <unistd.h>

#include "batcher.h"
#include "request_log.h"
#include "http2.h"
#include "router.h"
#include "sstable.h"
#include "wire.h"

using namespace tfs;

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

static std::string make_request(std::mt19937& rng, int rows, int cols, bool filter, bool tc) {
  ModelSpecView spec;
  spec.name = "m";
  spec.has_version = rng() % 2;
  spec.version = 7;
  spec.signature_name = rng() % 2 ? "serving_default" : "";
  std::vector<float> data(size_t(rows) * cols);
  for (auto& v : data) v = float(rng() % 1000) / 7.f;
  OutTensor t;
  t.alias = "x";
  t.dtype = DT_FLOAT;
  t.shape = {rows, cols};
  t.data = data.data();
  t.count = data.size();
  std::vector<std::string> of;
  if (filter) of.push_back("y");
  return encode_predict_request(spec, {t}, of, tc);
}

static void fuzz_codec() {
  std::mt19937 rng(1234);
  for (int iter = 0; iter < 60; ++iter) {
    const int rows = 1 + rng() % 3, cols = 1 + rng() % 300;
    const bool filter = rng() % 4 == 0, tc = rng() % 2;
    std::string body = make_request(rng, rows, cols, filter, tc);
    PredictRequestView req;
    parse_predict_request(reinterpret_cast<const uint8_t*>(body.data()), body.size(), req);
    CHECK(req.has_spec && req.spec.name == "m");
    CHECK(req.inputs.size() == 1 && req.inputs[0].second.count == size_t(rows) * cols);
    // every truncation: throw or parse, never crash
    for (size_t n = 0; n < body.size(); n += 1 + body.size() / 97) {
      std::vector<uint8_t> cut(body.begin(), body.begin() + n);   // exact-size heap copy: ASan sees overreads
      try {
        PredictRequestView r2;
        parse_predict_request(cut.data(), cut.size(), r2);
      } catch (const std::exception&) {
      }
    }
    // random byte flips
    for (int f = 0; f < 40; ++f) {
      std::vector<uint8_t> bad(body.begin(), body.end());
      const int nflip = 1 + rng() % 4;
      for (int k = 0; k < nflip; ++k) bad[rng() % bad.size()] ^= uint8_t(1 + rng() % 255);
      try {
        PredictRequestView r3;
        parse_predict_request(bad.data(), bad.size(), r3);
      } catch (const std::exception&) {
      }
    }
    // streaming probe over every prefix of the framed message
    std::string framed(5, '\0');
    grpc_frame_header(reinterpret_cast<uint8_t*>(&framed[0]), uint32_t(body.size()));
    framed += body;
    bool found = false;
    for (size_t n = 0; n <= framed.size(); n += 1 + framed.size() / 211) {
      std::vector<uint8_t> cut(framed.begin(), framed.begin() + n);
      ProbeInfo pi;
      const Probe p = probe_predict_header(cut.data(), cut.size(), 1, pi);
      if (p == Probe::kFound) {
        found = true;
        CHECK(pi.payload_off + pi.payload_len == framed.size());
        CHECK(pi.payload_len == size_t(rows) * cols * 4);
      }
    }
    CHECK(found || filter);   // an output_filter after the inputs disables streaming
  }
}

static void fuzz_sstable() {
  std::mt19937 rng(99);
  std::vector<std::pair<std::string, std::string>> kvs;
  for (int i = 0; i < 500; ++i) {
    char k[32];
    std::snprintf(k, sizeof(k), "key/%06d", i);
    kvs.emplace_back(k, std::string(rng() % 300, char('a' + i % 26)));
  }
  const std::string t = sstable_build(kvs, 4096, 8);
  auto back = sstable_read(reinterpret_cast<const uint8_t*>(t.data()), t.size(), true);
  CHECK(back == kvs);
  for (int f = 0; f < 200; ++f) {
    std::vector<uint8_t> bad(t.begin(), t.end());
    bad[rng() % bad.size()] ^= 0x5a;
    try {
      sstable_read(bad.data(), bad.size(), true);
    } catch (const std::exception&) {
    }
  }
}

// Streams that are neither committed nor abandoned must never reach the batcher,
// so this drives reserve -> write -> commit/abandon exactly as the IO thread does.
static void stress_batcher() {
  Server srv("127.0.0.1", 0, 1, size_t(1) << 30);
  const int COLS = 64, ROWS = 8, SLOTS = 3;
  TensorSpecC in{"x", DT_FLOAT, {COLS}, size_t(COLS), size_t(COLS) * 4};
  TensorSpecC out{"y", DT_FLOAT, {COLS}, size_t(COLS), size_t(COLS) * 4};
  auto ep = std::make_shared<Endpoint>(1, "m", 7, "serving_default", std::vector<TensorSpecC>{in},
                                       std::vector<TensorSpecC>{out}, ROWS, 300, 100);
  ep->set_server(&srv);
  std::vector<std::vector<float>> bufs(SLOTS * 2, std::vector<float>(ROWS * COLS));
  for (int s = 0; s < SLOTS; ++s)
    ep->set_slot_buffers(s, {reinterpret_cast<uint8_t*>(bufs[2 * s].data())},
                         {reinterpret_cast<const uint8_t*>(bufs[2 * s + 1].data())});
  // request logging on, toggled off / on while lanes submit (writer thread + lane threads)
  const std::string log_path = "/tmp/sanitize_reqlog_" + std::to_string(getpid()) + ".tfrecord";
  auto rlog = std::make_shared<RequestLog>(log_path, 0.5);
  ep->set_log(rlog);
  std::atomic<bool> stop{false};
  std::atomic<int> batches{0};
  std::thread toggler([&] {
    for (int k = 0; !stop; ++k) {
      ep->set_log(k % 3 == 2 ? nullptr : rlog);
      std::this_thread::sleep_for(std::chrono::milliseconds(3));
    }
  });
  std::vector<std::thread> lanes;
  for (int s = 0; s < SLOTS; ++s)
    lanes.emplace_back([&, s] {
      while (!stop) {
        const int n = ep->acquire(s, 5);
        if (n < 0) return;
        if (n == 0) continue;
        std::memcpy(bufs[2 * s + 1].data(), bufs[2 * s].data(), size_t(n) * COLS * 4);
        if (n % 5 == 0) ep->fail(s, srv, 13, "x");
        else ep->complete(s, srv);
        batches++;
      }
    });
  std::vector<std::thread> io;
  for (int t = 0; t < 4; ++t)
    io.emplace_back([&, t] {
      std::mt19937 rng(t);
      for (int i = 0; i < 400; ++i) {
        const int rows = 1 + rng() % 3;
        if (rng() % 2) {   // buffered offer
          std::string body = make_request(rng, rows, COLS, false, rng() % 2);
          auto call = std::make_unique<Call>();
          call->body = body;
          PredictRequestView req;
          parse_predict_request(call->data(), call->size(), req);
          ep->offer(call, req);
        } else {           // streamed row: reserve, write in chunks, commit or abandon
          ProbeInfo pi;
          pi.spec.name = "m";
          pi.alias = "x";
          pi.dtype = DT_FLOAT;
          pi.shape = {rows, COLS};
          pi.payload_len = size_t(rows) * COLS * 4;
          auto r = ep->reserve_stream(ep, pi);
          if (!r) continue;
          std::vector<float> src(size_t(rows) * COLS, float(i));
          const uint8_t* p = reinterpret_cast<const uint8_t*>(src.data());
          size_t left = r->len;
          while (left) {
            const size_t n = std::min<size_t>(left, 1 + rng() % 700);
            r->write(p + (r->len - left), n);
            left -= n;
          }
          if (rng() % 7 == 0) {
            r->abandon();
          } else {
            auto call = std::make_unique<Call>();
            if (r->keep_header()) call->head = "\0\0\0\0\0hdr";   // what request_done keeps
            r->commit(std::move(call));
          }
        }
      }
    });
  for (auto& t : io) t.join();
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  stop = true;
  ep->close(&srv);
  for (auto& t : lanes) t.join();
  toggler.join();
  rlog->flush();
  rlog->close();
  CHECK(batches.load() > 0);
  CHECK(rlog->written.load() > 0);
  std::remove(log_path.c_str());
}

static void stress_router() {
  const std::string group = "san" + std::to_string(getpid());
  Server a("127.0.0.1", 0, 1, size_t(1) << 30), b("127.0.0.1", 0, 1, size_t(1) << 30);
  auto ra = std::make_unique<Router>(&a, group, 0, 2, 8, 4096, 4096, 0);
  auto rb = std::make_unique<Router>(&b, group, 1, 2, 8, 4096, 4096, 0);
  a.set_router(ra.get());
  b.set_router(rb.get());
  ra->start();
  rb->start();
  std::atomic<bool> stop{false};
  std::atomic<int> answered{0};
  std::vector<std::thread> th;
  for (Server* s : {&a, &b})
    for (int k = 0; k < 2; ++k)
      th.emplace_back([&, s] {
        while (!stop) {
          auto c = s->next_call(2);
          if (!c) continue;
          CHECK(c->size() >= 1 && c->data()[0] == 'p');
          std::this_thread::sleep_for(std::chrono::microseconds(200));
          s->respond(*c, 0, std::string(), std::string(c->size() > 64 ? 64 : c->size(), 'r'));
          answered++;
        }
      });
  std::this_thread::sleep_for(std::chrono::milliseconds(300));   // routers map each other
  std::vector<std::thread> drivers;
  for (int t = 0; t < 4; ++t)
    drivers.emplace_back([&, t] {
      std::mt19937 rng(77 + t);
      Server& s = t % 2 ? b : a;
      for (int i = 0; i < 300; ++i) {
        if (rng() % 3) {   // a buffered call
          auto c = std::make_unique<Call>();
          c->method = "/tensorflow.serving.PredictionService/Predict";
          c->body.assign(5, '\0');
          c->body += "p" + std::string(1 + rng() % 2000, char('a' + i % 26));
          c->off = 5;
          c->arrival = Clock::now();
          s.dispatch(std::move(c));
        } else {           // a streamed call whose payload lands in whichever row the router picks
          std::string head(5, '\0');
          head += "p" + std::string(20, 'h');
          ProbeInfo pi;
          pi.payload_off = head.size();
          pi.payload_len = 1 + rng() % 1500;
          auto r = s.reserve_stream(pi, reinterpret_cast<const uint8_t*>(head.data()), head.size(),
                                    "/tensorflow.serving.PredictionService/Predict");
          if (!r) continue;     // stays local: no batch slots in this harness
          std::vector<uint8_t> payload(r->len, uint8_t('z'));
          size_t left = r->len;
          while (left) {
            const size_t n = std::min<size_t>(left, 1 + rng() % 400);
            r->write(payload.data() + (r->len - left), n);
            left -= n;
          }
          if (rng() % 9 == 0) {
            r->abandon();
          } else {
            auto c = std::make_unique<Call>();
            c->method = "/tensorflow.serving.PredictionService/Predict";
            c->arrival = Clock::now();
            r->commit(std::move(c));
          }
        }
      }
    });
  for (auto& d : drivers) d.join();
  std::this_thread::sleep_for(std::chrono::milliseconds(500));
  CHECK(ra->stats.forwarded.load() + rb->stats.forwarded.load() > 0);
  CHECK(ra->stats.returned.load() == ra->stats.forwarded.load());
  CHECK(rb->stats.returned.load() == rb->stats.forwarded.load());
  rb->stop();                      // a peer goes away with the other still routing
  for (int i = 0; i < 50; ++i) {
    auto c = std::make_unique<Call>();
    c->method = "/tensorflow.serving.PredictionService/Predict";
    c->body = std::string(5, '\0') + "pzz";
    c->off = 5;
    c->arrival = Clock::now();
    a.dispatch(std::move(c));
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  stop = true;
  for (auto& t : th) t.join();
  ra->stop();
  a.set_router(nullptr);
  b.set_router(nullptr);
  ra.reset();
  rb.reset();
  const std::string dir = "/dev/shm/tfs_" + group + "_dir";
  std::remove(dir.c_str());
  CHECK(answered.load() > 0);
}

int main() {
  fuzz_codec();
  fuzz_sstable();
  stress_batcher();
  stress_router();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("sanitize_main: ok\n");
  return 0;
}
