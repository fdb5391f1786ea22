// Native PredictionLog TFRecord writer (see request_log.h).
#include "request_log.h"

#include <cerrno>
#include <cmath>
#include <cstring>
#include <random>
#include <stdexcept>

namespace tfs {

namespace {

uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

uint64_t seed_of() {
  std::random_device rd;
  return (uint64_t(rd()) << 32) ^ rd();
}

const uint64_t kSeed = seed_of();

}  // namespace

RequestLog::RequestLog(const std::string& path_, double rate_, size_t max_pending)
    : path(path_), rate(rate_), max_pending_(max_pending) {
  f_ = std::fopen(path.c_str(), "ab");
  if (!f_) throw std::runtime_error("request log: cannot open " + path + ": " + std::strerror(errno));
  if (!(rate > 0)) threshold_ = 0;
  else if (rate >= 1.0) threshold_ = ~uint64_t(0);
  else threshold_ = uint64_t(std::ldexp(rate, 64));
  th_ = std::thread([this] { run(); });
}

RequestLog::~RequestLog() { close(); }

bool RequestLog::sample() {
  if (threshold_ == ~uint64_t(0)) return true;
  if (threshold_ == 0) return false;
  return splitmix64(kSeed ^ (draws_.fetch_add(1, std::memory_order_relaxed) * 0x2545f4914f6cdd1dull)) < threshold_;
}

bool RequestLog::push(Item&& it) {
  const size_t n = it.size();
  std::lock_guard<std::mutex> g(mu_);
  if (stop_ || pending_ + n > max_pending_) {
    dropped++;
    return false;
  }
  pending_ += n;
  ++seq_in_;
  q_.push_back(std::move(it));
  cv_.notify_one();
  return true;
}

bool RequestLog::submit_predict(const ModelSpecView& spec, std::string head, std::string payload,
                                std::string response) {
  Item it;
  it.spec = spec;
  it.a = std::move(head);
  it.b = std::move(payload);
  it.c = std::move(response);
  return push(std::move(it));
}

bool RequestLog::submit_record(std::string record) {
  Item it;
  it.raw = true;
  it.a = std::move(record);
  return push(std::move(it));
}

void RequestLog::flush() {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t want = seq_in_;
  cv_done_.wait(lk, [&] { return seq_out_ >= want || done_; });
}

void RequestLog::close() {
  std::lock_guard<std::mutex> c(close_mu_);
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    cv_.notify_all();
  }
  if (th_.joinable()) th_.join();   // the writer drains the queue first
  if (f_) {
    std::fclose(f_);
    f_ = nullptr;
  }
}

void RequestLog::run() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
    if (q_.empty()) {          // stop_ and drained
      done_ = true;
      cv_done_.notify_all();
      return;
    }
    std::deque<Item> batch;
    batch.swap(q_);
    lk.unlock();
    size_t n = 0;
    for (auto& it : batch) {
      write_item(it);
      n += it.size();
    }
    std::fflush(f_);
    lk.lock();
    pending_ -= n;
    seq_out_ += batch.size();
    cv_done_.notify_all();
  }
}

// TFRecord: u64 length, masked crc32c(length), data, masked crc32c(data)
void RequestLog::write_record(const std::string_view* parts, size_t nparts) {
  uint64_t len = 0;
  for (size_t i = 0; i < nparts; ++i) len += parts[i].size();
  uint8_t hdr[12];
  std::memcpy(hdr, &len, 8);   // little-endian host
  const uint32_t hc = crc32c_mask(crc32c(hdr, 8));
  std::memcpy(hdr + 8, &hc, 4);
  std::fwrite(hdr, 1, 12, f_);
  uint32_t crc = 0;
  for (size_t i = 0; i < nparts; ++i) {
    std::fwrite(parts[i].data(), 1, parts[i].size(), f_);
    crc = crc32c_extend(crc, parts[i].data(), parts[i].size());
  }
  const uint32_t pc = crc32c_mask(crc);
  std::fwrite(&pc, 1, 4, f_);
  written++;
  bytes += 16 + len;
}

void RequestLog::write_item(const Item& it) {
  if (it.raw) {
    const std::string_view v(it.a);
    write_record(&v, 1);
    return;
  }
  // PredictionLog { log_metadata = 1 { model_spec = 1, sampling_config = 2 { sampling_rate = 1 },
  //                 saved_model_tags = 3 }, predict_log = 6 { request = 1, response = 2 } }
  Writer meta;
  write_model_spec(meta, 1, it.spec);
  Writer sc;
  sc.tag(1, 1);
  sc.raw(&rate, 8);
  meta.bytes_field(2, sc.out);
  meta.bytes_field(3, "serve");
  const size_t req = it.a.size() + it.b.size();
  const size_t pl = 1 + varint_size(req) + req + 1 + varint_size(it.c.size()) + it.c.size();
  Writer pre;
  pre.bytes_field(1, meta.out);
  pre.tag(6, 2);
  pre.varint(pl);
  pre.tag(1, 2);
  pre.varint(req);
  Writer mid;
  mid.tag(2, 2);
  mid.varint(it.c.size());
  const std::string_view parts[5] = {pre.out, it.a, it.b, mid.out, it.c};
  write_record(parts, 5);
}

}  // namespace tfs
