// Request logging (ModelConfig.logging_config, reference
// protos/tensorflow_serving/config/logging_config.proto:15,
// model_server_config.proto:67): sampled (request, response) pairs written as
// PredictionLog TFRecords by a native writer thread.
//
// The fast path's lane thread decides per request whether it is sampled
// (sampling_rate, a counter-hashed draw: no lock, no shared RNG state) and
// hands the sampled request / response bytes to submit(); framing, crc32c and
// file IO happen on the writer thread, never on an IO or lane thread.  The
// Python slow path (server/core.py) writes its already-serialised
// PredictionLog records through the same writer, so one file per model holds
// both.  A writer that falls `max_pending` bytes behind drops records (counted)
// rather than stalling serving.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>

#include "wire.h"

namespace tfs {

class RequestLog {
 public:
  RequestLog(const std::string& path, double sampling_rate, size_t max_pending = size_t(256) << 20);
  ~RequestLog();
  RequestLog(const RequestLog&) = delete;
  RequestLog& operator=(const RequestLog&) = delete;

  // One draw per request: true with probability sampling_rate.
  bool sample();
  // A predict pair: the request message is `head` + `payload` (a streamed
  // request's header bytes and its row; `payload` empty otherwise).
  bool submit_predict(const ModelSpecView& spec, std::string head, std::string payload, std::string response);
  // An already-serialised PredictionLog (the Python slow path).
  bool submit_record(std::string record);
  // Blocks until everything submitted so far is on disk (fflush'ed).
  void flush();
  void close();

  const std::string path;
  const double rate;
  std::atomic<uint64_t> written{0}, dropped{0}, bytes{0};

 private:
  struct Item {
    bool raw = false;
    ModelSpecView spec;
    std::string a, b, c;   // raw: a = record; predict: head, payload, response
    size_t size() const { return a.size() + b.size() + c.size(); }
  };
  bool push(Item&& it);
  void run();
  void write_item(const Item& it);
  void write_record(const std::string_view* parts, size_t nparts);

  std::FILE* f_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_, cv_done_;
  std::deque<Item> q_;
  size_t pending_ = 0, max_pending_;
  uint64_t seq_in_ = 0, seq_out_ = 0;
  bool stop_ = false, done_ = false;
  std::mutex close_mu_;
  std::atomic<uint64_t> draws_{0};
  uint64_t threshold_ = 0;
  std::thread th_;
};

}  // namespace tfs
