// LevelDB-format immutable table (the container of TensorFlow's TensorBundle
// `variables/variables.index`), reader + writer, plus bundle data-file helpers.
//
// Layout written (and accepted when reading):
//   [data block]* [metaindex block] [index block] [footer 48 B]
//   block   = entries (shared:v32, non_shared:v32, value_len:v32, key_delta, value)
//             + restart offsets (u32 LE each) + num_restarts (u32 LE)
//   trailer = compression type (u8, 0 = none) + masked crc32c(block||type) (u32 LE)
//   footer  = metaindex handle + index handle (varint64 offset,size each),
//             zero padded to 40 B, then magic 0xdb4775248b80fb57 (u64 LE)
// This is the format TF's table::TableBuilder emits for checkpoint indexes;
// the reference's fixture (resnet SavedModel, serving/fetch.sh:22-26) ships
// such an index next to saved_model.pb.
#include "sstable.h"

#include <algorithm>
#include <cstdio>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "wire.h"

namespace tfs {

static constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
static constexpr size_t kFooterLen = 48;

namespace {

void put_fixed32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
void put_fixed64(std::string& s, uint64_t v) { s.append(reinterpret_cast<const char*>(&v), 8); }
void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) { s.push_back(char(v | 0x80)); v >>= 7; }
  s.push_back(char(v));
}

class BlockBuilder {
 public:
  explicit BlockBuilder(int restart_interval) : interval_(restart_interval) { restarts_.push_back(0); }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter_ < interval_) {
      const size_t mx = std::min(last_key_.size(), key.size());
      while (shared < mx && last_key_[shared] == key[shared]) ++shared;
    } else {
      restarts_.push_back(uint32_t(buf_.size()));
      counter_ = 0;
    }
    const size_t non_shared = key.size() - shared;
    put_varint(buf_, shared);
    put_varint(buf_, non_shared);
    put_varint(buf_, value.size());
    buf_.append(key.data() + shared, non_shared);
    buf_.append(value);
    last_key_ = key;
    ++counter_;
    ++entries_;
  }
  std::string finish() {
    std::string out = buf_;
    for (uint32_t r : restarts_) put_fixed32(out, r);
    put_fixed32(out, uint32_t(restarts_.size()));
    return out;
  }
  size_t size_estimate() const { return buf_.size() + restarts_.size() * 4 + 4; }
  bool empty() const { return entries_ == 0; }
  void reset() {
    buf_.clear(); restarts_.assign(1, 0); counter_ = 0; entries_ = 0; last_key_.clear();
  }

 private:
  int interval_;
  std::string buf_;
  std::vector<uint32_t> restarts_;
  int counter_ = 0;
  size_t entries_ = 0;
  std::string last_key_;
};

void emit_block(std::string& file, const std::string& contents, uint64_t& off, uint64_t& size) {
  off = file.size();
  size = contents.size();
  file.append(contents);
  const char type = 0;
  uint32_t crc = crc32c_extend(crc32c(contents.data(), contents.size()), &type, 1);
  file.push_back(type);
  put_fixed32(file, crc32c_mask(crc));
}

struct Handle { uint64_t off = 0, size = 0; };

Handle read_handle(Reader& r) {
  Handle h;
  h.off = r.varint();
  h.size = r.varint();
  return h;
}

std::string_view read_block(const uint8_t* data, size_t n, const Handle& h, bool verify) {
  if (h.off + h.size + 5 > n) throw WireError("sstable: block handle out of range");
  const uint8_t* b = data + h.off;
  const uint8_t type = b[h.size];
  if (type != 0) throw WireError("sstable: compressed blocks are not supported");
  if (verify) {
    uint32_t stored; std::memcpy(&stored, b + h.size + 1, 4);
    uint32_t crc = crc32c_extend(crc32c(b, h.size), &type, 1);
    if (crc32c_mask(crc) != stored) throw WireError("sstable: block checksum mismatch (DATA_LOSS)");
  }
  return std::string_view(reinterpret_cast<const char*>(b), h.size);
}

void iterate_block(std::string_view blk, std::vector<std::pair<std::string, std::string>>& out) {
  if (blk.size() < 4) throw WireError("sstable: block too small");
  uint32_t nrest; std::memcpy(&nrest, blk.data() + blk.size() - 4, 4);
  const size_t limit = blk.size() - 4 - size_t(nrest) * 4;
  if (size_t(nrest) * 4 + 4 > blk.size()) throw WireError("sstable: bad restart count");
  Reader r(reinterpret_cast<const uint8_t*>(blk.data()), limit);
  std::string key;
  while (!r.done()) {
    uint64_t shared = r.varint(), non_shared = r.varint(), vlen = r.varint();
    if (shared > key.size()) throw WireError("sstable: bad shared prefix");
    if (uint64_t(r.end - r.p) < non_shared + vlen) throw WireError("sstable: truncated entry");
    key.resize(shared);
    key.append(reinterpret_cast<const char*>(r.p), non_shared);
    r.p += non_shared;
    out.emplace_back(key, std::string(reinterpret_cast<const char*>(r.p), vlen));
    r.p += vlen;
  }
}

}  // namespace

std::string sstable_build(const std::vector<std::pair<std::string, std::string>>& sorted_kvs,
                          size_t block_size, int restart_interval) {
  std::string file;
  BlockBuilder data(restart_interval), index(1);
  std::string last_key;
  bool pending_index = false;
  Handle pending;
  auto flush = [&]() {
    if (data.empty()) return;
    emit_block(file, data.finish(), pending.off, pending.size);
    data.reset();
    pending_index = true;
  };
  for (size_t i = 0; i < sorted_kvs.size(); ++i) {
    const auto& kv = sorted_kvs[i];
    if (i > 0 && !(last_key < kv.first)) throw WireError("sstable: keys must be strictly increasing");
    if (pending_index) {
      std::string h; put_varint(h, pending.off); put_varint(h, pending.size);
      index.add(last_key, h);     // separator = last key of the finished block
      pending_index = false;
    }
    data.add(kv.first, kv.second);
    last_key = kv.first;
    if (data.size_estimate() >= block_size) flush();
  }
  flush();
  if (pending_index) {
    std::string h; put_varint(h, pending.off); put_varint(h, pending.size);
    index.add(last_key, h);
  }
  Handle meta_h, index_h;
  BlockBuilder meta(restart_interval);
  emit_block(file, meta.finish(), meta_h.off, meta_h.size);
  emit_block(file, index.finish(), index_h.off, index_h.size);
  std::string footer;
  put_varint(footer, meta_h.off); put_varint(footer, meta_h.size);
  put_varint(footer, index_h.off); put_varint(footer, index_h.size);
  footer.resize(40, '\0');
  put_fixed64(footer, kTableMagic);
  file.append(footer);
  return file;
}

std::vector<std::pair<std::string, std::string>> sstable_read(const uint8_t* data, size_t n, bool verify) {
  if (n < kFooterLen) throw WireError("sstable: file too short");
  const uint8_t* f = data + n - kFooterLen;
  uint64_t magic; std::memcpy(&magic, f + 40, 8);
  if (magic != kTableMagic) throw WireError("sstable: bad magic number");
  Reader r(f, 40);
  read_handle(r);                       // metaindex (unused)
  Handle index_h = read_handle(r);
  std::vector<std::pair<std::string, std::string>> index_entries, out;
  iterate_block(read_block(data, n, index_h, verify), index_entries);
  for (auto& ie : index_entries) {
    Reader hr(reinterpret_cast<const uint8_t*>(ie.second.data()), ie.second.size());
    Handle h = read_handle(hr);
    iterate_block(read_block(data, n, h, verify), out);
  }
  return out;
}

// ---------------------------------------------------------------- MappedFile
MappedFile::MappedFile(const std::string& path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw WireError("cannot open " + path);
  struct stat st;
  if (fstat(fd_, &st) != 0) { ::close(fd_); throw WireError("cannot stat " + path); }
  size_ = size_t(st.st_size);
  if (size_) {
    void* p = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (p == MAP_FAILED) { ::close(fd_); throw WireError("cannot mmap " + path); }
    data_ = static_cast<const uint8_t*>(p);
  }
}

MappedFile::~MappedFile() {
  if (data_) munmap(const_cast<uint8_t*>(data_), size_);
  if (fd_ >= 0) ::close(fd_);
}

}  // namespace tfs
