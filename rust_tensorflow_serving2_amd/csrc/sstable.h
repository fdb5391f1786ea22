#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace tfs {

// Build a LevelDB-format table from strictly increasing keys.
std::string sstable_build(const std::vector<std::pair<std::string, std::string>>& sorted_kvs,
                          size_t block_size = 256 * 1024, int restart_interval = 16);

// Read every (key, value) of a table; `verify` checks block crc32c (DATA_LOSS on mismatch).
std::vector<std::pair<std::string, std::string>> sstable_read(const uint8_t* data, size_t n,
                                                              bool verify = true);

// Read-only mmap of a file (bundle data shards are mapped, never slurped).
class MappedFile {
 public:
  explicit MappedFile(const std::string& path);
  ~MappedFile();
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
  const uint8_t* data() const { return data_; }
  size_t size() const { return size_; }

 private:
  int fd_ = -1;
  const uint8_t* data_ = nullptr;
  size_t size_ = 0;
};

}  // namespace tfs
