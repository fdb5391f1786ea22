// Protobuf wire-format primitives + the hot-path codecs for the serving API.
//
// The reference client builds PredictRequest with prost (src/lib.rs:244-263):
// a single TensorProto with `float_val` (field 5, packed) holding the image as
// raw little-endian f32.  A packed fixed-width field on the wire *is* the raw
// array, so the decoder hands out (offset, length) views into the received
// buffer instead of materialising 150k-element repeated fields.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace tfs {

struct WireError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// TensorFlow DataType enum values used on the wire (types.proto).
enum DType : int {
  DT_INVALID = 0, DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_UINT8 = 4,
  DT_INT16 = 5, DT_INT8 = 6, DT_STRING = 7, DT_COMPLEX64 = 8, DT_INT64 = 9,
  DT_BOOL = 10, DT_BFLOAT16 = 14, DT_UINT16 = 17, DT_COMPLEX128 = 18,
  DT_HALF = 19, DT_UINT32 = 22, DT_UINT64 = 23,
};

// Bytes per element of a numeric dtype (0 for string / unsupported).
int dtype_size(int dtype);

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const uint8_t* b, size_t n) : p(b), end(b + n) {}
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t r = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= end) throw WireError("truncated varint");
      uint8_t b = *p++;
      r |= uint64_t(b & 0x7f) << shift;
      if (!(b & 0x80)) return r;
    }
    throw WireError("varint too long");
  }
  uint32_t fixed32() {
    if (end - p < 4) throw WireError("truncated fixed32");
    uint32_t v; std::memcpy(&v, p, 4); p += 4; return v;
  }
  uint64_t fixed64() {
    if (end - p < 8) throw WireError("truncated fixed64");
    uint64_t v; std::memcpy(&v, p, 8); p += 8; return v;
  }
  std::string_view bytes() {
    uint64_t n = varint();
    if (uint64_t(end - p) < n) throw WireError("truncated length-delimited field");
    std::string_view s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: if (end - p < 8) throw WireError("truncated"); p += 8; break;
      case 2: bytes(); break;
      case 5: if (end - p < 4) throw WireError("truncated"); p += 4; break;
      default: throw WireError("unsupported wire type " + std::to_string(wt));
    }
  }
};

struct Writer {
  std::string out;
  void varint(uint64_t v) {
    while (v >= 0x80) { out.push_back(char(v | 0x80)); v >>= 7; }
    out.push_back(char(v));
  }
  void tag(int field, int wt) { varint((uint64_t(field) << 3) | wt); }
  void bytes_field(int field, std::string_view s) {
    tag(field, 2); varint(s.size()); out.append(s.data(), s.size());
  }
  void varint_field(int field, uint64_t v) { tag(field, 0); varint(v); }
  void raw(const void* p, size_t n) { out.append(reinterpret_cast<const char*>(p), n); }
};

inline size_t varint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) { v >>= 7; ++n; }
  return n;
}

// ---------------------------------------------------------------- ModelSpec
struct ModelSpecView {
  std::string name;
  bool has_version = false;
  int64_t version = 0;
  bool has_label = false;
  std::string version_label;
  std::string signature_name;
};
void parse_model_spec(std::string_view buf, ModelSpecView& ms);
void write_model_spec(Writer& w, int field, const ModelSpecView& ms);

// ---------------------------------------------------------------- TensorProto
// Where the element data of a decoded tensor lives.
enum class Storage : int {
  kEmpty = 0,      // no values at all (zeros / fill rule)
  kView = 1,       // raw little-endian array at [offset, offset+nbytes) of the input buffer
  kOwned = 2,      // decoded into `owned` (varint fields / unpacked / multi-chunk)
  kStrings = 3,    // string_val entries (offset,len pairs into input buffer)
};

struct TensorView {
  int dtype = 0;
  std::vector<int64_t> shape;
  bool unknown_rank = false;
  Storage storage = Storage::kEmpty;
  size_t offset = 0;        // kView
  size_t nbytes = 0;        // kView / kOwned payload size
  size_t count = 0;         // number of values present on the wire
  std::string owned;        // kOwned
  std::vector<std::pair<size_t, size_t>> strings;  // kStrings (offset, len)
};

// Decode a TensorProto located at [base+off, base+off+len) of the request buffer.
void parse_tensor(const uint8_t* base, size_t off, size_t len, TensorView& t);

// ---------------------------------------------------------------- Predict
struct PredictRequestView {
  ModelSpecView spec;
  bool has_spec = false;
  std::vector<std::pair<std::string, TensorView>> inputs;
  std::vector<std::string> output_filter;
};
void parse_predict_request(const uint8_t* buf, size_t n, PredictRequestView& req);

// ---------------------------------------------------------------- streaming probe
// Header of a gRPC-framed PredictRequest whose LAST bytes are one large raw
// tensor payload (the reference client's shape: ModelSpec, then one inputs
// entry {alias, TensorProto{dtype, shape, float_val}} ending the message).
// For such requests the payload can be copied from the socket buffer straight
// into a batch slot as DATA frames arrive.
struct ProbeInfo {
  ModelSpecView spec;
  std::string alias;
  int dtype = 0;
  std::vector<int64_t> shape;
  size_t payload_off = 0;   // offset of the payload in the framed message (incl. the 5-byte prefix)
  size_t payload_len = 0;
};
enum class Probe : int { kNeedMore = 0, kNoStream = 1, kFound = 2 };
// `buf` = the first `n` bytes of the gRPC-framed message received so far.
Probe probe_predict_header(const uint8_t* buf, size_t n, size_t min_payload, ProbeInfo& out);

struct OutTensor {
  std::string alias;
  int dtype;
  std::vector<int64_t> shape;
  const void* data;      // numeric: contiguous little-endian array
  size_t count;          // element count
  const std::vector<std::string>* strings = nullptr;  // DT_STRING
};
// Serialise a PredictResponse.  `use_tensor_content` selects TF's
// AsProtoTensorContent form instead of typed repeated fields.
std::string encode_predict_response(const ModelSpecView* spec,
                                    const std::vector<OutTensor>& outs,
                                    bool use_tensor_content);
// Encode one TensorProto (shared by the response encoder and the client encoder).
void write_tensor(Writer& w, const OutTensor& t, bool use_tensor_content);

// Client-side request encoder (the Rust client's PredictRequest, src/lib.rs:244-263).
std::string encode_predict_request(const ModelSpecView& spec,
                                   const std::vector<OutTensor>& inputs,
                                   const std::vector<std::string>& output_filter,
                                   bool use_tensor_content);

// ---------------------------------------------------------------- gRPC framing
// 5-byte length prefix: [compressed:u8][len:u32 big-endian]
inline void grpc_frame_header(uint8_t* dst, uint32_t len) {
  dst[0] = 0;
  dst[1] = uint8_t(len >> 24); dst[2] = uint8_t(len >> 16);
  dst[3] = uint8_t(len >> 8);  dst[4] = uint8_t(len);
}

// ---------------------------------------------------------------- crc32c
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
inline uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }
inline uint32_t crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
inline uint32_t crc32c_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

}  // namespace tfs
