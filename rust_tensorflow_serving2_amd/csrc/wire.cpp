// Protobuf wire codecs for the TF-Serving hot path (see wire.h).
#include "wire.h"

#include <algorithm>

#if defined(__SSE4_2__)
#include <nmmintrin.h>
#endif

namespace tfs {

int dtype_size(int dtype) {
  switch (dtype) {
    case DT_FLOAT: case DT_INT32: case DT_UINT32: return 4;
    case DT_DOUBLE: case DT_INT64: case DT_UINT64: case DT_COMPLEX64: return 8;
    case DT_COMPLEX128: return 16;
    case DT_UINT8: case DT_INT8: case DT_BOOL: return 1;
    case DT_INT16: case DT_UINT16: case DT_HALF: case DT_BFLOAT16: return 2;
    default: return 0;
  }
}

// ---------------------------------------------------------------- ModelSpec
void parse_model_spec(std::string_view buf, ModelSpecView& ms) {
  Reader r(reinterpret_cast<const uint8_t*>(buf.data()), buf.size());
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = int(key >> 3), wt = int(key & 7);
    if (field == 1 && wt == 2) {
      ms.name = std::string(r.bytes());
    } else if (field == 2 && wt == 2) {          // google.protobuf.Int64Value
      std::string_view sub = r.bytes();
      Reader rr(reinterpret_cast<const uint8_t*>(sub.data()), sub.size());
      ms.has_version = true;
      ms.version = 0;
      while (!rr.done()) {
        uint64_t k2 = rr.varint();
        if ((k2 >> 3) == 1 && (k2 & 7) == 0) ms.version = int64_t(rr.varint());
        else rr.skip(int(k2 & 7));
      }
      ms.has_label = false;
    } else if (field == 3 && wt == 2) {
      ms.signature_name = std::string(r.bytes());
    } else if (field == 4 && wt == 2) {
      ms.version_label = std::string(r.bytes());
      ms.has_label = true;
      ms.has_version = false;
    } else {
      r.skip(wt);
    }
  }
}

void write_model_spec(Writer& w, int field, const ModelSpecView& ms) {
  Writer sub;
  if (!ms.name.empty()) sub.bytes_field(1, ms.name);
  if (ms.has_version) {
    Writer v;
    if (ms.version != 0) v.varint_field(1, uint64_t(ms.version));
    sub.bytes_field(2, v.out);
  }
  if (!ms.signature_name.empty()) sub.bytes_field(3, ms.signature_name);
  if (ms.has_label) sub.bytes_field(4, ms.version_label);
  w.bytes_field(field, sub.out);
}

// ---------------------------------------------------------------- TensorProto
namespace {

struct Seg {
  int wt;
  size_t off, len;   // wt==2: payload span (relative to base)
  uint64_t val;      // wt 0/1/5: scalar value bits
};

constexpr int kMaxField = 18;

int field_for_dtype(int dtype) {
  switch (dtype) {
    case DT_FLOAT: return 5;
    case DT_DOUBLE: return 6;
    case DT_INT32: case DT_INT16: case DT_INT8: case DT_UINT8: case DT_UINT16: return 7;
    case DT_STRING: return 8;
    case DT_COMPLEX64: return 9;
    case DT_INT64: return 10;
    case DT_BOOL: return 11;
    case DT_COMPLEX128: return 12;
    case DT_HALF: case DT_BFLOAT16: return 13;
    case DT_UINT32: return 16;
    case DT_UINT64: return 17;
    default: return -1;
  }
}

// Wire width of one element of a fixed-width repeated field (0 = varint field).
int fixed_width(int field) {
  switch (field) {
    case 5: case 9: return 4;
    case 6: case 12: return 8;
    default: return 0;
  }
}

template <typename T>
void append_value(std::string& out, T v) {
  out.append(reinterpret_cast<const char*>(&v), sizeof(T));
}

void append_converted(std::string& out, int dtype, uint64_t raw) {
  switch (dtype) {
    case DT_INT32: append_value<int32_t>(out, int32_t(raw)); break;
    case DT_INT16: append_value<int16_t>(out, int16_t(raw)); break;
    case DT_INT8: append_value<int8_t>(out, int8_t(raw)); break;
    case DT_UINT8: append_value<uint8_t>(out, uint8_t(raw)); break;
    case DT_UINT16: case DT_HALF: case DT_BFLOAT16:
      append_value<uint16_t>(out, uint16_t(raw)); break;
    case DT_INT64: append_value<int64_t>(out, int64_t(raw)); break;
    case DT_UINT32: append_value<uint32_t>(out, uint32_t(raw)); break;
    case DT_UINT64: append_value<uint64_t>(out, raw); break;
    case DT_BOOL: append_value<uint8_t>(out, raw ? 1 : 0); break;
    default: throw WireError("unsupported dtype for varint values: " + std::to_string(dtype));
  }
}

}  // namespace

void parse_tensor(const uint8_t* base, size_t off, size_t len, TensorView& t) {
  Reader r(base + off, len);
  std::vector<Seg> segs[kMaxField];
  bool have_content = false;
  size_t content_off = 0, content_len = 0;
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = int(key >> 3), wt = int(key & 7);
    if (field == 1 && wt == 0) {
      t.dtype = int(r.varint());
    } else if (field == 2 && wt == 2) {
      std::string_view sh = r.bytes();
      Reader rs(reinterpret_cast<const uint8_t*>(sh.data()), sh.size());
      while (!rs.done()) {
        uint64_t k2 = rs.varint();
        if ((k2 >> 3) == 2 && (k2 & 7) == 2) {
          std::string_view dim = rs.bytes();
          Reader rd(reinterpret_cast<const uint8_t*>(dim.data()), dim.size());
          int64_t size = 0;
          while (!rd.done()) {
            uint64_t k3 = rd.varint();
            if ((k3 >> 3) == 1 && (k3 & 7) == 0) size = int64_t(rd.varint());
            else rd.skip(int(k3 & 7));
          }
          t.shape.push_back(size);
        } else if ((k2 >> 3) == 3 && (k2 & 7) == 0) {
          t.unknown_rank = rs.varint() != 0;
        } else {
          rs.skip(int(k2 & 7));
        }
      }
    } else if (field == 4 && wt == 2) {
      std::string_view c = r.bytes();
      content_off = size_t(reinterpret_cast<const uint8_t*>(c.data()) - base);
      content_len = c.size();
      have_content = true;
    } else if (field >= 5 && field < kMaxField && field != 14 && field != 15) {
      Seg s{wt, 0, 0, 0};
      if (wt == 2) {
        std::string_view c = r.bytes();
        s.off = size_t(reinterpret_cast<const uint8_t*>(c.data()) - base);
        s.len = c.size();
      } else if (wt == 0) {
        s.val = r.varint();
      } else if (wt == 5) {
        s.val = r.fixed32();
      } else if (wt == 1) {
        s.val = r.fixed64();
      } else {
        throw WireError("bad wire type in TensorProto");
      }
      segs[field].push_back(s);
    } else {
      r.skip(wt);
    }
  }

  const int esz = dtype_size(t.dtype);
  if (have_content && content_len > 0) {
    if (t.dtype == DT_STRING) throw WireError("tensor_content is not valid for DT_STRING");
    if (esz == 0) throw WireError("unsupported dtype " + std::to_string(t.dtype));
    if (content_len % esz) throw WireError("tensor_content size is not a multiple of the element size");
    t.storage = Storage::kView;
    t.offset = content_off;
    t.nbytes = content_len;
    t.count = content_len / esz;
    return;
  }
  const int field = field_for_dtype(t.dtype);
  if (field < 0) throw WireError("unsupported dtype " + std::to_string(t.dtype));
  auto& fs = segs[field];
  if (fs.empty()) {
    t.storage = Storage::kEmpty;
    return;
  }
  if (field == 8) {  // string_val: each segment is one element
    t.storage = Storage::kStrings;
    for (auto& s : fs) {
      if (s.wt != 2) throw WireError("string_val must be length-delimited");
      t.strings.emplace_back(s.off, s.len);
    }
    t.count = t.strings.size();
    return;
  }
  const int fw = fixed_width(field);
  if (fw) {
    // float/double/complex: packed payload == raw LE array of the element type
    if (fs.size() == 1 && fs[0].wt == 2) {
      if (fs[0].len % fw) throw WireError("packed fixed-width field has a ragged length");
      t.storage = Storage::kView;
      t.offset = fs[0].off;
      t.nbytes = fs[0].len;
      t.count = fs[0].len / fw;
      if (t.dtype == DT_COMPLEX64 || t.dtype == DT_COMPLEX128) t.count /= 2;
      return;
    }
    t.storage = Storage::kOwned;
    for (auto& s : fs) {
      if (s.wt == 2) {
        if (s.len % fw) throw WireError("packed fixed-width field has a ragged length");
        t.owned.append(reinterpret_cast<const char*>(base + s.off), s.len);
      } else if ((fw == 4 && s.wt == 5) || (fw == 8 && s.wt == 1)) {
        if (fw == 4) append_value<uint32_t>(t.owned, uint32_t(s.val));
        else append_value<uint64_t>(t.owned, s.val);
      } else {
        throw WireError("wire type mismatch for fixed-width field");
      }
    }
    t.nbytes = t.owned.size();
    t.count = t.nbytes / fw;
    if (t.dtype == DT_COMPLEX64 || t.dtype == DT_COMPLEX128) t.count /= 2;
    return;
  }
  // varint-encoded repeated scalars
  t.storage = Storage::kOwned;
  for (auto& s : fs) {
    if (s.wt == 2) {
      Reader rv(base + s.off, s.len);
      while (!rv.done()) append_converted(t.owned, t.dtype, rv.varint());
    } else if (s.wt == 0) {
      append_converted(t.owned, t.dtype, s.val);
    } else {
      throw WireError("wire type mismatch for varint field");
    }
  }
  t.nbytes = t.owned.size();
  t.count = t.nbytes / esz;
}

// ---------------------------------------------------------------- Predict
void parse_predict_request(const uint8_t* buf, size_t n, PredictRequestView& req) {
  Reader r(buf, n);
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = int(key >> 3), wt = int(key & 7);
    if (field == 1 && wt == 2) {
      parse_model_spec(r.bytes(), req.spec);
      req.has_spec = true;
    } else if (field == 2 && wt == 2) {
      std::string_view entry = r.bytes();
      Reader re(reinterpret_cast<const uint8_t*>(entry.data()), entry.size());
      std::string alias;
      TensorView tv;
      bool have_value = false;
      while (!re.done()) {
        uint64_t k2 = re.varint();
        int f2 = int(k2 >> 3), w2 = int(k2 & 7);
        if (f2 == 1 && w2 == 2) {
          alias = std::string(re.bytes());
        } else if (f2 == 2 && w2 == 2) {
          std::string_view tb = re.bytes();
          tv = TensorView();
          parse_tensor(buf, size_t(reinterpret_cast<const uint8_t*>(tb.data()) - buf), tb.size(), tv);
          have_value = true;
        } else {
          re.skip(w2);
        }
      }
      (void)have_value;
      // proto3 map semantics: last entry for a key wins
      bool replaced = false;
      for (auto& kv : req.inputs) {
        if (kv.first == alias) { kv.second = std::move(tv); replaced = true; break; }
      }
      if (!replaced) req.inputs.emplace_back(std::move(alias), std::move(tv));
    } else if (field == 3 && wt == 2) {
      req.output_filter.emplace_back(r.bytes());
    } else {
      r.skip(wt);
    }
  }
}

void write_tensor(Writer& w, const OutTensor& t, bool use_tensor_content) {
  Writer tp;
  if (t.dtype) tp.varint_field(1, uint64_t(t.dtype));
  {
    Writer sh;
    for (int64_t d : t.shape) {
      Writer dim;
      if (d != 0) dim.varint_field(1, uint64_t(d));
      sh.bytes_field(2, dim.out);
    }
    tp.bytes_field(2, sh.out);
  }
  const int esz = dtype_size(t.dtype);
  if (t.dtype == DT_STRING) {
    if (t.strings)
      for (auto& s : *t.strings) tp.bytes_field(8, s);
  } else if (t.count > 0) {
    if (esz == 0) throw WireError("unsupported output dtype " + std::to_string(t.dtype));
    const size_t nbytes = t.count * size_t(esz);
    const int field = field_for_dtype(t.dtype);
    if (use_tensor_content) {
      tp.tag(4, 2); tp.varint(nbytes); tp.raw(t.data, nbytes);
    } else if (fixed_width(field)) {
      tp.tag(field, 2); tp.varint(nbytes); tp.raw(t.data, nbytes);
    } else {
      // varint-packed: size first, then values
      Writer vals;
      vals.out.reserve(t.count * 2);
      const uint8_t* p = static_cast<const uint8_t*>(t.data);
      for (size_t i = 0; i < t.count; ++i) {
        uint64_t v = 0;
        switch (t.dtype) {
          case DT_INT32: { int32_t x; std::memcpy(&x, p + 4 * i, 4); v = uint64_t(int64_t(x)); break; }
          case DT_INT16: { int16_t x; std::memcpy(&x, p + 2 * i, 2); v = uint64_t(int64_t(x)); break; }
          case DT_INT8: { int8_t x = int8_t(p[i]); v = uint64_t(int64_t(x)); break; }
          case DT_UINT8: v = p[i]; break;
          case DT_BOOL: v = p[i] ? 1 : 0; break;
          case DT_UINT16: case DT_HALF: case DT_BFLOAT16: { uint16_t x; std::memcpy(&x, p + 2 * i, 2); v = x; break; }
          case DT_INT64: { int64_t x; std::memcpy(&x, p + 8 * i, 8); v = uint64_t(x); break; }
          case DT_UINT32: { uint32_t x; std::memcpy(&x, p + 4 * i, 4); v = x; break; }
          case DT_UINT64: { std::memcpy(&v, p + 8 * i, 8); break; }
          default: throw WireError("unsupported output dtype");
        }
        vals.varint(v);
      }
      tp.bytes_field(field, vals.out);
    }
  }
  w.out.append(tp.out);   // TensorProto body (caller wraps it in a field)
}

namespace {
void write_map_entry(Writer& w, int field, const OutTensor& t, bool use_tc) {
  Writer val;
  write_tensor(val, t, use_tc);
  Writer entry;
  entry.bytes_field(1, t.alias);
  entry.bytes_field(2, val.out);
  w.bytes_field(field, entry.out);
}
}  // namespace

std::string encode_predict_response(const ModelSpecView* spec,
                                    const std::vector<OutTensor>& outs,
                                    bool use_tensor_content) {
  Writer w;
  size_t hint = 64;
  for (auto& o : outs) hint += o.count * 8 + 64;
  w.out.reserve(hint);
  for (auto& o : outs) write_map_entry(w, 1, o, use_tensor_content);
  if (spec) write_model_spec(w, 2, *spec);
  return std::move(w.out);
}

std::string encode_predict_request(const ModelSpecView& spec,
                                   const std::vector<OutTensor>& inputs,
                                   const std::vector<std::string>& output_filter,
                                   bool use_tensor_content) {
  Writer w;
  size_t hint = 64;
  for (auto& o : inputs) hint += o.count * 8 + 64;
  w.out.reserve(hint);
  write_model_spec(w, 1, spec);
  for (auto& o : inputs) write_map_entry(w, 2, o, use_tensor_content);
  for (auto& f : output_filter) w.bytes_field(3, f);
  return std::move(w.out);
}

// ---------------------------------------------------------------- crc32c
namespace {
struct Crc32cTable {
  uint32_t t[8][256];
  Crc32cTable() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82f63b78u : (c >> 1);
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Crc32cTable& table() {
  static Crc32cTable tab;
  return tab;
}
}  // namespace

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~crc;
#if defined(__SSE4_2__)
  while (n >= 8) {
    uint64_t v; std::memcpy(&v, p, 8);
    c = uint32_t(_mm_crc32_u64(c, v));
    p += 8; n -= 8;
  }
  while (n--) c = _mm_crc32_u8(c, *p++);
#else
  const auto& T = table().t;
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4); std::memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = T[7][lo & 0xff] ^ T[6][(lo >> 8) & 0xff] ^ T[5][(lo >> 16) & 0xff] ^ T[4][lo >> 24] ^
        T[3][hi & 0xff] ^ T[2][(hi >> 8) & 0xff] ^ T[1][(hi >> 16) & 0xff] ^ T[0][hi >> 24];
    p += 8; n -= 8;
  }
  while (n--) c = T[0][(c ^ *p++) & 0xff] ^ (c >> 8);
#endif
  return ~c;
}

// ---------------------------------------------------------------- streaming probe
Probe probe_predict_header(const uint8_t* buf, size_t n, size_t min_payload, ProbeInfo& out) {
  if (n < 5) return Probe::kNeedMore;
  if (buf[0] != 0) return Probe::kNoStream;   // compressed
  const size_t msglen = (size_t(buf[1]) << 24) | (size_t(buf[2]) << 16) | (size_t(buf[3]) << 8) | buf[4];
  const uint8_t* base = buf + 5;
  const size_t avail = std::min(n - 5, msglen);
  bool have_spec = false;
  try {
    Reader r(base, avail);
    while (true) {
      if (r.done()) return avail == msglen ? Probe::kNoStream : Probe::kNeedMore;
      const uint64_t key = r.varint();
      const int field = int(key >> 3), wt = int(key & 7);
      if (field == 1 && wt == 2) {
        std::string_view sv = r.bytes();
        parse_model_spec(sv, out.spec);
        have_spec = true;
        continue;
      }
      if (field != 2 || wt != 2 || !have_spec) return Probe::kNoStream;
      // inputs map entry: must be the last field of the message
      const uint64_t elen = r.varint();
      const size_t estart = size_t(r.p - base);
      if (estart + elen != msglen) return Probe::kNoStream;
      Reader re(r.p, std::min<size_t>(elen, size_t(r.end - r.p)));
      while (true) {
        if (re.done()) return Probe::kNeedMore;
        const uint64_t k2 = re.varint();
        const int f2 = int(k2 >> 3), w2 = int(k2 & 7);
        if (f2 == 1 && w2 == 2) {
          std::string_view a = re.bytes();
          out.alias.assign(a.data(), a.size());
          continue;
        }
        if (f2 != 2 || w2 != 2 || out.alias.empty()) return Probe::kNoStream;
        const uint64_t tlen = re.varint();
        const size_t tstart = size_t(re.p - base);
        if (tstart + tlen != msglen) return Probe::kNoStream;   // value ends the entry (and message)
        Reader rt(re.p, std::min<size_t>(tlen, size_t(re.end - re.p)));
        while (true) {
          if (rt.done()) return Probe::kNeedMore;
          const uint64_t k3 = rt.varint();
          const int f3 = int(k3 >> 3), w3 = int(k3 & 7);
          if (f3 == 1 && w3 == 0) {
            out.dtype = int(rt.varint());
          } else if (f3 == 2 && w3 == 2) {
            std::string_view sh = rt.bytes();
            Reader rs(reinterpret_cast<const uint8_t*>(sh.data()), sh.size());
            out.shape.clear();
            while (!rs.done()) {
              const uint64_t k4 = rs.varint();
              if ((k4 >> 3) == 2 && (k4 & 7) == 2) {
                std::string_view dim = rs.bytes();
                Reader rd(reinterpret_cast<const uint8_t*>(dim.data()), dim.size());
                int64_t size = 0;
                while (!rd.done()) {
                  const uint64_t k5 = rd.varint();
                  if ((k5 >> 3) == 1 && (k5 & 7) == 0) size = int64_t(rd.varint());
                  else rd.skip(int(k5 & 7));
                }
                out.shape.push_back(size);
              } else if ((k4 >> 3) == 3 && (k4 & 7) == 0) {
                if (rs.varint() != 0) return Probe::kNoStream;   // unknown_rank
              } else {
                rs.skip(int(k4 & 7));
              }
            }
          } else if (f3 == 3 && w3 == 0) {
            rt.varint();   // version_number
          } else if ((f3 == 4 || f3 == 5 || f3 == 6) && w3 == 2) {
            const bool raw_ok = f3 == 4 ? (dtype_size(out.dtype) > 0 && out.dtype != DT_STRING)
                                        : (f3 == 5 ? out.dtype == DT_FLOAT : out.dtype == DT_DOUBLE);
            if (!raw_ok) return Probe::kNoStream;
            const uint64_t plen = rt.varint();
            const size_t poff = size_t(rt.p - base);
            if (poff + plen != msglen || plen < min_payload) return Probe::kNoStream;
            out.payload_off = 5 + poff;
            out.payload_len = size_t(plen);
            return Probe::kFound;
          } else {
            return Probe::kNoStream;
          }
        }
      }
    }
  } catch (const WireError&) {
    return Probe::kNeedMore;   // truncated so far (the caller bounds how long it waits)
  }
}

}  // namespace tfs
