// pybind11 bindings of the CPU-side native data plane (`_C`):
//   wire codec (PredictRequest/PredictResponse), crc32c, LevelDB tables
//   (TensorBundle index), mmap'd bundle shards, the HTTP/2 gRPC front end
//   and the dynamic batcher (see server.cpp / batcher.cpp).
#include <pthread.h>
#include <cstring>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "ingest.h"
#include "sstable.h"
#include "wire.h"

namespace py = pybind11;
using namespace tfs;

void register_server(py::module_& m);   // server.cpp

namespace {

struct ConstBuf {
  const uint8_t* ptr;
  size_t len;
  py::buffer_info info;
};

ConstBuf get_buf(const py::buffer& b) {
  py::buffer_info info = b.request();
  if (info.ndim > 1) {
    // require C-contiguous
    ssize_t expect = info.itemsize;
    for (ssize_t i = info.ndim - 1; i >= 0; --i) {
      if (info.strides[i] != expect) throw std::invalid_argument("buffer must be C-contiguous");
      expect *= info.shape[i];
    }
  }
  size_t len = size_t(info.size) * size_t(info.itemsize);
  return ConstBuf{static_cast<const uint8_t*>(info.ptr), len, std::move(info)};
}

py::object spec_to_py(const ModelSpecView& s) {
  return py::make_tuple(py::bytes(s.name),
                        s.has_version ? py::object(py::int_(s.version)) : py::object(py::none()),
                        s.has_label ? py::object(py::bytes(s.version_label)) : py::object(py::none()),
                        py::bytes(s.signature_name));
}

ModelSpecView spec_from_py(const py::handle& o) {
  ModelSpecView s;
  auto t = o.cast<py::tuple>();
  if (t.size() != 4) throw std::invalid_argument("model spec tuple must be (name, version, label, signature)");
  s.name = t[0].cast<std::string>();
  if (!t[1].is_none()) { s.has_version = true; s.version = t[1].cast<int64_t>(); }
  if (!t[2].is_none()) { s.has_label = true; s.version_label = t[2].cast<std::string>(); }
  s.signature_name = t[3].cast<std::string>();
  return s;
}

// outputs: list of (alias, dtype, shape, data) where data is a buffer (numeric)
// or a list of bytes (DT_STRING).
struct OutHolder {
  std::vector<OutTensor> outs;
  std::vector<py::buffer_info> keep;
  std::vector<std::vector<std::string>> strings;
};

void outs_from_py(const py::list& lst, OutHolder& h) {
  h.outs.reserve(lst.size());
  h.strings.reserve(lst.size());
  for (auto item : lst) {
    auto t = item.cast<py::tuple>();
    OutTensor o;
    o.alias = t[0].cast<std::string>();
    o.dtype = t[1].cast<int>();
    o.shape = t[2].cast<std::vector<int64_t>>();
    if (o.dtype == DT_STRING) {
      h.strings.emplace_back();
      for (auto s : t[3].cast<py::list>()) h.strings.back().push_back(s.cast<std::string>());
      o.strings = &h.strings.back();
      o.count = h.strings.back().size();
      o.data = nullptr;
    } else {
      ConstBuf b = get_buf(t[3].cast<py::buffer>());
      int esz = dtype_size(o.dtype);
      if (esz == 0) throw std::invalid_argument("unsupported dtype " + std::to_string(o.dtype));
      if (b.len % esz) throw std::invalid_argument("buffer size is not a multiple of the dtype size");
      o.data = b.ptr;
      o.count = b.len / size_t(esz);
      h.keep.push_back(std::move(b.info));
    }
    h.outs.push_back(std::move(o));
  }
}

py::tuple parse_predict(const py::buffer& buf) {
  ConstBuf b = get_buf(buf);
  PredictRequestView req;
  {
    py::gil_scoped_release nogil;
    parse_predict_request(b.ptr, b.len, req);
  }
  py::list inputs;
  for (auto& kv : req.inputs) {
    const TensorView& t = kv.second;
    py::object owned = py::none(), strs = py::none();
    if (t.storage == Storage::kOwned) owned = py::bytes(t.owned);
    if (t.storage == Storage::kStrings) {
      py::list l;
      for (auto& s : t.strings) l.append(py::bytes(reinterpret_cast<const char*>(b.ptr + s.first), s.second));
      strs = l;
    }
    inputs.append(py::make_tuple(py::bytes(kv.first), t.dtype, py::cast(t.shape), t.unknown_rank,
                                 int(t.storage), t.offset, t.nbytes, t.count, owned, strs));
  }
  py::list filt;
  for (auto& f : req.output_filter) filt.append(py::bytes(f));
  return py::make_tuple(req.has_spec ? spec_to_py(req.spec) : py::object(py::none()), inputs, filt);
}

py::bytes encode_response(const py::object& spec, const py::list& outputs, bool use_tc) {
  OutHolder h;
  outs_from_py(outputs, h);
  ModelSpecView s;
  const bool has = !spec.is_none();
  if (has) s = spec_from_py(spec);
  std::string out;
  {
    py::gil_scoped_release nogil;
    out = encode_predict_response(has ? &s : nullptr, h.outs, use_tc);
  }
  return py::bytes(out);
}

py::bytes encode_request(const py::object& spec, const py::list& inputs, const py::list& filt, bool use_tc) {
  OutHolder h;
  outs_from_py(inputs, h);
  ModelSpecView s = spec_from_py(spec);
  std::vector<std::string> f;
  for (auto x : filt) f.push_back(x.cast<std::string>());
  std::string out;
  {
    py::gil_scoped_release nogil;
    out = encode_predict_request(s, h.outs, f, use_tc);
  }
  return py::bytes(out);
}

// The reference's image hot loop (src/lib.rs:237-242: raw_pixels() u8 -> f32
// -> preprocessing_fn -> float_val) in one native pass: `lut` holds the
// preprocessing function's value for each of the 256 possible pixel values
// (any f32 -> f32 function of a u8 pixel is exactly a 256-entry table), so
// every pixel is one table lookup written straight into the float_val array.
// `dims` is the shape the reference sends ([1, width, height, 3]) even when
// the pixel count disagrees (grayscale / RGBA: the server must reject it).
py::bytes encode_image_request(const py::object& spec, const std::string& alias, const py::buffer& pixels,
                               const std::vector<int64_t>& dims, const py::buffer& lut) {
  ConstBuf px = get_buf(pixels);
  ConstBuf lb = get_buf(lut);
  if (lb.len != 256 * sizeof(float)) throw std::invalid_argument("lut must hold 256 float32 values");
  ModelSpecView s = spec_from_py(spec);
  std::string out;
  {
    py::gil_scoped_release nogil;
    std::vector<float> vals(px.len);
    float table[256];
    std::memcpy(table, lb.ptr, sizeof(table));
    for (size_t i = 0; i < px.len; ++i) vals[i] = table[px.ptr[i]];
    OutTensor t;
    t.alias = alias;
    t.dtype = DT_FLOAT;
    t.shape = dims;
    t.data = vals.data();
    t.count = vals.size();
    out = encode_predict_request(s, {t}, {}, false);
  }
  return py::bytes(out);
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "rust_tensorflow_serving2_amd native CPU data plane";
  py::register_exception<WireError>(m, "WireError", PyExc_ValueError);

  m.def("parse_predict_request", &parse_predict, py::arg("buf"),
        "Decode PredictRequest bytes -> (spec, inputs, output_filter). Numeric inputs come back as "
        "(offset, nbytes) views into `buf` when the wire bytes are already the raw array.");
  m.def("encode_predict_response", &encode_response, py::arg("spec"), py::arg("outputs"),
        py::arg("use_tensor_content") = false);
  m.def("encode_predict_request", &encode_request, py::arg("spec"), py::arg("inputs"),
        py::arg("output_filter") = py::list(), py::arg("use_tensor_content") = false);
  m.def("encode_image_request", &encode_image_request, py::arg("spec"), py::arg("alias"), py::arg("pixels"),
        py::arg("dims"), py::arg("lut"),
        "PredictRequest of one DT_FLOAT float_val tensor from u8 pixels mapped through a 256-entry table");

  m.def("ingest_f32_to_bf16", [](py::bytes b) {
    const std::string in = b;
    std::string out(in.size() / 4 * 2, '\0');
    {
      py::gil_scoped_release nogil;
      tfs::ingest_f32_to_bf16(reinterpret_cast<uint16_t*>(&out[0]), reinterpret_cast<const uint8_t*>(in.data()),
                              in.size() / 4);
    }
    return py::bytes(out);
  }, py::arg("f32_bytes"), "fp32 bytes -> bf16 bytes (the fast path's ingest conversion, csrc/ingest.h)");
  m.def("set_thread_name", [](const std::string& name) {
    // OS-level thread name (<= 15 chars), visible in /proc/<pid>/task/*/comm
    pthread_setname_np(pthread_self(), name.substr(0, 15).c_str());
  });
  m.def("crc32c", [](const py::buffer& b, uint32_t init) {
    ConstBuf cb = get_buf(b);
    py::gil_scoped_release nogil;
    return crc32c_extend(init, cb.ptr, cb.len);
  }, py::arg("data"), py::arg("init") = 0);
  m.def("crc32c_mask", &crc32c_mask);
  m.def("crc32c_unmask", &crc32c_unmask);

  m.def("sstable_build", [](const std::vector<std::pair<py::bytes, py::bytes>>& kvs, size_t block_size) {
    std::vector<std::pair<std::string, std::string>> v;
    v.reserve(kvs.size());
    for (auto& kv : kvs) v.emplace_back(std::string(kv.first), std::string(kv.second));
    std::string out;
    {
      py::gil_scoped_release nogil;
      out = sstable_build(v, block_size);
    }
    return py::bytes(out);
  }, py::arg("kvs"), py::arg("block_size") = 256 * 1024);
  m.def("sstable_read", [](const py::buffer& b, bool verify) {
    ConstBuf cb = get_buf(b);
    std::vector<std::pair<std::string, std::string>> kvs;
    {
      py::gil_scoped_release nogil;
      kvs = sstable_read(cb.ptr, cb.len, verify);
    }
    py::list out;
    for (auto& kv : kvs) out.append(py::make_tuple(py::bytes(kv.first), py::bytes(kv.second)));
    return out;
  }, py::arg("data"), py::arg("verify") = true);

  py::class_<MappedFile>(m, "MappedFile", py::buffer_protocol())
      .def(py::init<const std::string&>())
      .def("__len__", &MappedFile::size)
      .def("crc32c", [](const MappedFile& f, size_t off, size_t n) {
        if (off + n > f.size()) throw std::out_of_range("range outside mapped file");
        py::gil_scoped_release nogil;
        return crc32c(f.data() + off, n);
      })
      .def_buffer([](MappedFile& f) -> py::buffer_info {
        return py::buffer_info(const_cast<uint8_t*>(f.data()), 1, py::format_descriptor<uint8_t>::format(),
                               1, {ssize_t(f.size())}, {ssize_t(1)}, /*readonly=*/true);
      });

  register_server(m);
}
