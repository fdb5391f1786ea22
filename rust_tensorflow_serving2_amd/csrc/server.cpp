// pybind11 registration of the HTTP/2 front end, Predict fast path and load generator.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>

#include "batcher.h"
#include "http2.h"

namespace py = pybind11;
using namespace tfs;

namespace {

struct PyServer {
  std::unique_ptr<Server> srv;
  std::unique_ptr<FastPath> fast;
};

// A slow-path call handed to Python.
struct PyCall {
  std::unique_ptr<Call> call;
};

std::vector<TensorSpecC> specs_from(const py::list& l) {
  std::vector<TensorSpecC> out;
  for (auto it : l) {
    auto t = it.cast<py::tuple>();
    TensorSpecC s;
    s.alias = t[0].cast<std::string>();
    s.dtype = t[1].cast<int>();
    s.row_shape = t[2].cast<std::vector<int64_t>>();
    s.row_elems = 1;
    for (auto d : s.row_shape) s.row_elems *= size_t(d);
    const int esz = dtype_size(s.dtype);
    if (esz == 0) throw std::invalid_argument("fast path: unsupported dtype for " + s.alias);
    s.row_bytes = s.row_elems * size_t(esz);
    out.push_back(std::move(s));
  }
  std::sort(out.begin(), out.end(), [](const TensorSpecC& a, const TensorSpecC& b) { return a.alias < b.alias; });
  return out;
}

}  // namespace

void register_server(py::module_& m) {
  py::class_<PyCall>(m, "Call")
      .def_property_readonly("method", [](const PyCall& c) { return c.call->method; })
      .def_property_readonly("body", [](const PyCall& c) {
        return py::bytes(reinterpret_cast<const char*>(c.call->data()), c.call->size());
      })
      .def_property_readonly("timeout_us", [](const PyCall& c) { return c.call->timeout_us; });

  py::class_<PyServer>(m, "Http2Server")
      .def(py::init([](const std::string& host, int port, int io_threads, size_t max_message) {
             auto p = std::make_unique<PyServer>();
             p->srv = std::make_unique<Server>(host, port, io_threads, max_message);
             p->fast = std::make_unique<FastPath>(p->srv.get());
             FastPath* fp = p->fast.get();
             p->srv->set_fast_dispatch([fp](std::unique_ptr<Call>& c) { return fp->try_dispatch(c); });
             p->srv->set_stream_reserve([fp](const ProbeInfo& pi) { return fp->reserve_stream(pi); });
             return p;
           }),
           py::arg("host"), py::arg("port"), py::arg("io_threads") = 4, py::arg("max_message") = size_t(2147483647))
      .def_property_readonly("port", [](const PyServer& s) { return s.srv->port(); })
      .def("start", [](PyServer& s) { s.srv->start(); })
      .def("stop", [](PyServer& s) {
        py::gil_scoped_release nogil;
        s.srv->stop();
      })
      .def("next_call", [](PyServer& s, int timeout_ms) -> py::object {
        std::unique_ptr<Call> c;
        {
          py::gil_scoped_release nogil;
          c = s.srv->next_call(timeout_ms);
        }
        if (!c) return py::none();
        auto pc = std::make_unique<PyCall>();
        pc->call = std::move(c);
        return py::cast(std::move(pc));
      }, py::arg("timeout_ms") = 100)
      .def("respond", [](PyServer& s, PyCall& c, int status, const std::string& message, const py::bytes& body) {
        if (!c.call) throw std::runtime_error("call already answered");
        std::string b = body;
        s.srv->respond(*c.call, status, message, std::move(b));
        c.call.reset();
      }, py::arg("call"), py::arg("status"), py::arg("message"), py::arg("body"))
      .def("stats", [](PyServer& s) {
        auto& st = s.srv->stats;
        py::dict d;
        d["connections"] = st.connections.load(); d["requests"] = st.requests.load();
        d["fast_path"] = st.fast_path.load(); d["slow_path"] = st.slow_path.load();
        d["streamed"] = st.streamed.load();
        d["responses"] = st.responses.load(); d["errors"] = st.errors.load();
        d["bytes_in"] = st.bytes_in.load(); d["bytes_out"] = st.bytes_out.load();
        d["io_s_recv"] = st.ns_recv.load() * 1e-9; d["io_s_h2"] = st.ns_h2.load() * 1e-9;
        d["io_s_dispatch"] = st.ns_dispatch.load() * 1e-9; d["io_s_send"] = st.ns_send.load() * 1e-9;
        return d;
      })
      // ---- fast path endpoints
      .def("add_endpoint", [](PyServer& s, const std::string& model, int64_t version, const std::string& sig,
                              const py::list& inputs, const py::list& outputs, int max_rows, int64_t timeout_us,
                              int max_wait_ms) {
        const int id = s.fast->next_id();
        auto ep = std::make_shared<Endpoint>(id, model, version, sig, specs_from(inputs), specs_from(outputs),
                                             max_rows, timeout_us, max_wait_ms);
        return s.fast->add_endpoint(ep);
      }, py::arg("model"), py::arg("version"), py::arg("signature"), py::arg("inputs"), py::arg("outputs"),
         py::arg("max_rows"), py::arg("timeout_us"), py::arg("max_wait_ms") = 200)
      .def("endpoint_io_order", [](PyServer& s, int id) {
        auto ep = s.fast->endpoint(id);
        if (!ep) throw std::invalid_argument("no such endpoint");
        py::list ins, outs;
        for (auto& t : ep->inputs) ins.append(t.alias);
        for (auto& t : ep->outputs) outs.append(t.alias);
        return py::make_tuple(ins, outs);
      })
      .def("set_slot_buffers", [](PyServer& s, int id, int slot, const std::vector<uintptr_t>& in_ptrs,
                                  const std::vector<uintptr_t>& out_ptrs) {
        auto ep = s.fast->endpoint(id);
        if (!ep) throw std::invalid_argument("no such endpoint");
        if (in_ptrs.size() != ep->inputs.size() || out_ptrs.size() != ep->outputs.size())
          throw std::invalid_argument("buffer count mismatch");
        std::vector<uint8_t*> in;
        std::vector<const uint8_t*> out;
        for (auto p : in_ptrs) in.push_back(reinterpret_cast<uint8_t*>(p));
        for (auto p : out_ptrs) out.push_back(reinterpret_cast<const uint8_t*>(p));
        ep->set_slot_buffers(slot, in, out);
      })
      .def("set_route", [](PyServer& s, const std::string& model, const std::string& sig, int64_t version, int id) {
        s.fast->set_route(model, sig, version, id);
      })
      .def("clear_routes", [](PyServer& s, const std::string& model) { s.fast->clear_routes(model); })
      .def("remove_endpoint", [](PyServer& s, int id) {
        py::gil_scoped_release nogil;
        s.fast->remove_endpoint(id);
      })
      .def("acquire", [](PyServer& s, int id, int slot, int timeout_ms) {
        auto ep = s.fast->endpoint(id);
        if (!ep) return -1;
        py::gil_scoped_release nogil;
        return ep->acquire(slot, timeout_ms);
      })
      .def("complete", [](PyServer& s, int id, int slot) {
        auto ep = s.fast->endpoint(id);
        if (!ep) return;
        py::gil_scoped_release nogil;
        ep->complete(slot, *s.srv);
      })
      .def("fail", [](PyServer& s, int id, int slot, int code, const std::string& msg) {
        auto ep = s.fast->endpoint(id);
        if (!ep) return;
        py::gil_scoped_release nogil;
        ep->fail(slot, *s.srv, code, msg);
      })
      .def("endpoint_stats", [](PyServer& s, int id) {
        auto ep = s.fast->endpoint(id);
        py::dict d;
        if (!ep) return d;
        auto st = ep->stats();
        d["requests"] = st.requests; d["batches"] = st.batches; d["rows"] = st.rows; d["rejected"] = st.rejected;
        return d;
      });

  m.def("run_loadgen", [](const std::string& host, int port, const std::string& method, const py::list& bodies,
                          uint64_t total, int concurrency, int connections, int threads, double timeout_s) {
    std::vector<std::string> b;
    for (auto x : bodies) b.push_back(x.cast<std::string>());
    LoadGenResult r;
    {
      py::gil_scoped_release nogil;
      r = run_loadgen(host, port, method, b, total, concurrency, connections, threads, timeout_s);
    }
    py::dict d;
    d["ok"] = r.ok; d["errors"] = r.errors; d["elapsed_s"] = r.elapsed_s;
    d["latency_us"] = r.latency_us; d["first_error"] = r.first_error;
    d["bytes_sent"] = r.bytes_sent; d["bytes_recv"] = r.bytes_recv; d["cpu_s"] = r.cpu_s;
    return d;
  }, py::arg("host"), py::arg("port"), py::arg("method"), py::arg("bodies"), py::arg("total"),
     py::arg("concurrency") = 64, py::arg("connections") = 8, py::arg("threads") = 4, py::arg("timeout_s") = 120.0);
}
