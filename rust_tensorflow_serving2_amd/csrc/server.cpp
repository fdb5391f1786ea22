// placeholder: HTTP/2 front end lands in a later commit
#include <pybind11/pybind11.h>
namespace py = pybind11;
void register_server(py::module_& m) { (void)m; }
