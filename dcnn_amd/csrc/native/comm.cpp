// placeholder: TCP control plane is added in a later milestone
#include <pybind11/pybind11.h>
namespace py = pybind11;
void bind_comm(py::module_& m) {}
