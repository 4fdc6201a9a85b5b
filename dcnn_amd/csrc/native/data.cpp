// placeholder: dataset parsers / augmentation are added in a later milestone
#include <pybind11/pybind11.h>
namespace py = pybind11;
void bind_data(py::module_& m) {}
