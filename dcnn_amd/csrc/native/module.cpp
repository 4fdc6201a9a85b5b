// pybind11 module of the host C++ runtime.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "native.h"

namespace py = pybind11;
using namespace dcnn_native;

void bind_comm(py::module_& m);   // comm.cpp
void bind_data(py::module_& m);   // data.cpp
void bind_cpu(py::module_& m);    // cpu_bind.cpp

PYBIND11_MODULE(_native, m) {
  m.doc() = "dcnn_amd host runtime (C++)";
  m.def("parse_env_text", &parse_env_text);
  m.def("load_env_file", &load_env_file, py::arg("path"), py::arg("overwrite") = false);
  m.def("read_cpu_info", []() {
    CpuInfo c = read_cpu_info();
    py::dict d;
    d["vendor"] = c.vendor;
    d["model_name"] = c.model_name;
    d["logical_cores"] = c.logical_cores;
    d["physical_cores"] = c.physical_cores;
    d["sockets"] = c.sockets;
    d["base_mhz"] = c.base_mhz;
    d["max_mhz"] = c.max_mhz;
    d["flags"] = c.flags;
    d["caches_kb"] = c.caches_kb;
    d["total_mem_kb"] = c.total_mem_kb;
    d["avail_mem_kb"] = c.avail_mem_kb;
    d["cgroup_mem_limit_bytes"] = c.cgroup_mem_limit_bytes;
    d["cgroup_cpu_quota"] = c.cgroup_cpu_quota;
    d["pcores"] = c.pcores;
    d["ecores"] = c.ecores;
    return d;
  });
  m.def("cpu_utilization", &cpu_utilization, py::arg("sample_ms") = 100, py::call_guard<py::gil_scoped_release>());
  m.def("cpu_utilization_total", &cpu_utilization_total, py::arg("sample_ms") = 100,
        py::call_guard<py::gil_scoped_release>());
  m.def("process_rss_kb", &process_rss_kb);
  m.def("thermal_zones", &thermal_zones);
  m.def("set_thread_affinity", &set_thread_affinity);
  m.def("get_thread_affinity", &get_thread_affinity);
  bind_comm(m);
  bind_data(m);
  bind_cpu(m);
}
