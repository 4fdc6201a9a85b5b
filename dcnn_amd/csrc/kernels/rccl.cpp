// Python binding of the in-tree RCCL communicator (collective.h): parallel/rccl.py's data plane.
// Collectives take raw device pointers and the caller's hipStream_t (uintptr_t), exactly like the
// compute kernels of this library; the communicator constructor releases the GIL while it waits
// for the other ranks.
#include <cstdint>
#include <string>

#include <pybind11/pybind11.h>

#include "collective.h"

namespace py = pybind11;

namespace {
using dcnn::coll::Comm;
void* S(uintptr_t s) { return reinterpret_cast<void*>(s); }
const void* C(uintptr_t p) { return reinterpret_cast<const void*>(p); }
void* M(uintptr_t p) { return reinterpret_cast<void*>(p); }
}  // namespace

void bind_rccl(py::module_& m) {
  namespace coll = dcnn::coll;
  auto r = m.def_submodule("rccl", "in-tree RCCL communicator (librccl.so, dlopen'ed)");
  r.def("available", &coll::available);
  r.def("load_error", &coll::load_error);
  r.def("version", &coll::version);
  r.def("unique_id", [] { return py::bytes(coll::unique_id()); });
  r.def("group_start", &coll::group_start);
  r.def("group_end", &coll::group_end);
  py::class_<Comm>(r, "Comm")
      .def(py::init([](py::bytes uid, int world, int rank, int device) {
             std::string s = uid;
             py::gil_scoped_release nogil;  // blocks until every rank has joined
             return new Comm(s, world, rank, device);
           }),
           py::arg("unique_id"), py::arg("world"), py::arg("rank"), py::arg("device"))
      .def_property_readonly("world", &Comm::world)
      .def_property_readonly("rank", &Comm::rank)
      .def("all_reduce",
           [](Comm& c, uintptr_t send, uintptr_t recv, size_t count, int dt, int op, uintptr_t st) {
             c.all_reduce(C(send), M(recv), count, dt, op, S(st));
           },
           py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("stream"))
      .def("broadcast", [](Comm& c, uintptr_t send, uintptr_t recv, size_t count, int dt, int root,
                           uintptr_t st) { c.broadcast(C(send), M(recv), count, dt, root, S(st)); })
      .def("all_gather", [](Comm& c, uintptr_t send, uintptr_t recv, size_t count, int dt, uintptr_t st) {
        c.all_gather(C(send), M(recv), count, dt, S(st));
      })
      .def("reduce_scatter", [](Comm& c, uintptr_t send, uintptr_t recv, size_t count, int dt, int op,
                                uintptr_t st) { c.reduce_scatter(C(send), M(recv), count, dt, op, S(st)); })
      .def("send", [](Comm& c, uintptr_t buf, size_t count, int dt, int peer, uintptr_t st) {
        c.send(C(buf), count, dt, peer, S(st));
      })
      .def("recv", [](Comm& c, uintptr_t buf, size_t count, int dt, int peer, uintptr_t st) {
        c.recv(M(buf), count, dt, peer, S(st));
      })
      .def("destroy", &Comm::destroy);
}
