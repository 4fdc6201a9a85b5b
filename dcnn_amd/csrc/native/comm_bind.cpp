// pybind11 bindings of the control plane (comm.h).  Tensor payloads are exposed through the
// buffer protocol (zero-copy numpy views that keep the Message alive).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "comm.h"

namespace py = pybind11;
using namespace dcnn_native;

static void set_tensor(Message& m, uint64_t mb_id, py::buffer buf, int dtype, int codec, int level, bool legacy) {
  py::buffer_info bi = buf.request();
  std::vector<uint64_t> shape;
  for (auto d : bi.shape) shape.push_back(static_cast<uint64_t>(d));
  // require C-contiguous
  ssize_t expect = bi.itemsize;
  for (ssize_t i = bi.ndim - 1; i >= 0; --i) {
    if (bi.shape[i] > 1 && bi.strides[i] != expect) throw std::runtime_error("set_tensor: buffer must be C-contiguous");
    expect *= bi.shape[i];
  }
  const size_t nbytes = static_cast<size_t>(bi.size * bi.itemsize);
  m.mb_id = mb_id;
  m.shape = std::move(shape);
  m.dtype = static_cast<uint8_t>(dtype);
  {
    py::gil_scoped_release nogil;
    std::string raw(static_cast<const char*>(bi.ptr), nbytes);
    if (legacy) {
      if (dtype != 0 || codec != CODEC_NONE) throw std::runtime_error("legacy Job<float> payload is float32/raw only");
      m.payload_type = P_JOB;
      m.codec = CODEC_NONE;
      m.data = std::move(raw);
    } else {
      m.payload_type = P_TYPED_JOB;
      m.codec = static_cast<uint8_t>(codec);
      m.data = codec == CODEC_NONE ? std::move(raw) : compress(raw, static_cast<Codec>(codec), level);
    }
  }
}

void bind_comm(py::module_& m) {
  auto c = m.def_submodule("comm", "pipeline control plane (messages, TCP / in-process communicators)");
  py::dict cmds;
  for (uint16_t i = 0; i < CMD_COUNT; ++i) cmds[command_name(i)] = i;
  c.attr("COMMANDS") = cmds;
  c.def("command_name", &command_name);
  c.def("zstd_available", &zstd_available);

  py::class_<Message>(c, "Message", py::buffer_protocol())
      .def(py::init<>())
      .def(py::init([](std::string recipient, uint16_t cmd) {
             Message x;
             x.recipient = std::move(recipient);
             x.command = cmd;
             return x;
           }),
           py::arg("recipient"), py::arg("command"))
      .def_readwrite("recipient", &Message::recipient)
      .def_readwrite("sender", &Message::sender)
      .def_readwrite("command", &Message::command)
      .def_readwrite("payload_type", &Message::payload_type)
      .def_readwrite("mb_id", &Message::mb_id)
      .def_readwrite("dtype", &Message::dtype)
      .def_readwrite("codec", &Message::codec)
      .def_readwrite("shape", &Message::shape)
      .def_property(
          "text", [](const Message& x) { return py::bytes(x.text); },
          [](Message& x, py::bytes s) {
            x.text = std::string(s);
            x.payload_type = P_STRING;
          })
      .def_property(
          "flag", [](const Message& x) { return x.flag; },
          [](Message& x, bool f) {
            x.flag = f;
            x.payload_type = P_BOOL;
          })
      .def_property(
          "load",
          [](const Message& x) {
            return py::make_tuple(x.load.avg_forward_ms, x.load.avg_backward_ms, x.load.avg_cpu_utilization,
                                  x.load.max_memory_mb);
          },
          [](Message& x, std::tuple<float, float, float, float> t) {
            x.load = {std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)};
            x.payload_type = P_LOAD;
          })
      .def("set_tensor", &set_tensor, py::arg("mb_id"), py::arg("buffer"), py::arg("dtype") = 0,
           py::arg("codec") = 0, py::arg("level") = 3, py::arg("legacy") = false)
      .def("set_job_meta",
           [](Message& x, uint64_t mb, std::vector<uint64_t> shape, int dtype) {
             x.payload_type = P_TYPED_JOB;
             x.mb_id = mb;
             x.shape = std::move(shape);
             x.dtype = static_cast<uint8_t>(dtype);
             x.codec = CODEC_NONE;
             x.data.clear();
           })
      .def("decompress",
           [](Message& x) {
             if (x.codec == CODEC_NONE) return;
             py::gil_scoped_release nogil;
             x.data = decompress(x.data, static_cast<Codec>(x.codec), 0);
             x.codec = CODEC_NONE;
           })
      .def_property_readonly("nbytes", [](const Message& x) { return x.data.size(); })
      .def("body_size", &Message::body_size)
      .def_buffer([](Message& x) -> py::buffer_info {
        return py::buffer_info(x.data.empty() ? nullptr : &x.data[0], 1, py::format_descriptor<uint8_t>::format(), 1,
                               {static_cast<ssize_t>(x.data.size())}, {1});
      })
      .def("__repr__", [](const Message& x) {
        return "<Message " + std::string(command_name(x.command)) + " " + x.sender + "->" + x.recipient +
               " payload=" + std::to_string(x.payload_type) + " bytes=" + std::to_string(x.data.size()) + ">";
      });

  c.def("serialize", [](const Message& x) { return py::bytes(serialize(x)); });
  c.def("deserialize", [](py::bytes b) { return deserialize(std::string(b)); });
  c.def("compress", [](py::bytes b, int codec, int level) {
    std::string in(b);
    std::string out;
    {
      py::gil_scoped_release nogil;
      out = compress(in, static_cast<Codec>(codec), level);
    }
    return py::bytes(out);
  }, py::arg("data"), py::arg("codec") = 2, py::arg("level") = 3);
  c.def("decompress", [](py::bytes b, int codec, size_t hint) {
    std::string in(b);
    std::string out;
    {
      py::gil_scoped_release nogil;
      out = decompress(in, static_cast<Codec>(codec), hint);
    }
    return py::bytes(out);
  }, py::arg("data"), py::arg("codec") = 2, py::arg("raw_size") = 0);

  py::class_<Communicator>(c, "Communicator")
      .def_property_readonly("id", &Communicator::id)
      .def("send",
           [](Communicator& self, Message& msg) {
             Message tmp = std::move(msg);  // a sent message's payload is consumed
             py::gil_scoped_release nogil;
             self.send(std::move(tmp));
           })
      .def("recv",
           [](Communicator& self, int timeout_ms) -> py::object {
             Message out;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = self.queue().pop(out, timeout_ms);
             }
             if (!ok) return py::none();
             return py::cast(std::move(out));
           },
           py::arg("timeout_ms") = -1)
      .def("recv_command",
           [](Communicator& self, uint16_t cmd, int timeout_ms) -> py::object {
             Message out;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = self.queue().pop_command(cmd, out, timeout_ms);
             }
             if (!ok) return py::none();
             return py::cast(std::move(out));
           },
           py::arg("command"), py::arg("timeout_ms") = -1)
      .def("recv_any",
           [](Communicator& self, std::vector<uint16_t> cmds, int timeout_ms) -> py::object {
             Message out;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = self.queue().pop_any(cmds, out, timeout_ms);
             }
             if (!ok) return py::none();
             return py::cast(std::move(out));
           },
           py::arg("commands"), py::arg("timeout_ms") = -1)
      .def("deliver_local", [](Communicator& self, Message& msg) { self.queue().push(std::move(msg)); })
      .def("pending", [](Communicator& self) { return self.queue().size(); })
      .def("count", [](Communicator& self, uint16_t cmd) { return self.queue().count(cmd); })
      .def("peers", &Communicator::peers)
      .def_property_readonly("bytes_sent", &Communicator::bytes_sent)
      .def_property_readonly("bytes_received", &Communicator::bytes_received)
      .def_property_readonly("messages_sent", &Communicator::messages_sent)
      .def_property_readonly("messages_received", &Communicator::messages_received)
      .def("close", &Communicator::close, py::call_guard<py::gil_scoped_release>());

  py::class_<InProcessCommunicator, Communicator>(c, "InProcessCommunicator")
      .def(py::init<std::string>(), py::arg("id"))
      .def("alias", &InProcessCommunicator::alias);

  py::class_<TcpCommunicator, Communicator>(c, "TcpCommunicator")
      .def("set_id", &TcpCommunicator::set_id)
      .def(py::init<std::string, const std::string&, int>(), py::arg("id"), py::arg("host") = "0.0.0.0",
           py::arg("port") = 0)
      .def_property_readonly("port", &TcpCommunicator::port)
      .def("connect", &TcpCommunicator::connect, py::arg("name"), py::arg("host"), py::arg("port"),
           py::arg("timeout_ms") = 30000, py::call_guard<py::gil_scoped_release>())
      .def("alias", &TcpCommunicator::alias)
      .def("wait_for_peer", &TcpCommunicator::wait_for_peer, py::arg("name"), py::arg("timeout_ms") = 30000,
           py::call_guard<py::gil_scoped_release>());
}
