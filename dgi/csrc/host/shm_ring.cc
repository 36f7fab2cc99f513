// Node-local control plane: single-producer / single-consumer message rings in
// POSIX shared memory (one ring per directed rank pair and tag).
//
// Replaces the round-2 control channel, which put every P/D header, credit and
// pipeline hop through the c10d TCPStore on rank 0 (one TCP round trip per
// poll).  All ranks of a node share /dev/shm, so a message is a memcpy into the
// ring plus one release store of the producer cursor; a poll is one acquire
// load.  Reference counterpart: the HTTP/gRPC hops between shard workers
// (reference worker/distributed/session.py:102-166, grpc_server.py:66-140).
//
// The ring itself lives in shm_ring.h (shared with the sanitizer stress driver).
#include <pybind11/pybind11.h>

#include "shm_ring.h"

namespace py = pybind11;
using dgi_shm::Ring;
using dgi_shm::wait_until;

PYBIND11_MODULE(_shm, m) {
  m.doc() = "dgi node-local control plane: SPSC message rings in POSIX shared memory";
  py::class_<Ring>(m, "Ring")
      .def_static("create", &Ring::create, py::arg("name"), py::arg("capacity"),
                  "Create the producer end (the name must not exist).")
      .def_static("try_open", &Ring::try_open, py::arg("name"), py::return_value_policy::take_ownership,
                  "Open the consumer end, or None while the producer has not created it.")
      .def_property_readonly("capacity", &Ring::capacity)
      .def_property_readonly("name", &Ring::name)
      .def_property_readonly("messages", &Ring::messages)
      .def("pending_bytes", &Ring::pending_bytes)
      .def("try_send", [](Ring& r, py::bytes b) {
             char* p;
             ssize_t n;
             PYBIND11_BYTES_AS_STRING_AND_SIZE(b.ptr(), &p, &n);
             return r.try_write(p, static_cast<uint64_t>(n));
           })
      .def("send", [](Ring& r, py::bytes b, double timeout_s) {
             char* p;
             ssize_t n;
             PYBIND11_BYTES_AS_STRING_AND_SIZE(b.ptr(), &p, &n);
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = r.write(p, static_cast<uint64_t>(n), timeout_s);
             }
             if (!ok) throw std::runtime_error("ring " + r.name() + " full for " + std::to_string(timeout_s) + " s");
           }, py::arg("data"), py::arg("timeout_s") = 600.0)
      .def("poll", [](Ring& r) -> py::object {
             if (!r.has_message()) return py::none();
             std::string s = r.read_one();
             return py::bytes(s);
           }, "Next message as bytes, or None.")
      .def("wait", [](Ring& r, double timeout_s) -> py::object {
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = wait_until([&] { return r.has_message(); }, timeout_s);
             }
             if (!ok) return py::none();
             std::string s = r.read_one();
             return py::bytes(s);
           }, py::arg("timeout_s") = -1.0, "Block (GIL released) until a message arrives; None on timeout.");
  m.def("unlink", [](const std::string& name) { return shm_unlink(name.c_str()) == 0; });
}
