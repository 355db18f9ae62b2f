// pybind11 module dtg._runtime: the C++ parameter-server service/client and TensorBundle I/O.
// Blocking calls release the GIL so Python threads (hooks, heartbeats, the chief's SyncReplicas
// aggregation thread) keep running while a call waits on the network or a server-side queue.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "dtg/bundle.h"
#include "dtg/ps.h"

namespace py = pybind11;
using namespace dtg;

namespace {

uint8_t np_to_wire(const py::dtype& dt) {
  if (dt.is(py::dtype::of<float>())) return wire::F32;
  if (dt.is(py::dtype::of<double>())) return wire::F64;
  if (dt.is(py::dtype::of<int32_t>())) return wire::I32;
  if (dt.is(py::dtype::of<int64_t>())) return wire::I64;
  if (dt.is(py::dtype::of<uint16_t>())) return wire::BF16;  // raw bf16 bits
  throw std::runtime_error("unsupported numpy dtype for the PS wire format");
}

py::dtype wire_to_np(uint8_t dt) {
  switch (dt) {
    case wire::F32: return py::dtype::of<float>();
    case wire::F64: return py::dtype::of<double>();
    case wire::I32: return py::dtype::of<int32_t>();
    case wire::I64: return py::dtype::of<int64_t>();
    case wire::BF16: return py::dtype::of<uint16_t>();
  }
  throw std::runtime_error("bad wire dtype");
}

void put_array(wire::Writer& w, py::array a) {
  a = py::array::ensure(a, py::array::c_style);
  std::vector<int64_t> shape(a.shape(), a.shape() + a.ndim());
  w.tensor(np_to_wire(a.dtype()), shape, a.data(), (uint64_t)a.nbytes());
}

py::array to_array(const wire::Tensor& t) {
  std::vector<py::ssize_t> shape(t.shape.begin(), t.shape.end());
  py::array a(wire_to_np(t.dtype), shape);
  if (!t.data.empty()) memcpy(a.mutable_data(), t.data.data(), t.data.size());
  return a;
}

class PyClient {
 public:
  PyClient(const std::string& host, int port, double timeout) {
    py::gil_scoped_release nogil;
    c_ = std::make_unique<ps::Client>(host, port, timeout);
  }

  // returns (status, reader-owned buffer)
  int32_t call(uint16_t op, const wire::Writer& w, std::vector<uint8_t>* resp) {
    int32_t st;
    {
      py::gil_scoped_release nogil;
      st = c_->call(op, w.buf, resp);
    }
    if (st == wire::ERR) {
      wire::Reader r(resp->data(), resp->size());
      throw std::runtime_error("ps server error: " + r.str());
    }
    return st;
  }

  bool ping() {
    wire::Writer w;
    std::vector<uint8_t> r;
    return call(wire::PING, w, &r) == wire::OK;
  }

  bool create(const std::string& name, py::array init, bool overwrite) {
    wire::Writer w;
    w.str(name);
    put_array(w, init);
    w.i64(overwrite);
    std::vector<uint8_t> r;
    call(wire::CREATE, w, &r);
    wire::Reader rd(r.data(), r.size());
    return rd.i64() != 0;
  }

  py::list read(const std::vector<std::string>& names) {
    wire::Writer w;
    w.i64((int64_t)names.size());
    for (auto& n : names) w.str(n);
    std::vector<uint8_t> r;
    call(wire::READ, w, &r);
    wire::Reader rd(r.data(), r.size());
    py::list out;
    for (size_t i = 0; i < names.size(); ++i) out.append(to_array(rd.tensor()));
    return out;
  }

  void assign(const std::vector<std::pair<std::string, py::array>>& items) {
    wire::Writer w;
    w.i64((int64_t)items.size());
    for (auto& kv : items) {
      w.str(kv.first);
      put_array(w, kv.second);
    }
    std::vector<uint8_t> r;
    call(wire::ASSIGN, w, &r);
  }

  py::array assign_add(const std::string& name, py::array delta) {
    wire::Writer w;
    w.str(name);
    put_array(w, delta);
    std::vector<uint8_t> r;
    call(wire::ASSIGN_ADD, w, &r);
    wire::Reader rd(r.data(), r.size());
    return to_array(rd.tensor());
  }

  py::tuple apply(int64_t opt, const std::vector<double>& hyper, bool locking, const std::string& global_step,
                  const std::vector<std::pair<std::string, py::array>>& grads, bool read_back) {
    wire::Writer w;
    w.i64(opt);
    for (int i = 0; i < 5; ++i) w.f64(i < (int)hyper.size() ? hyper[i] : 0.0);
    w.i64(locking);
    w.str(global_step);
    w.i64((int64_t)grads.size());
    for (auto& kv : grads) {
      w.str(kv.first);
      put_array(w, kv.second);
    }
    std::vector<uint8_t> r;
    call(read_back ? wire::APPLY_READ : wire::APPLY, w, &r);
    wire::Reader rd(r.data(), r.size());
    const int64_t step = rd.i64();
    py::list vals;
    if (read_back)
      for (size_t i = 0; i < grads.size(); ++i) vals.append(to_array(rd.tensor()));
    return py::make_tuple(step, vals);
  }

  std::vector<bool> is_init(const std::vector<std::string>& names) {
    wire::Writer w;
    w.i64((int64_t)names.size());
    for (auto& n : names) w.str(n);
    std::vector<uint8_t> r;
    call(wire::IS_INIT, w, &r);
    wire::Reader rd(r.data(), r.size());
    std::vector<bool> out;
    for (size_t i = 0; i < names.size(); ++i) out.push_back(rd.i64() != 0);
    return out;
  }

  py::list list() {
    wire::Writer w;
    std::vector<uint8_t> r;
    call(wire::LIST, w, &r);
    wire::Reader rd(r.data(), r.size());
    const int64_t n = rd.i64();
    py::list out;
    for (int64_t i = 0; i < n; ++i) {
      std::string name = rd.str();
      const int64_t dt = rd.i64();
      const int64_t nd = rd.i64();
      std::vector<int64_t> shape;
      for (int64_t k = 0; k < nd; ++k) shape.push_back(rd.i64());
      out.append(py::make_tuple(name, dt, shape));
    }
    return out;
  }

  void acc_create(const std::string& name, py::array tmpl, int64_t step) {
    wire::Writer w;
    w.str(name);
    put_array(w, tmpl);
    w.i64(step);
    std::vector<uint8_t> r;
    call(wire::ACC_CREATE, w, &r);
  }

  bool acc_apply(const std::string& name, int64_t local_step, py::array g) {
    wire::Writer w;
    w.str(name);
    w.i64(local_step);
    put_array(w, g);
    std::vector<uint8_t> r;
    call(wire::ACC_APPLY, w, &r);
    wire::Reader rd(r.data(), r.size());
    return rd.i64() != 0;
  }

  py::object acc_take(const std::string& name, int64_t num_required, double timeout) {
    wire::Writer w;
    w.str(name);
    w.i64(num_required);
    w.f64(timeout);
    std::vector<uint8_t> r;
    if (call(wire::ACC_TAKE, w, &r) != wire::OK) return py::none();
    wire::Reader rd(r.data(), r.size());
    return to_array(rd.tensor());
  }

  void acc_set_step(const std::string& name, int64_t step) {
    wire::Writer w;
    w.str(name);
    w.i64(step);
    std::vector<uint8_t> r;
    call(wire::ACC_SET_STEP, w, &r);
  }

  py::tuple acc_num(const std::string& name) {
    wire::Writer w;
    w.str(name);
    std::vector<uint8_t> r;
    call(wire::ACC_NUM, w, &r);
    wire::Reader rd(r.data(), r.size());
    const int64_t c = rd.i64();
    const int64_t d = rd.i64();
    return py::make_tuple(c, d);
  }

  void q_enqueue(const std::string& name, const std::vector<int64_t>& vals) {
    wire::Writer w;
    w.str(name);
    w.i64((int64_t)vals.size());
    for (auto v : vals) w.i64(v);
    std::vector<uint8_t> r;
    call(wire::Q_ENQ, w, &r);
  }

  py::object q_dequeue(const std::string& name, double timeout) {
    wire::Writer w;
    w.str(name);
    w.f64(timeout);
    std::vector<uint8_t> r;
    if (call(wire::Q_DEQ, w, &r) != wire::OK) return py::none();
    wire::Reader rd(r.data(), r.size());
    return py::int_(rd.i64());
  }

  int64_t q_size(const std::string& name) {
    wire::Writer w;
    w.str(name);
    std::vector<uint8_t> r;
    call(wire::Q_SIZE, w, &r);
    wire::Reader rd(r.data(), r.size());
    return rd.i64();
  }

  bool barrier(const std::string& name, int64_t count, double timeout) {
    wire::Writer w;
    w.str(name);
    w.i64(count);
    w.f64(timeout);
    std::vector<uint8_t> r;
    return call(wire::BARRIER, w, &r) == wire::OK;
  }

  int64_t worker_done(int64_t task) {
    wire::Writer w;
    w.i64(task);
    std::vector<uint8_t> r;
    call(wire::WORKER_DONE, w, &r);
    wire::Reader rd(r.data(), r.size());
    return rd.i64();
  }

  void shutdown() {
    wire::Writer w;
    std::vector<uint8_t> r;
    call(wire::SHUTDOWN, w, &r);
  }

  void watch(const std::string& queue, int64_t token) {
    wire::Writer w;
    w.str(queue);
    w.i64(token);
    std::vector<uint8_t> r;
    call(wire::WATCH, w, &r);
  }

  void unwatch() {
    wire::Writer w;
    std::vector<uint8_t> r;
    call(wire::UNWATCH, w, &r);
  }

  int64_t heartbeat(int64_t task) {
    wire::Writer w;
    w.i64(task);
    std::vector<uint8_t> r;
    call(wire::HEARTBEAT, w, &r);
    wire::Reader rd(r.data(), r.size());
    return rd.i64();
  }

  py::dict stats() {
    wire::Writer w;
    std::vector<uint8_t> r;
    call(wire::STATS, w, &r);
    wire::Reader rd(r.data(), r.size());
    py::dict d;
    d["requests"] = rd.i64();
    d["bytes_in"] = rd.i64();
    d["bytes_out"] = rd.i64();
    d["applies"] = rd.i64();
    return d;
  }

  void close() { c_->close(); }

 private:
  std::unique_ptr<ps::Client> c_;
};

}  // namespace

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "dtg native runtime: parameter-server service and TensorBundle checkpoint I/O";

  py::class_<ps::Server>(m, "PSServer")
      .def(py::init<const std::string&, int, int>(), py::arg("host") = "127.0.0.1", py::arg("port") = 0,
           py::arg("num_workers") = 0)
      .def("start", &ps::Server::start)
      .def("join", &ps::Server::join, py::arg("timeout") = -1.0, py::call_guard<py::gil_scoped_release>())
      .def("stop", &ps::Server::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &ps::Server::port)
      .def("stats", &ps::Server::stats)
      .def("list_vars", &ps::Server::list_vars)
      .def("read_var",
           [](ps::Server& s, const std::string& name) -> py::object {
             wire::Tensor t;
             if (!s.read_var(name, &t)) return py::none();
             return to_array(t);
           })
      .def("assign_var", [](ps::Server& s, const std::string& name, py::array a) {
        a = py::array::ensure(a, py::array::c_style);
        wire::Tensor t;
        t.dtype = np_to_wire(a.dtype());
        t.shape.assign(a.shape(), a.shape() + a.ndim());
        t.data.assign((const uint8_t*)a.data(), (const uint8_t*)a.data() + a.nbytes());
        s.assign_var(name, t);
      });

  py::class_<PyClient>(m, "PSClient")
      .def(py::init<const std::string&, int, double>(), py::arg("host"), py::arg("port"), py::arg("timeout") = 60.0)
      .def("ping", &PyClient::ping)
      .def("create", &PyClient::create, py::arg("name"), py::arg("init"), py::arg("overwrite") = false)
      .def("read", &PyClient::read)
      .def("assign", &PyClient::assign)
      .def("assign_add", &PyClient::assign_add)
      .def("apply", &PyClient::apply, py::arg("opt"), py::arg("hyper"), py::arg("locking"), py::arg("global_step"),
           py::arg("grads"), py::arg("read_back") = false)
      .def("is_init", &PyClient::is_init)
      .def("list", &PyClient::list)
      .def("acc_create", &PyClient::acc_create)
      .def("acc_apply", &PyClient::acc_apply)
      .def("acc_take", &PyClient::acc_take, py::arg("name"), py::arg("num_required"), py::arg("timeout") = -1.0)
      .def("acc_set_step", &PyClient::acc_set_step)
      .def("acc_num", &PyClient::acc_num)
      .def("q_enqueue", &PyClient::q_enqueue)
      .def("q_dequeue", &PyClient::q_dequeue, py::arg("name"), py::arg("timeout") = -1.0)
      .def("q_size", &PyClient::q_size)
      .def("barrier", &PyClient::barrier, py::arg("name"), py::arg("count"), py::arg("timeout") = -1.0)
      .def("worker_done", &PyClient::worker_done)
      .def("shutdown", &PyClient::shutdown)
      .def("heartbeat", &PyClient::heartbeat)
      .def("watch", &PyClient::watch, py::arg("queue"), py::arg("token"))
      .def("unwatch", &PyClient::unwatch)
      .def("stats", &PyClient::stats)
      .def("close", &PyClient::close);

  m.attr("SGD") = (int64_t)wire::SGD;
  m.attr("ADAGRAD") = (int64_t)wire::ADAGRAD;
  m.attr("MOMENTUM") = (int64_t)wire::MOMENTUM;
  m.attr("ADAM") = (int64_t)wire::ADAM;
  m.attr("RAW_ADD") = (int64_t)wire::RAW_ADD;

  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return ckpt::crc32c(s.data(), s.size());
  });
  m.def("crc_mask", &ckpt::crc_mask);
  m.def("write_bundle", [](const std::string& prefix, const std::vector<py::tuple>& items) {
    // items: (name, tf_dtype, shape, bytes)
    std::vector<ckpt::NamedTensor> ts;
    for (auto& it : items) {
      ckpt::NamedTensor t;
      t.name = it[0].cast<std::string>();
      t.dtype = it[1].cast<int>();
      t.shape = it[2].cast<std::vector<int64_t>>();
      t.bytes = it[3].cast<std::string>();
      ts.push_back(std::move(t));
    }
    py::gil_scoped_release nogil;
    ckpt::write_bundle(prefix, ts);
  });
  m.def("read_bundle", [](const std::string& prefix, bool verify) {
    std::vector<ckpt::NamedTensor> ts;
    {
      py::gil_scoped_release nogil;
      ts = ckpt::read_bundle(prefix, verify);
    }
    py::list out;
    for (auto& t : ts) out.append(py::make_tuple(t.name, t.dtype, t.shape, py::bytes(t.bytes)));
    return out;
  }, py::arg("prefix"), py::arg("verify") = true);
  m.def("read_index", [](const std::string& prefix) {
    auto idx = ckpt::read_index(prefix);
    py::dict d;
    for (auto& kv : idx)
      d[py::str(kv.first)] = py::make_tuple(kv.second.dtype, kv.second.shape, kv.second.offset, kv.second.size,
                                            kv.second.crc32c);
    return d;
  });
}
