// dtg parameter-server service (see dtg/ps.h).  One thread per connection: blocking ops
// (accumulator take, token dequeue, barrier) park only their own connection, which is exactly the
// semantics of the TF queue/accumulator ops they replace.
//
// Hogwild (Hogwild/README.md:3, TF use_locking=False default): unlocked applies read and write
// each element with relaxed atomic 32-bit accesses -- concurrent workers may lose updates (the
// algorithm's intended race) but there is no undefined behaviour and TSan stays clean.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstring>
#include <iostream>

#include "dtg/ps.h"

namespace dtg {
namespace wire {

bool send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

}  // namespace wire

namespace ps {
using namespace wire;

namespace {

inline float ld_relaxed(const float* p) {
  uint32_t u = __atomic_load_n(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED);
  float f;
  memcpy(&f, &u, 4);
  return f;
}
inline void st_relaxed(float* p, float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  __atomic_store_n(reinterpret_cast<uint32_t*>(p), u, __ATOMIC_RELAXED);
}

template <class F>
void for_each_locked(Variable& v, bool locking, F f) {
  if (locking) {
    std::lock_guard<std::mutex> g(v.mu);
    f();
  } else {
    f();
  }
}

void add_into(Variable& v, const Tensor& t) {
  const int64_t n = v.numel();
  if ((int64_t)t.data.size() != n * (int64_t)dtype_size(v.dtype) || t.dtype != v.dtype)
    throw std::runtime_error("assign_add: shape/dtype mismatch");
  switch (v.dtype) {
    case F32: {
      float* d = (float*)v.data.data();
      const float* s = (const float*)t.data.data();
      for (int64_t i = 0; i < n; ++i) d[i] += s[i];
      break;
    }
    case F64: {
      double* d = (double*)v.data.data();
      const double* s = (const double*)t.data.data();
      for (int64_t i = 0; i < n; ++i) d[i] += s[i];
      break;
    }
    case I32: {
      int32_t* d = (int32_t*)v.data.data();
      const int32_t* s = (const int32_t*)t.data.data();
      for (int64_t i = 0; i < n; ++i) d[i] += s[i];
      break;
    }
    case I64: {
      int64_t* d = (int64_t*)v.data.data();
      const int64_t* s = (const int64_t*)t.data.data();
      for (int64_t i = 0; i < n; ++i) d[i] += s[i];
      break;
    }
    default:
      throw std::runtime_error("assign_add: unsupported dtype");
  }
}

int64_t scalar_i64(const Variable& v) {
  if (v.dtype == I64) return *(const int64_t*)v.data.data();
  if (v.dtype == I32) return *(const int32_t*)v.data.data();
  if (v.dtype == F32) return (int64_t)*(const float*)v.data.data();
  return (int64_t)*(const double*)v.data.data();
}

void set_timeout(int fd, double s) {
  struct timeval tv;
  tv.tv_sec = (time_t)s;
  tv.tv_usec = (suseconds_t)((s - (double)tv.tv_sec) * 1e6);
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
}

}  // namespace

Server::Server(const std::string& host, int port, int num_workers)
    : host_(host), port_(port), num_workers_(num_workers), worker_done_(num_workers > 0 ? num_workers : 0, false) {}

Server::~Server() { stop(); }

void Server::start() {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("ps: socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port_);
  // all interfaces only when asked for explicitly ("0.0.0.0" / "*": a multi-host ClusterSpec); an
  // unspecified host binds the loopback interface -- the service has no authentication
  if (host_ == "0.0.0.0" || host_ == "*") {
    a.sin_addr.s_addr = htonl(INADDR_ANY);
  } else {
    std::string h = (host_.empty() || host_ == "localhost") ? "127.0.0.1" : host_;
    if (inet_pton(AF_INET, h.c_str(), &a.sin_addr) != 1) {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      if (getaddrinfo(h.c_str(), nullptr, &hints, &res) != 0 || !res)
        throw std::runtime_error("ps: cannot resolve host " + h);
      a.sin_addr = ((sockaddr_in*)res->ai_addr)->sin_addr;
      freeaddrinfo(res);
    }
  }
  if (::bind(listen_fd_, (sockaddr*)&a, sizeof(a)) != 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
    throw std::runtime_error("ps: bind() failed on port " + std::to_string(port_) + ": " + strerror(errno));
  }
  socklen_t len = sizeof(a);
  getsockname(listen_fd_, (sockaddr*)&a, &len);
  port_ = ntohs(a.sin_port);
  if (::listen(listen_fd_, 128) != 0) throw std::runtime_error("ps: listen() failed");
  acceptor_ = std::thread([this] { accept_loop(); });
}

void Server::accept_loop() {
  while (!stopping_.load()) {
    sockaddr_in ca{};
    socklen_t cl = sizeof(ca);
    int fd = ::accept(listen_fd_, (sockaddr*)&ca, &cl);
    if (fd < 0) {
      if (stopping_.load()) break;
      if (errno == EINTR || errno == ECONNABORTED) continue;
      break;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::lock_guard<std::mutex> g(conns_mu_);
    conn_fds_.push_back(fd);
    conns_.emplace_back([this, fd] { serve(fd); });
  }
}

void Server::serve(int fd) {
  std::vector<uint8_t> body;
  // connection watch (failure detection): a client registers (queue, token); if its connection ends
  // without UNWATCH -- the process died or dropped off the network -- the token is enqueued, so a
  // consumer blocked on that queue learns about the loss instead of waiting out a timeout
  bool watching = false;
  std::string watch_q;
  int64_t watch_tok = 0;
  bool clean = false;
  while (!stopping_.load()) {
    ReqHdr h;
    if (!recv_all(fd, &h, sizeof(h))) break;
    if (h.magic != kMagic) break;
    body.resize(h.body_len);
    if (h.body_len && !recv_all(fd, body.data(), h.body_len)) break;
    n_requests_++;
    bytes_in_ += (int64_t)(sizeof(h) + h.body_len);
    Writer wr;
    int32_t st = OK;
    try {
      Reader rd(body.data(), body.size());
      if (h.op == WATCH) {
        watch_q = rd.str();
        watch_tok = rd.i64();
        watching = true;
      } else if (h.op == UNWATCH) {
        watching = false;
      } else {
        st = dispatch(h.op, rd, wr);
      }
    } catch (const std::exception& e) {
      st = ERR;
      wr.buf.clear();
      wr.str(e.what());
    }
    RespHdr r{kMagic, st, (uint64_t)wr.buf.size()};
    if (!send_all(fd, &r, sizeof(r))) break;
    if (!wr.buf.empty() && !send_all(fd, wr.buf.data(), wr.buf.size())) break;
    bytes_out_ += (int64_t)(sizeof(r) + wr.buf.size());
    if (h.op == SHUTDOWN) {
      clean = true;
      break;
    }
  }
  ::shutdown(fd, SHUT_RDWR);
  if (watching && !clean && !stopping_.load() && watch_q == "__worker__") {
    // a worker task's process is gone: count it as finished so join() does not wait for it forever
    std::lock_guard<std::mutex> lk(done_mu_);
    if (watch_tok >= 0 && watch_tok < (int64_t)worker_done_.size() && !worker_done_[watch_tok]) {
      worker_done_[watch_tok] = true;
      done_count_++;
      n_lost_++;
    }
    done_cv_.notify_all();
  } else if (watching && !clean && !stopping_.load()) {
    auto q = get_q(watch_q);
    std::lock_guard<std::mutex> lk(q->mu);
    q->q.push_back(watch_tok);
    q->cv.notify_all();
  }
}

std::shared_ptr<Variable> Server::get_var(const std::string& name) {
  std::shared_lock<std::shared_mutex> g(vars_mu_);
  auto it = vars_.find(name);
  if (it == vars_.end()) throw std::runtime_error("ps: no variable '" + name + "'");
  return it->second;
}

std::shared_ptr<Variable> Server::get_or_create_slot(const std::shared_ptr<Variable>& base, const std::string& name,
                                                     float init) {
  {
    std::shared_lock<std::shared_mutex> g(vars_mu_);
    auto it = vars_.find(name);
    if (it != vars_.end()) return it->second;
  }
  std::unique_lock<std::shared_mutex> g(vars_mu_);
  auto it = vars_.find(name);
  if (it != vars_.end()) return it->second;
  auto v = std::make_shared<Variable>();
  v->dtype = F32;
  v->shape = base->shape;
  v->data.resize((size_t)base->numel() * 4);
  float* d = (float*)v->data.data();
  for (int64_t i = 0; i < base->numel(); ++i) d[i] = init;
  v->initialized = true;
  vars_[name] = v;
  return v;
}

std::shared_ptr<Accumulator> Server::get_acc(const std::string& name, bool create) {
  std::lock_guard<std::mutex> g(misc_mu_);
  auto it = accs_.find(name);
  if (it != accs_.end()) return it->second;
  if (!create) throw std::runtime_error("ps: no accumulator '" + name + "'");
  auto a = std::make_shared<Accumulator>();
  accs_[name] = a;
  return a;
}

std::shared_ptr<TokenQueue> Server::get_q(const std::string& name) {
  std::lock_guard<std::mutex> g(misc_mu_);
  auto& q = queues_[name];
  if (!q) q = std::make_shared<TokenQueue>();
  return q;
}

std::shared_ptr<Barrier> Server::get_barrier(const std::string& name) {
  std::lock_guard<std::mutex> g(misc_mu_);
  auto& b = barriers_[name];
  if (!b) b = std::make_shared<Barrier>();
  return b;
}

// Applies gradients for n variables; returns the incremented global step (or -1).
// hyper: [lr, p1, p2, p3, t]  SGD: -, ADAGRAD: p1 = initial accumulator,
// MOMENTUM: p1 = momentum, ADAM: p1=b1 p2=b2 p3=eps t=step, RAW_ADD: w += lr*g
int64_t Server::apply(int64_t opt, const double* hyper, bool locking, const std::string& gstep, Reader& rd,
                      std::vector<std::string>* names) {
  const int64_t n = rd.i64();
  const float lr = (float)hyper[0];
  for (int64_t k = 0; k < n; ++k) {
    const std::string name = rd.str();
    Tensor g = rd.tensor();
    if (names) names->push_back(name);
    auto v = get_var(name);
    if (v->dtype != F32 || g.dtype != F32 || g.numel() != v->numel() || g.data.size() != v->data.size())
      throw std::runtime_error("apply: '" + name + "' needs matching float32 gradient");
    float* w = (float*)v->data.data();
    const float* gr = (const float*)g.data.data();
    const int64_t m = v->numel();
    switch (opt) {
      case SGD:
      case RAW_ADD: {
        const float s = opt == SGD ? -lr : lr;
        for_each_locked(*v, locking, [&] {
          for (int64_t i = 0; i < m; ++i) st_relaxed(w + i, ld_relaxed(w + i) + s * gr[i]);
        });
        break;
      }
      case ADAGRAD: {
        auto acc = get_or_create_slot(v, name + "/Adagrad", (float)hyper[1]);
        float* a = (float*)acc->data.data();
        for_each_locked(*v, locking, [&] {
          for (int64_t i = 0; i < m; ++i) {
            const float an = ld_relaxed(a + i) + gr[i] * gr[i];
            st_relaxed(a + i, an);
            st_relaxed(w + i, ld_relaxed(w + i) - lr * gr[i] / std::sqrt(an));
          }
        });
        break;
      }
      case MOMENTUM: {
        auto acc = get_or_create_slot(v, name + "/Momentum", 0.f);
        float* a = (float*)acc->data.data();
        const float mu = (float)hyper[1];
        for_each_locked(*v, locking, [&] {
          for (int64_t i = 0; i < m; ++i) {
            const float an = mu * ld_relaxed(a + i) + gr[i];
            st_relaxed(a + i, an);
            st_relaxed(w + i, ld_relaxed(w + i) - lr * an);
          }
        });
        break;
      }
      case ADAM: {
        auto m1 = get_or_create_slot(v, name + "/Adam", 0.f);
        auto m2 = get_or_create_slot(v, name + "/Adam_1", 0.f);
        float* a = (float*)m1->data.data();
        float* b = (float*)m2->data.data();
        const float b1 = (float)hyper[1], b2 = (float)hyper[2], eps = (float)hyper[3];
        const double t = hyper[4] < 1 ? 1 : hyper[4];
        const float lrt = (float)(lr * std::sqrt(1 - std::pow((double)b2, t)) / (1 - std::pow((double)b1, t)));
        for_each_locked(*v, locking, [&] {
          for (int64_t i = 0; i < m; ++i) {
            const float an = b1 * ld_relaxed(a + i) + (1 - b1) * gr[i];
            const float bn = b2 * ld_relaxed(b + i) + (1 - b2) * gr[i] * gr[i];
            st_relaxed(a + i, an);
            st_relaxed(b + i, bn);
            st_relaxed(w + i, ld_relaxed(w + i) - lrt * an / (std::sqrt(bn) + eps));
          }
        });
        break;
      }
      default:
        throw std::runtime_error("apply: unknown optimizer");
    }
    n_applies_++;
  }
  if (gstep.empty()) return -1;
  auto gs = get_var(gstep);
  std::lock_guard<std::mutex> g(gs->mu);
  if (gs->dtype == I64) return ++*(int64_t*)gs->data.data();
  if (gs->dtype == I32) return ++*(int32_t*)gs->data.data();
  throw std::runtime_error("global_step must be an integer variable");
}

int32_t Server::dispatch(uint16_t op, Reader& rd, Writer& wr) {
  switch (op) {
    case PING:
      wr.i64(1);
      return OK;
    case CREATE: {
      const std::string name = rd.str();
      Tensor t = rd.tensor();
      const bool overwrite = rd.i64() != 0;
      std::unique_lock<std::shared_mutex> g(vars_mu_);
      auto it = vars_.find(name);
      if (it != vars_.end() && !overwrite) {
        wr.i64(0);
        return OK;
      }
      auto v = std::make_shared<Variable>();
      v->dtype = t.dtype;
      v->shape = t.shape;
      v->data = std::move(t.data);
      v->initialized = true;
      vars_[name] = v;
      wr.i64(1);
      return OK;
    }
    case READ: {
      const int64_t n = rd.i64();
      for (int64_t k = 0; k < n; ++k) {
        auto v = get_var(rd.str());
        // unlocked read: a concurrent Hogwild apply may be mid-update (TF reads are racy too)
        std::vector<uint8_t> snap(v->data.size());
        const uint32_t* s = (const uint32_t*)v->data.data();
        uint32_t* d = (uint32_t*)snap.data();
        const size_t nw = v->data.size() / 4;
        for (size_t i = 0; i < nw; ++i) d[i] = __atomic_load_n(s + i, __ATOMIC_RELAXED);
        for (size_t i = nw * 4; i < v->data.size(); ++i) snap[i] = v->data[i];
        wr.tensor(v->dtype, v->shape, snap.data(), snap.size());
      }
      return OK;
    }
    case ASSIGN: {
      const int64_t n = rd.i64();
      for (int64_t k = 0; k < n; ++k) {
        const std::string name = rd.str();
        Tensor t = rd.tensor();
        auto v = get_var(name);
        if (t.data.size() != v->data.size() || t.dtype != v->dtype)
          throw std::runtime_error("assign: size/dtype mismatch for " + name);
        std::lock_guard<std::mutex> g(v->mu);
        uint32_t* d = (uint32_t*)v->data.data();
        const uint32_t* s = (const uint32_t*)t.data.data();
        const size_t nw = t.data.size() / 4;
        for (size_t i = 0; i < nw; ++i) __atomic_store_n(d + i, s[i], __ATOMIC_RELAXED);
        for (size_t i = nw * 4; i < t.data.size(); ++i) v->data[i] = t.data[i];
        v->initialized = true;
      }
      return OK;
    }
    case ASSIGN_ADD: {
      const std::string name = rd.str();
      Tensor t = rd.tensor();
      auto v = get_var(name);
      std::lock_guard<std::mutex> g(v->mu);
      add_into(*v, t);
      wr.tensor(v->dtype, v->shape, v->data.data(), v->data.size());
      return OK;
    }
    case APPLY:
    case APPLY_READ: {
      const int64_t opt = rd.i64();
      double hyper[5];
      for (double& h : hyper) h = rd.f64();
      const bool locking = rd.i64() != 0;
      const std::string gstep = rd.str();
      std::vector<std::string> names;
      const int64_t step = apply(opt, hyper, locking, gstep, rd, &names);
      wr.i64(step);
      if (op == APPLY_READ) {
        for (auto& nm : names) {
          auto v = get_var(nm);
          std::vector<uint8_t> snap(v->data.size());
          const uint32_t* s = (const uint32_t*)v->data.data();
          uint32_t* d = (uint32_t*)snap.data();
          for (size_t i = 0; i < snap.size() / 4; ++i) d[i] = __atomic_load_n(s + i, __ATOMIC_RELAXED);
          wr.tensor(v->dtype, v->shape, snap.data(), snap.size());
        }
      }
      return OK;
    }
    case IS_INIT: {
      const int64_t n = rd.i64();
      std::shared_lock<std::shared_mutex> g(vars_mu_);
      for (int64_t k = 0; k < n; ++k) {
        auto it = vars_.find(rd.str());
        wr.i64(it != vars_.end() && it->second->initialized ? 1 : 0);
      }
      return OK;
    }
    case LIST: {
      std::shared_lock<std::shared_mutex> g(vars_mu_);
      wr.i64((int64_t)vars_.size());
      for (auto& kv : vars_) {
        wr.str(kv.first);
        wr.i64(kv.second->dtype);
        wr.i64((int64_t)kv.second->shape.size());
        for (auto d : kv.second->shape) wr.i64(d);
      }
      return OK;
    }
    case ACC_CREATE: {
      const std::string name = rd.str();
      Tensor tmpl = rd.tensor();
      const int64_t step = rd.i64();
      auto a = get_acc(name, true);
      std::lock_guard<std::mutex> g(a->mu);
      if (a->sum.empty()) {
        a->shape = tmpl.shape;
        a->sum.assign((size_t)tmpl.numel(), 0.0);
        a->global_step = step;
      }
      return OK;
    }
    case ACC_APPLY: {
      const std::string name = rd.str();
      const int64_t local_step = rd.i64();
      Tensor g = rd.tensor();
      auto a = get_acc(name, false);
      std::lock_guard<std::mutex> lk(a->mu);
      if (g.dtype != F32 || (size_t)g.numel() != a->sum.size() || g.data.size() != a->sum.size() * 4)
        throw std::runtime_error("acc_apply: shape mismatch");
      if (local_step < a->global_step) {  // stale gradient: dropped (ConditionalAccumulator)
        a->dropped++;
        wr.i64(0);
        return OK;
      }
      const float* s = (const float*)g.data.data();
      for (size_t i = 0; i < a->sum.size(); ++i) a->sum[i] += s[i];
      a->count++;
      a->cv.notify_all();
      wr.i64(1);
      return OK;
    }
    case ACC_TAKE: {
      const std::string name = rd.str();
      const int64_t need = rd.i64();
      const double to = rd.f64();
      auto a = get_acc(name, false);
      std::unique_lock<std::mutex> lk(a->mu);
      auto pred = [&] { return a->count >= need || stopping_.load(); };
      if (to < 0) a->cv.wait(lk, pred);
      else if (!a->cv.wait_for(lk, std::chrono::duration<double>(to), pred)) return TIMEOUT;
      if (stopping_.load() && a->count < need) return CLOSED;
      std::vector<float> mean(a->sum.size());
      const double inv = a->count ? 1.0 / (double)a->count : 0.0;
      for (size_t i = 0; i < mean.size(); ++i) mean[i] = (float)(a->sum[i] * inv);
      std::fill(a->sum.begin(), a->sum.end(), 0.0);
      a->count = 0;
      wr.tensor(F32, a->shape, mean.data(), mean.size() * 4);
      return OK;
    }
    case ACC_SET_STEP: {
      const std::string name = rd.str();
      const int64_t step = rd.i64();
      auto a = get_acc(name, false);
      std::lock_guard<std::mutex> lk(a->mu);
      if (step > a->global_step) a->global_step = step;
      return OK;
    }
    case ACC_NUM: {
      auto a = get_acc(rd.str(), false);
      std::lock_guard<std::mutex> lk(a->mu);
      wr.i64(a->count);
      wr.i64(a->dropped);
      return OK;
    }
    case Q_ENQ: {
      auto q = get_q(rd.str());
      const int64_t n = rd.i64();
      std::lock_guard<std::mutex> lk(q->mu);
      for (int64_t k = 0; k < n; ++k) q->q.push_back(rd.i64());
      q->cv.notify_all();
      return OK;
    }
    case Q_DEQ: {
      auto q = get_q(rd.str());
      const double to = rd.f64();
      std::unique_lock<std::mutex> lk(q->mu);
      auto pred = [&] { return !q->q.empty() || stopping_.load(); };
      if (to < 0) q->cv.wait(lk, pred);
      else if (!q->cv.wait_for(lk, std::chrono::duration<double>(to), pred)) return TIMEOUT;
      if (q->q.empty()) return CLOSED;
      wr.i64(q->q.front());
      q->q.pop_front();
      return OK;
    }
    case Q_SIZE: {
      auto q = get_q(rd.str());
      std::lock_guard<std::mutex> lk(q->mu);
      wr.i64((int64_t)q->q.size());
      return OK;
    }
    case BARRIER: {
      auto b = get_barrier(rd.str());
      const int64_t count = rd.i64();
      const double to = rd.f64();
      std::unique_lock<std::mutex> lk(b->mu);
      const int64_t gen = b->generation;
      if (++b->arrived >= count) {
        b->arrived = 0;
        b->generation++;
        b->cv.notify_all();
        return OK;
      }
      auto pred = [&] { return b->generation != gen || stopping_.load(); };
      if (to < 0) b->cv.wait(lk, pred);
      else if (!b->cv.wait_for(lk, std::chrono::duration<double>(to), pred)) {
        b->arrived--;
        return TIMEOUT;
      }
      return b->generation != gen ? OK : CLOSED;
    }
    case WORKER_DONE: {
      const int64_t task = rd.i64();
      std::lock_guard<std::mutex> lk(done_mu_);
      if (task >= 0 && task < (int64_t)worker_done_.size() && !worker_done_[task]) {
        worker_done_[task] = true;
        done_count_++;
      }
      done_cv_.notify_all();
      wr.i64(done_count_);
      return OK;
    }
    case SHUTDOWN: {
      std::lock_guard<std::mutex> lk(done_mu_);
      shutdown_ = true;
      done_cv_.notify_all();
      return OK;
    }
    case STATS: {
      wr.i64(n_requests_.load());
      wr.i64(bytes_in_.load());
      wr.i64(bytes_out_.load());
      wr.i64(n_applies_.load());
      return OK;
    }
    case HEARTBEAT: {
      (void)rd.i64();
      wr.i64((int64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
                 std::chrono::steady_clock::now().time_since_epoch())
                 .count());
      return OK;
    }
    default:
      throw std::runtime_error("ps: unknown op " + std::to_string(op));
  }
}

bool Server::join(double timeout_s) {
  std::unique_lock<std::mutex> lk(done_mu_);
  auto pred = [&] {
    return shutdown_ || (num_workers_ > 0 && done_count_ >= num_workers_);
  };
  if (timeout_s < 0) {
    done_cv_.wait(lk, pred);
    return true;
  }
  return done_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred);
}

void Server::stop() {
  if (stopping_.exchange(true)) return;
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
    ::close(listen_fd_);
  }
  if (acceptor_.joinable()) acceptor_.join();
  // wake every blocked op so connection threads can exit
  {
    std::lock_guard<std::mutex> g(misc_mu_);
    for (auto& kv : accs_) { std::lock_guard<std::mutex> l(kv.second->mu); kv.second->cv.notify_all(); }
    for (auto& kv : queues_) { std::lock_guard<std::mutex> l(kv.second->mu); kv.second->cv.notify_all(); }
    for (auto& kv : barriers_) { std::lock_guard<std::mutex> l(kv.second->mu); kv.second->cv.notify_all(); }
  }
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : conns_)
    if (t.joinable()) t.join();
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (int fd : conn_fds_) ::close(fd);
    conn_fds_.clear();
  }
  {
    std::lock_guard<std::mutex> lk(done_mu_);
    shutdown_ = true;
    done_cv_.notify_all();
  }
}

std::map<std::string, int64_t> Server::stats() {
  int64_t lost;
  {
    std::lock_guard<std::mutex> lk(done_mu_);
    lost = n_lost_;
  }
  return {{"requests", n_requests_.load()},
          {"workers_lost", lost},
          {"bytes_in", bytes_in_.load()},
          {"bytes_out", bytes_out_.load()},
          {"applies", n_applies_.load()}};
}

std::vector<std::string> Server::list_vars() {
  std::shared_lock<std::shared_mutex> g(vars_mu_);
  std::vector<std::string> out;
  for (auto& kv : vars_) out.push_back(kv.first);
  return out;
}

bool Server::read_var(const std::string& name, Tensor* out) {
  std::shared_ptr<Variable> v;
  {
    std::shared_lock<std::shared_mutex> g(vars_mu_);
    auto it = vars_.find(name);
    if (it == vars_.end()) return false;
    v = it->second;
  }
  out->dtype = v->dtype;
  out->shape = v->shape;
  out->data.resize(v->data.size());
  const uint32_t* s = (const uint32_t*)v->data.data();
  uint32_t* d = (uint32_t*)out->data.data();
  for (size_t i = 0; i < out->data.size() / 4; ++i) d[i] = __atomic_load_n(s + i, __ATOMIC_RELAXED);
  for (size_t i = out->data.size() / 4 * 4; i < out->data.size(); ++i) out->data[i] = v->data[i];
  return true;
}

void Server::assign_var(const std::string& name, const Tensor& t) {
  std::unique_lock<std::shared_mutex> g(vars_mu_);
  auto v = std::make_shared<Variable>();
  v->dtype = t.dtype;
  v->shape = t.shape;
  v->data = t.data;
  v->initialized = true;
  vars_[name] = v;
}

// ---------------------------------------------------------------------------------------------
Client::Client(const std::string& host, int port, double connect_timeout_s) {
  std::string h = host == "localhost" ? "127.0.0.1" : host;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, h.c_str(), &a.sin_addr) != 1) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(h.c_str(), nullptr, &hints, &res) != 0 || !res)
      throw std::runtime_error("ps client: cannot resolve " + h);
    a.sin_addr = ((sockaddr_in*)res->ai_addr)->sin_addr;
    freeaddrinfo(res);
  }
  // retry with backoff until the server is up (replaces the reference's startup sleeps)
  auto t0 = std::chrono::steady_clock::now();
  double backoff = 0.01;
  while (true) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd_, (sockaddr*)&a, sizeof(a)) == 0) break;
    ::close(fd_);
    fd_ = -1;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > connect_timeout_s)
      throw std::runtime_error("ps client: cannot connect to " + h + ":" + std::to_string(port));
    std::this_thread::sleep_for(std::chrono::duration<double>(backoff));
    backoff = std::min(backoff * 2, 0.5);
  }
  int one = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  (void)set_timeout;
}

Client::~Client() { close(); }

void Client::close() {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ >= 0) {
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    fd_ = -1;
  }
}

int32_t Client::call(uint16_t op, const std::vector<uint8_t>& body, std::vector<uint8_t>* resp) {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ < 0) throw std::runtime_error("ps client: closed");
  ReqHdr h{kMagic, op, 0, (uint64_t)body.size()};
  if (!send_all(fd_, &h, sizeof(h)) || (!body.empty() && !send_all(fd_, body.data(), body.size())))
    throw std::runtime_error("ps client: send failed (server gone?)");
  RespHdr r;
  if (!recv_all(fd_, &r, sizeof(r)) || r.magic != kMagic) throw std::runtime_error("ps client: connection lost");
  resp->resize(r.body_len);
  if (r.body_len && !recv_all(fd_, resp->data(), r.body_len)) throw std::runtime_error("ps client: truncated reply");
  return r.status;
}

}  // namespace ps
}  // namespace dtg
