// dtg parameter-server service: the native stand-in for the TF-1.x runtime services the
// reference exercises: gRPC Server + join (N1), variable resource store with
// assign / assign_add / is_initialized (N3, N8), ApplyGradientDescent / ApplyAdagrad (N4, N5),
// ConditionalAccumulator (N6), the SyncReplicas token FIFOQueue (N7), plus a named barrier
// (replaces the reference's rendezvous sleeps) and worker-done accounting so
// join() returns when training ends (the reference's PS never exits, README.md:55-59).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "dtg/wire.h"

namespace dtg {
namespace ps {

struct Variable {
  uint8_t dtype = wire::F32;
  std::vector<int64_t> shape;
  std::vector<uint8_t> data;  // 64-byte aligned storage is not required on the host path
  std::mutex mu;              // taken only for use_locking applies / assign_add
  bool initialized = false;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    return n;
  }
};

struct Accumulator {
  std::vector<int64_t> shape;
  std::vector<double> sum;
  int64_t count = 0;
  int64_t global_step = 0;
  int64_t dropped = 0;
  std::mutex mu;
  std::condition_variable cv;
};

struct TokenQueue {
  std::deque<int64_t> q;
  std::mutex mu;
  std::condition_variable cv;
};

struct Barrier {
  int64_t arrived = 0;
  int64_t generation = 0;
  std::mutex mu;
  std::condition_variable cv;
};

class Server {
 public:
  Server(const std::string& host, int port, int num_workers);
  ~Server();
  void start();
  // blocks until SHUTDOWN or every worker reported done; timeout_s < 0 = forever.
  // returns true if the server is finished.
  bool join(double timeout_s);
  void stop();
  int port() const { return port_; }
  std::map<std::string, int64_t> stats();

  // direct (in-process) access used by checkpointing on the PS task and by tests
  std::vector<std::string> list_vars();
  bool read_var(const std::string& name, wire::Tensor* out);
  void assign_var(const std::string& name, const wire::Tensor& t);

 private:
  void accept_loop();
  void serve(int fd);
  int32_t dispatch(uint16_t op, wire::Reader& rd, wire::Writer& wr);
  std::shared_ptr<Variable> get_var(const std::string& name);
  std::shared_ptr<Variable> get_or_create_slot(const std::shared_ptr<Variable>& base, const std::string& name,
                                               float init);
  std::shared_ptr<Accumulator> get_acc(const std::string& name, bool create);
  std::shared_ptr<TokenQueue> get_q(const std::string& name);
  std::shared_ptr<Barrier> get_barrier(const std::string& name);
  int64_t apply(int64_t opt, const double* hyper, bool locking, const std::string& gstep, wire::Reader& rd,
                std::vector<std::string>* names);

  std::string host_;
  int port_;
  int num_workers_;
  int listen_fd_ = -1;
  std::atomic<bool> stopping_{false};
  std::thread acceptor_;
  std::vector<std::thread> conns_;
  std::vector<int> conn_fds_;
  std::mutex conns_mu_;

  std::shared_mutex vars_mu_;
  std::map<std::string, std::shared_ptr<Variable>> vars_;
  std::mutex misc_mu_;
  std::map<std::string, std::shared_ptr<Accumulator>> accs_;
  std::map<std::string, std::shared_ptr<TokenQueue>> queues_;
  std::map<std::string, std::shared_ptr<Barrier>> barriers_;

  std::mutex done_mu_;
  std::condition_variable done_cv_;
  std::vector<bool> worker_done_;
  int64_t done_count_ = 0;
  bool shutdown_ = false;

  std::atomic<int64_t> n_requests_{0}, bytes_in_{0}, bytes_out_{0}, n_applies_{0};
  int64_t n_lost_ = 0;  // worker tasks whose watched connection dropped before they reported done
};

class Client {
 public:
  Client(const std::string& host, int port, double connect_timeout_s);
  ~Client();
  // returns status; fills response body
  int32_t call(uint16_t op, const std::vector<uint8_t>& body, std::vector<uint8_t>* resp);
  void close();

 private:
  int fd_ = -1;
  std::mutex mu_;
};

}  // namespace ps
}  // namespace dtg
