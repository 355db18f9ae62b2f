// Wire format of dtg's parameter-server control/data channel (TCP).
//
// Replaces the TF-1.x gRPC master/worker services the reference relies on (SURVEY §2.4, §2.5
// N1): a request is a fixed header followed by a body of typed fields; the response carries a
// status and a body.  Fields are little-endian and written back to back:
//   str  : u32 len, bytes
//   i64  : 8 bytes          f64 : 8 bytes
//   tensor: u8 dtype, u8 ndim, i64 dims[ndim], u64 nbytes, bytes
#pragma once
#include <stdint.h>
#include <string.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace dtg {
namespace wire {

constexpr uint32_t kMagic = 0x50475444;  // "DTGP"

enum Op : uint16_t {
  PING = 0,
  CREATE = 1,        // name, tensor(init), i64 overwrite -> i64 created
  READ = 2,          // n, names... -> n tensors
  ASSIGN = 3,        // n, (name, tensor)...
  ASSIGN_ADD = 4,    // name, tensor -> tensor(new value)
  APPLY = 5,         // i64 opt, f64 hyper[5], i64 locking, str global_step ("" = none), n, (name, grad)... -> i64 step
  IS_INIT = 6,       // n, names -> n x i64
  LIST = 7,          // -> n, (name, dtype, shape)
  ACC_CREATE = 8,    // name, tensor template (dtype/shape), i64 initial global step
  ACC_APPLY = 9,     // name, i64 local_step, tensor grad -> i64 accepted
  ACC_TAKE = 10,     // name, i64 num_required, f64 timeout_s -> tensor mean
  ACC_SET_STEP = 11, // name, i64 step
  Q_ENQ = 12,        // name, n, i64 values...
  Q_DEQ = 13,        // name, f64 timeout_s -> i64 value (status 2 on timeout)
  BARRIER = 14,      // name, i64 count, f64 timeout_s
  WORKER_DONE = 15,  // i64 task
  SHUTDOWN = 16,
  APPLY_READ = 17,   // APPLY then READ the same names (fused push+pull round trip)
  ACC_NUM = 18,      // name -> i64 num accumulated
  STATS = 19,        // -> i64 requests, i64 bytes_in, i64 bytes_out, i64 applies
  HEARTBEAT = 20,    // i64 task -> i64 server time ms
  Q_SIZE = 21,       // name -> i64
  WATCH = 40,        // name, i64 token: if THIS connection closes before UNWATCH, enqueue token on queue name
  UNWATCH = 41,      // clears this connection's watch
};

enum DType : uint8_t { F32 = 1, F64 = 2, I32 = 3, I64 = 9, BF16 = 14 };

inline size_t dtype_size(uint8_t dt) {
  switch (dt) {
    case F32: case I32: return 4;
    case F64: case I64: return 8;
    case BF16: return 2;
    default: throw std::runtime_error("bad dtype");
  }
}

enum Status : int32_t { OK = 0, ERR = 1, TIMEOUT = 2, NOT_FOUND = 3, CLOSED = 4 };

enum OptKind : int64_t { SGD = 0, ADAGRAD = 1, MOMENTUM = 2, ADAM = 3, RAW_ADD = 4 };

#pragma pack(push, 1)
struct ReqHdr {
  uint32_t magic;
  uint16_t op;
  uint16_t flags;
  uint64_t body_len;
};
struct RespHdr {
  uint32_t magic;
  int32_t status;
  uint64_t body_len;
};
#pragma pack(pop)

struct Tensor {
  uint8_t dtype = F32;
  std::vector<int64_t> shape;
  std::vector<uint8_t> data;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    return n;
  }
};

class Writer {
 public:
  std::vector<uint8_t> buf;
  void raw(const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    buf.insert(buf.end(), b, b + n);
  }
  void i64(int64_t v) { raw(&v, 8); }
  void f64(double v) { raw(&v, 8); }
  void str(const std::string& s) {
    uint32_t n = (uint32_t)s.size();
    raw(&n, 4);
    raw(s.data(), n);
  }
  void tensor(uint8_t dt, const std::vector<int64_t>& shape, const void* data, uint64_t nbytes) {
    raw(&dt, 1);
    uint8_t nd = (uint8_t)shape.size();
    raw(&nd, 1);
    for (auto d : shape) i64(d);
    raw(&nbytes, 8);
    raw(data, nbytes);
  }
  void tensor(const Tensor& t) { tensor(t.dtype, t.shape, t.data.data(), t.data.size()); }
};

class Reader {
 public:
  Reader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  // off_ <= n_ always holds, so n_ - off_ cannot wrap; off_ + k could for a hostile k
  void need(size_t k) {
    if (k > n_ - off_) throw std::runtime_error("wire: truncated message");
  }
  void raw(void* dst, size_t k) {
    need(k);
    memcpy(dst, p_ + off_, k);
    off_ += k;
  }
  int64_t i64() { int64_t v; raw(&v, 8); return v; }
  double f64() { double v; raw(&v, 8); return v; }
  std::string str() {
    uint32_t k;
    raw(&k, 4);
    need(k);
    std::string s((const char*)p_ + off_, k);
    off_ += k;
    return s;
  }
  Tensor tensor() {
    Tensor t;
    raw(&t.dtype, 1);
    uint8_t nd;
    raw(&nd, 1);
    t.shape.resize(nd);
    // validate before anything dereferences the payload: every dim non-negative, numel bounded (no
    // overflow in numel * dtype_size), and the byte count exactly numel * dtype_size
    constexpr int64_t kMaxNumel = (int64_t)1 << 40;
    int64_t numel = 1;
    for (int i = 0; i < nd; ++i) {
      t.shape[i] = i64();
      if (t.shape[i] < 0 || (t.shape[i] > 0 && numel > kMaxNumel / t.shape[i]))
        throw std::runtime_error("wire: bad tensor shape");
      numel *= t.shape[i];
    }
    uint64_t nb;
    raw(&nb, 8);
    if (nb != (uint64_t)numel * dtype_size(t.dtype)) throw std::runtime_error("wire: tensor byte count mismatch");
    need(nb);
    t.data.assign(p_ + off_, p_ + off_ + nb);
    off_ += nb;
    return t;
  }
  bool done() const { return off_ >= n_; }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t off_ = 0;
};

// blocking full send/recv helpers (return false on EOF / error)
bool send_all(int fd, const void* p, size_t n);
bool recv_all(int fd, void* p, size_t n);

}  // namespace wire
}  // namespace dtg
