// Concurrency stress test of the native PS service (csrc/ps/server.cc), built by
// tools/build_sanitizers.sh with -fsanitize=thread and -fsanitize=address (host code only; SURVEY
// §5.2 "Build the C++ PS with -fsanitize=thread and address targets").  N client threads hammer one
// server over loopback TCP with every op family at once:
//   * locked RAW_ADD applies (exact: the final value must equal the number of applies),
//   * lock-free (Hogwild) SGD applies with the global step incremented under the lock (exact count),
//   * conditional-accumulator apply/take with stale drops, token-queue enqueue/dequeue, barriers,
//   * concurrent READ / ASSIGN_ADD / LIST / STATS.
// Exit status 0 = all invariants hold; sanitizer reports make the process exit non-zero.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "dtg/ps.h"
#include "dtg/wire.h"

using namespace dtg;

static std::vector<uint8_t> body(const wire::Writer& w) { return w.buf; }

static wire::Tensor f32(const std::vector<int64_t>& shape, float v) {
  wire::Tensor t;
  t.dtype = wire::F32;
  t.shape = shape;
  int64_t n = t.numel();
  t.data.resize(n * 4);
  for (int64_t i = 0; i < n; ++i) memcpy(&t.data[i * 4], &v, 4);
  return t;
}

static int check(bool ok, const char* what) {
  if (!ok) fprintf(stderr, "FAILED: %s\n", what);
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  const int kThreads = argc > 1 ? atoi(argv[1]) : 8;
  const int kIters = argc > 2 ? atoi(argv[2]) : 200;
  ps::Server srv("127.0.0.1", 0, kThreads);
  srv.start();
  const int port = srv.port();
  {
    ps::Client c("127.0.0.1", port, 10.0);
    std::vector<uint8_t> r;
    for (const char* n : {"counter", "w"}) {
      wire::Writer w;
      w.str(n);
      w.tensor(f32({16}, 0.f));
      w.i64(1);
      c.call(wire::CREATE, body(w), &r);
    }
    {
      wire::Writer w;
      const int64_t zero = 0;
      w.str("global_step");
      w.tensor(wire::I64, {}, &zero, 8);
      w.i64(1);
      c.call(wire::CREATE, body(w), &r);
    }
    wire::Writer w;
    w.str("acc");
    w.tensor(f32({4}, 0.f));
    w.i64(0);  // initial global step
    c.call(wire::ACC_CREATE, body(w), &r);
  }
  std::atomic<int> failures{0};
  std::atomic<int64_t> acc_accepted{0}, tokens_taken{0};
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t) {
    th.emplace_back([&, t] {
      ps::Client c("127.0.0.1", port, 10.0);
      std::vector<uint8_t> r;
      for (int i = 0; i < kIters; ++i) {
        {  // locked exact add
          wire::Writer w;
          w.i64(wire::RAW_ADD);
          w.f64(1.0);  // w += 1.0 * g
          for (int k = 0; k < 4; ++k) w.f64(0.0);
          w.i64(1);
          w.str("");
          w.i64(1);
          w.str("counter");
          w.tensor(f32({16}, 1.f));
          if (c.call(wire::APPLY, body(w), &r) != wire::OK) failures++;
        }
        {  // Hogwild SGD + global step
          wire::Writer w;
          w.i64(wire::SGD);
          w.f64(0.01);
          for (int k = 0; k < 4; ++k) w.f64(0.0);
          w.i64(0);
          w.str("global_step");
          w.i64(1);
          w.str("w");
          w.tensor(f32({16}, 1.f));
          if (c.call(wire::APPLY, body(w), &r) != wire::OK) failures++;
        }
        {  // accumulator (local_step 0 vs global step possibly advanced -> some dropped)
          wire::Writer w;
          w.str("acc");
          w.i64(i);
          w.tensor(f32({4}, 1.f));
          const int32_t st = c.call(wire::ACC_APPLY, body(w), &r);
          if (st != wire::OK) failures++;
          if (st == wire::OK && r.size() >= 8) {
            int64_t a;
            memcpy(&a, r.data(), 8);
            acc_accepted += a;
          }
        }
        {  // tokens: enqueue 1, dequeue 1 (never blocks for long)
          wire::Writer w;
          w.str("tokens");
          w.i64(1);
          w.i64(t * 100000 + i);
          c.call(wire::Q_ENQ, body(w), &r);
          wire::Writer d;
          d.str("tokens");
          d.f64(5.0);
          if (c.call(wire::Q_DEQ, body(d), &r) == wire::OK) tokens_taken++;
        }
        if (i % 16 == 0) {  // readers and misc
          wire::Writer w;
          w.i64(2);
          w.str("counter");
          w.str("w");
          if (c.call(wire::READ, body(w), &r) != wire::OK) failures++;
          wire::Writer l;
          c.call(wire::LIST, body(l), &r);
          c.call(wire::STATS, body(l), &r);
          if (t == 0) {  // the chief advances the accumulator's global step
            wire::Writer s;
            s.str("acc");
            s.i64(i);
            c.call(wire::ACC_SET_STEP, body(s), &r);
          }
        }
      }
      wire::Writer b;
      b.str("end");
      b.i64(kThreads);
      b.f64(30.0);
      if (c.call(wire::BARRIER, body(b), &r) != wire::OK) failures++;
      wire::Writer d;
      d.i64(t);
      c.call(wire::WORKER_DONE, body(d), &r);
    });
  }
  for (auto& x : th) x.join();
  int bad = failures.load();
  wire::Tensor counter, gs;
  bad += check(srv.read_var("counter", &counter), "read counter");
  bad += check(srv.read_var("global_step", &gs), "read global_step");
  float cv0;
  int64_t gs0;
  memcpy(&cv0, counter.data.data(), 4);
  memcpy(&gs0, gs.data.data(), 8);
  bad += check(cv0 == (float)(kThreads * kIters), "locked RAW_ADD applies are exact");
  bad += check(gs0 == (int64_t)kThreads * kIters, "global step increments are exact");
  bad += check(tokens_taken.load() == (int64_t)kThreads * kIters, "every enqueued token dequeued");
  bad += check(acc_accepted.load() > 0, "accumulator accepted gradients");
  bad += check(srv.join(5.0), "join returns once all workers are done");
  srv.stop();
  printf("ps_stress: threads=%d iters=%d failures=%d counter=%.0f global_step=%lld acc_accepted=%lld tokens=%lld -> %s\n",
         kThreads, kIters, failures.load(), cv0, (long long)gs0, (long long)acc_accepted.load(), (long long)tokens_taken.load(),
         bad ? "FAIL" : "OK");
  return bad ? 1 : 0;
}
