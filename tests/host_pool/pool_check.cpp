// Exactly-once check of libstark_hip's host worker pool (csrc/host_pool.cpp, built here with the
// STARK_POOL_TEST race-window hook) against a restatement of the round-4 pool it replaced, whose handoff
// is the hazard DESIGN.md 7.1 names: one claim counter served every call, so a worker still leaving call
// k could claim, run and count an item of call k + 1 (round-4 csrc/api.hip HostWorkers::drain).
// Test infrastructure (tests/test_host_pool.py).
//   usage: pool_check product|r4 [calls]
// Interleaved small (3-7 items) and large (24-64 items) host_parallel calls from two caller threads while
// the side thread runs HostTasks that make calls of their own.  Every item records its call and index;
// when a call returns, each of its items must have run exactly once and none may still be running.  The
// hook widens the window between a worker's claim and its bound check (a worker descheduled there, which
// oversubscribed rank processes make possible), so the r4 pool's stale claims show within a few calls.
// Exit 0: no violation; 1: a violation (printed); ThreadSanitizer builds exit 66 on a data race.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "host_pool.h"

static std::atomic<uint64_t> g_seed{12345};
static bool g_window = true;  // off for the latency diagnostic

// a short random pause in the claim window on about one claim in four
void stark_pool_test_window() {
  if (!g_window) return;
  thread_local std::minstd_rand rng((uint32_t)g_seed.fetch_add(7919));
  if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
}

namespace r4 {
// The round-4 pool (api.hip at the round-4 verdict commit, HostWorkers::run/drain/loop), restated with
// the same window hook after the claim.
class Pool {
 public:
  static Pool& get() {
    static Pool* p = new Pool();
    return *p;
  }
  void run(unsigned n, const std::function<void(unsigned)>& fn) {
    if (n == 0) return;
    if (n == 1 || workers_ == 0 || in_job()) {
      for (unsigned k = 0; k < n; ++k) fn(k);
      return;
    }
    std::lock_guard<std::mutex> serial(call_);
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &fn;
      n_ = n;
      next_.store(1);
      pending_ = n - 1;
      ++gen_;
    }
    cv_.notify_all();
    in_job() = true;
    fn(0);
    drain();
    in_job() = false;
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  Pool() {
    unsigned hw = std::thread::hardware_concurrency();
    hw = hw < 1 ? 1 : (hw > 16 ? 16 : hw);
    workers_ = hw - 1;
    for (unsigned i = 0; i < workers_; ++i) std::thread([this] { loop(); }).detach();
  }
  static bool& in_job() {
    thread_local bool flag = false;
    return flag;
  }
  void drain() {
    for (;;) {
      const unsigned k = next_.fetch_add(1);
      stark_pool_test_window();
      if (k >= n_) break;
      (*job_)(k);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
      }
      in_job() = true;
      drain();
      in_job() = false;
    }
  }
  size_t workers_ = 0;
  std::mutex call_, m_;
  std::condition_variable cv_, done_;
  const std::function<void(unsigned)>* job_ = nullptr;
  unsigned n_ = 0, pending_ = 0;
  std::atomic<unsigned> next_{0};
  uint64_t gen_ = 0;
};
}  // namespace r4

static bool g_r4 = false;
static void par(unsigned n, const std::function<void(unsigned)>& fn) {
  if (g_r4) {
    r4::Pool::get().run(n, fn);
  } else {
    stark::host_parallel(n, fn);
  }
}

static std::atomic<int> g_fail{0};
static std::atomic<uint64_t> g_done_calls{0};  // progress, for the watchdog

// One call of n items; checks exactly-once and nothing running after return.
static void one_call(unsigned n, unsigned spin_us, const char* who, unsigned id) {
  std::unique_ptr<std::atomic<int>[]> hits(new std::atomic<int>[n]);
  for (unsigned i = 0; i < n; ++i) hits[i] = 0;
  std::atomic<int> running{0};
  par(n, [&, n](unsigned k) {
    running.fetch_add(1);
    if (k >= n) g_fail.store(1);
    if (spin_us) {
      const auto t0 = std::chrono::steady_clock::now();
      while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(spin_us)) {
      }
    }
    if (k < n) hits[k].fetch_add(1);
    running.fetch_sub(1);
  });
  const int still = running.load();
  int bad = still != 0;
  for (unsigned i = 0; i < n; ++i) bad |= hits[i].load() != 1;
  if (bad && g_fail.exchange(1) == 0) {
    fprintf(stderr, "%s call %u (%u items): %d item(s) still running at return; hits:", who, id, n, still);
    for (unsigned i = 0; i < n; ++i)
      if (hits[i].load() != 1) fprintf(stderr, " [%u]=%d", i, hits[i].load());
    fprintf(stderr, "\n");
    fflush(stderr);
    std::_Exit(1);  // (a broken pool may also hang or crash from here on: stop at the first violation)
  }
  // (a late item of a returned call may still touch hits/running: give it time before they go)
  if (bad) std::this_thread::sleep_for(std::chrono::milliseconds(50));
  g_done_calls.fetch_add(1);
}

static void caller(unsigned calls, unsigned seed, const char* who) {
  std::minstd_rand rng(seed);
  for (unsigned c = 0; c < calls && !g_fail.load(); ++c) {
    const bool small = c % 2 == 0;
    const unsigned n = small ? 3 + rng() % 5 : 24 + rng() % 41;
    one_call(n, rng() % 20, who, c);
  }
}

// Dispatch latency of the product pool (a diagnostic, not a test): wall time of host_parallel(16, ~2 us
// items), back to back and after an idle gap that lets the workers fall asleep.
static int latency() {
  g_window = false;
  const unsigned n = std::min(16u, stark::host_threads());
  for (int gap_us : {0, 300}) {
    std::vector<double> ts;
    for (int i = 0; i < 400; ++i) {
      if (gap_us) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
      const auto t0 = std::chrono::steady_clock::now();
      stark::host_parallel(n, [](unsigned) {
        const auto s0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - s0 < std::chrono::microseconds(2)) {
        }
      });
      ts.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(ts.begin(), ts.end());
    printf("host_parallel(%u) after %d us idle: median %.1f us, p90 %.1f us, min %.1f us\n", n, gap_us,
           ts[ts.size() / 2], ts[ts.size() * 9 / 10], ts[0]);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && !strcmp(argv[1], "latency")) return latency();
  if (argc < 2 || (strcmp(argv[1], "product") && strcmp(argv[1], "r4"))) {
    fprintf(stderr, "usage: pool_check product|r4|latency [calls]\n");
    return 2;
  }
  g_r4 = strcmp(argv[1], "r4") == 0;
  const unsigned calls = argc > 2 ? (unsigned)atoi(argv[2]) : 400;
  // A broken pool can also lose an item's completion and wait forever (the round-4 pool's double-counted
  // pending_): no call finishing for 10 s is reported as a violation too.
  std::thread([] {
    uint64_t last = g_done_calls.load();
    for (;;) {
      std::this_thread::sleep_for(std::chrono::seconds(10));
      const uint64_t now = g_done_calls.load();
      if (now == last) {
        fprintf(stderr, "no call returned in 10 s after %llu calls (a lost completion); hits: hang\n",
                (unsigned long long)now);
        fflush(stderr);
        std::_Exit(1);
      }
      last = now;
    }
  }).detach();
  std::thread a([&] { caller(calls, 1, "caller A"); });
  std::thread b([&] { caller(calls, 2, "caller B"); });
  // side-thread tasks that make host_parallel calls of their own while the callers run
  if (!g_r4) {
    for (unsigned t = 0; t < calls / 8 && !g_fail.load(); ++t) {
      stark::HostTask task([&, t] { caller(4, 100 + t, "side task"); });
      caller(2, 200 + t, "main");
      task.wait();
    }
  }
  a.join();
  b.join();
  if (g_fail.load()) return 1;
  printf("ok: %u calls per caller, %s pool\n", calls, g_r4 ? "round-4" : "product");
  return 0;
}
