// Host worker pool and side thread (declared in host_pool.h).  Host-only: libstark_hip links it, and
// tests/host_pool builds it alone with a race-window hook (STARK_POOL_TEST) and under ThreadSanitizer.
#include "host_pool.h"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>

#ifdef STARK_POOL_TEST
void stark_pool_test_window();  // provided by the test harness
#define STARK_POOL_WINDOW() stark_pool_test_window()
#else
#define STARK_POOL_WINDOW() ((void)0)
#endif

namespace stark {

namespace {

// Spin-then-block: poll for up to kSpinUs before sleeping on a condition variable.  A proof makes its
// host_parallel calls and side tasks in bursts, and a wake-up through a condition variable costs each
// thread tens of microseconds (tests/host_pool/pool_check latency).
constexpr int kSpinUs = 40;
template <class Pred>
bool spin_until(Pred pred) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0;; ++i) {
    if (pred()) return true;
    if ((i & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs)) return false;
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
}

class HostWorkers {
 public:
  static HostWorkers& get() {
    static HostWorkers* w = new HostWorkers();  // never destroyed: workers live for the process
    return *w;
  }
  unsigned threads() const { return (unsigned)workers_ + 1; }
  // One call at a time (call_).  A call is published as a 64-bit ticket (generation << 32 | next item);
  // an item is claimed by a compare-exchange of the ticket, which fails for a worker still holding a
  // ticket of an earlier call, so a late worker can neither run nor skip an item of the current call
  // (the round-4 pool's shared counter let it do both: DESIGN.md 7.1, tests/host_pool).  The call
  // returns once `done` counts all of its items; nothing of a call is read after its last item ends.
  // Workers and the caller spin briefly before they sleep: a proof makes its calls in bursts, and a
  // wake-up through a condition variable costs each worker tens of microseconds.
  void run(unsigned n, const std::function<void(unsigned)>& fn) {
    if (n == 0) return;
    if (n == 1 || workers_ == 0 || in_job()) {  // a job that calls host_parallel runs the inner one serially
      for (unsigned k = 0; k < n; ++k) fn(k);
      return;
    }
    std::lock_guard<std::mutex> serial(call_);
    // Seal the previous call's ticket first: a worker that read that call's exhausted ticket and then
    // this call's n_ (below) could otherwise claim "item n_old" of the old generation, i.e. run an item
    // of this call under the old ticket, and count it twice (tests/host_pool caught exactly this).
    ticket_.store((ticket_.load(std::memory_order_relaxed) & ~(uint64_t)0xFFFFFFFFu) | 0xFFFFFFFFu,
                  std::memory_order_relaxed);
    fn_.store(&fn, std::memory_order_release);
    n_.store(n, std::memory_order_release);  // (a worker that sees this n also sees the seal)
    done_.store(0, std::memory_order_relaxed);
    const uint64_t gen = ++gen_;
    ticket_.store(gen << 32, std::memory_order_release);  // (publishes fn_, n_, done_)
    { std::lock_guard<std::mutex> g(m_); }  // a worker between its check and its sleep is asleep now
    wake_.notify_all();
    in_job() = true;
    work(gen);
    in_job() = false;
    auto finished = [&] { return done_.load(std::memory_order_acquire) == n; };
    if (!spin_until(finished)) {
      std::unique_lock<std::mutex> g(m_);
      finished_.wait(g, finished);
    }
  }

 private:
  HostWorkers() {
    unsigned hw = std::thread::hardware_concurrency();
    hw = hw < 1 ? 1 : (hw > 16 ? 16 : hw);
    workers_ = hw - 1;
    for (unsigned i = 0; i < workers_; ++i) std::thread([this] { loop(); }).detach();
  }
  static bool& in_job() {
    thread_local bool flag = false;
    return flag;
  }
  // Claims and runs items of call `gen` until none is left (or the call is no longer current).
  void work(uint64_t gen) {
    uint64_t t = ticket_.load(std::memory_order_acquire);
    for (;;) {
      const unsigned n = n_.load(std::memory_order_acquire);  // (validated by the exchange below)
      if ((t >> 32) != gen || (uint32_t)t >= n) return;
      if (!ticket_.compare_exchange_weak(t, t + 1, std::memory_order_acq_rel, std::memory_order_acquire)) continue;
      STARK_POOL_WINDOW();  // (tests/host_pool: a claimant descheduled before it runs the item)
#ifdef STARK_POOL_TEST
      {
        const uint64_t now = ticket_.load(std::memory_order_acquire);
        if ((now >> 32) != gen) {  // the call ended early
          fprintf(stderr, "pool: claimed (%llu, %u) of n %u, ticket now (%llu, %u), done %u, n_ %u\n",
                  (unsigned long long)gen, (unsigned)(uint32_t)t, n, (unsigned long long)(now >> 32),
                  (unsigned)(uint32_t)now, done_.load(), n_.load());
          __builtin_trap();
        }
      }
#endif
      (*fn_.load(std::memory_order_acquire))((uint32_t)t);
      const unsigned prev = done_.fetch_add(1, std::memory_order_acq_rel);
#ifdef STARK_POOL_TEST
      if (prev >= n) {
        fprintf(stderr, "pool: done %u >= n %u after item (%llu, %u); ticket (%llu, %u)\n", prev, n,
                (unsigned long long)gen, (unsigned)(uint32_t)t, (unsigned long long)(ticket_.load() >> 32),
                (unsigned)(uint32_t)ticket_.load());
        __builtin_trap();
      }
#endif
      if (prev + 1 == n) {
        std::lock_guard<std::mutex> g(m_);
        finished_.notify_all();
      }
      t = ticket_.load(std::memory_order_acquire);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      auto fresh = [&] { return (ticket_.load(std::memory_order_acquire) >> 32) != seen; };
      if (!spin_until(fresh)) {
        std::unique_lock<std::mutex> g(m_);
        wake_.wait(g, fresh);
      }
      seen = ticket_.load(std::memory_order_acquire) >> 32;
      in_job() = true;
      work(seen);
      in_job() = false;
    }
  }
  size_t workers_ = 0;
  std::mutex call_, m_;
  std::condition_variable wake_, finished_;
  std::atomic<const std::function<void(unsigned)>*> fn_{nullptr};
  std::atomic<unsigned> n_{0}, done_{0};
  std::atomic<uint64_t> ticket_{0};
  uint64_t gen_ = 0;  // under call_
};

// One side thread for HostTask: one task at a time, tickets in submission order.
class SideWorker {
 public:
  static SideWorker& get() {
    static SideWorker* w = new SideWorker();  // never destroyed, like HostWorkers
    return *w;
  }
  uint64_t submit(std::function<void()>& fn) {  // 0 when busy (the caller then runs fn itself)
    std::lock_guard<std::mutex> g(m_);
    if (task_) return 0;
    task_ = std::move(fn);
    const uint64_t t = ++submitted_;
    submitted_a_.store(t, std::memory_order_release);
    cv_.notify_all();
    return t;
  }
  void wait(uint64_t ticket) {
    if (spin_until([&] { return done_a_.load(std::memory_order_acquire) >= ticket; })) return;
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [&] { return done_ >= ticket; });
  }

 private:
  SideWorker() { std::thread([this] { loop(); }).detach(); }
  void loop() {
    for (uint64_t seen = 0;; ++seen) {
      spin_until([&] { return submitted_a_.load(std::memory_order_acquire) > seen; });
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return (bool)task_; });
        fn = task_;
      }
      fn();
      std::lock_guard<std::mutex> g(m_);
      task_ = nullptr;
      ++done_;
      done_a_.store(done_, std::memory_order_release);
      done_cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::function<void()> task_;
  std::atomic<uint64_t> submitted_a_{0}, done_a_{0};
  uint64_t submitted_ = 0, done_ = 0;
};

}  // namespace

HostTask::HostTask(std::function<void()> fn) {
  ticket_ = SideWorker::get().submit(fn);
  if (!ticket_) fn();
}

void HostTask::wait() {
  if (ticket_) SideWorker::get().wait(ticket_);
  ticket_ = 0;
}

unsigned host_threads() { return HostWorkers::get().threads(); }
void host_parallel(unsigned n, const std::function<void(unsigned)>& fn) { HostWorkers::get().run(n, fn); }

void host_memcpy(void* dst, const void* src, size_t n) {
  constexpr size_t kPiece = (size_t)256 << 10;
  if (n < ((size_t)1 << 20)) {
    memcpy(dst, src, n);
    return;
  }
  const size_t pieces = (n + kPiece - 1) / kPiece;
  std::atomic<size_t> next{0};
  const unsigned nt = (unsigned)std::min<size_t>(host_threads(), pieces);
  host_parallel(nt, [&](unsigned) {
    for (size_t i; (i = next.fetch_add(1)) < pieces;) {
      const size_t o = i * kPiece;
      memcpy((char*)dst + o, (const char*)src + o, std::min(kPiece, n - o));
    }
  });
}

}  // namespace stark
