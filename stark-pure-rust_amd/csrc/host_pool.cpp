// Host worker pool and side thread (declared in host_pool.h).  Host-only: libstark_hip links it, and
// tests/host_pool builds it alone with a race-window hook (STARK_POOL_TEST) and under ThreadSanitizer.
#include "host_pool.h"

#include <string.h>

#include <algorithm>
#include <atomic>
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

class HostWorkers {
 public:
  static HostWorkers& get() {
    static HostWorkers* w = new HostWorkers();  // never destroyed: workers live for the process
    return *w;
  }
  unsigned threads() const { return (unsigned)workers_ + 1; }
  // Each call is a Job of its own (on the caller's stack): a worker takes a reference to the current
  // job under the lock and claims items from that job's counter only, and the caller returns once
  // every item is done AND every worker that joined has let go of the job.  (The previous form kept
  // one counter for all calls: a worker still leaving call k could claim, run and count an item of
  // call k + 1 while that call was being set up, so the call could return with an item unfinished.)
  void run(unsigned n, const std::function<void(unsigned)>& fn) {
    if (n == 0) return;
    if (n == 1 || workers_ == 0 || in_job()) {  // a job that calls host_parallel runs the inner one serially
      for (unsigned k = 0; k < n; ++k) fn(k);
      return;
    }
    std::lock_guard<std::mutex> serial(call_);  // one parallel call at a time
    Job job{&fn, n};
    {
      std::lock_guard<std::mutex> g(m_);
      cur_ = &job;
      ++gen_;
    }
    cv_.notify_all();
    in_job() = true;
    work(job);
    in_job() = false;
    std::unique_lock<std::mutex> g(m_);
    cur_ = nullptr;  // no worker joins from here on
    done_.wait(g, [&] { return job.done == job.n && job.refs == 0; });
  }

 private:
  struct Job {
    const std::function<void(unsigned)>* fn;
    unsigned n;
    std::atomic<unsigned> next{0};
    unsigned done = 0, refs = 0;  // under m_
  };
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
  void work(Job& job) {
    unsigned mine = 0;
    for (;; ++mine) {
      const unsigned k = job.next.fetch_add(1);
      STARK_POOL_WINDOW();  // (tests/host_pool: a claim descheduled before its bound check)
      if (k >= job.n) break;
      (*job.fn)(k);
    }
    if (mine) {
      std::lock_guard<std::mutex> g(m_);
      job.done += mine;
      if (job.done == job.n) done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      Job* job;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        job = cur_;
        if (!job) continue;  // that call has already finished
        ++job->refs;
      }
      in_job() = true;
      work(*job);
      in_job() = false;
      std::lock_guard<std::mutex> g(m_);
      if (--job->refs == 0) done_.notify_all();
    }
  }
  size_t workers_ = 0;
  std::mutex call_, m_;
  std::condition_variable cv_, done_;
  Job* cur_ = nullptr;
  uint64_t gen_ = 0;
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
    cv_.notify_all();
    return t;
  }
  void wait(uint64_t ticket) {
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [&] { return done_ >= ticket; });
  }

 private:
  SideWorker() { std::thread([this] { loop(); }).detach(); }
  void loop() {
    for (;;) {
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
      done_cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::function<void()> task_;
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
