// Host worker threads of libstark_hip (host_pool.cpp): host-only C++, no HIP, so the pool is built and
// tested on its own on the CPU (tests/host_pool: exactly-once checks and a ThreadSanitizer build).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>

namespace stark {

// Host worker threads shared by the host-side stages (trace build, proof
// JSON): host_parallel(n, fn) runs fn(0) .. fn(n-1), fn(0) on the caller, the
// rest on persistent workers (spawning threads per call costs more than the
// millisecond-scale work it splits).  host_threads() = workers + 1 (<= 16).
unsigned host_threads();
void host_parallel(unsigned n, const std::function<void(unsigned)>& fn);
// memcpy, split over the host workers from 1 MB on (a multi-MB proof text into caller memory).
void host_memcpy(void* dst, const void* src, size_t n);
// A task run on the process's side thread while the caller goes on (the caller waits for it with
// wait() or the destructor, so the task may use the caller's locals).  When the side thread is busy
// with another caller's task, the task runs inline in the constructor.
class HostTask {
 public:
  explicit HostTask(std::function<void()> fn);
  ~HostTask() { wait(); }
  void wait();
  HostTask(const HostTask&) = delete;
  HostTask& operator=(const HostTask&) = delete;

 private:
  uint64_t ticket_ = 0;  // 0: ran inline or already waited for
};

}  // namespace stark
