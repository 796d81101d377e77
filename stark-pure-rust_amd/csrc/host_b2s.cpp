// b2s_paths: the widest vector the CPU runs (host_b2s.h).
#include "host_b2s.h"

namespace stark {
namespace b2s_w16 { void paths(const PathJob* jobs, size_t n, uint8_t* ok); }
namespace b2s_w8 { void paths(const PathJob* jobs, size_t n, uint8_t* ok); }
namespace b2s_w4 { void paths(const PathJob* jobs, size_t n, uint8_t* ok); }

int b2s_paths_width() {
  static const int w = __builtin_cpu_supports("avx512f") ? 16 : __builtin_cpu_supports("avx2") ? 8 : 4;
  return w;
}

void b2s_paths(const PathJob* jobs, size_t n, uint8_t* ok) {
  switch (b2s_paths_width()) {
    case 16: b2s_w16::paths(jobs, n, ok); break;
    case 8: b2s_w8::paths(jobs, n, ok); break;
    default: b2s_w4::paths(jobs, n, ok); break;
  }
}

}  // namespace stark
