// b2s_paths: the widest vector the CPU runs (host_b2s.h).
#include "host_b2s.h"

#include <stdlib.h>

namespace stark {
namespace b2s_w16 { void paths(const PathJob* jobs, size_t n, uint8_t* ok); }
namespace b2s_w8 { void paths(const PathJob* jobs, size_t n, uint8_t* ok); }
namespace b2s_w4 { void paths(const PathJob* jobs, size_t n, uint8_t* ok); }

// STARK_B2S_WIDTH=4|8|16 narrows the choice (tests cover every width on one host); a width the CPU
// lacks is never taken.
static int pick_width() {
  const int have = __builtin_cpu_supports("avx512f") ? 16 : __builtin_cpu_supports("avx2") ? 8 : 4;
  const char* e = getenv("STARK_B2S_WIDTH");
  const int want = e ? atoi(e) : 16;
  return want >= 16 ? have : want >= 8 ? (have >= 8 ? 8 : 4) : 4;
}

int b2s_paths_width() {
  static const int w = pick_width();
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
