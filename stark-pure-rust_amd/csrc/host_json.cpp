// json_simd_width: the JSON byte-array writer's path on this CPU (host_json.h).
#include "host_json.h"

#include <stdlib.h>

namespace stark {

static int pick_json_width() {
  const bool have = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                    __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512vbmi") &&
                    __builtin_cpu_supports("avx512vbmi2") && __builtin_cpu_supports("bmi") &&
                    __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("popcnt");
  const char* e = getenv("STARK_JSON_SIMD");
  const bool want = !(e && e[0] == '0');
  return have && want ? 64 : 1;
}

int json_simd_width() {
  static const int w = pick_json_width();
  return w;
}

}  // namespace stark
