// b2s_paths at 4 lanes (host_b2s_impl.inc)
#include "host_b2s.h"

namespace stark {
namespace b2s_w4 {
#define B2S_W 4
#include "host_b2s_impl.inc"
#undef B2S_W
}  // namespace b2s_w4
}  // namespace stark
