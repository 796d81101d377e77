// b2s_paths at 16 lanes (host_b2s_impl.inc), built with -mavx512f
#include "host_b2s.h"

namespace stark {
namespace b2s_w16 {
#define B2S_W 16
#include "host_b2s_impl.inc"
#undef B2S_W
}  // namespace b2s_w16
}  // namespace stark
