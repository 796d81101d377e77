// b2s_paths at 8 lanes (host_b2s_impl.inc), built with -mavx2
#include "host_b2s.h"

namespace stark {
namespace b2s_w8 {
#define B2S_W 8
#include "host_b2s_impl.inc"
#undef B2S_W
}  // namespace b2s_w8
}  // namespace stark
