// fleet6_h3.hip -- the 6-DoF rollout kernels (fleet6_n.h) for horizons N = 21 .. 25:
// every horizon is its own compile-time instance (fleet6.h), split over a few
// translation units so that they build in parallel.
#include "fleet6.h"
namespace r6n21 {
#define R6_N 21
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n21
namespace r6n22 {
#define R6_N 22
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n22
namespace r6n23 {
#define R6_N 23
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n23
namespace r6n24 {
#define R6_N 24
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n24
namespace r6n25 {
#define R6_N 25
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n25
