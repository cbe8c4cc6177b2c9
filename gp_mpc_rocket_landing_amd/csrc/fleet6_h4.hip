// fleet6_h4.hip -- the 6-DoF rollout kernels (fleet6_n.h) for horizons N = 26 .. 30:
// every horizon is its own compile-time instance (fleet6.h), split over a few
// translation units so that they build in parallel.
#include "fleet6.h"
namespace r6n26 {
#define R6_N 26
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n26
namespace r6n27 {
#define R6_N 27
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n27
namespace r6n28 {
#define R6_N 28
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n28
namespace r6n29 {
#define R6_N 29
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n29
namespace r6n30 {
#define R6_N 30
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n30
