// fleet6_h2.hip -- the 6-DoF rollout kernels (fleet6_n.h) for horizons N = 16 .. 20:
// every horizon is its own compile-time instance (fleet6.h), split over a few
// translation units so that they build in parallel.
#include "fleet6.h"
namespace r6n16 {
#define R6_N 16
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n16
namespace r6n17 {
#define R6_N 17
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n17
namespace r6n18 {
#define R6_N 18
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n18
namespace r6n19 {
#define R6_N 19
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n19
namespace r6n20 {
#define R6_N 20
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n20
