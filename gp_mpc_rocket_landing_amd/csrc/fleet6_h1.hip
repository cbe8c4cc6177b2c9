// fleet6_h1.hip -- the 6-DoF rollout kernels (fleet6_n.h) for horizons N = 10 .. 15:
// every horizon is its own compile-time instance (fleet6.h), split over a few
// translation units so that they build in parallel.
#include "fleet6.h"
namespace r6n10 {
#define R6_N 10
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n10
namespace r6n11 {
#define R6_N 11
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n11
namespace r6n12 {
#define R6_N 12
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n12
namespace r6n13 {
#define R6_N 13
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n13
namespace r6n14 {
#define R6_N 14
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n14
namespace r6n15 {
#define R6_N 15
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n15
