// fleet6_h0.hip -- the 6-DoF rollout kernels (fleet6_n.h) for horizons N = 2 .. 9:
// every horizon is its own compile-time instance (fleet6.h), split over a few
// translation units so that they build in parallel.
#include "fleet6.h"
namespace r6n2 {
#define R6_N 2
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n2
namespace r6n3 {
#define R6_N 3
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n3
namespace r6n4 {
#define R6_N 4
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n4
namespace r6n5 {
#define R6_N 5
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n5
namespace r6n6 {
#define R6_N 6
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n6
namespace r6n7 {
#define R6_N 7
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n7
namespace r6n8 {
#define R6_N 8
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n8
namespace r6n9 {
#define R6_N 9
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n9
