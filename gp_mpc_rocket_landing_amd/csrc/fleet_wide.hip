// fleet_wide.hip -- the fleet's control kernel (fleet.hip, k_fleet_control2) built for
// small fleets: 256 threads per landing (one variable and at most one dynamics row per
// thread, fleet_qp.h FQ_T) and one wave per SIMD, so the register budget is 512 per lane
// (VGPRs + AGPRs) and nothing spills.  One landing per CU: fleet.hip launches it when the
// fleet has at most one landing per CU (gpmpc_fleet.wide).  Same algorithm and parity as
// the 128-thread build; the block-wide sums run over four waves instead of two.
#define FQ_T 256
#define FQ_WPE 1
#define FQ_KNS fq_wide
#define FLEET_WIDE_TU 1
#include "fleet.hip"
