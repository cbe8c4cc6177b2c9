// qp.h -- internal QP interfaces shared by qp.hip and fleet.hip.
#pragma once
#include "internal.h"
#include "qp_device.h"

// LDS caps of the single compiled instantiation: 3-DoF MPC up to N = 20
// (n = 10N + 7, m = 17N + 14, nnz = 36N + 14; NMAX also holds n rounded up to
// whole stage blocks), sized so that the fleet's control kernel stays under
// 80 KB and two workgroups share a CU
#define QP_NMAX 216
#define QP_MMAX 360
#define QP_NNZMAX 896
#define QP_W 16
typedef QPSmem<QP_NMAX, QP_MMAX, QP_NNZMAX, QP_W> QPSmemStd;
// factor slots available in QPSmem (its factor area minus the 4 zero columns)
#define QP_FAC_CAP (QP_NMAX * (QP_W + 1) + 64)

struct QPPatternHost {
  int n = 0, m = 0, nnz = 0, w = 0, maxrow = 0, maxcol = 0;
  int mode = 0, fac_len = 0, nblk = 0;
  bool fits() const {
    return n <= QP_NMAX && m <= QP_MMAX && nnz <= QP_NNZMAX && maxrow <= QP_RMAX &&
           maxcol <= QP_CMAX &&
           (mode == 1 ? nblk * QP_BLK_SZ <= QP_NMAX : (w <= QP_W && fac_len <= QP_FAC_CAP));
  }
  DevBuf buf;
  QPPattern dev{};
  int build(int n, int m, const int *rowptr, const int *colidx, hipStream_t s);
};

QPSettingsDev to_dev(const gpmpc_qp_settings &s);
// the fleet's specialised solver for batched QPs on its pattern (fleet.hip k_qp_fleet): the
// 128-thread build (four problems per CU) and the 256-thread one (one per CU)
bool qp_is_fleet_pattern(int n, int m, const int *rowptr, const int *colidx);
#define QP_FLEET_MD 147  // its dynamics rows (fleet_qp.h FQ_MD)
#define QP_FLEET_DECL(name)                                                                                    \
  hipError_t name(hipStream_t s, int batch, const QPPattern &pt, const QPSettingsDev &st, const double *Aval,  \
                  const double *Pd, const double *q, const double *l, const double *u, const double *xws,      \
                  double *rho, double *yst, double *xo, double *yo, int *iters, int *status, double *obj);
QP_FLEET_DECL(launch_qp_fleet_narrow)
QP_FLEET_DECL(launch_qp_fleet_wide)
