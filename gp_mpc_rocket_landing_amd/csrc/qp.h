// qp.h -- internal QP interfaces shared by qp.hip and fleet.hip.
#pragma once
#include "internal.h"
#include "qp_device.h"

// LDS caps of the single compiled instantiation (3-DoF MPC up to N = 21)
#define QP_NMAX 224
#define QP_MMAX 384
#define QP_NNZMAX 800
#define QP_W 16
typedef QPSmem<QP_NMAX, QP_MMAX, QP_NNZMAX, QP_W> QPSmemStd;

struct QPPatternHost {
  int n = 0, m = 0, nnz = 0, w = 0;
  DevBuf buf;
  QPPattern dev{};
  int build(int n, int m, const int *rowptr, const int *colidx, hipStream_t s);
};

QPSettingsDev to_dev(const gpmpc_qp_settings &s);
