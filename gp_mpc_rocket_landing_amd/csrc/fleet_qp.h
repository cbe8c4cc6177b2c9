// fleet_qp.h -- the fleet's OSQP-0.6 ADMM, specialised to the 3-DoF MPC QP so
// that FOUR landings share a CU.
//
// The generic solver (qp_device.h) keeps every vector in LDS: 78 KB per QP,
// two QPs per CU.  With 1024 landings on 512 slots and ~64% of solves running
// the full 50 iterations (490 us vs 240 us for 25), 142 slots must run two
// long solves back to back (measured span 916-967 us; no dispatch order can
// beat 2 x 490 us).  At four per CU every landing starts at once.
//
// The MPC QP has a fixed row layout (fleet.hip mpc_pattern): rows 0..MD-1 are
// the initial-state and dynamics equalities, rows MD..MD+n-1 are the identity
// bound rows of variables 0..n-1.  A bound row touches only its own variable,
// so a thread that owns variable j also owns row MD+j: the bound row's A entry,
// l, u, E, y, z, rho z - y and delta y live in that thread's registers, as do
// x, dx, P, q, D of the variable.  Only what crosses threads stays in LDS: the
// dynamics rows' A values, their rho z - y (the A' operand), x~ (the block
// solve's right-hand side) and the block-tridiagonal factor.  Checks stage x,
// y, delta y, delta x through the x~ / (rho z - y) slots, which are dead then.
//
// 128 threads (2 waves): thread t owns variables t, t+128 and dynamics rows
// 127-t, 255-t.  Every arithmetic expression is the generic solver's, in the
// same order (same rounding), except the block-wide sums, whose tree now has
// two waves.  The dynamics rows are equalities (l = u, built so by the fleet),
// so one bound value serves both.  The row scaling E lives in LDS (only the
// scaling and the checks read it); the row / column patterns are packed in
// 16-bit pairs to keep the register budget at 256.  LDS ~39.7 KB.
#pragma once
#include "qp_device.h"

#ifndef FQ_T
#define FQ_T 128      // threads per landing: 128 (two items per thread) or 256 (one)
#endif
#define FQ_H (FQ_T >= 256 ? 1 : 2)  // item slots per thread
#define FQ_NW (FQ_T / 64)           // waves per landing
#define FQ_MD 147     // dynamics rows: NX (N+1) at N = 20
#define FQ_NNZD 527   // their nonzeros: NX + 26 N
#define FQ_NMAX 224   // x~: n = 207 padded to whole blocks (210) + the solve's look-ahead reads
#define FQ_NBLK 21
#define FQ_FAC (FQ_NBLK * (QP_BLK_SZ * QP_BLK_SZ + QP_BLK_SZ * QP_BLK_CM) + 16)
#define FQ_CMAX 6     // dynamics entries per column (<= 5) + 1
#define FQ_RMAX 5     // entries per dynamics row
#ifndef FQ_DIAG_SPLIT
#define FQ_DIAG_SPLIT 1  // the KKT diagonal products on both waves (needs !FQ_FUSED_DIAG)
#endif
// LDS-only workgroup barrier (no wait on outstanding global memory operations)
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// FQ_RHS_PAIR 1: the right-hand side's two column dot products with all their reads in flight
// (measured 295.2 -> 293.6 us at 1024 landings, two runs each: within the noise; off)
#ifndef FQ_RHS_PAIR
#define FQ_RHS_PAIR 0
#endif
#ifndef FQ_FUSED_DIAG
#define FQ_FUSED_DIAG false  // block solve: G chain first, then the diagonal blocks 4 at a time
#endif
// FQ_LAUNDER bit 0: the diagonal phase's thread index, bit 1: the items' indices (once per
// ADMM iteration) made opaque, so that the addresses derived from them are formed inside
// the loop rather than hoisted out of it into spilled registers.  Measured
// (profiles/r5_fleet_launder_ab.log, 3 runs each at 1024 landings): spills 54 -> 3,
// traffic 47 -> 17 MB per launch, but the kernel 291 -> 303 us (the 17 packed-row
// addresses of a diagonal round recomputed on the phase's path); off.  The 6-DoF
// kernel, where the hoisted values were the loop's live state, keeps it (fleet6.h).
// FQ_AREG 1: each item's column of scaled dynamics values in registers for the solve
// (the right-hand side's column dots then read only rho z - y from LDS).  Measured
// (profiles/r5_fleet_areg_ab.log, 3 runs each): 291 -> 322 us (306 with the diagonal
// phase rolled): the registers are worth more than the LDS reads; off.
#ifndef FQ_AREG
#define FQ_AREG 0
#endif
#ifndef FQ_LAUNDER
#define FQ_LAUNDER 0
#endif
__device__ __forceinline__ int fq_tid() {
  int t = threadIdx.x;
#if FQ_LAUNDER & 1
  asm volatile("" : "+v"(t));
#endif
  return t;
}
// FQ_TWIST: the two-ended factor / solve of fleet_twist.h (10-block chains instead of 20)
#ifndef FQ_TWIST
#define FQ_TWIST 1
#endif
#include "fleet_twist.h"
// FQ_PART: the partitioned solve of fleet_part.h, opt-in for the wide build (-DFQ_PART=1).
// Measured (profiles/r6_partitioned_kkt.md): its substitution takes 4235 cycles against the
// twisted solve's 5560, but its factor (segment chains, spikes, the 30 x 30 Shat^-1) 85.9K
// against 41.7K and the consumers' V x_S terms add ~550 a iteration: 194 us a single-landing
// step against 177 us.  Kept for the record and the probe (scripts/hip/fp_probe.hip).
#ifndef FQ_PART
#define FQ_PART 0
#endif
#if FQ_PART
static_assert(FQ_T >= 256, "the partitioned solve's correction takes one variable per thread");
#include "fleet_part.h"
#endif

struct FleetSmem {
  double A[FQ_NNZD + 1];
  double rhs[FQ_NMAX];   // x~ (block solve b); check-time scratch for x / dx
  double zt[FQ_MD + 1];  // rho z - y of the dynamics rows; check-time scratch for y / dy
  double E[FQ_MD + FQ_NMAX];  // row scaling: dynamics rows, then bound row MD + j
  double band_store[FQ_FAC];
  double gzero[64];      // zero "-G rows" of the non-coupled lanes (they read gzero[0..63])
  double zslot, sink;
  double red[FQ_NW][16];
  double c, rho_s;
  int flag;
#if FQ_PART
  double spk[FP_SPK];          // spikes V = M_II^-1 M_IS (fleet_part.h)
  double sinv[FP_NS * FP_NS];  // Shat^-1
  alignas(16) double xs[32];   // x_S (read as 16-byte pairs)
  double bh[64];               // bhat_S; the Shat inverse's pivot rows
  double brhs[FQ_NMAX];        // copy of the KKT right-hand side (the spike partial sums read it)
  double part[80];             // the partial sums L_k^T b_k of segments B and C
#endif
  __device__ double *band() { return band_store; }
};

template <int K>
__device__ __forceinline__ void fq_max(double (&v)[K], double (*red)[16]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] = fmax(v[k], __shfl_xor(v[k], o));
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[wv][k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double m = red[0][k];
#pragma unroll
    for (int w = 1; w < FQ_NW; ++w) m = fmax(m, red[w][k]);
    v[k] = m;
  }
  __syncthreads();
}

template <int K>
__device__ __forceinline__ void fq_sum(double (&v)[K], double (*red)[16]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[wv][k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double t = red[0][k];
#pragma unroll
    for (int w = 1; w < FQ_NW; ++w) t += red[w][k];
    v[k] = t;
  }
  __syncthreads();
}

// block-wide sum of a and max of b in one exchange (3 barriers instead of 6);
// each tree is fq_sum's / fq_max's
__device__ __forceinline__ void fq_sum_max(double &a, double &b, double (*red)[16]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b = fmax(b, __shfl_xor(b, o));
  }
  __syncthreads();
  if (lane == 0) { red[wv][0] = a; red[wv][1] = b; }
  __syncthreads();
  a = red[0][0];
  b = red[0][1];
#pragma unroll
  for (int w = 1; w < FQ_NW; ++w) {
    a += red[w][0];
    b = fmax(b, red[w][1]);
  }
  __syncthreads();
}

__device__ __forceinline__ double fq_rho(double l, double u, double rs) {
  if (l < -QP_OSQP_INFTY * QP_MIN_SCALING && u > QP_OSQP_INFTY * QP_MIN_SCALING) return QP_RHO_MIN;
  if (u - l < QP_RHO_TOL) return QP_RHO_EQ * rs;
  return rs;
}

// per-thread state: 2 variable slots (+ their bound rows), 2 dynamics-row slots
struct FleetRegs {
  bool vok[2], rok[2];
  int vj[2], rr[2];
  // variable j and bound row MD + j
  double x[2], dx[2], P[2], q[2], D[2];
  double Ab[2], lb[2], ub[2];
  // the bound row's y, z, delta y as scalars per slot, not arrays: an array whose slot-1
  // element also serves the aliased dynamics row (yr / zr / dyr below) was kept in scratch
  double yb0, yb1, zb0, zb1, dyb0, dyb1;  // (rho z - y of the bound row: recomputed)
  __device__ __forceinline__ double &yb_(int h) { return h ? yb1 : yb0; }
  __device__ __forceinline__ double &zb_(int h) { return h ? zb1 : zb0; }
  __device__ __forceinline__ double &dyb_(int h) { return h ? dyb1 : dyb0; }
  // dynamics row 0 (l = u = ur).  No thread owns both a second variable and a
  // second dynamics row (t < 79: 2 variables + 1 row; t >= 109: 1 + 2), so row
  // slot 1 lives in variable slot 1's registers: ur <- P, yr <- yb, zr <- zb,
  // dyr <- dyb, its pattern in cp[1][0..3]
  double ur0, yr0, zr0, dyr0;
  // patterns: column j's dynamics entries, (CSR value index) | (row << 16);
  // row r: first value index | count << 16, column indices two per int
  int cn[2], cp[2][FQ_CMAX];
#if FQ_AREG
  double av[2][FQ_CMAX];  // the column's scaled dynamics values (FQ_AREG: read once per solve)
#endif
#if FQ_PART
  double vsp[17];         // the variable's spike row (fleet_part.h), reloaded after each factor
  double wsp[17];         // dynamics row 0's: sum_e A[r][e] (spike row of column e)
  int vseg, rseg;         // the segments those spikes belong to
#endif
  int rbn0, rcp0[(FQ_RMAX + 1) / 2];
  __device__ __forceinline__ double &ur(int h) { return h ? P[1] : ur0; }
  __device__ __forceinline__ double &yr(int h) { return h ? yb1 : yr0; }
  __device__ __forceinline__ double &zr(int h) { return h ? zb1 : zr0; }
  __device__ __forceinline__ double &dyr(int h) { return h ? dyb1 : dyr0; }
  __device__ __forceinline__ int &rbn(int h) { return h ? cp[1][3] : rbn0; }
  __device__ __forceinline__ int &rcp(int h, int e) { return h ? cp[1][e] : rcp0[e]; }
  __device__ __forceinline__ int ca(int h, int e) const { return cp[h][e] & 0xffff; }
  __device__ __forceinline__ int cr(int h, int e) const { return cp[h][e] >> 16; }
  __device__ __forceinline__ int rb(int h) { return rbn(h) & 0xffff; }
  __device__ __forceinline__ int rn(int h) { return rbn(h) >> 16; }
  __device__ __forceinline__ int rc(int h, int e) { return (rcp(h, e >> 1) >> (16 * (e & 1))) & 0xffff; }
};
static_assert((FQ_RMAX + 1) / 2 + 1 <= FQ_CMAX, "row slot 1 pattern must fit variable slot 1's");

__device__ __forceinline__ void fq_init_pattern(const QPPattern &pt, FleetRegs &R, int n) {
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    const int j = t + h * FQ_T;
    R.vj[h] = j;
    R.vok[h] = j < n;
    R.cn[h] = 0;
    if (R.vok[h]) {
      const int k0 = pt.colptr[j], k1 = pt.colptr[j + 1] - 1;  // the last entry is the bound row
      R.cn[h] = k1 - k0;
#pragma unroll
      for (int e = 0; e < FQ_CMAX; ++e)  // past the column: the zero pads A[FQ_NNZD], zt[FQ_MD]
        R.cp[h][e] = (e < R.cn[h]) ? (pt.csc2csr[k0 + e] | (pt.cscrow[k0 + e] << 16))
                                   : (FQ_NNZD | (FQ_MD << 16));
    } else {
#pragma unroll
      for (int e = 0; e < FQ_CMAX; ++e) R.cp[h][e] = 0;
    }
    const int r = (FQ_T - 1 - t) + h * FQ_T;
    R.rr[h] = r;
    R.rok[h] = r < FQ_MD;
    if (h == 0 || R.rok[h]) {  // slot 1: only when this thread's second item is a row
      const int rb = R.rok[h] ? pt.rowptr[r] : 0;
      const int rn = R.rok[h] ? pt.rowptr[r + 1] - rb : 0;
      R.rbn(h) = rb | (rn << 16);
#pragma unroll
      for (int e = 0; e < (FQ_RMAX + 1) / 2; ++e) {
        // past the row: column FQ_NMAX - 1, a zero slot of x~ (never written)
        const int c0 = (2 * e < rn) ? pt.colidx[rb + 2 * e] : FQ_NMAX - 1;
        const int c1 = (2 * e + 1 < rn) ? pt.colidx[rb + 2 * e + 1] : FQ_NMAX - 1;
        R.rcp(h, e) = c0 | (c1 << 16);
      }
    }
  }
}

// K-term LDS dot products with all 2K reads in flight at once.  The empty asm
// takes every loaded value as an operand, so the reads issue before it and one
// wait covers them; left alone, the compiler (at the 256-VGPR budget)
// serialises read -> wait -> FMA per term.  Same terms, same order as the
// plain loop.
__device__ __forceinline__ double fq_col_dot(const FleetSmem &s, const FleetRegs &R, int h) {
  static_assert(FQ_CMAX == 6, "fq_col_dot holds 6 terms");
  double a[FQ_CMAX], z[FQ_CMAX];
#pragma unroll
  for (int e = 0; e < FQ_CMAX; ++e) {
#if FQ_AREG
    a[e] = R.av[h][e];
#else
    a[e] = s.A[R.ca(h, e)];
#endif
    z[e] = s.zt[R.cr(h, e)];
  }
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                    "+v"(z[0]), "+v"(z[1]), "+v"(z[2]), "+v"(z[3]), "+v"(z[4]), "+v"(z[5]));
  double acc = 0.0;
#pragma unroll
  for (int e = 0; e < FQ_CMAX; ++e) acc += a[e] * z[e];
  return acc;
}
// both slots' column dot products with all 4K reads in flight at once (FQ_RHS_PAIR)
__device__ __forceinline__ void fq_col_dot2(const FleetSmem &s, const FleetRegs &R, double &d0, double &d1) {
  double a[2][FQ_CMAX], z[2][FQ_CMAX];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < FQ_CMAX; ++e) {
      a[h][e] = s.A[R.ca(h, e)];
      z[h][e] = s.zt[R.cr(h, e)];
    }
  asm volatile("" : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(a[0][2]), "+v"(a[0][3]), "+v"(a[0][4]), "+v"(a[0][5]),
                    "+v"(z[0][0]), "+v"(z[0][1]), "+v"(z[0][2]), "+v"(z[0][3]), "+v"(z[0][4]), "+v"(z[0][5]),
                    "+v"(a[1][0]), "+v"(a[1][1]), "+v"(a[1][2]), "+v"(a[1][3]), "+v"(a[1][4]), "+v"(a[1][5]),
                    "+v"(z[1][0]), "+v"(z[1][1]), "+v"(z[1][2]), "+v"(z[1][3]), "+v"(z[1][4]), "+v"(z[1][5]));
  double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
  for (int e = 0; e < FQ_CMAX; ++e) {
    acc0 += a[0][e] * z[0][e];
    acc1 += a[1][e] * z[1][e];
  }
  d0 = acc0;
  d1 = acc1;
}
__device__ __forceinline__ double fq_row_dot(const FleetSmem &s, FleetRegs &R, int h) {
  static_assert(FQ_RMAX == 5, "fq_row_dot holds 5 terms");
  double a[FQ_RMAX], v[FQ_RMAX];
  const int rb = R.rb(h);
#pragma unroll
  for (int e = 0; e < FQ_RMAX; ++e) {
    a[e] = s.A[rb + e];
    v[e] = s.rhs[R.rc(h, e)];
  }
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]),
                    "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]));
  double acc = 0.0;
#pragma unroll
  for (int e = 0; e < FQ_RMAX; ++e) acc += a[e] * v[e];
  return acc;
}

// scaling.c scale_data over the split storage (qp_device.h qp_scale, same order)
__device__ __forceinline__ void fq_scale(const QPPattern &pt, FleetSmem &s, FleetRegs &R, int iters) {
  const int n = pt.n, tid = threadIdx.x;
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    R.D[h] = 1.0;
    if (R.vok[h]) s.E[FQ_MD + R.vj[h]] = 1.0;
    if (R.rok[h]) s.E[R.rr[h]] = 1.0;
  }
  if (tid == 0) s.c = 1.0;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    // column factors -> rhs (scratch), row factors -> zt (dynamics) / register (bound)
    double eb[2];
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) {
      if (R.vok[h]) {
        double v = fabs(R.P[h]);  // padded entries read the zero A[FQ_NNZD]: fmax(v, 0) = v
        _Pragma("unroll") for (int e = 0; e < FQ_CMAX; ++e) v = fmax(v, fabs(s.A[R.ca(h, e)]));
        v = fmax(v, fabs(R.Ab[h]));
        s.rhs[R.vj[h]] = 1.0 / sqrt(qp_limit(v));
        eb[h] = 1.0 / sqrt(qp_limit(fmax(0.0, fabs(R.Ab[h]))));
      }
      if (R.rok[h]) {
        double v = 0.0;  // all FQ_RMAX reads issue at once (in bounds); entries past the row count 0
        const int rb = R.rb(h), rn = R.rn(h);
        _Pragma("unroll") for (int e = 0; e < FQ_RMAX; ++e) {
          const double a = fabs(s.A[rb + e]);
          v = fmax(v, e < rn ? a : 0.0);
        }
        s.zt[R.rr[h]] = 1.0 / sqrt(qp_limit(v));
      }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) {
      if (R.rok[h]) {
        const double e = s.zt[R.rr[h]];
        _Pragma("unroll") for (int k = 0; k < FQ_RMAX; ++k) if (k < R.rn(h)) {
          const int a = R.rb(h) + k;
          s.A[a] = e * s.A[a] * s.rhs[R.rc(h, k)];
        }
        s.E[R.rr[h]] *= e;
      }
      if (R.vok[h]) {
        const double d = s.rhs[R.vj[h]];
        R.Ab[h] = eb[h] * R.Ab[h] * d;
        s.E[FQ_MD + R.vj[h]] *= eb[h];
      }
    }
    double v[1] = {0.0};
#pragma unroll
    for (int h = 0; h < FQ_H; ++h)
      if (R.vok[h]) {
        const double d = s.rhs[R.vj[h]];
        R.P[h] = d * R.P[h] * d;
        R.q[h] = d * R.q[h];
        R.D[h] *= d;
        v[0] += fabs(R.P[h]);
      }
    double mx[1] = {0.0};
#pragma unroll
    for (int h = 0; h < FQ_H; ++h)
      if (R.vok[h]) mx[0] = fmax(mx[0], fabs(R.q[h]));
    fq_sum_max(v[0], mx[0], s.red);  // (its barriers also order the A / rhs updates above)
    double ct = v[0] / n;
    const double nq = qp_limit(mx[0]);
    ct = qp_limit(fmax(ct, nq));
    ct = 1.0 / ct;
#pragma unroll
    for (int h = 0; h < FQ_H; ++h)
      if (R.vok[h]) { R.P[h] *= ct; R.q[h] *= ct; }
    if (tid == 0) s.c *= ct;
    __syncthreads();
  }
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (R.vok[h]) {
      const double e = s.E[FQ_MD + R.vj[h]];
      R.lb[h] = e * R.lb[h]; R.ub[h] = e * R.ub[h];
    }
    if (R.rok[h]) R.ur(h) = s.E[R.rr[h]] * R.ur(h);
  }
}

// assemble M = P + sigma I + A' R A into the block slots and factor it
// (qp_device.h qp_factor, mode 1).  Diagonal slots are assembled by the owner
// of their variable (its bound row is the slot's last term); the rest by all.
__device__ __forceinline__ int fq_factor(const QPPattern &pt, FleetSmem &s, FleetRegs &R, double sigma,
                                         int cw, QPStamps *T = nullptr) {
  constexpr int SZ = QP_BLK_SZ, BS = SZ * SZ + SZ * QP_BLK_CM;
  const int tid = threadIdx.x;
  const double rs = s.rho_s;
  if (pt.n_offd >= 0) {
    // zero every slot, then the listed non-diagonal slots (<= 3 terms each,
    // packed in one int4, four items in flight per thread); same terms in the
    // same order as the walk below
    for (int e = tid; e < pt.fac_len; e += FQ_T) s.band_store[e] = 0.0;
    __syncthreads();
    const double re = QP_RHO_EQ * rs;
    for (int i0 = tid; i0 < pt.n_offd; i0 += 4 * FQ_T) {
      int4 it[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * FQ_T;
        it[u] = i < pt.n_offd ? pt.offd[i] : make_int4(-1, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (it[u].x < 0) continue;
        const int e = it[u].x & 0x7fff, nt = it[u].x >> 16;
        double v = (it[u].x & 0x8000) ? 1.0 : 0.0;
        if (nt > 0) v += re * s.A[it[u].y & 0xffff] * s.A[it[u].y >> 16];
        if (nt > 1) v += re * s.A[it[u].z & 0xffff] * s.A[it[u].z >> 16];
        if (nt > 2) v += re * s.A[it[u].w & 0xffff] * s.A[it[u].w >> 16];
        s.band_store[e] = v;
      }
    }
  }
  for (int e = tid; pt.n_offd < 0 && e < pt.fac_len; e += FQ_T) {
    const int d = pt.facdiag[e];
    if (d >= 0) continue;
    double v = (d == -2) ? 1.0 : 0.0;
    for (int k = pt.facptr[e]; k < pt.facptr[e + 1]; ++k) {
      const int r = pt.terms[3 * k], a = pt.terms[3 * k + 1], b = pt.terms[3 * k + 2];
      const int h = 0;
      (void)h;
      v += QP_RHO_EQ * rs * s.A[a] * s.A[b];  // off-diagonal terms come from dynamics rows only
      (void)r;
    }
    s.band_store[e] = v;
  }
  // diagonal slot of variable j: P + sigma, then its terms in row order -- the
  // dynamics rows of column j (the owner's column pattern; pads add re * 0 * 0)
  // and last its bound row -- with no pattern reads
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (!R.vok[h]) continue;
    const int j = R.vj[h], e = (j / SZ) * BS + (j % SZ) * (SZ + 1);
    double a[FQ_CMAX];
#pragma unroll
    for (int k = 0; k < FQ_CMAX; ++k) a[k] = s.A[R.ca(h, k)];
    asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]));
    const double re = QP_RHO_EQ * rs;
    double v = R.P[h] + sigma;
#pragma unroll
    for (int k = 0; k < FQ_CMAX; ++k) v += re * a[k] * a[k];
    v += fq_rho(R.lb[h], R.ub[h], rs) * R.Ab[h] * R.Ab[h];
    s.band_store[e] = v;
  }
  if (tid == 0) s.zslot = 0.0;
  if (tid < 64) s.gzero[tid] = 0.0;
  __syncthreads();
  if (T) T->mark(13);
  int f = 0;
#if FQ_PART
  f = fp_factor(s, cw);
#elif FQ_TWIST && !defined(FT_OLD_FACTOR)
  f = ft_factor(s, cw);
#else
  if ((tid >> 6) == cw) f = blk_factor_dispatch(pt, s);
#endif
  if ((tid & 63) == 0 && (tid >> 6) == cw) s.flag = f;  // the chain wave's lane 0 reports
  __syncthreads();
#if FQ_PART
  fp_load_spikes(s, R.vj[0], R.vsp);
  R.vseg = fp_seg(R.vj[0] / FT_SZ);
  {
    int cols[FQ_RMAX];
#pragma unroll
    for (int e = 0; e < FQ_RMAX; ++e) cols[e] = R.rc(0, e);
    R.rseg = fp_load_rowspikes(s, R.rb(0), R.rok[0] ? R.rn(0) : 0, cols, R.wsp);
  }
#endif
  return s.flag;
}

// residual norms (auxil.c update_info) and the rho-estimate quantities in one pass:
// o: 0 pri  1 |z/E|  2 |Ax/E|  3 dua*c  4 |q/D|  5 |A'y/D|  6 |Px/D|
// re: 0 |Ax - z|  1 max(|z|,|Ax|)  2 |q + Px + A'y|  3 max(|q|,|A'y|,|Px|)   (scaled)
__device__ __forceinline__ void fq_update_info(FleetSmem &s, FleetRegs &R, double (&o)[8], double (&re)[4]) {
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (R.vok[h]) s.rhs[R.vj[h]] = R.x[h];
    if (R.rok[h]) s.zt[R.rr[h]] = R.yr(h);
  }
  __syncthreads();
  double v[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (R.rok[h]) {  // dynamics row: (A x)_r
      double ax = 0.0;
      _Pragma("unroll") for (int e = 0; e < FQ_RMAX; ++e) ax += s.A[R.rb(h) + e] * s.rhs[R.rc(h, e)];
      const double e = s.E[R.rr[h]], z = R.zr(h);
      v[0] = fmax(v[0], fabs((ax - z) / e));
      v[1] = fmax(v[1], fabs(z / e));
      v[2] = fmax(v[2], fabs(ax / e));
      v[8] = fmax(v[8], fabs(ax - z));
      v[9] = fmax(v[9], fmax(fabs(z), fabs(ax)));
    }
    if (R.vok[h]) {
      {  // bound row
        const double ax = 0.0 + R.Ab[h] * R.x[h];
        const double e = s.E[FQ_MD + R.vj[h]], z = R.zb_(h);
        v[0] = fmax(v[0], fabs((ax - z) / e));
        v[1] = fmax(v[1], fabs(z / e));
        v[2] = fmax(v[2], fabs(ax / e));
        v[8] = fmax(v[8], fabs(ax - z));
        v[9] = fmax(v[9], fmax(fabs(z), fabs(ax)));
      }
      double aty = 0.0;  // (A' y)_j in CSC order, the bound row last
      _Pragma("unroll") for (int e = 0; e < FQ_CMAX; ++e) aty += s.A[R.ca(h, e)] * s.zt[R.cr(h, e)];
      aty += R.Ab[h] * R.yb_(h);
      const double px = R.P[h] * R.x[h], d = R.D[h], q = R.q[h];
      v[3] = fmax(v[3], fabs((q + px + aty) / d));
      v[4] = fmax(v[4], fabs(q / d));
      v[5] = fmax(v[5], fabs(aty / d));
      v[6] = fmax(v[6], fabs(px / d));
      v[10] = fmax(v[10], fabs(q + px + aty));
      v[11] = fmax(v[11], fmax(fmax(fabs(q), fabs(aty)), fabs(px)));
    }
  }
  fq_max<12>(v, s.red);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = v[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) re[k] = v[8 + k];
}

__device__ __forceinline__ bool fq_primal_infeasible(FleetSmem &s, FleetRegs &R, double eps) {
  double v[1] = {0.0};
  auto proj = [](double d, double l, double u) {
    const bool bu = u > QP_OSQP_INFTY * QP_MIN_SCALING;
    const bool bl = l < -QP_OSQP_INFTY * QP_MIN_SCALING;
    if (bu && bl) return 0.0;
    if (bu) return fmin(d, 0.0);
    if (bl) return fmax(d, 0.0);
    return d;
  };
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (R.rok[h]) {
      R.dyr(h) = proj(R.dyr(h), R.ur(h), R.ur(h));
      v[0] = fmax(v[0], fabs(s.E[R.rr[h]] * R.dyr(h)));
    }
    if (R.vok[h]) {
      R.dyb_(h) = proj(R.dyb_(h), R.lb[h], R.ub[h]);
      v[0] = fmax(v[0], fabs(s.E[FQ_MD + R.vj[h]] * R.dyb_(h)));
    }
  }
  fq_max<1>(v, s.red);
  const double nrm = v[0];
  if (!(nrm > QP_DIV_TOL)) return false;
  double sm[1] = {0.0};
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (R.rok[h]) sm[0] += R.ur(h) * fmax(R.dyr(h), 0.0) + R.ur(h) * fmin(R.dyr(h), 0.0);
    if (R.vok[h]) sm[0] += R.ub[h] * fmax(R.dyb_(h), 0.0) + R.lb[h] * fmin(R.dyb_(h), 0.0);
  }
  fq_sum<1>(sm, s.red);
  if (!(sm[0] < -eps * nrm)) return false;
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
    if (R.rok[h]) s.zt[R.rr[h]] = R.dyr(h);
  __syncthreads();
  double mx[1] = {0.0};
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
    if (R.vok[h]) {
      double acc = 0.0;
      _Pragma("unroll") for (int e = 0; e < FQ_CMAX; ++e) acc += s.A[R.ca(h, e)] * s.zt[R.cr(h, e)];
      acc += R.Ab[h] * R.dyb_(h);
      mx[0] = fmax(mx[0], fabs(acc / R.D[h]));
    }
  fq_max<1>(mx, s.red);
  return mx[0] < eps * nrm;
}

__device__ __forceinline__ bool fq_dual_infeasible(FleetSmem &s, FleetRegs &R, double eps) {
  double v[1] = {0.0};
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
    if (R.vok[h]) v[0] = fmax(v[0], fabs(R.D[h] * R.dx[h]));
  fq_max<1>(v, s.red);
  const double nrm = v[0];
  if (!(nrm > QP_DIV_TOL)) return false;
  double a[1] = {0.0}, pm[1] = {0.0};
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
    if (R.vok[h]) {
      a[0] += R.q[h] * R.dx[h];
      pm[0] = fmax(pm[0], fabs(R.P[h] * R.dx[h] / R.D[h]));
    }
  fq_sum<1>(a, s.red);
  fq_max<1>(pm, s.red);
  if (!(a[0] < s.c * eps * nrm)) return false;
  if (!(pm[0] < s.c * eps * nrm)) return false;
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
    if (R.vok[h]) s.rhs[R.vj[h]] = R.dx[h];
  __syncthreads();
  double bad[1] = {0.0};
  auto test = [&](double vv, double l, double u) {
    if ((u < QP_OSQP_INFTY * QP_MIN_SCALING && vv > eps * nrm) ||
        (l > -QP_OSQP_INFTY * QP_MIN_SCALING && vv < -eps * nrm))
      bad[0] = 1.0;
  };
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (R.rok[h]) {
      double adx = 0.0;
      _Pragma("unroll") for (int e = 0; e < FQ_RMAX; ++e) adx += s.A[R.rb(h) + e] * s.rhs[R.rc(h, e)];
      test(adx / s.E[R.rr[h]], R.ur(h), R.ur(h));
    }
    if (R.vok[h]) test((0.0 + R.Ab[h] * R.dx[h]) / s.E[FQ_MD + R.vj[h]], R.lb[h], R.ub[h]);
  }
  fq_max<1>(bad, s.red);
  return bad[0] == 0.0;
}

__device__ __forceinline__ bool fq_check(FleetSmem &s, FleetRegs &R, const QPSettingsDev &st, const double (&o)[8],
                         bool approx, int &status) {
  const double pri = o[0], dua = o[3] / s.c;
  double ea = st.eps_abs, er = st.eps_rel, epi = st.eps_prim_inf, edi = st.eps_dual_inf;
  if (pri > QP_OSQP_INFTY || dua > QP_OSQP_INFTY) {
    status = -7;
    return true;
  }
  if (approx) { ea *= 10; er *= 10; epi *= 10; edi *= 10; }
  bool prim_ok = false, prim_inf = false, dual_ok = false, dual_inf = false;
  if (pri < ea + er * fmax(o[1], o[2])) prim_ok = true;
  else prim_inf = fq_primal_infeasible(s, R, epi);
  if (dua < ea + er * fmax(fmax(o[4], o[5]), o[6]) / s.c) dual_ok = true;
  else dual_inf = fq_dual_infeasible(s, R, edi);
  if (prim_ok && dual_ok) { status = approx ? 2 : 1; return true; }
  if (prim_inf) { status = approx ? 3 : -3; return true; }
  if (dual_inf) { status = approx ? 4 : -4; return true; }
  return false;
}

__device__ __forceinline__ double fq_rho_estimate(const FleetSmem &s, const double (&re)[4]) {
  const double pr = re[0] / (re[1] + 1e-10);
  const double du = re[2] / (re[3] + 1e-10);
  const double est = s.rho_s * sqrt(pr / (du + 1e-10));
  return fmin(fmax(est, QP_RHO_MIN), QP_RHO_MAX);
}

__device__ __forceinline__ void fq_rebuild_zt(FleetSmem &s, FleetRegs &R) {
  const double rs = s.rho_s;
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (R.rok[h]) s.zt[R.rr[h]] = QP_RHO_EQ * rs * R.zr(h) - R.yr(h);
  }
  __syncthreads();
}

// The solve (qp_device.h qp_solve): on entry R holds the unscaled P, q, l, u,
// bound-row A entries, the warm-start x and the persistent scaled y, s.A the
// unscaled dynamics rows, s.rho_s the persistent rho.  On exit R.x / R.y* hold
// the scaled iterates, R.D / E* and s.c the scaling.
__device__ __forceinline__ QPResult fq_solve(const QPPattern &pt, FleetSmem &s, FleetRegs &R,
                             const QPSettingsDev &st, QPStamps *ts, int cw = 0) {
  const int n = pt.n, tid = threadIdx.x;
  QPResult res{-10, 0, 0.0, 0};
  QPStamps &T = *ts;  // the caller's (no pointer select: a null `out` folds the stamps away)
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    R.lb[h] = fmax(R.lb[h], -QP_OSQP_INFTY); R.ub[h] = fmin(R.ub[h], QP_OSQP_INFTY);
    if (R.rok[h]) R.ur(h) = fmin(fmax(R.ur(h), -QP_OSQP_INFTY), QP_OSQP_INFTY);
  }
  if (tid == 0) {  // the zero pads the padded column patterns point at (fq_init_pattern)
    s.A[FQ_NNZD] = 0.0;
    s.zt[FQ_MD] = 0.0;
  }
  if (st.scaling) fq_scale(pt, s, R, st.scaling);
  else {
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) {
      R.D[h] = 1.0;
      if (R.vok[h]) s.E[FQ_MD + R.vj[h]] = 1.0;
      if (R.rok[h]) s.E[R.rr[h]] = 1.0;
    }
    if (tid == 0) s.c = 1.0;
  }
  // the block solve reads b in whole blocks (plus look-ahead): zero the tail
  for (int j = n + tid; j < FQ_NMAX; j += FQ_T) s.rhs[j] = 0.0;

  if (tid == 0) s.rho_s = fmin(fmax(s.rho_s, QP_RHO_MIN), QP_RHO_MAX);
  __syncthreads();
#if FQ_AREG
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
#pragma unroll
    for (int e = 0; e < FQ_CMAX; ++e) R.av[h][e] = s.A[R.ca(h, e)];
#endif
  T.mark(1);
  int f = fq_factor(pt, s, R, st.sigma, cw);
  T.mark(2);
  if (f) { res.factor_fail = f; return res; }
  if (st.warm_start) {
#pragma unroll
    for (int h = 0; h < FQ_H; ++h)
      if (R.vok[h]) { R.x[h] = R.x[h] / R.D[h]; s.rhs[R.vj[h]] = R.x[h]; }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) {  // z = A x
      if (R.rok[h]) {
        double acc = 0.0;
        _Pragma("unroll") for (int e = 0; e < FQ_RMAX; ++e) acc += s.A[R.rb(h) + e] * s.rhs[R.rc(h, e)];
        R.zr(h) = acc;
      }
      if (R.vok[h]) R.zb_(h) = 0.0 + R.Ab[h] * R.x[h];
    }
  } else {
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) {
      R.x[h] = 0.0; R.zr(h) = 0.0; R.yr(h) = 0.0; R.zb_(h) = 0.0; R.yb_(h) = 0.0;
    }
  }
  __syncthreads();
  const double sig = st.sigma, al = st.alpha;
  fq_rebuild_zt(s, R);
  bool can_check = false;
  int it;
  double o[8], re[4];
  for (it = 1; it <= st.max_iter; ++it) {
#if FQ_LAUNDER & 2
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) asm volatile("" : "+v"(R.vj[h]), "+v"(R.rr[h]));
#endif
    // rhs = sigma x - q + A'(rho z - y)
#if FQ_RHS_PAIR && FQ_T < 256
    {
      double cd[2];
      fq_col_dot2(s, R, cd[0], cd[1]);  // (a slot past n reads the zero pads: harmless)
#pragma unroll
      for (int h = 0; h < FQ_H; ++h)
        if (R.vok[h]) {
          double acc = cd[h];
          acc += R.Ab[h] * (fq_rho(R.lb[h], R.ub[h], s.rho_s) * R.zb_(h) - R.yb_(h));
          s.rhs[R.vj[h]] = sig * R.x[h] - R.q[h] + acc;
        }
    }
#else
#pragma unroll
    for (int h = 0; h < FQ_H; ++h)
      if (R.vok[h]) {
        double acc = fq_col_dot(s, R, h);
        acc += R.Ab[h] * (fq_rho(R.lb[h], R.ub[h], s.rho_s) * R.zb_(h) - R.yb_(h));
        const double rv = sig * R.x[h] - R.q[h] + acc;
        s.rhs[R.vj[h]] = rv;
#if FQ_PART
        s.brhs[R.vj[h]] = rv;
#endif
      }
#endif
    T.mark(11);
    __syncthreads();
    T.mark(3);
#if FQ_PART
    // x~ but the separator correction: the segment chains (wave cw) and the separators'
    // Schur solve beside them (fleet_part.h), LDS-only barriers between; each consumer
    // below subtracts its V x_S itself (fp_corr)
    fp_solve<1>(s, s.rhs, cw);
    T.mark(8);
    lds_sync();
    fp_solve<2>(s, s.rhs, cw);
    T.mark(9);
    lds_sync();
    fp_solve<4>(s, s.rhs, cw);
    T.mark(10);
#elif FQ_TWIST
    // x~: two-ended forward chains (wave cw), diagonal products (both waves),
    // two-ended backward chains (wave cw), LDS-only barriers between
    ft_solve<1>(s, s.rhs, cw);
    T.mark(8);
    lds_sync();
    ft_solve<2>(s, s.rhs, cw);
    T.mark(9);
    lds_sync();
    ft_solve<4>(s, s.rhs, cw);
    T.mark(10);
#elif FQ_DIAG_SPLIT
    // x~: forward chain (wave cw), diagonal products (both waves, eight blocks
    // a round), backward chain (wave cw), LDS-only barriers between
    blk_solve_dispatch<false, FQ_NBLK, 1>(pt, s, s.rhs, &T, cw);
    lds_sync();
    blk_solve_dispatch<false, FQ_NBLK, 2>(pt, s, s.rhs, &T, cw);
    lds_sync();
    blk_solve_dispatch<false, FQ_NBLK, 4>(pt, s, s.rhs, &T, cw);
#else
    blk_solve_dispatch<FQ_FUSED_DIAG, FQ_NBLK>(pt, s, s.rhs, &T, cw);  // x~ (wave cw)
#endif
    __syncthreads();
    T.mark(4);
    const double rs = s.rho_s;
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) {
      if (R.vok[h]) {
#if FQ_PART
        const double xt = s.rhs[R.vj[h]] - fp_corr(s, R.vseg, R.vsp);
#else
        const double xt = s.rhs[R.vj[h]];
#endif
        const double xo = R.x[h];
        const double xn = al * xt + (1.0 - al) * xo;
        R.dx[h] = xn - xo;
        R.x[h] = xn;
        // bound row: z~ = A_b x~_j
        const double ztl = 0.0 + R.Ab[h] * xt;
        const double rho = fq_rho(R.lb[h], R.ub[h], rs), zo = R.zb_(h), yo = R.yb_(h);
        const double zr = al * ztl + (1.0 - al) * zo;
        double zn = zr + yo / rho;
        zn = fmin(fmax(zn, R.lb[h]), R.ub[h]);
        const double d = rho * (zr - zn);
        const double yn = yo + d;
        R.dyb_(h) = d; R.yb_(h) = yn; R.zb_(h) = zn;
      }
      if (R.rok[h]) {
#if FQ_PART
        const double ztl = fq_row_dot(s, R, h) - fp_corr(s, R.rseg, R.wsp);
#else
        const double ztl = fq_row_dot(s, R, h);
#endif
        const double rho = QP_RHO_EQ * rs, zo = R.zr(h), yo = R.yr(h);
        const double zr = al * ztl + (1.0 - al) * zo;
        double zn = zr + yo / rho;
        zn = fmin(fmax(zn, R.ur(h)), R.ur(h));
        const double d = rho * (zr - zn);
        const double yn = yo + d;
        R.dyr(h) = d; R.yr(h) = yn; R.zr(h) = zn;
        s.zt[R.rr[h]] = rho * zn - yn;
      }
    }
    T.mark(12);
    __syncthreads();
    T.mark(5);
    can_check = st.check_termination && (it % st.check_termination == 0);
    const bool adapt = st.adaptive_rho && st.adaptive_rho_interval && (it % st.adaptive_rho_interval == 0);
    if (can_check || adapt) {
      res.iter = it;
      fq_update_info(s, R, o, re);
    }
    if (can_check && fq_check(s, R, st, o, false, res.status)) break;
    if (adapt) {
      const double est = fq_rho_estimate(s, re);
      if (est > s.rho_s * st.adaptive_rho_tolerance || est < s.rho_s / st.adaptive_rho_tolerance) {
        __syncthreads();
        if (tid == 0) s.rho_s = est;
        __syncthreads();
        // at max_iter the loop ends here: rho_s persists and the next solve
        // factors from scratch, so this factorisation would never be used
        if (it < st.max_iter) {
          f = fq_factor(pt, s, R, st.sigma, cw);
          if (f) { res.factor_fail = f; return res; }
        }
      }
    }
    if (can_check || adapt) fq_rebuild_zt(s, R);
    T.mark(6);
  }
  if (!can_check) {
    res.iter = it - 1;
    fq_update_info(s, R, o, re);
    fq_check(s, R, st, o, false, res.status);
  }
  if (res.status == -10) {
    // the residuals of the last check iteration, recomputed from the unchanged
    // iterates (rebuilding rho z - y touches none of them) so that o[] is not
    // live across the iteration loop (register pressure)
    if (can_check) fq_update_info(s, R, o, re);
    if (!fq_check(s, R, st, o, true, res.status)) res.status = -2;
  }
  double ob[1] = {0.0};
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
    if (R.vok[h]) ob[0] += 0.5 * R.x[h] * (R.P[h] * R.x[h]) + R.q[h] * R.x[h];
  fq_sum<1>(ob, s.red);
  res.obj = ob[0] / s.c;
  return res;
}
