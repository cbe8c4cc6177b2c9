// fleet_twist.h -- twisted (two-ended) block factor / solve of the fleet's reduced
// KKT matrix, M block tridiagonal in the 21 stage blocks of SZ = 10 ([x_k, u_k]),
// block k+1 coupled to block k through its first CM = 7 rows (x_{k+1}).
//
// The one-ended recursion of qp_block.h walks 21 blocks per chain.  Here the top
// half (blocks 0..9) is eliminated downwards and the bottom half (blocks 20..11)
// upwards AT THE SAME TIME, by two 16-lane DPP rows of the one chain wave: row 0
// runs the top, row 1 the bottom, with the same instruction stream (the DPP
// row_newbcast broadcasts stay inside each row).  They meet in block 10.  Every
// chain -- the factor sweep, the forward and the backward substitution -- is 10
// block steps instead of 20.
//
//   top    S_0 = M_00,  S_k+1 = M_k+1 - G_k C_k^T,  G_k = C_k S_k^-1       (k < 10)
//   bottom T_20 = M_20, T_k-1 = M_k-1 - K_k^T C_k-1, K_k^T = C_k-1^T T_k^-1 (k > 10)
//   middle Z = M_10 - G_9 C_9^T - K_11^T C_10
//   forward   y_0 = b_0,   y_k+1 = b_k+1 - G_k y_k            (k = 0..9)
//             z_20 = b_20, z_k-1 = b_k-1 - K_k^T z_k          (k = 20..12)
//             z'_10 = - K_11^T z_11
//   diagonal  u_k = S_k^-1 y_k (k < 10), x_10 = Z^-1 (y_10 + z'_10), w_k = T_k^-1 z_k (k > 10)
//   backward  x_k = u_k - G_k^T x_k+1 (k = 9..0),  x_k = w_k - K_k x_k-1 (k = 11..20)
//
// Storage: the assembled M_kk (100, column-major) and C_k (70, 7 rows
// column-major) of block k sit at k * 170 (fleet_qp.h / qp_block.h layout); the
// factor overwrites block k's slots with
//   [0, 55)    S_k^-1 / T_k^-1 / Z^-1, packed lower (row r: r (r + 1) / 2 + c, c <= r)
//   [55, 155)  top: -G_k padded to 10 rows (rows 7..9 zero), bottom: -K_k^T,
//              both column-major: slot 55 + j * 10 + r = (-G_k or -K_k^T)[r][j]
// so both rows read their forward operands at the same immediate offsets, and
// their backward operands ((-G_k)^T and -K_k rows) at the same offsets too.
// Everything a block step reads from another block is consumed before that
// block is overwritten (block k-1's C is read by the bottom's step k, block
// k-1 is rewritten one step later; the middle block last).
#pragma once

#define FT_SZ 10
#define FT_CM 7
#define FT_NB 21
#define FT_MID 10
#define FT_BS (FT_SZ * FT_SZ + FT_SZ * FT_CM)
#define FT_GO 55          // -G / -K^T slots within a block
#define FT_ZS 210         // b scratch for z'_10 (the rhs padding)

__device__ __forceinline__ int ft_tri(int r, int c) { return r >= c ? r * (r + 1) / 2 + c : c * (c + 1) / 2 + r; }

// Gauss-Jordan inverse of the row block held one row per lane (SZ lanes of
// each DPP row); returns the first non-positive pivot (1-based) or 0
__device__ __forceinline__ int ft_gj(double (&a)[FT_SZ], int rr) {
  int bad = 0;
#pragma unroll
  for (int p = 0; p < FT_SZ; ++p) {
    const double piv = bc16_rt(a[p], p);
    if (!(piv > 0.0) && !bad) bad = p + 1;
    const double inv = blk_recip(piv);
    const double f = (rr == p) ? inv - 1.0 : -a[p] * inv;
    fq_gj_update<FT_SZ>(a, f, p);
    a[p] = (rr == p) ? inv : f;
  }
  return bad;
}

// factor (chain wave only): returns 0 or a positive code
template <class S>
__device__ __forceinline__ int ft_factor(S &s, int cw) {
  if ((int)(threadIdx.x >> 6) != cw) return 0;
  const int lane = threadIdx.x & 63, rr = lane & 15;
  const bool top = lane < 16, act = lane < 32 && rr < FT_SZ;
  const int rs = rr < FT_SZ ? rr : FT_SZ - 1, rc = rr < FT_CM ? rr : FT_CM - 1;
  double *F = s.band();
  double u[FT_SZ];  // this lane's row of the pending Schur update of the next block
#pragma unroll
  for (int j = 0; j < FT_SZ; ++j) u[j] = 0.0;
  int bad = 0;
#pragma unroll 1
  for (int t = 0; t < FT_MID; ++t) {
    const int k = top ? t : FT_NB - 1 - t;
    double *Bk = F + k * FT_BS;
    double a[FT_SZ];
#pragma unroll
    for (int j = 0; j < FT_SZ; ++j) a[j] = Bk[j * FT_SZ + rs];
    if (t > 0) {
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j)
        if (!top || (rr < FT_CM && j < FT_CM)) a[j] -= u[j];
    }
    // the coupling operand, before anything of block k is overwritten:
    // top: row rc of C_k;  bottom: column rr of C_k-1 (its 7 rows, zero past them)
    double c[FT_SZ];
    if (top) {
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) c[j] = Bk[FT_SZ * FT_SZ + j * FT_CM + rc];
    } else {
      const double *Cp = F + (k - 1) * FT_BS + FT_SZ * FT_SZ + rs * FT_CM;
#pragma unroll
      for (int l = 0; l < FT_SZ; ++l) c[l] = l < FT_CM ? Cp[l] : 0.0;
    }
    const int b = ft_gj(a, rr);
    if (b && !bad) bad = k * FT_SZ + b;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // every lane's reads of block k done
    if (act) {
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j)
        if (j <= rr) Bk[rr * (rr + 1) / 2 + j] = a[j];
    }
    // top: G row rr = sum_l C[rr][l] S^-1[l][:];  bottom: K^T row rr = sum_l C[l][rr] T^-1[l][:]
    double g[FT_SZ];
#pragma unroll
    for (int j = 0; j < FT_SZ; ++j) g[j] = 0.0;
    blk_gmul<FT_SZ>(g, a, c, std::make_integer_sequence<int, FT_SZ>{});
    if (act) {
      const bool zero = top && rr >= FT_CM;
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) Bk[FT_GO + j * FT_SZ + rr] = zero ? 0.0 : -g[j];
    }
    // next block's update: top u[i] = sum_j G[rr][j] C[i][j] (i < 7 used),
    // bottom u[i] = sum_j K^T[rr][j] C[j][i]
    blk_schur<FT_SZ, FT_SZ>(u, g, c, std::make_integer_sequence<int, FT_SZ>{});
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // middle block: the bottom's update goes through the b scratch (the rhs is
  // rebuilt before every solve)
  double *Sc = s.rhs;
  if (!top && act) {
#pragma unroll
    for (int j = 0; j < FT_SZ; ++j) Sc[rr * FT_SZ + j] = u[j];
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  double *Bm = F + FT_MID * FT_BS;
  double a[FT_SZ];
#pragma unroll
  for (int j = 0; j < FT_SZ; ++j) {
    double v = Bm[j * FT_SZ + rs] - Sc[rs * FT_SZ + j];
    if (rr < FT_CM && j < FT_CM) v -= u[j];  // the top's corner (row 0 lanes' u)
    a[j] = v;
  }
  const int b = ft_gj(a, rr);
  if (top && b && !bad) bad = FT_MID * FT_SZ + b;
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (top && act) {
#pragma unroll
    for (int j = 0; j < FT_SZ; ++j)
      if (j <= rr) Bm[rr * (rr + 1) / 2 + j] = a[j];
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // any lane's failure
  const unsigned long long m = __ballot(act && bad != 0);
  if (!m) return 0;
  return __shfl(bad, __ffsll((long long)m) - 1);
}

// FT_PF2 1: chain operands two block steps ahead (measured 318 us against 314 us
// for the one-step form at 1024 landings: spills 3 -> 9 VGPRs, nothing gained)
#ifndef FT_PF2
#define FT_PF2 0
#endif
// FT_DIAG_UNROLL 1: the diagonal phase's three rounds unrolled, their LDS reads in flight
// together (control kernel 306 -> 293 us at 1024 landings, two runs each, although the
// unrolled rounds' registers raise the kernel's spills 7 -> 54 VGPRs, its scratch traffic
// 19.9 -> 47 MB per launch, L2-resident; a two-deep software pipeline of the rounds spills
// 52 as well; same bits)
#ifndef FT_DIAG_UNROLL
#define FT_DIAG_UNROLL 1
#endif

// init + sum_j g[j] bcast_j(src) (two accumulators, as dot_bc_init), reloading
// g[j] from nx[j * ST] right after its FMA when rl
template <int ST, int... J>
__device__ __forceinline__ double ft_dot_reload(double init, double src, double (&g)[FT_SZ], const double *nx,
                                                bool rl, std::integer_sequence<int, J...>) {
  double a0 = init, a1 = 0.0;
  (((J % 2 == 0 ? fmac_bc<J, J == 0>(a0, src, g[J]) : fmac_bc<J, false>(a1, src, g[J])),
    (rl ? (void)(g[J] = nx[J * ST]) : (void)0)), ...);
  return a0 + a1;
}
template <int ST>
__device__ __forceinline__ double ft_dot_reload(double init, double src, double (&g)[FT_SZ], const double *nx,
                                                bool rl) {
  return ft_dot_reload<ST>(init, src, g, nx, rl, std::make_integer_sequence<int, FT_SZ>{});
}

// b <- M^-1 b, by phases (PH: 1 forward | 2 diagonal | 4 backward).  PH 1 / 4 run
// on the chain wave only; PH 2 on both waves of the workgroup (caller barriers).
template <int PH, class S>
__device__ __forceinline__ void ft_solve(S &s, double *b, int cw) {
  // the diagonal phase's thread index is opaque (its unrolled rounds otherwise keep
  // hoisted addresses live across the loop); the chains keep threadIdx.x, whose wave
  // index the compiler knows to be uniform
  const int tid = PH == 2 ? fq_tid() : (int)threadIdx.x, lane = tid & 63, rr = lane & 15;
  const int rs = rr < FT_SZ ? rr : FT_SZ - 1;
  const double *F = s.band();
  if constexpr (PH == 1 || PH == 4) {
    if ((tid >> 6) != cw || lane >= 32 || rr >= FT_SZ) return;
    const bool top = lane < 16;
    // Block offsets are element indices advanced step by step behind an empty asm:
    // the two rows walk in opposite directions, so a step's address is not an
    // immediate offset from one base, and left alone the compiler hoists all
    // twenty of them out of the ADMM loop as live registers (spilled elsewhere).
#if FT_PF2
    // Two steps ahead: each term's operand for step t + 2 loads right after the
    // term's FMA of step t, into the register it frees (two buffers, as the
    // one-step-ahead form, but twice the latency cover for the LDS reads).
    if constexpr (PH == 1) {
      // top: y over blocks 0..10;  bottom: z over blocks 20..11, then z'_10
      int ib = (top ? 0 : (FT_NB - 1) * FT_SZ) + rs;
      const int db = top ? FT_SZ : -FT_SZ;
      int ig = (top ? 0 : (FT_NB - 1) * FT_BS) + FT_GO + rs;
      const int dg = top ? FT_BS : -FT_BS;
      double y = b[ib];
      double gA[FT_SZ], gB[FT_SZ], cA, cB;
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) { gA[j] = F[ig + j * FT_SZ]; gB[j] = F[ig + dg + j * FT_SZ]; }
      cA = b[ib + db];
      cB = b[ib + 2 * db];
#pragma unroll
      for (int t = 0; t < FT_MID; ++t) {
        double (&g)[FT_SZ] = (t & 1) ? gB : gA;
        double &c = (t & 1) ? cB : cA;
        const double init = (t == FT_MID - 1 && !top) ? 0.0 : c;  // z'_10 = -K_11^T z_11
        const bool rl = t + 2 < FT_MID;
        if (rl) c = b[ib + 3 * db];
        const double yn = ft_dot_reload<FT_SZ>(init, y, g, F + ig + 2 * dg, rl);
        b[ib] = y;
        y = yn;
        ib += db;
        ig += dg;
        asm volatile("" : "+v"(ib), "+v"(ig));
      }
      if (top) b[ib] = y;            // y_10 over b_10
      else b[FT_ZS + rs] = y;        // z'_10
    } else {
      // top: x_9 .. x_0 from x_10;  bottom: x_11 .. x_20
      double x = b[FT_MID * FT_SZ + rs];
      int iu = (top ? (FT_MID - 1) : (FT_MID + 1)) * FT_SZ + rs;
      const int du = top ? -FT_SZ : FT_SZ;
      int ig = (top ? (FT_MID - 1) : (FT_MID + 1)) * FT_BS + FT_GO + rs * FT_SZ;
      const int dg = top ? -FT_BS : FT_BS;
      double gA[FT_SZ], gB[FT_SZ], cA, cB;
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) { gA[j] = F[ig + j]; gB[j] = F[ig + dg + j]; }
      cA = b[iu];
      cB = b[iu + du];
#pragma unroll
      for (int t = 0; t < FT_MID; ++t) {
        double (&g)[FT_SZ] = (t & 1) ? gB : gA;
        double &c = (t & 1) ? cB : cA;
        const double init = c;
        const bool rl = t + 2 < FT_MID;
        if (rl) c = b[iu + 2 * du];
        x = ft_dot_reload<1>(init, x, g, F + ig + 2 * dg, rl);
        b[iu] = x;
        iu += du;
        ig += dg;
        asm volatile("" : "+v"(iu), "+v"(ig));
      }
    }
#else
    if constexpr (PH == 1) {
      // top: y over blocks 0..10;  bottom: z over blocks 20..11, then z'_10
      int ib = (top ? 0 : (FT_NB - 1) * FT_SZ) + rs;
      const int db = top ? FT_SZ : -FT_SZ;
      int ig = (top ? 0 : (FT_NB - 1) * FT_BS) + FT_GO + rs;
      const int dg = top ? FT_BS : -FT_BS;
      double y = b[ib];
      double gA[FT_SZ], gB[FT_SZ], cA, cB;
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) gA[j] = F[ig + j * FT_SZ];
      cA = b[ib + db];
#pragma unroll
      for (int t = 0; t < FT_MID; ++t) {
        double *gc = (t & 1) ? gB : gA, *gn = (t & 1) ? gA : gB;
        double &cc = (t & 1) ? cB : cA, &cn = (t & 1) ? cA : cB;
        if (t + 1 < FT_MID) {
          const int ign = ig + dg;
#pragma unroll
          for (int j = 0; j < FT_SZ; ++j) gn[j] = F[ign + j * FT_SZ];
          cn = b[ib + 2 * db];
        }
        const double init = (t == FT_MID - 1 && !top) ? 0.0 : cc;  // z'_10 = -K_11^T z_11
        const double yn = dot_bc_init<FT_SZ>(init, y, gc);
        b[ib] = y;
        y = yn;
        ib += db;
        ig += dg;
        asm volatile("" : "+v"(ib), "+v"(ig));
      }
      if (top) b[ib] = y;            // y_10 over b_10
      else b[FT_ZS + rs] = y;        // z'_10
    } else {
      // top: x_9 .. x_0 from x_10;  bottom: x_11 .. x_20
      double x = b[FT_MID * FT_SZ + rs];
      int iu = (top ? (FT_MID - 1) : (FT_MID + 1)) * FT_SZ + rs;
      const int du = top ? -FT_SZ : FT_SZ;
      int ig = (top ? (FT_MID - 1) : (FT_MID + 1)) * FT_BS + FT_GO + rs * FT_SZ;
      const int dg = top ? -FT_BS : FT_BS;
      double gA[FT_SZ], gB[FT_SZ], cA, cB;
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) gA[j] = F[ig + j];
      cA = b[iu];
#pragma unroll
      for (int t = 0; t < FT_MID; ++t) {
        double *gc = (t & 1) ? gB : gA, *gn = (t & 1) ? gA : gB;
        double &cc = (t & 1) ? cB : cA, &cn = (t & 1) ? cA : cB;
        if (t + 1 < FT_MID) {
          const int ign = ig + dg;
#pragma unroll
          for (int j = 0; j < FT_SZ; ++j) gn[j] = F[ign + j];
          cn = b[iu + du];
        }
        x = dot_bc_init<FT_SZ>(cc, x, gc);
        b[iu] = x;
        iu += du;
        ig += dg;
        asm volatile("" : "+v"(iu), "+v"(ig));
      }
    }
#endif
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  } else {
    // diagonal: u_k / x_10 / w_k, eight blocks a round (one per DPP row of
    // either wave); rows past the last block read the last block and do not store
    const int q = tid >> 4;
    constexpr int RB = FQ_T / 16, NR = (FT_NB + RB - 1) / RB;
#if FT_DIAG_UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int t = 0; t < NR; ++t) {
      const int kk = RB * t + q, k = kk < FT_NB ? kk : FT_NB - 1;
      const double *Sk = F + k * FT_BS;
      // packed row rs: (rs, j) at rs (rs + 1) / 2 + j for j <= rs, else j (j + 1) / 2 + rs
      const double *pr = Sk + rs * (rs + 1) / 2, *pc = Sk + rs;
      double sv[FT_SZ];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) sv[j] = j <= rs ? pr[j] : pc[j * (j + 1) / 2];
      double y = b[k * FT_SZ + rs];
      if (k == FT_MID) y += b[FT_ZS + rs];
      const double v = dot_bc<FT_SZ>(y, sv);
      if (kk < FT_NB && rr < FT_SZ) b[kk * FT_SZ + rr] = v;
    }
  }
}
