// fleet_part.h -- partitioned (nested-dissection) factor / solve of the fleet's reduced KKT
// matrix for the wide control build (fleet_wide.hip: one landing per CU, 256 threads, LDS
// to spare).  M is block tridiagonal in the 21 stage blocks of SZ = 10 ([x_k, u_k]), block
// k+1 coupled to block k through its first CM = 7 rows (x_{k+1}): C_k = M[k+1][k] (7 x 10).
//
// The twisted solve (fleet_twist.h) walks two chains of 10 block steps.  Here blocks 5, 10
// and 15 are separators and the 18 blocks between them four independent segments,
//   A = 0..4 (top-down)  B = 6..9 (top-down)  C = 11..14 (top-down)  D = 20..16 (bottom-up),
// one per 16-lane DPP row of the chain wave, so every chain is at most 4 block steps.
// With I the segment blocks and S the separators (30 unknowns):
//   spikes   V = M_II^-1 M_IS          per segment block k: L_k (10 x 10, the coupling to the
//                                      separator left of its segment) and R_k (10 x 7, right)
//   Schur    Shat = M_SS - M_SI V      (30 x 30, SPD), kept as its inverse
//   solve    z_I = M_II^-1 b_I         (segment chains: forward, diagonal, backward)
//            bhat_S = b_S - M_SI z_I   (the separators' neighbour blocks; the two whose z
//                                      the backward chains finish last through their spikes,
//                                      beside the forward chains)
//            x_S = Shat^-1 bhat_S      (beside the backward chains)
//            x_I = z_I - V x_S         (every variable's owner, its spike row in registers)
// so one ADMM iteration's substitution is 4 + 4 dependent block steps instead of 10 + 10.
//
// Storage: the factor area keeps the twisted layout per segment block (fleet_twist.h): the
// block's S^-1 packed lower at [0, 55), -G_k (top-down) / -K_k^T (bottom-up) at [55, 155);
// a segment's last block keeps its coupling to the separator (C_k at [100, 170)), which
// the spikes and Shat read.  Separator blocks keep M_ss and C_s as assembled.  Spikes in
// spk, column-major (a column's 10 rows contiguous: the per-iteration readers take a
// column per lane, or a row per lane across consecutive lanes, without bank conflicts):
// block k's L_k[r][c] at k * 170 + c * 10 + r, R_k[r][c] at k * 170 + 100 + c * 10 + r.
#pragma once

#define FP_SPK (FT_NB * FT_BS)
#define FP_NS 30                // separator unknowns: blocks 5, 10, 15

// section timestamps of fp_factor (scripts/hip/fp_probe.hip defines it)
#ifndef FP_MARK
#define FP_MARK(k)
#endif

// segment q: its first block in elimination order, its length and direction
__device__ __forceinline__ int fp_k0(int q) { return q == 0 ? 0 : q == 1 ? 6 : q == 2 ? 11 : 20; }
__device__ __forceinline__ int fp_len(int q) { return (q == 0 || q == 3) ? 5 : 4; }
// the lowest-numbered block of segment q, and the segment's separators (block numbers)
__device__ __forceinline__ int fp_lo(int q) { return q == 0 ? 0 : q == 1 ? 6 : q == 2 ? 11 : 16; }
// interior block idx (0..17) -> block number
__device__ __forceinline__ int fp_iblk(int idx) { return idx + (idx >= 5) + (idx >= 9) + (idx >= 13); }

// 10-wide DPP product of the row block held one row per lane: out[c] = init[c] + sum_j
// m[j] bcast_j(v[c]) for c < NC (two accumulators per column, dot_bc_init's order)
template <int NC>
__device__ __forceinline__ void fp_rowmul(double (&out)[10], const double (&init)[10], const double (&m)[10],
                                          const double (&v)[10]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) out[c] = dot_bc_init<FT_SZ>(init[c], v[c], m);
}

// Factor: segment chains, spikes, Shat^-1.  Chain wave only (the caller barriers after);
// returns 0 or a positive code (the first non-positive pivot's block * 10 + row + 1).
template <class S>
__device__ __forceinline__ int fp_factor(S &s, int cw) {
  if ((int)(threadIdx.x >> 6) != cw) return 0;
  const int lane = threadIdx.x & 63, rr = lane & 15, q = lane >> 4;
  const bool top = q < 3, act = rr < FT_SZ;
  const int rs = rr < FT_SZ ? rr : FT_SZ - 1, rc = rr < FT_CM ? rr : FT_CM - 1;
  const int k0 = fp_k0(q), L = fp_len(q), dir = top ? 1 : -1;
  double *F = s.band();
  double *spk = s.spk;
  int bad = 0;
  FP_MARK(0);
  // ---- segment factor: the twisted factor's top (rows 0-2) / bottom (row 3) recursion
  {
    double u[FT_SZ];
#pragma unroll
    for (int j = 0; j < FT_SZ; ++j) u[j] = 0.0;
#pragma unroll 1
    for (int t = 0; t < 5; ++t) {
      const bool on = t < L, cpl = t + 1 < L;  // cpl: the next block is in the segment
      const int k = k0 + dir * (on ? t : L - 1);  // a finished row re-reads its last block, stores nothing
      double *Bk = F + k * FT_BS;
      double a[FT_SZ];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) a[j] = Bk[j * FT_SZ + rs];
      if (t > 0) {
#pragma unroll
        for (int j = 0; j < FT_SZ; ++j)
          if (!top || (rr < FT_CM && j < FT_CM)) a[j] -= u[j];
      }
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
      if (on && b && !bad) bad = k * FT_SZ + b;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (on && act) {
#pragma unroll
        for (int j = 0; j < FT_SZ; ++j)
          if (j <= rr) Bk[rr * (rr + 1) / 2 + j] = a[j];
      }
      double g[FT_SZ];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) g[j] = 0.0;
      blk_gmul<FT_SZ>(g, a, c, std::make_integer_sequence<int, FT_SZ>{});
      // a segment's last block keeps C_k (its coupling to the separator) in [100, 170)
      if (on && cpl && act) {
        const bool zero = top && rr >= FT_CM;
#pragma unroll
        for (int j = 0; j < FT_SZ; ++j) Bk[FT_GO + j * FT_SZ + rr] = zero ? 0.0 : -g[j];
      }
      blk_schur<FT_SZ, FT_SZ>(u, g, c, std::make_integer_sequence<int, FT_SZ>{});
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  FP_MARK(1);
  // ---- spikes.  The start spike (rows 1, 2: the left separator's coupling C_sep at the
  // segment's first block) needs the forward chain: y_0 = E, y_t = -G y_t-1, and u_t =
  // S^-1 y_t, parked in the L slots; the end spike (every row: at the segment's last block,
  // R for rows 0-2 = C_b^T, L for row 3 = C_15) starts with S_b^-1 E.  Then one backward
  // chain carries both: v_k = u_k + (-G_k)^T v_k+1 (start), w_k = (-G_k)^T w_k+1 (end).
  const bool has_start = q == 1 || q == 2;
  const int sep_l = q == 1 ? 5 : 10;  // (rows 1, 2)
  {
    double y[FT_SZ], u[FT_SZ], z[FT_SZ];
#pragma unroll
    for (int c = 0; c < FT_SZ; ++c) {
      z[c] = 0.0;
      y[c] = rr < FT_CM ? F[sep_l * FT_BS + FT_SZ * FT_SZ + c * FT_CM + rc] : 0.0;  // C_sep[rr][c]
    }
#pragma unroll 1
    for (int t = 0; t < 4; ++t) {
      const int k = k0 + dir * t;  // rows 1, 2 only (rows 0, 3 compute on their own blocks, store nothing)
      if (t > 0) {
        double g[FT_SZ];
        const double *gp = F + (k - dir) * FT_BS + FT_GO + rs;  // (-G_k-1)[rs][j] at j * 10
#pragma unroll
        for (int j = 0; j < FT_SZ; ++j) g[j] = gp[j * FT_SZ];
        double yn[FT_SZ];
        fp_rowmul<FT_SZ>(yn, z, g, y);
#pragma unroll
        for (int c = 0; c < FT_SZ; ++c) y[c] = yn[c];
      }
      const double *Sk = F + k * FT_BS;
      const double *pr = Sk + rs * (rs + 1) / 2, *pc = Sk + rs;
      double sv[FT_SZ];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) sv[j] = j <= rs ? pr[j] : pc[j * (j + 1) / 2];
      fp_rowmul<FT_SZ>(u, z, sv, y);
      if (has_start && act) {
#pragma unroll
        for (int c = 0; c < FT_SZ; ++c) spk[k * FT_BS + c * FT_SZ + rr] = u[c];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  FP_MARK(2);
  {
    const int kb = k0 + dir * (L - 1);  // the segment's last block
    const double *Bb = F + kb * FT_BS;
    double e[FT_SZ], w[FT_SZ], v[FT_SZ], z[FT_SZ];
#pragma unroll
    for (int c = 0; c < FT_SZ; ++c) {
      z[c] = 0.0;
      if (top) e[c] = c < FT_CM ? Bb[FT_SZ * FT_SZ + rs * FT_CM + c] : 0.0;       // C_b[c][rr]
      else e[c] = rr < FT_CM ? F[15 * FT_BS + FT_SZ * FT_SZ + c * FT_CM + rc] : 0.0;  // C_15[rr][c]
    }
    {
      const double *pr = Bb + rs * (rs + 1) / 2, *pc = Bb + rs;
      double sv[FT_SZ];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) sv[j] = j <= rs ? pr[j] : pc[j * (j + 1) / 2];
      fp_rowmul<FT_SZ>(w, z, sv, e);
    }
#pragma unroll
    for (int c = 0; c < FT_SZ; ++c) v[c] = has_start ? spk[kb * FT_BS + c * FT_SZ + rs] : 0.0;
    auto store = [&](int k) {
      if (!act) return;
      if (top) {
#pragma unroll
        for (int c = 0; c < FT_CM; ++c) spk[k * FT_BS + FT_SZ * FT_SZ + c * FT_SZ + rr] = w[c];
        if (has_start) {
#pragma unroll
          for (int c = 0; c < FT_SZ; ++c) spk[k * FT_BS + c * FT_SZ + rr] = v[c];
        } else {
#pragma unroll
          for (int c = 0; c < FT_SZ; ++c) spk[k * FT_BS + c * FT_SZ + rr] = 0.0;   // segment A: no L
        }
      } else {
#pragma unroll
        for (int c = 0; c < FT_SZ; ++c) spk[k * FT_BS + c * FT_SZ + rr] = w[c];
#pragma unroll
        for (int c = 0; c < FT_CM; ++c) spk[k * FT_BS + FT_SZ * FT_SZ + c * FT_SZ + rr] = 0.0;  // D: no R
      }
    };
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // the u_b reads above before the stores
    store(kb);
#pragma unroll 1
    for (int t = 1; t < 5; ++t) {
      const bool on = t < L;
      const int k = kb - dir * (on ? t : L - 1);
      double g[FT_SZ];
      const double *gp = F + k * FT_BS + FT_GO + rs * FT_SZ;  // (-G_k)[j][rs] / (-K_k^T)[j][rs]
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) g[j] = gp[j];
      double wn[FT_SZ], vn[FT_SZ], ui[FT_SZ];
#pragma unroll
      for (int c = 0; c < FT_SZ; ++c) ui[c] = has_start ? spk[k * FT_BS + c * FT_SZ + rs] : 0.0;
      fp_rowmul<FT_SZ>(wn, z, g, w);
      fp_rowmul<FT_SZ>(vn, ui, g, v);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (on) {
#pragma unroll
        for (int c = 0; c < FT_SZ; ++c) { w[c] = wn[c]; v[c] = vn[c]; }
        store(k);
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  FP_MARK(3);
  // ---- Shat = M_SS - M_SI V, lane i < 30 its row (separator sg = i / 10, component r)
  double a[FP_NS];
  const int sg = lane / FT_SZ, r = lane % FT_SZ, sb = 5 + 5 * sg;
  const bool srow = lane < FP_NS;
  {
    const int sgc = srow ? sg : 0, sbc = 5 + 5 * sgc;
#pragma unroll
    for (int j = 0; j < FP_NS; ++j) a[j] = 0.0;
#pragma unroll
    for (int j = 0; j < FT_SZ; ++j) {
      const double m = F[sbc * FT_BS + j * FT_SZ + r];
#pragma unroll
      for (int g = 0; g < 3; ++g)
        if (g == sgc) a[10 * g + j] = m;
    }
    // left neighbour kl = sb - 1 (last block of segment sg): M[sb][kl] = C_kl (rows r < 7);
    // right neighbour kr = sb + 1 (first block of segment sg + 1): M[sb][kr] = C_sb^T.
    // Row-wise products: spike row l (contiguous) times the coupling's l-th element
    const int kl = sbc - 1, kr = sbc + 1;
    double cl[FT_SZ], cr[FT_CM];
#pragma unroll
    for (int l = 0; l < FT_SZ; ++l) cl[l] = r < FT_CM ? F[kl * FT_BS + FT_SZ * FT_SZ + l * FT_CM + r] : 0.0;
#pragma unroll
    for (int l = 0; l < FT_CM; ++l) cr[l] = F[sbc * FT_BS + FT_SZ * FT_SZ + r * FT_CM + l];  // C_sb[l][r]
    double tR[FT_CM], tL[FT_SZ], uL[FT_SZ], uR[FT_CM];
#pragma unroll
    for (int j = 0; j < FT_SZ; ++j) { tL[j] = 0.0; uL[j] = 0.0; }
#pragma unroll
    for (int j = 0; j < FT_CM; ++j) { tR[j] = 0.0; uR[j] = 0.0; }
#pragma unroll
    for (int l = 0; l < FT_SZ; ++l) {
      double rv[FT_CM], lv[FT_SZ];
#pragma unroll
      for (int j = 0; j < FT_CM; ++j) rv[j] = spk[kl * FT_BS + FT_SZ * FT_SZ + j * FT_SZ + l];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) lv[j] = spk[kl * FT_BS + j * FT_SZ + l];
#pragma unroll
      for (int j = 0; j < FT_CM; ++j) tR[j] = fma(cl[l], rv[j], tR[j]);   // C_kl R_kl
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) tL[j] = fma(cl[l], lv[j], tL[j]);   // C_kl L_kl
    }
#pragma unroll
    for (int l = 0; l < FT_CM; ++l) {
      double lv[FT_SZ], rv[FT_CM];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) lv[j] = spk[kr * FT_BS + j * FT_SZ + l];
#pragma unroll
      for (int j = 0; j < FT_CM; ++j) rv[j] = spk[kr * FT_BS + FT_SZ * FT_SZ + j * FT_SZ + l];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) uL[j] = fma(cr[l], lv[j], uL[j]);   // C_sb^T L_kr
#pragma unroll
      for (int j = 0; j < FT_CM; ++j) uR[j] = fma(cr[l], rv[j], uR[j]);   // C_sb^T R_kr
    }
#pragma unroll
    for (int g = 0; g < 3; ++g) {
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) {
        if (g == sgc) a[10 * g + j] = (a[10 * g + j] - (j < FT_CM ? tR[j] : 0.0)) - uL[j];
        if (g == sgc - 1) a[10 * g + j] -= tL[j];                    // (segment sg has a left separator)
        if (g == sgc + 1 && j < FT_CM) a[10 * g + j] -= uR[j];       // (segment sg + 1 has a right one)
      }
    }
  }
  FP_MARK(4);
  // ---- Shat^-1 by Gauss-Jordan (SPD, no pivoting: the ft_gj step), the pivot row through
  // LDS (two alternating buffers: a step's stores never overtake the previous step's reads)
  {
    double *pb = s.bh;  // 2 x 32 scratch
#pragma unroll
    for (int p = 0; p < FP_NS; ++p) {
      double *buf = pb + (p & 1) * 32;
      if (lane == p) {
#pragma unroll
        for (int j = 0; j < FP_NS; ++j) buf[j] = a[j];
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      double prow[FP_NS];
#pragma unroll
      for (int j = 0; j < FP_NS; ++j) prow[j] = buf[j];
      const double piv = prow[p];
      if (srow && lane == p && !(piv > 0.0) && !bad) bad = sb * FT_SZ + r + 1;
      const double inv = blk_recip(piv);
      const double f = (lane == p) ? inv - 1.0 : -a[p] * inv;
#pragma unroll
      for (int j = 0; j < FP_NS; ++j)
        if (j != p) a[j] = fma(prow[j], f, a[j]);
      a[p] = (lane == p) ? inv : f;
    }
    if (srow) {
#pragma unroll
      for (int j = 0; j < FP_NS; ++j) s.sinv[lane * FP_NS + j] = a[j];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  FP_MARK(5);
  const unsigned long long m = __ballot(bad != 0);
  if (!m) return 0;
  return __shfl(bad, __ffsll((long long)m) - 1);
}

// The spike row of variable j (block j / 10, row j % 10) into registers: its L_k row
// (10, zeros in segment A) then its R_k row (7, zeros in segment D); zeros for the
// separators' and the padding's rows.  Loaded by every variable's owner after each factor.
template <class S>
__device__ __forceinline__ void fp_load_spikes(const S &s, int j, double (&vsp)[17]) {
  const int k = j / FT_SZ, r = j % FT_SZ;
  const bool in = j < FT_NB * FT_SZ && k != 5 && k != 10 && k != 15;
  const double *sp = s.spk + (in ? k : 0) * FT_BS + r;
#pragma unroll
  for (int c = 0; c < FT_SZ; ++c) vsp[c] = in ? sp[c * FT_SZ] : 0.0;
#pragma unroll
  for (int c = 0; c < FT_CM; ++c) vsp[FT_SZ + c] = in ? sp[FT_SZ * FT_SZ + c * FT_SZ] : 0.0;
}

// b <- M^-1 b by phases (the caller barriers between them):
//  PH 1  chain wave: each segment's forward chain y (one DPP row each).  The other three
//        waves: bhat_S's terms that only a finished backward chain would give otherwise --
//        the middle segments' first blocks (6, 11) couple to separators 5 and 10 -- as
//        spike products L_k^T b_k over those segments (= C_s^T z_(s+1)), from brhs, the
//        copy of b the right-hand side phase leaves (b itself is being overwritten);
//  PH 2  every wave: the segment blocks' diagonal products u = S^-1 y (z of each segment's
//        last block, 4, 9, 14, 16, is final from here on); then the next wave (w1, which
//        formed those four) bhat_S = b_S - M_SI z_I from them and the partial sums;
//  PH 4  chain wave: the backward chains z = u - G^T z'.  Beside them, w1:
//        x_S = Shat^-1 bhat_S, written over b_S.
// The caller applies x_I = z_I - V x_S where x~ is consumed (fp_corr): no further phase.
template <int PH, class S>
__device__ __forceinline__ void fp_solve(S &s, double *b, int cw) {
  const int tid = threadIdx.x, lane = tid & 63, rr = lane & 15, q = lane >> 4, wv = tid >> 6;
  const int rs = rr < FT_SZ ? rr : FT_SZ - 1;
  const double *F = s.band();
  const double *spk = s.spk;
  if constexpr (PH == 1) {
    if (wv == cw) {
      if (rr >= FT_SZ) return;
      const bool top = q < 3;
      const int k0 = fp_k0(q), L = fp_len(q);
      const int db = top ? FT_SZ : -FT_SZ, dg = top ? FT_BS : -FT_BS;
      int ib = k0 * FT_SZ + rs, ig = k0 * FT_BS + FT_GO + rs;
      double y = b[ib];
      double gA[FT_SZ], gB[FT_SZ], cA, cB;
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) gA[j] = F[ig + j * FT_SZ];
      cA = b[ib + db];
#pragma unroll
      for (int t = 0; t < 4; ++t) {  // up to 4 steps; segments of 4 blocks stop after 3
        double *gc = (t & 1) ? gB : gA, *gn = (t & 1) ? gA : gB;
        double &cc = (t & 1) ? cB : cA, &cn = (t & 1) ? cA : cB;
        const bool on = t + 1 < L;
        if (t + 1 < 4) {
          const int ign = on ? ig + dg : ig;
#pragma unroll
          for (int j = 0; j < FT_SZ; ++j) gn[j] = F[ign + j * FT_SZ];
          cn = b[on && t + 2 < L ? ib + 2 * db : ib];
        }
        const double yn = dot_bc_init<FT_SZ>(cc, y, gc);
        if (on) {
          b[ib] = y;
          y = yn;
          ib += db;
          ig += dg;
        }
        asm volatile("" : "+v"(ib), "+v"(ig));
      }
      b[ib] = y;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    } else {
      // item j = seg * 40 + c * 4 + i: sum_r L_k[r][c] b_k[r], k block i of segment B (seg 0,
      // separator 5) or C (seg 1, separator 10)
      const int j = ((wv - cw - 1) & 3) * 64 + lane;
      if (j >= 80) return;
      const int sgm = j / 40, c = (j / 4) % FT_SZ, k = (sgm ? 11 : 6) + j % 4;
      const double *sp = spk + k * FT_BS + c * FT_SZ, *bk = s.brhs + k * FT_SZ;
      double sv[FT_SZ], bv[FT_SZ];
#pragma unroll
      for (int rw = 0; rw < FT_SZ; ++rw) { sv[rw] = sp[rw]; bv[rw] = bk[rw]; }
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int rw = 0; rw < FT_SZ; rw += 2) {
        a0 = fma(sv[rw], bv[rw], a0);
        a1 = fma(sv[rw + 1], bv[rw + 1], a1);
      }
      s.part[j] = a0 + a1;
    }
  } else if constexpr (PH == 2) {
    // the 18 segment blocks' S^-1 y products, one per DPP row: round 1 sixteen blocks,
    // the next wave (w1) taking the four whose z bhat_S needs (4, 9, 14, 16: the last blocks
    // of their segments, final from here on); round 2 the last two, on the chain wave.
    // Then w1 forms bhat_S = b_S - M_SI z_I: lane pair (o, h), h = 0 C_(s-1) z_(s-1)
    // (components < 7), h = 1 the right neighbour's term -- the spike partial sums of
    // segments B / C for separators 5 / 10, C_15^T z_16 for 15
    const int d = (wv - cw) & 3, rq = (tid >> 4) & 3;
    const int tab[16] = {0, 1, 2, 3, 4, 9, 14, 16, 6, 7, 8, 11, 12, 13, 17, 18};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (t == 1 && (d != 0 || rq >= 2)) break;
      const int k = t == 0 ? tab[d * 4 + rq] : 19 + rq;
      const double *Sk = F + k * FT_BS;
      const double *pr = Sk + rs * (rs + 1) / 2, *pc = Sk + rs;
      double sv[FT_SZ];
#pragma unroll
      for (int j = 0; j < FT_SZ; ++j) sv[j] = j <= rs ? pr[j] : pc[j * (j + 1) / 2];
      const double y = b[k * FT_SZ + rs];
      const double v = dot_bc<FT_SZ>(y, sv);
      if (rr < FT_SZ) b[k * FT_SZ + rr] = v;
    }
    if (d != 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const int o = lane >> 1, h = lane & 1, oc = o < FP_NS ? o : 0, sg = oc / FT_SZ, c = oc % FT_SZ;
    const int sb = 5 + 5 * sg;
    double part;
    {
      double cv[FT_SZ], zv[FT_SZ];
      if (h == 0) {
        const double *cp = F + (sb - 1) * FT_BS + FT_SZ * FT_SZ + (c < FT_CM ? c : 0);
#pragma unroll
        for (int l = 0; l < FT_SZ; ++l) { cv[l] = c < FT_CM ? cp[l * FT_CM] : 0.0; zv[l] = b[(sb - 1) * FT_SZ + l]; }
      } else if (sg == 2) {
        const double *cp = F + sb * FT_BS + FT_SZ * FT_SZ + c * FT_CM;
#pragma unroll
        for (int l = 0; l < FT_SZ; ++l) { cv[l] = l < FT_CM ? cp[l] : 0.0; zv[l] = l < FT_CM ? b[(sb + 1) * FT_SZ + l] : 0.0; }
      } else {
        const double *pp = s.part + sg * 40 + c * 4;
#pragma unroll
        for (int l = 0; l < FT_SZ; ++l) { cv[l] = l < 4 ? 1.0 : 0.0; zv[l] = l < 4 ? pp[l] : 0.0; }
      }
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int l = 0; l < FT_SZ; l += 2) {
        a0 = fma(cv[l], zv[l], a0);
        a1 = fma(cv[l + 1], zv[l + 1], a1);
      }
      part = a0 + a1;
    }
    const double other = __shfl_xor(part, 1);
    if (o < FP_NS && h == 0) s.bh[o] = (b[sb * FT_SZ + c] - part) - other;
  } else {
    if (wv == ((cw + 1) & 3)) {
      // beside the backward chains: x_S = Shat^-1 bhat_S, lane pair (i, h) sums the
      // columns [15 h, 15 h + 15) of row i; written over b_S
      const int o = lane >> 1, h = lane & 1, oc = o < FP_NS ? o : 0, sg = oc / FT_SZ, c = oc % FT_SZ;
      const double *si = s.sinv + oc * FP_NS + 15 * h, *bv = s.bh + 15 * h;
      double sr[15], br[15];
#pragma unroll
      for (int j = 0; j < 15; ++j) { sr[j] = si[j]; br[j] = bv[j]; }
      double x0 = 0.0, x1 = 0.0;
#pragma unroll
      for (int j = 0; j < 14; j += 2) {
        x0 = fma(sr[j], br[j], x0);
        x1 = fma(sr[j + 1], br[j + 1], x1);
      }
      x0 = fma(sr[14], br[14], x0);
      const double xp = x0 + x1;
      const double xo = __shfl_xor(xp, 1);
      if (o < FP_NS && h == 0) {
        const double xs = xp + xo;
        s.xs[o] = xs;
        b[(5 + 5 * sg) * FT_SZ + c] = xs;
      }
      return;
    }
    if (wv != cw || rr >= FT_SZ) return;
    const bool top = q < 3;
    const int k0 = fp_k0(q), L = fp_len(q);
    const int kb = top ? k0 + L - 1 : k0 - (L - 1);
    const int du = top ? -FT_SZ : FT_SZ, dg = top ? -FT_BS : FT_BS;
    double x = b[kb * FT_SZ + rs];
    int iu = kb * FT_SZ + du + rs;
    int ig = kb * FT_BS + dg + FT_GO + rs * FT_SZ;
    double gA[FT_SZ], gB[FT_SZ], cA, cB;
#pragma unroll
    for (int j = 0; j < FT_SZ; ++j) gA[j] = F[ig + j];
    cA = b[iu];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      double *gc = (t & 1) ? gB : gA, *gn = (t & 1) ? gA : gB;
      double &cc = (t & 1) ? cB : cA, &cn = (t & 1) ? cA : cB;
      const bool on = t + 1 < L;
      if (t + 1 < 4) {
        const bool nx = t + 2 < L;
        const int ign = nx ? ig + dg : ig;
#pragma unroll
        for (int j = 0; j < FT_SZ; ++j) gn[j] = F[ign + j];
        cn = b[nx ? iu + du : iu];
      }
      const double xn = dot_bc_init<FT_SZ>(cc, x, gc);
      if (on) {
        x = xn;
        b[iu] = x;
        iu += du;
        ig += dg;
      }
      asm volatile("" : "+v"(iu), "+v"(ig));
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
}

// The separator correction V x_S of one consumer (fp_correct_value): v is a spike row
// (fp_load_spikes) or a dynamics row's product with its columns' spike rows
// (fp_load_rowspikes), both against the separators of segment qs: the L part (10) the
// one left of it, the R part (7) the one right of it.  x_S read as 16-byte pairs.
template <class S>
__device__ __forceinline__ double fp_corr(const S &s, int qs, const double (&v)[17]) {
  const double2 *xl = (const double2 *)(s.xs + (qs >= 1 ? qs - 1 : 0) * FT_SZ);
  const double2 *xr = (const double2 *)(s.xs + (qs <= 2 ? qs : 2) * FT_SZ);
  double2 l2[5], r2[4];
#pragma unroll
  for (int c = 0; c < 5; ++c) l2[c] = xl[c];
#pragma unroll
  for (int c = 0; c < 4; ++c) r2[c] = xr[c];
  double acc[4] = {0.0, 0.0, 0.0, 0.0};   // (segment A's L and D's R parts are zeros)
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    acc[(2 * c) & 3] = fma(v[2 * c], l2[c].x, acc[(2 * c) & 3]);
    acc[(2 * c + 1) & 3] = fma(v[2 * c + 1], l2[c].y, acc[(2 * c + 1) & 3]);
  }
#pragma unroll
  for (int c = 0; c < FT_CM; ++c) {
    const double xv = (c & 1) ? r2[c >> 1].y : r2[c >> 1].x;
    acc[(c + 2) & 3] = fma(v[FT_SZ + c], xv, acc[(c + 2) & 3]);
  }
  return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// the segment (0..3) of variable j's block, or that of a dynamics row's non-separator block
__device__ __forceinline__ int fp_seg(int k) { return (k > 5) + (k > 10) + (k > 15); }

// A dynamics row's correction vector: sum over its columns e of A[r][e] times column e's
// spike row (separator columns have none), and the segment those spikes belong to (a row
// couples blocks k, k + 1: at most one of them is a segment block's... or both of one segment)
template <class S>
__device__ __forceinline__ int fp_load_rowspikes(const S &s, int rb, int rn, const int (&cols)[5],
                                                 double (&w)[17]) {
#pragma unroll
  for (int c = 0; c < 17; ++c) w[c] = 0.0;
  int seg = 0;
#pragma unroll
  for (int e = 0; e < 5; ++e) {
    if (e >= rn) break;
    const int col = cols[e], k = col / FT_SZ;
    if (k == 5 || k == 10 || k == 15) continue;
    seg = fp_seg(k);
    double v[17];
    fp_load_spikes(s, col, v);
    const double a = s.A[rb + e];
#pragma unroll
    for (int c = 0; c < 17; ++c) w[c] = fma(a, v[c], w[c]);
  }
  return seg;
}
