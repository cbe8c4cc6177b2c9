// qp_block.h -- block-tridiagonal factor/solve of the reduced KKT matrix
//     M = P + sigma I + A' R A
// for QPs whose variables split into uniform blocks of SZ (the MPC stages
// [x_k, u_k]) such that M couples only neighbouring blocks, and block k+1
// couples to block k only through its first CM rows (x_{k+1}).  Included by
// qp_device.h; used when the host pattern analysis selects mode 1.
//
//   S_0 = M_00,  S_{k+1} = M_{k+1,k+1} - G_k C_k^T,   G_k = C_k S_k^-1,
//   C_k = M[block k+1 (first CM rows)][block k]
// solve  M x = b :
//   forward   y_0 = b_0,  y_{k+1} = b_{k+1} - G_k y_k         (chain, SZ FMAs/block)
//   diagonal  u_k = S_k^-1 y_k                                 (independent blocks)
//   backward  x_K = u_K,  x_k = u_k - G_k^T x_{k+1}            (chain, CM FMAs/block)
//
// Everything runs in wave 0 with one block row per lane of a 16-lane DPP row
// (the four rows of the wave replicate the chain, or work on four blocks at
// once in the diagonal step).  The vector operand of every block product is
// broadcast with DPP row_newbcast straight into v_fmac_f64, so the chains
// need no readlane, no LDS round trip and no barrier: a forward block is 10
// dependent-free FMAs + one add.
//
// Storage (doubles, in the factor area of QPSmem), block stride
// BS = SZ*SZ + SZ*CM:
//   [k*BS, +SZ*SZ)       S_k^-1  column-major (symmetric)   slot j*SZ + r = S^-1[r][j]
//   [k*BS + SZ*SZ, +SZ*CM) -G_k  column-major               slot j*CM + r = -G_k[r][j]
// (before factoring the same slots hold M_kk and C_k; a last block shorter
// than SZ is padded with identity rows by the host).
#pragma once

// accumulators of the KKT chains' block products (1, 2 or 4).  Measured on the
// fleet control kernel: 4 is 2.4% slower than 2 (more instructions on the
// chain); 1 needs an s_nop between dependent DPP FMAs, so 2 it is
#ifndef QP_CHAIN_ACC
#define QP_CHAIN_ACC 2
#endif
// QP_CHAIN_PF2: operands two blocks ahead in the runtime-count forward chain
// (measured 2.6% slower on the fleet: the extra index math costs more than the
// LDS latency it hides)
#ifndef QP_CHAIN_PF2
#define QP_CHAIN_PF2 0
#endif

// value of lane J of each 16-lane row, in every lane of that row
template <int J>
__device__ __forceinline__ double bc16(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xf, 0xf, true);
}
__device__ __forceinline__ double bc16_rt(double v, int j) {
  switch (j) {  // j is a constant after unrolling
    case 0: return bc16<0>(v);
    case 1: return bc16<1>(v);
    case 2: return bc16<2>(v);
    case 3: return bc16<3>(v);
    case 4: return bc16<4>(v);
    case 5: return bc16<5>(v);
    case 6: return bc16<6>(v);
    case 7: return bc16<7>(v);
    case 8: return bc16<8>(v);
    case 9: return bc16<9>(v);
    case 10: return bc16<10>(v);
    case 11: return bc16<11>(v);
    case 12: return bc16<12>(v);
    case 13: return bc16<13>(v);
    case 14: return bc16<14>(v);
    default: return bc16<15>(v);
  }
}

// acc += bcast_J(src) * mul as ONE v_fmac_f64_dpp.  The compiler does not see
// the DPP read of src inside the asm, so the first FMA of a chain carries the
// two wait states a DPP read of a just-written VGPR needs.
template <int J, bool NOP>
__device__ __forceinline__ void fmac_bc(double &acc, double src, double mul) {
  if (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "i"(J));
  else
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "i"(J));
}
// returns sum_j mul[j] * bcast_j(src), two interleaved accumulators
template <int... J>
__device__ __forceinline__ double dot_bc(double src, const double *mul, std::integer_sequence<int, J...>) {
  double a0 = 0.0, a1 = 0.0;
  ((J % 2 == 0 ? fmac_bc<J, J == 0>(a0, src, mul[J]) : fmac_bc<J, false>(a1, src, mul[J])), ...);
  return a0 + a1;
}
// init + sum_j mul[j] * bcast_j(src)
template <int... J>
__device__ __forceinline__ double dot_bc_init(double init, double src, const double *mul,
                                              std::integer_sequence<int, J...>) {
#if QP_CHAIN_ACC == 4
  // four accumulators: the chain's dependent depth is ceil(K/4) FMAs + 2 adds
  // instead of ceil(K/2) + 1 (the sum order differs from the generic solver's)
  double a0 = init, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  ((J % 4 == 0   ? fmac_bc<J, J == 0>(a0, src, mul[J])
    : J % 4 == 1 ? fmac_bc<J, false>(a1, src, mul[J])
    : J % 4 == 2 ? fmac_bc<J, false>(a2, src, mul[J])
                 : fmac_bc<J, false>(a3, src, mul[J])), ...);
  return (a0 + a1) + (a2 + a3);
#elif QP_CHAIN_ACC == 1
  // one accumulator: K dependent FMAs, no closing add
  double a0 = init;
  (fmac_bc<J, J == 0>(a0, src, mul[J]), ...);
  return a0;
#else
  double a0 = init, a1 = 0.0;
  ((J % 2 == 0 ? fmac_bc<J, J == 0>(a0, src, mul[J]) : fmac_bc<J, false>(a1, src, mul[J])), ...);
  return a0 + a1;
#endif
}
template <int K>
__device__ __forceinline__ double dot_bc_init(double init, double src, const double *mul) {
  return dot_bc_init(init, src, mul, std::make_integer_sequence<int, K>{});
}
// two products of the same broadcast source, interleaved (4 accumulators):
//   r0 = init0 + sum_j m0[j] bcast_j(src),  r1 = sum_j m1[j] bcast_j(src)
template <int... J>
__device__ __forceinline__ void dot2_bc(double init0, double src, const double *m0,
                                        const double *m1, double &r0, double &r1,
                                        std::integer_sequence<int, J...>) {
  double a0 = init0, a1 = 0.0, c0 = 0.0, c1 = 0.0;
  ((J % 2 == 0 ? (fmac_bc<J, J == 0>(a0, src, m0[J]), fmac_bc<J, false>(c0, src, m1[J]))
               : (fmac_bc<J, false>(a1, src, m0[J]), fmac_bc<J, false>(c1, src, m1[J]))), ...);
  r0 = a0 + a1;
  r1 = c0 + c1;
}
template <int K>
__device__ __forceinline__ void dot2_bc(double init0, double src, const double *m0, const double *m1,
                                        double &r0, double &r1) {
  dot2_bc(init0, src, m0, m1, r0, r1, std::make_integer_sequence<int, K>{});
}
// same with compiler-visible DPP moves (2 VALU per term, exact waitcnts)
template <int... J>
__device__ __forceinline__ double dot_bcv(double src, const double *mul, std::integer_sequence<int, J...>) {
  double a0 = 0.0, a1 = 0.0;
  ((J % 2 == 0 ? (void)(a0 = fma(bc16<J>(src), mul[J], a0)) : (void)(a1 = fma(bc16<J>(src), mul[J], a1))), ...);
  return a0 + a1;
}
#ifndef QP_FAST_RECIP
#define QP_FAST_RECIP 1
#endif
#ifndef QP_CHAIN_ROW0
#define QP_CHAIN_ROW0 1
#endif
#ifndef QP_DOT_ASM
#define QP_DOT_ASM 1
#endif
template <int K>
__device__ __forceinline__ double dot_bc(double src, const double *mul) {
  if (QP_DOT_ASM) return dot_bc(src, mul, std::make_integer_sequence<int, K>{});
  return dot_bcv(src, mul, std::make_integer_sequence<int, K>{});
}

// 1/p for a positive, normal pivot: v_rcp_f64 + two Newton steps (4 dependent
// FMAs instead of the ~10-instruction IEEE division sequence on the factor's
// critical path); within an ulp of the division.
__device__ __forceinline__ double blk_recip(double p) {
#if QP_FAST_RECIP
  double r = __builtin_amdgcn_rcp(p);
  double e = fma(-p, r, 1.0);
  r = fma(r, e, r);
  e = fma(-p, r, 1.0);
  return fma(r, e, r);
#else
  return 1.0 / p;
#endif
}

// ---- factor helpers: every broadcast-multiply-add is one v_fmac_f64_dpp.
// Gauss-Jordan step p: a[c] += bcast_p(a[c]) * f for c != p (the source and the
// accumulator are the same register: DPP reads all lanes before the write).
// The first FMA of a step waits the two DPP states after the last VALU write.
template <int P, int... C>
__device__ __forceinline__ void fq_gj_step(double *a, double f, std::integer_sequence<int, C...>) {
  ((C != P ? fmac_bc<P, C == (P == 0 ? 1 : 0)>(a[C], a[C], f) : (void)0), ...);
}
template <int SZ, int... P>
__device__ __forceinline__ void fq_gj_dispatch(double *a, double f, int p, std::integer_sequence<int, P...>) {
  ((p == P ? fq_gj_step<P>(a, f, std::make_integer_sequence<int, SZ>{}) : (void)0), ...);
}
template <int SZ>
__device__ __forceinline__ void fq_gj_update(double *a, double f, int p) {
  fq_gj_dispatch<SZ>(a, f, p, std::make_integer_sequence<int, SZ>{});
}
// g[j] += c[l] * bcast_l(a[j]) for l = 0..SZ-1, j = 0..SZ-1
template <int L, int... J>
__device__ __forceinline__ void blk_gmul_l(double *g, const double *a, double cl, std::integer_sequence<int, J...>) {
  ((fmac_bc<L, L == 0 && J == 0>(g[J], a[J], cl)), ...);
}
template <int SZ, int... L>
__device__ __forceinline__ void blk_gmul(double *g, const double *a, const double *c, std::integer_sequence<int, L...>) {
  (blk_gmul_l<L>(g, a, c[L], std::make_integer_sequence<int, SZ>{}), ...);
}
// u[i] = sum_j g[j] * bcast_i(c[j]) for i = 0..CM-1
template <int I, int... J>
__device__ __forceinline__ double blk_schur_i(const double *g, const double *c, std::integer_sequence<int, J...>) {
  double t = 0.0;
  ((fmac_bc<I, I == 0 && J == 0>(t, c[J], g[J])), ...);
  return t;
}
template <int SZ, int CM, int... I>
__device__ __forceinline__ void blk_schur(double *u, const double *g, const double *c, std::integer_sequence<int, I...>) {
  ((u[I] = blk_schur_i<I>(g, c, std::make_integer_sequence<int, SZ>{})), ...);
}

// factor: returns 0 or the 1-based failing (non-positive pivot) variable.
// Wave 0 only, all 64 lanes (rows replicate).
template <int SZ, int CM, class S>
__device__ __forceinline__ int blk_factor(const QPPattern &pt, S &s) {
  constexpr int BS = SZ * SZ + SZ * CM;
  const int lane = threadIdx.x & 63, rr = lane & 15;
  const bool wr = lane < 16;
  const int rs = rr < SZ ? rr : SZ - 1, rc = rr < CM ? rr : CM - 1;
  double *F = s.band();
  const int nblk = pt.nblk;
  double u[CM];  // Schur update of the next block's CM x CM corner, row rr
#pragma unroll
  for (int i = 0; i < CM; ++i) u[i] = 0.0;
  for (int k = 0; k < nblk; ++k) {
    double *Sk = F + k * BS;
    double a[SZ];
#pragma unroll
    for (int j = 0; j < SZ; ++j) a[j] = Sk[j * SZ + rs];
    if (rr < CM) {
#pragma unroll
      for (int j = 0; j < CM; ++j) a[j] -= u[j];
    }
    // in-place Gauss-Jordan inverse (SPD: no pivoting); pivot row by DPP
#pragma unroll
    for (int p = 0; p < SZ; ++p) {
      const double piv = bc16_rt(a[p], p);
      if (!(piv > 0.0)) return k * SZ + p + 1;
      const double inv = blk_recip(piv);
      // lane p: row *= inv  (= row + row*(inv-1));  other lanes: row -= a[p]/piv * row_p
      const double f = (rr == p) ? inv - 1.0 : -a[p] * inv;
      fq_gj_update<SZ>(a, f, p);
      a[p] = (rr == p) ? inv : f;
    }
    if (wr && rr < SZ) {
#pragma unroll
      for (int j = 0; j < SZ; ++j) Sk[j * SZ + rr] = a[j];
    }
    if (k + 1 < nblk) {
      double *Ck = Sk + SZ * SZ;
      double c[SZ], g[SZ];
#pragma unroll
      for (int j = 0; j < SZ; ++j) {
        c[j] = Ck[j * CM + rc];
        g[j] = 0.0;
      }
      // G[rr][j] = sum_l C[rr][l] S^-1[l][j]   (one v_fmac_f64_dpp per term)
      blk_gmul<SZ>(g, a, c, std::make_integer_sequence<int, SZ>{});
      if (wr && rr < CM) {  // stored negated: the solve's chains accumulate into b / u
#pragma unroll
        for (int j = 0; j < SZ; ++j) Ck[j * CM + rr] = -g[j];
      }
      // u[rr][i] = sum_j G[rr][j] C[i][j]   (one v_fmac_f64_dpp per term)
      blk_schur<SZ, CM>(u, g, c, std::make_integer_sequence<int, CM>{});
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  return 0;
}

// b <- M^-1 b.  Wave 0 only.  The block loops are unrolled by two with
// ping-pong operand registers, so the next block's operands load under the
// current block's FMA chain without register copies.  b is zero-padded to
// nblk*SZ entries (qp_solve), so lanes read it without bounds selects; lanes
// rr >= SZ (never a broadcast source) read clamped addresses and only the
// stores are masked.  Per-lane pointers advance by constants; operands sit at
// immediate offsets.
//  NBC > 0: the block count is known at compile time (the fleet's N = 20
//  MPC); when pt.nblk matches, the !FUSED chains run fully unrolled -- no loop
//  counter, branch or pointer updates, every operand at an immediate offset.
//  PH (!FUSED only): the phases run by this call, 1 forward | 2 diagonal |
//  4 backward.  A PH == 2 call is made by BOTH waves of the workgroup (caller
//  barriers around it): eight blocks per round, one per DPP row of either wave.
template <int SZ, int CM, bool FUSED = true, int NBC = 0, int PH = 7, class S>
__device__ __forceinline__ void blk_solve(const QPPattern &pt, S &s, double *b, QPStamps *T = nullptr, int cw = 0) {
  static_assert(!FUSED || PH == 7, "the fused solve runs all phases in one call");
  if (PH != 2 && (int)(threadIdx.x >> 6) != cw) return;
  constexpr int BS = SZ * SZ + SZ * CM;
  // non-coupled lanes keep pg = gzero (gstep 0) and read gzero[j * CM], j < SZ
  static_assert((SZ - 1) * CM + 1 <= sizeof(s.gzero) / sizeof(double), "gzero too small");
  const int lane = threadIdx.x & 63, rr = lane & 15, row = lane >> 4;
  const int rs = rr < SZ ? rr : SZ - 1, rc = rr < CM ? rr : CM - 1;
  const bool wr = rr < SZ;
  const int nblk = pt.nblk;
  const double *F = s.band();
  if (nblk == 1) {
    if (!(PH & 1) || (int)(threadIdx.x >> 6) != cw) return;
    double sv[SZ];
#pragma unroll
    for (int j = 0; j < SZ; ++j) sv[j] = F[j * SZ + rs];
    const double uv = dot_bc<SZ>(b[rs], sv);
    if (wr) b[rr] = uv;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    return;
  }
  // ---- forward + diagonal in one pass over the blocks:
  //        y_{k+1} = b_{k+1} + (-G_k) y_k     (first CM rows of block k+1)
  //        u_k     = S_k^-1 y_k               (stored over b_k)
  //      both products broadcast the same y_k, so their two FMA chains
  //      interleave.  Lanes rr >= CM read their "-G row" from a zero region
  //      (their y is exactly b); lanes rr >= SZ compute bit-identical values
  //      to lane SZ-1 (same clamped inputs), so every store is unconditional.
  //  !FUSED: the chain carries the G product only (half the FMAs and operand
  //      registers on the critical path) and the diagonal products run after
  //      it, four independent blocks per round, one per DPP row.
  if constexpr (!FUSED) {
    if constexpr ((PH & 1) != 0) {
    // the chains need the SZ lanes of one 16-lane row: the other lanes would
    // only replicate them, and their LDS operand reads would multiply the
    // chain's LDS traffic (the CU's LDS is shared by the four landings' chains)
    if (!QP_CHAIN_ROW0 || lane < SZ) {
    double *pb = b + rs;
    const bool cpl = rr < CM;
    if (NBC > 0 && nblk == NBC) {
      // every lane reads a real -G row (rc is clamped to CM - 1); the
      // non-coupled lanes then keep b_{k+1}, which is what their zero row gave
      const double *pgu = F + SZ * SZ + rc;
      double y = pb[0];
      double g0[SZ], g1[SZ], c0, c1 = 0.0;
#pragma unroll
      for (int j = 0; j < SZ; ++j) g0[j] = pgu[j * CM];
      c0 = pb[SZ];
#pragma unroll
      for (int k = 0; k < NBC - 1; ++k) {
        double *gc = (k & 1) ? g1 : g0, *gn = (k & 1) ? g0 : g1;
        double &cc = (k & 1) ? c1 : c0, &cn = (k & 1) ? c0 : c1;
        if (k + 1 < NBC - 1) {
#pragma unroll
          for (int j = 0; j < SZ; ++j) gn[j] = pgu[(k + 1) * BS + j * CM];
          cn = pb[(k + 2) * SZ];
        }
        const double yn = dot_bc_init<SZ>(cc, y, gc);
        pb[k * SZ] = y;
        y = cpl ? yn : cc;
      }
      pb[(NBC - 1) * SZ] = y;
    } else {
    const double *pg = cpl ? F + SZ * SZ + rc : s.gzero;
    const int gstep = cpl ? BS : 0;
    double y = pb[0];
#if QP_CHAIN_PF2
    // operands two blocks ahead (three rotating sets): under four landings per
    // CU an LDS read takes longer than one block product.  Step k reads G_k and
    // b_{k+1}; the look-ahead index is clamped to the last step (no over-read).
    double g0[SZ], g1[SZ], g2[SZ], c0, c1, c2;
    auto ld = [&](double (&g)[SZ], double &c, int kk) {
      const int kc = min(kk, nblk - 2);
      const double *p = pg + kc * gstep;
#pragma unroll
      for (int j = 0; j < SZ; ++j) g[j] = p[j * CM];
      c = pb[(kc + 1) * SZ];
    };
    ld(g0, c0, 0);
    ld(g1, c1, 1);
    for (int k = 0;;) {
      ld(g2, c2, k + 2);
      { const double yn = dot_bc_init<SZ>(c0, y, g0); pb[k * SZ] = y; y = yn; }
      if (++k >= nblk - 1) break;
      ld(g0, c0, k + 2);
      { const double yn = dot_bc_init<SZ>(c1, y, g1); pb[k * SZ] = y; y = yn; }
      if (++k >= nblk - 1) break;
      ld(g1, c1, k + 2);
      { const double yn = dot_bc_init<SZ>(c2, y, g2); pb[k * SZ] = y; y = yn; }
      if (++k >= nblk - 1) break;
    }
    pb[(nblk - 1) * SZ] = y;
#else
    double gA[SZ], gB[SZ];
    double bA = pb[SZ], bB;
#pragma unroll
    for (int j = 0; j < SZ; ++j) gA[j] = pg[j * CM];
    for (int k = 0;;) {
      {
        bB = pb[2 * SZ];
#pragma unroll
        for (int j = 0; j < SZ; ++j) gB[j] = pg[gstep + j * CM];
        const double yn = dot_bc_init<SZ>(bA, y, gA);
        pb[0] = y;
        y = yn;
        pb += SZ;
        pg += gstep;
        if (++k >= nblk - 1) break;
      }
      {
        bA = pb[2 * SZ];
#pragma unroll
        for (int j = 0; j < SZ; ++j) gA[j] = pg[gstep + j * CM];
        const double yn = dot_bc_init<SZ>(bB, y, gB);
        pb[0] = y;
        y = yn;
        pb += SZ;
        pg += gstep;
        if (++k >= nblk - 1) break;
      }
    }
    pb[0] = y;
#endif
    }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (T) T->mark(8);
    }
    if constexpr ((PH & 2) != 0) {
    // diagonal: u_k = S_k^-1 y_k, block RB t + q in round t (q: this lane's
    // DPP row, over both waves when PH == 2).  Rows past the last block read
    // the last block (in bounds) and do not store.
    constexpr int RB = PH == 2 ? 8 : 4;
    const int q = PH == 2 ? (int)(threadIdx.x >> 4) : row;
    const int nr = (nblk + RB - 1) / RB;
    auto blk = [&](int t) { return min(RB * t + q, nblk - 1); };
    double sA[SZ], sB[SZ];
    {
      const double *ps = F + blk(0) * BS + rs;
#pragma unroll
      for (int j = 0; j < SZ; ++j) sA[j] = ps[j * SZ];
    }
    double yA = b[blk(0) * SZ + rs], yB = 0.0;
    for (int t = 0;;) {
      {
        const int kn = blk(t + 1 < nr ? t + 1 : t);
        const double *ps = F + kn * BS + rs;
#pragma unroll
        for (int j = 0; j < SZ; ++j) sB[j] = ps[j * SZ];
        yB = b[kn * SZ + rs];
        const double uv = dot_bc<SZ>(yA, sA);
        if (RB * t + q < nblk) b[(RB * t + q) * SZ + rs] = uv;
        if (++t >= nr) break;
      }
      {
        const int kn = blk(t + 1 < nr ? t + 1 : t);
        const double *ps = F + kn * BS + rs;
#pragma unroll
        for (int j = 0; j < SZ; ++j) sA[j] = ps[j * SZ];
        yA = b[kn * SZ + rs];
        const double uv = dot_bc<SZ>(yB, sB);
        if (RB * t + q < nblk) b[(RB * t + q) * SZ + rs] = uv;
        if (++t >= nr) break;
      }
    }
    }
  } else {
    double *pb = b + rs;                          // block k of b
    const bool cpl = rr < CM;
    const double *pg = cpl ? F + SZ * SZ + rc : s.gzero;   // -G_k row rc
    const int gstep = cpl ? BS : 0;
    const double *ps = F + rs;                    // S_k^-1 row rs: ps[k*BS + j*SZ]
    double y = pb[0];
    double gA[SZ], gB[SZ], sA[SZ], sB[SZ];
    double bA = pb[SZ], bB;                       // b_{k+1}: the next accumulator's start
#pragma unroll
    for (int j = 0; j < SZ; ++j) {
      gA[j] = pg[j * CM];
      sA[j] = ps[j * SZ];
    }
    for (int k = 0;;) {
      {
        bB = pb[2 * SZ];                           // b_{k+2} (past the end: unused)
#pragma unroll
        for (int j = 0; j < SZ; ++j) {
          gB[j] = pg[gstep + j * CM];              // -G_{k+1} (past the end: unused)
          sB[j] = ps[BS + j * SZ];                 // S_{k+1}^-1
        }
        double yn, u;
        dot2_bc<SZ>(bA, y, gA, sA, yn, u);
        pb[0] = u;
        y = yn;
        pb += SZ;
        pg += gstep;
        ps += BS;
        if (++k >= nblk - 1) break;
      }
      {
        bA = pb[2 * SZ];
#pragma unroll
        for (int j = 0; j < SZ; ++j) {
          gA[j] = pg[gstep + j * CM];
          sA[j] = ps[BS + j * SZ];
        }
        double yn, u;
        dot2_bc<SZ>(bB, y, gB, sB, yn, u);
        pb[0] = u;
        y = yn;
        pb += SZ;
        pg += gstep;
        ps += BS;
        if (++k >= nblk - 1) break;
      }
    }
    // last block: u = S^-1 y (its operands were prefetched into whichever buffer is current)
    double sl[SZ];
#pragma unroll
    for (int j = 0; j < SZ; ++j) sl[j] = ps[j * SZ];
    pb[0] = dot_bc<SZ>(y, sl);
    if (T) T->mark(8);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (T) T->mark(9);
  if constexpr ((PH & 4) == 0) return;
  // ---- backward: x_k = u_k + (-G_k)^T x_{k+1}
  if ((!QP_CHAIN_ROW0 || lane < SZ) && NBC > 0 && nblk == NBC && !FUSED) {
    // fully unrolled (see NBC above): x_k = u_k + (-G_k)^T x_{k+1}, k = NBC-2..0
    double *pb = b + rs;
    const double *pgu = F + SZ * SZ + rs * CM;   // column rs of -G_k at k * BS
    double x = pb[(NBC - 1) * SZ];
    double g0[CM], g1[CM], u0, u1 = 0.0;
#pragma unroll
    for (int i = 0; i < CM; ++i) g0[i] = pgu[(NBC - 2) * BS + i];
    u0 = pb[(NBC - 2) * SZ];
#pragma unroll
    for (int t = 0; t < NBC - 1; ++t) {
      const int k = NBC - 2 - t;
      double *gc = (t & 1) ? g1 : g0, *gn = (t & 1) ? g0 : g1;
      double &uc = (t & 1) ? u1 : u0, &un = (t & 1) ? u0 : u1;
      if (k > 0) {
#pragma unroll
        for (int i = 0; i < CM; ++i) gn[i] = pgu[(k - 1) * BS + i];
        un = pb[(k - 1) * SZ];
      }
      const double xn = dot_bc_init<CM>(uc, x, gc);
      pb[(k + 1) * SZ] = x;
      x = xn;
    }
    pb[0] = x;
  } else if (!QP_CHAIN_ROW0 || lane < SZ) {
    double *pb = b + (nblk - 1) * SZ + rs;        // block k+1 of b
    const double *pg = F + (nblk - 2) * BS + SZ * SZ + rs * CM;  // -G_k column rs
    double x = pb[0];
    double gA[CM], gB[CM];
    double uA = pb[-SZ], uB;                      // u_k: the next accumulator's start
#pragma unroll
    for (int i = 0; i < CM; ++i) gA[i] = pg[i];
    for (int k = nblk - 2;;) {
      {
        uB = pb[-2 * SZ];                          // u_{k-1} (before the start: unused)
#pragma unroll
        for (int i = 0; i < CM; ++i) gB[i] = pg[i - BS];  // -G_{k-1} (before the start: unused)
        const double xn = dot_bc_init<CM>(uA, x, gA);
        pb[0] = x;
        x = xn;
        pb -= SZ;
        pg -= BS;
        if (--k < 0) break;
      }
      {
        uA = pb[-2 * SZ];
#pragma unroll
        for (int i = 0; i < CM; ++i) gA[i] = pg[i - BS];
        const double xn = dot_bc_init<CM>(uB, x, gB);
        pb[0] = x;
        x = xn;
        pb -= SZ;
        pg -= BS;
        if (--k < 0) break;
      }
    }
    pb[0] = x;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (T) T->mark(10);
}

// the compiled (SZ, CM) instantiations; the host only selects mode 1 for these
#define QP_BLK_SZ 10  // 3-DoF MPC stage [x_k (7), u_k (3)]
#define QP_BLK_CM 7   // coupled through x_{k+1}
#define QP_NBLK_MPC20 21  // its block count at N = 20 (207 variables), unrolled by the generic solver

template <class S>
__device__ __forceinline__ int blk_factor_dispatch(const QPPattern &pt, S &s) {
  return blk_factor<QP_BLK_SZ, QP_BLK_CM>(pt, s);
}
template <bool FUSED = true, int NBC = 0, int PH = 7, class S>
__device__ __forceinline__ void blk_solve_dispatch(const QPPattern &pt, S &s, double *b, QPStamps *T = nullptr,
                                   int cw = 0) {
  blk_solve<QP_BLK_SZ, QP_BLK_CM, FUSED, NBC, PH>(pt, s, b, T, cw);
}
