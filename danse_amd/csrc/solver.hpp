// Lane-group small Hermitian solvers for the DANSE filter update
// (update_w / update_w_gevd, danse_toolbox/d_classes.py:3320-3387).
//
// Layout: one frequency bin per group of G lanes, lane i of the group holds
// ROW i of every DMAX x DMAX matrix in registers (cf A[DMAX]).  Every loop is
// compile-time unrolled to DMAX and carries no runtime bound: a problem of
// size D < DMAX is embedded by the caller (pad_identity) so that the padded
// block is decoupled and inert:
//   Rnn (GEVD) / Ryy (MWF) padded with the identity, the other matrix with 0,
//   so L = diag(L_D, I), C = diag(C_D, 0), T = diag(T_D, 0), and the padded
//   eigenvalues are 0 (never among the top R of the PSD C_D after the
//   update gate) with eigenvector components exactly 0.
// Row broadcasts are DPP row_newbcast (G = 16) or quad_perm (G = 4);
// reductions are DPP butterflies (common.hpp).  No LDS except the one
// transpose tile and the Householder vectors.
//
// GEVD path (rank R):
//   Rnn = L L^H (Cholesky)                      [replaces LAPACK zpotrf]
//   C   = L^{-1} Ryy L^{-H}  (2 forward solves + one LDS transpose) [zhegst]
//   C   = Q T Q^H, Householder, T complex tridiagonal            [zhetrd]
//   top-R eigenvalues of T by multisection (Sturm counts, one point per lane)
//   eigenvectors by inverse iteration on the real-symmetric T' = P^H T P,
//   back-transformed v = Q P x
//   w = sum_r (1 - 1/s_r) L^{-H} v_r (v_r^H L^H e_ref)
// which equals the reference's W = X diag(1-1/s) X^{-1}, w = W[:, ref] with
// X^H Rnn X = I (scipy.linalg.eigh(Ryy, Rnn), descending order).
//
// MWF path: w = Ryy^{-1}(Ryy - Rnn) e_ref = L^{-H} L^{-1} (Ryy - Rnn) e_ref
// with Ryy = L L^H.
#pragma once
#include <type_traits>
#include "common.hpp"

namespace danse {

template <int B, int E, typename Fn>
DANSE_DEV void sfor(Fn&& fn) {
  if constexpr (B < E) {
    fn(std::integral_constant<int, B>{});
    sfor<B + 1, E>(fn);
  }
}
// B-1, B-2, ..., E
template <int B, int E, typename Fn>
DANSE_DEV void sfor_down(Fn&& fn) {
  if constexpr (B > E) {
    fn(std::integral_constant<int, B - 1>{});
    sfor_down<B - 1, E>(fn);
  }
}

constexpr int kRMax = 4;   // largest supported GEVD rank

template <int DMAX>
struct SolverLDS {
  cf U[DMAX][DMAX + 1];     // transpose tile, then Householder vectors U[j][i]
  float x[kRMax][DMAX];     // real tridiagonal eigenvectors (Gram-Schmidt of rank > 1)
  cf tb[DMAX];              // complex sub-diagonal T[i+1][i] (phase fix)
};

// Embed a size-D problem: rows D..DMAX-1 of X (zero on entry) become unit
// rows.  Written as an add so that the unrolled selects are not merged into
// one dynamically indexed store (which would demote X to scratch).
template <int DMAX>
DANSE_DEV void pad_identity(cf (&X)[DMAX], int li, int D) {
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    X[c].re += (li == c && c >= D) ? 1.0f : 0.0f;
  });
}

// ---- Cholesky, rows in registers: on exit B[c] (c <= li) = L[li][c], 0 above,
// invd = 1 / L[li][li] (lane-local).
template <int G, int DMAX>
DANSE_DEV bool chol_rows(cf (&B)[DMAX], int li, float& invd) {
  bool ok = true;
  invd = 0.0f;
  sfor<0, DMAX>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const float p0 = gbcast<G, j>(B[j].re);
    ok = ok && (p0 > 1e-37f);
    const float piv = fmaxf(p0, 1e-37f);
    const float inv = frsq(piv);
    if (li == j) { B[j] = cf{piv * inv, 0.0f}; invd = inv; }
    else if (li > j) B[j] = inv * B[j];
    // trailing update B[li][c] -= L[li][j] conj(L[c][j]); rows li < c only touch
    // the (discarded) upper triangle
    sfor<j + 1, DMAX>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const cf lcj = gbcast<G, c>(B[j]);
      fms_cc(B[c], B[j], lcj);
    });
  });
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c > li) B[c] = cf{0.0f, 0.0f};
  });
  return ok;
}

// Substitution multiplier for step J on lane li: lanes i != J eliminate with
// L[i][J] / L[J][J] applied to the raw row J, lane J itself scales by
// 1 / L[J][J] through x_J - (1 - 1/L[J][J]) x_J.  No divide, no row scaling.
template <int G, int J>
DANSE_DEV cf elim_mult(cf lij, float invd, int li) {
  const float ij = gbcast<G, J>(invd);
  return (li == J) ? cf{1.0f - ij, 0.0f} : ij * lij;
}

// X <- L^{-1} X (rows of X and L in registers; rows li < j have L[li][j] = 0).
template <int G, int DMAX>
DANSE_DEV void fwd_rows(cf (&X)[DMAX], const cf (&L)[DMAX], float invd, int li) {
  sfor<0, DMAX>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const cf lm = elim_mult<G, j>(L[j], invd, li);
    sfor<0, DMAX>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const cf xjc = gbcast<G, j>(X[c]);
      fms_c(X[c], lm, xjc);
    });
  });
}

// vector x (one value per lane) <- L^{-1} x
template <int G, int DMAX>
DANSE_DEV cf fwd_vec(cf x, const cf (&L)[DMAX], float invd, int li) {
  sfor<0, DMAX>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const cf lm = elim_mult<G, j>(L[j], invd, li);
    const cf xj = gbcast<G, j>(x);
    fms_c(x, lm, xj);
  });
  return x;
}

// vector v (one value per lane) <- L^{-H} v  (back substitution with L^H),
// given Lt with Lt[c] = conj(L[c][li]) on lane li (column li of L, conjugated;
// herm_transpose of the Cholesky rows).  Lanes i > j have Lt[j] = 0, so a
// lane's value is final once its own step has passed.
template <int G, int DMAX>
DANSE_DEV cf bwd_vec_h(cf v, const cf (&Lt)[DMAX], float invd, int li) {
  sfor_down<DMAX, 0>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const cf lm = elim_mult<G, j>(Lt[j], invd, li);
    const cf uj = gbcast<G, j>(v);
    fms_c(v, lm, uj);
  });
  return v;
}

// Transpose-conjugate rows through LDS: X[li][c] <- conj(X[c][li]).
template <int G, int DMAX>
DANSE_DEV void herm_transpose(cf (&X)[DMAX], cf (*U)[DMAX + 1], int li) {
  if (li < DMAX) {
    sfor<0, DMAX>([&](auto cc) { U[li][decltype(cc)::value] = X[decltype(cc)::value]; });
  }
  __syncthreads();
  if (li < DMAX) {
    sfor<0, DMAX>([&](auto cc) { X[decltype(cc)::value] = conjg(U[decltype(cc)::value][li]); });
  }
  __syncthreads();
}

// Householder reduction of the Hermitian C (rows in A; rows of lanes >= DMAX
// are zero) to tridiagonal form.  Stores u_j in S.U[j][i]; returns the
// diagonal a = T[li][li] and sub-diagonal b = T[li][li-1] of my row.
// Branch-free: a zero column gives u = 0 (identity reflector).
template <int G, int DMAX>
DANSE_DEV void tridiag_rows(cf (&A)[DMAX], SolverLDS<DMAX>& S, int li, float& a, cf& b) {
  sfor<0, (DMAX >= 2 ? DMAX - 2 : 0)>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const cf xi = (li > j) ? A[j] : cf{0.0f, 0.0f};
    const float nrm2 = gsum<G>(abs2(xi));
    const cf x0 = gbcast<G, j + 1>(A[j]);
    const float ax02 = abs2(x0);
    const float nx = fsqrt(nrm2);
    const float ax0 = fsqrt(ax02);
    const float iax0 = frsq(ax02);
    const cf e = (ax02 > 0.0f) ? cf{x0.re * iax0, x0.im * iax0} : cf{1.0f, 0.0f};
    const float invn = (nrm2 > 1e-30f) ? frsq(2.0f * nx * (nx + ax0)) : 0.0f;
    cf u = xi;
    if (li == j + 1) u = u + nx * e;
    u = invn * u;
    // p = A u  (u_c = 0 for c <= j)
    cf p = cf{0.0f, 0.0f};
    sfor<j + 1, DMAX>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      fma_c(p, A[c], gbcast<G, c>(u));
    });
    const float Kr = gsum<G>(cmul(u, p).re);
    const cf q = p - Kr * u;
    const cf u2 = 2.0f * u, q2 = 2.0f * q;
    sfor<j, DMAX>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const cf qc = gbcast<G, c>(q);
      const cf uc = gbcast<G, c>(u);
      // A[i][c] -= 2 (u_i conj(q_c) + q_i conj(u_c))
      fms_cc(A[c], u2, qc);
      fms_cc(A[c], q2, uc);
    });
    if (li < DMAX) S.U[j][li] = u;
  });
  a = 0.0f;
  b = cf{0.0f, 0.0f};
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (li == c) a = A[c].re;
    if constexpr (c >= 1) {
      if (li == c) b = A[c - 1];
    }
  });
  __syncthreads();   // Householder vectors in S.U visible to the back-transform
}

// The real tridiagonal, replicated in the registers of every lane of the
// group; the complex sub-diagonal (needed once, for the phase fix) goes to LDS.
template <int DMAX>
struct Tri {
  float a[DMAX];    // diagonal
  float e2[DMAX];   // |sub-diagonal|^2, e2[i] = |T[i+1][i]|^2
};

template <int G, int DMAX>
DANSE_DEV void gather_tri(Tri<DMAX>& T, float a, cf b, cf* tb, int li) {
  const float e2 = abs2(b);
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    T.a[c] = gbcast<G, c>(a);
    if constexpr (c + 1 < DMAX) T.e2[c] = gbcast<G, c + 1>(e2);
    else T.e2[c] = 0.0f;
  });
  if (li >= 1 && li < DMAX) tb[li - 1] = b;
  if (li == DMAX - 1) tb[DMAX - 1] = cf{0.0f, 0.0f};
  __syncthreads();
}

// Number of eigenvalues of the real symmetric tridiagonal (a, sqrt(e2)) below x.
template <int DMAX>
DANSE_DEV int sturm_reg(const Tri<DMAX>& T, float x, float pivmin) {
  int cnt = 0;
  float q = 1.0f;
  sfor<0, DMAX>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    float qn;
    if constexpr (i == 0) qn = T.a[0] - x;
    else qn = (T.a[i] - x) - T.e2[i - 1] * frcp(q);
    if (fabsf(qn) <= pivmin) qn = -pivmin;
    q = qn;
    cnt += (q < 0.0f) ? 1 : 0;
  });
  return cnt;
}

// Top-R eigenvalues (descending) by multisection: every lane of the group
// evaluates one Sturm count per pass, the bracket shrinks by (G + 1).
template <int G, int DMAX, int RMAX>
DANSE_DEV void top_eigvals(const Tri<DMAX>& T, int li, int R, float (&lam)[kRMax], float& tnorm) {
  float lo = 3.0e38f, hi = -3.0e38f, e2max = 0.0f;
  tnorm = 0.0f;
  sfor<0, DMAX>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    float em = 0.0f;
    if constexpr (i >= 1) em = fsqrt(T.e2[i - 1]);
    const float ep = fsqrt(T.e2[i]);
    lo = fminf(lo, T.a[i] - em - ep);
    hi = fmaxf(hi, T.a[i] + em + ep);
    e2max = fmaxf(e2max, T.e2[i]);
    tnorm = fmaxf(tnorm, fabsf(T.a[i]) + em + ep);
  });
  const float scale = fmaxf(fabsf(lo), fabsf(hi));
  const float pivmin = 1.0e-30f * fmaxf(1.0f, e2max);
  lo -= 2.0f * 1.2e-7f * scale + pivmin;
  hi += 2.0f * 1.2e-7f * scale + pivmin;
  constexpr int NIT = (G >= 64) ? 5 : (G >= 16 ? 7 : 12);
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if (r < R) {
      float a = lo, b = hi;
      constexpr int target = DMAX - r;   // count(x) >= target  <=>  x > lambda_r
      for (int it = 0; it < NIT; ++it) {
        const float step = (b - a) * (1.0f / (float)(G + 1));
        const float x = a + step * (float)(li + 1);
        const int cnt = sturm_reg<DMAX>(T, x, pivmin);
        const uint64_t m = gballot<G>(cnt >= target);
        if (m == 0ull) {
          a = a + step * (float)G;
        } else {
          const int first = __builtin_ctzll(m);
          const float na = a + step * (float)first;
          b = a + step * (float)(first + 1);
          a = na;
        }
      }
      lam[r] = 0.5f * (a + b);
      hi = b;
    }
  });
}

// Eigenvector of the real tridiagonal for eigenvalue lam by inverse
// iteration (LAPACK dgtsv elimination with partial pivoting, written with
// selects so that the groups of a wave never diverge), Gram-Schmidt against
// the R previous vectors in LDS.  All lanes of a group compute the same x.
// The start vector is zero on the padded block, which keeps it zero.
template <int DMAX>
DANSE_DEV void tri_eigvec(const Tri<DMAX>& T, int D, float lam, float pert, int r, const float (*prev)[DMAX],
                          float (&x)[DMAX]) {
  sfor<0, DMAX>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    x[i] = (i < D) ? 1.0f + 0.1f * (float)((i * 7919 + r * 104729) % 13) / 13.0f : 0.0f;
  });
  float e[DMAX];
  sfor<0, DMAX>([&](auto ic) { e[decltype(ic)::value] = fsqrt(T.e2[decltype(ic)::value]); });
  for (int it = 0; it < 2; ++it) {
    float d[DMAX], dl[DMAX], du[DMAX], rhs[DMAX];
    sfor<0, DMAX>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      d[i] = T.a[i] - lam;
      dl[i] = e[i];
      du[i] = e[i];
      rhs[i] = x[i];
    });
    sfor<0, DMAX - 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const bool swap = fabsf(d[i]) < fabsf(dl[i]);
      const float di = (d[i] == 0.0f) ? pert : d[i];
      const float f1 = dl[i] * frcp(di);       // no interchange
      const float f2 = d[i] * frcp(dl[i]);     // interchange rows i, i+1
      const float d1 = d[i + 1];
      const float duI = du[i];
      float du1 = 0.0f;
      if constexpr (i + 2 < DMAX) du1 = du[i + 1];
      d[i] = swap ? dl[i] : di;
      d[i + 1] = swap ? (duI - f2 * d1) : (d1 - f1 * duI);
      dl[i] = swap ? du1 : 0.0f;   // second super-diagonal
      if constexpr (i + 2 < DMAX) du[i + 1] = swap ? -f2 * du1 : du1;
      du[i] = swap ? d1 : duI;
      const float ri = rhs[i], ri1 = rhs[i + 1];
      rhs[i] = swap ? ri1 : ri;
      rhs[i + 1] = swap ? (ri - f2 * ri1) : (ri1 - f1 * ri);
    });
    // back solve
    sfor_down<DMAX, 0>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      float acc = rhs[i];
      if constexpr (i + 1 < DMAX) acc -= du[i] * rhs[i + 1];
      if constexpr (i + 2 < DMAX) acc -= dl[i] * rhs[i + 2];
      const float di = (d[i] == 0.0f) ? pert : d[i];
      rhs[i] = acc * frcp(di);
    });
    for (int q = 0; q < r; ++q) {
      float dot = 0.0f;
      sfor<0, DMAX>([&](auto ic) { constexpr int i = decltype(ic)::value; dot += prev[q][i] * rhs[i]; });
      sfor<0, DMAX>([&](auto ic) { constexpr int i = decltype(ic)::value; rhs[i] -= dot * prev[q][i]; });
    }
    float mx = 0.0f;
    sfor<0, DMAX>([&](auto ic) { mx = fmaxf(mx, fabsf(rhs[decltype(ic)::value])); });
    mx = (mx > 0.0f) ? mx : 1.0f;
    const float imx = frcp(mx);
    float nrm = 0.0f;
    sfor<0, DMAX>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      rhs[i] *= imx;
      nrm += rhs[i] * rhs[i];
    });
    const float inv = frsq(nrm);
    sfor<0, DMAX>([&](auto ic) { constexpr int i = decltype(ic)::value; x[i] = rhs[i] * inv; });
  }
}

// Full GEVD filter: A = Ryy rows, B = Rnn rows (both destroyed; rows of
// lanes >= D zero on entry).  Returns w_li.  RMAX bounds the runtime rank R.
template <int G, int DMAX, int RMAX>
DANSE_DEV cf gevd_filter(cf (&A)[DMAX], cf (&B)[DMAX], SolverLDS<DMAX>& S, int li, int D, int R, int ref,
                         bool& ok) {
  const bool act = li < D;
  pad_identity<DMAX>(B, li, D);
  float invd;
  ok = chol_rows<G, DMAX>(B, li, invd);
  fwd_rows<G, DMAX>(A, B, invd, li);          // A = L^{-1} Ryy
  herm_transpose<G, DMAX>(A, S.U, li);        // A = Ryy L^{-H}
  fwd_rows<G, DMAX>(A, B, invd, li);          // A = L^{-1} Ryy L^{-H} = C
  herm_transpose<G, DMAX>(B, S.U, li);        // B[c] = conj(L[c][li]) (columns of L)
  float ta;
  cf tb;
  tridiag_rows<G, DMAX>(A, S, li, ta, tb);
  Tri<DMAX> T;
  gather_tri<G, DMAX>(T, ta, tb, S.tb, li);
  float lam[kRMax];
  float tnorm;
  top_eigvals<G, DMAX, RMAX>(T, li, R, lam, tnorm);
  const float pert = 1.2e-7f * fmaxf(tnorm, 1e-30f);
  // g = L^H e_ref : g_i = conj(L[ref][i]) = B[ref] on lane i
  cf g = cf{0.0f, 0.0f};
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c == ref) g = B[c];
  });
  cf w = cf{0.0f, 0.0f};
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if (r >= R) return;
    float x[DMAX];
    tri_eigvec<DMAX>(T, D, lam[r], pert, r, S.x, x);
    // phase fix v_i = phi_i x_i (phi_{i+1} = phi_i * b_i / |b_i|); lane li keeps v_li
    cf v = cf{0.0f, 0.0f};
    cf phi = cf{1.0f, 0.0f};
    sfor<0, DMAX>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if (li == i) v = x[i] * phi;
      if constexpr (i + 1 < DMAX) {
        const cf b = S.tb[i];
        const float ab2 = abs2(b);
        const float iab = frsq(ab2);
        if (ab2 > 0.0f) phi = phi * cf{b.re * iab, b.im * iab};
      }
    });
    if (r + 1 < R) {
      // keep x for Gram-Schmidt of the next eigenvectors
      float xi = 0.0f;
      sfor<0, DMAX>([&](auto ic) { constexpr int i = decltype(ic)::value; if (li == i) xi = x[i]; });
      if (li < DMAX) S.x[r][li] = xi;
      __syncthreads();
    }
    // back-transform with the Householder vectors, last first
    sfor_down<(DMAX >= 2 ? DMAX - 2 : 0), 0>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const cf u = (li < DMAX) ? S.U[j][li] : cf{0.0f, 0.0f};
      const cf s = gsum<G>(cmul(u, v));
      fms_c(v, 2.0f * u, s);
    });
    const cf sr = gsum<G>(cmul(v, g));
    const cf u = bwd_vec_h<G, DMAX>(v, B, invd, li);
    const float coef = 1.0f - frcp(lam[r]);
    w = w + coef * (u * sr);
  });
  return act ? w : cf{0.0f, 0.0f};
}

// MWF filter: A = Ryy rows, B = Rnn rows (rows of lanes >= D zero).  Returns w_li.
// w = Ryy^{-1} (Ryy - Rnn) e_ref: the difference column is formed first, as
// the reference does (np.linalg.inv(Ryy) @ (Ryy - Rnn)), which keeps the
// speech-dominated cancellation out of the solve.
template <int G, int DMAX>
DANSE_DEV cf mwf_filter(cf (&A)[DMAX], const cf (&B)[DMAX], SolverLDS<DMAX>& S, int li, int D, int ref, bool& ok) {
  const bool act = li < D;
  cf r = cf{0.0f, 0.0f};
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c == ref) r = A[c] - B[c];
  });
  pad_identity<DMAX>(A, li, D);
  float invd;
  ok = chol_rows<G, DMAX>(A, li, invd);
  cf t = fwd_vec<G, DMAX>(r, A, invd, li);
  herm_transpose<G, DMAX>(A, S.U, li);        // columns of L
  cf w = bwd_vec_h<G, DMAX>(t, A, invd, li);
  return act ? w : cf{0.0f, 0.0f};
}

}  // namespace danse
