// Lane-group small Hermitian solvers for the DANSE filter update
// (update_w / update_w_gevd, danse_toolbox/d_classes.py:3320-3387).
//
// Layout: one frequency bin per group of G lanes, lane i of the group holds
// ROW i of every D x D matrix in registers (cf A[DMAX]).  All loops over
// matrix columns are compile-time unrolled to DMAX (runtime D <= DMAX is
// wave-uniform), so register arrays are indexed by constants only.  Row
// broadcasts are DPP row_newbcast (G = 16) or v_readlane (G = 64).
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
// MWF path: w = Ryy^{-1}(Ryy - Rnn) e_ref = e_ref - L^{-H} L^{-1} Rnn e_ref
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
  float ta[DMAX];           // tridiagonal diagonal
  float te2[DMAX];          // squared |sub-diagonal|
  cf tb[DMAX];              // complex sub-diagonal T[i+1][i]
  float x[kRMax][DMAX];     // eigenvectors of the real tridiagonal
  float d[DMAX], dl[DMAX], du[DMAX], rhs[DMAX];   // inverse-iteration scratch
  cf v[kRMax][DMAX];        // complex eigenvectors of T (after the phase fix)
  float lam[kRMax];
};

// ---- Cholesky, rows in registers: on exit B[c] (c <= li) = L[li][c], 0 above.
template <int G, int DMAX>
DANSE_DEV bool chol_rows(cf (&B)[DMAX], int li, int D) {
  bool ok = true;
  sfor<0, DMAX>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    if (j < D) {
      const float piv = gbcast<G, j>(B[j].re);
      ok = ok && (piv > 0.0f);
      const float ljj = sqrtf(fmaxf(piv, 1e-37f));
      const float inv = 1.0f / ljj;
      if (li == j) B[j] = cf{ljj, 0.0f};
      else if (li > j) B[j] = inv * B[j];
      sfor<j + 1, DMAX>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if (c < D) {
          const cf lcj = gbcast<G, c>(B[j]);
          if (li >= c) fms_cc(B[c], B[j], lcj);
        }
      });
    }
  });
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c > li || c >= D) B[c] = cf{0.0f, 0.0f};
  });
  return ok;
}

// X <- L^{-1} X (rows of X and L in registers).
template <int G, int DMAX>
DANSE_DEV void fwd_rows(cf (&X)[DMAX], const cf (&L)[DMAX], int li, int D) {
  sfor<0, DMAX>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    if (j < D) {
      if (li == j) {
        const float inv = 1.0f / L[j].re;
        sfor<0, DMAX>([&](auto cc) { X[decltype(cc)::value] = inv * X[decltype(cc)::value]; });
      }
      sfor<0, DMAX>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if (c < D) {
          const cf xjc = gbcast<G, j>(X[c]);
          if (li > j) fms_c(X[c], L[j], xjc);
        }
      });
    }
  });
}

// vector x (one value per lane) <- L^{-1} x
template <int G, int DMAX>
DANSE_DEV cf fwd_vec(cf x, const cf (&L)[DMAX], int li, int D) {
  sfor<0, DMAX>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    if (j < D) {
      if (li == j) x = (1.0f / L[j].re) * x;
      const cf xj = gbcast<G, j>(x);
      if (li > j) fms_c(x, L[j], xj);
    }
  });
  return x;
}

// vector v (one value per lane) <- L^{-H} v  (back substitution with L^H)
template <int G, int DMAX>
DANSE_DEV cf bwd_vec_h(cf v, const cf (&L)[DMAX], int li, int D) {
  sfor_down<DMAX, 0>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    if (j < D) {
      if (li == j) v = (1.0f / L[j].re) * v;
      const cf uj = gbcast<G, j>(v);
      // lanes i < j: v_i -= conj(L[j][i]) * u_j ; L[j][i] is lane j's B[i]
      sfor<0, j>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const cf lji = gbcast<G, j>(L[i]);
        if (li == i) v = v - cmul(lji, uj);
      });
    }
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

// Householder reduction of the Hermitian C (rows in A) to tridiagonal form.
// Stores u_j in S.U[j][i], diag in S.ta, sub-diagonal in S.tb, |sub|^2 in S.te2.
template <int G, int DMAX>
DANSE_DEV void tridiag_rows(cf (&A)[DMAX], SolverLDS<DMAX>& S, int li, int D) {
  const bool act = li < D;
  sfor<0, (DMAX >= 2 ? DMAX - 2 : 0)>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    if (j < D - 2) {
      const cf xi = (act && li > j) ? A[j] : cf{0.0f, 0.0f};
      const float nrm2 = gsum<G>(abs2(xi));
      const cf x0 = gbcast<G, j + 1>(A[j]);
      const float nx = sqrtf(nrm2);
      const float ax0 = sqrtf(abs2(x0));
      cf u = cf{0.0f, 0.0f};
      if (nx > 0.0f) {
        const cf e = (ax0 > 0.0f) ? cf{x0.re / ax0, x0.im / ax0} : cf{1.0f, 0.0f};
        const float invn = 1.0f / sqrtf(2.0f * nx * (nx + ax0));
        u = xi;
        if (li == j + 1) u = u + nx * e;
        u = invn * u;
        // p = A u
        cf p = cf{0.0f, 0.0f};
        sfor<j + 1, DMAX>([&](auto cc) {
          constexpr int c = decltype(cc)::value;
          if (c < D) fma_c(p, A[c], gbcast<G, c>(u));
        });
        if (!act) p = cf{0.0f, 0.0f};
        const float Kr = gsum<G>(cmul(u, p).re);
        const cf q = p - Kr * u;
        sfor<j, DMAX>([&](auto cc) {
          constexpr int c = decltype(cc)::value;
          if (c < D) {
            const cf qc = gbcast<G, c>(q);
            const cf uc = gbcast<G, c>(u);
            // A[i][c] -= 2 (u_i conj(q_c) + q_i conj(u_c))
            cf t = mulc(u, qc) + mulc(q, uc);
            A[c] = A[c] - 2.0f * t;
          }
        });
      }
      if (li < DMAX) S.U[j][li] = u;
    }
  });
  // diagonal and sub-diagonal
  float a = 0.0f;
  cf b = cf{0.0f, 0.0f};
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (li == c) a = A[c].re;
    if constexpr (c >= 1) {
      if (li == c) b = A[c - 1];
    }
  });
  if (li < DMAX && li < D) S.ta[li] = a;
  if (li >= 1 && li < D && li < DMAX) {
    S.tb[li - 1] = b;
    S.te2[li - 1] = abs2(b);
  }
  __syncthreads();
}

// Number of eigenvalues of the real symmetric tridiagonal (ta, sqrt(te2)) below x.
template <int DMAX>
DANSE_DEV int sturm_count(const SolverLDS<DMAX>& S, int D, float x, float pivmin) {
  int cnt = 0;
  float q = S.ta[0] - x;
  if (fabsf(q) <= pivmin) q = -pivmin;
  cnt += (q < 0.0f);
  for (int i = 1; i < D; ++i) {
    q = (S.ta[i] - x) - S.te2[i - 1] / q;
    if (fabsf(q) <= pivmin) q = -pivmin;
    cnt += (q < 0.0f);
  }
  return cnt;
}

// Top-R eigenvalues (descending) by multisection; stored in S.lam.
template <int G, int DMAX>
DANSE_DEV void top_eigvals(SolverLDS<DMAX>& S, int li, int D, int R) {
  const bool act = li < D;
  float lo_i = 0.0f, hi_i = 0.0f, e2max = 0.0f;
  if (act) {
    const float em = (li >= 1) ? sqrtf(S.te2[li - 1]) : 0.0f;
    const float ep = (li + 1 < D) ? sqrtf(S.te2[li]) : 0.0f;
    lo_i = S.ta[li] - em - ep;
    hi_i = S.ta[li] + em + ep;
    e2max = (li + 1 < D) ? S.te2[li] : 0.0f;
  }
  float lo = gmin<G>(act ? lo_i : 3.0e38f);
  float hi = gmax<G>(act ? hi_i : -3.0e38f);
  const float scale = fmaxf(fabsf(lo), fabsf(hi));
  const float pivmin = 1.0e-30f * fmaxf(1.0f, gmax<G>(e2max));
  lo -= 2.0f * 1.2e-7f * scale + pivmin;
  hi += 2.0f * 1.2e-7f * scale + pivmin;
  // iterations: each shrinks the bracket by (G + 1)
  constexpr int NIT = (G >= 64) ? 5 : (G >= 16 ? 7 : 12);
  for (int r = 0; r < R; ++r) {
    float a = lo, b = hi;
    const int target = D - r;   // count(x) >= target  <=>  x > lambda_r
    for (int it = 0; it < NIT; ++it) {
      const float x = a + (b - a) * (float)(li + 1) / (float)(G + 1);
      const int cnt = sturm_count<DMAX>(S, D, x, pivmin);
      const uint64_t m = gballot<G>(cnt >= target);
      if (m == 0ull) {
        a = a + (b - a) * (float)G / (float)(G + 1);
      } else {
        const int first = __builtin_ctzll(m);
        const float xf = a + (b - a) * (float)(first + 1) / (float)(G + 1);
        const float xp = a + (b - a) * (float)first / (float)(G + 1);
        b = xf;
        a = xp;
      }
    }
    if (li == 0) S.lam[r] = 0.5f * (a + b);
    hi = b;   // next eigenvalue is not above this one
  }
  __syncthreads();
}

// Eigenvectors of the real tridiagonal for S.lam[0..R), by inverse iteration
// with partial pivoting (LAPACK dgtsv elimination) on lane 0 of the group,
// Gram-Schmidt against earlier vectors; then the complex phase fix
// v_i = phi_i x_i (phi_{i+1} = phi_i * tb_i / |tb_i|).  Results in S.v[r].
template <int DMAX>
DANSE_DEV void tri_eigvecs_lane(SolverLDS<DMAX>& S, int D, int R, float tnorm) {
  const float pert = 1.2e-7f * fmaxf(tnorm, 1e-30f);
  for (int r = 0; r < R; ++r) {
    const float lam = S.lam[r];
    for (int i = 0; i < D; ++i) S.x[r][i] = 1.0f + 0.1f * (float)((i * 7919 + r * 104729) % 13) / 13.0f;
    for (int it = 0; it < 3; ++it) {
      for (int i = 0; i < D; ++i) {
        S.d[i] = S.ta[i] - lam;
        S.rhs[i] = S.x[r][i];
        if (i + 1 < D) {
          const float e = sqrtf(S.te2[i]);
          S.dl[i] = e;
          S.du[i] = e;
        }
      }
      // elimination (dgtsv), rows i, i+1
      for (int i = 0; i + 1 < D; ++i) {
        if (fabsf(S.d[i]) >= fabsf(S.dl[i])) {
          if (S.d[i] == 0.0f) S.d[i] = pert;
          const float fact = S.dl[i] / S.d[i];
          S.d[i + 1] -= fact * S.du[i];
          S.rhs[i + 1] -= fact * S.rhs[i];
          S.dl[i] = 0.0f;
        } else {
          const float fact = S.d[i] / S.dl[i];
          S.d[i] = S.dl[i];
          const float temp = S.d[i + 1];
          S.d[i + 1] = S.du[i] - fact * temp;
          if (i + 2 < D) {
            S.dl[i] = S.du[i + 1];
            S.du[i + 1] = -fact * S.dl[i];
          } else {
            S.dl[i] = 0.0f;
          }
          S.du[i] = temp;
          const float tb = S.rhs[i];
          S.rhs[i] = S.rhs[i + 1];
          S.rhs[i + 1] = tb - fact * S.rhs[i + 1];
        }
      }
      if (S.d[D - 1] == 0.0f) S.d[D - 1] = pert;
      // back solve (upper, two super-diagonals du, dl)
      S.rhs[D - 1] = S.rhs[D - 1] / S.d[D - 1];
      if (D > 1) S.rhs[D - 2] = (S.rhs[D - 2] - S.du[D - 2] * S.rhs[D - 1]) / S.d[D - 2];
      for (int i = D - 3; i >= 0; --i)
        S.rhs[i] = (S.rhs[i] - S.du[i] * S.rhs[i + 1] - S.dl[i] * S.rhs[i + 2]) / S.d[i];
      // Gram-Schmidt against earlier vectors, normalise
      for (int q = 0; q < r; ++q) {
        float dot = 0.0f;
        for (int i = 0; i < D; ++i) dot += S.x[q][i] * S.rhs[i];
        for (int i = 0; i < D; ++i) S.rhs[i] -= dot * S.x[q][i];
      }
      float nrm = 0.0f, mx = 0.0f;
      for (int i = 0; i < D; ++i) mx = fmaxf(mx, fabsf(S.rhs[i]));
      mx = (mx > 0.0f) ? mx : 1.0f;
      for (int i = 0; i < D; ++i) {
        const float t = S.rhs[i] / mx;
        nrm += t * t;
      }
      const float inv = 1.0f / (mx * sqrtf(nrm));
      for (int i = 0; i < D; ++i) S.x[r][i] = S.rhs[i] * inv;
    }
    // phase fix
    cf phi = cf{1.0f, 0.0f};
    for (int i = 0; i < D; ++i) {
      S.v[r][i] = S.x[r][i] * phi;
      if (i + 1 < D) {
        const cf b = S.tb[i];
        const float ab = sqrtf(abs2(b));
        if (ab > 0.0f) phi = phi * cf{b.re / ab, b.im / ab};
      }
    }
  }
}

// Full GEVD filter: A = Ryy rows, B = Rnn rows (both destroyed).  Returns w_li.
template <int G, int DMAX>
DANSE_DEV cf gevd_filter(cf (&A)[DMAX], cf (&B)[DMAX], SolverLDS<DMAX>& S, int li, int D, int R, int ref,
                         bool& ok) {
  const bool act = li < D;
  ok = chol_rows<G, DMAX>(B, li, D);
  fwd_rows<G, DMAX>(A, B, li, D);             // A = L^{-1} Ryy
  herm_transpose<G, DMAX>(A, S.U, li);        // A = Ryy L^{-H}
  fwd_rows<G, DMAX>(A, B, li, D);             // A = L^{-1} Ryy L^{-H} = C
  tridiag_rows<G, DMAX>(A, S, li, D);
  top_eigvals<G, DMAX>(S, li, D, R);
  float tn = act ? (fabsf(S.ta[li]) + ((li + 1 < D) ? sqrtf(S.te2[li]) : 0.0f)) : 0.0f;
  tn = gmax<G>(tn);
  if (li == 0) tri_eigvecs_lane<DMAX>(S, D, R, tn);
  __syncthreads();
  // g = L^H e_ref : g_i = conj(L[ref][i])
  cf g = cf{0.0f, 0.0f};
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    const cf v = gbcast_rt<G>(B[c], ref);
    if (li == c) g = conjg(v);
  });
  cf w = cf{0.0f, 0.0f};
  for (int r = 0; r < R; ++r) {
    cf v = (act && li < DMAX) ? S.v[r][li] : cf{0.0f, 0.0f};
    // back-transform with the Householder vectors, last first
    for (int j = D - 3; j >= 0; --j) {
      const cf u = (act && li < DMAX) ? S.U[j][li] : cf{0.0f, 0.0f};
      const cf s = gsum<G>(cmul(u, v));
      v = v - 2.0f * (u * s);
    }
    const cf sr = gsum<G>(act ? cmul(v, g) : cf{0.0f, 0.0f});
    cf u = bwd_vec_h<G, DMAX>(v, B, li, D);
    const float coef = 1.0f - 1.0f / S.lam[r];
    w = w + coef * (u * sr);
  }
  return act ? w : cf{0.0f, 0.0f};
}

// MWF filter: A = Ryy rows, B = Rnn rows.  Returns w_li.
template <int G, int DMAX>
DANSE_DEV cf mwf_filter(cf (&A)[DMAX], const cf (&B)[DMAX], int li, int D, int ref, bool& ok) {
  const bool act = li < D;
  ok = chol_rows<G, DMAX>(A, li, D);
  cf r = cf{0.0f, 0.0f};
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c == ref) r = B[c];
  });
  if (!act) r = cf{0.0f, 0.0f};
  cf t = fwd_vec<G, DMAX>(r, A, li, D);
  cf u = bwd_vec_h<G, DMAX>(t, A, li, D);
  cf w = cf{(li == ref) ? 1.0f : 0.0f, 0.0f} - u;
  return act ? w : cf{0.0f, 0.0f};
}

}  // namespace danse
