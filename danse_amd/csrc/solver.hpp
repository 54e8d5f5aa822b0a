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
  float x[kRMax][DMAX];     // real tridiagonal eigenvectors (Gram-Schmidt of rank > 1)
  cf tb[DMAX];              // complex sub-diagonal T[i+1][i] (phase fix)
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
DANSE_DEV void tridiag_rows(cf (&A)[DMAX], SolverLDS<DMAX>& S, int li, int D, float& a, cf& b) {
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
  // diagonal and sub-diagonal element of my row
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
DANSE_DEV void gather_tri(Tri<DMAX>& T, float a, cf b, int D, cf* tb, int li) {
  const float e2 = abs2(b);
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    T.a[c] = (c < D) ? gbcast<G, c>(a) : 0.0f;
    if constexpr (c + 1 < DMAX) {
      const float ec = gbcast<G, c + 1>(e2);
      T.e2[c] = (c + 1 < D) ? ec : 0.0f;
    } else {
      T.e2[c] = 0.0f;
    }
  });
  if (li >= 1 && li < DMAX) tb[li - 1] = (li < D) ? b : cf{0.0f, 0.0f};
  if (li == DMAX - 1 || li == D - 1) tb[DMAX - 1] = cf{0.0f, 0.0f};
  __syncthreads();
}

// Number of eigenvalues of the real symmetric tridiagonal (a, sqrt(e2)) below x.
template <int DMAX>
DANSE_DEV int sturm_reg(const Tri<DMAX>& T, int D, float x, float pivmin) {
  int cnt = 0;
  float q = 1.0f;
  sfor<0, DMAX>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if (i < D) {
      float qn;
      if constexpr (i == 0) qn = T.a[0] - x;
      else qn = (T.a[i] - x) - __fdividef(T.e2[i - 1], q);
      if (fabsf(qn) <= pivmin) qn = -pivmin;
      q = qn;
      cnt += (q < 0.0f) ? 1 : 0;
    }
  });
  return cnt;
}

// Top-R eigenvalues (descending) by multisection: every lane of the group
// evaluates one Sturm count per pass, the bracket shrinks by (G + 1).
template <int G, int DMAX, int RMAX>
DANSE_DEV void top_eigvals(const Tri<DMAX>& T, int li, int D, int R, float (&lam)[kRMax], float& tnorm) {
  float lo = 3.0e38f, hi = -3.0e38f, e2max = 0.0f;
  tnorm = 0.0f;
  sfor<0, DMAX>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if (i < D) {
      float em = 0.0f;
      if constexpr (i >= 1) em = sqrtf(T.e2[i - 1]);
      const float ep = (i + 1 < D) ? sqrtf(T.e2[i]) : 0.0f;
      lo = fminf(lo, T.a[i] - em - ep);
      hi = fmaxf(hi, T.a[i] + em + ep);
      if (i + 1 < D) e2max = fmaxf(e2max, T.e2[i]);
      tnorm = fmaxf(tnorm, fabsf(T.a[i]) + em + ep);
    }
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
      const int target = D - r;   // count(x) >= target  <=>  x > lambda_r
      for (int it = 0; it < NIT; ++it) {
        const float step = (b - a) / (float)(G + 1);
        const float x = a + step * (float)(li + 1);
        const int cnt = sturm_reg<DMAX>(T, D, x, pivmin);
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
template <int DMAX>
DANSE_DEV void tri_eigvec(const Tri<DMAX>& T, int D, float lam, float pert, int r, const float (*prev)[DMAX],
                          float (&x)[DMAX]) {
  sfor<0, DMAX>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    x[i] = (i < D) ? 1.0f + 0.1f * (float)((i * 7919 + r * 104729) % 13) / 13.0f : 0.0f;
  });
  for (int it = 0; it < 3; ++it) {
    float d[DMAX], dl[DMAX], du[DMAX], rhs[DMAX];
    sfor<0, DMAX>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      d[i] = T.a[i] - lam;
      const float e = sqrtf(T.e2[i]);
      dl[i] = e;
      du[i] = e;
      rhs[i] = x[i];
    });
    sfor<0, DMAX - 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if (i + 1 < D) {
        const bool swap = fabsf(d[i]) < fabsf(dl[i]);
        const float di = (d[i] == 0.0f) ? pert : d[i];
        const float f1 = dl[i] / di;           // no interchange
        const float f2 = d[i] / dl[i];         // interchange rows i, i+1
        const float d1 = d[i + 1];
        const float duI = du[i];
        float du1 = 0.0f;
        if constexpr (i + 1 < DMAX) du1 = du[i + 1];
        const bool has2 = (i + 2 < D);
        d[i] = swap ? dl[i] : di;
        d[i + 1] = swap ? (duI - f2 * d1) : (d1 - f1 * duI);
        dl[i] = (swap && has2) ? du1 : 0.0f;   // second super-diagonal
        if constexpr (i + 1 < DMAX) {
          if (has2) du[i + 1] = swap ? -f2 * du1 : du1;
        }
        du[i] = swap ? d1 : duI;
        const float ri = rhs[i], ri1 = rhs[i + 1];
        rhs[i] = swap ? ri1 : ri;
        rhs[i + 1] = swap ? (ri - f2 * ri1) : (ri1 - f1 * ri);
      }
    });
    // back solve
    sfor_down<DMAX, 0>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if (i < D) {
        float acc = rhs[i];
        if constexpr (i + 1 < DMAX) {
          if (i + 1 < D) acc -= du[i] * rhs[i + 1];
        }
        if constexpr (i + 2 < DMAX) {
          if (i + 2 < D) acc -= dl[i] * rhs[i + 2];
        }
        const float di = (d[i] == 0.0f) ? pert : d[i];
        rhs[i] = acc / di;
      }
    });
    for (int q = 0; q < r; ++q) {
      float dot = 0.0f;
      sfor<0, DMAX>([&](auto ic) { constexpr int i = decltype(ic)::value; dot += prev[q][i] * rhs[i]; });
      sfor<0, DMAX>([&](auto ic) { constexpr int i = decltype(ic)::value; rhs[i] -= dot * prev[q][i]; });
    }
    float mx = 0.0f;
    sfor<0, DMAX>([&](auto ic) { mx = fmaxf(mx, fabsf(rhs[decltype(ic)::value])); });
    mx = (mx > 0.0f) ? mx : 1.0f;
    const float imx = 1.0f / mx;
    float nrm = 0.0f;
    sfor<0, DMAX>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      rhs[i] *= imx;
      nrm += rhs[i] * rhs[i];
    });
    const float inv = 1.0f / sqrtf(nrm);
    sfor<0, DMAX>([&](auto ic) { constexpr int i = decltype(ic)::value; x[i] = (i < D) ? rhs[i] * inv : 0.0f; });
  }
}

// Full GEVD filter: A = Ryy rows, B = Rnn rows (both destroyed).  Returns w_li.
// RMAX bounds the (runtime) rank R at compile time.
template <int G, int DMAX, int RMAX>
DANSE_DEV cf gevd_filter(cf (&A)[DMAX], cf (&B)[DMAX], SolverLDS<DMAX>& S, int li, int D, int R, int ref,
                         bool& ok) {
  const bool act = li < D;
  ok = chol_rows<G, DMAX>(B, li, D);
  fwd_rows<G, DMAX>(A, B, li, D);             // A = L^{-1} Ryy
  herm_transpose<G, DMAX>(A, S.U, li);        // A = Ryy L^{-H}
  fwd_rows<G, DMAX>(A, B, li, D);             // A = L^{-1} Ryy L^{-H} = C
  float ta;
  cf tb;
  tridiag_rows<G, DMAX>(A, S, li, D, ta, tb);
  Tri<DMAX> T;
  gather_tri<G, DMAX>(T, ta, tb, D, S.tb, li);
  float lam[kRMax];
  float tnorm;
  top_eigvals<G, DMAX, RMAX>(T, li, D, R, lam, tnorm);
  const float pert = 1.2e-7f * fmaxf(tnorm, 1e-30f);
  // g = L^H e_ref : g_i = conj(L[ref][i])
  cf g = cf{0.0f, 0.0f};
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    const cf v = gbcast_rt<G>(B[c], ref);
    if (li == c) g = conjg(v);
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
      const cf b = (i + 1 < D) ? S.tb[i] : cf{0.0f, 0.0f};
      const float ab2 = abs2(b);
      if (ab2 > 0.0f) {
        const float iab = rsqrtf(ab2);
        phi = phi * cf{b.re * iab, b.im * iab};
      }
    });
    if (r + 1 < R) {
      // keep x for Gram-Schmidt of the next eigenvectors
      float xi = 0.0f;
      sfor<0, DMAX>([&](auto ic) { constexpr int i = decltype(ic)::value; if (li == i) xi = x[i]; });
      if (li < DMAX) S.x[r][li] = xi;
      __syncthreads();
    }
    if (!act) v = cf{0.0f, 0.0f};
    // back-transform with the Householder vectors, last first
    for (int j = D - 3; j >= 0; --j) {
      const cf u = (act && li < DMAX) ? S.U[j][li] : cf{0.0f, 0.0f};
      const cf s = gsum<G>(cmul(u, v));
      v = v - 2.0f * (u * s);
    }
    const cf sr = gsum<G>(act ? cmul(v, g) : cf{0.0f, 0.0f});
    cf u = bwd_vec_h<G, DMAX>(v, B, li, D);
    const float coef = 1.0f - 1.0f / lam[r];
    w = w + coef * (u * sr);
  });
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
