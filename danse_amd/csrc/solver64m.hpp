// Mixed-precision wavefront solver for large filter dimensions
// (16 < D <= 64): one frequency bin per wavefront, lane i holds ROW i.
// (update_w / update_w_gevd, danse_toolbox/d_classes.py:3320-3387.)
//
// Same precision plan as the lane-per-bin classes (solver_mixed.hpp,
// DESIGN.md "Precision"): Rnn arrives in float64 and is factored and
// inverted in float64; Li = L^-1 is rounded to float32 and everything after
// it is float32 (C = Li Ryy Li^H, Householder tridiagonalisation,
// multisection, inverse iteration, back-transform, x = Li^H v).
//
// Dynamic (runtime D, pivot j) indexing goes through LDS, never through
// registers:
//   Cholesky   rows in registers (RowD), column j broadcast by readlane,
//              columns of L collected in LDS (U64[c][i] = L[i][c]);
//   inverse    in place in U64, column-descending: lane i forms
//              Li[i][j] = -(1/L[j][j]) sum_{k>j} Li[i][k] L[k][j], every L[k][j]
//              a broadcast LDS read;
//   congruence Y = Li A with the rows of A broadcast from LDS, then
//              C[i][c] = sum_k Y[i][k] conj(Li[c][k]) with the rows of Li
//              broadcast from LDS.
#pragma once
#include "solver64.hpp"
#include "solver_mixed.hpp"

namespace danse {
namespace big {

template <int DMAX>
struct RowD {
  static constexpr int NC = DMAX / 8;
  double re[DMAX], im[DMAX];
};
template <int C, int DMAX>
DANSE_DEV cd rsd(const RowD<DMAX>& X) {
  return cd{X.re[C], X.im[C]};
}
template <int C, int DMAX>
DANSE_DEV void wsd(RowD<DMAX>& X, cd v) {
  X.re[C] = v.re;
  X.im[C] = v.im;
}
template <int DMAX, int C = 0>
DANSE_DEV double rget1d(const double (&x)[DMAX], int j) {
  if constexpr (C == DMAX - 1) return x[C];
  else return (j == C) ? x[C] : rget1d<DMAX, C + 1>(x, j);
}
template <int DMAX>
DANSE_DEV cd rgetd(const RowD<DMAX>& X, int j) {
  return cd{rget1d<DMAX>(X.re, j), rget1d<DMAX>(X.im, j)};
}
DANSE_DEV double rld(double x, int lane) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
DANSE_DEV cd rld(cd x, int lane) { return cd{rld(x.re, lane), rld(x.im, lane)}; }

template <int DMAX>
struct LDSM {
  union {
    cd U64[DMAX][DMAX + 1];   // L, then Li (float64), by columns: U64[c][i] = X[i][c]
    struct {
      cf As[DMAX][DMAX + 1];  // rows of Ryy; then the Householder vectors
      cf Ls[DMAX][DMAX + 1];  // rows of Li (float32)
    } f;
  } m;
  float x[kRMax][DMAX];       // tridiagonal eigenvectors (Gram-Schmidt, rank > 1)
  cf g[64];                   // g = L^H e_ref (lane i: g_i)
};

// float64 Cholesky, rows in registers; on exit U64[c][i] = L[i][c] (c <= i,
// 0 above), the pivots' inverses in invd (lane i: 1 / L[i][i]).
template <int DMAX>
DANSE_DEV bool chol64_rows(RowD<DMAX>& B, cd (*U)[DMAX + 1], int li, int D, double& invd) {
  bool ok = true;
  invd = 0.0;
  for (int j = 0; j < D; ++j) {
    cd bj = rgetd(B, j);
    const double p0 = rld(bj.re, j);
    ok = ok && (p0 > 1e-300);
    const double piv = p0 > 1e-300 ? p0 : 1e-300;
    const double inv = lane::rsqrt64(piv);
    if (li == j) {
      bj = cd{piv * inv, 0.0};
      invd = inv;
    } else if (li > j) {
      bj = inv * bj;
    }
    if (li < DMAX) U[j][li] = (li >= j) ? bj : cd{0.0, 0.0};   // column j of L
    cols_after<DMAX>(j, [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      cd lcj = rld(bj, c);
      if (!(c > j)) lcj = cd{0.0, 0.0};
      cd x = rsd<c>(B);
      fms_cc(x, bj, lcj);
      wsd<c>(B, x);
    });
  }
  __syncthreads();
  return ok;
}

// In-place inverse of L held by columns in U (U[c][i] = L[i][c]), float64:
// column j from the last; lane i (> j) reads its row of Li (columns > j,
// already inverted) and the broadcast column j of L.
template <int DMAX>
DANSE_DEV void tri_inv64_cols(cd (*U)[DMAX + 1], int li, int D, double invd) {
  for (int j = D - 1; j >= 0; --j) {
    const double ajj = rld(invd, j);
    cd acc = cd{0.0, 0.0};
    if (li > j && li < D) {
      for (int k = j + 1; k <= li; ++k) fma_c(acc, U[k][li], U[j][k]);   // Li[i][k] L[k][j]
    }
    __syncthreads();   // every read of column j before it is replaced
    if (li == j) U[j][li] = cd{ajj, 0.0};
    else if (li > j && li < D) U[j][li] = (-ajj) * acc;
    __syncthreads();
  }
}

// Rank-R GEVD filter: A = Ryy rows (float32, destroyed), N = Rnn rows
// (float64, destroyed).  Returns w_li.
template <int DMAX, int RMAX>
DANSE_DEV cf gevd_filter_mixed(Row<DMAX>& A, RowD<DMAX>& N, LDSM<DMAX>& S, int li, int D, int R, int ref, bool& ok) {
  const bool act = li < D;
  double invd;
  ok = chol64_rows<DMAX>(N, S.m.U64, li, D, invd);
  // g = L^H e_ref: g_i = conj(L[ref][i]) = conj(U[i][ref]) for i <= ref
  const cf gi = (li <= ref && li < D) ? conjg(cfk(S.m.U64[li][ref])) : cf{0.0f, 0.0f};
  tri_inv64_cols<DMAX>(S.m.U64, li, D, invd);
  // rows of Li in float32: registers (Lr) and, after the union switches to
  // its float32 view, LDS (Ls)
  Row<DMAX> Lr;
  rzero(Lr);
  cols_below<DMAX>(D, [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c < D && li < DMAX) ws<c>(Lr, cfk(S.m.U64[c][li]));
  });
  __syncthreads();
  if (li < DMAX) {
    sfor<0, DMAX>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      S.m.f.Ls[li][c] = rs<c>(Lr);
      S.m.f.As[li][c] = rs<c>(A);
    });
  }
  S.g[li] = gi;
  __syncthreads();
  // Y = Li A: Y[i][c] = sum_{k <= i} Li[i][k] A[k][c]
  Row<DMAX> Y;
  rzero(Y);
  cols_below<DMAX>(D, [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if (k < D) {
      const cf lik = rs<k>(Lr);
      cols_below<DMAX>(D, [&](auto cc) {
        constexpr int c = decltype(cc)::value;
        cf y = rs<c>(Y);
        fma_c(y, lik, S.m.f.As[k][c]);
        ws<c>(Y, y);
      });
    }
  });
  // C[i][c] = sum_{k <= c} Y[i][k] conj(Li[c][k])  (rows into A)
  rzero(A);
  cols_below<DMAX>(D, [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c < D) {
      cf acc = cf{0.0f, 0.0f};
      sfor<0, c + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        acc = acc + mulc(rs<k>(Y), S.m.f.Ls[c][k]);
      });
      if (!act) acc = cf{0.0f, 0.0f};
      if (li == c) acc.im = 0.0f;
      ws<c>(A, acc);
    }
  });
  __syncthreads();
  // float32 eigen part (solver64.hpp)
  float ta;
  cf tb;
  tridiag<DMAX>(A, S.m.f.As, li, D, ta, tb);   // Householder vectors over the rows of Ryy
  const float e2own = abs2(tb);
  float te2 = __shfl_down(e2own, 1);
  if (li + 1 >= D) te2 = 0.0f;
  const float ta_ = act ? ta : 0.0f;
  float lam[kRMax];
  float tnorm;
  top_eigvals<RMAX>(ta_, te2, li, D, R, lam, tnorm);
  const float pert = 1.2e-7f * fmaxf(tnorm, 1e-30f);
  const float te = fsqrt(te2);
  cf w = cf{0.0f, 0.0f};
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (r > 0) {
      if (r >= R) return;
    }
    const float x = tri_eigvec<DMAX>(ta_, te, li, D, lam[r], pert, r, S.x);
    cf phi = cf{1.0f, 0.0f};
    cf v = cf{0.0f, 0.0f};
    for (int i = 0; i < D; ++i) {
      if (li == i) v = x * phi;
      if (i + 1 < D) {
        const cf bb = rl(tb, i + 1);
        const float ab2 = abs2(bb);
        const float iab = frsq(ab2);
        if (ab2 > 0.0f) phi = phi * cf{bb.re * iab, bb.im * iab};
      }
    }
    if (r + 1 < R) {
      if (li < DMAX) S.x[r][li] = x;
      __syncthreads();
    }
    for (int j = D - 3; j >= 0; --j) {
      const cf u = (li < DMAX) ? S.m.f.As[j][li] : cf{0.0f, 0.0f};
      const cf s = gsum<64>(cmul(u, v));
      fms_c(v, 2.0f * u, s);
    }
    const cf sr = gsum<64>(cmul(v, S.g[li]));
    // x = Li^H v: x_i = sum_{k >= i} conj(Li[k][i]) v_k
    cf xv = cf{0.0f, 0.0f};
    cols_below<DMAX>(D, [&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if (k < D) {
        const cf vk = rl(v, k);
        const cf lki = (li <= k && li < DMAX) ? S.m.f.Ls[k][li] : cf{0.0f, 0.0f};
        xv = xv + cmul(lki, vk);
      }
    });
    const float coef = 1.0f - frcp(lam[r]);
    w = w + coef * (xv * sr);
  });
  return act ? w : cf{0.0f, 0.0f};
}

// MWF filter, float64: X = Ryy rows (float64, destroyed), ncol_li = Rnn[li][ref].
// w = Ryy^-1 (Ryy - Rnn) e_ref: Cholesky of Ryy, then the two substitutions
// with the columns of L in LDS.
template <int DMAX>
DANSE_DEV cf mwf_filter64(RowD<DMAX>& X, cd ncol, LDSM<DMAX>& S, int li, int D, int ref, bool& ok) {
  const bool act = li < D;
  cd r = rgetd(X, ref) - ncol;   // (Ryy - Rnn)[li][ref], as the reference forms it
  if (!act) r = cd{0.0, 0.0};
  double invd;
  ok = chol64_rows<DMAX>(X, S.m.U64, li, D, invd);
  // r <- L^-1 r (forward): r_j final at step j
  for (int j = 0; j < D; ++j) {
    const double ij = rld(invd, j);
    if (li == j) r = ij * r;
    const cd rj = rld(r, j);
    if (li > j && li < D) fms_c(r, S.m.U64[j][li], rj);   // r_i -= L[i][j] r_j
  }
  // r <- L^-H r (backward): (L^H)[i][k] = conj(L[k][i]) = conj(U[i][k])
  for (int j = D - 1; j >= 0; --j) {
    const double ij = rld(invd, j);
    if (li == j) r = ij * r;
    const cd rj = rld(r, j);
    if (li < j) fms_c(r, conjg(S.m.U64[li][j]), rj);
  }
  return act ? cfk(r) : cf{0.0f, 0.0f};
}
// ... with the float32 Ryy rows of the online engine (promoted)
template <int DMAX>
DANSE_DEV cf mwf_filter_mixed(const Row<DMAX>& A, cd ncol, LDSM<DMAX>& S, int li, int D, int ref, bool& ok) {
  RowD<DMAX> X;
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    wsd<c>(X, cdk(rs<c>(A)));
  });
  return mwf_filter64<DMAX>(X, ncol, S, li, D, ref, ok);
}

}  // namespace big
}  // namespace danse
