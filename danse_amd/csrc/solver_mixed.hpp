// Mixed-precision lane-per-bin filter update (D <= kLaneMaxD): one frequency
// bin per LANE, update_w / update_w_gevd (danse_toolbox/d_classes.py:
// 3320-3387).
//
// Precision plan (measured with scripts/precision_probe.py on the float64
// oracle, DESIGN.md "Precision"): the GEVD filter is conditioned by
// cond(Rnn), so
//   * Rnn is stored and averaged in float64 (PTriD), factored in float64:
//       Rnn = L L^H, Li = L^-1 (in place, float64),
//   * Li is then rounded to float32, and everything after it runs in
//     float32: C = Li Ryy Li^H (congruence, from the float32 Ryy), the
//     Householder tridiagonalisation, bisection, inverse iteration and
//     back-transform (solver1.hpp), x = Li^H v and g = L^H e_ref.
// That plan leaves the float64 oracle's filters unchanged to p99 3e-6
// (D = 11) / 6e-6 (D = 19); rounding Rnn to float32 anywhere before the
// factorisation and inverse costs p99 3e-5 .. 4e-4 (SCM storage alone 1e-4
// at D = 11, 4e-4 at D = 19).
//
// MWF: w = Ryy^-1 (Ryy - Rnn) e_ref, Cholesky of Ryy and both solves in
// float64 (Ryy promoted), the difference column formed in float64.
#pragma once
#include "solver1.hpp"

namespace danse {
namespace lane {

// Packed lower triangle of complex doubles in this lane's registers.
template <int D>
struct PTriD {
  cd a[tri_n(D)];
};

template <int I, int J, int D>
DANSE_DEV cd hermd(const PTri<D>& X) {
  if constexpr (I >= J) return cdk(X.a[P(I, J)]);
  else return conjg(cdk(X.a[P(J, I)]));
}
template <int I, int J, int D>
DANSE_DEV cd hermd(const PTriD<D>& X) {
  if constexpr (I >= J) return X.a[P(I, J)];
  else return conjg(X.a[P(J, I)]);
}

// 1 / sqrt(x), float64: hardware estimate + two Newton steps (no IEEE
// divide / sqrt sequences on the pivot chain).
DANSE_DEV double rsqrt64(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = y * fma(-0.5 * x * y, y, 1.5);
  y = y * fma(-0.5 * x * y, y, 1.5);
  return y;
}

// Right-looking Cholesky in place, float64: X = L L^H (lower, real diagonal);
// invd[j] = 1 / L[j][j].
template <int D>
DANSE_DEV bool chol64(PTriD<D>& X, double (&invd)[D]) {
  bool ok = true;
  sfor<0, D>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const double p0 = X.a[P(j, j)].re;
    ok = ok && (p0 > 1e-300);
    const double piv = p0 > 1e-300 ? p0 : 1e-300;
    const double inv = rsqrt64(piv);
    invd[j] = inv;
    X.a[P(j, j)] = cd{piv * inv, 0.0};
    sfor<j + 1, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      X.a[P(i, j)] = inv * X.a[P(i, j)];
    });
    sfor<j + 1, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const cd lij = X.a[P(i, j)];
      sfor<j + 1, i + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        fms_cc(X.a[P(i, k)], lij, X.a[P(k, j)]);   // X[i][k] -= L[i][j] conj(L[k][j])
      });
    });
  });
  return ok;
}

// g = L^H e_ref (g_i = conj(L[ref][i]), i <= ref), float32; ref is a runtime
// value, selected through a static chain (no dynamic register indexing).
template <int D>
DANSE_DEV void ref_row(const PTriD<D>& L, int ref, cf (&g)[D]) {
  sfor<0, D>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    cf v = cf{0.0f, 0.0f};
    sfor<i, D>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if (r == ref) v = conjg(cfk(L.a[P(r, i)]));
    });
    g[i] = v;
  });
}

// In-place inverse of the lower-triangular L, float64:
// Li[i][j] = -(1 / L[j][j]) sum_{k=j+1..i} Li[i][k] L[k][j], columns from the
// last, rows from the bottom (so every L entry is read before it is replaced).
template <int D>
DANSE_DEV void tri_inv64(PTriD<D>& X, const double (&invd)[D]) {
  sfor_down<D, 0>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const double ajj = invd[j];
    X.a[P(j, j)] = cd{ajj, 0.0};
    sfor_down<D, j + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      cd acc = cd{0.0, 0.0};
      sfor<j + 1, i + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        fma_c(acc, X.a[P(i, k)], X.a[P(k, j)]);
      });
      X.a[P(i, j)] = (-ajj) * acc;
    });
  });
}

// The float32 copy of Li lives in LDS, one 8-byte column per lane
// ([entry][lane]: every access of a wave is 512 contiguous bytes, conflict
// free; a lane only touches its own column, so no barrier is needed), which
// leaves the register file to C and the Householder work.
template <int D>
struct LdsTri {
  cf (*p)[64];
  int lane;
  template <int I, int J>
  DANSE_DEV cf at() const { return p[P(I, J)][lane]; }
};
template <int D>
DANSE_DEV void store_tri(const PTriD<D>& X, cf (*p)[64], int lane) {
  sfor<0, tri_n(D)>([&](auto ec) { p[decltype(ec)::value][lane] = cfk(X.a[decltype(ec)::value]); });
}

// A <- Li A Li^H (A: packed Hermitian, Li: lower; float32).  Lower column j
// of the result needs A's columns 0..j only, so the columns are produced
// from the last to the first and each overwrites the one it no longer needs
// (no second triangle in registers).
//   u = A conj(Li[j][0..j])^T,  C[i][j] = sum_{k<=i} Li[i][k] u[k]  (i >= j)
// (The compiler barriers keep each row of Li in registers for one use only:
// otherwise the LDS loads are merged over all rows, and Li's 2 D(D+1)
// floats join C's in the register file.)
template <int D, typename LM>
DANSE_DEV void congruence(PTri<D>& A, const LM& Li) {
  sfor_down<D, 0>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    asm volatile("" ::: "memory");
    cf u[D];
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      cf acc = cf{0.0f, 0.0f};
      sfor<0, j + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        herm_mac<i, k, true, false>(acc, A, Li.template at<j, k>());
      });
      u[i] = acc;
    });
    sfor<j, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      asm volatile("" ::: "memory");
      cf acc = cf{0.0f, 0.0f};
      sfor<0, i + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        cmac<false, false, false>(acc, Li.template at<i, k>(), u[k]);
      });
      if constexpr (i == j) acc.im = 0.0f;
      A.a[P(i, j)] = acc;
    });
  });
}

// Rank-R GEVD filter from C (in A, destroyed), Li (float32 copy of L^-1) and
// g = L^H e_ref:  w = sum_r (1 - 1/l_r) (Li^H v_r) (v_r^H g).
template <int D, int RMAX, typename LM>
DANSE_DEV void gevd_filter_mixed(PTri<D>& A, const LM& Li, const cf (&g)[D], int R, cf (&wv)[D]) {
  sfor<0, D>([&](auto ic) { wv[decltype(ic)::value] = cf{0.0f, 0.0f}; });
  gevd_eig<D, RMAX>(A, R, [&](int r, float lam, cf (&v)[D]) {
    cf sr = cf{0.0f, 0.0f};
    sfor<0, D>([&](auto ic) { sr = sr + cmul(v[decltype(ic)::value], g[decltype(ic)::value]); });
    const cf cs = (1.0f - 1.0f / lam) * sr;
    // x_i = sum_{k >= i} conj(Li[k][i]) v_k
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      asm volatile("" ::: "memory");
      cf x = cf{0.0f, 0.0f};
      sfor<i, D>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        cmac<true, false, false>(x, Li.template at<k, i>(), v[k]);
      });
      fma_c(wv[i], x, cs);
    });
  });
}

// MWF filter in float64: X = Ryy (float64, destroyed), ncol = Rnn[:, ref].
template <int D>
DANSE_DEV bool mwf_filter64(PTriD<D>& X, const cd (&ncol)[D], int ref, cf (&wv)[D]) {
  cd r[D];
  sfor<0, D>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    cd c = cd{0.0, 0.0};
    sfor<0, D>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if (k == ref) c = hermd<i, k>(X);
    });
    r[i] = c - ncol[i];
  });
  double invd[D];
  const bool ok = chol64<D>(X, invd);
  // r <- L^-1 r
  sfor<0, D>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    cd acc = r[i];
    sfor<0, i>([&](auto kc) { fms_c(acc, X.a[P(i, decltype(kc)::value)], r[decltype(kc)::value]); });
    r[i] = invd[i] * acc;
  });
  // r <- L^-H r
  sfor_down<D, 0>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    cd acc = r[i];
    sfor<i + 1, D>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      fms_c(acc, conjg(X.a[P(k, i)]), r[k]);
    });
    r[i] = invd[i] * acc;
  });
  sfor<0, D>([&](auto ic) { wv[decltype(ic)::value] = cfk(r[decltype(ic)::value]); });
  return ok;
}
// ... with the float32 Ryy of the online engine (promoted)
template <int D>
DANSE_DEV bool mwf_filter_mixed(const PTri<D>& A, const cd (&ncol)[D], int ref, cf (&wv)[D]) {
  PTriD<D> X;
  sfor<0, tri_n(D)>([&](auto ec) { X.a[decltype(ec)::value] = cdk(A.a[decltype(ec)::value]); });
  return mwf_filter64<D>(X, ncol, ref, wv);
}

}  // namespace lane
}  // namespace danse
