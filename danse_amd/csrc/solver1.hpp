// Lane-per-bin solvers for small filter dimensions (D <= kLaneMaxD): one
// frequency bin per LANE, both SCMs as packed lower triangles in that lane's
// registers.  (update_w / update_w_gevd, danse_toolbox/d_classes.py:
// 3320-3387.)  No cross-lane traffic at all: every instruction does useful
// work for 64 bins, where the lane-group solvers (solver.hpp) spend most of
// their issue slots on row broadcasts and idle lanes.
//
// This file holds the float32 eigen part of the GEVD, statically unrolled on
// D (the float64 factorisation in front of it is solver_mixed.hpp):
//   C = Q T Q^H                               (Householder, complex subdiag)
//   top-R eigenvalues of |T| by bisection     (Sturm counts)
//   x_r by inverse iteration on |T|, v_r = Q P x_r (P: subdiagonal phases)
#pragma once
#include "solver.hpp"

namespace danse {
namespace lane {

constexpr int tri_n(int D) { return D * (D + 1) / 2; }
constexpr int P(int i, int j) { return i * (i + 1) / 2 + j; }   // i >= j

// Packed lower triangle in this lane's registers ...
template <int D>
struct PTri {
  cf a[tri_n(D)];
  template <int I, int J>
  DANSE_DEV cf at() const { return a[P(I, J)]; }
};
// Full Hermitian element (i, j) from the packed lower triangle.
template <int I, int J, int D>
DANSE_DEV cf herm(const PTri<D>& X) {
  if constexpr (I >= J) return X.a[P(I, J)];
  else return conjg(X.a[P(J, I)]);
}
// acc += (NEG ? -1 : 1) herm(X)[i][j] op(b) (op = conj where CB), one packed
// complex MAC with the conjugation folded into its modifiers
template <int I, int J, bool CB, bool NEG, int D>
DANSE_DEV void herm_mac(cf& acc, const PTri<D>& X, cf b) {
  if constexpr (I >= J) cmac<false, CB, NEG>(acc, X.a[P(I, J)], b);
  else cmac<true, CB, NEG>(acc, X.a[P(J, I)], b);
}

// Householder tridiagonalisation of the Hermitian A (packed lower), in
// place: on exit A[i][i].re is the diagonal, b[i] = T[i][i-1] (complex) for
// i >= 1, and reflector j (H_j = I - 2 u u^H, ||u|| = 1, u supported on rows
// j+1..D-1) is stored as u0[j] = u_{j+1} and A[i][j] = u_i for i >= j+2.
template <int D>
DANSE_DEV void tridiag(PTri<D>& A, cf (&u0)[D], cf (&b)[D]) {
  b[0] = cf{0.0f, 0.0f};
  sfor<0, (D >= 2 ? D - 2 : 0)>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    float nrm2 = 0.0f;
    sfor<j + 1, D>([&](auto ic) { nrm2 += abs2(A.a[P(decltype(ic)::value, j)]); });
    const cf x0 = A.a[P(j + 1, j)];
    const float ax02 = abs2(x0);
    const float nx = fsqrt(nrm2);
    const float ax0 = fsqrt(ax02);
    const float iax0 = frsq(ax02);
    const cf e = csel(ax02 > 0.0f, cf{x0.re * iax0, x0.im * iax0}, cf{1.0f, 0.0f});
    const float invn = (nrm2 > 1e-30f) ? frsq(2.0f * nx * (nx + ax0)) : 0.0f;
    cf u[D];
    sfor<j + 1, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      cf v = A.a[P(i, j)];
      if constexpr (i == j + 1) v = v + nx * e;
      u[i] = invn * v;
    });
    // p = A~ u on the trailing block
    cf p[D];
    sfor<j + 1, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      cf acc = cf{0.0f, 0.0f};
      sfor<j + 1, D>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        herm_mac<i, k, false, false>(acc, A, u[k]);
      });
      p[i] = acc;
    });
    float Kr = 0.0f;
    sfor<j + 1, D>([&](auto ic) { Kr += cmul(u[decltype(ic)::value], p[decltype(ic)::value]).re; });
    cf q[D], u2[D];
    sfor<j + 1, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      q[i] = p[i] - Kr * u[i];
      u2[i] = 2.0f * u[i];
    });
    // A~ -= 2 (u q^H + q u^H), lower part
    sfor<j + 1, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      sfor<j + 1, i + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        cf t = A.a[P(i, k)];
        cmac<false, true, true>(t, u2[i], q[k]);
        cmac<false, true, true>(t, q[i], u2[k]);
        if constexpr (i == k) t.im = 0.0f;
        A.a[P(i, k)] = t;
      });
    });
    b[j + 1] = cf{-nx * e.re, -nx * e.im};
    u0[j] = u[j + 1];
    sfor<j + 2, D>([&](auto ic) { A.a[P(decltype(ic)::value, j)] = u[decltype(ic)::value]; });
  });
  if constexpr (D >= 2) b[D - 1] = A.a[P(D - 1, D - 2)];
}

// Sturm count of the real symmetric tridiagonal (a, e2 = |b|^2) below x.
template <int D>
DANSE_DEV int sturm(const float (&a)[D], const float (&e2)[D], float x, float pivmin) {
  int cnt = 0;
  float q = 1.0f;
  sfor<0, D>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    float qn;
    if constexpr (i == 0) qn = a[0] - x;
    else qn = (a[i] - x) - e2[i] * frcp(q);
    if (fabsf(qn) <= pivmin) qn = -pivmin;
    q = qn;
    cnt += (q < 0.0f) ? 1 : 0;
  });
  return cnt;
}

// Eigenvector of the tridiagonal (a, |b| = sqrt(e2)) for eigenvalue lam by inverse
// iteration: the pivoted elimination of solver.hpp::tri_eigvec, per lane.
template <int D, int RMAX>
DANSE_DEV void tri_eigvec(const float (&a)[D], const float (&e2)[D], float lam, float pert, int r,
                          const float (&prev)[RMAX][D], float (&x)[D]) {
  sfor<0, D>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    x[i] = 1.0f + 0.1f * (float)((i * 7919 + r * 104729) % 13) / 13.0f;
  });
  for (int it = 0; it < 2; ++it) {
    float d[D], dl[D], du[D], rhs[D];
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      d[i] = a[i] - lam;
      if constexpr (i + 1 < D) dl[i] = fsqrt(e2[i + 1]);   // |T[i+1][i]|
      else dl[i] = 0.0f;
      du[i] = dl[i];
      rhs[i] = x[i];
    });
    sfor<0, D - 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const bool swap = fabsf(d[i]) < fabsf(dl[i]);
      const float di = (d[i] == 0.0f) ? pert : d[i];
      const float f1 = dl[i] * frcp(di);
      const float f2 = d[i] * frcp(dl[i]);
      const float d1 = d[i + 1];
      const float duI = du[i];
      float du1 = 0.0f;
      if constexpr (i + 2 < D) du1 = du[i + 1];
      d[i] = swap ? dl[i] : di;
      d[i + 1] = swap ? (duI - f2 * d1) : (d1 - f1 * duI);
      dl[i] = swap ? du1 : 0.0f;
      if constexpr (i + 2 < D) du[i + 1] = swap ? -f2 * du1 : du1;
      du[i] = swap ? d1 : duI;
      const float ri = rhs[i], ri1 = rhs[i + 1];
      rhs[i] = swap ? ri1 : ri;
      rhs[i + 1] = swap ? (ri - f2 * ri1) : (ri1 - f1 * ri);
    });
    sfor_down<D, 0>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      float acc = rhs[i];
      if constexpr (i + 1 < D) acc -= du[i] * rhs[i + 1];
      if constexpr (i + 2 < D) acc -= dl[i] * rhs[i + 2];
      const float di = (d[i] == 0.0f) ? pert : d[i];
      rhs[i] = acc * frcp(di);
    });
    sfor<0, RMAX>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      if (q < r) {
        float dot = 0.0f;
        sfor<0, D>([&](auto ic) { dot += prev[q][decltype(ic)::value] * rhs[decltype(ic)::value]; });
        sfor<0, D>([&](auto ic) { rhs[decltype(ic)::value] -= dot * prev[q][decltype(ic)::value]; });
      }
    });
    float mx = 0.0f;
    sfor<0, D>([&](auto ic) { mx = fmaxf(mx, fabsf(rhs[decltype(ic)::value])); });
    mx = (mx > 0.0f) ? mx : 1.0f;
    const float imx = frcp(mx);
    float nrm = 0.0f;
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      rhs[i] *= imx;
      nrm += rhs[i] * rhs[i];
    });
    const float inv = frsq(nrm);
    sfor<0, D>([&](auto ic) { x[decltype(ic)::value] = rhs[decltype(ic)::value] * inv; });
  }
}

// Top-R eigenpairs of the Hermitian C (packed lower, destroyed):
// Householder tridiagonalisation, bisection for the eigenvalues (descending),
// inverse iteration on |T|, subdiagonal phases and the back-transform.
// fn(r, lambda_r, v_r) is called once per rank r < R (v_r unit 2-norm).
template <int D, int RMAX, typename Fn>
DANSE_DEV void gevd_eig(PTri<D>& A, int R, Fn&& fn) {
  cf u0[D], b[D];
  tridiag<D>(A, u0, b);
  float ta[D], e2[D];
  sfor<0, D>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    ta[i] = A.a[P(i, i)].re;
    e2[i] = abs2(b[i]);   // e2[0] = 0
  });
  // Gershgorin bracket
  float lo = 3.0e38f, hi = -3.0e38f, e2max = 0.0f, tnorm = 0.0f;
  sfor<0, D>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    float ep = 0.0f;
    if constexpr (i + 1 < D) ep = fsqrt(e2[i + 1]);
    const float em = fsqrt(e2[i]);
    lo = fminf(lo, ta[i] - em - ep);
    hi = fmaxf(hi, ta[i] + em + ep);
    e2max = fmaxf(e2max, e2[i]);
    tnorm = fmaxf(tnorm, fabsf(ta[i]) + em + ep);
  });
  const float scale = fmaxf(fabsf(lo), fabsf(hi));
  const float pivmin = 1.0e-30f * fmaxf(1.0f, e2max);
  lo -= 2.0f * 1.2e-7f * scale + pivmin;
  hi += 2.0f * 1.2e-7f * scale + pivmin;
  const float pert = 1.2e-7f * fmaxf(tnorm, 1e-30f);
  float prev[RMAX][D];
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    // (rank >= 1 is checked at create time: no runtime test for r = 0, which
    // would keep the whole eigen work behind a branch and double its
    // register footprint)
    if constexpr (r > 0) {
      if (r >= R) return;
    }
    // bisection for the (r+1)-th largest eigenvalue: count(x) >= D - r <=> x > lambda_r
    float lo_r = lo, hi_r = hi;
    for (int it = 0; it < 32; ++it) {
      const float mid = 0.5f * (lo_r + hi_r);
      const int cnt = sturm<D>(ta, e2, mid, pivmin);
      if (cnt >= D - r) hi_r = mid;
      else lo_r = mid;
    }
    const float lam = 0.5f * (lo_r + hi_r);
    hi = hi_r;
    float x[D];
    tri_eigvec<D, RMAX>(ta, e2, lam, pert, r, prev, x);
    sfor<0, D>([&](auto ic) { prev[r][decltype(ic)::value] = x[decltype(ic)::value]; });
    // phases: v_i = phi_i x_i, phi_{i+1} = phi_i b_{i+1} / |b_{i+1}|
    cf v[D];
    cf phi = cf{1.0f, 0.0f};
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i >= 1) {
        const float ab2 = e2[i];
        const float iab = frsq(ab2);
        if (ab2 > 0.0f) phi = phi * cf{b[i].re * iab, b[i].im * iab};
      }
      v[i] = x[i] * phi;
    });
    // back-transform: v <- H_0 ... H_{D-3} v (last reflector first)
    sfor_down<(D >= 2 ? D - 2 : 0), 0>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      cf s = cmul(u0[j], v[j + 1]);
      sfor<j + 2, D>([&](auto ic) { cmac<true, false, false>(s, A.a[P(decltype(ic)::value, j)], v[decltype(ic)::value]); });
      const cf s2 = 2.0f * s;
      cmac<false, false, true>(v[j + 1], u0[j], s2);
      sfor<j + 2, D>([&](auto ic) { cmac<false, false, true>(v[decltype(ic)::value], A.a[P(decltype(ic)::value, j)], s2); });
    });
    fn(r, lam, v);
  });
}

}  // namespace lane
}  // namespace danse
