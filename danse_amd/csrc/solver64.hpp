// Wavefront building blocks for large filter dimensions (12 < D <= 64): one
// frequency bin per wavefront, lane i holds ROW i.  (The filter update that
// uses them is solver64m.hpp.)  Householder tridiagonalisation, Sturm
// multisection for the top-R eigenvalues, inverse iteration, written for
// code size: the pivot loops run at RUN time over the actual D (no padding),
// the column loops are unrolled over DMAX.  A row lives in chunked vector
// registers (Row<DMAX>, processed in chunks of 8 columns) so that the
// pivot column j -- a wave-uniform runtime index -- is read through a tree
// of uniform branches (no scratch) and written back through LDS.  Row
// broadcasts are v_readlane into SGPRs (uniform lane index j), reductions
// are DPP butterflies.  The tridiagonal is lane-distributed (lane i holds
// a_i and |b_i|^2) and the inverse iteration is a serial Thomas sweep over
// readlane and lane selects.
#pragma once
#include "solver.hpp"

namespace danse {
namespace big {

template <int DMAX>
struct Row {
  static_assert(DMAX % 8 == 0, "DMAX must be a multiple of 8");
  static constexpr int NC = DMAX / 8;   // chunks of 8 columns (uniform skipping)
  float re[DMAX], im[DMAX];
};

template <int C, int DMAX>
DANSE_DEV cf rs(const Row<DMAX>& X) {
  return cf{X.re[C], X.im[C]};
}
template <int C, int DMAX>
DANSE_DEV void ws(Row<DMAX>& X, cf v) {
  X.re[C] = v.re;
  X.im[C] = v.im;
}
// Dynamic, wave-uniform column index: a select chain the compiler lowers to
// a binary tree of uniform (scalar) branches ending in one v_mov -- no
// scratch, no per-element selects.  (There is no dynamic WRITE: columns are
// written back through LDS, see chol.)
template <int DMAX, int C = 0>
DANSE_DEV float rget1(const float (&x)[DMAX], int j) {
  if constexpr (C == DMAX - 1) return x[C];
  else return (j == C) ? x[C] : rget1<DMAX, C + 1>(x, j);
}
template <int DMAX>
DANSE_DEV cf rget(const Row<DMAX>& X, int j) {
  return cf{rget1<DMAX>(X.re, j), rget1<DMAX>(X.im, j)};
}
template <int DMAX>
DANSE_DEV void rzero(Row<DMAX>& X) {
  sfor<0, DMAX>([&](auto cc) {
    X.re[decltype(cc)::value] = 0.0f;
    X.im[decltype(cc)::value] = 0.0f;
  });
}

DANSE_DEV float rl(float x, int lane) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), lane)); }
DANSE_DEV cf rl(cf x, int lane) { return cf{rl(x.re, lane), rl(x.im, lane)}; }
// value v into lane `lane` of x (v wave-uniform)
DANSE_DEV float wl(float x, float v, int lane) {
  return (lane_id() == lane) ? v : x;
}

// Apply fn(c) for every static column c of chunks that hold a column > j
// (uniform skip of finished chunks).
template <int DMAX, typename Fn>
DANSE_DEV void cols_after(int j, Fn&& fn) {
  sfor<0, Row<DMAX>::NC>([&](auto cc) {
    constexpr int c0 = decltype(cc)::value * 8;
    if (c0 + 7 > j) {
      sfor<c0, c0 + 8>(fn);
    }
  });
}
// ... every static column c < D (uniform skip of padding chunks)
template <int DMAX, typename Fn>
DANSE_DEV void cols_below(int D, Fn&& fn) {
  sfor<0, Row<DMAX>::NC>([&](auto cc) {
    constexpr int c0 = decltype(cc)::value * 8;
    if (c0 < D) {
      sfor<c0, c0 + 8>(fn);
    }
  });
}

template <int DMAX>
struct LDS {
  cf U[DMAX][DMAX + 1];   // transpose tile, then Householder vectors U[j][i]
  float x[kRMax][DMAX];   // tridiagonal eigenvectors (Gram-Schmidt)
};

// Householder tridiagonalisation of the Hermitian A (first D rows/cols).
// u_j -> U[j][i]; returns a = T[li][li], b = T[li][li-1].
template <int DMAX>
DANSE_DEV void tridiag(Row<DMAX>& A, cf (*U)[DMAX + 1], int li, int D, float& a, cf& b) {
  for (int j = 0; j + 2 < D; ++j) {
    const cf aj = rget(A, j);
    const cf xi = (li > j) ? aj : cf{0.0f, 0.0f};
    const float nrm2 = gsum<64>(abs2(xi));
    const cf x0 = rl(aj, j + 1);
    const float ax02 = abs2(x0);
    const float nx = fsqrt(nrm2);
    const float ax0 = fsqrt(ax02);
    const float iax0 = frsq(ax02);
    const cf e = (ax02 > 0.0f) ? cf{x0.re * iax0, x0.im * iax0} : cf{1.0f, 0.0f};
    const float invn = (nrm2 > 1e-30f) ? frsq(2.0f * nx * (nx + ax0)) : 0.0f;
    cf u = xi;
    if (li == j + 1) u = u + nx * e;
    u = invn * u;
    cf p = cf{0.0f, 0.0f};
    cols_after<DMAX>(j, [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      fma_c(p, rs<c>(A), rl(u, c));
    });
    const float Kr = gsum<64>(cmul(u, p).re);
    const cf q = p - Kr * u;
    const cf u2 = 2.0f * u, q2 = 2.0f * q;
    cols_after<DMAX>(j - 1, [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      cf qc = rl(q, c), uc = rl(u, c);
      if (c < j) {   // columns already reduced: leave them bit-exact
        qc = cf{0.0f, 0.0f};
        uc = cf{0.0f, 0.0f};
      }
      cf x = rs<c>(A);
      fms_cc(x, u2, qc);
      fms_cc(x, q2, uc);
      ws<c>(A, x);
    });
    if (li < DMAX) U[j][li] = u;
  }
  a = 0.0f;
  b = cf{0.0f, 0.0f};
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (li == c) a = rs<c>(A).re;
    if constexpr (c >= 1) {
      if (li == c) b = rs<c - 1>(A);
    }
  });
  __syncthreads();
}

// Sturm count of the lane-distributed tridiagonal (a_i, e2_i = |b_{i+1}|^2 on
// lane i) below x (one x per lane).
DANSE_DEV int sturm(float ta, float te2, int D, float x, float pivmin) {
  int cnt = 0;
  float q = 1.0f;
  for (int i = 0; i < D; ++i) {
    const float ai = rl(ta, i);
    float qn = ai - x;
    if (i > 0) qn -= rl(te2, i - 1) * frcp(q);
    if (fabsf(qn) <= pivmin) qn = -pivmin;
    q = qn;
    cnt += (q < 0.0f) ? 1 : 0;
  }
  return cnt;
}

template <int RMAX>
DANSE_DEV void top_eigvals(float ta, float te2, int li, int D, int R, float (&lam)[kRMax], float& tnorm) {
  const bool act = li < D;
  const float e2m = __shfl_up(te2, 1);   // |b_li|^2 (lane li - 1)
  const float em = (li >= 1 && act) ? fsqrt(e2m) : 0.0f;
  const float ep = (li + 1 < D) ? fsqrt(te2) : 0.0f;
  const float lo0 = gmin<64>(act ? ta - em - ep : 3.0e38f);
  const float hi0 = gmax<64>(act ? ta + em + ep : -3.0e38f);
  const float e2max = gmax<64>((li + 1 < D) ? te2 : 0.0f);
  tnorm = gmax<64>(act ? fabsf(ta) + em + ep : 0.0f);
  const float scale = fmaxf(fabsf(lo0), fabsf(hi0));
  const float pivmin = 1.0e-30f * fmaxf(1.0f, e2max);
  float lo = lo0 - (2.0f * 1.2e-7f * scale + pivmin);
  float hi = hi0 + (2.0f * 1.2e-7f * scale + pivmin);
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if (r >= R) return;
    float a = lo, b = hi;
    const int target = D - r;   // count(x) >= target  <=>  x > lambda_r
    for (int it = 0; it < 5; ++it) {
      const float step = (b - a) * (1.0f / 65.0f);
      const float x = a + step * (float)(li + 1);
      const int cnt = sturm(ta, (li + 1 < D) ? te2 : 0.0f, D, x, pivmin);
      const uint64_t m = __ballot(cnt >= target);
      if (m == 0ull) {
        a = a + step * 64.0f;
      } else {
        const int first = __builtin_ctzll(m);
        const float na = a + step * (float)first;
        b = a + step * (float)(first + 1);
        a = na;
      }
    }
    lam[r] = 0.5f * (a + b);
    hi = b;
  });
}

// Eigenvector (lane-distributed, x_li) of the tridiagonal for eigenvalue lam:
// inverse iteration with the partial-pivoting tridiagonal elimination of
// solver.hpp::tri_eigvec, as a serial sweep over readlane and lane selects.
template <int DMAX>
DANSE_DEV float tri_eigvec(float ta, float te, int li, int D, float lam, float pert, int r, const float (*prev)[DMAX]) {
  // te: |b_{li+1}| on lane li (0 for li >= D-1)
  float x = (li < D) ? 1.0f + 0.1f * (float)((li * 7919 + r * 104729) % 13) / 13.0f : 0.0f;
  for (int it = 0; it < 2; ++it) {
    float d = (li < D) ? ta - lam : 0.0f;
    float dl = te, du = te, dl2 = 0.0f;
    float rhs = x;
    for (int i = 0; i + 1 < D; ++i) {
      const float di0 = rl(d, i), dli = rl(dl, i), dui = rl(du, i);
      const float d1 = rl(d, i + 1), du1 = (i + 2 < D) ? rl(du, i + 1) : 0.0f;
      const float ri = rl(rhs, i), ri1 = rl(rhs, i + 1);
      const bool swap = fabsf(di0) < fabsf(dli);
      const float di = (di0 == 0.0f) ? pert : di0;
      const float f1 = dli * frcp(di);
      const float f2 = di0 * frcp(dli);
      const float nd_i = swap ? dli : di;
      const float nd_i1 = swap ? (dui - f2 * d1) : (d1 - f1 * dui);
      const float ndl2_i = swap ? du1 : 0.0f;
      const float ndu_i1 = swap ? -f2 * du1 : du1;
      const float ndu_i = swap ? d1 : dui;
      const float nr_i = swap ? ri1 : ri;
      const float nr_i1 = swap ? (ri - f2 * ri1) : (ri1 - f1 * ri);
      d = wl(wl(d, nd_i, i), nd_i1, i + 1);
      dl2 = wl(dl2, ndl2_i, i);
      du = wl(du, ndu_i, i);
      if (i + 2 < D) du = wl(du, ndu_i1, i + 1);
      rhs = wl(wl(rhs, nr_i, i), nr_i1, i + 1);
    }
    // back solve
    float xn1 = 0.0f, xn2 = 0.0f;   // x[i+1], x[i+2]
    float sol = 0.0f;
    for (int i = D - 1; i >= 0; --i) {
      float acc = rl(rhs, i);
      acc -= rl(du, i) * xn1;
      acc -= rl(dl2, i) * xn2;
      const float di0 = rl(d, i);
      const float di = (di0 == 0.0f) ? pert : di0;
      const float xi = acc * frcp(di);
      sol = wl(sol, xi, i);
      xn2 = xn1;
      xn1 = xi;
    }
    for (int q = 0; q < r; ++q) {
      const float pq = (li < DMAX) ? prev[q][li] : 0.0f;
      const float dot = gsum<64>(pq * sol);
      sol -= dot * pq;
    }
    const float mx0 = gmax<64>(fabsf(sol));
    const float mx = (mx0 > 0.0f) ? mx0 : 1.0f;
    sol *= frcp(mx);
    const float nrm = gsum<64>(sol * sol);
    x = sol * frsq(nrm);
  }
  return x;
}

}  // namespace big
}  // namespace danse
