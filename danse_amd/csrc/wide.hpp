// Filters of the wide classes, 64 < D <= 256: the centralised family and the
// best-performance estimate at sum(M) up to 256 (d_core.py:602-627,
// d_batch.py:81-125, d_classes.py:2139-2201), and the stand-alone filter
// operator at those sizes.  One 256-thread workgroup per (SCM pair, bin),
// float64 throughout; the matrices live in a global workspace of 2 D^2
// complex doubles per workgroup (Lc: the Cholesky factor, column-major;
// Cw: the right-hand sides / the congruence C).
//
//   GEVD (update_w_gevd, d_classes.py:3343-3387; scipy.linalg.eigh reads the
//   lower triangles):
//     Rnn = L L^H              left-looking Cholesky, one column per step
//     C = L^-1 Ryy L^-H        two triangular solves, one column per thread,
//                              rows in register chunks of kCh
//     C = Q T Q^H              Householder steps of LAPACK zhetd2 ('L'),
//                              real off-diagonal
//     top-R eigenvalues of T   multisection: 256 Sturm counts per pass
//     their vectors            inverse iteration (one thread per vector),
//                              Gram-Schmidt between them, y = Q z
//     x = L^-H y               (Xmat's columns: x^H Rnn x = 1)
//     w = sum_r (1 - 1/sigma_r) x_r conj((Rnn x_r)[ref]),  Rnn x = L y
//   (Qmat^H = Xmat^-1 = Xmat^H Rnn, so X D Q^H e_ref is that sum.)
//   MWF (update_w, d_classes.py:3320-3340): Ryy = L L^H,
//     w = L^-H L^-1 (Ryy - Rnn) e_ref, one right-hand side per output.
#pragma once
#include "solver.hpp"
#include "wide_api.hpp"
#include "../../include/danse_mi355x_defs.h"

namespace danse {
namespace wide {

DANSE_DEV cd cmulx(cd a, cd b) { return cd{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }

// element (i, c) of an item's SCM from its lower triangle (the diagonal real)
DANSE_DEV cd src_el(const WideArgs& a, bool ryy, long long base, int i, int c) {
  const int hi = i >= c ? i : c, lo = i >= c ? c : i;
  cd v;
  if (a.layout == 0) {
    const long long e = base + (long long)hi * a.D + lo;
    v = ryy ? a.RyyD[e] : a.Rnn[e];
  } else if (a.layout == 2) {
    const long long e = base + (long long)hi * (hi + 1) / 2 + lo;
    v = ryy ? a.RyyD[e] : a.Rnn[e];
  } else {
    const long long e = base + (long long)hi * (hi + 1) / 2 + lo;
    v = ryy ? cdk(a.RyyF[e]) : a.Rnn[e];
  }
  if (i < c) v = conjg(v);
  if (i == c) v.im = 0.0;
  return v;
}

// sum over the workgroup (every thread gets it); red: 4 doubles of LDS
DANSE_DEV double bsum(double x, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// Column c of Cw ([D][D] row-major) <- L^-1 Cw[:, c] (FWD) or L^-H Cw[:, c]
// (!FWD), in place, by thread c alone.  Rows are taken kCh at a time into
// registers: the solved rows' contributions stream in (one load of x_k per
// chunk, the L entries are the same for every thread), then the chunk's own
// triangle.  invd[i] = 1 / L[i][i].
template <bool FWD>
// (restrict: the factor and the workspace are distinct buffers, so the L
// reads of the chunk's triangle need not wait behind the solved-row stores;
// the reads are unconditional at clamped rows, their values selected)
DANSE_DEV void trsv_col(const cd* __restrict__ Lc, const double* __restrict__ invd, int D, cd* __restrict__ Cw, int c) {
  for (int b0 = 0; b0 < D; b0 += kCh) {
    cd acc[kCh];
#pragma unroll
    for (int r = 0; r < kCh; ++r) {
      const int i = FWD ? b0 + r : D - 1 - (b0 + r);
      const bool ok = FWD ? i < D : i >= 0;
      acc[r] = ok ? Cw[(long long)i * D + c] : cd{0.0, 0.0};
    }
    for (int kk = 0; kk < b0; ++kk) {
      const int k = FWD ? kk : D - 1 - kk;
      const cd xk = Cw[(long long)k * D + c];
#pragma unroll
      for (int r = 0; r < kCh; ++r) {
        const int i = FWD ? b0 + r : D - 1 - (b0 + r);
        const bool ok = FWD ? i < D : i >= 0;
        // FWD: L[i][k] = Lc[k][i];  !FWD: (L^H)[i][k] = conj(L[k][i]) = conj(Lc[i][k])
        const int ic = ok ? i : (FWD ? D - 1 : 0);
        const cd l = csel(ok, FWD ? Lc[(long long)k * D + ic] : conjg(Lc[(long long)ic * D + k]), cd{0.0, 0.0});
        fms_c(acc[r], l, xk);
      }
    }
#pragma unroll
    for (int r = 0; r < kCh; ++r) {
      const int i = FWD ? b0 + r : D - 1 - (b0 + r);
      const bool ok = FWD ? i < D : i >= 0;
#pragma unroll
      for (int q = 0; q < r; ++q) {
        const int k = FWD ? b0 + q : D - 1 - (b0 + q);
        const int ic = ok ? i : (FWD ? D - 1 : 0);
        const cd l = csel(ok, FWD ? Lc[(long long)k * D + ic] : conjg(Lc[(long long)ic * D + k]), cd{0.0, 0.0});
        fms_c(acc[r], l, acc[q]);
      }
      if (ok) {
        acc[r] = invd[i] * acc[r];
        Cw[(long long)i * D + c] = acc[r];
      }
    }
  }
}

// Sturm count: eigenvalues of T (d, e2 = e^2) below x
DANSE_DEV int sturm(const double* d, const double* e2, int n, double x, double pivmin) {
  int cnt = 0;
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  cnt += q < 0.0;
  for (int i = 1; i < n; ++i) {
    q = d[i] - x - e2[i - 1] / q;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
  }
  return cnt;
}

struct WideLds {
  cd vec[kMaxD];            // broadcast vector (Cholesky column, Householder v)
  cd y[kRMax][kMaxD];       // eigenvectors: z (real) -> y = Q z -> x = L^-H y
  cd ly[kRMax][kMaxD];      // L y
  double invd[kMaxD];       // 1 / L[i][i]
  double td[kMaxD];         // tridiagonal: diagonal
  double te[kMaxD];         //              off-diagonal (real)
  double te2[kMaxD];        //              its squares
  cd tau[kMaxD];            // Householder scalars
  double zs[kRMax][kMaxD];  // inverse iteration iterates
  unsigned char piv[kRMax][kMaxD];   //                   row interchanges
  double lam[kRMax];        // eigenvalues, descending
  double red[4];
  double sh[4];
  int ish[4];
};

#ifdef DANSE_WIDE_KERNEL
__global__ void __launch_bounds__(kThr) wide_filter_kernel(const WideArgs a) {
  __shared__ WideLds S;
  const long long b = a.item0 + blockIdx.x;
  if (b >= a.nItems) return;   // workgroup-uniform
  const int t = threadIdx.x;
  const int D = a.D;
  const int s = (int)(b / a.F), f = (int)(b % a.F);
  if (a.flags) {   // workgroup-uniform
    const unsigned char fl = a.flags[(long long)s * a.flagStride];
    if (!(fl & DANSE_FLAG_SOLVE) || (fl & DANSE_FLAG_PREGIVEN)) return;
  }
  const long long base = (long long)s * a.srcScene + (long long)f * a.srcBin;
  cd* Lc = a.work + (long long)blockIdx.x * 2 * D * D;   // Lc[k * D + i] = L[i][k]
  cd* Cw = Lc + (long long)D * D;
  const bool gevd = a.gevd != 0;

  // ---- factor: Rnn (GEVD) or Ryy (MWF), lower triangle into Lc ----------
  for (long long e = t; e < (long long)D * D; e += kThr) {
    const int k = (int)(e / D), i = (int)(e % D);
    Lc[e] = i >= k ? src_el(a, !gevd, base, i, k) : cd{0.0, 0.0};
  }
  if (t == 0) S.ish[0] = 1;
  __syncthreads();
  for (int j = 0; j < D; ++j) {
    cd s0 = cd{0.0, 0.0}, s1 = cd{0.0, 0.0};
    if (t >= j && t < D) {
      s0 = Lc[(long long)j * D + t];
      int k = 0;
      for (; k + 1 < j; k += 2) {
        fms_cc(s0, Lc[(long long)k * D + t], Lc[(long long)k * D + j]);
        fms_cc(s1, Lc[(long long)(k + 1) * D + t], Lc[(long long)(k + 1) * D + j]);
      }
      if (k < j) fms_cc(s0, Lc[(long long)k * D + t], Lc[(long long)k * D + j]);
      s0 = s0 + s1;
    }
    if (t == j) {
      const double p = s0.re;
      if (!(p > 0.0) || !isfinite(p)) S.ish[0] = 0;
      const double dj = sqrt(p > 1e-300 ? p : 1e-300);
      S.invd[j] = 1.0 / dj;
      Lc[(long long)j * D + j] = cd{dj, 0.0};
    }
    __syncthreads();
    if (t > j && t < D) Lc[(long long)j * D + t] = S.invd[j] * s0;
    __syncthreads();
  }
  const bool okFactor = S.ish[0] != 0;

  if (!gevd) {
    // ---- MWF: column j of Cw = (Ryy - Rnn)[:, ref_j]; two solves --------
    for (long long e = t; e < (long long)D * a.nOut; e += kThr) {
      const int i = (int)(e / a.nOut), j = (int)(e % a.nOut);
      const int rf = a.refs[j];
      const cd v = src_el(a, true, base, i, rf) - src_el(a, false, base, i, rf);
      Cw[(long long)i * D + j] = v;
    }
    __syncthreads();
    if (t < a.nOut) {
      trsv_col<true>(Lc, S.invd, D, Cw, t);
      trsv_col<false>(Lc, S.invd, D, Cw, t);
    }
    __syncthreads();
    for (long long e = t; e < (long long)D * a.nOut; e += kThr) {
      const int i = (int)(e % D), j = (int)(e / D);
      a.w[a.wOff[j] + s * a.wScene + f * a.wBin + i] = cfk(Cw[(long long)i * D + j]);
    }
    if (a.diag && t == 0) a.diag[b] = okFactor ? 0 : 1;
    return;
  }

  // ---- GEVD: C = L^-1 Ryy L^-H ------------------------------------------
  for (long long e = t; e < (long long)D * D; e += kThr) {
    const int i = (int)(e / D), c = (int)(e % D);
    Cw[e] = src_el(a, true, base, i, c);
  }
  __syncthreads();
  if (t < D) trsv_col<true>(Lc, S.invd, D, Cw, t);   // X = L^-1 Ryy
  __syncthreads();
  for (long long e = t; e < (long long)D * D; e += kThr) {   // X^H in place (= Ryy L^-H)
    const int i = (int)(e / D), c = (int)(e % D);
    if (i < c) {
      const cd u = Cw[e], v = Cw[(long long)c * D + i];
      Cw[e] = conjg(v);
      Cw[(long long)c * D + i] = conjg(u);
    } else if (i == c) {
      Cw[e] = conjg(Cw[e]);
    }
  }
  __syncthreads();
  if (t < D) trsv_col<true>(Lc, S.invd, D, Cw, t);   // C = L^-1 X^H
  __syncthreads();
  // exact Hermitian: the lower triangle (what eigh reads) mirrored up
  for (long long e = t; e < (long long)D * D; e += kThr) {
    const int i = (int)(e / D), c = (int)(e % D);
    if (i < c) Cw[e] = conjg(Cw[(long long)c * D + i]);
    else if (i == c) Cw[e].im = 0.0;
  }
  __syncthreads();

  // ---- Householder tridiagonalisation (zhetd2, lower) -------------------
  // step j: v = (1, x / (alpha - beta)) over rows j+1 .. D-1, stored in row j
  // of Cw (dead after the step) for the back-transform; T: td, te (real).
  for (int j = 0; j + 1 < D; ++j) {
    const int n1 = j + 1;
    // column j below the diagonal = conj(row j) right of it
    const cd xi = (t > n1 && t < D) ? conjg(Cw[(long long)j * D + t]) : cd{0.0, 0.0};
    const double xn2 = bsum(xi.re * xi.re + xi.im * xi.im, S.red);
    const cd alpha = conjg(Cw[(long long)j * D + n1]);
    cd tau = cd{0.0, 0.0};
    double beta = alpha.re;
    cd scal = cd{0.0, 0.0};
    if (xn2 > 0.0 || alpha.im != 0.0) {
      const double nrm = sqrt(alpha.re * alpha.re + alpha.im * alpha.im + xn2);
      beta = alpha.re >= 0.0 ? -nrm : nrm;
      tau = cd{(beta - alpha.re) / beta, -alpha.im / beta};
      // 1 / (alpha - beta)
      const cd dd = cd{alpha.re - beta, alpha.im};
      const double den = dd.re * dd.re + dd.im * dd.im;
      scal = cd{dd.re / den, -dd.im / den};
    }
    if (t >= n1 && t < D) S.vec[t] = (t == n1) ? cd{1.0, 0.0} : cmulx(scal, xi);
    if (t == 0) {
      S.td[j] = Cw[(long long)j * D + j].re;
      S.te[j] = beta;
      S.te2[j] = beta * beta;
      S.tau[j] = tau;
    }
    __syncthreads();
    if (tau.re != 0.0 || tau.im != 0.0) {
      // p = tau C22 v: thread i, C[i][k] = conj(C[k][i]) read down column i
      cd p = cd{0.0, 0.0};
      if (t >= n1 && t < D) {
        cd q0 = cd{0.0, 0.0}, q1 = cd{0.0, 0.0};
        int k = n1;
        for (; k + 1 < D; k += 2) {
          fma_c(q0, conjg(Cw[(long long)k * D + t]), S.vec[k]);
          fma_c(q1, conjg(Cw[(long long)(k + 1) * D + t]), S.vec[k + 1]);
        }
        if (k < D) fma_c(q0, conjg(Cw[(long long)k * D + t]), S.vec[k]);
        p = cmulx(tau, q0 + q1);
      }
      // alpha2 = -tau / 2 * (p^H v)
      const cd pv = (t >= n1 && t < D) ? cmulx(conjg(p), S.vec[t]) : cd{0.0, 0.0};
      const double pvr = bsum(pv.re, S.red), pvi = bsum(pv.im, S.red);
      const cd a2 = cmulx(cd{-0.5 * tau.re, -0.5 * tau.im}, cd{pvr, pvi});
      // w = p + a2 v, staged in y[0] (free until the eigenvectors)
      if (t >= n1 && t < D) S.y[0][t] = p + cmulx(a2, S.vec[t]);
      __syncthreads();
      // C22 -= v w^H + w v^H (thread k: column k)
      if (t >= n1 && t < D) {
        const cd vk = S.vec[t], wk = S.y[0][t];
        for (int i = n1; i < D; ++i) {
          cd c = Cw[(long long)i * D + t];
          fms_cc(c, S.vec[i], wk);
          fms_cc(c, S.y[0][i], vk);
          Cw[(long long)i * D + t] = c;
        }
      }
    }
    // v into row j (right of the diagonal) for the back-transform
    if (t >= n1 && t < D) Cw[(long long)j * D + t] = S.vec[t];
    __syncthreads();
  }
  if (t == 0) S.td[D - 1] = Cw[(long long)(D - 1) * D + D - 1].re;
  __syncthreads();

  // ---- top-R eigenvalues of T: multisection --------------------------------
  const int R = a.rank;
  double lo = 0.0, hi = 0.0, pivmin = 0.0;
  {
    double glo = 1e300, ghi = -1e300, emax = 0.0;
    for (int i = 0; i < D; ++i) {
      const double r = (i > 0 ? fabs(S.te[i - 1]) : 0.0) + (i + 1 < D ? fabs(S.te[i]) : 0.0);
      glo = fmin(glo, S.td[i] - r);
      ghi = fmax(ghi, S.td[i] + r);
      if (i + 1 < D) emax = fmax(emax, S.te2[i]);
    }
    const double wdt = ghi - glo, pad = 2.0e-15 * fmax(fabs(glo), fabs(ghi)) + 1e-300;
    lo = glo - pad - 1e-14 * wdt;
    hi = ghi + pad + 1e-14 * wdt;
    pivmin = 2.2250738585072014e-308 * fmax(1.0, emax);
  }
  for (int r = 0; r < R; ++r) {
    const int m = D - 1 - r;   // ascending index of the r-th largest
    double aa = lo, bb = hi;
    for (int pass = 0; pass < 24; ++pass) {
      const double x = aa + (bb - aa) * (double)(t + 1) / (double)(kThr + 1);
      const int c = sturm(S.td, S.te2, D, x, pivmin);
      // first point with count > m
      int first = (c > m) ? t : kThr;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o));
      __syncthreads();
      if ((t & 63) == 0) S.ish[t >> 6] = first;
      __syncthreads();
      const int fm = min(min(S.ish[0], S.ish[1]), min(S.ish[2], S.ish[3]));
      const double na = fm == 0 ? aa : aa + (bb - aa) * (double)fm / (double)(kThr + 1);
      const double nb = fm == kThr ? bb : aa + (bb - aa) * (double)(fm + 1) / (double)(kThr + 1);
      aa = na;
      bb = nb;
      if (bb - aa <= 4.0e-16 * fmax(fabs(aa), fabs(bb)) + pivmin) break;
    }
    if (t == 0) S.lam[r] = 0.5 * (aa + bb);
  }
  __syncthreads();

  // ---- tridiagonal eigenvectors: inverse iteration, thread r --------------
  // (T - lam I) z = b by Gaussian elimination with row interchanges (dgttrf:
  // U's rows in d / u1 / u2, the multipliers l, the interchanges in piv),
  // three solves from a fixed pseudo-random start; the LU rows overlay y[r] /
  // ly[r], the iterate lives in zs[r].
  if (t < R) {
    const double lam = S.lam[t];
    double tn = 0.0;
    for (int i = 0; i < D; ++i)
      tn = fmax(tn, fabs(S.td[i]) + (i > 0 ? fabs(S.te[i - 1]) : 0.0) + (i + 1 < D ? fabs(S.te[i]) : 0.0));
    const double tiny = 2.2e-16 * fmax(tn, 1e-300);
    double* du = &S.y[t][0].re;    // du[2 i] = U[i][i], du[2 i + 1] = U[i][i + 1]
    double* dl = &S.ly[t][0].re;   // dl[2 i] = U[i][i + 2], dl[2 i + 1] = l_i
    double* z = S.zs[t];
    double c0 = S.td[0] - lam, c1 = (D > 1) ? S.te[0] : 0.0;
    for (int i = 0; i < D; ++i) {
      if (i + 1 < D) {
        const double sub = S.te[i];   // T[i + 1][i]
        const double nd = S.td[i + 1] - lam, nu = (i + 2 < D) ? S.te[i + 1] : 0.0;
        if (fabs(c0) >= fabs(sub)) {
          const double pv = (c0 == 0.0) ? tiny : c0;
          const double l = sub / pv;
          du[2 * i] = pv; du[2 * i + 1] = c1; dl[2 * i] = 0.0; dl[2 * i + 1] = l;
          S.piv[t][i] = 0;
          c0 = nd - l * c1;
          c1 = nu;
        } else {
          const double l = c0 / sub;
          du[2 * i] = sub; du[2 * i + 1] = nd; dl[2 * i] = nu; dl[2 * i + 1] = l;
          S.piv[t][i] = 1;
          c0 = c1 - l * nd;
          c1 = -l * nu;
        }
      } else {
        du[2 * i] = c0; du[2 * i + 1] = 0.0; dl[2 * i] = 0.0; dl[2 * i + 1] = 0.0;
        S.piv[t][i] = 0;
      }
      if (fabs(du[2 * i]) < tiny) du[2 * i] = du[2 * i] < 0.0 ? -tiny : tiny;
    }
    unsigned h = 0x9E3779B9u * (unsigned)(t + 1);
    for (int i = 0; i < D; ++i) {
      h = h * 1664525u + 1013904223u;
      z[i] = 0.5 + (double)(h >> 8) * (1.0 / 16777216.0);
    }
    for (int it = 0; it < 3; ++it) {
      for (int i = 0; i + 1 < D; ++i) {
        double bi = z[i], bn = z[i + 1];
        if (S.piv[t][i]) { const double x = bi; bi = bn; bn = x; }
        z[i] = bi;
        z[i + 1] = bn - dl[2 * i + 1] * bi;
      }
      double nrm = 0.0;
      for (int i = D - 1; i >= 0; --i) {
        double v = z[i];
        if (i + 1 < D) v -= du[2 * i + 1] * z[i + 1];
        if (i + 2 < D) v -= dl[2 * i] * z[i + 2];
        v /= du[2 * i];
        z[i] = v;
        nrm = fmax(nrm, fabs(v));
      }
      const double sc = 1.0 / nrm;
      for (int i = 0; i < D; ++i) z[i] *= sc;
    }
  }
  __syncthreads();
  for (int r = 0; r < R; ++r) S.y[r][t] = cd{t < D ? S.zs[r][t] : 0.0, 0.0};
  __syncthreads();
  // Gram-Schmidt (descending eigenvalue order) and unit norm
  for (int r = 0; r < R; ++r) {
    for (int q = 0; q < r; ++q) {
      const double dp = bsum(S.y[q][t].re * S.y[r][t].re, S.red);
      S.y[r][t].re -= dp * S.y[q][t].re;
    }
    const double n2 = bsum(S.y[r][t].re * S.y[r][t].re, S.red);
    S.y[r][t].re *= 1.0 / sqrt(n2);
  }
  __syncthreads();

  // ---- y = Q z = H(0) .. H(D-2) z ---------------------------------------
  for (int j = D - 2; j >= 0; --j) {
    const cd tj = S.tau[j];
    if (tj.re == 0.0 && tj.im == 0.0) continue;   // workgroup-uniform
    const int n1 = j + 1;
    const cd vj = (t >= n1 && t < D) ? Cw[(long long)j * D + t] : cd{0.0, 0.0};
    for (int r = 0; r < R; ++r) {
      const cd pr = (t >= n1 && t < D) ? cmulx(conjg(vj), S.y[r][t]) : cd{0.0, 0.0};
      const double dr = bsum(pr.re, S.red), di = bsum(pr.im, S.red);
      const cd sc = cmulx(tj, cd{dr, di});
      if (t >= n1 && t < D) fms_c(S.y[r][t], vj, sc);
    }
    __syncthreads();
  }

  // ---- L y (for (Rnn x)[ref]) and x = L^-H y --------------------------------
  for (int r = 0; r < R; ++r) {
    cd acc = cd{0.0, 0.0};
    if (t < D)
      for (int k = 0; k <= t; ++k) fma_c(acc, Lc[(long long)k * D + t], S.y[r][k]);
    S.ly[r][t] = acc;
  }
  __syncthreads();
  cd yv[kRMax];
#pragma unroll
  for (int r = 0; r < kRMax; ++r) yv[r] = (r < R && t < D) ? S.y[r][t] : cd{0.0, 0.0};
  for (int i = D - 1; i >= 0; --i) {
    if (t == i) {
#pragma unroll
      for (int r = 0; r < kRMax; ++r)
        if (r < R) {
          yv[r] = S.invd[i] * yv[r];
          S.y[r][i] = yv[r];   // x_i
        }
    }
    __syncthreads();
    if (t < i) {
      const cd l = conjg(Lc[(long long)t * D + i]);   // (L^H)[t][i] = conj(L[i][t])
#pragma unroll
      for (int r = 0; r < kRMax; ++r)
        if (r < R) fms_c(yv[r], l, S.y[r][i]);
    }
  }
  __syncthreads();

  // ---- filters ------------------------------------------------------------
  if (t < D) {
    for (int j = 0; j < a.nOut; ++j) {
      const int rf = a.refs[j];
      cd wv = cd{0.0, 0.0};
      for (int r = 0; r < R; ++r) {
        const double g = 1.0 - 1.0 / S.lam[r];
        fma_cc(wv, g * S.y[r][t], S.ly[r][rf]);
      }
      a.w[a.wOff[j] + s * a.wScene + f * a.wBin + t] = cfk(wv);
    }
  }
  if (a.diag && t == 0) a.diag[b] = okFactor ? 0 : 1;
}

#endif  // DANSE_WIDE_KERNEL

}  // namespace wide
}  // namespace danse
