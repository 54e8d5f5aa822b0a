// Condition numbers of the SCMs Ryy (the reference's ConditionNumbers:
// get_new_cond_number / compute_condition_numbers, d_classes.py:19-130, called
// after the SCM update of every saveConditionNumberEvery-th iteration,
// d_classes.py:2126-2186): np.linalg.cond (2-norm, sigma_max / sigma_min) of
// every bin's Ryy as stored after the round's recursion.  Ryy is Hermitian
// (the engine keeps the lower triangle, as eigh reads it), so the singular
// values are the absolute eigenvalues: cyclic complex Jacobi in float64, one
// bin per wavefront, the matrix in LDS, row k on lane k (D <= 64).
//
// A Jacobi step on (p, q) first turns a_pq real by the unitary scaling of
// row / column q with exp(-i arg a_pq), then applies the real rotation of
// the 2 x 2 block [[a_pp, |a_pq|], [|a_pq|, a_qq]]; both are similarities,
// so the eigenvalues are those of Ryy.  Host translation unit only.
#pragma once
#include "kernels.hpp"

namespace danse {

constexpr int kCondMaxSweeps = 30;

// out: [S][nFN][R][F] float64 (NaN for the SSBC family: not saved by the reference)
__global__ void __launch_bounds__(64) cond_kernel(const UpdateArgs a, const FamNode* fns, int nFN, double* out) {
  extern __shared__ cd cA[];   // [D][D + 1]
  const int li = threadIdx.x;
  const int f = blockIdx.x;
  const int fni = blockIdx.y % nFN;
  const int s = blockIdx.y / nFN;
  const FamNode d = fns[fni];
  const int D = d.D, P = D + 1, F = a.F;
  double* o = out + (((long long)s * nFN + fni) * a.R + a.r) * F + f;
  if (d.fam == DANSE_FAM_SSBC) {
    if (li == 0) *o = __builtin_nan("");
    return;
  }
  const bool act = li < D;
  // Hermitian completion of the stored lower triangle (diagonal real)
  if (act) {
    const int i = li;
    for (int j = 0; j <= i; ++j) {
      const long long e = scm_lower(d, a.scmStride, s, F, f, i, j);
      cd x = scm_entry(a, d, true, e);
      if (i == j) x.im = 0.0;
      cA[i * P + j] = x;
      cA[j * P + i] = conjg(x);
    }
  }
  __syncthreads();
  for (int sweep = 0; sweep < kCondMaxSweeps; ++sweep) {
    double off = 0.0, dg = 0.0;
    if (act) {
      for (int j = 0; j < D; ++j) {
        const cd x = cA[li * P + j];
        const double m = x.re * x.re + x.im * x.im;
        if (j == li) dg += m;
        else off += m;
      }
    }
    for (int w = 32; w >= 1; w >>= 1) {
      off += __shfl_xor(off, w);
      dg += __shfl_xor(dg, w);
    }
    if (!(off > 1e-32 * dg)) break;   // converged (or a NaN matrix: stop)
    for (int p = 0; p < D - 1; ++p) {
      for (int q = p + 1; q < D; ++q) {
        const cd apq = cA[p * P + q];
        const double r = sqrt(apq.re * apq.re + apq.im * apq.im);
        const double app = cA[p * P + p].re, aqq = cA[q * P + q].re;
        if (r == 0.0) continue;   // wave-uniform
        const cd ph = cd{apq.re / r, -apq.im / r};   // exp(-i arg a_pq)
        const double th = (aqq - app) / (2.0 * r);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), sn = t * c;
        cd nkp = cd{0.0, 0.0}, nkq = cd{0.0, 0.0};
        const bool row = act && li != p && li != q;
        if (row) {
          const cd akp = cA[li * P + p];
          const cd x = cA[li * P + q];
          const cd akq = cd{x.re * ph.re - x.im * ph.im, x.re * ph.im + x.im * ph.re};
          nkp = cd{c * akp.re - sn * akq.re, c * akp.im - sn * akq.im};
          nkq = cd{sn * akp.re + c * akq.re, sn * akp.im + c * akq.im};
        }
        __syncthreads();
        if (row) {
          cA[li * P + p] = nkp;
          cA[p * P + li] = conjg(nkp);
          cA[li * P + q] = nkq;
          cA[q * P + li] = conjg(nkq);
        }
        if (li == 0) {
          cA[p * P + p] = cd{app - t * r, 0.0};
          cA[q * P + q] = cd{aqq + t * r, 0.0};
          cA[p * P + q] = cd{0.0, 0.0};
          cA[q * P + p] = cd{0.0, 0.0};
        }
        __syncthreads();
      }
    }
  }
  double lmax = act ? fabs(cA[li * P + li].re) : 0.0;
  double lmin = act ? fabs(cA[li * P + li].re) : __builtin_inf();
  bool nan = act && (cA[li * P + li].re != cA[li * P + li].re);
  for (int w = 32; w >= 1; w >>= 1) {
    lmax = fmax(lmax, __shfl_xor(lmax, w));
    lmin = fmin(lmin, __shfl_xor(lmin, w));
  }
  nan = __ballot(nan) != 0ull;
  if (li == 0) *o = nan ? __builtin_nan("") : lmax / lmin;
}

}  // namespace danse
