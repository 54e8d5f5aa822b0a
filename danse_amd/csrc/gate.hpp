// The reference's start-of-updates gate (check_covariance_matrices,
// danse_toolbox/d_classes.py:1430-1540): once the frame counters allow it,
// a family-node starts updating only if, over ALL bins,
//   GEVD: Rnn and Ryy are Hermitian (np.allclose(X^H, X): |X^H - X| <=
//         1e-8 + 1e-5 |X| elementwise), eigvalsh >= 0 and full rank;
//   MWF:  Rnn and Ryy are full rank.
// Evaluated on the device for one round, on the SCMs as the reference holds
// them after that round's recursion (the kernel applies the round's update
// to a private copy; the update kernel then repeats it for real).
//
// Storage: the engine keeps the LOWER triangle (eigh reads it).  The
// reference matrix is X = H + Q with Q anti-Hermitian; Q = q Q0, Q0 = (R0 -
// R0^H) / 2 from the init slice R0, q = beta^m (m recursion steps since the
// init, 0 after a first-frame SET) -- the recursion adds only Hermitian terms.
// So conj(X_ji) - X_ij = -2 Q_ij, and X_ji = conj(X_ij - 2 Q_ij).
//
// eigvalsh >= 0 and the rank test become one float64 Cholesky of the
// lower-triangle Hermitian matrix with every pivot above D eps trace(X) (the
// matrix_rank tolerance sigma_max max(M, N) eps with sigma_max <= trace).
// MWF runs the rank test alone: a signed elimination that accepts negative
// pivots (an indefinite full-rank SCM passes, as in the reference).
// One (candidate, bin) per wavefront, the matrix in LDS.
#pragma once
#include <type_traits>

#include "kernels.hpp"

namespace danse {

struct GateCand {
  int fni;      // index into the engine's family-node table
  int s;        // scene
  double qY;    // beta^m of Ryy's init residue (0: a SET wiped it)
  double qN;    // ... of Rnn's
};

// (lower) triangle entry e = i (i + 1) / 2 + j -> (i, j)
DANSE_DEV void tri_ij(int e, int& i, int& j) {
  int r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  while (r * (r + 1) / 2 > e) --r;
  while ((r + 1) * (r + 2) / 2 <= e) ++r;
  i = r;
  j = e - r * (r + 1) / 2;
}

// All 64 lanes share every step: the loads, the recursion and the Hermitian
// test go over the packed lower triangle in storage order (coalesced), the
// Cholesky's trailing updates over the trailing triangle's entries.
// (filter dimensions up to kGateMaxD: the online centralised family above
// 64 channels -- [D][D + 1] complex doubles of dynamic LDS, 147 KiB at 96;
// gate_wide_kernel below takes the larger ones)
constexpr int kGateMaxD = 96;
__global__ void __launch_bounds__(64) gate_kernel(const UpdateArgs a, const FamNode* fns, const GateCand* cand,
                                                 const long long* initOff, const cd* scm0, int perBin, int* verdict) {
  extern __shared__ cd gX[];   // [D][D + 1]
  const int li = threadIdx.x;
  const int f = blockIdx.x;
  const GateCand c = cand[blockIdx.y];
  const FamNode d = fns[c.fni];
  if (!node_in(a.nodeMask, d.k)) return;   // (fewSamples: checked before its node's update step)
  const int D = d.D, s = c.s, F = a.F;
  const int P = D + 1;
  const int T = D * (D + 1) / 2;
  const uint8_t fl = a.flags[(((long long)a.r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  __shared__ cf gy[kGateMaxD];
  __shared__ double gd[kGateMaxD];   // diagonal entries (the trace)
  for (int i = li; i < D; i += 64) gy[i] = load_y(a, d, s, f, i, true);
  __syncthreads();
  const double beta = a.beta[s * a.K + d.k];
  const cd* R0 = scm0 + initOff[c.fni] + (perBin ? (long long)f * D * D : 0ll);
  bool pass = true;
  for (int which = 0; which < 2; ++which) {   // 0: Ryy, 1: Rnn
    const int op = which == 0 ? (fl & 3) : ((fl >> 2) & 3);
    const double q = which == 0 ? c.qY : c.qN;
    const double cy = (op == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (op == DANSE_OP_SET) ? 0.0 : beta;
    bool herm = true;
    for (int i = li; i < D; i += 64) gd[i] = 0.0;
    __syncthreads();
    for (int e = li; e < T; e += 64) {
      int i, j;
      tri_ij(e, i, j);
      const long long ee = scm_lower(d, a.scmStride, s, F, f, i, j);
      cd x = scm_entry(a, d, which == 0, ee);
      if (i == j) x.im = 0.0;   // the stored diagonal is real; its init residue is Q_ii
      if (op != DANSE_OP_KEEP) {
        cd yy = cd{0.0, 0.0};
        fma_cc(yy, cdk(gy[i]), cdk(gy[j]));
        x = cx * x;
        x.re = fma(cy, yy.re, x.re);
        x.im = fma(cy, (i == j) ? 0.0 : yy.im, x.im);
      }
      const cd r0ij = R0[i * D + j], r0ji = R0[j * D + i];
      const cd Q = cd{0.5 * q * (r0ij.re - r0ji.re), 0.5 * q * (r0ij.im + r0ji.im)};   // q (R0 - R0^H)_ij / 2
      if (i == j) {
        const double qi = q * r0ij.im;   // X_ii = x.re + i qi
        herm = herm && (2.0 * fabs(qi) <= 1e-8 + 1e-5 * sqrt(x.re * x.re + qi * qi));
        gd[i] = x.re;
        gX[i * P + j] = cd{x.re, 0.0};
      } else {
        const double aq = 2.0 * sqrt(Q.re * Q.re + Q.im * Q.im);
        const double xr = x.re, xi = x.im;                        // X_ij = H_ij + Q_ij (stored)
        const double mr = xr - 2.0 * Q.re, mi = xi - 2.0 * Q.im;   // conj(X_ji) = X_ij - 2 Q_ij
        herm = herm && (aq <= 1e-8 + 1e-5 * sqrt(xr * xr + xi * xi)) && (aq <= 1e-8 + 1e-5 * sqrt(mr * mr + mi * mi));
        gX[i * P + j] = cd{xr, xi};
      }
    }
    // GEVD: Hermitian over every entry of every bin
    if (a.gevd && __ballot(!herm) != 0ull) pass = false;
    __syncthreads();
    // full rank (+ positive definite): float64 Cholesky of the lower triangle
    double tr = 0.0;
    for (int i = li; i < D; i += 64) tr += gd[i];
    for (int o = 32; o >= 1; o >>= 1) tr += __shfl_xor(tr, o);
    const double tol = (double)D * 2.220446049250313e-16 * fabs(tr);
    // GEVD (eigvalsh >= 0 and full rank): every pivot above tol.  MWF (rank
    // only, _check_validity_nogevd, d_classes.py:1473-1480): a signed
    // (LDL^H) elimination -- negative pivots are accepted, |pivot| > tol
    for (int j = 0; j < D && pass; ++j) {
      const double pj = gX[j * P + j].re;
      if (!(a.gevd ? pj > tol : fabs(pj) > tol)) {
        pass = false;   // (wave-uniform: every lane read the same pivot)
        break;
      }
      const double inv = 1.0 / sqrt(fabs(pj));
      for (int row = li; row < D; row += 64)
        if (row > j) gX[row * P + j] = inv * gX[row * P + j];
      __syncthreads();
      // trailing lower triangle (rows and columns j + 1 .. D - 1), entry by entry
      const int n = D - 1 - j;
      for (int e = li; e < n * (n + 1) / 2; e += 64) {
        int i2, k2;
        tri_ij(e, i2, k2);
        const int row = j + 1 + i2, col = j + 1 + k2;
        const cd lij = gX[row * P + j];
        if (pj > 0.0) fms_cc(gX[row * P + col], lij, gX[col * P + j]);
        else fma_cc(gX[row * P + col], lij, gX[col * P + j]);
      }
      __syncthreads();
    }
    __syncthreads();
    if (!pass) break;
  }
  if (li == 0 && !pass) atomicAnd(&verdict[blockIdx.y], 0);
}

// The same checks above kGateMaxD (the online centralised family up to 256
// channels, wide classes): one 256-thread workgroup per (candidate, bin), the
// packed lower triangle in a global workspace (T complex doubles per
// workgroup, launched in chunks), the Cholesky right-looking over the packed
// trailing triangle with the pivot test of gate_kernel (same entry-wise
// arithmetic, so the same verdicts).
constexpr int kGateWideThr = 256;
DANSE_DEV long long pk_lo(int i, int j) { return (long long)i * (i + 1) / 2 + j; }
__global__ void __launch_bounds__(kGateWideThr) gate_wide_kernel(const UpdateArgs a, const FamNode* fns,
                                                                 const GateCand* cand, const long long* initOff,
                                                                 const cd* scm0, int perBin, int* verdict,
                                                                 long long item0, cd* work) {
  const long long item = item0 + blockIdx.x;
  const int F = a.F;
  const int ci = (int)(item / F), f = (int)(item % F);
  const GateCand c = cand[ci];
  const FamNode d = fns[c.fni];
  if (!node_in(a.nodeMask, d.k)) return;   // (workgroup-uniform)
  const int tid = threadIdx.x;
  const int D = d.D, s = c.s;
  const int T = D * (D + 1) / 2;
  cd* X = work + (long long)blockIdx.x * T;
  const uint8_t fl = a.flags[(((long long)a.r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  __shared__ cf gy[256];
  __shared__ double red[kGateWideThr / 64];
  __shared__ int flag;
  for (int i = tid; i < D; i += kGateWideThr) gy[i] = load_y(a, d, s, f, i, true);
  __syncthreads();
  const double beta = a.beta[s * a.K + d.k];
  const cd* R0 = scm0 + initOff[c.fni] + (perBin ? (long long)f * D * D : 0ll);
  bool pass = true;
  for (int which = 0; which < 2 && pass; ++which) {   // 0: Ryy, 1: Rnn
    const int op = which == 0 ? (fl & 3) : ((fl >> 2) & 3);
    const double q = which == 0 ? c.qY : c.qN;
    const double cy = (op == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (op == DANSE_OP_SET) ? 0.0 : beta;
    bool herm = true;
    double tr = 0.0;
    for (int e = tid; e < T; e += kGateWideThr) {
      int i, j;
      tri_ij(e, i, j);
      const long long ee = scm_lower(d, a.scmStride, s, F, f, i, j);
      cd x = scm_entry(a, d, which == 0, ee);
      if (i == j) x.im = 0.0;
      if (op != DANSE_OP_KEEP) {
        cd yy = cd{0.0, 0.0};
        fma_cc(yy, cdk(gy[i]), cdk(gy[j]));
        x = cx * x;
        x.re = fma(cy, yy.re, x.re);
        x.im = fma(cy, (i == j) ? 0.0 : yy.im, x.im);
      }
      const cd r0ij = R0[i * D + j], r0ji = R0[j * D + i];
      const cd Q = cd{0.5 * q * (r0ij.re - r0ji.re), 0.5 * q * (r0ij.im + r0ji.im)};
      if (i == j) {
        const double qi = q * r0ij.im;
        herm = herm && (2.0 * fabs(qi) <= 1e-8 + 1e-5 * sqrt(x.re * x.re + qi * qi));
        tr += x.re;
        X[e] = cd{x.re, 0.0};
      } else {
        const double aq = 2.0 * sqrt(Q.re * Q.re + Q.im * Q.im);
        const double xr = x.re, xi = x.im;
        const double mr = xr - 2.0 * Q.re, mi = xi - 2.0 * Q.im;
        herm = herm && (aq <= 1e-8 + 1e-5 * sqrt(xr * xr + xi * xi)) && (aq <= 1e-8 + 1e-5 * sqrt(mr * mr + mi * mi));
        X[e] = cd{xr, xi};
      }
    }
    if (a.gevd && __syncthreads_or(!herm)) pass = false;
    // the trace (every diagonal entry, summed over the workgroup)
    for (int o = 32; o >= 1; o >>= 1) tr += __shfl_xor(tr, o);
    if ((tid & 63) == 0) red[tid >> 6] = tr;
    __syncthreads();
    tr = 0.0;
    for (int w = 0; w < kGateWideThr / 64; ++w) tr += red[w];
    const double tol = (double)D * 2.220446049250313e-16 * fabs(tr);
    __threadfence_block();
    __syncthreads();
    for (int j = 0; j < D && pass; ++j) {
      const double pj = X[pk_lo(j, j)].re;   // (every thread reads the same pivot: uniform)
      if (!(a.gevd ? pj > tol : fabs(pj) > tol)) {
        pass = false;
        break;
      }
      const double inv = 1.0 / sqrt(fabs(pj));
      for (int row = j + 1 + tid; row < D; row += kGateWideThr) X[pk_lo(row, j)] = inv * X[pk_lo(row, j)];
      __threadfence_block();
      __syncthreads();
      const int n = D - 1 - j;
      for (int e = tid; e < n * (n + 1) / 2; e += kGateWideThr) {
        int i2, k2;
        tri_ij(e, i2, k2);
        const int row = j + 1 + i2, col = j + 1 + k2;
        const cd lij = X[pk_lo(row, j)];
        if (pj > 0.0) fms_cc(X[pk_lo(row, col)], lij, X[pk_lo(col, j)]);
        else fma_cc(X[pk_lo(row, col)], lij, X[pk_lo(col, j)]);
      }
      __threadfence_block();
      __syncthreads();
    }
    __syncthreads();
  }
  (void)flag;
  if (tid == 0 && !pass) atomicAnd(&verdict[ci], 0);
}

// The same checks for D <= kGateRegMaxD with the matrix in REGISTERS: lane li
// holds the packed lower entries e = li + 64 m (m < NE, NE = ceil(T / 64)
// rounded to 2, 4, 8 or 13) of its
// (candidate, bin), their (row, column) found once; per Cholesky step only
// column j goes through LDS (its owners write it, every lane reads the
// entries its updates need).  The arithmetic of every entry is gate_kernel's
// (the column scaled by 1 / sqrt|p_j| as each lane reads it, then
// X[i][c] -= l_i conj(l_c)), so the verdicts are the same; no per-entry
// index arithmetic and no LDS read-modify-write per step (gate_kernel keeps
// the larger D).
constexpr int kGateRegMaxD = 40;
// entries per lane, NE = ceil(T / 64) rounded up to an instantiated size
constexpr int gate_reg_ne(int dmax) {
  const int n = (dmax * (dmax + 1) / 2 + 63) / 64;
  return n <= 2 ? 2 : n <= 4 ? 4 : n <= 8 ? 8 : 13;
}
template <int kGateRegNE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kGateRegNE <= 4 ? 4 : 2)))
gate_kernel_reg(const UpdateArgs a, const FamNode* fns, const GateCand* cand, const long long* initOff, const cd* scm0,
                int perBin, int* verdict) {
  const int li = threadIdx.x;
  const int f = blockIdx.x;
  const GateCand c = cand[blockIdx.y];
  const FamNode d = fns[c.fni];
  if (!node_in(a.nodeMask, d.k)) return;
  const int D = d.D, s = c.s, F = a.F;
  const int T = D * (D + 1) / 2;
  const uint8_t fl = a.flags[(((long long)a.r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  __shared__ cf gy[kGateRegMaxD];
  __shared__ cd colv[kGateRegMaxD];
  for (int i = li; i < D; i += 64) gy[i] = load_y(a, d, s, f, i, true);
  // this lane's entries: rows / columns (T <= 1176: 11 bits each)
  int rc[kGateRegNE];
  sfor<0, kGateRegNE>([&](auto mc) {
    constexpr int m = decltype(mc)::value;
    const int e = li + 64 * m;
    int i = 0, j = 0;
    if (e < T) tri_ij(e, i, j);
    rc[m] = (e < T) ? (i << 16) | j : -1;
  });
  __syncthreads();
  const double beta = a.beta[s * a.K + d.k];
  const cd* R0 = scm0 + initOff[c.fni] + (perBin ? (long long)f * D * D : 0ll);
  bool pass = true;
  for (int which = 0; which < 2 && pass; ++which) {   // 0: Ryy, 1: Rnn
    const int op = which == 0 ? (fl & 3) : ((fl >> 2) & 3);
    const double q = which == 0 ? c.qY : c.qN;
    const double cy = (op == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (op == DANSE_OP_SET) ? 0.0 : beta;
    bool herm = true;
    double tr = 0.0;
    cd X[kGateRegNE];
    sfor<0, kGateRegNE>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      // (a compiler fence every 4 entries: their loads are not all hoisted
      // over the earlier entries' arithmetic, which would spill)
      if constexpr (m % 4 == 0) asm volatile("" ::: "memory");
      X[m] = cd{0.0, 0.0};
      if (rc[m] >= 0) {
        const int i = rc[m] >> 16, j = rc[m] & 0xffff;
        const long long ee = scm_lower(d, a.scmStride, s, F, f, i, j);
        cd x = scm_entry(a, d, which == 0, ee);
        if (i == j) x.im = 0.0;
        if (op != DANSE_OP_KEEP) {
          cd yy = cd{0.0, 0.0};
          fma_cc(yy, cdk(gy[i]), cdk(gy[j]));
          x = cx * x;
          x.re = fma(cy, yy.re, x.re);
          x.im = fma(cy, (i == j) ? 0.0 : yy.im, x.im);
        }
        const cd r0ij = R0[i * D + j], r0ji = R0[j * D + i];
        const cd Q = cd{0.5 * q * (r0ij.re - r0ji.re), 0.5 * q * (r0ij.im + r0ji.im)};
        if (i == j) {
          const double qi = q * r0ij.im;
          herm = herm && (2.0 * fabs(qi) <= 1e-8 + 1e-5 * sqrt(x.re * x.re + qi * qi));
          tr += x.re;
          X[m] = cd{x.re, 0.0};
        } else {
          const double aq = 2.0 * sqrt(Q.re * Q.re + Q.im * Q.im);
          const double xr = x.re, xi = x.im;
          const double mr = xr - 2.0 * Q.re, mi = xi - 2.0 * Q.im;
          herm = herm && (aq <= 1e-8 + 1e-5 * sqrt(xr * xr + xi * xi)) &&
                 (aq <= 1e-8 + 1e-5 * sqrt(mr * mr + mi * mi));
          X[m] = cd{xr, xi};
        }
      }
    });
    if (a.gevd && __ballot(!herm) != 0ull) pass = false;
    for (int o = 32; o >= 1; o >>= 1) tr += __shfl_xor(tr, o);
    const double tol = (double)D * 2.220446049250313e-16 * fabs(tr);
    for (int j = 0; j < D && pass; ++j) {
      // column j (rows >= j) from its owners to LDS
      sfor<0, kGateRegNE>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        if (rc[m] >= 0 && (rc[m] & 0xffff) == j) colv[rc[m] >> 16] = X[m];
      });
      __syncthreads();
      const double pj = colv[j].re;   // (uniform)
      if (!(a.gevd ? pj > tol : fabs(pj) > tol)) {
        pass = false;
        break;
      }
      const double inv = 1.0 / sqrt(fabs(pj));
      sfor<0, kGateRegNE>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        if constexpr (m % 4 == 0) asm volatile("" ::: "memory");
        const int i = rc[m] >> 16, cc = rc[m] & 0xffff;
        if (rc[m] >= 0 && cc > j) {
          const cd xi = colv[i], xc = colv[cc];
          const cd lij = cd{inv * xi.re, inv * xi.im}, lcj = cd{inv * xc.re, inv * xc.im};
          if (pj > 0.0) fms_cc(X[m], lij, lcj);
          else fma_cc(X[m], lij, lcj);
        }
      });
      __syncthreads();   // (every read of column j before the next column's writes)
    }
  }
  if (li == 0 && !pass) atomicAnd(&verdict[blockIdx.y], 0);
}

// The same checks for D <= 11 with one (candidate, bin) per LANE: the lane's
// packed lower triangle in float64 registers and its Cholesky sequential in
// the lane; for the lane classes' bin-minor SCMs every entry is one
// coalesced wave access.  When one init slice serves every bin (PB false),
// the wave's (at most two) candidates' slices are staged in LDS and the
// Hermitian test runs on the factorisation's registers, one entry at a time
// (scheduling barriers: the square-root sequences of many entries
// interleaved would spill); per-bin slices (PB) take a pass of their own over
// the triangle and the slice.  Per entry the arithmetic of gate_kernel (the
// column scaled by 1 / sqrt|p_j|, then X[i][c] -= l_i conj(l_c)); the trace
// is summed in row order.  The triangle is padded to DMAX with a decoupled
// identity block above the tolerance (the real pivots are unchanged, the
// factorisation runs without per-lane guards, a failed pivot only clears
// pass).  DMAX is the launch's largest D (4, 8 or 11; a launch with D = 12
// takes gate_kernel_reg, whose registers it fits); each lane runs its own
// candidate's D.
constexpr int kGateLaneMaxD = 12;
template <int DMAX, bool PB>
__global__ void __launch_bounds__(64) gate_kernel_lane(const UpdateArgs a, const FamNode* fns, const GateCand* cand,
                                                      int nCand, const long long* initOff, const cd* scm0, int perBin,
                                                      int* verdict) {
  constexpr int NT = DMAX * (DMAX + 1) / 2;
  constexpr auto P = [](int i, int j) { return i * (i + 1) / 2 + j; };
  const int F = a.F;
  const long long total = (long long)nCand * F;
  const long long gid0 = (long long)blockIdx.x * 64 + threadIdx.x;
  const bool live = gid0 < total;
  const long long gid = live ? gid0 : total - 1;
  const int ci = (int)(gid / F), f = (int)(gid % F);
  const GateCand c = cand[ci];
  const FamNode d = fns[c.fni];
  const int D = d.D, s = c.s;
  // the init slices of the wave's (at most two) candidates in LDS, when one
  // slice serves every bin (perBin = 0): the Hermitian test reads them there
  __shared__ cd r0s[2][kGateLaneMaxD * kGateLaneMaxD];
  const int c0 = __builtin_amdgcn_readfirstlane(ci);
  const int c1 = __shfl(ci, 63);
  if constexpr (!PB) {
    sfor<0, 2>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int ck = k == 0 ? c0 : c1;
      const int fk = cand[ck].fni;
      const int Dk = fns[fk].D;
      const cd* src = scm0 + initOff[fk];
      for (int e = threadIdx.x; e < Dk * Dk; e += 64) r0s[k][e] = src[e];
    });
  }
  __syncthreads();
  if (!live || !node_in(a.nodeMask, d.k)) return;
  const cd* R0s = r0s[ci == c0 ? 0 : 1];
  const uint8_t fl = a.flags[(((long long)a.r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  // the observation vector (entries past D: a valid channel, unused), also in
  // LDS for pass 1's runtime-indexed rows (this lane's column)
  __shared__ cf ys[DMAX][64];
  cf y[DMAX];
  load_y_all<DMAX>(a, d, s, f, y, D);
  sfor<0, DMAX>([&](auto ic) { ys[decltype(ic)::value][threadIdx.x] = y[decltype(ic)::value]; });
  const double beta = a.beta[s * a.K + d.k];
  const cd* R0 = scm0 + initOff[c.fni] + (perBin ? (long long)f * D * D : 0ll);
  bool pass = true;
  // Ryy (float32 storage), then Rnn (float64): one code path each, so that no
  // entry load sits behind a per-entry test of which matrix it reads
  auto check = [&](auto ryyc) {
    constexpr bool RYY = decltype(ryyc)::value;
    auto ld = [&](long long ee) -> cd { if constexpr (RYY) return cdk(a.Ryy[ee]); else return a.Rnn[ee]; };
    const int op = RYY ? (fl & 3) : ((fl >> 2) & 3);
    const double q = RYY ? c.qY : c.qN;
    const double cy = (op == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (op == DANSE_OP_SET) ? 0.0 : beta;
    // pass 1 (per-bin init slices only), a runtime loop over the entries
    // (each one's Hermitian test runs three square roots: unrolled, their
    // sequences interleave and spill): the Hermitian test against the init
    // residue and the trace; the entries are read again for the factorisation
    bool herm = true;
    double tr = 0.0;
#pragma unroll 1
    for (int i = 0; i < (PB ? D : 0); ++i) {
      const cf yi = ys[i][threadIdx.x];
#pragma unroll 6
      for (int j = 0; j <= i; ++j) {
        cd x = ld(scm_lower(d, a.scmStride, s, F, f, i, j));
        if (i == j) x.im = 0.0;
        if (op != DANSE_OP_KEEP) {
          cd yy = cd{0.0, 0.0};
          fma_cc(yy, cdk(yi), cdk(ys[j][threadIdx.x]));
          x = cx * x;
          x.re = fma(cy, yy.re, x.re);
          x.im = fma(cy, (i == j) ? 0.0 : yy.im, x.im);
        }
        const cd r0ij = R0[i * D + j], r0ji = R0[j * D + i];
        const cd Q = cd{0.5 * q * (r0ij.re - r0ji.re), 0.5 * q * (r0ij.im + r0ji.im)};
        if (i == j) {
          const double qi = q * r0ij.im;
          herm = herm && (2.0 * fabs(qi) <= 1e-8 + 1e-5 * sqrt(x.re * x.re + qi * qi));
          tr += x.re;
        } else {
          const double aq = 2.0 * sqrt(Q.re * Q.re + Q.im * Q.im);
          const double xr = x.re, xi = x.im;
          const double mr = xr - 2.0 * Q.re, mi = xi - 2.0 * Q.im;
          herm = herm && (aq <= 1e-8 + 1e-5 * sqrt(xr * xr + xi * xi)) &&
                 (aq <= 1e-8 + 1e-5 * sqrt(mr * mr + mi * mi));
        }
      }
    }
    // pass 2: the triangle into registers (rows past D read row D - 1's
    // entries; the padding replaces them below)
    cd X[NT];
    sfor<0, DMAX>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      asm volatile("" ::: "memory");   // (one row's loads in flight at a time)
      sfor<0, i + 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        cd x = ld(scm_lower(d, a.scmStride, s, F, f, min(i, D - 1), min(j, D - 1)));
        if constexpr (i == j) x.im = 0.0;
        if (op != DANSE_OP_KEEP) {
          cd yy = cd{0.0, 0.0};
          fma_cc(yy, cdk(ys[i][threadIdx.x]), cdk(ys[j][threadIdx.x]));
          x = cx * x;
          x.re = fma(cy, yy.re, x.re);
          x.im = fma(cy, (i == j) ? 0.0 : yy.im, x.im);
        }
        X[P(i, j)] = x;
      });
    });
    if constexpr (!PB) {
      // the Hermitian test and the trace on the registers, the init residues
      // from LDS, one entry at a time (scheduling barriers: the square-root
      // sequences of many entries interleaved would spill)
      sfor<0, DMAX>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        sfor<0, i + 1>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          __builtin_amdgcn_sched_barrier(0);
          if (i < D) {
            const cd x = X[P(i, j)];
            const cd r0ij = R0s[i * D + j], r0ji = R0s[j * D + i];
            const cd Q = cd{0.5 * q * (r0ij.re - r0ji.re), 0.5 * q * (r0ij.im + r0ji.im)};
            if constexpr (i == j) {
              const double qi = q * r0ij.im;
              herm = herm && (2.0 * fabs(qi) <= 1e-8 + 1e-5 * sqrt(x.re * x.re + qi * qi));
              tr += x.re;
            } else {
              const double aq = 2.0 * sqrt(Q.re * Q.re + Q.im * Q.im);
              const double xr = x.re, xi = x.im;
              const double mr = xr - 2.0 * Q.re, mi = xi - 2.0 * Q.im;
              herm = herm && (aq <= 1e-8 + 1e-5 * sqrt(xr * xr + xi * xi)) &&
                     (aq <= 1e-8 + 1e-5 * sqrt(mr * mr + mi * mi));
            }
          }
        });
      });
      __builtin_amdgcn_sched_barrier(0);
    }
    if (a.gevd && !herm) pass = false;
    const double tol = (double)D * 2.220446049250313e-16 * fabs(tr);
    // the padding past D: an identity block scaled above the tolerance
    // (decoupled: the real pivots are the same, the padded ones pass), so
    // that the factorisation below runs without per-lane guards
    const double pad = 1.0 + 2.0 * tol;
    sfor<1, DMAX>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      sfor<0, i + 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if (i >= D) X[P(i, j)] = cd{(i == j) ? pad : 0.0, 0.0};
      });
    });
    // right-looking Cholesky (GEVD) / signed elimination (MWF), every step
    // run: a failed pivot only clears pass
    sfor<0, DMAX>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const double pj = X[P(j, j)].re;
      pass = pass && (a.gevd ? pj > tol : fabs(pj) > tol);
      const double inv = 1.0 / sqrt(fabs(pj));
      sfor<j + 1, DMAX>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        X[P(i, j)] = cd{inv * X[P(i, j)].re, inv * X[P(i, j)].im};
      });
      sfor<j + 1, DMAX>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        // X[i][k] -= l_i conj(l_k) for a positive pivot (fma_cc with -l_i:
        // the same fused operations as fms_cc), += for a negative one
        const cd lij = X[P(i, j)];
        const cd ls = (pj > 0.0) ? cd{-lij.re, -lij.im} : lij;
        sfor<j + 1, i + 1>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          fma_cc(X[P(i, k)], ls, X[P(k, j)]);
        });
      });
    });
  };
  check(std::true_type{});
  if (pass) check(std::false_type{});
  if (!pass) atomicAnd(&verdict[ci], 0);
}

}  // namespace danse

