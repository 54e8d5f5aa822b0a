// CohDrift SRO estimation, closed or open loop, least-squares fit over bins
// (update_sro_estimates + build_phase_shifts_for_srocomp,
// danse_toolbox/d_classes.py:2364-2621; cohdrift_sro_estimation with
// method 'ls', danse_toolbox/d_sros.py:19-95), one workgroup per (scene,
// owned node k, neighbour q), launched after every round's update (a
// receiver needs its own local spectrum and the all-gathered fused spectra
// only, so a node-sharded engine estimates for its own nodes):
//   * the coherence of the compensated observation, yyH[0, q] /
//     sqrt(yyH[0, 0] yyH[q, q]) with yyH = y y^H / D, goes to a ring of
//     segLength + 1 rounds;
//   * on estimation rounds, res_f = coh_f(i) conj(coh_f(i - ld)) laid out as
//     the reference's 2 (F - 1)-bin spectrum [res_0 .. res_{F-2},
//     conj(res_{F-1}) .. conj(res_1)], exponentially averaged; the LS fit
//     reads its last F entries, which are res_{F-2} and conj(res_{F-1} ..
//     res_1) (kept as avgTail[kappa]);  sro = -sum b angle / sum b^2,
//     b_kappa = pi kappa ld Ns / (2 F);
//   * eps = sro / (1 + sro) alphaEps; the sender's phase accumulator
//     (added to zPhase in load_y from the next round on) loses eps Ns.
// Open loop (cohDrift.loop 'open', d_classes.py:2439-2450,2580-2584): the
// coherence of the UNcompensated observation (no zPhase / accumulator
// rotation), every residual-product entry n of the 2 (F - 1)-bin spectrum
// times exp(j 2 pi n W / (2 (F - 1))) with W = bufferFlagPos - bufferFlagPri
// (flagWin, the full-sample drifts inside the segment; d_sros.py:19-95), and
// eps = sro / (1 + sro) (no alphaEps).
#pragma once
#include "kernels.hpp"

namespace danse {

struct CohDriftArgs {
  int S, K, MT, F, r, ld, start, every, nIter, compensate;
  int k0, nOwn;         // receivers k0 .. k0 + nOwn - 1 (a node-sharded engine owns a block)
  double alpha, alphaEps, Ns;
  const int* base;      // [K] first channel of node k
  cd* ring;             // [ld + 1][S][K][K - 1][F]
  cd* avgTail;          // [S][K][K - 1][F]
  double* phase;        // [S][K][K] accumulator
  double* est;          // [S][K][R][K - 1]
  double* res;          // [S][K][R][K - 1]
  int R;
  int open;                     // 1: open loop
  const double* flagWin;        // open loop: [R][K][K] bufferFlagPos - bufferFlagPri
};

constexpr int kCdThreads = 576;   // >= F = 513, nine waves

__global__ void __launch_bounds__(kCdThreads) cohdrift_kernel(const UpdateArgs a, const CohDriftArgs c) {
  __shared__ cd coh[kCdThreads];
  __shared__ double red[2][kCdThreads / 64];
  const int K = c.K, F = c.F, r = c.r;
  const int qi = blockIdx.x % (K - 1);
  const int k = c.k0 + (int)((blockIdx.x / (K - 1)) % c.nOwn);
  const int s = blockIdx.x / ((K - 1) * c.nOwn);
  const int qg = qi < k ? qi : qi + 1;
  const int t = threadIdx.x;
  const long long ringStride = (long long)c.S * K * (K - 1) * F;
  const long long chunk = (((long long)s * K + k) * (K - 1) + qi) * F;
  if (t < F) {
    // local reference mic (channel base[k]) and sender qg's fused frame, as load_y
    const cf y0 = a.Yspec[(((long long)((r + 1) & 1) * a.S + s) * a.MT + c.base[k]) * F + t];
    const long long lk = ((long long)r * K + k) * K + qg;
    const int lag = a.zLag ? a.zLag[lk] : 0;
    cf yq = a.Zspec[((((long long)((r - lag) & 1)) * K + qg) * a.S + s) * F + t];
    if (a.zPhase && !c.open) {
      double ph = a.zPhase[lk];
      if (a.cdPhase) ph += a.cdPhase[((long long)s * K + k) * K + qg];
      double tt = (double)t * ph / (double)(2 * (F - 1));
      tt -= rint(tt);
      float sn, cs;
      sincospif(-2.0f * (float)tt, &sn, &cs);
      yq = yq * cf{cs, sn};
    }
    const cd a0 = cdk(y0), aq = cdk(yq);
    const cd yy0q = cd{a0.re * aq.re + a0.im * aq.im, a0.im * aq.re - a0.re * aq.im};   // y0 conj(yq)
    const double yy00 = a0.re * a0.re + a0.im * a0.im, yyqq = aq.re * aq.re + aq.im * aq.im;
    const double den = sqrt(yy00 * yyqq);
    const cd v = cd{yy0q.re / den, yy0q.im / den};
    coh[t] = v;
    c.ring[(long long)(r % (c.ld + 1)) * ringStride + chunk + t] = v;
  }
  __syncthreads();
  const bool estRound = r >= c.start && r < c.nIter && ((r - c.start) % c.every) == 0;
  if (!estRound) return;
  const bool first = r == c.start;
  double num = 0.0, bb = 0.0;
  if (t < F) {
    const int kap = t;
    const int f = (kap == 0) ? F - 2 : F - kap;
    const cd pri = c.ring[(long long)((r - c.ld) % (c.ld + 1)) * ringStride + chunk + f];
    const cd cp = coh[f];
    cd rv = cd{cp.re * pri.re + cp.im * pri.im, cp.im * pri.re - cp.re * pri.im};   // coh conj(pri)
    if (kap != 0) rv.im = -rv.im;                                                    // conj for the mirrored half
    if (c.open) {
      // entry n = F - 2 + kap of the 2 (F - 1)-bin spectrum times
      // exp(j 2 pi n W / (2 (F - 1))), in double (the reference's complex128)
      const double W = c.flagWin[((long long)r * K + k) * K + qg];
      const double ang = 2.0 * M_PI * (double)(F - 2 + kap) * W / (double)(2 * (F - 1));
      double sn, cs;
      sincos(ang, &sn, &cs);
      rv = cd{rv.re * cs - rv.im * sn, rv.re * sn + rv.im * cs};
    }
    cd* av = c.avgTail + chunk + kap;
    const cd avg = first ? rv : cd{c.alpha * av->re + (1.0 - c.alpha) * rv.re, c.alpha * av->im + (1.0 - c.alpha) * rv.im};
    *av = avg;
    const double b = M_PI * (double)kap * (double)(c.ld * c.Ns) / ((double)F * 2.0);
    num = b * atan2(avg.im, avg.re);
    bb = b * b;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    num += __shfl_xor(num, o);
    bb += __shfl_xor(bb, o);
  }
  if ((t & 63) == 0) {
    red[0][t >> 6] = num;
    red[1][t >> 6] = bb;
  }
  __syncthreads();
  if (t == 0) {
    double sn = 0.0, sb = 0.0;
    for (int w = 0; w < kCdThreads / 64; ++w) {
      sn += red[0][w];
      sb += red[1][w];
    }
    const double sro = -sn / sb;
    const double eps = c.open ? sro / (1.0 + sro) : sro / (1.0 + sro) * c.alphaEps;
    const long long o = (((long long)s * K + k) * c.R + r) * (K - 1) + qi;
    c.res[o] = sro;
    c.est[o] = c.compensate ? eps : 0.0;
    if (c.compensate) c.phase[((long long)s * K + k) * K + qg] -= eps * c.Ns;
  }
}

}  // namespace danse
