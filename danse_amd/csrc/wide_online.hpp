// The online centralised family above 64 channels (SURVEY §8(f) rank 3,
// d_classes.py:1542-1585 build_ycentr, 2139-2201 the centralised SCM
// recursion, 3343-3387 its GEVD filter, 2657-2709 the centralised estimate):
// the family-nodes of filter dimension sum(M) > 64 stay out of the lane and
// lane-grid classes.  Per round:
//   wide_rec_kernel   one 256-thread workgroup per (scene, family-node, bin):
//                     the centralised vector into LDS, then the recursion of
//                     the SCM this round's VAD selects over its packed lower
//                     triangle (bin-major, FamNode.packed 2: Ryy and Rnn
//                     complex128, kernels.hpp wide_fn);
//   wide_filter_kernel (wide.hpp) per family-node over its solving (scene,
//                     bin) items, float64, writing w[r + 1];
//   wide_tail_kernel  one wave per (scene, family-node, bin): the filter of
//                     the rounds without a solve carried over, dhat = w^H y.
#pragma once
#include "gate.hpp"

namespace danse {

constexpr int kWideRecThr = 256;

__global__ void __launch_bounds__(kWideRecThr) wide_rec_kernel(const UpdateArgs a, const FamNode* fns, const int* ids,
                                                               int nW) {
  const int f = blockIdx.x;
  const int s = blockIdx.y / nW;
  const FamNode d = fns[ids[blockIdx.y % nW]];
  if (!node_in(a.nodeMask, d.k)) return;
  const uint8_t fl = a.flags[(((long long)a.r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  const int opY = fl & 3, opN = (fl >> 2) & 3;
  if (!opY && !opN) return;   // (workgroup-uniform)
  const int D = d.D, F = a.F;
  __shared__ cf ys[256];
  for (int i = threadIdx.x; i < D; i += kWideRecThr) ys[i] = load_y(a, d, s, f, i, true);
  __syncthreads();
  const double beta = a.beta[s * a.K + d.k];
  const int T = D * (D + 1) / 2;
  const long long base = (long long)s * a.scmStride + d.scmOff + (long long)f * T;
  if (opY) {
    // (float64, in the Rnn array past this fn's Rnn: kernels.hpp wide_fn)
    cd* RyyD = a.Rnn + wide_ryy_shift(d, F);
    const double cy = (opY == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (opY == DANSE_OP_SET) ? 0.0 : beta;
    for (int e = threadIdx.x; e < T; e += kWideRecThr) {
      int i, j;
      tri_ij(e, i, j);
      cd x = RyyD[base + e];
      if (i == j) x.im = 0.0;
      cd yy = cd{0.0, 0.0};
      fma_cc(yy, cdk(ys[i]), cdk(ys[j]));
      x = cx * x;
      x.re = fma(cy, yy.re, x.re);
      x.im = (i == j) ? 0.0 : fma(cy, yy.im, x.im);
      RyyD[base + e] = x;
    }
  }
  if (opN) {
    const double cy = (opN == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (opN == DANSE_OP_SET) ? 0.0 : beta;
    for (int e = threadIdx.x; e < T; e += kWideRecThr) {
      int i, j;
      tri_ij(e, i, j);
      cd x = a.Rnn[base + e];
      if (i == j) x.im = 0.0;
      cd yy = cd{0.0, 0.0};
      fma_cc(yy, cdk(ys[i]), cdk(ys[j]));
      x = cx * x;
      x.re = fma(cy, yy.re, x.re);
      x.im = (i == j) ? 0.0 : fma(cy, yy.im, x.im);
      a.Rnn[base + e] = x;
    }
  }
  (void)F;
}

__global__ void __launch_bounds__(64) wide_tail_kernel(const UpdateArgs a, const FamNode* fns, const int* ids, int nW) {
  const int f = blockIdx.x;
  const int s = blockIdx.y / nW;
  const FamNode d = fns[ids[blockIdx.y % nW]];
  if (!node_in(a.nodeMask, d.k)) return;
  const int li = threadIdx.x, D = d.D, F = a.F, r = a.r;
  const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;
  const bool solve = (fl & DANSE_FLAG_SOLVE) != 0 && !pregiven;
  const bool initslot = (fl & DANSE_FLAG_INITSLOT) != 0;
  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotPrev = a.wHistory ? r : (r & 1);
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  const cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  cf acc = cf{0.0f, 0.0f};
  for (int i = li; i < D; i += 64) {
    cf w;
    // a solve's filter was written by wide_filter_kernel; pre-given and
    // init-slot filters are already in the next slot
    if (solve || pregiven || initslot) {
      w = wNext[i];
    } else {
      w = wPrev[i];
      wNext[i] = w;
    }
    acc = acc + cmul(w, load_y(a, d, s, f, i, true));
  }
  cf dh = gsum<64>(acc);
  if (f == 0 || f == F - 1) dh.im = 0.0f;
  if (li == 0) a.dhat[((((long long)d.fam * a.S + s) * a.K + d.k) * a.R + r) * F + f] = dh;
}

}  // namespace danse
