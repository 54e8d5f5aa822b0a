// update / filter kernels for large filter dimensions (16 < D <= 64): one
// frequency bin per wavefront, rows in chunked vector registers.  Since the
// two-dimensional layout (kernels_2d.hpp) took over the GEVD of D <= 48,
// these serve the MWF filter of every large class and the GEVD of D > 48
// (solver64m.hpp: Rnn in float64, mixed-precision filter update).  Same per-bin work as update_kernel in kernels.hpp:
// SCM update (d_classes.py:2048-2267), filter update (d_classes.py:
// 3320-3387), external filters (d_classes.py:1627-1694), dhat = w^H yhat.
#pragma once
#include "kernels.hpp"
#include "solver64m.hpp"

namespace danse {

template <int DMAX, int RMAX, bool GEVD>
__global__ void __launch_bounds__(64) update_kernel_big(const UpdateArgs a) {
  using namespace big;
  __shared__ LDSM<DMAX> lds;
  const int li = threadIdx.x;
  const int F = a.F;
  const int f = blockIdx.x % F;
  const int t = blockIdx.x / F;
  const int fni = t % a.nFN;
  const int s = t / a.nFN;
  const FamNode d = a.fn[fni];
  if (!node_in(a.nodeMask, d.k)) return;   // one bin per wave
  const int D = d.D;
  const bool act = li < D;
  const int r = a.r;
  const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  // noRec: a prefix round (span.hpp) -- its recursion is deferred to
  // span_rec_kernel, this launch runs the tail only (no item solves there)
  const int opY = a.noRec ? 0 : (fl & 3), opN = a.noRec ? 0 : ((fl >> 2) & 3);
  const bool solve = (fl & DANSE_FLAG_SOLVE) != 0;

  const cf y = load_y(a, d, s, f, li, act);
  const double beta = a.beta[s * a.K + d.k];
  // SCMs: packed lower triangles, bin-major (FamNode.packed 2): row li's
  // entry c is (li, c) for c <= li, conj((c, li)) above the diagonal
  const long long triOff = (long long)s * a.scmStride + d.scmOff + (long long)f * (D * (D + 1) / 2);
  const int rowc = act ? li : 0;
  auto ent = [&](int c) -> long long {
    return triOff + (c <= rowc ? rowc * (rowc + 1) / 2 + c : c * (c + 1) / 2 + rowc);
  };

  // Ryy row in float32; Rnn row in float64
  Row<DMAX> A;
  RowD<DMAX> B;
  const bool needY = (opY != 0) || solve;
  const bool needN = (opN != 0) || solve;
  if (needY) {
    rzero(A);
    cols_below<DMAX>(D, [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const int cl = (c < D) ? c : D - 1;
      cf v = a.Ryy[ent(cl)];
      if (cl > rowc) v = conjg(v);
      if (cl == rowc) v.im = 0.0f;
      ws<c>(A, (act && c < D) ? v : cf{0.0f, 0.0f});
    });
  }
  if (opY) {
    const float by = (float)beta, cy = (opY == DANSE_OP_SET) ? (float)(1.0 / D) : (float)((1.0 - beta) / D);
    cols_below<DMAX>(D, [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const cf yy = cy * mulc(y, rl(y, c));   // y = 0 on lanes >= D
      cf x = (opY == DANSE_OP_SET) ? yy : by * rs<c>(A) + yy;
      if (c == li) x.im = 0.0f;
      ws<c>(A, x);
    });
    if (act) {
      cols_below<DMAX>(D, [&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if (c <= li) a.Ryy[ent(c)] = rs<c>(A);
      });
    }
  }
  if (needN) {
    sfor<0, DMAX>([&](auto cc) { wsd<decltype(cc)::value>(B, cd{0.0, 0.0}); });
    const double cy = (opN == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (opN == DANSE_OP_SET) ? 0.0 : beta;
    const cd yl = cdk(y);
    cols_below<DMAX>(D, [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const int cl = (c < D) ? c : D - 1;
      cd x = a.Rnn[ent(cl)];
      if (cl > rowc) x = conjg(x);
      if (cl == rowc) x.im = 0.0;
      if (!(act && c < D)) x = cd{0.0, 0.0};
      if (opN) {
        cd yy = cd{0.0, 0.0};
        fma_cc(yy, yl, cdk(rl(y, c)));
        x = cx * x;
        x.re = fma(cy, yy.re, x.re);
        x.im = (c == li) ? 0.0 : fma(cy, yy.im, x.im);
        if (act && c <= li) a.Rnn[ent(c)] = x;
      }
      wsd<c>(B, x);
    });
  }

  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotPrev = a.wHistory ? r : (r & 1);
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  cf w = cf{0.0f, 0.0f};
  const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;
  const bool initslot = (fl & DANSE_FLAG_INITSLOT) != 0;
  if (pregiven || initslot) {
    w = csel(act, wNext[rowc], cf{0.0f, 0.0f});
  } else if (solve) {
    bool ok = true;
    if constexpr (GEVD) w = gevd_filter_mixed<DMAX, RMAX>(A, B, lds, li, D, a.rank, d.ref, ok);
    else w = mwf_filter_mixed<DMAX>(A, rgetd(B, d.ref), lds, li, D, d.ref, ok);
    if (!ok && li == 0) atomicOr(&a.diag[(s * a.K + d.k) * kMaxFam + d.fam], 1);
  } else {
    w = act ? wPrev[rowc] : cf{0.0f, 0.0f};
  }
  if (act && !pregiven && !initslot) wNext[li] = w;
  node_bin_tail(a, d, s, f, li, fl, pregiven, true, w, y, gsum<64>(act ? cmul(w, y) : cf{0.0f, 0.0f}));
}

template <int DMAX, int RMAX, bool GEVD>
__global__ void __launch_bounds__(64) filter_update_kernel_big(const cd* Ryy, const cd* Rnn, int B, int D, int gevd,
                                                              int rank, int ref, cf* w, int* diag) {
  using namespace big;
  __shared__ LDSM<DMAX> lds;
  const int li = threadIdx.x;
  const int b = blockIdx.x;
  const bool act = li < D;
  const int row = act ? li : 0;
  RowD<DMAX> Y, N;
  sfor<0, DMAX>([&](auto cc) {
    wsd<decltype(cc)::value>(Y, cd{0.0, 0.0});
    wsd<decltype(cc)::value>(N, cd{0.0, 0.0});
  });
  cols_below<DMAX>(D, [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    const int cl = (c < D) ? c : D - 1;
    const cd va = Ryy[((long long)b * D + row) * D + cl];
    const cd vn = Rnn[((long long)b * D + row) * D + cl];
    wsd<c>(Y, (act && c < D) ? va : cd{0.0, 0.0});
    wsd<c>(N, (act && c < D) ? vn : cd{0.0, 0.0});
  });
  bool ok = true;
  cf wv;
  (void)gevd;
  if constexpr (GEVD) {
    Row<DMAX> A;
    sfor<0, DMAX>([&](auto cc) { ws<decltype(cc)::value>(A, cfk(rsd<decltype(cc)::value>(Y))); });
    wv = gevd_filter_mixed<DMAX, RMAX>(A, N, lds, li, D, rank, ref, ok);
  } else {
    wv = mwf_filter64<DMAX>(Y, rgetd(N, ref), lds, li, D, ref, ok);
  }
  if (act) w[(long long)b * D + li] = wv;
  if (diag && li == 0) diag[b] = ok ? 0 : 1;
}

}  // namespace danse
