// update / filter kernels for large filter dimensions (16 < D <= 64): one
// frequency bin per wavefront, rows in chunked vector registers
// (solver64.hpp).  Same per-bin work as update_kernel in kernels.hpp:
// SCM update (d_classes.py:2048-2267), filter update (d_classes.py:
// 3320-3387), external filters (d_classes.py:1627-1694), dhat = w^H yhat.
#pragma once
#include "kernels.hpp"
#include "solver64.hpp"

namespace danse {

template <int DMAX, int RMAX>
__global__ void __launch_bounds__(64) update_kernel_big(const UpdateArgs a) {
  using namespace big;
  __shared__ LDS<DMAX> lds;
  const int li = threadIdx.x;
  const int F = a.F;
  const int f = blockIdx.x % F;
  const int t = blockIdx.x / F;
  const int fni = t % a.nFN;
  const int s = t / a.nFN;
  const FamNode d = a.fn[fni];
  const int D = d.D;
  const bool act = li < D;
  const int r = a.r;
  const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  const int opY = fl & 3, opN = (fl >> 2) & 3;
  const bool solve = (fl & DANSE_FLAG_SOLVE) != 0;

  const cf y = load_y(a, d, s, f, li, act);
  const float beta = a.beta[s * a.K + d.k];
  const float invD = 1.0f / (float)D;
  const long long matOff = (long long)s * a.scmStride + d.scmOff + (long long)f * D * D;
  const int rowc = act ? li : 0;

  Row<DMAX> A, B;
  auto load_rows = [&](const cf* P, Row<DMAX>& X) {
    rzero(X);
    cols_below<DMAX>(D, [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const int cl = (c < D) ? c : D - 1;
      const cf v = P[matOff + (long long)rowc * D + cl];
      ws<c>(X, (act && c < D) ? v : cf{0.0f, 0.0f});
    });
  };
  auto store_rows = [&](cf* P, const Row<DMAX>& X) {
    if (act) {
      cols_below<DMAX>(D, [&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if (c < D) P[matOff + (long long)li * D + c] = rs<c>(X);
      });
    }
  };
  auto apply_op = [&](Row<DMAX>& X, int op) {
    cols_below<DMAX>(D, [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const cf yc = rl(y, c);
      const cf yy = invD * mulc(y, yc);   // y = 0 on lanes >= D
      if (op == DANSE_OP_SET) ws<c>(X, yy);
      else ws<c>(X, beta * rs<c>(X) + (1.0f - beta) * yy);
    });
  };
  const bool needY = (opY != 0) || solve;
  const bool needN = (opN != 0) || solve;
  if (needY) load_rows(a.Ryy, A);
  if (needN) load_rows(a.Rnn, B);
  if (opY) {
    apply_op(A, opY);
    store_rows(a.Ryy, A);
  }
  if (opN) {
    apply_op(B, opN);
    store_rows(a.Rnn, B);
  }

  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotPrev = a.wHistory ? r : (r & 1);
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  cf w;
  const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;
  if (pregiven) {
    w = act ? wNext[rowc] : cf{0.0f, 0.0f};
  } else if (solve) {
    bool ok = true;
    if (a.gevd) w = gevd_filter<DMAX, RMAX>(A, B, lds, li, D, a.rank, d.ref, ok);
    else w = mwf_filter<DMAX>(A, B, lds, li, D, d.ref, ok);
    if (!ok && li == 0) atomicOr(&a.diag[(s * a.K + d.k) * kMaxFam + d.fam], 1);
  } else {
    w = act ? wPrev[rowc] : cf{0.0f, 0.0f};
  }
  if (act && !pregiven) wNext[li] = w;
  node_bin_tail(a, d, s, f, li, fl, pregiven, true, w, y, gsum<64>(act ? cmul(w, y) : cf{0.0f, 0.0f}));
}

template <int DMAX, int RMAX>
__global__ void __launch_bounds__(64) filter_update_kernel_big(const cf* Ryy, const cf* Rnn, int B, int D, int gevd,
                                                              int rank, int ref, cf* w, int* diag) {
  using namespace big;
  __shared__ LDS<DMAX> lds;
  const int li = threadIdx.x;
  const int b = blockIdx.x;
  const bool act = li < D;
  const int row = act ? li : 0;
  Row<DMAX> A, Bm;
  rzero(A);
  rzero(Bm);
  cols_below<DMAX>(D, [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    const int cl = (c < D) ? c : D - 1;
    const cf va = Ryy[((long long)b * D + row) * D + cl];
    const cf vn = Rnn[((long long)b * D + row) * D + cl];
    ws<c>(A, (act && c < D) ? va : cf{0.0f, 0.0f});
    ws<c>(Bm, (act && c < D) ? vn : cf{0.0f, 0.0f});
  });
  bool ok = true;
  cf wv;
  if (gevd) wv = gevd_filter<DMAX, RMAX>(A, Bm, lds, li, D, rank, ref, ok);
  else wv = mwf_filter<DMAX>(A, Bm, lds, li, D, ref, ok);
  if (act) w[(long long)b * D + li] = wv;
  if (diag && li == 0) diag[b] = ok ? 0 : 1;
}

}  // namespace danse
