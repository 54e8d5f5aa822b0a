// GEVD update / filter kernels for 16 < D <= 48 on the two-dimensional
// wavefront layout of solver2d.hpp: one frequency bin per wavefront, lane
// (p, q) owns the SCM entries (p + 8 s, q + 8 t).  Same per-bin work as
// update_kernel_big (kernels_big.hpp): SCM update (d_classes.py:2048-2267),
// GEVD filter update (d_classes.py:3343-3387), external filters
// (d_classes.py:1627-1694), dhat = w^H yhat (d_base.py:2075).  The MWF
// filter of these classes stays on update_kernel_big.
//
// Register phases (the float64 block and the float32 Ryy block are never
// live together): Rnn recursion (+ store) -> float64 Cholesky + inverse ->
// Li in float32 -> Ryy recursion (+ store) -> congruence, tridiagonal,
// eigen part, back-transform.
#pragma once
#include "kernels.hpp"

#ifndef DANSE_2D_WPE
#define DANSE_2D_WPE 2
#endif
#include "solver2d.hpp"

namespace danse {

template <int NB, int RMAX>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NB <= 5 ? DANSE_2D_WPE : 1)))
update_kernel_2d(const UpdateArgs a) {
  using namespace t2d;
  __shared__ LDS2<NB> S;
  const int li = threadIdx.x;
  const int p = li >> 3, q = li & 7;
  const int F = a.F;
  const int f = blockIdx.x % F;
  const int tt = blockIdx.x / F;
  const int fni = tt % a.nFN;
  const int s = tt / a.nFN;
  const FamNode d = a.fn[fni];
  const int D = d.D;
  const bool act = li < D;
  const int r = a.r;
  const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  const int opY = fl & 3, opN = (fl >> 2) & 3;
  const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;
  const bool solve = (fl & DANSE_FLAG_SOLVE) != 0 && !pregiven;
  const bool initslot = (fl & DANSE_FLAG_INITSLOT) != 0;
  // factor cache (kernels.hpp li_reusable): per bin the float32 Li blocks in
  // lane order [NB * NB][64] and g [64]
  const bool reuse = solve && li_reusable(a, d, s, opN);
  cf* liC = a.liCache ? a.liCache + (long long)s * a.liStride + d.liOff + (long long)f * (64 * NB * NB + 64) : nullptr;

  const cf y = load_y(a, d, s, f, li, act);
  S.vb[li] = y;
  t2d::wsync();
  cf yr[NB], yc[NB];
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    yr[sb] = S.vb[p + 8 * sb];
    yc[sb] = S.vb[q + 8 * sb];
  });
  t2d::wsync();
  const double beta = a.beta[s * a.K + d.k];
  const long long matOff = (long long)s * a.scmStride + d.scmOff + (long long)f * D * D;

  // ---- Rnn (float64): recursion, store, factor --------------------------
  Blk<NB> Lf;
  bool ok = true;
  if (opN || (solve && !reuse)) {
    BlkD<NB> M;
    const double cy = (opN == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (opN == DANSE_OP_SET) ? 0.0 : beta;
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p + 8 * sb, c = q + 8 * tb;
        const bool in = i < D && c < D;
        cd x = csel(in, a.Rnn[matOff + (in ? (long long)i * D + c : 0ll)], cd{0.0, 0.0});
        if (opN) {
          cd yy = cd{0.0, 0.0};
          fma_cc(yy, cdk(yr[sb]), cdk(yc[tb]));
          x = cx * x;
          x.re = fma(cy, yy.re, x.re);
          x.im = fma(cy, yy.im, x.im);
          if (in) a.Rnn[matOff + (long long)i * D + c] = x;
        }
        M.v[sb][tb] = x;
      });
    });
    if (solve && !reuse) {
      ok = gevd2d_factor<NB>(M, Lf, S, li, D, d.ref);
      if (liC) {
        sfor<0, NB>([&](auto sc) {
          sfor<0, NB>([&](auto tc) {
            constexpr int sb = decltype(sc)::value, tb = decltype(tc)::value;
            liC[(sb * NB + tb) * 64 + li] = Lf.v[sb][tb];
          });
        });
        liC[64 * NB * NB + li] = S.g[li];
      }
    }
  }
  if (reuse) {
    sfor<0, NB>([&](auto sc) {
      sfor<0, NB>([&](auto tc) {
        constexpr int sb = decltype(sc)::value, tb = decltype(tc)::value;
        Lf.v[sb][tb] = liC[(sb * NB + tb) * 64 + li];
      });
    });
    S.g[li] = liC[64 * NB * NB + li];
    t2d::wsync();
  }

  // ---- Ryy (float32): recursion, store, filter ---------------------------
  cf w = cf{0.0f, 0.0f};
  if (opY || solve) {
    Blk<NB> A;
    const float by = (float)beta, cy = (opY == DANSE_OP_SET) ? (float)(1.0 / D) : (float)((1.0 - beta) / D);
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p + 8 * sb, c = q + 8 * tb;
        const bool in = i < D && c < D;
        cf x = csel(in, a.Ryy[matOff + (in ? (long long)i * D + c : 0ll)], cf{0.0f, 0.0f});
        if (opY) {
          const cf yy = cy * mulc(yr[sb], yc[tb]);
          x = csel(opY == DANSE_OP_SET, yy, by * x + yy);
          if (in) a.Ryy[matOff + (long long)i * D + c] = x;
        }
        A.v[sb][tb] = x;
      });
    });
    if (solve) w = gevd2d_filter<NB, RMAX>(A, Lf, S, li, D, a.rank);
  }

  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotPrev = a.wHistory ? r : (r & 1);
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  const int rowc = act ? li : 0;
  if (pregiven || initslot) {
    w = csel(act, wNext[rowc], cf{0.0f, 0.0f});
  } else if (solve) {
    if (!ok && li == 0) atomicOr(&a.diag[(s * a.K + d.k) * kMaxFam + d.fam], 1);
  } else {
    w = csel(act, wPrev[rowc], cf{0.0f, 0.0f});
  }
  if (act && !pregiven && !initslot) wNext[li] = w;
  node_bin_tail(a, d, s, f, li, fl, pregiven, true, w, y, gsum<64>(csel(act, cmul(w, y), cf{0.0f, 0.0f})));
}

// Stand-alone GEVD filter update (danse_filter_update): float64 SCM pairs
// [B][D][D], one bin per wavefront.
template <int NB, int RMAX>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NB <= 5 ? DANSE_2D_WPE : 1)))
filter_update_kernel_2d(const cd* Ryy, const cd* Rnn, int B, int D, int rank, int ref, cf* w, int* diag) {
  using namespace t2d;
  __shared__ LDS2<NB> S;
  const int li = threadIdx.x;
  const int p = li >> 3, q = li & 7;
  const int b = blockIdx.x;
  Blk<NB> Lf;
  bool ok;
  {
    BlkD<NB> M;
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p + 8 * sb, c = q + 8 * tb;
        const bool in = i < D && c < D;
        M.v[sb][tb] = csel(in, Rnn[(long long)b * D * D + (in ? i * D + c : 0)], cd{0.0, 0.0});
      });
    });
    ok = gevd2d_factor<NB>(M, Lf, S, li, D, ref);
  }
  Blk<NB> A;
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    sfor<0, NB>([&](auto tc) {
      constexpr int tb = decltype(tc)::value;
      const int i = p + 8 * sb, c = q + 8 * tb;
      const bool in = i < D && c < D;
      A.v[sb][tb] = csel(in, cfk(Ryy[(long long)b * D * D + (in ? i * D + c : 0)]), cf{0.0f, 0.0f});
    });
  });
  const cf wv = gevd2d_filter<NB, RMAX>(A, Lf, S, li, D, rank);
  if (li < D) w[(long long)b * D + li] = wv;
  if (diag && li == 0) diag[b] = ok ? 0 : 1;
}

}  // namespace danse
