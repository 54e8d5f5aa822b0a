// update / filter kernels for small filter dimensions (D <= kLaneMaxD):
// one (scene, family-node, bin) per LANE (solver1.hpp).  Same per-bin work as
// update_kernel in kernels.hpp -- SCM update (d_classes.py:2048-2267), filter
// update (d_classes.py:3320-3387), external filters (d_classes.py:1627-1694),
// dhat = w^H yhat (d_base.py:2075) -- with the SCMs of this class stored as
// packed lower triangles, bin-minor ([D(D+1)/2][F] per family-node), so a
// wave's 64 lanes read and write every SCM entry as one coalesced 512-byte
// access.
#pragma once
#include "kernels.hpp"
#include "solver1.hpp"

namespace danse {

template <int D, int RMAX, bool GEVD>
__global__ void __launch_bounds__(64) update_kernel_lane(const UpdateArgs a) {
  using namespace lane;
  constexpr int NT = tri_n(D);
  const int F = a.F;
  const long long total = (long long)a.S * a.nFN * F;
  long long gid = (long long)blockIdx.x * 64 + threadIdx.x;
  const bool valid = gid < total;
  if (!valid) gid = total - 1;
  const int f = (int)(gid % F);
  const long long t = gid / F;
  const int fni = (int)(t % a.nFN);
  const int s = (int)(t / a.nFN);
  const FamNode d = a.fn[fni];
  const int r = a.r;
  const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  const int opY = fl & 3, opN = (fl >> 2) & 3;
  const bool solve = (fl & DANSE_FLAG_SOLVE) != 0;
  const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;

  cf y[D];
  if (opY || opN) {
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      y[i] = load_y(a, d, s, f, i, true);
    });
  }
  const float beta = a.beta[s * a.K + d.k];
  const float invD = 1.0f / (float)D;
  const long long base = (long long)s * a.scmStride + d.scmOff + f;

  // Rnn first, then Ryy, so that at most one triangle plus the Cholesky
  // factor's LDS copy is live: the GEVD keeps L in LDS, the MWF only the
  // column Rnn[:, ref].
  __shared__ cf Ls[(D * (D - 1) / 2 > 0) ? D * (D - 1) / 2 : 1][64];
  const int lane_ = threadIdx.x;
  PTri<D> X;
  auto load = [&](const cf* Pm) {
    sfor<0, NT>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      X.a[e] = Pm[base + (long long)e * F];
    });
  };
  auto store = [&](cf* Pm) {
    if (valid) {
      sfor<0, NT>([&](auto ec) {
        constexpr int e = decltype(ec)::value;
        Pm[base + (long long)e * F] = X.a[e];
      });
    }
  };
  // X <- yy^H (first-frame basis) or beta X + (1 - beta) yy^H, yy^H = y y^H / D
  auto apply = [&](int op) {
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      sfor<0, i + 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const cf yy = invD * mulc(y[i], y[j]);
        X.a[P(i, j)] = (op == DANSE_OP_SET) ? yy : beta * X.a[P(i, j)] + (1.0f - beta) * yy;
      });
    });
  };
  const bool gsolve = solve && GEVD;
  bool ok = true;
  float invd[D], ldiag[D];
  cf ncol[D];
  if (opN || solve) {
    load(a.Rnn);
    if (opN) {
      apply(opN);
      store(a.Rnn);
    }
    if (gsolve) {
      ok = chol<D>(X, invd);
      to_lds<D>(X, Ls, lane_, ldiag);
    } else if (solve) {
      herm_col<D>(X, d.ref, ncol);
    }
  }
  if (opY || solve) {
    load(a.Ryy);
    if (opY) {
      apply(opY);
      store(a.Ryy);
    }
  }

  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotPrev = a.wHistory ? r : (r & 1);
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  cf w[D];
  if (pregiven) {
    sfor<0, D>([&](auto ic) { w[decltype(ic)::value] = wNext[decltype(ic)::value]; });
  } else if (solve) {
    if constexpr (GEVD) gevd_filter<D, RMAX>(X, LTri<D>{Ls, lane_}, invd, ldiag, a.rank, d.ref, w);
    else ok = mwf_filter<D>(X, ncol, d.ref, w);
    if (!ok && valid) atomicOr(&a.diag[(s * a.K + d.k) * kMaxFam + d.fam], 1);
  } else {
    sfor<0, D>([&](auto ic) { w[decltype(ic)::value] = wPrev[decltype(ic)::value]; });
  }
  if (valid && !pregiven) {
    sfor<0, D>([&](auto ic) { wNext[decltype(ic)::value] = w[decltype(ic)::value]; });
  }

  // external filters (DANSE family), d_classes.py:1627-1694
  if (d.extMode >= 0 && !pregiven && valid) {
    const int M = d.M;
    const long long eb = (long long)s * a.wExtStride + d.wExtOff;
    const int eP = a.wExtHistory ? r : (r & 1);
    const int eN = a.wExtHistory ? r + 1 : ((r + 1) & 1);
    cf* eprev = a.wExtHist + eb + ((long long)eP * F + f) * M;
    cf* enext = a.wExtHist + eb + ((long long)eN * F + f) * M;
    cf* tgt = a.wExtTarget + (long long)s * a.tgtStride + d.tgtOff + (long long)f * M;
    const float be = a.betaExt[s * a.K + d.k];
    sfor<0, D>([&](auto ic) {
      constexpr int m = decltype(ic)::value;
      if (m < M) {
        cf ne;
        if (d.extMode == 0) ne = w[m];
        else if (d.extMode == 2) ne = eprev[m];
        else if (d.extMode == 3) ne = cf{(m == d.ref) ? 1.0f : 0.0f, 0.0f};
        else {
          const cf tg = tgt[m];
          ne = be * eprev[m] + (1.0f - be) * tg;
          if (fl & DANSE_FLAG_EXT_TARGET) tgt[m] = (1.0f - a.alphaExt) * tg + a.alphaExt * w[m];
        }
        enext[m] = ne;
      }
    });
  }
  // dhat = w^H yhat, DC / Nyquist forced real (quirk Q7); yhat re-read (L2)
  // rather than held in registers across the solve
  cf dh = cf{0.0f, 0.0f};
  sfor<0, D>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    dh = dh + cmul(w[i], load_y(a, d, s, f, i, true));
  });
  if (f == 0 || f == F - 1) dh.im = 0.0f;
  if (valid) a.dhat[((((long long)d.fam * a.S + s) * a.K + d.k) * a.R + r) * F + f] = dh;
}

// Stand-alone batched filter update (danse_filter_update) on full [B][D][D]
// SCM pairs: one batch item per lane.
template <int D, int RMAX>
__global__ void __launch_bounds__(64) filter_update_kernel_lane(const cf* Ryy, const cf* Rnn, int Bn, int gevd,
                                                               int rank, int ref, cf* w, int* diag) {
  using namespace lane;
  int b = blockIdx.x * 64 + threadIdx.x;
  const bool valid = b < Bn;
  if (!valid) b = Bn - 1;
  __shared__ cf Ls[(D * (D - 1) / 2 > 0) ? D * (D - 1) / 2 : 1][64];
  const int lane_ = threadIdx.x;
  PTri<D> X;
  auto load = [&](const cf* M) {
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      sfor<0, i + 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        X.a[P(i, j)] = M[((long long)b * D + i) * D + j];
      });
    });
  };
  cf wv[D];
  bool ok = true;
  load(Rnn);
  if (gevd) {
    float invd[D], ldiag[D];
    ok = chol<D>(X, invd);
    to_lds<D>(X, Ls, lane_, ldiag);
    load(Ryy);
    gevd_filter<D, RMAX>(X, LTri<D>{Ls, lane_}, invd, ldiag, rank, ref, wv);
  } else {
    cf ncol[D];
    herm_col<D>(X, ref, ncol);
    load(Ryy);
    ok = mwf_filter<D>(X, ncol, ref, wv);
  }
  if (valid) {
    sfor<0, D>([&](auto ic) { w[(long long)b * D + decltype(ic)::value] = wv[decltype(ic)::value]; });
    if (diag) diag[b] = ok ? 0 : 1;
  }
}

}  // namespace danse
