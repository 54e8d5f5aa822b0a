// update / filter kernels for small filter dimensions (D <= kLaneMaxD):
// one (scene, family-node, bin) per LANE (solver_mixed.hpp).  Same per-bin
// work as update_kernel in kernels.hpp -- SCM update (d_classes.py:
// 2048-2267), filter update (d_classes.py:3320-3387), external filters
// (d_classes.py:1627-1694), dhat = w^H yhat (d_base.py:2075) -- with the
// SCMs of this class stored as packed lower triangles, bin-minor
// ([D(D+1)/2][F] per family-node), so a wave's 64 lanes read and write
// every SCM entry as one coalesced access (512 B for the float32 Ryy, 1 KiB
// for the float64 Rnn).
//
// Per lane, in two phases that never hold their big arrays at once:
//   1. SCM recursion (Ryy float32 or Rnn float64, as the VAD selects); on
//      solve frames the float64 Cholesky + inverse of Rnn, handed to phase 2
//      through LDS as the float32 Li = L^-1 and g = L^H e_ref ([entry][lane],
//      39 KiB per wave at D = 11) -- or, when Rnn is unchanged since the
//      last factorisation, that record from the factor cache (below);
//      MWF solves completely here, in float64;
//   2. Ryy's recursion, C = Li Ryy Li^H, eigen part, w, external filters
//      (their loads issued ahead of the solve), dhat (from the observation
//      vector kept since phase 1).
// (No SLP packing in these classes -- build.py -- and no runtime rank test
// for r = 0 in gevd_eig: either one doubles the register footprint.)
#pragma once
#include "kernels.hpp"
#include "solver_mixed.hpp"

namespace danse {

// The float32 factor record of a lane class (Li entries 0..NT-1, g entries
// NT..NT+D-1) is cached in wave order, UpdateArgs.liLane: block b's record
// is [entry][64 lanes] contiguous, exactly the LDS array the solve reads, so
// it reaches LDS by LDS-DMA in 1 KiB pieces (global_load_lds_dwordx4, lane l
// carrying bytes 16 l .. 16 l + 15 of a piece: two bins' entries), issued
// right behind the Ryy loads.  A piece carries other lanes' bins, so the DMA
// runs only in waves whose every lane takes the cached factor (the whole
// wave in the branch); other waves copy their record through registers.
namespace lane {
constexpr int lr_rows(int D) { return (tri_n(D) + D + 1) & ~1; }   // whole pieces
template <int D>
DANSE_DEV void li_dma_lane(cf (*Lr)[64], const cf* rec) {
  const char* src = reinterpret_cast<const char*>(rec) + 16 * threadIdx.x;
  char* dst = reinterpret_cast<char*>(&Lr[0][0]);
  sfor<0, lr_rows(D) / 2>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + 1024 * j),
                                     (__attribute__((address_space(3))) void*)(dst + 1024 * j), 16, 0, 0);
  });
}
}  // namespace lane

struct LaneIdx {
  int f, s, fni;
  bool valid;
};
DANSE_DEV LaneIdx lane_index(const UpdateArgs& a) {
  const long long total = (long long)a.S * a.nFN * a.F;
  long long gid = (long long)blockIdx.x * 64 + threadIdx.x;
  LaneIdx x;
  x.valid = gid < total;
  if (!x.valid) gid = total - 1;
  x.f = (int)(gid % a.F);
  const long long t = gid / a.F;
  x.fni = (int)(t % a.nFN);
  x.s = (int)(t / a.nFN);
  return x;
}

// RO: the recursion-only variant for rounds in which no item of the launch
// solves (UpdateArgs.noSolve): the SCM entries are updated one at a time, so
// the launch runs at the occupancy of a streaming kernel instead of the
// solver's one wave per SIMD
template <int D, int RMAX, bool GEVD, bool RO = false>
__global__ void __launch_bounds__(64) update_kernel_lane(const UpdateArgs a) {
  using namespace lane;
  constexpr int NT = tri_n(D);
  // DANSE_STAMP builds (kernels_2d.hpp): per-wave phase clocks
  unsigned long long tsv[kStampN];
  auto stamp = [&](int i) {
    if constexpr (DANSE_STAMP) tsv[i] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  const LaneIdx ix = lane_index(a);
  const int F = a.F, f = ix.f, s = ix.s, r = a.r;
  const FamNode d = a.fn[ix.fni];
  // (lanes of nodes outside the launch's node mask compute and store nothing)
  const bool valid = ix.valid && node_in(a.nodeMask, d.k);
  const long long flIdx = (((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k;
  const uint8_t fl = a.flags[flIdx];
  // (the previous round's flags in the same round trip: li_reusable's first step)
  const uint8_t flPrev = a.flags[r > 0 ? flIdx - (long long)a.S * kMaxFam * a.K : flIdx];
  const int opY = fl & 3, opN = (fl >> 2) & 3;
  const bool solve = !RO && (fl & DANSE_FLAG_SOLVE) != 0 && (fl & DANSE_FLAG_PREGIVEN) == 0;
  if (a.splitSolve && solve) return;   // this item's round runs on update_kernel_2d<.., PK = true>
  // GEVD: reuse the cached float32 Li / g when Rnn has not changed since the
  // last factorisation (skips the float64 load, Cholesky and inverse)
  const bool reuse = GEVD && solve && a.liLane && li_reusable_prev(a, d, s, opN, flPrev);
  // this block's record in the wave-ordered cache, this lane's column
  cf* const liRec = a.liLane ? a.liLane + (long long)blockIdx.x * lr_rows(D) * 64 : nullptr;
  cf* const liC = liRec ? liRec + threadIdx.x : nullptr;
  // the float32 factor record: Li (entries 0..NT-1) and g (NT..NT+D-1)
  __shared__ __attribute__((aligned(16))) cf Lr[lr_rows(D)][64];
  cf (*const Ls)[64] = Lr;
  cf (*const Gs)[64] = Lr + NT;
  const bool dma = GEVD && !RO && __any(reuse) && !__any(!reuse);   // (every lane: __all, spelled so that it allocates without spills)

  // the observation vector: the recursion's and, kept in registers, dhat's
  cf y[D];
  if (!RO || ((opY || opN) && !a.noRec)) {
    load_y_all<D>(a, d, s, f, y);
  }
  stamp(1);
  const double beta = a.beta[s * a.K + d.k];
  const long long base = (long long)s * a.scmStride + d.scmOff + f;
  // Ryy (float32) of this frame into A: load, the recursion when the VAD
  // selects it, store
  // (dma: the factor record's DMA, issued right behind these loads, so that
  // the two share one round trip; waited for after the recursion, before the
  // stores join the count)
  auto ryy_update = [&](PTri<D>& A, bool dma = false) {
    sfor<0, NT>([&](auto ec) { A.a[decltype(ec)::value] = a.Ryy[base + (long long)decltype(ec)::value * F]; });
    if (dma) {
      asm volatile("" ::: "memory");
      li_dma_lane<D>(Lr, liRec);
      hold(A.a);
    }
    if (opY) {
      const float by = (float)beta, cy = (opY == DANSE_OP_SET) ? (float)(1.0 / D) : (float)((1.0 - beta) / D);
      sfor<0, D>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        sfor<0, i + 1>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const cf yy = cy * mulc(y[i], y[j]);
          A.a[P(i, j)] = csel(opY == DANSE_OP_SET, yy, by * A.a[P(i, j)] + yy);
          if constexpr (i == j) A.a[P(i, j)].im = 0.0f;
        });
      });
      if (dma) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the record has landed
      if (valid) {
        sfor<0, NT>([&](auto ec) { a.Ryy[base + (long long)decltype(ec)::value * F] = A.a[decltype(ec)::value]; });
      }
    } else if (dma) {
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
  };

  // ---- SCM recursion (the VAD selects one of Ryy / Rnn per frame):
  // SCM <- yy^H (first-frame basis) or beta SCM + (1 - beta) yy^H, yy^H = y y^H / D.
  // Rnn (float64) first, with the factor of a solve; then Ryy, which a solve
  // uses straight from the registers it was updated in (one Ryy read per
  // frame: the recursion, the store and the congruence share it)
  if constexpr (RO) {
    // one entry at a time (loads, recursion, store): no triangle is held
    // (noRec: the prefix's recursion is deferred to span_rec_kernel)
    if ((opY || opN) && !a.noRec) {
      const bool isY = opY != 0;
      const int op = isY ? opY : opN;
      const double cy = (op == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
      const double cx = (op == DANSE_OP_SET) ? 0.0 : beta;
      // row by row: the row's entries loaded first (one round trip per
      // row, hold()), then the recursion and the stores
      sfor<0, D>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if (isY) {
          cf old[i + 1];
          sfor<0, i + 1>([&](auto jc) { old[decltype(jc)::value] = a.Ryy[base + (long long)P(i, decltype(jc)::value) * F]; });
          hold(old);
          sfor<0, i + 1>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            const cf yy = (float)cy * mulc(y[i], y[j]);
            cf x = csel(op == DANSE_OP_SET, yy, (float)beta * old[j] + yy);
            if constexpr (i == j) x.im = 0.0f;
            if (valid) a.Ryy[base + (long long)P(i, j) * F] = x;
          });
        } else {
          cd old[i + 1];
          sfor<0, i + 1>([&](auto jc) { old[decltype(jc)::value] = a.Rnn[base + (long long)P(i, decltype(jc)::value) * F]; });
          hold(old);
          sfor<0, i + 1>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            cd yy = cd{0.0, 0.0};
            fma_cc(yy, cdk(y[i]), cdk(y[j]));
            cd x = cx * old[j];
            if constexpr (i == j) x.im = 0.0;
            x.re = fma(cy, yy.re, x.re);
            x.im = (i == j) ? 0.0 : fma(cy, yy.im, x.im);
            if (valid) a.Rnn[base + (long long)P(i, j) * F] = x;
          });
        }
      });
    }
  }
  PTriD<D> N;
  if (!RO && (opN || (solve && !reuse))) {
    sfor<0, NT>([&](auto ec) { N.a[decltype(ec)::value] = a.Rnn[base + (long long)decltype(ec)::value * F]; });
    sfor<0, D>([&](auto ic) { N.a[P(decltype(ic)::value, decltype(ic)::value)].im = 0.0; });
  }
  if (!RO && opN) {
    const double cy = (opN == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (opN == DANSE_OP_SET) ? 0.0 : beta;
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const cd yi = cdk(y[i]);
      sfor<0, i + 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        cd yy = cd{0.0, 0.0};
        fma_cc(yy, yi, cdk(y[j]));
        cd x = cx * N.a[P(i, j)];
        x.re = fma(cy, yy.re, x.re);
        x.im = (i == j) ? 0.0 : fma(cy, yy.im, x.im);
        N.a[P(i, j)] = x;
      });
    });
    if (valid) {
      sfor<0, NT>([&](auto ec) { a.Rnn[base + (long long)decltype(ec)::value * F] = N.a[decltype(ec)::value]; });
    }
  }
  stamp(2);
  bool ok = true;
  if (solve) {
  if constexpr (GEVD) {
    asm volatile("" ::: "memory");   // (the float64 triangle is dead before the float32 work below)
    if (reuse && !dma) {
      sfor<0, NT + D>([&](auto ec) { Lr[decltype(ec)::value][threadIdx.x] = liC[decltype(ec)::value * 64]; });
    } else if (!reuse) {
      // float64 Cholesky + inverse of Rnn; hand-over in float32 (LDS, and
      // the factor cache for later solves on the same Rnn)
      double invd[D];
      ok = chol64<D>(N, invd);
      {
        cf g[D];   // out of the registers before the inverse
        ref_row<D>(N, d.ref, g);
        sfor<0, D>([&](auto ic) { Gs[decltype(ic)::value][threadIdx.x] = g[decltype(ic)::value]; });
        if (liC && valid) sfor<0, D>([&](auto ic) { liC[(NT + decltype(ic)::value) * 64] = g[decltype(ic)::value]; });
      }
      asm volatile("" ::: "memory");
      tri_inv64<D>(N, invd);
      store_tri<D>(N, Ls, threadIdx.x);
      if (liC && valid) {
        sfor<0, NT>([&](auto ec) { liC[decltype(ec)::value * 64] = cfk(N.a[decltype(ec)::value]); });
      }
    }
  } else {
    // MWF, float64 throughout: w = Ryy^-1 (Ryy - Rnn) e_ref
    cd ncol[D];
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      cd c = cd{0.0, 0.0};
      sfor<0, D>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k == d.ref) c = hermd<i, k>(N);
      });
      ncol[i] = c;
    });
    asm volatile("" ::: "memory");
    PTri<D> A;
    ryy_update(A);
    cf w[D];
    ok = mwf_filter_mixed<D>(A, ncol, d.ref, w);
    const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
    cf* wNext = a.wHist + (long long)s * a.wStride + d.wOff + ((long long)slotNext * F + f) * D;
    if (valid) sfor<0, D>([&](auto ic) { wNext[decltype(ic)::value] = w[decltype(ic)::value]; });
  }
  if (!ok && valid) atomicOr(&a.diag[(s * a.K + d.k) * kMaxFam + d.fam], 1);
  }
  stamp(3);
  if (!RO && !solve && opY) {   // (a solve updates Ryy where it uses it)
    PTri<D> A;
    ryy_update(A);
  }
  asm volatile("" ::: "memory");
  const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;
  const bool solveT = !RO && (fl & DANSE_FLAG_SOLVE) != 0;   // (RO: pre-given histories only)
  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotPrev = a.wHistory ? r : (r & 1);
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  // the tail's external-filter loads (previous entries and targets, d_classes.py:
  // 1627-1694), issued here so that they share the Ryy loads' round trip
  // instead of taking one of their own after the solve: clamped indices, this
  // lane's filter history standing in for a lane without a tail
  const bool extOn = d.extMode >= 0 && !pregiven && valid;
  const int eP = a.wExtHistory ? r : (r & 1);
  const int eN = a.wExtHistory ? r + 1 : ((r + 1) & 1);
  const long long eb = (long long)s * a.wExtStride + d.wExtOff;
  cf ep[D], tq[D];
  if constexpr (!RO) {
    const int Mx = extOn ? d.M : D;
    const cf* epSrc = extOn ? a.wExtHist + eb + ((long long)eP * F + f) * d.M : wPrev;
    const cf* tqSrc = (extOn && a.wExtTarget) ? a.wExtTarget + (long long)s * a.tgtStride + d.tgtOff + (long long)f * d.M
                                              : wPrev;
#pragma unroll
    for (int m = 0; m < D; ++m) ep[m] = epSrc[min(m, Mx - 1)], tq[m] = tqSrc[min(m, Mx - 1)];
    if (!a.wExtTarget) {
#pragma unroll
      for (int m = 0; m < D; ++m) tq[m] = cf{0.0f, 0.0f};
    }
  }
  cf w[D];
  if (pregiven || (solveT && !GEVD)) {
    // pre-given history, or the MWF filter scm_factor_kernel_lane solved
    sfor<0, D>([&](auto ic) { w[decltype(ic)::value] = wNext[decltype(ic)::value]; });
  } else if (solveT) {
    if constexpr (GEVD) {
      const LdsTri<D> Li{Ls, (int)threadIdx.x};
      PTri<D> A;
      ryy_update(A, dma);
      cf g[D];
      sfor<0, D>([&](auto ic) { g[decltype(ic)::value] = Gs[decltype(ic)::value][threadIdx.x]; });
      stamp(4);
      congruence<D>(A, Li);
      stamp(5);
      gevd_filter_mixed<D, RMAX>(A, Li, g, a.rank, w);
      stamp(6);
    }
    if (valid) sfor<0, D>([&](auto ic) { wNext[decltype(ic)::value] = w[decltype(ic)::value]; });
  } else if (fl & DANSE_FLAG_INITSLOT) {
    sfor<0, D>([&](auto ic) { w[decltype(ic)::value] = wNext[decltype(ic)::value]; });
  } else {
    sfor<0, D>([&](auto ic) { w[decltype(ic)::value] = wPrev[decltype(ic)::value]; });
    if (valid) sfor<0, D>([&](auto ic) { wNext[decltype(ic)::value] = w[decltype(ic)::value]; });
  }
  asm volatile("" ::: "memory");

  // external filters (DANSE family), d_classes.py:1627-1694
  if (extOn) {
    const int M = d.M;
    cf* enext = a.wExtHist + eb + ((long long)eN * F + f) * M;
    cf* tgt = a.wExtTarget + (long long)s * a.tgtStride + d.tgtOff + (long long)f * M;
    const float be = a.betaExt[s * a.K + d.k];
    if constexpr (RO) {
      // the previous entries and targets first (clamped, hold())
      const cf* eprev = a.wExtHist + eb + ((long long)eP * F + f) * M;
#pragma unroll
      for (int m = 0; m < D; ++m) ep[m] = eprev[min(m, M - 1)], tq[m] = cf{0.0f, 0.0f};
      if (a.wExtTarget) {
#pragma unroll
        for (int m = 0; m < D; ++m) tq[m] = tgt[min(m, M - 1)];
      }
      hold(ep);
      hold(tq);
    }
    sfor<0, D>([&](auto ic) {
      constexpr int m = decltype(ic)::value;
      if (m < M) {
        cf ne;
        if (d.extMode == 0) ne = w[m];
        else if (d.extMode == 2) ne = ep[m];
        else if (d.extMode == 3) ne = cf{(m == d.ref) ? 1.0f : 0.0f, 0.0f};
        else {
          const cf tg = tq[m];
          ne = be * ep[m] + (1.0f - be) * tg;
          if (fl & DANSE_FLAG_EXT_TARGET) tgt[m] = (1.0f - a.alphaExt) * tg + a.alphaExt * w[m];
        }
        enext[m] = ne;
      }
    });
  }
  // dhat = w^H yhat, DC / Nyquist forced real (quirk Q7)
  cf dh = cf{0.0f, 0.0f};
  if constexpr (RO) {
    cf yo[D];
    load_y_all<D>(a, d, s, f, yo);
    sfor<0, D>([&](auto ic) { dh = dh + cmul(w[decltype(ic)::value], yo[decltype(ic)::value]); });
  } else {
    sfor<0, D>([&](auto ic) { dh = dh + cmul(w[decltype(ic)::value], y[decltype(ic)::value]); });
  }
  if (f == 0 || f == F - 1) dh.im = 0.0f;
  if (valid) a.dhat[((((long long)d.fam * a.S + s) * a.K + d.k) * a.R + r) * F + f] = dh;
  if constexpr (DANSE_STAMP) {
    stamp(7);
    __builtin_amdgcn_s_waitcnt(0);
    stamp(8);
    // path code over the wave's lanes: 1 any noise frame, 8 any cached
    // factor, 16 any solve, 4 any factorisation
    const unsigned long long code = (__ballot(opN != 0) ? 1ull : 0ull) | (__ballot(reuse) ? 8ull : 0ull) |
                                    (__ballot(solve) ? 16ull : 0ull) | (__ballot(solve && !reuse) ? 4ull : 0ull);
    if (a.stamps && threadIdx.x <= kStampN) {
      unsigned long long v = code;
      sfor<0, kStampN>([&](auto ic) { v = (threadIdx.x == decltype(ic)::value) ? tsv[decltype(ic)::value] : v; });
      a.stamps[(long long)blockIdx.x * (kStampN + 1) + threadIdx.x] = v;
    }
  }
}


// Stand-alone batched filter update (danse_filter_update) on full [B][D][D]
// complex double SCM pairs: one batch item per lane, the same precision plan
// (GEVD: Rnn factored in float64, Ryy used in float32; MWF: Ryy factored in
// float64) in one kernel (the operator is not performance critical).
template <int D, int RMAX>
__global__ void __launch_bounds__(64) filter_update_kernel_lane(const cd* Ryy, const cd* Rnn, int Bn, int gevd,
                                                               int rank, int ref, cf* w, int* diag) {
  using namespace lane;
  int b = blockIdx.x * 64 + threadIdx.x;
  const bool valid = b < Bn;
  if (!valid) b = Bn - 1;
  __shared__ cf Ls[tri_n(D)][64];
  __shared__ cf Gs[D][64];
  const LdsTri<D> Li{Ls, (int)threadIdx.x};
  auto load = [&](const cd* src, PTriD<D>& X) {
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      sfor<0, i + 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        X.a[P(i, j)] = src[((long long)b * D + i) * D + j];
      });
    });
  };
  cf wv[D];
  bool ok = true;
  if (gevd) {
    {
      PTriD<D> N;
      load(Rnn, N);
      double invd[D];
      ok = chol64<D>(N, invd);
      cf g[D];
      ref_row<D>(N, ref, g);
      sfor<0, D>([&](auto ic) { Gs[decltype(ic)::value][threadIdx.x] = g[decltype(ic)::value]; });
      tri_inv64<D>(N, invd);
      store_tri<D>(N, Ls, threadIdx.x);
    }
    asm volatile("" ::: "memory");
    PTri<D> A;
    sfor<0, D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      sfor<0, i + 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        A.a[P(i, j)] = cfk(Ryy[((long long)b * D + i) * D + j]);
      });
    });
    cf g[D];
    sfor<0, D>([&](auto ic) { g[decltype(ic)::value] = Gs[decltype(ic)::value][threadIdx.x]; });
    congruence<D>(A, Li);
    gevd_filter_mixed<D, RMAX>(A, Li, g, rank, wv);
  } else {
    cd ncol[D];
    sfor<0, D>([&](auto ic) { ncol[decltype(ic)::value] = Rnn[((long long)b * D + decltype(ic)::value) * D + ref]; });
    PTriD<D> X;
    load(Ryy, X);
    ok = mwf_filter64<D>(X, ncol, ref, wv);
  }
  if (valid) {
    sfor<0, D>([&](auto ic) { w[(long long)b * D + decltype(ic)::value] = wv[decltype(ic)::value]; });
    if (diag) diag[b] = ok ? 0 : 1;
  }
}

}  // namespace danse
