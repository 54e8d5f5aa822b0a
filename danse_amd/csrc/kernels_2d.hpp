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
// Li in float32 (LDS) -> Ryy recursion (+ store) -> congruence, tridiagonal,
// eigen part, back-transform.
#pragma once
#include "kernels.hpp"

#ifndef DANSE_2D_WPE
#define DANSE_2D_WPE 2
#endif

#include "solver2d.hpp"

namespace danse {

// G = 8: one bin per wave on the 8 x 8 lane grid; G = 4: four bins per wave
// (bins f0 .. f0 + 3 of one scene / family-node), each on a 16-lane DPP row,
// lane-layout vectors with vpl entries per lane (solver2d.hpp).
// Split solves (UpdateArgs.splitSolve; in asy updating one node of K solves
// per round, the others only run the recursion):
//   SM = 1  recursion-only launch over every item: the items that solve this
//           round return at once, the solver is compiled out, so the launch
//           is not held to the solver's register budget;
//   SM = 2  the solving items only, launch item b / FG = solveItems[b / FG].
// SCMs: packed lower triangles (the upper entries of a lane's blocks are the
// conjugates of the stored lower ones, only the lower ones are written back,
// the diagonals are kept real), bin-major; PK (with SM = 2): a lane class's
// bin-minor triangles (kernels_lane.hpp).
// The C cache of a bin (UpdateArgs.cCache): the lane-layout blocks sb >= tb
// of C, [NB (NB + 1) / 2][64] (the blocks above come back by an 8 x 8 lane
// transpose: entry (p + 8 sb, q + 8 tb) of an upper block is the conjugate of
// lane (q, p)'s entry of block (tb, sb)).  cC points at this lane's column.
template <int NB>
constexpr int c_record() { return NB * (NB + 1) / 2 * 64; }
template <int NB>
DANSE_DEV void c_store(cf* cC, const t2d::Blk<NB>& A) {
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    sfor<0, sb + 1>([&](auto tc) {
      constexpr int tb = decltype(tc)::value;
      cC[(sb * (sb + 1) / 2 + tb) * 64] = A.v[sb][tb];
    });
  });
}
template <int NB>
DANSE_DEV void c_load_lower(t2d::Blk<NB>& A, const cf* cC) {
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    sfor<0, sb + 1>([&](auto tc) {
      constexpr int tb = decltype(tc)::value;
      A.v[sb][tb] = cC[(sb * (sb + 1) / 2 + tb) * 64];
    });
  });
}
// the upper blocks from the lower ones through buf (LDS, (NB - 1) * G * G
// entries; li the bin-local lane: G = 4 runs four bins per wave, each with
// its own buf)
template <int NB, int G = 8>
DANSE_DEV void c_fill_upper(t2d::Blk<NB>& A, cf* buf, int li) {
  const int p = li / G, q = li % G;
  sfor<1, NB>([&](auto tc) {
    constexpr int tb = decltype(tc)::value;
    t2d::wsync();
    sfor<0, tb>([&](auto sc) { buf[decltype(sc)::value * G * G + q * G + p] = A.v[tb][decltype(sc)::value]; });
    t2d::wsync();
    sfor<0, tb>([&](auto sc) { A.v[decltype(sc)::value][tb] = conjg(buf[decltype(sc)::value * G * G + p * G + q]); });
  });
  t2d::wsync();
}
// G = 4 (four bins per wave, kernels' bin group fg): the cache holds the
// wave's lower blocks [NB (NB + 1) / 2][64] per bin GROUP, so that each block
// is one 512-byte wave access; cC points at this lane's entry of block 0
template <int NB>
DANSE_DEV cf* c4_ptr(const UpdateArgs& a, const FamNode& d, int s, int fg) {
  return a.cCache + (long long)s * a.cStride + d.cOff + (long long)fg * c_record<NB>() + threadIdx.x;
}

// G = 4: the four bins' float32 factor records (S.Ls | S.g, li_record
// entries each, contiguous per bin in the cache and in LDS2) straight into
// LDS by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave instruction, no
// VGPR staging); the last chunk of a bin runs into its S.U, which the solver
// writes before it reads.  Waited for by the caller (s_waitcnt vmcnt(0)).
template <int NB>
DANSE_DEV void li_dma4(char* ldsRaw, const cf* rec0, int fg, int F) {
  constexpr int G = 4, W = 4;
  constexpr int kRec = t2d::li_record<NB, G>();
  constexpr int kChunks = (kRec * (int)sizeof(cf) + 1023) / 1024;
  static_assert(kRec % 2 == 0, "16-byte pieces of the record");
  static_assert(sizeof(t2d::LDS2<NB, G>) % 16 == 0 && __builtin_offsetof(t2d::LDS2<NB, G>, Ls) % 16 == 0,
                "every bin's S.Ls 16-byte aligned in LDS");
  static_assert(kChunks * 1024 <= (int)sizeof(t2d::LDS2<NB, G>) - (int)__builtin_offsetof(t2d::LDS2<NB, G>, Ls),
                "the record's last chunk stays inside the bin's LDS2");
  const int lane = threadIdx.x;
  sfor<0, W>([&](auto bc) {
    constexpr int b = decltype(bc)::value;
    const int fb = min(fg * W + b, F - 1);
    const cf* rec = rec0 + (long long)fb * kRec;
    char* dst = ldsRaw + b * (int)sizeof(t2d::LDS2<NB, G>) + (int)__builtin_offsetof(t2d::LDS2<NB, G>, Ls);
    sfor<0, kChunks>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const int e = 2 * (64 * j + lane);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(rec + (e + 1 < kRec ? e : kRec - 2)),
                                       (__attribute__((address_space(3))) void*)(dst + 1024 * j), 16, 0, 0);
    });
  });
}

template <int NB, int RMAX, int G = 8, bool PK = false, int SM = 0>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NB <= 5 ? DANSE_2D_WPE : 1)))
update_kernel_2d(const UpdateArgs a) {
  using namespace t2d;
  constexpr int L = bin_lanes<G>(), W = 64 / L, V = vpl<NB, G>();
  // (the recursion-only launch needs only the y staging vector: its LDS
  // stays small so that the launch is not held to the solver's LDS budget)
  constexpr int kLds = (SM == 1) ? (int)sizeof(cf) * W * L * V : (int)sizeof(LDS2<NB, G>) * W;
  __shared__ __attribute__((aligned(16))) char ldsRaw[kLds];
  const int bw = threadIdx.x / L;
  const int li = threadIdx.x % L;
  LDS2<NB, G>& S = reinterpret_cast<LDS2<NB, G>*>(ldsRaw)[bw];   // (not touched when SM == 1)
  cf* const vb = (SM == 1) ? reinterpret_cast<cf*>(ldsRaw) + bw * L * V : S.vb;
  const int p = li / G, q = li % G;
  unsigned long long tsv[kStampN];
  int tcode = 0;
  auto stamp = [&](int i) {
    if constexpr (DANSE_STAMP) tsv[i] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  const int F = a.F;
  const int FG = (F + W - 1) / W;
  const int fg = blockIdx.x % FG;
  const int tt = (SM == 2) ? a.solveItems[blockIdx.x / FG] : blockIdx.x / FG;
  const int f0 = fg * W + bw;
  const bool fvalid = (W == 1) || f0 < F;   // the last group's tail bins compute on bin F-1, store nothing
  const int f = (W == 1 || f0 < F) ? f0 : F - 1;
  const int fni = tt % a.nFN;
  const int s = tt / a.nFN;
  const FamNode d = a.fn[fni];
  if (!node_in(a.nodeMask, d.k)) return;   // wave-uniform: one item per wave
  const int D = d.D;
  const int r = a.r;
  const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  const int opY = fl & 3, opN = (fl >> 2) & 3;
  const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;
  bool solve = (fl & DANSE_FLAG_SOLVE) != 0 && !pregiven;
  if constexpr (SM == 1) {
    if (solve) return;   // wave-uniform: the SM = 2 launch runs this item
    solve = false;
  }
  const bool initslot = (fl & DANSE_FLAG_INITSLOT) != 0;
  // factor cache (kernels.hpp li_reusable): per bin S.Ls (packed Li, float32)
  // and g (solver2d.hpp li_record / li_store2d)
  const bool reuse = solve && li_reusable(a, d, s, opN);
  cf* liC = a.liCache ? a.liCache + (long long)s * a.liStride + d.liOff + (long long)f * li_record<NB, G>() : nullptr;
  // float64 factor record (solver2d.hpp li_rank1_2d): a solve one noise
  // frame after the last factorisation updates it by rank one
  cd* l64 = (!PK && SM == 0 && a.l64Cache && d.l64Off >= 0)
                ? a.l64Cache + (long long)s * a.l64Stride + d.l64Off + (long long)f * l64_record<NB, G>()
                : nullptr;
  // eigenvector cache of the warm-started rank-1 path (solver2d.hpp lanczos2d)
  cf* vC = (!PK && SM == 0 && a.vCache && d.vOff >= 0)
               ? a.vCache + (long long)s * a.vStride + d.vOff + (long long)f * (G * NB)
               : nullptr;
  // C = Li Ryy Li^H per bin ([NB * NB][64], this lane layout), stored after
  // every congruence: the solves on the cached factor and C (kernels.hpp
  // c_reusable) run on update_kernel_2dc (kernels_2dc.hpp) and skip this one
  const bool hasC = G == 8 && !PK && SM == 0 && a.cCache && d.cOff >= 0;
  if (hasC && (a.leanOn || a.leanNoise) && r % kCRefresh != 0 && c_reusable(a, d, s) &&
      ((a.leanOn && reuse) || (a.leanNoise && solve && opN == DANSE_OP_AVG && opY == DANSE_OP_KEEP)))
    return;   // wave-uniform: update_kernel_2dc runs this item
  // G = 4 (four bins per wave, DMAX 20): the C cache in this kernel -- a solve
  // on the cached factor whose item solved last round with no SCM update
  // since (kernels.hpp c_reusable) moves the cached C by this round's rank
  // one (C' = by C + cy (Li y)(Li y)^H) instead of the O(D^3) congruence
  const bool hasC4 = G == 4 && !PK && SM == 0 && a.cCache && d.cOff >= 0;
  const bool useC4 = hasC4 && reuse && r % kCRefresh != 0 && c_reusable(a, d, s);
  // G = 4: the cached factor records of the four bins by LDS-DMA, issued
  // before the observation loads (they land while the y chain runs)
  constexpr bool kDma4 = G == 4 && !PK && SM == 0;
  if constexpr (kDma4) {
    if (reuse) li_dma4<NB>(ldsRaw, a.liCache + (long long)s * a.liStride + d.liOff, fg, F);
  }

  // Loads of the solve on a cached factor (the common solve: a VAD frame,
  // Rnn unchanged since the last factorisation) issued with the observation's:
  // the factor record (S.Ls + g) and the Ryy block, so that the record, the
  // block and the spectra are one memory round trip instead of three.
  constexpr int kRec = t2d::li_record<NB, G>(), kRecL = (kRec + L - 1) / L, kNL = G * NB * (G * NB + 1) / 2;
  // (G = 4 keeps the separate loads: its 16-entry record chunk next to the
  // Ryy block spilled)
  constexpr bool kPre = (SM != 1) && G == 8;
  const long long triOff0 = PK ? (long long)s * a.scmStride + d.scmOff + f
                               : (long long)s * a.scmStride + d.scmOff + (long long)f * (D * (D + 1) / 2);
  auto entA = [&](int i, int c) -> long long {
    const int hi = i >= c ? i : c, lo = i >= c ? c : i;
    const long long t = hi * (hi + 1) / 2 + lo;
    return PK ? triOff0 + t * F : triOff0 + t;
  };
  Blk<NB> A;
  cf lrec[kRecL];
  int ych[V];
  sfor<0, V>([&](auto vc) {
    constexpr int v = decltype(vc)::value;
    const int i = li + L * v;
    ych[v] = chan_of(a, d, i, i < D);
  });
  if constexpr (kPre) {
    if (reuse) {
      sfor<0, kRecL>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const int e = li + L * j;
        lrec[j] = liC[e < kRec ? e : 0];
      });
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        sfor<0, NB>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          const int i = p + G * sb, c = q + G * tb;
          const bool in = i < D && c < D;
          A.v[sb][tb] = a.Ryy[in ? entA(i, c) : triOff0];
        });
      });
    }
  }
  cf y[V];
  sfor<0, V>([&](auto vc) {
    constexpr int v = decltype(vc)::value;
    const int i = li + L * v;
    y[v] = load_y_c(a, d, s, f, ych[v], i < D);
  });
  if constexpr (kPre) {
    if (reuse) {
      hold(lrec);
      sfor<0, NB>([&](auto sc) { hold(A.v[decltype(sc)::value]); });
      // the record into LDS (li_load2d's layout: [0, kNL) S.Ls, then g)
      sfor<0, kRecL>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const int e = li + L * j;
        if (e < kNL) S.Ls[e] = lrec[j];
        else if (e < kRec) S.g[e - kNL] = lrec[j];
      });
    }
  }
  sfor<0, V>([&](auto vc) {
    constexpr int v = decltype(vc)::value;
    vb[li + L * v] = y[v];
  });
  t2d::wsync();
  cf yr[NB], yc[NB];
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    yr[sb] = vb[p + G * sb];
    yc[sb] = vb[q + G * sb];
  });
  t2d::wsync();
  stamp(1);
  const double beta = a.beta[s * a.K + d.k];
  // entry (i, c) of the SCM (both in range): the stored lower entry (hi, lo)
  // -- packed lower triangles, bin-major ([F][D(D+1)/2], FamNode.packed 2), or
  // with PK the lane class's bin-minor [D(D+1)/2][F]; the upper entries are
  // the conjugates of the stored lower ones
  const long long triOff = PK ? (long long)s * a.scmStride + d.scmOff + f
                              : (long long)s * a.scmStride + d.scmOff + (long long)f * (D * (D + 1) / 2);
  auto ent = [&](int i, int c) -> long long {
    const int hi = i >= c ? i : c, lo = i >= c ? c : i;
    const long long t = hi * (hi + 1) / 2 + lo;
    return PK ? triOff + t * F : triOff + t;
  };
  const long long safe = triOff;   // (an in-bounds address for the padding entries)

  // ---- Rnn (float64): recursion, store, factor -> Li in S.Ls -------------
  bool ok = true;
  const bool rec = !(SM == 1 && a.noRec);   // (span.hpp: the prefix's recursion deferred)
  if (rec && (opN || (solve && !reuse))) {
    BlkD<NB> M;
    const double cy = (opN == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
    const double cx = (opN == DANSE_OP_SET) ? 0.0 : beta;
    // (every block entry loaded before the first store -- a load after a
    // store to the same array is not moved above it, and the block was one
    // memory round trip per entry; the recursion-only variant SM = 1 loads
    // row by row, its register budget is a streaming kernel's)
    auto ld_row_Rnn = [&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p + G * sb, c = q + G * tb;
        const bool in = i < D && c < D;
        M.v[sb][tb] = a.Rnn[in ? ent(i, c) : safe];
      });
    };
    if constexpr (SM != 1) {
      sfor<0, NB>(ld_row_Rnn);
      sfor<0, NB>([&](auto sc) { hold(M.v[decltype(sc)::value]); });
    }
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      if constexpr (SM == 1) {
        ld_row_Rnn(sc);
        hold(M.v[sb]);
      }
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p + G * sb, c = q + G * tb;
        const bool in = i < D && c < D;
        cd x = csel(in, M.v[sb][tb], cd{0.0, 0.0});
        if (i < c) x = conjg(x);
        if (i == c) x.im = 0.0;
        if (opN) {
          cd yy = cd{0.0, 0.0};
          fma_cc(yy, cdk(yr[sb]), cdk(yc[tb]));
          x = cx * x;
          x.re = fma(cy, yy.re, x.re);
          x.im = (i == c) ? 0.0 : fma(cy, yy.im, x.im);
          if (in && fvalid && i >= c) a.Rnn[ent(i, c)] = x;
        }
        M.v[sb][tb] = x;
      });
    });
    stamp(2);
    if (solve && !reuse) {
      if (l64 && beta > 0.0 && li_updatable(a, d, s, opN)) {
        ok = li_rank1_2d<NB, G>(S, li, yc, beta, cy, l64, fvalid);
        tcode |= 2;
      } else {
        ok = gevd2d_factor<NB, G>(M, S, li, D, d.ref, fvalid ? l64 : nullptr);
        tcode |= 4;
      }
      if (liC && fvalid) li_store2d<NB, G>(S, liC, li);
    }
  } else {
    stamp(2);
  }
  if constexpr (kDma4) {
    if (reuse) {
      __builtin_amdgcn_s_waitcnt(0);   // (the records' LDS-DMA landed)
      t2d::wsync();
    }
  } else {
    if (!kPre && reuse) li_load2d<NB, G>(S, liC, li);
  }
  tcode |= (opN ? 1 : 0) | (reuse ? 8 : 0) | (solve ? 16 : 0);
  stamp(3);

  // ---- Ryy (float32): recursion, store, filter ---------------------------
  cf w[V];
  sfor<0, V>([&](auto vc) { w[decltype(vc)::value] = cf{0.0f, 0.0f}; });
  if (rec && (opY || solve)) {
    const float by = (float)beta, cy = (opY == DANSE_OP_SET) ? (float)(1.0 / D) : (float)((1.0 - beta) / D);
    auto ld_row_Ryy = [&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p + G * sb, c = q + G * tb;
        const bool in = i < D && c < D;
        A.v[sb][tb] = a.Ryy[in ? ent(i, c) : safe];
      });
    };
    if constexpr (SM != 1) {
      if (!kPre || !reuse) {   // (kPre and reuse: loaded with the observation above)
        sfor<0, NB>(ld_row_Ryy);
        sfor<0, NB>([&](auto sc) { hold(A.v[decltype(sc)::value]); });
      }
    }
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      if constexpr (SM == 1) {
        ld_row_Ryy(sc);
        hold(A.v[sb]);
      }
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p + G * sb, c = q + G * tb;
        const bool in = i < D && c < D;
        cf x = csel(in, A.v[sb][tb], cf{0.0f, 0.0f});
        if (i < c) x = conjg(x);
        if (opY) {
          const cf yy = cy * mulc(yr[sb], yc[tb]);
          x = csel(opY == DANSE_OP_SET, yy, by * x + yy);
          if (i == c) x.im = 0.0f;
          if (in && fvalid && i >= c) a.Ryy[ent(i, c)] = x;
        }
        A.v[sb][tb] = x;
      });
    });
    stamp(4);
    if (solve) {
      if (useC4) {
        // C' = by C + cy u u^H, u = Li y (Ryy' = by Ryy + cy y y^H; the
        // factor is unchanged): u in the row layout by row-group sums, the
        // column layout through LDS (as kernels_2dc.hpp)
        cf* cC = c4_ptr<NB>(a, d, s, fg);
        c_load_lower<NB>(A, cC);
        c_fill_upper<NB, G>(A, S.U, li);
        if (opY) {
          constexpr int DMc = G * NB;
          const float by = (float)beta, cy = (opY == DANSE_OP_SET) ? (float)(1.0 / D) : (float)((1.0 - beta) / D);
          cf ur[NB], uc[NB];
          sfor<0, NB>([&](auto sc) {
            constexpr int sb = decltype(sc)::value;
            cf acc = cf{0.0f, 0.0f};
            sfor<0, sb + 1>([&](auto tc) {
              constexpr int tb = decltype(tc)::value;
              acc = acc + ls_get<DMc>(S.Ls, p + G * sb, q + G * tb) * yc[tb];   // (cmul would conjugate Li)
            });
            ur[sb] = sumq<G>(acc);
            if (q == 0) S.vb[p + G * sb] = ur[sb];
          });
          t2d::wsync();
          sfor<0, NB>([&](auto tc) { uc[decltype(tc)::value] = S.vb[q + G * decltype(tc)::value]; });
          t2d::wsync();
          sfor<0, NB>([&](auto sc) {
            constexpr int sb = decltype(sc)::value;
            sfor<0, NB>([&](auto tc) {
              constexpr int tb = decltype(tc)::value;
              const cf uu = cy * mulc(ur[sb], uc[tb]);
              cf x = csel(opY == DANSE_OP_SET, uu, by * A.v[sb][tb] + uu);
              if (sb == tb && p == q) x.im = 0.0f;
              A.v[sb][tb] = x;
            });
          });
          c_store<NB>(cC, A);
        }
        tcode |= 128;
      } else {
        congruence2d<NB, G>(A, S, li, D);
        if (hasC && fvalid)
          c_store<NB>(a.cCache + (long long)s * a.cStride + a.fn[fni].cOff + (long long)f * c_record<NB>() + li, A);
        if (hasC4) c_store<NB>(c4_ptr<NB>(a, d, s, fg), A);   // (each bin of the group its own slot)
      }
      stamp(5);
      const int path = gevd2d_solve<NB, RMAX, G>(A, S, li, D, a.rank, w, vC, fvalid);
      // (one atomic per wave -- the path is wave-uniform -- into one of
      // kLzSlots counters per round and path: a single counter took every
      // wave's add and stalled config C's launches 2x)
      if (path && a.lzStats && threadIdx.x == 0) {
        const int nb = (W == 1) ? 1 : min(W, F - fg * W);
        atomicAdd(&a.lzStats[((long long)(2 * r + path - 1)) * kLzSlots + (blockIdx.x & (kLzSlots - 1))], nb);
      }
      tcode |= path << 5;
    } else {
      stamp(5);
    }
  } else {
    stamp(4);
    stamp(5);
  }
  stamp(6);

  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotPrev = a.wHistory ? r : (r & 1);
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  if (solve && !pregiven && !initslot && !ok && li == 0 && fvalid)
    atomicOr(&a.diag[(s * a.K + d.k) * kMaxFam + d.fam], 1);
  cf dsum;
  sfor<0, V>([&](auto vc) {
    constexpr int v = decltype(vc)::value;
    const int i = li + L * v;
    const bool act = i < D;
    const int rowc = act ? i : 0;
    if (pregiven || initslot) w[v] = csel(act, wNext[rowc], cf{0.0f, 0.0f});
    else if (!solve) w[v] = csel(act, wPrev[rowc], cf{0.0f, 0.0f});
    if (act && !pregiven && !initslot && fvalid) wNext[i] = w[v];
    const cf t = csel(act, cmul(w[v], y[v]), cf{0.0f, 0.0f});
    dsum = (v == 0) ? t : dsum + t;
  });
  const cf dh = gsum<L>(dsum);
  sfor<0, V>([&](auto vc) {
    constexpr int v = decltype(vc)::value;
    node_bin_tail(a, d, s, f, li + L * v, fl, pregiven, fvalid, w[v], y[v], dh);
  });
  if constexpr (DANSE_STAMP) {
    stamp(7);
    __builtin_amdgcn_s_waitcnt(0);   // (the stores drained: the last mark includes them)
    stamp(8);
    if (a.stamps && threadIdx.x <= kStampN) {
      // lane i stores mark i (vector stores), lane kStampN the path code
      unsigned long long v = (unsigned long long)tcode;
      sfor<0, kStampN>([&](auto ic) { v = (threadIdx.x == decltype(ic)::value) ? tsv[decltype(ic)::value] : v; });
      a.stamps[(long long)blockIdx.x * (kStampN + 1) + threadIdx.x] = v;
    }
  }
}

// Stand-alone GEVD filter update (danse_filter_update): float64 SCM pairs
// [B][D][D], one bin per wavefront (G = 8) or four per wavefront (G = 4).
template <int NB, int RMAX, int G = 8>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NB <= 5 ? DANSE_2D_WPE : 1)))
filter_update_kernel_2d(const cd* Ryy, const cd* Rnn, int B, int D, int rank, int ref, cf* w, int* diag) {
  using namespace t2d;
  constexpr int L = bin_lanes<G>(), W = 64 / L, V = vpl<NB, G>();
  __shared__ LDS2<NB, G> Sall[W];
  const int bw = threadIdx.x / L, li = threadIdx.x % L;
  LDS2<NB, G>& S = Sall[bw];
  const int p = li / G, q = li % G;
  const int b0 = blockIdx.x * W + bw;
  const bool valid = (W == 1) || b0 < B;
  const int b = (W == 1 || b0 < B) ? b0 : B - 1;
  bool ok;
  {
    BlkD<NB> M;
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p + G * sb, c = q + G * tb;
        const bool in = i < D && c < D;
        M.v[sb][tb] = csel(in, Rnn[(long long)b * D * D + (in ? i * D + c : 0)], cd{0.0, 0.0});
      });
    });
    ok = gevd2d_factor<NB, G>(M, S, li, D, ref);
  }
  Blk<NB> A;
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    sfor<0, NB>([&](auto tc) {
      constexpr int tb = decltype(tc)::value;
      const int i = p + G * sb, c = q + G * tb;
      const bool in = i < D && c < D;
      A.v[sb][tb] = csel(in, cfk(Ryy[(long long)b * D * D + (in ? i * D + c : 0)]), cf{0.0f, 0.0f});
    });
  });
  cf wv[V];
  gevd2d_filter<NB, RMAX, G>(A, S, li, D, rank, wv);
  sfor<0, V>([&](auto vc) {
    const int i = li + L * decltype(vc)::value;
    if (valid && i < D) w[(long long)b * D + i] = wv[decltype(vc)::value];
  });
  if (diag && valid && li == 0) diag[b] = ok ? 0 : 1;
}

}  // namespace danse
