// Lean solve kernel of the 8 x 8 lane-grid GEVD classes (rank 1, warm
// Lanczos): the solves on the cached factor Li and the cached
// C = Li Ryy Li^H (kernels.hpp c_reusable -- the common solve of a run, a
// VAD-active frame after a solve on the same factor).  Same arithmetic as the
// solve path of update_kernel_2d (update_w_gevd, d_classes.py:3343-3387;
// SCM update d_classes.py:2048-2267; dhat = w^H yhat, d_base.py:2075), but
// C moves by this round's rank one instead of being recomputed:
//   Ryy' = by Ryy + cy y y^H  =>  C' = by C + cy (Li y)(Li y)^H,
// an O(D^2) step in place of the O(D^3) congruence (update_kernel_2d stores C
// after each of its congruences, so the cache is the exact congruence of the
// last factorisation, moved by at most the VAD-active frames since).
//
// Registers and LDS: no float64 state (the factor is cached), no Householder
// reflectors (LDS2 allocated up to the Lanczos basis, solver2d.hpp), so the
// kernel runs at 3 waves per SIMD instead of 2.  A bin whose warm solve the
// Lanczos acceptance test sends back is listed (fbList) for
// fallback_kernel_2d, which runs the Householder path on the cached C and
// writes that bin's filter and estimate: this kernel writes neither for it.
#pragma once
#include "kernels_2d.hpp"

#ifndef DANSE_LEAN_DMA
#define DANSE_LEAN_DMA 1   // the factor record by LDS-DMA (0: through VGPRs, diagnostics)
#endif

namespace danse {

// Lanczos steps of the first attempt: kLz (8) on VAD frames; two more on the
// noise frames, whose transform moves C further (most of the restarts were
// there; the VAD variant would spill at its 3-waves-per-SIMD budget)
#ifndef DANSE_LEAN_LZ_VAD_DELTA
#define DANSE_LEAN_LZ_VAD_DELTA 0   // (A/B builds: steps added to kLz on VAD frames)
#endif
template <int NB, bool NZ>
constexpr int lean_lz() { return t2d::kLz<8 * NB>() + (NZ ? 2 : DANSE_LEAN_LZ_VAD_DELTA); }
template <int NB, bool NZ = true>
constexpr int lean_lds_bytes() {
  return (int)__builtin_offsetof(t2d::LDS2<NB>, U) + lean_lz<NB, NZ>() * 8 * NB * (int)sizeof(cf);
}

// w[r + 1], its history slot, and the per-bin tail (external filters, dhat)
template <int NB>
DANSE_DEV void lean_tail(const UpdateArgs& a, const FamNode& d, int s, int f, int li, uint8_t fl, cf w, cf y) {
  const int F = a.F, D = d.D, r = a.r;
  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  const bool act = li < D;
  if (act) wNext[li] = w;
  const cf dh = gsum<64>(act ? cmul(w, y) : cf{0.0f, 0.0f});
  node_bin_tail(a, d, s, f, li, fl, false, true, w, y, dh);
}

// float32 prefix sums over the lanes of a bin: over the row groups p' < p
// (lanes q + G p', inclusive) and over the lanes q' < q of the row group
template <int G>
DANSE_DEV float scan_pf(float x, int p) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const float u = __shfl_up(x, o * G, G * G);
    if (p >= o) x += u;
  }
  return x;
}
template <int G>
DANSE_DEV float scan_qf(float x, int q) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const float u = __shfl_up(x, o, G);
    if (q >= o) x += u;
  }
  return x;
}

// NZ = false: a VAD-active frame (Ryy update, cached factor):
//   C' = by C + cy (Li y)(Li y)^H.
// NZ = true: a noise frame one solve after the last (Rnn update by rank one,
// Ryy kept): the float64 factor record moves by li_rank1_2d (solver2d.hpp),
// Li' = beta^-1/2 T Li with T = Mf^-1 = diag(dd) - tril(pe p^H, -1), so
//   C' = Li' Ryy Li'^H = beta^-1 T C T^H,
// two O(D^2) passes with prefix sums: Y = T C (over the rows), C' = Y T^H / beta
// (over the columns).
template <int NB, bool NZ>
// (the noise-frame variant's float64 factor move and two prefix passes need
// the 2-waves-per-SIMD register budget)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NZ ? 2 : 3))) update_kernel_2dc(const UpdateArgs a) {
  using namespace t2d;
  constexpr int G = 8, DM = G * NB;
  static_assert(vpl<NB, G>() == 1, "one lane-layout entry per lane");
  __shared__ __attribute__((aligned(16))) char ldsRaw[lean_lds_bytes<NB, NZ>()];
  LDS2<NB, G>& S = *reinterpret_cast<LDS2<NB, G>*>(ldsRaw);   // (members up to the Lanczos basis)
  const int li = threadIdx.x, p = li / G, q = li % G;
  // DANSE_STAMP builds (kernels_2d.hpp, scripts/update_trace.py): marks 0
  // start, 1 y staged (VAD: the record landed), 2 VAD: C upper blocks /
  // noise: the factor moved and cached, 3 noise: C loaded, 4 C moved and
  // stored, 5 Lanczos, 6 w, 7 tail issued, 8 recursion and stores drained
  unsigned long long tsv[kStampN];
  auto stamp = [&](int i) {
    if constexpr (DANSE_STAMP) tsv[i] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  const int F = a.F;
  const int f = blockIdx.x % F;
  const int tt = (NZ ? a.cnItems : a.creItems)[blockIdx.x / F];
  const int fni = tt % a.nFN, s = tt / a.nFN;
  const FamNode d = a.fn[fni];
  const int D = d.D, r = a.r;
  const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  const int opY = fl & 3;
  constexpr int kRec = li_record<NB, G>();
  cf* liC = a.liCache + (long long)s * a.liStride + d.liOff + (long long)f * kRec;
  cf* cC = a.cCache + (long long)s * a.cStride + d.cOff + (long long)f * c_record<NB>() + li;
  const long long tri = (long long)s * a.scmStride + d.scmOff + (long long)f * (D * (D + 1) / 2);
  auto ent = [&](int i, int c) -> long long {
    const int hi = i >= c ? i : c, lo = i >= c ? c : i;
    return tri + hi * (hi + 1) / 2 + lo;
  };
  const double beta = a.beta[s * a.K + d.k];

  if constexpr (!NZ) {
    // the factor record straight into LDS (LDS-DMA, [S.Ls | S.g] is the
    // record's layout; no VGPR staging)
#if DANSE_LEAN_DMA
    constexpr int kChunks = (kRec * (int)sizeof(cf) + 1023) / 1024;   // 16 B per lane per instruction
    static_assert(kChunks * 1024 <= lean_lds_bytes<NB, NZ>() - (int)__builtin_offsetof(LDS2<NB>, Ls),
                  "the record's last chunk stays inside the lean LDS");
    sfor<0, kChunks>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const int e = 2 * (64 * j + li);   // first record entry of this lane's 16 bytes
      const cf* src = liC + (e + 1 < kRec ? e : kRec - 2);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(S.Ls) + 1024 * j),
                                       16, 0, 0);
    });
#else
    constexpr int kRecL = (kRec + 63) / 64, kNL = DM * (DM + 1) / 2;
    cf lrec[kRecL];
    sfor<0, kRecL>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const int e = li + 64 * j;
      lrec[j] = liC[e < kRec ? e : 0];
    });
    hold(lrec);
    sfor<0, kRecL>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const int e = li + 64 * j;
      if (e < kNL) S.Ls[e] = lrec[j];
      else if (e < kRec) S.g[e - kNL] = lrec[j];
    });
#endif
  }
  const int ych = chan_of(a, d, li, li < D);
  Blk<NB> A;
  if constexpr (!NZ) c_load_lower<NB>(A, cC);
  const cf y = load_y_c(a, d, s, f, ych, li < D);
  S.vb[li] = y;
  if constexpr (!NZ) __builtin_amdgcn_s_waitcnt(0);   // (the record's LDS-DMA landed)
  wsync();
  cf yc[NB];
  sfor<0, NB>([&](auto sc) { yc[decltype(sc)::value] = S.vb[q + G * decltype(sc)::value]; });
  wsync();
  stamp(1);
  // (after the record's LDS-DMA drained: its last chunk runs into S.U)
  if constexpr (!NZ) c_fill_upper<NB>(A, S.U, li);
  stamp(2);

  bool ok = true;
  if constexpr (!NZ) {
    if (opY) {
      const float by = (float)beta, cy = (opY == DANSE_OP_SET) ? (float)(1.0 / D) : (float)((1.0 - beta) / D);
      // u = Li y: partial sums over the row group (row layout: every lane of
      // row group p holds u[p + G sb]), the column layout through LDS
      cf ur[NB], uc[NB];
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        cf acc = cf{0.0f, 0.0f};
        sfor<0, sb + 1>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          acc = acc + ls_get<DM>(S.Ls, p + G * sb, q + G * tb) * yc[tb];   // (cmul would conjugate Li)
        });
        ur[sb] = sumq<G>(acc);
        if (q == 0) S.vb[p + G * sb] = ur[sb];
      });
      wsync();
      sfor<0, NB>([&](auto tc) { uc[decltype(tc)::value] = S.vb[q + G * decltype(tc)::value]; });
      wsync();
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
  } else {
    // the float64 factor record by rank one (Li', g in S.Ls / S.g, record
    // rewritten), then the float32 factor cache of the later solves
    const double cyN = (1.0 - beta) / D;
    cd* l64 = a.l64Cache + (long long)s * a.l64Stride + d.l64Off + (long long)f * l64_record<NB, G>();
    ok = li_rank1_2d<NB, G>(S, li, yc, beta, cyN, l64, true);
    li_store2d<NB, G>(S, liC, li);
    stamp(2);
    c_load_lower<NB>(A, cC);
    c_fill_upper<NB>(A, S.U, li);
    stamp(3);
    // T's coefficients from li_rank1_2d's LDS (S.invd: a_i = alpha |p_i|^2,
    // S.rb64[0]: p_i): t_i = 1 + sum_(k < i) a_k, dd_i = sqrt(t_i / t_(i+1)),
    // pe_i = alpha p_i / sqrt(t_i t_(i+1)); this lane's rows i = p + G sb
    const double alpha = cyN / beta;
    float ddr[NB];
    cf per[NB], pcr[NB];   // pe_i, conj(p_i)
    double tlo[NB];
    {
      double carry = 1.0;
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        const double av = S.invd[p + G * sb];
        const double inc = scan_p<G>(av, p);
        tlo[sb] = carry + (inc - av);
        carry += __shfl(inc, (G - 1) * G + q, G * G);
        const double thi = tlo[sb] + av;
        const cd pi = S.rb64[0][p + G * sb];
        ddr[sb] = (float)sqrt(tlo[sb] / thi);
        per[sb] = cfk((alpha / sqrt(tlo[sb] * thi)) * pi);
        pcr[sb] = conjg(cfk(pi));
      });
    }
    // Y = T C: Y[i][c] = dd_i C[i][c] - pe_i sum_(k < i) conj(p_k) C[k][c]
    // (a prefix over the row groups plus the earlier block rows' sums)
    {
      cf carP[NB];
      sfor<0, NB>([&](auto tc) { carP[decltype(tc)::value] = cf{0.0f, 0.0f}; });
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        sfor<0, NB>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          const cf x = A.v[sb][tb];
          const cf u = pcr[sb] * x;
          const float ire = scan_pf<G>(u.re, p), iim = scan_pf<G>(u.im, p);
          const float tre = __shfl(ire, (G - 1) * G + q, G * G), tim = __shfl(iim, (G - 1) * G + q, G * G);
          const cf ex = cf{carP[tb].re + (ire - u.re), carP[tb].im + (iim - u.im)};
          carP[tb] = cf{carP[tb].re + tre, carP[tb].im + tim};
          A.v[sb][tb] = ddr[sb] * x - per[sb] * ex;
        });
      });
    }
    // C' = Y T^H / beta: C'[i][c] = (dd_c Y[i][c] - conj(pe_c) sum_(k < c) Y[i][k] p_k) / beta
    // (a prefix over the lanes of the row group plus the earlier block
    // columns' sums); the column coefficients from row group q
    {
      const float ib = (float)(1.0 / beta);
      cf carQ[NB];
      sfor<0, NB>([&](auto sc) { carQ[decltype(sc)::value] = cf{0.0f, 0.0f}; });
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const float ddc = __shfl(ddr[tb], G * q, G * G);
        const cf pec = cf{__shfl(per[tb].re, G * q, G * G), __shfl(per[tb].im, G * q, G * G)};
        const cf pc = conjg(cf{__shfl(pcr[tb].re, G * q, G * G), __shfl(pcr[tb].im, G * q, G * G)});   // p_c
        sfor<0, NB>([&](auto sc) {
          constexpr int sb = decltype(sc)::value;
          const cf yv = A.v[sb][tb];
          const cf v = yv * pc;
          const float ire = scan_qf<G>(v.re, q), iim = scan_qf<G>(v.im, q);
          const float tre = __shfl(ire, G - 1, G), tim = __shfl(iim, G - 1, G);
          const cf ex = cf{carQ[sb].re + (ire - v.re), carQ[sb].im + (iim - v.im)};
          carQ[sb] = cf{carQ[sb].re + tre, carQ[sb].im + tim};
          cf x = ib * (ddc * yv - conjg(pec) * ex);
          if (sb == tb && p == q) x.im = 0.0f;
          A.v[sb][tb] = x;
        });
      });
      c_store<NB>(cC, A);
    }
  }

  if constexpr (!NZ) stamp(3);
  stamp(4);
  cf* vC = a.vCache + (long long)s * a.vStride + d.vOff + (long long)f * DM;
  cf vv[1];
  float lam1;
  bool warm;
  // this round's SCM recursion (as update_kernel_2d: Ryy in float32, or on a
  // noise frame Rnn in float64), after the solve: none of its registers is
  // live across the Lanczos phase
  auto recursion = [&]() {
    if constexpr (!NZ) {
      if (!opY) return;
    }
    constexpr int kLo = NB * (NB + 1) / 2;
    wsync();   // (the solve's LDS reads before the staging write)
    S.vb[li] = y;
    wsync();
    cf yr[NB], yq[NB];
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      yr[sb] = S.vb[p + G * sb];
      yq[sb] = S.vb[q + G * sb];
    });
    if constexpr (!NZ) {
      cf rlo[kLo];
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        sfor<0, sb + 1>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          const int i = p + G * sb, c = q + G * tb;
          const bool lo = i < D && c < D && i >= c;
          rlo[sb * (sb + 1) / 2 + tb] = a.Ryy[lo ? ent(i, c) : tri];
        });
      });
      const float by = (float)beta, cy = (opY == DANSE_OP_SET) ? (float)(1.0 / D) : (float)((1.0 - beta) / D);
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        sfor<0, sb + 1>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          const int i = p + G * sb, c = q + G * tb;
          const cf yy = cy * mulc(yr[sb], yq[tb]);
          cf x = csel(opY == DANSE_OP_SET, yy, by * rlo[sb * (sb + 1) / 2 + tb] + yy);
          if (i == c) x.im = 0.0f;
          if (i < D && c < D && i >= c) a.Ryy[ent(i, c)] = x;
        });
      });
    } else {
      // Rnn' = beta Rnn + cy y y^H (opN = AVG), float64, lower entries
      const double cy = (1.0 - beta) / D;
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        cd rn[sb + 1];
        sfor<0, sb + 1>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          const int i = p + G * sb, c = q + G * tb;
          const bool lo = i < D && c < D && i >= c;
          rn[tb] = ld_cd(a.Rnn + (lo ? ent(i, c) : tri));
        });
        hold(rn);
        sfor<0, sb + 1>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          const int i = p + G * sb, c = q + G * tb;
          cd yy = cd{0.0, 0.0};
          fma_cc(yy, cdk(yr[sb]), cdk(yq[tb]));
          cd x = beta * rn[tb];
          x.re = fma(cy, yy.re, x.re);
          x.im = (i == c) ? 0.0 : fma(cy, yy.im, x.im);
          if (i < D && c < D && i >= c) st_cd(a.Rnn + ent(i, c), x);
        });
      });
    }
  };
  if constexpr (NZ) {
    if (!ok && li == 0) atomicOr(&a.diag[(s * a.K + d.k) * kMaxFam + d.fam], 1);
  }
  const bool conv = lanczos2d<NB, G, lean_lz<NB, NZ>()>(A, S, li, D, vC, vv, lam1, warm);
  stamp(5);
  if (!conv) {
    // (wave-uniform) fallback_kernel_2d writes this bin: a restart from this
    // attempt's Ritz vector, else the Householder path
    if (warm && li < DM) vC[li] = vv[0];
    recursion();
    if (li == 0) {
      const int e = atomicAdd(&a.fbCount[r], 1);
      a.fbList[e] = tt * F + f;
    }
    return;
  }
  cf w[1];
  rank1_w2d<NB, G>(S, li, D, vv, lam1, w);
  stamp(6);
  if (li < DM) vC[li] = vv[0];
  if (a.lzStats && li == 0) atomicAdd(&a.lzStats[((long long)(2 * r)) * kLzSlots + (blockIdx.x & (kLzSlots - 1))], 1);
  lean_tail<NB>(a, d, s, f, li, fl, w[0], y);
  stamp(7);
  recursion();
  if constexpr (DANSE_STAMP) {
    __builtin_amdgcn_s_waitcnt(0);
    stamp(8);
    if (a.stamps && threadIdx.x <= kStampN) {
      // lane i stores mark i (vector stores), lane kStampN the path code
      // (128 lean, 256 noise frame, 32 Lanczos accepted)
      unsigned long long v = 128ull | (NZ ? 256ull : 0ull) | 32ull;
      sfor<0, kStampN>([&](auto ic) { v = (threadIdx.x == decltype(ic)::value) ? tsv[decltype(ic)::value] : v; });
      a.stamps[(long long)blockIdx.x * (kStampN + 1) + threadIdx.x] = v;
    }
  }
}

// The warm solves update_kernel_2dc sent back: the Householder path
// (tridiagonalisation, eigen part, back-transform; gevd2d_solve path 2) on
// the C and factor it cached, then the filter and the tail.  A fixed grid
// strides over this round's list.
template <int NB>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) fallback_kernel_2d(const UpdateArgs a) {
  using namespace t2d;
  constexpr int G = 8, DM = G * NB;
  __shared__ LDS2<NB, G> S;
  const int li = threadIdx.x;
  const int F = a.F, r = a.r;
  const int n = a.fbCount[r];
  for (int e = blockIdx.x; e < n; e += gridDim.x) {
    const int code = a.fbList[e];
    const int tt = code / F, f = code % F;
    const int fni = tt % a.nFN, s = tt / a.nFN;
    const FamNode d = a.fn[fni];
    const int D = d.D;
    const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
    const cf* cC = a.cCache + (long long)s * a.cStride + d.cOff + (long long)f * c_record<NB>() + li;
    Blk<NB> A;
    c_load_lower<NB>(A, cC);
    const cf y = load_y(a, d, s, f, li, li < D);
    wsync();   // the previous item's LDS reads before this item's writes
    c_fill_upper<NB>(A, S.U, li);
    li_load2d<NB, G>(S, a.liCache + (long long)s * a.liStride + d.liOff + (long long)f * li_record<NB, G>(), li);
    cf* vC = a.vCache + (long long)s * a.vStride + d.vOff + (long long)f * DM;
    cf w[1];
    // kLz more Lanczos steps from update_kernel_2dc's Ritz vector (counted as
    // accepted warm solves), else the Householder path (counted sent back)
    cf vv[1];
    float lam1;
    bool warm;
    if (lanczos2d<NB, G>(A, S, li, D, vC, vv, lam1, warm)) {
      rank1_w2d<NB, G>(S, li, D, vv, lam1, w);
      if (li < DM) vC[li] = vv[0];
      if (a.lzStats && li == 0)
        atomicAdd(&a.lzStats[((long long)(2 * r)) * kLzSlots + (blockIdx.x & (kLzSlots - 1))], 1);
    } else {
      tridiag2d<NB, G>(A, S, li, D);
      eigen2d<NB, 1, G>(S, li, D, 1, w, vC, true);
      if (a.lzStats && li == 0)
        atomicAdd(&a.lzStats[((long long)(2 * r + 1)) * kLzSlots + (blockIdx.x & (kLzSlots - 1))], 1);
    }
    lean_tail<NB>(a, d, s, f, li, fl, w[0], y);
  }
  // the last block to finish has seen every block read n: it zeroes this
  // round's counter (and the done counter fbCount[R]), so a later run without
  // danse_engine_reset starts from an empty list
  if (li == 0) {
    __threadfence();
    if (atomicAdd(&a.fbCount[a.R], 1) == (int)gridDim.x - 1) {
      atomicExch(&a.fbCount[r], 0);
      atomicExch(&a.fbCount[a.R], 0);
    }
  }
}

}  // namespace danse
