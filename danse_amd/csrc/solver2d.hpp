// Two-dimensional wavefront solver for large filter dimensions
// (16 < D <= 48): one frequency bin per wavefront, the matrix spread over
// the 64 lanes as an 8 x 8 lane grid with a CYCLIC block layout.
// (update_w_gevd, danse_toolbox/d_classes.py:3343-3387.)
//
//   lane li = 8 p + q owns the NB x NB entries (p + 8 s, q + 8 t), s, t < NB
//   (DM = 8 NB, the class size).
//
// Every lane does useful work at every pivot (the row-per-lane layout of
// solver64m.hpp keeps 64 - D lanes idle and broadcasts one column element
// per v_readlane).  A pivot step j = 8 sj + rj is split into a STATIC block
// index sj (the outer loop is unrolled over it, so every register index is a
// compile-time constant and blocks left of the pivot are skipped at compile
// time) and a runtime lane index rj.  Cross-lane traffic:
//   * pivot column -> every lane: its 8 owners (q == rj) write it to a
//     double-buffered LDS vector, every lane reads its NB row and NB column
//     entries (broadcast reads, one barrier per step);
//   * sums over the 8 lanes of a row group (q): three DPP steps
//     (quad_perm, quad_perm, row_half_mirror), no LDS;
//   * sums over the 8 row groups (p): DPP row_ror:8, then two bpermutes.
//
// Precision plan (as solver64m.hpp): Rnn factored and
// inverted in float64 (Cholesky, Li = L^-1 in place), Li rounded to float32
// once; C = Li Ryy Li^H, the Householder tridiagonalisation, multisection,
// inverse iteration and back-transform in float32.
#pragma once
#include "solver64m.hpp"   // big::rld, big::top_eigvals / tri_eigvec, lane::rsqrt64

namespace danse {
namespace t2d {

template <int NB>
struct BlkD {
  cd v[NB][NB];
};
template <int NB>
struct Blk {
  cf v[NB][NB];
};

template <int NB>
struct LDS2 {
  static constexpr int DM = 8 * NB;
  cd cb64[2][DM];   // float64 pivot column (double-buffered)
  cd rb64[2][DM];   // float64 pivot row
  double invd[DM];  // 1 / L[j][j]
  cf cb[2][DM];     // float32 pivot column
  cf qb[2][DM];     // row -> column layout transpose of q
  union {
    cf Ls[DM][DM + 1];   // Li (float32) during the congruence
    cf U[DM][DM + 1];    // then the Householder vectors U[j][i]
  } m;
  float a[DM];        // tridiagonal: diagonal
  cf b[DM];           //              subdiagonal b[i] = T[i][i-1]
  float e2[DM];       //              |b[i+1]|^2
  float ev[DM];       //              |b[i+1]|
  cf phi[DM];         //              phases phi_i = prod_{k<=i} b_k / |b_k|
  float4 fac[DM];     // inverse iteration: eliminated rows (d, du, dl2, rhs)
  float xs[64];       //                    right-hand side of the next sweep
  cf g[64];           // g = L^H e_ref (lane layout)
  cf vb[64];          // lane layout -> row layout
  cf wb[64];          // column layout -> lane layout
  float x[kRMax][DM]; // tridiagonal eigenvectors (Gram-Schmidt, rank > 1)
};

// ---- cross-lane helpers ---------------------------------------------------
// LDS hand-off inside the one-wave workgroup: LDS operations of a wavefront
// execute in order, so a wavefront-scope fence pair (no s_waitcnt, no
// s_barrier) only has to stop the compiler from moving LDS accesses across.
DANSE_DEV void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int CTRL>
DANSE_DEV double dpp_d(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(v & 0xffffffffll), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// sum over the 8 lanes of my row group (lanes 8p .. 8p+7)
DANSE_DEV float sumq(float x) {
  x += dpp_x<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_x<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp_x<0x141>(x);   // row_half_mirror (quads 0/1 of each half-row)
  return x;
}
DANSE_DEV cf sumq(cf x) { return cf{sumq(x.re), sumq(x.im)}; }
DANSE_DEV double sumq(double x) {
  x += dpp_d<0xB1>(x);
  x += dpp_d<0x4E>(x);
  x += dpp_d<0x141>(x);
  return x;
}
DANSE_DEV cd sumq(cd x) { return cd{sumq(x.re), sumq(x.im)}; }
// sum over the 8 row groups (lanes q, q+8, ..., q+56)
DANSE_DEV float sump(float x) {
  x += dpp_x<0x128>(x);   // row_ror:8 == xor 8 inside a 16-lane row
  x += __shfl_xor(x, 16);
  x += __shfl_xor(x, 32);
  return x;
}
DANSE_DEV cf sump(cf x) { return cf{sump(x.re), sump(x.im)}; }

// ---- float64 Cholesky, in place: M = L (lower, upper part zeroed) -----------
template <int NB>
DANSE_DEV bool chol2d(BlkD<NB>& M, LDS2<NB>& S, int li, int D) {
  const int p = li >> 3, q = li & 7;
  bool ok = true;
  int buf = 0;
  sfor<0, NB>([&](auto sjc) {
    constexpr int sj = decltype(sjc)::value;
    for (int rj = 0; rj < 8; ++rj) {
      const int j = 8 * sj + rj;
      if (j >= D) break;
      const double p0 = big::rld(M.v[sj][sj].re, 9 * rj);   // lane (rj, rj)
      ok = ok && (p0 > 1e-300);
      const double piv = p0 > 1e-300 ? p0 : 1e-300;
      const double inv = lane::rsqrt64(piv);
      if (li == 0) S.invd[j] = inv;
      if (q == rj) {
        sfor<sj, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const int i = p + 8 * s;
          const cd v0 = M.v[s][sj];
          const cd v = csel(i == j, cd{piv * inv, 0.0}, csel(i > j, inv * v0, cd{0.0, 0.0}));
          M.v[s][sj] = v;
          S.cb64[buf][i] = csel(i > j, v, cd{0.0, 0.0});
        });
      }
      wsync();
      cd rv[NB], cv[NB];
      sfor<sj, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        rv[s] = S.cb64[buf][p + 8 * s];
        cv[s] = S.cb64[buf][q + 8 * s];
      });
      sfor<sj, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        sfor<sj, s + 1>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          fms_cc(M.v[s][t], rv[s], cv[t]);
        });
      });
      buf ^= 1;
    }
  });
  sfor<0, NB>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if (p + 8 * s < q + 8 * t) M.v[s][t] = cd{0.0, 0.0};
    });
  });
  return ok;
}

// ---- float64 in-place inverse of the lower-triangular L, right-looking
// (forward elimination of L X = I, no reductions): at step k
//   X[k][:] = X[k][:] / L[k][k]                        (row k is final)
//   X[i][c] -= L[i][k] X[k][c]   for i > k, c <= k      (X[i][k] replaces L[i][k])
// Row k (owners p == rk) and column k of L (owners q == rk) are broadcast
// through LDS, one barrier per step.
template <int NB>
DANSE_DEV void trinv2d(BlkD<NB>& M, LDS2<NB>& S, int li, int D) {
  const int p = li >> 3, q = li & 7;
  int buf = 0;
  sfor<0, NB>([&](auto skc) {
    constexpr int sk = decltype(skc)::value;
    for (int rk = 0; rk < 8; ++rk) {
      const int k = 8 * sk + rk;
      if (k >= D) break;
      const double ik = S.invd[k];
      if (p == rk) {
        sfor<0, NB>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          const int c = q + 8 * t;
          const cd v = csel(c == k, cd{ik, 0.0}, csel(c < k, ik * M.v[sk][t], cd{0.0, 0.0}));
          M.v[sk][t] = v;
          S.rb64[buf][c] = v;
        });
      }
      if (q == rk) {
        sfor<sk, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const int i = p + 8 * s;
          S.cb64[buf][i] = csel(i > k, M.v[s][sk], cd{0.0, 0.0});
        });
      }
      wsync();
      cd lc[NB], xr[NB];
      sfor<sk, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        lc[s] = S.cb64[buf][p + 8 * s];
      });
      sfor<0, sk + 1>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        xr[t] = S.rb64[buf][q + 8 * t];
      });
      sfor<sk, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        const int i = p + 8 * s;
        sfor<0, sk + 1>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          cd x = M.v[s][t];
          if constexpr (t == sk) x = csel(q == rk && i > k, cd{0.0, 0.0}, x);
          fms_c(x, lc[s], xr[t]);
          M.v[s][t] = x;
        });
      });
      buf ^= 1;
    }
  });
}

// ---- phase 1: Rnn block (float64, destroyed) -> Li (float32 block), g in LDS
template <int NB>
DANSE_DEV bool gevd2d_factor(BlkD<NB>& M, Blk<NB>& Lf, LDS2<NB>& S, int li, int D, int ref) {
  const int p = li >> 3, q = li & 7;
  const bool ok = chol2d<NB>(M, S, li, D);
  // g = L^H e_ref: g_c = conj(L[ref][c]) (c <= ref; the upper part is zero)
  S.g[li] = cf{0.0f, 0.0f};
  wsync();
  {
    // row ref of L: block row ref >> 3 (a select chain over the static
    // block index, no branches) on the row group p == ref & 7
    const int sr = ref >> 3;
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      cd v = M.v[0][t];
      sfor<1, NB>([&](auto sc) { v = csel(decltype(sc)::value == sr, M.v[decltype(sc)::value][t], v); });
      if (p == (ref & 7)) S.g[q + 8 * t] = conjg(cfk(v));
    });
  }
  trinv2d<NB>(M, S, li, D);
  sfor<0, NB>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      Lf.v[s][t] = cfk(M.v[s][t]);
    });
  });
  return ok;
}

// ---- C = Li A Li^H in place of A (float32); Li staged in LDS ---------------
template <int NB>
DANSE_DEV void congruence2d(Blk<NB>& A, const Blk<NB>& Lf, LDS2<NB>& S, int li, int D) {
  const int p = li >> 3, q = li & 7;
  // scipy.linalg.eigh reads the lower triangle: A[i][c] = conj(A[c][i]) for
  // i < c (the SCMs are Hermitian except for the random init's residue).
  // Element (c, i) lives on lane (q, p), register [t][s], and is never one
  // that this loop rewrites.
  {
    const int tl = 8 * q + p;
    sfor<0, NB>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const cf v = cf{__shfl(A.v[t][s].re, tl), __shfl(A.v[t][s].im, tl)};
        A.v[s][t] = csel(p + 8 * s < q + 8 * t, conjg(v), A.v[s][t]);
      });
    });
  }
  // Li -> LDS (row-major, pitch DM + 1)
  sfor<0, NB>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      S.m.Ls[p + 8 * s][q + 8 * t] = Lf.v[s][t];
    });
  });
  wsync();
  // Z = A Li^H: Z[i][c] = sum_k A[i][k] conj(Li[c][k]), Li[c][k] = 0 for k > c
  Blk<NB> Z;
  sfor<0, NB>([&](auto sc) {
    sfor<0, NB>([&](auto tc) { Z.v[decltype(sc)::value][decltype(tc)::value] = cf{0.0f, 0.0f}; });
  });
  sfor<0, NB>([&](auto skc) {
    constexpr int sk = decltype(skc)::value;
    for (int rk = 0; rk < 8; ++rk) {
      const int k = 8 * sk + rk;
      if (k >= D) break;
      const int src = (li & ~7) | rk;   // lane (p, rk) holds A[p + 8 s][k]
      cf ak[NB], lc[NB];
      sfor<0, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        ak[s] = cf{__shfl(A.v[s][sk].re, src), __shfl(A.v[s][sk].im, src)};
      });
      sfor<sk, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        lc[t] = S.m.Ls[q + 8 * t][k];
      });
      sfor<0, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        sfor<sk, NB>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          cf z = Z.v[s][t];
          z.re = fmaf(ak[s].re, lc[t].re, fmaf(ak[s].im, lc[t].im, z.re));
          z.im = fmaf(ak[s].im, lc[t].re, fmaf(-ak[s].re, lc[t].im, z.im));
          Z.v[s][t] = z;
        });
      });
    }
  });
  // C = Li Z: C[i][c] = sum_k Li[i][k] Z[k][c], Li[i][k] = 0 for k > i  (into A)
  sfor<0, NB>([&](auto sc) {
    sfor<0, NB>([&](auto tc) { A.v[decltype(sc)::value][decltype(tc)::value] = cf{0.0f, 0.0f}; });
  });
  sfor<0, NB>([&](auto skc) {
    constexpr int sk = decltype(skc)::value;
    for (int rk = 0; rk < 8; ++rk) {
      const int k = 8 * sk + rk;
      if (k >= D) break;
      const int src = rk * 8 + q;   // lane (rk, q) holds Z[k][q + 8 t]
      cf zk[NB], lr[NB];
      sfor<0, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        zk[t] = cf{__shfl(Z.v[sk][t].re, src), __shfl(Z.v[sk][t].im, src)};
      });
      sfor<sk, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        lr[s] = S.m.Ls[p + 8 * s][k];
      });
      sfor<sk, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        sfor<0, NB>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          fma_c(A.v[s][t], lr[s], zk[t]);
        });
      });
    }
  });
  sfor<0, NB>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (p == q) A.v[s][s].im = 0.0f;
  });
  wsync();   // every Ls read before the Householder vectors overwrite it
}

// ---- Householder tridiagonalisation of the Hermitian block A (destroyed):
// diagonal -> S.a, subdiagonal -> S.b, reflectors -> S.m.U[j][*]
template <int NB>
DANSE_DEV void tridiag2d(Blk<NB>& A, LDS2<NB>& S, int li, int D) {
  constexpr int DM = 8 * NB;
  const int p = li >> 3, q = li & 7;
  int buf = 0;
  cf ph = cf{1.0f, 0.0f};   // phi_j (wave-uniform)
  if (li == 0) S.phi[0] = ph;
  sfor<0, NB>([&](auto sjc) {
    constexpr int sj = decltype(sjc)::value;
    for (int rj = 0; rj < 8; ++rj) {
      const int j = 8 * sj + rj;
      if (j + 2 >= D) break;
      if (q == rj) {
        sfor<sj, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const int i = p + 8 * s;
          S.cb[buf][i] = csel(i > j, A.v[s][sj], cf{0.0f, 0.0f});
        });
        if (p == rj) S.a[j] = A.v[sj][sj].re;
      }
      wsync();
      cf xr[NB], xc[NB];
      sfor<sj, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        xr[s] = S.cb[buf][p + 8 * s];
        xc[s] = S.cb[buf][q + 8 * s];
      });
      const cf x0 = S.cb[buf][j + 1];
      float n2 = 0.0f;
      sfor<sj, NB>([&](auto tc) { n2 += abs2(xc[decltype(tc)::value]); });
      const float nrm2 = sumq(n2);
      const float ax02 = abs2(x0);
      const float nx = fsqrt(nrm2);
      const float ax0 = fsqrt(ax02);
      const float iax0 = frsq(ax02);
      const cf e = csel(ax02 > 0.0f, cf{x0.re * iax0, x0.im * iax0}, cf{1.0f, 0.0f});
      const bool refl = nrm2 > 1e-30f;
      const float invn = refl ? frsq(2.0f * nx * (nx + ax0)) : 0.0f;
      if (li == 0) S.b[j + 1] = csel(refl, cf{-nx * e.re, -nx * e.im}, x0);
      const cf ne = nx * e;
      cf ur[NB], uc[NB];
      sfor<sj, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        ur[s] = invn * csel(p + 8 * s == j + 1, xr[s] + ne, xr[s]);
        uc[s] = invn * csel(q + 8 * s == j + 1, xc[s] + ne, xc[s]);
      });
      if (q == 0) {
        sfor<0, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          if constexpr (s < sj) S.m.U[j][p + 8 * s] = cf{0.0f, 0.0f};
          else S.m.U[j][p + 8 * s] = ur[s];
        });
      }
      // p = C u (rows > j); its column-layout copy through LDS gives
      // K = Re(u^H p) as a sum over q (DPP), then q = p - K u in both layouts
      cf pr[NB];
      sfor<sj, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        cf acc = cf{0.0f, 0.0f};
        sfor<sj, NB>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          fma_c(acc, A.v[s][t], uc[t]);
        });
        acc = sumq(acc);
        acc = csel(p + 8 * s > j, acc, cf{0.0f, 0.0f});
        pr[s] = acc;
        if (q == 0) S.qb[buf][p + 8 * s] = acc;
      });
      // phase of the subdiagonal: phi_{j+1} = phi_j b_{j+1} / |b_{j+1}|
      {
        const cf bb = csel(refl, cf{-nx * e.re, -nx * e.im}, x0);
        const float ab2 = abs2(bb);
        const float iab = frsq(ab2);
        ph = csel(ab2 > 0.0f, ph * cf{bb.re * iab, bb.im * iab}, ph);
        if (li == 0) S.phi[j + 1] = ph;
      }
      wsync();
      cf pc[NB];
      float kp = 0.0f;
      sfor<sj, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        pc[t] = S.qb[buf][q + 8 * t];
        kp += cmul(uc[t], pc[t]).re;
      });
      const float Kr = sumq(kp);
      sfor<sj, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const cf qc = pc[t] - Kr * uc[t];
        const cf u2c = 2.0f * uc[t], q2c = 2.0f * qc;
        sfor<sj, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const cf qrs = pr[s] - Kr * ur[s];
          cf x = A.v[s][t];
          fms_cc(x, ur[s], q2c);
          fms_cc(x, qrs, u2c);
          A.v[s][t] = x;
        });
      });
      buf ^= 1;
    }
  });
  // trailing 2 x 2 (or 1 x 1) block, and b[0] = 0
  sfor<0, NB>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      const int i = p + 8 * s, c = q + 8 * t;
      if (i == c && i >= D - 2 && i < D) S.a[i] = A.v[s][t].re;
      if (i == D - 1 && c == D - 2) S.b[i] = A.v[s][t];
    });
  });
  if (li == 0) S.b[0] = cf{0.0f, 0.0f};
  wsync();
  if (D >= 2) {
    const cf bb = S.b[D - 1];
    const float ab2 = abs2(bb);
    const float iab = frsq(ab2);
    ph = csel(ab2 > 0.0f, ph * cf{bb.re * iab, bb.im * iab}, ph);
    if (li == 0) S.phi[D - 1] = ph;
  }
  // the tridiagonal for the eigen part: S.ev[i] = |b_{i+1}|, S.e2[i] = |b_{i+1}|^2
  if (li < DM) {
    const float e2 = (li + 1 < D) ? abs2(S.b[li + 1]) : 0.0f;
    S.e2[li] = e2;
    S.ev[li] = fsqrt(e2);
  }
  wsync();
}

// ---- eigen part of the real tridiagonal (a_i, |b_i|) held in LDS ----------
// Sturm count below x (one x per lane), the recurrence of solver64.hpp::sturm
// with the coefficients read from LDS (broadcast reads, independent of the
// recurrence, so the unrolled loop issues them ahead of it).
template <int DM>
DANSE_DEV int sturm2d(const float* a, const float* e2, int D, float x, float pivmin) {
  int cnt = 0;
  float q = 1.0f;
  sfor<0, DM>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    float qn = a[i] - x;
    if constexpr (i > 0) qn -= e2[i - 1] * frcp(q);
    if (fabsf(qn) <= pivmin) qn = -pivmin;
    const bool on = i < D;
    q = on ? qn : q;
    cnt += (on && q < 0.0f) ? 1 : 0;
  });
  return cnt;
}

// top-R eigenvalues by 64-point multisection (solver64.hpp::top_eigvals)
template <int DM, int RMAX>
DANSE_DEV void top_eigvals2d(const float* a, const float* e2, float ta, float te2, int li, int D, int R,
                             float (&lam)[kRMax], float& tnorm) {
  const bool act = li < D;
  const float e2m = __shfl_up(te2, 1);
  const float em = (li >= 1 && act) ? fsqrt(e2m) : 0.0f;
  const float ep = (li + 1 < D) ? fsqrt(te2) : 0.0f;
  const float lo0 = gmin<64>(act ? ta - em - ep : 3.0e38f);
  const float hi0 = gmax<64>(act ? ta + em + ep : -3.0e38f);
  const float e2max = gmax<64>((li + 1 < D) ? te2 : 0.0f);
  tnorm = gmax<64>(act ? fabsf(ta) + em + ep : 0.0f);
  const float scale = fmaxf(fabsf(lo0), fabsf(hi0));
  const float pivmin = 1.0e-30f * fmaxf(1.0f, e2max);
  float lo = lo0 - (2.0f * 1.2e-7f * scale + pivmin);
  float hi = hi0 + (2.0f * 1.2e-7f * scale + pivmin);
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if (r >= R) return;
    float al = lo, bl = hi;
    const int target = D - r;   // count(x) >= target  <=>  x > lambda_r
    for (int it = 0; it < 5; ++it) {
      const float step = (bl - al) * (1.0f / 65.0f);
      const float x = al + step * (float)(li + 1);
      const int cnt = sturm2d<DM>(a, e2, D, x, pivmin);
      const uint64_t m = __ballot(cnt >= target);
      if (m == 0ull) {
        al = al + step * 64.0f;
      } else {
        const int first = __builtin_ctzll(m);
        const float na = al + step * (float)first;
        bl = al + step * (float)(first + 1);
        al = na;
      }
    }
    lam[r] = 0.5f * (al + bl);
    hi = bl;
  });
}

// Eigenvector x_li of the tridiagonal for eigenvalue lam: two sweeps of
// inverse iteration with partial pivoting (solver64.hpp::tri_eigvec), the
// elimination computed redundantly by every lane from LDS (wave-uniform
// values, no readlane / lane-select chains), the eliminated rows kept in LDS
// for the back substitution.
template <int DM>
DANSE_DEV float tri_eigvec2d(const float* a, const float* ev, float4* fac, float* xs, int li, int D, float lam,
                             float pert, int r, const float (*prev)[DM]) {
  float x = (li < D) ? 1.0f + 0.1f * (float)((li * 7919 + r * 104729) % 13) / 13.0f : 0.0f;
  for (int it = 0; it < 2; ++it) {
    if (it > 0) {
      if (li < 64) xs[li] = x;
      wsync();
    }
    auto rhs = [&](int i) {
      return (it == 0) ? 1.0f + 0.1f * (float)((i * 7919 + r * 104729) % 13) / 13.0f : xs[i];
    };
    float dc = a[0] - lam, duc = ev[0], rc = rhs(0);
    sfor<0, DM - 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if (i + 1 < D) {
        const float dli = ev[i];
        const float d1 = a[i + 1] - lam;
        const float du1 = (i + 2 < D) ? ev[i + 1] : 0.0f;
        const float r1 = rhs(i + 1);
        const bool swap = fabsf(dc) < fabsf(dli);
        const float di = (dc == 0.0f) ? pert : dc;
        const float f1 = dli * frcp(di);
        const float f2 = dc * frcp(dli);
        if (li == 0) fac[i] = swap ? make_float4(dli, d1, du1, r1) : make_float4(di, duc, 0.0f, rc);
        const float ndc = swap ? (duc - f2 * d1) : (d1 - f1 * duc);
        const float nduc = swap ? -f2 * du1 : du1;
        const float nrc = swap ? (rc - f2 * r1) : (r1 - f1 * rc);
        dc = ndc;
        duc = nduc;
        rc = nrc;
      }
    });
    if (li == 0) fac[D - 1] = make_float4(dc, 0.0f, 0.0f, rc);
    wsync();
    float xn1 = 0.0f, xn2 = 0.0f, sol = 0.0f;
    sfor_down<DM, 0>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const float4 fr = fac[i];
      const float acc = fr.w - fr.y * xn1 - fr.z * xn2;
      const float di = (fr.x == 0.0f) ? pert : fr.x;
      const float xi = acc * frcp(di);
      const bool on = i < D;
      sol = (on && li == i) ? xi : sol;
      xn2 = on ? xn1 : xn2;
      xn1 = on ? xi : xn1;
    });
    for (int qq = 0; qq < r; ++qq) {
      const float pq = (li < DM) ? prev[qq][li] : 0.0f;
      const float dot = gsum<64>(pq * sol);
      sol -= dot * pq;
    }
    const float mx0 = gmax<64>(fabsf(sol));
    const float mx = (mx0 > 0.0f) ? mx0 : 1.0f;
    sol *= frcp(mx);
    const float nrm = gsum<64>(sol * sol);
    x = sol * frsq(nrm);
    wsync();   // fac / xs reads before the next sweep rewrites them
  }
  return x;
}

// ---- eigen part, back-transform, x = Li^H v,
// w = sum_r (1 - 1/lambda_r) x_r (x_r^H Rnn e_ref)
template <int NB, int RMAX>
DANSE_DEV cf eigen2d(const Blk<NB>& Lf, LDS2<NB>& S, int li, int D, int R) {
  constexpr int DM = 8 * NB;
  const int p = li >> 3, q = li & 7;
  const bool act = li < D;
  const float ta = act ? S.a[li] : 0.0f;
  const float te2 = (li + 1 < D) ? S.e2[li] : 0.0f;
  float lam[kRMax];
  float tnorm;
  top_eigvals2d<DM, RMAX>(S.a, S.e2, ta, te2, li, D, R, lam, tnorm);
  const float pert = 1.2e-7f * fmaxf(tnorm, 1e-30f);
  const cf gl = S.g[li];
  const cf phl = csel(act, S.phi[act ? li : 0], cf{0.0f, 0.0f});
  cf wc[NB];
  sfor<0, NB>([&](auto tc) { wc[decltype(tc)::value] = cf{0.0f, 0.0f}; });
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (r > 0) {
      if (r >= R) return;
    }
    const float x = tri_eigvec2d<DM>(S.a, S.ev, S.fac, S.xs, li, D, lam[r], pert, r, S.x);
    cf v = x * phl;
    if (r + 1 < R) {
      if (li < DM) S.x[r][li] = x;
      wsync();
    }
    for (int j = D - 3; j >= 0; --j) {
      const cf u = (li < DM ? 1.0f : 0.0f) * S.m.U[j][li < DM ? li : 0];
      const cf sdot = gsum<64>(cmul(u, v));
      fms_c(v, 2.0f * u, sdot);
    }
    const cf sr = gsum<64>(cmul(v, gl));
    // x = Li^H v: x_c = sum_i conj(Li[i][c]) v_i (column layout)
    S.vb[li] = v;
    wsync();
    cf vr[NB];
    sfor<0, NB>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      vr[s] = S.vb[p + 8 * s];
    });
    const float coef = 1.0f - frcp(lam[r]);
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      cf acc = cf{0.0f, 0.0f};
      sfor<t, NB>([&](auto sc) {   // Li[i][c] = 0 for i < c
        constexpr int s = decltype(sc)::value;
        acc = acc + cmul(Lf.v[s][t], vr[s]);
      });
      acc = sump(acc);
      wc[t] = wc[t] + coef * (acc * sr);
    });
    wsync();   // vb reads before the next rank's write
  });
  if (p == 0) {
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      S.wb[q + 8 * t] = wc[t];
    });
  }
  wsync();
  const cf w = S.wb[li];
  return csel(act, w, cf{0.0f, 0.0f});
}

// ---- phase 2: A = Ryy block (float32, destroyed), Lf = Li -> w (lane layout)
template <int NB, int RMAX>
DANSE_DEV cf gevd2d_filter(Blk<NB>& A, const Blk<NB>& Lf, LDS2<NB>& S, int li, int D, int R) {
  congruence2d<NB>(A, Lf, S, li, D);
  tridiag2d<NB>(A, S, li, D);
  return eigen2d<NB, RMAX>(Lf, S, li, D, R);
}

}  // namespace t2d
}  // namespace danse
