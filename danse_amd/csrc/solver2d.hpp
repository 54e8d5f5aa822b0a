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

// lanes per bin and lane-layout vector entries per lane (G = 8: one bin
// per wave, one entry per lane; G = 4: four bins per wave, DM <= 32)
template <int G>
constexpr int bin_lanes() { return G * G; }
template <int NB, int G>
constexpr int vpl() { return (G * NB + G * G - 1) / (G * G); }

template <int NB>
struct BlkD {
  cd v[NB][NB];
};
template <int NB>
struct Blk {
  cf v[NB][NB];
};
DANSE_DEV cd cmulx2(cd a, cd b) { return cd{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
// complex double to / from global memory as two doubles (a struct copy of a
// register-array element becomes a memcpy from its address, which moves the
// whole array to scratch)
DANSE_DEV void st_cd(cd* p, cd v) {
  double* o = reinterpret_cast<double*>(p);
  o[0] = v.re;
  o[1] = v.im;
}
DANSE_DEV cd ld_cd(const cd* p) {
  const double* o = reinterpret_cast<const double*>(p);
  return cd{o[0], o[1]};
}

// LDS of one bin.  The float64 factor phase, the congruence and the float32
// phases never overlap, so their scratch shares one union; inside the
// float32 phases the pivot vectors of the tridiagonalisation, the inverse
// iteration's rows and the layout-change vectors (y staging, back-transform)
// are used one after the other and share a second one.  NB = 5: 16.3 KB per
// wave at G = 8; G = 4: 19.9 KB for the wave's four bins, so a CU holds 8
// waves (2 per SIMD, the VGPR limit) in both.
template <int NB, int G = 8>
struct LDS2 {
  static constexpr int DM = G * NB;
  static constexpr int VL = bin_lanes<G>() * vpl<NB, G>();   // lane-layout vectors
  union {
    struct {                // float64 factor phase (chol2d, trinv2d)
      cd cb64[2][DM];       // pivot column (double-buffered)
      cd rb64[2][DM];       // pivot row
      double invd[DM];      // 1 / L[j][j]
    };
    struct {                // float32 phases (tridiagonalisation .. back-transform)
      union {
        struct {
          cf cb[2][DM];     // pivot column
          cf qb[2][DM];     // row -> column layout transpose of q
        };
        struct {
          float4 fac[DM];   // inverse iteration: eliminated rows (d, du, dl2, rhs)
          float xs[VL];     //                    right-hand side of the next sweep
        };
        struct {
          cf vb[VL];        // lane layout -> row layout (y staging, Li^H v)
          cf wb[VL];        // column layout -> lane layout
        };
      };
      float a[DM];          // tridiagonal: diagonal
      cf b[DM];             //              subdiagonal b[i] = T[i][i-1]
      float e2[DM];         //              |b[i+1]|^2
      float ev[DM];         //              |b[i+1]|
      cf phi[DM];           //              phases phi_i = prod_{k<=i} b_k / |b_k|
      float x[kRMax][DM];   // tridiagonal eigenvectors (Gram-Schmidt, rank > 1)
    };
    struct {                // congruence: one block column of A / block row of Z
      cf cz[G][DM];
    };
  };
  // Li (float32) from the factor to the back-transform, lower triangle packed
  // by columns (ls_col); it never lives in registers, so the float32 phases
  // hold one NB x NB block (the Ryy / C block) instead of two.
  alignas(16) cf Ls[DM * (DM + 1) / 2];   // (16-byte aligned: LDS-DMA destination, kernels_2dc.hpp)
  cf g[VL];           // g = L^H e_ref (lane layout), written by the factor phase
  // Householder vectors u_j (i > j), packed by j (u_row); the warm Lanczos
  // keeps its basis in the first kLz DM entries.  Last member: the lean
  // kernel (kernels_2dc.hpp) allocates the struct up to that basis only.
  cf U[DM * (DM - 1) / 2];
};

// column-packed lower triangle: (i, c), i >= c, column c at c DM - c (c - 1) / 2
template <int DM>
DANSE_DEV int ls_col(int c) { return c * DM - ((c * (c - 1)) >> 1); }
// Li[i][c] from LDS (zero above the diagonal; the load always stays in bounds)
template <int DM>
DANSE_DEV cf ls_get(const cf* Ls, int i, int c) {
  const bool lo = i >= c;
  return csel(lo, Ls[lo ? ls_col<DM>(c) + i - c : 0], cf{0.0f, 0.0f});
}
// Householder vector j, entries i = j + 1 .. DM - 1
template <int DM>
DANSE_DEV int u_row(int j) { return j * (DM - 1) - ((j * (j - 1)) >> 1) - j - 1; }

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
// sum over the G lanes of my row group (lanes G p .. G p + G - 1 of the bin)
template <int G>
DANSE_DEV float sumq(float x) {
  x += dpp_x<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_x<0x4E>(x);    // quad_perm [2,3,0,1]
  if constexpr (G == 8) x += dpp_x<0x141>(x);   // row_half_mirror (quads 0/1 of each half-row)
  return x;
}
template <int G>
DANSE_DEV cf sumq(cf x) { return cf{sumq<G>(x.re), sumq<G>(x.im)}; }
template <int G>
DANSE_DEV double sumq(double x) {
  x += dpp_d<0xB1>(x);
  x += dpp_d<0x4E>(x);
  if constexpr (G == 8) x += dpp_d<0x141>(x);
  return x;
}
template <int G>
DANSE_DEV cd sumq(cd x) { return cd{sumq<G>(x.re), sumq<G>(x.im)}; }
// sum over the G row groups of the bin (lanes q, q + G, ...)
template <int G>
DANSE_DEV float sump(float x) {
  if constexpr (G == 8) {
    // row_ror:8 == xor 8 inside a 16-lane row; the xor-16 and xor-32
    // butterflies by v_permlane16_swap / v_permlane32_swap (VALU, no LDS:
    // with vdst = src = x the two results are x and its partner lane's x, so
    // each sum adds the same two operands as the former ds_bpermute form)
    x += dpp_x<0x128>(x);
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(b[0]) + __uint_as_float(b[1]);
  } else {
    x += dpp_x<0x124>(x);   // row_ror:4
    x += dpp_x<0x128>(x);   // row_ror:8: the four quads of the 16-lane row
  }
  return x;
}
template <int G>
DANSE_DEV cf sump(cf x) { return cf{sump<G>(x.re), sump<G>(x.im)}; }
// value of bin-local lane src (runtime, bin-uniform): v_readlane when the bin
// is the whole wave, a bpermute inside the 16-lane row otherwise
template <int G>
DANSE_DEV double bin_rld(double x, int src) {
  if constexpr (G == 8) return big::rld(x, src);
  else return __shfl(x, (__lane_id() & ~15) | src);
}

// ---- float64 Cholesky, in place: M = L (lower, upper part zeroed) -----------
template <int NB, int G = 8>
DANSE_DEV bool chol2d(BlkD<NB>& M, LDS2<NB, G>& S, int li, int D) {
  const int p = li / G, q = li % G;
  bool ok = true;
  int buf = 0;
  sfor<0, NB>([&](auto sjc) {
    constexpr int sj = decltype(sjc)::value;
    for (int rj = 0; rj < G; ++rj) {
      const int j = G * sj + rj;
      if (j >= D) break;
      const double p0 = bin_rld<G>(M.v[sj][sj].re, (G + 1) * rj);   // lane (rj, rj)
      ok = ok && (p0 > 1e-300);
      const double piv = p0 > 1e-300 ? p0 : 1e-300;
      const double inv = lane::rsqrt64(piv);
      if (li == 0) S.invd[j] = inv;
      if (q == rj) {
        sfor<sj, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const int i = p + G * s;
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
        rv[s] = S.cb64[buf][p + G * s];
        cv[s] = S.cb64[buf][q + G * s];
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
      if (p + G * s < q + G * t) M.v[s][t] = cd{0.0, 0.0};
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
template <int NB, int G = 8>
DANSE_DEV void trinv2d(BlkD<NB>& M, LDS2<NB, G>& S, int li, int D) {
  const int p = li / G, q = li % G;
  int buf = 0;
  sfor<0, NB>([&](auto skc) {
    constexpr int sk = decltype(skc)::value;
    for (int rk = 0; rk < G; ++rk) {
      const int k = G * sk + rk;
      if (k >= D) break;
      const double ik = S.invd[k];
      if (p == rk) {
        sfor<0, NB>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          const int c = q + G * t;
          const cd v = csel(c == k, cd{ik, 0.0}, csel(c < k, ik * M.v[sk][t], cd{0.0, 0.0}));
          M.v[sk][t] = v;
          S.rb64[buf][c] = v;
        });
      }
      if (q == rk) {
        sfor<sk, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const int i = p + G * s;
          S.cb64[buf][i] = csel(i > k, M.v[s][sk], cd{0.0, 0.0});
        });
      }
      wsync();
      cd lc[NB], xr[NB];
      sfor<sk, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        lc[s] = S.cb64[buf][p + G * s];
      });
      sfor<0, sk + 1>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        xr[t] = S.rb64[buf][q + G * t];
      });
      sfor<sk, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        const int i = p + G * s;
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

// ---- float64 factor record (kernels.hpp li_updatable): Li packed by
// columns (ls_col order) + g64 = conj(L[ref][:]) = L^H e_ref, DM entries
template <int NB, int G = 8>
constexpr int l64_record() { return G * NB * (G * NB + 1) / 2 + G * NB; }
template <int NB, int G = 8>
DANSE_DEV void l64_store2d(const BlkD<NB>& M, cd* l64, int li) {
  constexpr int DM = G * NB;
  const int p = li / G, q = li % G;
  sfor<0, NB>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    const int c = q + G * t;
    const int col = ls_col<DM>(c) - c;
    sfor<t, NB>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      const int i = p + G * s;
      if (s > t || i >= c) st_cd(l64 + col + i, M.v[s][t]);
    });
  });
}
// scans over the lanes of a bin (float64): inclusive prefix over the row
// groups p' <= p (lanes q + G p'), and the suffix over q' >= q inside the row
// group
template <int G>
DANSE_DEV double scan_p(double x, int p) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const double u = __shfl_up(x, o * G, G * G);
    if (p >= o) x += u;
  }
  return x;
}
template <int G>
DANSE_DEV double scan_q_down(double x, int q) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const double u = __shfl_down(x, o, G);
    if (q + o < G) x += u;
  }
  return x;
}

// ---- rank-one update of the float64 factor (a noise frame one solve after
// the last factorisation): Rnn' = beta Rnn + cy y y^H.  With L the Cholesky
// factor of Rnn, Li = L^-1, p = Li y and alpha = cy / beta,
//   L' = sqrt(beta) L Mf,   Mf Mf^H = I + alpha p p^H,
// whose factor has closed forms (t_0 = 1, t_(i+1) = t_i + alpha |p_i|^2):
//   Mf[c][c] = sqrt(t_(c+1) / t_c),  Mf[k][c] = alpha p_k conj(p_c) / sqrt(t_c t_(c+1))  (k > c),
//   Mf^-1[i][i] = sqrt(t_i / t_(i+1)),  Mf^-1[i][k] = -alpha p_i conj(p_k) / sqrt(t_i t_(i+1))  (k < i), so
//   Li'[i][c] = (sqrt(t_i / t_(i+1)) Li[i][c] - alpha p_i / sqrt(t_i t_(i+1)) P[i][c]) / sqrt(beta),
//     P[i][c] = sum_(k < i) conj(p_k) Li[k][c]          (a column prefix sum)
//   L'[ref][c] = sqrt(beta) (sqrt(t_(c+1) / t_c) L[ref][c]
//                + alpha conj(p_c) / sqrt(t_c t_(c+1)) sum_(c < k <= ref) L[ref][k] p_k)
// O(D^2) with running sums (LDS, shuffles), instead of the O(D^3) Cholesky and
// inverse (alpha > 0: an update, the stable direction).  The record l64 holds
// Li and g64 = conj(L[ref][:]) on entry and (store) this frame's on exit;
// Li' (float32) and g go to S.Ls / S.g as gevd2d_factor leaves them.
template <int NB, int G = 8>
DANSE_DEV bool li_rank1_2d(LDS2<NB, G>& S, int li, const cf (&yc)[NB], double beta, double cy, cd* l64,
                           bool store) {
  constexpr int DM = G * NB, L = bin_lanes<G>(), V = vpl<NB, G>();
  const int p = li / G, q = li % G;
  const double alpha = cy / beta;
  double* av = S.invd;    // a_i = alpha |p_i|^2
  cd* pv = S.rb64[0];     // p_i
  // Li entry (p + G sb, q + G t) of the record (zero above the diagonal):
  // the blocks are streamed from the record (L2) as they are needed, never
  // all held in registers (the register budget of the 2 waves / SIMD kernel)
  auto li_at = [&](int sb, int t) -> cd {
    const int i = p + G * sb, c = q + G * t;
    const bool lo = sb > t || (sb == t && i >= c);
    return csel(lo, ld_cd(l64 + (lo ? ls_col<DM>(c) - c + i : 0)), cd{0.0, 0.0});
  };
  // p_i (to LDS: pv[i], and a_i in av[i])
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    cd acc = cd{0.0, 0.0};
    sfor<0, sb + 1>([&](auto tc) { fma_c(acc, li_at(sb, decltype(tc)::value), cdk(yc[decltype(tc)::value])); });
    const cd pi = sumq<G>(acc);
    if (q == 0) {
      av[p + G * sb] = alpha * (pi.re * pi.re + pi.im * pi.im);
      pv[p + G * sb] = pi;
    }
  });
  wsync();
  // t_i = 1 + sum_(k < i) a_k (exclusive prefix) of this lane's rows, in the
  // row order i = p + G s: a scan over the row groups plus the carry over the
  // block rows
  double tlo[NB];
  {
    double carry = 1.0;
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      const double a = av[p + G * sb];
      const double inc = scan_p<G>(a, p);
      tlo[sb] = carry + (inc - a);
      carry += __shfl(inc, (G - 1) * G + q, G * G);
    });
  }
  // Li' block row by block row: P[i][c] = sum_(k < i) conj(p_k) Li[k][c],
  // a prefix over the row groups of the block row (shuffles) plus the earlier
  // block rows' column sums carried in carP
  const double rb = 1.0 / sqrt(beta);
  {
    cd carP[NB];
    sfor<0, NB>([&](auto tc) { carP[decltype(tc)::value] = cd{0.0, 0.0}; });
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      const cd ps = pv[p + G * sb];
      const double thi = tlo[sb] + av[p + G * sb];
      const double dd = sqrt(tlo[sb] / thi);
      const cd pe = (alpha / sqrt(tlo[sb] * thi)) * ps;
      // the block row's old entries first (one round trip, hold()): the
      // record stores below would otherwise keep each load behind the
      // previous entry's store
      cd mrow[sb + 1];
      sfor<0, sb + 1>([&](auto tc) { mrow[decltype(tc)::value] = li_at(sb, decltype(tc)::value); });
      hold(mrow);
      sfor<0, sb + 1>([&](auto tc) {   // (blocks right of the diagonal block are zero)
        constexpr int t = decltype(tc)::value;
        const int c = q + G * t;
        const cd m = mrow[t];
        const cd u = cd{ps.re * m.re + ps.im * m.im, ps.re * m.im - ps.im * m.re};   // conj(p_i) Li[i][c]
        // prefix over the row groups of this block row (lanes q + G p', p' < p)
        const double ire = scan_p<G>(u.re, p), iim = scan_p<G>(u.im, p);
        const double tre = __shfl(ire, (G - 1) * G + q, G * G), tim = __shfl(iim, (G - 1) * G + q, G * G);
        const cd ex = cd{carP[t].re + (ire - u.re), carP[t].im + (iim - u.im)};
        carP[t] = cd{carP[t].re + tre, carP[t].im + tim};
        cd x = dd * m;
        fms_c(x, pe, ex);
        x = rb * x;
        // float32 Li where gevd2d_factor leaves it (S.Ls), float64 record
        // (this block row's old entries were all read above)
        const int i = p + G * sb;
        if (sb > t || i >= c) {
          S.Ls[ls_col<DM>(c) - c + i] = cfk(x);
          if (store) st_cd(l64 + ls_col<DM>(c) - c + i, x);
        }
      });
    });
  }
  const double tN = tlo[NB - 1] + av[p + G * (NB - 1)];
  // row ref of L (its record entries are read and rewritten here):
  // L'[ref][c] = sqrt(beta) (sqrt(t_(c+1) / t_c) L[ref][c] + alpha conj(p_c) / sqrt(t_c t_(c+1)) sum_(k > c) L[ref][k] p_k)
  // column c = q + G t: t_c, t_(c+1) from row group q (block t), the suffix
  // sum over the columns by a scan inside the row group plus the carry over
  // the blocks (descending)
  {
    const double sbeta = sqrt(beta);
    double czr = 0.0, czi = 0.0;
    cd lrv[NB];   // L[ref][q + G t], all read before the first store (hold())
    sfor<0, NB>([&](auto tc) { lrv[decltype(tc)::value] = ld_cd(l64 + DM * (DM + 1) / 2 + q + G * decltype(tc)::value); });
    hold(lrv);
    sfor_down<NB, 0>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      const int c = q + G * t;
      const double t0 = __shfl(tlo[t], G * q, G * G);
      const double t1 = t0 + av[c];
      const cd pc = pv[c];
      const cd lr = conjg(lrv[t]);   // L[ref][c]
      const cd z = cmulx2(lr, pc);
      const double sre = scan_q_down<G>(z.re, q), sim = scan_q_down<G>(z.im, q);
      const cd sfx = cd{czr + (sre - z.re), czi + (sim - z.im)};   // sum_(k > c) L[ref][k] p_k
      czr += __shfl(sre, 0, G);
      czi += __shfl(sim, 0, G);
      cd x = sqrt(t1 / t0) * lr;
      fma_c(x, (alpha / sqrt(t0 * t1)) * conjg(pc), sfx);
      const cd g = conjg(sbeta * x);
      if (p == 0) {
        S.g[c] = cfk(g);
        if (store) st_cd(l64 + DM * (DM + 1) / 2 + c, g);
      }
    });
    sfor<0, V>([&](auto vc) {
      const int i = li + L * decltype(vc)::value;
      if (i >= DM) S.g[i] = cf{0.0f, 0.0f};
    });
  }
  wsync();
  return tN > 0.0 && tN < 1e300;
}

// ---- phase 1: Rnn block (float64, destroyed) -> Li (float32, S.Ls), g in LDS
template <int NB, int G = 8>
DANSE_DEV bool gevd2d_factor(BlkD<NB>& M, LDS2<NB, G>& S, int li, int D, int ref, cd* l64 = nullptr) {
  constexpr int DM = G * NB;
  const int p = li / G, q = li % G;
  constexpr int L = bin_lanes<G>(), V = vpl<NB, G>();
  const bool ok = chol2d<NB, G>(M, S, li, D);
  // g = L^H e_ref: g_c = conj(L[ref][c]) (c <= ref; the upper part is zero)
  sfor<0, V>([&](auto vc) { S.g[li + L * decltype(vc)::value] = cf{0.0f, 0.0f}; });
  wsync();
  {
    // row ref of L: block row ref / G (a select chain over the static
    // block index, no branches) on the row group p == ref & 7
    const int sr = ref / G;
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      cd v = M.v[0][t];
      sfor<1, NB>([&](auto sc) { v = csel(decltype(sc)::value == sr, M.v[decltype(sc)::value][t], v); });
      if (p == (ref % G)) {
        S.g[q + G * t] = conjg(cfk(v));
        if (l64) st_cd(l64 + DM * (DM + 1) / 2 + q + G * t, conjg(v));
      }
    });
  }
  trinv2d<NB, G>(M, S, li, D);
  if (l64) {
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      const int c = q + G * t;
      const int col = ls_col<DM>(c) - c;
      sfor<t, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        const int i = p + G * s;
        if (s > t || i >= c) st_cd(l64 + col + i, M.v[s][t]);
      });
    });
  }
  sfor<0, NB>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    const int c = q + G * t;
    const int col = ls_col<DM>(c) - c;
    sfor<t, NB>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      const int i = p + G * s;
      if (s > t || i >= c) S.Ls[col + i] = cfk(M.v[s][t]);
    });
  });
  wsync();
  return ok;
}

// factor cache (kernels.hpp li_reusable): S.Ls and g as one contiguous
// record per bin (li_record entries), copied with coalesced stores / loads
template <int NB, int G = 8>
constexpr int li_record() { return G * NB * (G * NB + 1) / 2 + bin_lanes<G>() * vpl<NB, G>(); }
template <int NB, int G = 8>
DANSE_DEV void li_store2d(const LDS2<NB, G>& S, cf* liC, int li) {
  constexpr int NL = G * NB * (G * NB + 1) / 2, L = bin_lanes<G>();
  for (int i = li; i < NL; i += L) liC[i] = S.Ls[i];
  sfor<0, vpl<NB, G>()>([&](auto vc) { liC[NL + li + L * decltype(vc)::value] = S.g[li + L * decltype(vc)::value]; });
}
template <int NB, int G = 8>
DANSE_DEV void li_load2d(LDS2<NB, G>& S, const cf* liC, int li) {
  constexpr int NL = G * NB * (G * NB + 1) / 2, L = bin_lanes<G>();
  for (int i = li; i < NL; i += L) S.Ls[i] = liC[i];
  sfor<0, vpl<NB, G>()>([&](auto vc) { S.g[li + L * decltype(vc)::value] = liC[NL + li + L * decltype(vc)::value]; });
  wsync();
}

// ---- C = Li A Li^H in place of A (float32); Li staged in LDS ---------------
template <int NB, int G = 8>
DANSE_DEV void congruence2d(Blk<NB>& A, LDS2<NB, G>& S, int li, int D) {
  constexpr int DM = G * NB;
  const int p = li / G, q = li % G;
  // Z = A Li^H: Z[i][c] = sum_k A[i][k] conj(Li[c][k]), Li[c][k] = 0 for k > c.
  // scipy.linalg.eigh reads the lower triangle, so A[i][k] = conj(A[k][i])
  // for i < k (the SCMs are Hermitian except for the random init's residue).
  // Block column sk of that Hermitian completion is staged in S.cz: entry
  // (i, k = 8 sk + r) comes from lane (p, r) (i >= k) or, mirrored, from
  // lane (r, q) (i < k); one LDS write pass per block, one read per k and
  // block row instead of two bpermutes.
  Blk<NB> Z;
  sfor<0, NB>([&](auto sc) {
    sfor<0, NB>([&](auto tc) { Z.v[decltype(sc)::value][decltype(tc)::value] = cf{0.0f, 0.0f}; });
  });
  sfor<0, NB>([&](auto skc) {
    constexpr int sk = decltype(skc)::value;
    if (G * sk >= D) return;
    wsync();   // the previous block's reads before this block's writes
    sfor<0, NB>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      const int i = p + G * s;
      if (i >= G * sk + q) S.cz[q][i] = A.v[s][sk];          // (i, 8 sk + q), lower
      const int c = q + G * s;
      if (c < G * sk + p) S.cz[p][c] = conjg(A.v[sk][s]);    // (c, 8 sk + p) from (8 sk + p, c)
    });
    wsync();
    // (pivots unrolled at compile time: k is a constant and the next
    // pivot's LDS reads can go out under this one's multiply-adds; the
    // padding pivots k >= D add exact zeros -- Li and A are zero there)
    sfor<0, G>([&](auto rkc) {
      constexpr int rk = decltype(rkc)::value;
      constexpr int k = G * sk + rk;
      cf ak[NB], lc[NB];
      sfor<0, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        ak[s] = S.cz[rk][p + G * s];
      });
      sfor<sk, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        lc[t] = ls_get<DM>(S.Ls, q + G * t, k);
      });
      sfor<0, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        sfor<sk, NB>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          pk_fma_cc(Z.v[s][t], ak[s], lc[t]);
        });
      });
    });
  });
  // C = Li Z: C[i][c] = sum_k Li[i][k] Z[k][c], Li[i][k] = 0 for k > i  (into A);
  // block row sk of Z staged in S.cz the same way
  sfor<0, NB>([&](auto sc) {
    sfor<0, NB>([&](auto tc) { A.v[decltype(sc)::value][decltype(tc)::value] = cf{0.0f, 0.0f}; });
  });
  sfor<0, NB>([&](auto skc) {
    constexpr int sk = decltype(skc)::value;
    if (G * sk >= D) return;
    wsync();
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      S.cz[p][q + G * t] = Z.v[sk][t];
    });
    wsync();
    sfor<0, G>([&](auto rkc) {
      constexpr int rk = decltype(rkc)::value;
      constexpr int k = G * sk + rk;
      cf zk[NB], lr[NB];
      sfor<0, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        zk[t] = S.cz[rk][q + G * t];
      });
      sfor<sk, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        lr[s] = ls_get<DM>(S.Ls, p + G * s, k);
      });
      sfor<sk, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        sfor<0, NB>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          pk_fma_c(A.v[s][t], lr[s], zk[t]);
        });
      });
    });
  });
  sfor<0, NB>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (p == q) A.v[s][s].im = 0.0f;
  });
}

// ---- Householder tridiagonalisation of the Hermitian block A (destroyed):
// diagonal -> S.a, subdiagonal -> S.b, reflectors -> S.U (u_row)
template <int NB, int G = 8>
DANSE_DEV void tridiag2d(Blk<NB>& A, LDS2<NB, G>& S, int li, int D) {
  constexpr int DM = G * NB;
  const int p = li / G, q = li % G;
  int buf = 0;
  cf ph = cf{1.0f, 0.0f};   // phi_j (wave-uniform)
  if (li == 0) S.phi[0] = ph;
  sfor<0, NB>([&](auto sjc) {
    constexpr int sj = decltype(sjc)::value;
    for (int rj = 0; rj < G; ++rj) {
      const int j = G * sj + rj;
      if (j + 2 >= D) break;
      if (q == rj) {
        sfor<sj, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const int i = p + G * s;
          S.cb[buf][i] = csel(i > j, A.v[s][sj], cf{0.0f, 0.0f});
        });
        if (p == rj) S.a[j] = A.v[sj][sj].re;
      }
      wsync();
      cf xr[NB], xc[NB];
      sfor<sj, NB>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        xr[s] = S.cb[buf][p + G * s];
        xc[s] = S.cb[buf][q + G * s];
      });
      const cf x0 = S.cb[buf][j + 1];
      float n2 = 0.0f;
      sfor<sj, NB>([&](auto tc) { n2 += abs2(xc[decltype(tc)::value]); });
      const float nrm2 = sumq<G>(n2);
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
        ur[s] = invn * csel(p + G * s == j + 1, xr[s] + ne, xr[s]);
        uc[s] = invn * csel(q + G * s == j + 1, xc[s] + ne, xc[s]);
      });
      if (q == 0) {
        const int ub = u_row<DM>(j);
        sfor<sj, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const int i = p + G * s;
          if (i > j) S.U[ub + i] = ur[s];
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
          pk_fma_c(acc, A.v[s][t], uc[t]);
        });
        acc = sumq<G>(acc);
        acc = csel(p + G * s > j, acc, cf{0.0f, 0.0f});
        pr[s] = acc;
        if (q == 0) S.qb[buf][p + G * s] = acc;
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
        pc[t] = S.qb[buf][q + G * t];
        kp += cmul(uc[t], pc[t]).re;
      });
      const float Kr = sumq<G>(kp);
      sfor<sj, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const cf qc = pc[t] - Kr * uc[t];
        const cf u2c = 2.0f * uc[t], q2c = 2.0f * qc;
        sfor<sj, NB>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const cf qrs = pr[s] - Kr * ur[s];
          cf x = A.v[s][t];
          pk_fms_cc(x, ur[s], q2c);
          pk_fms_cc(x, qrs, u2c);
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
      const int i = p + G * s, c = q + G * t;
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
  sfor<0, vpl<NB, G>()>([&](auto vc) {
    const int i = li + bin_lanes<G>() * decltype(vc)::value;
    if (i < DM) {
      const float e2 = (i + 1 < D) ? abs2(S.b[i + 1]) : 0.0f;
      S.e2[i] = e2;
      S.ev[i] = fsqrt(e2);
    }
  });
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

// top-R eigenvalues by (L)-point multisection over the bin's L lanes
// (solver64.hpp::top_eigvals): 5 rounds of 64 points (G = 8), 8 rounds of
// 16 points (G = 4); lane li holds the tridiagonal entries li + L v
template <int DM, int RMAX, int G>
DANSE_DEV void top_eigvals2d(const float* a, const float* e2, int li, int D, int R, float (&lam)[kRMax],
                             float& tnorm) {
  constexpr int L = bin_lanes<G>(), V = (DM + L - 1) / L;
  float lo1 = 3.0e38f, hi1 = -3.0e38f, e2m1 = 0.0f, tn1 = 0.0f;
  sfor<0, V>([&](auto vc) {
    const int i = li + L * decltype(vc)::value;
    const bool act = i < D;
    const float ta = act ? a[i] : 0.0f;
    const float te2 = (i + 1 < D) ? e2[i] : 0.0f;
    const float em = (i >= 1 && act) ? fsqrt(e2[i >= 1 ? i - 1 : 0]) : 0.0f;
    const float ep = (i + 1 < D) ? fsqrt(te2) : 0.0f;
    lo1 = fminf(lo1, act ? ta - em - ep : 3.0e38f);
    hi1 = fmaxf(hi1, act ? ta + em + ep : -3.0e38f);
    e2m1 = fmaxf(e2m1, (i + 1 < D) ? te2 : 0.0f);
    tn1 = fmaxf(tn1, act ? fabsf(ta) + em + ep : 0.0f);
  });
  const float lo0 = gmin<L>(lo1);
  const float hi0 = gmax<L>(hi1);
  const float e2max = gmax<L>(e2m1);
  tnorm = gmax<L>(tn1);
  const float scale = fmaxf(fabsf(lo0), fabsf(hi0));
  const float pivmin = 1.0e-30f * fmaxf(1.0f, e2max);
  float lo = lo0 - (2.0f * 1.2e-7f * scale + pivmin);
  float hi = hi0 + (2.0f * 1.2e-7f * scale + pivmin);
  constexpr int kRounds = (G == 8) ? 5 : 8;
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if (r >= R) return;
    float al = lo, bl = hi;
    const int target = D - r;   // count(x) >= target  <=>  x > lambda_r
    for (int it = 0; it < kRounds; ++it) {
      const float step = (bl - al) * (1.0f / (float)(L + 1));
      const float x = al + step * (float)(li + 1);
      const int cnt = sturm2d<DM>(a, e2, D, x, pivmin);
      const uint64_t m = gballot<L>(cnt >= target);
      if (m == 0ull) {
        al = al + step * (float)L;
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

// Eigenvector of the tridiagonal for eigenvalue lam (entries li + L v of
// lane li): two sweeps of inverse iteration with partial pivoting
// (solver64.hpp::tri_eigvec), the elimination computed redundantly by every
// lane from LDS (bin-uniform values, no readlane / lane-select chains), the
// eliminated rows kept in LDS for the back substitution.
template <int DM, int G>
DANSE_DEV void tri_eigvec2d(const float* a, const float* ev, float4* fac, float* xs, int li, int D, float lam,
                            float pert, int r, const float (*prev)[DM], float (&x)[(DM + G * G - 1) / (G * G)]) {
  constexpr int L = bin_lanes<G>(), V = (DM + L - 1) / L;
  sfor<0, V>([&](auto vc) {
    const int i = li + L * decltype(vc)::value;
    x[decltype(vc)::value] = (i < D) ? 1.0f + 0.1f * (float)((i * 7919 + r * 104729) % 13) / 13.0f : 0.0f;
  });
  for (int it = 0; it < 2; ++it) {
    if (it > 0) {
      sfor<0, V>([&](auto vc) { xs[li + L * decltype(vc)::value] = x[decltype(vc)::value]; });
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
    float xn1 = 0.0f, xn2 = 0.0f, sol[V];
    sfor<0, V>([&](auto vc) { sol[decltype(vc)::value] = 0.0f; });
    sfor_down<DM, 0>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const float4 fr = fac[i];
      const float acc = fr.w - fr.y * xn1 - fr.z * xn2;
      const float di = (fr.x == 0.0f) ? pert : fr.x;
      const float xi = acc * frcp(di);
      const bool on = i < D;
      sfor<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        sol[v] = (on && li + L * v == i) ? xi : sol[v];
      });
      xn2 = on ? xn1 : xn2;
      xn1 = on ? xi : xn1;
    });
    for (int qq = 0; qq < r; ++qq) {
      float pq[V], dp = 0.0f;
      sfor<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        const int i = li + L * v;
        pq[v] = (i < DM) ? prev[qq][i < DM ? i : 0] : 0.0f;
        dp = (v == 0) ? pq[v] * sol[v] : dp + pq[v] * sol[v];
      });
      const float dot = gsum<L>(dp);
      sfor<0, V>([&](auto vc) { sol[decltype(vc)::value] -= dot * pq[decltype(vc)::value]; });
    }
    float am = 0.0f;
    sfor<0, V>([&](auto vc) { am = (decltype(vc)::value == 0) ? fabsf(sol[0]) : fmaxf(am, fabsf(sol[decltype(vc)::value])); });
    const float mx0 = gmax<L>(am);
    const float mx = (mx0 > 0.0f) ? mx0 : 1.0f;
    float n2 = 0.0f;
    sfor<0, V>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      sol[v] *= frcp(mx);
      n2 = (v == 0) ? sol[v] * sol[v] : n2 + sol[v] * sol[v];
    });
    const float nrm = gsum<L>(n2);
    sfor<0, V>([&](auto vc) { x[decltype(vc)::value] = sol[decltype(vc)::value] * frsq(nrm); });
    wsync();   // fac / xs reads before the next sweep rewrites them
  }
}

// ---- eigen part, back-transform, x = Li^H v,
// w = sum_r (1 - 1/lambda_r) x_r (x_r^H Rnn e_ref); w[v] = entry li + L v
template <int NB, int RMAX, int G = 8>
DANSE_DEV void eigen2d(LDS2<NB, G>& S, int li, int D, int R, cf (&w)[vpl<NB, G>()], cf* vOut = nullptr,
                       bool store = false) {
  constexpr int DM = G * NB, L = bin_lanes<G>(), V = vpl<NB, G>();
  const int p = li / G, q = li % G;
  float lam[kRMax];
  float tnorm;
  top_eigvals2d<DM, RMAX, G>(S.a, S.e2, li, D, R, lam, tnorm);
  const float pert = 1.2e-7f * fmaxf(tnorm, 1e-30f);
  cf gl[V], phl[V];
  sfor<0, V>([&](auto vc) {
    constexpr int v = decltype(vc)::value;
    const int i = li + L * v;
    const bool act = i < D;
    gl[v] = S.g[i];
    phl[v] = csel(act, S.phi[act ? i : 0], cf{0.0f, 0.0f});
  });
  cf wc[NB];
  sfor<0, NB>([&](auto tc) { wc[decltype(tc)::value] = cf{0.0f, 0.0f}; });
  sfor<0, RMAX>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (r > 0) {
      if (r >= R) return;
    }
    float x[V];
    tri_eigvec2d<DM, G>(S.a, S.ev, S.fac, S.xs, li, D, lam[r], pert, r, S.x, x);
    cf vv[V];
    sfor<0, V>([&](auto vc) { vv[decltype(vc)::value] = x[decltype(vc)::value] * phl[decltype(vc)::value]; });
    if (r + 1 < R) {
      sfor<0, V>([&](auto vc) {
        const int i = li + L * decltype(vc)::value;
        if (i < DM) S.x[r][i] = x[decltype(vc)::value];
      });
      wsync();
    }
    for (int j = D - 3; j >= 0; --j) {
      cf u[V], sd;
      sfor<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        const int i = li + L * v;
        const bool in = i > j && i < DM;
        u[v] = csel(in, S.U[in ? u_row<DM>(j) + i : 0], cf{0.0f, 0.0f});
        const cf t = cmul(u[v], vv[v]);
        sd = (v == 0) ? t : sd + t;
      });
      const cf sdot = gsum<L>(sd);
      sfor<0, V>([&](auto vc) { fms_c(vv[decltype(vc)::value], 2.0f * u[decltype(vc)::value], sdot); });
    }
    if (r == 0 && vOut && store) {
      // the eigenvector of C: the next frame's Lanczos start (lanczos2d)
      sfor<0, V>([&](auto vc) {
        const int i = li + L * decltype(vc)::value;
        if (i < DM) vOut[i] = (i < D) ? vv[decltype(vc)::value] : cf{0.0f, 0.0f};
      });
    }
    cf sg;
    sfor<0, V>([&](auto vc) {
      const cf t = cmul(vv[decltype(vc)::value], gl[decltype(vc)::value]);
      sg = (decltype(vc)::value == 0) ? t : sg + t;
    });
    const cf sr = gsum<L>(sg);
    // x = Li^H v: x_c = sum_i conj(Li[i][c]) v_i (column layout)
    sfor<0, V>([&](auto vc) {
      const int i = li + L * decltype(vc)::value;
      if (i < DM) S.vb[i] = vv[decltype(vc)::value];
    });
    wsync();
    cf vr[NB];
    sfor<0, NB>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      vr[s] = S.vb[p + G * s];
    });
    const float coef = 1.0f - frcp(lam[r]);
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      cf acc = cf{0.0f, 0.0f};
      sfor<t, NB>([&](auto sc) {   // Li[i][c] = 0 for i < c
        constexpr int s = decltype(sc)::value;
        acc = acc + cmul(ls_get<DM>(S.Ls, p + G * s, q + G * t), vr[s]);
      });
      acc = sump<G>(acc);
      wc[t] = wc[t] + coef * (acc * sr);
    });
    wsync();   // vb reads before the next rank's write
  });
  if (p == 0) {
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      S.wb[q + G * t] = wc[t];
    });
  }
  wsync();
  sfor<0, V>([&](auto vc) {
    const int i = li + L * decltype(vc)::value;
    w[decltype(vc)::value] = (i < D) ? S.wb[i < D ? i : 0] : cf{0.0f, 0.0f};
  });
}

// ---- warm-started Lanczos for the top eigenpair (rank-1 GEVD) ------------
// The SCMs move by a factor (1 - beta) ~ 2 % per frame, so the previous
// frame's eigenvector of C (kept per bin, eigen2d / this function) is a close
// start: kLz<DM>() Lanczos steps on C (one block matvec each, the vector moved
// between the row and column layouts through LDS, one reorthogonalisation
// pass against the stored basis), the top Ritz pair of the small tridiagonal
// by the multisection / inverse iteration of the full path, and the Lanczos
// residual |beta_m s_m| as the acceptance test.  Replaces the D-step
// Householder tridiagonalisation and the D-point eigen part (the bulk of the
// per-bin instruction count) when it converges; the caller
// falls back to them otherwise.  Accuracy: the residual bound kLzTol theta is
// a few float32 roundings of ||C||, the floor the Householder path reaches.
template <int DM>
constexpr int kLz() { return (DM - 1) / 2 < 8 ? (DM - 1) / 2 : 8; }
// reorthogonalisation of each Lanczos step: 1 = one classical Gram-Schmidt
// pass against the whole basis; 0 = against the last two basis vectors only
// (the three-term recurrence; A/B builds)
#ifndef DANSE_LZ_FULL_REORTH
#define DANSE_LZ_FULL_REORTH 1
#endif
template <int k>
constexpr int lz_j0() { return (DANSE_LZ_FULL_REORTH || k < 1) ? 0 : k - 1; }
constexpr float kLzTol = 3.0e-6f;
constexpr float kLzBreak = 1.0e-6f;   // first-step breakdown test (relative to theta)

// true (wave-uniform) if every bin of the wave converged: then vv (lane
// layout) is the unit eigenvector of C and lam1 its eigenvalue
template <int NB, int G = 8, int M = kLz<G * NB>()>
DANSE_DEV bool lanczos2d(const Blk<NB>& A, LDS2<NB, G>& S, int li, int D, const cf* vIn, cf (&vv)[vpl<NB, G>()],
                         float& lam1, bool& warm) {
  constexpr int DM = G * NB, L = bin_lanes<G>(), V = vpl<NB, G>();
  static_assert(M * DM <= DM * (DM - 1) / 2, "the Lanczos basis lives in the reflector space");
  const int p = li / G, q = li % G;
  cf* Q = S.U;   // [M][DM] basis vectors (the Householder vectors' space: unused on this path)
  wsync();       // the congruence's staging reads (S.cz aliases S.qb / S.a) before the writes below
  // start vector, column layout (entries q + G t), unit norm
  cf vc[NB];
  float n0 = 0.0f;
  sfor<0, NB>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    const int i = q + G * t;
    vc[t] = (i < D) ? vIn[i] : cf{0.0f, 0.0f};
    n0 += abs2(vc[t]);
  });
  n0 = sumq<G>(n0);
  bool ok = n0 > 1e-30f && n0 < 1e30f;
  warm = __ballot(n0 > 1e-30f) != 0ull;   // (a bin's first solve has no start vector: a cold solve)
  const float s0 = ok ? frsq(n0) : 0.0f;
  sfor<0, NB>([&](auto tc) { vc[decltype(tc)::value] = s0 * vc[decltype(tc)::value]; });
  if (p == 0) sfor<0, NB>([&](auto tc) { Q[q + G * decltype(tc)::value] = vc[decltype(tc)::value]; });
  float blast = 0.0f, b0 = 0.0f;
  // largest diagonal entry of C: a lower bound of lambda_1 (the Rayleigh
  // quotient of a unit vector), checked against the Ritz value below
  float dmax1 = -3.0e38f;
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    if (p == q && p + G * sb < D) dmax1 = fmaxf(dmax1, A.v[sb][sb].re);
  });
  const float dmax = gmax<L>(dmax1);
  // k = 0 .. M - 1, unrolled (the orthogonalisation's loops get static bounds)
  sfor<0, M>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    // w = C v: row-layout partial sums over the row group, then the column
    // layout through LDS
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      cf acc = cf{0.0f, 0.0f};
      sfor<0, NB>([&](auto tc) { pk_fma_c(acc, A.v[sb][decltype(tc)::value], vc[decltype(tc)::value]); });
      acc = sumq<G>(acc);
      if (q == 0) S.qb[k & 1][p + G * sb] = acc;
    });
    wsync();
    cf wc[NB];
    sfor<0, NB>([&](auto tc) { wc[decltype(tc)::value] = S.qb[k & 1][q + G * decltype(tc)::value]; });
    // one classical Gram-Schmidt pass against the basis Q_0 .. Q_k: the
    // coefficients are independent (one reduction each, side by side);
    // h_k is the Lanczos alpha_k, h_(k-1) its beta_(k-1)
    cf h[k + 1];
    constexpr int j0 = lz_j0<k>();
    sfor<j0, k + 1>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      cf acc = cf{0.0f, 0.0f};
      sfor<0, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const cf qj = (j == k) ? vc[t] : Q[j * DM + q + G * t];
        acc = acc + cmul(qj, wc[t]);
      });
      h[j] = acc;
    });
    sfor<j0, k + 1>([&](auto jc) { h[decltype(jc)::value] = sumq<G>(h[decltype(jc)::value]); });
    // (the basis entries are read again below, not kept in registers from the
    // coefficient pass: at k = 7 they were 80 VGPRs)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    sfor<j0, k + 1>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const cf qj = (j == k) ? vc[t] : Q[j * DM + q + G * t];
        fms_c(wc[t], h[j], qj);
      });
    });
    float nb = 0.0f;
    sfor<0, NB>([&](auto tc) { nb += abs2(wc[decltype(tc)::value]); });
    nb = sumq<G>(nb);
    const float b = fsqrt(nb);
    if (li == 0) {
      S.a[k] = h[k].re;
      if (k + 1 < M) {
        S.e2[k] = nb;
        S.ev[k] = b;
      }
    }
    // (a breakdown -- an invariant subspace, b ~ 0 -- leaves the remaining
    // basis vectors zero: the small tridiagonal splits and its top Ritz pair
    // is exact)
    const float ib = (b > 1e-20f) ? frcp(b) : 0.0f;
    sfor<0, NB>([&](auto tc) { vc[decltype(tc)::value] = ib * wc[decltype(tc)::value]; });
    if (k + 1 < M && p == 0) sfor<0, NB>([&](auto tc) { Q[(k + 1) * DM + q + G * decltype(tc)::value] = vc[decltype(tc)::value]; });
    blast = b;
    if constexpr (k == 0) b0 = b;
    wsync();
  });
  // top Ritz pair of the M x M tridiagonal (the full path's eigen routines)
  float lam[kRMax], tnorm;
  top_eigvals2d<M, 1, G>(S.a, S.e2, li, M, 1, lam, tnorm);
  float x[(M + L - 1) / L];
  tri_eigvec2d<M, G>(S.a, S.ev, S.fac, S.xs, li, M, lam[0], 1.2e-7f * fmaxf(tnorm, 1e-30f), 0,
                     reinterpret_cast<const float(*)[M]>(S.x), x);
  if (li < M) S.x[0][li] = x[0];
  wsync();
  const float sm = S.x[0][M - 1];
  // Ritz vector y = sum_k s_k Q_k (column layout), unit norm
  cf yc[NB];
  sfor<0, NB>([&](auto tc) { yc[decltype(tc)::value] = cf{0.0f, 0.0f}; });
  for (int k = 0; k < M; ++k) {
    const float sk = S.x[0][k];
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      yc[t] = yc[t] + sk * Q[k * DM + q + G * t];
    });
  }
  float ny = 0.0f;
  sfor<0, NB>([&](auto tc) { ny += abs2(yc[decltype(tc)::value]); });
  ny = sumq<G>(ny);
  const float theta = lam[0];
  const float res = blast * fabsf(sm);
  // Accept on the Lanczos residual, and only when nothing says the Ritz pair
  // may be a lower eigenpair (an eigenvalue crossing since the start vector
  // was the top one): a first step that already breaks down (the start
  // vector spans an invariant subspace on its own: exact, but not
  // necessarily the top pair) and a Ritz value below a diagonal entry of C
  // (a Rayleigh quotient: lambda_1 is at least that) send the bin back.
  ok = ok && ny > 0.5f && theta > 0.0f && theta < 3.0e38f && res <= kLzTol * theta;
  ok = ok && b0 > kLzBreak * theta && theta >= dmax * (1.0f - 4.0e-6f);
  const float sy = frsq(fmaxf(ny, 1e-30f));
  // lane layout through LDS
  if (p == 0) sfor<0, NB>([&](auto tc) { S.vb[q + G * decltype(tc)::value] = sy * yc[decltype(tc)::value]; });
  wsync();
  sfor<0, V>([&](auto vc2) {
    constexpr int v = decltype(vc2)::value;
    const int i = li + L * v;
    vv[v] = (i < D) ? S.vb[i < DM ? i : 0] : cf{0.0f, 0.0f};
  });
  wsync();   // vb reads before the caller's next write
  lam1 = theta;
  // wave-uniform verdict (G = 4: four bins per wave fall back together)
  return __ballot(!ok) == 0ull;
}

// w from the rank-1 eigenpair (lam1, vv) of C: w = (1 - 1/lam1) x (v^H g),
// x = Li^H v (the tail of eigen2d for one rank)
template <int NB, int G = 8>
DANSE_DEV void rank1_w2d(LDS2<NB, G>& S, int li, int D, const cf (&vv)[vpl<NB, G>()], float lam1,
                         cf (&w)[vpl<NB, G>()]) {
  constexpr int DM = G * NB, L = bin_lanes<G>(), V = vpl<NB, G>();
  const int p = li / G, q = li % G;
  cf sg;
  sfor<0, V>([&](auto vc) {
    constexpr int v = decltype(vc)::value;
    const int i = li + L * v;
    const cf t = cmul(vv[v], S.g[i]);
    sg = (v == 0) ? t : sg + t;
  });
  const cf sr = gsum<L>(sg);
  sfor<0, V>([&](auto vc) {
    const int i = li + L * decltype(vc)::value;
    if (i < DM) S.vb[i] = vv[decltype(vc)::value];
  });
  wsync();
  cf vr[NB];
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    vr[sb] = S.vb[p + G * sb];
  });
  const float coef = 1.0f - frcp(lam1);
  cf wc[NB];
  sfor<0, NB>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    cf acc = cf{0.0f, 0.0f};
    sfor<t, NB>([&](auto sc) {   // Li[i][c] = 0 for i < c
      constexpr int sb = decltype(sc)::value;
      acc = acc + cmul(ls_get<DM>(S.Ls, p + G * sb, q + G * t), vr[sb]);
    });
    acc = sump<G>(acc);
    wc[t] = coef * (acc * sr);
  });
  wsync();   // vb reads before the wb writes (they share the union)
  if (p == 0) {
    sfor<0, NB>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      S.wb[q + G * t] = wc[t];
    });
  }
  wsync();
  sfor<0, V>([&](auto vc) {
    const int i = li + L * decltype(vc)::value;
    w[decltype(vc)::value] = (i < D) ? S.wb[i < D ? i : 0] : cf{0.0f, 0.0f};
  });
}

// ---- phase 2: A = Ryy block (float32, destroyed), Li in S.Ls -> w[v] = entry li + L v
// vCache (rank 1, or null): this bin's eigenvector of C from its previous
// solve (the Lanczos start; zero = none), rewritten with this solve's (store:
// the bin is real, not a padding copy)
// Returns the path (wave-uniform): 0 the Householder path (no warm start
// tried, or none to try from), 1 the warm Lanczos solve accepted, 2 the warm
// solve tried and sent back to the Householder path.
template <int NB, int RMAX, int G = 8>
DANSE_DEV int gevd2d_solve(Blk<NB>& A, LDS2<NB, G>& S, int li, int D, int R, cf (&w)[vpl<NB, G>()],
                           cf* vCache = nullptr, bool store = false);
template <int NB, int RMAX, int G = 8>
DANSE_DEV int gevd2d_filter(Blk<NB>& A, LDS2<NB, G>& S, int li, int D, int R, cf (&w)[vpl<NB, G>()],
                            cf* vCache = nullptr, bool store = false) {
  congruence2d<NB, G>(A, S, li, D);
  return gevd2d_solve<NB, RMAX, G>(A, S, li, D, R, w, vCache, store);
}
// the part after the congruence (C in A)
template <int NB, int RMAX, int G>
DANSE_DEV int gevd2d_solve(Blk<NB>& A, LDS2<NB, G>& S, int li, int D, int R, cf (&w)[vpl<NB, G>()], cf* vCache,
                           bool store) {
  constexpr int V = vpl<NB, G>(), L = bin_lanes<G>(), DM = G * NB;
  int path = 0;
  // (classes below 20: too few Lanczos steps fit, and the D-step Householder
  // path is short there -- measured slower with the warm start)
  if (G * NB >= 20 && vCache && R == 1) {
    cf vv[V];
    float lam1;
    bool warm;
    if (lanczos2d<NB, G>(A, S, li, D, vCache, vv, lam1, warm)) {
      rank1_w2d<NB, G>(S, li, D, vv, lam1, w);
      if (store) {
        sfor<0, V>([&](auto vc) {
          const int i = li + L * decltype(vc)::value;
          if (i < DM) vCache[i] = vv[decltype(vc)::value];
        });
      }
      return 1;
    }
    path = warm ? 2 : 0;
  }
  tridiag2d<NB, G>(A, S, li, D);
  eigen2d<NB, RMAX, G>(S, li, D, R, w, R == 1 ? vCache : nullptr, store);
  return path;
}

}  // namespace t2d
}  // namespace danse
