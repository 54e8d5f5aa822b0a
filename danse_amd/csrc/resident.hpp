// Resident-SCM persistent engine (BASELINE north_star: "a
// persistent kernel that keeps each bin's small Hermitian matrix resident in
// registers/LDS while STFT frames stream from HBM").  The reference's round
// loop (danse_toolbox/d_core.py:66-90: broadcast, then every node's
// update_and_estimate) runs INSIDE one launch:
//
//   * every update wave owns four bins of one (scene, family-node) on 4 x 4
//     lane grids (solver2d.hpp, G = 4) for the whole run: its Rnn block
//     (float64) and Ryy block (float32) stay in VGPRs across all R rounds
//     (the recursion of d_classes.py:2086-2090 never touches HBM), and the
//     GEVD factor Li / g of its last factorisation stays in the wave's LDS
//     (reused while Rnn is unchanged, kernels.hpp li_reusable);
//   * one Z wave per (scene, node) does the broadcast of round r: the z
//     synthesis + OLA of the fused spectrum (d_base.py:1829-1852), the stream
//     append (fill_buffers, d_classes.py:1185-1224) and the analysis of the z
//     frame the receivers use (d_classes.py:1701-1807);
//   * the fused spectrum zhat = wExt^H yhat of round r + 1 is formed by the
//     update waves themselves right after they produce wExt[r + 1], from the
//     broadcast-frame spectra analysed before the launch (they do not depend
//     on any filter), so the Z wave only sums nothing and transforms;
//   * only yhat / z / dhat / w / wExt touch HBM inside the loop; the WOLA
//     analyses of every round run before the launch (resident_analysis_kernel)
//     and the estimate synthesis after it (resident_synth_* kernels).
//
// Hand-offs (all inside one launch, agent-coherent sc1 payload stores and
// loads, per-wave round flags stored after s_waitcnt vmcnt(0);
// MI355X_MICROARCH.md "inter-workgroup visibility"):
//   update wave (s, fn, bin group) -> uFlag = r + 1 after round r
//   Z wave (s, k) waits for every bin group of (s, DANSE family, k) >= r,
//     transforms, writes Zspec slot r + 1, sets zFlag[s][k] = r
//   update waves of round r wait for zFlag[s][q] >= r, every q.
// Every wave of the grid must be resident at once (the host checks the
// occupancy); every wait gives up after kSpinCap polls and flags an error,
// so a wave that never arrives drains the grid instead of hanging it.
//
// The per-bin arithmetic is update_kernel_2d's (kernels_2d.hpp) in the same
// order, so the resident run reproduces the launch-per-round engine.
#pragma once
#include "bcast.hpp"
#include "kernels.hpp"
#include "solver2d.hpp"

namespace danse {
namespace res {

#ifndef RES_WPE
#define RES_WPE 2
#endif
constexpr int kG = 4;          // 4 x 4 lane grids, four bins per wave
constexpr int kBins = 4;       // bins per update wave
constexpr unsigned kSpinCap = 1u << 22;   // polls (s_sleep 2 each) before a wait gives up

struct ResArgs {
  UpdateArgs u;               // Yall = update-frame spectra, zAll = 1, Zspec = [R + 1][K][S][F]
  BcastArgs b;                // windows, twiddles, zPrev / zStream of the Z waves
  const FamNode* fn;          // [nFN] every family-node of the engine
  const int* danseFni;        // [K] family-node index of node k's DANSE filter
  int nFN, FG, nZ, R;
  const cf* YB;               // [R][S][MT][F] broadcast-frame spectra
  cf* zhat;                   // [S][K][F] fused spectrum of the next round
  unsigned* uFlag;            // [S][nFN][FG]
  unsigned* zFlag;            // [S][K]
  const int* gateRound;       // [S][nFN]: round whose pre-update SCMs go to RyyG / RnnG (-1: none)
  cf* RyyG;
  cd* RnnG;
  int* err;                   // [1]: a wait gave up
  unsigned long long* trace;  // diagnostics (DANSE_RESIDENT_TRACE): [R][grid][2] wall clock after the
                              // wait / at the publish of every wave and round, or null
};

DANSE_DEV void trace_mark(const ResArgs& ra, int r, int slot) {
  if (ra.trace && __lane_id() == 0)
    ra.trace[((long long)r * gridDim.x + blockIdx.x) * 2 + slot] = wall_clock64();
}

// Wave-uniform wait until flags[0 .. n) >= target (each lane polls every
// 64th flag with sc1 loads).  False if it gave up.
DANSE_DEV bool wait_all(const unsigned* flags, int n, unsigned target, int* err) {
  for (unsigned it = 0;; ++it) {
    bool ok = true;
    for (int i = __lane_id(); i < n; i += 64) ok = ok && (ld_flag(flags + i) >= target);
    if (__ballot(!ok) == 0ull) return true;
    if (it > kSpinCap) {
      if (__lane_id() == 0) atomicOr(err, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Drain this wave's stores, then publish a round flag (one lane).
DANSE_DEV void publish(unsigned* flag, unsigned v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (__lane_id() == 0) st_flag(flag, v);
}

// ---- the Z wave of (scene s, node k): rounds 1 .. R - 1 (round 0's
// broadcast is the ordinary bcast_kernel before the launch).  Everything it
// re-reads every round stays on the chip: the FFT twiddles and the window
// values of its lanes in registers, the OLA state (the previous z frame,
// zPrev of bcast_kernel) in LDS, double-buffered by round parity; from HBM
// it reads only the fused spectrum and writes the stream and the spectra.
DANSE_DEV void z_role(const ResArgs& ra, int s, int k, cf* L, float* zqb, float* nvL) {
  const BcastArgs& a = ra.b;
  const int N = a.N, Ns = a.Ns, F = a.F, K = a.K, S = a.S;
  const float sqNs = sqrtf((float)Ns);
  const float invSqNs = 1.0f / sqNs;
  const float sc = sqNs / (float)N;
  const int l0 = __lane_id();
  const unsigned* uf = ra.uFlag + ((long long)s * ra.nFN + ra.danseFni[k]) * ra.FG;
  const cf* zh = ra.zhat + ((long long)s * K + k) * F;
  float* zs = a.zStream + ((long long)s * K + k) * a.zLen;
  wfft::TwReg tw;
  tw.load(a.tw);
  float hA[16], hS[16];   // (the OLA normalisation goes to LDS: registers are the limit here)
#pragma unroll
  for (int j = 0; j < 16; ++j) hA[j] = a.hA[l0 + 64 * j];
#pragma unroll
  for (int c = 0; c < 16; ++c) hS[c] = a.hS[wfft::out_index(c)];
  for (int n = l0; n < Ns; n += 64) nvL[n] = a.normVal[n];
  // round 0's z frame (bcast_kernel left it in zPrev) -> buffer 0
  {
    const float* zpv = a.zPrev + ((long long)s * K + k) * N;
#pragma unroll
    for (int j = 0; j < 16; ++j) zqb[l0 + 64 * j] = zpv[l0 + 64 * j];
  }
  for (int r = 1; r < ra.R; ++r) {
    // (lane index laundered per round, as in the update waves: no
    // lane-derived addresses hoisted out of the round loop)
    int l = l0, zo = (r & 1) * 1024;
    asm volatile("" : "+v"(l), "+v"(zo));
    float* zq = zqb + zo;                  // this round's frame
    const float* zp = zqb + (1024 - zo);   // the previous round's
    if (!wait_all(uf, ra.FG, (unsigned)r, ra.err)) return;
    trace_mark(ra, r, 0);
    // z synthesis: sqrt(Ns) * real(ifft(herm-ext(zhat))) * f, OLA with the previous frame
    cf v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = l + 64 * j;
      const int nn = (n < F) ? n : N - n;
      cf z = ld_sc1(zh + nn);
      if (nn == 0 || nn == F - 1) z.im = 0.0f;
      v[j] = (n < F) ? conjg(z) : z;
    }
    wfft::fft1024_tw(v, L, tw);
    bool nz = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) nz |= (zp[l + 64 * j] != 0.0f);
    const bool prevNZ = __ballot(nz) != 0ull;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int n = wfft::out_index(c);
      float zc = sc * v[c].re * hS[c];
      // (unconditional reads at clamped indices: no read waited for under a branch)
      const float zo = zp[min(n + Ns, N - 1)];
      const float nv = nvL[min(n, Ns - 1)];
      if (prevNZ) {
        float t = (n < N - Ns) ? zo : 0.0f;
        t += zc;
        if (n < Ns) t = t / nv;
        zc = t;
      }
      zq[n] = zc;
    }
    wfft::wave_sync();
    // the z frame the receivers consume at round r: stream [(r-1)Ns, (r+1)Ns)
    // = the previous frame's first Ns samples, then this one's
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = l + 64 * j;
      const float t = (n < Ns) ? zp[n] : zq[n - Ns];
      if (n < Ns) zs[(long long)r * Ns + n] = zq[n];
      v[j] = cf{t * hA[j], 0.0f};
    }
    wfft::fft1024_tw(v, L, tw);
    cf* Zs = const_cast<cf*>(ra.u.Zspec) + (((long long)(r + 1) * K + k) * S + s) * F;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int f = wfft::out_index(c);
      if (f < F) st_sc1(Zs + f, invSqNs * v[c]);
    }
    publish(ra.zFlag + (long long)s * K + k, (unsigned)r);
    trace_mark(ra, r, 1);
  }
}

template <int NB>
constexpr int lds_bytes() {
  constexpr int u = (int)sizeof(t2d::LDS2<NB, kG>) * kBins + (int)sizeof(cf) * kBins * 16 * t2d::vpl<NB, kG>();
  constexpr int z = (int)sizeof(cf) * wfft::kLdsElems + (int)sizeof(float) * (2048 + 512);
  return u > z ? u : z;
}

// The fused spectrum of round r + 1 for this wave's bins from the new
// external filter entries ne (lane li: mic li + L v) and the prefetched
// broadcast-frame spectra: bcast.hpp phase 1 + the part[] sum of phase 2 in
// the same order (per broadcast wave w the mics m = w, w + 4, ..., then the
// four partial sums left to right).  Stored sc1 for the Z wave.
template <int V>
DANSE_DEV void fused_next(const ResArgs& ra, const UpdateArgs& a, const FamNode& d, int s, int f, int li, bool fvalid,
                          int r, cf* zt, const cf (&ne)[V], const cf (&yb)[V]) {
  constexpr int L = 16;
  if (r + 1 >= ra.R) return;
  const int M = d.M;
  sfor<0, V>([&](auto vc) {
    constexpr int v = decltype(vc)::value;
    const int m = li + L * v;
    if (m < M) zt[m] = cmul(ne[v], yb[v]);
  });
  t2d::wsync();
  if (li == 0 && fvalid) {
    cf z = cf{0.0f, 0.0f};
    for (int wv = 0; wv < kBcWaves; ++wv) {
      cf part = cf{0.0f, 0.0f};
      for (int m = wv; m < M; m += kBcWaves) part = part + zt[m];
      z = (wv == 0) ? part : z + part;
    }
    st_sc1(ra.zhat + ((long long)s * a.K + d.k) * a.F + f, z);
  }
  t2d::wsync();
}

template <int NB, int RMAX>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RES_WPE)))
resident_kernel(const ResArgs ra) {
  using namespace t2d;
  constexpr int G = kG, L = bin_lanes<G>(), W = 64 / L, V = vpl<NB, G>();
  static_assert(W == kBins, "four bins per wave");
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes<NB>()];
  const int id = blockIdx.x;
#ifndef RES_NOZ
  if (id < ra.nZ) {
    const int K = ra.b.K;
    float* zqb = reinterpret_cast<float*>(smem + sizeof(cf) * wfft::kLdsElems);
    z_role(ra, id / K, id % K, reinterpret_cast<cf*>(smem), zqb, zqb + 2048);
    return;
  }
#endif
  const int bw = threadIdx.x / L;
  const int li0 = threadIdx.x % L;
  cf* zt = reinterpret_cast<cf*>(smem + sizeof(LDS2<NB, G>) * W) + bw * L * V;   // this bin's mic products
  const int u = id - ra.nZ;
  const int fg = u % ra.FG;
  const int tt = u / ra.FG;
  const int fni = tt % ra.nFN;
  const int s = tt / ra.nFN;
  const int p0 = li0 / G, q0 = li0 % G;
  UpdateArgs a = ra.u;
  const int F = a.F, K = a.K;
  const int f0 = fg * W + bw;
  const bool fvalid = f0 < F;   // the last group's tail bins compute on bin F-1, store nothing
  const int f = fvalid ? f0 : F - 1;
  const FamNode d = ra.fn[fni];
  const int D0 = d.D;
  const double beta = a.beta[s * K + d.k];
  // SCMs: packed lower triangles, bin-major (FamNode.packed 2); a lane's
  // blocks above the diagonal start from the conjugates of the stored entries
  const long long triOff = (long long)s * a.scmStride + d.scmOff + (long long)f * (D0 * (D0 + 1) / 2);
  auto ent = [&](int i, int c) -> long long {
    return triOff + (i >= c ? i * (i + 1) / 2 + c : c * (c + 1) / 2 + i);
  };
  const int gateR = ra.gateRound ? ra.gateRound[s * ra.nFN + fni] : -1;
  const bool isDanse = d.fam == DANSE_FAM_DANSE;

  // resident state: this lane's NB x NB blocks of Rnn (float64) and Ryy (float32)
  BlkD<NB> Rn;
  Blk<NB> Ry;
  sfor<0, NB>([&](auto sc) {
    constexpr int sb = decltype(sc)::value;
    sfor<0, NB>([&](auto tc) {
      constexpr int tb = decltype(tc)::value;
      const int i = p0 + G * sb, c = q0 + G * tb;
      const bool in = i < D0 && c < D0;
      cd xn = csel(in, a.Rnn[in ? ent(i, c) : triOff], cd{0.0, 0.0});
      cf xy = csel(in, a.Ryy[in ? ent(i, c) : triOff], cf{0.0f, 0.0f});
      if (i < c) { xn = conjg(xn); xy = conjg(xy); }
      if (i == c) { xn.im = 0.0; xy.im = 0.0f; }
      Rn.v[sb][tb] = xn;
      Ry.v[sb][tb] = xy;
    });
  });
  bool liValid = false;     // S.Ls / S.g hold the factor of the current Rnn
  unsigned* myFlag = ra.uFlag + ((long long)s * ra.nFN + fni) * ra.FG + fg;

  for (int r = 0; r < ra.R; ++r) {
    a.r = r;
    // the lane index, the filter size and the LDS base are laundered per
    // round: otherwise the solver's lane-derived addresses and masks are
    // hoisted out of the round loop and stay live across all of it
    // (an integer offset, so that the accesses stay LDS instructions: a
    // laundered pointer loses its address space and turns into flat ones)
    int li = li0, D = D0, sOff = bw * (int)sizeof(LDS2<NB, G>);
    asm volatile("" : "+v"(li), "+v"(sOff));
    asm volatile("" : "+s"(D));
    LDS2<NB, G>& S = *reinterpret_cast<LDS2<NB, G>*>(smem + sOff);
    const int p = li / G, q = li % G;
    if (r > 0 && !wait_all(ra.zFlag + (long long)s * K, K, (unsigned)r, ra.err)) break;
    trace_mark(ra, r, 0);
    // the next round's broadcast-frame spectra of this node's mics (for the
    // fused spectrum at the end of the round): issued now, used after the solve
    cf ybPre[V];
    sfor<0, V>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      const int m = li + L * v;
      const bool use = isDanse && r + 1 < ra.R && m < d.M;
      const int ch = a.chanList[d.chanOff + (use ? m : 0)];
      ybPre[v] = use ? ra.YB[(((long long)(r + 1) * a.S + s) * a.MT + ch) * F + f] : cf{0.0f, 0.0f};
    });
    const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * K + d.k];
    const int opY = fl & 3, opN = (fl >> 2) & 3;
    const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;
    // Relaxed (and kept / reference-only) external filters do not depend on
    // this round's solve: wExt[r + 1] = b wExt[r] + (1 - b) target, with the
    // target as it stood before this round (d_classes.py:1627-1694).  So
    // the fused spectrum of round r + 1 is formed and published FIRST, and
    // the broadcast of round r + 1 runs while this round's solve does.
    const bool early = isDanse && !pregiven && d.extMode != DANSE_EXT_COPY;
    if (early) {
      const long long eb = (long long)s * a.wExtStride + d.wExtOff;
      const cf* eprev = a.wExtHist + eb + ((long long)(a.wExtHistory ? r : (r & 1)) * F + f) * d.M;
      const cf* tgt = a.wExtTarget + (long long)s * a.tgtStride + d.tgtOff + (long long)f * d.M;
      const float be = a.betaExt[s * K + d.k];
      cf neE[V];
      sfor<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        const int m = li + L * v;
        const bool in = m < d.M;
        const int mm = in ? m : 0;
        cf ne;
        if (d.extMode == DANSE_EXT_KEEP) ne = eprev[mm];
        else if (d.extMode == DANSE_EXT_REFONLY) ne = cf{(m == d.ref) ? 1.0f : 0.0f, 0.0f};
        else ne = ext_relax(be, eprev[mm], tgt[mm]);
        neE[v] = ne;
      });
      fused_next(ra, a, d, s, f, li, fvalid, r, zt, neE, ybPre);
      publish(myFlag, (unsigned)(r + 1));
    }
    const bool solve = (fl & DANSE_FLAG_SOLVE) != 0 && !pregiven;
    const bool initslot = (fl & DANSE_FLAG_INITSLOT) != 0;
    if (opN) liValid = false;

    cf y[V];
    sfor<0, V>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      const int i = li + L * v;
      y[v] = load_y(a, d, s, f, i, i < D);
      S.vb[i] = y[v];
    });
    t2d::wsync();
    cf yr[NB], yc[NB];
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      yr[sb] = S.vb[p + G * sb];
      yc[sb] = S.vb[q + G * sb];
    });
    t2d::wsync();

    if (r == gateR && fvalid) {
      // the speculative start gate is checked after the launch on the SCMs
      // as they stood before this round's recursion (gate.hpp applies it)
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        sfor<0, NB>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          const int i = p + G * sb, c = q + G * tb;
          if (i < D && c <= i) {
            ra.RnnG[ent(i, c)] = Rn.v[sb][tb];
            ra.RyyG[ent(i, c)] = Ry.v[sb][tb];
          }
        });
      });
    }

    // ---- Rnn (float64): recursion in registers, factor -> Li in S.Ls ----
    bool ok = true;
    if (opN) {
      const double cy = (opN == DANSE_OP_SET) ? 1.0 / D : (1.0 - beta) / D;
      const double cx = (opN == DANSE_OP_SET) ? 0.0 : beta;
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        sfor<0, NB>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          cd yy = cd{0.0, 0.0};
          fma_cc(yy, cdk(yr[sb]), cdk(yc[tb]));
          cd x = cx * Rn.v[sb][tb];
          x.re = fma(cy, yy.re, x.re);
          x.im = fma(cy, yy.im, x.im);
          Rn.v[sb][tb] = x;
        });
      });
    }
#ifndef RES_NOSOLVE
    if (solve && !liValid) {
      BlkD<NB> M = Rn;
      ok = gevd2d_factor<NB, G>(M, S, li, D, d.ref);
      liValid = true;
    }
#endif

    // ---- Ryy (float32): recursion in registers, filter --------------------
    cf w[V];
    sfor<0, V>([&](auto vc) { w[decltype(vc)::value] = cf{0.0f, 0.0f}; });
    if (opY) {
      const float by = (float)beta, cy = (opY == DANSE_OP_SET) ? (float)(1.0 / D) : (float)((1.0 - beta) / D);
      sfor<0, NB>([&](auto sc) {
        constexpr int sb = decltype(sc)::value;
        sfor<0, NB>([&](auto tc) {
          constexpr int tb = decltype(tc)::value;
          const cf yy = cy * mulc(yr[sb], yc[tb]);
          Ry.v[sb][tb] = csel(opY == DANSE_OP_SET, yy, by * Ry.v[sb][tb] + yy);
        });
      });
    }
#ifndef RES_NOSOLVE2
    if (solve) {
      Blk<NB> A = Ry;
      // (no warm-started Lanczos here: at D <= 12 the Householder path is
      // short and the few Lanczos steps that fit were measured slower)
      gevd2d_filter<NB, RMAX, G>(A, S, li, D, a.rank, w);
    }
#endif

    const long long wBase = (long long)s * a.wStride + d.wOff;
    const int slotPrev = a.wHistory ? r : (r & 1);
    const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
    cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
    cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
    if (solve && !initslot && !ok && li == 0 && fvalid) atomicOr(&a.diag[(s * K + d.k) * kMaxFam + d.fam], 1);
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
    cf ne[V];
    sfor<0, V>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      ne[v] = node_bin_tail(a, d, s, f, li + L * v, fl, pregiven, fvalid, w[v], y[v], dh);
    });

    if (!early) {
      // wExt[r + 1] = w[r + 1] (EXT_COPY): after the solve
      if (isDanse) fused_next(ra, a, d, s, f, li, fvalid, r, zt, ne, ybPre);
      publish(myFlag, (unsigned)(r + 1));
    }
    trace_mark(ra, r, 1);
  }

  // final SCMs back to HBM (the engine's state after the run)
  if (fvalid) {
    sfor<0, NB>([&](auto sc) {
      constexpr int sb = decltype(sc)::value;
      sfor<0, NB>([&](auto tc) {
        constexpr int tb = decltype(tc)::value;
        const int i = p0 + G * sb, c = q0 + G * tb;
        if (i < D0 && c <= i) {
          a.Rnn[ent(i, c)] = Rn.v[sb][tb];
          a.Ryy[ent(i, c)] = Ry.v[sb][tb];
        }
      });
    });
  }
}

}  // namespace res
}  // namespace danse
