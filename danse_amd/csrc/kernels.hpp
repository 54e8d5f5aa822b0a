// Device kernels of the DANSE frame-update engine.
//
// Per DANSE round r (all nodes of all scenes in parallel; round-synchronous
// fully connected schedule):
//   bcast_kernel  (one 256-thread workgroup per (scene, node)):
//       [synthesis of the estimates of round r-1 (get_desired_sig_chunk,
//        d_base.py:2027-2084)]
//       WOLA analysis of the broadcast frame of every local mic
//        (d_base.py:1821-1826), fused-signal spectrum zhat = wExt^H yhat,
//       WOLA synthesis + OLA normalisation of z (d_base.py:1829-1852),
//       append z[:Ns] to the node's stream (fill_buffers, d_classes.py:1185),
//       analysis of the z frame every receiver will use
//        (process_incoming_signals_buffers + build_ytilde,
//         d_classes.py:1701-1807,1893-1934).
//   update_kernel (one wavefront per 64/G frequency bins of one family-node):
//       SCM update (d_classes.py:2048-2267), filter update (update_w /
//       update_w_gevd, d_classes.py:3320-3387), external filters
//       (d_classes.py:1627-1694), dhat = w^H yhat (d_base.py:2075).
#pragma once
#include "common.hpp"
#include "fft.hpp"
#include "solver.hpp"
#include "../../include/danse_mi355x.h"

namespace danse {

constexpr int kMaxFam = 4;

struct FamNode {
  int fam, k, D, ref;
  int chanOff;        // offset into chanList
  int extMode;        // DANSE family only (else -1)
  int M;              // local mics of node k
  int pad;
  long long scmOff;   // complex-element offset within one scene's SCM block
  long long wOff;     // complex-element offset within one scene's w-history block
  long long wExtOff;  // DANSE only: offset within one scene's wExt-history block
  long long tgtOff;   // DANSE only: offset within one scene's target block
};

struct BcastArgs {
  int S, K, MT, T, N, Ns, F, R;
  int r;
  int k0, k1;
  int families;            // bitmask
  int doSynth;             // synthesise dhat of round r-1
  int doBcast;             // perform the broadcast of round r
  const int* M;            // [K]
  const int* base;         // [K] first channel of node k
  const int* bcEnd;        // [R*K]
  const int* upEnd;        // [R*K]
  const float* y;          // [S][MT][T]
  cf* Yspec;               // [2][S][MT][F]
  cf* Zspec;               // [K][S][F]
  float* zPrev;            // [S][K][N]
  float* zStream;          // [S][K][R*Ns]
  const cf* wExtHist;      // per scene block (stride wExtStride) : node offsets wExtNodeOff
  const long long* wExtNodeOff;  // [K]
  long long wExtStride;
  int wExtHistory;         // 1: index by r, 0: single slot
  const cf* dhat;          // [fam][S][K][R][F]
  float* d;                // [fam][S][K][T]
  const float* hA;         // analysis window [N]
  const float* hS;         // synthesis window [N]
  const float* normVal;    // [Ns] OLA normalisation h^2[n] + h^2[n+Ns]
  const cf* tw;            // [N] twiddles
};

// y[(frame end - N) .. frame end) * win, zero before sample 0 -> buf (complex, imag 0)
DANSE_DEV void load_frame(cf* buf, const float* __restrict__ x, int end, int N, int T,
                          const float* __restrict__ win) {
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const int idx = end - N + n;
    const float v = (idx >= 0 && idx < T) ? x[idx] : 0.0f;
    buf[n] = cf{v * win[n], 0.0f};
  }
}

__global__ void __launch_bounds__(256) bcast_kernel(const BcastArgs a) {
  __shared__ cf b0[1024];
  __shared__ cf b1[1024];
  __shared__ cf zacc[513];
  __shared__ float zq[1024];
  __shared__ int anyNZ;
  const int tid = threadIdx.x;
  const int N = a.N, Ns = a.Ns, F = a.F;
  const int nOwn = a.k1 - a.k0;
  const int s = blockIdx.x / nOwn;
  const int k = a.k0 + blockIdx.x % nOwn;
  const float sqNs = sqrtf((float)Ns);
  const float invSqNs = 1.0f / sqNs;
  const int r = a.r;

  // ---- synthesis of the estimates of round r-1, all families
  if (a.doSynth) {
    const int rp = r - 1;
    const int end = a.upEnd[rp * a.K + k];
    for (int fam = 0; fam < kMaxFam; ++fam) {
      if (!((a.families >> fam) & 1)) continue;
      const cf* dh = a.dhat + ((((long long)fam * a.S + s) * a.K + k) * a.R + rp) * F;
      // forward FFT of conj(Hermitian extension) gives N * conj(ifft); real part is what we need
      for (int n = tid; n < N; n += blockDim.x) {
        cf X;
        if (n < F) X = conjg(dh[n]);
        else X = dh[N - n];
        b0[n] = X;
      }
      __syncthreads();
      cf* out = fft1024(b0, b1, a.tw);
      float* dd = a.d + (((long long)fam * a.S + s) * a.K + k) * a.T;
      const float sc = sqNs / (float)N;
      for (int n = tid; n < N; n += blockDim.x) {
        const int idx = end - N + n;
        if (idx >= 0 && idx < a.T) dd[idx] += sc * a.hS[n] * out[n].re;
      }
      __syncthreads();
    }
  }
  if (!a.doBcast) return;

  // ---- local analysis + fused spectrum
  const int Mk = a.M[k];
  const int bEnd = a.bcEnd[r * a.K + k];
  const cf* wx = a.wExtHist + (long long)s * a.wExtStride + a.wExtNodeOff[k] +
                 (a.wExtHistory ? (long long)r * F * Mk : 0);
  for (int f = tid; f < F; f += blockDim.x) zacc[f] = cf{0.0f, 0.0f};
  for (int m = 0; m < Mk; ++m) {
    const int c = a.base[k] + m;
    const float* x = a.y + ((long long)s * a.MT + c) * a.T;
    load_frame(b0, x, bEnd, N, a.T, a.hA);
    __syncthreads();
    cf* out = fft1024(b0, b1, a.tw);
    cf* Ys = a.Yspec + (((long long)(r & 1) * a.S + s) * a.MT + c) * F;
    for (int f = tid; f < F; f += blockDim.x) {
      const cf Y = invSqNs * out[f];
      Ys[f] = Y;
      zacc[f] = zacc[f] + cmul(wx[(long long)f * Mk + m], Y);
    }
    __syncthreads();
    const bool needUp = (r == 0) || (a.upEnd[r * a.K + k] != a.bcEnd[(r - 1) * a.K + k]);
    if (needUp) {
      // update-local frame of round r (only when it is not the broadcast frame of r-1)
      const int uEnd = a.upEnd[r * a.K + k];
      load_frame(b0, x, uEnd, N, a.T, a.hA);
      __syncthreads();
      cf* o2 = fft1024(b0, b1, a.tw);
      cf* Yu = a.Yspec + (((long long)((r + 1) & 1) * a.S + s) * a.MT + c) * F;
      for (int f = tid; f < F; f += blockDim.x) Yu[f] = invSqNs * o2[f];
      __syncthreads();
    }
  }
  // ---- z synthesis: sqrt(Ns) * real(ifft(herm-ext(zhat))) * f
  for (int n = tid; n < N; n += blockDim.x) {
    cf X;
    if (n < F) {
      X = zacc[n];
      if (n == 0 || n == F - 1) X.im = 0.0f;
      X = conjg(X);
    } else {
      X = zacc[N - n];
    }
    b0[n] = X;
  }
  if (tid == 0) anyNZ = 0;
  __syncthreads();
  float* zp = a.zPrev + ((long long)s * a.K + k) * N;
  {
    int nz = 0;
    for (int n = tid; n < N; n += blockDim.x) nz |= (zp[n] != 0.0f);
    if (nz) atomicOr(&anyNZ, 1);
  }
  cf* out = fft1024(b0, b1, a.tw);
  const float sc = sqNs / (float)N;
  const bool prevNZ = anyNZ != 0;
  for (int n = tid; n < N; n += blockDim.x) {
    float zc = sc * out[n].re * a.hS[n];
    if (prevNZ) {
      float v = (n < N - Ns) ? zp[n + Ns] : 0.0f;
      v += zc;
      if (n < Ns) v = v / a.normVal[n];
      zc = v;
    }
    zq[n] = zc;
  }
  __syncthreads();
  float* zs = a.zStream + ((long long)s * a.K + k) * ((long long)a.R * Ns);
  for (int n = tid; n < N; n += blockDim.x) {
    zp[n] = zq[n];
    if (n < Ns) zs[(long long)r * Ns + n] = zq[n];
  }
  // ---- z frame the receivers consume at round r: stream samples [(r+1)Ns - N, (r+1)Ns)
  for (int n = tid; n < N; n += blockDim.x) {
    const long long idx = (long long)(r + 1) * Ns - N + n;
    float v;
    if (idx < 0) v = 0.0f;
    else if (idx >= (long long)r * Ns) v = zq[idx - (long long)r * Ns];
    else v = zs[idx];
    b0[n] = cf{v * a.hA[n], 0.0f};
  }
  __syncthreads();
  out = fft1024(b0, b1, a.tw);
  cf* Zs = a.Zspec + ((long long)k * a.S + s) * F;
  for (int f = tid; f < F; f += blockDim.x) Zs[f] = invSqNs * out[f];
}

struct UpdateArgs {
  int S, K, MT, F, R, r;
  int nFN;                 // family-nodes in this launch
  const FamNode* fn;       // [nFN]
  const int* famNodeId;    // [nFN] index into the global family-node list (for flags/dhat)
  const int* chanList;
  const uint8_t* flags;    // [R][S][kMaxFam][K]
  const cf* Yspec;         // [2][S][MT][F]
  const cf* Zspec;         // [K][S][F]
  cf* Ryy;                 // per scene stride scmStride
  cf* Rnn;
  long long scmStride;
  cf* wHist;               // per scene stride wStride
  long long wStride;
  int wHistory;            // 1: [R+1][F][D] per family-node; 0: 2 slots
  cf* wExtHist;
  long long wExtStride;
  int wExtHistory;
  cf* wExtTarget;
  long long tgtStride;
  cf* dhat;                // [fam][S][K][R][F]
  const float* beta;       // [S*K]
  const float* betaExt;    // [S*K]
  float alphaExt;
  int gevd, rank;
  int* diag;               // [S*K*kMaxFam]
};

template <int G, int DMAX, int RMAX>
__global__ void __launch_bounds__(64) update_kernel(const UpdateArgs a) {
  static_assert(DMAX <= G, "a lane group must hold every row");
  constexpr int NB = 64 / G;
  __shared__ SolverLDS<DMAX> lds[NB];
  const int lane = threadIdx.x;
  const int li = lane & (G - 1);
  const int gi = lane / G;
  const int F = a.F;
  const int nBB = (F + NB - 1) / NB;
  const int bb = blockIdx.x % nBB;
  const int t = blockIdx.x / nBB;
  const int fni = t % a.nFN;
  const int s = t / a.nFN;
  const FamNode d = a.fn[fni];
  const int D = d.D;
  int f = bb * NB + gi;
  const bool valid = f < F;
  if (!valid) f = F - 1;
  const bool act = li < D;
  const int r = a.r;
  const uint8_t fl = a.flags[(((long long)r * a.S + s) * kMaxFam + d.fam) * a.K + d.k];
  const int opY = fl & 3, opN = (fl >> 2) & 3;
  const bool solve = (fl & DANSE_FLAG_SOLVE) != 0;

  // ---- observation vector yhat_li
  cf y = cf{0.0f, 0.0f};
  {
    const int c = a.chanList[d.chanOff + (act ? li : 0)];
    const cf* src = (c < a.MT) ? a.Yspec + (((long long)((r + 1) & 1) * a.S + s) * a.MT + c) * F
                               : a.Zspec + ((long long)(c - a.MT) * a.S + s) * F;
    const cf v = src[f];
    y = act ? v : cf{0.0f, 0.0f};
  }
  const float beta = a.beta[s * a.K + d.k];
  const float invD = 1.0f / (float)D;
  const long long matOff = (long long)s * a.scmStride + d.scmOff + (long long)f * D * D;
  const int rowc = act ? li : 0;

  // yy^H row li: invD * y_li * conj(y_c)
  cf yy[DMAX];
  sfor<0, DMAX>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    const cf yc = gbcast<G, c>(y);
    yy[c] = (c < D) ? invD * mulc(y, yc) : cf{0.0f, 0.0f};
  });

  cf A[DMAX], B[DMAX];
  auto load_rows = [&](const cf* P, cf (&X)[DMAX]) {
    sfor<0, DMAX>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      const int cl = (c < D) ? c : D - 1;
      const cf v = P[matOff + (long long)rowc * D + cl];
      X[c] = (act && c < D) ? v : cf{0.0f, 0.0f};
    });
  };
  auto store_rows = [&](cf* P, const cf (&X)[DMAX]) {
    if (act && valid) {
      sfor<0, DMAX>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if (c < D) P[matOff + (long long)li * D + c] = X[c];
      });
    }
  };
  auto apply_op = [&](cf (&X)[DMAX], int op) {
    sfor<0, DMAX>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if (op == DANSE_OP_SET) X[c] = yy[c];
      else X[c] = beta * X[c] + (1.0f - beta) * yy[c];
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

  // ---- filter
  const long long wBase = (long long)s * a.wStride + d.wOff;
  const int slotPrev = a.wHistory ? r : (r & 1);
  const int slotNext = a.wHistory ? r + 1 : ((r + 1) & 1);
  cf* wPrev = a.wHist + wBase + ((long long)slotPrev * F + f) * D;
  cf* wNext = a.wHist + wBase + ((long long)slotNext * F + f) * D;
  cf w;
  const bool pregiven = (fl & DANSE_FLAG_PREGIVEN) != 0;
  if (pregiven) {
    w = act ? wNext[act ? li : 0] : cf{0.0f, 0.0f};
  } else if (solve) {
    bool ok = true;
    if (a.gevd) w = gevd_filter<G, DMAX, RMAX>(A, B, lds[gi], li, D, a.rank, d.ref, ok);
    else w = mwf_filter<G, DMAX>(A, B, li, D, d.ref, ok);
    if (!ok && li == 0 && valid) atomicOr(&a.diag[(s * a.K + d.k) * kMaxFam + d.fam], 1);
  } else {
    w = act ? wPrev[act ? li : 0] : cf{0.0f, 0.0f};
  }
  if (act && valid && !pregiven) wNext[li] = w;

  // ---- external filters (DANSE family)
  if (d.extMode >= 0 && !pregiven) {
    const int M = d.M;
    const long long eb = (long long)s * a.wExtStride + d.wExtOff;
    const int eP = a.wExtHistory ? r : (r & 1);
    const int eN = a.wExtHistory ? r + 1 : ((r + 1) & 1);
    cf* eprev = a.wExtHist + eb + ((long long)eP * F + f) * M;
    cf* enext = a.wExtHist + eb + ((long long)eN * F + f) * M;
    cf* tgt = a.wExtTarget + (long long)s * a.tgtStride + d.tgtOff + (long long)f * M;
    if (li < M && valid) {
      cf ne;
      if (d.extMode == 0) ne = w;
      else if (d.extMode == 2) ne = eprev[li];
      else if (d.extMode == 3) ne = cf{(li == d.ref) ? 1.0f : 0.0f, 0.0f};
      else {
        const float be = a.betaExt[s * a.K + d.k];
        const cf tg = tgt[li];
        ne = be * eprev[li] + (1.0f - be) * tg;
        if (fl & DANSE_FLAG_EXT_TARGET) tgt[li] = (1.0f - a.alphaExt) * tg + a.alphaExt * w;
      }
      enext[li] = ne;
    }
  }

  // ---- dhat = w^H yhat (DC / Nyquist forced real, quirk Q7)
  cf dh = gsum<G>(act ? cmul(w, y) : cf{0.0f, 0.0f});
  if (f == 0 || f == F - 1) dh.im = 0.0f;
  if (li == 0 && valid) {
    a.dhat[((((long long)d.fam * a.S + s) * a.K + d.k) * a.R + r) * F + f] = dh;
  }
}

}  // namespace danse
