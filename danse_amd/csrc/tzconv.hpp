// T(z) few-samples compression building blocks, shared by the stand-alone
// operators (tz.hip: danse_tz_ir / danse_tz_compress) and the online engine's
// fewSamples broadcasts (danse_engine.hip).  SURVEY §8a row a14.
//
// dist_fct_approx (d_base.py:1941-1991) sums the offset diagonals of
// diag(f) C diag(h), C the circulant of flip(w_td), w_td = real(IFFT(
// Hermitian-extended conj(wHat))).  The tau-th diagonal has the constant
// circulant entry c[(-tau) mod N], so
//     wIR[i] = w_td[i mod N] * S[i] / R,   i = tau + N - 1 in [0, 2N - 2],
//     S[i]   = sum_n f[n] h[n + i - N + 1]       (window cross-correlation)
// and, w_td being real, w_td = Re(FFT(Y)) / N with Y the Hermitian extension
// of wHat itself: one wave FFT (wfft.hpp), then 2N - 1 scaled stores.
// sn = S / (N R) is a host-built table (windows only).
//
// The convolution (extract_few_samples_from_convolution, d_base.py:1538-1566)
// keeps only the L samples the node broadcasts:
//     z[ii] = sum_m sum_q yq[q][m] wIR[id_ii - q][m],  id_ii = 2N - 1 - L + 1 + ii
// (taps outside [0, 2N - 2] are the reference's zero padding).  One 256-thread
// workgroup per filter; the frame and the IR of up to kMC sensors sit in LDS.
// A thread owns kR = 16 consecutive outputs over a contiguous range of q and
// slides a 23-tap window through the IR, so every LDS read feeds 5.6 FMAs;
// the IR is stored with one pad slot per 16 taps so the lanes of a wave
// (output blocks 16 apart, stride 17 after padding) hit distinct banks.  Partial sums over the q ranges are
// reduced through LDS.
#pragma once
#include "wfft.hpp"

namespace danse {
namespace tzc {

constexpr int kN = 1024;
constexpr int kA = 2 * kN - 1;          // IR length
constexpr int kR = 16;                  // outputs per thread
constexpr int kMC = 2;                  // sensors per LDS pass (26.6 KB of LDS: 6 workgroups per CU)
constexpr int kThr = 256;
constexpr int kIrPad = 16;              // zero taps past the IR end (tile overhang)
constexpr int kIrSlots = kA + kIrPad;
DANSE_DEV int phys(int x) { return x + (x >> 4); }
constexpr int kIrPhys = kIrSlots + kIrSlots / 16 + 1;

union ConvLds {
  struct {
    float ys[kMC][kN];
    float as[kMC][kIrPhys];
  } in;
  float red[kThr * kR];   // partial sums, after the last pass
};

// One wave: IR of one (filter, sensor).  wAt(k) = wHat[k] for k in [0, N/2];
// out(t, v) stores tap t in [0, 2N - 2].
template <class WF, class OF>
DANSE_DEV void ir_wave(cf* lds, const cf* __restrict__ tw, const float* __restrict__ sn, WF wAt, OF out) {
  const int l = __lane_id();
  // (every read issued unconditionally, then held: a read under a branch, or
  // after a store, is one memory round trip per element)
  cf v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = l + 64 * j;
    v[j] = wAt(k <= kN / 2 ? k : kN - k);
  }
  hold(v);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = l + 64 * j;
    if (k == 0 || k == kN / 2) v[j].im = 0.f;   // DC / Nyquist forced real (d_base.py:1522-1523)
    else if (k > kN / 2) v[j] = conjg(v[j]);
  }
  float s0[16], s1[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int t = wfft::out_index(c);
    s0[c] = sn[t];
    s1[c] = sn[min(t + kN, kA - 1)];
  }
  wfft::fft1024(v, lds, tw);
  hold(s0);
  hold(s1);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int t = wfft::out_index(c);
    const float wt = v[c].re;
    out(t, wt * s0[c]);
    if (t < kN - 1) out(t + kN, wt * s1[c]);
  }
}

// One workgroup (kThr threads): the last L (1 <= L <= N) outputs of the
// M-sensor convolution.  yAt(q, m): frame sample q of sensor m, read at a
// valid address for every q < N (yKeep(q, m) false: the sample is zero, its
// read value discarded -- the read stays unconditional); aAt(i, m): IR tap
// i < kA of sensor m; out(e, v): output e in [0, L).
// nTiles = ceil(L / kR) output tiles, G = kThr / nTiles q ranges (G >= 1).
// off: 0 for the broadcast chunks (idDesired = kA - L + 1 .. kA,
// d_base.py:1924-1927), -1 for the 'conv' desired-signal chunk (kA - Ns ..
// kA - 1, d_base.py:2092).
template <class YF, class YK, class AF, class OF>
DANSE_DEV void conv_block(ConvLds& sm, int M, int L, YF yAt, YK yKeep, AF aAt, OF out, int off = 0) {
  const int t = threadIdx.x;
  const int nTiles = (L + kR - 1) / kR;
  const int G = kThr / nTiles;
  const int tile = t % nTiles, g = t / nTiles;
  const bool active = g < G;
  const int qc = (kN + G - 1) / G;
  const int q0 = min(kN, g * qc), q1 = min(kN, q0 + qc);
  const int d0 = kA - L + 1 + off + tile * kR;   // convolution index of this thread's first output
  float acc[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) acc[r] = 0.f;
  for (int m0 = 0; m0 < M; m0 += kMC) {
    const int mc = min(kMC, M - m0);
    __syncthreads();   // previous pass's reads are done
    // staging: every thread's reads issued together at clamped (valid)
    // indices and held, then the LDS writes -- a strided loop keeps one read
    // in flight per thread (one memory round trip per iteration)
    {
      constexpr int kYIt = kN * kMC / kThr;
      float yv[kYIt];
#pragma unroll
      for (int u = 0; u < kYIt; ++u) {
        const int e = min(t + u * kThr, kN * mc - 1);
        const int q = e / mc, mm = e - q * mc;
        yv[u] = yAt(q, m0 + mm);
      }
      hold(yv);
#pragma unroll
      for (int u = 0; u < kYIt; ++u) {
        const int e = t + u * kThr;
        const int q = e / mc, mm = e - q * mc;
        if (e < kN * mc) sm.in.ys[mm][q] = yKeep(q, m0 + mm) ? yv[u] : 0.0f;
      }
    }
    {
      constexpr int kAIt = (kIrSlots * kMC + kThr - 1) / kThr;
      float av[kAIt];
#pragma unroll
      for (int u = 0; u < kAIt; ++u) {
        const int e = t + u * kThr;
        const int i = min(e / mc, kA - 1), mm = min(e - (e / mc) * mc, mc - 1);
        av[u] = aAt(i, m0 + mm);
      }
      hold(av);
#pragma unroll
      for (int u = 0; u < kAIt; ++u) {
        const int e = t + u * kThr;
        const int i = e / mc, mm = e - i * mc;
        if (e < kIrSlots * mc) sm.in.as[mm][phys(i)] = i < kA ? av[u] : 0.f;
      }
    }
    __syncthreads();
    if (active) {
      for (int mm = 0; mm < mc; ++mm) {
        const float* ym = sm.in.ys[mm];
        const float* am = sm.in.as[mm];
        // win[s] = a[d0 - q - 7 + s], s = 0..kR+6, for the block q .. q + 7:
        // a[d0 + r - (q + u)] = win[r - u + 7]
        int q = q0;
        for (; q + 8 <= q1; q += 8) {
          float win[kR + 7];
#pragma unroll
          for (int s = 0; s < kR + 7; ++s) {
            const int x = d0 - q - 7 + s;   // >= 1 always: d0 >= N, q <= N - 8
            win[s] = am[phys(x)];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float yv = ym[q + u];
#pragma unroll
            for (int r = 0; r < kR; ++r) acc[r] = fmaf(yv, win[r - u + 7], acc[r]);
          }
        }
        for (; q < q1; ++q) {
          const float yv = ym[q];
#pragma unroll
          for (int r = 0; r < kR; ++r) acc[r] = fmaf(yv, am[phys(d0 + r - q)], acc[r]);
        }
      }
    }
  }
  // reduce over the G q ranges (red aliases the frame / IR tiles)
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kR; ++r) sm.red[t * kR + r] = acc[r];
  __syncthreads();
  for (int e = t; e < L; e += kThr) {
    const int tl = e / kR, r = e - tl * kR;
    float s = 0.f;
    for (int gg = 0; gg < G; ++gg) s += sm.red[(gg * nTiles + tl) * kR + r];
    out(e, s);
  }
}

}  // namespace tzc
}  // namespace danse
