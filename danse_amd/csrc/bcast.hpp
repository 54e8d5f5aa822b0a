// Broadcast-phase kernel of the DANSE frame-update engine (see kernels.hpp
// for the round structure): WOLA analysis, compression z = wExt^H y, WOLA
// synthesis of z and of the estimates, and the analysis of the z frame that
// every receiving node uses.  Host translation unit only (danse_engine.hip).
#pragma once
#include "fft.hpp"
#include "kernels.hpp"

namespace danse {

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
  cf* Zspec;               // [2][K][S][F] (slot r & 1)
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
  cf* Zs = a.Zspec + (((long long)(r & 1) * a.K + k) * a.S + s) * F;
  for (int f = tid; f < F; f += blockDim.x) Zs[f] = invSqNs * out[f];
}

}  // namespace danse
