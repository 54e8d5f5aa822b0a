// Broadcast-phase kernel of the DANSE frame-update engine (see kernels.hpp
// for the round structure): WOLA analysis, compression z = wExt^H y, WOLA
// synthesis of z and of the estimates, and the analysis of the z frame that
// every receiving node uses.  Host translation unit only (danse_engine.hip).
//
// One workgroup of 4 or 8 waves per (scene, node); every 1024-point FFT is
// owned by ONE wavefront (wfft.hpp), so the waves run independent transforms
// side by side:
//   phase 1  the broadcast-frame analyses of the node's M mics (and the
//            update-frame analyses when the update frame is not the previous
//            broadcast frame), round-robin over the waves; each wave keeps
//            its partial sum of conj(wExt) yhat in registers;
//   phase 2  wave 0: fused spectrum = sum of the wave partials (wave order),
//            z synthesis + OLA normalisation (d_base.py:1759-1868), stream
//            append (fill_buffers, d_classes.py:1185-1224) and the analysis of
//            the z frame the receivers consume (d_classes.py:1701-1807,
//            1893-1934); waves 1..3: synthesis of the previous round's
//            estimates (get_desired_sig_chunk, d_base.py:2027-2084).
//            waves 1..NW-1 take the families round-robin.
#pragma once
#include <cstdlib>

#include "fft.hpp"
#include "kernels.hpp"
#include "wfft.hpp"

namespace danse {

constexpr int kBcWaves = 4;   // waves per (scene, node) of the resident broadcast / the default bcast_kernel
// bcast_kernel's waves per workgroup: 8 when S K <= 128 workgroups would
// leave most CUs idle (N2: 32, config C: 128), else 4 (decided on the global
// S K so that node-sharded engines sum the fused spectra in the same order)
// (DANSE_BCAST_WAVES=4 / 8 forces one form: A/B timing only)
inline int bcast_waves(int S, int K) {
  static const int forced = [] {
    const char* e = std::getenv("DANSE_BCAST_WAVES");
    return e ? std::atoi(e) : 0;
  }();
  if (forced == 4 || forced == 8) return forced;
  return S * K <= 128 ? 8 : 4;
}

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
  float* zStream;          // [S][K][zLen]
  int zLen;                // samples per node stream (R*Ns for wholeChunk)
  const int* fsTab;        // fewSamples: [R][K][DANSE_FS_FIELDS] (null: wholeChunk)
  const cf* wExtHist;      // per scene block (stride wExtStride) : node offsets wExtNodeOff
  const long long* wExtNodeOff;  // [K]
  long long wExtStride;
  int wExtHistory;         // 1: index by r, 0: single slot
  const cf* dhat;          // [fam][S][K][R][F]
  float* d;                // [fam][S][K][T]
  const float* hA;         // analysis window [N]
  const float* hS;         // synthesis window [N]
  const float* normVal;    // [Ns] OLA normalisation h^2[n] + h^2[n+Ns]
  const cf* tw;            // wave-FFT twiddle table (wfft::kTwElems)
  int dbg;                 // diagnostic ablation mask (DANSE_BCAST_ABLATE; 0 in production)
  const int* cEnd;         // [R*K] raw stream end of the centralised frame (danse_cfg.cEnd) or null
  cf* Cspec;               // [2][S][MT][F] (slot r & 1)
  const float* rawStream;  // fewSamples raw streams [S][MT][zLen] (danse_cfg.rawStreams): the
                           // centralised frame is rawStream[cEnd - N, cEnd) instead of y
  // fewSamples step lists: the senders whose z frame this launch analyses
  // (bit k), and zOnly = that analysis alone (a late z frame: no local-frame
  // analyses, no estimate synthesis)
  unsigned zMask;
  int zOnly;
  // node-sharded DXCP (danse_engine_set_zchunk): the round's new z samples of
  // every owned node also go to zChunk [K][S][Ns] (node-major: a rank's block
  // is one all-gather chunk), for the other ranks' estimators
  float* zChunk;
  // node-sharded engines with centralised / SSBC families (the vectors of
  // the owned nodes read every node's raw spectra): the grid covers every
  // node, and the blocks of the nodes this engine does not own run the
  // analyses of phase 1 alone (no fused spectrum, no z, no estimates)
  int foreign;
};

// y[(frame end - N) .. frame end) * win, zero before sample 0 -> buf (complex, imag 0)
// (workgroup-cooperative form, used by the stand-alone analysis operator)
DANSE_DEV void load_frame(cf* buf, const float* __restrict__ x, int end, int N, int T,
                          const float* __restrict__ win) {
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const int idx = end - N + n;
    const float v = (idx >= 0 && idx < T) ? x[idx] : 0.0f;
    buf[n] = cf{v * win[n], 0.0f};
  }
}

// The same frame in the wave-FFT input layout (lane l: samples l + 64 j).
DANSE_DEV void load_frame_wave(cf (&v)[16], const float* __restrict__ x, int end, int T,
                               const float* __restrict__ win) {
  const int l = __lane_id();
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int n = l + 64 * j;
    const int idx = end - 1024 + n;
    const float s = (idx >= 0 && idx < T) ? x[idx] : 0.0f;
    v[j] = cf{s * win[n], 0.0f};
  }
}

// sqrt(Ns) * real(ifft(Hermitian extension of X[0..F))) through a forward
// FFT of the conjugate: input element n of the wave layout.
DANSE_DEV cf herm_ext_conj(const cf* __restrict__ X, int n, int F) {
  const cf x = X[(n < F) ? n : 1024 - n];   // (one load at a selected index: no branch)
  return (n < F) ? conjg(x) : x;
}

#ifndef DANSE_BCAST_HELPERS_ONLY   // resident.hip uses the helpers above, not the kernel
// NW waves per (scene, node): 4, or 8 when the grid is small (few scenes x
// nodes: one analysis per wave instead of two; bcast_waves)
template <int NW>
__global__ void __launch_bounds__(NW * 64) bcast_kernel(const BcastArgs a) {
  __shared__ cf fftLds[NW][wfft::kLdsElems];
  __shared__ cf part[NW][513];
  __shared__ float zq[1024];
  const int wv = threadIdx.x >> 6;
  const int N = a.N, Ns = a.Ns, F = a.F;
  const int nGrid = a.foreign ? a.K : a.k1 - a.k0;
  const int s = blockIdx.x / nGrid;
  const int k = (a.foreign ? 0 : a.k0) + blockIdx.x % nGrid;
  const bool owned = k >= a.k0 && k < a.k1;
  const float sqNs = sqrtf((float)Ns);
  const float invSqNs = 1.0f / sqNs;
  const float sc = sqNs / (float)N;
  const int r = a.r;
  cf* L = fftLds[wv];

  // ---- phase 1: analyses, per-wave partial fused spectra
  if (a.doBcast && !(a.dbg & 1)) {
    const int Mk = a.M[k];
    const int bEnd = a.bcEnd[r * a.K + k];
    const int uEnd = a.upEnd[r * a.K + k];
    const bool needUp = (r == 0) || (uEnd != a.bcEnd[(r - 1) * a.K + k]);
    // wExt[r]: history slot r, or ring slot r & 1 (the update kernels write
    // wExt[r + 1] into slot (r + 1) & 1 when the history is not kept)
    const cf* wx = a.wExtHist + (long long)s * a.wExtStride + a.wExtNodeOff[k] +
                   (long long)(a.wExtHistory ? r : (r & 1)) * F * Mk;
    cf zp[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) zp[c] = cf{0.0f, 0.0f};
    // jobs: [0, Mk) broadcast frames, then the update frames (needUp), then
    // the raw frames y[cEnd - N, cEnd) of the centralised buffers (cEnd; of
    // the senders in zMask, whose received streams are complete); a zOnly
    // launch (a late fewSamples z frame) runs only the last kind
    const bool zk = ((a.zMask >> k) & 1u) != 0u;
    const int nBc = a.zOnly ? 0 : Mk;
    const int nUp = (needUp && !a.zOnly) ? Mk : 0;
    const int nJobs = nBc + nUp + ((a.cEnd && zk) ? Mk : 0);
    for (int j = wv; j < nJobs; j += NW) {
      const int kind = (j < nBc) ? 0 : (j < nBc + nUp ? 1 : 2);
      const bool up = kind == 1;
      const int m = j - (kind == 0 ? 0 : (kind == 1 ? nBc : nBc + nUp));
      const int ch = a.base[k] + m;
      const int fend = kind == 0 ? bEnd : (kind == 1 ? uEnd : a.cEnd[r * a.K + k]);
      cf v[16];
      if (a.dbg & 8) {
        for (int jj = 0; jj < 16; ++jj) v[jj] = cf{(float)(jj + threadIdx.x), 0.0f};
      } else if (kind == 2 && a.rawStream) {
        load_frame_wave(v, a.rawStream + ((long long)s * a.MT + ch) * a.zLen, fend, a.zLen, a.hA);
      } else {
        load_frame_wave(v, a.y + ((long long)s * a.MT + ch) * a.T, fend, a.T, a.hA);
      }
      if (!(a.dbg & 64)) wfft::fft1024(v, L, a.tw);
      cf* dst = (kind == 2) ? a.Cspec + (((long long)(r & 1) * a.S + s) * a.MT + ch) * F
                            : a.Yspec + (((long long)((up ? r + 1 : r) & 1) * a.S + s) * a.MT + ch) * F;
      // (fewSamples: z comes from the T(z) chunk, no fused spectrum here)
      const bool zk0 = kind == 0 && !a.fsTab;   // (a foreign block's partial sums go unused)
      if (zk0) {
        cf w[16];   // the weights first, at clamped bins (hold())
#pragma unroll
        for (int c = 0; c < 16; ++c) w[c] = wx[(long long)min(wfft::out_index(c), F - 1) * Mk + m];
        hold(w);
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int f = wfft::out_index(c);
          if (f < F) {
            const cf Y = invSqNs * v[c];
            if (!(a.dbg & 32)) dst[f] = Y;
            zp[c] = zp[c] + ((a.dbg & 16) ? Y : cmul(w[c], Y));
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int f = wfft::out_index(c);
          if (f < F && !(a.dbg & 32)) dst[f] = invSqNs * v[c];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int f = wfft::out_index(c);
      if (f < F) part[wv][f] = zp[c];
    }
  }
  __syncthreads();
  if (!owned) return;   // (block-uniform)

  if (a.doBcast && wv == 0 && a.fsTab) {
    // (a sender outside zMask: its z frame is analysed by a later step)
    if (((a.zMask >> k) & 1u) != 0u) {
    // ---- fewSamples: the chunks are already in the stream (fs_chunk_kernel);
    // the receivers' z frame is stream[ZEND - N, ZEND) (process_incoming_
    // signals_buffers, d_classes.py:1701-1807: the last N received samples)
    const int l = __lane_id();
    const float* zs = a.zStream + ((long long)s * a.K + k) * a.zLen;
    const int zEnd = a.fsTab[((long long)r * a.K + k) * DANSE_FS_FIELDS + DANSE_FS_ZEND];
    float t[16], h[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      t[j] = zs[max(zEnd - N + l + 64 * j, 0)];
      h[j] = a.hA[l + 64 * j];
    }
    hold(t);
    hold(h);
    cf v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = cf{(zEnd - N + l + 64 * j >= 0) ? t[j] * h[j] : 0.0f, 0.0f};
    wfft::fft1024(v, L, a.tw);
    cf* Zs = a.Zspec + (((long long)(r & 1) * a.K + k) * a.S + s) * F;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int f = wfft::out_index(c);
      if (f < F) Zs[f] = invSqNs * v[c];
    }
    }
  } else if (a.doBcast && wv == 0 && !(a.dbg & 2)) {
    // ---- z synthesis: sqrt(Ns) * real(ifft(herm-ext(zhat))) * f, OLA with the previous frame
    const int l = __lane_id();
    cf v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = l + 64 * j;
      const int nn = (n < F) ? n : N - n;
      cf z = part[0][nn];
#pragma unroll
      for (int w = 1; w < NW; ++w) z = z + part[w][nn];
      if (nn == 0 || nn == F - 1) z.im = 0.0f;
      v[j] = (n < F) ? conjg(z) : z;
    }
    wfft::fft1024(v, L, a.tw);
    float* zpv = a.zPrev + ((long long)s * a.K + k) * N;
    float* zs = a.zStream + ((long long)s * a.K + k) * a.zLen;
    // every global read of the chain in one straight run (hold()): the OLA
    // state (the previous frame), the synthesis window and normalisation at
    // this lane's output positions, and the old stream samples and analysis
    // window of the z frame analysed below.  (The old samples lie before
    // r Ns; the append below writes [r Ns, (r+1) Ns).)
    const long long rs = (long long)r * Ns;
    float zpr[16], hsv[16], nvv[16], olds[16], hav[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = l + 64 * j, o = wfft::out_index(j);
      const long long idx = (long long)(r + 1) * Ns - N + n;
      zpr[j] = zpv[n];
      hsv[j] = a.hS[o];
      nvv[j] = a.normVal[min(o, Ns - 1)];
      olds[j] = zs[(idx >= 0 && idx < rs) ? idx : 0];
      hav[j] = a.hA[n];
    }
    hold(zpr);
    hold(hsv);
    hold(nvv);
    hold(olds);
    hold(hav);
    // the previous frame through LDS (zq is free until the new frame is built)
    bool nz = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      nz |= (zpr[j] != 0.0f);
      zq[l + 64 * j] = zpr[j];
    }
    const bool prevNZ = __ballot(nz) != 0ull;
    wfft::wave_sync();
    float zo[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int n = wfft::out_index(c);
      const float t = zq[min(n + Ns, N - 1)];
      zo[c] = (n < N - Ns) ? t : 0.0f;
    }
    wfft::wave_sync();
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int n = wfft::out_index(c);
      float zc = sc * v[c].re * hsv[c];
      if (prevNZ) {
        float t = zo[c];
        t += zc;
        if (n < Ns) t = t / nvv[c];
        zc = t;
      }
      zq[n] = zc;
    }
    wfft::wave_sync();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = l + 64 * j;
      zpv[n] = zq[n];
      if (n < Ns) zs[rs + n] = zq[n];
      if (n < Ns && a.zChunk) a.zChunk[((long long)k * a.S + s) * Ns + n] = zq[n];
    }
    // ---- z frame the receivers consume at round r: stream samples [(r+1)Ns - N, (r+1)Ns)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = l + 64 * j;
      const long long idx = (long long)(r + 1) * Ns - N + n;
      const float cur = zq[(idx >= rs) ? (int)(idx - rs) : 0];
      const float t = (idx < 0) ? 0.0f : (idx >= rs ? cur : olds[j]);
      v[j] = cf{t * hav[j], 0.0f};
    }
    wfft::fft1024(v, L, a.tw);
    cf* Zs = a.Zspec + (((long long)(r & 1) * a.K + k) * a.S + s) * F;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int f = wfft::out_index(c);
      if (f < F) Zs[f] = invSqNs * v[c];
    }
  }

  // ---- synthesis of the estimates of round r-1, one family per wave
  if (a.doSynth && !a.zOnly && !(a.dbg & 4)) {
    const int rp = r - 1;
    const int end = a.upEnd[rp * a.K + k];
    const int w0 = a.doBcast ? 1 : 0;
    const int nW = NW - w0;
    int job = 0;
    for (int fam = 0; fam < kMaxFam; ++fam) {
      if (!((a.families >> fam) & 1)) continue;
      if (wv == w0 + (job % nW)) {
        const cf* dh = a.dhat + ((((long long)fam * a.S + s) * a.K + k) * a.R + rp) * F;
        const int l = __lane_id();
        cf v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = herm_ext_conj(dh, l + 64 * j, F);
        wfft::fft1024(v, L, a.tw);
        float* dd = a.d + (((long long)fam * a.S + s) * a.K + k) * a.T;
        // (all reads first, at clamped indices: distinct n, so no element
        // is both read and written twice)
        float old[16], hsv[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int n = wfft::out_index(c);
          old[c] = dd[min(max(end - N + n, 0), a.T - 1)];
          hsv[c] = a.hS[n];
        }
        hold(old);
        hold(hsv);
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int idx = end - N + wfft::out_index(c);
          if (idx >= 0 && idx < a.T) dd[idx] = old[c] + sc * hsv[c] * v[c].re;
        }
      }
      ++job;
    }
  }
}
#endif

}  // namespace danse
