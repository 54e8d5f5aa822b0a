// DXCP-PhaT sampling-rate-offset estimator on the device
// (dxcpphat/sro_estimation.py:130-345, class DXCPPhaT, default parameters:
// fs 16 kHz, 2048-sample frames and hop, 8192-point FFT, 5 s accumulation),
// batched over P independent node pairs: one 512-thread workgroup per pair
// and input frame.  Per frame (sro_estimation.py:_stateupdate):
//   GCSD-PhaT of the Blackman-windowed 8192-sample two-channel buffer,
//     recursive average (0.53), pushed into a 40-frame container
//   CSD-2 = newest x conj(oldest), averaged (0.99), incoherent bins zeroed
//     (in the running average itself: the reference aliases it), IFFT,
//     +-80 lags, Kaiser-windowed 4x FFT upsampling (scipy.signal.resample),
//     argmax + parabolic interpolation -> SRO (ppm)
//   CCF-1 with the SRO-induced offset removed, averaged (0.99), argmax of
//     its magnitude + parabolic interpolation -> STO (samples)
// The 8192-point FFTs are eight one-wave 1024-point FFTs (wfft.hpp) of the
// decimated sequences x[8m + r] followed by radix-8 butterflies across them.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/danse_mi355x.h"
#include "wfft.hpp"
#include "fill.hpp"

using namespace danse;

namespace {

constexpr int kN = 8192;          // FFTsize_dxcp
constexpr int kFrame = 2048;      // FrameSize_input = FFTshift_dxcp
constexpr int kCont = 40;         // Cont_NumFr = AccumTime_B_NumFr + 1
constexpr int kLam = 80;          // Lambda
constexpr int kUps = 4095;        // Upsilon
constexpr int kStart = 43;        // Cont_NumFr + InvShiftFactor_NumFr - 1 + AddContWait_NumFr
constexpr int kSettle = 47;       // + SettlingCSD2avg_NumFr
constexpr double kBsmpls = 79872.0;   // B_smpls = 39 * 2048
constexpr int kNUp = 644;         // (2 Lambda + 1) * p_upsmpFac
constexpr int kThreads = 512;

// bins without coherent components (zeroed before each IFFT)
DANSE_DEV bool incoherent(int k) { return k < 40 || k >= 8153 || (k >= 3890 && k < 4303); }

struct DxcpConst {
  const float* win;     // [8192] Blackman, periodic
  const cf* tw8192;     // [8192] exp(-2 pi i m / 8192)
  const cf* wtw;        // wave-FFT table (wfft::kTwElems)
  const float* wres;    // [81] folded Kaiser(161, 5) spectrum window
  const cf* t161;       // [161] exp(-2 pi i m / 161)
  const cf* t644;       // [644] exp(+2 pi i m / 644)
};

struct DxcpPairState {
  int ell;
  int initiated;
  double sro;
  double sto;
};

struct DxcpState {
  float* ring;          // [P][2][4][2048] last four input frames
  cf* gavg;             // [P][8192]       GCSD_PhaT_avg
  cf* cont;             // [P][40][8192]   container ring
  cf* g2;               // [P][8192]       GCSD2_avg
  float* c1;            // [P][8191]       GCCF1_smShftAvg
  DxcpPairState* ps;    // [P]
};

// 8192-point FFT of z (natural order, in LDS `buf`), result in `buf`.
// Each of the 8 waves transforms x[8m + r] (r = its index), twiddles by
// W8192^(r k'), then every thread finishes two columns k' with a radix-8 DFT
// over r (in place: a thread reads and writes only its own columns).
DANSE_DEV void fft8192(cf* buf, cf (*scratch)[wfft::kLdsElems], const DxcpConst& c) {
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  cf v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = buf[8 * (l + 64 * j) + wv];
  __syncthreads();
  wfft::fft1024(v, scratch[wv], c.wtw);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int kp = wfft::out_index(q);
    buf[wv * 1024 + kp] = v[q] * c.tw8192[wv * kp];
  }
  __syncthreads();
  for (int kp = threadIdx.x; kp < 1024; kp += kThreads) {
    cf y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) y[r] = buf[r * 1024 + kp];
    // X[kp + 1024 s] = sum_r W8^(r s) y_r
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      cf acc = y[0];
#pragma unroll
      for (int r = 1; r < 8; ++r) acc = acc + y[r] * c.tw8192[((r * s) & 7) * 1024];
      buf[s * 1024 + kp] = acc;
    }
  }
  __syncthreads();
}

// argmax (first maximum) over the workgroup: value / index pairs in LDS.
DANSE_DEV int block_argmax(float v, int idx, float* rv, int* ri) {
  const int t = threadIdx.x;
  rv[t] = v;
  ri[t] = idx;
  __syncthreads();
  for (int w = kThreads / 2; w > 0; w >>= 1) {
    if (t < w) {
      const float a = rv[t], b = rv[t + w];
      const int ia = ri[t], ib = ri[t + w];
      if (b > a || (b == a && ib < ia)) {
        rv[t] = b;
        ri[t] = ib;
      }
    }
    __syncthreads();
  }
  const int r = ri[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(kThreads) dxcp_kernel(const float* __restrict__ x, DxcpState st, DxcpConst c,
                                                        const double* __restrict__ tdoa, double* __restrict__ out) {
  __shared__ cf buf[kN];
  __shared__ cf scratch[8][wfft::kLdsElems];
  __shared__ float up[kNUp];
  __shared__ float g161[2 * kLam + 1];
  __shared__ cf X81[81];
  __shared__ float rv[kThreads];
  __shared__ int ri[kThreads];
  const int p = blockIdx.x;
  const int tid = threadIdx.x;
  DxcpPairState ps = st.ps[p];
  const int ell = ps.ell;
  const bool init = ps.initiated != 0;
  const float* xin = x + (size_t)p * 2 * kFrame;
  const float* ring = st.ring + (size_t)p * 2 * 4 * kFrame;

  // ---- windowed two-channel buffer (frames ell-3 .. ell), packed x1 + i x2
  for (int n = tid; n < kN; n += kThreads) {
    const int fi = n / kFrame, o = n % kFrame;
    float a, b;
    if (fi == 3) {
      a = xin[o];
      b = xin[kFrame + o];
    } else {
      const int slot = (ell + fi) & 3;
      a = ring[(0 * 4 + slot) * kFrame + o];
      b = ring[(1 * 4 + slot) * kFrame + o];
    }
    buf[n] = cf{a * c.win[n], b * c.win[n]};
  }
  __syncthreads();
  fft8192(buf, scratch, c);

  // ---- GCSD-PhaT, its average, the container, CSD-2
  cf* gavg = st.gavg + (size_t)p * kN;
  cf* cont = st.cont + (size_t)p * kCont * kN;
  cf* g2 = st.g2 + (size_t)p * kN;
  const int slotNew = (ell - 1) % kCont, slotOld = ell % kCont;
  const bool do2 = ell >= kStart;
  cf avgr[kN / kThreads], g2r[kN / kThreads];
  // the state a chunk of this thread's bins reads, loaded before the chunk's
  // first store (a store holds every later load behind it: one memory round
  // trip per bin); init / do2 are uniform per pair.  Two chunks of eight:
  // the registers of all sixteen would spill.
  constexpr int kPer = kN / kThreads, kChunk = 8;
#pragma unroll
  for (int i0 = 0; i0 < kPer; i0 += kChunk) {
    cf gavgOld[kChunk], contOld[kChunk], g2Old[kChunk];
    if (init) {
#pragma unroll
      for (int u = 0; u < kChunk; ++u) gavgOld[u] = gavg[tid + (i0 + u) * kThreads];
      hold(gavgOld);
    }
    if (do2) {
#pragma unroll
      for (int u = 0; u < kChunk; ++u) contOld[u] = cont[(size_t)slotOld * kN + tid + (i0 + u) * kThreads];
      hold(contOld);
    }
    if (do2 && init) {
#pragma unroll
      for (int u = 0; u < kChunk; ++u) g2Old[u] = g2[tid + (i0 + u) * kThreads];
      hold(g2Old);
    }
#pragma unroll
    for (int u = 0; u < kChunk; ++u) {
      const int i = i0 + u;
      const int k = tid + i * kThreads;
      const cf zk = buf[k], zm = buf[(kN - k) & (kN - 1)];
      const cf x1 = 0.5f * (zk + conjg(zm));
      const cf dd = zk - conjg(zm);
      const cf x2 = cf{0.5f * dd.im, -0.5f * dd.re};   // (zk - conj zm) / (2i)
      const cf x12 = mulc(x1, x2);
      float a = sqrtf(abs2(x12));
      if (a < 1e-12f) a = 1e-12f;
      const cf g = cf{x12.re / a, x12.im / a};
      const cf avg = init ? 0.53f * gavgOld[u] + 0.47f * g : g;
      gavg[k] = avg;
      avgr[i] = avg;
      if (do2) {
        const cf act = mulc(avg, contOld[u]);
        cf v = init ? 0.99f * g2Old[u] + 0.01f * act : act;
        if (incoherent(k)) v = cf{0.0f, 0.0f};
        g2[k] = v;
        g2r[i] = conjg(v);
      }
      cont[(size_t)slotNew * kN + k] = avg;
    }
  }
  __syncthreads();

  double sro = ps.sro, sto = ps.sto;
  if (do2) {
    // ---- CCF-2: real(ifft(GCSD2)), lags -80..80
#pragma unroll
    for (int i = 0; i < kN / kThreads; ++i) buf[tid + i * kThreads] = g2r[i];
    __syncthreads();
    fft8192(buf, scratch, c);
    if (tid < 2 * kLam + 1) g161[tid] = buf[(tid - kLam + kN) & (kN - 1)].re * (1.0f / kN);
    __syncthreads();
    if (ell >= kSettle) {
      // scipy.signal.resample(x, 644, window=kaiser(161, 5)): rfft, folded
      // window, zero-padded irfft times 644 / 161
      if (tid < 81) {
        cf acc = cf{0.0f, 0.0f};
        // (unrolled: the table reads of 7 taps issue together, the sum keeps its order)
#pragma unroll 7
        for (int m = 0; m < 2 * kLam + 1; ++m) acc = acc + g161[m] * c.t161[(tid * m) % 161];
        X81[tid] = c.wres[tid] * acc;
      }
      __syncthreads();
      for (int n = tid; n < kNUp; n += kThreads) {
        float acc = X81[0].re;
#pragma unroll 8
        for (int k = 1; k < 81; ++k) {
          const cf e = c.t644[(k * n) % kNUp];
          acc += 2.0f * (X81[k].re * e.re - X81[k].im * e.im);
        }
        up[n] = acc * (4.0f / kNUp);
      }
      __syncthreads();
      float bv = -3.0e38f;
      int bi = 0x7fffffff;
      for (int n = tid; n < kNUp; n += kThreads)
        if (up[n] > bv) { bv = up[n]; bi = n; }
      const int im = block_argmax(bv, bi, rv, ri);
      double frac = 0.0;
      if (im > 0 && im < kNUp - 1) {
        const double s0 = up[im - 1], s1 = up[im], s2 = up[im + 1];
        frac = (s2 - s0) / 2.0 / (2.0 * s1 - s2 - s0);
      }
      sro = ((-kLam + 0.25 * im) + frac / 4.0) / kBsmpls * 1e6;

      // ---- STO: CCF-1 with the SRO-induced time offset removed
      const double tOff = sro * 1e-6 * kFrame * (ell - 1);
#pragma unroll
      for (int i = 0; i < kN / kThreads; ++i) {
        const int k = tid + i * kThreads;
        double t = tOff * (double)k / (double)kN;
        t -= floor(t);
        float sn, cs;
        sincospif(2.0f * (float)t, &sn, &cs);
        cf v = avgr[i] * cf{cs, sn};
        if (incoherent(k)) v = cf{0.0f, 0.0f};
        buf[k] = conjg(v);
      }
      __syncthreads();
      fft8192(buf, scratch, c);
      float* c1 = st.c1 + (size_t)p * (2 * kUps + 1);
      float ar[16];
      float bv1 = -1.0f;
      int bi1 = 0x7fffffff;
      float c1Old[16];   // (read before the stores below, clamped; hold())
      if (init) {
#pragma unroll
        for (int i = 0; i < 16; ++i) c1Old[i] = c1[min(tid + i * kThreads, 2 * kUps)];
        hold(c1Old);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int j = tid + i * kThreads;
        ar[i] = 0.0f;
        if (j < 2 * kUps + 1) {
          const float cur = buf[(j - kUps + kN) & (kN - 1)].re * (1.0f / kN);
          const float a = init ? 0.99f * c1Old[i] + 0.01f * cur : cur;
          c1[j] = a;
          ar[i] = fabsf(a);
          if (ar[i] > bv1) { bv1 = ar[i]; bi1 = j; }
        }
      }
      const int im1 = block_argmax(bv1, bi1, rv, ri);
      // the three supporting points, from the registers of their owners
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int j = tid + i * kThreads;
        if (j >= im1 - 1 && j <= im1 + 1) rv[j - im1 + 1] = ar[i];
      }
      __syncthreads();
      if (im1 == 0 || im1 == 2 * kUps) {
        sto = (double)(im1 - kUps);
      } else {
        const double s0 = rv[0], s1 = rv[1], s2 = rv[2];
        sto = (double)(im1 - kUps) + (s2 - s0) / 2.0 / (2.0 * s1 - s2 - s0);
        // TDOA correction, interior maxima only (sro_estimation.py:338-339)
        if (tdoa) sto += tdoa[p] * 16000.0;
      }
    }
  }

  // ---- keep the frame for the next calls, advance the counters
  float* wring = st.ring + (size_t)p * 2 * 4 * kFrame;
  const int slot = (ell + 3) & 3;
  for (int o = tid; o < kFrame; o += kThreads) {
    wring[(0 * 4 + slot) * kFrame + o] = xin[o];
    wring[(1 * 4 + slot) * kFrame + o] = xin[kFrame + o];
  }
  if (tid == 0) {
    DxcpPairState n = ps;
    n.ell = ell + 1;
    n.initiated = 1;
    n.sro = sro;
    n.sto = sto;
    st.ps[p] = n;
    out[2 * p] = sro;
    out[2 * p + 1] = sto;
  }
}

// ---- closed loop (CL_DXCPPhaT, sro_estimation.py:12-72) -------------------
// Per pair: OnlineResampler (online_resampler.py:4-77) of z_i with the
// controller's current estimate, DelayBuffer (delay_buffer.py:8-26) of z_j,
// DXCP-PhaT on the synchronised pair, IMC controller (PIT1, Tf = 8).
struct ClPair {
  double shift;          // Resampler.shift
  double dS[3], S[3];    // dSRO_est, SRO_est (newest first)
  double sroCurr;        // SRO_est_curr
  int ell;               // CL_DXCPPhaT.ell
  int zjPtr;             // DelayBuffer.pointer
};

struct ClState {
  float* inBuf;          // [P][4 * 2048]  prev - current - next - next2
  float* outBuf;         // [P][3 * 2048]
  float* zj;             // [P][3][2048]   delay ring (2 + 1 frames)
  float* x12;            // [P][2][2048]   the DXCP input of this frame
  ClPair* cp;            // [P]
};

constexpr int kB = kFrame;   // blockSize

// hann(4096, sym=False)
DANSE_DEV float hann4096(int n) { return (float)(0.5 - 0.5 * cos(2.0 * M_PI * (double)n / (double)(2 * kB))); }

__global__ void __launch_bounds__(kThreads) cl_resample_kernel(const float* __restrict__ x, ClState st, DxcpConst c,
                                                               float* __restrict__ ziOut) {
  __shared__ cf buf[kN];
  __shared__ cf scratch[8][wfft::kLdsElems];
  __shared__ int sel0;
  __shared__ double rest;
  const int p = blockIdx.x, tid = threadIdx.x;
  float* in = st.inBuf + (size_t)p * 4 * kB;
  float* ob = st.outBuf + (size_t)p * 3 * kB;
  const float* zi = x + ((size_t)p * 2 + 1) * kB;
  const float* zjIn = x + ((size_t)p * 2 + 0) * kB;
  // the input buffer shifted by one block, the new block appended
  auto nin = [&](int n) { return (n < 3 * kB) ? in[n + kB] : zi[n - 3 * kB]; };
  if (tid == 0) {
    ClPair cp = st.cp[p];
    const double sro = -cp.sroCurr;
    cp.shift += sro * 1e-6 * kB;
    const double acc = cp.shift;
    const double ish = rint(acc);   // np.round: half to even
    rest = ish - acc;
    long long s0 = (long long)kB + (long long)ish, s1 = (long long)3 * kB + (long long)ish;
    if (s0 < 0) {
      cp.shift -= sro * 1e-6 * kB;
      s1 -= s0;
      s0 = 0;
    } else if (s1 >= 4 * kB) {
      cp.shift -= sro * 1e-6 * kB;
      s0 -= s1 - 4 * kB;
      s1 = 4 * kB;
    }
    sel0 = (int)s0;
    st.cp[p] = cp;
  }
  __syncthreads();
  for (int n = tid; n < kN; n += kThreads) buf[n] = cf{n < 2 * kB ? hann4096(n) * nin(sel0 + n) : 0.0f, 0.0f};
  {
    // shift the stored buffer in place: every read before any write
    float v[4 * kB / kThreads];
#pragma unroll
    for (int i = 0; i < 4 * kB / kThreads; ++i) v[i] = nin(tid + i * kThreads);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4 * kB / kThreads; ++i) in[tid + i * kThreads] = v[i];
  }
  __syncthreads();
  fft8192(buf, scratch, c);
  // linear phase of the rest shift on the fftshift'ed bin index, then
  // ifft = conj(fft(conj(.))) / N
  const double rs = rest;
  for (int m = tid; m < kN; m += kThreads) {
    const int k = m < kN / 2 ? m : m - kN;
    double t = (double)k * rs / (double)kN;
    t -= rint(t);
    float sn, cs;
    sincospif(-2.0f * (float)t, &sn, &cs);
    buf[m] = conjg(buf[m] * cf{cs, sn});
  }
  __syncthreads();
  fft8192(buf, scratch, c);
  // overlap-add into blocks 2-3 of the output buffer, shift it by one block
  float* zo = st.x12 + ((size_t)p * 2 + 1) * kB;
  for (int n = tid; n < 2 * kB; n += kThreads) {
    const float y = buf[n].re * (1.0f / kN);   // real(conj(.)) / N
    const float v = ob[kB + n] + y;
    if (n < kB) {
      zo[n] = v;
      if (ziOut) ziOut[(size_t)p * kB + n] = v;
    }
    __syncthreads();   // every read of ob before the shifted writes
    ob[n] = v;
  }
  for (int n = tid; n < kB; n += kThreads) ob[2 * kB + n] = 0.0f;
  // z_j through the delay ring: write at the pointer, read the oldest
  const int ptr = st.cp[p].zjPtr;
  float* ring = st.zj + (size_t)p * 3 * kB;
  float* zjo = st.x12 + ((size_t)p * 2 + 0) * kB;
  for (int n = tid; n < kB; n += kThreads) {
    ring[(size_t)ptr * kB + n] = zjIn[n];
    zjo[n] = ring[(size_t)((ptr + 1) % 3) * kB + n];
  }
  __syncthreads();
  if (tid == 0) st.cp[p].zjPtr = (ptr + 1) % 3;
}

// IMC controller update after DXCP-PhaT (sro_estimation.py:56-70)
__global__ void cl_control_kernel(ClState st, int P, int startDelay, const int* __restrict__ acs,
                                  const double* __restrict__ dx, double* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const double kNom[3] = {0.0, 0.0251941968627353, -0.0249422548941180};
  const double kDen[3] = {1.0, -1.96825464010938, 0.968254640109407};
  ClPair cp = st.cp[p];
  const double raw = dx[2 * p];
  double d = (!acs || acs[p] == 1) ? raw : 0.0;
  if (cp.ell <= startDelay) d = 0.0;
  cp.dS[2] = cp.dS[1];
  cp.dS[1] = cp.dS[0];
  cp.dS[0] = d;
  cp.S[2] = cp.S[1];
  cp.S[1] = cp.S[0];
  cp.S[0] = (kNom[0] * cp.dS[0] + kNom[1] * cp.dS[1] + kNom[2] * cp.dS[2]) - (kDen[1] * cp.S[1] + kDen[2] * cp.S[2]);
  cp.sroCurr = cp.S[0] + 0.0;   // + SRO_est_op
  cp.ell += 1;
  st.cp[p] = cp;
  out[3 * p] = raw;
  out[3 * p + 1] = cp.sroCurr;
  out[3 * p + 2] = cp.shift;
}

}  // namespace

struct danse_dxcp {
  int dev = 0;
  int P = 0;
  std::string err;
  DxcpState st{};
  DxcpConst c{};
  float *dWin = nullptr, *dWres = nullptr;
  cf *dTw = nullptr, *dWtw = nullptr, *dT161 = nullptr, *dT644 = nullptr;
  // closed loop (danse_cl_dxcp_*): resampler / delay / controller state
  ClState cl{};
  int startDelay = 0;
  double* dxOut = nullptr;   // [P][2] DXCP output of the current frame
};

static thread_local std::string g_derr;

#define DCHK(expr)                                                                  \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      std::string m = std::string(#expr) + ": " + hipGetErrorString(_e);            \
      if (eng) eng->err = m;                                                        \
      g_derr = m;                                                                   \
      return -2;                                                                    \
    }                                                                               \
  } while (0)

extern "C" {

const char* danse_dxcp_last_error(const danse_dxcp* eng) {
  if (eng && !eng->err.empty()) return eng->err.c_str();
  return g_derr.c_str();
}

int danse_dxcp_create(int32_t P, int device, danse_dxcp** out) {
  danse_dxcp* eng = nullptr;
  if (P < 1 || !out) {
    g_derr = "bad arguments";
    return -1;
  }
  eng = new danse_dxcp();
  eng->dev = device;
  eng->P = P;
  DCHK(hipSetDevice(device));
  std::vector<float> win(kN), wres(81);
  std::vector<cf> tw(kN), t161(161), t644(kNUp), wtw;
  for (int n = 0; n < kN; ++n) {   // scipy.signal.windows.blackman(8192, sym=False)
    const double a = 2.0 * M_PI * n / kN;
    win[n] = (float)(0.42 - 0.5 * std::cos(a) + 0.08 * std::cos(2.0 * a));
    tw[n] = cf{(float)std::cos(-a), (float)std::sin(-a)};
  }
  {
    // kaiser(161, 5), symmetric; folded as scipy.signal.resample does for real input
    std::vector<double> kw(161);
    auto i0 = [](double x) {
      double s = 1.0, t = 1.0;
      for (int k = 1; k < 60; ++k) {
        t *= (x / 2.0) * (x / 2.0) / ((double)k * k);
        s += t;
      }
      return s;
    };
    for (int n = 0; n < 161; ++n) {
      const double r = 2.0 * n / 160.0 - 1.0;
      kw[n] = i0(5.0 * std::sqrt(std::max(0.0, 1.0 - r * r))) / i0(5.0);
    }
    std::vector<double> wr = kw;
    for (int n = 1; n < 161; ++n) wr[n] += kw[161 - n];
    for (int n = 1; n < 161; ++n) wr[n] *= 0.5;
    for (int n = 0; n < 81; ++n) wres[n] = (float)wr[n];
  }
  for (int m = 0; m < 161; ++m) t161[m] = cf{(float)std::cos(-2.0 * M_PI * m / 161.0), (float)std::sin(-2.0 * M_PI * m / 161.0)};
  for (int m = 0; m < kNUp; ++m)
    t644[m] = cf{(float)std::cos(2.0 * M_PI * m / kNUp), (float)std::sin(2.0 * M_PI * m / kNUp)};
  for (int k1 = 0; k1 < 16; ++k1)
    for (int l = 0; l < 64; ++l) {
      const double ang = -2.0 * M_PI * (double)(l * k1) / 1024.0;
      wtw.push_back(cf{(float)std::cos(ang), (float)std::sin(ang)});
    }
  for (int a4 = 0; a4 < 4; ++a4)
    for (int cc = 0; cc < 16; ++cc) {
      const double ang = -2.0 * M_PI * (double)(a4 * cc) / 64.0;
      wtw.push_back(cf{(float)std::cos(ang), (float)std::sin(ang)});
    }
  DCHK(hipMalloc((void**)&eng->dWin, kN * sizeof(float)));
  DCHK(hipMalloc((void**)&eng->dWres, 81 * sizeof(float)));
  DCHK(hipMalloc((void**)&eng->dTw, kN * sizeof(cf)));
  DCHK(hipMalloc((void**)&eng->dWtw, wtw.size() * sizeof(cf)));
  DCHK(hipMalloc((void**)&eng->dT161, 161 * sizeof(cf)));
  DCHK(hipMalloc((void**)&eng->dT644, kNUp * sizeof(cf)));
  DCHK(hipMemcpy(eng->dWin, win.data(), kN * sizeof(float), hipMemcpyHostToDevice));
  DCHK(hipMemcpy(eng->dWres, wres.data(), 81 * sizeof(float), hipMemcpyHostToDevice));
  DCHK(hipMemcpy(eng->dTw, tw.data(), kN * sizeof(cf), hipMemcpyHostToDevice));
  DCHK(hipMemcpy(eng->dWtw, wtw.data(), wtw.size() * sizeof(cf), hipMemcpyHostToDevice));
  DCHK(hipMemcpy(eng->dT161, t161.data(), 161 * sizeof(cf), hipMemcpyHostToDevice));
  DCHK(hipMemcpy(eng->dT644, t644.data(), kNUp * sizeof(cf), hipMemcpyHostToDevice));
  eng->c = DxcpConst{eng->dWin, eng->dTw, eng->dWtw, eng->dWres, eng->dT161, eng->dT644};
  const size_t nRing = (size_t)P * 2 * 4 * kFrame, nG = (size_t)P * kN, nC = (size_t)P * kCont * kN,
               nC1 = (size_t)P * (2 * kUps + 1);
  DCHK(hipMalloc((void**)&eng->st.ring, nRing * sizeof(float)));
  DCHK(hipMalloc((void**)&eng->st.gavg, nG * sizeof(cf)));
  DCHK(hipMalloc((void**)&eng->st.cont, nC * sizeof(cf)));
  DCHK(hipMalloc((void**)&eng->st.g2, nG * sizeof(cf)));
  DCHK(hipMalloc((void**)&eng->st.c1, nC1 * sizeof(float)));
  DCHK(hipMalloc((void**)&eng->st.ps, (size_t)P * sizeof(DxcpPairState)));
  DCHK(hipMemset(eng->st.ring, 0, nRing * sizeof(float)));
  DCHK(hipMemset(eng->st.gavg, 0, nG * sizeof(cf)));
  DCHK(hipMemset(eng->st.cont, 0, nC * sizeof(cf)));
  DCHK(hipMemset(eng->st.g2, 0, nG * sizeof(cf)));
  DCHK(hipMemset(eng->st.c1, 0, nC1 * sizeof(float)));
  std::vector<DxcpPairState> ps(P, DxcpPairState{1, 0, 0.0, 0.0});
  DCHK(hipMemcpy(eng->st.ps, ps.data(), (size_t)P * sizeof(DxcpPairState), hipMemcpyHostToDevice));
  *out = eng;
  return 0;
}

void danse_dxcp_destroy(danse_dxcp* eng) {
  if (!eng) return;
  (void)hipSetDevice(eng->dev);
  void* ptrs[] = {eng->dWin, eng->dWres, eng->dTw, eng->dWtw, eng->dT161, eng->dT644, eng->st.ring, eng->st.gavg,
                  eng->st.cont, eng->st.g2, eng->st.c1, eng->st.ps, eng->cl.inBuf, eng->cl.outBuf, eng->cl.zj,
                  eng->cl.x12, eng->cl.cp, eng->dxOut};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  delete eng;
}

__global__ void dxcp_reset_ps_kernel(DxcpPairState* ps, int P) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < P) ps[p] = DxcpPairState{1, 0, 0.0, 0.0};
}

int danse_dxcp_reset(danse_dxcp* eng, void* stream) {
  if (!eng) {
    g_derr = "null argument";
    return -1;
  }
  DCHK(hipSetDevice(eng->dev));
  hipStream_t st = (hipStream_t)stream;
  const size_t P = (size_t)eng->P;
  DCHK(fill_async(eng->st.ring, 0, P * 2 * 4 * kFrame * sizeof(float), st));
  DCHK(fill_async(eng->st.gavg, 0, P * kN * sizeof(cf), st));
  DCHK(fill_async(eng->st.cont, 0, P * kCont * kN * sizeof(cf), st));
  DCHK(fill_async(eng->st.g2, 0, P * kN * sizeof(cf), st));
  DCHK(fill_async(eng->st.c1, 0, P * (2 * kUps + 1) * sizeof(float), st));
  hipLaunchKernelGGL(dxcp_reset_ps_kernel, dim3((eng->P + 63) / 64), dim3(64), 0, st, eng->st.ps, eng->P);
  DCHK(hipGetLastError());
  if (eng->cl.cp) {
    DCHK(fill_async(eng->cl.inBuf, 0, P * 4 * kB * sizeof(float), st));
    DCHK(fill_async(eng->cl.outBuf, 0, P * 3 * kB * sizeof(float), st));
    DCHK(fill_async(eng->cl.zj, 0, P * 3 * kB * sizeof(float), st));
    DCHK(fill_async(eng->cl.cp, 0, P * sizeof(ClPair), st));
  }
  return 0;
}

int danse_dxcp_process(danse_dxcp* eng, const float* x, double* out, void* stream) {
  if (!eng || !x || !out) {
    g_derr = "null argument";
    return -1;
  }
  DCHK(hipSetDevice(eng->dev));
  hipLaunchKernelGGL(dxcp_kernel, dim3(eng->P), dim3(kThreads), 0, (hipStream_t)stream, x, eng->st, eng->c,
                     (const double*)nullptr, out);
  DCHK(hipGetLastError());
  return 0;
}

int danse_dxcp_process_tdoa(danse_dxcp* eng, const float* x, const double* tdoa, double* out, void* stream) {
  if (!eng || !x || !out) {
    g_derr = "null argument";
    return -1;
  }
  DCHK(hipSetDevice(eng->dev));
  hipLaunchKernelGGL(dxcp_kernel, dim3(eng->P), dim3(kThreads), 0, (hipStream_t)stream, x, eng->st, eng->c, tdoa, out);
  DCHK(hipGetLastError());
  return 0;
}

int danse_cl_dxcp_create(int32_t P, int32_t startDelay, int device, danse_dxcp** out) {
  danse_dxcp* eng = nullptr;
  const int rc = danse_dxcp_create(P, device, &eng);
  if (rc) return rc;
  eng->startDelay = startDelay;
  ClState& c = eng->cl;
  DCHK(hipMalloc((void**)&c.inBuf, (size_t)P * 4 * kB * sizeof(float)));
  DCHK(hipMalloc((void**)&c.outBuf, (size_t)P * 3 * kB * sizeof(float)));
  DCHK(hipMalloc((void**)&c.zj, (size_t)P * 3 * kB * sizeof(float)));
  DCHK(hipMalloc((void**)&c.x12, (size_t)P * 2 * kB * sizeof(float)));
  DCHK(hipMalloc((void**)&c.cp, (size_t)P * sizeof(ClPair)));
  DCHK(hipMalloc((void**)&eng->dxOut, (size_t)P * 2 * sizeof(double)));
  DCHK(hipMemset(c.inBuf, 0, (size_t)P * 4 * kB * sizeof(float)));
  DCHK(hipMemset(c.outBuf, 0, (size_t)P * 3 * kB * sizeof(float)));
  DCHK(hipMemset(c.zj, 0, (size_t)P * 3 * kB * sizeof(float)));
  DCHK(hipMemset(c.x12, 0, (size_t)P * 2 * kB * sizeof(float)));
  DCHK(hipMemset(c.cp, 0, (size_t)P * sizeof(ClPair)));
  *out = eng;
  return 0;
}

int danse_cl_dxcp_process(danse_dxcp* eng, const float* x, const int32_t* acs, double* out, float* zi, void* stream) {
  if (!eng || !x || !out || !eng->cl.cp) {
    g_derr = "null argument or not a closed-loop engine";
    return -1;
  }
  DCHK(hipSetDevice(eng->dev));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(cl_resample_kernel, dim3(eng->P), dim3(kThreads), 0, st, x, eng->cl, eng->c, zi);
  hipLaunchKernelGGL(dxcp_kernel, dim3(eng->P), dim3(kThreads), 0, st, (const float*)eng->cl.x12, eng->st, eng->c,
                     (const double*)nullptr, eng->dxOut);
  hipLaunchKernelGGL(cl_control_kernel, dim3((eng->P + 63) / 64), dim3(64), 0, st, eng->cl, eng->P, eng->startDelay, acs,
                     (const double*)eng->dxOut, out);
  DCHK(hipGetLastError());
  return 0;
}

}  // extern "C"
