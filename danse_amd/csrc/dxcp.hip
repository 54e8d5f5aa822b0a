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
                                                        double* __restrict__ out) {
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
#pragma unroll
  for (int i = 0; i < kN / kThreads; ++i) {
    const int k = tid + i * kThreads;
    const cf zk = buf[k], zm = buf[(kN - k) & (kN - 1)];
    const cf x1 = 0.5f * (zk + conjg(zm));
    const cf dd = zk - conjg(zm);
    const cf x2 = cf{0.5f * dd.im, -0.5f * dd.re};   // (zk - conj zm) / (2i)
    const cf x12 = mulc(x1, x2);
    float a = sqrtf(abs2(x12));
    if (a < 1e-12f) a = 1e-12f;
    const cf g = cf{x12.re / a, x12.im / a};
    const cf avg = init ? 0.53f * gavg[k] + 0.47f * g : g;
    gavg[k] = avg;
    avgr[i] = avg;
    if (do2) {
      const cf old = cont[(size_t)slotOld * kN + k];
      const cf act = mulc(avg, old);
      cf v = init ? 0.99f * g2[k] + 0.01f * act : act;
      if (incoherent(k)) v = cf{0.0f, 0.0f};
      g2[k] = v;
      g2r[i] = conjg(v);
    }
    cont[(size_t)slotNew * kN + k] = avg;
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
        for (int m = 0; m < 2 * kLam + 1; ++m) acc = acc + g161[m] * c.t161[(tid * m) % 161];
        X81[tid] = c.wres[tid] * acc;
      }
      __syncthreads();
      for (int n = tid; n < kNUp; n += kThreads) {
        float acc = X81[0].re;
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
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int j = tid + i * kThreads;
        ar[i] = 0.0f;
        if (j < 2 * kUps + 1) {
          const float cur = buf[(j - kUps + kN) & (kN - 1)].re * (1.0f / kN);
          const float a = init ? 0.99f * c1[j] + 0.01f * cur : cur;
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

}  // namespace

struct danse_dxcp {
  int dev = 0;
  int P = 0;
  std::string err;
  DxcpState st{};
  DxcpConst c{};
  float *dWin = nullptr, *dWres = nullptr;
  cf *dTw = nullptr, *dWtw = nullptr, *dT161 = nullptr, *dT644 = nullptr;
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
                  eng->st.cont, eng->st.g2, eng->st.c1, eng->st.ps};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  delete eng;
}

int danse_dxcp_process(danse_dxcp* eng, const float* x, double* out, void* stream) {
  if (!eng || !x || !out) {
    g_derr = "null argument";
    return -1;
  }
  DCHK(hipSetDevice(eng->dev));
  hipLaunchKernelGGL(dxcp_kernel, dim3(eng->P), dim3(kThreads), 0, (hipStream_t)stream, x, eng->st, eng->c, out);
  DCHK(hipGetLastError());
  return 0;
}

}  // extern "C"
