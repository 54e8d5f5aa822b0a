// T(z) few-samples compression on the device:
//   danse_tz_ir       = dist_fct_approx        (d_base.py:1941-1991)
//   danse_tz_compress = danse_compression_few_samples' convolution
//                       (d_base.py:1871-1938, 1538-1566)
//
// dist_fct_approx sums the offset diagonals of diag(f) C diag(h), C the
// circulant of flip(w_td), w_td = real(IFFT(Hermitian-extended conj(wHat))).
// The tau-th diagonal of that matrix has the constant circulant entry
// c[(-tau) mod N], so
//     wIR[i] = w_td[i mod N] * S[i] / R,   i = tau + N - 1 in [0, 2N - 2],
//     S[i]   = sum_n f[n] h[n + i - N + 1]       (window cross-correlation)
// and, w_td being real, w_td = Re(FFT(Y)) / N with Y the Hermitian extension
// of wHat itself.  One wavefront per (filter, sensor): one wave FFT
// (wfft.hpp), then 2N - 1 scaled stores.  S / (N R) is a host-built double
// table (windows only, like the twiddles).
//
// The convolution keeps only the L samples the node broadcasts:
//     z[ii] = sum_m sum_q yq[q][m] wIR[id_ii - q][m],  id_ii = 2N - 1 - L + 1 + ii
// (taps outside [0, 2N - 2] are the reference's zero padding).  One 256-thread
// workgroup per filter; the frame and the IR of up to kMC sensors sit in LDS.
// A thread owns kR = 8 consecutive outputs over a contiguous range of q and
// slides a 15-tap window through the IR, so every LDS read feeds 4 FMAs; the
// IR is stored with one pad slot per 8 taps so the 64 lanes of a wave (output
// blocks 8 apart) hit 64 distinct banks.  Partial sums over the q ranges are
// reduced through LDS.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/danse_mi355x.h"
#include "wfft.hpp"

using namespace danse;

namespace {

constexpr int kN = 1024;
constexpr int kA = 2 * kN - 1;          // IR length
constexpr int kR = 8;                   // outputs per thread
constexpr int kMC = 4;                  // sensors per LDS pass
constexpr int kThr = 256;
constexpr int kIrPad = 16;              // zero taps past the IR end (tile overhang)
constexpr int kIrSlots = kA + kIrPad;
DANSE_DEV int phys(int x) { return x + (x >> 3); }
constexpr int kIrPhys = kIrSlots + kIrSlots / 8 + 1;

// ---- dist_fct_approx --------------------------------------------------------
// grid: (ceil(B*M / 4)), block 256: wave w handles item (b, m) = blockIdx*4 + w
__global__ __launch_bounds__(256) void tz_ir_kernel(const cf* __restrict__ wHat, int BM, int M,
                                                    const cf* __restrict__ tw, const float* __restrict__ sn,
                                                    float* __restrict__ wIR) {
  __shared__ cf lds[4][wfft::kLdsElems];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + wv;
  if (item >= BM) return;   // whole wave exits together
  const int b = item / M, m = item - b * M;
  const cf* w = wHat + (size_t)b * (kN / 2 + 1) * M + m;
  cf v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = l + 64 * j;
    cf y;
    if (k == 0 || k == kN / 2) {
      y = cf{w[(size_t)k * M].re, 0.f};            // DC / Nyquist forced real (d_base.py:1522-1523)
    } else if (k < kN / 2) {
      y = w[(size_t)k * M];
    } else {
      y = conjg(w[(size_t)(kN - k) * M]);
    }
    v[j] = y;
  }
  wfft::fft1024(v, lds[wv], tw);
  float* o = wIR + (size_t)b * kA * M + m;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int t = wfft::out_index(c);
    const float wt = v[c].re;
    o[(size_t)t * M] = wt * sn[t];
    if (t < kN - 1) o[(size_t)(t + kN) * M] = wt * sn[t + kN];
  }
}

// ---- few-samples convolution ---------------------------------------------
// grid: B, block 256.  nTiles = ceil(L / kR) output tiles, G = 256 / nTiles
// q ranges (G >= 1 since L <= N = 1024 -> nTiles <= 128).
__global__ __launch_bounds__(kThr) void tz_compress_kernel(const float* __restrict__ yq, const float* __restrict__ wIR,
                                                           int M, int L, float* __restrict__ z) {
  __shared__ float ys[kMC][kN];
  __shared__ float as[kMC][kIrPhys];
  __shared__ float red[kThr * kR];
  const int b = blockIdx.x, t = threadIdx.x;
  const int nTiles = (L + kR - 1) / kR;
  const int G = kThr / nTiles;
  const int tile = t % nTiles, g = t / nTiles;
  const bool active = g < G;
  const int qc = (kN + G - 1) / G;
  const int q0 = min(kN, g * qc), q1 = min(kN, q0 + qc);
  const int d0 = kA - L + 1 + tile * kR;   // convolution index of this thread's first output
  float acc[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) acc[r] = 0.f;
  const float* y = yq + (size_t)b * kN * M;
  const float* a = wIR + (size_t)b * kA * M;
  for (int m0 = 0; m0 < M; m0 += kMC) {
    const int mc = min(kMC, M - m0);
    __syncthreads();   // previous pass's reads are done
    for (int e = t; e < kN * mc; e += kThr) {
      const int q = e / mc, mm = e - q * mc;
      ys[mm][q] = y[(size_t)q * M + m0 + mm];
    }
    for (int e = t; e < kIrSlots * mc; e += kThr) {
      const int i = e / mc, mm = e - i * mc;
      as[mm][phys(i)] = i < kA ? a[(size_t)i * M + m0 + mm] : 0.f;
    }
    __syncthreads();
    if (active) {
      for (int mm = 0; mm < mc; ++mm) {
        const float* ym = ys[mm];
        const float* am = as[mm];
        // win[s] = a[d0 - q - 7 + s], s = 0..14, for the block q .. q + 7:
        // a[d0 + r - (q + u)] = win[r - u + 7]
        int q = q0;
        for (; q + 8 <= q1; q += 8) {
          float win[15];
#pragma unroll
          for (int s = 0; s < 15; ++s) {
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
  // reduce over the G q ranges
#pragma unroll
  for (int r = 0; r < kR; ++r) red[t * kR + r] = acc[r];
  __syncthreads();
  for (int e = t; e < L; e += kThr) {
    const int tl = e / kR, r = e - tl * kR;
    float s = 0.f;
    for (int gg = 0; gg < G; ++gg) s += red[(gg * nTiles + tl) * kR + r];
    z[(size_t)b * L + e] = s;
  }
}

}  // namespace

struct danse_tz {
  int dev = 0;
  int R = 1;
  std::string err;
  cf* dTw = nullptr;
  float* dSn = nullptr;
};

static thread_local std::string g_terr;

#define TCHK(expr)                                                                  \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      std::string m_ = std::string(#expr) + ": " + hipGetErrorString(_e);           \
      if (eng) eng->err = m_;                                                       \
      g_terr = m_;                                                                  \
      return -2;                                                                    \
    }                                                                               \
  } while (0)

extern "C" {

const char* danse_tz_last_error(const danse_tz* eng) {
  if (eng && !eng->err.empty()) return eng->err.c_str();
  return g_terr.c_str();
}

int danse_tz_create(int32_t N, const float* h, const float* f, int32_t R, int device, danse_tz** out) {
  danse_tz* eng = nullptr;
  if (!out || !h || !f || R < 1) {
    g_terr = "bad arguments";
    return -1;
  }
  if (N != kN) {
    g_terr = "only DFTsize 1024 is supported by the HIP FFT";
    return -1;
  }
  eng = new danse_tz();
  eng->dev = device;
  eng->R = R;
  TCHK(hipSetDevice(device));
  // S[i] / (N R), i = tau + N - 1: sum_n f[n] h[n + tau]
  std::vector<float> sn(kA);
  for (int i = 0; i < kA; ++i) {
    const int tau = i - (kN - 1);
    double s = 0.0;
    for (int n = std::max(0, -tau); n < std::min(kN, kN - tau); ++n) s += (double)f[n] * (double)h[n + tau];
    sn[i] = (float)(s / ((double)kN * (double)R));
  }
  std::vector<cf> wtw;
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
  TCHK(hipMalloc((void**)&eng->dTw, wtw.size() * sizeof(cf)));
  TCHK(hipMalloc((void**)&eng->dSn, kA * sizeof(float)));
  TCHK(hipMemcpy(eng->dTw, wtw.data(), wtw.size() * sizeof(cf), hipMemcpyHostToDevice));
  TCHK(hipMemcpy(eng->dSn, sn.data(), kA * sizeof(float), hipMemcpyHostToDevice));
  *out = eng;
  return 0;
}

void danse_tz_destroy(danse_tz* eng) {
  if (!eng) return;
  (void)hipSetDevice(eng->dev);
  if (eng->dTw) (void)hipFree(eng->dTw);
  if (eng->dSn) (void)hipFree(eng->dSn);
  delete eng;
}

int danse_tz_ir(danse_tz* eng, const float* wHat, int32_t B, int32_t M, float* wIR, void* stream) {
  if (!eng || !wHat || !wIR || B < 0 || M < 1) {
    g_terr = "bad arguments";
    if (eng) eng->err = g_terr;
    return -1;
  }
  if (B == 0) return 0;
  TCHK(hipSetDevice(eng->dev));
  const int BM = B * M;
  hipLaunchKernelGGL(tz_ir_kernel, dim3((BM + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const cf*>(wHat), BM, M, eng->dTw, eng->dSn, wIR);
  TCHK(hipGetLastError());
  return 0;
}

int danse_tz_compress(danse_tz* eng, const float* yq, const float* wIR, int32_t B, int32_t M, int32_t L, float* z,
                      void* stream) {
  if (!eng || !yq || !wIR || !z || B < 0 || M < 1 || L < 1 || L > kN) {
    g_terr = "bad arguments (1 <= L <= N)";
    if (eng) eng->err = g_terr;
    return -1;
  }
  if (B == 0) return 0;
  TCHK(hipSetDevice(eng->dev));
  hipLaunchKernelGGL(tz_compress_kernel, dim3(B), dim3(kThr), 0, (hipStream_t)stream, yq, wIR, M, L, z);
  TCHK(hipGetLastError());
  return 0;
}

}  // extern "C"
