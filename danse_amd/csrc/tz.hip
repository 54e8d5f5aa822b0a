// T(z) few-samples compression on the device:
//   danse_tz_ir       = dist_fct_approx        (d_base.py:1941-1991)
//   danse_tz_compress = danse_compression_few_samples' convolution
//                       (d_base.py:1871-1938, 1538-1566)
// The wave IR and the LDS sliding-window convolution live in tzconv.hpp
// (shared with the online engine's fewSamples broadcasts).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/danse_mi355x.h"
#include "tzconv.hpp"

using namespace danse;

namespace {

using tzc::kA;
using tzc::kN;
using tzc::kThr;

// ---- dist_fct_approx --------------------------------------------------------
// grid: (ceil(B*M / 4)), block 256: wave w handles item (b, m) = blockIdx*4 + w
__global__ __launch_bounds__(256) void tz_ir_kernel(const cf* __restrict__ wHat, int BM, int M,
                                                    const cf* __restrict__ tw, const float* __restrict__ sn,
                                                    float* __restrict__ wIR) {
  __shared__ cf lds[4][wfft::kLdsElems];
  const int wv = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + wv;
  if (item >= BM) return;   // whole wave exits together
  const int b = item / M, m = item - b * M;
  const cf* w = wHat + (size_t)b * (kN / 2 + 1) * M + m;
  float* o = wIR + (size_t)b * kA * M + m;
  tzc::ir_wave(lds[wv], tw, sn, [&](int k) { return w[(size_t)k * M]; },
               [&](int t, float v) { o[(size_t)t * M] = v; });
}

// ---- few-samples convolution ---------------------------------------------
__global__ __launch_bounds__(kThr) void tz_compress_kernel(const float* __restrict__ yq, const float* __restrict__ wIR,
                                                           int M, int L, float* __restrict__ z) {
  __shared__ tzc::ConvLds sm;
  const int b = blockIdx.x;
  const float* y = yq + (size_t)b * kN * M;
  const float* a = wIR + (size_t)b * kA * M;
  float* zb = z + (size_t)b * L;
  tzc::conv_block(sm, M, L, [&](int q, int m) { return y[(size_t)q * M + m]; }, [](int, int) { return true; },
                  [&](int i, int m) { return a[(size_t)i * M + m]; }, [&](int e, float v) { zb[e] = v; });
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
