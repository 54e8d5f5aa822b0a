// Enhancement metrics on the device, float64 like the
// reference:
//   danse_snr      = get_snr        (danse_toolbox/d_eval.py:573-624)
//   danse_fwsnrseg = get_fwsnrseg   (danse_toolbox/d_eval.py:660-778)
// The fwSNRseg kernel takes one frame of one signal pair per workgroup: the
// clean and the enhanced frame each go through a radix-2 FFT in LDS (two
// passes: packing both into one complex FFT loses the clean spectrum of
// silent frames -- eps-level samples -- in the enhanced one's rounding),
// then the 25 critical-band energies, the weighted log-SNR and the [0, 35]
// dB clip.  Metrics are not on the update path: the
// kernels are sized for the E battery (thousands of frames per launch).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "../../include/danse_mi355x.h"

namespace {

thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return 1;
}

#define MCHK(x)                                                          \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr int kThr = 256;
constexpr int kCrit = 25;

// critical bands of d_eval.py:690-716 and their weights (717-718)
__constant__ double kCent[kCrit] = {50.0000, 120.000, 190.000, 260.000, 330.000, 400.000, 470.000, 540.000, 617.372,
                                    703.378, 798.717, 904.128, 1020.38, 1148.30, 1288.72, 1442.54, 1610.70, 1794.16,
                                    1993.93, 2211.08, 2446.71, 2701.97, 2978.04, 3276.17, 3597.63};
__constant__ double kBw[kCrit] = {70.0000, 70.0000, 70.0000, 70.0000, 70.0000, 70.0000, 70.0000, 77.3724, 86.0056,
                                  95.3398, 105.411, 116.256, 127.914, 140.423, 153.823, 168.154, 183.457, 199.776,
                                  217.153, 235.631, 255.255, 276.072, 298.126, 321.465, 346.136};

struct FwParams {
  int W;          // winlength = round(frameLen fs)
  int skip;       // floor((1 - overlap) frameLen fs)
  int nfft;       // 2^ceil(log2(2 W))
  int logn;
  int nf;         // int(T / skip - W / skip)
  double maxFreq, gamma;
};

__device__ double block_sum(double v, double* red) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < kThr / 64; ++w) s += red[w];
  return s;
}

// grid (nf, nSig), block 256, dynamic LDS: nfft complex + nfft / 2 x 2 magnitudes
__global__ void __launch_bounds__(kThr) fwsnrseg_kernel(const double* __restrict__ clean,
                                                        const double* __restrict__ enh, long long T, FwParams p,
                                                        double* __restrict__ perFrame) {
  extern __shared__ double2 sm[];
  __shared__ double red[kThr / 64];
  __shared__ double band[2][kCrit];
  const int n = p.nfft, h = n / 2, t = threadIdx.x;
  double2* z = sm;                          // [n]
  double* cm = (double*)(sm + n);           // [h]
  double* em = cm + h;                      // [h]
  const long long sig = blockIdx.y;
  const long long st = (long long)blockIdx.x * p.skip;
  const double eps = 2.220446049250313e-16;
  for (int pass = 0; pass < 2; ++pass) {
    const double* x = (pass == 0 ? clean : enh) + sig * T + st;
    double* mag = pass == 0 ? cm : em;
    // windowed frame (+ eps, d_eval.py:672-673), zero-padded to nfft, bit-reversed
    for (int i = t; i < n; i += kThr) {
      double2 v = make_double2(0.0, 0.0);
      if (i < p.W) {
        const double w = 0.5 * (1.0 - cos(2.0 * M_PI * (double)(i + 1) / (double)(p.W + 1)));
        v.x = (x[i] + eps) * w;
      }
      const int r = (int)(__brev((unsigned)i) >> (32 - p.logn));
      z[r] = v;
  }
  __syncthreads();
  for (int len = 2; len <= n; len <<= 1) {
    const int hl = len >> 1;
    for (int b = t; b < h; b += kThr) {
      const int grp = b / hl, j = b - grp * hl;
      const int i0 = grp * len + j, i1 = i0 + hl;
      double sn, cs;
      sincospi(-2.0 * (double)j / (double)len, &sn, &cs);
      const double2 u = z[i0], v = z[i1];
      const double2 vw = make_double2(v.x * cs - v.y * sn, v.x * sn + v.y * cs);
      z[i0] = make_double2(u.x + vw.x, u.y + vw.y);
      z[i1] = make_double2(u.x - vw.x, u.y - vw.y);
    }
    __syncthreads();
  }
  // magnitudes of bins 0..n/2-1 (the reference drops the Nyquist bin, d_eval.py:752,757)
  for (int k = t; k < h; k += kThr) mag[k] = hypot(z[k].x, z[k].y);
  __syncthreads();
  }
  double sc = 0.0, se = 0.0;
  for (int k = t; k < h; k += kThr) {
    sc += cm[k];
    se += em[k];
  }
  sc = block_sum(sc, red);
  se = block_sum(se, red);
  // critical-band energies (d_eval.py:722-733,759-760): one wave per band
  const double minFactor = exp(-30.0 / (2.0 * 2.303));
  const int wv = t >> 6, ln = t & 63;
  for (int i = wv; i < kCrit; i += kThr / 64) {
    const double f0 = floor((kCent[i] / p.maxFreq) * (double)h);
    const double bw = (kBw[i] / p.maxFreq) * (double)h;
    const double nrm = log(kBw[0]) - log(kBw[i]);
    double ce = 0.0, pe = 0.0;
    for (int j = ln; j < h; j += 64) {
      const double q = ((double)j - f0) / bw;
      double c = exp(-11.0 * (q * q) + nrm);
      c = c * (double)(c > minFactor);
      ce += c * (cm[j] / sc);
      pe += c * (em[j] / se);
    }
    for (int o = 32; o >= 1; o >>= 1) {
      ce += __shfl_xor(ce, o);
      pe += __shfl_xor(pe, o);
    }
    if (ln == 0) {
      band[0][i] = ce;
      band[1][i] = pe;
    }
  }
  __syncthreads();
  if (t == 0) {
    double num = 0.0, den = 0.0;
    for (int i = 0; i < kCrit; ++i) {
      const double ce = band[0][i], pe = band[1][i];
      double err = (ce - pe) * (ce - pe);
      if (err < eps) err = eps;
      const double w = pow(ce, p.gamma);
      num += w * (10.0 * log10((ce * ce) / err));
      den += w;
    }
    double d = num / den;
    if (d < 0.0) d = 0.0;
    if (d > 35.0) d = 35.0;
    perFrame[sig * p.nf + blockIdx.x] = d;
  }
}

// mean over frames per signal (np.mean, d_eval.py:239,243)
__global__ void __launch_bounds__(kThr) frame_mean_kernel(const double* __restrict__ perFrame, int nf,
                                                          double* __restrict__ mean) {
  __shared__ double red[kThr / 64];
  double s = 0.0;
  for (int i = threadIdx.x; i < nf; i += kThr) s += perFrame[(long long)blockIdx.x * nf + i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) mean[blockIdx.x] = s / (double)nf;
}

// get_snr: one workgroup per channel, float64 sums of s^2 and n^2 over vad
__global__ void __launch_bounds__(kThr) snr_kernel(const double* __restrict__ s, const double* __restrict__ nz,
                                                   const uint8_t* __restrict__ vad, long long T,
                                                   double* __restrict__ out) {
  __shared__ double red[kThr / 64];
  const long long c = blockIdx.x;
  double ss = 0.0, sn = 0.0, cnt = 0.0;
  for (long long i = threadIdx.x; i < T; i += kThr) {
    if (vad && !vad[c * T + i]) continue;
    const double a = s[c * T + i], b = nz[c * T + i];
    ss += a * a;
    sn += b * b;
    cnt += 1.0;
  }
  ss = block_sum(ss, red);
  sn = block_sum(sn, red);
  cnt = block_sum(cnt, red);
  if (threadIdx.x == 0) out[c] = 10.0 * log10((ss / cnt) / (sn / cnt));
}

int fw_params(long long T, double fs, double frameLen, double overlap, double gamma, FwParams* p) {
  if (!(fs > 0.0) || !(frameLen > 0.0) || !(overlap >= 0.0 && overlap < 1.0)) return fail("bad fwSNRseg parameters");
  p->W = (int)nearbyint(frameLen * fs);                              // round(): ties to even
  p->skip = (int)floor((1.0 - overlap) * frameLen * fs);
  if (p->W < 1 || p->skip < 1) return fail("fwSNRseg window or hop below one sample");
  const double nfft = pow(2.0, ceil(log2(2.0 * (double)p->W)));
  p->nfft = (int)nfft;
  p->logn = (int)lround(log2(nfft));
  if (p->nfft > 4096) return fail("fwSNRseg FFT longer than 4096 points");
  const double nf = (double)T / (double)p->skip - ((double)p->W / (double)p->skip);
  p->nf = nf > 0.0 ? (int)nf : 0;
  p->maxFreq = fs / 2.0;
  p->gamma = gamma;
  if (p->nf < 1) return fail("signal shorter than one fwSNRseg frame");
  return 0;
}

}  // namespace

extern "C" {

const char* danse_metrics_last_error(void) { return g_err.c_str(); }

int danse_fwsnrseg_frames(int64_t T, double fs, double frameLen, double overlap, int32_t* nFrames) {
  FwParams p;
  if (fw_params(T, fs, frameLen, overlap, 0.2, &p)) return 1;
  *nFrames = p.nf;
  return 0;
}

int danse_fwsnrseg(const double* clean, const double* enhanced, int64_t T, int32_t nSig, double fs, double frameLen,
                   double overlap, double gamma, double* perFrame, double* mean, void* stream) {
  if (!clean || !enhanced || !perFrame || nSig < 1) return fail("null argument or no signal");
  FwParams p;
  if (fw_params(T, fs, frameLen, overlap, gamma, &p)) return 1;
  // every frame's last sample is inside the signal: (nf - 1) skip + W <= T
  if ((long long)(p.nf - 1) * p.skip + p.W > T) return fail("fwSNRseg frame table exceeds the signal");
  const size_t lds = (size_t)p.nfft * sizeof(double2) + (size_t)p.nfft * sizeof(double);
  if (nSig > 65535) return fail("fwSNRseg: more than 65535 signal pairs in one call");
  {
    int dev = 0, maxLds = 0;
    MCHK(hipGetDevice(&dev));
    MCHK(hipDeviceGetAttribute(&maxLds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
    if (lds > (size_t)maxLds) return fail("fwSNRseg: the FFT workspace exceeds the device's LDS per workgroup");
    if (lds > 65536) MCHK(hipFuncSetAttribute((const void*)fwsnrseg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(fwsnrseg_kernel, dim3(p.nf, nSig), dim3(kThr), lds, st, clean, enhanced, (long long)T, p,
                     perFrame);
  MCHK(hipGetLastError());
  if (mean) {
    hipLaunchKernelGGL(frame_mean_kernel, dim3(nSig), dim3(kThr), 0, st, perFrame, p.nf, mean);
    MCHK(hipGetLastError());
  }
  return 0;
}

int danse_snr(const double* s, const double* n, const uint8_t* vad, int64_t T, int32_t C, double* out, void* stream) {
  if (!s || !n || !out || C < 1 || T < 1) return fail("null argument or empty signal");
  hipLaunchKernelGGL(snr_kernel, dim3(C), dim3(kThr), 0, (hipStream_t)stream, s, n, vad, (long long)T, out);
  MCHK(hipGetLastError());
  return 0;
}

}  // extern "C"
