// (e)STOI on the device, float64 like the reference:
//   danse_stoi = stoi / stoi_any_fs (danse_toolbox/mypystoi/stoi.py:18-239,
//                utils.py), extended = eSTOI (what get_metrics reports,
//                d_eval.py:254-331)
// for nSig (clean, processed) pairs per call, so the E battery's
// before / after / centralised / local scores of every scene stay on the GPU.
// Pipeline (one launch per stage, every stage batched over the pairs):
//   1. resample to 10 kHz (fs != 10000): resample_poly(x, 10000, fs) with the
//      Octave Kaiser window of utils.resample_oct (utils.py:8-47) -- stoi()'s
//      resampler; stoi_any_fs uses resampy, absent offline (unpinned there);
//   2. silent-frame removal (utils.py:102-126): 256-sample Hann frames every
//      128, energies in dB, frames within 40 dB of the loudest kept, the kept
//      frames overlap-added back to back -- one workgroup per pair (energy
//      pass, max, ordered compaction, overlap-add);
//   3. STFT (utils.py:87-99): 512-point radix-2 FFT in LDS of each 256-sample
//      Hann frame, the 15 one-third-octave band magnitudes (thirdoct,
//      utils.py:57-84) -- one workgroup per (frame, pair);
//   4. 30-frame segments: eSTOI row / column mean-variance normalisation
//      (row_col_normalize without its EPS-scale random perturbation) or the
//      classic normalise-clip-correlate -- one wave per (segment, pair);
//   5. the mean over segments, in order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/danse_mi355x.h"

namespace {

thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return 1;
}

#define SCHK(x)                                                                         \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr int kFs = 10000;
constexpr int kW = 256;        // N_FRAME
constexpr int kHop = 128;
constexpr int kNfft = 512;
constexpr int kBands = 15;
constexpr int kSeg = 30;       // N
constexpr double kDyn = 40.0;  // DYN_RANGE
constexpr double kEps = 2.220446049250313e-16;
constexpr int kThr = 256;

struct Bands {
  int lo[kBands], hi[kBands];   // bins [lo, hi) of each 1/3-octave band
};

// np.hanning(256 + 2)[1:-1]
__device__ __forceinline__ double hann(int n) {
  return 0.5 - 0.5 * cos(2.0 * M_PI * (double)(n + 1) / (double)(kW + 1));
}

__device__ double block_sum(double v, double* red) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < kThr / 64; ++w) s += red[w];
  __syncthreads();
  return s;
}

__device__ double block_max(double v, double* red) {
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = red[0];
  for (int w = 1; w < kThr / 64; ++w) s = fmax(s, red[w]);
  __syncthreads();
  return s;
}

// upfirdn(h, x, up, down)[pre + i] (scipy resample_poly, padtype constant):
// out[i] = sum_j h[j] xu[(i + pre) down - j], xu = x zero-stuffed by up
__global__ void __launch_bounds__(kThr) resample_kernel(const double* __restrict__ x, long long T, int nSig,
                                                        const double* __restrict__ h, int nh, int up, int down,
                                                        long long pre, long long nOut, double* __restrict__ out) {
  const long long n = (long long)nSig * nOut;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long i = e % nOut, s = e / nOut;
    const long long m = (i + pre) * down;   // position in the upsampled signal
    // taps j with (m - j) % up == 0, 0 <= j < nh, 0 <= (m - j) / up < T
    long long j = m % up;
    long long xi = (m - j) / up;
    if (xi >= T) {
      const long long skip = xi - (T - 1);
      j += skip * up;
      xi -= skip;
    }
    const double* xs = x + s * T;
    double acc = 0.0;
    for (; j < nh && xi >= 0; j += up, --xi) acc += h[j] * xs[xi];
    out[s * nOut + i] = acc;
  }
}

// Silent-frame removal of one pair per workgroup; frames i in range(0, T -
// 256, 128).  kept[s][q] = original frame of kept slot q; nKept[s].
__global__ void __launch_bounds__(kThr) silent_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                      long long T, int nFr, double* __restrict__ energy,
                                                      int* __restrict__ kept, int* __restrict__ nKept,
                                                      double* __restrict__ xs, double* __restrict__ ys) {
  __shared__ double red[kThr / 64];
  __shared__ int scan[kThr];
  const int s = blockIdx.x, t = threadIdx.x;
  const double* xx = x + (long long)s * T;
  const double* yy = y + (long long)s * T;
  double* en = energy + (long long)s * nFr;
  int* km = kept + (long long)s * nFr;
  // energies 20 log10(||w x_frame|| + EPS), one frame per wave
  const int wv = t >> 6, ln = t & 63;
  for (int f = wv; f < nFr; f += kThr / 64) {
    double a = 0.0;
    for (int n = ln; n < kW; n += 64) {
      const double v = hann(n) * xx[(long long)f * kHop + n];
      a += v * v;
    }
    for (int o = 32; o >= 1; o >>= 1) a += __shfl_xor(a, o);
    if (ln == 0) en[f] = 20.0 * log10(sqrt(a) + kEps);
  }
  __syncthreads();
  double mx = -INFINITY;
  for (int f = t; f < nFr; f += kThr) mx = fmax(mx, en[f]);
  mx = block_max(mx, red);
  // ordered compaction of the kept frames (mask: max - dyn - e < 0)
  int base = 0;
  for (int c0 = 0; c0 < nFr; c0 += kThr) {
    const int f = c0 + t;
    const int keep = (f < nFr && (mx - kDyn - en[f]) < 0.0) ? 1 : 0;
    scan[t] = keep;
    __syncthreads();
    for (int o = 1; o < kThr; o <<= 1) {
      const int v = (t >= o) ? scan[t - o] : 0;
      __syncthreads();
      scan[t] += v;
      __syncthreads();
    }
    if (keep) km[base + scan[t] - 1] = f;
    base += scan[kThr - 1];
    __syncthreads();
  }
  if (t == 0) nKept[s] = base;
  __syncthreads();
  // overlap-add of the kept frames: sample j of the output gets slot j / 128
  // (offset < 128) and slot j / 128 - 1 (offset >= 128)
  const long long nSil = (long long)(base - 1) * kHop + kW;
  double* xo = xs + (long long)s * T;
  double* yo = ys + (long long)s * T;
  for (long long j = t; j < nSil; j += kThr) {
    const int q1 = (int)(j / kHop);
    double ax = 0.0, ay = 0.0;
    for (int q = q1 - 1; q <= q1; ++q) {
      if (q < 0 || q >= base) continue;
      const int o = (int)(j - (long long)q * kHop);
      if (o >= kW) continue;
      const long long src = (long long)km[q] * kHop + o;
      const double w = hann(o);
      ax += w * xx[src];
      ay += w * yy[src];
    }
    xo[j] = ax;
    yo[j] = ay;
  }
}

// One STFT frame of one pair: the 15 band magnitudes sqrt(sum |X_k|^2) of
// the clean (tob[s][0]) and processed (tob[s][1]) signal.  grid (frames, nSig)
__global__ void __launch_bounds__(kThr) band_kernel(const double* __restrict__ xs, const double* __restrict__ ys,
                                                    long long T, const int* __restrict__ nKept, int maxFr2, Bands b,
                                                    double* __restrict__ tob) {
  __shared__ double2 z[kNfft];
  __shared__ double pw[kNfft / 2 + 1];
  const int s = blockIdx.y, f = blockIdx.x, t = threadIdx.x;
  const long long nSil = (long long)(nKept[s] - 1) * kHop + kW;
  // frames in range(0, nSil - 256, 128)
  const long long nFr2 = nSil - kW > 0 ? (nSil - kW + kHop - 1) / kHop : 0;
  if (f >= nFr2) return;   // whole workgroup
  for (int pass = 0; pass < 2; ++pass) {
    const double* src = (pass ? ys : xs) + (long long)s * T + (long long)f * kHop;
    for (int i = t; i < kNfft; i += kThr) {
      const double v = (i < kW) ? hann(i) * src[i] : 0.0;
      const int r = (int)(__brev((unsigned)i) >> (32 - 9));
      z[r] = make_double2(v, 0.0);
    }
    __syncthreads();
    for (int len = 2; len <= kNfft; len <<= 1) {
      const int hl = len >> 1;
      for (int bb = t; bb < kNfft / 2; bb += kThr) {
        const int grp = bb / hl, j = bb - grp * hl;
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
    for (int k = t; k <= kNfft / 2; k += kThr) pw[k] = z[k].x * z[k].x + z[k].y * z[k].y;
    __syncthreads();
    if (t < kBands) {
      double a = 0.0;
      for (int k = b.lo[t]; k < b.hi[t]; ++k) a += pw[k];
      tob[(((long long)s * 2 + pass) * kBands + t) * maxFr2 + f] = sqrt(a);
    }
    __syncthreads();
  }
}

// One 30-frame segment of one pair per wave: its contribution to the sum
// over segments.  eSTOI: sum(x_n y_n) / 30 after row then column
// mean / norm normalisation (row_col_normalize, utils.py:134-149); classic:
// the correlation summed over bands of the normalised, clipped vectors
// (stoi.py:208-239).  grid (segments, nSig), block 64
__global__ void __launch_bounds__(64) seg_kernel(const double* __restrict__ tob, const int* __restrict__ nKept,
                                                 int maxFr2, int extended, double* __restrict__ seg, int maxSeg) {
  __shared__ double X[kBands][kSeg], Y[kBands][kSeg];
  const int s = blockIdx.y, m = blockIdx.x, l = threadIdx.x;
  const long long nSil = (long long)(nKept[s] - 1) * kHop + kW;
  const long long nFr2 = nSil - kW > 0 ? (nSil - kW + kHop - 1) / kHop : 0;
  if (m + kSeg > nFr2) return;
  const double* xt = tob + ((long long)s * 2 + 0) * kBands * maxFr2;
  const double* yt = tob + ((long long)s * 2 + 1) * kBands * maxFr2;
  for (int e = l; e < kBands * kSeg; e += 64) {
    const int bnd = e / kSeg, c = e % kSeg;
    X[bnd][c] = xt[(long long)bnd * maxFr2 + m + c];
    Y[bnd][c] = yt[(long long)bnd * maxFr2 + m + c];
  }
  __syncthreads();
  double part = 0.0;
  if (extended) {
    // rows (bands): zero mean, unit norm over the 30 frames
    if (l < 2 * kBands) {
      double (*A)[kSeg] = (l < kBands) ? X : Y;
      const int bnd = l % kBands;
      double mu = 0.0;
      for (int c = 0; c < kSeg; ++c) mu += A[bnd][c];
      mu /= (double)kSeg;
      double nn = 0.0;
      for (int c = 0; c < kSeg; ++c) {
        const double v = A[bnd][c] - mu;
        A[bnd][c] = v;
        nn += v * v;
      }
      const double inv = 1.0 / sqrt(nn);
      for (int c = 0; c < kSeg; ++c) A[bnd][c] *= inv;
    }
    __syncthreads();
    // columns (frames): zero mean, unit norm over the 15 bands
    if (l < 2 * kSeg) {
      double (*A)[kSeg] = (l < kSeg) ? X : Y;
      const int c = l % kSeg;
      double mu = 0.0;
      for (int bnd = 0; bnd < kBands; ++bnd) mu += A[bnd][c];
      mu /= (double)kBands;
      double nn = 0.0;
      for (int bnd = 0; bnd < kBands; ++bnd) {
        const double v = A[bnd][c] - mu;
        A[bnd][c] = v;
        nn += v * v;
      }
      const double inv = 1.0 / sqrt(nn);
      for (int bnd = 0; bnd < kBands; ++bnd) A[bnd][c] *= inv;
    }
    __syncthreads();
    if (l < kSeg)
      for (int bnd = 0; bnd < kBands; ++bnd) part += X[bnd][l] * Y[bnd][l] / (double)kSeg;
  } else if (l < kBands) {
    const double clip = 1.0 + pow(10.0, 15.0 / 20.0);   // 1 + 10^(-BETA / 20)
    double nx = 0.0, ny = 0.0;
    for (int c = 0; c < kSeg; ++c) {
      nx += X[l][c] * X[l][c];
      ny += Y[l][c] * Y[l][c];
    }
    const double alpha = sqrt(nx) / (sqrt(ny) + kEps);
    double yp[kSeg];
    double my = 0.0, mx = 0.0;
    for (int c = 0; c < kSeg; ++c) {
      yp[c] = fmin(Y[l][c] * alpha, X[l][c] * clip);
      my += yp[c];
      mx += X[l][c];
    }
    my /= (double)kSeg;
    mx /= (double)kSeg;
    double n2y = 0.0, n2x = 0.0;
    for (int c = 0; c < kSeg; ++c) {
      yp[c] -= my;
      n2y += yp[c] * yp[c];
      const double v = X[l][c] - mx;
      n2x += v * v;
    }
    const double iy = 1.0 / (sqrt(n2y) + kEps), ix = 1.0 / (sqrt(n2x) + kEps);
    for (int c = 0; c < kSeg; ++c) part += (yp[c] * iy) * ((X[l][c] - mx) * ix);
  }
  for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o);
  if (l == 0) seg[(long long)s * maxSeg + m] = part;
}

// mean over the segments (in order); fewer than 30 STFT frames -> 1e-5
// (stoi.py:69-75)
__global__ void __launch_bounds__(kThr) final_kernel(const double* __restrict__ seg, const int* __restrict__ nKept,
                                                     int maxSeg, int extended, double* __restrict__ out) {
  __shared__ double red[kThr / 64];
  const int s = blockIdx.x;
  const long long nSil = (long long)(nKept[s] - 1) * kHop + kW;
  const long long nFr2 = nSil - kW > 0 ? (nSil - kW + kHop - 1) / kHop : 0;
  const long long J = nFr2 - kSeg + 1;
  if (nFr2 < kSeg) {
    if (threadIdx.x == 0) out[s] = 1e-5;
    return;
  }
  double a = 0.0;
  for (long long j = threadIdx.x; j < J; j += kThr) a += seg[(long long)s * maxSeg + j];
  a = block_sum(a, red);
  if (threadIdx.x == 0) out[s] = extended ? a / (double)J : a / ((double)J * kBands);
}

// utils.thirdoct(10000, 512, 15, 150)
Bands third_octave() {
  Bands b{};
  const int nb = kNfft / 2 + 1;
  for (int i = 0; i < kBands; ++i) {
    const double lo = 150.0 * std::pow(2.0, (2.0 * i - 1.0) / 6.0), hi = 150.0 * std::pow(2.0, (2.0 * i + 1.0) / 6.0);
    int bl = 0, bh = 0;
    double dl = 1e300, dh = 1e300;
    for (int k = 0; k < nb; ++k) {
      const double f = (double)kFs * (double)k / (double)kNfft;   // np.linspace(0, fs, nfft + 1)[k]
      const double el = (f - lo) * (f - lo), eh = (f - hi) * (f - hi);
      if (el < dl) { dl = el; bl = k; }
      if (eh < dh) { dh = eh; bh = k; }
    }
    b.lo[i] = bl;
    b.hi[i] = bh;
  }
  return b;
}

// utils._resample_window_oct(p, q) / sum, then resample_poly's filter
// preparation (h *= up, centring pads) -> the padded filter and the first
// kept output sample
struct Resampler {
  int up, down;
  std::vector<double> h;
  long long pre, nOut;
};

double bessel_i0(double x) {
  double s = 1.0, t = 1.0;
  for (int k = 1; k < 200; ++k) {
    t *= (x / (2.0 * k)) * (x / (2.0 * k));
    s += t;
    if (t < 1e-17 * s) break;
  }
  return s;
}

Resampler make_resampler(int p, int q, long long nIn) {
  const int g = std::gcd(p, q);
  p /= g;
  q /= g;
  const double rej = 60.0;   // -20 log10_rejection, log10_rejection = -3
  const double stop = 1.0 / (2.0 * std::max(p, q));
  const double roll = stop / 10.0;
  const long long L = (long long)std::ceil((rej - 8.0) / (28.714 * roll));
  const double beta = 0.1102 * (rej - 8.7);
  const long long n = 2 * L + 1;
  std::vector<double> h(n);
  double sum = 0.0;
  for (long long i = 0; i < n; ++i) {
    const double t = (double)(i - L);
    const double a = 2.0 * stop * t;
    const double sinc = (a == 0.0) ? 1.0 : std::sin(M_PI * a) / (M_PI * a);
    // np.kaiser(n, beta)[i] = I0(beta sqrt(1 - ((i - (n-1)/2) / ((n-1)/2))^2)) / I0(beta)
    const double r = (double)(i - L) / (double)L;
    const double w = bessel_i0(beta * std::sqrt(std::max(0.0, 1.0 - r * r))) / bessel_i0(beta);
    h[i] = w * (2.0 * p * stop * sinc);
    sum += h[i];
  }
  for (auto& v : h) v = v / sum * (double)p;   // window / sum(window), then h *= up
  Resampler rs;
  rs.up = p;
  rs.down = q;
  const long long halfLen = (n - 1) / 2;
  const long long preP = q - halfLen % q;
  long long postP = 0;
  const long long preRemove = (halfLen + preP) / q;
  long long nOut = nIn * p;
  nOut = nOut / q + ((nOut % q) ? 1 : 0);
  auto outLen = [&](long long lh) { return ((nIn - 1) * p + lh - 1) / q + 1; };
  while (outLen(n + preP + postP) < nOut + preRemove) ++postP;
  rs.h.assign(preP, 0.0);
  rs.h.insert(rs.h.end(), h.begin(), h.end());
  rs.h.insert(rs.h.end(), postP, 0.0);
  rs.pre = preRemove;
  rs.nOut = nOut;
  return rs;
}

}  // namespace

extern "C" {

const char* danse_stoi_last_error(void) { return g_err.c_str(); }

int danse_stoi(const double* x, const double* y, int64_t T, int32_t nSig, double fs, int32_t extended, double* out,
               void* stream) {
  if (!x || !y || !out || nSig < 1 || T < 1) return fail("null argument or empty signal");
  if (!(fs > 0.0) || fs != std::floor(fs)) return fail("fs must be a positive integer rate");
  if (nSig > 65535) return fail("more than 65535 signal pairs in one call");
  hipStream_t st = (hipStream_t)stream;
  const double *xr = x, *yr = y;
  long long Tr = T;
  double *bufX = nullptr, *bufY = nullptr, *dh = nullptr;
  std::vector<void*> owned;
  auto cleanup = [&]() {
    for (void* p : owned) (void)hipFree(p);
  };
  auto alloc = [&](void** p, size_t bytes) -> bool {
    if (hipMalloc(p, std::max<size_t>(bytes, 8)) != hipSuccess) return false;
    owned.push_back(*p);
    return true;
  };
  if ((int)fs != kFs) {
    const Resampler rs = make_resampler(kFs, (int)fs, T);
    Tr = rs.nOut;
    if (!alloc((void**)&bufX, (size_t)nSig * Tr * sizeof(double)) || !alloc((void**)&bufY, (size_t)nSig * Tr * sizeof(double)) ||
        !alloc((void**)&dh, rs.h.size() * sizeof(double))) {
      cleanup();
      return fail("stoi: device allocation failed");
    }
    if (hipMemcpyAsync(dh, rs.h.data(), rs.h.size() * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess) {
      cleanup();
      return fail("stoi: filter upload failed");
    }
    const long long n = (long long)nSig * Tr;
    const unsigned g = (unsigned)std::min<long long>((n + kThr - 1) / kThr, 65535);
    hipLaunchKernelGGL(resample_kernel, dim3(g), dim3(kThr), 0, st, x, (long long)T, nSig, dh, (int)rs.h.size(), rs.up,
                       rs.down, rs.pre, Tr, bufX);
    hipLaunchKernelGGL(resample_kernel, dim3(g), dim3(kThr), 0, st, y, (long long)T, nSig, dh, (int)rs.h.size(), rs.up,
                       rs.down, rs.pre, Tr, bufY);
    xr = bufX;
    yr = bufY;
  }
  // frames of the silent-frame pass: range(0, Tr - 256, 128)
  const int nFr = Tr > kW ? (int)((Tr - kW + kHop - 1) / kHop) : 0;
  if (nFr < 1) {
    cleanup();
    return fail("stoi: signal shorter than one 256-sample frame at 10 kHz");
  }
  const int maxFr2 = std::max(nFr - 1, 1);          // STFT frames of the longest possible output
  const int maxSeg = std::max(maxFr2 - kSeg + 1, 1);
  double *energy = nullptr, *xs = nullptr, *ys = nullptr, *tob = nullptr, *seg = nullptr;
  int *kept = nullptr, *nKept = nullptr;
  if (!alloc((void**)&energy, (size_t)nSig * nFr * sizeof(double)) || !alloc((void**)&kept, (size_t)nSig * nFr * sizeof(int)) ||
      !alloc((void**)&nKept, (size_t)nSig * sizeof(int)) || !alloc((void**)&xs, (size_t)nSig * Tr * sizeof(double)) ||
      !alloc((void**)&ys, (size_t)nSig * Tr * sizeof(double)) ||
      !alloc((void**)&tob, (size_t)nSig * 2 * kBands * maxFr2 * sizeof(double)) ||
      !alloc((void**)&seg, (size_t)nSig * maxSeg * sizeof(double))) {
    cleanup();
    return fail("stoi: device allocation failed");
  }
  hipLaunchKernelGGL(silent_kernel, dim3(nSig), dim3(kThr), 0, st, xr, yr, Tr, nFr, energy, kept, nKept, xs, ys);
  hipLaunchKernelGGL(band_kernel, dim3(maxFr2, nSig), dim3(kThr), 0, st, xs, ys, Tr, nKept, maxFr2, third_octave(), tob);
  hipLaunchKernelGGL(seg_kernel, dim3(maxSeg, nSig), dim3(64), 0, st, tob, nKept, maxFr2, (int)(extended != 0), seg,
                     maxSeg);
  hipLaunchKernelGGL(final_kernel, dim3(nSig), dim3(kThr), 0, st, seg, nKept, maxSeg, (int)(extended != 0), out);
  const hipError_t le = hipGetLastError();
  // the scratch buffers are freed once the launches have drained
  const hipError_t se = hipStreamSynchronize(st);
  cleanup();
  if (le != hipSuccess) return fail(std::string("stoi launch: ") + hipGetErrorString(le));
  if (se != hipSuccess) return fail(std::string("stoi: ") + hipGetErrorString(se));
  return 0;
}

}  // extern "C"
