// Resident engine translation unit (resident.hpp): the persistent round-loop
// kernel on 4 x 4 lane grids with 3 x 3 blocks per lane (D <= 12),
// the WOLA analyses of every round before it and the estimate synthesis
// after it.
#define DANSE_BCAST_HELPERS_ONLY
#include "resident.hpp"
#include "resident_api.hpp"

namespace danse {
namespace res {

// WOLA analysis of every round's broadcast frame (kind 0) and update frame
// (kind 1) of every channel: bcast_kernel phase 1's analysis (window, one
// wave FFT, 1 / sqrt(Ns)) for all rounds at once, one wave per
// (kind, round, scene, channel).
__global__ void __launch_bounds__(256) resident_analysis_kernel(const BcastArgs a, const int* chanNode, cf* YB, cf* YU) {
  __shared__ cf fftLds[4][wfft::kLdsElems];
  const int wv = threadIdx.x >> 6;
  const long long job = (long long)blockIdx.x * 4 + wv;
  const long long per = (long long)a.R * a.S * a.MT;
  if (job >= 2 * per) return;
  const int kind = (int)(job / per);
  const long long t = job % per;
  const int ch = (int)(t % a.MT);
  const int s = (int)((t / a.MT) % a.S);
  const int r = (int)(t / ((long long)a.MT * a.S));
  const int k = chanNode[ch];
  const int end = kind == 0 ? a.bcEnd[r * a.K + k] : a.upEnd[r * a.K + k];
  const float invSqNs = 1.0f / sqrtf((float)a.Ns);
  cf v[16];
  load_frame_wave(v, a.y + ((long long)s * a.MT + ch) * a.T, end, a.T, a.hA);
  wfft::fft1024(v, fftLds[wv], a.tw);
  cf* dst = (kind == 0 ? YB : YU) + (((long long)r * a.S + s) * a.MT + ch) * a.F;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int f = wfft::out_index(c);
    if (f < a.F) dst[f] = invSqNs * v[c];
  }
}

// Estimate synthesis, step 1: the real part of the inverse transform of
// every round's dhat (bcast_kernel's synthesis without the accumulation),
// one wave per (family, scene, node, round), into frames [..][R][N].
__global__ void __launch_bounds__(256) resident_synth_frames_kernel(const BcastArgs a, const int* fams, int nFam,
                                                                     float* frames) {
  __shared__ cf fftLds[4][wfft::kLdsElems];
  const int wv = threadIdx.x >> 6;
  const long long job = (long long)blockIdx.x * 4 + wv;
  const long long total = (long long)nFam * a.S * a.K * a.R;
  if (job >= total) return;
  const int rp = (int)(job % a.R);
  const long long t = job / a.R;
  const int k = (int)(t % a.K);
  const int s = (int)((t / a.K) % a.S);
  const int fam = fams[t / ((long long)a.K * a.S)];
  const cf* dh = a.dhat + ((((long long)fam * a.S + s) * a.K + k) * a.R + rp) * a.F;
  const int l = __lane_id();
  cf v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = herm_ext_conj(dh, l + 64 * j, a.F);
  wfft::fft1024(v, fftLds[wv], a.tw);
  float* fr = frames + job * a.N;
#pragma unroll
  for (int c = 0; c < 16; ++c) fr[wfft::out_index(c)] = v[c].re;
}

// Step 2: overlap-add in round order (the launch-per-round engine adds
// round rp's frame at round rp + 1, so every sample receives its frames in
// increasing rp): d[idx] += sc h_S[n] v_rp[n] over the rounds whose frame
// [upEnd - N, upEnd) covers idx (upEnd is non-decreasing in rp; the host
// checks it), one thread per (family, scene, node, sample).
__global__ void __launch_bounds__(256) resident_synth_ola_kernel(const BcastArgs a, const int* fams, int nFam,
                                                                  const float* frames) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)nFam * a.S * a.K * a.T;
  if (i >= total) return;
  const int idx = (int)(i % a.T);
  const long long t = i / a.T;
  const int k = (int)(t % a.K);
  const int s = (int)((t / a.K) % a.S);
  const int fam = fams[t / ((long long)a.K * a.S)];
  const int N = a.N, R = a.R;
  const float sc = sqrtf((float)a.Ns) / (float)N;
  // first round whose frame ends after idx
  int lo = 0, hi = R;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a.upEnd[mid * a.K + k] > idx) hi = mid;
    else lo = mid + 1;
  }
  float* dd = a.d + (((long long)fam * a.S + s) * a.K + k) * a.T;
  float acc = dd[idx];
  const float* fr = frames + t * (long long)R * N;
  for (int rp = lo; rp < R; ++rp) {
    const int n = idx - (a.upEnd[rp * a.K + k] - N);
    if (n < 0) break;
    acc += sc * a.hS[n] * fr[(long long)rp * N + n];
  }
  dd[idx] = acc;
}

template <int NB, int RMAX>
static int launch_nb(const ResArgs& ra, int grid, hipStream_t st, bool check, int* fits) {
  if (check) {
    int dev = 0, per = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)resident_kernel<NB, RMAX>, 64, 0) != hipSuccess)
      return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    *fits = per * cus;
    if (grid > *fits) return 1;
    return 0;
  }
  hipLaunchKernelGGL((resident_kernel<NB, RMAX>), dim3(grid), dim3(64), 0, st, ra);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace res

int resident_launch(int NB, int rank1, const res::ResArgs& ra, int grid, hipStream_t st, bool check, int* fits) {
  using namespace res;
  // NB = 3 only (D <= 12): the resident Rnn / Ryy blocks of NB = 4 / 5 (36 /
  // 150 VGPRs with the solver's ~160) no longer fit 256 VGPRs at two waves
  // per SIMD without spilling
  if (NB != 3) return -1;
  return rank1 ? launch_nb<3, 1>(ra, grid, st, check, fits) : launch_nb<3, kRMax>(ra, grid, st, check, fits);
}

void resident_analysis(const BcastArgs& a, const int* chanNode, cf* YB, cf* YU, hipStream_t st) {
  const long long jobs = 2LL * a.R * a.S * a.MT;
  hipLaunchKernelGGL(res::resident_analysis_kernel, dim3((unsigned)((jobs + 3) / 4)), dim3(256), 0, st, a, chanNode,
                     YB, YU);
}

void resident_synth(const BcastArgs& a, const int* fams, int nFam, float* frames, hipStream_t st) {
  const long long jobs = (long long)nFam * a.S * a.K * a.R;
  hipLaunchKernelGGL(res::resident_synth_frames_kernel, dim3((unsigned)((jobs + 3) / 4)), dim3(256), 0, st, a, fams,
                     nFam, frames);
  const long long n = (long long)nFam * a.S * a.K * a.T;
  hipLaunchKernelGGL(res::resident_synth_ola_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, fams,
                     nFam, frames);
}

}  // namespace danse
