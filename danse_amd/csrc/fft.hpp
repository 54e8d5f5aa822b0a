// Workgroup-level 1024-point complex FFT in LDS (radix-4 Stockham, natural
// order in and out), used by the WOLA analysis / synthesis stages.
//
// 256 threads, one radix-4 butterfly per thread per pass, log4(1024) = 5
// passes, ping-pong between two 8 KB LDS buffers.  Twiddles come from a
// 1024-entry table exp(-2*pi*i*m/N) computed in double on the host.
#pragma once
#include "common.hpp"

namespace danse {

constexpr int kFftThreads = 256;

// Forward DFT X[k] = sum_n x[n] exp(-2 pi i k n / N) of buf0 (N = 1024).
// Returns the LDS buffer holding the result (buf1 after 5 passes).
// Caller must __syncthreads() after filling buf0.
DANSE_DEV cf* fft1024(cf* buf0, cf* buf1, const cf* __restrict__ tw) {
  constexpr int N = 1024;
  const int j = threadIdx.x;
  cf* src = buf0;
  cf* dst = buf1;
#pragma unroll
  for (int p = 0; p < 5; ++p) {
    const int Ns = 1 << (2 * p);
    cf v0 = src[j], v1 = src[j + 256], v2 = src[j + 512], v3 = src[j + 768];
    const int k = j & (Ns - 1);
    if (p > 0) {
      const int m = k * (N / (Ns * 4));
      v1 = v1 * tw[m];
      v2 = v2 * tw[2 * m];
      v3 = v3 * tw[3 * m];
    }
    const cf a0 = v0 + v2, a1 = v0 - v2, a2 = v1 + v3, d13 = v1 - v3;
    const cf a3 = cf{d13.im, -d13.re};  // -i * (v1 - v3)
    const int idx = (j / Ns) * Ns * 4 + k;
    dst[idx] = a0 + a2;
    dst[idx + Ns] = a1 + a3;
    dst[idx + 2 * Ns] = a0 - a2;
    dst[idx + 3 * Ns] = a1 - a3;
    __syncthreads();
    cf* t = src;
    src = dst;
    dst = t;
  }
  return src;
}

}  // namespace danse
