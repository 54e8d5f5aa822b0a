// Check + timing of the 4 x 4 lane-grid GEVD solver (solver2d.hpp, G = 4,
// four bins per wave) against the row-per-lane wavefront solver
// (solver64m.hpp) and the 8 x 8 grid (G = 8) on the random Hermitian pairs
// of t2d_check.hip.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I danse_amd/csrc
//        -DPH_NB4=5 -DPH_NB8=3 scripts/micro/t2g_check.hip -o scripts/micro/bin/t2g_check5
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "kernels_2d.hpp"
#include "kernels_big.hpp"

using namespace danse;

#ifndef PH_NB4
#define PH_NB4 5
#endif
#ifndef PH_NB8
#define PH_NB8 3
#endif
constexpr int NB4 = PH_NB4, NB8 = PH_NB8;
constexpr int DMB = (4 * NB4 + 7) / 8 * 8 > 8 * NB8 ? (4 * NB4 + 7) / 8 * 8 : 8 * NB8;

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    printf("HIP error %s: %s\n", what, hipGetErrorString(e));
    exit(1);
  }
}

int main(int argc, char** argv) {
  const int D = argc > 1 ? atoi(argv[1]) : 4 * NB4 - 1;
  const int B = argc > 2 ? atoi(argv[2]) : 16416;
  const int R = argc > 3 ? atoi(argv[3]) : 1;
  const int ref = argc > 4 ? atoi(argv[4]) : 0;
  if (D > 4 * NB4 || D > 8 * NB8 || D > DMB || (R != 1 && R > kRMax) || ref >= D) {
    printf("bad arguments\n");
    return 2;
  }
  std::mt19937 rng(7);
  std::normal_distribution<double> nd;
  std::uniform_real_distribution<double> ud(0.0, 1.0);
  const int NU = 256;
  std::vector<cd> hY((size_t)B * D * D), hN((size_t)B * D * D);
  for (int u = 0; u < NU; ++u) {
    std::vector<cd> X((size_t)D * 2 * D), h(D), Z((size_t)D * 2 * D);
    for (auto& v : X) v = cd{nd(rng), nd(rng)};
    for (auto& v : Z) v = cd{nd(rng), nd(rng)};
    for (auto& v : h) v = cd{nd(rng), nd(rng)};
    const double sig = std::pow(10.0, 2.0 * ud(rng) - 1.0);
    const bool full = (u % 4) == 3;
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        cd n{0, 0}, z{0, 0};
        for (int t = 0; t < 2 * D; ++t) {
          const cd xi = X[i * 2 * D + t], xj = X[j * 2 * D + t];
          n.re += xi.re * xj.re + xi.im * xj.im;
          n.im += xi.im * xj.re - xi.re * xj.im;
          const cd zi = Z[i * 2 * D + t], zj = Z[j * 2 * D + t];
          z.re += zi.re * zj.re + zi.im * zj.im;
          z.im += zi.im * zj.re - zi.re * zj.im;
        }
        n = cd{n.re / (2 * D), n.im / (2 * D)};
        cd yv;
        if (full) {
          yv = cd{n.re + z.re / (2 * D), n.im + z.im / (2 * D)};
        } else {
          const cd hh{h[i].re * h[j].re + h[i].im * h[j].im, h[i].im * h[j].re - h[i].re * h[j].im};
          yv = cd{n.re + sig * hh.re, n.im + sig * hh.im};
        }
        for (int b = u; b < B; b += NU) {
          hN[((size_t)b * D + i) * D + j] = n;
          hY[((size_t)b * D + i) * D + j] = yv;
        }
      }
  }
  cd *dY, *dN;
  cf* dW[3];
  int* dDiag;
  check(hipMalloc(&dY, hY.size() * sizeof(cd)), "malloc");
  check(hipMalloc(&dN, hN.size() * sizeof(cd)), "malloc");
  for (auto& p : dW) check(hipMalloc(&p, (size_t)B * D * sizeof(cf)), "malloc");
  check(hipMalloc(&dDiag, (size_t)B * sizeof(int)), "malloc");
  check(hipMemcpy(dY, hY.data(), hY.size() * sizeof(cd), hipMemcpyHostToDevice), "h2d");
  check(hipMemcpy(dN, hN.data(), hN.size() * sizeof(cd), hipMemcpyHostToDevice), "h2d");
  hipEvent_t e0, e1;
  check(hipEventCreate(&e0), "event");
  check(hipEventCreate(&e1), "event");
  auto run = [&](int which) {
    if (which == 0) {
      if (R == 1) hipLaunchKernelGGL((filter_update_kernel_big<DMB, 1, true>), dim3(B), dim3(64), 0, 0, dY, dN, B, D, 1, R, ref, dW[0], dDiag);
      else hipLaunchKernelGGL((filter_update_kernel_big<DMB, kRMax, true>), dim3(B), dim3(64), 0, 0, dY, dN, B, D, 1, R, ref, dW[0], dDiag);
    } else if (which == 1) {
      if (R == 1) hipLaunchKernelGGL((filter_update_kernel_2d<NB8, 1>), dim3(B), dim3(64), 0, 0, dY, dN, B, D, R, ref, dW[1], dDiag);
      else hipLaunchKernelGGL((filter_update_kernel_2d<NB8, kRMax>), dim3(B), dim3(64), 0, 0, dY, dN, B, D, R, ref, dW[1], dDiag);
    } else {
      const int nb = (B + 3) / 4;
      if (R == 1) hipLaunchKernelGGL((filter_update_kernel_2d<NB4, 1, 4>), dim3(nb), dim3(64), 0, 0, dY, dN, B, D, R, ref, dW[2], dDiag);
      else hipLaunchKernelGGL((filter_update_kernel_2d<NB4, kRMax, 4>), dim3(nb), dim3(64), 0, 0, dY, dN, B, D, R, ref, dW[2], dDiag);
    }
  };
  float best[3] = {1e30f, 1e30f, 1e30f};
  for (int which = 0; which < 3; ++which) {
    for (int rep = 0; rep < 4; ++rep) {
      check(hipEventRecord(e0), "record");
      run(which);
      check(hipEventRecord(e1), "record");
      check(hipEventSynchronize(e1), "sync");
      float ms;
      check(hipEventElapsedTime(&ms, e0, e1), "elapsed");
      if (rep > 0) best[which] = std::min(best[which], ms);
    }
  }
  check(hipGetLastError(), "launch");
  std::vector<cf> w[3];
  for (int k = 0; k < 3; ++k) {
    w[k].resize((size_t)B * D);
    check(hipMemcpy(w[k].data(), dW[k], w[k].size() * sizeof(cf), hipMemcpyDeviceToHost), "d2h");
  }
  printf("D=%d B=%d R=%d ref=%d  row-per-lane %.3f ms  grid8 NB=%d %.3f ms  grid4 NB=%d %.3f ms (%.2fx vs grid8)\n", D, B, R,
         ref, best[0], NB8, best[1], NB4, best[2], best[1] / best[2]);
  for (int k = 1; k < 3; ++k) {
    std::vector<double> err(NU);
    for (int u = 0; u < NU; ++u) {
      double num = 0, den = 0;
      for (int i = 0; i < D; ++i) {
        const cf a = w[0][(size_t)u * D + i], b = w[k][(size_t)u * D + i];
        num += (double)(a.re - b.re) * (a.re - b.re) + (double)(a.im - b.im) * (a.im - b.im);
        den += (double)a.re * a.re + (double)a.im * a.im;
      }
      err[u] = std::sqrt(num / std::max(den, 1e-300));
    }
    double dmax = 0;
    for (int b = NU; b < B; ++b)
      for (int i = 0; i < D; ++i) {
        const cf a = w[k][(size_t)(b % NU) * D + i], c = w[k][(size_t)b * D + i];
        dmax = std::max(dmax, (double)std::fabs(a.re - c.re) + std::fabs(a.im - c.im));
      }
    std::sort(err.begin(), err.end());
    printf("  %s vs row-per-lane: median %.2e p99 %.2e max %.2e   tiled-copy max diff %.2e\n", k == 1 ? "grid8" : "grid4",
           err[NU / 2], err[(NU * 99) / 100], err[NU - 1], dmax);
  }
  return 0;
}
