// Phase cost of the wavefront (D 13..64) mixed-precision GEVD filter update
// (danse_amd/csrc/solver64m.hpp) at N2's batch: B independent bins, one per
// wavefront, the production occupancy (one kernel, the phase to stop after
// is a runtime argument, so every variant has the full kernel's registers).
//   stop 0: load only, 1: + float64 Cholesky, 2: + float64 inverse,
//   3: + Li rows to float32 + LDS, 4: + Y = Li A, 5: + C = Y Li^H,
//   6: + Householder tridiagonalisation, 7: full filter (eigen + back-transform)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I danse_amd/csrc big_phases.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include "solver64m.hpp"

using namespace danse;
using namespace danse::big;

#ifndef PH_DMAX
#define PH_DMAX 40
#endif
constexpr int DM = PH_DMAX;

__global__ void __launch_bounds__(64) phases(const cf* __restrict__ Ryy, const cd* __restrict__ Rnn, int D, int stop,
                                             cf* __restrict__ out) {
  __shared__ LDSM<DM> S;
  const int li = threadIdx.x, b = blockIdx.x;
  const bool act = li < D;
  const int row = act ? li : 0;
  Row<DM> A;
  RowD<DM> N;
  rzero(A);
  sfor<0, DM>([&](auto cc) { wsd<decltype(cc)::value>(N, cd{0.0, 0.0}); });
  cols_below<DM>(D, [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    const int cl = (c < D) ? c : D - 1;
    const cf va = Ryy[((long long)b * D + row) * D + cl];
    const cd vn = Rnn[((long long)b * D + row) * D + cl];
    ws<c>(A, (act && c < D) ? va : cf{0.0f, 0.0f});
    wsd<c>(N, (act && c < D) ? vn : cd{0.0, 0.0});
  });
  cf res = cf{0.0f, 0.0f};
  if (stop == 0) {
    sfor<0, DM>([&](auto cc) { res = res + rs<decltype(cc)::value>(A) + cfk(rsd<decltype(cc)::value>(N)); });
    if (act) out[(long long)b * 64 + li] = res;
    return;
  }
  double invd;
  bool ok = chol64_rows<DM>(N, S.m.U64, li, D, invd);
  if (stop == 1) {
    if (act) out[(long long)b * 64 + li] = cfk(S.m.U64[li][li]) + cf{(float)invd, ok ? 1.0f : 0.0f};
    return;
  }
  const cf gi = (li <= 0 && li < D) ? conjg(cfk(S.m.U64[li][0])) : cf{0.0f, 0.0f};
  tri_inv64_cols<DM>(S.m.U64, li, D, invd);
  if (stop == 2) {
    if (act) out[(long long)b * 64 + li] = cfk(S.m.U64[0][li]) + gi;
    return;
  }
  Row<DM> Lr;
  rzero(Lr);
  cols_below<DM>(D, [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c < D && li < DM) ws<c>(Lr, cfk(S.m.U64[c][li]));
  });
  __syncthreads();
  if (li < DM) {
    sfor<0, DM>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      S.m.f.Ls[li][c] = rs<c>(Lr);
      S.m.f.As[li][c] = rs<c>(A);
    });
  }
  S.g[li] = gi;
  __syncthreads();
  if (stop == 3) {
    if (act) out[(long long)b * 64 + li] = S.m.f.Ls[li][0] + S.m.f.As[0][li];
    return;
  }
  Row<DM> Y;
  rzero(Y);
  cols_below<DM>(D, [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if (k < D) {
      const cf lik = rs<k>(Lr);
      cols_below<DM>(D, [&](auto cc) {
        constexpr int c = decltype(cc)::value;
        cf y = rs<c>(Y);
        fma_c(y, lik, S.m.f.As[k][c]);
        ws<c>(Y, y);
      });
    }
  });
  if (stop == 4) {
    sfor<0, DM>([&](auto cc) { res = res + rs<decltype(cc)::value>(Y); });
    if (act) out[(long long)b * 64 + li] = res;
    return;
  }
  rzero(A);
  cols_below<DM>(D, [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if (c < D) {
      cf acc = cf{0.0f, 0.0f};
      sfor<0, c + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        acc = acc + mulc(rs<k>(Y), S.m.f.Ls[c][k]);
      });
      if (!act) acc = cf{0.0f, 0.0f};
      if (li == c) acc.im = 0.0f;
      ws<c>(A, acc);
    }
  });
  __syncthreads();
  if (stop == 5) {
    sfor<0, DM>([&](auto cc) { res = res + rs<decltype(cc)::value>(A); });
    if (act) out[(long long)b * 64 + li] = res;
    return;
  }
  float ta;
  cf tb;
  tridiag<DM>(A, S.m.f.As, li, D, ta, tb);
  if (stop == 6) {
    if (act) out[(long long)b * 64 + li] = tb + cf{ta, 0.0f};
    return;
  }
  // stop 7: the production routine from the start (same loads)
  out[(long long)b * 64 + li] = res;
}

__global__ void __launch_bounds__(64) full(const cf* __restrict__ Ryy, const cd* __restrict__ Rnn, int D, cf* __restrict__ out) {
  __shared__ LDSM<DM> S;
  const int li = threadIdx.x, b = blockIdx.x;
  const bool act = li < D;
  const int row = act ? li : 0;
  Row<DM> A;
  RowD<DM> N;
  rzero(A);
  sfor<0, DM>([&](auto cc) { wsd<decltype(cc)::value>(N, cd{0.0, 0.0}); });
  cols_below<DM>(D, [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    const int cl = (c < D) ? c : D - 1;
    const cf va = Ryy[((long long)b * D + row) * D + cl];
    const cd vn = Rnn[((long long)b * D + row) * D + cl];
    ws<c>(A, (act && c < D) ? va : cf{0.0f, 0.0f});
    wsd<c>(N, (act && c < D) ? vn : cd{0.0, 0.0});
  });
  bool ok;
  const cf w = gevd_filter_mixed<DM, 1>(A, N, S, li, D, 1, 0, ok);
  if (act) out[(long long)b * 64 + li] = w;
}

int main(int argc, char** argv) {
  const int D = argc > 1 ? atoi(argv[1]) : 39;
  const int B = argc > 2 ? atoi(argv[2]) : 16416;
  std::mt19937 rng(1);
  std::normal_distribution<double> nd;
  // random Hermitian positive-definite pairs (a few distinct ones, tiled)
  const int NU = 64;
  std::vector<cf> hA((size_t)B * D * D);
  std::vector<cd> hN((size_t)B * D * D);
  for (int u = 0; u < NU; ++u) {
    std::vector<cd> X((size_t)D * 2 * D), Z((size_t)D * 2 * D);
    for (auto& v : X) v = cd{nd(rng), nd(rng)};
    for (auto& v : Z) v = cd{nd(rng), nd(rng)};
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        cd a{0, 0}, n{0, 0};
        for (int t = 0; t < 2 * D; ++t) {
          const cd xi = X[i * 2 * D + t], xj = X[j * 2 * D + t];
          const cd zi = Z[i * 2 * D + t], zj = Z[j * 2 * D + t];
          a.re += xi.re * xj.re + xi.im * xj.im; a.im += xi.im * xj.re - xi.re * xj.im;
          n.re += zi.re * zj.re + zi.im * zj.im; n.im += zi.im * zj.re - zi.re * zj.im;
        }
        for (int b = u; b < B; b += NU) {
          hA[((size_t)b * D + i) * D + j] = cf{(float)(a.re + n.re), (float)(a.im + n.im)};
          hN[((size_t)b * D + i) * D + j] = n;
        }
      }
  }
  cf *dA, *dOut;
  cd* dN;
  hipMalloc(&dA, hA.size() * sizeof(cf));
  hipMalloc(&dN, hN.size() * sizeof(cd));
  hipMalloc(&dOut, (size_t)B * 64 * sizeof(cf));
  hipMemcpy(dA, hA.data(), hA.size() * sizeof(cf), hipMemcpyHostToDevice);
  hipMemcpy(dN, hN.data(), hN.size() * sizeof(cd), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"load", "+chol64", "+inv64", "+Li to LDS", "+Y=LiA", "+C=YLi^H", "+tridiag"};
  for (int stop = 0; stop <= 6; ++stop) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(phases, dim3(B), dim3(64), 0, 0, dA, dN, D, stop, dOut);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    printf("D=%d B=%d stop %d %-12s %8.3f ms\n", D, B, stop, names[stop], best);
  }
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(full, dim3(B), dim3(64), 0, 0, dA, dN, D, dOut);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  printf("D=%d B=%d full gevd_filter_mixed  %8.3f ms\n", D, B, best);
  hipError_t err = hipGetLastError();
  printf("status %s\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
