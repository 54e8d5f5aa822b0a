// One size class of the update / filter kernels (see classes.hpp); compiled
// once per DMAX with -DDANSE_DMAX=N.
#include "classes.hpp"
#include "kernels_big.hpp"

#ifndef DANSE_DMAX
#error "compile with -DDANSE_DMAX=<2..16>"
#endif

namespace danse {

namespace {
constexpr int kD = DANSE_DMAX;
constexpr int kG = class_group(kD);
constexpr int kNB = 64 / kG;
static_assert(kD >= 2 && kD <= kMaxDMax, "class out of range");
}  // namespace

#define DANSE_CAT2(a, b) a##b
#define DANSE_CAT(a, b) DANSE_CAT2(a, b)

void DANSE_CAT(launch_update_d, DANSE_DMAX)(const UpdateArgs& a, hipStream_t st) {
  const int nBB = (a.F + kNB - 1) / kNB;
  const unsigned grid = (unsigned)(a.S * a.nFN * nBB);
  if constexpr (kG == 64) {
    if (!a.gevd || a.rank == 1)
      hipLaunchKernelGGL((update_kernel_big<kD, 1>), dim3(grid), dim3(64), 0, st, a);
    else
      hipLaunchKernelGGL((update_kernel_big<kD, kRMax>), dim3(grid), dim3(64), 0, st, a);
  } else {
    if (!a.gevd || a.rank == 1)
      hipLaunchKernelGGL((update_kernel<kG, kD, 1>), dim3(grid), dim3(64), 0, st, a);
    else
      hipLaunchKernelGGL((update_kernel<kG, kD, kRMax>), dim3(grid), dim3(64), 0, st, a);
  }
}

void DANSE_CAT(launch_filter_update_d, DANSE_DMAX)(const cf* Ryy, const cf* Rnn, int B, int D, int gevd, int rank,
                                                   int ref, cf* w, int* diag, hipStream_t st) {
  const unsigned grid = (unsigned)((B + kNB - 1) / kNB);
  if constexpr (kG == 64) {
    if (!gevd || rank == 1)
      hipLaunchKernelGGL((filter_update_kernel_big<kD, 1>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, gevd, rank,
                         ref, w, diag);
    else
      hipLaunchKernelGGL((filter_update_kernel_big<kD, kRMax>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, gevd,
                         rank, ref, w, diag);
  } else {
    if (!gevd || rank == 1)
      hipLaunchKernelGGL((filter_update_kernel<kG, kD, 1>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, gevd,
                         rank, ref, w, diag);
    else
      hipLaunchKernelGGL((filter_update_kernel<kG, kD, kRMax>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, gevd,
                         rank, ref, w, diag);
  }
}

}  // namespace danse
