// One size class of the update / filter kernels (see classes.hpp); compiled
// once per DMAX with -DDANSE_DMAX=N.
#include "classes.hpp"
#include "kernels_2d.hpp"
#include "kernels_big.hpp"
#include "kernels_lane.hpp"

#ifndef DANSE_DMAX
#error "compile with -DDANSE_DMAX=<1..12, 16..64 step 8>"
#endif

namespace danse {

namespace {
constexpr int kD = DANSE_DMAX;
constexpr int kG = class_group(kD);
// GEVD of the wavefront classes up to 48 on the 8 x 8 lane grid (kernels_2d.hpp)
constexpr bool k2D = (kG == 64) && kD <= 48;
constexpr int kNB = k2D ? kD / 8 : 2;
static_assert(kD >= 1 && kD <= kMaxDMax, "class out of range");
}  // namespace

#define DANSE_CAT2(a, b) a##b
#define DANSE_CAT(a, b) DANSE_CAT2(a, b)

void DANSE_CAT(launch_update_d, DANSE_DMAX)(const UpdateArgs& a, hipStream_t st) {
  const bool r1 = !a.gevd || a.rank == 1;
  if constexpr (kG == 1) {
    const long long lanes = (long long)a.S * a.nFN * a.F;
    const unsigned grid = (unsigned)((lanes + 63) / 64);
    if (!a.gevd) hipLaunchKernelGGL((update_kernel_lane<kD, 1, false>), dim3(grid), dim3(64), 0, st, a);
    else if (r1) hipLaunchKernelGGL((update_kernel_lane<kD, 1, true>), dim3(grid), dim3(64), 0, st, a);
    else hipLaunchKernelGGL((update_kernel_lane<kD, kRMax, true>), dim3(grid), dim3(64), 0, st, a);
  } else if constexpr (kG == 64) {
    const unsigned grid = (unsigned)(a.S * a.nFN * a.F);
    if (!a.gevd) {
      hipLaunchKernelGGL((update_kernel_big<kD, 1, false>), dim3(grid), dim3(64), 0, st, a);
    } else if constexpr (k2D) {
      if (r1) hipLaunchKernelGGL((update_kernel_2d<kNB, 1>), dim3(grid), dim3(64), 0, st, a);
      else hipLaunchKernelGGL((update_kernel_2d<kNB, kRMax>), dim3(grid), dim3(64), 0, st, a);
    } else {
      if (r1) hipLaunchKernelGGL((update_kernel_big<kD, 1, true>), dim3(grid), dim3(64), 0, st, a);
      else hipLaunchKernelGGL((update_kernel_big<kD, kRMax, true>), dim3(grid), dim3(64), 0, st, a);
    }
  }
}

void DANSE_CAT(launch_filter_update_d, DANSE_DMAX)(const cd* Ryy, const cd* Rnn, int B, int D, int gevd, int rank,
                                                   int ref, cf* w, int* diag, hipStream_t st) {
  const bool r1 = !gevd || rank == 1;
  if constexpr (kG == 1) {
    const unsigned grid = (unsigned)((B + 63) / 64);
    if (r1)
      hipLaunchKernelGGL((filter_update_kernel_lane<kD, 1>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, gevd, rank,
                         ref, w, diag);
    else
      hipLaunchKernelGGL((filter_update_kernel_lane<kD, kRMax>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, gevd,
                         rank, ref, w, diag);
  } else if constexpr (kG == 64) {
    const unsigned grid = (unsigned)B;
    if (!gevd) {
      hipLaunchKernelGGL((filter_update_kernel_big<kD, 1, false>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, gevd,
                         rank, ref, w, diag);
    } else if constexpr (k2D) {
      if (r1)
        hipLaunchKernelGGL((filter_update_kernel_2d<kNB, 1>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, rank, ref,
                           w, diag);
      else
        hipLaunchKernelGGL((filter_update_kernel_2d<kNB, kRMax>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, rank,
                           ref, w, diag);
    } else {
      if (r1)
        hipLaunchKernelGGL((filter_update_kernel_big<kD, 1, true>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, gevd,
                           rank, ref, w, diag);
      else
        hipLaunchKernelGGL((filter_update_kernel_big<kD, kRMax, true>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D,
                           gevd, rank, ref, w, diag);
    }
  }
}

}  // namespace danse
