// One size class of the update / filter kernels (see classes.hpp); compiled
// once per DMAX with -DDANSE_DMAX=N.
#include "classes.hpp"
#include "kernels_2d.hpp"
#include "kernels_2dc.hpp"
#include "kernels_big.hpp"
#include "kernels_lane.hpp"

#ifndef DANSE_DMAX
#error "compile with -DDANSE_DMAX=<1..12, 16, 20, 24..64 step 8>"
#endif

namespace danse {

namespace {
constexpr int kD = DANSE_DMAX;
constexpr int kG = class_group(kD);
static_assert(class_dmax(kD) == kD, "DANSE_DMAX is not a class size");
// GEVD of the wavefront classes up to 48 on a lane grid (kernels_2d.hpp):
// 4 x 4 (four bins per wave) for DMAX 16 / 20, 8 x 8 above
constexpr int kGrid = class_grid(kD);
constexpr bool k2D = (kG == 64) && kGrid > 0;
constexpr int kNB = k2D ? kD / kGrid : 2;
constexpr int kBinsPerWave = (kGrid == 4) ? 4 : 1;
// the row-per-lane kernels (MWF of D > 12) unroll over multiples of 8
constexpr int kDBig = ((kD + 7) / 8) * 8;
static_assert(kD >= 1 && kD <= kMaxDMax, "class out of range");
}  // namespace

#define DANSE_CAT2(a, b) a##b
#define DANSE_CAT(a, b) DANSE_CAT2(a, b)

void DANSE_CAT(launch_update_d, DANSE_DMAX)(const UpdateArgs& a, hipStream_t st) {
  const bool r1 = !a.gevd || a.rank == 1;
  if constexpr (kG == 1) {
    const long long lanes = (long long)a.S * a.nFN * a.F;
    const unsigned grid = (unsigned)((lanes + 63) / 64);
    if (a.noSolve) hipLaunchKernelGGL((update_kernel_lane<kD, 1, true, true>), dim3(grid), dim3(64), 0, st, a);
    else if (!a.gevd) hipLaunchKernelGGL((update_kernel_lane<kD, 1, false>), dim3(grid), dim3(64), 0, st, a);
    else if (r1) hipLaunchKernelGGL((update_kernel_lane<kD, 1, true>), dim3(grid), dim3(64), 0, st, a);
    else hipLaunchKernelGGL((update_kernel_lane<kD, kRMax, true>), dim3(grid), dim3(64), 0, st, a);
  } else if constexpr (kG == 64) {
    const unsigned grid = (unsigned)(a.S * a.nFN * a.F);
    if (!a.gevd) {
      hipLaunchKernelGGL((update_kernel_big<kDBig, 1, false>), dim3(grid), dim3(64), 0, st, a);
    } else if constexpr (k2D) {
      const unsigned g2 = (unsigned)(a.S * a.nFN * ((a.F + kBinsPerWave - 1) / kBinsPerWave));
      if (a.splitSolve || a.noSolve) {   // recursion only: the split solves' first launch, or no solver this round
        if (r1) hipLaunchKernelGGL((update_kernel_2d<kNB, 1, kGrid, false, 1>), dim3(g2), dim3(64), 0, st, a);
        else hipLaunchKernelGGL((update_kernel_2d<kNB, kRMax, kGrid, false, 1>), dim3(g2), dim3(64), 0, st, a);
      } else if (r1) {
        hipLaunchKernelGGL((update_kernel_2d<kNB, 1, kGrid>), dim3(g2), dim3(64), 0, st, a);
      } else {
        hipLaunchKernelGGL((update_kernel_2d<kNB, kRMax, kGrid>), dim3(g2), dim3(64), 0, st, a);
      }
    } else {
      if (r1) hipLaunchKernelGGL((update_kernel_big<kDBig, 1, true>), dim3(grid), dim3(64), 0, st, a);
      else hipLaunchKernelGGL((update_kernel_big<kDBig, kRMax, true>), dim3(grid), dim3(64), 0, st, a);
    }
  }
}

// Split solves of a lane class (UpdateArgs.splitSolve): the GEVD rounds of the
// nItems solving items on 4 x 4 lane grids (four bins per wave, NB = 3:
// D 9..12) over the lane class's packed SCMs.  Returns false if the class
// has no split kernel.
bool DANSE_CAT(launch_split_solve_d, DANSE_DMAX)(const UpdateArgs& a, int nItems, hipStream_t st) {
  if (!a.gevd) return false;
  if constexpr (kG == 1 && kD >= 9) {
    const unsigned g2 = (unsigned)(nItems * ((a.F + 3) / 4));
    if (a.rank == 1) hipLaunchKernelGGL((update_kernel_2d<3, 1, 4, true, 2>), dim3(g2), dim3(64), 0, st, a);
    else hipLaunchKernelGGL((update_kernel_2d<3, kRMax, 4, true, 2>), dim3(g2), dim3(64), 0, st, a);
    return true;
  } else if constexpr (k2D) {
    // the solving items of a lane-grid class (full storage)
    const unsigned g2 = (unsigned)(nItems * ((a.F + kBinsPerWave - 1) / kBinsPerWave));
    if (a.rank == 1) hipLaunchKernelGGL((update_kernel_2d<kNB, 1, kGrid, false, 2>), dim3(g2), dim3(64), 0, st, a);
    else hipLaunchKernelGGL((update_kernel_2d<kNB, kRMax, kGrid, false, 2>), dim3(g2), dim3(64), 0, st, a);
    return true;
  } else {
    (void)a; (void)nItems; (void)st;
    return false;
  }
}

bool DANSE_CAT(launch_lean_solve_d, DANSE_DMAX)(const UpdateArgs& a, int nCre, int nCn, int fbGrid, hipStream_t st) {
  if constexpr (k2D && kGrid == 8) {
    if (nCre > 0) hipLaunchKernelGGL((update_kernel_2dc<kNB, false>), dim3((unsigned)(nCre * a.F)), dim3(64), 0, st, a);
    if (nCn > 0) hipLaunchKernelGGL((update_kernel_2dc<kNB, true>), dim3((unsigned)(nCn * a.F)), dim3(64), 0, st, a);
    hipLaunchKernelGGL((fallback_kernel_2d<kNB>), dim3((unsigned)fbGrid), dim3(64), 0, st, a);
    return true;
  } else {
    (void)a; (void)nCre; (void)nCn; (void)fbGrid; (void)st;
    return false;
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
      hipLaunchKernelGGL((filter_update_kernel_big<kDBig, 1, false>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, gevd,
                         rank, ref, w, diag);
    } else if constexpr (k2D) {
      const unsigned g2 = (unsigned)((B + kBinsPerWave - 1) / kBinsPerWave);
      if (r1)
        hipLaunchKernelGGL((filter_update_kernel_2d<kNB, 1, kGrid>), dim3(g2), dim3(64), 0, st, Ryy, Rnn, B, D, rank,
                           ref, w, diag);
      else
        hipLaunchKernelGGL((filter_update_kernel_2d<kNB, kRMax, kGrid>), dim3(g2), dim3(64), 0, st, Ryy, Rnn, B, D,
                           rank, ref, w, diag);
    } else {
      if (r1)
        hipLaunchKernelGGL((filter_update_kernel_big<kDBig, 1, true>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D, gevd,
                           rank, ref, w, diag);
      else
        hipLaunchKernelGGL((filter_update_kernel_big<kDBig, kRMax, true>), dim3(grid), dim3(64), 0, st, Ryy, Rnn, B, D,
                           gevd, rank, ref, w, diag);
    }
  }
}

}  // namespace danse
