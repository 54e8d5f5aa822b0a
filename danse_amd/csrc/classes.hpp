// Size classes of the update / filter kernels, one translation unit each
// (update_class.hip compiled with -DDANSE_DMAX=N, so the build parallelises;
// the engine dispatches by DMAX at launch time):
//   D <= kLaneMaxD   one bin per LANE, packed-triangle SCMs (kernels_lane.hpp,
//                    solver_mixed.hpp)
//   D in 13..20      GEVD: four bins per wavefront on 4 x 4 lane grids
//                    (kernels_2d.hpp / solver2d.hpp, G = 4), DMAX 16 or 20
//   D in 21..48      GEVD: one bin per wavefront on the 8 x 8 lane grid (G = 8),
//                    DMAX = D rounded up to a multiple of 8
//   otherwise        one bin per wavefront, runtime pivot loops (kernels_big.hpp,
//                    solver64m.hpp): the MWF of D > 12, the GEVD of D > 48
#pragma once
#include "kernels.hpp"

namespace danse {

constexpr int kMaxDMax = 64;
constexpr int kLaneMaxD = 12;
constexpr int class_dmax(int D) { return D <= kLaneMaxD ? D : D <= 20 ? ((D + 3) / 4) * 4 : ((D + 7) / 8) * 8; }
constexpr int class_group(int DMAX) { return DMAX <= kLaneMaxD ? 1 : 64; }
// lane-grid side of the GEVD solver of a wavefront class (8 x 8 or 4 x 4),
// 0 for the row-per-lane classes
constexpr int class_grid(int DMAX) { return (DMAX == 16 || DMAX == 20) ? 4 : (DMAX > kLaneMaxD && DMAX <= 48) ? 8 : 0; }
// GEVD factor cache record per bin of a grid class (solver2d.hpp li_record)
constexpr long long class_li_record(int DMAX) {
  return (long long)DMAX * (DMAX + 1) / 2 +
         (class_grid(DMAX) == 4 ? 16LL * ((DMAX + 15) / 16) : 64LL);
}
// SCM storage of a class: packed lower triangle, bin-minor ([D(D+1)/2][F])
// for the lane kernels; full rows ([F][D][D]) otherwise.
constexpr bool class_packed(int D) { return D <= kLaneMaxD; }

#define DANSE_FOR_EACH_CLASS(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(16) X(20) X(24) X(32) X(40) X(48) X(56) X(64)

#define DANSE_DECLARE_CLASS(N)                                                                      \
  void launch_update_d##N(const UpdateArgs& a, hipStream_t st);                                     \
  bool launch_split_solve_d##N(const UpdateArgs& a, int nItems, hipStream_t st);                    \
  bool launch_lean_solve_d##N(const UpdateArgs& a, int nCre, int nCn, int fbGrid, hipStream_t st);  \
  void launch_filter_update_d##N(const cd* Ryy, const cd* Rnn, int B, int D, int gevd, int rank,   \
                                 int ref, cf* w, int* diag, hipStream_t st);
DANSE_FOR_EACH_CLASS(DANSE_DECLARE_CLASS)
#undef DANSE_DECLARE_CLASS

inline bool launch_update_class(int DMAX, const UpdateArgs& a, hipStream_t st) {
  switch (DMAX) {
#define DANSE_CASE(N) \
  case N: launch_update_d##N(a, st); return true;
    DANSE_FOR_EACH_CLASS(DANSE_CASE)
#undef DANSE_CASE
    default: return false;
  }
}

inline bool launch_split_solve_class(int DMAX, const UpdateArgs& a, int nItems, hipStream_t st) {
  switch (DMAX) {
#define DANSE_CASE(N) \
  case N: return launch_split_solve_d##N(a, nItems, st);
    DANSE_FOR_EACH_CLASS(DANSE_CASE)
#undef DANSE_CASE
    default: return false;
  }
}
// the solves on the cached factor and C of an 8 x 8 grid class
// (kernels_2dc.hpp): update_kernel_2dc over the nCre VAD-frame and nCn
// noise-frame items, then
// fallback_kernel_2d (fbGrid workgroups) over the bins it sent back
inline bool launch_lean_solve_class(int DMAX, const UpdateArgs& a, int nCre, int nCn, int fbGrid, hipStream_t st) {
  switch (DMAX) {
#define DANSE_CASE(N) \
  case N: return launch_lean_solve_d##N(a, nCre, nCn, fbGrid, st);
    DANSE_FOR_EACH_CLASS(DANSE_CASE)
#undef DANSE_CASE
    default: return false;
  }
}
// the classes with split solves (update_class.hip): the GEVD of the lane
// classes D 9..12 and of the lane-grid classes
constexpr bool class_split(int DMAX) { return (DMAX >= 9 && DMAX <= kLaneMaxD) || class_grid(DMAX) > 0; }
constexpr long long class_split_li_record() { return 12LL * 13 / 2 + 16; }   // li_record<3, 4>

inline bool launch_filter_update_class(int DMAX, const cd* Ryy, const cd* Rnn, int B, int D, int gevd, int rank,
                                       int ref, cf* w, int* diag, hipStream_t st) {
  switch (DMAX) {
#define DANSE_CASE(N) \
  case N: launch_filter_update_d##N(Ryy, Rnn, B, D, gevd, rank, ref, w, diag, st); return true;
    DANSE_FOR_EACH_CLASS(DANSE_CASE)
#undef DANSE_CASE
    default: return false;
  }
}

}  // namespace danse
