// Host entry points of the resident engine translation unit (resident.hip),
// called by danse_engine.hip's danse_engine_run_resident.
#pragma once
#include "bcast.hpp"

namespace danse {
namespace res {
struct ResArgs;
}
// NB: lane-grid blocks per lane (3, 4, 5); rank1: RMAX = 1 instantiation.
// check: only compute *fits (waves the device holds at once) and return 1
// if grid exceeds it.  0 on success.
int resident_launch(int NB, int rank1, const res::ResArgs& ra, int grid, hipStream_t st, bool check, int* fits);
void resident_analysis(const BcastArgs& a, const int* chanNode, cf* YB, cf* YU, hipStream_t st);
void resident_synth(const BcastArgs& a, const int* fams, int nFam, float* frames, hipStream_t st);
}  // namespace danse
