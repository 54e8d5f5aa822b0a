// Host-side interface of the wide filter classes (wide.hpp): filter
// dimensions 64 < D <= 256, one 256-thread workgroup per (SCM pair, bin).
#pragma once
#include <hip/hip_runtime.h>
#include "common.hpp"

namespace danse {
namespace wide {

constexpr int kThr = 256;    // threads per workgroup (one per row / column)
constexpr int kMaxD = 256;   // largest filter dimension
constexpr int kCh = 16;      // rows per register chunk of the column solves
constexpr int kMaxOut = 64;  // outputs (reference indices) per item

struct WideArgs {   // (passed by value: the per-output tables ride in the kernel arguments)
  int D, rank, gevd, F;
  long long nItems, item0;   // item b = item0 + blockIdx.x; (scene, bin) = (b / F, b % F)
  int layout;                // 0: full rows [D][D] (RyyD, Rnn); 1: packed lower, bin-major (RyyF, Rnn);
                             // 2: packed lower, bin-major (RyyD, Rnn)
  const cd* RyyD;
  const cf* RyyF;
  const cd* Rnn;
  long long srcScene, srcBin;   // element strides of the sources
  int nOut;                     // outputs per item (<= kMaxOut, <= D for MWF)
  int refs[kMaxOut];            // reference index of output j
  long long wOff[kMaxOut];      // w[wOff[j] + s * wScene + f * wBin + i]
  cf* w;
  long long wScene, wBin;
  int* diag;                    // [nItems] or null: 1 = factor / eigen failure, 0 ok
  cd* work;                     // [gridDim.x][2][D][D]
  // online engine (scene items): item (s, f) solves only when the flag byte
  // flags[s * flagStride] has DANSE_FLAG_SOLVE and not DANSE_FLAG_PREGIVEN;
  // null = every item solves
  const unsigned char* flags;
  long long flagStride;
};

// Launch wide_filter_kernel over a.nItems items, `chunk` workgroups per
// launch (a.work holds chunk * work_elems(D) complex doubles).
hipError_t launch_wide_filters(const WideArgs& a, long long chunk, hipStream_t st);
inline size_t work_elems(int D) { return (size_t)2 * D * D; }
// workgroups per launch for nItems items: at most 1024 and at most a 1 GiB
// float64 workspace (512 at D = 256), at least one per CU (256)
constexpr size_t kWorkBudget = (size_t)1 << 30;
inline long long chunk_for(int D, long long nItems) {
  long long c = (long long)(kWorkBudget / (work_elems(D) * sizeof(cd)));
  c = c < 256 ? 256 : (c > 1024 ? 1024 : c);
  return nItems < c ? (nItems > 0 ? nItems : 1) : c;
}

}  // namespace wide
}  // namespace danse
