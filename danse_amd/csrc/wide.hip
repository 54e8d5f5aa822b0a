// Wide filter classes (64 < D <= 256): the kernel of wide.hpp and its
// chunked launcher (wide_api.hpp).
#define DANSE_WIDE_KERNEL
#include "wide.hpp"

#include <algorithm>

namespace danse {
namespace wide {

hipError_t launch_wide_filters(const WideArgs& a0, long long chunk, hipStream_t st) {
  if (a0.D < 1 || a0.D > kMaxD || a0.nOut < 1 || a0.nOut > kMaxOut || chunk < 1) return hipErrorInvalidValue;
  if (a0.gevd && (a0.rank < 1 || a0.rank > kRMax || a0.rank > a0.D)) return hipErrorInvalidValue;
  WideArgs a = a0;
  for (long long i0 = 0; i0 < a0.nItems; i0 += chunk) {
    a.item0 = i0;
    const long long n = std::min(chunk, a0.nItems - i0);
    hipLaunchKernelGGL(wide_filter_kernel, dim3((unsigned)n), dim3(kThr), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace wide
}  // namespace danse
