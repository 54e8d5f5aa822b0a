// Graph-safe device fills.
//
// A hipMemsetAsync captured into a HIP graph (stream capture) became a memset
// node that the FIRST launch of the graph applied and later launches did not
// apply correctly (scripts/graph_replay_check.py on MI355X, DESIGN.md §6.2:
// zero fills and 0xff fills, torch-allocated and engine-allocated buffers).
// The online engine's state reset, the speculative gate's verdict reset and
// the DXCP estimator reset can all end up inside captured round sequences
// (danse_engine_run's own graph, dist.ShardedRun's CUDA graph), so they fill
// through this kernel instead: a kernel node replays like any other.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace {   // internal linkage: one copy per translation unit
namespace fillk {

__global__ void __launch_bounds__(256) fill32_kernel(uint32_t* __restrict__ p, uint32_t v, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

__global__ void __launch_bounds__(256) fill8_kernel(uint8_t* __restrict__ p, uint8_t v, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

__global__ void __launch_bounds__(256) copy32_kernel(uint32_t* __restrict__ d, const uint32_t* __restrict__ s, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) d[i] = s[i];
}

__global__ void __launch_bounds__(256) copy8_kernel(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) d[i] = s[i];
}

}  // namespace fillk
}  // namespace

// Device-to-device copy as a kernel node (a captured hipMemcpyAsync becomes a
// memcpy node: the same node type family as the memset nodes above, so the
// copies on capturable paths -- the DXCP input recording -- go through this).
static inline hipError_t copy_async(void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (bytes == 0) return hipSuccess;
  if ((((uintptr_t)dst | (uintptr_t)src) & 3u) == 0 && (bytes & 3u) == 0) {
    const size_t n = bytes / 4;
    const unsigned blocks = (unsigned)(n < (size_t)256 * 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(fillk::copy32_kernel, dim3(blocks), dim3(256), 0, st, (uint32_t*)dst, (const uint32_t*)src, n);
  } else {
    const unsigned blocks = (unsigned)(bytes < (size_t)256 * 4096 ? (bytes + 255) / 256 : 4096);
    hipLaunchKernelGGL(fillk::copy8_kernel, dim3(blocks), dim3(256), 0, st, (uint8_t*)dst, (const uint8_t*)src, bytes);
  }
  return hipGetLastError();
}

// hipMemsetAsync's signature: every byte of [p, p + bytes) set to (uint8_t)value.
static inline hipError_t fill_async(void* p, int value, size_t bytes, hipStream_t st) {
  if (bytes == 0) return hipSuccess;
  const uint32_t b = (uint32_t)(value & 0xff);
  if (((uintptr_t)p & 3u) == 0 && (bytes & 3u) == 0) {
    const size_t n = bytes / 4;
    const unsigned blocks = (unsigned)(n < (size_t)256 * 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(fillk::fill32_kernel, dim3(blocks), dim3(256), 0, st, (uint32_t*)p, b * 0x01010101u, n);
  } else {
    const unsigned blocks = (unsigned)(bytes < (size_t)256 * 4096 ? (bytes + 255) / 256 : 4096);
    hipLaunchKernelGGL(fillk::fill8_kernel, dim3(blocks), dim3(256), 0, st, (uint8_t*)p, (uint8_t)b, bytes);
  }
  return hipGetLastError();
}
