// probe.hip — the same-device streaming copy bench.py times beside the codec (fury_hbm_copy): 16-B
// non-temporal loads and stores, four in flight per lane, grid-stride over whole 4 KB blocks.  It is
// the box's achievable copy rate for the roofline line (`roofline.copy_GBps`): the codec kernels'
// 1.0x-traffic streams cannot beat it, so `frac_of_copy` separates a slow box from a slow kernel
// (VERDICT r5 item 6).  tools/hbm_probe.hip measured the same shape at 5.5-6.1 TB/s in round 1.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "kernels.h"

namespace fury {
namespace {

using v4 = __attribute__((ext_vector_type(4))) uint32_t;
constexpr int kCopyThreads = 256, kCopyUnroll = 4;

__global__ __launch_bounds__(kCopyThreads) void hbm_copy_kernel(const v4* __restrict__ s,
                                                                v4* __restrict__ d, int64_t n) {
  const int64_t block = static_cast<int64_t>(kCopyThreads) * kCopyUnroll;
  int64_t i = static_cast<int64_t>(blockIdx.x) * block + threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * block;
  for (; i + (kCopyUnroll - 1) * kCopyThreads < n; i += stride) {
    v4 t[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; u++) t[u] = __builtin_nontemporal_load(s + i + u * kCopyThreads);
#pragma unroll
    for (int u = 0; u < kCopyUnroll; u++) __builtin_nontemporal_store(t[u], d + i + u * kCopyThreads);
  }
}

}  // namespace
}  // namespace fury

extern "C" int fury_hbm_copy(void* dst, const void* src, int64_t bytes, void* stream) {
  using namespace fury;
  const int64_t block = static_cast<int64_t>(kCopyThreads) * kCopyUnroll * 16;
  if (!dst || !src || bytes <= 0 || bytes % block || (reinterpret_cast<uintptr_t>(dst) & 15) ||
      (reinterpret_cast<uintptr_t>(src) & 15))
    return set_error(FURY_ERR_INVALID_ARGUMENT,
                     "fury_hbm_copy: 16-byte aligned buffers, bytes a positive multiple of 16 KB");
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int64_t blocks = bytes / block;
  const int64_t grid = blocks < 16LL * cus ? blocks : 16LL * cus;     // 16 groups per CU in flight
  hipLaunchKernelGGL(hbm_copy_kernel, dim3(static_cast<unsigned>(grid)), dim3(kCopyThreads), 0,
                     static_cast<hipStream_t>(stream), static_cast<const v4*>(src),
                     static_cast<v4*>(dst), bytes / 16);
  return check_hip(hipGetLastError(), "fury_hbm_copy launch");
}
