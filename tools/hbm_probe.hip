// hbm_probe.hip — measures what plain streaming kernels reach on this MI355X, to calibrate the
// row codec's roofline fraction: copy (read+write), read-only, write-only, 16 B per lane,
// with/without non-temporal hints, several grid shapes.  Standalone binary:
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe && tools/hbm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

using v4 = __attribute__((ext_vector_type(4))) uint32_t;

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const v4* __restrict__ s, v4* __restrict__ d,
                                              size_t n) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (; i + (U - 1) * 256 < n; i += stride) {
    v4 t[U];
#pragma unroll
    for (int u = 0; u < U; u++) t[u] = NT ? __builtin_nontemporal_load(s + i + u * 256) : s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (NT) __builtin_nontemporal_store(t[u], d + i + u * 256);
      else d[i + u * 256] = t[u];
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_k(const v4* __restrict__ s, size_t n, uint32_t* out) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256 * U;
  uint32_t acc = 0;
  for (; i + (U - 1) * 256 < n; i += stride) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      v4 t = s[i + u * 256];
      acc ^= t.x ^ t.y ^ t.z ^ t.w;
    }
  }
  if (acc == 0x12345678u) *out = acc;
}

template <int U>
__global__ __launch_bounds__(256) void write_k(v4* __restrict__ d, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256 * U;
  v4 z = {1, 2, 3, 4};
  for (; i + (U - 1) * 256 < n; i += stride) {
#pragma unroll
    for (int u = 0; u < U; u++) d[i + u * 256] = z;
  }
}

// 8-byte-per-lane streams (the encode kernel's column reads / decode kernel's column writes),
// for calibrating FETCH_SIZE / WRITE_SIZE at that access width.
__global__ __launch_bounds__(256) void read8_k(const uint64_t* __restrict__ s, size_t n, uint32_t* out) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t acc = 0;
  for (; i < n; i += (size_t)gridDim.x * 256) acc ^= __builtin_nontemporal_load(s + i);
  if (acc == 0x12345678ull) *out = 1;
}
__global__ __launch_bounds__(256) void write8_k(uint64_t* __restrict__ d, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * 256) __builtin_nontemporal_store((uint64_t)i, d + i);
}

template <typename F>
float time_ms(F f, int iters) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; i++) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : (size_t)816 << 20;
  const size_t n = bytes / 16;
  v4 *s, *d;
  uint32_t* o;
  CHECK(hipMalloc(&s, bytes));
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&o, 4));
  CHECK(hipMemset(s, 1, bytes));
  CHECK(hipMemset(d, 0, bytes));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("{\"bytes_per_buffer\": %zu, \"cus\": %d, \"results\": [\n", bytes, cus);
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  bool first = true;
  auto rep = [&](const char* name, int grid, double moved, float ms) {
    printf("%s {\"kernel\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
           first ? "" : ",", name, grid, ms, moved / ms / 1e6);
    first = false;
  };
  for (int grid : {cus * 4, cus * 8, cus * 16, (int)((n + 1023) / 1024)}) {
    rep("copy_u4", grid, 2.0 * bytes, time_ms([&] { copy_k<4, false><<<grid, 256>>>(s, d, n); }, iters));
    rep("copy_u4_nt", grid, 2.0 * bytes, time_ms([&] { copy_k<4, true><<<grid, 256>>>(s, d, n); }, iters));
    rep("copy_u8", grid, 2.0 * bytes, time_ms([&] { copy_k<8, false><<<grid, 256>>>(s, d, n); }, iters));
    rep("read_u4", grid, 1.0 * bytes, time_ms([&] { read_k<4><<<grid, 256>>>(s, n, o); }, iters));
    rep("write_u4", grid, 1.0 * bytes, time_ms([&] { write_k<4><<<grid, 256>>>(d, n); }, iters));
  }
  rep("read8_nt", cus * 16, 1.0 * bytes,
      time_ms([&] { read8_k<<<cus * 16, 256>>>((const uint64_t*)s, bytes / 8, o); }, iters));
  rep("write8_nt", cus * 16, 1.0 * bytes,
      time_ms([&] { write8_k<<<cus * 16, 256>>>((uint64_t*)d, bytes / 8); }, iters));
  rep("hipMemcpyD2D", 0, 2.0 * bytes,
      time_ms([&] { CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); }, iters));
  printf("]}\n");
  return 0;
}
