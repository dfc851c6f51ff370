// gather_probe.hip — known-byte read patterns for calibrating rocprofv3's FETCH_SIZE on gfx950
// (VERDICT r4 item 6).  The guide calibrates FETCH_SIZE only for 16 B/lane streaming reads
// (FETCH_SIZE = TCC_EA0_RDREQ x 64 B, half the bytes); the row-walk decode reads 1-8 B per lane at
// scattered row addresses.  Each kernel below reads a buffer far larger than the 256 MiB Infinity
// Cache with a known set of lines, so its true memory-side bytes are known:
//   stream16    16 B per lane, coalesced, every byte once                    -> B bytes
//   gather128   8 B per lane at the start of each 128-B line, lines in a     -> B bytes of lines
//               bijective pseudo-random order (one lane per line)               (8 B of each used)
//   gather64    8 B per lane at the start of each 64-B half line, random     -> B bytes of lines
//   gather32    8 B per lane at the start of each 32-B sector, random        -> B bytes of lines
//   rowwalk     a lane per 296-B row (rows contiguous), each lane reading     -> B bytes
//               its row's 37 words one after the other (the walk's pattern)
// Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
// TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum` (separate passes); scripts/r05_gather_probe.sh.
//   hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o tools/gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

using v4 = __attribute__((ext_vector_type(4))) uint32_t;

__global__ __launch_bounds__(256) void stream16(const v4* __restrict__ s, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const v4 t = s[i];
    acc ^= t.x ^ t.y ^ t.z ^ t.w;
  }
  if (acc == 0x12345678u) *out = acc;
}

// one 8-B load from each of `units` (a power of two) units of `ub` bytes, in the bijective order
// u -> (u * odd) mod units
__global__ __launch_bounds__(256) void gather(const uint8_t* __restrict__ s, size_t units, int ub,
                                              uint32_t* out) {
  uint64_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < units; i += (size_t)gridDim.x * 256) {
    const size_t u = (i * 0x9E3779B97F4A7C15ull) & (units - 1);
    acc ^= *reinterpret_cast<const uint64_t*>(s + u * ub);
  }
  if (acc == 0x1234567812345678ull) *out = 1;
}

constexpr int kRow = 296;
__global__ __launch_bounds__(256) void rowwalk(const uint8_t* __restrict__ s, size_t rows, uint32_t* out) {
  const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const uint64_t* p = reinterpret_cast<const uint64_t*>(s + r * kRow);
  uint64_t acc = 0;
  for (int w = 0; w < kRow / 8; w++) acc = (acc ^ p[w]) * 3;   // dependent, like the walk
  if (acc == 0x1234567812345678ull) *out = 1;
}

int main() {
  const size_t bytes = size_t(1) << 30;              // 1 GiB, 4x the Infinity Cache
  uint8_t* buf = nullptr;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&buf, bytes + 4096));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(buf, 1, bytes + 4096));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto time = [&](const char* name, double known, auto launch) {
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"kernel\": \"%s\", \"known_bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n", name, known,
           ms, known / (ms * 1e-3) / 1e9);
  };
  time("stream16", double(bytes), [&] {
    hipLaunchKernelGGL(stream16, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const v4*>(buf), bytes / 16, out);
  });
  for (int ub : {128, 64, 32}) {
    const size_t units = bytes / ub;
    const char* nm = ub == 128 ? "gather128" : ub == 64 ? "gather64" : "gather32";
    time(nm, double(bytes), [&] {
      hipLaunchKernelGGL(gather, dim3(8192), dim3(256), 0, 0, buf, units, ub, out);
    });
  }
  const size_t rows = bytes / kRow;
  time("rowwalk", double(rows * kRow), [&] {
    hipLaunchKernelGGL(rowwalk, dim3((rows + 255) / 256), dim3(256), 0, 0, buf, rows, out);
  });
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
