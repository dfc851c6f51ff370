// transpose_probe.hip — DIAGNOSTIC: the Struct-100 encode/decode access patterns without LDS,
// to separate the cost of the memory pattern from the cost of the kernels' LDS staging.
//   gather_read   each workgroup reads 100 columns x 64 rows x 8 B (the encode's column reads)
//   contig_read   each workgroup reads one contiguous 52,224-B tile (the decode's row reads)
//   gather_copy   column reads + the tile written contiguously (the encode's pattern)
//   contig_scatter  contiguous tile read + 100 column chunks written (the decode's pattern)
// 1M rows, 100 columns of 8 MB (separate allocations), rows 816 B; nt loads/stores throughout.
// Prints one JSON line: ms and GB/s (bytes actually moved) per kernel.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

namespace {

constexpr int kThreads = 256;
constexpr int kCols = 100;
constexpr int kR = 64;
constexpr int kRow = 816;
constexpr int kTile = kR * kRow;     // 52,224 B

struct Cols {
  const uint64_t* c[kCols];
};
struct OutCols {
  uint64_t* c[kCols];
};

using v4u = __attribute__((ext_vector_type(4))) uint32_t;

__global__ __launch_bounds__(kThreads) void gather_read(Cols a, uint64_t* sink) {
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kR;
  uint64_t acc = 0;
  for (int base = threadIdx.x; base < kCols * kR; base += kThreads * 8) {
    uint64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = base + u * kThreads;
      const int c = __builtin_amdgcn_readfirstlane(min(idx, kCols * kR - 1) / kR);
      v[u] = idx < kCols * kR ? __builtin_nontemporal_load(a.c[c] + r0 + (idx - c * kR)) : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) acc ^= v[u];
  }
  if (acc == 0x123456789abcdefull) sink[threadIdx.x] = acc;   // never true: keeps the loads
}

__global__ __launch_bounds__(kThreads) void contig_read(const uint8_t* rows, uint64_t* sink) {
  const v4u* t = reinterpret_cast<const v4u*>(rows + static_cast<int64_t>(blockIdx.x) * kTile);
  uint32_t acc = 0;
  constexpr int n16 = kTile / 16;
  v4u x[13];
#pragma unroll
  for (int k = 0; k < 13; k++) {
    const int i = threadIdx.x + k * kThreads;
    x[k] = i < n16 ? __builtin_nontemporal_load(t + i) : v4u{0, 0, 0, 0};
  }
#pragma unroll
  for (int k = 0; k < 13; k++) acc ^= x[k].x ^ x[k].y ^ x[k].z ^ x[k].w;
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

template <int R>
__global__ __launch_bounds__(kThreads) void gather_copy(Cols a, uint8_t* rows) {
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  uint64_t acc = 0;
  for (int base = threadIdx.x; base < kCols * R; base += kThreads * 8) {
    uint64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = base + u * kThreads;
      const int c = __builtin_amdgcn_readfirstlane(min(idx, kCols * R - 1) / R);
      v[u] = idx < kCols * R ? __builtin_nontemporal_load(a.c[c] + r0 + (idx - c * R)) : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) acc ^= v[u];
  }
  v4u* t = reinterpret_cast<v4u*>(rows + static_cast<int64_t>(blockIdx.x) * R * kRow);
  const v4u w = {static_cast<uint32_t>(acc), static_cast<uint32_t>(acc >> 32), 0u, 0u};
  for (int i = threadIdx.x; i < R * kRow / 16; i += kThreads) __builtin_nontemporal_store(w, t + i);
}

__global__ __launch_bounds__(kThreads) void contig_scatter(const uint8_t* rows, OutCols o) {
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kR;
  const v4u* t = reinterpret_cast<const v4u*>(rows + static_cast<int64_t>(blockIdx.x) * kTile);
  constexpr int n16 = kTile / 16;
  v4u x[13];
#pragma unroll
  for (int k = 0; k < 13; k++) {
    const int i = threadIdx.x + k * kThreads;
    x[k] = i < n16 ? __builtin_nontemporal_load(t + i) : v4u{0, 0, 0, 0};
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 13; k++) acc ^= x[k].x ^ x[k].y ^ x[k].z ^ x[k].w;
  // pair mode: a lane stores rows 2q, 2q + 1 of one column (half a wave per column)
  const int lane = threadIdx.x & 63;
  for (int base = threadIdx.x; base < kCols * kR / 2; base += kThreads) {
    const int c = __builtin_amdgcn_readfirstlane((base - lane) / 32) + (lane >> 5);
    const int q = base - c * 32;
    const v4u w = {acc, acc, acc, acc};
    __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(o.c[c] + r0 + 2 * q));
  }
}

}  // namespace

int main() {
  const int64_t n = 1000000, ntiles = n / kR + 1;
  std::vector<uint64_t*> cols(kCols);
  for (auto& c : cols) hipMalloc(&c, (ntiles * kR) * 8);
  uint8_t* rows = nullptr;
  hipMalloc(&rows, ntiles * kTile);
  uint64_t* sink = nullptr;
  hipMalloc(&sink, 4096);
  hipMemset(rows, 1, ntiles * kTile);
  for (auto& c : cols) hipMemset(c, 2, (ntiles * kR) * 8);
  Cols a;
  OutCols o;
  for (int i = 0; i < kCols; i++) {
    a.c[i] = cols[i];
    o.c[i] = cols[i];
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int g = static_cast<int>(n / kR);
  const double colb = static_cast<double>(g) * kR * 8 * kCols, rowb = static_cast<double>(g) * kTile;
  struct Leg { const char* name; double bytes; int which; };
  const Leg legs[] = {{"gather_read", colb, 0}, {"contig_read", rowb, 1},
                      {"gather_copy", colb + rowb, 2}, {"contig_scatter", rowb + colb, 3},
                      {"gather_copy_R32", colb + rowb, 4}, {"gather_copy_R128", colb + rowb, 5},
                      {"gather_copy_R256", colb + rowb, 6}};
  printf("{\"rows\": %lld", static_cast<long long>(g) * kR);
  for (const Leg& L : legs) {
    float best = 1e30f;
    for (int rep = 0; rep < 7; rep++) {
      hipEventRecord(e0);
      for (int it = 0; it < 10; it++) {
        switch (L.which) {
          case 0: hipLaunchKernelGGL(gather_read, dim3(g), dim3(kThreads), 0, 0, a, sink); break;
          case 1: hipLaunchKernelGGL(contig_read, dim3(g), dim3(kThreads), 0, 0, rows, sink); break;
          case 2: hipLaunchKernelGGL(gather_copy<64>, dim3(g), dim3(kThreads), 0, 0, a, rows); break;
          case 4: hipLaunchKernelGGL(gather_copy<32>, dim3(2 * g), dim3(kThreads), 0, 0, a, rows); break;
          case 5: hipLaunchKernelGGL(gather_copy<128>, dim3(g / 2), dim3(kThreads), 0, 0, a, rows); break;
          case 6: hipLaunchKernelGGL(gather_copy<256>, dim3(g / 4), dim3(kThreads), 0, 0, a, rows); break;
          case 3: hipLaunchKernelGGL(contig_scatter, dim3(g), dim3(kThreads), 0, 0, rows, o); break;
        }
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 10;
      if (rep > 0 && ms < best) best = ms;
    }
    printf(", \"%s\": {\"ms\": %.4f, \"GBps\": %.1f}", L.name, best, L.bytes / (best * 1e-3) / 1e9);
  }
  printf("}\n");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
