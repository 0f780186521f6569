// Microbenchmark (diagnostics only): random 4/16-byte loads per lane from a
// table of T bytes, 16 waves per CU, D independent loads in flight per lane.
// Prints G loads/s per table size -- the rate a per-position HBM probe gets.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int D, typename V>
__global__ __launch_bounds__(1024) void rl(const V* __restrict__ t, uint32_t mask, uint32_t iters, uint32_t* sink) {
  uint32_t x = (blockIdx.x * 1024u + threadIdx.x) * 2654435761u + 12345u;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < iters; ++i) {
    V v[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      x = x * 1664525u + 1013904223u;
      v[d] = t[(x >> 3) & mask];
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if constexpr (sizeof(V) == 4) acc += (uint32_t)v[d];
      else acc += v[d].x ^ v[d].w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int D, typename V>
void run(size_t bytes, const char* name) {
  V* t;
  hipMalloc(&t, bytes);
  hipMemset(t, 1, bytes);
  uint32_t* sink;
  hipMalloc(&sink, 4);
  const uint32_t n = (uint32_t)(bytes / sizeof(V));
  const uint32_t iters = 64;
  dim3 g(256 * 2), b(1024);
  hipLaunchKernelGGL((rl<D, V>), g, b, 0, 0, t, n - 1, iters, sink);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((rl<D, V>), g, b, 0, 0, t, n - 1, iters, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double loads = 5.0 * g.x * b.x * (double)iters * D;
  printf("%-6s D=%d table %7.1f MiB: %7.1f G loads/s (%.1f GB/s useful)\n", name, D, bytes / 1048576.0,
         loads / (ms * 1e-3) / 1e9, loads * sizeof(V) / (ms * 1e-3) / 1e9);
  hipFree(t);
  hipFree(sink);
}

int main() {
  for (size_t mb : {1, 2, 4, 8, 16, 64, 1024}) {
    run<8, uint32_t>(mb << 20, "u32");
    run<8, uint4>(mb << 20, "u32x4");
  }
  run<16, uint32_t>(2 << 20, "u32");
  run<4, uint32_t>(2 << 20, "u32");
  return 0;
}
