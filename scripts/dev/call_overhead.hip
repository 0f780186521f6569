// Diagnostics: the fixed cost of one host-driven call on this box -- what a
// per-call decode() (xcg_decode_call) pays around its kernel.  Each line is
// the median of 2000 iterations, us:
//   launch+sync        empty kernel, hipStreamSynchronize
//   h2d+launch+d2h     64 KiB in, kernel, 88 KiB back (pinned staging), sync
//   launch+poll        empty kernel that stores a flag into pinned host memory; the host spins on it
//   zc 64K in/out+poll kernel reads 64 KiB from pinned host memory into LDS, writes 64 KiB + 24 KiB back
//                      to pinned host memory, stores the flag; host spins
// Build: hipcc --offload-arch=gfx950 -O2 -o call_overhead call_overhead.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s at %d\n", #x, __LINE__); return 1; } } while (0)

__global__ void empty_kernel(int* p) { if (threadIdx.x == 0 && p) p[0] = 0; }

__global__ __launch_bounds__(1024) void flag_kernel(volatile uint32_t* flag, uint32_t seq) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store((uint32_t*)flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(1024) void zc_kernel(const uint4* in, uint32_t nin, uint4* out, uint32_t nout,
                                                  uint32_t* flag, uint32_t seq) {
  __shared__ uint4 x[65536 / 16];
  for (uint32_t i = threadIdx.x; i < nin; i += 1024) x[i] = in[i];
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nout; i += 1024) {
    uint4 v = x[i & (nin - 1)];
    v.x ^= i;
    out[i] = v;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static int spin(volatile uint32_t* f, uint32_t seq, hipStream_t st) {
  for (uint64_t n = 1;; ++n) {
    if (__atomic_load_n((uint32_t*)f, __ATOMIC_ACQUIRE) == seq) return 0;
    if ((n & 4095) == 0) {
      const hipError_t e = hipStreamQuery(st);
      if (e == hipSuccess) return __atomic_load_n((uint32_t*)f, __ATOMIC_ACQUIRE) == seq ? 0 : 1;
      if (e != hipErrorNotReady) return 1;
    }
  }
}

int main() {
  const int N = 2000;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint8_t *h = nullptr, *hc = nullptr, *d = nullptr;
  CK(hipHostMalloc((void**)&h, 1 << 20, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&hc, 1 << 20, hipHostMallocCoherent));
  CK(hipMalloc((void**)&d, 1 << 20));
  memset(h, 1, 1 << 20);
  memset(hc, 1, 1 << 20);
  std::vector<double> t;
  // warm
  for (int i = 0; i < 50; ++i) {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr);
    CK(hipStreamSynchronize(st));
  }
  t.clear();
  for (int i = 0; i < N; ++i) {
    const double a = now_us();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr);
    CK(hipStreamSynchronize(st));
    t.push_back(now_us() - a);
  }
  printf("launch+sync                 %8.1f us\n", median(t));
  t.clear();
  for (int i = 0; i < N; ++i) {
    const double a = now_us();
    CK(hipMemcpyAsync(d, h, 65536, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr);
    CK(hipMemcpyAsync(h + 65536, d + 65536, 90112, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    t.push_back(now_us() - a);
  }
  printf("h2d+launch+d2h+sync         %8.1f us\n", median(t));
  for (int pass = 0; pass < 2; ++pass) {
    uint8_t* hb = pass ? hc : h;
    const char* nm = pass ? "coherent" : "default ";
    volatile uint32_t* flag = (volatile uint32_t*)(hb + (1 << 20) - 64);
    *flag = 0;
    uint32_t seq = 0;
    t.clear();
    for (int i = 0; i < N; ++i) {
      ++seq;
      const double a = now_us();
      hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(1024), 0, st, flag, seq);
      if (spin(flag, seq, st)) { printf("flag never arrived (%s)\n", nm); return 1; }
      t.push_back(now_us() - a);
    }
    CK(hipStreamSynchronize(st));
    printf("launch+poll (%s)        %8.1f us\n", nm, median(t));
    t.clear();
    for (int i = 0; i < N; ++i) {
      ++seq;
      const double a = now_us();
      hipLaunchKernelGGL(zc_kernel, dim3(1), dim3(1024), 0, st, (const uint4*)hb, 4096u, (uint4*)(hb + 65536),
                         (65536u + 24576u) / 16, (uint32_t*)flag, seq);
      if (spin(flag, seq, st)) { printf("flag never arrived (%s)\n", nm); return 1; }
      t.push_back(now_us() - a);
    }
    CK(hipStreamSynchronize(st));
    bool ok = true;
    for (uint32_t i = 0; i < (65536u + 24576u) / 16 && ok; ++i) {
      const uint32_t* o = (const uint32_t*)(hb + 65536) + 4 * i;
      ok = o[0] == (0x01010101u ^ i) && o[1] == 0x01010101u;
    }
    printf("zc 64K in / 88K out+poll (%s) %8.1f us  %s\n", nm, median(t), ok ? "ok" : "WRONG");
    t.clear();
    for (int i = 0; i < N; ++i) {
      ++seq;
      const double a = now_us();
      hipLaunchKernelGGL(zc_kernel, dim3(1), dim3(1024), 0, st, (const uint4*)hb, 4096u, (uint4*)(hb + 65536),
                         (65536u + 24576u) / 16, (uint32_t*)flag, seq);
      CK(hipStreamSynchronize(st));
      t.push_back(now_us() - a);
    }
    printf("zc 64K in / 88K out+sync (%s) %8.1f us\n", nm, median(t));
  }
  // device-side in/out, d2h of the same sizes (the current path's shape)
  t.clear();
  for (int i = 0; i < N; ++i) {
    const double a = now_us();
    CK(hipMemcpyAsync(d, h, 65536, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(zc_kernel, dim3(1), dim3(1024), 0, st, (const uint4*)d, 4096u, (uint4*)(d + 65536),
                       (65536u + 24576u) / 16, (uint32_t*)(d + (1 << 20) - 64), 1u);
    CK(hipMemcpyAsync(h + 65536, d + 65536, 90112, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    t.push_back(now_us() - a);
  }
  printf("h2d+kernel(dev)+d2h+sync    %8.1f us\n", median(t));
  return 0;
}
