// Memory ceiling of the headline kernel's access pattern (diagnostics): 4096
// waves, each streams one 64 KiB chunk in 2 KiB pieces (32 B per lane) and
// writes 2050-byte records (a 2-byte header + the 2 KiB body: an EXTRACT),
// with the next D pieces' loads in flight.  Variants: prefetch depth D,
// record stride 2050 (unaligned bodies) or 2048 (aligned), waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o copy_pattern copy_pattern.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4_u;

template <int D, int STRIDE, int WORK>
__global__ __launch_bounds__(256) void copy_kernel(const uint8_t* in, uint8_t* out, uint32_t n) {
  const uint32_t wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t chunk = blockIdx.x * 4 + wv;
  if (chunk >= n) return;
  const uint8_t* x = in + (uint64_t)chunk * 65536;
  uint8_t* o = out + (uint64_t)chunk * (32 * STRIDE + 16);
  u32x4 buf[D + 1][2];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    buf[k][0] = *(const u32x4*)(x + 2048 * k + 32 * l);
    buf[k][1] = *(const u32x4*)(x + 2048 * k + 32 * l + 16);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int pc = 0; pc < 32; ++pc) {
    if (pc + D < 32) {
      buf[(pc + D) % (D + 1)][0] = *(const u32x4*)(x + 2048 * (pc + D) + 32 * l);
      buf[(pc + D) % (D + 1)][1] = *(const u32x4*)(x + 2048 * (pc + D) + 32 * l + 16);
    }
    const u32x4 a = buf[pc % (D + 1)][0], b = buf[pc % (D + 1)][1];
    // stand-in compute: WORK dependent VALU ops per piece
#pragma unroll
    for (int w = 0; w < WORK; ++w) acc = acc * 3u + (a[w & 3] ^ b[(w >> 2) & 3]);
    uint8_t* dst = o + (uint64_t)pc * STRIDE;
    if (l < 2) dst[l] = (uint8_t)(0xF1 + l + (acc & 1));
    *(u32x4_u*)(dst + 2 + 32 * l) = a;
    *(u32x4_u*)(dst + 2 + 32 * l + 16) = b;
  }
}

template <int D, int STRIDE, int WORK>
static void run(const char* name, const uint8_t* in, uint8_t* out, uint32_t n) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((copy_kernel<D, STRIDE, WORK>), dim3(n / 4), dim3(256), 0, 0, in, out, n);
  hipEventRecord(e0, 0);
  const int R = 20;
  for (int i = 0; i < R; ++i) hipLaunchKernelGGL((copy_kernel<D, STRIDE, WORK>), dim3(n / 4), dim3(256), 0, 0, in, out, n);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / R;
  const double bytes = (double)n * 65536 * 2;
  printf("%-34s %7.1f us per launch  %6.2f TB/s (in + out)\n", name, us, bytes / us / 1e6);
}

int main() {
  const uint32_t n = 4096;
  uint8_t *in = nullptr, *out = nullptr;
  if (hipMalloc(&in, (size_t)n * 65536) != hipSuccess || hipMalloc(&out, (size_t)n * (32 * 2050 + 16)) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(in, 7, (size_t)n * 65536);
  run<1, 2050, 0>("D=1 stride 2050 work 0", in, out, n);
  run<2, 2050, 0>("D=2 stride 2050 work 0", in, out, n);
  run<4, 2050, 0>("D=4 stride 2050 work 0", in, out, n);
  run<1, 2048, 0>("D=1 stride 2048 work 0", in, out, n);
  run<4, 2048, 0>("D=4 stride 2048 work 0", in, out, n);
  run<1, 2050, 64>("D=1 stride 2050 work 64", in, out, n);
  run<2, 2050, 64>("D=2 stride 2050 work 64", in, out, n);
  run<4, 2050, 64>("D=4 stride 2050 work 64", in, out, n);
  run<1, 2050, 200>("D=1 stride 2050 work 200", in, out, n);
  run<2, 2050, 200>("D=2 stride 2050 work 200", in, out, n);
  run<4, 2050, 200>("D=4 stride 2050 work 200", in, out, n);
  hipFree(in);
  hipFree(out);
  return 0;
}
