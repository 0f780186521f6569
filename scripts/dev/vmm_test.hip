// Diagnostics: can one physical allocation (a shared disk pool) be mapped
// behind two different front pools so `pool + id * 2048` stays one linear
// address range per front?  hipMemCreate / hipMemMap / hipMemSetAccess.
// Build: hipcc --offload-arch=gfx950 -O2 -o vmm_test vmm_test.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);          \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void fill(uint32_t* p, uint64_t n, uint32_t tag) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i ^ tag;
}
__global__ void check(const uint32_t* p, uint64_t n, uint32_t tag, uint32_t* bad) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (p[i] != ((uint32_t)i ^ tag)) atomicAdd(bad, 1u);
}

int main(int argc, char** argv) {
  int dev = 0;
  CK(hipSetDevice(dev));
  const bool host_part = argc > 1;
  int vmm = 0;
  CK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev));
  printf("VMM supported attr: %d\n", vmm);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0, rgran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  CK(hipMemGetAllocationGranularity(&rgran, &prop, hipMemAllocationGranularityRecommended));
  printf("granularity min %zu recommended %zu\n", gran, rgran);
  const size_t prim = 8 * gran, disk = 64 * gran;   // front primary, shared disk
  hipMemGenericAllocationHandle_t hp1, hp2, hd;
  CK(hipMemCreate(&hp1, prim, &prop, 0));
  CK(hipMemCreate(&hp2, prim, &prop, 0));
  CK(hipMemCreate(&hd, disk, &prop, 0));
  void *va1 = nullptr, *va2 = nullptr;
  CK(hipMemAddressReserve(&va1, prim + disk, 0, nullptr, 0));
  CK(hipMemAddressReserve(&va2, prim + disk, 0, nullptr, 0));
  CK(hipMemMap(va1, prim, 0, hp1, 0));
  CK(hipMemMap((char*)va1 + prim, disk, 0, hd, 0));
  CK(hipMemMap(va2, prim, 0, hp2, 0));
  CK(hipMemMap((char*)va2 + prim, disk, 0, hd, 0));
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va1, prim + disk, &acc, 1));
  CK(hipMemSetAccess(va2, prim + disk, &acc, 1));
  uint32_t* bad = nullptr;
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  const uint64_t n = (prim + disk) / 4;
  // front 1 writes its whole range; front 2 must see front 1's disk part
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, (uint32_t*)va1, n, 0x1234u);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, 0, (const uint32_t*)va1, n, 0x1234u, bad);
  uint32_t h = 0;
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
  printf("front 1 readback mismatches: %u\n", h);
  CK(hipMemset(bad, 0, 4));
  // front 2's disk part == front 1's disk part (same physical pages)
  hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, 0, (const uint32_t*)((char*)va2 + prim), disk / 4, 0u, bad);
  CK(hipDeviceSynchronize());
  // compare against the expected tag pattern of front 1 shifted by prim / 4
  uint32_t* host = (uint32_t*)malloc(disk);
  CK(hipMemcpy(host, (char*)va2 + prim, disk, hipMemcpyDeviceToHost));
  uint64_t mism = 0;
  for (uint64_t i = 0; i < disk / 4; ++i)
    if (host[i] != ((uint32_t)(i + prim / 4) ^ 0x1234u)) ++mism;
  printf("front 2 sees front 1's disk writes: mismatches %llu of %llu\n", (unsigned long long)mism,
         (unsigned long long)(disk / 4));
  // front 2's primary must be untouched by front 1 (fill it, check front 1's primary unchanged)
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, (uint32_t*)va2, prim / 4, 0x9999u);
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, 0, (const uint32_t*)va1, prim / 4, 0x1234u, bad);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
  printf("front 1 primary after front 2 fill: mismatches %u\n", h);
  // hipMemcpy / hipMemset on the mapped range
  CK(hipMemsetAsync((char*)va2 + prim - 4096, 0, 8192, 0));
  CK(hipDeviceSynchronize());
  CK(hipMemUnmap(va1, prim));
  CK(hipMemUnmap((char*)va1 + prim, disk));
  CK(hipMemUnmap(va2, prim));
  CK(hipMemUnmap((char*)va2 + prim, disk));
  CK(hipMemAddressFree(va1, prim + disk));
  CK(hipMemAddressFree(va2, prim + disk));
  CK(hipMemRelease(hp1));
  CK(hipMemRelease(hp2));
  CK(hipMemRelease(hd));
  printf("VMM OK\n");
  // a host-memory physical allocation mapped into the device VA (a spill tier)
  if (host_part) {
    hipMemAllocationProp hp = {};
    hp.type = hipMemAllocationTypePinned;
    hp.location.type = hipMemLocationTypeHost;
    hp.location.id = 0;
    size_t hg = 0;
    hipError_t e = hipMemGetAllocationGranularity(&hg, &hp, hipMemAllocationGranularityMinimum);
    printf("host granularity: %s %zu\n", hipGetErrorString(e), hg);
    hipMemGenericAllocationHandle_t hh;
    e = hipMemCreate(&hh, 64 * (hg ? hg : gran), &hp, 0);
    printf("host hipMemCreate: %s\n", hipGetErrorString(e));
    if (e == hipSuccess) {
      void* hv = nullptr;
      const size_t hs = 64 * (hg ? hg : gran);
      CK(hipMemAddressReserve(&hv, hs, 0, nullptr, 0));
      e = hipMemMap(hv, hs, 0, hh, 0);
      printf("host hipMemMap: %s\n", hipGetErrorString(e));
      if (e == hipSuccess) {
        hipMemAccessDesc da = {};
        da.location.type = hipMemLocationTypeDevice;
        da.location.id = dev;
        da.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess(hv, hs, &da, 1);
        printf("host hipMemSetAccess(device): %s\n", hipGetErrorString(e));
        if (e == hipSuccess) {
          CK(hipMemset(bad, 0, 4));
          hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, (uint32_t*)hv, hs / 4, 0x4242u);
          hipLaunchKernelGGL(check, dim3(256), dim3(256), 0, 0, (const uint32_t*)hv, hs / 4, 0x4242u, bad);
          CK(hipDeviceSynchronize());
          CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
          printf("host-backed range via the device: mismatches %u\n", h);
        }
        (void)hipMemUnmap(hv, hs);
      }
      (void)hipMemAddressFree(hv, hs);
      (void)hipMemRelease(hh);
    }
  }
  return 0;
}
