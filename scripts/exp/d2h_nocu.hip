// Probe: does a D2H copy into pinned host memory overlap a kernel that holds every CU?
// (round 3: hipMemcpyAsync D2H ran as blit kernels that waited for the engine kernels'
// CU slots).  Times a 1 GB D2H alone and beside a persistent busy kernel, with the copy
// kind DeviceToHost and DeviceToDeviceNoCU (SDMA, no compute units), and checks the bytes.
// build: hipcc -O2 --offload-arch=gfx950 -o scripts/exp/d2h_nocu scripts/exp/d2h_nocu.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void busy(unsigned long long ticks, unsigned int* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned int x = threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
  if (x == 0xFFFFFFFFu) sink[0] = x;
}

__global__ void fill(unsigned int* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (unsigned int)(i * 2654435761u);
}

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 4;
  unsigned int *d = nullptr, *h = nullptr, *sink = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipHostMalloc((void**)&h, bytes, hipHostMallocDefault));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, d, n);
  CK(hipDeviceSynchronize());
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  hipStream_t sk, sc;
  CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  hipEvent_t a, b, c, k0, k1;
  for (hipEvent_t* e : {&a, &b, &c, &k0, &k1}) CK(hipEventCreate(e));
  const hipMemcpyKind kinds[2] = {hipMemcpyDeviceToHost, hipMemcpyDeviceToDeviceNoCU};
  const char* names[2] = {"DeviceToHost", "DeviceToDeviceNoCU"};
  for (int ki = 0; ki < 2; ++ki) {
    for (int rep = 0; rep < 2; ++rep) {
      std::memset(h, 0, bytes);
      // alone
      CK(hipEventRecord(a, sc));
      CK(hipMemcpyAsync(h, d, bytes, kinds[ki], sc));
      CK(hipEventRecord(b, sc));
      CK(hipStreamSynchronize(sc));
      float alone = 0;
      CK(hipEventElapsedTime(&alone, a, b));
      size_t bad = 0;
      for (size_t i = 0; i < n; i += 4097) bad += h[i] != (unsigned int)(i * 2654435761u);
      // beside a kernel holding every CU for ~100 ms (8 waves per SIMD)
      std::memset(h, 0, bytes);
      const int grid = pr.multiProcessorCount * 32;
      CK(hipEventRecord(k0, sk));
      hipLaunchKernelGGL(busy, dim3(grid), dim3(64), 0, sk, 10000000ull /* 100 ms at 100 MHz */, sink);
      CK(hipEventRecord(k1, sk));
      CK(hipEventRecord(a, sc));
      CK(hipMemcpyAsync(h, d, bytes, kinds[ki], sc));
      CK(hipEventRecord(c, sc));
      CK(hipDeviceSynchronize());
      float kern = 0, copy = 0, kstart_to_copyend = 0;
      CK(hipEventElapsedTime(&kern, k0, k1));
      CK(hipEventElapsedTime(&copy, a, c));
      CK(hipEventElapsedTime(&kstart_to_copyend, k0, c));
      for (size_t i = 0; i < n; i += 4097) bad += h[i] != (unsigned int)(i * 2654435761u);
      std::printf("{\"kind\": \"%s\", \"rep\": %d, \"alone_ms\": %.2f, \"alone_GBs\": %.1f, "
                  "\"kernel_ms\": %.2f, \"copy_beside_kernel_ms\": %.2f, "
                  "\"kernel_start_to_copy_end_ms\": %.2f, \"bad\": %zu}\n",
                  names[ki], rep, alone, bytes / alone / 1e6, kern, copy, kstart_to_copyend, bad);
    }
  }
  return 0;
}
