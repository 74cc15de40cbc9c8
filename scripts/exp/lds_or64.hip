// Probe: 64 lanes of one wave OR distinct bits into shared 64-bit LDS words in one
// instruction (the band replay's bitmap insert); prints the words that lost bits.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(unsigned long long* out, int mode) {
  extern __shared__ unsigned long long w[];
  const unsigned lane = threadIdx.x;
  if (lane < 4) w[lane] = 0;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  unsigned id = mode == 0 ? lane : (mode == 1 ? 38 + lane / 2 * 2 + (lane & 1) : lane * 2 % 128);
  atomicOr(&w[(id >> 6) & 3], 1ull << (id & 63));
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < 4) out[lane] = w[lane];
}
int main() {
  unsigned long long* d;
  hipMalloc(&d, 64);
  for (int mode = 0; mode < 3; ++mode) {
    probe<<<1, 64, 64>>>(d, mode);
    unsigned long long h[4];
    hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    unsigned long long e[4] = {0, 0, 0, 0};
    for (unsigned lane = 0; lane < 64; ++lane) {
      unsigned id = mode == 0 ? lane : (mode == 1 ? 38 + lane / 2 * 2 + (lane & 1) : lane * 2 % 128);
      e[(id >> 6) & 3] |= 1ull << (id & 63);
    }
    for (int i = 0; i < 4; ++i)
      printf("mode %d word %d got %016llx expect %016llx %s\n", mode, i, h[i], e[i], h[i] == e[i] ? "ok" : "LOST");
  }
  return 0;
}
