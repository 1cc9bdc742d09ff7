// Microbenchmark: cost of claiming workgroup tickets through global atomic counters, 16384
// workgroups of 512 threads: one counter; 8 counters (b % 8) at a given stride; per-XCD counters.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(512) void k_claim(unsigned* counter, unsigned* sink, int stride) {
  __shared__ unsigned t;
  if (threadIdx.x == 0) {
    unsigned* c = counter;
    if (MODE == 1) c += (blockIdx.x % 8) * stride;
    if (MODE == 2) c += __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) % 8 * stride;  // XCC_ID
    if (MODE != 3) t = atomicAdd(c, 1u); else t = blockIdx.x;
  }
  __syncthreads();
  if (threadIdx.x == 0 && t == 0xffffffffu) sink[0] = 1;
}

int main() {
  unsigned *c, *sink;
  (void)hipMalloc(&c, 1 << 20);
  (void)hipMalloc(&sink, 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int n = 16384;
  struct { const char* name; int mode, stride; } cases[] = {
      {"one counter", 0, 0},        {"8 counters, 256 B apart", 1, 64},  {"8 counters, 4 KiB apart", 1, 1024},
      {"8 counters, 64 KiB apart", 1, 16384}, {"per-XCD counters, 4 KiB apart", 2, 1024}, {"no atomic", 3, 0}};
  for (int rep = 0; rep < 2; ++rep)
    for (auto& cs : cases) {
      (void)hipMemset(c, 0, 1 << 20);
      (void)hipEventRecord(a);
      if (cs.mode == 0) k_claim<0><<<n, 512>>>(c, sink, cs.stride);
      if (cs.mode == 1) k_claim<1><<<n, 512>>>(c, sink, cs.stride);
      if (cs.mode == 2) k_claim<2><<<n, 512>>>(c, sink, cs.stride);
      if (cs.mode == 3) k_claim<3><<<n, 512>>>(c, sink, cs.stride);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      printf("%-32s %8.1f us\n", cs.name, ms * 1e3);
    }
  return 0;
}
