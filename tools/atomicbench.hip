// Claim-counter probe: 256 blocks (one per CU), lane 0 of each issues N
// returning atomicAdds on shared counters (1 counter, or one per XCD), each
// waiting for its result (a dependent chain, like a loader claiming its next
// batch). Reports claims per second over the grid and the mean latency.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/atomicbench tools/atomicbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void claim(unsigned* ctr, int n, int spread, unsigned long long* sink) {
  if (threadIdx.x != 0) return;
  unsigned* c = ctr + (spread ? (blockIdx.x & 7) * 64 : 0);
  unsigned acc = 0;
  for (int i = 0; i < n; ++i) acc += atomicAdd(c, 4u + (acc & 0));
  sink[blockIdx.x] = acc;
}

int main() {
  unsigned* ctr;
  unsigned long long* sink;
  hipMalloc(&ctr, 8 * 64 * sizeof(unsigned));
  hipMalloc(&sink, 4096 * sizeof(unsigned long long));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int spread = 0; spread < 2; ++spread)
    for (int blocks : {64, 256}) {
      const int n = 2000;
      hipMemset(ctr, 0, 8 * 64 * sizeof(unsigned));
      claim<<<blocks, 64>>>(ctr, 10, spread, sink);
      hipEventRecord(a);
      claim<<<blocks, 64>>>(ctr, n, spread, sink);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double claims = double(blocks) * n;
      printf("counters %d blocks %4d: %.1f M claims/s, %.2f us per dependent claim\n", spread ? 8 : 1, blocks,
             claims / (ms * 1e-3) / 1e6, ms * 1e3 / n);
    }
  return 0;
}
