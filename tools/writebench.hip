// writebench.hip -- write-only HBM ceiling sweep on MI355X: is there a store
// shape that writes faster than the codec's (grid-stride 16-B stores, 1 KiB
// per wave instruction)? The codec's mix model prices its
// writes at the write-only rate, so a faster write shape would lift it.
// hipcc --offload-arch=gfx950 -O3 tools/writebench.hip -o tools/writebench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

// grid-stride: each iteration a block writes B*U contiguous 16-B elements
template <int U, int B>
__global__ void __launch_bounds__(B) w_gs(uint4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * B * U;
  for (size_t base = (size_t)blockIdx.x * B * U + threadIdx.x; base < n; base += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + (size_t)u * B < n) b[base + (size_t)u * B] = make_uint4((uint32_t)base, u, 1, 2);
  }
}

// block-contiguous: block k owns one contiguous range
template <int U, int B>
__global__ void __launch_bounds__(B) w_blk(uint4* __restrict__ b, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t v0 = per * blockIdx.x, v1 = v0 + per < n ? v0 + per : n;
  for (size_t base = v0 + threadIdx.x; base < v1; base += (size_t)B * U) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + (size_t)u * B < v1) b[base + (size_t)u * B] = make_uint4((uint32_t)base, u, 1, 2);
  }
}

// S streams written side by side (like an encode's e output cells): each
// iteration writes B*U elements into each of S equal-size regions
template <int S, int U, int B>
__global__ void __launch_bounds__(B) w_streams(uint4* __restrict__ b, size_t n) {
  const size_t m = n / S;
  const size_t stride = (size_t)gridDim.x * B * U;
  for (size_t base = (size_t)blockIdx.x * B * U + threadIdx.x; base < m; base += stride) {
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (base + (size_t)u * B < m) b[(size_t)s * m + base + (size_t)u * B] = make_uint4((uint32_t)base, u, s, 2);
  }
}

// the encode's memory pattern without the GF math: R input streams read,
// combined by XOR, W output streams written, each stream its own region
template <int R, int W, int U, int B>
__global__ void __launch_bounds__(B) rw_streams(uint4* __restrict__ b, size_t n) {
  const size_t m = n / (R + W);
  const size_t stride = (size_t)gridDim.x * B * U;
  for (size_t base = (size_t)blockIdx.x * B * U + threadIdx.x; base < m; base += stride) {
    uint4 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (base + (size_t)u * B < m) {
          uint4 t = b[(size_t)r * m + base + (size_t)u * B];
          acc[u].x ^= t.x; acc[u].y ^= t.y; acc[u].z ^= t.z; acc[u].w ^= t.w;
        }
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (base + (size_t)u * B < m) {
          uint4 t = acc[u];
          t.x += w;
          b[(size_t)(R + w) * m + base + (size_t)u * B] = t;
        }
  }
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / reps;
}

#define RUN(NAME, KER, G, B)                                                                         \
  {                                                                                                  \
    float ms = time_it([&] { hipLaunchKernelGGL(KER, dim3(G), dim3(B), 0, 0, buf, n); }, reps);     \
    printf("%-22s G=%5d  %7.3f ms  %7.1f GB/s\n", NAME, G, ms, bytes / ms / 1e6);                   \
    fflush(stdout);                                                                                  \
  }

int main() {
  const size_t bytes = 2ull << 30;  // 2 GiB written per launch
  const size_t n = bytes / 16;
  uint4* buf;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMemset(buf, 0, bytes));
  const int reps = 10;
  // streams side by side at the smallest write front
  for (int g : {128, 256, 512}) {
    RUN("streams1 U=1 B=256", (w_streams<1, 1, 256>), g, 256)
    RUN("streams2 U=1 B=256", (w_streams<2, 1, 256>), g, 256)
    RUN("streams3 U=1 B=256", (w_streams<3, 1, 256>), g, 256)
  }
  // 8 reads + 3 writes (encode) and 8 + 2 (rebuild): GB/s = (R+W) streams' bytes
  printf("-- read/write mix (bytes = all streams)\n");
  for (int g : {256, 512, 1024, 2048}) {
    RUN("r8w3 U=1 B=256", (rw_streams<8, 3, 1, 256>), g, 256)
    RUN("r8w3 U=1 B=512", (rw_streams<8, 3, 1, 512>), g, 512)
    RUN("r8w3 U=2 B=256", (rw_streams<8, 3, 2, 256>), g, 256)
    RUN("r8w3 U=2 B=512", (rw_streams<8, 3, 2, 512>), g, 512)
    RUN("r8w2 U=1 B=512", (rw_streams<8, 2, 1, 512>), g, 512)
    RUN("r8w2 U=2 B=256", (rw_streams<8, 2, 2, 256>), g, 256)
  }
  for (int round = 0; round < 1; ++round) {
    printf("-- round %d (write-only GB/s)\n", round);
    for (int g : {256, 512, 1024, 2048, 4096}) {
      RUN("gs U=1 B=256", (w_gs<1, 256>), g, 256)
      RUN("gs U=4 B=256", (w_gs<4, 256>), g, 256)
      RUN("gs U=8 B=256", (w_gs<8, 256>), g, 256)
      RUN("gs U=2 B=512", (w_gs<2, 512>), g, 512)
      RUN("gs U=4 B=1024", (w_gs<4, 1024>), g, 1024)
      RUN("blk U=4 B=256", (w_blk<4, 256>), g, 256)
      RUN("streams3 U=1 B=512", (w_streams<3, 1, 512>), g, 512)
      RUN("streams3 U=2 B=512", (w_streams<3, 2, 512>), g, 512)
    }
  }
  CHECK(hipFree(buf));
  return 0;
}
