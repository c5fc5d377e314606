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

// S streams, each written by its own third of the grid (block b -> stream
// b % S): same fronts, each 1/S as wide as in w_streams
template <int S, int B>
__global__ void __launch_bounds__(B) w_split(uint4* __restrict__ b, size_t n) {
  const size_t m = n / S;
  const int s = blockIdx.x % S, nb = gridDim.x / S;
  const size_t stride = (size_t)nb * B;
  for (size_t base = (size_t)(blockIdx.x / S) * B + threadIdx.x; base < m; base += stride)
    b[(size_t)s * m + base] = make_uint4((uint32_t)base, s, 1, 2);
}

// S streams one after another (one front at a time), same grid
template <int S, int B>
__global__ void __launch_bounds__(B) w_seq(uint4* __restrict__ b, size_t n) {
  const size_t m = n / S;
  const size_t stride = (size_t)gridDim.x * B;
  for (int s = 0; s < S; ++s)
    for (size_t base = (size_t)blockIdx.x * B + threadIdx.x; base < m; base += stride)
      b[(size_t)s * m + base] = make_uint4((uint32_t)base, s, 1, 2);
}

// R reads + W writes per position like rw_streams, but each half of a
// 512-thread block sweeps its own half of the regions: two fronts per
// stream, each G*256*16 B wide (HALVES=1: one front G*512*16 B wide)
template <int R, int W, int HALVES>
__global__ void __launch_bounds__(512) rw_halves(uint4* __restrict__ b, size_t n) {
  const size_t m = n / (R + W);
  const int h = HALVES ? threadIdx.x / 256 : 0;
  const int t = HALVES ? threadIdx.x % 256 : threadIdx.x;
  const int BW = HALVES ? 256 : 512;
  const size_t lo = HALVES ? (h ? m / 2 : 0) : 0, hi = HALVES ? (h ? m : m / 2) : m;
  const size_t stride = (size_t)gridDim.x * BW;
  for (size_t base = lo + (size_t)blockIdx.x * BW + t; base < hi; base += stride) {
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      uint4 v = b[(size_t)r * m + base];
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint4 v = acc;
      v.x += w;
      b[(size_t)(R + w) * m + base] = v;
    }
  }
}

// split roles: waves 0-3 of a 512-thread block only load (R streams, U
// positions per iteration) and XOR into an LDS ring; waves 4-7 only store
// the W outputs of the previous iteration (one wave per SIMD writing)
template <int R, int W, int U>
__global__ void __launch_bounds__(512) rw_roles(uint4* __restrict__ b, size_t n) {
  __shared__ uint4 ring[2][U][256];
  const size_t m = n / (R + W);
  const bool loader = threadIdx.x < 256;
  const int t = threadIdx.x & 255;
  const size_t stride = (size_t)gridDim.x * 256 * U;
  const size_t first = (size_t)blockIdx.x * 256 * U;
  const long iters = first < m ? (long)((m - first + stride - 1) / stride) : 0;
  for (long it = 0; it <= iters; ++it) {
    if (loader && it < iters) {
      const size_t base = first + (size_t)it * stride + t;
      uint4 acc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (base + (size_t)u * 256 < m) {
            uint4 v = b[(size_t)r * m + base + (size_t)u * 256];
            acc[u].x ^= v.x; acc[u].y ^= v.y; acc[u].z ^= v.z; acc[u].w ^= v.w;
          }
#pragma unroll
      for (int u = 0; u < U; ++u) ring[it & 1][u][t] = acc[u];
    }
    if (!loader && it > 0) {
      const size_t base = first + (size_t)(it - 1) * stride + t;
#pragma unroll
      for (int w = 0; w < W; ++w)
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (base + (size_t)u * 256 < m) {
            uint4 v = ring[(it - 1) & 1][u][t];
            v.x += w;
            b[(size_t)(R + w) * m + base + (size_t)u * 256] = v;
          }
    }
    __syncthreads();
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
  for (int round = 0; round < 3; ++round) {
    printf("-- round %d: split roles (4 load waves + 4 store waves per 512-thread block) vs one front\n", round);
    RUN("r8w3 one front G=256", (rw_halves<8, 3, 0>), 256, 512)
    RUN("r8w3 roles U=1 G=256", (rw_roles<8, 3, 1>), 256, 512)
    RUN("r8w3 roles U=2 G=256", (rw_roles<8, 3, 2>), 256, 512)
    RUN("r8w3 roles U=4 G=256", (rw_roles<8, 3, 4>), 256, 512)
    RUN("r8w3 roles U=2 G=512", (rw_roles<8, 3, 2>), 512, 512)
    RUN("r8w2 one front G=256", (rw_halves<8, 2, 0>), 256, 512)
    RUN("r8w2 roles U=2 G=256", (rw_roles<8, 2, 2>), 256, 512)
  }
  CHECK(hipFree(buf));
  return 0;
}
