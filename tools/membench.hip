// membench.hip -- HBM ceilings on MI355X for streaming shapes relevant to the
// codec: copy / read-only / write-only with grid, block, unroll and access
// layout sweeps. hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// grid-stride copy, U independent elements per thread per iteration
template <int U, int B>
__global__ void __launch_bounds__(B) copy_gs(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * B * U;
  for (size_t base = (size_t)blockIdx.x * B * U + threadIdx.x; base < n; base += stride) {
    uint4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = (base + (size_t)u * B < n) ? a[base + (size_t)u * B] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + (size_t)u * B < n) b[base + (size_t)u * B] = t[u];
  }
}

// block-contiguous copy: block k owns [k*per, (k+1)*per)
template <int U, int B>
__global__ void __launch_bounds__(B) copy_blk(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t v0 = per * blockIdx.x, v1 = v0 + per < n ? v0 + per : n;
  for (size_t base = v0 + threadIdx.x; base < v1; base += (size_t)B * U) {
    uint4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = (base + (size_t)u * B < v1) ? a[base + (size_t)u * B] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + (size_t)u * B < v1) b[base + (size_t)u * B] = t[u];
  }
}

template <int U, int B>
__global__ void __launch_bounds__(B) read_gs(const uint4* __restrict__ a, uint4* __restrict__ sink, size_t n) {
  const size_t stride = (size_t)gridDim.x * B * U;
  uint32_t acc = 0;
  for (size_t base = (size_t)blockIdx.x * B * U + threadIdx.x; base < n; base += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + (size_t)u * B < n) {
        uint4 t = a[base + (size_t)u * B];
        acc ^= t.x ^ t.y ^ t.z ^ t.w;
      }
    }
  }
  if (acc == 0x9E3779B9u) sink[0] = make_uint4(acc, 0, 0, 0);
}

template <int U, int B>
__global__ void __launch_bounds__(B) write_gs(uint4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * B * U;
  for (size_t base = (size_t)blockIdx.x * B * U + threadIdx.x; base < n; base += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + (size_t)u * B < n) b[base + (size_t)u * B] = make_uint4((uint32_t)base, u, 1, 2);
  }
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
// copy with explicit cache-policy bits on the store / load (inline asm)
#define STORE_VARIANT(NAME, MODS)                                                          \
  __global__ void __launch_bounds__(256) NAME(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) { \
    const size_t stride = (size_t)gridDim.x * 256;                                         \
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {          \
      v4u t = reinterpret_cast<const v4u*>(a)[i];                                          \
      asm volatile("global_store_dwordx4 %0, %1, off " MODS :: "v"(b + i), "v"(t) : "memory"); \
    }                                                                                      \
  }
STORE_VARIANT(st_plain, "")
STORE_VARIANT(st_sc0, "sc0")
STORE_VARIANT(st_sc1, "sc1")
STORE_VARIANT(st_nt, "nt")
STORE_VARIANT(st_sc0sc1, "sc0 sc1")
STORE_VARIANT(st_sc1nt, "sc1 nt")
STORE_VARIANT(st_sc0nt, "sc0 nt")
STORE_VARIANT(st_all, "sc0 sc1 nt")
#define LOAD_VARIANT(NAME, MODS)                                                           \
  __global__ void __launch_bounds__(256) NAME(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) { \
    const size_t stride = (size_t)gridDim.x * 256;                                         \
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {          \
      v4u t;                                                                               \
      asm volatile("global_load_dwordx4 %0, %1, off " MODS "\n\ts_waitcnt vmcnt(0)" : "=v"(t) : "v"(a + i) : "memory"); \
      reinterpret_cast<v4u*>(b)[i] = t;                                                    \
    }                                                                                      \
  }
LOAD_VARIANT(ld_nt, "nt")
LOAD_VARIANT(ld_sc1, "sc1")
LOAD_VARIANT(ld_sc0sc1, "sc0 sc1")

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
  return ms / reps;
}

#define COPY(KER, U, B, G)                                                                              \
  {                                                                                                     \
    float ms = time_it([&] { hipLaunchKernelGGL((KER<U, B>), dim3(G), dim3(B), 0, 0, a, b, n); }, reps); \
    printf("%-9s U=%d B=%4d G=%5d  %7.3f ms  %7.1f GB/s\n", #KER, U, B, G, ms, 2.0 * bytes / ms / 1e6); \
  }

int main() {
  const size_t bytes = 2ull << 30;  // 2 GiB each way
  const size_t n = bytes / 16;
  uint4 *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 0x5a, bytes));
  CHECK(hipMemset(b, 0, bytes));
  const int reps = 10;
  for (int round = 0; round < 2; ++round) {
    printf("-- round %d (bytes = read + write)\n", round);
    COPY(copy_gs, 1, 256, 1024)
    COPY(copy_gs, 4, 256, 512)
#define V(K) { for (int g : {1024, 2048}) { float ms = time_it([&] { hipLaunchKernelGGL(K, dim3(g), dim3(256), 0, 0, a, b, n); }, reps); \
    printf("%-12s G=%5d %7.3f ms  %7.1f GB/s\n", #K, g, ms, 2.0 * bytes / ms / 1e6); } }
    V(st_plain) V(st_sc0) V(st_sc1) V(st_nt) V(st_sc0sc1) V(st_sc1nt) V(st_sc0nt) V(st_all)
    V(ld_nt) V(ld_sc1) V(ld_sc0sc1)
    for (int g : {1024, 2048}) {
      float ms = time_it([&] { hipLaunchKernelGGL((read_gs<4, 256>), dim3(g), dim3(256), 0, 0, a, b, n); }, reps);
      printf("read-only U=4 B=256 G=%5d  %7.3f ms  %7.1f GB/s\n", g, ms, bytes / ms / 1e6);
      ms = time_it([&] { hipLaunchKernelGGL((write_gs<4, 256>), dim3(g), dim3(256), 0, 0, b, n); }, reps);
      printf("write-only U=4 B=256 G=%5d %7.3f ms  %7.1f GB/s\n", g, ms, bytes / ms / 1e6);
    }
  }
  return 0;
}
