// codec_kernels.hip -- host-side launchers of the codec kernels (the kernels
// themselves: codec_device.h, instantiated by codec_sets_*.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "codec_kernels.h"

namespace redset_hip {

const KernelSet* kernel_sets_a(int nin);
const KernelSet* kernel_sets_b(int nin);
const KernelSet* kernel_sets_c(int nin);
const KernelSet* kernel_sets_d(int nin);
const KernelSet* kernel_sets_e(int nin);
const KernelSet* kernel_sets_f(int nin);
const KernelSet* kernel_sets_g(int nin);

namespace {

const KernelSet& kernel_set(int nin) {
  static const KernelSet* table[kMaxIn] = {};
  if (!table[nin - 1]) {
    const KernelSet* s = nullptr;
    for (auto fn : {kernel_sets_a, kernel_sets_b, kernel_sets_c, kernel_sets_d, kernel_sets_e, kernel_sets_f,
                    kernel_sets_g})
      if (!s) s = fn(nin);
    table[nin - 1] = s;
  }
  return *table[nin - 1];
}

// jobs one launch covers (the last launch may get fewer)
template <class Launch>
int jobs_per_launch(const Launch& L) {
  if (L.sequential == kJobsStreamed || L.sequential == kJobsClaimed) return L.group > 0 ? L.group : L.njobs;
  return L.sequential == kJobsInLaunches ? std::max(1, L.group) : L.njobs;
}

// The kernels' fault words, two per device: [0] capped loader-ring spins
// (codec_device.h ring_sweep; a fallback ran, outputs right), [1] capped hang
// waits (no fallback, outputs wrong; kRingHangCap). The kernels get the
// address in GfLaunch / XorLaunch::fault. Launches come from several threads
// (the pipeline's compute thread, per-rank backends, callers), so the
// per-device address cache is atomic; a racing first lookup resolves the
// same address twice, which is harmless.
__device__ unsigned g_ring_fault[2];

unsigned* ring_fault_word() {
  static std::atomic<unsigned*> addr[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  unsigned* a = addr[dev].load(std::memory_order_acquire);
  if (!a) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_ring_fault)) == hipSuccess) {
      a = static_cast<unsigned*>(p);
      addr[dev].store(a, std::memory_order_release);
    }
  }
  return a;
}
// Test builds (REDSET_HIP_TEST_KNOBS, the twin library of the test suite):
// the loader ring's poll cap and a claimer delay from the environment
// (REDSET_HIP_TEST_SPIN_CAP, REDSET_HIP_TEST_CLAIM_DELAY), so the suite can
// drive the ring's fallbacks and the claimed kernel's claim/record window on
// every launch. Read at every launch, so one test process can change them.
// The product library reads no environment here.
unsigned test_env(const char* name, unsigned dflt) {
#if REDSET_HIP_TEST_KNOBS
  const char* s = std::getenv(name);
  const long v = s ? std::atol(s) : 0;
  return v > 0 ? static_cast<unsigned>(v) : dflt;
#else
  (void) name;
  return dflt;
#endif
}

unsigned spin_cap() { return test_env("REDSET_HIP_TEST_SPIN_CAP", 1u << 24); }
unsigned claim_delay() { return test_env("REDSET_HIP_TEST_CLAIM_DELAY", 0); }

// Test builds: the hang cap (REDSET_HIP_TEST_HANG_CAP polls) and the
// loader's table delay (REDSET_HIP_TEST_TABLE_DELAY), so the suite can make
// the hang waits fire (codec_device.h kRingHangCap).
unsigned hang_cap() { return test_env("REDSET_HIP_TEST_HANG_CAP", 1u << 26); }
unsigned table_delay() { return test_env("REDSET_HIP_TEST_TABLE_DELAY", 0); }

template <class Launch>
void set_launch_knobs(Launch& one) {
  one.fault = ring_fault_word();
  one.spin_cap = spin_cap();
  one.claim_delay = claim_delay();
  one.hang_cap = hang_cap();
  one.table_delay = table_delay();
}
}  // namespace

int test_knobs() { return REDSET_HIP_TEST_KNOBS ? 1 : 0; }

int read_ring_faults(unsigned* count, int clear) {
  unsigned v = 0;
  hipError_t e = hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ring_fault), sizeof(v), 0, hipMemcpyDeviceToHost);
  if (e == hipSuccess && clear && v) {
    const unsigned zero = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_ring_fault), &zero, sizeof(zero), 0, hipMemcpyHostToDevice);
  }
  if (count) *count = v;
  return e;
}

// a non-blocking stream of the library's own per device, for reads of the
// hang word that must not wait for unrelated work (created once, kept)
static hipStream_t own_stream() {
  static std::atomic<hipStream_t> streams[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  hipStream_t s = streams[dev].load(std::memory_order_acquire);
  if (!s) {
    hipStream_t made = nullptr;
    if (hipStreamCreateWithFlags(&made, hipStreamNonBlocking) != hipSuccess) return nullptr;
    if (streams[dev].compare_exchange_strong(s, made, std::memory_order_acq_rel)) s = made;
    else (void) hipStreamDestroy(made);  // another thread made one first
  }
  return s;
}

int read_hang_faults(void* stream, unsigned* count, int clear) {
  const hipStream_t s = stream ? static_cast<hipStream_t>(stream) : own_stream();
  if (!s) return hipErrorInvalidResourceHandle;
  unsigned v = 0;
  const size_t off = sizeof(unsigned);
  hipError_t e = hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_ring_fault), sizeof(v), off, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess && clear && v) {
    const unsigned zero = 0;
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ring_fault), &zero, sizeof(zero), off, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
  }
  if (count) *count = v;
  return e;
}


int device_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
    cus = prop.multiProcessorCount;
  }
  return cus;
}

int gf_blocks_per_cu(int nin) {
  if (nin < 1 || nin > kMaxIn) return 1;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(kernel_set(nin).gf[kMaxOut - 1][1]), kBlock,
                                                   0) != hipSuccess ||
      n < 1)
    n = 1;
  return n;
}

// L.sequential (codec_kernels.h): kJobsInLaunches = the jobs go one after
// another, one launch each on the whole grid (or L.group per launch), so
// only one stripe's ~11 cell streams are in flight instead of every
// stripe's ~120: same bytes, fewer concurrent DRAM streams (A/B in profiles/r01_sequential_jobs.txt);
// kJobsInKernel = one launch on the whole grid whose blocks loop over the
// jobs (codec_device.h); 0 = one launch, jobs side by side, blocks_per_job
// blocks each.
int launch_gf(const GfLaunch& L, void* stream) {
  if (L.nin < 1 || L.nin > kMaxIn || L.nout < 1 || L.nout > kMaxOut) return hipErrorInvalidValue;
  if (L.njobs == 0 || L.nbytes == 0) return hipSuccess;
  const GfKernel k = kernel_set(L.nin).gf[L.nout - 1][L.accumulate ? 1 : 0];
  const int per = jobs_per_launch(L);
  for (int j = 0; j < L.njobs; j += per) {
    GfLaunch one = L;
    one.job0 = j;
    set_launch_knobs(one);
    if (L.sequential == kJobsStreamed || L.sequential == kJobsClaimed) one.njobs = std::min(per, L.njobs - j);
    if (L.sequential == kJobsClaimed && L.claim) {
      // the claim queues start at zero for every launch, whatever an earlier
      // launch left (aborted, replayed from a graph, another stream's)
      const hipError_t e = hipMemsetAsync(L.claim, 0, kClaimWords * sizeof(unsigned), static_cast<hipStream_t>(stream));
      if (e != hipSuccess) return e;
    }
    const int n = (L.sequential == kJobsInKernel || L.sequential == kJobsStreamed || L.sequential == kJobsClaimed)
                      ? 1
                      : std::min(per, L.njobs - j);
    const dim3 grid(static_cast<unsigned>(n * L.blocks_per_job));
    hipLaunchKernelGGL(k, grid, dim3(kBlock), 0, static_cast<hipStream_t>(stream), one);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

int launch_gf_single(const GfLaunch& L, const GfJob& J, void* stream) {
  if (L.nin < 1 || L.nin > kMaxIn || L.nout < 1 || L.nout > kMaxOut) return hipErrorInvalidValue;
  if (L.nbytes == 0) return hipSuccess;
  GfLaunch one = L;
  set_launch_knobs(one);
  hipLaunchKernelGGL(kernel_set(L.nin).gf_arg[L.nout - 1][L.accumulate ? 1 : 0], dim3(static_cast<unsigned>(L.blocks_per_job)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), one, J);
  return hipGetLastError();
}

int launch_xor_single(const XorLaunch& L, const XorJob& J, void* stream) {
  if (L.nin < 1 || L.nin > kMaxIn) return hipErrorInvalidValue;
  if (L.nbytes == 0) return hipSuccess;
  XorLaunch one = L;
  set_launch_knobs(one);
  hipLaunchKernelGGL(kernel_set(L.nin).xr_arg[L.accumulate ? 1 : 0], dim3(static_cast<unsigned>(L.blocks_per_job)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), one, J);
  return hipGetLastError();
}

int launch_xor(const XorLaunch& L, void* stream) {
  if (L.nin < 1 || L.nin > kMaxIn) return hipErrorInvalidValue;
  if (L.njobs == 0 || L.nbytes == 0) return hipSuccess;
  const XorKernel k = kernel_set(L.nin).xr[L.accumulate ? 1 : 0];
  const int per = jobs_per_launch(L);
  for (int j = 0; j < L.njobs; j += per) {
    XorLaunch one = L;
    one.job0 = j;
    set_launch_knobs(one);
    if (L.sequential == kJobsClaimed && L.claim) {
      const hipError_t e = hipMemsetAsync(L.claim, 0, kClaimWords * sizeof(unsigned), static_cast<hipStream_t>(stream));
      if (e != hipSuccess) return e;
    }
    if (L.sequential == kJobsStreamed || L.sequential == kJobsClaimed) one.njobs = std::min(per, L.njobs - j);
    const int n = (L.sequential == kJobsInKernel || L.sequential == kJobsStreamed || L.sequential == kJobsClaimed)
                      ? 1
                      : std::min(per, L.njobs - j);
    const dim3 grid(static_cast<unsigned>(n * L.blocks_per_job));
    hipLaunchKernelGGL(k, grid, dim3(kBlock), 0, static_cast<hipStream_t>(stream), one);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace redset_hip
