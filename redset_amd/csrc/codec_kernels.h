// codec_kernels.h -- device-side job descriptors shared by the kernels
// (codec_kernels.hip) and the host planner (redset_hip.cpp).
#pragma once

// REDSET_HIP_TEST_KNOBS=1 builds the test twin library (redset_amd/lib_test):
// its planner and launchers honour the REDSET_HIP_* / REDSET_HIP_TEST_*
// environment knobs the test suite uses to force job orders, ring fallbacks
// and injected failures. The product library reads none of them.
#ifndef REDSET_HIP_TEST_KNOBS
#define REDSET_HIP_TEST_KNOBS 0
#endif

#include <cstddef>
#include <cstdint>

namespace redset_hip {

// Most inputs one kernel pass combines, and most outputs it produces.
// An output's 4 partial products are packed into one LDS dword per table
// entry, so 4 outputs cost the same lookups as 1. Wider stripes or more
// erasures are split into passes by the planner.
constexpr int kMaxIn = 16;
constexpr int kMaxOut = 4;

// Job order of a launch (GfLaunch / XorLaunch::sequential). 0: all jobs side
// by side in one grid, blocks_per_job blocks each. kJobsInLaunches: one
// launch per job over the whole grid (or per `group` jobs side by side).
// kJobsInKernel: one launch whose every block sweeps the jobs in turn. The
// last two keep one stripe's cells in flight at a time.
constexpr int kJobsInLaunches = 1;
constexpr int kJobsInKernel = 2;
// kJobsStreamed: one launch whose blocks stream their items of all the jobs
// through one continuous loader ring (codec_device.h gf_mac_stream; GF jobs
// of <= 8 inputs over whole 16-B vectors, else as kJobsInKernel).
constexpr int kJobsStreamed = 3;
// kJobsClaimed: as kJobsStreamed, but the blocks of each XCD claim their
// items in batches from a shared per-XCD queue (GfLaunch::claim), so no block
// runs ahead of the others or idles at the end (codec_device.h claimed_sweep;
// GF and XOR jobs of <= 8 inputs over whole 16-B vectors).
constexpr int kJobsClaimed = 4;
// claim queues: one counter per XCD, 128 B apart (kClaimWords words per
// launch, plan-owned; the launcher zeroes them on the launch's stream before
// every claimed launch, so no state carries from one launch to the next)
constexpr int kClaimQueues = 8;
constexpr int kClaimStride = 32;
constexpr int kClaimWords = kClaimQueues * kClaimStride;

// One stripe (or one pass over a slice of a stripe's members):
// out[j] (^)= sum_i coef[j][i] * in[i] over GF(2^8), byte by byte.
struct GfJob {
  const uint8_t* in[kMaxIn];
  uint8_t* out[kMaxOut];
  uint8_t coef[kMaxOut][kMaxIn];
};

// One launch of the GF multiply-accumulate kernel over `njobs` jobs.
struct GfLaunch {
  const GfJob* jobs;        // device array
  int njobs;
  int nin;                  // inputs per job (all jobs of a launch agree)
  int nout;                 // outputs per job
  int accumulate;           // 0: out = sum, 1: out ^= sum
  int bytes_only;           // 1: a pointer is not 16-B aligned, use the byte path
  int blocks_per_job;
  int sequential;           // job order: 0 side by side, kJobsInLaunches, kJobsInKernel (launch_gf)
  int job0;                 // first job of this launch (set by the launcher)
  int group;                // kJobsInLaunches: jobs per launch, side by side (0 = 1);
                            // kJobsStreamed / kJobsClaimed: jobs per launch, in turn (0 = all)
  size_t nbytes;            // bytes per cell
  unsigned* fault;          // set by the launcher: two device words, [0] capped ring spins (a direct-load
                            // fallback ran), [1] capped hang waits (outputs wrong; codec_device.h kRingHangCap)
  unsigned* claim;          // kJobsClaimed: kClaimWords device words (plan; zeroed per launch)
  unsigned spin_cap;        // set by the launcher; read by test builds only (codec_device.h kRingSpinCap)
  unsigned claim_delay;     // test builds: s_sleep rounds the claimer waits between claiming and recording
  unsigned hang_cap;        // test builds: polls before a wait with no fallback gives up (kRingHangCap)
  unsigned table_delay;     // test builds: s_sleep rounds before a loader publishes a job's tables
};

// XOR of `nin` inputs into one output (the XOR scheme's parity / rebuild).
struct XorJob {
  const uint8_t* in[kMaxIn];
  uint8_t* out;
};

struct XorLaunch {
  const XorJob* jobs;
  int njobs;
  int nin;
  int accumulate;
  int bytes_only;
  int blocks_per_job;
  int sequential;
  int job0;
  int group;
  size_t nbytes;
  unsigned* fault;          // set by the launcher (see GfLaunch)
  unsigned* claim;          // kJobsClaimed (see GfLaunch)
  unsigned spin_cap;        // (see GfLaunch)
  unsigned claim_delay;     // (see GfLaunch)
  unsigned hang_cap;        // (see GfLaunch)
  unsigned table_delay;     // (see GfLaunch)
};

// launchers (codec_kernels.hip); return hipError_t as int
int launch_gf(const GfLaunch& L, void* stream);
int launch_xor(const XorLaunch& L, void* stream);
// one job passed by value (L.jobs / L.njobs ignored; grid = blocks_per_job)
int launch_gf_single(const GfLaunch& L, const GfJob& J, void* stream);
int launch_xor_single(const XorLaunch& L, const XorJob& J, void* stream);
// device properties used to size grids
int device_cu_count();
// the current device's count of capped loader-ring spins since the last
// clearing read (a handshake that took the direct-load fallback; outputs
// right); `clear` resets it. Synchronises the device. Returns hipError_t.
int read_ring_faults(unsigned* count, int clear);
// the current device's count of capped hang waits (no fallback: that
// launch's outputs are wrong), read in order on `stream` after the work
// already there, which this waits for (nullptr: on the library's own
// non-blocking stream, ordered after nothing); `clear` resets it. Returns
// hipError_t as int.
int read_hang_faults(void* stream, unsigned* count, int clear);
// occupancy of the GF kernel for a given input count (blocks per CU)
int gf_blocks_per_cu(int nin);
// 1 in the test twin library (built with REDSET_HIP_TEST_KNOBS), else 0
int test_knobs();

// Threads per block, one block per CU: the kernels stream their inputs
// through a loader-wave LDS-DMA ring (codec_device.h ring_sweep) run by 1
// loader + 15 consumer waves. 7 or 11 consumers cannot keep up with the GF
// math; the per-wave sweep this replaced ran 8 waves of 512 threads
// (profiles/r02_ab_ring.txt, r02_ab_block_waves.txt).
constexpr int kBlock = 1024;

// The kernels of one input count: [nout - 1][accumulate] for gf_mac,
// [accumulate] for xor_reduce; *_arg take the job by value.
using GfKernel = void (*)(GfLaunch);
using XorKernel = void (*)(XorLaunch);
using GfKernelArg = void (*)(GfLaunch, GfJob);
using XorKernelArg = void (*)(XorLaunch, XorJob);
struct KernelSet {
  GfKernel gf[kMaxOut][2];
  GfKernelArg gf_arg[kMaxOut][2];
  XorKernel xr[2];
  XorKernelArg xr_arg[2];
};

}  // namespace redset_hip
