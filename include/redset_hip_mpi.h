/*
 * redset_hip_mpi.h -- per-rank backends with the reference's calling
 * convention, for MPI builds of redset (library libredset_hip_mpi.so).
 *
 * These are what the reference's backend slot calls per rank
 * (src/redset_internal.h:345-381: redset_{reedsolomon,xor}_{encode,decode}_gpu),
 * with redset's own types replaced by plain arguments:
 *   d->comm / d->ranks / d->rank   -> comm (its size and rank)
 *   d->state (GF tables, mat)      -> rs (redset_hip_rs_create(ranks, encoding))
 *   redset_lofi rsf                -> lofi: this rank's logical file as a
 *                                     redset_hip_io (rank argument 0; kind DATA,
 *                                     index = segment, offset within segment)
 *   chunk_file, fd_chunk           -> same; fd_chunk is positioned just after
 *                                     the header on entry and the header size is
 *                                     taken as lseek(fd_chunk, 0, SEEK_CUR)
 *                                     (src/redset_reedsolomon.c:295, :588)
 *   redset_mpi_buf_size            -> buf_size (0 = 1 MiB, src/redset.c:45)
 * The message pattern of every MPI exchange is the reference's (RS encode
 * ring :329-363, RS decode ring + gather :646-733), each cell sent straight
 * to the member that combines it; the RS backends size their own slices from
 * buf_size (rank_mpi.c slice_bytes). XOR uses one all-to-all per slice for
 * encode, and for decode a gather to the root (small sets, short chunks) or
 * the reference's pipelined chain through the survivors (src/redset_xor.c:
 * 466-524, a slice of every stripe per message). All arithmetic runs on the
 * GPU.
 * Collective over comm; returns REDSET_SUCCESS / REDSET_FAILURE; I/O errors
 * fail the call but the collective loop continues, as in the reference.
 */
#ifndef REDSET_HIP_MPI_H
#define REDSET_HIP_MPI_H

#include <mpi.h>

#include "redset_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* replaces redset_reedsolomon_encode (src/redset_reedsolomon.c:280-402) */
int redset_hip_rs_encode_rank(const redset_hip_rs* rs, MPI_Comm comm, const redset_hip_io* lofi,
                              const char* chunk_file, int fd_chunk, size_t chunk_size, size_t buf_size);

/* replaces redset_reedsolomon_decode (src/redset_reedsolomon.c:570-785) */
int redset_hip_rs_decode_rank(const redset_hip_rs* rs, MPI_Comm comm, int missing, const int* rebuild_ranks,
                              int need_rebuild, const redset_hip_io* lofi, const char* chunk_file, int fd_chunk,
                              size_t chunk_size, size_t buf_size);

/* replaces redset_xor_encode (src/redset_xor.c:220-295) */
int redset_hip_xor_encode_rank(MPI_Comm comm, const redset_hip_io* lofi, const char* chunk_file, int fd_chunk,
                               size_t chunk_size, size_t buf_size);

/* replaces redset_xor_decode (src/redset_xor.c:441-531) */
int redset_hip_xor_decode_rank(MPI_Comm comm, int root, const redset_hip_io* lofi, const char* chunk_file,
                               int fd_chunk, size_t chunk_size, size_t buf_size);

/* The exchange of the four backends above.
 * REDSET_HIP_EXCHANGE_AUTO (the default): a DECODE whose members are on one
 * node, each owning a distinct GPU (PCI bus id), with librccl loadable on
 * every member, runs as the sharded plan over RCCL / xGMI: every member reads
 * the cells the call needs into HBM, the plan gathers column slices of them
 * onto every member's GPU, runs gf_mac (or the XOR) on each slice and returns
 * the rebuilt slices to the lost members (replacing the decode ring and
 * gather, src/redset_reedsolomon.c:646-733, and the XOR reduce to the root,
 * src/redset_xor.c:466-524); decodes elsewhere take the host-MPI paths
 * above. An RS ENCODE with d, e >= 2 and p <= 32 runs as the sharded plan over
 * host slabs (_SHARDED_HOST below: it sends (d + e)(p - 1)/p cells per member
 * where the reference's ring sends d*e, RS(8+3) 10 against 24); XOR and e = 1
 * encodes, where the two send the same, and wider sets, whose windows would
 * cut small messages, take the host ring. AUTO never sends an
 * encode over RCCL (north_star: RCCL only for the multi-rank rebuild).
 * _HOST_MPI and _SHARDED_RCCL force a path for every call (the encodes too:
 * the parity slices then return to their holders, replacing the encode
 * rings, :329-377, src/redset_xor.c:251-285); _SHARDED_MPI runs the sharded
 * plan over the MPI transport with device buffers (members may share a GPU);
 * _SHARDED_HOST runs it over the MPI transport with every slab in page-locked
 * host memory, read and written in place by the kernels over PCIe (no
 * staging, no copies; windows on two slab sets, one window's kernels under
 * the next one's reads and gather).
 * After a local device error a member still takes part in the exchange it
 * is in, so no member waits forever. The RCCL decision is made once per
 * communicator (cached on it as an MPI attribute, with the RCCL
 * communicator, freed with it). Process-wide; every member of a set must
 * pass the same mode (every call checks and fails otherwise). The exchange
 * the last call used on this thread: redset_hip_rank_last_exchange. */
enum {
  REDSET_HIP_EXCHANGE_AUTO = 0,
  REDSET_HIP_EXCHANGE_HOST_MPI = 1,
  REDSET_HIP_EXCHANGE_SHARDED_MPI = 2,
  REDSET_HIP_EXCHANGE_SHARDED_RCCL = 3,
  REDSET_HIP_EXCHANGE_SHARDED_HOST = 4
};
int redset_hip_rank_set_exchange(int mode);
int redset_hip_rank_last_exchange(void);

/* What the calling thread's last backend call moved and where it waited
 * (one member's view): bytes read from the logical file and the redundancy
 * file, sent and received over MPI (or, sharded, over the exchange's
 * transport), copied to and from the GPU (over host slabs, _SHARDED_HOST: the
 * kernels' own reads and writes across PCIe), written; and the seconds its host
 * thread spent blocked, in disjoint classes whose sum is at most the call:
 *   read / write_seconds   file I/O
 *   mpi_seconds            MPI waits: the exchanges' Waitall (the MPI
 *                          transport's too) and the per-window agreements
 *   gpu_seconds            waiting for the GPU's copies and kernels (event
 *                          and stream waits; a stream-ordered RCCL exchange
 *                          is waited for here)
 *   stage_seconds          the MPI transport's staging of device messages
 *                          through pinned memory (D2H / H2D copies, waited)
 *   copy_seconds           enqueueing the sharded windows' H2D / D2H copies
 *   plan_seconds           planning the sharded exchanges
 *   setup_seconds          the call's own resources: choosing the exchange
 *                          (and creating / destroying a _SHARDED_MPI
 *                          transport), scratch buffers and stream from the
 *                          cache or new, events, tearing the plans down
 * exchange_seconds is the host time inside redset_hip_sharded_execute and
 * its phases (the sharded calls' exchanges and kernels; it contains their
 * mpi, gpu and stage time and is not one of the classes). */
typedef struct {
  double seconds;
  double read_seconds, mpi_seconds, gpu_seconds, write_seconds;
  unsigned long long read_bytes, sent_bytes, recv_bytes, h2d_bytes, d2h_bytes, write_bytes;
  double stage_seconds, copy_seconds, plan_seconds, exchange_seconds, setup_seconds;
} redset_hip_rank_stats;
int redset_hip_rank_last_stats(redset_hip_rank_stats* out);

/* Page-locked host memory one call takes per member (and about as much
 * device memory): the RS host paths at most 256 MiB of slice buffers (encode
 * (2e+1)*G + 2e slices, decode 4p + 2*missing; rank_mpi.c cuts the slice to
 * fit: RS(8+3) at 64 MiB chunks takes 248 MiB to encode); the XOR host
 * paths a few buffers of buf_size; the sharded exchanges two window images
 * of 96 MiB, plus, over the MPI transport (_SHARDED_MPI), a staging buffer of
 * one exchange's bytes sent and received (up to ~2 x 96 MiB); over host slabs
 * (_SHARDED_HOST) two slab sets of ~192 MiB (a 96 MiB window of the p cells,
 * hosted and gathered: ~384 MiB) and no device memory. The
 * sharded windows are cut from these budgets whatever buf_size is (a window
 * never grows to the MPI buffer).
 * The host paths keep a successful call's pinned host buffers, device
 * buffers and stream for the next call (at most 256 MiB pinned, 1 GiB of
 * device memory). The sharded exchanges keep, per communicator, the last
 * call shape's context -- its plans and their streams, the two window images
 * (192 MiB pinned), the device slabs (about 4 x 96 MiB) and, for
 * _SHARDED_MPI, the transport with its staging -- so a checkpoint loop plans
 * and allocates once; another shape replaces it, a failed call frees it, and
 * freeing the communicator frees it. REDSET_HIP_SCRATCH_CACHE=0 allocates
 * and frees all of it per call instead, as the reference does
 * (src/redset_reedsolomon.c:298-302, :397-399). This frees every cache (and
 * redset_hip_release_scratch's), e.g. from redset_finalize; a communicator
 * whose sharded call is running in another thread keeps its context and
 * transport until it is freed. */
void redset_hip_rank_scratch_release(void);

/* Transport of the sharded path (redset_hip_rs_sharded_plan) over MPI
 * point-to-point: MPI_Isend / MPI_Irecv of every message of an exchange,
 * then MPI_Waitall -- the reference's own primitives (src/redset_reedsolomon.c:
 * 690-694, :713-733) for builds without RCCL or across nodes. Buffers are
 * host memory (device_buffers = 0; the exchange waits for `stream` only if
 * one is passed, and a host-only caller needs no HIP runtime), device memory
 * staged through pinned host buffers with hipMemcpyAsync (device_buffers = 1;
 * no GPU-aware MPI needed), or page-locked host memory that HIP kernels read
 * and write in place (device_buffers = 2: every exchange first waits for
 * `stream`, the null stream included). Messages above 1 GiB are split alike
 * on both sides. */
typedef struct redset_hip_mpi_transport redset_hip_mpi_transport;
int redset_hip_mpi_transport_create(MPI_Comm comm, int device_buffers, redset_hip_transport* out,
                                    redset_hip_mpi_transport** handle);
/* Size the transport's staging (device mode) and MPI request buffers for
 * exchanges of up to `bytes` of messages to and from other processes and
 * `messages` such messages (redset_hip_sharded_info: bytes sent + received,
 * messages sent + received, of the largest exchange). Local; agree on the
 * result before the first exchange. An exchange that finds its buffers too
 * small allocates them itself, and a failure there returns before any
 * message is posted -- the peers then wait in that exchange -- so callers
 * that can fail must reserve first (the per-rank backends do). */
int redset_hip_mpi_transport_reserve(redset_hip_mpi_transport* handle, size_t bytes, size_t messages);
void redset_hip_mpi_transport_destroy(redset_hip_mpi_transport* handle);

#ifdef __cplusplus
}
#endif
#endif /* REDSET_HIP_MPI_H */
