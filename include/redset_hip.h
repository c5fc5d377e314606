/*
 * redset_hip.h -- C ABI of the MI355X (gfx950) Reed-Solomon / XOR codec that
 * replaces redset's encode/decode backends.
 *
 * Everything here is plain C: integers, sizes and pointers. Buffers named
 * "device" are HIP device pointers; `stream` is a hipStream_t passed as
 * void* (NULL = the default stream). Return codes follow redset:
 * REDSET_SUCCESS (0, src/redset.h:24) or REDSET_FAILURE (1,
 * src/redset_util.h:19); HIP errors map to REDSET_FAILURE and
 * redset_hip_last_error() says why.
 *
 * Where the reference dispatches to a backend (src/redset_reedsolomon.c:
 * 522-545, :986-1006; src/redset_xor.c:399-420, :650-671), a maintainer adds
 * a REDSET_ENCODE_HIP case that calls these functions; INTEGRATION.md shows
 * that glue.
 *
 * Data layout in HBM ("set layout"): member r of a redundancy set of p
 * members owns a logical-file region lofi[r] holding its data cells
 * (p-e for RS, p-1 for XOR) and a redundancy region parity[r] holding its
 * e parity cells (1 for XOR). Cell s of either region starts at
 * base + s * cell_stride, cell_stride >= chunk_size. This mirrors the
 * reference's logical file (segment s at s*chunk_size, src/redset_
 * reedsolomon.c:334-335) and redundancy file (slot i at header + i*chunk_size,
 * :380-381) with an optional pad so every cell can start 16-B aligned.
 * Cells at a 16-B aligned address take the vector path; others work, slowly.
 */
#ifndef REDSET_HIP_H
#define REDSET_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef REDSET_SUCCESS
#define REDSET_SUCCESS (0)
#endif
#ifndef REDSET_FAILURE
#define REDSET_FAILURE (1)
#endif

typedef struct redset_hip_rs redset_hip_rs;      /* GF tables + encoding matrix */
typedef struct redset_hip_plan redset_hip_plan;  /* prepared kernel launches */

enum {
  REDSET_HIP_PLAN_RS_ENCODE = 1,
  REDSET_HIP_PLAN_RS_REBUILD = 2,
  REDSET_HIP_PLAN_XOR_ENCODE = 3,
  REDSET_HIP_PLAN_XOR_REBUILD = 4
};

typedef struct {
  int kind;                          /* REDSET_HIP_PLAN_* */
  int ranks;                         /* p */
  int encoding;                      /* e (1 for XOR) */
  int missing;                       /* erased members (rebuild plans) */
  int launches;                      /* kernel launches per execute */
  int jobs;                          /* stripe jobs over all launches */
  size_t chunk_size;                 /* bytes per cell */
  unsigned long long bytes_read;     /* algorithmic bytes read per execute */
  unsigned long long bytes_written;  /* algorithmic bytes written per execute */
} redset_hip_plan_info;

/* ---- field, matrix, layout ------------------------------------------- */

/* Build GF(2^8) tables and the (p+e) x p encoding matrix.
 * Replaces redset_rs_gf_alloc (src/redset_reedsolomon_common.c:727-757) as
 * called from redset_construct_rs (src/redset_reedsolomon.c:169-185); same
 * validity rule: 1 <= encoding < ranks, ranks + encoding <= 256. */
int redset_hip_rs_create(int ranks, int encoding, redset_hip_rs** out);
/* Replaces redset_rs_gf_delete (src/redset_reedsolomon_common.c:759-769). */
void redset_hip_rs_destroy(redset_hip_rs* rs);
/* Copies the (p+e) x p matrix (state->mat, src/redset_internal.h:88) as bytes. */
int redset_hip_rs_matrix(const redset_hip_rs* rs, unsigned char* mat_out);
/* ranks (p) and encoding (e) of a codec (d->ranks, state->encoding). */
int redset_hip_rs_shape(const redset_hip_rs* rs, int* ranks, int* encoding);
/* Same results as redset_rs_get_encoding_id / redset_rs_get_data_id
 * (src/redset_reedsolomon_common.c:822-853). */
int redset_hip_rs_get_encoding_id(int ranks, int encoding, int rank, int chunk_id);
int redset_hip_rs_get_data_id(int ranks, int encoding, int rank, int chunk_id);

/* ---- whole-set plans (all members' cells resident on one device) ----- */

/* Recommended cell_stride for a set held in one device allocation: chunk_size
 * rounded up to 256 B, plus 16 MiB when that is a multiple of 16 MiB. Cells
 * of a power-of-two size such as 64 MiB otherwise start at addresses equal
 * modulo 2^24..2^26, and a stripe's 11 streams then share DRAM channels and
 * banks; the pad staggers them (+2.0% on the RS(8+3) step at 64 MiB cells,
 * profiles/r02_ab_cell_pad.txt; the bench uses this layout). Any stride >=
 * chunk_size is correct; this one is only faster. */
size_t redset_hip_cell_stride(size_t chunk_size);

/* Parity of every stripe of the set: the work redset_reedsolomon_encode
 * (src/redset_reedsolomon.c:280-402) does across all p ranks; member r's
 * parity slot i = stripe (r+i) mod p, row p+i. lofi/parity: p device pointers. */
int redset_hip_rs_plan_encode(const redset_hip_rs* rs, unsigned char* const* lofi,
                              unsigned char* const* parity, size_t chunk_size,
                              size_t cell_stride, redset_hip_plan** out);

/* Rebuild the cells of `missing` erased members (ascending, as
 * redset_recover_rs builds them, src/redset_reedsolomon.c:1111-1119) in every
 * stripe; replaces redset_reedsolomon_decode (src/redset_reedsolomon.c:
 * 570-785) / redset_recover_rs_rebuild_serial (src/redset_reedsolomon_
 * serial.c:165-343). Outputs land in the erased members' lofi/parity cells.
 * Fails if missing > encoding (src/redset_reedsolomon.c:1096). */
int redset_hip_rs_plan_rebuild(const redset_hip_rs* rs, int missing, const int* rebuild_ranks,
                               unsigned char* const* lofi, unsigned char* const* parity,
                               size_t chunk_size, size_t cell_stride, redset_hip_plan** out);

/* XOR parity of every stripe: member r's cell = XOR of every other member's
 * cell of stripe r (src/redset_xor.c:220-295). xorc: p device pointers. */
int redset_hip_xor_plan_encode(int ranks, unsigned char* const* lofi, unsigned char* const* xorc,
                               size_t chunk_size, size_t cell_stride, redset_hip_plan** out);

/* Rebuild member `root` (src/redset_xor.c:441-531,
 * src/redset_xor_serial.c:161-275). */
int redset_hip_xor_plan_rebuild(int ranks, int root, unsigned char* const* lofi,
                                unsigned char* const* xorc, size_t chunk_size, size_t cell_stride,
                                redset_hip_plan** out);

/* Enqueue the plan's kernels on `stream`; no host synchronisation, no
 * allocation (safe inside hipStreamBeginCapture). A big-cell RS(8+3)
 * encode plan runs as one launch whose blocks claim their rows at run time
 * (DESIGN.md §4), with the claim counters in the plan: one plan must not
 * execute on two streams at once (its outputs would race anyway). */
int redset_hip_plan_execute(const redset_hip_plan* plan, void* stream);
int redset_hip_plan_get_info(const redset_hip_plan* plan, redset_hip_plan_info* info);
void redset_hip_plan_destroy(redset_hip_plan* plan);

/* ---- stripe primitives (one stripe, device pointers) ----------------- */

/* out[j] = (out[j] ^) sum_i coeffs[j*nin + i] * in[i] over GF(2^8), for
 * nbytes bytes; 1 <= nin, nout <= 256. Up to 16 inputs x 4 outputs run as
 * one kernel pass; wider calls run 16-input accumulate passes per group of
 * 4 outputs (outputs must not alias inputs then). One pass replaces nout*nin
 * calls of redset_rs_reduce_buffer_multadd (src/redset_reedsolomon_common.c:
 * 786-819) and, with a decode matrix, redset_rs_reduce_decode +
 * redset_rs_gaussian_solve (:855-899, :570-630). */
int redset_hip_gf_combine(const unsigned char* const* in, int nin, unsigned char* const* out,
                          int nout, const unsigned char* coeffs, size_t nbytes, int accumulate,
                          void* stream);

/* out = (out ^) XOR of nin inputs, 1 <= nin <= 256 (reduce_xor, src/redset_xor.c:35-42). */
int redset_hip_xor_combine(const unsigned char* const* in, int nin, unsigned char* out,
                           size_t nbytes, int accumulate, void* stream);

/* Many stripe combines of nbytes each as one plan (the gf_mac / xor kernels
 * with the set plans' job orders: jobs of one shape share a launch): job k is
 * out[j] = (out[j] ^) sum_i coef[j*nin + i] * in[i], as redset_hip_gf_combine;
 * a job with one output and every coefficient 1 runs on the XOR kernel. No
 * job's output may be another job's input. The arrays are copied; the
 * buffers must outlive the plan. Used by the sharded plans' partial-sum
 * shape (REDSET_HIP_SHAPE_REDUCE). */
typedef struct {
  int nin, nout;
  const unsigned char* const* in;   /* nin device pointers */
  unsigned char* const* out;        /* nout device pointers */
  const unsigned char* coef;        /* nout x nin */
  int accumulate;                   /* XOR into the outputs */
} redset_hip_combine_job;
int redset_hip_plan_combine(const redset_hip_combine_job* jobs, int njobs, size_t nbytes,
                            redset_hip_plan** out);

/* Host-side decode matrix for one stripe: rows = missing outputs, columns =
 * the p members (0 for erased members / unused cells). coef_out: missing x p
 * bytes. Equals the reference's reduce_decode + gaussian_solve as one linear
 * map. */
int redset_hip_rs_decode_matrix(const redset_hip_rs* rs, int missing, const int* rebuild_ranks,
                                int chunk_id, unsigned char* coef_out);

/* ---- host-resident streaming pipeline (pinned staging <-> HBM) ------- */
/*
 * Encode / rebuild a set whose cells live outside the GPU (host memory or
 * files): cells stream through pinned host buffers, hipMemcpyAsync to HBM,
 * the gf_mac / xor kernel, and back, with reads, H2D, compute, D2H and writes
 * of successive (stripe, slice) units overlapped. This is the shape of the
 * reference's own loop -- slices of redset_mpi_buf_size read via
 * redset_lofi_pread, combined, written after the header
 * (src/redset_reedsolomon.c:309-391) -- with the arithmetic on the GPU.
 */
#define REDSET_HIP_CELL_DATA (0)    /* logical-file segment `index` */
#define REDSET_HIP_CELL_PARITY (1)  /* redundancy slot `index` */

typedef struct {
  /* Read / write `len` bytes at byte `offset` of a cell of member `rank`
   * (kind DATA: logical-file offset index*chunk_size + offset; kind PARITY:
   * redundancy-file offset header + index*chunk_size + offset). Return 0 on
   * success. Called concurrently from the pipeline's I/O threads. */
  int (*read)(void* ctx, int rank, int kind, int index, unsigned long long offset, size_t len, void* dst);
  int (*write)(void* ctx, int rank, int kind, int index, unsigned long long offset, size_t len, const void* src);
  /* Optional (may be NULL): host address of the cell bytes at `offset` if
   * that memory is page-locked, so the pipeline can DMA it directly instead
   * of staging it through read/write; NULL = use read/write. */
  void* (*map)(void* ctx, int rank, int kind, int index, unsigned long long offset);
  void* ctx;
} redset_hip_io;

typedef struct {
  double seconds;                    /* wall time of the call */
  unsigned long long bytes_read;     /* algorithmic bytes of cells read */
  unsigned long long bytes_written;  /* algorithmic bytes of cells written */
  unsigned long long units;          /* (stripe, slice) units */
  double read_seconds;               /* summed time inside io->read */
  double write_seconds;              /* summed time inside io->write */
  double gpu_seconds;                /* H2D + kernels + D2H, event-timed */
} redset_hip_stream_stats;

/* Stripes [first_stripe, first_stripe + nstripes) (nstripes <= 0: all).
 * slice_bytes: per-cell slice (0 = 8 MiB); io_threads (0 = 8). */
int redset_hip_rs_encode_stream(const redset_hip_rs* rs, size_t chunk_size, int first_stripe, int nstripes,
                                size_t slice_bytes, int io_threads, const redset_hip_io* io,
                                redset_hip_stream_stats* stats);
int redset_hip_rs_rebuild_stream(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, size_t chunk_size,
                                 int first_stripe, int nstripes, size_t slice_bytes, int io_threads,
                                 const redset_hip_io* io, redset_hip_stream_stats* stats);
int redset_hip_xor_encode_stream(int ranks, size_t chunk_size, int first_stripe, int nstripes, size_t slice_bytes,
                                 int io_threads, const redset_hip_io* io, redset_hip_stream_stats* stats);
int redset_hip_xor_rebuild_stream(int ranks, int root, size_t chunk_size, int first_stripe, int nstripes,
                                  size_t slice_bytes, int io_threads, const redset_hip_io* io,
                                  redset_hip_stream_stats* stats);

/* The streaming calls keep a successful call's three streams and (up to
 * 256 MiB pinned, 1 GiB of device memory) its staging buffers for the next
 * call; REDSET_HIP_SCRATCH_CACHE=0 allocates and frees per call. This frees
 * what is cached. */
void redset_hip_release_scratch(void);

/* Built-in I/O over host memory laid out like the device set layout
 * (lofi[r] + s*cell_stride, parity[r] + i*cell_stride). pinned != 0 declares
 * the memory page-locked (hipHostMalloc / hipHostRegister): cells are then
 * DMAed directly, with no staging copy. */
typedef struct redset_hip_hostio redset_hip_hostio;
int redset_hip_hostio_create(int ranks, unsigned char* const* lofi, unsigned char* const* parity, size_t cell_stride,
                             int pinned, redset_hip_io* io_out, redset_hip_hostio** out);
void redset_hip_hostio_destroy(redset_hip_hostio* h);

/* Built-in I/O over files with redset's logical-file semantics
 * (src/redset_lofi.c:30-173): member r's logical file is the concatenation
 * of its nfiles[r] data files (paths/sizes flattened member by member);
 * reads past a file's recorded size return zeros, writes past it are
 * dropped. Member r's parity goes to redundancy_paths[r] at
 * header_sizes[r] + slot*chunk_size (src/redset_reedsolomon.c:380-381).
 * Data files of members with writable[r] != 0 are created / extended to their
 * recorded size (rebuild targets); other data files are opened read-only.
 * redundancy_paths may be NULL (data-only I/O, e.g. for the per-rank MPI
 * backends, which use their own fd_chunk). */
typedef struct redset_hip_fileio redset_hip_fileio;
int redset_hip_fileio_create(int ranks, const int* nfiles, const char* const* paths,
                             const unsigned long long* sizes, const char* const* redundancy_paths,
                             const unsigned long long* header_sizes, size_t chunk_size, const int* writable,
                             redset_hip_io* io_out, redset_hip_fileio** out);
void redset_hip_fileio_destroy(redset_hip_fileio* f);

/* ---- sets sharded over the GPUs of a node (multi-rank rebuild) ------- */
/*
 * Replaces the reference's MPI rings for a redundancy set whose members live
 * on different GPUs: the decode's reduce ring (src/redset_reedsolomon.c:
 * 646-703) becomes ONE grouped exchange that gathers, onto every GPU, its
 * column slice of each cell the decode reads; every GPU runs the gf_mac
 * kernel on its slice of every stripe; a second grouped exchange returns the
 * rebuilt slices to the GPUs hosting the lost members (the gather of :713-733).
 * Byte j of an output depends only on byte j of its stripe's inputs
 * (SURVEY.md §8e), so the column slices are independent. Encode works the
 * same way (all data cells in, all parity cells back; replaces :329-377).
 *
 * World: `world` processes (one per GPU), this one is `rank`. The caller
 * places `nsets` sets of p members: member r of set k is hosted by process
 * host[k*p + r] at hosted index slot[k*p + r] (< max_hosted). Every cell is
 * cut into `world` column slices of `slice_bytes` (W) bytes
 * (redset_hip_shard_slice_bytes); slice q covers cell bytes [q*W, q*W + W)
 * clipped to chunk_size. Buffers of this process (device memory for the HIP
 * compute and RCCL; any memory the transport and compute can address):
 *   hosted_data     [world][max_hosted][d][W]   slice q of data cell s of my
 *                                               hosted member j
 *   hosted_parity   [world][max_hosted][e][W]   same for parity slot i
 *   gathered_data   [world][max_hosted][d][W]   my slice of data cell s of the
 *                                               member hosted at (h, j)
 *   gathered_parity [world][max_hosted][e][W]
 * (d = p - e). A member's logical file is thus stored as `world` column slabs.
 */
typedef struct {
  int peer;     /* process in the transport's world; == own rank: a local copy */
  int send;     /* 1: send buf to peer; 0: receive buf from peer (local copy:
                   the send entry is the source, the receive entry right after
                   it the destination) */
  void* buf;
  size_t len;
} redset_hip_xfer;

typedef struct {
  int world, rank;
  /* Run one exchange: every transfer of the list concurrently (sends and
   * receives between a pair of processes are listed in the same order on
   * both sides, with equal lengths). Stream-ordered transports (RCCL) enqueue
   * on `stream` and return; others complete before returning, after waiting
   * for work already on `stream`. Return 0 on success. */
  int (*exchange)(void* ctx, const redset_hip_xfer* xfers, int n, void* stream);
  void* ctx;
} redset_hip_transport;

typedef struct {
  /* Optional compute (NULL run = the HIP gf_mac plans): encode (kind
   * REDSET_HIP_PLAN_RS_ENCODE) or rebuild (..._RS_REBUILD, `missing` erased
   * members) of one set whose cells are at lofi/parity in the set layout
   * (cell_stride apart, nbytes each). Tests put the CPU oracle here. */
  int (*run)(void* ctx, int kind, int missing, const int* rebuild_ranks, unsigned char* const* lofi,
             unsigned char* const* parity, size_t nbytes, size_t cell_stride, void* stream);
  void* ctx;
} redset_hip_compute;

typedef struct {
  int nsets;
  const int* host;              /* [nsets * p] */
  const int* slot;              /* [nsets * p] */
  int max_hosted;
  size_t chunk_size;
  size_t slice_bytes;           /* W */
  unsigned char* hosted_data;
  unsigned char* hosted_parity;
  unsigned char* gathered_data;
  unsigned char* gathered_parity;
} redset_hip_shard_layout;

typedef struct {
  int kind;                               /* REDSET_HIP_PLAN_RS_ENCODE / _REBUILD */
  int world, rank, nsets, missing;
  size_t my_slice_len;                    /* cell bytes of this process's slice */
  int gather_messages, return_messages;   /* peer messages after merging (no local copies) */
  unsigned long long gather_bytes_sent;   /* to other processes, per execute */
  unsigned long long gather_bytes_recv;
  unsigned long long return_bytes_sent;
  unsigned long long return_bytes_recv;
  unsigned long long local_bytes;         /* copied within this process: 0 (own slices computed in place) */
  unsigned long long compute_bytes;       /* algorithmic bytes of this process's slice */
  unsigned long long gather_msg_max;      /* largest / smallest peer message this process sends */
  unsigned long long gather_msg_min;
  unsigned long long return_msg_max;
  unsigned long long return_msg_min;
  int gather_recv_messages, return_recv_messages; /* peer messages this process receives */
} redset_hip_sharded_info;

typedef struct redset_hip_sharded redset_hip_sharded;

/* Phases of one execute, in this order. The gather shape: gather the input
 * slices, compute, return the output slices (ACCUMULATE does nothing). The
 * partial-sum shape (REDSET_HIP_SHAPE_REDUCE): GATHER does nothing, COMPUTE
 * makes this process's partial sums, RETURN sends them to the outputs' hosts,
 * ACCUMULATE adds what arrived (and this process's own inputs) into the
 * outputs. Running the four in order is one execute in either shape. */
enum {
  REDSET_HIP_PHASE_GATHER = 0,
  REDSET_HIP_PHASE_COMPUTE = 1,
  REDSET_HIP_PHASE_RETURN = 2,
  REDSET_HIP_PHASE_ACCUMULATE = 3
};

/* Column slice width for chunk_size bytes over `world` processes: ceil(C/world)
 * rounded up to 256 B (so every slice starts 16-B aligned). */
size_t redset_hip_shard_slice_bytes(size_t chunk_size, int world);

/* Plan the sharded encode (kind REDSET_HIP_PLAN_RS_ENCODE, missing 0) or
 * rebuild of `missing` members (ascending rebuild_ranks, the same in every
 * set) of every set. Collective in the sense that every process plans with
 * the same placement; planning itself does no communication. The rebuild
 * gathers only the cells some stripe's decode reads (surviving data and the
 * parity rows identify_rows selects, src/redset_reedsolomon_common.c:
 * 425-564) and never a lost member's. */
int redset_hip_rs_sharded_plan(const redset_hip_rs* rs, int kind, int missing, const int* rebuild_ranks,
                               const redset_hip_shard_layout* layout, const redset_hip_transport* transport,
                               const redset_hip_compute* compute, redset_hip_sharded** out);
/* The same for an XOR set (e = 1; kind REDSET_HIP_PLAN_XOR_ENCODE, or
 * REDSET_HIP_PLAN_XOR_REBUILD of member `root`): the layout's cells are the
 * p - 1 logical-file segments and the one XOR chunk of every member. The
 * rebuild gathers every survivor's every cell; it replaces the pipelined
 * reduce to the lost member (src/redset_xor.c:466-524). */
int redset_hip_xor_sharded_plan(int ranks, int kind, int root, const redset_hip_shard_layout* layout,
                                const redset_hip_transport* transport, const redset_hip_compute* compute,
                                redset_hip_sharded** out);
/* The same plans with only some processes computing: compute_on[g] != 0 for
 * the K processes that take a column slice each (in rank order, slices
 * 0 .. K - 1; slice_bytes >= ceil(chunk_size / K); NULL: all of them, as
 * above). The others only send the cells they host and receive their
 * members' outputs -- e.g. a rebuild whose lost members then receive just
 * their own cells instead of also gathering a slice of every decode input.
 * Every process must pass the same mask. */
int redset_hip_rs_sharded_plan_on(const redset_hip_rs* rs, int kind, int missing, const int* rebuild_ranks,
                                  const redset_hip_shard_layout* layout, const int* compute_on,
                                  const redset_hip_transport* transport, const redset_hip_compute* compute,
                                  redset_hip_sharded** out);
int redset_hip_xor_sharded_plan_on(int ranks, int kind, int root, const redset_hip_shard_layout* layout,
                                   const int* compute_on, const redset_hip_transport* transport,
                                   const redset_hip_compute* compute, redset_hip_sharded** out);
/* The exchange's shape (redset_hip_sharded_opts.shape).
 * GATHER: every computing process gathers its column slice of every cell a
 *   stripe reads and returns its slice of every output -- (inputs + outputs)
 *   x (world - 1) / world cells per stripe cross the fabric.
 * REDUCE: the code is linear, so every process combines the inputs IT hosts
 *   into partial outputs (the stripe's own coefficients) and sends one
 *   partial per output and contributing process to the output's host, which
 *   XORs them in: outputs x (contributing processes - 1) cells per stripe,
 *   the shape of the reference's XOR ring, which moves partial sums
 *   (src/redset_xor.c:251-279), where its RS decode gathers inputs
 *   (src/redset_reedsolomon.c:690-733). The partials use the gathered slabs
 *   as scratch; a plan whose partials do not fit them, or with over 64
 *   processes, cannot take it.
 * AUTO: whichever moves fewer bytes through the busiest process (max over
 *   processes of max(bytes sent, bytes received) per execute; ties: GATHER).
 *   Every process computes every process's counts, so all choose alike. */
enum { REDSET_HIP_SHAPE_AUTO = 0, REDSET_HIP_SHAPE_GATHER = 1, REDSET_HIP_SHAPE_REDUCE = 2 };

typedef struct {
  size_t struct_size;             /* sizeof(redset_hip_sharded_opts): checked */
  int shape;                      /* REDSET_HIP_SHAPE_* */
  const int* compute_on;          /* as redset_hip_rs_sharded_plan_on (GATHER only; NULL = all) */
  const redset_hip_compute* compute; /* whole-set compute callback (GATHER; NULL = HIP plans) */
  /* the REDUCE shape's compute callback (NULL = HIP plans, redset_hip_plan_combine):
   * run the `njobs` combines of one phase of one set, each over nbytes */
  int (*combine)(void* ctx, const redset_hip_combine_job* jobs, int njobs, size_t nbytes, void* stream);
  void* combine_ctx;
} redset_hip_sharded_opts;

/* The plans above with options: the exchange's shape and the callbacks. The
 * four-argument forms above are this with shape GATHER (their callers run the
 * gather shape's phases themselves, e.g. the per-rank slot). AUTO (or REDUCE)
 * with a whole-set `compute` callback and no `combine` plans GATHER. */
int redset_hip_rs_sharded_plan_ex(const redset_hip_rs* rs, int kind, int missing, const int* rebuild_ranks,
                                  const redset_hip_shard_layout* layout, const redset_hip_transport* transport,
                                  const redset_hip_sharded_opts* opts, redset_hip_sharded** out);
int redset_hip_xor_sharded_plan_ex(int ranks, int kind, int root, const redset_hip_shard_layout* layout,
                                   const redset_hip_transport* transport, const redset_hip_sharded_opts* opts,
                                   redset_hip_sharded** out);

/* Both shapes' byte counts and the one planned. */
typedef struct {
  size_t struct_size;                       /* set by the library */
  int shape;                                /* REDSET_HIP_SHAPE_GATHER or _REDUCE */
  int reduce_possible;                      /* the partial sums fit the scratch */
  unsigned long long gather_busiest_bytes;  /* max over processes of max(sent, received), per execute */
  unsigned long long reduce_busiest_bytes;  /* the same for REDUCE (0 if not possible) */
  unsigned long long gather_bytes_sent, gather_bytes_recv;  /* this process, GATHER */
  unsigned long long reduce_bytes_sent, reduce_bytes_recv;  /* this process, REDUCE */
  unsigned long long scratch_bytes_needed;  /* REDUCE: this process's partial-sum rows */
  unsigned long long scratch_bytes;         /* the gathered slabs */
  int reduce_messages, reduce_recv_messages; /* REDUCE: peer messages per execute, after merging */
  int reduce_fused;                         /* REDUCE: a host folds its own inputs in with the
                                               partials it makes (its inputs read once; needs
                                               more scratch), else it combines them again after
                                               the exchange */
} redset_hip_sharded_shape_info;
/* Copies min(size, sizeof) bytes: callers built against an older header get
 * the fields they know, never a write past their struct. */
int redset_hip_sharded_get_shape(const redset_hip_sharded* plan, redset_hip_sharded_shape_info* info, size_t size);

/* All phases, ordered after the work already on `stream`; work
 * enqueued on `stream` afterwards sees the results. With the HIP plans as
 * compute (compute == NULL at plan time) the sets are pipelined: every set's
 * gather and return is an exchange of its own on a second stream the plan
 * owns, so set k+1's gather (and the first returns) overlap set k's gf_mac on
 * `stream`; in the partial-sum shape set k's exchange overlaps set k+1's
 * combines and set k's accumulate follows its exchange. With a compute (or
 * combine) callback the phases run one after another. */
int redset_hip_sharded_execute(redset_hip_sharded* plan, void* stream);
/* One phase (REDSET_HIP_PHASE_*), so callers can time them apart; the four in
 * order are one execute. */
int redset_hip_sharded_execute_phase(redset_hip_sharded* plan, int phase, void* stream);
int redset_hip_sharded_get_info(const redset_hip_sharded* plan, redset_hip_sharded_info* info);
void redset_hip_sharded_destroy(redset_hip_sharded* plan);

/* RCCL transport over xGMI (grouped ncclSend / ncclRecv on the caller's
 * stream; local copies as hipMemcpyAsync). One process calls
 * redset_hip_rccl_unique_id, the caller distributes the 128 bytes (any
 * channel: MPI_Bcast, torch.distributed, a file), then every process creates
 * its transport collectively (ncclCommInitRank) on its current device. */
typedef struct redset_hip_rccl redset_hip_rccl;
/* 1 if librccl can be loaded in this process (no communication), else 0 */
int redset_hip_rccl_available(void);
int redset_hip_rccl_unique_id(unsigned char id_out[128]);
int redset_hip_rccl_transport_create(const unsigned char id[128], int world, int rank, redset_hip_transport* out,
                                     redset_hip_rccl** handle);
void redset_hip_rccl_transport_destroy(redset_hip_rccl* handle);

/* The kernels count two kinds of capped waits, per device and process-wide
 * (concurrent callers share the counts):
 *
 * Capped handshake SPINS of the loader-wave ring (redset_hip_ring_faults),
 * since the last clearing read. A capped spin never costs correctness: the
 * waiting consumer (or, after a capped loader, every consumer of the rest of
 * the launch) loads its bytes straight from HBM. A nonzero count in the
 * shipped build (cap 2^24 polls) means a ring stalled and ran slower -- a
 * performance event worth reporting, not an error. It happened once in
 * development, from a since-fixed missing barrier (round 2). Synchronises the
 * device; `clear` resets the count. */
int redset_hip_ring_faults(unsigned* count, int clear);

/* Capped HANG waits (redset_hip_hang_faults): waits that end by construction
 * and have no fallback -- the streamed and claimed kernels' table hand-over,
 * claim records and end-of-sequence agreement. Their cap (2^26 polls) only
 * keeps a bug from hanging the GPU; a capped one proceeds with another job's
 * tables or drops rows, so THAT LAUNCH'S OUTPUTS ARE WRONG. The synchronous
 * entry points that run kernels -- the streaming calls, the per-rank backends
 * of redset_hip_mpi.h (host and sharded exchanges) and the offline rebuild
 * tool -- read this count before and after their work and return
 * REDSET_FAILURE when it moved, so they never report success with wrong
 * bytes (a concurrent caller's hang on the same device fails them too). The
 * asynchronous ones (redset_hip_plan_execute, redset_hip_sharded_execute,
 * the stripe primitives) cannot: their caller reads this after its own sync.
 * The read is ordered on `stream` after the work already there and waits
 * for it; NULL reads on the library's own non-blocking stream, ordered after
 * nothing (sync the work to be counted first). `clear` resets the count. */
int redset_hip_hang_faults(void* stream, unsigned* count, int clear);

/* 1 if this is the test twin library (built with REDSET_HIP_TEST_KNOBS: it
 * honours the environment knobs the test suite uses to force job orders,
 * ring fallbacks and injected failures), 0 for the product library, which
 * reads none of them. */
int redset_hip_test_build(void);

/* Text of the last failure on this thread ("" if none). */
const char* redset_hip_last_error(void);
/* For layers built on this library (the per-rank backends of
 * redset_hip_mpi.h): record `msg` as this thread's last failure; returns
 * REDSET_FAILURE. */
int redset_hip_record_error(const char* msg);
/* Library version string. */
const char* redset_hip_version(void);
/* The revision of this header's struct layouts (REDSET_HIP_ABI_VERSION) the
 * library was built with. It changes whenever a struct that crosses this
 * ABI changes size or layout; a caller compares it with the header it was
 * built against and refuses to run on a mismatch (the Python binding and the
 * per-rank backends do), so a stale caller fails loudly instead of writing
 * past a struct. 6: round 6 (combine jobs, sharded options and
 * shape info; PHASE_ACCUMULATE). */
#define REDSET_HIP_ABI_VERSION 6
int redset_hip_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* REDSET_HIP_H */
