/*
 * redset_hip_backend.c -- redset's REDSET_ENCODE=HIP backend slot: the glue a
 * redset maintainer compiles into libredset. It turns
 * redset's own types into the plain arguments of the per-rank backends in
 * libredset_hip_mpi.so (include/redset_hip_mpi.h), which keep the
 * reference's MPI message patterns and run every GF(2^8) operation on the
 * GPU. Dispatch: redset_apply_rs (src/redset_reedsolomon.c:522-545),
 * redset_recover_rs_rebuild (:986-1006), redset_apply_xor (src/redset_xor.c:
 * 399-420) and redset_recover_xor_rebuild (:650-671) each get a
 * `case REDSET_ENCODE_HIP:` calling the function of the same role below.
 *
 * Compiled here only by tests/test_integration_adapter.py (-fsyntax-only
 * against the reference's own headers, with -DHAVE_CUDA so the reference's
 * CUDA prototypes are in scope and checked against ours).
 */
#include "redset_hip_backend.h"

#include "redset_hip_mpi.h"

/* The reference's redset_lofi (src/redset_lofi.h:10-16) as a redset_hip_io:
 * the backends address this rank's logical file as (rank 0, DATA, index =
 * segment, offset within segment); chunk_size maps that to the logical-file
 * offsets redset_lofi_pread / redset_lofi_pwrite take (src/redset_lofi.c:
 * 424-451), which pad reads with zeros and drop writes past the end. */
struct lofi_ctx {
  redset_lofi* rsf;
  size_t chunk_size;
};

static int lofi_read(void* c, int rank, int kind, int index, unsigned long long off, size_t n, void* dst) {
  struct lofi_ctx* x = (struct lofi_ctx*) c;
  (void) rank;
  (void) kind;
  return redset_lofi_pread(x->rsf, dst, n, (off_t) (x->chunk_size * (size_t) index + off));
}

static int lofi_write(void* c, int rank, int kind, int index, unsigned long long off, size_t n, const void* src) {
  struct lofi_ctx* x = (struct lofi_ctx*) c;
  (void) rank;
  (void) kind;
  return redset_lofi_pwrite(x->rsf, (void*) src, n, (off_t) (x->chunk_size * (size_t) index + off));
}

/* GF tables + encoding matrix for (ranks, encoding): built once and reused,
 * the role redset_rs_gf_alloc plays for d->state (src/redset_reedsolomon.c:
 * 169-171). Kept here rather than in redset_reedsolomon so the reference's
 * struct stays as it is; redset calls backends from one thread per rank
 * (SURVEY.md §8b), so a single cached codec suffices. */
static redset_hip_rs* cached_rs = NULL;

static redset_hip_rs* codec_for(int ranks, int encoding) {
  int p = 0, e = 0;
  if (cached_rs && redset_hip_rs_shape(cached_rs, &p, &e) == REDSET_SUCCESS && p == ranks && e == encoding)
    return cached_rs;
  redset_hip_rs_destroy(cached_rs);
  cached_rs = NULL;
  if (redset_hip_rs_create(ranks, encoding, &cached_rs) != REDSET_SUCCESS) cached_rs = NULL;
  return cached_rs;
}

void redset_hip_backend_finalize(void) {
  redset_hip_rs_destroy(cached_rs);
  cached_rs = NULL;
  redset_hip_rank_scratch_release();
}

int redset_reedsolomon_encode_hip(const redset_base* d, redset_lofi rsf, const char* chunk_file, int fd_xor,
                                  size_t chunk_size) {
  struct lofi_ctx x = {&rsf, chunk_size};
  redset_hip_io io = {lofi_read, lofi_write, NULL, &x};
  const redset_reedsolomon* st = (const redset_reedsolomon*) d->state;
  redset_hip_rs* rs = codec_for(d->ranks, st->encoding);
  if (!rs) return REDSET_FAILURE;
  return redset_hip_rs_encode_rank(rs, d->comm, &io, chunk_file, fd_xor, chunk_size, (size_t) redset_mpi_buf_size);
}

int redset_reedsolomon_decode_hip(const redset_base* d, int missing, int* rebuild_ranks, int need_rebuild,
                                  redset_lofi rsf, const char* chunk_file, int fd_chunk, size_t chunk_size) {
  struct lofi_ctx x = {&rsf, chunk_size};
  redset_hip_io io = {lofi_read, lofi_write, NULL, &x};
  const redset_reedsolomon* st = (const redset_reedsolomon*) d->state;
  redset_hip_rs* rs = codec_for(d->ranks, st->encoding);
  if (!rs) return REDSET_FAILURE;
  return redset_hip_rs_decode_rank(rs, d->comm, missing, rebuild_ranks, need_rebuild, &io, chunk_file, fd_chunk,
                                   chunk_size, (size_t) redset_mpi_buf_size);
}

int redset_xor_encode_hip(const redset_base* d, redset_lofi rsf, const char* chunk_file, int fd_xor,
                          size_t chunk_size) {
  struct lofi_ctx x = {&rsf, chunk_size};
  redset_hip_io io = {lofi_read, lofi_write, NULL, &x};
  return redset_hip_xor_encode_rank(d->comm, &io, chunk_file, fd_xor, chunk_size, (size_t) redset_mpi_buf_size);
}

int redset_xor_decode_hip(const redset_base* d, int root, redset_lofi rsf, const char* chunk_file, int fd_chunk,
                          size_t chunk_size) {
  struct lofi_ctx x = {&rsf, chunk_size};
  redset_hip_io io = {lofi_read, lofi_write, NULL, &x};
  return redset_hip_xor_decode_rank(d->comm, root, &io, chunk_file, fd_chunk, chunk_size,
                                    (size_t) redset_mpi_buf_size);
}

#ifdef HAVE_CUDA
/* The reference's CUDA backend prototypes are in scope (src/redset_internal.h:
 * 345-381): each HIP function must have exactly the type of the function it
 * stands beside in the dispatch switches. */
static __typeof__(redset_reedsolomon_encode_gpu)* const check_rs_encode __attribute__((unused)) =
    redset_reedsolomon_encode_hip;
static __typeof__(redset_reedsolomon_decode_gpu)* const check_rs_decode __attribute__((unused)) =
    redset_reedsolomon_decode_hip;
static __typeof__(redset_xor_encode_gpu)* const check_xor_encode __attribute__((unused)) = redset_xor_encode_hip;
static __typeof__(redset_xor_decode_gpu)* const check_xor_decode __attribute__((unused)) = redset_xor_decode_hip;
#endif
