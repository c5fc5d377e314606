/*
 * redset_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of ECP-VeloC/redset's Reed-Solomon / XOR arithmetic and
 * stripe layout, used as the parity checker for the HIP path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The
 * product library (redset_amd/) never links or calls this code.
 *
 * Every function cites the reference file:line it restates
 * (paths relative to the reference root, v0.4.0 @ 2024-08-07).
 *
 * Pinning: the reference cannot be compiled in this image without writing
 * stand-ins for its generated config.h and the absent KVTree headers, so it
 * is treated as unbuildable (DESIGN.md "Oracle"). The restatement is pinned
 * by the reference's own known-answer encoding matrix (p=4, e=2:
 * doc/rst/schemes.rst:381-388 and src/redset_reedsolomon_common.c:684-694),
 * by GF(2^8) table identities, and by an independent numpy restatement in
 * tests/. Byte-level parity beyond the matrix KAT is "partially pinned".
 */
#ifndef REDSET_ORACLE_H
#define REDSET_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* mirrors the GF-relevant fields of redset_reedsolomon
 * (src/redset_internal.h:73-89) */
typedef struct {
  int ranks;            /* p: members of the redundancy set */
  int encoding;         /* e: parity chunks per stripe */
  unsigned int log[256];
  unsigned int exp[256];
  unsigned int imult[256];
  unsigned int* mat;    /* (p+e) x p row-major encoding matrix */
} ro_rs;

/* GF(2^8)/0x11D tables (src/redset_reedsolomon_common.c:79-150) */
void ro_gf_tables(unsigned int* log_out, unsigned int* exp_out, unsigned int* imult_out);
unsigned int ro_gf_mult(const ro_rs* st, unsigned int a, unsigned int b);

/* redset_rs_gf_alloc / redset_rs_gf_delete (:727-769) */
int  ro_rs_init(ro_rs* st, int ranks, int encoding);
void ro_rs_free(ro_rs* st);
/* convenience for ctypes: heap-allocated state */
ro_rs* ro_rs_new(int ranks, int encoding);
void   ro_rs_delete(ro_rs* st);
const unsigned int* ro_rs_matrix(const ro_rs* st);

/* layout maps (src/redset_reedsolomon_common.c:822-853) */
int ro_rs_get_encoding_id(int ranks, int encoding, int rank, int chunk_id);
int ro_rs_get_data_id(int ranks, int encoding, int rank, int chunk_id);

/* buf ^= coeff*data (src/redset_reedsolomon_common.c:786-819) */
void ro_rs_multadd(const ro_rs* st, size_t count, uint8_t* buf, unsigned int coeff, const uint8_t* data);
/* 256-entry product table (src/redset_reedsolomon_common.c:184-233) */
void ro_rs_premult_table(const ro_rs* st, unsigned int v, uint8_t* prods);

/* row selection + elimination (src/redset_reedsolomon_common.c:425-630) */
void ro_rs_identify_rows(const ro_rs* st, int missing, const int* unknowns,
                         unsigned int* m_out /* missing*missing */, int* rows_out /* missing */);
void ro_rs_gaussian_solve(const ro_rs* st, unsigned int* m, int missing, size_t count, uint8_t** bufs);

/* ---- whole-set operations (all p members in one address space) ----
 * lofi[r]   : rank r's logical file, (p-e) cells of chunk_size bytes
 * parity[r] : rank r's redundancy payload, e cells (file offset header+i*C)
 * slice     : bytes per pass (redset_mpi_buf_size, src/redset.c:45); the
 *             result does not depend on it.                                */
/* restates redset_reedsolomon_encode (src/redset_reedsolomon.c:280-402) */
void ro_rs_encode_set(const ro_rs* st, size_t chunk_size, uint8_t* const* lofi,
                      uint8_t* const* parity, size_t slice);
/* restates redset_reedsolomon_decode (src/redset_reedsolomon.c:570-785):
 * erased members listed ascending in rebuild_ranks; their lofi/parity are
 * overwritten. Returns 0 on success, 1 if missing > encoding. */
int  ro_rs_rebuild_set(const ro_rs* st, size_t chunk_size, int missing, const int* rebuild_ranks,
                       uint8_t* const* lofi, uint8_t* const* parity, size_t slice);

/* XOR: restates redset_xor_encode (src/redset_xor.c:220-295);
 * lofi[r] holds (p-1) cells, xorc[r] one cell. */
void ro_xor_encode_set(int ranks, size_t chunk_size, uint8_t* const* lofi, uint8_t* const* xorc, size_t slice);
/* restates redset_recover_xor_rebuild_serial (src/redset_xor_serial.c:161-275) */
void ro_xor_rebuild_set(int ranks, size_t chunk_size, int root, uint8_t* const* lofi, uint8_t* const* xorc, size_t slice);

/* CPU baseline: restates redset_reedsolomon_encode_pthreads
 * (src/redset_reedsolomon_pthreads.c:567-699; pool :184-224, :388-564):
 * min(nprocs,10) workers, each multadd split into contiguous jobs with a
 * private premult table, a barrier after every ring step. Computes the
 * parity of members [rank_lo, rank_hi). Returns number of threads used. */
int ro_rs_encode_pthreads(const ro_rs* st, size_t chunk_size, uint8_t* const* lofi,
                          uint8_t* const* parity, size_t slice, int nthreads,
                          int rank_lo, int rank_hi);
/* XOR pthreads baseline (src/redset_xor_pthreads.c:311-392) */
int ro_xor_encode_pthreads(int ranks, size_t chunk_size, uint8_t* const* lofi, uint8_t* const* xorc,
                           size_t slice, int nthreads, int rank_lo, int rank_hi);

/* CRC32 (zlib polynomial), as redset_crc32 (src/redset_io.c:478-521) uses */
uint32_t ro_crc32(uint32_t crc, const uint8_t* buf, size_t len);

#ifdef __cplusplus
}
#endif
#endif
