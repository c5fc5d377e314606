/*
 * redset_hip_backend.h -- the four backend-slot functions of redset's
 * REDSET_ENCODE=HIP variant, with exactly the signatures of the CUDA ones
 * they stand beside (src/redset_internal.h:345-381). A redset maintainer adds
 * this header's declarations to src/redset_internal.h under HAVE_HIP and
 * compiles integration/redset_hip_backend.c into libredset.
 */
#ifndef REDSET_HIP_BACKEND_H
#define REDSET_HIP_BACKEND_H

#include "redset_internal.h"

#ifdef __cplusplus
extern "C" {
#endif

#ifndef REDSET_ENCODE_HIP
#define REDSET_ENCODE_HIP (5) /* next to REDSET_ENCODE_CUDA (4), src/redset_internal.h:34-37 */
#endif

/* replaces redset_reedsolomon_encode_gpu (src/redset_internal.h:362-368) */
int redset_reedsolomon_encode_hip(const redset_base* d, redset_lofi rsf, const char* chunk_file, int fd_xor,
                                  size_t chunk_size);

/* replaces redset_reedsolomon_decode_gpu (:370-379) */
int redset_reedsolomon_decode_hip(const redset_base* d, int missing, int* rebuild_ranks, int need_rebuild,
                                  redset_lofi rsf, const char* chunk_file, int fd_chunk, size_t chunk_size);

/* replaces redset_xor_encode_gpu (:345-351) */
int redset_xor_encode_hip(const redset_base* d, redset_lofi rsf, const char* chunk_file, int fd_xor,
                          size_t chunk_size);

/* replaces redset_xor_decode_gpu (:353-360) */
int redset_xor_decode_hip(const redset_base* d, int root, redset_lofi rsf, const char* chunk_file, int fd_chunk,
                          size_t chunk_size);

/* release the codec state the RS functions cache per (ranks, encoding) and
 * the backends' scratch cache; call from redset_finalize (src/redset.c) */
void redset_hip_backend_finalize(void);

#ifdef __cplusplus
}
#endif
#endif /* REDSET_HIP_BACKEND_H */
