/* TEST-ONLY stand-in for redset's cmake-generated config.h, used solely to
 * syntax-check integration/redset_hip_backend.c against the reference's
 * headers (tests/test_integration_adapter.py); nothing is built or linked
 * with it. HAVE_CUDA exposes the CUDA backend prototypes for the type check. */
#define HAVE_CUDA 1
