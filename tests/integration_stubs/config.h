/* TEST-ONLY stand-in for redset's cmake-generated config.h, used solely to
 * compile integration/redset_hip_backend.c against the reference's headers:
 * its syntax check (tests/test_integration_adapter.py) and the test driver
 * that runs it (tests/adapter/). No reference source is compiled with it.
 * HAVE_CUDA exposes the CUDA backend prototypes for the type check. */
#define HAVE_CUDA 1
