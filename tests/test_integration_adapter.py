"""The reference-side adapter (integration/redset_hip_backend.c) compiles
against the reference's own headers (src/redset_internal.h, redset_lofi.h,
redset.h, redset_util.h) and its four functions have exactly the types of the
CUDA backend functions they stand beside (src/redset_internal.h:345-381).

CPU only, and only where /root/reference exists (this container; never on
the GPU box). Two test-only stand-ins fill the gaps the reference's headers
leave in this image -- an empty cmake config.h (plus HAVE_CUDA to expose the
CUDA prototypes) and KVTree's opaque typedef (tests/integration_stubs/) --
and the compile is -fsyntax-only: nothing of the reference is built."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/src"
MPI_INC = "/opt/conda/include"


def _gcc(src, tmp_path=None, extra=()):
    cmd = ["gcc", "-std=gnu99", "-Wall", "-Wextra", "-Werror", "-fsyntax-only", "-DREDSET_ENABLE_MPI",
           "-I", os.path.join(ROOT, "tests", "integration_stubs"), "-I", REF_SRC,
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "integration"), "-I", MPI_INC,
           *extra, src]
    return subprocess.run(cmd, capture_output=True, text=True)


def _need():
    if not os.path.isdir(REF_SRC) or not os.path.exists(os.path.join(REF_SRC, "redset_internal.h")):
        pytest.skip("reference sources not present (GPU box)")
    if not shutil.which("gcc") or not os.path.exists(os.path.join(MPI_INC, "mpi.h")):
        pytest.skip("gcc or mpi.h missing")


def test_adapter_compiles_against_reference_headers():
    _need()
    res = _gcc(os.path.join(ROOT, "integration", "redset_hip_backend.c"))
    assert res.returncode == 0, res.stderr


def test_prototype_check_rejects_a_mismatch(tmp_path):
    """The adapter's HAVE_CUDA block is a real check: a function whose type
    differs from the CUDA backend's (here fd as long) does not compile."""
    _need()
    bad = tmp_path / "bad.c"
    bad.write_text('#include "redset_internal.h"\n'
                   "int wrong(const redset_base* d, redset_lofi rsf, const char* f, long fd, size_t c);\n"
                   "static __typeof__(redset_xor_encode_gpu)* const chk __attribute__((unused)) = wrong;\n")
    res = _gcc(str(bad))
    assert res.returncode != 0 and "incompatible" in res.stderr


def test_adapter_declares_the_four_backend_functions():
    text = open(os.path.join(ROOT, "integration", "redset_hip_backend.h")).read()
    for name in ("redset_reedsolomon_encode_hip", "redset_reedsolomon_decode_hip", "redset_xor_encode_hip",
                 "redset_xor_decode_hip"):
        assert f"int {name}(" in text
