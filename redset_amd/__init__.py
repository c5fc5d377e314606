"""redset_amd -- MI355X-native (gfx950) Reed-Solomon / XOR codec for
ECP-VeloC/redset's encode / rebuild path.

The product is the C-ABI shared library ``redset_amd/lib/libredset_hip.so``
(header: ``include/redset_hip.h``): a host C++ planner plus hand-written HIP
kernels. This package binds it for Python callers (tests, bench, the RCCL
multi-GPU rebuild driver in :mod:`redset_amd.dist`), and holds the
redundancy-file headers (:mod:`redset_amd.header`) and the whole-set apply /
header-driven rebuild over files (:mod:`redset_amd.setfiles`).
"""
from ._lib import LIB_PATH, RedsetHipError, RedsetHipUnavailable, load  # noqa: F401
from .codec import (  # noqa: F401
    Plan,
    RSCodec,
    SetLayout,
    gf_combine,
    cell_stride,
    ring_faults,
    hang_faults,
    xor_combine,
    xor_plan_encode,
    xor_plan_rebuild,
)

__version__ = "0.1.0"
