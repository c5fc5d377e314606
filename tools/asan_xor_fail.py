"""Replays tests/test_gpu_mpi.py's XOR rebuild with a failing read on rank 0
with the given rank_test build, every step under its own time limit, output
to files (debugging aid for tools/gpu_asan.sh)."""
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_mpi as T  # noqa: E402

drv, out = sys.argv[1], sys.argv[2]
tmp = os.path.join("/tmp", "asan_xor_fail")
os.makedirs(tmp, exist_ok=True)
p, e, d = 4, 1, 3
rng = np.random.default_rng(3)
files, chunk = T._setup(tmp, p, d, rng, 300_000)
reds = [os.path.join(tmp, f"r{r}.xor.redset") for r in range(p)]
T._manifests(tmp, files, chunk, [512] * p, reds)


def run(tag, args, env):
    with open(os.path.join(out, f"{tag}.out"), "w") as fo, open(os.path.join(out, f"{tag}.err"), "w") as fe:
        cmd = ["timeout", "-k", "5", "60", T.MPIRUN, "-np", str(p), "-host", "localhost", drv] + [str(a) for a in args]
        rc = subprocess.run(cmd, stdout=fo, stderr=fe, env={**os.environ, **env}).returncode
    print(tag, "rc", rc, flush=True)
    return rc


if run("encode", ["xor", "encode", e, tmp, 16384], {}) == 0:
    for pth, _ in files[2]:
        os.unlink(pth)
    os.unlink(reds[2])
    run("rebuild_fail0", ["xor", "rebuild", e, tmp, 16384, 2], {"RANK_TEST_FAIL_READ": "0"})
