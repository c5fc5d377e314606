"""bench.py as the driver runs it, on the one-GPU box.

* `--gpus 2` WITHOUT torchrun: bench.py starts its two ranks itself (one
  torch.distributed.run child, before it touches the GPU), the ranks share the
  box's GPU over gloo, and exactly one JSON line comes back whose sharded leg
  (configs[3], the column-sharded rebuild, src/redset_reedsolomon.c:646-733
  replaced) is bit-exact and carries its message counts and HBM fraction.
* `--gpus 1`: the sharded leg runs at N=1 over the world-1 RCCL transport
  (configs[3]'s base point) and is bit-exact.
Small chunks keep both runs to seconds (gloo moves device tensors at tens of
MB/s); the CPU baseline, pair sweep and XOR leg are off.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "2", "--warmup", "1", "--chunk-mib", "0.5", "--cpu-baseline", "0", "--pairs", "0", "--xor", "0"]


def _bench(args, timeout):
    from conftest import gpu_available

    if not gpu_available():
        pytest.skip("needs an MI355X")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def _check_sharded(sh, world, auto=True):
    assert "error" not in sh, sh
    assert sh["bit_exact"] is True
    assert sh["value"] > 0 and 0 < sh["frac_of_hbm"] < 1  # gloo moves tens of MB/s: a tiny fraction
    assert sh["hbm_peak_GBps"] == world * 8000.0
    # the decode on slices in place and the exchange, timed apart
    assert sh["decode"]["value"] > 0 and 0 < sh["decode"]["frac_of_hbm"] < 1, sh["decode"]
    assert sh["exchange_only"]["ms_per_step"] >= 0
    msgs = sh["exchange"]["messages_per_gpu"]["rebuild"]
    if world > 1:
        if sh["shape"] == "gather":
            # every GPU gathers slices from its peer and returns rebuilt slices
            assert msgs["gather_messages"] > 0 and msgs["return_messages"] > 0, msgs
        else:
            # partial sums of each GPU's own inputs to the outputs' hosts: one exchange
            assert sh["shape"] == "reduce" and msgs["gather_messages"] == 0 and msgs["return_messages"] > 0, msgs
        # the planner's choice: the shape whose busiest GPU moves fewer bytes
        by = sh["model"]["xgmi_ms_by_shape"]
        if auto and by["reduce"] is not None:
            assert sh["shape"] == ("reduce" if by["reduce"] < by["gather"] else "gather"), by
        assert sh["exchange"]["bytes_sent_per_gpu_per_step"] > 0
        assert sh["exchange_only"]["send_GBps_per_gpu"] > 0, sh["exchange_only"]
        # BASELINE.md C4 word for word: one set over every GPU (strong scaling)
        one = sh["one_set"]
        assert one["bit_exact"] is True and one["value"] > 0 and one["decode"]["value"] > 0, one
        assert one["exchange_only"]["bytes_sent_per_gpu"] > 0, one
    else:
        assert msgs["gather_messages"] == 0 and msgs["return_messages"] == 0, msgs
        assert sh["roofline"]["bound"] == "hbm" and sh["exchange"]["bytes_sent_per_gpu_per_step"] == 0
        assert sh["exchange_only"]["send_GBps_per_gpu"] is None


@pytest.mark.timeout(420)
def test_bench_two_ranks_self_launched_over_gloo():
    """...and, at N > 1 too, the CPU baseline on rank 0 and configs[3]'s
    scaling number (sharded.value) next to `value`."""
    i = SMALL.index("--cpu-baseline")
    args = SMALL[:i] + ["--cpu-baseline", "1", "--cpu-seconds", "1"] + SMALL[i + 2:]
    line = _bench(["--gpus", "2", "--dist-backend", "gloo", "--sharded-timeout", "300"] + args, 400)
    assert line["n_gpus"] == 2 and line["round_trip_bit_exact"] is True
    assert line["config"]["sets"] == 2
    assert line["config"]["scaling_value"].startswith("sharded.value")
    _check_sharded(line["sharded"], 2)
    assert line["config"]["scaling_value_GBps"] == line["sharded"]["value"] == line["scaling_value_GBps"]
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1, cb
    # the shape the planner did not take, measured beside it, bit-exact
    other = line["sharded"]["other_shape"]
    assert other["bit_exact"] is True and other["shape"] != line["sharded"]["shape"], other
    assert other["value"] > 0 and other["decode"]["value"] > 0, other


@pytest.mark.timeout(420)
@pytest.mark.parametrize("shape", ["gather", "reduce"])
def test_bench_two_ranks_over_the_rccl_transport(shape):
    """The bench's N = 2 sharded leg as the 8-GPU node runs it -- RcclTransport,
    grouped ncclSend / ncclRecv -- on this box's one GPU: the test twin loads
    tests/rcclstub by path (REDSET_HIP_TEST_RCCL_LIBRARY; the real RCCL
    refuses two ranks on one device), the process group is gloo. Each shape
    once, bit-exact."""
    twin = os.path.join(ROOT, "redset_amd", "lib_test", "libredset_hip.so")
    stub = os.path.join(ROOT, "tests", "rcclstub", "lib", "librccl.so.1")
    if not os.path.exists(twin) or not os.path.exists(stub):
        pytest.skip("needs the test twin and tests/rcclstub")
    old = {k: os.environ.get(k) for k in ("REDSET_HIP_LIBRARY", "REDSET_HIP_TEST_RCCL_LIBRARY")}
    os.environ["REDSET_HIP_LIBRARY"] = twin
    os.environ["REDSET_HIP_TEST_RCCL_LIBRARY"] = stub
    try:
        line = _bench(["--gpus", "2", "--dist-backend", "gloo", "--sharded-timeout", "300", "--sharded-transport",
                       "rccl", "--sharded-shape", shape] + SMALL, 400)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    _check_sharded(line["sharded"], 2, auto=False)
    assert line["sharded"]["transport"].startswith("RcclTransport"), line["sharded"]["transport"]
    assert line["sharded"]["shape"] == shape


@pytest.mark.timeout(300)
def test_bench_one_gpu_runs_the_sharded_leg():
    line = _bench(["--gpus", "1"] + SMALL, 280)
    assert line["n_gpus"] == 1 and line["round_trip_bit_exact"] is True
    _check_sharded(line["sharded"], 1)
    assert line["sharded"]["transport"].startswith("RcclTransport")
