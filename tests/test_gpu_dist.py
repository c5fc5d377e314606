"""The sharded path with the HIP compute AND a real multi-rank exchange: 2 and
3 ranks spawned on the one GPU, each running redset_hip_rs_sharded_plan's
gather -> gf_mac -> return with the library's own kernels (no compute
callback), the exchange over torch.distributed gloo (TorchTransport; RCCL
refuses two ranks on one device, so the box's single GPU cannot host an RCCL
world > 1). The parity and the rebuilt members are checked against the CPU
oracle, cell by cell (tests/test_dist.py runs the same placement with the
oracle as the compute, on CPU)."""
import json
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import FALLBACK_RUN
from test_dist import _assemble, _free_port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, p, e, chunk, lost, outdir):
    import sys

    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import redset_amd
    from redset_amd.dist import ShardedSetRunner

    runner = ShardedSetRunner(p, e, chunk, lost, world=world, rank=rank, device="cuda:0", backend=None,
                              seed=7, transport="torch")
    if rank == 0:
        with open(os.path.join(outdir, "where.json"), "w") as f:
            json.dump({str(m): list(v) for m, v in runner._where.items()}, f)
    save = lambda name, t: np.save(os.path.join(outdir, f"{name}_{rank}.npy"), t.cpu().numpy())
    save("data", runner.D_host)
    runner.encode()
    torch.cuda.synchronize()
    save("par", runner.P_host)
    snap = runner.lost_snapshot()
    runner.erase()
    runner.D_gath.fill_(0xA5)
    runner.P_gath.fill_(0x5A)
    runner.rebuild()
    torch.cuda.synchronize()
    save("data2", runner.D_host)
    save("par2", runner.P_host)
    with open(os.path.join(outdir, f"faults_{rank}.json"), "w") as f:
        json.dump({"ring_faults": int(redset_amd.ring_faults()),
                   "matches": bool(runner.matches(snap))}, f)
    runner.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,p,e,chunk,lost", [(2, 11, 3, 65536 + 48, [1, 2]), (3, 5, 2, 40000, [0, 4]),
                                                   (2, 4, 2, 3001, [3])])
def test_sharded_hip_compute_over_gloo(oracle, world, p, e, chunk, lost):
    port = _free_port()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(world, port, p, e, chunk, lost, td), nprocs=world, join=True)
        load = lambda name: [np.load(os.path.join(td, f"{name}_{g}.npy")) for g in range(world)]
        data, par, data2, par2 = load("data"), load("par"), load("data2"), load("par2")
        W = data[0].shape[-1]
        with open(os.path.join(td, "where.json")) as f:
            where = json.load(f)
        for g in range(world):
            with open(os.path.join(td, f"faults_{g}.json")) as f:
                rec = json.load(f)
            assert rec["matches"], g
            if not FALLBACK_RUN:  # the spin-cap twin counts capped spins by design
                assert rec["ring_faults"] == 0, g
        st = oracle.OracleRS(p, e)
        for k in range(world):
            lofi = [_assemble(data, where, world, p, chunk, W, k, r) for r in range(p)]
            want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
            st.encode_set(lofi, want, chunk)
            for r in range(p):
                assert np.array_equal(_assemble(par, where, world, p, chunk, W, k, r), want[r]), (k, r)
                assert np.array_equal(_assemble(data2, where, world, p, chunk, W, k, r), lofi[r]), (k, r)
                assert np.array_equal(_assemble(par2, where, world, p, chunk, W, k, r), want[r]), (k, r)
