"""World-size 2/3/4/8 gloo tests of the sharded path on CPU: the C ABI's
planner (redset_hip_rs_sharded_plan, redset_amd/csrc/sharded.c) drives a
torch.distributed (gloo) callback transport, and the HIP compute is replaced
by a CPU checker callback (the oracle), so these tests exercise the C
placement, column slicing and exchange plans; tests/test_gpu_parity.py covers
the HIP compute with the RCCL transport."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleBackend:
    """CPU stand-in for the HIP compute of the sharded plan (the C ABI's
    redset_hip_compute callback), built on the oracle (test-only)."""

    def __init__(self, p, e):
        import oracle_lib

        self.st = oracle_lib.OracleRS(p, e)
        self.p, self.e = p, e

    def run(self, kind, lost, lofi, parity, n, W, bufs):
        from redset_amd import _lib

        d, e = self.p - self.e, self.e
        lv = [bufs.view(a, d * W).numpy().reshape(d, W) for a in lofi]
        pv = [bufs.view(a, e * W).numpy().reshape(e, W) for a in parity]
        lf = [np.ascontiguousarray(v[:, :n]).reshape(-1) for v in lv]
        pr = [np.ascontiguousarray(v[:, :n]).reshape(-1) for v in pv]
        if kind == _lib.PLAN_RS_ENCODE:
            self.st.encode_set(lf, pr, n)
        else:
            assert self.st.rebuild_set(list(lost), lf, pr, n) == 0
        for v, a in zip(lv, lf):
            v[:, :n] = a.reshape(d, n)
        for v, a in zip(pv, pr):
            v[:, :n] = a.reshape(e, n)

    def combine(self, jobs, n, bufs):
        """The partial-sum shape's combines: out[j] = (out[j] ^) sum_i
        coef[j][i] * in[i] by the oracle's multadd
        (src/redset_reedsolomon_common.c:786-819)."""
        for ins, outs, coef, acc in jobs:
            iv = [bufs.view(a, n).numpy() for a in ins]
            for j, a in enumerate(outs):
                ov = bufs.view(a, n).numpy()
                if not acc:
                    ov[:] = 0
                for i, x in enumerate(iv):
                    if coef[j, i]:
                        self.st.multadd(ov, int(coef[j, i]), x)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, p, e, chunk, lost, outdir, sets=None, shape="gather"):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from redset_amd.dist import ShardedSetRunner

    runner = ShardedSetRunner(p, e, chunk, lost, world=world, rank=rank, device="cpu",
                              backend=OracleBackend(p, e), seed=99, transport="torch", sets=sets, shape=shape)
    if rank == 0:
        import json

        with open(os.path.join(outdir, "where.json"), "w") as f:
            json.dump({str(m): list(v) for m, v in runner._where.items()}, f)
    np.save(os.path.join(outdir, f"data_{rank}.npy"), runner.D_host.numpy())
    runner.encode()
    np.save(os.path.join(outdir, f"par_{rank}.npy"), runner.P_host.numpy())
    snap = runner.lost_snapshot()
    runner.erase()
    assert not snap or not runner.matches(snap)
    # nothing from the encode may survive into the rebuild's gathered slices
    runner.D_gath.fill_(0xA5)
    runner.P_gath.fill_(0x5A)
    runner.rebuild()
    assert runner.matches(snap)
    with open(os.path.join(outdir, f"sent_{rank}.json"), "w") as f:
        import json

        json.dump({"rebuild": runner.exchanged_bytes("rebuild"), "W": runner.W,
                   "shape": {o: runner.shape(o) for o in ("encode", "rebuild")}}, f)
    np.save(os.path.join(outdir, f"data2_{rank}.npy"), runner.D_host.numpy())
    np.save(os.path.join(outdir, f"par2_{rank}.npy"), runner.P_host.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _assemble(host_arrays, where, world, p, chunk, W, k, r):
    """full cells of member r of set k from the per-GPU column slabs"""
    h, j = where[str(k * p + r)]
    a = host_arrays[h]  # [g][j][cell][W]
    cells = []
    for c in range(a.shape[2]):
        parts = [a[g, j, c, :max(0, min(chunk, (g + 1) * W) - g * W)] for g in range(world)]
        cells.append(np.concatenate(parts))
    return np.concatenate(cells)


def _reduce_sent(p, e, lost, where, world, nsets, chunk, W):
    """All GPUs' bytes of the partial-sum shape's rebuild, counted here from
    the decode maps and the placement: one W-byte row per output cell,
    remote contributor and slice with cell bytes (independent of sharded.c)."""
    from redset_amd.codec import RSCodec

    rs = RSCodec(p, e)
    nslices = sum(1 for q in range(world) if q * W < chunk)
    rows = 0
    for k in range(nsets):
        for c in range(p):
            D = rs.decode_matrix(list(lost), c)
            for i, l in enumerate(lost):
                host = where[str(k * p + l)][0]
                contrib = {where[str(k * p + s)][0] for s in range(p) if D[i, s]}
                rows += len(contrib - {host}) * nslices
    rs.close()
    return rows * W


@pytest.mark.parametrize("world,p,e,chunk,lost,sets,shape", [
    (2, 4, 2, 3000, [1], None, "gather"), (2, 11, 3, 4096, [1, 2], None, "gather"),
    (4, 11, 3, 2048, [1, 2], None, "gather"),
    (8, 11, 3, 4096, [1, 2], None, "gather"),  # the driver's 8-GPU shape
    (3, 5, 2, 1000, [0, 4], None, "gather"),
    # one set spread over every GPU (strong scaling, BASELINE.md's C4)
    (2, 11, 3, 4096, [1, 2], 1, "gather"), (3, 5, 2, 1000, [0, 4], 1, "gather"), (8, 11, 3, 4096, [1, 2], 1, "gather"),
    # the partial-sum shape (each GPU sends partial sums of its own inputs to
    # the outputs' hosts), forced, and AUTO's choice at the bench's shapes
    (2, 11, 3, 4096, [1, 2], None, "reduce"), (4, 11, 3, 2048, [1, 2], None, ("auto", "reduce")),
    (3, 5, 2, 1000, [0, 4], None, "reduce"), (2, 11, 3, 4096, [1, 2], 1, "reduce"),
    # (AUTO at N = 2 and 4 takes the partial sums: the forced cases above
    # run that path; here the N = 8 cases, where it keeps gathering)
    (8, 11, 3, 4096, [1, 2], None, "auto"), (8, 11, 3, 4096, [1, 2], 1, "auto")])
def test_sharded_encode_rebuild_gloo(oracle, world, p, e, chunk, lost, sets, shape):
    port = _free_port()
    nsets = world if sets is None else sets
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(world, port, p, e, chunk, lost, td, sets, shape), nprocs=world, join=True)
        load = lambda name: [np.load(os.path.join(td, f"{name}_{g}.npy")) for g in range(world)]
        data, par, data2, par2 = load("data"), load("par"), load("data2"), load("par2")
        W = data[0].shape[-1]
        import json

        with open(os.path.join(td, "where.json")) as f:
            where = json.load(f)
        # fabric bytes: each decode input's slices go to the other GPUs once,
        # each rebuilt cell's slices come back from them once
        from redset_amd.dist import rebuild_inputs

        need_d, need_p = rebuild_inputs(p, e, lost)
        cells_in = sum(int(need_d[r].sum() + need_p[r].sum()) for r in range(p))
        gather_sent = nsets * (world - 1) * W * (cells_in + len(lost) * p)
        reduce_sent = _reduce_sent(p, e, lost, where, world, nsets, chunk, W)
        sent, shapes = 0, []
        for g in range(world):
            with open(os.path.join(td, f"sent_{g}.json")) as f:
                rec = json.load(f)
            sent += rec["rebuild"]
            shapes.append(rec["shape"])
        got = {sh["rebuild"]["shape"] for sh in shapes}
        assert len(got) == 1, shapes  # every GPU planned the same shape
        got = got.pop()
        want_shape = shape if isinstance(shape, str) else shape[1]
        if want_shape != "auto":
            assert got == want_shape
        else:
            # AUTO: the shape whose busiest GPU moves fewer bytes (ties: gather)
            sh = shapes[0]["rebuild"]
            better = sh["reduce_possible"] and sh["reduce_busiest_bytes"] < sh["gather_busiest_bytes"]
            assert got == ("reduce" if better else "gather"), sh
        assert sent == (reduce_sent if got == "reduce" else gather_sent), (got, sent, gather_sent, reduce_sent)
        assert cells_in == p * (p - e)
        st = oracle.OracleRS(p, e)
        for k in range(nsets):
            lofi = [_assemble(data, where, world, p, chunk, W, k, r) for r in range(p)]
            want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
            st.encode_set(lofi, want, chunk)
            for r in range(p):
                assert np.array_equal(_assemble(par, where, world, p, chunk, W, k, r), want[r]), (k, r)
                # rebuild restored every member, lost ones included
                assert np.array_equal(_assemble(data2, where, world, p, chunk, W, k, r), lofi[r]), (k, r)
                assert np.array_equal(_assemble(par2, where, world, p, chunk, W, k, r), want[r]), (k, r)


@pytest.mark.parametrize("p,e,lost", [(11, 3, [1, 2]), (4, 2, [1]), (20, 4, [0, 5, 19]), (6, 3, [2]), (11, 3, [4, 7, 10])])
def test_rebuild_inputs_read_d_cells_per_stripe(p, e, lost):
    """The sharded rebuild moves only the cells the decode reads: exactly d
    surviving cells per stripe (an MDS decode from an information set uses
    every one of them with a nonzero coefficient), all surviving data among
    them, never a lost member's."""
    from redset_amd import codec
    from redset_amd.dist import rebuild_inputs

    need_d, need_p = rebuild_inputs(p, e, lost)
    d = p - e
    rs = codec.RSCodec(p, e)
    for s in lost:
        assert not need_d[s].any() and not need_p[s].any()
    for c in range(p):
        used = 0
        for s in range(p):
            enc = rs.encoding_id(s, c)
            used += bool(need_d[s, rs.data_id(s, c)]) if enc < p else bool(need_p[s, enc - p])
        assert used == d, c
    for s in range(p):
        if s not in lost:
            assert need_d[s].all()
