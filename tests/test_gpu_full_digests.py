"""Bit-exact parity at BASELINE.json's full sizes: configs[2] (RS(8+3), 64 MiB
chunks) and configs[1] (XOR, 8 ranks, 64 MiB chunks). The inputs are
regenerated from the seeds of tests/full_size.py; the HIP plans' parity, and
the cells a rebuild restores, must hash to the SHA-256 digests the CPU oracle
produced for the same inputs (tests/golden/full_size_digests.json, made by
tests/golden/make_full_digests.py)."""
import json
import os

import pytest

import full_size

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

torch = pytest.importorskip("torch")

DIGESTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full_size_digests.json")


@pytest.fixture(scope="module")
def rd():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import redset_amd

    redset_amd.load()
    return redset_amd


@pytest.mark.parametrize("name", sorted(full_size.CASES))
def test_full_size_parity_digests(rd, name):
    case = full_size.CASES[name]
    with open(DIGESTS) as f:
        want = json.load(f)[name]
    p, e, C = case["ranks"], case["encoding"], case["chunk"]
    d = full_size.data_cells(case)
    lay = rd.SetLayout.allocate(p, d, e, C)
    S = lay.cell_stride

    def cells(region, n):  # the n cells of a member region, padding dropped
        return region.view(n, S)[:, :C]

    for r in range(p):
        x = full_size.member_lofi(case, r)
        assert full_size.sha256(x) == want["lofi_sha256"][r], f"regenerated input of member {r} differs"
        cells(lay.lofi(r), d).copy_(torch.from_numpy(x).view(d, C))
        del x
    if case["kind"] == "rs":
        codec = rd.RSCodec(p, e)
        enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), C, S)
        reb = codec.plan_rebuild(case["lost"], lay.lofi_ptrs(), lay.parity_ptrs(), C, S)
    else:
        enc = rd.xor_plan_encode(p, lay.lofi_ptrs(), lay.parity_ptrs(), C, S)
        reb = rd.xor_plan_rebuild(p, case["lost"][0], lay.lofi_ptrs(), lay.parity_ptrs(), C, S)
    enc.execute()
    torch.cuda.synchronize()
    for r in range(p):
        got = full_size.sha256(cells(lay.parity(r), e).cpu().numpy())
        assert got == want["parity_sha256"][r], f"parity of member {r}"
    for r in case["lost"]:
        lay.lofi(r).fill_(0)
        lay.parity(r).fill_(0)
    reb.execute()
    torch.cuda.synchronize()
    for r in case["lost"]:
        assert full_size.sha256(cells(lay.lofi(r), d).cpu().numpy()) == want["lofi_sha256"][r], r
        assert full_size.sha256(cells(lay.parity(r), e).cpu().numpy()) == want["parity_sha256"][r], r


def test_full_size_sharded_rebuild_digests(rd):
    """BASELINE.json configs[3] (RS(8+3), erase 2 ranks, sharded rebuild) at
    its 64 MiB chunks through the C sharded plan and the RCCL transport at
    world size 1 (a one-rank communicator; the multi-GPU slicing is covered at
    world 2-4 by tests/test_gpu_mpi.py and test_mpi_sharded.py). Same inputs
    and oracle digests as configs[2]'s case above."""
    from redset_amd.dist import ShardedSetRunner

    case = full_size.CASES["rs_p11_e3_c64MiB"]
    with open(DIGESTS) as f:
        want = json.load(f)["rs_p11_e3_c64MiB"]
    p, e, C = case["ranks"], case["encoding"], case["chunk"]
    d = p - e
    run = ShardedSetRunner(p, e, C, case["lost"], world=1, rank=0, fill=False)
    try:
        assert run.W >= C  # world 1: the slab pitch carries the cell pad
        slot = [run.host_of(0, r)[1] for r in range(p)]
        for r in range(p):
            run.D_host[0, slot[r], :, :C].copy_(torch.from_numpy(full_size.member_lofi(case, r)).view(d, C))
        run.encode()
        torch.cuda.synchronize()
        for r in range(p):
            assert full_size.sha256(run.P_host[0, slot[r], :, :C].cpu().numpy()) == want["parity_sha256"][r], r
        run.erase()
        run.rebuild()
        torch.cuda.synchronize()
        for r in range(p):
            assert full_size.sha256(run.D_host[0, slot[r], :, :C].cpu().numpy()) == want["lofi_sha256"][r], r
            assert full_size.sha256(run.P_host[0, slot[r], :, :C].cpu().numpy()) == want["parity_sha256"][r], r
    finally:
        run.close()
