"""The reference's integration loop, test/test_redset.c test_sequence
(:591-659) with test_recover_loss_k_ranks (:459-589), over our file-level
apply / rebuild (redset_amd.setfiles, HIP streaming pipeline) for a set of
8 members (the reference creates its sets with set size 8, :624-634):

* for every protection level of the scheme (XOR: 1; RS: 1 .. p-1) and every
  number of lost members lose_k in 0 .. p-1, files are created with a CRC,
  a distinctive mode and mtime (:60-173), and the set is applied;
* lose_k <= level: EVERY lose_k-subset of members (increment_index, :426-455)
  loses its data files, recovery must succeed and restore CRC, mode and mtime
  (check_crcs / check_meta) and the redundancy files; then the same members
  lose data AND redundancy files, and recovery must succeed again;
* lose_k > level: the first subset loses its files and recovery must fail
  (the reference stops its enumeration there, :549-553).

Like the reference it checks the round trip only; parity bytes against the
oracle are tests/test_gpu_setfiles.py's job."""
import itertools
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

P = 8


@pytest.fixture(scope="module")
def sf():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import redset_amd
    from redset_amd import setfiles

    redset_amd.load()
    return setfiles


def _create(tmp, seed):
    """test_redset.c create_files / set_meta: member r writes (P + r) units of
    random bytes (the reference: (ranks + rank) MiB of rand() seeded by rank;
    4 KiB units + r bytes here to keep ~900 rebuilds quick)."""
    rng = np.random.default_rng(seed)
    files = []
    for r in range(P):
        path = os.path.join(tmp, "data", f"testfile_{r}.out")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        rng.integers(0, 256, (P + r) * 4096 + r, dtype=np.uint8).tofile(path)
        os.chmod(path, 0o640 if r % 2 else 0o604)
        os.utime(path, ns=(1_600_000_000_000_000_000 + 7 * r, 1_600_000_000_123_456_789 + r))
        files.append([path])
    return files


def _state(paths):
    out = {}
    for p in paths:
        st = os.stat(p)
        with open(p, "rb") as f:
            data = f.read()
        out[p] = (data, st.st_mode, st.st_mtime_ns) if not p.endswith(".redset") else (data,)
    return out


def _delete(members, reds, lost, redundancy):
    for r in lost:
        for f in members[r]:
            os.unlink(f)
        if redundancy:
            os.unlink(reds[r])


def _levels():
    yield "XOR", 1
    for k in range(1, P):
        yield "RS", k


@pytest.mark.parametrize("scheme,level", list(_levels()))
def test_redset_sequence(sf, tmp_path, scheme, level):
    tmp = str(tmp_path)
    rebuilds = 0
    for lose_k in range(P):
        members = _create(tmp, seed=97 * level + lose_k)
        res = sf.apply_set(scheme, members, os.path.join(tmp, "ckpt."), encoding=level)
        reds = res["redundancy"]
        allpaths = [f for fl in members for f in fl] + reds
        before = _state(allpaths)
        if lose_k == 0:  # test_recover_no_loss
            assert sf.rebuild_set(reds)["missing"] == []
            assert _state(allpaths) == before
            continue
        if lose_k > level:
            lost = list(range(lose_k))  # the first subset of the enumeration
            _delete(members, reds, lost, redundancy=False)
            with pytest.raises(ValueError, match="tolerates"):
                sf.rebuild_set(reds)
            continue
        for lost in itertools.combinations(range(P), lose_k):
            for redundancy in (False, True):
                _delete(members, reds, lost, redundancy)
                out = sf.rebuild_set(reds)
                rebuilds += 1
                assert out["missing"] == list(lost) and out["ok"], (lost, redundancy, out)
                assert _state(allpaths) == before, (lost, redundancy)
    assert rebuilds == 2 * sum(len(list(itertools.combinations(range(P), k))) for k in range(1, level + 1))
