"""Redundancy sets on disk, in one process: write every member's redundancy
file (header + parity chunks) and rebuild lost members from whatever
redundancy files survive, learning the set from their headers.

This is the file-level job of redset_apply over a whole set
(src/redset_reedsolomon.c:405-566, src/redset_xor.c:298-439) and of the
single-process rebuild redset_rebuild_rs / redset_rebuild_xor
(src/redset_reedsolomon_serial.c:345-693, src/redset_xor_serial.c:277-622),
with the byte work done by the HIP streaming pipeline (redset_amd.stream:
files -> pinned host buffers -> HBM -> gf_mac / xor kernels -> files).
Headers: redset_amd.header (tree content pinned by the reference's documented
examples; KVTree's byte layout unpinned)."""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

from . import header as H
from . import stream


def _codec(scheme: str, ranks: int, encoding: int):
    if scheme == "RS":
        from .codec import RSCodec

        return RSCodec(ranks, encoding)
    return None


def apply_set(scheme: str, member_files: Sequence[Sequence[str]], prefix: str, encoding: int = 1,
              world_ranks: Optional[Sequence[int]] = None, world_size: Optional[int] = None,
              group_id: int = 0, groups: int = 1, slice_bytes: int = 0) -> Dict:
    """Encode a set whose members' data files are ``member_files[r]``: write
    member r's redundancy file ``redundancy_filename(prefix, ...)`` with its
    header and its parity chunks. Returns the file names, CHUNK and the
    pipeline statistics."""
    scheme = scheme.upper()
    if scheme not in ("RS", "XOR"):
        raise ValueError(f"unknown scheme {scheme!r}")
    p = len(member_files)
    k = encoding if scheme == "RS" else 1
    wr = list(world_ranks) if world_ranks is not None else list(range(p))
    ws = world_size if world_size is not None else max(wr) + 1
    metas = [[H.FileMeta.stat(f) for f in fl] for fl in member_files]
    members = [H.member_hash(H.Descriptor(scheme, r, p, wr[r], ws, group_id, groups, k), metas[r])
               for r in range(p)]
    chunk = H.chunk_size(scheme, max(sum(m.size for m in ms) for ms in metas), p, k)
    reds, hsize = [], []
    for r in range(p):
        red = H.redundancy_filename(scheme, prefix, wr[r], group_id, groups, r, p)
        fd = os.open(red, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        try:
            hsize.append(H.write_header(fd, H.header_tree(scheme, r, members, wr, chunk, k)))
        finally:
            os.close(fd)
        reds.append(red)
    io = stream.FileIO([[(m.path, m.size) for m in ms] for ms in metas], reds, hsize, chunk)
    try:
        if scheme == "RS":
            st = stream.rs_encode_stream(_codec(scheme, p, k), chunk, io, slice_bytes=slice_bytes)
        else:
            st = stream.xor_encode_stream(p, chunk, io, slice_bytes=slice_bytes)
    finally:
        io.close()
    return {"redundancy": reds, "chunk": chunk, "header_bytes": hsize, "stats": st}


def _files_ok(files) -> bool:
    """redset_lofi_check_mapped: every data file exists with its recorded
    size (src/redset_lofi.c:219-297)."""
    for path, size in files:
        try:
            if os.stat(path).st_size != size:
                return False
        except OSError:
            return False
    return True


def _apply_meta(path: str, meta: H.Tree) -> List[str]:
    """redset_meta_apply (src/redset_util.c:292-380): mode, owner, size check,
    access / modification times. Returns the failures (the reference logs
    them and reports failure)."""
    errs = []
    try:
        os.chmod(path, H.get_int(meta, "MODE") & 0o7777)
    except OSError as e:
        errs.append(f"chmod({path}): {e}")
    try:
        uid, gid = H.get_int(meta, "UID"), H.get_int(meta, "GID")
        st = os.stat(path)
        if (st.st_uid, st.st_gid) != (uid, gid):
            os.chown(path, uid, gid)
    except OSError as e:
        errs.append(f"chown({path}): {e}")
    if os.stat(path).st_size != H.get_int(meta, "SIZE"):
        errs.append(f"{path}: size {os.stat(path).st_size} expected {H.get_int(meta, 'SIZE')}")
    ns = lambda s, n: H.get_int(meta, s) * 1_000_000_000 + H.get_int(meta, n)  # noqa: E731
    os.utime(path, ns=(ns("ATIME_SECS", "ATIME_NSECS"), ns("MTIME_SECS", "MTIME_NSECS")))
    return errs


def rebuild_set(redundancy_files: Sequence[str], slice_bytes: int = 0) -> Dict:
    """Rebuild the lost members of one set from the redundancy files that can
    still be read (``redundancy_files`` may name lost ones too). A member is
    lost when its redundancy file is unreadable or shorter than header + k
    chunks, or one of its data files is absent or the wrong size. More lost
    members than the scheme tolerates is an error
    (src/redset_reedsolomon_serial.c:496-519). Lost members get
    their data files, file metadata and redundancy file (header regenerated
    from the set facts, so it matches what apply_set wrote) back."""
    heads, paths = [], {}
    for path in redundancy_files:
        try:
            t, n = H.read_header(path)
        except (OSError, ValueError):
            continue
        heads.append((t, n))
        paths[H.get_int(t, "RANK")] = path
    f = H.set_facts(heads)
    p, k = f.ranks, f.encoding
    # every member's redundancy file name, from a survivor's name and the descriptors
    any_rank, any_path = next(iter(paths.items()))
    d0 = f.descriptor(any_rank)
    g, gs = H.get_int(d0, "GROUP"), H.get_int(d0, "GROUPS")
    tail = H.redundancy_filename(f.scheme, "", f.world_ranks[any_rank], g, gs, any_rank, p)
    if not any_path.endswith(tail):
        raise ValueError(f"{any_path}: name does not follow the redundancy file pattern")
    prefix = any_path[:len(any_path) - len(tail)]
    reds = [paths.get(r) or H.redundancy_filename(f.scheme, prefix, f.world_ranks[r], g, gs, r, p)
            for r in range(p)]
    files = [f.files(r) for r in range(p)]

    def parity_ok(r: int) -> bool:  # header + k chunks present
        try:
            return os.stat(reds[r]).st_size >= f.header_size[r] + k * f.chunk
        except OSError:
            return False

    lost = [r for r in range(p) if not f.have_header[r] or not parity_ok(r) or not _files_ok(files[r])]
    out = {"scheme": f.scheme, "ranks": p, "encoding": k, "chunk": f.chunk, "missing": lost,
           "redundancy": reds, "errors": []}
    if not lost:
        return out
    if len(lost) > k:
        raise ValueError(f"{len(lost)} members lost but {f.scheme} tolerates {k}")
    hsize = [f.header_size.get(r, 0) for r in range(p)]
    for r in lost:
        for path, _ in files[r]:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            os.close(os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600))
        fd = os.open(reds[r], os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        try:
            hsize[r] = H.write_header(fd, H.header_tree(f.scheme, r, f.members, f.world_ranks, f.chunk, k))
        finally:
            os.close(fd)
    io = stream.FileIO(files, reds, hsize, f.chunk, writable=[r in lost for r in range(p)])
    try:
        if f.scheme == "RS":
            out["stats"] = stream.rs_rebuild_stream(_codec("RS", p, k), lost, f.chunk, io, slice_bytes=slice_bytes)
        else:
            out["stats"] = stream.xor_rebuild_stream(p, lost[0], f.chunk, io, slice_bytes=slice_bytes)
    finally:
        io.close()
    for r in lost:
        for i, (path, _) in enumerate(files[r]):
            (_, meta), = f.members[r]["FILE"][str(i)].items()
            out["errors"] += _apply_meta(path, meta)
    out["ok"] = not out["errors"]
    return out
