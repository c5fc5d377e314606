"""Redundancy-file headers: the kvtree that redset writes in front of the
parity chunks of every RS / XOR redundancy file, and the set facts a
single-process rebuild learns from the surviving headers.

What is pinned and what is not:

* The **tree content** (keys, nesting, which members' descriptors a header
  carries, CHUNK, GROUP map, RANK) follows the reference's construction
  (src/redset_reedsolomon.c:430-516, src/redset_xor.c:310-393,
  src/redset.c:628-680, src/redset_lofi.c:175-197, src/redset_util.c:264-290)
  and is checked against the two example headers the reference documents
  (doc/rst/schemes.rst:262-327 XOR, :520-603 RS) -- tests/test_header.py.
* The **text form** is kvtree_print's layout as those examples show it
  (``KEY = VALUE`` for a key whose only child is a leaf, otherwise the key on
  its own line and its children two spaces deeper).
* The **on-disk bytes** of kvtree_write_fd belong to ECP-VeloC/KVTree, an
  un-vendored dependency with no pinned version: byte parity
  is **unpinned**. :func:`encode` writes the text form behind a small frame of
  our own (``RSHIPHDR`` magic, u64 length) so our own files carry a header the
  rebuild can read back; a redset-side integration keeps calling
  kvtree_write_fd, which the backend slot never sees (the slot receives an fd
  already positioned after the header, src/redset_reedsolomon.c:295).
* Sibling order: redset_sort_kvtree (src/redset_util.c:191-205) sorts with
  KVTREE_SORT_ASCENDING; we sort keys as byte strings (strcmp order).
  Identical to the documented examples (all keys there sort the same either
  way); for sets of 10+ members whether KVTree compares member numbers as
  strings is unpinned.

Host-side control logic only: one small tree per redundancy file, built once
per encode; nothing here is on the byte path.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

Tree = Dict[str, "Tree"]

MAGIC = b"RSHIPHDR"
_FRAME = struct.Struct("<8sQ")


# ---------------------------------------------------------------- tree basics

def set_kv(t: Tree, key: str, value) -> Tree:
    """kvtree_set_kv / kvtree_util_set_*: key -> single leaf child ``value``
    (replacing what the key held)."""
    t[key] = {str(value): {}}
    return t


def get_kv(t: Tree, key: str) -> Optional[str]:
    """kvtree_get_val: the single child's name of ``key`` (None if absent)."""
    sub = t.get(key)
    if not sub:
        return None
    if len(sub) != 1:
        raise ValueError(f"key {key!r} holds {len(sub)} values, expected one")
    return next(iter(sub))


def get_int(t: Tree, key: str) -> int:
    v = get_kv(t, key)
    if v is None:
        raise KeyError(key)
    return int(v)


def merge(dst: Tree, src: Tree) -> Tree:
    """kvtree_merge: recursive union, src's leaves added under dst."""
    for k, sub in src.items():
        merge(dst.setdefault(k, {}), sub)
    return dst


def copy(t: Tree) -> Tree:
    return {k: copy(v) for k, v in t.items()}


def _sort_key(k: str) -> bytes:
    return k.encode("utf-8", "surrogateescape")


def render(t: Tree, indent: int = 0) -> str:
    """kvtree_print layout of a sorted tree (doc/rst/schemes.rst:262-327)."""
    out: List[str] = []
    pad = " " * indent
    for k in sorted(t, key=_sort_key):
        sub = t[k]
        if len(sub) == 1:
            (v, leaf), = sub.items()
            if not leaf:
                out.append(f"{pad}{k} = {v}\n")
                continue
        out.append(f"{pad}{k}\n")
        out.append(render(sub, indent + 2))
    return "".join(out)


def parse(text: str) -> Tree:
    """Inverse of :func:`render` (keys must not contain " = ")."""
    root: Tree = {}
    stack: List[Tuple[int, Tree]] = [(-1, root)]
    for line in text.splitlines():
        if not line.strip():
            continue
        ind = len(line) - len(line.lstrip(" "))
        body = line[ind:]
        while stack[-1][0] >= ind:
            stack.pop()
        parent = stack[-1][1]
        if " = " in body:
            k, v = body.split(" = ", 1)
            parent.setdefault(k, {})[v] = {}
        else:
            node = parent.setdefault(body, {})
            stack.append((ind, node))
    return root


def encode(t: Tree) -> bytes:
    """Header bytes of our own redundancy files: frame + text form + NUL
    (KVTree's binary layout is unpinned here, see the module docstring)."""
    body = render(t).encode("utf-8", "surrogateescape") + b"\0"
    return _FRAME.pack(MAGIC, len(body)) + body


def decode(buf: bytes) -> Tuple[Tree, int]:
    """(tree, header size in bytes) from the start of a redundancy file."""
    if len(buf) < _FRAME.size:
        raise ValueError("short header")
    magic, n = _FRAME.unpack_from(buf)
    if magic != MAGIC or len(buf) < _FRAME.size + n or n == 0 or buf[_FRAME.size + n - 1] != 0:
        raise ValueError("not a redset_amd redundancy-file header")
    text = buf[_FRAME.size:_FRAME.size + n - 1].decode("utf-8", "surrogateescape")
    return parse(text), _FRAME.size + n


def write_header(fd: int, t: Tree) -> int:
    """kvtree_write_fd's role: write the header at the fd's position; the
    chunks follow it (the caller's fd is left just past the header, as the
    backend slot expects, src/redset_reedsolomon.c:295)."""
    b = encode(t)
    view = memoryview(b)
    while view:
        n = os.write(fd, view)
        view = view[n:]
    return len(b)


def read_header(path: str) -> Tuple[Tree, int]:
    """kvtree_read_fd's role for one redundancy file."""
    with open(path, "rb") as f:
        head = f.read(_FRAME.size)
        if len(head) < _FRAME.size:
            raise ValueError(f"{path}: short header")
        magic, n = _FRAME.unpack(head)
        if magic != MAGIC:
            raise ValueError(f"{path}: not a redset_amd redundancy-file header")
        return decode(head + f.read(n))


# ------------------------------------------------------ redset's header trees

@dataclass
class FileMeta:
    """redset_meta_encode's fields (src/redset_util.c:264-290)."""
    path: str
    size: int
    mode: int = 0o100600
    uid: int = 0
    gid: int = 0
    atime: Tuple[int, int] = (0, 0)
    ctime: Tuple[int, int] = (0, 0)
    mtime: Tuple[int, int] = (0, 0)

    @classmethod
    def stat(cls, path: str) -> "FileMeta":
        st = os.stat(path)

        def split(ns: int) -> Tuple[int, int]:
            return ns // 1_000_000_000, ns % 1_000_000_000

        return cls(path, st.st_size, st.st_mode, st.st_uid, st.st_gid,
                   split(st.st_atime_ns), split(st.st_ctime_ns), split(st.st_mtime_ns))

    def tree(self) -> Tree:
        t: Tree = {}
        for k, v in (("MODE", self.mode), ("UID", self.uid), ("GID", self.gid), ("SIZE", self.size),
                     ("ATIME_SECS", self.atime[0]), ("ATIME_NSECS", self.atime[1]),
                     ("CTIME_SECS", self.ctime[0]), ("CTIME_NSECS", self.ctime[1]),
                     ("MTIME_SECS", self.mtime[0]), ("MTIME_NSECS", self.mtime[1])):
            set_kv(t, k, v)
        return t


@dataclass
class Descriptor:
    """The redundancy descriptor fields redset_store_to_kvtree records
    (src/redset.c:628-680; CKSUM from redset_store_to_kvtree_rs,
    src/redset_reedsolomon.c:211-222). ``scheme`` is "RS" or "XOR"."""
    scheme: str
    rank: int
    ranks: int
    world_rank: int
    world_ranks: int
    group_id: int = 0
    groups: int = 1
    encoding: int = 1
    enabled: int = 1

    def tree(self) -> Tree:
        t: Tree = {}
        set_kv(t, "ENABLED", self.enabled)
        set_kv(t, "TYPE", self.scheme)
        if self.scheme == "RS":
            set_kv(t, "CKSUM", self.encoding)
        set_kv(t, "GROUPS", self.groups)
        set_kv(t, "GROUP", self.group_id)
        set_kv(t, "RANKS", self.ranks)
        set_kv(t, "RANK", self.rank)
        set_kv(t, "WRANK", self.world_rank)
        set_kv(t, "WRANKS", self.world_ranks)
        return t


def member_hash(desc: Descriptor, files: Sequence[FileMeta]) -> Tree:
    """The per-member "current_hash": redset_lofi_encode_kvtree
    (src/redset_lofi.c:175-197) plus the descriptor under DESC
    (src/redset_reedsolomon.c:430-449, src/redset_xor.c:313-332)."""
    t: Tree = {}
    set_kv(t, "FILES", len(files))
    ft: Tree = {}
    for i, fm in enumerate(files):
        if " = " in fm.path or "\n" in fm.path or fm.path != fm.path.strip(" ") or not fm.path:
            raise ValueError(f"file name {fm.path!r} has no representation in the header text form")
        ft[str(i)] = {fm.path: fm.tree()}
    t["FILE"] = ft
    t["DESC"] = desc.tree()
    return t


def group_map(world_ranks: Sequence[int]) -> Tree:
    """GROUP kvtree: RANKS and member -> parent-rank map
    (src/redset_reedsolomon.c:95-121, same for XOR)."""
    g: Tree = {}
    set_kv(g, "RANKS", len(world_ranks))
    g["RANK"] = {str(i): {str(w): {}} for i, w in enumerate(world_ranks)}
    return {"GROUP": g}


def chunk_size(scheme: str, max_bytes: int, ranks: int, encoding: int = 1) -> int:
    """ceil(max_bytes / data segments), at least 1: RS segments = ranks - k
    (src/redset_reedsolomon.c:485-493), XOR segments = ranks - 1
    (src/redset_xor.c:358-370)."""
    seg = ranks - (encoding if scheme == "RS" else 1)
    if seg < 1:
        raise ValueError(f"too few ranks ({ranks}) for {scheme} with {encoding} encoding blocks")
    c = max_bytes // seg
    if c * seg < max_bytes:
        c += 1
    return max(1, c)


def header_tree(scheme: str, rank: int, members: Sequence[Tree], world_ranks: Sequence[int],
                chunk: int, encoding: int = 1) -> Tree:
    """Member ``rank``'s header: its own hash and its left neighbours' under
    DESC <member> (RS: k neighbours, src/redset_reedsolomon.c:453-474; XOR:
    one, src/redset_xor.c:337-348), GROUP map, CHUNK, RANK."""
    p = len(members)
    left = encoding if scheme == "RS" else 1
    h: Tree = {}
    set_kv(h, "RANK", rank)
    desc: Tree = {str(rank): copy(members[rank])}
    for i in range(1, left + 1):
        lhs = (rank - i + p) % p
        desc[str(lhs)] = copy(members[lhs])
    h["DESC"] = desc
    merge(h, group_map(world_ranks))
    set_kv(h, "CHUNK", chunk)
    return h


def redundancy_filename(scheme: str, prefix: str, world_rank: int, group_id: int, groups: int,
                        rank: int, ranks: int) -> str:
    """<prefix><rank>.<rs|xor>.grp_<g+1>_of_<G>.mem_<r+1>_of_<p>.redset
    (src/redset_reedsolomon.c:34-44, src/redset_xor.c:45-55)."""
    kind = "rs" if scheme == "RS" else "xor"
    return f"{prefix}{world_rank}.{kind}.grp_{group_id + 1}_of_{groups}.mem_{rank + 1}_of_{ranks}.redset"


# ------------------------------------------------ set facts from the headers

@dataclass
class SetFacts:
    """What the single-process rebuild learns from the headers it can read
    (src/redset_reedsolomon_serial.c:355-500, src/redset_xor_serial.c)."""
    scheme: str
    ranks: int
    encoding: int
    chunk: int
    world_ranks: List[int]
    members: List[Tree]                      # every member's current_hash
    have_header: List[bool]                  # member's redundancy file read
    header_size: Dict[int, int] = field(default_factory=dict)

    def files(self, r: int) -> List[Tuple[str, int]]:
        """Member r's data files in logical-file order: (path, SIZE)."""
        m = self.members[r]
        n = get_int(m, "FILES")
        out = []
        for i in range(n):
            (path, meta), = m["FILE"][str(i)].items()
            out.append((path, get_int(meta, "SIZE")))
        return out

    def descriptor(self, r: int) -> Tree:
        return self.members[r]["DESC"]


def set_facts(headers: Sequence[Tuple[Tree, int]]) -> SetFacts:
    """Collect the set from any readable headers, as the serial rebuild does:
    ranks / CHUNK / CKSUM / GROUP from the first header, each member's hash
    from whichever header carries it (its own, or a right neighbour's copy).
    Raises when no header was readable or some member's hash is in none
    (src/redset_reedsolomon_serial.c:436-466)."""
    first = None
    got: Dict[int, Tree] = {}
    have: Dict[int, int] = {}
    for h, size in headers:
        if first is None:
            first = h
        r = get_int(h, "RANK")
        have[r] = size
        for k, mh in h.get("DESC", {}).items():
            got.setdefault(int(k), copy(mh))
    if first is None:
        raise ValueError("no readable redundancy-file header")
    g = first["GROUP"]
    ranks = get_int(g, "RANKS")
    world = [int(get_kv(g["RANK"], str(i))) for i in range(ranks)]
    me = get_int(first, "RANK")
    d = first["DESC"][str(me)]["DESC"]
    scheme = get_kv(d, "TYPE")
    encoding = get_int(d, "CKSUM") if scheme == "RS" else 1
    lost = [i for i in range(ranks) if i not in got]
    if lost:
        raise ValueError(f"no header carries the file list of member(s) {lost}")
    return SetFacts(scheme, ranks, encoding, get_int(first, "CHUNK"), world,
                    [got[i] for i in range(ranks)], [i in have for i in range(ranks)], have)
