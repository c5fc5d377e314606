"""Multi-GPU encode / rebuild of redundancy sets spread over the GPUs of a node.

Replaces the reference's MPI rings (encode: src/redset_reedsolomon.c:346-363;
decode reduce + gather: :690-733) with one all-to-all gather of cell column
slices over RCCL/xGMI, a local gf_mac pass on each GPU's column slice of
every stripe, and one exchange that returns the result slices to their owners.

World layout (weak scaling): ``world`` sets of ``p`` members; member m of the
world (set m // p, index m % p) lives on GPU m % world, so every GPU hosts p
members and a set's members spread over the GPUs. Every cell is cut into
``world`` column slices of ``W`` bytes; GPU g computes slice g of every stripe
of every set. Byte j of a parity/rebuilt cell depends only on byte j of its
stripe's inputs, so the slices are independent.

HBM layout per GPU (so each exchange is one contiguous all-to-all):
  hosted data   D_host[g][j][s][W]  slice g of data cell s of hosted member j
  hosted parity P_host[g][j][i][W]  slice g of parity cell i of hosted member j
  gathered      D_gath[h][j][s][W]  my slice of data cell s of member j hosted on h
                P_gath[h][j][i][W]  my slice of parity cell i of that member
A member's logical file is therefore stored as `world` column slabs; the
single-GPU path (bench N=1) keeps cells contiguous.

The compute backend is pluggable so the exchange logic can be tested with
gloo on CPU (tests/test_dist.py injects a CPU checker backend); the default
backend is the HIP library.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

SLICE_ALIGN = 256


@dataclass
class SetViews:
    """Per-member base tensors of one set in a gathered layout (stride W)."""

    lofi: List[torch.Tensor]    # member r: d cells of W bytes, contiguous
    parity: List[torch.Tensor]  # member r: e cells of W bytes


class HipBackend:
    """Default compute: the HIP plans of redset_amd (gf_mac kernel)."""

    def __init__(self, p: int, e: int):
        from . import codec

        self.codec = codec.RSCodec(p, e)

    def prepare_encode(self, views: SetViews, nbytes: int, stride: int) -> Callable[[], None]:
        plan = self.codec.plan_encode([t.data_ptr() for t in views.lofi], [t.data_ptr() for t in views.parity],
                                      nbytes, stride)
        return lambda: plan.execute()

    def prepare_rebuild(self, views: SetViews, lost: Sequence[int], nbytes: int, stride: int) -> Callable[[], None]:
        plan = self.codec.plan_rebuild(list(lost), [t.data_ptr() for t in views.lofi],
                                       [t.data_ptr() for t in views.parity], nbytes, stride)
        return lambda: plan.execute()


def rebuild_inputs(p: int, e: int, lost: Sequence[int]) -> Tuple[np.ndarray, np.ndarray]:
    """Which cells of each surviving member some stripe's decode reads.

    Returns (data[p][d], parity[p][e]) boolean masks. A stripe's decode
    (redset_rs_reduce_decode + redset_rs_gaussian_solve as one linear map,
    redset_hip_rs_decode_matrix) reads the stripe's surviving data cells and
    the parity rows redset_rs_gaussian_solve_identify_rows selects
    (src/redset_reedsolomon_common.c:425-564); the parity rows it leaves out
    never have to cross the fabric. Member s's cell in stripe c is data cell
    get_data_id(s, c) when get_encoding_id(s, c) < p, else parity slot
    get_encoding_id(s, c) - p (src/redset_reedsolomon_common.c:822-853)."""
    from .codec import RSCodec

    d = p - e
    need_d = np.zeros((p, d), dtype=bool)
    need_p = np.zeros((p, e), dtype=bool)
    if not lost:
        return need_d, need_p
    codec = RSCodec(p, e)
    for c in range(p):
        M = codec.decode_matrix(list(lost), c)
        for s in range(p):
            if s in lost or not M[:, s].any():
                continue
            enc = codec.encoding_id(s, c)
            if enc < p:
                need_d[s, codec.data_id(s, c)] = True
            else:
                need_p[s, enc - p] = True
    codec.close()
    return need_d, need_p


def _runs(flags: Sequence[bool]) -> List[Tuple[int, int]]:
    """[a, b) index ranges of the True entries"""
    out, a = [], None
    for i, f in enumerate(list(flags) + [False]):
        if f and a is None:
            a = i
        elif not f and a is not None:
            out.append((a, i))
            a = None
    return out


class ShardedSetRunner:
    """Encode + rebuild of `world` sets column-sharded over `world` ranks."""

    def __init__(self, p: int, e: int, chunk: int, lost: Sequence[int], world: int, rank: int,
                 device=None, backend=None, seed: int = 1234, fill: bool = True):
        self.p, self.e, self.d = p, e, p - e
        self.chunk, self.world, self.rank = chunk, world, rank
        self.lost = sorted(lost)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        W = -(-chunk // world)
        self.W = -(-W // SLICE_ALIGN) * SLICE_ALIGN
        # bytes of my column slice of each cell (the last slice may be short)
        self.my_len = self.slice_len(rank)
        self.backend = backend if backend is not None else HipBackend(p, e)
        self._place()
        self.timing = self.device.type == "cuda"
        self._events = []
        self._gather_ops = None
        self._return_ops = None
        d, W, ph = self.d, self.W, p  # every GPU hosts p members
        u8 = dict(dtype=torch.uint8, device=self.device)
        self.D_host = torch.zeros(world, ph, d, W, **u8)
        self.P_host = torch.zeros(world, ph, e, W, **u8)
        self.D_gath = torch.zeros(world, ph, d, W, **u8)
        self.P_gath = torch.zeros(world, ph, e, W, **u8)
        if fill:
            g = torch.Generator(device=self.device)
            g.manual_seed(seed + rank)
            self.D_host.copy_(torch.randint(0, 256, self.D_host.shape, generator=g, **u8))
        # my slice of every stripe of every set, as per-set views
        self._encode, self._rebuild = [], []
        for k in range(world):
            views = self.set_views(k)
            if self.my_len > 0:
                self._encode.append(self.backend.prepare_encode(views, self.my_len, W))
                if self.lost:
                    self._rebuild.append(self.backend.prepare_rebuild(views, self.lost, self.my_len, W))

    # ---- placement -------------------------------------------------------
    def _place(self) -> None:
        """member m of the world (set m // p, index m % p) lives on GPU
        m % world; each GPU lists its hosted members with the lost ones last,
        so an exchange can skip them with contiguous views."""
        self._where = {}
        self.n_alive = []
        self._hosted = []
        for g in range(self.world):
            mine = [m for m in range(self.world * self.p) if m % self.world == g]
            alive = [m for m in mine if (m % self.p) not in self.lost]
            dead = [m for m in mine if (m % self.p) in self.lost]
            for j, m in enumerate(alive + dead):
                self._where[m] = (g, j)
            self.n_alive.append(len(alive))
            self._hosted.append(alive + dead)

    def host_of(self, k: int, r: int):
        """(GPU, hosted index) of member r of set k."""
        return self._where[k * self.p + r]

    def set_views(self, k: int) -> SetViews:
        lofi, parity = [], []
        for r in range(self.p):
            h, j = self.host_of(k, r)
            lofi.append(self.D_gath[h, j].view(-1))
            parity.append(self.P_gath[h, j].view(-1))
        return SetViews(lofi, parity)

    # ---- exchanges -------------------------------------------------------
    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """out[h] <- inp[me] of rank h, for every h (encode: every cell)."""
        if self.world == 1:
            out.copy_(inp)
            return
        dist.all_to_all_single(out, inp)

    def _build_rebuild_gather(self) -> None:
        """The rebuild's gather as one batch of P2P ops: my column slice of
        every cell some decode reads (rebuild_inputs), from every survivor's
        host. Lost members are hosted last and never sent; parity rows no
        decode selects stay home. Cells are flattened per GPU as
        (hosted member, cell), so neighbouring needed cells merge into one op."""
        p, d, e, W, me = self.p, self.d, self.e, self.W, self.rank
        need_d, need_p = rebuild_inputs(p, e, self.lost)

        def runs(h):
            alive = self._hosted[h][:self.n_alive[h]]
            fd = [bool(need_d[m % p, s]) for m in alive for s in range(d)]
            fp = [bool(need_p[m % p, i]) for m in alive for i in range(e)]
            return _runs(fd), _runs(fp)

        def rows(t, g):  # GPU g's slab of t as [hosted member * cell, W]
            return t[g].view(-1, W)

        self._gather_local = []
        self._gather_ops = []
        self._gather_sent = 0
        my_d, my_p = runs(me)
        for a, b in my_d:
            self._gather_local.append((rows(self.D_gath, me)[a:b], rows(self.D_host, me)[a:b]))
        for a, b in my_p:
            self._gather_local.append((rows(self.P_gath, me)[a:b], rows(self.P_host, me)[a:b]))
        for g in range(self.world):
            if g == me:
                continue
            for a, b in my_d:
                self._gather_ops.append(dist.P2POp(dist.isend, rows(self.D_host, g)[a:b], g))
                self._gather_sent += (b - a) * W
            for a, b in my_p:
                self._gather_ops.append(dist.P2POp(dist.isend, rows(self.P_host, g)[a:b], g))
                self._gather_sent += (b - a) * W
            their_d, their_p = runs(g)
            for a, b in their_d:
                self._gather_ops.append(dist.P2POp(dist.irecv, rows(self.D_gath, g)[a:b], g))
            for a, b in their_p:
                self._gather_ops.append(dist.P2POp(dist.irecv, rows(self.P_gath, g)[a:b], g))

    def _gather_rebuild_inputs(self) -> None:
        if self._gather_ops is None:
            self._build_rebuild_gather()
        for dst, src in self._gather_local:
            dst.copy_(src)
        if self._gather_ops:
            for req in dist.batch_isend_irecv(self._gather_ops):
                req.wait()

    def _mark(self, name: str) -> None:
        if self.timing:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._events.append((name, ev))

    def _build_return(self) -> None:
        """Rebuilt slices of lost members go to their hosts (the reference's
        gather to the failed ranks, src/redset_reedsolomon.c:713-733): my own
        slice is a local copy, the others arrive from their peers."""
        self._return_local, self._return_ops, self._return_sent = [], [], 0
        for k in range(self.world):
            for r in self.lost:
                h, j = self.host_of(k, r)
                if h == self.rank:
                    self._return_local.append((self.D_host[self.rank, j], self.D_gath[h, j]))
                    self._return_local.append((self.P_host[self.rank, j], self.P_gath[h, j]))
                    for g in range(self.world):
                        if g != self.rank:
                            self._return_ops.append(dist.P2POp(dist.irecv, self.D_host[g, j], g))
                            self._return_ops.append(dist.P2POp(dist.irecv, self.P_host[g, j], g))
                else:
                    self._return_ops.append(dist.P2POp(dist.isend, self.D_gath[h, j], h))
                    self._return_ops.append(dist.P2POp(dist.isend, self.P_gath[h, j], h))
                    self._return_sent += self.D_gath[h, j].numel() + self.P_gath[h, j].numel()

    def _return_lost(self) -> None:
        if self._return_ops is None:
            self._build_return()
        for dst, src in self._return_local:
            dst.copy_(src)
        if self._return_ops:
            for req in dist.batch_isend_irecv(self._return_ops):
                req.wait()

    # ---- operations ------------------------------------------------------
    def encode(self) -> None:
        """Parity of every stripe of every set: gather data slices, compute my
        column slice, return parity slices to their hosts."""
        self._mark("encode_start")
        self._all_to_all(self.D_gath, self.D_host)
        self._mark("encode_gathered")
        for fn in self._encode:
            fn()
        self._mark("encode_computed")
        self._all_to_all(self.P_host, self.P_gath)
        self._mark("encode_done")

    def erase(self) -> None:
        """Model the loss of the lost members' files on their hosts."""
        for k in range(self.world):
            for r in self.lost:
                h, j = self.host_of(k, r)
                if h == self.rank:
                    self.D_host[:, j].zero_()
                    self.P_host[:, j].zero_()

    def rebuild(self) -> None:
        """Rebuild the lost members of every set from the survivors."""
        self._mark("rebuild_start")
        self._gather_rebuild_inputs()
        self._mark("rebuild_gathered")
        for fn in self._rebuild:
            fn()
        self._mark("rebuild_computed")
        self._return_lost()
        self._mark("rebuild_done")

    def step(self) -> None:
        self.encode()
        self.rebuild()

    # ---- verification --------------------------------------------------
    def lost_snapshot(self) -> List[Tuple[int, torch.Tensor, torch.Tensor]]:
        """Copies of this GPU's hosted slabs of the members `erase` destroys."""
        snap = []
        for k in range(self.world):
            for r in self.lost:
                h, j = self.host_of(k, r)
                if h == self.rank:
                    snap.append((j, self.D_host[:, j].clone(), self.P_host[:, j].clone()))
        return snap

    def slice_len(self, g: int) -> int:
        """Bytes of cell column slice g that are cell bytes (the rest of the
        last slice's W is padding)."""
        return max(0, min(self.chunk, (g + 1) * self.W) - g * self.W)

    def matches(self, snap) -> bool:
        """Every cell byte of the hosted slabs in `snap` is back, bit for bit."""
        for j, dd, pp in snap:
            for g in range(self.world):
                n = self.slice_len(g)
                if not (torch.equal(self.D_host[g, j, :, :n], dd[g, :, :n])
                        and torch.equal(self.P_host[g, j, :, :n], pp[g, :, :n])):
                    return False
        return True

    # ---- accounting ------------------------------------------------------
    def algorithmic_bytes(self, op: str = "step") -> int:
        """Per-GPU algorithmic bytes (one set's worth, p stripes): encode
        (d+e)*C per stripe, rebuild (d+m)*C per stripe;
        "step" = both."""
        p, d, e, m, C = self.p, self.d, self.e, len(self.lost), self.chunk
        enc = p * (d + e) * C
        reb = p * (d + m) * C if m else 0
        return {"encode": enc, "rebuild": reb, "step": enc + reb}[op]

    def exchanged_bytes(self, op: str = "step") -> int:
        """Bytes this GPU sends over the fabric per operation."""
        if self.world == 1:
            return 0
        if self._gather_ops is None:
            self._build_rebuild_gather()
        if self._return_ops is None:
            self._build_return()
        enc = (self.world - 1) * (self.D_host[0].numel() + self.P_host[0].numel())
        reb = self._gather_sent + self._return_sent
        return {"encode": enc, "rebuild": reb, "step": enc + reb}[op]

    def phase_ms(self) -> dict:
        """Mean milliseconds per phase over the steps marked so far."""
        torch.cuda.synchronize()
        acc, n = {}, {}
        ev = self._events
        for (a, ea), (b, eb) in zip(ev, ev[1:]):
            if a.split("_")[0] != b.split("_")[0] or a.endswith("_done"):
                continue
            key = f"{a}->{b.split('_', 1)[1]}"
            acc[key] = acc.get(key, 0.0) + ea.elapsed_time(eb)
            n[key] = n.get(key, 0) + 1
        return {k: round(acc[k] / n[k], 3) for k in acc}

    def reset_timing(self) -> None:
        self._events = []

    def report(self, step_seconds: float, op: str = "step") -> dict:
        coll = {"encode": "RCCL all_to_all (data slices, then parity slices)",
                "rebuild": "batched RCCL P2P: decode inputs' slices in, rebuilt slices back to their hosts"}
        phases = self.phase_ms() if self.timing else None
        out = {
            "exchange": {
                "bytes_sent_per_gpu_per_step": self.exchanged_bytes(op),
                "column_slice_bytes": self.W,
                "collective": coll.get(op, coll["encode"] + "; " + coll["rebuild"]),
                "phase_ms_rank0": phases,
            },
            "per_gpu_GBps": round(self.algorithmic_bytes(op) / step_seconds / 1e9, 2),
        }
        if phases and op == "rebuild" and self.world > 1:
            # rank 0's send rate over the fabric in each exchange phase (what
            # bounds the sharded rebuild; compare with xGMI, 7 links per GPU)
            if self._gather_ops is None:
                self._build_rebuild_gather()
            if self._return_ops is None:
                self._build_return()
            g_ms = phases.get("rebuild_start->gathered")
            r_ms = phases.get("rebuild_computed->done")
            out["exchange"]["gather_send_GBps_rank0"] = (round(self._gather_sent / (g_ms * 1e-3) / 1e9, 1)
                                                         if g_ms else None)
            out["exchange"]["return_send_GBps_rank0"] = (round(self._return_sent / (r_ms * 1e-3) / 1e9, 1)
                                                         if r_ms and self._return_sent else None)
        return out
