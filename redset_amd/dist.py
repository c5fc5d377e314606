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
from typing import Callable, List, Sequence

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
        self.my_len = max(0, min(chunk, (rank + 1) * self.W) - rank * self.W)
        self.backend = backend if backend is not None else HipBackend(p, e)
        self._place()
        self.timing = self.device.type == "cuda"
        self._events = []
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
        for g in range(self.world):
            mine = [m for m in range(self.world * self.p) if m % self.world == g]
            alive = [m for m in mine if (m % self.p) not in self.lost]
            dead = [m for m in mine if (m % self.p) in self.lost]
            for j, m in enumerate(alive + dead):
                self._where[m] = (g, j)
            self.n_alive.append(len(alive))

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
    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor, skip_lost: bool = False) -> None:
        """out[h] <- inp[me] of rank h, for every h. With skip_lost, the lost
        members (hosted last, see host_of) are not sent: their cells are gone."""
        if self.world == 1:
            out.copy_(inp)
            return
        if not skip_lost or not self.lost:
            dist.all_to_all_single(out, inp)
            return
        # uneven all-to-all as one batch of P2P ops (gloo has no uneven
        # all_to_all; RCCL groups the batch into one launch)
        me, n_send = self.rank, self.n_alive[self.rank]
        out[me, :n_send].copy_(inp[me, :n_send])
        ops = []
        for g in range(self.world):
            if g != me:
                ops.append(dist.P2POp(dist.isend, inp[g, :n_send], g))
                ops.append(dist.P2POp(dist.irecv, out[g, :self.n_alive[g]], g))
        for req in dist.batch_isend_irecv(ops):
            req.wait()

    def _mark(self, name: str) -> None:
        if self.timing:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._events.append((name, ev))

    def _return_lost(self) -> None:
        """Send rebuilt slices of lost members to their hosts (the reference's
        gather to the failed ranks, src/redset_reedsolomon.c:713-733)."""
        ops = []
        for k in range(self.world):
            for r in self.lost:
                h, j = self.host_of(k, r)
                if h == self.rank:
                    # my own slice: local copy; other slices arrive from peers
                    self.D_host[self.rank, j].copy_(self.D_gath[h, j])
                    self.P_host[self.rank, j].copy_(self.P_gath[h, j])
                    for g in range(self.world):
                        if g != self.rank:
                            ops.append(dist.P2POp(dist.irecv, self.D_host[g, j], g))
                            ops.append(dist.P2POp(dist.irecv, self.P_host[g, j], g))
                else:
                    ops.append(dist.P2POp(dist.isend, self.D_gath[h, j], h))
                    ops.append(dist.P2POp(dist.isend, self.P_gath[h, j], h))
        if ops:
            for req in dist.batch_isend_irecv(ops):
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
        self._all_to_all(self.D_gath, self.D_host, skip_lost=True)
        self._all_to_all(self.P_gath, self.P_host, skip_lost=True)
        self._mark("rebuild_gathered")
        for fn in self._rebuild:
            fn()
        self._mark("rebuild_computed")
        self._return_lost()
        self._mark("rebuild_done")

    def step(self) -> None:
        self.encode()
        self.rebuild()

    # ---- accounting ------------------------------------------------------
    @property
    def algorithmic_bytes(self) -> int:
        """Per-GPU algorithmic bytes of one step (one set's worth: encode
        (d+e)*C per stripe + rebuild (d+m)*C per stripe, p stripes)."""
        p, d, e, m, C = self.p, self.d, self.e, len(self.lost), self.chunk
        return p * (d + e) * C + (p * (d + m) * C if m else 0)

    @property
    def exchanged_bytes(self) -> int:
        """Bytes this GPU sends per step over the fabric (average GPU)."""
        if self.world == 1:
            return 0
        frac = (self.world - 1) / self.world
        p, d, e, C, m = self.p, self.d, self.e, self.chunk, len(self.lost)
        enc = (p * d + p * e) * C * frac
        reb = ((p - m) * (d + e) + m * (d + e)) * C * frac
        return int(enc + reb)

    def phase_ms(self) -> dict:
        """Mean milliseconds per phase over the steps marked so far."""
        torch.cuda.synchronize()
        acc, n = {}, {}
        ev = self._events
        for (a, ea), (b, eb) in zip(ev, ev[1:]):
            if a.split("_")[0] != b.split("_")[0]:
                continue
            key = f"{a}->{b.split('_', 1)[1]}"
            acc[key] = acc.get(key, 0.0) + ea.elapsed_time(eb)
            n[key] = n.get(key, 0) + 1
        return {k: round(acc[k] / n[k], 3) for k in acc}

    def reset_timing(self) -> None:
        self._events = []

    def report(self, step_seconds: float) -> dict:
        return {
            "exchange": {
                "bytes_sent_per_gpu_per_step": self.exchanged_bytes,
                "column_slice_bytes": self.W,
                "collective": "RCCL all_to_all (data / parity slices) + batched P2P (rebuilt slices)",
                "phase_ms_rank0": self.phase_ms() if self.timing else None,
            },
            "per_gpu_GBps": round(self.algorithmic_bytes / step_seconds / 1e9, 2),
        }
