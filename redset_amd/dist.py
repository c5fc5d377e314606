"""Multi-GPU encode / rebuild of redundancy sets spread over the GPUs of a node.

A thin Python face of the C ABI's sharded path (include/redset_hip.h, "sets
sharded over the GPUs of a node"; redset_amd/csrc/sharded.c): the C library
plans which column slices go where, runs the exchanges through a transport
and the gf_mac kernel on this GPU's slice of every stripe. This module only
chooses the placement, allocates the slabs (torch tensors in HBM) and picks
the transport: RCCL over xGMI (redset_hip_rccl_*, the production path), or,
for CPU tests, a callback transport over torch.distributed (gloo).

Replaces the reference's MPI rings (encode: src/redset_reedsolomon.c:329-377;
decode reduce + gather: :646-733) with one grouped gather of cell column
slices, a local gf_mac pass, and one grouped return.

World layout (weak scaling): ``world`` sets of ``p`` members; member m of the
world (set m // p, index m % p) lives on GPU m % world, so every GPU hosts p
members and a set's members spread over the GPUs. Each GPU lists its hosted
members with the lost ones last. Every cell is cut into ``world`` column
slices of ``W`` bytes; GPU g computes slice g of every stripe of every set.

HBM layout per GPU (include/redset_hip.h):
  hosted data   D_host[q][j][s][W]  slice q of data cell s of hosted member j
  hosted parity P_host[q][j][i][W]  slice q of parity cell i of hosted member j
  gathered      D_gath[h][j][s][W]  my slice of data cell s of member j hosted on h
                P_gath[h][j][i][W]  my slice of parity cell i of that member
"""
from __future__ import annotations

import ctypes
from ctypes import c_int, c_ubyte, c_void_p
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def rebuild_inputs(p: int, e: int, lost: Sequence[int]) -> Tuple[np.ndarray, np.ndarray]:
    """Which cells of each surviving member some stripe's decode reads.

    Returns (data[p][d], parity[p][e]) boolean masks (a cross-check of the C
    planner's gather, tests/test_dist.py). A stripe's decode
    (redset_rs_reduce_decode + redset_rs_gaussian_solve as one linear map,
    redset_hip_rs_decode_matrix) reads the stripe's surviving data cells and
    the parity rows redset_rs_gaussian_solve_identify_rows selects
    (src/redset_reedsolomon_common.c:425-564). Member s's cell in stripe c is
    data cell get_data_id(s, c) when get_encoding_id(s, c) < p, else parity
    slot get_encoding_id(s, c) - p (src/redset_reedsolomon_common.c:822-853)."""
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


class _Buffers:
    """Address -> tensor view over the runner's four slabs, for callbacks."""

    def __init__(self, tensors):
        self.spans = sorted((t.data_ptr(), t.data_ptr() + t.numel(), t.view(-1)) for t in tensors)

    def view(self, addr: int, n: int) -> torch.Tensor:
        for lo, hi, flat in self.spans:
            if lo <= addr and addr + n <= hi:
                return flat[addr - lo: addr - lo + n]
        raise ValueError(f"address {addr:#x}+{n} is outside the sharded buffers")


class TorchTransport:
    """redset_hip_transport over torch.distributed point-to-point
    (batch_isend_irecv): for gloo runs on CPU; the C planner is unchanged."""

    def __init__(self, world: int, rank: int, bufs: _Buffers):
        self.bufs = bufs
        self._fn = _lib.EXCHANGE_FN(self._exchange)
        self.struct = _lib.Transport(world, rank, ctypes.cast(self._fn, c_void_p), None)
        self.rank = rank

    def _exchange(self, ctx, xfers, n, stream) -> int:
        try:
            ops = []
            i = 0
            while i < n:
                x = xfers[i]
                if x.peer == self.rank:  # local copy: source, then destination
                    y = xfers[i + 1]
                    self.bufs.view(y.buf, y.len).copy_(self.bufs.view(x.buf, x.len))
                    i += 2
                    continue
                t = self.bufs.view(x.buf, x.len)
                ops.append(dist.P2POp(dist.isend if x.send else dist.irecv, t, x.peer))
                i += 1
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            return 0
        except Exception as exc:  # noqa: BLE001 -- reported through the C error path
            _lib.load().redset_hip_record_error(f"torch transport: {exc}".encode())
            return 1

    def close(self):
        pass


class RcclTransport:
    """redset_hip_rccl_*: grouped ncclSend / ncclRecv over xGMI. Rank 0's
    unique id reaches the others through the torch process group (any
    channel would do)."""

    def __init__(self, world: int, rank: int):
        L = _lib.load()
        uid = (c_ubyte * 128)()
        if rank == 0:
            _lib.check(L.redset_hip_rccl_unique_id(uid), "rccl_unique_id")
        if world > 1:
            t = torch.tensor(list(bytes(uid)), dtype=torch.uint8,
                             device="cuda" if dist.get_backend() == "nccl" else "cpu")
            dist.broadcast(t, src=0)
            uid = (c_ubyte * 128)(*t.cpu().tolist())
        self.struct = _lib.Transport()
        h = c_void_p()
        _lib.check(L.redset_hip_rccl_transport_create(uid, world, rank, ctypes.byref(self.struct), ctypes.byref(h)),
                   "rccl_transport_create")
        self._h = h

    def close(self):
        if self._h:
            _lib.load().redset_hip_rccl_transport_destroy(self._h)
            self._h = None


class CallbackCompute:
    """redset_hip_compute over a Python backend with
    ``run(kind, lost, lofi_views, parity_views, nbytes, stride)`` (tests put
    the CPU oracle here), and, if the backend has
    ``combine(jobs, nbytes, bufs)`` with jobs as (input addresses, output
    addresses, nout x nin coefficients, accumulate), the partial-sum shape's
    combine callback too."""

    def __init__(self, backend, p: int, bufs: _Buffers):
        self.backend, self.p, self.bufs = backend, p, bufs
        self._fn = _lib.COMPUTE_FN(self._run)
        self.struct = _lib.Compute(ctypes.cast(self._fn, c_void_p), None)
        self._cfn = _lib.COMBINE_FN(self._combine) if hasattr(backend, "combine") else None

    @property
    def combine_ptr(self):
        return ctypes.cast(self._cfn, c_void_p) if self._cfn is not None else None

    def _combine(self, ctx, jobs, njobs, nbytes, stream) -> int:
        try:
            lst = []
            for k in range(njobs):
                J = jobs[k]
                ins = [J.inp[i] for i in range(J.nin)]
                outs = [J.out[j] for j in range(J.nout)]
                coef = np.ctypeslib.as_array(J.coef, shape=(J.nout * J.nin,)).reshape(J.nout, J.nin).copy()
                lst.append((ins, outs, coef, bool(J.accumulate)))
            self.backend.combine(lst, nbytes, self.bufs)
            return 0
        except Exception as exc:  # noqa: BLE001
            _lib.load().redset_hip_record_error(f"combine callback: {exc}".encode())
            return 1

    def _run(self, ctx, kind, missing, ranks, lofi, parity, nbytes, stride, stream) -> int:
        try:
            lost = [ranks[i] for i in range(missing)]
            lv = [lofi[r] for r in range(self.p)]
            pv = [parity[r] for r in range(self.p)]
            self.backend.run(kind, lost, lv, pv, nbytes, stride, self.bufs)
            return 0
        except Exception as exc:  # noqa: BLE001
            _lib.load().redset_hip_record_error(f"compute callback: {exc}".encode())
            return 1


class ShardedSetRunner:
    """Encode + rebuild of `sets` sets (default `world`: weak scaling, one
    set's worth of work per GPU) column-sharded over `world` ranks; sets = 1
    spreads one set over all of them (strong scaling, BASELINE.md's C4)."""

    def __init__(self, p: int, e: int, chunk: int, lost: Sequence[int], world: int, rank: int,
                 device=None, backend=None, seed: int = 1234, fill: bool = True, transport: Optional[str] = None,
                 parity_gap: Optional[int] = 0, sets: Optional[int] = None, shape: str = "auto"):
        self.p, self.e, self.d = p, e, p - e
        self.chunk, self.world, self.rank = chunk, world, rank
        self.nsets = world if sets is None else sets
        self.lost = sorted(lost)
        # the exchange's shape (include/redset_hip.h REDSET_HIP_SHAPE_*):
        # "auto" lets the planner take whichever moves fewer bytes through
        # the busiest GPU -- gathering column slices of the inputs, or
        # sending partial sums of each GPU's own inputs to the outputs' hosts
        # (one name for both plans, or an (encode, rebuild) pair)
        names = {"auto": _lib.SHAPE_AUTO, "gather": _lib.SHAPE_GATHER, "reduce": _lib.SHAPE_REDUCE}
        enc_s, reb_s = (shape, shape) if isinstance(shape, str) else shape
        self.shape_req = {_lib.PLAN_RS_ENCODE: names[enc_s], _lib.PLAN_RS_REBUILD: names[reb_s]}
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        L = _lib.load()
        self.W = int(L.redset_hip_shard_slice_bytes(chunk, world))
        if world == 1:
            # one process: no slice crosses a link, so the slab pitch can carry
            # the library's cell pad (redset_hip_cell_stride: 64 MiB cells
            # otherwise start at equal addresses modulo 2^26 and crowd the
            # same DRAM channels, the whole-set plans' 2% lesson)
            self.W = int(L.redset_hip_cell_stride(chunk))
        self.my_len = self.slice_len(rank)
        self._place()
        self.timing = self.device.type == "cuda"
        self.phased = False
        self._events = []
        # members per GPU: p when there are `world` sets
        d, W, mh = self.d, self.W, -(-self.nsets * p // world)
        u8 = dict(dtype=torch.uint8, device=self.device)
        if parity_gap is None:
            self.D_host = torch.zeros(world, mh, d, W, **u8)
            self.P_host = torch.zeros(world, mh, e, W, **u8)
        else:
            # the hosted slabs as one allocation, parity `parity_gap` bytes
            # after the data (None: two allocations, as the allocator places
            # them). At N = 1 the rebuild runs over these slabs in place, and
            # as two allocations its rate depended on where they landed:
            # 6.01-6.44 TB/s, against 6.33-6.40 for one allocation at any gap
            # (profiles/r05s18_*, r05s19_placement.json)
            nd, npar = world * mh * d * W, world * mh * e * W
            self._hosted_buf = torch.zeros(nd + parity_gap + npar, **u8)
            self.D_host = self._hosted_buf[:nd].view(world, mh, d, W)
            self.P_host = self._hosted_buf[nd + parity_gap:].view(world, mh, e, W)
        self.D_gath = torch.zeros(world, mh, d, W, **u8)
        self.P_gath = torch.zeros(world, mh, e, W, **u8)
        if fill:
            g = torch.Generator(device=self.device)
            g.manual_seed(seed + rank)
            self.D_host.copy_(torch.randint(0, 256, self.D_host.shape, generator=g, **u8))
        self._bufs = _Buffers([self.D_host, self.P_host, self.D_gath, self.P_gath])
        if transport is None:
            transport = "rccl" if self.device.type == "cuda" and (world == 1 or dist.get_backend() == "nccl") \
                else "torch"
        self._transport = RcclTransport(world, rank) if transport == "rccl" else \
            TorchTransport(world, rank, self._bufs)
        self._compute = CallbackCompute(backend, p, self._bufs) if backend is not None else None
        self._codec_h = c_void_p()
        _lib.check(L.redset_hip_rs_create(p, e, ctypes.byref(self._codec_h)), "rs_create")
        nm = self.nsets * p
        self._host_arr = (c_int * nm)(*[self._where[m][0] for m in range(nm)])
        self._slot_arr = (c_int * nm)(*[self._where[m][1] for m in range(nm)])
        self._layout = _lib.ShardLayout(self.nsets, self._host_arr, self._slot_arr, mh, chunk, W,
                                        self.D_host.data_ptr(), self.P_host.data_ptr(),
                                        self.D_gath.data_ptr(), self.P_gath.data_ptr())
        self._plans = {"encode": self._plan(_lib.PLAN_RS_ENCODE, [])}
        if self.lost:
            self._plans["rebuild"] = self._plan(_lib.PLAN_RS_REBUILD, self.lost)

    def _plan(self, kind: int, lost: List[int]) -> c_void_p:
        L = _lib.load()
        arr = (c_int * max(1, len(lost)))(*lost)
        h = c_void_p()
        opts = _lib.ShardedOpts()
        opts.struct_size = ctypes.sizeof(_lib.ShardedOpts)
        opts.shape = self.shape_req[kind]
        if self._compute is not None:
            opts.compute = ctypes.pointer(self._compute.struct)
            opts.combine = self._compute.combine_ptr
        _lib.check(L.redset_hip_rs_sharded_plan_ex(self._codec_h, kind, len(lost), arr, ctypes.byref(self._layout),
                                                   ctypes.byref(self._transport.struct), ctypes.byref(opts),
                                                   ctypes.byref(h)),
                   "rs_sharded_plan_ex")
        return h

    def info(self, op: str) -> dict:
        inf = _lib.ShardedInfo()
        _lib.check(_lib.load().redset_hip_sharded_get_info(self._plans[op], ctypes.byref(inf)), "sharded_get_info")
        return inf.as_dict()

    def shape(self, op: str) -> dict:
        """The planned shape and both shapes' byte counts (redset_hip_sharded_get_shape)."""
        si = _lib.ShapeInfo()
        _lib.check(_lib.load().redset_hip_sharded_get_shape(self._plans[op], ctypes.byref(si), ctypes.sizeof(si)),
                   "sharded_get_shape")
        return si.as_dict()

    def close(self):
        L = _lib.load()
        for h in self._plans.values():
            L.redset_hip_sharded_destroy(h)
        self._plans = {}
        self._transport.close()
        if self._codec_h:
            L.redset_hip_rs_destroy(self._codec_h)
            self._codec_h = None

    # ---- placement -------------------------------------------------------
    def _place(self) -> None:
        """member m of the world (set m // p, index m % p) lives on GPU
        m % world; each GPU lists its hosted members with the lost ones last,
        so an exchange can skip them with contiguous views."""
        self._where = {}
        self.n_alive = []
        self._hosted = []
        for g in range(self.world):
            mine = [m for m in range(self.nsets * self.p) if m % self.world == g]
            alive = [m for m in mine if (m % self.p) not in self.lost]
            dead = [m for m in mine if (m % self.p) in self.lost]
            for j, m in enumerate(alive + dead):
                self._where[m] = (g, j)
            self.n_alive.append(len(alive))
            self._hosted.append(alive + dead)

    def host_of(self, k: int, r: int):
        """(GPU, hosted index) of member r of set k."""
        return self._where[k * self.p + r]

    # ---- operations ------------------------------------------------------
    def _mark(self, name: str) -> None:
        if self.timing:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._events.append((name, ev))

    def _run(self, op: str) -> None:
        """One execute: pipelined over the sets (redset_hip_sharded_execute:
        set k+1's gather overlaps set k's gf_mac), or, with ``self.phased``,
        the four phases one after another with events between them so
        phase_ms() can split the time."""
        L = _lib.load()
        h = self._plans[op]
        stream = torch.cuda.current_stream().cuda_stream if self.device.type == "cuda" else None
        self._mark(f"{op}_start")
        if not self.phased:
            _lib.check(L.redset_hip_sharded_execute(h, stream), f"sharded {op}")
            self._mark(f"{op}_done")
            return
        _lib.check(L.redset_hip_sharded_execute_phase(h, _lib.PHASE_GATHER, stream), f"sharded {op} gather")
        self._mark(f"{op}_gathered")
        _lib.check(L.redset_hip_sharded_execute_phase(h, _lib.PHASE_COMPUTE, stream), f"sharded {op} compute")
        self._mark(f"{op}_computed")
        _lib.check(L.redset_hip_sharded_execute_phase(h, _lib.PHASE_RETURN, stream), f"sharded {op} return")
        self._mark(f"{op}_returned")
        _lib.check(L.redset_hip_sharded_execute_phase(h, _lib.PHASE_ACCUMULATE, stream), f"sharded {op} accumulate")
        self._mark(f"{op}_done")

    def run_phases(self, op: str, phases) -> None:
        """Only the given phases of one execute (redset_hip_sharded_execute_phase),
        in order, with no marks: the bench times the decode on slices already in
        place (PHASE_COMPUTE + PHASE_ACCUMULATE) and the exchange (PHASE_GATHER,
        PHASE_RETURN) apart, as BASELINE.md's C4 asks."""
        L = _lib.load()
        h = self._plans[op]
        stream = torch.cuda.current_stream().cuda_stream if self.device.type == "cuda" else None
        for ph in phases:
            _lib.check(L.redset_hip_sharded_execute_phase(h, ph, stream), f"sharded {op} phase {ph}")

    def encode(self) -> None:
        """Parity of every stripe of every set: gather data slices, compute my
        column slice, return parity slices to their hosts."""
        self._run("encode")

    def erase(self) -> None:
        """Model the loss of the lost members' files on their hosts."""
        for k in range(self.nsets):
            for r in self.lost:
                h, j = self.host_of(k, r)
                if h == self.rank:
                    self.D_host[:, j].zero_()
                    self.P_host[:, j].zero_()

    def rebuild(self) -> None:
        """Rebuild the lost members of every set from the survivors."""
        self._run("rebuild")

    def step(self) -> None:
        self.encode()
        self.rebuild()

    # ---- verification --------------------------------------------------
    def lost_snapshot(self) -> List[Tuple[int, torch.Tensor, torch.Tensor]]:
        """Copies of this GPU's hosted slabs of the members `erase` destroys."""
        snap = []
        for k in range(self.nsets):
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
        """One set's algorithmic bytes (p stripes; per GPU when there are
        `world` sets): encode
        (d+e)*C per stripe, rebuild (d+m)*C per stripe;
        "step" = both."""
        p, d, e, m, C = self.p, self.d, self.e, len(self.lost), self.chunk
        enc = p * (d + e) * C
        reb = p * (d + m) * C if m else 0
        return {"encode": enc, "rebuild": reb, "step": enc + reb}[op]

    def total_algorithmic_bytes(self, op: str = "step") -> int:
        """All GPUs' algorithmic bytes per operation: every set's."""
        return self.nsets * self.algorithmic_bytes(op)

    def exchanged_bytes(self, op: str = "step") -> int:
        """Bytes this GPU sends over the fabric per operation (C planner's count)."""
        def sent(o):
            if o not in self._plans:
                return 0
            i = self.info(o)
            return i["gather_bytes_sent"] + i["return_bytes_sent"]
        if op == "step":
            return sent("encode") + sent("rebuild")
        return sent(op)

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
        tname = type(self._transport).__name__

        def what(o, gather_text):
            if o in self._plans and self.shape(o)["shape"] == "reduce":
                return (f"{tname}: grouped P2P, partial sums of each GPU's own inputs to the outputs' hosts "
                        "(redset_hip_rs_sharded_plan_ex, REDUCE shape)")
            return f"{tname}: grouped P2P, {gather_text} (redset_hip_rs_sharded_plan_ex, GATHER shape)"
        coll = {"encode": what("encode", "data slices in, parity slices back"),
                "rebuild": what("rebuild", "decode inputs' slices in, rebuilt slices back to their hosts")}
        phases = self.phase_ms() if self.timing else None
        ops = ["encode", "rebuild"] if op == "step" else [op]
        msgs = {}
        for o in ops:
            if o in self._plans:
                i = self.info(o)
                # peer messages this GPU sends per execute after the planner's
                # row merging (every set's gather and return is an exchange
                # of its own), and their size range
                msgs[o] = {"gather_messages": i["gather_messages"], "return_messages": i["return_messages"],
                           "gather_msg_bytes": [i["gather_msg_min"], i["gather_msg_max"]],
                           "return_msg_bytes": [i["return_msg_min"], i["return_msg_max"]],
                           "exchanges": 2 * self.nsets}
        out = {
            "exchange": {
                "bytes_sent_per_gpu_per_step": self.exchanged_bytes(op),
                # the shape each plan took and both shapes' counts (busiest
                # GPU's max(sent, received) per execute, every GPU's view)
                "shape": {o: self.shape(o) for o in ops if o in self._plans},
                "messages_per_gpu": msgs,
                "column_slice_bytes": self.W,
                "collective": coll.get(op, coll["encode"] + "; " + coll["rebuild"]),
                "phase_ms_rank0": phases,
            },
            "per_gpu_GBps": round(self.algorithmic_bytes(op) / step_seconds / 1e9, 2),
        }
        if phases and op in self._plans and self.world > 1:
            # rank 0's send rate over the fabric in each exchange phase (what
            # bounds the sharded rebuild; compare with xGMI, 7 links per GPU)
            i = self.info(op)
            g_ms = phases.get(f"{op}_start->gathered")
            r_ms = phases.get(f"{op}_computed->returned")
            out["exchange"]["gather_send_GBps_rank0"] = (round(i["gather_bytes_sent"] / (g_ms * 1e-3) / 1e9, 1)
                                                         if g_ms else None)
            out["exchange"]["return_send_GBps_rank0"] = (round(i["return_bytes_sent"] / (r_ms * 1e-3) / 1e9, 1)
                                                         if r_ms and i["return_bytes_sent"] else None)
        return out
