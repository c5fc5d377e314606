#!/usr/bin/env python3
"""What one member moves per call of the drop-in slot's sharded exchange on a
node with a GPU per member (the RCCL path of rank_mpi.c sharded_slot), from
the C planner itself: redset_hip_rs_sharded_plan / redset_hip_xor_sharded_plan
are planned for every member r of one set at world = p (host[m] = m, one
hosted slot), with a compute callback and a no-op transport, so no GPU and no
process group are needed and nothing executes. Per member:

  file_read   the cells it reads: the decode's wanted cells (a cell is read iff
              some stripe's decode map reads it, rank_mpi.c `want`), the
              encode's d data cells
  pcie_h2d    the same bytes, copied to HBM column slab by column slab
  xgmi_sent / xgmi_recv   gather + return bytes to / from other GPUs
              (redset_hip_sharded_info, the planner's own count)
  pcie_d2h    the cells it gets back: a lost member's p cells (decode), the
              e parity cells (encode)
  file_write  the same bytes

and the seconds each would take at its ceiling: PCIe 55 GB/s per direction
(profiles/r01_pcie_probe.json), xGMI 153 GB/s per link and direction with
one link per GPU pair: a member's exchange with its p - 1
peers spreads over p - 1 links. This is the model the first
redset_recover() on such a node is to be read against
(redset_hip_rank_last_stats gives the measured side).

usage: python tools/slot_model.py [--chunk-mib 64] [--network] -> one JSON line per case
(--network: the encode's bytes per member with a node per member, the
reference's ring against the sharded plan, network_encode)
"""
import argparse
import ctypes
import json
import os
import sys
from ctypes import c_int, c_void_p

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PCIE_GBPS = 55.0
XGMI_LINK_GBPS = 153.0


def plan_info(L, lib, rs, p, e, kind, lost, chunk, rank):
    """the planner's info block of member `rank` at world = p"""
    W = int(lib.redset_hip_shard_slice_bytes(chunk, p))
    host = (c_int * p)(*range(p))
    slot = (c_int * p)(*([0] * p))
    d = p - e
    base = 1 << 40  # addresses only: nothing is executed
    bufs = [base, base + (1 << 38), base + (2 << 38), base + (3 << 38)]
    lay = L.ShardLayout(1, host, slot, 1, chunk, W, *bufs)
    tr = L.Transport(p, rank, ctypes.cast(L.EXCHANGE_FN(lambda *a: 0), c_void_p), None)
    cfn = L.COMPUTE_FN(lambda *a: 0)
    comp = L.Compute(ctypes.cast(cfn, c_void_p), None)
    out = c_void_p()
    arr = (c_int * max(1, len(lost)))(*lost)
    if rs is None:
        rc = lib.redset_hip_xor_sharded_plan(p, kind, lost[0] if lost else 0, ctypes.byref(lay), ctypes.byref(tr),
                                             ctypes.byref(comp), ctypes.byref(out))
    else:
        rc = lib.redset_hip_rs_sharded_plan(rs, kind, len(lost), arr, ctypes.byref(lay), ctypes.byref(tr),
                                            ctypes.byref(comp), ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(lib.redset_hip_last_error().decode())
    info = L.ShardedInfo()
    lib.redset_hip_sharded_get_info(out, ctypes.byref(info))
    lib.redset_hip_sharded_destroy(out)
    _ = d
    return info.as_dict()


def wanted_cells(codec, p, e, lost, r):
    """cells of member r the sharded decode reads (rank_mpi.c sharded_slot)"""
    if codec is None:
        return p  # XOR: every cell of every survivor
    n = 0
    for c in range(p):
        M = codec.decode_matrix(lost, c)
        if M[:, r].any():
            n += 1
    return n


def model(scheme, p, e, lost, chunk, op):
    from redset_amd import _lib as L
    from redset_amd.codec import RSCodec

    lib = L.load()
    rs = c_void_p()
    codec = None
    if scheme == "rs":
        lib.redset_hip_rs_create(p, e, ctypes.byref(rs))
        codec = RSCodec(p, e)
        kind = L.PLAN_RS_REBUILD if op == "rebuild" else L.PLAN_RS_ENCODE
    else:
        rs = None
        kind = L.PLAN_XOR_REBUILD if op == "rebuild" else L.PLAN_XOR_ENCODE
    d = p - e
    rows = []
    for r in range(p):
        inf = plan_info(L, lib, rs, p, e, kind, lost if op == "rebuild" else [], chunk, r)
        if op == "rebuild":
            reads = 0 if r in lost else wanted_cells(codec, p, e, lost, r) * chunk
            back = p * chunk if r in lost else 0
        else:
            reads, back = d * chunk, e * chunk
        sent = inf["gather_bytes_sent"] + inf["return_bytes_sent"]
        recv = inf["gather_bytes_recv"] + inf["return_bytes_recv"]
        rows.append({"member": r, "file_read": reads, "pcie_h2d": reads, "xgmi_sent": sent, "xgmi_recv": recv,
                     "pcie_d2h": back, "file_write": back})
    if rs is not None:
        lib.redset_hip_rs_destroy(rs)
    mx = {k: max(x[k] for x in rows) for k in rows[0] if k != "member"}
    links = max(1, p - 1)
    secs = {"pcie_h2d": mx["pcie_h2d"] / (PCIE_GBPS * 1e9), "pcie_d2h": mx["pcie_d2h"] / (PCIE_GBPS * 1e9),
            "xgmi": max(mx["xgmi_sent"], mx["xgmi_recv"]) / (links * XGMI_LINK_GBPS * 1e9)}
    alg = p * (d + (len(lost) if op == "rebuild" else e)) * chunk
    bound = max(secs, key=secs.get)
    return {
        "case": f"{scheme.upper()}" + (f"({d}+{e})" if scheme == "rs" else "") + f" p={p} {op}"
                + (f" lost {lost}" if op == "rebuild" else "") + f", chunk {chunk >> 20} MiB, world {p} (a GPU per member)",
        "bytes_per_member_max": mx,
        "bytes_per_member": rows,
        "seconds_at_ceiling_max": {k: round(v, 5) for k, v in secs.items()},
        "bound": bound,
        "model_call_seconds": round(secs[bound], 5),
        "model_GBps": round(alg / secs[bound] / 1e9, 1),
        "ceilings": {"pcie_GBps_per_direction": PCIE_GBPS, "xgmi_GBps_per_link": XGMI_LINK_GBPS, "links": links},
    }


NIC_GBPS = 25.0  # a 200 Gb/s NIC per node and direction: an assumption, not measured here


def network_encode(p, e, chunk):
    """The encode's network bytes per member with every member on its own
    node (redset's usual placement): the reference's ring, which the host
    exchange keeps, sends each of a member's d data cells to the e parity
    holders of its stripe and receives as much (src/redset_reedsolomon.c:
    329-363: d ring steps x e sends of one segment), d*e cells each way; the
    sharded plan over host slabs (rank_mpi.c sharded_slot_host, AUTO for RS
    encodes with e >= 2) sends the column slices the C planner lists."""
    from redset_amd import _lib as L

    lib = L.load()
    rs = c_void_p()
    lib.redset_hip_rs_create(p, e, ctypes.byref(rs))
    d = p - e
    sent = recv = 0
    for r in range(p):
        inf = plan_info(L, lib, rs, p, e, L.PLAN_RS_ENCODE, [], chunk, r)
        sent = max(sent, inf["gather_bytes_sent"] + inf["return_bytes_sent"])
        recv = max(recv, inf["gather_bytes_recv"] + inf["return_bytes_recv"])
    lib.redset_hip_rs_destroy(rs)
    ring = d * e * chunk
    sharded = max(sent, recv)
    return {
        "case": f"RS({d}+{e}) p={p} encode, chunk {chunk >> 20} MiB, a node per member",
        "ring_bytes_per_member_each_way": ring,
        "sharded_bytes_per_member_each_way": {"sent": sent, "recv": recv},
        "cells_each_way": {"ring": d * e, "sharded": round(sharded / chunk, 3)},
        "ratio_ring_over_sharded": round(ring / sharded, 3),
        "seconds_at_nic": {"ring": round(ring / (NIC_GBPS * 1e9), 4), "sharded": round(sharded / (NIC_GBPS * 1e9), 4)},
        "nic_GBps_per_direction": NIC_GBPS,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--network", action="store_true",
                    help="the encode's network bytes with a node per member: ring vs sharded plan")
    a = ap.parse_args()
    C = a.chunk_mib << 20
    if a.network:
        for p, e in [(4, 2), (6, 2), (8, 3), (11, 3), (10, 2), (20, 4)]:
            print(json.dumps(network_encode(p, e, C)))
        return
    for scheme, p, e, lost, op in [("rs", 8, 3, [1, 2], "rebuild"), ("rs", 8, 2, [1, 2], "rebuild"),
                                   ("rs", 8, 3, [], "encode"), ("xor", 8, 1, [3], "rebuild")]:
        print(json.dumps(model(scheme, p, e, lost, C, op)))


if __name__ == "__main__":
    main()
