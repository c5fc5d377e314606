#!/usr/bin/env python3
"""What bench.py's sharded leg (configs[3]) should show at N = 1/2/4/8 on a
node of MI355X GPUs, from the C planner itself: for every GPU g the
rebuild plan of redset_amd/dist.py's placement (N sets of p members, member
m of the world on GPU m mod N, each GPU's lost members last) is planned with
a compute callback and a no-op transport, so no GPU and no process group are
needed and nothing executes. Per GPU it reports the bytes sent and received
over the fabric per step (redset_hip_sharded_info) and the algorithmic
bytes of its compute, and prices them:

  xgmi   max(sent, recv) / ((N - 1) x 153 GB/s): an all-to-all over the
         fully connected mesh, one link per GPU pair
  hbm    compute bytes / the measured gf_mac rebuild rate (6.3 TB/s,
         profiles/r05s24_bench_kernel_stats.csv)

The leg pipelines its sets (set k + 1's gather under set k's gf_mac), so a
step costs about the larger of the two; `model_value` is then N sets'
algorithmic rebuild bytes over that. SCALE_rNN's sharded.value at each N is
to be read against it. --one-set: one set spread over the N GPUs instead
(the leg's `one_set`, BASELINE.md's C4 word for word).

Both exchange shapes are planned (include/redset_hip.h REDSET_HIP_SHAPE_*):
"gather" (every GPU gathers its column slice of each decode input and
returns its slice of each output) and "reduce" (every GPU sends partial sums
of its own inputs to the outputs' hosts); `auto` names the one the planner
takes (the busiest GPU's max(sent, received) is smaller; ties: gather).

usage: python tools/sharded_model.py [--chunk-mib 64] [--ranks 11] [--encoding 3] [--lost 1,2] [--one-set]
"""
import argparse
import ctypes
import json
import os
import sys
from ctypes import c_int, c_void_p

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

XGMI_LINK_GBPS = 153.0
GF_MAC_REBUILD_GBPS = 6300.0


def placement(p, lost, world, nsets):
    """dist.py ShardedSetRunner._place: (host, slot) of every member"""
    where = {}
    for g in range(world):
        mine = [m for m in range(nsets * p) if m % world == g]
        alive = [m for m in mine if (m % p) not in lost]
        dead = [m for m in mine if (m % p) in lost]
        for j, m in enumerate(alive + dead):
            where[m] = (g, j)
    return where


def plan_gpu(L, lib, rs, p, lost, chunk, world, rank, nsets, shape):
    where = placement(p, lost, world, nsets)
    nm = nsets * p
    host = (c_int * nm)(*[where[m][0] for m in range(nm)])
    slot = (c_int * nm)(*[where[m][1] for m in range(nm)])
    W = int(lib.redset_hip_shard_slice_bytes(chunk, world))
    base = 1 << 40  # addresses only: nothing is executed
    lay = L.ShardLayout(nsets, host, slot, -(-nsets * p // world), chunk, W, base, base + (1 << 38),
                        base + (2 << 38), base + (3 << 38))
    tr = L.Transport(world, rank, ctypes.cast(L.EXCHANGE_FN(lambda *a: 0), c_void_p), None)
    cfn = L.COMPUTE_FN(lambda *a: 0)
    kfn = L.COMBINE_FN(lambda *a: 0)
    comp = L.Compute(ctypes.cast(cfn, c_void_p), None)
    opts = L.ShardedOpts()
    opts.struct_size = ctypes.sizeof(L.ShardedOpts)
    opts.shape = shape
    opts.compute = ctypes.pointer(comp)
    opts.combine = ctypes.cast(kfn, c_void_p)
    out = c_void_p()
    arr = (c_int * len(lost))(*lost)
    if lib.redset_hip_rs_sharded_plan_ex(rs, L.PLAN_RS_REBUILD, len(lost), arr, ctypes.byref(lay), ctypes.byref(tr),
                                         ctypes.byref(opts), ctypes.byref(out)) != 0:
        raise RuntimeError(lib.redset_hip_last_error().decode())
    info = L.ShardedInfo()
    lib.redset_hip_sharded_get_info(out, ctypes.byref(info))
    si = L.ShapeInfo()
    lib.redset_hip_sharded_get_shape(out, ctypes.byref(si), ctypes.sizeof(si))
    lib.redset_hip_sharded_destroy(out)
    return info.as_dict(), si.as_dict()


def price(rows, world, alg):
    sent = max(r["gather_bytes_sent"] + r["return_bytes_sent"] for r in rows)
    recv = max(r["gather_bytes_recv"] + r["return_bytes_recv"] for r in rows)
    comp = max(r["compute_bytes"] for r in rows)
    t_hbm = comp / (GF_MAC_REBUILD_GBPS * 1e9)
    t_xgmi = max(sent, recv) / ((world - 1) * XGMI_LINK_GBPS * 1e9) if world > 1 else 0.0
    step = max(t_hbm, t_xgmi)
    return {
        "per_gpu_max": {"bytes_sent": sent, "bytes_recv": recv, "compute_bytes": comp,
                        "messages_sent": max(r["gather_messages"] + r["return_messages"] for r in rows)},
        "seconds": {"hbm": round(t_hbm, 6), "xgmi": round(t_xgmi, 6)},
        "bound": "xgmi" if t_xgmi > t_hbm else "hbm",
        "model_ms_per_step": round(step * 1e3, 4),
        "model_value_GBps": round(alg / step / 1e9, 1),
        "model_frac_of_hbm": round(alg / step / 1e9 / (world * 8000.0), 4),
    }


def model(p, e, lost, chunk, world, one_set=False):
    from redset_amd import _lib as L

    lib = L.load()
    rs = c_void_p()
    lib.redset_hip_rs_create(p, e, ctypes.byref(rs))
    nsets = 1 if one_set else world
    alg = nsets * p * (p - e + len(lost)) * chunk
    out = {
        "n_gpus": world,
        "workload": (f"{nsets} set(s) of RS({p - e}+{e}) over {world} GPUs, chunk {chunk >> 20} MiB, rebuild {lost}, "
                     "members round-robin"),
        "ceilings": {"xgmi_GBps_per_link": XGMI_LINK_GBPS, "gf_mac_rebuild_GBps": GF_MAC_REBUILD_GBPS},
    }
    plans = [plan_gpu(L, lib, rs, p, lost, chunk, world, g, nsets, L.SHAPE_AUTO) for g in range(world)]
    out["auto"] = plans[0][1]["shape"]
    out["reduce_possible"] = bool(plans[0][1]["reduce_possible"])
    for name, sh in (("gather", L.SHAPE_GATHER), ("reduce", L.SHAPE_REDUCE)):
        if name == "reduce" and not out["reduce_possible"]:
            out[name] = None
            continue
        out[name] = price([plan_gpu(L, lib, rs, p, lost, chunk, world, g, nsets, sh)[0] for g in range(world)],
                          world, alg)
    lib.redset_hip_rs_destroy(rs)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--ranks", type=int, default=11)
    ap.add_argument("--encoding", type=int, default=3)
    ap.add_argument("--lost", default="1,2")
    ap.add_argument("--one-set", action="store_true", help="one set over the N GPUs (the leg's one_set, C4)")
    a = ap.parse_args()
    lost = sorted(int(x) for x in a.lost.split(","))
    for n in (1, 2, 4, 8):
        print(json.dumps(model(a.ranks, a.encoding, lost, a.chunk_mib << 20, n, a.one_set)))


if __name__ == "__main__":
    main()
