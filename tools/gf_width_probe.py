"""gf_mac at a given input / output count: gf_combine of NIN 64 MiB cells
into NOUT, event-timed on the stream it runs on; GB/s of (NIN + NOUT) cells.
Cells one recommended stride apart in one allocation. Library from
REDSET_HIP_LIBRARY (A/B). Output checked against a small CPU spot check.
usage: python tools/gf_width_probe.py NOUT NIN [NIN ...]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import redset_amd  # noqa: E402


def gf_mul(a, b):
    r = 0
    for _ in range(8):
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
    return r


def probe(nin, nout, cell=64 << 20, reps=20):
    stride = redset_amd.cell_stride(cell)
    buf = torch.randint(0, 256, ((nin + nout) * stride,), dtype=torch.uint8, device="cuda")
    ins = [buf.data_ptr() + i * stride for i in range(nin)]
    outs = [buf.data_ptr() + (nin + j) * stride for j in range(nout)]
    coef = np.random.default_rng(nin * 16 + nout).integers(1, 256, (nout, nin), dtype=np.uint8)
    for _ in range(3):
        redset_amd.gf_combine(ins, outs, coef, cell)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        redset_amd.gf_combine(ins, outs, coef, cell)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    # spot check 64 positions of every output
    host = buf.cpu().numpy()
    ok = True
    for pos in np.random.default_rng(7).integers(0, cell, 64):
        for j in range(nout):
            want = 0
            for i in range(nin):
                want ^= gf_mul(int(coef[j, i]), int(host[i * stride + pos]))
            ok &= want == host[(nin + j) * stride + pos]
    return {"nin": nin, "nout": nout, "us": round(ms * 1e3, 1),
            "GBps": round((nin + nout) * cell / (ms * 1e-3) / 1e9, 1), "ok": bool(ok), "faults": redset_amd.ring_faults()}


if __name__ == "__main__":
    lib = os.path.basename(os.environ.get("REDSET_HIP_LIBRARY", "new"))
    nout = int(sys.argv[1])
    for n in [int(x) for x in sys.argv[2:]]:
        print(json.dumps({"lib": lib, **probe(n, nout)}), flush=True)
