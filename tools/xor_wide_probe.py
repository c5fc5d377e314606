"""XOR kernel at a given input count (wide XOR sets and the ring's
two-row items): xor_combine of NIN 64 MiB cells into one, event-timed on the
stream it runs on, GB/s of (NIN + 1) * cell bytes. Library from
REDSET_HIP_LIBRARY (A/B). usage: python tools/xor_wide_probe.py [nin ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import redset_amd  # noqa: E402


def probe(nin, cell=64 << 20, reps=20):
    stride = redset_amd.cell_stride(cell)
    buf = torch.randint(0, 256, ((nin + 1) * stride,), dtype=torch.uint8, device="cuda")
    ins = [buf.data_ptr() + i * stride for i in range(nin)]
    out = buf.data_ptr() + nin * stride
    for _ in range(3):
        redset_amd.xor_combine(ins, out, cell)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        redset_amd.xor_combine(ins, out, cell)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    want = buf[:cell].clone()
    for i in range(1, nin):
        want ^= buf[i * stride:i * stride + cell]
    ok = torch.equal(want, buf[nin * stride:nin * stride + cell])
    return {"nin": nin, "us": round(ms * 1e3, 1), "GBps": round((nin + 1) * cell / (ms * 1e-3) / 1e9, 1), "ok": ok,
            "faults": redset_amd.ring_faults()}


if __name__ == "__main__":
    lib = os.environ.get("REDSET_HIP_LIBRARY", "new")
    for n in [int(x) for x in sys.argv[1:]] or [7, 12, 16]:
        print(json.dumps({"lib": os.path.basename(lib), **probe(n)}), flush=True)
