#!/usr/bin/env python3
"""Where does the run-to-run spread of the bench come from? In ONE process,
allocate the bench's set K times (fresh storage each round; HOLD=1 keeps the
earlier sets allocated) and time the encode two ways on each: the whole-set
plan (all 11 stripes in one launch, ~121 concurrent cell streams) and one
full-GPU gf_combine launch per stripe (11 concurrent streams). Prints one
line per round."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import redset_amd  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
HOLD = int(sys.argv[2]) if len(sys.argv) > 2 else 0
p, e, chunk, lost = 11, 3, 64 << 20, [1, 2]
d = p - e
redset_amd.load()
codec = redset_amd.RSCodec(p, e)
mat = codec.matrix()
s = torch.cuda.current_stream()


def stripe_ops(lay):
    ops = []
    for c in range(p):
        ins, outs, cols = [], [None] * e, []
        for r in range(p):
            enc = codec.encoding_id(r, c)
            if enc < p:
                ins.append(lay.data_cell(r, codec.data_id(r, c)))
                cols.append(r)
            else:
                outs[enc - p] = lay.parity_cell(r, enc - p)
        coef = np.array([[mat[p + i, r] for r in cols] for i in range(e)], dtype=np.uint8)
        ops.append((ins, outs, coef))
    return ops


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(n):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


keep = []
for k in range(K):
    lay = redset_amd.SetLayout.allocate(p, d, e, chunk, pad=16 << 20)
    lay.storage.random_(0, 256)
    enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    nb = enc.bytes_read + enc.bytes_written
    ops = stripe_ops(lay)
    t_plan = timeit(lambda: enc.execute(s))
    ref = [lay.parity(r).clone() for r in range(p)]

    def per_stripe():
        for ins, outs, coef in ops:
            redset_amd.gf_combine(ins, outs, coef, chunk, stream=s)

    t_str = timeit(per_stripe)
    same = all(torch.equal(lay.parity(r), ref[r]) for r in range(p))
    print(f"pid {os.getpid()} round {k} base {lay.storage.data_ptr():#x}: plan {nb / t_plan / 1e6:7.1f} GB/s  "
          f"per-stripe {nb / t_str / 1e6:7.1f} GB/s  same parity {same}", flush=True)
    if HOLD:
        keep.append((lay, enc))
    else:
        del enc, lay, ref, ops
        torch.cuda.empty_cache()
