"""How the set's placement in one HBM allocation moves the codec's rate.

RS(8+3), p = 11, 64 MiB cells: encode (11 launches) and rebuild of members
{1, 2} (11 launches) through the whole-set plans, event-timed on the stream
they run on, for several placements of the same cells:
  member  -- member-major: member r's d data cells then e parity cells,
             cells `gap` apart (SetLayout; the bench uses gap = 80 MiB)
  cell    -- cell-major: cell s of every member side by side, member r's
             cells p * gap apart (lofi[r] = r * gap, parity[r] = (d*p + r) * gap)
Also XOR p = 8 encode in both placements. Prints one JSON line per case.
usage: python tools/layout_probe.py [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import redset_amd  # noqa: E402

MiB = 1 << 20


def placements(p, d, e, gap, kind):
    """(lofi offsets, parity offsets, cell stride, total bytes)"""
    if kind == "member":
        per = (d + e) * gap
        return [r * per for r in range(p)], [r * per + d * gap for r in range(p)], gap, p * per
    return [r * gap for r in range(p)], [(d * p + r) * gap for r in range(p)], p * gap, p * (d + e) * gap


def time_plan(plan, reps):
    plan.execute()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        plan.execute()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    C = 64 * MiB
    p, e = 11, 3
    d = p - e
    codec = redset_amd.RSCodec(p, e)
    for kind in ("member", "cell"):
        for gap_mib in (64, 80, 72, 68):
            gap = gap_mib * MiB
            lo, po, stride, total = placements(p, d, e, gap, kind)
            buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
            base = buf.data_ptr()
            lofi = [base + o for o in lo]
            par = [base + o for o in po]
            enc = codec.plan_encode(lofi, par, C, stride)
            reb = codec.plan_rebuild([1, 2], lofi, par, C, stride)
            te, tr = time_plan(enc, reps), time_plan(reb, reps)
            eb, rb = p * (d + e) * C, p * (d + 2) * C
            print(json.dumps({"scheme": "rs", "placement": kind, "gap_mib": gap_mib,
                              "encode_us_per_launch": round(te * 1e3 / enc.launches, 1),
                              "encode_GBps": round(eb / (te * 1e-3) / 1e9, 1),
                              "rebuild_us_per_launch": round(tr * 1e3 / reb.launches, 1),
                              "rebuild_GBps": round(rb / (tr * 1e-3) / 1e9, 1),
                              "step_GBps": round((eb + rb) / ((te + tr) * 1e-3) / 1e9, 1)}), flush=True)
            del enc, reb, buf
            torch.cuda.empty_cache()
    px = 8
    for kind in ("member", "cell"):
        for gap_mib in (64, 80):
            gap = gap_mib * MiB
            lo, po, stride, total = placements(px, px - 1, 1, gap, kind)
            buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
            base = buf.data_ptr()
            enc = redset_amd.xor_plan_encode(px, [base + o for o in lo], [base + o for o in po], C, stride)
            te = time_plan(enc, reps)
            print(json.dumps({"scheme": "xor", "placement": kind, "gap_mib": gap_mib,
                              "encode_us_per_launch": round(te * 1e3 / enc.launches, 1),
                              "encode_GBps": round(px * px * C / (te * 1e-3) / 1e9, 1)}), flush=True)
            del enc, buf
            torch.cuda.empty_cache()
    assert redset_amd.ring_faults() == 0


if __name__ == "__main__":
    main()
