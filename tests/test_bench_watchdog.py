"""bench.py's sharded-leg watchdog (host logic only, no GPU): a hung RCCL
exchange must still leave rank 0's one JSON line on stdout, printed once, and
end the process with a non-zero status (a hang is never a clean run)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code):
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60)


def test_expired_leg_prints_main_line_and_exits():
    r = _run("import bench, time\n"
             "bench.sharded_expired({'metric': 'm', 'value': 1.0}, 0, 2.0)\n"
             "time.sleep(5)\n"
             "print('not reached')\n")
    assert r.returncode == 3
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["value"] == 1.0 and line["sharded"] == {"error": "timed out after 2 s"}


def test_watchdog_after_print_exits_without_second_line():
    r = _run("import bench\n"
             "res = {'metric': 'm', 'value': 2.0, 'sharded': {'value': 3.0}}\n"
             "bench.emit(res, 0)\n"
             "bench.sharded_expired(res, 0, 1.0)\n")
    assert r.returncode == 3
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1 and json.loads(lines[0])["sharded"] == {"value": 3.0}
    assert "timed out" in r.stderr


def test_other_ranks_print_nothing():
    r = _run("import bench\nbench.sharded_expired({'value': 1.0}, 3, 1.0)\n")
    assert r.returncode == 3 and r.stdout == ""
