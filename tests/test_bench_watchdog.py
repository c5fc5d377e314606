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


def test_relay_passes_one_result_line():
    """self_launch's relay: rank 0's result line to stdout once, every other
    line (logs, a second JSON line) to stderr."""
    r = _run("import bench, io\n"
             "out, err = io.StringIO(), io.StringIO()\n"
             "lines = ['log a\\n', '{\"metric\": \"m\", \"value\": 1}\\n', '{\"metric\": \"m\", \"value\": 2}\\n',"
             " '{not json\\n']\n"
             "seen = bench.relay(lines, out, err)\n"
             "print(seen, repr(out.getvalue()), repr(err.getvalue()))\n")
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == ("True '{\"metric\": \"m\", \"value\": 1}\\n' "
                                "'log a\\n{\"metric\": \"m\", \"value\": 2}\\n{not json\\n'")


def test_self_launch_relays_child_line_and_status(tmp_path):
    """The launcher runs its ranks as one child process and returns the
    child's status; no result line is a failure even with status 0, and a
    child past the timeout is stopped."""
    ok = tmp_path / "ok.py"
    ok.write_text("import json; print('rank log'); print(json.dumps({'metric': 'm', 'value': 5}))\n")
    silent = tmp_path / "silent.py"
    silent.write_text("print('nothing to report')\n")
    hang = tmp_path / "hang.py"
    hang.write_text("import time; time.sleep(60)\n")
    code = ("import bench, sys\n"
            f"rc1 = bench.self_launch([], 2, 30, cmd=[sys.executable, {str(ok)!r}])\n"
            f"rc2 = bench.self_launch([], 2, 30, cmd=[sys.executable, {str(silent)!r}])\n"
            f"rc3 = bench.self_launch([], 2, 2, cmd=[sys.executable, {str(hang)!r}])\n"
            "print('rcs', rc1, rc2, rc3)\n")
    r = _run(code)
    assert r.returncode == 0, r.stderr
    out = r.stdout.strip().splitlines()
    assert json.loads(out[0]) == {"metric": "m", "value": 5}
    assert "printed no result line" in out[1] and "printed no result line" in out[2]
    assert out[3] == "rcs 0 1 -9"
    assert "rank log" in r.stderr


def test_claimed_stdout_carries_only_the_result_line():
    """RCCL prints a version banner to stdout (C stdio) when a communicator is
    created; after claim_stdout() anything written to fd 1 -- C printf or
    Python print -- goes to stderr, and only the result line to stdout."""
    r = _run("import bench, ctypes\n"
             "bench.claim_stdout()\n"
             "libc = ctypes.CDLL(None)\n"
             "libc.printf(b'RCCL version : banner\\n')\n"
             "libc.fflush(None)\n"
             "print('a stray python print')\n"
             "bench.emit({'metric': 'm', 'value': 7.0}, 0)\n")
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines() == ['{"metric": "m", "value": 7.0}'], r.stdout
    assert "RCCL version" in r.stderr and "stray" in r.stderr
