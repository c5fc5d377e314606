"""Run a test's child command (mpirun and its ranks, a tool) in a process
group of its own, so a hang ends at the time limit with the whole group
killed and the output so far reported -- subprocess.run(timeout=...) kills
only mpirun, then waits forever on the pipes its ranks still hold."""
import os
import signal
import subprocess

import pytest


def run_group(cmd, timeout, env=None, cwd=None):
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, errors="replace", env=env,
                         cwd=cwd, start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        pytest.fail(f"timed out after {timeout} s: {' '.join(map(str, cmd))}\n{out[-3000:]}\n{err[-3000:]}")
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


def locked_make(directory, jobs=8, timeout=600):
    """`make -s -C directory` under an exclusive file lock, so parallel test
    workers (pytest -n) that need the same build do not relink it under each
    other."""
    import fcntl

    with open(os.path.join(directory, ".make.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        return subprocess.run(["make", "-s", f"-j{jobs}", "-C", directory], capture_output=True, text=True,
                              timeout=timeout)
