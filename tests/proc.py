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


def stub_shm():
    """tests/rcclstub's shared-memory objects (/dev/shm/rcclstub_<pid>_<id>,
    <pid> = the process that made the unique id)"""
    return {f for f in os.listdir("/dev/shm") if f.startswith("rcclstub_")}


def leaked_stub_shm(before):
    """objects made since `before` (a stub_shm() snapshot) whose maker has
    exited or is this process: what a finished run left behind. Another
    pytest worker's run still in progress (pytest -n) is not counted."""
    leaked = []
    for f in sorted(stub_shm() - before):
        try:
            pid = int(f.split("_")[1])
        except (IndexError, ValueError):
            leaked.append(f)
            continue
        if pid == os.getpid() or not os.path.exists(f"/proc/{pid}"):
            leaked.append(f)
    return leaked


def locked_make(directory, jobs=8, timeout=600):
    """`make -s -C directory` under an exclusive file lock, so parallel test
    workers (pytest -n) that need the same build do not relink it under each
    other."""
    import fcntl

    with open(os.path.join(directory, ".make.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        return subprocess.run(["make", "-s", f"-j{jobs}", "-C", directory], capture_output=True, text=True,
                              timeout=timeout)
