"""The C ABI under concurrent host callers, as the reference's own race tests
use its codec (race_test.go:33 TestConcurrentEncodeDeterminism, :137-193):
six host threads with their own streams make a fresh process's first library
calls at once (the one-time table uploads race) and repeat them; outputs
must be byte-identical to a serial run.  And the timeout report of the
persistent kernels: reported once, then clean launches succeed again
(ADVICE r03).  Both run in a fresh child process (tests/concurrency_worker.py)
so that no earlier test has initialised the library's process-wide state."""
import json
import os
import subprocess
import sys

import pytest

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "concurrency_worker.py")


def run_worker(mode):
    p = subprocess.run([sys.executable, "-u", WORKER, mode], capture_output=True, text=True, timeout=110)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    rep = json.loads(lines[-1])
    assert p.returncode == 0 and rep["ok"], (rep, p.stderr[-2000:])
    return rep


@pytest.mark.gpu
def test_gpu_concurrent_callers_are_deterministic(cuda):
    rep = run_worker("race")
    assert rep["threads"] == 6 and not rep["mismatches"]


@pytest.mark.gpu
def test_gpu_timeout_reported_once_then_recovers(cuda):
    rep = run_worker("diag")
    assert rep["checks"] == {"decode_unaffected": True, "reported": True, "recovered": True}
