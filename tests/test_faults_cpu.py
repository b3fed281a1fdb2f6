"""Failure detection and aux subsystems on CPU.

* a rank that crashes mid-training makes the launcher fail fast (non-zero exit, no hang);
* a rank that hangs inside training is detected by a progress watchdog (its own or its peer's),
  which aborts with the watchdog exit code; the launcher then tears the job down;
* unit checks of the watchdog, the fault-spec parser, step metrics and tracing."""
import os
import random
import re
import subprocess
import sys
import time

import pytest
from conftest import free_port
import torch

from pytorch_distributed_tutorials_amd.utils import trace
from pytorch_distributed_tutorials_amd.utils.metrics import StepTimer
from pytorch_distributed_tutorials_amd.utils.watchdog import (EXIT_CODE, FaultInjector, Watchdog,
                                                              parse_faults)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**extra):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "2"
    env.update(extra)
    return env


def _launch(tmp_path, extra_args, **env):
    port = free_port()
    cmd = [sys.executable, "-m", "pytorch_distributed_tutorials_amd.launch", "--nproc_per_node=2",
           "--master_port", str(port),
           "--arch", "resnet18", "--data", "synthetic-cifar", "--synthetic-samples", "64",
           "--batch-size", "8", "--num_epochs", "1", "--eval-every", "1000",
           "--model_dir", str(tmp_path), "--num-classes", "10", "--backend", "gloo"] + extra_args
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=_env(**env), timeout=300, capture_output=True, text=True)
    return r, time.time() - t0


def test_parse_faults():
    assert parse_faults("1:3:crash, 0:5:hang") == [(1, 3, "crash"), (0, 5, "hang")]
    assert parse_faults("") == []
    with pytest.raises(ValueError):
        parse_faults("0:1:explode")
    inj = FaultInjector(1, "1:2:crash,0:1:hang")
    inj(0)
    inj(1)  # the hang is for rank 0
    with pytest.raises(RuntimeError):
        inj(2)


def test_watchdog_fires_and_heartbeat_defers():
    fired = []
    wd = Watchdog(0.4, rank=3, on_timeout=lambda: fired.append(1), poll=0.05, exit_process=False)
    for _ in range(6):  # steady heartbeats keep it quiet
        time.sleep(0.1)
        wd.heartbeat("train")
    assert not wd.fired
    time.sleep(0.8)
    assert wd.fired and fired == [1] and wd.phase == "train"
    wd.stop()


def test_step_timer_and_trace():
    timer = StepTimer(torch.device("cpu"))
    timer.start()
    for _ in range(3):
        time.sleep(0.01)
        timer.tick()
    r = timer.report()
    assert r["step_ms"] >= 5.0
    s = timer.stats.summary(images_per_step=32)
    assert s["steps"] == 3 and s["img_per_s"] > 0 and s["comm_ms"] is None
    trace.enable(True)
    try:
        with trace.trace_range("unit-test-range"):
            x = torch.ones(4).sum()
        trace.mark("unit-test-mark")
    finally:
        trace.enable(False)
    assert float(x) == 4.0


@pytest.mark.slow
def test_rank_crash_fails_fast(tmp_path):
    r, dt = _launch(tmp_path, ["--max-steps-per-epoch", "6"], PDT_FAULT="1:2:crash")
    assert r.returncode != 0
    assert "injected fault on rank 1 at step 2" in r.stderr
    assert dt < 240


@pytest.mark.slow
def test_rank_hang_detected_by_watchdog(tmp_path):
    r, dt = _launch(tmp_path, ["--max-steps-per-epoch", "6", "--watchdog-timeout", "8"],
                    PDT_FAULT="1:2:hang")
    assert r.returncode != 0
    # the hung rank and its blocked peer both stop progressing: whichever watchdog fires first
    # aborts the job (the launcher then tears the other rank down)
    assert re.search(r"\[watchdog\] rank [01]: no progress", r.stderr), r.stderr[-2000:]
    assert dt < 240
