"""Native-communicator bring-up must fail loudly and consistently, never hang (CPU, gloo).

The reference inherits ProcessGroupNCCL's watchdog and timeouts (``resnet/main.py:74``); our own
RCCL communicator replaces them (``parallel/comm.py``, ``csrc/comm/rccl_comm.cpp``).  These tests
drive the real agreement protocol over the launcher's TCPStore with 2 processes:

* every rank can build -> all build, with the same unique id;
* rank 1 reports "cannot build" -> EVERY rank gets the same refusal naming rank 1 (DDP then falls
  back on all ranks, or raises on all with comm='rccl') -- no rank enters the RCCL init alone;
* rank 1 never reaches setup -> rank 0 raises within the timeout with a message naming rank 1 and
  the launcher exits non-zero (instead of rank 0 blocking in ncclCommInitRank forever).

The RCCL-level halves (non-blocking init deadline, collective timeout / abort) are GPU tests in
``tests/test_rccl_gpu.py``."""
import json
import os
import subprocess
import sys
import time

import pytest
from conftest import free_port, parse_results

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(fault=None, timeout=5.0, nproc=2):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    env.pop("PDT_FAULT_NATIVE", None)
    if fault:
        env["PDT_FAULT_NATIVE"] = fault
    cmd = [sys.executable, "-m", "pytorch_distributed_tutorials_amd.launch", f"--nproc_per_node={nproc}",
           "--master_port", str(free_port()), os.path.join(ROOT, "tests", "comm_worker.py"),
           "--timeout", str(timeout)]
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, timeout=240, capture_output=True, text=True)
    res = parse_results(r.stdout)  # interleaved rank output: see conftest.parse_results
    return r, {x["rank"]: x for x in res}, time.time() - t0


def test_all_ranks_build_with_one_uid():
    r, res, _ = _run()
    assert r.returncode == 0, r.stderr[-3000:]
    assert {res[0]["outcome"], res[1]["outcome"]} == {"built"}
    assert res[0]["init"]["uid"] == res[1]["init"]["uid"]
    assert res[0]["init"]["world"] == 2 and res[1]["init"]["rank"] == 1


def test_rank_that_cannot_build_refuses_on_every_rank():
    r, res, _ = _run(fault="1:cannot")
    assert r.returncode == 0, r.stderr[-3000:]
    for k in (0, 1):
        assert res[k]["outcome"] == "refused", res
        assert "rank 1: fault injection" in res[k]["error"]


def test_rank_that_never_arrives_times_out_loudly():
    r, res, dt = _run(fault="1:never", timeout=4.0)
    assert r.returncode != 0
    assert res[0]["outcome"] == "timeout"
    assert "ranks [1] never reached the RCCL communicator setup" in res[0]["error"]
    assert 3.5 < res[0]["seconds"] < 30
    assert dt < 120


def test_comm_options_from_env(monkeypatch):
    from pytorch_distributed_tutorials_amd.parallel.comm import CommOptions
    monkeypatch.setenv("PDT_COMM_TIMEOUT", "7")
    monkeypatch.setenv("PDT_RCCL_CHANNELS", "8,16")
    o = CommOptions.from_env()
    assert (o.init_timeout, o.op_timeout, o.min_channels, o.max_channels) == (7.0, 7.0, 8, 16)
    monkeypatch.setenv("PDT_RCCL_CHANNELS", "4")
    assert CommOptions.from_env().max_channels == 4
