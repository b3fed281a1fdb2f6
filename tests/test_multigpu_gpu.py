"""Data-parallel collectives between SEPARATE GPUs (make the first multi-GPU
box self-verifying).

Every other multi-rank GPU test runs its ranks on cuda:0 (the gpurun boxes have one GPU).  These
run one process per device -- ranks = min(device count, 8) -- and skip cleanly below two devices:

* our RCCL communicator between devices vs gloo (all_reduce sum exact on integer data, avg within
  reassociation, broadcast exact);
* the direct xGMI backend with peer buffers on other GPUs: bitwise vs the rank-order fp32 sum,
  tiny unaligned buckets leave their neighbours alone, and the POISON protocol of a late peer;
* native ResNet-18 DDP training over RCCL and over xGMI: every rank ends bit-identical, and the
  step-1 averaged gradient matches the mean of the ranks' single-process gradients.
Worker: tests/multigpu_worker.py.
"""
import os
import subprocess
import sys

import pytest
import torch
from conftest import free_port, parse_results

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _ndev():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


needs_two = pytest.mark.skipif(_ndev() < 2, reason="needs >= 2 GPUs (one process per device)")


def _launch(mode, *extra, timeout=240, nproc=None):
    n = nproc or min(_ndev(), 8)
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "multigpu_worker.py"), "--mode", mode, *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, timeout=timeout, capture_output=True, text=True)
    res = {x["rank"]: x for x in parse_results(r.stdout)}
    assert len(res) == n, r.stdout[-3000:] + r.stderr[-3000:]
    for x in res.values():
        assert x["status"] == "ok", x
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert sorted(x["device"] for x in res.values()) == list(range(n))
    return n, res


@needs_two
def test_rccl_between_devices_matches_gloo():
    n, res = _launch("rccl")
    for x in res.values():
        assert x["comm_count"] == n, x
        assert x["sum_exact"] and x["broadcast_exact"], x
        assert x["avg_max_abs"] < 1e-5, x


@needs_two
def test_xgmi_between_devices_bitwise_and_poison():
    n, res = _launch("xgmi")
    for r, x in res.items():
        assert x["bitwise_vs_rank_order"] and x["untouched_kept"] and x["error_code"] == 0, x
        assert x["flags_uncached"], x
        assert x["poison_nan"], x
        if r == 0:
            assert "never marked their gradients ready" in x["poison_msg"], x
        else:
            assert "peer rank 0 failed first" in x["poison_msg"] and x["poison_code"] & 0x80000000, x


@needs_two
@pytest.mark.parametrize("comm", ["auto", "xgmi"])
def test_ddp_between_devices_ranks_bit_identical(comm):
    n, res = _launch("ddp", "--comm", comm)
    cs = {x["checksum"] for x in res.values()}
    assert len(cs) == 1, res
    for x in res.values():
        assert x["finite"], x
        assert x["xgmi"] if comm == "xgmi" else x["native_comm"], x
        # the averaged gradient is right (vs the mean of per-rank single-process native twins),
        # and distinguishable from a reducer that did not average or did not reduce at all
        assert x["grad_rel_vs_reference"] < 2e-2, x
        assert x["grad_rel_vs_local"] > 5 * x["grad_rel_vs_reference"], x
        assert x["grad_rel_vs_sum"] > 0.3, x


def test_ddp_worker_gradient_reference_single_rank():
    """The separate-device worker's gradient check itself, exercised on any GPU box: at world 1
    the DDP gradient must equal the rank's own single-process gradient within tolerance (the
    parameter-name mapping, the pre-re-layout state copy and the per-rank reference run)."""
    if _ndev() < 1:
        pytest.skip("needs a GPU")
    n, res = _launch("ddp", "--comm", "auto", nproc=1)
    x = res[0]
    assert x["finite"], x
    assert x["grad_rel_vs_reference"] < 2e-2, x
    assert abs(x["grad_rel_vs_local"] - x["grad_rel_vs_reference"]) < 1e-6, x  # world 1: local == mean
