"""Multi-rank data parallelism on the GPU path (2 ranks sharing cuda:0, gloo collectives).

RCCL cannot put two ranks on one device, and gpurun boxes have one GPU, so this
exercises everything of the multi-GPU path except RCCL itself: native kernels,
in-place gradient sinks, the side-stream weight gradients the reducer must join
before each bucket's collective, bucket ordering and the fused optimizer.  The
RCCL communicator + C++ reducer path itself is executed on one GPU by
test_rccl_gpu.py (forced world-1 communicator: bitwise gradients, bf16 wire,
timing, launch order, strict duplicate-mark checking).
"""
import json
import os
import subprocess
import sys

import pytest
from conftest import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_ddp_two_ranks_one_gpu(tmp_path, gpu):
    out = str(tmp_path / "res")
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "ddp_gpu_worker.py"), "--out", out]
    r = subprocess.run(cmd, cwd=ROOT, env=env, timeout=110, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.load(open(f"{out}.rank{i}.json")) for i in range(2)]
    for x in res:
        assert x["finite"]
        assert x["grad_rel_err"] < 2e-2, x["worst_params"]
        assert x["launch_order"] == list(range(x["bucket_info"]["num_buckets"]))
    cs = res[0]["checksums"]
    assert cs[0] == cs[1], cs


def test_bench_two_ranks_share_device_ranks_identical(tmp_path, gpu):
    """bench.py at N>1 proves its ranks ended bit-identical (all-gathered
    parameter checksum in the JSON) -- rehearsed with 2 gloo ranks sharing cuda:0 on the native
    kernels, the same bench path the driver's 8-GPU run takes."""
    out = tmp_path / "b.json"
    env = dict(os.environ, MASTER_PORT=str(free_port()), OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--backend", "gloo", "--arch", "resnet18", "--image-size", "64", "--batch", "16",
                        "--steps", "2", "--warmup", "1", "--json-out", str(out)],
                       cwd=ROOT, env=env, timeout=110, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["n_gpus"] == 2 and d["config"]["shared_device"]
    assert d["config"]["ranks_identical"] is True, d["config"]
