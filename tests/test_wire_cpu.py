"""bf16 gradient wire format: accuracy at the world size of one MI355X node (8 ranks, gloo, CPU).

``--wire-dtype bf16`` halves the all-reduce bytes over xGMI (``csrc/ddp/reducer.cpp``: cast,
``ncclBfloat16`` sum, cast back with the 1/world scale).  At world 1 the sum is an identity, so
the GPU test cannot see its error; here 8 real processes sum bf16 gradients through gloo (which,
like RCCL's ring, rounds to bf16 after every partial sum) and the averaged gradient is compared
with the exact fp64 average of the per-rank fp32 gradients.

Bound: relative L2 error below 1 % and within 4x of the irreducible error of rounding the exact
average to bf16 once (the multi-hop sums cost a small constant factor, not a blow-up with N)."""
import json
import os
import subprocess
import sys

import pytest
from conftest import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_bf16_wire_error_at_8_ranks(tmp_path):
    out = str(tmp_path / "w")
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "pytorch_distributed_tutorials_amd.launch", "--nproc_per_node=8",
           "--master_port", str(free_port()), os.path.join(ROOT, "tests", "wire_worker.py"), "--out", out]
    r = subprocess.run(cmd, cwd=ROOT, env=env, timeout=600, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.load(open(f"{out}.rank{i}.json")) for i in range(8)]
    for x in res:
        assert x["world"] == 8
        assert x["rel_fp32"] < 1e-6, x          # fp32 wire: exact up to fp32 summation order
        assert x["rel_bf16"] < 1e-2, x          # bf16 wire: < 1 % relative L2
        assert x["rel_bf16"] < 4 * x["rel_bf16_once"], x
        assert x["rel_bf16"] > x["rel_fp32"]    # the bf16 wire really was used
    # every rank holds the same averaged gradient error (identical reduced gradients)
    assert len({round(x["rel_bf16"], 12) for x in res}) == 1
    print("bf16 wire @8 ranks: rel L2 %.3e (one rounding: %.3e)" % (res[0]["rel_bf16"], res[0]["rel_bf16_once"]))
