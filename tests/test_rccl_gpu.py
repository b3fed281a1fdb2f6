"""The RCCL data-parallel path executed on ONE GPU (forced world-1 communicator).

The multi-GPU hot path -- our C++ ``Reducer`` launching bucket all-reduces on our own RCCL
communicator (``csrc/ddp/reducer.cpp``, ``csrc/comm/rccl_comm.cpp``), the bf16 wire format,
``ncclAvg``, the side-stream join before each bucket, the comm-timing events and the per-forward
BN-buffer broadcast with its deferred wait -- is what the reference's ``init_process_group("nccl")``
+ DDP wrap + overlapped all-reduce (``resnet/main.py:74,80,123``) become here.  A single-process
``DistributedDataParallel(force_reducer=True)`` runs all of it through a world-1 RCCL
communicator, where every collective is an identity: the gradients must be BITWISE those of the
same model without the reducer (deterministic kernels), bf16 on the wire must stay within bf16
rounding, and the bookkeeping (launch order, duplicate marks, timing) must be exact.
"""
import json
import math
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _build(dev, arch="resnet50", force=False, wire="fp32", last_mb=None, seed=0):
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.optim import SGD
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    torch.manual_seed(seed)
    m = build_model(arch, num_classes=1000, impl="native").to(dev)
    m.set_impl("native")
    ddp = DistributedDataParallel(m, device_ids=[dev.index], output_device=dev.index,
                                  comm="rccl" if force else "auto", force_reducer=force,
                                  wire_dtype=wire, last_bucket_mb=last_mb)
    opt = SGD(ddp.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-5)
    return ddp, opt


def _data(dev, n=16, hw=112):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, 3, hw, hw, generator=g).to(dev)
    y = torch.randint(0, 1000, (n,), generator=g).to(dev)
    return x, y


def _train(ddp, opt, x, y, steps=2):
    from pytorch_distributed_tutorials_amd import ops
    grads, losses = [], []
    for _ in range(steps):
        opt.zero_grad()
        loss = ops.cross_entropy(ddp(x), y)
        loss.backward()
        grads.append(ddp.space.grad_flat.clone())
        losses.append(float(loss.item()))
        opt.step()
    torch.cuda.synchronize()
    bufs = {str(k): v.clone() for k, v in ddp.buffer_flats.items()}
    return grads, losses, ddp.space.param_flat.clone(), bufs


@pytest.fixture
def det():
    from pytorch_distributed_tutorials_amd.utils import seed
    seed.set_random_seeds(0, deterministic=True)   # slab split-K weight gradients: bitwise repeatable
    yield
    seed.set_random_seeds(0, deterministic=False)


def test_forced_reducer_fp32_wire_bitwise(gpu, det):
    x, y = _data(gpu)
    ddp0, opt0 = _build(gpu, force=False)
    # world 1 without force: no communicator (a local-mode reducer may exist for the optimizer's
    # per-bucket update, optim/sgd.py overlap)
    assert ddp0.comm is None and not ddp0.bucket_info()["native_comm"]
    ref = _train(ddp0, opt0, x, y)
    del ddp0, opt0

    ddp1, opt1 = _build(gpu, force=True)
    info = ddp1.bucket_info()
    assert info["native_comm"] and info["reducer"] == "Reducer" and info["forced"]
    assert ddp1.enable_comm_timing(True)
    ddp1.reducer.set_strict(True)     # a gradient marked again after its all-reduce raises
    got = _train(ddp1, opt1, x, y)

    for s in range(2):
        assert torch.equal(ref[0][s], got[0][s]), f"step {s}: gradients differ through the reducer"
        assert ref[1][s] == got[1][s]
    assert torch.equal(ref[2], got[2]), "parameters differ after two SGD steps"
    for k in ref[3]:
        assert torch.equal(ref[3][k], got[3][k]), f"BN buffers ({k}) differ"
    nb = ddp1.reducer.num_buckets
    assert nb == len(ddp1.bucket_sizes) > 1
    assert ddp1.reducer.last_launch_order() == list(range(nb))
    assert ddp1.reducer.duplicate_marks == 0
    assert ddp1.reducer.iterations == 2
    st = ddp1.comm_stats()
    assert st is not None and math.isfinite(st["comm_ms"]) and math.isfinite(st["exposed_ms"])
    assert st["comm_ms"] >= 0 and 0 <= st["exposed_ms"] <= st["comm_ms"] + 1e-3


def test_forced_reducer_bf16_wire(gpu, det):
    x, y = _data(gpu)
    ddp0, opt0 = _build(gpu, force=True, wire="fp32")
    ref = _train(ddp0, opt0, x, y, steps=1)
    del ddp0, opt0
    ddp1, opt1 = _build(gpu, force=True, wire="bf16")
    got = _train(ddp1, opt1, x, y, steps=1)
    g0, g1 = ref[0][0], got[0][0]
    rel = float((g1 - g0).norm() / g0.norm())
    assert rel < 1e-2, rel
    # bf16 on the wire: every gradient element is a bf16 value (round trip of the wire copy)
    assert torch.equal(g1, g1.to(torch.bfloat16).float())
    assert not torch.equal(g0, g1)  # the wire copy really was bf16
    assert ddp1.reducer.last_launch_order() == list(range(ddp1.reducer.num_buckets))


def test_last_bucket_cap_layout_and_grads(gpu, det):
    x, y = _data(gpu, n=8, hw=64)
    ddp0, opt0 = _build(gpu, force=True)
    ref = _train(ddp0, opt0, x, y, steps=1)
    n0 = ddp0.reducer.num_buckets
    del ddp0, opt0
    ddp1, opt1 = _build(gpu, force=True, last_mb=1.0)
    got = _train(ddp1, opt1, x, y, steps=1)
    assert ddp1.reducer.num_buckets == n0 + 1
    assert ddp1.bucket_bytes[-1] <= 1 << 20
    assert ddp1.reducer.last_launch_order() == list(range(n0 + 1))
    # splitting the tail keeps the readiness order, so the flat layout is unchanged
    assert torch.equal(ref[0][0], got[0][0])


def test_rccl_world1_collectives(gpu, native_ext):
    from pytorch_distributed_tutorials_amd.parallel import comm as pcomm
    c = pcomm.native_comm(gpu)
    assert c.world == 1 and c.rank == 0
    x = torch.randn(4096, device=gpu)
    out = torch.empty(4096, device=gpu)
    c.reduce_scatter(x, out, "sum")
    back = torch.empty(4096, device=gpu)
    c.all_gather(out, back)
    c.all_reduce(back, "avg")
    c.broadcast(back, 0)
    c.current_wait_comm()
    torch.cuda.synchronize()
    assert torch.equal(back, x)
    xb = x.to(torch.bfloat16)
    c.all_reduce(xb, "max")
    c.current_wait_comm()
    assert torch.equal(xb, x.to(torch.bfloat16))
    c.barrier()


def _py(code, timeout=120, **env_extra):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.update(env_extra)
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, timeout=timeout,
                          capture_output=True, text=True)


def test_rccl_init_times_out_when_peer_never_joins(gpu):
    # rank 0 of a 2-rank communicator whose rank 1 never calls init: the deadline-bounded init
    # (helper-thread init of a blocking communicator, or PDT_RCCL_NONBLOCKING=1 polling) must give
    # up at its deadline with a clear error (a bare ncclCommInitRank would wait forever)
    code = (
        "import time, torch\n"
        "from pytorch_distributed_tutorials_amd.ops import _ext\n"
        "C = _ext.native()\n"
        "t0 = time.time()\n"
        "try:\n"
        "    C.RcclComm(C.RcclComm.unique_id(), 0, 2, 0, init_timeout=4.0)\n"
        "    print('BUILT')\n"
        "except RuntimeError as e:\n"
        "    print('ERR', round(time.time() - t0, 1), e)\n")
    r = _py(code, timeout=150)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith(("ERR", "BUILT"))][-1]
    assert line.startswith("ERR"), line
    assert "init timed out" in line and "never joined" in line, line
    assert 3.5 <= float(line.split()[1]) < 60, line


def test_rccl_collective_timeout_aborts_and_raises(gpu):
    # a collective that does not complete within op_timeout (a stalled peer, simulated by a
    # sleeping host callback on the comm stream: no GPU kernel spins) -> the monitor aborts the
    # communicator, records the error, and every later call raises it
    code = (
        "import time, torch\n"
        "from pytorch_distributed_tutorials_amd.ops import _ext\n"
        "C = _ext.native()\n"
        "c = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0, init_timeout=30.0, op_timeout=1.0)\n"
        "x = torch.ones(1024, device='cuda')\n"
        "c.all_reduce(x, 'sum'); c.synchronize(); assert c.healthy\n"
        "c.inject_delay(4.0)\n"
        "time.sleep(2.5)\n"
        "print('HEALTHY', c.healthy)\n"
        "print('ERROR', c.error)\n"
        "try:\n"
        "    c.all_reduce(x, 'sum'); print('NO_RAISE')\n"
        "except RuntimeError as e:\n"
        "    print('RAISED', e)\n"
        "time.sleep(2.5)\n")
    r = _py(code)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = r.stdout
    assert "HEALTHY False" in out, out
    assert "did not complete within" in out, out
    assert "RAISED" in out and "unusable" in out, out
    assert "[rccl] rank 0:" in r.stderr


def test_rccl_collective_timeout_exits_process(gpu):
    # exit_on_error (default when world > 1): the monitor ends the process with the watchdog's
    # exit code so the launcher's fail-fast tears the job down
    code = (
        "import time, torch\n"
        "from pytorch_distributed_tutorials_amd.ops import _ext\n"
        "C = _ext.native()\n"
        "c = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0, op_timeout=1.0, exit_on_error=True)\n"
        "c.inject_delay(3.0)\n"
        "time.sleep(20)\n"
        "print('STILL_ALIVE')\n")
    r = _py(code)
    assert r.returncode == 124, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "STILL_ALIVE" not in r.stdout
    assert "did not complete within" in r.stderr


def test_rccl_channel_bounds(gpu):
    # the per-communicator RCCL channel knob (ncclConfig_t minCTAs/maxCTAs) is accepted and the
    # communicator still reduces correctly
    from pytorch_distributed_tutorials_amd.ops import _ext
    C = _ext.native()
    c = C.RcclComm(C.RcclComm.unique_id(), 0, 1, gpu.index, min_channels=4, max_channels=8)
    x = torch.randn(1 << 16, device=gpu)
    y = x.clone()
    c.all_reduce(y, "sum")
    c.synchronize()
    assert torch.equal(x, y) and c.healthy and c.init_seconds >= 0


def test_bn_counter_banks_never_shared(gpu):
    # a 9th stream must not share a completion-counter bank with another stream; it
    # takes the two-launch BN reduction path instead, and the results stay bitwise equal
    from pytorch_distributed_tutorials_amd.ops import _ext
    C = _ext.native()
    streams = [torch.cuda.Stream(device=gpu) for _ in range(12)]
    banks = [C.bn_counter_bank(s.cuda_stream) for s in streams]
    used = [b for b in banks if b >= 0]
    assert len(used) == len(set(used)), banks          # no bank handed out twice
    assert banks.count(-1) >= 12 - 8                   # streams past the 8 banks get none
    # a BN finalize over many groups on a bank-less stream equals the same one on a banked stream
    K, G = 256, 1200
    part = torch.rand(G, 2, K, device=gpu)
    gamma = torch.rand(K, device=gpu)
    beta = torch.rand(K, device=gpu)
    outs = []
    banked = [s for s, b in zip(streams, banks) if b >= 0] or [torch.cuda.current_stream(gpu)]
    for s in (streams[banks.index(-1)], banked[0]):
        s.wait_stream(torch.cuda.current_stream(gpu))
        with torch.cuda.stream(s):
            rm = torch.zeros(K, device=gpu)
            rv = torch.ones(K, device=gpu)
            st = C.bn_finalize(part, G * 64, rm, rv, gamma, beta, 0.1, 1e-5)  # > 512 groups: 2-level
        torch.cuda.current_stream(gpu).wait_stream(s)
        outs.append((st.clone(), rm.clone(), rv.clone()))
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


def test_bench_force_comm_json(gpu, tmp_path):
    out = tmp_path / "b.json"
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--force-comm", "--comm-timing",
           "--steps", "2", "--warmup", "1", "--batch", "16", "--image-size", "64",
           "--last-bucket-mb", "2", "--json-out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, timeout=110, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    cfg = res["config"]
    assert cfg["force_comm"] and cfg["comm"]["native_comm"] and cfg["comm"]["reducer"] == "Reducer"
    assert cfg["comm"]["buckets_mb"][-1] <= 2.0
    assert cfg["comm"]["last_step"] is not None
    assert res["value"] > 0 and math.isfinite(cfg["final_loss"])


def test_rccl_abort_spam_while_issuing(gpu):
    # abort() from other threads while a thread issues collectives on the same
    # world-1 communicator.  Every use goes through the abort gate: the issuing thread must end
    # with the recorded error (never a crash / use-after-free), repeatedly, and the process must
    # exit cleanly.  all_reduce and abort release the GIL, so the threads really overlap.
    code = (
        "import threading, time, torch\n"
        "from pytorch_distributed_tutorials_amd.ops import _ext\n"
        "C = _ext.native()\n"
        "x = torch.ones(4096, device='cuda')\n"
        "ok = 0\n"
        "for rnd in range(6):\n"
        "    c = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0, init_timeout=60.0, op_timeout=30.0)\n"
        "    assert c.comm_count() == 1\n"
        "    res = {}\n"
        "    def issue():\n"
        "        n = 0\n"
        "        try:\n"
        "            while True:\n"
        "                c.all_reduce(x, 'sum'); n += 1\n"
        "        except RuntimeError as e:\n"
        "            res['err'] = str(e); res['n'] = n\n"
        "    t = threading.Thread(target=issue); t.start()\n"
        "    time.sleep(0.05 + 0.02 * rnd)\n"
        "    spam = [threading.Thread(target=lambda: [c.abort() for _ in range(200)]) for _ in range(3)]\n"
        "    [s.start() for s in spam]; [s.join() for s in spam]\n"
        "    t.join(timeout=30)\n"
        "    assert not t.is_alive(), 'issuing thread hung'\n"
        "    assert 'abort' in res.get('err', ''), res\n"
        "    assert not c.healthy and c.comm_count() == -1\n"
        "    del c\n"
        "    ok += 1\n"
        "torch.cuda.synchronize()\n"
        "print('ABORT_SPAM_OK', ok, C.RcclComm.version())\n")
    r = _py(code, timeout=150)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ABORT_SPAM_OK 6" in r.stdout, r.stdout


def test_bench_force_comm_reports_diagnostics(gpu, tmp_path):
    # bench.py's JSON carries what RCCL itself reports (ncclCommCount, version,
    # channel bounds) and one untimed step's all-reduce time / exposed tail from the reducer's
    # events, so the driver's first 8-GPU run is diagnosable
    import json
    out = tmp_path / "b.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--arch", "resnet18", "--image-size", "64",
                        "--batch", "32", "--steps", "2", "--warmup", "1", "--force-comm", "--json-out", str(out)],
                       cwd=ROOT, timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    cfg = json.loads(out.read_text())["config"]
    # a world-1 --force-comm run executes the 8-rank bucket layout, tail bucket
    # included (auto_last_bucket_mb planned for 8 ranks), and reports the parameter checksum
    assert cfg["plan_world"] == 8 and cfg["last_bucket_mb"] is not None
    assert cfg["comm"]["buckets_mb"][-1] <= cfg["last_bucket_mb"] + 1e-6
    assert cfg["ranks_identical"] is True
    c = cfg["comm"]
    assert c["backend"] == "rccl" and c["native_comm"] and c["comm_count"] == 1 and c["count_matches_world"]
    assert c["rccl_version"] >= 20000 and c["healthy"]
    assert c["comm_ms"] >= 0 and 0 <= c["exposed_ms"] <= c["comm_ms"] + 1e-3
    assert len(c["channels"]) == 2
