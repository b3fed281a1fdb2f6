"""CPU tests of the non-kernel plumbing: sampler, bucket planner, model spec,
checkpoint schema, CLI contract, flat parameter space, fused-SGD semantics."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

from pytorch_distributed_tutorials_amd.data import DistributedSampler
from pytorch_distributed_tutorials_amd.models import build_model
from pytorch_distributed_tutorials_amd.optim import SGD
from pytorch_distributed_tutorials_amd.parallel import FlatParamSpace, ddp_bucket_plan
from pytorch_distributed_tutorials_amd.train import build_parser
from pytorch_distributed_tutorials_amd.utils.checkpoint import load_checkpoint, save_checkpoint


# ------------------------------------------------------------------ sampler
@pytest.mark.parametrize("n,world,shuffle,drop_last", [
    (50000, 2, True, False), (10, 3, True, False), (10, 3, False, False), (11, 4, True, True),
    (7, 8, True, False), (100, 1, True, False)])
def test_sampler_matches_torch(n, world, shuffle, drop_last):
    from torch.utils.data.distributed import DistributedSampler as TorchDS
    ds = list(range(n))
    for epoch in (0, 3):
        for r in range(world):
            ours = DistributedSampler(n, num_replicas=world, rank=r, shuffle=shuffle, seed=7,
                                      drop_last=drop_last)
            theirs = TorchDS(ds, num_replicas=world, rank=r, shuffle=shuffle, seed=7, drop_last=drop_last)
            ours.set_epoch(epoch)
            theirs.set_epoch(epoch)
            assert list(iter(ours)) == list(iter(theirs))
            assert len(ours) == len(theirs)


def test_sampler_shards_cover_dataset():
    n, world = 1003, 4
    allidx = []
    for r in range(world):
        allidx += DistributedSampler(n, world, r).indices()
    assert sorted(set(allidx)) == list(range(n))  # padded by wrap-around, covers everything


# ------------------------------------------------------------------ buckets
@pytest.mark.parametrize("arch", ["resnet18", "resnet50", "resnet152"])
def test_bucket_plan_matches_torch(arch):
    m = build_model(arch)
    params = list(m.parameters())
    sizes = [p.numel() * p.element_size() for p in params]
    ours = ddp_bucket_plan(sizes, 25.0, 1.0)
    rev = list(reversed(range(len(params))))
    theirs, _ = dist._compute_bucket_assignment_by_size(
        [params[i] for i in rev], [1 << 20, 25 << 20], [False] * len(params), rev)
    assert ours == [list(b) for b in theirs]


def test_resnet50_bucket_sizes_from_survey():
    m = build_model("resnet50")
    params = list(m.parameters())
    plan = ddp_bucket_plan([p.numel() * 4 for p in params])
    assert [sum(params[i].numel() for i in b) for b in plan] == \
        [2049000, 7875584, 6563840, 6637568, 2431040]


def test_last_bucket_cap_hand_layout():
    MiB = 1 << 20
    # definition order sizes 1..6 MiB -> readiness order 6,5,4,3,2,1 MiB; caps [1, 8] MiB:
    # [6] | [5,4] | [3,2,1]; a 3 MiB tail cap carves [2,1] off the last bucket
    sizes = [k * MiB for k in range(1, 7)]
    assert ddp_bucket_plan(sizes, 8.0, 1.0) == [[5], [4, 3], [2, 1, 0]]
    assert ddp_bucket_plan(sizes, 8.0, 1.0, last_bucket_mb=3.0) == [[5], [4, 3], [2], [1, 0]]
    # a tail cap at or above the last bucket changes nothing; one oversized item stays alone
    assert ddp_bucket_plan(sizes, 8.0, 1.0, last_bucket_mb=6.0) == [[5], [4, 3], [2, 1, 0]]
    assert ddp_bucket_plan(sizes, 8.0, 1.0, last_bucket_mb=0.5) == [[5], [4, 3], [2, 1], [0]]


def test_resnet50_tail_bucket_and_model():
    from pytorch_distributed_tutorials_amd.parallel.buckets import allreduce_us, tail_time_us
    m = build_model("resnet50")
    params = list(m.parameters())
    sizes = [p.numel() * 4 for p in params]
    base = ddp_bucket_plan(sizes)
    capped = ddp_bucket_plan(sizes, last_bucket_mb=2.0)
    # same readiness order (the flat layout does not move), only the tail is split
    assert [i for b in base for i in b] == [i for b in capped for i in b]
    assert len(capped) == len(base) + 1
    tail = sum(sizes[i] for i in capped[-1])
    assert tail <= 2 << 20
    # the exposed tail shrinks with the cap; a 1-link ring is 7x slower than all links
    t_base = tail_time_us([sum(sizes[i] for i in b) for b in base], 8)
    t_cap = tail_time_us([sum(sizes[i] for i in b) for b in capped], 8)
    assert t_cap < t_base
    big = 100 << 20
    assert allreduce_us(big, 8, 1, latency_us=0) == pytest.approx(7 * allreduce_us(big, 8, 7, latency_us=0))
    # 2(n-1)/n * 102.2 MB over one 153 GB/s link = 1.17 ms
    assert allreduce_us(102_228_128, 8, 1, latency_us=0) == pytest.approx(1169, rel=1e-2)


def test_forced_reducer_world1_cpu(native_ext):
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    assert not (dist.is_available() and dist.is_initialized())
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 10, (4,))
    res = []
    for force in (False, True):
        torch.manual_seed(0)
        m = build_model("resnet18", num_classes=10)
        ddp = DistributedDataParallel(m, force_reducer=force, last_bucket_mb=1.0)
        assert (ddp.reducer is not None) == force
        nn.functional.cross_entropy(ddp(x), y).backward()
        res.append(ddp.space.grad_flat.clone())
        if force:
            nb = ddp.reducer.num_buckets
            assert ddp.reducer.last_launch_order() == list(range(nb))
            assert ddp.bucket_info()["forced"]
    assert torch.equal(res[0], res[1])


# -------------------------------------------------------------------- model
@pytest.mark.parametrize("arch,count,keys", [("resnet18", 11689512, 122), ("resnet50", 25557032, 320),
                                             ("resnet152", 60192808, 932)])
def test_model_spec(arch, count, keys):
    m = build_model(arch)
    assert sum(p.numel() for p in m.parameters()) == count
    assert len(m.state_dict()) == keys


def test_native_impl_is_pure_memory_format_change():
    torch.manual_seed(0)
    m = build_model("resnet18")
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    m.set_impl("native")
    assert m.conv1.weight.is_contiguous(memory_format=torch.channels_last)
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd0[k])


def test_native_cpu_forward_matches_torch():
    torch.manual_seed(0)
    m = build_model("resnet18", num_classes=10)
    import copy
    m2 = copy.deepcopy(m).set_impl("native")
    x = torch.randn(3, 3, 32, 32)
    assert torch.allclose(m(x), m2(x), atol=1e-4, rtol=1e-4)
    for b1, b2 in zip(m.buffers(), m2.buffers()):
        assert torch.allclose(b1.float(), b2.float(), atol=1e-5)


# --------------------------------------------------------------- flat + sgd
def test_flat_space_and_fused_sgd_semantics():
    torch.manual_seed(0)
    m1 = build_model("resnet18", num_classes=10).set_impl("native")
    import copy
    m2 = copy.deepcopy(m1)
    sp = FlatParamSpace(list(reversed(list(m1.parameters()))))
    assert sp.numel == sum(p.numel() for p in m1.parameters())
    assert m1.conv1.weight.is_contiguous(memory_format=torch.channels_last)
    o1 = SGD(m1.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    o2 = torch.optim.SGD(m2.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(2, 3, 32, 32)
    y = torch.tensor([1, 2])
    for _ in range(2):
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad()
            nn.functional.cross_entropy(m(x), y).backward()
            o.step()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p1, p2, atol=1e-5)
    assert all(p.grad is g for p, g in zip(sp.params, sp.grad_views))
    # optimizer state round trip keeps torch's format
    st = o1.state_dict()
    assert all("momentum_buffer" in v for v in st["state"].values())


# --------------------------------------------------------------- checkpoint
def test_checkpoint_schema_and_roundtrip(tmp_path):
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    m = build_model("resnet18").set_impl("native")
    ddp = DistributedDataParallel(m)
    opt = SGD(ddp.parameters(), lr=0.1, momentum=0.9)
    path = str(tmp_path / "saved_models" / "resnet_distributed.pth")
    save_checkpoint(ddp, path, opt, epoch=10)
    sd = torch.load(path, weights_only=True)
    assert len(sd) == 122
    assert all(k.startswith("module.") for k in sd)
    assert sd["module.conv1.weight"].shape == (64, 3, 7, 7)
    assert sd["module.conv1.weight"].is_contiguous()
    assert sd["module.fc.weight"].shape == (1000, 512)
    assert sd["module.bn1.num_batches_tracked"].dtype == torch.int64
    n_f32 = sum(1 for v in sd.values() if v.dtype == torch.float32)
    n_i64 = sum(1 for v in sd.values() if v.dtype == torch.int64)
    assert (n_f32, n_i64) == (102, 20)
    # loads into a plain (torchvision-layout) model after stripping the prefix
    plain = build_model("resnet18")
    plain.load_state_dict({k[len("module."):]: v for k, v in sd.items()})
    # and back into a fresh DDP-wrapped native model, with the training sidecar
    m2 = build_model("resnet18").set_impl("native")
    ddp2 = DistributedDataParallel(m2)
    opt2 = SGD(ddp2.parameters(), lr=0.1, momentum=0.9)
    ep = load_checkpoint(ddp2, path, torch.device("cpu"), opt2)
    assert ep == 10
    for a, b in zip(ddp.parameters(), ddp2.parameters()):
        assert torch.equal(a, b)


# ---------------------------------------------------------------------- CLI
def test_cli_contract(monkeypatch):
    p = build_parser()
    a = p.parse_args([])
    assert (a.num_epochs, a.batch_size, a.learning_rate, a.seed) == (10000, 256, 0.01, 0)
    assert (a.model_dir, a.model_filename, a.resume) == ("saved_models", "resnet_distributed.pth", False)
    assert p.parse_args(["--local_rank", "3"]).local_rank == 3
    assert p.parse_args(["--local-rank=2"]).local_rank == 2
    assert p.parse_args(["--learning_rate", "0.1"]).learning_rate == 0.1
    from pytorch_distributed_tutorials_amd.utils.env import dist_env
    monkeypatch.setenv("LOCAL_RANK", "5")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "5")
    assert dist_env(None).local_rank == 5
    assert dist_env(1).local_rank == 1


# ------------------------------------------------------------------ bench.py contract, N>1
def test_bench_two_ranks_gloo(tmp_path):
    """``bench.py --gpus 2`` self-launches torchrun, takes the max time over ranks and has rank 0
    print one JSON line with the whole-job aggregate (driver contract)."""
    import json
    import subprocess
    import sys
    from conftest import free_port
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_PORT=str(free_port()), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    out = tmp_path / "b.json"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--arch", "resnet18",
                        "--image-size", "32", "--num-classes", "10", "--batch", "4", "--steps", "2",
                        "--warmup", "1", "--impl", "torch", "--backend", "gloo", "--json-out", str(out)],
                       cwd=root, env=env, timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d == json.loads(out.read_text())
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 8 and d["config"]["parallelism"] == "dp2"
    assert abs(d["value"] - 8 * 2 / (d["ms_per_step"] * 2 / 1000.0)) / d["value"] < 1e-2
    # every rank ends with bit-identical parameters (all-gathered checksum)
    assert d["config"]["ranks_identical"] is True and isinstance(d["config"]["param_checksum"], int)


def test_bench_two_ranks_native_reports_comm_diagnostics(tmp_path):
    """the scaling run's JSON must be diagnosable -- the rank count the
    communicator itself reports (vs WORLD_SIZE), backend, wire format and bucket sizes ride in
    config.comm (native impl, 2 gloo ranks on the CPU; the RCCL twin is
    tests/test_rccl_gpu.py::test_bench_force_comm_reports_diagnostics)."""
    import json
    import subprocess
    import sys
    from conftest import free_port
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_PORT=str(free_port()), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--arch", "resnet18",
                        "--image-size", "32", "--num-classes", "10", "--batch", "4", "--steps", "2",
                        "--warmup", "1", "--impl", "native", "--backend", "gloo"],
                       cwd=root, env=env, timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    cfg = json.loads(lines[0])["config"]
    assert cfg["ranks_identical"] is True and cfg["plan_world"] == 2
    c = cfg["comm"]
    assert c["world_size"] == 2 and c["comm_count"] == 2 and c["count_matches_world"]
    assert c["backend"] == "python-gloo" and c["wire_dtype"] == "fp32"
    assert len(c["buckets_mb"]) >= 2 and all(b > 0 for b in c["buckets_mb"])
    assert "WARNING" not in r.stdout


def test_bn_counter_list_cache_follows_mode_and_surgery():
    """bump_bn_counters caches the model's BatchNorm list (host issue); the cached counters follow
    train()/eval() and a replaced counter buffer, and forget_bn_modules picks up new modules."""
    import torch.nn as nn
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    m = build_model("resnet18", num_classes=10)
    nbn = sum(isinstance(x, nn.BatchNorm2d) for x in m.modules())
    assert len(ops.bump_bn_counters(m).counters) == nbn
    m.eval()
    assert ops.bump_bn_counters(m).counters == []
    m.train()
    c = ops.bump_bn_counters(m).counters
    assert len(c) == nbn and c[0] is m.bn1.num_batches_tracked
    m.bn1.num_batches_tracked = torch.zeros((), dtype=torch.long)  # re-homed buffer
    assert ops.bump_bn_counters(m).counters[0] is m.bn1.num_batches_tracked
    m.bn1 = nn.BatchNorm2d(64)  # module surgery: invisible until forgotten
    ops.forget_bn_modules(m)
    assert ops.bump_bn_counters(m).counters[0] is m.bn1.num_batches_tracked


def test_sgd_flat_space_check_cache_tracks_the_param_list():
    """optim.SGD caches 'this group is exactly one flat space' per group (host issue); a changed
    member invalidates it, and nothing of the cache leaks into state_dict()."""
    from pytorch_distributed_tutorials_amd.optim import SGD

    class _Space:
        pass

    ps = [nn.Parameter(torch.zeros(2)) for _ in range(3)]
    sp = _Space()
    sp.params = list(ps)
    for p in ps:
        p._pdt_flat = sp
    opt = SGD(ps, lr=0.1, momentum=0.9)
    g = opt.param_groups[0]
    assert opt._flat_space_of(g) is sp
    assert opt._flat_space_of(g) is sp  # cached path
    other = nn.Parameter(torch.zeros(2))
    other._pdt_flat = sp
    g["params"][2] = other  # same length, different member: not the space any more
    assert opt._flat_space_of(g) is None
    g["params"][2] = ps[2]
    assert opt._flat_space_of(g) is sp
    assert set(opt.state_dict()["param_groups"][0]) == set(g) - {"params"} | {"params"}
    assert not any(k.startswith("_pdt") for k in opt.state_dict()["param_groups"][0])


def test_auto_last_bucket_cap_from_tail_model():
    # DDP's default last_bucket_mb="auto": the tail model caps the last-launched bucket (stem and
    # early layer1 gradients, produced at the very end of backward) so its exposed all-reduce
    # shrinks; at world 1 there is no all-reduce and the torch layout is kept
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.parallel.buckets import auto_last_bucket_mb, tail_time_us
    sizes = [p.numel() * 4 for p in build_model("resnet50", num_classes=1000).parameters()]
    assert auto_last_bucket_mb(sizes, 1) is None
    for world in (2, 8):
        cap = auto_last_bucket_mb(sizes, world)
        assert cap is not None and cap <= 2.0
        base = [sum(sizes[i] for i in b) for b in ddp_bucket_plan(sizes)]
        capped = [sum(sizes[i] for i in b) for b in ddp_bucket_plan(sizes, last_bucket_mb=cap)]
        assert capped[-1] <= cap * 2**20 and sum(capped) == sum(base)
        assert tail_time_us(capped, world, 7) < tail_time_us(base, world, 7)


def test_critical_priority_policy(monkeypatch):
    """Normal priority by default since round 5 (profiles/r7q_priority_ab.jsonl: the plain bf16
    step is faster without it and the N>1 path matches it); only the eager fp8 step without
    collectives keeps it; PDT_MAIN_PRIO forces it either way."""
    from pytorch_distributed_tutorials_amd.ops import streams
    monkeypatch.delenv("PDT_MAIN_PRIO", raising=False)
    assert not streams.critical_priority_wanted(collective=False, graph=False)
    assert not streams.critical_priority_wanted(collective=True, graph=False)
    assert not streams.critical_priority_wanted(collective=False, graph=True)
    assert streams.critical_priority_wanted(collective=False, graph=False, fp8=True)
    assert not streams.critical_priority_wanted(collective=True, graph=False, fp8=True)
    monkeypatch.setenv("PDT_MAIN_PRIO", "0")
    assert not streams.critical_priority_wanted(collective=False, graph=False)
    monkeypatch.setenv("PDT_MAIN_PRIO", "1")
    assert streams.critical_priority_wanted(collective=True, graph=True)
    # CPU device: nothing to make current
    assert streams.use_critical_stream(torch.device("cpu")) is None


def test_fp8_dgrad_policy(monkeypatch):
    """fp8 input gradient: whole 128-byte K-steps per tap, or any 16-multiple at stride 1
    (the generic loader's dgrad tap walk covers one parity class only)."""
    from pytorch_distributed_tutorials_amd.ops import fused
    monkeypatch.setattr(fused, "_FP8_DGRAD_NARROW", True)
    assert fused._fp8_dgrad_ok(256, 2) and fused._fp8_dgrad_ok(128, 1)
    assert fused._fp8_dgrad_ok(64, 1) and fused._fp8_dgrad_ok(80, 1)
    assert not fused._fp8_dgrad_ok(64, 2) and not fused._fp8_dgrad_ok(72, 1)
    monkeypatch.setattr(fused, "_FP8_DGRAD_NARROW", False)
    assert not fused._fp8_dgrad_ok(64, 1) and fused._fp8_dgrad_ok(128, 1)
