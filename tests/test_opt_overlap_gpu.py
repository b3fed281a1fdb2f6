"""Optimizer in backward: the fused SGD runs per gradient bucket inside
backward -- behind each bucket's all-reduce on the comm stream, or in one process on the reducer's
local stream as soon as the bucket's gradients are final -- and ``step()`` only joins.

Pinned here: parameters and momentum after several steps are BITWISE equal to the classic
post-backward flat SGD (deterministic mode, so both runs see bit-identical gradients), in local
mode and behind the forced world-1 RCCL communicator; and the contract violations that would make
the early update wrong (a second backward without step(), an LR change or a gradient edit between
backward and step) raise instead of training silently differently.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def det_mode():
    from pytorch_distributed_tutorials_amd.utils import seed
    old = seed._DETERMINISTIC
    yield seed
    seed.set_random_seeds(0, deterministic=old)


def _build(gpu, overlap, force=False, arch="resnet50"):
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.optim import SGD
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    model = build_model(arch, num_classes=100, impl="native").to(gpu)
    model.set_impl("native")
    ddp = DistributedDataParallel(model, force_reducer=force)
    opt = SGD(ddp.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4, overlap=overlap)
    return ddp, opt


def _data(gpu, steps, batch=8, size=64):
    g = torch.Generator().manual_seed(7)
    xs = [torch.randn(batch, 3, size, size, generator=g).to(gpu) for _ in range(steps)]
    ys = [torch.randint(0, 100, (batch,), generator=g).to(gpu) for _ in range(steps)]
    return xs, ys


def _train(ddp, opt, xs, ys):
    from pytorch_distributed_tutorials_amd import ops
    for x, y in zip(xs, ys):
        opt.zero_grad()
        loss = ops.cross_entropy(ddp(x), y)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    return loss.item()


@pytest.mark.parametrize("force", [False, True], ids=["local", "rccl_world1"])
def test_overlap_bitwise_equals_post_backward_step(gpu, det_mode, force):
    det_mode.set_random_seeds(0, deterministic=True)
    xs, ys = _data(gpu, 6)
    ddp_a, opt_a = _build(gpu, overlap=False, force=force)
    la = _train(ddp_a, opt_a, xs, ys)
    ddp_b, opt_b = _build(gpu, overlap=None, force=force)
    assert opt_b._overlap_owner is not None, "the per-bucket update did not attach"
    assert ddp_b.reducer is not None and ddp_b.reducer.num_buckets >= 2
    if not force:
        assert ddp_b.reducer.local
    lb = _train(ddp_b, opt_b, xs, ys)
    assert la == lb
    pa, pb = ddp_a.space.param_flat, ddp_b.space.param_flat
    assert torch.equal(pa, pb), (pa - pb).abs().max().item()
    ma = opt_a._flat_bufs[id(ddp_a.space)]
    mb = opt_b._flat_bufs[id(ddp_b.space)]
    assert torch.equal(ma, mb)
    # the bf16 weight mirror the per-bucket kernel wrote is the one the classic step writes
    assert torch.equal(ddp_a.space.mirror().krsc, ddp_b.space.mirror().krsc)
    # torch-format optimizer state: momentum_buffer entries are views of the flat buffer
    sd = opt_b.state_dict()
    assert len(sd["state"]) == len(list(ddp_b.parameters()))


def test_overlap_contract_violations_raise(gpu):
    from pytorch_distributed_tutorials_amd import ops
    xs, ys = _data(gpu, 3)
    ddp, opt = _build(gpu, overlap=None, arch="resnet18")
    assert opt._overlap_owner is not None
    # a second synced backward before step()
    loss = ops.cross_entropy(ddp(xs[0]), ys[0])
    loss.backward()
    with pytest.raises(RuntimeError, match="step\\(\\) was not called"):
        ddp(xs[1])
    ddp2, opt2 = _build(gpu, overlap=None, arch="resnet18")
    # an LR change between backward and step()
    loss = ops.cross_entropy(ddp2(xs[0]), ys[0])
    loss.backward()
    opt2.param_groups[0]["lr"] = 0.5
    with pytest.raises(RuntimeError, match="hyperparameters changed"):
        opt2.step()
    # a gradient edit (clipping) between backward and step()
    ddp3, opt3 = _build(gpu, overlap=None, arch="resnet18")
    loss = ops.cross_entropy(ddp3(xs[0]), ys[0])
    loss.backward()
    torch.nn.utils.clip_grad_norm_(ddp3.parameters(), 0.1)
    with pytest.raises(RuntimeError, match="gradients were modified"):
        opt3.step()
    # no_sync() backwards are not updated; the synced one after them applies the whole step
    ddp4, opt4 = _build(gpu, overlap=None, arch="resnet18")
    p0 = ddp4.space.param_flat.clone()
    with ddp4.no_sync():
        ops.cross_entropy(ddp4(xs[0]), ys[0]).backward()
    torch.cuda.synchronize()
    assert torch.equal(p0, ddp4.space.param_flat)
    ops.cross_entropy(ddp4(xs[1]), ys[1]).backward()
    opt4.step()
    torch.cuda.synchronize()
    assert not torch.equal(p0, ddp4.space.param_flat)
