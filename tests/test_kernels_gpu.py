"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Inputs are rounded to bf16 first so the reference sees exactly the kernel's
operands; tolerances cover the fp32-accumulate vs fp32-reference ordering and the
final bf16 rounding of outputs.
"""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_tutorials_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CONV_SHAPES = [
    # N, H, W, C, K, R, S, stride, pad
    (2, 8, 8, 64, 64, 3, 3, 1, 1),
    (2, 8, 8, 64, 128, 1, 1, 2, 0),
    (2, 9, 9, 128, 128, 3, 3, 2, 1),
    (3, 7, 7, 256, 512, 1, 1, 1, 0),
    (4, 56, 56, 64, 256, 1, 1, 1, 0),     # 128x128 tile config
    (8, 32, 32, 64, 64, 3, 3, 1, 1),      # 256x64 tile config
    (2, 14, 14, 256, 256, 3, 3, 1, 1),
    (2, 15, 15, 128, 256, 3, 3, 2, 1),
    (2, 16, 16, 512, 64, 1, 1, 1, 0),
]


def _make(shape, dev, seed=0):
    n, h, w, c, k, r, s, st, pd = shape
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, h, w, c, generator=g).to(torch.bfloat16).to(dev)
    wt = (torch.randn(k, c, r, s, generator=g) / (c * r * s) ** 0.5).to(dev)
    wt = wt.to(torch.bfloat16).float().contiguous(memory_format=torch.channels_last)
    return x, wt


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_fwd_and_stats(gpu, native_ext, shape):
    C = native_ext
    x, w = _make(shape, gpu)
    st, pd = shape[7], shape[8]
    wk = C.pack_weight(w, x.shape[3])
    y, part = C.conv_fwd(x, wk, st, pd, True)
    yr = ref.conv2d_nhwc(x, w, st, pd)
    assert y.shape == yr.shape
    assert _rel_err(y, yr) < 1e-2
    # BN finalize from the epilogue partials
    k = w.shape[0]
    m = yr.numel() // k
    rm = torch.zeros(k, device=gpu)
    rv = torch.ones(k, device=gpu)
    gamma = torch.rand(k, device=gpu) + 0.5
    beta = torch.randn(k, device=gpu)
    stats = C.bn_finalize(part, m, rm, rv, gamma, beta, 0.1, 1e-5)
    mean_r, var_r = ref.bn_batch_stats(yr)
    assert torch.allclose(stats[0], mean_r, atol=2e-3, rtol=1e-2)
    invstd_r = torch.rsqrt(var_r + 1e-5)
    assert torch.allclose(stats[1], invstd_r, rtol=2e-2)
    assert torch.allclose(rm, 0.1 * mean_r, atol=1e-3, rtol=1e-2)
    assert torch.allclose(rv, 0.9 + 0.1 * var_r * m / (m - 1), rtol=1e-2)


def test_conv_fwd_stem(gpu, native_ext):
    C = native_ext
    g = torch.Generator().manual_seed(1)
    img = torch.randn(2, 3, 32, 32, generator=g).to(gpu)
    x = C.image_to_nhwc(img)
    assert x.shape == (2, 32, 32, 8)
    assert torch.equal(x[..., :3].float(), img.permute(0, 2, 3, 1).to(torch.bfloat16).float())
    assert x[..., 3:].abs().max().item() == 0
    w = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(gpu).to(torch.bfloat16).float()
    w = w.contiguous(memory_format=torch.channels_last)
    wk = C.pack_weight(w, 8)
    y, _ = C.conv_fwd(x, wk, 2, 3, False)
    yr = ref.conv2d_nhwc(x, w, 2, 3)
    assert _rel_err(y, yr) < 1e-2
    # wgrad of the stem (C padded to 8 internally, sliced back to 3)
    dy = torch.randn(yr.shape, generator=g).to(torch.bfloat16).to(gpu)
    dw = C.conv_wgrad(dy, x, list(w.shape), 2, 3)
    dwr = ref.conv2d_nhwc_wgrad(dy, x, w.shape, 2, 3)
    assert dw.shape == dwr.shape
    assert _rel_err(dw, dwr) < 1e-2


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_dgrad(gpu, native_ext, shape):
    C = native_ext
    x, w = _make(shape, gpu, seed=3)
    st, pd = shape[7], shape[8]
    yr = ref.conv2d_nhwc(x, w, st, pd)
    g = torch.Generator().manual_seed(5)
    dy = torch.randn(yr.shape, generator=g).to(torch.bfloat16).to(gpu)
    dx = C.conv_dgrad(dy, w, list(x.shape), st, pd)
    dxr = ref.conv2d_nhwc_dgrad(dy, w, x.shape, st, pd)
    assert dx.shape == dxr.shape
    assert _rel_err(dx, dxr) < 1e-2


@pytest.mark.parametrize("deterministic", [False, True])
@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_wgrad(gpu, native_ext, shape, deterministic):
    C = native_ext
    x, w = _make(shape, gpu, seed=7)
    st, pd = shape[7], shape[8]
    yr = ref.conv2d_nhwc(x, w, st, pd)
    g = torch.Generator().manual_seed(9)
    dy = torch.randn(yr.shape, generator=g).to(torch.bfloat16).to(gpu)
    dw = C.conv_wgrad(dy, x, list(w.shape), st, pd, deterministic)
    dwr = ref.conv2d_nhwc_wgrad(dy, x, w.shape, st, pd)
    assert dw.shape == dwr.shape
    if deterministic:
        assert torch.equal(dw, C.conv_wgrad(dy, x, list(w.shape), st, pd, True))
    assert dw.is_contiguous(memory_format=torch.channels_last)
    assert _rel_err(dw, dwr) < 1e-2


@pytest.mark.parametrize("nhwk", [(16, 56, 56, 64), (8, 28, 28, 128), (8, 14, 14, 256), (4, 7, 7, 512), (3, 5, 7, 64)])
def test_bn_act_fwd_column_sums(gpu, native_ext, nhwk):
    """bn_act_fwd(csum=): the same z bit for bit, and per-channel sums of the STORED bf16 z added into
    C.bn_csum_slots() fp32 slots (accumulating over calls: the consumer re-zeroes them) -- the folded weight
    gradient's sum_m x, against an fp64 sum of z."""
    C = native_ext
    g = torch.Generator().manual_seed(21)
    n, h, w, k = nhwk
    y = torch.randn(n, h, w, k, generator=g).to(torch.bfloat16).to(gpu)
    scale = (torch.rand(k, generator=g) + 0.5).to(gpu)
    shift = (0.2 * torch.randn(k, generator=g)).to(gpu)
    z0 = C.bn_act_fwd(y, scale, shift, None, True)
    cs = torch.zeros(C.bn_csum_slots(), k, device=gpu)
    z1 = C.bn_act_fwd(y, scale, shift, None, True, None, None, cs)
    assert torch.equal(z0, z1)
    want = z0.double().sum((0, 1, 2))
    assert torch.allclose(cs.double().sum(0), want, rtol=1e-5, atol=1e-3), (cs.sum(0) - want).abs().max()
    C.bn_act_fwd(y, scale, shift, None, True, None, None, cs)  # accumulates
    assert torch.allclose(cs.double().sum(0), 2 * want, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("relu,res,nhwk", [
    (True, False, (4, 7, 9, 128)), (True, True, (4, 7, 9, 128)), (False, False, (4, 7, 9, 128)),
    # channel-chunked reduction grid (K8 > 32) and a many-row-block case
    (False, False, (16, 7, 7, 2048)), (True, True, (8, 14, 14, 512)), (True, False, (64, 28, 28, 64)),
])
def test_bn_act_fwd_bwd(gpu, native_ext, relu, res, nhwk):
    C = native_ext
    g = torch.Generator().manual_seed(11)
    n, h, w, k = nhwk
    y = torch.randn(n, h, w, k, generator=g).to(torch.bfloat16).to(gpu)
    r = torch.randn(n, h, w, k, generator=g).to(torch.bfloat16).to(gpu) if res else None
    gamma = (torch.rand(k, generator=g) + 0.5).to(gpu)
    beta = torch.randn(k, generator=g).to(gpu)
    mean, var = ref.bn_batch_stats(y)
    invstd = torch.rsqrt(var + 1e-5)
    scale = gamma * invstd
    shift = beta - mean * scale
    z = C.bn_act_fwd(y, scale, shift, r, relu)
    zr = ref.bn_act_fwd(y, mean, invstd, gamma, beta, r, relu, torch.float32)
    assert ((z.float() - zr).abs() / zr.abs().clamp_min(1.0)).max().item() < 1.6e-2  # bf16 output
    stats = torch.stack([mean, invstd, scale, shift]).contiguous()
    dz = torch.randn(n, h, w, k, generator=g).to(torch.bfloat16).to(gpu)
    dyr, dgr, dbr, dresr = ref.bn_act_bwd(dz, z, y, mean, invstd, gamma, relu, True, res, torch.float32)
    modes = ([1, 2] if not res else [1]) if relu else [0]
    for mask in modes:  # 1: mask from z, 2: mask recomputed from y (must agree)
        sums = C.bn_act_bwd_reduce(dz, z, y, stats, mask)
        dy, dres = C.bn_act_bwd_apply(dz, z, y, stats, gamma, sums, mask, True, res)
        assert torch.allclose(sums[0], dbr, rtol=1e-3, atol=1e-2)
        assert torch.allclose(sums[1] * invstd, dgr, rtol=1e-3, atol=1e-2)
        assert _rel_err(dy, dyr) < 1e-2
        if res:
            assert _rel_err(dres, dresr) < 1e-2


def test_bn_against_torch_batchnorm(gpu, native_ext):
    """Full BN fwd/bwd semantics vs torch.nn.functional.batch_norm (training)."""
    C = native_ext
    g = torch.Generator().manual_seed(12)
    x = torch.randn(8, 64, 6, 6, generator=g).to(gpu)
    xb = x.to(torch.bfloat16).float().requires_grad_(True)
    gamma = (torch.rand(64, generator=g) + 0.5).to(gpu).requires_grad_(True)
    beta = torch.randn(64, generator=g).to(gpu).requires_grad_(True)
    out = F.relu(F.batch_norm(xb, None, None, gamma, beta, training=True, eps=1e-5))
    gout = torch.randn(out.shape, generator=g).to(gpu)
    out.backward(gout)
    y = xb.detach().permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    mean, var = ref.bn_batch_stats(y)
    invstd = torch.rsqrt(var + 1e-5)
    z = C.bn_act_fwd(y, gamma.detach() * invstd, beta.detach() - mean * gamma.detach() * invstd, None, True)
    assert _rel_err(z.permute(0, 3, 1, 2), out) < 1e-2
    dz = gout.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    sc = gamma.detach() * invstd
    stats = torch.stack([mean, invstd, sc, beta.detach() - mean * sc]).contiguous()
    sums = C.bn_act_bwd_reduce(dz, z, y, stats, 2)
    dy, _ = C.bn_act_bwd_apply(dz, z, y, stats, gamma.detach(), sums, 2, True, False)
    assert _rel_err(dy.permute(0, 3, 1, 2), xb.grad) < 3e-2
    assert _rel_err(sums[1] * invstd, gamma.grad) < 3e-2
    assert _rel_err(sums[0], beta.grad) < 3e-2


def test_maxpool(gpu, native_ext):
    C = native_ext
    g = torch.Generator().manual_seed(13)
    x = torch.randn(2, 17, 16, 64, generator=g)
    x = torch.relu(x).to(torch.bfloat16).to(gpu)  # many exact zeros -> exercises tie-breaking
    y, idx = C.maxpool_fwd(x)
    yr = ref.maxpool3x3s2_fwd(x)
    assert torch.equal(y, yr)
    dy = torch.randn(y.shape, generator=g).to(torch.bfloat16).to(gpu)
    dx = C.maxpool_bwd(dy, idx, x.shape[1], x.shape[2])
    dxr = ref.maxpool3x3s2_bwd(dy, x)
    assert (dx.float() - dxr.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("hw", [(17, 16), (112, 112)])
def test_bn_relu_maxpool_matches_unfused(gpu, native_ext, hw):
    """Fused stem BN + ReLU + max pool == bn_act_fwd then maxpool_fwd, bit for bit (values and
    argmax), and its backward (pooled gradient gathered inside the BN passes) matches
    maxpool_bwd -> bn_act_bwd_reduce/apply (mask mode 2) up to the bf16 rounding of dz."""
    C = native_ext
    g = torch.Generator().manual_seed(21)
    n, (h, w), k = 4, hw, 64
    y = torch.randn(n, h, w, k, generator=g).to(torch.bfloat16).to(gpu)
    gamma = (torch.rand(k, generator=g) + 0.5).to(gpu)
    beta = torch.randn(k, generator=g).to(gpu)
    mean, var = ref.bn_batch_stats(y)
    invstd = torch.rsqrt(var + 1e-5)
    scale = (gamma * invstd).contiguous()
    shift = (beta - mean * scale).contiguous()
    out, idx = C.bn_relu_maxpool(y, scale, shift)
    z = C.bn_act_fwd(y, scale, shift, None, True)
    out_r, idx_r = C.maxpool_fwd(z)
    assert torch.equal(out, out_r) and torch.equal(idx, idx_r)
    stats = torch.stack([mean, invstd, scale, shift]).contiguous()
    dpool = torch.randn(out.shape, generator=g).to(torch.bfloat16).to(gpu)
    dz = C.maxpool_bwd(dpool, idx, h, w)
    sums_r = C.bn_act_bwd_reduce(dz, dz, y, stats, 2)
    dy_r, _ = C.bn_act_bwd_apply(dz, dz, y, stats, gamma, sums_r, 2, True, False)
    sums = C.pool_bn_bwd_reduce(dpool, idx, y, stats)
    dy = C.pool_bn_bwd_apply(dpool, idx, y, stats, gamma, sums, True)
    assert torch.allclose(sums, sums_r, rtol=2e-2, atol=0.5)
    assert _rel_err(dy, dy_r) < 1e-2
    # in-place parameter-gradient accumulation variant
    dgs = torch.ones(k, device=gpu)
    dbs = torch.ones(k, device=gpu)
    sums2 = C.pool_bn_bwd_reduce(dpool, idx, y, stats, dgs, dbs)
    assert torch.equal(sums2, sums)
    assert torch.allclose(dgs, 1 + sums[1] * invstd, rtol=1e-5, atol=1e-5)
    assert torch.allclose(dbs, 1 + sums[0], rtol=1e-5, atol=1e-5)


def test_stem_pool_fused_matches_unfused_model_path(gpu, native_ext, monkeypatch):
    """ResNet-50 stem through the fused BN/ReLU/pool node vs the unfused node + max pool:
    same pooled output, same conv1/bn1 gradients (up to dz's bf16 rounding)."""
    import copy
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.ops import fused
    from pytorch_distributed_tutorials_amd.models import build_model
    torch.manual_seed(3)
    m = build_model("resnet50", num_classes=10).to(gpu).set_impl("native")
    m2 = copy.deepcopy(m)
    x = torch.randn(8, 3, 64, 64, device=gpu)
    a = ops.stem_conv_bn_pool(x, m.conv1, m.bn1, m.maxpool)
    monkeypatch.setattr(fused, "_STEM_POOL", False)
    b = ops.stem_conv_bn_pool(x, m2.conv1, m2.bn1, m2.maxpool)
    assert torch.equal(a, b)
    gout = torch.randn(a.shape, device=gpu).to(torch.bfloat16)
    a.backward(gout)
    b.backward(gout)
    for p1, p2 in [(m.conv1.weight, m2.conv1.weight), (m.bn1.weight, m2.bn1.weight), (m.bn1.bias, m2.bn1.bias)]:
        assert _rel_err(p1.grad, p2.grad) < 2e-2
    assert torch.equal(m.bn1.running_mean, m2.bn1.running_mean)


def test_avgpool(gpu, native_ext):
    C = native_ext
    x = torch.randn(4, 7, 7, 2048, device=gpu).to(torch.bfloat16)
    y = C.avgpool_fwd(x)
    assert torch.allclose(y, x.float().mean((1, 2)), atol=1e-3)
    x2 = torch.randn(3, 3, 5, 40, device=gpu).to(torch.bfloat16)  # odd spatial size, 5 vectors per pixel
    assert torch.allclose(C.avgpool_fwd(x2), x2.float().mean((1, 2)), atol=1e-3)
    dy = torch.randn(4, 2048, device=gpu)
    dx = C.avgpool_bwd(dy, 7, 7)
    assert torch.allclose(dx.float(), (dy / 49)[:, None, None, :].expand(4, 7, 7, 2048), atol=1e-3, rtol=1e-2)


def test_softmax_xent_and_top1(gpu, native_ext):
    C = native_ext
    g = torch.Generator().manual_seed(17)
    logits = (torch.randn(64, 1000, generator=g) * 3).to(gpu)
    labels = torch.randint(0, 1000, (64,), generator=g).to(gpu)
    loss, dl = C.softmax_xent(logits, labels)
    lr_, dlr = ref.softmax_xent(logits, labels)
    assert abs(loss.item() - lr_.item()) < 1e-4
    assert torch.allclose(dl, dlr, atol=1e-6)
    labels[:10] = logits[:10].argmax(1)
    cnt = C.top1_correct(logits, labels)
    assert cnt.item() == (logits.argmax(1) == labels).sum().item()


@pytest.mark.parametrize("nesterov", [False, True])
def test_sgd_flat(gpu, native_ext, nesterov):
    C = native_ext
    n = 10001
    p = torch.randn(n, device=gpu)
    gr = torch.randn(n, device=gpu)
    buf = torch.empty(n, device=gpu)
    p2, b2 = p.clone(), torch.empty(n, device=gpu)
    for first in (True, False):
        C.sgd_step(p, gr, buf, 0.1, 0.9, 0.0, 1e-4, nesterov, first, 1.0)
        ref.sgd_momentum_([p2], [gr], [b2], 0.1, 0.9, 0.0, 1e-4, nesterov, first)
    assert torch.allclose(p, p2, atol=1e-6)
    assert torch.allclose(buf, b2, atol=1e-6)


def test_sgd_flat_without_momentum(gpu, native_ext):
    """momentum 0 (torch.optim.SGD's default): no momentum buffer at all -- p -= lr * (g + wd * p)"""
    C = native_ext
    n = 10001
    p = torch.randn(n, device=gpu)
    gr = torch.randn(n, device=gpu)
    want = p - 0.1 * (gr + 1e-4 * p)
    C.sgd_step(p, gr, None, 0.1, 0.0, 0.0, 1e-4, False, True, 1.0)
    assert torch.allclose(p, want, atol=1e-6)


def test_rccl_comm_single_rank(gpu, native_ext):
    C = native_ext
    comm = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0)
    t = torch.arange(1024, dtype=torch.float32, device=gpu)
    comm.all_reduce(t, "avg")
    comm.broadcast(t, 0)
    comm.current_wait_comm()
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(1024, dtype=torch.float32, device=gpu))


def test_resnet18_native_matches_torch(gpu, native_ext):
    """Native NHWC bf16 model vs the stock fp32 torch model with identical weights."""
    import copy
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    torch.manual_seed(0)
    mt = build_model("resnet18", num_classes=10)
    mn = copy.deepcopy(mt).to(gpu).set_impl("native")
    x = torch.randn(16, 3, 32, 32)
    y = torch.randint(0, 10, (16,))
    lt = F.cross_entropy(mt(x), y)
    lt.backward()
    ln = ops.cross_entropy(mn(x.to(gpu)), y.to(gpu))
    ln.backward()
    assert abs(ln.item() - lt.item()) < 5e-2 * max(1.0, abs(lt.item()))
    for (name, pt), (_, pn) in zip(mt.named_parameters(), mn.named_parameters()):
        a, b = pn.grad.float().cpu().flatten(), pt.grad.flatten()
        cos = torch.nn.functional.cosine_similarity(a, b, dim=0).item()
        # bf16 activations at random init: the CPU model with bf16-rounded activations
        # (same algorithm) lands at ~0.93 for the stem vs fp32, so 0.85 is the noise floor
        assert cos > 0.85, f"{name}: cosine {cos}"
    for (name, bt), (_, bn) in zip(mt.named_buffers(), mn.named_buffers()):
        assert torch.allclose(bn.float().cpu(), bt.float(), atol=5e-2, rtol=5e-2), name


@pytest.mark.parametrize("arch,idx", [("resnet50", (1, 0)), ("resnet50", (1, 1)), ("resnet50", (2, 0)),
                                      ("resnet18", (2, 0))])
def test_residual_block_matches_unit_path(gpu, native_ext, arch, idx):
    """The fused block autograd node == the per-unit conv_bn composition (same kernels)."""
    import copy
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    torch.manual_seed(0)
    m = build_model(arch).to(gpu).set_impl("native")
    blk = getattr(m, f"layer{idx[0]}")[idx[1]]
    blk2 = copy.deepcopy(blk)
    cin = blk.conv1.in_channels
    x = torch.randn(4, 16, 16, cin, device=gpu).to(torch.bfloat16).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    out = blk.forward_native(x)                       # fused block node
    chain = [(blk2.conv1, blk2.bn1), (blk2.conv2, blk2.bn2)]
    if hasattr(blk2, "conv3"):
        chain.append((blk2.conv3, blk2.bn3))
    ident = x2
    if blk2.downsample is not None:
        ident = ops.conv_bn(x2, blk2.downsample[0], blk2.downsample[1], relu=False)
    h = x2
    for i, (c, b) in enumerate(chain):
        h = ops.conv_bn(h, c, b, relu=True, residual=ident if i == len(chain) - 1 else None)
    assert torch.equal(out, h)
    g = torch.randn(out.shape, device=gpu).to(torch.bfloat16)
    out.backward(g)
    h.backward(g)
    assert _rel_err(x.grad, x2.grad) < 1e-2
    for (n1, p1), (n2, p2) in zip(blk.named_parameters(), blk2.named_parameters()):
        assert _rel_err(p1.grad, p2.grad) < 1e-2, n1
    for b1, b2 in zip(blk.buffers(), blk2.buffers()):
        assert torch.equal(b1, b2)


@pytest.mark.parametrize("deterministic", [False, True])
def test_inplace_grad_sinks_match_autograd(gpu, native_ext, deterministic):
    """Block backward writing weight/BN grads straight into the flat buffer (DDP flat space) must
    equal the autograd-returned gradients, including accumulation over two backward passes."""
    import copy
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    from pytorch_distributed_tutorials_amd.utils import seed as seedmod
    old = seedmod._DETERMINISTIC
    seedmod._DETERMINISTIC = deterministic
    try:
        torch.manual_seed(0)
        m1 = build_model("resnet50", num_classes=10).to(gpu).set_impl("native")
        m2 = copy.deepcopy(m1)
        ddp = DistributedDataParallel(m2)   # world 1: flat space, grads sunk in place
        x = torch.randn(2, 3, 64, 64, device=gpu)
        y = torch.randint(0, 10, (2,), device=gpu)
        for _ in range(2):  # no zero_grad in between: gradients must accumulate
            ops.cross_entropy(m1(x), y).backward()
            ops.cross_entropy(ddp(x), y).backward()
        # The flat-buffer path also fuses each BN backward into the producing dgrad epilogue
        # (different fp32 summation order -> occasional 1-ulp bf16 flips of dy that propagate):
        # same math, not bitwise.  BN-parameter gradients at batch 2 are cancellation-dominated
        # sums (a BN feeding another BN has ~zero net mean gradient), so they get a wider bound;
        # a race or a wrong mask would break the global cosine and the weight bounds.
        a_all, b_all = [], []
        for (n1, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
            assert p2.grad is not None, n1
            tol = 3e-2 if p1.dim() > 1 else 0.15
            assert _rel_err(p2.grad, p1.grad) < tol, n1
            a_all.append(p2.grad.float().flatten())
            b_all.append(p1.grad.float().flatten())
        cos = torch.nn.functional.cosine_similarity(torch.cat(a_all), torch.cat(b_all), dim=0).item()
        assert cos > 0.999, cos
    finally:
        seedmod._DETERMINISTIC = old


@pytest.mark.parametrize("mask", [0, 1, 2])
@pytest.mark.parametrize("cfg", [(256, 128, 3, 1, 1), (256, 128, 1, 2, 0), (64, 64, 3, 1, 1)])
def test_conv_dgrad_bn_matches_composition(gpu, native_ext, mask, cfg):
    """dgrad with the producer's BN backward (relu mask + reduction) fused into the epilogue ==
    plain dgrad followed by the standalone BN backward reduction."""
    C = native_ext
    cin, k, r, stride, pad = cfg
    g_ = torch.Generator().manual_seed(5 + mask)
    n, h = 4, 14
    ho = (h + 2 * pad - r) // stride + 1
    dy = torch.randn(n, ho, ho, k, generator=g_).to(gpu).bfloat16()
    w = (torch.randn(k, cin, r, r, generator=g_) * 0.05).to(gpu).contiguous(memory_format=torch.channels_last)
    y = torch.randn(n, h, h, cin, generator=g_).to(gpu).bfloat16()
    mean = torch.randn(cin, generator=g_).to(gpu) * 0.1
    invstd = torch.rand(cin, generator=g_).to(gpu) + 0.5
    gamma = torch.randn(cin, generator=g_).to(gpu)
    scale = gamma * invstd
    shift = torch.randn(cin, generator=g_).to(gpu) * 0.1 - mean * scale
    stats = torch.stack([mean, invstd, scale, shift]).contiguous()
    z = torch.relu(torch.randn(n, h, h, cin, generator=g_)).to(gpu).bfloat16()
    dx = C.conv_dgrad(dy, w, [n, h, h, cin], stride, pad)
    sums_ref = C.bn_act_bwd_reduce(dx, z, y, stats, mask)
    if mask == 1:
        g_ref = torch.where(z.float() > 0, dx.float(), 0.0).bfloat16()
    elif mask == 2:
        on = torch.addcmul(shift, y.float(), scale) > 0  # fma order differs: compare masked set
        g_ref = None
    else:
        g_ref = dx
    g, sums = C.conv_dgrad_bn(dy, w, [n, h, h, cin], stride, pad, None, y, z if mask == 1 else None,
                              stats, mask)
    if g_ref is not None:
        assert torch.equal(g, g_ref)
    else:
        agree = (g.float() == torch.where(on, dx.float(), 0.0)).float().mean().item()
        assert agree > 0.999
    assert torch.allclose(sums, sums_ref, rtol=2e-3, atol=2e-3 * sums_ref.abs().max().item())


def test_block_handoff_with_extra_consumer(gpu, native_ext):
    """Cross-block BN-backward handoff: correct when the block output feeds the next block only
    (fused path) and when it has another consumer too (fallback undoes the deposit)."""
    import copy
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    m1 = build_model("resnet50", num_classes=10).to(gpu).set_impl("native")
    m2 = copy.deepcopy(m1)
    DistributedDataParallel(m2)  # world 1: flat space -> grad sinks -> handoff enabled
    x = torch.randn(4, 56, 56, 64, device=gpu).bfloat16()
    c = torch.randn(4, 56, 56, 256, device=gpu)
    for extra in (False, True):
        for m in (m1, m2):
            for p in m.parameters():
                p.grad = None
            b0, b1 = m.layer1[0], m.layer1[1]
            h0 = b0.forward_native(x)
            h1 = b1.forward_native(h0)
            loss = (h1.float() * c).sum()
            if extra:
                loss = loss + (h0.float() * c).sum() * 0.5
            loss.backward()
        for (n1, p1), (_, p2) in zip(m1.layer1[:2].named_parameters(), m2.layer1[:2].named_parameters()):
            assert p2.grad is not None, n1
            assert _rel_err(p2.grad, p1.grad) < 2e-2, (extra, n1)


def test_weight_mirror_matches_packs(gpu, native_ext):
    """The bf16 conv-weight mirror (written by the fused SGD step + one batched transpose) equals
    the per-layer packs bit for bit, and is refreshed after a torch in-place weight update."""
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.optim import SGD
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    C = native_ext
    torch.manual_seed(0)
    m = build_model("resnet50", num_classes=10).to(gpu).set_impl("native")
    ddp = DistributedDataParallel(m)
    opt = SGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(2, 3, 64, 64, device=gpu)
    y = torch.randint(0, 10, (2,), device=gpu)
    sp = m.conv1.weight._pdt_flat

    def check():
        mir = sp.mirror()
        assert mir.valid()
        n = 0
        for mod in m.modules():
            if isinstance(mod, torch.nn.Conv2d) and mir.krsc_view(mod.weight) is not None:
                w = mod.weight
                assert torch.equal(mir.krsc_view(w), C.pack_weight(w, w.shape[1]))
                assert torch.equal(mir.crsk_view(w), C.pack_weight_t(w))
                n += 1
        assert n == 52  # every conv but the 3-channel stem

    for _ in range(2):
        opt.zero_grad()
        ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        check()
    with torch.no_grad():
        m.layer2[0].conv2.weight.mul_(0.5)   # torch in-place write: bumps the shared version
    assert not sp.mirror().valid()
    ddp(x)
    check()


def test_stem_superpixel_matches_generic(gpu, native_ext):
    """Super-pixel stem (K = 224 implicit GEMM on a re-laid-out image) == channel-padded generic
    stem (image_to_nhwc + conv_bn): forward output, running stats and parameter gradients."""
    import copy
    from pytorch_distributed_tutorials_amd import ops
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(gpu)
    conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
    bn = torch.nn.BatchNorm2d(64).to(gpu)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(4, 3, 64, 96, device=gpu)
    z1 = ops.stem_conv_bn(x, conv, bn)
    z2 = ops.conv_bn(ops.image_to_nhwc(x), conv2, bn2, relu=True)
    assert z1.shape == z2.shape == (4, 32, 48, 64)
    assert _rel_err(z1, z2) < 1e-2
    assert torch.allclose(bn.running_mean, bn2.running_mean, atol=1e-3, rtol=1e-2)
    assert torch.allclose(bn.running_var, bn2.running_var, atol=1e-3, rtol=1e-2)
    g = torch.randn(z1.shape, device=gpu).bfloat16()
    z1.backward(g)
    z2.backward(g)
    assert _rel_err(conv.weight.grad, conv2.weight.grad) < 2e-2
    assert _rel_err(bn.weight.grad, bn2.weight.grad) < 2e-2
    assert _rel_err(bn.bias.grad, bn2.bias.grad) < 2e-2


@pytest.mark.parametrize("arch,fp8", [("resnet18", False), ("resnet50", False), ("resnet18", True)])
def test_captured_step_matches_eager(gpu, native_ext, arch, fp8):
    """A training step captured in a HIP graph and replayed == the same steps run eagerly
    (deterministic kernels: bitwise), including the fused SGD and the weight mirror.  fp8: the
    delayed-scaling slot ring cycles every 3 steps, so the step is captured as 3 graphs replayed
    round-robin (CapturedStep period=3); 5 replays cover a full cycle and a wrap."""
    import copy
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.optim import SGD
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    from pytorch_distributed_tutorials_amd.utils import seed as seedmod
    from pytorch_distributed_tutorials_amd.ops.fused import FP8_RING
    from pytorch_distributed_tutorials_amd.utils.graph import CapturedStep
    old = seedmod._DETERMINISTIC
    seedmod._DETERMINISTIC = True
    old_fp8 = ops.fp8_enabled()
    ops.set_fp8(fp8)
    try:
        torch.manual_seed(0)
        base = build_model(arch, num_classes=10).to(gpu).set_impl("native")
        x = torch.randn(32, 3, 32, 32, device=gpu)
        y = torch.randint(0, 10, (32,), device=gpu)
        runs = []
        for graphed in (False, True):
            m = copy.deepcopy(base)
            ddp = DistributedDataParallel(m)
            opt = SGD(ddp.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)

            def step():
                opt.zero_grad()
                loss = ops.cross_entropy(ddp(x), y)
                loss.backward()
                opt.step()
                return loss
            for _ in range(2):
                step()
            run = CapturedStep(step, warmup=0, period=3 if fp8 else 1,
                               ring=FP8_RING if fp8 else None) if graphed else step
            losses = [float(run()) for _ in range(5 if fp8 else 3)]
            runs.append((losses, [p.detach().clone() for p in m.parameters()]))
        (l0, p0), (l1, p1) = runs
        assert l0 == l1, (l0, l1)
        for a, b in zip(p0, p1):
            assert torch.equal(a, b)
    finally:
        seedmod._DETERMINISTIC = old
        ops.set_fp8(old_fp8)


@pytest.mark.parametrize("n_eval", [1, 3])
def test_captured_fp8_step_with_evaluation_between_replays(gpu, native_ext, n_eval):
    """fp8 under graph replay with eager work in between: an evaluation advances the forward
    slot rings by n_eval steps.  The host ring counters follow the replays (CapturedStep ring),
    so the evaluation uses the slots the device expects; n_eval = 1 leaves the graphs out of phase
    (in_phase() False -> capture again, whose first step must still quantize the weights the
    evaluation already saw), n_eval = 3 keeps them in phase.  Bitwise equal to eager."""
    import copy
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.ops.fused import FP8_RING
    from pytorch_distributed_tutorials_amd.optim import SGD
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    from pytorch_distributed_tutorials_amd.utils import seed as seedmod
    from pytorch_distributed_tutorials_amd.utils.graph import CapturedStep
    old, old_fp8 = seedmod._DETERMINISTIC, ops.fp8_enabled()
    seedmod._DETERMINISTIC = True
    ops.set_fp8(True)
    try:
        torch.manual_seed(0)
        base = build_model("resnet18", num_classes=10).to(gpu).set_impl("native")
        x = torch.randn(32, 3, 32, 32, device=gpu)
        y = torch.randint(0, 10, (32,), device=gpu)
        xe = torch.randn(32, 3, 32, 32, device=gpu)
        runs = []
        for graphed in (False, True):
            m = copy.deepcopy(base)
            ddp = DistributedDataParallel(m)
            opt = SGD(ddp.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)

            def step():
                opt.zero_grad()
                loss = ops.cross_entropy(ddp(x), y)
                loss.backward()
                opt.step()
                return loss
            for _ in range(2):
                step()
            mk = lambda: CapturedStep(step, warmup=0, period=3, ring=FP8_RING)  # noqa: E731
            run = mk() if graphed else step
            losses, recaptures = [], 0
            for i in range(8):
                if i == 4:
                    m.eval()
                    with torch.no_grad():
                        for _ in range(n_eval):
                            ddp(xe)
                    m.train()
                if graphed and not run.in_phase():
                    run = mk()
                    recaptures += 1
                losses.append(float(run().detach()))
            runs.append((losses, [p.detach().clone() for p in m.parameters()], recaptures))
        (l0, p0, _), (l1, p1, rc) = runs
        assert rc == (1 if n_eval % 3 else 0)
        assert l0 == l1, (l0, l1)
        for a, b in zip(p0, p1):
            assert torch.equal(a, b)
    finally:
        seedmod._DETERMINISTIC = old
        ops.set_fp8(old_fp8)


@pytest.mark.parametrize("deterministic", [True, False])
def test_wgrad_into_sink_ignores_uninitialised_workspace(gpu, native_ext, deterministic):
    """Regression: split-K slabs are private partials and must be overwritten, never accumulated
    into, when the result accumulates into a caller-owned gradient buffer (NaN-filled fresh
    allocations make any read of uninitialised workspace visible)."""
    C = native_ext
    old_det = torch.are_deterministic_algorithms_enabled()
    old_fill = torch.utils.deterministic.fill_uninitialized_memory
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = True
    try:
        x = torch.randn(32, 8, 8, 64, device=gpu).bfloat16()
        dy = torch.randn(32, 8, 8, 64, device=gpu).bfloat16()
        want = ref.conv2d_nhwc_wgrad(dy.float(), x.float(), (64, 64, 3, 3), 1, 1)
        sink = torch.full((64, 64, 3, 3), 0.5, device=gpu).contiguous(memory_format=torch.channels_last)
        C.conv_wgrad(dy, x, [64, 64, 3, 3], 1, 1, deterministic, sink)
        assert not torch.isnan(sink).any()
        assert _rel_err(sink - 0.5, want) < 1e-4
    finally:
        torch.use_deterministic_algorithms(old_det)
        torch.utils.deterministic.fill_uninitialized_memory = old_fill


@pytest.mark.parametrize("normalized", [False, True])
@pytest.mark.parametrize("augment", [True, False])
def test_fused_augment_matches_torch_loader(gpu, native_ext, normalized, augment):
    """The fused HIP gather/crop/flip/normalize kernel == the batched torch loader, bit for bit."""
    from pytorch_distributed_tutorials_amd.data import DeviceLoader, TensorImageDataset
    g = torch.Generator().manual_seed(21)
    if normalized:
        imgs = torch.randn(40, 3, 32, 32, generator=g)
    else:
        imgs = torch.randint(0, 256, (40, 3, 32, 32), generator=g, dtype=torch.uint8)
    ds = TensorImageDataset(imgs, torch.randint(0, 10, (40,), generator=g), normalized=normalized)
    kw = dict(batch_size=16, shuffle=True, augment=augment, device=gpu, seed=3)
    fused = list(DeviceLoader(ds, fused=True, **kw))
    plain = list(DeviceLoader(ds, fused=False, **kw))
    assert len(fused) == len(plain) == 3
    for (xa, ya), (xb, yb) in zip(fused, plain):
        assert torch.equal(ya, yb)
        assert xa.dtype == torch.float32 and xa.shape == xb.shape
        assert torch.equal(xa, xb)


def test_relu_bitmask_dgrad_matches_z_mask(gpu, native_ext):
    """bn_act_fwd_mask == bn_act_fwd + packed (z > 0) bits, and the BN-fused dgrad reading the
    bits (mask 3) is bit-identical to reading z (mask 1)."""
    C = native_ext
    g = torch.Generator().manual_seed(31)
    n, h, w_, c, k = 2, 14, 14, 256, 64
    y = torch.randn(n, h, w_, c, generator=g).to(torch.bfloat16).to(gpu)
    res = torch.randn(n, h, w_, c, generator=g).to(torch.bfloat16).to(gpu)
    sc = (torch.rand(c, generator=g) + 0.5).to(gpu)
    sh = torch.randn(c, generator=g).to(gpu)
    z, zm = C.bn_act_fwd_mask(y, sc, sh, res)
    assert torch.equal(z, C.bn_act_fwd(y, sc, sh, res, True))
    bits = (z.reshape(-1, 8) > 0).to(torch.int32) << torch.arange(8, device=gpu, dtype=torch.int32)
    assert torch.equal(zm.to(torch.int32), bits.sum(1))
    dy = torch.randn(n, h, w_, k, generator=g).to(torch.bfloat16).to(gpu)
    wt = (torch.randn(k, c, 1, 1, generator=g) * 0.05).to(gpu).contiguous(memory_format=torch.channels_last)
    addend = torch.randn(n, h, w_, c, generator=g).to(torch.bfloat16).to(gpu)
    stats = torch.stack([torch.randn(c, generator=g) * 0.1, torch.rand(c, generator=g) + 0.5, sc.cpu(),
                         sh.cpu()]).to(gpu)
    g1, s1 = C.conv_dgrad_bn(dy, wt, [n, h, w_, c], 1, 0, addend, y, z, stats, 1)
    g3, s3 = C.conv_dgrad_bn(dy, wt, [n, h, w_, c], 1, 0, addend, y, zm, stats, 3)
    assert torch.equal(g1, g3)
    assert torch.equal(s1, s3)


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_trainer_graph_matches_eager(gpu, native_ext, tmp_path, dtype):
    """train.py --graph (HIP-graph replay of the whole step, eager warm-up and partial batches)
    trains every batch exactly once: same weights as the eager trainer, bit for bit (the default
    deterministic kernels), across an epoch boundary with a partial last batch and an evaluation.
    The checkpoint is written at the start of each epoch, so the one of epoch 2 holds the state
    after epochs 0 and 1.  fp8: three graphs, one per delayed-scaling slot phase."""
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.train import main
    base = ["--arch", "resnet18", "--data", "synthetic-cifar", "--synthetic-samples", "200",
            "--batch-size", "32", "--num_epochs", "3", "--eval-every", "1", "--num-classes", "10",
            "--dtype", dtype]
    old_fp8 = ops.fp8_enabled()
    sds = []
    try:
        for extra, sub in (([], "eager"), (["--graph"], "graph")):
            d = tmp_path / sub
            assert main(base + extra + ["--model_dir", str(d)]) == 0
            sds.append(torch.load(d / "resnet_distributed.pth", weights_only=True))
    finally:
        ops.set_fp8(old_fp8)
    assert sds[0].keys() == sds[1].keys()
    for k in sds[0]:
        assert torch.equal(sds[0][k], sds[1][k]), k


def test_graph_step_recaptures_on_hyperparameter_change(gpu, native_ext):
    """The captured fused-SGD launch bakes lr / momentum / weight decay in as kernel arguments:
    a changed param group must trigger a fresh capture, never a stale replay."""
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.optim import SGD
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    from pytorch_distributed_tutorials_amd.train import _GraphStep
    torch.manual_seed(0)
    m = build_model("resnet18", num_classes=10).to(gpu).set_impl("native")
    ddp = DistributedDataParallel(m)
    opt = SGD(ddp.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    gs = _GraphStep(ddp, ops.cross_entropy, opt)
    x = torch.randn(16, 3, 32, 32, device=gpu)
    y = torch.randint(0, 10, (16,), device=gpu)
    for _ in range(gs.WARMUP + 2):
        gs(x, y)
    first = gs.captured
    assert first is not None and first.calls == 2
    gs(x, y)
    assert gs.captured is first  # unchanged hyperparameters: replay
    for g in opt.param_groups:
        g["lr"] = 0.01
    gs(x, y)
    assert gs.captured is not first and gs.captured.calls == 1
    assert dict(gs.hyper[0])["lr"] == 0.01


@pytest.mark.parametrize("mask", [False, True])
def test_bn_act_fwd_residual_bn_matches_materialised(gpu, native_ext, mask):
    """Projection-shortcut BN applied inside the block-tail apply == applying it in its own pass
    first (bit for bit: the fused kernel rounds the normalised shortcut to bf16 the same way)."""
    C = native_ext
    g = torch.Generator().manual_seed(21)
    y = torch.randn(8, 14, 14, 256, generator=g).to(torch.bfloat16).to(gpu)
    r = torch.randn(8, 14, 14, 256, generator=g).to(torch.bfloat16).to(gpu)
    sc, sh = (torch.rand(256, generator=g) + 0.5).to(gpu), torch.randn(256, generator=g).to(gpu)
    rsc, rsh = (torch.rand(256, generator=g) * 2 - 1).to(gpu), torch.randn(256, generator=g).to(gpu)
    res = C.bn_act_fwd(r, rsc, rsh, None, False)
    if mask:
        z0, m0 = C.bn_act_fwd_mask(y, sc, sh, res)
        z1, m1 = C.bn_act_fwd_mask(y, sc, sh, r, rsc, rsh)
        assert torch.equal(m0, m1)
    else:
        z0 = C.bn_act_fwd(y, sc, sh, res, True)
        z1 = C.bn_act_fwd(y, sc, sh, r, True, rsc, rsh)
    assert torch.equal(z0, z1)


@pytest.mark.parametrize("cfg", [(2, 28, 28, 256, 128, 1, 1, 1, 0),    # bottleneck conv1 (dense dgrad)
                                 (2, 28, 28, 128, 128, 3, 3, 2, 1),    # BasicBlock conv1 (parity classes)
                                 (2, 13, 13, 64, 64, 3, 3, 2, 1)])     # odd extent
def test_compact_stride2_addend(gpu, native_ext, cfg):
    """A stride-2 shortcut gradient passed as a compact [N, ceil(H/2), ceil(W/2), C] map == the same
    values zero-interleaved at full resolution, for plain and BN-fused dgrad."""
    C = native_ext
    n, h, w, c, k, r, s, st, pd = cfg
    g = torch.Generator().manual_seed(22)
    ho, wo = (h + 2 * pd - r) // st + 1, (w + 2 * pd - s) // st + 1
    dy = torch.randn(n, ho, wo, k, generator=g).to(torch.bfloat16).to(gpu)
    wt = (torch.randn(k, c, r, s, generator=g) * 0.05).to(gpu).contiguous(memory_format=torch.channels_last)
    comp = torch.randn(n, (h + 1) // 2, (w + 1) // 2, c, generator=g).to(torch.bfloat16).to(gpu)
    full = torch.zeros(n, h, w, c, dtype=torch.bfloat16, device=gpu)
    full[:, ::2, ::2, :] = comp
    assert torch.equal(C.conv_dgrad(dy, wt, [n, h, w, c], st, pd, comp),
                       C.conv_dgrad(dy, wt, [n, h, w, c], st, pd, full))
    y = torch.randn(n, h, w, c, generator=g).to(torch.bfloat16).to(gpu)
    stats = torch.stack([torch.zeros(c), torch.ones(c), torch.rand(c, generator=g) + 0.5,
                         torch.randn(c, generator=g) * 0.1]).to(gpu).contiguous()
    a = C.conv_dgrad_bn(dy, wt, [n, h, w, c], st, pd, comp, y, None, stats, 2)
    b = C.conv_dgrad_bn(dy, wt, [n, h, w, c], st, pd, full, y, None, stats, 2)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("n,c,v", [(256, 2048, 1000), (32, 512, 10), (7, 72, 33)])
def test_fc_gemms_match_fp32_linear(gpu, native_ext, n, c, v):
    """Hand-written head GEMMs (bf16 MFMA, fp32 accumulate, split-K) vs fp32 F.linear and its
    gradients; dW/db accumulate into given buffers; the dgrad partials feed avgpool_bwd."""
    C = native_ext
    g = torch.Generator().manual_seed(31)
    pooled = torch.randn(n, c, generator=g).to(gpu)
    w = (torch.randn(v, c, generator=g) / c ** 0.5).to(gpu)
    b = torch.randn(v, generator=g).to(gpu)
    logits = C.fc_forward(pooled, w, b)
    assert _rel_err(logits, F.linear(pooled, w, b)) < 1e-2
    dl = (torch.randn(n, v, generator=g) * 1e-2).to(gpu)
    dp, dw, db = C.fc_backward(dl, pooled, w)
    assert _rel_err(dw, dl.t() @ pooled) < 1e-2
    assert torch.allclose(db, dl.sum(0), rtol=1e-5, atol=1e-6)
    assert _rel_err(dp.sum(0), dl @ w) < 1e-2
    dw0, db0 = torch.randn(v, c, device=gpu), torch.randn(v, device=gpu)
    dw1, db1 = dw0.clone(), db0.clone()
    C.fc_backward(dl, pooled, w, dw1, db1)
    assert torch.allclose(dw1, dw0 + dw, rtol=1e-5, atol=1e-6)
    assert torch.allclose(db1, db0 + db, rtol=1e-5, atol=1e-6)
    dx = C.avgpool_bwd(dp, 3, 5)
    ref_dx = ((dl @ w) / 15)[:, None, None, :].expand(n, 3, 5, c)
    assert _rel_err(dx, ref_dx) < 1.5e-2


def test_avgpool_linear_and_ce_autograd(gpu, native_ext):
    from pytorch_distributed_tutorials_amd import ops
    g = torch.Generator().manual_seed(32)
    x = torch.randn(16, 7, 7, 256, generator=g).to(torch.bfloat16).to(gpu).requires_grad_(True)
    w = (torch.randn(100, 256, generator=g) * 0.05).to(gpu).requires_grad_(True)
    b = torch.randn(100, generator=g).to(gpu).requires_grad_(True)
    y = torch.randint(0, 100, (16,), generator=g).to(gpu)
    loss = ops.cross_entropy(ops.avgpool_linear(x, w, b), y) * 3.0   # non-unit upstream gradient
    loss.backward()
    xr = x.detach().float().requires_grad_(True)
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    lr = F.cross_entropy(F.linear(xr.mean((1, 2)), wr, br), y) * 3.0
    lr.backward()
    assert abs(loss.item() - lr.item()) < 1e-2 * lr.item()
    assert _rel_err(w.grad, wr.grad) < 1e-2 and _rel_err(b.grad, br.grad) < 1e-2
    assert _rel_err(x.grad, xr.grad) < 2e-2


@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (3, 64, 96), (2, 62, 250), (1, 40, 300)])
def test_stem_halo_conv_vs_fp32(gpu, native_ext, n, h, w):
    """Halo-staged stem forward (csrc/kernels/stem.hip) vs fp32 conv2d on the same bf16-rounded
    image and weights, plus its per-output-row BN partials (sum, M2) vs fp32; the Wo > 128 case
    falls back to the generic implicit GEMM (row-tile partials)."""
    C = native_ext
    torch.manual_seed(1)
    x = torch.randn(n, 3, h, w, device=gpu)
    wt = (torch.randn(64, 3, 7, 7, device=gpu) * 0.1).contiguous(memory_format=torch.channels_last)
    xsp, y, part, grows = C.stem_conv_fwd(x, wt, 2, 3, True)
    ref = torch.nn.functional.conv2d(x.bfloat16().float(), wt.bfloat16().float(), stride=2, padding=3)
    ho, wo = ref.shape[2], ref.shape[3]
    assert y.shape == (n, ho, wo, 64)
    assert _rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2
    rows = ref.permute(0, 2, 3, 1).reshape(-1, 64)  # [N*Ho*Wo, K] in NHWC row order
    assert grows == (wo if wo <= 128 else grows)
    g = part.shape[0]
    assert g == (rows.shape[0] + grows - 1) // grows
    pad = g * grows - rows.shape[0]
    rr = torch.cat([rows, rows.new_full((pad, 64), float("nan"))]).view(g, grows, 64)
    cnt = (~rr.isnan()).sum(1).float()
    s = torch.nansum(rr, 1)
    mean = s / cnt
    m2 = torch.nansum((rr - mean[:, None, :]) ** 2, 1)
    assert _rel_err(part[:, 0], s) < 1e-2
    assert _rel_err(part[:, 1], m2) < 1e-2


@pytest.mark.parametrize("det", [False, True])
# 24 x 224 and 40 x 64x96: more items than the 512 workgroups, so the next item's halo and raw
# loads are prefetched under the current item's MFMAs (both halo buffers in use)
@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (3, 64, 96), (24, 224, 224), (40, 64, 96)])
def test_stem_bwd_fused_matches_unfused(gpu, native_ext, n, h, w, det):
    """Fused stem backward (BN/pool apply inside the weight gradient, csrc/kernels/stem.hip) vs the
    unfused pool_bn_bwd_apply + stem_wgrad on identical inputs (same bf16 dy values, different
    summation order), and vs an fp32 reference weight gradient of the same bf16 dy."""
    C = native_ext
    torch.manual_seed(2)
    x = torch.randn(n, 3, h, w, device=gpu)
    wt = (torch.randn(64, 3, 7, 7, device=gpu) * 0.1).contiguous(memory_format=torch.channels_last)
    xsp, y, part, grows = C.stem_conv_fwd(x, wt, 2, 3, True)
    gamma = torch.rand(64, device=gpu) + 0.5
    beta = torch.rand(64, device=gpu) - 0.5
    rm, rv = torch.zeros(64, device=gpu), torch.ones(64, device=gpu)
    cnt = y.shape[0] * y.shape[1] * y.shape[2]
    stats = C.bn_finalize(part, cnt, rm, rv, gamma, beta, 0.1, 1e-5, grows)
    pooled, idx = C.bn_relu_maxpool(y, stats[2], stats[3])
    dpool = torch.randn(pooled.shape, device=gpu).bfloat16()
    sums = C.pool_bn_bwd_reduce(dpool, idx, y, stats)
    dy = C.pool_bn_bwd_apply(dpool, idx, y, stats, gamma, sums, True)
    ref = C.stem_wgrad(dy, xsp, [64, 3, 7, 7], det)
    got = C.stem_bwd_fused(dpool, idx, y, stats, gamma, sums, True, xsp, [64, 3, 7, 7], det)
    torch.cuda.synchronize()
    assert _rel_err(got, ref) < 1e-3
    # fp32 reference: weight gradient of the same (bf16) dy on the bf16 image
    xb = x.bfloat16().float().requires_grad_(False)
    w32 = wt.bfloat16().float().requires_grad_(True)
    yy = torch.nn.functional.conv2d(xb, w32, stride=2, padding=3)
    yy.backward(dy.float().permute(0, 3, 1, 2))
    assert _rel_err(got, w32.grad) < 1e-2
    if det:  # deterministic slabs: bitwise repeatable
        again = C.stem_bwd_fused(dpool, idx, y, stats, gamma, sums, True, xsp, [64, 3, 7, 7], det)
        assert torch.equal(got, again)
    # eval-mode apply (k1 * g only)
    dy_e = C.pool_bn_bwd_apply(dpool, idx, y, stats, gamma, sums, False)
    ref_e = C.stem_wgrad(dy_e, xsp, [64, 3, 7, 7], det)
    got_e = C.stem_bwd_fused(dpool, idx, y, stats, gamma, sums, False, xsp, [64, 3, 7, 7], det)
    assert _rel_err(got_e, ref_e) < 1e-3


@pytest.mark.parametrize("n,h,w", [(4, 112, 112), (3, 57, 45)])  # odd sizes: clipped edge windows
def test_stem_pool_argmax_y_reduction(gpu, native_ext, n, h, w):
    """The stem's BN backward reduction from the pooled tensors: bn_relu_maxpool(argmax_y=True)
    also returns u = y at every window's argmax (bitwise a copy of y's element), and the plain
    streaming reduction bn_act_bwd_reduce(dpool, -, u, mask=2) equals the gather over y
    (pool_bn_bwd_reduce) up to fp32 summation order."""
    C = native_ext
    torch.manual_seed(5)
    y = torch.randn(n, h, w, 64, device=gpu).bfloat16()
    scale = torch.randn(64, device=gpu)
    shift = torch.randn(64, device=gpu) * 0.3
    mean = torch.randn(64, device=gpu) * 0.1
    stats = torch.stack([mean, torch.rand(64, device=gpu) + 0.5, scale, shift]).contiguous()
    out, idx = C.bn_relu_maxpool(y, scale, shift)
    out2, idx2, u = C.bn_relu_maxpool(y, scale, shift, True)
    assert torch.equal(out, out2) and torch.equal(idx, idx2)
    ho, wo = out.shape[1], out.shape[2]
    k = idx.long()
    ii = torch.arange(ho, device=gpu).view(1, ho, 1, 1)
    jj = torch.arange(wo, device=gpu).view(1, 1, wo, 1)
    hh = (2 * ii - 1 + k // 3).clamp(0, h - 1)
    ww = (2 * jj - 1 + k % 3).clamp(0, w - 1)
    nn_ = torch.arange(n, device=gpu).view(n, 1, 1, 1).expand_as(k)
    cc = torch.arange(64, device=gpu).view(1, 1, 1, 64).expand_as(k)
    assert torch.equal(u, y[nn_, hh, ww, cc])
    dpool = torch.randn(out.shape, device=gpu).bfloat16()
    ref = C.pool_bn_bwd_reduce(dpool, idx, y, stats)
    got = C.bn_act_bwd_reduce(dpool, u, u, stats, 2)
    torch.cuda.synchronize()
    assert _rel_err(got, ref) < 1e-4


@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 256), (2, 7, 9, 128, 512), (3, 28, 28, 64, 256),
                                   (2, 7, 7, 512, 2048), (9, 32, 32, 128, 512), (16, 56, 56, 256, 1024)])
def test_folded_bn_backward_dgrad_matches_apply_then_dgrad(gpu, native_ext, shape):
    """DgradFold (ops/fused.py, last unit of a bottleneck): dx = [g | z] x [wt*k1 | G]^T + bias with
    G = W^T diag(a) W equals the BN-backward apply (dy = k1 g + a y + b) followed by the 1x1 dgrad,
    against an fp32 reference of that composition; the fused epilogue's BN sums (acc mode) too."""
    C = native_ext
    n, h, w_, c, k = shape
    g_ = torch.Generator().manual_seed(21)
    z_in = torch.relu(torch.randn(n, h, w_, c, generator=g_)).to(torch.bfloat16).to(gpu)
    w = (torch.randn(k, c, 1, 1, generator=g_) / c ** 0.5).to(gpu).contiguous(memory_format=torch.channels_last)
    y, part = C.conv_fwd(z_in, C.pack_weight(w, c), 1, 0, True)
    M = n * h * w_
    gamma = (1 + 0.2 * torch.randn(k, generator=g_)).to(gpu)
    beta = (0.1 * torch.randn(k, generator=g_)).to(gpu)
    stats = C.bn_finalize(part, M, torch.zeros(k, device=gpu), torch.ones(k, device=gpu), gamma, beta, 0.1, 1e-5)
    g = (torch.randn(n, h, w_, k, generator=g_) * (torch.rand(n, h, w_, k, generator=g_) > 0.4)).to(torch.bfloat16).to(gpu)
    sums = C.bn_act_bwd_reduce(g, g, y, stats, 0)
    # the unit before (whose BN the dgrad epilogue reduces): y_prev, its stats, mask 2
    y_prev = torch.randn(n, h, w_, c, generator=g_).to(torch.bfloat16).to(gpu)
    st_prev = torch.stack([torch.zeros(c), torch.ones(c), torch.ones(c) * 0.7, torch.ones(c) * 0.05]).to(gpu).contiguous()
    # reference composition on the native kernels: apply, then BN-fused dgrad
    dy, _ = C.bn_act_bwd_apply(g, g, y, stats, gamma, sums, 0, True, False)
    acc_a = torch.zeros(2, c, device=gpu)
    dx_a, _ = C.conv_dgrad_bn(dy, w, [n, h, w_, c], 1, 0, None, y_prev, None, st_prev, 2, acc=acc_a)
    # folded
    wt = C.pack_weight_t(w).view(c, k)
    wfold, bias = C.bn_fold_weights(wt, stats, gamma, sums, M)
    acc_b = torch.zeros(2, c, device=gpu)
    dx_b, s_b = C.conv_dgrad_bn_fold(g, z_in, wfold, bias, y_prev, None, st_prev, 2, acc_b)
    assert s_b.data_ptr() == acc_b.data_ptr()
    # fp32 reference: BN backward apply in fp32 from the same bf16 g and y, dgrad in fp32, mask 2
    mu, inv = stats[0], stats[1]
    gf, yf = g.float().reshape(-1, k), y.float().reshape(-1, k)
    s0, s1 = gf.sum(0), (gf * (yf - mu)).sum(0)
    k1 = gamma * inv
    dyf = k1 * (gf - s0 / M - (yf - mu) * (s1 * inv * inv / M))
    dxf = (dyf @ w.reshape(k, c).float()).reshape(n, h, w_, c)
    on = (y_prev.float() * st_prev[2] + st_prev[3]) > 0
    dxf = torch.where(on, dxf, 0.0)
    rel = lambda a_, b_: ((a_.float() - b_).norm() / b_.norm()).item()  # noqa: E731
    assert rel(dx_a, dxf) < 1e-2
    assert rel(dx_b, dxf) < 1e-2, (rel(dx_b, dxf), rel(dx_a, dxf))
    assert rel(dx_b, dx_a.float()) < 1e-2
    # the epilogue's BN sums (sum g, sum g*y at mean 0): within 1 % of the summed magnitudes (the sums
    # themselves cancel), and as close to the unfolded path's
    d2, yp = dxf.reshape(-1, c), y_prev.float().reshape(-1, c)
    ref_sums = torch.stack([d2.sum(0), (d2 * yp).sum(0)])
    mag = torch.stack([d2.abs().sum(0), (d2 * yp).abs().sum(0)])
    assert ((acc_b - ref_sums).abs() <= 1e-2 * mag + 1e-6).all(), ((acc_b - ref_sums).abs() / mag).max()
    assert ((acc_a - ref_sums).abs() <= 1e-2 * mag + 1e-6).all(), ((acc_a - ref_sums).abs() / mag).max()
