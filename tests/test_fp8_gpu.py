"""FP8 (OCP e4m3 / e5m2) MX-rate MFMA path: operand lane map, scale semantics, kernels.

The lane map of v_mfma_scale_f32_16x16x128_f8f6f4 is pinned with exact small-integer
data (every product and sum is exact in fp32), so a wrong map cannot pass by rounding.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lane_maps(name):
    """(lane, byte) -> (row/col, k) under a hypothesis for the 16x16x128 operand layout."""
    lanes = torch.arange(64)[:, None].expand(64, 32)
    j = torch.arange(32)[None, :].expand(64, 32)
    rc = lanes & 15
    q = lanes >> 4
    if name == "contig32":      # k = 32*(lane/16) + j
        k = 32 * q + j
    elif name == "halves":      # bytes 0-15 -> k = 16q + j, bytes 16-31 -> 64 + 16q + (j-16)
        k = torch.where(j < 16, 16 * q + j, 64 + 16 * q + (j - 16))
    else:                       # 8-byte groups interleaved over the lane groups
        k = (j >> 3) * 32 + 8 * q + (j & 7)
    return rc, k


def _reference(a_regs, b_regs, hyp):
    rc, k = _lane_maps(hyp)
    A = torch.zeros(16, 128)
    B = torch.zeros(128, 16)
    A[rc.reshape(-1), k.reshape(-1)] = a_regs.reshape(-1)
    B[k.reshape(-1), rc.reshape(-1)] = b_regs.reshape(-1)
    D = A @ B
    lanes = torch.arange(64)
    out = torch.zeros(64, 4)
    for e in range(4):
        out[:, e] = D[(lanes >> 4) * 4 + e, lanes & 15]
    return out


def _fp8_bytes(vals, dtype):
    return vals.to(dtype).view(torch.uint8)


@pytest.mark.parametrize("fmt", [(0, 0), (1, 0), (0, 1)])
def test_mfma_f8_lane_map_and_unit_scale(gpu, native_ext, fmt):
    C = native_ext
    g = torch.Generator().manual_seed(3)
    dts = {0: torch.float8_e4m3fn, 1: torch.float8_e5m2}
    av = torch.randint(-4, 5, (64, 32), generator=g).float()
    bv = torch.randint(-4, 5, (64, 32), generator=g).float()
    a = _fp8_bytes(av, dts[fmt[0]]).to(gpu)
    b = _fp8_bytes(bv, dts[fmt[1]]).to(gpu)
    d_unit = C.mfma_f8_probe(a, b, fmt[0], fmt[1], 127, 127, True).cpu()
    d_lit0 = C.mfma_f8_probe(a, b, fmt[0], fmt[1], 0, 0, False).cpu()
    # rows/cols on lanes l&15, the four lane groups l>>4 partition k; the k order inside a
    # lane's 32 bytes is free as long as A and B use the same one (every hypothesis below is a
    # consistent k permutation, so they all give the same product -- the kernels use contig32)
    for hyp in ("contig32", "halves", "groups8"):
        assert torch.equal(d_unit, _reference(av, bv, hyp)), hyp
    # mismatched k orders between A and B must NOT give the product (the check has teeth)
    rc, k1 = _lane_maps("contig32")
    _, k2 = _lane_maps("halves")
    A = torch.zeros(16, 128)
    B = torch.zeros(128, 16)
    A[rc.reshape(-1), k1.reshape(-1)] = av.reshape(-1)
    B[k2.reshape(-1), rc.reshape(-1)] = bv.reshape(-1)
    lanes = torch.arange(64)
    mixed = torch.stack([(A @ B)[(lanes >> 4) * 4 + e, lanes & 15] for e in range(4)], 1)
    assert not torch.equal(d_unit, mixed)
    # composable_kernel's literal-0 scale operands mean "unscaled" (== E8M0 127 = 1.0)
    assert torch.equal(d_lit0, d_unit)
    # E8M0 128 = 2.0 on A, 126 = 0.5 on B
    d_s = C.mfma_f8_probe(a, b, fmt[0], fmt[1], 128, 126, True).cpu()
    assert torch.equal(d_s, d_unit)
    d_2 = C.mfma_f8_probe(a, b, fmt[0], fmt[1], 128, 127, True).cpu()
    assert torch.equal(d_2, 2 * d_unit)


# ----------------------------------------------------------------------------- kernels
from pytorch_distributed_tutorials_amd.ops import reference as ref  # noqa: E402


def _deq_e4m3(q):
    return q.view(torch.float8_e4m3fn).float()


def test_pack_weight_fp8(gpu, native_ext):
    C = native_ext
    g = torch.Generator().manual_seed(5)
    w = (torch.randn(96, 40, 3, 3, generator=g) * 0.05).to(gpu).contiguous(memory_format=torch.channels_last)
    act = torch.tensor([0.25], device=gpu)
    wq, osc = C.pack_weight_fp8(w, 48, act)
    assert wq.shape == (96, 3, 3, 48) and wq.dtype == torch.uint8
    ws = w.abs().amax(dim=(1, 2, 3)) / 448.0
    assert torch.allclose(osc, ws * 0.25, rtol=1e-6)
    deq = _deq_e4m3(wq)[..., :40] * ws[:, None, None, None]
    assert _deq_e4m3(wq)[..., 40:].abs().max().item() == 0
    w_krsc = w.permute(0, 2, 3, 1)
    rel = ((deq - w_krsc).norm() / w_krsc.norm()).item()
    assert rel < 0.04, rel
    # the per-channel max maps to +-448 exactly
    assert _deq_e4m3(wq).abs().amax(dim=(1, 2, 3)).eq(448).all()


def test_quant_e4m3_delayed_scaling(gpu, native_ext):
    C = native_ext
    g = torch.Generator().manual_seed(6)
    x = (torch.randn(2, 4, 4, 32, generator=g) * 3).to(torch.bfloat16).to(gpu)
    state = torch.zeros(C.fp8_state_floats(), device=gpu)
    D = C.fp8_deq_offset()
    slot_amax = lambda k: state[k * (D // 3):(k + 1) * (D // 3)].max().item()  # noqa: E731
    q0 = C.quant_e4m3(x, state, 0)                   # no history: scale 1
    amax = x.float().abs().max().item()
    torch.cuda.synchronize()
    assert state[D].item() == 1.0
    assert slot_amax(0) == amax
    ref0 = x.float().clamp(-448, 448).to(torch.float8_e4m3fn).float()
    assert torch.equal(_deq_e4m3(q0), ref0)
    q1 = C.quant_e4m3(x, state, 1)                   # scale from call 0's amax
    s = 2.0 ** torch.floor(torch.log2(torch.tensor(224.0 / amax))).item()
    torch.cuda.synchronize()
    assert state[D + 1].item() == 1.0 / s
    assert slot_amax(2) == 0.0                       # slot of the next call cleared
    ref1 = (x.float() * s).clamp(-448, 448).to(torch.float8_e4m3fn).float()
    assert torch.equal(_deq_e4m3(q1), ref1)
    # saturation instead of inf/NaN when the data outgrows the delayed scale
    big = torch.full((1, 1, 1, 16), 1e4, device=gpu).to(torch.bfloat16)
    qb = C.quant_e4m3(big, state, 2)
    assert _deq_e4m3(qb).eq(448).all()


FP8_CONV_SHAPES = [
    # N, H, W, C, K, R, S, stride, pad
    (2, 8, 8, 64, 64, 3, 3, 1, 1),        # C=64: generic (non-128) loader path, 256x64 tile
    (2, 9, 9, 128, 128, 3, 3, 2, 1),      # 128-byte channel blocks, 64x128 tile
    (3, 7, 7, 256, 512, 1, 1, 1, 0),
    (4, 56, 56, 64, 256, 1, 1, 1, 0),     # 128x128 tile
    (8, 28, 28, 128, 512, 1, 1, 1, 0),    # M = 6272 <= 8192: 64x128 tile (256x256: test_tiles_gpu.py)
    (2, 16, 16, 512, 1024, 1, 1, 2, 0),
    (2, 14, 14, 256, 256, 3, 3, 1, 1),
]


@pytest.mark.parametrize("shape", FP8_CONV_SHAPES)
def test_conv_fwd_fp8(gpu, native_ext, shape):
    C = native_ext
    n, h, w_, c, k, r, s, st, pd = shape
    g = torch.Generator().manual_seed(7)
    x = torch.relu(torch.randn(n, h, w_, c, generator=g)).to(torch.bfloat16).to(gpu)
    w = (torch.randn(k, c, r, s, generator=g) / (c * r * s) ** 0.5).to(gpu)
    w = w.contiguous(memory_format=torch.channels_last)
    state = torch.zeros(C.fp8_state_floats(), device=gpu)
    D = C.fp8_deq_offset()
    C.quant_e4m3(x, state, 0)                         # history -> a real (non-unit) scale
    xq = C.quant_e4m3(x, state, 1)
    deq = state[D + 1:D + 2].clone()
    wq, osc = C.pack_weight_fp8(w, c, deq)
    y, part = C.conv_fwd_fp8(xq, wq, osc, st, pd, True)
    # exact operand semantics: conv of the dequantized operands
    xd = (_deq_e4m3(xq) * deq).to(gpu)
    wd = (_deq_e4m3(wq).permute(0, 3, 1, 2) * (osc / deq)[:, None, None, None])
    yr = ref.conv2d_nhwc(xd, wd.contiguous(memory_format=torch.channels_last), st, pd)
    assert y.shape == yr.shape
    rel = ((y.float() - yr).norm() / yr.norm()).item()
    assert rel < 1e-2, rel
    # and close to the unquantized bf16 conv
    y16 = ref.conv2d_nhwc(x, w, st, pd)
    rel16 = ((y.float() - y16).norm() / y16.norm()).item()
    assert rel16 < 0.08, rel16
    # BN partial statistics from the dequantized accumulators
    stats = C.bn_finalize(part, yr.numel() // k, torch.zeros(k, device=gpu), torch.ones(k, device=gpu),
                          torch.ones(k, device=gpu), torch.zeros(k, device=gpu), 0.1, 1e-5)
    mean_r, _ = ref.bn_batch_stats(yr)
    assert torch.allclose(stats[0], mean_r, atol=5e-3, rtol=2e-2)
    # the same conv with the BN finalize fused (fp64 sums, last workgroup per channel tile)
    acc = torch.zeros(8, 2, k, dtype=torch.float64, device=gpu)
    rm, rv = torch.zeros(k, device=gpu), torch.ones(k, device=gpu)
    ones, zeros = torch.ones(k, device=gpu), torch.zeros(k, device=gpu)
    y2, st2 = C.conv_fwd_fp8(xq, wq, osc, st, pd, True, None,
                             (yr.numel() // k, rm, rv, ones, zeros, 0.1, 1e-5, acc))
    assert torch.equal(y2, y)
    assert torch.allclose(st2, stats, rtol=2e-4, atol=1e-5)
    assert torch.count_nonzero(acc) == 0


def test_bn_act_fwd_q8_matches_bf16_apply(gpu, native_ext):
    C = native_ext
    g = torch.Generator().manual_seed(8)
    y = torch.randn(4, 6, 6, 64, generator=g).to(torch.bfloat16).to(gpu)
    res = torch.randn(4, 6, 6, 64, generator=g).to(torch.bfloat16).to(gpu)
    sc = (torch.rand(64, generator=g) + 0.5).to(gpu)
    sh = torch.randn(64, generator=g).to(gpu)
    state = torch.zeros(C.fp8_state_floats(), device=gpu)
    z, q, zm = C.bn_act_fwd_q8(y, sc, sh, res, True, state, 0, True)
    z_ref = C.bn_act_fwd(y, sc, sh, res, True)
    assert torch.equal(z, z_ref)
    bits = (z.reshape(-1, 8) > 0).to(torch.int32) << torch.arange(8, device=gpu, dtype=torch.int32)
    assert torch.equal(zm.to(torch.int32), bits.sum(1))
    assert torch.equal(_deq_e4m3(q), z.float().clamp(-448, 448).to(torch.float8_e4m3fn).float())
    torch.cuda.synchronize()
    D = C.fp8_deq_offset()
    assert state[:D // 3].max().item() == z.float().abs().max().item()


def test_resnet50_fp8_forward_close_to_bf16(gpu, native_ext):
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    torch.manual_seed(0)
    m = build_model("resnet50", num_classes=10, impl="native").to(gpu).set_impl("native")
    x = torch.randn(8, 3, 64, 64, device=gpu)
    yl = torch.randint(0, 10, (8,), device=gpu)
    m.eval()
    with torch.no_grad():
        ref_logits = m(x).float()
        try:
            ops.set_fp8(True)
            for _ in range(3):  # delayed scaling settles after the first call
                out = m(x).float()
        finally:
            ops.set_fp8(False)
    rel = ((out - ref_logits).norm() / ref_logits.norm()).item()
    assert rel < 0.1, rel
    m.train()
    try:
        ops.set_fp8(True)
        loss = ops.cross_entropy(m(x), yl)
        loss.backward()
    finally:
        ops.set_fp8(False)
    assert torch.isfinite(loss).item()
    assert all(torch.isfinite(p.grad).all().item() for p in m.parameters() if p.grad is not None)


# ----------------------------------------------------------------------------- fp8 backward
def _deq_e5m2(q):
    return q.view(torch.float8_e5m2).float()


FP8_DGRAD_SHAPES = [
    # N, H, W, C, K, R, S, stride, pad   (K % 128 == 0: dy rows fill 128-byte fp8 steps)
    (2, 9, 9, 64, 128, 3, 3, 2, 1),
    (3, 7, 7, 256, 512, 1, 1, 1, 0),
    (2, 14, 14, 256, 256, 3, 3, 1, 1),
    (2, 15, 15, 128, 256, 3, 3, 2, 1),
    (4, 28, 28, 512, 128, 1, 1, 1, 0),
    (2, 16, 16, 512, 1024, 1, 1, 2, 0),
    # K % 128 != 0 at stride 1 (the 64-channel layer-1 convs): generic loader, K-steps across taps
    (2, 14, 14, 64, 64, 3, 3, 1, 1),
    (3, 9, 9, 256, 64, 1, 1, 1, 0),
    (2, 8, 8, 64, 80, 3, 3, 1, 1),
]


def _dgrad_operands(C, shape, gpu, seed=11):
    from pytorch_distributed_tutorials_amd.ops.fused import _packed_crsk8
    n, h, w_, c, k, r, s, st, pd = shape
    g = torch.Generator().manual_seed(seed)
    ho, wo = (h + 2 * pd - r) // st + 1, (w_ + 2 * pd - s) // st + 1
    dy = (torch.randn(n, ho, wo, k, generator=g) * 1e-3).to(torch.bfloat16).to(gpu)
    w = (torch.randn(k, c, r, s, generator=g) / (c * r * s) ** 0.5).to(gpu)
    w = w.contiguous(memory_format=torch.channels_last)
    sc = 2.0 ** 14  # e5m2 scale for ~1e-3 gradients
    dy8 = (dy.float() * sc).clamp(-57344, 57344).to(torch.float8_e5m2).view(torch.uint8)
    ascale = torch.tensor([1.0 / sc], device=gpu)
    wt8, wsc = _packed_crsk8(C, w)
    dyd = _deq_e5m2(dy8) / sc
    wd = (_deq_e4m3(wt8) * wsc[:, None, None, None]).permute(3, 0, 1, 2)  # [K,C,R,S]
    return dy, w, dy8, ascale, wt8, wsc, dyd.to(torch.bfloat16), wd.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", FP8_DGRAD_SHAPES)
def test_conv_dgrad_fp8(gpu, native_ext, shape):
    C = native_ext
    n, h, w_, c, k, r, s, st, pd = shape
    dy, w, dy8, ascale, wt8, wsc, dyd, wd = _dgrad_operands(C, shape, gpu)
    dx = C.conv_dgrad_fp8(dy8, wt8, wsc, ascale, [n, h, w_, c], st, pd)
    ref_q = ref.conv2d_nhwc_dgrad(dyd, wd, (n, h, w_, c), st, pd)
    rel = ((dx.float() - ref_q).norm() / ref_q.norm()).item()
    assert rel < 1e-2, rel
    ref16 = ref.conv2d_nhwc_dgrad(dy, w, (n, h, w_, c), st, pd)
    rel16 = ((dx.float() - ref16).norm() / ref16.norm()).item()
    assert rel16 < 0.12, rel16


@pytest.mark.parametrize("mask", [1, 2])
@pytest.mark.parametrize("shape", [(2, 14, 14, 256, 256, 3, 3, 1, 1), (2, 14, 14, 64, 64, 3, 3, 1, 1)])
def test_conv_dgrad_bn_fp8_matches_bf16_on_dequantized(gpu, native_ext, mask, shape):
    C = native_ext
    n, h, w_, c, k, r, s, st, pd = shape
    dy, w, dy8, ascale, wt8, wsc, dyd, wd = _dgrad_operands(C, shape, gpu, seed=12)
    g = torch.Generator().manual_seed(13)
    y = torch.randn(n, h, w_, c, generator=g).to(torch.bfloat16).to(gpu)
    stats = torch.stack([torch.randn(c, generator=g) * 0.1, torch.rand(c, generator=g) + 0.5,
                         torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1]).to(gpu)
    z = torch.relu(y.float() * stats[2] + stats[3]).to(torch.bfloat16)
    g8, sums8 = C.conv_dgrad_bn_fp8(dy8, wt8, wsc, ascale, [n, h, w_, c], st, pd, None, y,
                                    z if mask == 1 else None, stats, mask)
    g16, sums16 = C.conv_dgrad_bn(dyd, wd, [n, h, w_, c], st, pd, None, y, z if mask == 1 else None,
                                  stats, mask)
    assert ((g8.float() - g16.float()).norm() / g16.float().norm()).item() < 2e-2
    assert ((sums8 - sums16).norm() / sums16.norm()).item() < 2e-2


def test_bn_act_bwd_apply_q8(gpu, native_ext):
    C = native_ext
    g = torch.Generator().manual_seed(14)
    K = 128
    dz = (torch.randn(4, 6, 6, K, generator=g) * 1e-3).to(torch.bfloat16).to(gpu)
    y = torch.randn(4, 6, 6, K, generator=g).to(torch.bfloat16).to(gpu)
    stats = torch.stack([torch.randn(K, generator=g) * 0.1, torch.rand(K, generator=g) + 0.5,
                         torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1]).to(gpu)
    gamma = (torch.rand(K, generator=g) + 0.5).to(gpu)
    sums = C.bn_act_bwd_reduce(dz, dz, y, stats, 2)
    state = torch.zeros(C.fp8_state_floats(), device=gpu)
    D = C.fp8_deq_offset()
    dy, dres, dy8 = C.bn_act_bwd_apply_q8(dz, dz, y, stats, gamma, sums, 2, False, state, 0)
    dy_ref, _ = C.bn_act_bwd_apply(dz, dz, y, stats, gamma, sums, 2, True, False)
    assert torch.equal(dy, dy_ref)
    assert torch.equal(_deq_e5m2(dy8), dy.float().to(torch.float8_e5m2).float())  # first call: scale 1
    amax = dy.float().abs().max().item()
    dy2, _, dy82 = C.bn_act_bwd_apply_q8(dz, dz, y, stats, gamma, sums, 2, False, state, 1)
    s = 2.0 ** torch.floor(torch.log2(torch.tensor(28672.0 / amax))).item()
    torch.cuda.synchronize()
    assert state[D + 1].item() == 1.0 / s
    assert torch.equal(_deq_e5m2(dy82), (dy2.float() * s).to(torch.float8_e5m2).float())


def test_resnet50_fp8_dgrad_matches_bf16_dgrad_on_same_forward(gpu, native_ext):
    """fp8 dgrads (e5m2 dy, flat-mirror e4m3 weights) vs bf16 dgrads behind the SAME fp8
    forward.  (Comparing against a bf16 forward is meaningless here: a random-init ResNet-50 in
    BN training mode is chaotic -- perturbing the input at 0.4% already drops the gradient
    cosine to ~0.1, scripts/diag_fp8.py.)"""
    import pytorch_distributed_tutorials_amd.ops.fused as fused
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    m = build_model("resnet50", num_classes=10, impl="native").to(gpu).set_impl("native")
    ddp = DistributedDataParallel(m)
    x = torch.randn(16, 3, 64, 64, device=gpu)
    yl = torch.randint(0, 10, (16,), device=gpu)

    def grads(bwd8):
        ops.set_fp8(True)
        fused._FP8_BWD = bwd8
        try:
            # delayed scaling: later calls use real amax history; the scales settle after one call
            # per quantized layer in a dependency chain (4 calls on this net, scripts/diag_fp8_det.py)
            for _ in range(6):
                ddp.space.zero_grad()
                loss = ops.cross_entropy(ddp(x), yl)
                loss.backward()
        finally:
            ops.set_fp8(False)
            fused._FP8_BWD = True
        return loss.item(), ddp.space.grad_flat.clone()

    l_a, g_a = grads(False)
    l_b, g_b = grads(True)
    assert l_a == l_b  # identical forward
    assert torch.isfinite(g_b).all()
    cos = torch.nn.functional.cosine_similarity(g_b, g_a, dim=0).item()
    assert cos > 0.9, cos


def test_resnet18_fp8_training_reduces_loss(gpu, native_ext):
    """End-to-end fp8 training (fwd + dgrad on fp8) fits a fixed batch like bf16 does."""
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.optim import SGD
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel

    def run(fp8):
        torch.manual_seed(0)
        m = build_model("resnet18", num_classes=10, impl="native").to(gpu).set_impl("native")
        ddp = DistributedDataParallel(m)
        opt = SGD(ddp.parameters(), lr=0.05, momentum=0.9)
        g = torch.Generator().manual_seed(1)
        x = torch.randn(64, 3, 32, 32, generator=g).to(gpu)
        yl = torch.randint(0, 10, (64,), generator=g).to(gpu)
        ops.set_fp8(fp8)
        losses = []
        try:
            for _ in range(30):
                opt.zero_grad()
                loss = ops.cross_entropy(ddp(x), yl)
                loss.backward()
                opt.step()
                losses.append(loss.item())
        finally:
            ops.set_fp8(False)
        return losses

    l16, l8 = run(False), run(True)
    assert l8[-1] < 0.5 * l8[0], l8
    assert l8[-1] < 2.0 * l16[-1] + 0.1, (l8[-1], l16[-1])
