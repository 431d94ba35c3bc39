"""Kernel-level numerics on the MI355X: each libdfcsa GEMM/kernel against a plain PyTorch
fp32 CPU reference of the same op.  fp32 mode must match to ~1e-5 relative; bf16 mode to the
bf16 input rounding (operands are rounded to bf16 in the reference too)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dfcsa_ops = pytest.importorskip("dfcsa.ops")
from dfcsa import ops  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def nhwc(x, dtype):
    return x.permute(0, 2, 3, 1).contiguous().to("cuda", dtype)


def nchw(y):
    return y.permute(0, 3, 1, 2).float().cpu()


def q(x, dtype):  # round to the compute dtype (reference sees the same operands)
    return x.to(dtype).float()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,Cs,nsrc,C,H,W", [(2, 8, 1, 16, 9, 7), (1, 64, 2, 64, 14, 14), (2, 16, 2, 136, 5, 11)])
def test_conv3x3_multisource(dtype, tol, B, Cs, nsrc, C, H, W):
    torch.manual_seed(0)
    xs = [q(torch.randn(B, Cs, H, W), dtype) for _ in range(nsrc)]
    w = q(torch.randn(C, nsrc * Cs, 3, 3) * 0.1, dtype)
    b = torch.randn(C)
    ref = F.conv2d(torch.cat(xs, 1), w, b, padding=1)
    Kp = ops.rup(9 * nsrc * Cs, ops.KALIGN)
    wp = ops.pack_conv_w(dtype, w.cuda(), nsrc * Cs, Kp)
    y = torch.empty((B, H, W, C), dtype=dtype, device="cuda")
    M = B * H * W
    stats = torch.empty(ops.ntiles_gemm(M) * 2 * C, device="cuda")
    xh = [nhwc(x, dtype) for x in xs]
    segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xh]
    rows = ops.conv_gemm(dtype, segs, Cs, (B, H, W), (H, W), wp, Kp, C, [y], C, bias=b.cuda(), stats=stats)
    torch.cuda.synchronize()
    assert rel(nchw(y), ref) < tol
    st = stats[:rows * 2 * C].view(-1, 2, C).sum(0).cpu()
    acc = ref - b.view(1, -1, 1, 1)
    assert rel(st[0], acc.sum((0, 2, 3))) < max(tol, 1e-5) * 10
    assert rel(st[1], (acc * acc).sum((0, 2, 3))) < max(tol, 1e-5) * 10


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
def test_conv1x1_three_dests_accumulate(dtype, tol):
    torch.manual_seed(1)
    B, H, W, Cin, C = 2, 6, 10, 24, 16
    x = q(torch.randn(B, Cin, H, W), dtype)
    w = q(torch.randn(3 * C, Cin, 1, 1) * 0.2, dtype)
    ref = F.conv2d(x, w)
    base = [q(torch.randn(B, C, H, W), dtype) for _ in range(3)]
    Kp = ops.rup(Cin, ops.KALIGN)
    wp = ops.pack_conv_w(dtype, w.cuda(), Cin, Kp)
    dests = [nhwc(t, dtype) for t in base]
    ops.conv_gemm(dtype, [(nhwc(x, dtype), 0, 0)], Cin, (B, H, W), (H, W), wp, Kp, 3 * C, dests, C,
                  accumulate=True)
    torch.cuda.synchronize()
    for i in range(3):
        assert rel(nchw(dests[i]), ref[:, i * C:(i + 1) * C] + base[i]) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
def test_conv_transpose_fwd_bwd(dtype, tol):
    from dfcsa.functions import ConvTranspose2x2
    torch.manual_seed(2)
    B, h, w, Cin, Cout = 2, 5, 7, 32, 16
    mod = torch.nn.ConvTranspose2d(Cin, Cout, 2, 2)
    with torch.no_grad():
        mod.weight.copy_(q(mod.weight, dtype))
    x = q(torch.randn(B, Cin, h, w), dtype)
    xr = x.clone().requires_grad_(True)
    ref = mod(xr)
    g = q(torch.randn_like(ref), dtype)
    ref.backward(g)
    modg = torch.nn.ConvTranspose2d(Cin, Cout, 2, 2).cuda()
    with torch.no_grad():
        modg.weight.copy_(mod.weight)
        modg.bias.copy_(mod.bias)
    xh = nhwc(x, dtype).requires_grad_(True)
    y = ConvTranspose2x2.apply(xh, modg, dtype, *modg.parameters())
    y.backward(nhwc(g, dtype))
    torch.cuda.synchronize()
    assert rel(nchw(y), ref) < tol
    assert rel(nchw(xh.grad), xr.grad) < tol
    assert rel(modg.weight.grad, mod.weight.grad) < tol
    assert rel(modg.bias.grad, mod.bias.grad) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,Cs,C,H,fuse_all", [(2, 512, 256, 14, 0), (4, 256, 512, 16, 0), (16, 64, 64, 56, 1),
                                               (1, 64, 64, 8, 0)])
def test_wgrad_fused_split_reduction(dtype, B, Cs, C, H, fuse_all):
    """The split-K reduction inside the wgrad kernel (last-arriving workgroup per output tile sums
    the partials in split order): against torch fp32, bitwise reproducible run to run, and it
    ACCUMULATES into the gradient.  Shapes: deep layers (2-16 splits), a high-split shallow layer
    forced through the fused path (tuning knob 12), and a single-split case (direct store)."""
    import ctypes

    import dfcsa
    from dfcsa._lib import LIB
    torch.manual_seed(5)
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    x = q(torch.randn(B, Cs, H, H), dtype)
    g = q(torch.randn(B, C, H, H), dtype)
    w = torch.zeros(C, Cs, 3, 3, requires_grad=True)
    F.conv2d(x.requires_grad_(False), w, padding=1).backward(g)
    ref = w.grad + 0.25
    xh, gh = nhwc(x, dtype), nhwc(g, dtype)
    segs = [(xh, kh - 1, kw - 1) for kh in range(3) for kw in range(3)]
    sp, mc, fl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    LIB.dfcsa_wgrad_plan(B * H * H, C, 9 * Cs, ops.dt(dtype), ctypes.addressof(sp), ctypes.addressof(mc),
                         ctypes.addressof(fl))
    outs = []
    dfcsa.set_tuning(12, fuse_all)
    dfcsa.set_tuning(13, 16)      # exercise the in-kernel reduction up to 16 splits
    assert fuse_all or sp.value <= LIB.dfcsa_wgrad_fuse_max()
    try:
        for _ in range(2):
            gw = torch.full((C, Cs, 3, 3), 0.25, device="cuda")
            ops.conv_wgrad_into(dtype, [gh], C, segs, Cs, (B, H, H), (H, H), [gw], 9, Cs, Cs)
            outs.append(gw)
        torch.cuda.synchronize()
    finally:
        dfcsa.set_tuning(12, 0)
        dfcsa.set_tuning(13, 0)
    assert rel(outs[0], ref) < tol, (sp.value, rel(outs[0], ref))
    assert torch.equal(outs[0], outs[1]), "fused split-K reduction is not bitwise reproducible"


@pytest.mark.parametrize("B,Cs,nsrc,C,H,W,taps", [(16, 64, 2, 64, 56, 56, 1), (16, 64, 1, 128, 56, 56, 1),
                                                   (8, 64, 2, 64, 28, 28, 9), (4, 512, 1, 256, 14, 14, 9),
                                                   (4, 256, 3, 512, 14, 14, 1), (3, 64, 1, 72, 17, 13, 9)])
def test_wgrad_cooperative_reduction(B, Cs, nsrc, C, H, W, taps):
    """Split-K weight gradients reduced INSIDE the launch (knob 31, opt-in -- the library default is
    off -- and used only when the grid fits the chip): every split reduces one slice of its tile over all splits in split order.  bf16-exact
    operands against torch fp32 (1e-5: fp32 accumulation only), the separate slab reduction (knob 31 =
    0) to 1e-6, bitwise repeatable, accumulating into the gradient, no bounded wait ever exceeded.
    Shapes: the 224^2-like many-split 1x1 (hundreds of splits of one tile), multi-source 3x3, the deep
    3x3 with few splits, ragged channel counts (C = 72)."""
    import dfcsa
    from dfcsa._lib import LIB
    torch.manual_seed(11)
    dtype = torch.bfloat16
    xs = [q(torch.randn(B, Cs, H, W), dtype) for _ in range(nsrc)]
    g = q(torch.randn(B, C, H, W), dtype)
    w = torch.zeros(C, nsrc * Cs, 3 if taps == 9 else 1, 3 if taps == 9 else 1, requires_grad=True)
    F.conv2d(torch.cat(xs, 1), w, padding=1 if taps == 9 else 0).backward(g)
    ref = w.grad + 0.5
    xh = [nhwc(t, dtype) for t in xs]
    gh = nhwc(g, dtype)
    segs = ([(t, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for t in xh] if taps == 9
            else [(t, 0, 0) for t in xh])
    from dfcsa import streams
    LIB.dfcsa_wgrad_coop_errors(1)
    outs = {}
    saved = LIB.dfcsa_get_tuning(31)   # restore the library's setting (default 0), not a fixed value
    # knob 31 is refused while the side / branch streams are on (dfcsa.set_tuning): this standalone
    # launch runs alone on the device
    sstate = (streams.ENABLED[0], streams.BRANCH_ENABLED[0])
    streams.ENABLED[0] = streams.BRANCH_ENABLED[0] = False
    try:
        for coop in (1, 0, 1):
            dfcsa.set_tuning(31, coop)
            before = LIB.dfcsa_get_tuning(32)
            gw = torch.full(w.shape, 0.5, device="cuda")
            ops.conv_wgrad_into(dtype, [gh], C, segs, Cs, (B, H, W), (H, W), [gw], taps, nsrc * Cs, nsrc * Cs)
            torch.cuda.synchronize()
            used = LIB.dfcsa_get_tuning(32) - before
            outs.setdefault(coop, []).append((gw, used))
    finally:
        dfcsa.set_tuning(31, saved)
        streams.ENABLED[0], streams.BRANCH_ENABLED[0] = sstate
    assert LIB.dfcsa_wgrad_coop_errors(1) == 0
    (a, ua), (b, _) = outs[1]
    (c, uc), = outs[0]
    assert ua >= 1 and uc == 0, (ua, uc)
    assert rel(a, ref) < 1e-5, rel(a, ref)
    assert rel(a, c) < 1e-6, rel(a, c)
    assert torch.equal(a, b), "cooperative split-K reduction is not bitwise reproducible"


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,Cs,nsrc,C,H,W", [(2, 8, 1, 16, 9, 7), (3, 64, 2, 64, 14, 14), (2, 32, 1, 136, 20, 20)])
@pytest.mark.parametrize("variant", [(0, 0, 1), (1, 4, 1), (1, 8, 1), (0, 4, 1), (0, 8, 0)])  # knobs 7, 6, 8
def test_wgrad_3x3(dtype, tol, B, Cs, nsrc, C, H, W, variant):
    import dfcsa
    if dtype == torch.float32 and variant[0] == 0 and variant[1]:
        pytest.skip("fp32 always runs the register-staged kernel")
    torch.manual_seed(3)
    xs = [q(torch.randn(B, Cs, H, W), dtype) for _ in range(nsrc)]
    x = torch.cat(xs, 1).requires_grad_(True)
    w = torch.randn(C, nsrc * Cs, 3, 3, requires_grad=True)
    g = q(torch.randn(B, C, H, W), dtype)
    F.conv2d(x, w, padding=1).backward(g)
    xh = [nhwc(t, dtype) for t in xs]
    segs = [(t, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for t in xh]
    gw = torch.zeros(C, nsrc * Cs, 3, 3, device="cuda")
    dfcsa.set_tuning(7, variant[0])
    dfcsa.set_tuning(6, variant[1])
    dfcsa.set_tuning(8, variant[2])
    try:
        ops.conv_wgrad_into(dtype, [nhwc(g, dtype)], C, segs, Cs, (B, H, W), (H, W), [gw], 9, nsrc * Cs, nsrc * Cs)
        torch.cuda.synchronize()
    finally:
        dfcsa.set_tuning(7, 0)
        dfcsa.set_tuning(6, 0)
        dfcsa.set_tuning(8, 1)
    assert rel(gw, w.grad) < tol


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("B,Cs,C,H,W,fuse", [(2, 256, 256, 14, 14, 0), (2, 128, 512, 12, 10, 16), (3, 64, 264, 9, 11, 0),
                                             (1, 64, 128, 8, 8, 16)])
def test_wgrad_big_tiles(mode, B, Cs, C, H, W, fuse):
    """bf16 weight gradient on the big output tiles (tuning knob 17: 256x256, 256x128, 128x256; one
    512-thread workgroup per CU) against torch fp32 on bf16-exact operands: full and ragged tiles
    (C = 264), the slab reduction and the in-kernel split reduction (knob 13), bitwise repeatable."""
    import dfcsa
    torch.manual_seed(6)
    dtype = torch.bfloat16
    x = q(torch.randn(B, Cs, H, W), dtype)
    g = q(torch.randn(B, C, H, W), dtype)
    w = torch.zeros(C, Cs, 3, 3, requires_grad=True)
    F.conv2d(x, w, padding=1).backward(g)
    xh, gh = nhwc(x, dtype), nhwc(g, dtype)
    segs = [(xh, kh - 1, kw - 1) for kh in range(3) for kw in range(3)]
    outs = []
    dfcsa.set_tuning(17, mode)
    dfcsa.set_tuning(13, fuse)
    try:
        for _ in range(2):
            gw = torch.zeros(C, Cs, 3, 3, device="cuda")
            ops.conv_wgrad_into(dtype, [gh], C, segs, Cs, (B, H, W), (H, W), [gw], 9, Cs, Cs)
            outs.append(gw)
        torch.cuda.synchronize()
    finally:
        dfcsa.set_tuning(17, 0)
        dfcsa.set_tuning(13, 0)
    assert rel(outs[0], w.grad) < 1e-5, rel(outs[0], w.grad)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
def test_dgrad_3x3_plus_1x1(dtype, tol):
    """the fused input-gradient GEMM: 3x3 dgrad + two 1x1 dgrads into two destination sources"""
    torch.manual_seed(4)
    B, H, W, Cs, C = 2, 11, 9, 16, 24
    x = torch.randn(B, 2 * Cs, H, W, requires_grad=True)
    w1 = q(torch.randn(C, 2 * Cs, 3, 3) * 0.1, dtype)
    w2 = q(torch.randn(C, 2 * Cs, 1, 1) * 0.1, dtype)
    w3 = q(torch.randn(C, 2 * Cs, 1, 1) * 0.1, dtype)
    g1, g2, g3 = (q(torch.randn(B, C, H, W), dtype) for _ in range(3))
    (F.conv2d(x, w1, padding=1) * g1 + F.conv2d(x, w2) * g2 + F.conv2d(x, w3) * g3).sum().backward()
    Kx = ops.rup(11 * C, ops.KALIGN)
    Wdx = torch.zeros((2 * Cs, Kx), dtype=dtype, device="cuda")
    ops.pack_conv_w_t(dtype, w1.cuda(), Kx, Wdx, 0)
    ops.pack_conv_w_t(dtype, w2.cuda(), Kx, Wdx, 9 * C)
    ops.pack_conv_w_t(dtype, w3.cuda(), Kx, Wdx, 10 * C)
    d1, d2, d3 = (nhwc(t, dtype) for t in (g1, g2, g3))
    segs = [(d1, 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(d2, 0, 0), (d3, 0, 0)]
    dx = [torch.empty((B, H, W, Cs), dtype=dtype, device="cuda") for _ in range(2)]
    ops.conv_gemm(dtype, segs, C, (B, H, W), (H, W), Wdx, Kx, 2 * Cs, dx, Cs)
    torch.cuda.synchronize()
    assert rel(torch.cat([nchw(dx[0]), nchw(dx[1])], 1), x.grad) < tol


def test_maxpool_ties_and_odd_sizes():
    from dfcsa.functions import MaxPool2x2
    torch.manual_seed(5)
    x = torch.randint(-2, 3, (2, 16, 9, 7)).float()  # many ties
    xr = x.clone().requires_grad_(True)
    ref = F.max_pool2d(xr, 2, 2)
    g = torch.randn_like(ref)
    ref.backward(g)
    xh = nhwc(x, torch.float32).requires_grad_(True)
    y = MaxPool2x2.apply(xh, torch.float32)
    y.backward(nhwc(g, torch.float32))
    assert torch.equal(nchw(y), ref)
    assert torch.equal(nchw(xh.grad), xr.grad)


def test_maxpool_fork_accumulates_into_skip_gradient():
    """MaxPoolFork (encoder output -> pooled + skip): dx = maxpool_bwd(d pooled) + d skip, formed
    in place in the skip gradient; also with the skip unused (no skip gradient)."""
    from dfcsa.functions import MaxPoolFork
    torch.manual_seed(7)
    x = torch.randint(-2, 3, (2, 16, 10, 8)).float()  # ties
    xr = x.clone().requires_grad_(True)
    ref = F.max_pool2d(xr, 2, 2)
    g1, g2 = torch.randn_like(ref), torch.randn_like(x)
    (ref * g1).sum().backward()
    want = xr.grad + g2
    xh = nhwc(x, torch.float32).requires_grad_(True)
    pooled, skip = MaxPoolFork.apply(xh, torch.float32)
    assert torch.equal(nchw(pooled), ref) and torch.equal(nchw(skip), x)
    ((pooled * nhwc(g1, torch.float32)).sum() + (skip * nhwc(g2, torch.float32)).sum()).backward()
    assert torch.equal(nchw(xh.grad), want)
    xh2 = nhwc(x, torch.float32).requires_grad_(True)
    pooled2, _ = MaxPoolFork.apply(xh2, torch.float32)
    (pooled2 * nhwc(g1, torch.float32)).sum().backward()
    assert torch.equal(nchw(xh2.grad), xr.grad)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-6), (torch.bfloat16, 1e-2)])
def test_resize_bilinear(dtype, tol):
    from dfcsa.functions import ResizeBilinear
    torch.manual_seed(6)
    x = q(torch.randn(2, 8, 4, 5), dtype)
    xr = x.clone().requires_grad_(True)
    ref = F.interpolate(xr, size=(9, 11), mode="bilinear", align_corners=False)
    g = q(torch.randn_like(ref), dtype)
    ref.backward(g)
    xh = nhwc(x, dtype).requires_grad_(True)
    y = ResizeBilinear.apply(xh, (9, 11), dtype)
    y.backward(nhwc(g, dtype))
    assert rel(nchw(y), ref) < tol
    assert rel(nchw(xh.grad), xr.grad) < tol


def test_loss_and_metrics_kernel(golden):
    from dfcsa.loss import bce_dice, metrics_from_stats
    fx = golden("metrics_bce_dice.npz")
    for c in sorted({k.split(".")[0] for k in fx}):
        p = torch.tensor(fx[c + ".p"], device="cuda", requires_grad=True)
        t = torch.tensor(fx[c + ".t"], device="cuda")
        loss, stats = bce_dice(p, t, float(fx[c + ".wbce"]), float(fx[c + ".wdice"]))
        loss.backward()
        iou, dice = metrics_from_stats(stats)
        assert abs(loss.item() - float(fx[c + ".loss"])) < 1e-5 * max(1.0, abs(float(fx[c + ".loss"])))
        assert abs(iou - float(fx[c + ".iou"])) < 1e-9 and abs(dice - float(fx[c + ".dice"])) < 1e-9
        ref = torch.tensor(fx[c + ".dp"])
        assert rel(p.grad, ref) < 1e-5


def test_dice_loss_type_matches_reference(golden):
    """calculate_metrics(..., 'dice') (reference utils/metrics.py:251-252 -> dice_loss :6-24) against
    the reference's own outputs (metrics_dice.npz): loss, IoU, Dice, dL/dp -- p at exactly 0 and 1 (the
    zero-weight BCE term must not leak a non-finite value) and an empty mask included."""
    from dfcsa.loss import metrics_from_stats
    from utils.metrics import calculate_metrics, calculate_metrics_device
    fx = golden("metrics_dice.npz")
    for c in sorted({k.split(".")[0] for k in fx}):
        p = torch.tensor(fx[c + ".p"], device="cuda", requires_grad=True)
        t = torch.tensor(fx[c + ".t"], device="cuda")
        met = calculate_metrics_device(p, t, "dice", {})
        met["loss"].backward()
        iou, dice = metrics_from_stats(met["stats"])
        assert abs(met["loss"].item() - float(fx[c + ".loss"])) < 1e-5 * max(1.0, abs(float(fx[c + ".loss"]))), c
        assert abs(iou - float(fx[c + ".iou"])) < 1e-9 and abs(dice - float(fx[c + ".dice"])) < 1e-9, c
        assert torch.isfinite(p.grad).all(), c
        assert rel(p.grad, torch.tensor(fx[c + ".dp"])) < 1e-5, c
        m2 = calculate_metrics(p.detach(), t, "dice")
        assert abs(m2["dice"] - float(fx[c + ".dice"])) < 1e-9


def test_clip_sgd_matches_torch():
    from dfcsa.flat import FlatParams
    from dfcsa.optim import FusedSGD
    torch.manual_seed(7)
    ref = torch.nn.Sequential(torch.nn.Linear(37, 50), torch.nn.Linear(50, 3))
    mine = torch.nn.Sequential(torch.nn.Linear(37, 50), torch.nn.Linear(50, 3)).cuda()
    mine.load_state_dict(ref.state_dict())
    flat = FlatParams(mine)
    opt_r = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    opt_m = FusedSGD(mine.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    for step in range(3):
        gs = [torch.randn_like(p) * (3.0 if step == 1 else 0.01) for p in ref.parameters()]
        for p, g in zip(ref.parameters(), gs):
            p.grad = g.clone()
        nr = torch.nn.utils.clip_grad_norm_(ref.parameters(), max_norm=1.0)
        opt_r.step()
        opt_m.zero_grad()
        for p, g in zip(mine.parameters(), gs):
            p.grad.copy_(g)
        opt_m.step(max_norm=1.0)
        torch.cuda.synchronize()
        assert abs(opt_m.last_norm.item() - nr.item()) < 1e-5 * nr.item()
        for pr, pm in zip(ref.parameters(), mine.parameters()):
            assert rel(pm, pr) < 1e-6
    assert flat.valid()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("C,Cout", [(64, 1), (8, 1), (32, 3), (24, 1)])
def test_head_fwd_bwd(dtype, tol, C, Cout):
    from dfcsa.functions import Head1x1
    torch.manual_seed(8)
    B, H, W = 2, 13, 9
    mod = torch.nn.Conv2d(C, Cout, 1)
    x = q(torch.randn(B, C, H, W), dtype)
    xr = x.clone().requires_grad_(True)
    ref = mod(xr)
    g = torch.randn_like(ref)
    ref.backward(g)
    modg = torch.nn.Conv2d(C, Cout, 1).cuda()
    modg.load_state_dict(mod.state_dict())
    xh = nhwc(x, dtype).requires_grad_(True)
    y = Head1x1.apply(xh, modg, dtype, *modg.parameters())
    y.backward(g.cuda())
    assert rel(y, ref) < tol
    assert rel(nchw(xh.grad), xr.grad) < tol
    assert rel(modg.weight.grad, mod.weight.grad) < max(tol, 1e-5)
    assert rel(modg.bias.grad, mod.bias.grad) < 1e-5


@pytest.mark.parametrize("B,H,Cs,nsrc,C,k3", [(8, 128, 64, 1, 64, False),    # 256x64 LDS-DMA tile
                                              (4, 128, 64, 1, 256, False),   # 256x128 tile
                                              (4, 128, 16, 2, 128, True),    # 256x128, 3x3, 2 sources
                                              (2, 96, 8, 1, 64, True)])      # Cseg 8 < K stage
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19])
def test_conv_large_tiles_bf16(B, H, Cs, nsrc, C, k3, cfg):
    """Every bf16 tile configuration (tuning knob 1; 0 = automatic) on the same problems."""
    import dfcsa
    dtype = torch.bfloat16
    torch.manual_seed(9)
    xs = [q(torch.randn(B, Cs, H, H), dtype) for _ in range(nsrc)]
    ks = 3 if k3 else 1
    w = q(torch.randn(C, nsrc * Cs, ks, ks) * 0.1, dtype)
    b = torch.randn(C)
    ref = F.conv2d(torch.cat(xs, 1), w, b, padding=ks // 2)
    taps = [(kh - 1, kw - 1) for kh in range(3) for kw in range(3)] if k3 else [(0, 0)]
    Kp = ops.rup(len(taps) * nsrc * Cs, ops.KALIGN)
    wp = ops.pack_conv_w(dtype, w.cuda(), nsrc * Cs, Kp)
    M = B * H * H
    y = torch.empty((B, H, H, C), dtype=dtype, device="cuda")
    stats = torch.empty(ops.ntiles_gemm(M) * 2 * C, device="cuda")
    xh = [nhwc(x, dtype) for x in xs]
    segs = [(x, dh, dw) for dh, dw in taps for x in xh]
    dfcsa.set_tuning(1, cfg)
    try:
        rows = ops.conv_gemm(dtype, segs, Cs, (B, H, H), (H, H), wp, Kp, C, [y], C, bias=b.cuda(), stats=stats)
        torch.cuda.synchronize()
    finally:
        dfcsa.set_tuning(1, 0)
    assert rel(nchw(y), ref) < 1e-2
    st = stats[:rows * 2 * C].view(-1, 2, C).sum(0).cpu()
    acc = ref - b.view(1, -1, 1, 1)
    assert rel(st[0], acc.sum((0, 2, 3))) < 1e-4
    assert rel(st[1], (acc * acc).sum((0, 2, 3))) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,C", [(40, 64), (64, 64), (8, 16), (3, 16), (512, 64)])
def test_pack_plan_matches_single_packs(dtype, cin, C):
    """The two-phase pack plan (row permutes, then 64x64 tile transposes) reproduces the
    per-weight pack kernels bit for bit for a DFC block (with and without a residual conv), its
    LightSelfAttention projections and a ConvTranspose2d."""
    import torch.nn as nn
    from dfcsa import _lib
    from dfcsa.block import _build_block_packs
    from dfcsa.functions import _convT_packs
    from dfcsa.packs import PackSet
    from models.unet_dfc_sa_res import DynamicFusionConvAttnBlock
    torch.manual_seed(cin + C)
    blk = DynamicFusionConvAttnBlock(cin, C, pool_size=4).cuda()
    has_res = cin != C
    ps = PackSet(("t",), torch.device("cuda"))
    _build_block_packs(ps, blk, dtype, cin, C, has_res)
    up = nn.ConvTranspose2d(96, 32, 2, 2).cuda()
    ps2 = PackSet(("u",), torch.device("cuda"))
    _convT_packs(ps2, up, dtype, 128, 128)
    ps.run()
    ps2.run()
    torch.cuda.synchronize()
    conv1, conv2, conv3, conv4 = blk.conv_branch[0], blk.attn_branch[0], blk.gate[0], blk.fusion_conv[0]
    K = lambda n: ops.rup(n, 64)  # noqa: E731
    assert torch.equal(ps["W1p"], ops.pack_conv_w(dtype, conv1.weight, cin, K(9 * cin)))
    w2 = torch.zeros((2 * C if has_res else C, K(cin)), dtype=dtype, device="cuda")
    ops.pack_conv_w(dtype, conv2.weight, cin, K(cin), out=w2, row0=0)
    if has_res:
        ops.pack_conv_w(dtype, blk.residual_conv.weight, cin, K(cin), out=w2, row0=C)
        assert torch.equal(ps["b2"][:C], conv2.bias) and not ps["b2"][C:].any()
    assert torch.equal(ps["W2p"], w2)
    assert torch.equal(ps["W3p"], ops.pack_conv_w(dtype, conv3.weight, 2 * C, K(2 * C)))
    assert torch.equal(ps["W4p"], ops.pack_conv_w(dtype, conv4.weight, 3 * C, K(3 * C)))
    assert torch.equal(ps["W4t"], ops.pack_t3(dtype, 3 * C, K(C), [conv4.weight]))
    assert torch.equal(ps["W3t"], ops.pack_t3(dtype, 2 * C, K(C), [conv3.weight]))
    want = ops.pack_t3(dtype, cin, K(11 * C), [conv1.weight, conv2.weight,
                                                blk.residual_conv.weight if has_res else None],
                       identity_last=not has_res)
    if "Wdx" in ps.t:
        assert torch.equal(ps["Wdx"], want)
    else:   # the split block-input gradient operands: [W1 taps | Wres or I] and W2
        wa, wb = ps["WdxA"], ps["WdxB"]
        assert torch.equal(wa[:, :9 * C], want[:, :9 * C]) and torch.equal(wa[:, 9 * C:10 * C], want[:, 10 * C:11 * C])
        assert not wa[:, 10 * C:].any()
        assert torch.equal(wb[:, :C], want[:, 9 * C:10 * C]) and not wb[:, C:].any()
    lsa = blk.attn_branch[3]
    qw, kw, vw = lsa.query_conv.weight, lsa.key_conv.weight, lsa.value_conv.weight
    Cq = qw.shape[0]
    J = 2 * Cq + C
    assert torch.equal(ps["bqkv"], torch.cat([lsa.query_conv.bias, lsa.key_conv.bias, lsa.value_conv.bias]))
    if "Wp" in ps.t:
        wp = torch.zeros((J, K(C)), device="cuda")
        for w, off in ((qw, 0), (kw, Cq), (vw, 2 * Cq)):
            ops.pack_conv_w(torch.float32, w, C, K(C), out=wp, row0=off)
        assert torch.equal(ps["Wp"], wp)
        assert torch.equal(ps["WT"], ops.pack_t3(torch.float32, C, K(J), [qw, kw, vw]))
    else:
        assert torch.equal(ps["WqkvT"], ops.pack_t3(torch.float32, C, J, [qw, kw, vw]))
    fv = torch.empty((4 * 32, 96), dtype=dtype, device="cuda")
    bv = torch.empty((96, 128), dtype=dtype, device="cuda")
    b4 = torch.empty(128, device="cuda")
    _lib.call("dfcsa_pack_convT_w", ops.dt(dtype), ops.P(up.weight), ops.P(up.bias), 96, 32, ops.P(fv), ops.P(bv),
              ops.P(b4), ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(ps2["Wf"][:, :96], fv) and not ps2["Wf"][:, 96:].float().any()
    assert torch.equal(ps2["Wb"], bv)
    assert torch.equal(ps2["b4"], b4)


@pytest.mark.parametrize("Cs,nsrc,C,nd,acc,bias,stats", [
    (64, 1, 64, 2, True, False, False),     # W3t dgrad: 1 source, 2 accumulated dests
    (64, 1, 64, 3, False, False, False),    # W4t dgrad: 3 dests
    (64, 3, 64, 1, False, True, True),      # fusion conv fwd: 3 sources (K = 192), stats
    (8, 1, 64, 2, False, True, True),       # first block 1x1: K = 8 padded to 64
    (128, 1, 256, 1, False, True, True),    # K = 128, N = 256
    (128, 1, 96, 2, False, True, True),     # N = 192 -> 48 columns per wave
    (256, 1, 256, 2, False, True, True),    # K = 256, N = 512
])
@pytest.mark.parametrize("force", [1, 0])
def test_conv1x1_streaming_kernel(Cs, nsrc, C, nd, acc, bias, stats, force):
    """bf16 1x1 GEMMs with M >= 65536: the persistent streaming kernel (forced for every template
    variant) and the automatic choice, ragged last tile."""
    import dfcsa
    torch.manual_seed(Cs + C + nd)
    B, H, W = 3, 150, 147                      # M = 66150: 1034 tiles, last one partial
    dtype = torch.bfloat16
    xs = [q(torch.randn(B, Cs, H, W), dtype) for _ in range(nsrc)]
    N = nd * C
    w = q(torch.randn(N, nsrc * Cs, 1, 1) * 0.1, dtype)
    b = torch.randn(N) if bias else None
    ref = F.conv2d(torch.cat(xs, 1), w, b)
    base = [q(torch.randn(B, C, H, W), dtype) for _ in range(nd)]
    Kp = ops.rup(nsrc * Cs, ops.KALIGN)
    wp = ops.pack_conv_w(dtype, w.cuda(), nsrc * Cs, Kp)
    dests = [nhwc(t, dtype) if acc else torch.empty((B, H, W, C), dtype=dtype, device="cuda") for t in base]
    M = B * H * W
    st = torch.full((ops.ntiles_gemm(M) * 2 * N,), float("nan"), device="cuda") if stats else None
    dfcsa.set_tuning(5, force)
    try:
        rows = ops.conv_gemm(dtype, [(nhwc(x, dtype), 0, 0) for x in xs], Cs, (B, H, W), (H, W), wp, Kp, N, dests,
                             C, bias=b.cuda() if bias else None, accumulate=acc, stats=st)
        torch.cuda.synchronize()
    finally:
        dfcsa.set_tuning(5, 0)
    for i in range(nd):
        want = ref[:, i * C:(i + 1) * C] + (base[i] if acc else 0)
        assert rel(nchw(dests[i]), want) < 1e-2
    if stats:
        assert not torch.isnan(st[:rows * 2 * N]).any()     # every reported row written
        s = st[:rows * 2 * N].view(-1, 2, N).sum(0).cpu()
        a = ref - (b.view(1, -1, 1, 1) if bias else 0)
        assert rel(s[0], a.sum((0, 2, 3))) < 1e-3
        assert rel(s[1], (a * a).sum((0, 2, 3))) < 1e-3


@pytest.mark.parametrize("stream_shift", [1, 0])
@pytest.mark.parametrize("B,H,W", [(3, 150, 147), (2, 224, 224)])
def test_first_layer_3x3_streaming(B, H, W, stream_shift):
    """The first-layer 3x3 conv (Cin = 3 padded to 8, K = 72): the streaming GEMM with shifted
    segments (knob 30 on) and the tile kernel (off) against torch fp32 on the bf16-rounded
    operands, bias and BN partial sums, ragged last tile and image borders."""
    import dfcsa
    torch.manual_seed(H + W)
    dtype = torch.bfloat16
    x = q(torch.randn(B, 3, H, W), dtype)
    w = q(torch.randn(64, 3, 3, 3) * 0.2, dtype)
    b = torch.randn(64)
    ref = F.conv2d(x, w, b, padding=1)
    xp = torch.zeros(B, H, W, 8, dtype=dtype, device="cuda")
    xp[..., :3] = nhwc(x, dtype)
    w8 = torch.zeros(64, 8, 3, 3)
    w8[:, :3] = w
    Kp = ops.rup(9 * 8, ops.KALIGN)
    wp = ops.pack_conv_w(dtype, w8.cuda(), 8, Kp)
    M = B * H * W
    out = torch.empty((B, H, W, 64), dtype=dtype, device="cuda")
    st = torch.full((ops.ntiles_gemm(M) * 2 * 64,), float("nan"), device="cuda")
    segs = [(xp, kh - 1, kw - 1) for kh in range(3) for kw in range(3)]
    dfcsa.set_tuning(30, stream_shift)
    try:
        rows = ops.conv_gemm(dtype, segs, 8, (B, H, W), (H, W), wp, Kp, 64, [out], 64, bias=b.cuda(), stats=st)
        torch.cuda.synchronize()
    finally:
        dfcsa.set_tuning(30, 1)
    assert rel(nchw(out), ref) < 1e-2
    s = st[:rows * 2 * 64].view(-1, 2, 64).sum(0).cpu()
    a = ref - b.view(1, -1, 1, 1)
    assert rel(s[0], a.sum((0, 2, 3))) < 1e-3
    assert rel(s[1], (a * a).sum((0, 2, 3))) < 1e-3


@pytest.mark.parametrize("M,C", [(65536 + 37, 64), (4 * 28 * 28, 128), (2 * 56 * 56 + 5, 256), (300, 64),
                                 (16 * 224 * 224, 64), (16 * 112 * 112, 128), (16 * 56 * 56, 256)])
def test_dgrad_gate_fused_equals_gemm_plus_gate(M, C):
    """dfcsa_dgrad_gate (fusion-conv input gradient with the gate backward in its epilogue) against
    the unfused pair it replaces (dfcsa_conv_gemm -> [dfused, dlocal, dattn], then
    dfcsa_bwd_gate): dlocal, dattn and dz3 bit-identical (same MFMA order, same bf16 roundings),
    the BN3-backward sums equal to fp32 summation-order noise; ragged M (M % 64 != 0)."""
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P, S, stream
    torch.manual_seed(11)
    bf = torch.bfloat16
    dev = "cuda"
    Kp = ops.rup(C, ops.KALIGN)
    dy4 = torch.randn(M, C, device=dev).to(bf)
    w4t = (torch.randn(3 * C, Kp, device=dev) * 0.1).to(bf)
    y3, loc, att = (torch.randn(M, C, device=dev).to(bf) for _ in range(3))
    sc, sh, mu = (torch.randn(C, device=dev) for _ in range(3))
    istd = torch.rand(C, device=dev) + 0.5
    # unfused reference path
    dfu, dl0, da0, dz0 = (torch.empty(M, C, device=dev, dtype=bf) for _ in range(4))
    ops.conv_gemm(bf, [(dy4.view(1, M, 1, C), 0, 0)], C, (1, M, 1), (M, 1), w4t, Kp, 3 * C,
                  [dfu.view(1, M, 1, C), dl0.view(1, M, 1, C), da0.view(1, M, 1, C)], C)
    nte = ops.ntiles_ew(M, C)
    part0 = torch.empty(nte * 2 * C, device=dev)
    call("dfcsa_bwd_gate", ops.dt(bf), M, C, P(dfu), P(y3), P(sc), P(sh), P(mu), P(istd), P(loc), P(att), P(dl0),
         P(da0), P(dz0), *S(part0), stream())
    # fused
    npart = LIB.dfcsa_dgrad_gate_parts(M, C)
    assert 1 <= npart <= (M + 63) // 64
    dl1, da1, dz1 = (torch.empty(M, C, device=dev, dtype=bf) for _ in range(3))
    part1 = torch.empty(npart * 2 * C, device=dev)
    call("dfcsa_dgrad_gate", M, C, P(dy4), P(w4t), Kp, P(y3), P(sc), P(sh), P(mu), P(istd), P(loc), P(att), P(dl1),
         P(da1), P(dz1), *S(part1), stream())
    torch.cuda.synchronize()
    assert torch.equal(dl1, dl0) and torch.equal(da1, da0) and torch.equal(dz1, dz0)
    s0 = part0.view(nte, 2, C).double().sum(0)
    s1 = part1.view(npart, 2, C).double().sum(0)
    assert rel(s1, s0) < 1e-5


@pytest.mark.parametrize("M,C", [(65536 + 37, 64), (16 * 112 * 112, 128), (2 * 56 * 56 + 5, 256), (300, 64),
                                 (16 * 224 * 224, 64)])
def test_dgrad_acc_relu_bn_fused_equals_gemm_plus_sums(M, C):
    """dfcsa_dgrad_acc_relu_bn (gate-conv input gradient added into [dlocal, dattn] with the BN1
    relu-backward sums in its epilogue) against the unfused pair it replaces (accumulate-mode
    dfcsa_conv_gemm, then dfcsa_bwd_relu_bn's sums): dlocal and dattn bit-identical, the sums equal
    to fp32 summation-order noise; ragged M."""
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P, S, stream
    torch.manual_seed(12)
    bf = torch.bfloat16
    dev = "cuda"
    Kp = ops.rup(C, ops.KALIGN)
    dy3 = torch.randn(M, C, device=dev).to(bf)
    w3t = (torch.randn(2 * C, Kp, device=dev) * 0.1).to(bf)
    y1, dl_in, da_in = (torch.randn(M, C, device=dev).to(bf) for _ in range(3))
    sc, sh, mu = (torch.randn(C, device=dev) for _ in range(3))
    istd = torch.rand(C, device=dev) + 0.5
    dl0, da0 = dl_in.clone(), da_in.clone()
    ops.conv_gemm(bf, [(dy3.view(1, M, 1, C), 0, 0)], C, (1, M, 1), (M, 1), w3t, Kp, 2 * C,
                  [dl0.view(1, M, 1, C), da0.view(1, M, 1, C)], C, accumulate=True)
    nte = ops.ntiles_ew(M, C)
    part0 = torch.empty(nte * 2 * C, device=dev)
    call("dfcsa_bwd_relu_bn", ops.dt(bf), M, C, P(dl0), P(y1), P(sc), P(sh), P(mu), P(istd), None, *S(part0), stream())
    npart = LIB.dfcsa_dgrad_acc_relu_bn_parts(M, C)
    assert 1 <= npart <= (M + 63) // 64
    dl1, da1 = dl_in.clone(), da_in.clone()
    part1 = torch.empty(npart * 2 * C, device=dev)
    call("dfcsa_dgrad_acc_relu_bn", M, C, P(dy3), P(w3t), Kp, P(y1), P(sc), P(sh), P(mu), P(istd), P(dl1), P(da1),
         *S(part1), stream())
    torch.cuda.synchronize()
    assert torch.equal(dl1, dl0) and torch.equal(da1, da0)
    s0 = part0.view(nte, 2, C).double().sum(0)
    s1 = part1.view(npart, 2, C).double().sum(0)
    assert rel(s1, s0) < 1e-5


@pytest.mark.parametrize("wide", [0, 1])
@pytest.mark.parametrize("B,H,W,nsrc,NI", [(2, 20, 18, 3, 64), (1, 9, 7, 2, 40), (4, 16, 16, 3, 16)])
def test_wgrad_1x1_multisource_wide_tile(wide, B, H, W, nsrc, NI):
    """1x1 weight gradient over 2-3 concatenated 64-channel sources (the fusion / gate convs) with
    the 64x256 tile of tuning knob 18 (one column tile: the output gradient read once) and without,
    against torch fp32 on bf16-exact operands."""
    import dfcsa
    torch.manual_seed(8)
    bf = torch.bfloat16
    xs = [q(torch.randn(B, 64, H, W), bf) for _ in range(nsrc)]
    g = q(torch.randn(B, NI, H, W), bf)
    w = torch.zeros(NI, 64 * nsrc, 1, 1, requires_grad=True)
    F.conv2d(torch.cat(xs, 1), w).backward(g)
    segs = [(nhwc(x, bf), 0, 0) for x in xs]
    gw = torch.zeros(NI, 64 * nsrc, device="cuda")
    dfcsa.set_tuning(18, wide)
    try:
        ops.conv_wgrad_into(bf, [nhwc(g, bf)], NI, segs, 64, (B, H, W), (H, W), [gw], 1, 64 * nsrc, 64 * nsrc)
        torch.cuda.synchronize()
    finally:
        dfcsa.set_tuning(18, 0)
    assert rel(gw.view(NI, -1, 1, 1), w.grad) < 1e-5


@pytest.mark.parametrize("M,C", [(16 * 224 * 224, 64), (65536 + 37, 64), (300, 64), (16 * 112 * 112, 128),
                                 (4133, 128)])
def test_gate_fusion_fwd_equals_gate_fuse_plus_gemm(M, C):
    """dfcsa_gate_fusion_fwd (fusion conv forward with the gate fusion in its A-operand prologue,
    C = 64) against the pair it replaces (dfcsa_gate_fuse, then the [fused, local, attn] GEMM with
    BN statistics): fused, y4 and the statistics totals; ragged M; C = 64 and 128."""
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P, S, stream
    torch.manual_seed(13)
    bf = torch.bfloat16
    dev = "cuda"
    Kp = 3 * C
    y3, loc, att = (torch.randn(M, C, device=dev).to(bf) for _ in range(3))
    sc, sh = torch.randn(C, device=dev), torch.randn(C, device=dev)
    w4 = (torch.randn(C, Kp, device=dev) * 0.1).to(bf)
    b4 = torch.randn(C, device=dev)
    nt = ops.ntiles_gemm(M)
    f0, y0 = (torch.empty(M, C, device=dev, dtype=bf) for _ in range(2))
    st0 = torch.empty(nt * 2 * C, device=dev)
    call("dfcsa_gate_fuse", ops.dt(bf), M, C, P(y3), P(sc), P(sh), P(loc), P(att), P(f0), stream())
    v = lambda t: t.view(1, M, 1, C)
    rows = ops.conv_gemm(bf, [(v(f0), 0, 0), (v(loc), 0, 0), (v(att), 0, 0)], C, (1, M, 1), (M, 1), w4, Kp, C,
                         [v(y0)], C, bias=b4, stats=st0)
    f1, y1 = (torch.empty(M, C, device=dev, dtype=bf) for _ in range(2))
    st1 = torch.empty(nt * 2 * C, device=dev)
    call("dfcsa_gate_fusion_fwd", M, C, P(y3), P(sc), P(sh), P(loc), P(att), P(w4), Kp, P(b4), P(f1), P(y1), *S(st1),
         stream())
    torch.cuda.synchronize()
    assert rel(f1, f0) < 1e-6 and (f1.float() - f0.float()).abs().max().item() <= 2 ** -7 * f0.float().abs().max().item()
    assert rel(y1, y0) < 2e-3
    npart = LIB.dfcsa_fwd_pro_parts(M, C, 0)     # one statistics row per workgroup
    assert 1 <= npart <= nt
    tot = lambda st, n: st[:n * 2 * C].view(n, 2, C).double().sum(0)  # noqa: E731
    assert rel(tot(st1, npart), tot(st0, rows)) < 1e-4


@pytest.mark.parametrize("B,H,W,P", [(16, 224, 224, 4), (2, 36, 36, 4), (3, 14, 9, 8), (1, 5, 7, 4)])
def test_local_attn_gate_fwd_equals_merge_plus_gemm(B, H, W, P):
    """dfcsa_local_attn_gate_fwd (gate conv forward with the local/attention merge in its A-operand
    prologue, C = 64) against the pair it replaces (dfcsa_block_local_attn, then the [local, attn]
    GEMM with BN statistics): local, attn, y3 and the statistics totals; ragged M, P > H."""
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P as Ptr, S, stream
    torch.manual_seed(14)
    bf = torch.bfloat16
    dev = "cuda"
    C, Kp = 64, 128
    M = B * H * W
    y1, y2 = (torch.randn(M, C, device=dev).to(bf) for _ in range(2))
    sc1, sh1, sc2, sh2 = (torch.randn(C, device=dev) for _ in range(4))
    o = torch.randn(B, P, P, C, device=dev)
    gamma = torch.tensor([0.37], device=dev)
    w3 = (torch.randn(C, Kp, device=dev) * 0.1).to(bf)
    b3 = torch.randn(C, device=dev)
    nt = ops.ntiles_gemm(M)
    l0, a0, y30 = (torch.empty(M, C, device=dev, dtype=bf) for _ in range(3))
    st0 = torch.empty(nt * 2 * C, device=dev)
    call("dfcsa_block_local_attn", ops.dt(bf), B, H, W, C, Ptr(y1), Ptr(sc1), Ptr(sh1), Ptr(y2), Ptr(sc2), Ptr(sh2),
         Ptr(o), P, Ptr(gamma), 1, Ptr(l0), Ptr(a0), stream())
    v = lambda t: t.view(B, H, W, C)
    rows = ops.conv_gemm(bf, [(v(l0), 0, 0), (v(a0), 0, 0)], C, (B, H, W), (H, W), w3, Kp, C, [v(y30)], C, bias=b3,
                         stats=st0)
    l1, a1, y31 = (torch.empty(M, C, device=dev, dtype=bf) for _ in range(3))
    st1 = torch.empty(nt * 2 * C, device=dev)
    call("dfcsa_local_attn_gate_fwd", B, H, W, C, Ptr(y1), Ptr(sc1), Ptr(sh1), Ptr(y2), Ptr(sc2), Ptr(sh2), Ptr(o), P,
         Ptr(gamma), Ptr(w3), Kp, Ptr(b3), Ptr(l1), Ptr(a1), Ptr(y31), *S(st1), stream())
    torch.cuda.synchronize()
    assert torch.equal(l1, l0)
    assert rel(a1, a0) < 1e-6
    assert rel(y31, y30) < 2e-3
    npart = LIB.dfcsa_fwd_pro_parts(M, C, 1)     # one statistics row per workgroup
    tot = lambda st, n: st[:n * 2 * C].view(n, 2, C).double().sum(0)  # noqa: E731
    assert rel(tot(st1, npart), tot(st0, rows)) < 1e-4


@pytest.mark.parametrize("M", [16 * 224 * 224, 65536 + 37, 300])
def test_dgrad_apply_prologue_equals_apply_plus_gemm(M):
    """C = 64: dfcsa_dgrad_gate_apply / dfcsa_dgrad_acc_relu_bn_apply (the BatchNorm-backward apply of
    the A operand formed in the GEMM's prologue) against dfcsa_bn_bwd_apply_relu / _apply followed by
    dfcsa_dgrad_gate / dfcsa_dgrad_acc_relu_bn: dy, the GEMM outputs and the partial sums."""
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P, S, stream
    torch.manual_seed(15)
    bf = torch.bfloat16
    dev = "cuda"
    C = Kp = 64
    src, y, y3, loc, att, y1 = (torch.randn(M, C, device=dev).to(bf) for _ in range(6))
    gamma, k, mu, sc, sh, mu3, sc3, sh3 = (torch.randn(C if i != 1 else 3 * C, device=dev) for i in range(8))
    istd, istd3 = torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) + 0.5
    w4t = (torch.randn(3 * C, Kp, device=dev) * 0.1).to(bf)
    w3t = (torch.randn(2 * C, Kp, device=dev) * 0.1).to(bf)
    T = ops.dt(bf)
    # gate: reference path
    dy0 = torch.empty(M, C, device=dev, dtype=bf)
    call("dfcsa_bn_bwd_apply_relu", T, M, C, P(src), P(y), P(sc), P(sh), P(mu), P(istd), P(gamma), P(k), P(dy0), None, 0,
         stream())
    n0 = LIB.dfcsa_dgrad_gate_parts(M, C)
    dl0, da0, dz0 = (torch.empty(M, C, device=dev, dtype=bf) for _ in range(3))
    p0 = torch.empty(n0 * 2 * C, device=dev)
    call("dfcsa_dgrad_gate", M, C, P(dy0), P(w4t), Kp, P(y3), P(sc3), P(sh3), P(mu3), P(istd3), P(loc), P(att),
         P(dl0), P(da0), P(dz0), *S(p0), stream())
    n1 = LIB.dfcsa_dgrad_apply_parts(M, 0)
    dy1, dl1, da1, dz1 = (torch.empty(M, C, device=dev, dtype=bf) for _ in range(4))
    p1 = torch.empty(n1 * 2 * C, device=dev)
    call("dfcsa_dgrad_gate_apply", M, P(src), P(y), P(gamma), P(k), P(mu), P(istd), P(sc), P(sh), P(dy1), P(w4t),
         P(y3), P(sc3), P(sh3), P(mu3), P(istd3), P(loc), P(att), P(dl1), P(da1), P(dz1), *S(p1), stream())
    # acc: reference path (plain apply of dz3 = src)
    dyb0 = torch.empty(M, C, device=dev, dtype=bf)
    call("dfcsa_bn_bwd_apply", T, M, C, P(src), P(y), P(mu), P(istd), P(gamma), P(k), P(dyb0), None, 0, stream())
    dlb0, dab0 = loc.clone(), att.clone()
    m0 = LIB.dfcsa_dgrad_acc_relu_bn_parts(M, C)
    q0 = torch.empty(m0 * 2 * C, device=dev)
    call("dfcsa_dgrad_acc_relu_bn", M, C, P(dyb0), P(w3t), Kp, P(y1), P(sc3), P(sh3), P(mu3), P(istd3), P(dlb0),
         P(dab0), *S(q0), stream())
    m1 = LIB.dfcsa_dgrad_apply_parts(M, 1)
    dyb1 = torch.empty(M, C, device=dev, dtype=bf)
    dlb1, dab1 = loc.clone(), att.clone()
    q1 = torch.empty(m1 * 2 * C, device=dev)
    call("dfcsa_dgrad_acc_relu_bn_apply", M, P(src), P(y), P(gamma), P(k), P(mu), P(istd), P(dyb1), P(w3t), P(y1),
         P(sc3), P(sh3), P(mu3), P(istd3), P(dlb1), P(dab1), *S(q1), stream())
    torch.cuda.synchronize()
    for a, b in ((dy1, dy0), (dl1, dl0), (da1, da0), (dz1, dz0), (dyb1, dyb0), (dlb1, dlb0), (dab1, dab0)):
        assert rel(a, b) < 1e-5
    assert rel(p1.view(n1, 2, C).double().sum(0), p0.view(n0, 2, C).double().sum(0)) < 1e-5
    assert rel(q1.view(m1, 2, C).double().sum(0), q0.view(m0, 2, C).double().sum(0)) < 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,H,W,C,skip", [(2, 16, 12, 64, True), (1, 8, 10, 128, False), (3, 6, 4, 16, True)])
def test_block_out_pool_fused_equals_separate(dtype, B, H, W, C, skip):
    """dfcsa_block_out_pool / dfcsa_bwd_block_out_pool (encoder block output + 2x2 max-pool, forward
    and backward in one pass each) against the separate launches (dfcsa_block_out + dfcsa_maxpool2_fwd;
    dfcsa_maxpool2_bwd into the skip gradient + dfcsa_bwd_block_out): out, pooled, dout, dres exact
    (ties included: y4 has repeated values), the three per-channel sums to summation-order noise."""
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P, S, stream
    torch.manual_seed(16)
    dev = "cuda"
    T = ops.dt(dtype)
    M = B * H * W
    y4 = (torch.randint(-3, 4, (M, C), device=dev).float() * 0.5).to(dtype)   # ties in the windows
    res = torch.randn(M, C, device=dev).to(dtype)
    sc, sh, mu = (torch.randn(C, device=dev) for _ in range(3))
    istd = torch.rand(C, device=dev) + 0.5
    rs = torch.tensor([0.3], device=dev)
    Mp = B * (H // 2) * (W // 2)
    out0, out1 = (torch.empty(M, C, device=dev, dtype=dtype) for _ in range(2))
    p0, p1 = (torch.empty(Mp, C, device=dev, dtype=dtype) for _ in range(2))
    call("dfcsa_block_out", T, M, C, P(y4), P(sc), P(sh), P(res), P(rs), P(out0), stream())
    call("dfcsa_maxpool2_fwd", T, B, H, W, C, P(out0), P(p0), stream())
    call("dfcsa_block_out_pool", T, B, H, W, C, P(y4), P(sc), P(sh), P(res), P(rs), P(out1), P(p1), stream())
    gp = torch.randn(Mp, C, device=dev).to(dtype)
    gs = torch.randn(M, C, device=dev).to(dtype) if skip else None
    d0 = gs.clone() if skip else torch.zeros(M, C, device=dev, dtype=dtype)
    call("dfcsa_maxpool2_bwd", T, B, H, W, C, P(out0), P(gp), P(d0), stream())
    nte = ops.ntiles_ew(M, C)
    dr0 = torch.empty(M, C, device=dev, dtype=dtype)
    q0 = torch.empty(nte * 3 * C, device=dev)
    call("dfcsa_bwd_block_out", T, M, C, P(d0), P(y4), P(sc), P(sh), P(mu), P(istd), P(res), P(rs), None, P(dr0),
         *S(q0), stream())
    ntp = LIB.dfcsa_bwd_block_out_pool_ntiles(B, H, W, C)
    d1, dr1 = (torch.empty(M, C, device=dev, dtype=dtype) for _ in range(2))
    q1 = torch.empty(ntp * 3 * C, device=dev)
    call("dfcsa_bwd_block_out_pool", T, B, H, W, C, P(gs), P(out1), P(gp), P(y4), P(sc), P(sh), P(mu), P(istd),
         P(res), P(rs), P(d1), P(dr1), *S(q1), stream())
    torch.cuda.synchronize()
    assert torch.equal(out1, out0) and torch.equal(p1, p0)
    assert torch.equal(d1, d0) and torch.equal(dr1, dr0)
    assert rel(q1.view(ntp, 3, C).double().sum(0), q0.view(nte, 3, C).double().sum(0)) < 1e-5


def _reduce_ref(slab, splits, NI, NJ, layout, ntaps, Ctot, Creal, ndst):
    """torch restatement of dfcsa_wgrad_reduce: sum the split slabs, then map the [NI][NJ] GEMM
    element (i, j) into the reference weight layouts (wgrad.hip reduce_dst_add)."""
    s = slab[:splits * NI * NJ].view(splits, NI, NJ).double().sum(0)
    if layout == 0:
        rows = NI // ndst
        g = s[:, :ntaps * Ctot].view(NI, ntaps, Ctot)[:, :, :Creal].permute(0, 2, 1)   # [NI][Creal][taps]
        return [g[d * rows:(d + 1) * rows].reshape(-1) for d in range(ndst)]
    g = s.view(NI, 4, Ctot).permute(0, 2, 1)                                        # ConvT [Cin][Cout][4]
    return [g.reshape(-1)]


@pytest.mark.parametrize("layout,ntaps,NI,Ctot,Creal,ndst,extra", [
    (0, 9, 64, 128, 128, 1, 0), (0, 9, 96, 72, 67, 2, 8), (0, 1, 48, 512, 512, 3, 0), (0, 9, 16, 8, 3, 1, 0),
    (1, 4, 40, 96, 96, 1, 0)])
@pytest.mark.parametrize("splits", [1, 3, 7, 16, 17, 40, 56, 70])
def test_wgrad_reduce_layouts(layout, ntaps, NI, Ctot, Creal, ndst, extra, splits):
    """The split-K reduction into the reference weight layouts (Conv2d [Cout][Cin][kh][kw] with K
    padding columns and channel padding, three stacked destinations, ConvTranspose2d [Cin][Cout][2][2]):
    the tap-transposing kernel (<= 16 splits) and the element-order kernel (knob 23 / > 16 splits)
    against a float64 torch reduction; each destination starts non-zero (the reduction adds)."""
    import dfcsa
    torch.manual_seed(splits + 31 * NI)
    T = ntaps if layout == 0 else 4
    NJ = T * Ctot + extra
    slab = torch.randn(splits * NI * NJ, device="cuda")
    ref = _reduce_ref(slab.cpu(), splits, NI, NJ, layout, ntaps, Ctot, Creal, ndst)
    for old in (0, 1):
        dfcsa.set_tuning(23, old)
        try:
            dsts = [torch.full((r.numel(),), 0.5, device="cuda") for r in ref]
            ops.wgrad_reduce(slab, splits, NI, NJ, layout, ntaps, Ctot, Creal, dsts)
            torch.cuda.synchronize()
        finally:
            dfcsa.set_tuning(23, 0)
        for d, r in zip(dsts, ref):
            assert (d.double().cpu() - 0.5 - r).abs().max().item() < 1e-5 * max(1.0, splits ** 0.5)


@pytest.mark.parametrize("B,H,Cs,nsrc,taps,N", [(4, 14, 512, 2, 9, 512), (16, 14, 1024, 1, 11, 512), (3, 13, 256, 1, 9, 136),
                                               (8, 14, 1024, 3, 1, 1024)])
def test_conv_splitk_matches_unsplit(B, H, Cs, nsrc, taps, N):
    """Split-K launch (few 128x128 tiles, long K: the 14^2 bottleneck / 28^2 layers) against the
    unsplit kernel (knob 25 = 0) and a torch fp32 reference: outputs and BN statistics; partial M /
    N tiles included; the split plan is visible through dfcsa_conv_work_floats."""
    import ctypes

    import dfcsa
    from dfcsa import _lib
    torch.manual_seed(5)
    bf = torch.bfloat16
    xs = [q(torch.randn(B, Cs, H, H), bf) for _ in range(nsrc)]
    xh = [nhwc(x, bf) for x in xs]
    if taps == 9:
        segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xh]
    elif taps == 11:
        segs = [(xh[0], 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(xh[0], 0, 0), (xh[0], 0, 0)]
    else:
        segs = [(x, 0, 0) for x in xh]
    K = len(segs) * Cs
    Kp = ops.rup(K, 64)
    w = q(torch.randn(N, Kp) * 0.02, bf)
    b = torch.randn(N)
    M = B * H * H
    outs, sts = [], []
    for knob in (1, 0):
        dfcsa.set_tuning(25, knob)
        try:
            y = torch.full((B, H, H, N), float("nan"), dtype=bf, device="cuda")
            stats = torch.full((ops.ntiles_gemm(M) * 2 * N,), float("nan"), device="cuda")
            rows = ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w.to("cuda", bf), Kp, N, [y], N, bias=b.cuda(),
                                 stats=stats)
            torch.cuda.synchronize()
        finally:
            dfcsa.set_tuning(25, 1)
        outs.append(y.float().cpu())
        sts.append(stats[:rows * 2 * N].view(-1, 2, N).sum(0).cpu())
    # the reference: the same gathered operand as one GEMM
    cols = []
    for t, dh, dw in segs:
        tc = t.float().cpu()
        sh = torch.zeros_like(tc)
        hs, he = max(0, -dh), H - max(0, dh)
        ws, we = max(0, -dw), H - max(0, dw)
        sh[:, hs:he, ws:we] = tc[:, hs + dh:he + dh, ws + dw:we + dw]
        cols.append(sh.reshape(M, Cs))
    A = torch.cat(cols, 1)
    acc = A @ w[:, :K].t()
    ref = acc + b
    for o, st in zip(outs, sts):
        assert torch.isfinite(o).all()
        assert rel(o.reshape(M, N), ref) < 1e-2
        assert rel(st[0], acc.sum(0)) < 1e-4 and rel(st[1], (acc * acc).sum(0)) < 1e-4
    assert rel(outs[0], outs[1]) < 5e-3


@pytest.mark.parametrize("B,H,C", [(2, 20, 64), (1, 37, 128), (16, 56, 64)])
def test_wgrad_pair_layout3(B, H, C):
    """The fusion conv's and the gate conv's weight gradients as one GEMM (G = [dy4 | dy3] over
    [fused | local | attn], layout 3) against the two separate launches and a torch fp32 reference."""
    torch.manual_seed(C + H)
    bf = torch.bfloat16
    xs = [q(torch.randn(B, C, H, H), bf) for _ in range(3)]            # fused, local, attn
    g4, g3 = (q(torch.randn(B, C, H, H) * 0.1, bf) for _ in range(2))
    xh = [nhwc(x, bf) for x in xs]
    segs = [(x, 0, 0) for x in xh]
    w4 = torch.zeros(C, 3 * C, 1, 1, device="cuda")
    w3 = torch.zeros(C, 2 * C, 1, 1, device="cuda")
    ops.conv_wgrad_into(bf, [nhwc(g4, bf), nhwc(g3, bf)], C, segs, C, (B, H, H), (H, H), [w4, w3], 1, C, 3 * C,
                        layout=3)
    s4 = torch.zeros_like(w4)
    s3 = torch.zeros_like(w3)
    ops.conv_wgrad_into(bf, [nhwc(g4, bf)], C, segs, C, (B, H, H), (H, H), [s4], 1, 3 * C, 3 * C)
    ops.conv_wgrad_into(bf, [nhwc(g3, bf)], C, segs[1:], C, (B, H, H), (H, H), [s3], 1, 2 * C, 2 * C)
    torch.cuda.synchronize()
    X = torch.cat(xs, 1).permute(0, 2, 3, 1).reshape(-1, 3 * C)
    r4 = g4.permute(0, 2, 3, 1).reshape(-1, C).t() @ X
    r3 = g3.permute(0, 2, 3, 1).reshape(-1, C).t() @ X[:, C:]
    assert rel(w4.view(C, -1), r4) < 1e-5 and rel(w3.view(C, -1), r3) < 1e-5
    assert rel(w4, s4) < 1e-6 and rel(w3, s3) < 1e-6


@pytest.mark.parametrize("B,H,W,Cs,nsrc,taps,NI,NG", [(2, 20, 20, 64, 2, 9, 64, 1), (3, 14, 14, 128, 1, 9, 128, 1),
                                                      (1, 37, 29, 64, 1, 9, 256, 1), (4, 28, 28, 64, 2, 1, 64, 2),
                                                      (2, 56, 56, 64, 3, 1, 64, 1), (16, 7, 7, 256, 1, 9, 512, 1)])
def test_wgrad_buffer_descriptor_kernel(B, H, W, Cs, nsrc, taps, NI, NG):
    """The buffer-descriptor weight-gradient kernel (64-channel sub-images, knob 26) against the
    pointer-DMA kernel: bit-identical (same images, same MFMA order), and against torch fp32."""
    import dfcsa
    torch.manual_seed(B * H + Cs)
    bf = torch.bfloat16
    xs = [q(torch.randn(B, Cs, H, W), bf) for _ in range(nsrc)]
    gs = [q(torch.randn(B, NI, H, W) * 0.1, bf) for _ in range(NG)]
    xh = [nhwc(x, bf) for x in xs]
    gh = [nhwc(g, bf) for g in gs]
    if taps == 9:
        segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xh]
    else:
        segs = [(x, 0, 0) for x in xh]
    k = 3 if taps == 9 else 1
    outs = []
    for bd in (1, 0):
        dfcsa.set_tuning(26, bd)
        try:
            grads = [torch.zeros(NI, nsrc * Cs, k, k, device="cuda") for _ in range(NG)]
            ops.conv_wgrad_into(bf, gh, NI, segs, Cs, (B, H, W), (H, W), grads, taps, nsrc * Cs, nsrc * Cs)
            torch.cuda.synchronize()
        finally:
            dfcsa.set_tuning(26, 1)
        outs.append(grads)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    x = torch.cat(xs, 1)
    for g, dw in zip(gs, outs[0]):
        ref = torch.nn.grad.conv2d_weight(x, (NI, nsrc * Cs, k, k), g, padding=k // 2)
        assert rel(dw, ref) < 1e-5


@pytest.mark.parametrize("B,H,C,P", [(2, 14, 64, 4), (3, 37, 128, 4), (16, 224, 64, 4), (4, 14, 1024, 4), (2, 9, 64, 2),
                                     (2, 11, 16, 3), (16, 28, 512, 4)])
def test_lsa_core_bwd_fused_matches_three_launches(B, H, C, P):
    """dfcsa_lsa_core_bwd (one launch per image) against dfcsa_lsa_up_bwd_cols + dfcsa_lsa_attn_bwd
    on the same upsample-backward rows: dq / dk / dv and dgamma."""
    from dfcsa._lib import LIB  # noqa: F401
    from dfcsa._lib import call
    from dfcsa.ops import P as ptr, stream
    torch.manual_seed(B + H + C)
    N, Cq = P * P, C // 8
    J = 2 * Cq + C
    rows = torch.randn(B * H * P * C, device="cuda")
    o = torch.randn(B, N, C, device="cuda")
    gamma = torch.tensor([0.37], device="cuda")
    qkv = torch.randn(B, N, J, device="cuda")
    A = torch.softmax(torch.randn(B, N, N, device="cuda"), -1)
    d1 = torch.full((B, N, J), float("nan"), device="cuda")
    g1 = torch.zeros(1, device="cuda")
    gp1 = torch.empty(B, device="cuda")
    sdO = torch.empty(B, N, C, device="cuda")
    sdE = torch.empty(B, N, N, device="cuda")
    gp1 = torch.empty(B * N, device="cuda")
    call("dfcsa_lsa_core_bwd", B, H, C, Cq, P, ptr(rows), ptr(o), ptr(gamma), ptr(qkv), ptr(A), ptr(d1), ptr(sdO),
         ptr(sdE), ptr(gp1), ptr(g1), stream())
    dO = torch.empty(B, N, C, device="cuda")
    gp2 = torch.empty(B * N, device="cuda")
    g2 = torch.zeros(1, device="cuda")
    call("dfcsa_lsa_up_bwd_cols", B, H, C, P, ptr(rows), ptr(o), ptr(gamma), ptr(dO), ptr(gp2), None, ptr(g2),
         stream())
    dE = torch.empty(B, N, N, device="cuda")
    d2 = torch.full((B, N, J), float("nan"), device="cuda")
    call("dfcsa_lsa_attn_bwd", B, N, C, Cq, ptr(qkv), ptr(A), ptr(dO), ptr(dE), ptr(d2), stream())
    torch.cuda.synchronize()
    assert torch.isfinite(d1).all()
    assert rel(d1, d2) < 1e-5
    assert abs(g1.item() - g2.item()) <= 1e-5 * max(1.0, abs(g2.item()))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,H,W,C,P,relu", [(2, 224, 224, 64, 32, 1), (2, 112, 112, 128, 16, 1), (3, 28, 28, 512, 32, 1),
                                            (2, 14, 14, 1024, 32, 0), (2, 30, 17, 256, 16, 1), (1, 9, 13, 16, 16, 1),
                                            (2, 56, 56, 8, 16, 0), (3, 56, 56, 256, 8, 1), (2, 28, 30, 512, 8, 1),
                                            (2, 14, 14, 1024, 8, 1)])
def test_lsa_pool_direct_matches_sliced_pool(B, H, W, C, P, relu, dtype):
    """dfcsa_lsa_pool_direct (one wave per window: P >= 16, or P = 8 with windows of <= 8 x 8) against the sliced pool + pooled launches
    (dfcsa_lsa_pool_ws + dfcsa_lsa_pooled_ws) and an fp64 adaptive average pool: the window means,
    their bf16 copy, and the window sums (sum r exactly: a pixel count)."""
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P as ptr, dt, stream
    assert LIB.dfcsa_lsa_pool_direct_ok(C, P, H, W) == 1
    torch.manual_seed(B + H + C + P)
    y = torch.randn(B, H, W, C, device="cuda").to(dtype)
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda") * 0.3
    N = P * P
    pooled = torch.full((B, N, C), float("nan"), device="cuda")
    p16 = torch.empty((B, N, C), device="cuda", dtype=torch.bfloat16)
    wsum = torch.full((B, N, 2, C), float("nan"), device="cuda")
    call("dfcsa_lsa_pool_direct", dt(dtype), B, H, W, C, ptr(y), ptr(sc), ptr(sh), P, relu, ptr(pooled), ptr(p16),
         ptr(wsum), stream())
    S = LIB.dfcsa_lsa_pool_splits(H, P)
    part = torch.empty(B * N * S * C, device="cuda")
    wpart = torch.empty(B * N * S * 2 * C, device="cuda")
    pooled2 = torch.empty((B, N, C), device="cuda")
    wsum2 = torch.empty((B, N, 2, C), device="cuda")
    call("dfcsa_lsa_pool_ws", dt(dtype), B, H, W, C, ptr(y), ptr(sc), ptr(sh), P, relu, ptr(part), ptr(wpart), stream())
    call("dfcsa_lsa_pooled_ws", B, H, W, C, P, ptr(part), ptr(pooled2), ptr(wpart), ptr(wsum2), stream())
    torch.cuda.synchronize()
    t = y.double() * sc.double() + sh.double()
    a = t.clamp_min(0) if relu else t
    ref = F.adaptive_avg_pool2d(a.permute(0, 3, 1, 2).cpu(), (P, P)).permute(0, 2, 3, 1).reshape(B, N, C)
    assert rel(pooled.cpu(), ref) < 1e-6
    assert rel(pooled, pooled2) < 1e-6
    assert torch.equal(p16, pooled.bfloat16())
    assert torch.equal(wsum[:, :, 0], wsum2[:, :, 0])
    assert rel(wsum[:, :, 1], wsum2[:, :, 1]) < 1e-6


def _bilinear_matrix(out, inp):
    """[out][inp] weights of F.interpolate(bilinear, align_corners=False) along one axis."""
    eye = torch.eye(inp, dtype=torch.float64).view(inp, 1, inp, 1)
    return F.interpolate(eye, size=(out, 1), mode="bilinear", align_corners=False)[:, 0, :, 0].T


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,H,W,C,P", [(16, 224, 224, 64, 4), (2, 14, 14, 1024, 4), (3, 28, 28, 512, 4),
                                       (2, 13, 17, 24, 3), (2, 9, 11, 192, 2), (1, 7, 5, 2048, 4), (2, 10, 6, 8, 1),
                                       (2, 20, 12, 64, 8)])
def test_lsa_up_bwd_rows_and_pool(B, H, W, C, P, dtype):
    """The column-owner upsample-backward row kernel (and the item-owner one, knob 28) against the
    transposed bilinear matrix, and the BN+ReLU adaptive average pool against PyTorch (fp64 CPU)."""
    import dfcsa
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P as ptr, stream
    torch.manual_seed(H * W + C)
    d = torch.randn(B, H, W, C).to(dtype)
    ref = torch.einsum("bhwc,wp->bhpc", d.double(), _bilinear_matrix(W, P))
    dc = d.cuda()
    for old in (0, 1):
        dfcsa.set_tuning(28, old)
        try:
            rows = torch.full((B * H * P * C,), float("nan"), device="cuda")
            call("dfcsa_lsa_up_bwd_rows", ops.dt(dtype), B, H, W, C, ptr(dc), P, ptr(rows), stream())
            torch.cuda.synchronize()
        finally:
            dfcsa.set_tuning(28, 0)
        assert rel(rows.view(B, H, P, C), ref) < 1e-6, old
    sc = torch.rand(C) + 0.5
    sh = torch.randn(C) * 0.3
    scc, shc = sc.cuda(), sh.cuda()   # kept alive across the launches
    S = LIB.dfcsa_lsa_pool_splits(H, P)
    part = torch.full((B * P * P * S * C,), float("nan"), device="cuda")
    pooled = torch.empty(B, P * P, C, device="cuda")
    call("dfcsa_lsa_pool", ops.dt(dtype), B, H, W, C, ptr(dc), ptr(scc), ptr(shc), P, 1, ptr(part),
         stream())
    call("dfcsa_lsa_pooled", B, H, W, C, P, ptr(part), ptr(pooled), stream())
    torch.cuda.synchronize()
    act = torch.relu(d.double() * sc.double() + sh.double()).permute(0, 3, 1, 2)
    pref = F.adaptive_avg_pool2d(act, P).permute(0, 2, 3, 1).reshape(B, P * P, C)
    assert rel(pooled, pref) < 1e-6


@pytest.mark.parametrize("M,Cq,C", [(256, 8, 64), (256, 16, 128), (5000, 8, 64)])
def test_wgrad_layout2_bias_sums(M, Cq, C):
    """The LightSelfAttention projection backward: q/k/v weight gradients (layout 2) and, in the same
    dfcsa_conv_wgrad call, the bias gradients (pixel sums of dqkv) -- inside the small fp32 kernel at
    M <= 4096, by the column-sum launch after the weight gradient otherwise -- against torch fp32 and
    the separate dfcsa_slab_colsum3 launch, accumulated onto existing gradients."""
    from dfcsa._lib import call
    torch.manual_seed(M + C)
    J = 2 * Cq + C
    g = torch.randn(M, J, device="cuda")
    x = torch.randn(M, C, device="cuda")
    ws = [torch.randn(Cq, C, 1, 1, device="cuda"), torch.randn(Cq, C, 1, 1, device="cuda"),
          torch.randn(C, C, 1, 1, device="cuda")]
    bs = [torch.randn(Cq, device="cuda"), torch.randn(Cq, device="cuda"), torch.randn(C, device="cuda")]
    w0 = [w.clone() for w in ws]
    b0 = [b.clone() for b in bs]
    ops.conv_wgrad_into(torch.float32, [g], J, [(x, 0, 0)], C, (1, M, 1), (M, 1), ws, 1, Cq, C, layout=2,
                        bias_grads=bs)
    sep = [b.clone() for b in b0]
    call("dfcsa_slab_colsum3", ops.P(g), M, J, Cq, Cq, ops.P(sep[0]), ops.P(sep[1]), ops.P(sep[2]), ops.stream())
    torch.cuda.synchronize()
    dw = g.t() @ x
    db = g.sum(0)
    for k, (lo, hi) in enumerate(((0, Cq), (Cq, 2 * Cq), (2 * Cq, J))):
        assert rel(ws[k].view(hi - lo, C) - w0[k].view(hi - lo, C), dw[lo:hi]) < 1e-5
        assert rel(bs[k] - b0[k], db[lo:hi]) < 1e-5
        assert (bs[k] - sep[k]).abs().max().item() <= 1e-5 * (1 + sep[k].abs().max().item())


@pytest.mark.parametrize("M,Cq,C", [(256, 8, 64), (64, 16, 128), (5000, 8, 64)])
def test_wgrad_dgrad1x1_one_launch(M, Cq, C):
    """dfcsa_conv_wgrad_dgrad1x1 (the LightSelfAttention projection backward): the layout-2 weight and
    bias gradients and dpooled = dqkv * W in one launch (M <= 4096) or two (M > 4096), against torch
    fp32 and the separate calls."""
    from dfcsa.block import rup
    torch.manual_seed(M + Cq)
    J = 2 * Cq + C
    g = torch.randn(M, J, device="cuda")
    x = torch.randn(M, C, device="cuda")
    W = torch.randn(J, C, device="cuda")               # stacked q/k/v weights [J][C]
    Kj = rup(J, ops.KALIGN)
    WT = torch.zeros(C, Kj, device="cuda")
    WT[:, :J] = W.t()
    ws = [torch.zeros(Cq, C, 1, 1, device="cuda"), torch.zeros(Cq, C, 1, 1, device="cuda"),
          torch.zeros(C, C, 1, 1, device="cuda")]
    bs = [torch.zeros(Cq, device="cuda"), torch.zeros(Cq, device="cuda"), torch.zeros(C, device="cuda")]
    dx = torch.empty(M, C, device="cuda")
    ops.conv_wgrad_dgrad1x1(torch.float32, g, J, x, C, M, ws, 1, Cq, C, WT, Kj, C, dx, layout=2, bias_grads=bs)
    ws2 = [torch.zeros_like(w) for w in ws]
    bs2 = [torch.zeros_like(b) for b in bs]
    ops.conv_wgrad_into(torch.float32, [g], J, [(x, 0, 0)], C, (1, M, 1), (M, 1), ws2, 1, Cq, C, layout=2,
                        bias_grads=bs2)
    dx2 = torch.empty(M, C, device="cuda")
    ops.conv_gemm(torch.float32, [(g, 0, 0)], J, (1, M, 1), (M, 1), WT, Kj, C, [dx2], C)
    torch.cuda.synchronize()
    assert rel(dx, g @ W) < 1e-5 and rel(dx, dx2) < 1e-6   # (the one-launch kernel splits K over 8 waves)
    dw = g.t() @ x
    for k, (lo, hi) in enumerate(((0, Cq), (Cq, 2 * Cq), (2 * Cq, J))):
        assert rel(ws[k].view(hi - lo, C), dw[lo:hi]) < 1e-5 and torch.equal(ws[k], ws2[k])
        assert rel(bs[k], g[:, lo:hi].sum(0)) < 1e-5 and torch.equal(bs[k], bs2[k])


@pytest.mark.parametrize("B,h,w,Cin,Cout", [(2, 5, 7, 64, 16), (4, 28, 28, 256, 128), (3, 13, 9, 128, 64),
                                            (16, 56, 56, 128, 64)])
def test_conv_transpose_fwd_streaming(B, h, w, Cin, Cout):
    """The ConvTranspose2d(2, 2) forward GEMM on the streaming 1x1 kernel (shuffle store, knob 34;
    knob 33 = 0 lets it take every M) against the tile kernel (knob 34 = 0) and torch."""
    from dfcsa.functions import ConvTranspose2x2
    bf = torch.bfloat16
    torch.manual_seed(Cin + h)
    mod = torch.nn.ConvTranspose2d(Cin, Cout, 2, 2).cuda()
    with torch.no_grad():
        mod.weight.copy_(q(mod.weight.cpu(), bf).cuda())
    x = q(torch.randn(B, Cin, h, w), bf)
    xh = nhwc(x, bf)
    outs = []
    old33 = ops._lib.LIB.dfcsa_get_tuning(33)
    try:
        for knob34 in (1, 0):
            ops._lib.LIB.dfcsa_set_tuning(33, 0)
            ops._lib.LIB.dfcsa_set_tuning(34, knob34)
            with torch.no_grad():
                outs.append(ConvTranspose2x2.apply(xh, mod, bf, *mod.parameters()).clone())
        torch.cuda.synchronize()
    finally:
        ops._lib.LIB.dfcsa_set_tuning(33, old33)
        ops._lib.LIB.dfcsa_set_tuning(34, 1)
    with torch.no_grad():
        ref = torch.nn.functional.conv_transpose2d(x, mod.weight.cpu(), mod.bias.cpu(), stride=2)
    assert rel(outs[0].float(), outs[1].float()) < 4e-3   # same K order; a bf16 rounding flip at most
    assert rel(nchw(outs[0]), ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,C", [(4096, 64), (3000, 128), (50176, 256)])
def test_bwd_relu_bn_pair_equals_two_launches(dtype, M, C):
    """dfcsa_bwd_relu_bn_pair: two BatchNorm-backward statistics passes in one launch, bit-identical
    to two dfcsa_bwd_relu_bn launches."""
    from dfcsa._lib import LIB, call
    from dfcsa.ops import P, stream
    torch.manual_seed(M + C)
    t = lambda: torch.randn(M, C, device="cuda").to(dtype)   # noqa: E731
    v = lambda: torch.randn(C, device="cuda")                 # noqa: E731
    d0, y0, d1, y1 = t(), t(), t(), t()
    bn = [(v(), v(), v(), v().abs() + 0.5) for _ in range(2)]
    nt = LIB.dfcsa_ew_ntiles(M, C)
    pa, pb = torch.empty(nt * 2 * C, device="cuda"), torch.empty(nt * 2 * C, device="cuda")
    qa, qb = torch.empty_like(pa), torch.empty_like(pb)
    dt = 1 if dtype == torch.bfloat16 else 0
    call("dfcsa_bwd_relu_bn_pair", dt, M, C, P(d0), P(y0), *[P(x) for x in bn[0]], P(pa), P(d1), P(y1),
         *[P(x) for x in bn[1]], P(pb), pa.numel(), stream())
    call("dfcsa_bwd_relu_bn", dt, M, C, P(d0), P(y0), *[P(x) for x in bn[0]], None, P(qa), qa.numel(), stream())
    call("dfcsa_bwd_relu_bn", dt, M, C, P(d1), P(y1), *[P(x) for x in bn[1]], None, P(qb), qb.numel(), stream())
    torch.cuda.synchronize()
    assert torch.equal(pa, qa) and torch.equal(pb, qb)
