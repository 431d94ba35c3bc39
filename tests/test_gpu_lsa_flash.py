"""Pooled attention for large pools (configs/config_dfc-sa-res-block-p16.yaml / -p32.yaml: N = 256 /
1024 tokens) on the flash kernels (dfcsa_lsa_flash_fwd / _bwd, csrc/fra.hip).

fp32 (parity) mode keeps the per-row kernels (pinned by the reference's LightSelfAttention fixtures at
P = 16 / 32, tests/test_gpu_model.py::test_lsa_fp32, and the model-level float64 oracle checks,
tests/test_gpu_qk_ratio.py::test_large_pool_model_matches_oracle); the flash kernels' fp32 variant is
checked against them below.  Here: the bf16 MFMA
kernels at the widths the model uses (C = 64 .. 1024, q/k width C / 8; C >= 512 takes the
value-chunked backward) against the oracle's LightSelfAttention (oracle/dfcsa_oracle.py:68-81) in
float64 on the same bf16-rounded input.  Tolerance per quantity: max(2e-2, 2x the reference's own
error under CPU bf16 autocast on the same layer and input, 1.5x the bf16 rounding of the output
itself) -- the reference's bmm q k^T / v A^T run in bf16 there too, as do our MFMA kernels
(tools/lsa_flash_err.py: at C = 256 .. 1024 the flash kernels are 2-3x closer to float64 than the
reference's autocast; at C = 64 the bf16 storage of y dominates both our paths alike).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _module(C, P, seed):
    from models.unet_dfc_sa_res import LightSelfAttention
    torch.manual_seed(seed)
    m = LightSelfAttention(C, pool_size=P)
    with torch.no_grad():
        m.gamma.fill_(0.7)
        for conv in (m.query_conv, m.key_conv, m.value_conv):
            conv.weight.mul_(2.0)   # sharper softmax rows than the default init
    return m


@pytest.mark.parametrize("C,P,H,B,alike", [(64, 16, 28, 2, 0), (128, 16, 14, 3, 0), (256, 32, 14, 2, 0),
                                           (512, 32, 28, 2, 0), (1024, 32, 14, 1, 0), (512, 16, 7, 2, 0),
                                           (64, 8, 28, 2, 1), (256, 16, 14, 2, 1), (1024, 32, 14, 1, 1)])
def test_flash_bf16_matches_oracle(C, P, H, B, alike):
    """alike = 1: inputs 1 + 0.05 N(0, 1), so the pooled value rows are nearly the same for every key (as
    pooled features after BatchNorm + ReLU are in the model) and dS = P (dP - r) is a small difference
    of large terms: the rounding of dO must enter dP and r alike (dfcsa_lsa_flash_bwd's prep kernel)."""
    from dfcsa import _lib
    from oracle import dfcsa_oracle as O
    assert _lib.LIB.dfcsa_lsa_flash_path(C, C // 8, 2 * (C // 8) + C) == 1
    m = _module(C, P, 100 + C + P)
    g0 = torch.Generator().manual_seed(7 + C)
    x = torch.randn(B, C, H, H + 1, generator=g0)
    x = (1 + 0.05 * x if alike else x).bfloat16().float()
    gy = torch.randn(B, C, H, H + 1, generator=g0)
    # oracle in float64: y = gamma * up(attn(pool(x))) + x and its gradients
    sd = {"a." + k: v.detach().double().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    xr = x.double().clone().requires_grad_(True)
    yr = O.light_self_attention(xr, sd, "a", P)
    yr.backward(gy.double())
    # the reference's own bf16-autocast error on this layer (fp32 weights, CPU autocast)
    sa = {k: v.detach().float().clone().requires_grad_(True) for k, v in sd.items()}
    xa = x.clone().requires_grad_(True)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        ya = O.light_self_attention(xa, sa, "a", P)
    ya.float().backward(gy)
    # bf16 mode stores y and dx in bf16: where the attention term is small against x (dx against
    # the residual's gy) that rounding alone is a large part of the term -- 1.5x of it is admitted
    bf = lambda t: t.bfloat16().double()   # noqa: E731
    floor_y = rel(bf(yr.detach()) - xr.detach(), (yr - xr).detach())
    floor_dx = rel(bf(xr.grad) - gy.double(), xr.grad - gy.double())
    bar_y = max(2e-2, 2 * rel(ya.float() - x, (yr - xr).detach()), 1.5 * floor_y)
    bar_dx = max(2e-2, 2 * rel(xa.grad - gy, xr.grad - gy.double()), 1.5 * floor_dx)
    mg = m.cuda()
    mg.compute_dtype = torch.bfloat16
    xg = x.cuda().requires_grad_(True)
    y = mg(xg)
    y.backward(gy.cuda())
    torch.cuda.synchronize()
    # the attention term alone (y - x), where the bf16 error lives
    assert rel(y.float().cpu() - x, (yr - xr).detach()) < bar_y, bar_y
    assert rel(xg.grad - gy.cuda(), xr.grad - gy.double()) < bar_dx, bar_dx
    for n, p in mg.named_parameters():
        if n == "key_conv.bias":   # true gradient 0 (softmax is shift-invariant over keys)
            continue
        bar = max(2e-2, 2 * rel(sa["a." + n].grad, sd["a." + n].grad))
        assert rel(p.grad, sd["a." + n].grad) < bar, (n, bar)


@pytest.mark.parametrize("P", [16, 32])
def test_flash_fp32_equals_per_row_kernels(P, monkeypatch):
    """fp32 mode: the flash kernels' fp32 variant (opt-in, DFCSA_LSA_FLASH_FP32) and the per-row
    kernels (the fp32 path) agree on the same layer to fp32 rounding."""
    from dfcsa import block
    C, H, B = 64, 14, 2
    outs = []
    monkeypatch.setattr(block, "LSA_FLASH_FP32", [True])   # the fp32 flash kernels (opt-in)
    for min_n in (1 << 30, 64):
        monkeypatch.setattr(block, "LSA_FLASH_MIN_N", [min_n])
        m = _module(C, P, 5).cuda()
        m.compute_dtype = torch.float32
        g0 = torch.Generator().manual_seed(11)
        x = torch.randn(B, C, H, H, generator=g0).cuda().requires_grad_(True)
        y = m(x)
        y.backward(torch.randn(B, C, H, H, generator=g0).cuda())
        outs.append((y.detach(), x.grad.detach(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    (ya, dxa, ga), (yb, dxb, gb) = outs
    assert rel(yb, ya) < 1e-5 and rel(dxb, dxa) < 1e-5
    for n in ga:
        if n != "key_conv.bias":
            assert rel(gb[n], ga[n]) < 1e-4, n


def test_flash_rejects_bad_shapes():
    from dfcsa import _lib
    import ctypes
    nb = ctypes.c_int64()
    L = _lib.LIB
    assert L.dfcsa_lsa_flash_path(48, 6, 60) == 0            # q/k width not a power of two: fp32 kernels
    assert L.dfcsa_lsa_flash_bwd_bytes(_lib.DT_BF16, 2, 256, 48, 6, 60, ctypes.byref(nb)) != 0
    assert L.dfcsa_lsa_flash_bwd_bytes(_lib.DT_F32, 2, 256, 48, 6, 61, ctypes.byref(nb)) != 0   # ldq != 2Cq + C
    assert L.dfcsa_lsa_flash_bwd_bytes(_lib.DT_F32, 2, 256, 48, 6, 60, ctypes.byref(nb)) == 0 and nb.value > 0
    assert np.isfinite(nb.value)


def _cos(a, b):
    a, b = a.reshape(-1).double().cpu(), b.reshape(-1).double().cpu()
    return (a @ b / (a.norm() * b.norm() + 1e-300)).item()


@pytest.mark.parametrize("P", [8, 16, 32])
def test_flash_model_bf16_step_vs_float64(P, monkeypatch):
    """The whole bf16 train step at pool size P (64..512 features, 64 x 64, B = 2) with the pooled
    attention on the flash kernels (bf16 projections, the entry's pool-backward BatchNorm rows from
    dfcsa_lsa_pool_rows), against the float64 oracle (oracle/dfcsa_oracle.py) beside the same bf16 step
    with the per-row fp32 attention kernels: logits and loss within the per-row path's own distance to
    float64 plus 1e-2; the whole gradient's cosine distance to float64 at most 1.5x the per-row path's
    + 2e-3; every non-scalar attention-branch tensor's at most 2x + 1e-2 where the per-row path is within
    1-cos 0.05 of float64 (see below for the rest).  (At 64 x 64 with pools as
    large as the maps the bf16 step itself is far from float64 -- whole-gradient cosine ~0.96 on both
    paths -- so the bar is relative to the per-row path, not absolute.)"""
    from dfcsa import block
    from dfcsa.loss import sigmoid
    from models.unet_dfc_sa_res import UNetDFCSARes
    from oracle import dfcsa_oracle as O
    from utils.metrics import calculate_metrics
    torch.manual_seed(500 + P)
    m0 = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=P, precision="bf16")
    with torch.no_grad():
        for i, (n, p) in enumerate(sorted(m0.named_parameters())):
            if n.endswith("gamma"):
                p.fill_(0.3 + 0.05 * (i % 5))
    sd = {k: v.detach().clone() for k, v in m0.state_dict().items()}
    g0 = torch.Generator().manual_seed(600 + P)
    x = torch.randn(2, 3, 64, 64, generator=g0)
    t = (torch.rand(2, 1, 64, 64, generator=g0) > 0.5).float()
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    logits64, met64, g64, _ = O.forward_backward(sd64, x.double(), t.double(), P, {})
    runs = {}
    for tag, min_n in (("row", 1 << 30), ("flash", 32)):
        monkeypatch.setattr(block, "LSA_FLASH_MIN_N", [min_n])
        m = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=P, precision="bf16")
        m.load_state_dict(sd)
        m = m.cuda().train()
        logits = m(x.cuda())
        met = calculate_metrics(sigmoid(logits), t.cuda(), "bce_dice", {})
        met["loss"].backward()
        torch.cuda.synchronize()
        runs[tag] = (logits.float(), met["loss"].item(), {n: p.grad.detach() for n, p in m.named_parameters()})
    names = [n for n in g64 if not n.endswith(("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias",
                                                  "fusion_conv.0.bias", "key_conv.bias"))]
    ref = torch.cat([g64[n].reshape(-1) for n in names])
    dist = {}
    for tag, (lg, loss, gr) in runs.items():
        whole = 1 - _cos(torch.cat([gr[n].reshape(-1).double().cpu() for n in names]), ref)
        # non-scalar attention-branch tensors (a scalar's "cosine" is its sign: gamma's gradient is one
        # cancelling sum whose sign bf16 noise can flip on either path)
        attn = {n: 1 - _cos(gr[n], g64[n]) for n in names
                if ".attn_branch." in n and g64[n].numel() > 1 and g64[n].norm() > 0}
        dist[tag] = (rel(lg, logits64), abs(loss - met64["loss"].item()) / abs(met64["loss"].item()), whole, attn)
        print(f"P={P} {tag}: logits {dist[tag][0]:.3e} loss {dist[tag][1]:.3e} whole-gradient 1-cos {whole:.3e} "
              f"worst attention tensor 1-cos {max(attn.values()):.3e}")
    (lr, sr, wr, ar), (lf, sf, wf, af) = dist["row"], dist["flash"]
    assert lf <= lr + 1e-2 and sf <= sr + 1e-2
    assert wf <= 1.5 * wr + 2e-3, (wf, wr)
    for n in af:
        if ar[n] < 0.05:   # signal-dominated on the per-row path
            assert af[n] <= 2 * ar[n] + 1e-2, (n, af[n], ar[n])
        else:
            # noise-dominated on both paths: the query-bias gradient of a 64-channel layer at P = 32 (8
            # entries, a sum over 1024 queries of dq that mostly cancels) is 1-cos 0.12 from float64 on the
            # per-row path and ~0.45 on the flash path; that only the direction is still positively
            # correlated is checked here
            assert af[n] < 0.7, (n, af[n], ar[n])


@pytest.mark.parametrize("C,N,B", [(64, 256, 2), (256, 1024, 1), (512, 1024, 1)])
def test_flash_bwd_centred_dq_on_alike_keys(C, N, B):
    """Keys that are nearly the same (mean key + 2% spread, as pooled features give): dQ = sum_k dS K_k
    is then a small difference of large terms and the bf16 rounding residue of each dS row times the
    mean key is coherent.  The centred backward (knob 48, dQ = sum_k dS (K_k - kbar)) must stay close to
    float64 on the same bf16 operands, and closer than the uncentred one; dK / dV are unchanged by it."""
    import ctypes
    import dfcsa
    from dfcsa import _lib
    from dfcsa.ops import P as ptr, stream
    L = _lib.LIB
    Cq = C // 8
    ldq = 2 * Cq + C
    g0 = torch.Generator().manual_seed(C + N)
    q = torch.randn(B, N, Cq, generator=g0) * 0.5
    kb = torch.randn(B, 1, Cq, generator=g0) * 3
    k = kb + 0.06 * torch.randn(B, N, Cq, generator=g0)
    v = torch.randn(B, N, C, generator=g0)
    qkv16 = torch.cat([q, k, v], -1).bfloat16()
    dO = torch.randn(B, N, C, generator=g0)
    # float64 reference on the same bf16 operands
    q64, k64, v64 = (t.double().requires_grad_(True) for t in qkv16.double().split([Cq, Cq, C], -1))
    o64 = torch.softmax(q64 @ k64.transpose(1, 2), -1) @ v64
    o64.backward(dO.double())
    ref = [q64.grad, k64.grad, v64.grad]
    qg = qkv16.cuda().contiguous()
    o = torch.empty(B, N, C, device="cuda")
    lse = torch.empty(B, N, device="cuda")
    assert L.dfcsa_lsa_flash_fwd(_lib.DT_BF16, B, N, C, Cq, ldq, ptr(qg), ptr(o), ptr(lse), stream()) == 0
    nb = ctypes.c_int64()
    assert L.dfcsa_lsa_flash_bwd_bytes(_lib.DT_BF16, B, N, C, Cq, ldq, ctypes.byref(nb)) == 0
    work = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
    errs = {}
    old = L.dfcsa_get_tuning(48)
    try:
        for centre in (1, 0):
            dfcsa.set_tuning(48, centre)
            d = torch.full((B, N, ldq), float("nan"), device="cuda").bfloat16()
            dOg = dO.cuda()
            assert L.dfcsa_lsa_flash_bwd(_lib.DT_BF16, B, N, C, Cq, ldq, ptr(qg), ptr(dOg), ptr(o), ptr(lse), ptr(d),
                                         ptr(work), nb.value, stream()) == 0
            torch.cuda.synchronize()
            errs[centre] = [rel(t.float(), r) for t, r in zip(d.float().cpu().split([Cq, Cq, C], -1), ref)]
    finally:
        dfcsa.set_tuning(48, old)
    print(f"C={C} N={N}: dq/dk/dv rel err centred {errs[1]} uncentred {errs[0]}")
    assert errs[1][0] < 3e-2 and errs[1][0] <= errs[0][0]
    assert errs[1][1] == pytest.approx(errs[0][1], rel=1e-6, abs=1e-7)
    assert errs[1][2] == pytest.approx(errs[0][2], rel=1e-6, abs=1e-7)


@pytest.mark.parametrize("C,P,H,B", [(64, 16, 224, 2), (128, 32, 112, 2), (512, 32, 28, 2), (1024, 32, 14, 1),
                                     (256, 8, 56, 3), (64, 8, 224, 1)])
def test_flash_bwd_up_matches_separate_passes(C, P, H, B):
    """dfcsa_lsa_flash_bwd_up (column pass writing the bf16 dO / r itself) against dfcsa_lsa_up_bwd_cols +
    dfcsa_lsa_flash_bwd on the same rows / o / q,k,v: the q/k/v gradients (bf16 outputs: the fp32 du may
    differ in its last bits between the two summation orders, so a bf16 dO element can round the other
    way) and the dgamma partials."""
    import ctypes
    from dfcsa import _lib
    from dfcsa.ops import P as ptr, stream
    L = _lib.LIB
    N, Cq = P * P, C // 8
    J = 2 * Cq + C
    g0 = torch.Generator().manual_seed(C + P + H)
    rows = torch.randn(B * H * P * C, generator=g0).cuda()
    o = torch.randn(B, N, C, generator=g0).cuda()
    gamma = torch.tensor([0.7]).cuda()
    qkv16 = (torch.randn(B, N, J, generator=g0) * 0.5).bfloat16().cuda()
    lse = torch.empty(B * N, device="cuda")
    o2 = torch.empty(B, N, C, device="cuda")
    assert L.dfcsa_lsa_flash_fwd(_lib.DT_BF16, B, N, C, Cq, J, ptr(qkv16), ptr(o2), ptr(lse), stream()) == 0
    nb = ctypes.c_int64()
    assert L.dfcsa_lsa_flash_bwd_bytes(_lib.DT_BF16, B, N, C, Cq, J, ctypes.byref(nb)) == 0
    work = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
    d1 = torch.full((B, N, J), float("nan"), device="cuda").bfloat16()
    gp1 = torch.full((B * N,), float("nan"), device="cuda")
    assert L.dfcsa_lsa_flash_bwd_up(B, H, C, Cq, P, ptr(rows), ptr(o), ptr(gamma), ptr(qkv16), ptr(lse), ptr(d1),
                                    ptr(gp1), ptr(work), nb.value, stream()) == 0
    dO = torch.empty(B, N, C, device="cuda")
    gp2 = torch.empty(B * N, device="cuda")
    assert L.dfcsa_lsa_up_bwd_cols(B, H, C, P, ptr(rows), ptr(o), ptr(gamma), ptr(dO), ptr(gp2), None, None,
                                   stream()) == 0
    d2 = torch.full((B, N, J), float("nan"), device="cuda").bfloat16()
    assert L.dfcsa_lsa_flash_bwd(_lib.DT_BF16, B, N, C, Cq, J, ptr(qkv16), ptr(dO), ptr(o), ptr(lse), ptr(d2),
                                 ptr(work), nb.value, stream()) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(d1.float()).all()
    assert rel(gp1, gp2) < 1e-5
    for a, b_ in zip(d1.float().split([Cq, Cq, C], -1), d2.float().split([Cq, Cq, C], -1)):
        assert rel(a, b_) < 5e-3


@pytest.mark.parametrize("P", [8, 32])
def test_bf16_dpooled_path_is_bitwise_the_widened_one(P, monkeypatch):
    """The window-sum path of a bf16 flash layer reads the projection dgrad's bf16 dpooled as it is
    (dfcsa_lsa_pool_rows with dtype bf16, dfcsa_bn_bwd_apply_entry16) instead of widening it to fp32 first
    (DFCSA_LSA_DP16=0): bf16 -> fp32 is exact, so the whole train step's gradients are bitwise equal."""
    from dfcsa import block
    from dfcsa.loss import sigmoid
    from models.unet_dfc_sa_res import UNetDFCSARes
    from utils.metrics import calculate_metrics
    torch.manual_seed(900 + P)
    m0 = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=P, precision="bf16")
    with torch.no_grad():
        for n, p in m0.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.4)
    sd = {k: v.detach().clone() for k, v in m0.state_dict().items()}
    g0 = torch.Generator().manual_seed(910 + P)
    x = torch.randn(2, 3, 64, 64, generator=g0)
    t = (torch.rand(2, 1, 64, 64, generator=g0) > 0.5).float()
    grads = []
    for on in (True, False):
        monkeypatch.setattr(block, "LSA_DP16", [on])
        m = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=P, precision="bf16")
        m.load_state_dict(sd)
        m = m.cuda().train()
        met = calculate_metrics(sigmoid(m(x.cuda())), t.cuda(), "bce_dice", {})
        met["loss"].backward()
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    for n in grads[0]:
        assert torch.equal(grads[0][n], grads[1][n]), n
