"""MI355X parity of the TransUNet path (BASELINE config 4; reference models/transformer_unet.py).

Kernel level: every csrc/transunet.hip entry point against a plain PyTorch fp32 reference of the same
op (GroupNorm, LayerNorm, multi-head attention, MaxPool2d(3,2,1), UpsamplingBilinear2d, strided-conv
column gradient, 3x3 head, dropout).  Model level: the reduced R50-ViT configuration against the
golden fixture made by the reference itself (tests/golden/make_golden.py gen_transunet): logits and
loss 1e-4 (fp32 mode), Dice exact, every gradient against the reference re-run in float64 within
max(2e-3, 4x the reference's own fp32 error), BatchNorm running statistics 1e-5; bf16 mode 3e-2 on
logits.  Then the full 105 M-parameter model through the factory for a few bf16 train steps.
"""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
LP = {"bce_weight": 0.5, "dice_weight": 0.5}


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b).detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def T(a, dev="cuda"):
    return torch.from_numpy(np.asarray(a)).to(dev)


def lib():
    from dfcsa._lib import call
    from dfcsa.ops import P, dt, stream
    return call, P, dt, stream


# ----------------------------------------------------------------------------- kernels
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,C,G,H,eps", [(3, 64, 32, 14, 1e-6), (3, 256, 32, 7, 1e-6), (3, 64, 64, 9, 1e-5),
                                         (3, 32, 32, 5, 1e-6), (8, 1024, 32, 14, 1e-6), (8, 256, 32, 56, 1e-6),
                                         (8, 64, 32, 112, 1e-6), (3, 256, 1, 7, 1e-6), (2, 512, 2, 9, 1e-6),
                                         (2, 512, 16, 11, 1e-6)])
def test_groupnorm_fwd_bwd(B, C, G, H, eps, dtype, tol, fused):
    """GroupNorm fwd (+ReLU) and bwd against F.group_norm + ReLU autograd: the fused launches
    (dfcsa_gn_stats_fused / dfcsa_gn_bwd_reduce_fused: the finalisation by the last workgroup of each
    image and 128-channel chunk, dgamma / dbeta by the last image) and the four-launch path, at the test
    sizes and the TransUNet bench's (B = 8: 14^2 x 1024, 56^2 x 256, 112^2 x 64), plus groups wider than a
    chunk (G = 1; C = 512, G = 2: one chunk); the fused path twice, bitwise."""
    from dfcsa import transunet_ops as TU
    torch.manual_seed(C + G + H)
    gn = torch.nn.GroupNorm(G, C, eps=eps).cuda()
    with torch.no_grad():
        gn.weight.uniform_(0.5, 1.5)
        gn.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(B, H, H + 1, C, device="cuda") * 2 + 0.3).to(dtype)
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = F.relu(F.group_norm(xr, G, gn.weight, gn.bias, eps))
    g = torch.randn_like(yr)
    gw, gb = torch.autograd.grad(yr, [xr, gn.weight, gn.bias], g)[1:]
    dxr = torch.autograd.grad(F.relu(F.group_norm(xr, G, gn.weight, gn.bias, eps)), xr, g)[0]
    saved = TU.GN_FUSED[0]
    TU.GN_FUSED[0] = fused
    try:
        runs = []
        for _ in range(2 if fused else 1):
            st = TU.gn_forward(dtype, x.contiguous(), gn)
            out = TU.gn_apply(dtype, x.contiguous(), st, 1)
            gn.weight.grad = torch.zeros_like(gn.weight)
            gn.bias.grad = torch.zeros_like(gn.bias)
            dy = TU.gn_backward(dtype, g.permute(0, 2, 3, 1).contiguous().to(dtype), out, x.contiguous(), st, gn)
            torch.cuda.synchronize()
            runs.append((out.clone(), dy.clone(), gn.weight.grad.clone(), gn.bias.grad.clone()))
    finally:
        TU.GN_FUSED[0] = saved
    out, dy, gwo, gbo = runs[0]
    assert rel(out.float().permute(0, 3, 1, 2), yr) < tol
    assert rel(dy.float().permute(0, 3, 1, 2), dxr) < 5 * tol
    assert rel(gwo, gw) < 5 * tol and rel(gbo, gb) < 5 * tol
    if fused:
        assert all(torch.equal(a, b) for a, b in zip(runs[0], runs[1])), "fused GroupNorm is not bitwise repeatable"


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("rows,C", [(392, 768), (37, 64), (8, 32)])
def test_layernorm_fwd_bwd(rows, C, dtype, tol):
    from dfcsa import transunet_ops as TU
    torch.manual_seed(rows + C)
    ln = torch.nn.LayerNorm(C, eps=1e-6).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    h = torch.randn(rows, C, device="cuda") * 3 + 1
    hr = h.clone().requires_grad_(True)
    yr = F.layer_norm(hr, (C,), ln.weight, ln.bias, 1e-6)
    g = torch.randn_like(yr)
    dres = torch.randn_like(yr)
    dxr, dgr, dbr = torch.autograd.grad(yr, [hr, ln.weight, ln.bias], g)
    y, mr = TU._ln_forward(dtype, h, ln, (rows, C))
    assert rel(y, yr) < tol
    ln.weight.grad = torch.zeros_like(ln.weight)
    ln.bias.grad = torch.zeros_like(ln.bias)
    dx = TU._ln_backward(dtype, g.to(dtype), h, mr, ln, dres)
    assert rel(dx - dres, dxr) < 5 * tol
    assert rel(ln.weight.grad, dgr) < 5 * tol and rel(ln.bias.grad, dbr) < 5 * tol


def _mha_torch(qkv, B, N, heads, dh):
    D = heads * dh
    q, k, v = (qkv[..., i * D:(i + 1) * D].reshape(B, N, heads, dh).permute(0, 2, 1, 3) for i in range(3))
    a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(dh), dim=-1)
    return (a @ v).permute(0, 2, 1, 3).reshape(B, N, D)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,N,heads,dh", [(2, 196, 12, 64), (2, 50, 4, 32), (3, 4, 2, 16), (1, 130, 2, 16)])
def test_mha_fwd_bwd(B, N, heads, dh, dtype, tol):
    """Attention core (Attention.forward :146-154) with N not a multiple of the 64-row tiles."""
    call, P, dt, stream = lib()
    torch.manual_seed(N + heads)
    D = heads * dh
    qkv = (torch.randn(B, N, 3 * D, device="cuda") * 1.5).to(dtype)
    qr = qkv.float().clone().requires_grad_(True)
    yr = _mha_torch(qr, B, N, heads, dh)
    g = torch.randn_like(yr)
    dqr = torch.autograd.grad(yr, qr, g)[0]
    ctx = torch.empty((B, N, D), dtype=dtype, device="cuda")
    lse = torch.empty(B * heads * N, device="cuda")
    scale = 1.0 / math.sqrt(dh)
    call("dfcsa_mha_fwd", dt(dtype), B, N, heads, dh, 3 * D, scale, P(qkv), P(ctx), P(lse), stream())
    assert rel(ctx, yr) < tol
    dqkv = torch.empty_like(qkv)
    dvec = torch.empty(B * heads * N, device="cuda")
    call("dfcsa_mha_bwd", dt(dtype), B, N, heads, dh, 3 * D, scale, P(qkv), P(ctx), P(g.to(dtype)), P(lse), P(dvec),
         P(dqkv), stream())
    for i in range(3):
        assert rel(dqkv[..., i * D:(i + 1) * D], dqr[..., i * D:(i + 1) * D]) < 3 * tol, i


def _keep_mask(rng0, rng1, site, n, p):
    """numpy restatement of the counter-based dropout keep(i) of csrc/transunet.hip (drop_key,
    mix64, keep_elem) for element indices 0 .. n-1."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        key = (np.uint64(rng0) * np.uint64(0x100000001B3)) ^ (np.uint64(rng1) << np.uint64(20)) ^ \
            (np.uint64(site) << np.uint64(52))
        z = key ^ (np.arange(n, dtype=np.uint64) * np.uint64(0xD6E8FEB86659FD93))
        z = (z + np.uint64(0x9E3779B97F4A7C15)) & M
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M
        z = z ^ (z >> np.uint64(31))
    u = ((z >> np.uint64(32)) >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return u >= np.float32(p)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,N,heads,dh,p", [(2, 196, 12, 64, 0.1), (3, 50, 4, 32, 0.3), (1, 7, 2, 16, 0.5)])
def test_mha_attention_dropout(B, N, heads, dh, p, dtype, tol):
    """Attention-probability dropout (Attention.forward :146-151 with attention_dropout_rate = p):
    the kernel's mask regenerated here from the same counter-based key, ctx = (keep * P / (1 - p)) v
    and the q / k / v gradients against torch autograd with that mask; the stored probabilities are
    the undropped softmax; the keep rate is 1 - p."""
    call, P, dt, stream = lib()
    torch.manual_seed(N + 7 * heads)
    D = heads * dh
    qkv = (torch.randn(B, N, 3 * D, device="cuda") * 1.5).to(dtype)
    rng = torch.tensor([987654321, 5], dtype=torch.int64, device="cuda")
    site = 19
    keep = torch.from_numpy(_keep_mask(987654321, 5, site, B * heads * N * N, p)).view(B, heads, N, N)
    qr = qkv.float().cpu().clone().requires_grad_(True)
    q, k, v = (qr[..., i * D:(i + 1) * D].reshape(B, N, heads, dh).permute(0, 2, 1, 3) for i in range(3))
    a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(dh), dim=-1)
    yr = ((a * keep / (1 - p)) @ v).permute(0, 2, 1, 3).reshape(B, N, D)
    g = torch.randn_like(yr)
    dqr = torch.autograd.grad(yr, qr, g)[0]
    ctx = torch.empty((B, N, D), dtype=dtype, device="cuda")
    probs = torch.empty(B * heads * N * N, device="cuda")
    scale = 1.0 / math.sqrt(dh)
    call("dfcsa_mha_drop_fwd", dt(dtype), B, N, heads, dh, 3 * D, scale, P(qkv), p, P(rng), site, P(probs), P(ctx),
         stream())
    torch.cuda.synchronize()
    assert rel(probs.cpu().view(B, heads, N, N), a.detach()) < max(tol, 1e-6)
    assert rel(ctx, yr) < tol
    dqkv = torch.empty_like(qkv)
    dscores = torch.empty_like(probs)
    call("dfcsa_mha_drop_bwd", dt(dtype), B, N, heads, dh, 3 * D, scale, P(qkv), P(g.to("cuda", dtype)), P(probs), p,
         P(rng), site, P(dscores), P(dqkv), stream())
    torch.cuda.synchronize()
    for i in range(3):
        assert rel(dqkv[..., i * D:(i + 1) * D], dqr[..., i * D:(i + 1) * D]) < 3 * tol, i
    if B * heads * N * N > 100000:
        assert abs(keep.float().mean().item() - (1 - p)) < 0.01


def test_transunet_attention_dropout_train_step():
    """TransUNet with attention_dropout_rate > 0 (attn_dropout on the probabilities + proj_dropout):
    a train-mode forward/backward runs on the dropout path with finite gradients that differ from
    the p = 0 step, two steps draw different masks, and eval mode ignores the rate."""
    torch.manual_seed(0)
    m, fx = _small_model("fp32")
    x = torch.from_numpy(fx["x"]).cuda()
    m.config.transformer["attention_dropout_rate"] = 0.0
    m.eval()
    with torch.no_grad():
        y_eval0 = m(x).clone()
    m.config.transformer["attention_dropout_rate"] = 0.2
    with torch.no_grad():
        y_eval = m(x).clone()
    assert torch.equal(y_eval, y_eval0)
    m.train()
    outs, grads = [], []
    for _ in range(2):
        m.zero_grad(set_to_none=False)
        y = m(x)
        y.square().mean().backward()
        outs.append(y.detach().clone())
        grads.append(m.transformer.encoder.layer[0].attn.query.weight.grad.detach().clone())
    assert all(torch.isfinite(o).all() for o in outs) and all(torch.isfinite(gq).all() for gq in grads)
    assert not torch.equal(outs[0], outs[1])
    m.config.transformer["attention_dropout_rate"] = 0.0


@pytest.mark.parametrize("B,N,heads", [(2, 196, 12), (1, 130, 2), (3, 4, 2)])
def test_mha_flash_bf16(B, N, heads):
    """bf16 ViT attention on the MFMA flash kernels (head-major relayout, q pre-scaled): against the
    plain PyTorch fp32 attention of the same bf16 inputs, bf16 tolerances."""
    from dfcsa.transunet_ops import mha_flash_backward, mha_flash_forward
    torch.manual_seed(N + heads + B)
    dh = 64
    D = heads * dh
    qkv = (torch.randn(B, N, 3 * D, device="cuda") * 1.5).to(torch.bfloat16)
    qr = qkv.float().clone().requires_grad_(True)
    yr = _mha_torch(qr, B, N, heads, dh)
    g = torch.randn_like(yr)
    dqr = torch.autograd.grad(yr, qr, g)[0]
    cx, saved = mha_flash_forward(torch.bfloat16, qkv.view(B * N, 3 * D), B, N, heads, dh)
    assert rel(cx.view(B, N, D), yr) < 1e-2
    dqkv = mha_flash_backward(torch.bfloat16, saved, g.to(torch.bfloat16).view(B * N, D), B, N, heads, dh)
    dqkv = dqkv.view(B, N, 3 * D)
    for i in range(3):
        assert rel(dqkv[..., i * D:(i + 1) * D], dqr[..., i * D:(i + 1) * D]) < 3e-2, i


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,W", [(112, 112), (7, 9), (2, 3)])
def test_maxpool3s2(H, W, dtype):
    call, P, dt, stream = lib()
    torch.manual_seed(H * W)
    x = torch.randn(2, H, W, 16, device="cuda").to(dtype)
    x[0, :2, :2, :] = x[0, 0, 0, :]        # ties: the first maximum (scan order) takes the gradient
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    g = torch.randn_like(yr)
    dxr = torch.autograd.grad(yr, xr, g)[0]
    Ho, Wo = yr.shape[2], yr.shape[3]
    out = torch.empty((2, Ho, Wo, 16), dtype=dtype, device="cuda")
    idx = torch.empty((2, Ho, Wo, 16), dtype=torch.uint8, device="cuda")
    call("dfcsa_maxpool3s2_fwd", dt(dtype), 2, H, W, 16, P(x), P(out), P(idx), stream())
    assert torch.equal(out.float().permute(0, 3, 1, 2), yr)
    dx = torch.empty_like(x)
    gb = g.permute(0, 2, 3, 1).contiguous().to(dtype)
    call("dfcsa_maxpool3s2_bwd", dt(dtype), 2, H, W, 16, P(idx), P(gb), P(dx), stream())
    ref = torch.autograd.grad(F.max_pool2d(xr, 3, 2, 1), xr, gb.float().permute(0, 3, 1, 2))[0]
    # bf16: a pixel that is the maximum of several windows sums their gradients in fp32 and rounds once
    tol = dict(atol=1e-2, rtol=1e-2) if dtype == torch.bfloat16 else dict(atol=1e-6, rtol=0)
    d = dx.float().permute(0, 3, 1, 2)
    assert torch.allclose(d, ref, **tol), ((d - ref).abs().max().item(), (d != ref).sum().item())
    assert dxr is not None


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("H,W", [(14, 14), (1, 3), (5, 8)])
def test_upsample2_align_corners(H, W, dtype, tol):
    """nn.UpsamplingBilinear2d(scale_factor=2) (align_corners=True) and its gather backward."""
    call, P, dt, stream = lib()
    torch.manual_seed(H + W)
    x = torch.randn(2, H, W, 24, device="cuda").to(dtype)
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = torch.nn.UpsamplingBilinear2d(scale_factor=2)(xr)
    g = torch.randn_like(yr)
    dxr = torch.autograd.grad(yr, xr, g)[0]
    out = torch.empty((2, 2 * H, 2 * W, 24), dtype=dtype, device="cuda")
    call("dfcsa_upsample2_ac", dt(dtype), 2, 24, H, W, P(x), P(out), stream())
    assert rel(out.float().permute(0, 3, 1, 2), yr) < tol
    dx = torch.empty_like(x)
    call("dfcsa_upsample2_ac_bwd", dt(dtype), 2, 24, H, W, P(g.permute(0, 2, 3, 1).contiguous().to(dtype)), P(dx),
         stream())
    assert rel(dx.float().permute(0, 3, 1, 2), dxr) < 2 * tol


@pytest.mark.parametrize("k,s,p,H", [(3, 2, 1, 9), (3, 2, 1, 8), (1, 2, 0, 7), (3, 1, 1, 5)])
def test_col2im_matches_conv_input_grad(k, s, p, H):
    """dx of a k x k / stride s conv from the column gradient dcols = dY @ W (one GEMM + col2im)."""
    call, P, dt, stream = lib()
    torch.manual_seed(k * 10 + H)
    C, Co = 16, 8
    # reference on the host in float64 (ATen's CPU convolution)
    w = torch.randn(Co, C, k, k, dtype=torch.float64)
    x = torch.randn(2, C, H, H + 1, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, w, None, s, p)
    g = torch.randn_like(y)
    dxr = torch.autograd.grad(y, x, g)[0].float().cuda()
    w, g = w.float().cuda(), g.float().cuda()
    Ho, Wo = y.shape[2], y.shape[3]
    # dcols[b, oh, ow, (kh*k + kw)*C + c] = sum_o g[b, o, oh, ow] * w[o, c, kh, kw]
    dcols = torch.einsum("bohw,ocij->bhwijc", g, w).reshape(2, Ho, Wo, k * k * C).contiguous()
    dx = torch.full((2, H, H + 1, C), 0.5, device="cuda")
    call("dfcsa_col2im", 0, 2, H, H + 1, C, Ho, Wo, k, s, p, P(dcols), P(dx), 1, stream())
    assert rel(dx - 0.5, dxr.permute(0, 2, 3, 1)) < 1e-5


def test_dropout_masks():
    """keep rate 1-p, inverse scaling, backward reuses the forward mask, a new step draws a new mask,
    p = 0 is the identity."""
    call, P, dt, stream = lib()
    n = 1 << 20
    a = torch.randn(n, device="cuda")
    res = torch.randn(n, device="cuda")
    rng = torch.tensor([12345, 0], dtype=torch.int64, device="cuda")
    out = torch.empty(n, device="cuda")
    call("dfcsa_drop_add_fwd", 0, n, P(a), None, 0, P(res), 0.1, P(rng), 7, P(out), stream())
    kept = (out - res) != 0
    frac = kept.float().mean().item()
    assert abs(frac - 0.9) < 0.003, frac
    assert torch.allclose((out - res)[kept], a[kept] / 0.9, rtol=1e-5, atol=1e-5)
    g = torch.randn(n, device="cuda")
    da = torch.empty(n, device="cuda")
    call("dfcsa_drop_bwd", 0, n, P(g), 0.1, P(rng), 7, P(da), stream())
    assert torch.equal(da != 0, kept & (g != 0))
    call("dfcsa_rng_advance", P(rng), stream())
    out2 = torch.empty(n, device="cuda")
    call("dfcsa_drop_add_fwd", 0, n, P(a), None, 0, P(res), 0.1, P(rng), 7, P(out2), stream())
    assert ((out2 - res) != 0).ne(kept).float().mean().item() > 0.1
    call("dfcsa_drop_add_fwd", 0, n, P(a), None, 0, P(res), 0.0, P(rng), 7, P(out2), stream())
    assert torch.allclose(out2, a + res)
    x = torch.randn(n, device="cuda")
    gl = torch.empty(n, device="cuda")
    call("dfcsa_gelu_drop_fwd", 0, n, P(x), 0.0, P(rng), 3, P(gl), stream())
    assert torch.allclose(gl, F.gelu(x), atol=1e-6)
    dx = torch.empty(n, device="cuda")
    xr = x.clone().requires_grad_(True)
    ref = torch.autograd.grad(F.gelu(xr), xr, g)[0]
    call("dfcsa_gelu_drop_bwd", 0, n, P(x), P(g), 0.0, P(rng), 3, P(dx), stream())
    assert torch.allclose(dx, ref, atol=1e-5)


@pytest.mark.parametrize("B,H,W,C,Cout", [(2, 20, 24, 16, 1), (1, 37, 224, 16, 1), (1, 30, 100, 64, 3), (3, 9, 7, 8, 4)])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
def test_head3(dtype, tol, B, H, W, C, Cout):
    """3x3 segmentation head fwd/bwd vs torch fp32; (1, 30, 100, 64, 3) exceeds head3_bwd's LDS halo
    staging (the global-load weight-partial path), the others take the staged path."""
    from dfcsa.transunet_ops import SegHead3x3
    torch.manual_seed(4)
    conv = torch.nn.Conv2d(C, Cout, 3, padding=1).cuda()
    x = torch.randn(B, H, W, C, device="cuda").to(dtype)
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = conv(xr)
    g = torch.randn_like(yr)
    dxr, dwr, dbr = torch.autograd.grad(yr, [xr, conv.weight, conv.bias], g)
    xk = x.clone().requires_grad_(True)
    conv.weight.grad, conv.bias.grad = torch.zeros_like(conv.weight), torch.zeros_like(conv.bias)
    y = SegHead3x3.apply(xk, conv, dtype, *conv.parameters())
    assert rel(y, yr) < tol
    y.backward(g)
    assert rel(xk.grad.float().permute(0, 3, 1, 2), dxr) < tol
    assert rel(conv.weight.grad, dwr) < 2 * tol and rel(conv.bias.grad, dbr) < 2 * tol


# ----------------------------------------------------------------------------- model
def _small_model(precision):
    from models.transformer_unet import TransUNet
    from test_oracle_golden import transunet_small_config
    fx = dict(np.load(os.path.join(GOLDEN, "transunet_small.npz")))
    m = TransUNet(transunet_small_config(), img_size=32, num_classes=1, precision=precision)
    m.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")})
    return m.cuda().train(), fx


def test_transunet_small_fp32_matches_reference():
    from dfcsa.loss import sigmoid
    from utils.metrics import calculate_metrics
    m, fx = _small_model("fp32")
    logits = m(T(fx["x"]))
    met = calculate_metrics(sigmoid(logits), T(fx["t"]), "bce_dice", LP)
    met["loss"].backward()
    torch.cuda.synchronize()
    assert rel(logits, fx["logits"]) < 1e-4
    assert abs(met["loss"].item() - float(fx["loss"])) < 1e-4 * abs(float(fx["loss"]))
    assert abs(met["dice"] - float(fx["dice"])) < 1e-6
    ours, refs = [], []
    for n, p in m.named_parameters():
        ref = fx["grad64." + n]
        if n.endswith("attn.key.bias"):   # true gradient 0 (softmax shift invariance per query)
            assert p.grad.abs().max().item() < 1e-3 * np.abs(fx["grad64." + n[:-4] + "weight"]).max() + 1e-9, n
            continue
        lim = max(2e-3 if ref.size > 1 else 1e-2, 4 * max(float(fx["noise." + n]), float(fx["noise.all"])))
        r = rel(p.grad, ref)
        assert r < lim, (n, r, lim)
        ours.append(p.grad.double().cpu().reshape(-1))
        refs.append(torch.from_numpy(ref.astype(np.float64)).reshape(-1))
    assert rel(torch.cat(ours), torch.cat(refs)) < 1e-3
    for k, v in m.state_dict().items():
        if "running" in k:
            assert rel(v.float(), fx["buf." + k]) < 1e-5, k


def test_transunet_small_bf16_close_to_reference():
    from dfcsa.loss import sigmoid
    from utils.metrics import calculate_metrics
    m, fx = _small_model("bf16")
    logits = m(T(fx["x"]))
    met = calculate_metrics(sigmoid(logits), T(fx["t"]), "bce_dice", LP)
    met["loss"].backward()
    assert rel(logits, fx["logits"]) < 3e-2
    assert abs(met["loss"].item() - float(fx["loss"])) < 2e-2 * abs(float(fx["loss"]))
    g = torch.cat([p.grad.reshape(-1).double().cpu() for n, p in m.named_parameters()])
    r = torch.cat([torch.from_numpy(fx["grad64." + n].astype(np.float64)).reshape(-1) for n, _ in m.named_parameters()])
    cos = (g @ r / (g.norm() * r.norm())).item()
    # the reference itself under CPU bf16 autocast reaches bf16_autocast_grad_cos (0.959) against
    # its float64 run: bf16 rounding, not a kernel error, sets this bar
    assert cos > float(fx["bf16_autocast_grad_cos"]) - 0.01, (cos, float(fx["bf16_autocast_grad_cos"]))


def test_transunet_single_channel_input_repeats():
    """x.size(1) == 1 -> x.repeat(1, 3, 1, 1) (reference :363-364)."""
    m, fx = _small_model("fp32")
    m.eval()
    x1 = T(fx["x"])[:, :1]
    with torch.no_grad():
        a = m(x1)
        b = m(x1.repeat(1, 3, 1, 1))
    assert torch.equal(a, b)


def test_transunet_full_factory_bf16_train_steps():
    """config_transunet.yaml through the factory (R50-ViT-B/16, 224x224, 105.3 M parameters), batch 2,
    dropout 0.1 active: finite loss that decreases on a fixed batch over a few fused SGD steps."""
    from dfcsa.loss import sigmoid
    from dfcsa.optim import FusedSGD
    from models.model_factory import ModelFactory
    from utils.metrics import calculate_metrics_device
    torch.manual_seed(0)
    cfg = {"model": {"name": "TransformerUNet", "in_channels": 3, "out_channels": 1},
           "dataset": {"img_size": [224, 224]}, "training": {}}
    m = ModelFactory.get_model(cfg).cuda().train()
    assert sum(p.numel() for p in m.parameters()) == 105275921
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(2, 3, 224, 224, device="cuda")
    t = (x[:, :1] > 0.3).float()
    losses = []
    for _ in range(4):
        opt.zero_grad()
        met = calculate_metrics_device(sigmoid(m(x)), t, "bce_dice", {})
        met["loss"].backward()
        opt.step(max_norm=1.0, skip_if_nan=met["loss"])
        losses.append(met["loss"].item())
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,C,n0,n1", [(1568, 768, 768, 0), (1568, 2304, 768, 768), (1568, 3072, 3072, 0),
                                       (37, 64, 16, 16), (4096, 4104, 4000, 100)])
def test_colsum_fused(M, C, n0, n1, dtype):
    """dfcsa_colsum_fused (the Linear bias gradients in one launch, last workgroup per column block)
    against the column sums in float64, added into three destinations; bitwise repeatable."""
    call, P, dt, stream = lib()
    from dfcsa._lib import LIB
    torch.manual_seed(M + C)
    x = torch.randn(M, C, device="cuda").to(dtype)
    ref = x.double().sum(0)
    outs = []
    for _ in range(2):
        d = [torch.full((n,), 0.5, device="cuda") for n in (n0, n1, C - n0 - n1)]
        part = torch.empty(LIB.dfcsa_colsum_ntiles(M) * C, device="cuda")
        call("dfcsa_colsum_fused", dt(dtype), M, C, P(x), P(part), n0, n1, P(d[0]), P(d[1]) if n1 else None,
             P(d[2]) if C - n0 - n1 else None, stream())
        torch.cuda.synchronize()
        outs.append(torch.cat(d))
    assert (outs[0].double() - 0.5 - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())
    assert torch.equal(outs[0], outs[1])


# ----------------------------------------------------------------------------- off-config edges
def test_transunet_patch_size_2_raises_like_reference():
    """img = 2 x 16 x grid (patch size 2): the reference builds the model and its forward raises
    the position-embedding broadcast error (tests/golden/transunet_patch2_error.json, recorded from
    reference models/transformer_unet.py:179-181,196); ours raises the same type and message."""
    import json
    from models.transformer_unet import TransUNet
    from test_oracle_golden import transunet_small_config
    rec = json.load(open(os.path.join(GOLDEN, "transunet_patch2_error.json")))
    m = TransUNet(transunet_small_config(), img_size=rec["img"], num_classes=1, precision="fp32").cuda().train()
    assert list(m.transformer.embeddings.patch_embeddings.kernel_size) == rec["patch_kernel"]
    with pytest.raises(RuntimeError) as ei:
        m(torch.randn(1, 3, rec["img"], rec["img"], device="cuda"))
    assert type(ei.value).__name__ == rec["raised"]["type"] and str(ei.value) == rec["raised"]["message"]


@pytest.mark.parametrize("up", [2, 3])
def test_segmentation_head_upsampling_matches_reference(up):
    """SegmentationHead(upsampling > 1) standalone (reference :272-276): conv 3x3 + bias, then
    UpsamplingBilinear2d(up) (align_corners), forward and gradients against the reference's fp32
    CPU run (tests/golden/seghead_up.npz)."""
    from models.transformer_unet import SegmentationHead
    fx = np.load(os.path.join(GOLDEN, "seghead_up.npz"))
    k = f"up{up}_"
    head = SegmentationHead(16, 2, kernel_size=3, upsampling=up).cuda()
    with torch.no_grad():
        head[0].weight.copy_(T(fx[k + "conv_w"]))
        head[0].bias.copy_(T(fx[k + "conv_b"]))
    x = T(fx[k + "x"]).requires_grad_(True)
    out = head(x)
    assert tuple(out.shape) == fx[k + "out"].shape
    assert rel(out, fx[k + "out"]) < 1e-5
    (out * T(fx[k + "w"])).sum().backward()
    assert rel(x.grad, fx[k + "dx"]) < 1e-5
    assert rel(head[0].weight.grad, fx[k + "dconv_w"]) < 1e-5
    assert rel(head[0].bias.grad, fx[k + "dconv_b"]) < 1e-5


@pytest.mark.parametrize("H,W,s", [(7, 9, 2), (14, 14, 4), (5, 8, 3), (1, 6, 2)])
def test_upsample_ac_planes_vs_torch(H, W, s):
    """dfcsa_upsample_ac_f32(_bwd) against torch's UpsamplingBilinear2d (fp32, align_corners)."""
    x = torch.randn(3, 5, H, W, device="cuda", requires_grad=True)
    from dfcsa.transunet_ops import UpsampleAC
    y = UpsampleAC.apply(x, s)
    xr = x.detach().clone().requires_grad_(True)
    yr = torch.nn.UpsamplingBilinear2d(scale_factor=s)(xr)
    assert y.shape == yr.shape and rel(y, yr) < 1e-6
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    assert rel(x.grad, xr.grad) < 1e-6


@pytest.mark.parametrize("gelu", [False, True])
@pytest.mark.parametrize("M,C,p", [(1568, 768, 0.1), (1568, 3072, 0.1), (200, 64, 0.0), (77, 136, 0.3)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_drop_bwd_column_partials(M, C, p, gelu, dtype):
    """dfcsa_(gelu_)drop_bwd_cs: the same output as the flat dropout / GELU-dropout backward, and column
    partials (16-row tiles) whose fp64 total equals the column sums of that output."""
    call, P, dt, stream = lib()
    from dfcsa._lib import LIB
    torch.manual_seed(M + C)
    rng = torch.tensor([12345, 0], dtype=torch.int64, device="cuda")
    x = torch.randn(M, C, device="cuda").to(dtype)
    dout = torch.randn(M, C, device="cuda")
    if gelu:
        dout = dout.to(dtype)
    ref = torch.empty(M, C, device="cuda", dtype=dtype)
    got = torch.empty_like(ref)
    pgot = torch.empty(LIB.dfcsa_cs_ntiles(M) * C, device="cuda")
    if gelu:
        call("dfcsa_gelu_drop_bwd", dt(dtype), M * C, P(x), P(dout), float(p), P(rng), 7, P(ref), stream())
        call("dfcsa_gelu_drop_bwd_cs", dt(dtype), M, C, P(x), P(dout), float(p), P(rng), 7, P(got), P(pgot),
             pgot.numel(), stream())
    else:
        call("dfcsa_drop_bwd", dt(dtype), M * C, P(dout), float(p), P(rng), 7, P(ref), stream())
        call("dfcsa_drop_bwd_cs", dt(dtype), M, C, P(dout), float(p), P(rng), 7, P(got), P(pgot), pgot.numel(),
             stream())
    torch.cuda.synchronize()
    assert torch.equal(ref, got)
    tot = pgot.view(-1, C).double().sum(0)
    want = ref.double().sum(0)
    assert ((tot - want).abs().max() / want.abs().max().clamp_min(1e-30)).item() < 1e-5


@pytest.mark.parametrize("B,N,heads,dh", [(8, 196, 12, 64), (2, 50, 3, 16)])
def test_heads_unpack_column_partials(B, N, heads, dh):
    """dfcsa_heads_unpack_cs: the token-major unpack of dfcsa_heads_relayout (dq scaled), bitwise, and
    column partials (16-row tiles) whose fp64 total equals the column sums of that output."""
    call, P, dt, stream = lib()
    from dfcsa._lib import LIB
    torch.manual_seed(B * N)
    src = torch.randn(heads * B, N, 3 * dh, device="cuda").to(torch.bfloat16)
    M, ld = B * N, 3 * heads * dh
    ref = torch.empty(M, ld, device="cuda", dtype=torch.bfloat16)
    got = torch.empty_like(ref)
    pgot = torch.empty(LIB.dfcsa_cs_ntiles(M) * ld, device="cuda")
    scale = 1.0 / math.sqrt(dh)
    call("dfcsa_heads_relayout", 1, B, N, heads, dh, 3, float(scale), P(src), P(ref), stream())
    call("dfcsa_heads_unpack_cs", B, N, heads, dh, 3, float(scale), P(src), P(got), P(pgot), pgot.numel(), stream())
    torch.cuda.synchronize()
    assert torch.equal(ref, got)
    tot = pgot.view(-1, ld).double().sum(0)
    want = ref.double().sum(0)
    assert ((tot - want).abs().max() / want.abs().max().clamp_min(1e-30)).item() < 1e-5
