"""The 2-D halo-tile 3x3 implicit GEMM (conv_halo_kernel, csrc/conv_gemm.hip) against a torch
reference of the same GEMM and against the row-tile kernels it replaces.

Covers the three tile shapes (16 x 16 when 16 | W and 16 | H -- the 224^2 / 112^2 levels --, 8 x 28
at 56^2, 14 x 14 at 28^2 / 14^2; tiles never straddle images, halo pixels outside the image are
zero), non-square images, a shape no tile fits (the row-tile kernel runs), the two-source forward
(the decoder's skip concat), the fused 3x3 + 1x1 data gradient (three sources, 11 segments),
bias / statistics / three destinations / accumulate / N tails, NaN guards around every output,
and the full-size layers of the benchmark against the row-tile kernel.
Reference: models/unet_dfc_sa_res.py:58-59 (3x3 conv), :182-200 (cat), the conv backward.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("dfcsa.ops")
import dfcsa  # noqa: E402
from dfcsa._lib import LIB  # noqa: E402

bf = torch.bfloat16
dev = "cuda"


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def ref_gemm(segs, Cseg, w, K):
    """C[m][n] = sum_s sum_c src_s[b, y+dh, x+dw, c] * w[n][s*Cseg + c], float64."""
    B, H, W, _ = segs[0][0].shape
    out = None
    for s, (x, dh, dw) in enumerate(segs):
        xp = F.pad(x.double(), (0, 0, 1, 1, 1, 1))           # [B, H+2, W+2, C]
        sh = xp[:, 1 + dh:1 + dh + H, 1 + dw:1 + dw + W, :].reshape(-1, Cseg)
        part = sh @ w[:, s * Cseg:(s + 1) * Cseg].double().t()
        out = part if out is None else out + part
    return out


def run(segs, Cseg, grid, w, Kp, N, dests, Nd, bias=None, stats=None, accumulate=False, halo=True):
    prev = LIB.dfcsa_get_tuning(19)
    LIB.dfcsa_set_tuning(19, 1 if halo else 0)   # 1: every M
    try:
        rows = ops.conv_gemm(bf, segs, Cseg, grid, grid[1:], w, Kp, N, dests, Nd, bias=bias, stats=stats,
                             accumulate=accumulate)
        torch.cuda.synchronize()
    finally:
        LIB.dfcsa_set_tuning(19, prev)
    return rows


def halo_tiles(B, H, W):
    """statistics rows of the halo kernel (one per tile), or None when no tile shape fits"""
    for tw, tr in ((16, 16), (8, 28), (14, 14)):
        if W % tw == 0 and H % tr == 0:
            return B * (H // tr) * (W // tw)
    return None


def guarded(shape, fill=float("nan")):
    n = 1
    for s in shape:
        n *= s
    buf = torch.full((n + 8192,), fill, dtype=bf, device=dev)
    return buf, buf[4096:4096 + n].view(*shape)


def intact(buf, n):
    return bool(torch.isnan(buf[:4096]).all()) and bool(torch.isnan(buf[4096 + n:]).all())


@pytest.mark.parametrize("B,H,W,Cs,nsrc,N", [
    (16, 14, 14, 64, 1, 128), (3, 28, 28, 64, 2, 64), (2, 56, 56, 128, 1, 256), (1, 112, 112, 64, 2, 128),
    (1, 20, 36, 64, 1, 64), (2, 12, 32, 128, 1, 192), (1, 224, 224, 64, 1, 64), (2, 32, 48, 64, 1, 64),
    (1, 28, 56, 64, 1, 192), (3, 14, 28, 128, 2, 64)])
def test_halo_forward_vs_torch(B, H, W, Cs, nsrc, N):
    torch.manual_seed(B * 1000 + H * 10 + W + N)
    xs = [torch.randn(B, H, W, Cs, device=dev).to(bf) for _ in range(nsrc)]
    segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
    K = len(segs) * Cs
    Kp = ops.rup(K, 64)
    w = (torch.randn(N, Kp, device=dev) * 0.05).to(bf)
    bias = torch.randn(N, device=dev)
    M = B * H * W
    ref = ref_gemm(segs, Cs, w, K)
    buf, y = guarded((B, H, W, N))
    st = torch.full((ops.ntiles_gemm(M) * 2 * N,), float("nan"), device=dev)
    rows = run(segs, Cs, (B, H, W), w, Kp, N, [y], N, bias=bias, stats=st)
    assert rows <= ops.ntiles_gemm(M)
    if halo_tiles(B, H, W) is not None:
        assert rows == halo_tiles(B, H, W), "the halo kernel did not run"
    assert intact(buf, y.numel()) and not torch.isnan(y).any()
    assert rel(y.reshape(M, N), ref + bias.double()) < 5e-3
    s = st[:rows * 2 * N].view(rows, 2, N).double().sum(0)
    assert not torch.isnan(s).any()
    assert rel(s[0], ref.sum(0)) < 1e-4 and rel(s[1], (ref * ref).sum(0)) < 1e-4
    # the same GEMM on the row-tile kernel
    y0 = torch.empty_like(y)
    run(segs, Cs, (B, H, W), w, Kp, N, [y0], N, bias=bias, halo=False)
    assert rel(y, y0) < 4e-3


@pytest.mark.parametrize("B,H,W,C,Cin,nd", [(2, 28, 28, 64, 128, 2), (1, 56, 56, 128, 64, 1),
                                            (9, 14, 14, 128, 256, 2), (1, 112, 112, 64, 128, 2),
                                            (2, 32, 16, 64, 192, 3)])
def test_halo_fused_dgrad_vs_torch(B, H, W, C, Cin, nd):
    """The block input gradient: 9 taps of dy1 (shifts 1-kh, 1-kw) + dy2 + dres (1x1) in one GEMM,
    the N = Cin columns split over nd source gradients."""
    torch.manual_seed(C + Cin + H)
    dy1, dy2, dres = (torch.randn(B, H, W, C, device=dev).to(bf) for _ in range(3))
    segs = [(dy1, 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(dy2, 0, 0), (dres, 0, 0)]
    K = 11 * C
    Kp = ops.rup(K, 64)
    w = (torch.randn(Cin, Kp, device=dev) * 0.05).to(bf)
    ref = ref_gemm(segs, C, w, K)
    Cs = Cin // nd
    outs = [guarded((B, H, W, Cs)) for _ in range(nd)]
    run(segs, C, (B, H, W), w, Kp, Cin, [o for _, o in outs], Cs)
    got = torch.cat([o.reshape(-1, Cs) for _, o in outs], 1)
    for b, o in outs:
        assert intact(b, o.numel())
    assert rel(got, ref) < 5e-3


def test_halo_accumulate_three_dests():
    torch.manual_seed(5)
    B, H, W, Cs, N = 2, 32, 32, 64, 192
    x = torch.randn(B, H, W, Cs, device=dev).to(bf)
    segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3)]
    Kp = ops.rup(9 * Cs, 64)
    w = (torch.randn(N, Kp, device=dev) * 0.05).to(bf)
    base = [torch.randn(B, H, W, 64, device=dev).to(bf) for _ in range(3)]
    dests = [b.clone() for b in base]
    run(segs, Cs, (B, H, W), w, Kp, N, dests, 64, accumulate=True)
    ref = ref_gemm(segs, Cs, w, 9 * Cs)
    for i in range(3):
        assert rel(dests[i].reshape(-1, 64), ref[:, 64 * i:64 * (i + 1)] + base[i].reshape(-1, 64).double()) < 5e-3


@pytest.mark.parametrize("name,H,Cs,nsrc,N,dgrad", [
    ("L1 fwd up_conv1", 224, 64, 2, 64, False), ("L1 dgrad up_conv1", 224, 64, 1, 128, True),
    ("L2 fwd up_conv2", 112, 128, 2, 128, False), ("L2 fwd down2", 112, 64, 1, 128, False),
    ("L2 dgrad up_conv2", 112, 128, 1, 256, True), ("L3 fwd up_conv3", 56, 256, 2, 256, False),
    ("L3 dgrad up_conv3", 56, 256, 1, 512, True), ("L4 fwd up_conv4", 28, 512, 2, 512, False)])
def test_halo_bench_layers_vs_row_tile_kernel(name, H, Cs, nsrc, N, dgrad):
    """The benchmark's 3x3 layers (B = 16) on the halo kernel against the row-tile kernels: the same
    GEMM in a different accumulation order, bf16 outputs within rounding."""
    torch.manual_seed(H + N)
    B = 16
    if dgrad:
        src = [torch.randn(B, H, H, Cs, device=dev).to(bf) for _ in range(3)]
        segs = [(src[0], 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(src[1], 0, 0), (src[2], 0, 0)]
    else:
        xs = [torch.randn(B, H, H, Cs, device=dev).to(bf) for _ in range(nsrc)]
        segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
    Kp = ops.rup(len(segs) * Cs, 64)
    w = (torch.randn(N, Kp, device=dev) * 0.03).to(bf)
    ya = torch.empty(B, H, H, N, device=dev, dtype=bf)
    yb = torch.empty_like(ya)
    run(segs, Cs, (B, H, H), w, Kp, N, [ya], N, halo=True)
    run(segs, Cs, (B, H, H), w, Kp, N, [yb], N, halo=False)
    assert rel(ya, yb) < 4e-3, name


# ------------------------------------------------------------------ weight gradient (knob 20)
def wgrad_run(dy, xs, gw, Cin_real, halo):
    B, H, W, C = dy.shape
    Cs = xs[0].shape[-1]
    segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
    prev = LIB.dfcsa_get_tuning(20)
    LIB.dfcsa_set_tuning(20, 1 if halo else 0)
    try:
        ops.conv_wgrad_into(bf, [dy], C, segs, Cs, (B, H, W), (H, W), [gw], 9, len(xs) * Cs, Cin_real)
        torch.cuda.synchronize()
    finally:
        LIB.dfcsa_set_tuning(20, prev)


@pytest.mark.parametrize("B,H,W,Cs,nsrc,C", [
    (2, 128, 128, 64, 1, 64), (1, 224, 224, 64, 2, 64), (4, 112, 112, 128, 1, 128), (16, 56, 56, 64, 2, 256),
    (48, 28, 28, 64, 1, 128), (170, 14, 14, 64, 1, 192), (3, 96, 120, 64, 1, 64)])
def test_halo_wgrad_vs_torch(B, H, W, Cs, nsrc, C):
    """3x3 weight gradient on halo tiles (M >= 32768): against torch's conv2d weight gradient in
    float64 (bf16-exact operands) and against the row-tile kernel; the gradient is ADDED into the
    existing buffer (accumulate semantics of p.grad)."""
    torch.manual_seed(H * 7 + C + nsrc)
    xs = [torch.randn(B, H, W, Cs, device=dev).to(bf) for _ in range(nsrc)]
    dy = torch.randn(B, H, W, C, device=dev).to(bf)
    Cin = nsrc * Cs
    if B * H * W < 32768:
        pytest.skip("below the halo kernel's M threshold")
    xc = torch.cat([x.double() for x in xs], -1).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xc, (C, Cin, 3, 3), dy.double().permute(0, 3, 1, 2), padding=1)
    base = torch.randn(C, Cin, 3, 3, device=dev)
    ga = base.clone()
    wgrad_run(dy, xs, ga, Cin, True)
    assert rel(ga - base, ref) < 1e-5
    gb = base.clone()
    wgrad_run(dy, xs, gb, Cin, False)
    assert rel(ga - base, gb - base) < 1e-5
