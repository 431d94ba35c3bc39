"""Small-M fp32 GEMMs (csrc/small_gemm.h): the LightSelfAttention q/k/v projections, their dgrad
and their weight gradient run on M = B*P*P pooled rows through split-reduction 16x64 tiles.
Checked against fp64 PyTorch on the CPU and against the generic tile kernels (tuning knobs 1=26
and 16 route the same calls to the generic paths)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

dfcsa_ops = pytest.importorskip("dfcsa.ops")
from dfcsa import ops  # noqa: E402
from dfcsa._lib import LIB  # noqa: E402

f32 = torch.float32


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def proj(x, w, b, dests):
    """x [M][K] fp32 -> dests (column split of the N = w.shape[0] outputs) via dfcsa_conv_gemm."""
    M, K = x.shape
    N = w.shape[0]
    Kp = ops.rup(K, ops.KALIGN)
    wp = torch.zeros(N, Kp, device="cuda", dtype=f32)
    wp[:, :K] = w
    Nd = N // len(dests)
    ops.conv_gemm(f32, [(x, 0, 0)], K, (1, M, 1), (M, 1), wp, Kp, N, dests, Nd, bias=b)


@pytest.mark.parametrize("M,K,N,ndest", [(256, 512, 640, 1), (32, 64, 80, 1), (1040, 1280, 1280, 1),
                                         (256, 640, 512, 1), (48, 96, 192, 3)])
def test_small_conv_f32_vs_fp64(M, K, N, ndest):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    dests = [torch.full((M, N // ndest), float("nan"), device="cuda") for _ in range(ndest)]
    proj(x, w, b, dests)
    ref = x.double().cpu() @ w.double().cpu().t() + b.double().cpu()
    out = torch.cat([d.cpu() for d in dests], 1)
    assert rel(out, ref) < 2e-6
    # the generic 64x64 tile path on the same call
    LIB.dfcsa_set_tuning(1, 26)
    try:
        dests2 = [torch.full((M, N // ndest), float("nan"), device="cuda") for _ in range(ndest)]
        proj(x, w, b, dests2)
    finally:
        LIB.dfcsa_set_tuning(1, 0)
    assert rel(out, torch.cat([d.cpu() for d in dests2], 1)) < 2e-6


@pytest.mark.parametrize("M,NI,NJ,Cq", [(256, 640, 512, 64), (32, 80, 64, 8), (1024, 1280, 1024, 128)])
def test_small_wgrad_f32_layout2_accumulates(M, NI, NJ, Cq):
    """dW = G^T X over M rows, stacked q/k/v rows added into three gradients (layout 2)."""
    torch.manual_seed(1)
    G = torch.randn(M, NI, device="cuda")
    X = torch.randn(M, NJ, device="cuda")
    C = NI - 2 * Cq
    base = [torch.randn(Cq, NJ, device="cuda"), torch.randn(Cq, NJ, device="cuda"), torch.randn(C, NJ, device="cuda")]
    grads = [t.clone() for t in base]
    ops.conv_wgrad_into(f32, [G], NI, [(X, 0, 0)], NJ, (1, M, 1), (M, 1), grads, 1, Cq, C, layout=2)
    ref = G.double().cpu().t() @ X.double().cpu()
    want = [base[0].double().cpu() + ref[:Cq], base[1].double().cpu() + ref[Cq:2 * Cq],
            base[2].double().cpu() + ref[2 * Cq:]]
    for g, r in zip(grads, want):
        assert rel(g, r) < 2e-6
    LIB.dfcsa_set_tuning(16, 1)
    try:
        grads2 = [t.clone() for t in base]
        ops.conv_wgrad_into(f32, [G], NI, [(X, 0, 0)], NJ, (1, M, 1), (M, 1), grads2, 1, Cq, C, layout=2)
    finally:
        LIB.dfcsa_set_tuning(16, 0)
    for g, g2 in zip(grads, grads2):
        assert rel(g, g2) < 2e-6


def test_small_wgrad_f32_layout0_1x1():
    """plain 1x1 conv weight gradient [Cout][Cin][1][1] (layout 0, one tap) over few pixels."""
    torch.manual_seed(2)
    M, Cout, Cin = 200, 96, 48
    G = torch.randn(M, Cout, device="cuda")
    X = torch.randn(M, Cin, device="cuda")
    gw = torch.zeros(Cout, Cin, 1, 1, device="cuda")
    ops.conv_wgrad_into(f32, [G], Cout, [(X, 0, 0)], Cin, (1, M, 1), (M, 1), [gw], 1, Cin, Cin)
    ref = (G.double().cpu().t() @ X.double().cpu()).view(Cout, Cin, 1, 1)
    assert rel(gw, ref) < 2e-6


def test_small_gemm_deterministic():
    torch.manual_seed(3)
    x = torch.randn(256, 512, device="cuda")
    w = torch.randn(640, 512, device="cuda")
    outs = []
    for _ in range(3):
        o = torch.empty(256, 640, device="cuda")
        proj(x, w, None, [o])
        outs.append(o)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
