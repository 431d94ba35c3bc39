"""The round-2 fused block kernels against a plain torch reference (float64 on the GPU, operands
bf16-exact), slab-capacity enforcement, and out-of-bounds canaries.

Round 2 checked these kernels only against the separate HIP launches they replace; here every one
is compared with the reference arithmetic of the block it implements
(models/unet_dfc_sa_res.py:97-114 forward, its autograd backward) at ragged M (not a multiple of the
64-row tile, with several tiles per workgroup) and C in {64, 128, 256} where the kernel serves it:
  dfcsa_dgrad_gate, dfcsa_dgrad_acc_relu_bn, dfcsa_dgrad_gate_apply, dfcsa_dgrad_acc_relu_bn_apply,
  dfcsa_gate_fusion_fwd, dfcsa_local_attn_gate_fwd.
Every output and every per-workgroup partial slab sits between NaN guard regions; after the call
the guards must be untouched and every slab row written.  A slab one float short of the launch
grid must be refused (DFCSA_EINVAL) without a launch: the round-2 HIP error 700 was exactly such a
slab (a partial buffer sized for the fused kernel's grid reused by dfcsa_bwd_relu_bn, whose grid is
larger).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("dfcsa.ops")
from dfcsa._lib import LIB, DfcsaError, call  # noqa: E402
from dfcsa.ops import P, S, stream  # noqa: E402

bf = torch.bfloat16
dev = "cuda"
GUARD = 4096


class Guarded:
    """A [n] tensor (viewed as `shape`) between two NaN guard regions of GUARD elements."""

    def __init__(self, shape, dtype, init=None):
        n = 1
        for s in shape:
            n *= s
        self.n = n
        self.buf = torch.full((n + 2 * GUARD,), float("nan"), dtype=dtype, device=dev)
        self.t = self.buf[GUARD:GUARD + n].view(*shape)
        if init is not None:
            self.t.copy_(init)

    def intact(self):
        return bool(torch.isnan(self.buf[:GUARD]).all()) and bool(torch.isnan(self.buf[GUARD + self.n:]).all())

    def written(self):
        return not bool(torch.isnan(self.t).any())


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(bf)


def r16(x):
    """round to bf16 and back (what the kernels store)"""
    return x.to(bf).double()


def short_by_one(t):
    return (P(t), t.numel() - 1)


def gate_ref(G, C, y3, loc, att, sc, sh, mu, istd):
    """Gate backward (reference :102-106 autograd) on the bf16-rounded fusion-conv input gradient."""
    df, dl, da = (r16(G[:, i * C:(i + 1) * C]) for i in range(3))
    g = torch.sigmoid(y3.double() * sc.double() + sh.double())
    dz = df * (loc.double() - att.double()) * g * (1 - g)
    xh = (y3.double() - mu.double()) * istd.double()
    return dl + df * g, da + df * (1 - g), dz, dz.sum(0), (dz * xh).sum(0)


def acc_ref(G, C, dl_in, da_in, y1, sc, sh, mu, istd):
    """Gate-conv input gradient added into [dlocal | dattn], then the BN1 relu-backward sums."""
    gl = r16(r16(G[:, :C]) + dl_in.double())
    ga = r16(G[:, C:]) + da_in.double()
    z = torch.where(y1.double() * sc.double() + sh.double() > 0, gl, torch.zeros_like(gl))
    xh = (y1.double() - mu.double()) * istd.double()
    return gl, ga, z.sum(0), (z * xh).sum(0)


def check_sums(part, npart, C, s0, s1, tol=2e-3):
    p = part.view(npart, 2, C).double().sum(0)
    assert rel(p[0], s0) < tol and rel(p[1], s1) < tol, (rel(p[0], s0), rel(p[1], s1))


MS = [64 * 97 + 13, 65536 * 3 + 37]


@pytest.mark.parametrize("C", [64, 128, 256])
@pytest.mark.parametrize("M", MS)
def test_dgrad_gate_vs_torch(M, C):
    torch.manual_seed(100 + C)
    Kp = ops.rup(C, ops.KALIGN)
    dy4 = rnd(M, C)
    w4t = rnd(3 * C, Kp, scale=0.1)
    y3, loc, att = rnd(M, C), rnd(M, C), rnd(M, C)
    sc, sh, mu = (torch.randn(C, device=dev) for _ in range(3))
    istd = torch.rand(C, device=dev) + 0.5
    outs = [Guarded((M, C), bf) for _ in range(3)]
    npart = LIB.dfcsa_dgrad_gate_parts(M, C)
    part = Guarded((npart * 2 * C,), torch.float32)
    call("dfcsa_dgrad_gate", M, C, P(dy4), P(w4t), Kp, P(y3), P(sc), P(sh), P(mu), P(istd), P(loc), P(att),
         P(outs[0].t), P(outs[1].t), P(outs[2].t), *S(part.t), stream())
    torch.cuda.synchronize()
    G = dy4.double() @ w4t[:, :C].double().t()
    dl, da, dz, s0, s1 = gate_ref(G, C, y3, loc, att, sc, sh, mu, istd)
    for o, r in zip(outs, (dl, da, dz)):
        assert o.intact() and o.written()
        assert rel(o.t, r) < 4e-3, rel(o.t, r)
    assert part.intact() and part.written()
    check_sums(part.t, npart, C, s0, s1)
    with pytest.raises(DfcsaError, match="invalid"):
        call("dfcsa_dgrad_gate", M, C, P(dy4), P(w4t), Kp, P(y3), P(sc), P(sh), P(mu), P(istd), P(loc), P(att),
             P(outs[0].t), P(outs[1].t), P(outs[2].t), *short_by_one(part.t), stream())


@pytest.mark.parametrize("C", [64, 128, 256])
@pytest.mark.parametrize("M", MS)
def test_dgrad_acc_relu_bn_vs_torch(M, C):
    torch.manual_seed(200 + C)
    Kp = ops.rup(C, ops.KALIGN)
    dy3 = rnd(M, C)
    w3t = rnd(2 * C, Kp, scale=0.1)
    y1, dl_in, da_in = rnd(M, C), rnd(M, C), rnd(M, C)
    sc, sh, mu = (torch.randn(C, device=dev) for _ in range(3))
    istd = torch.rand(C, device=dev) + 0.5
    dl, da = Guarded((M, C), bf, dl_in), Guarded((M, C), bf, da_in)
    npart = LIB.dfcsa_dgrad_acc_relu_bn_parts(M, C)
    part = Guarded((npart * 2 * C,), torch.float32)
    call("dfcsa_dgrad_acc_relu_bn", M, C, P(dy3), P(w3t), Kp, P(y1), P(sc), P(sh), P(mu), P(istd), P(dl.t),
         P(da.t), *S(part.t), stream())
    torch.cuda.synchronize()
    G = dy3.double() @ w3t[:, :C].double().t()
    gl, ga, s0, s1 = acc_ref(G, C, dl_in, da_in, y1, sc, sh, mu, istd)
    for o, r in ((dl, gl), (da, ga)):
        assert o.intact() and o.written()
        assert rel(o.t, r) < 4e-3
    assert part.intact() and part.written()
    check_sums(part.t, npart, C, s0, s1)
    with pytest.raises(DfcsaError, match="invalid"):
        call("dfcsa_dgrad_acc_relu_bn", M, C, P(dy3), P(w3t), Kp, P(y1), P(sc), P(sh), P(mu), P(istd), P(dl.t),
             P(da.t), *short_by_one(part.t), stream())


def apply_ref(src, y, gamma, k, mu, istd, C, sc=None, sh=None):
    """BatchNorm-backward apply dy = gamma*invstd*(dz - coef0 - xh*coef1) (dz relu-masked)."""
    dz = src.double()
    if sc is not None:
        dz = torch.where(y.double() * sc.double() + sh.double() > 0, dz, torch.zeros_like(dz))
    xh = (y.double() - mu.double()) * istd.double()
    return gamma.double() * istd.double() * (dz - k[:C].double() - xh * k[C:2 * C].double())


@pytest.mark.parametrize("M", MS)
def test_dgrad_apply_prologues_vs_torch(M):
    torch.manual_seed(300)
    C = Kp = 64
    src, y, y3, loc, att, y1 = (rnd(M, C) for _ in range(6))
    gamma, mu, sc, sh, mu3, sc3, sh3 = (torch.randn(C, device=dev) for _ in range(7))
    k = torch.randn(3 * C, device=dev) * 0.1
    istd, istd3 = torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) + 0.5
    w4t, w3t = rnd(3 * C, Kp, scale=0.1), rnd(2 * C, Kp, scale=0.1)
    # gate: dy4 = apply_relu(dout) in the prologue, the gate backward in the epilogue
    dy4 = Guarded((M, C), bf)
    outs = [Guarded((M, C), bf) for _ in range(3)]
    n0 = LIB.dfcsa_dgrad_apply_parts(M, 0)
    p0 = Guarded((n0 * 2 * C,), torch.float32)
    args = [M, P(src), P(y), P(gamma), P(k), P(mu), P(istd), P(sc), P(sh), P(dy4.t), P(w4t), P(y3), P(sc3), P(sh3),
            P(mu3), P(istd3), P(loc), P(att), P(outs[0].t), P(outs[1].t), P(outs[2].t)]
    call("dfcsa_dgrad_gate_apply", *args, *S(p0.t), stream())
    # acc: dy3 = apply(dz3) in the prologue, accumulate + BN1 sums in the epilogue
    dy3 = Guarded((M, C), bf)
    dl, da = Guarded((M, C), bf, loc), Guarded((M, C), bf, att)
    n1 = LIB.dfcsa_dgrad_apply_parts(M, 1)
    p1 = Guarded((n1 * 2 * C,), torch.float32)
    args1 = [M, P(src), P(y), P(gamma), P(k), P(mu), P(istd), P(dy3.t), P(w3t), P(y1), P(sc3), P(sh3), P(mu3),
             P(istd3), P(dl.t), P(da.t)]
    call("dfcsa_dgrad_acc_relu_bn_apply", *args1, *S(p1.t), stream())
    torch.cuda.synchronize()
    r4 = apply_ref(src, y, gamma, k, mu, istd, C, sc, sh)
    assert dy4.intact() and dy4.written() and rel(dy4.t, r4) < 4e-3
    G = r16(r4) @ w4t[:, :C].double().t()
    rl, ra, rz, s0, s1 = gate_ref(G, C, y3, loc, att, sc3, sh3, mu3, istd3)
    for o, r in zip(outs, (rl, ra, rz)):
        assert o.intact() and o.written() and rel(o.t, r) < 6e-3
    assert p0.intact() and p0.written()
    check_sums(p0.t, n0, C, s0, s1, 4e-3)
    r3 = apply_ref(src, y, gamma, k, mu, istd, C)
    assert dy3.intact() and dy3.written() and rel(dy3.t, r3) < 4e-3
    G = r16(r3) @ w3t[:, :C].double().t()
    gl, ga, s0, s1 = acc_ref(G, C, loc, att, y1, sc3, sh3, mu3, istd3)
    for o, r in ((dl, gl), (da, ga)):
        assert o.intact() and o.written() and rel(o.t, r) < 6e-3
    assert p1.intact() and p1.written()
    check_sums(p1.t, n1, C, s0, s1, 4e-3)
    with pytest.raises(DfcsaError, match="invalid"):
        call("dfcsa_dgrad_gate_apply", *args, *short_by_one(p0.t), stream())
    with pytest.raises(DfcsaError, match="invalid"):
        call("dfcsa_dgrad_acc_relu_bn_apply", *args1, *short_by_one(p1.t), stream())


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("M", MS)
def test_gate_fusion_fwd_vs_torch(M, C):
    torch.manual_seed(400 + C)
    Kp = 3 * C
    y3, loc, att = rnd(M, C), rnd(M, C), rnd(M, C)
    sc, sh = torch.randn(C, device=dev), torch.randn(C, device=dev)
    w4 = rnd(C, Kp, scale=0.1)
    b4 = torch.randn(C, device=dev)
    fused, y4 = Guarded((M, C), bf), Guarded((M, C), bf)
    npart = LIB.dfcsa_fwd_pro_parts(M, C, 0)
    st = Guarded((npart * 2 * C,), torch.float32)
    args = [M, C, P(y3), P(sc), P(sh), P(loc), P(att), P(w4), Kp, P(b4), P(fused.t), P(y4.t)]
    call("dfcsa_gate_fusion_fwd", *args, *S(st.t), stream())
    torch.cuda.synchronize()
    g = torch.sigmoid(y3.double() * sc.double() + sh.double())
    rf = g * loc.double() + (1 - g) * att.double()
    acc = torch.cat([r16(rf), loc.double(), att.double()], 1) @ w4.double().t()
    assert fused.intact() and fused.written() and rel(fused.t, rf) < 4e-3
    assert y4.intact() and y4.written() and rel(y4.t, acc + b4.double()) < 4e-3
    assert st.intact() and st.written()
    check_sums(st.t, npart, C, acc.sum(0), (acc * acc).sum(0), 1e-3)
    with pytest.raises(DfcsaError, match="invalid"):
        call("dfcsa_gate_fusion_fwd", *args, *short_by_one(st.t), stream())


@pytest.mark.parametrize("B,H,W,Pp,C", [(3, 37, 29, 4, 64), (4, 112, 112, 4, 64), (2, 14, 9, 8, 64),
                                        (3, 37, 29, 4, 128), (4, 56, 56, 4, 128), (2, 14, 9, 8, 128)])
def test_local_attn_gate_fwd_vs_torch(B, H, W, Pp, C):
    torch.manual_seed(500 + H + C)
    Kp = 2 * C
    M = B * H * W
    y1, y2 = rnd(M, C), rnd(M, C)
    sc1, sh1, sc2, sh2 = (torch.randn(C, device=dev) for _ in range(4))
    o = torch.randn(B, Pp, Pp, C, device=dev)
    gamma = torch.tensor([0.37], device=dev)
    w3 = rnd(C, Kp, scale=0.1)
    b3 = torch.randn(C, device=dev)
    local, attn, y3 = Guarded((M, C), bf), Guarded((M, C), bf), Guarded((M, C), bf)
    npart = LIB.dfcsa_fwd_pro_parts(M, C, 1)
    st = Guarded((npart * 2 * C,), torch.float32)
    args = [B, H, W, C, P(y1), P(sc1), P(sh1), P(y2), P(sc2), P(sh2), P(o), Pp, P(gamma), P(w3), Kp, P(b3),
            P(local.t), P(attn.t), P(y3.t)]
    call("dfcsa_local_attn_gate_fwd", *args, *S(st.t), stream())
    torch.cuda.synchronize()
    rl = torch.relu(y1.double() * sc1.double() + sh1.double())
    up = F.interpolate(o.double().permute(0, 3, 1, 2), size=(H, W), mode="bilinear", align_corners=False)
    ra = 0.37 * up.permute(0, 2, 3, 1).reshape(M, C) + torch.relu(y2.double() * sc2.double() + sh2.double())
    acc = torch.cat([r16(rl), r16(ra)], 1) @ w3.double().t()
    assert local.intact() and local.written() and rel(local.t, rl) < 4e-3
    assert attn.intact() and attn.written() and rel(attn.t, ra) < 4e-3
    assert y3.intact() and y3.written() and rel(y3.t, acc + b3.double()) < 4e-3
    assert st.intact() and st.written()
    check_sums(st.t, npart, C, acc.sum(0), (acc * acc).sum(0), 1e-3)
    with pytest.raises(DfcsaError, match="invalid"):
        call("dfcsa_local_attn_gate_fwd", *args, *short_by_one(st.t), stream())


# ------------------------------------------------------------------ elementwise reduction passes
def test_ew_reduction_slabs_guarded_and_capacity_checked():
    """The elementwise backward passes that write [ntiles][nsum][C] partial slabs: every slab row
    written, guards intact, a slab one float short refused."""
    torch.manual_seed(600)
    T = ops.dt(bf)
    B, H, W, C, Pp = 3, 38, 26, 64, 4
    M = B * H * W
    nte = ops.ntiles_ew(M, C)
    a, y, r3, loc, att = (rnd(M, C) for _ in range(5))
    sc, sh, mu = (torch.randn(C, device=dev) for _ in range(3))
    istd = torch.rand(C, device=dev) + 0.5
    rs = torch.tensor([0.3], device=dev)
    dpool = torch.randn(B, Pp, Pp, C, device=dev)
    cases = [
        ("dfcsa_bwd_relu_bn", 2, lambda o: [T, M, C, P(a), P(y), P(sc), P(sh), P(mu), P(istd), P(o[0])]),
        ("dfcsa_bwd_gate", 2, lambda o: [T, M, C, P(a), P(y), P(sc), P(sh), P(mu), P(istd), P(loc), P(att), P(o[0]),
                                         P(o[1]), P(o[2])]),
        ("dfcsa_bwd_block_out", 3, lambda o: [T, M, C, P(a), P(y), P(sc), P(sh), P(mu), P(istd), P(r3), P(rs),
                                              P(o[0]), P(o[1])]),
        ("dfcsa_bwd_attn_entry", 2, lambda o: [T, B, H, W, C, P(a), P(dpool), Pp, P(y), P(sc), P(sh), P(mu), P(istd),
                                               1, P(o[0])]),
    ]
    for name, ns, mk in cases:
        outs = [Guarded((M, C), bf, torch.zeros(M, C, dtype=bf, device=dev)) for _ in range(3)]
        part = Guarded((nte * ns * C,), torch.float32)
        call(name, *mk([o.t for o in outs]), *S(part.t), stream())
        torch.cuda.synchronize()
        assert part.intact() and part.written(), name
        assert all(o.intact() and o.written() for o in outs), name
        with pytest.raises(DfcsaError, match="invalid"):
            call(name, *mk([o.t for o in outs]), *short_by_one(part.t), stream())
    # the pooled block-output backward (its own tile size)
    ntp = LIB.dfcsa_bwd_block_out_pool_ntiles(B, H, W, C)
    out = rnd(M, C)
    dpo = rnd(B * (H // 2) * (W // 2), C)
    dout, dres = Guarded((M, C), bf), Guarded((M, C), bf)
    part = Guarded((ntp * 3 * C,), torch.float32)
    args = [T, B, H, W, C, None, P(out), P(dpo), P(y), P(sc), P(sh), P(mu), P(istd), P(r3), P(rs), P(dout.t),
            P(dres.t)]
    call("dfcsa_bwd_block_out_pool", *args, *S(part.t), stream())
    torch.cuda.synchronize()
    assert part.intact() and part.written() and dout.intact() and dres.intact()
    with pytest.raises(DfcsaError, match="invalid"):
        call("dfcsa_bwd_block_out_pool", *args, *short_by_one(part.t), stream())


def test_conv_gemm_stats_capacity():
    """dfcsa_conv_gemm writes one statistics row per M tile of the kernel it picks (the count it
    returns, at most ceil(M/64)) and refuses a slab shorter than that many rows * 2 * N floats."""
    M, C = 64 * 5 + 3, 64
    x = rnd(1, M, 1, C)
    w = rnd(C, 64, scale=0.1)
    y = torch.empty(1, M, 1, C, dtype=bf, device=dev)
    st = Guarded((ops.ntiles_gemm(M) * 2 * C,), torch.float32)
    rows = ops.conv_gemm(bf, [(x, 0, 0)], C, (1, M, 1), (M, 1), w, 64, C, [y], C, stats=st.t)
    torch.cuda.synchronize()
    assert 1 <= rows <= ops.ntiles_gemm(M)
    assert st.intact() and not torch.isnan(st.t[:rows * 2 * C]).any()
    with pytest.raises(DfcsaError, match="invalid"):
        ops.conv_gemm(bf, [(x, 0, 0)], C, (1, M, 1), (M, 1), w, 64, C, [y], C, stats=st.t[:rows * 2 * C - 1])
