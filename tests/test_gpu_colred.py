"""Fused column reduction + per-channel finalisation (csrc/block_ew.hip colred_block): the
BatchNorm statistics finalize, the BatchNorm-backward finalize (with the res_scale scalar) and the
bias column sums, each one launch over many row groups with a cross-workgroup hand-off.

Checked against float64 torch sums of the same fp32 partial rows, at row counts that give one
group, a few groups and the 64-group cap, with channel counts that leave a partial channel block;
every case runs repeatedly with the hand-off ring advancing between calls (so a stale read of an
older launch's hand-off would show up as a difference) and must be bitwise repeatable.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [(40, 64), (300, 64), (6272, 64), (20000, 100), (1568, 1024), (392, 2048)]


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.mark.parametrize("T,C", CASES, ids=[f"T{t}_C{c}" for t, c in CASES])
def test_bn_finalize_fused_reduction(T, C):
    from dfcsa._lib import call
    from dfcsa.ops import P, stream
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(T + C)
    ld = C + 8
    stats = torch.randn(T, 2, ld, device=dev, generator=g)
    stats[:, 1] = stats[:, 1].abs() * 4 + 2.0   # sum of squares dominates: positive variance
    count = T * 50
    s = stats[:, 0, :C].double().sum(0)
    q = stats[:, 1, :C].double().sum(0)
    mu_ref = s / count
    var_ref = (q / count - mu_ref * mu_ref).clamp_min(0)
    istd_ref = 1.0 / torch.sqrt(var_ref + 1e-5)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    outs = []
    for it in range(6):
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros(1, device=dev, dtype=torch.int64)
        sc, sh, mean, inv = (torch.empty(C, device=dev) for _ in range(4))
        call("dfcsa_bn_finalize", P(stats), T, C, ld, count, None, P(gamma), P(beta), P(rm), P(rv), P(nbt),
             0.1, 1e-5, 1, P(sc), P(sh), P(mean), P(inv), stream())
        # another launch in between: the next call's hand-off lands elsewhere in the ring
        call("dfcsa_bn_finalize", P(stats), T, C, ld, count, None, P(gamma), P(beta), P(rm), P(rv), P(nbt),
             0.1, 1e-5, 1, P(torch.empty(C, device=dev)), P(torch.empty(C, device=dev)),
             P(torch.empty(C, device=dev)), P(torch.empty(C, device=dev)), stream())
        torch.cuda.synchronize()
        assert int(nbt.item()) == 2
        outs.append(torch.stack([sc, sh, mean, inv]))
    assert rel(outs[0][2], mu_ref) < 1e-6
    assert rel(outs[0][3], istd_ref) < 1e-6
    assert rel(outs[0][0], gamma.double() * istd_ref) < 1e-6
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("nsum", [2, 3])
@pytest.mark.parametrize("T,C", CASES, ids=[f"T{t}_C{c}" for t, c in CASES])
def test_bn_bwd_finalize_fused_reduction(T, C, nsum):
    from dfcsa._lib import call
    from dfcsa.ops import P, stream
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(3 * T + C + nsum)
    part = torch.randn(T, nsum, C, device=dev, generator=g)
    sums = part.double().sum(0)
    count = T * 10
    outs = []
    for it in range(6):
        coef = torch.empty(3 * C, device=dev)
        dgamma, dbeta = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        extra = torch.full((1,), 0.5, device=dev) if nsum == 3 else None
        call("dfcsa_bn_bwd_finalize", P(part), T, nsum, C, count, P(coef), P(dgamma), P(dbeta), P(extra), stream())
        torch.cuda.synchronize()
        outs.append((coef[:2 * C].clone(), dgamma, dbeta, extra))
    coef, dgamma, dbeta, extra = outs[0]
    assert rel(coef[:C], sums[0] / count) < 1e-6 and rel(coef[C:2 * C], sums[1] / count) < 1e-6
    assert rel(dgamma, sums[1]) < 1e-6 and rel(dbeta, sums[0]) < 1e-6
    if nsum == 3:
        ref = 0.5 + sums[2].sum().item()
        assert abs(extra.item() - ref) <= 1e-5 * max(1.0, abs(ref)), (extra.item(), ref)
    for o in outs[1:]:
        for a, b in zip(o, outs[0]):
            if a is not None:
                assert torch.equal(a, b)


@pytest.mark.parametrize("T,C", CASES + [(3000, 5000)], ids=[f"T{t}_C{c}" for t, c in CASES + [(3000, 5000)]])
def test_slab_colsum3_fused_reduction(T, C):
    from dfcsa._lib import call
    from dfcsa.ops import P, stream
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(7 * T + C)
    slab = torch.randn(T, C, device=dev, generator=g)
    ref = slab.double().sum(0)
    n0, n1 = C // 4, C // 2
    res = []
    for it in range(4):
        d0, d1, d2 = (torch.zeros(n, device=dev) for n in (n0, n1, C - n0 - n1))
        call("dfcsa_slab_colsum3", P(slab), T, C, n0, n1, P(d0), P(d1), P(d2), stream())
        torch.cuda.synchronize()
        res.append(torch.cat([d0, d1, d2]))
    assert rel(res[0], ref) < 1e-6
    for r in res[1:]:
        assert torch.equal(r, res[0])
