"""Diagnostic for the round-5 opt-in batched-GEMM pooled attention (DFCSA_LSA_GEMM_MIN_N): at P = 16,
B = 2 (fp32 model step, tools/pool_path_diag2.py's setup), every lsa_core_forward / lsa_core_backward
call of the model runs BOTH the per-row kernels and the GEMM path on the same inputs, compares their
outputs (A, o; dpooled and the q/k/v/gamma gradient contributions), and continues with the one USE
names (row | bmm).  SYNC=1 synchronises the device around each call (separates a stream-ordering
cause from an arithmetic one).  Prints the worst per-tensor model gradient errors against the
float64 oracle at the end."""
import os
import sys

import torch

sys.path[:0] = ["dfc-sa-unet_amd", ".", "tests"]
import dfcsa.block as blk  # noqa: E402
from dfcsa.loss import sigmoid  # noqa: E402
from models.unet_dfc_sa_res import UNetDFCSARes  # noqa: E402
from oracle import dfcsa_oracle as O  # noqa: E402
from test_gpu_fra_unet import LP, T, rel  # noqa: E402
from utils.metrics import calculate_metrics  # noqa: E402

USE = os.environ.get("USE", "row")
USE_F = os.environ.get("USE_F", USE)   # the forward's saved state the model keeps (row | bmm)
USE_B = os.environ.get("USE_B", USE)   # the backward whose outputs the model continues with
FLASH = os.environ.get("FLASH", "0") == "1"   # no wrapping: the shipped flash kernels for P >= 9
SYNC = os.environ.get("SYNC", "0") == "1"
BIG = 1 << 30
orig_f, orig_b = blk.lsa_core_forward, blk.lsa_core_backward


def sync():
    if SYNC:
        torch.cuda.synchronize()


def wf(lsa, y, scale, shift, relu, pool_size, dtype, pk, window_sums=False):
    sync()
    blk.LSA_GEMM_MIN_N = 64
    sb = orig_f(lsa, y, scale, shift, relu, pool_size, dtype, pk, window_sums)
    blk.LSA_GEMM_MIN_N = BIG
    sr = orig_f(lsa, y, scale, shift, relu, pool_size, dtype, pk, window_sums)
    sync()
    torch.cuda.synchronize()
    C = y.shape[-1]
    ws = f" wsum {rel(sb[5], sr[5]):.2e}" if len(sb) > 5 and sb[5] is not None else ""
    print(f"fwd C={C}: pooled {rel(sb[0], sr[0]):.2e} qkv {rel(sb[1], sr[1]):.2e} A {rel(sb[2], sr[2]):.2e} "
          f"o {rel(sb[3], sr[3]):.2e}{ws}", flush=True)
    if os.environ.get("STRIDES"):
        print("   strides bmm", [tuple(t.stride()) if torch.is_tensor(t) else None for t in sb],
              "row", [tuple(t.stride()) if torch.is_tensor(t) else None for t in sr], flush=True)
    if os.environ.get("COPY") == "1":      # the GEMM path's saved tensors, holding the per-row values
        for a, b in zip(sb, sr):
            if torch.is_tensor(a):
                a.copy_(b)
    if os.environ.get("COPY") == "2":      # the per-row path's saved tensors, holding the GEMM values
        for a, b in zip(sr, sb):
            if torch.is_tensor(a):
                a.copy_(b)
        return sr
    return sb if USE_F == "bmm" else sr


def wb(lsa, saved, dattn, pool_size, dtype, pk, pool_rows=None):
    ps = [lsa.gamma, lsa.query_conv.weight, lsa.query_conv.bias, lsa.key_conv.weight, lsa.key_conv.bias,
          lsa.value_conv.weight, lsa.value_conv.bias]
    sync()
    before = [blk.grad_of(p).clone() for p in ps]
    blk.LSA_GEMM_MIN_N = 64
    db = orig_b(lsa, saved, dattn, pool_size, dtype, pk, pool_rows)
    torch.cuda.synchronize()
    gb = [blk.grad_of(p) - b for p, b in zip(ps, before)]
    for p, b in zip(ps, before):
        p.grad.copy_(b)
    blk.LSA_GEMM_MIN_N = BIG
    dr = orig_b(lsa, saved, dattn, pool_size, dtype, pk, pool_rows)
    torch.cuda.synchronize()
    gr = [blk.grad_of(p) - b for p, b in zip(ps, before)]
    print(f"bwd C={dattn.shape[-1]}: dpooled {rel(db, dr):.2e} grads "
          + " ".join(f"{rel(a, b):.1e}" for a, b in zip(gb, gr)), flush=True)
    if USE_B == "bmm":
        for p, b, g in zip(ps, before, gb):
            p.grad.copy_(b + g)
        return db
    return dr


if os.environ.get("POISON") == "1":
    # every torch.empty / empty_like buffer starts as NaN (ints: -1): a kernel that reads memory it
    # did not write first then shows up as NaN gradients
    _empty, _empty_like = torch.empty, torch.empty_like

    def _fill(t):
        if t.is_floating_point():
            t.fill_(float("nan"))
        elif t.dtype != torch.bool:
            t.fill_(-1)
        return t

    torch.empty = lambda *a, **k: _fill(_empty(*a, **k))
    torch.empty_like = lambda *a, **k: _fill(_empty_like(*a, **k))
if not FLASH:
    blk.lsa_core_forward, blk.lsa_core_backward = wf, wb
    blk.LSA_FLASH_MIN_N[0] = BIG   # compare the per-row kernels with the GEMM path
else:
    blk.LSA_FLASH_MIN_N[0] = int(os.environ.get("FLASH_MIN_N", "64"))

POOL_OUTS = []
if os.environ.get("TIES"):
    # record every encoder block output (the max-pool's argmax source) for the argmax comparison
    import models.unet_dfc_sa_res as _mr
    _orig_pool_fn = _mr.DFCBlockPoolFunction

    class _Rec:
        @staticmethod
        def apply(*a):
            r = _orig_pool_fn.apply(*a)
            POOL_OUTS.append(r[1].detach().float().cpu())
            return r

    _mr.DFCBlockPoolFunction = _Rec
P, B = int(os.environ.get("P", 16)), int(os.environ.get("B", 2))
torch.manual_seed(4300 + 16)
m0 = UNetDFCSARes(3, 1, [16, 32, 48, 64], pool_size=P, precision="fp32")
with torch.no_grad():
    for i, (n, p) in enumerate(sorted(m0.named_parameters())):
        if n.endswith("gamma"):
            p.fill_(0.2 + 0.05 * (i % 9))
sd = {k: v.detach().clone() for k, v in m0.state_dict().items()}
gen = torch.Generator().manual_seed(4400 + 16)
x = torch.randn(B, 3, 64, 64, generator=gen)
t = (torch.rand(B, 1, 64, 64, generator=gen) > 0.5).float()
sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
_, _, g64, _ = O.forward_backward(sd64, x.double(), t.double(), P, LP)
_, _, g32, _ = O.forward_backward(sd, x, t, P, LP)
m = UNetDFCSARes(3, 1, [16, 32, 48, 64], pool_size=P, precision="fp32")
m.load_state_dict(sd)
m = m.cuda().train()
logits = m(T(x.numpy()))
met = calculate_metrics(sigmoid(logits), T(t.numpy()), "bce_dice", LP)
met["loss"].backward()
torch.cuda.synchronize()
g = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}
bad = [n for n in g if not torch.isfinite(g[n]).all()]
print(f"non-finite gradients: {len(bad)} {bad[:6]}; logits finite: {bool(torch.isfinite(logits).all())}", flush=True)
rows = sorted(((rel(g[n], g64[n]), n) for n in g
               if not n.endswith(("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias", "fusion_conv.0.bias",
                                  "key_conv.bias"))), reverse=True)
print(f"USE_F={USE_F} USE_B={USE_B} FLASH={int(FLASH)} SYNC={int(SYNC)} P={P} B={B}: worst model gradients vs "
      "float64", flush=True)
for r, n in rows[:5]:
    print(f"   {r:.2e} (torch fp32 {rel(g32[n], g64[n]):.2e}) {n}", flush=True)
if os.environ.get("SAVE"):
    torch.save(g, os.environ["SAVE"])
    if POOL_OUTS:
        torch.save(POOL_OUTS, os.environ["SAVE"] + ".pool")
        cmp = os.environ.get("CMP", "") + ".pool"
        if os.path.exists(cmp):
            for i, (a, b) in enumerate(zip(POOL_OUTS, torch.load(cmp, weights_only=True))):
                Bn, Hh, Ww, Cc = a.shape
                wa = a.reshape(Bn, Hh // 2, 2, Ww // 2, 2, Cc).permute(0, 1, 3, 5, 2, 4).reshape(-1, 4)
                wb = b.reshape(Bn, Hh // 2, 2, Ww // 2, 2, Cc).permute(0, 1, 3, 5, 2, 4).reshape(-1, 4)
                flips = (wa.argmax(1) != wb.argmax(1)).nonzero().flatten()
                top = wa.topk(2, 1).values
                gap = (top[flips, 0] - top[flips, 1]).abs() / a.abs().max()
                print(f"encoder block {i + 1}: out rel diff {rel(a, b):.1e}, max-pool argmax flips {flips.numel()}"
                      f" (top-2 gaps / max|out| {[f'{v:.1e}' for v in gap.tolist()[:4]]})", flush=True)
    if os.environ.get("CMP") and os.path.exists(os.environ["CMP"]):
        o = torch.load(os.environ["CMP"], weights_only=True)
        d = sorted(((rel(g[n], o[n]), n) for n in g if not n.endswith("key_conv.bias")), reverse=True)
        print("vs", os.environ["CMP"], [(f"{r:.1e}", n) for r, n in d[:5]], flush=True)
