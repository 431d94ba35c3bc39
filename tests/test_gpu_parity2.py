"""Round-2 parity on the MI355X: the bf16 bar, the config-2 geometry, reference checkpoint interop,
the data-parallel step's HIP backward + grad_scale path, and the graph-captured RCCL reducer.

bf16 bar (north star: 1e-2 bf16).  PyTorch's own bf16 autocast of the REFERENCE misses 1e-2 on
logits on this network: tests/golden/bf16_calib.npz holds its error on the small model over the
fixture batch and 5 seeded batches (1.20e-2 .. 1.33e-2), cfg2_step.npz at the config-2 geometry
(1.81e-2).  The bar is therefore max(1e-2, the reference's own autocast error on the same batch),
per batch; loss, IoU and Dice are held to the plain 1e-2; thresholded predictions must agree
exactly on every pixel whose fp32 logit is farther than EPS from the 0.5-probability boundary.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
LP = {"bce_weight": 0.5, "dice_weight": 0.5}
ZERO = ("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias", "fusion_conv.0.bias", "key_conv.bias")
EPS = 0.05   # |logit| margin of the thresholded-metric rule (SURVEY.md section 7, bf16 parity)


def T(a, dev="cuda"):
    return torch.from_numpy(np.asarray(a)).to(dev)


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b).detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name)))


def small_model(precision):
    from models.unet_dfc_sa_res import UNetDFCSARes
    fx = load("model_small.npz")
    m = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, ablation_on_qk_channels=8, precision=precision)
    m.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")})
    return m.cuda().train()


def bf16_bar_check(logits, loss, stats, ref_logits, ref_loss, ref_iou, ref_dice, ac_rel, t):
    """The bf16 bar of the module docstring.  Returns (logits rel, bar)."""
    from dfcsa.loss import metrics_from_stats
    r = rel(logits, ref_logits)
    bar = max(1e-2, float(ac_rel))
    assert r <= bar, (r, bar)
    assert abs(loss - float(ref_loss)) <= 1e-2 * abs(float(ref_loss))
    iou, dice = metrics_from_stats(stats)
    assert abs(iou - float(ref_iou)) <= 1e-2 * max(abs(float(ref_iou)), 1e-2), (iou, ref_iou)
    assert abs(dice - float(ref_dice)) <= 1e-2 * max(abs(float(ref_dice)), 1e-2), (dice, ref_dice)
    lr = torch.as_tensor(np.asarray(ref_logits))
    confident = lr.abs() > EPS
    ours = logits.detach().float().cpu() > 0
    assert torch.equal(ours[confident], (lr > 0)[confident]), "thresholded prediction flipped on a confident pixel"
    return r, bar


# ----------------------------------------------------------------------------- bf16 bar
@pytest.mark.parametrize("tag", ["x1", "s0", "s1", "s2", "s3", "s4"])
def test_bf16_small_model_within_reference_autocast(tag):
    from dfcsa.loss import sigmoid
    from utils.metrics import calculate_metrics_device
    fx = load("bf16_calib.npz")
    model = small_model("bf16")
    with torch.no_grad():
        logits = model(T(fx[f"{tag}.x"]))
        met = calculate_metrics_device(sigmoid(logits), T(fx[f"{tag}.t"]), "bce_dice", {})
    r, bar = bf16_bar_check(logits, met["loss"].item(), met["stats"], fx[f"{tag}.logits"], fx[f"{tag}.loss"],
                            fx[f"{tag}.iou"], fx[f"{tag}.dice"], fx[f"{tag}.ac_logits_rel"], fx[f"{tag}.t"])
    print(f"{tag}: bf16 logits rel {r:.4e}, reference autocast {float(fx[tag + '.ac_logits_rel']):.4e}")


def test_bf16_small_model_no_worse_than_autocast_on_average():
    """Over the 6 calibration batches our bf16 mode is, on average, at least as close to the fp32
    reference as the reference's own bf16 autocast."""
    fx = load("bf16_calib.npz")
    model = small_model("bf16")
    ratios = []
    for tag in [str(t) for t in fx["tags"]]:
        with torch.no_grad():
            logits = model(T(fx[f"{tag}.x"]))
        ratios.append(rel(logits, fx[f"{tag}.logits"]) / float(fx[f"{tag}.ac_logits_rel"]))
    assert np.mean(ratios) <= 1.0, ratios


# ----------------------------------------------------------------------------- config-2 geometry
def cfg2_model(precision):
    """The fixture's model: torch.manual_seed(12000), DFC-SA-Res 64..512, P=4, gammas 0.5 (same
    module tree / creation order as the reference, so the seeded init is the reference's)."""
    from models.unet_dfc_sa_res import UNetDFCSARes
    fx = load("cfg2_step.npz")
    torch.manual_seed(12000)
    m = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4, ablation_on_qk_channels=8, precision=precision)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    for k, v in m.state_dict().items():
        if v.is_floating_point():
            assert abs(v.double().sum().item() - float(fx["init_sum." + k])) <= 1e-6 * max(1.0, abs(float(fx["init_sum." + k]))), k
    return m, fx


def scalar_or(base, n, p_numel, fx):
    """Tolerance of one gradient tensor at the config-2 geometry.  Scalars (res_scale, gamma) are a
    single sum over a whole block of cancelling terms: for down4.res_scale the terms' condition
    number sum|d*r| / |sum d*r| is 2.7e3 (measured on the reference), and the reference's OWN fp32
    gradient at the block output is 0.37 % off its float64 re-run (ours: 0.51 %), so the worst-case
    fp32 error of such a scalar is ~10x; they are held to 5e-2 against float64 instead of 5x the
    reference's one-sample fp32 error."""
    lim = max(base, 5.0 * float(fx["noise." + n]))
    return max(lim, 5e-2) if p_numel == 1 else lim


def test_cfg2_geometry_fp32_train_step():
    """Config-2 geometry (64..512, 224^2, P=4, B=2), fp32 compute mode, one full Trainer step:
    against the reference's own run (cfg2_step.npz) -- logits/loss 1e-4, IoU/Dice, pre-clip
    per-tensor gradient norms and the small tensors' full gradients against the reference re-run
    in float64, BN running stats, per-tensor SGD update norms -- and against the CPU oracle run
    here on the box (full per-tensor gradients, parameters after clip + SGD)."""
    from dfcsa.loss import metrics_from_stats, sigmoid
    from dfcsa.optim import FusedSGD
    from oracle import dfcsa_oracle as O
    from utils.metrics import calculate_metrics_device
    m, fx = cfg2_model("fp32")
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.cuda().train()
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    x, t = T(fx["x"]), T(fx["t"])
    opt.zero_grad()
    logits = m(x)
    met = calculate_metrics_device(sigmoid(logits), t, "bce_dice", LP)
    met["loss"].backward()
    torch.cuda.synchronize()
    assert rel(logits, fx["logits"]) < 1e-4
    assert abs(met["loss"].item() - float(fx["loss"])) < 1e-4 * abs(float(fx["loss"]))
    iou, dice = metrics_from_stats(met["stats"])
    assert abs(iou - float(fx["iou"])) < 1e-4 and abs(dice - float(fx["dice"])) < 1e-4
    pre = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    for n, g in pre.items():
        if n.endswith(ZERO):
            continue
        lim = scalar_or(5e-3, n, g.numel(), fx)
        ref_norm = float(fx["gnorm64." + n])
        assert abs(g.double().norm().item() - ref_norm) <= lim * ref_norm, (n, g.norm().item(), ref_norm)
        if "grad64." + n in fx:
            assert rel(g, fx["grad64." + n]) < lim, n
    opt.step(max_norm=1.0, skip_if_nan=met["loss"])
    torch.cuda.synchronize()
    assert abs(opt.last_norm.item() - float(fx["norm"])) < 1e-3 * float(fx["norm"])
    sd = m.state_dict()
    for k, v in sd.items():
        if "running" in k:
            assert rel(v.float(), fx["buf." + k]) < 1e-4, k
    for n, p in m.named_parameters():
        if n.endswith(ZERO):
            continue
        d = (p.detach().double().cpu() - sd0[n].double()).norm().item()
        assert abs(d - float(fx["dnorm." + n])) <= scalar_or(5e-3, n, p.numel(), fx) * float(fx["dnorm." + n]), n

    # the CPU oracle on this host: full gradient tensors and parameters after clip + SGD
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    sd1, _, ref = O.train_step(sd0, {}, x.cpu(), t.cpu(), 4, LP)
    clipped = {n: p.grad.detach().cpu() for n, p in m.named_parameters()}
    for n in O.param_names(sd0):
        if n.endswith(ZERO):
            continue
        lim = max(scalar_or(5e-3, n, clipped[n].numel(), fx), 10.0 * float(fx["noise." + n]))
        assert rel(clipped[n], ref["grads"][n]) < lim, n
        # the SGD update itself; both sides are fp32 parameters, so each update is quantised to the
        # parameter's ulp (BN weights = 1.0 take updates ~1e-5: 0.6 % resolution) -- allow that
        upd, upd_ref = sd[n].cpu().double() - sd0[n].double(), sd1[n].double() - sd0[n].double()
        quant = 2.0 * 2.0 ** -23 * sd0[n].double().norm().item()
        assert (upd - upd_ref).norm().item() <= lim * upd_ref.norm().item() + quant, n


def test_cfg2_geometry_bf16_within_reference_autocast():
    """Config-2 geometry in the benchmark dtype (bf16): logits within max(1e-2, the reference's
    autocast error at this geometry), loss/IoU/Dice 1e-2, confident pixels agree."""
    from dfcsa.loss import sigmoid
    from utils.metrics import calculate_metrics_device
    m, fx = cfg2_model("bf16")
    m = m.cuda().train()
    with torch.no_grad():
        logits = m(T(fx["x"]))
        met = calculate_metrics_device(sigmoid(logits), T(fx["t"]), "bce_dice", LP)
    r, bar = bf16_bar_check(logits, met["loss"].item(), met["stats"], fx["logits"], fx["loss"], fx["iou"], fx["dice"],
                            fx["calib.ac_logits_rel"], fx["t"])
    print(f"cfg2 bf16 logits rel {r:.4e} (bar {bar:.4e})")


def seeded_model(precision, pool, seed, fx):
    """A fixture's 64..512 model: torch.manual_seed(seed), pool ``pool``, gammas 0.5, checked against
    the fixture's seeded-init checksums (same module tree / creation order as the reference)."""
    from models.unet_dfc_sa_res import UNetDFCSARes
    torch.manual_seed(seed)
    m = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=pool, ablation_on_qk_channels=8, precision=precision)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    for k, v in m.state_dict().items():
        if v.is_floating_point():
            assert abs(v.double().sum().item() - float(fx["init_sum." + k])) <= 1e-6 * max(1.0, abs(float(fx["init_sum." + k]))), k
    return m


def _bf16_step(m, fx, xt=None):
    """One bf16 train step of model ``m`` on the fixture batch (or ``xt`` = (x, t) on the host; every
    bf16 block fusion on); returns (sd0, pre-clip grads, state after, x, t, logits, metrics)."""
    from dfcsa.loss import sigmoid
    from dfcsa.optim import FusedSGD
    from utils.metrics import calculate_metrics_device
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.cuda().train()
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    x, t = (T(fx["x"]), T(fx["t"])) if xt is None else (xt[0].cuda(), xt[1].cuda())
    opt.zero_grad()
    logits = m(x)
    met = calculate_metrics_device(sigmoid(logits), t, "bce_dice", LP)
    met["loss"].backward()
    torch.cuda.synchronize()
    pre = {n: p.grad.detach().double().cpu().clone() for n, p in m.named_parameters()}
    opt.step(max_norm=1.0, skip_if_nan=met["loss"])
    torch.cuda.synchronize()
    return sd0, pre, {k: v.detach().cpu() for k, v in m.state_dict().items()}, x, t, logits.detach(), met


def _cos_rel(g, r):
    g, r = g.reshape(-1), r.double().reshape(-1)
    return (g @ r / (g.norm() * r.norm() + 1e-300)).item(), ((g - r).norm() / (r.norm() + 1e-30)).item()


def _check_bf16_step_vs_autocast(tag, fb, pool, sd0, pre, sd, x, t, bufs_fp32, oracle=None):
    """The bar of test_cfg2_geometry_bf16_train_step_vs_reference_autocast (docstring there), against
    the fp32 oracle re-run on this host at pool size ``pool`` (or its result ``oracle`` =
    O.forward_backward(...) when the caller already ran it); ``fb`` holds the reference's autocast
    distances.  Prints every tensor's distances (worst first)."""
    from oracle import dfcsa_oracle as O
    SMALL = 4096
    if "x" in fb:
        assert torch.equal(x.cpu(), torch.from_numpy(fb["x"])) and torch.equal(t.cpu(), torch.from_numpy(fb["t"]))
    if oracle is None:
        torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
        oracle = O.forward_backward(sd0, x.cpu(), t.cpu(), pool, LP)
    _, _, gref, _ = oracle
    sd1, _, _, _ = O.clip_and_sgd(sd0, gref, {})
    rows, fails, scal = [], [], []
    sm = {"err": 0.0, "ac": 0.0, "uerr": 0.0, "uac": 0.0}
    for n in O.param_names(sd0):
        if n.endswith(ZERO):
            assert pre[n].abs().max().item() <= 1e-6 * max(1.0, gref[n].abs().max().item()), n
            continue
        cs, rr = _cos_rel(pre[n], gref[n])
        ac_rel, ac_cos = float(fb["ac_rel." + n]), float(fb["ac_cos." + n])
        ac_urel = float(fb["ac_upd_rel." + n])
        upd, upd_ref = sd[n].double() - sd0[n].double(), sd1[n].double() - sd0[n].double()
        quant = 2.0 * 2.0 ** -23 * sd0[n].double().norm().item()
        uerr = max(0.0, (upd - upd_ref).norm().item() - quant)
        ur = uerr / (upd_ref.norm().item() + 1e-30)
        if pre[n].numel() < SMALL:
            gn = gref[n].double().norm().item()
            sm["err"] += (rr * gn) ** 2
            sm["ac"] += (ac_rel * gn) ** 2
            sm["uerr"] += uerr ** 2
            sm["uac"] += (ac_urel * upd_ref.norm().item()) ** 2
            if pre[n].numel() == 1:
                # a scalar (gamma, res_scale): judged below against the pooled autocast noise
                scal.append((n, rr * gn, ac_rel * gn, uerr, ac_urel * upd_ref.norm().item()))
                ok = True
            else:
                ok = rr <= 5 * ac_rel + 2e-2 and ur <= 5 * ac_urel + 2e-2
        else:
            ok = rr <= max(1.25 * ac_rel, 2e-2) and 1 - cs <= 1.25 * (1 - ac_cos) + 1e-3
            if ur > max(1.25 * ac_urel, 2e-2):
                fails.append(f"{n}: update rel {ur:.3e} (autocast {ac_urel:.3e})")
        rows.append((rr / max(ac_rel, 1e-30), n, f"{n}: cos {cs:.5f} (autocast {ac_cos:.5f}) rel {rr:.3e} "
                                                 f"(autocast {ac_rel:.3e}) update rel {ur:.3e} (autocast "
                                                 f"{ac_urel:.3e})"))
        if not ok:
            fails.append(rows[-1][2])
    rows.sort(reverse=True)
    print(f"{tag} bf16 step, every tensor relative to the reference autocast (worst first):")
    for r in rows:
        print("   ", r[2])
    # scalars: each is ONE cancelling sum over B*H*W pixels, so one autocast distance is a single draw
    # of the bf16 noise (cfg2: 0.02 .. 6.3 relative across the 18 of them); the sanity bar per scalar
    # is 5 x the autocast's absolute error pooled (RMS) over all the model's scalars, for the gradient
    # and for the SGD update
    if scal:
        ac_g = (sum(c[2] ** 2 for c in scal) / len(scal)) ** 0.5
        ac_u = (sum(c[4] ** 2 for c in scal) / len(scal)) ** 0.5
        print(f"{tag} bf16 step, scalars: pooled autocast abs error gradient {ac_g:.3e}, update {ac_u:.3e}")
        for n, eg, _, eu, _ in scal:
            if eg > 5 * ac_g or eu > 5 * ac_u + 1e-12:
                fails.append(f"{n}: abs gradient error {eg:.3e} (pooled autocast {ac_g:.3e}), update {eu:.3e} "
                             f"(pooled autocast {ac_u:.3e})")
    g_small, g_ac = sm["err"] ** 0.5, sm["ac"] ** 0.5
    u_small, u_ac = sm["uerr"] ** 0.5, sm["uac"] ** 0.5
    print(f"{tag} bf16 step, small tensors as one vector: gradient error {g_small:.4e} (autocast {g_ac:.4e}), "
          f"update error {u_small:.4e} (autocast {u_ac:.4e})")
    if g_small > 1.25 * g_ac:
        fails.append(f"small-tensor gradient error {g_small:.4e} > 1.25 x autocast {g_ac:.4e}")
    if u_small > 1.25 * u_ac + 1e-12:
        fails.append(f"small-tensor update error {u_small:.4e} > 1.25 x autocast {u_ac:.4e}")
    names = [n for n in O.param_names(sd0) if not n.endswith(ZERO)]
    ga = torch.cat([pre[n].reshape(-1) for n in names])
    gb = torch.cat([gref[n].double().reshape(-1) for n in names])
    cos_all, rel_all = _cos_rel(ga, gb)
    print(f"{tag} bf16 step: whole-gradient cos {cos_all:.6f} (autocast {float(fb['ac_cos_all']):.6f}), "
          f"rel {rel_all:.4e} (autocast {float(fb['ac_rel_all']):.4e})")
    for k, v in sd.items():
        if "running" in k:
            bar = max(1.25 * float(fb["ac_buf_rel." + k]), 1e-3)
            if rel(v.float(), bufs_fp32["buf." + k]) > bar:
                fails.append(f"{k}: {rel(v.float(), bufs_fp32['buf.' + k]):.3e} > {bar:.3e}")
    assert not fails, fails
    assert cos_all >= float(fb["ac_cos_all"]) and rel_all <= float(fb["ac_rel_all"])


def test_cfg2_geometry_bf16_train_step_vs_reference_autocast():
    """The benchmark path itself: one bf16 train step at the config-2 geometry (64..512, 224^2, P=4,
    B=2, gammas 0.5) with every bf16 block fusion on (C = 64/128/256 blocks take dfcsa_dgrad_gate,
    dfcsa_dgrad_acc_relu_bn, the gate-fusion and local/attention prologue GEMMs, the apply prologues
    at C = 64, the fused max-pool passes).  Pinned to the reference's own bf16 error
    (tests/golden/cfg2_bf16.npz: the reference under CPU bf16 autocast against its float64 run),
    against the fp32 reference re-run here on the CPU oracle:
      * weight tensors (>= 4096 elements, pre-clip gradient): relative distance <= max(1.25 x the
        autocast's, 2e-2) and cosine distance 1 - cos <= 1.25 x the autocast's + 1e-3, every one of
        them (no fall-back bar);
      * the small tensors (biases, BatchNorm affine, the gamma / res_scale scalars): each of their
        elements is one reduction over B*H*W pixels whose bf16 error is rounding noise around a
        small, heavily cancelling sum, so one tensor's distance is a single noise sample (the
        autocast's own distance on down4's gamma is 6.3).  They are pinned as ONE vector:
        || ours - fp32 || <= 1.25 x || autocast - fp32 || over all of them (the autocast's per-tensor
        distances recombined exactly: sum_i (ac_rel_i * ||g_i||)^2), each vector tensor within 5 x its
        autocast distance + 2e-2 as a sanity bar, each scalar within 5 x the autocast's absolute
        error pooled (RMS) over the model's scalars (one scalar's autocast distance is a single
        noise draw), and the same for the SGD update;
      * over the whole gradient vector: no worse than the autocast;
      * BatchNorm running statistics after the step vs the reference fp32 step (cfg2_step.npz):
        <= max(1.25 x the autocast's distance, 1e-3);
      * the SGD update (clip 1.0 + momentum SGD) per weight tensor vs the oracle's update from the
        fp32 gradients: <= max(1.25 x the autocast update's distance, 2e-2).
    The conv biases that feed a train-mode BatchNorm have an exactly-zero gradient (ours is the
    exact zero; autocast's is rounding noise): they are held to zero."""
    fx = load("cfg2_step.npz")
    fb = load("cfg2_bf16.npz")
    sd0, pre, sd, x, t, _, _ = _bf16_step(seeded_model("bf16", 4, 12000, fx), fx)
    _check_bf16_step_vs_autocast("cfg2", fb, 4, sd0, pre, sd, x, t, fx)


def test_cfg3_geometry_bf16_train_step_vs_reference_autocast():
    """Config 3 (config_dfc-sa-res-block.yaml: pool_size 8) at its benchmark geometry -- 64..512,
    224^2, B = 2 per GPU, bf16 -- one train step through the benchmark path: the P = 8 attention (N =
    64 tokens, non-divisible 28 -> 8 / 14 -> 8 pooling windows) and every bf16 block fusion.  Pinned
    to tests/golden/cfg3_bf16.npz (the reference under CPU bf16 autocast against its float64 run,
    plus its fp32 step): logits within max(1e-2, the autocast's own logits error), loss / IoU / Dice
    1e-2, confident pixels identical; then the gradient / update / BatchNorm bar of the config-2 test
    (no fall-back bar)."""
    fb = load("cfg3_bf16.npz")
    sd0, pre, sd, x, t, logits, met = _bf16_step(seeded_model("bf16", 8, 14000, fb), fb)
    r, bar = bf16_bar_check(logits, met["loss"].item(), met["stats"], fb["logits"], fb["loss"], fb["iou"], fb["dice"],
                            fb["ac_logits_rel"], fb["t"])
    print(f"cfg3 bf16 logits rel {r:.4e} (bar {bar:.4e}; reference autocast {float(fb['ac_logits_rel']):.4e})")
    _check_bf16_step_vs_autocast("cfg3", fb, 8, sd0, pre, sd, x, t, fb)


def test_timed_config_b16_bf16_train_step_vs_oracle_and_reference_autocast():
    """The configuration bench.py times, end to end: 64..512, 224^2, P = 4, **B = 16**, bf16, every
    default route.  At B = 16 the step takes routes no B = 2 test reaches -- M = 16 x H x W puts the
    56^2 N >= 512 1x1 GEMMs and ConvTransposes on the mid-M streaming kernel (M >= 32768), and the
    weight-gradient split plans and split-K choices are functions of M.  One step from a seeded init
    (torch.manual_seed(16000), gammas 0.5; init checksums vs the reference's), on the batch
    tests/golden/make_golden.py (12d) drew from seed 16001 (regenerated here, checked against the
    fixture's checksums), against:
      * the fp32 oracle run on this host's CPU (~12 s on 16 threads), itself pinned here to the
        reference's fp32 step at B = 16 (image 0's logits 1e-4, logits checksums, loss);
      * the bf16 bar of bf16_bar_check -- logits within max(1e-2, the reference's own CPU bf16
        autocast error at B = 16, tests/golden/cfg2b16_bf16.npz), loss / IoU / Dice 1e-2, confident
        pixels identical;
      * the gradient / SGD-update / BatchNorm bar of test_cfg2_geometry_bf16_train_step_vs_reference_
        autocast against the reference autocast's distances AT B = 16 (same fixture): weight tensors
        per tensor, small tensors as one vector, whole gradient no worse than autocast.
    Reference: utils/trainer.py:115-151, models/unet_dfc_sa_res.py:161-204, train.py:73-78."""
    from oracle import dfcsa_oracle as O
    fb = load("cfg2b16_bf16.npz")
    B = int(fb["B"])
    assert B == 16 and int(fb["pool"]) == 4
    g = torch.Generator().manual_seed(int(fb["bseed"]))
    x = torch.randn(B, 3, 224, 224, generator=g)
    t = (torch.rand(B, 1, 224, 224, generator=g) > 0.5).float()
    assert abs(x.double().sum().item() - float(fb["x_sum"])) <= 1e-9 * float(fb["x_sqsum"])
    assert abs((x.double() ** 2).sum().item() - float(fb["x_sqsum"])) <= 1e-12 * float(fb["x_sqsum"])
    assert t.double().sum().item() == float(fb["t_sum"])
    m = seeded_model("bf16", 4, int(fb["seed"]), fb)
    sd0, pre, sd, x, t, logits, met = _bf16_step(m, fb, (x, t))
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    orc = O.forward_backward(sd0, x.cpu(), t.cpu(), 4, LP)
    lref, mref = orc[0], orc[1]
    # the oracle against the reference's own fp32 step at B = 16
    assert rel(lref[0], fb["logits0"]) < 1e-4, rel(lref[0], fb["logits0"])
    assert abs(lref.double().norm().item() - float(fb["logits_norm"])) <= 1e-4 * float(fb["logits_norm"])
    assert abs(float(mref["loss"]) - float(fb["loss"])) <= 1e-4 * abs(float(fb["loss"]))
    r, bar = bf16_bar_check(logits, met["loss"].item(), met["stats"], lref.numpy(), fb["loss"], fb["iou"], fb["dice"],
                            fb["ac_logits_rel"], None)
    print(f"timed config B=16 bf16 logits rel {r:.4e} (bar {bar:.4e}; reference autocast "
          f"{float(fb['ac_logits_rel']):.4e})")
    _check_bf16_step_vs_autocast("b16", fb, 4, sd0, pre, sd, x, t, fb, oracle=orc)


# ----------------------------------------------------------------------------- checkpoint interop
def test_reference_checkpoint_resume(tmp_path):
    """A checkpoint written by the reference's own Trainer.save_checkpoint (tests/golden/
    ref_checkpoint_epoch_1.pth, utils/trainer.py:267-298) loads with weights_only=True into our
    Trainer (model, torch.optim.SGD converted to the fused pass, histories), and one more epoch
    reproduces the reference's resumed epoch (its own load_checkpoint + train_epoch): loss and
    every parameter -- which requires the SGD momentum to be restored from the checkpoint.  Our own
    checkpoint of that state keeps the reference's metrics layout (best/worst samples)."""
    from utils.trainer import Trainer
    from models.unet_dfc_sa_res import UNetDFCSARes
    fx = load("ref_checkpoint_resume.npz")
    model = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, precision="fp32")
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    cfg = {"training": {"num_epochs": 2, "save_checkpoint_freq": 1, "loss": {"type": "bce_dice", "params": LP}},
           "logging": {"log_dir": str(tmp_path / "logs"), "images_dir": str(tmp_path / "img"),
                       "save_best_worst_samples": 1}}
    b3 = [{"image": torch.from_numpy(fx["x3"]), "mask": torch.from_numpy(fx["t3"]), "filename": ["a3", "b3"]}]
    tr = Trainer(model, b3, b3, opt, torch.device("cuda"), cfg)
    ep = tr.load_checkpoint(os.path.join(GOLDEN, "ref_checkpoint_epoch_1.pth"))
    assert ep == int(fx["epoch"])
    assert abs(tr.train_losses[0] - float(fx["train_loss1"])) < 1e-12
    assert abs(tr.val_dice_scores[0] - float(fx["val_dice1"])) < 1e-12
    loss, iou, dice = tr.train_epoch(ep + 1)
    torch.cuda.synchronize()
    assert abs(loss - float(fx["loss3"])) < 1e-4 * abs(float(fx["loss3"]))
    assert abs(dice - float(fx["dice3"])) < 1e-6 and abs(iou - float(fx["iou3"])) < 1e-6
    sd = model.state_dict()
    for k, v in fx.items():
        if k.startswith("sd3.") and "num_batches" not in k:
            assert rel(sd[k[4:]].float(), torch.from_numpy(np.asarray(v)).float()) < 1e-4, k
    va = tr.validate_epoch(b3)
    tr.save_checkpoint(ep + 1, va, is_best=False)
    ck = torch.load(str(tmp_path / "logs" / "checkpoints" / f"checkpoint_epoch_{ep + 2}.pth"), weights_only=True)
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "train_losses", "val_losses",
                       "train_dice_scores", "val_dice_scores", "train_iou_scores", "val_iou_scores", "best_val_loss",
                       "metrics"}
    assert set(ck["metrics"]) == {"loss", "iou", "dice", "best_samples", "worst_samples"}
    assert len(ck["metrics"]["best_samples"]) == 1 and "image" in ck["metrics"]["best_samples"][0]


def test_fused_sgd_resume_matches_torch_sgd():
    """FusedSGD.load_state_dict before the first forward keeps the loaded momentum (the
    step after resuming equals torch.optim.SGD loaded from the same state)."""
    from dfcsa.loss import sigmoid
    from dfcsa.optim import FusedSGD
    from utils.metrics import calculate_metrics_device
    fx = load("model_small.npz")
    ck = torch.load(os.path.join(GOLDEN, "ref_checkpoint_epoch_1.pth"), weights_only=True)
    model = small_model("fp32")
    model.load_state_dict(ck["model_state_dict"])
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    opt.load_state_dict(ck["optimizer_state_dict"])   # before the first forward: no flat storage yet
    x, t = T(fx["x2"]), T(fx["t2"])
    opt.zero_grad()
    met = calculate_metrics_device(sigmoid(model(x)), t, "bce_dice", LP)
    met["loss"].backward()
    g = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    w = {n: p.detach().clone() for n, p in model.named_parameters()}
    opt.step(max_norm=1.0, skip_if_nan=met["loss"])
    # the same step with torch's clip_grad_norm_ + SGD from the same state
    ps = [torch.nn.Parameter(w[n].clone()) for n, _ in model.named_parameters()]
    for p, n in zip(ps, g):
        p.grad = g[n].clone()
    topt = torch.optim.SGD(ps, lr=0.01, momentum=0.9, weight_decay=1e-4)
    topt.load_state_dict(ck["optimizer_state_dict"])
    torch.nn.utils.clip_grad_norm_(ps, max_norm=1.0)
    topt.step()
    for (n, p), q in zip(model.named_parameters(), ps):
        assert rel(p, q) < 1e-6, n


def test_clip_sgd_nan_semantics():
    """a NaN loss skips the update (reference trainer.py:134-139); an inf loss does not;
    a NaN gradient norm gives NaN gradients/weights like torch's clip_grad_norm_ (coef = NaN)."""
    from dfcsa.optim import FusedSGD
    model = small_model("fp32")
    model(T(load("model_small.npz")["x1"]))    # materialise the flat storage
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    opt.zero_grad()
    for p in model.parameters():
        p.grad.fill_(0.01)
    w0 = [p.detach().clone() for p in model.parameters()]
    opt.step(max_norm=1.0, skip_if_nan=torch.tensor([float("nan")], device="cuda"))
    assert all(torch.equal(p, q) for p, q in zip(model.parameters(), w0))
    opt.step(max_norm=1.0, skip_if_nan=torch.tensor([float("inf")], device="cuda"))
    assert not all(torch.equal(p, q) for p, q in zip(model.parameters(), w0))
    opt.zero_grad()
    next(iter(model.parameters())).grad.view(-1)[0] = float("nan")
    opt.step(max_norm=1.0)
    assert torch.isnan(opt.last_norm).all()
    assert all(torch.isnan(p).all() for p in model.parameters())


def test_clip_sgd_zero_after_step_same_update():
    """zero_after_step (bench.py, Trainer): the fused pass writes zeros to the gradients instead of
    the clipped values -- on a NaN-skipped step too -- and the weights and momentum are bit-identical
    to the default pass over the same steps (resumed momentum included)."""
    from dfcsa.optim import FusedSGD
    x = T(load("model_small.npz")["x1"])
    models, opts = [], []
    for zero in (False, True):
        torch.manual_seed(0)
        m = small_model("fp32")
        m(x)
        models.append(m)
        opts.append(FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4, zero_after_step=zero))
    gen = torch.Generator(device="cuda").manual_seed(3)
    skips = [None, torch.tensor([float("nan")], device="cuda"), torch.tensor([0.5], device="cuda"), None]
    for skip in skips:
        grads = [torch.randn(p.shape, device="cuda", generator=gen) * 0.05 for p in models[0].parameters()]
        for m, opt in zip(models, opts):
            opt.zero_grad()
            assert all(torch.count_nonzero(p.grad) == 0 for p in m.parameters())
            for p, g in zip(m.parameters(), grads):
                p.grad.copy_(g)
            opt.step(max_norm=1.0, skip_if_nan=skip)
        torch.cuda.synchronize()
        assert torch.equal(opts[0]._mom, opts[1]._mom)
        assert torch.equal(opts[0].last_norm, opts[1].last_norm)
        for p, q in zip(*(m.parameters() for m in models)):
            assert torch.equal(p, q)
        assert all(torch.count_nonzero(p.grad) == 0 for p in models[1].parameters())
    assert any(torch.count_nonzero(p.grad) > 0 for p in models[0].parameters())


def test_eval_mode_backward_is_refused():
    """the backward kernels are train-mode BatchNorm; a backward through an eval-mode
    forward raises instead of returning wrong gradients."""
    from dfcsa.loss import sigmoid
    model = small_model("fp32").eval()
    x = T(load("model_small.npz")["x1"]).requires_grad_(True)
    out = sigmoid(model(x)).sum()
    with pytest.raises(NotImplementedError):
        out.backward()


# ----------------------------------------------------------------------------- data parallel
def test_ddp_step_hip_backward_with_grad_scale():
    """The DP step without a second GPU: the HIP backward of each half of ddp_shards.npz accumulates
    into the flat gradient buffer (what the all-reduce SUM of 2 ranks produces), then the fused
    clip + SGD applies grad_scale = 1/2.  Gradients vs the reference's mean of per-shard gradients;
    parameters after the step vs the reference SGD step taken with those mean gradients."""
    from dfcsa.loss import sigmoid
    from dfcsa.optim import FusedSGD
    from oracle import dfcsa_oracle as O
    from utils.metrics import calculate_metrics_device
    dd = load("ddp_shards.npz")
    model = small_model("fp32")
    sd0 = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    x, t = T(dd["x"]), T(dd["t"])
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    opt.zero_grad()
    for r in range(2):
        met = calculate_metrics_device(sigmoid(model(x[4 * r:4 * r + 4])), t[4 * r:4 * r + 4], "bce_dice", LP)
        met["loss"].backward()
    torch.cuda.synchronize()
    mean = {}
    for n, p in model.named_parameters():
        ref = dd[f"w2.mean_grad.{n}"]
        mean[n] = torch.from_numpy(ref)
        if n.endswith(ZERO):
            continue
        assert rel(p.grad * 0.5, ref) < 2e-3, n
    opt.step(max_norm=1.0, grad_scale=0.5, skip_if_nan=met["loss"])
    torch.cuda.synchronize()
    sd1, _, norm, _ = O.clip_and_sgd(sd0, mean, {})
    assert abs(opt.last_norm.item() - norm.item()) < 1e-3 * norm.item()
    for n, p in model.named_parameters():
        if n.endswith(ZERO):
            continue
        assert rel(p.detach().cpu() - sd0[n], sd1[n] - sd0[n]) < 3e-3, n   # the SGD update


def _run_child_logged(name, argv, timeout):
    """Run a child process with its FULL stdout / stderr kept in files next to the test log
    (gpurun_out/<name>.{out,err}; DFCSA_TEST_LOGDIR overrides), so an abort's own message survives."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    logdir = os.environ.get("DFCSA_TEST_LOGDIR", os.path.join(root, "gpurun_out"))
    os.makedirs(logdir, exist_ok=True)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("MASTER_PORT", None)
    out_p, err_p = os.path.join(logdir, name + ".out"), os.path.join(logdir, name + ".err")
    with open(out_p, "w") as fo, open(err_p, "w") as fe:
        r = subprocess.run([sys.executable] + argv, stdout=fo, stderr=fe, text=True, timeout=timeout, env=env, cwd=root)
    out, err = open(out_p).read(), open(err_p).read()
    line = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and line, (r.returncode, f"full logs: {out_p} {err_p}", out[-1500:], err[-3000:])
    return json.loads(line[-1])


def test_rccl_bucket_reducer_graph_replay_equals_eager():
    """The multi-GPU step rehearsed on one GPU (tools/rccl_graph_check.py, in a child process so the
    RCCL communicator lives and dies with it): an RCCL (backend 'nccl') group of world size 1, the
    bucket reducer forced to several buckets, the NaN-agreement flag, and the whole step captured in
    one HIP graph (thread_local capture, watchdog drained: dfcsa.ddp.capture_step); 2 graph replays
    after 1 eager step equal 3 eager steps; the drop-in Trainer with training.data_parallel captures
    and replays its reducer step equal to its eager step; the child tears down as bench.py does
    (dfcsa.ddp.shutdown) and must exit 0."""
    res = _run_child_logged("rccl_graph_check", [os.path.join("tools", "rccl_graph_check.py")], 300)
    assert res["ok"], res


def test_bench_ddp_path_exits_cleanly():
    """bench.py's N > 1 code path on one GPU (--ddp-rehearsal: RCCL group of world size 1, bucket
    reducer, graph-captured step with its collectives, the max-over-ranks timing all-reduce, the
    kernel-timing leg, then the teardown): one JSON line and exit status 0."""
    res = _run_child_logged("bench_ddp_rehearsal",
                            ["bench.py", "--ddp-rehearsal", "--img", "64", "--batch", "4", "--steps", "3",
                             "--warmup", "2", "--bucket-mb", "4", "--no-cpu-baseline", "--no-val-dice",
                             "--no-trainer-faithful"], 300)
    assert res["config"]["ddp_path"] is True and res["launch"] == "hip_graph", res
    assert res["value"] > 0 and res["roofline"] is not None, res
