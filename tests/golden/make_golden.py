"""Generate golden fixtures by running the REFERENCE implementation (CPU, fp32).

Runs only in the build container, where the read-only reference checkout lives at
/root/reference.  The reference itself never travels: only the .npz outputs written next to
this script are committed and used by the tests (inputs + expected outputs, i.e. data).

Reference files imported (file-by-file, via importlib, because the reference's package
``__init__`` files import modules that do not exist):
  * models/unet_dfc_sa_res.py   LightSelfAttention :5-39, DynamicFusionConvAttnBlock :41-116,
                                UNetDFCSA :118-204, UNetDFCSARes :207-220
  * utils/metrics.py            dice_loss :6-24, BCEDiceLoss :52-78, calculate_metrics :211-264
  * models/unet.py              UNet :69-101 (config 1)
  * models/transformer_unet.py  TransUNet :347-368 with get_r50_b16_config :318-342 (config 4;
                                ml_collections replaced by a dict-with-attributes ConfigDict)
  * models/unet_dfc_sa_ablation_attention.py   FullResolutionAttention :7-26, FullResAttnDFCBlock
                                :29-92, UNet_FullResAttention :95-97 (config 5; imported under a stub
                                package because it uses a package-relative import of
                                unet_dfc_sa_ablation_branches.py)
  * models/unet_dfc_sa_ablation_branches.py / _fusion.py / _placement.py   the ablation zoo (seven
                                models; imported under the stub package like the attention ablation)
  * inference.py                calculate_segmentation_metrics :73-91, predict_large_image :104-153
                                (those two functions only, taken from the source with ast: the module
                                imports cv2 / matplotlib / torchvision, which are not installed)
The train-step semantics follow utils/trainer.py:115-151 and train.py:73-78.

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz, ~a few MB)
"""
import importlib.util
import os
import sys

import numpy as np
import torch

REF = os.environ.get("DFCSA_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ref_res = _load("ref_unet_dfc_sa_res", "models/unet_dfc_sa_res.py")
ref_metrics = _load("ref_metrics", "utils/metrics.py")
ref_unet = _load("ref_unet", "models/unet.py")


def _load_models_pkg(relmod):
    """Import reference models/<relmod>.py inside a stub package so its relative imports resolve
    (the reference's own models/__init__.py imports a module that does not exist)."""
    import types
    if "refmodels" not in sys.modules:
        pkg = types.ModuleType("refmodels")
        pkg.__path__ = [os.path.join(REF, "models")]
        sys.modules["refmodels"] = pkg
    name = "refmodels." + relmod
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, "models", relmod + ".py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {name}: {sum(np.asarray(v).nbytes for v in arrays.values())/1e6:.2f} MB raw")


def sd_arrays(module, prefix="sd."):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def grad_arrays(module, prefix="grad."):
    return {prefix + n: np32(p.grad) for n, p in module.named_parameters() if p.grad is not None}


def fp64_noise(module32, module64, prefix="noise."):
    """Per-tensor relative distance between the reference's fp32 gradients and the same reference
    run in float64 on the same weights and inputs: the reference's own fp32 rounding floor.  The GPU
    tests scale their gradient tolerance by it (deep nets with train-mode BatchNorm amplify fp32
    summation-order differences into gradient noise of a few 1e-3 on some tensors)."""
    g64 = dict(module64.named_parameters())
    out = {}
    for n, p in module32.named_parameters():
        if p.grad is None:
            continue
        a, b = p.grad.double(), g64[n].grad
        out[prefix + n] = np.float64(((a - b).norm() / (b.norm() + 1e-30)).item())
    a = torch.cat([p.grad.double().reshape(-1) for n, p in module32.named_parameters() if p.grad is not None])
    b = torch.cat([g64[n].grad.reshape(-1) for n, p in module32.named_parameters() if p.grad is not None])
    out[prefix + "all"] = np.float64(((a - b).norm() / (b.norm() + 1e-30)).item())
    return out


def bf16_autocast_cosine(model, x, t, loss_params, m64):
    """Gradient cosine between the reference run under CPU bf16 autocast and the float64 reference:
    what bf16 arithmetic alone does to the gradient (the bar for the build's bf16 mode)."""
    import copy
    mb = copy.deepcopy(model)
    mb.zero_grad()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        out = mb(x)
    met = ref_metrics.calculate_metrics(torch.sigmoid(out.float()), t, "bce_dice", loss_params)
    met["loss"].backward()
    g = torch.cat([p.grad.double().reshape(-1) for p in mb.parameters()])
    r = torch.cat([p.grad.reshape(-1) for p in m64.parameters()])
    return np.float64((g @ r / (g.norm() * r.norm())).item())


def fp64_twin(module):
    import copy
    return copy.deepcopy(module).double()


# ----------------------------------------------------------------------------------------
# (1) LightSelfAttention forward/backward, gamma = 0.7 (gamma inits to 0, which would hide
#     the attention path).  Non-divisible adaptive-pool windows at H=14 (P=4,8) and H=28 (P=8),
#     and P > H (pool upsamples) at H=14, P=16/32.
# ----------------------------------------------------------------------------------------
def gen_lsa():
    cases = [(8, 14, p) for p in (4, 8, 16, 32)] + [(8, 28, p) for p in (4, 8, 16, 32)] + \
            [(8, 56, p) for p in (4, 8)] + [(64, 14, p) for p in (4, 8, 32)] + [(64, 28, 8)]
    for (C, H, P) in cases:
        torch.manual_seed(1000 + C * 7 + H * 3 + P)
        m = ref_res.LightSelfAttention(C, pool_size=P, ablation_on_qk_channels=8)
        with torch.no_grad():
            m.gamma.fill_(0.7)
        x = torch.randn(2, C, H, H, requires_grad=True)
        y = m(x)
        g = torch.randn_like(y)
        y.backward(g)
        save(f"lsa_C{C}_H{H}_P{P}.npz", x=np32(x), g=np32(g), y=np32(y), dx=np32(x.grad),
             **sd_arrays(m), **grad_arrays(m))


# ----------------------------------------------------------------------------------------
# (2) DynamicFusionConvAttnBlock, train-mode forward + backward + BN running stats.
# ----------------------------------------------------------------------------------------
def gen_block():
    for (cin, cout, H, P) in [(3, 8, 32, 4), (16, 8, 16, 8), (16, 16, 14, 4)]:
        torch.manual_seed(2000 + cin * 11 + cout + H)
        blk = ref_res.DynamicFusionConvAttnBlock(cin, cout, pool_size=P, ablation_on_qk_channels=8)
        with torch.no_grad():
            blk.attn_branch[3].gamma.fill_(0.7)
        sd0 = sd_arrays(blk, "sd0.")
        blk.train()
        x = torch.randn(2, cin, H, H, requires_grad=True)
        y = blk(x)
        g = torch.randn_like(y)
        y.backward(g)
        save(f"block_{cin}to{cout}_H{H}_P{P}.npz", x=np32(x), g=np32(g), y=np32(y),
             dx=np32(x.grad), **sd0, **sd_arrays(blk, "sd1."), **grad_arrays(blk))


# ----------------------------------------------------------------------------------------
# (3) Whole model: two full train steps exactly as Trainer.train_epoch + SGD do them.
# ----------------------------------------------------------------------------------------
LOSS_PARAMS = {"bce_weight": 0.5, "dice_weight": 0.5}  # as in the DFC yaml configs (ignored keys)


def perturb_gammas(model):
    with torch.no_grad():
        for i, (n, p) in enumerate(sorted(model.named_parameters())):
            if n.endswith("gamma"):
                p.fill_(0.2 + 0.05 * (i % 9))


def train_step(model, opt, x, t):
    """utils/trainer.py:120-151."""
    opt.zero_grad()
    out = model(x)
    prob = torch.sigmoid(out)
    met = ref_metrics.calculate_metrics(prob, t, "bce_dice", LOSS_PARAMS)
    loss = met["loss"]
    loss.backward()
    norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
    grads = grad_arrays(model)  # post-clip grads
    opt.step()
    return out, met, norm, grads


def base_model(P=4):
    """The one initial model every whole-model fixture starts from (stored once, as sd0)."""
    torch.manual_seed(3000)
    model = ref_res.UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, ablation_on_qk_channels=8)
    perturb_gammas(model)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    m = ref_res.UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=P, ablation_on_qk_channels=8)
    m.load_state_dict(sd)  # pool_size does not change the parameter set
    return m


def batch(gen, shape):
    x = torch.randn(*shape, generator=gen)
    t = (torch.rand(shape[0], 1, shape[2], shape[3], generator=gen) > 0.5).float()
    return x, t


def gen_model():
    # Two full train steps (P=4): step-1 post-clip grads, params + momentum after step 2.
    model = base_model(4)
    sd0 = sd_arrays(model, "sd0.")
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    model.train()
    gen = torch.Generator().manual_seed(3001)
    x1, t1 = batch(gen, (2, 3, 32, 32))
    x2, t2 = batch(gen, (2, 3, 32, 32))
    out1, met1, norm1, g1 = train_step(model, opt, x1, t1)
    bn1 = {"bn1." + k: v.numpy().copy() for k, v in model.state_dict().items() if "running" in k or "num_batches" in k}
    out2, met2, norm2, _ = train_step(model, opt, x2, t2)
    sd2 = sd_arrays(model, "sd2.")
    save("model_small.npz", x1=np32(x1), t1=np32(t1), x2=np32(x2), t2=np32(t2),
         logits1=np32(out1), loss1=np32(met1["loss"]), iou1=np.float64(met1["iou"]),
         dice1=np.float64(met1["dice"]), norm1=np32(norm1),
         logits2=np32(out2), loss2=np32(met2["loss"]), iou2=np.float64(met2["iou"]),
         dice2=np.float64(met2["dice"]), norm2=np32(norm2),
         **sd0, **bn1, **sd2, **{"step1." + k: v for k, v in g1.items()})

    # P=8 (non-divisible pool windows at 4x4/2x2 maps, P > H at the bottleneck): fwd + grads.
    model = base_model(8)
    model.train()
    out = model(x1)
    met = ref_metrics.calculate_metrics(torch.sigmoid(out), t1, "bce_dice", LOSS_PARAMS)
    met["loss"].backward()
    save("model_p8.npz", logits=np32(out), loss=np32(met["loss"]), iou=np.float64(met["iou"]),
         dice=np.float64(met["dice"]), **grad_arrays(model))

    # Non-divisible input (36 -> 18 -> 9 -> 4 -> 2): exercises the bilinear shape fix
    # (unet_dfc_sa_res.py:180-199) and floor max-pooling of odd sizes.  Forward + grads.
    model = base_model(4)
    model.train()
    gen = torch.Generator().manual_seed(3100)
    x, t = batch(gen, (1, 3, 36, 36))
    out = model(x)
    met = ref_metrics.calculate_metrics(torch.sigmoid(out), t, "bce_dice", LOSS_PARAMS)
    met["loss"].backward()
    save("model_odd36.npz", x=np32(x), t=np32(t), logits=np32(out), loss=np32(met["loss"]),
         iou=np.float64(met["iou"]), dice=np.float64(met["dice"]), **grad_arrays(model))

    # Eval-mode forward (BN running statistics) after perturbing the running stats.
    model = base_model(4)
    torch.manual_seed(3200)
    with torch.no_grad():
        for n, b in model.named_buffers():
            if n.endswith("running_mean"):
                b.normal_(0, 0.1)
            elif n.endswith("running_var"):
                b.uniform_(0.5, 1.5)
    model.eval()
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        out = model(x)
    save("model_eval.npz", x=np32(x), logits=np32(out),
         **{"buf." + k: v.numpy() for k, v in model.state_dict().items() if "running" in k})


# ----------------------------------------------------------------------------------------
# (4) calculate_metrics edge cases (BCE log clamp at -100, p == 0.5 threshold, empty masks,
#     the weight_bce/weight_dice vs bce_weight/dice_weight key gotcha).
# ----------------------------------------------------------------------------------------
def gen_metrics():
    rng = np.random.default_rng(4000)
    p = rng.uniform(0, 1, size=(2, 1, 16, 16)).astype(np.float32)
    t = (rng.uniform(size=(2, 1, 16, 16)) > 0.5).astype(np.float32)
    p_edge = p.copy()
    p_edge[0, 0, 0, :4] = [0.0, 1.0, 0.5, 0.5]
    t_edge = t.copy()
    t_edge[0, 0, 0, :4] = [1.0, 0.0, 1.0, 0.0]
    cases = {
        "random_default": (p, t, {}),
        "random_keygotcha": (p, t, {"bce_weight": 0.5, "dice_weight": 0.5}),
        "random_weighted": (p, t, {"weight_bce": 0.3, "weight_dice": 2.0}),
        "edge_clamp": (p_edge, t_edge, {}),
        "empty_mask": (p, np.zeros_like(t), {}),
        "all_low": (p * 0.4, t, {}),
    }
    out = {}
    for k, (pp, tt, params) in cases.items():
        pt = torch.tensor(pp, requires_grad=True)
        tt_ = torch.tensor(tt)
        met = ref_metrics.calculate_metrics(pt, tt_, "bce_dice", params)
        met["loss"].backward()
        out[k + ".p"] = pp
        out[k + ".t"] = tt
        out[k + ".wbce"] = np.float32(params.get("weight_bce", 1.0))
        out[k + ".wdice"] = np.float32(params.get("weight_dice", 1.0))
        out[k + ".loss"] = np32(met["loss"])
        out[k + ".iou"] = np.float64(met["iou"])
        out[k + ".dice"] = np.float64(met["dice"])
        out[k + ".dp"] = np32(pt.grad)
    save("metrics_bce_dice.npz", **out)


def gen_metrics_dice():
    """The reference's 'dice' loss type (calculate_metrics :251-252 -> dice_loss :6-24): loss, IoU,
    Dice and dL/dp on the cases of gen_metrics (p at exactly 0 and 1 included, an empty mask)."""
    rng = np.random.default_rng(4000)
    p = rng.uniform(0, 1, size=(2, 1, 16, 16)).astype(np.float32)
    t = (rng.uniform(size=(2, 1, 16, 16)) > 0.5).astype(np.float32)
    p_edge = p.copy()
    p_edge[0, 0, 0, :4] = [0.0, 1.0, 0.5, 0.5]
    t_edge = t.copy()
    t_edge[0, 0, 0, :4] = [1.0, 0.0, 1.0, 0.0]
    out = {}
    for k, (pp, tt) in {"random": (p, t), "edge_clamp": (p_edge, t_edge), "empty_mask": (p, np.zeros_like(t)),
                        "all_low": (p * 0.4, t)}.items():
        pt = torch.tensor(pp, requires_grad=True)
        met = ref_metrics.calculate_metrics(pt, torch.tensor(tt), "dice", {})
        met["loss"].backward()
        out.update({k + ".p": pp, k + ".t": tt, k + ".loss": np32(met["loss"]), k + ".iou": np.float64(met["iou"]),
                    k + ".dice": np.float64(met["dice"]), k + ".dp": np32(pt.grad)})
    save("metrics_dice.npz", **out)


# ----------------------------------------------------------------------------------------
# (5) DDP parity target: mean over 4 shards (2 images each) of per-shard gradients (local BN,
#     per-shard Dice), from identical initial weights.  Also 2 shards of 4.
# ----------------------------------------------------------------------------------------
def gen_ddp():
    sd = {k: v.clone() for k, v in base_model(4).state_dict().items()}  # = model_small sd0
    gen = torch.Generator().manual_seed(5001)
    x, t = batch(gen, (8, 3, 32, 32))
    res = {"x": np32(x), "t": np32(t)}
    for world in (2, 4):
        acc = None
        per = x.shape[0] // world
        for r in range(world):
            m = ref_res.UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, ablation_on_qk_channels=8)
            m.load_state_dict(sd)
            m.train()
            out = m(x[r * per:(r + 1) * per])
            met = ref_metrics.calculate_metrics(torch.sigmoid(out), t[r * per:(r + 1) * per],
                                                "bce_dice", LOSS_PARAMS)
            met["loss"].backward()
            g = grad_arrays(m)
            acc = g if acc is None else {k: acc[k] + g[k] for k in acc}
        for k, v in acc.items():
            res[f"w{world}.mean_{k}"] = v / world
    save("ddp_shards.npz", **res)


# ----------------------------------------------------------------------------------------
# (6) Config 1 plumbing: plain UNet (widths hard-coded 64..1024) at 64x64, batch 2.
# ----------------------------------------------------------------------------------------
def _unet_run(seed, shape, name, bilinear=False):
    """One seeded reference UNet forward/backward at `shape` (see gen_unet)."""
    torch.manual_seed(seed)
    m = ref_unet.UNet(3, 1, bilinear=bilinear)
    init = {"init_sum." + k: np.float64(v.double().sum()) for k, v in m.state_dict().items()
            if v.is_floating_point()}
    m.train()
    m64 = fp64_twin(m)
    x = torch.randn(*shape)
    t = (torch.rand(shape[0], 1, shape[2], shape[3]) > 0.5).float()
    out = m(x)
    met = ref_metrics.calculate_metrics(torch.sigmoid(out), t, "bce_dice", {})
    met["loss"].backward()
    met64 = ref_metrics.calculate_metrics(torch.sigmoid(m64(x.double())), t.double(), "bce_dice", {})
    met64["loss"].backward()
    n = sum(p.numel() for p in m.parameters())
    keep = [k for k, p in m.named_parameters()
            if p.numel() <= 4096 or k in ("inc.conv.0.weight", "outc.conv.weight")]
    g64 = dict(m64.named_parameters())
    small = {"grad." + k: np32(p.grad) for k, p in m.named_parameters() if k in keep}
    small.update({"grad64." + k: np32(g64[k].grad) for k in keep})
    norms = {"gnorm." + k: np.float64(p.grad.double().norm()) for k, p in m.named_parameters()}
    bufs = {"buf." + k: v.numpy().copy() for k, v in m.state_dict().items() if "running" in k}
    extra = {}
    if bilinear:   # the reference's own bf16 error on this batch (CPU autocast, same weights): the bf16 bar
        torch.manual_seed(seed)
        mac = ref_unet.UNet(3, 1, bilinear=True).train()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            extra["logits_bf16_autocast"] = np32(mac(x).float())
    save(name, x=np32(x), t=np32(t), logits=np32(out), loss=np32(met["loss"]), iou=np.float64(met["iou"]),
         dice=np.float64(met["dice"]), nparams=np.int64(n), **init, **small, **norms, **bufs,
         **fp64_noise(m, m64), **extra)


def gen_unet():
    """20x20 (odd sizes: ceil-mode pooling 20->10->5->3->2 and both crop branches) and the
    config-1 size 64x64, batch 2.  The 31 M parameters are not stored: the test builds the model
    under the same seed (module tree and init order are the reference's) and checks per-tensor
    init sums first; gradients are stored for the small tensors plus per-tensor norms."""
    _unet_run(6000, (2, 3, 20, 20), "unet_small.npz")
    _unet_run(6001, (2, 3, 64, 64), "unet_cfg1.npz")


def gen_unet_bilinear():
    """UNet(bilinear=True) (nn.Upsample align_corners=True in Up, unet.py:36-37; half-width down4 and
    decoder): 20x20 (ceil-mode pooling and both crop branches) and 64x64, batch 2."""
    _unet_run(6002, (2, 3, 20, 20), "unet_bilinear_small.npz", bilinear=True)
    _unet_run(6003, (2, 3, 64, 64), "unet_bilinear_64.npz", bilinear=True)


# ----------------------------------------------------------------------------------------
# (7) Config 5: full-resolution attention (module, block, small model), gamma != 0.
# ----------------------------------------------------------------------------------------
def gen_fullres():
    fra = _load_models_pkg("unet_dfc_sa_ablation_attention")
    for (C, H) in [(16, 6), (32, 8), (64, 12)]:   # C = 16: q/k width 2 (padded GEMM width)
        torch.manual_seed(7000 + C + H)
        m = fra.FullResolutionAttention(C)
        with torch.no_grad():
            m.gamma.fill_(0.7)
            m.query_conv.weight.mul_(3.0)   # sharper softmax than the default init
            m.key_conv.weight.mul_(3.0)
        x = torch.randn(2, C, H, H + 1, requires_grad=True)   # non-square map, N = H * (H + 1)
        y = m(x)
        g = torch.randn_like(y)
        y.backward(g)
        save(f"fra_C{C}_H{H}.npz", x=np32(x), g=np32(g), y=np32(y), dx=np32(x.grad), **sd_arrays(m),
             **grad_arrays(m))
    for (cin, cout, H) in [(8, 32, 10), (16, 16, 8)]:   # (16, 16): identity residual
        torch.manual_seed(7100 + cin + cout + H)
        blk = fra.FullResAttnDFCBlock(cin, cout)
        with torch.no_grad():
            blk.attn_branch[3].gamma.fill_(0.7)
        sd0 = sd_arrays(blk, "sd0.")
        blk.train()
        x = torch.randn(2, cin, H, H, requires_grad=True)
        y = blk(x)
        g = torch.randn_like(y)
        y.backward(g)
        save(f"frablock_{cin}to{cout}_H{H}.npz", x=np32(x), g=np32(g), y=np32(y), dx=np32(x.grad), **sd0,
             **sd_arrays(blk, "sd1."), **grad_arrays(blk))
    torch.manual_seed(7200)
    model = fra.UNet_FullResAttention(3, 1, [8, 16, 32, 64])
    perturb_gammas(model)
    sd0 = sd_arrays(model, "sd0.")
    model.train()
    m64 = fp64_twin(model)
    gen = torch.Generator().manual_seed(7201)
    x, t = batch(gen, (2, 3, 32, 32))   # 32x32: the 2x2 bottleneck gives BatchNorm 8 samples per channel
    out = model(x)
    met = ref_metrics.calculate_metrics(torch.sigmoid(out), t, "bce_dice", LOSS_PARAMS)
    met["loss"].backward()
    met64 = ref_metrics.calculate_metrics(torch.sigmoid(m64(x.double())), t.double(), "bce_dice", LOSS_PARAMS)
    met64["loss"].backward()
    save("fullres_model.npz", x=np32(x), t=np32(t), logits=np32(out), loss=np32(met["loss"]),
         iou=np.float64(met["iou"]), dice=np.float64(met["dice"]), **sd0, **grad_arrays(model),
         **fp64_noise(model, m64), **grad_arrays(m64, "grad64."))


# ----------------------------------------------------------------------------------------
# (8) Config 4: TransUNet (R50-ViT hybrid) on a reduced configuration of the reference's own
#     get_r50_b16_config (same code paths: StdConv2d + GroupNorm bottlenecks with stride-2 and
#     projection units, ViT blocks, DecoderCup with concat skips of unequal widths, 3x3 head).
#     ml_collections is not installed: a dict-with-attributes stand-in provides ConfigDict.
#     Dropout p = 0 (the masks are random; the GPU tests check the dropout kernels separately).
# ----------------------------------------------------------------------------------------
TRANSUNET_SMALL = dict(img=32, num_layers=(2, 2, 1), width_factor=0.5, hidden=32, mlp=64, heads=2, layers=2,
                       decoder=(16, 16, 8, 8), skip=[256, 128, 32, 8])


def _transunet_module():
    import types

    class ConfigDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    if "ml_collections" not in sys.modules:
        mlc = types.ModuleType("ml_collections")
        mlc.ConfigDict = ConfigDict
        sys.modules["ml_collections"] = mlc
    return _load("ref_transformer_unet", "models/transformer_unet.py")


def gen_transunet():
    tu = _transunet_module()
    c = TRANSUNET_SMALL
    cfg = tu.get_r50_b16_config()
    cfg.patches.grid = (c["img"] // 16, c["img"] // 16)
    cfg.resnet.num_layers = c["num_layers"]
    cfg.resnet.width_factor = c["width_factor"]
    cfg.hidden_size = c["hidden"]
    cfg.transformer.mlp_dim = c["mlp"]
    cfg.transformer.num_heads = c["heads"]
    cfg.transformer.num_layers = c["layers"]
    cfg.transformer.dropout_rate = 0.0
    cfg.transformer.attention_dropout_rate = 0.0
    cfg.decoder_channels = c["decoder"]
    cfg.skip_channels = list(c["skip"])
    cfg.n_classes = 1
    torch.manual_seed(7500)
    model = tu.TransUNet(cfg, img_size=c["img"], num_classes=1)
    with torch.no_grad():   # zero-initialised in the reference; random here so it is exercised
        model.transformer.embeddings.position_embeddings.normal_(0.0, 0.05)
    sd0 = sd_arrays(model, "sd0.")
    model.train()
    m64 = fp64_twin(model)
    gen = torch.Generator().manual_seed(7501)
    x, t = batch(gen, (2, 3, c["img"], c["img"]))
    out = model(x)
    met = ref_metrics.calculate_metrics(torch.sigmoid(out), t, "bce_dice", LOSS_PARAMS)
    met["loss"].backward()
    met64 = ref_metrics.calculate_metrics(torch.sigmoid(m64(x.double())), t.double(), "bce_dice", LOSS_PARAMS)
    met64["loss"].backward()
    bufs = {"buf." + k: v.detach().numpy().copy() for k, v in model.state_dict().items() if "running" in k}
    m_ac = tu.TransUNet(cfg, img_size=c["img"], num_classes=1)
    m_ac.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in sd0.items()})
    m_ac.train()
    cos_ac = bf16_autocast_cosine(m_ac, x, t, LOSS_PARAMS, m64)
    save("transunet_small.npz", bf16_autocast_grad_cos=cos_ac, x=np32(x), t=np32(t), logits=np32(out), loss=np32(met["loss"]),
         iou=np.float64(met["iou"]), dice=np.float64(met["dice"]), **sd0, **bufs, **fp64_noise(model, m64),
         **grad_arrays(m64, "grad64."), nparams_full=np.int64(sum(
             p.numel() for p in tu.TransUNet(_n_classes_1(tu.get_r50_b16_config()), img_size=224,
                                             num_classes=1).parameters())))


def _n_classes_1(cfg):
    cfg.n_classes = 1
    return cfg


# ----------------------------------------------------------------------------------------
# (9) The ablation model zoo (unet_dfc_sa_ablation_branches.py, _fusion.py, _placement.py): every
#     model at features 8..64, pool 4, 32x32 input, one train-mode forward + backward, fp32 and
#     the float64 re-run (grad64.* / noise.*), like fullres_model.npz.
# ----------------------------------------------------------------------------------------
ZOO = ("UNet_Baseline", "UNet_AttentionOnly", "UNet_AdditionFusion", "UNet_ConcatFusion", "UNet_EncoderOnlyDFC",
       "UNet_DecoderOnlyDFC", "UNet_BothStandardConv")


def _zoo_model(name):
    mods = {"UNet_Baseline": "unet_dfc_sa_ablation_branches", "UNet_AttentionOnly": "unet_dfc_sa_ablation_branches",
            "UNet_AdditionFusion": "unet_dfc_sa_ablation_fusion", "UNet_ConcatFusion": "unet_dfc_sa_ablation_fusion",
            "UNet_EncoderOnlyDFC": "unet_dfc_sa_ablation_placement",
            "UNet_DecoderOnlyDFC": "unet_dfc_sa_ablation_placement",
            "UNet_BothStandardConv": "unet_dfc_sa_ablation_placement"}
    cls = getattr(_load_models_pkg(mods[name]), name)
    if name in ("UNet_Baseline", "UNet_BothStandardConv"):   # model_factory.py:162-187 argument lists
        return cls(3, 1, [8, 16, 32, 64])
    return cls(3, 1, [8, 16, 32, 64], 4)


def gen_transunet_edges():
    """Reference behaviour off the shipped TransUNet configuration (VERDICT r4 "missing" 1-2):
    (a) patch size 2 (img = 2 x 16 x grid): the reference constructs the model, then its forward
    raises at the position-embedding add -> transunet_patch2_error.json (exception type, message,
    patch kernel, position-embedding shape);
    (b) SegmentationHead(upsampling = 2, 3) standalone: conv 3x3 + UpsamplingBilinear2d on a
    seeded input, forward and input/weight gradients of sum(out * w) -> seghead_up.npz."""
    import json
    tu = _transunet_module()
    c = TRANSUNET_SMALL
    cfg = tu.get_r50_b16_config()
    img = 2 * c["img"]
    cfg.patches.grid = (c["img"] // 16, c["img"] // 16)
    cfg.resnet.num_layers = c["num_layers"]
    cfg.resnet.width_factor = c["width_factor"]
    cfg.hidden_size = c["hidden"]
    cfg.transformer.mlp_dim = c["mlp"]
    cfg.transformer.num_heads = c["heads"]
    cfg.transformer.num_layers = c["layers"]
    cfg.decoder_channels = c["decoder"]
    cfg.skip_channels = list(c["skip"])
    cfg.n_classes = 1
    torch.manual_seed(7500)
    model = tu.TransUNet(cfg, img_size=img, num_classes=1)
    e = model.transformer.embeddings
    rec = {"img": img, "grid": list(cfg.patches.grid), "patch_kernel": list(e.patch_embeddings.kernel_size),
           "position_embeddings": list(e.position_embeddings.shape), "config": dict(c)}
    try:
        with torch.no_grad():
            model(torch.randn(1, 3, img, img))
        rec["raised"] = None
    except Exception as ex:   # the reference's own failure, recorded as data
        rec["raised"] = {"type": type(ex).__name__, "message": str(ex)}
    with open(os.path.join(OUT, "transunet_patch2_error.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print("patch2:", rec["raised"])
    arrays = {}
    for up in (2, 3):
        torch.manual_seed(7600 + up)
        head = tu.SegmentationHead(16, 2, kernel_size=3, upsampling=up)
        x = torch.randn(2, 16, 7, 9, requires_grad=True)
        out = head(x)
        w = torch.randn(out.shape)
        (out * w).sum().backward()
        arrays.update({f"up{up}_x": np32(x), f"up{up}_w": np32(w), f"up{up}_conv_w": np32(head[0].weight),
                       f"up{up}_conv_b": np32(head[0].bias), f"up{up}_out": np32(out), f"up{up}_dx": np32(x.grad),
                       f"up{up}_dconv_w": np32(head[0].weight.grad), f"up{up}_dconv_b": np32(head[0].bias.grad)})
    save("seghead_up.npz", **arrays)


def gen_zoo():
    for i, name in enumerate(ZOO):
        torch.manual_seed(9100 + i)
        model = _zoo_model(name)
        perturb_gammas(model)
        sd0 = sd_arrays(model, "sd0.")
        model.train()
        m64 = fp64_twin(model)
        gen = torch.Generator().manual_seed(9200 + i)
        x, t = batch(gen, (2, 3, 32, 32))
        out = model(x)
        met = ref_metrics.calculate_metrics(torch.sigmoid(out), t, "bce_dice", LOSS_PARAMS)
        met["loss"].backward()
        met64 = ref_metrics.calculate_metrics(torch.sigmoid(m64(x.double())), t.double(), "bce_dice", LOSS_PARAMS)
        met64["loss"].backward()
        bufs = {"buf." + k: v.detach().numpy().copy() for k, v in model.state_dict().items() if "running" in k}
        save(f"zoo_{name}.npz", x=np32(x), t=np32(t), logits=np32(out), loss=np32(met["loss"]),
             iou=np.float64(met["iou"]), dice=np.float64(met["dice"]), **sd0, **bufs, **grad_arrays(model),
             **fp64_noise(model, m64), **grad_arrays(m64, "grad64."), nparams_full=np.int64(sum(p.numel() for p in _zoo_full(name).parameters())))


# ----------------------------------------------------------------------------------------
# (9b) Feature widths that are not multiples of 8 (VERDICT r4 missing 3): the reference at
#      features 10, 12, 20, 27 (padded internally to 16, 16, 24, 32; bottleneck 54 -> 56; attention
#      q/k widths 1, 1, 2, 3, 6 -> 8), pool 4, 32x32, batch 2: the initial gammas under the seed
#      (initg.*: every other entry of the fresh state dict is sd0.*), then gammas perturbed (sd0.*),
#      one train-mode forward + backward re-run in float64 (grad64.*, stored fp32; noise.* = the
#      fp32 run's distance to it), and one reference train step (clip 1.0 + SGD lr 0.05, momentum
#      0.9, wd 1e-4): the momentum buffers mom1.* (the new parameters are sd0 - 0.05 mom1).
# ----------------------------------------------------------------------------------------
ODD_FEATURES = [10, 12, 20, 27]
ODD = ("UNetDFCSARes", "UNet_ConcatFusion", "UNet_DecoderOnlyDFC", "UNet_FullResAttention", "UNet_AttentionOnly")


def _odd_model(name):
    if name == "UNetDFCSARes":
        return ref_res.UNetDFCSARes(3, 1, ODD_FEATURES, pool_size=4, ablation_on_qk_channels=8)
    if name == "UNet_FullResAttention":
        return _load_models_pkg("unet_dfc_sa_ablation_attention").UNet_FullResAttention(3, 1, ODD_FEATURES)
    mods = {"UNet_ConcatFusion": "unet_dfc_sa_ablation_fusion", "UNet_DecoderOnlyDFC": "unet_dfc_sa_ablation_placement",
            "UNet_AttentionOnly": "unet_dfc_sa_ablation_branches"}
    return getattr(_load_models_pkg(mods[name]), name)(3, 1, ODD_FEATURES, 4)


def gen_oddwidth():
    for i, name in enumerate(ODD):
        torch.manual_seed(9500 + i)
        model = _odd_model(name)
        initg = {"initg." + k: v.detach().numpy().copy() for k, v in model.state_dict().items() if k.endswith("gamma")}
        perturb_gammas(model)
        sd0 = sd_arrays(model, "sd0.")
        model.train()
        m64 = fp64_twin(model)
        gen = torch.Generator().manual_seed(9600 + i)
        x, t = batch(gen, (2, 3, 32, 32))
        opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        opt.zero_grad()   # utils/trainer.py:120-151, with the pre-clip gradients recorded
        out = model(x)
        met = ref_metrics.calculate_metrics(torch.sigmoid(out), t, "bce_dice", LOSS_PARAMS)
        met["loss"].backward()
        met64 = ref_metrics.calculate_metrics(torch.sigmoid(m64(x.double())), t.double(), "bce_dice", LOSS_PARAMS)
        met64["loss"].backward()
        noise = fp64_noise(model, m64)
        bufs = {"buf." + k: v.detach().numpy().copy() for k, v in model.state_dict().items() if "running" in k}
        norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        opt.step()
        mom = {"mom1." + n: np32(opt.state[p]["momentum_buffer"]) for n, p in model.named_parameters()}
        save(f"oddw_{name}.npz", x=np32(x), t=np32(t), logits=np32(out), loss=np32(met["loss"]),
             iou=np.float64(met["iou"]), dice=np.float64(met["dice"]), norm=np.float64(float(norm)), **initg, **sd0,
             **bufs, **noise, **grad_arrays(m64, "grad64."), **mom)


def gen_oddwidth_standalone():
    """LightSelfAttention / DynamicFusionConvAttnBlock built ON THEIR OWN at widths that are not
    multiples of 8 (reference :5-116 accepts any): the initial state dict under a seed (the build's
    construction must consume the RNG identically), one train-mode forward + backward in fp32 and
    the same run in float64 (grad64.*, the gradient reference; noise.* = the fp32 run's distance)."""
    for C, H, P in ((12, 17, 4), (20, 13, 8), (27, 9, 16)):
        torch.manual_seed(9700 + C)
        m = ref_res.LightSelfAttention(C, pool_size=P, ablation_on_qk_channels=8)
        sd0 = sd_arrays(m, "sd0.")
        with torch.no_grad():
            m.gamma.fill_(0.6)
        m64 = fp64_twin(m)
        gen = torch.Generator().manual_seed(9800 + C)
        x = torch.randn(2, C, H, H + 2, generator=gen)
        g = torch.randn(2, C, H, H + 2, generator=gen)
        xr = x.clone().requires_grad_(True)
        y = m(xr)
        y.backward(g)
        x64 = x.double().requires_grad_(True)
        y64 = m64(x64)
        y64.backward(g.double())
        save(f"oddw_lsa_C{C}_P{P}.npz", x=np32(x), g=np32(g), y=np32(y), dx=np32(xr.grad), y64=y64.detach().numpy(),
             dx64=x64.grad.numpy(), **sd0, **grad_arrays(m64, "grad64."), **fp64_noise(m, m64))
    for cin, cout, H, P in ((5, 12, 12, 4), (12, 20, 10, 8), (16, 27, 8, 4)):
        torch.manual_seed(9900 + cin * 10 + cout)
        blk = ref_res.DynamicFusionConvAttnBlock(cin, cout, pool_size=P, ablation_on_qk_channels=8)
        sd0 = sd_arrays(blk, "sd0.")
        with torch.no_grad():
            blk.attn_branch[3].gamma.fill_(0.5)
        blk.train()
        b64 = fp64_twin(blk)
        gen = torch.Generator().manual_seed(9950 + cout)
        x = torch.randn(2, cin, H, H + 1, generator=gen)
        g = torch.randn(2, cout, H, H + 1, generator=gen)
        xr = x.clone().requires_grad_(True)
        y = blk(xr)
        y.backward(g)
        x64 = x.double().requires_grad_(True)
        y64 = b64(x64)
        y64.backward(g.double())
        save(f"oddw_block_{cin}to{cout}_P{P}.npz", x=np32(x), g=np32(g), y=np32(y), dx=np32(xr.grad),
             y64=y64.detach().numpy(), dx64=x64.grad.numpy(), **sd0, **grad_arrays(b64, "grad64."),
             **fp64_noise(blk, b64), **sd_arrays(blk, "sd1."))


def _zoo_full(name):
    m = _zoo_model(name)
    cls = type(m)
    if name in ("UNet_Baseline", "UNet_BothStandardConv"):
        return cls(3, 1, [64, 128, 256, 512])
    return cls(3, 1, [64, 128, 256, 512], 8)


# ----------------------------------------------------------------------------------------
# Sliding-window inference (inference.py:73-153).  The module itself imports cv2, matplotlib
# and torchvision, none of which is installed here, so only the two functions under test are
# taken from its source (ast) and run with the reference's own code.  torchvision's ToTensor /
# Normalize, the only torchvision pieces they use, are restated below with torchvision's
# arithmetic (uint8 -> float / 255; (x - mean) / std).  The "model" is a fixed 3x3 conv.
# ----------------------------------------------------------------------------------------
def _reference_inference_functions():
    import ast
    import types

    from PIL import Image
    from tqdm import tqdm

    class Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, x):
            for t in self.ts:
                x = t(x)
            return x

    class ToTensor:
        def __call__(self, pic):
            a = torch.from_numpy(np.array(pic, dtype=np.uint8, copy=True))
            return a.permute(2, 0, 1).contiguous().float().div(255)

    class Normalize:
        def __init__(self, mean, std):
            self.mean, self.std = mean, std

        def __call__(self, t):
            m = torch.as_tensor(self.mean, dtype=t.dtype).view(-1, 1, 1)
            s = torch.as_tensor(self.std, dtype=t.dtype).view(-1, 1, 1)
            return t.sub(m).div(s)

    transforms = types.SimpleNamespace(Compose=Compose, ToTensor=ToTensor, Normalize=Normalize)
    src = open(os.path.join(REF, "inference.py"), encoding="utf-8").read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef)
            and n.name in ("calculate_segmentation_metrics", "predict_large_image")]
    ns = {"np": np, "torch": torch, "Image": Image, "transforms": transforms, "tqdm": tqdm}
    exec(compile(ast.Module(body=keep, type_ignores=[]), "reference/inference.py", "exec"), ns)
    return ns["predict_large_image"], ns["calculate_segmentation_metrics"]


def gen_inference():
    predict_large_image, calc_counts = _reference_inference_functions()
    torch.manual_seed(9000)
    conv = torch.nn.Conv2d(3, 1, 3, padding=1)
    with torch.no_grad():
        conv.weight.mul_(3.0)
    g = np.random.default_rng(9001)
    cases = {"a": ((150, 230), 64, 20), "b": ((40, 50), 64, 20), "c": ((128, 128), 64, 0), "d": ((97, 301), 48, 10)}
    out = {"conv.weight": np32(conv.weight), "conv.bias": np32(conv.bias)}
    for name, ((h, w), tile, overlap) in cases.items():
        img = g.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        out[f"{name}.image"] = img
        out[f"{name}.cfg"] = np.array([tile, overlap], dtype=np.int64)
        for tta in (False, True):
            out[f"{name}.canvas.tta{int(tta)}"] = predict_large_image(conv, img, tile, overlap, "cpu", use_tta=tta)
        gt = g.integers(0, 2, size=(h, w), dtype=np.uint8) * 255
        out[f"{name}.gt"] = gt
        c = calc_counts((out[f"{name}.canvas.tta0"] > 0.5).astype(np.uint8), (gt > 128).astype(np.uint8))
        out[f"{name}.counts"] = np.array([c["tp"], c["fp"], c["fn"], c["tn"]], dtype=np.int64)
    save("inference.npz", **out)


# ----------------------------------------------------------------------------------------
# (11) bf16 calibration: what PyTorch's own bf16 autocast does to the reference's logits, loss and
#      metrics on the small model (sd0 of model_small.npz) over the fixture batch and 5 seeded
#      batches.  The GPU tests hold the build's bf16 mode to max(1e-2, this error) per batch.
# ----------------------------------------------------------------------------------------
def _autocast_errors(model, x, t):
    import copy
    with torch.no_grad():
        o32 = copy.deepcopy(model)(x)
        m64 = fp64_twin(model)
        o64 = m64(x.double())
        with torch.autocast("cpu", dtype=torch.bfloat16):
            ob = copy.deepcopy(model)(x)
    ob = ob.float()
    a = ref_metrics.calculate_metrics(torch.sigmoid(o32), t, "bce_dice", {})
    b = ref_metrics.calculate_metrics(torch.sigmoid(ob), t, "bce_dice", {})
    rel = lambda u, v: np.float64(((u.double() - v.double()).norm() / v.double().norm()).item())  # noqa: E731
    return o32, a, {"ac_logits_rel": rel(ob, o32), "ac_logits_rel64": rel(ob, o64),
                    "ac_loss_rel": np.float64(abs(b["loss"].item() - a["loss"].item()) / abs(a["loss"].item())),
                    "ac_iou": np.float64(b["iou"]), "ac_dice": np.float64(b["dice"])}


def gen_bf16calib():
    fx = dict(np.load(os.path.join(OUT, "model_small.npz")))
    model = base_model(4)
    model.train()
    out = {}
    batches = [("x1", torch.from_numpy(fx["x1"]), torch.from_numpy(fx["t1"]))]
    for s in range(5):
        gen = torch.Generator().manual_seed(11000 + s)
        batches.append((f"s{s}",) + batch(gen, (2, 3, 32, 32)))
    for tag, x, t in batches:
        o32, met, e = _autocast_errors(model, x, t)
        out.update({f"{tag}.x": np32(x), f"{tag}.t": np32(t), f"{tag}.logits": np32(o32),
                    f"{tag}.loss": np32(met["loss"]), f"{tag}.iou": np.float64(met["iou"]),
                    f"{tag}.dice": np.float64(met["dice"])})
        out.update({f"{tag}.{k}": v for k, v in e.items()})
        print(tag, {k: float(v) for k, v in e.items()})
    save("bf16_calib.npz", tags=np.array([b[0] for b in batches]), **out)


# ----------------------------------------------------------------------------------------
# (12) Config-2 geometry: DFC-SA-Res features 64..512, P = 4, 224 x 224, batch 2, gammas 0.5,
#      one reference train step (fwd, sigmoid, bce_dice, backward, clip 1.0, SGD).  The 29 M
#      parameters are not stored: the test builds the model under the same seed (same module tree
#      and creation order) and checks the per-tensor init sums first.  Stored: logits, loss, IoU,
#      Dice, pre-clip per-tensor gradient norms (+ float64 run and the fp32-vs-fp64 noise), the full
#      gradients of the small tensors, the total norm, the BN running stats after the step, the
#      per-tensor norms of the SGD update, and the autocast bf16 calibration at this geometry.
# ----------------------------------------------------------------------------------------
def gen_cfg2():
    torch.manual_seed(12000)
    m = ref_res.UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4, ablation_on_qk_channels=8)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    init = {"init_sum." + k: np.float64(v.double().sum()) for k, v in m.state_dict().items() if v.is_floating_point()}
    m.train()
    gen = torch.Generator().manual_seed(12001)
    x, t = batch(gen, (2, 3, 224, 224))
    _, _, calib = _autocast_errors(m, x, t)
    print("cfg2 autocast", {k: float(v) for k, v in calib.items()})
    m64 = fp64_twin(m)
    w0 = {n: p.detach().clone() for n, p in m.named_parameters()}
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    opt.zero_grad()
    out = m(x)
    met = ref_metrics.calculate_metrics(torch.sigmoid(out), t, "bce_dice", LOSS_PARAMS)
    met["loss"].backward()
    met64 = ref_metrics.calculate_metrics(torch.sigmoid(m64(x.double())), t.double(), "bce_dice", LOSS_PARAMS)
    met64["loss"].backward()
    gnorm = {"gnorm." + n: np.float64(p.grad.double().norm()) for n, p in m.named_parameters()}
    g64 = dict(m64.named_parameters())
    gnorm64 = {"gnorm64." + n: np.float64(g64[n].grad.norm()) for n, _ in m.named_parameters()}
    small = {"grad." + n: np32(p.grad) for n, p in m.named_parameters() if p.numel() <= 4096}
    small.update({"grad64." + n: np32(g64[n].grad) for n, p in m.named_parameters() if p.numel() <= 4096})
    noise = fp64_noise(m, m64)
    norm = torch.nn.utils.clip_grad_norm_(m.parameters(), max_norm=1.0)
    opt.step()
    upd = {"dnorm." + n: np.float64((p.detach().double() - w0[n].double()).norm()) for n, p in m.named_parameters()}
    bufs = {"buf." + k: v.numpy().copy() for k, v in m.state_dict().items() if "running" in k}
    save("cfg2_step.npz", x=np32(x), t=np32(t), logits=np32(out), loss=np32(met["loss"]),
         iou=np.float64(met["iou"]), dice=np.float64(met["dice"]), norm=np32(norm),
         nparams=np.int64(sum(p.numel() for p in m.parameters())), **init, **gnorm, **gnorm64, **small, **noise,
         **upd, **bufs, **{"calib." + k: v for k, v in calib.items()})


# ----------------------------------------------------------------------------------------
# (12b) bf16 BACKWARD calibration at the config-2 geometry (the benchmark path's dtype): the same
#      model and batch as (12), one reference train step run three ways -- float64 (the truth), the
#      reference under PyTorch's CPU bf16 autocast (what bf16 arithmetic alone does to it), and
#      fp32 (cfg2_step.npz).  Stored per parameter tensor: the autocast gradient's cosine and
#      relative distance to float64 (pre-clip), the relative distance of the autocast SGD update
#      (clip 1.0 + SGD) to the float64 update, and per BN buffer the autocast running statistics'
#      distance to float64's after the step.  The GPU test holds the build's bf16 step to these
#      (utils/trainer.py:120-151, train.py:73-78).
# ----------------------------------------------------------------------------------------
def _bf16_step_fixture(fname, pool, seed, bseed, extra=False, B=2, store_xt=True):
    import copy
    import gc
    torch.manual_seed(seed)
    m = ref_res.UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=pool, ablation_on_qk_channels=8)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    init = {"init_sum." + k: np.float64(v.double().sum()) for k, v in m.state_dict().items() if v.is_floating_point()}
    m.train()
    gen = torch.Generator().manual_seed(bseed)
    x, t = batch(gen, (B, 3, 224, 224))

    def step(model, xx, tt, autocast):
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        w0 = {n: p.detach().clone() for n, p in model.named_parameters()}
        opt.zero_grad()
        if autocast:
            with torch.autocast("cpu", dtype=torch.bfloat16):
                out = model(xx)
            out = out.float()
        else:
            out = model(xx)
        met = ref_metrics.calculate_metrics(torch.sigmoid(out), tt, "bce_dice", LOSS_PARAMS)
        met["loss"].backward()
        g = {n: p.grad.detach().double().clone() for n, p in model.named_parameters()}
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        opt.step()
        upd = {n: (p.detach().double() - w0[n].double()) for n, p in model.named_parameters()}
        bufs = {k: v.detach().double().clone() for k, v in model.state_dict().items() if "running" in k}
        return g, upd, bufs, out.detach(), met

    m64 = fp64_twin(m)
    g64, u64, b64, o64, _ = step(m64, x.double(), t.double(), False)
    del m64
    gc.collect()
    mac = copy.deepcopy(m)
    gac, uac, bac, oac, _ = step(mac, x, t, True)
    del mac
    gc.collect()
    reln = lambda a, b: np.float64(((a - b).norm() / (b.norm() + 1e-30)).item())  # noqa: E731
    out = {}
    for n in g64:
        a, b = gac[n].reshape(-1), g64[n].reshape(-1)
        out["ac_cos." + n] = np.float64((a @ b / (a.norm() * b.norm() + 1e-300)).item())
        out["ac_rel." + n] = reln(a, b)
        out["ac_upd_rel." + n] = reln(uac[n], u64[n])
        out["gnorm64." + n] = np.float64(b.norm().item())
    for k in b64:
        out["ac_buf_rel." + k] = reln(bac[k], b64[k])
    ga = torch.cat([gac[n].reshape(-1) for n in g64])
    gb = torch.cat([g64[n].reshape(-1) for n in g64])
    out["ac_cos_all"] = np.float64((ga @ gb / (ga.norm() * gb.norm())).item())
    out["ac_rel_all"] = reln(ga, gb)
    if extra:
        # the fp32 reference step on the same weights (the forward bar and the BN buffers after it)
        m32 = copy.deepcopy(m)
        _, _, b32, o32, met32 = step(m32, x, t, False)
        out.update(init)
        if store_xt:
            out["logits"] = np32(o32)
        else:
            # the batch is regenerated by the test from bseed (checksums below); of the logits only
            # the first image and whole-batch checksums are stored (the test's fp32 logits come from
            # the oracle re-run on the box, which these pin to the reference)
            out["logits0"] = np32(o32[0])
            out["logits_sum"] = np.float64(o32.double().sum().item())
            out["logits_norm"] = np.float64(o32.double().norm().item())
        out["loss"] = np32(met32["loss"])
        out["iou"], out["dice"] = np.float64(met32["iou"]), np.float64(met32["dice"])
        out["ac_logits_rel"] = reln(oac.double(), o32.double())
        out["ac_logits_rel64"] = reln(oac.double(), o64.double())
        out.update({"buf." + k: np32(v) for k, v in b32.items()})
        print(fname, "autocast logits rel", float(out["ac_logits_rel"]))
    print(fname, "bf16 autocast: global grad cos", float(out["ac_cos_all"]), "rel", float(out["ac_rel_all"]))
    if store_xt:
        save(fname, x=np32(x), t=np32(t), **out)
    else:
        save(fname, B=np.int64(B), bseed=np.int64(bseed), seed=np.int64(seed), pool=np.int64(pool),
             x_sum=np.float64(x.double().sum().item()), x_sqsum=np.float64((x.double() ** 2).sum().item()),
             t_sum=np.float64(t.double().sum().item()), **out)


def gen_cfg2bf16():
    _bf16_step_fixture("cfg2_bf16.npz", 4, 12000, 12001)


# (12c) Config-3 geometry (config_dfc-sa-res-block.yaml: pool_size 8) at 224^2, 64..512, B = 2 -- the
#       P = 8 path (N = 64 tokens, non-divisible 28 -> 8 and 14 -> 8 pooling windows) of the DDP
#       benchmark: the same three-way step as (12b) from its own seed, plus the fp32 reference's logits,
#       loss / IoU / Dice, BN buffers and the seeded-init checksums.
def gen_cfg3bf16():
    _bf16_step_fixture("cfg3_bf16.npz", 8, 14000, 14001, extra=True)


# (12d) The TIMED configuration itself: 64..512, 224^2, P = 4, B = 16 (bench.py's per-GPU batch), so the
#       GPU test runs every B = 16 route (the mid-M streaming 1x1 GEMMs, the B = 16 weight-gradient split
#       plans and split-K choices) -- the same three-way reference step as (12b) from its own seed.  The
#       batch (39 MB) is not stored: the test regenerates it from bseed with this file's batch() and
#       checks the stored checksums; the fp32 logits are pinned by image 0 and checksums.
def gen_cfg2b16():
    _bf16_step_fixture("cfg2b16_bf16.npz", 4, 16000, 16001, extra=True, B=16, store_xt=False)


# ----------------------------------------------------------------------------------------
# (13) Checkpoint interop: the reference Trainer (utils/trainer.py) trains the small model for one
#      epoch of two batches, validates, and writes its checkpoint with its own save_checkpoint
#      (:267-298; metrics with best/worst samples).  A second reference Trainer loads it with its own
#      load_checkpoint (:300-324) and trains one more epoch on a third batch: the expected loss and
#      parameters after resuming (SGD momentum restored from the checkpoint).
#      utils/visualization.py needs cv2 (absent): the Trainer's plotting imports are stubbed (no
#      plotting is called by train_epoch / validate_epoch / save_checkpoint / load_checkpoint).
# ----------------------------------------------------------------------------------------
def _reference_trainer():
    import types
    if "utils" not in sys.modules or not hasattr(sys.modules["utils"], "_refstub"):
        pkg = types.ModuleType("utils")
        pkg.__path__ = [os.path.join(REF, "utils")]
        pkg._refstub = True
        sys.modules["utils"] = pkg
        sys.modules["utils.metrics"] = ref_metrics
        vis = types.ModuleType("utils.visualization")
        for f in ("save_loss_plot", "save_metrics_plot", "save_prediction_samples"):
            setattr(vis, f, lambda *a, **k: None)
        sys.modules["utils.visualization"] = vis
    return _load("ref_trainer", "utils/trainer.py")


def gen_ckpt():
    import shutil
    import tempfile
    tr_mod = _reference_trainer()
    fx = dict(np.load(os.path.join(OUT, "model_small.npz")))
    gen = torch.Generator().manual_seed(13000)
    x3, t3 = batch(gen, (2, 3, 32, 32))
    batches = [{"image": torch.from_numpy(fx[f"x{s}"]), "mask": torch.from_numpy(fx[f"t{s}"]),
                "filename": [f"a{s}.png", f"b{s}.png"]} for s in (1, 2)]
    b3 = [{"image": x3, "mask": t3, "filename": ["a3.png", "b3.png"]}]
    tmp = tempfile.mkdtemp()
    cfg = {"training": {"num_epochs": 1, "save_checkpoint_freq": 1,
                        "loss": {"type": "bce_dice", "params": LOSS_PARAMS}},
           "logging": {"log_dir": os.path.join(tmp, "logs"), "images_dir": os.path.join(tmp, "img"),
                       "save_best_worst_samples": 1}}
    model = base_model(4)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    tr = tr_mod.Trainer(model, batches, batches[:1], opt, torch.device("cpu"), cfg)
    loss, iou, dice = tr.train_epoch(0)
    tr.train_losses.append(loss)
    tr.train_dice_scores.append(dice)
    tr.train_iou_scores.append(iou)
    val = tr.validate_epoch(batches[:1])
    tr.val_losses.append(val["loss"])
    tr.val_dice_scores.append(val["dice"])
    tr.val_iou_scores.append(val["iou"])
    tr.epochs.append(1)
    tr.save_checkpoint(0, val, is_best=True)
    src = os.path.join(tmp, "logs", "checkpoints", "checkpoint_epoch_1.pth")
    shutil.copy(src, os.path.join(OUT, "ref_checkpoint_epoch_1.pth"))
    # resume with the reference's own loader, one more epoch on batch 3
    model2 = ref_res.UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, ablation_on_qk_channels=8)
    opt2 = torch.optim.SGD(model2.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    tr2 = tr_mod.Trainer(model2, b3, b3, opt2, torch.device("cpu"), cfg)
    ep = tr2.load_checkpoint(src)
    loss3, iou3, dice3 = tr2.train_epoch(ep + 1)
    save("ref_checkpoint_resume.npz", epoch=np.int64(ep), x3=np32(x3), t3=np32(t3), loss3=np.float64(loss3),
         iou3=np.float64(iou3), dice3=np.float64(dice3), train_loss1=np.float64(loss), val_dice1=np.float64(val["dice"]),
         **sd_arrays(model2, "sd3."))
    shutil.rmtree(tmp)


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["lsa", "block", "model", "metrics", "ddp", "unet", "unet_bilinear", "fullres", "transunet", "inference", "zoo",
                             "bf16calib", "cfg2", "ckpt"]
    for w in which:
        globals()["gen_" + w]()
    print("torch", torch.__version__)
