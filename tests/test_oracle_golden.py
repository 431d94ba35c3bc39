"""Pin the CPU oracle (oracle/dfcsa_oracle.py) against golden vectors produced by running the
reference implementation itself (tests/golden/make_golden.py).  CPU only."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import dfcsa_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def T(a):
    return torch.from_numpy(np.asarray(a))


def sd_from(fx, prefix):
    return {k[len(prefix):]: T(v) for k, v in fx.items() if k.startswith(prefix)}


def close(a, b, rtol=1e-5, atol=1e-5):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, np.asarray(b), rtol=rtol, atol=atol)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "lsa_*.npz"))),
                         ids=os.path.basename)
def test_lsa(path):
    fx = dict(np.load(path))
    P = int(os.path.basename(path).split("_P")[1].split(".")[0])
    sd = {k[3:]: T(v).requires_grad_(True) for k, v in fx.items() if k.startswith("sd.")}
    x = T(fx["x"]).requires_grad_(True)
    sdp = {"m." + k: v for k, v in sd.items()}
    y = O.light_self_attention(x, sdp, "m", P)
    close(y, fx["y"])
    y.backward(T(fx["g"]))
    close(x.grad, fx["dx"], rtol=1e-4, atol=1e-5)
    for k in sd:
        close(sd[k].grad, fx["grad." + k], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "block_*.npz"))),
                         ids=os.path.basename)
def test_block(path):
    fx = dict(np.load(path))
    P = int(os.path.basename(path).split("_P")[1].split(".")[0])
    sd0 = {"b." + k: v for k, v in sd_from(fx, "sd0.").items()}
    params = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v)
              for k, v in sd0.items()}
    x = T(fx["x"]).requires_grad_(True)
    bufs = {}
    y = O.dfc_block(x, params, "b", P, True, bufs)
    close(y, fx["y"], rtol=1e-4, atol=1e-5)
    y.backward(T(fx["g"]))
    close(x.grad, fx["dx"], rtol=1e-4, atol=1e-4)
    for k, v in fx.items():
        if k.startswith("grad."):
            close(params["b." + k[5:]].grad, v, rtol=1e-3, atol=1e-4)
        if k.startswith("sd1.") and ("running" in k or "num_batches" in k):
            close(bufs["b." + k[4:]], v, rtol=1e-5, atol=1e-6)


def test_model_two_steps():
    fx = dict(np.load(os.path.join(GOLDEN, "model_small.npz")))
    sd = sd_from(fx, "sd0.")
    lp = {"bce_weight": 0.5, "dice_weight": 0.5}
    sd1, bufs, m1 = O.train_step(sd, {}, T(fx["x1"]), T(fx["t1"]), 4, lp)
    close(m1["logits"], fx["logits1"], rtol=1e-4, atol=1e-5)
    close(m1["loss"], fx["loss1"], rtol=1e-5, atol=1e-6)
    assert abs(m1["iou"] - fx["iou1"]) < 1e-6 and abs(m1["dice"] - fx["dice1"]) < 1e-6
    close(m1["norm"], fx["norm1"], rtol=1e-4)
    for k in O.param_names(sd):
        close(m1["grads"][k], fx["step1.grad." + k], rtol=1e-3, atol=1e-5)
    for k, v in fx.items():
        if k.startswith("bn1."):
            close(sd1[k[4:]], v, rtol=1e-5, atol=1e-6)
    sd2, bufs, m2 = O.train_step(sd1, bufs, T(fx["x2"]), T(fx["t2"]), 4, lp)
    close(m2["loss"], fx["loss2"], rtol=1e-4, atol=1e-6)
    for k in sd:
        close(sd2[k], fx["sd2." + k], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name,P", [("model_p8.npz", 8), ("model_odd36.npz", 4)])
def test_model_grads(name, P):
    base = dict(np.load(os.path.join(GOLDEN, "model_small.npz")))
    sd = sd_from(base, "sd0.")
    fx = dict(np.load(os.path.join(GOLDEN, name)))
    x = T(fx["x"]) if "x" in fx else T(base["x1"])
    t = T(fx["t"]) if "t" in fx else T(base["t1"])
    logits, met, grads, _ = O.forward_backward(sd, x, t, P, {"bce_weight": 0.5})
    close(logits, fx["logits"], rtol=1e-4, atol=1e-5)
    close(met["loss"], fx["loss"], rtol=1e-5)
    for k in O.param_names(sd):
        close(grads[k], fx["grad." + k], rtol=1e-3, atol=1e-5)


def test_model_eval():
    base = dict(np.load(os.path.join(GOLDEN, "model_small.npz")))
    sd = sd_from(base, "sd0.")
    fx = dict(np.load(os.path.join(GOLDEN, "model_eval.npz")))
    sd.update(sd_from(fx, "buf."))
    with torch.no_grad():
        y = O.unet_dfc_sa_res(T(fx["x"]), sd, 4, training=False)
    close(y, fx["logits"], rtol=1e-4, atol=1e-5)


def test_metrics():
    fx = dict(np.load(os.path.join(GOLDEN, "metrics_bce_dice.npz")))
    cases = sorted({k.split(".")[0] for k in fx})
    for c in cases:
        p = T(fx[c + ".p"]).requires_grad_(True)
        params = {"weight_bce": float(fx[c + ".wbce"]), "weight_dice": float(fx[c + ".wdice"])}
        m = O.calculate_metrics(p, T(fx[c + ".t"]), "bce_dice", params)
        close(m["loss"], fx[c + ".loss"], rtol=1e-6)
        assert abs(m["iou"] - fx[c + ".iou"]) < 1e-9 and abs(m["dice"] - fx[c + ".dice"]) < 1e-9
        m["loss"].backward()
        close(p.grad, fx[c + ".dp"], rtol=1e-5, atol=1e-7)


def test_metrics_dice_type():
    """The reference's 'dice' loss type (metrics_dice.npz: p at exactly 0 / 1, an empty mask)."""
    fx = dict(np.load(os.path.join(GOLDEN, "metrics_dice.npz")))
    for c in sorted({k.split(".")[0] for k in fx}):
        p = T(fx[c + ".p"]).requires_grad_(True)
        m = O.calculate_metrics(p, T(fx[c + ".t"]), "dice", {})
        close(m["loss"], fx[c + ".loss"], rtol=1e-6)
        assert abs(m["iou"] - fx[c + ".iou"]) < 1e-9 and abs(m["dice"] - fx[c + ".dice"]) < 1e-9
        m["loss"].backward()
        close(p.grad, fx[c + ".dp"], rtol=1e-5, atol=1e-7)


def test_ddp_shard_means():
    base = dict(np.load(os.path.join(GOLDEN, "model_small.npz")))
    sd = sd_from(base, "sd0.")
    fx = dict(np.load(os.path.join(GOLDEN, "ddp_shards.npz")))
    x, t = T(fx["x"]), T(fx["t"])
    for world in (2, 4):
        per = x.shape[0] // world
        acc = None
        for r in range(world):
            _, _, g, _ = O.forward_backward(sd, x[r * per:(r + 1) * per], t[r * per:(r + 1) * per], 4)
            acc = g if acc is None else {k: acc[k] + g[k] for k in acc}
        for k in acc:
            close(acc[k] / world, fx[f"w{world}.mean_grad.{k}"], rtol=1e-3, atol=1e-5)


# ----------------------------------------------------------------------------- config 5 / config 1
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "fra_*.npz"))), ids=os.path.basename)
def test_full_resolution_attention(path):
    fx = dict(np.load(path))
    sd = {k[3:]: T(v).requires_grad_(True) for k, v in fx.items() if k.startswith("sd.")}
    x = T(fx["x"]).requires_grad_(True)
    y = O.full_resolution_attention(x, {"m." + k: v for k, v in sd.items()}, "m")
    close(y, fx["y"], rtol=1e-4, atol=1e-5)
    y.backward(T(fx["g"]))
    close(x.grad, fx["dx"], rtol=1e-4, atol=1e-4)
    for k in sd:
        close(sd[k].grad, fx["grad." + k], rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "frablock_*.npz"))), ids=os.path.basename)
def test_full_res_block(path):
    fx = dict(np.load(path))
    sd0 = {"b." + k: v for k, v in sd_from(fx, "sd0.").items()}
    params = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v)
              for k, v in sd0.items()}
    x = T(fx["x"]).requires_grad_(True)
    bufs = {}
    y = O.dfc_block(x, params, "b", 0, True, bufs, full_res=True)
    close(y, fx["y"], rtol=1e-4, atol=1e-5)
    y.backward(T(fx["g"]))
    close(x.grad, fx["dx"], rtol=1e-4, atol=1e-4)
    for k, v in fx.items():
        if k.startswith("grad."):
            close(params["b." + k[5:]].grad, v, rtol=1e-3, atol=1e-4)
        if k.startswith("sd1.") and ("running" in k or "num_batches" in k):
            close(bufs["b." + k[4:]], v, rtol=1e-5, atol=1e-6)


def test_full_res_model():
    fx = dict(np.load(os.path.join(GOLDEN, "fullres_model.npz")))
    sd = sd_from(fx, "sd0.")
    logits, met, grads, _ = O.forward_backward(sd, T(fx["x"]), T(fx["t"]), 0, {"bce_weight": 0.5}, model="fullres")
    close(logits, fx["logits"], rtol=1e-4, atol=1e-5)
    close(met["loss"], fx["loss"], rtol=1e-5)
    assert abs(met["dice"] - fx["dice"]) < 1e-9
    for k in O.param_names(sd):
        close(grads[k], fx["grad." + k], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("name,seed,bilinear", [("unet_small.npz", 6000, False), ("unet_cfg1.npz", 6001, False),
                                                ("unet_bilinear_small.npz", 6002, True),
                                                ("unet_bilinear_64.npz", 6003, True)])
def test_unet_oracle_and_seeded_init(name, seed, bilinear):
    """The build's UNet module tree reproduces the reference's seeded initialisation (per-tensor
    sums) and the oracle reproduces the reference's logits, loss, metrics and gradients; bilinear:
    nn.Upsample(align_corners=True) in Up and the half-width decoder (reference unet.py:36-37, 78-88)."""
    from models.unet import UNet
    fx = dict(np.load(os.path.join(GOLDEN, name)))
    torch.manual_seed(seed)
    m = UNet(3, 1, bilinear=bilinear)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    assert sum(p.numel() for p in m.parameters()) == int(fx["nparams"]) == (13395329 if bilinear else 31043521)
    for k, v in sd.items():
        if v.is_floating_point():
            assert abs(v.double().sum().item() - float(fx["init_sum." + k])) <= 1e-9 * max(1.0, abs(float(fx["init_sum." + k]))), k
    logits, met, grads, bufs = O.forward_backward(sd, T(fx["x"]), T(fx["t"]), 0, {}, model="unet")
    close(logits, fx["logits"], rtol=1e-4, atol=1e-5)
    close(met["loss"], fx["loss"], rtol=1e-5)
    assert abs(met["dice"] - fx["dice"]) < 1e-9 and abs(met["iou"] - fx["iou"]) < 1e-9
    for k, g in grads.items():
        ref = float(fx["gnorm." + k])
        assert abs(g.double().norm().item() - ref) <= 1e-3 * ref + 1e-7, k
        if "grad." + k in fx:
            close(g, fx["grad." + k], rtol=1e-3, atol=1e-5 * max(1.0, ref))
    for k, v in bufs.items():
        if "running" in k:
            close(v, fx["buf." + k], rtol=1e-5, atol=1e-6)


def transunet_small_config():
    """The reduced get_r50_b16_config of tests/golden/make_golden.py TRANSUNET_SMALL (32x32 input)."""
    from models.transformer_unet import get_r50_b16_config
    c = get_r50_b16_config()
    c.patches.grid = (2, 2)
    c.resnet.num_layers = (2, 2, 1)
    c.resnet.width_factor = 0.5
    c.hidden_size = 32
    c.transformer.mlp_dim = 64
    c.transformer.num_heads = 2
    c.transformer.num_layers = 2
    c.transformer.dropout_rate = 0.0
    c.decoder_channels = (16, 16, 8, 8)
    c.skip_channels = [256, 128, 32, 8]
    c.n_classes = 1
    return c


def test_transunet_oracle_and_seeded_init():
    """TransUNet (config 4) on the reference's reduced R50-ViT config: the build's module tree
    reproduces the reference's seeded initialisation exactly and the full-size model has the
    reference's 105,275,921 parameters; the oracle reproduces logits / loss / Dice and the float64
    reference gradients within 4x the reference's own fp32 error (min 1e-4), BN running stats."""
    from models.transformer_unet import TransUNet, get_r50_b16_config
    fx = dict(np.load(os.path.join(GOLDEN, "transunet_small.npz")))
    torch.manual_seed(7500)
    m = TransUNet(transunet_small_config(), img_size=32, num_classes=1)
    sd0 = sd_from(fx, "sd0.")
    for k, v in m.state_dict().items():
        if k != "transformer.embeddings.position_embeddings":   # re-drawn by the generator
            assert torch.equal(v, sd0[k]), k
    full = get_r50_b16_config()
    full.n_classes = 1
    assert sum(p.numel() for p in TransUNet(full, 224, 1).parameters()) == 105275921
    logits, met, grads, bufs = O.forward_backward(sd0, T(fx["x"]), T(fx["t"]), 0, {"bce_weight": 0.5},
                                                  model="transunet", heads=2)
    close(logits, fx["logits"], rtol=1e-4, atol=1e-5)
    close(met["loss"], fx["loss"], rtol=1e-5)
    assert abs(met["dice"] - fx["dice"]) < 1e-9
    for k, g in grads.items():
        if k.endswith("attn.key.bias"):      # true gradient 0 (softmax is shift-invariant per query)
            continue
        ref = torch.from_numpy(fx["grad64." + k]).double()
        r = ((g.double() - ref).norm() / (ref.norm() + 1e-30)).item()
        assert r < max(1e-4, 4 * float(fx["noise." + k])), (k, r)
    for k, v in bufs.items():
        if "running" in k:
            close(v, fx["buf." + k], rtol=1e-5, atol=1e-6)


# --------------------------------------------------------------------- sliding-window inference
def test_inference_oracle_matches_reference_predict_large_image(golden):
    """oracle/inference_oracle.py restates inference.py:73-153; the fixture is the reference's own
    predict_large_image (tiles, TTA, overlap averaging) run with a fixed 3x3 conv as the model."""
    from oracle import inference_oracle as IO
    fx = golden("inference.npz")
    conv = torch.nn.Conv2d(3, 1, 3, padding=1)
    conv.weight.data = torch.from_numpy(fx["conv.weight"])
    conv.bias.data = torch.from_numpy(fx["conv.bias"])

    def predict(b):
        with torch.no_grad():
            return conv(torch.from_numpy(np.ascontiguousarray(b))).numpy()

    for name in ("a", "b", "c", "d"):
        img = fx[f"{name}.image"]
        tile, overlap = (int(v) for v in fx[f"{name}.cfg"])
        for tta in (0, 1):
            got = IO.predict_large_image(predict, img, tile, overlap, use_tta=bool(tta))
            want = fx[f"{name}.canvas.tta{tta}"]
            assert got.shape == want.shape and got.dtype == np.float32
            assert np.abs(got - want).max() < 2e-6, (name, tta)
        pb = (fx[f"{name}.canvas.tta0"] > 0.5).astype(np.uint8)
        c = IO.calculate_segmentation_metrics(pb, (fx[f"{name}.gt"] > 128).astype(np.uint8))
        assert [c[k] for k in ("tp", "fp", "fn", "tn")] == fx[f"{name}.counts"].tolist()


def test_inference_tile_grid_matches_oracle_loop():
    """utils.inference.tile_grid (host logic) reproduces the reference loop's tile origins."""
    from utils.inference import tile_grid
    for (h, w, tile, ov) in [(150, 230, 64, 20), (40, 50, 64, 20), (128, 128, 64, 0), (1000, 777, 224, 50),
                             (224, 224, 224, 50), (225, 223, 224, 50)]:
        stride = tile - ov
        want = []
        for y in range(0, h, stride):
            for x in range(0, w, stride):
                ye, xe = min(y + tile, h), min(x + tile, w)
                want.append((max(0, ye - tile), max(0, xe - tile), ye - max(0, ye - tile), xe - max(0, xe - tile)))
        ys, xs, th, tw = tile_grid(h, w, tile, ov)
        assert [(y, x, th, tw) for y in ys for x in xs] == want
    with pytest.raises(ValueError):
        tile_grid(10, 10, 50, 50)


# --------------------------------------------------------------------- paired transforms
def test_augment_restatement_matches_pillow():
    """oracle/augment_oracle.py's restatement of Pillow's Resample.c / Geometry.c arithmetic (what the
    dfcsa_aug_* kernels implement) is bit-exact with Pillow itself (the reference's library)."""
    from PIL import Image

    from oracle import augment_oracle as A
    g = np.random.default_rng(0)
    for (H, W, h, w) in [(300, 400, 224, 224), (100, 150, 224, 224), (224, 224, 224, 224), (500, 223, 224, 224),
                         (37, 1000, 64, 32), (224, 300, 224, 224), (7, 5, 24, 20)]:
        img = g.integers(0, 256, (H, W, 3), dtype=np.uint8)
        ref = np.asarray(Image.fromarray(img).resize((w, h), Image.BILINEAR))
        mine = A.resize_bilinear(img, w, h)
        assert np.array_equal(ref, mine), (H, W, h, w)
        m = (g.random((H, W)) > 0.5).astype(np.uint8) * 255
        refm = np.array(Image.fromarray(m, "L").resize((w, h), Image.NEAREST))
        assert np.array_equal(refm, m[A.scale_nearest_tables(H, h)][:, A.scale_nearest_tables(W, w)])
        for ang in (37.3, -81.25, 12.0001, -0.5, 89.9):
            M = A.rotate_matrix(ang, w, h)
            assert np.array_equal(np.asarray(Image.fromarray(ref).rotate(ang, Image.BILINEAR)), A.rotate_bilinear(ref, M))
            assert np.array_equal(np.array(Image.fromarray(refm, "L").rotate(ang, Image.NEAREST)), A.rotate_nearest(refm, M))


def test_augment_host_tables_match_restatement():
    """The product's host-side tables (utils/augment.py) equal the pinned restatement."""
    from oracle import augment_oracle as A
    from utils import augment as G
    for (i, o) in [(400, 224), (150, 224), (224, 224), (1000, 32), (5, 20), (3, 1)]:
        b0, k0 = A.resample_coeffs(i, o)
        b1, k1 = G.resample_coeffs(i, o)
        assert np.array_equal(b0, b1) and np.array_equal(k0, k1)
        assert np.array_equal(A.scale_nearest_tables(i, o), G.nearest_table(i, o))
    for ang in (37.3, -81.25, 0.5):
        mode, m, fix = G.rotation(ang, 224, 200)
        assert mode == 1 and m == A.rotate_matrix(ang, 224, 200)
        assert tuple(fix) == A.rotate_fixed_coeffs(m)
    assert G.rotation(None, 9, 9)[0] == 0 and G.rotation(-360.0, 9, 9)[0] == 0
    assert G.rotation(180.0, 9, 7)[0] == 2 and G.rotation(90.0, 9, 9)[0] == 3 and G.rotation(-90.0, 9, 9)[0] == 4
    assert G.rotation(90.0, 9, 7)[0] == 1  # non-square: Pillow takes the affine path


def test_augmentation_draw_order_matches_reference():
    """draw_augmentation makes the reference's np.random calls in its order (data_loader.py:41-53)."""
    from utils.augment import draw_augmentation
    np.random.seed(11)
    got = [draw_augmentation(True) for _ in range(50)]
    np.random.seed(11)
    want = []
    for _ in range(50):
        angle = np.random.uniform(-90, 90) if np.random.random() < 0.5 else None
        want.append((angle, bool(np.random.random() < 0.5)))
    assert got == want and draw_augmentation(False) == (None, False)


@pytest.mark.parametrize("name", ["UNet_Baseline", "UNet_AttentionOnly", "UNet_AdditionFusion", "UNet_ConcatFusion",
                                  "UNet_EncoderOnlyDFC", "UNet_DecoderOnlyDFC", "UNet_BothStandardConv"])
def test_zoo_oracle_matches_reference(golden, name):
    """oracle.unet_dfc_sa_res(zoo=name) restates the seven ablation models: logits, loss and every
    gradient of the reference's own run (tests/golden/zoo_*.npz)."""
    fx = golden(f"zoo_{name}.npz")
    sd = {k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")}
    x, t = torch.from_numpy(fx["x"]), torch.from_numpy(fx["t"])
    logits, met, grads, _ = O.forward_backward(sd, x, t, 4, {"bce_weight": 0.5, "dice_weight": 0.5}, model=name)
    assert ((logits - torch.from_numpy(fx["logits"])).norm() / torch.from_numpy(fx["logits"]).norm()).item() < 1e-5
    assert abs(met["loss"].item() - float(fx["loss"])) < 1e-5 * abs(float(fx["loss"]))
    for n, g in grads.items():
        ref = fx.get("grad." + n)
        if ref is None:
            continue
        ref = torch.from_numpy(ref)
        assert ((g - ref).norm() / (ref.norm() + 1e-12)).item() < 1e-4 or (g - ref).abs().max().item() < 1e-7, n


def test_oracle_timed_config_b16_forward():
    """The oracle at the configuration bench.py times (64..512, 224^2, P = 4, B = 16), against the
    reference's own fp32 step of tests/golden/cfg2b16_bf16.npz (make_golden.py (12d)): the seeded init
    (state-dict checksums), the regenerated batch (checksums), image 0's logits, the logits norm and
    the loss.  Forward only (a few seconds on the CPU); the GPU test runs the full step."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), "..", "dfc-sa-unet_amd"))
    from models.unet_dfc_sa_res import UNetDFCSARes
    fx = dict(np.load(os.path.join(GOLDEN, "cfg2b16_bf16.npz")))
    B = int(fx["B"])
    torch.manual_seed(int(fx["seed"]))
    m = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4, ablation_on_qk_channels=8)
    sd = {}
    for k, v in m.state_dict().items():
        v = v.detach().clone()
        if k.endswith("gamma"):
            v.fill_(0.5)
        if v.is_floating_point():
            ref = float(fx["init_sum." + k])
            assert abs(v.double().sum().item() - ref) <= 1e-6 * max(1.0, abs(ref)), k
        sd[k] = v
    g = torch.Generator().manual_seed(int(fx["bseed"]))
    x = torch.randn(B, 3, 224, 224, generator=g)
    t = (torch.rand(B, 1, 224, 224, generator=g) > 0.5).float()
    assert abs(x.double().sum().item() - float(fx["x_sum"])) <= 1e-9 * float(fx["x_sqsum"])
    assert t.double().sum().item() == float(fx["t_sum"])
    with torch.no_grad():
        logits = O.unet_dfc_sa_res(x, sd, pool_size=4, training=True, bufs={})
        met = O.calculate_metrics(torch.sigmoid(logits), t, "bce_dice", {"bce_weight": 0.5, "dice_weight": 0.5})
    close(logits[0], fx["logits0"], rtol=1e-4, atol=1e-4)
    assert abs(logits.double().norm().item() - float(fx["logits_norm"])) <= 1e-5 * float(fx["logits_norm"])
    assert abs(float(met["loss"]) - float(fx["loss"])) <= 1e-5 * abs(float(fx["loss"]))
    assert abs(float(met["dice"]) - float(fx["dice"])) <= 1e-5
