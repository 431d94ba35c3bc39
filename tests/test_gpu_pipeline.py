"""GPU parity of the inference pipeline (utils/inference.py on the dfcsa_tiles_* / dfcsa_seg_counts
kernels) against the reference's own predict_large_image output (tests/golden/inference.npz) and
the CPU restatement in oracle/inference_oracle.py.

Tolerances: the canvas is fp32 probability; the GPU and the CPU evaluate the same model in a
different summation order and expf vs numpy exp differ in the last ulp, so canvases agree to
1e-5 absolute (probabilities are in [0, 1]).  Counts are integers and must be exact.
"""
import numpy as np
import pytest
import torch

from oracle import inference_oracle as IO

pytestmark = pytest.mark.gpu


def _conv_model(fx):
    conv = torch.nn.Conv2d(3, 1, 3, padding=1)
    conv.weight.data = torch.from_numpy(fx["conv.weight"])
    conv.bias.data = torch.from_numpy(fx["conv.bias"])
    return conv.cuda()


@pytest.mark.parametrize("tiles_per_batch", [1, 5, 64])
def test_predict_large_image_matches_reference(golden, tiles_per_batch):
    from utils.inference import predict_large_image
    fx = golden("inference.npz")
    model = _conv_model(fx)
    for name in ("a", "b", "c", "d"):
        img = fx[f"{name}.image"]
        tile, overlap = (int(v) for v in fx[f"{name}.cfg"])
        for tta in (0, 1):
            got = predict_large_image(model, img, tile, overlap, "cuda", use_tta=bool(tta),
                                      tiles_per_batch=tiles_per_batch)
            want = fx[f"{name}.canvas.tta{tta}"]
            assert got.shape == want.shape and got.dtype == np.float32
            assert np.abs(got - want).max() < 1e-5, (name, tta, np.abs(got - want).max())


def test_predict_large_image_dfc_model_matches_oracle():
    """The DFC-SA-Res model (fp32 mode, eval) over a 100 x 130 image with 64-pixel tiles, TTA on:
    batched tiles through the kernels == the reference loop run tile by tile."""
    from models.unet_dfc_sa_res import UNetDFCSARes
    from utils.inference import predict_large_image
    torch.manual_seed(3)
    model = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, precision="fp32").cuda()
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    model.eval()
    img = np.random.default_rng(4).integers(0, 256, size=(100, 130, 3), dtype=np.uint8)

    def predict(b):
        with torch.no_grad():
            return model(torch.from_numpy(np.ascontiguousarray(b)).cuda()).cpu().numpy()

    want = IO.predict_large_image(predict, img, 64, 16, use_tta=True)
    got = predict_large_image(model, img, 64, 16, "cuda", use_tta=True, tiles_per_batch=4)
    assert np.abs(got - want).max() < 1e-5


@pytest.mark.parametrize("gc", [1, 3])
def test_segmentation_counts_exact(gc):
    from utils.inference import calculate_segmentation_metrics, segmentation_counts
    g = np.random.default_rng(5 + gc)
    H, W = 333, 517
    prob = g.random((H, W), dtype=np.float32)
    prob[::7, ::5] = 0.5  # ties at the threshold: 0.5 > 0.5 is false
    gt = g.integers(0, 256, size=(H, W, gc) if gc == 3 else (H, W), dtype=np.uint8)
    if gc == 3:
        gt[::3] = gt[::3, :, :1]  # some gray pixels (R = G = B), as binary mask files hold
    got = segmentation_counts(torch.from_numpy(prob).cuda(), gt, threshold=0.5, gt_threshold=128)
    gray = IO.rgb2gray(gt) if gc == 3 else gt
    want = IO.calculate_segmentation_metrics((prob > 0.5).astype(np.uint8), (gray > 128).astype(np.uint8))
    assert got == want
    pb = (prob > 0.3).astype(np.uint8)
    gb = (gray > 100).astype(np.uint8)
    assert calculate_segmentation_metrics(pb, gb) == IO.calculate_segmentation_metrics(pb, gb)


def test_counts_match_reference_fixture(golden):
    from utils.inference import calculate_segmentation_metrics
    fx = golden("inference.npz")
    for name in ("a", "b", "c", "d"):
        c = calculate_segmentation_metrics((fx[f"{name}.canvas.tta0"] > 0.5).astype(np.uint8),
                                           (fx[f"{name}.gt"] > 128).astype(np.uint8))
        assert [c[k] for k in ("tp", "fp", "fn", "tn")] == fx[f"{name}.counts"].tolist()


def test_evaluate_image_and_global_metrics(golden):
    from utils.inference import evaluate_image, global_metrics
    fx = golden("inference.npz")
    model = _conv_model(fx)
    img, gt = fx["a.image"], fx["a.gt"]
    tile, overlap = (int(v) for v in fx["a.cfg"])
    prob, m = evaluate_image(model, img, gt, tile, overlap, threshold=0.5, use_tta=False)
    assert prob.is_cuda and tuple(prob.shape) == gt.shape
    want = IO.calculate_segmentation_metrics((prob.cpu().numpy() > 0.5).astype(np.uint8),
                                             (gt > 128).astype(np.uint8))
    assert {k: m[k] for k in want} == want
    gm = global_metrics([m, m])
    tp, fp, fn = 2 * m["tp"], 2 * m["fp"], 2 * m["fn"]
    assert abs(gm["dice_f1"] - 2 * tp / (2 * tp + fp + fn + 1e-7)) < 1e-12


def test_predict_single_image():
    from utils.inference import predict_single_image
    torch.manual_seed(6)
    conv = torch.nn.Conv2d(3, 1, 3, padding=1).cuda()
    x = torch.randn(1, 3, 40, 56)
    got = predict_single_image(conv, x, "cuda")
    with torch.no_grad():
        want = torch.sigmoid(conv(x.cuda())).cpu().numpy()[0, 0]
    assert got.shape == (40, 56) and np.abs(got - want).max() < 1e-6


# --------------------------------------------------------------------- paired transforms
def _smooth_image(g, H, W):
    """A natural-looking uint8 image (smooth gradients + noise) so interpolation weights matter."""
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    base = np.stack([127 + 120 * np.sin(x / 7.0 + c) * np.cos(y / 11.0 - c) for c in range(3)], -1)
    return np.clip(base + g.normal(0, 12, (H, W, 3)), 0, 255).astype(np.uint8)


def test_paired_transform_gpu_bit_exact_with_pillow():
    """The GPU batch transform equals the reference's Pillow chain (resize BILINEAR / NEAREST,
    rotate BILINEAR / NEAREST, h-flip, ToTensor, Normalize, mask / 255 > 0.5) bit for bit, on a
    batch of different source sizes (up- and down-scaling, identity), angles (incl. Pillow's exact
    0 / 90 / 180 / 270 fast paths) and flips."""
    from oracle import augment_oracle as A
    from utils.augment import PairedTransformGPU
    g = np.random.default_rng(21)
    sizes = [(300, 400), (100, 150), (224, 224), (500, 223), (37, 1000), (224, 300), (7, 5), (640, 480), (224, 224)]
    angles = [37.3, -81.25, None, 90.0, -90.0, 180.0, 0.0, -12.5, 44.999]
    samples = []
    for i, ((H, W), ang) in enumerate(zip(sizes, angles)):
        img = _smooth_image(g, H, W)
        mask = g.choice(np.array([0, 127, 128, 255], dtype=np.uint8), size=(H, W))
        samples.append({"image": img, "mask": mask, "angle": ang, "flip": bool(i % 2)})
    for size in ((224, 224), (160, 96)):
        images, masks = PairedTransformGPU(size)(samples)
        images, masks = images.cpu().numpy(), masks.cpu().numpy()
        for i, s in enumerate(samples):
            x, m = A.reference_transform(s["image"], s["mask"], size, s["angle"], s["flip"])
            assert np.array_equal(images[i], x), (size, i, np.abs(images[i] - x).max())
            assert np.array_equal(masks[i], m), (size, i)


def test_dataset_gpu_augment_matches_pillow_loader(tmp_path):
    """DataLoaderFactory with dataset.gpu_augment: same seeds -> the same batches as the reference's
    Pillow transforms (same np.random draw order, same shuffling), as device tensors."""
    from PIL import Image

    from utils.data_loader import DataLoaderFactory
    g = np.random.default_rng(22)
    for split in ("train", "val"):
        for sub in ("original", "mask"):
            (tmp_path / split / sub).mkdir(parents=True)
        for i, (H, W) in enumerate([(120, 160), (300, 260), (224, 224), (90, 90), (400, 333)]):
            Image.fromarray(_smooth_image(g, H, W)).save(tmp_path / split / "original" / f"im{i}.png")
            Image.fromarray((g.random((H, W)) > 0.6).astype(np.uint8) * 255, "L").save(
                tmp_path / split / "mask" / f"im{i}.png")
    cfg = {"dataset": {"train_dir": str(tmp_path / "train"), "val_dir": str(tmp_path / "val"), "img_size": [128, 96],
                       "augmentation": True},
           "training": {"batch_size": 2, "num_workers": 0}}
    for loader_name in ("get_train_loader", "get_val_loader"):
        cpu = getattr(DataLoaderFactory(cfg), loader_name)()
        gpu = getattr(DataLoaderFactory(dict(cfg, dataset=dict(cfg["dataset"], gpu_augment=True))), loader_name)()
        assert len(cpu) == len(gpu) == 3
        for seed in (5, 6):
            torch.manual_seed(seed)
            np.random.seed(seed)
            a = list(cpu)
            torch.manual_seed(seed)
            np.random.seed(seed)
            b = list(gpu)
            for ba, bb in zip(a, b):
                assert list(ba["filename"]) == list(bb["filename"])
                assert bb["image"].is_cuda and bb["mask"].is_cuda
                assert torch.equal(ba["image"], bb["image"].cpu()) and torch.equal(ba["mask"], bb["mask"].cpu())
