"""CPU tests of the data pipeline (utils/data_loader.py, reference utils/data_loader.py).

The reference's dataset module is absent from its checkout and torchvision is not installed, so
parity is pinned on the arithmetic the reference composes (PIL resize/rotate/flip, ToTensor =
uint8/255 CHW, mask/255 > 0.5, ImageNet Normalize) restated with numpy here."""
import numpy as np
import pytest
import torch

PIL = pytest.importorskip("PIL")
from PIL import Image  # noqa: E402


def _write_dataset(root, n=3, size=(40, 30)):
    rng = np.random.default_rng(0)
    for sub in ("original", "mask"):
        (root / sub).mkdir(parents=True)
    for i in range(n):
        img = rng.integers(0, 256, size=(size[1], size[0], 3), dtype=np.uint8)
        m = (rng.random((size[1], size[0])) > 0.5).astype(np.uint8) * 255
        Image.fromarray(img).save(root / "original" / f"im{i}.png")
        Image.fromarray(m).save(root / "mask" / f"im{i}.png")
    (root / "original" / "orphan.png").write_bytes((root / "original" / "im0.png").read_bytes())


def test_dataset_and_eval_transform(tmp_path):
    from utils.data_loader import DataLoaderFactory, IMAGENET_MEAN, IMAGENET_STD
    _write_dataset(tmp_path / "train")
    _write_dataset(tmp_path / "val")
    cfg = {"dataset": {"train_dir": str(tmp_path / "train"), "val_dir": str(tmp_path / "val"),
                       "img_size": [32, 24], "augmentation": False},
           "training": {"batch_size": 2, "num_workers": 0}}
    fac = DataLoaderFactory(cfg)
    ds = fac.get_val_loader().dataset
    assert ds.names == ["im0.png", "im1.png", "im2.png"]  # orphan (no mask) skipped
    item = ds[1]
    assert item["image"].shape == (3, 24, 32) and item["mask"].shape == (1, 24, 32)
    img = Image.open(tmp_path / "val" / "original" / "im1.png").convert("RGB").resize((32, 24), Image.BILINEAR)
    want = (np.asarray(img, dtype=np.float32).transpose(2, 0, 1) / 255.0 - IMAGENET_MEAN[:, None, None]) \
        / IMAGENET_STD[:, None, None]
    assert np.allclose(item["image"].numpy(), want, atol=1e-6)
    m = Image.open(tmp_path / "val" / "mask" / "im1.png").convert("L").resize((32, 24), Image.NEAREST)
    assert np.array_equal(item["mask"][0].numpy(), (np.asarray(m) / 255.0 > 0.5).astype(np.float32))
    batch = next(iter(fac.get_val_loader()))
    assert batch["image"].shape == (2, 3, 24, 32) and batch["filename"] == ["im0.png", "im1.png"]


def test_augmentation_keeps_pairs_aligned(tmp_path):
    from utils.data_loader import ExtRandomHorizontalFlip, ExtRandomRotation
    img = Image.fromarray(np.tile(np.arange(16, dtype=np.uint8)[None, :, None] * 16, (16, 1, 3)))
    mask = Image.fromarray((np.arange(16)[None, :] < 4).repeat(16, 0).astype(np.uint8) * 255)
    np.random.seed(1)
    flips = 0
    for _ in range(20):
        i2, m2 = ExtRandomHorizontalFlip()(img, mask)
        a, b = np.asarray(i2)[..., 0], np.asarray(m2)
        flipped = a[0, 0] > a[0, -1]
        flips += flipped
        assert bool(b[0, -1] > 0) == bool(flipped)
        i3, m3 = ExtRandomRotation(90)(img, mask)
        assert set(np.unique(np.asarray(m3))) <= {0, 255}   # nearest keeps the mask binary
    assert 0 < flips < 20


def test_synthetic_ellipses_deterministic():
    from utils.data_loader import DataLoaderFactory, SyntheticEllipses
    a, b = SyntheticEllipses(4, (64, 48), seed=42), SyntheticEllipses(4, (64, 48), seed=42)
    x, y = a[3], b[3]
    assert torch.equal(x["image"], y["image"]) and torch.equal(x["mask"], y["mask"])
    assert x["image"].shape == (3, 48, 64) and 0 < x["mask"].mean() < 1
    assert not torch.equal(SyntheticEllipses(4, (64, 48), seed=43)[3]["mask"], x["mask"])
    cfg = {"dataset": {"synthetic": 8, "img_size": [32, 32], "augmentation": True},
           "training": {"batch_size": 4, "num_workers": 0}}
    fac = DataLoaderFactory(cfg)
    assert len(fac.get_train_loader().dataset) == 8 and len(fac.get_val_loader().dataset) == 2
