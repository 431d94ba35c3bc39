"""Data loading (drop-in for the reference's utils/data_loader.py:1-181).

``DataLoaderFactory(config)`` with ``get_train_loader()`` / ``get_val_loader()`` and the paired
image/mask transforms of the reference (data_loader.py:10-73, :119-135):
  resize (image bilinear, mask nearest) -> [train + augmentation: p=0.5 rotation by U(-90, 90)
  degrees (bilinear / nearest), p=0.5 horizontal flip] -> image to [0, 1] CHW float, mask
  /255 > 0.5 -> ImageNet normalisation.

The reference's ``datasets.segmentation_dataset.SegmentationDataset`` is absent from its
checkout; it is defined here by its use (README.md "Dataset Structure"): ``root/original/<name>``
and ``root/mask/<name>`` share file names; items are ``{'image', 'mask', 'filename'}``.
torchvision is not needed: ToTensor / Normalize are restated with numpy (same arithmetic).

``dataset.gpu_augment: true`` (optional, new) moves the transforms to the GPU
(``utils/augment.py``): the dataset then returns the decoded uint8 arrays plus the random draws
(made in the reference's order), and ``DeviceBatches`` turns each batch into the device tensors
the trainer consumes with three HIP launches, bit-exact with the Pillow path.

``SyntheticEllipses`` is the learnable synthetic task of SURVEY.md section 8d (1-4 random
ellipses per image, mask-conditioned colour + N(0, 0.5) noise) used to measure validation Dice
without a dataset.
"""
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None

IMAGENET_MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
IMAGENET_STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)
IMG_EXTS = (".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff")


# ------------------------------------------------------------------ paired transforms
class ExtTransform:
    def __call__(self, img, mask):
        return img, mask


class ExtCompose(ExtTransform):
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, img, mask):
        for t in self.transforms:
            img, mask = t(img, mask)
        return img, mask


class ExtResize(ExtTransform):
    def __init__(self, size):
        self.size = tuple(size)

    def __call__(self, img, mask):
        return img.resize(self.size, Image.BILINEAR), mask.resize(self.size, Image.NEAREST)


class ExtRandomRotation(ExtTransform):
    def __init__(self, degrees):
        self.degrees = degrees

    def __call__(self, img, mask):
        if np.random.random() < 0.5:
            angle = np.random.uniform(-self.degrees, self.degrees)
            img = img.rotate(angle, Image.BILINEAR)
            mask = mask.rotate(angle, Image.NEAREST)
        return img, mask


class ExtRandomHorizontalFlip(ExtTransform):
    def __call__(self, img, mask):
        if np.random.random() < 0.5:
            img = img.transpose(Image.FLIP_LEFT_RIGHT)
            mask = mask.transpose(Image.FLIP_LEFT_RIGHT)
        return img, mask


class ExtToTensor(ExtTransform):
    """image: uint8 HWC -> float CHW in [0, 1]; mask: uint8 -> {0, 1} float [1, H, W]."""

    def __call__(self, img, mask):
        a = np.asarray(img, dtype=np.uint8)
        if a.ndim == 2:
            a = a[:, :, None]
        x = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1))).float().div_(255.0)
        m = torch.from_numpy(np.array(mask, dtype=np.uint8)).float().unsqueeze(0) / 255.0
        return x, (m > 0.5).float()


class ExtNormalize(ExtTransform):
    def __init__(self, mean=IMAGENET_MEAN, std=IMAGENET_STD):
        self.mean = torch.as_tensor(np.asarray(mean, dtype=np.float32)).view(-1, 1, 1)
        self.std = torch.as_tensor(np.asarray(std, dtype=np.float32)).view(-1, 1, 1)

    def __call__(self, img, mask):
        return (img - self.mean) / self.std, mask


# ------------------------------------------------------------------ datasets
class SegmentationDataset(Dataset):
    """root/original/<name> + root/mask/<name> (identical file names)."""

    def __init__(self, root, transform=None, img_size=(224, 224), raw_augmentation=None):
        if Image is None:
            raise ImportError("PIL is required to read image files")
        self.root = root.replace("\\", "/")
        self.img_dir = os.path.join(self.root, "original")
        self.mask_dir = os.path.join(self.root, "mask")
        if not os.path.isdir(self.img_dir) or not os.path.isdir(self.mask_dir):
            raise FileNotFoundError(f"expected {self.img_dir} and {self.mask_dir} (README 'Dataset Structure')")
        self.names = sorted(n for n in os.listdir(self.img_dir) if n.lower().endswith(IMG_EXTS)
                            and os.path.exists(os.path.join(self.mask_dir, n)))
        self.transform = transform
        self.img_size = tuple(img_size)
        # raw mode (gpu_augment): None = off, else whether the random draws are made
        self.raw_augmentation = raw_augmentation

    def __len__(self):
        return len(self.names)

    def __getitem__(self, i):
        name = self.names[i]
        img = Image.open(os.path.join(self.img_dir, name)).convert("RGB")
        mask = Image.open(os.path.join(self.mask_dir, name)).convert("L")
        if self.raw_augmentation is not None:
            from utils.augment import draw_augmentation
            angle, flip = draw_augmentation(self.raw_augmentation)
            return {"image": np.asarray(img, dtype=np.uint8), "mask": np.asarray(mask, dtype=np.uint8),
                    "angle": angle, "flip": flip, "filename": name}
        if self.transform is not None:
            img, mask = self.transform(img, mask)
        return {"image": img, "mask": mask, "filename": name}


class SyntheticEllipses(Dataset):
    """Deterministic learnable segmentation task: 1-4 ellipses per image; the image is a
    mask-conditioned colour plus N(0, 0.5) noise (already in the normalised range)."""

    def __init__(self, n, img_size=(224, 224), seed=42):
        self.n, self.size, self.seed = n, tuple(img_size), seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = np.random.default_rng((self.seed, i))
        H, W = self.size[1], self.size[0]
        yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
        mask = np.zeros((H, W), dtype=bool)
        for _ in range(int(g.integers(1, 5))):
            cy, cx = g.uniform(0.15, 0.85) * H, g.uniform(0.15, 0.85) * W
            ry, rx = g.uniform(0.06, 0.22) * H, g.uniform(0.06, 0.22) * W
            th = g.uniform(0, np.pi)
            c, s = np.cos(th), np.sin(th)
            u = ((xx - cx) * c + (yy - cy) * s) / rx
            v = (-(xx - cx) * s + (yy - cy) * c) / ry
            mask |= (u * u + v * v) <= 1.0
        fg = g.normal(0.0, 1.0, size=3).astype(np.float32)
        bg = g.normal(0.0, 1.0, size=3).astype(np.float32)
        img = np.where(mask[None], fg[:, None, None], bg[:, None, None])
        img = img + g.normal(0.0, 0.5, size=(3, H, W)).astype(np.float32)
        return {"image": torch.from_numpy(img.astype(np.float32)),
                "mask": torch.from_numpy(mask[None].astype(np.float32)), "filename": f"synthetic_{self.seed}_{i}"}


class DeviceBatches:
    """Iterates a DataLoader of raw samples (lists) and yields device batches
    {'image': [B,3,h,w] fp32, 'mask': [B,1,h,w] fp32, 'filename': [...]} built by the GPU
    transforms."""

    def __init__(self, loader, transform):
        self.loader, self.transform = loader, transform

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for samples in self.loader:
            images, masks = self.transform(samples)
            yield {"image": images, "mask": masks, "filename": [s["filename"] for s in samples]}


def _collate_list(batch):
    return batch


class RankShardedLoader:
    """The training loader of one data-parallel rank: every rank draws the SAME global permutation
    (a torch.Generator seeded with seed + epoch, identical on every rank, independent of the
    process's global RNG), cuts it into global batches of ``batch_size`` and loads only its own rows
    of each (``dfcsa.ddp.shard_rows``: as even as possible, the last ragged batch included, as the
    reference's DataLoader keeps it).  Each batch carries ``global_rows`` = the global batch's size,
    so the Trainer neither re-shards it nor mis-weights a short shard; a rank without rows in a batch
    gets {'image': None, 'mask': None, 'global_rows': n} and steps with zero gradients."""

    def __init__(self, dataset, batch_size, rank, world, seed=0, shuffle=True, wrap=None, **dl_kwargs):
        self.dataset, self.batch_size, self.rank, self.world = dataset, int(batch_size), rank, world
        self.seed, self.shuffle, self.wrap, self.dl_kwargs = int(seed), shuffle, wrap, dl_kwargs
        self.epoch = 0

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def global_batches(self):
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            order = torch.randperm(n, generator=g).tolist()
        else:
            order = list(range(n))
        return [order[i:i + self.batch_size] for i in range(0, n, self.batch_size)]

    def __iter__(self):
        from dfcsa.ddp import shard_rows
        glob = self.global_batches()
        local = []
        for b in glob:
            lo, hi = shard_rows(len(b), self.rank, self.world)
            local.append(b[lo:hi])
        loader = DataLoader(self.dataset, batch_sampler=[ix for ix in local if ix], **self.dl_kwargs)
        if self.wrap is not None:
            loader = self.wrap(loader)
        it = iter(loader)
        for b, ix in zip(glob, local):
            if not ix:
                yield {"image": None, "mask": None, "filename": [], "global_rows": len(b)}
                continue
            batch = next(it)
            batch["global_rows"] = len(b)
            yield batch


# ------------------------------------------------------------------ factory
class DataLoaderFactory:
    """Same config keys as the reference (data_loader.py:75-98): dataset.{train_dir, val_dir,
    img_size, augmentation}, training.{batch_size, num_workers}.  ``dataset.synthetic: N``
    (optional, new) swaps in SyntheticEllipses of N training / N // 4 validation images."""

    def __init__(self, config):
        self.config = config
        ds = config["dataset"]
        self.train_dir = str(ds.get("train_dir", "")).replace("\\", "/")
        self.val_dir = str(ds.get("val_dir", "")).replace("\\", "/")
        self.batch_size = config["training"]["batch_size"]
        self.num_workers = config["training"].get("num_workers", 0)
        self.img_size = tuple(ds.get("img_size", [224, 224]))
        self.use_augmentation = ds.get("augmentation", False)
        self.synthetic = ds.get("synthetic")
        self.gpu_augment = bool(ds.get("gpu_augment", False))
        print(f"數據增強: {'啟用' if self.use_augmentation else '禁用'}")

    def get_transforms(self, is_train=True):
        if is_train and self.use_augmentation:
            print("使用數據增強進行訓練")
            return ExtCompose([ExtResize(self.img_size), ExtRandomRotation(degrees=90), ExtRandomHorizontalFlip(),
                               ExtToTensor(), ExtNormalize()])
        return ExtCompose([ExtResize(self.img_size), ExtToTensor(), ExtNormalize()])

    @staticmethod
    def _rank_world():
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return dist.get_rank(), dist.get_world_size()
        return 0, 1

    def _loader(self, is_train):
        rank, world = self._rank_world()
        if is_train and world > 1:
            return self._sharded_train_loader(rank, world)
        if self.synthetic:
            n = int(self.synthetic) if is_train else max(1, int(self.synthetic) // 4)
            dataset = SyntheticEllipses(n, self.img_size, seed=42 if is_train else 43)
        elif self.gpu_augment:
            from utils.augment import PairedTransformGPU
            dataset = SegmentationDataset(self.train_dir if is_train else self.val_dir, img_size=self.img_size,
                                          raw_augmentation=bool(is_train and self.use_augmentation))
            loader = DataLoader(dataset, batch_size=self.batch_size, shuffle=is_train,
                                num_workers=self.num_workers, collate_fn=_collate_list)
            return DeviceBatches(loader, PairedTransformGPU(self.img_size, device="cuda"))
        else:
            dataset = SegmentationDataset(self.train_dir if is_train else self.val_dir,
                                          transform=self.get_transforms(is_train), img_size=self.img_size)
        return DataLoader(dataset, batch_size=self.batch_size, shuffle=is_train, num_workers=self.num_workers,
                          pin_memory=torch.cuda.is_available())

    def _sharded_train_loader(self, rank, world):
        """Data parallel (a process group of > 1 ranks): this rank's rows of every global batch."""
        seed = int(self.config["training"].get("seed", 0))
        if self.synthetic:
            ds = SyntheticEllipses(int(self.synthetic), self.img_size, seed=42)
            return RankShardedLoader(ds, self.batch_size, rank, world, seed, num_workers=self.num_workers)
        if self.gpu_augment:
            from utils.augment import PairedTransformGPU
            ds = SegmentationDataset(self.train_dir, img_size=self.img_size, raw_augmentation=bool(self.use_augmentation))
            tf = PairedTransformGPU(self.img_size, device="cuda")
            return RankShardedLoader(ds, self.batch_size, rank, world, seed, num_workers=self.num_workers,
                                     collate_fn=_collate_list, wrap=lambda dl: DeviceBatches(dl, tf))
        ds = SegmentationDataset(self.train_dir, transform=self.get_transforms(True), img_size=self.img_size)
        return RankShardedLoader(ds, self.batch_size, rank, world, seed, num_workers=self.num_workers,
                                 pin_memory=torch.cuda.is_available())

    def get_train_loader(self):
        return self._loader(True)

    def get_val_loader(self):
        return self._loader(False)
