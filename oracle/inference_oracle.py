"""CPU oracle for sliding-window inference.  TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the checker; the product path
(``dfc-sa-unet_amd/utils/inference.py``) runs the HIP kernels of ``libdfcsa.so``.

A literal numpy restatement of the reference (inference.py under the reference checkout):
  * calculate_segmentation_metrics          :73-91   -> calculate_segmentation_metrics
  * predict_large_image (tiles, TTA, canvas) :104-153 -> predict_large_image
  * ToTensor + Normalize of its transform    :116-119 -> to_tensor_normalize (torchvision's
    arithmetic: uint8 -> fp32 / 255, then (x - mean) / std in fp32)
  * cv2.cvtColor(RGB2GRAY) of the mask       :300      -> rgb2gray (OpenCV's 14-bit fixed point)
The model is a callable ``predict(batch NCHW fp32 numpy) -> logits numpy [n, 1, h, w]`` so the
same restatement checks the GPU path with any model.  Pinned against the reference's own
predict_large_image run in the build container (tests/golden/inference.npz, make_golden.py
gen_inference).
"""
import numpy as np

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def to_tensor_normalize(tile_u8):
    x = tile_u8.astype(np.float32).transpose(2, 0, 1) / np.float32(255.0)
    return (x - MEAN[:, None, None]) / STD[:, None, None]


def sigmoid(x):
    x = x.astype(np.float32)
    return (np.float32(1.0) / (np.float32(1.0) + np.exp(-x))).astype(np.float32)


def predict_large_image(predict, image, tile_size, overlap, use_tta=False):
    h, w, _ = image.shape
    stride = tile_size - overlap
    canvas = np.zeros((h, w), dtype=np.float32)
    counts = np.zeros((h, w), dtype=np.float32)
    for y in range(0, h, stride):
        for x in range(0, w, stride):
            y_end, x_end = min(y + tile_size, h), min(x + tile_size, w)
            y_start, x_start = max(0, y_end - tile_size), max(0, x_end - tile_size)
            t = to_tensor_normalize(image[y_start:y_end, x_start:x_end])[None]
            if use_tta:
                p0 = sigmoid(predict(t))
                ph = sigmoid(predict(np.ascontiguousarray(t[..., ::-1])))[..., ::-1]
                pv = sigmoid(predict(np.ascontiguousarray(t[..., ::-1, :])))[..., ::-1, :]
                pred = ((p0 + ph) + pv) / np.float32(3.0)
            else:
                pred = sigmoid(predict(t))
            canvas[y_start:y_end, x_start:x_end] += pred[0, 0]
            counts[y_start:y_end, x_start:x_end] += 1
    counts[counts == 0] = 1
    return canvas / counts


def calculate_segmentation_metrics(pred_binary, gt_binary):
    p = (pred_binary > 0).astype(np.uint8).ravel().astype(np.int64)
    g = (gt_binary > 0).astype(np.uint8).ravel().astype(np.int64)
    tp = int(np.sum(p * g))
    fp = int(np.sum(p)) - tp
    fn = int(np.sum(g)) - tp
    return {"tp": tp, "fp": fp, "fn": fn, "tn": len(p) - (tp + fp + fn)}


def rgb2gray(rgb):
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14).astype(np.uint8)
