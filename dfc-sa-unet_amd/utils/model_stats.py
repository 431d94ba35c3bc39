"""Model statistics: parameters, serialized size and forward FLOPs/MACs.

Mirrors the reference's reporting tool (model_stats.py:15-43 count_parameters / get_model_size,
:146-197 main) without its plotting and third-party counters (thop, ptflops, prettytable and
seaborn are not part of this build):

* ``count_parameters(model)`` -> {'total', 'trainable', 'non_trainable', 'table'} (reference :15-36;
  the table is a list of (name, numel) rows plus ``format_table`` for the text report);
* ``get_model_size(model)`` -> MB of the serialized state_dict (reference :38-43, written to memory
  instead of a temporary file);
* ``forward_flops(model, input_size)`` -> analytic forward FLOPs of the convolutions, transposed
  convolutions and attention matrix products of the DFC-SA U-Net family (UNetDFCSA / UNetDFCSARes
  and UNet_FullResAttention), counted as torch.utils.flop_counter counts them (2 x MACs, no bias
  or elementwise terms).  The GPU models run on hand-written kernels that forward hooks and flop
  counters cannot see, so the count walks the module tree with the spatial sizes the reference
  forward produces (models/unet_dfc_sa_res.py:118-204).  MACs = FLOPs / 2.  Other model families
  return None.
* ``main(config_path, output_dir, input_size)`` writes model_stats.txt / model_stats.csv in the
  reference's layout (:116-144) and prints the summary.
"""
import argparse
import io
import os

import torch
import yaml


def count_parameters(model):
    """Parameter totals (reference model_stats.py:15-36)."""
    rows, total, trainable = [], 0, 0
    for name, p in model.named_parameters():
        n = p.numel()
        rows.append((name, n))
        total += n
        if p.requires_grad:
            trainable += n
    return {"total": total, "trainable": trainable, "non_trainable": total - trainable, "table": rows}


def format_table(rows):
    w = max([len("Module")] + [len(n) for n, _ in rows])
    lines = [f"{'Module':<{w}}  Parameters", "-" * (w + 12)]
    lines += [f"{n:<{w}}  {c:>10,}" for n, c in rows]
    return "\n".join(lines)


def get_model_size(model):
    """Size of the serialized state_dict in MB (reference :38-43)."""
    buf = io.BytesIO()
    torch.save(model.state_dict(), buf)
    return buf.tell() / (1024 * 1024.0)


def _conv(cin, cout, k, h, w):
    return 2.0 * h * w * cout * cin * k * k


def _block_flops(blk, h, w):
    """One DynamicFusionConvAttnBlock at h x w (reference :95-116, :20-39)."""
    conv1 = blk.conv_branch[0]
    cin, c = conv1.in_channels, conv1.out_channels
    f = _conv(cin, c, 3, h, w)                          # local 3x3 branch
    f += _conv(cin, c, 1, h, w)                         # attention entry 1x1
    if hasattr(blk.residual_conv, "in_channels"):
        f += _conv(cin, c, 1, h, w)                     # residual 1x1
    f += _conv(2 * c, c, 1, h, w) + _conv(3 * c, c, 1, h, w)   # gate, fusion
    att = blk.attn_branch[3]
    cq = att.query_conv.out_channels
    if getattr(att, "full_resolution", False):
        n, hp, wp = h * w, h, w                         # unet_dfc_sa_ablation_attention.py:15-26
    else:
        p = att.pool_size
        n, hp, wp = p * p, p, p                         # adaptive pool to P x P
    f += 2 * _conv(c, cq, 1, hp, wp) + _conv(c, c, 1, hp, wp)   # q, k, v projections
    f += 2.0 * n * n * cq + 2.0 * c * n * n             # q k^T, v A^T
    return f


def forward_flops(model, input_size):
    """Forward FLOPs per batch for input_size = (B, C, H, W); None for unsupported families."""
    from models.unet_dfc_sa_res import DynamicFusionConvAttnBlock, UNetDFCSA
    if not isinstance(model, UNetDFCSA):
        return None
    b, _, h, w = input_size
    enc = [model.down1, model.down2, model.down3, model.down4]
    if not all(isinstance(m, DynamicFusionConvAttnBlock) for m in enc + [model.bottleneck]):
        return None
    f, sizes = 0.0, []
    for blk in enc:
        f += _block_flops(blk, h, w)
        sizes.append((h, w))
        h, w = h // 2, w // 2                            # MaxPool2d(2, 2)
    f += _block_flops(model.bottleneck, h, w)
    for up, blk, (sh, sw) in zip((model.up4, model.up3, model.up2, model.up1),
                                 (model.up_conv4, model.up_conv3, model.up_conv2, model.up_conv1),
                                 reversed(sizes)):
        f += 2.0 * h * w * up.in_channels * up.out_channels * 4   # ConvTranspose2d(k2, s2)
        h, w = sh, sw                                    # (bilinear fix to the skip size)
        f += _block_flops(blk, h, w)
    fc = model.final_conv
    f += _conv(fc.in_channels, fc.out_channels, 1, h, w)
    return b * f


def _fmt(v, unit):
    for s, d in (("T", 1e12), ("G", 1e9), ("M", 1e6), ("K", 1e3)):
        if v >= d:
            return f"{v / d:.2f} {s}{unit}"
    return f"{v:.0f} {unit}"


def save_stats_report(stats, output_dir, model_name):
    """model_stats.csv / model_stats.txt as the reference writes them (:116-144)."""
    import pandas as pd
    model_dir = os.path.join(output_dir, model_name)
    os.makedirs(model_dir, exist_ok=True)
    pd.DataFrame({k: [v] for k, v in stats.items() if k != "table"}).to_csv(os.path.join(model_dir, "model_stats.csv"))
    with open(os.path.join(model_dir, "model_stats.txt"), "w", encoding="utf-8") as f:
        f.write(f"Model Statistics Report - {model_name}\n" + "=" * 50 + "\n\n")
        f.write("Parameter Statistics:\n" + "-" * 30 + "\n")
        f.write(f"Total Parameters: {stats['total_params']:,}\n")
        f.write(f"Trainable Parameters: {stats['trainable_params']:,}\n")
        f.write(f"Non-trainable Parameters: {stats['non_trainable_params']:,}\n\n")
        f.write("Model Size:\n" + "-" * 30 + "\n" + f"Size: {stats['model_size']:.2f} MB\n\n")
        f.write("Computational Complexity:\n" + "-" * 30 + "\n")
        f.write(f"FLOPs: {stats['flops']}\n" + f"MACs: {stats['macs']}\n\n")
        f.write(format_table(stats["table"]) + "\n")


def main(config_path, output_dir, input_size):
    """Reference model_stats.py:146-197 (no plots)."""
    from models.model_factory import ModelFactory
    with open(config_path, "r", encoding="utf-8") as f:
        config = yaml.safe_load(f)
    model_name = config["model"]["name"]
    model = ModelFactory.get_model(config)
    model.eval()
    ps = count_parameters(model)
    fl = forward_flops(model, input_size)
    stats = {"total_params": ps["total"], "trainable_params": ps["trainable"],
             "non_trainable_params": ps["non_trainable"], "model_size": get_model_size(model),
             "flops": _fmt(fl, "FLOPs") if fl is not None else "n/a",
             "macs": _fmt(fl / 2, "MACs") if fl is not None else "n/a", "table": ps["table"]}
    save_stats_report(stats, output_dir, model_name)
    print(f"\nModel Statistics Summary - {model_name}:\n" + "=" * 50)
    print(f"Total Parameters: {stats['total_params']:,}")
    print(f"Trainable Parameters: {stats['trainable_params']:,}")
    print(f"Non-trainable Parameters: {stats['non_trainable_params']:,}")
    print(f"Model Size: {stats['model_size']:.2f} MB")
    print(f"Computational Complexity:\n  - MACs: {stats['macs']}\n  - FLOPs: {stats['flops']}")
    print(f"\nDetailed report saved to: {os.path.join(output_dir, model_name)}")
    return stats


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="model statistics (parameters, size, FLOPs)")
    ap.add_argument("--config", required=True)
    ap.add_argument("--output_dir", default="model_stats")
    ap.add_argument("--input_size", type=int, nargs=4, default=[1, 3, 224, 224])
    a = ap.parse_args()
    main(a.config, a.output_dir, tuple(a.input_size))
