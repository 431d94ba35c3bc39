"""Model statistics: parameters, serialized size and forward FLOPs/MACs.

Mirrors the reference's reporting tool (model_stats.py:15-43 count_parameters / get_model_size,
:146-197 main) without its plotting and third-party counters (thop, ptflops, prettytable and
seaborn are not part of this build):

* ``count_parameters(model)`` -> {'total', 'trainable', 'non_trainable', 'table'} (reference :15-36;
  the table is a list of (name, numel) rows plus ``format_table`` for the text report);
* ``get_model_size(model)`` -> MB of the serialized state_dict (reference :38-43, written to memory
  instead of a temporary file);
* ``forward_flops(model, input_size)`` -> analytic forward FLOPs of the convolutions, transposed
  convolutions, linear layers and attention matrix products, counted as torch.utils.flop_counter
  counts them (2 x MACs, no bias or elementwise terms), for every model the factory builds: the
  DFC-SA U-Net family (UNetDFCSA / UNetDFCSARes, UNet_FullResAttention and the ablation zoo, whose
  blocks are walked by the branches they own), UNet (config 1) and TransUNet R50-ViT (config 4).
  The GPU models run on hand-written kernels that forward hooks and flop counters cannot see, so
  the count walks the module tree with the spatial sizes the reference forward produces
  (models/unet_dfc_sa_res.py:118-204, models/unet.py:69-101, models/transformer_unet.py:97-106,
  :137-157, :193-200, :300-312, :362-368).  MACs = FLOPs / 2.  The reference counts with ptflops
  (model_stats.py:164-165), which adds BatchNorm / activation terms; this count is the
  convolution / matmul work only.
* ``main(config_path, output_dir, input_size)`` writes model_stats.txt / model_stats.csv in the
  reference's layout (:116-144) and prints the summary.
"""
import argparse
import io
import os

import torch
import yaml

from dfcsa import chanpad


def count_parameters(model):
    """Parameter totals (reference model_stats.py:15-36)."""
    rows, total, trainable = [], 0, 0
    for name, p in model.named_parameters():
        n = chanpad.numel(p)   # reference shape for channel-padded widths (dfcsa/chanpad.py)
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


def _out(h, k, s, p):
    return (h + 2 * p - k) // s + 1


def _conv_mod(m, h, w):
    """FLOPs and output size of an nn.Conv2d at input h x w (flop_counter: 2 * out * Cin/g * k^2)."""
    kh, kw = m.kernel_size
    ho, wo = _out(h, kh, m.stride[0], m.padding[0]), _out(w, kw, m.stride[1], m.padding[1])
    cin, cout = chanpad.io_channels(m)
    return 2.0 * ho * wo * cout * (cin // m.groups) * kh * kw, ho, wo


def _block_flops(blk, h, w):
    """One block of the DFC-SA U-Net family at h x w, by the branches it owns: the DFC block
    (reference unet_dfc_sa_res.py:95-116, :20-39) and the ablation blocks (local-only, attention-
    only, addition / concat fusion: unet_dfc_sa_ablation_branches.py, _fusion.py)."""
    f = 0.0
    conv_branch = getattr(blk, "conv_branch", None)
    attn_branch = getattr(blk, "attn_branch", None)
    if conv_branch is not None:
        f += _conv_mod(conv_branch[0], h, w)[0]        # local 3x3 branch
    if attn_branch is not None:
        entry = attn_branch[0]
        cin, c = chanpad.io_channels(entry)
        f += _conv(cin, c, 1, h, w)                     # attention entry 1x1
        att = attn_branch[3]
        cq = chanpad.io_channels(att.query_conv)[1]
        if getattr(att, "full_resolution", False):
            n, hp, wp = h * w, h, w                     # unet_dfc_sa_ablation_attention.py:15-26
        else:
            p = att.pool_size
            n, hp, wp = p * p, p, p                     # adaptive pool to P x P
        f += 2 * _conv(c, cq, 1, hp, wp) + _conv(c, c, 1, hp, wp)   # q, k, v projections
        f += 2.0 * n * n * cq + 2.0 * c * n * n         # q k^T, v A^T
    if hasattr(blk.residual_conv, "in_channels"):
        f += _conv_mod(blk.residual_conv, h, w)[0]      # residual 1x1
    if getattr(blk, "gate", None) is not None:
        f += _conv_mod(blk.gate[0], h, w)[0]            # gate 1x1 over [local | attn]
    if getattr(blk, "fusion_conv", None) is not None:
        f += _conv_mod(blk.fusion_conv[0], h, w)[0]     # fusion 1x1 (3C for DFC, 2C for concat)
    return f


def _dfc_unet_flops(model, h, w):
    """UNetDFCSA.forward (reference unet_dfc_sa_res.py:161-204) and AblationUNetBase.forward."""
    enc = [model.down1, model.down2, model.down3, model.down4]
    f, sizes = 0.0, []
    for blk in enc:
        f += _block_flops(blk, h, w)
        sizes.append((h, w))
        h, w = h // 2, w // 2                            # MaxPool2d(2, 2)
    f += _block_flops(model.bottleneck, h, w)
    for up, blk, (sh, sw) in zip((model.up4, model.up3, model.up2, model.up1),
                                 (model.up_conv4, model.up_conv3, model.up_conv2, model.up_conv1),
                                 reversed(sizes)):
        f += 2.0 * h * w * chanpad.io_channels(up)[0] * chanpad.io_channels(up)[1] * 4   # ConvTranspose2d(k2, s2)
        h, w = sh, sw                                    # (bilinear fix to the skip size)
        f += _block_flops(blk, h, w)
    fc = model.final_conv
    f += _conv(*chanpad.io_channels(fc), 1, h, w)
    return f


def _unet_flops(model, h, w):
    """UNet.forward (reference unet.py:69-101, bilinear=False): DoubleConv, Down = MaxPool2d(2,
    ceil_mode=True) + DoubleConv, Up = ConvTranspose2d(k2, s2) + crop to the smaller of the two +
    DoubleConv over the concat, OutConv 1x1."""
    def dconv(dc, h, w):
        f0, h, w = _conv_mod(dc.conv[0], h, w)
        f1, h, w = _conv_mod(dc.conv[3], h, w)
        return f0 + f1, h, w
    f, h, w = dconv(model.inc, h, w)
    sizes = [(h, w)]
    for d in (model.down1, model.down2, model.down3, model.down4):
        h, w = (h + 1) // 2, (w + 1) // 2                # ceil_mode pooling
        g, h, w = dconv(d.mpconv[1], h, w)
        f += g
        sizes.append((h, w))
    for up, (sh, sw) in zip((model.up1, model.up2, model.up3, model.up4), reversed(sizes[:4])):
        t = up.up
        f += 2.0 * h * w * t.in_channels * t.out_channels * t.kernel_size[0] * t.kernel_size[1]
        h, w = min(h * 2, sh), min(w * 2, sw)            # crop (unet.py:44-56)
        g, h, w = dconv(up.conv, h, w)
        f += g
    f += _conv_mod(model.outc.conv, h, w)[0]
    return f


def _transunet_flops(model, h, w):
    """TransUNet.forward (reference transformer_unet.py:362-368): ResNetV2 root + bottleneck units
    (:58-68, :97-106; StdConv2d counts as a conv, its weight standardisation is elementwise),
    patch embeddings (:193-200), ViT blocks (Attention :137-157: q, k, v, out projections and the
    two score products; Mlp :167-173), DecoderCup (:300-312: conv_more, per block two 3x3 convs
    after the 2x upsample) and the 3x3 segmentation head."""
    emb = model.transformer.embeddings
    hyb = emb.hybrid_model
    f, h, w = _conv_mod(hyb.root.conv, h, w)
    h, w = _out(h, 3, 2, 1), _out(w, 3, 2, 1)            # MaxPool2d(3, 2, 1)
    for blk in hyb.body.children():
        for u in blk.children():
            if getattr(u, "downsample", None) is not None:
                f += _conv_mod(u.downsample, h, w)[0]
            g1, h1, w1 = _conv_mod(u.conv1, h, w)
            g2, h, w = _conv_mod(u.conv2, h1, w1)
            g3 = _conv_mod(u.conv3, h, w)[0]
            f += g1 + g2 + g3
    g, h, w = _conv_mod(emb.patch_embeddings, h, w)
    f += g
    n = h * w
    for layer in model.transformer.encoder.layer:
        a = layer.attn
        for lin in (a.query, a.key, a.value, a.out, layer.ffn.fc1, layer.ffn.fc2):
            f += 2.0 * n * lin.in_features * lin.out_features
        f += 2 * (2.0 * n * n * a.all_head_size)          # q k^T and P v over all heads
    dec = model.decoder
    g, h, w = _conv_mod(dec.conv_more[0], h, w)
    f += g
    for blk in dec.blocks:
        h, w = 2 * h, 2 * w                              # UpsamplingBilinear2d(scale_factor=2)
        g1, h, w = _conv_mod(blk.conv1[0], h, w)
        g2, h, w = _conv_mod(blk.conv2[0], h, w)
        f += g1 + g2
    f += _conv_mod(model.segmentation_head[0], h, w)[0]
    return f


def forward_flops(model, input_size):
    """Forward FLOPs per batch for input_size = (B, C, H, W); None for a model outside the
    factory's families."""
    from models.transformer_unet import TransUNet
    from models.unet import UNet
    from models.unet_dfc_sa_res import UNetDFCSA
    b, _, h, w = input_size
    if isinstance(model, UNetDFCSA):
        return b * _dfc_unet_flops(model, h, w)
    if isinstance(model, UNet):
        return b * _unet_flops(model, h, w)
    if isinstance(model, TransUNet):
        return b * _transunet_flops(model, h, w)
    return None


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
