"""CPU fp32 oracle for the DFC-SA-Res training step.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker (or the timed CPU baseline) -- never as part of the product
path.  The product path (``dfc-sa-unet_amd/``) runs the HIP kernels of ``libdfcsa.so`` and fails
loudly when they are missing.

What it is: a functional restatement of the reference algorithm in eager PyTorch on the CPU
(NCHW, fp32; autograd supplies the backward), keyed by the reference's ``state_dict`` names so
that golden fixtures and our GPU modules can be fed to it directly.  It is *pinned* against
golden vectors produced by running the reference itself in the build container
(``tests/golden/make_golden.py``; ``tests/test_oracle_golden.py`` checks it).

Reference functions restated (file:line under the reference checkout):
  * LightSelfAttention.forward            models/unet_dfc_sa_res.py:20-39   -> light_self_attention
  * DynamicFusionConvAttnBlock.forward    models/unet_dfc_sa_res.py:95-116  -> dfc_block
  * UNetDFCSA.forward                     models/unet_dfc_sa_res.py:161-204 -> unet_dfc_sa_res
  * dice_loss / BCEDiceLoss               utils/metrics.py:6-24, 52-78      -> bce_dice_loss
  * calculate_metrics ('bce_dice')        utils/metrics.py:211-264          -> calculate_metrics
  * train step (zero_grad, fwd, sigmoid, loss, backward, clip_grad_norm_(1.0), SGD)
                                          utils/trainer.py:115-151, train.py:73-78 -> train_step
  * FullResolutionAttention.forward       models/unet_dfc_sa_ablation_attention.py:15-26
                                                                   -> full_resolution_attention
  * FullResAttnDFCBlock / UNet_FullResAttention (AblationUNetBase.forward,
    models/unet_dfc_sa_ablation_branches.py:129-164)          -> dfc_block / unet_dfc_sa_res(full_res=True)
  * UNet.forward (DoubleConv, Down, Up, OutConv)  models/unet.py:6-101        -> unet
  * TransUNet.forward (StdConv2d, PreActBottleneck, ResNetV2, Attention, Mlp, Block, Embeddings,
    Encoder, DecoderCup, SegmentationHead)    models/transformer_unet.py:21-368 -> transunet
  * the ablation zoo: LocalOnlyBlock / AttentionOnlyBlock (unet_dfc_sa_ablation_branches.py:62-101),
    AdditionFusionBlock / ConcatFusionBlock (unet_dfc_sa_ablation_fusion.py:35-100), placement models
    (unet_dfc_sa_ablation_placement.py:85-284)          -> *_block, unet_dfc_sa_res(zoo=name)
"""
import math

import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1


# ------------------------------------------------------------------------------------------
# building blocks
# ------------------------------------------------------------------------------------------
def conv(x, sd, name, padding=0, bias=True):
    w = sd[name + ".weight"]
    b = sd.get(name + ".bias") if bias else None
    return F.conv2d(x, w, b, padding=padding)


def batch_norm(x, sd, name, training, bufs):
    """nn.BatchNorm2d semantics: train mode normalises with the biased batch variance and
    updates running stats with momentum 0.1 using the unbiased variance; eval mode uses the
    running statistics.  ``bufs`` (dict) receives the updated running stats."""
    rm = sd[name + ".running_mean"].clone()
    rv = sd[name + ".running_var"].clone()
    y = F.batch_norm(x, rm, rv, sd[name + ".weight"], sd[name + ".bias"], training,
                     BN_MOMENTUM, BN_EPS)
    if training and bufs is not None:
        bufs[name + ".running_mean"] = rm
        bufs[name + ".running_var"] = rv
        nbt = sd.get(name + ".num_batches_tracked")
        if nbt is not None:
            bufs[name + ".num_batches_tracked"] = nbt + 1
    return y


def light_self_attention(a, sd, name, pool_size):
    """models/unet_dfc_sa_res.py:20-39: pooled self-attention, no 1/sqrt(d) scale,
    softmax over keys, bilinear (align_corners=False) back to H x W, gamma-scaled residual."""
    B, C, H, W = a.shape
    p = F.adaptive_avg_pool2d(a, (pool_size, pool_size))
    N = pool_size * pool_size
    q = conv(p, sd, name + ".query_conv").reshape(B, -1, N).permute(0, 2, 1)   # [B,N,C']
    k = conv(p, sd, name + ".key_conv").reshape(B, -1, N)                      # [B,C',N]
    att = torch.softmax(torch.bmm(q, k), dim=-1)                               # [B,N,N]
    v = conv(p, sd, name + ".value_conv").reshape(B, C, N)                     # [B,C,N]
    o = torch.bmm(v, att.permute(0, 2, 1)).reshape(B, C, pool_size, pool_size)
    o = F.interpolate(o, size=(H, W), mode="bilinear", align_corners=False)
    return sd[name + ".gamma"] * o + a


def full_resolution_attention(a, sd, name, q_chunk=8192):
    """models/unet_dfc_sa_ablation_attention.py:15-26: attention over all H*W positions, q/k with
    C//8 channels, softmax over keys without a 1/sqrt(d) scale, gamma-scaled residual.  Past
    q_chunk positions the [N, N] map is formed q_chunk query rows at a time (each row's softmax over
    every key, as the reference's): at 512^2 the whole map would be 275 GB."""
    B, C, H, W = a.shape
    N = H * W
    q = conv(a, sd, name + ".query_conv").reshape(B, -1, N).permute(0, 2, 1)    # [B,N,C']
    k = conv(a, sd, name + ".key_conv").reshape(B, -1, N)                       # [B,C',N]
    v = conv(a, sd, name + ".value_conv").reshape(B, -1, N)                     # [B,C,N]
    if N <= q_chunk:
        att = torch.softmax(torch.bmm(q, k), dim=-1)                            # [B,N,N]
        o = torch.bmm(v, att.permute(0, 2, 1)).reshape(B, C, H, W)
    else:
        o = torch.cat([torch.bmm(v, torch.softmax(torch.bmm(q[:, i:i + q_chunk], k), dim=-1).permute(0, 2, 1))
                       for i in range(0, N, q_chunk)], dim=2).reshape(B, C, H, W)
    return sd[name + ".gamma"] * o + a


def dfc_block(x, sd, name, pool_size, training, bufs, full_res=False):
    """models/unet_dfc_sa_res.py:95-116 (DynamicFusionConvAttnBlock.forward); with full_res the
    attention branch is FullResolutionAttention (unet_dfc_sa_ablation_attention.py:71-92, otherwise
    identical)."""
    local = F.relu(batch_norm(conv(x, sd, name + ".conv_branch.0", padding=1), sd,
                              name + ".conv_branch.1", training, bufs))
    a = F.relu(batch_norm(conv(x, sd, name + ".attn_branch.0"), sd, name + ".attn_branch.1",
                          training, bufs))
    if full_res:
        attn = full_resolution_attention(a, sd, name + ".attn_branch.3")
    else:
        attn = light_self_attention(a, sd, name + ".attn_branch.3", pool_size)
    comb = torch.cat([local, attn], dim=1)
    g = torch.sigmoid(batch_norm(conv(comb, sd, name + ".gate.0"), sd, name + ".gate.1",
                                 training, bufs))
    fused = g * local + (1 - g) * attn
    out = F.relu(batch_norm(conv(torch.cat([fused, comb], dim=1), sd, name + ".fusion_conv.0"),
                            sd, name + ".fusion_conv.1", training, bufs))
    if (name + ".residual_conv.weight") in sd:
        res = conv(x, sd, name + ".residual_conv", bias=False)
    else:
        res = x
    return out + sd[name + ".res_scale"] * res


def _residual(x, sd, name):
    if (name + ".residual_conv.weight") in sd:
        return conv(x, sd, name + ".residual_conv", bias=False)
    return x


def _local_branch(x, sd, name, training, bufs):
    return F.relu(batch_norm(conv(x, sd, name + ".conv_branch.0", padding=1), sd, name + ".conv_branch.1",
                             training, bufs))


def _attn_branch(x, sd, name, pool_size, training, bufs):
    a = F.relu(batch_norm(conv(x, sd, name + ".attn_branch.0"), sd, name + ".attn_branch.1", training, bufs))
    return light_self_attention(a, sd, name + ".attn_branch.3", pool_size)


def local_only_block(x, sd, name, pool_size, training, bufs):
    """models/unet_dfc_sa_ablation_branches.py:93-101 (LocalOnlyBlock.forward)."""
    return _local_branch(x, sd, name, training, bufs) + sd[name + ".res_scale"] * _residual(x, sd, name)


def attention_only_block(x, sd, name, pool_size, training, bufs):
    """models/unet_dfc_sa_ablation_branches.py:62-70 (AttentionOnlyBlock.forward)."""
    return _attn_branch(x, sd, name, pool_size, training, bufs) + sd[name + ".res_scale"] * _residual(x, sd, name)


def addition_fusion_block(x, sd, name, pool_size, training, bufs):
    """models/unet_dfc_sa_ablation_fusion.py:35-49 (AdditionFusionBlock.forward)."""
    fused = _local_branch(x, sd, name, training, bufs) + _attn_branch(x, sd, name, pool_size, training, bufs)
    return fused + sd[name + ".res_scale"] * _residual(x, sd, name)


def concat_fusion_block(x, sd, name, pool_size, training, bufs):
    """models/unet_dfc_sa_ablation_fusion.py:86-100 (ConcatFusionBlock.forward)."""
    comb = torch.cat([_local_branch(x, sd, name, training, bufs),
                      _attn_branch(x, sd, name, pool_size, training, bufs)], dim=1)
    fused = F.relu(batch_norm(conv(comb, sd, name + ".fusion_conv.0"), sd, name + ".fusion_conv.1", training, bufs))
    return fused + sd[name + ".res_scale"] * _residual(x, sd, name)


def _zoo_blocks(model):
    """(encoder/bottleneck block, decoder block) of the ablation models (model_factory.py:160-187;
    placement: unet_dfc_sa_ablation_placement.py:85-284)."""
    dfc = lambda x, sd, n, p, tr, b: dfc_block(x, sd, n, p, tr, b)  # noqa: E731
    return {"UNet_Baseline": (local_only_block, local_only_block),
            "UNet_AttentionOnly": (attention_only_block, attention_only_block),
            "UNet_AdditionFusion": (addition_fusion_block, addition_fusion_block),
            "UNet_ConcatFusion": (concat_fusion_block, concat_fusion_block),
            "UNet_EncoderOnlyDFC": (dfc, local_only_block),
            "UNet_DecoderOnlyDFC": (local_only_block, dfc),
            "UNet_BothStandardConv": (local_only_block, local_only_block)}[model]


def conv_transpose2x2(x, sd, name):
    return F.conv_transpose2d(x, sd[name + ".weight"], sd[name + ".bias"], stride=2)


def unet_dfc_sa_res(x, sd, pool_size=8, training=True, bufs=None, full_res=False, zoo=None):
    """models/unet_dfc_sa_res.py:161-204 (UNetDFCSA.forward; UNetDFCSARes adds nothing).  With
    full_res: UNet_FullResAttention (AblationUNetBase.forward, unet_dfc_sa_ablation_branches.py:
    129-164, the same graph with FullResAttnDFCBlock blocks).  With zoo = an ablation model name:
    the same graph with that model's blocks (encoder + bottleneck, decoder)."""
    if zoo:
        enc, dec = _zoo_blocks(zoo)
        blk = lambda t, n: (enc if not n.startswith("up_conv") else dec)(t, sd, n, pool_size, training, bufs)  # noqa
    else:
        blk = lambda t, n: dfc_block(t, sd, n, pool_size, training, bufs, full_res)  # noqa: E731
    d1 = blk(x, "down1")
    d2 = blk(F.max_pool2d(d1, 2, 2), "down2")
    d3 = blk(F.max_pool2d(d2, 2, 2), "down3")
    d4 = blk(F.max_pool2d(d3, 2, 2), "down4")
    u = blk(F.max_pool2d(d4, 2, 2), "bottleneck")
    for lvl, skip in ((4, d4), (3, d3), (2, d2), (1, d1)):
        u = conv_transpose2x2(u, sd, f"up{lvl}")
        if u.shape[2:] != skip.shape[2:]:
            u = F.interpolate(u, size=skip.shape[2:], mode="bilinear", align_corners=False)
        u = blk(torch.cat([u, skip], dim=1), f"up_conv{lvl}")
    return conv(u, sd, "final_conv")


def unet(x, sd, training=True, bufs=None):
    """models/unet.py:69-101: DoubleConv (:6-18), Down = MaxPool2d(2, ceil_mode=True) + DoubleConv
    (:21-30), Up = ConvTranspose2d(k2, s2) -- or, bilinear=True (no up.weight in the state_dict),
    nn.Upsample(scale_factor=2, bilinear, align_corners=True) (:36-37) -- + crop + cat([skip, up])
    + DoubleConv (:33-58), OutConv 1x1 (:61-66)."""
    def dconv(t, n):
        for i in (0, 3):
            t = F.relu(batch_norm(conv(t, sd, f"{n}.conv.{i}", padding=1), sd, f"{n}.conv.{i + 1}", training, bufs))
        return t
    xs = [dconv(x, "inc")]
    for i in range(1, 5):
        xs.append(dconv(F.max_pool2d(xs[-1], 2, ceil_mode=True), f"down{i}.mpconv.1"))
    u = xs[4]
    for i, skip in zip(range(1, 5), (xs[3], xs[2], xs[1], xs[0])):
        if f"up{i}.up.weight" in sd:
            u = F.conv_transpose2d(u, sd[f"up{i}.up.weight"], sd[f"up{i}.up.bias"], stride=2)
        else:
            u = F.interpolate(u, scale_factor=2, mode="bilinear", align_corners=True)
        dy, dx = skip.shape[2] - u.shape[2], skip.shape[3] - u.shape[3]
        if dy < 0 or dx < 0:
            u = u[:, :, :skip.shape[2], :skip.shape[3]]
        else:
            skip = skip[:, :, dy // 2:dy // 2 + u.shape[2], dx // 2:dx // 2 + u.shape[3]]
        u = dconv(torch.cat([skip, u], dim=1), f"up{i}.conv")
    return conv(u, sd, "outc.conv")


# ------------------------------------------------------------------------------------------
# TransUNet R50-ViT (models/transformer_unet.py, BASELINE config 4), dropout p = 0 (eval-mode
# dropout; the fixtures are generated with dropout_rate 0)
# ------------------------------------------------------------------------------------------
def std_conv(x, w, stride=1, padding=0):
    """StdConv2d.forward :21-27: per-output-channel standardised weight (biased var, eps 1e-5)."""
    v, m = torch.var_mean(w, dim=[1, 2, 3], keepdim=True, unbiased=False)
    return F.conv2d(x, (w - m) / torch.sqrt(v + 1e-5), None, stride, padding)


def _gn(x, sd, name, groups, eps):
    return F.group_norm(x, groups, sd[name + ".weight"], sd[name + ".bias"], eps)


def bottleneck_unit(x, sd, n, stride):
    """PreActBottleneck.forward :58-68 (GroupNorm(32, .) eps 1e-6; gn_proj GroupNorm(C, C) eps 1e-5)."""
    cout = sd[n + ".conv3.weight"].shape[0]
    if (n + ".downsample.weight") in sd:
        res = _gn(std_conv(x, sd[n + ".downsample.weight"], stride), sd, n + ".gn_proj", cout, 1e-5)
    else:
        res = x
    y = F.relu(_gn(std_conv(x, sd[n + ".conv1.weight"]), sd, n + ".gn1", 32, 1e-6))
    y = F.relu(_gn(std_conv(y, sd[n + ".conv2.weight"], stride, 1), sd, n + ".gn2", 32, 1e-6))
    y = _gn(std_conv(y, sd[n + ".conv3.weight"]), sd, n + ".gn3", 32, 1e-6)
    return F.relu(res + y)


def vit_block(h, sd, n, heads):
    """Block.forward :211-220 with Attention :137-157 (scores / sqrt(head size)) and Mlp :167-173."""
    B, N, D = h.shape
    dh = D // heads
    x = F.layer_norm(h, (D,), sd[n + ".attention_norm.weight"], sd[n + ".attention_norm.bias"], 1e-6)

    def proj(t, name):
        return F.linear(t, sd[f"{n}.attn.{name}.weight"], sd[f"{n}.attn.{name}.bias"])

    q, k, v = (proj(x, nm).view(B, N, heads, dh).permute(0, 2, 1, 3) for nm in ("query", "key", "value"))
    a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(dh), dim=-1)
    c = (a @ v).permute(0, 2, 1, 3).reshape(B, N, D)
    h = proj(c, "out") + h
    x = F.layer_norm(h, (D,), sd[n + ".ffn_norm.weight"], sd[n + ".ffn_norm.bias"], 1e-6)
    x = F.linear(F.gelu(F.linear(x, sd[n + ".ffn.fc1.weight"], sd[n + ".ffn.fc1.bias"])),
                 sd[n + ".ffn.fc2.weight"], sd[n + ".ffn.fc2.bias"])
    return x + h


def transunet(x, sd, heads, n_skip=3, training=True, bufs=None):
    """TransUNet.forward :362-368: ResNetV2 hybrid (:97-106) -> Embeddings (:193-200) -> Encoder
    (:231-237) -> DecoderCup (:300-312, UpsamplingBilinear2d = bilinear align_corners=True) ->
    SegmentationHead 3x3 (:272-276)."""
    if x.shape[1] == 1:
        x = x.repeat(1, 3, 1, 1)
    hp = "transformer.embeddings.hybrid_model"
    r = F.relu(_gn(std_conv(x, sd[hp + ".root.conv.weight"], 2, 3), sd, hp + ".root.gn", 32, 1e-6))
    feats = [r]
    h = F.max_pool2d(r, 3, 2, 1)
    nblocks = 1 + max(int(k.split(".body.block")[1].split(".")[0]) for k in sd if ".body.block" in k) - 1
    for b in range(1, nblocks + 1):
        nunits = max(int(k.split(f".body.block{b}.unit")[1].split(".")[0]) for k in sd if f".body.block{b}.unit" in k)
        for u in range(1, nunits + 1):
            h = bottleneck_unit(h, sd, f"{hp}.body.block{b}.unit{u}", 2 if (u == 1 and b > 1) else 1)
        if b < nblocks:
            feats.append(h)
    feats = feats[::-1]
    e = F.conv2d(h, sd["transformer.embeddings.patch_embeddings.weight"],
                 sd["transformer.embeddings.patch_embeddings.bias"])
    B, D, gh, gw = e.shape
    t = e.flatten(2).transpose(-1, -2) + sd["transformer.embeddings.position_embeddings"]
    nl = 1 + max(int(k.split("encoder.layer.")[1].split(".")[0]) for k in sd if "encoder.layer." in k)
    for i in range(nl):
        t = vit_block(t, sd, f"transformer.encoder.layer.{i}", heads)
    t = F.layer_norm(t, (D,), sd["transformer.encoder.encoder_norm.weight"], sd["transformer.encoder.encoder_norm.bias"],
                     1e-6)
    u = t.permute(0, 2, 1).reshape(B, D, gh, gw)

    def conv_bn_relu(z, n):
        return F.relu(batch_norm(F.conv2d(z, sd[n + ".0.weight"], None, padding=1), sd, n + ".1", training, bufs))

    u = conv_bn_relu(u, "decoder.conv_more")
    nb = 1 + max(int(k.split("decoder.blocks.")[1].split(".")[0]) for k in sd if "decoder.blocks." in k)
    for i in range(nb):
        u = F.interpolate(u, scale_factor=2, mode="bilinear", align_corners=True)
        if i < n_skip:
            u = torch.cat([u, feats[i]], dim=1)
        u = conv_bn_relu(conv_bn_relu(u, f"decoder.blocks.{i}.conv1"), f"decoder.blocks.{i}.conv2")
    return F.conv2d(u, sd["segmentation_head.0.weight"], sd["segmentation_head.0.bias"], padding=1)


# ------------------------------------------------------------------------------------------
# loss and metrics
# ------------------------------------------------------------------------------------------
def bce_dice_loss(p, t, w_bce=1.0, w_dice=1.0, smooth=1.0):
    """utils/metrics.py:52-78 + :6-24: mean BCE (log clamped at -100 inside F.binary_cross_
    entropy) + Dice loss over the whole flattened batch."""
    bce = F.binary_cross_entropy(p, t)
    pf, tf = p.reshape(-1), t.reshape(-1)
    inter = (pf * tf).sum()
    dice = (2.0 * inter + smooth) / (pf.sum() + tf.sum() + smooth)
    return w_bce * bce + w_dice * (1 - dice)


def calculate_metrics(p, t, loss_type="bce_dice", loss_params=None):
    """utils/metrics.py:211-264 for loss_type 'bce_dice' (the type every config uses) and 'dice'
    (the Trainer's default type, :251-252).
    Note the reference reads 'weight_bce'/'weight_dice' (defaults 1.0), NOT the yaml's
    'bce_weight'/'dice_weight' keys."""
    if loss_type not in ("bce_dice", "dice"):
        raise ValueError(f"oracle only restates loss_types 'bce_dice' and 'dice', got {loss_type!r}")
    loss_params = loss_params or {}
    b = (p > 0.5).float()
    inter = (b * t).sum().item()
    union = (b + t).sum().item() - inter
    iou = inter / (union + 1e-7)
    dice = (2.0 * inter) / (b.sum().item() + t.sum().item() + 1e-7)
    if loss_type == "dice":   # utils/metrics.py:251-252 -> dice_loss :6-24
        loss = bce_dice_loss(p, t, 0.0, 1.0)
    else:
        loss = bce_dice_loss(p, t, loss_params.get("weight_bce", 1.0),
                             loss_params.get("weight_dice", 1.0))
    return {"loss": loss, "iou": iou, "dice": dice}


# ------------------------------------------------------------------------------------------
# the train step
# ------------------------------------------------------------------------------------------
def param_names(sd):
    """Trainable entries of a DFC-SA-Res state_dict (everything but BN buffers)."""
    return [k for k in sd if not (k.endswith("running_mean") or k.endswith("running_var")
                                  or k.endswith("num_batches_tracked"))]


def forward_backward(sd, x, t, pool_size, loss_params=None, model="dfc", heads=12):
    """fwd -> sigmoid -> calculate_metrics -> backward.  Returns (logits, metrics, grads,
    updated BN buffers).  model: 'dfc' (UNetDFCSARes), 'fullres' (UNet_FullResAttention), 'unet',
    'transunet' (TransUNet with `heads` attention heads), or an ablation-zoo model name
    ('UNet_Baseline', ...)."""
    params = {k: (v.detach().clone().requires_grad_(True) if k in set(param_names(sd)) else v)
              for k, v in sd.items()}
    bufs = {}
    if model == "unet":
        logits = unet(x, params, training=True, bufs=bufs)
    elif model == "transunet":
        logits = transunet(x, params, heads, training=True, bufs=bufs)
    elif model.startswith("UNet_"):
        logits = unet_dfc_sa_res(x, params, pool_size, training=True, bufs=bufs, zoo=model)
    else:
        logits = unet_dfc_sa_res(x, params, pool_size, training=True, bufs=bufs, full_res=(model == "fullres"))
    met = calculate_metrics(torch.sigmoid(logits), t, "bce_dice", loss_params)
    met["loss"].backward()
    grads = {k: params[k].grad.detach().clone() for k in param_names(sd)}
    return logits.detach(), met, grads, bufs


def clip_and_sgd(sd, grads, mom_bufs, lr=0.01, momentum=0.9, weight_decay=1e-4, max_norm=1.0):
    """torch.nn.utils.clip_grad_norm_ (utils/trainer.py:149) + torch.optim.SGD step
    (train.py:73-78): total L2 norm, coef = max_norm/(norm+1e-6) clamped to <= 1;
    d = g + wd*w; buf = d on the first step else momentum*buf + d; w -= lr*buf."""
    names = param_names(sd)
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(grads[k]) for k in names]))
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    new_sd = dict(sd)
    new_bufs = dict(mom_bufs)
    clipped = {}
    for k in names:
        g = grads[k] * coef
        clipped[k] = g
        d = g + weight_decay * sd[k]
        buf = d.clone() if k not in mom_bufs else momentum * mom_bufs[k] + d
        new_bufs[k] = buf
        new_sd[k] = sd[k] - lr * buf
    return new_sd, new_bufs, total, clipped


def train_step(sd, mom_bufs, x, t, pool_size, loss_params=None, lr=0.01, momentum=0.9,
               weight_decay=1e-4):
    logits, met, grads, bufs = forward_backward(sd, x, t, pool_size, loss_params)
    new_sd, new_bufs, norm, clipped = clip_and_sgd(sd, grads, mom_bufs, lr, momentum, weight_decay)
    new_sd.update(bufs)
    return new_sd, new_bufs, {"logits": logits, "norm": norm, "grads": clipped, **met}


def num_params(sd):
    return sum(sd[k].numel() for k in param_names(sd))


def gflop_per_image(features, H, pool_size):
    """Analytic fwd conv+bmm FLOPs per image (2*MACs), for documentation cross-checks."""
    f = features
    chans = [(None, f[0]), (f[0], f[1]), (f[1], f[2]), (f[2], f[3]), (f[3], 2 * f[3]),
             (2 * f[3], f[3]), (2 * f[2], f[2]), (2 * f[1], f[1]), (2 * f[0], f[0])]
    sizes = [H, H // 2, H // 4, H // 8, H // 16, H // 8, H // 4, H // 2, H]
    total = 0.0
    for (cin, cout), s in zip(chans, sizes):
        cin = 3 if cin is None else cin
        px = s * s
        total += px * cout * (9 * cin + cin + 2 * cout + 3 * cout + cin)
        n = pool_size * pool_size
        cq = cout // 8
        total += n * cout * (2 * cq + cout) + n * n * (cq + cout)
    for cin, s in ((2 * f[3], H // 16), (f[3], H // 8), (f[2], H // 4), (f[1], H // 2)):
        total += s * s * cin * (cin // 2) * 4
    total += H * H * f[0]
    return 2 * total / 1e9
