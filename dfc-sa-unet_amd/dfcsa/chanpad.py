"""Feature widths that are not multiples of 8, behind the reference's parameter shapes.

The reference accepts any ``features`` list (models/unet_dfc_sa_res.py:118-159, the ablation
models through AblationUNetBase, unet_dfc_sa_ablation_branches.py:104-164).  Every NHWC kernel
here moves 16-byte channel chunks, so an activation's channel count must be a multiple of 8.

A model built with such widths is first constructed exactly as the reference builds it (same
modules, same creation order, so the same default initialisation under a given seed); then
``pad_model`` zero-pads every channel dimension to the next multiple of 8, segment by segment
where a dimension is a concatenation (the skip concat [up | skip], the gate's [local | attn],
the fusion conv's [fused | local | attn]).  The padded channels stay exactly zero for the whole
of training:
  * a padded output channel has zero weight rows and zero bias, so its conv output is 0;
    train-mode BatchNorm of an all-zero channel is 0 (mean 0, variance 0) times gamma plus a
    zero beta; ReLU keeps 0; the sigmoid gate gives 0.5 but multiplies zero features;
  * every weight column that reads a padded channel is zero, so it adds nothing downstream, and
    its gradient (dy x_pad) is exactly 0 -- as are the gradients of the padded rows, bias, BN
    gamma / beta entries (their upstream gradient is the transpose of those zero columns);
  * weight decay and momentum of a zero parameter with a zero gradient stay zero, and the global
    gradient norm (clipping) is unchanged.
The query/key width C // 8 of the attention modules is padded like any other output width; the
attention energy is q.k over those channels, unscaled (reference :26-31), so zero channels do not
change it.

What the user sees stays the reference's: ``state_dict()`` (at any module level) returns the
logical shapes, ``load_state_dict`` accepts them (and padded ones), the FusedSGD momentum in
an optimizer state dict is logical-shaped.  ``named_parameters()`` and ``.grad`` hold the padded
storage; ``logical(p, t)`` slices a tensor of a parameter's padded shape back.
"""
import contextlib

import torch
import torch.nn as nn


def rup8(n):
    return (n + 7) // 8 * 8


# construction depth of the modules that pad their children themselves (the U-Net pads every block
# after the reference's construction, pad_model): a block or attention module built at depth 0 is
# standalone and pads itself (pad_standalone)
_BUILD = [0]


@contextlib.contextmanager
def building():
    _BUILD[0] += 1
    try:
        yield
    finally:
        _BUILD[0] -= 1


def standalone():
    return _BUILD[0] == 0


def build_inside(fn, *args, **kw):
    """fn(*args, **kw) with its blocks / attention modules marked as parts of a larger model."""
    with building():
        return fn(*args, **kw)


class Segs:
    """One channel dimension: logical widths of its concatenated segments; ``raw`` keeps them
    unpadded (the model's 3-channel image input and 1-channel logits, which the input pack and
    the 1x1 head already handle)."""

    def __init__(self, widths, raw=False):
        self.widths = list(widths)
        self.raw = raw

    @property
    def logical(self):
        return sum(self.widths)

    @property
    def padded(self):
        return self.logical if self.raw else sum(rup8(w) for w in self.widths)

    def index(self):
        """padded positions of the logical channels, in order"""
        idx, off = [], 0
        for w in self.widths:
            idx.extend(range(off, off + w))
            off += w if self.raw else rup8(w)
        return idx


class _Spec:
    """How one parameter / buffer is padded: {dim: Segs} plus its logical shape."""

    def __init__(self, shape, dims, fill=0.0):
        self.logical_shape = tuple(shape)
        self.dims = {d: s for d, s in dims.items() if s.padded != s.logical}
        self.fill = fill
        shp = list(shape)
        for d, s in dims.items():
            shp[d] = s.padded
        self.padded_shape = tuple(shp)

    def pad(self, t):
        for d, s in self.dims.items():
            shape = list(t.shape)
            shape[d] = s.padded
            out = torch.full(shape, self.fill, dtype=t.dtype, device=t.device)
            out.index_copy_(d, torch.tensor(s.index(), device=t.device), t)
            t = out
        return t

    def unpad(self, t):
        for d, s in self.dims.items():
            t = t.index_select(d, torch.tensor(s.index(), device=t.device))
        return t


def _state_dict_post_hook(module, state_dict, prefix, local_metadata):
    for name, spec in module._dfcsa_pad.items():
        key = prefix + name
        if key in state_dict and tuple(state_dict[key].shape) == spec.padded_shape:
            state_dict[key] = spec.unpad(state_dict[key].detach())


def _load_pre_hook(module, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs):
    for name, spec in module._dfcsa_pad.items():
        key = prefix + name
        if key in state_dict and tuple(state_dict[key].shape) == spec.logical_shape:
            state_dict[key] = spec.pad(state_dict[key])


def _pad_tensors(mod, dims_of):
    """Replace mod's parameters / buffers named in dims_of ({name: {dim: Segs}}) by padded copies
    and register the state_dict hooks that translate between the two shapes."""
    specs = {}
    for name, dims in dims_of.items():
        t = getattr(mod, name, None)
        if t is None:
            continue
        spec = _Spec(t.shape, dims, fill=1.0 if name == "running_var" else 0.0)
        if not spec.dims:
            continue
        with torch.no_grad():
            new = spec.pad(t.data)
        if isinstance(t, nn.Parameter):
            p = nn.Parameter(new, requires_grad=t.requires_grad)
            p._dfcsa_pad = spec
            setattr(mod, name, p)
        else:
            mod.register_buffer(name, new)
        specs[name] = spec
    if not specs:
        return
    if not hasattr(mod, "_dfcsa_pad"):
        mod.register_state_dict_post_hook(_state_dict_post_hook)
        mod.register_load_state_dict_pre_hook(_load_pre_hook)
        mod._dfcsa_pad = {}
    mod._dfcsa_pad.update(specs)


def _pad_conv(conv, out_segs, in_segs):
    if isinstance(conv, nn.ConvTranspose2d):          # weight [Cin, Cout, kh, kw]
        wd = {0: in_segs, 1: out_segs}
    else:                                             # weight [Cout, Cin, kh, kw]
        wd = {0: out_segs, 1: in_segs}
    _pad_tensors(conv, {"weight": wd, "bias": {0: out_segs}})
    conv._dfcsa_logical = (in_segs.logical, out_segs.logical)
    conv.out_channels, conv.in_channels = out_segs.padded, in_segs.padded


def _pad_bn(bn, segs):
    d = {0: segs}
    _pad_tensors(bn, {"weight": d, "bias": d, "running_mean": d, "running_var": d})
    bn.num_features = segs.padded


def pad_block(block, in_segs, C):
    """Pad one U-Net block (the DFC block or an ablation block: every block class of the
    reference's models shares the submodule names used here) whose input is the concatenation
    ``in_segs`` and whose output width is C."""
    out = Segs([C])
    for name, mod in block.named_modules():
        leaf = name.rsplit(".", 1)[-1]
        if isinstance(mod, nn.Conv2d):
            if leaf in ("query_conv", "key_conv"):
                if mod.out_channels < 1:
                    raise ValueError(f"feature width {C}: the attention's C // 8 query/key width is 0")
                _pad_conv(mod, Segs([mod.out_channels]), out)
            elif leaf == "value_conv":
                _pad_conv(mod, out, out)
            elif name.startswith(("conv_branch.", "attn_branch.0")) or name == "residual_conv":
                _pad_conv(mod, out, in_segs)
            elif name.startswith(("gate.", "fusion_conv.")):
                k, r = divmod(mod.in_channels, C)
                if r:
                    raise NotImplementedError(f"{name}: {mod.in_channels} input channels over width {C}")
                _pad_conv(mod, out, Segs([C] * k))
            else:
                raise NotImplementedError(f"channel padding: unknown conv {name!r} in {type(block).__name__}")
        elif isinstance(mod, nn.BatchNorm2d):
            _pad_bn(mod, out)
        elif isinstance(mod, nn.ConvTranspose2d):
            raise NotImplementedError(f"channel padding: unexpected {name!r} in {type(block).__name__}")


def pad_standalone(mod, cin, cout):
    """A DFC block (cin -> cout) or a LightSelfAttention / FullResolutionAttention (cin = cout = C)
    built on its own, outside a U-Net (reference models/unet_dfc_sa_res.py:5-116 accepts any
    width): zero-pad it like pad_block when cout is not a multiple of 8.  Its standalone forward
    takes the logical NCHW input (padded to a multiple of 8 on the way in) and returns the logical
    cout channels (``mod._dfcsa_out``).  cout % 8 == 0 needs nothing: the input side's padding is the
    NCHW -> NHWC pack's."""
    if cout % 8 == 0:
        return
    pad_block(mod, Segs([cin]), cout)
    mod._dfcsa_out = cout


def pad_model(model, features, in_channels, out_channels):
    """Pad a UNetDFCSA-family model (UNetDFCSA / UNetDFCSARes, UNet_FullResAttention and the
    ablation zoo): block inputs follow the forward's wiring (reference :118-204)."""
    f = list(features)
    src = Segs([in_channels], raw=True)
    for name, cin, c in (("down1", src, f[0]), ("down2", Segs([f[0]]), f[1]), ("down3", Segs([f[1]]), f[2]),
                         ("down4", Segs([f[2]]), f[3]), ("bottleneck", Segs([f[3]]), 2 * f[3]),
                         ("up_conv4", Segs([f[3], f[3]]), f[3]), ("up_conv3", Segs([f[2], f[2]]), f[2]),
                         ("up_conv2", Segs([f[1], f[1]]), f[1]), ("up_conv1", Segs([f[0], f[0]]), f[0])):
        pad_block(getattr(model, name), cin, c)
    for name, cin, c in (("up4", 2 * f[3], f[3]), ("up3", f[3], f[2]), ("up2", f[2], f[1]), ("up1", f[1], f[0])):
        _pad_conv(getattr(model, name), Segs([c]), Segs([cin]))
    _pad_conv(model.final_conv, Segs([out_channels], raw=True), Segs([f[0]]))


def io_channels(conv):
    """(in_channels, out_channels) of a conv as the reference built it (before padding)."""
    return getattr(conv, "_dfcsa_logical", (conv.in_channels, conv.out_channels))


def numel(p):
    """Element count of parameter p in its reference shape."""
    spec = getattr(p, "_dfcsa_pad", None)
    return p.numel() if spec is None else int(torch.Size(spec.logical_shape).numel())


def logical(p, t=None):
    """``t`` (default ``p.data``), a tensor of parameter p's stored shape, in p's reference shape."""
    t = p.data if t is None else t
    spec = getattr(p, "_dfcsa_pad", None)
    return t if spec is None else spec.unpad(t)


def padded(p, t):
    """A tensor of parameter p's reference shape, in p's stored (padded) shape."""
    spec = getattr(p, "_dfcsa_pad", None)
    if spec is None or tuple(t.shape) == spec.padded_shape:
        return t
    return spec.pad(t)
