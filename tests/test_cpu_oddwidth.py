"""Feature widths that are not multiples of 8 (dfcsa/chanpad.py; the reference accepts any width,
models/unet_dfc_sa_res.py:118-159): host-side checks against the reference's own models at
features 10, 12, 20, 27 (tests/golden/oddw_*.npz, make_golden.py gen_oddwidth).

  * the build consumes the seed exactly as the reference does: the fresh state dict equals the
    reference's, key for key, shape for shape and value for value;
  * state_dict() is logical at every module level; load_state_dict round-trips bitwise; the
    padded storage is zero outside the logical channels and every stored channel dimension is a
    multiple of 8 (what the NHWC kernels address);
  * the FusedSGD state dict translates momentum buffers between the two shapes.
"""
import numpy as np
import pytest
import torch

ODD = ("UNetDFCSARes", "UNet_ConcatFusion", "UNet_DecoderOnlyDFC", "UNet_FullResAttention", "UNet_AttentionOnly")
FEATURES = [10, 12, 20, 27]


def odd_model(name):
    from models.model_factory import ModelFactory
    fname = "DFC-SA-Res-Block" if name == "UNetDFCSARes" else name
    return ModelFactory.get_model({"model": {"name": fname, "features": FEATURES, "pool_size": 4}, "training": {}})


def sd_of(fx, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.asarray(fx[k])) for k in fx if k.startswith(prefix)}


@pytest.mark.parametrize("i,name", list(enumerate(ODD)))
def test_odd_width_init_matches_reference(golden, i, name):
    fx = golden(f"oddw_{name}.npz")
    ref = sd_of(fx, "sd0.")
    ref.update(sd_of(fx, "initg."))   # the fixture perturbed the gammas after recording them
    torch.manual_seed(9500 + i)
    m = odd_model(name)
    got = m.state_dict()
    assert list(got) == list(ref)
    for k, v in ref.items():
        assert tuple(got[k].shape) == tuple(v.shape), k
        assert torch.equal(got[k], v.to(got[k].dtype)), k


@pytest.mark.parametrize("name", ODD)
def test_odd_width_storage_and_roundtrip(golden, name):
    from dfcsa import chanpad
    fx = golden(f"oddw_{name}.npz")
    ref = sd_of(fx, "sd0.")
    m = odd_model(name)
    m.load_state_dict(ref)
    got = m.state_dict()
    assert all(torch.equal(got[k], v.to(got[k].dtype)) for k, v in ref.items())
    npad = 0
    for n, p in m.named_parameters():
        spec = getattr(p, "_dfcsa_pad", None)
        if spec is None:
            continue
        npad += 1
        assert tuple(chanpad.logical(p).shape) == tuple(ref[n].shape), n
        # zero outside the logical channels: the padded tensor re-padded from its logical slice
        assert torch.equal(spec.pad(chanpad.logical(p)), p.data), n
        for d in spec.dims:
            assert p.shape[d] % 8 == 0, (n, tuple(p.shape))
    assert npad > 0
    # submodule-level state dicts are logical too
    blk = m.down2
    for k, v in blk.state_dict().items():
        assert tuple(v.shape) == tuple(ref["down2." + k].shape), k
    # a padded model's conv sees multiples of 8 on both sides except the image input and logits
    for n, mod in m.named_modules():
        if isinstance(mod, (torch.nn.Conv2d, torch.nn.ConvTranspose2d)):
            assert mod.out_channels % 8 == 0 or n == "final_conv", n
            assert mod.in_channels % 8 == 0 or n.startswith("down1."), n


def test_odd_width_optimizer_state_translation(golden):
    """FusedSGD.state_dict / load_state_dict with padded parameters: logical momentum out, padded
    momentum in (the flat momentum storage itself needs the GPU; the translation does not)."""
    from dfcsa import chanpad
    fx = golden("oddw_UNetDFCSARes.npz")
    m = odd_model("UNetDFCSARes")
    m.load_state_dict(sd_of(fx, "sd0."))
    mom = sd_of(fx, "mom1.")
    for n, p in m.named_parameters():
        b = chanpad.padded(p, mom[n])
        assert b.shape == p.shape, n
        assert torch.equal(chanpad.logical(p, b), mom[n]), n


@pytest.mark.parametrize("fname", ["oddw_lsa_C12_P4.npz", "oddw_lsa_C20_P8.npz", "oddw_lsa_C27_P16.npz",
                                   "oddw_block_5to12_P4.npz", "oddw_block_12to20_P8.npz", "oddw_block_16to27_P4.npz"])
def test_standalone_odd_width_init_and_storage(golden, fname):
    """A block / attention module built on its own at a width that is not a multiple of 8: the fresh
    state dict equals the reference's under the same seed (key, shape and value); the stored
    parameters are padded to multiples of 8 (zeros outside the logical channels); load_state_dict of
    the reference's shapes round-trips bitwise."""
    from test_gpu_oddwidth import standalone_module
    fx = golden(fname)
    ref = sd_of(fx, "sd0.")
    m = standalone_module(fname)
    got = m.state_dict()
    assert list(got) == list(ref)
    for k, v in ref.items():
        assert tuple(got[k].shape) == tuple(v.shape), k
        assert torch.equal(got[k], v.to(got[k].dtype)), k
    for n, p in m.named_parameters():
        if p.dim() > 1:
            assert p.shape[0] % 8 == 0 and (p.shape[1] % 8 == 0 or n.endswith("conv_branch.0.weight")
                                           or n.endswith("attn_branch.0.weight") or n.endswith("residual_conv.weight")), n
    m.load_state_dict(ref)
    assert all(torch.equal(a, ref[k].to(a.dtype)) for k, a in m.state_dict().items())
