"""CPU-only tests: the C-ABI library and the host-side logic (no GPU compute here)."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dfcsa.h")
LIB = os.path.join(ROOT, "dfc-sa-unet_amd", "libdfcsa.so")


def header_symbols():
    text = re.sub(r"/\*.*?\*/", " ", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(dfcsa_\w+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    assert os.path.exists(LIB), "build libdfcsa.so first (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dfcsa_\w+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    assert len(header_symbols()) >= 50


def test_ctypes_binding_loads_and_parses_header():
    from dfcsa import _lib
    assert set(_lib.PROTOS) == set(header_symbols())
    assert _lib.version().startswith("libdfcsa")
    for name in _lib.PROTOS:
        assert getattr(_lib.LIB, name).argtypes is not None


def test_descriptor_layouts_match_c(tmp_path):
    from dfcsa import _lib
    fields = [("dfcsa_conv_desc", _lib.ConvDesc, ("weight", "Wout")),
              ("dfcsa_wgrad_desc", _lib.WgradDesc, ("slab", "mchunk", "ndst", "dst", "bias_dst")),
              ("dfcsa_pack_entry", _lib.PackEntry, ("w0", "a")),
              ("dfcsa_wstd_entry", _lib.WstdEntry, ("K", "pad")),
              ("dfcsa_resample_desc", _lib.ResampleDesc, ("kk", "row0")),
              ("dfcsa_aug_desc", _lib.AugDesc, ("m", "fix", "rotate", "mask_w")),
              ("dfcsa_pool_contract", _lib.PoolContract, ("rows", "H", "P")),
              ("dfcsa_bn_fold", _lib.BnFold, ("conv_bias", "num_batches_tracked", "momentum", "eps", "scale",
                                              "invstd"))]
    exprs = []
    want = []
    for cname, py, names in fields:
        exprs.append(f"sizeof({cname})")
        want.append(ctypes.sizeof(py))
        for n in names:
            exprs.append(f"offsetof({cname}, {n})")
            want.append(getattr(py, n).offset)
    src = tmp_path / "lay.c"
    src.write_text('#include "dfcsa.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(){'
                   + "".join(f'printf("%zu\\n", (size_t){e});' for e in exprs) + "}\n")
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == want


def test_host_side_planning_functions():
    """Pure host entry points (no device work) can run without a GPU."""
    from dfcsa._lib import LIB as L
    s, mc, fl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    A = ctypes.addressof
    assert L.dfcsa_wgrad_plan(802816, 64, 1152, 1, A(s), A(mc), A(fl)) == 0
    assert mc.value % 64 == 0 and s.value * mc.value >= 802816 and (s.value - 1) * mc.value < 802816
    assert fl.value >= s.value * 64 * 1152
    assert L.dfcsa_wgrad_plan(3136, 1024, 4608, 0, A(s), A(mc), A(fl)) == 0
    assert mc.value % 32 == 0 and s.value >= 1
    # a deep bf16 layer: few splits; the slab also covers the tile-ordered partials of the
    # in-kernel reduction (off by default: dfcsa_wgrad_fuse_max() == 0, tuning knob 13)
    assert L.dfcsa_wgrad_plan(3136, 1024, 4608, 1, A(s), A(mc), A(fl)) == 0
    assert 1 < s.value <= 16 and fl.value >= s.value * 1024 * 4608
    assert L.dfcsa_wgrad_fuse_max() == 0
    assert L.dfcsa_wgrad_plan(0, 1, 1, 1, A(s), A(mc), A(fl)) != 0
    assert L.dfcsa_ew_ntiles(802816, 64) == 3136   # 16384-element tiles: 256 pixels of 64 channels
    assert L.dfcsa_lsa_pool_splits(224, 4) >= 1 and L.dfcsa_lsa_pool_splits(14, 32) == 1
    assert 1 <= L.dfcsa_sumsq_nparts(29052083) <= 1024
    assert L.dfcsa_bce_dice_partial_count(16 * 224 * 224) == 512


def test_state_dict_matches_reference_layout(golden):
    from models.unet_dfc_sa_res import UNetDFCSARes
    fx = golden("model_small.npz")
    m = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4)
    ref_keys = [k[4:] for k in fx if k.startswith("sd0.")]
    assert sorted(m.state_dict().keys()) == sorted(ref_keys)
    for k, v in m.state_dict().items():
        assert tuple(v.shape) == fx["sd0." + k].shape, k
    big = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4)
    assert len(big.state_dict()) == 343
    assert sum(p.numel() for p in big.parameters()) == 29052083


def test_seeded_init_matches_oracle_param_count():
    from models.unet_dfc_sa_res import UNetDFCSARes
    from oracle import dfcsa_oracle as O
    torch.manual_seed(0)
    m = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4)
    assert O.num_params(m.state_dict()) == sum(p.numel() for p in m.parameters())


def test_model_factory_contract():
    from models.model_factory import ModelFactory
    cfg = {"model": {"name": "DFC-SA-Res-Block", "features": [8, 16, 32, 64], "pool_size": 4}, "training": {}}
    m = ModelFactory.get_model(cfg)
    assert type(m).__name__ == "UNetDFCSARes" and m.pool_size == 4
    assert m.compute_dtype == torch.bfloat16
    cfg32 = {"model": dict(cfg["model"], precision="fp32"), "training": {}}
    assert ModelFactory(cfg32).create_model().compute_dtype == torch.float32
    with pytest.raises(ValueError):
        ModelFactory().create_model()
    with pytest.raises(ValueError):
        ModelFactory.get_model({"model": {"name": "NoSuchModel"}, "training": {}})
    with pytest.raises(NotImplementedError):
        ModelFactory.get_model({"model": {"name": "VisionTransformerSegmentation"}, "training": {}})
    # config_transunet.yaml: 'TransformerUNet', img_size from the dataset section (:113-137)
    tu = ModelFactory.get_model({"model": {"name": "TransformerUNet", "in_channels": 3, "out_channels": 1},
                                 "dataset": {"img_size": [224, 224]}, "training": {}})
    assert type(tu).__name__ == "TransUNet" and tu.config.patches.grid == (14, 14)
    assert sum(p.numel() for p in tu.parameters()) == 105275921
    # defaults (model_factory.py:87-91): pool 8, qk ratio 8, features 64..512
    d = ModelFactory.get_model({"model": {"name": "DFC-SA-Res-Block"}, "training": {}})
    assert d.pool_size == 8 and d.down1.attn_branch[3].query_conv.out_channels == 8


def test_ablation_zoo_state_dicts_match_reference(golden):
    """Every ablation model (model_factory.py:160-187) builds with the reference's module tree:
    state_dict keys and shapes of the fixture (features 8..64) and the full-size parameter count."""
    from models.model_factory import ModelFactory
    for name in ("UNet_Baseline", "UNet_AttentionOnly", "UNet_AdditionFusion", "UNet_ConcatFusion",
                 "UNet_EncoderOnlyDFC", "UNet_DecoderOnlyDFC", "UNet_BothStandardConv"):
        fx = golden(f"zoo_{name}.npz")
        m = ModelFactory.get_model({"model": {"name": name, "features": [8, 16, 32, 64], "pool_size": 4},
                                    "training": {}})
        ref = {k[4:]: fx[k].shape for k in fx if k.startswith("sd0.")}
        got = {k: tuple(v.shape) for k, v in m.state_dict().items()}
        assert got == ref, name
        full = ModelFactory.get_model({"model": {"name": name}, "training": {}})
        assert sum(p.numel() for p in full.parameters()) == int(fx["nparams_full"]), name


def test_pretrained_failure_is_reported_not_raised(tmp_path, capsys):
    from models.model_factory import ModelFactory
    cfg = {"model": {"name": "DFC-SA-Res-Block", "features": [8, 16, 32, 64],
                     "pretrained_path": str(tmp_path / "missing.pth")}, "training": {}}
    ModelFactory.get_model(cfg)
    assert "載入預訓練權重失敗" in capsys.readouterr().out


def test_pretrained_roundtrip(tmp_path):
    from models.model_factory import ModelFactory
    cfg = {"model": {"name": "DFC-SA-Res-Block", "features": [8, 16, 32, 64]}, "training": {}}
    torch.manual_seed(1)
    a = ModelFactory.get_model(cfg)
    torch.save(a.state_dict(), tmp_path / "w.pth")
    cfg["model"]["pretrained_path"] = str(tmp_path / "w.pth")
    torch.manual_seed(2)
    b = ModelFactory.get_model(cfg)
    assert all(torch.equal(a.state_dict()[k], b.state_dict()[k]) for k in a.state_dict())


def test_no_cpu_fallback():
    from models.unet_dfc_sa_res import UNetDFCSARes
    m = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4)
    with pytest.raises(RuntimeError, match="MI355X"):
        m(torch.randn(1, 3, 32, 32))


def test_metrics_loss_types():
    from utils.metrics import calculate_metrics
    p, t = torch.rand(1, 1, 4, 4), torch.ones(1, 1, 4, 4)
    with pytest.raises(ValueError):
        calculate_metrics(p, t, "no-such-loss")
    with pytest.raises(NotImplementedError):
        calculate_metrics(p, t, "tversky")
    with pytest.raises(RuntimeError):  # bce_dice on host tensors: no CPU fallback
        calculate_metrics(p, t, "bce_dice")
    with pytest.raises(RuntimeError):  # 'dice' runs on the same kernel: no CPU fallback either
        calculate_metrics(p, t, "dice")


def test_flat_params_views_and_grads():
    from dfcsa.flat import ALIGN, FlatParams
    net = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Linear(7, 3))
    before = [p.detach().clone() for p in net.parameters()]
    flat = FlatParams(net)
    assert flat.valid()
    for p, b, off in zip(net.parameters(), before, flat.offsets):
        assert torch.equal(p.detach(), b) and off % ALIGN == 0
        assert p.data_ptr() == flat.data.data_ptr() + 4 * off
    flat.grad.fill_(1.0)
    for p in net.parameters():
        p.grad = None
    flat.attach_grads()
    assert all(torch.all(p.grad == 0) for p in net.parameters())  # None -> zeroed view
    net[0].weight.grad.fill_(2.0)
    flat.zero_grad()
    assert torch.all(flat.grad == 0)


def test_ddp_bucket_plan():
    from dfcsa.ddp import GradBucketReducer

    class FakeFlat:
        def __init__(self, n):
            self.grad = torch.zeros(n)

    class FakeModel:
        def __init__(self, sizes):
            self.mods = [torch.nn.Module() for _ in sizes]
            o, self.units = 0, []
            for m, s in zip(self.mods, sizes):
                self.units.append((m, o, o + s))
                o += s
            self.flat = FakeFlat(o)

        def flat_params(self):
            return self.flat

        def grad_units(self):
            return self.units

    import torch.distributed as dist
    model = FakeModel([10, 20, 30, 1000, 5])
    orig = dist.get_world_size
    dist.get_world_size = lambda group=None: 2
    try:
        r = GradBucketReducer(model, bucket_mb=100 * 4 / (1 << 20))  # 100-float buckets
    finally:
        dist.get_world_size = orig
    spans = [(lo, hi) for lo, hi, _ in r.buckets]
    assert spans[0][1] == 1065 and spans[-1][0] == 0          # from the end of the buffer
    assert all(a[0] == b[1] for a, b in zip(spans, spans[1:]))  # contiguous, no gaps
    assert r.grad_scale == 0.5

    # ARMED accounting: one count per armed reducer whatever happens between start()
    # and finish() -- a failed pass (abort), a re-arm without finish, an exception inside finish()
    from dfcsa import ddp as D
    base = D.ARMED[0]
    r.start()
    assert D.ARMED[0] == base + 1
    r.abort()
    assert D.ARMED[0] == base and r._pending is None
    r.abort()                                   # idempotent
    assert D.ARMED[0] == base
    r.start()
    r.start()                                   # re-arming does not leak a count
    assert D.ARMED[0] == base + 1

    class Boom:
        def wait(self):
            raise RuntimeError("collective failed")
    r._works = [Boom() for _ in r.buckets]
    with pytest.raises(RuntimeError):
        r.finish()
    assert D.ARMED[0] == base and r._pending is None


def _ddp_worker(rank, world, port, out_q):
    import torch.distributed as dist
    sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dfcsa.ddp import GradBucketReducer, shard_rows
        from dfcsa.flat import FlatParams
        from models.unet_dfc_sa_res import UNetDFCSARes
        from oracle import dfcsa_oracle as O
        fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "model_small.npz")))
        dd = dict(np.load(os.path.join(ROOT, "tests", "golden", "ddp_shards.npz")))
        sd = {k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")}
        model = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4)
        model.load_state_dict(sd)
        model._flat = FlatParams(model)
        red = GradBucketReducer(model, bucket_mb=0.25)
        x, t = torch.from_numpy(dd["x"]), torch.from_numpy(dd["t"])
        lo, hi = shard_rows(x.shape[0], rank, world)
        # the oracle stands in for the GPU backward: per-shard grads, written into the flat buffer
        _, _, grads, _ = O.forward_backward(sd, x[lo:hi], t[lo:hi], 4)
        red.start()
        named = dict(model.named_parameters())
        for mod, _, _ in reversed(model.grad_units()):      # backward order: last module first
            for n, p in named.items():
                if any(p is q for q in mod.parameters()):
                    p.grad.copy_(grads[n])
            red.unit_ready(mod)
        # NaN agreement: rank 1 reports a NaN loss, every rank gets the NaN skip scalar
        loss = torch.tensor(float("nan") if rank == 1 else 0.5)
        skip = red.finish(loss)
        nan_agreed = bool(torch.isnan(skip).all())
        worst = 0.0
        for n, p in named.items():
            ref = torch.from_numpy(dd[f"w{world}.mean_grad.{n}"]).double()
            g = p.grad.double() * red.grad_scale
            if n.endswith(("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias", "fusion_conv.0.bias",
                           "key_conv.bias")):
                continue
            worst = max(worst, ((g - ref).norm() / (ref.norm() + 1e-30)).item())
        red.start()
        ok_skip = red.finish(torch.tensor(float("inf")))   # inf is not NaN: the reference still steps
        inf_steps = bool((ok_skip == 0).all())
        # buffer broadcast: rank-specific running stats -> rank 0's everywhere
        with torch.no_grad():
            for b in model.buffers():
                if b.is_floating_point():
                    b.fill_(float(rank + 1))
        red.broadcast_buffers()
        bufs_ok = all(bool((b == 1.0).all()) for b in model.buffers() if b.is_floating_point())
        out_q.put((rank, (worst, nan_agreed, inf_steps, bufs_ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_ddp_gloo_two_ranks_matches_sharded_reference():
    """world_size 2 over gloo: bucketed all-reduce of the flat gradient buffer reproduces the
    reference's mean of per-shard gradients (tests/golden/ddp_shards.npz)."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=500) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in (0, 1):
        worst, nan_agreed, inf_steps, bufs_ok = res[r]
        assert worst < 1e-3, res
        assert nan_agreed and inf_steps and bufs_ok, res


def test_cfg2_seeded_init_matches_reference(golden):
    """The config-2 parity test (tests/test_gpu_parity2.py) rebuilds the reference's 29 M-parameter
    model from its seed instead of storing it: same module tree, creation order and init."""
    from models.unet_dfc_sa_res import UNetDFCSARes
    fx = golden("cfg2_step.npz")
    torch.manual_seed(12000)
    m = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4, ablation_on_qk_channels=8)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    assert sum(p.numel() for p in m.parameters()) == int(fx["nparams"])
    for k, v in m.state_dict().items():
        if v.is_floating_point():
            want = float(fx["init_sum." + k])
            assert abs(v.double().sum().item() - want) <= 1e-6 * max(1.0, abs(want)), k


def test_reference_checkpoint_loads_weights_only():
    """The reference-written checkpoint (its Trainer.save_checkpoint, trainer.py:267-298) loads with
    the non-executing loader and its model state fits our module tree key for key."""
    from models.unet_dfc_sa_res import UNetDFCSARes
    ck = torch.load(os.path.join(ROOT, "tests", "golden", "ref_checkpoint_epoch_1.pth"), weights_only=True)
    m = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4)
    m.load_state_dict(ck["model_state_dict"])
    assert set(ck["metrics"]) == {"loss", "iou", "dice", "best_samples", "worst_samples"}
    assert len(ck["optimizer_state_dict"]["state"]) == len(list(m.parameters()))


@pytest.mark.parametrize("features,pool,hw,full_res", [((8, 16, 32, 64), 4, 32, False), ((8, 16, 32, 64), 8, 48, False),
                                                       ((10, 12, 20, 27), 4, 32, False), ((10, 12, 20, 27), 4, 32, True),
                                                       ((8, 16, 16, 32), 4, 16, True)])
def test_model_stats_flops_match_flop_counter(features, pool, hw, full_res):
    """utils.model_stats.forward_flops (analytic walk of the GPU model's module tree) against
    torch.utils.flop_counter on the CPU restatement of the same forward (oracle/dfcsa_oracle.py),
    and parameter totals / serialized size (reference model_stats.py:15-43)."""
    from torch.utils.flop_counter import FlopCounterMode

    from models.model_factory import ModelFactory
    from oracle import dfcsa_oracle as O
    from utils import model_stats as S
    name = "UNet_FullResAttention" if full_res else "DFC-SA-Res-Block"
    cfg = {"model": {"name": name, "features": list(features), "pool_size": pool}, "training": {}}
    m = ModelFactory.get_model(cfg)
    sd = {k: v.detach().float() for k, v in m.state_dict().items()}
    x = torch.randn(2, 3, hw, hw)
    with FlopCounterMode(display=False) as fc:
        with torch.no_grad():
            O.unet_dfc_sa_res(x, sd, pool_size=pool, training=True, bufs=None, full_res=full_res)
    ref = fc.get_total_flops()
    ours = S.forward_flops(m, (2, 3, hw, hw))
    assert abs(ours - ref) <= 1e-9 * ref, (ours, ref)
    ps = S.count_parameters(m)
    # reference-shape totals (equal to the stored ones unless widths were channel-padded)
    assert ps["total"] == sum(v.numel() for k, v in sd.items() if "running" not in k and "num_batches" not in k) \
        == ps["trainable"]
    assert 0 < S.get_model_size(m) < 10


ZOO_NAMES = ["UNet_Baseline", "UNet_AttentionOnly", "UNet_AdditionFusion", "UNet_ConcatFusion",
             "UNet_EncoderOnlyDFC", "UNet_DecoderOnlyDFC", "UNet_BothStandardConv"]


@pytest.mark.parametrize("name", ZOO_NAMES)
def test_model_stats_flops_zoo(name):
    """forward_flops of every ablation-zoo model (the reference counts each with ptflops,
    model_stats.py:164-165) against torch.utils.flop_counter on the oracle's restatement of the
    same graph with that model's blocks."""
    from torch.utils.flop_counter import FlopCounterMode

    from models.model_factory import ModelFactory
    from oracle import dfcsa_oracle as O
    from utils import model_stats as S
    cfg = {"model": {"name": name, "features": [8, 16, 32, 64], "pool_size": 4}, "training": {}}
    m = ModelFactory.get_model(cfg)
    sd = {k: v.detach().float() for k, v in m.state_dict().items()}
    x = torch.randn(2, 3, 32, 32)
    with FlopCounterMode(display=False) as fc:
        with torch.no_grad():
            O.unet_dfc_sa_res(x, sd, pool_size=4, training=True, bufs=None, zoo=name)
    ref = fc.get_total_flops()
    ours = S.forward_flops(m, (2, 3, 32, 32))
    assert abs(ours - ref) <= 1e-9 * ref, (ours, ref)


@pytest.mark.parametrize("hw", [64, 37])
def test_model_stats_flops_unet(hw):
    """forward_flops of UNet (config 1; odd sizes exercise the ceil-mode pooling and the crop)
    against torch.utils.flop_counter on the oracle's UNet."""
    from torch.utils.flop_counter import FlopCounterMode

    from models.model_factory import ModelFactory
    from oracle import dfcsa_oracle as O
    from utils import model_stats as S
    m = ModelFactory.get_model({"model": {"name": "UNet"}, "training": {}})
    sd = {k: v.detach().float() for k, v in m.state_dict().items()}
    x = torch.randn(1, 3, hw, hw)
    with FlopCounterMode(display=False) as fc:
        with torch.no_grad():
            O.unet(x, sd, training=True, bufs=None)
    ref = fc.get_total_flops()
    ours = S.forward_flops(m, (1, 3, hw, hw))
    assert abs(ours - ref) <= 1e-9 * ref, (ours, ref)


def test_model_stats_flops_transunet():
    """forward_flops of TransUNet on the reduced R50-ViT config of the fixtures (32x32 input, two
    ViT layers) against torch.utils.flop_counter on the oracle's TransUNet."""
    from torch.utils.flop_counter import FlopCounterMode

    from models.transformer_unet import TransUNet
    from oracle import dfcsa_oracle as O
    from test_oracle_golden import transunet_small_config
    from utils import model_stats as S
    c = transunet_small_config()
    m = TransUNet(c, img_size=32, num_classes=1)
    sd = {k: v.detach().float() for k, v in m.state_dict().items()}
    x = torch.randn(2, 3, 32, 32)
    with FlopCounterMode(display=False) as fc:
        with torch.no_grad():
            O.transunet(x, sd, heads=c.transformer.num_heads, training=True, bufs=None)
    ref = fc.get_total_flops()
    ours = S.forward_flops(m, (2, 3, 32, 32))
    assert abs(ours - ref) <= 1e-9 * ref, (ours, ref)


def test_model_stats_headline_flops_pinned():
    """The config-2 model at 224^2, P=4: 67.29 GFLOP per image forward (measured there
    with torch.utils.flop_counter on the reference) -- fwd+bwd 201.66 = 3x forward minus the input
    gradient of the first block."""
    from models.model_factory import ModelFactory
    from utils import model_stats as S
    m = ModelFactory.get_model({"model": {"name": "DFC-SA-Res-Block", "features": [64, 128, 256, 512],
                                          "pool_size": 4}, "training": {}})
    f = S.forward_flops(m, (1, 3, 224, 224))
    assert abs(f / 1e9 - 67.29) < 0.01, f / 1e9


def test_shard_rows_ragged_and_weights():
    """ragged global batches split as evenly as possible (the last ranks may get none); the
    per-rank loss weights make (sum of weighted replica gradients) / world the row-weighted mean."""
    from dfcsa.ddp import shard_rows, shard_weight
    for n in (1, 3, 7, 8, 16, 17):
        for world in (1, 2, 3, 8):
            spans = [shard_rows(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
            ws = [shard_weight(n, r, world) for r in range(world)]
            assert abs(sum(ws) / world - 1.0) < 1e-12
            assert all(abs(w * world / world - s / n * world) < 1e-12 for w, s in zip(ws, sizes))
            if n % world == 0:
                assert all(w == 1.0 for w in ws)


def test_rank_sharded_loader_partitions_global_batches():
    """Every rank draws the same global permutation (seed + epoch, independent of the global RNG) and
    loads only its rows; the ranks' rows of each batch together are that global batch; a rank without
    rows in a batch gets a placeholder carrying global_rows."""
    from utils.data_loader import RankShardedLoader

    class DS(torch.utils.data.Dataset):
        def __len__(self):
            return 9

        def __getitem__(self, i):
            return {"image": torch.full((1, 2, 2), float(i)), "mask": torch.zeros(1, 2, 2)}

    world = 4
    for epoch in (0, 1):
        per_rank = []
        for r in range(world):
            torch.manual_seed(1000 + r)   # a rank's own RNG state must not matter
            ld = RankShardedLoader(DS(), 5, r, world, seed=3)
            ld.set_epoch(epoch)
            per_rank.append(list(ld))
        glob = RankShardedLoader(DS(), 5, 0, world, seed=3)
        glob.set_epoch(epoch)
        gb = glob.global_batches()
        assert len(gb) == 2 and [len(b) for b in gb] == [5, 4]
        for bi, b in enumerate(gb):
            got = []
            for r in range(world):
                batch = per_rank[r][bi]
                assert batch["global_rows"] == len(b)
                if batch["image"] is not None:
                    got += [int(v) for v in batch["image"][:, 0, 0, 0].tolist()]
            assert got == b
    e0 = RankShardedLoader(DS(), 5, 0, world, seed=3).global_batches()
    ld = RankShardedLoader(DS(), 5, 0, world, seed=3)
    ld.set_epoch(1)
    assert ld.global_batches() != e0


def test_transunet_off_config_modules_match_reference():
    """Off-config TransUNet pieces build the reference's module tree on the host: patch size 2
    (img = 2 x 16 x grid) gives the patch conv and position embeddings the reference records in
    tests/golden/transunet_patch2_error.json (its forward then raises there and here, the GPU test);
    SegmentationHead(upsampling > 1) holds conv + UpsamplingBilinear2d with the reference's keys and
    refuses a CPU tensor (no CPU fallback)."""
    import json
    from models.transformer_unet import SegmentationHead, TransUNet
    from test_oracle_golden import transunet_small_config
    rec = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "transunet_patch2_error.json")))
    assert rec["raised"]["type"] == "RuntimeError"
    m = TransUNet(transunet_small_config(), img_size=rec["img"], num_classes=1)
    e = m.transformer.embeddings
    assert list(e.patch_embeddings.kernel_size) == rec["patch_kernel"]
    assert list(e.position_embeddings.shape) == rec["position_embeddings"]
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "seghead_up.npz"))
    for up in (2, 3):
        h = SegmentationHead(16, 2, kernel_size=3, upsampling=up)
        assert isinstance(h[1], torch.nn.UpsamplingBilinear2d) and h[1].scale_factor == up
        assert sorted(h.state_dict()) == ["0.bias", "0.weight"]
        assert tuple(h[0].weight.shape) == fx[f"up{up}_conv_w"].shape
        with pytest.raises(RuntimeError):
            h(torch.zeros(1, 16, 4, 4))
