"""Benchmark: DFC-SA-Res U-Net training throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], config_dfc-sa-res-block-p4.yaml overlaid): DFC-SA-Res,
features [64, 128, 256, 512], pool_size 4, 3x224x224 -> 1x224x224, bf16 activations with fp32
master weights/statistics, 16 images per GPU.  One step = the full Trainer step
(utils/trainer.py:115-151): forward, sigmoid, BCE+Dice loss + IoU/Dice counts, backward,
[bucketed RCCL all-reduce for N > 1], clip_grad_norm_(1.0) + SGD(0.01, 0.9, 1e-4).
Synthetic data: the GLOBAL batch (16 x N images, N(0,1); masks Bernoulli(0.5)) is generated
from fixed seeds and sharded by rank, resident in HBM before timing.

Launch: `python bench.py` (N=1) or, for N > 1, `python -m torch.distributed.run --nproc-per-node N
... bench.py --gpus N`.  Rank 0 prints ONE JSON line.  The line carries:
  roofline      the dominant kernel class (implicit-GEMM conv or weight-gradient GEMM): its
                algorithmic FLOPs (2*M*N*K per launch, counted by the library in an eager pass) / its
                kernel time per step in the timed HIP-graph replays, from a rocprofv3 kernel trace of
                this benchmark run as a child process before the timed run (live_replay_classes), vs
                the 2.5 PFLOP/s dense bf16 MFMA peak; the HIP-event timing of the eager pass with the
                streams serialised is kept as roofline.serialised_events;
  cpu_baseline  the CPU oracle (oracle/dfcsa_oracle.py, fp32 eager PyTorch = the reference
                algorithm) timed on this host on the same B=16 workload (rank 0, N = 1 only);
  step_roofline whole-step fractions: mfma_frac = model FLOP/s / dense bf16
                peak, hbm_frac = the step's rocprofv3-counted HBM bytes/s / 8 TB/s (profiles/
                rNN_pmc_step.json), roofline_frac = img/s / the per-layer roofline ceiling (6.1 k);
  trainer_faithful  the same model/optimizer driven by utils.trainer.Trainer.train_epoch over host
                batches (H2D copy + the reference's per-step .item() syncs, eager launches), beside
                the device-resident HIP-graph rate that is `value`.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md, chip-level parameters)
MFMA_F32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0
FWD_BWD_GFLOP_PER_IMG = 201.66   # SURVEY.md section 8d (torch.utils.flop_counter, P=4, 224^2)
ALG_GB_PER_IMG = 1.07            # minimum bf16 bytes per image
ROOFLINE_CEILING_IMG_S = 6100.0  # per-layer max(F/P, B/BW) ceiling per GPU

# --model: the BASELINE configs.  Only 'dfc' is the headline line the driver records;
# the others put the secondary configs' training step on the same clock.  GFLOP/img fwd+bwd
# from SURVEY.md section 6 (torch.utils.flop_counter) where the survey measured it at that size.
MODELS = {
    "dfc": dict(name="DFC-SA-Res-Block", label="DFC-SA-Res", gflop={224: FWD_BWD_GFLOP_PER_IMG}),
    "unet": dict(name="UNet", label="UNet (config 1)", gflop={64: 18.05}),
    "transunet": dict(name="TransformerUNet", label="TransUNet R50-ViT-B/16 (config 4)", gflop={224: 174.94}),
    "fullres": dict(name="UNet_FullResAttention", label="UNet_FullResAttention (config 5)", gflop={}),
    # the ablation zoo (configs/config_ablation{1,2,4}_*.yaml): reported, not the headline
    **{k: dict(name=n, label=n, gflop={}) for k, n in (
        ("baseline", "UNet_Baseline"), ("attn_only", "UNet_AttentionOnly"), ("addition", "UNet_AdditionFusion"),
        ("concat", "UNet_ConcatFusion"), ("encoder_only", "UNet_EncoderOnlyDFC"),
        ("decoder_only", "UNet_DecoderOnlyDFC"), ("both_standard", "UNet_BothStandardConv"))},
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(cls):
    """HBM bytes per launch of a kernel class from the committed rocprofv3 PMC passes
    (profiles/rNN_pmc_traffic.json, written by tools/rocpd_export.py from separate FETCH_SIZE and
    WRITE_SIZE passes over this benchmark, gfx950 correction: reads = 2 x FETCH_SIZE)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))[cls]
        return round(d["hbm_bytes_per_launch"]), os.path.relpath(files[-1], ROOT)
    except (KeyError, ValueError, OSError):
        return None, None


def live_replay_classes(args, timeout_s=420):
    """Kernel time per step of each roofline class in the timed HIP-graph replays of THIS build on
    THIS box: this benchmark's own timed loop (same workload, streams concurrent) run under
    `rocprofv3 --kernel-trace` as a child process, started before this process touches the GPU
    (no exec from a GPU-initialised process), classified by tools/rocpd_export.py.  Returns
    (classes, info) or (None, reason)."""
    import glob
    import shutil
    import sqlite3
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import rocpd_export as R
    finally:
        sys.path.pop(0)
    if any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ):
        return None, "this command already runs under a profiler"
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    steps = max(args.steps, 6)
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        cmd = [prof, "--kernel-trace", "-d", tmp, "-o", "run", "--", sys.executable, os.path.join(ROOT, "bench.py"),
               "--steps", str(steps), "--warmup", str(args.warmup), "--batch", str(args.batch), "--img", str(args.img),
               "--pool", str(args.pool), "--precision", args.precision, "--no-cpu-baseline", "--no-val-dice",
               "--no-trainer-faithful", "--no-kernel-timing", "--no-live-trace"]
        env = dict(os.environ, TMPDIR="/tmp")
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=timeout_s)
        except (OSError, subprocess.SubprocessError) as e:
            return None, f"rocprofv3 child failed: {e}"
        if r.returncode != 0:
            return None, f"rocprofv3 child rc={r.returncode}: {r.stderr[-400:]}"
        dbs = sorted(glob.glob(os.path.join(tmp, "**", "*.db"), recursive=True))
        if not dbs:
            return None, "rocprofv3 wrote no trace database"
        out = os.path.join(tmp, "replay.json")
        try:
            R.replay(dbs[-1], out, steps=min(5, steps - 1))
            res = json.load(open(out))
        except (SystemExit, sqlite3.Error, OSError, ValueError, KeyError) as e:
            return None, f"trace parse failed: {e}"
        try:
            child = json.loads(r.stdout.strip().splitlines()[-1])
            child_ms = child.get("ms_per_step")
        except (ValueError, IndexError):
            child_ms = None
    info = {"steps": res["steps"], "launches_per_step": res["launches_per_step"],
            "first_to_last_kernel_ms_per_step": round(res["first_to_last_kernel_ms_per_step"], 3),
            "child_ms_per_step_under_profiler": child_ms, "seconds": round(time.perf_counter() - t0, 1),
            "groups": {k: {kk: round(vv, 4) for kk, vv in v.items()} for k, v in res["groups"].items()}}
    return res["classes"], info


def cpu_model_name():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return None


def cpu_baseline(batch=16, timed_steps=2):
    """Time the CPU oracle's full train step (fp32 eager PyTorch, the reference algorithm) on the
    headline workload: B=16 images of 3x224x224, P=4, features 64..512, 1 warm-up + `timed_steps`
    steps.  Threads: this process's CPU affinity, capped by OMP_NUM_THREADS when the launcher sets
    it (the GPU box gives one GPU's job a 16-core share of a larger machine)."""
    from oracle import dfcsa_oracle as O
    aff = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(aff, omp) if omp > 0 else aff)
    torch.set_num_threads(threads)
    from models.unet_dfc_sa_res import UNetDFCSARes
    torch.manual_seed(0)
    ref = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4)
    sd = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(batch, 3, 224, 224, generator=g)
    t = (torch.rand(batch, 1, 224, 224, generator=g) > 0.5).float()
    sd, bufs, _ = O.train_step(sd, {}, x, t, 4)   # warm-up step
    t0 = time.perf_counter()
    for _ in range(timed_steps):
        sd, bufs, _ = O.train_step(sd, bufs, x, t, 4)
    el = time.perf_counter() - t0
    return {"value": round(timed_steps * batch / el, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model_name(), "affinity_cpus": aff,
            "core_share": (f"{threads}-core share (OMP_NUM_THREADS={omp} of {aff} affinity CPUs: the box's CPU "
                           f"share for one GPU's job)" if omp > 0 and omp < aff else f"all {aff} affinity CPUs"),
            "sample": f"{timed_steps} timed train steps (after 1 warm-up) of B={batch} 3x224x224 images, P=4, "
                      f"features 64..512: oracle/dfcsa_oracle.py fp32 eager PyTorch on {threads} host threads"}


def trainer_faithful_leg(model, opt, x, t, steps):
    """The reference's step loop as a user runs it: utils.trainer.Trainer.train_epoch over host
    (pinned) batches -- H2D copy per batch, the device step, and the reference's per-step host
    syncs (loss .item(), IoU/Dice as Python floats, trainer.py:142,154-156); the Trainer replays
    the step as a HIP graph (captured during the two warm-up batches)."""
    import contextlib
    import io

    from utils.trainer import Trainer
    os.environ.setdefault("TQDM_DISABLE", "1")   # the epoch progress bar would flood stderr
    xb, tb = x.cpu().pin_memory(), t.cpu().pin_memory()
    loader = [{"image": xb, "mask": tb} for _ in range(steps)]
    with contextlib.redirect_stdout(io.StringIO()), tempfile.TemporaryDirectory() as tmp:
        cfg = {"training": {"num_epochs": 1, "loss": {"type": "bce_dice", "params": {}}},
               "logging": {"log_dir": os.path.join(tmp, "l"), "images_dir": os.path.join(tmp, "i")}}
        tr = Trainer(model, loader[:2], loader[:1], opt, x.device, cfg)
        tr.train_epoch(0)                      # warm-up: one eager step, then the graph capture
        torch.cuda.synchronize()
        tr.train_loader = loader
        t0 = time.perf_counter()
        tr.train_epoch(0)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    return {"value": round(steps * x.shape[0] / el, 2), "unit": "images/s", "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 3),
            "how": "utils.trainer.Trainer.train_epoch over pinned host batches: H2D copy + per-step "
                   ".item() syncs as the reference (trainer.py:115-163), the step replayed as a HIP graph "
                   "(Trainer default, training.cuda_graph)"}


def step_pmc_bytes():
    """HBM bytes per step from the newest committed whole-step PMC pass (profiles/rNN_pmc_step.json,
    FETCH_SIZE and WRITE_SIZE summed over every kernel of a step, gfx950 read correction)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_step.json")))
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
        return float(d["hbm_bytes_per_step"]), os.path.relpath(files[-1], ROOT)
    except (KeyError, ValueError, OSError):
        return None, None


def val_dice_leg(cfg, dev, steps=600, batch=16, img=224, n_train=512, n_val=64):
    """BASELINE.json metric's "val Dice": train the same model/config from the same seed on the
    learnable synthetic task (utils.data_loader.SyntheticEllipses, seed 42 train / 43 val) for
    `steps` Trainer steps, then validation Dice exactly as Trainer.validate_epoch reports it (eval-mode
    BatchNorm, mean over batches of the batch-micro Dice, reference trainer.py:219,249)."""
    from dfcsa.loss import metrics_from_stats, sigmoid
    from dfcsa.optim import FusedSGD
    from models.model_factory import ModelFactory
    from utils.data_loader import SyntheticEllipses
    from utils.metrics import calculate_metrics_device

    def stack(ds, n):
        items = [ds[i] for i in range(n)]
        return (torch.stack([it["image"] for it in items]).to(dev), torch.stack([it["mask"] for it in items]).to(dev))

    t0 = time.perf_counter()
    xtr, ttr = stack(SyntheticEllipses(n_train, (img, img), seed=42), n_train)
    xva, tva = stack(SyntheticEllipses(n_val, (img, img), seed=43), n_val)
    torch.manual_seed(0)
    model = ModelFactory.get_model(cfg).to(dev).train()
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4, zero_after_step=True)
    g = torch.Generator().manual_seed(7)
    for s in range(steps):
        idx = torch.randint(0, n_train, (batch,), generator=g).to(dev)
        opt.zero_grad()
        met = calculate_metrics_device(sigmoid(model(xtr[idx])), ttr[idx], "bce_dice", {})
        met["loss"].backward()
        opt.step(max_norm=1.0, skip_if_nan=met["loss"])
    train_loss = float(met["stats"][0].item())
    model.eval()
    dices = []
    with torch.no_grad():
        for i in range(0, n_val, batch):
            st = calculate_metrics_device(sigmoid(model(xva[i:i + batch])), tva[i:i + batch], "bce_dice", {})["stats"]
            dices.append(metrics_from_stats(st)[1])
    return {"value": round(sum(dices) / len(dices), 4), "train_steps": steps, "batch": batch,
            "final_train_loss": round(train_loss, 4), "train_images": n_train, "val_images": n_val,
            "task": "SyntheticEllipses 1-4 ellipses/image, seed 42 train / 43 val (utils/data_loader.py)",
            "seconds": round(time.perf_counter() - t0, 1)}


# v_exp_f32 issue: 8 cycles per 64-lane wave-instruction on one SIMD (MI355X_MICROARCH.md, constants table
# row 'vector-instruction ISSUE cost') -> 8 exp / clk / SIMD x 4 SIMDs x 256 CUs x 2.4 GHz
EXP_PEAK_PER_S = 256 * 4 * 64 / 8 * 2.4e9


def fra_exp_roofline(roof, fra_cls, args, B, L):
    """Config 5's full-resolution attention is transcendental-bound (d_qk = C/8 = 8 at level 1: one
    v_exp_f32 per score element against 144 MFMA flops), so its roofline is in exp/s, not MFMA flop/s.
    Executed exps per step: forward N^2 per attention; backward recomputes P from the saved row
    log-sum-exp twice (dK/dV pass and dQ pass), and the C > 256 levels once per 128-wide value chunk
    and pass (dfcsa_fra_bwd_wide).  Attention blocks: 4 encoder + 4 decoder at img / 2^l, l = 0..3,
    and the bottleneck at img / 16 (models/unet_dfc_sa_ablation_attention.py)."""
    feats = [64, 128, 256, 512]
    blocks = [(args.img >> l, feats[l], 2) for l in range(4)] + [(args.img >> 4, 1024, 1)]
    fwd = bwd = 0.0
    for hw, C, nb in blocks:
        n2 = float(hw * hw) ** 2
        path = L.LIB.dfcsa_fra_path(1 if args.precision == "bf16" else 0, C, C // 8, 2 * (C // 8) + C, 1)
        fwd += nb * n2
        bwd += nb * n2 * (2 * (C // 128) if path == 2 else 2)
    name, ms, n, _, _, _ = fra_cls
    sec = ms * 1e-3 / args.steps
    executed = B * (fwd + bwd)
    ach = executed / sec
    return {"bound": "exp", "kernel": name, "achieved": round(ach / 1e12, 3), "peak": round(EXP_PEAK_PER_S / 1e12, 3),
            "unit": "Texp/s", "frac": round(ach / EXP_PEAK_PER_S, 4),
            "executed_exps_per_step": executed, "forward_exps_per_img": fwd,
            "algorithmic_frac": round(B * fwd / sec / EXP_PEAK_PER_S, 4),
            "note": "peak = v_exp_f32 issue rate (8 clk per wave-instruction per SIMD, 2.4 GHz, 256 CUs); achieved = "
                    "every exp the kernels execute (forward N^2 + two backward recomputations of P) / the fra class's "
                    "time; algorithmic_frac counts the forward N^2 only (the reference stores P instead of recomputing, "
                    "which at 512^2 is 274.9 GB per image)",
            "mfma_view": {k: roof[k] for k in ("achieved", "peak", "unit", "frac")},
            "timing": roof["timing"], "launches_per_step": roof["launches_per_step"],
            "avg_launch_ms": roof["avg_launch_ms"], "ms_per_step": roof["ms_per_step"],
            "share_of_step": roof["share_of_step"], "traffic": None, "other_class": {}}


def main():
    # stdout carries exactly ONE JSON line (rank 0).  RCCL prints its version banner to stdout when a
    # communicator comes up, and other libraries may print too: keep a private handle on the real
    # stdout for the JSON line and point fd 1 at stderr for everything else.
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--img", type=int, default=224)
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one HIP graph per step")
    ap.add_argument("--no-val-dice", action="store_true", help="skip the synthetic-task validation Dice leg")
    ap.add_argument("--model", default="dfc", choices=sorted(MODELS),
                    help="dfc = the BASELINE headline (config 2/3); unet / transunet / fullres = configs 1 / 4 / 5")
    ap.add_argument("--val-steps", type=int, default=600)
    ap.add_argument("--no-trainer-faithful", action="store_true", help="skip the Trainer.train_epoch rate")
    ap.add_argument("--sync-bn", action="store_true",
                    help="opt-in SyncBatchNorm over the ranks (default: per-replica BN, standard DDP)")
    ap.add_argument("--ddp-rehearsal", action="store_true",
                    help="one GPU: run the N > 1 code path (RCCL group of world size 1, bucket reducer, "
                         "graph-captured collectives, teardown) -- the multi-GPU path's test on a one-GPU box")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--no-live-trace", action="store_true",
                    help="skip the rocprofv3 kernel trace of the timed replay (roofline.frac then falls back to "
                         "the serialised HIP-event timing)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    live = (None, None)
    if (world == 1 and args.model == "dfc" and not args.no_kernel_timing and not args.no_live_trace
            and not args.ddp_rehearsal and not args.no_graph):
        # before this process initialises the GPU: the child owns the device while it runs
        log("[rank 0] kernel trace of the timed replay (rocprofv3 child) ...")
        live = live_replay_classes(args)
        log(f"[rank 0] live replay trace: {live[1] if live[0] is None else 'ok'}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ddp = world > 1 or args.ddp_rehearsal
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    elif ddp:   # world size 1: an in-process store, no rendezvous
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)

    import dfcsa._lib as L
    from dfcsa.ddp import GradBucketReducer, capture_step, shard_rows, shutdown
    from dfcsa.loss import bce_dice, sigmoid
    from dfcsa.optim import FusedSGD
    from models.model_factory import ModelFactory

    spec = MODELS[args.model]
    cfg = {"model": {"name": spec["name"], "in_channels": 3, "out_channels": 1,
                     "features": [64, 128, 256, 512], "pool_size": args.pool, "ablation_on_qk_channels": 8,
                     "precision": args.precision},
           "dataset": {"img_size": [args.img, args.img]},
           "training": {"learning_rate": 0.01, "momentum": 0.9, "weight_decay": 1e-4}}
    headline = args.model == "dfc"
    torch.manual_seed(0)
    model = ModelFactory.get_model(cfg).to(dev).train()   # its messages go to stderr (fd 1 redirected)
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4, zero_after_step=True)

    B, S = args.batch, args.img
    gb = B * world
    g = torch.Generator().manual_seed(1234)
    xg = torch.randn(gb, 3, S, S, generator=g)
    g2 = torch.Generator().manual_seed(1235)
    tg = (torch.rand(gb, 1, S, S, generator=g2) > 0.5).float()
    lo, hi = shard_rows(gb, rank, world)
    x = xg[lo:hi].to(dev)
    t = tg[lo:hi].to(dev)
    del xg, tg

    if ddp and args.sync_bn:
        from dfcsa import ops as dfops
        dfops.set_sync_bn()
    model(x)  # materialise the flat parameter/gradient storage and packed operands first
    reducer = GradBucketReducer(model, bucket_mb=args.bucket_mb) if ddp else None
    scale = reducer.grad_scale if reducer else 1.0

    one = torch.ones((), device=dev)   # the root gradient, a persistent tensor (no fill per step)

    def step():
        opt.zero_grad()
        p = sigmoid(model(x))
        loss, stats = bce_dice(p, t, 1.0, 1.0)   # 'bce_dice' with the yaml's (ignored) weight keys
        if reducer:
            reducer.start()
        loss.backward(one)
        skip = reducer.finish(loss) if reducer else loss   # NaN on any rank -> every rank skips
        opt.step(max_norm=1.0, grad_scale=scale, skip_if_nan=skip)
        return stats

    def barrier():
        if ddp:
            dist.barrier()

    for _ in range(args.warmup):
        stats = step()
    torch.cuda.synchronize()
    log(f"[rank {rank}] warm-up done; loss {stats[0].item():.4f}")

    # One HIP graph per training step: the whole step (forward, loss, backward, [RCCL buckets],
    # clip + SGD) is captured once and replayed, so the ~500 kernel launches of a step cost one
    # graph launch.  Inputs are static (resident) tensors; nothing in the step syncs the host.
    graph = None
    if not args.no_graph:
        side = torch.cuda.Stream(priority=int(os.environ.get("DFCSA_PRIO_MAIN", "0")))
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        try:
            # thread_local capture with the NCCL watchdog drained first (dfcsa.ddp.capture_step)
            graph, gstats = capture_step(step)
        except RuntimeError as e:  # e.g. a collective the runtime cannot capture: time eager steps
            log(f"[rank {rank}] HIP graph capture failed ({e}); timing eager steps")
            graph = None
            torch.cuda.synchronize()

    def run_step():
        if graph is None:
            return step()
        graph.replay()
        return gstats

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        stats = run_step()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    if ddp:
        te = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        el = te.item()
    final_loss = stats[0].item()
    import dfcsa
    dfcsa.check_wgrad_coop()   # knob 31 (opt-in) must not have produced a partially reduced tile

    # Dominant-kernel timing: the same K steps again, launched eagerly with the per-class HIP
    # event hook on (a graph replay cannot bracket individual kernels).
    roof = None
    if not args.no_kernel_timing:
        import ctypes
        # kernel classes (bound, unit of the "flops" slot): the tile GEMMs are MFMA-bound; the 1x1
        # streaming GEMMs are HBM-bound and report algorithmic bytes
        classes = ((1, "conv_gemm (implicit-GEMM conv fwd/dgrad, LDS-DMA tiles)", "conv_gemm", "mfma"),
                   (2, "conv_wgrad (weight-gradient GEMM)", "conv_wgrad", "mfma"),
                   (3, "fra (full-resolution attention fwd/bwd, bf16 MFMA)", "fra", "mfma"),
                   (4, "conv1x1_stream (1x1 conv GEMMs with K <= 256 and the fused block GEMMs -- gate backward "
                       "in the dgrad epilogue, gate fusion / local-attention merge in the forward prologue; HBM-streaming)",
                    "conv1x1_stream", "hbm"))
        # the side / branch streams are serialised for this pass: a class's launch durations are then
        # its kernels' own (concurrent with the other streams' work, a launch's event-to-event time
        # also counts the CUs it shares)
        from dfcsa import streams as _streams
        saved = (_streams.ENABLED[0], _streams.BRANCH_ENABLED[0])
        _streams.ENABLED[0] = _streams.BRANCH_ENABLED[0] = False
        for c, _, _, _ in classes:
            L.LIB.dfcsa_prof_enable(c, 1)
        try:
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
        finally:
            _streams.ENABLED[0], _streams.BRANCH_ENABLED[0] = saved
        cls = {}
        for c, name, key, bound in classes:
            ms, n, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
            L.LIB.dfcsa_prof_read(c, ctypes.addressof(ms), ctypes.addressof(n), ctypes.addressof(fl))
            if n.value:
                cls[c] = (name, ms.value, n.value, fl.value, key, bound)
            L.LIB.dfcsa_prof_enable(c, 0)

        def rate(v):
            """(achieved, peak, unit) of a class: TFLOP/s against the dense MFMA peak, or GB/s
            against HBM."""
            _, ms_, _, units, _, bound_ = v
            if bound_ == "hbm":
                return (units / (ms_ * 1e-3) / 1e9 if ms_ > 0 else 0.0), HBM_PEAK_GBS, "GB/s"
            pk = MFMA_BF16_PEAK_TFLOPS if args.precision == "bf16" else MFMA_F32_PEAK_TFLOPS
            return (units / (ms_ * 1e-3) / 1e12 if ms_ > 0 else 0.0), pk, "TFLOP/s"

        dom = max(cls.values(), key=lambda v: v[1])
        name, ms, n, fl, dom_key, bound = dom
        ach, peak, unit = rate(dom)
        traffic, tsrc = pmc_traffic(dom_key) if headline else (None, None)   # PMC passes cover the headline
        roof = {"bound": bound, "kernel": name, "achieved": round(ach, 2), "peak": peak, "unit": unit,
                "timing": "HIP events around each launch of the class, the same K steps launched eagerly "
                          "with the side and branch streams serialised",
                "frac": round(ach / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": tsrc,
                "launches_per_step": n // args.steps, "avg_launch_ms": round(ms / max(n, 1), 4),
                "ms_per_step": round(ms / args.steps, 3), "share_of_step": round(ms / (el * 1e3), 3),
                "other_class": {}}
        rep, rinfo = live
        if rep and dom_key in rep and rep[dom_key]["ms_per_step"] > 0:
            # the headline figure: the class's FLOPs per step over its kernel time in the timed HIP-graph
            # replays of this build on this box (streams concurrent, so a launch also counts the CUs
            # it shares) -- where the step runs.  The serialised HIP-event timing stays as secondary.
            r = rep[dom_key]
            a_rep = fl / args.steps / (r["ms_per_step"] * 1e-3) / (1e12 if unit == "TFLOP/s" else 1e9)
            roof["serialised_events"] = {"achieved": roof["achieved"], "frac": roof["frac"],
                                         "avg_launch_ms": roof["avg_launch_ms"], "ms_per_step": roof["ms_per_step"],
                                         "timing": roof["timing"]}
            roof.update({"achieved": round(a_rep, 2), "frac": round(a_rep / peak, 4),
                         "ms_per_step": round(r["ms_per_step"], 3),
                         "launches_per_step": r["launches_per_step"],
                         "avg_launch_ms": round(r["ms_per_step"] / max(r["launches_per_step"], 1), 4),
                         "share_of_step": round(r["ms_per_step"] / (el * 1e3 / args.steps), 3),
                         "timing": "rocprofv3 --kernel-trace of this benchmark's timed HIP-graph replays, run as a "
                                   "child process of this command on this box (side and branch streams concurrent); "
                                   "FLOPs per step from this run's per-launch 2*M*N*K counts"})
            roof["replay_trace"] = rinfo
        elif headline:
            roof["replay_trace"] = {"error": rinfo}
        if args.model == "fullres" and 3 in cls:
            roof = fra_exp_roofline(roof, cls[3], args, B, L)
        for v in cls.values():
            if v is dom:
                continue
            a_, p_, u_ = rate(v)
            tr_, _ = pmc_traffic(v[4]) if headline else (None, None)
            roof["other_class"][v[0]] = {"bound": v[5], "ms_per_step": round(v[1] / args.steps, 3),
                                         "achieved": round(a_, 2), "unit": u_, "frac": round(a_ / p_, 4),
                                         "avg_launch_ms": round(v[1] / max(v[2], 1), 4), "traffic": tr_}

    faithful = None
    if world == 1 and not args.no_trainer_faithful and headline:
        log(f"[rank {rank}] Trainer-faithful leg (Trainer.train_epoch, host batches, .item() syncs) ...")
        faithful = trainer_faithful_leg(model, opt, x, t, args.steps)

    vdice = None
    if rank == 0 and world == 1 and not args.no_val_dice and headline:
        log("[rank 0] validation Dice leg (synthetic ellipses) ...")
        vdice = val_dice_leg(cfg, dev, steps=args.val_steps, batch=B, img=S)

    imgs = args.steps * B * world
    value = imgs / el
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline:
        log("[rank 0] timing the CPU oracle baseline ...")
        cpu = cpu_baseline()
    if rank == 0:
        gflop = spec["gflop"].get(S)
        step_roof = None
        if headline and gflop:
            per_gpu = value / world
            pmc, psrc = step_pmc_bytes()
            step_roof = {"mfma_frac": round(per_gpu * gflop * 1e9 / (MFMA_BF16_PEAK_TFLOPS * 1e12), 4),
                         "hbm_frac": round(per_gpu * pmc / B / (HBM_PEAK_GBS * 1e9), 4) if pmc else None,
                         "hbm_frac_algorithmic": round(per_gpu * ALG_GB_PER_IMG / HBM_PEAK_GBS, 4),
                         "roofline_frac": round(per_gpu / ROOFLINE_CEILING_IMG_S, 4),
                         "ceiling_img_s_per_gpu": ROOFLINE_CEILING_IMG_S,
                         "hbm_bytes_per_step": pmc, "hbm_source": psrc}
        out = {"metric": f"training images/sec (fwd+bwd) 3x{S}x{S} {spec['label']}", "value": round(value, 2),
               "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
               "launch": "eager" if graph is None else "hip_graph",
               "config": {"workload": (f"DFC-SA-Res P={args.pool} features 64..512 {S}x{S} train step" if headline
                                       else f"{spec['label']} {S}x{S} train step"),
                          "per_gpu_batch": B, "global_batch": B * world, "img": S, "pool_size": args.pool,
                          "parallelism": f"dp{world}", "sync_bn": bool(ddp and args.sync_bn), "final_loss": round(final_loss, 5),
                          "ddp_path": ddp,
                          "model_tflops": round(value * gflop / 1e3, 2) if gflop else None},
               "roofline": roof, "step_roofline": step_roof, "trainer_faithful": faithful,
               "cpu_baseline": cpu, "val_dice": vdice}
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    # release the step graph (its RCCL kernels reference the communicator) before the process
    # group is destroyed; then every rank exits 0
    shutdown(graph)


if __name__ == "__main__":
    main()
