"""Trainer (drop-in for the reference's utils/trainer.py:19-461).

Same constructor (model, train_loader, val_loader, optimizer, device, config), same methods
(train_epoch -> (loss, iou, dice), validate_epoch -> dict, save_checkpoint, load_checkpoint,
train) and the same step semantics (trainer.py:115-151):

    zero_grad -> forward -> sigmoid -> calculate_metrics -> [NaN loss: skip] -> backward
    -> clip_grad_norm_(max_norm=1.0) -> optimizer.step()

On the MI355X path the step is device-resident (``train_step``): the NaN check skips the SGD
update on the device and the metrics stay on the device; the epoch loop reads them back once
per batch for the running averages, as the reference's ``.item()`` calls do.  With a
``dfcsa.optim.FusedSGD`` optimizer, clipping + SGD is one fused pass; with any other
torch optimizer the reference's clip_grad_norm_ + step() are called.  A plain
``torch.optim.SGD`` (what the reference's train.py builds) is converted to FusedSGD.

Differences kept deliberately small and listed: plots are written only when matplotlib is
importable; best/worst validation samples are kept (tensors on the host, stored in the
checkpoint's ``metrics`` like the reference's) but image dumps (cv2 in the reference) are not
written; ``train(resume_from)`` restores the histories, the
start epoch and the best validation Dice (the reference resets histories and best Dice,
trainer.py:334-349 -- pass ``training.reference_resume_semantics: true`` to keep that behaviour).

Data parallelism (north_star: every configs/*.yaml drops in unchanged on 1..8 GPUs; SURVEY section
8e).  The reference is single-device (train.py:56-59).  When ``torch.distributed`` is initialised
with more than one rank (one process per GPU, e.g. under torchrun), the same Trainer runs the
data-parallel step: each rank takes its rows of every global batch (``dfcsa.ddp.shard_rows``;
a loader from ``DataLoaderFactory`` under the process group already yields only this rank's rows),
the flat gradient buffer is all-reduced in buckets during backward (``GradBucketReducer``; RCCL on
its own stream, captured in the step's HIP graph), a NaN loss on any rank skips the update on every
rank, 1/world is applied inside the fused clip + SGD pass, the per-step metric vector is summed over
the ranks (IoU / Dice of the global batch, the mean of the replica losses), rank 0's BatchNorm
running statistics are broadcast before validation, and only rank 0 writes checkpoints and plots.
Replicas start from rank 0's parameters (broadcast when the reducer is built).  A global batch that
does not divide evenly (the last batch of most epochs) is split as evenly as it can be; each rank's
loss gradient is weighted by n_rank * world / n so the reduced step is the row-weighted mean of the
replica gradients, and a rank left without rows takes part in the collectives with zero gradients.
``training.data_parallel: true`` builds the reducer even in a one-rank group (a rehearsal of the
multi-GPU step on one GPU).  Call ``close()`` before ``dist.destroy_process_group()``: it releases
the captured graphs, which hold RCCL kernels referencing the communicator.
"""
import csv
import os
import time
import weakref

import torch
import torch.distributed as dist

import dfcsa
from dfcsa import streams
from dfcsa.ddp import GradBucketReducer, allreduce_stats, capture_step, shard_rows, shard_weight
from dfcsa.loss import metrics_from_stats, sigmoid
from dfcsa.optim import FusedSGD
from utils.metrics import calculate_metrics_device

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    def tqdm(it, **kw):
        return it

_LIVE = weakref.WeakSet()   # constructed Trainers (close_all)


def close_all():
    """Trainer.close() on every Trainer still alive (e.g. before dist.destroy_process_group() or at the
    end of a test): captured graphs and copy streams are released now, in order, not by a finalizer."""
    for tr in list(_LIVE):
        tr.close()


class Trainer:
    def __init__(self, model, train_loader, val_loader, optimizer, device, config):
        self.config = config
        self.device = device
        self.model = model.to(device)
        # the reference's train.py builds torch.optim.SGD(model.parameters(), ...): run it as the
        # fused device pass (same update; clip_grad_norm_ included)
        self.optimizer = FusedSGD.from_torch_sgd(optimizer) or optimizer
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.loss_type = config["training"].get("loss", {}).get("type", "dice")
        self.loss_params = config["training"].get("loss", {}).get("params", {}) or {}
        print(f"使用損失函數: {self.loss_type}")
        if self.loss_type == "bce_dice":
            print(f"BCE+Dice 損失參數: weight_bce={self.loss_params.get('weight_bce', 1.0)}, "
                  f"weight_dice={self.loss_params.get('weight_dice', 1.0)}")
        self.train_losses, self.val_losses = [], []
        self.train_dice_scores, self.val_dice_scores = [], []
        self.train_iou_scores, self.val_iou_scores = [], []
        self.epochs = []
        self.log_dir = config["logging"]["log_dir"].replace("\\", "/")
        self.images_dir = config["logging"]["images_dir"].replace("\\", "/")
        os.makedirs(self.log_dir, exist_ok=True)
        os.makedirs(self.images_dir, exist_ok=True)
        self.best_model_path = os.path.join(self.log_dir, "best_model.pth").replace("\\", "/")
        self.best_val_loss = float("inf")
        self.checkpoint_dir = os.path.join(self.log_dir, "checkpoints").replace("\\", "/")
        os.makedirs(self.checkpoint_dir, exist_ok=True)
        self.start_time = time.time()
        self.num_epochs = config["training"]["num_epochs"]
        self.max_norm = 1.0
        # data parallelism: one process per GPU under an initialised process group
        self.world, self.rank, self.reducer = 1, 0, None
        if dist.is_available() and dist.is_initialized() and (
                dist.get_world_size() > 1 or config["training"].get("data_parallel", False)):
            self.world, self.rank = dist.get_world_size(), dist.get_rank()
            if not isinstance(self.optimizer, FusedSGD):
                raise NotImplementedError("data-parallel training needs the fused SGD (torch.optim.SGD as built by "
                                          "the reference's train.py, or dfcsa.optim.FusedSGD)")
            self.reducer = GradBucketReducer(self.model, bucket_mb=config["training"].get("bucket_mb", 32.0))
        # HIP-graph replay of the training step (train_step); training.cuda_graph: false disables.
        # Host-staged (gloo) collectives cannot be captured: graphs are off for them.
        use_graphs = config["training"].get("cuda_graph", True)
        if self.reducer is not None and dist.get_backend() == "gloo":
            use_graphs = False
        self._weight = 1.0   # this rank's loss-gradient weight for the current batch (shard_weight)
        self._graphs = {} if use_graphs else None
        self._graph_seen = set()
        self._copy_stream = None   # host batches are uploaded on it, one step ahead (_prefetch)
        _LIVE.add(self)
        print(f"模型將在 {self.device} 上訓練" + (f" (rank {self.rank}/{self.world})" if self.world > 1 else ""))

    # ------------------------------------------------------------------ one step
    def train_step(self, images, masks):
        """One device-resident training step.  Returns {'loss': 0-d tensor, 'stats': fp32[8]}
        (see dfcsa.loss) without synchronising with the host.

        With the fused optimizer on a GPU (``training.cuda_graph``, default on) the step is
        captured once per input shape as a HIP graph (the first batch of a shape runs eagerly,
        the second is captured and replayed, later ones replay): the ~430 kernel launches of a
        step become one graph launch, the kernels and their order are the same, so the results
        are the eager step's.  If capture fails the trainer keeps stepping eagerly."""
        if (self._graphs is not None and isinstance(self.optimizer, FusedSGD) and images.is_cuda
                and self.model.training):
            return self._graph_step(images, masks)
        return self._eager_step(images, masks)

    def close(self):
        """Release the captured step graphs and the upload stream (call before
        dist.destroy_process_group()).  Idempotent; the Trainer can keep training afterwards (it
        captures again)."""
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        if self._graphs:
            for g in self._graphs.values():
                g[0].reset()
            self._drop_graphs()
        self._copy_stream = None
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def _storage(self):
        """The device storage a captured step reads and writes through raw pointers: the model's
        pack plan (tables + packed operands), the flat parameter/gradient buffers and the fused
        optimizer's momentum / norm scratch.  Returns (signature, keep-alive objects), or
        (None, None) when any of it is missing or stale (a plan invalidated by a new PackSet, a
        re-flattened model after ``.to()`` / ``load_state_dict`` into new storage, an optimizer
        re-resolved after ``load_state_dict``, a parameter frozen): the step then runs eagerly,
        which rebuilds what is stale, and later batches capture again."""
        m, opt = self.model, self.optimizer
        params = opt.param_groups[0]["params"]
        flat = getattr(params[0], "_dfcsa_flat", None)
        plan = getattr(m, "_dfcsa_plan", None)
        if flat is None or not flat.valid() or opt._flat is not flat or opt._mom is None:
            return None, None
        if hasattr(m, "_dfcsa_plan") and (plan is None or not plan.valid()):
            return None, None
        if not all(p.requires_grad for p in params):
            return None, None
        keep = (plan, flat, opt._mom, opt._partial, opt.last_norm)
        sig = (id(plan), plan.epoch if plan is not None else -1, id(flat), flat.data.data_ptr(),
               flat.grad.data_ptr(), opt._mom.data_ptr(), opt._partial.data_ptr(),
               opt.last_norm.data_ptr())
        return sig, keep

    def _drop_graphs(self):
        self._graphs.clear()
        self._graph_seen.clear()

    def _graph_step(self, images, masks):
        # the SGD hyper-parameters are kernel arguments baked into a capture: part of the key
        hp = tuple(float(self.optimizer.param_groups[0][k]) for k in ("lr", "momentum", "weight_decay"))
        shapes = (tuple(images.shape), tuple(masks.shape), images.dtype, masks.dtype, hp, self._weight)
        sig, keep = self._storage()
        if sig is None:                           # storage changed or not yet resolved: eager
            self._drop_graphs()
            met = self._eager_step(images, masks)
            sig, _ = self._storage()              # resolved by that step: it counts as the warm-up
            if sig is not None:
                self._graph_seen.add(shapes + (sig,))
            return met
        key = shapes + (sig,)
        g = self._graphs.get(key)
        if g is None:
            if key not in self._graph_seen:       # first batch of this shape: eager (warm-up)
                self._graph_seen.add(key)
                return self._eager_step(images, masks)
            si, sm = images.clone(), masks.clone()
            try:
                # thread_local capture (a DataLoader pin-memory thread and ProcessGroupNCCL's watchdog
                # keep running during the capture), see dfcsa.ddp.capture_step
                graph, met = capture_step(lambda: self._eager_step(si, sm))   # replayed below
            except RuntimeError as e:
                print(f"HIP graph capture of the training step failed ({e}); stepping eagerly")
                self._graphs = None
                self._reset_host_state()
                torch.cuda.synchronize()
                return self._eager_step(images, masks)
            if len(self._graphs) >= 2:           # e.g. a short last batch: keep the newest two
                self._graphs.pop(next(iter(self._graphs)))
            g = self._graphs[key] = (graph, si, sm, met, keep)
        graph, si, sm, met, _ = g
        si.copy_(images, non_blocking=True)
        sm.copy_(masks, non_blocking=True)
        graph.replay()
        return met

    def _reset_host_state(self):
        """After a failed capture: forget host-side state the half-recorded step changed (packed
        operands marked fresh by a plan launch that never ran, an armed bucket reducer)."""
        for mod in self.model.modules():
            ps = getattr(mod, "_dfcsa_pk", None)
            if ps is not None:
                ps.fresh = False
        if self.reducer is not None:
            self.reducer.abort()
        streams.clear_deferred()   # closures of the half-recorded step must not run in a later backward

    def _eager_step(self, images, masks):
        self.optimizer.zero_grad()
        logits = self.model(images)
        probs = sigmoid(logits)
        met = calculate_metrics_device(probs, masks, self.loss_type, self.loss_params)
        loss = met["loss"]
        if self.reducer is not None:
            # data parallel: buckets all-reduced as backward finalises them, NaN agreement over the
            # ranks, 1/world inside the fused clip + SGD, the metric vector summed over the ranks
            self.reducer.start()
            try:
                # a ragged global batch: row-weighted mean over the replicas
                loss.backward(self._root_grad(loss, self._weight))
                skip = self.reducer.finish(loss)
            except BaseException:
                self.reducer.abort()   # no leaked ARMED count / bucket state after a failed pass
                raise
            self.optimizer.step(max_norm=self.max_norm, grad_scale=self.reducer.grad_scale, skip_if_nan=skip)
            return {"loss": loss, "stats": allreduce_stats(met["stats"], weight=self._weight)}
        loss.backward(self._root_grad(loss, 1.0))
        if isinstance(self.optimizer, FusedSGD):
            self.optimizer.step(max_norm=self.max_norm, skip_if_nan=loss)
        else:
            if not torch.isnan(loss):  # host sync; reference behaviour with a foreign optimizer
                torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=self.max_norm)
                self.optimizer.step()
        return met

    def _root_grad(self, loss, w):
        """The loss's root gradient (w), a persistent device scalar per value: no fill kernel per
        step, and a fixed address inside a captured step."""
        cache = self.__dict__.setdefault("_root_grads", {})
        key = (float(w), loss.device, loss.dtype, tuple(loss.shape))
        g = cache.get(key)
        if g is None:
            g = cache[key] = torch.full_like(loss, float(w))
        return g

    def _null_step(self):
        """Data parallel, a rank without rows in this global batch: zero gradients through the same
        collective sequence (every bucket, the NaN flag, the metric vector) and the same SGD step,
        so the replicas stay identical."""
        self.optimizer.zero_grad()
        zero = torch.zeros((), dtype=torch.float32, device=self.device)
        self.reducer.start()
        skip = self.reducer.finish(zero)
        self.optimizer.step(max_norm=self.max_norm, grad_scale=self.reducer.grad_scale, skip_if_nan=skip)
        stats = torch.zeros(8, dtype=torch.float32, device=self.device)
        return {"loss": zero, "stats": allreduce_stats(stats, weight=0.0)}

    def _local_rows(self, batch):
        """(images, masks) of this rank and its loss-gradient weight.  A batch from a rank-sharded
        loader carries 'global_rows' (its rows are already this rank's, possibly none)."""
        images, masks = batch["image"], batch["mask"]
        if self.reducer is None:
            return images, masks, 1.0
        n = batch.get("global_rows")
        if n is None:     # a global batch: take this rank's rows
            n = images.shape[0]
            lo, hi = shard_rows(n, self.rank, self.world)
            images, masks = images[lo:hi], masks[lo:hi]
        return images, masks, shard_weight(n, self.rank, self.world)

    def _prefetch(self, batch):
        """(images, masks, weight, event) of a loader batch on the device, or None at the end.  Host
        (pinned) tensors are uploaded on a copy stream so the upload overlaps the running step; the
        event marks its completion and the tensors are recorded on the compute stream."""
        if batch is None:
            return None
        images, masks, w = self._local_rows(batch)
        if images is None or images.shape[0] == 0:
            return images, masks, w, None
        dev = torch.device(self.device)
        if dev.type != "cuda" or images.is_cuda or not torch.cuda.is_available():
            return images.to(self.device, non_blocking=True), masks.to(self.device, non_blocking=True), w, None
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(device=dev)
        main = torch.cuda.current_stream(dev)
        with torch.cuda.stream(self._copy_stream):
            di = images.to(dev, non_blocking=True)
            dm = masks.to(dev, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._copy_stream)
        di.record_stream(main)
        dm.record_stream(main)
        return di, dm, w, ev

    def train_epoch(self, epoch):
        self.model.train()
        if hasattr(self.train_loader, "set_epoch"):   # a rank-sharded loader reshuffles per epoch
            self.train_loader.set_epoch(epoch)
        running_loss = running_iou = running_dice = 0.0
        bar = tqdm(self.train_loader, desc=f"Epoch {epoch + 1}/{self.num_epochs} [Train]")
        it = iter(bar)
        nxt = self._prefetch(next(it, None))
        batch_idx = -1
        while nxt is not None:
            batch_idx += 1
            images, masks, self._weight, ready = nxt
            if images is None or images.shape[0] == 0:
                met = self._null_step()
            else:
                if ready is not None:   # the copy-stream upload of this batch
                    torch.cuda.current_stream(self.device).wait_event(ready)
                met = self.train_step(images, masks)
            # the next batch is fetched and uploaded while this step runs (the reference's loop
            # uploads it after the .item() below); the results are the same
            nxt = self._prefetch(next(it, None))
            loss = float(met["stats"][0].item())
            if loss != loss:  # NaN: the device already skipped the update (trainer.py:134-139)
                print(f"Warning: NaN loss detected at batch {batch_idx}\n  Skipping this batch...")
                continue
            if loss > 100:
                print(f"Warning: Very large loss detected: {loss:.6f} at batch {batch_idx}")
            iou, dice = metrics_from_stats(met["stats"])
            running_loss += loss
            running_iou += iou
            running_dice += dice
            if hasattr(bar, "set_postfix"):
                bar.set_postfix({"loss": running_loss / (batch_idx + 1), "iou": running_iou / (batch_idx + 1),
                                 "dice": running_dice / (batch_idx + 1)})
        dfcsa.check_wgrad_coop()
        n = len(self.train_loader)
        return running_loss / n, running_iou / n, running_dice / n

    @torch.no_grad()
    def validate_epoch(self, dataloader):
        if self.reducer is not None:
            # every rank evaluates rank 0's model: the BatchNorm running statistics (per replica
            # while training) are broadcast first, as torch DDP's broadcast_buffers does
            self.reducer.broadcast_buffers()
        self.model.eval()
        running_loss = running_iou = running_dice = 0.0
        samples = []
        for batch_idx, batch in enumerate(tqdm(dataloader, desc="Validation")):
            images = batch["image"].to(self.device)
            masks = batch["mask"].to(self.device)
            probs = sigmoid(self.model(images))
            met = calculate_metrics_device(probs, masks, self.loss_type, self.loss_params)
            loss = float(met["stats"][0].item())
            if loss != loss:
                print(f"Warning: NaN loss detected in validation at batch {batch_idx}")
                continue
            iou, dice = metrics_from_stats(met["stats"])
            running_loss += loss
            running_iou += iou
            running_dice += dice
            names = batch.get("filename", [f"{batch_idx}_{i}" for i in range(images.shape[0])])
            for i in range(images.shape[0]):
                m = calculate_metrics_device(probs[i:i + 1], masks[i:i + 1], self.loss_type, self.loss_params)
                si, sd = metrics_from_stats(m["stats"])
                samples.append({"batch_idx": batch_idx, "sample_idx": i, "image": images[i].cpu(),
                                "mask": masks[i].cpu(), "output": probs[i].cpu(), "filename": names[i],
                                "metrics": {"loss": float(m["stats"][0].item()), "iou": si, "dice": sd}})
        n = len(dataloader)
        samples.sort(key=lambda s: s["metrics"]["dice"])
        k = self.config["logging"].get("save_best_worst_samples", 0)
        return {"loss": running_loss / n, "iou": running_iou / n, "dice": running_dice / n,
                "best_samples": samples[-k:] if k else [], "worst_samples": samples[:k]}

    # ------------------------------------------------------------------ checkpoints
    def save_checkpoint(self, epoch, metrics, is_best=False):
        if self.rank != 0:   # data parallel: the replicas are identical, rank 0 writes
            return
        ckpt = {"epoch": epoch, "model_state_dict": self.model.state_dict(),
                "optimizer_state_dict": self.optimizer.state_dict(),
                "train_losses": self.train_losses, "val_losses": self.val_losses,
                "train_dice_scores": self.train_dice_scores, "val_dice_scores": self.val_dice_scores,
                "train_iou_scores": self.train_iou_scores, "val_iou_scores": self.val_iou_scores,
                "best_val_loss": self.best_val_loss,
                "metrics": metrics}   # incl. best/worst samples (host tensors), as trainer.py:276-288
        path = os.path.join(self.checkpoint_dir, f"checkpoint_epoch_{epoch + 1}.pth").replace("\\", "/")
        torch.save(ckpt, path)
        if is_best:
            torch.save(self.model.state_dict(), self.best_model_path)
            torch.save(ckpt, os.path.join(self.checkpoint_dir, "best_checkpoint.pth").replace("\\", "/"))

    def load_checkpoint(self, checkpoint_path):
        ckpt = torch.load(checkpoint_path.replace("\\", "/"), map_location=self.device, weights_only=True)
        self.model.load_state_dict(ckpt["model_state_dict"])
        self.optimizer.load_state_dict(ckpt["optimizer_state_dict"])
        if self._graphs is not None:   # optimizer storage may be new: capture again
            self._drop_graphs()
        for k in ("train_losses", "val_losses", "train_dice_scores", "val_dice_scores", "train_iou_scores",
                  "val_iou_scores", "best_val_loss"):
            setattr(self, k, ckpt[k])
        # the reference does not store the epoch axis of the histories: rebuild it
        self.epochs = list(range(ckpt["epoch"] + 2 - len(self.train_losses), ckpt["epoch"] + 2))
        return ckpt["epoch"]

    # ------------------------------------------------------------------ loop
    def _write_history(self):
        if self.rank != 0:
            return
        with open(os.path.join(self.images_dir, "metrics.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["epoch", "train_loss", "val_loss", "train_dice", "val_dice", "train_iou", "val_iou"])
            for row in zip(self.epochs, self.train_losses, self.val_losses, self.train_dice_scores,
                           self.val_dice_scores, self.train_iou_scores, self.val_iou_scores):
                w.writerow(row)
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except ImportError:
            return
        for name, tr, va in (("loss", self.train_losses, self.val_losses),
                             ("dice", self.train_dice_scores, self.val_dice_scores),
                             ("iou", self.train_iou_scores, self.val_iou_scores)):
            plt.figure(figsize=(8, 5))
            plt.plot(self.epochs, tr, label=f"train {name}")
            plt.plot(self.epochs, va, label=f"val {name}")
            plt.legend()
            plt.savefig(os.path.join(self.images_dir, f"{name}_plot.png"))
            plt.close()

    def train(self, resume_from=None):
        start_epoch = 0
        if resume_from:
            start_epoch = self.load_checkpoint(resume_from) + 1
            print(f"從 epoch {start_epoch} 恢復訓練")
        reference_semantics = self.config["training"].get("reference_resume_semantics", False)
        if not resume_from or reference_semantics:
            self.epochs, self.train_losses, self.val_losses = [], [], []
            self.train_dice_scores, self.val_dice_scores = [], []
            self.train_iou_scores, self.val_iou_scores = [], []
        # the reference restarts the best-Dice tracking at 0 on resume (trainer.py:334-349)
        best_val_dice = 0.0 if reference_semantics else max(self.val_dice_scores, default=0.0)
        for epoch in range(start_epoch, self.num_epochs):
            tr = self.train_epoch(epoch)
            va = self.validate_epoch(self.val_loader)
            self.epochs.append(epoch + 1)
            self.train_losses.append(tr[0])
            self.val_losses.append(va["loss"])
            self.train_dice_scores.append(tr[2])
            self.val_dice_scores.append(va["dice"])
            self.train_iou_scores.append(tr[1])
            self.val_iou_scores.append(va["iou"])
            print(f"Epoch [{epoch + 1}/{self.num_epochs}]")
            print(f"  Train Loss: {tr[0]:.4f}, Dice: {tr[2]:.4f}, IoU: {tr[1]:.4f}")
            print(f"  Val Loss: {va['loss']:.4f}, Dice: {va['dice']:.4f}, IoU: {va['iou']:.4f}")
            is_best = va["dice"] > best_val_dice
            if is_best:
                best_val_dice = va["dice"]
            if (epoch + 1) % self.config["training"]["save_checkpoint_freq"] == 0 or is_best:
                self.save_checkpoint(epoch, va, is_best)
            self._write_history()
        total = time.time() - self.start_time
        print(f"Training completed in {total:.0f}s; best validation dice: {best_val_dice:.4f}")
        return best_val_dice
