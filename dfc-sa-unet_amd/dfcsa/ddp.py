"""Data parallelism for the DFC-SA-Res step: one process per GPU, gradients all-reduced over
torch.distributed ('nccl' backend = RCCL on ROCm, xGMI between the MI355X GPUs of a node).

The reference has no parallelism (single device, train.py:56-59); this is the build's own
design:
  * the minibatch is sharded over ranks; BatchNorm statistics and the batch Dice loss stay
    per-replica (standard DDP semantics -- the multi-GPU step equals the mean of per-shard
    reference gradients, which is what tests/golden/ddp_shards.npz pins);
  * all gradients live in one flat fp32 buffer (dfcsa.flat), cut into contiguous buckets from
    its END, because backward produces gradients from the last layer to the first;
  * every module backward (DFC block, transposed conv, head) reports when its parameters'
    gradients are final; a bucket whose modules are all final is all-reduced immediately with
    async_op=True, so RCCL runs on its own stream underneath the remaining backward kernels;
  * ``finish(loss)`` makes the compute stream wait for every bucket (no host synchronisation);
    the optimizer then applies 1/world_size inside the fused clip+SGD pass.  With ``loss`` it
    also all-reduces (MAX) a NaN indicator of every rank's loss and returns the device scalar the
    optimizer's NaN skip reads, so a NaN loss on ANY rank skips the update on EVERY rank (the
    reference's NaN ``continue``, utils/trainer.py:134-139, made consistent across replicas; a
    rank-local decision would let the other ranks apply the NaN gradients they received);
  * BatchNorm running statistics are per replica between syncs (each rank normalises its own
    shard, as torch DDP does).  ``broadcast_buffers()`` copies rank 0's running statistics to
    every rank (torch DDP's broadcast_buffers); call it before validation or checkpointing so all
    ranks evaluate and save the same model.
"""
import time

import torch
import torch.distributed as dist

from . import streams

# armed bucket reducers (between start() and finish()): a bucket is all-reduced as soon as its
# modules' backward has issued their gradient launches, so no gradient launch may be deferred then
ARMED = [0]

# ProcessGroupNCCL's watchdog thread polls the completion events of the eager collectives it
# tracks about every 100 ms and drops completed ones.  A HIP-graph capture must not begin while it
# still holds any (see capture_step): waiting this long after a device synchronisation lets it
# drain its list first.
WATCHDOG_DRAIN_S = 0.3


class GradBucketReducer:
    def __init__(self, model, bucket_mb=32.0, group=None):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        self.flat = model.flat_params()
        # [(module, lo, hi)] in flat-buffer order; a model without per-module units is one unit
        # (its single bucket is reduced by finish())
        units = model.grad_units() if hasattr(model, "grad_units") else [(model, 0, self.flat.numel)]
        self.unit_of = {}
        self.buckets = []           # [(lo, hi, n_units)]
        cap = int(bucket_mb * (1 << 20) / 4)
        cur, lo, hi = [], None, None
        for mod, a, b in reversed(units):
            if cur and (hi - a) > cap:
                self.buckets.append([lo, hi, cur])
                cur = []
            if not cur:
                hi = b
            lo = a
            cur.append(mod)
        if cur:
            self.buckets.append([lo, hi, cur])
        for i, (_, _, mods) in enumerate(self.buckets):
            for m in mods:
                self.unit_of[id(m)] = i
                m._dfcsa_reducer = self
        self._pending = None
        self._works = []
        self.broadcast_parameters()

    @torch.no_grad()
    def broadcast_parameters(self, src=0):
        """Make every replica start from rank ``src``'s parameters and BatchNorm buffers (torch
        DDP does this at construction): one broadcast of the flat parameter buffer, one of the
        floating-point buffers.  Replica consistency then does not rest on every process having
        drawn the same initialisation from its RNG."""
        if self.world <= 1 or not dist.is_initialized():
            return
        data = self.flat.data
        if data.is_cuda and dist.get_backend(self.group) == "gloo":
            h = data.cpu()
            dist.broadcast(h, src=src, group=self.group)
            data.copy_(h)
        else:
            dist.broadcast(data, src=src, group=self.group)
        self.broadcast_buffers(src)

    def start(self):
        """Arm for one backward pass (re-arming an armed reducer first disarms it: the ARMED count
        stays one per armed reducer whatever happened to the previous pass)."""
        self._disarm()
        ARMED[0] += 1
        self._pending = [len(b[2]) for b in self.buckets]
        self._works = []
        self._launched = [False] * len(self.buckets)

    def unit_ready(self, module):
        if self._pending is None:
            return
        i = self.unit_of.get(id(module))
        if i is None:
            return
        self._pending[i] -= 1
        # launch in bucket order only (every rank issues the same collective sequence)
        j = len(self._works)
        while j < len(self.buckets) and self._pending[j] == 0:
            lo, hi, _ = self.buckets[j]
            self._works.append(self._launch(lo, hi))
            j += 1

    def _launch(self, lo, hi):
        """all_reduce a bucket once both the compute stream (BN / attention grads) and the side
        stream (weight-gradient GEMMs, dfcsa.streams) have produced it."""
        main = torch.cuda.current_stream() if self.flat.grad.is_cuda else None
        if main is None:
            return dist.all_reduce(self.flat.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if dist.get_backend(self.group) == "gloo":
            # CPU-transport rehearsal (several ranks on one GPU): host-staged and synchronous
            streams.join()
            return _host_allreduce(self.flat.grad[lo:hi], dist.ReduceOp.SUM, self.group)
        side = streams.side_stream(self.flat.grad.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            return dist.all_reduce(self.flat.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _disarm(self):
        """Idempotent: drop this reducer's ARMED count iff it is armed."""
        if self._pending is not None:
            ARMED[0] -= 1
            self._pending = None

    def abort(self):
        """Forget an armed backward without reducing (an exception between start() and finish(), a
        failed graph capture): the ARMED count returns, so deferred weight gradients are allowed
        again, and no stale bucket state leaks into the next pass."""
        self._disarm()
        self._works = []

    def finish(self, loss=None):
        """Ensure every bucket has been reduced (launch stragglers), make the current stream wait.
        With ``loss``: returns a device scalar that is NaN iff some rank's loss is NaN (else 0),
        for ``FusedSGD.step(skip_if_nan=...)``."""
        if self._pending is not None:
            for j in range(len(self._works), len(self.buckets)):
                lo, hi, _ = self.buckets[j]
                self._works.append(self._launch(lo, hi))
        flag = None
        if loss is not None:
            # the NaN agreement runs whether or not the reducer was armed: a caller handing the
            # result to FusedSGD.step(skip_if_nan=...) must never get None for a NaN loss
            flag = torch.isnan(loss.detach().reshape(1)).float()
            if flag.is_cuda and dist.get_backend(self.group) == "gloo":
                self._works.append(_host_allreduce(flag, dist.ReduceOp.MAX, self.group))
            else:
                self._works.append(dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group, async_op=True))
        try:
            if self.flat.grad.is_cuda:
                streams.join()
            for w in self._works:
                w.wait()
        finally:
            self._disarm()
        if flag is None:
            return None
        return torch.where(flag > 0, torch.full_like(flag, float("nan")), torch.zeros_like(flag))

    @torch.no_grad()
    def broadcast_buffers(self, src=0):
        """Copy rank ``src``'s floating-point buffers (BatchNorm running_mean / running_var) to every
        rank in one collective."""
        bufs = [b for b in self.model.buffers() if b.is_floating_point()]
        if not bufs:
            return
        flat = torch.cat([b.reshape(-1) for b in bufs])
        if flat.is_cuda and dist.get_backend(self.group) == "gloo":
            h = flat.cpu()
            dist.broadcast(h, src=src, group=self.group)
            flat.copy_(h)
        else:
            dist.broadcast(flat, src=src, group=self.group)
        o = 0
        for b in bufs:
            b.copy_(flat[o:o + b.numel()].view_as(b))
            o += b.numel()

    @property
    def grad_scale(self):
        return 1.0 / self.world


class _Done:
    def wait(self):
        return True


def _host_allreduce(t, op, group):
    """all_reduce of a device tensor through the host (gloo carries CPU tensors); synchronous."""
    h = t.cpu()
    dist.all_reduce(h, op=op, group=group)
    t.copy_(h)
    return _Done()


def allreduce_stats(stats, group=None, weight=1.0):
    """The Trainer's per-step metric vector (dfcsa.loss stats, fp32[8]) summed over the ranks, the
    loss entry averaged: IoU / Dice from the summed counts are the global batch's, the loss the
    mean of the per-replica losses, each weighted by its ``shard_weight`` (the
    4-scalar metric all-reduce).  A rank without rows passes zeros."""
    world = dist.get_world_size(group)
    out = stats.detach().clone()
    if weight != 1.0:
        out[0] *= weight
    if out.is_cuda and dist.get_backend(group) == "gloo":
        _host_allreduce(out, dist.ReduceOp.SUM, group)
    else:
        dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
    out[0] /= world
    return out


def notify_grads_ready(module):
    r = getattr(module, "_dfcsa_reducer", None)
    if r is not None:
        r.unit_ready(module)


def shard_rows(n, rank, world):
    """Rows [lo, hi) of a global batch of n owned by `rank`.  The split is as even as it can be:
    the first n % world ranks take one row more, and with n < world the last ranks take none (a
    dataset whose length is not a multiple of batch x world ends on such a ragged batch; the
    reference's DataLoader keeps it, utils/data_loader.py:153-159)."""
    per, rem = divmod(int(n), world)
    lo = rank * per + min(rank, rem)
    return lo, lo + per + (1 if rank < rem else 0)


def shard_weight(n, rank, world):
    """The factor this rank's loss gradient is scaled by so that the all-reduced SUM times 1/world
    is the row-weighted mean of the per-replica gradients, sum_r (n_r / n) g_r (= the plain mean
    when the batch divides evenly, where the factor is exactly 1)."""
    lo, hi = shard_rows(n, rank, world)
    return (hi - lo) * world / n if n else 0.0


def capture_step(fn):
    """Capture one call of ``fn`` (a whole training step) as a HIP graph; returns (graph, fn's
    result).

    The fix for the round-3 abort is the capture mode: ``thread_local``.  In torch's default
    global mode the HIP runtime refuses stream-unsafe calls from EVERY thread while a capture is
    open, and ProcessGroupNCCL's watchdog thread calls hipEventQuery on the eager collectives it
    tracks -- the refusal surfaced as an exception in the watchdog, which terminated the process
    (SIGABRT, "Exception raised from run at ProcessGroupNCCL.cpp").  In thread-local mode only the
    capturing thread is restricted, so the watchdog's polls are legal.

    The device synchronisation and the WATCHDOG_DRAIN_S pause before the capture are a margin, not
    the fix: they let the watchdog drop the completed warm-up collectives first, so nothing it
    tracks is in flight while the capture is open (collectives issued during a capture are not
    handed to the watchdog)."""
    torch.cuda.synchronize()
    if dist.is_available() and dist.is_initialized():
        time.sleep(WATCHDOG_DRAIN_S)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        out = fn()
    torch.cuda.synchronize()
    return graph, out


def shutdown(*graphs):
    """Leave a (data-parallel) run cleanly: release the captured graphs first -- a graph holding
    RCCL kernels references the communicator, and tearing the communicator down under it aborts
    -- then drain the device, meet the other ranks and destroy the process group."""
    for g in graphs:
        if g is not None:
            g.reset()
    torch.cuda.synchronize()
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
