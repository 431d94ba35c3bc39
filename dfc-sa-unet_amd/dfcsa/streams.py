"""Optional side HIP stream for the weight-gradient work of the backward pass.

In a block's backward the weight-gradient GEMMs (pixel reductions dW = dY^T X) depend only on
the activation gradient dY and saved forward tensors; nothing on the data-gradient chain waits
for them.  They are therefore issued on a second stream forked from the compute stream at the
point dY exists, so the MFMA-bound wgrad kernels fill the CUs left idle by the latency- and
HBM-bound elementwise / reduction kernels of the dgrad chain.  Tensors read on the side stream
are ``record_stream``-ed (the caching allocator must not hand their memory to the compute
stream before the side stream is done), and the compute stream joins the side stream when the
autograd pass ends (``queue_callback``), so any consumer of ``param.grad`` -- the fused
optimizer, ``clip_grad_norm_``, a DDP reducer -- sees complete gradients.  The fork/join is
event-based and captures into HIP graphs.
"""
import contextlib

import torch

_SIDE = {}
_JOIN_QUEUED = [False]
import os

# On by default since round 4: with the round-3 kernels the backward's dgrad chain is a string of
# latency-bound launches (BatchNorm finalizers on 1-16 workgroups, the pooled-attention backward on
# 16-224) that leave most CUs idle, and the HBM-streaming weight-gradient GEMMs fill them (same-box
# A/B of the default bench: 1497 / 1499 on vs 1469 / 1473 img/s off; round 2, when the dgrad chain
# was GEMM-bound: 1245 on vs 1251 off).  DFCSA_SIDE_STREAM=0 disables.
ENABLED = [os.environ.get("DFCSA_SIDE_STREAM", "1") == "1"]


# HIP stream priorities (torch: lower value = higher priority): the weight-gradient side stream and
# the attention branch stream are created with these (DFCSA_PRIO_SIDE / DFCSA_PRIO_BRANCH)
PRIO_SIDE = int(os.environ.get("DFCSA_PRIO_SIDE", "0"))
PRIO_BRANCH = int(os.environ.get("DFCSA_PRIO_BRANCH", "0"))


# The TransUNet (config 4) and plain UNet (config 1) backward passes issue their weight gradients
# through side_or_main: measured slower on the side stream there (config 4 bf16, same box: 559-563
# vs 568 img/s with everything on one stream -- its small M = 1568 ViT GEMMs fill the chip on
# their own), so DFCSA_SIDE_STREAM_TU=1 opts in.
SIDE_TU = [os.environ.get("DFCSA_SIDE_STREAM_TU", "0") == "1"]


def side_or_main(device, *tensors):
    """on_side for the TransUNet / UNet weight gradients when SIDE_TU is set, else the current stream."""
    if SIDE_TU[0]:
        return on_side(device, *tensors)
    return contextlib.nullcontext()


def side_stream(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx, priority=PRIO_SIDE)
        _SIDE[idx] = s
    return s


# side-stream work deferred to a later point of the backward (block_backward, DFCSA_DEFER_WGRAD):
# run by the next flush_deferred() and, at the latest, by the end-of-backward join
_DEFERRED = []


def defer(fn):
    _DEFERRED.append(fn)


def clear_deferred():
    """Drop queued deferred launches without running them (after an aborted / failed capture)."""
    _DEFERRED.clear()


def flush_deferred():
    while _DEFERRED:
        _DEFERRED.pop(0)()


def _join():
    flush_deferred()
    _JOIN_QUEUED[0] = False
    cur = torch.cuda.current_stream()
    for s in _SIDE.values():
        if s.device == cur.device:
            cur.wait_stream(s)


def join():
    """Make the current stream wait for all side-stream work (idempotent, cheap)."""
    _join()


@contextlib.contextmanager
def on_side(device, *tensors):
    """Run the enclosed launches on the side stream, after everything issued so far on the
    current stream; `tensors` (allocated elsewhere) are marked as used by the side stream."""
    if not ENABLED[0]:
        yield
        return
    main = torch.cuda.current_stream(device)
    side = side_stream(device)
    side.wait_stream(main)
    if not _JOIN_QUEUED[0]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(_join)
            _JOIN_QUEUED[0] = True
        except RuntimeError:
            pass  # not inside a backward pass: the caller joins explicitly
    with torch.cuda.stream(side):
        yield side
    for t in tensors:
        if t is not None:
            t.record_stream(side)


# ---------------------------------------------------------------------------------------------
# Branch stream: concurrency INSIDE a block.  The LightSelfAttention chain of a DFC-SA block
# (pooled statistics, q/k/v projections on B*P*P rows, the N = P*P softmax core and their
# backward) is a string of latency-bound launches that use a few dozen workgroups each, and it
# is independent of the local 3x3 branch in both directions (forward: after the 1x1 attention
# entry conv, until the local/attention merge; backward: after the gate backward, until the
# input-gradient GEMM).  It is forked onto this stream so that it runs beside the local branch's
# GEMM / elementwise kernels instead of between them.  DFCSA_BRANCH_STREAM=0 disables it.
BRANCH_ENABLED = [os.environ.get("DFCSA_BRANCH_STREAM", "1") == "1"]
_BRANCH = {}


def branch_stream(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _BRANCH.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx, priority=PRIO_BRANCH)
        _BRANCH[idx] = s
    return s


def _record(obj, stream):
    if obj is None:
        return
    if isinstance(obj, torch.Tensor):
        obj.record_stream(stream)
    elif isinstance(obj, (tuple, list)):
        for o in obj:
            _record(o, stream)
    else:  # a plain record object (e.g. ops.BNState, __slots__ of tensors)
        names = list(getattr(obj, "__slots__", ())) + list(getattr(obj, "__dict__", {}).keys())
        for n in names:
            o = getattr(obj, n, None)
            if isinstance(o, (torch.Tensor, tuple, list)):
                _record(o, stream)


@contextlib.contextmanager
def on_branch(device, enabled, *inputs):
    """Run the enclosed launches on the branch stream, after everything issued so far on the
    current stream.  `inputs` (allocated on the current stream, read on the branch) are
    record_stream-ed.  The caller joins with join_branch(device, enabled, *outputs)."""
    if not (enabled and BRANCH_ENABLED[0]):
        yield None
        return
    main = torch.cuda.current_stream(device)
    br = branch_stream(device)
    br.wait_stream(main)
    with torch.cuda.stream(br):
        yield br
    _record(inputs, br)


def join_branch(device, enabled, *outputs):
    """The current stream waits for the branch; `outputs` (allocated on the branch, used on the
    current stream from here on) are record_stream-ed."""
    if not (enabled and BRANCH_ENABLED[0]):
        return
    main = torch.cuda.current_stream(device)
    main.wait_stream(branch_stream(device))
    _record(outputs, main)
