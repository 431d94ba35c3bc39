"""dfcsa: MI355X-native runtime for the DFC-SA-Res U-Net training step.

Importing this package loads libdfcsa.so (HIP kernels for gfx950) and fails loudly if it is
missing.  Public pieces:
  dfcsa.block       DFC block forward/backward on the kernels
  dfcsa.functions   U-Net plumbing (pooling, transposed conv, head, ...)
  dfcsa.loss        sigmoid + BCE/Dice loss and metrics
  dfcsa.flat        flat fp32 parameter / gradient storage
  dfcsa.optim       fused clip_grad_norm_ + momentum SGD
  dfcsa.ddp         data parallelism over RCCL (torch.distributed 'nccl' backend)
"""
import os

from ._lib import LIB as _LIB
from ._lib import version  # noqa: F401


def set_tuning(knob, value):
    """Benchmark-only kernel selection overrides (include/dfcsa.h, dfcsa_set_tuning).  Knob 31 (the
    cooperative split-K weight-gradient reduction) is refused while the side or branch stream is on:
    it assumes every workgroup of its grid is co-resident, which concurrent streams do not guarantee."""
    if int(knob) == 31 and int(value):
        from . import streams
        if streams.ENABLED[0] or streams.BRANCH_ENABLED[0]:
            raise ValueError("tuning knob 31 needs DFCSA_SIDE_STREAM=0 and DFCSA_BRANCH_STREAM=0")
    if _LIB.dfcsa_set_tuning(int(knob), int(value)) != 0:
        raise ValueError(f"unknown tuning knob {knob}")


def check_wgrad_coop():
    """Fail loudly if the opt-in cooperative split-K weight-gradient reduction (knob 31) ever ran
    out of its bounded wait.  That reduction assumes every workgroup of its grid is co-resident;
    with the side and branch streams sharing the CUs a split can wait past the bound, and the tile
    is then reduced from partial sums -- a wrong gradient whose only trace is this sticky device
    flag.  No-op when the knob is off (the default), so it costs nothing on the shipped path."""
    if _LIB.dfcsa_get_tuning(31) and _LIB.dfcsa_wgrad_coop_errors(0):
        raise RuntimeError("cooperative split-K weight-gradient reduction (knob 31) exceeded its bounded "
                           "wait: gradients of this run are wrong; leave knob 31 off with concurrent streams")


for _kv in filter(None, os.environ.get("DFCSA_TUNE", "").split(",")):   # e.g. DFCSA_TUNE=2=1024
    _k, _v = _kv.split("=")
    set_tuning(_k, _v)

PRECISIONS = {"bf16": "bfloat16", "bfloat16": "bfloat16", "fp32": "float32", "float32": "float32"}


def resolve_dtype(precision):
    import torch
    if precision is None:
        return torch.bfloat16
    if isinstance(precision, torch.dtype):
        if precision not in (torch.bfloat16, torch.float32):
            raise ValueError(f"unsupported compute dtype {precision}")
        return precision
    key = str(precision).lower()
    if key not in PRECISIONS:
        raise ValueError(f"unsupported precision {precision!r} (use 'bf16' or 'fp32')")
    return getattr(torch, PRECISIONS[key])
