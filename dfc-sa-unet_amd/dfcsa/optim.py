"""Fused clip_grad_norm_ + momentum SGD over a model's flat parameter buffer.

Replaces, in one device pass and without host synchronisation:
  torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)   utils/trainer.py:149
  torch.optim.SGD(lr, momentum, weight_decay).step()                  train.py:73-78, trainer.py:151
with torch's semantics (weight decay added to the gradient before momentum; first step
initialises the buffer to the gradient -- the buffer starts at zero, so momentum * 0 + d is that
first step exactly; p.grad holds the clipped gradient afterwards).

``zero_after_step=True`` (bench.py) has the same pass write zeros to the gradients
instead of the clipped values, and the next ``zero_grad`` then skips its memset; the weights and
momentum are the same either way.
"""
import ctypes

import torch

from . import chanpad, streams
from ._lib import LIB, call
from .ops import P, stream


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=0.01, momentum=0.0, weight_decay=0.0, dampening=0.0, nesterov=False,
                 zero_after_step=False):
        if dampening != 0.0 or nesterov:
            raise NotImplementedError("FusedSGD implements the reference's SGD (no dampening/nesterov)")
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, dampening=0.0,
                                      nesterov=False, maximize=False, foreach=None, differentiable=False,
                                      fused=None))
        if len(self.param_groups) != 1:
            raise NotImplementedError("FusedSGD supports a single parameter group")
        self._flat = None
        self._mom = None
        self._mom_init = None
        self._partial = None
        self._pending_mom = None   # momentum buffers loaded before the flat storage existed
        self.last_norm = None
        self.zero_after_step = zero_after_step
        self._grads_zeroed = False  # the last step() zeroed the gradients (zero_after_step)

    def add_param_group(self, param_group):
        if getattr(self, "_flat", "init") != "init" or self.param_groups:
            raise NotImplementedError("FusedSGD supports a single parameter group (the model's flat buffer)")
        super().add_param_group(param_group)

    @classmethod
    def from_torch_sgd(cls, opt):
        """The fused equivalent of a ``torch.optim.SGD`` built as in the reference's train.py:73-78
        (one group, no dampening/nesterov); None if the optimizer is something else."""
        if type(opt) is not torch.optim.SGD or len(opt.param_groups) != 1:
            return None
        g = opt.param_groups[0]
        if g.get("dampening", 0.0) or g.get("nesterov", False) or g.get("maximize", False) or any(opt.state.values()):
            return None
        return cls(g["params"], lr=g["lr"], momentum=g["momentum"], weight_decay=g["weight_decay"])

    # ------------------------------------------------------------------ helpers
    def _resolve(self):
        params = self.param_groups[0]["params"]
        flat = getattr(params[0], "_dfcsa_flat", None)
        if flat is None or not flat.valid() or len(flat.params) != len(params) or \
                any(a is not b for a, b in zip(flat.params, params)):
            raise RuntimeError("FusedSGD needs the parameters of a dfcsa model after its first forward "
                               "(they live in one flat buffer); got foreign parameters")
        frozen = [i for i, p in enumerate(params) if not p.requires_grad]
        if frozen:
            # torch's SGD skips parameters without a gradient; the fused pass updates the whole
            # flat buffer, so frozen parameters would drift under weight decay / momentum
            raise NotImplementedError(f"FusedSGD: {len(frozen)} parameter(s) have requires_grad=False; "
                                      "freeze nothing or use torch.optim.SGD")
        if flat is not self._flat:
            self._flat = flat
            self._mom = torch.zeros_like(flat.data)
            self._partial = torch.empty(LIB.dfcsa_sumsq_nparts(flat.numel), dtype=torch.float64,
                                        device=flat.device)
            self.last_norm = torch.zeros(1, dtype=torch.float32, device=flat.device)
            pending, self._pending_mom = self._pending_mom, None
            for p, off in zip(flat.params, flat.offsets):
                view = self._mom[off:off + p.numel()].view_as(p)
                if pending is not None:
                    view.copy_(pending[id(p)])
                self.state[p]["momentum_buffer"] = view
        return flat

    def zero_grad(self, set_to_none=True):
        flat = getattr(self.param_groups[0]["params"][0], "_dfcsa_flat", None)
        if flat is not None and flat.valid():
            if self._grads_zeroed and flat is self._flat:
                flat.attach_grads()   # the last step() already wrote zeros
            else:
                flat.zero_grad()  # one memset; grads stay views of the flat buffer
            self._grads_zeroed = False
        else:
            super().zero_grad(set_to_none)

    @torch.no_grad()
    def step(self, closure=None, max_norm=None, grad_scale=1.0, skip_if_nan=None):
        """max_norm: clip the global L2 norm first (None = no clipping).
        grad_scale: multiply gradients first (1/world_size after an all-reduce sum).
        skip_if_nan: device scalar; the update is skipped on the device if it is NaN (the
        reference's NaN-loss skip, utils/trainer.py:134-139; an inf loss still steps)."""
        loss = closure() if closure is not None else None
        flat = self._resolve()
        streams.join()  # weight gradients may still be in flight on the side stream
        g = self.param_groups[0]
        n = flat.numel
        if max_norm is not None:
            call("dfcsa_sumsq_partial", ctypes.c_int64(n), P(flat.grad), P(self._partial), stream())
            nparts, mn = self._partial.numel(), float(max_norm)
        else:
            nparts, mn = 0, float("inf")
        call("dfcsa_clip_sgd2", ctypes.c_int64(n), P(flat.data), P(flat.grad), P(self._mom), P(self._partial),
             nparts, mn, float(grad_scale), float(g["lr"]), float(g["momentum"]), float(g["weight_decay"]),
             int(bool(self.zero_after_step)), P(skip_if_nan), P(self.last_norm), stream())
        self._grads_zeroed = bool(self.zero_after_step)
        return loss

    def state_dict(self):
        """torch.optim.SGD's format; momentum buffers of channel-padded parameters (dfcsa.chanpad)
        in their reference shapes."""
        sd = super().state_dict()
        # torch numbers the state by a running index over every group's parameters
        params = [p for g in self.param_groups for p in g["params"]]
        for i, p in enumerate(params):
            st = sd["state"].get(i)
            if st is not None and st.get("momentum_buffer") is not None and hasattr(p, "_dfcsa_pad"):
                sd["state"][i] = dict(st, momentum_buffer=chanpad.logical(p, st["momentum_buffer"]).clone())
        return sd

    def load_state_dict(self, state_dict):
        """torch.optim.SGD state (e.g. a reference checkpoint's optimizer_state_dict): the loaded
        momentum buffers are copied into the flat momentum storage -- now if it exists, otherwise
        when the model's first forward has created it (the next step() resolves it)."""
        super().load_state_dict(state_dict)
        params = self.param_groups[0]["params"]
        bufs = [self.state[p].get("momentum_buffer") if p in self.state else None for p in params]
        if not all(b is not None for b in bufs):
            # no momentum in the checkpoint (taken before the first step): start fresh, as
            # torch.optim.SGD does from an empty state -- forget any momentum already held
            self._pending_mom = None
            if self._mom is not None:
                self._mom.zero_()
            return
        flat = getattr(params[0], "_dfcsa_flat", None)
        self._pending_mom = {id(p): chanpad.padded(p, b.detach()).clone() for p, b in zip(params, bufs)}
        self._flat = None
        if flat is not None and flat.valid():
            self._resolve()
