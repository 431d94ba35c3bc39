"""Flat fp32 storage for all parameters (and their gradients) of a model.

Every nn.Parameter becomes a view into one contiguous buffer (offsets aligned to 64 floats),
and every ``param.grad`` a view into a second one, in ``model.parameters()`` order (the
order torch.optim.SGD and clip_grad_norm_ see, utils/trainer.py:149).  Gradient clipping,
the SGD update and the data-parallel all-reduce then run as single passes over one buffer.
Kernels accumulate into ``param.grad`` in place, so gradients keep PyTorch's accumulate
semantics; ``zero_grad`` is one memset.
"""
import torch

ALIGN = 64


class FlatParams:
    def __init__(self, module):
        params = [p for p in module.parameters()]
        if not params:
            raise ValueError("module has no parameters")
        dev = params[0].device
        offs, o = [], 0
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise TypeError("flat parameters must all be fp32 on one device")
            offs.append(o)
            o += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = o
        self.params = params
        self.offsets = offs
        self.device = dev
        self.data = torch.zeros(o, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(o, dtype=torch.float32, device=dev)
        self.views = []
        with torch.no_grad():
            for p, off in zip(params, offs):
                n = p.numel()
                self.data[off:off + n].copy_(p.data.reshape(-1))
                p.data = self.data[off:off + n].view_as(p)
                gv = self.grad[off:off + n].view_as(p)
                if p.grad is not None:
                    gv.copy_(p.grad)
                p.grad = gv
                self.views.append(gv)
                p._dfcsa_flat = self

    def valid(self):
        return all(p.data_ptr() == self.data.data_ptr() + 4 * off for p, off in zip(self.params, self.offsets))

    def attach_grads(self):
        """Re-point every param.grad at its flat view (zeroing views whose grad was None)."""
        for p, gv in zip(self.params, self.views):
            g = p.grad
            if g is None:
                gv.zero_()
                p.grad = gv
            elif g.data_ptr() != gv.data_ptr():
                gv.copy_(g)
                p.grad = gv

    def zero_grad(self):
        self.grad.zero_()
        self.attach_grads()
