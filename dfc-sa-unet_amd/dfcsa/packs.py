"""Persistent GEMM weight operands and the one-launch pack plan.

Every conv of the model is consumed by the implicit GEMMs as a packed, K-padded operand in the
compute dtype (forward rows [Cout][Kpad], transposed dgrad rows [Cin][Kpad], the fused 3x3 + 1x1
dgrad operand, ConvTranspose fwd/bwd layouts, concatenated bias vectors).  The fp32 master
weights change once per step (optimizer), so the packed operands are rebuilt once per forward.

A ``PackSet`` owns the packed tensors of one module and the table entries that fill them
(``dfcsa_pack_entry``, include/dfcsa.h).  The model gathers the PackSets of all its modules into
one ``PackPlan`` whose two device-resident tables are processed by two ``dfcsa_pack_plan``
launches at the start of each forward (instead of ~100 small pack launches): phase A permutes
the fp32 master weights into the forward operands (coalesced row reads), phase B transposes
those into the dgrad operands with 64x64 LDS tiles.  Modules used outside a model
(a standalone block) run their own PackSet.
"""
import ctypes

import torch

from . import _lib
from ._lib import call
from .ops import P, dt, stream

_EPOCH = [0]   # bumped whenever a PackSet is (re)created: invalidates gathered plans


def _table(entries, device):
    """Assign element ranges and upload the entry array; returns (uint8 device tensor, n, total)."""
    arr = (_lib.PackEntry * len(entries))()
    start = 0
    for i, e in enumerate(entries):
        arr[i] = e
        arr[i].start = start
        start += e.count
    raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(device)
    return raw, len(entries), start


class PackSet:
    """Packed operands of one module.  Phase-A entries read the fp32 master weights (ROWS,
    CONCAT, BIAS4); phase-B entries transpose phase-A outputs (so they run in a second launch)."""

    def __init__(self, key, device):
        self.key = key
        self.device = device
        self.t = {}
        self.entries = ([], [])
        self.fresh = False
        self._tabs = None
        _EPOCH[0] += 1

    def __getitem__(self, name):
        return self.t[name]

    def buffer(self, name, shape, dtype):
        """A zero-initialised persistent operand (padding stays zero: entries never write it)."""
        out = self.t.get(name)
        if out is None:
            out = torch.zeros(shape, dtype=dtype, device=self.device)
            self.t[name] = out
        return out

    def _entry(self, phase, kind, dtype, out_ptr, count, w0=None, w1=None, w2=None, a=()):
        e = _lib.PackEntry()
        e.count, e.kind, e.dtype = count, kind, dt(dtype)
        e.w0, e.w1, e.w2, e.out = w0, w1, w2, out_ptr
        for i, v in enumerate(a):
            e.a[i] = int(v)
        self.entries[phase].append(e)

    # ---- entry builders (semantics: include/dfcsa.h, DFCSA_PACK_*) ----
    def rows(self, name, dtype, w, Cpad, Kpad, row0=0, rows=None):
        """out[row0 + r][tap*Cpad + c] = w[r][c][tap] (conv weight [Cout][Cin][kh][kw]; for a
        ConvTranspose weight [Cin][Cout][2][2] this is its dgrad operand)."""
        out = self.buffer(name, (rows or w.shape[0], Kpad), dtype)
        R, Cc = w.shape[0], w.shape[1]
        ntaps = w.shape[2] * w.shape[3] if w.dim() == 4 else 1
        if ntaps * Cpad > Kpad or Cc > Cpad or row0 + R > out.shape[0]:
            raise ValueError("pack plan: rows entry does not fit its operand")
        per = max(1, 4096 // (Cc * ntaps))
        self._entry(0, 0, dtype, P(out), (R + per - 1) // per, w0=P(w),
                    a=(R, Cc, ntaps, Cpad, Kpad, row0, per))
        return out

    def transpose(self, src, r0, c0, R, C, name, shape, dr0=0, dc0=0):
        """dst[dr0 + c][dc0 + r] = src[r0 + r][c0 + c] (same dtype; src is a phase-A operand)."""
        dst = self.buffer(name, shape, src.dtype)
        if r0 + R > src.shape[0] or c0 + C > src.shape[1] or dr0 + C > dst.shape[0] or dc0 + R > dst.shape[1]:
            raise ValueError("pack plan: transpose out of range")
        es = src.element_size()
        tc = (C + 63) // 64
        self._entry(1, 1, src.dtype, dst.data_ptr() + (dr0 * dst.shape[1] + dc0) * es, ((R + 63) // 64) * tc,
                    w0=src.data_ptr() + (r0 * src.shape[1] + c0) * es, a=(R, C, src.shape[1], dst.shape[1], tc))
        return dst

    def concat(self, name, parts, total):
        """fp32 out = cat(parts) zero-padded to `total` (parts: up to three 1-D tensors)."""
        parts = list(parts) + [None] * (3 - len(parts))
        lens = [p.numel() if p is not None else 0 for p in parts]
        out = self.buffer(name, (total,), torch.float32)
        self._entry(0, 4, torch.float32, P(out), 1, w0=P(parts[0]), w1=P(parts[1]), w2=P(parts[2]),
                    a=(lens[0], lens[1], lens[2], total))
        return out

    def bias4(self, name, b):
        out = self.buffer(name, (4 * b.numel(),), torch.float32)
        self._entry(0, 5, torch.float32, P(out), 1, w0=P(b), a=(b.numel(),))
        return out

    # ---- execution ----
    def run(self):
        if self._tabs is None:
            self._tabs = [_table(es, self.device) for es in self.entries if es]
        for raw, n, total in self._tabs:
            call("dfcsa_pack_plan", P(raw), n, total, stream())


class PackPlan:
    """All PackSets of a model packed by one launch."""

    def __init__(self, sets, device):
        self.sets = list(sets)
        self.epoch = _EPOCH[0]
        self.tabs = []
        for phase in (0, 1):
            entries = [e for s in self.sets for e in s.entries[phase]]
            if entries:
                self.tabs.append(_table(entries, device))

    def valid(self):
        return self.epoch == _EPOCH[0]

    def run(self):
        for raw, n, total in self.tabs:
            call("dfcsa_pack_plan", P(raw), n, total, stream())
        for s in self.sets:
            s.fresh = True


def param_key(mod):
    return tuple(p.data_ptr() for p in mod.parameters())


def get_packset(mod, key, build):
    """The module's PackSet for `key` (built by build(PackSet) if absent/stale); packs it now
    unless a model-level plan already did for this forward."""
    ps = getattr(mod, "_dfcsa_pk", None)
    if ps is None or ps.key != key:
        dev = next(mod.parameters()).device
        ps = PackSet(key, dev)
        build(ps)
        mod._dfcsa_pk = ps
    if not ps.fresh:
        ps.run()
    ps.fresh = False
    return ps


def sync_model_plan(model):
    """Run the model-wide plan if valid (marks its sets fresh); returns False if it must be rebuilt
    after this forward (call rebuild_model_plan then)."""
    plan = getattr(model, "_dfcsa_plan", None)
    if plan is not None and plan.valid():
        plan.run()
        return True
    return False


def rebuild_model_plan(model, device):
    sets = [m._dfcsa_pk for m in model.modules() if getattr(m, "_dfcsa_pk", None) is not None]
    model._dfcsa_plan = PackPlan(sets, device)
