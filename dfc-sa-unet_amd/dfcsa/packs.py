"""Persistent GEMM weight operands and the one-launch pack plan.

Every conv of the model is consumed by the implicit GEMMs as a packed, K-padded operand in the
compute dtype (forward rows [Cout][Kpad], transposed dgrad rows [Cin][Kpad], the fused 3x3 + 1x1
dgrad operand, ConvTranspose fwd/bwd layouts, concatenated bias vectors).  The fp32 master
weights change once per step (optimizer), so the packed operands are rebuilt once per forward.

A ``PackSet`` owns the packed tensors of one module and the table entries that fill them
(``dfcsa_pack_entry``, include/dfcsa.h).  The model gathers the PackSets of all its modules into
one ``PackPlan`` whose device-resident table is processed by ONE ``dfcsa_pack_plan`` launch at
the start of each forward (instead of ~100 small pack launches).  Modules used outside a model
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
    def __init__(self, key, device):
        self.key = key
        self.device = device
        self.t = {}
        self.entries = []
        self.fresh = False
        self._tab = None
        _EPOCH[0] += 1

    def __getitem__(self, name):
        return self.t[name]

    def _new(self, name, shape, dtype):
        out = torch.empty(shape, dtype=dtype, device=self.device)
        self.t[name] = out
        return out

    def _entry(self, kind, dtype, out, count, w0=None, w1=None, w2=None, a=()):
        e = _lib.PackEntry()
        e.count, e.kind, e.dtype = count, kind, dt(dtype)
        e.w0, e.w1, e.w2, e.out = P(w0), P(w1), P(w2), P(out)
        for i, v in enumerate(a):
            e.a[i] = int(v)
        self.entries.append(e)

    # ---- entry builders (semantics: include/dfcsa.h, DFCSA_PACK_*) ----
    def rows(self, name, dtype, w, Cpad, Kpad, row0=0, rows=None):
        """forward operand: out[row0 + co][tap*Cpad + ci] = w[co][ci][tap]"""
        out = self.t.get(name)
        if out is None:
            out = self._new(name, (rows or w.shape[0], Kpad), dtype)
        ntaps = w.shape[2] * w.shape[3] if w.dim() == 4 else 1
        self._entry(0, dtype, out, w.shape[0] * Kpad, w0=w, a=(w.shape[0], w.shape[1], ntaps, Cpad, Kpad, row0))
        return out

    def t3(self, name, dtype, Cin, Kpad, ws, identity_last=False):
        """transposed dgrad operand of up to three weights side by side (pack_t3 semantics)."""
        ws = list(ws) + [None] * (3 - len(ws))
        wcin = next(w.shape[1] for w in ws if w is not None)
        t0 = (ws[0].shape[2] * ws[0].shape[3]) if ws[0].dim() == 4 else 1
        for w in ws[1:]:
            if w is not None and w.dim() == 4 and w.shape[2] * w.shape[3] != 1:
                raise ValueError("pack plan: segments 1 and 2 must be 1x1 weights")
        c = [w.shape[0] if w is not None else 0 for w in ws]
        if identity_last:
            c[2] = Cin
        if t0 * c[0] + c[1] + c[2] > Kpad:
            raise ValueError("pack plan: t3 segments exceed Kpad")
        out = self._new(name, (Cin, Kpad), dtype)
        self._entry(1, dtype, out, Cin * Kpad, w0=ws[0], w1=ws[1], w2=ws[2],
                    a=(Cin, Kpad, wcin, c[0], c[1], c[2], t0, int(identity_last)))
        return out

    def convT(self, dtype, w, bias, Kf, Kb):
        Cin, Cout = w.shape[0], w.shape[1]
        wf = self._new("Wf", (4 * Cout, Kf), dtype)
        self._entry(2, dtype, wf, 4 * Cout * Kf, w0=w, a=(Cin, Cout, Kf))
        wb = self._new("Wb", (Cin, Kb), dtype)
        self._entry(3, dtype, wb, Cin * Kb, w0=w, a=(Cin, Cout, Kb))
        b4 = self._new("b4", (4 * Cout,), torch.float32)
        self._entry(5, torch.float32, b4, 4 * Cout, w0=bias, a=(Cout,))

    def concat(self, name, parts, total):
        """fp32 out = cat(parts) zero-padded to `total` (parts: up to three 1-D tensors or None)."""
        parts = list(parts) + [None] * (3 - len(parts))
        lens = [p.numel() if p is not None else 0 for p in parts]
        out = self._new(name, (total,), torch.float32)
        self._entry(4, torch.float32, out, total, w0=parts[0], w1=parts[1], w2=parts[2],
                    a=(lens[0], lens[1], lens[2], total))
        return out

    # ---- execution ----
    def run(self):
        if self._tab is None:
            self._tab = _table(self.entries, self.device)
        raw, n, total = self._tab
        call("dfcsa_pack_plan", P(raw), n, total, stream())


class PackPlan:
    """All PackSets of a model packed by one launch."""

    def __init__(self, sets, device):
        self.sets = list(sets)
        self.epoch = _EPOCH[0]
        entries = [e for s in self.sets for e in s.entries]
        self.tab = _table(entries, device) if entries else None

    def valid(self):
        return self.epoch == _EPOCH[0]

    def run(self):
        if self.tab is not None:
            raw, n, total = self.tab
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
