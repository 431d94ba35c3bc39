"""Repeat the folded forward prologue GEMMs (tests/test_gpu_fold.py::_run_pro) over small / ragged
grids and report runs whose BatchNorm outputs are not finite or differ from the first run."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "dfc-sa-unet_amd")]
import torch  # noqa: E402

from test_gpu_fold import _run_pro  # noqa: E402

for pro, B, H, C in [(1, 3, 17, 128), (0, 3, 17, 128), (1, 3, 17, 64), (0, 3, 17, 64), (1, 16, 28, 128),
                     (1, 1, 8, 128), (1, 2, 30, 128)]:
    first = None
    bad = []
    for rep in range(8):
        out = _run_pro(pro, B, H, C, fold=True)
        fin = all(bool(torch.isfinite(t.float()).all()) for t in out[:6])
        same = first is None or all(torch.equal(a, b) for a, b in zip(first, out))
        if first is None:
            first = out
        if not fin or not same:
            bad.append((rep, fin, same))
    ref = _run_pro(pro, B, H, C, fold=False)
    err = max((a.double() - b.double()).abs().max().item() for a, b in zip(ref[:6], first[:6]))
    print(pro, B, H, C, "bad", bad, "max err vs unfolded", err, flush=True)
