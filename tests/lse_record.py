"""softmax_lse deviation records.

The folded calls (attn_folds_q: head dim 64 / 128, no dropout) score from Q' = bf16/f16(scale
log2(e) Q), one rounding of Q the reference does not make, so their LSE can leave the plain 2x rule
of ``oracle.attention_ref.check_lse_within_bound`` (|lse - ref| <= max(2 |lse_pt - ref|,
atol + rtol |ref|)) on rows where the PyTorch path's own LSE error happens to be small.  ``lse_ratio``
measures by how much, row by row, and ``record`` appends the figures as one JSON line to the file
named by FA_LSE_LOG (unset: nothing is written), so a GPU run leaves the distribution behind
(``tools/lse_summary.py`` summarises it; DESIGN.md deviation 8 quotes it)."""
import json
import os

import torch


def lse_ratio(lse, ref, pt, atol=1e-3, rtol=1e-4):
    """(worst err / bound, rows over the bound, live rows, max err, pt err) of the plain 2x rule."""
    lse, ref, pt = (x.detach().double().cpu() for x in (lse, ref, pt))
    live = ~torch.isinf(ref)
    if not live.any():
        return 0.0, 0, 0, 0.0, 0.0
    err = (lse[live] - ref[live]).abs()
    pt_err = float((pt[live] - ref[live]).abs().max())
    bound = torch.clamp(atol + rtol * ref[live].abs(), min=2.0 * pt_err)
    r = err / bound
    return float(r.max()), int((r > 1).sum()), int(live.sum()), float(err.max()), pt_err


def record(test, case, ratio, over, rows, err, pt_err):
    path = os.environ.get("FA_LSE_LOG")
    if not path:
        return
    with open(path, "a") as f:
        f.write(json.dumps(dict(test=test, case=str(case), ratio=ratio, rows_over=over, rows=rows, err=err,
                                pt_err=pt_err)) + "\n")
