"""GPU-box diagnostic: the exemplar shapes of tests/test_gpu_exemplar.py, reporting per case and per glob which rows
differ from the oracle (missing / extra (ts, glob) pairs) instead of stopping at the first mismatch."""
import json
import os
import sys
import tempfile
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lakeside_amd import LK_PER_GLOB_ROWS, synth
    from lakeside_amd.evaluator import Engine
    from oracle import dataexpr as dx
    from oracle import exemplar as ex
    from tests.test_gpu_exemplar import SVC, _logs_files, _request
    tmp = Path(tempfile.mkdtemp())
    paths, blobs = _logs_files(tmp)
    eng = Engine(0)
    for p in paths:
        eng.load_segment(p)
    name_eq = synth.leaf(dx.NAME, "eq", "metric_02")
    svc_re = synth.leaf(SVC, "regex", "^svc-a")
    cases = [("default", name_eq, {}, 2), ("reverse_sort", svc_re, {"limit": 50, "reverse": True}, 3),
             ("reverse_nolimit", svc_re, {"limit": 100000, "reverse": True}, 3),
             ("everything", {"k": SVC, "v": [], "op": "exists"}, {"limit": 100_000}, 4),
             ("everything3", {"k": SVC, "v": [], "op": "exists"}, {"limit": 100_000}, 3)]
    for label, filt, kw, gs in cases:
        req = _request(filt, len(paths), limit=kw.get("limit"), order=kw.get("order"), reverse=kw.get("reverse", False))
        pr = dx.parse_pushdown(req)
        want = ex.evaluate_exemplar(pr, paths, gs, sources=blobs)
        got = eng.eval_pushdown(req, paths, gs, LK_PER_GLOB_ROWS)
        g = list(zip(got.ts.tolist(), got.globs.tolist()))
        w = [(r[0], r[3]) for r in want]
        sg, sw = set(g), set(w)
        print(f"{label}: got {len(g)} want {len(w)}; missing {sorted(sw - sg)[:8]} extra {sorted(sg - sw)[:8]}; "
              f"order equal {g == w}; stats {got.stats}", flush=True)
        if g != w:
            for i in range(min(6, len(g), len(w))):
                print(f"   {i}: got {g[i]} want {w[i]}")
    eng.close()


if __name__ == "__main__":
    main()
