"""Profiling driver (no torch): load N synthetic C2 segments, run the query K times, print per-step stats.
Used under rocprofv3; LK_ABLATE=1/2 time the kernel with a phase removed (diagnostics)."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lakeside_amd import LK_MERGED, synth
from lakeside_amd.evaluator import Engine
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench

ap = argparse.ArgumentParser()
ap.add_argument("--segments", type=int, default=16)
ap.add_argument("--rows", type=int, default=1 << 24)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--query", default="c2")
ap.add_argument("--ablate", default="0")
a = ap.parse_args()
eng = Engine(0)
for i in range(a.segments):
    s = synth.make_segment(synth.segment_spec(i, rows=a.rows, threads=8))
    eng.put_segment_ptr(f"seg/{i}", s.ptr, s.size)
    s.free()
q = bench.QUERIES[a.query]
req = json.dumps(synth.pushdown(q["filter"], [synth.segment_request(i) for i in range(a.segments)], q["agg"], q["group_bys"]))
keys = [f"seg/{i}" for i in range(a.segments)]
for ab in a.ablate.split(","):
    os.environ["LK_ABLATE"] = ab
    for k in range(a.steps):
        r = eng.eval_pushdown(req, keys, 10, LK_MERGED)
    st = r.stats
    print(f"ablate={ab} scan_ms={st['scan_ms']:.3f} GB/s={st['algorithmic_bytes']/st['scan_ms']/1e6:.0f} tiles={st['tiles']} rows={len(r)}", flush=True)
eng.close()
