"""Profiling driver (no torch): load N synthetic segments of a bench query's shape, run the query K times, print per-step stats.
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
ap.add_argument("--env", action="append", default=[], help="K=V set before the engine starts (A/B switches)")
a = ap.parse_args()
for kv in a.env:
    k, v = kv.split("=", 1)
    os.environ[k] = v
eng = Engine(0)
for i in range(a.segments):
    s = synth.make_segment(synth.segment_spec(i, rows=a.rows, threads=8, hour=bench.QUERIES[a.query].get("hour"),
                                              highcard_n=bench.QUERIES[a.query].get("highcard_n", 0)))
    eng.put_segment_ptr(f"seg/{i}", s.ptr, s.size)
    s.free()
q = bench.QUERIES[a.query]
segs = [synth.segment_request(i, step=q.get("step", 60000), hour=q.get("hour")) for i in range(a.segments)]
req = json.dumps(synth.pushdown(q["filter"], segs, q["agg"] or "sum", q["group_bys"], tag=q.get("tag")))
keys = [f"seg/{i}" for i in range(a.segments)]
for ab in a.ablate.split(","):
    os.environ["LK_ABLATE"] = ab
    for k in range(a.steps):
        r = eng.eval_pushdown(req, keys, 10, LK_MERGED)
    st = r.stats
    print(f"ablate={ab} scan_ms={st['scan_ms']:.3f} tiles={st.get('tiles')} rows={len(r)}", flush=True)
eng.close()
