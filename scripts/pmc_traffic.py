"""HBM traffic of the scan kernel from rocprofv3 PMC passes over the bench command (scripts/gpu_bench_prof.sh).

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch. On gfx950 FETCH_SIZE counts half the bytes of a
wide coalesced read (MI355X_MICROARCH.md, HBM section) and other widths are uncalibrated, so the factor is
measured here: the dense query reads every timestamp and value (all rows pass), whose byte count is the
algorithmic bytes of the launch; factor = algorithmic / FETCH_SIZE on that run, applied to the query's run.
"""
import csv, glob, json, os, statistics, sys

root, query = sys.argv[1], sys.argv[2]


def counter(d, name):
    vals = []
    for f in glob.glob(os.path.join(root, d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "scan_tiles" in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]) * 1024.0)
    return vals


def bench_line(name):
    with open(os.path.join(root, name)) as f:
        return json.loads(f.read().strip().splitlines()[-1])


q_fetch = counter("bench_fetch", "FETCH_SIZE")
q_write = counter("bench_write", "WRITE_SIZE")
d_fetch = counter("dense_fetch", "FETCH_SIZE")
q_alg = bench_line("bench_fetch.json")["roofline"]["algorithmic_bytes_per_launch"]
d_alg = bench_line("dense_fetch.json")["roofline"]["algorithmic_bytes_per_launch"]
factor = d_alg / statistics.median(d_fetch)
read = statistics.median(q_fetch) * factor
write = statistics.median(q_write)
out = {
    "query": query,
    "dispatches": len(q_fetch),
    "fetch_size_bytes_raw": statistics.median(q_fetch),
    "write_size_bytes_raw": write,
    "calibration": {"query": "dense", "algorithmic_bytes": d_alg, "fetch_size_bytes_raw": statistics.median(d_fetch),
                    "factor": factor},
    "hbm_read_bytes_per_launch": read,
    "hbm_bytes_per_launch": read + write,
    "algorithmic_bytes_per_launch": q_alg,
    "traffic_over_algorithmic": (read + write) / q_alg,
}
print(json.dumps(out, indent=1))
