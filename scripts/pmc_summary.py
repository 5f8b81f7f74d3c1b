"""Summarise rocprofv3 --pmc CSVs: per directory, the mean counter values of the scan kernel's dispatches
(the last dispatch of each counter set; scan_tiles / scan_lean)."""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
for d in sorted(glob.glob(os.path.join(root, "pmc*"))):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    vals = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if "scan_tiles" not in row["Kernel_Name"] and "scan_lean" not in row["Kernel_Name"]:
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not vals:
        continue
    out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    waves = out.get("SQ_WAVES")
    line = " ".join(f"{k}={v:.4g}" for k, v in out.items())
    print(f"{os.path.basename(d)}: {line}")
    if waves:
        per = " ".join(f"{k}/wave={v / waves:.1f}" for k, v in out.items() if k.startswith("SQ_INSTS"))
        print(f"    {per}")
