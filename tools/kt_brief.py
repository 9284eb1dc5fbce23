"""Summarise a rocprofv3 --kernel-trace --stats output directory: per kernel
the dispatch count, mean / median / min / max duration (us); for the step
kernels the duration of every dispatch in launch order (kt_dispatches.json)."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if not paths:
    sys.exit(f"no kernel_trace.csv under {d}")
rows = []
for p in paths:
    with open(p) as f:
        rows += list(csv.DictReader(f))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = {}
for r in rows:
    per.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
summary = {}
for k, v in per.items():
    summary[k] = {"n": len(v), "mean_us": statistics.fmean(v), "median_us": statistics.median(v),
                  "min_us": min(v), "max_us": max(v)}
steps = {k: v for k, v in per.items() if "k_step" in k}
with open(os.path.join(d, "kt_dispatches.json"), "w") as f:
    json.dump({"summary": summary, "step_dispatches_us": steps}, f, indent=1)
for k, s in sorted(summary.items(), key=lambda kv: -kv[1]["mean_us"] * kv[1]["n"])[:6]:
    print(f"  {k[:90]:90s} n={s['n']:5d} mean {s['mean_us']:9.2f} med {s['median_us']:9.2f} "
          f"min {s['min_us']:9.2f} max {s['max_us']:9.2f}")
for k, v in steps.items():
    print("  step dispatches:", " ".join(f"{x:.1f}" for x in v[:12]), "..." if len(v) > 12 else "")
