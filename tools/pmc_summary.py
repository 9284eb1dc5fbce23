"""Summarise a tools/prof.sh run (rocprofv3 CSVs under gpurun_out/prof) into
profiles/: kernel stats, per-dispatch PMC means, and profiles/pmc_traffic.json
(HBM bytes per launch of the step kernel, the bench's roofline.traffic).

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half of the
bytes of a wide coalesced streaming read, so bytes = 2*FETCH_SIZE*1024 +
WRITE_SIZE*1024 (WRITE_SIZE is exact for streaming stores).  The step kernel's
reads are mostly small (state once per launch, int8 actions), so the doubled
read term is an upper bound; it is a small fraction of the total either way.

    python tools/pmc_summary.py --tag r01 --workload C3_trendou_8192x8_fuse64
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(prof):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(prof, "pmc*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "k_step" not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
            names[r["Counter_Name"]] = r["Kernel_Name"]
    return {c: sum(d.values()) / len(d) for c, d in agg.items()}, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prof", default=os.path.join(ROOT, "gpurun_out", "prof"))
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--workload", default="C3_trendou_8192x8_fuse64")
    ap.add_argument("--bytes-per-launch", type=float, default=None,
                    help="algorithmic bytes per launch, for the ratio")
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    ks = os.path.join(a.prof, "kt", "kt_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
    c, _ = counters(a.prof)
    summary = {"per_dispatch_mean": c}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        traffic = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        summary["hbm_bytes_per_launch"] = traffic
        summary["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
        summary["write_bytes"] = c["WRITE_SIZE"] * 1024
        if a.bytes_per_launch:
            summary["traffic_over_algorithmic"] = traffic / a.bytes_per_launch
        tj = os.path.join(out, "pmc_traffic.json")
        d = json.load(open(tj)) if os.path.exists(tj) else {}
        d[a.workload] = traffic
        json.dump(d, open(tj, "w"), indent=1, sort_keys=True)
    if "SQ_WAVES" in c and "SQ_INSTS_VALU" in c:
        summary["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        vj = os.path.join(out, "pmc_valu.json")
        d = json.load(open(vj)) if os.path.exists(vj) else {}
        d[a.workload] = c["SQ_INSTS_VALU"]  # wave-level VALU instructions per launch
        json.dump(d, open(vj, "w"), indent=1, sort_keys=True)
    json.dump(summary, open(os.path.join(out, f"{a.tag}_pmc_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
