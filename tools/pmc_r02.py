"""Summarise the rocprofv3 PMC passes of tools/gpu_r02.sh (separate FETCH_SIZE,
WRITE_SIZE and SQ passes of the driver-shape bench) into profiles/.

    python tools/pmc_r02.py [--src gpurun_out/r02] [--tag r02]

Per step-kernel dispatch (the timed launch: the last k_step dispatch of the
20-step run; the mean over all dispatches of the 1-step run):
  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes  (MI355X_MICROARCH.md,
            HBM: gfx950 FETCH_SIZE counts half the bytes of wide streaming
            reads; WRITE_SIZE is exact for streaming stores);
  SQ_INSTS_VALU, SQ_WAIT_ANY / SQ_WAVE_CYCLES, SQ_WAVES.
Updates profiles/pmc_traffic.json and profiles/pmc_valu.json under the
bench's keys (C3_trendou_8192x8_fuse{K}).
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path):
    d = {}
    for r in csv.DictReader(open(path)):
        if "k_step" not in r["Kernel_Name"]:
            continue
        d.setdefault(int(r["Dispatch_Id"]), {})
        c = d[int(r["Dispatch_Id"])]
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "r02"))
    ap.add_argument("--tag", default="r02")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    tj, vj = os.path.join(prof, "pmc_traffic.json"), os.path.join(prof, "pmc_valu.json")
    traffic = json.load(open(tj)) if os.path.exists(tj) else {}
    valu = json.load(open(vj)) if os.path.exists(vj) else {}
    out = {}
    for K, pick in (("20", "last"), ("1", "mean"), ("256", "mean")):
        merged = {}
        for part in ("fetch", "write", "sq"):
            f = os.path.join(a.src, f"pmc{K}", part, "p_counter_collection.csv")
            if not os.path.exists(f):
                continue
            d = per_dispatch(f)
            ids = sorted(d)
            sel = [d[ids[-1]]] if pick == "last" else [d[i] for i in ids]
            for c in sel[0]:
                merged[c] = sum(s[c] for s in sel) / len(sel)
        if not merged:
            continue
        key = f"C3_trendou_8192x8_fuse{K}"
        s = {"counters_per_dispatch": merged, "dispatches": pick}
        if "FETCH_SIZE" in merged and "WRITE_SIZE" in merged:
            s["hbm_bytes_per_launch"] = (2 * merged["FETCH_SIZE"] + merged["WRITE_SIZE"]) * 1024
            s["hbm_bytes_per_env_step"] = s["hbm_bytes_per_launch"] / (8192 * int(K))
            traffic[key] = s["hbm_bytes_per_launch"]
        if "SQ_INSTS_VALU" in merged:
            valu[key] = merged["SQ_INSTS_VALU"]
            s["valu_wave_insts_per_wave_step"] = merged["SQ_INSTS_VALU"] / merged["SQ_WAVES"] / int(K)
            s["wait_any_frac"] = merged["SQ_WAIT_ANY"] / merged["SQ_WAVE_CYCLES"]
        out[key] = s
    for K in ("20", "1", "256"):
        ks = os.path.join(a.src, f"kt{K}", "kt_kernel_stats.csv")
        if os.path.exists(ks):
            shutil.copy(ks, os.path.join(prof, f"{a.tag}_kernel_stats_fuse{K}.csv"))
    json.dump(traffic, open(tj, "w"), indent=1, sort_keys=True)
    json.dump(valu, open(vj, "w"), indent=1, sort_keys=True)
    json.dump(out, open(os.path.join(prof, f"{a.tag}_pmc_driver_shape.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
