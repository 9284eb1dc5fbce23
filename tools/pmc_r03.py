"""Summarise tools/gpu_r03_final.sh into profiles/ (round 3).

    python tools/pmc_r03.py [--src gpurun_out/r03final] [--tag r03]

Per kernel dispatch (the C3 step kernel: the last dispatch of the 20-step run,
the mean over the 1- and 256-step runs; C4 / C5: the mean over every
k_hist_gather and every step-kernel dispatch of the timed launches):
  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes  (MI355X_MICROARCH.md
            HBM section: gfx950 FETCH_SIZE counts half the bytes of wide
            streaming reads; WRITE_SIZE is exact), separate PMC passes;
  SQ_INSTS_VALU, SQ_WAIT_ANY / SQ_WAVE_CYCLES, SQ_WAVES.
Updates profiles/pmc_traffic.json / pmc_valu.json under the bench's keys and
copies the kernel-stat summaries, bench lines and the GPU test log.
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, match):
    d = {}
    for r in csv.DictReader(open(path)):
        if match not in r["Kernel_Name"]:
            continue
        c = d.setdefault(int(r["Dispatch_Id"]), {})
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return d


def merged(src, tag, match, pick):
    out = {}
    for part in ("fetch", "write", "sq"):
        f = os.path.join(src, f"pmc{tag}", part, "p_counter_collection.csv")
        if not os.path.exists(f):
            continue
        d = per_dispatch(f, match)
        if not d:
            continue
        ids = sorted(d)
        sel = [d[ids[-1]]] if pick == "last" else [d[i] for i in ids]
        for c in sel[0]:
            out[c] = sum(s.get(c, 0.0) for s in sel) / len(sel)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "r03final"))
    ap.add_argument("--tag", default="r03")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    tj, vj = os.path.join(prof, "pmc_traffic.json"), os.path.join(prof, "pmc_valu.json")
    traffic = json.load(open(tj)) if os.path.exists(tj) else {}
    valu = json.load(open(vj)) if os.path.exists(vj) else {}
    summary = {}
    plan = [("20", "k_step", "last", "C3_trendou_8192x8_fuse20", 8192 * 20),
            ("1", "k_step", "mean", "C3_trendou_8192x8_fuse1", 8192),
            ("256", "k_step", "mean", "C3_trendou_8192x8_fuse256", 8192 * 256),
            ("C2", "k_hist_gather", "mean", "C2_gather_4096x4_W64", 4096 * 64),
            ("C2", "k_step", "mean", "C2_step_4096x4_fuse64", 4096 * 64),
            ("C4", "k_hist_gather", "mean", "C4_gather_8192x8_W64", 8192 * 64),
            ("C4", "k_step", "mean", "C4_step_8192x8_fuse64", 8192 * 64),
            ("C5", "k_hist_gather", "mean", "C5_gather_8192x16_W64", 8192 * 64),
            ("C5", "k_step", "mean", "C5_step_8192x16_fuse64", 8192 * 64),
            ("a16", "k_step", "mean", "C3_trendou_8192x16_fuse64", 8192 * 64)]
    for tag, match, pick, key, units in plan:
        m = merged(a.src, tag, match, pick)
        if not m:
            continue
        s = {"counters_per_dispatch": m, "dispatches": pick, "kernel": match}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            s["hbm_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
            s["hbm_bytes_per_env_step"] = s["hbm_bytes_per_launch"] / units
            traffic[key] = s["hbm_bytes_per_launch"]
        if "SQ_INSTS_VALU" in m and m.get("SQ_WAVES"):
            valu[key] = m["SQ_INSTS_VALU"]
            steps = 64 if key.startswith("C2") else units // 8192
            s["valu_wave_insts_per_wave_step"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"] / steps
            s["wait_any_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        summary[key] = s
    for tag in ("20", "1", "256", "C2", "C4", "C5", "a16"):
        ks = os.path.join(a.src, f"kt{tag}", "kt_kernel_stats.csv")
        if os.path.exists(ks):
            shutil.copy(ks, os.path.join(prof, f"{a.tag}_kernel_stats_{tag}.csv"))
    for f in sorted(os.listdir(a.src)):
        if f.startswith("bench_") and f.endswith(".json"):
            shutil.copy(os.path.join(a.src, f), os.path.join(prof, f"{a.tag}_{f}"))
    lg = os.path.join(a.src, "pytest_gpu.log")
    if os.path.exists(lg):
        shutil.copy(lg, os.path.join(prof, f"{a.tag}_pytest_gpu.txt"))
    json.dump(traffic, open(tj, "w"), indent=1, sort_keys=True)
    json.dump(valu, open(vj, "w"), indent=1, sort_keys=True)
    json.dump(summary, open(os.path.join(prof, f"{a.tag}_pmc_summary.json"), "w"), indent=1)
    print(json.dumps({k: {kk: v for kk, v in s.items() if kk != "counters_per_dispatch"}
                      for k, s in summary.items()}, indent=1))


if __name__ == "__main__":
    main()
