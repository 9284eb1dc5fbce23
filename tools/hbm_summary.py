"""Summarise tools/gpu_hbm.sh (C3 at N beyond the Infinity Cache) into
profiles/<tag>_hbm_bound_c3.json: per N the bench line, the kernel-trace
average launch, and the PMC traffic (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per
launch (MI355X_MICROARCH.md gfx950 correction), mean of the last 8 launches.

    python tools/hbm_summary.py [--src gpurun_out/hbm] [--tag r02]
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, name):
    d = {}
    for r in csv.DictReader(open(path)):
        if "k_step" in r["Kernel_Name"] and r["Counter_Name"] == name:
            d[int(r["Dispatch_Id"])] = d.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    v = [d[i] for i in sorted(d)][-8:]
    return sum(v) / len(v), len(d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "hbm"))
    ap.add_argument("--tag", default="r02")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    out = {}
    for N in (262144, 524288):
        bj = os.path.join(a.src, f"bench_{N}.json")
        if not os.path.exists(bj):
            continue
        b = json.load(open(bj))
        f, nl = counters(os.path.join(a.src, f"pmc_{N}", "fetch", "p_counter_collection.csv"), "FETCH_SIZE")
        w, _ = counters(os.path.join(a.src, f"pmc_{N}", "write", "p_counter_collection.csv"), "WRITE_SIZE")
        tr = (2 * f + w) * 1024
        ks = [r for r in csv.DictReader(open(os.path.join(a.src, f"kt_{N}", "kt_kernel_stats.csv")))
              if "k_step" in r["Name"]][0]
        avg_ns = float(ks["AverageNs"])
        spl = b["config"]["steps_per_launch"]
        out[N] = dict(n_envs=N, steps_per_launch=spl, kernel=b["roofline"]["kernel"], launches_pmc=nl,
                      hbm_bytes_per_launch=tr, hbm_bytes_per_env_step=tr / (N * spl),
                      trace_avg_launch_us=avg_ns / 1e3, bench_avg_launch_us=b["roofline"]["avg_launch_us"],
                      counter_GBs=tr / (avg_ns * 1e-9) / 1e9, counter_frac_of_8TBs=tr / (avg_ns * 1e-9) / 8e12,
                      survey_bytes_GBs=b["roofline"]["achieved"], survey_bytes_frac=b["roofline"]["frac"],
                      value=b["value"])
        shutil.copy(bj, os.path.join(prof, f"{a.tag}_bench_c3_{N}.json"))
        shutil.copy(os.path.join(a.src, f"kt_{N}", "kt_kernel_stats.csv"),
                    os.path.join(prof, f"{a.tag}_kernel_stats_c3_{N}.csv"))
    json.dump(out, open(os.path.join(prof, f"{a.tag}_hbm_bound_c3.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
