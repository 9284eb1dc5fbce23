"""Print the numbers DESIGN section 5 quotes from one evidence pass.

    python tools/evidence_summary.py gpurun_out/r03final4

Bench lines (value, launch us, frac, schedules, view mode), rocprof kernel
averages / minima and the PMC summary (tools/pmc_r03.py's computation).
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_r03 as P  # noqa: E402


def main():
    src = sys.argv[1]
    for f in ("bench_driver", "bench_fuse256", "bench_nstep20", "bench_a16", "bench_C1", "bench_C2",
              "bench_C4", "bench_C5"):
        path = os.path.join(src, f + ".json")
        if not os.path.exists(path):
            continue
        d = json.load(open(path))
        r = d.get("roofline") or {}
        print(f, "%.4g" % d["value"], "launch_us", r.get("avg_launch_us"), "frac", r.get("frac"),
              "of_copy", r.get("frac_of_attainable"), "kus/step", d.get("kernel_us_per_step"),
              "step_launch", d.get("step_launch_avg_us"), "view", (d.get("view_mode") or {}).get("value"),
              "sched", (d.get("config") or {}).get("schedule"), "eps", d.get("episodes_completed"),
              "cpu", (d.get("cpu_baseline") or {}).get("value"))
    for t in ("20", "1", "256", "C2", "C4", "C5"):
        ks = os.path.join(src, f"kt{t}", "kt_kernel_stats.csv")
        if os.path.exists(ks):
            for r in csv.DictReader(open(ks)):
                if "k_step" in r["Name"] or "gather" in r["Name"]:
                    print("kt", t, r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2),
                          round(float(r["MinNs"]) / 1e3, 2), round(float(r["MaxNs"]) / 1e3, 2))
    for tag, units in (("20", 8192 * 20), ("256", 8192 * 256), ("1", 8192)):
        m = P.merged(src, tag, "k_step", "last" if tag == "20" else "mean")
        if m:
            print("pmc", tag, "valu/wave-step", round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"] / (units // 8192), 1),
                  "wait", round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3), "B/env-step",
                  round((2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024 / units, 1))


if __name__ == "__main__":
    main()
