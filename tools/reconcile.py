"""Reconcile a bench.py line with a rocprofv3 kernel trace of the same command.

    python bench.py ARGS > line.json                      # the un-profiled line
    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o kt -- python3 bench.py ARGS > kt.json
    python tools/reconcile.py line.json DIR [--trace-line kt.json] [--out profiles/rNN_reconcile.json]

The line's `launch_log` lists every step-kernel launch in issue order (label,
steps per launch, launches); the trace's step-kernel dispatches, sorted by
start time, are assigned to those entries in that order (the traced run's
log, --trace-line, must hold the same entries).  For each figure the line
reports from the launches' own HIP events -- the timed region's launch
(roofline.avg_launch_us), the episode-age launches (episode_age, the steady
state among them), the launch-length sweep (launch_lengths) -- the trace's
mean and median over the same dispatches and their ratio to the line's
figure.  (Under the profiler the launch events themselves read longer -- about
4 us per launch on this box -- so the line to compare is the un-profiled one;
the traced run's own figures are reported beside it as `profiled_line_us`.)
"""
import csv
import glob
import json
import os
import statistics
import sys


def dispatches(d):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            rows += [r for r in csv.DictReader(f) if "k_step" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"]) for r in rows]


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    tline = line
    if "--trace-line" in sys.argv:
        tline = json.loads(open(sys.argv[sys.argv.index("--trace-line") + 1]).read().strip().splitlines()[-1])
        if [e[:2] for e in tline["launch_log"]] != [e[:2] for e in line["launch_log"]]:
            sys.exit("the traced run's launch log differs from the line's")
    disp = dispatches(sys.argv[2])
    log = tline["launch_log"]
    need = sum(n for _, _, n in log)
    if len(disp) != need:
        sys.exit(f"trace holds {len(disp)} step dispatches, the launch log {need}")
    groups, i = {}, 0
    for label, K, n in log:
        g = groups.setdefault(label, {"steps_per_launch": K, "us": []})
        g["us"] += [u for u, _ in disp[i:i + n]]
        i += n
    res = {"line": sys.argv[1], "trace": sys.argv[2], "figures": {}}

    def fig(name, label, get):
        us = groups[label]["us"]
        mean, med = statistics.fmean(us), statistics.median(us)
        line_us = get(line)
        res["figures"][name] = {"launches": len(us), "steps_per_launch": groups[label]["steps_per_launch"],
                                "line_us": line_us, "trace_mean_us": mean, "trace_median_us": med,
                                "trace_over_line": mean / line_us, "profiled_line_us": get(tline)}

    # the line's kernel figure comes from the launches after the timed region
    # ("probe", the timed plan repeated with launch events; older lines timed
    # the timed launches themselves)
    kl = "probe" if "probe" in groups else "timed"
    fig("timed_region_launch", kl, lambda d: d["roofline"]["avg_launch_us"])
    if kl == "probe":
        us = groups["timed"]["us"]
        res["figures_trace_only"] = {"timed_launches_trace_mean_us": statistics.fmean(us),
                                     "note": "the timed region's own launches (no events) in the trace"}
    for age in line.get("episode_age", {}):
        key = age if age in tline.get("episode_age", {}) else None
        if key:
            fig(f"episode_age_{age}", f"age_{age}", lambda d, a=age: d["episode_age"][a]["kernel_us_per_launch"])
    for K in line.get("launch_lengths", {}):
        fig(f"launch_length_{K}", f"sweep_{K}", lambda d, k=K: d["launch_lengths"][k]["kernel_us_per_launch"])
    res["within_3pct"] = all(abs(f["trace_over_line"] - 1) <= 0.03 for f in res["figures"].values())
    res["kernels"] = sorted({k for _, k in disp})
    out = json.dumps(res, indent=1)
    if "--out" in sys.argv:
        open(sys.argv[sys.argv.index("--out") + 1], "w").write(out + "\n")
    for n, f in res["figures"].items():
        print(f"{n:28s} n={f['launches']:4d} line {f['line_us']:9.2f} us  trace mean {f['trace_mean_us']:9.2f} "
              f"med {f['trace_median_us']:9.2f}  ratio {f['trace_over_line']:.4f}")
    print("within 3 %:", res["within_3pct"])


if __name__ == "__main__":
    main()
