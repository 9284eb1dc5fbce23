"""Summarise tools/pmc_pass.sh: per library, the mean over the probe's
measured step-kernel dispatches (the last REPS), per wave and step.

    python tools/pmc_brief.py gpurun_out/pmc_TAG [--json out.json]

SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* count quad-cycles
(MI355X_MICROARCH.md); they are reported x4 as cycles.  The effective clock
is GRBM_GUI_ACTIVE / 8 (the sum over the XCDs) / the dispatch's duration when
the CSV carries its timestamps.  For role-ablation libraries (name ablG /
ablL / ablF) the role's own VALU per role-wave-step is estimated as
3 x (base - ablX) per wave-step (a third of the waves hold each role)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def probe_cfg(d, name):
    for f in sorted(glob.glob(os.path.join(d, f"{name}_g*.log"))):
        for line in open(f):
            if line.startswith("{") and '"fuse"' in line:
                return json.loads(line)
    return {}


def dispatches(gdir):
    rows = defaultdict(dict)
    ts = {}
    for f in glob.glob(os.path.join(gdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if os.environ.get("PMC_KERNEL", "k_step") not in r.get("Kernel_Name", ""):
                continue
            i = int(r["Dispatch_Id"])
            c = rows[i]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if "Start_Timestamp" in r and r["Start_Timestamp"]:
                ts[i] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return rows, ts


def main():
    d = sys.argv[1]
    res = {}
    for vdir in sorted(glob.glob(os.path.join(d, "*", ""))):
        name = os.path.basename(os.path.dirname(vdir))
        cfg = probe_cfg(d, name)
        reps, fuse = cfg.get("reps", 8), cfg.get("fuse", 20)
        acc = {}
        dur = []
        for gdir in sorted(glob.glob(os.path.join(vdir, "g*"))):
            rows, ts = dispatches(gdir)
            ids = sorted(rows)[-reps:]
            for i in ids:
                for k, v in rows[i].items():
                    acc.setdefault(k, []).append(v)
                if i in ts:
                    dur.append(ts[i])
        m = {k: sum(v) / len(v) for k, v in acc.items()}
        waves = m.get("SQ_WAVES")
        out = {"config": cfg}
        if waves:
            per = lambda k: m[k] / waves / fuse if k in m else None  # noqa: E731
            out.update({
                "valu_per_wave_step": per("SQ_INSTS_VALU"),
                "salu_per_wave_step": per("SQ_INSTS_SALU"),
                "lds_per_wave_step": per("SQ_INSTS_LDS"),
                "vmem_wr_per_wave_step": per("SQ_INSTS_VMEM_WR"),
                "vmem_rd_per_wave_step": per("SQ_INSTS_VMEM_RD"),
                "wave_cycles_per_wave_step": 4 * per("SQ_WAVE_CYCLES") if "SQ_WAVE_CYCLES" in m else None,
                "valu_active_cycles_per_wave_step": 4 * per("SQ_ACTIVE_INST_VALU") if "SQ_ACTIVE_INST_VALU" in m else None,
                "any_active_cycles_per_wave_step": 4 * per("SQ_ACTIVE_INST_ANY") if "SQ_ACTIVE_INST_ANY" in m else None,
                "wait_inst_any_frac": m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]
                if "SQ_WAIT_INST_ANY" in m and "SQ_WAVE_CYCLES" in m else None,
                "wait_any_frac": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
                if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m else None,
            })
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            # gfx950: FETCH_SIZE reports half the bytes of a wide streaming read
            # (MI355X_MICROARCH.md, HBM): doubled; WRITE_SIZE exact; kilobytes
            out["hbm_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
            out["fetch_kb_raw"] = m["FETCH_SIZE"]
            out["write_kb"] = m["WRITE_SIZE"]
        if "SQ_INSTS_VALU" in m:
            out["valu_wave_insts_per_launch"] = m["SQ_INSTS_VALU"]
        if dur:
            out["dispatch_us"] = 1e6 * sum(dur) / len(dur)
            if "GRBM_GUI_ACTIVE" in m:
                out["clock_GHz"] = m["GRBM_GUI_ACTIVE"] / 8 / (sum(dur) / len(dur)) / 1e9
        out["raw_mean"] = m
        res[name] = out
    base = res.get("base")
    if base and base.get("valu_per_wave_step"):
        for n, r in res.items():
            mm = re.match(r"abl([GLF])$", n)
            if mm and r.get("valu_per_wave_step") is not None:
                r["role_valu_per_role_wave_step"] = 3 * (base["valu_per_wave_step"] - r["valu_per_wave_step"])
                r["role_salu_per_role_wave_step"] = 3 * (base["salu_per_wave_step"] - r["salu_per_wave_step"])
    for n, r in res.items():
        brief = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items() if k not in ("raw_mean", "config")}
        print(n, json.dumps(brief))
    if "--json" in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    if "--update" in sys.argv:
        # the bench's lookups (bench.load_pmc_traffic / valu_issue): per workload
        # key (the library name of the pass), per launch
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        for fname, field in (("pmc_traffic.json", "hbm_bytes_per_launch"),
                             ("pmc_valu.json", "valu_wave_insts_per_launch")):
            path = os.path.join(root, "profiles", fname)
            d = json.load(open(path)) if os.path.exists(path) else {}
            for n, r in res.items():
                if r.get(field) and re.match(r"(C\d|R1)_", n):
                    d[n] = r[field]
            json.dump(d, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
