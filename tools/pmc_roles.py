"""Per-role VALU / LDS / SALU wave-instructions of the three-role kernel from
the role-ablation builds (tools/_var/abl{G,L,F}: -DMGN_TRIO_ABL_{G,L,F}, the
role's work skipped, outputs wrong) against the product build, from the
rocprofv3 --pmc runs of tools/gpu_r04_roles.sh.

    python tools/pmc_roles.py gpurun_out/roles

Per variant: mean per dispatch of the k_step_trio launches, per wave and step
(SQ_WAVES counts every wave of the three roles).  base - ablX estimates role
X's own instructions (per wave of the whole kernel; x3 per wave of the role)."""
import csv
import glob
import json
import os
import sys


def load(path):
    d = {}
    for r in csv.DictReader(open(path)):
        if "k_step_trio" not in r["Kernel_Name"]:
            continue
        c = d.setdefault(int(r["Dispatch_Id"]), {})
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return d


def main():
    src = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    res = {}
    for f in sorted(glob.glob(os.path.join(src, "*", "p_counter_collection.csv"))):
        name = os.path.basename(os.path.dirname(f))
        d = load(f)
        # the timed launches: every dispatch of the full launch length (the
        # last ones); per wave and step
        ids = sorted(d)[-4:]
        rows = [d[i] for i in ids]
        waves = sum(r.get("SQ_WAVES", 0) for r in rows) / len(rows)
        out = {"waves": waves}
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            v = sum(r.get(c, 0) for r in rows) / len(rows)
            out[c + "_per_wave_step"] = v / waves / steps if waves else None
        res[name] = out
    if "base" in res:
        b = res["base"]
        for r in ("G", "L", "F"):
            k = "abl" + r
            if k in res:
                res[k]["role_valu_per_role_wave_step"] = 3 * (b["SQ_INSTS_VALU_per_wave_step"] -
                                                              res[k]["SQ_INSTS_VALU_per_wave_step"])
                res[k]["role_lds_per_role_wave_step"] = 3 * (b["SQ_INSTS_LDS_per_wave_step"] -
                                                             res[k]["SQ_INSTS_LDS_per_wave_step"])
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
