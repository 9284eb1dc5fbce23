"""One-line summary of a bench.py JSON line (tools/gpu_pass.sh)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
out = [f"{d['value']:.4g} {d['unit']}", f"ms/step {d['ms_per_step']:.5f}"]
if "avg_launch_us" in r:
    out.append(f"launch {r['avg_launch_us']:.2f} us frac {r.get('frac', 0):.4f}")
if "step_launch_avg_us" in d:
    out.append(f"step launch {d['step_launch_avg_us']:.1f} us")
if "steady_state" in d:
    s = d["steady_state"]
    out.append(f"steady {s['kernel_us_per_launch']:.2f} us ({s['kernel_us_per_step']:.3f}/step, ep {s['episodes_completed']})")
if "episode_age" in d:
    out.append("ages " + " ".join(f"{k}:{v['kernel_us_per_step']:.3f}" for k, v in d["episode_age"].items()))
if "launch_lengths" in d:
    out.append("K " + " ".join(f"{k}:{v['kernel_us_per_launch']:.2f}/{v['back_to_back_us_per_step']:.3f}"
                               for k, v in d["launch_lengths"].items()))
if "view_mode" in d:
    out.append(f"view {d['view_mode']['value']:.4g}")
if "cpu_baseline" in d:
    out.append(f"cpu {d['cpu_baseline']['value']:.3g}")
print(sys.argv[1].rsplit("/", 1)[-1], " | ".join(out))
