"""Benchmark: batched madigan market-simulation step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--fuse F] [--n-envs 8192]
                    [--workload C3|C2|C4|C5]

Workload (BASELINE.json configs[2], SURVEY 8d "C3"): 8192 envs x 8 assets per
GPU, TrendOU generators (config.yaml:116-138), Broker with 1e-4 relative
slippage and 2% transaction cost, DDR reward (eta=.001, n=1), discrete actions
U{0,1,2} (Philox, pre-generated on device) turned into units by DQN's
action_to_transaction (unit_size .05 of available margin), in-kernel
auto-reset.  A "step" advances every env by one tick and materialises every
per-step output of the reference's Env.step (State row, reward, done,
BrokerResponse) plus the shaped reward; `--fuse` (256) steps run per launch
with the state held in registers (every step's outputs are written to a
(K, N, ...) trajectory).

For N>1 (torchrun, one process per GPU) envs are sharded by global index
(env_offset) with no per-step collective; one RCCL all-gather of the
per-env episode statistics closes the timed region.  Prints one JSON line.

The other BASELINE.json configs are selectable with --workload;
they carry a W = 64 sliding window, so a step there is one Env step plus
StackerDiscrete.current_data of every env, as the agent reads one window per
step: `--win-fuse` (64) steps per launch append every ring push to a launch
history, and a second kernel writes all K windows (mgn_rollout_hist /
mgn_window_hist):
  C2  4096 envs x 4 OU (mu 10, theta .08, phi .04), 2% cost, DSR, norm none
  C4  8192 envs/GPU x 8 Composite (Synth 2 + OU 3 + TrendOU 3), 2% cost,
      PPC (target [1,0..0], alpha .01) over the env log reward, norm log
  C5  8192 envs/GPU x 16 HDF replay (synthetic OU paths written to an HDF5
      file in the HDFSourceSingle layout generalised to (T, 16), staged to HBM
      once, per-env start stride), 2% cost, DDR, norm none
  R1  the reference's own experiment shape (scripts/ou_ddr_.001_nstep20.yaml):
      --n-envs envs x 1 OU (mu 10, theta .08, phi .04), W = 64 (norm false:
      raw prices), n = 20 step returns (discount .99) of the summed agent
      reward, DDR eta .001 (--shaper sortino_shaperB: sortino_exp 1.1), 2% cost
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (batched) at 8192 envs × 8 assets; % HBM roofline"
TRENDOU_P = [0.001, 100, 500, 0.001, 0.005, 5.0, 0.15, 0.04, 0.001, 0.99]  # config.yaml:116-138
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
GUIDE_COPY_GBS = 6290.0  # MI355X_MICROARCH.md: 6.29 TB/s measured (float4 copy)


def c3_kwargs():
    return dict(required_margin=1.0, maintenance_margin=0.25, slippage_rel=1e-4,
                transaction_cost_rel=0.02, reward_shaper="DDR", adaptation_rate=0.001,
                unit_size=0.05, auto_reset=True, init_cash=1_000_000.0)


def bytes_per_env_step(A: int, fuse: int, D: int = 1, agent_reward: bool = False) -> float:
    """Algorithmic HBM bytes of the fused step kernel per env-step.

    per step: actions A*1 B read; outputs reward 8, shaped 8*D (+ agent_reward 8*D when
    requested; the C3 workload feeds the env log reward to DDR and does not),
    done 1, obs_price 8A, obs_port 8(A+1), timestamp 8, tprice/tunits/tcost 24A,
    risk A, marginCall 1.  Per launch (amortised over `fuse` steps): state read +
    write of L, meanEntry, borrowed, price, sine_x, ouMean, dY (7*8A), trend len
    4A + flags A, cash 8, timestamp 8, shaper A/B 16*D, running stats 16, plus
    the episode-stat counter read 8 and the stats row write 32."""
    per_step = A + 8 + 8 * D * (2 if agent_reward else 1) + 1 + 8 * A + 8 * (A + 1) + 8 + 24 * A + A + 1
    state = 2 * (7 * 8 * A + 4 * A + A + 8 + 8 + 16 * D + 16) + 8 + 32
    return per_step + state / fuse


def survey_bytes_per_env_step(env) -> float:
    """SURVEY 8d's algorithmic bytes per env-step: per asset 113 (ledger,
    meanEntry, borrowed, price read + write 64; action 8; broker response 25;
    observation row + ledgerNormedFull entry 16) plus the generator's state
    (OU 0, Sine 16, TrendOU 48), per env 105 (cash r/w 16, DSR/DDR A,B 32,
    reward 8, done 1, ledgerNormedFull cash entry 8, timestamp r/w 16, episode
    stats 24).  C3: 8 x (113 + 48) + 105 = 1393."""
    from madigan_amd import _lib as L
    extra = {L.SRC_OU: 0, L.SRC_SINE: 16, L.SRC_TRENDOU: 48}
    return float(sum(113 + extra.get(k, 48) for k in env.spec.kinds) + 105)


def load_pmc_traffic(workload: str):
    """(HBM bytes per launch, key) from the committed rocprofv3 PMC summary:
    the workload's own entry, else the entry with the nearest steps per launch
    of the same shape (its key says which)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if workload in d:
        return d[workload], workload
    stem, _, k = workload.rpartition("_fuse")
    cands = [(abs(int(key.rpartition("_fuse")[2]) - int(k)), key) for key in d
             if key.startswith(stem + "_fuse") and key.rpartition("_fuse")[2].isdigit()]
    if not cands or not k.isdigit():
        return None, None
    key = min(cands)[1]
    return d[key], key


def bandwidth_probe(dev, nbytes: int = 2 << 30, reps: int = 10):
    """Attainable HBM bandwidth on this box: the library's
    16-B-per-lane copy kernel over two 1 GiB buffers; (read + write) GB/s."""
    import ctypes as C
    import torch
    from madigan_amd import _lib as L
    lib = L.load()
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev).fill_(1)
    dst = torch.empty_like(src)
    out = C.c_double()
    L.check(lib.mgn_bandwidth_probe(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), nbytes,
                                    reps, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream),
                                    C.byref(out)))
    del src, dst
    return out.value


SCHED_NAMES = {1: "single", 2: "duo", 3: "trio"}

# MI355X: 256 CUs x 4 SIMDs; a wave64 VALU instruction occupies its SIMD for
# at least 4 cycles (16 lanes per cycle; fp64 FMA at full rate, transcendental
# and fp64 divide / sqrt steps longer); peak engine clock 2.4 GHz
N_SIMD = 1024
SIMD_CYCLES_PER_VALU = 4
CLOCK_HZ = 2.4e9


def valu_issue(workload: str, launch_s: float):
    """The step kernel's VALU issue against the SIMDs' capacity, from the
    committed rocprofv3 PMC SQ_INSTS_VALU per launch (profiles/pmc_valu.json):
    a lower bound on the fraction of SIMD cycles spent issuing VALU work (the
    bound that limits this kernel; the HBM roofline above is far from it)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_valu.json")) as f:
            n = json.load(f).get(workload)
    except (OSError, ValueError):
        n = None
    if not n:
        return None
    busy = n * SIMD_CYCLES_PER_VALU / N_SIMD / (launch_s * CLOCK_HZ)
    return {"valu_wave_insts_per_launch": n, "simd_cycles_per_launch": launch_s * CLOCK_HZ,
            "valu_busy_frac_lower_bound": busy,
            "note": "SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x launch cycles at 2.4 GHz)"}


def host_threads() -> int:
    """The host-core share this process may use: OMP_NUM_THREADS where set (16
    on the GPU box, whose `nproc` shows the whole machine's CPUs, many times
    this process's share), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def host_cpu_info() -> dict:
    """The box's CPU counts beside the threads the baseline used (SURVEY 8d:
    the core count stated)."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}
    try:
        with open("/proc/cpuinfo") as f:
            names = [ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")]
        if names:
            info["model"] = names[0]
    except OSError:
        pass
    return info


def cpu_baseline(n_envs: int, A: int, budget_s: float = 12.0):
    """The oracle's C restatement (fast-math build, the reference's flags), one
    Env object per env, same C3 workload, bounded samples: all host cores
    (OpenMP over envs; the reported value) and one core."""
    from oracle import oracle as O
    cfg = dict(n_envs=n_envs, seed=0x6D6164 + 3, transaction_cost_rel=0.02, **{
        k: v for k, v in c3_kwargs().items() if k not in ("transaction_cost_rel", "auto_reset")})
    cfg["auto_reset"] = 1
    srcs = [(O.SRC_TRENDOU, TRENDOU_P)] * A
    b = O.OracleBatch(cfg, srcs, fast=True)
    rng = np.random.default_rng(0)
    chunk = 4
    acts = rng.integers(0, 3, (chunk, n_envs, A)).astype(np.int8)
    b.rollout(acts[:1])  # warm

    def timed(threads, budget):
        steps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget:
            b.rollout(acts, threads=threads)
            steps += chunk
        dt = time.perf_counter() - t0
        return n_envs * steps / dt, steps, dt

    T = host_threads()
    T_all = len(os.sched_getaffinity(0))
    parts = 3 if T_all > T else 2
    v1, s1, d1 = timed(1, budget_s / parts)
    vT, sT, dT = timed(T, budget_s / parts) if T > 1 else (v1, s1, d1)
    out = dict(value=vT, unit="env-steps/s", cores=T, kind="port",
               single_core=v1, host=host_cpu_info(),
               sample=f"C3 workload, {n_envs} envs x {A} assets: {sT} steps on {T} host threads "
                      f"(OpenMP over envs, {dT:.1f} s) and {s1} steps on one core ({d1:.1f} s); "
                      f"oracle/madigan_oracle.c built -O3 -march=x86-64-v3 -ffast-math")
    if T_all > T:
        # every host core the process may run on (the affinity set;
        # on a shared box the threads beyond its share contend with others)
        vA, sA, dA = timed(T_all, budget_s / parts)
        out["all_cores"] = {"value": vA, "threads": T_all,
                            "sample": f"{sA} steps on {T_all} threads (the affinity set), {dA:.1f} s"}
    return out


def composite_spec():
    """C4: Synth(2, DataSource.cpp:477-480 first two) + OU(3) + TrendOU(3)."""
    from madigan_amd.config import SourceSpec, ou_spec, synth_spec, trendou_spec
    s = SourceSpec()
    s.extend(synth_spec([1., 0.3], [2., 2.1], [1., 1.2], [0., 1.], 0.01, 0.0))
    s.extend(ou_spec([10.0] * 3, [0.15] * 3, [0.04] * 3))
    s.extend(trendou_spec(*[[p] * 3 for p in TRENDOU_P]))
    return s


def c5_paths(A: int, T: int):
    """Synthetic OU paths (mu 10, theta .08, phi .04, as C2): price (T, A)
    and 1-minute-bar timestamps (T,)."""
    from scipy.signal import lfilter
    rng = np.random.default_rng(0x6D6164 + 5)
    mu, th, phi = 10.0, 0.08, 0.04
    z = rng.standard_normal((T, A))
    # x_t = (1 - theta) x_{t-1} + theta mu + mu phi z_t, x_0 = mu
    x = lfilter([1.0], [1.0, -(1.0 - th)], th * mu + mu * phi * z, axis=0,
                zi=np.full((1, A), (1.0 - th) * mu))[0]
    ts = (np.arange(T, dtype=np.uint64) + np.uint64(27_000_000)) * np.uint64(60_000_000_000)
    return x, ts


def c5_replay_file(A: int, T: int, path: str) -> None:
    """c5_paths in the replay layout: price (T, A), features = prices."""
    from madigan_amd import write_hdf
    x, ts = c5_paths(A, T)
    write_hdf(path, "synth/ou", [f"OU_{i}" for i in range(A)], x, x, ts,
              price_key="price", feature_key="features", timestamp_key="timestamps")


def workload_env(name, N, A, rank, dev, **extra):
    """(BatchedEnv, description, window) for a --workload (extra: C3 overrides,
    e.g. nstep_return for the n-step diagnostic lines)."""
    from madigan_amd import BatchedEnv
    from madigan_amd.config import ou_spec, spec_from_config, trendou_spec
    seed = 0x6D6164 + int(name[1])
    off = rank * N
    if name == "C3":
        spec = trendou_spec(*[[p] * A for p in TRENDOU_P])
        return (BatchedEnv(spec, N, device=dev, seed=seed, env_offset=off, **{**c3_kwargs(), **extra}),
                "C3: TrendOU x8 assets per env, slippage 1e-4 + 2% cost broker, DDR eta=.001 n=1, "
                "discrete actions via action_to_transaction, auto-reset", 0)
    base = dict(required_margin=1.0, maintenance_margin=0.25, transaction_cost_rel=0.02,
                unit_size=0.05, auto_reset=True, init_cash=1_000_000.0, window=64,
                adaptation_rate=0.001)
    if name == "C2":
        spec = ou_spec([10.0] * A, [0.08] * A, [0.04] * A)
        return (BatchedEnv(spec, N, device=dev, seed=seed, env_offset=off, reward_shaper="DSR",
                           **base),
                f"C2: OU x{A} (mu 10, theta .08, phi .04), 2% cost, DSR eta=.001, W=64 window "
                "(norm none) gathered every step, auto-reset", 64)
    if name == "C4":
        spec = composite_spec()
        return (BatchedEnv(spec, N, device=dev, seed=seed, env_offset=off, reward_shaper="PPC",
                           cosine_temp=0.01, desired_portfolio=[1.0] + [0.0] * spec.n_assets,
                           norm_type="log", **base),
                "C4: Composite Synth(2)+OU(3)+TrendOU(3), 2% cost, PPC alpha=.01 target [1,0..0] "
                "over the env log reward, W=64 window (norm log) gathered every step, auto-reset", 64)
    if name == "R1":
        shaper = extra.pop("shaper", "DDR")
        sx = {"sortino_exp": 1.1} if shaper.startswith("sortino") else {}
        spec = ou_spec([10.0], [0.08], [0.04])
        pop = extra.pop("nstep_pop", "exact")
        return (BatchedEnv(spec, N, device=dev, seed=seed, env_offset=off, reward_shaper=shaper,
                           nstep_return=20, discount=0.99, reward_mode="agent_sum", nstep_pop=pop, **sx, **base),
                f"R1: OU x1 (mu 10, theta .08, phi .04), W=64 window (norm none), n=20 returns "
                f"(discount .99, {pop} pop) of the summed agent reward, {shaper} eta=.001{' exp 1.1' if sx else ''}, "
                "2% cost, unit .05 avM, auto-reset (scripts/ou_ddr_.001_nstep20.yaml)", 64)
    if name == "C5":
        import tempfile
        T = 200_000
        path = os.path.join(tempfile.gettempdir(), f"madigan_c5_{A}x{T}_r{rank}.h5")
        if not os.path.exists(path):
            c5_replay_file(A, T, path)
        cfg = {"data_source_type": "HDFSourceSingle",
               "data_source_config": {"filepath": path, "group_key": "synth/ou",
                                      "price_key": "price", "feature_key": "features",
                                      "timestamp_key": "timestamps", "cache_size": 10_000}}
        t0 = time.perf_counter()
        env = BatchedEnv(spec_from_config(cfg), N, device=dev, seed=seed, env_offset=off,
                         reward_shaper="DDR", replay_stride=997, **base)
        import torch
        torch.cuda.synchronize()
        env._stage_s = time.perf_counter() - t0
        return (env, f"C5: HDF replay x{A} (synthetic OU paths, {T} rows, HDFSourceSingle layout "
                     f"(T,{A}), cache_size 10000, staged to HBM once by pinned double-buffered H2D, "
                     "env start stride 997 rows), 2% cost, DDR eta=.001, W=64 window (norm none) "
                     "gathered every step, auto-reset", 64)
    raise SystemExit(f"unknown workload {name}")


def gather_bytes(env, K: int) -> float:
    """Algorithmic bytes of one k_hist_gather launch (K windows per env): write
    every step's window, W*(F+A+2)*8 per env-step (price, portfolio,
    timestamps), and read each history row once, (W + K)*(F+A+2)*8 per env
    (the window before the launch plus one row per step; reset refill rows,
    which add to it, are not counted).  The kernel re-reads the rows that
    consecutive windows share; those re-reads are not algorithmic bytes."""
    C1 = env.F + env.A + 2
    return env.N * 8.0 * C1 * (K * env.W + env.W + K)


def kernel_name(env, A: int) -> str:
    """The step kernel as rocprofv3 names it: the two-role k_step_duo where the
    handle's schedule picked it (mgn_get_schedule), else k_step<M, S, RQ1, NST>."""
    from madigan_amd import _lib as L
    m = int(env.lib.mgn_get_layout(env.h))
    apad = 1 << max(0, (A - 1).bit_length())
    rq1 = "true" if env.cfg.required_margin == 1.0 else "false"
    if int(env.lib.mgn_get_schedule(env.h)) == L.SCHED_TRIO:
        return f"mgn::k_step_trio<{apad}, {rq1}, true>"
    if int(env.lib.mgn_get_schedule(env.h)) == L.SCHED_DUO:
        # <S, RQ1, ABL, DISC, RP, NST>: the bench launches discrete actions
        rp = "true" if env.spec.replay else "false"
        nst = "true" if env.nstep > 1 else "false"
        return f"mgn::k_step_duo<{apad}, {rq1}, false, true, {rp}, {nst}>"
    nst = "true" if env.nstep > 1 else "false"
    return f"mgn::k_step<{m}, {apad // m}, {rq1}, {nst}>"


def free_port() -> int:
    """A free TCP port on 127.0.0.1 for the ranks' rendezvous."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def gather_stats(D, env, n_total):
    """The episode-statistics all-gather after the timed region: the C ABI's
    mgn_stats_allgather on RCCL where torch's nccl group exposes its
    communicator, else torch's all-gather (the path is recorded in the line);
    an all-gather that fails does not lose the measured line -- it is
    recorded instead, with this rank's own rows."""
    try:
        return D.allgather_env_stats(env, n_total=n_total), D.last_allgather_path
    except D.CollectiveUnavailable as e:
        try:
            g = D.allgather_env_stats(env, n_total=n_total, allow_torch_fallback=True)
            return g, f"{D.last_allgather_path} (no RCCL communicator: {e})"
        except Exception as e2:  # noqa: BLE001
            return env.episode_stats, f"failed: {type(e2).__name__}: {e2}"
    except Exception as e:  # noqa: BLE001
        return env.episode_stats, f"failed: {type(e).__name__}: {e}"


def spawn_ranks(n: int, argv, backend: str) -> int:
    """`bench.py --gpus N` without a launcher: start N child ranks of this
    script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR 127.0.0.1 /
    MASTER_PORT in their environment, one process per GPU), and wait.  This
    process never touches the GPU (no HIP call: it only counts devices, which
    does not initialise the runtime on this image) and never execs; rank 0
    prints the JSON line on the inherited stdout.  When a rank fails, the
    others are ended (by their own PIDs: the survivors would wait in a
    collective) and the worst exit status is returned."""
    if backend == "nccl":
        import torch  # device count only (no runtime initialisation)
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py --gpus {n}: {have} GPU(s) visible; one rank per GPU needs {n} "
                  "(--dist-backend gloo lets ranks share a GPU)", file=sys.stderr)
            return 2
    port = free_port()
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = []
    every_rank = "--rank-probe" in argv  # (the test hook: every rank reports)
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 or every_rank else subprocess.DEVNULL))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [abs(rc) for rc in rcs if rc]
    return max(bad) if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without a launcher's WORLD_SIZE, N > 1 starts "
                         "N child ranks of this script itself (spawn_ranks)")
    ap.add_argument("--rank-probe", action="store_true",
                    help="test hook: each rank prints its rank / world as JSON and exits before any "
                         "GPU call")
    ap.add_argument("--steps", type=int, default=2048)
    ap.add_argument("--warmup", type=int, default=256)
    ap.add_argument("--fuse", type=int, default=256)
    ap.add_argument("--win-fuse", type=int, default=64,
                    help="steps per launch of the windowed workloads (capped by --fuse)")
    ap.add_argument("--win-assets", type=int, default=0,
                    help="C2 only (diagnostic): OU assets per env, at --n-envs envs")
    ap.add_argument("--win-overlap", action="store_true",
                    help="windowed workloads: gather on a second stream beside the next step launch")
    ap.add_argument("--n-envs", type=int, default=8192, help="envs per GPU")
    ap.add_argument("--assets", type=int, default=8)
    ap.add_argument("--layout", type=int, default=0, help="assets per lane (0 = auto)")
    ap.add_argument("--schedule", default="auto", choices=["auto", "single", "duo", "trio"],
                    help="C3 diagnostics: pin the step kernel (results are bit-identical)")
    ap.add_argument("--nstep", type=int, default=1,
                    help="C3 diagnostics: n-step aggregation (nstep_return), not the headline")
    ap.add_argument("--nstep-pop", default="exact", choices=["exact", "running"],
                    help="n-step lines (C3 --nstep > 1, R1): the exact pop or the running-sum pop "
                         "(MGN_NSTEP_POP_RUNNING, within 1e-6 of the exact pop)")
    ap.add_argument("--k1-hist", dest="k1_ring", action="store_false",
                    help="windowed workloads at --win-fuse 1: the launch-history path (mgn_rollout_hist + "
                         "mgn_window_hist) instead of mgn_rollout + mgn_window")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-k-sweep", dest="k_sweep", action="store_false",
                    help="skip the K = 1 / 16 / 256 launch-length block of the line")
    ap.add_argument("--sweep", action="store_true",
                    help="also time 1/16/64/256 steps per launch (separate launches; keep it off "
                         "when profiling, so the kernel's rocprof average is the headline's)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--workload", default="C3", choices=["C1", "C2", "C3", "C4", "C5", "R1"])
    ap.add_argument("--shaper", default="DDR", help="R1: DDR or sortino_shaperB")
    ap.add_argument("--dump-stats", default=None,
                    help="rank 0 saves the gathered (n_total, 4) episode statistics (.npy)")
    ap.add_argument("--no-probe", dest="probe", action="store_false",
                    help="skip the attainable-bandwidth copy probe")
    ap.add_argument("--timing", default="launch", choices=["launch", "marker"],
                    help="kernel duration events: recorded by the step launch itself "
                         "(hipExtLaunchKernel, the kernel's begin / end) or marker events around it")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: nccl (RCCL; the statistics all-gather is the C ABI's "
                         "mgn_stats_allgather) or gloo (several ranks may share one GPU)")
    ap.add_argument("--wait", default="stream", choices=["stream", "spin"],
                    help="the timed region's closing wait on the handle's stream: "
                         "hipStreamSynchronize or polling hipStreamQuery (mgn_synchronize_spin)")
    ap.add_argument("--sched-spin", action="store_true",
                    help="diagnostic: hipSetDeviceFlags(hipDeviceScheduleSpin) before the device is used "
                         "(the host waits by spinning)")
    args = ap.parse_args()

    # ranks: a launcher (torch.distributed.run) sets WORLD_SIZE; without one,
    # --gpus N > 1 starts the N ranks here, before anything touches the GPU
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], args.dist_backend))
    if world_env is not None and int(world_env) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks")
    if args.rank_probe:
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": int(world_env or 1),
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}),
              flush=True)
        return

    import torch
    import torch.distributed as dist
    if args.sched_spin:
        # (the runtime torch loaded -- by its soname -- before the device is used)
        import ctypes
        ctypes.CDLL("libamdhip64.so.7").hipSetDeviceFlags(1)  # hipDeviceScheduleSpin

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.dist_backend == "gloo":
        # gloo rehearsal of the sharded path: ranks may share one GPU
        dist.init_process_group("gloo")
        local_rank = local_rank % max(1, torch.cuda.device_count())
    elif world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    dev = torch.device(f"cuda:{local_rank}")
    torch.cuda.set_device(dev)

    if args.workload == "C1":
        return c1_latency(args, world, rank, dev)
    if args.workload != "C3":
        return windowed(args, world, rank, dev)
    N, A, F = args.n_envs, args.assets, args.fuse
    extra = dict(nstep_return=args.nstep, discount=0.99, nstep_pop=args.nstep_pop) if args.nstep > 1 else {}
    env, _, _ = workload_env("C3", N, A, rank, dev, **extra)
    if args.layout:
        env.lib.mgn_set_layout(env.h, args.layout)
    if args.schedule != "auto":
        from madigan_amd import _lib as L
        L.check(env.lib.mgn_set_schedule(env.h, {"single": L.SCHED_SINGLE, "duo": L.SCHED_DUO,
                                                  "trio": L.SCHED_TRIO}[args.schedule]), env.h)
    import ctypes as C
    from madigan_amd import _lib as L
    lib, h = env.lib, env.h
    total = args.warmup + args.steps
    # rows [total, total + steps): the kernel-timing launches after the timed
    # region (the same launch plan on the next rows)
    actions = env.generate_actions(total + args.steps, seed=0x6D6164)
    traj = env.alloc_traj(F, fields=[f for f in ("reward", "shaped", "done", "obs_price", "obs_port",
                                                 "timestamp", "tprice", "tunits", "tcost", "risk",
                                                 "margin_call")])

    # one launcher per launch length (the mgn_traj and the action buffer are
    # validated once, outside the timed region; a launch's action rows are
    # bounds-checked by the launcher); the timed loop is one call per launch
    outs, launchers = {}, {}

    def launcher(n):
        if n not in launchers:
            outs[n] = traj if n == F else {k: v[:n] for k, v in traj.items()}
            launchers[n] = env.rollout_launcher(outs[n], n, actions)
        return launchers[n]

    def plan(k0, k1):
        seq, k = [], k0
        while k < k1:
            n = min(F, k1 - k)
            seq.append((launcher(n), k, n))
            k += n
        return seq

    # every step-kernel launch in issue order, (label, steps per launch,
    # launches): tools/reconcile.py matches a kernel trace of this command to
    # the line's figures launch by launch
    launch_log = []

    def logl(label, K, n):
        if launch_log and launch_log[-1][0] == label and launch_log[-1][1] == K:
            launch_log[-1][2] += n
        else:
            launch_log.append([label, K, n])

    def run(seq, label):
        rc = 0
        for fn, k, n in seq:
            rc |= fn(k)
            logl(label, n, 1)
        return rc

    warm, timed = plan(0, args.warmup), plan(args.warmup, total)
    probe_plan = plan(total, total + args.steps)
    # the handle's stream (every launch is on it); --wait spin polls it
    sync = env.stream_synchronizer(spin=args.wait == "spin")
    # kernel durations: HIP events around each step launch on the handle's
    # stream (mgn_set_timing; pooled events, created during the warmup) -- on
    # the kernel-timing launches after the timed region only: the timed
    # region issues the product path exactly as a caller does, with no events
    tmode = 2 if args.timing == "launch" else 1
    L.check(lib.mgn_set_timing(h, tmode), h)
    L.check(run(warm, "warmup"), h)
    torch.cuda.synchronize()
    L.check(lib.mgn_set_timing(h, 0), h)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = run(timed, "timed")
    # the closing wait is on the handle's stream, the only one the steps use
    # (a device-wide synchronize costs ~3 us more on an idle device)
    rc |= sync()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()
    L.check(rc, h)
    # the sharded path's one collective, issued at log intervals
    # in a training loop, not per step: after the timed steps, timed on its own
    from madigan_amd import distributed as D
    ta = time.perf_counter()
    gathered, allgather_path = gather_stats(D, env, world * N)
    torch.cuda.synchronize()
    # reported only when a collective ran ("local": one rank, no exchange)
    allgather_us = (time.perf_counter() - ta) * 1e6 if allgather_path != "local" else None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        if args.dist_backend == "gloo":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the step kernel's duration: the timed region's launch plan once more,
    # right after it, on the next action rows, with the launches' own events
    L.check(lib.mgn_set_timing(h, tmode), h)
    tp = time.perf_counter()
    L.check(run(probe_plan, "probe"), h)
    L.check(sync(), h)
    probe_s = time.perf_counter() - tp
    torch.cuda.synchronize()
    tm = (C.c_double * 4)()
    L.check(lib.mgn_get_timing(h, tm), h)
    L.check(lib.mgn_set_timing(h, 0), h)
    n_launch = int(tm[1])
    avg_launch_s = tm[0] / max(n_launch, 1) / 1e3
    steps_per_launch = args.steps / max(n_launch, 1)
    units_per_launch = N * steps_per_launch
    bpes = survey_bytes_per_env_step(env)
    achieved_gbs = units_per_launch * bpes / avg_launch_s / 1e9
    fused = bytes_per_env_step(A, steps_per_launch, env.D)
    value = world * N * args.steps / elapsed
    episodes = int(gathered[:, 3].sum().item())
    age = total + args.steps  # steps the handle has run

    # after the timed region, rank 0 only: the same handle continues on fresh
    # actions (T_ACT rows, each launch on the next rows, as an agent loop's
    # launches read fresh actions -- one action row repeated launch after
    # launch drives every env into margin calls and auto-resets)
    T_ACT = 1024
    sw_actions = env.generate_actions(T_ACT, seed=0x6D6165) if rank == 0 and args.k_sweep else None
    sw_at = [0]

    def sw_launches(fn, K, n, label):
        """n K-step launches of `fn` (bound to sw_actions), fresh rows each."""
        rc = 0
        logl(label, K, n)
        for _ in range(n):
            if sw_at[0] + K > T_ACT:
                sw_at[0] = 0
            rc |= fn(sw_at[0])
            sw_at[0] += K
        return rc

    def kernel_launch_us(fn, K, n, label):
        """The step kernel's own duration (HIP events recorded by the launch)
        averaged over n launches."""
        L.check(lib.mgn_set_timing(h, 2), h)
        L.check(sw_launches(fn, K, n, label), h)
        torch.cuda.synchronize()
        tk = (C.c_double * 4)()
        L.check(lib.mgn_get_timing(h, tk), h)
        L.check(lib.mgn_set_timing(h, 0), h)
        return tk[0] / max(int(tk[1]), 1) * 1e3

    sw_traj = env.alloc_traj(256, fields=list(traj.keys())) if sw_actions is not None else None
    sw_fns = {}

    def sw_fn(K):
        if K not in sw_fns:
            sw_fns[K] = env.rollout_launcher({kk: v[:K] for kk, v in sw_traj.items()}, K, sw_actions)
        return sw_fns[K]

    def advance_to(target):
        nonlocal age
        while age < target:
            n = min(256, target - age)
            L.check(sw_launches(sw_fn(n), n, 1, "advance"), h)
            age += n
        torch.cuda.synchronize()

    def at_age(target, n=8):
        """The headline's launch (steps_per_launch steps) at episode age
        `target`: kernel time per launch and step, HBM fraction on SURVEY bytes,
        the episodes ended so far (episode age sets the per-step cost: positions
        grow, more orders are refused, rollbacks follow episode ends)."""
        nonlocal age
        advance_to(target)
        Kh = int(round(steps_per_launch))
        us = kernel_launch_us(sw_fn(Kh), Kh, n, f"age_{target}")
        a0 = age
        age += Kh * n
        ep = int(env.episode_stats[:, 3].sum().item())
        return {"age_steps": a0, "launches": n, "steps_per_launch": Kh, "kernel_us_per_launch": us,
                "kernel_us_per_step": us / Kh,
                "frac_survey_bytes": N * Kh * bpes / (us * 1e-6) / 1e9 / PEAK_HBM_GBS,
                "episodes_completed": ep}

    ages, steady, sweep = {}, None, {}
    if sw_actions is not None:
        # per-step cost against episode age; the steady-state figure is the
        # headline's launch after >= 2000 untimed steps
        for tgt in (1000, 2000):
            ages[str(tgt)] = at_age(tgt)
        steady = ages["2000"]
        # steps fused per launch (K in {1, 16, 256} beside the
        # headline; K = 1 is the agent loop's shape, one env.step per policy
        # step, offpolicy_q.py:143), all at steady state: per launch length the
        # step kernel's own duration (launch events) and the per-step time of
        # launches issued back to back through the same per-launch binding as
        # the timed loop
        stream = torch.cuda.current_stream(dev)
        for K in ((1, 16, 64, 256) if args.sweep else (1, 16, 256)):
            reps = max(4, 512 // K)
            fn = sw_fn(K)
            L.check(sw_launches(fn, K, 1, f"sweep_{K}_warm"), h)  # warm
            torch.cuda.synchronize()
            a0 = age + K
            launch_us = kernel_launch_us(fn, K, reps, f"sweep_{K}")
            s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_ev.record(stream)
            L.check(sw_launches(fn, K, reps, f"sweep_{K}_back_to_back"), h)
            e_ev.record(stream)
            torch.cuda.synchronize()
            age += K * (1 + 2 * reps)
            us = s_ev.elapsed_time(e_ev) * 1e3 / (reps * K)
            sweep[str(K)] = {"age_steps": a0, "kernel_us_per_launch": launch_us,
                             "kernel_us_per_step": launch_us / K,
                             "kernel_frac_survey_bytes": N * K * bpes / (launch_us * 1e-6) / 1e9 / PEAK_HBM_GBS,
                             "back_to_back_us_per_step": us, "env_steps_per_s": N / us * 1e6,
                             "achieved_GBs_survey_bytes": N * bpes / us / 1e3,
                             "fused_bytes_per_env_step": bytes_per_env_step(A, K, env.D),
                             "launches": reps}
        tgt = max(5000, age)
        ages[str(tgt)] = at_age(tgt)
        del sw_fns, sw_traj, sw_actions

    if rank == 0 and args.dump_stats:
        np.save(args.dump_stats, gathered.cpu().numpy())
    if rank == 0:
        K = int(round(steps_per_launch))
        # (n-step handles have PMC entries of their own: the pops' rows)
        workload = (f"C3_trendou_{N}x{A}" + (f"_n{args.nstep}" if args.nstep > 1 else "")
                    + ("_running" if args.nstep > 1 and args.nstep_pop == "running" else "") + f"_fuse{K}")
        traffic, traffic_key = load_pmc_traffic(workload)
        probe = bandwidth_probe(dev) if args.probe else None
        roof = {"bound": "hbm", "achieved": achieved_gbs, "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": achieved_gbs / PEAK_HBM_GBS,
                "traffic": traffic, "traffic_key": traffic_key,
                "kernel": kernel_name(env, A),
                "bytes_per_env_step": bpes,
                "bytes_note": "SURVEY 8d algorithmic bytes per env-step (C3: 8 x (113 + 48) + 105): "
                              "state r/w + actions + outputs per step",
                "units_per_launch": units_per_launch, "avg_launch_us": avg_launch_s * 1e6,
                "timing": ("HIP events recorded by the step launch (hipExtLaunchKernel start / stop), "
                           "on the timed plan repeated right after the timed region"
                           if args.timing == "launch" else "HIP marker events around the step launch"),
                "fused_bytes_per_env_step": fused,
                "fused_achieved_GBs": units_per_launch * fused / avg_launch_s / 1e9,
                "fused_note": "what the fused kernel must move (state held in registers across "
                              "the launch's steps; PMC traffic matches this figure)",
                "compute_issue": valu_issue(workload, avg_launch_s)}
        if traffic:
            # the bytes the kernel really moves (PMC, per launch) over the same
            # launch time: `achieved`/`frac` stay on the algorithmic bytes the
            # roofline contract prices, this is the HBM the launch used
            roof["measured_traffic_GBs"] = traffic / avg_launch_s / 1e9
            roof["measured_traffic_frac"] = roof["measured_traffic_GBs"] / PEAK_HBM_GBS
            roof["measured_traffic_note"] = ("PMC (2*FETCH_SIZE + WRITE_SIZE) * 1024 B per launch / "
                                             "avg_launch_us; below `achieved` because the fused "
                                             "kernel keeps the state in registers across steps")
        # the resource that binds the launch, from the PMC figures: fp64 VALU
        # issue (SQ_INSTS_VALU) against the HBM the launch really moved
        # (FETCH_SIZE / WRITE_SIZE); `achieved` / `frac` stay priced on the
        # algorithmic bytes either way
        ci = roof["compute_issue"]
        if ci and traffic:
            busy = ci["valu_busy_frac_lower_bound"]
            roof["bound"] = "valu" if busy > roof["measured_traffic_frac"] else "hbm"
            roof["bound_note"] = (f"PMC: VALU issue >= {busy:.2f} of SIMD cycles vs HBM traffic "
                                  f"{roof['measured_traffic_frac']:.2f} of 8 TB/s")
        if probe:
            # attainable: the better of this box's copy probe and the guide's
            # float4 copy (6.29 TB/s, MI355X_MICROARCH.md)
            roof["attainable_copy_GBs"] = probe
            roof["attainable_GBs"] = max(probe, GUIDE_COPY_GBS)
            roof["frac_of_attainable"] = achieved_gbs / roof["attainable_GBs"]
        res = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "C3: TrendOU x8 assets per env, slippage 1e-4 + 2% cost broker, "
                                   + (f"DDR eta=.001 n={args.nstep} (discount .99, {args.nstep_pop} pop; "
                                      "a diagnostic line, not the headline)" if args.nstep > 1 else
                                      "DDR eta=.001 n=1")
                                   + ", discrete actions via action_to_transaction, auto-reset",
                       "nstep": args.nstep, "nstep_pop": args.nstep_pop if args.nstep > 1 else None,
                       "n_envs_per_gpu": N, "n_envs_total": world * N, "n_assets": A, "window": 0,
                       "steps_per_launch": steps_per_launch,
                       "assets_per_lane": int(lib.mgn_get_layout(h)),
                       "schedule": SCHED_NAMES[int(lib.mgn_get_schedule(h))],
                       "parallelism": f"env-sharded x{world} (no per-step collective)"
                                      + (f", {args.dist_backend}" if world > 1 else "")},
            "roofline": roof,
            "kernel_us_per_step": avg_launch_s * 1e6 / steps_per_launch,
            "timed_region_us_per_launch": elapsed * 1e6 / max(n_launch, 1),
            "kernel_timing": {
                "launches": n_launch, "avg_launch_us": avg_launch_s * 1e6,
                "region_us_with_events": probe_s * 1e6,
                "note": "the timed region issues the product path with no timing events; the kernel "
                        "figure (roofline.avg_launch_us) comes from the same launch plan issued right "
                        "after it on the next action rows, each launch recording its own HIP events "
                        "(region_us_with_events: that plan's wall time, events included)"},
            "episodes_completed": episodes,
            "stats_allgather_us": allgather_us,
            "allgather_path": allgather_path,
        }
        if steady:
            res["steady_state"] = steady
            res["episode_age"] = ages
            res["episode_age_note"] = (
                "the headline's launch on the same handle after the timed region, at the handle's step "
                "index age_steps (fresh actions): kernel time from the launch's own HIP events; the "
                "steady-state figure is the one after >= 2000 untimed steps (episodes ended)")
        res["launch_log"] = launch_log
        if sweep:
            res["launch_lengths"] = sweep
            res["launch_lengths_note"] = (
                "K steps per launch on the same handle at steady state (age_steps: the handle's step "
                "index): kernel_us_per_launch from the launch's own HIP events; back_to_back_us_per_step "
                "from events around `launches` launches issued by the per-launch binding (host + "
                "dispatch included); frac on SURVEY 8d bytes (1393 B per C3 env-step) over the kernel time")
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(N, A, args.cpu_budget)
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


def c1_latency(args, world, rank, dev):
    """C1: the Python-level Env.step latency of one env -- the
    drop-in madigan_amd.Env (one 1-asset sine, no costs, env log reward)
    called per step from Python as the reference agent calls its pybind11 Env
    (each step returns host State / reward / done / EnvInfo, so it launches
    and synchronises once per step).  Beside it the oracle's one-env step
    through ctypes on one host core.  Rank 0 only; latency, lower is better."""
    import torch
    from madigan_amd import Env
    if rank != 0:
        return
    T = max(1000, args.steps * 5)
    cfg = {"data_source_type": "Synth",
           "data_source_config": {"freq": [1.0], "mu": [2.0], "amp": [1.0], "phase": [0.0],
                                  "dX": 0.01, "noise": 0.0}}
    env = Env("Synth", 1_000_000.0, cfg, device=dev, seed=0x6D6165)
    rng = np.random.default_rng(1)
    units = rng.integers(-1, 2, size=(T + 200, 1)).astype(np.float64) * 10.0
    for t in range(200):
        env.step(units[t])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(T):
        env.step(units[200 + t])
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / T * 1e6
    res = {"metric": "Env.step latency (C1: 1 env x 1 asset, Python per-step call)", "value": us,
           "unit": "us/step", "n_gpus": 1, "steps": T, "warmup": 200, "ms_per_step": us / 1e3,
           "higher_is_better": False, "scaling": "none", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic",
           "config": {"workload": "C1: Synth sine freq 1 mu 2 amp 1 phase 0 dX .01 noise 0, no costs, "
                                  "env log reward, Env.step(units) from Python"}}
    if not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle import oracle as O
        orc = O.OracleBatch(dict(n_envs=1, seed=0x6D6165), [(O.SRC_SINE, [1.0, 2.0, 1.0, 0.0, 0.01, 0.0])])
        for t in range(200):
            orc.step(units[t].reshape(1, 1))
        t0 = time.perf_counter()
        for t in range(T):
            orc.step(units[200 + t].reshape(1, 1))
        cus = (time.perf_counter() - t0) / T * 1e6
        res["cpu_baseline"] = {"value": cus, "unit": "us/step", "cores": 1, "kind": "port",
                               "sample": f"C1, {T} steps of the oracle's one-env step through ctypes"}
    print(json.dumps(res))


def windowed(args, world, rank, dev):
    """C2 / C4 / C5: per launch `fuse` steps, each followed by its window
    (StackerDiscrete.current_data) -- mgn_rollout_hist (the K steps, every
    ring push kept in the launch history) then mgn_window_hist (all K windows
    to (K,N,W,·)).  Every step's window is materialised, as the agent reads one
    per step."""
    import torch
    import torch.distributed as dist
    wl = args.workload
    N = {"C2": 4096}.get(wl, args.n_envs)
    A = {"C2": 4, "C4": 8, "C5": 16, "R1": 1}[wl]
    if wl == "C2" and args.win_assets:
        # diagnostic: OU windows at another asset count, at --n-envs envs
        N, A = args.n_envs, args.win_assets
    env, desc, W = workload_env(wl, N, A, rank, dev, **({"shaper": args.shaper, "nstep_pop": args.nstep_pop}
                                                         if wl == "R1" else {}))
    Kf = max(1, min(args.fuse, args.win_fuse))
    n_warm = max(1, -(-args.warmup // Kf))
    n_time = max(1, -(-args.steps // Kf))
    args.warmup, args.steps = n_warm * Kf, n_time * Kf
    total = args.warmup + args.steps
    actions = env.generate_actions(total, seed=0x6D6164)
    traj = env.alloc_traj(Kf, fields=["reward", "shaped", "done", "obs_price", "obs_port",
                                      "timestamp", "tprice", "tunits", "tcost", "risk",
                                      "margin_call", "data_end"] + (["n_shaped"] if env.nstep > 1 else []))
    wp = torch.empty((Kf, N, W, env.F), dtype=torch.float64, device=dev)
    wo = torch.empty((Kf, N, W, A + 1), dtype=torch.float64, device=dev)
    wt = torch.empty((Kf, N, W), dtype=torch.int64, device=dev)
    import ctypes as C
    from madigan_amd import _lib as L
    lib, h = env.lib, env.h
    if args.schedule != "auto":
        L.check(lib.mgn_set_schedule(h, {"single": L.SCHED_SINGLE, "duo": L.SCHED_DUO,
                                         "trio": L.SCHED_TRIO}[args.schedule]), h)
    if args.win_overlap:
        # gathers on a second stream, the history double-buffered: launch L's
        # gather (HBM-bound) runs beside launch L+1's steps (latency-bound).
        # Measured: +7 % at C4, -5 % at C5 (the step kernel's latency rises
        # under the gather's traffic), so it is off by default.
        wstream = torch.cuda.Stream(dev)
        L.check(lib.mgn_set_window_stream(h, C.c_void_p(wstream.cuda_stream)), h)
    tstruct = C.byref(env._traj_struct(traj))
    per = env.N * env.A
    base = actions.data_ptr()
    wptr = [C.c_void_p(x.data_ptr()) for x in (wp, wo, wt)]

    # one step per launch (--win-fuse 1, the reference's own driving:
    # offpolicy_q.py:143, 193-194 -- env.step, then stream_state /
    # current_data): mgn_rollout then mgn_window, the window gathered from the
    # ring the step kernel pushed to (no launch history to copy into)
    agent_k1 = Kf == 1 and args.k1_ring

    def run(l0, l1):
        rc = 0
        for l in range(l0, l1):
            if agent_k1:
                rc |= lib.mgn_rollout(h, C.c_void_p(base + l * per), 1, tstruct)
                rc |= lib.mgn_window(h, *wptr)
            else:
                rc |= lib.mgn_rollout_hist(h, C.c_void_p(base + l * Kf * per), Kf, tstruct)
                rc |= lib.mgn_window_hist(h, *wptr)
        L.check(rc, h)

    run(0, n_warm)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # kernel durations: HIP events on each kernel's own stream (mgn_set_timing)
    L.check(lib.mgn_set_timing(h, 1), h)
    t0 = time.perf_counter()
    run(n_warm, n_warm + n_time)
    torch.cuda.synchronize()
    if world > 1:
        # barrier + synchronize; at one rank the synchronize above is both
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the episode-statistics all-gather (log intervals, not per step): after the timed steps
    from madigan_amd import distributed as D
    gathered, allgather_path = gather_stats(D, env, world * N)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        if args.dist_backend == "gloo":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    tm = (C.c_double * 4)()
    L.check(lib.mgn_get_timing(h, tm), h)
    L.check(lib.mgn_set_timing(h, 0), h)
    step_us = tm[0] / max(tm[1], 1) * 1e3
    gather_us = tm[2] / max(tm[3], 1) * 1e3
    # the zero-copy form (element-wise normalisers, preprocessor.py:183-189):
    # the same launches with the windows read in place from the launch
    # history (mgn_window_hist_view) instead of materialised -- measured after
    # the timed region, reported beside the line, never as its value
    view = None
    if env.cfg.norm_type in (L.NORM_NONE, L.NORM_LOG):
        hv = L.HistView()

        def run_view(l0, l1):
            rc = 0
            for l in range(l0, l1):
                rc |= lib.mgn_rollout_hist(h, C.c_void_p(base + l * Kf * per), Kf, tstruct)
                rc |= lib.mgn_window_hist_view(h, C.byref(hv))
            L.check(rc, h)
        n_view = n_time  # the timed launches' actions again
        run_view(n_warm, n_warm + 1)
        torch.cuda.synchronize()
        tv = time.perf_counter()
        run_view(n_warm, n_warm + n_view)
        torch.cuda.synchronize()
        view_s = time.perf_counter() - tv
        view = {"value": N * n_view * Kf / view_s, "unit": "env-steps/s",
                "ms_per_step": view_s * 1e3 / (n_view * Kf), "launches": n_view,
                "note": "mgn_rollout_hist + mgn_window_hist_view: each step's window is the history "
                        "row range [hend - hlen, hend), read in place by the consumer (no k_hist_gather); "
                        "measured after the timed region on this rank"}
    gb = gather_bytes(env, Kf)
    achieved = gb / (gather_us * 1e-6) / 1e9
    value = world * N * args.steps / elapsed
    if rank == 0:
        C = env.F + env.A + 1
        res = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": desc, "n_envs_per_gpu": N, "n_envs_total": world * N, "n_assets": A,
                       "n_feats": env.F,
                       "window": W, "steps_per_launch": Kf, "nstep": env.nstep,
                       "nstep_pop": args.nstep_pop if env.nstep > 1 else None,
                       "drive": ("mgn_rollout (one step) + mgn_window (the ring's window) per step, as "
                                 "offpolicy_q.py:143,193-194 drives env.step / current_data") if agent_k1 else
                                "mgn_rollout_hist (K steps) + mgn_window_hist (every step's window)",
                       "schedule": SCHED_NAMES[int(lib.mgn_get_schedule(h))],
                       "parallelism": f"env-sharded x{world} (no per-step collective)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                         "traffic": load_pmc_traffic(f"{wl}_gather_{N}x{A}_W{W}")[0],
                         "kernel": "mgn::k_ring_gather_lds" if agent_k1 else "mgn::k_hist_gather",
                         "bytes_per_env_step": gb / (N * Kf),
                         "avg_launch_us": gather_us},
            "step_launch_avg_us": step_us,
            "step_launch_traffic": load_pmc_traffic(f"{wl}_step_{N}x{A}_fuse{Kf}")[0],
            "step_launch_note": "the K-step step kernel" + (
                " (the previous launch's k_hist_gather runs beside it on a second stream)"
                if args.win_overlap else ""),
            "episodes_completed": int(gathered[:, 3].sum().item()),
            "allgather_path": allgather_path,
        }
        if view is not None:
            res["view_mode"] = view
        if wl == "C5":
            tape_bytes = sum(t.numel() * t.element_size() for t in env._tape.values())
            res["replay_staging"] = {"tape_rows": int(env._tape["ts"].shape[0]),
                                     "tape_bytes": tape_bytes, "stage_s": env._stage_s,
                                     "pcie_inclusive_GBs": tape_bytes / env._stage_s / 1e9}
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
