"""Generate golden vectors from the reference's own Python implementations.

Run in the build container (the reference checkout is at /root/reference):

    python tests/golden/make_golden.py

It imports madigan/utils/buffers/nstep_buffer.py (DSR, DDR, cosine PPC) and
madigan/utils/preprocessor.py (StackerDiscrete) with stub modules for the two
third-party imports that are absent offline and unused by that arithmetic
(numba decorators; rollers.Roller, used only by RollerDiscrete).  Outputs are
plain .npz data (inputs and expected outputs) -- no reference source is
copied.  Rewards are fed as float64 ndarrays, as the reference agent does
(offpolicy_q.py:160-164); a python-float reward would hit NumPy-2 scalar
promotion with the float32 EPS (NEP 50), which the pinned numpy 1.18 did not.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REF = os.environ.get("MADIGAN_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _stub_modules():
    nb = types.ModuleType("numba")

    def deco(*a, **k):
        if a and callable(a[0]) and not k:
            return a[0]
        return lambda f: f

    class _T:
        def __call__(self, *a, **k):
            return self

        def __getitem__(self, k):
            return self

    for n in ("njit", "jit", "guvectorize", "vectorize", "prange"):
        setattr(nb, n, deco)
    for n in ("float64", "float32", "int64", "int32", "boolean", "void"):
        setattr(nb, n, _T())
    sys.modules["numba"] = nb
    r = types.ModuleType("rollers")
    r.Roller = object
    sys.modules["rollers"] = r
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)


def shaper_vectors(nstep_buffer, data):
    """Drive NStepBuffer exactly like ReplayBuffer.add (replay_buffer.py:68-80)."""
    from madigan.utils.data import SARSD, State
    rng = np.random.default_rng(20261015)
    cases = []
    # (shaper type, sortino_exp, case-key prefix); the naive shapers (sharpe_shaper,
    # sortino_shaperA/B, nstep_buffer.py:207-312) follow the original three so the
    # earlier cases keep their random draws
    shapers = [("DSR", 2, "DSR"), ("DDR", 2, "DDR"), ("cosine", 2, "cosine"),
               ("sharpe_shaper", 2, "sharpe"), ("sortino_shaperA", 2, "sortinoA"),
               ("sortino_shaperB", 2, "sortinoB"), ("sortino_shaperA", 3, "sortinoA3"),
               ("sortino_shaperB", 3, "sortinoB3")]
    for shaper, sexp, prefix in shapers:
        for n in (1, 5, 20):
            for D in (1, 4):
                T = 64
                rewards = rng.normal(0, 0.01, (T, D))
                rewards[rng.random((T, D)) < 0.1] = 0.0          # r == 0 takes DDR's 2nd branch
                rewards[5] = 0.5                                  # clip saturation
                ports = rng.normal(0, 0.5, (T, D + 1))
                dones = np.zeros(T, bool)
                dones[[17, 40]] = True                            # done-flush
                cfg = {"reward_shaper": shaper, "adaptation_rate": 0.01,
                       "desired_portfolio": list(np.linspace(1, 0, D + 1)), "cosine_temp": 0.05,
                       "sortino_exp": sexp}
                nb = nstep_buffer.NStepBuffer(n, 0.99, cfg)
                outs, out_steps = [], []
                for t in range(T):
                    st = State(ports[t][None, :], ports[t][None, :], np.array([t]))
                    s = SARSD(st, 0, rewards[t].copy(), st, bool(dones[t]))
                    nb.add(s)
                    if nb.full():
                        outs.append(np.atleast_1d(np.asarray(nb.pop_nstep_sarsd().reward, float)))
                        out_steps.append(t)
                    if dones[t]:
                        while len(nb) > 0:
                            outs.append(np.atleast_1d(np.asarray(nb.pop_nstep_sarsd().reward, float)))
                            out_steps.append(t)
                key = f"{prefix}_n{n}_D{D}"
                data[key + "_shaper"] = np.array(shaper)
                data[key + "_exp"] = np.array(float(sexp))
                data[key + "_rewards"] = rewards
                data[key + "_ports"] = ports
                data[key + "_dones"] = dones
                data[key + "_out"] = np.array(outs)
                data[key + "_out_step"] = np.array(out_steps)
                data[key + "_cfg"] = np.array([n, 0.99, 0.01, 0.05])
                data[key + "_desired"] = np.array(cfg["desired_portfolio"])
                cases.append(key)
    data["shaper_cases"] = np.array(cases)


def window_vectors(preprocessor, data):
    from madigan.utils.data import State
    rng = np.random.default_rng(7)
    T, F, W = 40, 3, 8
    prices = 10 + np.cumsum(rng.normal(0, 0.3, (T, F)), axis=0)
    prices[11, 1] = -0.5                     # log_norm clamp max(x, 1e-5)
    prices[:, 2] = np.where(np.arange(T) < 20, 5.0, prices[:, 2])  # std == 0 -> nan_to_num
    ports = rng.normal(0, 0.3, (T, F + 1))
    data["win_prices"] = prices
    data["win_ports"] = ports
    data["win_W"] = np.array(W)
    for norm_type in ("log", "lookback", "standard_normal", "lookback_log"):
        sd = preprocessor.StackerDiscrete(W, F, norm=True, norm_type=norm_type)
        outs_p, outs_port, outs_ts = [], [], []
        for t in range(T):
            sd.stream_state(State(prices[t], ports[t], t + 2))
            cur = sd.current_data()
            pad = W - cur.price.shape[0]
            outs_p.append(np.vstack([cur.price, np.zeros((pad, F))]))
            outs_port.append(np.vstack([cur.portfolio, np.zeros((pad, F + 1))]))
            outs_ts.append(np.concatenate([cur.timestamp, np.zeros(pad, int)]))
        data[f"win_{norm_type}_price"] = np.array(outs_p)
        data[f"win_{norm_type}_port"] = np.array(outs_port)
        data[f"win_{norm_type}_ts"] = np.array(outs_ts)
    # make_normalizer(None) raises (preprocessor.py:53-77): pinned behaviour
    try:
        preprocessor.StackerDiscrete(W, F, norm=False, norm_type=None)
        data["win_none_raises"] = np.array(False)
    except NotImplementedError:
        data["win_none_raises"] = np.array(True)
    # 'expanding' builds, but its lambda calls _expanding_mean(x) with one of
    # two required arguments (preprocessor.py:73, :475): current_data raises TypeError
    sd = preprocessor.StackerDiscrete(W, F, norm=True, norm_type="expanding")
    sd.stream_state(State(prices[0], ports[0], 2))
    try:
        sd.current_data()
        data["win_expanding_raises"] = np.array(False)
    except TypeError:
        data["win_expanding_raises"] = np.array(True)


def stacker_variant_vectors(preprocessor, data):
    """log_standard_normal, StackerDiscreteReturns, StackerDiscretePairs and
    MultiStackerDiscrete (preprocessor.py:95-107, :202-327) over one stream."""
    from madigan.utils.data import State
    rng = np.random.default_rng(11)
    T, F, W = 40, 3, 8
    prices = 10 + np.cumsum(rng.normal(0, 0.3, (T, F)), axis=0)
    prices[13, 0] = -0.5                     # log(x < 0) = nan: nanmean / nanstd skip it
    ports = rng.normal(0, 0.3, (T, F + 1))
    data["var_prices"] = prices
    data["var_ports"] = ports
    data["var_W"] = np.array(W)

    def store(key, outs):
        """outs: per step (price (r, c), port (r2, P), ts (r2,)); zero-padded to
        (T, W, cmax) / (T, W, P) / (T, W) with the row and column counts."""
        cmax = max([o[0].shape[1] for o in outs if o[0].ndim == 2] + [1])
        pr = np.zeros((T, W, cmax))
        po = np.zeros((T, W, F + 1))
        ts = np.zeros((T, W), np.int64)
        shape = np.zeros((T, 3), np.int64)   # price rows, price cols, port/ts rows
        for t, (p, q, s) in enumerate(outs):
            p = p.reshape(p.shape[0], -1) if p.size else np.zeros((0, 0))
            pr[t, :p.shape[0], :p.shape[1]] = p
            po[t, :q.shape[0], :q.shape[1]] = q.reshape(q.shape[0], -1) if q.size else 0
            ts[t, :s.shape[0]] = s
            shape[t] = (p.shape[0], p.shape[1], q.shape[0])
        data[key + "_price"], data[key + "_port"], data[key + "_ts"] = pr, po, ts
        data[key + "_shape"] = shape

    def run(pp, feed, key):
        outs = []
        for t in range(T):
            pp.stream_state(State(feed[t], ports[t], t + 2))
            cur = pp.current_data()
            outs.append((np.asarray(cur.price, float), np.asarray(cur.portfolio, float),
                         np.asarray(cur.timestamp, np.int64)))
        store(key, outs)

    with np.errstate(all="ignore"):
        run(preprocessor.StackerDiscrete(W, F, norm=True, norm_type="log_standard_normal"),
            prices, "var_lsn")
        for nt in ("log", "lookback", "standard_normal"):
            run(preprocessor.StackerDiscreteReturns(W, F, norm=True, norm_type=nt), prices,
                f"var_returns_{nt}")
        for nt in ("lookback", "log"):
            run(preprocessor.StackerDiscretePairs(W, 2, norm=True, norm_type=nt), prices[:, :2],
                f"var_pairs_{nt}")
    # MultiStackerDiscrete allocates its counters with np.int (numpy < 1.24, the
    # reference pins 1.18.1); numpy 2 dropped the alias, so restore it for the run
    if not hasattr(np, "int"):
        np.int = int
    dil = [1, 3, 4]
    data["var_multi_dilations"] = np.array(dil)
    for nt in ("lookback", "standard_normal"):
        ms = preprocessor.MultiStackerDiscrete(W, dil, F, norm=True, norm_type=nt)
        outs, ok = [], []
        for t in range(T):
            ms.stream_state(State(prices[t], ports[t], t + 2))
            try:
                cur = ms.current_data()
                outs.append((np.asarray(cur.price, float), np.asarray(cur.portfolio, float),
                             np.asarray(cur.timestamp, np.int64)))
                ok.append(True)
            except ValueError:  # dilation buffers of unequal length cannot be concatenated
                outs.append((np.zeros((0, F * len(dil))), np.zeros((0, F + 1)), np.zeros(0, np.int64)))
                ok.append(False)
        data[f"var_multi_{nt}_ok"] = np.array(ok)
        store(f"var_multi_{nt}", outs)


def main():
    _stub_modules()
    from madigan.utils import preprocessor
    from madigan.utils.buffers import nstep_buffer
    data = {"eps": np.array(float(nstep_buffer.EPS))}
    shaper_vectors(nstep_buffer, data)
    window_vectors(preprocessor, data)
    stacker_variant_vectors(preprocessor, data)
    path = os.path.join(OUT, "reference_vectors.npz")
    np.savez_compressed(path, **data)
    print(f"wrote {path}: {len(data)} arrays")


if __name__ == "__main__":
    main()
