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
    for shaper in ("DSR", "DDR", "cosine"):
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
                       "desired_portfolio": list(np.linspace(1, 0, D + 1)), "cosine_temp": 0.05}
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
                key = f"{shaper}_n{n}_D{D}"
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


def main():
    _stub_modules()
    from madigan.utils import preprocessor
    from madigan.utils.buffers import nstep_buffer
    data = {"eps": np.array(float(nstep_buffer.EPS))}
    shaper_vectors(nstep_buffer, data)
    window_vectors(preprocessor, data)
    path = os.path.join(OUT, "reference_vectors.npz")
    np.savez_compressed(path, **data)
    print(f"wrote {path}: {len(data)} arrays")


if __name__ == "__main__":
    main()
