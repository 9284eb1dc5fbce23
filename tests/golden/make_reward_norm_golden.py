"""Golden vectors of the reference's reward normalisers
(madigan/environments/reward_normalization.pyx), from the reference itself
compiled by `make -C oracle ref_normalizers` into oracle/_ref/.

    python tests/golden/make_reward_norm_golden.py

For each class and window: 8 reward streams of 300 log-return-like values
(one stream per reference object, one `stream` call per value), with the
object reset at fixed steps of some streams (an episode end); the inputs, the
reset schedule and every output go to tests/golden/reward_norm_vectors.npz.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle", "_ref"))
import reward_normalization as R  # noqa: E402  (the compiled reference)

CASES = [("SharpeFixedWindow", 5), ("SharpeFixedWindow", 32), ("SortinoFixedWindowA", 7),
         ("SortinoFixedWindowB", 4), ("SortinoFixedWindowB", 16), ("SortinoFixedWindowC", 6),
         ("SharpeEWMA", 10), ("SharpeEWMA", 3)]


def main():
    rng = np.random.default_rng(20261017)
    S, T = 8, 300
    rewards = rng.normal(0.0, 0.01, (S, T))
    rewards[:, ::17] = 0.0           # exact zeros
    rewards[3, 40:60] = -0.02        # a run below the mean
    resets = np.zeros((S, T), dtype=bool)
    resets[1, 100] = resets[2, 37] = resets[2, 38] = resets[5, 250] = True
    out = {"rewards": rewards, "resets": resets}
    for name, w in CASES:
        res = np.zeros((S, T))
        for e in range(S):
            obj = getattr(R, name)(w)
            for t in range(T):
                if resets[e, t]:
                    obj.reset()
                res[e, t] = obj.stream(float(rewards[e, t]))
        out[f"{name}_{w}"] = res
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reward_norm_vectors.npz")
    np.savez_compressed(path, **out)
    print(path, sorted(out))


if __name__ == "__main__":
    main()
