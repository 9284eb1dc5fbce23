"""n-step reward aggregation (n > 1) in the oracle's batch
path, checked against NStepBuffer semantics as ReplayBuffer.add drives them
(replay_buffer.py:68-80, nstep_buffer.py:315-356), restated here with the
shaper kernels that tests/test_golden.py pins to the reference's own Python
(O.dsr / O.ppc).  The per-step rewards, dones and portfolio rows come from an
n == 1 run of the same configuration (shaping never feeds back into state)."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests.configs import trendou_sources

DONE_P = [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99]
DONE_KW = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02,
               unit_size=0.9, auto_reset=1, init_cash=1e5)


def expected_emissions(traj, shaper, mode, n, gamma, eta, temp, desired):
    """Per step and env, the list of shaped rewards NStepBuffer pops."""
    rin = traj["reward"] if mode == "env_log" else traj["agent_reward"]
    K, N = traj["done"].shape
    D = 1 if rin.ndim == 2 else rin.shape[2]
    disc = np.array([math.pow(gamma, i) for i in range(n)])
    out = [[[] for _ in range(N)] for _ in range(K)]
    for e in range(N):
        A_, B_ = np.zeros(D), np.zeros(D)
        buf = []
        for k in range(K):
            buf.append(k)

            def pop():
                L = len(buf)
                r = np.array([rin[t, e] for t in buf]).reshape(L, D)
                if shaper in ("DSR", "DDR"):
                    v = O.dsr(r, disc[:L], eta, A_, B_, ddr=shaper == "DDR")
                elif shaper == "PPC":
                    v = O.ppc(r, np.array([traj["obs_port"][t, e] for t in buf]), desired, temp,
                              disc[:L])
                else:
                    v = np.zeros(D)
                    for j in range(L):
                        v = v + disc[j] * r[j]
                buf.pop(0)
                return v

            if len(buf) >= n:
                out[k][e].append(pop())
            if traj["done"][k, e]:
                while buf:
                    out[k][e].append(pop())
    return out


@pytest.mark.parametrize("shaper,mode,n", [("DSR", "env_log", 3), ("DDR", "env_log", 5),
                                          ("DDR", "agent_per_asset", 4), ("PPC", "env_log", 3),
                                          ("none", "agent_sum", 4), ("DSR", "agent_sum", 20)])
def test_nstep_batch_matches_replay_semantics(shaper, mode, n):
    N, A, K = 24, 3, 60
    gamma, eta, temp = 0.97, 0.01, 0.05
    desired = [0.5, 0.2, 0.2, 0.1]
    cfg = dict(n_envs=N, seed=9, reward_shaper=shaper, reward_mode=mode, adaptation_rate=eta,
               cosine_temp=temp, desired_portfolio=desired, discount=gamma, **DONE_KW)
    acts = np.random.default_rng(3).integers(0, 3, (K, N, A)).astype(np.int8)
    one = O.OracleBatch(dict(cfg, nstep_return=1), trendou_sources(A, DONE_P)).rollout(acts)
    assert one["done"].sum() > 0
    got = O.OracleBatch(dict(cfg, nstep_return=n), trendou_sources(A, DONE_P)).rollout(acts)
    exp = expected_emissions(one, shaper, mode, n, gamma, eta, temp, np.array(desired))
    D = A if mode == "agent_per_asset" else 1
    sh = got["shaped"].reshape(K, N, n, D)
    for k in range(K):
        for e in range(N):
            c = int(got["n_shaped"][k, e])
            assert c == len(exp[k][e]), (k, e)
            if c:
                np.testing.assert_allclose(sh[k, e, :c], np.array(exp[k][e]), rtol=1e-13,
                                           atol=1e-16)
            assert not sh[k, e, c:].any()


def test_nstep_one_matches_single_step_path():
    """nstep_return == 1 emits exactly one shaped reward per step."""
    N, A, K = 16, 2, 30
    cfg = dict(n_envs=N, seed=2, reward_shaper="DDR", nstep_return=1, **DONE_KW)
    acts = np.random.default_rng(4).integers(0, 3, (K, N, A)).astype(np.int8)
    got = O.OracleBatch(cfg, trendou_sources(A, DONE_P)).rollout(acts)
    assert (got["n_shaped"] == 1).all()
    assert got["shaped"].shape == (K, N)
