"""The random-variate specification and the generators' statistics.

The reference seeds std::default_random_engine from the wall clock
(DataSource.cpp:472, :1131, :1407), so its draws cannot be replayed: generator
parity with the reference is distributional ("parity unpinned" bitwise), and
bitwise between the oracle and the HIP kernels (tests/test_gpu_parity.py).
These tests pin the specification itself: Philox4x32-10 against the Random123
known-answer vectors, the fdlibm log/sin/cos against libm, the variates'
moments, and each generator's statistics against its reference formula.
"""
import ctypes as C
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests.configs import ou_sources, trendou_sources


@pytest.mark.parametrize("ctr,key,expect", [  # Random123 kat_vectors, philox4x32 10 rounds
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
])
def test_philox_kat(ctr, key, expect):
    assert list(O.philox(ctr, key)) == expect


def test_fdlibm_accuracy_vs_libm():
    L = O.lib()
    rng = np.random.default_rng(0)
    for x in rng.uniform(1e-300, 1.0, 5000):
        assert abs(L.orc_log(x) - math.log(x)) <= 2 * np.spacing(abs(math.log(x)))
    for x in np.concatenate([rng.uniform(-1e5, 1e5, 5000), np.arange(1, 200) * math.pi]):
        assert abs(L.orc_sin(x) - math.sin(x)) <= 2e-16 + 2 * np.spacing(abs(math.sin(x)))
    # the variates' fma-form kernels (specification v3)
    sn, cs = C.c_double(), C.c_double()
    for u in rng.uniform(0, 1, 5000):
        L.orc_vsincos2pi(u, C.byref(sn), C.byref(cs))
        assert abs(cs.value - math.cos(2 * math.pi * u)) < 1e-15
        assert abs(sn.value - math.sin(2 * math.pi * u)) < 1e-15
    for x in rng.uniform(1e-300, 1.0, 5000):
        assert abs(L.orc_vlog(x) - math.log(x)) <= 2 * np.spacing(abs(math.log(x)))


def _draws(n, d_of):
    L = O.lib()
    z, ut = np.zeros(n), np.zeros(n)
    bit = np.zeros(n, np.uint32)
    zz, uu, bb = C.c_double(), C.c_double(), C.c_uint32()
    for i in range(n):
        env, asset, d = d_of(i)
        L.orc_draw0(11, env, asset, d, C.byref(zz), C.byref(uu), C.byref(bb))
        z[i], ut[i], bit[i] = zz.value, uu.value, bb.value
    return z, ut, bit


def test_variates_moments():
    """Specification v3: the even and odd draw index of a pair are the
    Box-Muller pair (r cos, r sin) of one block, each with its own switch
    uniform and direction bit."""
    z, ut, bit = _draws(200_000, lambda i: (i % 1000, i // 1000 % 8, i // 8000))
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    assert abs(np.mean(z ** 4) - 3) < 0.1        # normal kurtosis
    assert abs(ut.mean() - 0.5) < 0.005 and ut.min() >= 0 and ut.max() < 1
    assert abs(bit.mean() - 0.5) < 0.01
    # consecutive draw indices of one (env, asset): both halves of every pair
    zs, us, bs = _draws(200_000, lambda i: (i // 500, 3, i % 500))
    e, o = zs[0::2], zs[1::2]                    # (even, odd) halves of each pair
    for x in (e, o):
        assert abs(x.mean()) < 0.01 and abs(x.std() - 1) < 0.01
    assert abs(np.corrcoef(e, o)[0, 1]) < 0.01   # the Box-Muller pair is independent
    assert abs(np.corrcoef(e ** 2, o ** 2)[0, 1]) < 0.01
    assert abs(np.corrcoef(zs[1:-1:2], zs[2::2])[0, 1]) < 0.01  # across pairs
    assert abs(np.corrcoef(us[0::2], us[1::2])[0, 1]) < 0.01    # the halves' switch uniforms
    assert abs(np.corrcoef(us[1::2], np.abs(o))[0, 1]) < 0.01   # odd uniform vs the odd normal
    assert abs(bs[1::2].mean() - 0.5) < 0.01


def test_variates_pair_definition():
    """The pair's halves are r cos(2 pi u2) and r sin(2 pi u2) of block A at
    counter d >> 1 (restated here from the Philox block in Python)."""
    L = O.lib()
    zz, uu, bb = C.c_double(), C.c_double(), C.c_uint32()
    sn, cs = C.c_double(), C.c_double()
    seed, env, asset = 0x1234_5678_9ABC, 77, 5
    for P in (0, 1, 12345, 2 ** 33 + 7):
        x = O.philox([P & 0xFFFFFFFF, env, asset, (P >> 32) ^ 0], [seed & 0xFFFFFFFF, seed >> 32])
        a = ((int(x[1]) << 32) | int(x[0])) >> 11
        r = math.sqrt(-2.0 * L.orc_vlog((a + 1) * 2.0 ** -53))
        L.orc_vsincos2pi(int(x[2]) * 2.0 ** -32, C.byref(sn), C.byref(cs))
        L.orc_draw0(seed, env, asset, 2 * P, C.byref(zz), C.byref(uu), C.byref(bb))
        assert zz.value == r * cs.value and uu.value == int(x[3]) * 2.0 ** -32 and bb.value == x[0] & 1
        L.orc_draw0(seed, env, asset, 2 * P + 1, C.byref(zz), C.byref(uu), C.byref(bb))
        y = O.philox([P & 0xFFFFFFFF, env, asset | (3 << 16), (P >> 32) ^ 0],
                     [seed & 0xFFFFFFFF, seed >> 32])
        assert zz.value == r * sn.value and uu.value == int(y[3]) * 2.0 ** -32 and bb.value == y[0] & 1


def test_ou_stationary_moments():
    """x += theta(mu-x) + mu*phi*N(0,1) (DataSource.cpp:1173-1180): stationary
    mean mu, variance (mu phi)^2 / (1 - (1-theta)^2)."""
    mu, theta, phi = 10.0, 0.08, 0.04
    b = O.OracleBatch(dict(n_envs=400, seed=3), ou_sources(2, mu, theta, phi))
    for _ in range(200):
        b.step()
    xs = []
    for _ in range(300):
        b.step()
        xs.append(b.field(O.F_PRICE).copy())
    x = np.array(xs)
    var = (mu * phi) ** 2 / (1 - (1 - theta) ** 2)
    assert abs(x.mean() - mu) < 0.05
    assert abs(x.var() / var - 1) < 0.05


def test_trendou_regime_switching_rate():
    """Trend starts with probability trendProb per OU-regime tick and lasts
    U{min..max} ticks (DataSource.cpp:1457-1493)."""
    p = [0.01, 5, 15, 0.001, 0.005, 5.0, 0.15, 0.04, 0.001, 0.99]
    b = O.OracleBatch(dict(n_envs=500, seed=7), trendou_sources(4, p))
    starts = 0
    ou_ticks = 0
    lens = []
    prev = b.field(O.F_TRENDING)
    for _ in range(400):
        ou_ticks += int((prev == 0).sum())
        b.step()
        cur = b.field(O.F_TRENDING)
        new = (prev == 0) & (cur == 1)
        starts += int(new.sum())
        lens.extend(b.field(O.F_TLEN)[new].tolist())
        prev = cur
    rate = starts / ou_ticks
    assert abs(rate - 0.01) < 0.001
    assert min(lens) >= 5 and max(lens) <= 15 and abs(np.mean(lens) - 10) < 0.3
    dirs = b.field(O.F_DIR)
    assert set(np.unique(dirs)) <= {-1.0, 1.0}


def test_rollout_threads_identical():
    """The all-cores CPU baseline (OpenMP over envs) computes the same
    trajectories as the single-threaded oracle."""
    p = [0.01, 5, 15, 0.001, 0.005, 5.0, 0.15, 0.04, 0.001, 0.99]
    cfg = dict(n_envs=64, seed=5, transaction_cost_rel=0.02, slippage_rel=1e-4,
               maintenance_margin=0.25, required_margin=1.0, reward_shaper="DDR",
               adaptation_rate=0.001, unit_size=0.05, auto_reset=1)
    acts = np.random.default_rng(1).integers(0, 3, (40, 64, 3)).astype(np.int8)
    outs = []
    for threads in (1, 4):
        b = O.OracleBatch(dict(cfg), trendou_sources(3, p))
        outs.append(b.rollout(acts, threads=threads))
    for k in outs[0]:
        np.testing.assert_array_equal(outs[0][k], outs[1][k])
