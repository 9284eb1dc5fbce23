"""C1 on the GPU: the drop-in ``madigan_amd.Env`` (one env, N = 1 view of the
batched handle) run through the reference's own known-answer tests and Python
surface.

The accounting KATs of madigan/environments/cpp/tests/envTest.py:101-566 are
written against a Portfolio / Broker holding a fixed price vector.  Here the
same transactions go through ``Env.step(assetIdx, units)`` /
``Env.step(assetCode, units)`` / ``Env.step(units)`` on the GPU, with the
prices held fixed between ticks in one of two ways:
  * "synth": the device Synth generator of envTest.py:11-21 with dX = 0 (its
    price never moves: p = mu + amp sin(2 pi phase freq));
  * "host": a host DataSourceTick subclass whose getData() returns a price
    vector the test controls, plugged in with Env.setDataSource (Env.h:174-179,
    PyDataSource.h:9-15) -- the route the risk KATs (envTest.py:512-566) need,
    since they move prices between checks.
Expected values are the reference's own closed forms with its tolerances.
The four step overloads, reset() -> State and setDataSource mid-episode are
also checked against the oracle step by step.
"""
import math

import numpy as np
import pytest
from numpy.testing import assert_allclose

from oracle import oracle as O
from tests.configs import sine_sources

pytestmark = pytest.mark.gpu

FREQ, MU, AMP, PHASE = [1., 0.3, 2., 0.5], [2., 2.1, 2.2, 2.3], [1., 1.2, 1.3, 1.], [0., 1., 2., 1.]
PI2 = 3.141592653589793238463 * 2
SYNTH_PRICES = np.array([m + a * math.sin(PI2 * p * f) for f, m, a, p in zip(FREQ, MU, AMP, PHASE)])


def synth_cfg(dX=0.0, noise=0.0):
    return {"data_source_type": "Synth",
            "data_source_config": {"freq": FREQ, "mu": MU, "amp": AMP, "phase": PHASE, "dX": dX,
                                   "noise": noise}}


class HostPrices:
    """A host DataSourceTick (DataSource.h:48-64) whose prices the test sets."""

    def __new__(cls, prices):
        from madigan_amd import DataSourceTick

        class _Src(DataSourceTick):
            def __init__(self, p):
                self.p = np.array(p, dtype=np.float64)
                self.t = 0
                self.calls = 0

            def getData(self):
                self.calls += 1
                self.t += 1
                return self.p

            def currentPrices(self):
                return self.p

            def currentTime(self):
                return self.t
        return _Src(prices)


def make(route, reqM=1.0, mainM=0.25, prices=None):
    from madigan_amd import Env
    env = Env("Synth", 1_000_000, synth_cfg())
    env.setRequiredMargin(reqM)
    env.setMaintenanceMargin(mainM)
    src = None
    if route == "host":
        src = HostPrices(SYNTH_PRICES if prices is None else prices)
        env.setDataSource(src)
    return env, src


def ref_transaction(units, init_cash, prices, assetIdx=0, margin=1.):
    """envTest.py:101-117 (transaction helper), same arithmetic."""
    cash = init_cash
    price = prices[assetIdx]
    cost = margin * (price * units)
    cash -= cost
    borrowed_margin = (1 - margin) * (price * units)
    if borrowed_margin < 0.:
        cash -= borrowed_margin
        borrowed_margin = 0.
    equity = cash + units * price - borrowed_margin
    return cash, borrowed_margin, equity


ROUTES = ["synth", "host"]


@pytest.mark.parametrize("route", ROUTES)
def test_env_prices_are_the_reference_synth(gpu, route):
    env, _ = make(route)
    assert_allclose(env.currentPrices, SYNTH_PRICES, rtol=0, atol=1e-15)
    env.step()
    assert_allclose(env.currentPrices, SYNTH_PRICES, rtol=0, atol=1e-15)


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("overload", ["index", "vector"])
def test_env_accounting_logic(gpu, route, overload):
    """envTest.py:120-145 (Portfolio) and :303-330 (Broker): one buy / sell on
    cash and on 10 % margin; cash, borrowed margin and equity exactly equal."""
    for units, reqM in ((1000., 1.), (-1000., 1.), (1000., .1), (-1000., .1)):
        env, _ = make(route, reqM=reqM)
        prices = env.currentPrices
        if overload == "index":
            _, _, _, info = env.step(0, units)
        else:
            _, _, _, info = env.step(np.array([units, 0., 0., 0.]))
        r = info.brokerResponse
        risk = r.riskInfo if overload == "index" else r.riskInfo[0]
        assert int(risk) == O.GREEN
        cash, borrowed, equity = ref_transaction(units, 1_000_000, prices, 0, reqM)
        assert env.cash == cash
        assert env.borrowedMargin == borrowed
        assert env.equity == equity


@pytest.mark.parametrize("route", ROUTES)
def test_env_ledger_normed(gpu, route):
    """envTest.py:148-178: ledgerNormed(Full) identities after four orders."""
    ATOL = 1e-8
    for reqM in (1., .1):
        env, _ = make(route, reqM=reqM)
        env.step(np.array([1000., 2000., -4000., 1000.]))
        lnf = env.ledgerNormedFull
        ln = env.ledgerNormed
        eq = env.equity
        assert abs((1 - ln.sum()) * eq - (env.cash - env.borrowedMargin)) < ATOL
        if reqM == 1.:
            assert abs((1 - ln.sum()) * eq - env.cash) < ATOL
        assert abs(lnf.sum() - 1.) < ATOL
        assert_allclose(lnf[1:], ln, rtol=1e-15)


@pytest.mark.parametrize("route", ROUTES)
def test_env_successive_accounting1(gpu, route):
    """envTest.py:404-443: buy, buy, sell to flat, sell short, buy back."""
    env, _ = make(route, reqM=0.1)
    p = env.currentPrices[0]
    env.step(0, 10_000)
    assert env.assetValue == p * 10_000
    env.step(0, 10_000)
    assert env.cash == 1_000_000. - 0.1 * p * 20_000
    assert env.assetValue == p * 20_000
    assert env.usedMargin == 0.1 * p * 20_000
    assert env.borrowedMargin == 0.9 * p * 20_000
    assert env.borrowedAssetValue == 0.
    env.step(0, -20_000)
    for k, v in (("cash", 1_000_000.), ("assetValue", 0.), ("usedMargin", 0.), ("borrowedMargin", 0.),
                 ("borrowedAssetValue", 0.)):
        assert_allclose(getattr(env, k), v, rtol=1e-12, err_msg=k)
    env.step(0, -20_000)
    assert_allclose(env.cash, 1_000_000 + p * 20_000., rtol=1e-12)
    assert_allclose(env.assetValue, p * -20_000, rtol=1e-12)
    assert_allclose(env.usedMargin, 0.1 * p * 20_000, rtol=1e-12)
    assert_allclose(env.borrowedMargin, 0.)
    assert_allclose(env.borrowedAssetValue, p * -20_000, rtol=1e-12)
    env.step(0, 10_000)
    env.step(0, 10_000)
    for k, v in (("cash", 1_000_000.), ("assetValue", 0.), ("usedMargin", 0.), ("borrowedMargin", 0.),
                 ("borrowedAssetValue", 0.)):
        assert_allclose(getattr(env, k), v, rtol=1e-12, err_msg=k)


@pytest.mark.parametrize("route", ROUTES)
def test_env_successive_accounting2_and_3(gpu, route):
    """envTest.py:446-472: reversals short -> long and long -> short."""
    env, _ = make(route, reqM=0.1)
    p = env.currentPrices[0]
    env.step(0, -10_000)
    env.step(0, 20_000)
    assert env.cash == 1_000_000. - 0.1 * p * 10_000
    assert env.assetValue == p * 10_000
    assert env.usedMargin == 0.1 * p * 10_000
    assert env.borrowedMargin == 0.9 * p * 10_000
    assert env.borrowedAssetValue == 0.
    env, _ = make(route, reqM=0.1)
    env.step(0, 10_000)
    env.step(0, -20_000)
    assert env.cash == 1_000_000. + p * 10_000
    assert env.assetValue == -p * 10_000
    assert env.usedMargin == 0.1 * p * 10_000
    assert env.borrowedMargin == 0.
    assert env.borrowedAssetValue == -p * 10_000


@pytest.mark.parametrize("route", ROUTES)
def test_env_multiasset_accounting(gpu, route):
    """envTest.py:475-509, orders addressed by asset code (step(assetCode, units))."""
    env, _ = make(route, reqM=0.1)
    prices = env.currentPrices
    codes = [a.code for a in env.assets]
    env.step(codes[0], 20_000)
    assert env.cash == 1_000_000. - 0.1 * prices[0] * 20_000
    assert env.assetValue == prices[0] * 20_000
    assert env.usedMargin == 0.1 * prices[0] * 20_000
    assert env.borrowedMargin == 0.9 * prices[0] * 20_000
    assert env.borrowedAssetValue == 0.
    env.step(codes[3], -20_000)
    expect = dict(cash=1_000_000. - (0.1 * prices[0] * 20_000) + (prices[3] * 20_000),
                  balance=1_000_000 - (0.1 * prices[0] * 20_000),
                  assetValue=prices[0] * 20_000 + prices[3] * -20_000,
                  usedMargin=0.1 * prices[0] * 20_000 + 0.1 * prices[3] * 20_000,
                  borrowedMargin=0.9 * prices[0] * 20_000,
                  borrowedAssetValue=prices[3] * -20_000)
    for k, v in expect.items():
        assert_allclose(getattr(env, k), v, rtol=1e-12, err_msg=k)
    with pytest.raises(IndexError):
        env.step("NOT_AN_ASSET", 1.0)
    with pytest.raises(IndexError):
        env.step(7, 1.0)
    with pytest.raises(ValueError):
        env.step(np.ones(3))


def test_env_risk_handling(gpu):
    """envTest.py:512-547 through Env: asset 1 priced 4, bought 1e6 units on 10 %
    margin; order checks at the insuff_margin threshold; the price drops to
    3.71 (green) then 3.69 (margin call); closing at 3.69 leaves cash = equity
    = 1e6 - loss.  The prices move through a host DataSourceTick.  (The
    reference's checkRisk("ETHUSD", 0.) is a Portfolio-level probe: a zero
    order never reaches the risk check through the Broker, Broker.cpp:126.)"""
    reqM, mainM, price = 0.1, 1., 4.
    start = SYNTH_PRICES.copy()
    start[1] = price

    def setup():
        env, src = make("host", reqM=reqM, mainM=mainM, prices=start)
        _, _, done, info = env.step(1, 1_000_000)
        assert int(info.brokerResponse.riskInfo) == O.GREEN and not done
        return env, src

    env, src = setup()
    bp = env.balance + env.pnl
    ledger0, cash0 = env.ledger, env.cash
    # green probe on a replica (a green order executes)
    env2, _ = setup()
    _, _, _, info = env2.step(1, (-1. + bp / reqM) / price)
    assert int(info.brokerResponse.riskInfo) == O.GREEN
    for units in ((0. + bp / reqM) / price, (1. + bp / reqM) / price):
        _, _, done, info = env.step(1, units)
        assert int(info.brokerResponse.riskInfo) == O.INSUFF_MARGIN and not done
        assert info.brokerResponse.transactionUnits == 0.0
    assert np.array_equal(env.ledger, ledger0) and env.cash == cash0
    src.p[1] = 3.71
    env.step()
    assert int(env.checkRisk()) == O.GREEN
    env3, src3 = setup()
    src3.p[1] = 3.71
    env3.step()
    _, _, _, info = env3.step(1, 1_000_000 / price)
    assert int(info.brokerResponse.riskInfo) == O.GREEN
    new_price = 3.69
    src.p[1] = new_price
    _, _, done, _ = env.step()
    assert done  # Env.h:196-197: checkRisk() != green
    assert int(env.checkRisk()) == O.MARGIN_CALL
    bp = env.balance + env.pnl
    _, _, done, info = env.step(1, (-1. + bp / reqM) / price)
    assert int(info.brokerResponse.riskInfo) == O.MARGIN_CALL and done
    loss = 1_000_000 * (price - new_price)
    equity = 1_000_000 - loss
    assert_allclose(-loss, env.pnl, rtol=1e-12)
    env.step(1, -1_000_000)
    assert_allclose(equity, env.equity, rtol=1e-12)
    assert_allclose(equity, env.cash, rtol=1e-12)


def test_env_broker_risk_handling(gpu):
    """envTest.py:550-566: the response of a green order at price 4."""
    start = SYNTH_PRICES.copy()
    start[1] = 4.
    env, _ = make("host", reqM=0.1, mainM=1., prices=start)
    codes = [a.code for a in env.assets]
    _, _, _, info = env.step(codes[1], 1_000_000)
    r = info.brokerResponse
    assert r.transactionPrice == 4
    assert r.transactionCost == 0.
    assert r.transactionUnits == 1_000_000
    assert int(r.riskInfo) == O.GREEN


def _c1_pair(seed):
    from madigan_amd import Env
    cfg = {"data_source_type": "Synth",
           "data_source_config": {"freq": [1.0], "mu": [2.0], "amp": [1.0], "phase": [0.0],
                                  "dX": 0.01, "noise": 0.0}}
    env = Env("Synth", 1_000_000.0, cfg, seed=seed)
    env.setRequiredMargin(1.0)
    env.setMaintenanceMargin(0.25)
    orc = O.OracleBatch(dict(n_envs=1, seed=seed, required_margin=1.0, maintenance_margin=0.25),
                        sine_sources([1.0], [2.0], [1.0], [0.0], 0.01, 0.0))
    return env, orc


def _check_srdi(srdi, ref, what, single=None):
    state, reward, done, info = srdi
    assert np.array_equal(state.price.view(np.int64), ref["obs_price"][0].view(np.int64)), what
    assert np.array_equal(state.portfolio.view(np.int64), ref["obs_port"][0].view(np.int64)), what
    assert state.timestamp == int(ref["timestamp"][0]), what
    assert_allclose(reward, ref["reward"][0], rtol=1e-12, err_msg=what)
    assert done == bool(ref["done"][0]), what
    r = info.brokerResponse
    if single is None:
        assert np.array_equal(np.asarray(r.transactionPrice), ref["tprice"][0]), what
        assert np.array_equal(np.asarray(r.transactionUnits), ref["tunits"][0]), what
        assert [int(x) for x in r.riskInfo] == list(ref["risk"][0]), what
    else:
        assert r.transactionPrice == ref["tprice"][0, single], what
        assert r.transactionCost == ref["tcost"][0, single], what
        assert int(r.riskInfo) == ref["risk"][0, single], what
    assert r.marginCall == bool(ref["margin_call"][0]), what
    assert info.dataEnd is False


def test_c1_step_overloads_vs_oracle(gpu):
    """C1 (BASELINE configs[0]): 1 env x 1-asset Sine, env log reward; 300
    steps cycling step(), step(units), step(assetIdx, units), step(assetCode,
    units) and two reset()s, every State / reward / done / EnvInfo against the
    oracle (prices and portfolio bit-exact, reward rtol 1e-12)."""
    env, orc = _c1_pair(5)
    rng = np.random.default_rng(0)
    code = env.assets[0].code
    for t in range(300):
        u = float(rng.integers(-3, 4)) * 5_000.
        kind = t % 4
        if t in (97, 211):
            s = env.reset()
            orc.reset()
            assert np.array_equal(s.price, orc.field(O.F_PRICE)[0]) and s.timestamp == int(
                orc.scalar("timestamp")[0])
            assert_allclose(s.portfolio, orc.ledger_normed_full(0), rtol=0)
            continue
        if kind == 0:
            _check_srdi(env.step(), orc.step(), f"t={t} step()", single=0)
        elif kind == 1:
            _check_srdi(env.step(np.array([u])), orc.step(np.array([[u]])), f"t={t} step(units)")
        elif kind == 2:
            _check_srdi(env.step(0, u), orc.step(np.array([u]), np.array([0], np.int32)),
                        f"t={t} step(i,u)", single=0)
        else:
            _check_srdi(env.step(code, u), orc.step(np.array([u]), np.array([0], np.int32)),
                        f"t={t} step(code,u)", single=0)
        assert env.cash == orc.scalar("cash")[0]
        assert env.equity == orc.scalar("equity")[0]
        assert np.array_equal(env.ledger, orc.field(O.F_LEDGER)[0])
    from madigan_amd import get_env_info
    info = get_env_info(env)
    assert info["equity"] == env.equity and info["timestamp"] == env.timestamp


def test_set_data_source_mid_episode_keeps_portfolio(gpu):
    """Env.setDataSource after 25 steps on the device OU source: the ledger,
    cash, mean entry and borrowed margin survive (Env.h:174-179 keeps the
    Broker), the portfolio is revalued at the new source's currentPrices(),
    and from then on every tick's prices come from the host source's
    getData().  The oracle receives the identical price path."""
    from madigan_amd import Env
    from tests.configs import ou_sources
    cfg = {"data_source_type": "OU", "data_source_config": {"mean": [10.] * 4, "theta": [.08] * 4,
                                                            "phi": [.04] * 4}}
    env = Env("OU", 1_000_000, cfg, seed=77)
    env.setRequiredMargin(0.2)
    env.setMaintenanceMargin(0.25)
    orc = O.OracleBatch(dict(n_envs=1, seed=77, required_margin=0.2, maintenance_margin=0.25),
                        ou_sources(4))
    rng = np.random.default_rng(4)
    for t in range(25):
        u = rng.normal(0, 5e3, 4)
        _check_srdi(env.step(u), orc.step(u[None]), f"pre t={t}")
    ledger, cash, mep = env.ledger, env.cash, env.meanEntryPrices
    assert np.count_nonzero(ledger) > 0
    path = 10.0 + np.cumsum(rng.normal(0, 0.05, (41, 4)), axis=0)

    from madigan_amd import DataSourceTick

    class Path(DataSourceTick):
        def __init__(self):
            self.i = 0

        def getData(self):
            self.i += 1
            return path[self.i]

        def currentPrices(self):
            return path[self.i]

    src = Path()
    env.setDataSource(src)
    orc.set_sources([(O.SRC_EXTERNAL, [])] * 4, path[0][None])
    assert np.array_equal(env.ledger, ledger) and env.cash == cash
    assert np.array_equal(env.meanEntryPrices, mep)
    assert np.array_equal(env.currentPrices, path[0])
    assert env.equity == orc.scalar("equity")[0]
    assert env.dataSource is src
    for t in range(40):
        u = rng.normal(0, 5e3, 4)
        orc.set_prices(path[t + 1][None])
        _check_srdi(env.step(u), orc.step(u[None]), f"post t={t}")
        assert np.array_equal(env.currentPrices, path[t + 1])
        assert np.array_equal(env.ledger.view(np.int64), orc.field(O.F_LEDGER)[0].view(np.int64))
    with pytest.raises(ValueError):
        env.setDataSource(HostPrices([1.0, 2.0]))


def test_batched_host_source_n_envs(gpu):
    """A host source for N envs (mgn_set_sources + mgn_set_prices): 96 envs
    switched from TrendOU to host prices mid-run keep their portfolios and then
    follow the host path bit-exactly against the oracle."""
    from tests.test_gpu_parity import make_pair, out_check, state_check
    from tests.configs import TRENDOU_P, trendou_sources, spec_from_sources
    N, A = 96, 4
    g, orc = make_pair(trendou_sources(A, [0.05] + TRENDOU_P[1:]), N, required_margin=0.5,
                       maintenance_margin=0.25, transaction_cost_rel=0.01, seed=3)
    rng = np.random.default_rng(8)
    for t in range(12):
        u = rng.normal(0, 2e3, (N, A))
        g.step(u)
        orc.step(u)
    state_check(g, orc, "pre")
    ext = [(O.SRC_EXTERNAL, [])] * A
    p0 = 5.0 + rng.random((N, A))
    g.set_sources(spec_from_sources(ext), p0)
    orc.set_sources(ext, p0)
    state_check(g, orc, "switched")
    for t in range(20):
        p = 5.0 + rng.random((N, A))
        g.set_prices(p)
        orc.set_prices(p)
        u = rng.normal(0, 2e3, (N, A))
        g.step(u)
        ref = orc.step(u)
        out_check(g.host_outputs(), ref, f"host t={t}")
        state_check(g, orc, f"host t={t}")
    with pytest.raises(RuntimeError):  # only EXTERNAL or the same kind
        g.set_sources(spec_from_sources([(O.SRC_OU, [10., .1, .04])] * A))
