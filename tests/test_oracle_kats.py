"""Pin the oracle to the reference's own known-answer tests.

Every case restates an assertion of madigan/environments/cpp/tests/envTest.py
(or envTest.cpp) with the same inputs and the same tolerance; the reference's
Synth() default source (DataSource.cpp:475-482) supplies the prices exactly as
in those tests (its first getData at x = phase).
"""
import math

import numpy as np
from numpy.testing import assert_allclose

from oracle import oracle as O
from tests.configs import sine_sources

SYNTH_DEFAULT = sine_sources([1., 0.3, 2., 0.5], [2., 2.1, 2.2, 2.3], [1., 1.2, 1.3, 1.],
                             [0., 1., 2., 1.], 0.01, 0.)


def port(reqM=1.0, mainM=0.25, cash=1_000_000, n_envs=1, **kw):
    return O.OracleBatch(dict(n_envs=n_envs, required_margin=reqM, maintenance_margin=mainM,
                              init_cash=cash, **kw), SYNTH_DEFAULT)


def synth_prices():
    PI2 = 3.141592653589793238463 * 2
    return np.array([m + a * math.sin(PI2 * p * f) for f, m, a, p in
                     zip([1., 0.3, 2., 0.5], [2., 2.1, 2.2, 2.3], [1., 1.2, 1.3, 1.], [0., 1., 2., 1.])])


def ref_transaction(units, init_cash, prices, assetIdx=0, margin=1.):
    """envTest.py:101-117 helper, verbatim arithmetic."""
    cash = init_cash
    price = prices[assetIdx]
    cost = margin * (price * units)
    cash -= cost
    borrowed_margin = (1 - margin) * (price * units)
    if borrowed_margin < 0.:
        cash -= borrowed_margin
        borrowed_margin = 0.
    equity = cash + units * (price) - borrowed_margin
    return cash, borrowed_margin, equity


def test_synth_prices_match_reference_formula():
    b = port()
    assert_allclose(b.field(O.F_PRICE)[0], synth_prices(), rtol=0, atol=1e-15)


def test_port_accounting_logic():  # envTest.py:120-145
    for units, reqM in ((1000., 1.), (-1000., 1.), (1000., .1), (-1000., .1)):
        b = port(reqM=reqM)
        prices = b.field(O.F_PRICE)[0]
        b.port_handle_transaction(0, 0, prices[0], units, 0.)
        cash, borrowed, equity = ref_transaction(units, 1_000_000, prices, 0, reqM)
        assert cash == b.scalar("cash")[0]
        assert borrowed == b.scalar("borrowedMargin")[0]
        assert equity == b.scalar("equity")[0]


def test_broker_accounting_logic():  # envTest.py:282-330
    for units, reqM in ((1000., 1.), (-1000., 1.), (1000., .1), (-1000., .1)):
        b = port(reqM=reqM)
        prices = b.field(O.F_PRICE)[0]
        b.broker_handle_transaction(0, 0, units)
        cash, borrowed, equity = ref_transaction(units, 1_000_000, prices, 0, reqM)
        assert cash == b.scalar("cash")[0]
        assert borrowed == b.scalar("borrowedMargin")[0]
        assert equity == b.scalar("equity")[0]


def test_port_ledger():  # envTest.py:148-178
    ATOL = 1e-8
    for reqM in (1., .1):
        b = port(reqM=reqM)
        prices = b.field(O.F_PRICE)[0]
        for idx, units in zip([0, 1, 2, 3], [1000, 2000, -4000, 1000]):
            b.port_handle_transaction(0, idx, prices[idx], units, 0.)
        lnf = b.ledger_normed_full()
        ln = lnf[1:]
        eq = b.scalar("equity")[0]
        cash, bm = b.scalar("cash")[0], b.scalar("borrowedMargin")[0]
        assert abs((1 - ln.sum()) * eq - (cash - bm)) < ATOL
        if reqM == 1.:
            assert abs((1 - ln.sum()) * eq - cash) < ATOL
        assert abs(lnf.sum() - 1.) < ATOL


def test_successive_accounting1():  # envTest.py:404-443
    b = port(reqM=0.1)
    p = b.field(O.F_PRICE)[0][0]
    b.port_handle_transaction(0, 0, p, 10_000)
    assert b.scalar("assetValue")[0] == p * 10_000
    b.port_handle_transaction(0, 0, p, 10_000)
    assert b.scalar("cash")[0] == 1_000_000. - 0.1 * p * 20_000
    assert b.scalar("assetValue")[0] == p * 20_000
    assert b.scalar("usedMargin")[0] == 0.1 * p * 20_000
    assert b.scalar("borrowedMargin")[0] == 0.9 * p * 20_000
    assert b.scalar("borrowedAssetValue")[0] == 0.
    b.port_handle_transaction(0, 0, p, -20_000)
    for k, v in (("cash", 1_000_000.), ("assetValue", 0.), ("usedMargin", 0.), ("borrowedMargin", 0.),
                 ("borrowedAssetValue", 0.)):
        assert_allclose(b.scalar(k)[0], v, rtol=1e-12)
    b.port_handle_transaction(0, 0, p, -20_000)
    assert_allclose(b.scalar("cash")[0], 1_000_000 + p * 20_000., rtol=1e-12)
    assert_allclose(b.scalar("assetValue")[0], p * -20_000, rtol=1e-12)
    assert_allclose(b.scalar("usedMargin")[0], 0.1 * p * 20_000, rtol=1e-12)
    assert_allclose(b.scalar("borrowedMargin")[0], 0.)
    assert_allclose(b.scalar("borrowedAssetValue")[0], p * -20_000, rtol=1e-12)
    b.port_handle_transaction(0, 0, p, 10_000)
    b.port_handle_transaction(0, 0, p, 10_000)
    for k, v in (("cash", 1_000_000.), ("assetValue", 0.), ("usedMargin", 0.), ("borrowedMargin", 0.),
                 ("borrowedAssetValue", 0.)):
        assert_allclose(b.scalar(k)[0], v, rtol=1e-12)


def test_successive_accounting2():  # envTest.py:446-458, short then reverse to long
    b = port(reqM=0.1)
    p = b.field(O.F_PRICE)[0][0]
    b.port_handle_transaction(0, 0, p, -10_000)
    b.port_handle_transaction(0, 0, p, 20_000)
    assert b.scalar("cash")[0] == 1_000_000. - 0.1 * p * 10_000
    assert b.scalar("assetValue")[0] == p * 10_000
    assert b.scalar("usedMargin")[0] == 0.1 * p * 10_000
    assert b.scalar("borrowedMargin")[0] == 0.9 * p * 10_000
    assert b.scalar("borrowedAssetValue")[0] == 0.


def test_successive_accounting3():  # envTest.py:461-472, long then reverse to short
    b = port(reqM=0.1)
    p = b.field(O.F_PRICE)[0][0]
    b.port_handle_transaction(0, 0, p, 10_000)
    b.port_handle_transaction(0, 0, p, -20_000)
    assert b.scalar("cash")[0] == 1_000_000. + p * 10_000
    assert b.scalar("assetValue")[0] == -p * 10_000
    assert b.scalar("usedMargin")[0] == 0.1 * p * 10_000
    assert b.scalar("borrowedMargin")[0] == 0.
    assert b.scalar("borrowedAssetValue")[0] == -p * 10_000


def test_multiasset_accounting():  # envTest.py:475-509
    b = port(reqM=0.1)
    prices = b.field(O.F_PRICE)[0]
    b.port_handle_transaction(0, 0, prices[0], 20_000)
    assert b.scalar("cash")[0] == 1_000_000. - 0.1 * prices[0] * 20_000
    assert b.scalar("assetValue")[0] == prices[0] * 20_000
    assert b.scalar("usedMargin")[0] == 0.1 * prices[0] * 20_000
    assert b.scalar("borrowedMargin")[0] == 0.9 * prices[0] * 20_000
    assert b.scalar("borrowedAssetValue")[0] == 0.
    b.port_handle_transaction(0, 3, prices[3], -20_000)
    expect = dict(cash=1_000_000. - (0.1 * prices[0] * 20_000) + (prices[3] * 20_000),
                  balance=1_000_000 - (0.1 * prices[0] * 20_000),
                  assetValue=prices[0] * 20_000 + prices[3] * -20_000,
                  usedMargin=0.1 * prices[0] * 20_000 + 0.1 * prices[3] * 20_000,
                  borrowedMargin=0.9 * prices[0] * 20_000,
                  borrowedAssetValue=prices[3] * -20_000)
    for k, v in expect.items():
        assert_allclose(b.scalar(k)[0], v, rtol=1e-12, err_msg=k)


def test_port_risk_handling():  # envTest.py:512-547
    b = port(reqM=0.1, mainM=1.)
    prices = b.field(O.F_PRICE)[0]
    prices[1] = 4
    b.set_field(O.F_PRICE, prices[None])
    price = 4.
    reqM = 0.1
    b.port_handle_transaction(0, 1, price, 1_000_000)

    def bp():
        return b.scalar("balance")[0] + b.scalar("pnl")[0]

    assert b.port_check_risk(0, 1, (-1. + bp() / reqM) / price) == O.GREEN
    assert b.port_check_risk(0, 1, (0. + bp() / reqM) / price) == O.INSUFF_MARGIN
    assert b.port_check_risk(0, 1, (1. + bp() / reqM) / price) == O.INSUFF_MARGIN
    prices[1] = 3.71
    b.set_field(O.F_PRICE, prices[None])
    assert b.port_check_risk(0) == O.GREEN
    assert b.port_check_risk(0, 1, 1_000_000 / price) == O.GREEN
    new_price = 3.69
    prices[1] = new_price
    b.set_field(O.F_PRICE, prices[None])
    assert b.port_check_risk(0) == O.MARGIN_CALL
    assert b.port_check_risk(0, 1, (-1. + bp() / reqM) / price) == O.MARGIN_CALL
    assert b.port_check_risk(0, 1, 0.) == O.MARGIN_CALL
    loss = 1_000_000 * (price - new_price)
    equity = 1_000_000 - loss
    assert_allclose(-loss, b.scalar("pnl")[0], rtol=1e-12)
    b.port_handle_transaction(0, 1, new_price, -1_000_000)
    assert_allclose(equity, b.scalar("equity")[0], rtol=1e-12)
    assert_allclose(equity, b.scalar("cash")[0], rtol=1e-12)


def test_broker_risk_handling():  # envTest.py:550-566
    b = port(reqM=0.1, mainM=1.)
    prices = b.field(O.F_PRICE)[0]
    prices[1] = 4
    b.set_field(O.F_PRICE, prices[None])
    tp, tu, tc, risk = b.broker_handle_transaction(0, 1, 1_000_000)
    assert tp == 4 and tc == 0. and risk == O.GREEN and tu == 1_000_000


def test_opposite_sign_quirk():
    """Portfolio.cpp:257-265: a long->short over-sale is green
    without any margin test, a short->long over-cover is margin checked."""
    b = port(reqM=0.1, mainM=1.)
    p = b.field(O.F_PRICE)[0][0]
    b.port_handle_transaction(0, 0, p, 10_000)
    huge = 1e12
    assert b.port_check_risk(0, 0, -huge) == O.GREEN           # u <= -cur: unchecked
    b2 = port(reqM=0.1, mainM=1.)
    b2.port_handle_transaction(0, 0, p, -10_000)
    assert b2.port_check_risk(0, 0, huge) == O.INSUFF_MARGIN   # u > -cur: checked


def test_transaction_cost_uses_pre_slippage_price():  # Broker.cpp:130-131 (quirk 8)
    b = port(reqM=1.0, slippage_rel=0.01, transaction_cost_rel=0.02)
    p = b.field(O.F_PRICE)[0][1]
    tp, tu, tc, risk = b.broker_handle_transaction(0, 1, 100.)
    assert tp == p + (p * 0.01 + 0.0)
    assert tc == abs(100. * p) * 0.02 + 0.0


def test_env_step_reward_and_done():  # Env.h:206-230
    b = port(reqM=1.0, mainM=0.25)
    eq0 = b.scalar("equity")[0]
    o = b.step(np.array([[10_000, 20_000, -20_000, -40_000]], float))
    eq1 = b.scalar("equity")[0]
    assert o["reward"][0] == math.log(max(eq1 / eq0, 0.3))
    assert o["done"][0] == 0
    assert list(o["risk"][0]) == [O.GREEN] * 4
    # single-asset overload clamps at 0.01 (Env.h:238)
    o = b.step(np.array([1e9]), np.array([0], np.int32))
    assert o["risk"][0][0] == O.INSUFF_MARGIN and o["done"][0] == 0


def test_env_equity_floor_done():  # Env.h:221-223: equity < 0.1 * initCash
    b = port(reqM=1.0, mainM=0.0)
    b.set_cash(np.array([50_000.]))
    o = b.step()
    assert o["done"][0] == 1


def test_reset_restores_accounting():  # Env.h:181-187
    b = port(reqM=0.1)
    b.step(np.array([[1000., 0, 0, 0]]))
    ts = b.scalar("timestamp")[0]
    b.reset()
    assert b.scalar("cash")[0] == 1_000_000
    assert not b.field(O.F_LEDGER).any()
    assert b.scalar("timestamp")[0] == ts + 1  # reset ticks the source once (Env.h:160)


def test_broker_close_kat():  # Broker.cpp:160-169 (bound at env.cpp:825-829)
    """Broker::close(assetIdx): the position closed at the current price with
    slippage and transaction cost applied as for an order, always green; the
    closed form below follows Portfolio.cpp:284-323 statement by statement."""
    sr, tc = 1e-4, 0.02
    for units in (1000., -1000.):
        b = port(reqM=1.0, slippage_rel=sr, transaction_cost_rel=tc)
        P = b.field(O.F_PRICE)[0][0]
        tp1, u1, c1, r1 = b.broker_handle_transaction(0, 0, units)
        slip = P * sr + 0.0
        assert tp1 == (P - slip if units < 0 else P + slip) and u1 == units and r1 == O.GREEN
        assert c1 == abs(units * P) * tc + 0.0
        cash1 = 1_000_000 - ((tp1 * units) * 1.0 + c1)
        assert b.scalar("cash")[0] == cash1
        tp2, u2, c2, r2 = b.broker_close(0, 0)
        cu = -units
        assert u2 == cu and r2 == O.GREEN
        assert tp2 == (P - slip if cu < 0 else P + slip)
        assert c2 == abs(P * cu) * tc + 0.0
        amt = tp2 * cu
        assert b.scalar("cash")[0] == cash1 - (amt * 1.0 + c2)
        assert b.field(O.F_LEDGER)[0][0] == 0.0 and b.field(O.F_MEP)[0][0] == 0.0
        # closing a flat position moves nothing and still answers green
        tp3, u3, c3, r3 = b.broker_close(0, 0)
        assert u3 == 0.0 and r3 == O.GREEN and b.scalar("cash")[0] == cash1 - (amt * 1.0 + c2)


def test_port_close_kat():  # Portfolio.cpp:327-333
    b = port(reqM=.1)
    P = b.field(O.F_PRICE)[0]
    b.port_handle_transaction(0, 2, P[2], -4000., 0.)
    b.port_close(0, 2, P[2] * 1.01, 5.0)
    assert b.field(O.F_LEDGER)[0][2] == 0.0
    assert b.field(O.F_BORROWED)[0][2] == 0.0
