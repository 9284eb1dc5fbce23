"""HDF replay DataSource on the CPU: the reader / writer (libmadigan_hdf.so),
HDFSourceSingle's time bounds and cache walk against the reference's own
known answers (madigan/environments/cpp/tests/envTest.cpp:319-400) and against
the oracle's restatement (oracle/oracle.py hdf_bounds, the C oracle's
iterCache), and the replay tape's visiting order."""
import numpy as np
import pytest

from madigan_amd import HDFSourceSingle, write_hdf
from madigan_amd.hdf import HDFFile
from oracle import oracle as O

KEYS = dict(price_key="midprice", feature_key="feats", timestamp_key="timestamp")


def kat_file(tmp_path):
    """testHDFSourceSingle's fixture (envTest.cpp:322-351): price i, feats i^3,
    timestamps i^2, 10 rows, one asset "Test", group "group/dataset"."""
    path = str(tmp_path / "test_envTest.h5")
    i = np.arange(10)
    write_hdf(path, "group/dataset", ["Test"], i.astype(float), (i ** 3).astype(float).reshape(-1, 1),
              (i * i).astype(np.uint64), **KEYS)
    return path


def src(path, cache, start=0, end=0):
    return HDFSourceSingle(path, "group/dataset", "midprice", "feats", "timestamp", cache, start, end)


def test_reference_kat(tmp_path):
    path = kat_file(tmp_path)
    ds = src(path, 10)
    for _ in range(3):
        ds.getData()
    assert ds.currentPrices().tolist() == [2.0]          # envTest.cpp:381-383
    assert ds.currentData().tolist() == [8.0]
    assert [a.code for a in ds.assets] == ["Test"]
    assert (ds.startTime, ds.endTime) == (0, 81)
    assert ds.boundsIdx == (0, 9)
    ds2 = src(path, 10, 1, 63)                            # envTest.cpp:386-397
    for _ in range(3):
        ds2.getData()
    assert ds2.boundsIdx == (1, 7)
    assert ds2.currentPrices().tolist() == [3.0] and ds2.currentData().tolist() == [27.0]
    with pytest.raises(IndexError):                       # envTest.cpp:399-409
        src(path, 10, 0, 82)


def test_reader_roundtrip_and_layout(tmp_path):
    rng = np.random.default_rng(1)
    T, A, F = 37, 3, 5
    price = rng.normal(10, 1, (T, A))
    feats = rng.normal(0, 1, (T, F))
    ts = np.cumsum(rng.integers(1, 9, T)).astype(np.uint64)
    path = str(tmp_path / "m.h5")
    write_hdf(path, "fx/daily", ["A", "BB", "CCC"], price, feats, ts, **KEYS)
    f = HDFFile(path, "fx/daily", "midprice", "feats", "timestamp")
    assert (f.n_assets, f.n_feats, f.info.n_rows, f.info.price_1d) == (A, F, T, 0)
    assert f.asset_codes == ["A", "BB", "CCC"]
    p, x, t = f.read(5, 20)
    assert np.array_equal(p, price[5:25]) and np.array_equal(x, feats[5:25])
    assert np.array_equal(t, ts[5:25])
    with pytest.raises(IndexError):
        f.read(30, 10)


def test_missing_keys_raise_config_error(tmp_path):
    path = kat_file(tmp_path)
    with pytest.raises(RuntimeError, match="not found"):
        HDFSourceSingle(path, "group/dataset", "nope", "feats", "timestamp", 5)
    with pytest.raises(RuntimeError, match="not found"):
        HDFSourceSingle(path, "group/other", "midprice", "feats", "timestamp", 5)
    with pytest.raises(RuntimeError, match="Missing keys"):
        HDFSourceSingle({"filepath": path, "group_key": "group/dataset"})


@pytest.mark.parametrize("seed", range(6))
def test_time_bounds_match_restatement(tmp_path, seed):
    rng = np.random.default_rng(seed)
    T = int(rng.integers(5, 200))
    ts = np.cumsum(rng.integers(1, 5, T)).astype(np.uint64)
    path = str(tmp_path / "b.h5")
    write_hdf(path, "g", ["X"], np.arange(T, dtype=float), np.zeros((T, 1)), ts, **KEYS)
    for _ in range(20):
        a, b = sorted(int(v) for v in rng.integers(int(ts[0]), int(ts[-1]) + 1, 2))
        try:
            want = O.hdf_bounds(ts, a, b)
        except (IndexError, ValueError) as e:
            with pytest.raises(type(e)):
                HDFFile(path, "g", "midprice", "feats", "timestamp", a, b)
            continue
        if want[1] <= want[0]:  # empty range: undefined in the reference, rejected here
            with pytest.raises(ValueError):
                HDFFile(path, "g", "midprice", "feats", "timestamp", a, b)
            continue
        f = HDFFile(path, "g", "midprice", "feats", "timestamp", a, b)
        assert (f.info.first, f.info.second, f.info.start_time, f.info.end_time) == want


@pytest.mark.parametrize("cache,bounds", [(10, (0, 0)), (3, (0, 0)), (4, (0, 0)), (5, (0, 0)),
                                          (1, (0, 0)), (2, (1, 63)), (4, (4, 81))])
def test_tape_is_one_period_of_the_cache_walk(tmp_path, cache, bounds):
    path = kat_file(tmp_path)
    f = HDFFile(path, "group/dataset", "midprice", "feats", "timestamp", *bounds)
    rows = f.tape_index(cache)
    # the host HDFSourceSingle walk, 3 periods
    ds = src(path, cache, *bounds)
    seen = []
    for _ in range(3 * len(rows)):
        ds.getData()
        seen.append(int(ds.currentPrices()[0]))   # price i == row i
    assert seen == list(rows) * 3
    first, second = f.bounds
    assert rows[0] == first and rows[-1] <= second - 1 and np.all(np.diff(rows) == 1)
    # the oracle's C restatement of iterCache over the same arrays
    i = np.arange(10)
    orc = O.OracleBatch(dict(n_envs=1, n_feats=1), [(O.SRC_REPLAY, [])])
    period = orc.set_replay(i.astype(float), (i ** 3).astype(float), (i * i).astype(np.uint64),
                            first, second, cache)
    assert period == len(rows)
    got = [int(orc.step()["obs_price"][0, 0]) for _ in range(2 * period)]
    # the constructor consumed tape row 0; steps continue from row 1
    want = [int(r) ** 3 for r in (list(rows) * 3)[1:2 * period + 1]]
    assert got == want


def test_skip_quirk_period(tmp_path):
    """A refill that starts at second - 1 rewinds (DataSource.cpp:369): with
    bounds (0, 9) and cacheSize 4 the chunks are [0,4), [4,8) and row 8 is
    never served."""
    path = kat_file(tmp_path)
    f = HDFFile(path, "group/dataset", "midprice", "feats", "timestamp")
    assert f.bounds == (0, 9)
    assert f.tape_index(4).tolist() == list(range(8))
    assert f.tape_index(3).tolist() == list(range(9))


def test_adjust_config_datetimes():
    import pandas as pd
    from madigan_amd.env import adjust_config
    cfg = {"data_source_type": "HDFSourceSingle",
           "data_source_config": {"start_time": "1995-01-03", "end_time": "2015-01-01"},
           "data_source_config_test": {"start_time": "2015-01-01", "end_time": "2020-10-01"}}
    a = adjust_config(cfg)
    assert a["data_source_config"]["start_time"] == pd.to_datetime("1995-01-03").value
    t = adjust_config(cfg, test=True)
    assert t["data_source_config"]["end_time"] == pd.to_datetime("2020-10-01").value
    assert cfg["data_source_config"]["start_time"] == "1995-01-03"  # deep copy
