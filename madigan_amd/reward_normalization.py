"""Streaming reward normalisers: madigan/environments/reward_normalization.pyx.

The reference's Cython classes transform a stream of (log-return) rewards by a
rolling estimate of their spread -- one object per environment, one scalar per
call.  These keep the same names, constructors, ``from_config`` /
``make_reward_normalizer`` entry points and ``reset()`` / ``stream()``
methods, and batch over environments: ``stream`` takes a float (one env, as
the reference) or an (N,) array (N envs, each with its own window and
estimates), ``reset`` an optional boolean env mask (the envs whose episode
ended).  Every env's arithmetic is the reference's, statement by statement, in
float64 (numpy element-wise operations are IEEE binary64 like the Cython's C
doubles), so the outputs match the compiled reference bit for bit
(tests/test_reward_normalization.py against tests/golden/reward_norm_vectors.npz,
generated from the reference built by ``make -C oracle ref_normalizers``).

Host-side agent plumbing (the reference calls these from the agent, off the
env step): numpy, no device work.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

__all__ = ["make_reward_normalizer", "RewardShaper", "NullShaper", "SharpeFixedWindow",
           "SortinoFixedWindowA", "SortinoFixedWindowB", "SortinoFixedWindowC", "SharpeEWMA"]


def make_reward_normalizer(config, n_envs: Optional[int] = None):
    """reward_normalization.pyx:14-22: config['reward_shaper_config'] names the
    class ('None' / 'none' / None: NullShaper)."""
    conf = config["reward_shaper_config"]
    name = conf["reward_shaper"]
    if name in ("None", "none", None):
        return NullShaper()
    cls = _CLASSES.get(name)
    if cls is None:
        raise NotImplementedError(f"reward_shaper {name} has not been implemented")
    return cls.from_config(conf, n_envs)


class RewardShaper:
    """reward_normalization.pyx:25-47: running estimates of a reward stream."""

    @classmethod
    def from_config(cls, config, n_envs: Optional[int] = None):
        raise NotImplementedError

    def reset(self, mask=None):
        raise NotImplementedError

    def stream(self, reward):
        raise NotImplementedError


class NullShaper(RewardShaper):
    """reward_normalization.pyx:50-58."""

    @classmethod
    def from_config(cls, config, n_envs: Optional[int] = None):
        return cls()

    def reset(self, mask=None):
        pass

    def stream(self, reward):
        return reward


class _Batch:
    """The env batch of a windowed normaliser: a scalar call is a batch of one."""

    def __init__(self, window: int, n_envs: Optional[int]):
        self.window = int(window)
        self.scalar = n_envs is None
        self.N = 1 if n_envs is None else int(n_envs)
        # std::queue<double> per env as a ring of `window` slots
        self.buf = np.zeros((self.N, max(self.window, 1)), dtype=np.float64)
        self.head = np.zeros(self.N, dtype=np.int64)  # front (oldest) slot
        self.size = np.zeros(self.N, dtype=np.int64)

    def _in(self, reward):
        r = np.asarray(reward, dtype=np.float64)
        if self.scalar:
            if r.ndim != 0:
                raise ValueError("this normaliser streams one env (built with n_envs=None)")
            return r.reshape(1)
        if r.shape != (self.N,):
            raise ValueError(f"reward must be ({self.N},), got {r.shape}")
        return r

    def _out(self, v):
        return float(v[0]) if self.scalar else v

    def _mask(self, mask):
        if mask is None:
            return np.ones(self.N, dtype=bool)
        m = np.asarray(mask, dtype=bool).reshape(-1)
        if m.shape != (self.N,):
            raise ValueError(f"mask must be ({self.N},)")
        return m

    def _push(self, idx, value):
        slot = (self.head[idx] + self.size[idx]) % self.window
        self.buf[idx, slot] = value[idx]
        self.size[idx] += 1

    def _pop(self, idx):
        front = self.buf[idx, self.head[idx]]
        self.head[idx] = (self.head[idx] + 1) % self.window
        self.size[idx] -= 1
        return front


class SharpeFixedWindow(_Batch, RewardShaper):
    """reward_normalization.pyx:61-118: reward / sqrt((ssq + 1e-8) / size) with
    a rolling-window (Welford add / remove) mean and sum of squares; 0 while
    the window holds <= 1 reward."""

    def __init__(self, window: int, n_envs: Optional[int] = None):
        _Batch.__init__(self, window, n_envs)
        self.mean_est = np.zeros(self.N, dtype=np.float64)
        self.ssq = np.zeros(self.N, dtype=np.float64)
        self.reset()

    @classmethod
    def from_config(cls, config, n_envs: Optional[int] = None):
        return cls(config["window"], n_envs)

    def reset(self, mask=None):
        m = self._mask(mask)
        self.size[m] = 0
        self.head[m] = 0
        self.mean_est[m] = 0.
        self.ssq[m] = 0.

    def _head_add(self, value, idx):  # :105-110
        self._push(idx, value)
        delt = value[idx] - self.mean_est[idx]
        self.mean_est[idx] += delt / self.size[idx].astype(np.float64)
        self.ssq[idx] += delt * (value[idx] - self.mean_est[idx])

    def _tail_adjust(self, idx):  # :112-118
        remove = self._pop(idx)
        delt = remove - self.mean_est[idx]
        self.mean_est[idx] -= delt / self.size[idx].astype(np.float64)
        self.ssq[idx] -= delt * (remove - self.mean_est[idx])

    def _update(self, r):
        full = np.nonzero(self.size == self.window)[0]
        if full.size:
            self._tail_adjust(full)
        self._head_add(r, np.arange(self.N))

    def _scaled(self, r):
        return r / np.sqrt((self.ssq + 1e-8) / self.size.astype(np.float64))

    def stream(self, reward):  # :95-103
        r = self._in(reward)
        self._update(r)
        with np.errstate(divide="ignore", invalid="ignore"):
            out = np.where(self.size <= 1, 0., self._scaled(r))
        return self._out(out)


class SortinoFixedWindowA(SharpeFixedWindow):
    """reward_normalization.pyx:121-146: as SharpeFixedWindow, negative scaled
    rewards squared in magnitude."""

    def stream(self, reward):  # :135-146
        r = self._in(reward)
        self._update(r)
        with np.errstate(divide="ignore", invalid="ignore"):
            s = self._scaled(r)
            out = np.where(self.size <= 1, 0., np.where(s < 0, -1 * (s * s), s))
        return self._out(out)


class SortinoFixedWindowB(_Batch, RewardShaper):
    """reward_normalization.pyx:149-202: the spread from rewards below the
    running mean only (count, mean, ssq move only on those; the window holds
    them), negative scaled rewards squared."""

    def __init__(self, window: int, n_envs: Optional[int] = None):
        _Batch.__init__(self, window, n_envs)
        self.mean_est = np.zeros(self.N, dtype=np.float64)
        self.ssq = np.zeros(self.N, dtype=np.float64)
        self.count = np.zeros(self.N, dtype=np.int64)
        self.reset()

    @classmethod
    def from_config(cls, config, n_envs: Optional[int] = None):
        return cls(config["window"], n_envs)

    def reset(self, mask=None):
        m = self._mask(mask)
        self.size[m] = 0
        self.head[m] = 0
        self.mean_est[m] = 0.
        self.count[m] = 0
        self.ssq[m] = 0.

    def _update(self, value):  # :189-202
        with np.errstate(divide="ignore", invalid="ignore"):
            self._update_(value)

    def _update_(self, value):
        delt = value - self.mean_est
        idx = np.nonzero(delt < 0)[0]
        if idx.size == 0:
            return
        d = delt[idx]
        self.count[idx] += 1
        self.mean_est[idx] += d / self.count[idx].astype(np.float64)
        self.ssq[idx] += d * (value[idx] - self.mean_est[idx])
        full = idx[self.size[idx] == self.window]
        if full.size:
            self.count[full] -= 1
            remove = self._pop(full)
            d2 = remove - self.mean_est[full]
            self.mean_est[full] -= d2 / self.count[full].astype(np.float64)
            self.ssq[full] -= d2 * (remove - self.mean_est[full])
        self._push(idx, value)

    def _scaled(self, r):
        return r / np.sqrt((self.ssq + 1e-8) / self.count.astype(np.float64))

    def stream(self, reward):  # :178-187
        r = self._in(reward)
        self._update(r)
        with np.errstate(divide="ignore", invalid="ignore"):
            s = self._scaled(r)
            out = np.where(self.size <= 1, 0., np.where(s < 0, -1 * (s * s), s))
        return self._out(out)


class SortinoFixedWindowC(SortinoFixedWindowB):
    """reward_normalization.pyx:205-218: as B without the squaring."""

    def stream(self, reward):  # :213-218
        r = self._in(reward)
        self._update(r)
        with np.errstate(divide="ignore", invalid="ignore"):
            out = np.where(self.size <= 1, 0., self._scaled(r))
        return self._out(out)


class SharpeEWMA(RewardShaper):
    """reward_normalization.pyx:221-272: reward / sqrt of an exponentially
    weighted (alpha = 2 / (window + 1)) bias-corrected variance estimate; 0
    for the first reward.  The weight powers (1 - alpha) ** count are Python's
    float power (C pow), evaluated per distinct count."""

    def __init__(self, window: int, n_envs: Optional[int] = None):
        self.alpha = 2 / (float(window + 1))
        self.scalar = n_envs is None
        self.N = 1 if n_envs is None else int(n_envs)
        z = lambda: np.zeros(self.N, dtype=np.float64)  # noqa: E731
        self.count = np.zeros(self.N, dtype=np.int64)
        self.ewma, self.ewma_old, self.ewssq_old, self.ewssq, self.std_est = z(), z(), z(), z(), z()
        self.w1, self.w2 = z(), z()
        self.reset()

    @classmethod
    def from_config(cls, config, n_envs: Optional[int] = None):
        # the reference reads config.reward_shape_window (attribute access)
        w = getattr(config, "reward_shape_window", None)
        if w is None:
            w = config["reward_shape_window"] if "reward_shape_window" in config else config["window"]
        return cls(w, n_envs)

    def reset(self, mask=None):  # :238-246
        m = np.ones(self.N, dtype=bool) if mask is None else np.asarray(mask, dtype=bool).reshape(-1)
        self.count[m] = 0
        for a in (self.ewma, self.ewma_old, self.ewssq_old, self.ewssq, self.std_est):
            a[m] = 0.
        self.w1[m] = 1.
        self.w2[m] = 1.

    def _update(self, value):  # :260-272
        a = self.alpha
        self.count += 1
        p = np.empty(self.N, dtype=np.float64)
        for c in np.unique(self.count):
            p[self.count == c] = (1 - a) ** int(c)
        self.w1 += p
        pp = np.empty(self.N, dtype=np.float64)
        for c in np.unique(self.count):
            pp[self.count == c] = ((1 - a) ** int(c)) ** 2
        self.w2 += pp
        ewma_prev = self.ewma.copy()
        self.ewma_old = self.ewma_old * (1 - a) + value
        self.ewma = self.ewma_old / self.w1
        self.ewssq_old = self.ewssq_old * (1 - a) + ((value - self.ewma) * (value - ewma_prev))
        self.ewssq = self.ewssq_old / (self.w1 - self.w2 / self.w1)

    def stream(self, reward):  # :248-252
        r = np.asarray(reward, dtype=np.float64)
        r = r.reshape(1) if self.scalar else r
        if r.shape != (self.N,):
            raise ValueError(f"reward must be ({self.N},), got {r.shape}")
        self._update(r)
        with np.errstate(divide="ignore", invalid="ignore"):
            out = np.where(self.count <= 1, 0., r / np.sqrt(self.ewssq))
        # the .pyx divides by sqrt(ewssq) with Cython's checked division: a
        # zero variance (a constant reward stream) raises ZeroDivisionError
        # there, after _update advanced the statistics, never a nan / inf into
        # the caller's data.  Batched, each env behaves as its own shaper: every
        # env's statistics advance, and the error names the envs whose call
        # would have raised, carrying the other envs' values (nan at the named
        # ones) -- a caller that catches it has the batch's step, not a retry
        bad = (self.count > 1) & (self.ewssq == 0.)
        if np.any(bad):
            err = ZeroVarianceError("float division by zero (SharpeEWMA: zero reward variance"
                                    + ("" if self.scalar else f" in envs {np.flatnonzero(bad).tolist()[:8]}") + ")")
            err.envs = np.flatnonzero(bad)
            err.out = np.where(bad, np.nan, out)
            raise err
        return float(out[0]) if self.scalar else out


class ZeroVarianceError(ZeroDivisionError):
    """SharpeEWMA.stream on a zero-variance reward stream (the reference's
    ZeroDivisionError).  ``envs``: the envs whose shaper raised (batched mode;
    [0] in scalar mode); ``out``: the batch's values, nan at those envs.  Every
    env's statistics have advanced, as the reference's _update runs before its
    division."""
    envs: np.ndarray
    out: np.ndarray


_CLASSES = {c.__name__: c for c in (SharpeFixedWindow, SortinoFixedWindowA, SortinoFixedWindowB,
                                     SortinoFixedWindowC, SharpeEWMA)}
