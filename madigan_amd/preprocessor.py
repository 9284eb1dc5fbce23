"""Device-backed StackerDiscrete family (madigan/utils/preprocessor.py:143-327).

Keeps the last ``window_len`` States of every env in a device ring
(N, W, F + A+1) and assembles ``current_data()`` with the HIP gather kernel
(normalisers log / lookback / lookback_log / standard_normal /
log_standard_normal applied on device).  StackerDiscretePairs stores the pair
ratio at push, StackerDiscreteReturns differences the gathered price columns
(mgn_feat_diff), MultiStackerDiscrete gathers one ring per dilation side by
side.  Works for the drop-in single ``Env`` (numpy State in, numpy State
out, ``len(self)`` rows like the reference deque) and for batched States of
device tensors (N, ...) -> (N, W, ...).
"""
from __future__ import annotations

import ctypes as C
from abc import ABC, abstractmethod
from typing import List

import numpy as np

from . import _lib as L
from .config import norm_code
from .env import State


class PreProcessor(ABC):
    """PreProcessor ABC (preprocessor.py:110-140)."""

    @property
    def feature_output_shape(self):
        """Returns the output shape for features in state.price"""

    @abstractmethod
    def stream(self, data):
        """Ingests either a State or SRDI"""

    @abstractmethod
    def stream_state(self, state):
        """Ingests data given as State"""

    @abstractmethod
    def current_data(self):
        """Performs normalisation (if indicated) and returns current data."""

    @classmethod
    def from_config(cls, config, n_feats):
        return make_preprocessor(config, n_feats)

    @abstractmethod
    def initialize_history(self, env):
        """Steps the env with empty actions until the window is full."""


def _get(c, k, d=None):
    if isinstance(c, dict):
        return c.get(k, d)
    return getattr(c, k, d)


def make_preprocessor(config, n_feats):
    """make_preprocessor (preprocessor.py:28-50) for the StackerDiscrete family.
    The reference's tests are reproduced as written: "StackerDiscreteReturns"
    maps to plain StackerDiscrete (:36-38), and the later checks are substring
    tests on one string (``x in ("StackerDiscretePairs")``, :39-42)."""
    ptype = _get(config, "preprocessor_type")
    if ptype in ("WindowedStacker", "StackerDiscrete", "StackerDiscreteReturns"):
        return StackerDiscrete.from_config(config, n_feats)
    if isinstance(ptype, str) and ptype in "StackerDiscretePairs":
        return StackerDiscretePairs.from_config(config, n_feats)
    if isinstance(ptype, str) and ptype in "MultiStackerDiscrete":
        return MultiStackerDiscrete.from_config(config, n_feats)
    raise NotImplementedError(f"{ptype} is not implemented ")


def _pconf(config):
    pconf = _get(config, "preprocessor_config")
    keys = pconf.keys() if isinstance(pconf, dict) else vars(pconf).keys()
    norm = _get(pconf, "norm") if "norm" in keys else False
    norm_type = _get(pconf, "norm_type") if "norm_type" in keys else None
    return pconf, norm, norm_type


def _norm_code_or_raise(norm_type):
    """make_normalizer (preprocessor.py:53-77): unknown types, including None,
    raise NotImplementedError.  'expanding' constructs (its lambda fails later)."""
    if norm_type == "expanding":
        return "expanding"
    code = norm_code(norm_type) if norm_type is not None else None
    if code is None:
        raise NotImplementedError(
            f"norm_type {norm_type} is not implemented.choose from : 'lookback', "
            "'lookback_log', 'standard_normal', 'expanding'")
    return code


class _DeviceRing:
    """One deque(maxlen=W) of (price, portfolio, timestamp) rows per env, on
    device (mgn_ring): ring (N, W, F + P), timestamps, head / len."""

    def __init__(self, n_envs, n_price, n_port, window, norm, device, transform=0,
                 out_stride=0, out_offset=0):
        import torch
        self.torch, self.dev = torch, device
        self.N, self.F, self.P, self.W = n_envs, n_price, n_port, window
        self.ring = torch.zeros((n_envs, window, n_price + n_port), dtype=torch.float64, device=device)
        self.ts = torch.zeros((n_envs, window), dtype=torch.int64, device=device)
        self.head = torch.full((n_envs,), window - 1, dtype=torch.int32, device=device)
        self.len = torch.zeros((n_envs,), dtype=torch.int32, device=device)
        r = L.Ring()
        r.n_envs, r.n_price, r.n_port, r.window = n_envs, n_price, n_port, window
        r.norm_type, r.transform = norm, transform
        r.out_stride, r.out_offset = out_stride, out_offset
        r.ring, r.ring_ts = self.ring.data_ptr(), self.ts.data_ptr()
        r.head, r.len = self.head.data_ptr(), self.len.data_ptr()
        self.r = r
        self.lib = L.load()

    def stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def push(self, price, port, ts):
        L.check(self.lib.mgn_ring_push(C.byref(self.r), C.c_void_p(price.data_ptr()),
                                       C.c_void_p(port.data_ptr()), C.c_void_p(ts.data_ptr()),
                                       self.stream()))

    def clear(self):
        L.check(self.lib.mgn_ring_clear(C.byref(self.r), None, self.stream()))

    def gather(self, price, port=None, ts=None):
        ptr = (lambda t: None if t is None else C.c_void_p(t.data_ptr()))
        L.check(self.lib.mgn_ring_gather(C.byref(self.r), ptr(price), ptr(port), ptr(ts),
                                         self.stream()))


class StackerDiscrete(PreProcessor):
    def __init__(self, window_len: int, n_features: int, norm: bool = True,
                 norm_type: str = "standard_normal"):
        self.k = int(window_len)
        self.min_tf = self.k
        self.norm = norm
        self.norm_code = _norm_code_or_raise(norm_type)
        self._feature_output_shape = (self.k, n_features)
        self._len = 0
        self._ring = None

    @property
    def feature_output_shape(self):
        return self._feature_output_shape

    @classmethod
    def from_config(cls, config, n_feats):
        pconf, norm, norm_type = _pconf(config)
        return cls(_get(pconf, "window_length"), n_feats, norm, norm_type)

    def __len__(self):
        return self._len

    # ---- device ring ---------------------------------------------------------
    _transform = L.RING_PLAIN

    def _ring_cols(self, n_in):
        return n_in

    def _alloc(self, n_envs, n_price, n_port, device):
        import torch
        W = self.k
        self._torch = torch
        self._dev = device
        self._n = n_envs
        self._Fin, self._P = n_price, n_port
        self._F = self._ring_cols(n_price)
        norm = self.norm_code if (self.norm and self.norm_code != "expanding") else L.NORM_NONE
        self._ring = _DeviceRing(n_envs, self._F, n_port, W, norm, device, self._transform)
        self._out_price = torch.empty((n_envs, W, self._F), dtype=torch.float64, device=device)
        self._out_port = torch.empty((n_envs, W, n_port), dtype=torch.float64, device=device)
        self._out_ts = torch.empty((n_envs, W), dtype=torch.int64, device=device)

    def _to_dev(self, x, dtype, shape):
        torch = self._torch
        t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
        return t.to(self._dev, dtype).reshape(shape).contiguous()

    def _rows(self, state):
        """(price, port, ts) device rows of a State, allocating on first use."""
        import torch
        price, port, ts = state.price, state.portfolio, state.timestamp
        batched = isinstance(price, torch.Tensor) and price.dim() == 2
        if self._ring is None:
            n = price.shape[0] if batched else 1
            f = price.shape[-1] if batched else int(np.asarray(price).reshape(-1).shape[0])
            p = port.shape[-1] if batched else int(np.asarray(port).reshape(-1).shape[0])
            dev = price.device if isinstance(price, torch.Tensor) and price.is_cuda else torch.device("cuda")
            self._alloc(n, f, p, dev)
            self._batched = batched
        pr = self._to_dev(price, torch.float64, (self._n, self._Fin))
        po = self._to_dev(port, torch.float64, (self._n, self._P))
        tt = self._to_dev(np.asarray(ts, dtype=np.int64) if not isinstance(ts, torch.Tensor) else ts,
                          torch.int64, (self._n,))
        return pr, po, tt

    def stream_state(self, state):
        pr, po, tt = self._rows(state)
        self._ring.push(pr, po, tt)
        self._len = min(self._len + 1, self.k)

    def stream(self, data):
        if isinstance(data, tuple):
            self.stream_state(data[0])
        else:
            self.stream_state(data)

    def _gather(self):
        if self.norm and self.norm_code == "expanding":
            # x / _expanding_mean(x): _expanding_mean(arr, ma) needs two arguments
            # (preprocessor.py:73, :475), so the reference raises here
            raise TypeError("_expanding_mean() missing 1 required positional argument: 'ma'")
        self._ring.gather(self._out_price, self._out_port, self._out_ts)
        return self._out_price, self._out_port, self._out_ts

    def current_data(self):
        if self._ring is None:
            return State(np.zeros((0, self._feature_output_shape[1])), np.zeros((0, 0)),
                         np.zeros((0,), np.int64))
        price, port, ts = self._gather()
        if self._batched:
            return State(price, port, ts)
        n = self._len
        return State(price[0, :n].cpu().numpy(), port[0, :n].cpu().numpy(), ts[0, :n].cpu().numpy())

    def initialize_history(self, env):
        while len(self) < self.k:
            _state, reward, done, info = env.step()
            self.stream_state(_state)

    def reset_state(self):
        if self._ring is not None:
            self._ring.clear()
        self._len = 0


class StackerDiscretePairs(StackerDiscrete):
    """preprocessor.py:291-316: the price is the ratio of a pair's two
    features (normalised after), one column.  The ratio is row-wise, so the
    ring stores it at push (MGN_RING_PAIR_RATIO)."""
    _transform = L.RING_PAIR_RATIO

    def __init__(self, window_len: int, n_feats: int, norm: bool = True,
                 norm_type: str = "standard_normal"):
        assert n_feats == 2
        super().__init__(window_len, n_feats, norm, norm_type)
        self._feature_output_shape = (self.k, 1)

    def _ring_cols(self, n_in):
        if n_in != 2:
            raise IndexError("StackerDiscretePairs needs 2 price features per State")
        return 1


class StackerDiscreteReturns(StackerDiscrete):
    """preprocessor.py:319-327: normalise, then np.diff with numpy's default
    axis -1 -- across the price columns, not time (reproduced) -- and drop the
    first portfolio / timestamp row."""

    def current_data(self):
        if self._ring is None:
            return super().current_data()
        price, port, ts = self._gather()
        N, W, F = price.shape
        diff = self._torch.empty((N, W, max(F - 1, 0)), dtype=self._torch.float64, device=self._dev)
        L.check(L.load().mgn_feat_diff(C.c_void_p(price.data_ptr()), C.c_void_p(diff.data_ptr()),
                                       N * W, F, self._ring.stream()))
        if self._batched:
            return State(diff, port[:, 1:], ts[:, 1:])
        n = self._len
        return State(diff[0, :n].cpu().numpy(), port[0, 1:n].cpu().numpy(),
                     ts[0, 1:n].cpu().numpy())


class MultiStackerDiscrete(PreProcessor):
    """preprocessor.py:202-288: one window per dilation d, fed every d-th
    State (per-dilation countdown, not reset by reset_state); current_data
    concatenates the dilations' price windows along the features (the device
    rings gather side by side into one (N, W, F * n_dilations) array) and
    returns the first dilation's portfolio and timestamps."""

    def __init__(self, window_len: int, dilations: List[int], n_feats: int, norm: bool = True,
                 norm_type: str = "standard_normal"):
        self.k = int(window_len)
        self.dilations = list(dilations)
        self.dilation_counter = np.zeros(len(self.dilations), dtype=np.int64)
        self.min_tf = self.k
        self.norm = norm
        self.norm_code = _norm_code_or_raise(norm_type)
        self.max_dilation = max(self.dilations)
        self._lens = [0] * len(self.dilations)
        self._feature_output_shape = (self.k, n_feats * len(self.dilations))
        self._rings = None

    @property
    def feature_output_shape(self):
        return self._feature_output_shape

    @classmethod
    def from_config(cls, config, n_feats):
        pconf, norm, norm_type = _pconf(config)
        return cls(_get(pconf, "window_length"), _get(pconf, "dilations"), n_feats, norm,
                   norm_type)

    def __len__(self):
        return self._lens[self.dilations.index(self.max_dilation)]

    def stream_state(self, state):
        if self._rings is None:
            self._base = StackerDiscrete(self.k, 1, False, "lookback")  # row staging only
            pr, po, tt = self._base._rows(state)
            self._batched, self._dev, self._torch = self._base._batched, self._base._dev, self._base._torch
            N, F, P = self._base._n, self._base._Fin, self._base._P
            self._N, self._F, self._P = N, F, P
            D = len(self.dilations)
            norm = self.norm_code if (self.norm and self.norm_code != "expanding") else L.NORM_NONE
            self._rings = [_DeviceRing(N, F, P, self.k, norm, self._dev, out_stride=F * D,
                                       out_offset=i * F) for i in range(D)]
            torch = self._torch
            self._out_price = torch.empty((N, self.k, F * D), dtype=torch.float64, device=self._dev)
            self._out_port = torch.empty((N, self.k, P), dtype=torch.float64, device=self._dev)
            self._out_ts = torch.empty((N, self.k), dtype=torch.int64, device=self._dev)
        else:
            pr, po, tt = self._base._rows(state)
        for i, d in enumerate(self.dilations):
            if self.dilation_counter[i] == 0:
                self._rings[i].push(pr, po, tt)
                self._lens[i] = min(self._lens[i] + 1, self.k)
                self.dilation_counter[i] = d - 1
            else:
                self.dilation_counter[i] -= 1

    def stream(self, data):
        if isinstance(data, tuple):
            self.stream_state(data[0])
        else:
            self.stream_state(data)

    def current_data(self):
        if self._rings is None or len(set(self._lens)) != 1:
            # np.concatenate of windows of different lengths
            raise ValueError("all the input array dimensions except for the concatenation axis "
                             "must match exactly")
        if self.norm and self.norm_code == "expanding":
            raise TypeError("_expanding_mean() missing 1 required positional argument: 'ma'")
        for i, r in enumerate(self._rings):
            r.gather(self._out_price, self._out_port if i == 0 else None,
                     self._out_ts if i == 0 else None)
        if self._batched:
            return State(self._out_price, self._out_port, self._out_ts)
        n = self._lens[0]
        return State(self._out_price[0, :n].cpu().numpy(), self._out_port[0, :n].cpu().numpy(),
                     self._out_ts[0, :n].cpu().numpy())

    def initialize_history(self, env):
        while len(self) < self.k:
            _state, reward, done, info = env.step()
            self.stream_state(_state)

    def reset_state(self):
        if self._rings is not None:
            for r in self._rings:
                r.clear()
        self._lens = [0] * len(self.dilations)
