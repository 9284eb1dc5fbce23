"""Device-backed StackerDiscrete (madigan/utils/preprocessor.py:143-199).

Keeps the last ``window_len`` States of every env in a device ring
(N, W, F + A+1) and assembles ``current_data()`` with the HIP gather kernel
(normalisers log / lookback / lookback_log / standard_normal applied on
device).  Works for the drop-in single ``Env`` (numpy State in, numpy State
out, ``len(self)`` rows like the reference deque) and for batched States of
device tensors (N, ...) -> (N, W, ...).
"""
from __future__ import annotations

import ctypes as C
from abc import ABC, abstractmethod

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
    """make_preprocessor (preprocessor.py:28-50) for the StackerDiscrete family."""
    ptype = _get(config, "preprocessor_type")
    if ptype in ("WindowedStacker", "StackerDiscrete", "StackerDiscreteReturns"):
        return StackerDiscrete.from_config(config, n_feats)
    raise NotImplementedError(f"{ptype} is not implemented ")


class StackerDiscrete(PreProcessor):
    def __init__(self, window_len: int, n_features: int, norm: bool = True,
                 norm_type: str = "standard_normal"):
        self.k = int(window_len)
        self.min_tf = self.k
        self.norm = norm
        # make_normalizer raises for unknown types, including None (preprocessor.py:53-77)
        self.norm_code = norm_code(norm_type) if norm_type is not None else None
        if self.norm_code is None:
            raise NotImplementedError(
                f"norm_type {norm_type} is not implemented.choose from : 'lookback', "
                "'lookback_log', 'standard_normal', 'expanding'")
        self._feature_output_shape = (self.k, n_features)
        self._len = 0
        self._ring = None

    @property
    def feature_output_shape(self):
        return self._feature_output_shape

    @classmethod
    def from_config(cls, config, n_feats):
        pconf = _get(config, "preprocessor_config")
        keys = pconf.keys() if isinstance(pconf, dict) else vars(pconf).keys()
        norm = _get(pconf, "norm") if "norm" in keys else False
        norm_type = _get(pconf, "norm_type") if "norm_type" in keys else None
        return cls(_get(pconf, "window_length"), n_feats, norm, norm_type)

    def __len__(self):
        return self._len

    # ---- device ring ---------------------------------------------------------
    def _alloc(self, n_envs, n_price, n_port, device):
        import torch
        W = self.k
        self._torch = torch
        self._dev = device
        self._n = n_envs
        self._F, self._P = n_price, n_port
        self._ring_t = torch.zeros((n_envs, W, n_price + n_port), dtype=torch.float64, device=device)
        self._ts_t = torch.zeros((n_envs, W), dtype=torch.int64, device=device)
        self._head = torch.full((n_envs,), W - 1, dtype=torch.int32, device=device)
        self._lent = torch.zeros((n_envs,), dtype=torch.int32, device=device)
        self._out_price = torch.empty((n_envs, W, n_price), dtype=torch.float64, device=device)
        self._out_port = torch.empty((n_envs, W, n_port), dtype=torch.float64, device=device)
        self._out_ts = torch.empty((n_envs, W), dtype=torch.int64, device=device)
        r = L.Ring()
        r.n_envs, r.n_price, r.n_port, r.window = n_envs, n_price, n_port, W
        r.norm_type = self.norm_code if self.norm else L.NORM_NONE
        r.ring, r.ring_ts = self._ring_t.data_ptr(), self._ts_t.data_ptr()
        r.head, r.len = self._head.data_ptr(), self._lent.data_ptr()
        self._ring = r
        self._lib = L.load()

    def _stream(self):
        return C.c_void_p(self._torch.cuda.current_stream(self._dev).cuda_stream)

    def _to_dev(self, x, dtype, shape):
        torch = self._torch
        t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
        return t.to(self._dev, dtype).reshape(shape).contiguous()

    def stream_state(self, state):
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
        pr = self._to_dev(price, torch.float64, (self._n, self._F))
        po = self._to_dev(port, torch.float64, (self._n, self._P))
        tt = self._to_dev(np.asarray(ts, dtype=np.int64) if not isinstance(ts, torch.Tensor) else ts,
                          torch.int64, (self._n,))
        L.check(self._lib.mgn_ring_push(C.byref(self._ring), C.c_void_p(pr.data_ptr()),
                                        C.c_void_p(po.data_ptr()), C.c_void_p(tt.data_ptr()),
                                        self._stream()))
        self._len = min(self._len + 1, self.k)

    def stream(self, data):
        if isinstance(data, tuple):
            self.stream_state(data[0])
        else:
            self.stream_state(data)

    def current_data(self):
        if self._ring is None:
            return State(np.zeros((0, self._feature_output_shape[1])), np.zeros((0, 0)),
                         np.zeros((0,), np.int64))
        L.check(self._lib.mgn_ring_gather(C.byref(self._ring), C.c_void_p(self._out_price.data_ptr()),
                                          C.c_void_p(self._out_port.data_ptr()),
                                          C.c_void_p(self._out_ts.data_ptr()), self._stream()))
        if self._batched:
            return State(self._out_price, self._out_port, self._out_ts)
        n = self._len
        return State(self._out_price[0, :n].cpu().numpy(), self._out_port[0, :n].cpu().numpy(),
                     self._out_ts[0, :n].cpu().numpy())

    def initialize_history(self, env):
        while len(self) < self.k:
            _state, reward, done, info = env.step()
            self.stream_state(_state)

    def reset_state(self):
        if self._ring is not None:
            L.check(self._lib.mgn_ring_clear(C.byref(self._ring), None, self._stream()))
        self._len = 0
