"""HDF replay DataSource (libmadigan_hdf.so, include/madigan_hdf.h).

``HDFSourceSingle`` keeps the reference's Python binding surface
(madigan/environments/cpp/env.cpp:395-431; class DataSource.h:89-149): the
constructor runs checkKeys / loadAssets / loadDimsInfo / getTimeBounds /
findBounds in the C++ reader, and ``getData`` walks the cache exactly as
iterCache / loadData do (DataSource.cpp:368-408), reading the file through
the same reader.  On the MI355X path an env does not call it: the period of
that walk is staged once into HBM as a replay tape (``stage_tape``, pinned
double-buffered H2D) and the step kernels read the tape in place.

``write_hdf`` writes the reference's layout (envTest.cpp:322-368) generalised
to price (T, A).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

from . import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
HDF_LIB_PATH = os.path.join(HERE, "libmadigan_hdf.so")


class HdfInfo(C.Structure):
    _fields_ = [("n_rows", C.c_int64), ("n_assets", C.c_int32), ("n_feats", C.c_int32),
                ("first", C.c_int64), ("second", C.c_int64), ("start_time", C.c_uint64),
                ("end_time", C.c_uint64), ("price_1d", C.c_int32), ("pad_", C.c_int32)]


HDF_SYMBOLS = {
    "mgn_hdf_open": (C.c_int, [C.c_char_p] * 5 + [C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p)]),
    "mgn_hdf_close": (C.c_int, [C.c_void_p]),
    "mgn_hdf_get_info": (C.c_int, [C.c_void_p, C.POINTER(HdfInfo)]),
    "mgn_hdf_asset": (C.c_int, [C.c_void_p, C.c_int32, C.c_char_p, C.c_size_t]),
    "mgn_hdf_read": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                               C.c_void_p]),
    "mgn_hdf_tape_rows": (C.c_int64, [C.c_void_p, C.c_int64]),
    "mgn_hdf_tape_index": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p]),
    "mgn_hdf_stage": (C.c_int, [C.c_void_p, C.c_int64] + [C.c_void_p] * 5),
    "mgn_hdf_write": (C.c_int, [C.c_char_p] * 5 + [C.POINTER(C.c_char_p), C.c_int32, C.c_int64,
                                                   C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                                   C.c_int32]),
    "mgn_hdf_last_error": (C.c_char_p, []),
}

_hlib = None


def load_hdf(path: str = HDF_LIB_PATH):
    global _hlib
    if _hlib is not None:
        return _hlib
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build it with `python -m madigan_amd.build`")
    lib = C.CDLL(path)
    for name, (res, args) in HDF_SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _hlib = lib
    return lib


def _check(status: int) -> None:
    if status == L.OK:
        return
    msg = (load_hdf().mgn_hdf_last_error() or b"").decode(errors="replace")
    if status == L.ERR_CONFIG:
        raise RuntimeError(msg)        # ConfigError
    if status == L.ERR_INDEX:
        raise IndexError(msg)          # std::out_of_range
    if status == L.ERR_LENGTH:
        raise ValueError(msg)          # std::length_error
    if status == L.ERR_ARG:
        raise TypeError(msg)
    raise L.MadiganError(msg)


def _b(s: str) -> bytes:
    return str(s).encode()


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else C.c_void_p(a.ctypes.data)


def write_hdf(path: str, group: str, assets: Sequence[str], price, feats, timestamps,
              price_key: str = "midprice", feature_key: str = "feats",
              timestamp_key: str = "timestamp") -> None:
    """Write a replay file: attribute ``assets``, price (T,) for one asset given
    as a 1-D array, else (T, A), features (T, F), timestamps uint64 (T,)."""
    price = np.ascontiguousarray(price, dtype=np.float64)
    feats = np.ascontiguousarray(feats, dtype=np.float64)
    if feats.ndim == 1:
        feats = feats.reshape(-1, 1)
    ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
    T = ts.shape[0]
    price_1d = price.ndim == 1
    A = 1 if price_1d else price.shape[1]
    if len(assets) != A or price.shape[0] != T or feats.shape[0] != T:
        raise ValueError("assets / price / feats / timestamps shapes disagree")
    arr = (C.c_char_p * A)(*[_b(a) for a in assets])
    _check(load_hdf().mgn_hdf_write(_b(path), _b(group), _b(price_key), _b(feature_key),
                                    _b(timestamp_key), arr, A, T, feats.shape[1], _ptr(price),
                                    _ptr(feats), _ptr(ts), 1 if price_1d else 0))


class HDFFile:
    """An open replay file with its time bounds (HDFSourceSingle::init)."""

    def __init__(self, filepath: str, groupKey: str, priceKey: str, featureKey: str,
                 timestampKey: str, startTime: int = 0, endTime: int = 0):
        lib = load_hdf()
        h = C.c_void_p()
        _check(lib.mgn_hdf_open(_b(filepath), _b(groupKey), _b(priceKey), _b(featureKey),
                                _b(timestampKey), int(startTime), int(endTime), C.byref(h)))
        self.h = h
        info = HdfInfo()
        _check(lib.mgn_hdf_get_info(h, C.byref(info)))
        self.info = info
        buf = C.create_string_buffer(512)
        self.asset_codes = []
        for i in range(info.n_assets):
            _check(lib.mgn_hdf_asset(h, i, buf, 512))
            self.asset_codes.append(buf.value.decode())

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            try:
                load_hdf().mgn_hdf_close(h)
            except Exception:
                pass
            self.h = None

    @property
    def n_assets(self) -> int:
        return self.info.n_assets

    @property
    def n_feats(self) -> int:
        return self.info.n_feats

    @property
    def bounds(self):
        return (int(self.info.first), int(self.info.second))

    def read(self, row0: int, n: int):
        """rows [row0, row0+n): price (n,A), feats (n,F), timestamps (n,)."""
        A, F = self.info.n_assets, self.info.n_feats
        p = np.empty((n, A)); f = np.empty((n, F)); t = np.empty(n, np.uint64)
        _check(load_hdf().mgn_hdf_read(self.h, int(row0), int(n), _ptr(p), _ptr(f), _ptr(t)))
        return p, f, t

    def tape_index(self, cache_size: int) -> np.ndarray:
        """File rows of one period of getData's visiting order."""
        n = load_hdf().mgn_hdf_tape_rows(self.h, int(cache_size))
        out = np.empty(n, np.int64)
        _check(load_hdf().mgn_hdf_tape_index(self.h, int(cache_size), _ptr(out)))
        return out

    def stage_tape(self, cache_size: int, device, stream=None) -> dict:
        """The period as device tensors (pinned double-buffered H2D)."""
        import torch
        lib = load_hdf()
        P = lib.mgn_hdf_tape_rows(self.h, int(cache_size))
        A, F = self.info.n_assets, self.info.n_feats
        t = dict(price=torch.empty((P, A), dtype=torch.float64, device=device),
                 feats=torch.empty((P, F), dtype=torch.float64, device=device),
                 ts=torch.empty((P,), dtype=torch.int64, device=device),
                 data_end=torch.empty((P,), dtype=torch.uint8, device=device))
        st = stream if stream is not None else torch.cuda.current_stream(device)
        _check(lib.mgn_hdf_stage(self.h, int(cache_size), C.c_void_p(t["price"].data_ptr()),
                                 C.c_void_p(t["feats"].data_ptr()), C.c_void_p(t["ts"].data_ptr()),
                                 C.c_void_p(t["data_end"].data_ptr()), C.c_void_p(st.cuda_stream)))
        return t


class HDFSourceSingle:
    """madigan.environments.cpp.HDFSourceSingle (env.cpp:395-431)."""

    def __init__(self, filepath, groupKey=None, priceKey=None, featureKey=None, timestampKey=None,
                 cacheSize=None, startTime: int = 0, endTime: int = 0):
        if isinstance(filepath, dict):  # HDFSourceSingle(Config), DataSource.cpp:227-262
            cfg = dict(filepath.get("data_source_config", filepath))
            missing = [k for k in ("filepath", "group_key", "feature_key", "timestamp_key",
                                   "price_key", "cache_size") if k not in cfg]
            if missing:
                raise RuntimeError("Missing keys in call to HDFSourceSingle: \n" +
                                   ", ".join(missing) + ", \n")
            filepath, groupKey, priceKey = cfg["filepath"], cfg["group_key"], cfg["price_key"]
            featureKey, timestampKey = cfg["feature_key"], cfg["timestamp_key"]
            cacheSize = cfg["cache_size"]
            if "start_time" in cfg and "end_time" in cfg:
                startTime, endTime = cfg["start_time"], cfg["end_time"]
        self.filepath, self.groupKey, self.priceKey = filepath, groupKey, priceKey
        self.featureKey, self.timestampKey = featureKey, timestampKey
        self.file = HDFFile(filepath, groupKey, priceKey, featureKey, timestampKey,
                            int(startTime), int(endTime))
        i = self.file.info
        self.startTime, self.endTime = int(i.start_time), int(i.end_time)
        self._first, self._second = int(i.first), int(i.second)
        self._full = self._second - self._first
        self.cacheSize = min(int(cacheSize), self._full)           # :299
        self._idx = self._first
        self._cidx = 0
        self._load()                                                # init -> loadData
        self._cur_data = np.zeros(i.n_feats)
        self._cur_price = np.zeros(i.n_assets)
        self._ts = 0

    def _load(self):  # loadData, DataSource.cpp:368-379
        if self._idx >= self._second - 1:
            self._idx = self._first
        self._ccs = min(self.cacheSize, self._second - self._idx)
        self._cache = self.file.read(self._idx, self._ccs)

    def _iter_cache(self):  # iterCache, DataSource.cpp:391-408
        if self._cidx == self._ccs or self._idx == self._second:
            if self._ccs >= self._full:
                self._idx = self._first
                self._cidx = 0
            else:
                self._load()
                self._cidx = 0

    def getData(self):  # DataSource.cpp:381-389
        self._iter_cache()
        p, f, t = self._cache
        self._cur_price = p[self._cidx].copy()
        self._cur_data = f[self._cidx].copy()
        self._ts = int(t[self._cidx])
        self._idx += 1
        self._cidx += 1
        return self._cur_data

    def currentData(self):
        return self._cur_data

    def currentPrices(self):
        return self._cur_price

    def reset(self):  # "Carry on" (DataSource.cpp:200-206)
        pass

    def dataEnd(self) -> bool:  # DataSource.h:126
        return self._idx == self._second

    @property
    def size(self):
        return self._full

    @property
    def currentCacheSize(self):
        return self._ccs

    @property
    def nFeats(self):
        return self.file.n_feats

    @property
    def nAssets(self):
        return self.file.n_assets

    @property
    def currentIdx(self):
        return self._idx

    @property
    def currentCacheIdx(self):
        return self._cidx

    @property
    def currentTime(self):
        return self._ts

    @property
    def boundsIdx(self):
        return (self._first, self._second)

    @property
    def isDateTime(self):
        return True

    @property
    def assets(self):
        from .env import Asset
        return [Asset(a) for a in self.file.asset_codes]
