"""Batched MI355X environments and the drop-in ``Env`` (N = 1 view).

``BatchedEnv`` owns one handle of the C ABI: N independent envs whose state
lives in HBM (struct-of-arrays, env-major) and which one HIP launch advances by
one step (``step``) or K steps (``rollout``).  Outputs are device tensors that
alias the handle's buffers (valid until the next launch), mirroring the
reference's zero-copy property views (madigan/environments/cpp/env.cpp:897-913).

``Env`` keeps the reference's Python surface (env.cpp:843-1005,
madigan/environments/__init__.py) for one environment: ``reset()``,
``step()``, ``step(units)``, ``step(assetIdx, units)``, ``step(assetCode,
units)`` and the property accessors, returning host numpy values exactly like
the pybind11 module did.
"""
from __future__ import annotations

import ctypes as C
from collections import namedtuple
from typing import Any, Optional

import numpy as np

from . import _lib as L
from .config import SourceSpec, build_config, default_spec, spec_from_config

RISK_NAMES = {L.GREEN: "green", L.INSUFF_MARGIN: "insuff_margin", L.MARGIN_CALL: "margin_call",
              L.BLOWN_OUT: "blown_out"}

VALUATION_FIELDS = ("cash", "equity", "pnl", "balance", "availableMargin", "usedMargin",
                    "borrowedMargin", "borrowedAssetValue", "assetValue", "checkRisk")

StepOutput = namedtuple("StepOutput", ["reward", "done", "obs_price", "obs_port", "timestamp",
                                       "tprice", "tunits", "tcost", "risk", "margin_call",
                                       "shaped", "agent_reward", "n_shaped", "data_end"])


def _torch():
    import torch
    return torch


class RiskInfo(int):
    """RiskInfo enum (DataTypes.h:70-75) with the pybind11 names."""
    green = L.GREEN
    insuff_margin = L.INSUFF_MARGIN
    margin_call = L.MARGIN_CALL
    blown_out = L.BLOWN_OUT

    def __repr__(self):
        return f"RiskInfo.{RISK_NAMES.get(int(self), int(self))}"

    __str__ = __repr__


for _v, _n in RISK_NAMES.items():
    setattr(RiskInfo, _n, RiskInfo(_v))


class State:
    """State{price, portfolio, timestamp} (DataTypes.h:52-63)."""
    __slots__ = ("price", "portfolio", "timestamp")

    def __init__(self, price, portfolio, timestamp):
        self.price = price
        self.portfolio = portfolio
        self.timestamp = timestamp

    def __iter__(self):
        return iter((self.price, self.portfolio, self.timestamp))

    def __repr__(self):
        return f"State(price={self.price!r}, portfolio={self.portfolio!r}, timestamp={self.timestamp!r})"


class BrokerResponse:
    """BrokerResponse<T> (DataTypes.h:103-135)."""

    def __init__(self, transactionPrice, transactionUnits, transactionCost, riskInfo, marginCall,
                 timestamp=0, event=""):
        self.transactionPrice = transactionPrice
        self.transactionUnits = transactionUnits
        self.transactionCost = transactionCost
        self.riskInfo = riskInfo
        self.marginCall = marginCall
        self.timestamp = timestamp
        self.event = event

    def __repr__(self):
        return (f"timestamp:        {self.timestamp}\ntransactionPrice: \n{self.transactionPrice}\n"
                f"transactionUnits:  \n{self.transactionUnits}\ntransactionCost:  \n"
                f"{self.transactionCost}\nriskInfo:         \n{self.riskInfo}\nmarginCall:         \n"
                f"{self.marginCall}\n")


class EnvInfo:
    """EnvInfo<T> (DataTypes.h:141-149)."""

    def __init__(self, brokerResponse=None, dataEnd=False):
        self.brokerResponse = brokerResponse
        self.dataEnd = dataEnd


class Asset:
    def __init__(self, code):
        self.code = code

    def __repr__(self):
        return self.code

    def __eq__(self, other):
        return getattr(other, "code", other) == self.code

    def __hash__(self):
        return hash(self.code)


class BatchedEnv:
    """N independent madigan Envs on one GPU (one handle of the C ABI)."""

    def __init__(self, spec: SourceSpec, n_envs: int, *, device=None, seed: int = 0,
                 env_offset: int = 0, init_cash: float = 1_000_000.0,
                 required_margin: float = 0.0, maintenance_margin: float = 0.0,
                 slippage_rel: float = 0.0, slippage_abs: float = 0.0,
                 transaction_cost_rel: float = 0.0, transaction_cost_abs: float = 0.0,
                 reward_shaper=None, reward_mode: str = "env_log",
                 adaptation_rate: float = 0.001, cosine_temp: float = 0.0,
                 desired_portfolio=None, window: int = 0, norm_type=None,
                 auto_reset: bool = False, action_atoms: int = 3, unit_size: float = 0.05,
                 nstep_return: int = 1, discount: float = 0.99, replay_tape: Optional[dict] = None,
                 replay_stride: int = 0, sortino_exp=None, nstep_pop: str = "exact"):
        """nstep_pop: "exact" (default) re-evaluates every n-step pop's
        summands as nstep_buffer.py does; "running" lets the three-role kernel
        pop DSR / DDR / PPC / none from discounted running sums (O(1) per pop,
        within 1e-6 of the exact pop; include/madigan_amd.h MGN_NSTEP_POP_*).

        A replay spec (``config.replay_spec`` / HDFSourceSingle) reads its
        prices, features and timestamps from a device replay tape: staged from
        the spec's HDF file (``spec.hdf``, cache_size chunks, pinned
        double-buffered H2D) or given as ``replay_tape`` = {price (P,A),
        feats (P,F), ts (P,), data_end (P,)} device tensors.  Env g starts at
        tape row (g * replay_stride) mod P."""
        torch = _torch()
        self.lib = L.load()
        if not torch.cuda.is_available():
            raise RuntimeError("madigan_amd needs a ROCm GPU (gfx950); there is no CPU fallback")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.spec = spec
        self.cfg, self._srcs = build_config(
            spec, n_envs=n_envs, init_cash=init_cash, required_margin=required_margin,
            maintenance_margin=maintenance_margin, slippage_rel=slippage_rel,
            slippage_abs=slippage_abs, transaction_cost_rel=transaction_cost_rel,
            transaction_cost_abs=transaction_cost_abs, reward_shaper=reward_shaper,
            reward_mode=reward_mode, adaptation_rate=adaptation_rate, cosine_temp=cosine_temp,
            desired_portfolio=desired_portfolio, window=window, norm_type=norm_type,
            auto_reset=auto_reset, action_atoms=action_atoms, unit_size=unit_size, seed=seed,
            env_offset=env_offset, nstep_return=nstep_return, discount=discount,
            sortino_exp=sortino_exp, nstep_pop=nstep_pop)
        self.N = int(n_envs)
        self.A = spec.n_assets
        self.F = int(spec.n_feats) if spec.replay else self.A
        self.W = int(window)
        nbytes = self.lib.mgn_arena_bytes(C.byref(self.cfg))
        if nbytes == 0:
            raise ValueError("invalid env dimensions")
        # the arena and, after it (256-B aligned), the (N, 10) valuation rows,
        # so a host snapshot of both is one copy (Env)
        self._val_off = (nbytes + 255) // 256 * 256
        with torch.cuda.device(self.device):
            self._arena_buf = torch.empty(self._val_off + self.N * 80, dtype=torch.uint8, device=self.device)
            self.arena = self._arena_buf[:nbytes]
            self.stream = torch.cuda.current_stream(self.device)
        h = C.c_void_p()
        L.check(self.lib.mgn_create(C.byref(self.cfg), self._srcs, C.c_void_p(self.stream.cuda_stream),
                                    C.c_void_p(self.arena.data_ptr()), nbytes, C.byref(h)))
        self.h = h
        v = L.Views()
        L.check(self.lib.mgn_get_views(self.h, C.byref(v)), self.h)
        self._v = v
        self.D = v.reward_dim
        self.nstep = v.nstep
        self._build_views()
        self._val = self._arena_buf[self._val_off:].view(torch.float64).view(self.N, 10)
        self._traj_cache = {}
        # host-array inputs (_dev): pinned twins of the staging buffers, copied
        # asynchronously on the handle's stream, each guarded by an event
        self._pinned = {}
        self._tape = None
        if spec.replay:
            self._attach_replay(replay_tape, int(replay_stride))
        elif replay_tape is not None:
            raise RuntimeError("replay_tape given for a generator source spec")

    def _attach_replay(self, tape: Optional[dict], stride: int):
        torch = _torch()
        if tape is None:
            if not self.spec.hdf:
                raise RuntimeError("replay source needs an HDF config or a replay_tape")
            from .hdf import HDFFile
            h = self.spec.hdf
            f = HDFFile(h["filepath"], h["group_key"], h["price_key"], h["feature_key"],
                        h["timestamp_key"], int(h.get("start_time", 0)), int(h.get("end_time", 0)))
            with torch.cuda.device(self.device):
                tape = f.stage_tape(int(h["cache_size"]), self.device, self.stream)
            stride = int(h.get("replay_stride", stride))
        want = dict(price=(torch.float64, 2, self.A), feats=(torch.float64, 2, self.F),
                    ts=(torch.int64, 1, None), data_end=(torch.uint8, 1, None))
        rows = None
        for k, (dt, nd, cols) in want.items():
            t = tape.get(k)
            if t is None or t.dtype != dt or t.dim() != nd or t.device != self.device \
                    or not t.is_contiguous() or (cols is not None and t.shape[1] != cols):
                raise ValueError(f"replay_tape[{k!r}] must be a contiguous {dt} tensor of "
                                 f"{nd} dims on {self.device}" + (f" with {cols} columns" if cols else ""))
            if rows is not None and t.shape[0] != rows:
                raise ValueError("replay_tape arrays differ in rows")
            rows = t.shape[0]
        self._tape = tape
        rt = L.ReplayTape(price=tape["price"].data_ptr(), feats=tape["feats"].data_ptr(),
                          ts=tape["ts"].data_ptr(), data_end=tape["data_end"].data_ptr(),
                          rows=int(rows), stride=int(stride))
        L.check(self.lib.mgn_attach_replay(self.h, C.byref(rt)), self.h)

    # ---- tensor views over the arena --------------------------------------
    def _t(self, ptr, dtype, shape):
        torch = _torch()
        if not ptr:
            return None
        n = int(np.prod(shape))
        item = torch.empty((), dtype=dtype).element_size()
        off = ptr - self.arena.data_ptr()
        return self.arena[off:off + n * item].view(dtype).view(shape)

    def _build_views(self):
        torch = _torch()
        f64, i32, u8, i64 = torch.float64, torch.int32, torch.uint8, torch.int64
        N, A, W, D, F, v = self.N, self.A, self.W, self.D, self.F, self._v
        NA = (N, A)
        Dsh = (N,) if D == 1 else (N, A)
        self.ledger = self._t(v.ledger, f64, NA)
        self.mean_entry = self._t(v.mean_entry, f64, NA)
        self.borrowed = self._t(v.borrowed, f64, NA)
        self.prices = self._t(v.prices, f64, NA)
        self.sine_x = self._t(v.sine_x, f64, NA)
        self.ou_mean = self._t(v.ou_mean, f64, NA)
        self.trend_dy = self._t(v.trend_dy, f64, NA)
        self.trend_len = self._t(v.trend_len, i32, NA)
        self.trend_flags = self._t(v.trend_flags, u8, NA)
        self.cash = self._t(v.cash, f64, (N,))
        self.timestamp = self._t(v.timestamp, i64, (N,))
        # resets so far: the variates' draw index is timestamp + draw_skip (DESIGN, variates v3)
        self.draw_skip = self._t(v.draw_skip, i64, (N,))
        self.shaper_a = self._t(v.shaper_a, f64, Dsh)
        self.shaper_b = self._t(v.shaper_b, f64, Dsh)
        self.ep_stats = self._t(v.ep_stats, f64, (N, 2))
        self.episode_stats = self._t(v.episode_stats, f64, (N, 4))
        self.ext_prices = self._t(v.ext_prices, f64, NA)
        self.units_buf = self._t(v.units, f64, NA)
        self.asset_idx_buf = self._t(v.asset_idx, i32, (N,))
        self.reset_mask_buf = self._t(v.reset_mask, u8, (N,))
        if W:
            self.ring = self._t(v.ring, f64, (N, W, F + A + 1))
            self.win_price = self._t(v.win_price, f64, (N, W, F))
            self.win_port = self._t(v.win_port, f64, (N, W, A + 1))
            self.win_ts = self._t(v.win_ts, i64, (N, W))
            self.ring_len = self._t(v.ring_len, i32, (N,))
        o = v.out
        self.out = StepOutput(
            reward=self._t(o.reward, f64, (N,)), done=self._t(o.done, u8, (N,)),
            obs_price=self._t(o.obs_price, f64, (N, F)), obs_port=self._t(o.obs_port, f64, (N, A + 1)),
            timestamp=self._t(o.timestamp, i64, (N,)), tprice=self._t(o.tprice, f64, NA),
            tunits=self._t(o.tunits, f64, NA), tcost=self._t(o.tcost, f64, NA),
            risk=self._t(o.risk, u8, NA), margin_call=self._t(o.margin_call, u8, (N,)),
            shaped=self._t(o.shaped, f64, self._shaped_shape()),
            agent_reward=self._t(o.agent_reward, f64, Dsh), n_shaped=self._t(o.n_shaped, u8, (N,)),
            data_end=self._t(o.data_end, u8, (N,)))
        self.replay_cursor = self._t(v.replay_cursor, i64, (N,))
        # the whole step-output block is contiguous in the arena: one D2H copy
        lo = o.reward - self.arena.data_ptr()
        hi = o.data_end - self.arena.data_ptr() + N
        self._out_span = (lo, hi)

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            try:
                self.lib.mgn_destroy(h)
            except Exception:
                pass
            self.h = None

    # ---- inputs -------------------------------------------------------------
    def _dev(self, x, dtype, shape, staging):
        torch = _torch()
        if isinstance(x, torch.Tensor) and x.device == self.device and x.dtype == dtype \
                and x.is_contiguous() and tuple(x.shape) == tuple(shape):
            return x
        n = int(np.prod(shape))
        dst = staging.view(-1)[:n]
        if isinstance(x, torch.Tensor) and x.device.type != "cpu":
            if x.numel() != n:
                raise ValueError(f"expected {n} values, got {x.numel()}")
            dst.copy_(x.reshape(-1).to(dtype), non_blocking=False)
            return dst.view(shape)
        xa = np.asarray(x.detach().numpy() if isinstance(x, torch.Tensor) else x).reshape(-1)
        if xa.size != n:
            raise ValueError(f"expected {n} values, got {xa.size}")
        # a host array: into the pinned twin of the staging buffer (after the
        # previous asynchronous copy out of it has run), then one asynchronous
        # H2D copy on the handle's stream, ordered before the launch that
        # reads it -- no synchronous pageable copy per step
        key = staging.data_ptr()
        twin = self._pinned.get(key)
        if twin is None:
            hb = torch.empty(staging.numel(), dtype=staging.dtype, pin_memory=True)
            twin = (hb, hb.numpy(), torch.cuda.Event())
            self._pinned[key] = twin
        else:
            twin[2].synchronize()
        hb, hnp, ev = twin
        hnp[:n] = xa  # numpy casts to the staging dtype (exact for the int8 / int32 / f64 inputs)
        hip = L.hip()
        st = C.c_void_p(self.stream.cuda_stream)
        nbytes = n * hb.element_size()
        if hip.hipMemcpyAsync(C.c_void_p(dst.data_ptr()), C.c_void_p(hb.data_ptr()), C.c_size_t(nbytes),
                              1, st) != 0:  # hipMemcpyHostToDevice
            raise RuntimeError("hipMemcpyAsync (input staging) failed")
        ev.record(self.stream)
        return dst.view(shape)

    # ---- API ------------------------------------------------------------------
    def set_broker(self, required_margin=None, maintenance_margin=None, slippage_rel=None,
                   slippage_abs=None, transaction_cost_rel=None, transaction_cost_abs=None):
        c = self.cfg
        if required_margin is not None:
            c.required_margin = float(required_margin)
        if maintenance_margin is not None:
            c.maintenance_margin = float(maintenance_margin)
        if slippage_rel is not None:
            c.slippage_rel = float(slippage_rel)
        if slippage_abs is not None:
            c.slippage_abs = float(slippage_abs)
        if transaction_cost_rel is not None:
            c.tc_rel = float(transaction_cost_rel)
        if transaction_cost_abs is not None:
            c.tc_abs = float(transaction_cost_abs)
        L.check(self.lib.mgn_set_broker(self.h, c.required_margin, c.maintenance_margin,
                                        c.slippage_rel, c.slippage_abs, c.tc_rel, c.tc_abs), self.h)

    def reset(self, mask=None):
        """Env::reset for every env (mask None) or the masked ones."""
        torch = _torch()
        ptr = None
        if mask is not None:
            m = self._dev(mask, torch.uint8, (self.N,), self.reset_mask_buf)
            ptr = C.c_void_p(m.data_ptr())
        L.check(self.lib.mgn_reset(self.h, ptr), self.h)

    def step(self, units=None, asset_idx=None) -> StepOutput:
        """Env::step() (units None), step(units (N,A)) or step(asset_idx (N), units (N))."""
        torch = _torch()
        if units is None:
            L.check(self.lib.mgn_step(self.h, L.STEP_NONE, None, None), self.h)
        elif asset_idx is None:
            u = self._dev(units, torch.float64, (self.N, self.A), self.units_buf)
            L.check(self.lib.mgn_step(self.h, L.STEP_UNITS, C.c_void_p(u.data_ptr()), None), self.h)
        else:
            u = self._dev(units, torch.float64, (self.N,), self.units_buf)
            ix = self._dev(asset_idx, torch.int32, (self.N,), self.asset_idx_buf)
            L.check(self.lib.mgn_step(self.h, L.STEP_SINGLE, C.c_void_p(u.data_ptr()),
                                      C.c_void_p(ix.data_ptr())), self.h)
        return self.out

    def ledger_op(self, op: int, asset_idx=None, units=None, tprice=None, tcost=None) -> dict:
        """A Broker / Portfolio operation outside a step on every env
        (mgn_ledger_op; no tick, no reward).  op: L.OP_*.  units (N, A) for
        OP_BROKER_UNITS, else (N,); asset_idx / tprice / tcost (N,).  Returns
        the responses as device tensors (tprice / tunits / tcost / risk of
        shape (N, A) for OP_BROKER_UNITS, else (N,); margin_call (N,)), valid
        until the next ledger_op."""
        torch = _torch()
        N, A = self.N, self.A
        if not hasattr(self, "_op"):
            f64, u8 = torch.float64, torch.uint8
            self._op = dict(tprice=torch.zeros((N, A), dtype=f64, device=self.device),
                            tunits=torch.zeros((N, A), dtype=f64, device=self.device),
                            tcost=torch.zeros((N, A), dtype=f64, device=self.device),
                            risk=torch.zeros((N, A), dtype=u8, device=self.device),
                            margin_call=torch.zeros((N,), dtype=u8, device=self.device))
            self._op_in = dict(tprice=torch.zeros(N, dtype=f64, device=self.device),
                               tcost=torch.zeros(N, dtype=f64, device=self.device))
            self._op_traj = self._traj_struct(self._op)
        multi = op == L.OP_BROKER_UNITS
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        u = ix = tp = tc = None
        if units is not None:
            u = self._dev(units, torch.float64, (N, A) if multi else (N,), self.units_buf)
        if asset_idx is not None:
            ix = self._dev(asset_idx, torch.int32, (N,), self.asset_idx_buf)
            bad = (ix < 0) | (ix >= A)
            if bool(bad.any()):
                raise IndexError(f"asset index out of range [0, {A})")
        if tprice is not None:
            tp = self._dev(tprice, torch.float64, (N,), self._op_in["tprice"])
        if tcost is not None:
            tc = self._dev(tcost, torch.float64, (N,), self._op_in["tcost"])
        L.check(self.lib.mgn_ledger_op(self.h, int(op), ptr(ix), ptr(u), ptr(tp), ptr(tc),
                                       C.byref(self._op_traj)), self.h)
        o = self._op
        if multi:
            return dict(o)
        return {k: (v.view(-1)[:N] if k != "margin_call" else v) for k, v in o.items()}

    def _shaped_shape(self) -> tuple:
        N, A, D, n = self.N, self.A, self.D, self.nstep
        col = (N,) if D == 1 else (N, A)
        return col if n == 1 else ((N, n) if D == 1 else (N, n, A))

    def _traj_shapes(self, K: int) -> dict:
        torch = _torch()
        N, A, D, n, F = self.N, self.A, self.D, self.nstep, self.F
        col = (N,) if D == 1 else (N, A)
        sh = col if n == 1 else ((N, n) if D == 1 else (N, n, A))
        return dict(reward=((K, N), torch.float64), agent_reward=((K,) + col, torch.float64),
                    shaped=((K,) + sh, torch.float64), done=((K, N), torch.uint8),
                    obs_price=((K, N, F), torch.float64), obs_port=((K, N, A + 1), torch.float64),
                    timestamp=((K, N), torch.int64), tprice=((K, N, A), torch.float64),
                    tunits=((K, N, A), torch.float64), tcost=((K, N, A), torch.float64),
                    risk=((K, N, A), torch.uint8), margin_call=((K, N), torch.uint8),
                    n_shaped=((K, N), torch.uint8), data_end=((K, N), torch.uint8))

    def alloc_traj(self, k_steps: int, fields=None):
        """(K, ...) device buffers for rollout outputs (None fields are skipped).
        shaped is (K,N[,A]) for n == 1 and (K,N,n[,A]) for n-step, with
        n_shaped (K,N) the number of entries popped per step."""
        torch = _torch()
        fields = L.TRAJ_FIELDS if fields is None else fields
        return {k: torch.empty(s, dtype=dt, device=self.device)
                for k, (s, dt) in self._traj_shapes(k_steps).items() if k in fields}

    def _check_traj(self, out: dict, K: int) -> None:
        """Every output the kernel will write must hold K steps of its field."""
        shapes = self._traj_shapes(K)
        for k, v in out.items():
            if v is None:
                continue
            if k not in shapes:
                raise ValueError(f"unknown output field {k!r}")
            s, dt = shapes[k]
            n = 1
            for d in s:
                n *= d
            if v.dtype != dt or v.device != self.device or not v.is_contiguous() or v.numel() < n:
                raise ValueError(f"output {k!r} must be a contiguous {dt} tensor on {self.device} "
                                 f"with >= {n} elements {s}, got {tuple(v.shape)} {v.dtype}")

    @staticmethod
    def _traj_struct(out: dict) -> L.Traj:
        t = L.Traj()
        for k in L.TRAJ_FIELDS:
            v = out.get(k)
            setattr(t, k, None if v is None else v.data_ptr())
        return t

    # caller-owned output dicts whose validated mgn_traj is kept (the most
    # recently used ones; an evicted dict is released, so a loop that builds a
    # fresh dict per launch holds at most this many)
    TRAJ_CACHE_SLOTS = 4

    def _traj_for(self, out: dict, K: int, cache: bool = True):
        """The validated mgn_traj of an output dict: validated and built once per
        (dict, K, buffer addresses), then reused, so a loop over launches with
        the same buffers pays one address comparison per launch.  cache=False
        (buffers allocated by the call itself): validate and build, keep nothing."""
        if not cache:
            self._check_traj(out, K)
            return self._traj_struct(out)
        key = (id(out), K)
        ptrs = tuple(None if v is None else v.data_ptr() for v in out.values())
        tc = self._traj_cache
        hit = tc.pop(key, None)
        if hit is not None and hit[0] is out and hit[1] == ptrs:
            tc[key] = hit  # most recently used last
            return hit[2]
        self._check_traj(out, K)
        t = self._traj_struct(out)
        tc[key] = (out, ptrs, t, C.byref(t))
        while len(tc) > self.TRAJ_CACHE_SLOTS:
            tc.pop(next(iter(tc)))
        return t

    def rollout(self, actions, out: Optional[dict] = None) -> dict:
        """K fused steps from discrete actions (K,N,A) int8 via action_to_transaction."""
        torch = _torch()
        if not (isinstance(actions, torch.Tensor) and actions.device == self.device
                and actions.dtype == torch.int8 and actions.is_contiguous()):
            actions = torch.as_tensor(actions).to(self.device, torch.int8).contiguous()
        if actions.dim() != 3 or actions.shape[1] != self.N or actions.shape[2] != self.A:
            raise ValueError(f"actions must be (K, {self.N}, {self.A}), got {tuple(actions.shape)}")
        K = int(actions.shape[0])
        own = out is None
        out = self.alloc_traj(K) if own else out
        t = self._traj_for(out, K, cache=not own)
        L.check(self.lib.mgn_rollout(self.h, C.c_void_p(actions.data_ptr()), K, C.byref(t)), self.h)
        return out

    def rollout_launcher(self, out: dict, k_steps: int, actions=None):
        """A launcher for repeated K-step rollouts into the same output buffers,
        with the mgn_traj validated once here (the per-launch host work is the
        call itself).  The caller keeps ``out`` (and ``actions``) alive.

        With ``actions`` -- a (T, N, A) int8 device tensor, T >= K -- the
        launcher is ``launch(t)``: K steps from rows [t, t + K) of it, t checked
        against T - K on every call.  Without it, ``launch(actions_ptr)`` reads
        (K, N, A) int8 at a raw device address the caller vouches for (an
        address whose buffer holds fewer than K steps is read past its end:
        round 4's bench fault)."""
        torch = _torch()
        K = int(k_steps)
        t = self._traj_for(out, K)
        pc = L.pycall()
        if pc is not None:  # the CPython binding: no ctypes conversion per call
            f, hv, tv = pc.rollout, self.h.value, C.addressof(t)

            def raw(actions_ptr: int) -> int:
                return f(hv, actions_ptr, K, tv)
        else:
            ref = C.byref(t)
            fn, h = self.lib.mgn_rollout, self.h

            def raw(actions_ptr: int) -> int:
                return fn(h, actions_ptr, K, ref)
        if actions is None:
            raw._keep = t  # the mgn_traj the address points at
            return raw
        if not (isinstance(actions, torch.Tensor) and actions.device == self.device
                and actions.dtype == torch.int8 and actions.is_contiguous() and actions.dim() == 3
                and actions.shape[1] == self.N and actions.shape[2] == self.A):
            raise ValueError(f"actions must be a contiguous (T, {self.N}, {self.A}) int8 tensor on {self.device}")
        T = int(actions.shape[0])
        if T < K:
            raise ValueError(f"actions hold {T} steps, a launch reads {K}")
        base, row, tmax = actions.data_ptr(), self.N * self.A, T - K

        def launch(t0: int) -> int:
            if not 0 <= t0 <= tmax:
                raise IndexError(f"launch at step {t0}: rows [{t0}, {t0 + K}) outside the {T} action steps")
            return raw(base + t0 * row)
        launch._keep = (t, actions)
        return launch

    def stream_synchronizer(self, spin: bool = False):
        """A zero-argument callable that waits for the handle's stream
        (mgn_synchronize) -- every launch of the handle is on it -- rather than
        the whole device (torch.cuda.synchronize); returns the status code.
        spin: poll the stream instead (mgn_synchronize_spin: the thread
        busy-waits), for short waits such as an agent loop's per step."""
        name = "synchronize_spin" if spin else "synchronize"
        pc = L.pycall()
        if pc is not None and hasattr(pc, name):
            f, hv = getattr(pc, name), self.h.value
            return lambda: f(hv)
        fn, h = getattr(self.lib, "mgn_" + name), self.h
        return lambda: fn(h)

    # ---- Env::setDataSource / checkpoint --------------------------------------------
    def set_sources(self, spec: SourceSpec, prices=None):
        """Env::setDataSource for every env (Env.h:174-179): swap the price
        source in place and keep the portfolios.  spec: per asset
        MGN_SRC_EXTERNAL (host prices through set_prices before each tick) or
        the current kind with new parameters; prices (N,A): the new source's
        currentPrices (None keeps the device prices)."""
        torch = _torch()
        if spec.n_assets != self.A:
            raise ValueError(f"the new source has {spec.n_assets} assets, the env {self.A}")
        srcs = (L.AssetSource * self.A)()
        for i, (k, p) in enumerate(zip(spec.kinds, spec.params)):
            srcs[i].kind = k
            for j, v in enumerate(p):
                srcs[i].p[j] = v
        ptr = None
        if prices is not None:
            stage = torch.empty((self.N, self.A), dtype=torch.float64, device=self.device)
            ptr = C.c_void_p(self._dev(prices, torch.float64, (self.N, self.A), stage).data_ptr())
        L.check(self.lib.mgn_set_sources(self.h, srcs, ptr), self.h)
        self.spec = spec

    def state_dict(self) -> dict:
        """The handle's whole state (mgn_save_state) as a host uint8 array plus
        the library ABI: every episode resumes bit-exactly after load_state_dict."""
        n = int(self.lib.mgn_state_bytes(self.h))
        blob = np.empty(n, dtype=np.uint8)
        L.check(self.lib.mgn_save_state(self.h, blob.ctypes.data_as(C.c_void_p), n), self.h)
        return {"state": blob, "abi": L.ABI_VERSION}

    def load_state_dict(self, sd: dict) -> None:
        blob = np.ascontiguousarray(sd["state"], dtype=np.uint8)
        if int(sd.get("abi", L.ABI_VERSION)) != L.ABI_VERSION:
            raise RuntimeError("state_dict of another ABI version")
        L.check(self.lib.mgn_load_state(self.h, blob.ctypes.data_as(C.c_void_p), blob.nbytes), self.h)
        c = L.Config()
        C.memmove(C.byref(c), blob.ctypes.data + 24, C.sizeof(c))
        self.cfg = c

    def rollout_units(self, units, out: Optional[dict] = None) -> dict:
        """K fused Env::step(units) from units (K,N,A) fp64."""
        torch = _torch()
        u = torch.as_tensor(units).to(self.device, torch.float64).contiguous()
        if u.dim() != 3 or u.shape[1] != self.N or u.shape[2] != self.A:
            raise ValueError(f"units must be (K, {self.N}, {self.A}), got {tuple(u.shape)}")
        K = int(u.shape[0])
        own = out is None
        out = self.alloc_traj(K) if own else out
        t = self._traj_for(out, K, cache=not own)
        L.check(self.lib.mgn_rollout_units(self.h, C.c_void_p(u.data_ptr()), K, C.byref(t)), self.h)
        return out

    def generate_actions(self, k_steps: int, seed: int = 0x6D6164):
        torch = _torch()
        a = torch.empty((k_steps, self.N, self.A), dtype=torch.int8, device=self.device)
        L.check(self.lib.mgn_generate_actions(self.h, C.c_void_p(a.data_ptr()), k_steps, seed), self.h)
        return a

    def set_prices(self, prices):
        torch = _torch()
        p = self._dev(prices, torch.float64, (self.N, self.A), self.ext_prices)
        if p.data_ptr() != self.ext_prices.data_ptr():
            L.check(self.lib.mgn_set_prices(self.h, C.c_void_p(p.data_ptr())), self.h)

    def valuation(self) -> dict:
        """Portfolio accessors for every env as (N,) device tensors."""
        L.check(self.lib.mgn_valuation(self.h, C.c_void_p(self._val.data_ptr())), self.h)
        return {k: self._val[:, i] for i, k in enumerate(VALUATION_FIELDS)}

    def window(self):
        """StackerDiscrete.current_data of the handle's ring: (N,W,A), (N,W,A+1), (N,W)."""
        if not self.W:
            raise RuntimeError("env built with window=0")
        L.check(self.lib.mgn_window(self.h, None, None, None), self.h)
        return self.win_price, self.win_port, self.win_ts

    def rollout_window(self, actions, out: Optional[dict] = None, per_step: bool = False):
        """The agent loop of a windowed env in one native call (mgn_rollout_window):
        per step k, step k of `rollout(actions)` then `window()`.  Returns the
        trajectory and the window: the last step's (N,W,·) views of the handle's
        buffers, or with per_step=True fresh (K,N,W,·) tensors of every step's."""
        torch = _torch()
        if not self.W:
            raise RuntimeError("env built with window=0")
        if not (isinstance(actions, torch.Tensor) and actions.device == self.device
                and actions.dtype == torch.int8 and actions.is_contiguous()):
            actions = torch.as_tensor(actions).to(self.device, torch.int8).contiguous()
        if actions.dim() != 3 or actions.shape[1] != self.N or actions.shape[2] != self.A:
            raise ValueError(f"actions must be (K, {self.N}, {self.A}), got {tuple(actions.shape)}")
        K = int(actions.shape[0])
        out = self.alloc_traj(K) if out is None else out
        self._check_traj(out, K)
        t = self._traj_struct(out)
        if per_step:
            wp = torch.empty((K,) + tuple(self.win_price.shape), dtype=torch.float64, device=self.device)
            wo = torch.empty((K,) + tuple(self.win_port.shape), dtype=torch.float64, device=self.device)
            wt = torch.empty((K,) + tuple(self.win_ts.shape), dtype=self.win_ts.dtype, device=self.device)
            ptrs = [C.c_void_p(x.data_ptr()) for x in (wp, wo, wt)]
            win = (wp, wo, wt)
        else:
            ptrs = [None, None, None]
            win = (self.win_price, self.win_port, self.win_ts)
        L.check(self.lib.mgn_rollout_window(self.h, C.c_void_p(actions.data_ptr()), K, C.byref(t),
                                            *ptrs, int(per_step)), self.h)
        return out, win

    def window_hist_view(self) -> dict:
        """The last mgn_rollout_hist's launch history, read in place
        (mgn_window_hist_view; norm none / log): window k of env e is rows
        [hend[k, e] - hlen[k, e], hend[k, e]) of ``hist[e]`` (price columns
        first, then ledgerNormedFull), zero-padded to W rows.  Device tensors
        over the handle's buffers, valid until the next rollout_window /
        mgn_rollout_hist; no copy is made."""
        torch = _torch()
        v = L.HistView()
        L.check(self.lib.mgn_window_hist_view(self.h, C.byref(v)), self.h)

        class _Dev:  # __cuda_array_interface__ over the library's device buffer
            def __init__(self, ptr, shape, typestr):
                self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False),
                                                 "version": 2, "strides": None}

        def dev(ptr, shape, typestr):
            return torch.as_tensor(_Dev(int(ptr), shape, typestr), device=self.device)
        N, K = self.N, int(v.k_steps)
        return dict(hist=dev(v.hist, (N, int(v.rows), int(v.cols)), "<f8"),
                    hist_ts=dev(v.hist_ts, (N, int(v.rows)), "<i8"),
                    hend=dev(v.hend, (K, N), "<i4"), hlen=dev(v.hlen, (K, N), "<i4"),
                    window=int(v.window), n_feats=int(v.n_feats))

    @staticmethod
    def window_from_view(view: dict, k: int):
        """Window k of every env from a window_hist_view, as (N, W, F),
        (N, W, A+1), (N, W) tensors (a consumer-side gather; what
        mgn_window_hist writes)."""
        torch = _torch()
        hist, W, F = view["hist"], view["window"], view["n_feats"]
        end = view["hend"][k].long()
        ln = view["hlen"][k].long()
        w = torch.arange(W, device=hist.device)
        rows = (end - ln)[:, None] + w[None, :]
        ok = w[None, :] < ln[:, None]
        rows = torch.where(ok, rows, torch.zeros_like(rows))
        g = torch.gather(hist, 1, rows[:, :, None].expand(-1, -1, hist.shape[2]))
        g = torch.where(ok[:, :, None], g, torch.zeros((), dtype=g.dtype, device=g.device))
        ts = torch.gather(view["hist_ts"], 1, rows)
        ts = torch.where(ok, ts, torch.zeros((), dtype=ts.dtype, device=ts.device))
        return g[:, :, :F], g[:, :, F:], ts

    def window_push(self, price=None, port=None, ts=None):
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        L.check(self.lib.mgn_window_push(self.h, ptr(price), ptr(port), ptr(ts)), self.h)

    def window_clear(self, mask=None):
        torch = _torch()
        ptr = None
        if mask is not None:
            m = self._dev(mask, torch.uint8, (self.N,), self.reset_mask_buf)
            ptr = C.c_void_p(m.data_ptr())
        L.check(self.lib.mgn_window_clear(self.h, ptr), self.h)

    def synchronize(self):
        L.check(self.lib.mgn_synchronize(self.h), self.h)

    def host_outputs(self) -> dict:
        """One D2H copy of the whole step-output block, sliced into numpy arrays."""
        lo, hi = self._out_span
        blob = self.arena[lo:hi].cpu().numpy()
        base = self.arena.data_ptr() + lo
        N, A, D, F = self.N, self.A, self.D, self.F
        o = self._v.out
        def arr(ptr, dtype, shape):  # noqa: E306
            off = ptr - base
            n = int(np.prod(shape)) * np.dtype(dtype).itemsize
            return blob[off:off + n].view(dtype).reshape(shape)
        Dsh = (N,) if D == 1 else (N, A)
        return dict(reward=arr(o.reward, np.float64, (N,)), agent_reward=arr(o.agent_reward, np.float64, Dsh),
                    shaped=arr(o.shaped, np.float64, self._shaped_shape()),
                    n_shaped=arr(o.n_shaped, np.uint8, (N,)), done=arr(o.done, np.uint8, (N,)),
                    obs_price=arr(o.obs_price, np.float64, (N, F)),
                    obs_port=arr(o.obs_port, np.float64, (N, A + 1)),
                    timestamp=arr(o.timestamp, np.uint64, (N,)), tprice=arr(o.tprice, np.float64, (N, A)),
                    tunits=arr(o.tunits, np.float64, (N, A)), tcost=arr(o.tcost, np.float64, (N, A)),
                    risk=arr(o.risk, np.uint8, (N, A)), margin_call=arr(o.margin_call, np.uint8, (N,)),
                    data_end=arr(o.data_end, np.uint8, (N,)))


# ---------------------------------------------------------------------------
# Drop-in single Env (pybind11 module surface, env.cpp:843-1005)


class DataSourceTick:
    """Plug-in base class for host data sources (DataSource.h:48-64).

    Subclass and override getData()/currentPrices(); pass an instance to
    Env.setDataSource (PyDataSource trampoline, PyDataSource.h:9-24).  Its
    prices are streamed to the device as the external source of every asset.
    """

    def getData(self):
        raise NotImplementedError

    def currentData(self):
        return self.currentPrices()

    def currentPrices(self):
        raise NotImplementedError

    def reset(self):
        pass

    def currentTime(self):
        return 0

    def dataEnd(self):
        return False

    @property
    def nAssets(self):
        return len(np.asarray(self.currentPrices()))

    @property
    def nFeats(self):
        return len(np.asarray(self.currentData()))

    @property
    def assets(self):
        return [Asset(f"asset_{i}") for i in range(self.nAssets)]


class _DeviceSourceView:
    """Env.dataSource for the device generators (read-only view)."""

    def __init__(self, env):
        self._env = env

    def currentData(self):
        return self._env.currentData.copy()

    def currentPrices(self):
        return self._env.currentPrices.copy()

    def currentTime(self):
        return self._env.timestamp

    def dataEnd(self):
        return self._env.dataEnd()

    @property
    def nAssets(self):
        return self._env.nAssets

    @property
    def nFeats(self):
        return self._env.nFeats

    @property
    def assets(self):
        return self._env.assets


class PortfolioView:
    """Env.portfolio / Env.account: the default Portfolio (env.cpp:440-570).

    Accessors read the Env's state; handleTransaction / close mutate the
    device ledger directly (Portfolio.cpp:284-333, no risk check, no tick)."""

    def __init__(self, env):
        self._env = env

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._env, name)

    def _idx(self, asset):
        return self._env._asset_index(asset)

    def checkRisk(self, *args):
        """checkRisk() (Portfolio.cpp:243-252) or checkRisk(assetIdx | assetCode,
        units) (:254-279)."""
        if len(args) == 0:
            return self._env.checkRisk()
        if len(args) != 2:
            raise TypeError("checkRisk() takes () or (assetIdx | assetCode, units)")
        e = self._env
        r = e._b.ledger_op(L.OP_CHECK_ORDER, asset_idx=[self._idx(args[0])], units=[float(args[1])])
        return RiskInfo(int(r["risk"][0].item()))

    def handleTransaction(self, asset, transactionPrice, units, transactionCost=0.0):
        """Portfolio::handleTransaction(assetIdx | asset, transactionPrice, units,
        transactionCost=0.) (Portfolio.cpp:284-323): the accounting alone."""
        e = self._env
        e._b.ledger_op(L.OP_PORT_TXN, asset_idx=[self._idx(asset)], units=[float(units)],
                       tprice=[float(transactionPrice)], tcost=[float(transactionCost)])
        e._dirty()

    def close(self, assetIdx, transactionPrice, transactionCost=0.0):
        """Portfolio::close(assetIdx, transactionPrice, transactionCost=0.)
        (Portfolio.cpp:327-333): sell / cover the whole position, if any."""
        e = self._env
        e._b.ledger_op(L.OP_PORT_CLOSE, asset_idx=[self._idx(assetIdx)],
                       tprice=[float(transactionPrice)], tcost=[float(transactionCost)])
        e._dirty()

    def setRequiredMargin(self, requiredMargin):
        self._env.setRequiredMargin(requiredMargin)

    def setMaintenanceMargin(self, maintenanceMargin):
        self._env.setMaintenanceMargin(maintenanceMargin)


class BrokerView:
    """Env.broker: the Env's Broker (Broker.h, env.cpp:700-840) over the
    default account and portfolio.  Orders run the reference's risk checks,
    slippage and transaction cost on the device ledger, without a tick."""

    def __init__(self, env):
        self._env = env

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._env, name)

    def _multi(self, units):
        e = self._env
        u = np.asarray(units, dtype=np.float64).reshape(-1)
        if u.shape[0] != e.nAssets:
            raise ValueError(f"units must have {e.nAssets} entries, got {u.shape[0]}")
        r = e._b.ledger_op(L.OP_BROKER_UNITS, units=u.reshape(1, -1))
        e._dirty()
        h = {k: v.cpu().numpy() for k, v in r.items()}
        return BrokerResponse(h["tprice"][0].copy(), h["tunits"][0].copy(), h["tcost"][0].copy(),
                              [RiskInfo(int(x)) for x in h["risk"][0]], bool(h["margin_call"][0]))

    def _single(self, op, asset, units=None):
        e = self._env
        r = e._b.ledger_op(op, asset_idx=[e._asset_index(asset)],
                           units=None if units is None else [float(units)])
        e._dirty()
        h = {k: v.cpu().numpy() for k, v in r.items()}
        return BrokerResponse(float(h["tprice"][0]), float(h["tunits"][0]), float(h["tcost"][0]),
                              RiskInfo(int(h["risk"][0])), bool(h["margin_call"][0]))

    def handleTransaction(self, *args):
        """handleTransaction(units) -> BrokerResponseMulti (Broker.cpp:144-158);
        handleTransaction(assetIdx | assetCode, units) -> BrokerResponseSingle
        (:124-142)."""
        if len(args) == 1:
            return self._multi(args[0])
        if len(args) == 2:
            return self._single(L.OP_BROKER_SINGLE, args[0], args[1])
        raise TypeError("handleTransaction takes (units) or (assetIdx | assetCode, units) "
                        "on the Env's default account / portfolio")

    def handleAction(self, units):
        """Broker::handleAction (Broker.h:99-101): handleTransaction(units)."""
        return self._multi(units)

    def handleEvent(self, units):
        """Broker::handleEvent (Broker.h:95-97): handleTransaction(units)."""
        return self._multi(units)

    def close(self, assetIdx):
        """Broker::close(assetIdx) (Broker.cpp:160-169): close the position at
        the current price with slippage and transaction cost; always green."""
        return self._single(L.OP_BROKER_CLOSE, assetIdx)

    def portfolio(self, *args):
        return PortfolioView(self._env)

    def account(self, *args):
        return PortfolioView(self._env)

    def setSlippage(self, relativeSlippage=0.0, absSlippage=0.0):
        self._env.setSlippage(relativeSlippage, absSlippage)

    def setTransactionCost(self, relativeCost=0.0, absCost=0.0):
        self._env.setTransactionCost(relativeCost, absCost)


class Env:
    """Drop-in for madigan.environments.cpp.Env (one env on the GPU).

    Host reads go through one snapshot per state change: the first step or
    accessor after a launch runs k_valuation and copies the handle's arena
    and the valuation row to pinned host memory with one stream synchronise;
    every accessor until the next mutating call reads that snapshot (the
    reference agent reads equity, availableMargin, currentPrices, ledger, ...
    around every step, offpolicy_q.py:140-164, dqn.py:165-176)."""

    def __init__(self, dataSourceType: str, initCash: float = 1_000_000.0, config_dict=None, *,
                 device=None, seed: int = 0):
        self._type = dataSourceType
        if config_dict is not None and len(dict(config_dict)) > 0:
            cfg = dict(config_dict)
            cfg.setdefault("data_source_type", dataSourceType)
            spec = spec_from_config(cfg)
        else:
            spec = default_spec(dataSourceType)
        self._init_cash = float(initCash)
        self._device = device
        self._seed = seed
        self._source = None
        # Env::requiredMargin_ / maintenanceMargin_ default to 0 (Env.h:131-132)
        self._broker = dict(required_margin=0.0, maintenance_margin=0.0, slippage_rel=0.0,
                            slippage_abs=0.0, transaction_cost_rel=0.0, transaction_cost_abs=0.0)
        self._spec = spec
        self._b = BatchedEnv(spec, 1, device=self._device, seed=self._seed,
                             init_cash=self._init_cash, **self._broker)
        self._init_snapshot()
        self._snap = None
        self._vsnap = None

    def _init_snapshot(self):
        """The pinned host image of the handle's arena + valuation row and numpy
        views of the fields the accessors read, built once (the snapshot then
        costs one valuation launch, one copy and one synchronise)."""
        torch = _torch()
        b = self._b
        n = b._val_off + 80
        self._h_buf = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        blob = self._h_buf.numpy()
        base = b.arena.data_ptr()

        def arr(ptr, dtype, shape):
            off = ptr - base
            k = int(np.prod(shape)) * np.dtype(dtype).itemsize
            return blob[off:off + k].view(dtype).reshape(shape)
        v, A, F = b._v, b.A, b.F
        o = v.out
        # step inputs read by the kernel in place from pinned host memory (Env.step
        # synchronises before it returns, so the next write never races a read)
        self._h_units = torch.zeros(max(A, 1), dtype=torch.float64, pin_memory=True)
        self._h_aidx = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._d_units = L.device_view(self._h_units.data_ptr())
        self._d_aidx = L.device_view(self._h_aidx.data_ptr())
        self._h_views = dict(
            val=blob[b._val_off:b._val_off + 80].view(np.float64),
            prices=arr(v.prices, np.float64, (A,)), ledger=arr(v.ledger, np.float64, (A,)),
            mean_entry=arr(v.mean_entry, np.float64, (A,)), timestamp=arr(v.timestamp, np.uint64, (1,)),
            reward=arr(o.reward, np.float64, (1,)), done=arr(o.done, np.uint8, (1,)),
            obs_price=arr(o.obs_price, np.float64, (F,)), obs_port=arr(o.obs_port, np.float64, (A + 1,)),
            obs_ts=arr(o.timestamp, np.uint64, (1,)), tprice=arr(o.tprice, np.float64, (A,)),
            tunits=arr(o.tunits, np.float64, (A,)), tcost=arr(o.tcost, np.float64, (A,)),
            risk=arr(o.risk, np.uint8, (A,)), margin_call=arr(o.margin_call, np.uint8, (1,)))

    # ---- host snapshot of the device state ------------------------------------------
    def _dirty(self):
        self._snap = None
        self._vsnap = None

    def _snapshot(self) -> dict:
        if self._snap is not None:
            return self._snap
        b = self._b
        hip = L.hip()
        st = C.c_void_p(b.stream.cuda_stream)
        if hip.hipMemcpyAsync(C.c_void_p(self._h_buf.data_ptr()), C.c_void_p(b._arena_buf.data_ptr()),
                              C.c_size_t(b._val_off), 2, st) != 0 or \
                hip.hipStreamSynchronize(st) != 0:  # hipMemcpyDeviceToHost
            raise RuntimeError("snapshot copy failed")
        h = self._h_views
        # the arrays stay views of the pinned image: State / accessors copy them
        self._snap = dict(h, timestamp=int(h["timestamp"][0]), reward=float(h["reward"][0]),
                          done=bool(h["done"][0]), obs_ts=int(h["obs_ts"][0]),
                          margin_call=bool(h["margin_call"][0]))
        return self._snap

    def _valuation(self) -> dict:
        """Portfolio valuation (k_valuation) of the current state, launched
        only when an accessor needs it (Env.step's own returns do not)."""
        if self._vsnap is not None:
            return self._vsnap
        b = self._b
        L.check(b.lib.mgn_valuation(b.h, C.c_void_p(b._val.data_ptr())), b.h)
        hip = L.hip()
        st = C.c_void_p(b.stream.cuda_stream)
        if hip.hipMemcpyAsync(C.c_void_p(self._h_buf.data_ptr() + b._val_off), C.c_void_p(b._val.data_ptr()),
                              C.c_size_t(80), 2, st) != 0 or hip.hipStreamSynchronize(st) != 0:
            raise RuntimeError("valuation copy failed")
        self._vsnap = dict(zip(VALUATION_FIELDS, self._h_views["val"].tolist()))
        return self._vsnap

    # ---- setters (Env.h:94-111) ------------------------------------------------
    def setRequiredMargin(self, requiredMargin):
        self._broker["required_margin"] = float(requiredMargin)
        self._b.set_broker(required_margin=requiredMargin)
        self._dirty()

    def setMaintenanceMargin(self, maintenanceMargin):
        self._broker["maintenance_margin"] = float(maintenanceMargin)
        self._b.set_broker(maintenance_margin=maintenanceMargin)
        self._dirty()

    def setSlippage(self, relativeSlippage=0.0, absSlippage=0.0):
        self._broker.update(slippage_rel=float(relativeSlippage), slippage_abs=float(absSlippage))
        self._b.set_broker(slippage_rel=relativeSlippage, slippage_abs=absSlippage)

    def setTransactionCost(self, relativeCost=0.0, absCost=0.0):
        self._broker.update(transaction_cost_rel=float(relativeCost),
                            transaction_cost_abs=float(absCost))
        self._b.set_broker(transaction_cost_rel=relativeCost, transaction_cost_abs=absCost)

    def setDataSource(self, dataSource):
        """Env::setDataSource (Env.h:174-179): the host DataSourceTick becomes the
        source of every asset; the Broker / Portfolio (ledger, cash, mean entry,
        borrowed margin) are kept and value the portfolio at the new source's
        currentPrices() from now on.  Its getData() runs before every step's
        tick (PyDataSource trampoline, PyDataSource.h:9-15)."""
        if self._spec.replay:
            raise RuntimeError("setDataSource: a replay Env cannot switch its data source")
        prices = np.asarray(dataSource.currentPrices(), dtype=np.float64).reshape(-1)
        if prices.shape[0] != self.nAssets:
            raise ValueError(f"the data source has {prices.shape[0]} assets, the Env {self.nAssets}")
        spec = SourceSpec(kinds=[L.SRC_EXTERNAL] * self.nAssets, params=[[]] * self.nAssets,
                          assets=list(self._spec.assets))
        self._b.set_sources(spec, prices.reshape(1, -1))
        self._source = dataSource
        self._spec = spec
        self._dirty()

    # ---- stepping -----------------------------------------------------------------
    def _feed_external(self):
        if self._source is not None:
            p = np.asarray(self._source.getData(), dtype=np.float64).reshape(1, -1)
            self._b.set_prices(p)

    def _state(self, o):
        return State(o["obs_price"].copy(), o["obs_port"].copy(), o["obs_ts"])

    def reset(self):
        if self._source is not None:
            self._source.reset()
            self._feed_external()
        self._b.reset()
        self._dirty()
        s = self._snapshot()
        return State(self.currentData.copy(), self.ledgerNormedFull, s["timestamp"])

    def step(self, *args):
        if len(args) == 0:
            self._feed_external()
            self._b.step()
            self._dirty()
            o = self._snapshot()
            return self._state(o), o["reward"], o["done"], EnvInfo(
                BrokerResponse(0.0, 0.0, 0.0, RiskInfo.green, False), self.dataEnd())
        if len(args) == 2:
            idx, units = args
            if isinstance(idx, str):
                codes = [a.code for a in self.assets]
                if idx not in codes:
                    raise IndexError(f"asset code {idx} not found")
                idx = codes.index(idx)
            idx = int(idx)
            if not 0 <= idx < self.nAssets:
                raise IndexError(f"asset index {idx} out of range")
            self._feed_external()
            if self._d_units and self._d_aidx:
                self._h_units.numpy()[0] = float(units)
                self._h_aidx.numpy()[0] = idx
                b = self._b
                L.check(b.lib.mgn_step(b.h, L.STEP_SINGLE, C.c_void_p(self._d_units),
                                       C.c_void_p(self._d_aidx)), b.h)
            else:
                self._b.step(units=np.array([float(units)]), asset_idx=np.array([idx], np.int32))
            self._dirty()
            o = self._snapshot()
            resp = BrokerResponse(float(o["tprice"][idx]), float(o["tunits"][idx]),
                                  float(o["tcost"][idx]), RiskInfo(int(o["risk"][idx])),
                                  o["margin_call"])
            return self._state(o), o["reward"], o["done"], EnvInfo(resp, self.dataEnd())
        if len(args) == 1:
            units = np.asarray(args[0], dtype=np.float64).reshape(-1)
            if units.shape[0] != self.nAssets:
                raise ValueError(f"units must have {self.nAssets} entries, got {units.shape[0]}")
            self._feed_external()
            if self._d_units:
                self._h_units.numpy()[:self.nAssets] = units
                b = self._b
                L.check(b.lib.mgn_step(b.h, L.STEP_UNITS, C.c_void_p(self._d_units), None), b.h)
            else:
                self._b.step(units=units.reshape(1, -1))
            self._dirty()
            o = self._snapshot()
            resp = BrokerResponse(o["tprice"].copy(), o["tunits"].copy(), o["tcost"].copy(),
                                  [RiskInfo(int(r)) for r in o["risk"]], o["margin_call"])
            return self._state(o), o["reward"], o["done"], EnvInfo(resp, self.dataEnd())
        raise TypeError("step() takes (), (units), (assetIdx, units) or (assetCode, units)")

    # ---- accessors (env.cpp:872-969) --------------------------------------------------
    def _vals(self):
        return self._valuation()

    @property
    def currentPrices(self):
        return self._snapshot()["prices"].copy()

    def _replay_row(self):
        b = self._b
        rows = b._tape["ts"].shape[0]
        return (int(b.replay_cursor[0].item()) - 1) % rows

    @property
    def currentData(self):
        """Env::currentData (Env.h:52): the source's features (= prices for the generators)."""
        if self._spec.replay:
            return self._b._tape["feats"][self._replay_row()].cpu().numpy()
        return self.currentPrices

    @property
    def ledger(self):
        return self._snapshot()["ledger"].copy()

    @property
    def meanEntryPrices(self):
        return self._snapshot()["mean_entry"].copy()

    @property
    def timestamp(self):
        return self._snapshot()["timestamp"]

    currentTime = timestamp

    @property
    def equity(self):
        return float(self._vals()["equity"])

    @property
    def cash(self):
        return float(self._vals()["cash"])

    @property
    def pnl(self):
        return float(self._vals()["pnl"])

    @property
    def balance(self):
        return float(self._vals()["balance"])

    @property
    def availableMargin(self):
        return float(self._vals()["availableMargin"])

    @property
    def usedMargin(self):
        return float(self._vals()["usedMargin"])

    @property
    def borrowedMargin(self):
        return float(self._vals()["borrowedMargin"])

    @property
    def borrowedAssetValue(self):
        return float(self._vals()["borrowedAssetValue"])

    @property
    def assetValue(self):
        return float(self._vals()["assetValue"])

    @property
    def requiredMargin(self):
        return self._broker["required_margin"]

    @property
    def maintenanceMargin(self):
        return self._broker["maintenance_margin"]

    @property
    def positionValues(self):
        return self.ledger * self.currentPrices

    @property
    def pnlPositions(self):
        return self.positionValues - self.meanEntryPrices * self.ledger

    @property
    def positionValuesFull(self):
        v = self._vals()
        return np.concatenate([[v["cash"] - v["borrowedMargin"]], self.positionValues])

    @property
    def ledgerFull(self):
        v = self._vals()
        return np.concatenate([[v["cash"] - v["borrowedMargin"]], self.ledger])

    @property
    def ledgerNormed(self):
        return self.positionValues / self._vals()["equity"]

    @property
    def ledgerNormedFull(self):
        v = self._vals()
        eq = v["equity"]
        return np.concatenate([[(v["cash"] - v["borrowedMargin"]) / eq], self.positionValues / eq])

    @property
    def ledgerAbsNormed(self):
        ln = self.ledgerNormed
        return ln / np.abs(ln).sum()

    @property
    def ledgerAbsNormedFull(self):
        ln = self.ledgerNormedFull
        return ln / np.abs(ln).sum()

    @property
    def nAssets(self):
        return self._spec.n_assets

    @property
    def nFeats(self):
        return self._b.F

    @property
    def assets(self):
        return [Asset(a) for a in self._spec.assets]

    @property
    def isDateTime(self):
        return self._spec.replay  # HDFSourceSingle::isDateTime (DataSource.h:124)

    @property
    def dataSource(self):
        return self._source if self._source is not None else _DeviceSourceView(self)

    @property
    def portfolio(self):
        return PortfolioView(self)

    @property
    def broker(self):
        return BrokerView(self)

    def _asset_index(self, asset) -> int:
        """An asset index or code -> index; IndexError out of range (the
        reference's std::out_of_range, envTest.py:246-248)."""
        if isinstance(asset, str):
            codes = [a.code for a in self.assets]
            if asset not in codes:
                raise IndexError(f"asset code {asset} not found")
            return codes.index(asset)
        idx = int(asset)
        if not 0 <= idx < self.nAssets:
            raise IndexError(f"asset index {idx} out of range")
        return idx

    @property
    def account(self):
        return PortfolioView(self)

    def dataEnd(self):
        """Env::dataEnd (Env.h:58) -> DataSource::dataEnd (DataSource.h:61, :126)."""
        if self._source is not None:
            return bool(self._source.dataEnd())
        if self._spec.replay:
            return bool(self._b._tape["data_end"][self._replay_row()].item())
        return False

    def checkRisk(self):
        return RiskInfo(int(self._vals()["checkRisk"]))

    @property
    def batched(self) -> BatchedEnv:
        return self._b


# ---------------------------------------------------------------------------
# madigan/environments/__init__.py surface


def _cfg_get(config: Any, key: str, default=None):
    if isinstance(config, dict):
        return config.get(key, default)
    return getattr(config, key, default)


def make_env(config, test: bool = False, **kw) -> Env:
    """make_env (madigan/environments/__init__.py:9-22)."""
    config = adjust_config(config, test)
    if config.get("env_type", "Synth") in ("Synth",):
        if config.get("data_source_config") is not None:
            env = Env(config["data_source_type"], config["init_cash"], config, **kw)
        else:
            env = Env(config["data_source_type"], config["init_cash"], **kw)
        env.setRequiredMargin(config["required_margin"])
        env.setMaintenanceMargin(config["maintenance_margin"])
        env.setTransactionCost(config["transaction_cost_rel"], config["transaction_cost_abs"])
        env.setSlippage(config["slippage_rel"], config["slippage_abs"])
        return env
    raise NotImplementedError(f"Env type {config.get('env_type')} not implemented")


def adjust_config(config, test: bool = False) -> dict:
    """adjust_config (madigan/environments/__init__.py:25-37): the test data
    config, and HDFSourceSingle start/end times as pd.to_datetime(x).value."""
    import copy
    config = copy.deepcopy(dict(config))
    if test and "data_source_config_test" in config:
        config["data_source_config"] = config["data_source_config_test"]
    if config.get("data_source_type") == "HDFSourceSingle" and config.get("data_source_config"):
        import pandas as pd
        dsc = dict(config["data_source_config"])
        for key in ("start_time", "end_time"):
            if key in dsc:
                dsc[key] = int(pd.to_datetime(dsc[key]).value)
        config["data_source_config"] = dsc
    return config


def make_batched_env(config, n_envs: int, **kw) -> BatchedEnv:
    """BatchedEnv from a reference experiment config (env, preprocessor and
    reward-shaper keys: madigan/utils/config.py:104-115, config.yaml:280-310)."""
    spec = spec_from_config(config)
    pconf = _cfg_get(config, "preprocessor_config") or {}
    rconf = _cfg_get(config, "reward_shaper_config") or {}
    window = int(kw.pop("window", _cfg_get(pconf, "window_length", 0) or 0))
    norm = _cfg_get(pconf, "norm", False)
    norm_type = kw.pop("norm_type", _cfg_get(pconf, "norm_type", None) if norm else None)
    shaper = kw.pop("reward_shaper", _cfg_get(rconf, "reward_shaper", None))
    aconf = _cfg_get(config, "agent_config") or {}
    nstep = int(kw.pop("nstep_return", _cfg_get(aconf, "nstep_return", 1) or 1))
    discount = float(kw.pop("discount", _cfg_get(aconf, "discount", 0.99)))
    unit = kw.pop("unit_size", _cfg_get(aconf, "unit_size_proportion_avM", 0.05))
    atoms = int(kw.pop("action_atoms", _cfg_get(aconf, "action_atoms", 3) or 3))
    return BatchedEnv(
        spec, n_envs, init_cash=_cfg_get(config, "init_cash", 1_000_000.0),
        required_margin=_cfg_get(config, "required_margin", 1.0),
        maintenance_margin=_cfg_get(config, "maintenance_margin", 0.25),
        slippage_rel=_cfg_get(config, "slippage_rel", 0.0),
        slippage_abs=_cfg_get(config, "slippage_abs", 0.0),
        transaction_cost_rel=_cfg_get(config, "transaction_cost_rel", 0.0),
        transaction_cost_abs=_cfg_get(config, "transaction_cost_abs", 0.0),
        reward_shaper=shaper, adaptation_rate=_cfg_get(rconf, "adaptation_rate", 0.001),
        cosine_temp=_cfg_get(rconf, "cosine_temp", 0.0),
        sortino_exp=_cfg_get(rconf, "sortino_exp", None),
        desired_portfolio=_cfg_get(rconf, "desired_portfolio", None) if shaper in (
            "cosine", "cosine_similarity", "cosine_port_shaper") else None,
        window=window, norm_type=norm_type, nstep_return=nstep, discount=discount,
        unit_size=unit, action_atoms=atoms, **kw)


def get_env_info(env: Env) -> dict:
    """get_env_info (madigan/environments/__init__.py:41-56)."""
    return {
        "timestamp": env.timestamp,
        "riskInfo": env.checkRisk(),
        "prices": np.array(env.currentPrices, copy=True),
        "equity": env.equity,
        "cash": env.cash,
        "pnl": env.pnl,
        "balance": env.portfolio.balance,
        "availableMargin": env.availableMargin,
        "usedMargin": env.usedMargin,
        "borrowedAssetValue": env.borrowedAssetValue,
        "borrowedMargin": env.borrowedMargin,
        "ledger": np.array(env.ledger, copy=True),
        "ledgerNormed": np.array(env.ledgerNormed, copy=True),
    }
