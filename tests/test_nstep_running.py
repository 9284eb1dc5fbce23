"""The running-sum n-step pop (MGN_NSTEP_POP_RUNNING, csrc/mgn_kernels.h
nrun_*), restated here in numpy (the kernel's algebra: the same sums, slides and re-sums), against
the reference's own pops: the golden vectors tests/golden/make_golden.py made
from madigan/utils/buffers/nstep_buffer.py (DSR :30-98, DDR :101-169, cosine
PPC :182-204; n = 5 and 20, done flushes, r = 0, A = B = 0, clip saturation)
and long random reward streams against the oracle's exact pop.  The bar is
north_star's 1e-6 relative on rewards.  The GPU kernel itself is checked
against the oracle in tests/test_gpu_nstep_running.py."""
import math
import os

import numpy as np
import pytest

from oracle import oracle as O

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.npz"))
EPS = float(np.finfo(np.float32).eps)  # nstep_buffer.py:20
RTOL, ATOL = 1e-6, 1e-10


class RunningPop:
    """One reward column's NStepBuffer with the kernel's running-sum pop:
    sums of g^k {1, r, r^2} split by r > 0, an entry enters at weight
    g^(len-1), a pop slides the rest by 1/g, the sums are formed afresh from
    the buffer every n pops (before the next append) and are zero once the
    buffer is flushed."""

    def __init__(self, shaper, n, gamma, eta, sexp=2.0):
        self.shaper, self.n, self.eta, self.sexp = shaper, n, eta, sexp
        self.disc = [math.pow(gamma, i) for i in range(n)]  # nstep_buffer.py:330
        self.disc2 = [math.pow(d, 1.0 / sexp) for d in self.disc]  # sortino_shaperB: (gamma^k)^(1/exp)
        self.rg = 1.0 / gamma
        self.rg2 = 1.0 / math.pow(gamma, 1.0 / sexp)
        self.buf = []
        self.s = np.zeros(6)  # p1 pr prr n1 nr nrr
        self.nsl = 0
        self.A = self.B = 0.0

    def _root(self, r):
        return (-r) ** (1.0 / self.sexp) if r < 0 else 0.0

    def _add(self, r, w, k=None):
        if self.shaper == "sortinoB":  # p1 = sum_{r>0} w r, n1 = sum_{r<0} w2 (-r)^(1/e), prr = #{r < -1}
            w2 = self.disc2[k]
            self.s[0] += w * r if r > 0 else 0.0
            self.s[3] += w2 * self._root(r) if r < 0 else 0.0
            self.s[2] += 1.0 if r < -1 else 0.0
            return
        c = 0 if r > 0 else 3
        self.s[c] += w
        self.s[c + 1] += w * r
        self.s[c + 2] += (w * r) * r

    def push(self, v):
        if self.nsl >= self.n:
            self.s[:] = 0
            for k, r in enumerate(self.buf):
                self._add(r, self.disc[k], k)
            self.nsl = 0
        self.buf.append(v)
        self._add(v, self.disc[len(self.buf) - 1], len(self.buf) - 1)

    def pop(self):
        p1, pr, prr, n1, nr, nrr = self.s
        A, B, L_ = self.A, self.B, len(self.buf)
        if self.shaper == "DSR":
            S1, Sr, Srr = p1 + n1, pr + nr, prr + nrr
            den = abs(B - A * A) ** 1.5 + EPS
            res = np.clip((B * (Sr - A * S1) - (A / 2) * (Srr - B * S1)) / den / L_, -1, 1)
        elif self.shaper == "sortinoB":
            if prr > 0:  # an entry below -1: the exact pop (the per-term clip may bind)
                acc = 0.0
                for k, r in enumerate(self.buf):
                    x = max(r * self.disc[k], -1.0)
                    acc += -((-x) ** (1.0 / self.sexp)) if x < 0 else x
                res = np.clip(acc, -1, 1)
            else:
                res = np.clip(p1 - n1, -1, 1)
        elif self.shaper == "DDR":
            up = (pr - (A / 2) * p1) / (math.sqrt(B) + EPS)
            dn = (B * (nr - (A / 2) * n1) - (A / 2) * nrr) / (B * math.sqrt(B) + EPS)
            res = np.clip((up + dn) / L_, -1, 1)
        else:
            res = pr + nr
        r0 = self.buf.pop(0)
        if self.shaper in ("DSR", "DDR"):  # update_parameters, exact
            self.A = A + self.eta * (r0 - A)
            m = min(r0, 0.0) if self.shaper == "DDR" else r0
            self.B = B + self.eta * (m * m - B)
        if not self.buf:
            self.s[:] = 0
            self.nsl = 0
        elif self.shaper == "sortinoB":
            self.s[0] = (self.s[0] - (r0 if r0 > 0 else 0.0)) * self.rg
            self.s[3] = (self.s[3] - self._root(r0)) * self.rg2
            self.s[2] -= 1.0 if r0 < -1 else 0.0
            self.nsl += 1
        else:
            self._add(r0, -1.0)
            self.s *= self.rg
            self.nsl += 1
        return float(res)


def drive(shaper, n, gamma, eta, values, dones, sexp=2.0):
    """ReplayBuffer.add's driving (replay_buffer.py:68-80): append, pop when
    full, flush on done."""
    rp = RunningPop(shaper, n, gamma, eta, sexp)
    outs = []
    for v, d in zip(values, dones):
        rp.push(float(v))
        if len(rp.buf) >= n:
            outs.append(rp.pop())
        if d:
            while rp.buf:
                outs.append(rp.pop())
    return np.array(outs)


def _cos(p, q):  # cosine_similarity (nstep_buffer.py:173-177) on one row
    return float((p * q).sum() / (np.sqrt((p ** 2).sum()) * np.sqrt((q ** 2).sum())))


CASES = [c for c in (str(x) for x in G["shaper_cases"])
         if c.split("_")[0] in ("DSR", "DDR", "cosine", "sortinoB", "sortinoB3") and not c.split("_")[1] == "n1"]


@pytest.mark.parametrize("case", CASES)
def test_running_pop_matches_reference_goldens(case):
    shaper = case.split("_")[0]
    sexp = float(G[case + "_exp"]) if case + "_exp" in G.files else 2.0
    if shaper == "sortinoB3":
        shaper = "sortinoB"
    rewards, ports, dones = G[case + "_rewards"], G[case + "_ports"], G[case + "_dones"]
    n, gamma, eta, temp = G[case + "_cfg"]
    n = int(n)
    desired = G[case + "_desired"]
    ref = G[case + "_out"]
    T, D = rewards.shape
    for d in range(D):  # the device's running pop is per scalar column
        if shaper == "cosine":  # the stored value r + temp * cos(port, target) (PPC)
            vals = [rewards[t, d] + temp * _cos(ports[t], desired) for t in range(T)]
            sh = "none"
        else:
            vals, sh = rewards[:, d], shaper
        got = drive(sh, n, gamma, eta, vals, dones, sexp)
        np.testing.assert_allclose(got, ref[:, d], rtol=RTOL, atol=ATOL, err_msg=f"{case} column {d}")


@pytest.mark.parametrize("shaper,n,gamma,sexp", [("DDR", 20, 0.99, 2.0), ("DSR", 20, 0.97, 2.0),
                                                 ("DDR", 5, 0.9, 2.0), ("DSR", 64, 0.9, 2.0),
                                                 ("none", 20, 0.99, 2.0), ("sortinoB", 20, 0.99, 1.1),
                                                 ("sortinoB", 20, 0.97, 2.0), ("sortinoB", 64, 0.95, 3.0)])
def test_running_pop_long_stream_vs_oracle(shaper, n, gamma, sexp):
    """20000 steps of rewards shaped like the env's (log returns, exact zeros,
    a few large moves that saturate the clip) with episode ends every ~300
    steps: every pop within 1e-6 of the oracle's exact pop, over hundreds of
    re-sums and flushes (the slides' drift stays bounded)."""
    rng = np.random.default_rng(7)
    T, eta = 20000, 0.01
    r = rng.normal(1e-4, 1e-2, T)
    r[rng.random(T) < 0.05] = 0.0
    r[rng.random(T) < 0.002] *= 30
    dones = rng.random(T) < 1 / 300
    if shaper == "sortinoB":
        r[rng.random(T) < 0.001] = -1.3  # entries below -1: the exact pops (the per-term clip)
    got = drive(shaper, n, gamma, eta, r, dones, sexp)
    disc = np.array([math.pow(gamma, i) for i in range(n)])
    A, B = np.zeros(1), np.zeros(1)
    buf, ref = [], []
    for t in range(T):
        buf.append(r[t])
        while len(buf) >= n or (dones[t] and buf):
            rr = np.array(buf)[:, None]
            if shaper == "none":
                ref.append(float((disc[:len(buf)] * rr[:, 0]).sum()))
            elif shaper == "sortinoB":
                ref.append(float(O.naive("sortino_shaperB", rr, disc[:len(buf)], sexp)[0]))
            else:
                ref.append(float(O.dsr(rr, disc[:len(buf)], eta, A, B, ddr=shaper == "DDR")[0]))
            buf.pop(0)
            if not dones[t]:
                break
    ref = np.array(ref)
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)
    if shaper != "none":
        assert (np.abs(ref) == 1.0).any(), "clip saturation exercised"
    assert not np.array_equal(got, ref), "the running pop is a different evaluation"
