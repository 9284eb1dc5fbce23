"""CPU checks of the drop-in boundary: the C-ABI library loads and exports
every entry point include/madigan_amd.h declares, the ctypes mirrors match the
C struct layouts byte for byte, and the product fails loudly without a GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

from madigan_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "madigan_amd.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mgn_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = L.load()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} declared in madigan_amd.h but not exported"
        assert n in L.SYMBOLS, f"{n} has no ctypes prototype"
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (mgn_\w+)", out))
    assert set(names) == exported, f"undeclared exports: {exported - set(names)}"


def test_hdf_library_exports_every_declared_symbol():
    from madigan_amd import hdf as H
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "madigan_hdf.h")).read(),
                 flags=re.S)
    names = sorted(set(re.findall(r"\b(mgn_hdf_[a-z_0-9]+)\s*\(", txt)))
    assert len(names) >= 9
    lib = H.load_hdf()
    for n in names:
        assert hasattr(lib, n) and n in H.HDF_SYMBOLS, n
    out = subprocess.run(["nm", "-D", "--defined-only", H.HDF_LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert set(re.findall(r" T (mgn_\w+)", out)) == set(names)


def test_abi_version():
    assert L.load().mgn_abi_version() == L.ABI_VERSION


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "madigan_amd.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("mgn_config %zu\nmgn_traj %zu\nmgn_views %zu\nmgn_asset_source %zu\nmgn_ring %zu\n"
         "mgn_replay_tape %zu\nmgn_hist_view %zu\n",
         sizeof(mgn_config), sizeof(mgn_traj), sizeof(mgn_views), sizeof(mgn_asset_source),
         sizeof(mgn_ring), sizeof(mgn_replay_tape), sizeof(mgn_hist_view));
  F(mgn_config, seed) F(mgn_config, shaper) F(mgn_config, adaptation_rate)
  F(mgn_config, desired_portfolio) F(mgn_config, window) F(mgn_config, unit_size)
  F(mgn_views, out) F(mgn_views, n_envs) F(mgn_views, reward_dim) F(mgn_views, reset_mask)
  F(mgn_ring, ring) F(mgn_ring, len) F(mgn_asset_source, p) F(mgn_config, n_feats)
  F(mgn_traj, data_end) F(mgn_views, replay_cursor) F(mgn_views, n_feats)
  F(mgn_replay_tape, rows) F(mgn_replay_tape, stride)
  F(mgn_hist_view, hlen) F(mgn_hist_view, rows) F(mgn_hist_view, n_feats)
  return 0;
}
"""


def test_struct_layouts_match_ctypes(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.splitlines())
    py = {"mgn_config": L.Config, "mgn_traj": L.Traj, "mgn_views": L.Views,
          "mgn_asset_source": L.AssetSource, "mgn_ring": L.Ring, "mgn_replay_tape": L.ReplayTape,
          "mgn_hist_view": L.HistView}
    for k, v in got.items():
        if "." in k:
            t, f = k.split(".")
            assert getattr(py[t], f).offset == int(v), k
        else:
            assert C.sizeof(py[k]) == int(v), k


def test_arena_bytes_scales():
    from madigan_amd.config import build_config, trendou_spec
    p = [0.001, 100, 500, 0.001, 0.005, 5.0, 0.15, 0.04, 0.001, 0.99]
    c1, _ = build_config(trendou_spec(*[[v] * 8 for v in p]), n_envs=1024)
    c2, _ = build_config(trendou_spec(*[[v] * 8 for v in p]), n_envs=2048, window=64)
    lib = L.load()
    b1 = lib.mgn_arena_bytes(C.byref(c1))
    b2 = lib.mgn_arena_bytes(C.byref(c2))
    assert b1 > 1024 * 8 * 8 * 10 and b2 > 2 * b1
    bad = L.Config()
    bad.n_envs, bad.n_assets = 4, 65
    assert lib.mgn_arena_bytes(C.byref(bad)) == 0


def test_create_rejects_bad_config_with_reference_exceptions():
    from madigan_amd.config import build_config, ou_spec
    lib = L.load()
    c, srcs = build_config(ou_spec([10.] * 2, [.1] * 2, [.04] * 2), n_envs=4)
    c.n_envs = 0
    h = C.c_void_p()
    with pytest.raises(ValueError):
        L.check(lib.mgn_create(C.byref(c), srcs, None, None, 0, C.byref(h)))
    c.n_envs = 4
    srcs[1].kind = 42
    with pytest.raises(RuntimeError, match="unknown data source"):
        L.check(lib.mgn_create(C.byref(c), srcs, None, None, 0, C.byref(h)))


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("host has a GPU")
    from madigan_amd import BatchedEnv, Env
    from madigan_amd.config import ou_spec
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        BatchedEnv(ou_spec([10.], [.1], [.04]), 4)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        Env("OU", 1_000_000)


def test_pycall_binding_links_the_in_tree_library():
    """The CPython binding of mgn_rollout (csrc/mgn_pycall.c) is built next to
    libmadigan_hip.so, resolves it through $ORIGIN and rejects a null handle
    before any HIP call (no GPU needed)."""
    import os
    from madigan_amd import _lib as L
    pc = L.pycall()
    assert pc is not None, "_mgn_pycall is not built (python -m madigan_amd.build)"
    assert os.path.dirname(pc.__file__) == os.path.dirname(L.LIB_PATH)
    with pytest.raises(ValueError):
        pc.rollout(0, 0, 1, 0)
    with pytest.raises(TypeError):
        pc.rollout(0, 0)
