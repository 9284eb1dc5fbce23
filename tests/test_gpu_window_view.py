"""Zero-copy per-step windows (mgn_window_hist_view): every window of a
K-step launch read in place from the launch history equals the materialised
mgn_window_hist output bit for bit (StackerDiscrete.current_data after each
step, preprocessor.py:177-189), for the element-wise normalisers none and log,
across auto-resets; the other normalisers are refused."""
import pytest

from tests.configs import composite_sources, ou_sources, spec_from_sources

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,norm,N", [("C4", "log", 2048), ("C2", None, 1024)])
def test_view_equals_materialised(gpu, name, norm, N):
    import torch
    from madigan_amd import BatchedEnv
    src = composite_sources() if name == "C4" else ou_sources(4)
    kw = dict(required_margin=0.05, maintenance_margin=0.25, transaction_cost_rel=0.02, unit_size=0.5,
              auto_reset=True, init_cash=1e5, window=64, norm_type=norm, seed=11)
    if name == "C4":
        kw.update(reward_shaper="PPC", cosine_temp=0.01, desired_portfolio=[1.0] + [0.0] * 8)
    else:
        kw.update(reward_shaper="DSR")
    g = BatchedEnv(spec_from_sources(src), N, device=gpu, **kw)
    K = 64
    acts = g.generate_actions(2 * K, seed=9)
    ends = 0
    for launch in range(2):
        out, (wp, wo, wt) = g.rollout_window(acts[launch * K:(launch + 1) * K], per_step=True)
        ends += int(out["done"].sum().item())
        view = g.window_hist_view()
        assert view["hend"].shape == (K, N) and view["window"] == 64
        for k in range(K):
            vp, vo, vt = g.window_from_view(view, k)
            assert torch.equal(vp.view(torch.int64), wp[k].view(torch.int64)), f"{name} price {launch}/{k}"
            assert torch.equal(vo.view(torch.int64), wo[k].view(torch.int64)), f"{name} port {launch}/{k}"
            assert torch.equal(vt, wt[k].view(torch.int64)), f"{name} ts {launch}/{k}"
    assert ends > 0


def test_view_refuses_lookback(gpu):
    from madigan_amd import BatchedEnv
    g = BatchedEnv(spec_from_sources(ou_sources(2)), 64, device=gpu, window=8, norm_type="lookback",
                   required_margin=1.0, maintenance_margin=0.25, auto_reset=True)
    g.rollout_window(g.generate_actions(4, seed=1), per_step=True)
    with pytest.raises(RuntimeError):
        g.window_hist_view()
    h = BatchedEnv(spec_from_sources(ou_sources(2)), 64, device=gpu, window=8,
                   required_margin=1.0, maintenance_margin=0.25)
    with pytest.raises(RuntimeError):  # no launch history yet
        h.window_hist_view()
