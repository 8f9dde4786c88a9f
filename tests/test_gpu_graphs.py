"""GPU: evaluations replayed from HIP graphs (phy_set_graphs) give bit for
bit the direct launches' rows -- on the small host-buffer path (copies in
the graph), the device-buffer path with new contents in the same buffers,
every engine, and across changes that must rebuild the graphs (output
layout, engine, draw count)."""
import numpy as np
import pytest
import torch  # noqa: F401 -- torch's own HIP runtime must load before the engine's

from tests import cases

pytestmark = pytest.mark.gpu


def _pair(case, max_draws):
    from phylostan_amd.engine import TreeLikelihood
    a = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, max_draws=max_draws)
    b = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, max_draws=max_draws)
    a.set_graphs(True)
    b.set_graphs(False)
    return a, b


def _inputs(case, n, seed):
    rng = np.random.default_rng(seed)
    bl = case.blens[None, :] * rng.uniform(0.6, 1.4, (n, case.blens.size))
    mv = np.repeat(case.model_vec()[None], n, axis=0)
    return bl, mv


@pytest.mark.parametrize("engine", ["pattern", "class"])
def test_graph_replay_host_path(engine):
    case = cases.fluA_case()
    a, b = _pair(case, 8)
    for e in (a, b):
        e.set_engine(engine)
        e.set_output(compact=True)
    for k, n in enumerate([4, 4, 4, 4, 2, 2, 2, 4]):  # capture on the second call of a size, replay after
        bl, mv = _inputs(case, n, k)
        ra, rb = a.evaluate_rows(bl, mv), b.evaluate_rows(bl, mv)
        np.testing.assert_array_equal(ra, rb)
        if k == 5:  # a layout change rebuilds
            a.set_output(compact=False)
            b.set_output(compact=False)
    a.submit_rows(*_inputs(case, 4, 99))
    b.submit_rows(*_inputs(case, 4, 99))
    np.testing.assert_array_equal(a.wait_rows(), b.wait_rows())


@pytest.mark.parametrize("engine", ["pattern", "class"])
def test_graph_replay_device_path(engine):
    from phylostan_amd import synthetic
    pd, prm = synthetic.simulate(n_sites=20_000)
    case = cases.Case("syn20k", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"], prm["freqs"],
                      prm["rates"], prm["rs"], prm["ps"])
    a, b = _pair(case, 2)
    for e in (a, b):
        e.set_engine(engine)
    d_bl = torch.zeros((2, a.B), dtype=torch.float64, device="cuda:0")
    d_mv = torch.zeros((2, a.model_len), dtype=torch.float64, device="cuda:0")
    outs = [torch.zeros((2, e.outlen), dtype=torch.float64, device="cuda:0") for e in (a, b)]
    for k in range(5):
        bl, mv = _inputs(case, 2, 10 + k)
        d_bl.copy_(torch.from_numpy(bl))
        d_mv.copy_(torch.from_numpy(mv))
        for e, o in zip((a, b), outs):
            e.evaluate_device(d_bl.data_ptr(), d_mv.data_ptr(), o.data_ptr(), 0, n_draws=2)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]), k
        if k == 2:
            a.set_engine("pattern" if engine == "class" else "class")
            b.set_engine("pattern" if engine == "class" else "class")
