"""GPU: the posterior, ADVI and NUTS driven by the HIP likelihood (C-ABI).

* the host posterior around ``TreeLikelihood`` equals the one around the
  CPU oracle (value rel 1e-10, gradient 1e-8 of its largest entry);
* ``phylostan run -a vb`` on fluA (HKY+W4, strict clock, constant
  coalescent, heterochronous -- the README.md:93-109 analysis) lands its
  posterior means inside the 95% credible intervals the reference prints
  there;
* a short multi-chain NUTS run on fluA is finite and moves uphill.
"""
import numpy as np
import pytest

from tests import cases, fixture_files
from tests.oracle_backend import OracleLikelihood

pytestmark = pytest.mark.gpu

README_CI = {  # README.md:104-108 (fluA meanfield ADVI)
    "wshape": (0.383, 0.616),
    "rate": (0.00432, 0.00577),
    "theta": (3.14, 5.05),
    "kappa": (4.37, 7.039),
    "root_height": (18.36, 19.74),
}


def _fluA_posterior(lik_cls, clock="strict", speciation=None, **kw):
    from phylostan_amd.posterior import ModelSpec, Posterior, TreeData
    d = cases.load_layout("fluA")
    S = d["tipbits"].shape[0]
    peel0 = d["peel"] - 1
    tree = TreeData(S, peel0, d["map"], d["lowers"], float(d["oldest"]))
    spec = ModelSpec(model="HKY", categories=4, clock=clock, estimate_rate=True, coalescent="constant",
                     heterochronous=True, speciation=speciation)
    return Posterior(spec, tree, lik_cls(d["tipbits"], d["weights"], peel0, True, "HKY", 4, **kw),
                     compact_rows=True), d


def test_posterior_gpu_equals_oracle():
    from phylostan_amd.engine import TreeLikelihood
    pg, d = _fluA_posterior(TreeLikelihood, max_draws=8)
    po, _ = _fluA_posterior(OracleLikelihood)
    case = cases.fluA_case()
    u0 = pg.unconstrain(dict(wshape=0.488, rate=0.00499, height=d["heights"][-1], theta=4.03, kappa=5.58,
                             freqs=case.freqs, props=pg.props_from_heights(d["heights"])))
    rng = np.random.default_rng(0)
    U = np.stack([u0] + [u0 + 0.05 * rng.standard_normal(pg.dim) for _ in range(3)])
    lg, Gg = pg.log_prob_grad(U)
    lo, Go = po.log_prob_grad(U)
    np.testing.assert_allclose(lg, lo, rtol=1e-10)
    for k in range(len(U)):
        assert np.max(np.abs(Gg[k] - Go[k])) <= 1e-8 * np.max(np.abs(Go[k]))


@pytest.mark.parametrize("clock,speciation", [("ucln", None), ("acln", None), ("hsmrf", "bd")])
def test_relaxed_clock_posterior_gpu_equals_oracle(clock, speciation):
    """Relaxed clocks (per-branch substrates in the blens) and the
    birth-death prior around the GPU likelihood: value and gradient equal
    the oracle-backed posterior's."""
    from phylostan_amd.engine import TreeLikelihood
    pg, d = _fluA_posterior(TreeLikelihood, clock=clock, speciation=speciation, max_draws=4)
    po, _ = _fluA_posterior(OracleLikelihood, clock=clock, speciation=speciation)
    rng = np.random.default_rng(1)
    case = cases.fluA_case()
    vals = dict(wshape=0.488, height=d["heights"][-1], theta=4.03, kappa=5.58, freqs=case.freqs,
                props=pg.props_from_heights(d["heights"]), substrates=rng.uniform(0.004, 0.006, pg.B),
                ucln_mean=0.005, ucln_stdev=0.3, nu=0.01, deltas=rng.normal(0, 0.001, 2 * pg.S - 3),
                rate=0.005, zeta=1.0, gammas=np.ones(pg.B - 1), netDiversificationRate=0.1,
                relativeExtinctionRate=0.5)
    u0 = pg.unconstrain({p.name: vals[p.name] for p in pg.params})
    U = np.stack([u0] + [u0 + 0.02 * rng.standard_normal(pg.dim) for _ in range(3)])
    lg, Gg = pg.log_prob_grad(U)
    lo, Go = po.log_prob_grad(U)
    assert np.all(np.isfinite(lg))
    np.testing.assert_allclose(lg, lo, rtol=1e-10)
    for k in range(len(U)):
        assert np.max(np.abs(Gg[k] - Go[k])) <= 1e-8 * np.max(np.abs(Go[k]))


def test_fluA_advi_within_readme_intervals(tmp_path):
    from phylostan_amd import cli, stan_io
    t, a = fixture_files.write_dataset("fluA", str(tmp_path))
    out = str(tmp_path / "fluA")
    cli.main(["run", "-s", str(tmp_path / "fluA.json"), "-m", "HKY", "-C", "4", "--heterochronous",
              "--estimate_rate", "--clock", "strict", "--coalescent", "constant", "-i", a, "-t", t, "-o", out,
              "-q", "meanfield", "-S", "1", "--iter", "30000"])
    res = stan_io.parse_log(out, 0.05)
    for key, (lo, hi) in README_CI.items():
        m = res[key][0]
        assert lo <= m <= hi, "%s mean %g outside the reference's 95%% CI (%g, %g)" % (key, m, lo, hi)


def test_fluA_nuts_short_multichain():
    from phylostan_amd.engine import TreeLikelihood
    from phylostan_amd.nuts import run_chains
    post, d = _fluA_posterior(TreeLikelihood, max_draws=4)
    rng = np.random.default_rng(5)
    q0s = [post.initial_point(rng) for _ in range(4)]
    lp0 = post.log_prob(np.stack(q0s))
    chains = run_chains(post, q0s, [11, 12, 13, 14], num_warmup=40, num_samples=10, max_depth=6)
    for c, ch in enumerate(chains):
        lps = np.array([dr[1] for dr in ch.draws])
        assert np.all(np.isfinite(lps)) and lps[-1] > lp0[c]


def test_fluA_native_nuts_loop_equals_python_rounds(monkeypatch):
    """The whole NUTS loop in C++ (phn_run: the posterior's native phases
    and phy_eval_submit / phy_eval_wait called from the sampler) gives the
    draws of the same native chains driven round by round from Python
    through Posterior.log_prob_grad -- bit for bit, on the GPU."""
    from phylostan_amd import nuts
    from phylostan_amd.engine import TreeLikelihood
    runs = []
    for mode in ("python", None):
        if mode:
            monkeypatch.setenv("PHYLO_NUTS_LOOP", mode)
        else:
            monkeypatch.delenv("PHYLO_NUTS_LOOP", raising=False)
        post, d = _fluA_posterior(TreeLikelihood, max_draws=4)
        if mode is None:
            assert nuts._native_loop_args(post, 4) is not None
        q0s = [post.initial_point(np.random.default_rng((3, c))) for c in range(4)]
        runs.append(nuts.run_chains(post, q0s, [(3, c) for c in range(4)], num_warmup=30, num_samples=10,
                                    max_depth=6))
    for ca, cb in zip(*runs):
        assert ca.n_grad == cb.n_grad and ca.eps == cb.eps
        for da, db in zip(ca.draws, cb.draws):
            np.testing.assert_array_equal(da[0], db[0])
            assert da[1:] == db[1:]


def test_fluA_fullrank_advi_runs_to_convergence(tmp_path):
    """-q fullrank (phylostan.py:311-313 algorithm='fullrank') on fluA with
    eta fixed at 0.1 (phylostan run --eta 0.1: no adaptation; the value the
    adaptation picks here): Stan's normal_fullrank SGA on GPU gradients runs
    until its relative-ELBO test stops it, writes the mean row plus 1000
    draws, and its posterior means land inside the 95% intervals the
    reference prints for meanfield (README.md:104-108).

    Why eta is fixed (tests/test_fullrank_fate.py, CPU): with adaptation the
    generator state SGA starts from depends on which of the adaptation's
    eta = 100 / 10 draws overflowed, which last-bit differences decide, and
    from some states SGA stops early in a poor state (ELBO -4,790 .. -4,890,
    clock rate 0.08 .. 0.15) -- the round-2 "stall".  With eta fixed the run
    is a function of the seed alone (ulp-perturbed gradients give the same
    ELBO trace) and seeds 1..12 all converge to ELBO -4,430 on the C port."""
    from phylostan_amd import cli, stan_io
    t, a = fixture_files.write_dataset("fluA", str(tmp_path))
    out = str(tmp_path / "fluA_fr")
    cli.main(["run", "-s", str(tmp_path / "fluA.json"), "-m", "HKY", "-C", "4", "--heterochronous",
              "--estimate_rate", "--clock", "strict", "--coalescent", "constant", "-i", a, "-t", t, "-o", out,
              "-q", "fullrank", "-S", "1", "--eta", "0.1"])
    header, data = stan_io.read_samples(out)
    assert data.shape[0] == 1001 and np.isfinite(data).all()
    with open(out + ".diag") as fp:
        rows = [ln.strip().split(",") for ln in fp if ln.strip() and not ln.startswith(("#", "iter"))]
    elbo = np.array([float(r[2]) for r in rows])
    assert np.isfinite(elbo).all() and elbo[-1] > elbo[0] + 5000.0
    assert len(elbo) < 1000  # stopped by tol_rel_obj, not by the iteration cap
    assert elbo[-1] > -4500.0  # the converged state, not the early stop (-4,790 .. -4,890)
    res = stan_io.parse_log(out, 0.05)
    for key, (lo, hi) in README_CI.items():
        m = res[key][0]
        assert lo <= m <= hi, "%s mean %g outside the reference's 95%% CI (%g, %g)" % (key, m, lo, hi)


def test_config1_ds1_jc69_unrooted_meanfield(tmp_path, capsys):
    """BASELINE config 1 as the reference runs it (examples/SConstruct:170-188,
    run_stan :71-88): `phylostan build -m JC69`, then `phylostan run -i DS1 -t
    tree0 -s jc69.stan -o tree0 -m JC69 --eta 0.1` -- no clock, so the
    unrooted model with the root branch merged (generate_script.py:1013-1023)
    and blens ~ exponential(10) (:1404) -- on DS1 and its first tree in the
    reference's form (trifurcating root, no branch lengths), every gradient
    from the GPU engine.  The posterior is parity-unpinned (the reference
    publishes no DS1 numbers); this checks the run's contract: Stan's progress
    lines (the regex SConstruct:128 parses), an ELBO that rises and stops by
    tol_rel_obj, `blens.k` columns, and `parse` giving the .trees file `run`
    wrote (same node numbering for the trifurcating root)."""
    import re
    from phylostan_amd import cli, stan_io
    t, a = fixture_files.write_dataset("DS1", str(tmp_path), reference_form=True)
    script = str(tmp_path / "jc69.stan")
    assert cli.main(["build", "-m", "JC69", "-s", script]) == 0
    out = str(tmp_path / "tree0")
    capsys.readouterr()
    cli.main(["run", "-i", a, "-t", t, "-s", script, "-o", out, "-m", "JC69", "--eta", "0.1", "--seed", "1"])
    printed = capsys.readouterr().out
    prog = [(int(m.group(1)), float(m.group(2))) for m in re.finditer(r"\s+(\d+)\s+(-\d+\.\d+)", printed)]
    assert len(prog) >= 5, printed[:2000]
    elbo = np.array([e for _, e in prog])
    assert np.isfinite(elbo).all() and elbo[-1] > elbo[0] + 1000.0
    assert "ELBO CONVERGED" in printed and prog[-1][0] < 100000
    header, data = stan_io.read_samples(out)
    B = 2 * 27 - 3
    assert header[:B + 1] == ["lp__"] + ["blens.%d" % k for k in range(1, B + 1)]
    assert data.shape == (1001, len(header)) and np.isfinite(data).all() and np.all(data[:, 1:B + 1] > 0)
    cli.main(["parse", "--samples", out, "-t", t, "-o", str(tmp_path / "parsed.trees")])
    ran = open(out + ".trees").read()
    parsed = open(str(tmp_path / "parsed.trees")).read()
    assert ran.count("tree ") == 1001 and ran == parsed


def test_config3_hcv_gtr_skyride_as_the_reference_runs_it(tmp_path, capsys):
    """BASELINE config 3 as the reference runs it (examples/SConstruct:215-218):
    `phylostan build -m GTR -C 4 --clock strict --coalescent skyride`, then
    `phylostan run -m GTR -C 4 --clock strict --rate 7.9e-4 --coalescent
    skyride` on HCV (contemporaneous tips, the clock rate fixed), every
    gradient from the GPU engine, meanfield ADVI at eta 0.1 (no adaptation:
    the run is a function of the seed).  The posterior is parity-unpinned (the
    reference publishes no HCV numbers); this checks the run's contract:
    Stan's progress lines, an ELBO that rises and stops by tol_rel_obj, the
    skyride's `thetas.k` / `tau` columns beside `heights.k`, `rates.k`,
    `freqs.k`, and `parse` giving the .trees file `run` wrote."""
    import argparse
    import re
    import sys
    import time
    from phylostan_amd import cli, stan_io
    t, a = fixture_files.write_dataset("HCV", str(tmp_path))
    script = str(tmp_path / "hcv.stan")
    assert cli.main(["build", "-m", "GTR", "-C", "4", "--clock", "strict", "--coalescent", "skyride",
                     "-s", script]) == 0
    out = str(tmp_path / "hcv")
    parser = argparse.ArgumentParser()
    sub = parser.add_subparsers()
    cli.create_run_parser(sub).set_defaults(func=cli.run)
    arg = parser.parse_args(["run", "-i", a, "-t", t, "-s", script, "-o", out, "-m", "GTR", "-C", "4", "--clock",
                             "strict", "--rate", "7.9e-4", "--coalescent", "skyride", "--eta", "0.1", "--seed", "1"])
    lines = []
    t0 = time.time()

    def log(msg):  # the run's printed lines, echoed past pytest's capture (a long run shows progress)
        lines.append(msg)
        with capsys.disabled():
            sys.stdout.write("[config3 %.1fs] %s\n" % (time.time() - t0, msg))
            sys.stdout.flush()
    cli.run(arg, log=log)
    printed = "\n".join(lines)
    prog = [(int(m.group(1)), float(m.group(2))) for m in re.finditer(r"\s+(\d+)\s+(-\d+\.\d+)", printed)]
    assert len(prog) >= 5, printed[:2000]
    elbo = np.array([e for _, e in prog])
    assert np.isfinite(elbo).all() and elbo[-1] > elbo[0]
    assert "ELBO CONVERGED" in printed and prog[-1][0] < 100000
    header, data = stan_io.read_samples(out)
    S = 63
    for k in (1, S - 1):
        assert "thetas.%d" % k in header
    assert "thetas.%d" % S not in header and "tau" in header
    assert "heights.%d" % (S - 1) in header and "rates.6" in header and "freqs.4" in header
    assert "rate" not in header  # --rate fixes the clock rate: no rate parameter
    assert data.shape == (1001, len(header)) and np.isfinite(data).all()
    tau = data[:, header.index("tau")]
    assert np.all(tau > 0)
    # parse with the run's fixed rate (phylostan.py parse --rate): the same .trees run wrote
    cli.main(["parse", "--samples", out, "-t", t, "--rate", "7.9e-4", "-o", str(tmp_path / "parsed.trees")])
    ran = open(out + ".trees").read()
    parsed = open(str(tmp_path / "parsed.trees")).read()
    assert ran.count("tree ") == 1001
    assert ran == parsed, "parse's .trees differ from run's"  # (no diff of two multi-MB strings in the report)
