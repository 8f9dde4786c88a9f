"""``python -m phylostan_amd build|run|parse``: flags, output files and their
formats (phylostan/phylostan.py:15-335, utils.py:193-409), on the CPU with the
oracle stand-in as the likelihood (the GPU run of the same CLI is in
tests/test_gpu_inference.py)."""
import json
import os

import numpy as np
import pytest

from phylostan_amd import cli, stan_io
from tests import fixture_files
from tests.oracle_backend import OracleLikelihood


def _run(argv, **kw):
    import argparse
    parser = argparse.ArgumentParser()
    sub = parser.add_subparsers()
    cli.create_run_parser(sub).set_defaults(func=cli.run)
    arg = parser.parse_args(["run"] + argv)
    lines = []
    post = cli.run(arg, likelihood_factory=OracleLikelihood, log=lines.append, **kw)
    return post, lines


def test_build_writes_model_description(tmp_path):
    script = str(tmp_path / "m.json")
    assert cli.main(["build", "-s", script, "-m", "HKY", "-C", "4", "--clock", "strict", "--estimate_rate",
                     "--coalescent", "constant", "--heterochronous"]) == 0
    doc = json.load(open(script))
    assert doc["options"]["model"] == "HKY" and doc["options"]["categories"] == 4


def test_run_vb_outputs(tmp_path, capsys):
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=1, S=6, sites=50)
    out = str(tmp_path / "rand")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "HKY", "-C", "2", "--clock", "strict",
                        "--estimate_rate", "--coalescent", "constant", "--heterochronous", "-t", t, "-i", a,
                        "-o", out, "-S", "7", "--iter", "300", "--elbo_samples", "20", "--samples", "50",
                        "--tol_rel_obj", "0.01"])
    assert any("Begin stochastic gradient ascent." in s for s in lines)
    assert any(s.startswith("   100") or s.startswith("  100") for s in lines)
    header, data = stan_io.read_samples(out)
    assert header[0] == "lp__" and header[1:4] == ["wshape", "props.1", "props.2"]
    assert "heights.5" in header and "rs.2" in header and "freqs.4" in header
    assert data.shape == (51, len(header)) and np.all(data[:, 0] == 0)
    diag = open(out + ".diag").read().splitlines()
    rows = [r for r in diag if not r.startswith("#")]
    assert rows[0] == "iter,time_in_seconds,ELBO" and rows[1].startswith("100,")
    trees = open(out + ".trees").read()
    assert trees.startswith("#NEXUS\nBegin trees;\nTranslate\n1 t") and trees.count("tree ") == 51
    assert "[&height=" in trees and ",rate=" in trees and trees.endswith("END;")
    printed = capsys.readouterr().out
    assert "Strict clock (rate) mean:" in printed and "Root height mean:" in printed


def test_run_nuts_two_chains_and_parse(tmp_path, capsys):
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=2, S=5, sites=40, hetero=False)
    out = str(tmp_path / "nuts")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "JC69", "-t", t, "-i", a, "-o", out, "-a", "nuts",
                        "--chains", "2", "--iter", "40", "-S", "3"])
    for c in range(2):
        path = out + "_%d.csv" % c
        header, data = stan_io.read_samples(path)
        assert header[:7] == ["lp__"] + stan_io.NUTS_COLUMNS
        assert header[7] == "blens.1" and data.shape[0] == 20
        txt = open(path).read()
        assert "# Adaptation terminated" in txt and "# Diagonal elements of inverse mass matrix:" in txt
        assert os.path.exists(out + "_%d.trees" % c)
    capsys.readouterr()
    cli.main(["parse", "--samples", out + "_0.csv", "-t", t, "-o", str(tmp_path / "p.trees")])
    printed = capsys.readouterr().out
    assert "Tree length mean:" in printed
    assert open(str(tmp_path / "p.trees")).read().count("tree ") == 20


def test_run_relaxed_clock_vb(tmp_path, capsys):
    """--clock ucln --estimate_rate: substrates in the sample CSV, per-branch
    rates in the trees file (utils.py:229-245)."""
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=3, S=6, sites=50)
    out = str(tmp_path / "ucln")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "JC69", "--clock", "ucln", "--estimate_rate",
                        "--coalescent", "constant", "--heterochronous", "-t", t, "-i", a,
                        "-o", out, "-S", "5", "--iter", "200", "--elbo_samples", "10", "--samples", "20",
                        "--tol_rel_obj", "0.01"])
    header, data = stan_io.read_samples(out)
    assert "substrates.10" in header and "ucln_stdev" in header
    assert data.shape == (21, len(header))
    trees = open(out + ".trees").read()
    assert trees.count("tree ") == 21 and ",rate=" in trees
    capsys.readouterr()


def test_unsupported_options_fail_loudly(tmp_path):
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=1, S=5, sites=20)
    with pytest.raises((SystemExit, ValueError)):
        _run(["-s", "x", "-t", t, "-i", a, "-o", str(tmp_path / "o"), "--clock", "acln"])  # needs --estimate_rate
    with pytest.raises(SystemExit):
        _run(["-s", "x", "-t", t, "-i", a, "-o", str(tmp_path / "o"), "--geo"])
    with pytest.raises(SystemExit):  # not one of the reference's algorithms
        _run(["-s", "x", "-t", t, "-i", a, "-o", str(tmp_path / "o"), "-a", "rwm"])


def test_parse_log_relaxed_clock_rate_summaries(tmp_path):
    """utils.py:354-380: with a tree and substrates, parse_log also prints the
    mean rate (sum rate*time / sum time per draw) and the variance of the
    branch rates -- accumulated over all draws so far, as the reference's
    never-reset list does.  Values checked against a hand computation."""
    import io
    from phylostan_amd import data as dataio
    from phylostan_amd import treeio
    tree = treeio.parse_newick("((A:1,B:1):1,C:2);")
    dataio.setup_indexes(tree)
    dataio.setup_dates(tree, None, False)
    # node ids: A=1 B=2 C=3 cherry=4 root=5; heights.1 = node 4, heights.2 = node 5
    rows = [[0.0, 1.0, 2.5, 0.1, 0.2, 0.3, 0.4],
            [0.0, 0.5, 3.0, 0.5, 0.1, 0.2, 0.6]]
    path = str(tmp_path / "relaxed.csv")
    with open(path, "w") as fp:
        fp.write("lp__,heights.1,heights.2,substrates.1,substrates.2,substrates.3,substrates.4\n")
        for r in rows:
            fp.write(",".join(str(x) for x in r) + "\n")
    buf = io.StringIO()
    res = stan_io.parse_log(path, 0.05, tree, out=buf)
    means, allr, variances = [], [], []
    for _, h4, h5, r1, r2, r3, r4 in rows:
        t = {1: h4, 2: h4, 3: h5, 4: h5 - h4}  # branch times: A, B under node 4; C, node 4 under root
        r = {1: r1, 2: r2, 3: r3, 4: r4}
        means.append(sum(r[b] * t[b] for b in t) / sum(t.values()))
        allr += [r[b] for b in (1, 2, 4, 3)]
        variances.append(np.var(allr))
    assert res["mean_rate"][0] == pytest.approx(np.mean(means), rel=1e-12)
    assert res["variance_rate"][0] == pytest.approx(np.mean(variances), rel=1e-12)
    text = buf.getvalue()
    assert "Mean rate mean:" in text and "Variance rate mean:" in text


def test_run_fullrank_vb(tmp_path, capsys):
    """-q fullrank (phylostan.py:311-313 algorithm=arg.variational): Stan's
    normal_fullrank family runs and writes the same files."""
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=4, S=5, sites=40)
    out = str(tmp_path / "fr")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "JC69", "--clock", "strict", "--estimate_rate",
                        "--coalescent", "constant", "--heterochronous", "-t", t, "-i", a, "-o", out, "-S", "3",
                        "--iter", "300", "--elbo_samples", "20", "--samples", "30", "--tol_rel_obj", "0.01",
                        "-q", "fullrank"])
    header, data = stan_io.read_samples(out)
    assert data.shape == (31, len(header))
    assert "# algorithm = fullrank" in open(out).read()
    assert any("Begin stochastic gradient ascent." in s for s in lines)
    capsys.readouterr()


def test_fullrank_family_gradient_matches_finite_differences():
    """normal_fullrank: the reparameterisation gradient of the ELBO (mean of
    g eta^T, lower triangle, + 1/L_dd) equals finite differences of the
    Monte-Carlo ELBO with the same eta on a Gaussian log density."""
    from phylostan_amd.advi import FullRank
    rng = np.random.default_rng(0)
    d = 3
    A = rng.standard_normal((d, d))
    Prec = A @ A.T + d * np.eye(d)
    logp = lambda Z: -0.5 * np.einsum("ni,ij,nj->n", Z, Prec, Z)
    q = FullRank(rng.standard_normal(d), np.tril(rng.standard_normal((d, d))) + 2 * np.eye(d))
    eta = rng.standard_normal((50, d))
    G = -(q.transform(eta) @ Prec)
    mu_g, L_g = q.grad(G, eta)

    def elbo(mu, L):
        qq = FullRank(mu, L)
        return logp(qq.transform(eta)).mean() + qq.entropy()
    h = 1e-6
    for i in range(d):
        e = np.zeros(d); e[i] = h
        fd = (elbo(q.mu + e, q.L) - elbo(q.mu - e, q.L)) / (2 * h)
        assert abs(fd - mu_g[i]) < 1e-5 * max(1, abs(fd))
        for j in range(i + 1):
            E = np.zeros((d, d)); E[i, j] = h
            fd = (elbo(q.mu, q.L + E) - elbo(q.mu, q.L - E)) / (2 * h)
            assert abs(fd - L_g[i, j]) < 1e-5 * max(1, abs(fd))
    assert np.all(np.triu(L_g, 1) == 0)


def test_run_static_hmc(tmp_path, capsys):
    """-a hmc (phylostan.py:319-321 algorithm=arg.algorithm.upper()): static
    HMC with Stan's HMC sampler columns."""
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=5, S=5, sites=40, hetero=False)
    out = str(tmp_path / "hmc.csv")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "JC69", "-t", t, "-i", a, "-o", out, "-a", "hmc",
                        "--iter", "60", "-S", "3"])
    header, data = stan_io.read_samples(out)
    assert header[:5] == ["lp__"] + stan_io.HMC_COLUMNS
    assert data.shape[0] == 30 and np.all(np.isfinite(data[:, 0]))
    assert np.all((data[:, 1] >= 0) & (data[:, 1] <= 1))
    assert np.allclose(data[:, 3], 2 * np.pi, rtol=1e-5)
    assert os.path.exists(str(tmp_path / "hmc.trees"))
    capsys.readouterr()


def test_dates_without_heterochronous_is_homochronous(tmp_path, capsys):
    """--dates alone (no --heterochronous): the model is homochronous, as in
    the reference where only --heterochronous adds lowers / lower_root to the
    data dict (phylostan.py:259-263)."""
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=6, S=5, sites=40, hetero=False)
    dates = str(tmp_path / "dates.csv")
    from phylostan_amd import treeio
    names = [tx.label for tx in treeio.read_tree(t).taxon_namespace]
    with open(dates, "w") as fp:
        fp.write("name,date\n" + "".join("%s,%g\n" % (n, 2000 + 3 * k) for k, n in enumerate(names)))
    out = str(tmp_path / "d")
    post, _ = _run(["-s", str(tmp_path / "x.stan"), "-m", "JC69", "--clock", "strict", "--estimate_rate",
                    "--coalescent", "constant", "-t", t, "-i", a, "-o", out, "--dates", dates, "-S", "2",
                    "--iter", "200", "--elbo_samples", "10", "--samples", "10", "--tol_rel_obj", "0.05"])
    assert post.tree.lowers is None
    rng = np.random.default_rng(0)
    lp = post.log_prob(np.stack([post.initial_point(rng) for _ in range(8)]))
    assert np.all(np.isfinite(lp))
    capsys.readouterr()


def test_compiled_model_artifact(tmp_path):
    """build --compile writes the compiled-model artifact under the
    reference's name (phylostan.py:154-161); run loads it and refuses flags
    describing another model (:292-300)."""
    script = str(tmp_path / "m.stan")
    assert cli.main(["build", "-s", script, "-m", "HKY", "-C", "4", "--clock", "strict", "--estimate_rate",
                     "--coalescent", "constant", "--heterochronous", "--compile"]) == 0
    assert cli.artifact_path(script) == str(tmp_path / "m.pkl")
    assert cli.artifact_path(str(tmp_path / "m.json")) == str(tmp_path / "m.json.pkl")
    doc = cli.load_artifact(script)
    assert doc["options"]["model"] == "HKY" and doc["options"]["categories"] == 4
    json.loads(open(str(tmp_path / "m.pkl")).read())  # JSON, never a pickle
    # a real pystan pickle (binary) at that path is refused cleanly, never unpickled
    with open(str(tmp_path / "p.pkl"), "wb") as fp:
        fp.write(b"\x80\x04\x95\x10\x00\x00\x00\x00\x00\x00\x00\xff\xfe")
    with pytest.raises(SystemExit):
        cli.load_artifact(str(tmp_path / "p.stan"))


def test_parse_reroots_a_multifurcating_root_like_the_reference():
    """phylostan.py:140-141: parse reroots a root with > 2 children at its
    first child's edge (DendroPy reroot_at_edge: new root (head, old root),
    the old root keeping its other children in order).  For a trifurcating
    root that is the shape -- and the node numbering -- run's
    resolve_polytomies gives (phylostan.py:175), so the sample columns of an
    unrooted run map to the same nodes."""
    from phylostan_amd import data as dataio
    from phylostan_amd import treeio

    def numbering(tree):
        dataio.setup_indexes(tree)
        return [(n.index, sorted(c.index for c in n.child_node_iter())) for n in tree.postorder_node_iter()
                if not n.is_leaf()]

    text = "((a:1,b:1):1,(c:1,d:1):1,e:2);"
    t1 = treeio.parse_newick(text)
    t1.resolve_polytomies()
    t2 = treeio.parse_newick(text)
    assert len(t2.seed_node.child_nodes()) == 3
    t2.reroot_at_edge(t2.seed_node.child_nodes()[0].edge)
    assert len(t2.seed_node.child_nodes()) == 2
    assert numbering(t1) == numbering(t2)
    # a four-way root keeps a trifurcation under the new root, as the reference does
    t3 = treeio.parse_newick("(a:1,b:1,c:1,d:1);")
    t3.reroot_at_edge(t3.seed_node.child_nodes()[0].edge)
    kids = t3.seed_node.child_nodes()
    assert kids[0].taxon.label == "a" and [c.taxon.label for c in kids[1].child_nodes()] == ["b", "c", "d"]


def test_ds1_reference_form_tree_round_trips(tmp_path):
    """The DS1 fixture written as the reference ships its trees (trifurcating
    root, no branch lengths: examples/DS1/DS1.trees) loads back, through the
    CLI's unrooted path (no --clock), to the fixture's peel and map -- the
    layout tests/test_data_prep.py pins to phylostan/utils.py."""
    from phylostan_amd import data as dataio
    from tests import cases
    t, a = fixture_files.write_dataset("DS1", str(tmp_path), reference_form=True)
    text = open(t).read()
    assert ":" not in text and text.count(",") == 26
    d = dataio.load(t, a, rooted=False, heterochronous=False)
    lay = cases.load_layout("DS1")
    np.testing.assert_array_equal(d.peel0, lay["peel"] - 1)
    np.testing.assert_array_equal(d.tipcodes, lay["tipbits"])
    np.testing.assert_array_equal(d.weights, lay["weights"])


def test_config3_hcv_skyride_columns_cpu(tmp_path):
    """Config 3's run shape (SConstruct:215-218: GTR+W4, strict clock at a
    fixed --rate, skyride) on the CPU stand-in, 150 iterations: the skyride's
    thetas.k (S-1 of them) and tau columns are written (the GPU test runs it
    to convergence)."""
    t, a = fixture_files.write_dataset("HCV", str(tmp_path))
    out = str(tmp_path / "hcv")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "GTR", "-C", "4", "--clock", "strict",
                        "--rate", "7.9e-4", "--coalescent", "skyride", "-t", t, "-i", a, "-o", out, "-S", "3",
                        "--iter", "150", "--elbo_samples", "10", "--samples", "20", "--eta", "0.1"])
    header, data = stan_io.read_samples(out)
    assert "thetas.62" in header and "thetas.63" not in header and "tau" in header
    assert "rate" not in header and "heights.62" in header and "rates.6" in header
    assert data.shape == (21, len(header)) and np.isfinite(data).all()
