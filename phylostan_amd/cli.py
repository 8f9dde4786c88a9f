"""``phylostan`` command line with the Stan runtime removed.

Same sub-commands, flags and output files as ``phylostan/phylostan.py``
(``build`` ``:149-161``, ``run`` ``:164-335``, ``parse`` ``:130-146``), driven
by the GPU likelihood engine instead of pystan:

* ``build -s SCRIPT ...`` writes SCRIPT as a JSON model description (the
  options that shape the model and the Stan parameter names it implies) in
  place of the emitted Stan program.  ``--compile`` "compiles" it: the HIP
  engine is loaded and the compiled-model artifact is written under the
  reference's name, SCRIPT with ``.stan`` replaced by ``.pkl`` (or SCRIPT +
  ``.pkl``; phylostan.py:154-161).  The artifact is JSON, never a pickle:
  the model options, the engine library and its kernel-source hash.
* ``run`` follows phylostan.py:292-300: if the artifact is missing or
  ``--compile`` is given it is (re)built, otherwise the existing one is
  loaded and its model is used -- a run whose flags describe a different
  model than the artifact is refused (the reference would hand Stan a data
  dict that does not fit the compiled model).
* ``run -s SCRIPT -t TREE -i ALN -o OUT ...`` reads and indexes the data
  exactly as the reference (``phylostan_amd.data.load``), builds the host
  posterior around ``TreeLikelihood`` and runs ``-a vb`` (ADVI,
  (``-q meanfield``, the default, or ``-q fullrank``), ``-a nuts`` or
  ``-a hmc`` (static HMC); it writes OUT (Stan-format sample CSV; ``OUT_{chain}.csv``
  for several chains, as pystan), ``OUT.diag`` (vb), ``OUT.trees`` and prints
  the ``parse_log`` summary.
* ``parse --samples CSV -t TREE -o OUT.trees`` post-processes a sample file.

Run as ``python -m phylostan_amd <command> ...``.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

from . import data as dataio
from . import stan_io
from .posterior import ModelSpec, Posterior, TreeData


def create_parse_parser(sub):
    p = sub.add_parser("parse", help="parse Stan log files")
    p.add_argument("--samples", required=True, help="Path to sample file from Stan")
    p.add_argument("-t", "--tree", required=True, help="Tree file")
    p.add_argument("-o", "--output", required=True, help="Nexus output file")
    p.add_argument("--alpha", type=float, default=0.05,
                   help="Controls level for 100*(1-alpha)%% Bayesian credible intervals")
    p.add_argument("--rate", type=float, help="Value of fixed rate")
    p.add_argument("--dates", help="Comma-separated (csv) file containing sequence dates with header 'name,date'")
    p.add_argument("--heterochronous", action="store_true",
                   help="Heterochronous data. Expect a date in the leaf names or a csv file containing dates")
    return p


def create_build_parser(sub, prog, help):
    p = sub.add_parser(prog, help=help)
    p.add_argument("-s", "--script", required=True, help="Model script file")
    p.add_argument("-m", "--model", choices=["JC69", "HKY", "GTR"], default="GTR",
                   help="Substitution model [default: %(default)s]")
    p.add_argument("-I", "--invariant", action="store_true", help="Include a proportion of invariant sites")
    p.add_argument("-C", "--categories", metavar="C", type=int, default=1, help="Number of categories")
    p.add_argument("--heterogeneity", choices=["weibull", "discrete"], default="weibull",
                   help="Weibull or discrete distribution to model rate heterogeneity across sites")
    p.add_argument("--heterochronous", action="store_true", help="Heterochronous data. Expect a date in the leaf names")
    p.add_argument("--clock", choices=["strict", "ace", "acln", "acg", "aoup", "ucln", "uced", "gmrf", "hsmrf"],
                   default=None, help="Type of clock")
    p.add_argument("--estimate_rate", action="store_true", help="Estimate substitution rate")
    p.add_argument("-c", "--coalescent", choices=["constant", "skyride", "skygrid"], default=None,
                   help="Type of coalescent (constant or skyride)")
    p.add_argument("--speciation", choices=["bd", "yule"], default=None, help="Speciation model")
    p.add_argument("--grid", metavar="I", type=int, help="Number of grid points in skygrid")
    p.add_argument("--cutoff", metavar="G", type=float, help="a cutoff for skygrid")
    p.add_argument("--compile", action="store_true", help="Check that the GPU engine loads")
    p.add_argument("--geo", action="store_true", help="Phylogeography (not supported)")
    p.add_argument("--rescaling_geo", action="store_true", help="Phylogeography (not supported)")
    return p


def create_run_parser(sub):
    p = create_build_parser(sub, "run", help="run an analysis")
    p.add_argument("-t", "--tree", required=True, help="Tree file")
    p.add_argument("-i", "--input", required=False, help="Sequence file")
    p.add_argument("-o", "--output", required=True, help="Stem for output files")
    p.add_argument("--lower_root", type=float, default=0.0, help="Lower bound of the root")
    p.add_argument("--rate", type=float, help="Substitution rate")
    p.add_argument("--dates", help="Comma-separated (csv) file containing sequence dates with header 'name,date'")
    p.add_argument("-a", "--algorithm", choices=["vb", "nuts", "hmc"], default="vb", type=str.lower,
                   help="Algorithm [default: %(default)s]")
    p.add_argument("-S", "--seed", type=int, help="Seed")
    p.add_argument("-q", "--variational", choices=["meanfield", "fullrank"], default="meanfield",
                   help="Variational distribution family")
    p.add_argument("-e", "--eta", type=float, help="eta (variational only)")
    p.add_argument("--elbo_samples", type=int, default=100, help="Monte Carlo draws per ELBO estimate")
    p.add_argument("--grad_samples", type=int, default=1, help="Monte Carlo draws per ELBO gradient")
    p.add_argument("--samples", type=int, default=1000, help="Draws from the variational distribution")
    p.add_argument("--tol_rel_obj", type=float, default=0.001, help="Relative ELBO convergence tolerance")
    p.add_argument("--chains", type=int, default=1, help="Number of chains (NUTS)")
    p.add_argument("--thin", type=int, default=1, help="Period for saving samples (NUTS)")
    p.add_argument("--iter", type=int, default=100000,
                   help="Maximum iterations (vb) or iterations including warmup (nuts)")
    p.add_argument("-M", "--metadata", help="Phylogeography metadata file (not supported)")
    p.add_argument("--metadata_key", help="Phylogeography (not supported)")
    p.add_argument("--device", type=int, default=None, help="HIP device (default LOCAL_RANK or 0)")
    return p


def _spec(arg):
    if arg.geo or getattr(arg, "metadata", None):
        raise SystemExit("phylogeography (--geo / -M) is not supported by this engine")
    return ModelSpec.from_args(arg)


def artifact_path(script):
    """phylostan.py:155-158 / :292-294: the compiled model's file name."""
    binary = script.replace(".stan", ".pkl")
    return script + ".pkl" if binary == script else binary


def compile_artifact(spec, script):
    """Load the HIP engine and write the compiled-model artifact (JSON)."""
    import hashlib
    from . import _lib
    _lib.load()
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "phylo_hip.hip")
    h = hashlib.sha1()
    if os.path.exists(src):
        with open(src, "rb") as fp:
            h.update(fp.read())
    doc = {"phylostan_amd_compiled": 1, "script": script, "options": dict(vars(spec)),
           "engine": _lib.LIB_PATH, "kernel_source_sha1": h.hexdigest()[:12],
           "note": "compiled-model artifact of the GPU engine (JSON; replaces the pickled pystan StanModel)"}
    path = artifact_path(script)
    with open(path, "w") as fp:
        json.dump(doc, fp, indent=1)
    return path


def load_artifact(script):
    path = artifact_path(script)
    try:
        with open(path) as fp:
            doc = json.load(fp)
    except (ValueError, UnicodeDecodeError):  # e.g. a real pystan pickle left at that path
        raise SystemExit("%s is not a compiled-model artifact of this engine" % path)
    if not isinstance(doc, dict) or doc.get("phylostan_amd_compiled") != 1:
        raise SystemExit("%s is not a compiled-model artifact of this engine" % path)
    from . import _lib
    _lib.load()
    return doc


def build(arg):
    spec = _spec(arg)
    doc = {"phylostan_amd_model": 1, "options": dict(vars(spec)),
           "note": "model description for the GPU engine (replaces the emitted Stan program)"}
    with open(arg.script, "w") as fp:
        json.dump(doc, fp, indent=1)
    if arg.compile:
        path = compile_artifact(spec, arg.script)
        print("GPU engine: %s (compiled model %s)" % (os.environ.get("PHYLO_HIP_LIB", "libphylo_hip.so"), path))


def _read_script(path):
    try:
        with open(path) as fp:
            doc = json.load(fp)
        return doc.get("options") if isinstance(doc, dict) and "phylostan_amd_model" in doc else None
    except (OSError, ValueError):
        return None


def load_run_data(arg):
    rooted = arg.clock is not None
    d = dataio.load(arg.tree, arg.input, rooted=rooted, heterochronous=arg.heterochronous or bool(arg.dates),
                    dates=arg.dates)
    return d


def run(arg, likelihood_factory=None, log=print):
    spec = _spec(arg)
    opts = _read_script(arg.script)
    if likelihood_factory is None:  # the GPU engine: compiled-model artifact (phylostan.py:292-300)
        if arg.compile or not os.path.lexists(artifact_path(arg.script)):
            compile_artifact(spec, arg.script)
        else:
            opts = load_artifact(arg.script)["options"]
    if opts is not None:
        for k in ("model", "categories", "invariant", "clock", "estimate_rate", "coalescent", "heterochronous"):
            if opts.get(k) != getattr(spec, k):
                raise SystemExit("run option %s=%r differs from the built model (%r)" % (k, getattr(spec, k),
                                                                                        opts.get(k)))
    if not arg.input:
        raise SystemExit("an alignment (-i) is required")
    d = load_run_data(arg)
    log("Number of sequences: {} length {} ".format(d.S, int(np.sum(d.weights))))
    log("Model: " + arg.model)
    C = spec.C
    chains = max(1, arg.chains) if arg.algorithm in ("nuts", "hmc") else 1
    # draws per likelihood call: one per chain (NUTS / HMC), else the ELBO / gradient samples
    max_draws = chains if arg.algorithm in ("nuts", "hmc") else max(arg.elbo_samples, arg.grad_samples, 1)
    if likelihood_factory is None:
        from .engine import TreeLikelihood
        dev = arg.device if arg.device is not None else int(os.environ.get("LOCAL_RANK", "0"))

        def make_lik():
            lk = TreeLikelihood(d.tipcodes, d.weights, d.peel0, d.rooted, arg.model, C, max_draws=max_draws,
                                device=dev)
            if max_draws * C <= 256:  # batches within one workgroup per CU: the lowest-latency engine
                lk.prefer_latency_engine()
            return lk
        lik = make_lik()
    else:
        make_lik = None
        lik = likelihood_factory(d.tipcodes, d.weights, d.peel0, d.rooted, arg.model, C)
    tree = TreeData.from_phylodata(d)
    if not spec.heterochronous:
        # --dates alone dates the tips (setup_dates) but, as in the reference,
        # only --heterochronous puts lowers / lower_root into the model's data
        # (phylostan.py:259-263): the model stays homochronous
        tree = TreeData(d.S, d.peel0, d.map, None, None)
    post = Posterior(spec, tree, lik, compact_rows=True)
    seed = arg.seed if arg.seed is not None else int(time.time()) % 100000
    rng = np.random.default_rng(seed)
    names = post.column_names()
    config = [("model", "phylostan_amd (GPU likelihood; Stan runtime removed)"), ("method", arg.algorithm),
              ("seed", seed), ("dimension", post.dim)]
    sample_path = arg.output
    tree_path = sample_path + ".trees"

    if arg.algorithm == "vb":
        from .advi import ADVI
        diag = stan_io.DiagWriter(sample_path + ".diag", config)
        adv = ADVI(post, rng, grad_samples=arg.grad_samples, elbo_samples=arg.elbo_samples, log=log)
        q0 = post.initialize(rng)
        t0 = time.time()
        q, eta, iters = adv.run(q0, eta=arg.eta, adapt_engaged=arg.eta is None, tol_rel_obj=arg.tol_rel_obj,
                                max_iterations=arg.iter, diag=diag, family=arg.variational)
        diag.close()
        log("TIME: %.3f" % (time.time() - t0))
        mean_row = post.flat_rows(q.mu[None])[0]
        draws = post.flat_rows(q.sample(rng, arg.samples)) if arg.samples > 0 else np.zeros((0, len(names)))
        stan_io.write_vb_csv(sample_path, names, mean_row, draws,
                             config + [("algorithm", arg.variational), ("iter", iters), ("eta", eta),
                                       ("elbo_samples", arg.elbo_samples),
                                       ("grad_samples", arg.grad_samples), ("tol_rel_obj", arg.tol_rel_obj),
                                       ("output_samples", arg.samples)], eta)
        stan_io.convert_samples_to_nexus(d.tree, sample_path, tree_path, arg.rate)
        stan_io.parse_log(sample_path, 0.05)
        return post
    from .nuts import run_chains
    num_warmup = arg.iter // 2
    num_samples = arg.iter - num_warmup
    q0s = [post.initialize(np.random.default_rng((seed, c, 0))) for c in range(chains)]
    t0 = time.time()
    # one batched context for all chains: every leapfrog round of all chains
    # is one small-batch likelihood call
    res = run_chains(post, q0s, [(seed, c) for c in range(chains)], num_warmup=num_warmup,
                     num_samples=num_samples, thin=arg.thin, progress=log, algorithm=arg.algorithm)
    el = time.time() - t0
    for c, ch in enumerate(res):
        rows = post.flat_rows(np.stack([dr[0] for dr in ch.draws]))
        path = sample_path if chains == 1 else sample_path + "_{}.csv".format(c)
        tpath = tree_path if chains == 1 else sample_path + "_{}.trees".format(c)
        if chains == 1 and sample_path.endswith(".csv"):
            tpath = sample_path.replace(".csv", ".trees")
        stan_io.write_nuts_csv(path, names, ch, rows,
                               config + [("chain", c), ("num_warmup", num_warmup), ("num_samples", num_samples),
                                         ("thin", arg.thin), ("gradient_evaluations", ch.n_grad)],
                               elapsed=(el / 2, el / 2), algorithm=arg.algorithm)
        stan_io.convert_samples_to_nexus(d.tree, path, tpath, arg.rate)
        stan_io.parse_log(path, 0.05)
    return post


def parse(arg):
    tree = dataio.read_tree(arg.tree)
    # phylostan.py:140-141: a root with more than two children is rerooted at
    # its first child's edge (run resolves polytomies instead, :175; for a
    # trifurcating root, e.g. DS1's, both give the same shape and numbering)
    if len(tree.seed_node.child_nodes()) > 2:
        tree.reroot_at_edge(tree.seed_node.child_nodes()[0].edge)
    dataio.setup_indexes(tree)
    dataio.setup_dates(tree, arg.dates, arg.heterochronous)
    stan_io.convert_samples_to_nexus(tree, arg.samples, arg.output, arg.rate)
    stan_io.parse_log(arg.samples, arg.alpha, tree)


def main(argv=None):
    parser = argparse.ArgumentParser(prog="phylostan", description="Phylogenetic inference on MI355X "
                                     "(GPU pruning likelihood, Stan runtime removed)")
    sub = parser.add_subparsers()
    create_build_parser(sub, "build", "build a model script").set_defaults(func=build)
    create_run_parser(sub).set_defaults(func=run)
    create_parse_parser(sub).set_defaults(func=parse)
    arg = parser.parse_args(argv)
    if not hasattr(arg, "func"):
        parser.print_help()
        return 1
    arg.func(arg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
