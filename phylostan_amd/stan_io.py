"""The output-file contract of ``phylostan run`` / ``phylostan parse``.

* Sample CSV (what pystan writes to ``sample_file``): ``#`` comment lines, a
  header ``lp__,<sampler columns>,<params>,<transformed params>`` with Stan's
  ``name.k`` flattening, one row per draw.  NUTS adds the sampler columns
  ``accept_stat__,stepsize__,treedepth__,n_leapfrog__,divergent__,energy__``
  and the adaptation comment block; ADVI writes ``lp__ = 0`` rows, the first
  one being the mean of the approximation (Stan ``advi::run``).
* ``.diag`` (ADVI ``diagnostic_file``): ``iter,time_in_seconds,ELBO`` rows.
* ``.trees``: NEXUS written by ``convert_samples_to_nexus``
  (``phylostan/utils.py:193-287``), restated here on our tree objects.
* ``parse_log`` (``utils.py:290-409``): mean / median / CI summaries printed
  after a run and by ``phylostan parse``.
"""
import sys

import numpy as np

NUTS_COLUMNS = ["accept_stat__", "stepsize__", "treedepth__", "n_leapfrog__", "divergent__", "energy__"]
HMC_COLUMNS = ["accept_stat__", "stepsize__", "int_time__", "energy__"]  # diag_e_static_hmc


def _fmt(v):
    return "%.6g" % v


def write_nuts_csv(path, colnames, chain, rows, config, elapsed=None, save_warmup=False, algorithm="nuts"):
    """``rows``: [n_draws, len(colnames)] constrained values of the recorded
    draws of ``chain`` (a ``nuts.Chain`` or ``nuts.StaticHMCChain``), in the
    same order.  Static HMC writes Stan's HMC sampler columns."""
    hmc = algorithm == "hmc"
    with open(path, "w") as fp:
        for k, v in config:
            fp.write("# %s = %s\n" % (k, v))
        fp.write(",".join(["lp__"] + (HMC_COLUMNS if hmc else NUTS_COLUMNS) + colnames) + "\n")
        adapt_written = False
        for d, vals in zip(chain.draws, rows):
            q, lp, acc, eps, depth, nlf, div, energy, warm = d
            if warm and not save_warmup:
                continue
            if not warm and not adapt_written:
                fp.write("# Adaptation terminated\n# Step size = %g\n# Diagonal elements of inverse mass matrix:\n# %s\n"
                         % (chain.eps, ", ".join("%g" % x for x in chain.inv_metric)))
                adapt_written = True
            if hmc:  # the depth slot holds int_time
                sampler = [_fmt(lp), _fmt(acc), _fmt(eps), _fmt(depth), _fmt(energy)]
            else:
                sampler = [_fmt(lp), _fmt(acc), _fmt(eps), "%d" % depth, "%d" % nlf, "%d" % div, _fmt(energy)]
            fp.write(",".join(sampler + [_fmt(x) for x in vals]) + "\n")
        if elapsed is not None:
            w, s = elapsed
            fp.write("# \n#  Elapsed Time: %g seconds (Warm-up)\n#                %g seconds (Sampling)\n"
                     "#                %g seconds (Total)\n# \n" % (w, s, w + s))


def write_vb_csv(path, colnames, mean_row, draw_rows, config, eta):
    with open(path, "w") as fp:
        for k, v in config:
            fp.write("# %s = %s\n" % (k, v))
        fp.write(",".join(["lp__"] + colnames) + "\n")
        fp.write("# Stepsize adaptation complete.\n# eta = %g\n" % eta)
        fp.write(",".join(["0"] + [_fmt(x) for x in mean_row]) + "\n")
        for r in draw_rows:
            fp.write(",".join(["0"] + [_fmt(x) for x in r]) + "\n")


class DiagWriter:
    """ADVI diagnostic file: ``iter,time_in_seconds,ELBO``."""

    def __init__(self, path, config=()):
        self.fp = open(path, "w")
        for k, v in config:
            self.fp.write("# %s = %s\n" % (k, v))
        self.fp.write("iter,time_in_seconds,ELBO\n")

    def __call__(self, it, seconds, elbo):
        self.fp.write("%d,%.3f,%.6f\n" % (it, seconds, elbo))
        self.fp.flush()

    def close(self):
        self.fp.close()


# --------------------------------------------------------------------------
# utils.py:193-287
# --------------------------------------------------------------------------
def to_nexus(node, fp):
    if not node.is_leaf():
        fp.write("(")
        for i, n in enumerate(node.child_node_iter()):
            to_nexus(n, fp)
            if i == 0:
                fp.write(",")
        fp.write(")")
    else:
        fp.write(str(node.index))
    if hasattr(node, "date"):  # setup_dates gives every node a date (0.0 when isochronous)
        fp.write("[&height={}".format(node.date))
        if getattr(node, "rate", None) is not None:
            fp.write(",rate={}".format(node.rate))
        fp.write("]")
    if node.parent_node is not None:
        fp.write(":{}".format(node.edge_length))
    else:
        fp.write(";")


def convert_samples_to_nexus(tree, input, output, rate=None):
    S = len(tree.taxon_namespace)
    with open(output, "w") as outp:
        outp.write("#NEXUS\nBegin trees;\nTranslate\n")
        outp.write(",\n".join([str(i + 1) + " " + x.label.replace("'", "") for i, x in enumerate(tree.taxon_namespace)]))
        outp.write("\n;\n")
        header = None
        rows = []
        with open(input) as fp:
            for line in fp:
                if line.startswith("lp"):
                    header = line.strip().split(",")
                elif not line.startswith("#") and line.strip() and header is not None:
                    rows.append(line.strip().split(","))
        if header is None:
            raise ValueError("%s has no header line" % input)
        time_tree = "blens.1" not in header
        count = 1
        nodes = list(tree.postorder_node_iter())
        if time_tree:
            hindex = header.index("heights.1")
            strict = True
            rindex = None
            if rate is None:
                if "substrates.1" in header:
                    rindex = header.index("substrates.1")
                    strict = False
                else:
                    rindex = header.index("rate") if "rate" in header else None
            for l in rows:
                for n in nodes:
                    if not n.is_leaf():
                        n.date = float(l[hindex + n.index - S - 1])
                for n in nodes:
                    if n.parent_node is not None:
                        if strict:
                            n.rate = float(l[rindex]) if rate is None and rindex is not None else rate
                        else:
                            n.rate = float(l[rindex + n.index - 1])
                for n in nodes:
                    if n.parent_node is not None:
                        n.edge_length = n.parent_node.date - n.date
                outp.write("tree {} = ".format(count))
                count += 1
                to_nexus(tree.seed_node, outp)
                outp.write("\n")
        else:
            bindex = header.index("blens.1")
            for l in rows:
                for n in nodes:
                    if n.parent_node is not None:
                        k = bindex + n.index - 1
                        n.edge_length = float(l[k]) if k < len(l) else 0.0
                outp.write("tree {} = ".format(count))
                count += 1
                to_nexus(tree.seed_node, outp)
                outp.write("\n")
        outp.write("END;")


# --------------------------------------------------------------------------
# utils.py:290-409
# --------------------------------------------------------------------------
def descriptive_stats(d, alpha):
    median, low, high = np.quantile(d, (0.5, alpha / 2.0, 1.0 - alpha / 2.0))
    return np.mean(d), median, low, high


VARIABLES = {
    "wshape": "Weibull (shape)",
    "pinv": "Proportion invariant",
    "kappa": "HKY (kappa)",
    "rate": "Strict clock (rate)",
    "theta": "Constant population size (theta)",
    "tau": "GMRF precision (tau)",
    "netDiversificationRate": "net diversification rate",
    "relativeExtinctionRate": "relative extinction rate",
    "ucln_mean": "UCLN mean",
    "ucln_stdev": "UCLN stdev",
    "R": "effective reproductive number",
    "delta": "rate of becoming uninfectious",
    "s": "probability of an individual being sampled",
    "thetas": "effective population size",
    "heights": "coalescence times of nodes",
}


def read_samples(inputfile):
    header, rows = None, []
    with open(inputfile) as fp:
        for line in fp:
            line = line.strip()
            if line.startswith("lp"):
                header = line.split(",")
            elif not line.startswith("#") and len(line) != 0:
                rows.append([float(h) for h in line.split(",")])
    return header, np.array(rows).reshape(len(rows), len(header) if header else 0)


def parse_log(inputfile, alpha=0.05, tree=None, out=None):
    """Print the summaries of ``utils.parse_log``; returns them as a dict
    ``label -> (mean, median, low, high)``."""
    out = out or sys.stdout
    header, data = read_samples(inputfile)
    res = {}
    GTR = ("AC", "AG", "AT", "CG", "CT", "GC")
    freqs = ("A", "C", "G", "T")
    pct = (1 - alpha) * 100
    for var in header:
        if var == "rates.1":
            print("GTR", file=out)
            for i in range(6):
                m, md, lo, hi = descriptive_stats(data[:, header.index("rates." + str(i + 1))], alpha)
                res["rates.%d" % (i + 1)] = (m, md, lo, hi)
                print("  {} mean: {:.3E} {}% CI: ({:.3E},{:.3E})".format(GTR[i], m, pct, lo, hi), file=out)
            for i in range(4):
                m, md, lo, hi = descriptive_stats(data[:, header.index("freqs." + str(i + 1))], alpha)
                res["freqs.%d" % (i + 1)] = (m, md, lo, hi)
                print("  {} mean: {:.4f} {}% CI: ({:.4f},{:.4f})".format(freqs[i], m, pct, lo, hi), file=out)
        elif var in VARIABLES:
            if "substrates.1" not in header or var != "rate":
                m, md, lo, hi = descriptive_stats(data[:, header.index(var)], alpha)
                res[var] = (m, md, lo, hi)
                print("{} mean: {} {}% CI: ({},{})".format(VARIABLES[var], m, pct, lo, hi), file=out)
    if "heights.1" in header:
        idx_root, max_h = 0, 0
        for idx, h in enumerate(header):
            if h.startswith("heights.") and data[0, idx] > max_h:
                idx_root, max_h = idx, data[0, idx]
        m, md, lo, hi = descriptive_stats(data[:, idx_root], alpha)
        res["root_height"] = (m, md, lo, hi)
        print("Root height mean: {} {}% CI: ({},{})".format(m, pct, lo, hi), file=out)
        if tree is not None and "substrates.1" in header:
            # relaxed clock (utils.py:354-380): per draw the mean rate
            # sum(rate * time) / sum(time) over the branches; the "variance"
            # is numpy.var of every branch rate seen in this and all earlier
            # draws (the reference's list is never reset between draws)
            rindex = header.index("substrates.1")
            hindex = header.index("heights.1")
            S = len(tree.taxon_namespace)
            nodes = list(tree.postorder_node_iter())
            mean_rates, variances, rates = [], [], []
            for i in range(data.shape[0]):
                for n in nodes:
                    if not n.is_leaf():
                        n.date = data[i, hindex + n.index - S - 1]
                    if n.parent_node is not None:
                        n.rate = data[i, rindex + n.index - 1]
                        rates.append(n.rate)
                dist = tm = 0.0
                for n in nodes:
                    if n.parent_node is not None:
                        el = n.parent_node.date - n.date
                        dist += n.rate * el
                        tm += el
                mean_rates.append(dist / tm)
                variances.append(np.var(rates))
            m, md, lo, hi = descriptive_stats(mean_rates, alpha)
            res["mean_rate"] = (m, md, lo, hi)
            print("Mean rate mean: {} {}% CI: ({},{})".format(m, pct, lo, hi), file=out)
            m, md, lo, hi = descriptive_stats(variances, alpha)
            res["variance_rate"] = (m, md, lo, hi)
            print("Variance rate mean: {} {}% CI: ({},{})".format(m, pct, lo, hi), file=out)
    else:
        idx = [k for k, h in enumerate(header) if h.startswith("blens")]
        sums = data[:, idx].sum(axis=1)
        m, md, lo, hi = descriptive_stats(sums, alpha)
        res["tree_length"] = (m, md, lo, hi)
        print("Tree length mean: {} {}% CI: ({},{})".format(m, pct, lo, hi), file=out)
    for var in ("R", "delta", "s", "thetas", "heights"):
        if "%s.1" % var in header:
            print(var, file=out)
            for k, h in enumerate(header):
                if h.startswith("%s." % var):
                    m, md, lo, hi = descriptive_stats(data[:, k], alpha)
                    print("  {} mean: {:.3E} {}% CI: ({:.3E},{:.3E})".format(h, m, pct, lo, hi), file=out)
    return res
