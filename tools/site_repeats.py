"""Site-repeat classes per node (pruner/tree.cpp:140-174).

For every internal node v and pattern i, the *lower class* of (v, i) is the
tuple of tip states under v; the forward partial p_v,i (and a_v,i = P_v p_v,i)
depends on pattern i only through it.  The *upper class* is the tuple of tip
states outside v's subtree (what the pre-order partial depends on).  Prints,
per dataset, the fraction of (node, pattern) forward work that is a repeat
(sum over nodes of P - distinct lower classes) and the same for the upper side.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def classes(tipcodes, peel0):
    S, P = tipcodes.shape
    N = 2 * S - 1
    low = [None] * N
    for t in range(S):
        _, low[t] = np.unique(tipcodes[t], return_inverse=True)
    nlow = {}
    for a, b, v in peel0:
        key = low[a].astype(np.int64) * (int(low[b].max()) + 1) + low[b]
        _, low[v] = np.unique(key, return_inverse=True)
        nlow[int(v)] = int(low[v].max()) + 1
    # upper classes: root has one class; child x of v: pair (up_v, low_sibling)
    up = [None] * N
    root = int(peel0[-1][2])
    up[root] = np.zeros(P, dtype=np.int64)
    nup = {}
    for a, b, v in peel0[::-1]:
        for ch, sib in ((a, b), (b, a)):
            key = up[v].astype(np.int64) * (int(low[sib].max()) + 1) + low[sib]
            _, up[ch] = np.unique(key, return_inverse=True)
            nup[int(ch)] = int(up[ch].max()) + 1
    return nlow, nup


def report(name, tipcodes, weights, peel0):
    S, P = tipcodes.shape
    nlow, nup = classes(tipcodes, peel0)
    root = int(peel0[-1][2])
    internal = [v for v in nlow if v != root]
    lw = sum(nlow[v] for v in internal)
    upi = sum(nup[v] for v in internal)
    upt = sum(nup[t] for t in range(S))
    return dict(dataset=name, taxa=S, patterns=P, sites=float(np.sum(weights)),
                forward_node_patterns=len(internal) * P, forward_distinct=lw,
                forward_repeat_frac=1 - lw / (len(internal) * P),
                upper_internal_distinct=upi, upper_internal_repeat_frac=1 - upi / (len(internal) * P),
                upper_tip_distinct=upt, upper_tip_repeat_frac=1 - upt / (S * P))


def main():
    from tests import cases
    out = []
    for name, fn in (("fluA", cases.fluA_case), ("HCV", cases.hcv_case), ("DS1", cases.ds1_case)):
        c = fn()
        out.append(report(name, c.tipcodes, c.weights, c.peel0))
    if "--synthetic" in sys.argv:
        from phylostan_amd import synthetic
        sites = int(os.environ.get("SITES", "1000000"))
        pd, _ = synthetic.simulate(n_sites=sites)
        out.append(report("synthetic%d" % sites, pd.tipcodes, pd.weights, pd.peel0))
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
