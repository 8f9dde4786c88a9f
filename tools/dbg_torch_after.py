"""Debug helper: does torch initialise the GPU after this library ran
evaluations (graphs on / off)?  python -m tools.dbg_torch_after {0|1} [n_calls] [import_first]"""
import sys

import numpy as np

from tests import cases


def main():
    graphs = int(sys.argv[1])
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    if len(sys.argv) > 3 and sys.argv[3] == "import_first":
        import torch  # noqa: F401  (loaded, not initialised)
    from phylostan_amd.engine import TreeLikelihood
    case = cases.fluA_case()
    e = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, max_draws=4)
    e.set_graphs(bool(graphs))
    bl = np.repeat(case.blens[None], 4, axis=0)
    mv = np.repeat(case.model_vec()[None], 4, axis=0)
    for _ in range(calls):
        e.evaluate_rows(bl, mv)
    import torch
    print("graphs", graphs, "calls", calls, "torch sees", torch.cuda.device_count(), flush=True)
    x = torch.ones(3, device="cuda:0")
    print("torch ok", float(x.sum()))


if __name__ == "__main__":
    main()
