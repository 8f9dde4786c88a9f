#!/usr/bin/env python
"""Benchmark: log-likelihood + full-gradient evaluations per second.

Metric (BASELINE.json): "log-lik+grad evals/sec (HKY+W4, 69 taxa) at 1/2/4/8
MI355X; HBM-BW fraction".  One *evaluation* = P-matrices + post-order sweep +
root + pre-order gradient pass + dL/dP accumulation + finalize (loglik,
dL/dP[C][B][16], dlogL/dblens, /drs, /dps, root-frequency term), outputs left
in HBM.  One *step* = one batched evaluation of ``--draws`` independent
parameter points (distinct branch lengths and kappa per draw, pre-generated
on the device so nothing is cached across steps).

Workloads:
  fluA (default)  examples/fluA: 69 taxa, 238 patterns, HKY+W4 strict clock at
                  the README.md:104-108 means.  Multi-GPU = independent draw
                  batches per rank (weak scaling, no collective: each rank's
                  evaluations are complete).
  synthetic       128 taxa x 1M simulated sites GTR+W4 (phylostan_amd/
                  synthetic.py).  Multi-GPU = patterns sharded over ranks +
                  one RCCL all-reduce of the output vector per step (strong
                  scaling of one evaluation).

Launched as ``python bench.py`` (N=1) or under torch.distributed.run with
one rank per GPU.  Rank 0 prints ONE JSON line.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec
PEAK_FP64_TFLOPS = 78.6  # MI355X fp64 vector peak (no MFMA on this path)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=["fluA", "synthetic", "HCV", "DS1"], default="fluA")
    ap.add_argument("--draws", type=int, default=None,
                    help="parameter points per step (default: fluA/HCV/DS1 8192, synthetic 1)")
    ap.add_argument("--sites", type=int, default=1_000_000, help="synthetic: simulated sites")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sampler-latency", action="store_true",
                    help="skip the small-batch (sampler path) latency probe of the batched workloads")
    ap.add_argument("--single-eval", action="store_true",
                    help="also time unbatched (draws=1) evaluations and report them")
    ap.add_argument("--wg-budget", type=int, default=0)
    ap.add_argument("--cols", type=int, default=0, help="pattern columns per lane (0 = automatic)")
    ap.add_argument("--lds-budget", type=int, default=0)
    ap.add_argument("--engine", choices=["auto", "pattern", "class"], default="auto",
                    help="pattern sweep, class sweep (site repeats) or the context's automatic choice")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--shard-of", type=int, default=0,
                    help="evaluate only the first of this many pattern shards on one GPU, with no collective -- "
                         "what each rank of a site-sharded N-GPU run computes (a projection, not the headline; "
                         "for the batched workloads, SURVEY 8e's site sharding beside the replicas)")
    ap.add_argument("--multi-device", type=int, default=0,
                    help="one process, ONE context over this many devices (phy_create_multi: pattern shards on "
                         "devices 0..N-1, one RCCL all-reduce of the output rows inside the C-ABI, or a device-side "
                         "sum when the box has fewer GPUs than shards -- the reference boundary's single handle, "
                         "eigen/prune_stan.hpp:9-17); parallelism multidevN")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check only: ranks join a gloo group on the CPU, all-reduce their rank "
                         "ids and exit (no GPU, no evaluation)")
    return ap.parse_args()


def kernel_source_hash():
    h = hashlib.sha1()
    for name in ("phylo_hip.hip", "class_engine.inc", "quad_engine.inc", "multi_device.inc"):
        with open(os.path.join(ROOT, "phylostan_amd", "csrc", name), "rb") as fp:
            h.update(fp.read())
    return h.hexdigest()[:12]


def fluA_problem():
    from tests import cases
    c = cases.fluA_case()
    return dict(tipcodes=c.tipcodes, weights=c.weights, peel0=c.peel0, rooted=True, model="HKY",
                C=4, blens=c.blens, freqs=c.freqs, kappa=5.58, rates=c.rates, rs=c.rs, ps=c.ps)


def hcv_problem():
    """BASELINE config 3: examples/HCV, GTR+W4 at rates (1,2,1,1,2,1)/8, pi = 1/4,
    alpha 0.5, clock rate 7.9e-4 on the input-tree heights (SConstruct:218)."""
    from tests import cases
    c = cases.hcv_case()
    return dict(tipcodes=c.tipcodes, weights=c.weights, peel0=c.peel0, rooted=True, model="GTR",
                C=4, blens=c.blens, freqs=c.freqs, kappa=None, rates=c.rates, rs=c.rs, ps=c.ps)


def ds1_problem():
    """BASELINE config 1: examples/DS1 tree 0, JC69 unrooted (root branch
    merged), blens ~ Exp(10) seed 0 -- the reference runs it on the CPU only."""
    from tests import cases
    c = cases.ds1_case()
    return dict(tipcodes=c.tipcodes, weights=c.weights, peel0=c.peel0, rooted=False, model="JC69",
                C=1, blens=c.blens, freqs=c.freqs, kappa=None, rates=c.rates, rs=np.asarray(c.rs),
                ps=np.asarray(c.ps))


BATCHED = {"fluA": fluA_problem, "HCV": hcv_problem, "DS1": ds1_problem}
METRIC = {
    "fluA": "log-lik+grad evals/sec (HKY+W4, 69 taxa) at 1/2/4/8 MI355X; HBM-BW fraction",
    "HCV": "log-lik+grad evals/sec (GTR+W4, 63 taxa, HCV)",
    "DS1": "log-lik+grad evals/sec (JC69 unrooted, 27 taxa, DS1)",
    "synthetic": "log-lik+grad evals/sec (GTR+W4, 128 taxa x 1M sites)",
}
DATA = {
    "fluA": "fluA alignment patterns + input-tree heights (tests/golden fixture of examples/fluA)",
    "HCV": "HCV alignment patterns + input-tree heights (tests/golden fixture of examples/HCV)",
    "DS1": "DS1 alignment patterns + tree 0, branch lengths ~ Exp(10) seed 0 (tests/golden fixture)",
    "synthetic": "synthetic (Kingman 128 taxa, simulated GTR+W4 sites, seed 0)",
}


def synthetic_problem(sites):
    from phylostan_amd import synthetic
    cache = "/tmp/phylostan_amd_synth_%d.npz" % sites
    if os.path.exists(cache):
        z = np.load(cache, allow_pickle=False)
        d = {k: z[k] for k in z.files}
    else:
        pd, prm = synthetic.simulate(n_sites=sites)
        d = dict(tipcodes=pd.tipcodes, weights=pd.weights, peel0=pd.peel0, **prm)
        try:
            np.savez(cache + ".tmp.npz", **d)
            os.replace(cache + ".tmp.npz", cache)
        except OSError:
            pass
    return dict(tipcodes=d["tipcodes"], weights=d["weights"], peel0=d["peel0"], rooted=True,
                model="GTR", C=4, blens=d["blens"], freqs=d["freqs"], kappa=None, rates=d["rates"],
                rs=d["rs"], ps=d["ps"])


def algorithmic_bytes(S, P, C, nslots, B, draws):
    """HBM bytes one sweep launch must move (DESIGN.md "Roofline"): every
    stored moved partial written once + read once (2 x 32 B per stored slot
    per column; ``nslots`` = the slots the plan stores, i.e. non-root internal
    nodes minus recomputed cherries), tip codes (S/2 B/pattern: 4-bit record
    indices), weights (8 B/pattern), P-matrices in + dL/dP out (2 x 128 B per
    branch-category)."""
    per_draw = 64 * nslots * C * P + S * P // 2 + 8 * P + 256 * B * C
    return per_draw * draws


def class_algorithmic_bytes(C, classes, stage, staged, draws):
    """HBM bytes of one class-sweep evaluation (DESIGN.md "Class sweep"):
    per category, every non-root subtree class's moved partial is written
    once (forward) and its aggregated upper partial written and read once --
    3 x 32 B per class; every contribution a parent class makes to an
    internal child (``stage`` of them) needs that child's vector gathered in
    the forward and again in the reverse -- 2 x 32 B; the ``staged`` ones
    (secondary children) are also stored and read back by the segmented
    reduction -- 2 x 32 B more (a primary child's are reduced in registers)."""
    return 32 * C * (3 * classes + 2 * stage + 2 * staged) * draws


def survey_bytes(S, P, C, draws):
    """SURVEY.md 8d model: B_eval = P (224 C (S-2) + 3 S + 16)."""
    return P * (224 * C * (S - 2) + 3 * S + 16) * draws


def survey_flops(S, P, C, draws):
    """SURVEY.md 8d's algorithmic flops: F_eval = 244 C P (S-1) (forward 60
    per node, reverse 92 per branch)."""
    return 244.0 * C * P * (S - 1) * draws


def host_cpu_info():
    """CPU model, nproc, and the host threads this job may use: the CPUs in
    its affinity mask, capped by a cgroup CPU quota when one is set (the GPU
    box gives each one-GPU job a share of a larger machine)."""
    model = None
    try:
        with open("/proc/cpuinfo") as fp:
            for line in fp:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fp:
            q, per = fp.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    threads = min(usable, quota) if quota else usable
    return dict(model=model, nproc=nproc, affinity=usable, cgroup_quota_cpus=quota, threads=threads)


def cpu_baseline(prob, seconds, nthreads=1, info=None):
    """The C oracle (oracle/cpu_pruner.c, 'port') on the same workload at the
    nominal parameter point (= the GPU's draw 0 of parameter set 0),
    single-threaded by default (Stan evaluates log_prob on one thread per
    chain); nthreads > 1 runs its OpenMP loop over patterns."""
    from oracle import cpu
    from phylostan_amd import models
    kind = models.MODEL_IDS[prob["model"]]
    mv = models.model_vector(prob["freqs"], prob["rates"], prob["rs"], prob["ps"])
    S, P = prob["tipcodes"].shape
    n = 0
    t0 = time.perf_counter()
    out = None
    while True:
        out, _ = cpu.evaluate(prob["tipcodes"], prob["weights"], prob["peel0"], prob["rooted"], kind, mv,
                              prob["blens"], prob["C"], nthreads=nthreads)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    rec = dict(value=n / el, unit="evals/s", cores=nthreads, kind="port",
               sample="%d full log-lik+grad evaluations of the %d-taxon x %d-pattern workload in %.1f s, "
                      "%d thread%s (oracle/cpu_pruner.c, gcc -O2%s)"
                      % (n, S, P, el, nthreads, "" if nthreads == 1 else "s",
                         "" if nthreads == 1 else ", OpenMP over patterns"))
    if info:
        rec.update(cpu_model=info["model"], nproc=info["nproc"], affinity_cpus=info["affinity"],
                   cgroup_quota_cpus=info["cgroup_quota_cpus"])
    return rec, out


def spawn_ranks(args):
    """``python bench.py --gpus N`` without a launcher: start N rank processes
    through torch.distributed.run (one per GPU) before anything touches HIP,
    and exit with the launcher's code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def parameter_sets(prob, nuniq, draws, B, C, rng):
    """Distinct parameter points for every step.  Draw 0 of set 0 is the
    nominal point the CPU baseline evaluates (the cross-check); every other
    draw scales the branch lengths by U(0.8, 1.25) and kappa (HKY) or the
    exchangeabilities (GTR/JC69) by random factors."""
    from phylostan_amd import models
    blens = np.empty((nuniq, draws, B))
    mvs = np.empty((nuniq, draws, 10 + 2 * C))
    for k in range(nuniq):
        scale = rng.uniform(0.8, 1.25, (draws, 1))
        if k == 0:
            scale[0] = 1.0
        blens[k] = prob["blens"][None, :] * scale
        for d in range(draws):
            nominal = k == 0 and d == 0
            if prob["kappa"] is not None:
                rates = models.hky_exchangeabilities(prob["kappa"] * (1.0 if nominal else rng.uniform(0.8, 1.25)))
            else:
                rates = prob["rates"] * (1.0 if nominal else rng.uniform(0.9, 1.1, 6))
            mvs[k, d] = models.model_vector(prob["freqs"], rates, prob["rs"], prob["ps"])
    return blens, mvs


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (one rank per GPU)" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    if args.dry_run:
        total = rank
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.tensor([rank], dtype=torch.int64)
            dist.all_reduce(t)
            total = int(t.item())
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "sum_of_ranks": total}), flush=True)
        return

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from phylostan_amd.distributed import ShardedLikelihood

    class MultiDeviceLikelihood:
        """bench's view of one phy_create_multi context (--multi-device N):
        shards on devices 0..N-1 (all on device 0 when the box has fewer GPUs:
        the device-side shard sum), inputs and rows on device 0."""

        def __init__(self, prob, C, n, max_draws):
            from phylostan_amd.engine import TreeLikelihood
            ndev = torch.cuda.device_count()
            self.devices = list(range(n)) if ndev >= n else [0] * n
            self.engine = TreeLikelihood(prob["tipcodes"], prob["weights"], prob["peel0"], prob["rooted"],
                                         prob["model"], C, max_draws=max_draws, devices=self.devices)
            self.p0, self.p1 = 0, prob["tipcodes"].shape[1]
            self.world = 1

        def evaluate(self, d_blens, d_model, d_out, stream=None):
            self.engine.evaluate_device(d_blens.data_ptr(), d_model.data_ptr(), d_out.data_ptr(), 0,
                                        n_draws=d_blens.shape[0], stream=stream or 0)

    batched = args.workload in BATCHED
    if batched:
        prob = BATCHED[args.workload]()
        draws = args.draws or 8192
        shard_world, shard_rank = 1, 0  # replicas: every rank runs complete evaluations
        if args.shard_of > 1:  # also report site sharding of a small alignment (projection)
            if world > 1:
                raise SystemExit("bench.py: --shard-of is a one-GPU projection; run it without a launcher")
            shard_world = args.shard_of
    else:
        prob = synthetic_problem(args.sites)
        draws = args.draws or 1
        shard_world, shard_rank = world, rank
        if args.shard_of > 1:
            if world > 1:
                raise SystemExit("bench.py: --shard-of is a one-GPU projection; run it without a launcher")
            shard_world = args.shard_of
    S, P = prob["tipcodes"].shape
    C = prob["C"]

    if args.multi_device:
        if world > 1 or args.shard_of > 1:
            raise SystemExit("bench.py: --multi-device is one process driving N devices; run it without a launcher "
                             "and without --shard-of")
        sl = MultiDeviceLikelihood(prob, C, args.multi_device, draws)
    else:
        sl = ShardedLikelihood(prob["tipcodes"], prob["weights"], prob["peel0"], prob["rooted"], prob["model"],
                               C, shard_rank, shard_world, device=local, max_draws=draws)
    if args.shard_of > 1:
        sl.world = 1  # the projection: one shard's evaluation, no collective
    eng = sl.engine
    if args.engine != "auto":
        eng.set_engine(args.engine)
    if args.wg_budget or args.cols or args.lds_budget:
        eng.set_tuning(args.wg_budget, args.cols, args.lds_budget)
    info = eng.program_info()
    info.update(eng.lds_plan())
    info["engine"] = eng.engine()
    if info["engine"] == "class":
        info.update({"class_" + k: v for k, v in eng.class_info().items()})
    B = eng.B
    P_local = sl.p1 - sl.p0

    # pre-generated, distinct parameter points for every step (seeded per rank)
    rng = np.random.default_rng(1234 + rank)
    nsets = args.warmup + args.steps
    nuniq = min(nsets, 16)
    blens, mvs = parameter_sets(prob, nuniq, draws, B, C, rng)
    d_blens = torch.tensor(blens, device=dev, dtype=torch.float64)
    d_model = torch.tensor(mvs, device=dev, dtype=torch.float64)
    d_out = torch.zeros((draws, eng.outlen), device=dev, dtype=torch.float64)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step(k):
        sl.evaluate(d_blens[k % nuniq], d_model[k % nuniq], d_out, stream=stream)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # the dominant kernel's duration: the same K steps again under the
    # engine's HIP-event timing (timed launches run direct, not from the
    # engine's HIP graphs -- so they do not share the throughput loop)
    eng.timing_start()
    for k in range(args.steps):
        step(args.warmup + k)
    torch.cuda.synchronize(dev)
    kern_ms, nlaunch = eng.timing_read()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        km = torch.tensor([kern_ms / max(nlaunch, 1)], device=dev, dtype=torch.float64)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kern_avg_ms = float(km.item())
    else:
        kern_avg_ms = kern_ms / max(nlaunch, 1)

    if batched:
        total_evals = world * draws * args.steps
    else:
        total_evals = draws * args.steps
    value = total_evals / elapsed

    # host-inclusive: the same steps with compact output rows (log-lik and
    # every parameter gradient, no dL/dP block: what a sampler consumes),
    # each followed by their D2H copy into pinned host memory
    full_len = eng.outlen
    eng.set_output(compact=True)
    d_out_c = torch.zeros((draws, eng.outlen), device=dev, dtype=torch.float64)
    h_out = torch.empty((draws, eng.outlen), dtype=torch.float64, pin_memory=True)
    nh = max(1, min(args.steps, 20))
    for k in range(2):
        sl.evaluate(d_blens[k % nuniq], d_model[k % nuniq], d_out_c, stream=stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ta = time.perf_counter()
    for k in range(nh):
        sl.evaluate(d_blens[k % nuniq], d_model[k % nuniq], d_out_c, stream=stream)
        h_out.copy_(d_out_c, non_blocking=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    tb = time.perf_counter()
    host_el = tb - ta
    if world > 1:
        t = torch.tensor([host_el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        host_el = float(t.item())
    host_inclusive = dict(value=(total_evals / args.steps) * nh / host_el, unit="evals/s", steps=nh,
                          bytes_to_host_per_eval=8 * eng.outlen, full_row_bytes=8 * full_len,
                          note="compact output rows (log-lik, branch / rate / mixture / frequency / "
                               "exchangeability gradients; no dL/dP block), each step followed by their D2H "
                               "copy into pinned host memory")
    eng.set_output(compact=False)

    # cross-check: parameter set 0, draw 0 is the nominal point
    step(0)
    torch.cuda.synchronize(dev)
    ll_nominal = float(d_out[0, 0].item())

    single = None
    if args.single_eval and rank == 0:
        d_out1 = torch.zeros((1, eng.outlen), device=dev, dtype=torch.float64)
        for k in range(10):
            eng.evaluate_device(d_blens[0, :1].data_ptr(), d_model[0, :1].data_ptr(), d_out1.data_ptr(), 0,
                                n_draws=1, stream=stream)
        torch.cuda.synchronize(dev)
        n1 = 200
        ta = time.perf_counter()
        for k in range(n1):
            eng.evaluate_device(d_blens[k % nuniq, :1].data_ptr(), d_model[k % nuniq, :1].data_ptr(),
                                d_out1.data_ptr(), 0, n_draws=1, stream=stream)
        torch.cuda.synchronize(dev)
        tb = time.perf_counter()
        single = dict(evals_per_s=n1 / (tb - ta), us_per_eval=1e6 * (tb - ta) / n1)

    # the sampler path (host buffers, compact rows -- what phylostan run
    # issues): µs per call of 4 draws (NUTS, one draw per chain) and the
    # evals/s of ADVI's ELBO estimate, elbo_samples = 100 draws per call
    # (phylostan.py:47), on the pattern sweep (its quad form for the 4-draw
    # call)
    sampler = draws_100 = None
    if batched and rank == 0 and world == 1 and not args.no_sampler_latency:
        from phylostan_amd.engine import TreeLikelihood
        sampler = {"draws_per_call": 4}
        draws_100 = {"draws_per_call": 100, "unit": "evals/s",
                     "note": "ADVI's ELBO estimate (elbo_samples = 100, phylostan.py:47): host buffers in, "
                             "compact rows out, one synchronous call each"}
        bl4, mv4 = blens[0][:4].copy(), mvs[0][:4].copy()
        bl100 = np.concatenate([blens[0]] * (1 + 100 // draws))[:100].copy()
        mv100 = np.concatenate([mvs[0]] * (1 + 100 // draws))[:100].copy()
        def sampler_ctx(name, n):
            # sized as the CLI sizes its contexts: max_draws = the draws of one call
            # (a 4-chain NUTS context plans for 4 draws, an ELBO context for 100)
            lk = TreeLikelihood(prob["tipcodes"], prob["weights"], prob["peel0"], prob["rooted"], prob["model"],
                                C, max_draws=n, device=local)
            lk.set_output(compact=True)
            lk.set_engine(name)
            return lk

        for name in ("pattern",):
            lk = sampler_ctx(name, 4)
            for _ in range(20):
                lk.evaluate_rows(bl4, mv4)
            ta = time.perf_counter()
            for _ in range(300):
                lk.evaluate_rows(bl4, mv4)
            sampler[name + "_us_per_call"] = 1e6 * (time.perf_counter() - ta) / 300
            lk.close()
            lk = sampler_ctx(name, 100)
            for _ in range(5):
                lk.evaluate_rows(bl100, mv100)
            ta = time.perf_counter()
            for _ in range(100):
                lk.evaluate_rows(bl100, mv100)
            el100 = (time.perf_counter() - ta) / 100
            draws_100[name] = 100 / el100
            draws_100[name + "_us_per_call"] = 1e6 * el100
            lk.close()

    if info["engine"] == "class":
        alg = class_algorithmic_bytes(C, info["class_classes"], info["class_stage"], info["class_staged"], draws)
        kernel_name = "class sweep: cls_clade_fwd/cls_fwd/cls_root/cls_red/cls_fix_list/cls_rev/cls_clade_rev kernels, forward through reverse"
    else:
        alg = algorithmic_bytes(S, P_local, C, info["nslots"] - info.get("recomputed", 0), B, draws)
        kernel_name = "sweep_kernel"
    achieved = alg / (kern_avg_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc) and args.shard_of <= 1:  # the PMC record is of the whole workload, not a shard
        try:
            with open(pmc) as fp:
                rec = json.load(fp)
            key = "%s:%d:%s" % (args.workload, draws, info["engine"])
            if rec.get("kernel_source") == kernel_source_hash() and key in rec.get("per_launch_bytes", {}):
                traffic = rec["per_launch_bytes"][key]
        except (OSError, ValueError):
            traffic = None

    # compute side of the same kernel (rocprofv3 SQ counters, tools/pmc_sq.py,
    # same kernel source only): fp64 FLOP rate against the vector peak and
    # the VALU's busy fraction -- the sweep is issue/latency-bound at two
    # waves per SIMD, not HBM-bound
    compute = None
    sqp = os.path.join(ROOT, "profiles", "sq_counters.json")
    if os.path.exists(sqp) and info["engine"] == "pattern" and batched:
        try:
            rec = json.load(open(sqp))
            sq = rec.get("per_launch", {}).get("%s:pattern" % args.workload)
            if rec.get("kernel_source") == kernel_source_hash() and sq:
                flops = 64.0 * (2.0 * sq["SQ_INSTS_VALU_FMA_F64"] + sq["SQ_INSTS_VALU_MUL_F64"]
                                + sq["SQ_INSTS_VALU_ADD_F64"])
                t = kern_avg_ms * 1e-3
                simd_cycles = t * 2.4e9 * 1024  # 256 CUs x 4 SIMDs at 2.4 GHz
                compute = {"fp64_tflops": flops / t / 1e12, "fp64_peak_tflops": PEAK_FP64_TFLOPS,
                           "fp64_frac": flops / t / 1e12 / PEAK_FP64_TFLOPS,
                           "valu_busy": 4.0 * sq["SQ_ACTIVE_INST_VALU"] / simd_cycles,
                           "instructions_per_wave": sq["SQ_INSTS"] / sq["SQ_WAVES"],
                           "source": "profiles/sq_counters.json (rocprofv3 --pmc SQ counters of this kernel source; "
                                     "SQ cycle counters in quad-cycles)"}
        except (OSError, ValueError, KeyError):
            compute = None

    cpu = cpu_mt = check = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the CPU baseline is an N=1 figure
        hinfo = host_cpu_info()
        cpu, cpu_out = cpu_baseline(prob, args.cpu_seconds, info=hinfo)
        # the same port on every host thread this job may use (reported beside it)
        if hinfo["threads"] > 1:
            cpu_mt, _ = cpu_baseline(prob, max(2.0, args.cpu_seconds / 2), nthreads=hinfo["threads"], info=hinfo)
        if shard_world == 1:
            ref = float(cpu_out[0])
            rel = abs(ll_nominal - ref) / max(abs(ref), 1e-300)
            check = dict(gpu_loglik_nominal=ll_nominal, cpu_loglik_nominal=ref, rel_err=rel, ok=rel <= 1e-10)

    if rank == 0:
        rec = {
            "metric": METRIC[args.workload],
            "value": value,
            "unit": "evals/s",
            "n_gpus": len(set(sl.devices)) if args.multi_device else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak" if batched and args.shard_of <= 1 and not args.multi_device else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": DATA[args.workload],
            "config": {
                "workload": {"fluA": "fluA HKY+W4 strict clock, %d parameter draws per step" % draws,
                             "HCV": "HCV GTR+W4 strict clock, %d parameter draws per step" % draws,
                             "DS1": "DS1 JC69 unrooted, %d parameter draws per step" % draws}.get(
                    args.workload, "synthetic 128 x %d sites GTR+W4, pattern-sharded" % args.sites),
                "taxa": S, "patterns": P, "patterns_per_rank": P_local, "categories": C,
                "branches": B, "draws_per_step": draws,
                "parallelism": ("multidev%d" % args.multi_device) if args.multi_device else
                               ("replicas%d" % world) if batched else ("patterns%d" % world),
                "devices": sl.devices if args.multi_device else None,
                "projection_shard_of": args.shard_of or None,
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBPS, "traffic": traffic,
                "kernel": kernel_name, "kernel_avg_ms": kern_avg_ms,
                "algorithmic_bytes_per_launch": alg,
                "survey_model_bytes_per_launch": survey_bytes(S, P_local, C, draws),
                # SURVEY.md 8d's flops per evaluation over the same launch time, against the fp64 vector peak
                "survey_flops_frac": survey_flops(S, P_local, C, draws) / (kern_avg_ms * 1e-3) / 1e12
                / PEAK_FP64_TFLOPS,
                # what actually limits the kernel: the byte roof above is the bound the
                # contract prices against; the counters say instruction issue / latency
                "limiter": ("issue/latency: SQ counters show the SIMDs issuing about half of the wave-cycles "
                            "and waiting on s_waitcnt most of the rest (profiles/sq_counters.json); counted HBM "
                            "traffic is below the 8 TB/s roof" if info["engine"] == "pattern" else
                            "latency / launch chain: one small dependent kernel per tree level (DESIGN.md 5b)"),
                "compute": compute,
            },
            "cpu_baseline": cpu,
            "cpu_baseline_all_threads": cpu_mt,
            "host_inclusive": host_inclusive,
            "nominal_check": check,
            "single_eval": single,
            "sampler_latency": sampler,
            "draws_100": draws_100,
            "program": info,
            "kernel_source": kernel_source_hash(),
        }
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fp:
                fp.write(line + "\n")
        if check is not None and not check["ok"]:
            print("bench.py: GPU nominal log-lik disagrees with the CPU port", file=sys.stderr)
            sys.exit(3)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
