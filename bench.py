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
    ap.add_argument("--no-synthetic", action="store_true",
                    help="skip the synthetic 128 x 1M sub-record of the default (fluA) run")
    ap.add_argument("--synthetic-steps", type=int, default=None,
                    help="timed steps of the synthetic sub-record (default: --steps, at least 20)")
    ap.add_argument("--synthetic-draws", type=int, default=1,
                    help="parameter points per step of the synthetic sub-record")
    ap.add_argument("--no-multidev", action="store_true",
                    help="skip the phy_create_multi leg of the synthetic sub-record under --gpus N > 1")
    ap.add_argument("--compact", action="store_true",
                    help="compact output rows (log-lik + every parameter gradient, no dL/dP block): the rows a "
                         "sampler consumes, and the payload of any reduction of them")
    ap.add_argument("--rehearse", action="store_true",
                    help="N > 1 rehearsal on a one-GPU box: every rank on device 0, gloo instead of RCCL for the "
                         "collectives (the line says so); checks the multi-rank path, measures nothing")
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
            tmp = "%s.%d.tmp.npz" % (cache, os.getpid())  # ranks may simulate side by side
            np.savez(tmp, **d)
            os.replace(tmp, cache)
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


TORCHRUN_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
                "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE",
                "TORCH_NCCL_ASYNC_ERROR_HANDLING", "TORCHELASTIC_ERROR_FILE")


def multidev_child(n, steps, warmup, sites, draws, timeout=300):
    """The in-boundary multi-device leg: ``bench.py --workload synthetic
    --multi-device n`` as a child process (one process, ONE phy_create_multi
    handle over devices 0..n-1, one ncclAllReduce of the output rows per
    evaluation inside the C-ABI -- eigen/prune_stan.hpp:9-17's single
    synchronous handle).  A child, with its own time limit, so a failure of
    that path is reported in the line instead of taking the run down."""
    import subprocess
    import tempfile
    env = {k: v for k, v in os.environ.items() if k not in TORCHRUN_ENV}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    fd, path = tempfile.mkstemp(prefix="phylo_multidev_", suffix=".json")
    os.close(fd)
    cmd = [sys.executable, os.path.abspath(__file__), "--workload", "synthetic", "--multi-device", str(n),
           "--steps", str(steps), "--warmup", str(warmup), "--sites", str(sites), "--draws", str(draws),
           "--no-cpu-baseline", "--compact", "--json-out", path]
    t0 = time.perf_counter()
    try:
        cp = subprocess.run(cmd, env=env, timeout=timeout, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        with open(path) as fp:
            txt = fp.read().strip()
        if cp.returncode != 0 or not txt:
            return dict(ok=False, returncode=cp.returncode, stderr_tail=cp.stderr.decode(errors="replace")[-600:])
        sub = json.loads(txt.splitlines()[-1])
        keep = ("value", "unit", "n_gpus", "ms_per_step", "steps", "warmup", "nominal_loglik", "row_doubles")
        out = {k: sub.get(k) for k in keep}
        out["devices"] = sub["config"].get("devices")
        out["reduction"] = sub["config"].get("reduction")
        out["roofline_kernel_avg_ms"] = sub["roofline"]["kernel_avg_ms"]
        out.update(ok=True, wall_s=time.perf_counter() - t0, command=" ".join(cmd[1:-2]))
        return out
    except subprocess.TimeoutExpired:
        return dict(ok=False, error="timed out after %d s" % timeout)
    except (OSError, ValueError, KeyError) as e:
        return dict(ok=False, error=repr(e))
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass


def synthetic_leg(args, world, rank, local, dev, cpu_group):
    """BASELINE.json config 4 inside the default run: the synthetic 128-taxon x
    1M-site GTR+W4 workload, ``--synthetic-draws``
    parameter points per step, its patterns sharded over the run's ranks
    (contiguous whole 128-pattern blocks) with ONE all-reduce(SUM) of the
    fp64 output rows per step over RCCL inside the timed
    region.  At N = 1 it is the one-GPU evaluation (no collective).  Returns
    the sub-record for rank 0's JSON line (None elsewhere)."""
    import torch
    import torch.distributed as dist
    from phylostan_amd.distributed import ShardedLikelihood

    t_setup = time.perf_counter()
    prob = synthetic_problem(args.sites)
    S, P = prob["tipcodes"].shape
    C = prob["C"]
    draws = max(1, args.synthetic_draws)
    # compact rows: log-lik and every parameter gradient (branch lengths, rates, mixture weights,
    # exchangeabilities, frequencies) -- a sampler's whole gradient -- without the dL/dP block, so the
    # step's one collective carries ~2 KB per draw instead of ~130 KB
    sl = ShardedLikelihood(prob["tipcodes"], prob["weights"], prob["peel0"], prob["rooted"], prob["model"], C,
                           rank, world, device=local, max_draws=draws, compact=True)
    eng = sl.engine
    info = {"engine": eng.engine()}
    if info["engine"] == "class":
        info.update({"class_" + k: v for k, v in eng.class_info().items()})
    B = eng.B
    rng = np.random.default_rng(4321)  # every rank evaluates the same points (its own patterns)
    steps = args.synthetic_steps or max(20, args.steps)
    warm = max(3, min(args.warmup, 10))
    nuniq = min(steps + warm, 8)
    blens, mvs = parameter_sets(prob, nuniq, draws, B, C, rng)
    d_blens = torch.tensor(blens, device=dev, dtype=torch.float64)
    d_model = torch.tensor(mvs, device=dev, dtype=torch.float64)
    d_out = torch.zeros((draws, eng.outlen), device=dev, dtype=torch.float64)
    stream = torch.cuda.Stream(device=dev)  # not the null stream: the engine and the collective share it
    setup_s = time.perf_counter() - t_setup

    def step(k):
        with torch.cuda.stream(stream):
            sl.evaluate(d_blens[k % nuniq], d_model[k % nuniq], d_out)

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(fn, n):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(n):
            fn(k)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        return max_over_ranks(time.perf_counter() - t0)

    for k in range(warm):
        step(k)
    elapsed = timed(lambda k: step(warm + k), steps)
    # the class sweep's launches (forward through reverse) on HIP events
    eng.timing_start()
    for k in range(steps):
        sl.engine.evaluate_device(d_blens[k % nuniq].data_ptr(), d_model[k % nuniq].data_ptr(), d_out.data_ptr(),
                                  0, n_draws=draws, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    kern_ms, nl = eng.timing_read()
    kern_avg_ms = max_over_ranks(kern_ms / max(nl, 1))
    allreduce = None
    if world > 1:  # the step's one collective alone (its payload: the compact rows), and the full rows beside it
        full_len = eng.outlen + 16 * C * B
        op = "all_reduce(SUM) fp64, %s" % ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend())
        allreduce = dict(op=op, payload="compact rows: log-lik + every parameter gradient, %d doubles per draw "
                                        "(the full rows' dL/dP block, %d doubles, is not reduced)"
                                        % (eng.outlen, 16 * C * B))
        for name, cols in (("compact", eng.outlen), ("full_rows", full_len)):
            buf = torch.zeros((draws, cols), device=dev, dtype=torch.float64)
            with torch.cuda.stream(stream):
                for _ in range(5):
                    dist.all_reduce(buf)
                ar = timed(lambda k: dist.all_reduce(buf), 50)
            allreduce[name] = dict(us_per_call=1e6 * ar / 50, bytes=buf.numel() * 8)
        allreduce["us_per_call"] = allreduce["compact"]["us_per_call"]
        allreduce["bytes"] = allreduce["compact"]["bytes"]
    step(0)  # parameter set 0, draw 0: the nominal point
    torch.cuda.synchronize(dev)
    row0 = d_out[0].double().cpu().numpy()
    value = draws * steps / elapsed  # whole-job: every step is one evaluation of the whole alignment

    alg = class_algorithmic_bytes(C, info["class_classes"], info["class_stage"], info["class_staged"], draws) \
        if info["engine"] == "class" else \
        algorithmic_bytes(S, sl.p1 - sl.p0, C, eng.program_info()["nslots"], B, draws)
    achieved = alg / (kern_avg_ms * 1e-3) / 1e9
    traffic = None
    if world == 1:
        traffic = pmc_record("synthetic", draws, info["engine"])

    if world > 1:
        dist.barrier(group=cpu_group)
    rec = None
    if rank == 0:
        hinfo = host_cpu_info()
        cpu = cpu_mt = None
        if world == 1 and not args.no_cpu_baseline:
            # bounded sample: ONE full evaluation of the whole alignment, one thread (~7 s)
            cpu, ref = cpu_baseline(prob, 0.0, info=hinfo)
            if hinfo["threads"] > 1:  # ... and one on every host thread this job may use (OpenMP over patterns)
                cpu_mt, _ = cpu_baseline(prob, 0.0, nthreads=hinfo["threads"], info=hinfo)
        else:  # the check only: the C port on every host thread this job may use
            from oracle import cpu as ocpu
            from phylostan_amd import models
            ref, _ = ocpu.evaluate(prob["tipcodes"], prob["weights"], prob["peel0"], prob["rooted"],
                                   models.MODEL_IDS[prob["model"]],
                                   models.model_vector(prob["freqs"], prob["rates"], prob["rs"], prob["ps"]),
                                   prob["blens"], C, nthreads=hinfo["threads"])
        rel = abs(row0[0] - ref[0]) / max(abs(ref[0]), 1e-300)
        g, gr = row0[1:1 + B], ref[1:1 + B]
        grel = float(np.max(np.abs(g - gr)) / max(np.max(np.abs(gr)), 1e-300))
        check = dict(gpu_loglik_nominal=float(row0[0]), cpu_loglik_nominal=float(ref[0]), rel_err=rel,
                     grad_blens_max_rel_err=grel, ok=bool(rel <= 1e-10 and grel <= 1e-8),
                     reference="oracle/cpu_pruner.c on the whole alignment (all-reduced rows at N > 1)")
        multidev = None
        if world > 1 and not args.no_multidev:
            multidev = multidev_child(world, max(10, steps // 2), 3, args.sites, draws)
            if multidev.get("ok") and multidev.get("nominal_loglik") is not None:
                r = abs(multidev["nominal_loglik"] - ref[0]) / abs(ref[0])
                multidev["nominal_rel_err"] = r
        rec = {
            "metric": METRIC["synthetic"],
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warm,
            "ms_per_step": 1e3 * elapsed / steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": DATA["synthetic"],
            "config": {"workload": "synthetic 128 x %d sites GTR+W4 (BASELINE config 4), %d draw%s per step, "
                                   "patterns sharded over %d rank%s, one all-reduce of the rows per step"
                                   % (args.sites, draws, "" if draws == 1 else "s", world,
                                      "" if world == 1 else "s"),
                       "taxa": S, "patterns": P, "patterns_per_rank": sl.p1 - sl.p0, "categories": C,
                       "branches": B, "draws_per_step": draws, "parallelism": "patterns%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBPS, "traffic": traffic, "per": "GPU (rank 0's shard)",
                         "kernel": "class sweep, forward through reverse (DESIGN.md 5b)" if info["engine"] == "class"
                         else "sweep_kernel",
                         "kernel_avg_ms": kern_avg_ms, "algorithmic_bytes_per_launch": alg,
                         "survey_model_bytes_per_launch": survey_bytes(S, sl.p1 - sl.p0, C, draws),
                         "hbm": counted_hbm(traffic, alg, kern_avg_ms),
                         "limiter": "latency / launch chain: dependent kernels per tree level (DESIGN.md 5b)"},
            "allreduce": allreduce,
            "cpu_baseline": cpu,
            "cpu_baseline_all_threads": cpu_mt,
            "nominal_check": check,
            "multidev": multidev,
            "program": info,
            "setup_s": setup_s,
        }
    if world > 1:
        dist.barrier(group=cpu_group)
    eng.close()
    return rec


def counted_hbm(traffic, alg, kern_avg_ms):
    """The rocprof-counted HBM rate of the dominant kernel: PMC bytes per
    launch (profiles/pmc_traffic.json, this kernel source) over the launch's
    average duration, and its fraction of the 8 TB/s peak; None-valued when
    no PMC record of this source exists."""
    if not traffic:
        return {"counted_gbps": None, "counted_frac": None, "traffic_over_algorithmic": None, "counted_note": None}
    g = traffic / (kern_avg_ms * 1e-3) / 1e9
    note = ("counted bytes below the algorithmic count: reuse in L2 / MALL (the small gathers of class vectors "
            "hit cache)" if traffic < alg else
            "counted bytes above the algorithmic count: re-read / re-staged bytes (DESIGN.md 7)")
    return {"counted_gbps": g, "counted_frac": g / PEAK_HBM_GBPS, "traffic_over_algorithmic": traffic / alg,
            "counted_note": note}


def pmc_record(workload, draws, engine):
    """The committed PMC HBM bytes per launch of this kernel source (None when
    profiles/pmc_traffic.json is of another source or lacks the key)."""
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(pmc) as fp:
            rec = json.load(fp)
        key = "%s:%d:%s" % (workload, draws, engine)
        if rec.get("kernel_source") == kernel_source_hash() and key in rec.get("per_launch_bytes", {}):
            return rec["per_launch_bytes"][key]
    except (OSError, ValueError):
        pass
    return None


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

    cpu_group = None
    if args.rehearse:
        local = 0  # the ranks share one GPU
    if world > 1:
        torch.cuda.set_device(local)
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        cpu_group = dist.new_group(backend="gloo")  # host-side waits (rank 0's CPU work, the multidev child)
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
            self.reduction = ("rccl all-reduce (ncclCommInitAll, distinct devices)" if len(set(self.devices)) > 1
                              else "device-side shard sum (one device)" if n > 1 else "none (one shard)")

        def evaluate(self, d_blens, d_model, d_out, stream=None):
            if stream is None:  # torch's current stream (bench.py's steps run under a non-null one)
                stream = torch.cuda.current_stream(d_out.device).cuda_stream
            self.engine.evaluate_device(d_blens.data_ptr(), d_model.data_ptr(), d_out.data_ptr(), 0,
                                        n_draws=d_blens.shape[0], stream=stream)

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
    if args.compact:
        eng.set_output(compact=True)
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

    # pre-generated, distinct parameter points for every step (seeded per rank for replicas; the
    # pattern shards of one evaluation share their points)
    rng = np.random.default_rng(1234 + (rank if batched else 0))
    nsets = args.warmup + args.steps
    nuniq = min(nsets, 16)
    blens, mvs = parameter_sets(prob, nuniq, draws, B, C, rng)
    d_blens = torch.tensor(blens, device=dev, dtype=torch.float64)
    d_model = torch.tensor(mvs, device=dev, dtype=torch.float64)
    d_out = torch.zeros((draws, eng.outlen), device=dev, dtype=torch.float64)
    stream = torch.cuda.Stream(device=dev)  # not the null stream: the engine and the collective share it

    def step(k):
        with torch.cuda.stream(stream):
            sl.evaluate(d_blens[k % nuniq], d_model[k % nuniq], d_out)

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
    full_len = 1 + B + 2 * C + 14 + 16 * C * B  # the full row (the dL/dP block included)
    eng.set_output(compact=True)
    d_out_c = torch.zeros((draws, eng.outlen), device=dev, dtype=torch.float64)
    h_out = torch.empty((draws, eng.outlen), dtype=torch.float64, pin_memory=True)
    nh = max(1, min(args.steps, 20))
    with torch.cuda.stream(stream):
        for k in range(2):
            sl.evaluate(d_blens[k % nuniq], d_model[k % nuniq], d_out_c)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ta = time.perf_counter()
    with torch.cuda.stream(stream):
        for k in range(nh):
            sl.evaluate(d_blens[k % nuniq], d_model[k % nuniq], d_out_c)
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
    eng.set_output(compact=args.compact)

    # cross-check: parameter set 0, draw 0 is the nominal point
    step(0)
    torch.cuda.synchronize(dev)
    ll_nominal = float(d_out[0, 0].item())

    single = None
    if args.single_eval and rank == 0:
        d_out1 = torch.zeros((1, eng.outlen), device=dev, dtype=torch.float64)
        for k in range(10):
            eng.evaluate_device(d_blens[0, :1].data_ptr(), d_model[0, :1].data_ptr(), d_out1.data_ptr(), 0,
                                n_draws=1, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        n1 = 200
        ta = time.perf_counter()
        for k in range(n1):
            eng.evaluate_device(d_blens[k % nuniq, :1].data_ptr(), d_model[k % nuniq, :1].data_ptr(),
                                d_out1.data_ptr(), 0, n_draws=1, stream=stream.cuda_stream)
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
            sampler["quad_plan"] = lk.quad_plan()  # the multi-wave small-call sweep
            for _ in range(20):
                lk.evaluate_rows(bl4, mv4)
            ta = time.perf_counter()
            for _ in range(300):
                lk.evaluate_rows(bl4, mv4)
            sampler[name + "_us_per_call"] = 1e6 * (time.perf_counter() - ta) / 300
            lk.close()
            # ADVI's gradient: grad_samples = 1 draw per call (phylostan.py:49), the
            # reference's commonest call (`phylostan run` defaults to -a vb)
            lk = sampler_ctx(name, 1)
            for _ in range(20):
                lk.evaluate_rows(bl4[:1], mv4[:1])
            ta = time.perf_counter()
            for _ in range(300):
                lk.evaluate_rows(bl4[:1], mv4[:1])
            sampler[name + "_us_per_call_1draw"] = 1e6 * (time.perf_counter() - ta) / 300
            lk.close()
            lk = sampler_ctx(name, 100)
            for _ in range(20):
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
    flops = survey_flops(S, P_local, C, draws)
    achieved_tf = flops / (kern_avg_ms * 1e-3) / 1e12
    traffic = None
    if args.shard_of <= 1 and not args.multi_device:  # the PMC record is of the whole workload, not a shard
        traffic = pmc_record(args.workload, draws, info["engine"])

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
                cflops = 64.0 * (2.0 * sq["SQ_INSTS_VALU_FMA_F64"] + sq["SQ_INSTS_VALU_MUL_F64"]
                                 + sq["SQ_INSTS_VALU_ADD_F64"])  # counted, not SURVEY 8d's algorithmic flops
                t = kern_avg_ms * 1e-3
                simd_cycles = t * 2.4e9 * 1024  # 256 CUs x 4 SIMDs at 2.4 GHz
                compute = {"fp64_tflops": cflops / t / 1e12, "fp64_peak_tflops": PEAK_FP64_TFLOPS,
                           "fp64_frac": cflops / t / 1e12 / PEAK_FP64_TFLOPS,
                           "valu_busy": 4.0 * sq["SQ_ACTIVE_INST_VALU"] / simd_cycles,
                           "instructions_per_wave": sq["SQ_INSTS"] / sq["SQ_WAVES"],
                           "source": "profiles/sq_counters.json (rocprofv3 --pmc SQ counters of this kernel source; "
                                     "SQ cycle counters in quad-cycles)"}
        except (OSError, ValueError, KeyError):
            compute = None

    if info["engine"] == "pattern":
        # The pattern sweep keeps p and q on chip (SURVEY.md 8d's byte model, which materialises them,
        # would put this kernel above the HBM peak), and its counters say fp64 VALU issue / latency
        # (profiles/sq_counters.json): it is priced against the fp64 vector roof with SURVEY.md 8d's
        # algorithmic flops, F = 244 C P (S-1) per evaluation; the HBM view is reported beside it.
        roofline = {
            "bound": "fp64-vector", "achieved": achieved_tf, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved_tf / PEAK_FP64_TFLOPS, "traffic": traffic,
            "kernel": kernel_name, "kernel_avg_ms": kern_avg_ms,
            "algorithmic_flops_per_launch": flops,
            "limiter": "fp64 VALU issue / latency at two waves per SIMD: the SIMDs issue about half of the "
                       "wave-cycles and wait on s_waitcnt most of the rest (profiles/sq_counters.json); counted "
                       "HBM traffic is far below the 8 TB/s roof",
            "hbm": dict({"achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBPS, "algorithmic_bytes_per_launch": alg,
                         "survey_model_bytes_per_launch": survey_bytes(S, P_local, C, draws)},
                        **counted_hbm(traffic, alg, kern_avg_ms)),
            "compute": compute,
        }
    else:
        roofline = {
            "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBPS, "traffic": traffic,
            "kernel": kernel_name, "kernel_avg_ms": kern_avg_ms,
            "algorithmic_bytes_per_launch": alg,
            "survey_model_bytes_per_launch": survey_bytes(S, P_local, C, draws),
            "survey_flops_frac": achieved_tf / PEAK_FP64_TFLOPS,
            "hbm": counted_hbm(traffic, alg, kern_avg_ms),
            "limiter": "latency / launch chain: one small dependent kernel per tree level (DESIGN.md 5b)",
        }

    synth = None
    if args.workload == "fluA" and not args.no_synthetic and args.shard_of <= 1 and not args.multi_device:
        eng.close()  # the headline's context is done: its memory back before the 1M-site shard's
        synth = synthetic_leg(args, world, rank, local, dev, cpu_group)

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
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_all_threads": cpu_mt,
            "host_inclusive": host_inclusive,
            "nominal_check": check,
            "single_eval": single,
            "sampler_latency": sampler,
            "draws_100": draws_100,
            "program": info,
            "nominal_loglik": ll_nominal,
            "row_doubles": eng.outlen,
            "kernel_source": kernel_source_hash(),
        }
        if args.multi_device:
            rec["config"]["reduction"] = sl.reduction
        if args.rehearse:
            rec["rehearsal"] = "every rank on device 0, gloo collectives: a check of the multi-rank path, not a measurement"
        if synth is not None:
            rec["synthetic"] = synth
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fp:
                fp.write(line + "\n")
        if check is not None and not check["ok"]:
            print("bench.py: GPU nominal log-lik disagrees with the CPU port", file=sys.stderr)
            sys.exit(3)
        if synth is not None and not synth["nominal_check"]["ok"]:
            print("bench.py: synthetic rows disagree with the CPU port", file=sys.stderr)
            sys.exit(3)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
