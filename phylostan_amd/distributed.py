"""Multi-GPU: one process per GPU, site patterns sharded, one RCCL all-reduce.

SURVEY.md 8e: patterns are independent, so each rank owns a contiguous,
count-balanced range of patterns and evaluates its shard with its own
``phy_ctx``.  Every entry of the per-draw output vector (log-likelihood,
dL/dP, branch / rate / mixture / root-frequency gradients) is a sum over
patterns, so a single ``all_reduce(SUM)`` of that vector -- over RCCL
(``torch.distributed`` backend "nccl" on ROCm) between MI355X GPUs on xGMI --
is the whole exchange.  With ``compact=True`` (what a sampler consumes: the
log-likelihood and every parameter gradient -- branch lengths, rates,
mixture weights, exchangeabilities, frequencies) the rows stop before the
dL/dP block: for S = 128, C = 4 that is 1 + 254 + 8 + 14 doubles = 2.2 KB
per draw instead of 132 KB with the block (1 + 254 + 8 + 14 + 16*4*254
doubles).  The model-parameter gradients are linear in dL/dP and the root
term, so the compact rows of the shards sum to the compact rows of the
whole (tests/test_distributed.py).

The reference has no distributed code at all ("Parallelism");
this module is the build's addition.  ``engine_factory`` lets the CPU tests
substitute a shard evaluator (gloo, world size 2) for the HIP one.
"""
import numpy as np


ALIGN = 128  # patterns per sweep block at two columns per lane


def shard_range(P, rank, world, align=ALIGN):
    """Contiguous pattern range [p0, p1) of ``rank``.

    Whole ``align``-pattern blocks are dealt out as evenly as possible (block
    counts differ by <= 1) so every shard but the last starts and ends on a
    sweep-block boundary and no rank carries a ragged block in the middle of
    the alignment; the last rank takes the ragged tail.  With fewer blocks
    than ranks the count-balanced split is used instead.
    """
    nblk = -(-P // align)
    if nblk < world:
        base, extra = divmod(P, world)
        p0 = rank * base + min(rank, extra)
        return p0, p0 + base + (1 if rank < extra else 0)
    base, extra = divmod(nblk, world)
    b0 = rank * base + min(rank, extra)
    b1 = b0 + base + (1 if rank < extra else 0)
    return min(P, b0 * align), min(P, b1 * align)


class ShardedLikelihood:
    """The pattern shard of one rank plus the cross-rank reduction.

    ``evaluate(out)`` runs the local shard into ``out`` (a torch tensor of
    shape [n_draws, outlen] on this rank's device) and all-reduces it in
    place.  ``site_ll`` stays sharded (gathered only for parity checks).
    """

    def __init__(self, tipcodes, weights, peel0, rooted, model, C, rank, world, device=0,
                 max_draws=1, engine_factory=None, compact=False):
        self.rank, self.world = rank, world
        P = np.asarray(tipcodes).shape[1]
        self.p0, self.p1 = shard_range(P, rank, world)
        if self.p1 <= self.p0:
            raise ValueError("more ranks than patterns")
        if engine_factory is None:
            import torch  # noqa: F401 -- torch's HIP runtime loads before the engine's
            from .engine import TreeLikelihood
            engine_factory = TreeLikelihood
        self.engine = engine_factory(np.ascontiguousarray(np.asarray(tipcodes)[:, self.p0:self.p1]),
                                     np.ascontiguousarray(np.asarray(weights)[self.p0:self.p1]),
                                     peel0, rooted, model, C, max_draws=max_draws, device=device)
        if compact:
            self.engine.set_output(compact=True)
        self._side = {}  # per device: the side stream that fences a null-stream caller

    @property
    def outlen(self):
        return self.engine.outlen

    def evaluate(self, blens, model, out, site_ll=None, stream=None, group=None):
        """blens [n, B], model [n, 10+2C], out [n, outlen]: device tensors.

        The sweep is ordered on torch's current stream of ``out``'s device
        (or on ``stream``, a hipStream_t handle), the stream the collective
        orders itself against, so the reduction reads ``out`` only after the
        kernels wrote it and the kernels read blens / model only after torch
        produced them.  torch's default stream is the null stream (handle 0),
        which the C boundary fences itself (include/phylo_hip.h
        phy_eval_device); the side stream here, fenced both ways with events,
        keeps that ordering explicit on torch's side as well.
        """
        import torch
        import torch.distributed as dist
        n = blens.shape[0]
        args = (blens.data_ptr(), model.data_ptr(), out.data_ptr(),
                site_ll.data_ptr() if site_ll is not None else 0)
        if stream is None and out.is_cuda:
            stream = torch.cuda.current_stream(out.device).cuda_stream
        if out.is_cuda and not stream:
            cur = torch.cuda.current_stream(out.device)
            side = self._side.get(out.device)
            if side is None:
                side = self._side[out.device] = torch.cuda.Stream(device=out.device)
            side.wait_stream(cur)
            self.engine.evaluate_device(*args, n_draws=n, stream=side.cuda_stream)
            for t in (blens, model, out) + ((site_ll,) if site_ll is not None else ()):
                t.record_stream(side)  # the caching allocator must not reuse them before the side stream is done
            cur.wait_stream(side)
        else:
            self.engine.evaluate_device(*args, n_draws=n, stream=stream)
        if self.world > 1:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        return out
