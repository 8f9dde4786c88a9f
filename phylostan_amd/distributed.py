"""Multi-GPU: one process per GPU, site patterns sharded, one RCCL all-reduce.

SURVEY.md 8e: patterns are independent, so each rank owns a contiguous,
count-balanced range of patterns and evaluates its shard with its own
``phy_ctx``.  Every entry of the per-draw output vector (log-likelihood,
dL/dP, branch / rate / mixture / root-frequency gradients) is a sum over
patterns, so a single ``all_reduce(SUM)`` of that vector -- over RCCL
(``torch.distributed`` backend "nccl" on ROCm) between MI355X GPUs on xGMI --
is the whole exchange: for S = 128, C = 4 it is 1 + 254 + 12 + 16*4*254
doubles = 130 KB per draw, latency-bound on xGMI.

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
                 max_draws=1, engine_factory=None):
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
        which the C boundary reads as "the context's own stream"
        (include/phylo_hip.h phy_eval_device): on it the sweep runs on a side
        stream fenced both ways with events instead.
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
            if getattr(self, "_side", None) is None:
                self._side = torch.cuda.Stream(device=out.device)
            self._side.wait_stream(cur)
            self.engine.evaluate_device(*args, n_draws=n, stream=self._side.cuda_stream)
            cur.wait_stream(self._side)
        else:
            self.engine.evaluate_device(*args, n_draws=n, stream=stream)
        if self.world > 1:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        return out
