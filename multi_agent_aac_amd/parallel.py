"""Multi-GPU data parallelism for the vectorised MADDPG.

Envs are independent, so each rank (one process per GPU) owns E envs, its own OD-bank seed and
its own replay shard: the env step, replay push/sample and the forward/backward never talk to
other ranks.  The only exchange is the mean of the flat gradient buffer of each network before
every Adam step (critic and actor, N times per update_myown): ONE all-reduce of one contiguous
buffer per network (~0.72 MB critic + ~0.26 MB actor at N = 5), over RCCL/xGMI with backend
"nccl" -- latency-bound at this size, so bucketing everything into one flat tensor is the lever.
Parameters start identical on every rank (same init seed) and stay identical because every rank
applies the same averaged gradient.
"""
import os

import torch
import torch.distributed as dist

# the gradient all-reduces of a world > 1 update captured INSIDE the update's HIP graph (RCCL kernels
# are graph nodes, ordered by the graph's edges) instead of issued eagerly between graph segments:
# 6 eager collectives + 7 segment replays cost ~117 us per update on one GPU, one graph with them
# captured ~27 us (tools/seg_overhead.py, profiles/r05_seg_overhead.json).  AAC_GRAPH_COLL=0 keeps
# the segmented replay
GRAPH_COLL = os.environ.get("AAC_GRAPH_COLL", "1") == "1"


def capturable(group=None):
    """Whether the collectives of ``group`` can be captured into a HIP graph: RCCL (backend "nccl")
    enqueues device work; gloo runs on the host and cannot be."""
    return GRAPH_COLL and dist.is_initialized() and dist.get_backend(group) == "nccl"


def allreduce_mean_(t, group=None):
    """In-place mean over the ranks of ``group`` (one collective)."""
    ws = dist.get_world_size(group)
    if ws > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(ws)
    return t


def allreduce_sum_(t, group=None):
    """In-place sum over the ranks of ``group`` (one collective).  The fused learners divide by the
    world size inside the Adam launch that consumes the sum (``gscale``), so the mean costs no
    separate division kernel per collective."""
    if dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def rank_seed(base, rank):
    """Per-rank seed for OD bank / replay sampling / exploration noise (env shards differ)."""
    return int(base) + 1009 * int(rank)


def broadcast_flat_(t, src=0, group=None):
    """Make every rank's flat parameter buffer identical to ``src``'s (e.g. after a reload)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(t, src=src, group=group)
    return t


def init_from_env(backend=None):
    """torch.distributed.run environment -> (world, rank, local_rank, device)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % ndev) if ndev else torch.device("cpu")
    if ws > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if ndev else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(dev)
            dist.init_process_group(backend, device_id=dev)
        else:
            dist.init_process_group(backend)
    elif ndev:
        torch.cuda.set_device(dev)
    return ws, rank, local, dev
