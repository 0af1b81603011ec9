"""Multi-GPU partitioning of a token batch: one process per GPU,
host-side sharding, no collective on the data path.

Tokens are independent, so a global batch is cut into contiguous per-rank
ranges weighted by each token's verify cost (the per-class cost model of
jg_verify_batch), every rank verifies its own range on its own
GPU, and the only collective is a MAX over ranks of the elapsed time for
reporting (bench.py).  The same cut is what jg_verify_batch applies across the
devices of one jg_ctx.
"""
import numpy as np

# relative verify cost per token by alg (jg_runtime.cpp cls_cost; RSA by key size)
ALG_COST = {"RS256": 3.6, "PS256": 3.6, "RS384": 8.0, "PS384": 8.0, "RS512": 16.0, "PS512": 16.0,
            "ES256": 1.0, "ES384": 3.6, "ES512": 8.4, "EdDSA": 1.9}


def shard_bounds(costs, world: int):
    """Cut points c[0]=0 <= c[1] <= ... <= c[world]=n so that each rank's
    summed cost is within one token of total/world.  `costs` is a sequence of
    per-token costs (or an int n for unit costs)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    if isinstance(costs, (int, np.integer)):
        n = int(costs)
        return [n * r // world for r in range(world + 1)]
    c = np.asarray(costs, dtype=np.float64)
    pre = np.concatenate([[0.0], np.cumsum(c)])
    targets = pre[-1] * np.arange(1, world) / world
    cuts = np.searchsorted(pre, targets, side="left")
    return [0] + [int(x) for x in cuts] + [len(c)]


def shard_range(costs, world: int, rank: int):
    b = shard_bounds(costs, world)
    return b[rank], b[rank + 1]


def max_over_ranks(value: float, device=None) -> float:
    """MAX all-reduce of a scalar (the bench's elapsed time); identity when
    torch.distributed is not initialised.  gloo on CPU tensors, RCCL on GPU."""
    try:
        import torch
        import torch.distributed as td
    except ImportError:
        return value
    if not (td.is_available() and td.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device or "cpu")
    td.all_reduce(t, op=td.ReduceOp.MAX)
    return float(t.item())
