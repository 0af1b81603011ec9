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

# Relative device time per token by kernel class (ES256 = 1), measured on one
# MI355X with every class alone filling the chip (tools/class_costs.py ->
# profiles/r03_class_costs.json).  The same table as jg_runtime.cpp CLS_COST,
# in its class order (reject, rsa2048, rsa3072, rsa4096, p256, p384, p521,
# ed25519); tests/test_shard_dist.py checks they agree.
CLASS_COST = {"reject": 0.01, "rsa2048": 4.2, "rsa3072": 9.0, "rsa4096": 15.5, "p256": 1.0, "p384": 3.4,
              "p521": 6.6, "ed25519": 1.1}


def rsa_class(bits):
    """jg_runtime.cpp build_keys: RSA-2K up to 2070 bits, RSA-3K up to 3134,
    else the RSA-4K+ class (148 / 296 / 592 limbs up to 4142 / 8286 / 16574)."""
    return "rsa2048" if bits <= 2070 else "rsa3072" if bits <= 3134 else "rsa4096"


def token_cost(alg, key_bits=None):
    """Predicted device time of one (alg, key) verification, ES256 = 1.  RSA by
    the key's modulus size (default: the alg's usual 2048 / 3072 / 4096); the
    RSA-4K+ class scales with the square of its layout's limbs."""
    if alg in ("ES256", "ES384", "ES512"):
        return CLASS_COST[{"ES256": "p256", "ES384": "p384", "ES512": "p521"}[alg]]
    if alg == "EdDSA":
        return CLASS_COST["ed25519"]
    if alg[:2] in ("RS", "PS"):
        bits = key_bits or {"256": 2048, "384": 3072, "512": 4096}[alg[2:]]
        cls = rsa_class(bits)
        w = CLASS_COST[cls]
        if cls == "rsa4096":
            limbs = 148 if bits <= 4142 else 296 if bits <= 8286 else 592
            w *= (limbs / 148) ** 2
        return w
    return CLASS_COST["reject"]


# by alg at the usual key sizes (RS/PS256 on 2048-bit keys, 384 on 3072, 512 on 4096)
ALG_COST = {a: token_cost(a) for a in ("RS256", "PS256", "RS384", "PS384", "RS512", "PS512", "ES256", "ES384",
                                       "ES512", "EdDSA")}


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
