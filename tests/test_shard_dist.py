"""N>1 path on CPU: world_size-2 `gloo` process group, host-side sharding with
no data-path collective, MAX-over-ranks timing (bench.py).
Each rank verifies its own shard of the golden tokens (the CPU oracle stands in
for the rank's GPU here); the gathered verdicts must equal the unsharded run."""
import os
import socket

import numpy as np
import pytest

from cap_amd import shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_bounds_cover_and_balance():
    rng = np.random.default_rng(3)
    algs = list(shard.ALG_COST)
    for world in (1, 2, 3, 4, 8):
        costs = [shard.ALG_COST[algs[i]] for i in rng.integers(0, len(algs), 5000)]
        b = shard.shard_bounds(costs, world)
        assert b[0] == 0 and b[-1] == len(costs) and all(x <= y for x, y in zip(b, b[1:]))
        tot = sum(costs)
        for r in range(world):
            part = sum(costs[b[r]:b[r + 1]])
            assert abs(part - tot / world) <= 2 * max(costs)
    assert shard.shard_bounds(10, 4) == [0, 2, 5, 7, 10]
    assert shard.shard_bounds([], 2) == [0, 0, 0]


def test_cost_table_matches_the_runtime():
    """cap_amd/shard.py CLASS_COST == jg_runtime.cpp CLS_COST (class order)"""
    import re
    src = open(os.path.join(ROOT, "cap_amd", "csrc", "jg_runtime.cpp")).read()
    m = re.search(r"CLS_COST\[NCLS\]\s*=\s*\{([^}]*)\}", src)
    vals = [float(x) for x in m.group(1).split(",")]
    order = ["reject", "rsa2048", "rsa3072", "rsa4096", "p256", "p384", "p521", "ed25519"]
    assert vals == [shard.CLASS_COST[c] for c in order]
    assert shard.token_cost("RS256", 8192) == shard.CLASS_COST["rsa4096"] * 4
    assert shard.token_cost("PS512", 16384) == shard.CLASS_COST["rsa4096"] * 16


def test_sorted_eddsa_es384_batch_splits_into_equal_time():
    """BASELINE configs[3]: a 50/50 EdDSA / ES384 batch sorted by alg (the
    worst case for a count split: all ES384 in the back half) is cut so every
    rank gets the same predicted device time, not the same token count."""
    n = 100000
    algs = ["EdDSA"] * (n // 2) + ["ES384"] * (n // 2)
    costs = [shard.token_cost(a) for a in algs]
    for world in (2, 4, 8):
        b = shard.shard_bounds(costs, world)
        t = [sum(costs[b[r]:b[r + 1]]) for r in range(world)]
        assert max(t) - min(t) <= 2 * max(costs), (world, t)
        assert b[1] > n // world          # the cheap EdDSA front gets more tokens than n / world


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import json
    import torch
    import torch.distributed as td
    from cap_amd import shard as S
    from oracle import jws
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    toks = json.load(open(os.path.join(ROOT, "tests", "golden", "tokens.json")))
    keys = {k["kid"]: jws.Key.from_fixture(k) for k in json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))}
    costs = [S.ALG_COST.get(t["alg"], 1.0) for t in toks]
    lo, hi = S.shard_range(costs, world, rank)
    verdicts = []
    for t in toks[lo:hi]:
        p = jws.parse_jws(t["token"])
        verdicts.append(int(jws.verify_sig(p, keys[t["key"]])) if p else 0)
    # results come back to the host by index: gather (lo, hi, verdicts) -- reporting, not the data path
    got = [None] * world
    td.all_gather_object(got, (lo, hi, verdicts))
    mx = S.max_over_ranks(float(rank) + 1.5)
    if rank == 0:
        q.put((got, mx))
    td.barrier()
    td.destroy_process_group()


def test_two_rank_gloo_sharded_verify(golden):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, mx = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mx == 2.5
    (lo0, hi0, v0), (lo1, hi1, v1) = got
    assert lo0 == 0 and hi0 == lo1 and hi1 == len(golden["tokens"])
    assert v0 + v1 == [t["verdict"] for t in golden["tokens"]]
