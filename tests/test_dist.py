"""Multi-rank sharding of the independent checker, world_size 2 on gloo
(CPU). The per-rank checker here is the oracle; on GPUs it is libjh on each
rank's device and the all-reduce runs on RCCL (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from jepsen_amd import _abi as A


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jepsen_amd import shard, synth
        from oracle import oracle
        cols, _ = synth.cas_register(n_keys=240, ops_per_key=80, p_invalid=0.1, seed=9)

        def check_fn(sub, init, budget):
            return oracle.check_cas_independent(sub)

        mine, v, g = shard.check_cas_independent_sharded(cols, rank, world, check_fn)
        load = int(shard.key_costs(cols)[mine].sum())      # this rank's share of the window-sum cost
        q.put((rank, mine.tolist(), v.tolist(), g, load))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_equals_single(built, world):
    from jepsen_amd import shard, synth
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cols, _ = synth.cas_register(n_keys=240, ops_per_key=80, p_invalid=0.1, seed=9)
    full, s = oracle.check_cas_independent(cols)
    seen = set()
    costs = shard.key_costs(cols)
    loads = [r[4] for r in res]
    # LPT on the window-sum estimate: the ranks' loads differ by at most one key's cost
    assert sum(loads) == int(costs.sum()) and max(loads) - min(loads) <= int(costs.max())
    for rank, mine, v, g, _ in res:
        v = np.array([tuple(x) for x in v], dtype=A.VERDICT_DTYPE)
        for i, k in enumerate(mine):
            assert tuple(v[i]) == tuple(full[k]), (rank, k)
            seen.add(k)
        # every rank sees the same global summary, equal to the unsharded one
        assert g["valid"] == s.valid and g["n_invalid"] == s.n_invalid
        assert g["n_unknown"] == s.n_unknown and g["n_keys"] == s.n_keys
        assert g["explored"] == s.explored and g["first_fail_entry"] == s.first_fail_entry
    assert seen == set(range(cols.n_keys))


def test_lpt_balances():
    from jepsen_amd import shard
    costs = np.array([9, 8, 7, 6, 5, 4, 3, 2, 1, 1], np.int64)
    owner = shard.assign_keys(costs, 3)
    loads = np.bincount(owner, weights=costs, minlength=3)
    assert loads.max() - loads.min() <= 2


def _worker2(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jepsen_amd import shard, synth
        from oracle import oracle
        cols, _ = synth.cas_register(n_keys=240, ops_per_key=120, p_invalid=0.1, p_info=0.05, seed=19)

        def check_fn(sub, init, budget, stage):
            # the oracle in libjh's two-stage contract: stage 1 hands keys past
            # the quick budget back deferred, stage 2 decides everything
            v, s = oracle.check_cas_independent(sub)
            if stage == 1:
                v = v.copy()
                d = v["explored"] > 300
                v["valid"][d] = A.UNKNOWN
                v["cause"][d] = A.CAUSE_DEFERRED
                v["explored"][d] = 0
                v["fail_entry"][d] = -1
            return v, s

        keys, v, g, st = shard.check_cas_independent_two_stage(cols, rank, world, check_fn)
        q.put((rank, keys.tolist(), v.tolist(), g, st))
    finally:
        dist.destroy_process_group()


def test_two_stage_pool(built):
    """VERDICT r2 item 4, the torchrun path: phase 1 on each rank's share, the
    deferred keys of both ranks pooled (all_gather_object) and pulled in
    batches through the rendezvous store's atomic counter. Every key is
    decided exactly once, equal to the unsharded check, the pool is split
    between the ranks, and both see the same summary."""
    from jepsen_amd import synth
    from oracle import oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker2, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cols, _ = synth.cas_register(n_keys=240, ops_per_key=120, p_invalid=0.1, p_info=0.05, seed=19)
    full, s = oracle.check_cas_independent(cols)
    seen = []
    for rank, keys, v, g, st in res:
        v = np.array([tuple(x) for x in v], dtype=A.VERDICT_DTYPE)
        for i, k in enumerate(keys):
            assert tuple(v[i]) == tuple(full[k]), (rank, k)
        seen += keys
        assert g["valid"] == s.valid and g["n_invalid"] == s.n_invalid and g["n_keys"] == s.n_keys
        assert g["explored"] == s.explored and g["first_fail_entry"] == s.first_fail_entry
    assert sorted(seen) == list(range(cols.n_keys))
    pool = res[0][4]["pool"]
    assert pool > 10 and res[0][4]["pool"] == res[1][4]["pool"]
    assert res[0][4]["pulled"] + res[1][4]["pulled"] == pool
    assert min(res[0][4]["pulled"], res[1][4]["pulled"]) > 0


def _worker3(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jepsen_amd import history as H
        from jepsen_amd import shard, synth
        from oracle import oracle
        # weak scaling as bench.py runs it: each rank its own history
        cols, _ = synth.cas_register(n_keys=160, ops_per_key=120, p_invalid=0.1, p_info=0.05, seed=31 + rank)
        dcols = {c: torch.from_numpy(getattr(cols, c).copy()) for c in shard.COLS}
        kr = shard.KeyRows(cols.key, cols.n_keys)

        def stage1():
            # libjh's JH_LIN_PHASE1_ONLY contract: keys past the quick budget
            # come back deferred with their progress as `explored`
            v, _ = oracle.check_cas_independent(cols)
            v = v.copy()
            d = v["explored"] > 300
            v["valid"][d] = A.UNKNOWN
            v["cause"][d] = A.CAUSE_DEFERRED
            v["explored"][d] = 1000 - (v["explored"][d] % 997)
            v["fail_entry"][d] = -1
            return v

        got = []

        def stage2(sub, m):
            c = H.Columns(n=int(sub["key"].numel()), n_keys=m, aux=np.zeros(1, np.int64),
                          **{k: sub[k].numpy().copy() for k in shard.COLS})
            v, _ = oracle.check_cas_independent(c)
            got.append(int(c.n))
            return v

        home = {}
        g, st = shard.two_stage_resident(rank, world, dcols, kr, stage1, stage2, home=home)
        # the pooled verdicts back on their home rank equal the history checked whole
        want, _ = oracle.check_cas_independent(cols)
        st["home_equal"] = all(bool((home["verdicts"][f] == want[f]).all()) for f in A.VERDICT_FIELDS)
        q.put((rank, g, st))
    finally:
        dist.destroy_process_group()


def test_two_stage_resident_pool(built):
    """bench.py --gpus N's own path (shard.two_stage_resident), world 2 over
    gloo: phase 1 on each rank's own history, the deferred keys' rows
    exchanged with all_gather, the pool ordered by phase-1 progress and dealt
    round-robin, one stage-2 call per rank. The all-reduced summary equals
    the two histories checked whole, and both ranks take a share."""
    from jepsen_amd import synth
    from oracle import oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker3, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {"valid": 0, "n_invalid": 0, "n_unknown": 0, "n_keys": 0, "explored": 0}
    ffs = []
    for r in range(world):
        cols, _ = synth.cas_register(n_keys=160, ops_per_key=120, p_invalid=0.1, p_info=0.05, seed=31 + r)
        _, s = oracle.check_cas_independent(cols)
        want["valid"] = max(want["valid"], s.valid)
        for f in ("n_invalid", "n_unknown", "n_keys", "explored"):
            want[f] += getattr(s, f)
        if s.first_fail_entry >= 0:
            ffs.append(s.first_fail_entry)
    for rank, g, st in res:
        for f, x in want.items():
            assert g[f] == x, (rank, f, g[f], x)
        assert g["first_fail_entry"] == (min(ffs) if ffs else -1)
        assert st["pool"] > 4 and st["checked_here"] >= st["pool"] // 2
        assert st["home_equal"], rank
    assert sum(st["checked_here"] for _, _, st in res) == res[0][2]["pool"]
