"""Benchmark: independent cas-register history verification on MI355X.

Metric (BASELINE.json): history ops verified/sec (node), independent
cas-register, 10k keys x 1k ops per GPU (config C3), 1/2/4/8 GPUs.

A "step" = one full jh_check_cas_independent_device call on a history that
is already resident in HBM: split by key, complete, per-key op/window
tables, WGL search for every key, verdict summary, then (N > 1) the RCCL
all-reduce of the verdict summary across ranks. Each rank checks its own
10k-key shard (keys are independent: weak scaling, no data-path collective).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: 8 TB/s HBM3E (spec)
BYTES_PER_ENTRY = 56           # 7 x int64 columns read once (the whole step)
BYTES_PER_PROBE = 16           # one memo entry {mask, t|state|gen}
# Round 6: a search phase reads the compact per-key
# tables the table pass built, not the history's columns -- ops {rq, fa} and
# layers {rq, hi}, at most 8 B per entry plus 32 B per key
# -- and phase 2 also the resume records of the searches it continues. Those
# are the bytes each phase's roofline charges; 56 B per entry is the whole
# step's (roofline.step).
BYTES_PER_TABLE_ENTRY = 8
BYTES_PER_KEY_TABLE = 32
# HBM bytes per launch of a kernel from the rocprofv3 FETCH_SIZE and
# WRITE_SIZE passes over the SAME history (tools/gpu_pmc.sh + pmc_traffic.py),
# one file per (workload, seed, kernel) under profiles/r05/: PMC counters
# cannot be read inside a timed run, and a file of another history (another
# workload, seed or rank) is never used. Under --pmc the kernels run one at a
# time (rocprofv3 serializes them), so the search phases take another
# schedule than the timed run's (e.g. no late helpers beside phase 2): the
# file's ratio is traffic over the algorithmic bytes of that serialized run,
# and the line also scales the measured bytes per memo probe to the timed
# run's probe count.
TRAFFIC_DIR = os.path.join(ROOT, "profiles", "r06")


def traffic_name(workload, seed, kernel):
    k = "".join(c if c.isalnum() else "_" for c in kernel).strip("_")
    return f"traffic_{workload}_s{seed}_{k}.json"


def pmc_traffic(workload, seed, kernel):
    path = os.path.join(TRAFFIC_DIR, traffic_name(workload, seed, kernel))
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d, os.path.relpath(path, ROOT)
    except (OSError, ValueError, KeyError):
        return None, None


# the search phases a bench line reports a roofline for: (summary field of
# the time, of the memo probes, of the entries of the keys searched, of the
# number of keys searched, kernel). The default schedule's kernels; the
# phase-2 LEAN and WIDE roles share the k_lin_seq_lw grid but keep their own
# timers (the WIDE waves' span, ABI 4). Round 5: that grid's LEAN memo is a
# template argument -- MemoCfg<10, 17> with LEAN keys alone, MemoCfg<10, 15>
# beside WIDE ones (phase_kernel names the instance rocprof shows).
PHASES = {
    "phase1": ("dfs_ms", "memo_probes", None, None, "k_lin_dfs<true, false>"),
    "phase2_lean": ("seq_ms", "seq_probes", "lean_entries", "n_lean_deferred", "k_lin_seq_lw<false, MemoCfg<10, 17>>"),
    "phase3_lean": ("p3_ms", "p3_probes", "p3_entries", "n_phase3", "k_lin_seq3<true>"),
    "wide": ("wide_ms", "wide_probes", "wide_entries", "n_deferred_wide", "k_lin_seq_lw<false, MemoCfg<10, 15>>"),
    "xw": ("xw_ms", "xw_probes", "xw_entries", "n_xw", "k_lin_xw"),
}


def phase_kernel(name, kern, sums):
    # a phase-2 LEAN role beside WIDE keys runs the MemoCfg<10, 15> instance
    if name == "phase2_lean" and float(np.mean([x["n_deferred_wide"] for x in sums])) > 0:
        return PHASES["wide"][4]
    return kern


def _field(x, f):
    if f == "n_lean_deferred":
        return x["n_deferred"] - x["n_deferred_wide"]
    return x[f]


def phase_alg_bytes(name, d, n_entries):
    """Algorithmic bytes of one search phase in one call (jh_summary fields in
    d): the compact tables of the keys it searches (8 B per entry + 32 B per
    key), 16 B per HBM memo probe, and for phase 2 the resume records it
    reads (round 6: not the 56 B per entry of the columns, which the table
    pass read once)."""
    tf, pf, ef, kf, kern = PHASES[name]
    ent = n_entries if ef is None else d[ef]
    keys = d["n_keys"] if kf is None else _field(d, kf)
    b = BYTES_PER_TABLE_ENTRY * ent + BYTES_PER_KEY_TABLE * keys + BYTES_PER_PROBE * d[pf]
    if name == "phase2_lean":
        b += d.get("resume_bytes", 0)
    return float(b)


def phase_rooflines(sums, n_entries):
    """Per search phase, from jh_summary's per-phase times and probe
    counters: algorithmic bytes (phase_alg_bytes) over the phase's HIP-event
    time in the timed run. A phase that searched no key is not a phase of
    this line (its launch may still have run empty): skipped."""
    out = {}
    for name, (tf, pf, ef, kf, kern) in PHASES.items():
        ms = float(np.mean([x[tf] for x in sums]))
        keys = float(np.mean([_field(x, kf) for x in sums])) if kf else float(np.mean([x["n_keys"] for x in sums]))
        if ms <= 0 or keys <= 0:
            continue
        probes = float(np.mean([x[pf] for x in sums]))
        ent = float(n_entries if ef is None else np.mean([x[ef] for x in sums]))
        alg = float(np.mean([phase_alg_bytes(name, x, n_entries) for x in sums]))
        ach = alg / (ms / 1e3) / 1e9
        out[name] = {"kernel": phase_kernel(name, kern, sums), "ms": ms, "alg_bytes": alg, "probes": probes, "entries": ent,
                     "keys": keys, "achieved": ach, "frac": ach / PEAK_HBM_GBS}
    return out


# SURVEY.md 8(d) configurations. Each rank checks its own shard (weak scaling).
WORKLOADS = {
    "c3": dict(desc="C3: independent cas-register, 10000 keys x ~1k entries per GPU", keys=10000,
               seed=3, cpu_keys=10000, cpu_keys_opt=10000,
               # round 5: C4's budget (SURVEY A.6 makes it this project's; no C3 key is
               # :unknown at 2^20 or 2^22). At 2^22 the reachable-set engine settles the
               # valid keys of 1.17 M reachable configurations (ranks 4 / 6) without the
               # count pass
               budget=1 << 22,
               gen=dict(threads_per_key=10, readers=5, n_values=5, process_limit=20, groups=10,
                        init_nil=True, p_info=0.02, p_invalid=0.01, nemesis_every=10000)),
    # round 6: the north_star's own configuration -- ONE
    # 10k-key history (C3's rank-0 history, seed 3) split by key over the N
    # GPUs (jh_key_costs + LPT, shard.assign_keys): strong scaling. --shard r/N
    # rehearses rank r's shard on one GPU
    "c3s": dict(desc="C3 strong: ONE independent cas-register history of 10000 keys x ~1k entries (seed 3) "
                     "split by key over the N GPUs with the window-sum cost model + LPT (jepsen_amd/shard.py)",
                keys=10000, seed=3, cpu_keys=10000, cpu_keys_opt=10000, global_history=True, strong=True,
                budget=1 << 22,
                gen=dict(threads_per_key=10, readers=5, n_values=5, process_limit=20, groups=10,
                         init_nil=True, p_info=0.02, p_invalid=0.01, nemesis_every=10000)),
    "c4": dict(desc="C4: independent cas-register, ONE history of 125000 x N keys (1M at N=8) generated "
                    "identically on every rank and split by key over the N GPUs with the window-sum cost "
                    "model + LPT (jepsen_amd/shard.py); each GPU checks its shard", keys=125000, seed=4,
               cpu_keys=3000, cpu_keys_opt=125000, global_history=True,
               # the budget is raised until every C1-C4 key resolves;
               # at 2^20 two or three keys of a shard stay :unknown (their WGL
               # caches hold 1.66 M / 1.72 M configurations; oracle and device agree)
               budget=1 << 22,
               gen=dict(threads_per_key=10, readers=5, n_values=5, process_limit=20, groups=10,
                        init_nil=True, p_info=0.02, p_invalid=0.01, nemesis_every=10000)),
    "c5": dict(desc="C5: independent cas-register, 1000 keys x ~1k entries, 50 threads per key, "
                    "p_info 0.2 (deep searches, HBM memo stress)", keys=1000, seed=5, cpu_keys=48, cpu_keys_opt=64,
               gen=dict(threads_per_key=50, readers=25, n_values=5, process_limit=100, groups=10,
                        init_nil=True, p_info=0.2, p_invalid=0.01, nemesis_every=10000)),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3",
                    help="c3 (default, BASELINE.json's metric): 10k keys per GPU; c4: a 125k-key "
                         "shard of the 1M-key history (1/8 per GPU); c5: 50 threads per key, many :info")
    ap.add_argument("--keys", type=int, default=None)
    ap.add_argument("--budget", type=int, default=None, help="insert budget per key (default per workload)")
    ap.add_argument("--ops-per-key", type=int, default=500)
    ap.add_argument("--cpu-sample-keys", type=int, default=None,
                    help="keys of the rank-0 history timed on the CPU (default per workload)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--e2e", type=int, default=1, help="also time one call from host buffers (PCIe-inclusive)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--seed-rank", type=int, default=None,
                    help="generate the history rank R of a multi-GPU run would check (rehearsal on one GPU)")
    ap.add_argument("--pool", type=int, default=0,
                    help="1: the two-stage pool (phase 1 per rank, deferred keys exchanged over RCCL and "
                         "dealt by estimated work, one stage-2 call per rank; shard.two_stage_resident); "
                         "0 (default since round 5): each rank checks its shard in one call -- the schedule "
                         "that continues deferred searches and hands long ones over, which the pool's "
                         "stage 2 (keys restarted on another rank) cannot")
    ap.add_argument("--shard", default=None, metavar="R/N",
                    help="one GPU rehearses rank R of an N-rank split of a global-history workload "
                         "(c3s, c4): the same history, cost model and LPT split, R's shard only")
    ap.add_argument("--opt", action="append", default=[], metavar="FIELD=INT",
                    help="a jh_lin_opts tuning field for A/B runs (e.g. handover_min=2048); "
                         "recorded in config.opts")
    a = ap.parse_args()
    a.tune = {k: int(v) for k, v in (o.split("=", 1) for o in a.opt)}
    a.shard_rn = tuple(int(x) for x in a.shard.split("/")) if a.shard else None
    return a


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    # JH_BENCH_REHEARSE=1: every rank on cuda:0 over gloo, to rehearse the
    # N-rank launch, barrier / max-over-ranks timing and the report on a
    # one-GPU box (RCCL refuses two ranks on one device); never a bench number
    rehearse = world > 1 and os.environ.get("JH_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    # JH_BENCH_DIST1=1 (under torchrun --nproc-per-node 1): the N > 1 code path
    # -- RCCL process group, the two-stage pool's all_gathers, the verdict
    # all-reduce -- on a one-rank communicator, the only RCCL run one GPU allows
    dist1 = world == 1 and os.environ.get("JH_BENCH_DIST1") == "1"
    if world > 1 or dist1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from jepsen_amd import _abi as A
    from jepsen_amd import _native, synth

    # ---- workload: this rank's shard of the C3 configuration -------------
    wl = WORKLOADS[args.workload]
    n_keys = args.keys or wl["keys"]
    budget = args.budget or wl.get("budget", A.DEFAULT_BUDGET)
    shard_info = None
    if wl.get("global_history"):
        # C4: one global history (every rank generates the same one, 16 host
        # threads), weighed by jh_key_costs, dealt out by LPT; this rank keeps
        # its keys' rows plus the un-keyed rows (shard.shard_history)
        from jepsen_amd import shard
        # the split this process takes: its own rank of the launch, or (--shard
        # R/N on one GPU) rank R of an N-rank split
        s_rank, s_world = (rank, world) if args.shard_rn is None else args.shard_rn
        if args.shard_rn is not None and (world != 1 or not 0 <= s_rank < s_world):
            raise SystemExit("--shard R/N: one process, 0 <= R < N")
        t_g = time.perf_counter()
        total_keys = n_keys if wl.get("strong") else n_keys * s_world
        # c3s: C3's own rank-0 history (one generator thread, as the c3 line's),
        # so its N = 1 case is the default line's history
        gcols, _ = synth.cas_register(n_keys=total_keys, ops_per_key=args.ops_per_key, seed=wl["seed"],
                                      parts=1 if wl.get("strong") else 16, **wl["gen"])
        t_s = time.perf_counter()
        costs = shard.key_costs(gcols)
        owner = shard.assign_keys(costs, s_world)
        cols, mine, _rows = shard.shard_history(gcols, owner, s_rank)
        loads = np.bincount(owner, weights=costs, minlength=s_world)
        shard_info = {"global_keys": int(gcols.n_keys), "global_entries": int(gcols.n),
                      "rank": s_rank, "world": s_world, "rehearsed": args.shard_rn is not None,
                      "shard_keys": int(len(mine)), "shard_entries": int(cols.n),
                      "generate_s": t_s - t_g, "cost_and_split_s": time.perf_counter() - t_s,
                      "cost_model": "entries + window sum (jh_key_costs), LPT",
                      "max_over_mean_load": float(loads.max() / max(loads.mean(), 1.0))}
        del gcols, _rows
    else:
        seed = wl["seed"] + 7919 * (rank if args.seed_rank is None else args.seed_rank)
        cols, truth = synth.cas_register(n_keys=n_keys, ops_per_key=args.ops_per_key, seed=seed, **wl["gen"])
    n_entries = int(cols.n)
    names = ["process", "type", "f", "key", "value", "value2"]
    dcols = {k: torch.from_numpy(getattr(cols, k)).to(dev) for k in names}

    class DCols:
        n = n_entries
        n_keys = cols.n_keys
        process = dcols["process"].data_ptr()
        type = dcols["type"].data_ptr()
        f = dcols["f"].data_ptr()
        key = dcols["key"].data_ptr()
        value = dcols["value"].data_ptr()
        value2 = dcols["value2"].data_ptr()
        aux = 0
        n_aux = 0

    verd = torch.empty(cols.n_keys * A.VERDICT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    ctx = _native.Context(local)
    torch.cuda.synchronize()

    red_max = torch.zeros(2, dtype=torch.int64, device=dev)
    red_sum = torch.zeros(4, dtype=torch.int64, device=dev)
    use_pool = dist is not None and args.pool
    pool_stats = []
    pool_home = {}          # this rank's keys' pooled verdicts (the measured ones), for the parity check
    if use_pool:
        from jepsen_amd import shard as _shard
        key_rows = _shard.KeyRows(cols.key, cols.n_keys)
        tune = dict(args.tune)
        flags0 = tune.pop("flags", 0)

        def _dev_view(t, n, k):
            class V:
                pass
            v = V()
            v.n, v.n_keys, v.aux, v.n_aux = n, k, 0, 0
            for c in _shard.COLS:
                setattr(v, c, t[c].data_ptr())
            return v

        def step_pool():
            got = {}

            def stage1():
                got[1] = ctx.check_cas_independent_device(DCols, verd.data_ptr(), budget=budget,
                                                          flags=flags0 | A.LIN_PHASE1_ONLY, exact_count=False, **tune)
                return np.frombuffer(verd.cpu().numpy().tobytes(), dtype=A.VERDICT_DTYPE).copy()

            def stage2(sub, m):
                v2 = torch.empty(m * A.VERDICT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
                got[2] = ctx.check_cas_independent_device(_dev_view(sub, int(sub["key"].numel()), m), v2.data_ptr(),
                                                          budget=budget, flags=flags0 | A.LIN_SKIP_PHASE1,
                                                          exact_count=False, **tune)
                return np.frombuffer(v2.cpu().numpy().tobytes(), dtype=A.VERDICT_DTYPE).copy()

            g, st = _shard.two_stage_resident(rank, world, dcols, key_rows, stage1, stage2, device=dev,
                                              home=pool_home)
            pool_stats.append(st)
            # one jh_summary for the report: phase 1 from stage 1, the heavy-key
            # pass from stage 2 (explored / counts are the all-reduced ones)
            s = got.get(2) or got[1]
            if 2 in got:
                for f in ("dfs_ms", "memo_probes"):
                    setattr(s, f, getattr(got[1], f))
                # both stages' device time (the exchange is in the pool stats)
                s.device_ms = got[1].device_ms + got[2].device_ms
            s.valid, s.n_invalid, s.n_unknown = g["valid"], g["n_invalid"], g["n_unknown"]
            s.explored = g["explored"]
            s.first_fail_entry = g["first_fail_entry"]      # all-reduced, in home-rank rows
            return s

    def step():
        if use_pool:
            return step_pool()
        # the checkers' path: no count pass for valid keys the reachable-set
        # engine settles (their map has no :explored); parity below
        s = ctx.check_cas_independent_device(DCols, verd.data_ptr(), budget=budget, exact_count=False, **args.tune)
        if dist is not None:
            # RCCL verdict summary all-reduce over xGMI: merge-valid (MAX),
            # failures/unknown/keys counts (SUM), first failing row (MIN as -MAX)
            ff = s.first_fail_entry if s.first_fail_entry >= 0 else (1 << 62)
            red_max.copy_(torch.tensor([s.valid, -ff], dtype=torch.int64))
            red_sum.copy_(torch.tensor([s.n_invalid, s.n_unknown, s.n_keys, s.explored],
                                       dtype=torch.int64))
            dist.all_reduce(red_max, op=dist.ReduceOp.MAX)
            dist.all_reduce(red_sum, op=dist.ReduceOp.SUM)
            # the line reports the whole job's verdict counts
            mx, sm = red_max.tolist(), red_sum.tolist()
            s.valid, s.n_invalid, s.n_unknown, s.explored = mx[0], sm[0], sm[1], sm[3]
        return s

    for _ in range(args.warmup):
        step()
    dfs_ms, dev_ms, probes, seq_ms, bfs_ms, seq_probes = [], [], [], [], [], []
    sums = []
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s = step()
        dfs_ms.append(s.dfs_ms)
        dev_ms.append(s.device_ms)
        probes.append(s.memo_probes)
        seq_ms.append(s.seq_ms)
        bfs_ms.append(s.bfs_ms)
        seq_probes.append(s.seq_probes)
        sums.append({f: (list(getattr(s, f)) if f == "waves" else getattr(s, f)) for f, _ in A.JhSummary._fields_})
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([n_entries], dtype=torch.int64, device=dev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        total_entries = int(tot.item())
    else:
        total_entries = n_entries
    value = total_entries * args.steps / elapsed

    # ---- rooflines from live HIP events (jh_summary), per search phase -----
    # each phase's kernel has its own events and probe counter (ABI 4); the
    # line's roofline is the dominant (longest) phase's
    dfs_avg = float(np.mean(dfs_ms)) / 1e3
    seq_avg = float(np.mean(seq_ms)) / 1e3
    phases = phase_rooflines(sums, n_entries)
    dom = max(phases, key=lambda k: phases[k]["ms"]) if phases else None
    seed_used = wl["seed"] + 7919 * (rank if args.seed_rank is None else args.seed_rank)
    tr, traffic_src = (pmc_traffic(args.workload, seed_used, phases[dom]["kernel"])
                       if dom and args.keys is None else (None, None))

    # host buffers to host verdicts (H2D copy + check + verdicts D2H), over K
    # calls: the boundary's host-buffer entry point, beside the HBM-resident value
    e2e = None
    if args.e2e:
        # one untimed call first: the context's host-buffer staging (pinned
        # chunk buffers, the packing pool) is made on its first packed call
        ctx.check_cas_independent(cols, budget=budget, exact_count=False)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            ctx.check_cas_independent(cols, budget=budget, exact_count=False)
        e2e_s = (time.perf_counter() - t1) / args.steps
        e2e = {"ms_per_call": e2e_s * 1e3, "entries_per_s_this_rank": n_entries / e2e_s,
               "calls": args.steps}

    out = None
    if rank == 0:
        parity = parity_detail = None
        if not args.no_parity:
            from oracle import oracle
            # the verdicts of the last timed step: rank 0's keys as the pool left
            # them on their home rank (shard.two_stage_resident), or the call's own
            timed = (pool_home["verdicts"] if use_pool else
                     np.frombuffer(verd.cpu().numpy().tobytes(), dtype=A.VERDICT_DTYPE).copy())
            ov, os_ = oracle.check_cas_independent(cols, budget=budget, threads=min(16, len(os.sched_getaffinity(0))))
            unc = timed["explored"] == A.EXPLORED_UNCOUNTED
            # every field of every key; explored wherever counted (an uncounted
            # key must be valid: JH_LIN_EXACT_COUNT's contract)
            timed_ok = bool(all((timed[f] == ov[f]).all() for f in A.VERDICT_FIELDS if f != "explored") and
                            (timed["explored"][~unc] == ov["explored"][~unc]).all() and
                            (ov["valid"][unc] == A.VALID).all())
            # and one more call with WGL's exact count for every key: every field
            ctx.check_cas_independent_device(DCols, verd.data_ptr(), budget=budget, exact_count=True, **args.tune)
            hv = np.frombuffer(verd.cpu().numpy().tobytes(), dtype=A.VERDICT_DTYPE)
            exact_ok = bool(all((hv[f] == ov[f]).all() for f in A.VERDICT_FIELDS))
            parity = timed_ok and exact_ok
            parity_detail = {"timed_verdicts": timed_ok, "exact_count_call": exact_ok,
                             "uncounted_valid_keys": int(unc.sum()),
                             "source": "the last timed step's per-key verdicts" +
                                       (" (pooled: gathered back to rank 0)" if use_pool else "")}
        cpu = cpu_faithful = None
        if not args.no_cpu and world == 1:
            cpu = cpu_baseline(cols, args.cpu_sample_keys or wl["cpu_keys_opt"], args.workload.upper(), mode=0, budget=budget)
            cpu_faithful = cpu_baseline(cols, args.cpu_sample_keys or wl["cpu_keys"], args.workload.upper(), mode=3, budget=budget)
        out = {
            "metric": "history ops verified/sec (node), independent cas-register 10k keys, 1/2/4/8 GPU",
            "value": value,
            "unit": "entries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if wl.get("strong") else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded jepsen-shaped histories, jepsen_amd/csrc/gen.cpp)",
            "config": {"workload": wl["desc"],
                       "keys_per_gpu": int(cols.n_keys), "entries_per_gpu": n_entries,
                       "threads_per_key": wl["gen"]["threads_per_key"],
                       "process_limit": wl["gen"]["process_limit"], "p_info": wl["gen"]["p_info"],
                       "p_invalid": wl["gen"]["p_invalid"], "budget": budget,
                       "explored_per_step": int(s.explored), "invalid_keys": int(s.n_invalid),
                       "unknown_keys": int(s.n_unknown), "device_ms": float(np.mean(dev_ms)),
                       "deferred_keys": int(s.n_deferred), "deferred_entries": int(s.deferred_entries),
                       "phase1_ms": dfs_avg * 1e3, "phase2_seq_ms": seq_avg * 1e3,
                       "phase2_bfs_ms": float(np.mean(bfs_ms)),
                       # ABI 5: heavy keys started while phase 1 ran (the streaming pass), when
                       "streamed": bool(s.streamed), "phase2_start_ms": float(np.mean([x["p2_start_ms"] for x in sums])),
                       "phase1_span_ms": float(np.mean([x["p1_span_ms"] for x in sums])),
                       # round 5: deferred searches continued from phase 1's state
                       "resumed_keys": int(s.resumed), "resume_bytes": int(s.resume_bytes),
                       # round 6: speculative dead-subtree enumerations by idle late helpers
                       "spec": {"jobs": int(s.spec_jobs), "dead": int(s.spec_dead), "merges": int(s.spec_merges),
                                "merged_nodes": int(s.spec_nodes), "takeovers": int(s.takeovers)},
                       "phases": phase_table(sums), "opts": args.tune or None},
            "shard": shard_info,
            "pool": ({"mode": "two-stage (shard.two_stage_resident): phase 1 per rank, deferred keys' rows "
                              "all-gathered over RCCL, dealt round-robin most estimated phase-1 work first, one "
                              "stage-2 call per rank", "rank0_last_step": pool_stats[-1]}
                     if use_pool and pool_stats else None),
            "value_kind": "history resident in HBM, verdicts left in HBM (kernel pipeline only); "
                          "host-to-host rate in e2e_host_buffers",
            "e2e_host_buffers": e2e,
            "roofline": ({"bound": "hbm", "phase": dom, "kernel": phases[dom]["kernel"],
                          "achieved": phases[dom]["achieved"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                          "frac": phases[dom]["frac"],
                          # round 6: the kernel time is this timed run's
                          # HIP events around the phase's launch; rocprofv3's average of the
                          # same kernel over a traced run of this command is in profiles/r06/
                          # (the traced run's own line carries the frac that average gives)
                          "time_source": "HIP events around the phase's launch, this timed run",
                          "bytes_model": "8 B per table entry + 32 B per key of the keys the phase searches "
                                         "+ 16 B per HBM memo probe (+ resume records read, phase 2)",
                          "step": {"alg_bytes": BYTES_PER_ENTRY * float(total_entries) / max(1, world),
                                   "achieved": BYTES_PER_ENTRY * total_entries / max(1, world) /
                                               (elapsed / args.steps) / 1e9,
                                   "note": "the whole step: 56 B per entry (7 int64 columns, SURVEY 8(d)) "
                                           "over the step time, per GPU"},
                          # FETCH_SIZE + WRITE_SIZE per launch over this same history (tools/gpu_pmc.sh),
                          # measured in rocprofv3's serialized --pmc schedule
                          "traffic": tr["traffic_bytes"] if tr else None,
                          "traffic_schedule": ("serialized (rocprofv3 --pmc runs one kernel at a time: "
                                               f"that run's phase took {tr['pmc_phase_ms']:.1f} ms, "
                                               f"{tr['pmc_probes']:.0f} memo probes)") if tr else None,
                          "traffic_over_alg_pmc_run": tr.get("traffic_over_alg") if tr else None,
                          # that run's traffic per algorithmic byte, times this run's algorithmic
                          # bytes (its memo writes follow the inserts, not the HBM probes: a
                          # per-probe scaling overstated it ~13x in round 5's first lines)
                          "traffic_scaled_to_timed_alg": (
                              tr["traffic_bytes"] / max(1.0, tr["alg_bytes_same_run"]) * phases[dom]["alg_bytes"])
                          if tr and tr.get("alg_bytes_same_run") else None,
                          "traffic_source": traffic_src,
                          "kernel_ms": phases[dom]["ms"], "alg_bytes": phases[dom]["alg_bytes"],
                          "note": "latency-bound tree search: one wave per key, LDS memo"}
                         if dom else None),
            "roofline_phases": phases,
            "cpu_baseline": cpu,
            "cpu_baseline_faithful": cpu_faithful,
            "parity_vs_oracle": parity,
            "parity_detail": parity_detail,
            "dist_selftest": ("JH_BENCH_DIST1: one-rank RCCL communicator, the N > 1 code path on one GPU"
                              if dist1 else None),
        }
        if rehearse:
            out["rehearsal"] = "JH_BENCH_REHEARSE: every rank on cuda:0 over gloo; not a bench number"
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    return out


def phase_table(sums):
    """Per-phase times, probes, entries and waves of the timed steps (jh_summary,
    ABI 4): each search kernel's own HIP events and probe counter."""
    if not sums:
        return None
    mean = lambda f: float(np.mean([x[f] for x in sums]))
    last = sums[-1]
    return {"phase1": {"ms": mean("dfs_ms"), "probes": mean("memo_probes")},
            "phase2_lean": {"ms": mean("seq_ms"), "probes": mean("seq_probes"), "keys": last["n_deferred"] - last["n_deferred_wide"],
                            "entries": last["lean_entries"], "waves": last["waves"][0], "helper_probes": mean("helper_probes")},
            "phase3_lean": {"ms": mean("p3_ms"), "probes": mean("p3_probes"), "keys": last["n_phase3"],
                            "entries": last["p3_entries"], "waves": last["waves"][2]},
            "bfs": {"ms": mean("bfs_ms")},
            "wide": {"ms": mean("wide_ms"), "probes": mean("wide_probes"), "keys": last["n_deferred_wide"],
                     "entries": last["wide_entries"], "waves": last["waves"][1], "phase3_keys": last["n_phase3_wide"]},
            "xw": {"ms": mean("xw_ms"), "probes": mean("xw_probes"), "keys": last["n_xw"], "entries": last["xw_entries"],
                   "waves": last["waves"][3]}}


def cpu_quota_cores():
    """CPUs this process may actually use: the cgroup v2 CPU quota (cpu.max)
    when there is one -- on the GPU box the affinity mask shows the whole
    machine while the quota is the job's share -- else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            return min(aff, max(1, int(round(int(q) / int(p))))), aff
    except (OSError, ValueError):
        pass
    return aff, aff


def cpu_baseline(cols, sample_keys, name="C3", mode=0, min_s=8.0, budget=None):
    """The CPU oracle on every host core this process may use, over a bounded
    sample of this rank's keys, repeated until min_s of wall time. mode 0 =
    optimized CPU (one O(N) split, canonical WGL); mode 3 =
    reference-faithful (independent.clj:234-245's O(K*N) per-key subhistory
    scan + knossos-style linked-list/BitSet WGL)."""
    from oracle import oracle
    cores, aff = cpu_quota_cores()
    threads = aff                      # one worker per visible CPU; the quota caps their sum
    k1 = min(sample_keys, cols.n_keys)
    reps = 0
    t0 = time.perf_counter()
    while True:
        oracle.check_cas_independent_range(cols, 0, k1, mode=mode, threads=threads,
                                           **({"budget": budget} if budget else {}))
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_s:
            break
    counts = np.bincount(cols.key[cols.key >= 0], minlength=cols.n_keys)
    ent = int(counts[:k1].sum())
    what = ("optimized CPU oracle (one O(N) split + canonical WGL)" if mode == 0 else
            "reference-faithful oracle (O(K*N) subhistory + list WGL)")
    return {"value": ent * reps / dt, "unit": "entries/s", "cores": cores, "kind": "port",
            "threads": threads, "nproc_visible": os.cpu_count(),
            "sample": f"keys 0..{k1 - 1} ({ent} entries) of the rank-0 {name} history, {what}, "
                      f"{reps} pass(es) in {dt:.2f} s, {threads} threads under a {cores}-CPU quota"}


if __name__ == "__main__":
    main()
