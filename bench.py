"""Benchmark: candidate pairs scored/sec on BASELINE.json configs[1] — 1M synthetic person
records deduplicated with two key functions, NAME JaroWinkler + ADDRESS/DOB Levenshtein.

One step = one dk_match over every query record of this rank (blocking-table build,
candidate generation, fused scoring, threshold, match gather to the host), with the index
already resident in HBM.  N>1: one process per GPU (torchrun), replicated index, query
records split into contiguous tiles per rank, match counts all-gathered and match lists
gathered to rank 0 over RCCL inside the step.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "sesam-duke-microservice_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

METRIC = "candidate pairs scored/sec (node) + records/sec deduped, 1/2/4/8 MI355X"
HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md chip-level parameters


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--records", type=int, default=1_000_000)
    ap.add_argument("--dup-frac", type=float, default=0.1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="target CPU time of the oracle baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    return ap.parse_args()


def build_data(n_records, dup_frac):
    from dukehip import synth
    n_dup = int(n_records * dup_frac)
    p = synth.persons(n_records - n_dup, n_dup)
    keys = synth.keys_config2(p)
    return p, keys


def schema():
    from dukehip import _abi as A
    # comparison order = record HashMap order of NAME/ADDRESS/DOB + synthetic properties
    from dukehip.config import java_hashmap_order
    order = [n for n in java_hashmap_order(["NAME", "ADDRESS", "DOB", "ID", "dukeOriginalEntityId",
                                            "dukeDatasetId"]) if n in ("NAME", "ADDRESS", "DOB")]
    spec = {"NAME": (A.CMP_JAROWINKLER, 0.1, 0.95), "ADDRESS": (A.CMP_LEVENSHTEIN, 0.2, 0.8),
            "DOB": (A.CMP_LEVENSHTEIN, 0.1, 0.85)}
    arr = (A.dk_property * 3)()
    for i, name in enumerate(order):
        c, lo, hi = spec[name]
        arr[i] = A.dk_property(c, 2, 0, 0, lo, hi, 0.0)
    s = A.dk_schema(3, arr, 0.9, 0.7, A.MODE_DEDUP, 2)
    s._keep = arr
    return s, order, spec


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import dukehip as dh
    from dukehip import synth

    t0 = time.time()
    p, keys = build_data(args.records, args.dup_frac)
    sch, order, spec = schema()
    cols = [synth.column(p[{"NAME": "name", "ADDRESS": "address", "DOB": "dob"}[n]]) for n in order]
    n = len(p["name"])
    eng = dh.GpuEngine(sch, device=local)
    eng.upsert(n, np.arange(n, dtype=np.uint64), cols,
               key_columns=[synth.column(k) for k in keys])
    t_index = time.time() - t0
    # contiguous query tile of this rank
    q0, q1 = n * rank // world, n * (rank + 1) // world
    queries = np.arange(q0, q1, dtype=np.uint32)

    from dukehip import dist as dshard
    nq_max = dshard.max_tile(n, world)
    holder = {}

    def step():
        old = holder.pop("res", None)
        if old is not None:
            old.close()                       # hand the result memory back to the pool
        if dist is None:
            res = eng.match(queries)          # entries land in pinned host memory
            holder["res"] = res
            return res, res.pairs_scored
        # N>1: entries stay in HBM; RCCL all-gathers the per-rank counts, then gathers
        # every rank's match list (first / candidate / prob / kind) to rank 0 over xGMI,
        # which moves the node's list to the host.
        res = eng.match(queries, on_device=True)

        def fill(first, cand, prob, kind):
            torch.cuda.synchronize()
            res.copy_to_device(first.data_ptr(), cand.data_ptr(), prob.data_ptr(), kind.data_ptr())

        _, total = dshard.gather_matches(dist, torch, dev, len(queries), res.n, res.pairs_scored,
                                         fill, world, rank, nq_max)
        holder["res"] = res
        return res, total

    for _ in range(args.warmup):
        step()
    eng.reset_profile()
    eng.set_profiling(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    total_scored = 0
    last = None
    for _ in range(args.steps):
        last, sc = step()
        total_scored += sc
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t
    eng.set_profiling(False)
    prof = eng.profile()
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms_step = el / args.steps * 1e3
    pairs_step = total_scored / args.steps
    value = pairs_step / (ms_step / 1e3)

    if rank == 0:
        launches = max(1, prof["score_launches"])
        score_s = prof["ms_score"] / 1e3
        achieved = prof["score_bytes"] / score_s if score_s > 0 else 0.0
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_k_score.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "BASELINE configs[1]: 1M synthetic person records dedup, "
                                   "key blocking K1=surname[0:3]+dob[0:4] K2=given[0:2]+dob[5:10]",
                       "records": n, "pairs_per_step": pairs_step,
                       "comparators": {k: ["Levenshtein", "JaroWinkler"][spec[k][0] == 2] for k in order},
                       "threshold": 0.9, "maybe_threshold": 0.7,
                       "parallelism": f"query-tile sharding x{world}, replicated index"},
            "records_per_s": n / (ms_step / 1e3),
            "matches_per_step": int(last.n) if last is not None else 0,
            "index_build_s": t_index,
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK,
                         "traffic": traffic,
                         "kernel": "k_score", "launches": prof["score_launches"],
                         "avg_launch_ms": prof["ms_score"] / launches,
                         "bytes_per_launch": prof["score_bytes"] / launches},
            "phases_ms_per_step": {k: prof[k] / args.steps for k in
                                   ("ms_index", "ms_generate", "ms_score", "ms_gather", "ms_total")},
        }
        if world == 1 and args.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(p, keys, order, spec, last, args)
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(p, keys, order, spec, gpu_res, args):
    """The C oracle (oracle/duke_oracle.c, a restatement of Duke's scoring loop) on a
    bounded sample: the first S query records, full candidate lists, host threads.  The
    same sample's match list is checked against the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    field = {"NAME": "name", "ADDRESS": "address", "DOB": "dob"}
    props = [{"comparator": spec[k][0], "low": spec[k][1], "high": spec[k][2]} for k in order]
    ot = O.OracleTable(props, [p[field[k]] for k in order], keys=keys, threshold=0.9, maybe=0.7)
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    n = ot.n
    probe = min(n, 2000)
    r = ot.match(np.arange(probe, dtype=np.uint32), nthreads=threads)
    rate = r["pairs_scored"] / max(r["ms_score"] / 1e3, 1e-9)
    per_q = r["pairs_scored"] / probe
    s = int(min(n, max(probe, args.cpu_seconds * rate / max(per_q, 1e-9))))
    r = ot.match(np.arange(s, dtype=np.uint32), nthreads=threads)
    e = int(gpu_res.first[s])
    gq = np.repeat(np.arange(s, dtype=np.uint32), np.diff(gpu_res.first[: s + 1]).astype(np.int64))
    ok = (np.array_equal(r["query"], gq) and np.array_equal(r["candidate"], gpu_res.candidate[:e])
          and np.array_equal(r["prob"], gpu_res.prob[:e]) and np.array_equal(r["kind"], gpu_res.kind[:e]))
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    return {"value": r["pairs_scored"] / (r["ms_score"] / 1e3), "unit": "pairs/s", "cores": threads,
            "kind": "port",
            "sample": f"first {s} of {n} query records ({r['pairs_scored']} pairs), "
                      f"scoring loop timed, blocking-index build excluded ({r['ms_index']:.0f} ms)",
            "seconds": r["ms_score"] / 1e3, "cpu_model": cpu, "host_nproc": os.cpu_count(),
            "matches_identical_to_gpu": bool(ok)}


if __name__ == "__main__":
    main()
