"""Benchmark: candidate pairs scored/sec on BASELINE.json's configurations.

Default (the driver's line): configs[1] — 1M synthetic person records deduplicated with two
key functions, NAME JaroWinkler + ADDRESS/DOB Levenshtein.  `--workload` selects the other
GPU configurations for measurement runs (not the headline line):
  linkage   configs[2]: person linkage, QGram DICE/JACCARD names/addresses + Numeric
            BIRTHYEAR/ZIP (min-ratio 0.9), cross-group key blocking (default 1M x 1M; the
            published shape is 10M x 10M over 8 GPUs: --records 10000000)
  allpairs  configs[3]: 200k x 200k unblocked (Duke InMemoryDatabase), one <=16-char a-z
            field, --comparator lev|jw
  longtext  configs[4]: text linkage, 64-256 chars, WeightedLevenshtein + QGram q=3
            JACCARD, key = first two tokens (default 200k x 200k; published 5M x 5M)
  reference configs[0]: the reference's own pipeline (testdukeconfig.xml, parsed into
            tests/golden/testdukeconfig_schema.json) over 2 x 10,000 stress-test entities,
            with its own Lucene candidate semantics (no key functions) on the GPU

One step = one dk_match over every query record of this rank (candidate generation, fused
scoring, threshold and the device-side compaction of the match list), with the index
already resident in HBM (its blocking tables are built by the first match after the
upsert, in the warmup) and the match list left in HBM: `value` is that rate.  The boundary
hands the MatchListener its list in host memory, so the same step with the list copied to
pinned host memory is timed after it and reported as `pcie_inclusive` (never `value`).
N>1: one process per GPU -- started by torch.distributed.run, or by this script itself when
`--gpus N` is given without a launcher (WORLD_SIZE unset) -- replicated index, query records
split into contiguous cost-weighted tiles per rank.  The result gather is inside the timed
step: by default (--gather shm) every GPU copies its tile's list into its slice
of one shared host mapping over its own host link, overlapped with scoring, and the per-rank
counts are all-gathered over RCCL, after which rank 0 holds the node list; --gather rccl
gathers the lists to GPU 0 over xGMI, --gather none leaves them in each rank's HBM.
Rank 0 prints one JSON line.
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
VALU_PEAK = 1024 * 2.4e9 / 2  # wave64 VALU instructions/s: 256 CUs x 4 SIMD-32, 2 cycles each
DEFAULT_RECORDS = {"dedup": 1_000_000, "linkage": 1_000_000, "allpairs": 200_000, "longtext": 200_000,
                   "reference": 20_000}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="dedup", choices=sorted(DEFAULT_RECORDS))
    ap.add_argument("--records", type=int, default=None,
                    help="dedup/allpairs: records; linkage/longtext: records per group")
    ap.add_argument("--comparator", default="lev", choices=["lev", "jw"],
                    help="allpairs: the field's comparator")
    ap.add_argument("--dup-frac", type=float, default=0.1)
    ap.add_argument("--utf16-frac", type=float, default=0.0,
                    help="dedup: fraction of given names drawn from a non-Latin-1 vocabulary "
                         "(SURVEY §8d's 1%% UTF-16 slice: the NAME column becomes width 2)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="target CPU time of the oracle baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (0 = the CPUs this job may use: the "
                         "smaller of its affinity set and its cgroup CPU quota)")
    ap.add_argument("--cpu-single-seconds", type=float, default=6.0,
                    help="target CPU time of the single-core baseline sample (0 = skip)")
    ap.add_argument("--gather", default=None, choices=["none", "shm", "rccl"],
                    help="N>1 result path inside the timed steps (default shm): shm = every "
                         "GPU copies its tile's list into its slice of one shared host mapping "
                         "(rank 0 reads the node list in place: SURVEY §8d's result gather); "
                         "rccl = device lists gathered to GPU 0 over xGMI; none = each rank's "
                         "list stays in its HBM, only the per-rank counts are all-gathered")
    ap.add_argument("--phase-steps", type=int, default=3,
                    help="untimed steps after the timed region that give phases_ms_per_step "
                         "(0: take the phases from the timed region, with every phase's events in it)")
    ap.add_argument("--pcie-steps", type=int, default=3,
                    help="N=1: extra steps with the match list copied to pinned host memory "
                         "(the PCIe-inclusive rate, reported beside `value`; 0 = skip)")
    ap.add_argument("--no-json-batch", action="store_true",
                    help="skip the POSTed-body ingestion leg (dk_pack_json + upsert + match)")
    ap.add_argument("--no-warm-batch", action="store_true",
                    help="skip the warm-context re-upsert + match after the timed steps "
                         "(PMC passes: one step's launches only)")
    ap.add_argument("--only", default=None,
                    help="diagnostic: comma-separated property names to keep (not a bench line)")
    return ap.parse_args()


def heartbeat(rank):
    """Progress on stderr every 60 s while a long workload builds or runs (a silent GPU
    command looks hung to the job runner)."""
    import threading
    t0 = time.time()

    def run():
        while True:
            time.sleep(60)
            print(f"[bench rank {rank}] {time.time() - t0:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def prop(name, op, low, high, **kw):
    return {"name": name, "comparator": op, "low": low, "high": high, **kw}


def build_workload(args):
    """The synthetic data, schema and queries of one BASELINE configuration."""
    from dukehip import _abi as A
    from dukehip import synth
    n = args.records or DEFAULT_RECORDS[args.workload]
    w = {"name": args.workload, "keys": [], "group": None, "threshold": 0.9, "maybe": 0.7}
    if args.workload == "dedup":
        n_dup = int(n * args.dup_frac)
        p = synth.persons(n - n_dup, n_dup, utf16_frac=args.utf16_frac)
        w.update(desc="BASELINE configs[1]: 1M synthetic person records dedup, key blocking "
                      "K1=surname[0:3]+dob[0:4] K2=given[0:2]+dob[5:10]"
                      + (f", {args.utf16_frac:.0%} UTF-16 names" if args.utf16_frac else ""),
                 props=[prop("NAME", A.CMP_JAROWINKLER, 0.1, 0.95),
                        prop("ADDRESS", A.CMP_LEVENSHTEIN, 0.2, 0.8),
                        prop("DOB", A.CMP_LEVENSHTEIN, 0.1, 0.85)],
                 values={"NAME": p["name"], "ADDRESS": p["address"], "DOB": p["dob"]},
                 keys=synth.keys_config2(p), mode=A.MODE_DEDUP, queries=np.arange(n),
                 # the same key functions over the NAME / DOB columns (POSTed-body ingestion):
                 # NAME = "given surname", so token -1 is the surname and token 0 the given name
                 kparts=[(("NAME", -1, 0, 3), ("DOB", None, 0, 4)),
                         (("NAME", 0, 0, 2), ("DOB", None, 5, 10))])
    elif args.workload == "linkage":
        p, group = synth.linkage_persons(n)
        # BIRTHYEAR's min-ratio rejects every non-equal year of 1930..2010 (2009 / 2010 =
        # 0.99950 < 0.9996): with 0.9 every same-bucket pair had a near-constant 0.69 factor and
        # the list held ~10 % of the scored pairs.  ADDRESS low = 0.05: a
        # pair whose addresses share under half their bigrams cannot reach the list however
        # alike the names are (with 0.1, same-name / same-year / near-zip strangers did, and
        # their number grew with the bucket size: 1.6 entries per query at 1M, 13 at 10M).
        # The list is then the perturbed copies (30 % of group 2): ~0.28 entries per query
        # at every size.  SURVEY §8d names the comparators, not these values.
        w.update(desc=f"BASELINE configs[2]: person record linkage {n} x {len(group) - n}, QGram "
                      "q=2 DICE/JACCARD + Numeric BIRTHYEAR (min-ratio 0.9996: equal years) / ZIP "
                      "(min-ratio 0.9), cross-group key blocking",
                 props=[prop("NAME", A.CMP_QGRAM, 0.1, 0.9, q=2, formula=A.QGRAM_DICE),
                        prop("ADDRESS", A.CMP_QGRAM, 0.05, 0.8, q=2, formula=A.QGRAM_JACCARD),
                        prop("BIRTHYEAR", A.CMP_NUMERIC, 0.2, 0.6, min_ratio=0.9996),
                        prop("ZIP", A.CMP_NUMERIC, 0.4, 0.75, min_ratio=0.9)],
                 values={"NAME": p["name"], "ADDRESS": p["address"], "BIRTHYEAR": p["birthyear"],
                         "ZIP": p["zip"]},
                 keys=synth.keys_config2(p), group=group, mode=A.MODE_LINKAGE,
                 queries=np.arange(n, len(group)),
                 # the same key functions over the POSTed columns (json_ingest): DOB is a
                 # column only the key functions read (a key-only property)
                 kparts=[(("NAME", -1, 0, 3), ("BIRTHYEAR", None, 0, 4)),
                         (("NAME", 0, 0, 2), ("DOB", None, 5, 10))],
                 json_extra={"DOB": p["dob"]})
    elif args.workload == "allpairs":
        vals = synth.short_strings(n)
        op = A.CMP_LEVENSHTEIN if args.comparator == "lev" else A.CMP_JAROWINKLER
        w.update(desc=f"BASELINE configs[3]: {n} x {n} unblocked all-pairs (InMemoryDatabase), "
                      f"one a-z field of 4-16 units, {args.comparator}",
                 props=[prop("FIELD", op, 0.1, 0.95)], values={"FIELD": vals},
                 mode=A.MODE_ALLPAIRS, queries=np.arange(n),
                 threshold=0.85 if args.comparator == "lev" else 0.93, maybe=0.0)
    elif args.workload == "reference":
        import dukehip as dh
        from dukehip.config import DukeConfig
        from dukehip.lucene import lookup_properties
        with open(os.path.join(ROOT, "tests", "golden", "testdukeconfig_schema.json")) as f:
            cfg = DukeConfig.from_dict(json.load(f)["pipelines"]["Deduplication/countries-dbpedia-mondial"])
        recs = []
        for src, seed in zip(cfg.data_sources, (1234, 4321)):
            recs += dh.records_from_entities(synth.stress_entities(n // 2, seed), src)
        props = cfg.scored_properties()
        ids = {}
        w.update(desc=f"BASELINE configs[0]: the reference's testdukeconfig.xml dedup pipeline over "
                      f"{len(recs)} stress-test entities, Lucene candidate semantics "
                      "(lookup NAME, top 10, min-relevance 0.9)",
                 props=[dict(name=p.name, **{k: getattr(p.comparator.to_c(p.low, p.high), f)
                                             for k, f in (("comparator", "comparator"), ("low", "low"),
                                                          ("high", "high"), ("q", "qgram_q"),
                                                          ("formula", "qgram_formula"),
                                                          ("tokenizer", "qgram_tokenizer"),
                                                          ("min_ratio", "min_ratio"))})
                        for p in props],
                 values={p.name: [r.get_value(p.name) for r in recs] for p in props},
                 ident=np.array([ids.setdefault(r.get_value("ID"), len(ids)) for r in recs], np.uint64),
                 deleted=np.array([r.get_value("dukeDeleted") == "true" for r in recs], np.uint8),
                 lucene=lookup_properties(cfg, props), mode=A.MODE_DEDUP,
                 queries=np.arange(len(recs)), threshold=cfg.threshold, maybe=cfg.maybe_threshold)
    else:  # longtext
        texts, group = synth.long_texts(n)
        w.update(desc=f"BASELINE configs[4]: text linkage {n} x {len(group) - n}, 64-256 units, "
                      "WeightedLevenshtein + QGram q=3 JACCARD, key = first two tokens",
                 props=[prop("TEXT", A.CMP_WEIGHTED_LEVENSHTEIN, 0.2, 0.9),
                        prop("TEXTGRAMS", A.CMP_QGRAM, 0.3, 0.8, q=3, formula=A.QGRAM_JACCARD)],
                 values={"TEXT": texts, "TEXTGRAMS": texts},
                 keys=synth.keys_first_two_tokens(texts), group=group, mode=A.MODE_LINKAGE,
                 queries=np.arange(n, len(group)))
    # the committed PMC summary this line's roofline reads (profiles/pmc_<key>.json) and the
    # dominant kernel of the workload
    w["pmc_key"] = {"dedup": "dedup_utf16" if args.utf16_frac else "dedup",
                    "allpairs": f"allpairs_{args.comparator}"}.get(args.workload, args.workload)
    w["kernel"] = {"dedup": ("k_score<40,true,false> (symmetric owner schedule, one query per wave)"
                             if args.utf16_frac else
                             "k_score_sym2<40> (symmetric owner schedule, a query per half-wave)"),
                   "linkage": "k_score_gq<2,2>", "allpairs": "k_score<16,false,*>",
                   "longtext": "k_score_long<16,16>",
                   "reference": "k_score (Lucene candidates)"}[args.workload]
    w["n"] = len(next(iter(w["values"].values())))
    w["nkeys"] = len(w["keys"])
    w["queries"] = np.asarray(w["queries"], dtype=np.uint32)
    # Processor.compare visits the record's HashMap order (data-source columns + ID and the
    # ignored synthetic properties, App.java:309-323; dukeGroupNo in linkage)
    from dukehip.config import java_hashmap_order
    synth_props = ["ID", "dukeOriginalEntityId", "dukeDatasetId"]
    if w["mode"] == A.MODE_LINKAGE:
        synth_props.append("dukeGroupNo")
    by = {p["name"]: p for p in w["props"]}
    if args.only:
        by = {k: v for k, v in by.items() if k in args.only.split(",")}
    w["props"] = [by[k] for k in java_hashmap_order(list(by) + synth_props) if k in by]
    return w


def make_schema(w):
    from dukehip import _abi as A
    arr = (A.dk_property * len(w["props"]))()
    for i, p in enumerate(w["props"]):
        arr[i] = A.dk_property(p["comparator"], p.get("q", 2), p.get("formula", A.QGRAM_OVERLAP),
                               p.get("tokenizer", A.QGRAM_BASIC), p["low"], p["high"],
                               p.get("min_ratio", 0.0))
    s = A.dk_schema(len(w["props"]), arr, w["threshold"], w["maybe"], w["mode"], w["nkeys"])
    s._keep = arr
    if w.get("lucene"):
        names = [p["name"] for p in w["props"]]
        A.lucene_source(s, [names.index(x) for x in w["lucene"]], 10, 0.9)
    return s


def bpair_s8d(w, counts):
    """SURVEY §8(d)'s algorithmic bytes per scored pair (the unamortised operand stream):
    B_pair = 8 (two u32 row ids) + 1 (decision) + per string property 2·(4 + L̄·w)
           + per numeric property 2·8 + per q-gram property 2·(4 + Ḡ·g),
    L̄ / Ḡ the mean units / unique grams per value over the scored pairs (here: the query
    side weighted by each query's candidate count -- both sides of a pair come from the same
    generator in every config), w the stored unit width (1 Latin-1, 2 UTF-16), g the packed
    gram bytes (u32 codes for q <= 2, u64 above).  Returns (B_pair, per-property detail)."""
    from dukehip import _abi as A
    qs = np.asarray(w["queries"], dtype=np.int64)
    wt = np.asarray(counts, dtype=np.float64)
    if len(qs) > 200_000:   # a uniform sample of the queries estimates the weighted means
        pick = np.sort(np.random.default_rng(8).choice(len(qs), 200_000, replace=False))
        qs, wt = qs[pick], wt[pick]
    tot = wt.sum()
    if tot <= 0:
        return None, {}
    b, detail = 9.0, {}
    for p in w["props"]:
        vals = w["values"][p["name"]]
        sel = [vals[i] for i in qs]
        if p["comparator"] == A.CMP_NUMERIC:
            b += 16.0
            detail[p["name"]] = {"bytes": 16.0}
            continue
        lens = np.fromiter((len(s) if s else 0 for s in sel), np.float64, len(sel))
        wid = 2 if any(s and max(map(ord, s)) > 255 for s in sel[:20000]) else 1
        if p["comparator"] == A.CMP_QGRAM:
            qq = int(p.get("q", 2))
            g = np.fromiter((len({s[i:i + qq] for i in range(len(s) - qq + 1)}) if s else 0
                             for s in sel), np.float64, len(sel))
            gbar = float((g * wt).sum() / tot)
            gb = 4 if qq <= 2 else 8
            pb = 2.0 * (4 + gbar * gb)
            detail[p["name"]] = {"grams": gbar, "gram_bytes": gb, "bytes": pb}
        else:
            lbar = float((lens * wt).sum() / tot)
            pb = 2.0 * (4 + lbar * wid)
            detail[p["name"]] = {"units": lbar, "width": wid, "bytes": pb}
        b += pb
    return b, detail


CMP_NAMES = {1: "Levenshtein", 2: "JaroWinkler", 3: "QGramComparator", 4: "ExactComparator",
             5: "NumericComparator", 6: "WeightedLevenshtein", 7: "DiceCoefficientComparator",
             8: "JaccardIndexComparator"}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nranks, argv=None, port=None, script=None):
    """`bench.py --gpus N` started without a launcher: start the N ranks here, one child
    process per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1), the
    same environment torch.distributed.run gives them.  This process never touches the GPU
    (no torch import, no HIP call), so the children start clean; rank 0 prints the line.
    Returns the first non-zero child exit status (the others are then stopped), else 0."""
    import signal
    import subprocess
    argv = sys.argv[1:] if argv is None else argv
    port = port or free_port()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__),
                                       *argv], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for o in live:            # one rank failed: the collectives would hang
                    o.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    if args.gather is None:
        args.gather = "shm" if world > 1 else "none"
    heartbeat(rank)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    # DUKEHIP_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share a device);
    # the driver's runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("DUKEHIP_DIST_BACKEND", "nccl")
    if world > 1:
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    cdev = dev if backend == "nccl" else torch.device("cpu")   # where collectives run
    if world > 1 and backend != "nccl" and args.gather == "rccl":
        raise SystemExit("--gather rccl needs the nccl (RCCL) backend")

    import dukehip as dh
    from dukehip import synth

    from dukehip import dist as dshard
    t0 = time.time()
    shared_batch = None
    t_synth = 0.0
    if dist is None:
        w = build_workload(args)
        t_synth = time.time() - t0
        # records/sec deduped: the batch's host pack (strings -> SoA columns)
        # and dk_upsert, plus one dk_match of the batch (the step below)
        t_pack = time.perf_counter()
        cols = [synth.column(w["values"][p["name"]]) for p in w["props"]]
        kcols = [synth.column(k) for k in w["keys"]] or None
        t_pack = time.perf_counter() - t_pack
    else:
        # pack once: rank 0 builds and packs the batch, every rank maps the same SoA arrays
        # (one shared file under /dev/shm) and upserts them into its replica of the index
        meta, arrays, t_pack = [None], None, 0.0
        if rank == 0:
            w = build_workload(args)
            t_synth = time.time() - t0
            t_pack = time.perf_counter()
            cols = [synth.column(w["values"][p["name"]]) for p in w["props"]]
            kcols = [synth.column(k) for k in w["keys"]]
            t_pack = time.perf_counter() - t_pack
            arrays = dshard.columns_to_arrays("p", cols)
            arrays.update(dshard.columns_to_arrays("k", kcols))
            arrays["queries"] = w["queries"]
            if w["group"] is not None:
                arrays["group"] = w["group"]
            meta = [{k: v for k, v in w.items() if k not in ("values", "keys", "queries", "group")}]
        dist.broadcast_object_list(meta, src=0)
        shared_batch = dshard.SharedBatch(dist, rank, arrays)
        cols = dshard.arrays_to_columns("p", shared_batch.arrays)
        kcols = dshard.arrays_to_columns("k", shared_batch.arrays) or None
        if rank != 0:
            w = dict(meta[0])
            w["queries"] = shared_batch.arrays["queries"]
            w["group"] = shared_batch.arrays.get("group")
    n = w["n"]
    eng = dh.GpuEngine(make_schema(w), device=local)
    torch.cuda.synchronize()
    t_up = time.perf_counter()
    eng.upsert(n, w.get("ident", np.arange(n, dtype=np.uint64)), cols, group=w["group"],
               deleted=w.get("deleted"), key_columns=kcols)
    t_upsert = time.perf_counter() - t_up
    del cols, kcols
    t_index = time.time() - t0 - t_synth   # shared-batch mapping + pack + upsert (no synthesis)
    # this rank's contiguous query tile: equal estimated cost (blocking's candidate counts,
    # identical on every rank's replica of the index), SURVEY §8e
    allq = w["queries"]
    if world > 1:
        counts = eng.candidate_counts(allq)
        bounds = dshard.cost_bounds(counts, world)
    else:
        bounds = [0, len(allq)]
    q0, q1 = bounds[rank], bounds[rank + 1]
    queries = allq[q0:q1]
    nq_max = max(bounds[r + 1] - bounds[r] for r in range(world))
    holder = {}
    shared = None
    # the first dk_match after dk_upsert also builds the blocking tables + candidate replica
    # (index state); timed separately so records/s end to end charges that build
    first_match_s = None
    if dist is not None and args.gather == "shm":
        # size this rank's result region from one untimed device-mode match (the same
        # queries every step), with headroom; the regions form one shared host mapping
        torch.cuda.synchronize()
        t_fm = time.perf_counter()
        probe = eng.match(queries, on_device=True)
        torch.cuda.synchronize()
        first_match_s = time.perf_counter() - t_fm
        cap = torch.tensor([probe.n], dtype=torch.int64, device=cdev)
        probe.close()
        dist.all_reduce(cap, op=dist.ReduceOp.MAX)
        try:
            shared = dshard.SharedRegionGather(dist, torch, cdev, eng, nq_max,
                                               int(cap.item() * 1.05) + 4096, world, rank)
        except dshard.RegionUnavailable as e:   # all ranks: RCCL gather instead
            if backend != "nccl":
                raise
            if rank == 0:
                print(f"shm result gather unavailable ({e}); using --gather rccl",
                      file=sys.stderr, flush=True)
            args.gather = "rccl"

    def step(host=False):
        old = holder.pop("res", None)
        if old is not None:
            old.close()                       # hand the result memory back to the pool
        if dist is None:
            # the list stays in HBM (`value`), or is copied to pinned host memory (PCIe-
            # inclusive line: the boundary hands the listener host buffers)
            res = eng.match(queries, on_device=not host)
            holder["res"] = res
            return res, res.pairs_scored
        if args.gather == "none":
            # each rank's list stays in its HBM; the exchange is the all-gather of counts
            res = eng.match(queries, on_device=True)
            cnt = torch.tensor([res.n, res.pairs_scored, len(queries)], dtype=torch.int64, device=cdev)
            allc = [torch.zeros_like(cnt) for _ in range(world)]
            dist.all_gather(allc, cnt)
            holder["res"] = res
            holder["counts"] = [tuple(int(v) for v in c.cpu()) for c in allc]
            return res, sum(c[1] for c in holder["counts"])
        if shared is not None:
            # N>1, shm gather: the list goes to this rank's slice of the shared host mapping
            # (overlapped chunk copies over this GPU's own link); the all-gather of counts
            # completes the exchange, after which rank 0 holds the node list in place (a
            # list that outgrows its region is handled collectively by shared.match)
            res, total = shared.match(eng, queries)
            holder["res"] = res
            return res, total
        # N>1: entries stay in HBM; RCCL all-gathers the per-rank counts, then gathers
        # every rank's match list (first / candidate / prob / kind) to rank 0 over xGMI,
        # which moves the node's list to the host.
        res = eng.match(queries, on_device=True)

        def fill(first, cand, prob, kind):
            torch.cuda.synchronize()
            res.copy_to_device(first.data_ptr(), cand.data_ptr(), prob.data_ptr(), kind.data_ptr())

        _, total = dshard.gather_matches(dist, torch, cdev, len(queries), res.n, res.pairs_scored,
                                         fill, world, rank, nq_max)
        holder["res"] = res
        return res, total

    for i in range(args.warmup):
        if i == 0 and first_match_s is None:
            torch.cuda.synchronize()
            t_fm = time.perf_counter()
            step()
            torch.cuda.synchronize()
            first_match_s = time.perf_counter() - t_fm
        else:
            step()
    eng.reset_profile()
    # the timed region records HIP events around the scoring kernels only (the roofline's
    # launch times); the phase split comes from its own untimed pass (--phase-steps), since
    # each phase's two events cost the stream a few microseconds between dependent kernels
    eng.set_profiling(2 if args.phase_steps > 0 else True)
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
    prof_ph, nph = prof, args.steps
    if args.phase_steps > 0:
        nph = args.phase_steps
        eng.reset_profile()
        eng.set_profiling(True)
        for _ in range(nph):
            last, _ = step()
        torch.cuda.synchronize()
        eng.set_profiling(False)
        prof_ph = eng.profile()
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms_step = el / args.steps * 1e3
    pairs_step = total_scored / args.steps
    value = pairs_step / (ms_step / 1e3)

    # PCIe-inclusive line (N=1): the same step with the match list copied to pinned host
    # memory, as the C-ABI hands it to the MatchListener replay; never `value`
    pcie = None
    if world == 1 and args.pcie_steps > 0:
        step(host=True)                      # sizes the pinned pool
        torch.cuda.synchronize()
        tp = time.perf_counter()
        sc_p = 0
        for _ in range(args.pcie_steps):
            last, sc = step(host=True)
            sc_p += sc
        torch.cuda.synchronize()
        elp = time.perf_counter() - tp
        pcie = {"value": sc_p / elp, "unit": "pairs/s", "steps": args.pcie_steps,
                "ms_per_step": elp / args.pcie_steps * 1e3,
                "note": "match list copied to pinned host memory inside the step (the "
                        "boundary's host buffers); not `value`"}

    if rank == 0:
        launches = max(1, prof["score_launches"])
        score_s = prof["ms_score"] / 1e3
        # roofline.achieved: SURVEY §8(d)'s B_pair x the pairs one k_score launch scores, over
        # the launch's HIP-event time on the ctx stream
        if world == 1:
            counts = eng.candidate_counts(allq)
        bpair, bdetail = bpair_s8d(w, counts)
        pairs_launch = prof["pairs_scored"] / launches
        avg_launch_s = score_s / launches
        # configs[2]'s k_score_gq keeps each query's operands in LDS and screens every pair on
        # one QGram role and the Numeric roles, the deferred role's keys read only for the pairs
        # that reach its exact pass: its algorithmic bytes are the schedule's own -- the kernel's
        # count (ids + decision 9 B, per role its candidate length / gram count / keys or numeric
        # operands, the deferred role's keys x the exact-pass pairs) plus each query's operands
        # once -- not §8(d)'s unamortised B_pair, which charges both sides of every pair
        qbytes = sum(d["bytes"] / 2.0 for d in bdetail.values()) if bdetail else 0.0
        s8d_basis = "SURVEY §8(d) B_pair (both sides' operands per directed pair)"
        bpair_s8d_unamortised = bpair
        if args.workload == "linkage" and prof["pairs_scored"] > 0 and prof.get("pairs_exact"):
            bpair = (prof["score_bytes"] + qbytes * len(queries) * args.steps) / prof["pairs_scored"]
            s8d_basis = ("k_score_gq schedule: the kernel's counted candidate operands (deferred role's "
                         "keys only for exact-pass pairs) + each query's operands once, per scored pair")
        achieved = bpair * pairs_launch / avg_launch_s if avg_launch_s > 0 and bpair else 0.0
        # the bytes this schedule REQUESTS (VERDICT r3's bound): every scored pair's candidate
        # operands at their stored width (the kernel's own count, score_bytes) plus each
        # query's operands once -- L2 serves part of these (the PMC's TCC hit rate), so this is
        # a request-bandwidth fraction, not an HBM one
        request_launch = (prof["score_bytes"] + qbytes * len(queries) * args.steps) / launches
        frac_request = request_launch / avg_launch_s / HBM_PEAK if avg_launch_s > 0 else None
        sched = prof["score_bytes"] / score_s if score_s > 0 else 0.0
        # roofline.frac: the CALIBRATED-COUNTER HBM fraction of the dominant kernel -- the
        # committed PMC summary of the kernel this workload runs (scripts/summarize_profiles.py:
        # FETCH_SIZE x 2 + WRITE_SIZE per scored pair, the factor from
        # profiles/r05/fetch_calib.json), at this run's pairs per launch, over the launch's
        # HIP-event time.  Measured bytes over measured time: <= 1 by construction.
        traffic = None
        valu = None
        pmc_info = None
        pj = None
        for cand in (f"pmc_{w['pmc_key']}_{n}.json", f"pmc_{w['pmc_key']}.json"):
            path = os.path.join(ROOT, "profiles", cand)
            if os.path.exists(path):
                with open(path) as f:
                    pj = json.load(f)
                pmc_path = path
                break
        if pj and pj.get("hbm_bytes_per_pair"):
            traffic = pj["hbm_bytes_per_pair"] * prof["pairs_scored"] / launches
            pmc_info = {"file": os.path.relpath(pmc_path, ROOT), "commit": pj.get("commit"),
                        "kernel_symbol": pj.get("kernel_symbol"), "records": pj.get("records"),
                        "hbm_bytes_per_pair": pj["hbm_bytes_per_pair"],
                        "tcc_hit_rate": pj.get("tcc_hit_rate"),
                        "wait_any_frac": pj.get("wait_any_frac"),
                        "lds_conflict_cycles_per_lds_inst": pj.get("lds_conflicts_per_lds_inst")}
            # VALU issue: wave-instructions per scored pair of the SAME PMC summary, at this
            # run's pairs and k_score time, against the chip's 2-cycle issue rate (1,024 SIMDs x
            # 2.4 GHz / 2) and against the achievable rate of that kernel's own instruction mix
            ipp = pj["counters"]["SQ_INSTS_VALU"] / pj["pairs_profiled"]
            rate = ipp * prof["pairs_scored"] / score_s if score_s > 0 else 0.0
            valu = {"insts_per_pair": ipp, "achieved": rate / 1e9, "peak": VALU_PEAK / 1e9,
                    "unit": "G wave-instructions/s", "frac": rate / VALU_PEAK,
                    "source": pmc_info["file"] + " (" + str(pj.get("commit")) + ")"}
            vm = os.path.join(ROOT, "profiles", "valu_mix.json")
            if os.path.exists(vm):
                with open(vm) as f:
                    mx = json.load(f).get(w["pmc_key"])
                if mx and mx.get("avg_cycles_per_valu"):
                    ach = 1024 * 2.4e9 / mx["avg_cycles_per_valu"]
                    valu.update(avg_cycles_per_valu=mx["avg_cycles_per_valu"],
                                peak_achievable=ach / 1e9, frac_achievable=rate / ach,
                                mix_kernel=mx["kernel"], mix_region=mx.get("region"),
                                mix_source="profiles/valu_mix.json (" + str(mx.get("commit")) + ")")
        hbm_rate = traffic / avg_launch_s if traffic and avg_launch_s > 0 else None
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
            "config": {"workload": w["desc"], "records": n, "queries": int(len(allq)),
                       "pairs_per_step": pairs_step,
                       "comparators": {p["name"]: CMP_NAMES[p["comparator"]] for p in w["props"]},
                       "threshold": w["threshold"], "maybe_threshold": w["maybe"],
                       "parallelism": f"query-tile sharding x{world} (cost-weighted tiles), replicated index"
                                      + (f", {args.gather} result gather" if world > 1 else "")},
            "records_per_s": len(allq) / (ms_step / 1e3),
            # host pack + dk_upsert + the first dk_match after it (table build included)
            "records_per_s_end_to_end": len(allq) / (t_pack + t_upsert + max(
                ms_step / 1e3, first_match_s or 0.0)),
            "first_match_s": first_match_s,
            "host_pack_s": t_pack,
            "upsert_s": t_upsert,
            "matches_per_step": (sum(c[0] for c in shared.counts) if shared is not None
                                 else sum(c[0] for c in holder["counts"]) if "counts" in holder
                                 else int(last.n) if last is not None else 0),
            "index_build_s": t_index,
            # the list: entries per query record, and its cost per step (device compaction of
            # the staged entries, k_compact + scan), apart from the scoring kernel
            "entries_per_query": ((sum(c[0] for c in shared.counts) if shared is not None
                                   else sum(c[0] for c in holder["counts"]) if "counts" in holder
                                   else int(last.n) if last is not None else 0) / max(1, len(allq))),
            "list_ms_per_step": prof_ph["ms_gather"] / nph,
            # k_score_gq: the scored pairs its single-precision screen sent to the exact pass
            "exact_pass_fraction": (prof["pairs_exact"] / prof["pairs_scored"]
                                    if prof.get("pairs_exact") and prof["pairs_scored"] else None),
            "synth_s": t_synth,
            "roofline": {"bound": "hbm",
                         "achieved": hbm_rate / 1e9 if hbm_rate else None,
                         "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": hbm_rate / HBM_PEAK if hbm_rate else None,
                         "traffic": traffic,
                         "frac_basis": ("calibrated HBM counter bytes of the dominant kernel (its "
                                        "committed PMC pass, `pmc`) over its HIP-event launch time"
                                        if hbm_rate else "no committed PMC summary for this "
                                        "workload: frac unmeasured"),
                         "kernel": prof.get("score_kernel") or w["kernel"],
                         "pmc": pmc_info, "pmc_key": w["pmc_key"],
                         "launches": prof["score_launches"],
                         "avg_launch_ms": prof["ms_score"] / launches,
                         "pairs_per_launch": pairs_launch,
                         # SURVEY §8(d)'s algorithmic bytes (B_pair charges each pair both
                         # sides' operands; a kernel holding the query in LDS can pass 1 here)
                         "achieved_s8d": achieved / 1e9, "frac_s8d": achieved / HBM_PEAK,
                         "b_pair_s8d": bpair, "s8d_basis": s8d_basis,
                         "b_pair_s8d_unamortised": bpair_s8d_unamortised, "b_pair_detail": bdetail,
                         "bytes_per_launch_s8d": bpair * pairs_launch if bpair else None,
                         "frac_step_s8d": (bpair * value / (HBM_PEAK * world)) if bpair else None,
                         # what the schedule requests (L2 serves part): not an HBM fraction
                         "frac_request": frac_request,
                         "request_bytes_per_launch": request_launch,
                         "query_bytes_per_query": qbytes,
                         "operand_bytes_per_launch": prof["score_bytes"] / launches,
                         "frac_operand_request": sched / HBM_PEAK,
                         "limiter": "valu" if valu else None, "valu": valu},
            "pcie_inclusive": pcie,
            # per-rank pairs scored of the last step (tile balance; N>1)
            "rank_pairs": ([c[1] for c in holder["counts"]] if "counts" in holder else
                           [c[1] for c in shared.counts] if shared is not None and shared.counts else None),
            # device time per phase, from the untimed phase pass (phase_steps steps)
            "phases_ms_per_step": {k: prof_ph[k] / nph for k in
                                   ("ms_index", "ms_generate", "ms_score", "ms_emit", "ms_gather", "ms_copy",
                                    "ms_total")},
            "phase_steps": nph,
        }
        if world == 1 and args.cpu_seconds > 0:
            if last is None or last.on_device:
                last, _ = step(host=True)    # the check needs the list on the host
            out["cpu_baseline"] = cpu_baseline(w, last, args)
        if world == 1 and not args.no_warm_batch:
            old = holder.pop("res", None)
            if old is not None:
                old.close()
            last = None
            out["warm_batch"] = warm_batch(eng, w, n, queries, torch)
            if w.get("kparts") and not args.no_json_batch:
                jb = json_batch(w, n, queries, local, torch)
                # the POSTed records must give the step's pairs (same records, same keys)
                jb["pairs_equal_to_step"] = jb["cold"]["pairs_scored"] == int(pairs_step)
                out["json_ingest"] = jb
                # records/sec deduped from the POSTed body: the end-to-end figure
                out["records_per_s_end_to_end_lists"] = out["records_per_s_end_to_end"]
                out["records_per_s_end_to_end"] = jb["cold"]["records_per_s"]
        print(json.dumps(out), flush=True)
    last = None
    holder.clear()
    if shared is not None:
        dist.barrier()   # rank 0 is done with the lists
        shared.close()
    if shared_batch is not None:
        shared_batch.close()
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def json_body(ids, cols):
    """A JSON array of entities {"_id": id, column: value, ...} (the POSTed body), built with
    one f-string per entity: the synthetic values hold no character JSON escapes."""
    names = list(cols)
    for k in names:
        assert not any(('"' in v or "\\" in v) for v in cols[k][:1000]), k
    vals = [cols[k] for k in names]
    keys = [json.dumps(k) for k in names]
    parts = []
    for i, row in zip(ids, zip(*vals)):
        parts.append('{"_id":"' + str(i) + '",' + ",".join(k + ':"' + v + '"' for k, v in zip(keys, row)) + "}")
    return ("[" + ",".join(parts) + "]").encode()


def json_batch(w, n, queries, device, torch):
    """records/sec from the POSTed body: the batch as the HTTP
    endpoint receives it (JSON bytes, serialised untimed; linkage: one body per group, as its
    two data sources receive them), then dk_pack_json (entities -> SoA columns, key functions,
    record-ID interning) + dk_upsert + the first dk_match of the batch on a fresh context
    (table build included; list left in HBM), timed; then the same bodies again on that
    now-warm context (every record re-posted: tombstones + delta tables)."""
    import dukehip as dh
    from dukehip import ingest
    from dukehip.config import DataSource, DataSourceColumn
    names = [p["name"] for p in w["props"]]
    extra = w.get("json_extra", {})
    cols = {k: w["values"][k] for k in names}
    cols.update(extra)
    total = len(next(iter(cols.values())))
    if w["group"] is None:
        groups = [(0, total, 0)]
    else:   # one body per group (its data source), in row order: group 1's rows come first
        g = np.asarray(w["group"])
        n1 = int((g == 1).sum())
        assert (g[:n1] == 1).all() and (g[n1:] == 2).all()
        groups = [(0, n1, 1), (n1, total, 2)]
    t_json = time.perf_counter()
    bodies = [json_body(range(a, b), {k: v[a:b] for k, v in cols.items()}) for a, b, _ in groups]
    t_json = time.perf_counter() - t_json
    kfs = [dh.PartsKey(*kp) for kp in w["kparts"]]
    srcs = [ingest.NativeSource(DataSource(f"persons{g}", [DataSourceColumn(k, k) for k in cols], g or None),
                                names, kfs) for _, _, g in groups]
    ids = ingest.Interner()
    eng = dh.GpuEngine(make_schema(w), device=device)
    out = {"path": "dk_pack_json -> dk_upsert -> dk_match", "body_bytes": sum(map(len, bodies)),
           "bodies": len(bodies), "records_posted": total, "queries": int(len(queries)),
           "json_build_s_untimed": t_json}
    try:
        for leg in ("cold", "warm"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pks = [src.pack(body, ids) for src, body in zip(srcs, bodies)]
            t1 = time.perf_counter()
            rows = np.concatenate([eng.upsert_packed(pk) for pk in pks])
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            qrows = rows[queries]
            t2a = time.perf_counter()
            res = eng.match(qrows, on_device=True)   # the batch's new rows
            t2b = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            out[leg] = {"pack_s": t1 - t0, "upsert_s": t2 - t1, "match_s": t3 - t2,
                        "match_parts_s": {"query_rows": t2a - t2, "dk_match": t2b - t2a, "sync": t3 - t2b},
                        "pairs_scored": int(res.pairs_scored),
                        "records_per_s": len(queries) / (t3 - t0),
                        "posted_records_per_s": total / (t3 - t0)}
            res.close()
            for pk in pks:
                pk.close()
    finally:
        eng.close()
        ids.close()
    return out


def warm_batch(eng, w, n, queries, torch):
    """records/sec deduped for a batch on a warm context (pools sized, kernels loaded): the
    same records upserted again under their IDs (delete-then-add, so the index changes and
    the next dk_match rebuilds the blocking tables and the replica), then that match.
    Untimed by the step loop; reported beside records_per_s_end_to_end (cold)."""
    from dukehip import synth
    t0 = time.perf_counter()
    cols = [synth.column(w["values"][p["name"]]) for p in w["props"]]
    kcols = [synth.column(k) for k in w["keys"]] or None
    t1 = time.perf_counter()
    rows = eng.upsert(n, w.get("ident", np.arange(n, dtype=np.uint64)), cols, group=w["group"],
                      deleted=w.get("deleted"), key_columns=kcols)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res = eng.match(rows[queries], on_device=True)   # the re-posted records' new rows
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    res.close()
    return {"host_pack_s": t1 - t0, "upsert_s": t2 - t1, "match_after_upsert_s": t3 - t2,
            "records_per_s_end_to_end": len(queries) / (t3 - t0)}


def cpu_baseline(w, gpu_res, args):
    """The C oracle (oracle/duke_oracle.c, a restatement of Duke's scoring loop) on a
    bounded sample: the first S query records, full candidate lists, host threads.  The
    same sample's match list is checked against the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from dukehip import _abi as A
    if w.get("lucene"):
        return cpu_baseline_lucene(w, gpu_res, O)
    mode = {A.MODE_DEDUP: "dedup", A.MODE_LINKAGE: "linkage", A.MODE_ALLPAIRS: "allpairs"}[w["mode"]]
    props = [{k: v for k, v in p.items() if k != "name"} for p in w["props"]]
    ot = O.OracleTable(props, [w["values"][p["name"]] for p in w["props"]], keys=w["keys"],
                       group=w["group"], threshold=w["threshold"], maybe=w["maybe"], mode=mode)
    nproc = os.cpu_count() or 1
    affinity, quota = host_cpus()
    effective = max(1, min(affinity or nproc, int(-(-quota // 1)) if quota else nproc))
    threads = args.cpu_threads or effective
    allq = w["queries"]

    def sample(nthreads, seconds):
        probe = min(len(allq), max(2000, 64 * nthreads) if mode != "allpairs" else max(64, 2 * nthreads))
        if nthreads == 1:
            probe = max(1, min(probe, 2000) // 16)
        r = ot.match(allq[:probe], nthreads=nthreads)
        rate = r["pairs_scored"] / max(r["ms_score"] / 1e3, 1e-9)
        per_q = r["pairs_scored"] / probe
        s = int(min(len(allq), max(probe, seconds * rate / max(per_q, 1e-9))))
        return s, ot.match(allq[:s], nthreads=nthreads)

    single = None
    if args.cpu_single_seconds > 0:
        s1, r1 = sample(1, args.cpu_single_seconds)
        single = {"value": r1["pairs_scored"] / (r1["ms_score"] / 1e3), "cores": 1,
                  "sample": f"first {s1} query records ({r1['pairs_scored']} pairs)",
                  "seconds": r1["ms_score"] / 1e3}
    s, r = sample(threads, args.cpu_seconds)
    e = int(gpu_res.first[s])
    gq = np.repeat(allq[:s], np.diff(gpu_res.first[: s + 1]).astype(np.int64))
    ok = (np.array_equal(r["query"], gq) and np.array_equal(r["candidate"], gpu_res.candidate[:e])
          and np.array_equal(r["prob"], gpu_res.prob[:e]) and np.array_equal(r["kind"], gpu_res.kind[:e]))
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    out = {"value": r["pairs_scored"] / (r["ms_score"] / 1e3), "unit": "pairs/s",
           # the CPUs the threads actually ran on: min(threads, affinity, cgroup quota)
           "cores": min(threads, effective), "threads": threads,
           "kind": "port",
           "sample": f"first {s} of {len(allq)} query records ({r['pairs_scored']} pairs), "
                     f"scoring loop timed, blocking-index build excluded ({r['ms_index']:.0f} ms)",
           "seconds": r["ms_score"] / 1e3, "cpu_model": cpu, "host_nproc": nproc,
           "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
           "matches_identical_to_gpu": bool(ok), "single_core": single}
    if single:
        # EXTRAPOLATION, not a measurement: the single-core rate x every hardware thread the
        # host reports (linear scaling, an upper bound of the whole node's CPU rate; this job
        # may only use `cores` of them)
        out["extrapolated_all_host_threads"] = {
            "value": single["value"] * nproc, "threads": nproc,
            "note": "single-core rate x host_nproc, linear (extrapolated, not measured)"}
    return out


def host_cpus():
    """(CPUs in this process's affinity set, cgroup v2 CPU quota in CPUs or None)."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except OSError:
        affinity = None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return affinity, quota


def cpu_baseline_lucene(w, gpu_res, O):
    """configs[0] on the CPU: the restated Lucene query (oracle/lucene_ref.py, pure Python)
    for candidates, the C oracle's Processor.compare for each hit, one thread; the whole list
    is checked against the GPU's."""
    import lucene_ref as R
    props = [{k: v for k, v in p.items() if k != "name"} for p in w["props"]]
    names = [p["name"] for p in w["props"]]
    vals = [w["values"][nm] for nm in names]
    n = len(vals[0])
    ident = w["ident"]
    alive = np.zeros(n, bool)
    last = {}
    for r in range(n):
        last[int(ident[r])] = r
    alive[list(last.values())] = True
    t0 = time.perf_counter()
    ref = R.LuceneIndexRef(w["lucene"], 10, 0.9)
    ref.set_docs([w["values"][f] for f in w["lucene"]], alive, w["deleted"])
    ot = O.OracleTable(props, vals, ident=ident, threshold=w["threshold"], maybe=w["maybe"])
    t1 = time.perf_counter()
    q_out, c_out, p_out, k_out = [], [], [], []
    scored = 0
    for q in w["queries"]:
        for c in ref.candidates(int(q)):
            if ident[c] == ident[q]:
                continue
            scored += 1
            p = ot.compare_rows(int(q), int(c))
            kind = 1 if p > w["threshold"] else (2 if w["maybe"] != 0.0 and p > w["maybe"] else 0)
            if kind:
                q_out.append(int(q)); c_out.append(int(c)); p_out.append(p); k_out.append(kind)
    el = time.perf_counter() - t1
    gq = np.repeat(w["queries"], np.diff(gpu_res.first).astype(np.int64))
    ok = (list(gq) == q_out and list(gpu_res.candidate) == c_out and list(gpu_res.prob) == p_out
          and list(gpu_res.kind) == k_out)
    return {"value": scored / el, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"all {len(w['queries'])} query records ({scored} pairs): Lucene query restated "
                      f"in Python + C Processor.compare; index build excluded ({t1 - t0:.1f} s)",
            "seconds": el, "matches_identical_to_gpu": bool(ok), "single_core": None}


if __name__ == "__main__":
    main()
