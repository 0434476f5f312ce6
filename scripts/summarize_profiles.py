"""Turn rocprofv3 outputs into the committed profile summaries.

usage: python scripts/summarize_profiles.py TRACE_DIR PMC_DIR OUT_DIR [PMC_KEY]
  TRACE_DIR: rocprofv3 --kernel-trace --stats --output-format csv -d TRACE_DIR
  PMC_DIR:   scripts/pmc_profile.sh PMC_DIR (valu / fetch / write / stall / l2 passes)
Writes OUT_DIR/kernel_stats.csv (copy of rocprofv3's stats), OUT_DIR/pmc_k_score.txt and
profiles/pmc_<PMC_KEY>.json (bench.py's roofline for that workload: dedup, dedup_utf16,
linkage, allpairs_lev, allpairs_jw, longtext, reference; PMC_KEY defaults to the workload
named by the profiled bench line).  The summary names the profiled kernel's symbol (the
most frequent k_score* dispatch), the commit (DK_COMMIT) and the records of the run.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB, and on gfx950 FETCH_SIZE reads exactly half the bytes of a coalesced row read -- the
guide calibrates 16 B per lane; scripts/micro/fetch_calib.hip calibrates the scoring kernels'
own widths (4- and 8-B-per-lane row reads: factor 2.000, profiles/r04/fetch_calib.json) --
so the read side is doubled.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


KERNELS = collections.Counter()


def pmc(pass_dir):
    f = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    agg, disp = collections.defaultdict(float), set()
    if not f:
        return agg, 0
    for r in csv.DictReader(open(f[0])):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Dispatch_Id"] not in disp:
            KERNELS[r["Kernel_Name"]] += 1
        disp.add(r["Dispatch_Id"])
    return agg, len(disp)


def main():
    trace, pmcdir, out = sys.argv[1:4]
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(trace, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(out, "kernel_stats.csv"))
    res = {}
    for name in ("valu", "fetch", "write", "stall", "l2"):
        agg, n = pmc(os.path.join(pmcdir, name))
        res[name] = (dict(agg), n)
    fetch_kb, n = res["fetch"][0].get("FETCH_SIZE", 0.0), max(1, res["fetch"][1])
    write_kb = res["write"][0].get("WRITE_SIZE", 0.0)
    v, s = res["valu"][0], res["stall"][0]
    per_launch = (2.0 * fetch_kb + write_kb) * 1024.0 / n
    # pairs scored by the profiled command (its bench.py JSON line), for a per-pair figure
    # that bench.py scales to its own launch mix
    pairs, workload, records, key = None, None, None, None
    try:
        for line in open(os.path.join(pmcdir, "fetch.log")):
            if line.startswith("{"):
                d = json.loads(line)
                pairs = d["config"]["pairs_per_step"] * d["steps"] + d["config"]["pairs_per_step"] * d["warmup"]
                workload = d["config"]["workload"].split(":")[0]
                records = d["config"].get("records")
                key = (d.get("roofline") or {}).get("pmc_key")
    except (OSError, ValueError, KeyError):
        pass
    names = {"BASELINE configs[1]": "dedup", "BASELINE configs[2]": "linkage",
             "BASELINE configs[3]": "allpairs", "BASELINE configs[4]": "longtext"}
    l2 = res["l2"][0]
    hits, misses = l2.get("TCC_HIT_sum", 0.0), l2.get("TCC_MISS_sum", 0.0)
    key = sys.argv[4] if len(sys.argv) > 4 else (key or names.get(workload, workload))
    summary = {
        "kernel": "k_score",
        "kernel_symbol": KERNELS.most_common(1)[0][0] if KERNELS else None,
        "workload": names.get(workload, workload),
        "pmc_key": key,
        "records": records,
        "commit": os.environ.get("DK_COMMIT", "?"),
        "launches_profiled": n,
        "fetch_size_kib_total": fetch_kb,
        "write_size_kib_total": write_kb,
        "hbm_bytes_per_launch": per_launch,
        "hbm_bytes_per_launch_uncorrected": (fetch_kb + write_kb) * 1024.0 / n,
        "pairs_profiled": pairs,
        "hbm_bytes_per_pair": (2.0 * fetch_kb + write_kb) * 1024.0 / pairs if pairs else None,
        "valu_insts_per_wave": v.get("SQ_INSTS_VALU", 0) / max(1.0, v.get("SQ_WAVES", 1)),
        # per 64 scored pairs (a wave of k_score, a quarter task of k_score_grouped)
        "valu_insts_per_64_pairs": v.get("SQ_INSTS_VALU", 0) * 64.0 / pairs if pairs else None,
        "fetch_calibration": "profiles/r05/fetch_calib.json (2/4/8/16 B per lane: x2.000; "
                             "scripts/fetch_calib_summary.py rejects launches under 1 % of their bytes)",
        "tcc_hit_rate": hits / (hits + misses) if hits + misses else None,
        "valu_thread_utilization": v.get("SQ_THREAD_CYCLES_VALU", 0) /
                                   max(1.0, v.get("SQ_ACTIVE_INST_VALU", 1) * 64),
        "wait_any_frac": s.get("SQ_WAIT_ANY", 0) / max(1.0, s.get("SQ_WAVE_CYCLES", 1)),
        "wait_inst_any_frac": s.get("SQ_WAIT_INST_ANY", 0) / max(1.0, s.get("SQ_WAVE_CYCLES", 1)),
        "active_inst_any_frac": s.get("SQ_ACTIVE_INST_ANY", 0) / max(1.0, s.get("SQ_WAVE_CYCLES", 1)),
        "lds_bank_conflict_cycles": s.get("SQ_LDS_BANK_CONFLICT", 0),
        "lds_conflicts_per_lds_inst": s.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_INSTS_LDS"]
                                      if v.get("SQ_INSTS_LDS") else None,
        "counters": {k: v for d in res.values() for k, v in d[0].items()},
    }
    with open(os.path.join(out, "pmc_k_score.txt"), "w") as f:
        for k, val in summary.items():
            f.write(f"{k}: {val}\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dest = os.environ.get("PMC_JSON", os.path.join(root, "profiles", f"pmc_{key}.json"))
    with open(dest, "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: summary[k] for k in list(summary)[:12]}, indent=1))


if __name__ == "__main__":
    main()
