"""Summarise scripts/micro/lds_probe.sh: per variant the measured LDS bank-conflict cycles
per LDS instruction (SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS), LDS-array cycles per instruction
(SQ_LDS_IDX_ACTIVE / SQ_INSTS_LDS), the Monte-Carlo expectation and the probe time."""
import csv, glob, json, os, re, sys

out = sys.argv[1]
timing = {}
for line in open(os.path.join(out, "timing.jsonl")):
    d = json.loads(line)
    timing[d["variant"].split("_")[0]] = d
names = {k: v["variant"] for k, v in timing.items()}
acc = {}
for path in glob.glob(os.path.join(out, "pmc", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        m = re.search(r"k_probe<(\d+)>", r["Kernel_Name"])
        if not m:
            continue
        v = "V" + m.group(1)
        acc.setdefault(v, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
res = []
for v in sorted(acc):
    c = {k: sum(x) / len(x) for k, x in acc[v].items()}  # warm-up and timed launch alike
    lds = c.get("SQ_INSTS_LDS", 0.0)
    t = timing.get(v, {})
    res.append({"variant": names.get(v, v),
                "conflict_cycles_per_lds_inst": c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else None,
                "lds_array_cycles_per_lds_inst": c.get("SQ_LDS_IDX_ACTIVE", 0.0) / lds if lds else None,
                "mc_extra_cycles": t.get("mc_extra_cycles"),
                "ns_per_probe_inst_per_cu": t.get("ns_per_probe_inst_per_cu")})
print(json.dumps(res, indent=1))
