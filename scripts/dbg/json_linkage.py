"""Debug: configs[2] json leg at a small size vs the column path (GPU)."""
import sys
import numpy as np
sys.path[:0] = ['sesam-duke-microservice_amd', '.']
import torch
import bench
import dukehip as dh
from dukehip import ingest
from dukehip.config import DataSource, DataSourceColumn
sys.argv = ['bench.py', '--workload', 'linkage', '--records', '3000']
a = bench.parse()
w = bench.build_workload(a)
w["nkeys"] = len(w["keys"])
n = 3000
queries = np.arange(n, 2 * n)
print(bench.json_batch(w, n, queries, 0, torch))
names = [p["name"] for p in w["props"]]
cols = {k: w["values"][k] for k in names}
cols.update(w["json_extra"])
kfs = [dh.PartsKey(*kp) for kp in w["kparts"]]
ids = ingest.Interner()
eng = dh.GpuEngine(bench.make_schema(w), device=0)
rows = []
for a0, b0, g in [(0, n, 1), (n, 2 * n, 2)]:
    src = ingest.NativeSource(DataSource(f"p{g}", [DataSourceColumn(k, k) for k in cols], g), names, kfs)
    pk = src.pack(bench.json_body(range(a0, b0), {k: v[a0:b0] for k, v in cols.items()}), ids)
    b = pk.batch()
    print("batch n", pk.n, "keys", pk.keys(0)[:2], pk.keys(1)[:2])
    rows.append(eng.upsert_packed(pk))
rows = np.concatenate(rows)
print("rows", rows[:5], rows[n:n + 5])
res = eng.match(rows[queries])
print("json path pairs", res.pairs_scored, "n", res.n)
eng2 = dh.GpuEngine(bench.make_schema(w), device=0)
r2 = eng2.upsert(2 * n, np.arange(2 * n, dtype=np.uint64), [dh.Column.from_strings(w["values"][k]) for k in names],
                 group=w["group"], key_columns=[dh.Column.from_strings(k) for k in w["keys"]])
res2 = eng2.match(r2[queries])
print("column path pairs", res2.pairs_scored, "n", res2.n)
