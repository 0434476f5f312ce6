"""Debug (CPU only): time dk_pack_json on configs[2]'s POSTed bodies at --records N."""
import sys, time
import numpy as np
sys.path[:0] = ['sesam-duke-microservice_amd', '.']
import bench
import dukehip as dh
from dukehip import ingest
from dukehip.config import DataSource, DataSourceColumn
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
sys.argv = ['bench.py', '--workload', 'linkage', '--records', str(n)]
a = bench.parse()
t = time.time()
w = bench.build_workload(a)
print("synth", round(time.time() - t, 2), flush=True)
names = [p["name"] for p in w["props"]]
cols = {k: w["values"][k] for k in names}
cols.update(w["json_extra"])
kfs = [dh.PartsKey(*kp) for kp in w["kparts"]]
groups = [(0, n, 1), (n, 2 * n, 2)]
t = time.time()
bodies = [bench.json_body(range(a0, b0), {k: v[a0:b0] for k, v in cols.items()}) for a0, b0, _ in groups]
print("json build", round(time.time() - t, 2), "bytes", sum(map(len, bodies)), flush=True)
srcs = [ingest.NativeSource(DataSource(f"p{g}", [DataSourceColumn(k, k) for k in cols], g), names, kfs)
        for _, _, g in groups]
for r in range(reps):
    ids = ingest.Interner()
    t = time.perf_counter()
    pks = []
    for src, body in zip(srcs, bodies):
        t1 = time.perf_counter()
        pks.append(src.pack(body, ids))
        print("  body", round(time.perf_counter() - t1, 3), flush=True)
    dt = time.perf_counter() - t
    print(f"rep {r}: pack {dt:.3f} s  {2 * n / dt / 1e6:.2f} M posted rec/s", flush=True)
    for pk in pks:
        pk.close()
    ids.close()
