"""Host-only timing of dk_pack_json on the configs[1] body (1M person records, 106 MB):
DK_INGEST_THREADS sweeps the worker count (the GPU box gives a job 16 CPUs).  Diagnostic."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sesam-duke-microservice_amd"))
import dukehip as dh  # noqa: E402
from dukehip import ingest, synth  # noqa: E402
from dukehip.config import DataSource, DataSourceColumn  # noqa: E402

n = int(os.environ.get("N", "1000000"))
p = synth.persons(n - n // 10, n // 10)
names = ["NAME", "ADDRESS", "DOB"]
cols = [p["name"], p["address"], p["dob"]]
body = json.dumps([{"_id": str(i), **{k: c[i] for k, c in zip(names, cols)}} for i in range(n)]).encode()
src = ingest.NativeSource(DataSource("persons", [DataSourceColumn(k, k) for k in names]), names,
                          [dh.PartsKey(("NAME", -1, 0, 3), ("DOB", None, 0, 4)),
                           dh.PartsKey(("NAME", 0, 0, 2), ("DOB", None, 5, 10))])
for threads in os.environ.get("THREADS", "4,8,12,16").split(","):
    os.environ["DK_INGEST_THREADS"] = threads
    for rep in range(3):
        it = ingest.Interner()
        t0 = time.perf_counter()
        pk = src.pack(body, it)
        t1 = time.perf_counter()
        pk2 = src.pack(body, it)
        t2 = time.perf_counter()
        print(f"threads {threads:>3} rep {rep}: cold {1e3 * (t1 - t0):7.1f} ms  warm {1e3 * (t2 - t1):7.1f} ms",
              flush=True)
        pk.close()
        pk2.close()
        it.close()
