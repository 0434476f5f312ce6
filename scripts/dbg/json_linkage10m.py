"""Debug: configs[2] json leg at 10M alone (no other engine on the GPU)."""
import sys, time
import numpy as np
sys.path[:0] = ['sesam-duke-microservice_amd', '.']
import torch
import bench
sys.argv = ['bench.py', '--workload', 'linkage', '--records', sys.argv[1] if len(sys.argv) > 1 else '10000000']
a = bench.parse()
t = time.time()
w = bench.build_workload(a)
w["nkeys"] = len(w["keys"])
n = a.records
print("synth", time.time() - t, flush=True)
out = bench.json_batch(w, n, np.arange(n, 2 * n), 0, torch)
print(out, flush=True)
