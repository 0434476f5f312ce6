"""Debug helper: all-pairs of a few values through the GPU and the oracle, printing the
pairs whose probabilities differ (test infrastructure; uses oracle/ as the checker)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sesam-duke-microservice_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import test_gpu_parity as T  # noqa: E402

cmp = int(sys.argv[1])
vals = sys.argv[2:]
if vals and vals[0].startswith("families:"):   # families:lo:hi  (test_weighted_levenshtein_allpairs)
    import random
    lo, hi = map(int, vals[0].split(":")[1:])
    rng = random.Random(lo * 1000 + hi)
    vals = T.families(rng, 20, 5, T.WL_ALPHA, lo, hi, max(2, hi // 8), 256)
res, ref = T.allpairs_single({"comparator": cmp, "low": 0.0, "high": 1.0}, vals)
g = {(int(q), int(c)): p for q, c, p in zip(res.query, res.candidate, res.prob)}
r = {(int(q), int(c)): p for q, c, p in zip(ref["query"], ref["candidate"], ref["prob"])}
bad = 0
for k in sorted(set(g) | set(r)):
    a, b = g.get(k), r.get(k)
    if a != b:
        bad += 1
        print(repr(vals[k[0]]), repr(vals[k[1]]), "gpu", a, "oracle", b)
print("pairs", len(r), "bad", bad)
