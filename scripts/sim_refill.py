"""Lane-utilisation model of the headline kernel's ADDRESS Levenshtein DP.

For a sample of configs[1] queries this computes, per owned candidate slot of the symmetric
schedule, the DP step at which compact_distance_pp's lane finishes (cutoff or last column),
then compares
  * the current schedule: one query per wave, 64 slots per wave, the wave runs until its
    slowest lane is done (padding lanes idle);
  * lane refill: one wave per query's whole owned list, a lane taking the next candidate
    when its DP ends, refilling at every G-th step when at least K lanes are idle, each
    refill costing `setup` column-equivalents (reset of the DP column, bias, lengths, first
    words).
Utilisation = useful lane-steps / (64 x wave steps).  Runs on CPU in a few minutes:
  python scripts/sim_refill.py [n_queries]
"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sesam-duke-microservice_amd"))
from dukehip import synth  # noqa: E402


def exit_step(s1, s2):
    """Step at which the lane of (query s1, candidate s2) ends in compact_distance_pp."""
    n1, n2 = len(s1), len(s2)
    if n1 == 0 or n2 == 0:
        return 0
    ln, mx = min(n1, n2), max(n1, n2)
    if 2 * ln <= mx or s1 == s2:  # decided before the DP (levenshtein_peq)
        return 0
    maxdist = ln >> 1
    R = (n1 + 1) // 2 * 2 if n1 <= 16 else ((n1 + 3) // 4 * 4 if n1 <= 32 else (n1 + 7) // 8 * 8)
    bottom = n1 > R // 2
    fin = n2 - 1 + (1 if bottom else 0)
    prev = list(range(n1 + 1))
    for j in range(n2):
        cur = [j + 1] + [0] * n1
        for i in range(1, n1 + 1):
            cost = 0 if s1[i - 1] == s2[j] else 1
            cur[i] = min(cur[i - 1], prev[i - 1], prev[i]) + cost
        if j >= 1 and min(cur[1:]) > maxdist:  # seen one step later in the packed DP
            return min(j + 1 + (1 if bottom else 0), fin)
        prev = cur
    return fin


def main():
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 150
    n = 1000000
    p = synth.persons(n - int(n * 0.3), int(n * 0.3))
    keys = synth.keys_config2(p)
    addr = p["address"]
    buckets = [collections.defaultdict(list) for _ in keys]
    for k, kk in enumerate(keys):
        for i, v in enumerate(kk):
            buckets[k][v].append(i)
    rng = np.random.default_rng(5)
    lists = []
    for q in rng.choice(n, nq, replace=False):
        seen, owned = set(), []
        for k in range(len(keys)):
            for c in buckets[k][keys[k][q]]:
                if c > q:  # the query owns the candidates after it (symmetric schedule)
                    owned.append(0 if c in seen else exit_step(addr[q], addr[c]))
                seen.add(c)
        lists.append(owned)
    work = sum(sum(w) for w in lists)
    cur = sum(max(w[i:i + 64]) * 64 for w in lists for i in range(0, len(w), 64))
    pairs = sum(len(w) for w in lists)
    slots = sum((len(w) + 63) // 64 * 64 for w in lists)
    print(f"{nq} queries, {pairs} owned pairs, {slots} slots: current utilisation {work / cur:.3f}")
    for G in (1, 2, 4):
        for setup in (0.0, 0.5, 1.0):
            for K in (1, 8, 16):
                t_total = 0
                for w in lists:
                    if not w:
                        continue
                    queue = collections.deque(w)
                    rem = [queue.popleft() if queue else None for _ in range(64)]
                    t = 0
                    while any(r is not None for r in rem):
                        t += G
                        for lane in range(64):
                            if rem[lane] is not None:
                                rem[lane] -= G
                                if rem[lane] <= 0:
                                    rem[lane] = None
                        idle = sum(1 for r in rem if r is None)
                        if queue and idle >= min(K, len(queue)):
                            for lane in range(64):
                                if rem[lane] is None and queue:
                                    rem[lane] = queue.popleft()
                            t += setup
                    t_total += t * 64
                print(f"refill G={G} setup={setup} K={K}: utilisation {work / t_total:.3f}")


if __name__ == "__main__":
    main()
