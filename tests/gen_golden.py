"""Generates tests/golden/*.jsonl from the pure-Python restatement oracle/duke_pyref.py.

The reference (sesam-duke-microservice) ships no golden vectors for this path and its
Duke 1.2 dependency is absent, so these fixtures pin the C oracle and the GPU path to an
independent restatement (PARITY UNPINNED against Duke itself).  Re-run with
`python tests/gen_golden.py` after a deliberate change to the restated semantics.
Strings are stored as lists of UTF-16 code units; floats as their repr and IEEE hex.
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import duke_pyref as R  # noqa: E402

OUT = os.path.join(HERE, "golden")


def fl(x):
    return {"repr": repr(x), "hex": float(x).hex()}


def rnd_str(rng, alpha, lo, hi):
    return "".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi)))


def string_cases(seed, n):
    rng = random.Random(seed)
    fixed = [("", ""), ("a", "b"), ("a", "a"), ("ab", "ba"), ("aab", "ab"), ("kitten", "sitting"),
             ("MARTHA", "MARHTA"), ("DWAYNE", "DUANE"), ("DIXON", "DICKSONX"), ("abc", ""),
             ("Norway", "Norwegian"), ("Oslo", "Olso"), ("ł\U0001F600a", "ła\U0001F600"),
             ("x" * 64, "x" * 63 + "y"), ("abcdefgh", "badcfehg"), ("a", "ab"), ("ab", "a"),
             ("a b c", "b c d e"), (" a  b ", "b a"), (" ", "  "), ("a a b", "a b"),
             ("12 main st.", "12 main street"), ("o'neil-smith", "oneil smith"), ("a\\b", "a/b"),
             ('"q"', "q")]
    out = list(fixed)
    alphas = ["ab", "abcd", "abcdefghijklmnopqrstuvwxyz", "ałé\U0001F600", "ab 1.-", "a b  "]
    for i in range(n):
        a = alphas[i % len(alphas)]
        out.append((rnd_str(rng, a, 0, 14), rnd_str(rng, a, 0, 14)))
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    cases = string_cases(1, 400)
    with open(os.path.join(OUT, "comparators.jsonl"), "w") as f:
        for s1, s2 in cases:
            u1, u2 = R.units(s1), R.units(s2)
            rec = {"s1": list(u1), "s2": list(u2),
                   "compact_distance": R.compact_distance(u1, u2),
                   "levenshtein": fl(R.levenshtein(u1, u2)) if (u1 or u2) else None,
                   "jarowinkler": fl(R.jarowinkler(u1, u2)),
                   "exact": fl(R.exact(u1, u2))}
            for q in (1, 2, 3):
                for form in (0, 1, 2):
                    rec[f"qgram_q{q}_f{form}"] = fl(R.qgram(u1, u2, q, form))
            rec["qgram_q2_f1_positional"] = fl(R.qgram(u1, u2, 2, 1, R.POSITIONAL))
            rec["qgram_q2_f1_ends"] = fl(R.qgram(u1, u2, 2, 1, R.ENDS))
            rec["qgram_q3_f2_ends"] = fl(R.qgram(u1, u2, 3, 2, R.ENDS))
            rec["weighted_levenshtein"] = fl(R.weighted_levenshtein(u1, u2))
            rec["dice_tokens"] = fl(R.token_set_similarity(u1, u2, False))
            rec["jaccard_tokens"] = fl(R.token_set_similarity(u1, u2, True))
            f.write(json.dumps(rec) + "\n")
    # long values for the long-value DP (WeightedLevenshtein, Levenshtein over 64 units)
    rng = random.Random(5)
    words = ["oslo", "bergen", "street", "42", "no.", "gate", "vei", "a/s", "-", "o'neil", "x"]
    with open(os.path.join(OUT, "long_values.jsonl"), "w") as f:
        for i in range(60):
            a = " ".join(rng.choice(words) for _ in range(rng.randint(1, 50)))[:256]
            b = list(a)
            for _ in range(rng.randint(0, 12)):
                if b and rng.random() < 0.5:
                    del b[rng.randrange(len(b))]
                else:
                    b.insert(rng.randrange(len(b) + 1), rng.choice("abc 1.-"))
            b = "".join(b)[:256] or "z"
            if i % 7 == 0:
                b = a[: max(1, len(a) // 2)]
            u1, u2 = R.units(a), R.units(b)
            f.write(json.dumps({"s1": list(u1), "s2": list(u2),
                                "compact_distance": R.compact_distance(u1, u2),
                                "levenshtein": fl(R.levenshtein(u1, u2)),
                                "weighted_levenshtein": fl(R.weighted_levenshtein(u1, u2))}) + "\n")
    nums = ["1", "2", "0", "-0", "0.0", "-3", "-4.5", "1e3", "1000", "abc", " 7 ", "7f", "NaN",
            "Infinity", "-Infinity", "0x1p3", "0x.8p1", "8", "1e", "", "1.", ".5", "0.5d",
            "3.3", "3.30", "+2", "1.e5", "1_0", "inf", "0x1", "1e-400", "1e400", "\t5\n"]
    with open(os.path.join(OUT, "numeric.jsonl"), "w") as f:
        for a in nums:
            v = R.parse_java_double(R.units(a))
            f.write(json.dumps({"parse": list(R.units(a)), "value": None if v is None else fl(v)}) + "\n")
        for a in nums:
            for b in nums[::3]:
                for mr in (0.0, 0.7):
                    f.write(json.dumps({"s1": list(R.units(a)), "s2": list(R.units(b)),
                                        "min_ratio": mr,
                                        "numeric": fl(R.numeric(R.units(a), R.units(b), mr))}) + "\n")
    rng = random.Random(3)
    with open(os.path.join(OUT, "bayes.jsonl"), "w") as f:
        pts = [0.0, 0.04, 0.09, 0.12, 0.5, 0.61, 0.73, 0.93, 1.0]
        pairs = [(a, b) for a in pts for b in pts] + [(rng.random(), rng.random()) for _ in range(100)]
        for a, b in pairs:
            f.write(json.dumps({"p1": fl(a), "p2": fl(b), "bayes": fl(R.compute_bayes(a, b))}) + "\n")
        # worked values of the default testdukeconfig.xml schema
        p = 0.5
        for h in (0.93, 0.73, 0.61):
            p = R.compute_bayes(p, h)
        f.write(json.dumps({"chain": [0.93, 0.73, 0.61], "bayes": fl(p)}) + "\n")
        p = 0.5
        for h in (0.93, 0.73, 0.12):
            p = R.compute_bayes(p, h)
        f.write(json.dumps({"chain": [0.93, 0.73, 0.12], "bayes": fl(p)}) + "\n")
    # end-to-end: small dedup with blocking, and a linkage case
    rng = random.Random(7)
    props = [{"comparator": R.JAROWINKLER, "low": 0.1, "high": 0.95},
             {"comparator": R.LEVENSHTEIN, "low": 0.2, "high": 0.8},
             {"comparator": R.NUMERIC, "low": 0.04, "high": 0.73}]
    with open(os.path.join(OUT, "e2e_small.jsonl"), "w") as f:
        for case in range(6):
            n = 40
            base = [rnd_str(rng, "abcde", 3, 8) for _ in range(12)]
            names, addrs, nums_, keys = [], [], [], [[], []]
            for i in range(n):
                b = rng.choice(base)
                nm = b if rng.random() < 0.6 else b[:-1] + rng.choice("abcde")
                names.append(nm)
                addrs.append(None if rng.random() < 0.1 else rnd_str(rng, "ab", 2, 6))
                nums_.append(str(rng.randint(1, 4)))
                keys[0].append(nm[:1])
                keys[1].append(nums_[-1])
            recs = [[R.units(names[i]), None if addrs[i] is None else R.units(addrs[i]),
                     R.units(nums_[i])] for i in range(n)]
            mode = "dedup" if case < 4 else "linkage"
            groups = [1 + (i % 2) for i in range(n)]
            deleted = [1 if rng.random() < 0.05 else 0 for _ in range(n)]
            kk = [[keys[0][i], keys[1][i]] for i in range(n)]
            out, scored = R.match(props, recs, kk, list(range(n)), 0.8, 0.6, mode=mode,
                                  groups=groups, deleted=deleted)
            f.write(json.dumps({"mode": mode, "props": props, "threshold": 0.8, "maybe": 0.6,
                                "names": names, "addrs": addrs, "nums": nums_, "keys": keys,
                                "groups": groups, "deleted": deleted, "pairs_scored": scored,
                                "links": [[q, c, fl(p), k] for q, c, p, k in out]}) + "\n")
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
