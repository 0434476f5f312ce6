"""Pure-Python restatement of Duke 1.2's scoring path — TEST INFRASTRUCTURE ONLY.

Used only to generate the golden fixtures under tests/golden/ (tests/gen_golden.py) and
inside tests as a second, independent restatement next to the C oracle
(oracle/duke_oracle.c).  Nothing in the product imports it.

PARITY UNPINNED against Duke itself: the algorithms live in the third-party jar
no.priv.garshol.duke:duke:1.2 (/root/reference/pom.xml:32-36), which is absent; the
reference ships no known-answer tests for this path (src/test/.../AppTest.java:34-37).
Functions follow the Duke 1.2 sources as recalled.

Strings are sequences of UTF-16 code units (Java ``char``); use :func:`units`.
"""
from __future__ import annotations

import math
import re

LEVENSHTEIN, JAROWINKLER, QGRAM, EXACT, NUMERIC, WEIGHTED_LEVENSHTEIN = 1, 2, 3, 4, 5, 6
DICE_TOKENS, JACCARD_TOKENS, GEOPOSITION = 7, 8, 9
OVERLAP, JACCARD, DICE = 0, 1, 2
BASIC, POSITIONAL, ENDS = 0, 1, 2
_CARET, _DOLLAR = ord("^"), ord("$")


def units(s: str) -> tuple:
    """Java String -> tuple of UTF-16 code units (surrogate pairs count as two)."""
    b = s.encode("utf-16-le", "surrogatepass")
    return tuple(int.from_bytes(b[i:i + 2], "little") for i in range(0, len(b), 2))


def compact_distance(s1, s2) -> int:
    """[Duke 1.2] Levenshtein.compactDistance (cost added to all three neighbours)."""
    if len(s1) == 0:
        return len(s2)
    if len(s2) == 0:
        return len(s1)
    maxdist = min(len(s1), len(s2)) // 2
    m = len(s1)
    col = [0] * (m + 1)
    col[0] = 1
    for i in range(1, m + 1):
        col[i] = min(col[i - 1], i - 1) + (0 if s1[i - 1] == s2[0] else 1)
    above = 0
    for j in range(1, len(s2)):
        above = j + 1
        smallest = 2 * m
        for i in range(1, m + 1):
            v = min(above, col[i - 1], col[i]) + (0 if s1[i - 1] == s2[j] else 1)
            col[i - 1] = above
            above = v
            smallest = min(smallest, v)
        col[m] = above
        if smallest > maxdist:
            return smallest
    return above


def levenshtein(s1, s2) -> float:
    """[Duke 1.2] Levenshtein.compare — divides by the SHORTER length."""
    n, mx = min(len(s1), len(s2)), max(len(s1), len(s2))
    ratio = n / mx if mx else float("nan")
    if ratio <= 0.5:
        return 0.0
    if n == mx and tuple(s1) == tuple(s2):
        return 1.0
    d = min(compact_distance(s1, s2), n)
    return 1.0 - (d / n)


def jarowinkler(s1, s2) -> float:
    """[Duke 1.2] JaroWinkler.similarity (first match in window, t not halved)."""
    if tuple(s1) == tuple(s2):
        return 1.0
    if len(s1) > len(s2):
        s1, s2 = s2, s1
    maxdist = len(s2) // 2
    c = t = 0
    prev = -1
    for i, ch in enumerate(s1):
        for j in range(max(0, i - maxdist), min(len(s2), i + maxdist)):
            if s2[j] == ch:
                c += 1
                if prev != -1 and j < prev:
                    t += 1
                prev = j
                break
    if c == 0:
        return 0.0
    score = ((c / len(s1)) + (c / len(s2)) + ((c - t) / c)) / 3.0
    p = 0
    last = min(4, len(s1))
    while p < last and s1[p] == s2[p]:
        p += 1
    score += (p * (1 - score)) / 10
    return score


def qgrams(s, q, tokenizer=BASIC) -> set:
    """QGramComparator.Tokenizer: BASIC substrings; POSITIONAL substring + index;
    ENDS [recalled, low confidence] BASIC plus the start gram "^" + s[0:q-1] and the end
    gram s[n-q+1:] + "$" — i.e. the q-grams of "^" + s + "$" (HashSet<String>, so marker
    grams may coincide with real ones)."""
    if tokenizer == ENDS:
        s = (_CARET,) + tuple(s) + (_DOLLAR,)
    out = set()
    for ix in range(0, len(s) - q + 1):
        g = tuple(s[ix:ix + q])
        out.add((g, ix) if tokenizer == POSITIONAL else g)
    return out


def qgram(s1, s2, q=2, formula=OVERLAP, tokenizer=BASIC) -> float:
    """[Duke 1.2] QGramComparator.compare + Formula.compute."""
    if tuple(s1) == tuple(s2):
        return 1.0
    g1, g2 = qgrams(s1, q, tokenizer), qgrams(s2, q, tokenizer)
    if not g1 or not g2:
        return 0.0
    common = len(g1 & g2)
    if formula == JACCARD:
        return common / (len(g1) + len(g2) - common)
    if formula == DICE:
        return (2.0 * common) / (len(g1) + len(g2))
    return common / min(float(len(g1)), float(len(g2)))


def exact(s1, s2) -> float:
    return 1.0 if tuple(s1) == tuple(s2) else 0.0


def _wl_weight(ch):
    """[Duke 1.2, recalled] WeightedLevenshtein.DefaultWeightEstimator: letters 1.0,
    digits 2.0, punctuation / space 0.1, anything else 1.0."""
    if ord("a") <= ch <= ord("z") or ord("A") <= ch <= ord("Z"):
        return 1.0
    if ord("0") <= ch <= ord("9"):
        return 2.0
    if chr(ch) in " '.-/\\,\"":
        return 0.1
    return 1.0


def weighted_distance(s1, s2):
    """[Duke 1.2, recalled] WeightedLevenshtein.distance, literally: one flat array
    addressed ix1 + s1len * ix2 (stride s1len, not s1len + 1), column init then row init,
    s1-major loop nest."""
    n1, n2 = len(s1), len(s2)
    if n1 == 0:
        return sum_weights(s2)
    if n2 == 0:
        return sum_weights(s1)
    m = [0.0] * ((n1 + 1) * (n2 + 1))
    for col in range(n2 + 1):
        m[col * n1] = float(col)
    for row in range(n1 + 1):
        m[row] = float(row)
    for ix1 in range(n1):
        ch1 = s1[ix1]
        for ix2 in range(n2):
            ch2 = s2[ix2]
            cost = 0.0 if ch1 == ch2 else max(_wl_weight(ch1), _wl_weight(ch2))
            left = m[ix1 + (ix2 + 1) * n1] + _wl_weight(ch1)
            above = m[ix1 + 1 + ix2 * n1] + _wl_weight(ch2)
            aboveleft = m[ix1 + ix2 * n1] + cost
            m[ix1 + 1 + (ix2 + 1) * n1] = min(left, min(above, aboveleft))
    return m[n1 + n2 * n1]


def sum_weights(s):
    e = 0.0
    for ch in s:
        e += _wl_weight(ch)
    return e


def weighted_levenshtein(s1, s2) -> float:
    """[Duke 1.2, recalled] WeightedLevenshtein.compare: 1 - dist / maxlen, 0 if dist >
    maxlen."""
    if tuple(s1) == tuple(s2):
        return 1.0
    dist = weighted_distance(s1, s2)
    maxlen = float(max(len(s1), len(s2)))
    if dist > maxlen:
        return 0.0
    return 1.0 - (dist / maxlen)


def split_tokens(s):
    """[Duke 1.2, recalled] utils.StringUtils.split: maximal runs of non-' ' units."""
    out, cur = [], []
    for ch in s:
        if ch == 0x20:
            if cur:
                out.append(tuple(cur))
            cur = []
        else:
            cur.append(ch)
    if cur:
        out.append(tuple(cur))
    return out


def token_set_similarity(s1, s2, jaccard):
    """[Duke 1.2, recalled, low confidence] DiceCoefficientComparator /
    JaccardIndexComparator with the default ExactComparator sub-comparator: t1 = the
    token list with fewer tokens (s1 on a tie); per t1 token the best sub-comparator score
    against t2; Dice = 2*sum / (|t1|+|t2|), Jaccard = sum / (|t1|+|t2| - sum) with the
    union reduced token by token."""
    if tuple(s1) == tuple(s2):
        return 1.0
    t1, t2 = split_tokens(s1), split_tokens(s2)
    if len(t1) > len(t2):
        t1, t2 = t2, t1
    total = 0.0
    union = float(len(t1) + len(t2))
    for a in t1:
        highest = 0.0
        for b in t2:
            highest = max(highest, exact(a, b))
        total += highest
        union -= highest
    if jaccard:
        return _div(total, union)
    return _div(total * 2, float(len(t1) + len(t2)))


def _div(num, den):
    if den == 0.0:
        return math.nan if num == 0.0 else math.copysign(math.inf, num)
    return num / den


_DEC = re.compile(r"^[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?[fFdD]?$")
_HEX = re.compile(r"^([+-]?)0[xX]([0-9a-fA-F]*)(?:\.([0-9a-fA-F]*))?[pP]([+-]?\d+)[fFdD]?$")


def parse_java_double(s):
    """java.lang.Double.parseDouble on code units; None for NumberFormatException."""
    a, b = 0, len(s)
    while a < b and s[a] <= 0x20:
        a += 1
    while b > a and s[b - 1] <= 0x20:
        b -= 1
    if a == b or any(u >= 0x80 for u in s[a:b]):
        return None
    t = "".join(chr(u) for u in s[a:b])
    body = t[1:] if t[:1] in "+-" else t
    neg = t.startswith("-")
    if body == "NaN":
        return float("nan")
    if body == "Infinity":
        return -math.inf if neg else math.inf
    m = _HEX.match(t)
    if m:
        ip, fp, ex = m.group(2), m.group(3) or "", m.group(4)
        if not ip and not fp:
            return None
        v = float.fromhex(f"{m.group(1)}0x{ip or '0'}.{fp or '0'}p{ex}")
        return v
    if _DEC.match(t):
        t2 = t[:-1] if t[-1] in "fFdD" else t
        return float(t2)
    return None


def numeric(s1, s2, min_ratio=0.0) -> float:
    """[Duke 1.2] NumericComparator.compare."""
    d1 = parse_java_double(s1)
    d2 = parse_java_double(s2)
    if d1 is None or d2 is None:
        return 0.5
    if d1 == 0.0 and d2 == 0.0:
        return 1.0
    if d2 < d1:
        d1, d2 = d2, d1
    try:
        ratio = d1 / d2
    except ZeroDivisionError:  # IEEE: x/0 -> +-inf, 0/0 -> nan
        ratio = math.nan if d1 == 0.0 or d1 != d1 else math.copysign(math.inf, d1) * math.copysign(1.0, d2)
    if ratio < min_ratio:
        return 0.0
    return ratio


def geoposition(s1, s2, max_distance) -> float:
    """[Duke 1.2, recalled, low confidence; parity unpinned] GeopositionComparator.compare:
    Geoposition.parse ("lat,lng" split at the first ','; Double.parseDouble each half;
    no ',' raises), haversine distance on a 6371000 m sphere with Java 8's Math.toRadians
    (angdeg / 180.0 * PI); unparsable -> 0.5; dist > max-distance -> 0.0; else
    ((1 - dist / max) * 0.5) + 0.5."""
    pos = []
    for s in (s1, s2):   # code units (or a str)
        u = [ord(ch) for ch in s] if isinstance(s, str) else list(s)
        if 0x2C not in u:
            raise ValueError(f"no comma in position {s!r}")
        c = u.index(0x2C)
        la, ln = parse_java_double(u[:c]), parse_java_double(u[c + 1:])
        if la is None or ln is None:
            return 0.5
        pos.append((la, ln))
    (la1, ln1), (la2, ln2) = pos
    lat1, lat2 = la1 / 180.0 * math.pi, la2 / 180.0 * math.pi
    dlat, dlng = (la2 - la1) / 180.0 * math.pi, (ln2 - ln1) / 180.0 * math.pi
    sl, sg = math.sin(dlat / 2), math.sin(dlng / 2)
    a = sl * sl + sg * sg * math.cos(lat1) * math.cos(lat2)
    dist = 6371000.0 * (2 * math.atan2(math.sqrt(a), math.sqrt(1 - a)))
    if dist > max_distance:
        return 0.0
    return ((1.0 - (dist / max_distance)) * 0.5) + 0.5


# --- RecordImpl's HashMap iteration order (SURVEY a-7; Processor.compare visits r1's map) ---
# Simulated as java.util.HashMap runs it (an independent restatement of the bucket-sort in
# dukehip/config.py): a table of per-bucket lists, puts appended at the bucket's tail, resize
# doubling and splitting each bucket into lo/hi lists that keep their order.  WHICH
# construction Duke's RecordImpl uses is unpinned (its source is absent): "incremental"
# (`new HashMap()` + one put per key) or "copy_jdk8" (`new HashMap(m)` of such a map on JDK
# 8..18: table sized tableSizeFor((int)(s / 0.75f + 1)), entries in m's iteration order).

def java_string_hashcode(s):
    h = 0
    for u in units(s):
        h = (31 * h + u) & 0xFFFFFFFF
    return h


class JavaHashMapOrder:
    def __init__(self, initial_threshold=0):
        self.table = None
        self.size = 0
        self.threshold = initial_threshold    # HashMap(int)/HashMap(Map): next table size

    def _resize(self):
        if self.table is None:
            cap = self.threshold if self.threshold > 0 else 16
            self.table = [[] for _ in range(cap)]
        else:
            old = self.table
            cap = 2 * len(old)
            self.table = [[] for _ in range(cap)]
            for j, b in enumerate(old):
                for k in b:                    # lo stays at j, hi moves to j + old cap
                    self.table[self._spread(k) & (cap - 1)].append(k)
        self.threshold = int(len(self.table) * 0.75)

    @staticmethod
    def _spread(k):
        h = java_string_hashcode(k)
        return h ^ (h >> 16)

    def put(self, k):
        if self.table is None:
            self._resize()
        b = self.table[self._spread(k) & (len(self.table) - 1)]
        if k in b:
            return
        b.append(k)
        self.size += 1
        if self.size > self.threshold:
            self._resize()

    def keys(self):
        return [k for b in (self.table or []) for k in b]


def _float32(x):
    import struct
    return struct.unpack("f", struct.pack("f", x))[0]


def record_map_order(keys, construction="incremental"):
    """Iteration order of a record map whose keys were put in `keys` order."""
    m = JavaHashMapOrder()
    for k in keys:
        m.put(k)
    if construction == "incremental":
        return m.keys()
    if construction == "copy_jdk8":
        t = int(_float32(_float32(float(len(keys))) / _float32(0.75)) + 1.0)
        cap = 1
        while cap < t:
            cap *= 2
        c = JavaHashMapOrder(cap if keys else 0)
        for k in m.keys():
            c.put(k)
        return c.keys()
    raise ValueError(construction)


def java_max(a, b):
    if a != a:
        return a
    if b != b:
        return b
    if a == 0.0 and b == 0.0:
        return b if math.copysign(1.0, a) < 0 else a
    return a if a >= b else b


def compute_bayes(p1, p2):
    """[Duke 1.2] Utils.computeBayes."""
    num = p1 * p2
    den = num + ((1.0 - p1) * (1.0 - p2))
    if den == 0.0:
        return math.nan if num == 0.0 else math.copysign(math.inf, num)
    return num / den


def property_compare(prop, v1, v2):
    """[Duke 1.2] PropertyImpl.compare.  prop: dict(comparator, low, high, ...)."""
    c = prop["comparator"]
    if c == LEVENSHTEIN:
        sim = levenshtein(v1, v2)
    elif c == JAROWINKLER:
        sim = jarowinkler(v1, v2)
    elif c == QGRAM:
        sim = qgram(v1, v2, prop.get("q", 2), prop.get("formula", OVERLAP), prop.get("tokenizer", BASIC))
    elif c == EXACT:
        sim = exact(v1, v2)
    elif c == NUMERIC:
        sim = numeric(v1, v2, prop.get("min_ratio", 0.0))
    elif c == WEIGHTED_LEVENSHTEIN:
        sim = weighted_levenshtein(v1, v2)
    elif c in (DICE_TOKENS, JACCARD_TOKENS):
        sim = token_set_similarity(v1, v2, c == JACCARD_TOKENS)
    elif c == GEOPOSITION:
        sim = geoposition(v1, v2, prop.get("min_ratio", 0.0))
    else:
        return 0.5
    if sim < 0.5:
        return prop["low"]
    return ((prop["high"] - 0.5) * (sim * sim)) + 0.5


def compare_records(props, r1, r2):
    """[Duke 1.2] Processor.compare.  r1/r2: list (per property, schema order) of a
    code-unit tuple or None (no value)."""
    prob = 0.5
    for i, prop in enumerate(props):
        v1, v2 = r1[i], r2[i]
        if v1 is None or v2 is None:
            continue
        high = 0.0
        if len(v1) and len(v2):
            high = java_max(high, property_compare(prop, v1, v2))
        prob = compute_bayes(prob, high)
    return prob


def match(props, records, keys, queries, threshold, maybe=0.0, mode="dedup",
          idents=None, groups=None, deleted=None):
    """Processor.deduplicate's match loop with exact-key blocking (SURVEY §8a-5 build
    contract).  records: list of per-property values; keys: per record list of key
    strings (tuples).  Returns (list of (q, c, prob, kind), pairs_scored)."""
    n = len(records)
    idents = idents if idents is not None else list(range(n))
    out, scored = [], 0
    for q in queries:
        cands = []
        if mode == "allpairs":
            cands = list(range(n))
        else:
            seen = set()
            for k in range(len(keys[q])):
                for c in range(n):
                    if keys[c][k] == keys[q][k] and c not in seen:
                        seen.add(c)
                        cands.append(c)
        for c in cands:
            if idents[c] == idents[q] or (deleted and deleted[c]):
                continue
            if mode == "linkage" and groups[c] == groups[q]:
                continue
            p = compare_records(props, records[q], records[c])
            scored += 1
            if p > threshold:
                out.append((q, c, p, 1))
            elif maybe != 0.0 and p > maybe:
                out.append((q, c, p, 2))
    return out, scored
