"""Lucene-compatible candidate generation, restated in Python (TEST INFRASTRUCTURE: the checker of
the GPU path's DK_CAND_LUCENE source; never imported by the product).

Follows the reference's IncrementalLuceneDatabase (src/main/java/io/sesam/dukemicroservice/):
  * findCandidateMatches (:459-492): BooleanQuery of MUST_NOT dukeGroupNo == g (linkage),
    MUST_NOT dukeDeleted == "true", and per lookup property, per value, the value's tokens as
    SHOULD TermQuerys (parseTokens :295-321 after escapeLucene :329-342); Lookup.REQUIRED
    (MUST clauses) and FUZZY_SEARCH are not restated;
  * doQuery (:377-414) with App.configureDatabase's defaults (App.java:550-563): max-search-
    hits 10 (any value <= 100: the first search's limit min(100, max) is final), keep hits
    while score >= min-relevance (0.9);
  * index (:505-575): every non-empty property value indexed ANALYZED with the same analyzer
    (no escaping at index time); ID / dataset / group / original-id NOT_ANALYZED.
[Lucene 4.x, recalled -- PARITY UNPINNED, Lucene is absent from /root/reference]:
  * StandardAnalyzer = StandardTokenizer (UAX#29 word boundaries; restated for U+0000-U+00FF,
    other code units are declined by the native path), LowerCaseFilter, StopFilter (English
    stop words);
  * DefaultSimilarity: idf = 1 + ln(maxDoc / (docFreq + 1)), queryNorm = 1/sqrt(sum over
    clauses of idf^2), clause weight = idf * queryNorm * idf, term score = sqrt(tf) * weight *
    decode(norm), norm byte = SmallFloat.floatToByte315(1/sqrt(#tokens)); float32 arithmetic
    except the per-document clause sum (double, in clause order: BooleanScorer's bucket) and
    its product with coord = overlap / #clauses;
  * collection statistics: by default those of a fully merged index (maxDoc = documents in
    the index: every live version, dukeDeleted ones included; superseded versions gone); with
    `in_stats` those of an unmerged one -- the superseded versions (deleted by ID on re-post,
    IncrementalLuceneDatabase.java:516-517, 578-590, never merged away: commit :146-165) still
    count in maxDoc and docFreq, but are never hits (liveDocs); ties by insertion order
    (doc id).
[Duke 1.2, recalled] lookup properties (ConfigurationImpl.findLookupProperties): the scored
properties sorted by <high> ascending; computeBayes over them from 0.5 until the result
reaches maybe-threshold (threshold when that is 0.0): that property and every later one.
"""
from __future__ import annotations

import math

import numpy as np

STOP_WORDS = frozenset(
    "a an and are as at be but by for if in into is it no not of on or such that the their "
    "then there these they this to was will with".split())

# UAX#29 word-break classes over Latin-1
_OTHER, _ALETTER, _NUMERIC, _MIDLETTER, _MIDNUMLET, _MIDNUM, _EXTENDNUMLET, _FORMAT, _NL = range(9)


def wb_class(c: int) -> int:
    if c in (0x0A, 0x0B, 0x0C, 0x0D, 0x85):
        return _NL
    if 0x30 <= c <= 0x39:
        return _NUMERIC
    if (0x41 <= c <= 0x5A) or (0x61 <= c <= 0x7A) or c in (0xAA, 0xB5, 0xBA) or \
            (0xC0 <= c <= 0xD6) or (0xD8 <= c <= 0xF6) or (0xF8 <= c <= 0xFF):
        return _ALETTER
    if c in (0x3A, 0xB7):
        return _MIDLETTER
    if c in (0x27, 0x2E):
        return _MIDNUMLET
    if c in (0x2C, 0x3B):
        return _MIDNUM
    if c == 0x5F:
        return _EXTENDNUMLET
    if c == 0xAD:
        return _FORMAT
    return _OTHER


def _lower(c: int) -> int:
    if 0x41 <= c <= 0x5A or 0xC0 <= c <= 0xD6 or 0xD8 <= c <= 0xDE:
        return c + 0x20
    return c


def tokenize(s: str):
    """StandardTokenizer (UAX#29) over a Latin-1 string: the word segments holding at least one
    ALetter or Numeric character; Format characters (soft hyphen) attach to their left
    neighbour and are kept in the token (WB4)."""
    cs = [ord(ch) for ch in s]
    if any(c > 0xFF for c in cs):
        raise ValueError("outside U+0000-U+00FF")
    n = len(cs)
    # WB4: the class a position contributes to the rules is that of its base character
    cls = [wb_class(c) for c in cs]
    out = []
    i = 0
    while i < n:
        # a segment starts at i; extend while no break
        j = i + 1
        while j < n and cls[j] == _FORMAT and cls[i] != _NL:
            j += 1
        while j < n:
            if not _joins(cls, i, j):
                break
            j += 1
            while j < n and cls[j] == _FORMAT:
                j += 1
        seg = cs[i:j]
        if any(cls[k] in (_ALETTER, _NUMERIC) for k in range(i, j)) and len(seg) <= 255:
            out.append("".join(chr(_lower(c)) for c in seg))
        i = j
    return out


def _base(cls, k, step):
    """Index of the nearest non-Format position from k in direction step (or -1 / len)."""
    while 0 <= k < len(cls) and cls[k] == _FORMAT:
        k += step
    return k


def _joins(cls, start, j):
    """No word break before position j (UAX#29 WB5-WB13b; WB4 skips Format characters)."""
    a = _base(cls, j - 1, -1)
    if a < start:
        return False
    A, B = cls[a], cls[j]
    if A == _NL or B == _NL:
        return False
    nxt = _base(cls, j + 1, 1)
    C = cls[nxt] if nxt < len(cls) else None
    prv = _base(cls, a - 1, -1) if a - 1 >= start else -1
    P = cls[prv] if prv >= start else None
    if A == _ALETTER and B == _ALETTER:                                            # WB5
        return True
    if A == _ALETTER and B in (_MIDLETTER, _MIDNUMLET) and C == _ALETTER:           # WB6
        return True
    if P == _ALETTER and A in (_MIDLETTER, _MIDNUMLET) and B == _ALETTER:           # WB7
        return True
    if A == _NUMERIC and B == _NUMERIC:                                            # WB8
        return True
    if A == _ALETTER and B == _NUMERIC:                                            # WB9
        return True
    if A == _NUMERIC and B == _ALETTER:                                            # WB10
        return True
    if P == _NUMERIC and A in (_MIDNUM, _MIDNUMLET) and B == _NUMERIC:              # WB11
        return True
    if A == _NUMERIC and B in (_MIDNUM, _MIDNUMLET) and C == _NUMERIC:              # WB12
        return True
    if A in (_ALETTER, _NUMERIC, _EXTENDNUMLET) and B == _EXTENDNUMLET:             # WB13a
        return True
    if A == _EXTENDNUMLET and B in (_ALETTER, _NUMERIC):                           # WB13b
        return True
    return False


def analyze(s: str):
    """StandardAnalyzer: tokens, lowercased, English stop words removed."""
    return [t for t in tokenize(s) if t not in STOP_WORDS]


_SPECIAL = set('*?!&()-+:"[]~{}^|')


def escape_lucene(q: str) -> str:
    """IncrementalLuceneDatabase.escapeLucene (:329-342): backslash before the query-syntax
    characters, then String.trim()."""
    out = "".join(("\\" + ch) if ch in _SPECIAL else ch for ch in q)
    a, b = 0, len(out)
    while a < b and ord(out[a]) <= 0x20:
        a += 1
    while b > a and ord(out[b - 1]) <= 0x20:
        b -= 1
    return out[a:b]


def query_tokens(value: str):
    """parseTokens(parent, field, value, required) (:295-321): the escaped value's tokens."""
    v = escape_lucene(value)
    return analyze(v) if v else []


# ---- similarity (float32 arithmetic) ------------------------------------------------------
F = np.float32


def float_to_byte315(f) -> int:
    bits = int(np.asarray(F(f)).view(np.int32))
    small = bits >> (24 - 3)
    if small <= ((63 - 15) << 3):
        return 0 if bits <= 0 else 1
    if small >= ((63 - 15) << 3) + 0x100:
        return 255
    return small - ((63 - 15) << 3)


def byte315_to_float(b: int):
    if b == 0:
        return F(0.0)
    bits = (b & 0xFF) << (24 - 3)
    bits += (63 - 15) << 24
    return np.asarray(np.int32(bits)).view(np.float32).item() * 1.0


def norm_byte(ntokens: int) -> int:
    """DefaultSimilarity.lengthNorm (boost 1) encoded: floatToByte315((float)(1/sqrt(n)))."""
    return float_to_byte315(F(1.0 / math.sqrt(ntokens)) if ntokens else F(np.inf))


def idf(df: int, max_doc: int):
    return F(math.log(max_doc / float(df + 1)) + 1.0)


def lookup_properties(props, threshold, maybe_threshold):
    """[Duke 1.2, recalled] ConfigurationImpl lookup properties: `props` = [(name, high, lookup)]
    of the scored properties (lookup: "default" / "true" / "false" / "required")."""
    cand = [p for p in props if p[2] != "false"]
    cand = sorted(cand, key=lambda p: p[1])            # HighComparator, stable
    limit = maybe_threshold if maybe_threshold != 0.0 else threshold
    prob, last = 0.5, -1
    for ix, p in enumerate(cand):
        if p[1] == 0.0:
            continue
        prob = (prob * p[1]) / ((prob * p[1]) + ((1.0 - prob) * (1.0 - p[1])))
        if prob >= limit:
            last = ix
            break
    out = [p[0] for p in cand[last:]] if last >= 0 else []
    for p in props:
        if p[2] in ("true", "required") and p[0] not in out:
            out.append(p[0])
    return out


class LuceneIndexRef:
    """The Lucene index of one pipeline, as the candidate source sees it."""

    def __init__(self, lookup_fields, max_hits=10, min_relevance=0.9, linkage=False):
        self.fields = list(lookup_fields)
        self.max_hits = max_hits
        self.min_relevance = F(min_relevance)
        self.linkage = linkage
        self.docs = []          # row -> dict or None (not in the index)

    def set_docs(self, values, in_index, deleted=None, group=None, in_stats=None):
        """values[f][row] (None = no value); in_index[row]: the row is a live version of an
        indexed record (superseded and transient rows are not); in_stats[row] (default
        in_index): the row counts in maxDoc / docFreq (unmerged: every version indexed)."""
        n = len(in_index)
        self.values = values
        self.in_index = np.asarray(in_index, bool)
        stats = self.in_index if in_stats is None else np.asarray(in_stats, bool)
        assert not (self.in_index & ~stats).any()
        self.deleted = np.zeros(n, bool) if deleted is None else np.asarray(deleted, bool)
        self.group = np.zeros(n, np.int64) if group is None else np.asarray(group, np.int64)
        self.max_doc = int(stats.sum())
        self.postings = [dict() for _ in self.fields]     # term -> {row: tf}
        self.norms = [dict() for _ in self.fields]
        for fi in range(len(self.fields)):
            for r in range(n):
                v = values[fi][r]
                if not stats[r] or v is None or v == "":
                    continue
                toks = analyze(v)
                self.norms[fi][r] = norm_byte(len(toks))
                for t in toks:
                    d = self.postings[fi].setdefault(t, {})
                    d[r] = d.get(r, 0) + 1

    def candidates(self, row):
        """findCandidateMatches(record of `row`): the hit rows in hit order."""
        clauses = []
        for fi in range(len(self.fields)):
            v = self.values[fi][row]
            if v is None:
                continue
            for t in query_tokens(v):
                clauses.append((fi, t))
        if not clauses:
            return []
        idfs = [idf(len(self.postings[fi].get(t, {})), self.max_doc) for fi, t in clauses]
        ssw = F(0.0)
        for w in idfs:
            ssw = F(ssw + F(w * w))
        qn = F(1.0 / math.sqrt(float(ssw)))
        if not np.isfinite(qn):
            qn = F(1.0)
        weights = [F(F(w * qn) * w) for w in idfs]
        coord = [F(k / F(len(clauses))) for k in range(len(clauses) + 1)]
        acc = {}
        for (fi, t), w in zip(clauses, weights):
            for r, tf in self.postings[fi].get(t, {}).items():
                s = F(F(F(math.sqrt(tf)) * w) * F(byte315_to_float(self.norms[fi][r])))
                a = acc.get(r)
                acc[r] = (float(s), 1) if a is None else (a[0] + float(s), a[1] + 1)
        hits = []
        g = self.group[row]
        for r, (s, k) in acc.items():
            if not self.in_index[r] or self.deleted[r] or (self.linkage and self.group[r] == g):
                continue
            hits.append((F(s * float(coord[k])), r))
        hits.sort(key=lambda h: (-float(h[0]), h[1]))
        out = []
        for s, r in hits[: self.max_hits]:
            if s >= self.min_relevance:
                out.append(r)
            else:
                break
        return out
