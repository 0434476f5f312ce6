"""ctypes binding to the C oracle (oracle/duke_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline.  PARITY UNPINNED against Duke
itself (see duke_oracle.h).  The packing here is deliberately independent of the
product's packer: every string is stored as UTF-16 code units.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libduke_oracle.so")

MODE = {"dedup": 0, "linkage": 1, "allpairs": 2}


class Prop(C.Structure):
    _fields_ = [("comparator", C.c_int), ("low", C.c_double), ("high", C.c_double),
                ("q", C.c_int), ("formula", C.c_int), ("tokenizer", C.c_int),
                ("min_ratio", C.c_double)]


class Schema(C.Structure):
    _fields_ = [("nprops", C.c_int), ("props", C.POINTER(Prop)), ("threshold", C.c_double),
                ("maybe_threshold", C.c_double), ("mode", C.c_int), ("nkeys", C.c_int),
                ("norders", C.c_int), ("orders", C.POINTER(C.c_int))]


class Table(C.Structure):
    _fields_ = [("n", C.c_uint64), ("ident", C.c_void_p), ("group", C.c_void_p),
                ("deleted", C.c_void_p), ("alive", C.c_void_p),
                ("off", C.POINTER(C.c_void_p)), ("chars", C.POINTER(C.c_void_p)),
                ("present", C.POINTER(C.c_void_p)), ("key_off", C.POINTER(C.c_void_p)),
                ("key_chars", C.POINTER(C.c_void_p)), ("oclass", C.c_void_p)]


class Result(C.Structure):
    _fields_ = [("n", C.c_uint64), ("query", C.POINTER(C.c_uint32)),
                ("candidate", C.POINTER(C.c_uint32)), ("prob", C.POINTER(C.c_double)),
                ("kind", C.POINTER(C.c_uint8)), ("pairs_scored", C.c_uint64),
                ("ms_index", C.c_double), ("ms_score", C.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        u16p = C.POINTER(C.c_uint16)
        for name in ("dko_levenshtein", "dko_jarowinkler", "dko_exact", "dko_weighted_levenshtein"):
            f = getattr(L, name)
            f.restype = C.c_double
            f.argtypes = [u16p, C.c_int, u16p, C.c_int]
        L.dko_compact_distance.restype = C.c_int
        L.dko_compact_distance.argtypes = [u16p, C.c_int, u16p, C.c_int]
        L.dko_token_similarity.restype = C.c_double
        L.dko_token_similarity.argtypes = [u16p, C.c_int, u16p, C.c_int, C.c_int]
        L.dko_qgram.restype = C.c_double
        L.dko_qgram.argtypes = [u16p, C.c_int, u16p, C.c_int, C.c_int, C.c_int, C.c_int]
        L.dko_numeric.restype = C.c_double
        L.dko_numeric.argtypes = [u16p, C.c_int, u16p, C.c_int, C.c_double]
        L.dko_geoposition.restype = C.c_double
        L.dko_geoposition.argtypes = [u16p, C.c_int, u16p, C.c_int, C.c_double]
        L.dko_parse_java_double.restype = C.c_int
        L.dko_parse_java_double.argtypes = [u16p, C.c_int, C.POINTER(C.c_double)]
        L.dko_compute_bayes.restype = C.c_double
        L.dko_compute_bayes.argtypes = [C.c_double, C.c_double]
        L.dko_java_max.restype = C.c_double
        L.dko_java_max.argtypes = [C.c_double, C.c_double]
        L.dko_property_compare.restype = C.c_double
        L.dko_property_compare.argtypes = [C.POINTER(Prop), u16p, C.c_int, u16p, C.c_int]
        L.dko_compare_rows.restype = C.c_double
        L.dko_compare_rows.argtypes = [C.POINTER(Schema), C.POINTER(Table), C.c_uint32, C.c_uint32]
        L.dko_match.restype = C.c_int
        L.dko_match.argtypes = [C.POINTER(Schema), C.POINTER(Table), C.POINTER(C.c_uint32),
                                C.c_uint64, C.c_int, C.POINTER(Result)]
        L.dko_free_result.restype = None
        L.dko_free_result.argtypes = [C.POINTER(Result)]
        _lib = L
    return _lib


def _u16(units):
    a = (C.c_uint16 * max(1, len(units)))(*units)
    return a, len(units)


def _units(s):
    if isinstance(s, str):
        b = s.encode("utf-16-le", "surrogatepass")
        return np.frombuffer(b, dtype=np.uint16)
    return np.asarray(s, dtype=np.uint16)


def _call2(name, s1, s2, *extra):
    a, na = _u16(list(_units(s1)))
    b, nb = _u16(list(_units(s2)))
    return getattr(lib(), name)(a, na, b, nb, *extra)


def compact_distance(s1, s2):
    return _call2("dko_compact_distance", s1, s2)


def levenshtein(s1, s2):
    return _call2("dko_levenshtein", s1, s2)


def jarowinkler(s1, s2):
    return _call2("dko_jarowinkler", s1, s2)


def qgram(s1, s2, q=2, formula=0, tokenizer=0):
    return _call2("dko_qgram", s1, s2, q, formula, tokenizer)


def exact(s1, s2):
    return _call2("dko_exact", s1, s2)


def numeric(s1, s2, min_ratio=0.0):
    return _call2("dko_numeric", s1, s2, min_ratio)


def geoposition(s1, s2, max_distance):
    return _call2("dko_geoposition", s1, s2, max_distance)


def weighted_levenshtein(s1, s2):
    return _call2("dko_weighted_levenshtein", s1, s2)


def token_similarity(s1, s2, jaccard):
    return _call2("dko_token_similarity", s1, s2, 1 if jaccard else 0)


def parse_java_double(s):
    a, n = _u16(list(_units(s)))
    out = C.c_double()
    rc = lib().dko_parse_java_double(a, n, C.byref(out))
    return None if rc != 0 else out.value


def compute_bayes(p1, p2):
    return lib().dko_compute_bayes(p1, p2)


def property_compare(prop: dict, v1, v2):
    p = Prop(prop["comparator"], prop["low"], prop["high"], prop.get("q", 2),
             prop.get("formula", 0), prop.get("tokenizer", 0), prop.get("min_ratio", 0.0))
    a, na = _u16(list(_units(v1)))
    b, nb = _u16(list(_units(v2)))
    return lib().dko_property_compare(C.byref(p), a, na, b, nb)


class OracleTable:
    """Column-packs records for the oracle.  values[p][r] is a str or None; keys[k][r]
    a str.  All strings stored as UTF-16 code units."""

    def __init__(self, props, values, keys=(), ident=None, group=None, deleted=None,
                 alive=None, threshold=0.9, maybe=0.0, mode="dedup", orders=None, oclass=None):
        """orders: per order class the visiting order of the props (indices); oclass: per
        record its class (Processor.compare follows the query record's HashMap order)."""
        n = len(values[0]) if values else len(keys[0])
        self.n = n
        self._keep = []
        self.props = (Prop * max(1, len(props)))()
        for i, pr in enumerate(props):
            self.props[i] = Prop(pr["comparator"], pr["low"], pr["high"], pr.get("q", 2),
                                 pr.get("formula", 0), pr.get("tokenizer", 0),
                                 pr.get("min_ratio", 0.0))
        self.schema = Schema(len(props), self.props, threshold, maybe, MODE[mode], len(keys))
        if orders:
            flat = (C.c_int * (len(orders) * len(props)))(*[int(x) for o in orders for x in o])
            self._orders = flat
            self.schema.norders = len(orders)
            self.schema.orders = flat

        def pack(col):
            if all(v is not None for v in col):
                try:  # fast path: Latin-1 strings
                    enc = [v.encode("latin-1") for v in col]
                    lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=n)
                    offs = np.zeros(n + 1, dtype=np.uint32)
                    np.cumsum(lens, out=offs[1:])
                    chars = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).astype(np.uint16)
                    pres = np.ones(n, dtype=np.uint8)
                    self._keep += [offs, chars, pres]
                    return offs, chars, pres
                except (UnicodeEncodeError, AttributeError):
                    pass
            offs = np.zeros(n + 1, dtype=np.uint32)
            parts = []
            pres = np.zeros(n, dtype=np.uint8)
            for r, v in enumerate(col):
                u = _units(v) if v is not None else np.zeros(0, np.uint16)
                pres[r] = v is not None
                parts.append(u)
                offs[r + 1] = offs[r] + len(u)
            chars = np.concatenate(parts) if parts else np.zeros(1, np.uint16)
            if chars.size == 0:
                chars = np.zeros(1, np.uint16)
            chars = np.ascontiguousarray(chars, dtype=np.uint16)
            self._keep += [offs, chars, pres]
            return offs, chars, pres

        P = len(values)
        self.off = (C.c_void_p * max(1, P))()
        self.chars = (C.c_void_p * max(1, P))()
        self.present = (C.c_void_p * max(1, P))()
        for p in range(P):
            o, c, pr = pack(values[p])
            self.off[p], self.chars[p], self.present[p] = o.ctypes.data, c.ctypes.data, pr.ctypes.data
        K = len(keys)
        self.key_off = (C.c_void_p * max(1, K))()
        self.key_chars = (C.c_void_p * max(1, K))()
        for k in range(K):
            o, c, _ = pack(keys[k])
            self.key_off[k], self.key_chars[k] = o.ctypes.data, c.ctypes.data

        def arr(x, dt):
            if x is None:
                return None
            a = np.ascontiguousarray(np.asarray(x, dtype=dt))
            self._keep.append(a)
            return a.ctypes.data

        ident = np.arange(n, dtype=np.uint64) if ident is None else ident
        self.table = Table(n, arr(ident, np.uint64), arr(group, np.uint8), arr(deleted, np.uint8),
                           arr(alive, np.uint8), self.off, self.chars, self.present,
                           self.key_off, self.key_chars, arr(oclass, np.uint8))

    @classmethod
    def from_packed(cls, props, columns, keys, ident, group=None, threshold=0.9, maybe=0.0,
                    mode="dedup"):
        """A table from already-packed columns (full-size tests): columns[p] / keys[k] =
        (offsets uint32 [n+1], UTF-16 units uint16), every value present."""
        self = cls.__new__(cls)
        n = len(ident)
        self.n = n
        self._keep = []
        self.props = (Prop * max(1, len(props)))()
        for i, pr in enumerate(props):
            self.props[i] = Prop(pr["comparator"], pr["low"], pr["high"], pr.get("q", 2),
                                 pr.get("formula", 0), pr.get("tokenizer", 0),
                                 pr.get("min_ratio", 0.0))
        self.schema = Schema(len(props), self.props, threshold, maybe, MODE[mode], len(keys))

        def keep(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            self._keep.append(a)
            return a.ctypes.data

        pres = np.ones(n, np.uint8)
        self.off = (C.c_void_p * max(1, len(columns)))()
        self.chars = (C.c_void_p * max(1, len(columns)))()
        self.present = (C.c_void_p * max(1, len(columns)))()
        for p, (o, u) in enumerate(columns):
            self.off[p], self.chars[p] = keep(o, np.uint32), keep(u, np.uint16)
            self.present[p] = keep(pres, np.uint8)
        self.key_off = (C.c_void_p * max(1, len(keys)))()
        self.key_chars = (C.c_void_p * max(1, len(keys)))()
        for k, (o, u) in enumerate(keys):
            self.key_off[k], self.key_chars[k] = keep(o, np.uint32), keep(u, np.uint16)
        self.table = Table(n, keep(ident, np.uint64), None if group is None else keep(group, np.uint8),
                           None, None, self.off, self.chars, self.present, self.key_off,
                           self.key_chars, None)
        return self

    def compare_rows(self, a, b):
        return lib().dko_compare_rows(C.byref(self.schema), C.byref(self.table), a, b)

    def match(self, queries=None, nthreads=1):
        q = np.arange(self.n, dtype=np.uint32) if queries is None else np.ascontiguousarray(queries, dtype=np.uint32)
        res = Result()
        rc = lib().dko_match(C.byref(self.schema), C.byref(self.table),
                             q.ctypes.data_as(C.POINTER(C.c_uint32)), len(q), nthreads, C.byref(res))
        if rc != 0:
            raise RuntimeError("dko_match failed")
        n = res.n
        out = {
            "query": np.ctypeslib.as_array(res.query, (n,)).copy() if n else np.zeros(0, np.uint32),
            "candidate": np.ctypeslib.as_array(res.candidate, (n,)).copy() if n else np.zeros(0, np.uint32),
            "prob": np.ctypeslib.as_array(res.prob, (n,)).copy() if n else np.zeros(0, np.float64),
            "kind": np.ctypeslib.as_array(res.kind, (n,)).copy() if n else np.zeros(0, np.uint8),
            "pairs_scored": res.pairs_scored,
            "ms_index": res.ms_index,
            "ms_score": res.ms_score,
        }
        lib().dko_free_result(C.byref(res))
        return out
