"""The httptransform response: match arrays -> ``duke_links``.

* ``EntityLinksListener``  <- the entityIdToMatches half of BaseLinkDatabaseMatchListener
  (BaseLinkDatabaseMatchListener.java:46, 53-56, 68-88, 115-135): per batch, r1's
  dukeOriginalEntityId -> [(r2, confidence)] in callback order.  Per-callback; it is the
  checker for the bulk path.
* ``entity_links``         <- the same map built in bulk from a MatchResult's arrays (one
  pass over the entries, candidate metadata looked up once per distinct row).
* ``http_transform_response`` <- App.writeHttpTransformResponse (App.java:1180-1200): each
  posted entity copied through Gson (null members dropped) with ``duke_links`` added; an
  object for a single-entity request, else an array.
* ``LinkDatabase``         <- the pipeline's SinceAwareInMemoryLinkDatabase written in bulk by
  ``dk_linkdb_apply`` (csrc/dk_links.cpp) from a MatchResult, in place of the per-callback
  LinkDatabaseMatchListener BaseLinkDatabaseMatchListener forwards to (:53-109);
  ``since_feed`` = the GET /deduplication/<name>?since= body (App.java:818-874).
* ``gson_dumps`` / ``java_double`` -- Gson 2.8.0's default writer (compact, HTML-safe
  escaping, serializeNulls off) and Double.toString for the confidences.  Digits are the
  shortest round-trip form (JDK >= 19); JDK 8's Double.toString can differ in the last
  digit for some values (JDK-4511638), so confidence text is "parity unpinned" there.
"""
from __future__ import annotations

import ctypes as C
import math
import time
from decimal import Decimal

import numpy as np

from . import _abi as A
from .config import DATASET_ID_PROPERTY_NAME, ORIGINAL_ENTITY_ID_PROPERTY_NAME
from .processor import MatchListener, MatchResult
from .records import JsonNumber, _gson_as_string

LINK_INFERRED, LINK_RETRACTED = 1, 2   # LinkStatus
LINK_SAME, LINK_MAYBE = 1, 2           # LinkKind


class dk_link_batch(C.Structure):
    _fields_ = [("nqueries", C.c_uint64), ("query_ident", C.c_void_p), ("first", C.c_void_p),
                ("candidate_ident", C.c_void_p), ("prob", C.c_void_p), ("kind", C.c_void_p)]


class dk_link_stats(C.Structure):
    _fields_ = [("asserted", C.c_uint64), ("unchanged", C.c_uint64), ("retracted", C.c_uint64)]


class dk_link_list(C.Structure):
    _fields_ = [("n", C.c_uint64), ("id1", C.c_void_p), ("id2", C.c_void_p), ("status", C.c_void_p),
                ("kind", C.c_void_p), ("confidence", C.c_void_p), ("timestamp", C.c_void_p)]


_bound = False


def _lib():
    global _bound
    L = A.load()
    if not _bound:
        vp = C.c_void_p
        L.dk_linkdb_create.argtypes = [vp, C.POINTER(vp)]
        L.dk_linkdb_create.restype = C.c_int
        L.dk_linkdb_destroy.argtypes = [vp]
        L.dk_linkdb_destroy.restype = None
        L.dk_linkdb_size.argtypes = [vp]
        L.dk_linkdb_size.restype = C.c_uint64
        L.dk_linkdb_apply.argtypes = [vp, C.POINTER(dk_link_batch), C.c_int64, C.POINTER(dk_link_stats)]
        L.dk_linkdb_apply.restype = C.c_int
        L.dk_linkdb_changes_since.argtypes = [vp, C.c_int64, C.POINTER(C.POINTER(dk_link_list))]
        L.dk_linkdb_changes_since.restype = C.c_int
        L.dk_linkdb_links_for.argtypes = [vp, C.c_uint64, C.POINTER(C.POINTER(dk_link_list))]
        L.dk_linkdb_links_for.restype = C.c_int
        L.dk_linkdb_retract.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_int64, C.POINTER(C.c_uint64)]
        L.dk_linkdb_retract.restype = C.c_int
        L.dk_free_link_list.argtypes = [C.POINTER(dk_link_list)]
        L.dk_free_link_list.restype = None
        L.dk_interner_string.argtypes = [vp, C.c_uint64, C.POINTER(C.POINTER(C.c_uint16)),
                                         C.POINTER(C.c_uint64)]
        L.dk_interner_string.restype = C.c_int
        _bound = True
    return L


def interned_string(interner, ident) -> str:
    """The record ID string of an interned id (dk_interner_string)."""
    L = _lib()
    p = C.POINTER(C.c_uint16)()
    n = C.c_uint64()
    A.check(L.dk_interner_string(interner.h, int(ident), C.byref(p), C.byref(n)))
    return C.string_at(p, 2 * n.value).decode("utf-16-le", "surrogatepass") if n.value else ""


class LinkDatabase:
    """SinceAwareInMemoryLinkDatabase (SinceAwareInMemoryLinkDatabase.java:12-41), written in
    bulk: ``apply`` runs a batch's listener stream -- per query record in batch order its
    matches / matchesPerhaps (or noMatchFor), reconciled with its stored links the way Duke's
    LinkDatabaseMatchListener does [recalled: parity unpinned] -- natively in one call.  IDs are
    the database's interned record IDs."""

    def __init__(self, interner):
        self.lib = _lib()
        self.interner = interner
        self.h = C.c_void_p()
        A.check(self.lib.dk_linkdb_create(interner.h, C.byref(self.h)))

    def __len__(self):
        return int(self.lib.dk_linkdb_size(self.h))

    def apply(self, query_ident, first, candidate_ident, prob, kind, timestamp=None):
        """One batch: query_ident[i] is query i's record ID id, its entries are
        [first[i], first[i+1]) with candidate_ident / prob / kind.  timestamp: ms since the
        epoch (System.currentTimeMillis), default now.  Returns the dk_link_stats counts."""
        q = np.ascontiguousarray(query_ident, dtype=np.uint64)
        f = np.ascontiguousarray(first, dtype=np.uint64)
        c = np.ascontiguousarray(candidate_ident, dtype=np.uint64)
        p = np.ascontiguousarray(prob, dtype=np.float64)
        k = np.ascontiguousarray(kind, dtype=np.uint8)
        if len(f) != len(q) + 1 or not (len(c) == len(p) == len(k) == (int(f[-1]) if len(f) else 0)):
            raise ValueError("inconsistent link batch arrays")
        b = dk_link_batch(len(q), A.ptr(q), A.ptr(f), A.ptr(c), A.ptr(p), A.ptr(k))
        st = dk_link_stats()
        ts = int(time.time() * 1000) if timestamp is None else int(timestamp)
        A.check(self.lib.dk_linkdb_apply(self.h, C.byref(b), ts, C.byref(st)))
        return {"asserted": st.asserted, "unchanged": st.unchanged, "retracted": st.retracted}

    def apply_result(self, res: MatchResult, query_ident, row_ident, timestamp=None):
        """``apply`` of a host MatchResult: query_ident per query, row_ident per index row."""
        if res.on_device:
            raise ValueError("LinkDatabase.apply_result needs a host MatchResult")
        row_ident = np.asarray(row_ident, dtype=np.uint64)
        cand = row_ident[res.candidate] if res.n else np.zeros(0, np.uint64)
        return self.apply(query_ident, res.first, cand, res.prob, res.kind, timestamp)

    def changes_since(self, since=0):
        """getChangesSince(since): dict of arrays id1, id2, status, kind, confidence, timestamp."""
        out = C.POINTER(dk_link_list)()
        A.check(self.lib.dk_linkdb_changes_since(self.h, int(since), C.byref(out)))
        return self._take(out)

    def links_for(self, ident):
        """InMemoryLinkDatabase.getAllLinksFor(id) of an interned record ID (same dict form)."""
        out = C.POINTER(dk_link_list)()
        A.check(self.lib.dk_linkdb_links_for(self.h, int(ident), C.byref(out)))
        return self._take(out)

    def retract(self, ident, other=None, timestamp=None):
        """The POST route's deleted-record branch (App.java:994-999): Link.retract() +
        assertLink on the link between two interned IDs, or (other None) on every link of
        `ident`.  Returns the number of links retracted."""
        n = C.c_uint64()
        ts = int(time.time() * 1000) if timestamp is None else int(timestamp)
        oth = 0xFFFFFFFFFFFFFFFF if other is None else int(other)
        A.check(self.lib.dk_linkdb_retract(self.h, int(ident), oth, ts, C.byref(n)))
        return int(n.value)

    def _take(self, out):
        try:
            L = out.contents
            n = int(L.n)

            def arr(ptr, ct, dt):
                if n == 0:
                    return np.zeros(0, dt)
                return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), (n,)).astype(dt, copy=True)

            return {"id1": arr(L.id1, C.c_uint64, np.uint64), "id2": arr(L.id2, C.c_uint64, np.uint64),
                    "status": arr(L.status, C.c_uint8, np.uint8), "kind": arr(L.kind, C.c_uint8, np.uint8),
                    "confidence": arr(L.confidence, C.c_double, np.float64),
                    "timestamp": arr(L.timestamp, C.c_int64, np.int64)}
        finally:
            self.lib.dk_free_link_list(out)

    def since_feed(self, since, find_record_by_id) -> str:
        """The GET /deduplication/<name>?since=<since> body (App.java:846-874): one JSON object
        per changed link joined by ",\\n", each JsonObject.toString -- a bare JsonWriter: members
        in insertion order, JsonNull written as null, no HTML escaping."""
        ch = self.changes_since(since)
        parts = []
        strs = {}

        def sid(i):
            i = int(i)
            if i not in strs:
                strs[i] = interned_string(self.interner, i)
            return strs[i]

        for j in range(len(ch["id1"])):
            id1, id2 = sid(ch["id1"][j]), sid(ch["id2"][j])
            r1, r2 = find_record_by_id(id1), find_record_by_id(id2)
            ent = {"_id": (id1 + "_" + id2).replace(":", "_"),
                   "_updated": int(ch["timestamp"][j]),
                   "_deleted": bool(ch["status"][j] == LINK_RETRACTED),
                   "entity1": r1.get_value(ORIGINAL_ENTITY_ID_PROPERTY_NAME) if r1 is not None else None,
                   "entity2": r2.get_value(ORIGINAL_ENTITY_ID_PROPERTY_NAME) if r2 is not None else None,
                   "dataset1": r1.get_value(DATASET_ID_PROPERTY_NAME) if r1 is not None else None,
                   "dataset2": r2.get_value(DATASET_ID_PROPERTY_NAME) if r2 is not None else None,
                   "confidence": float(ch["confidence"][j])}
            parts.append(gson_dumps(ent, html_safe=False, serialize_nulls=True))
        return "[" + ",\n".join(parts) + "]"

    def close(self):
        if self.h:
            self.lib.dk_linkdb_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EntityLinksListener(MatchListener):
    """BaseLinkDatabaseMatchListener's getLinksForObject bookkeeping, callback by callback."""

    def __init__(self):
        self.entity_matches = {}

    def batch_ready(self, size):
        self.entity_matches = {}                       # :55, reset per batch

    def matches(self, r1, r2, confidence):
        self._add(r1, r2, confidence)

    def matches_perhaps(self, r1, r2, confidence):
        self._add(r1, r2, confidence)

    def _add(self, r1, r2, confidence):               # :84-88
        self.entity_matches.setdefault(r1.get_value(ORIGINAL_ENTITY_ID_PROPERTY_NAME), []).append(
            {"datasetId": r2.get_value(DATASET_ID_PROPERTY_NAME),
             "entityId": r2.get_value(ORIGINAL_ENTITY_ID_PROPERTY_NAME),
             "confidence": float(confidence)})

    def links(self):
        return self.entity_matches


def entity_links(res: MatchResult, query_records, rows):
    """{r1 dukeOriginalEntityId: [link, ...]} from a host MatchResult; `query_records[i]` is
    the Record of the i-th query, `rows[r]` the Record of index row r.  Entity ids with no
    match or maybe-match get no entry (computeIfAbsent only on a callback, :86)."""
    if res.on_device:
        raise ValueError("entity_links needs a host MatchResult (DK_MATCH_HOST)")
    first = np.asarray(res.first, dtype=np.int64)
    out = {}
    if res.n == 0:
        return out
    uniq, inv = np.unique(res.candidate, return_inverse=True)
    meta = [(rows[int(r)].get_value(DATASET_ID_PROPERTY_NAME),
             rows[int(r)].get_value(ORIGINAL_ENTITY_ID_PROPERTY_NAME)) for r in uniq]
    prob = res.prob.tolist()
    inv = inv.tolist()
    has = np.flatnonzero(first[1:] > first[:-1])
    for i in has.tolist():
        lst = out.setdefault(query_records[i].get_value(ORIGINAL_ENTITY_ID_PROPERTY_NAME), [])
        for e in range(int(first[i]), int(first[i + 1])):
            ds, eid = meta[inv[e]]
            lst.append({"datasetId": ds, "entityId": eid, "confidence": prob[e]})
    return out


def http_transform_response(entities, single_entity, links) -> str:
    """App.writeHttpTransformResponse: the posted entities with ``duke_links`` set from
    `links` (an entity_links / EntityLinksListener map) by each entity's ``_id``."""
    out = []
    for ent in entities:
        obj = dict(ent)
        obj["duke_links"] = list(links.get(_gson_as_string(ent.get("_id")), ()))
        out.append(obj)
    if single_entity and len(out) == 1:
        return gson_dumps(out[0])
    return gson_dumps(out)


# ---------------------------------------------------------------------------------------
# Gson 2.8.0 default JsonWriter
# ---------------------------------------------------------------------------------------
_ESC = {i: "\\u%04x" % i for i in range(0x20)}
_ESC.update({ord('"'): '\\"', ord("\\"): "\\\\", ord("\t"): "\\t", ord("\b"): "\\b",
             ord("\n"): "\\n", ord("\r"): "\\r", ord("\f"): "\\f",
             # htmlSafe (Gson's default): < > & = '
             ord("<"): "\\u003c", ord(">"): "\\u003e", ord("&"): "\\u0026", ord("="): "\\u003d",
             ord("'"): "\\u0027", 0x2028: "\\u2028", 0x2029: "\\u2029"})


_ESC_RAW = {k: v for k, v in _ESC.items() if k not in (ord("<"), ord(">"), ord("&"), ord("="), ord("'"))}


def _gson_string(s, html_safe=True):
    return '"' + s.translate(_ESC if html_safe else _ESC_RAW) + '"'


def java_double(x: float) -> str:
    """java.lang.Double.toString (shortest round-trip digits)."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    d = Decimal(repr(abs(x)))
    if 1e-3 <= abs(x) < 1e7:
        s = format(d, "f")
        if "." not in s:
            s += ".0"
        return sign + s
    _, digits, exp = d.normalize().as_tuple()
    digits = "".join(map(str, digits))
    e10 = len(digits) + exp - 1
    return f"{sign}{digits[0]}.{digits[1:] or '0'}E{e10}"


def gson_dumps(v, html_safe=True, serialize_nulls=False) -> str:
    """Gson.toJson of a parsed JSON tree (parse_entities output + float confidences).
    html_safe=False, serialize_nulls=True is JsonElement.toString (a bare JsonWriter)."""
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, JsonNumber):
        return str.__str__(v)
    if isinstance(v, str):
        return _gson_string(v, html_safe)
    if isinstance(v, float):
        return java_double(v)
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, dict):
        # Gson.toJson: serializeNulls is off, a member whose value is JSON null is not written
        return "{" + ",".join(_gson_string(k, html_safe) + ":" + gson_dumps(x, html_safe, serialize_nulls)
                              for k, x in v.items() if x is not None or serialize_nulls) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(gson_dumps(x, html_safe, serialize_nulls) for x in v) + "]"
    raise TypeError(f"not a JSON value: {type(v).__name__}")


__all__ = ["EntityLinksListener", "entity_links", "http_transform_response", "gson_dumps",
           "java_double", "LinkDatabase", "interned_string", "LINK_INFERRED", "LINK_RETRACTED",
           "LINK_SAME", "LINK_MAYBE"]
