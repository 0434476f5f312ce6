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
* ``gson_dumps`` / ``java_double`` -- Gson 2.8.0's default writer (compact, HTML-safe
  escaping, serializeNulls off) and Double.toString for the confidences.  Digits are the
  shortest round-trip form (JDK >= 19); JDK 8's Double.toString can differ in the last
  digit for some values (JDK-4511638), so confidence text is "parity unpinned" there.
"""
from __future__ import annotations

import math
from decimal import Decimal

import numpy as np

from .config import DATASET_ID_PROPERTY_NAME, ORIGINAL_ENTITY_ID_PROPERTY_NAME
from .processor import MatchListener, MatchResult
from .records import JsonNumber, _gson_as_string


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


def _gson_string(s):
    return '"' + s.translate(_ESC) + '"'


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


def gson_dumps(v) -> str:
    """Gson.toJson of a parsed JSON tree (parse_entities output + float confidences)."""
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, JsonNumber):
        return str.__str__(v)
    if isinstance(v, str):
        return _gson_string(v)
    if isinstance(v, float):
        return java_double(v)
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, dict):
        # serializeNulls is off: a member whose value is JSON null is not written
        return "{" + ",".join(_gson_string(k) + ":" + gson_dumps(x)
                              for k, x in v.items() if x is not None) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(gson_dumps(x) for x in v) + "]"
    raise TypeError(f"not a JSON value: {type(v).__name__}")


__all__ = ["EntityLinksListener", "entity_links", "http_transform_response", "gson_dumps",
           "java_double"]
