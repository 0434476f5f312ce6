"""Records, JSON ingestion and key functions on the host side of the boundary.

`Record` mirrors Duke's RecordImpl (property name -> values).  `records_from_entities`
restates IncrementalDataSource.DatasetDataSourceRecordIterator.next
(IncrementalDataSource.java:50-101): the ``_id`` check, one value per column (a JSON array
is read with Gson's JsonArray.getAsString, so only 1-element arrays work, :69-72), cleaner
then RecordBuilder's "skip empty", and the synthetic ID / dukeGroupNo /
dukeOriginalEntityId / dukeDatasetId / dukeDeleted properties (:76-98).
"""
from __future__ import annotations

import json

from .config import (DATASET_ID_PROPERTY_NAME, DELETED_PROPERTY_NAME, GROUP_NO_PROPERTY_NAME,
                     ID_PROPERTY, ORIGINAL_ENTITY_ID_PROPERTY_NAME)


class Record:
    """[Duke 1.2] Record: property -> collection of string values."""

    __slots__ = ("_values",)

    def __init__(self, values=None):
        self._values = {}
        for k, v in (values or {}).items():
            self._values[k] = list(v) if isinstance(v, (list, tuple)) else [v]

    def add_value(self, prop, value):
        self._values.setdefault(prop, []).append(value)

    def get_value(self, prop):
        v = self._values.get(prop)
        return v[0] if v else None

    def get_values(self, prop):
        return list(self._values.get(prop, ()))

    def get_properties(self):
        return list(self._values)

    def __repr__(self):
        return f"Record({self._values!r})"


def _gson_as_string(el):
    """com.google.gson.JsonElement.getAsString for a parsed JSON value."""
    if isinstance(el, list):
        if len(el) != 1:
            raise ValueError("JsonArray.getAsString on an array of %d elements" % len(el))
        return _gson_as_string(el[0])
    if el is None:
        raise ValueError("JsonNull.getAsString is unsupported")
    if isinstance(el, bool):
        return "true" if el else "false"
    if isinstance(el, dict):
        raise ValueError("JsonObject.getAsString is unsupported")
    return str(el)


def _gson_as_boolean(el):
    """com.google.gson.JsonElement.getAsBoolean: booleans, Boolean.parseBoolean of a string
    or number's text, a one-element array's element; null / objects / other arrays throw."""
    if isinstance(el, bool):
        return el
    if isinstance(el, list) and len(el) == 1:
        return _gson_as_boolean(el[0])
    if isinstance(el, str):
        return el.lower() == "true"
    raise ValueError("getAsBoolean is unsupported on %s" % type(el).__name__)


class JsonNumber(str):
    """A JSON number kept as its source text (Gson's LazilyParsedNumber): getAsString and
    re-serialisation both give the literal back unchanged."""
    __slots__ = ()


def parse_entities(body: str):
    """POST body -> (entities, single_entity) like App.java:955-965: an array, or one object.
    Numbers keep their JSON text (Gson's LazilyParsedNumber.toString)."""
    doc = json.loads(body, parse_float=JsonNumber, parse_int=JsonNumber)
    if isinstance(doc, list):
        return doc, False
    return [doc], True


def records_from_entities(entities, source, cleaners=None):
    """IncrementalDataSource.DatasetDataSourceRecordIterator over one batch.  `cleaners`
    maps a column's cleaner class name to a function (default: CLEANERS)."""
    cleaners = CLEANERS if cleaners is None else cleaners
    out = []
    for entity in entities:
        if not isinstance(entity, dict):  # (JsonObject) cast, IncrementalDataSource.java:51
            raise ValueError("an entity of the batch is not a JSON object")
        eid = entity.get("_id")
        eid = None if eid is None else _gson_as_string(eid)
        if not eid:
            raise ValueError("Got an entity with no '_id' attribute!")
        rec = Record()
        for col in source.columns:
            el = entity.get(col.name)
            if col.name not in entity:
                continue
            if isinstance(el, list):
                vals = [_gson_as_string(el) for _ in el]  # getAsString on the array (:69-72)
            else:
                vals = [_gson_as_string(el)]
            for v in vals:
                cl = cleaners.get(col.cleaner) if col.cleaner else None
                if cl is not None:
                    v = cl(v)
                if v is None or v == "":  # RecordBuilder.addValue skips empty values
                    continue
                rec.add_value(col.property, v)
        if source.group_no is not None:
            g = str(int(source.group_no))
            rid = f"{g}__{source.dataset_id}__{eid}"
            rec.add_value(GROUP_NO_PROPERTY_NAME, g)
        else:
            rid = f"{source.dataset_id}__{eid}"
        rec.add_value(ID_PROPERTY, rid)
        rec.add_value(ORIGINAL_ENTITY_ID_PROPERTY_NAME, eid)
        rec.add_value(DATASET_ID_PROPERTY_NAME, source.dataset_id)
        if "_deleted" in entity and _gson_as_boolean(entity["_deleted"]):
            rec.add_value(DELETED_PROPERTY_NAME, "true")
        out.append(rec)
    return out


# ---------------------------------------------------------------------------------------
# cleaners named by the reference's config (testdukeconfig.xml:50,55,66).  [Duke 1.2,
# recalled; PARITY UNPINNED: Duke's cleaner sources are not in /root/reference]
# ---------------------------------------------------------------------------------------
_WS = (" ", "\t", "\n", "\r", "\u00a0")


def lowercase_normalize(value, strip_accents=True):
    """cleaners.LowerCaseNormalizeCleaner: strip accents (NFD, drop combining marks),
    lower-case, trim, and collapse every whitespace run to one space."""
    import unicodedata
    if strip_accents:
        value = "".join(ch for ch in unicodedata.normalize("NFD", value)
                        if not unicodedata.combining(ch))
    out, pending = [], False
    for ch in value:
        if ch in _WS:
            pending = True
            continue
        if pending and out:
            out.append(" ")
        pending = False
        out.append(ch.lower())
    return "".join(out)


def country_name_clean(value):
    """examples.CountryNameCleaner: lower-case normalised, without a leading "the " or a
    trailing ", the"."""
    v = lowercase_normalize(value)
    if v.startswith("the "):
        v = v[4:]
    if v.endswith(", the"):
        v = v[:-5]
    return v


def capital_clean(value):
    """examples.CapitalCleaner: lower-case normalised, cut at the first ',' or '('."""
    v = lowercase_normalize(value)
    for sep in (",", "("):
        i = v.find(sep)
        if i >= 0:
            v = v[:i]
    return v.strip()


CLEANERS = {
    "no.priv.garshol.duke.cleaners.LowerCaseNormalizeCleaner": lowercase_normalize,
    "no.priv.garshol.duke.examples.CountryNameCleaner": country_name_clean,
    "no.priv.garshol.duke.examples.CapitalCleaner": capital_clean,
}


# ---------------------------------------------------------------------------------------
# key functions: [Duke 1.2] KeyFunction.makeKey(Record) -> String
# ---------------------------------------------------------------------------------------
class KeyFunction:
    def make_key(self, record: Record) -> str:
        raise NotImplementedError


class PartsKey(KeyFunction):
    """Concatenation of substrings of property values.  Each part is
    (property, token, start, end): token None = whole value, else the token index
    (whitespace split, negative from the end); [start:end] slice of it.  A missing value
    contributes ""."""

    def __init__(self, *parts):
        self.parts = parts

    def part(self, value, token, start, end):
        if value is None:
            return ""
        if token is not None:
            toks = value.split()
            if not toks:
                return ""
            value = toks[token] if -len(toks) <= token < len(toks) else ""
        return value[start:end]

    def make_key(self, record):
        return "".join(self.part(record.get_value(p), t, a, b) for p, t, a, b in self.parts)
