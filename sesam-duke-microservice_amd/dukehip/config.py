"""The <duke> configuration the GPU path consumes, read with Duke's schema.

Mirrors what the microservice builds per pipeline (App.java:227-548, 613-647):
``ConfigLoader.load`` of the <duke> block (objects, schema/threshold, properties with
comparator/low/high), plus the synthetic ``ID`` property and the ignored ``dukeDatasetId``
/ ``dukeOriginalEntityId`` / ``dukeDeleted`` (+ ``dukeGroupNo`` for linkage) properties
(App.java:309-323, 426-444).  Only the scored properties reach the kernels, in the order
Processor.compare visits them: the iteration order of the record's HashMap.
"""
from __future__ import annotations

import os
import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

from . import _abi as A

DUKE_CMP = "no.priv.garshol.duke.comparators."
COMPARATOR_CLASSES = {
    DUKE_CMP + "Levenshtein": A.CMP_LEVENSHTEIN,
    DUKE_CMP + "JaroWinkler": A.CMP_JAROWINKLER,
    DUKE_CMP + "QGramComparator": A.CMP_QGRAM,
    DUKE_CMP + "ExactComparator": A.CMP_EXACT,
    DUKE_CMP + "NumericComparator": A.CMP_NUMERIC,
    DUKE_CMP + "WeightedLevenshtein": A.CMP_WEIGHTED_LEVENSHTEIN,
    DUKE_CMP + "DiceCoefficientComparator": A.CMP_DICE_TOKENS,
    DUKE_CMP + "JaccardIndexComparator": A.CMP_JACCARD_TOKENS,
    DUKE_CMP + "GeopositionComparator": A.CMP_GEOPOSITION,
}
EXACT_CLASS = DUKE_CMP + "ExactComparator"
FORMULAS = {"OVERLAP": A.QGRAM_OVERLAP, "JACCARD": A.QGRAM_JACCARD, "DICE": A.QGRAM_DICE}
TOKENIZERS = {"BASIC": A.QGRAM_BASIC, "POSITIONAL": A.QGRAM_POSITIONAL, "ENDS": A.QGRAM_ENDS}

ID_PROPERTY = "ID"
GROUP_NO_PROPERTY_NAME = "dukeGroupNo"               # IncrementalLuceneDatabase.java:449
DATASET_ID_PROPERTY_NAME = "dukeDatasetId"           # :450
ORIGINAL_ENTITY_ID_PROPERTY_NAME = "dukeOriginalEntityId"  # :451
DELETED_PROPERTY_NAME = "dukeDeleted"                # :452


class UnsupportedComparator(ValueError):
    """The pipeline names a comparator without a GPU kernel: not GPU-eligible."""


@dataclass
class Comparator:
    """A Duke comparator instance: class name + bean parameters (ConfigLoader <param>)."""
    klass: str
    params: dict = field(default_factory=dict)

    def to_c(self, low, high):
        op = COMPARATOR_CLASSES.get(self.klass)
        if op is None:
            raise UnsupportedComparator(f"comparator {self.klass} has no GPU kernel")
        p = A.dk_property(op, 2, A.QGRAM_OVERLAP, A.QGRAM_BASIC, low, high, 0.0)
        for name, value in self.params.items():
            key = name.replace("-", "").lower()   # bean setter: min-ratio -> setMinRatio
            if op == A.CMP_NUMERIC and key == "minratio":
                p.min_ratio = float(value)
            elif op == A.CMP_GEOPOSITION and key == "maxdistance":
                p.min_ratio = float(value)      # setMaxDistance (meters), the double parameter
            elif op == A.CMP_QGRAM and key == "q":
                p.qgram_q = int(value)
            elif op == A.CMP_QGRAM and key == "formula":
                p.qgram_formula = FORMULAS[value.strip().upper()]
            elif op == A.CMP_QGRAM and key == "tokenizer":
                p.qgram_tokenizer = TOKENIZERS[value.strip().upper()]
            elif op in (A.CMP_DICE_TOKENS, A.CMP_JACCARD_TOKENS) and key == "comparator":
                # the token sub-comparator: only the default ExactComparator has a kernel
                sub = value.klass if isinstance(value, Comparator) else str(value).strip()
                if sub != EXACT_CLASS:
                    raise UnsupportedComparator(f"{self.klass}: sub-comparator {sub} has no GPU kernel")
            else:
                raise UnsupportedComparator(f"{self.klass}: parameter {name!r}")
        return p


@dataclass
class Property:
    """[Duke 1.2] PropertyImpl: name, comparator, low, high, id / ignore flags, lookup
    behaviour (<property lookup="true|false|required">; "default" when absent)."""
    name: str
    comparator: Comparator | None = None
    low: float = 0.5
    high: float = 0.5
    is_id: bool = False
    ignore: bool = False
    lookup: str = "default"

    def scored(self):
        return not self.is_id and not self.ignore


@dataclass
class DataSourceColumn:
    name: str
    property: str
    cleaner: object = None


@dataclass
class DataSource:
    """An IncrementalDeduplicationDataSource / IncrementalRecordLinkageDataSource."""
    dataset_id: str
    columns: list
    group_no: int | None = None


@dataclass
class DukeConfig:
    properties: list
    threshold: float
    maybe_threshold: float = 0.0
    data_sources: list = field(default_factory=list)
    linkage: bool = False

    def property(self, name):
        for p in self.properties:
            if p.name == name:
                return p
        return None

    def scored_properties(self):
        return [p for p in self.properties if p.scored()]

    def to_dict(self):
        """JSON-able form (committed fixtures; the Java shim passes the same fields)."""
        def comp(c):
            if c is None:
                return None
            return {"class": c.klass, "params": {k: (comp(v) if isinstance(v, Comparator) else v)
                                                 for k, v in c.params.items()}}
        return {"threshold": self.threshold, "maybe_threshold": self.maybe_threshold,
                "linkage": self.linkage,
                "properties": [{"name": p.name, "comparator": comp(p.comparator), "low": p.low,
                                "high": p.high, "is_id": p.is_id, "ignore": p.ignore,
                                **({"lookup": p.lookup} if p.lookup != "default" else {})}
                               for p in self.properties],
                "data_sources": [{"dataset_id": d.dataset_id, "group_no": d.group_no,
                                  "columns": [{"name": c.name, "property": c.property,
                                               "cleaner": c.cleaner} for c in d.columns]}
                                 for d in self.data_sources]}

    @classmethod
    def from_dict(cls, d):
        def comp(c):
            if c is None:
                return None
            return Comparator(c["class"], {k: (comp(v) if isinstance(v, dict) else v)
                                           for k, v in c.get("params", {}).items()})
        props = [Property(p["name"], comp(p["comparator"]), p["low"], p["high"],
                          p.get("is_id", False), p.get("ignore", False), p.get("lookup", "default"))
                 for p in d["properties"]]
        sources = [DataSource(s["dataset_id"], [DataSourceColumn(c["name"], c["property"],
                                                                 c.get("cleaner"))
                                                for c in s["columns"]], s.get("group_no"))
                   for s in d["data_sources"]]
        return cls(props, d["threshold"], d.get("maybe_threshold", 0.0), sources,
                   d.get("linkage", False))

    def _record_keys(self, ds=None):
        """A record's possible HashMap keys in insertion order (IncrementalDataSource.java:
        67-98): the data source's column properties, then the synthetic ones (dukeDeleted,
        added last for deleted entities, is left to the caller), plus scored properties no
        column fills (never present; kept so every scored property has a place)."""
        names = []
        cols = (ds or (self.data_sources[0] if self.data_sources else None))
        for c in (cols.columns if cols else []):
            if c.property not in names:
                names.append(c.property)
        ncols = len(names)
        for p in self.scored_properties():
            if p.name not in names:
                names.append(p.name)
        if cols is None:   # no data source declared: any scored property may hold a value
            ncols = len(names)
        synth = ([GROUP_NO_PROPERTY_NAME] if self.linkage else []) + [
            ID_PROPERTY, ORIGINAL_ENTITY_ID_PROPERTY_NAME, DATASET_ID_PROPERTY_NAME]
        return names, synth, ncols

    def order_classes(self):
        """Processor.compare visits r1's properties in its RecordImpl HashMap's iteration
        order, which depends on the map's capacity: 16 up to 12 keys, 32 up to 24, 64 up to
        48 -- i.e. on how many properties the record holds values for.  Returns (caps,
        orders): the capacities a record of this pipeline can have (ascending) and for each
        the scored properties in visiting order (a record's missing ones are skipped)."""
        names, synth, ncols = self._record_keys()
        lo = len(synth)                      # no column value
        hi = ncols + len(synth) + 1          # every column + dukeDeleted
        if hi > 48:
            raise UnsupportedComparator(
                f"up to {hi} record properties: past 48 a record's HashMap grows past "
                "capacity 64 (not GPU-eligible)")
        caps = sorted({class_key(k) for k in range(lo, hi + 1)})
        keys = names + synth + [DELETED_PROPERTY_NAME]
        scored = {p.name: p for p in self.scored_properties()}
        orders = []
        for cap in caps:
            order = class_order(keys, cap)
            orders.append([scored[n] for n in order if n in scored])
        # every data source must give its records the same visiting orders (a different
        # column order only matters for keys sharing a HashMap bucket)
        for ds in self.data_sources[1:]:
            alt, _, _ = self._record_keys(ds)
            for cap, want in zip(caps, orders):
                got = [n for n in class_order(alt + synth + [DELETED_PROPERTY_NAME], cap)
                       if n in scored]
                if got != [p.name for p in want]:
                    raise UnsupportedComparator(
                        f"data source {ds.dataset_id!r} orders the record's properties "
                        "differently (HashMap bucket collision): one fixed comparison order "
                        "does not hold")
        return caps, orders

    def comparison_order(self):
        """Scored properties in Processor.compare's visiting order for a record of the
        smallest HashMap capacity the pipeline's records can have (the only one up to 12
        record properties): the schema's property order (dk_schema.props)."""
        return self.order_classes()[1][0]

    def record_class(self, record, caps):
        """The order class of a record (index into order_classes()[0]): its HashMap's
        capacity from the number of properties it holds values for."""
        return caps.index(class_key(len(record.get_properties())))

    def to_schema(self, mode, nkeys):
        """(dk_schema, props in its order); with several order classes the schema carries
        them (dk_schema.orders: class c visits props[orders[c][k]])."""
        caps, orders = self.order_classes()
        props = orders[0]
        arr = (A.dk_property * max(1, len(props)))()
        for i, p in enumerate(props):
            if p.comparator is None:
                arr[i] = A.dk_property(A.CMP_NONE, 2, 0, 0, p.low, p.high, 0.0)
            else:
                arr[i] = p.comparator.to_c(p.low, p.high)
        s = A.dk_schema(len(props), arr, self.threshold, self.maybe_threshold, mode, nkeys)
        s._keep = arr
        if len(orders) > 1:
            if len(orders) > A.MAX_ORDER_CLASSES:
                raise UnsupportedComparator(f"{len(orders)} HashMap order classes")
            idx = {p.name: i for i, p in enumerate(props)}
            A.order_classes(s, [[idx[p.name] for p in o] for o in orders])
        return s, props


def java_string_hash(s: str) -> int:
    h = 0
    b = s.encode("utf-16-le", "surrogatepass")
    for i in range(0, len(b), 2):
        h = (31 * h + int.from_bytes(b[i:i + 2], "little")) & 0xFFFFFFFF
    return h


# How a record's RecordImpl HashMap gets its capacity (SURVEY a-7).  Duke's source is absent,
# so which construction the reference's records go through is NOT pinned:
#   "incremental" -- `new HashMap<>()` then one put per key (IncrementalDataSource.java:67-98
#                    builds the property map key by key): 16, doubled when size > 0.75 * cap.
#                    A JDK 19+ copy constructor (`new HashMap<>(m)`, ceil(s / 0.75)) sizes
#                    every s the same way.
#   "copy_jdk8"   -- `new HashMap<>(m)` on JDK 8..18: putMapEntries sizes the table to
#                    tableSizeFor((int)(s / 0.75f + 1)), one doubling earlier at s = 12, 24, 48.
HASHMAP_CONSTRUCTIONS = ("incremental", "copy_jdk8")
HASHMAP_CONSTRUCTION = os.environ.get("DUKEHIP_HASHMAP_CONSTRUCTION", "incremental")


def _f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def _table_size_for(n):
    cap = 1
    while cap < n:
        cap *= 2
    return cap


def hashmap_capacity(nkeys, construction=None):
    """java.util.HashMap's table size for a map of `nkeys` keys built by `construction`
    (default HASHMAP_CONSTRUCTION; see above)."""
    construction = construction or HASHMAP_CONSTRUCTION
    if construction == "incremental":
        cap = 16
        while nkeys > cap * 0.75:
            cap *= 2
        return cap
    if construction == "copy_jdk8":
        # float arithmetic as putMapEntries: ft = s / 0.75f + 1.0f, t = (int) ft
        t = int(_f32(_f32(float(nkeys)) / _f32(0.75)) + 1.0)
        return _table_size_for(max(t, 1)) if nkeys else 16
    raise ValueError(f"unknown HashMap construction {construction!r} "
                     f"(one of {HASHMAP_CONSTRUCTIONS})")


def class_key(nkeys, construction=None):
    """What fixes the iteration order of a record map of `nkeys` keys: its capacity
    ("incremental"), or (capacity of the source map, capacity of the copy) ("copy_jdk8": a
    copy inserts the source's entries in the source's iteration order)."""
    construction = construction or HASHMAP_CONSTRUCTION
    if construction == "incremental":
        return hashmap_capacity(nkeys, "incremental")
    return (hashmap_capacity(nkeys, "incremental"), hashmap_capacity(nkeys, construction))


def class_order(keys, key):
    """Iteration order of the record map of order class `key` (class_key) holding `keys`
    (a record holding fewer keeps their relative order)."""
    if isinstance(key, tuple):
        src, cap = key
        return java_hashmap_order(java_hashmap_order(keys, src), cap)
    return java_hashmap_order(keys, key)


def java_hashmap_order(keys, cap=None):
    """Iteration order of a java.util.HashMap<String,?> filled with `keys` in this order
    (capacity `cap`, default: the one those puts give; buckets by (h ^ h>>>16) & (cap-1),
    insertion order inside a bucket -- a resize splits a bucket keeping its order).  A
    bucket of 8 or more keys is refused: a real map would treeify it at capacity >= 64 and
    resize below that (HashMap.treeifyBin), an order this model does not give."""
    cap = hashmap_capacity(len(keys)) if cap is None else cap
    buckets = {}
    for k in keys:
        h = java_string_hash(k)
        idx = (h ^ (h >> 16)) & (cap - 1)
        buckets.setdefault(idx, []).append(k)
    if any(len(b) >= 8 for b in buckets.values()):
        raise UnsupportedComparator("8 keys in one HashMap bucket (tree bin or resize): order not modelled")
    return [k for i in sorted(buckets) for k in buckets[i]]


def _text(el, tag, default=None):
    x = el.find(tag)
    return default if x is None or x.text is None else x.text.strip()


def parse_duke_config(xml, linkage=None) -> DukeConfig:
    """Parse a <duke> element (string or ElementTree element) the way ConfigLoader does
    for the parts the scoring path consumes."""
    root = ET.fromstring(xml) if isinstance(xml, str) else xml
    if root.tag != "duke":
        root = root.find(".//duke")
    objects = {}
    for ob in root.findall("object"):
        objects[ob.get("name")] = Comparator(
            ob.get("class"), {pa.get("name"): pa.get("value") for pa in ob.findall("param")})
    # ConfigLoader resolves a <param> value that names another <object> to that object
    # (e.g. the sub-comparator of DiceCoefficientComparator / JaccardIndexComparator)
    for ob in objects.values():
        for k, v in list(ob.params.items()):
            if isinstance(v, str) and v in objects:
                ob.params[k] = objects[v]
    schema = root.find("schema")
    threshold = float(_text(schema, "threshold"))
    maybe = float(_text(schema, "maybe-threshold", "0.0"))
    props = []
    for pe in schema.findall("property"):
        typ = pe.get("type", "")
        name = _text(pe, "name")
        cname = _text(pe, "comparator")
        comp = None
        if cname:
            # an <object> name wins, else the text is a class name with default params
            comp = objects.get(cname) or Comparator(cname, {})
        low = float(_text(pe, "low", "0.5"))
        high = float(_text(pe, "high", "0.5"))
        props.append(Property(name, comp, low, high, is_id=typ == "id", ignore=typ == "ignore",
                              lookup=(pe.get("lookup") or "default").strip().lower()))
    sources = []
    groups = root.findall("group")
    if linkage is None:
        linkage = bool(groups)
    containers = [(gi + 1, g) for gi, g in enumerate(groups)] if groups else [(None, root)]
    for gno, cont in containers:
        for ds in cont.findall("data-source"):
            params = {pa.get("name"): pa.get("value") for pa in ds.findall("param")}
            cols = [DataSourceColumn(c.get("name"), c.get("property"), c.get("cleaner"))
                    for c in ds.findall("column")]
            sources.append(DataSource(params.get("dataset-id"), cols, gno))
    return DukeConfig(props, threshold, maybe, sources, linkage)


def parse_microservice_config(xml: str):
    """<DukeMicroService> -> {("Deduplication"|"RecordLinkage", name): DukeConfig}
    (App.java:264-281, 291-293, 407-411)."""
    root = ET.fromstring(xml)
    out = {}
    for kind in ("Deduplication", "RecordLinkage"):
        for el in root.findall(kind):
            out[(kind, el.get("name"))] = parse_duke_config(el.find("duke"),
                                                            linkage=kind == "RecordLinkage")
    return out

