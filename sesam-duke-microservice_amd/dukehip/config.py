"""The <duke> configuration the GPU path consumes, read with Duke's schema.

Mirrors what the microservice builds per pipeline (App.java:227-548, 613-647):
``ConfigLoader.load`` of the <duke> block (objects, schema/threshold, properties with
comparator/low/high), plus the synthetic ``ID`` property and the ignored ``dukeDatasetId``
/ ``dukeOriginalEntityId`` / ``dukeDeleted`` (+ ``dukeGroupNo`` for linkage) properties
(App.java:309-323, 426-444).  Only the scored properties reach the kernels, in the order
Processor.compare visits them: the iteration order of the record's HashMap.
"""
from __future__ import annotations

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

    def comparison_order(self):
        """Scored properties in Processor.compare's visiting order: the key order of the
        record's java.util.HashMap (RecordImpl), whose keys are the data source's column
        properties followed by the synthetic ones IncrementalDataSource adds
        (IncrementalDataSource.java:76-98)."""
        names = []
        cols = self.data_sources[0].columns if self.data_sources else []
        for c in cols:
            if c.property not in names:
                names.append(c.property)
        for p in self.scored_properties():
            if p.name not in names:
                names.append(p.name)
        synth = ([GROUP_NO_PROPERTY_NAME] if self.linkage else []) + [
            ID_PROPERTY, ORIGINAL_ENTITY_ID_PROPERTY_NAME, DATASET_ID_PROPERTY_NAME]
        # A HashMap keeps capacity 16 up to 12 keys; past that its capacity (and so its
        # iteration order) depends on how many values a record holds, and computeBayes is
        # not associative: the GPU path runs one fixed order, so such schemas are not
        # eligible.  (+1: dukeDeleted is added for deleted entities.)
        if len(names + synth) + 1 > 12:
            raise UnsupportedComparator(
                f"{len(names + synth) + 1} record properties: past 12 a record's HashMap "
                "order depends on its value count (not GPU-eligible)")
        order = java_hashmap_order(names + synth)
        scored = {p.name: p for p in self.scored_properties()}
        out = [scored[n] for n in order if n in scored]
        # every data source must give its records the same visiting order (a different
        # column order only matters for keys sharing a HashMap bucket)
        for ds in self.data_sources[1:]:
            alt = []
            for c in ds.columns:
                if c.property not in alt:
                    alt.append(c.property)
            alt += [p.name for p in self.scored_properties() if p.name not in alt]
            if [n for n in java_hashmap_order(alt + synth) if n in scored] != [p.name for p in out]:
                raise UnsupportedComparator(
                    f"data source {ds.dataset_id!r} orders the record's properties differently "
                    "(HashMap bucket collision): one fixed comparison order does not hold")
        return out

    def to_schema(self, mode, nkeys):
        props = self.comparison_order()
        arr = (A.dk_property * max(1, len(props)))()
        for i, p in enumerate(props):
            if p.comparator is None:
                arr[i] = A.dk_property(A.CMP_NONE, 2, 0, 0, p.low, p.high, 0.0)
            else:
                arr[i] = p.comparator.to_c(p.low, p.high)
        s = A.dk_schema(len(props), arr, self.threshold, self.maybe_threshold, mode, nkeys)
        s._keep = arr
        return s, props


def java_string_hash(s: str) -> int:
    h = 0
    b = s.encode("utf-16-le", "surrogatepass")
    for i in range(0, len(b), 2):
        h = (31 * h + int.from_bytes(b[i:i + 2], "little")) & 0xFFFFFFFF
    return h


def java_hashmap_order(keys):
    """Iteration order of a java.util.HashMap<String,?> filled with `keys` in this order
    (default capacity 16, doubled past 0.75 load; buckets by (h ^ h>>>16) & (cap-1),
    insertion order inside a bucket)."""
    cap = 16
    while len(keys) > cap * 0.75:
        cap *= 2
    buckets = {}
    for k in keys:
        h = java_string_hash(k)
        idx = (h ^ (h >> 16)) & (cap - 1)
        buckets.setdefault(idx, []).append(k)
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

