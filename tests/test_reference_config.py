"""CPU: the reference's own pipelines (src/main/resources/testdukeconfig.xml) through the
config path the GPU drop-in uses.  The XML is parsed in place when /root/reference is
present (this container) and must equal the committed fixture
tests/golden/testdukeconfig_schema.json (tests/gen_reference_schema.py), which the GPU
parity test test_reference_schema_dedup_gpu runs on the box.

What the reference's config pins (App.java:264-281, 291-325, 613-647 + ConfigLoader):
  * thresholds: 0.9 (Deduplication, :23), 0.7 (RecordLinkage, :97); no maybe-threshold
    element, so Duke's 0.0 = none (Processor.compareCandidatesSimple emits no maybes);
  * NAME Levenshtein (0.09, 0.93), AREA Numeric (0.04, 0.73), CAPITAL Levenshtein
    (0.12, 0.61);
  * AREA names the CLASS NumericComparator (:33), not the <object name="AreaComparator">
    declared at :17-20 with min-ratio 0.7: the object is unused and min-ratio stays 0.0;
  * Processor.compare's visiting order is the record HashMap's: AREA, CAPITAL, NAME;
  * the dbpedia data source maps the misspelt column "capical" (:56), so entities carrying
    "capital" give dbpedia records no CAPITAL value.
"""
import json
import os

import pytest

from dukehip import _abi as A
from dukehip import config as cfgmod
from dukehip import records as R

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "testdukeconfig_schema.json")
REF_XML = "/root/reference/src/main/resources/testdukeconfig.xml"
DEDUP = "Deduplication/countries-dbpedia-mondial"
LINK = "RecordLinkage/countries-dbpedia-mondial"


def fixture():
    with open(FIXTURE) as f:
        return json.load(f)["pipelines"]


@pytest.mark.skipif(not os.path.exists(REF_XML), reason="/root/reference not present")
def test_reference_xml_parses_to_fixture():
    import gen_reference_schema
    assert gen_reference_schema.parsed(REF_XML) == fixture()


@pytest.mark.parametrize("key,thr,linkage", [(DEDUP, 0.9, False), (LINK, 0.7, True)])
def test_reference_schema_semantics(key, thr, linkage):
    cfg = cfgmod.DukeConfig.from_dict(fixture()[key])
    assert cfg.threshold == thr and cfg.maybe_threshold == 0.0 and cfg.linkage == linkage
    schema, props = cfg.to_schema(A.MODE_LINKAGE if linkage else A.MODE_DEDUP, 1)
    assert [p.name for p in props] == ["AREA", "CAPITAL", "NAME"]
    got = {p.name: schema.props[i] for i, p in enumerate(props)}
    assert (got["NAME"].comparator, got["NAME"].low, got["NAME"].high) == (A.CMP_LEVENSHTEIN, 0.09, 0.93)
    assert (got["CAPITAL"].comparator, got["CAPITAL"].low, got["CAPITAL"].high) == (
        A.CMP_LEVENSHTEIN, 0.12, 0.61)
    a = got["AREA"]
    assert (a.comparator, a.low, a.high, a.min_ratio) == (A.CMP_NUMERIC, 0.04, 0.73, 0.0)
    assert schema.threshold == thr and schema.maybe_threshold == 0.0
    # both data sources visit the properties in the same order
    assert [ds.dataset_id for ds in cfg.data_sources] == ["countries-dbpedia", "countries-mondial"]
    if linkage:
        assert [ds.group_no for ds in cfg.data_sources] == [1, 2]


def test_reference_capical_column_quirk():
    cfg = cfgmod.DukeConfig.from_dict(fixture()[DEDUP])
    dbpedia, mondial = cfg.data_sources
    ent = {"_id": "7", "country": "Norway", "capital": "Oslo", "area": "3"}
    r1 = R.records_from_entities([ent], dbpedia)[0]
    r2 = R.records_from_entities([ent], mondial)[0]
    assert r1.get_value("CAPITAL") is None and r2.get_value("CAPITAL") == "oslo"
    assert r1.get_value("NAME") == "norway" and r1.get_value("AREA") == "3"
    assert r1.get_value("ID") == "countries-dbpedia__7"
    assert r2.get_value("ID") == "countries-mondial__7"


def test_config_dict_round_trip():
    for key, d in fixture().items():
        assert cfgmod.DukeConfig.from_dict(d).to_dict() == d


def test_cleaners_recalled():
    assert R.lowercase_normalize("  Sào   Tomé\tE Príncipe ") == "sao tome e principe"
    assert R.country_name_clean("The Gambia") == "gambia"
    assert R.country_name_clean("Bahamas, The") == "bahamas"
    assert R.capital_clean("Washington, D.C.") == "washington"
    assert R.capital_clean("Kingston (Jamaica)") == "kingston"


def test_wide_schema_order_classes():
    """Past 12 record keys a HashMap's capacity depends on the record's value count: one
    order class per reachable capacity (dk_schema.orders), each the scored properties in
    the iteration order of a HashMap of that capacity holding every possible key; a record's
    class follows the number of properties it holds.  Past 48 keys: not GPU-eligible."""
    props = [cfgmod.Property(f"P{i}", cfgmod.Comparator(cfgmod.DUKE_CMP + "ExactComparator"), 0.3, 0.7)
             for i in range(14)]
    cols = [cfgmod.DataSourceColumn(f"c{i}", f"P{i}") for i in range(14)]
    cfg = cfgmod.DukeConfig(props, 0.9, data_sources=[cfgmod.DataSource("ds", cols)])
    caps, orders = cfg.order_classes()
    assert caps == [16, 32]                      # 3 .. 14 + 3 + 1 = 18 keys
    keys = [f"P{i}" for i in range(14)] + [cfgmod.ID_PROPERTY, cfgmod.ORIGINAL_ENTITY_ID_PROPERTY_NAME,
                                            cfgmod.DATASET_ID_PROPERTY_NAME, cfgmod.DELETED_PROPERTY_NAME]
    for cap, o in zip(caps, orders):
        assert [p.name for p in o] == [k for k in cfgmod.java_hashmap_order(keys, cap) if k.startswith("P")]
    assert [p.name for p in orders[0]] != [p.name for p in orders[1]]   # the classes differ here
    s, sp = cfg.to_schema(A.MODE_DEDUP, 1)
    assert s.nprops == 14 and s.norders == 2
    got = [[sp[s.orders[c * 14 + k]].name for k in range(14)] for c in range(2)]
    assert got == [[p.name for p in o] for o in orders]
    from dukehip.records import Record
    small = Record({"P0": "a", "ID": "x", "dukeOriginalEntityId": "1", "dukeDatasetId": "ds"})
    big = Record({**{f"P{i}": "a" for i in range(11)}, "ID": "x", "dukeOriginalEntityId": "1",
                  "dukeDatasetId": "ds"})
    assert cfg.record_class(small, caps) == 0 and cfg.record_class(big, caps) == 1   # 4 / 14 keys
    wide = [cfgmod.Property(f"W{i}", None, 0.3, 0.7) for i in range(46)]
    wcfg = cfgmod.DukeConfig(wide, 0.9, data_sources=[cfgmod.DataSource(
        "ds", [cfgmod.DataSourceColumn(f"w{i}", f"W{i}") for i in range(46)])])
    with pytest.raises(cfgmod.UnsupportedComparator):
        wcfg.to_schema(A.MODE_DEDUP, 1)
    narrow = cfgmod.DukeConfig(props[:8], 0.9)
    assert narrow.to_schema(A.MODE_DEDUP, 1)[0].norders == 0
