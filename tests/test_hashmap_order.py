"""CPU: the HashMap-capacity assumption behind order classes (SURVEY a-7).

Processor.compare visits r1's properties in its RecordImpl HashMap's iteration order, and
that order follows the map's capacity.  Which construction Duke's RecordImpl uses is
unpinned (Duke's source is absent), so it is a named option:
`dukehip.config.HASHMAP_CONSTRUCTION` ("incremental" by default, or "copy_jdk8").  These
tests check config.py's bucket sort against duke_pyref's simulated java.util.HashMap for
both, and show the choice is not cosmetic: the two disagree at 12 keys (capacity 16 vs 32)
while agreeing at 10 and 11.
"""
import random

import pytest

import duke_pyref as R
from dukehip import config as cfgmod

SYNTH = ["ID", "dukeOriginalEntityId", "dukeDatasetId"]


def _keys(rng, n):
    out = list(SYNTH[:min(3, n)])
    while len(out) < n:
        k = "".join(rng.choice("ABCDEFGHIJKLMNOPQRSTUVWXYZ_") for _ in range(rng.randint(2, 12)))
        if k not in out:
            out.insert(rng.randint(0, len(out)), k)
    return out


def _config_order(keys, construction):
    return cfgmod.class_order(keys, cfgmod.class_key(len(keys), construction))


@pytest.mark.parametrize("construction", cfgmod.HASHMAP_CONSTRUCTIONS)
def test_bucket_sort_matches_simulated_hashmap(construction):
    rng = random.Random(7)
    checked = 0
    for n in list(range(1, 49)) * 6:
        keys = _keys(rng, n)
        try:
            want = _config_order(keys, construction)
        except cfgmod.UnsupportedComparator:   # a tree bin: refused, not modelled
            continue
        assert want == R.record_map_order(keys, construction), (construction, keys)
        checked += 1
    assert checked > 250


def test_capacities_per_construction():
    inc = [cfgmod.hashmap_capacity(n, "incremental") for n in (3, 10, 11, 12, 13, 24, 25)]
    cpy = [cfgmod.hashmap_capacity(n, "copy_jdk8") for n in (3, 10, 11, 12, 13, 24, 25)]
    assert inc == [16, 16, 16, 16, 32, 32, 64]
    assert cpy == [8, 16, 16, 32, 32, 64, 64]   # putMapEntries: tableSizeFor((int)(s/.75f + 1))
    with pytest.raises(ValueError):
        cfgmod.hashmap_capacity(5, "treemap")


def test_orders_differ_at_12_keys_only_in_10_to_12():
    rng = random.Random(11)
    differ = {10: 0, 11: 0, 12: 0}
    for _ in range(200):
        for n in differ:
            keys = _keys(rng, n)
            a = R.record_map_order(keys, "incremental")
            b = R.record_map_order(keys, "copy_jdk8")
            differ[n] += a != b
    assert differ[10] == 0 and differ[11] == 0   # both capacity 16: same order
    assert differ[12] > 100                       # 16 vs 32: the choice is deliberate


def test_wide_schema_classes_follow_the_option(monkeypatch):
    """A 9-column pipeline (records of 3..13 keys) has one order class incrementally
    (capacity 16 up to 12 keys, 32 at 13) but several when records are copies."""
    cols = "".join(f'<column name="c{i}" property="P{i}"/>' for i in range(9))
    props = "".join(f"<property><name>P{i}</name><comparator>"
                    "no.priv.garshol.duke.comparators.ExactComparator</comparator>"
                    "<low>0.3</low><high>0.8</high></property>" for i in range(9))
    xml = (f"<duke><schema><threshold>0.8</threshold><property type='id'><name>ID</name>"
           f"</property>{props}</schema><data-source class='x'>"
           f"<param name='dataset-id' value='a'/>{cols}</data-source></duke>")
    cfg = cfgmod.parse_duke_config(xml)
    monkeypatch.setattr(cfgmod, "HASHMAP_CONSTRUCTION", "incremental")
    caps_i, orders_i = cfg.order_classes()
    assert caps_i == [16, 32]
    monkeypatch.setattr(cfgmod, "HASHMAP_CONSTRUCTION", "copy_jdk8")
    caps_c, orders_c = cfg.order_classes()
    assert caps_c == [(16, 8), (16, 16), (16, 32), (32, 32)]
    # every class's order is the simulated copy's, restricted to the scored properties
    keys = [f"P{i}" for i in range(9)] + SYNTH + [cfgmod.DELETED_PROPERTY_NAME]
    for key, order in zip(caps_c, orders_c):
        assert [p.name for p in order] == [k for k in cfgmod.class_order(keys, key)
                                           if k.startswith("P")]
