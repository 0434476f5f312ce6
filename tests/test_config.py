"""CPU: the <duke> configuration -> C-ABI schema mapping (ConfigLoader semantics the GPU
path relies on, App.java:613-647; comparator classes of SURVEY §8a rows a-10..a-16)."""
import pytest

from dukehip import _abi as A
from dukehip import config as cfgmod

XML = """
<duke>
  <object class="no.priv.garshol.duke.comparators.ExactComparator" name="Exact"/>
  <object class="no.priv.garshol.duke.comparators.DiceCoefficientComparator" name="Dice">
    <param name="comparator" value="Exact"/>
  </object>
  <object class="no.priv.garshol.duke.comparators.JaccardIndexComparator" name="Jacc"/>
  <object class="no.priv.garshol.duke.comparators.QGramComparator" name="Q3Ends">
    <param name="q" value="3"/>
    <param name="formula" value="JACCARD"/>
    <param name="tokenizer" value="ENDS"/>
  </object>
  <object class="no.priv.garshol.duke.comparators.NumericComparator" name="Zip">
    <param name="min-ratio" value="0.9"/>
  </object>
  <schema>
    <threshold>0.85</threshold>
    <maybe-threshold>0.6</maybe-threshold>
    <property type="id"><name>ID</name></property>
    <property><name>TEXT</name>
      <comparator>no.priv.garshol.duke.comparators.WeightedLevenshtein</comparator>
      <low>0.2</low><high>0.9</high></property>
    <property><name>TOKENS</name><comparator>Dice</comparator><low>0.3</low><high>0.8</high></property>
    <property><name>TAGS</name><comparator>Jacc</comparator><low>0.3</low><high>0.7</high></property>
    <property><name>NAME</name><comparator>Q3Ends</comparator><low>0.1</low><high>0.95</high></property>
    <property><name>ZIP</name><comparator>Zip</comparator><low>0.4</low><high>0.6</high></property>
  </schema>
  <data-source class="io.sesam.dukemicroservice.IncrementalDeduplicationDataSource">
    <param name="dataset-id" value="a"/>
    <column name="text" property="TEXT"/><column name="tokens" property="TOKENS"/>
    <column name="tags" property="TAGS"/><column name="name" property="NAME"/>
    <column name="zip" property="ZIP"/>
  </data-source>
</duke>
"""


def test_schema_from_duke_xml():
    c = cfgmod.parse_duke_config(XML)
    assert c.threshold == 0.85 and c.maybe_threshold == 0.6
    schema, props = c.to_schema(A.MODE_DEDUP, 1)
    assert schema.nprops == 5
    by = {p.name: schema.props[i] for i, p in enumerate(props)}
    assert by["TEXT"].comparator == A.CMP_WEIGHTED_LEVENSHTEIN
    assert by["TOKENS"].comparator == A.CMP_DICE_TOKENS
    assert by["TAGS"].comparator == A.CMP_JACCARD_TOKENS
    q = by["NAME"]
    assert (q.comparator, q.qgram_q, q.qgram_formula, q.qgram_tokenizer) == (
        A.CMP_QGRAM, 3, A.QGRAM_JACCARD, A.QGRAM_ENDS)
    assert by["ZIP"].comparator == A.CMP_NUMERIC and by["ZIP"].min_ratio == 0.9
    # Processor.compare visits the record's HashMap order, not the schema order
    assert [p.name for p in props] == [n for n in cfgmod.java_hashmap_order(
        ["TEXT", "TOKENS", "TAGS", "NAME", "ZIP", "ID", "dukeOriginalEntityId", "dukeDatasetId"])
        if n in by]


def test_token_sub_comparator_must_be_exact():
    xml = XML.replace('class="no.priv.garshol.duke.comparators.ExactComparator" name="Exact"',
                      'class="no.priv.garshol.duke.comparators.Levenshtein" name="Exact"')
    c = cfgmod.parse_duke_config(xml)
    with pytest.raises(cfgmod.UnsupportedComparator):
        c.to_schema(A.MODE_DEDUP, 1)


def test_unknown_comparator_is_not_gpu_eligible():
    xml = XML.replace("no.priv.garshol.duke.comparators.WeightedLevenshtein",
                      "no.priv.garshol.duke.comparators.SoundexComparator")
    with pytest.raises(cfgmod.UnsupportedComparator):
        cfgmod.parse_duke_config(xml).to_schema(A.MODE_DEDUP, 1)


def test_geoposition_comparator_maps_max_distance():
    """GeopositionComparator (DK_CMP_GEOPOSITION): max-distance travels in the property's
    double parameter; as the ONLY Lucene lookup property it stays on stock Duke, whose
    database raises for it (IncrementalLuceneDatabase.java:433-441, 460-463)."""
    from dukehip import lucene
    xml = XML.replace("</schema>", """<property><name>POS</name><comparator>Geo</comparator>
      <low>0.2</low><high>0.9</high></property></schema>""").replace(
        "<schema>", """<object class="no.priv.garshol.duke.comparators.GeopositionComparator" name="Geo">
    <param name="max-distance" value="2500"/></object><schema>""")
    c = cfgmod.parse_duke_config(xml)
    schema, props = c.to_schema(A.MODE_DEDUP, 1)
    pos = schema.props[[p.name for p in props].index("POS")]
    assert (pos.comparator, pos.min_ratio) == (A.CMP_GEOPOSITION, 2500.0)
    geo = [p for p in props if p.name == "POS"]
    geo[0].lookup = "true"
    with pytest.raises(cfgmod.UnsupportedComparator):
        lucene.lookup_properties(c, geo)
    geo[0].lookup = "default"
