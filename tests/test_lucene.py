"""The Lucene-compatible candidate source's host pieces (CPU): the native StandardAnalyzer
(dk_lucene_analyze) against its Python restatement (oracle/lucene_ref.py) and against UAX#29
word-boundary examples; the lookup-property selection on the reference's own schema.
PARITY UNPINNED against Lucene / Duke themselves (absent from /root/reference)."""
import json
import os
import random

import pytest

import lucene_ref as R
from dukehip.config import DukeConfig
from dukehip.lucene import LuceneOptions, analyze, lookup_properties

HERE = os.path.dirname(os.path.abspath(__file__))

# UAX#29 word segmentation examples (Unicode Standard Annex #29, WB5-WB13b), lowercased and
# English stop words removed as StandardAnalyzer does
KAT = [
    ("The quick brown fox", ["quick", "brown", "fox"]),
    ("O'Reilly's book", ["o'reilly's", "book"]),
    ("3.14 and 1,000.5", ["3.14", "1,000.5"]),
    ("e-mail wi-fi", ["e", "mail", "wi", "fi"]),
    ("U.S.A. a.b.c", ["u.s.a", "a.b.c"]),
    ("hello_world", ["hello_world"]),
    ("ab:cd", ["ab:cd"]),
    ("Café CRÈME brûlée", ["café", "crème", "brûlée"]),
    ("can't won't", ["can't", "won't"]),
    ("x1 2y 3.b", ["x1", "2y", "3", "b"]),
    ("  ", []),
]


@pytest.mark.parametrize("text,want", KAT)
def test_analyzer_word_boundaries(text, want):
    assert analyze(text) == want
    assert R.analyze(text) == want


def test_escaped_query_tokens():
    """escapeLucene (IncrementalLuceneDatabase.java:329-342) before the analyzer: a backslash
    in front of ':' splits what the index keeps as one token."""
    assert analyze("ab:cd", escape=True) == ["ab", "cd"] == R.query_tokens("ab:cd")
    assert analyze("  x-y  ", escape=True) == ["x", "y"]


def test_native_analyzer_equals_restatement():
    rng = random.Random(7)
    alphabet = list("abcXYZ019 .,:;'_-&()\"\t\nÀéÿ·ª\xad") + ["the", "and", "of"]
    for _ in range(3000):
        s = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 24)))
        for esc in (False, True):
            want = R.query_tokens(s) if esc else R.analyze(s)
            assert analyze(s, escape=esc) == want, (s, esc)


def test_non_latin1_declined():
    with pytest.raises(Exception):
        analyze("Δelta")


def test_norm_encoding():
    """SmallFloat.floatToByte315 of 1/sqrt(n): 1 token -> 124 (1.0), 2 -> 121 (0.625)."""
    assert [R.norm_byte(n) for n in (1, 2, 3, 4)] == [124, 121, 120, 120]
    assert R.byte315_to_float(124) == 1.0 and R.byte315_to_float(121) == 0.625


def test_lookup_properties_of_reference_schema():
    """testdukeconfig.xml: NAME (high 0.93), AREA (0.73), CAPITAL (0.61), threshold 0.9, no
    maybe-threshold: 0.5 -> CAPITAL 0.61 -> AREA 0.809 -> NAME 0.9825 >= 0.9, so NAME alone."""
    with open(os.path.join(HERE, "golden", "testdukeconfig_schema.json")) as f:
        cfg = DukeConfig.from_dict(json.load(f)["pipelines"]["Deduplication/countries-dbpedia-mondial"])
    props = cfg.scored_properties()
    assert lookup_properties(cfg, props) == ["NAME"]
    assert R.lookup_properties([(p.name, p.high, "default") for p in props], cfg.threshold,
                               cfg.maybe_threshold) == ["NAME"]


def test_options_from_environment():
    """App.configureDatabase (App.java:550-563)."""
    o = LuceneOptions.from_env({})
    assert (o.max_hits, o.min_relevance, o.fuzzy_search) == (10, 0.9, False)
    o = LuceneOptions.from_env({"MIN_RELEVANCE": "0.5", "MAX_SEARCH_HITS": "20", "FUZZY_SEARCH": "false"})
    assert (o.max_hits, o.min_relevance) == (20, 0.5)
    with pytest.raises(Exception):
        LuceneOptions.from_env({"FUZZY_SEARCH": "true"}).check()


# A re-posted ID under the two statistics modes: Q, A and B are indexed; four IDs
# first posted with name "anna" are re-posted as "finn".  Live versions alone (MERGED, the
# default): "anna" is in 2 documents and "oslo" in 4, so A (anna) outranks B (oslo) for Q.
# Counting the superseded versions too (UNMERGED, Lucene 4's deleted-but-unmerged documents):
# "anna" is in 6, so B outranks A, and with max_hits 2 the hit lists differ.
REPOST_NAMES = ["anna", "anna", "berit", "dag", "erik", "anna", "anna", "anna", "anna",
                "finn", "finn", "finn", "finn"]
REPOST_CITY = ["oslo", "bergen", "oslo", "oslo", "oslo"] + ["trondheim"] * 8
REPOST_ALIVE = [True] * 5 + [False] * 4 + [True] * 4       # rows 5..8 superseded by 9..12


def repost_hits(unmerged):
    ref = R.LuceneIndexRef(["name", "city"], max_hits=2, min_relevance=0.0)
    ref.set_docs([REPOST_NAMES, REPOST_CITY], REPOST_ALIVE,
                 in_stats=[True] * len(REPOST_NAMES) if unmerged else None)
    return ref.candidates(0)


def test_reposted_id_ranks_differently_merged_vs_unmerged():
    assert repost_hits(unmerged=False) == [0, 1]   # Q itself, then A
    assert repost_hits(unmerged=True) == [0, 2]    # Q itself, then B
