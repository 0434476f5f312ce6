"""The Lucene-compatible candidate source (DK_CAND_LUCENE, include/dukehip.h ``dk_lucene``):
pipelines that keep the reference's own IncrementalLuceneDatabase instead of key functions.

* ``lookup_properties``  <- [Duke 1.2, recalled] ConfigurationImpl's lookup properties: the
  scored properties sorted by <high> ascending (stable), computeBayes from 0.5 over them until
  the result reaches maybe-threshold (threshold when that is 0.0) -- that property and all
  later ones -- plus those marked lookup="true"/"required", minus lookup="false".
* ``LuceneOptions``      <- App.configureDatabase (App.java:550-563): max-search-hits 10,
  min-relevance 0.9, fuzzy search off; the MIN_RELEVANCE / MAX_SEARCH_HITS / FUZZY_SEARCH
  environment overrides.  FUZZY_SEARCH=true and Lookup.REQUIRED are not GPU-eligible.
* ``analyze``            <- the native StandardAnalyzer restatement (dk_lucene_analyze).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _abi as A
from .config import UnsupportedComparator


@dataclass
class LuceneOptions:
    max_hits: int = 10
    min_relevance: float = 0.9
    fuzzy_search: bool = False

    @classmethod
    def from_env(cls, env=None):
        """App.configureDatabase: the defaults, then MIN_RELEVANCE (Float.parseFloat),
        FUZZY_SEARCH (Boolean.parseBoolean), MAX_SEARCH_HITS (Integer.parseInt)."""
        env = os.environ if env is None else env
        o = cls()
        if env.get("MIN_RELEVANCE") is not None:
            o.min_relevance = float(env["MIN_RELEVANCE"])
        if env.get("FUZZY_SEARCH") is not None:
            o.fuzzy_search = env["FUZZY_SEARCH"].strip().lower() == "true"
        if env.get("MAX_SEARCH_HITS") is not None:
            o.max_hits = int(env["MAX_SEARCH_HITS"])
        return o

    def check(self):
        if self.fuzzy_search:
            raise UnsupportedComparator("FUZZY_SEARCH=true (FuzzyQuery) is not GPU-eligible")
        if not 1 <= self.max_hits <= 100:
            raise UnsupportedComparator(f"MAX_SEARCH_HITS={self.max_hits}: the GPU path holds 1..100 "
                                        "(larger limits grow adaptively, EstimateResultTracker)")


def lookup_properties(config, props):
    """Names of the lookup properties among `props` (the schema's scored properties)."""
    behaviour = {p.name: getattr(p, "lookup", "default") for p in props}
    if any(b == "required" for b in behaviour.values()):
        raise UnsupportedComparator("Lookup.REQUIRED (MUST clauses) is not GPU-eligible")
    cand = sorted([p for p in props if behaviour[p.name] != "false"], key=lambda p: p.high)
    limit = config.maybe_threshold if config.maybe_threshold != 0.0 else config.threshold
    prob, last = 0.5, -1
    for ix, p in enumerate(cand):
        if p.high == 0.0:
            continue
        prob = (prob * p.high) / ((prob * p.high) + ((1.0 - prob) * (1.0 - p.high)))
        if prob >= limit:
            last = ix
            break
    out = [p.name for p in cand[last:]] if last >= 0 else []
    for p in props:
        if behaviour[p.name] == "true" and p.name not in out:
            out.append(p.name)
    # a GeopositionComparator as the only lookup property: the reference's database searches
    # geo-spatially and raises (IncrementalLuceneDatabase.java:433-441, 460-463)
    if len(out) == 1:
        only = next(p for p in props if p.name == out[0])
        if only.comparator is not None and only.comparator.klass.endswith(".GeopositionComparator"):
            raise UnsupportedComparator("GeopositionComparator as the only lookup property "
                                        "(IncrementalLuceneDatabase.java:460-463 raises)")
    return out


_bound = False


def analyze(value: str, escape=False):
    """dk_lucene_analyze: StandardAnalyzer tokens of `value` (escape: escapeLucene first)."""
    global _bound
    L = A.load()
    if not _bound:
        L.dk_lucene_analyze.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_char_p, C.c_uint64,
                                        C.POINTER(C.c_uint64)]
        L.dk_lucene_analyze.restype = C.c_int
        _bound = True
    u = np.frombuffer(value.encode("utf-16-le", "surrogatepass"), dtype=np.uint16)
    cap = 4 * len(value) + 64
    out = C.create_string_buffer(cap)
    n = C.c_uint64()
    A.check(L.dk_lucene_analyze(u.ctypes.data if u.size else None, u.size, 1 if escape else 0, out,
                                cap, C.byref(n)))
    return out.value.decode("latin-1").split("\n") if n.value else []


__all__ = ["LuceneOptions", "lookup_properties", "analyze"]
