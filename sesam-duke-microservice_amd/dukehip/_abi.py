"""ctypes binding of libdukehip.so (include/dukehip.h).

This is the product path: there is no CPU fallback.  If the shared library is missing or
no GPU is visible, calls raise :class:`DukeHipError` loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("DUKEHIP_LIB", os.path.join(PKG_DIR, "build", "libdukehip.so"))

DK_OK = 0
DK_E_INVALID, DK_E_UNSUPPORTED, DK_E_NOMEM, DK_E_DEVICE, DK_E_STATE = -1, -2, -3, -4, -5

(CMP_NONE, CMP_LEVENSHTEIN, CMP_JAROWINKLER, CMP_QGRAM, CMP_EXACT, CMP_NUMERIC,
 CMP_WEIGHTED_LEVENSHTEIN, CMP_DICE_TOKENS, CMP_JACCARD_TOKENS, CMP_GEOPOSITION) = range(10)
QGRAM_OVERLAP, QGRAM_JACCARD, QGRAM_DICE = 0, 1, 2
QGRAM_BASIC, QGRAM_POSITIONAL, QGRAM_ENDS = 0, 1, 2
MODE_DEDUP, MODE_LINKAGE, MODE_ALLPAIRS = 0, 1, 2
MAX_ORDER_CLASSES = 4   # DK_MAX_ORDER_CLASSES
KIND_MATCH, KIND_MAYBE = 1, 2

MATCH_HOST, MATCH_DEVICE = 0, 1
LUCENE_STATS_MERGED, LUCENE_STATS_UNMERGED = 0, 1
ABI_VERSION = 9   # include/dukehip.h DK_ABI_VERSION

EXPORTS = ("dk_create", "dk_create_multi", "dk_num_devices", "dk_destroy", "dk_upsert", "dk_upsert_transient", "dk_drop_transient",
           "dk_lucene_set_stats", "dk_lucene_merge",
           "dk_match", "dk_candidate_counts", "dk_result_copy_to_device",
           "dk_free_result", "dk_result_region_layout", "dk_set_result_region",
           "dk_compare_rows", "dk_compare_values", "dk_property_similarity", "dk_set_overwrite", "dk_num_rows", "dk_row_of_ident", "dk_set_profiling", "dk_get_profile",
           "dk_reset_profile", "dk_last_error", "dk_abi_version",
           "dk_interner_create", "dk_interner_destroy", "dk_interner_size", "dk_interner_find",
           "dk_interner_intern", "dk_pack_json", "dk_free_packed", "dk_interner_string",
           "dk_linkdb_create", "dk_linkdb_destroy", "dk_linkdb_size", "dk_linkdb_apply",
           "dk_linkdb_changes_since", "dk_free_link_list", "dk_linkdb_links_for",
           "dk_linkdb_retract", "dk_lucene_analyze")


class DukeHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"dukehip error {code}: {msg}")
        self.code = code


class dk_property(C.Structure):
    _fields_ = [("comparator", C.c_int32), ("qgram_q", C.c_int32), ("qgram_formula", C.c_int32),
                ("qgram_tokenizer", C.c_int32), ("low", C.c_double), ("high", C.c_double),
                ("min_ratio", C.c_double)]


class dk_lucene(C.Structure):
    _fields_ = [("nlookup", C.c_int32), ("lookup_prop", C.POINTER(C.c_int32)),
                ("max_hits", C.c_int32), ("min_relevance", C.c_float)]


class dk_schema(C.Structure):
    _fields_ = [("nprops", C.c_int32), ("props", C.POINTER(dk_property)),
                ("threshold", C.c_double), ("maybe_threshold", C.c_double),
                ("mode", C.c_int32), ("nkeys", C.c_int32), ("lucene", C.POINTER(dk_lucene)),
                ("norders", C.c_int32), ("orders", C.POINTER(C.c_int32))]


def order_classes(schema, orders):
    """Give `schema` (a dk_schema) per order class the visiting order of its properties
    (dk_schema.orders; indices into schema.props)."""
    n = schema.nprops
    flat = (C.c_int32 * max(1, len(orders) * n))(*[int(x) for o in orders for x in o])
    schema.norders = len(orders)
    schema.orders = flat
    schema._keep_orders = flat
    return schema


def lucene_source(schema, lookup_props, max_hits=10, min_relevance=0.9):
    """Switch `schema` (a dk_schema with nkeys 0) to the Lucene-compatible candidate source
    over the schema properties `lookup_props` (indices, lookup order)."""
    idx = (C.c_int32 * max(1, len(lookup_props)))(*lookup_props)
    lu = dk_lucene(len(lookup_props), idx, int(max_hits), float(min_relevance))
    schema.lucene = C.pointer(lu)
    schema._keep_lucene = (idx, lu)
    return schema


class dk_column(C.Structure):
    _fields_ = [("offsets", C.c_void_p), ("units", C.c_void_p), ("width", C.c_int32),
                ("present", C.c_void_p)]


class dk_batch(C.Structure):
    _fields_ = [("n", C.c_uint64), ("ident", C.c_void_p), ("group", C.c_void_p),
                ("deleted", C.c_void_p), ("columns", C.POINTER(dk_column)),
                ("keys", C.c_void_p), ("key_columns", C.POINTER(dk_column)),
                ("order_class", C.c_void_p)]


class dk_result(C.Structure):
    _fields_ = [("nqueries", C.c_uint64), ("n", C.c_uint64), ("first", C.POINTER(C.c_uint64)),
                ("candidate", C.POINTER(C.c_uint32)), ("prob", C.POINTER(C.c_double)),
                ("kind", C.POINTER(C.c_uint8)), ("pairs_scored", C.c_uint64),
                ("pairs_generated", C.c_uint64)]


class dk_region_layout(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("first_offset", C.c_uint64),
                ("prob_offset", C.c_uint64), ("candidate_offset", C.c_uint64),
                ("kind_offset", C.c_uint64)]


class dk_profile(C.Structure):
    _fields_ = [("ms_index", C.c_double), ("ms_generate", C.c_double), ("ms_score", C.c_double),
                ("ms_gather", C.c_double), ("ms_total", C.c_double),
                ("score_launches", C.c_uint64), ("pairs_scored", C.c_uint64),
                ("pairs_generated", C.c_uint64), ("score_bytes", C.c_uint64),
                ("ms_copy", C.c_double), ("ms_emit", C.c_double), ("sym_matches", C.c_uint64),
                ("full_builds", C.c_uint64), ("delta_builds", C.c_uint64),
                ("replica_positions", C.c_uint64), ("gram_row_bytes", C.c_uint64),
                ("sym2_matches", C.c_uint64), ("pairs_exact", C.c_uint64)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


_lib = None


def load():
    """Load libdukehip.so (built by __graft_entry__.build() / `make -C csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("DUKEHIP_LIB") or LIB_PATH   # A/B builds (`make -C csrc variant`)
    if not os.path.exists(path):
        raise DukeHipError(DK_E_STATE, f"{path} not built: run `make -C "
                           f"{os.path.join(PKG_DIR, 'csrc')}` or __graft_entry__.build()")
    L = C.CDLL(path)
    vp = C.c_void_p
    L.dk_create.argtypes = [C.POINTER(dk_schema), C.c_int, C.POINTER(vp)]
    L.dk_create_multi.argtypes = [C.POINTER(dk_schema), C.POINTER(C.c_int), C.c_int, C.POINTER(vp)]
    L.dk_create_multi.restype = C.c_int
    L.dk_num_devices.argtypes = [vp]
    L.dk_num_devices.restype = C.c_int
    L.dk_destroy.argtypes = [vp]
    L.dk_destroy.restype = None
    L.dk_upsert.argtypes = [vp, C.POINTER(dk_batch), vp]
    L.dk_upsert_transient.argtypes = [vp, C.POINTER(dk_batch), vp]
    L.dk_drop_transient.argtypes = [vp]
    L.dk_lucene_set_stats.argtypes = [vp, C.c_int]
    L.dk_lucene_merge.argtypes = [vp]
    L.dk_match.argtypes = [vp, vp, C.c_uint64, C.c_int, C.POINTER(C.POINTER(dk_result))]
    L.dk_candidate_counts.argtypes = [vp, vp, C.c_uint64, vp]
    L.dk_candidate_counts.restype = C.c_int
    L.dk_result_copy_to_device.argtypes = [C.POINTER(dk_result), vp, vp, vp, vp]
    L.dk_result_copy_to_device.restype = C.c_int
    L.dk_free_result.argtypes = [C.POINTER(dk_result)]
    L.dk_free_result.restype = None
    L.dk_result_region_layout.argtypes = [C.c_uint64, C.c_uint64, C.POINTER(dk_region_layout)]
    L.dk_set_result_region.argtypes = [vp, vp, C.c_uint64, C.c_uint64]
    L.dk_compare_rows.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(C.c_double)]
    L.dk_compare_values.argtypes = [vp, C.POINTER(dk_batch), C.POINTER(C.c_double)]
    L.dk_set_overwrite.argtypes = [vp, C.c_int]
    L.dk_property_similarity.argtypes = [vp, C.c_int, C.c_uint32, C.c_uint32, C.POINTER(C.c_double)]
    L.dk_num_rows.argtypes = [vp]
    L.dk_num_rows.restype = C.c_uint64
    L.dk_row_of_ident.argtypes = [vp, C.c_uint64, C.POINTER(C.c_uint32)]
    L.dk_row_of_ident.restype = C.c_int
    L.dk_set_profiling.argtypes = [vp, C.c_int]
    L.dk_get_profile.argtypes = [vp, C.POINTER(dk_profile)]
    L.dk_reset_profile.argtypes = [vp]
    L.dk_last_error.restype = C.c_char_p
    L.dk_abi_version.restype = C.c_int
    for f in ("dk_create", "dk_upsert", "dk_upsert_transient", "dk_drop_transient", "dk_match",
              "dk_lucene_set_stats", "dk_lucene_merge",
              "dk_compare_rows", "dk_compare_values", "dk_property_similarity", "dk_set_overwrite",
              "dk_set_profiling",
              "dk_result_region_layout", "dk_set_result_region",
              "dk_get_profile", "dk_reset_profile"):
        getattr(L, f).restype = C.c_int
    if L.dk_abi_version() != ABI_VERSION:   # the struct layouts below are this version's
        raise ImportError(f"{path}: ABI version {L.dk_abi_version()}, dukehip expects {ABI_VERSION}")
    _lib = L
    return L


def check(rc):
    if rc != DK_OK:
        raise DukeHipError(rc, load().dk_last_error().decode("utf-8", "replace"))
    return rc


def region_layout(nbytes, max_queries):
    """dk_result_region_layout: where a result region keeps first / prob / candidate / kind."""
    out = dk_region_layout()
    check(load().dk_result_region_layout(int(nbytes), int(max_queries), C.byref(out)))
    return {name: int(getattr(out, name)) for name, _ in out._fields_}


def region_bytes(max_queries, capacity):
    """Smallest region holding max_queries queries and `capacity` entries."""
    return (int(max_queries) + 1) * 8 + int(capacity) * 13


def region_views(buf, max_queries, nq, n):
    """numpy views of a result region (any buffer, e.g. another rank's slice of a shared
    mapping): first[nq+1], candidate[n], prob[n], kind[n]."""
    lay = region_layout(len(buf), max_queries)
    if n > lay["capacity"] or nq > max_queries:
        raise ValueError("result larger than its region")
    b = np.frombuffer(buf, dtype=np.uint8)
    return {"first": b[:(nq + 1) * 8].view(np.uint64),
            "candidate": b[lay["candidate_offset"]:lay["candidate_offset"] + 4 * n].view(np.uint32),
            "prob": b[lay["prob_offset"]:lay["prob_offset"] + 8 * n].view(np.float64),
            "kind": b[lay["kind_offset"]:lay["kind_offset"] + n]}


def ptr(a):
    return None if a is None else a.ctypes.data


class Column:
    """Packed values of one property for a batch (owns its numpy buffers)."""

    def __init__(self, offsets, units, present=None):
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        self.units = np.ascontiguousarray(units)
        if self.units.dtype not in (np.uint8, np.uint16):
            raise ValueError("units must be uint8 or uint16")
        if self.units.size == 0:
            self.units = np.zeros(1, dtype=self.units.dtype)
        self.present = None if present is None else np.ascontiguousarray(present, dtype=np.uint8)

    @classmethod
    def from_strings(cls, values):
        """values: iterable of str or None.  Latin-1-only columns pack one byte per unit.

        One join + one encode for the whole column (no per-value encode): a Latin-1 column's
        per-value unit counts are the str lengths; a UTF-16 column's are too unless it holds
        characters outside the BMP (two units each), which falls back to per-value lengths."""
        vals = list(values)
        anymiss = None in vals
        missing = [v is None for v in vals] if anymiss else None
        joined = "".join("" if v is None else v for v in vals) if anymiss else "".join(vals)
        n = len(vals)
        try:
            units = np.frombuffer(joined.encode("latin-1"), dtype=np.uint8)
            lens = np.fromiter(((0 if v is None else len(v)) for v in vals) if anymiss
                               else map(len, vals), dtype=np.int64, count=n)
        except UnicodeEncodeError:
            units = np.frombuffer(joined.encode("utf-16-le", "surrogatepass"), dtype=np.uint16)
            if units.size == len(joined):
                lens = np.fromiter(((0 if v is None else len(v)) for v in vals), dtype=np.int64,
                                   count=n)
            else:
                lens = np.fromiter(((0 if v is None else
                                     len(v.encode("utf-16-le", "surrogatepass")) // 2)
                                    for v in vals), dtype=np.int64, count=n)
        offs = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        if units.size == 0:
            units = np.zeros(1, dtype=units.dtype)
        present = None
        if anymiss:
            present = (~np.asarray(missing, dtype=bool)).astype(np.uint8)
        return cls(offs, units, present)

    @classmethod
    def from_strings_per_value(cls, values):
        """Reference packing, one encode per value (tests compare from_strings with it)."""
        vals = list(values)
        enc = []
        wide = False
        for v in vals:
            if v is None:
                enc.append(None)
                continue
            b = v.encode("utf-16-le", "surrogatepass")
            u = np.frombuffer(b, dtype=np.uint16)
            if u.size and int(u.max()) > 0xFF:
                wide = True
            enc.append(u)
        dt = np.uint16 if wide else np.uint8
        lens = np.array([0 if u is None else u.size for u in enc], dtype=np.int64)
        offs = np.zeros(len(vals) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        units = np.concatenate([u for u in enc if u is not None]).astype(dt) if any(
            u is not None and u.size for u in enc) else np.zeros(1, dtype=dt)
        present = np.array([u is not None for u in enc], dtype=np.uint8)
        return cls(offs, units, None if present.all() else present)

    def c(self):
        return dk_column(ptr(self.offsets), ptr(self.units), self.units.itemsize,
                         ptr(self.present))
