"""Native ingestion: a POSTed entity batch (JSON text) -> the SoA columns dk_upsert takes, in
libdukehip.so's host code (dk_pack_json), without building Record objects (SURVEY §8f row
4).  Semantics: IncrementalDataSource.DatasetDataSourceRecordIterator.next
(IncrementalDataSource.java:50-101) as restated in dukehip.records.records_from_entities;
include/dukehip.h documents the contract.  A batch the native reader does not take (lenient
JSON, characters outside the cleaner tables, a second value for one property) raises
NativeUnsupported: callers pack it with records_from_entities instead.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi as A
from .config import DataSource, UnsupportedComparator
from .records import PartsKey

DK_CLEAN = {None: 0,
            "no.priv.garshol.duke.cleaners.LowerCaseNormalizeCleaner": 1,
            "no.priv.garshol.duke.examples.CountryNameCleaner": 2,
            "no.priv.garshol.duke.examples.CapitalCleaner": 3}
NONE_I32 = -(2 ** 31)


class NativeUnsupported(ValueError):
    """dk_pack_json declined the batch (DK_E_UNSUPPORTED): pack it on the Python path."""


class dk_source_column(C.Structure):
    _fields_ = [("name", C.c_char_p), ("prop", C.c_int32), ("cleaner", C.c_int32)]


class dk_key_part(C.Structure):
    _fields_ = [("prop", C.c_int32), ("token", C.c_int32), ("start", C.c_int32), ("end", C.c_int32)]


class dk_key_function(C.Structure):
    _fields_ = [("nparts", C.c_int32), ("parts", C.POINTER(dk_key_part))]


class dk_source(C.Structure):
    _fields_ = [("dataset_id", C.c_char_p), ("group_no", C.c_int32), ("ncolumns", C.c_int32),
                ("columns", C.POINTER(dk_source_column)), ("nprops", C.c_int32),
                ("nkeys", C.c_int32), ("keys", C.POINTER(dk_key_function))]


class dk_packed(C.Structure):
    _fields_ = [("n", C.c_uint64), ("columns", C.POINTER(A.dk_column)),
                ("key_columns", C.POINTER(A.dk_column)), ("ident", C.POINTER(C.c_uint64)),
                ("deleted", C.POINTER(C.c_uint8)), ("group", C.POINTER(C.c_uint8)),
                ("id", A.dk_column), ("entity_id", A.dk_column)]


_bound = False


def _lib():
    global _bound
    L = A.load()
    if not _bound:
        vp = C.c_void_p
        L.dk_interner_create.argtypes = [C.POINTER(vp)]
        L.dk_interner_create.restype = C.c_int
        L.dk_interner_destroy.argtypes = [vp]
        L.dk_interner_destroy.restype = None
        L.dk_interner_size.argtypes = [vp]
        L.dk_interner_size.restype = C.c_uint64
        L.dk_interner_find.argtypes = [vp, vp, C.c_uint64, C.POINTER(C.c_uint64)]
        L.dk_interner_find.restype = C.c_int
        L.dk_interner_intern.argtypes = [vp, C.POINTER(A.dk_column), C.c_uint64, vp]
        L.dk_interner_intern.restype = C.c_int
        L.dk_pack_json.argtypes = [C.POINTER(dk_source), C.c_char_p, C.c_uint64, vp,
                                   C.POINTER(C.POINTER(dk_packed))]
        L.dk_pack_json.restype = C.c_int
        L.dk_free_packed.argtypes = [C.POINTER(dk_packed)]
        L.dk_free_packed.restype = None
        _bound = True
    return L


class Interner:
    """Exact record-ID interning (string -> dense id), shared by every batch of a database."""

    def __init__(self):
        self.lib = _lib()
        self.h = C.c_void_p()
        A.check(self.lib.dk_interner_create(C.byref(self.h)))

    def __len__(self):
        return int(self.lib.dk_interner_size(self.h))

    def find(self, rid):
        u = np.frombuffer(rid.encode("utf-16-le", "surrogatepass"), dtype=np.uint16)
        out = C.c_uint64()
        rc = self.lib.dk_interner_find(self.h, u.ctypes.data if u.size else None, u.size, C.byref(out))
        return None if rc != 0 else int(out.value)

    def intern(self, ids):
        """Record ID strings -> their ids (new ones interned), as dk_pack_json numbers them."""
        col = A.Column.from_strings(ids)
        out = np.zeros(max(1, len(ids)), dtype=np.uint64)
        c = col.c()
        A.check(self.lib.dk_interner_intern(self.h, C.byref(c), len(ids), out.ctypes.data))
        return out[:len(ids)]

    def close(self):
        if self.h:
            self.lib.dk_interner_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _column_strings(col: A.dk_column, n):
    """A packed dk_column -> list of str / None (diagnostics, record materialisation)."""
    off = np.ctypeslib.as_array(C.cast(col.offsets, C.POINTER(C.c_uint32)), (n + 1,))
    dt = np.uint8 if col.width == 1 else np.uint16
    units = np.ctypeslib.as_array(C.cast(col.units, C.POINTER(C.c_uint8 if col.width == 1 else C.c_uint16)),
                                  (max(1, int(off[-1])),))
    pres = (np.ctypeslib.as_array(C.cast(col.present, C.POINTER(C.c_uint8)), (n,))
            if col.present else None)
    out = []
    for i in range(n):
        if pres is not None and not pres[i]:
            out.append(None)
            continue
        u = np.asarray(units[off[i]:off[i + 1]], dtype=dt)
        out.append(u.tobytes().decode("latin-1") if dt == np.uint8
                   else u.tobytes().decode("utf-16-le", "surrogatepass"))
    return out


class PackedBatch:
    """A dk_packed (library memory, freed on close / GC), ready for dk_upsert."""

    def __init__(self, lib, ptr, nprops, nkeys):
        self.lib, self.ptr = lib, ptr
        p = ptr.contents
        self.n, self.nprops, self.nkeys = int(p.n), nprops, nkeys

    def batch(self, ident=None):
        p = self.ptr.contents
        b = A.dk_batch(self.n, C.cast(p.ident, C.c_void_p) if ident is None else ident,
                       C.cast(p.group, C.c_void_p), C.cast(p.deleted, C.c_void_p),
                       p.columns if self.nprops else None, None,
                       p.key_columns if self.nkeys else None)
        return b

    @property
    def ident(self):
        return np.ctypeslib.as_array(self.ptr.contents.ident, (self.n,)) if self.n else np.zeros(0, np.uint64)

    @property
    def deleted(self):
        return np.ctypeslib.as_array(self.ptr.contents.deleted, (self.n,)) if self.n else np.zeros(0, np.uint8)

    def values(self, prop):
        return _column_strings(self.ptr.contents.columns[prop], self.n)

    def keys(self, k):
        return _column_strings(self.ptr.contents.key_columns[k], self.n)

    def ids(self):
        return _column_strings(self.ptr.contents.id, self.n)

    def entity_ids(self):
        return _column_strings(self.ptr.contents.entity_id, self.n)

    def close(self):
        if self.ptr:
            self.lib.dk_free_packed(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeSource:
    """A data source (+ the schema's scored properties and the key functions) compiled into
    a dk_source.  props: scored property names in schema order; key_functions: PartsKey."""

    def __init__(self, source: DataSource, props, key_functions=()):
        self.lib = _lib()
        names = list(props)
        # properties only key functions read (a column's property no comparator scores):
        # indices nprops + j, kept for the key parts, not packed
        colprops = {c.property for c in source.columns}
        keyonly = []
        for kf in key_functions:
            for prop, *_ in getattr(kf, "parts", ()):
                if prop not in names and prop in colprops and prop not in keyonly:
                    keyonly.append(prop)
        if len(keyonly) > 16:
            raise UnsupportedComparator("more than 16 key-only properties")
        allnames = names + keyonly
        cols = []
        for c in source.columns:
            if c.cleaner not in DK_CLEAN:
                raise UnsupportedComparator(f"cleaner {c.cleaner} has no native implementation")
            cols.append(dk_source_column(c.name.encode("utf-8"),
                                         allnames.index(c.property) if c.property in allnames else -1,
                                         DK_CLEAN[c.cleaner]))
        self._cols = (dk_source_column * max(1, len(cols)))(*cols)
        self._parts, kfs = [], []
        for kf in key_functions:
            if not isinstance(kf, PartsKey):
                raise UnsupportedComparator(f"key function {type(kf).__name__} has no native form")
            parts = []
            for prop, token, start, end in kf.parts:
                if prop not in allnames:
                    raise UnsupportedComparator(f"key part on {prop!r}: no column fills it")
                conv = lambda v: NONE_I32 if v is None else int(v)
                parts.append(dk_key_part(allnames.index(prop), conv(token), conv(start), conv(end)))
            arr = (dk_key_part * max(1, len(parts)))(*parts)
            self._parts.append(arr)
            kfs.append(dk_key_function(len(parts), arr))
        self._kfs = (dk_key_function * max(1, len(kfs)))(*kfs)
        self._ds = source.dataset_id.encode("utf-8")
        self.nprops, self.nkeys = len(names), len(kfs)
        self.src = dk_source(self._ds, int(source.group_no or 0), len(cols), self._cols,
                             self.nprops, self.nkeys, self._kfs)

    def pack(self, body, interner: Interner) -> PackedBatch:
        data = body.encode("utf-8") if isinstance(body, str) else bytes(body)
        out = C.POINTER(dk_packed)()
        rc = self.lib.dk_pack_json(C.byref(self.src), data, len(data), interner.h, C.byref(out))
        if rc == A.DK_E_UNSUPPORTED:
            raise NativeUnsupported(self.lib.dk_last_error().decode("utf-8", "replace"))
        A.check(rc)
        return PackedBatch(self.lib, out, self.nprops, self.nkeys)
