"""Host mirror of the Duke contracts the microservice drives, backed by libdukehip.so.

* ``GpuBlockingDatabase``  <- Duke ``Database`` as IncrementalLuceneDatabase implements it
  (setConfiguration :90, setOverwrite :99, isInMemory :139, commit :146,
  findRecordById :170, close :186, index :498): records are column-packed into the
  device-resident index; upsert by ID; key-function blocking replaces the Lucene query.
* ``GpuProcessor``         <- ``no.priv.garshol.duke.Processor`` as constructed and driven
  at App.java:342-345, 354, 1005, 1159: ``deduplicate(records)`` runs the whole batch on the
  GPU and replays the MatchListener callbacks in Duke's order on the calling thread.
* ``MatchListener``        <- the 7 callbacks of BaseLinkDatabaseMatchListener.java:53-109.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi as A
from .config import DukeConfig, ID_PROPERTY, GROUP_NO_PROPERTY_NAME, DELETED_PROPERTY_NAME
from .config import ORIGINAL_ENTITY_ID_PROPERTY_NAME, DATASET_ID_PROPERTY_NAME
from .ingest import Interner, NativeSource
from .records import Record


class MatchListener:
    """[Duke 1.2] matchers.MatchListener."""

    def batch_ready(self, size):
        pass

    def batch_done(self):
        pass

    def matches(self, r1, r2, confidence):
        pass

    def matches_perhaps(self, r1, r2, confidence):
        pass

    def no_match_for(self, record):
        pass

    def start_processing(self):
        pass

    def end_processing(self):
        pass


class CollectingListener(MatchListener):
    """Records every callback in order (what the reference's listeners observe)."""

    def __init__(self):
        self.events = []

    def batch_ready(self, size):
        self.events.append(("batchReady", size))

    def batch_done(self):
        self.events.append(("batchDone",))

    def matches(self, r1, r2, confidence):
        self.events.append(("matches", r1.get_value(ID_PROPERTY), r2.get_value(ID_PROPERTY), confidence))

    def matches_perhaps(self, r1, r2, confidence):
        self.events.append(("matchesPerhaps", r1.get_value(ID_PROPERTY), r2.get_value(ID_PROPERTY), confidence))

    def no_match_for(self, record):
        self.events.append(("noMatchFor", record.get_value(ID_PROPERTY)))


class MatchResult:
    """A dk_result: entries grouped per query (query order).  The arrays are zero-copy
    views of the library's pinned result memory, valid until :meth:`close` (called on
    garbage collection), which hands the memory back to the ctx's pool."""

    def __init__(self, lib, res, queries):
        self._lib, self._res = lib, res
        r = res.contents
        n, nq = r.n, r.nqueries
        self.n, self.nqueries = n, nq
        self.queries = queries
        self.pairs_scored, self.pairs_generated = r.pairs_scored, r.pairs_generated
        self.on_device = not bool(r.first)
        view = np.ctypeslib.as_array
        if self.on_device:
            self.first = self.candidate = self.prob = self.kind = None
        else:
            self.first = view(r.first, (nq + 1,))
            self.candidate = view(r.candidate, (n,)) if n else np.zeros(0, np.uint32)
            self.prob = view(r.prob, (n,)) if n else np.zeros(0, np.float64)
            self.kind = view(r.kind, (n,)) if n else np.zeros(0, np.uint8)

    @property
    def query(self):
        """Row of r1 for every entry (expanded from `first`)."""
        return np.repeat(np.asarray(self.queries, np.uint32), np.diff(self.first).astype(np.int64))

    def copy_to_device(self, first=None, candidate=None, prob=None, kind=None):
        """Device-to-device copy into caller buffers (device pointers as ints)."""
        A.check(self._lib.dk_result_copy_to_device(self._res, first, candidate, prob, kind))

    def close(self):
        if self._res is not None:
            self.first = self.candidate = self.prob = self.kind = None
            self._lib.dk_free_result(self._res)
            self._res = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GpuEngine:
    """Thin owner of one dk_ctx (one pipeline): on one device, or -- `devices`, a list --
    replicated over several devices of this process (dk_create_multi: one handle, the
    query tiles matched concurrently, one list back)."""

    def __init__(self, schema, device=0, devices=None):
        self.lib = A.load()
        self.ctx = C.c_void_p()
        if devices is not None:
            dv = (C.c_int * len(devices))(*[int(d) for d in devices])
            A.check(self.lib.dk_create_multi(C.byref(schema), dv, len(devices), C.byref(self.ctx)))
        else:
            A.check(self.lib.dk_create(C.byref(schema), int(device), C.byref(self.ctx)))
        self._schema = schema

    @property
    def num_devices(self):
        return int(self.lib.dk_num_devices(self.ctx))

    def close(self):
        if self.ctx:
            self.lib.dk_destroy(self.ctx)
            self._region = None
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_rows(self):
        return int(self.lib.dk_num_rows(self.ctx))

    def upsert(self, n, ident, columns, group=None, deleted=None, keys=None, key_columns=None,
               transient=False, order_class=None):
        """columns: list of A.Column (schema order); keys: uint64 array [nkeys, n] or
        key_columns: list of A.Column.  Returns the assigned rows.  transient=True appends
        query-only rows (dk_upsert_transient) that :meth:`drop_transient` removes.
        order_class: per record its Processor.compare order class (dk_schema.orders)."""
        ident = np.ascontiguousarray(ident, dtype=np.uint64)
        oc = None if order_class is None else np.ascontiguousarray(order_class, dtype=np.uint8)
        group = None if group is None else np.ascontiguousarray(group, dtype=np.uint8)
        deleted = None if deleted is None else np.ascontiguousarray(deleted, dtype=np.uint8)
        cols = (A.dk_column * max(1, len(columns)))(*[c.c() for c in columns])
        kc = None
        kptr = None
        if keys is not None:
            keys = np.ascontiguousarray(keys, dtype=np.uint64)
            kptr = keys.ctypes.data
        if key_columns is not None:
            kc = (A.dk_column * max(1, len(key_columns)))(*[c.c() for c in key_columns])
        b = A.dk_batch(n, ident.ctypes.data, A.ptr(group), A.ptr(deleted), cols, kptr, kc, A.ptr(oc))
        rows = np.zeros(max(1, n), dtype=np.uint32)
        fn = self.lib.dk_upsert_transient if transient else self.lib.dk_upsert
        A.check(fn(self.ctx, C.byref(b), rows.ctypes.data))
        return rows[:n]

    def upsert_packed(self, packed, transient=False):
        """dk_upsert of a natively packed batch (dukehip.ingest.PackedBatch)."""
        b = packed.batch()
        rows = np.zeros(max(1, packed.n), dtype=np.uint32)
        fn = self.lib.dk_upsert_transient if transient else self.lib.dk_upsert
        A.check(fn(self.ctx, C.byref(b), rows.ctypes.data))
        return rows[:packed.n]

    def row_of_ident(self, ident):
        """dk_row_of_ident: the row of the live version of an interned record ID, or None."""
        out = C.c_uint32()
        rc = self.lib.dk_row_of_ident(self.ctx, int(ident), C.byref(out))
        return None if rc != 0 else int(out.value)

    def drop_transient(self):
        A.check(self.lib.dk_drop_transient(self.ctx))

    def lucene_stats(self, unmerged):
        """dk_lucene_set_stats: Lucene collection statistics of a merged index (default), or
        unmerged -- superseded versions keep counting in maxDoc / docFreq until lucene_merge."""
        A.check(self.lib.dk_lucene_set_stats(self.ctx, A.LUCENE_STATS_UNMERGED if unmerged
                                             else A.LUCENE_STATS_MERGED))

    def lucene_merge(self):
        """dk_lucene_merge (IndexWriter.forceMerge): superseded versions leave the statistics."""
        A.check(self.lib.dk_lucene_merge(self.ctx))

    def match(self, query_rows, on_device=False):
        q = np.ascontiguousarray(query_rows, dtype=np.uint32)
        res = C.POINTER(A.dk_result)()
        A.check(self.lib.dk_match(self.ctx, q.ctypes.data if q.size else None, q.size,
                                  A.MATCH_DEVICE if on_device else A.MATCH_HOST, C.byref(res)))
        return MatchResult(self.lib, res, q)

    def candidate_counts(self, query_rows):
        """dk_candidate_counts: per query, the candidates blocking produces (cost model of
        the multi-GPU tiles)."""
        q = np.ascontiguousarray(query_rows, dtype=np.uint32)
        out = np.zeros(max(1, q.size), dtype=np.uint64)
        A.check(self.lib.dk_candidate_counts(self.ctx, q.ctypes.data if q.size else None, q.size,
                                             out.ctypes.data))
        return out[:q.size]

    def set_result_region(self, buf, max_queries):
        """dk_set_result_region: host-mode match lists land in `buf` (a writable buffer, e.g.
        this rank's slice of a node-wide shared mapping) instead of the library's pool.
        buf=None goes back to the pool.  The engine keeps a reference to `buf`."""
        if buf is None:
            A.check(self.lib.dk_set_result_region(self.ctx, None, 0, 0))
            self._region = None
            return
        arr = np.frombuffer(buf, dtype=np.uint8)
        A.check(self.lib.dk_set_result_region(self.ctx, arr.ctypes.data, arr.size, int(max_queries)))
        self._region = (buf, arr)

    def compare_rows(self, r1, r2):
        out = C.c_double()
        A.check(self.lib.dk_compare_rows(self.ctx, int(r1), int(r2), C.byref(out)))
        return out.value

    def compare_values(self, columns, order_class=(0, 0)):
        """dk_compare_values: Processor.compare(r1, r2) of two records given as columns of
        two values each (schema order; None = no value), r1's order class first.  The index
        is not touched."""
        cols = (A.dk_column * max(1, len(columns)))(*[c.c() for c in columns])
        ident = np.zeros(2, np.uint64)
        oc = np.ascontiguousarray(order_class, dtype=np.uint8)
        b = A.dk_batch(2, ident.ctypes.data, None, None, cols, None, None, oc.ctypes.data)
        out = C.c_double()
        A.check(self.lib.dk_compare_values(self.ctx, C.byref(b), C.byref(out)))
        return out.value

    def set_overwrite(self, on):
        A.check(self.lib.dk_set_overwrite(self.ctx, 1 if on else 0))

    def property_similarity(self, prop, r1, r2):
        """dk_property_similarity: Comparator.compare of schema property `prop` (index into
        the schema order) for two indexed rows; NaN when either value is missing/empty."""
        out = C.c_double()
        A.check(self.lib.dk_property_similarity(self.ctx, int(prop), int(r1), int(r2), C.byref(out)))
        return out.value

    def set_profiling(self, on):
        """on: False / True (every phase), or 2 (the scoring kernels only)."""
        A.check(self.lib.dk_set_profiling(self.ctx, 2 if on == 2 and on is not True else (1 if on else 0)))

    def profile(self):
        p = A.dk_profile()
        A.check(self.lib.dk_get_profile(self.ctx, C.byref(p)))
        return p.as_dict()

    def reset_profile(self):
        A.check(self.lib.dk_reset_profile(self.ctx))


class RowStore:
    """row -> Record for every indexed (and transient) row: Record objects of batches packed
    in Python, and natively packed batches (dukehip.ingest) whose Records are built only
    when a row is looked at (a listener callback, findRecordById)."""

    def __init__(self, props):
        self.props = props          # scored property names, schema order
        self.segs = []              # (row0, n, list of Record | (PackedBatch, [groupNo]))
        self.n = 0

    def append_records(self, recs):
        self.segs.append((self.n, len(recs), list(recs)))
        self.n += len(recs)

    def append_packed(self, packed, group_no=None, dataset_id=None):
        self.segs.append((self.n, packed.n, (packed, group_no, dataset_id)))
        self.n += packed.n

    def truncate(self, n):
        """Drop rows n.. (dk_drop_transient)."""
        while self.segs and self.segs[-1][0] >= n:
            self.segs.pop()
        if self.segs and self.segs[-1][0] + self.segs[-1][1] > n:
            r0, cnt, pay = self.segs[-1]
            self.segs[-1] = (r0, n - r0, pay[:n - r0] if isinstance(pay, list) else pay)
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, row):
        if isinstance(row, slice):
            return [self[i] for i in range(*row.indices(self.n))]
        if row < 0:
            row += self.n
        lo, hi = 0, len(self.segs)
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if self.segs[mid][0] <= row:
                lo = mid
            else:
                hi = mid
        r0, cnt, pay = self.segs[lo]
        if not (0 <= row - r0 < cnt):
            raise IndexError(row)
        if isinstance(pay, list):
            return pay[row - r0]
        return self._materialise(pay, row - r0)

    def _materialise(self, pay, i):
        packed, group_no, dataset_id = pay
        cache = getattr(packed, "_cols", None)
        if cache is None:
            cache = packed._cols = ([packed.values(p) for p in range(len(self.props))],
                                    packed.ids(), packed.entity_ids())
        vals, ids, eids = cache
        rec = Record({n: v[i] for n, v in zip(self.props, vals) if v[i] is not None})
        if group_no:
            rec.add_value(GROUP_NO_PROPERTY_NAME, str(group_no))
        rec.add_value(ID_PROPERTY, ids[i])
        rec.add_value(ORIGINAL_ENTITY_ID_PROPERTY_NAME, eids[i])
        # the source's dataset id as IncrementalDataSource sets it (:90), not parsed back out
        # of the record ID (a dataset id may itself contain "__")
        rec.add_value(DATASET_ID_PROPERTY_NAME, dataset_id)
        if packed.deleted[i]:
            rec.add_value(DELETED_PROPERTY_NAME, "true")
        return rec


class GpuBlockingDatabase:
    """Duke ``Database`` with key-function blocking, resident in HBM.

    ``index`` buffers records; ``commit`` upserts them (delete-by-ID then add,
    IncrementalLuceneDatabase.java:516-517, 578-590).  Records marked
    dukeDeleted=true stay indexed but are never candidates (:478)."""

    def __init__(self, config: DukeConfig, key_functions=(), mode=None, device=0, lucene=None,
                 devices=None):
        """key_functions: Duke blocking key functions (the GPU blocking contract); none ->
        the reference's own Lucene candidate semantics (IncrementalLuceneDatabase.
        findCandidateMatches, dukehip.lucene; `lucene` = LuceneOptions, default from the
        environment like App.configureDatabase).  devices: a list of GPUs of this process to
        replicate the index over (dk_create_multi), instead of the one `device`."""
        self.config = config
        self.key_functions = list(key_functions or ())
        if mode is None:
            mode = A.MODE_LINKAGE if config.linkage else A.MODE_DEDUP
        self.mode = mode
        nkeys = 0 if mode == A.MODE_ALLPAIRS else len(self.key_functions)
        self.schema, self.props = config.to_schema(mode, nkeys)
        self.caps = config.order_classes()[0]   # HashMap capacities -> order classes
        self.lookup = None
        if mode != A.MODE_ALLPAIRS and not self.key_functions:
            from .lucene import LuceneOptions, lookup_properties
            opts = lucene or LuceneOptions.from_env()
            opts.check()
            self.lookup = lookup_properties(config, self.props)
            if not self.lookup:
                raise ValueError("no lookup properties: the Lucene query would match nothing")
            idx = {p.name: i for i, p in enumerate(self.props)}
            A.lucene_source(self.schema, [idx[n] for n in self.lookup], opts.max_hits, opts.min_relevance)
        self.engine = GpuEngine(self.schema, device, devices=devices)
        self.pending = []
        self.rows = RowStore([p.name for p in self.props])   # row -> Record
        self.ids = Interner()   # ID string -> dense identity number (both packing paths)
        self.row_ident = np.zeros(0, np.uint64)   # row -> its record ID's interned id
        self._native = {}       # DataSource id -> NativeSource
        self.overwrite = False
        self.indexing_disabled = False
        self._transient_row0 = None

    # --- Database API (IncrementalLuceneDatabase.java) ---
    def set_indexing_is_disabled(self, disabled):
        """IncrementalLuceneDatabase.setIndexingIsDisabled (:95): while disabled, index()
        is a no-op (:499-502) and a processed batch is matched without entering the
        index (App.java:1130-1132, the httptransform endpoint)."""
        self.indexing_disabled = bool(disabled)
        if not self.indexing_disabled:
            self.drop_transient()

    def set_overwrite(self, overwrite):
        """Database.setOverwrite (IncrementalLuceneDatabase.java:99): with overwrite on,
        index() adds a record without first deleting the previous version by ID (:515)."""
        self.overwrite = bool(overwrite)
        self.engine.set_overwrite(self.overwrite)

    def is_in_memory(self):
        return True

    def index(self, record: Record):
        if self.indexing_disabled:
            return
        self.pending.append(record)

    def commit(self):
        recs, self.pending = self.pending, []
        return self.index_batch(recs)

    def find_record_by_id(self, rid):
        """IncrementalLuceneDatabase.findRecordById (:170-180): the row the index's ID map
        holds for the ID (dk_row_of_ident -- one source of truth for both packing paths: the
        live version, or the oldest under setOverwrite(true), Lucene's first hit)."""
        ident = self.ids.find(rid)
        row = None if ident is None else self.engine.row_of_ident(ident)
        return None if row is None else self.rows[row]

    def close(self):
        self.engine.close()

    def drop_transient(self):
        """Removes the query-only rows of a batch processed with indexing disabled."""
        if self._transient_row0 is not None:
            self.engine.drop_transient()
            self.rows.truncate(self._transient_row0)
            self.row_ident = self.row_ident[:self._transient_row0]
            self._transient_row0 = None

    # --- bulk path ---
    def index_batch(self, records, transient=None):
        """Column-packs and upserts `records`; with indexing disabled (or transient=True)
        they become query-only rows instead.  Returns their rows."""
        transient = self.indexing_disabled if transient is None else bool(transient)
        n = len(records)
        if n == 0:
            return np.zeros(0, np.uint32)
        rids = [r.get_value(ID_PROPERTY) for r in records]
        if any(rid is None for rid in rids):
            raise ValueError("record without ID property")
        ident = self.ids.intern(rids)
        cols = []
        for p in self.props:
            vals = []
            for r in records:
                vs = r.get_values(p.name)
                if len(vs) > 1:
                    raise ValueError(f"property {p.name}: {len(vs)} values (GPU path holds one)")
                vals.append(vs[0] if vs else None)
            cols.append(A.Column.from_strings(vals))
        group = None
        if self.mode == A.MODE_LINKAGE:
            # dukeGroupNo is "1" or "2" (IncrementalDataSource.java:80-84); a record without
            # it makes findCandidateMatches throw (IncrementalLuceneDatabase.java:469-471)
            gs = [r.get_value(GROUP_NO_PROPERTY_NAME) for r in records]
            bad = [g for g in gs if g not in ("1", "2")]
            if bad:
                raise ValueError(f"The '{GROUP_NO_PROPERTY_NAME}' property was missing or not "
                                 f"1/2: {bad[0]!r}")
            group = np.array([int(g) for g in gs], dtype=np.uint8)
        deleted = np.array([r.get_value(DELETED_PROPERTY_NAME) == "true" for r in records],
                           dtype=np.uint8)
        key_cols = None
        if self.mode != A.MODE_ALLPAIRS and self.key_functions:
            key_cols = [A.Column.from_strings([kf.make_key(r) for r in records])
                        for kf in self.key_functions]
        oc = None
        if len(self.caps) > 1:   # Processor.compare follows each query record's HashMap order
            oc = np.array([self.config.record_class(r, self.caps) for r in records], np.uint8)
        rows = self.engine.upsert(n, ident, cols, group=group, deleted=deleted,
                                  key_columns=key_cols, transient=transient, order_class=oc)
        if transient and self._transient_row0 is None:
            self._transient_row0 = len(self.rows)
        self.rows.append_records(records)
        self.row_ident = np.concatenate([self.row_ident, np.asarray(ident, np.uint64)])
        return rows

    def native_source(self, source):
        ns = self._native.get(id(source))
        if ns is None:
            ns = self._native[id(source)] = (NativeSource(source, [p.name for p in self.props],
                                                          self.key_functions), source)
        return ns[0]

    def index_json(self, body, source, transient=None):
        """The POSTed batch `body` (JSON text) of data source `source`, packed natively
        (dk_pack_json) and upserted (or appended as transient rows).  Returns (rows,
        packed).  Raises dukehip.ingest.NativeUnsupported for a batch the native reader
        declines (the caller then uses records_from_entities + index_batch)."""
        transient = self.indexing_disabled if transient is None else bool(transient)
        if len(self.caps) > 1:   # the native packer does not count a record's properties
            from .ingest import NativeUnsupported
            raise NativeUnsupported("several HashMap order classes: records path")
        packed = self.native_source(source).pack(body, self.ids)
        if packed.n == 0:
            return np.zeros(0, np.uint32), packed
        if self.mode == A.MODE_LINKAGE and not source.group_no:
            raise ValueError(f"The '{GROUP_NO_PROPERTY_NAME}' property was missing")
        rows = self.engine.upsert_packed(packed, transient=transient)
        if transient and self._transient_row0 is None:
            self._transient_row0 = len(self.rows)
        self.rows.append_packed(packed, source.group_no, source.dataset_id)
        self.row_ident = np.concatenate([self.row_ident, np.asarray(packed.ident, np.uint64)])
        return rows, packed


class _RowView:
    """records[i] of a batch whose rows are row0 .. row0+n-1 of a RowStore."""

    def __init__(self, rows, row0, n):
        self.rows, self.row0, self.n = rows, row0, n

    def __len__(self):
        return self.n

    def __iter__(self):
        return (self.rows[self.row0 + i] for i in range(self.n))

    def __getitem__(self, i):
        return self.rows[self.row0 + i]


class GpuProcessor:
    """``no.priv.garshol.duke.Processor`` with the matching loop on the GPU."""

    def __init__(self, config: DukeConfig, database: GpuBlockingDatabase):
        self.config = config
        self.database = database
        self.listeners = []
        self.threads = 1
        self.profiling = False
        self.link_database = None

    def add_match_listener(self, listener):
        self.listeners.append(listener)

    def get_database(self):
        return self.database

    def set_link_database(self, link_database):
        """The pipeline's LinkDatabase (dukehip.links.LinkDatabase), written in bulk after each
        batch's match -- what BaseLinkDatabaseMatchListener's wrapped
        LinkDatabaseMatchListener does per callback (BaseLinkDatabaseMatchListener.java:50,
        53-109).  Skipped while indexing is disabled (httptransform: App.java:1131-1132)."""
        self.link_database = link_database

    def _write_links(self, rows, res):
        db = self.database
        if self.link_database is not None and not db.indexing_disabled:
            self.link_database.apply_result(res, db.row_ident[np.asarray(rows, np.int64)], db.row_ident)

    def set_threads(self, n):
        self.threads = int(n)  # the GPU path does not use host threads for matching

    def set_performance_profiling(self, on):
        self.profiling = bool(on)
        self.database.engine.set_profiling(on)

    def get_profile(self):
        return self.database.engine.profile()

    def deduplicate(self, records):
        """[Duke 1.2] Processor.deduplicate(Collection<Record>): batchReady, index +
        commit every record, match each against the index (matchall), batchDone."""
        records = list(records)
        for l in self.listeners:
            l.batch_ready(len(records))
        # index every record, then commit (IncrementalLuceneDatabase.java:498-575, 146-165):
        # records handed to database.index() beforehand -- the deleted records of
        # App.java:988-1001, 1121-1137 -- become visible in the same commit
        db = self.database
        pending, db.pending = db.pending, []
        rows = db.index_batch(pending + records)[len(pending):]
        res = db.engine.match(rows)
        self._replay(records, res)
        self._write_links(rows, res)
        for l in self.listeners:
            l.batch_done()
        if self.database.indexing_disabled:
            self.database.drop_transient()   # the batch never entered the index
        return res

    def deduplicate_json(self, body, source):
        """Processor.deduplicate of a POSTed batch given as JSON text: packed natively
        (dk_pack_json, no Record objects on the way in), then the same index + commit +
        match + callback replay as deduplicate().  Records handed to the listeners are
        built only for the rows they name."""
        db = self.database
        pending, db.pending = db.pending, []
        if pending:
            db.index_batch(pending)
        rows, packed = db.index_json(body, source)
        n = len(rows)
        for l in self.listeners:
            l.batch_ready(n)
        res = db.engine.match(rows)
        if self.listeners:
            row0 = int(rows[0]) if n else 0
            self._replay(_RowView(db.rows, row0, n), res)
        self._write_links(rows, res)
        for l in self.listeners:
            l.batch_done()
        if db.indexing_disabled:
            db.drop_transient()
        return res

    def _replay(self, records, res: MatchResult):
        rows = self.database.rows
        for i, r in enumerate(records):
            a, b = int(res.first[i]), int(res.first[i + 1])
            if a == b:
                for l in self.listeners:
                    l.no_match_for(r)
                continue
            for e in range(a, b):
                cand = rows[int(res.candidate[e])]
                p = float(res.prob[e])
                for l in self.listeners:
                    if res.kind[e] == A.KIND_MATCH:
                        l.matches(r, cand, p)
                    else:
                        l.matches_perhaps(r, cand, p)

    def compare(self, r1: Record, r2: Record):
        """[Duke 1.2] Processor.compare(r1, r2) for any two records (indexed or not):
        dk_compare_values on their values; the index is not changed."""
        cols = []
        for p in self.database.props:
            vals = []
            for r in (r1, r2):
                vs = r.get_values(p.name)
                if len(vs) > 1:
                    raise ValueError(f"property {p.name}: {len(vs)} values (GPU path holds one)")
                vals.append(vs[0] if vs else None)
            cols.append(A.Column.from_strings(vals))
        return self.database.engine.compare_values(cols)
