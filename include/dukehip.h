/*
 * dukehip.h — C-ABI of libdukehip.so, the MI355X-native candidate-pair scoring engine
 * that replaces Duke 1.2's matching loop behind the sesam-duke-microservice.
 *
 * The microservice drives Duke through four contracts; each entry point below replaces
 * one reference interface (file:line under /root/reference/src/main/java/io/sesam/
 * dukemicroservice/ unless stated):
 *
 *   dk_create        <- `new Processor(config, false)` + `config.setDatabase(db)` +
 *                       `Processor.setThreads` (App.java:342-344, 463-465); the schema is
 *                       what ConfigLoader.load builds from the <duke> block (App.java:613-647)
 *                       with the synthetic ID / ignored properties removed (App.java:309-323).
 *   dk_upsert        <- `Database.index(Record)` per record + `Database.commit()`
 *                       (IncrementalLuceneDatabase.java:498-575, 146-165): delete-by-ID then
 *                       add (:516-517, 578-590), dukeDeleted kept as a flag (:478).
 *   dk_match         <- `Processor.deduplicate(Collection<Record>)`'s match loop
 *                       (App.java:1005, 1159): findCandidateMatches
 *                       (IncrementalDeduplicationLuceneDatabase.java:8-10,
 *                       IncrementalRecordLinkageLuceneDatabase.java:12-14) with the
 *                       key-function blocking contract of SURVEY §8a-5, then
 *                       Processor.compareCandidatesSimple -> compare -> threshold.
 *   dk_result        <- the MatchListener callbacks (BaseLinkDatabaseMatchListener.java:53-109):
 *                       entries grouped per query in batch order, candidate order inside;
 *                       result memory is pooled per ctx and recycled by dk_free_result.
 *   dk_compare_rows  <- `Processor.compare(Record, Record)` for one pair of indexed rows.
 *   dk_compare_values<- `Processor.compare(Record, Record)` for two records that need not be
 *                       indexed (SURVEY §8b dk_compare_pair): a dk_batch of 2.
 *   dk_set_overwrite <- `Database.setOverwrite` (IncrementalLuceneDatabase.java:99, 515):
 *                       with overwrite on, index() adds without the delete-by-ID.
 *   dk_set_profiling <- `Processor.setPerformanceProfiling` (App.java:345, 466).
 *   dk_last_error    <- DukeException / RuntimeException text (App.java:1007-1009).
 *
 * Strings cross the boundary as Java chars (UTF-16 code units) or, when every unit of
 * a column is <= 0xFF, as one byte per unit (width 1).  Plain pointers and sizes only;
 * the caller owns its buffers and may free them as soon as a call returns.
 * Every function returns DK_OK (0) or a negative DK_E* code; dk_last_error() then holds
 * a thread-local message.  Calls on one dk_ctx must be serialised by the caller (the
 * microservice's per-pipeline ReentrantLock, App.java:96,145,947,1096); distinct ctxs are
 * independent (one HIP stream each).
 */
#ifndef DUKEHIP_H
#define DUKEHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DK_ABI_VERSION 9

/* status codes */
#define DK_OK 0
#define DK_E_INVALID (-1)     /* bad argument / schema */
#define DK_E_UNSUPPORTED (-2) /* comparator or parameter the GPU path does not implement */
#define DK_E_NOMEM (-3)
#define DK_E_DEVICE (-4)      /* HIP runtime error, or no GPU */
#define DK_E_STATE (-5)       /* call not valid in the ctx's current state */

/* comparators: Duke 1.2 no.priv.garshol.duke.comparators.* class -> opcode */
#define DK_CMP_NONE 0                 /* property without comparator: PropertyImpl -> 0.5 */
#define DK_CMP_LEVENSHTEIN 1          /* comparators.Levenshtein */
#define DK_CMP_JAROWINKLER 2          /* comparators.JaroWinkler */
#define DK_CMP_QGRAM 3                /* comparators.QGramComparator */
#define DK_CMP_EXACT 4                /* comparators.ExactComparator */
#define DK_CMP_NUMERIC 5              /* comparators.NumericComparator */
#define DK_CMP_WEIGHTED_LEVENSHTEIN 6 /* comparators.WeightedLevenshtein (default weights) */
#define DK_CMP_DICE_TOKENS 7          /* comparators.DiceCoefficientComparator (Exact sub-comparator) */
#define DK_CMP_JACCARD_TOKENS 8       /* comparators.JaccardIndexComparator (Exact sub-comparator) */
#define DK_CMP_GEOPOSITION 9          /* comparators.GeopositionComparator ("lat,lng" degrees;
                                         max-distance in meters in dk_property.min_ratio) */

#define DK_QGRAM_OVERLAP 0 /* QGramComparator.Formula */
#define DK_QGRAM_JACCARD 1
#define DK_QGRAM_DICE 2
#define DK_QGRAM_BASIC 0 /* QGramComparator.Tokenizer */
#define DK_QGRAM_POSITIONAL 1
#define DK_QGRAM_ENDS 2

#define DK_MODE_DEDUP 0    /* <Deduplication>: every other record is a candidate */
#define DK_MODE_LINKAGE 1  /* <RecordLinkage>: candidates only from the other group */
#define DK_MODE_ALLPAIRS 2 /* Duke InMemoryDatabase: no blocking, all records */

#define DK_KIND_MATCH 1 /* MatchListener.matches */
#define DK_KIND_MAYBE 2 /* MatchListener.matchesPerhaps */

typedef struct dk_property {
  int32_t comparator;      /* DK_CMP_* */
  int32_t qgram_q;         /* QGramComparator.setQ (default 2; 1..4) */
  int32_t qgram_formula;   /* DK_QGRAM_OVERLAP/JACCARD/DICE */
  int32_t qgram_tokenizer; /* DK_QGRAM_BASIC/POSITIONAL/ENDS (POSITIONAL: q <= 3) */
  double low;              /* <low> */
  double high;             /* <high> */
  double min_ratio;        /* the comparator's double parameter: NumericComparator.setMinRatio
                              (default 0.0); GeopositionComparator.setMaxDistance (meters) */
} dk_property;

/* Lucene-compatible candidate source: the reference's own
 * IncrementalLuceneDatabase.findCandidateMatches (IncrementalLuceneDatabase.java:459-492) --
 * every lookup property value's StandardAnalyzer tokens as SHOULD TermQuerys (after
 * escapeLucene, :295-342), MUST_NOT the query's dukeGroupNo (LINKAGE) and dukeDeleted, the
 * top max_hits documents by Lucene's DefaultSimilarity TF-IDF score (doQuery :377-414) kept
 * while score >= min_relevance (App.configureDatabase :550-563 defaults: 10, 0.9).  Candidates
 * reach Processor.compare in hit order; the query itself can be a hit (isSameAs drops it
 * there, as in Duke).  [Lucene 4.x scoring / analysis recalled: parity unpinned.]  Values of
 * lookup properties must lie in U+0000-U+00FF (else DK_E_UNSUPPORTED) and give <= 256 query
 * clauses per record. */
typedef struct dk_lucene {
  int32_t nlookup;            /* lookup properties (Configuration.getLookupProperties order) */
  const int32_t* lookup_prop; /* their indices into dk_schema.props */
  int32_t max_hits;           /* setMaxSearchHits: 1..100 */
  float min_relevance;        /* setMinRelevance */
} dk_lucene;

#define DK_MAX_ORDER_CLASSES 4

typedef struct dk_schema {
  int32_t nprops;           /* scored properties, in Processor.compare iteration order */
  const dk_property* props;
  double threshold;         /* <threshold> */
  double maybe_threshold;   /* <maybe-threshold>; 0.0 = none (Duke's default) */
  int32_t mode;             /* DK_MODE_* */
  int32_t nkeys;            /* key functions (blocking); ignored in ALLPAIRS mode; <= 8 */
  const dk_lucene* lucene;  /* non-NULL: Lucene-compatible candidates instead of key
                               functions (nkeys 0; DEDUP or LINKAGE) */
  /* Processor.compare visits r1's properties in its RecordImpl HashMap's iteration order,
   * which depends on the map's capacity -- 16 up to 12 keys, 32 up to 24, 64 up to 48 --
   * i.e. on how many properties the record holds values for (IncrementalDataSource.java:
   * 67-98 adds its columns' values and the synthetic ID / dukeOriginalEntityId /
   * dukeDatasetId / dukeGroupNo / dukeDeleted).  norders <= DK_MAX_ORDER_CLASSES order
   * classes: orders[c * nprops + k] = the k-th property visited for a query record of class
   * c (a permutation of 0..nprops-1; a record's missing properties are skipped).  norders 0
   * = one class, the props' own order.  The batch gives each record's class. */
  int32_t norders;
  const int32_t* orders;
} dk_schema;

/* One property's values for the n records of a batch. */
typedef struct dk_column {
  const uint32_t* offsets; /* n+1 offsets, in code units, into units */
  const void* units;       /* width 1: uint8_t units (<= 0xFF); width 2: uint16_t */
  int32_t width;           /* 1 or 2 */
  const uint8_t* present;  /* n flags: 0 = record has no value; NULL = all present */
} dk_column;

typedef struct dk_batch {
  uint64_t n;
  const uint64_t* ident;    /* n: equal <=> same ID property value (Processor.isSameAs) */
  const uint8_t* group;     /* n: dukeGroupNo (1 or 2); NULL unless LINKAGE */
  const uint8_t* deleted;   /* n: dukeDeleted == "true"; NULL = none */
  const dk_column* columns; /* nprops */
  /* key functions: either keys (nkeys*n, key-function major, equal <=> same key
   * string) or key_columns (nkeys strings per record, interned exactly by the library) */
  const uint64_t* keys;
  const dk_column* key_columns;
  const uint8_t* order_class; /* n: the record's order class (dk_schema.orders); NULL = 0 */
} dk_batch;

/* dk_match flags */
#define DK_MATCH_HOST 0   /* entries copied to (pinned) host memory: first/candidate/prob/kind */
#define DK_MATCH_DEVICE 1 /* entries stay in HBM only (host arrays NULL); fetch them with
                             dk_result_copy_to_device, e.g. into buffers an RCCL gather sends */

/* Match list of one dk_match call, grouped per query record in query order; inside a
 * query, candidates in key-function order then index order (SURVEY §8a-5 contract).
 * Entry e of query i (first[i] <= e < first[i+1]) is one MatchListener callback
 * matches(r1 = query_rows[i], r2 = candidate[e], prob[e]) or matchesPerhaps(...);
 * a query with no entry gets noMatchFor(r1). */
typedef struct dk_result {
  uint64_t nqueries;         /* queries passed to dk_match */
  uint64_t n;                /* match + maybe entries */
  const uint64_t* first;     /* nqueries+1 entry offsets */
  const uint32_t* candidate; /* row of r2 */
  const double* prob;        /* Processor.compare(r1, r2) */
  const uint8_t* kind;       /* DK_KIND_MATCH / DK_KIND_MAYBE */
  uint64_t pairs_scored;     /* Processor.compare calls made (candidates after filters) */
  uint64_t pairs_generated;  /* candidate slots produced by blocking, before filters */
} dk_result;

typedef struct dk_profile {
  double ms_index;        /* blocking-table build (sort, segments) */
  double ms_generate;     /* candidate counting + pair emission */
  double ms_score;        /* fused scoring kernels (the dominant kernel) */
  double ms_gather;       /* match compaction (symmetric schedule: the emission's write
                             pass) + device->host copy */
  double ms_total;        /* wall time of dk_match */
  uint64_t score_launches;
  uint64_t pairs_scored;
  uint64_t pairs_generated;
  uint64_t score_bytes;   /* algorithmic operand bytes of the scored pairs */
  double ms_copy;         /* device->host copies of the match list (copy stream, overlapped) */
  double ms_emit;         /* symmetric dedup schedule: the emission's count pass + scan */
  uint64_t sym_matches;   /* dk_match calls that ran the symmetric dedup schedule */
  uint64_t full_builds;   /* blocking-table builds that sorted every usable row */
  uint64_t delta_builds;  /* builds that re-sorted only the rows added since the last full
                             one (sorted base + sorted delta) */
  uint64_t replica_positions; /* the last dk_match's candidate replica: positions (rstride) */
  uint64_t gram_row_bytes;    /* and the bytes of its largest QGram property's key-word rows
                                 (rows x positions x 8; past 4 GiB the grouped kernels address
                                 them through head / tail buffer resources) */
  uint64_t sym2_matches;  /* symmetric dedup calls with two queries per wave (k_score_sym2:
                             owner slots padded to 32; ABI 9) */
  uint64_t pairs_exact;   /* scored pairs that took k_score_gq's exact double-precision pass
                             (the rest were decided by its single-precision screen; ABI 9) */
} dk_profile;

typedef struct dk_ctx dk_ctx;

int dk_create(const dk_schema* schema, int device, dk_ctx** out);
/* One pipeline over several GPUs of this process (the reference's parallelism
 * is in-process -- THREADS -> Processor.setThreads, App.java:232,344,465 -- so a JVM reaches
 * every GPU of the node through ONE handle).  The index is replicated: every dk_upsert /
 * dk_upsert_transient / dk_drop_transient / dk_set_overwrite goes to every device, on one
 * host thread per device; a batch rejected on validation is rejected identically everywhere
 * (failure-atomic as dk_upsert), a device failure on some devices only leaves the ctx
 * unusable (DK_E_STATE afterwards).  dk_match splits the query rows into one contiguous tile
 * per device, balanced by dk_candidate_counts (+32 per query, the padded wave), runs the
 * tiles concurrently and returns ONE host list in query order -- each device copies its tile
 * into its slice of the list over its own host link (DK_MATCH_DEVICE and
 * dk_set_result_region are per-device features: DK_E_UNSUPPORTED here).  dk_compare_*,
 * dk_property_similarity, dk_candidate_counts, dk_row_of_ident and dk_num_rows use the
 * first device's replica; dk_get_profile sums counters and takes the largest time per
 * phase.  A device may be listed more than once (one stream set per entry).  ndev == 1 is
 * dk_create(devices[0]). */
int dk_create_multi(const dk_schema* schema, const int* devices, int ndev, dk_ctx** out);
int dk_num_devices(const dk_ctx* ctx);
void dk_destroy(dk_ctx* ctx);
/* Failure-atomic: a batch that is rejected (DK_E_INVALID / DK_E_UNSUPPORTED / DK_E_NOMEM)
 * leaves the index as it was -- no row added, no older version tombstoned -- so the caller
 * may run that batch on stock Duke and keep the ctx.  LINKAGE batches need group[i] in {1,2}. */
int dk_upsert(dk_ctx* ctx, const dk_batch* batch, uint32_t* rows_out);
/* IncrementalLuceneDatabase.setIndexingIsDisabled(true) (IncrementalLuceneDatabase.java:95,
 * 498-512) as the httptransform endpoint uses it (App.java:1130-1132): appends the batch as
 * query-only rows -- dk_match accepts them as queries, they are never candidates and do not
 * supersede the indexed version of their ID.  Normal dk_upsert is refused (DK_E_STATE)
 * until dk_drop_transient removes them again (App.java:1174-1175, indexing re-enabled). */
int dk_upsert_transient(dk_ctx* ctx, const dk_batch* batch, uint32_t* rows_out);
int dk_drop_transient(dk_ctx* ctx);
/* Collection statistics (maxDoc, docFreq) of the Lucene candidate source.  Every upsert of a
 * known ID deletes the older version and adds the new one (IncrementalLuceneDatabase.java:
 * 516-517, 578-590); the older version is never a hit again, but Lucene 4 keeps counting a
 * deleted document in maxDoc and docFreq until a merge of its segment reclaims it, and the
 * reference never forces one (commit, :146-165).
 *   DK_LUCENE_STATS_MERGED (default): the statistics of a fully merged index -- only the live
 *     version of each ID (dukeDeleted records included) counts;
 *   DK_LUCENE_STATS_UNMERGED: every version that entered the index counts until dk_lucene_merge
 *     (IndexWriter.forceMerge) reclaims the superseded ones.  Lucene's background merge policy
 *     reclaims them at times this ctx does not model: call dk_lucene_merge to follow it.
 * Both are index changes (the next dk_match rebuilds the statistics).  DK_E_STATE without a
 * Lucene source. */
#define DK_LUCENE_STATS_MERGED 0
#define DK_LUCENE_STATS_UNMERGED 1
int dk_lucene_set_stats(dk_ctx* ctx, int mode);
int dk_lucene_merge(dk_ctx* ctx);
int dk_match(dk_ctx* ctx, const uint32_t* query_rows, uint64_t nq, int flags, dk_result** out);
/* counts[i] = the candidates blocking produces for query_rows[i] (its buckets' sizes over
 * the key functions, before the isSameAs / already-a-candidate filters): the cost model for
 * splitting queries into balanced multi-GPU tiles.  Builds the blocking tables if the index
 * changed (as dk_match would). */
int dk_candidate_counts(dk_ctx* ctx, const uint32_t* query_rows, uint64_t nq, uint64_t* counts);
/* device-to-device copy of a result's entries (any of the pointers may be NULL); the
 * destination buffers live on the ctx's device */
int dk_result_copy_to_device(const dk_result* result, uint64_t* first, uint32_t* candidate,
                             double* prob, uint8_t* kind);
void dk_free_result(dk_result* result);

/* Caller-owned host memory for the entries of later DK_MATCH_HOST calls, instead of the
 * library's pinned pool: e.g. this rank's slice of one node-wide shared mapping, so every
 * GPU copies its query tile's match list over its own PCIe link into memory the listener
 * process (rank 0) reads directly -- the multi-GPU result gather of SURVEY §8e without a
 * second hop through one GPU (dukehip.dist).  The library registers the range with the
 * HIP runtime (page-locks it) until the region is replaced, cleared (base NULL) or the ctx
 * destroyed.  Layout: dk_result_region_layout.  The dk_result of a match in the region
 * points into it and is overwritten by the next dk_match.  A match list that does not fit
 * fails with DK_E_NOMEM; more than max_queries queries with DK_E_INVALID. */
typedef struct dk_region_layout {
  uint64_t capacity;         /* entries the region holds */
  uint64_t first_offset;     /* u64 first[max_queries + 1] */
  uint64_t prob_offset;      /* f64 prob[capacity] */
  uint64_t candidate_offset; /* u32 candidate[capacity] */
  uint64_t kind_offset;      /* u8 kind[capacity] */
} dk_region_layout;
int dk_result_region_layout(uint64_t bytes, uint64_t max_queries, dk_region_layout* out);
int dk_set_result_region(dk_ctx* ctx, void* base, uint64_t bytes, uint64_t max_queries);
/* Processor.compare(r1, r2) for two indexed rows; a record is compared with itself too
 * (no isSameAs).  Leaves the blocking tables and result pools of the ctx untouched. */
int dk_compare_rows(dk_ctx* ctx, uint32_t r1, uint32_t r2, double* prob);
/* Processor.compare(r1, r2) for records given as a dk_batch with n == 2 (records 0 and 1
 * are r1 and r2; ident / group / deleted / keys are ignored).  The ctx's index is not
 * changed. */
int dk_compare_values(dk_ctx* ctx, const dk_batch* pair, double* prob);
/* Comparator.compare(v1, v2) of schema property `prop` for two indexed rows (the raw
 * similarity PropertyImpl.compare maps to a probability), computed by the production
 * scoring kernel.  NaN when either row has no (or an empty) value: Processor.compare never
 * calls a comparator then.  Levenshtein: Duke's own value also where compactDistance's early
 * exit fires (its column minimum; the fused match kernels use maxdist + 1 there, which maps
 * to the same <low> probability). */
int dk_property_similarity(dk_ctx* ctx, int prop, uint32_t r1, uint32_t r2, double* sim);
int dk_set_overwrite(dk_ctx* ctx, int on);
uint64_t dk_num_rows(const dk_ctx* ctx);
/* IncrementalLuceneDatabase.findRecordById: the row of the live version of a record ID
 * (dk_batch.ident numbering); DK_E_INVALID when none is indexed */
int dk_row_of_ident(const dk_ctx* ctx, uint64_t ident, uint32_t* row);
/* on: 0 off, 1 every phase's device time (dk_profile.ms_*), 2 the scoring kernels only
 * (ms_score: no events between the other phases' dependent kernels) */
int dk_set_profiling(dk_ctx* ctx, int on);
int dk_get_profile(const dk_ctx* ctx, dk_profile* out);
int dk_reset_profile(dk_ctx* ctx);
/* ---- native ingestion: a POSTed entity batch (JSON text, UTF-8) ->
 * the SoA columns of a dk_batch, without building Duke Record objects.  Follows
 * IncrementalDataSource.DatasetDataSourceRecordIterator.next (IncrementalDataSource.java:
 * 50-101): `_id` (JsonElement.getAsString; missing/empty -> DK_E_INVALID "Got an entity
 * with no '_id' attribute!"), one value per column (a JSON array contributes
 * array.getAsString() per element: [] nothing, [x] x, longer -> DK_E_INVALID), the column's
 * cleaner then RecordBuilder's empty-value skip, the synthetic ID
 * "<group>__<dataset>__<entity>" and dukeDeleted (`_deleted`.getAsBoolean()).  Strict JSON
 * only; lenient-Gson input, characters a native cleaner does not cover (>= U+0370) and a
 * second value for one property return DK_E_UNSUPPORTED: that batch takes the caller's own
 * packing path.  Record IDs are interned exactly into dk_interner ids (dk_batch.ident). */
#define DK_CLEAN_NONE 0
#define DK_CLEAN_LOWERCASE_NORMALIZE 1 /* cleaners.LowerCaseNormalizeCleaner (recalled) */
#define DK_CLEAN_COUNTRY_NAME 2        /* examples.CountryNameCleaner (recalled) */
#define DK_CLEAN_CAPITAL 3             /* examples.CapitalCleaner (recalled) */

typedef struct dk_source_column {
  const char* name;   /* JSON attribute (<column name>), UTF-8 */
  int32_t prop;       /* schema property it fills (<column property>); -1 = not scored;
                         nprops + j (j < 16): a property only key functions read (its value
                         is kept for dk_key_part.prop = nprops + j, not packed) */
  int32_t cleaner;    /* DK_CLEAN_* (<column cleaner>) */
} dk_source_column;

/* one part of a key: the property's cleaned value, optionally its whitespace token number
 * `token` (Python str.split(); negative from the end; INT32_MIN = the whole value), sliced
 * [start, end) in code points with Python slice rules (INT32_MIN = open end) */
typedef struct dk_key_part {
  int32_t prop, token, start, end;
} dk_key_part;

typedef struct dk_key_function {
  int32_t nparts;
  const dk_key_part* parts; /* the key is the parts' concatenation */
} dk_key_function;

typedef struct dk_source {
  const char* dataset_id;          /* <param name="dataset-id">, UTF-8 */
  int32_t group_no;                /* 0: Deduplication; 1 / 2: the RecordLinkage <group> */
  int32_t ncolumns;
  const dk_source_column* columns; /* in data-source order */
  int32_t nprops;                  /* scored properties (schema order) of the packed batch */
  int32_t nkeys;
  const dk_key_function* keys;
} dk_source;

typedef struct dk_packed {
  uint64_t n;
  const dk_column* columns;     /* nprops, for dk_batch.columns */
  const dk_column* key_columns; /* nkeys, for dk_batch.key_columns */
  const uint64_t* ident;        /* interned record IDs, for dk_batch.ident */
  const uint8_t* deleted;       /* dukeDeleted, for dk_batch.deleted */
  const uint8_t* group;         /* dukeGroupNo (NULL in deduplication), for dk_batch.group */
  dk_column id;                 /* the ID property value of every record */
  dk_column entity_id;          /* dukeOriginalEntityId */
} dk_packed;

typedef struct dk_interner dk_interner;
int dk_interner_create(dk_interner** out);
void dk_interner_destroy(dk_interner* ids);
uint64_t dk_interner_size(const dk_interner* ids);
int dk_interner_find(const dk_interner* ids, const uint16_t* units, uint64_t n, uint64_t* id);
/* out[i] = the id of record ID string i of `column` (interned if new): the same numbering
 * dk_pack_json gives, for batches packed by the caller */
int dk_interner_intern(dk_interner* ids, const dk_column* column, uint64_t n, uint64_t* out);
int dk_pack_json(const dk_source* source, const char* json, uint64_t len, dk_interner* ids,
                 dk_packed** out);
void dk_free_packed(dk_packed* packed);
/* the record ID string of an interned id (UTF-16 code units; valid until the next call that
 * interns into `ids`: copy it out before packing another batch) */
int dk_interner_string(const dk_interner* ids, uint64_t id, const uint16_t** units, uint64_t* n);

/* ---- link sink: the pipeline's LinkDatabase written in bulk from a match
 * list.  Replaces the per-callback LinkDatabaseMatchListener that
 * BaseLinkDatabaseMatchListener.java:53-109 forwards to, writing into a
 * SinceAwareInMemoryLinkDatabase (SinceAwareInMemoryLinkDatabase.java:12-41; the
 * "in-memory" link-database-type, App.java:571-573).  Links are between interned record IDs
 * (dk_interner): ID1 is the smaller ID string (String.compareTo). */
#define DK_LINK_INFERRED 1   /* LinkStatus.INFERRED */
#define DK_LINK_RETRACTED 2  /* LinkStatus.RETRACTED */
#define DK_LINK_SAME 1       /* LinkKind.SAME (matches) */
#define DK_LINK_MAYBE 2      /* LinkKind.MAYBE (matchesPerhaps) */

typedef struct dk_link_batch {
  uint64_t nqueries;
  const uint64_t* query_ident;     /* interned ID of each query record, batch order */
  const uint64_t* first;           /* nqueries + 1 entry offsets (dk_result.first) */
  const uint64_t* candidate_ident; /* per entry: interned ID of the candidate */
  const double* prob;              /* per entry: confidence */
  const uint8_t* kind;             /* per entry: DK_KIND_MATCH / DK_KIND_MAYBE */
} dk_link_batch;

typedef struct dk_link_stats {
  uint64_t asserted;   /* links written (new, or changed status / kind / confidence) */
  uint64_t unchanged;  /* identical links kept with their old timestamp (1e-6 rule) */
  uint64_t retracted;  /* INFERRED links of a processed record it no longer produced */
} dk_link_stats;

typedef struct dk_link_list {
  uint64_t n;
  const uint64_t* id1;
  const uint64_t* id2;
  const uint8_t* status;     /* DK_LINK_INFERRED / DK_LINK_RETRACTED */
  const uint8_t* kind;       /* DK_LINK_SAME / DK_LINK_MAYBE */
  const double* confidence;
  const int64_t* timestamp;  /* ms since the epoch */
} dk_link_list;

typedef struct dk_linkdb dk_linkdb;
int dk_linkdb_create(const dk_interner* ids, dk_linkdb** out);
void dk_linkdb_destroy(dk_linkdb* db);
uint64_t dk_linkdb_size(const dk_linkdb* db);
/* Processor.deduplicate's listener stream of one batch (the query records in batch order,
 * each with its entries in candidate order), stamped `timestamp` */
int dk_linkdb_apply(dk_linkdb* db, const dk_link_batch* batch, int64_t timestamp, dk_link_stats* stats);
/* SinceAwareInMemoryLinkDatabase.getChangesSince: links with timestamp > since, ordered by
 * (timestamp, assertion order) -- the reference iterates a HashMap (order unpinned) */
int dk_linkdb_changes_since(const dk_linkdb* db, int64_t since, dk_link_list** out);
void dk_free_link_list(dk_link_list* list);
/* InMemoryLinkDatabase.getAllLinksFor: every link of one record ID (either side) */
int dk_linkdb_links_for(const dk_linkdb* db, uint64_t id, dk_link_list** out);
/* the POST route's deleted-record branch (App.java:994-999): Link.retract() + assertLink on
 * the link between `id` and `other`, or (other == UINT64_MAX) on every link of `id`, with the
 * given timestamp */
int dk_linkdb_retract(dk_linkdb* db, uint64_t id, uint64_t other, int64_t timestamp, uint64_t* nretracted);

/* the StandardAnalyzer tokens of one value (escape: escapeLucene first, the query side),
 * '\n'-joined into out (test hook of the DK_CAND_LUCENE analysis) */
int dk_lucene_analyze(const uint16_t* units, uint64_t n, int escape, char* out, uint64_t cap,
                      uint64_t* ntokens);

const char* dk_last_error(void);
int dk_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
