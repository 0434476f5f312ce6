package io.sesam.dukemicroservice.gpu;

/**
 * JNI mirror of include/dukehip.h (libdukehip.so), bound by integration/jni/dukehip_jni.c.
 * Java 8 compatible (the reference's pom.xml:85-86).  Strings cross as UTF-16 char[] arenas
 * (Java's own code units: width-2 dk_column), arrays as primitive arrays.  Every native
 * method throws DukeHipException(code, dk_last_error()) on a negative DK_E* code -- an
 * unchecked exception, which the reference maps to HTTP 500 like its DukeException
 * (App.java:1007-1009).
 *
 * Not compiled in this repository's build (no JDK in the image): shipped as source for the
 * maintainer, exercised here through the same entry points from Python ctypes and C
 * (integration/c/dk_harness.c).
 */
public final class DukeHip {
    static {
        System.loadLibrary("dukehip_jni");   // links against libdukehip.so
    }

    private DukeHip() {}

    public static final int CMP_NONE = 0, CMP_LEVENSHTEIN = 1, CMP_JAROWINKLER = 2, CMP_QGRAM = 3,
            CMP_EXACT = 4, CMP_NUMERIC = 5, CMP_WEIGHTED_LEVENSHTEIN = 6, CMP_DICE_TOKENS = 7,
            CMP_JACCARD_TOKENS = 8, CMP_GEOPOSITION = 9;
    public static final int MODE_DEDUP = 0, MODE_LINKAGE = 1, MODE_ALLPAIRS = 2;
    public static final int KIND_MATCH = 1, KIND_MAYBE = 2;
    public static final int E_INVALID = -1, E_UNSUPPORTED = -2, E_NOMEM = -3, E_DEVICE = -4, E_STATE = -5;
    public static final int MAX_ORDER_CLASSES = 4;                                 // DK_MAX_ORDER_CLASSES
    public static final int CLEAN_NONE = 0, CLEAN_LOWERCASE_NORMALIZE = 1, CLEAN_COUNTRY_NAME = 2,
            CLEAN_CAPITAL = 3;
    public static final int LINK_INFERRED = 1, LINK_RETRACTED = 2, LINK_SAME = 1, LINK_MAYBE = 2;
    /** dk_key_part: no token / open slice end (INT32_MIN) */
    public static final int KEY_ALL = Integer.MIN_VALUE;

    // ---- pipeline ctx -------------------------------------------------------------------

    /**
     * dk_create (devices.length == 1) or dk_create_multi (the index replicated over several
     * GPUs of this JVM, one handle).  One property per index, in Processor.compare's iteration
     * order.  lookupProps != null selects the Lucene candidate source (dk_schema.lucene:
     * IncrementalLuceneDatabase.findCandidateMatches on the device; nkeys 0) with the
     * database's maxSearchHits / minRelevance (App.configureDatabase, App.java:550-563).
     */
    public static native long create(int[] comparator, int[] q, int[] formula, int[] tokenizer,
                                     double[] low, double[] high, double[] minRatio,
                                     double threshold, double maybeThreshold, int mode, int nkeys,
                                     int[] lookupProps, int maxSearchHits, float minRelevance,
                                     int[] devices, int[] orders);   // orders: dk_schema.orders or null

    public static native void destroy(long ctx);                                    // dk_destroy

    public static native int numDevices(long ctx);                                  // dk_num_devices

    /**
     * dk_upsert (transient = false) / dk_upsert_transient (true) of n records.  Per scored
     * property p: offsets[p] (n + 1 code-unit offsets into units[p]) and present[p] (1 = the
     * record has a value); per key function k: keyOffsets[k] / keyUnits[k] (the key strings).
     * ident: the records' interned IDs (internerIntern).  group is null unless LINKAGE;
     * deleted may be null.  Returns the assigned rows.
     */
    public static native int[] upsert(long ctx, boolean transient, int n, long[] ident, byte[] group,
                                      byte[] deleted, int[][] offsets, char[][] units, byte[][] present,
                                      int[][] keyOffsets, char[][] keyUnits, byte[] orderClass);

    public static native void dropTransient(long ctx);                              // dk_drop_transient

    public static final int LUCENE_STATS_MERGED = 0, LUCENE_STATS_UNMERGED = 1;
    public static native void luceneSetStats(long ctx, int mode);                   // dk_lucene_set_stats

    public static native void luceneMerge(long ctx);                                // dk_lucene_merge

    public static native void setOverwrite(long ctx, boolean on);                   // dk_set_overwrite

    public static native long numRows(long ctx);                                    // dk_num_rows

    /** dk_row_of_ident: the row of the live version of an interned record ID, or -1. */
    public static native int rowOfIdent(long ctx, long ident);

    /** dk_match (DK_MATCH_HOST); the handle is released with freeResult. */
    public static native long match(long ctx, int[] queryRows);

    public static native long[] resultFirst(long result);

    public static native int[] resultCandidate(long result);

    public static native double[] resultProb(long result);

    public static native byte[] resultKind(long result);

    public static native long resultPairsScored(long result);

    public static native void freeResult(long result);                              // dk_free_result

    public static native double compareRows(long ctx, int r1, int r2);              // dk_compare_rows

    /** dk_compare_values: Processor.compare of two records given as one value per property
     *  (null = no value), not indexed. */
    public static native double compareValues(long ctx, String[] r1, String[] r2);

    public static native void setProfiling(long ctx, boolean on);                   // dk_set_profiling

    /** One ctx per device, each writing its tile's match list into its slice of one direct
     *  ByteBuffer (dk_result_region_layout gives the offsets).  Not for a create() over
     *  several devices, which gathers its tiles itself. */
    public static native void setResultRegion(long ctx, java.nio.ByteBuffer region, long maxQueries);

    // ---- record-ID interner (dk_interner): the identity numbering of both packing paths --

    public static native long internerCreate();

    public static native void internerDestroy(long ids);

    /** dk_interner_intern of n = offsets.length - 1 ID strings (UTF-16 arena). */
    public static native long[] internerIntern(long ids, int[] offsets, char[] units);

    /** dk_interner_find: the id of an ID string, or -1 when it was never interned. */
    public static native long internerFind(long ids, String id);

    public static native String internerString(long ids, long id);                 // dk_interner_string

    // ---- native ingestion of a POSTed body (dk_pack_json) --------------------------------

    /**
     * dk_pack_json: the request body (UTF-8 JSON array of entities) -> the SoA columns of one
     * batch, by IncrementalDataSource's rules (IncrementalDataSource.java:50-101), record IDs
     * interned into `ids`.  Columns: JSON attribute name, scored property index (-1 = not
     * scored) and DK_CLEAN_* cleaner, in data-source order.  keyParts[k] is key function k's
     * parts flattened as (prop, token, start, end)* (KEY_ALL = none).  Throws DukeHipException
     * E_UNSUPPORTED for a body the native reader declines (the route then builds Records).
     */
    public static native long packJson(long ids, byte[] body, String datasetId, int groupNo,
                                       String[] columnNames, int[] columnProp, int[] columnCleaner,
                                       int nprops, int[][] keyParts);

    public static native int packedSize(long packed);

    public static native long[] packedIdent(long packed);

    public static native byte[] packedDeleted(long packed);

    /** The batch's values of scored property p (null = no value), for Records built lazily. */
    public static native String[] packedValues(long packed, int p);

    public static native String[] packedIds(long packed);                           // ID property

    public static native String[] packedEntityIds(long packed);                     // dukeOriginalEntityId

    /** dk_upsert / dk_upsert_transient of a packed batch; returns the rows. */
    public static native int[] upsertPacked(long ctx, long packed, boolean transient);

    public static native void freePacked(long packed);                              // dk_free_packed

    // ---- link sink (dk_linkdb): SinceAwareInMemoryLinkDatabase written in bulk -----------

    public static native long linkdbCreate(long ids);

    public static native void linkdbDestroy(long db);

    /** dk_linkdb_apply: one batch's listener stream; returns {asserted, unchanged, retracted}. */
    public static native long[] linkdbApply(long db, long[] queryIdent, long[] first, long[] candidateIdent,
                                            double[] prob, byte[] kind, long timestamp);

    /** dk_linkdb_links_for: getAllLinksFor of an interned ID; released with freeLinkList. */
    public static native long linkdbLinksFor(long db, long ident);

    /** dk_linkdb_retract: Link.retract() + assertLink of the link ident-other (other = -1:
     *  every link of ident), App.java:994-999.  Returns the links retracted. */
    public static native long linkdbRetract(long db, long ident, long other, long timestamp);

    /** dk_linkdb_changes_since; the handle is released with freeLinkList. */
    public static native long linkdbChangesSince(long db, long since);

    public static native long[] linkListId1(long list);

    public static native long[] linkListId2(long list);

    public static native byte[] linkListStatus(long list);

    public static native byte[] linkListKind(long list);

    public static native double[] linkListConfidence(long list);

    public static native long[] linkListTimestamp(long list);

    public static native void freeLinkList(long list);
}
