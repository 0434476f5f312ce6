package io.sesam.dukemicroservice.gpu;

/**
 * JNI mirror of include/dukehip.h (libdukehip.so), bound by integration/jni/dukehip_jni.c.
 * Java 8 compatible (the reference's pom.xml:85-86).  Strings cross as UTF-16 char[] arenas
 * (Java's own code units: width-2 dk_column), arrays as primitive arrays.  Every native
 * method throws RuntimeException(dk_last_error()) on a negative DK_E* code -- the reference
 * maps DukeException to HTTP 500 the same way (App.java:1007-1009).
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
            CMP_JACCARD_TOKENS = 8;
    public static final int MODE_DEDUP = 0, MODE_LINKAGE = 1, MODE_ALLPAIRS = 2;
    public static final int KIND_MATCH = 1, KIND_MAYBE = 2;

    /** dk_create: one property per index, in Processor.compare's iteration order. */
    public static native long create(int[] comparator, int[] q, int[] formula, int[] tokenizer,
                                     double[] low, double[] high, double[] minRatio,
                                     double threshold, double maybeThreshold, int mode, int nkeys,
                                     int device);

    public static native void destroy(long ctx);                                    // dk_destroy

    /**
     * dk_upsert (transient = false) / dk_upsert_transient (true) of n records.  Per scored
     * property p: offsets[p] (n + 1 code-unit offsets into units[p]) and present[p] (1 = the
     * record has a value); per key function k: keyOffsets[k] / keyUnits[k] (the key strings).
     * group is null unless LINKAGE; deleted may be null.  Returns the assigned rows.
     */
    public static native int[] upsert(long ctx, boolean transient, int n, long[] ident, byte[] group,
                                      byte[] deleted, int[][] offsets, char[][] units, byte[][] present,
                                      int[][] keyOffsets, char[][] keyUnits);

    public static native void dropTransient(long ctx);                              // dk_drop_transient

    public static native void setOverwrite(long ctx, boolean on);                   // dk_set_overwrite

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

    /** Multi-GPU in one JVM: every device's ctx writes its tile's match list into its slice of
     *  one direct ByteBuffer (dk_result_region_layout gives the offsets). */
    public static native void setResultRegion(long ctx, java.nio.ByteBuffer region, long maxQueries);
}
