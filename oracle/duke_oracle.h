/*
 * duke_oracle.h — CPU restatement of Duke 1.2's candidate-pair scoring path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  Nothing in the product (sesam-duke-microservice_amd/) links or calls it.
 *
 * PARITY UNPINNED against Duke itself: the arithmetic lives in the third-party jar
 * no.priv.garshol.duke:duke:1.2 (/root/reference/pom.xml:32-36), which is absent from
 * /root/reference and cannot be fetched or run here (no JDK, no jar, no network), and
 * the reference ships no golden vectors for this path (AppTest.java:34-37 asserts true).
 * Every function below restates the published Duke 1.2 source as recalled and cites the
 * microservice call site it serves.  Golden fixtures under tests/golden/ are produced by
 * an independent pure-Python restatement (oracle/duke_pyref.py) and pin this C code to it.
 *
 * Strings are Java Strings: arrays of UTF-16 code units (uint16_t), compared by unit.
 */
#ifndef DUKE_ORACLE_H
#define DUKE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* comparator opcodes (same numbering as include/dukehip.h DK_CMP_*) */
enum {
  DKO_CMP_NONE = 0,          /* PropertyImpl with comparator == null -> 0.5 */
  DKO_CMP_LEVENSHTEIN = 1,
  DKO_CMP_JAROWINKLER = 2,
  DKO_CMP_QGRAM = 3,
  DKO_CMP_EXACT = 4,
  DKO_CMP_NUMERIC = 5,
  DKO_CMP_WEIGHTED_LEVENSHTEIN = 6,
  DKO_CMP_DICE_TOKENS = 7,   /* DiceCoefficientComparator (ExactComparator sub-comparator) */
  DKO_CMP_JACCARD_TOKENS = 8, /* JaccardIndexComparator (ExactComparator sub-comparator) */
  DKO_CMP_GEOPOSITION = 9     /* GeopositionComparator (max-distance in min_ratio) */
};
enum { DKO_QF_OVERLAP = 0, DKO_QF_JACCARD = 1, DKO_QF_DICE = 2 };
enum { DKO_QT_BASIC = 0, DKO_QT_POSITIONAL = 1, DKO_QT_ENDS = 2 };
enum { DKO_MODE_DEDUP = 0, DKO_MODE_LINKAGE = 1, DKO_MODE_ALLPAIRS = 2 };
enum { DKO_KIND_MATCH = 1, DKO_KIND_MAYBE = 2 };

/* ---- comparators ([Duke 1.2] no.priv.garshol.duke.comparators.*) ---- */
int    dko_compact_distance(const uint16_t* s1, int n1, const uint16_t* s2, int n2);
double dko_levenshtein(const uint16_t* s1, int n1, const uint16_t* s2, int n2);
double dko_jarowinkler(const uint16_t* s1, int n1, const uint16_t* s2, int n2);
double dko_qgram(const uint16_t* s1, int n1, const uint16_t* s2, int n2,
                 int q, int formula, int tokenizer);
double dko_exact(const uint16_t* s1, int n1, const uint16_t* s2, int n2);
/* Double.parseDouble; returns 0 and stores the value, or -1 for NumberFormatException */
int    dko_parse_java_double(const uint16_t* s, int n, double* out);
double dko_numeric(const uint16_t* s1, int n1, const uint16_t* s2, int n2, double min_ratio);
int dko_parse_geoposition(const uint16_t* s, int n, double* lat, double* lng);
double dko_geoposition(const uint16_t* s1, int n1, const uint16_t* s2, int n2, double maxdist);
double dko_weighted_levenshtein(const uint16_t* s1, int n1, const uint16_t* s2, int n2);
double dko_token_similarity(const uint16_t* s1, int n1, const uint16_t* s2, int n2, int jaccard);

/* ---- probability model ---- */
double dko_java_max(double a, double b);                 /* java.lang.Math.max */
double dko_compute_bayes(double p1, double p2);          /* [Duke 1.2] utils.Utils.computeBayes */

typedef struct dko_prop {
  int comparator;
  double low, high;
  int q, formula, tokenizer;   /* QGramComparator */
  double min_ratio;            /* NumericComparator min-ratio; GeopositionComparator max-distance */
} dko_prop;

/* [Duke 1.2] PropertyImpl.compare(v1, v2) */
double dko_property_compare(const dko_prop* p, const uint16_t* s1, int n1,
                            const uint16_t* s2, int n2);

typedef struct dko_schema {
  int nprops;
  const dko_prop* props;       /* in Processor.compare iteration order */
  double threshold;
  double maybe_threshold;
  int mode;                    /* DKO_MODE_* */
  int nkeys;                   /* key functions (blocking); 0 in ALLPAIRS mode */
  int norders;                 /* order classes (0: one, the props' order) */
  const int* orders;           /* norders x nprops: class c visits orders[c * nprops + k] */
} dko_schema;

/* Column-packed records.  Every array has n entries unless noted.
 *   off[p]   : n+1 offsets (code units) into chars[p]
 *   present[p]: 1 if record has a value for property p (a present value may be "")
 *   key_off[k]/key_chars[k]: the key string of key function k per record
 * group may be NULL (dedup), deleted/alive may be NULL (none deleted / all alive). */
typedef struct dko_table {
  uint64_t n;
  const uint64_t* ident;
  const uint8_t* group;
  const uint8_t* deleted;
  const uint8_t* alive;
  const uint32_t* const* off;
  const uint16_t* const* chars;
  const uint8_t* const* present;
  const uint32_t* const* key_off;
  const uint16_t* const* key_chars;
  const uint8_t* oclass;       /* per row: its order class (NULL: 0) */
} dko_table;

/* [Duke 1.2] Processor.compare(r1, r2) over rows a (r1) and b (r2) */
double dko_compare_rows(const dko_schema* s, const dko_table* t, uint32_t a, uint32_t b);

typedef struct dko_result {
  uint64_t n;                  /* emitted match/maybe callbacks */
  uint32_t* query;
  uint32_t* candidate;
  double* prob;
  uint8_t* kind;
  uint64_t pairs_scored;       /* Processor.compare calls */
  double ms_index;             /* blocking-index build (wall) */
  double ms_score;             /* candidate walk + compare + threshold (wall) */
} dko_result;

/* Processor.deduplicate's match loop for the given query rows (batch order): candidate
 * generation with exact-key blocking (or all rows in ALLPAIRS mode), isSameAs / deleted /
 * group filters, compare, threshold.  Uses nthreads host threads over contiguous query
 * slices; results are concatenated in query order.  Returns 0 or -1. */
int  dko_match(const dko_schema* s, const dko_table* t, const uint32_t* queries, uint64_t nq,
               int nthreads, dko_result* out);
void dko_free_result(dko_result* r);

#ifdef __cplusplus
}
#endif
#endif
