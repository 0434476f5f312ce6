/*
 * duke_oracle.c — CPU restatement of Duke 1.2's candidate-pair scoring path.
 *
 * TEST INFRASTRUCTURE ONLY (see duke_oracle.h).  PARITY UNPINNED against Duke itself:
 * the Duke 1.2 jar (/root/reference/pom.xml:32-36) is absent and nothing in
 * /root/reference pins these functions; the fixtures in tests/golden pin this file to the independent
 * Python restatement oracle/duke_pyref.py.
 *
 * Compiled with -O2 -ffp-contract=off: Java evaluates every double expression with one
 * rounding per operation, so no fused multiply-add may appear here (or in the GPU kernels).
 */
#include "duke_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_ms(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

static int u16eq(const uint16_t* a, int na, const uint16_t* b, int nb) {
  if (na != nb) return 0;
  for (int i = 0; i < na; i++)
    if (a[i] != b[i]) return 0;
  return 1;
}

/* [Duke 1.2] comparators.Levenshtein.compactDistance(s1, s2): single-column Wagner-Fischer
 * whose cell is min(above, aboveleft, left) + cost (cost added to all three neighbours),
 * first column min(column[ix1-1], ix1-1) + cost, and the cutoff "smallest value of the
 * column > min(|s1|,|s2|)/2 -> return it", checked after each column ix2 >= 1.  When
 * |s2| == 1 the column loop never runs and the function returns 0. */
int dko_compact_distance(const uint16_t* s1, int n1, const uint16_t* s2, int n2) {
  if (n1 == 0) return n2;
  if (n2 == 0) return n1;
  int maxdist = imin(n1, n2) / 2;
  int s1len = n1;
  int stackcol[257];
  int* column = s1len + 1 <= 257 ? stackcol : (int*)malloc(sizeof(int) * (size_t)(s1len + 1));

  int ix2 = 0;
  uint16_t ch2 = s2[ix2];
  column[0] = 1; /* virtual first row */
  for (int ix1 = 1; ix1 <= s1len; ix1++) {
    int cost = s1[ix1 - 1] == ch2 ? 0 : 1;
    column[ix1] = imin(column[ix1 - 1], ix1 - 1) + cost;
  }

  int above = 0;
  int result = -1;
  for (ix2 = 1; ix2 < n2; ix2++) {
    ch2 = s2[ix2];
    above = ix2 + 1; /* virtual first row */
    int smallest = s1len * 2;
    for (int ix1 = 1; ix1 <= s1len; ix1++) {
      int cost = s1[ix1 - 1] == ch2 ? 0 : 1;
      int value = imin(imin(above, column[ix1 - 1]), column[ix1]) + cost;
      column[ix1 - 1] = above;
      above = value;
      smallest = imin(smallest, value);
    }
    column[s1len] = above;
    if (smallest > maxdist) {
      result = smallest;
      break;
    }
  }
  if (result < 0) result = above;
  if (column != stackcol) free(column);
  return result;
}

/* [Duke 1.2] comparators.Levenshtein.compare: length-ratio shortcut, equality shortcut,
 * then 1 - min(compactDistance, len)/len with len = the SHORTER length. */
double dko_levenshtein(const uint16_t* s1, int n1, const uint16_t* s2, int n2) {
  int len = imin(n1, n2);
  int maxlen = imax(n1, n2);
  if ((double)len / (double)maxlen <= 0.5) return 0.0;
  if (len == maxlen && u16eq(s1, n1, s2, n2)) return 1.0;
  int dist = imin(dko_compact_distance(s1, n1, s2, n2), len);
  return 1.0 - ((double)dist / (double)len);
}

/* [Duke 1.2] comparators.JaroWinkler.similarity: s1 = the shorter string (s1 stays first
 * on equal length), window [max(0,i-maxdist), min(|s2|, i+maxdist)) with maxdist =
 * |s2|/2, FIRST equal character taken (no matched-marking), a transposition whenever the
 * match position moves backwards, t not halved, prefix bonus p*(1-score)/10 with p <= 4,
 * no long-string adjustment. */
double dko_jarowinkler(const uint16_t* s1, int n1, const uint16_t* s2, int n2) {
  if (u16eq(s1, n1, s2, n2)) return 1.0;
  if (n1 > n2) {
    const uint16_t* ts = s2; s2 = s1; s1 = ts;
    int tn = n2; n2 = n1; n1 = tn;
  }
  int maxdist = n2 / 2;
  int c = 0, t = 0, prevpos = -1;
  for (int ix = 0; ix < n1; ix++) {
    uint16_t ch = s1[ix];
    int hi = imin(n2, ix + maxdist);
    for (int ix2 = imax(0, ix - maxdist); ix2 < hi; ix2++) {
      if (ch == s2[ix2]) {
        c++;
        if (prevpos != -1 && ix2 < prevpos) t++;
        prevpos = ix2;
        break;
      }
    }
  }
  if (c == 0) return 0.0;
  double score = ((c / (double)n1) + (c / (double)n2) + ((c - t) / (double)c)) / 3.0;
  int p = 0;
  int last = imin(4, n1);
  for (; p < last && s1[p] == s2[p]; p++)
    ;
  score += ((p * (1 - score)) / 10);
  return score;
}

/* q-gram sets.  A gram is the q code units s[ix..ix+q) (java String.substring); the
 * POSITIONAL tokenizer also keys the gram by ix.  Sets are HashSet<String> in Duke, so
 * duplicate grams collapse.  Represented here as sorted unique arrays of 64-bit codes
 * (16 bits per code unit, q <= 4; POSITIONAL: q <= 3 and position in the top 16 bits). */
static int cmp_u64(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}

/* ENDS [recalled, low confidence]: the BASIC grams plus the start gram "^" + s[0, q-1)
 * and the end gram s[n-q+1, n) + "$" — exactly the grams of "^" + s + "$" (a Java
 * HashSet<String>, so a marker gram may coincide with a real one). */
static int qgram_set(const uint16_t* s0, int n0, int q, int tokenizer, uint64_t* out) {
  const uint16_t* s = s0;
  int n = n0;
  uint16_t ends_buf[260];
  uint16_t* ends = NULL;
  if (tokenizer == DKO_QT_ENDS) {
    ends = n0 + 2 <= 260 ? ends_buf : (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(n0 + 2));
    ends[0] = '^';
    memcpy(ends + 1, s0, sizeof(uint16_t) * (size_t)n0);
    ends[n0 + 1] = '$';
    s = ends;
    n = n0 + 2;
  }
  int m = 0;
  for (int ix = 0; ix < n - q + 1; ix++) {
    uint64_t g = 0;
    for (int k = 0; k < q; k++) g = (g << 16) | s[ix + k];
    if (tokenizer == DKO_QT_POSITIONAL) g |= (uint64_t)ix << 48;
    out[m++] = g;
  }
  if (ends && ends != ends_buf) free(ends);
  qsort(out, (size_t)m, sizeof(uint64_t), cmp_u64);
  int u = 0;
  for (int i = 0; i < m; i++)
    if (u == 0 || out[u - 1] != out[i]) out[u++] = out[i];
  return u;
}

/* [Duke 1.2] comparators.QGramComparator.compare + Formula.compute. */
double dko_qgram(const uint16_t* s1, int n1, const uint16_t* s2, int n2,
                 int q, int formula, int tokenizer) {
  if (u16eq(s1, n1, s2, n2)) return 1.0;
  uint64_t st1[264], st2[264];
  uint64_t* g1 = n1 < 260 ? st1 : (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n1 + 3));
  uint64_t* g2 = n2 < 260 ? st2 : (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n2 + 3));
  int m1 = qgram_set(s1, n1, q, tokenizer, g1);
  int m2 = qgram_set(s2, n2, q, tokenizer, g2);
  double r;
  if (m1 == 0 || m2 == 0) {
    r = 0.0;
  } else {
    int common = 0, i = 0, j = 0;
    while (i < m1 && j < m2) {
      if (g1[i] == g2[j]) { common++; i++; j++; }
      else if (g1[i] < g2[j]) i++;
      else j++;
    }
    if (formula == DKO_QF_JACCARD)
      r = (double)common / (double)(m1 + m2 - common);
    else if (formula == DKO_QF_DICE)
      r = (2.0 * (double)common) / (double)(m1 + m2);
    else
      r = (double)common / fmin((double)m1, (double)m2);
  }
  if (g1 != st1) free(g1);
  if (g2 != st2) free(g2);
  return r;
}

/* [Duke 1.2] comparators.ExactComparator */
double dko_exact(const uint16_t* s1, int n1, const uint16_t* s2, int n2) {
  return u16eq(s1, n1, s2, n2) ? 1.0 : 0.0;
}

/* java.lang.Double.parseDouble (FloatingDecimal.readJavaFormatString): String.trim()
 * (drops code units <= U+0020 at both ends), optional sign, then "NaN", "Infinity",
 * a hex literal 0x<hex>[.<hex>]p[+-]<dec> or a decimal literal
 * <dec>[.<dec>][(e|E)[+-]<dec>] (at least one mantissa digit), then an optional
 * f/F/d/D suffix for the numeric forms.  The value is the correctly rounded double
 * (glibc strtod is correctly rounded, like FloatingDecimal). */
int dko_parse_java_double(const uint16_t* s, int n, double* out) {
  int a = 0, b = n;
  while (a < b && s[a] <= 0x20) a++;
  while (b > a && s[b - 1] <= 0x20) b--;
  int len = b - a;
  if (len == 0) return -1;
  char buf[512];
  char* tmp = len < 511 ? buf : (char*)malloc((size_t)len + 1);
  for (int i = 0; i < len; i++) {
    uint16_t c = s[a + i];
    if (c >= 0x80) { if (tmp != buf) free(tmp); return -1; }
    tmp[i] = (char)c;
  }
  tmp[len] = 0;
  int i = 0, neg = 0, ok = 0;
  if (tmp[i] == '+' || tmp[i] == '-') { neg = tmp[i] == '-'; i++; }
  const char* rest = tmp + i;
  double v = 0.0;
  if (strcmp(rest, "NaN") == 0) {
    v = NAN; ok = 1;
  } else if (strcmp(rest, "Infinity") == 0) {
    v = neg ? -INFINITY : INFINITY; ok = 1;
  } else if (rest[0] == '0' && (rest[1] == 'x' || rest[1] == 'X')) {
    int j = i + 2, nd = 0;
    while (tmp[j] && ((tmp[j] >= '0' && tmp[j] <= '9') || (tmp[j] >= 'a' && tmp[j] <= 'f') ||
                      (tmp[j] >= 'A' && tmp[j] <= 'F'))) { j++; nd++; }
    if (tmp[j] == '.') {
      j++;
      while (tmp[j] && ((tmp[j] >= '0' && tmp[j] <= '9') || (tmp[j] >= 'a' && tmp[j] <= 'f') ||
                        (tmp[j] >= 'A' && tmp[j] <= 'F'))) { j++; nd++; }
    }
    if (nd > 0 && (tmp[j] == 'p' || tmp[j] == 'P')) {
      j++;
      if (tmp[j] == '+' || tmp[j] == '-') j++;
      int ne = 0;
      while (tmp[j] >= '0' && tmp[j] <= '9') { j++; ne++; }
      if (ne > 0) {
        if (tmp[j] == 'f' || tmp[j] == 'F' || tmp[j] == 'd' || tmp[j] == 'D') { tmp[j] = 0; j++; }
        if (tmp[j] == 0) { v = strtod(tmp, NULL); ok = 1; }
      }
    }
  } else {
    int j = i, nd = 0;
    while (tmp[j] >= '0' && tmp[j] <= '9') { j++; nd++; }
    if (tmp[j] == '.') {
      j++;
      while (tmp[j] >= '0' && tmp[j] <= '9') { j++; nd++; }
    }
    int good = nd > 0;
    if (good && (tmp[j] == 'e' || tmp[j] == 'E')) {
      j++;
      if (tmp[j] == '+' || tmp[j] == '-') j++;
      int ne = 0;
      while (tmp[j] >= '0' && tmp[j] <= '9') { j++; ne++; }
      if (ne == 0) good = 0;
    }
    if (good) {
      if (tmp[j] == 'f' || tmp[j] == 'F' || tmp[j] == 'd' || tmp[j] == 'D') { tmp[j] = 0; j++; }
      if (tmp[j] == 0) { v = strtod(tmp, NULL); ok = 1; }
    }
  }
  if (tmp != buf) free(tmp);
  if (!ok) return -1;
  *out = v;
  return 0;
}

/* [Duke 1.2] comparators.NumericComparator.compare: parse failure -> 0.5; both zero ->
 * 1.0; order so d1 <= d2 (by "d2 < d1" swap); ratio = d1/d2; ratio < minratio -> 0.0.
 * NaN, negative and infinite values flow through IEEE arithmetic exactly as in Java. */
double dko_numeric(const uint16_t* s1, int n1, const uint16_t* s2, int n2, double min_ratio) {
  double d1, d2;
  if (dko_parse_java_double(s1, n1, &d1) != 0) return 0.5;
  if (dko_parse_java_double(s2, n2, &d2) != 0) return 0.5;
  if (d1 == 0.0 && d2 == 0.0) return 1.0;
  if (d2 < d1) { double t = d2; d2 = d1; d1 = t; }
  double ratio = d1 / d2;
  if (ratio < min_ratio) return 0.0;
  return ratio;
}

/* [Duke 1.2, recalled, low confidence; parity unpinned: no Duke source or fixture here]
 * utils.Geoposition.parse: split at the first ',', Double.parseDouble of each half (degrees);
 * Geoposition.distance: haversine, R = 6371000 m, Math.toRadians as Java 8 (angdeg / 180.0 *
 * PI); comparators.GeopositionComparator.compare: unparsable -> 0.5, dist > maxdist -> 0.0,
 * else ((1.0 - (dist / maxdist)) * 0.5) + 0.5.  A value without ',' makes Geoposition.parse
 * raise: returns -1 here (the GPU path refuses such a value at upsert). */
int dko_parse_geoposition(const uint16_t* s, int n, double* lat, double* lng) {
  int comma = 0;
  while (comma < n && s[comma] != ',') comma++;
  if (comma == n) return -1;
  if (dko_parse_java_double(s, comma, lat) != 0) return 0;
  if (dko_parse_java_double(s + comma + 1, n - comma - 1, lng) != 0) return 0;
  return 1;
}

double dko_geoposition(const uint16_t* s1, int n1, const uint16_t* s2, int n2, double maxdist) {
  double la1, ln1, la2, ln2;
  if (dko_parse_geoposition(s1, n1, &la1, &ln1) != 1) return 0.5;
  if (dko_parse_geoposition(s2, n2, &la2, &ln2) != 1) return 0.5;
  const double pi = 3.141592653589793;
  double lat1 = la1 / 180.0 * pi, lat2 = la2 / 180.0 * pi;
  double dlat = (la2 - la1) / 180.0 * pi, dlng = (ln2 - ln1) / 180.0 * pi;
  double sl = sin(dlat / 2), sg = sin(dlng / 2);
  double a = sl * sl + sg * sg * cos(lat1) * cos(lat2);
  double dist = 6371000.0 * (2 * atan2(sqrt(a), sqrt(1 - a)));
  if (dist > maxdist) return 0.0;
  return ((1.0 - (dist / maxdist)) * 0.5) + 0.5;
}

/* [Duke 1.2, recalled, medium confidence] comparators.DefaultWeightEstimator.singleChar */
static double wl_weight(uint16_t ch) {
  if ((ch >= 'a' && ch <= 'z') || (ch >= 'A' && ch <= 'Z')) return 1.0;
  if (ch >= '0' && ch <= '9') return 2.0;
  if (ch == ' ' || ch == '\'' || ch == '.' || ch == '-' || ch == '/' || ch == '\\' ||
      ch == ',' || ch == '"')
    return 0.1;
  return 1.0;
}

/* [Duke 1.2, recalled, medium confidence] comparators.WeightedLevenshtein.distance: the
 * full flat matrix addressed s1ix + s1len*s2ix (stride s1len, so cell (s1len, c) aliases
 * cell (0, c+1)), evaluated s1-major exactly as the Java loop nest, including the
 * initialisation order that lets row init overwrite cell (0,1). */
static double wl_distance(const uint16_t* s1, int n1, const uint16_t* s2, int n2) {
  if (n1 == 0) { double e = 0.0; for (int i = 0; i < n2; i++) e += wl_weight(s2[i]); return e; }
  if (n2 == 0) { double e = 0.0; for (int i = 0; i < n1; i++) e += wl_weight(s1[i]); return e; }
  int s1len = n1;
  size_t sz = (size_t)(s1len + 1) * (size_t)(n2 + 1);
  double* m = (double*)malloc(sizeof(double) * sz);
  for (int col = 0; col <= n2; col++) m[(size_t)col * s1len] = col;
  for (int row = 0; row <= s1len; row++) m[row] = row;
  for (int ix1 = 0; ix1 < s1len; ix1++) {
    uint16_t ch1 = s1[ix1];
    for (int ix2 = 0; ix2 < n2; ix2++) {
      double cost = ch1 == s2[ix2] ? 0.0 : fmax(wl_weight(ch1), wl_weight(s2[ix2]));
      double left = m[ix1 + (size_t)(ix2 + 1) * s1len] + wl_weight(ch1);
      double above = m[ix1 + 1 + (size_t)ix2 * s1len] + wl_weight(s2[ix2]);
      double aboveleft = m[ix1 + (size_t)ix2 * s1len] + cost;
      double a = above < aboveleft ? above : aboveleft;
      m[ix1 + 1 + (size_t)(ix2 + 1) * s1len] = left < a ? left : a;
    }
  }
  double r = m[s1len + (size_t)n2 * s1len];
  free(m);
  return r;
}

/* [Duke 1.2, recalled, medium confidence] comparators.WeightedLevenshtein.compare */
double dko_weighted_levenshtein(const uint16_t* s1, int n1, const uint16_t* s2, int n2) {
  if (u16eq(s1, n1, s2, n2)) return 1.0;
  double dist = wl_distance(s1, n1, s2, n2);
  double maxlen = (double)imax(n1, n2);
  if (dist > maxlen) return 0.0;
  return 1.0 - (dist / maxlen);
}

/* [Duke 1.2, recalled] utils.StringUtils.split: the maximal runs of non-' ' units, as
 * (start, length) pairs; returns the token count. */
static int split_tokens(const uint16_t* s, int n, int* start, int* len) {
  int t = 0, i = 0;
  while (i < n) {
    while (i < n && s[i] == ' ') i++;
    if (i >= n) break;
    int a = i;
    while (i < n && s[i] != ' ') i++;
    start[t] = a;
    len[t] = i - a;
    t++;
  }
  return t;
}

/* [Duke 1.2, recalled, low confidence] comparators.DiceCoefficientComparator /
 * JaccardIndexComparator with the default ExactComparator sub-comparator: equal -> 1.0;
 * t1 = the token list with fewer tokens (s1 on a tie); for each t1 token the highest
 * sub-comparator score against t2 (Math.max from 0.0), summed; Dice = (sum * 2) /
 * (|t1| + |t2|); Jaccard = sum / union with union = |t1| + |t2| reduced by each highest. */
double dko_token_similarity(const uint16_t* s1, int n1, const uint16_t* s2, int n2, int jaccard) {
  if (u16eq(s1, n1, s2, n2)) return 1.0;
  int* b = (int*)malloc(sizeof(int) * (size_t)(2 * (n1 + n2) + 4));
  int *st1 = b, *ln1 = b + n1 + 1, *st2 = b + 2 * n1 + 2, *ln2 = st2 + n2 + 1;
  int m1 = split_tokens(s1, n1, st1, ln1);
  int m2 = split_tokens(s2, n2, st2, ln2);
  if (m1 > m2) {
    const uint16_t* ts = s1; s1 = s2; s2 = ts;
    int* tp = st1; st1 = st2; st2 = tp;
    tp = ln1; ln1 = ln2; ln2 = tp;
    int tm = m1; m1 = m2; m2 = tm;
  }
  double sum = 0.0, uni = (double)(m1 + m2);
  for (int i = 0; i < m1; i++) {
    double highest = 0.0;
    for (int j = 0; j < m2; j++)
      highest = dko_java_max(highest, dko_exact(s1 + st1[i], ln1[i], s2 + st2[j], ln2[j]));
    sum += highest;
    uni -= highest;
  }
  free(b);
  if (jaccard) return sum / uni;
  return (sum * 2) / (double)(m1 + m2);
}

/* java.lang.Math.max(double, double): NaN if either is NaN; +0.0 beats -0.0. */
double dko_java_max(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  if (a == 0.0 && b == 0.0) return signbit(a) ? b : a;
  return a >= b ? a : b;
}

/* [Duke 1.2] utils.Utils.computeBayes */
double dko_compute_bayes(double p1, double p2) {
  return (p1 * p2) / ((p1 * p2) + ((1.0 - p1) * (1.0 - p2)));
}

/* [Duke 1.2] PropertyImpl.compare: no comparator -> 0.5; sim < 0.5 -> low;
 * else ((high - 0.5) * (sim * sim)) + 0.5. */
double dko_property_compare(const dko_prop* p, const uint16_t* s1, int n1,
                            const uint16_t* s2, int n2) {
  double sim;
  switch (p->comparator) {
    case DKO_CMP_LEVENSHTEIN: sim = dko_levenshtein(s1, n1, s2, n2); break;
    case DKO_CMP_JAROWINKLER: sim = dko_jarowinkler(s1, n1, s2, n2); break;
    case DKO_CMP_QGRAM: sim = dko_qgram(s1, n1, s2, n2, p->q, p->formula, p->tokenizer); break;
    case DKO_CMP_EXACT: sim = dko_exact(s1, n1, s2, n2); break;
    case DKO_CMP_NUMERIC: sim = dko_numeric(s1, n1, s2, n2, p->min_ratio); break;
    case DKO_CMP_WEIGHTED_LEVENSHTEIN: sim = dko_weighted_levenshtein(s1, n1, s2, n2); break;
    case DKO_CMP_DICE_TOKENS: sim = dko_token_similarity(s1, n1, s2, n2, 0); break;
    case DKO_CMP_JACCARD_TOKENS: sim = dko_token_similarity(s1, n1, s2, n2, 1); break;
    case DKO_CMP_GEOPOSITION: sim = dko_geoposition(s1, n1, s2, n2, p->min_ratio); break;
    default: return 0.5;
  }
  if (sim < 0.5) return p->low;
  return ((p->high - 0.5) * (sim * sim)) + 0.5;
}

/* [Duke 1.2] Processor.compare(r1, r2): prob = 0.5; per property of r1 (in r1's RecordImpl
 * HashMap iteration order: the schema's order, or with order classes the one of r1's class,
 * which follows the map's capacity, IncrementalDataSource.java:67-98; ID / ignored
 * properties are not in the schema, App.java:309-323): skip if either side has no value;
 * high = 0.0, raised by Math.max with PropertyImpl.compare over the non-empty value pairs
 * (a record holds <= 1 value per property, IncrementalDataSource.java:69-72);
 * prob = computeBayes(prob, high). */
double dko_compare_rows(const dko_schema* s, const dko_table* t, uint32_t a, uint32_t b) {
  double prob = 0.5;
  const int oc = s->norders > 1 && t->oclass ? t->oclass[a] : 0;
  for (int k = 0; k < s->nprops; k++) {
    const int p = s->norders > 0 ? s->orders[oc * s->nprops + k] : k;
    if (!t->present[p][a] || !t->present[p][b]) continue;
    const uint32_t* off = t->off[p];
    const uint16_t* ch = t->chars[p];
    int n1 = (int)(off[a + 1] - off[a]);
    int n2 = (int)(off[b + 1] - off[b]);
    double high = 0.0;
    if (n1 > 0 && n2 > 0) {
      double v = dko_property_compare(&s->props[p], ch + off[a], n1, ch + off[b], n2);
      high = dko_java_max(high, v);
    }
    prob = dko_compute_bayes(prob, high);
  }
  return prob;
}

/* ------------------------------------------------------------------------------------ */
/* Candidate generation: exact-key blocking (SURVEY §8a-5 build contract).               */
/* cand(q) = U_k { r : key_k(r) == key_k(q), ident(r) != ident(q), alive(r), !deleted(r), */
/*                 group(r) != group(q) [linkage] }, listed key by key, rows ascending,   */
/*  a row already listed under an earlier key function skipped.                          */
/* ALLPAIRS (InMemoryDatabase semantics): every alive, non-deleted row, ascending.       */
/* ------------------------------------------------------------------------------------ */

typedef struct {
  const uint32_t* off;
  const uint16_t* ch;
} keycol;

static int key_cmp(const keycol* k, uint32_t a, uint32_t b) {
  int na = (int)(k->off[a + 1] - k->off[a]);
  int nb = (int)(k->off[b + 1] - k->off[b]);
  const uint16_t* pa = k->ch + k->off[a];
  const uint16_t* pb = k->ch + k->off[b];
  int n = imin(na, nb);
  for (int i = 0; i < n; i++)
    if (pa[i] != pb[i]) return pa[i] < pb[i] ? -1 : 1;
  return na < nb ? -1 : (na > nb ? 1 : 0);
}

static int key_eq(const dko_table* t, int k, uint32_t a, uint32_t b) {
  keycol kc = {t->key_off[k], t->key_chars[k]};
  return key_cmp(&kc, a, b) == 0;
}

typedef struct {
  const dko_table* t;
  keycol kc;
} sort_ctx;

/* merge sort of row ids by (key, row) — deterministic, no global state */
static void msort_rows(const sort_ctx* sc, uint32_t* a, uint32_t* tmp, uint64_t n) {
  if (n < 2) return;
  uint64_t h = n / 2;
  msort_rows(sc, a, tmp, h);
  msort_rows(sc, a + h, tmp, n - h);
  uint64_t i = 0, j = h, o = 0;
  while (i < h && j < n) {
    int c = key_cmp(&sc->kc, a[i], a[j]);
    if (c < 0 || (c == 0 && a[i] < a[j])) tmp[o++] = a[i++];
    else tmp[o++] = a[j++];
  }
  while (i < h) tmp[o++] = a[i++];
  while (j < n) tmp[o++] = a[j++];
  memcpy(a, tmp, sizeof(uint32_t) * n);
}

typedef struct {
  uint32_t* sorted;   /* alive rows sorted by (key, row) */
  uint64_t m;
  uint64_t* lo;       /* per row: block range in sorted[] */
  uint64_t* hi;
} block_index;

typedef struct {
  const dko_schema* s;
  const dko_table* t;
  const block_index* bi;
  const uint32_t* queries;
  uint64_t q0, q1;
  dko_result res;
  uint64_t cap;
  int err;
} work;

static void push(work* w, uint32_t q, uint32_t c, double p, uint8_t kind) {
  if (w->res.n == w->cap) {
    uint64_t nc = w->cap ? w->cap * 2 : 1024;
    w->res.query = (uint32_t*)realloc(w->res.query, nc * sizeof(uint32_t));
    w->res.candidate = (uint32_t*)realloc(w->res.candidate, nc * sizeof(uint32_t));
    w->res.prob = (double*)realloc(w->res.prob, nc * sizeof(double));
    w->res.kind = (uint8_t*)realloc(w->res.kind, nc);
    w->cap = nc;
  }
  w->res.query[w->res.n] = q;
  w->res.candidate[w->res.n] = c;
  w->res.prob[w->res.n] = p;
  w->res.kind[w->res.n] = kind;
  w->res.n++;
}

/* [Duke 1.2] Processor.compareCandidatesSimple for one (query, candidate). */
static void score_pair(work* w, uint32_t q, uint32_t c) {
  const dko_schema* s = w->s;
  double prob = dko_compare_rows(s, w->t, q, c);
  w->res.pairs_scored++;
  if (prob > s->threshold) push(w, q, c, prob, DKO_KIND_MATCH);
  else if (s->maybe_threshold != 0.0 && prob > s->maybe_threshold)
    push(w, q, c, prob, DKO_KIND_MAYBE);
}

static int row_usable(const dko_table* t, uint32_t q, uint32_t c) {
  if (t->alive && !t->alive[c]) return 0;
  if (t->deleted && t->deleted[c]) return 0;
  if (t->ident[c] == t->ident[q]) return 0; /* Processor.isSameAs on the ID property */
  return 1;
}

static void* worker(void* arg) {
  work* w = (work*)arg;
  const dko_schema* s = w->s;
  const dko_table* t = w->t;
  for (uint64_t qi = w->q0; qi < w->q1; qi++) {
    uint32_t q = w->queries[qi];
    if (s->mode == DKO_MODE_ALLPAIRS) {
      for (uint64_t c = 0; c < t->n; c++) {
        if (!row_usable(t, q, (uint32_t)c)) continue;
        score_pair(w, q, (uint32_t)c);
      }
      continue;
    }
    for (int k = 0; k < s->nkeys; k++) {
      const block_index* b = &w->bi[k];
      for (uint64_t pos = b->lo[q]; pos < b->hi[q]; pos++) {
        uint32_t c = b->sorted[pos];
        if (!row_usable(t, q, c)) continue;
        if (s->mode == DKO_MODE_LINKAGE && t->group[c] == t->group[q]) continue;
        int seen = 0;
        for (int j = 0; j < k && !seen; j++) seen = key_eq(t, j, q, c);
        if (seen) continue;
        score_pair(w, q, c);
      }
    }
  }
  return NULL;
}

int dko_match(const dko_schema* s, const dko_table* t, const uint32_t* queries, uint64_t nq,
              int nthreads, dko_result* out) {
  memset(out, 0, sizeof(*out));
  if (nthreads < 1) nthreads = 1;
  const double t0 = now_ms();
  int nk = s->mode == DKO_MODE_ALLPAIRS ? 0 : s->nkeys;
  block_index* bi = (block_index*)calloc((size_t)(nk > 0 ? nk : 1), sizeof(block_index));
  for (int k = 0; k < nk; k++) {
    sort_ctx sc = {t, {t->key_off[k], t->key_chars[k]}};
    uint32_t* rows = (uint32_t*)malloc(sizeof(uint32_t) * (t->n ? t->n : 1));
    uint64_t m = 0;
    for (uint64_t r = 0; r < t->n; r++)
      if (!t->alive || t->alive[r]) rows[m++] = (uint32_t)r;
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    msort_rows(&sc, rows, tmp, m);
    free(tmp);
    bi[k].sorted = rows;
    bi[k].m = m;
    bi[k].lo = (uint64_t*)calloc(t->n ? t->n : 1, sizeof(uint64_t));
    bi[k].hi = (uint64_t*)calloc(t->n ? t->n : 1, sizeof(uint64_t));
    uint64_t a = 0;
    while (a < m) {
      uint64_t e = a + 1;
      while (e < m && key_cmp(&sc.kc, rows[a], rows[e]) == 0) e++;
      for (uint64_t i = a; i < e; i++) { bi[k].lo[rows[i]] = a; bi[k].hi[rows[i]] = e; }
      a = e;
    }
  }
  /* a query row that is not alive still looks up its own key's block */
  for (int k = 0; k < nk; k++) {
    for (uint64_t qi = 0; qi < nq; qi++) {
      uint32_t q = queries[qi];
      if (t->alive && !t->alive[q]) {
        keycol kc = {t->key_off[k], t->key_chars[k]};
        uint64_t lo = 0, hi = bi[k].m;
        while (lo < hi) {
          uint64_t mid = (lo + hi) / 2;
          if (key_cmp(&kc, bi[k].sorted[mid], q) < 0) lo = mid + 1; else hi = mid;
        }
        uint64_t e = lo;
        while (e < bi[k].m && key_cmp(&kc, bi[k].sorted[e], q) == 0) e++;
        bi[k].lo[q] = lo; bi[k].hi[q] = e;
      }
    }
  }

  const double t1 = now_ms();
  work* ws = (work*)calloc((size_t)nthreads, sizeof(work));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int i = 0; i < nthreads; i++) {
    ws[i].s = s; ws[i].t = t; ws[i].bi = bi; ws[i].queries = queries;
    ws[i].q0 = nq * (uint64_t)i / (uint64_t)nthreads;
    ws[i].q1 = nq * (uint64_t)(i + 1) / (uint64_t)nthreads;
  }
  if (nthreads == 1) worker(&ws[0]);
  else {
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, worker, &ws[i]);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
  }
  const double t2 = now_ms();
  out->ms_index = t1 - t0;
  out->ms_score = t2 - t1;
  uint64_t total = 0;
  for (int i = 0; i < nthreads; i++) { total += ws[i].res.n; out->pairs_scored += ws[i].res.pairs_scored; }
  out->n = total;
  out->query = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
  out->candidate = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
  out->prob = (double*)malloc(sizeof(double) * (total ? total : 1));
  out->kind = (uint8_t*)malloc(total ? total : 1);
  uint64_t o = 0;
  for (int i = 0; i < nthreads; i++) {
    dko_result* r = &ws[i].res;
    if (r->n) {
      memcpy(out->query + o, r->query, r->n * sizeof(uint32_t));
      memcpy(out->candidate + o, r->candidate, r->n * sizeof(uint32_t));
      memcpy(out->prob + o, r->prob, r->n * sizeof(double));
      memcpy(out->kind + o, r->kind, r->n);
      o += r->n;
    }
    free(r->query); free(r->candidate); free(r->prob); free(r->kind);
  }
  for (int k = 0; k < nk; k++) { free(bi[k].sorted); free(bi[k].lo); free(bi[k].hi); }
  free(bi); free(ws); free(th);
  return 0;
}

void dko_free_result(dko_result* r) {
  free(r->query); free(r->candidate); free(r->prob); free(r->kind);
  memset(r, 0, sizeof(*r));
}
