/* dk_harness.c -- a plain C caller of libdukehip.so (no C++, no Python): the C-ABI exactly as a
 * JNI / cgo / N-API shim would bind it (include/dukehip.h).
 *
 * Input (argv[1], a text file):
 *   line 1: nprops nkeys mode threshold maybe_threshold
 *   nprops lines: comparator q formula tokenizer low high min_ratio
 *   then one record per line, tab separated: ident, deleted (0/1), group (0/1/2), nprops values
 *   ("\N" = no value), nkeys key strings; values are UTF-8 (ASCII here: width-1 columns).
 * Optional argv[2]: the batch boundaries as a comma list of record counts (upserts in order).
 * Output (stdout): for dk_match over every record, one line per query:
 *   q <query row> then " <candidate> <kind> <prob as %a>" per entry;
 *   then "scored <pairs_scored>" and, for row pair (0, 1), "compare <dk_compare_rows as %a>".
 * Exit status: 0, or 2 on a dk_* error (its dk_last_error on stderr).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dukehip.h"

#define MAXF 32

static void die(const char* what, int rc) {
  fprintf(stderr, "%s failed (%d): %s\n", what, rc, dk_last_error());
  exit(2);
}

typedef struct {
  uint64_t n, cap;
  uint64_t* ident;
  uint8_t *deleted, *group;
  char*** fields; /* [record][field] */
} Records;

static char* dupn(const char* s, size_t n) {
  char* o = (char*)malloc(n + 1);
  memcpy(o, s, n);
  o[n] = 0;
  return o;
}

/* one column (width 1) of records [a, b) of field f */
static dk_column pack(const Records* R, uint64_t a, uint64_t b, int f, uint32_t** off_out,
                      uint8_t** units_out, uint8_t** present_out) {
  uint64_t n = b - a, total = 0;
  for (uint64_t i = a; i < b; ++i)
    if (strcmp(R->fields[i][f], "\\N")) total += strlen(R->fields[i][f]);
  uint32_t* off = (uint32_t*)malloc((n + 1) * 4);
  uint8_t* units = (uint8_t*)malloc(total + 1);
  uint8_t* present = (uint8_t*)malloc(n + 1);
  off[0] = 0;
  for (uint64_t i = a; i < b; ++i) {
    const char* v = R->fields[i][f];
    const int has = strcmp(v, "\\N") != 0;
    const size_t l = has ? strlen(v) : 0;
    memcpy(units + off[i - a], v, l);
    off[i - a + 1] = off[i - a] + (uint32_t)l;
    present[i - a] = (uint8_t)has;
  }
  *off_out = off;
  *units_out = units;
  *present_out = present;
  dk_column c;
  c.offsets = off;
  c.units = units;
  c.width = 1;
  c.present = present;
  return c;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s input.txt [batch sizes]\n", argv[0]);
    return 1;
  }
  FILE* fp = fopen(argv[1], "r");
  if (!fp) {
    perror(argv[1]);
    return 1;
  }
  dk_schema schema;
  memset(&schema, 0, sizeof schema);
  int nprops = 0, nkeys = 0, mode = 0;
  if (fscanf(fp, "%d %d %d %lf %lf", &nprops, &nkeys, &mode, &schema.threshold, &schema.maybe_threshold) != 5)
    return 1;
  dk_property props[16];
  for (int p = 0; p < nprops; ++p) {
    dk_property* d = &props[p];
    if (fscanf(fp, "%d %d %d %d %lf %lf %lf", &d->comparator, &d->qgram_q, &d->qgram_formula,
               &d->qgram_tokenizer, &d->low, &d->high, &d->min_ratio) != 7)
      return 1;
  }
  schema.nprops = nprops;
  schema.props = props;
  schema.mode = mode;
  schema.nkeys = nkeys;
  Records R;
  memset(&R, 0, sizeof R);
  static char line[1 << 16];
  if (!fgets(line, sizeof line, fp)) return 1; /* rest of the header line */
  while (fgets(line, sizeof line, fp)) {
    size_t L = strlen(line);
    while (L && (line[L - 1] == '\n' || line[L - 1] == '\r')) line[--L] = 0;
    if (!L) continue;
    if (R.n == R.cap) {
      R.cap = R.cap ? 2 * R.cap : 1024;
      R.ident = (uint64_t*)realloc(R.ident, R.cap * 8);
      R.deleted = (uint8_t*)realloc(R.deleted, R.cap);
      R.group = (uint8_t*)realloc(R.group, R.cap);
      R.fields = (char***)realloc(R.fields, R.cap * sizeof(char**));
    }
    char* f[MAXF];
    int nf = 0;
    char* s = line;
    for (;;) {
      char* t = strchr(s, '\t');
      f[nf++] = s;
      if (!t || nf == MAXF) break;
      *t = 0;
      s = t + 1;
    }
    if (nf != 3 + nprops + nkeys) {
      fprintf(stderr, "record %llu: %d fields\n", (unsigned long long)R.n, nf);
      return 1;
    }
    R.ident[R.n] = strtoull(f[0], NULL, 10);
    R.deleted[R.n] = (uint8_t)atoi(f[1]);
    R.group[R.n] = (uint8_t)atoi(f[2]);
    R.fields[R.n] = (char**)malloc((size_t)(nprops + nkeys) * sizeof(char*));
    for (int i = 0; i < nprops + nkeys; ++i) R.fields[R.n][i] = dupn(f[3 + i], strlen(f[3 + i]));
    R.n++;
  }
  fclose(fp);

  if (dk_abi_version() != DK_ABI_VERSION) {
    fprintf(stderr, "library ABI %d, header %d\n", dk_abi_version(), DK_ABI_VERSION);
    return 2;
  }
  dk_ctx* ctx = NULL;
  int rc = dk_create(&schema, 0, &ctx);
  if (rc) die("dk_create", rc);

  /* upsert in the given batches (Processor.deduplicate's index + commit, batch by batch) */
  uint64_t at = 0;
  char* spec = argc > 2 ? argv[2] : NULL;
  while (at < R.n) {
    uint64_t b = R.n;
    if (spec && *spec) {
      b = at + strtoull(spec, &spec, 10);
      if (*spec == ',') spec++;
      if (b > R.n) b = R.n;
    }
    const uint64_t n = b - at;
    dk_column cols[16], kcols[8];
    uint32_t* offs[24];
    uint8_t *units[24], *pres[24];
    for (int p = 0; p < nprops; ++p) cols[p] = pack(&R, at, b, p, &offs[p], &units[p], &pres[p]);
    for (int k = 0; k < nkeys; ++k)
      kcols[k] = pack(&R, at, b, nprops + k, &offs[nprops + k], &units[nprops + k], &pres[nprops + k]);
    dk_batch batch;
    memset(&batch, 0, sizeof batch);
    batch.n = n;
    batch.ident = R.ident + at;
    batch.group = mode == DK_MODE_LINKAGE ? R.group + at : NULL;
    batch.deleted = R.deleted + at;
    batch.columns = cols;
    batch.key_columns = nkeys ? kcols : NULL;
    uint32_t* rows = (uint32_t*)malloc(n * 4 + 4);
    rc = dk_upsert(ctx, &batch, rows);
    if (rc) die("dk_upsert", rc);
    for (uint64_t i = 0; i < n; ++i)
      if (rows[i] != at + i) {
        fprintf(stderr, "row %u for record %llu\n", rows[i], (unsigned long long)(at + i));
        return 2;
      }
    free(rows);
    for (int i = 0; i < nprops + nkeys; ++i) {
      free(offs[i]);
      free(units[i]);
      free(pres[i]);
    }
    at = b;
  }

  uint32_t* q = (uint32_t*)malloc(R.n * 4 + 4);
  for (uint64_t i = 0; i < R.n; ++i) q[i] = (uint32_t)i;
  dk_result* res = NULL;
  rc = dk_match(ctx, q, R.n, DK_MATCH_HOST, &res);
  if (rc) die("dk_match", rc);
  for (uint64_t i = 0; i < res->nqueries; ++i) {
    printf("q %llu", (unsigned long long)q[i]);
    for (uint64_t e = res->first[i]; e < res->first[i + 1]; ++e)
      printf(" %u %u %a", res->candidate[e], (unsigned)res->kind[e], res->prob[e]);
    printf("\n");
  }
  printf("scored %llu\n", (unsigned long long)res->pairs_scored);
  dk_free_result(res);
  if (R.n >= 2) {
    double p = 0.0;
    rc = dk_compare_rows(ctx, 0, 1, &p);
    if (rc) die("dk_compare_rows", rc);
    printf("compare %a\n", p);
  }
  dk_destroy(ctx);
  free(q);
  return 0;
}
