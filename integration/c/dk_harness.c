/* dk_harness.c -- a plain C caller of libdukehip.so (no C++, no Python): the C-ABI exactly as a
 * JNI / cgo / N-API shim would bind it (include/dukehip.h).
 *
 * Input (argv[1], a text file):
 *   line 1: nprops nkeys mode threshold maybe_threshold
 *   nprops lines: comparator q formula tokenizer low high min_ratio
 *   then one record per line, tab separated: ident, deleted (0/1), group (0/1/2), nprops values
 *   ("\N" = no value), nkeys key strings; values are UTF-8 (a column holding a non-ASCII
 *   character is passed as UTF-16 units, width 2; ASCII columns as width 1).
 * Optional argv[2]: the batch boundaries as a comma list of record counts (upserts in order;
 * "-" = one batch).  Options after it:
 *   --devices D0,D1,...      dk_create_multi over these devices (one replicated handle)
 *   --lucene P,P:HITS:REL    the Lucene candidate source (dk_schema.lucene): lookup
 *                            properties (schema indices), max hits, min relevance; nkeys 0
 *   --per-batch              Processor.deduplicate per batch: after each upsert, dk_match over
 *                            that batch's rows (output "batch <i>" then its q lines)
 *   --linkdb                 (with --per-batch) the record ID strings are the ident columns;
 *                            they are interned (dk_interner_intern) into the batch idents, each
 *                            batch's list goes into a dk_linkdb (timestamp = batch number + 1)
 *                            and the feed (dk_linkdb_changes_since 0) is printed at the end
 * Output (stdout): per query "q <query row>" then " <candidate> <kind> <prob as %a>" per entry;
 *   "scored <pairs_scored>" per match; for row pair (0, 1), "compare <dk_compare_rows as %a>";
 *   with --linkdb, "link <id1> <id2> <status> <kind> <confidence as %a> <timestamp>" lines.
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
  char** idstr;   /* [record]: the ident column as given */
} Records;

static char* dupn(const char* s, size_t n) {
  char* o = (char*)malloc(n + 1);
  memcpy(o, s, n);
  o[n] = 0;
  return o;
}

/* UTF-8 -> UTF-16 code units (surrogate pairs above the BMP); returns the unit count */
static size_t utf16_of(const char* s, uint16_t* out) {
  const unsigned char* p = (const unsigned char*)s;
  size_t n = 0;
  while (*p) {
    uint32_t c = *p++;
    if (c >= 0xF0) {
      c = ((c & 0x07u) << 18) | ((uint32_t)(p[0] & 0x3F) << 12) | ((uint32_t)(p[1] & 0x3F) << 6) | (p[2] & 0x3Fu);
      p += 3;
    } else if (c >= 0xE0) {
      c = ((c & 0x0Fu) << 12) | ((uint32_t)(p[0] & 0x3F) << 6) | (p[1] & 0x3Fu);
      p += 2;
    } else if (c >= 0xC0) {
      c = ((c & 0x1Fu) << 6) | (p[0] & 0x3Fu);
      p += 1;
    }
    if (c >= 0x10000) {
      c -= 0x10000;
      if (out) {
        out[n] = (uint16_t)(0xD800 + (c >> 10));
        out[n + 1] = (uint16_t)(0xDC00 + (c & 0x3FF));
      }
      n += 2;
    } else {
      if (out) out[n] = (uint16_t)c;
      n += 1;
    }
  }
  return n;
}

static int is_ascii(const char* s) {
  for (; *s; ++s)
    if ((unsigned char)*s >= 0x80) return 0;
  return 1;
}

typedef struct {
  uint32_t* off;
  void* units;
  uint8_t* present;
} Packed;

/* one column of records [a, b): field f, or (f < 0) the record ID strings */
static dk_column pack(const Records* R, uint64_t a, uint64_t b, int f, Packed* pk) {
  uint64_t n = b - a, total = 0;
  int wide = 0;
  for (uint64_t i = a; i < b; ++i) {
    const char* v = f < 0 ? R->idstr[i] : R->fields[i][f];
    if (strcmp(v, "\\N")) {
      total += strlen(v);
      wide = wide || !is_ascii(v);
    }
  }
  uint32_t* off = (uint32_t*)malloc((n + 1) * 4);
  void* units = malloc(total * 2 + 2);
  uint8_t* present = (uint8_t*)malloc(n + 1);
  off[0] = 0;
  for (uint64_t i = a; i < b; ++i) {
    const char* v = f < 0 ? R->idstr[i] : R->fields[i][f];
    const int has = strcmp(v, "\\N") != 0;
    size_t l = 0;
    if (has && wide) l = utf16_of(v, (uint16_t*)units + off[i - a]);
    else if (has) {
      l = strlen(v);
      memcpy((uint8_t*)units + off[i - a], v, l);
    }
    off[i - a + 1] = off[i - a] + (uint32_t)l;
    present[i - a] = (uint8_t)has;
  }
  pk->off = off;
  pk->units = units;
  pk->present = present;
  dk_column c;
  c.offsets = off;
  c.units = units;
  c.width = wide ? 2 : 1;
  c.present = present;
  return c;
}

static void unpack(Packed* pk) {
  free(pk->off);
  free(pk->units);
  free(pk->present);
}

static void print_result(const dk_result* res, const uint32_t* q) {
  for (uint64_t i = 0; i < res->nqueries; ++i) {
    printf("q %llu", (unsigned long long)q[i]);
    for (uint64_t e = res->first[i]; e < res->first[i + 1]; ++e)
      printf(" %u %u %a", res->candidate[e], (unsigned)res->kind[e], res->prob[e]);
    printf("\n");
  }
  printf("scored %llu\n", (unsigned long long)res->pairs_scored);
}

static void print_string(const dk_interner* ids, uint64_t id) {
  const uint16_t* u = NULL;
  uint64_t n = 0;
  int rc = dk_interner_string(ids, id, &u, &n);
  if (rc) die("dk_interner_string", rc);
  for (uint64_t i = 0; i < n; ++i) putchar(u[i] < 0x80 ? (int)u[i] : '?');
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s input.txt [batch sizes|-] [--devices ..] [--lucene ..] [--per-batch] [--linkdb]\n",
            argv[0]);
    return 1;
  }
  int devices[16], ndev = 0, per_batch = 0, linkdb = 0;
  int32_t lookup[16];
  dk_lucene luc;
  memset(&luc, 0, sizeof luc);
  for (int a = 3; a < argc; ++a) {
    if (!strcmp(argv[a], "--devices") && a + 1 < argc) {
      char* s = argv[++a];
      while (*s && ndev < 16) {
        devices[ndev++] = (int)strtol(s, &s, 10);
        if (*s == ',') s++;
      }
    } else if (!strcmp(argv[a], "--lucene") && a + 1 < argc) {
      char* s = argv[++a];
      while (*s && *s != ':' && luc.nlookup < 16) {
        lookup[luc.nlookup++] = (int32_t)strtol(s, &s, 10);
        if (*s == ',') s++;
      }
      if (*s == ':') luc.max_hits = (int32_t)strtol(s + 1, &s, 10);
      if (*s == ':') luc.min_relevance = (float)strtod(s + 1, &s);
      luc.lookup_prop = lookup;
    } else if (!strcmp(argv[a], "--per-batch")) {
      per_batch = 1;
    } else if (!strcmp(argv[a], "--linkdb")) {
      linkdb = 1;
    } else {
      fprintf(stderr, "unknown option %s\n", argv[a]);
      return 1;
    }
  }
  if (linkdb && !per_batch) {
    fprintf(stderr, "--linkdb needs --per-batch\n");
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
  schema.lucene = luc.nlookup ? &luc : NULL;
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
      R.idstr = (char**)realloc(R.idstr, R.cap * sizeof(char*));
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
    R.idstr[R.n] = dupn(f[0], strlen(f[0]));
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
  int rc = ndev ? dk_create_multi(&schema, devices, ndev, &ctx) : dk_create(&schema, 0, &ctx);
  if (rc) die(ndev ? "dk_create_multi" : "dk_create", rc);
  dk_interner* ids = NULL;
  dk_linkdb* db = NULL;
  uint64_t* row_ident = NULL; /* row -> interned record ID (linkdb) */
  if (linkdb) {
    if ((rc = dk_interner_create(&ids))) die("dk_interner_create", rc);
    if ((rc = dk_linkdb_create(ids, &db))) die("dk_linkdb_create", rc);
    row_ident = (uint64_t*)malloc(R.n * 8 + 8);
  }

  /* upsert in the given batches (Processor.deduplicate's index + commit, batch by batch) */
  uint64_t at = 0;
  int batch_no = 0;
  char* spec = argc > 2 && strcmp(argv[2], "-") ? argv[2] : NULL;
  while (at < R.n) {
    uint64_t b = R.n;
    if (spec && *spec) {
      b = at + strtoull(spec, &spec, 10);
      if (*spec == ',') spec++;
      if (b > R.n) b = R.n;
    }
    const uint64_t n = b - at;
    dk_column cols[16], kcols[8];
    Packed pk[24];
    for (int p = 0; p < nprops; ++p) cols[p] = pack(&R, at, b, p, &pk[p]);
    for (int k = 0; k < nkeys; ++k) kcols[k] = pack(&R, at, b, nprops + k, &pk[nprops + k]);
    dk_batch batch;
    memset(&batch, 0, sizeof batch);
    batch.n = n;
    batch.ident = R.ident + at;
    if (linkdb) {  /* the record ID strings interned: equal idents <=> equal ID strings */
      Packed ip;
      dk_column idc = pack(&R, at, b, -1, &ip);
      if ((rc = dk_interner_intern(ids, &idc, n, row_ident + at))) die("dk_interner_intern", rc);
      unpack(&ip);
      batch.ident = row_ident + at;
    }
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
    for (int i = 0; i < nprops + nkeys; ++i) unpack(&pk[i]);
    if (per_batch) {  /* Processor.deduplicate: the batch's records against the index so far */
      dk_result* res = NULL;
      if ((rc = dk_match(ctx, rows, n, DK_MATCH_HOST, &res))) die("dk_match", rc);
      printf("batch %d\n", batch_no);
      print_result(res, rows);
      if (linkdb) {
        uint64_t* cid = (uint64_t*)malloc(res->n * 8 + 8);
        for (uint64_t e = 0; e < res->n; ++e) cid[e] = row_ident[res->candidate[e]];
        dk_link_batch lb;
        lb.nqueries = n;
        lb.query_ident = row_ident + at;
        lb.first = res->first;
        lb.candidate_ident = cid;
        lb.prob = res->prob;
        lb.kind = res->kind;
        dk_link_stats st;
        if ((rc = dk_linkdb_apply(db, &lb, batch_no + 1, &st))) die("dk_linkdb_apply", rc);
        free(cid);
      }
      dk_free_result(res);
    }
    free(rows);
    at = b;
    batch_no++;
  }

  if (!per_batch) {
    uint32_t* q = (uint32_t*)malloc(R.n * 4 + 4);
    for (uint64_t i = 0; i < R.n; ++i) q[i] = (uint32_t)i;
    dk_result* res = NULL;
    rc = dk_match(ctx, q, R.n, DK_MATCH_HOST, &res);
    if (rc) die("dk_match", rc);
    print_result(res, q);
    dk_free_result(res);
    free(q);
  }
  if (R.n >= 2) {
    double p = 0.0;
    rc = dk_compare_rows(ctx, 0, 1, &p);
    if (rc) die("dk_compare_rows", rc);
    printf("compare %a\n", p);
  }
  if (linkdb) {
    dk_link_list* ll = NULL;
    if ((rc = dk_linkdb_changes_since(db, 0, &ll))) die("dk_linkdb_changes_since", rc);
    for (uint64_t i = 0; i < ll->n; ++i) {
      printf("link ");
      print_string(ids, ll->id1[i]);
      putchar(' ');
      print_string(ids, ll->id2[i]);
      printf(" %u %u %a %lld\n", (unsigned)ll->status[i], (unsigned)ll->kind[i], ll->confidence[i],
             (long long)ll->timestamp[i]);
    }
    dk_free_link_list(ll);
    dk_linkdb_destroy(db);
    dk_interner_destroy(ids);
    free(row_ident);
  }
  dk_destroy(ctx);
  return 0;
}
