// dk_links.cpp — the link sink of the match path: a LinkDatabase written in
// bulk from dk_match's arrays instead of one JDBC / listener round trip per link.  Host C++.
//
// Semantics followed:
//   * SinceAwareInMemoryLinkDatabase (SinceAwareInMemoryLinkDatabase.java:12-41): assertLink
//     skips a link when the stored link between the same two IDs has the same status and kind
//     and a confidence within 1e-6 (so its timestamp survives); getChangesSince(since) =
//     every link with timestamp > since;
//   * [Duke 1.2, recalled -- PARITY UNPINNED, the Duke jar is absent] InMemoryLinkDatabase:
//     one link per unordered ID pair, assertLink replaces it; Link orders its two IDs
//     (String.compareTo: the smaller is ID1), status INFERRED / RETRACTED, kind SAME (matches)
//     / MAYBE (matchesPerhaps), timestamp at creation, retract() = RETRACTED + new timestamp;
//   * [Duke 1.2, recalled] LinkDatabaseMatchListener, which BaseLinkDatabaseMatchListener
//     forwards every callback to (BaseLinkDatabaseMatchListener.java:53-109): the links of one
//     query record (its matches / matchesPerhaps, or noMatchFor) are reconciled with the
//     record's stored links when the record ends -- stored INFERRED links between the same
//     IDs are replaced by the new ones, stored INFERRED links the record no longer produced
//     are retracted, then the new links are asserted -- record by record in batch order.
// One timestamp per batch (the caller's clock at the batch): Duke stamps each Link when it
// is built, milliseconds apart within one deduplicate call.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "dk_interner.h"
#include "dukehip.h"

extern "C" int dk_fail_ingest(int code, const char* msg);  // dk_api.cpp: sets dk_last_error

namespace {

struct PairHash {
  size_t operator()(const std::pair<uint64_t, uint64_t>& p) const {
    uint64_t h = p.first * 0x9E3779B97F4A7C15ull ^ (p.second + 0x632BE59BD9B4E019ull + (p.first << 6));
    return (size_t)(h ^ (h >> 29));
  }
};

struct LinkRec {
  uint64_t id1, id2;
  uint8_t status, kind;
  double confidence;
  int64_t timestamp;
  uint64_t seq;  // assertion order (the change feed's order among equal timestamps)
};

}  // namespace

struct dk_linkdb {
  const dk_interner* ids = nullptr;
  std::unordered_map<std::pair<uint64_t, uint64_t>, LinkRec, PairHash> links;
  std::unordered_map<uint64_t, std::vector<std::pair<uint64_t, uint64_t>>> by_id;  // links of an ID
  uint64_t seq = 0;

  // Link's ID order: String.compareTo of the two record IDs (UTF-16 code units)
  std::pair<uint64_t, uint64_t> key(uint64_t a, uint64_t b) const {
    return ids->compare(a, b) <= 0 ? std::make_pair(a, b) : std::make_pair(b, a);
  }

  // SinceAwareInMemoryLinkDatabase.assertLink, then InMemoryLinkDatabase.assertLink
  bool assert_link(const LinkRec& l) {
    const auto k = std::make_pair(l.id1, l.id2);
    auto it = links.find(k);
    if (it != links.end()) {
      const LinkRec& o = it->second;
      if (o.status == l.status && o.kind == l.kind && std::fabs(l.confidence - o.confidence) < 0.000001)
        return false;
      it->second = l;
      it->second.seq = seq++;
      return true;
    }
    LinkRec n = l;
    n.seq = seq++;
    links.emplace(k, n);
    by_id[l.id1].push_back(k);
    if (l.id2 != l.id1) by_id[l.id2].push_back(k);
    return true;
  }
};

extern "C" {

int dk_interner_string(const dk_interner* it, uint64_t id, const uint16_t** units, uint64_t* n) {
  if (!it || !units || !n) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  if (id >= it->size()) return dk_fail_ingest(DK_E_INVALID, "id not interned");
  *units = reinterpret_cast<const uint16_t*>(it->str(id));
  *n = it->len(id);
  return DK_OK;
}

int dk_linkdb_create(const dk_interner* ids, dk_linkdb** out) {
  if (!ids || !out) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  *out = new (std::nothrow) dk_linkdb();
  if (!*out) return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  (*out)->ids = ids;
  return DK_OK;
}

void dk_linkdb_destroy(dk_linkdb* db) { delete db; }

uint64_t dk_linkdb_size(const dk_linkdb* db) { return db ? db->links.size() : 0; }

int dk_linkdb_apply(dk_linkdb* db, const dk_link_batch* b, int64_t timestamp, dk_link_stats* stats) {
  if (!db || !b) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  if (b->nqueries && (!b->query_ident || !b->first)) return dk_fail_ingest(DK_E_INVALID, "NULL arrays");
  const uint64_t nq = b->nqueries;
  const uint64_t ne = nq ? b->first[nq] : 0;
  if (ne && (!b->candidate_ident || !b->prob || !b->kind)) return dk_fail_ingest(DK_E_INVALID, "NULL arrays");
  const uint64_t nid = db->ids->size();
  for (uint64_t i = 0; i < nq; ++i) {
    if (b->first[i] > b->first[i + 1]) return dk_fail_ingest(DK_E_INVALID, "first[] not monotone");
    if (b->query_ident[i] >= nid) return dk_fail_ingest(DK_E_INVALID, "query ident not interned");
  }
  for (uint64_t e = 0; e < ne; ++e) {
    if (b->candidate_ident[e] >= nid) return dk_fail_ingest(DK_E_INVALID, "candidate ident not interned");
    if (b->kind[e] != DK_KIND_MATCH && b->kind[e] != DK_KIND_MAYBE)
      return dk_fail_ingest(DK_E_INVALID, "entry kind not MATCH / MAYBE");
  }
  dk_link_stats st{};
  try {
    std::unordered_map<std::pair<uint64_t, uint64_t>, LinkRec, PairHash> cur;
    std::vector<std::pair<uint64_t, uint64_t>> order;
    for (uint64_t i = 0; i < nq; ++i) {
      const uint64_t q = b->query_ident[i];
      // the record's new links (a repeated pair keeps the later callback's link)
      cur.clear();
      order.clear();
      for (uint64_t e = b->first[i]; e < b->first[i + 1]; ++e) {
        const auto k = db->key(q, b->candidate_ident[e]);
        LinkRec l{k.first, k.second, (uint8_t)DK_LINK_INFERRED,
                  (uint8_t)(b->kind[e] == DK_KIND_MATCH ? DK_LINK_SAME : DK_LINK_MAYBE), b->prob[e],
                  timestamp, 0};
        if (cur.emplace(k, l).second) order.push_back(k);
        else cur[k] = l;
      }
      // stored INFERRED links of the record it did not produce again: retracted
      auto bi = db->by_id.find(q);
      if (bi != db->by_id.end()) {
        const std::vector<std::pair<uint64_t, uint64_t>> mine = bi->second;  // assert may append
        for (const auto& k : mine) {
          if (cur.count(k)) continue;
          auto it = db->links.find(k);
          if (it == db->links.end() || it->second.status != DK_LINK_INFERRED) continue;
          LinkRec r = it->second;
          r.status = DK_LINK_RETRACTED;
          r.timestamp = timestamp;
          if (db->assert_link(r)) st.retracted += 1;
        }
      }
      for (const auto& k : order) {
        if (db->assert_link(cur[k])) st.asserted += 1;
        else st.unchanged += 1;
      }
    }
  } catch (const std::bad_alloc&) {
    return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  }
  if (stats) *stats = st;
  return DK_OK;
}

namespace {
struct LinkList {
  dk_link_list pub{};
  std::vector<uint64_t> id1, id2;
  std::vector<uint8_t> status, kind;
  std::vector<double> confidence;
  std::vector<int64_t> timestamp;
};
}  // namespace

int dk_linkdb_changes_since(const dk_linkdb* db, int64_t since, dk_link_list** out) {
  if (!db || !out) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  *out = nullptr;
  LinkList* L = new (std::nothrow) LinkList();
  if (!L) return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  try {
    std::vector<const LinkRec*> sel;
    for (const auto& kv : db->links)
      if (kv.second.timestamp > since) sel.push_back(&kv.second);
    // Java HashMap iteration order in the reference (unpinned): here (timestamp, assertion)
    std::sort(sel.begin(), sel.end(), [](const LinkRec* a, const LinkRec* b) {
      return a->timestamp != b->timestamp ? a->timestamp < b->timestamp : a->seq < b->seq;
    });
    const size_t n = sel.size();
    L->id1.resize(n);
    L->id2.resize(n);
    L->status.resize(n);
    L->kind.resize(n);
    L->confidence.resize(n);
    L->timestamp.resize(n);
    for (size_t i = 0; i < n; ++i) {
      L->id1[i] = sel[i]->id1;
      L->id2[i] = sel[i]->id2;
      L->status[i] = sel[i]->status;
      L->kind[i] = sel[i]->kind;
      L->confidence[i] = sel[i]->confidence;
      L->timestamp[i] = sel[i]->timestamp;
    }
  } catch (const std::bad_alloc&) {
    delete L;
    return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  }
  L->pub.n = L->id1.size();
  L->pub.id1 = L->id1.data();
  L->pub.id2 = L->id2.data();
  L->pub.status = L->status.data();
  L->pub.kind = L->kind.data();
  L->pub.confidence = L->confidence.data();
  L->pub.timestamp = L->timestamp.data();
  *out = &L->pub;
  return DK_OK;
}

void dk_free_link_list(dk_link_list* l) { delete reinterpret_cast<LinkList*>(l); }

static int list_of(const std::vector<const LinkRec*>& sel, dk_link_list** out) {
  LinkList* L = new (std::nothrow) LinkList();
  if (!L) return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  try {
    for (const LinkRec* r : sel) {
      L->id1.push_back(r->id1);
      L->id2.push_back(r->id2);
      L->status.push_back(r->status);
      L->kind.push_back(r->kind);
      L->confidence.push_back(r->confidence);
      L->timestamp.push_back(r->timestamp);
    }
  } catch (const std::bad_alloc&) {
    delete L;
    return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  }
  L->pub.n = L->id1.size();
  L->pub.id1 = L->id1.data();
  L->pub.id2 = L->id2.data();
  L->pub.status = L->status.data();
  L->pub.kind = L->kind.data();
  L->pub.confidence = L->confidence.data();
  L->pub.timestamp = L->timestamp.data();
  *out = &L->pub;
  return DK_OK;
}

// InMemoryLinkDatabase.getAllLinksFor [recalled]: the links of one record ID, in the order
// they were first asserted
int dk_linkdb_links_for(const dk_linkdb* db, uint64_t id, dk_link_list** out) {
  if (!db || !out) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  *out = nullptr;
  std::vector<const LinkRec*> sel;
  try {
    auto bi = db->by_id.find(id);
    if (bi != db->by_id.end())
      for (const auto& k : bi->second) {
        auto it = db->links.find(k);
        if (it != db->links.end()) sel.push_back(&it->second);
      }
  } catch (const std::bad_alloc&) {
    return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  }
  return list_of(sel, out);
}

// The deleted-record branch of the POST route (App.java:994-999): for every link of the
// record, Link.retract() [recalled: status RETRACTED, timestamp now] on the stored link itself,
// then assertLink -- so even an already retracted link takes the new timestamp.  `other` ==
// UINT64_MAX: every link of `id`; else the one link between the two IDs.
int dk_linkdb_retract(dk_linkdb* db, uint64_t id, uint64_t other, int64_t timestamp, uint64_t* nretracted) {
  if (!db) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  uint64_t n = 0;
  auto bi = db->by_id.find(id);
  if (bi != db->by_id.end())
    for (const auto& k : bi->second) {
      if (other != UINT64_MAX && k != db->key(id, other)) continue;
      auto it = db->links.find(k);
      if (it == db->links.end()) continue;
      it->second.status = DK_LINK_RETRACTED;
      it->second.timestamp = timestamp;
      it->second.seq = db->seq++;
      ++n;
    }
  if (nretracted) *nretracted = n;
  return DK_OK;
}

}  // extern "C"
