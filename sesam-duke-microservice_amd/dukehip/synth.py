"""Deterministic synthetic person records (SURVEY §8d `synth_persons`).

No dataset can be fetched, so names, streets and cities are built from syllables with a
seeded PCG64 generator: 5,000 given names (Zipf s=1.1), 20,000 surnames (Zipf s=1.07),
3,000 streets, 1,000 cities, dob uniform 1930-01-01..2010-12-31.  Duplicates copy an
original and corrupt each field with p=0.3 by 1-2 edits (substitution / insertion /
deletion / adjacent swap over a-z); dob gets a day<->month swap with p=0.1.
"""
from __future__ import annotations

import datetime as _dt

import numpy as np

from ._abi import Column

SEED = 20261015
_CONS = list("bcdfghjklmnprstvwz") + ["ch", "sh", "th", "br", "tr", "st", "kr", "gr", "l", "n"]
_VOW = list("aeiou") + ["ai", "ea", "ou", "ie", "y"]
_SUFFIX = ["street", "avenue", "road", "lane", "drive", "way", "court", "place", "gate", "vei"]


def _vocab(rng, n, syl_lo, syl_hi, cap=True):
    out, seen = [], set()
    while len(out) < n:
        k = int(rng.integers(syl_lo, syl_hi + 1))
        w = "".join(_CONS[int(rng.integers(len(_CONS)))] + _VOW[int(rng.integers(len(_VOW)))]
                    for _ in range(k))
        if rng.random() < 0.4:
            w += _CONS[int(rng.integers(len(_CONS)))]
        if w in seen:
            continue
        seen.add(w)
        out.append(w.capitalize() if cap else w)
    return out


def _zipf_choice(rng, n_items, s, size):
    w = 1.0 / np.arange(1, n_items + 1, dtype=np.float64) ** s
    w /= w.sum()
    return rng.choice(n_items, size=size, p=w)


def _corrupt(rng, s):
    """1-2 random edits over a-z."""
    for _ in range(int(rng.integers(1, 3))):
        op = int(rng.integers(4))
        ch = chr(ord("a") + int(rng.integers(26)))
        if not s:
            s = ch
            continue
        i = int(rng.integers(len(s)))
        if op == 0:
            s = s[:i] + ch + s[i + 1:]
        elif op == 1:
            s = s[:i] + ch + s[i:]
        elif op == 2 and len(s) > 1:
            s = s[:i] + s[i + 1:]
        elif op == 3 and len(s) > 1:
            j = min(i + 1, len(s) - 1)
            i = j - 1
            s = s[:i] + s[j] + s[i] + s[j + 1:]
    return s


def persons(n_orig, n_dup, seed=SEED, utf16_frac=0.0, shuffle=True):
    """Returns dict with lists given/surname/name/address/dob and `orig` (index of the
    original each record duplicates, -1 for originals)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    given_v = _vocab(rng, 5000, 1, 3)
    sur_v = _vocab(rng, 20000, 2, 3)
    street_v = _vocab(rng, 3000, 2, 3)
    city_v = _vocab(rng, 1000, 2, 3)
    if utf16_frac > 0:
        # a slice of non-Latin-1 names, one with a surrogate pair (UTF-16 parity cases)
        k = max(1, int(len(given_v) * utf16_frac))
        for i in range(k):
            given_v[-1 - i] = given_v[-1 - i][:-1] + ("ł" if i % 3 else "\U0001F600")
    gi = _zipf_choice(rng, len(given_v), 1.1, n_orig)
    si = _zipf_choice(rng, len(sur_v), 1.07, n_orig)
    num = rng.integers(1, 1000, n_orig)
    sti = rng.integers(0, len(street_v), n_orig)
    suf = rng.integers(0, len(_SUFFIX), n_orig)
    ci = rng.integers(0, len(city_v), n_orig)
    d0 = _dt.date(1930, 1, 1).toordinal()
    d1 = _dt.date(2010, 12, 31).toordinal()
    dob_ord = rng.integers(d0, d1 + 1, n_orig)

    given = [given_v[i] for i in gi]
    surname = [sur_v[i] for i in si]
    address = [f"{n} {street_v[s]} {_SUFFIX[x]} {city_v[c]}" for n, s, x, c in zip(num, sti, suf, ci)]
    dob = [_dt.date.fromordinal(int(o)).isoformat() for o in dob_ord]
    orig = [-1] * n_orig

    src = rng.integers(0, n_orig, n_dup)
    for j in range(n_dup):
        i = int(src[j])
        g, s, a, d = given[i], surname[i], address[i], dob[i]
        if rng.random() < 0.3:
            g = _corrupt(rng, g)
        if rng.random() < 0.3:
            s = _corrupt(rng, s)
        if rng.random() < 0.3:
            a = _corrupt(rng, a)
        if rng.random() < 0.1:
            d = f"{d[:4]}-{d[8:10]}-{d[5:7]}"
        given.append(g)
        surname.append(s)
        address.append(a)
        dob.append(d)
        orig.append(i)
    n = n_orig + n_dup
    perm = rng.permutation(n) if shuffle else np.arange(n)
    pick = lambda xs: [xs[i] for i in perm]
    out = {"given": pick(given), "surname": pick(surname), "address": pick(address),
           "dob": pick(dob)}
    inv = np.empty(n, dtype=np.int64)
    inv[perm] = np.arange(n)
    o = np.asarray(orig)[perm]
    out["orig"] = np.where(o >= 0, inv[np.maximum(o, 0)], -1)
    out["name"] = [f"{g} {s}" for g, s in zip(out["given"], out["surname"])]
    return out


def linkage_persons(n_group1, dup_frac=0.3, seed=SEED + 2):
    """BASELINE config 3: group 1 = n_group1 persons; group 2 = n_group1 persons of which
    dup_frac are perturbed copies of group-1 records, the rest new.  Adds BIRTHYEAR
    (dob[0:4]) and ZIP (4 digits fixed per city) for the Numeric comparators.  Returns
    the persons dict (group-1 rows first) and the group array (1 / 2)."""
    n_dup = int(n_group1 * dup_frac)
    n_new = n_group1 - n_dup
    p = persons(n_group1 + n_new, 0, seed=seed, shuffle=False)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    src = rng.integers(0, n_group1, n_dup)
    fields = ("given", "surname", "address", "dob")
    out = {k: list(p[k][:n_group1]) for k in fields}
    extra = {k: list(p[k][n_group1:]) for k in fields}
    dup = {k: [] for k in fields}
    for j in range(n_dup):
        i = int(src[j])
        g, su, a, d = out["given"][i], out["surname"][i], out["address"][i], out["dob"][i]
        if rng.random() < 0.3:
            g = _corrupt(rng, g)
        if rng.random() < 0.3:
            su = _corrupt(rng, su)
        if rng.random() < 0.3:
            a = _corrupt(rng, a)
        if rng.random() < 0.1:
            d = f"{d[:4]}-{d[8:10]}-{d[5:7]}"
        for k, v in zip(fields, (g, su, a, d)):
            dup[k].append(v)
    for k in fields:
        out[k] = out[k] + dup[k] + extra[k]
    n = len(out["given"])
    out["name"] = [f"{g} {s}" for g, s in zip(out["given"], out["surname"])]
    out["birthyear"] = [d[:4] for d in out["dob"]]
    out["zip"] = [str(1000 + hash_str(a.rsplit(" ", 1)[-1]) % 9000) for a in out["address"]]
    group = np.concatenate([np.ones(n_group1, np.uint8), np.full(n - n_group1, 2, np.uint8)])
    return out, group


def _word_matrix(words):
    """(uint8 [len(words), W] zero padded, lengths) of Latin-1 words."""
    enc = [w.encode("latin-1") for w in words]
    L = np.fromiter(map(len, enc), dtype=np.int64, count=len(enc))
    M = np.zeros((len(enc), int(L.max())), np.uint8)
    for i, b in enumerate(enc):
        M[i, :len(b)] = np.frombuffer(b, np.uint8)
    return M, L


def _digits(v, width):
    """[n, width] ASCII digits of v (zero padded on the left)."""
    out = np.empty((len(v), width), np.uint8)
    for j in range(width):
        out[:, width - 1 - j] = 48 + (v // 10 ** j) % 10
    return out


def _pack(parts, n):
    """Column of the concatenation, per record, of `parts`: each (uint8 [n, W], lengths[n])
    or a bytes literal.  The parts side by side, then one row-major compress of the bytes
    inside each part's length."""
    Ms, Vs = [], []
    lens = np.zeros(n, np.int64)
    for p in parts:
        if isinstance(p, bytes):
            Ms.append(np.broadcast_to(np.frombuffer(p, np.uint8), (n, len(p))))
            Vs.append(np.ones((n, len(p)), bool))
            lens += len(p)
        else:
            M, L = p
            Ms.append(M)
            Vs.append(np.arange(M.shape[1])[None, :] < L[:, None])
            lens += L
    units = np.concatenate(Ms, axis=1)[np.concatenate(Vs, axis=1)]
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    return Column(offs, units)


def linkage_columns(n_group1, dup_frac=0.3, seed=SEED + 5, copies=1, long_every=0):
    """configs[2]-shaped linkage data at full size, built column-wise with numpy (no
    per-record Python): group 1 = n_group1 persons, group 2 = n_group1 persons of which
    dup_frac copy a group-1 record with, per field, p=0.3 of one a-z substitution (dob: p=0.1
    of a day<->month swap).  NAME = "given surname", ADDRESS = "num street suffix district
    city", BIRTHYEAR = dob's year, ZIP = 4 digits fixed per city; key columns K1 =
    surname[0:3] + year, K2 = given[0:2] + dob[5:10] (keys_config2) and their integer codes
    (k1 / k2: equal codes <=> equal key strings).
    copies > 1: n_group1 / copies persons per group, the whole set repeated `copies` times
    with the year moved by 100 per copy (K1 and BIRTHYEAR differ between copies, K2 does not:
    cross-copy candidates) -- full-size replicas at memcpy speed.  long_every > 0: every such
    record's ADDRESS gets two more words, cut at 65 units (sets of up to 64 bigrams: the
    longest key-word rows a replica holds).  Records: copy 0's group 1, its group 2, copy 1's
    group 1, ...  Returns (columns dict, key columns, group, k1, k2)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    given_v, sur_v = _word_matrix(_vocab(rng, 5000, 1, 3)), _word_matrix(_vocab(rng, 20000, 2, 3))
    street_v, city_v = _word_matrix(_vocab(rng, 3000, 2, 3)), _word_matrix(_vocab(rng, 1000, 2, 3))
    dist_v = _word_matrix(_vocab(rng, 2000, 2, 3))
    suf_v = _word_matrix(_SUFFIX)
    n1 = n_group1 // copies
    n_dup = int(n1 * dup_frac)
    n_src = 2 * n1 - n_dup                      # distinct persons drawn
    n = 2 * n1
    # group 1 rows, then the copies, then the new group-2 persons
    src = np.concatenate([np.arange(n1), rng.integers(0, n1, n_dup), np.arange(n1, n_src)])
    gi = _zipf_choice(rng, len(given_v[1]), 1.1, n_src)[src]
    si = _zipf_choice(rng, len(sur_v[1]), 1.07, n_src)[src]
    num = rng.integers(1, 1000, n_src)[src]
    sti = rng.integers(0, len(street_v[1]), n_src)[src]
    sfi = rng.integers(0, len(_SUFFIX), n_src)[src]
    di = rng.integers(0, len(dist_v[1]), n_src)[src]
    ci = rng.integers(0, len(city_v[1]), n_src)[src]
    day = (np.datetime64("1930-01-01") + rng.integers(0, 29584, n_src).astype("timedelta64[D]"))[src]
    year = day.astype("datetime64[Y]").astype(np.int64) + 1970
    month = (day.astype("datetime64[M]") - day.astype("datetime64[Y]")).astype(np.int64) + 1
    dom = (day - day.astype("datetime64[M]")).astype(np.int64) + 1
    dup = np.zeros(n, bool)
    dup[n1:n1 + n_dup] = True

    def field(V, idx):
        M, L = V[0][idx], V[1][idx].copy()
        hit = np.nonzero(dup & (rng.random(n) < 0.3))[0]   # one substitution, a-z
        at = (rng.random(len(hit)) * L[hit]).astype(np.int64)
        M[hit, at] = rng.integers(ord("a"), ord("z") + 1, len(hit), dtype=np.uint8)
        return M, L

    given, sur = field(given_v, gi), field(sur_v, si)
    street = field(street_v, sti)
    swap = dup & (rng.random(n) < 0.1) & (dom <= 12)
    mm = np.where(swap, dom, month)
    dd = np.where(swap, month, dom)
    nd = 1 + (num >= 10) + (num >= 100)
    numd = _digits(num, 3)
    numd = np.where((np.arange(3)[None, :] < nd[:, None]), np.take_along_axis(
        numd, (np.arange(3)[None, :] + (3 - nd)[:, None]) % 3, axis=1), 0).astype(np.uint8)
    dist = (dist_v[0][di], dist_v[1][di].copy())
    if long_every:
        lr = np.arange(0, n, long_every)
        extra = _pack([b" ", (dist_v[0][(di[lr] + 7) % len(dist_v[1])], dist_v[1][(di[lr] + 7) % len(dist_v[1])]),
                       b" ", (city_v[0][(ci[lr] + 3) % len(city_v[1])], city_v[1][(ci[lr] + 3) % len(city_v[1])]),
                       b" ", (street_v[0][(sti[lr] + 5) % len(street_v[1])], street_v[1][(sti[lr] + 5) % len(street_v[1])])],
                      len(lr))
        w = int(np.diff(extra.offsets.astype(np.int64)).max())
        X = np.zeros((len(lr), w), np.uint8)
        eo = extra.offsets.astype(np.int64)
        el = np.diff(eo)
        for j in range(w):
            sel = np.nonzero(j < el)[0]
            X[sel, j] = extra.units[eo[sel] + j]
        D = np.zeros((n, dist[0].shape[1] + w), np.uint8)
        D[:, :dist[0].shape[1]] = dist[0]
        for r, i in enumerate(lr):
            D[i, dist[1][i]:dist[1][i] + el[r]] = X[r, :el[r]]
        DL = dist[1].copy()
        DL[lr] += el
        dist = (D, DL)
    addr = _pack([(numd, nd), b" ", street, b" ", (suf_v[0][sfi], suf_v[1][sfi]), b" ", dist, b" ",
                  (city_v[0][ci], city_v[1][ci])], n)
    if long_every:  # cut at 65 units
        ao = addr.offsets.astype(np.int64)
        al = np.minimum(np.diff(ao), 65)
        keep = np.repeat(np.arange(n), al) if n else np.zeros(0, np.int64)
        pos = np.arange(int(al.sum())) - np.repeat(np.cumsum(al) - al, al)
        units = addr.units[ao[keep] + pos]
        no = np.zeros(n + 1, np.int64)
        np.cumsum(al, out=no[1:])
        addr = Column(no, units)
    cols = {"NAME": _pack([given, b" ", sur], n), "ADDRESS": addr,
            "ZIP": _pack([(_digits(1000 + (ci * 2654435761) % 9000, 4), np.full(n, 4))], n)}
    dob5 = np.concatenate([_digits(mm, 2), np.full((n, 1), ord("-"), np.uint8), _digits(dd, 2)], axis=1)
    s3 = sur[0][:, :3]
    g2 = given[0][:, :2]

    def tile(c):  # the column `copies` times
        o = c.offsets.astype(np.int64)
        return Column(np.concatenate([o[:-1] + k * o[-1] for k in range(copies)] + [[copies * o[-1]]]),
                      np.tile(c.units, copies))

    ys = [year + 100 * k for k in range(copies)]
    yd = np.concatenate([_digits(y, 4) for y in ys])
    N = n * copies
    out = {k: tile(c) for k, c in cols.items()}
    out["BIRTHYEAR"] = _pack([(yd, np.full(N, 4))], N)
    kcols = [_pack([(np.tile(s3, (copies, 1)), np.full(N, 3)), (yd, np.full(N, 4))], N),
             tile(_pack([(g2, np.full(n, 2)), (dob5, np.full(n, 5))], n))]
    s3i = s3.astype(np.int64)
    g2i = g2.astype(np.int64)
    k1 = np.concatenate([((s3i[:, 0] << 16 | s3i[:, 1] << 8 | s3i[:, 2]) << 16) | y for y in ys])
    k2 = np.tile(((g2i[:, 0] << 8 | g2i[:, 1]) << 16) | (mm * 100 + dd), copies)
    group = np.tile(np.concatenate([np.ones(n1, np.uint8), np.full(n - n1, 2, np.uint8)]), copies)
    return out, kcols, group, k1, k2


def hash_str(s):
    """Deterministic string hash (FNV-1a 32), stable across processes."""
    h = 0x811C9DC5
    for ch in s.encode("utf-8"):
        h = ((h ^ ch) * 0x01000193) & 0xFFFFFFFF
    return h


def short_strings(n, lo=4, hi=16, seed=SEED + 3):
    """BASELINE config 4: n strings over a-z with lengths U[lo, hi]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = rng.integers(lo, hi + 1, n)
    chars = rng.integers(ord("a"), ord("z") + 1, int(lens.sum()), dtype=np.uint8).tobytes()
    out, o = [], 0
    for L in lens:
        out.append(chars[o:o + int(L)].decode("latin-1"))
        o += int(L)
    return out


def long_texts(n_group1, dup_frac=0.3, lo=64, hi=256, vocab=50000, seed=SEED + 4):
    """BASELINE config 5: TEXT values of lo..hi characters (lognormal length, clipped) from
    a `vocab`-word list (Zipf s=1.05); group 2 holds dup_frac copies of group-1 texts with
    1-8 character edits, and new texts for the rest.  Returns (texts, group)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    words = _vocab(rng, vocab, 1, 4, cap=False)
    n_dup = int(n_group1 * dup_frac)
    total = 2 * n_group1 - n_dup
    target = np.clip(rng.lognormal(np.log(120.0), 0.35, total), lo, hi).astype(np.int64)
    w = _zipf_choice(rng, len(words), 1.05, int(target.sum() // 3 + 64 * total))
    texts, k = [], 0
    for t in target:
        parts, L = [], -1
        while L < t:
            wd = words[int(w[k])]
            k += 1
            parts.append(wd)
            L += len(wd) + 1
        texts.append(" ".join(parts)[:hi])
    g1 = texts[:n_group1]
    src = rng.integers(0, n_group1, n_dup)
    dups = []
    for j in range(n_dup):
        s = g1[int(src[j])]
        for _ in range(int(rng.integers(1, 9))):
            s = _corrupt(rng, s)
        dups.append(s[:hi])
    out = g1 + dups + texts[n_group1:]
    group = np.concatenate([np.ones(n_group1, np.uint8), np.full(len(out) - n_group1, 2, np.uint8)])
    return out, group


def stress_entities(n, seed):
    """configs[0]'s input: entities shaped like the reference's stress test
    (sesam_node_deduplication_stresstest_config.conf.json:18-71 -- country = a first name,
    capital = a last name, area in 1..10, ids from a 1..1,000,000 pool, so IDs recur), every
    97th one `_deleted`.  JSON-like dicts for records_from_entities / dk_pack_json."""
    from .records import JsonNumber
    rng = np.random.Generator(np.random.PCG64(seed))
    first = _vocab(rng, 3000, 1, 3)
    last = _vocab(rng, 8000, 2, 3)
    fi = _zipf_choice(rng, len(first), 1.1, n)
    li = _zipf_choice(rng, len(last), 1.07, n)
    ids = rng.integers(1, 1_000_001, n)
    area = rng.integers(1, 11, n)
    ents = []
    for i in range(n):
        e = {"_id": str(int(ids[i])), "country": first[fi[i]], "capital": last[li[i]],
             "area": JsonNumber(str(int(area[i]))), "id": str(int(ids[i]))}
        if i % 97 == 5:
            e["_deleted"] = True
        ents.append(e)
    return ents


def keys_first_two_tokens(texts):
    """BASELINE config 5 key: the first two tokens."""
    return [[" ".join(t.split(" ")[:2]) for t in texts]]


def keys_config2(p):
    """K1 = surname[0:3] + dob[0:4]; K2 = given[0:2] + dob[5:10]."""
    k1 = [s[:3] + d[:4] for s, d in zip(p["surname"], p["dob"])]
    k2 = [g[:2] + d[5:10] for g, d in zip(p["given"], p["dob"])]
    return [k1, k2]


def ascii_column(values):
    """Fast packing of a list of str (Latin-1 only) into a width-1 Column."""
    enc = [v.encode("latin-1") for v in values]
    lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    units = np.frombuffer(b"".join(enc), dtype=np.uint8) if offs[-1] else np.zeros(1, np.uint8)
    return Column(offs, units)


def column(values):
    return Column.from_strings(values)
