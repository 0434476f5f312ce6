"""CPU: the machinery of tests/test_gpu_fullsize.py at a small size -- the column-wise
configs[2] generator (synth.linkage_columns) and the oracle run on the rows sharing a key
with the queries give the same list as the oracle on every row."""
import numpy as np

import oracle as O
from dukehip import synth
from test_gpu_fullsize import NAMES, PROPS, _subset


def test_linkage_columns_shape():
    cols, kcols, group, k1, k2 = synth.linkage_columns(3000, copies=3, long_every=50)
    n = len(group)
    assert n == 6000 and all(len(c.offsets) == n + 1 for c in list(cols.values()) + kcols)
    assert (np.bincount(group) == [0, 3000, 3000]).all()
    o = cols["ADDRESS"].offsets.astype(np.int64)
    assert np.diff(o).max() == 65
    # equal key codes <=> equal key strings
    ks = [bytes(kcols[0].units[kcols[0].offsets[i]:kcols[0].offsets[i + 1]]) for i in range(n)]
    assert len(set(ks)) == len(np.unique(k1))
    by = [bytes(cols["BIRTHYEAR"].units[4 * i:4 * i + 4]) for i in (0, 2000, 4000)]
    assert int(by[1]) - int(by[0]) == 100 and int(by[2]) - int(by[1]) == 100   # year per copy


def test_subset_oracle_equals_full_oracle():
    cols, kcols, group, k1, k2 = synth.linkage_columns(4000, copies=2, long_every=40)
    n = len(group)
    allrows = np.arange(n)
    full = O.OracleTable.from_packed(PROPS, [_subset(cols[k], allrows) for k in NAMES],
                                     [_subset(c, allrows) for c in kcols],
                                     ident=np.arange(n, dtype=np.uint64), group=group,
                                     threshold=0.9, maybe=0.7, mode="linkage")
    q = np.sort(np.random.default_rng(1).choice(np.nonzero(group == 2)[0], 300, replace=False))
    want = full.match(q.astype(np.uint32), nthreads=4)
    rows = np.union1d(q, np.nonzero(np.isin(k1, k1[q]) | np.isin(k2, k2[q]))[0])
    sub = O.OracleTable.from_packed(PROPS, [_subset(cols[k], rows) for k in NAMES],
                                    [_subset(c, rows) for c in kcols], ident=rows.astype(np.uint64),
                                    group=group[rows], threshold=0.9, maybe=0.7, mode="linkage")
    got = sub.match(np.searchsorted(rows, q).astype(np.uint32), nthreads=4)
    assert got["pairs_scored"] == want["pairs_scored"] > 300
    assert np.array_equal(rows[got["query"]], want["query"])
    assert np.array_equal(rows[got["candidate"]], want["candidate"])
    assert np.array_equal(got["prob"], want["prob"]) and np.array_equal(got["kind"], want["kind"])
    assert len(want["query"]) > 10
