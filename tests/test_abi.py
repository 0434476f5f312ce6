"""CPU: libdukehip.so loads, exports every entry point include/dukehip.h declares, and the
ctypes mirror of every struct matches the C layout (checked with a gcc-compiled probe).
No compute calls: this container has no GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

from dukehip import _abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dukehip.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(dk_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_api():
    fns = declared_functions()
    assert set(A.EXPORTS) == set(fns), fns


def test_library_exports_every_symbol():
    lib = A.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", A.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}$", out, re.M), f"{name} not exported with C linkage"


def test_abi_version_and_error_text():
    lib = A.load()
    assert lib.dk_abi_version() == A.ABI_VERSION == 9
    assert isinstance(lib.dk_last_error(), bytes)


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "dukehip.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
#define S(T) printf(#T " %zu\n", sizeof(T));
int main(void) {
  S(dk_property) F(dk_property, comparator) F(dk_property, qgram_q) F(dk_property, qgram_formula)
  F(dk_property, qgram_tokenizer) F(dk_property, low) F(dk_property, high) F(dk_property, min_ratio)
  S(dk_schema) F(dk_schema, nprops) F(dk_schema, props) F(dk_schema, threshold)
  F(dk_schema, maybe_threshold) F(dk_schema, mode) F(dk_schema, nkeys)
  S(dk_column) F(dk_column, offsets) F(dk_column, units) F(dk_column, width) F(dk_column, present)
  S(dk_batch) F(dk_batch, n) F(dk_batch, ident) F(dk_batch, group) F(dk_batch, deleted)
  F(dk_batch, columns) F(dk_batch, keys) F(dk_batch, key_columns)
  S(dk_result) F(dk_result, nqueries) F(dk_result, first) F(dk_result, n)
  F(dk_result, candidate) F(dk_result, prob) F(dk_result, kind) F(dk_result, pairs_scored)
  F(dk_result, pairs_generated)
  S(dk_profile) F(dk_profile, ms_index) F(dk_profile, ms_generate) F(dk_profile, ms_score)
  F(dk_profile, ms_gather) F(dk_profile, ms_total) F(dk_profile, score_launches)
  F(dk_profile, pairs_scored) F(dk_profile, pairs_generated) F(dk_profile, score_bytes)
  F(dk_profile, ms_copy) F(dk_profile, ms_emit) F(dk_profile, sym_matches)
  F(dk_profile, full_builds) F(dk_profile, delta_builds) F(dk_profile, replica_positions)
  F(dk_profile, gram_row_bytes) F(dk_profile, sym2_matches) F(dk_profile, pairs_exact)
  S(dk_region_layout) F(dk_region_layout, capacity) F(dk_region_layout, first_offset)
  F(dk_region_layout, prob_offset) F(dk_region_layout, candidate_offset)
  F(dk_region_layout, kind_offset)
  return 0;
}
"""


def test_struct_layout_matches_ctypes(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    for line in filter(None, lines):
        key, val = line.rsplit(" ", 1)
        if "." in key:
            t, f = key.split(".")
            assert getattr(getattr(A, t), f).offset == int(val), key
        else:
            assert C.sizeof(getattr(A, key)) == int(val), key


def test_create_without_gpu_fails_loudly():
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is visible")
    except Exception:
        pass
    from dukehip.processor import GpuEngine
    arr = (A.dk_property * 1)(A.dk_property(A.CMP_LEVENSHTEIN, 2, 0, 0, 0.1, 0.9, 0.0))
    s = A.dk_schema(1, arr, 0.9, 0.0, A.MODE_DEDUP, 1)
    with pytest.raises(A.DukeHipError) as e:
        GpuEngine(s)
    assert e.value.code == A.DK_E_DEVICE


def test_schema_validation_rejects_unsupported():
    lib = A.load()
    ctx = C.c_void_p()
    arr = (A.dk_property * 1)(A.dk_property(99, 2, 0, 0, 0.1, 0.9, 0.0))
    s = A.dk_schema(1, arr, 0.9, 0.0, A.MODE_DEDUP, 1)
    assert lib.dk_create(C.byref(s), 0, C.byref(ctx)) == A.DK_E_UNSUPPORTED
    assert b"no GPU kernel" in lib.dk_last_error()
    s = A.dk_schema(1, arr, 0.9, 0.0, A.MODE_DEDUP, 0)
    assert lib.dk_create(C.byref(s), 0, C.byref(ctx)) == A.DK_E_INVALID


def test_result_region_layout():
    """dk_result_region_layout (host-only arithmetic): the four arrays are disjoint, aligned
    and inside the region; region_views reads them back."""
    import numpy as np
    lay = A.region_layout(A.region_bytes(10, 100), 10)
    assert lay["capacity"] == 100 and lay["first_offset"] == 0 and lay["prob_offset"] == 88
    assert lay["candidate_offset"] == 88 + 800 and lay["kind_offset"] == 88 + 1200
    assert lay["prob_offset"] % 8 == 0 and lay["candidate_offset"] % 4 == 0
    buf = bytearray(A.region_bytes(10, 100) + 5)
    v = A.region_views(buf, 10, 3, 7)
    v["first"][:] = [0, 2, 2, 7]
    v["candidate"][:] = np.arange(7)
    v["prob"][:] = 0.5
    v["kind"][:] = 1
    w = A.region_views(buf, 10, 3, 7)
    assert list(w["first"]) == [0, 2, 2, 7] and w["prob"].sum() == 3.5 and w["kind"].sum() == 7
    with pytest.raises(A.DukeHipError):
        A.region_layout(8, 10)
