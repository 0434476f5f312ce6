"""CPU: the whole-column string packer (one join + one encode) against the per-value packer,
on Latin-1, BMP, astral-plane and lone-surrogate values, missing and empty values."""
import random

import numpy as np
import pytest

from dukehip import _abi as A

ALPHABETS = {
    "ascii": "abcdefgh 0123",
    "latin1": "abcéÿæ 1",
    "bmp": "ab中éЖ ",
    "astral": "ab\U0001F600中\U00010348e",
    "surrogate": "ab𐏿c",
}


def rand_values(rng, alpha, n, none_frac=0.1, empty_frac=0.05):
    out = []
    for _ in range(n):
        r = rng.random()
        if r < none_frac:
            out.append(None)
        elif r < none_frac + empty_frac:
            out.append("")
        else:
            out.append("".join(rng.choice(alpha) for _ in range(rng.randint(1, 12))))
    return out


@pytest.mark.parametrize("alpha", sorted(ALPHABETS))
@pytest.mark.parametrize("none_frac", [0.0, 0.2])
def test_from_strings_matches_per_value(alpha, none_frac):
    rng = random.Random(hash((alpha, none_frac)) & 0xFFFF)
    vals = rand_values(rng, ALPHABETS[alpha], 500, none_frac=none_frac)
    a, b = A.Column.from_strings(vals), A.Column.from_strings_per_value(vals)
    assert a.units.dtype == b.units.dtype
    assert np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.units[: int(a.offsets[-1])], b.units[: int(b.offsets[-1])])
    assert (a.present is None) == (b.present is None)
    if a.present is not None:
        assert np.array_equal(a.present, b.present)


def test_from_strings_edge_cases():
    for vals in ([], [None], [""], ["", None, ""], ["\U0001F600"]):
        a, b = A.Column.from_strings(vals), A.Column.from_strings_per_value(vals)
        assert np.array_equal(a.offsets, b.offsets) and a.units.dtype == b.units.dtype
