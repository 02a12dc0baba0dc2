"""CPU lint of the HIP kernels: no short-circuit lexicographic compares.

The gfx950 backend (ROCm 7.2) miscompiled `a < A || (a == A && (...))` followed by
several assignments when a key was wave-uniform: tie-winning lanes kept stale
fields (MEASUREMENTS.md; reproducer tests/native/lexrepro.hip,
tests/test_gpu_lexrepro.py).  Every lexicographic compare in the kernels is written
branch-free (lex_less3 / lex_less2: bitwise & / | on bools, then selects); this test
keeps the short-circuit form from coming back."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# x < X || (x == X && ...   (any whitespace, identifiers / member / index expressions)
EXPR = r"[\w\.\[\]]+"
PATTERN = re.compile(rf"({EXPR})\s*<\s*({EXPR})\s*\|\|\s*\(\s*\1\s*==\s*\2\s*&&")


def kernel_sources():
    srcs = sorted(glob.glob(os.path.join(ROOT, "shadow_amd", "csrc", "spe", "kernels_*.inc")))
    srcs.append(os.path.join(ROOT, "shadow_amd", "csrc", "spe.hip"))
    return srcs


def test_no_short_circuit_lexicographic_compares():
    bad = []
    for p in kernel_sources():
        for i, line in enumerate(open(p), 1):
            code = line.split("//", 1)[0]
            if PATTERN.search(code):
                bad.append(f"{os.path.relpath(p, ROOT)}:{i}: {line.strip()}")
    assert not bad, "short-circuit lexicographic compares (write them branch-free, lex_less3):\n" + "\n".join(bad)


def test_lint_pattern_catches_the_form():
    assert PATTERN.search("if (alt < ba || (alt == ba && (du < bdu || (du == bdu && u < bu)))) {")
    assert PATTERN.search("(du < bdu || (du == bdu && u < bu))")
    assert not PATTERN.search("const bool b = (alt < ba) | ((alt == ba) & (du < bdu));")
