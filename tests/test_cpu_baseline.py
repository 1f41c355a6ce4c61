"""The CPU baseline engine (bench.py cpu_baseline): the oracle with every regex signature behind
its required-literal prefilter.  Its answers must equal the exhaustive checker's -- the factor
extraction is conservative -- and it must run the PCRE calls only where a factor occurs."""

import numpy as np

from gpumatch import records, sigs, workloads
from oracle_py import Oracle, regex_factor


def test_factor_extraction():
    assert regex_factor(r"union\s+(all\s+)?select") == b"select"
    assert regex_factor(r"abc+de") == b"abc"
    assert regex_factor(r"ab?cdef") == b"cdef"
    assert regex_factor(r"x{0,3}hello{2}") == b"hello"
    assert regex_factor(r"Etc/Pass(wd)?") == b"etc/pass"
    assert regex_factor(r"a|bcdef") == b""
    assert regex_factor(r"(?i)abcdef") == b""
    assert regex_factor(r"(z10ip3|suguep|30nrx3z)[a-z0-9]+--") == b"z10ip3|suguep|30nrx3z"
    assert regex_factor(r"(?:7viaa92q|0n2mczp)=[0-9a-f]{8,}") == b"7viaa92q|0n2mczp"
    assert regex_factor(r"(ab|cdef)?xyz") == b"xyz"
    assert regex_factor(r"(abc|d)xy") == b""
    assert regex_factor(r"[abc]def\.ghi") == b"def.ghi"
    assert regex_factor(r"\d{3}x") == b""
    assert regex_factor(r"foo.bar") == b"foo"


def test_prefiltered_equals_exhaustive():
    ss = workloads.c4_sigset()
    extra = [sigs.Rule("re", True, "uahb", r"sel(ect)?\s+[a-z]+_from"), sigs.Rule("re", False, "ab", r"a+b+c+d"),
             sigs.Rule("re", False, "uahb", r"[0-9]{3}x"), sigs.Rule("re", True, "ab", r"x\.y+z{2,}q")]
    ss = sigs.SigSet(ss.rules + extra)
    b = workloads.c4_blob(ss)
    reqs, arena = records.gen_c4(4000, ss, seed=records.SEED_BASE + 77, plant_rate=0.2)
    v0, h0 = Oracle(b, 1).match(reqs, arena, nthreads=8)
    v1, h1 = Oracle(b, 1, prefilter=True).match(reqs, arena, nthreads=8)
    assert v0.tobytes() == v1.tobytes() and np.array_equal(h0, h1)
    assert int((v0["n_hits"] > 0).sum()) > 500
