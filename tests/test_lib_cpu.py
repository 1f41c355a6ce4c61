"""libgpumatch.so on the CPU: it loads, exports every symbol include/*.h declares, and its
generation compiler (host code) behaves -- no classification calls without a GPU."""

import ctypes
import os
import re
import sys

import numpy as np
import pytest

from gpumatch import engine, sigs, workloads
from oracle_py import pcre_match

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    return set(re.findall(r"^\s*[\w\s\*]+?\b(gm_\w+)\s*\(", txt, flags=re.M))


def test_exports_every_declared_symbol():
    L = ctypes.CDLL(engine.LIB_PATH)
    syms = _declared("gpumatch.h") | _declared("gpumatch_debug.h")
    assert set(engine.EXPORTS) <= syms
    for s in sorted(syms):
        assert hasattr(L, s), s
    assert L.gm_abi_version() == engine.GM_ABI_VERSION


@pytest.fixture(scope="module")
def eng():
    return engine.Engine(compile_only=True)


def test_compile_cafe(eng):
    eng.load(workloads.c1_blob(), 7)
    s = eng.stats()
    # the default server, the stub_status server (nginx.tmpl:104-115, on by default), cafe's two
    assert s["gen"] == 7 and s["n_servers"] == 4 and s["n_locations"] == 5 and s["n_upstreams"] == 2
    assert s["n_rejected_other"] == 0 and s["n_rejected_pcre"] == 0


def test_compile_vs_routes(eng):
    eng.load(workloads.c2_blob(), 1)
    s = eng.stats()
    assert s["n_routes_rules"] == 3 and s["n_routes_split"] == 1 and s["n_rejected_other"] == 0


def test_bad_blob_keeps_previous_generation(eng):
    eng.load(workloads.c1_blob(), 11)
    with pytest.raises(engine.GmError):
        eng.load(b"GMB1garbage", 12)
    assert eng.stats()["gen"] == 11
    from gpumatch import blob
    with pytest.raises(engine.GmError):
        eng.load(blob.make_blob("http { server { listen 80; ", {}), 13)
    assert eng.stats()["gen"] == 11


def test_pcre_only_rules_rejected_and_counted(eng):
    rules = [sigs.Rule("re", False, "u", p) for p in
             [r"(a)\1", r"foo(?=bar)", r"(?<!x)abcd", r"a++b", r"(?>abc)", r"ab\Kcd", r"abcd"]]
    rules.append(sigs.Rule("lit", True, "u", b"abcdef"))
    b = workloads.c4_blob(sigs.SigSet(rules))
    eng.load(b, 2)
    s = eng.stats()
    assert s["n_rejected_pcre"] == 6
    assert s["n_sig_regex"] == 1 and s["n_sig_literals"] == 1 and s["n_sigs"] == 8


REGEX_CASES = [
    (r"union\s+select", False), (r"^/api/v[0-9]+/", False), (r"\.php$", False), (r"(?i)select.{0,8}from", False),
    (r"<script[^>]{0,16}on[a-z]{2,8}\s*=", True), (r"(abc|abd|xyz)[a-z0-9]+--", False), (r"a$", False),
    (r"^$", False), (r"x*", False), (r"[^a-c]+z", True), (r"\d{3}-\d{2}", False), (r"(?s)a.b", False),
    (r"colou?r", True), (r"a|^b|c$", False), (r"[\w.-]+@[\w-]+\.com", False), (r"\x41\x42", False),
    (r"a{2,}b{0,1}c{3}", False), (r"[]a]", False), (r"[a\-z]", False), (r"a\.b\*c", False),
]


def test_regex_dfa_matches_pcre_on_random_subjects():
    """The engine's DFA compiler agrees with PCRE 8.39 (the library nginx links)."""
    L = ctypes.CDLL(engine.LIB_PATH)
    L.gm_debug_regex.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    rng = np.random.default_rng(3)
    alpha = np.frombuffer(b"abcxyzABCz019-_.@ \t\n\x0b<>=/uniosetlcfrmphSELECTFROM*", dtype=np.uint8)
    seeds = [b"union  select", b"/api/v2/x", b"a.php", b"SELECT x FROM", b"<script a=1 onload =", b"abd9--",
             b"a\n", b"", b"zz", b"color", b"123-45", b"a\nb", b"b", b"ab@c-d.com", b"AB", b"aabccc",
             b"]", b"-", b"a.b*c"]
    for pat, ci in REGEX_CASES:
        subjects = list(seeds)
        for _ in range(300):
            k = int(rng.integers(0, 24))
            subjects.append(bytes(alpha[rng.integers(0, len(alpha), k)]))
        for s in subjects:
            got = L.gm_debug_regex(pat.encode(), 1 if ci else 0, s, len(s))
            assert got >= 0, (pat, got)
            assert got == pcre_match(pat, s, ci), (pat, ci, s)


def test_reversed_regex_matches_pcre():
    """X$ regex locations run backwards from the URI's end as ^(\\n)?rev(X) (gm_regex.hpp
    compile_regex_reversed): same answer as PCRE's forward search, the final-newline rule of '$'
    included; forms other than X$ are refused."""
    import random
    L = ctypes.CDLL(engine.LIB_PATH)
    L.gm_debug_regex_rev.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    extra = [("abc$", False), ("(a|bc)d*$", False), ("x[0-9]{2,3}$", True), ("a?$", False),
             (r"\.(php|html?)$", True), ("(foo|bar)+baz$", False), ("a.b$", False), ("[^/]+$", False)]
    for pat in ("^/a$", "abc", "a$|b", "(a$)b", "$"):
        assert L.gm_debug_regex_rev(pat.encode(), 0, b"x", 1) == -1, pat
    regs = workloads.c3_regexes()
    cases = extra + [(r[0], r[1]) for r in regs if not r[2] and not r[4] and r[5]]
    rng = random.Random(5)
    seeds = [b"", b"\n", b"abc\n", b"xabc", b"a\nb", b"ab\n\n", b"x12\n", b"foobaz", b"/v1/x.PHP", b"a.b\n"]
    n_hit = 0
    for pat, ci in cases:
        own = [r for r in regs if r[0] == pat]
        subjects = list(seeds) + [workloads.c3_uri(rng, regs, True).encode() for _ in range(12)]
        subjects += [workloads.c3_uri(rng, own, True).encode() for _ in range(6)] if own else []
        subjects += [x + b"\n" for x in subjects[-3:]]
        for s in subjects:
            got = L.gm_debug_regex_rev(pat.encode(), 1 if ci else 0, s, len(s))
            assert got >= 0, pat
            exp = pcre_match(pat, s, ci)
            assert got == exp, (pat, ci, s)
            n_hit += exp
    assert len(cases) > 100 and n_hit > 300


def test_regex_factors():
    L = ctypes.CDLL(engine.LIB_PATH)
    L.gm_debug_regex_factors.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    buf = ctypes.create_string_buffer(4096)

    def f(p):
        m = L.gm_debug_regex_factors(p.encode(), 0, buf, 4096)
        return m, sorted(x for x in buf.value.decode().split("\n") if x)
    assert f(r"union\s+select") == (6, ["select"])
    assert f(r"(abcd|efgh)x") == (5, ["abcdx", "efghx"])
    assert f(r"SeLect.{0,8}from")[1] == ["select"]
    assert f(r"[a-z]+\d+")[0] == 0
    for p in [r"(a)\1", r"x(?=y)"]:
        assert L.gm_debug_regex_factors(p.encode(), 0, buf, 4096) < 0


def test_c4_signature_set_compiles():
    ss = workloads.c4_sigset(800, 200)
    e = engine.Engine(compile_only=True)
    e.load(workloads.c4_blob(ss), 3)
    s = e.stats()
    assert s["n_sigs"] == 1000 and s["n_sig_literals"] == 800 and s["n_sig_regex"] == 200
    assert s["n_rejected_pcre"] == 0 and s["n_rejected_other"] == 0
    assert s["n_sig_regex_always"] == 0


def _prefilter(e, arena, stage2=False):
    L = ctypes.CDLL(engine.LIB_PATH)
    f = L.gm_debug_waf_prefilter2 if stage2 else L.gm_debug_waf_prefilter
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    a = np.ascontiguousarray(arena)
    n = f(e.h, a.ctypes.data, a.size, None, 0)
    out = np.zeros(max(n, 1), np.uint64)
    f(e.h, a.ctypes.data, a.size, out.ctypes.data, n)
    return out[:n]


@pytest.mark.parametrize("stage2", [False, True])
def test_prefilter_covers_every_literal_occurrence(stage2):
    """Host restatement of the scan kernel's candidate rule (and of k_waf_verify's stage-2
    context filter): every occurrence of every literal (any case for nocase rules) yields a
    candidate inside the occurrence, and the false-positive rate on the C4 traffic stays small."""
    from gpumatch import records
    ss = workloads.c4_sigset(800, 200)
    e = engine.Engine(compile_only=True)
    e.load(workloads.c4_blob(ss), 3)
    reqs, arena = records.gen_c4(3000, ss, plant_rate=0.3)
    cand = np.sort(_prefilter(e, arena, stage2))
    a = bytes(arena)
    al = a.lower()
    checked = 0
    for r in ss.rules:
        if r.kind != "lit":
            continue
        pat = bytes(r.pattern)
        hay, needle = (al, pat.lower()) if r.nocase else (a, pat)
        start = hay.find(needle)
        while start >= 0:
            # stride-2 scan: the candidate is an even offset in [start - 1, start + len - 3] (a key
            # window inside the pattern, or one of the one-byte-extended key families: the byte
            # before the pattern, or the byte after it -- gm_compile.cpp choose_keys)
            k = np.searchsorted(cand, start - 1)
            assert k < len(cand) and cand[k] <= start + len(pat) - 3, (pat, start)
            assert cand[k] % 2 == 0
            checked += 1
            start = hay.find(needle, start + 1)
    assert checked > 200
    assert len(cand) < len(a) * (5e-4 if stage2 else 2e-3)


def test_c3_regex_locations_compile(eng):
    """C3: 1k regex locations compile; the PCRE-only ones are rejected and
    counted, and the oracle's restated PCRE-only rule agrees with the compiler on every one."""
    import ctypes
    from oracle_py import lib as oracle_lib
    regs = workloads.c3_regexes()
    eng.load(workloads.c3_blob(regs), 3)
    s = eng.stats()
    ol = oracle_lib()
    ol.orc_pcre_only.restype = ctypes.c_int
    ol.orc_pcre_only.argtypes = [ctypes.c_char_p]
    flagged = [bool(ol.orc_pcre_only(p.encode())) for p, *_ in regs]
    assert flagged == [r[2] for r in regs]
    assert s["n_rejected_pcre"] == sum(flagged) > 0
    assert s["n_locations"] == len(regs) + 3
    # the anchored and the reversed slices carry head maps (k_rloc_heads): they run over
    # candidate lists
    assert s["n_rsl_reversed"] < s["n_rsl_heads"] <= s["n_rsl_slices"], s


def test_in_tree_library_is_the_default_build():
    """The in-tree libgpumatch.so carries no measurement or tuning macros (gm_stats build_flags = 0):
    what the tests, smoke() and bench.py load is the shipped pipeline (bench.py refuses otherwise)."""
    e = engine.Engine(compile_only=True)
    e.load(workloads.c1_blob(), 1)
    st = e.stats()
    assert st["build_flags"] == 0 and st["scratch_scale"] == 1.0 and st["set_shift"] == 0


# The largest private segment (scratch per lane) any shipped kernel may have. The route's realip
# instances are the largest (~1.8 KiB: the header walk's out-of-line leaves and their saves).
PRIVATE_SEGMENT_MAX = 2048
LLVM_BIN = "/opt/rocm/lib/llvm/bin"


def _kernel_metadata(lib_path, tmp_path):
    """The gfx950 code object's kernel descriptors: (name, uses_dynamic_stack, private bytes)."""
    import subprocess
    fb, co = str(tmp_path / "fatbin"), str(tmp_path / "gfx950.o")
    subprocess.check_call([f"{LLVM_BIN}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}",
                           lib_path, str(tmp_path / "stripped.so")])
    subprocess.check_call([f"{LLVM_BIN}/clang-offload-bundler", "--unbundle", "--type=o",
                           f"--input={fb}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                           f"--output={co}"])
    notes = subprocess.check_output([f"{LLVM_BIN}/llvm-readelf", "--notes", co], text=True)
    out = []
    for blk in notes.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        dyn = re.search(r"\.uses_dynamic_stack:\s+(\w+)", blk).group(1) == "true"
        priv = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk).group(1))
        out.append((name, dyn, priv))
    return out


@pytest.mark.skipif(not os.path.exists(f"{LLVM_BIN}/clang-offload-bundler"),
                    reason="ROCm LLVM tools absent")
def test_no_kernel_has_a_dynamic_stack(tmp_path):
    """Round 4's illegal memory access (test_peer_selection_long_sequential_runs): a recursive
    device function (parse_addr calling itself for an IPv6 address's dotted tail) gave k_peer_pick
    `uses_dynamic_stack: true` beside a 1536 B fixed private segment. The runtime sizes scratch
    from the fixed part, so the recursion's frames ran past the lane's scratch. Any recursive,
    alloca or indirect call brings the dynamic stack back: fail the build, and bound the fixed
    private segment every kernel may use."""
    md = _kernel_metadata(engine.LIB_PATH, tmp_path)
    assert len(md) > 100, "no gfx950 kernels found in libgpumatch.so"
    assert any(n.startswith("_ZN12_GLOBAL__N_111k_waf_scan") or "k_waf_scan" in n for n, _, _ in md)
    dyn = [n for n, d, _ in md if d]
    assert not dyn, f"kernels with a dynamic stack: {dyn}"
    big = [(n, p) for n, _, p in md if p > PRIVATE_SEGMENT_MAX]
    assert not big, f"kernels over {PRIVATE_SEGMENT_MAX} B of private segment: {big}"


def test_library_names_its_sources():
    """Evidence hygiene: libgpumatch.so carries the hash of the sources it was built
    from (gm_build_hash, gm_stats_t.csrc_hash); the shipped library must be built from this tree,
    so a profile stamped with the tree's hash describes the library that runs."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from scan_profile import csrc_hash
    assert engine.build_hash() == csrc_hash(ROOT)
