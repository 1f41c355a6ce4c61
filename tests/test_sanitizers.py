"""ASan + UBSan CPU builds of the code that parses untrusted text (VERDICT r1
item 10): the generation compiler (gm_compile.cpp, gm_regex.cpp) over every workload's
generation plus 300 mutated configs and signature sets, and the oracle (gm_oracle.c) over the
same generations with their traffic, the wire parser's edge messages, the balancers, the
upstream URIs and the $uri normaliser.  Any sanitizer report aborts the harness
(-fno-sanitize-recover=all)."""

import os
import subprocess

import numpy as np
import pytest

from gpumatch import blob, peers, records, sigs, wire, workloads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def harnesses():
    subprocess.run(["make", "-s", "-j3", "-C", SAN], check=True, timeout=1200)
    return os.path.join(SAN, "compile_harness"), os.path.join(SAN, "oracle_harness")


def _generations():
    from test_decoders import decoder_blob
    from test_rewrites import cafe_rewrites_blob
    ss = workloads.c4_sigset(800, 200)
    return {
        "c1": workloads.c1_blob(), "c2": workloads.c2_blob(), "c5": workloads.c5_blob(200),
        "c3": workloads.c3_blob(workloads.c3_regexes(150)), "c4": workloads.c4_blob(ss),
        "stress": workloads.c4_blob(sigs.SigSet(sigs.gen_waf_sigset_stress(800, 200).rules, ("percent", "base64"))),
        "peers": peers.peers_blob(), "decoders": decoder_blob(), "rewrites": cafe_rewrites_blob(),
    }


def _mutations(base: bytes, k: int, seed: int):
    """config / signature text with random deletions, insertions of syntax bytes and truncations"""
    rng = np.random.default_rng(seed)
    out = []
    ents = blob.parse_blob(base)
    for _ in range(k):
        new = []
        for kind, name, data in ents:
            d = bytearray(data)
            for _ in range(int(rng.integers(1, 6))):
                if not d:
                    break
                p = int(rng.integers(0, len(d)))
                op = int(rng.integers(0, 4))
                if op == 0:
                    del d[p]
                elif op == 1:
                    syn = b"{};\"'\\$~*()[]|"
                    d[p:p] = bytes([syn[int(rng.integers(0, len(syn)))]])
                elif op == 2:
                    d = d[:p]
                else:
                    d[p] = int(rng.integers(0, 256))
            new.append((kind, name, bytes(d)))
        main = next((d for kd, _, d in new if kd == blob.ENTRY_MAIN), None)
        confd = {n.decode()[:-5] if n.endswith(b".conf") else n.decode(): d for kd, n, d in new if kd == blob.ENTRY_CONFD}
        sg = next((d for kd, _, d in new if kd == blob.ENTRY_SIGS), None)
        out.append(blob.make_blob(main, confd, sg))
    return out


def test_compiler_under_sanitizers(harnesses, tmp_path):
    comp, _ = harnesses
    gens = _generations()
    files = []
    for name, b in gens.items():
        p = tmp_path / f"{name}.blob"
        p.write_bytes(b)
        files.append(str(p))
    for name in ("c1", "c2", "rewrites", "decoders", "peers", "c4"):
        for i, m in enumerate(_mutations(gens[name], 50, sum(name.encode()))):
            p = tmp_path / f"{name}_m{i}.blob"
            p.write_bytes(m)
            files.append(str(p))
    r = subprocess.run([comp] + files, capture_output=True, timeout=1800, env=ENV)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0 and "runtime error" not in err and "AddressSanitizer" not in err, err[-4000:]
    assert r.stdout.decode().count("ok=1") >= len(gens)


def test_oracle_under_sanitizers(harnesses, tmp_path):
    _, orc = harnesses
    gens = _generations()
    msgs, conn = wire.synthetic(1500, seed=77)
    w, m = wire.build(msgs + list(wire._EDGE), (conn + [None] * len(wire._EDGE)))
    (tmp_path / "wire.bin").write_bytes(w.tobytes())
    (tmp_path / "msgs.bin").write_bytes(m.tobytes())
    traffic = {"c1": records.gen_c1(2000), "c2": records.gen_c2(2000), "c5": workloads.gen_c5(2000, 200),
               "c4": records.gen_c4(1500, workloads.c4_sigset(800, 200), plant_rate=0.1, pool_mb=2),
               "peers": peers.gen_requests(3000)}
    args = [orc, str(tmp_path / "wire.bin"), str(tmp_path / "msgs.bin")]
    for name, (reqs, arena) in traffic.items():
        for suffix, data in (("blob", gens[name]), ("reqs", reqs.tobytes()), ("arena", arena.tobytes())):
            (tmp_path / f"{name}.{suffix}").write_bytes(data)
        args += [str(tmp_path / f"{name}.{x}") for x in ("blob", "reqs", "arena")]
    r = subprocess.run(args, capture_output=True, timeout=1800, env=ENV)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0 and "runtime error" not in err and "AddressSanitizer" not in err, err[-4000:]
    assert r.stdout.decode().count("requests ok") == len(traffic)


def test_union_dfa_under_sanitizers(harnesses, tmp_path):
    """The union DFAs (gm_regex.cpp build_multi + minimize_multi) under ASan/UBSan, and their
    answers: for groups of 1..32 regexes -- the always-run shapes of the WAF stress set and of the
    parity test, and C3's regex locations -- every member's bit equals its own search DFA's answer
    on random subjects (empty ones, a final newline, anchors)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_parity import always_rules
    pats = [(r.nocase, r.pattern) for r in always_rules()]
    pats += [(r.nocase, r.pattern) for r in sigs.gen_waf_sigset_stress(200, 300).rules if r.kind == "re"][:120]
    pats += [(ci, pat) for (pat, ci, *_r) in workloads.c3_regexes(300)]
    (tmp_path / "re.txt").write_text("".join(f"{int(ci)} {p}\n" for ci, p in pats))
    rng = np.random.Generator(np.random.PCG64(5))
    alpha = "abcdefghij0123456789-=<>/. xzqAB'\\"
    subj = []
    for _ in range(400):
        s = "".join(alpha[int(i)] for i in rng.integers(0, len(alpha), int(rng.integers(0, 60))))
        if rng.random() < 0.3:
            s = "/" + s
        if rng.random() < 0.2:
            s += "\\n"
        subj.append(s)
    (tmp_path / "subj.txt").write_text("\n".join(subj) + "\n")
    exe = os.path.join(SAN, "union_harness")
    r = subprocess.run([exe, str(tmp_path / "re.txt"), str(tmp_path / "subj.txt")], capture_output=True,
                       timeout=1200, env=ENV)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0 and "runtime error" not in err and "AddressSanitizer" not in err, err[-4000:]
    out = r.stdout.decode()
    assert "mismatches 0" in out and int(out.split("groups ")[1].split()[0]) >= 10, out
