"""WAF signature sets.

The Wallarm detection engine is a proprietary binary package that is not in the reference
(``build/DockerfileForPlus:7,75``), so the signature layer is build-defined.  What the
reference does fix is *where* it applies: ``wallarm_mode`` per server / location
(``annotations.go:294-330``, ``version1/nginx.ingress.tmpl:12-29,96-113``; modes off,
monitoring, safe_blocking, block).

Text format (one rule per line, ``#`` comments)::

    <kind> <flags> <zones> <pattern>
    lit  i  uahb  756e696f6e2073656c656374      # hex bytes of the literal
    re   -  ua    union\\s+(all\\s+)?select       # PCRE syntax, rest of the line

``flags``: ``i`` = ASCII case-insensitive, ``-`` = exact.  ``zones``: subset of ``u`` ($uri),
``a`` ($args), ``h`` (header block), ``b`` (body).  Rule ids are line order (0-based among
rules).  A rule hits a request if its literal occurs in / its regex matches anywhere in any of
its zones (PCRE 8.x search semantics, no DOTALL/MULTILINE).
"""

from __future__ import annotations

import numpy as np


class Rule:
    __slots__ = ("kind", "nocase", "zones", "pattern", "example")

    def __init__(self, kind, nocase, zones, pattern, example=None):
        self.kind = kind            # "lit" | "re"
        self.nocase = nocase
        self.zones = zones          # e.g. "uahb"
        self.pattern = pattern      # bytes for lit, str for re
        self.example = example      # bytes that match (generator only)


class SigSet:
    """``decoders``: the request parsers (Wallarm's names: percent, urlenc, json_doc, base64) whose
    decoded views of $args / the body the rules also scan ("@decoders" line, gm_decode.inc)."""

    def __init__(self, rules, decoders=()):
        self.rules = list(rules)
        self.decoders = list(decoders)

    def to_text(self) -> str:
        out = ["# gpumatch signature set v1"]
        if self.decoders:
            out.append("@decoders " + ",".join(self.decoders))
        for r in self.rules:
            fl = "i" if r.nocase else "-"
            if r.kind == "lit":
                out.append(f"lit {fl} {r.zones} {r.pattern.hex()}")
            else:
                out.append(f"re {fl} {r.zones} {r.pattern}")
        return "\n".join(out) + "\n"

    @staticmethod
    def from_text(text: str) -> "SigSet":
        rules, dec = [], []
        for line in text.splitlines():
            s = line.strip()
            if not s or s.startswith("#"):
                continue
            if s.startswith("@decoders"):
                dec += [x.strip() for x in s[9:].split(",") if x.strip()]
                continue
            kind, fl, zones, pat = s.split(" ", 3)
            if kind == "lit":
                rules.append(Rule("lit", fl == "i", zones, bytes.fromhex(pat)))
            else:
                rules.append(Rule("re", fl == "i", zones, pat))
        return SigSet(rules, dec)


# --------------------------------------------------------------------------- C4 generator

_TOKENS = ("union select", "select from", "information_schema", "' or '1'='1", "\" or \"1\"=\"1",
           "or 1=1--", "drop table", "insert into", "xp_cmdshell", "benchmark(", "sleep(", "waitfor delay",
           "load_file(", "into outfile", "<script", "</script>", "javascript:", "onerror=", "onload=",
           "<iframe", "<svg/onload", "document.cookie", "alert(", "eval(", "../../", "..\\..\\",
           "/etc/passwd", "/etc/shadow", "c:\\windows", "cmd.exe", "/bin/sh", "wget http", "curl http",
           "${jndi:", "%00", "php://input", "base64_decode(", "system(", "passthru(", "shell_exec(",
           "<?php", "${ifs}", ";cat ", "|id;", "`id`", "$(id)", "nslookup ", "ping -c", "/proc/self/",
           "<!entity", "<!doctype", "sqlmap", "nikto", "acunetix", "dirbuster", "masscan", "hydra",
           "/wp-admin", "/phpmyadmin", ".git/config", ".env", "web.config", "/actuator/", "select pg_",
           "utl_http", "dbms_pipe", "extractvalue(", "updatexml(", "group_concat(", "concat(0x",
           "char(", "chr(", "0x3c7363", "%3cscript", "&#x3c;", "\\x3c", "fromcharcode", "vbscript:",
           "expression(", "srcdoc=", "formaction=")

_ALPH = "abcdefghijklmnopqrstuvwxyz0123456789_"


def _rand_word(rng, lo, hi):
    k = int(rng.integers(lo, hi + 1))
    return "".join(_ALPH[int(c)] for c in rng.integers(0, len(_ALPH), k))


def _zones(rng):
    r = rng.random()
    if r < 0.6:
        return "uahb"
    if r < 0.8:
        return "ua"
    if r < 0.9:
        return "b"
    return "h"


def _regex_rule(rng, nocase):
    """RE2-compatible WAF-style regex with a >= 4-byte required literal, plus an example."""
    t = int(rng.integers(0, 6))
    w1 = _rand_word(rng, 4, 8)
    w2 = _rand_word(rng, 4, 8)
    w3 = _rand_word(rng, 4, 8)
    d = str(int(rng.integers(0, 9999)))
    if t == 0:
        pat, ex = f"{w1}\\s+{w2}", f"{w1}  {w2}"
    elif t == 1:
        pat, ex = f"{w1}\\s*\\(\\s*\\d{{1,4}}\\s*\\)", f"{w1}( {d} )"
    elif t == 2:
        pat, ex = f"<{w1}[^>]{{0,16}}on[a-z]{{2,8}}\\s*=", f"<{w1} x=1 onload ="
    elif t == 3:
        pat, ex = f"({w1}|{w2}|{w3})[a-z0-9]+--", f"{w2}abc9--"
    elif t == 4:
        pat, ex = f"{w1}.{{0,8}}{w2}", f"{w1}..x.{w2}"
    else:
        pat, ex = f"(?:{w1}|{w2})=[0-9a-f]{{8,}}", f"{w1}=deadbeef01"
    if nocase:
        ex = ex.upper()
    return pat, ex.encode()


def _job_regex_rule(rng, nocase):
    """A regex whose required >= 4-byte factor is NOT a prefix (a class or alternation comes
    first): the prefilter's factor hits become (request, zone, regex) jobs for k_waf_regex."""
    t = int(rng.integers(0, 4))
    w1 = _rand_word(rng, 4, 8)
    w2 = _rand_word(rng, 4, 8)
    if t == 0:
        pat, ex = f"\\d+{w1}\\s+{w2}", f"42{w1}  {w2}"
    elif t == 1:
        pat, ex = f"[a-z]+_{w1}\\s", f"abc_{w1} "
    elif t == 2:
        pat, ex = f"(?:%27|'){w1}[=(]", f"'{w1}("
    else:
        pat, ex = f"[0-9a-f]{{2,}}{w1}.{{0,6}}{w2}", f"0a{w1}..{w2}"
    if nocase:
        ex = ex.upper()
    return pat, ex.encode()


def gen_waf_sigset(n_lit: int = 8000, n_re: int = 2000, seed: int = 0xC0FFEE + 3, job_frac: float = 0.0) -> SigSet:
    """C4: literals 4-32 B (SQLi/XSS/traversal-style tokens + random tails so that benign
    text does not contain them) and RE2-subset regexes.  ``job_frac``: the share of regexes whose
    factor is not a prefix (k_waf_regex jobs; 0 keeps the headline set's random stream)."""
    rng = np.random.Generator(np.random.PCG64(seed ^ 0x5157))
    rules = []
    seen = set()
    while len(rules) < n_lit:
        tok = _TOKENS[int(rng.integers(0, len(_TOKENS)))]
        mode = rng.random()
        if mode < 0.15 and len(seen) < len(_TOKENS):
            s = tok
        elif mode < 0.55:
            s = tok + _rand_word(rng, 2, 10)
        else:
            s = _rand_word(rng, 2, 6) + tok + _rand_word(rng, 0, 6)
        s = s[:32]
        if len(s) < 4 or s in seen:
            continue
        seen.add(s)
        nocase = rng.random() < 0.7
        b = s.encode()
        ex = b.upper() if (nocase and rng.random() < 0.5) else b
        rules.append(Rule("lit", nocase, _zones(rng), b, ex))
    for _ in range(n_re):
        nocase = rng.random() < 0.5
        if job_frac > 0 and rng.random() < job_frac:
            pat, ex = _job_regex_rule(rng, nocase)
        else:
            pat, ex = _regex_rule(rng, nocase)
        rules.append(Rule("re", nocase, _zones(rng), pat, ex))
    order = rng.permutation(len(rules))
    return SigSet([rules[i] for i in order])


# --------------------------------------------------------------------------- C4 stress variant
# The headline C4 set keeps benign traffic nearly candidate-free (random literal tails, a random
# required word in every regex).  The stress variant drops both: literals are plain SQL / HTML /
# shell vocabulary (two or three words) that benign text (records.gen_c4(stress=True)) also
# speaks, and 10% of the regexes have no >= 4-byte factor, so every (request, zone) runs them
# (k_waf_always); another 10% have a factor that is not a prefix (k_waf_regex jobs); the other
# regexes keep the headline's shapes.  The prefilter passes far more
# windows, the exact stage verifies real matches, and the always-run DFAs carry the load.
VOCAB = ("select", "from", "where", "union", "insert", "into", "update", "delete", "drop", "table", "order",
         "group", "by", "having", "limit", "offset", "join", "inner", "outer", "left", "values", "set",
         "script", "iframe", "img", "src", "href", "onload", "onerror", "onclick", "alert", "document",
         "cookie", "window", "location", "eval", "function", "return", "var", "const", "style", "div",
         "span", "form", "input", "button", "action", "method", "post", "get", "http", "https", "www",
         "admin", "login", "password", "user", "passwd", "shadow", "etc", "bin", "bash", "cat", "echo",
         "curl", "wget", "exec", "system", "cmd", "shell", "php", "include", "require", "file", "path",
         "null", "true", "false", "and", "or", "not", "like", "count", "sum", "max", "min", "concat",
         "char", "sleep", "benchmark", "version", "database", "schema", "information", "columns")
_JOIN = (" ", "(", "=", "<", "/", "_", "'", " '", "--", ".")


def gen_waf_sigset_stress(n_lit: int = 8000, n_re: int = 2000, seed: int = 0xC0FFEE + 13) -> SigSet:
    rng = np.random.Generator(np.random.PCG64(seed ^ 0x5157))
    rules, seen = [], set()
    V = VOCAB
    while len(rules) < n_lit:
        k = int(rng.integers(2, 4))
        parts = [V[int(i)] for i in rng.integers(0, len(V), k)]
        s = parts[0]
        for w in parts[1:]:
            s += _JOIN[int(rng.integers(0, len(_JOIN)))] + w
        if rng.random() < 0.3:
            s = _JOIN[int(rng.integers(0, len(_JOIN)))] + s
        if len(s) < 4 or len(s) > 32 or s in seen:
            continue
        seen.add(s)
        nocase = rng.random() < 0.7
        b = s.encode()
        rules.append(Rule("lit", nocase, _zones(rng), b, b.upper() if nocase and rng.random() < 0.5 else b))
    n_always = n_re // 10
    n_jobs = n_re // 10
    for i in range(n_re):
        nocase = rng.random() < 0.5
        if i < n_always:   # no >= 4-byte factor: every (request, zone) runs it (k_waf_always)
            t = int(rng.integers(0, 4))
            k = int(rng.integers(2, 6))
            a2 = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, 2))
            b2 = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, 2))
            if t == 0:
                pat, ex = f"[0-9]{{{k},}}[a-f]x", "9" * k + "ax"
            elif t == 1:
                pat, ex = f"({a2}|{b2})[0-9]{{{k}}}--", a2 + "7" * k + "--"
            elif t == 2:
                pat, ex = f"=\\s*[0-9]{{{k}}}'\\s*or", "= " + "4" * k + "' or"
            else:
                pat, ex = f"<[a-z]{{1,3}}\\s+{a2}[a-z]{{{k}}}=", "<b " + a2 + "q" * k + "="
            if nocase:
                ex = ex.upper()
            rules.append(Rule("re", nocase, _zones(rng), pat, ex.encode()))
        elif i < n_always + n_jobs:   # the factor is not a prefix: k_waf_regex jobs
            pat, ex = _job_regex_rule(rng, nocase)
            rules.append(Rule("re", nocase, _zones(rng), pat, ex))
        else:
            pat, ex = _regex_rule(rng, nocase)
            rules.append(Rule("re", nocase, _zones(rng), pat, ex))
    order = rng.permutation(len(rules))
    return SigSet([rules[i] for i in order])
