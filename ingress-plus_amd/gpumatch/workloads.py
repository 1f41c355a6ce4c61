"""The five BASELINE.json configurations as (generation blob, request generator) pairs.

Config resources are the reference's own examples (examples/complete-example/cafe-ingress.yaml,
examples-of-custom-resources/advanced-routing + traffic-splitting, the e2e complex VS of
tests/data/virtual-server-advanced-routing/virtual-server-complex.yaml, examples/mergeable-
ingress-types), rendered through ``confgen`` exactly as the Configurator would hand them to
``nginx.Manager.CreateConfig``.
"""

from __future__ import annotations

import copy

import numpy as np

from . import blob, confgen, records, sigs

CAFE_INGRESS = {
    "apiVersion": "extensions/v1beta1", "kind": "Ingress",
    "metadata": {"name": "cafe-ingress", "namespace": "default"},
    "spec": {"tls": [{"hosts": ["cafe.example.com"], "secretName": "cafe-secret"}],
             "rules": [{"host": "cafe.example.com", "http": {"paths": [
                 {"path": "/tea", "backend": {"serviceName": "tea-svc", "servicePort": 80}},
                 {"path": "/coffee", "backend": {"serviceName": "coffee-svc", "servicePort": 80}}]}}]},
}

ADV_ROUTING_VS = {
    "metadata": {"name": "cafe", "namespace": "default"},
    "spec": {"host": "cafe.example.com",
             "tls": {"secret": "cafe-secret"},
             "upstreams": [{"name": "tea-post", "service": "tea-post-svc", "port": 80},
                           {"name": "tea", "service": "tea-svc", "port": 80},
                           {"name": "coffee-v1", "service": "coffee-v1-svc", "port": 80},
                           {"name": "coffee-v2", "service": "coffee-v2-svc", "port": 80}],
             "routes": [{"path": "/tea", "rules": {"conditions": [{"variable": "$request_method"}],
                                                   "matches": [{"values": ["POST"], "upstream": "tea-post"}],
                                                   "defaultUpstream": "tea"}},
                        {"path": "/coffee", "rules": {"conditions": [{"cookie": "version"}],
                                                      "matches": [{"values": ["v2"], "upstream": "coffee-v2"}],
                                                      "defaultUpstream": "coffee-v1"}}]},
}

SPLIT_VS = {
    "metadata": {"name": "cafe-split", "namespace": "default"},
    "spec": {"host": "split.example.com",
             "upstreams": [{"name": "coffee-v1", "service": "coffee-v1-svc", "port": 80},
                           {"name": "coffee-v2", "service": "coffee-v2-svc", "port": 80}],
             "routes": [{"path": "/coffee", "splits": [{"weight": 90, "upstream": "coffee-v1"},
                                                       {"weight": 10, "upstream": "coffee-v2"}]}]},
}

COMPLEX_VS = {
    "metadata": {"name": "virtual-server-adv-routing", "namespace": "default"},
    "spec": {"host": "virtual-server-adv-routing.example.com",
             "upstreams": [{"name": "backend2", "service": "backend2-svc", "port": 80},
                           {"name": "backend4-stable", "service": "backend4-stable-svc", "port": 80},
                           {"name": "backend1-future", "service": "backend1-future-svc", "port": 80},
                           {"name": "backend3-deprecated", "service": "backend3-deprecated-svc", "port": 80}],
             "routes": [{"path": "/backends", "rules": {
                 "conditions": [{"header": "x-version"}, {"cookie": "user"}, {"argument": "arg1"},
                                {"variable": "$request_method"}],
                 "matches": [{"values": ["future", "some", "v1", "get"], "upstream": "backend1-future"},
                             {"values": ["deprecated", "bad", "v2", "post"], "upstream": "backend3-deprecated"}],
                 "defaultUpstream": "backend4-stable"}},
                 {"path": "/backend2", "upstream": "backend2"}]},
}


def c1_blob(gen_params=None) -> bytes:
    files = confgen.ingress_files([CAFE_INGRESS], secrets=("cafe-secret",))
    return blob.make_blob(confgen.render_main(), files)


def c2_blob() -> bytes:
    files = confgen.virtual_server_files([ADV_ROUTING_VS, SPLIT_VS, COMPLEX_VS])
    return blob.make_blob(confgen.render_main(), files)


def c4_sample(sigset: sigs.SigSet, n: int = 2000, seed: int = records.SEED_BASE + 33, stress: bool = False) -> bytes:
    """A benign traffic sample for the WAF prefilter tuning (GM_ENTRY_SAMPLE): C4 requests from a
    seed disjoint from every pool the tests and the bench match (a deployment samples its own
    recent traffic the same way); the zone bytes only."""
    reqs, arena = records.gen_c4(n, sigset, seed=seed, plant_rate=0.0, pool_mb=2, stress=stress)
    parts = []
    for r in reqs:
        b = int(r["base"])
        z = int(r["uri_len"]) + int(r["args_len"]) + int(r["hdr_len"]) + int(r["body_len"])
        parts.append(arena[b:b + z].tobytes())
    return b"".join(parts)


def c4_blob(sigset: sigs.SigSet, mode: str = "block", sample: bytes | None = None, parser_disable: str = "") -> bytes:
    base = confgen.default_config_params()
    base["MainEnableWallarm"] = True
    ing = copy.deepcopy(CAFE_INGRESS)
    ing["metadata"]["annotations"] = {"wallarm.com/mode": mode}
    if parser_disable:
        ing["metadata"]["annotations"]["wallarm.com/parser-disable"] = parser_disable
    files = confgen.ingress_files([ing], base=base, secrets=("cafe-secret",))
    return blob.make_blob(confgen.render_main(base), files, sigset.to_text(), sample)


def c5_blob(n_hosts: int = 1000, seed: int = records.SEED_BASE + 4) -> bytes:
    """Mergeable Ingress: n masters x 1-8 minions, TLS without secretName -> wildcard secret."""
    rng = np.random.Generator(np.random.PCG64(seed))
    masters, minions = [], []
    for h in range(n_hosts):
        host = f"app{h}.example.com"
        masters.append({"metadata": {"name": f"m{h}", "namespace": "default",
                                     "annotations": {"nginx.org/mergeable-ingress-type": "master"}},
                        "spec": {"tls": [{"hosts": [host]}], "rules": [{"host": host}]}})
        k = int(rng.integers(1, 9))
        for j in range(k):
            paths = [{"path": f"/svc{j}/v{q}", "backend": {"serviceName": f"s{h}-{j}", "servicePort": 80}}
                     for q in range(int(rng.integers(1, 3)))]
            minions.append({"metadata": {"name": f"m{h}-{j}", "namespace": "default",
                                         "creationTimestamp": f"2019-01-01T00:{j:02d}:00Z",
                                         "annotations": {"nginx.org/mergeable-ingress-type": "minion"}},
                            "spec": {"rules": [{"host": host, "http": {"paths": paths}}]}})
    by_host = {}
    for m in minions:
        by_host.setdefault(m["spec"]["rules"][0]["host"], []).append(m)
    files = {}
    base = confgen.default_config_params()
    for m in masters:
        mins = confgen.get_minions_for_master(m, by_host.get(m["spec"]["rules"][0]["host"], []))
        cfg = confgen.generate_nginx_cfg_for_mergeable(
            {"Ingress": m, "Endpoints": {}}, [{"Ingress": x, "Endpoints": {}} for x in mins],
            confgen.tls_pems(m, wildcard=True), base)
        files[confgen.object_meta_to_file_name(m)] = confgen.render_ingress(cfg)
    return blob.make_blob(confgen.render_main(), files)


def gen_c5(n: int, n_hosts: int = 1000, seed: int = records.SEED_BASE + 4):
    """Zipf(1.1) over hosts; URIs hit minion paths, prefixes of them, or miss."""
    rng = np.random.Generator(np.random.PCG64(seed ^ 0xABCDEF))
    z = rng.zipf(1.1, n)
    host_idx = (z - 1) % n_hosts
    hosts = [f"app{h}.example.com" for h in range(n_hosts)] + ["unknown.example.com"]
    host_idx = np.where(rng.random(n) < 0.02, n_hosts, host_idx)
    https = rng.random(n) < 0.5
    uris = [f"/svc{j}/v{q}" for j in range(8) for q in range(2)] + ["/", "/svc1", "/svc1/", "/other"]
    uidx = rng.integers(0, len(uris), n)
    suf = records.geometric_lens(rng, n, 12, 0, 256)
    pool = records.alnum_pool(rng, 1 << 16)
    fields = {"uri": [records.choice_seg(uris, uidx), records.pool_seg(pool, suf, rng)],
              "host": [records.choice_seg(hosts, host_idx)],
              "method": [records.const_seg("GET", n)],
              "raddr": [records.const_seg("10.1.2.3", n)]}
    return records.build(n, fields, np.where(https, 443, 80), np.where(https, records.REQ_HTTPS, 0),
                         rng.integers(0, 256, (n, 16), dtype=np.uint8), rng.integers(1024, 65535, n))


def c4_sigset(n_lit=8000, n_re=2000) -> sigs.SigSet:
    return sigs.gen_waf_sigset(n_lit, n_re)


def c4_job_sigset(n_lit=200, n_re=300) -> sigs.SigSet:
    """A small C4-shaped set whose regexes are mostly factor-but-not-prefix shapes: the regex-job
    path (k_waf_regex) carries load (it had none in any benchmarked workload)."""
    return sigs.gen_waf_sigset(n_lit, n_re, seed=0xC0FFEE + 21, job_frac=0.8)


def c4_bench_generation():
    """The benchmarked C4 generation (bench.py): the 10k-rule set on the cafe Ingress in
    wallarm_mode block, with a benign traffic sample (disjoint seed) steering the prefilter's
    key choice.  Returns (sigset, blob)."""
    ss = c4_sigset()
    return ss, c4_blob(ss, "block", sample=c4_sample(ss))


C4_POOL_SEED = records.SEED_BASE + 3


def replicate_pool(preqs: np.ndarray, parena_len: int, n: int):
    """Headers of ``n`` requests that repeat a ``len(preqs)``-request pool: copy k of the pool's
    arena sits at k * plen (plen = the pool arena rounded up to 16 B).  Returns (reqs, plen,
    reps, arena_len); the caller lays the ``reps`` arena copies out in device memory."""
    pool_n = len(preqs)
    plen = (parena_len + 15) & ~15
    reps = (n + pool_n - 1) // pool_n
    reqs = np.tile(preqs, reps)[:n]
    reqs["base"] += (np.repeat(np.arange(reps, dtype=np.uint64), pool_n)[:n] * np.uint64(plen))
    last = reqs[-1]
    arena_len = int(last["base"]) + sum(int(last[f]) for f in ("uri_len", "args_len", "hdr_len", "body_len",
                                                                "host_len", "method_len", "ruri_len", "raddr_len"))
    return reqs, plen, reps, arena_len


# algorithmic bytes per request: 64 B header + payload of the fields the
# config reads + 32 B verdict (+ 4 B per hit id, added by the caller)
def algorithmic_bytes(reqs: np.ndarray, config: str) -> int:
    n = len(reqs)
    hdr = 64 * n + 32 * n
    if config in ("c1", "c5"):
        return hdr + int(reqs["host_len"].sum()) + int(reqs["uri_len"].sum())
    if config == "c4":
        return hdr + int(reqs["uri_len"].sum() + reqs["args_len"].sum() + reqs["hdr_len"].sum() +
                         reqs["body_len"].sum())
    if config == "c2":
        return hdr + int(reqs["host_len"].sum() + reqs["uri_len"].sum() + reqs["args_len"].sum() +
                         reqs["hdr_len"].sum() + reqs["method_len"].sum()) + 16 * n
    return hdr + int(reqs["uri_len"].sum())


# --------------------------------------------------------------------------- C3 regex locations

C3_HOST = "regex.example.com"
_C3_WORDS = ("api", "v1", "v2", "v3", "users", "items", "shop", "cart", "img", "static", "blog", "post",
             "search", "admin", "login", "docs", "files", "media", "video", "feed", "news", "order",
             "account", "profile", "catalog", "product", "assets", "report", "export", "tags",
             "comments", "upload", "download", "health", "status", "metrics", "session", "user",
             "group", "team", "project", "build", "release", "config", "settings", "page", "wiki")
_C3_EXT = ("json", "xml", "php", "html", "png", "jpg", "css", "js", "txt", "csv")
# PCRE-only constructs (rejected at compile time and counted)
_C3_PCRE_ONLY = ("(?=/)", "(?!x)", "(?<=/)", "(\\w+)/\\1", "[a-z]++", "(?>ab|a)", "\\Kz")


def c3_regexes(n: int = 1000, seed: int = records.SEED_BASE + 2):
    """C3: ``n`` regex locations from the RE2-compatible grammar of SURVEY.md §8(d): literal
    segments, ``[a-z0-9]+``, ``\\d{1,4}``, alternations of <= 4, optional groups, 70 % ``^``
    anchored; 20 % ``~*`` (caseless); 5 % carry a PCRE-only construct.  Returns
    ``[(pattern, caseless, pcre_only, segments, anchored, dollar)]``; ``segments`` is the sampler's
    view of the pattern (``c3_uri``)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    W = _C3_WORDS
    out, seen = [], set()
    while len(out) < n:
        anchored = rng.random() < 0.7
        segs = []
        # unanchored patterns get >= 3 segments, every pattern >= 1 literal segment: a pattern
        # like "(/a|/b)" alone would match most URIs and end every search at once
        for _ in range(int(rng.integers(2 if anchored else 3, 6))):
            r = rng.random()
            if r < 0.45:
                segs.append(("lit", "/" + W[rng.integers(len(W))]))
            elif r < 0.6:
                segs.append(("cls", "/"))
            elif r < 0.72:
                segs.append(("dig", "/" if rng.random() < 0.6 else "-"))
            elif r < 0.87:
                k = int(rng.integers(2, 5))
                segs.append(("alt", tuple(sorted(set("/" + W[i] for i in rng.choice(len(W), k, replace=False))))))
            else:
                segs.append(("opt", "/" + W[rng.integers(len(W))]))
        if not any(k == "lit" for k, _ in segs):
            segs[int(rng.integers(len(segs)))] = ("lit", "/" + W[rng.integers(len(W))])
        if rng.random() < 0.3:
            segs.append(("ext", tuple(sorted(set(_C3_EXT[i] for i in rng.choice(len(_C3_EXT), int(rng.integers(1, 4)),
                                                                               replace=False))))))
        dollar = rng.random() < 0.5
        caseless = rng.random() < 0.2
        pcre_only = rng.random() < 0.05
        body = []
        for kind, v in segs:
            if kind == "lit":
                body.append(v)
            elif kind == "cls":
                body.append(v + "[a-z0-9]+")
            elif kind == "dig":
                body.append(v + "\\d{1,4}")
            elif kind == "alt":
                body.append("(" + "|".join(v) + ")")
            elif kind == "opt":
                body.append("(" + v + ")?")
            else:
                body.append("\\.(" + "|".join(v) + ")")
        if pcre_only:
            body.insert(int(rng.integers(0, len(body) + 1)), _C3_PCRE_ONLY[rng.integers(len(_C3_PCRE_ONLY))])
        pat = ("^" if anchored else "") + "".join(body) + ("$" if dollar else "")
        if pat in seen:
            continue
        seen.add(pat)
        out.append((pat, caseless, pcre_only, tuple(segs), anchored, dollar))
    return out


def c3_conf(regexes) -> str:
    """nginx.conf text of the C3 server: ``location ~ / ~*`` blocks in config order (regex
    locations come from custom templates / snippets), plus prefix locations."""
    ups = "".join(f"  upstream c3-u{k} {{ server 10.3.0.{k + 1}:80; }}\n" for k in range(8))
    locs = []
    for i, (pat, ci, *_r) in enumerate(regexes):
        locs.append(f'    location {"~*" if ci else "~"} "{pat}" {{ proxy_pass http://c3-u{i % 8}; }}\n')
    return ("http {\n" + ups + "  server {\n    listen 80 default_server;\n"
            f"    server_name {C3_HOST};\n"
            "    location / { proxy_pass http://c3-u0; }\n"
            "    location ^~ /static/fixed/ { proxy_pass http://c3-u1; }\n"
            "    location = /exact { return 204; }\n" + "".join(locs) + "  }\n}\n")


def c3_blob(regexes=None) -> bytes:
    return blob.make_blob(c3_conf(regexes if regexes is not None else c3_regexes()), {})


_C3_ALNUM = "abcdefghijklmnopqrstuvwxyz0123456789"


def _c3_word(rng):
    return "".join(rng.choices(_C3_ALNUM, k=rng.randint(1, 8)))


def c3_uri(rng, regexes, crafted: bool) -> str:
    """One synthetic URI of 32-256 bytes (``rng`` a ``random.Random``): a string generated from a
    random regex of the set (``crafted``) or a random path of vocabulary words and alphanumeric
    segments."""
    W = _C3_WORDS
    target = rng.randint(32, 256)
    if not crafted:
        s = ""
        while len(s) < target:
            r = rng.random()
            s += "/" + (rng.choice(W) if r < 0.5 else str(rng.randrange(99999)) if r < 0.65 else _c3_word(rng))
        if rng.random() < 0.2:
            s += "." + rng.choice(_C3_EXT)
        return s[:256]
    pat, ci, pcre_only, segs, anchored, dollar = rng.choice(regexes)
    body = ""
    for kind, v in segs:
        if kind == "lit":
            body += v
        elif kind == "cls":
            body += v + _c3_word(rng)
        elif kind == "dig":
            body += v + str(rng.randrange(10 ** rng.randint(1, 4)))
        elif kind == "alt":
            body += rng.choice(v)
        elif kind == "opt":
            body += v if rng.random() < 0.5 else ""
        else:
            body += "." + rng.choice(v)
    if ci and rng.random() < 0.5:
        body = "".join(ch.upper() if rng.random() < 0.3 else ch for ch in body)
    pre = suf = ""
    room = max(0, target - len(body))
    if not anchored:
        k = rng.randint(0, room)
        while len(pre) < k:
            pre += "/" + rng.choice(W)
        room = max(0, target - len(body) - len(pre))
    if not dollar:
        while len(suf) < room:
            suf += "/" + _c3_word(rng)
    return (pre + body + suf)[:256] or "/"


def gen_c3(n: int, regexes=None, seed: int = records.SEED_BASE + 2, pool: int = 100_000):
    """C3 requests: host regex.example.com, URIs 32-256 B, 40 % crafted to hit a regex location.
    A pool of ``min(n, pool)`` distinct URIs is generated and indexed (vectorised for 10M)."""
    regexes = regexes if regexes is not None else c3_regexes()
    import random
    rnd = random.Random(seed)
    m = min(n, pool)
    uris = [c3_uri(rnd, regexes, rnd.random() < 0.4) for _ in range(m)]
    idx = np.arange(n) if n <= m else np.random.Generator(np.random.PCG64(seed)).integers(0, m, n)
    fields = {"uri": [records.choice_seg(uris, idx)],
              "host": [records.const_seg(C3_HOST, n)],
              "method": [records.const_seg("GET", n)]}
    return records.build(n, fields, np.full(n, 80), np.zeros(n, dtype=np.int64))


C4_STRESS_POOL_SEED = records.SEED_BASE + 23


def c4_stress_generation():
    """The C4 stress variant: gpumatch.sigs.gen_waf_sigset_stress on the same
    cafe Ingress (wallarm_mode block), traffic from records.gen_c4(stress=True)."""
    ss = sigs.gen_waf_sigset_stress()
    smp = c4_sample(ss, seed=records.SEED_BASE + 43, stress=True)
    return ss, c4_blob(ss, sample=smp)
