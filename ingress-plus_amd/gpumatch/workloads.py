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


def c4_sample(sigset: sigs.SigSet, n: int = 2000, seed: int = records.SEED_BASE + 33) -> bytes:
    """A benign traffic sample for the WAF prefilter tuning (GM_ENTRY_SAMPLE): C4 requests from a
    seed disjoint from every pool the tests and the bench match (a deployment samples its own
    recent traffic the same way); the zone bytes only."""
    reqs, arena = records.gen_c4(n, sigset, seed=seed, plant_rate=0.0, pool_mb=2)
    parts = []
    for r in reqs:
        b = int(r["base"])
        z = int(r["uri_len"]) + int(r["args_len"]) + int(r["hdr_len"]) + int(r["body_len"])
        parts.append(arena[b:b + z].tobytes())
    return b"".join(parts)


def c4_blob(sigset: sigs.SigSet, mode: str = "block", sample: bytes | None = None) -> bytes:
    base = confgen.default_config_params()
    base["MainEnableWallarm"] = True
    ing = copy.deepcopy(CAFE_INGRESS)
    ing["metadata"]["annotations"] = {"wallarm.com/mode": mode}
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
