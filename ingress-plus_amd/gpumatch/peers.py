"""Upstream peer-selection workloads.

The upstream blocks the templates render (``version1/nginx.ingress.tmpl:2-8``,
``version2/nginx.virtualserver.tmpl:2-10``): ``server <ip>:<port> max_fails=.. fail_timeout=..``
lines from the endpoints (``ingress.go:277-301``) behind every LBMethod ``ParseLBMethod`` accepts
(``parsing_helpers.go:89-161``; default ``random two least_conn``, ``config_params.go:123``), plus
the shapes the engine leaves to nginx (Plus-only methods, weights, ``$host`` keys).  Requests
vary what the balancers read: ``$remote_addr`` (IPv4, IPv6, unix), ``$request_uri``, ``$arg_*``,
``$cookie_*``, ``$http_*`` and ``$request_id``.
"""

from __future__ import annotations

import numpy as np

from . import blob, records

# (method directive, number of servers); "" = round robin
UPSTREAMS = [
    ("", 3), ("", 70), ("", 1), ("least_conn", 4), ("least_conn", 67), ("least_conn", 1),
    ("ip_hash", 5), ("ip_hash", 1), ("hash $request_uri", 6), ("hash $arg_user consistent", 7),
    ("hash $cookie_session$remote_addr", 4), ("hash ${http_x_user}-k consistent", 5),
    ("hash $request_id consistent", 64), ("random", 5), ("random two", 6), ("random two least_conn", 9),
    ("random two least_conn", 2), ("random", 1), ("random two", 1),
    ("hash $host", 3), ("least_time header", 3), ("hash $arg_user", 1), ("least_conn", 2),
]
# servers marked `down` in config: (upstream index, server index)
DOWN = {(0, 1), (3, 0), (6, 2), (9, 3), (13, 4), (15, 0), (4, 5), (4, 66)}
DEFER_WEIGHT = len(UPSTREAMS)   # one more upstream with weight=2: deferred


def _addr(u, j):
    if u == 2:
        return "unix:/var/run/nginx-502-server.sock"
    if u == 7:
        return "127.0.0.1:8181"
    return f"10.{u}.{j // 250}.{j % 250 + 1}:{8080 + (j % 3)}"


def upstream_name(u: int) -> str:
    return f"default-peers-u{u:02d}-svc-80"


def server_addrs(u: int) -> list:
    """The `server` addresses upstream u is rendered with (config order)."""
    return [_addr(u, j) for j in range(UPSTREAMS[u][1])]


def plus_order(old: list, new: list) -> list:
    """The server order of an upstream after an NGINX Plus API update from `old` to `new`
    (Manager.UpdateServersInPlus, manager.go:257-284 -> UpdateHTTPServers: the servers not listed
    are deleted, the new ones added, each appended to the peer list): the kept servers in their
    previous relative order, then the added ones in the order given -- gm_update_upstream's rule
    (parity-unpinned against a live Plus: no reference fixture covers the order)."""
    left = list(new)
    kept = []
    for a in old:
        if a in left:
            left.remove(a)
            kept.append(a)
    return kept + left


def conf_text(method: str | None = None, servers: dict | None = None, upstreams=None) -> str:
    """``method``: one LBMethod for every upstream (e.g. the default "random two least_conn").
    ``servers``: {upstream index: [address, ...]} -- the server list an NGINX Plus API update
    left (Manager.UpdateServersInPlus), rendered as a reload with those lines would be (no
    ``down``).  ``upstreams``: another (method, n) list in place of UPSTREAMS."""
    L = []
    names = []
    ups = UPSTREAMS if upstreams is None else upstreams
    for u, (m, k) in enumerate(ups):
        m = m if method is None else method
        name = upstream_name(u)
        names.append(name)
        L.append(f"upstream {name} {{")
        if m:
            L.append(f"\t{m};")
        if servers is not None and u in servers:
            for a in servers[u]:
                L.append(f"\tserver {a} max_fails=1 fail_timeout=10s;")
            L.append("\tkeepalive 32;")
            L.append("}")
            continue
        for j in range(k):
            down = " down" if (u, j) in DOWN else ""
            L.append(f"\tserver {_addr(u, j)} max_fails=1 fail_timeout=10s{down};")
        L.append("\tkeepalive 32;")
        L.append("}")
    name = upstream_name(len(ups))
    names.append(name)
    L.append(f"upstream {name} {{\n\tserver 10.99.0.1:80 weight=2;\n\tserver 10.99.0.2:80;\n}}")
    for u, name in enumerate(names):
        L.append(f"server {{\n\tlisten 80;\n\tserver_name u{u}.peers.example.com;\n"
                 f"\tlocation / {{\n\t\tproxy_pass http://{name};\n\t}}\n"
                 f"\tlocation /static/ {{\n\t\treturn 200;\n\t}}\n}}")
    return "\n".join(L) + "\n"


def peers_blob(method: str | None = None, servers: dict | None = None, upstreams=None) -> bytes:
    main = ("http {\n\tserver {\n\t\tlisten 80 default_server;\n\t\tserver_name _;\n"
            "\t\tlocation / {\n\t\t\treturn 404;\n\t\t}\n\t}\n\tinclude /etc/nginx/conf.d/*.conf;\n}\n")
    return blob.make_blob(main, {"default-peers": conf_text(method, servers, upstreams)})


def _raddrs(rng, m):
    out = []
    for _ in range(m):
        r = rng.random()
        if r < 0.6:
            out.append("%d.%d.%d.%d" % tuple(rng.integers(1, 255, 4)))
        elif r < 0.85:
            g = ["%x" % x for x in rng.integers(0, 65536, 8)]
            z = int(rng.integers(0, 4))
            out.append(":".join(g) if z == 0 else ":".join(g[:z]) + "::" + ":".join(g[z + 3:]))
        elif r < 0.9:
            out.append("::ffff:%d.%d.%d.%d" % tuple(rng.integers(1, 255, 4)))
        elif r < 0.95:
            out.append("unix:")
        else:
            out.append(["01.2.3.4", "1.2.3", "1:2::3::4", "::", "256.1.1.1", "fe80::1", ""][int(rng.integers(0, 7))])
    return out


def gen_requests(n: int, seed: int = records.SEED_BASE + 40, hot: tuple = (), upstreams=None):
    """n requests over the peers config.  ``hot``: upstream indices that get most of the traffic
    (long sequential runs for round robin / least_conn).  ``upstreams``: as for conf_text."""
    rng = np.random.default_rng(seed)
    nu = len(UPSTREAMS if upstreams is None else upstreams) + 1
    w = np.ones(nu)
    for h in hot:
        w[h] = 40.0 * nu
    w /= w.sum()
    ui = rng.choice(nu, size=n, p=w)
    hosts = [f"u{u}.peers.example.com" for u in range(nu)]
    uris = [f"/api/v{k}/item/{k * 7 % 13}" for k in range(40)] + ["/", "/static/x.css"]
    args = [""] + [f"user={k}" for k in range(25)] + [f"a=1&user=u{k}&b=2" for k in range(10)]
    ras = _raddrs(rng, 400)
    hdr_pool = []
    for k in range(60):
        h = b""
        if k % 3:
            h += f"Cookie: theme=dark; session=s{k % 17}\r\n".encode()
        if k % 4:
            h += f"X-User: user-{k % 11}\r\n".encode()
        if k % 7 == 0:
            h += b"Cookie: session=second\r\n"
        hdr_pool.append(h + b"Accept: */*\r\n")
    fields = {
        "uri": [records.choice_seg(uris, rng.integers(0, len(uris), n))],
        "args": [records.choice_seg(args, rng.integers(0, len(args), n))],
        "hdrs": [records.choice_seg(hdr_pool, rng.integers(0, len(hdr_pool), n))],
        "host": [records.choice_seg(hosts, ui)],
        "method": [records.const_seg("GET", n)],
        "raddr": [records.choice_seg(ras, rng.integers(0, len(ras), n))],
    }
    rid = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    return records.build(n, fields, np.full(n, 80), np.zeros(n, np.uint8), rid=rid,
                         remote_port=rng.integers(1024, 65535, n))


# ---------------------------------------------------------------- NGINX Plus sticky cookie
# Ingresses rendered by the Plus template (nginx-plus.ingress.tmpl:9-11) with
# nginx.com/sticky-cookie-services (annotations.go:387-399, 511-524) over three balancing methods.
STICKY_METHODS = ("round_robin", "least_conn", "random two least_conn")


def sticky_endpoints(k: int) -> list:
    return [f"10.9.{k}.{j + 1}:80" for j in range(5 + k)]


def sticky_ingresses():
    """(ingress objects, endpoints) for the sticky workload: ingress k balances svc-k with
    STICKY_METHODS[k] and sticky cookie srv_<k> (svc-x, never declared sticky, balances without);
    an invalid sticky declaration is ignored, as ParseConfigMap's log-and-ignore does."""
    ings, eps = [], {}
    for k, m in enumerate(STICKY_METHODS):
        ann = {"nginx.org/lb-method": m,
               "nginx.com/sticky-cookie-services": f"serviceName=svc-{k} srv_{k} expires=1h path=/;bad-entry"}
        ings.append({"metadata": {"name": f"sticky{k}", "namespace": "default", "annotations": ann},
                     "spec": {"rules": [{"host": f"s{k}.example.com", "http": {"paths": [
                         {"path": "/", "backend": {"serviceName": f"svc-{k}", "servicePort": 80}},
                         {"path": "/x", "backend": {"serviceName": "svc-x", "servicePort": 80}}]}}]}})
        eps[f"svc-{k}80"] = sticky_endpoints(k)
    eps["svc-x80"] = ["10.9.9.1:80", "10.9.9.2:80"]
    return ings, eps


def sticky_blob() -> bytes:
    from . import confgen
    ings, eps = sticky_ingresses()
    return blob.make_blob(confgen.render_main(), confgen.ingress_files(ings, endpoints=eps, is_plus=True))


def sticky_requests(n: int, seed: int = records.SEED_BASE + 77, down=()):
    """Requests to the sticky ingresses with a srv_<k> cookie that names a peer (its hex MD5), a
    down peer, another upstream's peer, no peer (stale), an uppercase or short value, or none."""
    import hashlib
    rng = np.random.Generator(np.random.PCG64(seed))
    items = []
    for i in range(n):
        k = int(rng.integers(0, len(STICKY_METHODS)))
        eps = sticky_endpoints(k)
        r = int(rng.integers(0, 10))
        hx = hashlib.md5(eps[int(rng.integers(0, len(eps)))].encode()).hexdigest()
        cookie = {0: hx, 1: hx, 2: hx, 3: hashlib.md5(b"10.9.9.1:80").hexdigest(), 4: "0" * 32, 5: hx.upper(),
                  6: hx[:31], 7: None, 8: hx, 9: hx}[r]
        hdrs = []
        if cookie is not None:
            name = f"srv_{k}" if r != 9 else f"srv_{(k + 1) % len(STICKY_METHODS)}"   # another upstream's cookie
            hdrs.append(("Cookie", f"a=b; {name}={cookie}" if rng.random() < 0.5 else f"{name}={cookie}"))
        uri = "/x" if rng.random() < 0.1 else "/"
        items.append({"host": f"s{k}.example.com", "uri": uri, "headers": hdrs, "port": 80,
                      "rid": bytes(rng.integers(0, 256, 16, dtype=np.uint8)), "raddr": f"10.200.{i % 200}.{i % 250 + 1}"})
    return records.from_dicts(items)
