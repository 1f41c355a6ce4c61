"""Rule-set shaping: Ingress / VirtualServer -> typed config -> nginx config text.

This is the fixture side of SURVEY.md §8 row A12: a Python restatement of the
reference Configurator's config *generation*, so that the engine can be fed
exactly the nginx text the reference would hand to ``nginx.Manager.CreateConfig``.
It is host tooling (used by tests, bench and the sample Manager), not part of the
device path.

Restated reference code (wallarm/ingress-plus 1.5.5-wallarm-r1):

* ``internal/configs/config_params.go:107-141``  NewDefaultConfigParams
* ``internal/configs/annotations.go:57-333``     parseAnnotations (verdict-affecting keys)
* ``internal/configs/ingress.go:47-231``         generateNginxCfg
* ``internal/configs/ingress.go:233-252``        createLocation
* ``internal/configs/ingress.go:329-362``        pathOrDefault / getNameForUpstream / upstreamMapToSlice
* ``internal/configs/ingress.go:364-432``        generateNginxCfgForMergeableIngresses
* ``internal/configs/virtualserver.go:41-82``    upstream / variable namers
* ``internal/configs/virtualserver.go:84-196``   generateVirtualServerConfig
* ``internal/configs/virtualserver.go:250-442``  split / rules / map-value generation
* ``internal/configs/virtualserver.go:444-472``  generateSSLConfig
* ``internal/configs/configurator.go:172-190,556-571`` TLS pem names, conf.d file names
* ``internal/k8s/controller.go:1827-1886``       getMinionsForMaster (path dedupe, first wins)
* ``internal/k8s/controller.go:1519-1591``       createVirtualServer (VSR resolution + endpoints)
* ``pkg/apis/configuration/validation/validation.go:15-476`` ValidateVirtualServer /
  ValidateVirtualServerRouteForVirtualServer (the legal input domain: what never reaches nginx)
* templates ``version1/nginx.ingress.tmpl``, ``version1/nginx.tmpl:81-129``,
  ``version2/nginx.virtualserver.tmpl`` -- rendered here by ``render_*``; only the
  directive *sequence* matters to the engine, whitespace is free.

Typed configs are plain dicts whose keys follow the Go struct field names, so the
Go unit tests' expected structs can be transcribed 1:1 into ``tests/golden``.
"""

from __future__ import annotations

import copy
import re

PEM_MISSING = "/etc/nginx/secrets/default"      # configurator.go:19
PEM_WILDCARD = "/etc/nginx/secrets/wildcard"    # configurator.go:20
NGINX502_SERVER = "unix:/var/run/nginx-502-server.sock"  # virtualserver.go:14


# --------------------------------------------------------------------------- params

def default_config_params() -> dict:
    """config_params.go:107-141 (verdict-relevant subset plus template fields)."""
    return {
        "ServerTokens": "on",
        "ProxyConnectTimeout": "60s",
        "ProxyReadTimeout": "60s",
        "ClientMaxBodySize": "1m",
        "SSLRedirect": True,
        "RedirectToHTTPS": False,
        "HTTP2": False,
        "ProxyProtocol": False,
        "ProxyBuffering": True,
        "ProxyBuffers": "",
        "ProxyBufferSize": "",
        "ProxyMaxTempFileSize": "",
        "Ports": [80],
        "SSLPorts": [443],
        "MaxFails": 1,
        "FailTimeout": "10s",
        "LBMethod": "random two least_conn",
        "Keepalive": 0,
        "HealthStatus": False,
        "MainEnableWallarm": False,
        "Wallarm": None,
        "ServerSnippets": [],
        "LocationSnippets": [],
        # realip (config_params.go:60-62, ConfigMap set-real-ip-from / real-ip-header /
        # real-ip-recursive, configmaps.go:153-169)
        "SetRealIPFrom": [], "RealIPHeader": "", "RealIPRecursive": False,
        "HSTS": False, "HSTSMaxAge": 2592000, "HSTSIncludeSubdomains": False, "HSTSBehindProxy": False,
        # the status server of the main template (nginx.tmpl:104-125), from the controller's flags:
        # -nginx-status (default true), -nginx-status-port (8080), -nginx-status-allow-cidrs
        # ("127.0.0.1"), and -enable-prometheus-metrics (false) for the unix-socket one
        # (cmd/nginx-ingress/main.go:108-113, 329-332)
        "NginxStatus": True, "NginxStatusPort": 8080, "NginxStatusAllowCIDRs": ["127.0.0.1"],
        "StubStatusOverUnixSocketForOSS": False,
    }


def new_wallarm() -> dict:
    """version1/config.go:208-222 NewWallarm."""
    return {"Mode": "off", "ModeAllowOverride": "on", "Fallback": "on", "Instance": "",
            "BlockPage": "", "ParseResponse": "on", "ParseWebsocket": "off",
            "UnpackResponse": "on", "ParserDisable": []}


def _as_bool(v):
    s = str(v).strip().lower()
    if s in ("true", "1", "t"):
        return True
    if s in ("false", "0", "f"):
        return False
    return None  # GetMapKeyAsBool error -> ignored (annotations.go logs and keeps default)


# --------------------------------------------------------------------------- load balancing

_LB_VALID = {"least_conn", "ip_hash", "random", "random two", "random two least_conn"}   # parsing_helpers.go:109-115
_LB_VALID_PLUS = _LB_VALID | {"random two least_time=header", "random two least_time=last_byte",
                              "least_time header", "least_time last_byte", "least_time header inflight",
                              "least_time last_byte inflight"}                          # :117-129


def _validate_hash_lb_method(method: str) -> str:
    """parsing_helpers.go:152-161: "hash <key>" or "hash <key> consistent" (split on single spaces)."""
    kw = method.split(" ")
    if kw[0] == "hash" and (len(kw) == 2 or (len(kw) == 3 and kw[2] == "consistent")):
        return method
    raise ValueError(f"Invalid load balancing method: {method!r}")


def parse_lb_method(method: str, plus: bool = False) -> str:
    """ParseLBMethod / ParseLBMethodForPlus (parsing_helpers.go:89-150): the directive the upstream
    block renders ("" = nginx's default round robin); ValueError for an invalid method."""
    method = method.strip(" \t\n\r\v\f")   # strings.TrimSpace
    if method == "round_robin":
        return ""
    if method.startswith("hash"):
        return _validate_hash_lb_method(method)
    if method in (_LB_VALID_PLUS if plus else _LB_VALID):
        return method
    raise ValueError(f"Invalid load balancing method: {method!r}")


_GO_INT = re.compile(r"[+-]?[0-9]+")


def _go_atoi(v):
    """strconv.Atoi / ParseInt(s, 10, 64) (GetMapKeyAsInt / GetMapKeyAsInt64): None on error."""
    s = str(v)
    return int(s) if _GO_INT.fullmatch(s) else None


def _string_slice(v, sep):
    """parsing_helpers.go:80-87 GetMapKeyAsStringSlice: strings.Split(value, sep)."""
    return str(v).split(sep)


def parse_annotations(ing: dict, base: dict) -> dict:
    """annotations.go:57-333, restricted to keys that change the request verdict:
    redirect-to-https (:176-182), ssl-redirect (:184-190), listen ports (:266-273),
    wallarm.* (:294-330).  Timeouts/buffers/etc. only feed non-verdict directives."""
    ann = (ing.get("metadata") or {}).get("annotations") or {}
    p = copy.deepcopy(base)
    if "nginx.org/redirect-to-https" in ann:
        b = _as_bool(ann["nginx.org/redirect-to-https"])
        if b is not None:
            p["RedirectToHTTPS"] = b
    if "ingress.kubernetes.io/ssl-redirect" in ann:
        b = _as_bool(ann["ingress.kubernetes.io/ssl-redirect"])
        if b is not None:
            p["SSLRedirect"] = b
    if "nginx.org/lb-method" in ann:   # annotations.go:60-74 (OSS: ParseLBMethod; errors keep the base)
        try:
            p["LBMethod"] = parse_lb_method(str(ann["nginx.org/lb-method"]), plus=False)
        except ValueError:
            pass
    if "nginx.org/keepalive" in ann:   # annotations.go:275-281
        v = _go_atoi(ann["nginx.org/keepalive"])
        if v is not None:
            p["Keepalive"] = v
    if "nginx.org/max-fails" in ann:   # annotations.go:283-289
        v = _go_atoi(ann["nginx.org/max-fails"])
        if v is not None:
            p["MaxFails"] = v
    if "nginx.org/fail-timeout" in ann:   # annotations.go:291-293
        p["FailTimeout"] = ann["nginx.org/fail-timeout"]
    # annotations.go:132-146 (GetMapKeyAsStringSlice with "\n")
    for key, field in (("nginx.org/server-snippets", "ServerSnippets"), ("nginx.org/location-snippets", "LocationSnippets")):
        if key in ann:
            p[field] = _string_slice(ann[key], "\n")
    if "nginx.org/client-max-body-size" in ann:
        p["ClientMaxBodySize"] = ann["nginx.org/client-max-body-size"]
    for key, field in (("nginx.org/listen-ports", "Ports"), ("nginx.org/listen-ports-ssl", "SSLPorts")):
        if key in ann:
            ports = []
            for v in str(ann[key]).split(","):
                try:
                    port = int(v)
                except ValueError:
                    continue
                if 1 <= port <= 65535:
                    ports.append(port)
            if ports:
                p[field] = ports
    if p["MainEnableWallarm"]:
        w = new_wallarm()
        for k, f in (("wallarm.com/mode", "Mode"), ("wallarm.com/mode-allow-override", "ModeAllowOverride"),
                     ("wallarm.com/fallback", "Fallback"), ("wallarm.com/instance", "Instance"),
                     ("wallarm.com/block-page", "BlockPage"), ("wallarm.com/parse-response", "ParseResponse"),
                     ("wallarm.com/parse-websocket", "ParseWebsocket"),
                     ("wallarm.com/unpack-response", "UnpackResponse")):
            if k in ann:
                w[f] = ann[k]
        if "wallarm.com/parser-disable" in ann:
            w["ParserDisable"] = [s.strip() for s in str(ann["wallarm.com/parser-disable"]).split(",")]
        p["Wallarm"] = w
    return p


# --------------------------------------------------------------------------- Ingress

def _meta(obj):
    m = obj.get("metadata") or {}
    return m.get("namespace", "default"), m["name"]


def object_meta_to_file_name(obj) -> str:
    """configurator.go:560-562."""
    ns, name = _meta(obj)
    return f"{ns}-{name}"


def _svc_port(backend) -> str:
    return str(backend["servicePort"])


def get_name_for_upstream(ing, host, backend) -> str:
    """ingress.go:336-338."""
    ns, name = _meta(ing)
    return f"{ns}-{name}-{host}-{backend['serviceName']}-{_svc_port(backend)}"


def path_or_default(path) -> str:
    """ingress.go:329-334."""
    return path if path else "/"


def parse_sticky_service(service: str):
    """annotations.go:511-524 parseStickyService: "serviceName=<svc> <cookie spec>" ->
    (service, cookie spec); ValueError for a bad declaration."""
    parts = service.split(" ", 1)
    if len(parts) != 2:
        raise ValueError(f"Invalid sticky-cookie service format: {service}")
    name_parts = parts[0].split("=")
    if len(name_parts) != 2:
        raise ValueError(f"Invalid sticky-cookie service format: {name_parts}")
    return name_parts[1], parts[1]


def get_session_persistence_services(ing: dict) -> dict:
    """annotations.go:387-399: nginx.com/sticky-cookie-services split on ";" (a bad entry is logged
    and ignored)."""
    out = {}
    v = ((ing.get("metadata") or {}).get("annotations") or {}).get("nginx.com/sticky-cookie-services")
    if v is not None:
        for svc in str(v).split(";"):
            try:
                name, sticky = parse_sticky_service(svc)
            except ValueError:
                continue
            out[name] = sticky
    return out


def _create_upstream(ing_ex, name, backend, p, sticky=""):
    """ingress.go:266-305: default server 127.0.0.1:8181 when no endpoints (version1/config.go:
    194-206); under NGINX Plus the service's sticky cookie (ingress.go:272)."""
    ups = {"Name": name, "UpstreamServers": [{"Address": "127.0.0.1", "Port": "8181",
                                              "MaxFails": 1, "FailTimeout": "10s"}],
           "LBMethod": p["LBMethod"], "StickyCookie": sticky}
    key = backend["serviceName"] + _svc_port(backend)
    endps = (ing_ex.get("Endpoints") or {}).get(key)
    if endps:
        ups["UpstreamServers"] = [{"Address": e.split(":")[0], "Port": e.split(":")[1],
                                   "MaxFails": p["MaxFails"], "FailTimeout": p["FailTimeout"]} for e in endps]
    return ups


def parse_rewrites(service: str):
    """annotations.go:526-544 parseRewrites: "serviceName=<svc> rewrite=<path>" -> (svc, path);
    ValueError on any other shape (strings.TrimSpace, SplitN(" ", 2), Split("="))."""
    parts = service.strip(" \t\n\r\v\f").split(" ", 1)
    if len(parts) != 2:
        raise ValueError(f"Invalid rewrite format: {service}")
    svc = parts[0].split("=")
    if len(svc) != 2:
        raise ValueError(f"Invalid rewrite format: {svc}")
    rw = parts[1].split("=")
    if len(rw) != 2:
        raise ValueError(f"Invalid rewrite format: {rw}")
    return svc[1], rw[1]


def get_rewrites(ing: dict) -> dict:
    """annotations.go:347-361 getRewrites: nginx.org/rewrites, ';'-separated; invalid entries are
    logged and skipped."""
    ann = (ing.get("metadata") or {}).get("annotations") or {}
    out = {}
    if "nginx.org/rewrites" in ann:
        for svc in str(ann["nginx.org/rewrites"]).split(";"):
            try:
                name, rw = parse_rewrites(svc)
            except ValueError:
                continue
            out[name] = rw
    return out


def _create_location(path, upstream, p, rewrite=""):
    """ingress.go:233-252 (Rewrite: the URI part of proxy_pass, version1/nginx.ingress.tmpl:194-196)."""
    return {"Path": path, "Upstream": upstream, "ProxyConnectTimeout": p["ProxyConnectTimeout"],
            "ProxyReadTimeout": p["ProxyReadTimeout"], "ClientMaxBodySize": p["ClientMaxBodySize"],
            "Rewrite": rewrite, "SSL": False, "GRPC": False, "Websocket": False,
            "ProxyBuffering": p["ProxyBuffering"], "Wallarm": None, "MinionIngress": None,
            "LocationSnippets": list(p["LocationSnippets"])}


def generate_nginx_cfg(ing_ex: dict, pems: dict, is_minion: bool, base: dict, is_plus: bool = False) -> dict:
    """ingress.go:47-231 generateNginxCfg (no JWT/health-check/grpc paths; is_plus: the session
    persistence services, ingress.go:50)."""
    ing = ing_ex["Ingress"]
    p = parse_annotations(ing, base)
    sp = get_session_persistence_services(ing) if is_plus else {}
    rewrites = get_rewrites(ing)   # ingress.go:51
    spec = ing.get("spec") or {}
    upstreams = {}
    default_backend = spec.get("backend")
    if default_backend is not None:
        name = get_name_for_upstream(ing, "", default_backend)
        upstreams[name] = _create_upstream(ing_ex, name, default_backend, p, sp.get(default_backend["serviceName"], ""))
    servers = []
    for rule in spec.get("rules") or []:
        if not rule.get("http"):
            continue
        host = rule.get("host", "")
        server = {"Name": host, "ServerTokens": p["ServerTokens"], "HTTP2": p["HTTP2"],
                  "RedirectToHTTPS": p["RedirectToHTTPS"], "SSLRedirect": p["SSLRedirect"],
                  "ProxyProtocol": p["ProxyProtocol"], "HSTS": p["HSTS"], "HSTSMaxAge": p["HSTSMaxAge"],
                  "HSTSIncludeSubdomains": p["HSTSIncludeSubdomains"], "HSTSBehindProxy": p["HSTSBehindProxy"],
                  "StatusZone": host,
                  "Ports": list(p["Ports"]), "SSLPorts": list(p["SSLPorts"]), "Wallarm": p["Wallarm"],
                  "SSL": False, "SSLCertificate": "", "SSLCertificateKey": "", "SSLCiphers": "",
                  "GRPCOnly": False, "ServerSnippets": list(p["ServerSnippets"]),
                  # ingress.go:100-102
                  "RealIPHeader": p["RealIPHeader"], "SetRealIPFrom": list(p["SetRealIPFrom"]),
                  "RealIPRecursive": p["RealIPRecursive"]}
        if host in pems:
            pem = pems[host]
            server.update(SSL=True, SSLCertificate=pem, SSLCertificateKey=pem)
            if pem == PEM_MISSING:
                server["SSLCiphers"] = "NULL"
        locations = []
        root = False
        for path in rule["http"].get("paths") or []:
            be = path["backend"]
            ups_name = get_name_for_upstream(ing, host, be)
            if ups_name not in upstreams:
                upstreams[ups_name] = _create_upstream(ing_ex, ups_name, be, p, sp.get(be["serviceName"], ""))
            loc = _create_location(path_or_default(path.get("path", "")), upstreams[ups_name], p,
                                   rewrites.get(be["serviceName"], ""))
            locations.append(loc)
            if loc["Path"] == "/":
                root = True
        if not root and default_backend is not None:
            ups_name = get_name_for_upstream(ing, "", default_backend)
            locations.append(_create_location("/", upstreams[ups_name], p,
                                              rewrites.get(default_backend["serviceName"], "")))
        server["Locations"] = locations
        servers.append(server)
    ns, name = _meta(ing)
    return {"Upstreams": [upstreams[k] for k in sorted(upstreams)], "Servers": servers,
            "Keepalive": str(p["Keepalive"]) if p["Keepalive"] > 0 else "",
            "Ingress": {"Name": name, "Namespace": ns,
                        "Annotations": (ing.get("metadata") or {}).get("annotations") or {}}}


# annotations.go:17-55
MASTER_DENY = ("nginx.org/rewrites", "nginx.org/ssl-services", "nginx.org/grpc-services",
               "nginx.org/websocket-services", "nginx.com/sticky-cookie-services",
               "nginx.com/health-checks", "nginx.com/health-checks-mandatory",
               "nginx.com/health-checks-mandatory-queue")
MINION_DENY = ("nginx.org/proxy-hide-headers", "nginx.org/proxy-pass-headers", "nginx.org/redirect-to-https",
               "ingress.kubernetes.io/ssl-redirect", "nginx.org/hsts", "nginx.org/hsts-max-age",
               "nginx.org/hsts-include-subdomains", "nginx.org/server-tokens", "nginx.org/listen-ports",
               "nginx.org/listen-ports-ssl", "nginx.org/server-snippets")
MINION_INHERIT = ("nginx.org/proxy-connect-timeout", "nginx.org/proxy-read-timeout",
                  "nginx.org/client-max-body-size", "nginx.org/proxy-buffering", "nginx.org/proxy-buffers",
                  "nginx.org/proxy-buffer-size", "nginx.org/proxy-max-temp-file-size",
                  "nginx.org/location-snippets", "nginx.org/lb-method", "nginx.org/keepalive",
                  "nginx.org/max-fails", "nginx.org/fail-timeout")


def get_minions_for_master(master: dict, candidates: list) -> list:
    """controller.go:1827-1886: minions with the master's host, oldest first; a path that an
    earlier minion already claimed is dropped (first wins, :1860-1871)."""
    host = master["spec"]["rules"][0]["host"]
    mins = [m for m in candidates if (m.get("spec") or {}).get("rules")
            and m["spec"]["rules"][0].get("host") == host]
    mins.sort(key=lambda m: (m["metadata"].get("creationTimestamp", ""), _meta(m)))
    seen = set()
    out = []
    for m in mins:
        m = copy.deepcopy(m)
        paths = []
        for pth in m["spec"]["rules"][0]["http"]["paths"]:
            if pth.get("path", "") in seen:
                continue
            seen.add(pth.get("path", ""))
            paths.append(pth)
        m["spec"]["rules"][0]["http"]["paths"] = paths
        if paths:
            out.append(m)
    return out


def generate_nginx_cfg_for_mergeable(master_ex: dict, minion_exs: list, master_pems: dict, base: dict) -> dict:
    """ingress.go:364-432 generateNginxCfgForMergeableIngresses."""
    master_ex = copy.deepcopy(master_ex)
    # controller.go:1933-1936: the master gets an empty path list so createIngress accepts it
    master_ex["Ingress"]["spec"]["rules"][0]["http"] = {"paths": []}
    mann = master_ex["Ingress"]["metadata"].setdefault("annotations", {})
    for k in MASTER_DENY:
        mann.pop(k, None)
    mcfg = generate_nginx_cfg(master_ex, master_pems, False, base)
    server = mcfg["Servers"][0]
    upstreams = list(mcfg["Upstreams"])
    locations = []
    for mx in minion_exs:
        mx = copy.deepcopy(mx)
        mx["Ingress"]["spec"].pop("backend", None)
        ann = mx["Ingress"]["metadata"].setdefault("annotations", {})
        for k in MINION_INHERIT:          # mergeMasterAnnotationsIntoMinion (annotations.go:439-465)
            if k in mann and k not in ann:
                ann[k] = mann[k]
        for k in MINION_DENY:             # filterMinionAnnotations (annotations.go:431-437)
            ann.pop(k, None)
        cfg = generate_nginx_cfg(mx, {}, True, base)
        for s in cfg["Servers"]:
            for loc in s["Locations"]:
                loc = dict(loc)
                loc["MinionIngress"] = cfg["Ingress"]   # Location.Wallarm is never set (ingress.go)
                locations.append(loc)
        upstreams.extend(cfg["Upstreams"])
    server["Locations"] = locations
    return {"Servers": [server], "Upstreams": upstreams, "Keepalive": mcfg["Keepalive"],
            "Ingress": mcfg["Ingress"]}


def tls_pems(ing: dict, wildcard: bool = False, secrets=()) -> dict:
    """configurator.go:172-190 updateTLSSecrets."""
    pems = {}
    ns, _ = _meta(ing)
    for tls in (ing.get("spec") or {}).get("tls") or []:
        sn = tls.get("secretName", "")
        pem = PEM_MISSING
        if sn == "" and wildcard:
            pem = PEM_WILDCARD
        elif sn in secrets:
            pem = f"/etc/nginx/secrets/{ns}-{sn}"
        for h in tls.get("hosts") or []:
            pems[h] = pem
    return pems


# --------------------------------------------------------------------------- VirtualServer

def _vs_upstream_prefix(vs):
    ns, name = _meta(vs)
    return f"vs_{ns}_{name}"


def _vsr_upstream_prefix(vs, vsr):
    ns, name = _meta(vs)
    rns, rname = _meta(vsr)
    return f"vs_{ns}_{name}_vsr_{rns}_{rname}"


def _safe_ns_name(vs):
    ns, name = _meta(vs)
    return f"{ns}_{name}".replace("-", "_")


SPECIAL_MAP_PARAMS = ("default", "hostnames", "include", "volatile")


def generate_value_for_rules_route_map(v: str):
    """virtualserver.go:387-402."""
    if len(v) == 0:
        return '""', False
    neg = False
    if v[0] == "!":
        neg = True
        v = v[1:]
    if v in SPECIAL_MAP_PARAMS:
        return "\\" + v, neg
    return f'"{v}"', neg


def generate_parameters_for_rules_route_map(v: str, ok: str):
    """virtualserver.go:404-426."""
    value, neg = generate_value_for_rules_route_map(v)
    vr, dr = (ok, "0") if not neg else ("0", ok)
    return [{"Value": value, "Result": vr}, {"Value": "default", "Result": dr}]


def source_for_condition(c: dict) -> str:
    """virtualserver.go:428-442."""
    if c.get("header"):
        return "$http_" + c["header"].replace("-", "_")
    if c.get("cookie"):
        return "$cookie_" + c["cookie"]
    if c.get("argument"):
        return "$arg_" + c["argument"]
    return c.get("variable", "")


def _vs_location(path, ups, p):
    """virtualserver.go:231-245 generateLocation."""
    return {"Path": path, "ProxyConnectTimeout": p["ProxyConnectTimeout"],
            "ProxyReadTimeout": p["ProxyReadTimeout"], "ClientMaxBodySize": p["ClientMaxBodySize"],
            "ProxyBuffering": p["ProxyBuffering"], "ProxyPass": f"http://{ups}",
            "Snippets": list(p["LocationSnippets"])}                    # virtualserver.go:231


def generate_split_route_config(route, prefix, safe, index, p):
    """virtualserver.go:250-291."""
    var = f"$vs_{safe}_splits_{index}"
    dists = [{"Weight": f"{s['weight']}%", "Value": f"@splits_{index}_split_{i}"}
             for i, s in enumerate(route["splits"])]
    locs = [_vs_location(f"@splits_{index}_split_{i}", f"{prefix}_{s['upstream']}", p)
            for i, s in enumerate(route["splits"])]
    return {"SplitClient": {"Source": "$request_id", "Variable": var, "Distributions": dists},
            "Locations": locs, "InternalRedirectLocation": {"Path": route["path"], "Destination": var}}


def generate_rules_route_config(route, prefix, safe, index, p):
    """virtualserver.go:299-378."""
    rules = route["rules"]
    conds = rules["conditions"]
    maps = []
    for i, m in enumerate(rules["matches"]):
        for j, c in enumerate(conds):
            ok = "1"
            if j < len(m["values"]) - 1:
                ok = f"$vs_{safe}_rules_{index}_match_{i}_cond_{j + 1}"
            maps.append({"Source": source_for_condition(c),
                         "Variable": f"$vs_{safe}_rules_{index}_match_{i}_cond_{j}",
                         "Parameters": generate_parameters_for_rules_route_map(m["values"][j], ok)})
    src = "".join(f"$vs_{safe}_rules_{index}_match_{i}_cond_0" for i in range(len(rules["matches"])))
    params = [{"Value": "~^" + "0" * i + "1", "Result": f"@rules_{index}_match_{i}"}
              for i in range(len(rules["matches"]))]
    params.append({"Value": "default", "Result": f"@rules_{index}_default"})
    var = f"$vs_{safe}_rules_{index}"
    maps.append({"Source": src, "Variable": var, "Parameters": params})
    locs = [_vs_location(f"@rules_{index}_match_{i}", f"{prefix}_{m['upstream']}", p)
            for i, m in enumerate(rules["matches"])]
    locs.append(_vs_location(f"@rules_{index}_default", f"{prefix}_{rules['defaultUpstream']}", p))
    return {"Maps": maps, "Locations": locs,
            "InternalRedirectLocation": {"Path": route["path"], "Destination": var}}


def generate_ssl_config(tls, pem_name, p):
    """virtualserver.go:444-472."""
    if not tls or not tls.get("secret"):
        return None
    name, ciphers = (pem_name, "") if pem_name else (PEM_MISSING, "NULL")
    return {"HTTP2": p["HTTP2"], "Certificate": name, "CertificateKey": name, "Ciphers": ciphers,
            "RedirectToHTTPS": p["SSLRedirect"]}


def generate_virtual_server_config(vs_ex: dict, pem_name: str, base: dict) -> dict:
    """virtualserver.go:84-196 (OSS)."""
    vs = vs_ex["VirtualServer"]
    spec = vs["spec"]
    p = base
    prefix = _vs_upstream_prefix(vs)
    safe = _safe_ns_name(vs)
    ups = []

    def mk_ups(name, ns, u):
        key = f"{ns}/{u['service']}:{u['port']}"
        eps = (vs_ex.get("Endpoints") or {}).get(key) or []
        servers = [{"Address": e, "MaxFails": p["MaxFails"], "FailTimeout": p["FailTimeout"]} for e in eps]
        if not servers:
            servers = [{"Address": NGINX502_SERVER, "MaxFails": p["MaxFails"], "FailTimeout": p["FailTimeout"]}]
        return {"Name": name, "Servers": servers, "LBMethod": p["LBMethod"]}

    vns, _ = _meta(vs)
    for u in spec.get("upstreams") or []:
        ups.append(mk_ups(f"{prefix}_{u['name']}", vns, u))
    vsrs = vs_ex.get("VirtualServerRoutes") or []
    for vsr in vsrs:
        rpre = _vsr_upstream_prefix(vs, vsr)
        rns, _ = _meta(vsr)
        for u in vsr["spec"].get("upstreams") or []:
            ups.append(mk_ups(f"{rpre}_{u['name']}", rns, u))
    locations, irls, splits, maps = [], [], [], []
    rules_routes = 0

    def add(r, pre):
        nonlocal rules_routes
        if r.get("splits"):
            cfg = generate_split_route_config(r, pre, safe, len(splits), p)
            splits.append(cfg["SplitClient"])
            locations.extend(cfg["Locations"])
            irls.append(cfg["InternalRedirectLocation"])
        elif r.get("rules") is not None:
            cfg = generate_rules_route_config(r, pre, safe, rules_routes, p)
            maps.extend(cfg["Maps"])
            locations.extend(cfg["Locations"])
            irls.append(cfg["InternalRedirectLocation"])
            rules_routes += 1
        else:
            locations.append(_vs_location(r["path"], f"{pre}_{r['upstream']}", p))

    for r in spec.get("routes") or []:
        if r.get("route"):
            continue
        add(r, prefix)
    for vsr in vsrs:
        rpre = _vsr_upstream_prefix(vs, vsr)
        for r in vsr["spec"].get("subroutes") or []:
            add(r, rpre)
    return {"Upstreams": ups, "SplitClients": splits, "Maps": maps,
            "Server": {"ServerName": spec["host"], "ProxyProtocol": p["ProxyProtocol"],
                       # virtualserver.go:187-189
                       "SetRealIPFrom": list(p["SetRealIPFrom"]), "RealIPHeader": p["RealIPHeader"],
                       "RealIPRecursive": p["RealIPRecursive"],
                       "SSL": generate_ssl_config(spec.get("tls"), pem_name, p),
                       "RedirectToHTTPSBasedOnXForwarderProto": p["RedirectToHTTPS"],
                       "ServerTokens": p["ServerTokens"], "Snippets": list(p["ServerSnippets"]),
                       "InternalRedirectLocations": irls, "Locations": locations},
            "Keepalive": str(p["Keepalive"]) if p["Keepalive"] > 0 else ""}


# --------------------------------------------------------------------------- validation
# pkg/apis/configuration/validation/validation.go: a VirtualServer (or a VirtualServerRoute for its
# VirtualServer) that fails validation is never rendered -- the controller deletes its config
# (controller.go:608-617) or skips the VSR (controller.go:1572-1577).  Each check returns a list
# of error strings (empty = valid), like the Go field.ErrorList.

_DNS1123_LABEL = r"[a-z0-9]([-a-z0-9]*[a-z0-9])?"
_DNS1123_SUBDOMAIN = re.compile(r"^" + _DNS1123_LABEL + r"(\." + _DNS1123_LABEL + r")*$")
_DNS1035_LABEL = re.compile(r"^[a-z]([-a-z0-9]*[a-z0-9])?$")
_QUALIFIED_NAME = re.compile(r"^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$")
_HTTP_HEADER_NAME = re.compile(r"^[-A-Za-z0-9]+$")
_PATH = re.compile(r"^/[^\s{};]*$")                      # validation.go:244-263 pathFmt
_COOKIE_ARG = re.compile(r"^[_A-Za-z0-9]+$")             # validation.go:327-349
_MATCH_VALUE = re.compile(r'^([^"\\]|\\.)*$', re.S)      # validation.go:381-398 matchValueFmt
VALID_VARIABLE_NAMES = frozenset(("$args", "$http2", "$https", "$remote_addr", "$remote_port", "$query_string",
                                  "$request", "$request_body", "$request_uri", "$request_method", "$scheme"))


def _is_dns1123_subdomain(s):
    return len(s) <= 253 and bool(_DNS1123_SUBDOMAIN.match(s))


def _is_dns1035_label(s):
    return len(s) <= 63 and bool(_DNS1035_LABEL.match(s))


def _is_qualified_name(s):
    """k8s IsQualifiedName: [prefix/]name, prefix a DNS-1123 subdomain, name <= 63."""
    parts = s.split("/")
    if len(parts) == 2:
        prefix, name = parts
        if not prefix or not _is_dns1123_subdomain(prefix):
            return False
    elif len(parts) == 1:
        name = parts[0]
    else:
        return False
    return 0 < len(name) <= 63 and bool(_QUALIFIED_NAME.match(name))


def validate_host(host):
    if host == "":
        return ["host: Required"]
    return [] if _is_dns1123_subdomain(host) else [f"host {host!r}: not a DNS-1123 subdomain"]


def validate_path(path):
    """validation.go:244-263."""
    if path == "":
        return ["path: Required"]
    return [] if _PATH.match(path) else [f"path {path!r}: must start with / and have no whitespace, {{, }} or ;"]


def is_valid_match_value(value):
    """validation.go:390-398: every '"' escaped, no trailing unescaped '\\'."""
    return [] if _MATCH_VALUE.match(value) else [f"value {value!r}: unescaped quote or trailing backslash"]


def _validate_name_1035(name, what):
    if name == "":
        return [f"{what}: Required"]
    return [] if _is_dns1035_label(name) else [f"{what} {name!r}: not a DNS-1035 label"]


def validate_upstreams(upstreams):
    """validation.go:76-100 -> (errors, names)."""
    errs, names = [], set()
    for u in upstreams or []:
        e = _validate_name_1035(u.get("name", ""), "upstream name")
        if e:
            errs += e
        elif u["name"] in names:
            errs.append(f"upstream name {u['name']!r}: Duplicate")
        else:
            names.add(u["name"])
        errs += _validate_name_1035(u.get("service", ""), "service")
        port = u.get("port", 0)
        if not (isinstance(port, int) and 1 <= port <= 65535):
            errs.append(f"port {port!r}: not a valid port number")
    return errs, names


def _validate_referenced_upstream(name, names):
    e = _validate_name_1035(name or "", "upstream")
    if e:
        return e
    return [] if name in names else [f"upstream {name!r}: Not found"]


def validate_splits(splits, names):
    """validation.go:216-242."""
    if len(splits or []) < 2:
        return ["splits: must include at least 2 splits"]
    errs, total = [], 0
    for s in splits:
        w = s.get("weight", 0)
        if not (1 <= w <= 99):
            errs.append(f"weight {w}: must be between 1 and 99")
        errs += _validate_referenced_upstream(s.get("upstream", ""), names)
        total += w
    if total != 100:
        errs.append("splits: the sum of the weights must be 100")
    return errs


def validate_condition(c):
    """validation.go:289-325."""
    errs, count = [], 0
    if c.get("header"):
        if not _HTTP_HEADER_NAME.match(c["header"]):
            errs.append(f"header {c['header']!r}: not a valid HTTP header name")
        count += 1
    if c.get("cookie"):
        if not _COOKIE_ARG.match(c["cookie"]):
            errs.append(f"cookie {c['cookie']!r}: invalid name")
        count += 1
    if c.get("argument"):
        if not _COOKIE_ARG.match(c["argument"]):
            errs.append(f"argument {c['argument']!r}: invalid name")
        count += 1
    if c.get("variable"):
        v = c["variable"]
        if not v.startswith("$"):
            errs.append(f"variable {v!r}: must start with $")
        elif v not in VALID_VARIABLE_NAMES:
            errs.append(f"variable {v!r}: not allowed")
        count += 1
    if count != 1:
        errs.append("condition: must specify exactly one of header, cookie, argument or variable")
    return errs


def validate_match(m, n_conditions, names):
    """validation.go:367-388."""
    errs = []
    vals = m.get("values") or []
    if len(vals) != n_conditions:
        errs.append(f"values: must specify {n_conditions} values")
    for v in vals:
        errs += is_valid_match_value(v)
    return errs + _validate_referenced_upstream(m.get("upstream", ""), names)


def validate_rules(rules, names):
    """validation.go:265-287."""
    errs = []
    conds = rules.get("conditions") or []
    if not conds:
        errs.append("conditions: Required")
    for c in conds:
        errs += validate_condition(c)
    matches = rules.get("matches") or []
    if not matches:
        errs.append("matches: Required")
    for m in matches:
        errs += validate_match(m, len(conds), names)
    return errs + _validate_referenced_upstream(rules.get("defaultUpstream", ""), names)


def validate_route(r, names, route_forbidden):
    """validation.go:148-190."""
    errs = validate_path(r.get("path", ""))
    count = 0
    if r.get("upstream"):
        errs += _validate_referenced_upstream(r["upstream"], names)
        count += 1
    if r.get("splits"):
        errs += validate_splits(r["splits"], names)
        count += 1
    if r.get("rules") is not None:
        errs += validate_rules(r["rules"], names)
        count += 1
    if r.get("route"):
        if route_forbidden:
            errs.append("route: is not allowed")
        else:
            if not _is_qualified_name(r["route"]):
                errs.append(f"route {r['route']!r}: not a qualified name")
            count += 1
    if count != 1:
        errs.append("route: must specify exactly one of upstream, splits, rules" + ("" if route_forbidden else " or route"))
    return errs


def validate_virtual_server(vs):
    """ValidateVirtualServer (validation.go:15-33)."""
    spec = vs.get("spec") or {}
    errs = validate_host(spec.get("host", ""))
    tls = spec.get("tls")
    if tls is not None:
        sec = tls.get("secret", "")
        errs += ["tls secret: Required"] if sec == "" else ([] if _is_dns1123_subdomain(sec) else ["tls secret: invalid"])
    ue, names = validate_upstreams(spec.get("upstreams"))
    errs += ue
    paths = set()
    for r in spec.get("routes") or []:
        re_ = validate_route(r, names, False)
        if re_:
            errs += re_
        elif r["path"] in paths:
            errs.append(f"path {r['path']!r}: Duplicate")
        else:
            paths.add(r["path"])
    return errs


def validate_virtual_server_route(vsr, vs_host="", path_prefix="/"):
    """ValidateVirtualServerRouteForVirtualServer (validation.go:411-476)."""
    spec = vsr.get("spec") or {}
    host = spec.get("host", "")
    errs = validate_host(host)
    if vs_host and host != vs_host:
        errs.append(f"host {host!r}: must be equal to {vs_host!r}")
    ue, names = validate_upstreams(spec.get("upstreams"))
    errs += ue
    paths = set()
    for r in spec.get("subroutes") or []:
        re_ = validate_route(r, names, True)
        if path_prefix and not r.get("path", "").startswith(path_prefix):
            re_.append(f"path {r.get('path')!r}: must start with {path_prefix!r}")
        if re_:
            errs += re_
        elif r["path"] in paths:
            errs.append(f"path {r['path']!r}: Duplicate")
        else:
            paths.add(r["path"])
    return errs


def generate_endpoints_key(ns, service, port):
    """configs.GenerateEndpointsKey: "<ns>/<service>:<port>"."""
    return f"{ns}/{service}:{port}"


def create_virtual_server(vs, vsr_store, endpoints_of=None):
    """controller.go:1519-1591: the VirtualServerEx the Configurator receives -- every `route:`
    reference resolved in the VSR store ({"ns/name": vsr}, a missing namespace meaning the VS's),
    skipped with a warning when missing or invalid for this VS (host, path prefix); endpoints for
    the VS's and the accepted VSRs' upstreams (endpoints_of(ns, service, port) -> ["ip:port"]).
    Returns (vs_ex, vsr_errors)."""
    endpoints_of = endpoints_of or (lambda ns, svc, port: [])
    vns, _ = _meta(vs)
    spec = vs["spec"]
    eps = {}
    for u in spec.get("upstreams") or []:
        eps[generate_endpoints_key(vns, u["service"], u["port"])] = endpoints_of(vns, u["service"], u["port"])
    vsrs, errors = [], []
    for r in spec.get("routes") or []:
        if not r.get("route"):
            continue
        key = r["route"] if "/" in r["route"] else f"{vns}/{r['route']}"
        vsr = vsr_store.get(key)
        if vsr is None:
            errors.append((key, "VirtualServerRoute doesn't exist"))
            continue
        e = validate_virtual_server_route(vsr, spec["host"], r["path"])
        if e:
            errors.append((key, "; ".join(e)))
            continue
        vsrs.append(vsr)
        rns, _ = _meta(vsr)
        for u in vsr["spec"].get("upstreams") or []:
            eps[generate_endpoints_key(rns, u["service"], u["port"])] = endpoints_of(rns, u["service"], u["port"])
    return {"VirtualServer": vs, "Endpoints": eps, "VirtualServerRoutes": vsrs}, errors


def vs_file_name(vs) -> str:
    """configurator.go:564-566."""
    ns, name = _meta(vs)
    return f"vs_{ns}_{name}"


# --------------------------------------------------------------------------- rendering

def _wallarm_lines(w, ind):
    if not w:
        return []
    out = [f"{ind}wallarm_mode {w['Mode']};", f"{ind}wallarm_mode_allow_override {w['ModeAllowOverride']};",
           f"{ind}wallarm_fallback {w['Fallback']};"]
    if w.get("Instance"):
        out.append(f"{ind}wallarm_instance {w['Instance']};")
    if w.get("BlockPage"):
        out.append(f'{ind}wallarm_block_page "{w["BlockPage"]}";')
    out += [f"{ind}wallarm_parse_response {w['ParseResponse']};",
            f"{ind}wallarm_parse_websocket {w['ParseWebsocket']};",
            f"{ind}wallarm_unpack_response {w['UnpackResponse']};"]
    out += [f"{ind}wallarm_parser_disable {x};" for x in w.get("ParserDisable") or []]
    return out


def render_ingress(cfg: dict) -> str:
    """Directive sequence of version1/nginx.ingress.tmpl (OSS, non-gRPC)."""
    ing = cfg["Ingress"]
    L = [f"# configuration for {ing['Namespace']}/{ing['Name']}"]
    for u in cfg["Upstreams"]:
        L.append(f"upstream {u['Name']} {{")
        if u.get("LBMethod"):
            L.append(f"\t{u['LBMethod']};")
        for s in u["UpstreamServers"]:
            L.append(f"\tserver {s['Address']}:{s['Port']} max_fails={s['MaxFails']} fail_timeout={s['FailTimeout']};")
        if u.get("StickyCookie"):   # nginx-plus.ingress.tmpl:9-11
            L.append(f"\tsticky cookie {u['StickyCookie']};")
        if cfg.get("Keepalive"):
            L.append(f"\tkeepalive {cfg['Keepalive']};")
        L.append("}")
    for s in cfg["Servers"]:
        L.append("server {")
        L += _wallarm_lines(s.get("Wallarm"), "\t")
        for port in s["Ports"]:
            L.append(f"\tlisten {port}{' proxy_protocol' if s['ProxyProtocol'] else ''};")
        if s["SSL"]:
            for port in s["SSLPorts"]:
                L.append(f"\tlisten {port} ssl{' http2' if s['HTTP2'] else ''}"
                         f"{' proxy_protocol' if s['ProxyProtocol'] else ''};")
            L.append(f"\tssl_certificate {s['SSLCertificate']};")
            L.append(f"\tssl_certificate_key {s['SSLCertificateKey']};")
            if s.get("SSLCiphers"):
                L.append(f"\tssl_ciphers {s['SSLCiphers']};")
        for cidr in s.get("SetRealIPFrom") or []:                 # nginx.ingress.tmpl:46-49
            L.append(f"\tset_real_ip_from {cidr};")
        if s.get("RealIPHeader"):
            L.append(f"\treal_ip_header {s['RealIPHeader']};")
        if s.get("RealIPRecursive"):
            L.append("\treal_ip_recursive on;")
        L.append(f"\tserver_tokens {s['ServerTokens']};")
        L.append(f"\tserver_name {s['Name']};")
        if s["SSL"] and s["SSLRedirect"]:
            L += ["\tif ($scheme = http) {", f"\t\treturn 301 https://$host:{s['SSLPorts'][0]}$request_uri;", "\t}"]
        if s["RedirectToHTTPS"]:
            L += ["\tif ($http_x_forwarded_proto = 'http') {", "\t\treturn 301 https://$host$request_uri;", "\t}"]
        for v in s.get("ServerSnippets") or []:
            L.append("\t" + v)
        for loc in s["Locations"]:
            L.append(f"\tlocation {loc['Path']} {{")
            L += _wallarm_lines(loc.get("Wallarm"), "\t\t")
            mi = loc.get("MinionIngress")
            if mi:
                L.append(f"\t\t# location for minion {mi['Namespace']}/{mi['Name']}")
            L.append("\t\tproxy_http_version 1.1;")
            if cfg.get("Keepalive"):
                L.append('\t\tproxy_set_header Connection "";')
            for v in loc.get("LocationSnippets") or []:                # nginx.ingress.tmpl:168-171
                L.append("\t\t" + v)
            L.append(f"\t\tproxy_connect_timeout {loc['ProxyConnectTimeout']};")
            L.append(f"\t\tproxy_read_timeout {loc['ProxyReadTimeout']};")
            L.append(f"\t\tclient_max_body_size {loc['ClientMaxBodySize']};")
            L.append("\t\tproxy_set_header Host $host;")
            L.append("\t\tproxy_set_header X-Real-IP $remote_addr;")
            L.append("\t\tproxy_set_header X-Forwarded-For $proxy_add_x_forwarded_for;")
            L.append("\t\tproxy_set_header X-Forwarded-Host $host;")
            L.append("\t\tproxy_set_header X-Forwarded-Port $server_port;")
            L.append(f"\t\tproxy_set_header X-Forwarded-Proto {'https' if s['RedirectToHTTPS'] else '$scheme'};")
            L.append(f"\t\tproxy_buffering {'on' if loc['ProxyBuffering'] else 'off'};")
            scheme = "https" if loc["SSL"] else "http"
            L.append(f"\t\tproxy_pass {scheme}://{loc['Upstream']['Name']}{loc['Rewrite']};")
            L.append("\t}")
        L.append("}")
    return "\n".join(L) + "\n"


def render_virtual_server(cfg: dict) -> str:
    """Directive sequence of version2/nginx.virtualserver.tmpl (OSS)."""
    L = []
    for u in cfg["Upstreams"]:
        L.append(f"upstream {u['Name']} {{")
        L.append(f"    zone {u['Name']} 256k;")
        if u.get("LBMethod"):
            L.append(f"    {u['LBMethod']};")
        for s in u["Servers"]:
            L.append(f"    server {s['Address']} max_fails={s['MaxFails']} fail_timeout={s['FailTimeout']};")
        if cfg.get("Keepalive"):
            L.append(f"    keepalive {cfg['Keepalive']};")
        L.append("}")
    for sc in cfg["SplitClients"]:
        L.append(f"split_clients {sc['Source']} {sc['Variable']} {{")
        for d in sc["Distributions"]:
            L.append(f"    {d['Weight']} {d['Value']};")
        L.append("}")
    for m in cfg["Maps"]:
        L.append(f"map {m['Source']} {m['Variable']} {{")
        for prm in m["Parameters"]:
            L.append(f"    {prm['Value']} {prm['Result']};")
        L.append("}")
    s = cfg["Server"]
    L.append("server {")
    L.append(f"    listen 80{' proxy_protocol' if s['ProxyProtocol'] else ''};")
    L.append(f"    server_name {s['ServerName']};")
    ssl = s.get("SSL")
    if ssl:
        L.append(f"    listen 443 ssl{' http2' if ssl['HTTP2'] else ''}{' proxy_protocol' if s['ProxyProtocol'] else ''};")
        L.append(f"    ssl_certificate {ssl['Certificate']};")
        L.append(f"    ssl_certificate_key {ssl['CertificateKey']};")
        if ssl.get("Ciphers"):
            L.append(f"    ssl_ciphers {ssl['Ciphers']};")
        if ssl["RedirectToHTTPS"]:
            L += ["    if ($scheme = http) {", "        return 301 https://$host$request_uri;", "    }"]
    if s["RedirectToHTTPSBasedOnXForwarderProto"]:
        L += ["    if ($http_x_forwarded_proto = 'http') {", "        return 301 https://$host$request_uri;", "    }"]
    L.append(f'    server_tokens "{s["ServerTokens"]}";')
    for cidr in s.get("SetRealIPFrom") or []:                      # nginx.virtualserver.tmpl:64-72
        L.append(f"    set_real_ip_from {cidr};")
    if s.get("RealIPHeader"):
        L.append(f"    real_ip_header {s['RealIPHeader']};")
    if s.get("RealIPRecursive"):
        L.append("    real_ip_recursive on;")
    for v in s.get("Snippets") or []:
        L.append("    " + v)
    for irl in s["InternalRedirectLocations"]:
        L += [f"    location {irl['Path']} {{", f"        error_page 418 = {irl['Destination']};",
              "        return 418;", "    }"]
    for loc in s["Locations"]:
        L.append(f"    location {loc['Path']} {{")
        for v in loc.get("Snippets") or []:                           # nginx.virtualserver.tmpl:87-89
            L.append("        " + v)
        L.append(f"        proxy_connect_timeout {loc['ProxyConnectTimeout']};")
        L.append(f"        proxy_read_timeout {loc['ProxyReadTimeout']};")
        L.append(f"        client_max_body_size {loc['ClientMaxBodySize']};")
        L.append(f"        proxy_buffering {'on' if loc['ProxyBuffering'] else 'off'};")
        L.append("        proxy_http_version 1.1;")
        if cfg.get("Keepalive"):
            L.append('        proxy_set_header Connection "";')
        L.append("        proxy_set_header Host $host;")
        L.append("        proxy_set_header X-Forwarded-Proto $scheme;")
        L.append(f"        proxy_pass {loc['ProxyPass']};")
        L.append("    }")
    L.append("}")
    return "\n".join(L) + "\n"


def _go_parse_bool(x: str):
    """strconv.ParseBool: 1 t T TRUE true True / 0 f F FALSE false False; None otherwise."""
    if x in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if x in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    return None


def configmap_params(data: dict, params: dict | None = None) -> dict:
    """ParseConfigMap for the PROXY protocol and realip keys (configmaps.go:145-169): proxy-protocol
    and real-ip-recursive through GetMapKeyAsBool (an invalid bool is logged and ignored),
    real-ip-header verbatim, set-real-ip-from split on "," (GetMapKeyAsStringSlice, no trimming)."""
    p = dict(params or default_config_params())
    for key, field in (("proxy-protocol", "ProxyProtocol"), ("real-ip-recursive", "RealIPRecursive")):
        if key in data:
            b = _go_parse_bool(data[key])
            if b is not None:
                p[field] = b
    if "real-ip-header" in data:
        p["RealIPHeader"] = data["real-ip-header"]
    if "set-real-ip-from" in data:
        p["SetRealIPFrom"] = data["set-real-ip-from"].split(",")
    return p


def render_main(params: dict | None = None, wallarm_global_mode: str | None = None) -> str:
    """The http{} part of version1/nginx.tmpl that affects request classification: the default
    server (:81-102), the stub_status server (:104-115, on by default: the controller's
    -nginx-status flag) and the conf.d include point (:128-129)."""
    p = params or default_config_params()
    L = []
    if p.get("MainEnableWallarm"):
        L.append("load_module /etc/nginx/modules/ngx_http_wallarm_module.so;")
    L += ["events {", "    worker_connections 1024;", "}", "http {"]
    if wallarm_global_mode:
        L.append(f"    wallarm_mode {wallarm_global_mode};")
    L += ["    map $http_upgrade $connection_upgrade {", "        default upgrade;", "        ''      close;", "    }",
          "    server {", f"        listen 80 default_server{' proxy_protocol' if p.get('ProxyProtocol') else ''};",
          f"        listen 443 ssl default_server{' http2' if p.get('HTTP2') else ''}"
          f"{' proxy_protocol' if p.get('ProxyProtocol') else ''};",
          "        ssl_certificate /etc/nginx/secrets/default;", "        ssl_certificate_key /etc/nginx/secrets/default;",
          "        server_name _;", f'        server_tokens "{p.get("ServerTokens", "on")}";', "        access_log off;"]
    if p.get("HealthStatus"):
        L += ["        location /nginx-health {", "            default_type text/plain;",
              '            return 200 "healthy\\n";', "        }"]
    L += ["        location / {", "           return 404;", "        }", "    }"]
    if p.get("NginxStatus", True):   # stub_status (nginx.tmpl:104-115)
        L += ["    server {", f"        listen {p.get('NginxStatusPort', 8080)};"]
        L += [f"        allow {c};" for c in p.get("NginxStatusAllowCIDRs", ["127.0.0.1"])]
        L += ["        deny all;", "        location /stub_status {", "            stub_status;", "        }", "    }"]
    if p.get("StubStatusOverUnixSocketForOSS"):   # (nginx.tmpl:117-125: a unix-socket listener, no TCP client)
        L += ["    server {", "        listen unix:/var/run/nginx-status.sock;", "        access_log off;",
              "        location /stub_status {", "            stub_status;", "        }", "    }"]
    L += ["    include /etc/nginx/config-version.conf;", "    include /etc/nginx/conf.d/*.conf;",
          "    server {", "        listen unix:/var/run/nginx-502-server.sock;", "        access_log off;",
          "        location / {", "            return 502;", "        }", "    }", "}"]
    return "\n".join(L) + "\n"


# --------------------------------------------------------------------------- convenience

def ingress_files(ingresses, base=None, wildcard=False, secrets=(), endpoints=None, is_plus=False):
    """Configurator.AddOrUpdateIngress for a list of plain Ingress objects -> {file stem: text};
    endpoints: {"<svc><port>": ["ip:port", ...]} (IngressEx.Endpoints)."""
    base = base or default_config_params()
    out = {}
    for ing in ingresses:
        ex = {"Ingress": ing, "Endpoints": endpoints or {}}
        cfg = generate_nginx_cfg(ex, tls_pems(ing, wildcard, secrets), False, base, is_plus=is_plus)
        out[object_meta_to_file_name(ing)] = render_ingress(cfg)
    return out


def mergeable_files(masters, minions, base=None, wildcard=False, secrets=()):
    """Configurator.AddOrUpdateMergeableIngress for masters + the minion pool."""
    base = base or default_config_params()
    out = {}
    for m in masters:
        mins = get_minions_for_master(m, minions)
        cfg = generate_nginx_cfg_for_mergeable({"Ingress": m, "Endpoints": {}},
                                               [{"Ingress": x, "Endpoints": {}} for x in mins],
                                               tls_pems(m, wildcard, secrets), base)
        out[object_meta_to_file_name(m)] = render_ingress(cfg)
    return out


def virtual_server_files(vss, base=None, vsrs_by_vs=None, pem_name="/etc/nginx/secrets/default-cafe-secret",
                         vsr_store=None, endpoints_of=None):
    """Configurator.AddOrUpdateVirtualServer for each VS -> {file stem: text}.  With a VSR store
    the controller's resolution applies (create_virtual_server); an invalid VS gets no file
    (controller.go:608-617).  ``vsrs_by_vs`` ({"ns/name": [vsr]}) bypasses the resolution."""
    base = base or default_config_params()
    out = {}
    for vs in vss:
        if validate_virtual_server(vs):
            continue
        if vsr_store is not None:
            ex, _ = create_virtual_server(vs, vsr_store, endpoints_of)
        else:
            key = "%s/%s" % _meta(vs)
            ex = {"VirtualServer": vs, "Endpoints": {}, "VirtualServerRoutes": (vsrs_by_vs or {}).get(key, [])}
        cfg = generate_virtual_server_config(ex, pem_name, base)
        out[vs_file_name(vs)] = render_virtual_server(cfg)
    return out
