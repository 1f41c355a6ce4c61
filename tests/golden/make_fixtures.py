"""Generate the committed golden fixtures from the reference's own test data and tests.

Run in the build container (reads /root/reference, writes tests/golden/*.json).  The GPU box
never runs this; it only reads the JSON.  Nothing here is reference *source*: the fixtures are
the reference's test inputs (YAML under tests/data, Go test structs) and the known answers its
tests assert, transcribed as data.

  advanced_routing.json   tests/data/virtual-server-advanced-routing/*.yaml +
                          tests/suite/test_virtual_server_advanced_routing.py:10-93 (expected backend)
  split_traffic.json      tests/data/virtual-server-split-traffic/standard/virtual-server.yaml +
                          tests/suite/test_virtual_server_split_traffic.py:46-66 (ratio +-0.2)
  match_values.json       docs/virtualserver-and-virtualserverroute.md:264-271 (value semantics)
  confgen_structs.json    internal/configs/virtualserver_test.go:1018-1399,
                          internal/configs/ingress_test.go:124-205 (expected typed configs)
  examples.json           examples/complete-example/cafe-ingress.yaml,
                          examples-of-custom-resources/{advanced-routing,traffic-splitting}/*.yaml,
                          examples/mergeable-ingress-types/{cafe-master,coffee-minion,tea-minion}.yaml
  reference_configs.json  internal/configs/virtualserver_test.go:163-731 (whole-VS configs incl.
                          VirtualServerRoutes), internal/configs/ingress_test.go:75-107 (missing /
                          wildcard TLS secret), :255-270 + :347-563 (mergeable master + minions),
                          pkg/apis/configuration/validation/validation_test.go:642-672 (paths),
                          :1157-1188 (match values)
  e2e_routes.json         tests/suite/test_v_s_route.py:260-322 with tests/data/virtual-server-route/
                          (VSR delegation, no-endpoint 502, deleted VSR 404) and
                          tests/suite/test_virtual_server.py:25-73 with tests/data/virtual-server/
                          standard/ (host change: old host 404, restore; backend port change 502)
"""

import json
import os

import yaml

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def y(path):
    with open(os.path.join(REF, path)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def dump(name, obj):
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
    print("wrote", name)


def main():
    d = "tests/data/virtual-server-advanced-routing/"
    vs = {
        "header": y(d + "standard/virtual-server.yaml")[0],
        "argument": y(d + "virtual-server-argument.yaml")[0],
        "cookie": y(d + "virtual-server-cookie.yaml")[0],
        "variable": y(d + "virtual-server-variable.yaml")[0],
        "complex": y(d + "virtual-server-complex.yaml")[0],
    }
    B1, B3, B4 = "backend1-future", "backend3-deprecated", "backend4-stable"
    cases = [
        # test_flow_with_header
        ("header", dict(headers=[["x-version", "future"]]), B1),
        ("header", dict(headers=[["x-version", "deprecated"]]), B3),
        ("header", dict(headers=[["x-version-invalid", "deprecated"]]), B4),
        # test_flow_with_argument
        ("argument", dict(args="arg1=v1"), B1),
        ("argument", dict(args="arg1=v2"), B3),
        ("argument", dict(args="argument1=v1"), B4),
        # test_flow_with_cookie (requests sends "Cookie: user=...")
        ("cookie", dict(headers=[["Cookie", "user=some"]]), B1),
        ("cookie", dict(headers=[["Cookie", "user=bad"]]), B3),
        ("cookie", dict(headers=[["Cookie", "user=anonymous"]]), B4),
        # test_flow_with_variable: values get / post vs methods GET POST PUT (case-insensitive)
        ("variable", dict(method="GET"), B1),
        ("variable", dict(method="POST"), B3),
        ("variable", dict(method="PUT"), B4),
        # test_flow_with_complex_conditions
        ("complex", dict(method="GET", args="arg1=v1", headers=[["x-version", "future"], ["Cookie", "user=some"]]), B1),
        ("complex", dict(method="POST", args="arg1=v2", headers=[["x-version", "deprecated"], ["Cookie", "user=bad"]]), B3),
        ("complex", dict(method="GET", args="arg1=v2", headers=[["x-version", "deprecated"], ["Cookie", "user=bad"]]), B4),
    ]
    dump("advanced_routing.json", {
        "source": "tests/suite/test_virtual_server_advanced_routing.py:10-93",
        "host": "virtual-server-adv-routing.example.com", "uri": "/backends",
        "virtual_servers": vs,
        "cases": [{"vs": v, "request": r, "expect_upstream": u} for v, r, u in cases],
    })

    sp = y("tests/data/virtual-server-split-traffic/standard/virtual-server.yaml")[0]
    dump("split_traffic.json", {"source": "tests/suite/test_virtual_server_split_traffic.py:46-66",
                                "virtual_server": sp, "tolerance": 0.2})

    # docs/virtualserver-and-virtualserverroute.md:264-271: (value, subject, matches)
    mv = [
        ("john", "john", True), ("john", "John", True), ("john", "JOHN", True), ("john", "bob", False),
        ("!john", "bob", True), ("!john", "anything", True), ("!john", "", True), ("!john", "John", False),
        ("~^yes", "yes", True), ("~^yes", "yes123", True), ("~^yes", "YES", False), ("~^yes", "noyes", False),
        ("!~^yes", "YES", True), ("!~^yes", "Yes123", True), ("!~^yes", "noyes", True), ("!~^yes", "yes", False),
        ("~*no$", "no", True), ("~*no$", "123no", True), ("~*no$", "123NO", True), ("~*no$", "nope", False),
    ]
    dump("match_values.json", {"source": "docs/virtualserver-and-virtualserverroute.md:264-271",
                               "cases": [{"value": a, "subject": b, "match": c} for a, b, c in mv]})

    # Go expected structs (transcribed from virtualserver_test.go / ingress_test.go)
    conds = [{"header": "x-version"}, {"cookie": "user"}, {"argument": "answer"}, {"variable": "$request_method"}]
    vals = [["v1", "john", "yes", "GET"], ["v2", "paul", "no", "POST"]]
    srcs = ["$http_x_version", "$cookie_user", "$arg_answer", "$request_method"]
    rules_maps = []
    for i in range(2):
        for j in range(4):
            ok = "1" if j == 3 else f"$vs_default_cafe_rules_1_match_{i}_cond_{j + 1}"
            rules_maps.append({"Source": srcs[j], "Variable": f"$vs_default_cafe_rules_1_match_{i}_cond_{j}",
                               "Parameters": [{"Value": f'"{vals[i][j]}"', "Result": ok},
                                              {"Value": "default", "Result": "0"}]})
    rules_maps.append({"Source": "$vs_default_cafe_rules_1_match_0_cond_0$vs_default_cafe_rules_1_match_1_cond_0",
                       "Variable": "$vs_default_cafe_rules_1",
                       "Parameters": [{"Value": "~^1", "Result": "@rules_1_match_0"},
                                      {"Value": "~^01", "Result": "@rules_1_match_1"},
                                      {"Value": "default", "Result": "@rules_1_default"}]})
    dump("confgen_structs.json", {
        "split_route": {  # virtualserver_test.go:1018-1079
            "route": {"path": "/", "splits": [{"weight": 90, "upstream": "coffee-v1"},
                                              {"weight": 10, "upstream": "coffee-v2"}]},
            "index": 1,
            "expected": {
                "SplitClient": {"Source": "$request_id", "Variable": "$vs_default_cafe_splits_1",
                                "Distributions": [{"Weight": "90%", "Value": "@splits_1_split_0"},
                                                  {"Weight": "10%", "Value": "@splits_1_split_1"}]},
                "Locations": [{"Path": "@splits_1_split_0", "ProxyPass": "http://vs_default_cafe_coffee-v1"},
                              {"Path": "@splits_1_split_1", "ProxyPass": "http://vs_default_cafe_coffee-v2"}],
                "InternalRedirectLocation": {"Path": "/", "Destination": "$vs_default_cafe_splits_1"}}},
        "rules_route": {  # virtualserver_test.go:1081-1291
            "route": {"path": "/", "rules": {"conditions": conds,
                                             "matches": [{"values": vals[0], "upstream": "coffee-v1"},
                                                         {"values": vals[1], "upstream": "coffee-v2"}],
                                             "defaultUpstream": "tea"}},
            "index": 1,
            "expected": {
                "Maps": rules_maps,
                "Locations": [{"Path": "@rules_1_match_0", "ProxyPass": "http://vs_default_cafe_coffee-v1"},
                              {"Path": "@rules_1_match_1", "ProxyPass": "http://vs_default_cafe_coffee-v2"},
                              {"Path": "@rules_1_default", "ProxyPass": "http://vs_default_cafe_tea"}],
                "InternalRedirectLocation": {"Path": "/", "Destination": "$vs_default_cafe_rules_1"}}},
        "value_for_map": [  # virtualserver_test.go:1293-1355
            ["default", "\\default", False], ["!default", "\\default", True], ["hostnames", "\\hostnames", False],
            ["include", "\\include", False], ["volatile", "\\volatile", False], ["abc", '"abc"', False],
            ["!abc", '"abc"', True], ["", '""', False], ["!", '""', True]],
        "params_for_map": [  # virtualserver_test.go:1357-1399
            ["abc", "1", [{"Value": '"abc"', "Result": "1"}, {"Value": "default", "Result": "0"}]],
            ["!abc", "1", [{"Value": '"abc"', "Result": "0"}, {"Value": "default", "Result": "1"}]]],
        "source_names": [  # virtualserver_test.go:1401-1437
            [{"header": "x-version"}, "$http_x_version"], [{"cookie": "mycookie"}, "$cookie_mycookie"],
            [{"argument": "arg"}, "$arg_arg"], [{"variable": "$request_method"}, "$request_method"]],
        "cafe_ingress": {  # ingress_test.go:124-253
            "ingress": {"metadata": {"name": "cafe-ingress", "namespace": "default",
                                     "annotations": {"kubernetes.io/ingress.class": "nginx"}},
                        "spec": {"tls": [{"hosts": ["cafe.example.com"], "secretName": "cafe-secret"}],
                                 "rules": [{"host": "cafe.example.com", "http": {"paths": [
                                     {"path": "/coffee", "backend": {"serviceName": "coffee-svc", "servicePort": "80"}},
                                     {"path": "/tea", "backend": {"serviceName": "tea-svc", "servicePort": "80"}}]}}]}},
            "endpoints": {"coffee-svc80": ["10.0.0.1:80"], "tea-svc80": ["10.0.0.2:80"]},
            "pems": {"cafe.example.com": "/etc/nginx/secrets/default-cafe-secret"},
            "expected": {
                "upstream_names": ["default-cafe-ingress-cafe.example.com-coffee-svc-80",
                                   "default-cafe-ingress-cafe.example.com-tea-svc-80"],
                "upstream_servers": [[["10.0.0.1", "80"]], [["10.0.0.2", "80"]]],
                "server": {"Name": "cafe.example.com", "SSL": True,
                           "SSLCertificate": "/etc/nginx/secrets/default-cafe-secret",
                           "Ports": [80], "SSLPorts": [443], "SSLRedirect": True, "StatusZone": "cafe.example.com"},
                "locations": [["/coffee", "default-cafe-ingress-cafe.example.com-coffee-svc-80"],
                              ["/tea", "default-cafe-ingress-cafe.example.com-tea-svc-80"]]}},
    })

    ex = {
        "cafe_ingress": y("examples/complete-example/cafe-ingress.yaml")[0],
        "advanced_routing_vs": y("examples-of-custom-resources/advanced-routing/cafe-virtual-server.yaml")[0],
        "traffic_splitting_vs": y("examples-of-custom-resources/traffic-splitting/cafe-virtual-server.yaml")[0],
        "mergeable_master": y("examples/mergeable-ingress-types/cafe-master.yaml")[0],
        "mergeable_minions": [y("examples/mergeable-ingress-types/coffee-minion.yaml")[0],
                              y("examples/mergeable-ingress-types/tea-minion.yaml")[0]],
    }
    dump("examples.json", ex)

    # ---- virtualserver_test.go:163-731: generateVirtualServerConfig on a VirtualServerEx
    def ups(name, svc):
        return {"name": name, "service": svc, "port": 80}
    vsr_coffee = lambda upstreams, sub: {"metadata": {"name": "coffee", "namespace": "default"},
                                         "spec": {"host": "cafe.example.com", "upstreams": upstreams,
                                                  "subroutes": [sub]}}
    vs_cafe = lambda upstreams, tea: {"metadata": {"name": "cafe", "namespace": "default"},
                                      "spec": {"host": "cafe.example.com", "upstreams": upstreams,
                                               "routes": [tea, {"path": "/coffee", "route": "default/coffee"}]}}
    eps4 = {"default/tea-svc-v1:80": ["10.0.0.20:80"], "default/tea-svc-v2:80": ["10.0.0.21:80"],
            "default/coffee-svc-v1:80": ["10.0.0.30:80"], "default/coffee-svc-v2:80": ["10.0.0.31:80"]}
    ups4 = [["vs_default_cafe_tea-v1", "10.0.0.20:80"], ["vs_default_cafe_tea-v2", "10.0.0.21:80"],
            ["vs_default_cafe_vsr_default_coffee_coffee-v1", "10.0.0.30:80"],
            ["vs_default_cafe_vsr_default_coffee_coffee-v2", "10.0.0.31:80"]]
    vsc = {}
    vsc["basic"] = {   # :163-282
        "source": "internal/configs/virtualserver_test.go:163-282",
        "vs": vs_cafe([ups("tea", "tea-svc")], {"path": "/tea", "upstream": "tea"}),
        "vsrs": [vsr_coffee([ups("coffee", "coffee-svc")], {"path": "/coffee", "upstream": "coffee"})],
        "endpoints": {"default/tea-svc:80": ["10.0.0.20:80"], "default/coffee-svc:80": ["10.0.0.30:80"]},
        "params": {"ServerTokens": "off", "Keepalive": 16, "ServerSnippets": ["# server snippet"],
                   "ProxyProtocol": True, "RedirectToHTTPS": True,
                   "SetRealIPFrom": ["0.0.0.0/0"], "RealIPHeader": "X-Real-IP", "RealIPRecursive": True},   # :230-232
        "expected": {
            "Upstreams": [["vs_default_cafe_tea", "10.0.0.20:80"],
                          ["vs_default_cafe_vsr_default_coffee_coffee", "10.0.0.30:80"]],
            "SplitClients": [], "Maps": [],
            "Server": {"ServerName": "cafe.example.com", "ProxyProtocol": True,
                       "RedirectToHTTPSBasedOnXForwarderProto": True, "ServerTokens": "off",
                       "SetRealIPFrom": ["0.0.0.0/0"], "RealIPHeader": "X-Real-IP", "RealIPRecursive": True,   # :260-262
                       "Snippets": ["# server snippet"], "InternalRedirectLocations": [],
                       "Locations": [["/tea", "http://vs_default_cafe_tea"],
                                     ["/coffee", "http://vs_default_cafe_vsr_default_coffee_coffee"]]},
            "Keepalive": "16"}}
    vsc["splits"] = {   # :283-487
        "source": "internal/configs/virtualserver_test.go:283-487",
        "vs": vs_cafe([ups("tea-v1", "tea-svc-v1"), ups("tea-v2", "tea-svc-v2")],
                      {"path": "/tea", "splits": [{"weight": 90, "upstream": "tea-v1"}, {"weight": 10, "upstream": "tea-v2"}]}),
        "vsrs": [vsr_coffee([ups("coffee-v1", "coffee-svc-v1"), ups("coffee-v2", "coffee-svc-v2")],
                            {"path": "/coffee", "splits": [{"weight": 40, "upstream": "coffee-v1"},
                                                            {"weight": 60, "upstream": "coffee-v2"}]})],
        "endpoints": eps4, "params": {},
        "expected": {
            "Upstreams": ups4,
            "SplitClients": [
                {"Source": "$request_id", "Variable": "$vs_default_cafe_splits_0",
                 "Distributions": [{"Weight": "90%", "Value": "@splits_0_split_0"}, {"Weight": "10%", "Value": "@splits_0_split_1"}]},
                {"Source": "$request_id", "Variable": "$vs_default_cafe_splits_1",
                 "Distributions": [{"Weight": "40%", "Value": "@splits_1_split_0"}, {"Weight": "60%", "Value": "@splits_1_split_1"}]}],
            "Maps": [],
            "Server": {"ServerName": "cafe.example.com",
                       "InternalRedirectLocations": [{"Path": "/tea", "Destination": "$vs_default_cafe_splits_0"},
                                                     {"Path": "/coffee", "Destination": "$vs_default_cafe_splits_1"}],
                       "Locations": [["@splits_0_split_0", "http://vs_default_cafe_tea-v1"],
                                     ["@splits_0_split_1", "http://vs_default_cafe_tea-v2"],
                                     ["@splits_1_split_0", "http://vs_default_cafe_vsr_default_coffee_coffee-v1"],
                                     ["@splits_1_split_1", "http://vs_default_cafe_vsr_default_coffee_coffee-v2"]]}}}
    def rmap(src_, var, val, res):
        return {"Source": src_, "Variable": var, "Parameters": [{"Value": val, "Result": res[0]},
                                                               {"Value": "default", "Result": res[1]}]}
    vsc["rules"] = {   # :489-731
        "source": "internal/configs/virtualserver_test.go:489-731",
        "vs": vs_cafe([ups("tea-v1", "tea-svc-v1"), ups("tea-v2", "tea-svc-v2")],
                      {"path": "/tea", "rules": {"conditions": [{"header": "x-version"}],
                                                 "matches": [{"values": ["v2"], "upstream": "tea-v2"}],
                                                 "defaultUpstream": "tea-v1"}}),
        "vsrs": [vsr_coffee([ups("coffee-v1", "coffee-svc-v1"), ups("coffee-v2", "coffee-svc-v2")],
                            {"path": "/coffee", "rules": {"conditions": [{"argument": "version"}],
                                                          "matches": [{"values": ["v2"], "upstream": "coffee-v2"}],
                                                          "defaultUpstream": "coffee-v1"}})],
        "endpoints": eps4, "params": {},
        "expected": {
            "Upstreams": ups4, "SplitClients": [],
            "Maps": [rmap("$http_x_version", "$vs_default_cafe_rules_0_match_0_cond_0", '"v2"', ["1", "0"]),
                     rmap("$vs_default_cafe_rules_0_match_0_cond_0", "$vs_default_cafe_rules_0", "~^1",
                          ["@rules_0_match_0", "@rules_0_default"]),
                     rmap("$arg_version", "$vs_default_cafe_rules_1_match_0_cond_0", '"v2"', ["1", "0"]),
                     rmap("$vs_default_cafe_rules_1_match_0_cond_0", "$vs_default_cafe_rules_1", "~^1",
                          ["@rules_1_match_0", "@rules_1_default"])],
            "Server": {"ServerName": "cafe.example.com",
                       "InternalRedirectLocations": [{"Path": "/tea", "Destination": "$vs_default_cafe_rules_0"},
                                                     {"Path": "/coffee", "Destination": "$vs_default_cafe_rules_1"}],
                       "Locations": [["@rules_0_match_0", "http://vs_default_cafe_tea-v2"],
                                     ["@rules_0_default", "http://vs_default_cafe_tea-v1"],
                                     ["@rules_1_match_0", "http://vs_default_cafe_vsr_default_coffee_coffee-v2"],
                                     ["@rules_1_default", "http://vs_default_cafe_vsr_default_coffee_coffee-v1"]]}}}

    # ---- ingress_test.go:255-270 + 347-563 (mergeable), :75-107 (TLS secrets)
    ann = lambda kind: {"kubernetes.io/ingress.class": "nginx", "nginx.org/mergeable-ingress-type": kind}
    minion = lambda name, path, svc: {"metadata": {"name": name, "namespace": "default", "annotations": ann("minion")},
                                      "spec": {"rules": [{"host": "cafe.example.com", "http": {"paths": [
                                          {"path": path, "backend": {"serviceName": svc, "servicePort": "80"}}]}}]}}
    mergeable = {
        "source": "internal/configs/ingress_test.go:255-270,347-563",
        "master": {"metadata": {"name": "cafe-ingress-master", "namespace": "default", "annotations": ann("master")},
                   "spec": {"tls": [{"hosts": ["cafe.example.com"], "secretName": "cafe-secret"}],
                            "rules": [{"host": "cafe.example.com", "http": {"paths": []}}]}},
        "master_endpoints": {"coffee-svc80": ["10.0.0.1:80"], "tea-svc80": ["10.0.0.2:80"]},
        "minions": [[minion("cafe-ingress-coffee-minion", "/coffee", "coffee-svc"), {"coffee-svc80": ["10.0.0.1:80"]}],
                    [minion("cafe-ingress-tea-minion", "/tea", "tea-svc"), {"tea-svc80": ["10.0.0.2:80"]}]],
        "pems": {"cafe.example.com": "/etc/nginx/secrets/default-cafe-secret"},
        "expected": {
            "upstreams": [["default-cafe-ingress-coffee-minion-cafe.example.com-coffee-svc-80", "random two least_conn",
                           [["10.0.0.1", "80", 1, "10s"]]],
                          ["default-cafe-ingress-tea-minion-cafe.example.com-tea-svc-80", "random two least_conn",
                           [["10.0.0.2", "80", 1, "10s"]]]],
            "server": {"Name": "cafe.example.com", "ServerTokens": "on", "SSL": True,
                       "SSLCertificate": "/etc/nginx/secrets/default-cafe-secret",
                       "SSLCertificateKey": "/etc/nginx/secrets/default-cafe-secret",
                       "StatusZone": "cafe.example.com", "HSTSMaxAge": 2592000, "Ports": [80], "SSLPorts": [443],
                       "SSLRedirect": True},
            "locations": [["/coffee", "default-cafe-ingress-coffee-minion-cafe.example.com-coffee-svc-80",
                           "cafe-ingress-coffee-minion", "60s", "60s", "1m", True],
                          ["/tea", "default-cafe-ingress-tea-minion-cafe.example.com-tea-svc-80",
                           "cafe-ingress-tea-minion", "60s", "60s", "1m", True]],
            "ingress": ["cafe-ingress-master", "default"]}}
    tls = {"source": "internal/configs/ingress_test.go:75-107, configurator.go:19-20",
           "missing": {"pem": "/etc/nginx/secrets/default", "expect_ciphers": "NULL"},
           "wildcard": {"pem": "/etc/nginx/secrets/wildcard", "expect_certificate": "/etc/nginx/secrets/wildcard",
                        "expect_certificate_key": "/etc/nginx/secrets/wildcard"}}
    validation = {
        "source": "pkg/apis/configuration/validation/validation_test.go:642-672,1157-1188",
        "valid_paths": ["/", "/path", "/a-1/_A/"],
        "invalid_paths": ["", " /", "/ ", "/{", "/}", "/abc;"],
        "valid_match_values": ["abc", "123", '\\" \n\t\tabc\\"'.replace("\\n", "\n").replace("\\t", "\t"), '\\"'],
        "invalid_match_values": ['"', "\\", 'abc"', "abc\\\\\\", 'a"b'],
    }
    dump("reference_configs.json", {"vs_configs": vsc, "mergeable": mergeable, "tls": tls, "validation": validation})

    # ---- e2e: VirtualServerRoute (test_v_s_route.py) and VirtualServer (test_virtual_server.py)
    vsr_dir = "tests/data/virtual-server-route/"
    vs_dir = "tests/data/virtual-server/standard/"
    dump("e2e_routes.json", {
        "v_s_route": {
            "source": "tests/suite/test_v_s_route.py:100-160,260-322",
            # the fixture creates the VS and VSR "backends" in the VS's first route namespace and
            # VSR "backend2" in the second (get_route_namespace_from_vs_yaml)
            "vs": y(vsr_dir + "standard/virtual-server.yaml")[0], "vs_namespace": "backends-namespace",
            "vsrs": [["backends-namespace", y(vsr_dir + "route-multiple.yaml")[0]],
                     ["backend2-namespace", y(vsr_dir + "route-single.yaml")[0]]],
            "steps": [
                {"step": "initial", "paths": [["/backends/backend1", 200], ["/backends/backend3", 200], ["/backend2", 200]]},
                # Step 4: backend1-svc port 80 -> 8080: no endpoints for backend1-svc:80 -> 502
                {"step": "backend1 port changed", "no_endpoints": ["backends-namespace/backend1-svc:80"],
                 "paths": [["/backends/backend1", 502], ["/backends/backend3", 200]]},
                # Step 6: VSR backends deleted -> its paths 404, the other VSR still 200
                {"step": "vsr deleted", "deleted": ["backends-namespace/backends"],
                 "paths": [["/backends/backend1", 404], ["/backends/backend3", 404], ["/backend2", 200]]}]},
        "virtual_server": {
            "source": "tests/suite/test_virtual_server.py:25-73",
            "vs": y(vs_dir + "virtual-server.yaml")[0], "vs_updated": y(vs_dir + "virtual-server-updated.yaml")[0],
            # the test builds URLs f"...:{port}/{path}" with paths that start with "/": the request
            # path is "//backend1" (nginx merges the slashes into $uri "/backend1")
            "steps": [
                {"step": "updated", "config": "vs_updated",
                 "requests": [["virtual-server.example.com", "//backend1", 404], ["virtual-server.example.com", "//backend2", 404],
                              ["virtual-server-up.example.com", "//updated-backend1", 200],
                              ["virtual-server-up.example.com", "//updated-backend2", 200]]},
                {"step": "restored", "config": "vs",
                 "requests": [["virtual-server-up.example.com", "//updated-backend1", 404],
                              ["virtual-server-up.example.com", "//updated-backend2", 404],
                              ["virtual-server.example.com", "//backend1", 200], ["virtual-server.example.com", "//backend2", 200]]},
                {"step": "backend1 port changed", "config": "vs", "no_endpoints": ["test-namespace/backend1-svc:80"],
                 "requests": [["virtual-server.example.com", "//backend1", 502], ["virtual-server.example.com", "//backend2", 200]]}],
            "vs_namespace": "test-namespace"},
    })


if __name__ == "__main__":
    main()
