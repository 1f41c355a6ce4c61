"""Config-generation KATs: confgen vs the reference's Go unit-test expected structs
(tests/golden/confgen_structs.json, transcribed from virtualserver_test.go / ingress_test.go)."""

import json
import os

from gpumatch import confgen

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "confgen_structs.json")))
VS = {"metadata": {"name": "cafe", "namespace": "default"}}


def _strip_loc(loc):
    return {"Path": loc["Path"], "ProxyPass": loc["ProxyPass"]}


def test_split_route_config():
    k = G["split_route"]
    got = confgen.generate_split_route_config(k["route"], "vs_default_cafe", "default_cafe", k["index"],
                                              confgen.default_config_params())
    exp = k["expected"]
    assert got["SplitClient"] == exp["SplitClient"]
    assert [_strip_loc(x) for x in got["Locations"]] == exp["Locations"]
    assert got["InternalRedirectLocation"] == exp["InternalRedirectLocation"]


def test_rules_route_config():
    k = G["rules_route"]
    got = confgen.generate_rules_route_config(k["route"], "vs_default_cafe", "default_cafe", k["index"],
                                              confgen.default_config_params())
    exp = k["expected"]
    assert got["Maps"] == exp["Maps"]
    assert [_strip_loc(x) for x in got["Locations"]] == exp["Locations"]
    assert got["InternalRedirectLocation"] == exp["InternalRedirectLocation"]


def test_value_for_rules_route_map():
    for inp, val, neg in G["value_for_map"]:
        assert confgen.generate_value_for_rules_route_map(inp) == (val, neg), inp


def test_parameters_for_rules_route_map():
    for inp, ok, exp in G["params_for_map"]:
        assert confgen.generate_parameters_for_rules_route_map(inp, ok) == exp


def test_source_names():
    for cond, exp in G["source_names"]:
        assert confgen.source_for_condition(cond) == exp


def test_cafe_ingress_config():
    k = G["cafe_ingress"]
    cfg = confgen.generate_nginx_cfg({"Ingress": k["ingress"], "Endpoints": k["endpoints"]}, k["pems"], False,
                                     confgen.default_config_params())
    e = k["expected"]
    assert [u["Name"] for u in cfg["Upstreams"]] == e["upstream_names"]
    assert [[[s["Address"], s["Port"]] for s in u["UpstreamServers"]] for u in cfg["Upstreams"]] == e["upstream_servers"]
    s = cfg["Servers"][0]
    for f, v in e["server"].items():
        assert s[f] == v, f
    assert [[l["Path"], l["Upstream"]["Name"]] for l in s["Locations"]] == e["locations"]


def test_namers_and_file_names():
    vs = {"metadata": {"name": "cafe-x", "namespace": "my-ns"}, "spec": {"host": "h", "routes": []}}
    assert confgen.vs_file_name(vs) == "vs_my-ns_cafe-x"                      # configurator.go:564-566
    assert confgen._safe_ns_name(vs) == "my_ns_cafe_x"                        # virtualserver.go:64-69
    assert confgen.object_meta_to_file_name({"metadata": {"name": "a", "namespace": "b"}}) == "b-a"


def test_mergeable_minion_dedupe():
    """controller.go:1860-1871: a path already claimed by an older minion is dropped."""
    master = {"metadata": {"name": "m", "namespace": "default"}, "spec": {"rules": [{"host": "h"}]}}
    m1 = {"metadata": {"name": "a", "namespace": "default", "creationTimestamp": "1"},
          "spec": {"rules": [{"host": "h", "http": {"paths": [{"path": "/x", "backend": {"serviceName": "s", "servicePort": 80}}]}}]}}
    m2 = {"metadata": {"name": "b", "namespace": "default", "creationTimestamp": "2"},
          "spec": {"rules": [{"host": "h", "http": {"paths": [{"path": "/x", "backend": {"serviceName": "t", "servicePort": 80}},
                                                              {"path": "/y", "backend": {"serviceName": "t", "servicePort": 80}}]}}]}}
    mins = confgen.get_minions_for_master(master, [m2, m1])
    assert [m["metadata"]["name"] for m in mins] == ["a", "b"]
    assert [p["path"] for p in mins[1]["spec"]["rules"][0]["http"]["paths"]] == ["/y"]
    cfg = confgen.generate_nginx_cfg_for_mergeable({"Ingress": master, "Endpoints": {}},
                                                   [{"Ingress": x, "Endpoints": {}} for x in mins], {},
                                                   confgen.default_config_params())
    assert [l["Path"] for l in cfg["Servers"][0]["Locations"]] == ["/x", "/y"]
