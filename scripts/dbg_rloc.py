import sys
sys.path.insert(0, "ingress-plus_amd"); sys.path.insert(0, "tests")
from gpumatch import blob, engine, records
from oracle_py import Oracle
conf = """http { upstream u1 { server 1.1.1.1; } upstream u2 { server 1.1.1.2; }
  server { listen 80 default_server; server_name t.example.com;
    location / { proxy_pass http://u1; }
    location ~ \\\\.php$ { proxy_pass http://u2; } } }"""
b = blob.make_blob(conf, {})
e = engine.Engine(0)
e.load(b, 1)
reqs, arena = records.from_dicts([{"host": "t.example.com", "uri": u} for u in ["/a.php", "/b"]])
print("gpu", e.match_host(reqs, arena)[0])
print("orc", Oracle(b, 1).match(reqs, arena)[0])
