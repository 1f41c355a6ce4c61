"""Shared test helpers: build KAT configs / requests and compare verdicts."""

from __future__ import annotations

import json
import os
import re

import numpy as np

from gpumatch import blob, confgen, records

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def upstream_table(b: bytes) -> list:
    """Sorted upstream names of a generation (the upstream_id space of verdicts)."""
    names = set()
    for kind, _, data in blob.parse_blob(b):
        if kind == blob.ENTRY_SIGS:
            continue
        names.update(re.findall(rb"^\s*upstream\s+(\S+)\s*\{", data, flags=re.M))
    return sorted(n.decode() for n in names)


def vs_blob(vs_list, base=None) -> bytes:
    return blob.make_blob(confgen.render_main(), confgen.virtual_server_files(vs_list, base=base))


def kat_request(host, uri, r):
    d = {"host": host, "uri": uri, "method": r.get("method", "GET"), "args": r.get("args", ""),
         "headers": [tuple(h) for h in r.get("headers", [])]}
    d.update({k: v for k, v in r.items() if k not in d})
    return d


def assert_verdicts_equal(got, exp, hits_got=None, hits_exp=None, label=""):
    fields = [f for f in records.VERDICT_DTYPE.names]
    for f in fields:
        bad = np.nonzero(got[f] != exp[f])[0]
        if len(bad):
            i = int(bad[0])
            raise AssertionError(f"{label}: field {f} differs at {len(bad)} requests; first i={i}: "
                                 f"got {got[i]} expected {exp[i]}")
    if hits_exp is not None:
        assert len(hits_got) == len(hits_exp), f"{label}: hit count {len(hits_got)} vs {len(hits_exp)}"
        assert np.array_equal(hits_got, hits_exp), f"{label}: hit ids differ"
