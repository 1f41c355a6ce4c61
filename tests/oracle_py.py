"""ctypes binding of oracle/liboracle.so (CPU oracle).  Test / baseline infrastructure only."""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB)
        L.orc_create.restype = ctypes.c_void_p
        L.orc_create.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
        L.orc_error.restype = ctypes.c_char_p
        L.orc_match.restype = ctypes.c_int64
        L.orc_match.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.orc_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_murmur2.restype = ctypes.c_uint32
        L.orc_murmur2.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_pcre_match.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.orc_set_prefilter.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_factor.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_proxy_ports.restype = ctypes.c_int
        L.orc_proxy_ports.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.orc_md5_hex.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
        _lib = L
    return _lib


class Oracle:
    def __init__(self, blob: bytes, gen: int = 1, prefilter: bool = False):
        """prefilter: the CPU-baseline engine (regexes behind their required-factor prefilter);
        off (the checker): every regex signature runs on every zone."""
        self._blob = blob
        self.h = lib().orc_create(blob, len(blob), gen)
        if not self.h:
            raise RuntimeError("oracle: " + lib().orc_error().decode())
        if prefilter:
            lib().orc_set_prefilter(ctypes.c_void_p(self.h), 1)
        info = np.zeros(4, dtype=np.uint32)
        lib().orc_info(self.h, info.ctypes.data)
        self.n_servers, self.n_locations, self.n_upstreams, self.n_sigs = (int(x) for x in info)

    def match(self, reqs: np.ndarray, arena: np.ndarray, nthreads: int = 0, hit_cap: int | None = None):
        from gpumatch.records import VERDICT_DTYPE
        n = len(reqs)
        out = np.zeros(n, dtype=VERDICT_DTYPE)
        cap = hit_cap if hit_cap is not None else max(1024, 4 * n)
        hits = np.zeros(cap, dtype=np.uint32)
        reqs = np.ascontiguousarray(reqs)
        arena = np.ascontiguousarray(arena) if len(arena) else np.zeros(16, np.uint8)
        nt = nthreads or min(os.cpu_count() or 1, 16)
        tot = lib().orc_match(self.h, reqs.ctypes.data, arena.ctypes.data, n, out.ctypes.data,
                              hits.ctypes.data, cap, nt)
        if tot < 0:
            raise RuntimeError("oracle hit buffer too small")
        return out, hits[:tot]

    def proxy_ports(self):
        """The listen ports with proxy_protocol, from the oracle's own reading of the config."""
        out = np.zeros(64, dtype=np.uint16)
        k = lib().orc_proxy_ports(self.h, out.ctypes.data, 64)
        return [int(x) for x in out[:k]]


def murmur2(b: bytes) -> int:
    return int(lib().orc_murmur2(b, len(b)))


def pcre_match(pat: str, subj: bytes, caseless: bool = False) -> int:
    return int(lib().orc_pcre_match(pat.encode(), 1 if caseless else 0, subj, len(subj)))


def parse_requests(wire: np.ndarray, msgs: np.ndarray, proxy_ports=()):
    """oracle/gm_oracle.c orc_parse_requests_pp: HTTP/1.x bytes -> (gm_req records, arena);
    proxy_ports: the listen ports with proxy_protocol (Oracle.proxy_ports())."""
    from gpumatch.records import REQ_DTYPE
    L = lib()
    L.orc_parse_requests_pp.restype = ctypes.c_int64
    L.orc_parse_requests_pp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    n = len(msgs)
    reqs = np.zeros(n, dtype=REQ_DTYPE)
    cap = int((2 * msgs["len"].astype(np.int64) + msgs["raddr_len"] + 64).sum()) + 16
    arena = np.zeros(cap, dtype=np.uint8)
    w = np.ascontiguousarray(wire)
    m = np.ascontiguousarray(msgs)
    pp = np.ascontiguousarray(np.asarray(list(proxy_ports) or [0], dtype=np.uint16))
    tot = L.orc_parse_requests_pp(w.ctypes.data, m.ctypes.data, n, reqs.ctypes.data, arena.ctypes.data, cap,
                                  pp.ctypes.data, len(proxy_ports))
    if tot < 0:
        raise RuntimeError("oracle parse: arena capacity")
    return reqs, arena[:tot]


def crc32(b: bytes) -> int:
    """nginx ngx_crc32 (the oracle's bitwise CRC-32/IEEE)."""
    L = lib()
    L.orc_crc32.restype = ctypes.c_uint32
    L.orc_crc32.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    return int(L.orc_crc32(b, len(b)))


class Balancer:
    """The oracle's upstream balancers (orc_select_peers): nginx's peer choice, request by request."""

    def __init__(self, oracle: Oracle):
        from gpumatch.engine import PEER_STATE_DTYPE
        L = lib()
        L.orc_n_peers.restype = ctypes.c_int
        L.orc_n_peers.argtypes = [ctypes.c_void_p]
        L.orc_peers_init.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        L.orc_select_peers.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        self.o = oracle
        self.n_peers = int(L.orc_n_peers(oracle.h))
        self.state = np.zeros(max(self.n_peers, 1), dtype=PEER_STATE_DTYPE)[:self.n_peers]
        L.orc_peers_init(oracle.h, self.state.ctypes.data, self.n_peers)

    def select(self, reqs: np.ndarray, arena: np.ndarray, verdicts: np.ndarray) -> np.ndarray:
        n = len(reqs)
        out = np.zeros(n, dtype=np.uint32)
        reqs = np.ascontiguousarray(reqs)
        arena = np.ascontiguousarray(arena) if len(arena) else np.zeros(16, np.uint8)
        verdicts = np.ascontiguousarray(verdicts)
        rc = lib().orc_select_peers(self.o.h, reqs.ctypes.data, arena.ctypes.data, verdicts.ctypes.data, n,
                                    self.state.ctypes.data, self.n_peers, out.ctypes.data)
        if rc != 0:
            raise RuntimeError("oracle: peer count mismatch")
        return out

    def release(self, ids: np.ndarray):
        for p in ids:
            if p < self.n_peers:
                self.state["conns"][p] -= 1


def upstream_uris(o: Oracle, reqs: np.ndarray, arena: np.ndarray, verdicts: np.ndarray):
    """oracle orc_upstream_uris: (out bytes, offsets, lengths) of the URIs sent upstream."""
    L = lib()
    L.orc_upstream_uris.restype = ctypes.c_int64
    L.orc_upstream_uris.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_void_p]
    n = len(reqs)
    reqs = np.ascontiguousarray(reqs)
    arena = np.ascontiguousarray(arena) if len(arena) else np.zeros(16, np.uint8)
    verdicts = np.ascontiguousarray(verdicts)
    cap = int(4 * len(arena) + 4096 * n + 16)
    out = np.zeros(cap, np.uint8)
    off = np.zeros(n, np.uint64)
    ln = np.zeros(n, np.uint32)
    tot = L.orc_upstream_uris(o.h, reqs.ctypes.data, arena.ctypes.data, verdicts.ctypes.data, n, out.ctypes.data,
                              cap, off.ctypes.data, ln.ctypes.data)
    if tot < 0:
        raise RuntimeError("oracle upstream URIs: capacity")
    return out[:tot], off, ln


def uri_list(out, off, ln):
    """per request: bytes, or None (not proxied) / "defer" """
    res = []
    for o, k in zip(off, ln):
        if k == 0xFFFFFFFF:
            res.append(None)
        elif k == 0xFFFFFFFE:
            res.append("defer")
        else:
            res.append(bytes(out[int(o):int(o) + int(k)]))
    return res


def regex_factor(pat: str) -> bytes:
    """the oracle's prefilter literals of a regex (lowercased, '|'-joined), b"" if none"""
    buf = ctypes.create_string_buffer(16 * 65 + 4)
    lib().orc_factor(pat.encode(), buf)
    return buf.value
