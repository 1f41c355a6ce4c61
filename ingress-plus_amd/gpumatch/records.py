"""Packed request records (``gm_req`` + byte arena) and the synthetic workloads C1..C5.

The layout is the one declared in ``include/gpumatch.h``: one 64-byte header per request and
a byte arena holding each request's payload contiguously in the order
``uri | args | hdrs | body | host | method | ruri | raddr`` at a 16-byte aligned ``base``.

Workloads follow SURVEY.md §8(d) "Synthetic inputs" (numpy PCG64, seed 0xC0FFEE + index).
All construction is vectorised: a field is a list of *segments*, each segment a slice of a
source pool per record, so a 10M-request batch is built with a handful of ragged scatters.
"""

from __future__ import annotations

import numpy as np

FIELDS = ("uri", "args", "hdrs", "body", "host", "method", "ruri", "raddr")
_FIELDS = FIELDS
SCAN_FIELDS = ("uri", "args", "hdrs", "body")

REQ_DTYPE = np.dtype([
    ("base", "<u8"), ("uri_len", "<u4"), ("args_len", "<u4"), ("hdr_len", "<u4"), ("body_len", "<u4"),
    ("host_len", "<u2"), ("method_len", "<u2"), ("ruri_len", "<u2"), ("raddr_len", "<u2"),
    ("port", "<u2"), ("remote_port", "<u2"), ("flags", "u1"), ("pad0", "u1", (3,)),
    ("rid", "u1", (16,)), ("pad1", "u1", (8,)),
])
assert REQ_DTYPE.itemsize == 64

LEN_FIELD = {"uri": "uri_len", "args": "args_len", "hdrs": "hdr_len", "body": "body_len",
             "host": "host_len", "method": "method_len", "ruri": "ruri_len", "raddr": "raddr_len"}

REQ_HTTPS, REQ_HTTP2, REQ_HTTP10, REQ_INVALID, REQ_CHUNKED = 0x01, 0x02, 0x04, 0x08, 0x10

VERDICT_DTYPE = np.dtype([
    ("gen", "<u4"), ("server_id", "<u4"), ("location_id", "<u4"), ("upstream_id", "<u4"),
    ("action", "u1"), ("route_kind", "u1"), ("split_bucket", "u1"), ("match_idx", "u1"),
    ("waf_mode", "<u2"), ("n_hits", "<u2"), ("first_hit_off", "<u4"), ("status", "<u4"),
])
assert VERDICT_DTYPE.itemsize == 32

SEED_BASE = 0xC0FFEE


# --------------------------------------------------------------------------- segments

class Seg:
    """Per-record slice ``src[off[i] : off[i] + lens[i]]``."""

    __slots__ = ("src", "off", "lens")

    def __init__(self, src: np.ndarray, off: np.ndarray, lens: np.ndarray):
        self.src = np.ascontiguousarray(src, dtype=np.uint8)
        self.off = np.asarray(off, dtype=np.int64)
        self.lens = np.asarray(lens, dtype=np.int64)


def choice_seg(strings, idx) -> Seg:
    """Record i gets ``strings[idx[i]]``."""
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strings]
    lens = np.array([len(b) for b in bs], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    src = np.frombuffer(b"".join(bs) or b"\0", dtype=np.uint8)
    idx = np.asarray(idx, dtype=np.int64)
    return Seg(src, offs[idx], lens[idx])


def const_seg(s, n) -> Seg:
    return choice_seg([s], np.zeros(n, dtype=np.int64))


def pool_seg(pool: np.ndarray, lens, rng) -> Seg:
    lens = np.asarray(lens, dtype=np.int64)
    hi = np.maximum(len(pool) - lens, 1)
    off = (rng.random(len(lens)) * hi).astype(np.int64)
    return Seg(pool, off, lens)


def list_seg(items) -> Seg:
    """Record i gets ``items[i]`` (bytes/str); for small hand-written batches."""
    return choice_seg(items, np.arange(len(items)))


# --------------------------------------------------------------------------- builder

def build(n: int, fields: dict, port, flags, rid=None, remote_port=None, chunk: int = 1 << 17, proxy_port=None):
    """Assemble headers + arena.  ``fields[name]`` is a list of Seg (concatenated per record); an
    optional "paddr" field ($proxy_protocol_addr, <= 46 bytes, after raddr) and proxy_port."""
    FIELDS = _FIELDS + (("paddr",) if "paddr" in fields else ())
    lens = {}
    for f in FIELDS:
        segs = fields.get(f, [])
        tot = np.zeros(n, dtype=np.int64)
        for s in segs:
            assert len(s.lens) == n, (f, len(s.lens), n)
            tot += s.lens
        lens[f] = tot
    limit16 = ("host", "method", "ruri", "raddr")
    for f in limit16:
        if lens[f].max(initial=0) > 0xFFFF:
            raise ValueError(f"field {f} longer than 65535")
    total = np.zeros(n, dtype=np.int64)
    for f in FIELDS:
        total += lens[f]
    padded = (total + 15) & ~np.int64(15)
    base = np.zeros(n, dtype=np.int64)
    if n > 1:
        np.cumsum(padded[:-1], out=base[1:])
    arena_len = int(base[-1] + padded[-1]) if n else 0
    arena = np.zeros(max(arena_len, 16), dtype=np.uint8)

    reqs = np.zeros(n, dtype=REQ_DTYPE)
    reqs["base"] = base
    for f in _FIELDS:
        reqs[LEN_FIELD[f]] = lens[f]
    if "paddr" in fields:
        if lens["paddr"].max(initial=0) > 46:
            raise ValueError("paddr longer than 46")
        reqs["pad0"][:, 0] = lens["paddr"]
        if proxy_port is not None:
            pp = np.asarray(proxy_port, dtype=np.int64) * (lens["paddr"] > 0)
            reqs["pad1"][:, 0] = pp & 0xFF
            reqs["pad1"][:, 1] = pp >> 8
    reqs["port"] = port
    reqs["flags"] = flags
    if remote_port is not None:
        reqs["remote_port"] = remote_port
    if rid is not None:
        reqs["rid"] = rid

    # ragged scatter, field by field, segment by segment, in record chunks
    cur = base.copy()
    for f in FIELDS:
        for s in fields.get(f, []):
            for a in range(0, n, chunk):
                b = min(n, a + chunk)
                L = s.lens[a:b]
                m = int(L.sum())
                if m == 0:
                    continue
                starts = np.repeat(cur[a:b] - np.concatenate([[0], np.cumsum(L)[:-1]]), L)
                srcst = np.repeat(s.off[a:b] - np.concatenate([[0], np.cumsum(L)[:-1]]), L)
                k = np.arange(m, dtype=np.int64)
                arena[starts + k] = s.src[srcst + k]
            cur += s.lens
    return reqs, arena[:arena_len] if arena_len else arena[:0]


# the payload as the wire parser writes it: the eight fields, then $proxy_protocol_addr (its length
# in pad0[0], gpumatch.h)
WIRE_FIELDS = FIELDS + ("paddr",)


def field_len(r, f: str) -> int:
    return int(r["pad0"][0]) if f == "paddr" else int(r[LEN_FIELD[f]])


def field_bytes(reqs, arena, i: int, name: str) -> bytes:
    """Python accessor used by tests."""
    r = reqs[i]
    off = int(r["base"])
    for f in WIRE_FIELDS:
        L = field_len(r, f)
        if f == name:
            return bytes(arena[off:off + L])
        off += L
    raise KeyError(name)


def proxy_port(r) -> int:
    """$proxy_protocol_port of a record (pad1[0..1])."""
    return int(r["pad1"][0]) | int(r["pad1"][1]) << 8


def from_dicts(items: list[dict]):
    """Build a batch from explicit requests (KAT fixtures).  Keys: host, method, uri, args,
    headers (list of (name, value)), body, https, http2, chunked, port, rid (bytes16/hex), raddr,
    ruri, remote_port, paddr / proxy_port (the PROXY protocol source)."""
    n = len(items)
    proxy = any("paddr" in it for it in items)
    cols = {f: [] for f in FIELDS + (("paddr",) if proxy else ())}
    ports, flags, rids, rports, pports = [], [], [], [], []
    for it in items:
        hdrs = it.get("headers", [])
        hb = b"".join((k.encode() if isinstance(k, str) else k) + b": " +
                      (v.encode() if isinstance(v, str) else v) + b"\r\n" for k, v in hdrs)
        host = it.get("host")
        cols["uri"].append(it.get("uri", "/"))
        cols["args"].append(it.get("args", ""))
        cols["hdrs"].append(hb)
        cols["body"].append(it.get("body", b""))
        cols["host"].append(host if host is not None else "")
        cols["method"].append(it.get("method", "GET"))
        cols["ruri"].append(it.get("ruri", ""))
        cols["raddr"].append(it.get("raddr", "10.0.0.1"))
        https = bool(it.get("https", False))
        ports.append(int(it.get("port", 443 if https else 80)))
        fl = (REQ_HTTPS if https else 0) | (REQ_HTTP2 if it.get("http2") else 0) | \
             (REQ_HTTP10 if it.get("http10") else 0) | (REQ_CHUNKED if it.get("chunked") else 0)
        flags.append(fl)
        rid = it.get("rid", bytes(16))
        if isinstance(rid, str):
            rid = bytes.fromhex(rid)
        rids.append(np.frombuffer(rid, dtype=np.uint8))
        rports.append(int(it.get("remote_port", 40000)))
        if proxy:   # $proxy_protocol_addr / port, as gm_parse_requests leaves them
            cols["paddr"].append(it.get("paddr", ""))
            pports.append(int(it.get("proxy_port", 0)))
    fields = {f: [list_seg(cols[f])] for f in cols}
    return build(n, fields, np.array(ports), np.array(flags), np.stack(rids) if n else None,
                 np.array(rports), proxy_port=np.array(pports) if proxy else None)


# --------------------------------------------------------------------------- text pools

_WORDS = ("the of and to in is it that for on with as was at by be this have from or one had not "
          "but what all were when we there can an your which their said if do will each about how up "
          "out them then she many some so these would other into has more her two like him see time "
          "could no make than first been its who now people my made over did down only way find use "
          "may water long little very after words called just where most know get through back much "
          "before go good new write our used me man too any day same right look think also around "
          "another came come work three word must because does part even place well such here take why "
          "things help put years different away again off went old number great tell men say small "
          "every found still between name should home big give air line set own under read last never "
          "us left end along while might next sound below saw something thought both few those always "
          "looked show large often together asked house world going want school important until form "
          "food keep children feet land side without boy once animals life enough took sometimes four "
          "head above kind began almost live page got earth need far hand high year mother light parts "
          "country father let night following picture being study second eyes soon times story boys "
          "since white days ever paper hard near sentence better best across during today others however "
          "sure means knew its try told young miles sun ways thing whole hear example heard several "
          "change answer room sea against top turned learn point city play toward five using himself "
          "usually money order product customer price cart checkout account login session token user "
          "email address phone items quantity total shipping billing status created updated id").split()


def text_pool(rng, size: int, vocab=()) -> np.ndarray:
    """Benign mixed text (words, JSON-ish and form-encoded fragments), all printable ASCII.
    ``vocab``: extra words drawn as often as all the plain words together (the C4 stress
    variant's SQL / HTML / shell vocabulary)."""
    words = np.array(list(_WORDS) + list(vocab) * max(1, len(_WORDS) // max(len(vocab), 1)) if vocab else _WORDS)
    seps = np.array([" ", " ", " ", ", ", ". ", "\": \"", "=", "&", "\n", "_", "-", "/", ":"] +
                    (["(", "'", " '", "<", "--"] if vocab else []))
    n = size // 5 + 16
    w = words[rng.integers(0, len(words), n)]
    s = seps[rng.integers(0, len(seps), n)]
    digits = rng.integers(0, 100000, n).astype(str)
    use_d = rng.random(n) < 0.08
    w = np.where(use_d, digits, w)
    txt = "".join(np.char.add(w, s).tolist())
    b = np.frombuffer(txt.encode(), dtype=np.uint8)
    while len(b) < size:
        b = np.concatenate([b, b])
    return b[:size].copy()


def alnum_pool(rng, size: int) -> np.ndarray:
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_.", dtype=np.uint8)
    return alpha[rng.integers(0, len(alpha), size)]


def geometric_lens(rng, n, mean, lo=0, hi=2048):
    L = rng.geometric(1.0 / max(mean, 1.0), n) - 1 + lo
    return np.minimum(L, hi).astype(np.int64)


_HDR_NAMES = ("User-Agent", "Accept", "Accept-Language", "Accept-Encoding", "Connection", "Referer",
              "Cache-Control", "Upgrade-Insecure-Requests", "X-Forwarded-For", "X-Request-Start",
              "Sec-Fetch-Mode", "Sec-Fetch-Site", "DNT", "Pragma", "X-Client-Version", "Origin",
              "Content-Type", "X-Trace-Id", "Authorization", "If-None-Match")
_HDR_VALUES = ("Mozilla/5.0 (X11; Linux x86_64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/76.0 Safari/537.36",
               "text/html,application/xhtml+xml,application/xml;q=0.9,image/webp,*/*;q=0.8",
               "en-US,en;q=0.9", "gzip, deflate, br", "keep-alive", "https://www.example.org/catalog/page",
               "no-cache", "1", "203.0.113.7, 198.51.100.23", "t=1571234567890", "navigate", "same-origin",
               "application/json", "W/\"5e1f-8c2d\"", "Bearer eyJhbGciOiJIUzI1NiJ9.e30.abcdef",
               "max-age=0")


def header_block_pool(rng, count: int, lo: int = 6, hi: int = 20):
    """``count`` distinct header blocks of lo..hi lines -> (pool bytes, offsets, lengths)."""
    blocks = []
    for _ in range(count):
        k = int(rng.integers(lo, hi + 1))
        names = rng.choice(len(_HDR_NAMES), size=min(k, len(_HDR_NAMES)), replace=False)
        lines = []
        for j in names:
            v = _HDR_VALUES[int(rng.integers(0, len(_HDR_VALUES)))]
            if rng.random() < 0.3:
                v = v + "-" + "".join(chr(97 + int(c)) for c in rng.integers(0, 26, int(rng.integers(4, 40))))
            lines.append(f"{_HDR_NAMES[j]}: {v}\r\n")
        blocks.append("".join(lines).encode())
    lens = np.array([len(b) for b in blocks], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    return np.frombuffer(b"".join(blocks), dtype=np.uint8).copy(), offs, lens


def _rid(rng, n):
    return rng.integers(0, 256, (n, 16), dtype=np.uint8)


def _host_variants(rng, name, n):
    """Host header variants per SURVEY §8(d) C1: 90% exact, 10% random case or :port suffix."""
    v = np.array([name, name.upper(), name.title(), name + ":443", name + ":80", name + "."], dtype=object)
    pick = np.where(rng.random(n) < 0.9, 0, rng.integers(1, len(v), n))
    return v, pick


# --------------------------------------------------------------------------- C1 cafe

def gen_c1(n: int, seed: int = SEED_BASE + 0):
    """C1 cafe Ingress: 85% cafe.example.com (10% of those case/port variants), 15% unknown;
    http/https 50/50; URI 35% /tea.., 35% /coffee.., 10% '/', 10% /teapot-style, 10% random."""
    rng = np.random.Generator(np.random.PCG64(seed))
    hv, hp = _host_variants(rng, "cafe.example.com", n)
    unknown = ["shop.example.com", "www.example.org", "10.0.0.5", "cafe.example.co", "", "bad..host"]
    is_unknown = rng.random(n) < 0.15
    host_strings = list(hv) + unknown
    hidx = np.where(is_unknown, len(hv) + rng.integers(0, len(unknown), n), hp)
    https = rng.random(n) < 0.5
    port = np.where(https, 443, 80)
    flags = np.where(https, REQ_HTTPS, 0)
    pre = ["/tea", "/coffee", "/", "/teapot", "/tea/", "/coffee/", "/t", "/coffe", "/Tea", "/random/"]
    r = rng.random(n)
    pidx = np.select([r < 0.35, r < 0.70, r < 0.80, r < 0.90], [0, 1, 2, 3],
                     default=rng.integers(4, len(pre), n))
    suf = geometric_lens(rng, n, 24, 0, 2048)
    suf = np.where(pidx == 2, 0, suf)
    pool = alnum_pool(rng, 1 << 16)
    slash = np.where(suf > 0, 1, 0)
    fields = {
        "uri": [choice_seg(pre, pidx), Seg(np.frombuffer(b"/", np.uint8), np.zeros(n), slash),
                pool_seg(pool, np.maximum(suf - 1, 0) * slash, rng)],
        "args": [pool_seg(pool, np.where(rng.random(n) < 0.3, rng.integers(3, 40, n), 0), rng)],
        "host": [choice_seg(host_strings, hidx)],
        "method": [choice_seg(["GET", "POST", "HEAD"], rng.choice(3, n, p=[0.7, 0.25, 0.05]))],
        "raddr": [choice_seg(["10.0.0.1", "192.168.1.20", "203.0.113.9"], rng.integers(0, 3, n))],
    }
    return build(n, fields, port, flags, _rid(rng, n), rng.integers(1024, 65535, n))


# --------------------------------------------------------------------------- C2 advanced routing

C2_HOSTS = ("cafe.example.com", "split.example.com", "virtual-server-adv-routing.example.com")


def gen_c2(n: int, seed: int = SEED_BASE + 1):
    """C2 advanced routing: methods GET 60 / POST 30 / other 10; 0-8 cookies (25% carry
    version=v2 at a random position with varied spacing); 0-4 args; 6-20 headers 300-900 B;
    random $request_id."""
    rng = np.random.Generator(np.random.PCG64(seed))
    host = rng.integers(0, len(C2_HOSTS), n)
    https = rng.random(n) < 0.3
    port = np.where(https, 443, 80)
    flags = np.where(https, REQ_HTTPS, 0)
    meth = rng.choice(6, n, p=[0.6, 0.3, 0.04, 0.03, 0.02, 0.01])
    uris = ["/tea", "/coffee", "/backends", "/backend2", "/tea/green", "/coffee/latte", "/", "/other"]
    uidx = rng.integers(0, len(uris), n)
    # args: 0-4 pairs built from a small vocabulary incl. the e2e arg1/argument1 cases
    arg_pairs = ["arg1=v1", "arg1=v2", "argument1=v1", "ARG1=v1", "page=2", "q=tea", "arg1=", "x=arg1=v1",
                 "sort=asc", "arg1=v3"]
    nargs = rng.integers(0, 5, n)
    arg_strs = []
    for k in range(5):
        arg_strs.append(rng.integers(0, len(arg_pairs), n))
    # cookie line variants: position of version=v2 / user=... varies
    ck_vocab = ["session=abc123", "version=v2", "version = v2", "version=v1", "user=some", "user=bad",
                "user=anonymous", "theme=dark", "versions=v2", "USER=some", "lang=en"]
    ncook = rng.integers(0, 9, n)
    want_v2 = rng.random(n) < 0.25
    hpool, hoff, hlen = header_block_pool(rng, 2048, 6, 18)
    hsel = rng.integers(0, len(hoff), n)
    xver = ["future", "deprecated", "FUTURE", "other", ""]
    has_x = rng.random(n) < 0.5
    xsel = rng.integers(0, len(xver), n)
    # per-request small strings are assembled in Python (C2 is a routing workload, headers small)
    args_l, cookie_l = [], []
    for i in range(n):
        k = int(nargs[i])
        args_l.append("&".join(arg_pairs[int(arg_strs[j][i])] for j in range(k)))
        c = int(ncook[i])
        toks = [ck_vocab[int(t)] for t in rng.integers(0, len(ck_vocab), c)] if c else []
        if want_v2[i]:
            toks.insert(int(rng.integers(0, len(toks) + 1)), "version=v2")
        sep = "; " if i % 3 else ";"
        cookie_l.append(("Cookie: " + sep.join(toks) + "\r\n") if toks else "")
    xh = [("X-Version: " + xver[int(xsel[i])] + "\r\n") if has_x[i] else "" for i in range(n)]
    fields = {
        "uri": [choice_seg(uris, uidx)],
        "args": [list_seg(args_l)],
        "hdrs": [Seg(hpool, hoff[hsel], hlen[hsel]), list_seg(xh), list_seg(cookie_l)],
        "host": [choice_seg(C2_HOSTS, host)],
        "method": [choice_seg(["GET", "POST", "PUT", "DELETE", "PATCH", "OPTIONS"], meth)],
        "raddr": [choice_seg(["10.0.0.1", "192.168.1.20"], rng.integers(0, 2, n))],
    }
    return build(n, fields, port, flags, _rid(rng, n), rng.integers(1024, 65535, n))


# --------------------------------------------------------------------------- C4 WAF

def gen_c4(n: int, sigs, seed: int = SEED_BASE + 3, plant_rate: float = 0.01, pool_mb: int = 32,
           stress: bool = False):
    """C4: cafe host/paths + URI, args, 6-20 headers, body 50% 0 B / 40% U(1,2K) / 10% U(2K,8K);
    ``plant_rate`` of requests carry one planted signature (rule chosen uniformly).  ``stress``:
    the benign text also speaks SQL / HTML / shell (gpumatch.sigs.VOCAB)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    if stress:
        from .sigs import VOCAB
        tpool = text_pool(rng, pool_mb << 20, VOCAB)
    else:
        tpool = text_pool(rng, pool_mb << 20)
    apool = alnum_pool(rng, 1 << 20)
    # TLS traffic: the cafe server redirects plain http (ssl-redirect) before the WAF phase
    https = rng.random(n) < 0.98
    port = np.where(https, 443, 80)
    flags = np.where(https, REQ_HTTPS, 0)
    pre = ["/tea/", "/coffee/", "/tea", "/coffee", "/"]
    pidx = rng.choice(len(pre), n, p=[0.45, 0.45, 0.04, 0.04, 0.02])
    suf = geometric_lens(rng, n, 24, 0, 512)
    r = rng.random(n)
    blen = np.where(r < 0.5, 0, np.where(r < 0.9, rng.integers(1, 2049, n), rng.integers(2049, 8193, n)))
    hpool, hoff, hlen = header_block_pool(rng, 4096, 6, 20)
    hsel = rng.integers(0, len(hoff), n)
    alen = np.where(rng.random(n) < 0.6, rng.integers(3, 80, n), 0)
    fields = {
        "uri": [choice_seg(pre, pidx), pool_seg(apool, suf, rng)],
        "args": [pool_seg(tpool, alen, rng)],
        "hdrs": [Seg(hpool, hoff[hsel], hlen[hsel])],
        "body": [pool_seg(tpool, blen, rng)],
        "host": [const_seg("cafe.example.com", n)],
        "method": [choice_seg(["GET", "POST"], (blen > 0).astype(np.int64))],
        "raddr": [const_seg("10.0.0.1", n)],
    }
    reqs, arena = build(n, fields, port, flags, _rid(rng, n), rng.integers(1024, 65535, n))
    if sigs is not None and plant_rate > 0:
        plant_signatures(reqs, arena, sigs, rng, plant_rate)
    return reqs, arena


def plant_signatures(reqs, arena, sigs, rng, rate):
    """Overwrite bytes inside one zone of ``rate`` of the requests with an example that
    matches a uniformly chosen signature (the generator's own example string)."""
    n = len(reqs)
    who = np.nonzero(rng.random(n) < rate)[0]
    rules = rng.integers(0, len(sigs.rules), len(who))
    zl = {"u": "uri_len", "a": "args_len", "h": "hdr_len", "b": "body_len"}
    order = "uahb"
    for i, ri in zip(who.tolist(), rules.tolist()):
        rule = sigs.rules[ri]
        ex = rule.example
        if ex is None:
            continue
        r = reqs[i]
        zones = [z for z in rule.zones if int(r[zl[z]]) >= len(ex)]
        if not zones:
            continue
        z = zones[int(rng.integers(0, len(zones)))]
        off = int(r["base"])
        for zz in order:
            if zz == z:
                break
            off += int(r[zl[zz]])
        L = int(r[zl[z]])
        pos = off + int(rng.integers(0, L - len(ex) + 1))
        arena[pos:pos + len(ex)] = np.frombuffer(ex, dtype=np.uint8)
