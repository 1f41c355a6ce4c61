"""CPU: nginx's address text rules for the realip module (ngx_parse_addr_port + ngx_sock_ntop),
as the device runs them (ingress-plus_amd/csrc/gm_inet.hpp, host build via gm_debug_inet) against
the oracle's independent restatement (orc_inet) on hand cases and 20k random texts, and against
Python's ipaddress where nginx and RFC 5952 agree (plain IPv4, IPv6 without an IPv4 form)."""

import ctypes
import ipaddress

import numpy as np
import pytest

from gpumatch import engine
import oracle_py


def _dev(t: bytes):
    L = engine.lib()
    L.gm_debug_inet.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    buf = ctypes.create_string_buffer(128)
    r = L.gm_debug_inet(t, len(t), buf, 128)
    return None if r < 0 else buf.value.decode()


def _orc(t: bytes):
    L = oracle_py.lib()
    L.orc_inet.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    buf = ctypes.create_string_buffer(128)
    r = L.orc_inet(t, len(t), buf, 128)
    return None if r < 0 else buf.value.decode()


KATS = [
    (b"1.2.3.4", "1.2.3.4 0"), (b"001.002.003.004", "1.2.3.4 0"), (b"1..2.3", "1.0.2.3 0"),
    (b"1.2.3.", "1.2.3.0 0"), (b"255.255.255.255", None), (b"256.1.1.1", None), (b"1.2.3", None),
    (b"1.2.3.4.5", None), (b"1.2.3.4:80", "1.2.3.4 80"), (b"1.2.3.4:0", None), (b"1.2.3.4:65536", None),
    (b"1.2.3.4:", None), (b"::", ":: 0"), (b"::1", "::1 0"), (b"1::", "1:: 0"), (b"::1::", None),
    (b"2001:DB8:0:0:0:0:0:1", "2001:db8::1 0"), (b"2001:db8:0:0:1:0:0:1", "2001:db8::1:0:0:1 0"),
    (b"0:0:1:0:0:0:0:0", "0:0:1:: 0"), (b"::ffff:1.2.3.4", "::ffff:1.2.3.4 0"), (b"::1.2.3.4", "::1.2.3.4 0"),
    (b"::0.0.0.1", "::1 0"), (b"[::1]:8080", "::1 8080"), (b"[::1]", None), (b"[::1]:", None),
    (b"12345::", None), (b"1:2:3:4:5:6:7:8", "1:2:3:4:5:6:7:8 0"), (b"1:2:3:4:5:6:7:8:9", None),
    (b":1", None), (b"", None), (b"unknown", None), (b"fe80::1%eth0", None),
]


@pytest.mark.parametrize("text,want", KATS)
def test_inet_kats(text, want):
    assert _dev(text) == want, text
    assert _orc(text) == want, text


def _rand(rng):
    k = int(rng.integers(0, 9))
    if k == 0:
        return b"%d.%d.%d.%d" % tuple(int(x) for x in rng.integers(0, 300, 4))
    if k in (1, 2, 3):
        g = [b"%x" % int(x) if rng.random() < 0.5 else b"0" for x in rng.integers(0, 65536, 8)]
        if k == 2:
            i, j = sorted(int(x) for x in rng.integers(0, 9, 2))
            return b":".join(g[:i]) + b"::" + b":".join(g[j:])
        if k == 3:
            return b"[" + b":".join(g) + b"]:%d" % int(rng.integers(0, 70000))
        return b":".join(g)
    if k == 4:
        return b"::ffff:%d.%d.%d.%d" % tuple(int(x) for x in rng.integers(0, 256, 4))
    if k == 5:
        return b"0:0:0:0:0:%x:%d.%d.%d.%d" % ((int(rng.integers(0, 2)) * 0xffff,) + tuple(int(x) for x in rng.integers(0, 256, 4)))
    alphabet = b"0123456789abcdefABCDEF:.[]% "
    return bytes(alphabet[int(x)] for x in rng.integers(0, len(alphabet), int(rng.integers(0, 20))))


def test_inet_random_device_vs_oracle_vs_python():
    rng = np.random.Generator(np.random.PCG64(42))
    n_py = 0
    for _ in range(20_000):
        t = _rand(rng)
        d, o = _dev(t), _orc(t)
        assert d == o, (t, d, o)
        if d is None or b"[" in t or b"." in t:
            continue
        try:
            a = ipaddress.ip_address(t.decode())
        except ValueError:
            continue
        # RFC 5952 text = nginx's for IPv6 that nginx does not print with an IPv4 tail
        if a.version == 6 and not str(d).startswith("::"):
            assert d == f"{a.compressed} 0", (t, d, a.compressed)
            n_py += 1
    assert n_py > 500
