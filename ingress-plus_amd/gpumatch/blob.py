"""Generation blob (GMB1) -- what the Manager wrapper hands to ``gm_load_generation``.

Layout (``include/gpumatch.h``): ``u32 magic 'GMB1' | u32 n | n x {u32 kind, u32 name_len,
u32 data_len, name, data}``.  conf.d entries are emitted in sorted file-name order, the order
``include /etc/nginx/conf.d/*.conf`` (``version1/nginx.tmpl:128-129``) reads them in, which
fixes duplicate-server-name precedence.
"""

from __future__ import annotations

import struct

MAGIC = 0x31424D47
ENTRY_MAIN, ENTRY_CONFD, ENTRY_SIGS, ENTRY_SAMPLE = 1, 2, 3, 4


def _b(x):
    return x.encode() if isinstance(x, str) else bytes(x)


def make_blob(main: str | bytes | None, confd: dict, sigs_text: str | bytes | None = None,
              sample: bytes | None = None) -> bytes:
    """``sample``: optional benign traffic bytes (GM_ENTRY_SAMPLE) -- the compiler uses them only to
    choose the WAF prefilter's key windows and hash multiplier; matching results never depend
    on it."""
    entries = []
    if main is not None:
        entries.append((ENTRY_MAIN, b"nginx.conf", _b(main)))
    for name in sorted(confd, key=lambda k: _b(k) + b".conf"):
        entries.append((ENTRY_CONFD, _b(name) + b".conf", _b(confd[name])))
    if sigs_text is not None:
        entries.append((ENTRY_SIGS, b"signatures", _b(sigs_text)))
    if sample is not None:
        entries.append((ENTRY_SAMPLE, b"sample", _b(sample)))
    out = [struct.pack("<II", MAGIC, len(entries))]
    for kind, name, data in entries:
        out.append(struct.pack("<III", kind, len(name), len(data)))
        out.append(name)
        out.append(data)
    return b"".join(out)


def parse_blob(blob: bytes):
    magic, n = struct.unpack_from("<II", blob, 0)
    if magic != MAGIC:
        raise ValueError("bad magic")
    off = 8
    out = []
    for _ in range(n):
        kind, nl, dl = struct.unpack_from("<III", blob, off)
        off += 12
        name = blob[off:off + nl]
        off += nl
        data = blob[off:off + dl]
        off += dl
        out.append((kind, name, data))
    return out
