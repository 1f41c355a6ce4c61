"""ctypes binding of libgpumatch.so (the C-ABI declared in include/gpumatch.h).

No fallback: if the HIP library is missing this module raises at import, and every compute
call goes through the gfx950 kernels.  torch is used only as the device-memory / stream
allocator in ``match_torch`` (plumbing, not the product).
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from .records import REQ_DTYPE, VERDICT_DTYPE

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GM_LIB") or os.path.join(os.path.dirname(HERE), "libgpumatch.so")

GM_OK = 0
GM_ABI_VERSION = 10   # include/gpumatch.h
GM_E_OVERFLOW = -4
GM_E_STALE = -9
GM_E_COMM = -7
GM_E_EARLIER = -10
GM_CREATE_COMPILE_ONLY = 0x1
GM_BATCH_HOST = 0x1

ACT = {0: "PROXY", 1: "REDIRECT", 2: "RETURN", 3: "AUTO_301", 4: "NOT_FOUND", 5: "BAD_REQUEST", 6: "BLOCK",
       7: "ERRPAGE", 8: "UNSUPPORTED", 9: "NO_LISTENER", 10: "TOO_LARGE", 11: "FORBIDDEN"}
GM_ACT_FORBIDDEN = 11
GM_ACT_TOO_LARGE = 10
GM_REQ_CHUNKED = 0x10
GM_BUILD_EXPERIMENT, GM_BUILD_TUNING = 0x1, 0x2

STATS_FIELDS = ["gen", "n_servers", "n_locations", "n_upstreams", "n_routes_rules", "n_routes_split", "n_sigs",
                "n_sig_literals", "n_sig_regex", "n_sig_regex_always", "n_rejected_pcre", "n_rejected_other",
                "n_dfa_states", "n_counters"]
STATS_FIELDS64 = ["table_bytes", "lds_bytes_scan", "last_candidates", "last_pairs", "last_hits"]


STATS_FIELDS_MS = ["last_ms_route", "last_ms_scan", "last_ms_verify", "last_ms_tail"]
STATS_FIELDS_WAF = ["n_waf_keys", "bloom_pk", "bloom_fp_ppm", "last_ctx_pass", "last_jobs", "n_peers",
                    "n_upstreams_deferred", "decoders", "n_alw_groups", "n_alw_states", "n_alw_slices",
                    "n_alw_single", "n_rsl_slices", "n_rk_prefilter", "n_rsl_reversed", "n_rsl_pref",
                    "n_realip", "build_flags"]
GM_CREATE_PROFILE = 0x2
GM_CREATE_SERIAL = 0x4


def GM_CREATE_SET_SHIFT(k: int) -> int:
    return (k & 0xFF) << 16


def GM_CREATE_SPILL_SHIFT(k: int) -> int:
    return (k & 0xFF) << 24


def GM_CREATE_SCRATCH_SHIFT(k: int) -> int:
    """Test hook: the internal WAF buffers at 2^-k of their default capacity (include/gpumatch.h)."""
    return (k & 0xFF) << 8


class GmStats(ctypes.Structure):
    _fields_ = ([(f, ctypes.c_uint32) for f in STATS_FIELDS] + [(f, ctypes.c_uint64) for f in STATS_FIELDS64] +
                [(f, ctypes.c_float) for f in STATS_FIELDS_MS] +
                [(f, ctypes.c_uint32) for f in STATS_FIELDS_WAF] +
                [("scratch_scale", ctypes.c_float), ("n_set_reruns", ctypes.c_uint32),
                 ("set_shift", ctypes.c_uint32), ("n_alw_members", ctypes.c_uint32),
                 ("last_redo", ctypes.c_uint32), ("last_spill", ctypes.c_uint32),
                 ("n_rsl_heads", ctypes.c_uint32), ("reserved0", ctypes.c_uint32),
                 ("csrc_hash", ctypes.c_uint64)])


class GmBatch(ctypes.Structure):
    _fields_ = [("reqs", ctypes.c_void_p), ("arena", ctypes.c_void_p), ("arena_len", ctypes.c_uint64),
                ("n", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("arena_len_dev", ctypes.c_void_p)]


EXPORTS = ["gm_create", "gm_destroy", "gm_abi_version", "gm_load_generation", "gm_match_batch", "gm_sync",
           "gm_counters", "gm_counters_reset", "gm_comm_unique_id", "gm_comm_init", "gm_counters_allreduce",
           "gm_stats", "gm_last_error", "gm_normalize_uris", "gm_counters_global", "gm_parse_requests",
           "gm_peers_init", "gm_select_peers", "gm_release_peers", "gm_peer_address", "gm_upstream_uris",
           "gm_update_upstream", "gm_peers_migrate", "gm_rejects", "gm_build_hash", "gm_sync_batches"]

# gm_peer_state (include/gpumatch.h)
PEER_STATE_DTYPE = np.dtype([("conns", "<u4"), ("current_weight", "<i4"), ("flags", "<u4"), ("reserved", "<u4")])
GM_PEER_DOWN = 0x1
GM_PEER_DEFER = 0xFFFFFFFE
GM_NONE = 0xFFFFFFFF

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libgpumatch.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        L.gm_create.restype = ctypes.c_void_p
        L.gm_create.argtypes = [ctypes.c_int, ctypes.c_uint32]
        L.gm_destroy.argtypes = [ctypes.c_void_p]
        L.gm_abi_version.restype = ctypes.c_uint32
        if L.gm_abi_version() != GM_ABI_VERSION:   # the structs below mirror this ABI exactly
            raise ImportError(f"{LIB_PATH}: ABI {L.gm_abi_version()}, this binding expects {GM_ABI_VERSION}")
        L.gm_load_generation.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
        L.gm_match_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(GmBatch), ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_void_p]
        L.gm_sync.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.gm_sync_batches.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.gm_counters.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.gm_counters_reset.argtypes = [ctypes.c_void_p]
        L.gm_comm_unique_id.argtypes = [ctypes.c_void_p]
        L.gm_comm_init.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.gm_counters_allreduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.gm_counters_global.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.gm_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(GmStats)]
        L.gm_normalize_uris.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.gm_parse_requests.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_void_p]
        L.gm_peers_init.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        L.gm_update_upstream.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p),
                                         ctypes.c_uint32]
        L.gm_peers_migrate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_void_p]
        L.gm_select_peers.argtypes = [ctypes.c_void_p, ctypes.POINTER(GmBatch), ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.gm_release_peers.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_void_p]
        L.gm_peer_address.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t,
                                      ctypes.c_void_p]
        L.gm_upstream_uris.argtypes = [ctypes.c_void_p, ctypes.POINTER(GmBatch), ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.gm_rejects.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.gm_build_hash.restype = ctypes.c_char_p
        L.gm_build_hash.argtypes = []
        L.gm_last_error.restype = ctypes.c_char_p
        L.gm_last_error.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def build_hash() -> str:
    """gm_build_hash: the source hash the loaded library was built from (16 hex digits)."""
    return lib().gm_build_hash().decode()


class GmError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"gpumatch error {code}: {msg}")
        self.code = code


class Engine:
    """One context per HIP device (one process per GPU)."""

    def __init__(self, device: int = 0, compile_only: bool = False, profile: bool = False, serial: bool = False,
                 scratch_shift: int = 0, set_shift: int = 0, spill_shift: int = 0):
        L = lib()
        fl = (GM_CREATE_COMPILE_ONLY if compile_only else 0) | (GM_CREATE_PROFILE if profile else 0) | \
             (GM_CREATE_SERIAL if serial else 0) | GM_CREATE_SCRATCH_SHIFT(scratch_shift) | \
             GM_CREATE_SET_SHIFT(set_shift) | GM_CREATE_SPILL_SHIFT(spill_shift)
        self.h = L.gm_create(device, fl)
        if not self.h:
            raise GmError(-1, L.gm_last_error(None).decode())
        self.device = device
        self.compile_only = compile_only

    def close(self):
        if self.h:
            lib().gm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != GM_OK:
            raise GmError(rc, lib().gm_last_error(self.h).decode())

    def load(self, blob: bytes, gen: int = 1):
        self._chk(lib().gm_load_generation(self.h, blob, len(blob), gen))

    def stats(self) -> dict:
        s = GmStats()
        self._chk(lib().gm_stats(self.h, ctypes.byref(s)))
        d = {f: getattr(s, f) for f in STATS_FIELDS + STATS_FIELDS64 + STATS_FIELDS_MS + STATS_FIELDS_WAF}
        d["scratch_scale"] = s.scratch_scale
        d["n_set_reruns"] = s.n_set_reruns
        d["last_redo"] = s.last_redo
        d["last_spill"] = s.last_spill
        d["n_rsl_heads"] = s.n_rsl_heads
        d["set_shift"] = s.set_shift
        d["n_alw_members"] = s.n_alw_members
        d["csrc_hash"] = f"{s.csrc_hash:016x}" if s.csrc_hash else "unknown"
        return d

    def rejects(self) -> list:
        """gm_rejects: the live generation's rejected constructs ("context: directive ...")."""
        n = lib().gm_rejects(self.h, None, 0)
        if n < 0:
            self._chk(n)
        buf = ctypes.create_string_buffer(n + 1)
        lib().gm_rejects(self.h, buf, n + 1)
        return [x for x in buf.value.decode().split("\n") if x]

    def match_ptr(self, reqs_ptr, arena_ptr, arena_len, n, out_ptr, hits_ptr, hit_cap, stream=0, host=False,
                  arena_len_dev=None):
        """gm_match_batch on pointers; ``arena_len_dev``: a device u64 holding the arena's length
        (then ``arena_len`` is the capacity), e.g. written by parse_ptr on the same stream."""
        b = GmBatch(reqs_ptr, arena_ptr, arena_len, n, GM_BATCH_HOST if host else 0, arena_len_dev)
        self._chk(lib().gm_match_batch(self.h, ctypes.byref(b), out_ptr, hits_ptr, hit_cap, stream))

    def sync(self, stream=0):
        self._chk(lib().gm_sync(self.h, stream))

    def sync_batches(self, stream=0, cap=256) -> list:
        """gm_sync_batches: the outcome (GM_OK / GM_E_OVERFLOW) of every batch completed since the
        stream's previous sync, in enqueue order."""
        st = (ctypes.c_int32 * cap)()
        n = lib().gm_sync_batches(self.h, stream, st, cap)
        if n < 0:
            self._chk(n)
        return [int(st[i]) for i in range(min(n, cap))]

    def match_host(self, reqs: np.ndarray, arena: np.ndarray, hit_cap: int | None = None):
        """Host numpy in, host numpy out (staged through HBM by the library)."""
        n = len(reqs)
        reqs = np.ascontiguousarray(reqs, dtype=REQ_DTYPE)
        arena = np.ascontiguousarray(arena) if len(arena) else np.zeros(16, np.uint8)
        out = np.zeros(n, dtype=VERDICT_DTYPE)
        cap = hit_cap if hit_cap is not None else max(1024, 4 * n)
        hits = np.zeros(cap, dtype=np.uint32)
        self.match_ptr(reqs.ctypes.data, arena.ctypes.data, len(arena), n, out.ctypes.data, hits.ctypes.data,
                       cap, 0, host=True)
        self.sync(0)
        total = self.stats()["last_hits"]
        return out, hits[:total]

    def parse_ptr(self, wire_ptr, msgs_ptr, n, reqs_ptr, arena_ptr, arena_cap, arena_len_dev_ptr, stream=0):
        """gm_parse_requests on device pointers (HTTP/1.x wire bytes -> gm_req records + arena)."""
        self._chk(lib().gm_parse_requests(self.h, wire_ptr, msgs_ptr, n, reqs_ptr, arena_ptr, arena_cap,
                                          arena_len_dev_ptr, stream))

    def peers_init_ptr(self, state_ptr, n_peers, stream=0):
        """gm_peers_init: the generation's initial balancer state into a device gm_peer_state array."""
        self._chk(lib().gm_peers_init(self.h, state_ptr, n_peers, stream))

    def update_upstream(self, name: str, servers):
        """gm_update_upstream: NGINX Plus UpdateServersInPlus(name, servers) without a reload."""
        arr = (ctypes.c_char_p * max(len(servers), 1))(*[x.encode() for x in servers])
        self._chk(lib().gm_update_upstream(self.h, name.encode(), arr, len(servers)))

    def peers_migrate_ptr(self, old_ptr, old_n, new_ptr, new_n, stream=0):
        """gm_peers_migrate: a balancer state array across the last update_upstream."""
        self._chk(lib().gm_peers_migrate(self.h, old_ptr, old_n, new_ptr, new_n, stream))

    def select_peers_ptr(self, reqs_ptr, arena_ptr, arena_len, n, verdicts_ptr, state_ptr, n_peers, out_ptr,
                         stream=0):
        """gm_select_peers on device pointers: the peer of every proxied verdict (async)."""
        b = GmBatch(reqs_ptr, arena_ptr, arena_len, n, 0, None)
        self._chk(lib().gm_select_peers(self.h, ctypes.byref(b), verdicts_ptr, state_ptr, n_peers, out_ptr, stream))

    def release_peers_ptr(self, ids_ptr, n, state_ptr, n_peers, stream=0):
        self._chk(lib().gm_release_peers(self.h, ids_ptr, n, state_ptr, n_peers, stream))

    def upstream_uris_ptr(self, reqs_ptr, arena_ptr, arena_len, n, verdicts_ptr, out_ptr, out_cap, off_ptr, len_ptr,
                          stream=0):
        """gm_upstream_uris on device pointers: the URI each proxied request goes upstream with."""
        b = GmBatch(reqs_ptr, arena_ptr, arena_len, n, 0, None)
        self._chk(lib().gm_upstream_uris(self.h, ctypes.byref(b), verdicts_ptr, out_ptr, out_cap, off_ptr, len_ptr,
                                         stream))

    def peer_address(self, peer: int):
        """(address, upstream id) of a global peer id."""
        buf = ctypes.create_string_buffer(512)
        up = ctypes.c_uint32(0)
        rc = lib().gm_peer_address(self.h, peer, buf, 512, ctypes.byref(up))
        if rc < 0:
            self._chk(rc)
        return buf.value.decode(), up.value

    def normalize_uris_ptr(self, arena_ptr, off_ptr, len_ptr, n, out_ptr, out_len_ptr, stream=0):
        """gm_normalize_uris on device pointers (nginx $uri normalisation, include/gpumatch.h)."""
        self._chk(lib().gm_normalize_uris(self.h, arena_ptr, off_ptr, len_ptr, n, out_ptr, out_len_ptr, stream))

    def match_torch(self, reqs_t, arena_t, arena_len: int, out_t, hits_t, stream=None):
        """Device tensors (torch.uint8 / structured views) -> verdicts in out_t (async)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        self.match_ptr(reqs_t.data_ptr(), arena_t.data_ptr(), arena_len, reqs_t.numel() // 64, out_t.data_ptr(),
                       hits_t.data_ptr(), hits_t.numel(), s.cuda_stream)

    def debug_status(self) -> np.ndarray:
        """The last batch's device status words (gm_waf.inc: counts and profiling counters)."""
        out = np.zeros(128, dtype=np.uint32)
        L = lib()
        L.gm_debug_status.restype = ctypes.c_int
        L.gm_debug_status.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        rc = L.gm_debug_status(self.h, out.ctypes.data, 128)
        if rc < 0:
            self._chk(rc)
        return out

    def counters(self) -> np.ndarray:
        n = self.stats()["n_counters"]
        out = np.zeros(max(n, 1), dtype=np.uint64)
        self._chk(lib().gm_counters(self.h, out.ctypes.data, n))
        return out[:n]

    def counters_reset(self):
        self._chk(lib().gm_counters_reset(self.h))

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        rc = lib().gm_comm_unique_id(buf)
        if rc != GM_OK:
            raise GmError(rc, lib().gm_last_error(None).decode())
        return buf.raw

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        self._chk(lib().gm_comm_init(self.h, uid, nranks, rank))

    def counters_allreduce(self, stream=0):
        """Enqueue the out-of-place sum of every rank's cumulative counters (RCCL)."""
        self._chk(lib().gm_counters_allreduce(self.h, stream))

    def counters_global(self) -> np.ndarray:
        """The job-wide counter totals computed by the last counters_allreduce."""
        n = self.stats()["n_counters"]
        out = np.zeros(max(n, 1), dtype=np.uint64)
        self._chk(lib().gm_counters_global(self.h, out.ctypes.data, n))
        return out[:n]
