/*
 * gpumatch.h -- C-ABI of libgpumatch.so, the MI355X (gfx950) batched request-matching engine.
 *
 * Drop-in boundary (SURVEY.md §8 b).  The reference's own plugin seam is the Go interface
 * nginx.Manager (internal/nginx/manager.go:34-50): the Configurator renders nginx config text
 * and hands it to CreateMainConfig / CreateConfig / DeleteConfig, then calls Reload().  The
 * classifier itself runs inside nginx worker processes (ngx_http_core_module location/server
 * lookup, ngx_http_map_module, ngx_http_split_clients_module, the Wallarm module).
 *
 * A Go wrapper `gpumatch.Manager{inner nginx.Manager}` binds these entry
 * points through cgo:
 *   - CreateMainConfig/CreateConfig/DeleteConfig (manager.go:97-129) -> cached in the wrapper,
 *     serialised into a generation blob (GMB1 format below) at Reload time;
 *   - Reload (manager.go:201-225)        -> gm_load_generation(ctx, blob, len, configVersion);
 *   - the nginx worker's per-request classification (external binary; templates
 *     version1/nginx.ingress.tmpl, version2/nginx.virtualserver.tmpl) -> gm_match_batch;
 *   - Prometheus-style counters (internal/metrics/collectors/manager.go:27-59) -> gm_counters,
 *     reduced across GPUs with gm_counters_allreduce (RCCL over xGMI).
 *
 * Conventions: plain C types only; 0 = OK, negative = error (GM_E_*); no C++ exception crosses
 * this boundary; gm_last_error() returns a thread-local message for the last failing call.
 */
#ifndef GPUMATCH_H
#define GPUMATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM_ABI_VERSION 10u  /* 10: gm_sync_batches, GM_E_EARLIER; 9: gm_stats_t.csrc_hash, gm_build_hash, GM_ACT_FORBIDDEN, GM_ROUTE_HELD; 8: PROXY protocol (gm_wire_msg 128 B, $proxy_protocol_addr in gm_req), last_redo;
                               7: GM_ACT_TOO_LARGE, GM_REQ_CHUNKED, gm_rejects, build flags; 6: n_rsl_reversed;
                               5: gm_update_upstream / gm_peers_migrate; 4: union-DFA stats */

/* ---------------------------------------------------------------- status codes */
#define GM_OK            0
#define GM_E_INVAL      -1   /* bad argument / malformed blob                          */
#define GM_E_HIP        -2   /* HIP runtime error                                      */
#define GM_E_NOGEN      -3   /* no generation loaded                                   */
#define GM_E_OVERFLOW   -4   /* candidate / hit buffer capacity exceeded (batch void)  */
#define GM_E_PARSE      -5   /* generation rejected: config text unparseable           */
#define GM_E_NOMEM      -6
#define GM_E_COMM       -7   /* RCCL error                                             */
#define GM_E_NODEVICE   -8   /* compute call on a compile-only context                 */
#define GM_E_STALE      -9   /* gm_update_upstream: the live generation changed under it
                                (a load or another update published first); nothing published */
#define GM_E_EARLIER   -10   /* gm_match_batch: an EARLIER batch of the stream completed void in the
                                sync this call forced (PENDING_MAX unsynced batches, or a GM_BATCH_HOST
                                batch behind device ones); this batch was not enqueued.
                                gm_sync_batches names the void batch(es) */

/* ---------------------------------------------------------------- gm_create flags */
#define GM_CREATE_COMPILE_ONLY  0x1u  /* no HIP device: compile + stats only (host tests) */
#define GM_CREATE_PROFILE       0x2u  /* record HIP events per stage (gm_stats_t.last_ms_*) */
#define GM_CREATE_SERIAL        0x4u  /* measurement: run the route stage alone before the WAF scan */
                                      /* (default: beside it on a side stream), so each stage's     */
                                      /* HIP-event time is its own                                  */
/* test hook: the internal WAF buffers (candidates, survivors, pairs, jobs) at 2^-k of their default
 * capacity, k = 1..31 (bits 8..15), so the overflow continuations run on batches small enough for
 * the oracle; reported in gm_stats_t.scratch_scale */
#define GM_CREATE_SCRATCH_SHIFT(k) (((uint32_t)(k) & 0xFFu) << 8)
/* test hook: the WAF dedupe set at 2^-k of its default capacity too (bits 16..23), so a batch
 * overflows it (OV_SET) and gm_sync's continuation is exercised */
#define GM_CREATE_SET_SHIFT(k) (((uint32_t)(k) & 0xFFu) << 16)
/* test hook: the spill of the pairs a full set refuses, and the always-run slices' match list, at
 * 2^-k of their capacity (bits 24..31), so that they overflow and gm_sync's continuation redoes the
 * requests they missed */
#define GM_CREATE_SPILL_SHIFT(k) (((uint32_t)(k) & 0xFFu) << 24)

/* ---------------------------------------------------------------- packed request record
 * One 64-byte header per request; payload bytes live in one byte arena.  The payload of a
 * record is contiguous at arena[base ...] in this fixed field order (so only lengths are
 * stored):
 *     uri | args | hdrs | body | host | method | ruri | raddr
 * followed by `paddr` (paddr_len = pad0[0] bytes): $proxy_protocol_addr, the source address of the
 * connection's PROXY protocol header (`listen ... proxy_protocol`), its source port in pad1[0..1]
 * (little-endian); paddr_len 0: no PROXY address (not a proxy_protocol listener, or "UNKNOWN").
 * The first four are the WAF-scanned zones.  `hdrs` is the header block exactly as parsed:
 * lines "Name: value\r\n" (the space after ':' optional; leading / trailing spaces of a value are
 * not part of it, tabs are -- nginx's header parser).
 * `uri` is nginx's normalised $uri; `args` is $args without '?'; `host` is the raw Host header
 * value (host_len == 0: header absent); `ruri` is the raw $request_uri (ruri_len == 0: derived
 * as uri ["?" args]); `raddr` is $remote_addr text.  $request_id is the 16 raw random bytes in
 * `rid` (nginx prints them as 32 lowercase hex digits).
 * Records must be stored with non-decreasing `base`, 16-byte aligned (coalesced dwordx4 scans).
 */
typedef struct gm_req {
    uint64_t base;          /* byte offset of the payload in the arena (16-B aligned)      */
    uint32_t uri_len;
    uint32_t args_len;
    uint32_t hdr_len;
    uint32_t body_len;
    uint16_t host_len;
    uint16_t method_len;
    uint16_t ruri_len;
    uint16_t raddr_len;
    uint16_t port;          /* local listen port ($server_port)                             */
    uint16_t remote_port;
    uint8_t  flags;         /* GM_REQ_*                                                    */
    uint8_t  pad0[3];       /* [0] paddr_len; [1..2] GM_REQ_INVALID's HTTP status           */
    uint8_t  rid[16];       /* $request_id raw bytes                                        */
    uint8_t  pad1[8];       /* [0..1] $proxy_protocol_port                                  */
} gm_req;

#define GM_REQ_HTTPS   0x01u  /* connection is TLS: $scheme = https, $https = on          */
#define GM_REQ_HTTP2   0x02u  /* $http2 = "h2"                                            */
#define GM_REQ_HTTP10  0x04u  /* request line protocol HTTP/1.0 (else HTTP/1.1 / HTTP/2.0) */
#define GM_REQ_INVALID 0x08u  /* the wire parser rejected the request (gm_parse_requests): the  */
                              /* HTTP status nginx answers is in pad0[1] | pad0[2] << 8, and   */
                              /* gm_match_batch answers GM_ACT_BAD_REQUEST with that status     */
#define GM_REQ_CHUNKED 0x10u  /* the body came chunked (Transfer-Encoding: chunked; body_len =  */
                              /* the decoded length): client_max_body_size applies when the     */
                              /* proxying location reads it, not to a Content-Length up front.  */
                              /* Set it for ANY body whose length was not announced up front --  */
                              /* an HTTP/2 request whose DATA frames came without a              */
                              /* content-length header included (nginx: content_length_n == -1);*/
                              /* without it body_len is taken as a Content-Length (413 at find-  */
                              /* config time, whatever the location does)                        */

typedef struct gm_batch {
    const gm_req  *reqs;      /* n headers (device pointer unless GM_BATCH_HOST)          */
    const uint8_t *arena;     /* payload arena (device pointer unless GM_BATCH_HOST)      */
    uint64_t       arena_len; /* bytes; with arena_len_dev: the arena's capacity          */
    uint32_t       n;
    uint32_t       flags;     /* GM_BATCH_*                                               */
    /* optional device u64 holding the arena's length (e.g. written by gm_parse_requests on
     * the same stream): the kernels read it on the device, so parse -> match needs no host
     * round trip.  NULL: arena_len is the length. */
    const uint64_t *arena_len_dev;
} gm_batch;

#define GM_BATCH_HOST  0x1u   /* reqs/arena/out/hit_ids are host memory: staged through HBM */

/* ---------------------------------------------------------------- verdict (32 B) */
typedef struct gm_verdict {
    uint32_t gen;               /* generation (= nginx configVersion) that produced it     */
    uint32_t server_id;         /* index of the selected server block (config order)       */
    uint32_t location_id;       /* index of the URI-selected location, GM_NONE if none     */
    uint32_t upstream_id;       /* index in the sorted upstream-name table, GM_NONE if none */
    uint8_t  action;            /* GM_ACT_*                                                */
    uint8_t  route_kind;        /* GM_ROUTE_*                                              */
    uint8_t  split_bucket;      /* split_clients part, 0xFF none                          */
    uint8_t  match_idx;         /* rules match index, 0xFF default / none                 */
    uint16_t waf_mode;          /* GM_WAF_* of the location that reached the access phase */
    uint16_t n_hits;            /* signature ids at hit_ids[first_hit_off ...]            */
    uint32_t first_hit_off;
    uint32_t status;            /* HTTP status the verdict implies (200 = proxied)         */
} gm_verdict;

#define GM_NONE 0xFFFFFFFFu

enum {
    GM_ACT_PROXY        = 0,  /* proxy_pass to upstream_id                                 */
    GM_ACT_REDIRECT     = 1,  /* server-level `return 301` (ssl-redirect / x-forwarded-proto) */
    GM_ACT_RETURN       = 2,  /* location `return <status>` (default server 404, health 200), or */
                              /* a content handler the engine answers itself (stub_status: 200) */
    GM_ACT_AUTO_301     = 3,  /* prefix location auto_redirect ($uri + "/")               */
    GM_ACT_NOT_FOUND    = 4,  /* no location matched                                       */
    GM_ACT_BAD_REQUEST  = 5,  /* invalid Host                                              */
    GM_ACT_BLOCK        = 6,  /* WAF block mode with >= 1 signature hit                    */
    GM_ACT_ERRPAGE      = 7,  /* error_page target empty (no split bucket) -> 302          */
    GM_ACT_UNSUPPORTED  = 8,  /* location uses a construct the compiler rejected, or the   */
                              /* regex search reached a PCRE-only regex location whose     */
                              /* superset pattern matches: the data plane defers to nginx  */
    GM_ACT_NO_LISTENER  = 9,  /* no server listens on the port / TLS on a plain port      */
    GM_ACT_TOO_LARGE    = 10, /* 413: the body exceeds client_max_body_size (nginx.ingress.tmpl:175, */
                              /* nginx.virtualserver.tmpl:93) -- no WAF phase, nothing proxied */
    GM_ACT_FORBIDDEN    = 11  /* 403: an allow / deny rule denies the client address (after realip): */
                              /* the stub_status server of nginx.tmpl:104-115 (-nginx-status-allow-cidrs) */
};

enum { GM_ROUTE_NONE = 0, GM_ROUTE_PLAIN = 1, GM_ROUTE_SPLIT = 2, GM_ROUTE_RULES = 3 };
/* route_kind bit, only between gm_match_batch and gm_sync: the batch's WAF dedupe set overflowed and
 * whether this wallarm_mode-block request is blocked is known only once gm_sync completes the batch
 * (its action reads PROXY meanwhile).  gm_select_peers / gm_upstream_uris enqueued before gm_sync
 * answer GM_PEER_DEFER for it (no balancer state moves); gm_sync clears the bit.  Every other action
 * is final when the batch's kernels end, so the match -> peers -> URI chain needs no gm_sync. */
#define GM_ROUTE_HELD 0x80u
enum { GM_WAF_OFF = 0, GM_WAF_MONITORING = 1, GM_WAF_SAFE_BLOCKING = 2, GM_WAF_BLOCK = 3 };

/* ---------------------------------------------------------------- generation blob (GMB1)
 *   u32 magic 'GMB1' (0x31424D47) | u32 n_entries | n x { u32 kind, u32 name_len, u32 data_len,
 *   name bytes, data bytes }     (all little-endian, no padding)
 * kinds: main nginx.conf (CreateMainConfig), conf.d file (CreateConfig; include order = sorted
 * file name, nginx.tmpl:128-129), signature set (text).
 */
#define GM_BLOB_MAGIC     0x31424D47u
#define GM_ENTRY_MAIN     1u
#define GM_ENTRY_CONFD    2u
#define GM_ENTRY_SIGS     3u
#define GM_ENTRY_SAMPLE   4u   /* optional: benign traffic sample bytes; tunes WAF key choice only */

typedef struct gm_stats_t {
    uint32_t gen;
    uint32_t n_servers;
    uint32_t n_locations;
    uint32_t n_upstreams;
    uint32_t n_routes_rules;
    uint32_t n_routes_split;
    uint32_t n_sigs;              /* signature rules accepted                           */
    uint32_t n_sig_literals;
    uint32_t n_sig_regex;
    uint32_t n_sig_regex_always;  /* regexes with no >=4-byte required factor           */
    uint32_t n_rejected_pcre;     /* regexes using PCRE-only constructs (rejected)      */
    uint32_t n_rejected_other;    /* other constructs rejected: every directive outside the     */
                                  /* known-neutral set (snippets: deny, auth_basic, ...), nested */
                                  /* locations; the requests reaching one are GM_ACT_UNSUPPORTED */
                                  /* (gm_rejects lists them)                                    */
    uint32_t n_dfa_states;
    uint32_t n_counters;          /* n_locations + n_sigs                               */
    uint64_t table_bytes;         /* device table bytes of the generation               */
    uint64_t lds_bytes_scan;      /* LDS bytes the WAF scan stage stages per workgroup  */
    uint64_t last_candidates;     /* WAF prefilter candidates in the last batch         */
    uint64_t last_pairs;          /* unique (request, rule) hits of scanning requests   */
    uint64_t last_hits;           /* hit ids written, last batch                        */
    /* GM_CREATE_PROFILE contexts: HIP-event times (ms) of the last synced batch's stages: route
     * kernel (side stream), WAF scan kernel, context filter + exact check, and everything after
     * it (regex confirm, hit emission). */
    float    last_ms_route, last_ms_scan, last_ms_verify, last_ms_tail;
    /* WAF prefilter shape: key windows in the Bloom filter, probes per window (K = 2 * pk bits),
     * and the modelled false-positive weight per probed window (ppm) the compiler chose on. */
    uint32_t n_waf_keys, bloom_pk, bloom_fp_ppm;
    /* last batch: candidate windows passing the stage-2 context filter; regex jobs queued */
    uint32_t last_ctx_pass, last_jobs;
    uint32_t n_peers;             /* upstream `server` peers: gm_peer_state entries     */
    uint32_t n_upstreams_deferred;/* upstreams whose balancing the engine leaves to nginx */
    uint32_t decoders;            /* request parsers the signature set runs (GM_DEC_*)  */
    /* always-run regexes: union-DFA groups (one pass over a zone answers a group), their states,
     * the LDS slices they are run in, and regexes left to the per-regex kernel (too big alone) */
    uint32_t n_alw_groups, n_alw_states, n_alw_slices, n_alw_single;
    /* regex locations of large servers (> RLOC_SEQ_MAX): union-DFA slices in LDS (0: the factor
     * prefilter runs them) */
    uint32_t n_rsl_slices;
    /* servers whose regex locations stay behind the factor prefilter (a regex no union group
     * can hold): k_rloc answers them */
    uint32_t n_rk_prefilter;
    /* of n_rsl_slices: slices of X$ regex locations run backwards from the URI's end, and forward
     * slices run only for requests whose $uri holds one of their regexes' factors */
    uint32_t n_rsl_reversed, n_rsl_pref;
    /* servers with a realip configuration (set_real_ip_from ...), and the build: GM_BUILD_* bits of
     * the measurement / test variants compiled into this library (0 = the product build) */
    uint32_t n_realip;
    uint32_t build_flags;
    /* the internal WAF capacity scale in effect (GM_CREATE_SCRATCH_SHIFT test hook; 1.0 normally) */
    float    scratch_scale;
    /* WAF passes gm_sync ran because a dedupe set overflowed (cumulative, this ctx): continuation
     * passes over the requests to redo, and whole re-runs of a stream's earlier batches */
    uint32_t n_set_reruns;
    uint32_t set_shift;          /* GM_CREATE_SET_SHIFT in effect (0 normally) */
    /* always-run union members: one per distinct (pattern, nocase) among the always-run regexes */
    uint32_t n_alw_members;
    /* the last dedupe-set continuation (gm_sync): requests redone (a sub-batch of their zones), and
     * pairs the full set refused that the spill held (emitted from it with no stage re-run) */
    uint32_t last_redo;
    uint32_t last_spill;
    /* of n_rsl_slices: anchored and reversed slices run only over the requests their head map
     * admits (the first, or for a reversed slice the last, three $uri bytes) */
    uint32_t n_rsl_heads;
    uint32_t reserved0;
    /* the source hash the library was built from (scripts/scan_profile.py csrc_hash: sha256 over
     * the files of ingress-plus_amd/csrc and include/gpumatch.h, first 16 hex digits as a number; 0 = unknown):
     * a profile or bench line names the build it measured, not the tree beside it */
    uint64_t csrc_hash;
} gm_stats_t;

/* gm_stats_t.build_flags: measurement / test variants compiled into the library.  bench.py refuses
 * a non-zero value unless told it measures a variant. */
#define GM_BUILD_EXPERIMENT   0x1u   /* a GM_EXP_* measurement macro (timing only) */
#define GM_BUILD_TUNING       0x2u   /* a non-default GM_SCAN_* / GM_ROUTE_* / GM_RLOC_* / GM_WIRE_* value */

/* Request parsers (Wallarm's) a signature set can declare ("@decoders" line of
 * the GM_ENTRY_SIGS text); wallarm_parser_disable <name> (annotations.go:320-329,
 * nginx.ingress.tmpl:26,111) turns one off for a server or location.  Their decoded views of
 * $args and the body are scanned by the same WAF stages (hits count for the request):
 *   percent   %XX -> byte in $args (and a form body)
 *   urlenc    '+' -> ' ' in $args and an application/x-www-form-urlencoded body
 *   json_doc  JSON string escapes (\" \\ \/ \b \f \n \r \t \uXXXX -> UTF-8) of a "json" body
 *   base64    every run of >= 16 base64 characters in $args / the body, decoded */
#define GM_DEC_PERCENT 0x1u
#define GM_DEC_URLENC  0x2u
#define GM_DEC_JSON    0x4u
#define GM_DEC_BASE64  0x8u

typedef struct gm_ctx gm_ctx;

/* Create a context bound to one HIP device (one ctx per device, one process per GPU). */
gm_ctx     *gm_create(int hip_device, uint32_t flags);
void        gm_destroy(gm_ctx *ctx);
uint32_t    gm_abi_version(void);

/* Copy-in a new table generation.  Atomic: on any error the previous generation stays
 * live; rejected rules are counted (gm_stats), never returned as an error. */
int         gm_load_generation(gm_ctx *ctx, const void *blob, size_t len, uint32_t gen);

/* Classify a batch.  Asynchronous on `stream` (hipStream_t; NULL = legacy default stream): the
 * call enqueues every stage and returns without waiting for the device (no host round trip for
 * intermediate counts -- they stay in device status words).  out[i] receives the verdict of
 * reqs[i]; the hit ids of request i are hit_ids[out[i].first_hit_off .. + n_hits), ascending,
 * requests in order.  gm_sync(ctx, stream) completes the stream's pending batches (the multi-batch
 * contract below) and reports capacity overflow (GM_E_OVERFLOW: a batch's verdicts are void; an internal WAF buffer that
 * overflowed is doubled for the stream's next batch, so a retry of the batch succeeds once the
 * buffers fit the traffic).
 * Thread-safe per (ctx, stream) pair: each stream has its own scratch buffers, so batches on
 * different streams may be enqueued from different threads and run concurrently.  A scratch
 * buffer that a batch outgrows is replaced after its stream drains (the first large batches).
 * Replaces the nginx worker's per-request classification (SURVEY.md §8 a): host/server
 * (nginx.ingress.tmpl:53), location (nginx.ingress.tmpl:96), map / split_clients
 * (nginx.virtualserver.tmpl:17-31), the Wallarm access phase (nginx.ingress.tmpl:12-29). */
int         gm_match_batch(gm_ctx *ctx, const gm_batch *in, gm_verdict *out,
                           uint32_t *hit_ids, size_t hit_cap, void *stream);
int         gm_sync(gm_ctx *ctx, void *stream);

/* The multi-batch contract.  A stream may hold up to 64 (PENDING_MAX) enqueued, unsynced batches;
 * gm_sync completes ALL of them (not just the last), in enqueue order, and its GM_E_OVERFLOW means
 * "at least one of them is void".  Until the gm_sync that completes a batch, its reqs / arena /
 * out / hit_ids buffers must stay allocated and unmodified: a batch whose WAF dedupe set overflowed
 * is completed inside gm_sync by re-running it (the stream's last batch by a continuation over its
 * scratch, earlier ones whole from their inputs).  The 65th unsynced gm_match_batch, and a
 * GM_BATCH_HOST batch behind device batches, first completes the earlier ones synchronously; if one
 * of those is void it returns GM_E_EARLIER and does not enqueue the new batch.
 * gm_sync_batches is gm_sync with the outcome per batch: it completes the stream's pending batches
 * and writes status[i] (GM_OK, or GM_E_OVERFLOW for a void batch -- its verdicts are garbage and its
 * counters were not committed: retry it, and only it) for every batch completed since the previous
 * gm_sync / gm_sync_batches on the stream, forced completions included, in enqueue order; it
 * returns that number of batches (entries past `cap` are not written), or a negative GM_E_* for an
 * error no batch status describes (HIP; gm_parse_requests / gm_upstream_uris capacity, which gm_sync
 * reports the same way; the statuses are then kept for the next call).  gm_sync discards them. */
int         gm_sync_batches(gm_ctx *ctx, void *stream, int32_t *status, size_t cap);

/* Per-location and per-signature hit counters of this device, u64, cumulative since the
 * generation was loaded (or gm_counters_reset): [0, n_locations) locations,
 * [n_locations, n_locations + n_sigs) signatures (gm_stats_t.n_counters entries).  The analogue
 * of the reference's monotonic Prometheus counters (internal/metrics/collectors/manager.go:27-59).
 * A batch's hits are committed once, when it completes whole: a batch gm_sync reports void
 * (GM_E_OVERFLOW) adds nothing, so its retry counts each request once; a batch whose WAF dedupe
 * set overflowed is re-run inside gm_sync (gm_stats_t.n_set_reruns) and counted on that run. */
int         gm_counters(gm_ctx *ctx, uint64_t *out, size_t n);
int         gm_counters_reset(gm_ctx *ctx);

/* Multi-GPU: ncclUniqueId (128 bytes) produced by rank 0 and shared by the caller. */
int         gm_comm_unique_id(void *out_128_bytes);
int         gm_comm_init(gm_ctx *ctx, const void *nccl_unique_id, int nranks, int rank);
/* Sum of every rank's cumulative counters (RCCL all-reduce over xGMI, enqueued on `stream`),
 * OUT OF PLACE: the local counters are untouched, so any number of calls give the true job
 * totals.  gm_counters_global() reads the result of the last call.  Collective: every rank calls
 * it, the same number of times.  The ranks' agreement on (gen, n_counters) travels inside the sum
 * (a 10-word block beside the counters), so a call is one collective with no host synchronisation;
 * the first call, and the call after one whose block showed the ranks apart, agree synchronously
 * first.  Ranks on different generations or counter spaces: that call's totals are void --
 * gm_counters_global returns GM_E_COMM on every rank -- and the next call re-agrees (GM_E_COMM on
 * every rank while they still differ; no collective of mismatched size is ever issued). */
int         gm_counters_allreduce(gm_ctx *ctx, void *stream);
int         gm_counters_global(gm_ctx *ctx, uint64_t *out, size_t n);

/* $uri normalisation of n raw request paths (nginx ngx_http_parse_complex_uri
 * with merge_slashes on -- the step that turns the request line's path into the `$uri` every
 * location rule matches, nginx.ingress.tmpl:96 `location {{Path}}`).  Path i is
 * arena[off[i] .. off[i] + len[i]); '?' or '#' ends it.  The normalised bytes go to
 * out[off[i] ..) (never longer than the input; out may equal arena) and out_len[i] = their
 * length, or GM_NONE where nginx answers 400 (bad %-escape, NUL, ".." above the root).
 * Device pointers; asynchronous on `stream`; gm_sync(ctx, stream) completes it (the call clears
 * the stream's batch status, so the sync reports no match-batch overflow). */
int         gm_normalize_uris(gm_ctx *ctx, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                              uint32_t n, uint8_t *out, uint32_t *out_len, void *stream);

/* ---------------------------------------------------------------- HTTP/1.x wire parser
 * (the on-the-wire step before the engine.)  nginx's request-line / header /
 * body handling (ngx_http_parse_request_line, ngx_http_parse_header_line,
 * ngx_http_parse_complex_uri, ngx_http_process_request_headers, the chunked body filter) turns
 * raw request bytes into exactly the fields the templates' rules read: $request_method, $uri,
 * $args, $request_uri, $host, the header lines behind $http_* / $cookie_* (nginx.virtualserver.
 * tmpl:25-31 maps) and the body the Wallarm phase scans.  See DESIGN.md §4 for the rules. */
typedef struct gm_wire_msg {
    uint64_t off;             /* the request's bytes: wire[off .. off + len)               */
    uint32_t len;
    uint16_t port;            /* local listen port ($server_port)                          */
    uint16_t remote_port;
    uint8_t  flags;           /* connection: GM_REQ_HTTPS, GM_REQ_HTTP2, GM_WIRE_PROXY_DONE */
    uint8_t  raddr_len;       /* $remote_addr text length, <= 40                           */
    uint8_t  paddr_len;       /* GM_WIRE_PROXY_DONE: the connection's $proxy_protocol_addr  */
    uint8_t  pad;
    uint8_t  rid[16];         /* $request_id raw bytes                                     */
    uint8_t  raddr[40];       /* $remote_addr text (the TCP peer)                          */
    uint16_t proxy_port;      /* GM_WIRE_PROXY_DONE: the connection's $proxy_protocol_port  */
    uint8_t  pad2[2];
    uint8_t  paddr[46];       /* GM_WIRE_PROXY_DONE: $proxy_protocol_addr text             */
    uint8_t  pad3[2];
} gm_wire_msg;                /* 128 B */
/* PROXY protocol (`listen <port> proxy_protocol`, ConfigMap proxy-protocol: configmaps.go:145,
 * nginx.ingress.tmpl:33,38, nginx.virtualserver.tmpl:35,40, nginx.tmpl:82-83).  A message on such a
 * port is the start of its connection: it begins with a PROXY v1 ("PROXY TCP4 <src> <dst> <sport>
 * <dport>\r\n", "PROXY UNKNOWN ...\r\n") or v2 (binary) header, which nginx reads before the
 * request (ngx_proxy_protocol_read): its source address and port go to the record (paddr); a
 * missing or broken header closes the connection with no response -- the record is GM_REQ_INVALID
 * with status 444 (nginx's "close without a response" code).  GM_WIRE_PROXY_DONE marks a later
 * (keep-alive) request of such a connection: no header is read, and the caller hands the
 * connection's address in paddr / paddr_len / proxy_port (e.g. from its first request's record). */
#define GM_WIRE_PROXY_DONE 0x40u

/* Parse n requests into gm_req records + a payload arena (field order of gm_req, records
 * 16-B aligned and packed in request order).  Device pointers, asynchronous on `stream`;
 * *arena_len_dev (device) receives the arena's length -- hand it to gm_match_batch through
 * gm_batch.arena_len_dev, with arena_cap as gm_batch.arena_len.  A request nginx would reject
 * gets GM_REQ_INVALID and its status (400 / 501 / 505).  arena_cap >= the sum over requests of
 * align16(2 * len + raddr_len + 46) always suffices (46: the record's $proxy_protocol_addr after
 * raddr); gm_sync reports GM_E_OVERFLOW if it is exceeded. */
int         gm_parse_requests(gm_ctx *ctx, const uint8_t *wire, const gm_wire_msg *msgs, uint32_t n,
                              gm_req *reqs, uint8_t *arena, uint64_t arena_cap, uint64_t *arena_len_dev,
                              void *stream);

/* ---------------------------------------------------------------- upstream request URI
 * (nginx.org/rewrites.)  The URI a proxied request is sent upstream with, as
 * ngx_http_proxy_create_request builds it: a location whose proxy_pass has a URI part (the
 * template's {{$location.Rewrite}}, version1/nginx.ingress.tmpl:194-196, from nginx.org/rewrites
 * "serviceName=<svc> rewrite=<uri>", annotations.go:347-361,526-544) sends <uri> + the rest of
 * $uri after the location's prefix (%-escaped when the request's path held a '%' the parser saw
 * before any "/.", "//", '?' or '#') + "?" $args; any other proxying location sends $request_uri
 * unchanged.  out_len[i] = the length at out[out_off[i]]; GM_NONE for a verdict that is not a
 * proxy (or past out_cap: gm_sync then reports GM_E_OVERFLOW), GM_PEER_DEFER for a proxy_pass
 * with variables or of an older generation.  out_cap >= sum over requests of (longest URI part +
 * 3 * uri_len + args_len + ruri_len + 1) always suffices.  Device pointers, asynchronous. */
int         gm_upstream_uris(gm_ctx *ctx, const gm_batch *in, const gm_verdict *verdicts, uint8_t *out,
                             uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, void *stream);

/* ---------------------------------------------------------------- upstream peer selection
 * (the step after the path.)  The upstream blocks the templates render
 * (version1/nginx.ingress.tmpl:2-8, version2/nginx.virtualserver.tmpl:2-10) -- `server` lines
 * from the endpoints (ingress.go:277-301) and the LBMethod (default "random two least_conn",
 * config_params.go:123; ParseLBMethod parsing_helpers.go:89-161) -- restated per request:
 * round robin and least_conn (nginx's smooth weighted round robin / least_conn with its
 * current_weight tie-break, in request order), ip_hash, hash <key> [consistent], random,
 * random two [least_conn].  Peer ids are global indices into the generation's peer table
 * (upstreams in sorted-name order, servers in config order; gm_peer_address names them).
 *
 * The balancing state nginx keeps per peer (active connections, current_weight, down) is a
 * caller-owned device array of gm_stats_t.n_peers gm_peer_state entries, so several
 * independent balancers (e.g. one per worker) can share one ctx.  gm_select_peers reads it at
 * the start of the batch, applies the batch's picks in request order (conns += picks,
 * current_weight as nginx would leave it) and gm_release_peers ends connections.  Calls that
 * share a state array must be ordered on one stream. */
typedef struct gm_peer_state {
    uint32_t conns;           /* active connections (nginx peer->conns)                   */
    int32_t  current_weight;  /* smooth-WRR / least_conn tie-break state                  */
    uint32_t flags;           /* GM_PEER_DOWN: unavailable (down, or max_fails reached)   */
    uint32_t reserved;
} gm_peer_state;
#define GM_PEER_DOWN   0x1u
#define GM_PEER_DEFER  0xFFFFFFFEu  /* peer_out: the engine does not model this upstream / stale gen */
/* peer_out: GM_NONE = no peer (not a proxied verdict, or no live peer: nginx's 502) */

/* (Re)initialise a state array for the live generation: conns 0, current_weight 0, DOWN for
 * `server ... down`.  n_peers must equal gm_stats_t.n_peers.  Device pointer, async. */
int         gm_peers_init(gm_ctx *ctx, gm_peer_state *state, uint32_t n_peers, void *stream);
/* peer_out[i] = the peer of verdicts[i] (proxied verdicts of the live generation only).  `in` is
 * the batch the verdicts came from (device pointers: hash keys read its variables).  Async. */
int         gm_select_peers(gm_ctx *ctx, const gm_batch *in, const gm_verdict *verdicts, gm_peer_state *state,
                            uint32_t n_peers, uint32_t *peer_out, void *stream);
/* conns -= 1 for each peer id in peer_ids[0 .. n) (GM_NONE / GM_PEER_DEFER skipped).  Async. */
int         gm_release_peers(gm_ctx *ctx, const uint32_t *peer_ids, uint32_t n, gm_peer_state *state,
                             uint32_t n_peers, void *stream);
/* NGINX Plus runtime server update of one upstream, with no reload (SURVEY.md §8 f3 + A11):
 * Configurator.UpdateEndpoints / UpdateEndpointsMergeableIngress / UpdateEndpointsForVirtualServers
 * push each upstream's endpoints through Manager.UpdateServersInPlus(upstream, servers, cfg)
 * (configurator.go:442,467,489; interface manager.go:47; LocalManager manager.go:257-284, the Plus
 * API's UpdateHTTPServers).  Publishes the live tables with upstream `upstream`'s `server` list
 * replaced by servers[0..n) ("10.0.0.7:8080"; none `down` -- the ServerConfig's max_fails /
 * fail_timeout / slow_start do not change a pick), RCU-style: calls already enqueued keep the
 * tables they started with.  configVersion does not change, so neither does `gen`: verdicts of
 * either table stay valid for gm_select_peers (same upstream ids).  Counters carry over.  The
 * peer table is renumbered (gm_stats_t.n_peers, gm_peer_address): carry every balancer state
 * array over with gm_peers_migrate before its next gm_select_peers.  GM_E_INVAL: no upstream of
 * that name (the previous tables stay live).  GM_E_STALE: a gm_load_generation or another
 * gm_update_upstream published between this call's read of the live tables and its publish -- the
 * newer tables stay, nothing is overwritten (the reference refuses a Plus update whose
 * configVersion no longer matches, verifyConfigVersion, manager.go:258); re-issue the update.
 * Peer order: the kept servers in their previous relative order, then the added ones in the order
 * given (the Plus API appends a POSTed server); that order is parity-unpinned against a live Plus. */
int         gm_update_upstream(gm_ctx *ctx, const char *upstream, const char *const *servers, uint32_t n);
/* new_state[j] = old_state[i] where peer j of the live table is the server of the same upstream
 * and address as peer i of the table before the last gm_update_upstream (NGINX Plus keeps a kept
 * server's conns / weights / flags), else the initial state.  old_n / new_n: that table's and
 * the live gm_stats_t.n_peers.  Device pointers (distinct arrays), asynchronous on `stream`. */
int         gm_peers_migrate(gm_ctx *ctx, const gm_peer_state *old_state, uint32_t old_n,
                             gm_peer_state *new_state, uint32_t new_n, void *stream);
/* Host: the `server` address of a peer id ("10.0.0.1:8080") and its upstream id. */
int         gm_peer_address(gm_ctx *ctx, uint32_t peer, char *buf, size_t cap, uint32_t *upstream_id);

int         gm_stats(gm_ctx *ctx, gm_stats_t *out);
/* The constructs the live generation's compile rejected (n_rejected_other / n_rejected_pcre), one
 * per line, "context: directive args" -- the Manager wrapper logs them after Reload (SURVEY §8 b:
 * counted and logged, never a Reload error).  Returns the text's length (written up to cap - 1
 * bytes, NUL-terminated), or a negative GM_E_*. */
int         gm_rejects(gm_ctx *ctx, char *buf, size_t cap);
/* The source hash the library was built from, 16 lowercase hex digits ("unknown" if the build had
 * none): the same value as gm_stats_t.csrc_hash, readable without a context or a generation. */
const char *gm_build_hash(void);
/* Message of the calling thread's last failing call (thread-local; ctx is not consulted). */
const char *gm_last_error(gm_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* GPUMATCH_H */
