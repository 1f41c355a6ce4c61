/*
 * gm_oracle.c -- CPU ORACLE for the gpumatch engine.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline.  The product path (libgpumatch.so) never
 * links, loads or calls it.
 *
 * What it restates.  The reference (wallarm/ingress-plus 1.5.5) renders nginx config text
 * (the internal/configs version1 and version2 templates) and nginx 1.17.3 (build/Dockerfile:1)
 * classifies each request.  nginx's C source is not in /root/reference (third-party, pinned by
 * build/Dockerfile:1), so the request-time algorithm restated here is nginx 1.17.3's, written
 * from its published behaviour and anchored on the reference's call sites:
 *   - config tokens: ngx_conf_read_token (quotes, \" \' \\ \t \r \n escapes, ')' after quote)
 *   - host validation:   ngx_http_validate_host            
 *   - server by name:    ngx_http_find_virtual_server; exact > *.x > x.* > ~regex, first wins
 *                        (server_name at nginx.ingress.tmpl:53, nginx.virtualserver.tmpl:37,
 *                         default server nginx.tmpl:81-102, conf.d order nginx.tmpl:128-129)
 *   - server rewrite:    `if ($scheme = http) { return 301 ...; }` / x-forwarded-proto
 *                        (nginx.ingress.tmpl:76-88, nginx.virtualserver.tmpl:49-60)
 *   - location lookup:   ngx_http_core_find_location: '=' exact, longest prefix, '^~',
 *                        regex in config order, auto_redirect
 *   - error_page 418 = $var + return 418 (nginx.virtualserver.tmpl:78-83) and named locations
 *   - map:               ngx_http_map_find: lowercased hash keys, then regexes (only for a
 *                        non-empty value), else default   (virtualserver.go:299-426)
 *   - split_clients:     ngx_murmur_hash2 over $request_id, percent*0xffffffff/10000 bounds
 *                        (virtualserver.go:250-291, nginx.virtualserver.tmpl:17-23)
 *   - variables:         $http_* (ngx_http_variable_unknown_header, cookie / x-forwarded-for
 *                        joins), $cookie_* (ngx_http_parse_multi_header_lines), $arg_*
 *                        (ngx_http_arg), the 11 whitelisted variables (validation.go:353-365)
 *   - regex:             the real PCRE 8.39 (libpcre.so.3, the library nginx:1.17.3 links)
 *   - WAF layer:         build-defined signature set (ingress-plus_amd/gpumatch/sigs.py):
 *                        Aho-Corasick for literals, PCRE for regexes, per zone; mode from
 *                        wallarm_mode (annotations.go:294-330, nginx.ingress.tmpl:12-29).
 * Pinning: tests/golden holds the reference's own known answers (e2e KATs of
 * tests/suite/test_virtual_server_advanced_routing.py, docs/virtualserver-and-
 * virtualserverroute.md:264-271, virtualserver_test.go map structs) and PCRE-generated
 * vectors; see DESIGN.md §Oracle for what remains unpinned.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <arpa/inet.h>

#include "../include/gpumatch.h"

/* ---- PCRE 8.39 (no headers in the image: declare the stable C API) ---- */
typedef struct real_pcre pcre;
typedef struct pcre_extra pcre_extra;
extern pcre *pcre_compile(const char *, int, const char **, int *, const unsigned char *);
extern pcre_extra *pcre_study(const pcre *, int, const char **);
extern int pcre_exec(const pcre *, const pcre_extra *, const char *, int, int, int, int *, int);
#define PCRE_CASELESS 0x00000001
#define PCRE_STUDY_JIT_COMPILE 0x0001


/* ------------------------------------------------------------------ small utils */
typedef struct { const char *p; int n; } sv;

static __thread char g_err[512];
const char *orc_error(void) { return g_err; }
static void seterr(const char *m, const char *a) { snprintf(g_err, sizeof g_err, "%s%s", m, a ? a : ""); }

static int sv_eq(sv a, const char *b) { int n = (int)strlen(b); return a.n == n && memcmp(a.p, b, n) == 0; }
static int sv_eqsv(sv a, sv b) { return a.n == b.n && memcmp(a.p, b.p, a.n) == 0; }
static char *xstrndup(const char *p, int n) { char *s = malloc(n + 1); memcpy(s, p, n); s[n] = 0; return s; }
static unsigned char lc(unsigned char c) { return (c >= 'A' && c <= 'Z') ? (unsigned char)(c | 0x20) : c; }

/* ------------------------------------------------------------------ config tokens (ngx_conf_read_token) */
typedef struct dir {
    int nargs; char **args; int *alen;
    struct dir *kids; int nkids, capkids; int block;
} dir_t;

typedef struct { const char *s; int n; int i; char *buf; } lexer;

static void dir_push_arg(dir_t *d, const char *p, int n) {
    d->args = realloc(d->args, sizeof(char *) * (d->nargs + 1));
    d->alen = realloc(d->alen, sizeof(int) * (d->nargs + 1));
    d->args[d->nargs] = xstrndup(p, n); d->alen[d->nargs] = n; d->nargs++;
}

/* copy token with nginx escape rules */
static int unescape(const char *src, int n, char *dst) {
    int o = 0;
    for (int i = 0; i < n; i++) {
        if (src[i] == '\\' && i + 1 < n) {
            char c = src[i + 1];
            if (c == '"' || c == '\'' || c == '\\') { dst[o++] = c; i++; continue; }
            if (c == 't') { dst[o++] = '\t'; i++; continue; }
            if (c == 'r') { dst[o++] = '\r'; i++; continue; }
            if (c == 'n') { dst[o++] = '\n'; i++; continue; }
        }
        dst[o++] = src[i];
    }
    return o;
}

/* returns 0 = ';' ended, 1 = '{' block start, 2 = '}' block end, 3 = EOF, -1 error */
static int read_directive(lexer *L, dir_t *d) {
    char *buf = L->buf;
    for (;;) {
        while (L->i < L->n && strchr(" \t\r\n", L->s[L->i])) L->i++;
        if (L->i >= L->n) { return d->nargs ? -1 : 3; }
        char c = L->s[L->i];
        if (c == '#') { while (L->i < L->n && L->s[L->i] != '\n') L->i++; continue; }
        if (c == ';') { L->i++; return d->nargs ? 0 : -1; }
        if (c == '{') { L->i++; return 1; }
        if (c == '}') { L->i++; if (d->nargs) return -1; return 2; }
        if (c == '"' || c == '\'') {
            char q = c; int st = ++L->i;
            while (L->i < L->n && L->s[L->i] != q) { if (L->s[L->i] == '\\') L->i++; L->i++; }
            if (L->i >= L->n) { return -1; }
            int m = unescape(L->s + st, L->i - st, buf); L->i++;
            dir_push_arg(d, buf, m);
            if (L->i < L->n && L->s[L->i] == ')') { dir_push_arg(d, ")", 1); L->i++; }
            else if (L->i < L->n && !strchr(" \t\r\n;{", L->s[L->i])) { return -1; }
            continue;
        }
        int st = L->i; int var = 0;
        while (L->i < L->n) {
            char ch = L->s[L->i];
            if (ch == '{' && var) { L->i++; continue; }
            var = 0;
            if (ch == '\\') { L->i += 2; continue; }
            if (ch == '$') { var = 1; L->i++; continue; }
            if (strchr(" \t\r\n;{", ch)) break;
            L->i++;
        }
        if (L->i > L->n) L->i = L->n;
        int m = unescape(L->s + st, L->i - st, buf);
        dir_push_arg(d, buf, m);
    }
}

static int parse_block(lexer *L, dir_t *parent, int depth) {
    for (;;) {
        dir_t d; memset(&d, 0, sizeof d);
        int r = read_directive(L, &d);
        if (r == 3) return depth == 0 ? 0 : -1;
        if (r == 2) return depth > 0 ? 0 : -1;
        if (r < 0) return -1;
        if (r == 1) { d.block = 1; if (parse_block(L, &d, depth + 1) < 0) return -1; }
        if (parent->nkids == parent->capkids) {
            parent->capkids = parent->capkids ? parent->capkids * 2 : 16;
            parent->kids = realloc(parent->kids, sizeof(dir_t) * parent->capkids);
        }
        parent->kids[parent->nkids++] = d;
    }
}

/* ------------------------------------------------------------------ model */
enum { LK_PREFIX, LK_EXACT, LK_NOREGEX, LK_REGEX, LK_REGEX_I, LK_NAMED };

/* an address block (ngx_cidr_t): set_real_ip_from, allow / deny */
typedef struct { uint8_t fam; uint8_t addr[16], mask[16]; } ocidr_t;
/* an ngx_http_access_module rule (allow / deny): `all`, `unix:`, or a CIDR */
typedef struct { int deny, all, unix_; ocidr_t c; } oacc_t;
typedef struct { int n; oacc_t *r; } oacl_t;

typedef struct {
    int kind; char *path; int plen; pcre *re;
    int id, server;
    int auto_redirect;
    char *proxy_ups; int upstream_id; int has_proxy;
    char *pass_uri;           /* proxy_pass URI part (nginx.org/rewrites), NULL none */
    int pass_defer;           /* variables in proxy_pass, or a URI part nginx rejects */
    int pd_mask, has_pd;      /* wallarm_parser_disable in the location (DEC bits) */
    int has_return; int ret_code;
    char *err418;             /* error_page 418 = <complex value> */
    int waf_mode;
    int pcre_only;            /* regex location the engine rejects (orc_pcre_only) */
    int nested;               /* contains location / if / rewrite: deferred (GM_ACT_UNSUPPORTED) */
    int unknown;              /* a directive outside the neutral set (default-deny): deferred */
    char *cmbs;               /* client_max_body_size written here, NULL: inherited */
    int64_t body_max;         /* the limit in effect (-1: none), set once the server is known */
    pcre *relaxed;            /* its superset pattern (orc_relax), NULL = none */
    oacl_t acc;               /* allow / deny written here (n 0: inherited) */
    int stub;                 /* stub_status: a content handler answering 200 */
} loc_t;

typedef struct { char *var; int op; char *val; pcre *re; int code; char *text; int is_return_only; int unsupported; } sif_t;

/* ngx_http_realip_module settings (set_real_ip_from / real_ip_header / real_ip_recursive) */
typedef struct {
    int nfrom; char **from;    /* NULL (nfrom 0) = unset */
    char *header;              /* NULL = unset */
    int recursive;             /* -1 unset */
} orip_t;

typedef struct {
    int id; int nports; int ports[16]; int ssl[16]; int def[16]; int pp[16];   /* pp: proxy_protocol */
    char *cmbs;               /* server-level client_max_body_size, NULL inherited */
    int64_t body_max;         /* limit in effect for a request with no location (-1 none) */
    orip_t rip;
    /* realip in effect: type 0 none, 1 X-Real-IP, 2 X-Forwarded-For, 3 proxy_protocol, 4 other
     * header (hdr lowercase), 5 unknowable (a set_real_ip_from that is no address) */
    int rtype, rrec; char hdr[128]; int ncidr; ocidr_t *cidr;
    int pd_mask;              /* server-level wallarm_parser_disable */
    int nnames; char **names; int *nlen; pcre **nre;
    int nifs; sif_t *ifs;
    int nlocs; int *locs;
    int waf_mode;
    oacl_t acc;               /* server-level allow / deny */
} srv_t;

typedef struct { char *key; int klen; pcre *re; int is_re; char *val; } mparam_t;
typedef struct { char *src; char *var; int np; mparam_t *p; char *defval; int hostnames; } map_t;
typedef struct { uint32_t bound; int star; char *val; } part_t;
typedef struct { char *src; char *var; int np; part_t *p; } split_t;

typedef struct {
    int kind; int nocase; int zones; uint8_t *lit; int len; pcre *re; pcre_extra *ex;
    /* prefilter: literals one of which every match of the regex contains (lowercased), nfac 0:
     * none (the regex runs on every zone) */
    char fac[16][64]; int flen[16]; int nfac;
    char *pattern_src;
} sig_t;

/* an upstream block (version1/nginx.ingress.tmpl:2-8, version2/nginx.virtualserver.tmpl:2-10) */
enum { OM_RR, OM_LEAST_CONN, OM_IP_HASH, OM_HASH, OM_CHASH, OM_RANDOM, OM_RANDOM2, OM_DEFER };
typedef struct { uint32_t hash; int peer; } opoint_t;
typedef struct {
    char *name; dir_t *d;
    int method; char *key;
    int npeers; char **addr; int *down;
    int first_peer;
    opoint_t *ring; int nring;
    char *sticky;             /* NGINX Plus `sticky cookie <name>`: "$cookie_<name>", NULL none */
} oups_t;

typedef struct orc_ctx {
    uint32_t gen;
    oups_t *udef; int nudef;        /* upstream blocks in config order */
    oups_t **uby; int total_peers;  /* per sorted upstream id (NULL: no block) */
    srv_t *srv; int nsrv;
    loc_t *loc; int nloc;
    map_t *map; int nmap;
    split_t *spl; int nspl;
    char **ups; int nups;
    int http_waf;
    char *http_cmbs; orip_t http_rip; int http_unknown;
    oacl_t http_acc;          /* http-level allow / deny */
    sig_t *sig; int nsig;
    int decoders;             /* the signature set's "@decoders" (DEC bits) */
    /* CPU-baseline engine (orc_set_prefilter): a regex runs on a zone only if its required factor
     * occurs there (Aho-Corasick over the factors), as a competent CPU WAF would do */
    int prefilter;
    int32_t *fac_next; int32_t *fac_out; int32_t *fac_dict; int32_t *fac_pat_next; int32_t *fac_pat_re;
    /* Aho-Corasick over case-folded bytes */
    int32_t *ac_next; int ac_states; int32_t *ac_out; int32_t *ac_dict; int32_t *ac_pat_next; int *ac_pat;
} orc_ctx;

static int waf_mode_of(const char *s) {
    if (!strcmp(s, "off")) return GM_WAF_OFF;
    if (!strcmp(s, "monitoring")) return GM_WAF_MONITORING;
    if (!strcmp(s, "safe_blocking")) return GM_WAF_SAFE_BLOCKING;
    if (!strcmp(s, "block")) return GM_WAF_BLOCK;
    return GM_WAF_OFF;
}

/* Wallarm parser names -> the engine's decoder bits (include/gpumatch.h GM_DEC_*) */
static int dec_bit(const char *nm) {
    if (!strcmp(nm, "percent")) return GM_DEC_PERCENT;
    if (!strcmp(nm, "urlenc")) return GM_DEC_URLENC;
    if (!strcmp(nm, "json_doc") || !strcmp(nm, "json")) return GM_DEC_JSON;
    if (!strcmp(nm, "base64")) return GM_DEC_BASE64;
    return 0;
}

static pcre *re_compile(const char *pat, int caseless) {
    const char *e; int eo;
    pcre *r = pcre_compile(pat, caseless ? PCRE_CASELESS : 0, &e, &eo, NULL);
    return r;
}

/* PCRE-only syntax, restated from the engine's contract (rejected at compile
 * time and counted): backreferences \1-\9 \g \k, \K, lookaround (?= (?! (?<= (?<!, atomic (?>,
 * recursion / conditionals / callouts / named groups (?R (?( (?C (?P (?& (?| (?<digit>,
 * possessive quantifiers *+ ++ ?+ }+.  A request that reaches such a regex location (no earlier
 * regex matched) is GM_ACT_UNSUPPORTED: nginx's answer depends on PCRE, the engine defers it. */
int orc_pcre_only(const char *p) {
    size_t n = strlen(p);
    int in_cls = 0;
    for (size_t i = 0; i < n; i++) {
        char ch = p[i];
        if (ch == '\\' && i + 1 < n) {
            char e = p[i + 1];
            if (!in_cls && ((e >= '1' && e <= '9') || e == 'g' || e == 'k' || e == 'K')) return 1;
            i++;
            continue;
        }
        if (in_cls) { if (ch == ']') in_cls = 0; continue; }
        if (ch == '[') { in_cls = 1; if (i + 1 < n && p[i + 1] == '^') i++; if (i + 1 < n && p[i + 1] == ']') i++; continue; }
        if (ch == '(' && i + 2 < n && p[i + 1] == '?') {
            char a = p[i + 2];
            if (a == '=' || a == '!' || a == '>' || a == 'R' || a == '(' || a == 'C' || a == 'P' || a == '&' ||
                a == '|' || (a >= '0' && a <= '9')) return 1;
            if (a == '<' && i + 3 < n && (p[i + 3] == '=' || p[i + 3] == '!')) return 1;
            continue;
        }
        if ((ch == '*' || ch == '+' || ch == '?' || ch == '}') && i + 1 < n && p[i + 1] == '+') {
            if (ch == '?' && i > 0 && p[i - 1] == '(') continue;
            return 1;
        }
    }
    return 0;
}

/* The engine's superset of a PCRE-only pattern (gm_compile.cpp relax_pcre_only, restated):
 * lookaround groups dropped, (?> -> (?:, possessive -> greedy, \K dropped, backreferences ->
 * (?:.|\n)*.  Returns a malloc'd string, or NULL when the engine has no superset. */
char *orc_relax(const char *p) {
    size_t n = strlen(p), k = 0;
    char *o = malloc(n * 10 + 16);
    int cls = 0;
    for (size_t i = 0; i < n; i++) {
        char ch = p[i];
        if (ch == '\\' && i + 1 < n) {
            char e = p[i + 1];
            if (!cls && e >= '1' && e <= '9') { memcpy(o + k, "(?:.|\\n)*", 9); k += 9; i++; continue; }
            if (!cls && e == 'K') { i++; continue; }
            if (!cls && (e == 'g' || e == 'k')) { free(o); return NULL; }
            o[k++] = ch; o[k++] = e; i++;
            continue;
        }
        if (cls) { o[k++] = ch; if (ch == ']') cls = 0; continue; }
        if (ch == '[') {
            cls = 1; o[k++] = ch;
            if (i + 1 < n && p[i + 1] == '^') o[k++] = p[++i];
            if (i + 1 < n && p[i + 1] == ']') o[k++] = p[++i];
            continue;
        }
        if (ch == '(' && i + 2 < n && p[i + 1] == '?') {
            char a = p[i + 2];
            int look = a == '=' || a == '!' || (a == '<' && i + 3 < n && (p[i + 3] == '=' || p[i + 3] == '!'));
            if (look) {
                int depth = 0, c2 = 0;
                size_t j = i;
                for (; j < n; j++) {
                    if (p[j] == '\\') { j++; continue; }
                    if (c2) { if (p[j] == ']') c2 = 0; continue; }
                    if (p[j] == '[') { c2 = 1; if (j + 1 < n && p[j + 1] == '^') j++; if (j + 1 < n && p[j + 1] == ']') j++; continue; }
                    if (p[j] == '(') depth++;
                    else if (p[j] == ')' && --depth == 0) break;
                }
                if (j >= n) { free(o); return NULL; }
                i = j;
                if (i + 1 < n && (p[i + 1] == '*' || p[i + 1] == '+' || p[i + 1] == '?' || p[i + 1] == '{')) { free(o); return NULL; }
                continue;
            }
            if (a == '>') { memcpy(o + k, "(?:", 3); k += 3; i += 2; continue; }
            if (a == 'R' || a == '(' || a == 'C' || a == 'P' || a == '&' || a == '|' || (a >= '0' && a <= '9')) { free(o); return NULL; }
        }
        if ((ch == '*' || ch == '+' || ch == '?' || ch == '}') && i + 1 < n && p[i + 1] == '+' &&
            !(ch == '?' && i > 0 && p[i - 1] == '(')) { o[k++] = ch; i++; continue; }
        o[k++] = ch;
    }
    o[k] = 0;
    return o;
}

static int cmp_str(const void *a, const void *b) { return strcmp(*(char *const *)a, *(char *const *)b); }

/* ------------------------------------------------------------------ default-deny
 * The engine's contract (gm_compile.cpp neutral_directive), restated: the directives known to
 * leave a request's verdict alone.  Any other directive in a server or location (snippets) makes
 * the requests reaching it GM_ACT_UNSUPPORTED; at http level it defers every server's requests
 * after their server rewrite phase. */
static int orc_neutral(const char *n, int ctx /* 0 http, 1 server, 2 location */) {
    static const char *pre[] = {"proxy_", "grpc_", "ssl_", "gzip", "http2_", "open_file_cache", "sub_filter",
                                "keepalive_", "wallarm_", NULL};
    static const char *any[] = {
        "add_header", "add_trailer", "access_log", "error_log", "log_not_found", "log_subrequest",
        "default_type", "charset", "charset_types", "source_charset", "override_charset", "expires", "etag",
        "send_timeout", "client_body_timeout", "client_body_buffer_size", "client_body_temp_path",
        "client_header_timeout", "sendfile", "sendfile_max_chunk", "tcp_nodelay", "tcp_nopush",
        "server_tokens", "status_zone", "chunked_transfer_encoding", "output_buffers", "postpone_output",
        "lingering_close", "lingering_time", "lingering_timeout", "reset_timedout_connection", "resolver",
        "resolver_timeout", "auth_jwt_key_file", "auth_jwt_leeway", "port_in_redirect",
        "server_name_in_redirect", "absolute_redirect", "msie_padding", "msie_refresh", NULL};
    static const char *http[] = {
        "log_format", "server_names_hash_max_size", "server_names_hash_bucket_size", "variables_hash_max_size",
        "variables_hash_bucket_size", "types_hash_max_size", "types_hash_bucket_size", "map_hash_max_size",
        "map_hash_bucket_size", "limit_req_zone", "limit_conn_zone", "proxy_cache_path", "geo", "match",
        "js_include", "js_import", "keyval_zone", "types", NULL};
    for (int i = 0; pre[i]; i++) if (!strncmp(n, pre[i], strlen(pre[i]))) return 1;
    for (int i = 0; any[i]; i++) if (!strcmp(n, any[i])) return 1;
    if (ctx == 2) return !strcmp(n, "health_check");
    if (ctx == 0) for (int i = 0; http[i]; i++) if (!strcmp(n, http[i])) return 1;
    return 0;
}

/* client_max_body_size (ngx_parse_offset): digits + optional k/m/g; 0 = unlimited (-1 here);
 * -2 = not a size */
static int64_t orc_size(const char *v) {
    int n = (int)strlen(v);
    if (n == 0) return -2;
    int64_t scale = 1;
    char u = v[n - 1];
    if (u == 'k' || u == 'K') { scale = 1024; n--; }
    else if (u == 'm' || u == 'M') { scale = 1 << 20; n--; }
    else if (u == 'g' || u == 'G') { scale = 1 << 30; n--; }
    if (n == 0) return -2;
    int64_t x = 0;
    for (int i = 0; i < n; i++) {
        if (!isdigit((unsigned char)v[i])) return -2;
        if (x < ((int64_t)1 << 50)) x = x * 10 + (v[i] - '0');
    }
    if (x >= ((int64_t)1 << 50)) return -1;
    x *= scale;
    return x == 0 ? -1 : x;
}

/* ------------------------------------------------------------------ addresses (nginx 1.17.3)
 * ngx_inet_addr, ngx_inet6_addr, ngx_parse_addr[_port], ngx_ptocidr, ngx_cidr_match,
 * ngx_inet6_ntop -- restated from nginx's behaviour for the realip module. */
static int o_inet4(const char *t, int n, uint8_t *out) {
    uint32_t a = 0, oct = 0; int dots = 0;
    for (const char *p = t; p < t + n; p++) {
        if (*p >= '0' && *p <= '9') { oct = oct * 10 + (uint32_t)(*p - '0'); if (oct > 255) return 0; }
        else if (*p == '.') { a = (a << 8) + oct; oct = 0; dots++; }
        else return 0;
    }
    if (dots != 3) return 0;
    a = (a << 8) + oct;
    if (a == 0xFFFFFFFFu) return 0;        /* INADDR_NONE */
    out[0] = a >> 24; out[1] = a >> 16; out[2] = a >> 8; out[3] = a;
    return 1;
}
static int o_inet6(const char *p, int len, uint8_t *addr) {
    if (len == 0) return 0;
    uint8_t *zero = NULL, *a0 = addr;
    const char *digit = NULL; int len4 = 0, nibbles = 0, n = 8; unsigned word = 0;
    if (p[0] == ':') { p++; len--; }
    for (; len; len--) {
        char c = *p++;
        if (c == ':') {
            if (nibbles) {
                digit = p; len4 = len;
                *addr++ = (uint8_t)(word >> 8); *addr++ = (uint8_t)word;
                if (--n) { nibbles = 0; word = 0; continue; }
            } else if (zero == NULL) { digit = p; len4 = len; zero = addr; continue; }
            return 0;
        }
        if (c == '.' && nibbles) {
            uint8_t v4[4];
            if (n < 2 || digit == NULL || !o_inet4(digit, len4 - 1, v4)) return 0;
            *addr++ = v4[0]; *addr++ = v4[1];
            word = (unsigned)v4[2] << 8 | v4[3];
            n--;
            break;
        }
        if (++nibbles > 4) return 0;
        if (c >= '0' && c <= '9') { word = word * 16 + (unsigned)(c - '0'); continue; }
        c |= 0x20;
        if (c >= 'a' && c <= 'f') { word = word * 16 + (unsigned)(c - 'a') + 10; continue; }
        return 0;
    }
    if (nibbles == 0 && zero == NULL) return 0;
    *addr++ = (uint8_t)(word >> 8); *addr++ = (uint8_t)word;
    if (--n) {
        if (zero) {
            n *= 2;
            uint8_t *s = addr - 1, *d = s + n;
            while (s >= zero) *d-- = *s--;
            memset(zero, 0, (size_t)n);
            return 1;
        }
    } else if (zero == NULL) return 1;
    (void)a0;
    return 0;
}
typedef struct { int fam; uint8_t b[16]; int port; } oaddr_t;
static int o_parse_addr(const char *t, int n, oaddr_t *a) {
    a->port = 0;
    if (o_inet4(t, n, a->b)) { a->fam = 4; return 1; }
    if (o_inet6(t, n, a->b)) { a->fam = 6; return 1; }
    return 0;
}
static int o_parse_addr_port(const char *text, int len, oaddr_t *a) {
    if (o_parse_addr(text, len, a)) return 1;
    const char *last = text + len, *p;
    if (len && text[0] == '[') {
        p = memchr(text, ']', (size_t)len);
        if (p == NULL || p == last - 1 || *++p != ':') return 0;
        text++; len -= 2;
    } else {
        p = memchr(text, ':', (size_t)len);
        if (p == NULL) return 0;
    }
    p++;
    int plen = (int)(last - p);
    if (plen <= 0 || plen > 9) return 0;
    long port = 0;
    for (int i = 0; i < plen; i++) { if (!isdigit((unsigned char)p[i])) return 0; port = port * 10 + (p[i] - '0'); }
    if (port < 1 || port > 65535) return 0;
    len -= plen + 1;
    if (!o_parse_addr(text, len, a)) return 0;
    a->port = (int)port;
    return 1;
}
static int o_ptocidr(const char *t, ocidr_t *c) {
    const char *sl = strchr(t, '/');
    int alen = sl ? (int)(sl - t) : (int)strlen(t);
    oaddr_t a;
    memset(c, 0, sizeof *c);
    if (!o_parse_addr(t, alen, &a)) return 0;
    int nb = a.fam == 4 ? 4 : 16, bits = nb * 8;
    if (sl) {
        const char *q = sl + 1;
        if (!*q) return 0;
        bits = 0;
        for (; *q; q++) { if (!isdigit((unsigned char)*q)) return 0; bits = bits * 10 + (*q - '0'); if (bits > 1000) return 0; }
        if (bits > nb * 8) return 0;
    }
    c->fam = (uint8_t)a.fam;
    for (int i = 0; i < nb; i++) {
        int k = bits - 8 * i;
        c->mask[i] = k >= 8 ? 0xFF : k <= 0 ? 0 : (uint8_t)(0xFF << (8 - k));
        c->addr[i] = a.b[i] & c->mask[i];
    }
    return 1;
}
static int o_cidr_match(const srv_t *S, const oaddr_t *a) {
    int fam = a->fam; const uint8_t *b = a->b;
    static const uint8_t mapped[12] = {0,0,0,0,0,0,0,0,0,0,0xFF,0xFF};
    if (fam == 6 && !memcmp(b, mapped, 12)) { fam = 4; b += 12; }
    for (int i = 0; i < S->ncidr; i++) {
        const ocidr_t *c = &S->cidr[i];
        if (c->fam != fam) continue;
        int ok = 1;
        for (int k = 0; k < (fam == 4 ? 4 : 16) && ok; k++) ok = (b[k] & c->mask[k]) == c->addr[k];
        if (ok) return 1;
    }
    return 0;
}
/* allow / deny <arg> (ngx_http_access_rule, nginx 1.17.3): `all`, `unix:`, or an address / CIDR */
/* 0: an argument the engine does not read (a host name): the directive is deferred like an
 * unknown one, and no rule is added */
static int oacl_add(oacl_t *L, const char *verb, const char *arg) {
    oacc_t a; memset(&a, 0, sizeof a);
    a.deny = !strcmp(verb, "deny");
    if (!strcmp(arg, "all")) a.all = 1;
    else if (!strcmp(arg, "unix:")) a.unix_ = 1;
    else if (!o_ptocidr(arg, &a.c)) return 0;
    L->r = realloc(L->r, sizeof(oacc_t) * (size_t)(L->n + 1));
    L->r[L->n++] = a;
    return 1;
}
/* ngx_http_access_handler with satisfy all: 1 = a deny rule matched the client address (403),
 * 0 = allowed.  An IPv4 client walks the rules for AF_INET in config order (IPv4 CIDRs and `all`);
 * an IPv4-mapped IPv6 client walks them too when there are any (and only them), other IPv6
 * clients the AF_INET6 ones (IPv6 CIDRs and `all`); `unix:` rules never see a TCP client. */
static int oacl_denies(const oacl_t *L, const oaddr_t *a) {
    int fam = a->fam; const uint8_t *b = a->b;
    static const uint8_t mapped[12] = {0,0,0,0,0,0,0,0,0,0,0xFF,0xFF};
    int has4 = 0;
    for (int i = 0; i < L->n; i++) if (L->r[i].all || (!L->r[i].unix_ && L->r[i].c.fam == 4)) has4 = 1;
    if (fam == 6 && has4 && !memcmp(b, mapped, 12)) { fam = 4; b += 12; }
    for (int i = 0; i < L->n; i++) {
        const oacc_t *r = &L->r[i];
        if (r->unix_) continue;
        if (!r->all) {
            if (r->c.fam != fam) continue;
            int ok = 1;
            for (int k = 0; k < (fam == 4 ? 4 : 16) && ok; k++) ok = (b[k] & r->c.mask[k]) == r->c.addr[k];
            if (!ok) continue;
        }
        return r->deny;
    }
    return 0;
}
static int o_ntop(const oaddr_t *a, char *out) {
    if (a->fam == 4) return sprintf(out, "%u.%u.%u.%u", a->b[0], a->b[1], a->b[2], a->b[3]);
    const uint8_t *p = a->b;
    int zero = -1, last = -1, max = 1, n = 0;
    for (int i = 0; i < 16; i += 2) {
        if (p[i] || p[i + 1]) { if (max < n) { zero = last; max = n; } n = 0; continue; }
        if (n++ == 0) last = i;
    }
    if (max < n) { zero = last; max = n; }
    char *d = out;
    n = 16;
    if (zero == 0) {
        if ((max == 5 && p[10] == 0xff && p[11] == 0xff) || max == 6 || (max == 7 && p[14] != 0 && p[15] != 1)) n = 12;
        *d++ = ':';
    }
    for (int i = 0; i < n; i += 2) {
        if (i == zero) { *d++ = ':'; i += (max - 1) * 2; continue; }
        d += sprintf(d, "%x", p[i] * 256 + p[i + 1]);
        if (i < 14) *d++ = ':';
    }
    if (n == 12) d += sprintf(d, "%u.%u.%u.%u", p[12], p[13], p[14], p[15]);
    *d = 0;
    return (int)(d - out);
}
/* test export: ngx_parse_addr_port + ngx_sock_ntop of a text -> "<text> <port>", -1 not an address */
int orc_inet(const char *t, int n, char *out, int cap) {
    oaddr_t a;
    if (!o_parse_addr_port(t, n, &a)) return -1;
    char x[64];
    o_ntop(&a, x);
    return snprintf(out, (size_t)cap, "%s %d", x, a.port);
}

/* ngx_http_get_forwarded_addr_internal, recursive as in nginx: 0 declined, 1 ok, 2 done */
static int o_fwd_internal(const srv_t *S, oaddr_t *addr, const char *xff, int xfflen) {
    if (!o_cidr_match(S, addr)) return 0;
    if (xfflen <= 0) return 0;     /* nginx reads the byte before an empty value: never an address */
    const char *p;
    for (p = xff + xfflen - 1; p > xff; p--, xfflen--) if (*p != ' ' && *p != ',') break;
    for (; p > xff; p--) if (*p == ' ' || *p == ',') { p++; break; }
    oaddr_t pa;
    if (!o_parse_addr_port(p, xfflen - (int)(p - xff), &pa)) return 0;
    *addr = pa;
    if (S->rrec && p > xff) {
        int rc = o_fwd_internal(S, addr, xff, (int)(p - 1 - xff));
        return rc == 0 ? 2 : rc;
    }
    return 1;
}

/* ------------------------------------------------------------------ build from directives */
typedef struct { orc_ctx *c; dir_t **confd; int nconfd; } build_t;

static void add_server(build_t *B, dir_t *s, int http_waf);

/* set_real_ip_from / real_ip_header / real_ip_recursive into R; 0 if d is none of them */
static int orc_realip_dir(orip_t *R, dir_t *d) {
    const char *n = d->args[0];
    if (d->nargs != 2) return 0;
    if (!strcmp(n, "set_real_ip_from")) {
        R->from = realloc(R->from, sizeof(char *) * (R->nfrom + 1));
        R->from[R->nfrom++] = strdup(d->args[1]);
        return 1;
    }
    if (!strcmp(n, "real_ip_header")) { R->header = strdup(d->args[1]); return 1; }
    if (!strcmp(n, "real_ip_recursive")) { R->recursive = !strcmp(d->args[1], "on"); return 1; }
    return 0;
}

static void walk_http(build_t *B, dir_t *h) {
    orc_ctx *c = B->c;
    for (int i = 0; i < h->nkids; i++) {
        dir_t *d = &h->kids[i];
        if (!d->nargs) continue;
        const char *n = d->args[0];
        if (!strcmp(n, "include") && d->nargs == 2 && strstr(d->args[1], "conf.d/")) {
            for (int k = 0; k < B->nconfd; k++) walk_http(B, B->confd[k]);
        } else if (!strcmp(n, "include") && d->nargs == 2 &&
                   (!strcmp(d->args[1], "/etc/nginx/mime.types") || !strcmp(d->args[1], "mime.types") ||
                    !strcmp(d->args[1], "/etc/nginx/config-version.conf"))) {
        } else if (!strcmp(n, "client_max_body_size") && d->nargs == 2) {
            c->http_cmbs = strdup(d->args[1]);
        } else if ((!strcmp(n, "allow") || !strcmp(n, "deny")) && d->nargs == 2 && oacl_add(&c->http_acc, n, d->args[1])) {
        } else if (orc_realip_dir(&c->http_rip, d)) {
        } else if (!strcmp(n, "wallarm_mode") && d->nargs == 2) {
            c->http_waf = waf_mode_of(d->args[1]);
        } else if (!strcmp(n, "upstream") && d->nargs == 2 && d->block) {
            c->ups = realloc(c->ups, sizeof(char *) * (c->nups + 1));
            c->ups[c->nups++] = strdup(d->args[1]);
            c->udef = realloc(c->udef, sizeof(oups_t) * (c->nudef + 1));
            memset(&c->udef[c->nudef], 0, sizeof(oups_t));
            c->udef[c->nudef].name = strdup(d->args[1]); c->udef[c->nudef].d = d;
            c->nudef++;
        } else if (!strcmp(n, "map") && d->nargs == 3 && d->block) {
            map_t m; memset(&m, 0, sizeof m);
            m.src = strdup(d->args[1]); m.var = strdup(d->args[2] + 1);
            for (int k = 0; k < d->nkids; k++) {
                dir_t *p = &d->kids[k];
                if (p->nargs == 1 && !strcmp(p->args[0], "hostnames")) { m.hostnames = 1; continue; }
                if (p->nargs == 1 && !strcmp(p->args[0], "volatile")) continue;
                if (p->nargs != 2) continue;
                if (!strcmp(p->args[0], "default")) { m.defval = strdup(p->args[1]); continue; }
                if (!strcmp(p->args[0], "include")) continue;
                mparam_t mp; memset(&mp, 0, sizeof mp);
                mp.val = strdup(p->args[1]);
                const char *k0 = p->args[0]; int kl = p->alen[0];
                if (kl && k0[0] == '~') {
                    int ci = (kl > 1 && k0[1] == '*');
                    mp.is_re = 1; mp.re = re_compile(k0 + 1 + ci, ci);
                } else {
                    if (kl && k0[0] == '\\') { k0++; kl--; }
                    mp.key = xstrndup(k0, kl); mp.klen = kl;
                    for (int q = 0; q < kl; q++) mp.key[q] = (char)lc((unsigned char)mp.key[q]);
                }
                m.p = realloc(m.p, sizeof(mparam_t) * (m.np + 1)); m.p[m.np++] = mp;
            }
            c->map = realloc(c->map, sizeof(map_t) * (c->nmap + 1)); c->map[c->nmap++] = m;
        } else if (!strcmp(n, "split_clients") && d->nargs == 3 && d->block) {
            split_t s; memset(&s, 0, sizeof s);
            s.src = strdup(d->args[1]); s.var = strdup(d->args[2] + 1);
            uint64_t last = 0; uint32_t sum = 0;
            for (int k = 0; k < d->nkids; k++) {
                dir_t *p = &d->kids[k];
                if (p->nargs != 2) continue;
                part_t pt; memset(&pt, 0, sizeof pt); pt.val = strdup(p->args[1]);
                if (!strcmp(p->args[0], "*")) { pt.star = 1; pt.bound = 0; }
                else {
                    /* ngx_atofp(value, len-1, 2): fixed point with 2 decimals */
                    const char *v = p->args[0]; int len = p->alen[0] - 1; uint32_t pc = 0; int dot = -1, dec = 0;
                    for (int q = 0; q < len; q++) {
                        if (v[q] == '.') { dot = q; continue; }
                        if (dot >= 0) { if (dec < 2) { pc = pc * 10 + (v[q] - '0'); dec++; } }
                        else pc = pc * 10 + (v[q] - '0');
                    }
                    while (dec < 2) { pc *= 10; dec++; }
                    sum += pc;
                    last += (uint64_t)pc * 0xffffffffull / 10000;
                    pt.bound = (uint32_t)last;
                }
                s.p = realloc(s.p, sizeof(part_t) * (s.np + 1)); s.p[s.np++] = pt;
            }
            (void)sum;
            c->spl = realloc(c->spl, sizeof(split_t) * (c->nspl + 1)); c->spl[c->nspl++] = s;
        } else if (!strcmp(n, "server") && d->block) {
            add_server(B, d, c->http_waf);
        } else if (!(!strcmp(n, "map") || !strcmp(n, "split_clients") || !strcmp(n, "upstream")) &&
                   !orc_neutral(n, 0)) {
            c->http_unknown = 1;
        }
    }
}

static void add_location(build_t *B, srv_t *S, dir_t *d, int srv_waf) {
    orc_ctx *c = B->c;
    loc_t L; memset(&L, 0, sizeof L);
    L.id = c->nloc; L.server = S->id; L.waf_mode = srv_waf; L.upstream_id = -1;
    const char *a1 = d->nargs > 1 ? d->args[1] : "";
    if (d->nargs == 3) {
        if (!strcmp(a1, "=")) L.kind = LK_EXACT;
        else if (!strcmp(a1, "^~")) L.kind = LK_NOREGEX;
        else if (!strcmp(a1, "~")) L.kind = LK_REGEX;
        else if (!strcmp(a1, "~*")) L.kind = LK_REGEX_I;
        L.path = strdup(d->args[2]); L.plen = d->alen[2];
    } else {
        L.path = strdup(a1); L.plen = d->alen[1];
        L.kind = (L.plen && L.path[0] == '@') ? LK_NAMED : LK_PREFIX;
    }
    if (L.kind == LK_REGEX || L.kind == LK_REGEX_I) {
        L.re = re_compile(L.path, L.kind == LK_REGEX_I);
        L.pcre_only = orc_pcre_only(L.path);
        if (L.pcre_only) {
            char *rp = orc_relax(L.path);
            if (rp) { L.relaxed = re_compile(rp, L.kind == LK_REGEX_I); free(rp); }
        }
    }
    for (int i = 0; i < d->nkids; i++) {
        dir_t *k = &d->kids[i];
        if (!k->nargs) continue;
        if ((!strcmp(k->args[0], "proxy_pass") || !strcmp(k->args[0], "grpc_pass")) && k->nargs == 2) {
            const char *u = k->args[1];
            const char *p = strstr(u, "://"); p = p ? p + 3 : u;
            int n = 0; while (p[n] && p[n] != '/' && p[n] != '$') n++;
            L.proxy_ups = xstrndup(p, n); L.has_proxy = 1;
            L.pass_uri = p[n] == '/' ? strdup(p + n) : NULL;
            L.pass_defer = strchr(u, '$') != NULL ||
                           (L.pass_uri && (!strcmp(k->args[0], "grpc_pass") || L.kind == LK_REGEX ||
                                           L.kind == LK_REGEX_I || L.kind == LK_NAMED));
        } else if (!strcmp(k->args[0], "return") && k->nargs >= 2) {
            L.has_return = 1; L.ret_code = atoi(k->args[1]);
            if (!isdigit((unsigned char)k->args[1][0])) L.ret_code = 302;
        } else if (!strcmp(k->args[0], "error_page") && k->nargs == 4 && !strcmp(k->args[1], "418") &&
                   !strcmp(k->args[2], "=")) {
            L.err418 = strdup(k->args[3]);
        } else if (!strcmp(k->args[0], "wallarm_mode") && k->nargs == 2) {
            L.waf_mode = waf_mode_of(k->args[1]);
        } else if (!strcmp(k->args[0], "wallarm_parser_disable") && k->nargs == 2) {
            L.pd_mask |= dec_bit(k->args[1]); L.has_pd = 1;
        } else if (!strcmp(k->args[0], "location") || !strcmp(k->args[0], "if") || !strcmp(k->args[0], "rewrite")) {
            L.nested = 1;   /* nested location / if / rewrite: outside the restated subset */
        } else if (!strcmp(k->args[0], "client_max_body_size") && k->nargs == 2) {
            L.cmbs = strdup(k->args[1]);
        } else if ((!strcmp(k->args[0], "allow") || !strcmp(k->args[0], "deny")) && k->nargs == 2 &&
                   oacl_add(&L.acc, k->args[0], k->args[1])) {
        } else if (!strcmp(k->args[0], "stub_status") && (k->nargs == 1 || (k->nargs == 2 && !strcmp(k->args[1], "on")))) {
            L.stub = 1;
        } else if (!strcmp(k->args[0], "error_page") && k->nargs >= 3 &&
                   !strncmp(k->args[k->nargs - 1], "@grpcerror", 10)) {
            /* gRPC error pages: a named location answering the same status */
        } else if (!strcmp(k->args[0], "auth_jwt") && k->nargs == 2 && !strcmp(k->args[1], "off")) {
        } else if (!orc_neutral(k->args[0], 2)) {
            L.unknown = 1;
        }
    }
    if (L.has_proxy && L.plen && L.path[L.plen - 1] == '/' && (L.kind == LK_PREFIX || L.kind == LK_EXACT ||
                                                               L.kind == LK_NOREGEX))
        L.auto_redirect = 1;
    c->loc = realloc(c->loc, sizeof(loc_t) * (c->nloc + 1)); c->loc[c->nloc++] = L;
    S->locs = realloc(S->locs, sizeof(int) * (S->nlocs + 1)); S->locs[S->nlocs++] = L.id;
}

static void add_server(build_t *B, dir_t *s, int http_waf) {
    orc_ctx *c = B->c;
    srv_t S; memset(&S, 0, sizeof S);
    S.id = c->nsrv; S.waf_mode = http_waf;
    S.rip.recursive = -1;
    for (int i = 0; i < s->nkids; i++) {
        dir_t *d = &s->kids[i];
        if (d->nargs == 2 && !strcmp(d->args[0], "wallarm_mode")) S.waf_mode = waf_mode_of(d->args[1]);
        if (d->nargs == 2 && !strcmp(d->args[0], "wallarm_parser_disable")) S.pd_mask |= dec_bit(d->args[1]);
    }
    c->srv = realloc(c->srv, sizeof(srv_t) * (c->nsrv + 1)); c->nsrv++;
    for (int i = 0; i < s->nkids; i++) {
        dir_t *d = &s->kids[i];
        if (!d->nargs) continue;
        const char *n = d->args[0];
        if (!strcmp(n, "listen") && d->nargs >= 2) {
            const char *a = d->args[1];
            if (!strncmp(a, "unix:", 5)) continue;
            const char *colon = strrchr(a, ':');
            int port = atoi(colon ? colon + 1 : a);
            int ssl = 0, def = 0, pp = 0;
            for (int k = 2; k < d->nargs; k++) {
                if (!strcmp(d->args[k], "ssl")) ssl = 1;
                if (!strcmp(d->args[k], "default_server") || !strcmp(d->args[k], "default")) def = 1;
                if (!strcmp(d->args[k], "proxy_protocol")) pp = 1;
            }
            if (S.nports < 16) {
                S.ports[S.nports] = port; S.ssl[S.nports] = ssl; S.def[S.nports] = def; S.pp[S.nports] = pp;
                S.nports++;
            }
        } else if (!strcmp(n, "server_name")) {
            for (int k = 1; k < d->nargs; k++) {
                S.names = realloc(S.names, sizeof(char *) * (S.nnames + 1));
                S.nlen = realloc(S.nlen, sizeof(int) * (S.nnames + 1));
                S.nre = realloc(S.nre, sizeof(pcre *) * (S.nnames + 1));
                char *nm = strdup(d->args[k]);
                S.nre[S.nnames] = NULL;
                if (nm[0] == '~') S.nre[S.nnames] = re_compile(nm + 1, 0);
                else for (char *q = nm; *q; q++) *q = (char)lc((unsigned char)*q);
                S.names[S.nnames] = nm; S.nlen[S.nnames] = (int)strlen(nm); S.nnames++;
            }
        } else if (!strcmp(n, "if") && d->block) {
            /* server rewrite phase: if (<var> [op value]) { return code [text]; } */
            sif_t f; memset(&f, 0, sizeof f);
            int a0 = 1, a1 = d->nargs - 1;
            char *first = d->args[a0]; char *last = d->args[a1];
            if (first[0] == '(') { if (first[1] == 0) a0++; else memmove(first, first + 1, strlen(first)); }
            int ll = (int)strlen(d->args[a1]);
            if (ll && d->args[a1][ll - 1] == ')') { if (ll == 1) a1--; else d->args[a1][ll - 1] = 0; }
            (void)last;
            f.var = strdup(d->args[a0]);
            if (a1 - a0 == 2) {
                const char *op = d->args[a0 + 1];
                f.val = strdup(d->args[a0 + 2]);
                if (!strcmp(op, "=")) f.op = 1;
                else if (!strcmp(op, "!=")) f.op = 2;
                else if (!strcmp(op, "~")) { f.op = 3; f.re = re_compile(f.val, 0); }
                else if (!strcmp(op, "~*")) { f.op = 3; f.re = re_compile(f.val, 1); }
                else if (!strcmp(op, "!~")) { f.op = 4; f.re = re_compile(f.val, 0); }
                else if (!strcmp(op, "!~*")) { f.op = 4; f.re = re_compile(f.val, 1); }
            }
            int has_ret = 0, other = 0;
            for (int k = 0; k < d->nkids; k++) {
                dir_t *r = &d->kids[k];
                if (r->nargs >= 2 && !strcmp(r->args[0], "return")) {
                    has_ret = 1;
                    if (isdigit((unsigned char)r->args[1][0])) f.code = atoi(r->args[1]); else f.code = 302;
                } else if (!(r->nargs >= 2 && !strcmp(r->args[0], "set") && !strcmp(r->args[1], "$hsts_header_val"))) {
                    other = 1;
                }
            }
            if (other) {   /* an `if` doing more than return / the HSTS header value: deferred here */
                memset(&f, 0, sizeof f); f.unsupported = 1;
                S.ifs = realloc(S.ifs, sizeof(sif_t) * (S.nifs + 1)); S.ifs[S.nifs++] = f;
                continue;
            }
            if (!has_ret) continue;   /* e.g. HSTS `if` only sets a header variable */
            S.ifs = realloc(S.ifs, sizeof(sif_t) * (S.nifs + 1)); S.ifs[S.nifs++] = f;
        } else if (!strcmp(n, "rewrite")) {
            /* server-level rewrite (server snippets): outside the restated subset, a request that
             * reaches it in the server rewrite phase is deferred (GM_ACT_UNSUPPORTED) */
            sif_t f; memset(&f, 0, sizeof f); f.unsupported = 1;
            S.ifs = realloc(S.ifs, sizeof(sif_t) * (S.nifs + 1)); S.ifs[S.nifs++] = f;
        } else if (!strcmp(n, "return") && d->nargs >= 2) {
            sif_t f; memset(&f, 0, sizeof f); f.is_return_only = 1;
            f.code = isdigit((unsigned char)d->args[1][0]) ? atoi(d->args[1]) : 302;
            S.ifs = realloc(S.ifs, sizeof(sif_t) * (S.nifs + 1)); S.ifs[S.nifs++] = f;
        } else if (!strcmp(n, "location") && d->block) {
            add_location(B, &S, d, S.waf_mode);
        } else if (!strcmp(n, "client_max_body_size") && d->nargs == 2) {
            S.cmbs = strdup(d->args[1]);
        } else if ((!strcmp(n, "allow") || !strcmp(n, "deny")) && d->nargs == 2 && oacl_add(&S.acc, n, d->args[1])) {
        } else if (orc_realip_dir(&S.rip, d)) {
        } else if ((!strcmp(n, "set") && d->nargs >= 2 && !strcmp(d->args[1], "$hsts_header_val")) ||
                   (!strcmp(n, "error_page") && d->nargs >= 3 && !strncmp(d->args[d->nargs - 1], "@grpcerror", 10)) ||
                   (!strcmp(n, "auth_jwt") && d->nargs == 2 && !strcmp(d->args[1], "off")) ||
                   !strcmp(n, "server_name") || !strcmp(n, "listen") || orc_neutral(n, 1)) {
        } else {
            /* any other directive (server snippets): deferred at its place in the server's
             * rewrite-phase order */
            sif_t f; memset(&f, 0, sizeof f); f.unsupported = 1;
            S.ifs = realloc(S.ifs, sizeof(sif_t) * (S.nifs + 1)); S.ifs[S.nifs++] = f;
        }
    }
    c->srv[S.id] = S;
}

/* ------------------------------------------------------------------ signatures + Aho-Corasick */
static int hexval(int ch) { return isdigit(ch) ? ch - '0' : (lc((unsigned char)ch) - 'a' + 10); }

static int load_sigs(orc_ctx *c, const char *t, int n) {
    int i = 0;
    while (i < n) {
        int e = i; while (e < n && t[e] != '\n') e++;
        int ls = i; while (ls < e && (t[ls] == ' ' || t[ls] == '\t' || t[ls] == '\r')) ls++;
        int le = e; while (le > ls && (t[le - 1] == '\r' || t[le - 1] == ' ' || t[le - 1] == '\t')) le--;
        i = e + 1;
        if (ls >= le || t[ls] == '#') continue;
        if (le - ls >= 9 && !strncmp(t + ls, "@decoders", 9)) {
            int p = ls + 9;
            while (p < le) {
                while (p < le && (t[p] == ' ' || t[p] == ',' || t[p] == '\t')) p++;
                int q = p; while (q < le && t[q] != ',' && t[q] != ' ' && t[q] != '\t') q++;
                if (q > p) { char nm[32] = {0}; memcpy(nm, t + p, (size_t)(q - p < 31 ? q - p : 31)); c->decoders |= dec_bit(nm); }
                p = q;
            }
            continue;
        }
        char kind[8] = {0}, fl[8] = {0}, zs[8] = {0};
        int p = ls, f = 0;
        char *dst[3] = {kind, fl, zs};
        for (f = 0; f < 3; f++) {
            int q = 0; while (p < le && t[p] != ' ') { if (q < 7) dst[f][q++] = t[p]; p++; }
            while (p < le && t[p] == ' ') p++;
        }
        sig_t s; memset(&s, 0, sizeof s);
        s.nocase = fl[0] == 'i';
        for (char *z = zs; *z; z++) s.zones |= (*z == 'u') ? 1 : (*z == 'a') ? 2 : (*z == 'h') ? 4 : (*z == 'b') ? 8 : 0;
        if (!strcmp(kind, "lit")) {
            s.kind = 0; s.len = (le - p) / 2; s.lit = malloc(s.len + 1);
            for (int k = 0; k < s.len; k++) s.lit[k] = (uint8_t)(hexval(t[p + 2 * k]) * 16 + hexval(t[p + 2 * k + 1]));
        } else {
            s.kind = 1;
            char *pat = xstrndup(t + p, le - p);
            s.re = re_compile(pat, s.nocase);
            s.pattern_src = pat;
            if (!s.re) { seterr("bad signature regex", NULL); return -1; }
            const char *er;
            s.ex = pcre_study(s.re, PCRE_STUDY_JIT_COMPILE, &er);
        }
        c->sig = realloc(c->sig, sizeof(sig_t) * (c->nsig + 1)); c->sig[c->nsig++] = s;
    }
    return 0;
}

/* A literal that every match of a PCRE pattern contains, or 0: the longest run of plain
 * characters at top level, each kept only if its quantifier has a minimum >= 1 (a '+' or {n,}
 * quantifier ends the run after its character, '*' '?' {0,} drop it); groups, classes, escapes
 * of letters and digits, '.', anchors end a run; a top-level '|', "(?" or \Q anywhere: no factor. */
static int skip_quant(const char *p, int i, int *min) {
    *min = 1;
    if (p[i] == '*' || p[i] == '?') { *min = 0; i++; }
    else if (p[i] == '+') { *min = 2; i++; }
    else if (p[i] == '{') {
        int j = i + 1, n = 0, dig = 0;
        while (p[j] >= '0' && p[j] <= '9') { n = n * 10 + (p[j] - '0'); j++; dig = 1; }
        if (!dig) return i;   /* a literal '{' */
        while (p[j] && p[j] != '}') j++;
        if (!p[j]) return i;
        *min = n == 0 ? 0 : 2;
        i = j + 1;
    } else return i;
    if (p[i] == '?' || p[i] == '+') i++;   /* lazy / possessive */
    return i;
}
/* a group body that is an alternation of plain literals (escaped punctuation allowed): its
 * alternatives, lowercased, into alts; 0 if any part is not a plain literal or is shorter than 3 */
static int literal_alts(const char *p, int n, char alts[16][64], int *alen) {
    int na = 0, cl = 0;
    char cur[64];
    for (int i = 0; i <= n; i++) {
        if (i == n || p[i] == '|') {
            if (cl < 3 || na == 16) return 0;
            memcpy(alts[na], cur, cl); alen[na++] = cl; cl = 0;
            continue;
        }
        char ch = p[i];
        if (ch == '\\') {
            if (i + 1 >= n || isalnum((unsigned char)p[i + 1])) return 0;
            ch = p[++i];
        } else if (strchr(".^$*+?{}[]()", ch)) return 0;
        if (cl == 63) return 0;
        cur[cl++] = (char)lc((unsigned char)ch);
    }
    return na;
}

static int extract_factor(const char *p, char alts[16][64], int *alen) {
    int depth = 0, cls = 0;
    for (int i = 0; p[i]; i++) {
        if (p[i] == '\\' && p[i + 1] == 'Q') return 0;
        if (p[i] == '\\' && p[i + 1]) { i++; continue; }
        if (cls) { if (p[i] == ']') cls = 0; continue; }
        if (p[i] == '[') { cls = 1; if (p[i + 1] == '^') i++; if (p[i + 1] == ']') i++; continue; }
        if (p[i] == '(') { if (p[i + 1] == '?' && p[i + 2] != ':') return 0; depth++; }
        else if (p[i] == ')') depth--;
        else if (p[i] == '|' && depth == 0) return 0;
    }
    char cur[256], best[256]; int cl = 0, bl = 0, i = 0, min;
    char galts[16][64]; int glen[16], gn = 0, gmin = 0;
#define FLUSH() do { if (cl > bl) { memcpy(best, cur, cl); bl = cl; } cl = 0; } while (0)
    while (p[i]) {
        char c = p[i], lit;
        if (c == '\\') {
            char e = p[i + 1];
            if (!e) break;
            if (isalnum((unsigned char)e)) { FLUSH(); i = skip_quant(p, i + 2, &min); continue; }
            lit = e; i += 2;
        } else if (c == '[') {
            int j = i + 1;
            if (p[j] == '^') j++;
            if (p[j] == ']') j++;
            while (p[j] && p[j] != ']') { if (p[j] == '\\' && p[j + 1]) j++; j++; }
            FLUSH(); i = skip_quant(p, p[j] ? j + 1 : j, &min); continue;
        } else if (c == '(') {
            int j = i, d = 0, k = 0;
            for (; p[j]; j++) {
                if (p[j] == '\\' && p[j + 1]) { j++; continue; }
                if (k) { if (p[j] == ']') k = 0; continue; }
                if (p[j] == '[') { k = 1; if (p[j + 1] == '^') j++; if (p[j + 1] == ']') j++; continue; }
                if (p[j] == '(') d++;
                else if (p[j] == ')' && --d == 0) break;
            }
            FLUSH();
            const int body = i + ((p[i + 1] == '?') ? 3 : 1);   /* "(?:" or "(" */
            i = skip_quant(p, p[j] ? j + 1 : j, &min);
            if (min > 0 && !gn) {   /* a required group of literal alternatives */
                char t[16][64]; int tl[16];
                const int na = p[j] ? literal_alts(p + body, j - body, t, tl) : 0;
                int mn = 64;
                for (int q = 0; q < na; q++) mn = tl[q] < mn ? tl[q] : mn;
                if (na) { memcpy(galts, t, sizeof t); memcpy(glen, tl, sizeof tl); gn = na; gmin = mn; }
            }
            continue;
        } else if (c == '.' || c == '^' || c == '$' || c == '*' || c == '+' || c == '?' || c == '{' || c == ')') {
            FLUSH(); i = skip_quant(p, i + 1, &min); continue;
        } else { lit = c; i++; }
        i = skip_quant(p, i, &min);
        if (min == 0) { FLUSH(); continue; }
        if (cl < 255) cur[cl++] = (char)lc((unsigned char)lit);
        if (min == 2) FLUSH();
    }
    FLUSH();
#undef FLUSH
    /* the longest plain run, unless a literal-alternation group has longer shortest members */
    if (bl >= 3 && (bl >= 4 || !gn || gmin <= bl)) {
        if (bl > 63) bl = 63;
        memcpy(alts[0], best, bl); alen[0] = bl;
        return 1;
    }
    if (gn) { memcpy(alts, galts, sizeof galts); memcpy(alen, glen, sizeof glen); return gn; }
    return 0;
}

static void build_ac(orc_ctx *c) {
    int total = 1;
    for (int i = 0; i < c->nsig; i++) if (c->sig[i].kind == 0) total += c->sig[i].len;
    int32_t *nx = malloc(sizeof(int32_t) * 256 * (size_t)total);
    for (size_t k = 0; k < 256 * (size_t)total; k++) nx[k] = -1;
    int32_t *out = malloc(sizeof(int32_t) * total), *fail = calloc(total, sizeof(int32_t));
    int32_t *dict = malloc(sizeof(int32_t) * total);
    for (int k = 0; k < total; k++) { out[k] = -1; dict[k] = -1; }
    int32_t *pnext = malloc(sizeof(int32_t) * (c->nsig + 1));
    int ns = 1;
    for (int i = 0; i < c->nsig; i++) {
        if (c->sig[i].kind != 0) continue;
        int s = 0;
        for (int k = 0; k < c->sig[i].len; k++) {
            int b = lc(c->sig[i].lit[k]);
            if (nx[(size_t)s * 256 + b] < 0) nx[(size_t)s * 256 + b] = ns++;
            s = nx[(size_t)s * 256 + b];
        }
        pnext[i] = out[s]; out[s] = i;
    }
    int32_t *q = malloc(sizeof(int32_t) * ns); int qh = 0, qt = 0;
    for (int b = 0; b < 256; b++) {
        int t = nx[b];
        if (t < 0) nx[b] = 0; else { fail[t] = 0; q[qt++] = t; }
    }
    while (qh < qt) {
        int s = q[qh++];
        dict[s] = (out[fail[s]] >= 0) ? fail[s] : dict[fail[s]];
        for (int b = 0; b < 256; b++) {
            int t = nx[(size_t)s * 256 + b];
            if (t < 0) nx[(size_t)s * 256 + b] = nx[(size_t)fail[s] * 256 + b];
            else { fail[t] = nx[(size_t)fail[s] * 256 + b]; q[qt++] = t; }
        }
    }
    free(q); free(fail);
    c->ac_next = nx; c->ac_states = ns; c->ac_out = out; c->ac_dict = dict; c->ac_pat_next = pnext;
}

static void build_fac_ac(orc_ctx *c) {
    int total = 1, npat = 0;
    for (int i = 0; i < c->nsig; i++) {
        sig_t *g = &c->sig[i];
        if (g->kind != 1) continue;
        g->nfac = extract_factor(g->pattern_src ? g->pattern_src : "", g->fac, g->flen);
        for (int k = 0; k < g->nfac; k++) { total += g->flen[k]; npat++; }
    }
    int32_t *nx = malloc(sizeof(int32_t) * 256 * (size_t)total);
    for (size_t k = 0; k < 256 * (size_t)total; k++) nx[k] = -1;
    int32_t *out = malloc(sizeof(int32_t) * total), *fail = calloc(total, sizeof(int32_t));
    int32_t *dict = malloc(sizeof(int32_t) * total);
    for (int k = 0; k < total; k++) { out[k] = -1; dict[k] = -1; }
    int32_t *pnext = malloc(sizeof(int32_t) * (npat + 1)), *pre = malloc(sizeof(int32_t) * (npat + 1));
    int ns = 1, pid = 0;
    for (int i = 0; i < c->nsig; i++) {
        sig_t *g = &c->sig[i];
        if (g->kind != 1) continue;
        for (int f = 0; f < g->nfac; f++, pid++) {
            int s = 0;
            for (int k = 0; k < g->flen[f]; k++) {
                int b = (unsigned char)g->fac[f][k];
                if (nx[(size_t)s * 256 + b] < 0) nx[(size_t)s * 256 + b] = ns++;
                s = nx[(size_t)s * 256 + b];
            }
            pre[pid] = i; pnext[pid] = out[s]; out[s] = pid;
        }
    }
    int32_t *q = malloc(sizeof(int32_t) * ns); int qh = 0, qt = 0;
    for (int b = 0; b < 256; b++) {
        int t = nx[b];
        if (t < 0) nx[b] = 0; else { fail[t] = 0; q[qt++] = t; }
    }
    while (qh < qt) {
        int s = q[qh++];
        dict[s] = (out[fail[s]] >= 0) ? fail[s] : dict[fail[s]];
        for (int b = 0; b < 256; b++) {
            int t = nx[(size_t)s * 256 + b];
            if (t < 0) nx[(size_t)s * 256 + b] = nx[(size_t)fail[s] * 256 + b];
            else { fail[t] = nx[(size_t)fail[s] * 256 + b]; q[qt++] = t; }
        }
    }
    free(q); free(fail);
    c->fac_next = nx; c->fac_out = out; c->fac_dict = dict; c->fac_pat_next = pnext; c->fac_pat_re = pre;
}

/* switch the CPU-baseline prefilter on (1) or off (0, the checker's exhaustive PCRE runs) */
int orc_set_prefilter(orc_ctx *c, int on) {
    if (on && !c->fac_next) build_fac_ac(c);
    c->prefilter = on;
    return 0;
}
/* the prefilter literals of a regex, '|'-joined into out (>= 16 * 65 bytes); returns their count */
int orc_factor(const char *pat, char *out) {
    char a[16][64]; int l[16];
    int n = extract_factor(pat, a, l), k = 0;
    for (int i = 0; i < n; i++) { if (i) out[k++] = '|'; memcpy(out + k, a[i], l[i]); k += l[i]; }
    out[k] = 0;
    return n;
}

/* ------------------------------------------------------------------ public: create */
/* ------------------------------------------------------------------ upstream balancers (§8 f3)
 * nginx 1.17.3's ngx_http_upstream_round_robin / least_conn / ip_hash / hash / random modules,
 * restated request by request (the engine's k_peer_* kernels batch the same algorithms).  What the
 * engine does not model defers (GM_PEER_DEFER): server parameters beyond max_fails /
 * fail_timeout / slow_start / down, Plus-only methods, hash keys with $host or variables outside
 * the engine's set, a consistent-hash upstream naming one address twice, more than 1024 peers
 * under round robin / least_conn, and a request of another method whose pick falls back to round
 * robin (empty hash key, > 20 tries on down peers) in an upstream of more than 1024 peers. */
static int is_var_ch(char ch);
static uint32_t crc32_bytes(uint32_t c, const void *p, size_t n) {   /* bitwise CRC-32/IEEE, running */
    const uint8_t *b = p;
    for (size_t i = 0; i < n; i++) {
        c ^= b[i];
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return c;
}
uint32_t orc_crc32(const void *p, size_t n) { return crc32_bytes(0xFFFFFFFFu, p, n) ^ 0xFFFFFFFFu; }

static int cmp_point(const void *a, const void *b) {
    const opoint_t *x = a, *y = b;
    if (x->hash != y->hash) return x->hash < y->hash ? -1 : 1;
    return x->peer - y->peer;
}

/* the engine's variable set for hash keys (gm_compile.cpp Compiler::src, minus $host) */
static int key_var_ok(const char *nm, int n) {
    static const char *vars[] = {"scheme", "https", "http2", "request_method", "args", "query_string", "uri",
                                 "document_uri", "request_uri", "request", "request_body", "remote_addr",
                                 "remote_port", "server_port", "request_id", NULL};
    char b[128];
    if (n <= 0 || n >= (int)sizeof b) return 0;
    for (int i = 0; i < n; i++) b[i] = (char)lc((unsigned char)nm[i]);
    b[n] = 0;
    for (int i = 0; vars[i]; i++) if (!strcmp(b, vars[i])) return 1;
    if ((!strncmp(b, "http_", 5) && n > 5) || (!strncmp(b, "cookie_", 7) && n > 7) || (!strncmp(b, "arg_", 4) && n > 4)) return 1;
    return 0;
}

static void build_upstreams(orc_ctx *c) {
    c->uby = calloc(c->nups ? c->nups : 1, sizeof(oups_t *));
    c->total_peers = 0;
    for (int u = 0; u < c->nups; u++) {
        oups_t *U = NULL;
        for (int k = 0; k < c->nudef && !U; k++) if (!strcmp(c->udef[k].name, c->ups[u])) U = &c->udef[k];
        c->uby[u] = U;
        if (!U) continue;
        dir_t *d = U->d;
        U->method = OM_RR;
        int defer = 0;
        for (int i = 0; i < d->nkids; i++) {
            dir_t *k = &d->kids[i];
            if (!k->nargs) continue;
            const char *m = k->args[0];
            if (!strcmp(m, "server") && k->nargs >= 2) {
                U->addr = realloc(U->addr, sizeof(char *) * (U->npeers + 1));
                U->down = realloc(U->down, sizeof(int) * (U->npeers + 1));
                U->addr[U->npeers] = strdup(k->args[1]); U->down[U->npeers] = 0;
                for (int q = 2; q < k->nargs; q++) {
                    const char *a = k->args[q];
                    if (!strcmp(a, "down")) U->down[U->npeers] = 1;
                    else if (!strncmp(a, "max_fails=", 10) || !strncmp(a, "fail_timeout=", 13) ||
                             !strncmp(a, "slow_start=", 11) || !strcmp(a, "weight=1") || !strcmp(a, "max_conns=0")) {}
                    else defer = 1;
                }
                U->npeers++;
            } else if (!strcmp(m, "least_conn") && k->nargs == 1) U->method = OM_LEAST_CONN;
            else if (!strcmp(m, "ip_hash") && k->nargs == 1) U->method = OM_IP_HASH;
            else if (!strcmp(m, "hash") && (k->nargs == 2 || (k->nargs == 3 && !strcmp(k->args[2], "consistent")))) {
                U->method = k->nargs == 3 ? OM_CHASH : OM_HASH;
                U->key = strdup(k->args[1]);
            } else if (!strcmp(m, "random")) {
                if (k->nargs == 1) U->method = OM_RANDOM;
                else if (!strcmp(k->args[1], "two") && (k->nargs == 2 || (k->nargs == 3 && !strcmp(k->args[2], "least_conn"))))
                    U->method = OM_RANDOM2;
                else defer = 1;
            } else if (!strcmp(m, "sticky") && k->nargs >= 3 && !strcmp(k->args[1], "cookie")) {
                /* expires= / domain= / path= / httponly / secure: the response's Set-Cookie only */
                char b[300];
                snprintf(b, sizeof b, "$cookie_%s", k->args[2]);
                free(U->sticky);
                U->sticky = strdup(b);
            } else if (!strcmp(m, "least_time") || !strcmp(m, "sticky") || !strcmp(m, "queue") ||
                       !strcmp(m, "ntlm") || !strcmp(m, "hash")) defer = 1;
        }
        U->first_peer = c->total_peers;
        c->total_peers += U->npeers;
        if ((U->method == OM_RR || U->method == OM_LEAST_CONN) && U->npeers > 1024) defer = 1;
        if (U->method == OM_HASH || U->method == OM_CHASH) {
            for (const char *p = U->key; *p && !defer; p++) {
                if (*p != '$') continue;
                const char *st; int n;
                p++;
                if (*p == '{') { st = ++p; while (*p && *p != '}') p++; if (!*p) { defer = 1; break; } n = (int)(p - st); }
                else { st = p; while (is_var_ch(*p)) p++; n = (int)(p - st); p--; }
                if (!key_var_ok(st, n)) defer = 1;
            }
            if (U->method == OM_CHASH)
                for (int a = 0; a < U->npeers; a++)
                    for (int b = 0; b < a; b++) if (!strcmp(U->addr[a], U->addr[b])) defer = 1;
        }
        if (U->method == OM_CHASH && !defer) {
            /* ngx_http_upstream_update_chash: 160 points per server */
            U->ring = malloc(sizeof(opoint_t) * 160 * (U->npeers ? U->npeers : 1));
            int np = 0;
            for (int j = 0; j < U->npeers; j++) {
                const char *sv = U->addr[j]; int sl = (int)strlen(sv);
                const char *host = sv, *port = ""; int hl = sl, pl = 0;
                if (sl >= 5 && !strncasecmp(sv, "unix:", 5)) { host = sv + 5; hl = sl - 5; }
                else {
                    for (int q = sl - 1; q >= 0; q--) {
                        if (sv[q] == ':') { hl = q; port = sv + q + 1; pl = sl - q - 1; break; }
                        if (sv[q] < '0' || sv[q] > '9') break;
                    }
                }
                uint32_t base = crc32_bytes(0xFFFFFFFFu, host, hl);
                base = crc32_bytes(base, "", 1);
                base = crc32_bytes(base, port, pl);
                uint32_t prev = 0;
                for (int q = 0; q < 160; q++) {
                    uint8_t pb[4] = {(uint8_t)prev, (uint8_t)(prev >> 8), (uint8_t)(prev >> 16), (uint8_t)(prev >> 24)};
                    uint32_t h = crc32_bytes(base, pb, 4) ^ 0xFFFFFFFFu;
                    U->ring[np].hash = h; U->ring[np].peer = j; np++;
                    prev = h;
                }
            }
            qsort(U->ring, np, sizeof(opoint_t), cmp_point);
            int m = 0;
            for (int q = 0; q < np; q++) if (q == 0 || U->ring[q].hash != U->ring[m - 1].hash) U->ring[m++] = U->ring[q];
            U->nring = m;
        }
        if (defer) U->method = OM_DEFER;
    }
}

orc_ctx *orc_create(const void *blob, size_t len, uint32_t gen) {
    const uint8_t *b = blob;
    if (len < 8) { seterr("short blob", NULL); return NULL; }
    uint32_t magic, n; memcpy(&magic, b, 4); memcpy(&n, b + 4, 4);
    if (magic != GM_BLOB_MAGIC) { seterr("bad magic", NULL); return NULL; }
    size_t off = 8;
    dir_t *mainroot = NULL; build_t B; memset(&B, 0, sizeof B);
    orc_ctx *c = calloc(1, sizeof *c); c->gen = gen; B.c = c;
    const char *sigt = NULL; int sign = 0;
    for (uint32_t e = 0; e < n; e++) {
        uint32_t kind, nl, dl;
        memcpy(&kind, b + off, 4); memcpy(&nl, b + off + 4, 4); memcpy(&dl, b + off + 8, 4); off += 12;
        const char *data = (const char *)b + off + nl; off += nl + dl;
        if (kind == GM_ENTRY_SIGS) { sigt = data; sign = (int)dl; continue; }
        if (kind == GM_ENTRY_SAMPLE) continue;   /* traffic sample: tunes the GPU prefilter only */
        dir_t *root = calloc(1, sizeof(dir_t));
        lexer L = {data, (int)dl, 0, malloc(dl + 1)};
        if (parse_block(&L, root, 0) < 0) { seterr("config parse error", NULL); return NULL; }
        if (kind == GM_ENTRY_MAIN) mainroot = root;
        else { B.confd = realloc(B.confd, sizeof(dir_t *) * (B.nconfd + 1)); B.confd[B.nconfd++] = root; }
    }
    if (mainroot) {
        for (int i = 0; i < mainroot->nkids; i++)
            if (mainroot->kids[i].nargs && !strcmp(mainroot->kids[i].args[0], "http") && mainroot->kids[i].block)
                walk_http(&B, &mainroot->kids[i]);
    } else {
        for (int k = 0; k < B.nconfd; k++) walk_http(&B, B.confd[k]);
    }
    /* upstream id = index in the sorted, de-duplicated upstream-name table */
    qsort(c->ups, c->nups, sizeof(char *), cmp_str);
    int u = 0;
    for (int i = 0; i < c->nups; i++) if (u == 0 || strcmp(c->ups[u - 1], c->ups[i])) c->ups[u++] = c->ups[i];
    c->nups = u;
    build_upstreams(c);
    for (int i = 0; i < c->nloc; i++) {
        loc_t *L = &c->loc[i];
        if (!L->has_proxy) continue;
        char *key = L->proxy_ups;
        char **hit = bsearch(&key, c->ups, c->nups, sizeof(char *), cmp_str);
        L->upstream_id = hit ? (int)(hit - c->ups) : -1;
    }
    /* limits and realip in effect per server / location (nginx's merge of http -> server ->
     * location settings) */
    for (int si = 0; si < c->nsrv; si++) {
        srv_t *S = &c->srv[si];
        const char *sv_size = S->cmbs ? S->cmbs : c->http_cmbs ? c->http_cmbs : "1m";
        int64_t x = orc_size(sv_size);
        S->body_max = x == -2 ? -1 : x;
        if (x == -2) {   /* not a size: the whole server defers */
            S->ifs = realloc(S->ifs, sizeof(sif_t) * (S->nifs + 1));
            memmove(S->ifs + 1, S->ifs, sizeof(sif_t) * S->nifs);
            memset(&S->ifs[0], 0, sizeof(sif_t)); S->ifs[0].unsupported = 1; S->nifs++;
        }
        for (int k = 0; k < S->nlocs; k++) {
            loc_t *L = &c->loc[S->locs[k]];
            int64_t y = orc_size(L->cmbs ? L->cmbs : sv_size);
            if (y == -2) { L->unknown = 1; y = -1; }
            L->body_max = (L->nested || L->pcre_only) ? -1 : y;
        }
        if (c->http_unknown) {
            S->ifs = realloc(S->ifs, sizeof(sif_t) * (S->nifs + 1));
            memset(&S->ifs[S->nifs], 0, sizeof(sif_t)); S->ifs[S->nifs].unsupported = 1; S->nifs++;
        }
        const orip_t *a = &S->rip, *h = &c->http_rip;
        const orip_t *fr = a->nfrom ? a : h;
        if (fr->nfrom) {
            const char *hd = a->header ? a->header : h->header ? h->header : "X-Real-IP";
            S->rrec = a->recursive >= 0 ? a->recursive : h->recursive >= 0 ? h->recursive : 0;
            if (!strcmp(hd, "X-Real-IP")) S->rtype = 1;
            else if (!strcmp(hd, "X-Forwarded-For")) S->rtype = 2;
            else if (!strcmp(hd, "proxy_protocol")) S->rtype = 3;
            else {
                S->rtype = 4;
                snprintf(S->hdr, sizeof S->hdr, "%s", hd);
                for (char *q = S->hdr; *q; q++) *q = (char)lc((unsigned char)*q);
            }
            S->cidr = calloc((size_t)fr->nfrom, sizeof(ocidr_t));
            for (int k = 0; k < fr->nfrom; k++) {
                if (!strncmp(fr->from[k], "unix:", 5)) continue;
                if (!o_ptocidr(fr->from[k], &S->cidr[S->ncidr])) { S->rtype = 5; continue; }
                S->ncidr++;
            }
        }
    }
    if (sigt && load_sigs(c, sigt, sign) < 0) return NULL;
    build_ac(c);
    return c;
}

void orc_destroy(orc_ctx *c) { (void)c; /* test process lifetime; intentionally leaked */ }

int orc_info(orc_ctx *c, uint32_t *out4) {
    out4[0] = c->nsrv; out4[1] = c->nloc; out4[2] = c->nups; out4[3] = c->nsig; return 0;
}

/* ------------------------------------------------------------------ request access */
typedef struct {
    const gm_req *r; const uint8_t *a;
    sv uri, args, hdrs, body, host, method, ruri, raddr, paddr;
    const srv_t *S;        /* the server (its realip settings), NULL before it is known */
    int rip;               /* 0 not evaluated, 1 unchanged, 2 replaced, 3 unknown to the engine */
    char ra[64]; int ra_len; oaddr_t raddr2;
} rq_t;

static void rq_init(rq_t *q, const gm_req *r, const uint8_t *arena) {
    q->r = r; q->a = arena;
    const char *p = (const char *)arena + r->base;
    q->uri = (sv){p, (int)r->uri_len}; p += r->uri_len;
    q->args = (sv){p, (int)r->args_len}; p += r->args_len;
    q->hdrs = (sv){p, (int)r->hdr_len}; p += r->hdr_len;
    q->body = (sv){p, (int)r->body_len}; p += r->body_len;
    q->host = (sv){p, r->host_len}; p += r->host_len;
    q->method = (sv){p, r->method_len}; p += r->method_len;
    q->ruri = (sv){p, r->ruri_len}; p += r->ruri_len;
    q->raddr = (sv){p, r->raddr_len}; p += r->raddr_len;
    q->paddr = (sv){p, r->pad0[0]};   /* $proxy_protocol_addr */
    q->S = NULL; q->rip = 0;
}

static int hdr_next(sv h, int *pos, sv *name, sv *val);

/* ngx_http_realip_handler for the request's server (post-read phase): q->rip */
static void orc_realip(rq_t *q) {
    const srv_t *S = q->S;
    q->rip = 1;
    if (!S || !S->rtype) return;
    if (S->rtype == 5) { q->rip = 3; return; }
    oaddr_t a;
    memset(&a, 0, sizeof a);
    if (!(q->raddr.n > 0 && q->raddr.n < 46 && o_parse_addr(q->raddr.p, q->raddr.n, &a))) a.fam = 0;
    int rc = 0;
    if (S->rtype == 3) {
        /* NGX_HTTP_REALIP_PROXY: the connection's PROXY address (none: declined) through
         * ngx_http_get_forwarded_addr, then the PROXY source port */
        if (!a.fam || q->paddr.n == 0) return;
        rc = o_fwd_internal(S, &a, q->paddr.p, q->paddr.n);
        if (rc == 0) return;
        a.port = q->r->pad1[0] | q->r->pad1[1] << 8;
        q->raddr2 = a;
        q->ra_len = o_ntop(&a, q->ra);
        q->rip = 2;
        return;
    }
    if (!a.fam) return;
    int pos = 0; sv hn, vv;
    if (S->rtype == 2) {
        /* every X-Forwarded-For line, last first (ngx_http_get_forwarded_addr over the array) */
        sv vals[256]; int nv = 0;
        while (hdr_next(q->hdrs, &pos, &hn, &vv))
            if (hn.n == 15 && !strncasecmp(hn.p, "x-forwarded-for", 15) && nv < 256) vals[nv++] = vv;
        int found = 0;
        for (int i = nv - 1; i >= 0; i--) {
            rc = o_fwd_internal(S, &a, vals[i].p, vals[i].n);
            if (!S->rrec) break;
            if (rc == 0 && found) { rc = 2; break; }
            if (rc != 1) break;
            found = 1;
        }
    } else {
        const char *want = S->rtype == 1 ? "x-real-ip" : S->hdr;
        int wl = (int)strlen(want);
        while (hdr_next(q->hdrs, &pos, &hn, &vv))
            if (hn.n == wl && !strncasecmp(hn.p, want, (size_t)wl)) { rc = o_fwd_internal(S, &a, vv.p, vv.n); break; }
    }
    if (rc == 0) return;
    q->raddr2 = a;
    q->ra_len = o_ntop(&a, q->ra);
    q->rip = 2;
}

/* scratch string arena, per thread: chunked so earlier views stay valid until reset */
typedef struct chunk { struct chunk *next; int cap, used; char data[]; } chunk_t;
typedef struct { chunk_t *head; } scratch_t;
static sv sc_put(scratch_t *s, const char *p, int n) {
    if (!s->head || s->head->used + n > s->head->cap) {
        int cap = n > (1 << 16) ? n : (1 << 16);
        chunk_t *c = malloc(sizeof(chunk_t) + cap); c->cap = cap; c->used = 0; c->next = s->head; s->head = c;
    }
    char *d = s->head->data + s->head->used;
    memcpy(d, p, n); s->head->used += n;
    return (sv){d, n};
}
static void sc_reset(scratch_t *s) {
    while (s->head && s->head->next) { chunk_t *n = s->head->next; free(s->head); s->head = n; }
    if (s->head) s->head->used = 0;
}

/* iterate header lines "Name: value\r\n"; the value without leading / trailing spaces (nginx
 * ngx_http_parse_header_line sw_space_before_value / sw_space_after_value skip ' ' only: a tab
 * is part of the value) */
static int hdr_next(sv h, int *pos, sv *name, sv *val) {
    while (*pos < h.n) {
        int st = *pos, e = st;
        while (e < h.n && h.p[e] != '\n') e++;
        *pos = e + 1;
        int le = e; if (le > st && h.p[le - 1] == '\r') le--;
        int c = st; while (c < le && h.p[c] != ':') c++;
        if (c >= le) continue;
        *name = (sv){h.p + st, c - st};
        int vs = c + 1; while (vs < le && h.p[vs] == ' ') vs++;
        int ve = le; while (ve > vs && h.p[ve - 1] == ' ') ve--;
        *val = (sv){h.p + vs, ve - vs};
        return 1;
    }
    return 0;
}

/* ngx_http_variable_unknown_header: lowercase, '-' -> '_' compare against var suffix */
static int hdr_name_match(sv name, const char *var, int vlen) {
    if (name.n != vlen) return 0;
    for (int i = 0; i < vlen; i++) {
        unsigned char ch = (unsigned char)name.p[i];
        if (ch >= 'A' && ch <= 'Z') ch |= 0x20; else if (ch == '-') ch = '_';
        if ((unsigned char)var[i] != ch) return 0;
    }
    return 1;
}

static uint32_t murmur2(const uint8_t *data, size_t len) {
    uint32_t h = 0 ^ (uint32_t)len, k;
    while (len >= 4) {
        k = data[0]; k |= data[1] << 8; k |= data[2] << 16; k |= (uint32_t)data[3] << 24;
        k *= 0x5bd1e995; k ^= k >> 24; k *= 0x5bd1e995;
        h *= 0x5bd1e995; h ^= k;
        data += 4; len -= 4;
    }
    switch (len) {
    case 3: h ^= data[2] << 16; /* fallthrough */
    case 2: h ^= data[1] << 8;  /* fallthrough */
    case 1: h ^= data[0]; h *= 0x5bd1e995;
    }
    h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
    return h;
}
uint32_t orc_murmur2(const uint8_t *d, size_t n) { return murmur2(d, n); }

typedef struct { orc_ctx *c; rq_t *q; scratch_t *sc; int depth; int *last_param; int *last_part; int unknown; } ev_t;

static sv eval_complex(ev_t *E, const char *tpl);

static sv get_var(ev_t *E, const char *name, int nlen) {
    rq_t *q = E->q; const gm_req *r = q->r; orc_ctx *c = E->c;
    char nm[256]; if (nlen > 255) nlen = 255; memcpy(nm, name, nlen); nm[nlen] = 0;
    for (int i = 0; i < nlen; i++) nm[i] = (char)lc((unsigned char)nm[i]);
    if (!strcmp(nm, "scheme")) return (r->flags & GM_REQ_HTTPS) ? (sv){"https", 5} : (sv){"http", 4};
    if (!strcmp(nm, "https")) return (r->flags & GM_REQ_HTTPS) ? (sv){"on", 2} : (sv){"", 0};
    if (!strcmp(nm, "http2")) return (r->flags & GM_REQ_HTTP2) ? (sv){"h2", 2} : (sv){"", 0};
    if (!strcmp(nm, "request_method")) return q->method;
    if (!strcmp(nm, "args") || !strcmp(nm, "query_string")) return q->args;
    if (!strcmp(nm, "uri") || !strcmp(nm, "document_uri")) return q->uri;
    if (!strcmp(nm, "request_body")) return (sv){"", 0};
    if (!strcmp(nm, "remote_addr") || !strcmp(nm, "remote_port")) {
        if (!q->rip) orc_realip(q);
        if (q->rip == 3) { E->unknown = 1; return (sv){"", 0}; }
        if (nm[7] == 'a') return q->rip == 2 ? (sv){q->ra, q->ra_len} : q->raddr;
        unsigned port = q->rip == 2 ? (unsigned)q->raddr2.port : r->remote_port;
        if (q->rip == 2 && port == 0) return (sv){"", 0};   /* no port in the header's address */
        char t[8]; int n = snprintf(t, 8, "%u", port); return sc_put(E->sc, t, n);
    }
    if (!strcmp(nm, "server_port")) { char t[8]; int n = snprintf(t, 8, "%u", r->port); return sc_put(E->sc, t, n); }
    if (!strcmp(nm, "request_uri")) {
        if (q->ruri.n) return q->ruri;
        char *t = malloc(q->uri.n + q->args.n + 2); int n = 0;
        memcpy(t, q->uri.p, q->uri.n); n = q->uri.n;
        if (q->args.n) { t[n++] = '?'; memcpy(t + n, q->args.p, q->args.n); n += q->args.n; }
        sv s = sc_put(E->sc, t, n); free(t); return s;
    }
    if (!strcmp(nm, "request")) {
        sv ru = get_var(E, "request_uri", 11);
        const char *proto = (r->flags & GM_REQ_HTTP2) ? "HTTP/2.0" : (r->flags & GM_REQ_HTTP10) ? "HTTP/1.0" : "HTTP/1.1";
        int pl = (int)strlen(proto);
        char *t = malloc(q->method.n + ru.n + pl + 3); int n = 0;
        memcpy(t + n, q->method.p, q->method.n); n += q->method.n; t[n++] = ' ';
        memcpy(t + n, ru.p, ru.n); n += ru.n; t[n++] = ' ';
        memcpy(t + n, proto, pl); n += pl;
        sv s = sc_put(E->sc, t, n); free(t); return s;
    }
    if (!strcmp(nm, "request_id")) {
        char t[32]; static const char hx[] = "0123456789abcdef";
        for (int i = 0; i < 16; i++) { t[2 * i] = hx[r->rid[i] >> 4]; t[2 * i + 1] = hx[r->rid[i] & 15]; }
        return sc_put(E->sc, t, 32);
    }
    if (!strncmp(nm, "http_", 5)) {
        const char *hv = nm + 5; int hl = nlen - 5;
        int joined = !strcmp(hv, "cookie") ? ';' : !strcmp(hv, "x_forwarded_for") ? ',' : 0;
        int pos = 0; sv hn, vv; sv acc = {"", 0}; int have = 0; char *tmp = NULL; int tn = 0;
        while (hdr_next(q->hdrs, &pos, &hn, &vv)) {
            if (!hdr_name_match(hn, hv, hl)) continue;
            if (!joined) return vv;
            tmp = realloc(tmp, tn + vv.n + 2);
            if (have) { tmp[tn++] = (char)joined; tmp[tn++] = ' '; }
            memcpy(tmp + tn, vv.p, vv.n); tn += vv.n; have = 1;
        }
        if (have) { acc = sc_put(E->sc, tmp, tn); }
        free(tmp);
        return acc;
    }
    if (!strncmp(nm, "cookie_", 7)) {
        /* ngx_http_parse_multi_header_lines over all Cookie lines */
        const char *cn = nm + 7; int cl = nlen - 7;
        int pos = 0; sv hn, vv;
        while (hdr_next(q->hdrs, &pos, &hn, &vv)) {
            if (!hdr_name_match(hn, "cookie", 6)) continue;
            if (cl > vv.n) continue;
            const char *start = vv.p, *end = vv.p + vv.n;
            while (start < end) {
                if (end - start < cl || strncasecmp(start, cn, cl) != 0) goto skip;
                for (start += cl; start < end && *start == ' '; start++) {}
                if (start == end || *start++ != '=') goto skip;
                while (start < end && *start == ' ') start++;
                const char *last = start;
                while (last < end && *last != ';') last++;
                return (sv){start, (int)(last - start)};
            skip:
                while (start < end) { char ch = *start++; if (ch == ';' || ch == ',') break; }
                while (start < end && *start == ' ') start++;
            }
        }
        return (sv){"", 0};
    }
    if (!strncmp(nm, "arg_", 4)) {
        /* ngx_http_arg */
        const char *an = nm + 4; int alen = nlen - 4;
        const char *a = q->args.p; int n = q->args.n;
        for (int p = 0; p + alen < n; p++) {
            if (strncasecmp(a + p, an, alen) != 0) continue;
            if ((p == 0 || a[p - 1] == '&') && a[p + alen] == '=') {
                int vs = p + alen + 1, ve = vs;
                while (ve < n && a[ve] != '&') ve++;
                return (sv){a + vs, ve - vs};
            }
        }
        return (sv){"", 0};
    }
    if (!strcmp(nm, "host")) {
        return q->host;   /* not verdict-relevant here (redirect Location text) */
    }
    /* map / split_clients variables */
    if (E->depth > 32) return (sv){"", 0};
    for (int i = 0; i < c->nmap; i++) {
        map_t *m = &c->map[i];
        if (strcmp(m->var, nm)) continue;
        E->depth++;
        sv src = eval_complex(E, m->src);
        const char *res = NULL; int pidx = -1;
        /* ngx_http_map_find: lowercased exact key, then regexes only for non-empty value */
        for (int k = 0; k < m->np && !res; k++) {
            if (m->p[k].is_re) continue;
            if (m->p[k].klen != src.n) continue;
            int ok = 1;
            for (int t = 0; t < src.n; t++) if (lc((unsigned char)src.p[t]) != (unsigned char)m->p[k].key[t]) { ok = 0; break; }
            if (ok) { res = m->p[k].val; pidx = k; }
        }
        if (!res && src.n) {
            for (int k = 0; k < m->np && !res; k++) {
                if (!m->p[k].is_re || !m->p[k].re) continue;
                int ov[30];
                if (pcre_exec(m->p[k].re, NULL, src.p, src.n, 0, 0, ov, 30) >= 0) { res = m->p[k].val; pidx = k; }
            }
        }
        if (!res) { res = m->defval ? m->defval : ""; pidx = -1; }
        if (E->last_param) *E->last_param = pidx;
        sv out = eval_complex(E, res);
        E->depth--;
        return out;
    }
    for (int i = 0; i < c->nspl; i++) {
        split_t *s = &c->spl[i];
        if (strcmp(s->var, nm)) continue;
        E->depth++;
        sv src = eval_complex(E, s->src);
        uint32_t h = murmur2((const uint8_t *)src.p, src.n);
        sv out = {"", 0}; int part = -1;
        for (int k = 0; k < s->np; k++) {
            if (h < s->p[k].bound || s->p[k].star) { part = k; out = eval_complex(E, s->p[k].val); break; }
        }
        if (E->last_part) *E->last_part = part;
        E->depth--;
        return out;
    }
    return (sv){"", 0};
}

static int is_var_ch(char ch) { return isalnum((unsigned char)ch) || ch == '_'; }

static sv eval_complex(ev_t *E, const char *tpl) {
    if (!strchr(tpl, '$')) return (sv){tpl, (int)strlen(tpl)};
    char *out = NULL; int on = 0;
    for (const char *p = tpl; *p;) {
        if (*p == '$') {
            p++;
            const char *st; int n;
            if (*p == '{') { st = ++p; while (*p && *p != '}') p++; n = (int)(p - st); if (*p) p++; }
            else { st = p; while (is_var_ch(*p)) p++; n = (int)(p - st); }
            sv v = get_var(E, st, n);
            out = realloc(out, on + v.n + 1); memcpy(out + on, v.p, v.n); on += v.n;
        } else {
            out = realloc(out, on + 2); out[on++] = *p++;
        }
    }
    sv r = sc_put(E->sc, out ? out : "", on); free(out); return r;
}

/* ------------------------------------------------------------------ host (ngx_http_validate_host) */
static int validate_host(sv h, char *out, int *outlen) {
    int dot_pos = h.n, host_len = h.n, state = 0; /* 0 usual, 1 literal, 2 rest */
    for (int i = 0; i < h.n; i++) {
        unsigned char ch = (unsigned char)h.p[i];
        switch (ch) {
        case '.':
            if (dot_pos == i - 1) return -1;
            dot_pos = i; break;
        case ':':
            if (state == 0) { host_len = i; state = 2; }
            break;
        case '[':
            if (i == 0) state = 1;
            break;
        case ']':
            if (state == 1) { host_len = i + 1; state = 2; }
            break;
        case '\0':
            return -1;
        default:
            if (ch == '/') return -1;
            break;
        }
    }
    if (dot_pos == host_len - 1) host_len--;
    if (host_len == 0) return -1;
    for (int i = 0; i < host_len; i++) out[i] = (char)lc((unsigned char)h.p[i]);
    *outlen = host_len;
    return 0;
}

static int find_server(orc_ctx *c, int port, int is_https, sv host, int *bad, int *port_ssl) {
    /* servers listening on port, config order */
    int def = -1, first = -1; int ssl = 0;
    for (int s = 0; s < c->nsrv; s++)
        for (int k = 0; k < c->srv[s].nports; k++)
            if (c->srv[s].ports[k] == port) {
                if (first < 0) first = s;
                if (c->srv[s].def[k] && def < 0) def = s;
                if (c->srv[s].ssl[k]) ssl = 1;
            }
    *port_ssl = ssl; (void)is_https;
    if (first < 0) return -1;
    if (def < 0) def = first;
    *bad = 0;
    if (host.n == 0) return def;
    char hn[65536]; int hl;
    if (validate_host(host, hn, &hl) < 0) { *bad = 1; return def; }
    int best = -1, bestlen = -1;
    /* exact */
    for (int s = 0; s < c->nsrv && best < 0; s++) {
        int on = 0; for (int k = 0; k < c->srv[s].nports; k++) if (c->srv[s].ports[k] == port) on = 1;
        if (!on) continue;
        for (int k = 0; k < c->srv[s].nnames; k++) {
            const char *nm = c->srv[s].names[k]; int nl = c->srv[s].nlen[k];
            if (nm[0] == '*' || nm[0] == '~' || nm[0] == '.' || (nl && nm[nl - 1] == '*')) continue;
            if (nl == hl && !memcmp(nm, hn, hl)) { best = s; break; }
        }
    }
    if (best >= 0) return best;
    /* wildcard head: "*.x" / ".x" -- longest suffix wins, earlier server on ties */
    for (int s = 0; s < c->nsrv; s++) {
        int on = 0; for (int k = 0; k < c->srv[s].nports; k++) if (c->srv[s].ports[k] == port) on = 1;
        if (!on) continue;
        for (int k = 0; k < c->srv[s].nnames; k++) {
            const char *nm = c->srv[s].names[k]; int nl = c->srv[s].nlen[k];
            const char *suf = NULL; int sl = 0, dotform = 0;
            if (nl > 2 && nm[0] == '*' && nm[1] == '.') { suf = nm + 1; sl = nl - 1; }
            else if (nl > 1 && nm[0] == '.') { suf = nm; sl = nl; dotform = 1; }
            if (!suf) continue;
            int m = 0;
            if (hl > sl && !memcmp(hn + hl - sl, suf, sl)) m = 1;
            if (dotform && hl == sl - 1 && !memcmp(hn, suf + 1, sl - 1)) m = 1;
            if (m && sl > bestlen) { best = s; bestlen = sl; }
        }
    }
    if (best >= 0) return best;
    /* wildcard tail "x.*" */
    for (int s = 0; s < c->nsrv; s++) {
        int on = 0; for (int k = 0; k < c->srv[s].nports; k++) if (c->srv[s].ports[k] == port) on = 1;
        if (!on) continue;
        for (int k = 0; k < c->srv[s].nnames; k++) {
            const char *nm = c->srv[s].names[k]; int nl = c->srv[s].nlen[k];
            if (nl < 3 || nm[nl - 1] != '*' || nm[nl - 2] != '.') continue;
            int pl = nl - 1;   /* "x." */
            if (hl > pl && !memcmp(hn, nm, pl) && pl > bestlen) { best = s; bestlen = pl; }
        }
    }
    if (best >= 0) return best;
    /* regex names in order */
    for (int s = 0; s < c->nsrv; s++) {
        int on = 0; for (int k = 0; k < c->srv[s].nports; k++) if (c->srv[s].ports[k] == port) on = 1;
        if (!on) continue;
        for (int k = 0; k < c->srv[s].nnames; k++) {
            if (!c->srv[s].nre[k]) continue;
            int ov[30];
            if (pcre_exec(c->srv[s].nre[k], NULL, hn, hl, 0, 0, ov, 30) >= 0) return s;
        }
    }
    return def;
}

/* ngx_http_core_find_location restated over the server's top-level locations */
static int find_location(orc_ctx *c, srv_t *S, sv uri, int *auto301) {
    *auto301 = 0;
    for (int i = 0; i < S->nlocs; i++) {
        loc_t *L = &c->loc[S->locs[i]];
        if (L->kind == LK_EXACT && L->plen == uri.n && !memcmp(L->path, uri.p, uri.n)) return L->id;
    }
    int best = -1, bestlen = -1, prefix_equal = 0;
    for (int i = 0; i < S->nlocs; i++) {
        loc_t *L = &c->loc[S->locs[i]];
        if (L->kind != LK_PREFIX && L->kind != LK_NOREGEX) continue;
        if (L->plen <= uri.n && !memcmp(L->path, uri.p, L->plen) && L->plen > bestlen) {
            best = L->id; bestlen = L->plen; prefix_equal = (L->plen == uri.n);
        }
    }
    /* auto_redirect: a location named uri + "/" and nothing (prefix or exact) named uri itself */
    if (!prefix_equal) {
        for (int i = 0; i < S->nlocs; i++) {
            loc_t *L = &c->loc[S->locs[i]];
            if (L->kind == LK_REGEX || L->kind == LK_REGEX_I || L->kind == LK_NAMED) continue;
            if (L->auto_redirect && L->plen == uri.n + 1 && !memcmp(L->path, uri.p, uri.n)) {
                *auto301 = 1; return L->id;
            }
        }
    }
    if (best >= 0 && c->loc[best].kind == LK_NOREGEX) return best;
    for (int i = 0; i < S->nlocs; i++) {
        loc_t *L = &c->loc[S->locs[i]];
        if ((L->kind != LK_REGEX && L->kind != LK_REGEX_I) || !L->re) continue;
        int ov[30];
        if (L->pcre_only) {   /* reached and its superset matches: deferred (GM_ACT_UNSUPPORTED) */
            if (!L->relaxed || pcre_exec(L->relaxed, NULL, uri.p, uri.n, 0, 0, ov, 30) >= 0) return L->id;
            continue;
        }
        if (pcre_exec(L->re, NULL, uri.p, uri.n, 0, 0, ov, 30) >= 0) return L->id;
    }
    return best;
}

static int find_named(orc_ctx *c, srv_t *S, sv name) {
    for (int i = 0; i < S->nlocs; i++) {
        loc_t *L = &c->loc[S->locs[i]];
        if (L->kind == LK_NAMED && L->plen == name.n && !memcmp(L->path, name.p, name.n)) return L->id;
    }
    return -1;
}

/* ------------------------------------------------------------------ per request */
typedef struct { uint32_t *ids; size_t n, cap; } hitbuf_t;

static void hb_push(hitbuf_t *h, uint32_t v) {
    if (h->n == h->cap) { h->cap = h->cap ? h->cap * 2 : 1024; h->ids = realloc(h->ids, h->cap * 4); }
    h->ids[h->n++] = v;
}

/* literal (Aho-Corasick) and regex signatures over four zones; skip_empty: regexes only on
 * non-empty zones (the decoded views' pass) */
static void waf_zones(orc_ctx *c, const sv *zones, uint8_t *mark, hitbuf_t *out, int skip_empty) {
    for (int z = 0; z < 4; z++) {
        sv Z = zones[z];
        int s = 0;
        for (int i = 0; i < Z.n; i++) {
            s = c->ac_next[(size_t)s * 256 + lc((unsigned char)Z.p[i])];
            int t = (c->ac_out[s] >= 0) ? s : c->ac_dict[s];
            while (t > 0) {
                for (int p = c->ac_out[t]; p >= 0; p = c->ac_pat_next[p]) {
                    sig_t *g = &c->sig[p];
                    if (mark[p] || !(g->zones & (1 << z))) continue;
                    int st = i - g->len + 1;
                    if (!g->nocase && memcmp(Z.p + st, g->lit, g->len)) continue;
                    mark[p] = 1; hb_push(out, (uint32_t)p);
                }
                t = c->ac_dict[t];
            }
        }
    }
    uint8_t *cand = c->prefilter ? mark + c->nsig + 1 : NULL;
    if (cand) {
        for (int z = 0; z < 4; z++) {
            sv Z = zones[z];
            int s = 0;
            for (int i = 0; i < Z.n; i++) {
                s = c->fac_next[(size_t)s * 256 + lc((unsigned char)Z.p[i])];
                for (int t = (c->fac_out[s] >= 0) ? s : c->fac_dict[s]; t > 0; t = c->fac_dict[t])
                    for (int p = c->fac_out[t]; p >= 0; p = c->fac_pat_next[p]) cand[c->fac_pat_re[p]] |= (uint8_t)(1 << z);
            }
        }
    }
    for (int p = 0; p < c->nsig; p++) {
        sig_t *g = &c->sig[p];
        if (g->kind != 1 || !g->re || mark[p]) { if (cand) cand[p] = 0; continue; }
        const int cz = cand ? cand[p] : 0;
        if (cand) cand[p] = 0;
        for (int z = 0; z < 4; z++) {
            if (!(g->zones & (1 << z))) continue;
            if (skip_empty && zones[z].n == 0) continue;
            if (cand && g->nfac && !(cz & (1 << z))) continue;   /* none of its factors is in the zone */
            int ov[30];
            if (pcre_exec(g->re, g->ex, zones[z].p ? zones[z].p : "", zones[z].n, 0, 0, ov, 30) >= 0) {
                mark[p] = 1; hb_push(out, (uint32_t)p); break;
            }
        }
    }
}

/* ------------------------------------------------------------------ request parsers (§8 f4)
 * The decoded views gm_decode.inc builds, restated: $args -> [percent / urlenc transform if it
 * changes a byte, '\n'] [each base64 run (>= 16 of [A-Za-z0-9+/]) decoded, '\n']; body -> the
 * form transform of an application/x-www-form-urlencoded body or the JSON unescape of a "json"
 * body (if it changes a byte, then '\n'), then the body's base64 runs. */
typedef struct { uint8_t *p; size_t n, cap; } dbuf_t;
static void db_put(dbuf_t *b, uint8_t ch) {
    if (b->n == b->cap) { b->cap = b->cap ? 2 * b->cap : 256; b->p = realloc(b->p, b->cap); }
    b->p[b->n++] = ch;
}
static int hexd(int c) { return c >= '0' && c <= '9' ? c - '0' : (c | 0x20) >= 'a' && (c | 0x20) <= 'f' ? (c | 0x20) - 'a' + 10 : -1; }
static int b64d(int c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    return c == '+' ? 62 : c == '/' ? 63 : -1;
}
static void dv_form(sv s, int mask, dbuf_t *o) {
    size_t st = o->n; int chg = 0;
    for (int i = 0; i < s.n; i++) {
        unsigned char ch = (unsigned char)s.p[i];
        if ((mask & GM_DEC_PERCENT) && ch == '%' && i + 2 < s.n && hexd((unsigned char)s.p[i + 1]) >= 0 &&
            hexd((unsigned char)s.p[i + 2]) >= 0) {
            ch = (unsigned char)(hexd((unsigned char)s.p[i + 1]) * 16 + hexd((unsigned char)s.p[i + 2])); i += 2; chg = 1;
        } else if ((mask & GM_DEC_URLENC) && ch == '+') { ch = ' '; chg = 1; }
        db_put(o, ch);
    }
    if (chg) db_put(o, '\n'); else o->n = st;
}
static void utf8(dbuf_t *o, unsigned cp) {
    if (cp < 0x80) db_put(o, (uint8_t)cp);
    else if (cp < 0x800) { db_put(o, (uint8_t)(0xC0 | cp >> 6)); db_put(o, (uint8_t)(0x80 | (cp & 63))); }
    else if (cp < 0x10000) { db_put(o, (uint8_t)(0xE0 | cp >> 12)); db_put(o, (uint8_t)(0x80 | (cp >> 6 & 63))); db_put(o, (uint8_t)(0x80 | (cp & 63))); }
    else { db_put(o, (uint8_t)(0xF0 | cp >> 18)); db_put(o, (uint8_t)(0x80 | (cp >> 12 & 63))); db_put(o, (uint8_t)(0x80 | (cp >> 6 & 63))); db_put(o, (uint8_t)(0x80 | (cp & 63))); }
}
static int u4(sv s, int i) {
    if (i + 4 > s.n) return -1;
    int v = 0;
    for (int k = 0; k < 4; k++) { int h = hexd((unsigned char)s.p[i + k]); if (h < 0) return -1; v = v * 16 + h; }
    return v;
}
static void dv_json(sv s, dbuf_t *o) {
    size_t st = o->n; int chg = 0;
    for (int i = 0; i < s.n; i++) {
        unsigned char ch = (unsigned char)s.p[i];
        if (ch != '\\' || i + 1 >= s.n) { db_put(o, ch); continue; }
        char e = s.p[i + 1];
        const char *from = "\"\\/bfnrt", *to = "\"\\/\b\f\n\r\t";
        const char *f = strchr(from, e);
        if (e && f) { db_put(o, (uint8_t)to[f - from]); i++; chg = 1; continue; }
        if (e == 'u') {
            int cp = u4(s, i + 2);
            if (cp >= 0) {
                int adv = 5;
                if (cp >= 0xD800 && cp <= 0xDBFF) {
                    int lo = (i + 7 < s.n && s.p[i + 6] == '\\' && s.p[i + 7] == 'u') ? u4(s, i + 8) : -1;
                    if (lo >= 0xDC00 && lo <= 0xDFFF) { cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); adv = 11; }
                    else cp = 0xFFFD;
                } else if (cp >= 0xDC00 && cp <= 0xDFFF) cp = 0xFFFD;
                utf8(o, (unsigned)cp); i += adv; chg = 1;
                continue;
            }
        }
        db_put(o, ch);
    }
    if (chg) db_put(o, '\n'); else o->n = st;
}
static void dv_b64(sv s, dbuf_t *o) {
    int i = 0;
    while (i < s.n) {
        if (b64d((unsigned char)s.p[i]) < 0) { i++; continue; }
        int j = i; while (j < s.n && b64d((unsigned char)s.p[j]) >= 0) j++;
        int L = j - i;
        if (L >= 16) {
            for (int q = i; q + 4 <= i + (L & ~3); q += 4) {
                unsigned v = (unsigned)b64d((unsigned char)s.p[q]) << 18 | (unsigned)b64d((unsigned char)s.p[q + 1]) << 12 |
                             (unsigned)b64d((unsigned char)s.p[q + 2]) << 6 | (unsigned)b64d((unsigned char)s.p[q + 3]);
                db_put(o, (uint8_t)(v >> 16)); db_put(o, (uint8_t)(v >> 8)); db_put(o, (uint8_t)v);
            }
            db_put(o, '\n');
        }
        i = j;
    }
}
/* 1 form, 2 json, 0 other: the first Content-Type line */
static int orc_body_kind(rq_t *q) {
    int pos = 0; sv hn, vv;
    while (hdr_next(q->hdrs, &pos, &hn, &vv)) {
        if (!hdr_name_match(hn, "content_type", 12)) continue;
        if (vv.n >= 33 && !strncasecmp(vv.p, "application/x-www-form-urlencoded", 33)) return 1;
        for (int k = 0; k + 4 <= vv.n; k++) if (!strncasecmp(vv.p + k, "json", 4)) return 2;
        return 0;
    }
    return 0;
}
static void decoded_views(rq_t *q, int mask, dbuf_t *a, dbuf_t *b) {
    if (mask & (GM_DEC_PERCENT | GM_DEC_URLENC)) dv_form(q->args, mask, a);
    if (mask & GM_DEC_BASE64) dv_b64(q->args, a);
    int kind = (mask & (GM_DEC_PERCENT | GM_DEC_URLENC | GM_DEC_JSON)) ? orc_body_kind(q) : 0;
    if (kind == 1 && (mask & (GM_DEC_PERCENT | GM_DEC_URLENC))) dv_form(q->body, mask, b);
    else if (kind == 2 && (mask & GM_DEC_JSON)) dv_json(q->body, b);
    if (mask & GM_DEC_BASE64) dv_b64(q->body, b);
}

static void waf_scan(orc_ctx *c, rq_t *q, uint8_t *mark, hitbuf_t *out, int dec_mask) {
    sv zones[4] = {q->uri, q->args, q->hdrs, q->body};
    size_t first = out->n;
    waf_zones(c, zones, mark, out, 0);
    if (dec_mask) {
        dbuf_t a = {0}, b = {0};
        decoded_views(q, dec_mask, &a, &b);
        if (a.n || b.n) {
            sv dz[4] = {{"", 0}, {(const char *)a.p, (int)a.n}, {"", 0}, {(const char *)b.p, (int)b.n}};
            waf_zones(c, dz, mark, out, 1);
        }
        free(a.p); free(b.p);
    }
    /* sort this request's ids ascending, clear marks */
    for (size_t i = first + 1; i < out->n; i++) {
        uint32_t v = out->ids[i]; size_t j = i;
        while (j > first && out->ids[j - 1] > v) { out->ids[j] = out->ids[j - 1]; j--; }
        out->ids[j] = v;
    }
    for (size_t i = first; i < out->n; i++) mark[out->ids[i]] = 0;
}

/* the allow / deny rules in effect at a location: its own, else its server's, else the http
 * block's (ngx_http_access_merge_loc_conf) */
static const oacl_t *loc_acl(const orc_ctx *c, const srv_t *S, const loc_t *L) {
    return L->acc.n ? &L->acc : S->acc.n ? &S->acc : &c->http_acc;
}
/* the engine's contract (gm_compile.cpp): a content location with rules beside wallarm_mode (the
 * two access-phase handlers' order is not fixed by the reference) is deferred */
static int loc_access_defer(const orc_ctx *c, const srv_t *S, const loc_t *L) {
    return loc_acl(c, S, L)->n && !L->has_return && L->waf_mode != GM_WAF_OFF;
}
/* the access phase for the address the connection has after realip: 0 allowed, 1 denied (403),
 * 2 unknown to the engine (realip from a source it cannot read, an unparseable address) */
static int access_phase(ev_t *E, const oacl_t *A) {
    if (!A->n) return 0;
    sv ra = get_var(E, "remote_addr", 11);
    oaddr_t a;
    if (E->unknown || !o_parse_addr(ra.p, ra.n, &a)) return 2;
    return oacl_denies(A, &a);
}
static void eval_one(orc_ctx *c, const gm_req *r, const uint8_t *arena, gm_verdict *v, scratch_t *sc,
                     uint8_t *mark, hitbuf_t *hits, uint32_t *nh) {
    rq_t q; rq_init(&q, r, arena);
    memset(v, 0, sizeof *v);
    v->gen = c->gen; v->location_id = GM_NONE; v->upstream_id = GM_NONE; v->split_bucket = 0xFF; v->match_idx = 0xFF;
    v->route_kind = GM_ROUTE_NONE; v->waf_mode = GM_WAF_OFF; *nh = 0;
    sc_reset(sc);
    int bad = 0, port_ssl = 0;
    int sidx = find_server(c, r->port, r->flags & GM_REQ_HTTPS, q.host, &bad, &port_ssl);
    if (sidx < 0 || ((r->flags & GM_REQ_HTTPS) && !port_ssl)) {
        v->server_id = GM_NONE; v->action = GM_ACT_NO_LISTENER; v->status = 0; return;
    }
    v->server_id = (uint32_t)sidx;
    if (r->flags & GM_REQ_INVALID) {   /* rejected by the wire parser: its status, from the default server */
        v->action = GM_ACT_BAD_REQUEST; v->status = (uint32_t)r->pad0[1] | (uint32_t)r->pad0[2] << 8; return;
    }
    if (bad || (port_ssl && !(r->flags & GM_REQ_HTTPS))) { v->action = GM_ACT_BAD_REQUEST; v->status = 400; return; }
    srv_t *S = &c->srv[sidx];
    q.S = S;
    ev_t E = {c, &q, sc, 0, NULL, NULL};
    for (int i = 0; i < S->nifs; i++) {
        sif_t *f = &S->ifs[i];
        int hit = 0;
        if (f->unsupported) { v->action = GM_ACT_UNSUPPORTED; v->status = 0; return; }
        if (f->is_return_only) hit = 1;
        else {
            const char *vn = f->var; sv val = {"", 0};
            if (vn[0] == '$') val = get_var(&E, vn + 1, (int)strlen(vn + 1));
            if (E.unknown) { v->action = GM_ACT_UNSUPPORTED; v->status = 0; return; }
            if (f->op == 0) hit = val.n && !(val.n == 1 && val.p[0] == '0');
            else if (f->op == 1) hit = sv_eq(val, f->val);
            else if (f->op == 2) hit = !sv_eq(val, f->val);
            else if (f->re) { int ov[30]; int m = pcre_exec(f->re, NULL, val.p ? val.p : "", val.n, 0, 0, ov, 30) >= 0; hit = (f->op == 3) ? m : !m; }
        }
        if (hit) {
            v->action = (f->code >= 301 && f->code <= 308 && f->code != 304 && f->code != 305 && f->code != 306) ? GM_ACT_REDIRECT : GM_ACT_RETURN;
            v->status = (uint32_t)f->code; return;
        }
    }
    /* client_max_body_size: a Content-Length body against the location found, before its rewrite
     * phase (ngx_http_core_find_config_phase); a chunked one when the proxying location reads it */
    const int chunked = (r->flags & GM_REQ_CHUNKED) != 0;
#define TOO_LARGE(lim) (!chunked && (lim) >= 0 && (int64_t)r->body_len > (lim))
    int a301 = 0;
    int lid = find_location(c, S, q.uri, &a301);
    if (lid < 0) {
        if (TOO_LARGE(S->body_max)) { v->action = GM_ACT_TOO_LARGE; v->status = 413; return; }
        /* no location: the server block's own configuration runs the access phase */
        const int ap = access_phase(&E, S->acc.n ? &S->acc : &c->http_acc);
        if (ap == 1) { v->action = GM_ACT_FORBIDDEN; v->status = 403; return; }
        if (ap == 2) { v->action = GM_ACT_UNSUPPORTED; v->status = 0; return; }
        v->action = GM_ACT_NOT_FOUND; v->status = 404; return;
    }
    v->location_id = (uint32_t)lid;
    loc_t *L = &c->loc[lid];
    if (TOO_LARGE(L->body_max)) { v->action = GM_ACT_TOO_LARGE; v->status = 413; return; }
#undef TOO_LARGE
    if (a301) { v->action = GM_ACT_AUTO_301; v->status = 301; return; }
    if (L->pcre_only || L->nested || L->unknown || loc_access_defer(c, S, L)) { v->action = GM_ACT_UNSUPPORTED; v->status = 0; return; }
    loc_t *F = L;   /* location that runs the content phase */
    if (L->has_return && L->ret_code == 418 && L->err418) {
        int pidx = -2, part = -2;
        E.last_param = &pidx; E.last_part = &part;
        sv target = eval_complex(&E, L->err418);
        E.last_param = NULL; E.last_part = NULL;
        if (E.unknown) {   /* a condition / split source the engine cannot know: deferred */
            v->route_kind = part != -2 ? GM_ROUTE_SPLIT : GM_ROUTE_RULES;
            v->action = GM_ACT_UNSUPPORTED; v->status = 0; return;
        }
        if (part != -2) { v->route_kind = GM_ROUTE_SPLIT; v->split_bucket = part < 0 ? 0xFF : (uint8_t)part; }
        else if (pidx != -2) { v->route_kind = GM_ROUTE_RULES; v->match_idx = pidx < 0 ? 0xFF : (uint8_t)pidx; }
        if (target.n && target.p[0] == '@') {
            int nl = find_named(c, S, target);
            if (nl < 0) { v->action = GM_ACT_NOT_FOUND; v->status = 404; return; }
            F = &c->loc[nl];
            if (F->nested || loc_access_defer(c, S, F)) { v->action = GM_ACT_UNSUPPORTED; v->status = 0; return; }
        } else if (target.n == 0) {
            v->action = GM_ACT_ERRPAGE; v->status = 302; return;
        } else {
            v->action = GM_ACT_UNSUPPORTED; v->status = 0; return;
        }
    } else if (L->has_return) {
        v->action = (L->ret_code == 301 || L->ret_code == 302 || L->ret_code == 303 || L->ret_code == 307 ||
                     L->ret_code == 308) ? GM_ACT_REDIRECT : GM_ACT_RETURN;
        v->status = (uint32_t)L->ret_code; return;
    } else if (L->has_proxy) {
        v->route_kind = GM_ROUTE_PLAIN;
    }
    if (F->has_return && F != L) {
        v->action = (F->ret_code == 301 || F->ret_code == 302 || F->ret_code == 303 || F->ret_code == 307 ||
                     F->ret_code == 308) ? GM_ACT_REDIRECT : GM_ACT_RETURN;
        v->status = (uint32_t)F->ret_code; return;
    }
    {   /* the access phase (after `return`, which answers in the rewrite phase) */
        const int ap = access_phase(&E, loc_acl(c, S, F));
        if (ap == 1) { v->action = GM_ACT_FORBIDDEN; v->status = 403; return; }
        if (ap == 2) { v->action = GM_ACT_UNSUPPORTED; v->status = 0; return; }
    }
    if (F->stub && !F->has_proxy) { v->action = GM_ACT_RETURN; v->status = 200; return; }
    if (!F->has_proxy) { v->action = GM_ACT_NOT_FOUND; v->status = 404; return; }
    if (chunked && F->body_max >= 0 && (int64_t)r->body_len > F->body_max) {
        v->action = GM_ACT_TOO_LARGE; v->status = 413; return;
    }
    v->action = GM_ACT_PROXY; v->status = 0;
    v->upstream_id = F->upstream_id < 0 ? GM_NONE : (uint32_t)F->upstream_id;
    v->waf_mode = (uint16_t)F->waf_mode;
    if (F->waf_mode != GM_WAF_OFF && c->nsig) {
        size_t before = hits->n;
        /* the request parsers of the URI-selected location (its own wallarm_parser_disable list,
         * else its server's) */
        int dmask = c->decoders & ~(L->has_pd ? L->pd_mask : S->pd_mask);
        waf_scan(c, &q, mark, hits, dmask);
        *nh = (uint32_t)(hits->n - before);
        v->n_hits = (uint16_t)*nh;
        if (*nh && F->waf_mode == GM_WAF_BLOCK) { v->action = GM_ACT_BLOCK; v->status = 403; }
    }
}

typedef struct {
    orc_ctx *c; const gm_req *reqs; const uint8_t *arena; gm_verdict *out;
    size_t lo, hi; hitbuf_t hits;
} job_t;

static void *worker(void *arg) {
    job_t *j = arg;
    scratch_t sc = {NULL};
    uint8_t *mark = calloc(2 * (size_t)(j->c->nsig + 1), 1);   /* marks + prefilter candidate bits */
    for (size_t i = j->lo; i < j->hi; i++) {
        uint32_t nh;
        eval_one(j->c, &j->reqs[i], j->arena, &j->out[i], &sc, mark, &j->hits, &nh);
    }
    sc_reset(&sc); free(sc.head); free(mark);
    return NULL;
}

/* Evaluate n requests.  Hit ids are laid out exactly as libgpumatch lays them out: request
 * order, ascending rule id, first_hit_off = running count.  Returns total hits, or -1 if
 * hit_cap is too small (hit_ids then untouched beyond hit_cap). */
int64_t orc_match(orc_ctx *c, const gm_req *reqs, const uint8_t *arena, uint32_t n, gm_verdict *out,
                  uint32_t *hit_ids, size_t hit_cap, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
    job_t *jobs = calloc(nthreads, sizeof(job_t));
    pthread_t *th = calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t].c = c; jobs[t].reqs = reqs; jobs[t].arena = arena; jobs[t].out = out;
        jobs[t].lo = (size_t)n * t / nthreads; jobs[t].hi = (size_t)n * (t + 1) / nthreads;
        if (nthreads > 1) pthread_create(&th[t], NULL, worker, &jobs[t]); else worker(&jobs[t]);
    }
    if (nthreads > 1) for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    size_t off = 0; int64_t rc = 0;
    for (int t = 0; t < nthreads; t++) {
        size_t k = 0;
        for (size_t i = jobs[t].lo; i < jobs[t].hi; i++) {
            out[i].first_hit_off = out[i].n_hits ? (uint32_t)off : 0;
            for (uint32_t h = 0; h < out[i].n_hits; h++, k++, off++) {
                if (off < hit_cap) hit_ids[off] = jobs[t].hits.ids[k];
                else rc = -1;
            }
        }
        free(jobs[t].hits.ids);
    }
    free(jobs); free(th);
    return rc < 0 ? -1 : (int64_t)off;
}

/* Regex probe used by tests to pin PCRE semantics: returns 1 match / 0 no match / -1 error */
int orc_pcre_match(const char *pat, int caseless, const char *subj, int n) {
    pcre *r = re_compile(pat, caseless);
    if (!r) return -1;
    int ov[30];
    int m = pcre_exec(r, NULL, subj, n, 0, 0, ov, 30);
    return m >= 0 ? 1 : 0;
}

/* ------------------------------------------------------------------------------------------
 * $uri normalisation oracle.  Restates nginx 1.17.3
 * src/http/ngx_http_parse.c ngx_http_parse_complex_uri() with merge_slashes on (the nginx
 * source is not in /root/reference; the reference renders `location {{Path}}`,
 * nginx.ingress.tmpl:96, and nginx matches those paths against this normalised $uri).
 * Parity unpinned: no reference test fixes these bytes; the hand vectors in tests/test_uri.py
 * restate nginx's documented behaviour.  Returns the normalised length, or -1 (nginx 400).
 * Test infrastructure only. */
enum { ON_USUAL, ON_SLASH, ON_DOT, ON_DOTDOT, ON_Q1, ON_Q2 };

static int on_hex(int c, int *v) {
    if (c >= '0' && c <= '9') { *v = c - '0'; return 1; }
    c |= 0x20;
    if (c >= 'a' && c <= 'f') { *v = c - 'a' + 10; return 2; }
    return 0;
}

/* "..": u points just past "/.."; back up over it and the previous segment (nginx u -= 4 loop) */
static int on_up(const uint8_t *o, int64_t *u) {
    int64_t k = *u - 4;
    for (;;) {
        if (k < 0) return 0;
        if (o[k] == '/') { *u = k + 1; return 1; }
        k--;
    }
}

int64_t orc_normalize_uri(const uint8_t *p, uint32_t n, uint8_t *o) {
    int state = ON_USUAL, quoted_state = ON_USUAL, hi = 0, v, kind;
    int64_t u = 0;
    uint32_t i = 0;
    int ch;
    while (i < n) {
        ch = p[i++];
    dispatch:
        switch (state) {
        case ON_Q1:
            if (!on_hex(ch, &v)) return -1;
            hi = v; state = ON_Q2;
            continue;
        case ON_Q2:
            kind = on_hex(ch, &v);
            if (!kind) return -1;
            ch = hi * 16 + v;
            if (kind == 1 && (ch == '%' || ch == '#')) { o[u++] = (uint8_t)ch; state = ON_USUAL; continue; }
            if (kind == 1 && ch == 0) return -1;
            if (kind == 2 && ch == '?') { o[u++] = (uint8_t)ch; state = ON_USUAL; continue; }
            state = quoted_state;
            goto dispatch;
        default:
            break;
        }
        if (ch == 0) return -1;
        if (ch == '?' || ch == '#') goto done;
        if (ch == '%') { quoted_state = state; state = ON_Q1; continue; }
        if (state == ON_USUAL) {
            o[u++] = (uint8_t)ch;
            if (ch == '/') state = ON_SLASH;
        } else if (state == ON_SLASH) {
            if (ch == '/') continue;                 /* merge_slashes */
            o[u++] = (uint8_t)ch;
            state = ch == '.' ? ON_DOT : ON_USUAL;
        } else if (state == ON_DOT) {
            if (ch == '/') { u--; state = ON_SLASH; continue; }
            o[u++] = (uint8_t)ch;
            state = ch == '.' ? ON_DOTDOT : ON_USUAL;
        } else {                                      /* ON_DOTDOT */
            if (ch == '/') { if (!on_up(o, &u)) return -1; state = ON_SLASH; continue; }
            o[u++] = (uint8_t)ch;
            state = ON_USUAL;
        }
    }
done:
    if (state == ON_Q1 || state == ON_Q2) return -1;
    if (state == ON_DOT) u--;
    else if (state == ON_DOTDOT && !on_up(o, &u)) return -1;
    return u;
}

/* batch form of orc_normalize_uri (CPU baseline of gm_normalize_uris, one thread); out_len[i] =
 * 0xFFFFFFFF for a 400.  Test / baseline infrastructure only. */
void orc_normalize_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t n,
                         uint8_t *out, uint32_t *out_len) {
    for (uint32_t i = 0; i < n; i++) {
        int64_t r = orc_normalize_uri(arena + off[i], len[i], out + off[i]);
        out_len[i] = r < 0 ? 0xFFFFFFFFu : (uint32_t)r;
    }
}

/* ------------------------------------------------------------------------------------------
 * HTTP/1.x wire-parser oracle.  TEST INFRASTRUCTURE ONLY.
 * Restates nginx 1.17.3's request intake (source not in /root/reference; the reference's
 * templates read its results: $request_method / $uri / $args / $request_uri / $host and the
 * header lines behind $http_* / $cookie_*, nginx.virtualserver.tmpl:25-31, and the body the
 * Wallarm phase scans, nginx.ingress.tmpl:12-29):
 *   - ngx_http_parse_request_line: leading CR/LF skipped; method [A-Z_-]+; 1+ spaces; target
 *     origin-form "/..." or absolute-form "scheme://host[:port][/...]"; 1+ spaces; "HTTP/"
 *     major "." minor; spaces; CRLF or LF.  No version (HTTP/0.9) -> 400 here (nginx serves a
 *     0.9 GET: a documented divergence); major > 1 -> 505; NUL in the line -> 400.
 *   - $uri = ngx_http_parse_complex_uri of the path (orc_normalize_uri, failure -> 400);
 *     $args = after the first '?' that precedes any '#'; $request_uri = the target from its
 *     path (absolute-form: the scheme and host are not part of it; no path -> "/").
 *   - ngx_http_parse_header_line + ngx_http_process_request_headers (ignore_invalid_headers on,
 *     underscores_in_headers off): a line whose name has a byte outside [A-Za-z0-9-] (incl. '_',
 *     a leading space -- obs-fold continuation lines -- or an empty name) is dropped; a NUL
 *     anywhere -> 400; the value loses leading / trailing spaces only; a line without ':' is a
 *     header with an empty value.  Kept lines are emitted "Name: value\r\n" in order.
 *   - Host: a second Host line -> 400; HTTP/1.1 without Host (and no absolute-form host) -> 400;
 *     the absolute-form host takes precedence.  Content-Length: a second one -> 400, not all
 *     digits -> 400.  Transfer-Encoding (the first): "chunked" (caseless) -> chunked body,
 *     Content-Length ignored; "identity" -> ignored; anything else -> 501.
 *   - body: Content-Length bytes (fewer present -> 400) or the chunked body decoded
 *     (hex size [;ext] CRLF data CRLF ... "0" CRLF trailers CRLF; malformed or short -> 400).
 *   - more than 255 header lines -> 400 (the device's line table; nginx's limit is its buffers).
 * A rejected request keeps its connection fields and gets GM_REQ_INVALID + its status.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    int status;                        /* 0 ok, else 400 / 501 / 505 */
    int minor;
    const uint8_t *method; int method_len;
    const uint8_t *target; int target_len;   /* $request_uri */
    const uint8_t *path; int path_len;       /* bytes normalised into $uri (stops at ? / #) */
    const uint8_t *args; int args_len;
    const uint8_t *uhost; int uhost_len;     /* absolute-form host */
    int body_start;                          /* offset of the first body byte */
    int chunked;                             /* Transfer-Encoding: chunked */
} orc_rl_t;

static int orc_rl_parse(const uint8_t *b, int n, orc_rl_t *r) {
    memset(r, 0, sizeof *r);
    int i = 0;
    while (i < n && (b[i] == '\r' || b[i] == '\n')) i++;
    int m0 = i;
    while (i < n && ((b[i] >= 'A' && b[i] <= 'Z') || b[i] == '_' || b[i] == '-')) i++;
    if (i == m0 || i >= n || b[i] != ' ') return 400;
    r->method = b + m0; r->method_len = i - m0;
    while (i < n && b[i] == ' ') i++;
    if (i >= n) return 400;
    int t0 = i;
    if (b[i] != '/') {                       /* absolute-form: scheme "://" host [":" port] */
        int s0 = i;
        while (i < n && ((b[i] | 0x20) >= 'a' && (b[i] | 0x20) <= 'z')) i++;
        if (i == s0 || i + 3 > n || b[i] != ':' || b[i + 1] != '/' || b[i + 2] != '/') return 400;
        i += 3;
        int h0 = i;
        if (i < n && b[i] == '[') {          /* sw_host_ip_literal: "[" ... "]", the brackets kept */
            for (i++; i < n && b[i] != ']'; i++) {
                const uint8_t ch = b[i], c = ch | 0x20;
                if ((ch >= '0' && ch <= '9') || (c >= 'a' && c <= 'z')) continue;
                if (ch && strchr(":-._~!$&'()*+,;=", ch)) continue;   /* unreserved, sub-delims */
                return 400;
            }
            if (i >= n) return 400;
            i++;
        } else {
            while (i < n && (isalnum(b[i]) || b[i] == '.' || b[i] == '-')) i++;
            if (i == h0) return 400;
        }
        r->uhost = b + h0; r->uhost_len = i - h0;
        if (i < n && b[i] == ':') { i++; while (i < n && b[i] >= '0' && b[i] <= '9') i++; }
        if (i >= n) return 400;
        if (b[i] != '/' && b[i] != ' ') return 400;
        t0 = i;
    }
    int te = t0;
    while (te < n && b[te] != ' ' && b[te] != '\r' && b[te] != '\n') { if (b[te] == 0) return 400; te++; }
    if (te >= n || b[te] != ' ') return 400;   /* HTTP/0.9 (no version) or truncated */
    if (te == t0) { static const uint8_t slash = '/'; r->target = &slash; r->target_len = 1; r->path = &slash; r->path_len = 1; }
    else {
        r->target = b + t0; r->target_len = te - t0;
        int q = t0; while (q < te && b[q] != '?' && b[q] != '#') q++;
        r->path = b + t0; r->path_len = q - t0;
        if (q < te && b[q] == '?') { r->args = b + q + 1; r->args_len = te - q - 1; }
    }
    i = te;
    while (i < n && b[i] == ' ') i++;
    if (i + 5 > n || memcmp(b + i, "HTTP/", 5)) return 400;
    i += 5;
    long major = 0, minor = 0; int d0 = i;
    while (i < n && b[i] >= '0' && b[i] <= '9') { major = major * 10 + (b[i] - '0'); if (major > 99) return 400; i++; }
    if (i == d0 || i >= n || b[i] != '.') return 400;
    i++; d0 = i;
    while (i < n && b[i] >= '0' && b[i] <= '9') { minor = minor * 10 + (b[i] - '0'); if (minor > 99) return 400; i++; }
    if (i == d0) return 400;
    while (i < n && b[i] == ' ') i++;
    if (i < n && b[i] == '\r') i++;
    if (i >= n || b[i] != '\n') return 400;
    if (major > 1) return 505;
    if (major < 1) return 400;
    r->minor = (int)minor;
    r->body_start = i + 1;   /* the first header line (the caller continues from here) */
    return 0;
}

static int orc_hname_ok(const uint8_t *p, int n) {
    if (n == 0) return 0;
    for (int k = 0; k < n; k++) if (!(isalnum(p[k]) || p[k] == '-')) return 0;
    return 1;
}
static int orc_ieq(const uint8_t *p, int n, const char *s) {
    int l = (int)strlen(s);
    if (n != l) return 0;
    for (int k = 0; k < n; k++) if (lc(p[k]) != (unsigned char)s[k]) return 0;
    return 1;
}

typedef struct { uint8_t *p; size_t n, cap; } obuf_t;
static void ob_put(obuf_t *o, const void *s, size_t n) {
    if (o->n + n > o->cap) { o->cap = (o->n + n) * 2 + 64; o->p = realloc(o->p, o->cap); }
    memcpy(o->p + o->n, s, n); o->n += n;
}

/* one request -> status and its fields (appended to the per-request buffers).  nginx's order:
 * the request line (400 / 505 / 414), its complex URI (400), header lines as they are read
 * (NUL, a second Host or Content-Length, an over-long line: 400), then after the header:
 * HTTP/1.1 without a Host header (400), an invalid Content-Length (400), an unknown
 * Transfer-Encoding (501), and the body (400 if short or malformed). */
static int orc_parse_one(const uint8_t *b, int n, orc_rl_t *R, obuf_t *uri, obuf_t *hdrs, obuf_t *body,
                         const uint8_t **host, int *host_len) {
    {   /* the request line (through its LF) must fit one 8 KiB large_client_header_buffers buffer */
        int s0 = 0; while (s0 < n && (b[s0] == '\r' || b[s0] == '\n')) s0++;
        int e = s0; while (e < n && b[e] != '\n') e++;
        if (e < n && e + 1 - s0 > 8192) return 414;
    }
    int st = orc_rl_parse(b, n, R);
    if (st) return st;
    int64_t u = uri->n;
    if (uri->n + R->path_len + 1 > uri->cap) { uri->cap = uri->n + R->path_len + 64; uri->p = realloc(uri->p, uri->cap); }
    int64_t nl = orc_normalize_uri(R->path, (uint32_t)R->path_len, uri->p + u);
    if (nl < 0) return 400;
    uri->n += (size_t)nl;
    int i = R->body_start, nlines = 0, hosts = 0, cls = 0, cl_bad = 0, te_kind = 0;
    int64_t clen = -1;
    *host = NULL; *host_len = 0;
    for (;;) {
        if (i >= n) return 400;                 /* no empty line: incomplete header */
        int e = i; while (e < n && b[e] != '\n') e++;
        if (e >= n) return 400;
        int le = e; if (le > i && b[le - 1] == '\r') le--;
        if (le == i) { i = e + 1; break; }      /* empty line: end of the header */
        if (e + 1 - i > 8192) return 400;       /* header line larger than a buffer */
        for (int k = i; k < le; k++) if (b[k] == 0) return 400;
        if (++nlines > 254) return 400;
        int c = i; while (c < le && b[c] != ':') c++;
        const uint8_t *nm = b + i; int nlen = c - i;
        int vs = c < le ? c + 1 : le;
        while (vs < le && b[vs] == ' ') vs++;
        int ve = le; while (ve > vs && b[ve - 1] == ' ') ve--;
        i = e + 1;
        if (!orc_hname_ok(nm, nlen)) continue;  /* invalid header line: ignored */
        ob_put(hdrs, nm, nlen); ob_put(hdrs, ": ", 2); ob_put(hdrs, b + vs, ve - vs); ob_put(hdrs, "\r\n", 2);
        if (orc_ieq(nm, nlen, "host")) {
            if (++hosts > 1) return 400;        /* "client sent duplicate host header" */
            if (!R->uhost) { *host = b + vs; *host_len = ve - vs; }
        } else if (orc_ieq(nm, nlen, "content-length")) {
            if (++cls > 1) return 400;          /* unique header line */
            clen = 0;
            if (ve == vs) cl_bad = 1;
            for (int k = vs; k < ve && !cl_bad; k++) {
                if (b[k] < '0' || b[k] > '9' || clen > (INT64_MAX - 9) / 10) cl_bad = 1;
                else clen = clen * 10 + (b[k] - '0');
            }
        } else if (orc_ieq(nm, nlen, "transfer-encoding") && !te_kind) {
            te_kind = orc_ieq(b + vs, ve - vs, "chunked") ? 1 : orc_ieq(b + vs, ve - vs, "identity") ? 2 : 3;
        }
    }
    if (!hosts && R->minor >= 1) return 400;    /* HTTP/1.1 without a Host header */
    if (R->uhost) { *host = R->uhost; *host_len = R->uhost_len; }   /* the absolute URI's host wins */
    if (cl_bad) return 400;
    if (te_kind == 3) return 501;
    R->chunked = te_kind == 1;
    if (te_kind == 1) {
        for (;;) {
            /* chunk-size line: hex digits, then CRLF / LF, or an extension (';', SP, HT ...) up
             * to LF (ngx_http_parse_chunked sw_chunk_size / sw_chunk_extension) */
            int64_t sz = 0; int d0 = i;
            while (i < n && isxdigit(b[i])) {
                int v = isdigit(b[i]) ? b[i] - '0' : (lc(b[i]) - 'a' + 10);
                if (sz > (INT64_MAX >> 4) - 1) return 400;
                sz = sz * 16 + v; i++;
            }
            if (i == d0 || i >= n) return 400;
            if (b[i] == '\r') { i++; if (i >= n || b[i] != '\n') return 400; }
            else if (b[i] == ';' || b[i] == ' ' || b[i] == '\t') { while (i < n && b[i] != '\n') i++; if (i >= n) return 400; }
            else if (b[i] != '\n') return 400;
            i++;
            if (sz == 0) {                        /* trailer lines up to the empty line */
                for (;;) {
                    if (i >= n) return 400;
                    int e = i; while (e < n && b[e] != '\n') e++;
                    if (e >= n) return 400;
                    int le = e; if (le > i && b[le - 1] == '\r') le--;
                    const int empty = le == i;
                    i = e + 1;
                    if (empty) break;
                }
                break;
            }
            if ((int64_t)(n - i) < sz) return 400;
            ob_put(body, b + i, (size_t)sz);
            i += (int)sz;
            if (i < n && b[i] == '\r') i++;
            if (i >= n || b[i] != '\n') return 400;
            i++;
        }
        if (body->n > 0xFFFFFFFFu) return 400;
    } else if (clen > 0) {
        if ((int64_t)(n - i) < clen) return 400;
        ob_put(body, b + i, (size_t)clen);
    }
    return 0;
}

/* ngx_proxy_protocol_read (nginx 1.17.3 src/core/ngx_proxy_protocol.c) over the connection's
 * first bytes b[0, n): the header's length, or -1 for a missing / broken header (nginx logs
 * "broken header" and closes the connection).  v1: "PROXY TCP4|TCP6 <src> <dst> <sport> <dport>"
 * CRLF -- the source address kept as sent (hex digits, ':' and '.'), the port a decimal 0..65535,
 * the destination fields not checked, the line's end the first CRLF after the source port;
 * "PROXY UNKNOWN" ... CRLF: no address.  v2: the 12-byte signature, version 2, a length that fits;
 * PROXY command over STREAM with AF_INET / AF_INET6 gives the source address (ngx_sock_ntop) and
 * port; LOCAL, other transports or families: no address.  *alen = 0 when there is no address. */
static int o_proxy_read(const uint8_t *b, int n, char *addr, int *alen, int *port) {
    static const uint8_t sig[12] = {'\r', '\n', '\r', '\n', 0, '\r', '\n', 'Q', 'U', 'I', 'T', '\n'};
    *alen = 0; *port = 0;
    if (n >= 16 && !memcmp(b, sig, 12)) {
        if (b[12] >> 4 != 2) return -1;
        int len = b[14] << 8 | b[15];
        if (n - 16 < len) return -1;
        int end = 16 + len;
        if ((b[12] & 15) != 1 || (b[13] & 15) != 1) return end;
        oaddr_t a; memset(&a, 0, sizeof a);
        int fam = b[13] >> 4;
        if (fam == 1) {
            if (len < 12) return -1;
            a.fam = 4; memcpy(a.b, b + 16, 4); *port = b[24] << 8 | b[25];
        } else if (fam == 2) {
            if (len < 36) return -1;
            a.fam = 6; memcpy(a.b, b + 16, 16); *port = b[48] << 8 | b[49];
        } else return end;
        *alen = o_ntop(&a, addr);
        return end;
    }
    if (n < 8 || memcmp(b, "PROXY ", 6)) return -1;
    int p = 6;
    if (n - 6 >= 7 && !memcmp(b + 6, "UNKNOWN", 7)) p += 7;
    else {
        if (n - 6 < 5 || memcmp(b + 6, "TCP", 3) || (b[9] != '4' && b[9] != '6') || b[10] != ' ') return -1;
        p = 11;
        int a0 = p;
        for (;;) {
            if (p == n) return -1;
            int ch = b[p++];
            if (ch == ' ') break;
            if (ch != ':' && ch != '.' && !isxdigit(ch)) return -1;
        }
        int al = p - a0 - 1;
        while (1) { if (p == n) return -1; if (b[p++] == ' ') break; }
        int p0 = p;
        while (1) { if (p == n) return -1; if (b[p++] == ' ') break; }
        int pl = p - p0 - 1;
        if (pl == 0) return -1;
        long v = 0;
        for (int k = 0; k < pl; k++) {
            if (!isdigit(b[p0 + k]) || v > 100000000L) return -1;
            v = v * 10 + (b[p0 + k] - '0');
        }
        if (v > 65535) return -1;
        *port = (int)v;
        if (al <= 46) { memcpy(addr, b + a0, (size_t)al); *alen = al; }   /* longer: never an address */
    }
    for (; p + 1 < n; p++) if (b[p] == '\r' && b[p + 1] == '\n') return p + 2;
    *alen = 0; *port = 0;
    return -1;
}

/* the generation's `listen ... proxy_protocol` ports (ORed over every listen of a port) */
int orc_proxy_ports(orc_ctx *c, uint16_t *out, int cap) {
    int k = 0;
    for (int s = 0; s < c->nsrv; s++)
        for (int i = 0; i < c->srv[s].nports; i++) {
            if (!c->srv[s].pp[i]) continue;
            int seen = 0;
            for (int j = 0; j < k; j++) seen |= out[j] == c->srv[s].ports[i];
            if (!seen && k < cap) out[k++] = (uint16_t)c->srv[s].ports[i];
        }
    return k;
}

/* n requests -> gm_req records + a packed payload arena (gm_req field order, 16-B aligned
 * bases).  Returns the arena length, or -1 if `cap` is too small.  pports[0, npp): the listen
 * ports with proxy_protocol: a message there starts with its connection's PROXY header (unless
 * GM_WIRE_PROXY_DONE: a keep-alive request, the caller's paddr / proxy_port) -- a broken or
 * missing one, or one with no request after it, gives an invalid record with status 444. */
int64_t orc_parse_requests_pp(const uint8_t *wire, const gm_wire_msg *msgs, uint32_t n, gm_req *reqs, uint8_t *arena,
                              uint64_t cap, const uint16_t *pports, int npp) {
    obuf_t uri = {0}, hdrs = {0}, body = {0};
    uint64_t o = 0;
    int64_t rc = 0;
    for (uint32_t k = 0; k < n; k++) {
        const gm_wire_msg *m = &msgs[k];
        orc_rl_t R;
        const uint8_t *host; int host_len;
        uri.n = hdrs.n = body.n = 0;
        int proxy = 0;
        for (int j = 0; j < npp; j++) proxy |= pports[j] == m->port;
        const uint8_t *mb = wire + m->off;
        int mn = (int)m->len;
        char pa[64]; int pal = 0, pport = 0, st;
        if (proxy && (m->flags & GM_WIRE_PROXY_DONE)) {
            pal = m->paddr_len <= 46 ? m->paddr_len : 0;
            memcpy(pa, m->paddr, (size_t)pal);
            pport = m->proxy_port;
            st = -1;
        } else if (proxy) {
            int used = o_proxy_read(mb, mn, pa, &pal, &pport);
            if (used < 0 || used >= mn) { st = 444; pal = 0; pport = 0; }
            else { mb += used; mn -= used; st = -1; }
        } else st = -1;
        if (st < 0) st = orc_parse_one(mb, mn, &R, &uri, &hdrs, &body, &host, &host_len);
        gm_req *r = &reqs[k];
        memset(r, 0, sizeof *r);
        r->base = o;
        r->port = m->port; r->remote_port = m->remote_port;
        memcpy(r->rid, m->rid, 16);
        const int ra = m->raddr_len > 40 ? 40 : m->raddr_len;
        r->flags = m->flags & (GM_REQ_HTTPS | GM_REQ_HTTP2);
        r->pad0[0] = (uint8_t)pal;
        if (pal) { r->pad1[0] = (uint8_t)pport; r->pad1[1] = (uint8_t)(pport >> 8); }
        const uint8_t *seg[9]; size_t len[9] = {0};
        if (st) {
            r->flags |= GM_REQ_INVALID;
            r->pad0[1] = (uint8_t)(st & 0xFF); r->pad0[2] = (uint8_t)(st >> 8);
        } else {
            if (R.minor == 0) r->flags |= GM_REQ_HTTP10;
            if (R.chunked) r->flags |= GM_REQ_CHUNKED;
            seg[0] = uri.p; len[0] = uri.n;
            seg[1] = R.args; len[1] = (size_t)R.args_len;
            seg[2] = hdrs.p; len[2] = hdrs.n;
            seg[3] = body.p; len[3] = body.n;
            seg[4] = host; len[4] = (size_t)host_len;
            seg[5] = R.method; len[5] = (size_t)R.method_len;
            seg[6] = R.target; len[6] = (size_t)R.target_len;
        }
        seg[7] = m->raddr; len[7] = (size_t)ra;
        seg[8] = (const uint8_t *)pa; len[8] = (size_t)pal;
        r->uri_len = (uint32_t)len[0]; r->args_len = (uint32_t)len[1]; r->hdr_len = (uint32_t)len[2];
        r->body_len = (uint32_t)len[3]; r->host_len = (uint16_t)len[4]; r->method_len = (uint16_t)len[5];
        r->ruri_len = (uint16_t)len[6]; r->raddr_len = (uint16_t)len[7];
        size_t tot = 0;
        for (int f = 0; f < 9; f++) tot += len[f];
        if (o + tot > cap) { rc = -1; break; }
        for (int f = 0; f < 9; f++) if (len[f]) { memcpy(arena + o, seg[f], len[f]); o += len[f]; }
        while (o & 15) { if (o < cap) arena[o] = 0; o++; }
    }
    free(uri.p); free(hdrs.p); free(body.p);
    return rc < 0 ? -1 : (int64_t)o;
}
int64_t orc_parse_requests(const uint8_t *wire, const gm_wire_msg *msgs, uint32_t n, gm_req *reqs, uint8_t *arena,
                           uint64_t cap) {
    return orc_parse_requests_pp(wire, msgs, n, reqs, arena, cap, NULL, 0);
}


/* RFC 1321 MD5, written from the RFC's round definitions (F, G, H, I and the four rounds of 16
 * operations), for the NGINX Plus sticky cookie: its value is the lowercase hex MD5 of the peer's
 * address text */
#define MD5_ROT(x, c) (((x) << (c)) | ((x) >> (32 - (c))))
static void o_md5_block(uint32_t st[4], const uint8_t b[64]) {
    uint32_t X[16];
    for (int i = 0; i < 16; i++) X[i] = (uint32_t)b[4 * i] | (uint32_t)b[4 * i + 1] << 8 | (uint32_t)b[4 * i + 2] << 16 | (uint32_t)b[4 * i + 3] << 24;
    uint32_t a = st[0], bb = st[1], c = st[2], d = st[3];
#define FF(a, b, c, d, k, s, t) a = b + MD5_ROT(a + (((b) & (c)) | (~(b) & (d))) + X[k] + (t), s)
#define GG(a, b, c, d, k, s, t) a = b + MD5_ROT(a + (((b) & (d)) | ((c) & ~(d))) + X[k] + (t), s)
#define HH(a, b, c, d, k, s, t) a = b + MD5_ROT(a + ((b) ^ (c) ^ (d)) + X[k] + (t), s)
#define II(a, b, c, d, k, s, t) a = b + MD5_ROT(a + ((c) ^ ((b) | ~(d))) + X[k] + (t), s)
    FF(a, bb, c, d, 0, 7, 0xd76aa478); FF(d, a, bb, c, 1, 12, 0xe8c7b756); FF(c, d, a, bb, 2, 17, 0x242070db); FF(bb, c, d, a, 3, 22, 0xc1bdceee);
    FF(a, bb, c, d, 4, 7, 0xf57c0faf); FF(d, a, bb, c, 5, 12, 0x4787c62a); FF(c, d, a, bb, 6, 17, 0xa8304613); FF(bb, c, d, a, 7, 22, 0xfd469501);
    FF(a, bb, c, d, 8, 7, 0x698098d8); FF(d, a, bb, c, 9, 12, 0x8b44f7af); FF(c, d, a, bb, 10, 17, 0xffff5bb1); FF(bb, c, d, a, 11, 22, 0x895cd7be);
    FF(a, bb, c, d, 12, 7, 0x6b901122); FF(d, a, bb, c, 13, 12, 0xfd987193); FF(c, d, a, bb, 14, 17, 0xa679438e); FF(bb, c, d, a, 15, 22, 0x49b40821);
    GG(a, bb, c, d, 1, 5, 0xf61e2562); GG(d, a, bb, c, 6, 9, 0xc040b340); GG(c, d, a, bb, 11, 14, 0x265e5a51); GG(bb, c, d, a, 0, 20, 0xe9b6c7aa);
    GG(a, bb, c, d, 5, 5, 0xd62f105d); GG(d, a, bb, c, 10, 9, 0x02441453); GG(c, d, a, bb, 15, 14, 0xd8a1e681); GG(bb, c, d, a, 4, 20, 0xe7d3fbc8);
    GG(a, bb, c, d, 9, 5, 0x21e1cde6); GG(d, a, bb, c, 14, 9, 0xc33707d6); GG(c, d, a, bb, 3, 14, 0xf4d50d87); GG(bb, c, d, a, 8, 20, 0x455a14ed);
    GG(a, bb, c, d, 13, 5, 0xa9e3e905); GG(d, a, bb, c, 2, 9, 0xfcefa3f8); GG(c, d, a, bb, 7, 14, 0x676f02d9); GG(bb, c, d, a, 12, 20, 0x8d2a4c8a);
    HH(a, bb, c, d, 5, 4, 0xfffa3942); HH(d, a, bb, c, 8, 11, 0x8771f681); HH(c, d, a, bb, 11, 16, 0x6d9d6122); HH(bb, c, d, a, 14, 23, 0xfde5380c);
    HH(a, bb, c, d, 1, 4, 0xa4beea44); HH(d, a, bb, c, 4, 11, 0x4bdecfa9); HH(c, d, a, bb, 7, 16, 0xf6bb4b60); HH(bb, c, d, a, 10, 23, 0xbebfbc70);
    HH(a, bb, c, d, 13, 4, 0x289b7ec6); HH(d, a, bb, c, 0, 11, 0xeaa127fa); HH(c, d, a, bb, 3, 16, 0xd4ef3085); HH(bb, c, d, a, 6, 23, 0x04881d05);
    HH(a, bb, c, d, 9, 4, 0xd9d4d039); HH(d, a, bb, c, 12, 11, 0xe6db99e5); HH(c, d, a, bb, 15, 16, 0x1fa27cf8); HH(bb, c, d, a, 2, 23, 0xc4ac5665);
    II(a, bb, c, d, 0, 6, 0xf4292244); II(d, a, bb, c, 7, 10, 0x432aff97); II(c, d, a, bb, 14, 15, 0xab9423a7); II(bb, c, d, a, 5, 21, 0xfc93a039);
    II(a, bb, c, d, 12, 6, 0x655b59c3); II(d, a, bb, c, 3, 10, 0x8f0ccc92); II(c, d, a, bb, 10, 15, 0xffeff47d); II(bb, c, d, a, 1, 21, 0x85845dd1);
    II(a, bb, c, d, 8, 6, 0x6fa87e4f); II(d, a, bb, c, 15, 10, 0xfe2ce6e0); II(c, d, a, bb, 6, 15, 0xa3014314); II(bb, c, d, a, 13, 21, 0x4e0811a1);
    II(a, bb, c, d, 4, 6, 0xf7537e82); II(d, a, bb, c, 11, 10, 0xbd3af235); II(c, d, a, bb, 2, 15, 0x2ad7d2bb); II(bb, c, d, a, 9, 21, 0xeb86d391);
#undef FF
#undef GG
#undef HH
#undef II
    st[0] += a; st[1] += bb; st[2] += c; st[3] += d;
}
/* lowercase hex of MD5(p[0, n)) into out[33] */
void orc_md5_hex(const char *p, int n, char *out) {
    uint32_t st[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
    int i = 0;
    for (; i + 64 <= n; i += 64) o_md5_block(st, (const uint8_t *)p + i);
    uint8_t tail[128] = {0};
    int r = n - i;
    memcpy(tail, p + i, (size_t)r);
    tail[r] = 0x80;
    int tl = r + 1 + 8 <= 64 ? 64 : 128;
    uint64_t bits = (uint64_t)n * 8;
    for (int k = 0; k < 8; k++) tail[tl - 8 + k] = (uint8_t)(bits >> (8 * k));
    o_md5_block(st, tail);
    if (tl == 128) o_md5_block(st, tail + 64);
    for (int k = 0; k < 16; k++) sprintf(out + 2 * k, "%02x", (st[k / 4] >> (8 * (k % 4))) & 0xFF);
    out[32] = 0;
}

/* ------------------------------------------------------------------ peer selection (§8 f3) */
static uint32_t orc_draw(const uint8_t rid[16], uint32_t j) {
    uint64_t lo = 0, hi = 0;
    for (int i = 7; i >= 0; i--) { lo = lo << 8 | rid[i]; hi = hi << 8 | rid[8 + i]; }
    uint64_t x = lo ^ (hi * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(j + 1) * 0xD1B54A32D192ED03ull);
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return (uint32_t)(x >> 32);
}

#define LIVE(j) (!(st[U->first_peer + (j)].flags & GM_PEER_DOWN))

/* ngx_http_upstream_get_round_robin_peer (weights 1): single peer, else smooth WRR */
static int orc_rr(oups_t *U, gm_peer_state *st) {
    int n = U->npeers;
    if (n == 1) return LIVE(0) ? 0 : -1;
    int best = -1, total = 0;
    for (int j = 0; j < n; j++) {
        if (!LIVE(j)) continue;
        gm_peer_state *e = &st[U->first_peer + j];
        e->current_weight += 1; total += 1;
        if (best < 0 || e->current_weight > st[U->first_peer + best].current_weight) best = j;
    }
    if (best < 0) return -1;
    st[U->first_peer + best].current_weight -= total;
    return best;
}

/* ngx_http_upstream_get_least_conn_peer (weights 1) */
static int orc_lc(oups_t *U, gm_peer_state *st) {
    int n = U->npeers, best = -1, many = 0;
    for (int j = 0; j < n; j++) {
        if (!LIVE(j)) continue;
        if (best < 0 || st[U->first_peer + j].conns < st[U->first_peer + best].conns) { best = j; many = 0; }
        else if (st[U->first_peer + j].conns == st[U->first_peer + best].conns) many = 1;
    }
    if (best < 0) return -1;
    if (many) {
        int b = best, total = 0;
        for (int j = best; j < n; j++) {
            if (!LIVE(j) || st[U->first_peer + j].conns != st[U->first_peer + b].conns) continue;
            st[U->first_peer + j].current_weight += 1; total += 1;
            if (st[U->first_peer + j].current_weight > st[U->first_peer + b].current_weight) b = j;
        }
        st[U->first_peer + b].current_weight -= total;
        best = b;
    }
    return best;
}

/* -1: round robin, -2: defer; st conns are the batch-start snapshot for random two */
static int orc_stateless(orc_ctx *c, oups_t *U, const gm_req *r, const uint8_t *arena, gm_peer_state *st,
                         const uint32_t *snap_conns, scratch_t *sc, uint32_t server) {
    int n = U->npeers;
    if (U->method == OM_RANDOM) {
        for (uint32_t tries = 0;;) {
            int x = (int)(orc_draw(r->rid, tries) % (uint32_t)n);
            if (LIVE(x)) return x;
            if (++tries > 20) return -1;
        }
    }
    if (U->method == OM_RANDOM2) {
        if (n < 2) return -1;
        int first = -1; uint32_t tries = 0;
        for (uint32_t j = 0;; j++) {
            int x = (int)(orc_draw(r->rid, j) % (uint32_t)n);
            if (LIVE(x) && x != first) {
                if (first < 0) { first = x; continue; }
                return snap_conns[U->first_peer + first] < snap_conns[U->first_peer + x] ? first : x;
            }
            if (++tries > 20) return -1;
        }
    }
    if (n == 1) return -1;
    rq_t q; rq_init(&q, r, arena);
    if (server < (uint32_t)c->nsrv) q.S = &c->srv[server];
    if (U->method == OM_IP_HASH) {
        uint8_t b[16] = {0}; int alen = 3;
        char t[64];
        orc_realip(&q);   /* ip_hash hashes the address the realip module set */
        if (q.rip == 3) return -2;
        if (q.rip == 2) {
            memcpy(b, q.raddr2.b, 16); alen = q.raddr2.fam == 4 ? 3 : 16;
        } else if (q.raddr.n < (int)sizeof t) {
            memcpy(t, q.raddr.p, q.raddr.n); t[q.raddr.n] = 0;
            uint8_t a6[16];
            if (inet_pton(AF_INET, t, b) == 1) alen = 3;
            else if (inet_pton(AF_INET6, t, a6) == 1) { memcpy(b, a6, 16); alen = 16; }
            else memset(b, 0, sizeof b);
        }
        uint32_t hash = 89;
        for (uint32_t tries = 0;;) {
            for (int i = 0; i < alen; i++) hash = (hash * 113 + b[i]) % 6271;
            int w = (int)(hash % (uint32_t)n);
            if (LIVE(w)) return w;
            if (++tries > 20) return -1;
        }
    }
    ev_t E = {c, &q, sc, 0, NULL, NULL};
    sv key = eval_complex(&E, U->key);
    if (E.unknown) return -2;
    if (key.n == 0) return -1;
    if (U->method == OM_CHASH) {
        uint32_t h = orc_crc32(key.p, key.n);
        int lo = 0, hi = U->nring;   /* ngx_http_upstream_find_chash_point */
        while (lo < hi) {
            int k = (lo + hi) / 2;
            if (h > U->ring[k].hash) lo = k + 1; else if (h < U->ring[k].hash) hi = k; else { lo = k; break; }
        }
        for (uint32_t tries = 0;; lo++) {
            int j = U->ring[lo % U->nring].peer;
            if (LIVE(j)) return j;
            if (++tries > 20) return -1;
        }
    }
    /* hash: ((crc32([REHASH] KEY) >> 16) & 0x7fff) + PREV_HASH */
    uint32_t acc = 0;
    for (uint32_t tries = 0, rehash = 0;;) {
        uint32_t cr = 0xFFFFFFFFu;
        if (rehash > 0) { char d[16]; int dn = snprintf(d, sizeof d, "%u", rehash); cr = crc32_bytes(cr, d, dn); }
        cr = crc32_bytes(cr, key.p, key.n) ^ 0xFFFFFFFFu;
        acc += (cr >> 16) & 0x7FFF;
        rehash++;
        int w = (int)(acc % (uint32_t)n);
        if (LIVE(w)) return w;
        if (++tries > 20) return -1;
    }
}

/* Select peers for n verdicts in request order, updating st (gm_peer_state per peer: conns +=
 * picks, current_weight).  Returns 0, or -1 if n_peers differs from the generation's. */
int orc_select_peers(orc_ctx *c, const gm_req *reqs, const uint8_t *arena, const gm_verdict *v, uint32_t n,
                     gm_peer_state *st, uint32_t n_peers, uint32_t *out) {
    if ((int)n_peers != c->total_peers) return -1;
    uint32_t *snap = malloc(sizeof(uint32_t) * (n_peers ? n_peers : 1));
    for (uint32_t j = 0; j < n_peers; j++) snap[j] = st[j].conns;
    uint32_t *picks = calloc(n_peers ? n_peers : 1, sizeof(uint32_t));
    scratch_t sc = {NULL};
    for (uint32_t i = 0; i < n; i++) {
        out[i] = GM_NONE;
        if (v[i].action != GM_ACT_PROXY || v[i].upstream_id == GM_NONE) continue;
        if (v[i].gen != c->gen || (int)v[i].upstream_id >= c->nups) { out[i] = GM_PEER_DEFER; continue; }
        oups_t *U = c->uby[v[i].upstream_id];
        if (!U || U->method == OM_DEFER) { out[i] = GM_PEER_DEFER; continue; }
        if (U->npeers == 0) continue;
        int p = -1;
        if (U->sticky) {
            /* the cookie names a live peer by the hex MD5 of its address: that peer, counted with
             * the batch (it does not take part in the round-robin / least_conn sequence) */
            rq_t q; rq_init(&q, &reqs[i], arena);
            if (v[i].server_id < (uint32_t)c->nsrv) q.S = &c->srv[v[i].server_id];
            ev_t E = {c, &q, &sc, 0, NULL, NULL};
            sv ck = eval_complex(&E, U->sticky);
            if (ck.n == 32) {
                for (int j = 0; j < U->npeers && p < 0; j++) {
                    char h[33];
                    orc_md5_hex(U->addr[j], (int)strlen(U->addr[j]), h);
                    if (!memcmp(h, ck.p, 32) && LIVE(j)) p = j;
                }
            }
            sc_reset(&sc);
            if (p >= 0) { picks[U->first_peer + p]++; out[i] = (uint32_t)(U->first_peer + p); continue; }
        }
        if (U->method == OM_LEAST_CONN) {
            p = orc_lc(U, st);
            if (p >= 0) st[U->first_peer + p].conns++;   /* least_conn sees its own picks at once */
        } else {
            p = U->method == OM_RR ? -1 : orc_stateless(c, U, &reqs[i], arena, st, snap, &sc, v[i].server_id);
            if (p == -2) { out[i] = GM_PEER_DEFER; continue; }
            /* the engine's round-robin fallback holds at most 1024 peers (SEQ_PEERS_MAX) */
            if (p == -1 && U->npeers > 1024) { out[i] = GM_PEER_DEFER; continue; }
            if (p == -1) p = orc_rr(U, st);
            if (p >= 0) picks[U->first_peer + p]++;
        }
        sc_reset(&sc);
        if (p >= 0) out[i] = (uint32_t)(U->first_peer + p);
    }
    for (uint32_t j = 0; j < n_peers; j++) st[j].conns += picks[j];
    free(snap); free(picks); sc_reset(&sc); free(sc.head);
    return 0;
}

int orc_n_peers(orc_ctx *c) { return c->total_peers; }

/* the initial state of a generation (gm_peers_init) */
int orc_peers_init(orc_ctx *c, gm_peer_state *st, uint32_t n_peers) {
    if ((int)n_peers != c->total_peers) return -1;
    memset(st, 0, sizeof(gm_peer_state) * n_peers);
    for (int u = 0; u < c->nups; u++) {
        oups_t *U = c->uby[u];
        if (!U) continue;
        for (int j = 0; j < U->npeers; j++) st[U->first_peer + j].flags = U->down[j] ? GM_PEER_DOWN : 0;
    }
    return 0;
}

/* ------------------------------------------------------------------ upstream request URI (§8 f1)
 * ngx_http_proxy_create_request restated: proxy_pass without a URI part sends the unparsed
 * $request_uri; with one (nginx.org/rewrites) the URI part + $uri after the location prefix
 * (ngx_escape_uri NGX_ESCAPE_URI when r->quoted_uri) + "?" $args.  r->quoted_uri: the request-line
 * parser (ngx_http_parse_request_line) met '%' in sw_check_uri / sw_after_slash_in_uri, i.e.
 * before any '?', '#', "/." or "//" moved it to sw_uri. */
static int orc_quoted(const char *p, int n) {
    int slash = 0;
    for (int i = 0; i < n; i++) {
        char c = p[i];
        if (c == '%') return 1;
        if (c == '?' || c == '#') return 0;
        if (slash && (c == '.' || c == '/')) return 0;
        slash = c == '/';
    }
    return 0;
}

static int orc_esc(unsigned char c) {   /* ngx_escape_uri's NGX_ESCAPE_URI table */
    static const uint32_t uri[] = {0xffffffff, 0x80000029, 0x00000000, 0x80000000,
                                   0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff};
    return (uri[c >> 5] >> (c & 0x1f)) & 1;
}

/* out_off[i] = running offset; out_len[i] = length, GM_NONE (not proxied / past cap) or
 * GM_PEER_DEFER.  Returns the total bytes, or -1 if cap was exceeded. */
int64_t orc_upstream_uris(orc_ctx *c, const gm_req *reqs, const uint8_t *arena, const gm_verdict *v, uint32_t n,
                          uint8_t *out, uint64_t cap, uint64_t *out_off, uint32_t *out_len) {
    uint64_t off = 0; int over = 0;
    static const char hex[] = "0123456789ABCDEF";
    for (uint32_t i = 0; i < n; i++) {
        out_off[i] = off; out_len[i] = GM_NONE;
        if (v[i].action != GM_ACT_PROXY || v[i].location_id == GM_NONE) continue;
        if (v[i].gen != c->gen || (int)v[i].location_id >= c->nloc) { out_len[i] = GM_PEER_DEFER; continue; }
        loc_t *L = &c->loc[v[i].location_id];
        if (L->pass_defer) { out_len[i] = GM_PEER_DEFER; continue; }
        rq_t q; rq_init(&q, &reqs[i], arena);
        uint8_t *buf = malloc(3 * (size_t)q.uri.n + q.args.n + q.ruri.n + (L->pass_uri ? strlen(L->pass_uri) : 0) + 8);
        size_t k = 0;
        if (!L->pass_uri) {
            if (q.ruri.n) { memcpy(buf, q.ruri.p, q.ruri.n); k = q.ruri.n; }
            else {
                memcpy(buf, q.uri.p, q.uri.n); k = q.uri.n;
                if (q.args.n) { buf[k++] = '?'; memcpy(buf + k, q.args.p, q.args.n); k += q.args.n; }
            }
        } else {
            size_t rl = strlen(L->pass_uri);
            memcpy(buf, L->pass_uri, rl); k = rl;
            int esc = q.ruri.n ? orc_quoted(q.ruri.p, q.ruri.n) : orc_quoted(q.uri.p, q.uri.n);
            int t0 = L->plen < q.uri.n ? L->plen : q.uri.n;
            for (int j = t0; j < q.uri.n; j++) {
                unsigned char ch = (unsigned char)q.uri.p[j];
                if (esc && orc_esc(ch)) { buf[k++] = '%'; buf[k++] = hex[ch >> 4]; buf[k++] = hex[ch & 15]; }
                else buf[k++] = ch;
            }
            if (q.args.n) { buf[k++] = '?'; memcpy(buf + k, q.args.p, q.args.n); k += q.args.n; }
        }
        if (off + k > cap) { over = 1; free(buf); continue; }
        memcpy(out + off, buf, k);
        out_len[i] = (uint32_t)k;
        off += k;
        free(buf);
    }
    return over ? -1 : (int64_t)off;
}
