// gm_device.hip -- gfx950 kernels + host runtime + C-ABI of libgpumatch.so.
//
// Pipeline of one gm_match_batch (all on the caller's HIP stream):
//   1. route   (lane per request)  host -> server, server rewrite `if`s, location trie / regex
//                                   locations, IRL -> rules truth table / split_clients, verdict;
//                                   per-location counters; arena block -> first record index.
//   2. scan    (wave per 1 KiB)    WAF prefilter over the flat arena: every byte position's
//                                   case-folded 4-gram probes an LDS bitmap (A) and, on a hit, a
//                                   second LDS bitmap (B); survivors are appended (ballot-free
//                                   wave prefix) to a candidate list.  HBM-bound by design.
//   3. verify  (lane per candidate) exact literal compare inside the record's zone -> (req, rule)
//                                   pairs; regex factor hits -> (req, zone, regex) jobs.
//   4. regex   (lane per job)      byte-class DFA over the zone -> pairs.  (+ always-run regexes)
//   5. finalize sort pairs, drop duplicates and requests whose location has WAF off, write the
//                                   hit-id list in request order, n_hits / first_hit_off / block.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/gpumatch.h"
#include "gm_compile.hpp"
#include "gm_inet.hpp"
#include "gm_tables.hpp"

using namespace gm;

// uint64_t is unsigned long here, for which HIP's device min / max have no overload: such calls
// (or a mix with unsigned long long) resolved to the double ones (v_cvt_f64 ... v_min_f64 per
// call, exact only below 2^53)
__device__ __forceinline__ unsigned long min(unsigned long a, unsigned long b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned long max(unsigned long a, unsigned long b) { return a > b ? a : b; }
__device__ __forceinline__ unsigned long min(unsigned long a, unsigned long long b) { return a < b ? a : (unsigned long)b; }
__device__ __forceinline__ unsigned long min(unsigned long long a, unsigned long b) { return a < b ? (unsigned long)a : b; }
__device__ __forceinline__ unsigned long max(unsigned long a, unsigned long long b) { return a > b ? a : (unsigned long)b; }
__device__ __forceinline__ unsigned long max(unsigned long long a, unsigned long b) { return a > b ? (unsigned long)a : b; }

// ============================================================================ device helpers
namespace {

struct Rec {
    uint64_t base;
    uint32_t uri_len, args_len, hdr_len, body_len;
    uint32_t host_len, method_len, ruri_len, raddr_len;
    uint32_t port, rport, flags;
    uint32_t bad_status;     // GM_REQ_INVALID: the wire parser's HTTP status (pad0[1..2])
    uint32_t rid[4];
    uint32_t paddr_len, pport;   // $proxy_protocol_addr (after raddr; pad0[0]) and its port (pad1[0..1])
};

__device__ __forceinline__ Rec load_rec(const gm_req *r) {
    const uint4 *p = reinterpret_cast<const uint4 *>(r);
    uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    Rec x;
    x.base = (uint64_t)a.x | ((uint64_t)a.y << 32);
    x.uri_len = a.z; x.args_len = a.w; x.hdr_len = b.x; x.body_len = b.y;
    x.host_len = b.z & 0xFFFF; x.method_len = b.z >> 16; x.ruri_len = b.w & 0xFFFF; x.raddr_len = b.w >> 16;
    x.port = c.x & 0xFFFF; x.rport = c.x >> 16; x.flags = c.y & 0xFF; x.bad_status = c.y >> 16;   // pad0[1] | pad0[2] << 8
    x.rid[0] = c.z; x.rid[1] = c.w; x.rid[2] = d.x; x.rid[3] = d.y;
    x.paddr_len = (c.y >> 8) & 0xFF; x.pport = d.z & 0xFFFF;
    return x;
}

__device__ __forceinline__ uint32_t lc(uint32_t c) { return (c - 'A' < 26u) ? (c | 0x20) : c; }

// value = up to MAXSEG byte segments (generic pointers: arena, table bytes or lane-private)
constexpr int MAXSEG = 12;
struct Val {
    const uint8_t *p[MAXSEG];
    uint32_t n[MAXSEG];
    int cnt;
    uint32_t total;
    bool overflow;
    bool unknown;            // a value the engine cannot know ($remote_addr under realip from the
                             // PROXY protocol header): the step that reads it defers the request
    __device__ void clear() { cnt = 0; total = 0; overflow = false; unknown = false; }
    __device__ void add(const uint8_t *q, uint32_t len) {
        if (len == 0) return;
        if (cnt == MAXSEG) { overflow = true; return; }
        p[cnt] = q; n[cnt] = len; cnt++; total += len;
    }
};

__constant__ uint8_t c_const[64] = "httpsonh2; , ?HTTP/2.0HTTP/1.0HTTP/1.1 0123456789abcdef";
// offsets into c_const: "http" 0, "https" 0(5), "on" 5, "h2" 7, "; " 9, ", " 11, "?" 13,
// "HTTP/2.0" 14, "HTTP/1.0" 22, "HTTP/1.1" 30, " " 38, hex digits 39

// realip outcome of a request (computed on first use): the connection address stays, the module
// replaced it (ra: the new address, its text and port), or the engine cannot know it
enum : uint32_t { RIPS_SAME = 1, RIPS_NEW = 2, RIPS_UNKNOWN = 3 };
struct Ctx {
    const uint8_t *A;
    Rec r;
    uint64_t uri, args, hdrs, body, host, method, ruri, raddr;
    uint8_t scratch[48];   // $request_id hex / $remote_port digits
    uint32_t rip;          // the server's DRealIp (GM_NONE: none)
    uint32_t rip_state;    // RIPS_*
    InetAddr ra, ra_tmp;   // (ra: the connection address, then the one the module takes)
    uint32_t ra_len;
    uint8_t ra_txt[48];
};

__device__ void realip_eval(Ctx &c, const GTab &t);
// rip: the server's realip settings -- evaluated here, at the top of the out-of-line step that
// needs the request's variables, where little else is live (called from deep inside the variable
// lookup, the call chain raised the route kernel's register allocation past its occupancy target)
__device__ __forceinline__ void ctx_init(Ctx &c, const uint8_t *A, const Rec &r, const GTab *t = nullptr,
                                         uint32_t rip = GM_NONE) {
    c.A = A; c.r = r;
    uint64_t o = r.base;
    c.uri = o; o += r.uri_len; c.args = o; o += r.args_len; c.hdrs = o; o += r.hdr_len;
    c.body = o; o += r.body_len; c.host = o; o += r.host_len; c.method = o; o += r.method_len;
    c.ruri = o; o += r.ruri_len; c.raddr = o;
    c.rip = rip; c.rip_state = RIPS_SAME;
    if (rip != GM_NONE) realip_eval(c, *t);
}

// exact per-byte flags (bit 7 of each byte) of the zero bytes of x
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// the first position of a byte flagged by `hit` (per-word flags) in A[p, e), or e: whole aligned
// 16-byte blocks (the first and the last masked to [p, e): an aligned block never leaves the
// allocation), exact SWAR flags per word
// NB = 2: 32 bytes a step, the second block's load out with the first -- for a header walk's LF
// search over a long value, otherwise a chain of dependent 16-byte loads (round 6); NB = 1 where
// the registers matter more (the FAST route pass)
template <int NB = 1, class F>
__device__ __forceinline__ uint64_t find_flagged(const uint8_t *A, uint64_t p, uint64_t e, F hit) {
    if (p >= e) return e;
    for (uint64_t b = p & ~15ull; b < e; b += 16 * NB) {
        uint32_t w[4 * NB];
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const uint4 q = j == 0 || b + 16 * j < e ? *reinterpret_cast<const uint4 *>(A + b + 16 * j) : make_uint4(0, 0, 0, 0);
            w[4 * j] = q.x; w[4 * j + 1] = q.y; w[4 * j + 2] = q.z; w[4 * j + 3] = q.w;
        }
#pragma unroll
        for (int k = 0; k < 4 * NB; k++) {
            uint32_t z = hit(w[k]);
            const uint64_t wb = b + 4 * k;   // bytes [wb, wb + 4)
            if (p > wb) z = p - wb >= 4 ? 0u : z & (~0u << (8 * (uint32_t)(p - wb)));
            if (wb + 4 > e) z = e <= wb ? 0u : z & ((1u << (8 * (uint32_t)(e - wb))) - 1u);
            if (z) return wb + (__builtin_ctz(z) >> 3);
        }
    }
    return e;
}

// first position of byte `ch` in A[p, e), or e
template <int NB = 1>
__device__ uint64_t find_byte(const uint8_t *A, uint64_t p, uint64_t e, uint32_t ch) {
    const uint32_t pat = ch * 0x01010101u;
    return find_flagged<NB>(A, p, e, [pat](uint32_t w) { return zero_bytes(w ^ pat); });
}

// first position of either byte in A[p, e), or e
__device__ uint64_t find_byte2(const uint8_t *A, uint64_t p, uint64_t e, uint32_t c1, uint32_t c2) {
    const uint32_t p1 = c1 * 0x01010101u, p2 = c2 * 0x01010101u;
    return find_flagged(A, p, e, [p1, p2](uint32_t w) { return zero_bytes(w ^ p1) | zero_bytes(w ^ p2); });
}

// the first ':' or LF in A[p, e) (e if neither); colon: it is the ':'
template <int NB = 1>
__device__ uint64_t find_colon_lf(const uint8_t *A, uint64_t p, uint64_t e, bool &colon) {
    colon = false;
    if (p >= e) return e;
    for (uint64_t b = p & ~15ull; b < e; b += 16 * NB) {   // (NB blocks a step, as find_flagged)
        uint32_t w[4 * NB];
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const uint4 q = j == 0 || b + 16 * j < e ? *reinterpret_cast<const uint4 *>(A + b + 16 * j) : make_uint4(0, 0, 0, 0);
            w[4 * j] = q.x; w[4 * j + 1] = q.y; w[4 * j + 2] = q.z; w[4 * j + 3] = q.w;
        }
#pragma unroll
        for (int k = 0; k < 4 * NB; k++) {
            const uint32_t zc = zero_bytes(w[k] ^ 0x3A3A3A3Au), zl = zero_bytes(w[k] ^ 0x0A0A0A0Au);
            uint32_t z = zc | zl;
            const uint64_t wb = b + 4 * k;   // bytes [wb, wb + 4)
            if (p > wb) z = p - wb >= 4 ? 0u : z & (~0u << (8 * (uint32_t)(p - wb)));
            if (wb + 4 > e) z = e <= wb ? 0u : z & ((1u << (8 * (uint32_t)(e - wb))) - 1u);
            if (z) {
                const uint32_t bit = (uint32_t)__builtin_ctz(z);
                colon = ((zc >> bit) & 1u) != 0;
                return wb + (bit >> 3);
            }
        }
    }
    return e;
}

// iterate "Name: value\r\n" lines (ngx_http_parse_header_line); returns false at end
struct HdrIt { uint64_t pos, end; };
// the next line's name only: [ns, ns + nl) up to its first ':' (c), the line ending at e (its LF,
// or the block's end); the value is read only for a line whose name matters (hdr_value) -- its CR
// check and space trims were three dependent byte loads per line of every walk (round 6)
template <int NB = 1>
__device__ bool hdr_next_name(const uint8_t *A, HdrIt &it, uint64_t &ns, uint32_t &nl, uint64_t &c, uint64_t &e) {
    while (it.pos < it.end) {
        const uint64_t st = it.pos;
        // the first ':' or LF: a ':' first names the line (its LF is searched from there on), a LF
        // first ends a line with no name (a ':' before the LF is before the line's CR too)
        bool colon;
        const uint64_t x = find_colon_lf(A, st, it.end, colon);
        if (!colon) { e = x; it.pos = e + 1; continue; }
        c = x;
        e = find_byte<NB>(A, c + 1, it.end, '\n');
        it.pos = e + 1;
        ns = st; nl = (uint32_t)(c - st);
        return true;
    }
    return false;
}
// (NB: the LF search's 16-byte blocks per step, find_flagged)
// the value of a line hdr_next_name returned: without the CR before its LF, without leading /
// trailing spaces (nginx skips ' ' only: a tab is value)
__device__ __forceinline__ void hdr_value(const uint8_t *A, uint64_t ns, uint64_t c, uint64_t e, uint64_t &vs, uint32_t &vl) {
    uint64_t le = e;
    if (le > ns && A[le - 1] == '\r') le--;
    uint64_t v0 = c + 1;
    while (v0 < le && A[v0] == ' ') v0++;
    uint64_t v1 = le;
    while (v1 > v0 && A[v1 - 1] == ' ') v1--;
    vs = v0; vl = (uint32_t)(v1 - v0);
}
__device__ bool hdr_next(const uint8_t *A, HdrIt &it, uint64_t &ns, uint32_t &nl, uint64_t &vs, uint32_t &vl) {
    uint64_t c, e;
    if (!hdr_next_name(A, it, ns, nl, c, e)) return false;
    hdr_value(A, ns, c, e, vs, vl);
    return true;
}

// header name vs a lowercase name, case-insensitively (the headers_in hash: lowcase_key)
__device__ bool hdr_name_ci(const uint8_t *A, uint64_t ns, uint32_t nl, const uint8_t *want, uint32_t wl) {
    if (nl != wl) return false;
    for (uint32_t i = 0; i < nl; i++) if (lc(A[ns + i]) != want[i]) return false;
    return true;
}

// header name vs variable suffix (lowercase, '-' -> '_'), ngx_http_variable_unknown_header
__device__ bool hdr_name_is(const uint8_t *A, uint64_t ns, uint32_t nl, const uint8_t *var, uint32_t vl) {
    if (nl != vl) return false;
    for (uint32_t i = 0; i < nl; i++) {
        uint32_t ch = A[ns + i];
        ch = (ch - 'A' < 26u) ? (ch | 0x20) : (ch == '-' ? '_' : ch);
        if (ch != var[i]) return false;
    }
    return true;
}

// A header (one line: no join), cookie or argument value as one arena span [vo, vo + vl):
// ngx_http_variable_unknown_header's first line, ngx_http_parse_multi_header_lines over every
// Cookie line, ngx_http_arg.  false: no such header / cookie / argument (the value "").  Spans
// stay in registers: rules_generic keeps them there instead of in a Val (lane-private memory).
template <int NB = 1>
__device__ bool span_http(const uint8_t *A, uint64_t hdrs, uint32_t hlen, const uint8_t *nm, uint32_t nml,
                          uint64_t &vo, uint32_t &vl) {
    HdrIt it{hdrs, hdrs + hlen};
    uint64_t ns, c, e; uint32_t nl;
    while (hdr_next_name<NB>(A, it, ns, nl, c, e))
        if (hdr_name_is(A, ns, nl, nm, nml)) { hdr_value(A, ns, c, e, vo, vl); return true; }
    return false;
}
// a cookie in one Cookie line's value [vs, vs + l): ngx_http_parse_multi_header_lines' loop
__device__ bool cookie_in_line(const uint8_t *A, uint64_t vs, uint32_t l, const uint8_t *nm, uint32_t nml,
                               uint64_t &vo, uint32_t &vl) {
    if (nml > l) return false;
    uint64_t start = vs, end = vs + l;
    while (start < end) {
        bool ok = end - start >= nml;
        for (uint32_t k = 0; ok && k < nml; k++) if (lc(A[start + k]) != nm[k]) ok = false;
        if (ok) {
            start += nml;
            while (start < end && A[start] == ' ') start++;
            // (nginx: `*start++ != '='` -- the byte tested is consumed even when it is not '=',
            // so a ';' or ',' there does not end the skip below)
            if (start < end && A[start++] == '=') {
                while (start < end && A[start] == ' ') start++;
                const uint64_t last = find_byte(A, start, end, ';');
                vo = start; vl = (uint32_t)(last - start);
                return true;
            }
        }
        start = find_byte2(A, start, end, ';', ',');
        if (start < end) start++;
        while (start < end && A[start] == ' ') start++;
    }
    return false;
}
template <int NB = 1>
__device__ bool span_cookie(const uint8_t *A, uint64_t hdrs, uint32_t hlen, const uint8_t *nm, uint32_t nml,
                            uint64_t &vo, uint32_t &vl) {
    HdrIt it{hdrs, hdrs + hlen};
    uint64_t ns, vs, c, e; uint32_t nl, l;
    const uint8_t cookie[7] = "cookie";
    while (hdr_next_name<NB>(A, it, ns, nl, c, e)) {
        if (!hdr_name_is(A, ns, nl, cookie, 6)) continue;
        hdr_value(A, ns, c, e, vs, l);
        if (cookie_in_line(A, vs, l, nm, nml, vo, vl)) return true;
    }
    return false;
}
// the first occurrence of the name at an argument start ("&" or the beginning) followed by '=':
// only argument starts can qualify, so they are visited directly
__device__ bool span_arg(const uint8_t *A, uint64_t a, uint32_t n, const uint8_t *nm, uint32_t L,
                         uint64_t &vo, uint32_t &vl) {
    for (uint32_t p = 0; p + L < n;) {
        bool ok = true;
        for (uint32_t k = 0; ok && k < L; k++) if (lc(A[a + p + k]) != nm[k]) ok = false;
        const uint32_t amp = (uint32_t)(find_byte(A, a + p, a + n, '&') - a);
        if (ok && A[a + p + L] == '=') { vo = a + p + L + 1; vl = amp - (p + L + 1); return true; }
        p = amp + 1;
    }
    return false;
}

__device__ void get_var(Ctx &c, const GTab &t, uint32_t src_id, Val &v) {
    v.clear();
    const DSrc s = t.srcs[src_id];
    const uint8_t *A = c.A;
    const Rec &r = c.r;
    if (s.kind == SRC_VAR) {
        switch (s.var) {
        case V_SCHEME: v.add(c_const, (r.flags & GM_REQ_HTTPS) ? 5 : 4); break;
        case V_HTTPS: if (r.flags & GM_REQ_HTTPS) v.add(c_const + 5, 2); break;
        case V_HTTP2: if (r.flags & GM_REQ_HTTP2) v.add(c_const + 7, 2); break;
        case V_METHOD: v.add(A + c.method, r.method_len); break;
        case V_ARGS: v.add(A + c.args, r.args_len); break;
        case V_URI: v.add(A + c.uri, r.uri_len); break;
        case V_REQUEST_BODY: break;
        case V_REMOTE_ADDR:
            if (c.rip_state == RIPS_UNKNOWN) v.unknown = true;
            else if (c.rip_state == RIPS_NEW) v.add(c.ra_txt, c.ra_len);
            else v.add(A + c.raddr, r.raddr_len);
            break;
        case V_HOST: v.add(A + c.host, r.host_len); break;
        case V_REQUEST_URI:
        case V_REQUEST:
            if (s.var == V_REQUEST) { v.add(A + c.method, r.method_len); v.add(c_const + 38, 1); }
            if (r.ruri_len) v.add(A + c.ruri, r.ruri_len);
            else {
                v.add(A + c.uri, r.uri_len);
                if (r.args_len) { v.add(c_const + 13, 1); v.add(A + c.args, r.args_len); }
            }
            if (s.var == V_REQUEST) {
                v.add(c_const + 38, 1);
                v.add(c_const + ((r.flags & GM_REQ_HTTP2) ? 14 : (r.flags & GM_REQ_HTTP10) ? 22 : 30), 8);
            }
            break;
        case V_REQUEST_ID:
            for (int i = 0; i < 16; i++) {
                uint32_t b = (r.rid[i >> 2] >> (8 * (i & 3))) & 0xFF;
                c.scratch[2 * i] = c_const[39 +(b >> 4)];
                c.scratch[2 * i + 1] = c_const[39 +(b & 15)];
            }
            v.add(c.scratch, 32);
            break;
        case V_REMOTE_PORT:
        case V_SERVER_PORT: {
            uint32_t x = s.var == V_REMOTE_PORT ? r.rport : r.port;
            if (s.var == V_REMOTE_PORT) {
                if (c.rip_state == RIPS_UNKNOWN) { v.unknown = true; break; }
                if (c.rip_state == RIPS_NEW) {
                    x = c.ra.port;
                    if (x == 0) break;   // ngx_http_variable_remote_port: no port -> ""
                }
            }
            uint8_t tmp[6]; int k = 0;
            do { tmp[k++] = (uint8_t)('0' + x % 10); x /= 10; } while (x);
            for (int i = 0; i < k; i++) c.scratch[i] = tmp[k - 1 - i];
            v.add(c.scratch, (uint32_t)k);
            break;
        }
        default: break;
        }
        return;
    }
    const uint8_t *nm = t.bytes + s.name_off;
    uint64_t vo = 0;
    uint32_t vl = 0;
    if (s.kind == SRC_HTTP) {
        if (!s.join) { if (span_http(A, c.hdrs, r.hdr_len, nm, s.name_len, vo, vl)) v.add(A + vo, vl); return; }
        HdrIt it{c.hdrs, c.hdrs + r.hdr_len};
        uint64_t ns, vs; uint32_t nl;
        bool have = false;
        while (hdr_next(A, it, ns, nl, vs, vl)) {
            if (!hdr_name_is(A, ns, nl, nm, s.name_len)) continue;
            if (have) v.add(c_const + (s.join == ';' ? 9 : 11), 2);
            v.add(A + vs, vl);
            have = true;
        }
        return;
    }
    if (s.kind == SRC_COOKIE) {
        if (span_cookie(A, c.hdrs, r.hdr_len, nm, s.name_len, vo, vl)) v.add(A + vo, vl);
        return;
    }
    if (s.kind == SRC_ARG) {
        if (span_arg(A, c.args, r.args_len, nm, s.name_len, vo, vl)) v.add(A + vo, vl);
    }
}

// ---- ngx_http_realip_module (post-read phase, nginx 1.17.3), for a server that configures it
// (set_real_ip_from, version1/nginx.ingress.tmpl:46-49, version2/nginx.virtualserver.tmpl:64-72).
// The client address comes from X-Real-IP (the first such header), a named header (the first),
// or X-Forwarded-For (every such header, the last one first).  A trusted (set_real_ip_from)
// connection address is replaced by the header's last address; with real_ip_recursive on, the
// list is walked leftwards past every trusted address (ngx_http_get_forwarded_addr).  $remote_addr
// then shows the new address as ngx_sock_ntop text, $remote_port its port (or "").  Out of line,
// run once per request that reads the address.  (The connection address is the record's raddr
// text; one that does not parse as an address is never trusted.)
// (register-light: the addresses live in the lane's Ctx -- private memory -- and the tables are read
// in place, so this rare step does not raise the route kernel's register allocation)
// out-of-line leaves: each keeps its own small register frame, so the call chain under
// realip_eval stays under the route kernel's occupancy target
// (out of line: realip_eval's own frame stays small -- a leaf holding all of them needs ~100
// VGPRs, which sets the route kernel's allocation above its target beside the scan)
#define GM_RIP_INL __noinline__
__device__ GM_RIP_INL bool d_parse_addr_port(const uint8_t *p, uint32_t n, InetAddr &a) { return ngx_parse_addr_port(p, n, a); }
__device__ GM_RIP_INL uint32_t d_parse_addr(const uint8_t *p, uint32_t n, uint8_t *b) { return ngx_parse_addr(p, n, b); }
__device__ GM_RIP_INL uint32_t d_addr_text(const InetAddr &a, uint8_t *out) { return ngx_addr_text(a, out); }
__device__ GM_RIP_INL bool rip_trusted(const GTab &t, const DRealIp *R, const InetAddr &a) {
    if (!a.fam) return false;
    for (uint32_t k = 0; k < R->n_cidr; k++) {
        const DCidr *c = t.cidrs + R->first_cidr + k;
        if (cidr_match1(a, c->family, reinterpret_cast<const uint8_t *>(c->addr), reinterpret_cast<const uint8_t *>(c->mask)))
            return true;
    }
    return false;
}
// ngx_http_get_forwarded_addr_internal over one header value, its recursion as a loop:
// 0 declined (a unchanged), 1 ok, 2 done (a = the last address taken); na: scratch
constexpr int RIP_DECLINED = 0, RIP_OK = 1, RIP_DONE = 2;
__device__ GM_RIP_INL int rip_forwarded(const GTab &t, const DRealIp *R, const uint8_t *x, uint32_t len, InetAddr &a,
                                          InetAddr &na) {
    for (int depth = 0;; depth++) {
        if (!rip_trusted(t, R, a) || len == 0) return depth ? RIP_DONE : RIP_DECLINED;
        uint32_t e = len;   // trailing ' ' and ',' (never the first byte)
        while (e > 1 && (x[e - 1] == ' ' || x[e - 1] == ',')) e--;
        uint32_t st = e - 1;   // the last address starts after the separator before it (byte 0
        while (st > 0) {       // is never taken for a separator)
            if (x[st] == ' ' || x[st] == ',') { st++; break; }
            st--;
        }
        if (!d_parse_addr_port(x + st, e - st, na)) return depth ? RIP_DONE : RIP_DECLINED;
        a = na;
        if (R->recursive && st > 0) { len = st - 1; continue; }
        return RIP_OK;
    }
}
// the k-th (0-based) header line named `want`: its value span; false if none
__device__ GM_RIP_INL bool hdr_nth(const Ctx &c, const uint8_t *want, uint32_t wl, uint32_t k, uint64_t &vs, uint32_t &vl) {
    HdrIt it{c.hdrs, c.hdrs + c.r.hdr_len};
    uint64_t ns; uint32_t nl;
    uint32_t seen = 0;
    while (hdr_next(c.A, it, ns, nl, vs, vl))
        if (hdr_name_ci(c.A, ns, nl, want, wl) && seen++ == k) return true;
    return false;
}
__device__ GM_RIP_INL uint32_t hdr_count(const Ctx &c, const uint8_t *want, uint32_t wl) {
    HdrIt it{c.hdrs, c.hdrs + c.r.hdr_len};
    uint64_t ns, vs; uint32_t nl, vl;
    uint32_t nh = 0;
    while (hdr_next(c.A, it, ns, nl, vs, vl)) nh += hdr_name_ci(c.A, ns, nl, want, wl);
    return nh;
}
// every X-Forwarded-For line, the last first (nginx's headers_in.x_forwarded_for array)
__device__ GM_RIP_INL int rip_xfwd(Ctx &c, const GTab &t, const DRealIp *R) {
    const uint8_t *want = (const uint8_t *)"x-forwarded-for";
    const uint32_t nh = hdr_count(c, want, 15);
    int rc = RIP_DECLINED;
    bool found = false;
    for (uint32_t k = nh; k-- > 0;) {
        uint64_t vs; uint32_t vl;
        hdr_nth(c, want, 15, k, vs, vl);
        rc = rip_forwarded(t, R, c.A + vs, vl, c.ra, c.ra_tmp);
        if (!R->recursive) break;
        if (rc == RIP_DECLINED && found) { rc = RIP_DONE; break; }
        if (rc != RIP_OK) break;
        found = true;
    }
    return rc;
}
// X-Real-IP or a named header: its first line
__device__ GM_RIP_INL int rip_one_header(Ctx &c, const GTab &t, const DRealIp *R) {
    const bool xr = R->type == RIP_XREALIP;
    uint64_t vs; uint32_t vl;
    if (!hdr_nth(c, xr ? (const uint8_t *)"x-real-ip" : t.bytes + R->hdr_off, xr ? 9u : R->hdr_len, 0, vs, vl))
        return RIP_DECLINED;
    return rip_forwarded(t, R, c.A + vs, vl, c.ra, c.ra_tmp);
}
__device__ __noinline__ void realip_eval(Ctx &c, const GTab &t) {
    const DRealIp *R = t.realip + c.rip;
    const uint8_t *A = c.A;
    InetAddr &a = c.ra;
    a.port = 0;
    a.fam = c.r.raddr_len <= 45 ? d_parse_addr(A + c.raddr, c.r.raddr_len, a.b) : 0u;
    c.rip_state = RIPS_SAME;
    const uint32_t type = R->type;
    if (type == RIP_UNKNOWN) { c.rip_state = RIPS_UNKNOWN; return; }
    int rc;
    if (type == RIP_PROXY) {
        // ngx_http_realip_handler, NGX_HTTP_REALIP_PROXY: the connection's PROXY header address
        // (none: declined) through ngx_http_get_forwarded_addr, then its port
        if (c.r.paddr_len == 0) return;
        rc = rip_forwarded(t, R, A + c.raddr + c.r.raddr_len, c.r.paddr_len, c.ra, c.ra_tmp);
        if (rc != RIP_DECLINED) a.port = c.r.pport;
    } else {
        rc = type == RIP_XFWD ? rip_xfwd(c, t, R) : rip_one_header(c, t, R);
    }
    if (rc == RIP_DECLINED) return;
    c.ra_len = d_addr_text(a, c.ra_txt);
    c.rip_state = RIPS_NEW;
}

__device__ bool val_eq(const Val &v, const uint8_t *key, uint32_t kl, bool nocase) {
    if (v.total != kl) return false;
    uint32_t k = 0;
    for (int s = 0; s < v.cnt; s++)
        for (uint32_t i = 0; i < v.n[s]; i++, k++) {
            uint32_t a = v.p[s][i];
            if (nocase) a = lc(a);
            if (a != key[k]) return false;
        }
    return true;
}

// PCRE search semantics on a byte stream given as segments (see gm_regex.cpp dfa_search)
__device__ bool dfa_run_val(const GTab &t, uint32_t dfa_id, const Val &v) {
    const DDfa d = t.dfas[dfa_id];
    const uint16_t *tr = t.dfa_trans + d.trans_off;
    const uint8_t *acc = t.dfa_acc + d.acc_off, *cls = t.dfa_cls + d.cls_off;
    uint32_t st = 1, fl = acc[1];   // fl: accept flags of st (packed into the transitions)
    if (fl & 1) return true;
    uint32_t pos = 0;
    for (int s = 0; s < v.cnt; s++)
        for (uint32_t i = 0; i < v.n[s]; i++, pos++) {
            uint8_t b = v.p[s][i];
            if ((fl & 2) && pos + 1 == v.total && b == '\n') return true;
            const uint32_t e = tr[st * d.n_classes + cls[b]];
            st = e & DFA_TRANS_STATE_MASK; fl = e >> 14;
            if (st == 0) return false;
            if (fl & 1) return true;
        }
    return (fl & 2) != 0;
}

// `steps` (optional) accumulates the bytes consumed -- profiling counters of the WAF verify
__device__ bool dfa_run_bytes(const GTab &t, uint32_t dfa_id, const uint8_t *p, uint32_t n, uint32_t *steps = nullptr) {
    const DDfa d = t.dfas[dfa_id];
    const uint16_t *tr = t.dfa_trans + d.trans_off;
    const uint8_t *acc = t.dfa_acc + d.acc_off, *cls = t.dfa_cls + d.cls_off;
    uint32_t st = 1, fl = acc[1];   // fl: accept flags of st (packed into the transitions)
    if (fl & 1) return true;
    uint32_t i = 0;
    bool r = false;
    // the next byte's class is loaded one step ahead: the only serial load per byte is the
    // transition itself
    uint32_t cn = n ? cls[p[0]] : 0u;
    for (; i < n; i++) {
        const uint32_t cc = cn;
        if (i + 1 < n) cn = cls[p[i + 1]];
        else if ((fl & 2) && p[i] == '\n') { r = true; break; }   // $ before a final newline
        const uint32_t e = tr[st * d.n_classes + cc];
        st = e & DFA_TRANS_STATE_MASK; fl = e >> 14;
        if (st == 0) break;
        if (fl & 1) { r = true; break; }
    }
    if (i == n) r = (fl & 2) != 0;
    if (steps) *steps += i;
    return r;
}

// Regex locations of a large server: the first regex in config
// order that matches `u`, behind the factor prefilter (gm_tables.hpp RLOC_SEQ_MAX).  One pass
// over the URI's folded 4-byte windows collects the RK_K smallest candidate indices >= lo
// (sorted in registers); they run in order, merged with the server's always list; if all RK_K
// fail the next pass collects the candidates after them.  Rejected (PCRE-only) regexes are in the
// always list with dfa GM_NONE and "match" when reached.  Out of line: the route fast path
// keeps its registers.
constexpr int RK_K = 8;
#ifndef GM_EXP_WPE
#define GM_EXP_WPE 3
#endif
#ifndef GM_EXP_GRIDMUL
#define GM_EXP_GRIDMUL 8
#endif
#ifdef GM_EXP_COUNT
__device__ unsigned long long g_exp[8];
#endif
__device__ __noinline__ int32_t rloc_prefiltered(const GTab &t, const DServer &S, uint32_t sid, const uint8_t *u,
                                                 uint32_t ulen, const uint32_t *rkb) {
    auto run = [&](uint32_t k) -> bool {
        const DRegexLoc rl = t.rlocs[S.first_rloc + k];
#ifdef GM_EXP_COUNT
        uint32_t steps = 0;
        const uint64_t t0 = __builtin_readcyclecounter();
        const bool m = rl.dfa == GM_NONE || dfa_run_bytes(t, rl.dfa, u, ulen, &steps);
        atomicAdd(&g_exp[1], 1ull); atomicAdd(&g_exp[2], (unsigned long long)steps);
        atomicAdd(&g_exp[3], (unsigned long long)(__builtin_readcyclecounter() - t0));
        return m;
#endif
        return rl.dfa == GM_NONE || dfa_run_bytes(t, rl.dfa, u, ulen);
    };
#ifdef GM_EXP_COUNT
    atomicAdd(&g_exp[0], 1ull);
#endif
    uint32_t lo = 0, ai = 0;
    for (;;) {
        uint32_t c[RK_K];
#pragma unroll
        for (int j = 0; j < RK_K; j++) c[j] = GM_NONE;
        uint32_t w = 0;
        for (uint32_t i = 0; i < ulen; i++) {
            w = (w >> 8) | ((uint32_t)u[i] << 24);
            if (i < 3) continue;
            const uint32_t key = fold4(w);
            const uint32_t kh = rk_hash(key, sid), bb = rk_bloom_bit(kh);
            if (rkb && !((rkb[bb >> 5] >> (bb & 31)) & 1u)) continue;   // LDS bit filter (k_route<, true>)
            for (uint32_t b = kh & t.rk_mask;; b = (b + 1) & t.rk_mask) {
                const DRlocKey e = t.rk[b];
                if (e.key == 0) break;
                if (e.key != key || e.server != sid) continue;
                for (uint32_t q = 0; q < e.count; q++) {
                    const DRlocEnt E = t.rk_ents[e.first + q];
                    const uint32_t k = E.k;
                    if (k < lo) continue;
                    if (k >= c[RK_K - 1]) break;   // ascending lists
                    // the whole folded factor at the window (a superset check: the DFA decides)
                    const int st = (int)i - 3 - (int)E.key_off;
                    if (st < 0 || (uint32_t)st + E.fac_len > ulen) continue;
                    bool fok = true;
                    for (uint32_t j = 0; j < E.fac_len && fok; j++) fok = (u[st + j] | 0x20u) == t.bytes[E.fac_off + j];
                    if (!fok) continue;
                    bool dup = false;
#pragma unroll
                    for (int j = 0; j < RK_K; j++) dup |= c[j] == k;
                    if (dup) continue;
                    c[RK_K - 1] = k;
#pragma unroll
                    for (int j = RK_K - 1; j > 0; j--)
                        if (c[j] < c[j - 1]) { const uint32_t x = c[j]; c[j] = c[j - 1]; c[j - 1] = x; }
                }
                break;
            }
        }
#pragma unroll
        for (int j = 0; j < RK_K; j++) {
            const uint32_t k = c[j];
            while (ai < S.n_ralw) {
                const uint32_t a = t.rk_ids[S.first_ralw + ai];
                if (a >= k) break;
                ai++;
                if (run(a)) return (int32_t)t.rlocs[S.first_rloc + a].loc;
            }
            if (k == GM_NONE) return -1;
            if (run(k)) return (int32_t)t.rlocs[S.first_rloc + k].loc;
        }
        lo = c[RK_K - 1] + 1;
    }
}

// The regex-location step of ngx_http_core_find_location: the first regex location in config
// order whose DFA matches the URI (-1: none).  Out of line, like the other rarely taken steps.
__device__ __noinline__ int32_t rloc_first_match(const GTab &t, const DServer &S, uint32_t sid, const uint8_t *u,
                                                 uint32_t ulen, const uint32_t *rkb) {
#ifdef GM_EXP_COUNT
    if (S.rk_on) {
        const uint64_t t0 = __builtin_readcyclecounter();
        const int32_t r = rloc_prefiltered(t, S, sid, u, ulen, rkb);
        atomicAdd(&g_exp[4], (unsigned long long)(__builtin_readcyclecounter() - t0));
        return r;
    }
#endif
    if (S.rk_on) return rloc_prefiltered(t, S, sid, u, ulen, rkb);
    for (uint32_t k = 0; k < S.n_rloc; k++) {
        const DRegexLoc rl = t.rlocs[S.first_rloc + k];
        if (rl.dfa == GM_NONE || dfa_run_bytes(t, rl.dfa, u, ulen)) return (int32_t)rl.loc;
    }
    return -1;
}

__device__ uint32_t murmur2_val(const Val &v, uint8_t *buf, bool &ok) {
    // gather to a contiguous lane-private buffer (values here are <= 64 bytes: $request_id)
    uint32_t n = v.total;
    if (n > 64) { ok = false; return 0; }
    uint32_t k = 0;
    for (int s = 0; s < v.cnt; s++) for (uint32_t i = 0; i < v.n[s]; i++) buf[k++] = v.p[s][i];
    uint32_t h = n, len = n;
    const uint8_t *d = buf;
    while (len >= 4) {
        uint32_t x = d[0] | (d[1] << 8) | (d[2] << 16) | ((uint32_t)d[3] << 24);
        x *= 0x5bd1e995u; x ^= x >> 24; x *= 0x5bd1e995u;
        h *= 0x5bd1e995u; h ^= x;
        d += 4; len -= 4;
    }
    switch (len) {
    case 3: h ^= d[2] << 16; [[fallthrough]];
    case 2: h ^= d[1] << 8; [[fallthrough]];
    case 1: h ^= d[0]; h *= 0x5bd1e995u;
    }
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    ok = true;
    return h;
}

// ngx_http_validate_host; returns normalised length or -1
__device__ int validate_host(const uint8_t *h, uint32_t n) {
    int dot_pos = (int)n, host_len = (int)n, state = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t ch = h[i];
        if (ch == '.') { if (dot_pos == (int)i - 1) return -1; dot_pos = (int)i; }
        else if (ch == ':') { if (state == 0) { host_len = (int)i; state = 2; } }
        else if (ch == '[') { if (i == 0) state = 1; }
        else if (ch == ']') { if (state == 1) { host_len = (int)i + 1; state = 2; } }
        else if (ch == 0 || ch == '/') return -1;
    }
    if (dot_pos == host_len - 1) host_len--;
    return host_len <= 0 ? -1 : host_len;
}

__device__ uint32_t name_probe(const DName *tab, uint32_t mask, const uint8_t *bytes, const uint8_t *h,
                               uint32_t off, uint32_t len, uint32_t port_idx) {
    uint32_t hs = name_hash_init(len);
    for (uint32_t i = 0; i < len; i += 4) {
        uint32_t w = 0;
        for (uint32_t q = 0; q < 4 && i + q < len; q++) w |= lc(h[off + i + q]) << (8 * q);
        hs = name_hash_word(hs, w);
    }
    hs = name_hash_fin(hs, port_idx);
    for (uint32_t i = hs & mask;; i = (i + 1) & mask) {
        const DName e = tab[i];
        if (e.hash == 0) return GM_NONE;
        if (e.hash == hs && e.port_idx == port_idx && e.name_len == len) {
            bool ok = true;
            for (uint32_t k = 0; ok && k < len; k++) if (lc(h[off + k]) != bytes[e.name_off + k]) ok = false;
            if (ok) return e.server;
        }
    }
}

__device__ __forceinline__ bool is_redirect(uint32_t code) {
    return code == 301 || code == 302 || code == 303 || code == 307 || code == 308;
}

struct RouteOut {
    uint32_t server, loc, ups, status;
    uint8_t action, kind, bucket, match;
    uint16_t waf;
    uint16_t slow, pad;  // FAST route_one: the request needs an out-of-line step (the SLOW pass)
    int32_t pend_best;   // a request deferred to the regex-location kernels: its longest prefix match
};

// 32 arena bytes starting at `off` (any alignment) as 8 little-endian dwords, from three aligned
// 16-B loads; blocks starting at or beyond `lim` are not read (zero).  Callers mask by length.
// w = the 32 bytes from byte r (0..15) of the 48 in d: the dword offset r >> 2 picked with bit
// selects (v_bfi: a per-lane select of registers, where `qd == 0 ? d[k] : ...` compiled to
// branches and scratch), then a byte funnel shift
__device__ __forceinline__ void funnel32(const uint32_t (&d)[12], uint32_t r, uint32_t (&w)[8]) {
    const uint32_t m1 = 0u - ((r >> 2) & 1u), m2 = 0u - ((r >> 3) & 1u);
    uint32_t sdw[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
        const uint32_t a = (d[k + 1] & m1) | (d[k] & ~m1);
        const uint32_t b = (d[k + 3] & m1) | (d[k + 2] & ~m1);
        sdw[k] = (b & m2) | (a & ~m2);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = __builtin_amdgcn_alignbyte(sdw[k + 1], sdw[k], r & 3);
}
__device__ __forceinline__ void load_span32(const uint8_t *A, uint64_t off, uint64_t lim, uint32_t (&w)[8]) {
    const uint64_t a = off & ~15ull;
    uint32_t d[12];
#pragma unroll
    for (int b = 0; b < 3; b++) {
        uint4 q = make_uint4(0, 0, 0, 0);
        if (a + 16 * b < lim) q = *reinterpret_cast<const uint4 *>(A + a + 16 * b);
        d[4 * b] = q.x; d[4 * b + 1] = q.y; d[4 * b + 2] = q.z; d[4 * b + 3] = q.w;
    }
    funnel32(d, (uint32_t)(off & 15), w);
}

// load_span32 restricted to the aligned 16-byte blocks that hold [off, off + nbytes) (nbytes <=
// 32): bytes past them read as 0.  Each skipped block is one random HBM transaction saved.
__device__ __forceinline__ void load_span_n(const uint8_t *A, uint64_t off, uint64_t lim, uint32_t nbytes,
                                            uint32_t (&w)[8]) {
    const uint64_t a = off & ~15ull;
    const uint32_t r = (uint32_t)(off & 15), nb = (r + nbytes + 15) >> 4;
    uint32_t d[12];
#pragma unroll
    for (int b = 0; b < 3; b++) {
        uint4 q = make_uint4(0, 0, 0, 0);
        if ((uint32_t)b < nb && a + 16 * b < lim) q = *reinterpret_cast<const uint4 *>(A + a + 16 * b);
        d[4 * b] = q.x; d[4 * b + 1] = q.y; d[4 * b + 2] = q.z; d[4 * b + 3] = q.w;
    }
    funnel32(d, r, w);
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[8], int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xFF; }

// exact per-byte equality flags of a word against a byte value: bit 8k+7 set iff byte k == c
__device__ __forceinline__ uint32_t byte_eq_flags(uint32_t w, uint32_t c) {
    const uint32_t t = w ^ (c * 0x01010101u);
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
// the four flags of a word as a nibble (bit k = byte k): the multiply gathers bits 7/15/23/31
__device__ __forceinline__ uint32_t flags_nibble(uint32_t f) { return ((f >> 7) * 0x10204080u) >> 28; }

// Host of <= 32 bytes held in registers: validate_host + exact-name probe (the common case).
// Returns the normalised length (-1 = invalid) and the exact-table server (GM_NONE = miss).
// SWAR: per 4-byte word, exact byte-equality flags for '.', ':', '/', NUL, gathered into 32-bit
// position masks; ngx_http_validate_host's rules then follow from the masks (".." = adjacent
// dots; the first ':' ends the host; the last '.' is stripped when it ends the host).  A host
// starting with '[' (IPv6 literal) takes the byte loop.
// The route's hot tables (gm_tables.hpp ROUTE_STAGE_BYTES): the block's LDS copy when they fit,
// else the image.  Kept apart from GTab and passed by value: a modified local copy of the whole
// GTab (~600 B) lived in scratch, and every table pointer the route read was a scratch load.
struct HotTabs {
    const DPort *ports; const DName *names; const DServer *servers; const DServerIf *server_ifs;
    const DSmallLoc *small; const DLoc *locs; const uint8_t *name_bytes;
};
// NOV6: an IPv6 literal returns -2 (the caller's slow path): its byte loop indexes hw by a
// variable, which puts the words in scratch for every request.  NW: the host's words in
// registers, 8 (<= 32 bytes, the route's prefetched window) or 16 (<= 64 bytes, loaded by the
// caller: round 6 -- C2's 38-byte VirtualServer host took the arena-byte path, a load per byte)
template <bool NOV6 = false, int NW = 8>
__device__ __forceinline__ int host_fast(const uint32_t (&hw)[NW], uint32_t n, const GTab &t, const HotTabs &h,
                                         uint32_t pi, uint32_t &server) {
    static_assert(NW == 8 || NW == 16, "host words");
    using M = typename std::conditional<NW == 8, uint32_t, uint64_t>::type;
    server = GM_NONE;
    int host_len;
    if ((NOV6 || NW != 8) && (hw[0] & 0xFF) == '[') return -2;
    if (!NOV6 && NW == 8 && (hw[0] & 0xFF) == '[') {
        int dot_pos = (int)n, state = 0;
        bool bad = false;
        host_len = (int)n;
        for (int i = 0; i < (int)n; i++) {
            const uint32_t ch = (hw[(i >> 2) & (NW - 1)] >> (8 * (i & 3))) & 0xFF;
            if (ch == '.') { bad |= dot_pos == i - 1; dot_pos = i; }
            else if (ch == ':') { if (state == 0) { host_len = i; state = 2; } }
            else if (ch == '[') { if (i == 0) state = 1; }
            else if (ch == ']') { if (state == 1) { host_len = i + 1; state = 2; } }
            else if (ch == 0 || ch == '/') bad = true;
        }
        if (dot_pos == host_len - 1) host_len--;
        if (bad || host_len <= 0) return -1;
    } else {
        M dots = 0, colons = 0;
        uint32_t badm = 0;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const int rem = (int)n - 4 * k;
            const uint32_t lm = rem >= 4 ? 0xFFFFFFFFu : rem > 0 ? (1u << (8 * rem)) - 1 : 0u;
            const uint32_t w = hw[k];
            dots |= (M)flags_nibble(byte_eq_flags(w, '.') & lm) << (4 * k);
            colons |= (M)flags_nibble(byte_eq_flags(w, ':') & lm) << (4 * k);
            badm |= (byte_eq_flags(w, '/') | byte_eq_flags(w, 0)) & lm;
        }
        if (badm || (dots & (dots >> 1))) return -1;
        host_len = colons ? (NW == 8 ? __builtin_ctz((uint32_t)colons) : __builtin_ctzll((uint64_t)colons)) : (int)n;
        if (dots && (NW == 8 ? 31 - __builtin_clz((uint32_t)dots) : 63 - __builtin_clzll((uint64_t)dots)) == host_len - 1)
            host_len--;
        if (host_len <= 0) return -1;
    }
    uint32_t hs = name_hash_init((uint32_t)host_len);
#pragma unroll
    for (int k = 0; k < NW; k++) {
        const int rem = host_len - 4 * k;
        if (rem <= 0) break;
        const uint32_t m = rem >= 4 ? 0xFFFFFFFFu : (1u << (8 * rem)) - 1;
        hs = name_hash_word(hs, lower4(hw[k]) & m);
    }
    hs = name_hash_fin(hs, pi);
    for (uint32_t i = hs & t.names_mask;; i = (i + 1) & t.names_mask) {
        const DName e = h.names[i];
        if (e.hash == 0) break;
        if (e.hash == hs && e.port_idx == pi && e.name_len == (uint32_t)host_len) {
            uint32_t diff = 0;
#pragma unroll
            for (int hlf = 0; hlf < NW / 8; hlf++) {
                uint32_t tw[8];
                load_span32(h.name_bytes, e.name_off + 32 * hlf, ~0ull, tw);   // the name strings end with 64 B of slack
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const int rem = host_len - 4 * (k + 8 * hlf);
                    const uint32_t m = rem >= 4 ? 0xFFFFFFFFu : rem > 0 ? (1u << (8 * rem)) - 1 : 0u;
                    diff |= (lower4(hw[k + 8 * hlf]) ^ tw[k]) & m;
                }
            }
            if (diff == 0) { server = e.server; break; }
        }
    }
    return host_len;
}

// Wildcard names (*.x / .x, then x.*) for a host that missed the exact table; byte-wise over
// the arena (rare path).
template <bool INL = false>
__device__ __forceinline__ uint32_t host_wildcards_body(const uint8_t *h, int hl, const GTab &t, uint32_t pi) {
    uint32_t s = GM_NONE;
    uint32_t w = name_probe(t.wild_head, t.wild_head_mask, t.name_bytes, h, 0, (uint32_t)hl, pi);
    if (w != GM_NONE && (w & 0x80000000u)) s = w & 0x7FFFFFFFu;      // ".x" matches x itself
    for (int d = 0; s == GM_NONE && d < hl; d++)
        if (h[d] == '.') {
            w = name_probe(t.wild_head, t.wild_head_mask, t.name_bytes, h, d + 1, (uint32_t)(hl - d - 1), pi);
            if (w != GM_NONE) s = w & 0x7FFFFFFFu;
        }
    for (int d = hl - 2; s == GM_NONE && d > 0; d--)
        if (h[d] == '.') s = name_probe(t.wild_tail, t.wild_tail_mask, t.name_bytes, h, 0, (uint32_t)d, pi);
    return s;
}
__device__ __noinline__ uint32_t host_wildcards(const uint8_t *h, int hl, const GTab &t, uint32_t pi) {
    return host_wildcards_body(h, hl, t, pi);
}

// Generic (variable-reading) steps live in non-inlined functions so that the Ctx / Val
// lane-private arrays only exist on these paths (scratch), never on the host/URI fast path.
// server rewrite `if` on a request variable: 1 hit, 0 miss
// (-1: the variable's value is unknown to the engine -- the request defers)
__device__ __noinline__ int server_if_generic(const uint8_t *A, const gm_req *rp, const GTab &t, uint32_t if_idx,
                                             uint32_t rip) {
    const Rec r = load_rec(rp);
    const DServerIf f = t.server_ifs[if_idx];
    Ctx c;
    ctx_init(c, A, r, &t, rip);
    Val v;
    get_var(c, t, f.src, v);
    if (v.unknown) return -1;
    if (f.op == SIF_EQ) return val_eq(v, t.bytes + f.val_off, f.val_len, false);
    if (f.op == SIF_NE) return !val_eq(v, t.bytes + f.val_off, f.val_len, false);
    if (f.op == 4) return v.total && !(v.total == 1 && v.p[0][0] == '0');
    const bool m = dfa_run_val(t, f.val_off, v);
    return f.op == 5 ? m : !m;
}

// rules route (compiled map chains) -> result index (0xFF default; -1 a condition read a value the
// engine cannot know)
template <int NB>
__device__ __noinline__ int rules_generic(const uint8_t *A, const gm_req *rp, const GTab &t, uint32_t rules_idx,
                                          uint32_t rip) {
#ifdef GM_EXP_NO_RULES   // measurement build: no conditions (timing only)
    return 0xFF;
#endif
    const Rec r = load_rec(rp);
    const DRules R = t.rules[rules_idx];
    const uint64_t o_args = r.base + r.uri_len, o_hdrs = o_args + r.args_len;
    // header (one line) / cookie / argument values are single arena spans, looked up once per
    // request (every match of a rules route repeats the route's conditions) and kept in registers;
    // the other variables go through a Val in the lane's private memory, as before (round 6:
    // C2's conditions read headers, cookies and arguments only)
    constexpr int MEMO = 4;
    uint32_t msrc[MEMO], mlen[MEMO];
    uint64_t moff[MEMO];
#pragma unroll
    for (int q = 0; q < MEMO; q++) { msrc[q] = GM_NONE; mlen[q] = 0; moff[q] = 0; }
    Ctx c;
    bool have_ctx = false;
    Val v;
    uint32_t bits = 0;
    bool walked = false;   // the route's header / cookie sources were resolved by one walk
    for (uint32_t ch = 0; ch < R.n_chains; ch++) {
        int32_t nd = (int32_t)t.chain_heads[R.first_chain + ch];
        int guard = 0;
        while (nd >= 0 && guard++ < 64) {
            const DCond cd = t.conds[nd];
            const DSrc sr = t.srcs[cd.src];
            bool m;
            if (sr.kind != SRC_VAR && !(sr.kind == SRC_HTTP && sr.join)) {
                uint64_t off = 0;
                uint32_t len = 0;
                bool hit = false;
#pragma unroll
                for (int q = 0; q < MEMO; q++) if (msrc[q] == cd.src) { off = moff[q]; len = mlen[q]; hit = true; }
                if (!hit && !walked && (sr.kind == SRC_HTTP || sr.kind == SRC_COOKIE)) {
                    // one header walk for every header (one line) and cookie source on the
                    // route's chains (their true paths; up to the free memo slots): C2's
                    // /backends route read X-Version and the Cookie lines in two walks
                    walked = true;
                    uint32_t ps[MEMO], pk[MEMO], pl[MEMO];
                    const uint8_t *pn[MEMO];
                    bool pf[MEMO];
                    uint64_t po[MEMO];
                    uint32_t pv[MEMO];
                    uint32_t np = 0;
#pragma unroll
                    for (int q = 0; q < MEMO; q++) { ps[q] = GM_NONE; pk[q] = 0; pl[q] = 0; pn[q] = nullptr; pf[q] = false; po[q] = 0; pv[q] = 0; }
                    uint32_t nfree = 0;
#pragma unroll
                    for (int q = 0; q < MEMO; q++) nfree += msrc[q] == GM_NONE ? 1u : 0u;
                    for (uint32_t c2 = 0; c2 < R.n_chains && np < nfree; c2++) {
                        int32_t n2 = (int32_t)t.chain_heads[R.first_chain + c2];
                        for (int g2 = 0; n2 >= 0 && g2 < 64 && np < nfree; g2++) {
                            const DCond d2 = t.conds[n2];
                            const DSrc s2 = t.srcs[d2.src];
                            if ((s2.kind == SRC_HTTP && !s2.join) || s2.kind == SRC_COOKIE) {
                                bool dup = false;
#pragma unroll
                                for (int q = 0; q < MEMO; q++) dup |= msrc[q] == d2.src || ps[q] == d2.src;
                                if (!dup) {
                                    bool put = false;
#pragma unroll
                                    for (int q = 0; q < MEMO; q++)
                                        if (!put && q == (int)np) {
                                            ps[q] = d2.src; pk[q] = s2.kind; pl[q] = s2.name_len; pn[q] = t.bytes + s2.name_off;
                                            put = true;
                                        }
                                    np++;
                                }
                            }
                            n2 = d2.next_true;
                        }
                    }
                    // line by line, LF first: a wanted name (a $http_ / $cookie_ suffix: no ':')
                    // of length L names the line iff its first ':' is at st + L, so the ':' probes
                    // at st + L go out beside the LF search instead of a ':' search before it
                    // (hdr_next_name's semantics; one dependent search per line instead of two)
                    uint32_t left = np;
                    const uint64_t he = o_hdrs + r.hdr_len;
                    const uint8_t cookie[7] = "cookie";
                    for (uint64_t st = o_hdrs; left && st < he;) {
                        const bool ck = st + 6 < he && A[st + 6] == ':';
                        bool cq[MEMO];
#pragma unroll
                        for (int q = 0; q < MEMO; q++)
                            cq[q] = !pf[q] && ps[q] != GM_NONE && pk[q] == SRC_HTTP && st + pl[q] < he && A[st + pl[q]] == ':';
                        const uint64_t e = find_byte<NB>(A, st, he, '\n');
                        const bool is_ck = ck && st + 6 < e && hdr_name_is(A, st, 6, cookie, 6);
                        uint64_t lvs = 0;
                        uint32_t lvl = 0;
                        if (is_ck) hdr_value(A, st, st + 6, e, lvs, lvl);
#pragma unroll
                        for (int q = 0; q < MEMO; q++) {
                            if (pf[q] || ps[q] == GM_NONE) continue;
                            if (pk[q] == SRC_HTTP) {
                                if (cq[q] && st + pl[q] < e && hdr_name_is(A, st, pl[q], pn[q], pl[q])) {
                                    hdr_value(A, st, st + pl[q], e, po[q], pv[q]); pf[q] = true; left--;
                                }
                            } else if (is_ck && cookie_in_line(A, lvs, lvl, pn[q], pl[q], po[q], pv[q])) {
                                pf[q] = true; left--;
                            }
                        }
                        st = e + 1;
                    }
                    // into the memo (not found: the empty value)
#pragma unroll
                    for (int q = 0; q < MEMO; q++) {
                        if (ps[q] == GM_NONE) continue;
                        bool put = false;
#pragma unroll
                        for (int q2 = 0; q2 < MEMO; q2++)
                            if (!put && msrc[q2] == GM_NONE) {
                                msrc[q2] = ps[q]; moff[q2] = pf[q] ? po[q] : 0; mlen[q2] = pf[q] ? pv[q] : 0; put = true;
                            }
                        if (ps[q] == cd.src) { off = pf[q] ? po[q] : 0; len = pf[q] ? pv[q] : 0; hit = true; }
                    }
                }
                if (!hit) {
                    const uint8_t *nm = t.bytes + sr.name_off;
                    bool f;
#ifdef GM_EXP_RULES_NOSPAN   // measurement build: every header / cookie / argument empty (timing only)
                    if (true) f = false; else
#endif
                    if (sr.kind == SRC_HTTP) f = span_http<NB>(A, o_hdrs, r.hdr_len, nm, sr.name_len, off, len);
                    else if (sr.kind == SRC_COOKIE) f = span_cookie<NB>(A, o_hdrs, r.hdr_len, nm, sr.name_len, off, len);
                    else f = span_arg(A, o_args, r.args_len, nm, sr.name_len, off, len);
                    if (!f) { off = 0; len = 0; }
                    bool put = false;
#pragma unroll
                    for (int q = 0; q < MEMO; q++)
                        if (!put && msrc[q] == GM_NONE) { msrc[q] = cd.src; moff[q] = off; mlen[q] = len; put = true; }
                }
                if (cd.is_regex) {
                    m = len > 0 && dfa_run_bytes(t, cd.dfa, A + off, len);
                } else {
                    m = len == cd.key_len;
                    const uint8_t *key = t.bytes + cd.key_off;
                    for (uint32_t k = 0; m && k < len; k++) m = lc(A[off + k]) == key[k];
                }
            } else {
#ifdef GM_EXP_RULES_NOVAR   // measurement build: every other variable empty (timing only)
                v.clear();
#else
                if (!have_ctx) { ctx_init(c, A, r, &t, rip); have_ctx = true; }
                get_var(c, t, cd.src, v);
#endif
                if (v.unknown) return -1;
                if (cd.is_regex) m = v.total > 0 && dfa_run_val(t, cd.dfa, v);
                else m = val_eq(v, t.bytes + cd.key_off, cd.key_len, true);
            }
            nd = m ? cd.next_true : cd.next_false;
        }
        if (nd == NEXT_1) bits |= 1u << ch;
    }
    if (R.table_off != GM_NONE) return t.rtab[R.table_off + bits];
    // more chains than a truth table holds: ngx_http_map_find over the '0'/'1' string -- the
    // exact keys first, then the regexes in config order
    uint8_t sb[RULES_CHAINS_MAX];
    for (uint32_t ch = 0; ch < R.n_chains; ch++) sb[ch] = (bits >> ch) & 1u ? '1' : '0';
    Val sv;
    sv.clear();
    sv.add(sb, R.n_chains);
    for (uint32_t k = 0; k < R.n_targets; k++) {
        const DCond cd = t.conds[R.pad[0] + k];
        if (!cd.is_regex && val_eq(sv, t.bytes + cd.key_off, cd.key_len, false)) return (int)k;
    }
    for (uint32_t k = 0; k < R.n_targets; k++) {
        const DCond cd = t.conds[R.pad[0] + k];
        if (cd.is_regex && dfa_run_val(t, cd.dfa, sv)) return (int)k;
    }
    return 0xFF;
}

// split_clients: murmur2 of the source -> part index (0xFF none, 0xFFFFFFFF unsupported value)
__device__ __noinline__ uint32_t split_generic(const uint8_t *A, const gm_req *rp, const GTab &t, uint32_t split_idx,
                                               uint32_t rip) {
#ifdef GM_EXP_NO_SPLIT   // measurement build: no split key (timing only)
    return 0;
#endif
    const Rec r = load_rec(rp);
    const DSplit Sp = t.splits[split_idx];
    Ctx c;
    ctx_init(c, A, r, &t, rip);
    Val v;
    get_var(c, t, Sp.src, v);
    if (v.unknown) return 0xFFFFFFFFu;
    uint8_t buf[64];
    bool ok;
    const uint32_t hsh = murmur2_val(v, buf, ok);
    if (!ok) return 0xFFFFFFFFu;
    for (uint32_t k = 0; k < Sp.n_parts; k++) {
        const DPart pt = t.parts[Sp.first_part + k];
        if (hsh < pt.bound || pt.star) return k;
    }
    return 0xFFu;
}

// The first 32 bytes of a request's Host and URI, both loaded as soon as its record is known (two
// independent HBM loads instead of host, then the server's tables, then the URI).  (Loading them
// one request ahead was measured slower: a wave's loads complete in order, so the prefetch made
// every table lookup of the current request wait for the next request's HBM loads.)
struct RoutePre { uint32_t hw[8], uw[8]; };
__device__ __forceinline__ void route_prefetch(const uint8_t *A, uint64_t alen, const Rec &r, RoutePre &p) {
    const uint64_t f_uri = r.base, f_host = r.base + r.uri_len + r.args_len + r.hdr_len + r.body_len;
    // (measured: loading all three blocks of both spans unconditionally, so that the compiler
    // issues the six loads together, made the route slower -- 1.10 vs 0.85 ms per 10M C4 requests
    // alone: the extra blocks are extra HBM lines)
    load_span_n(A, f_host, alen, min(r.host_len, 32u), p.hw);
    load_span_n(A, f_uri, alen, min(r.uri_len, 32u), p.uw);
}

// k_rloc's tile shape: URIs up to RLOC_URI_CAP bytes staged in LDS, candidate bitmaps of
// RLOC_BM_BITS regex locations (longer URIs / larger servers run rloc_prefiltered in the lane)
constexpr uint32_t RLOC_URI_CAP = 256, RLOC_BM_BITS = 2048;
constexpr uint32_t RLOC_STATUS_WORD = 16;   // batch status word: requests deferred to k_rloc
constexpr uint32_t SLOW_STATUS_WORD = 17;   // batch status word: requests for k_route's SLOW pass
// rk_in: RK_INLINE -- a prefiltered regex step runs here; RK_DEFER -- one that k_rloc can take
// (URI <= RLOC_URI_CAP, n_rloc <= RLOC_BM_BITS) sets *pend and returns; >= -1 -- k_rloc's answer
// (the location index, -1 none).  *sid_out: the server chosen (valid whenever *pend is set).
constexpr int32_t RK_INLINE = -3, RK_DEFER = -2;
template <bool FAST = false, bool LONGHOST = true>
__device__ __forceinline__ void route_loc(const uint8_t *A, const gm_req *rp, const GTab &t, const HotTabs h, int32_t loc,
                          RouteOut &o);
// the request's body length and whether it is chunked, re-read from its record where the 413
// check needs them (kept in registers across the location walk they cost the route spills)
__device__ __forceinline__ uint32_t req_body_len(const gm_req *rp) { return reinterpret_cast<const uint32_t *>(rp)[5]; }
__device__ __forceinline__ bool req_chunked(const gm_req *rp) { return reinterpret_cast<const uint32_t *>(rp)[9] & GM_REQ_CHUNKED; }
template <bool FAST, bool LONGHOST>
__device__ __forceinline__ void route_locphase(const uint8_t *A, const gm_req *rp, const Rec &r, const RoutePre &pre,
                                               const GTab &t, const HotTabs h, RouteOut &o, const uint32_t *rkb,
                                               int32_t rk_in, bool *pend, const DServer &S, uint32_t sid);
// client_max_body_size exceeded: 413, nothing proxied, no WAF phase
__device__ __forceinline__ void too_large(RouteOut &o) {
    o.action = GM_ACT_TOO_LARGE; o.status = 413; o.ups = GM_NONE; o.waf = GM_WAF_OFF;
}
// FAST: no out-of-line call at all.  A call anywhere in the step made the compiler keep the
// step's values (the record, the host / URI words, addresses) in scratch around it -- stored and
// reloaded for every request, whether it calls or not: the route took 1.05 ms alone per 10M C4
// requests with the calls in the kernel, 0.63 with none.  The wildcard step is inlined, an IPv6
// literal host takes the arena-byte path; a request that needs a generic server `if`, the
// regex-location prefilter or a rules / split route stops with o.slow set, and k_route's SLOW
// pass (a second launch over the list of such requests) routes it again with the calls.
// LONGHOST: hosts of 33..64 bytes through the 16-word SWAR path, and rules_generic's header walks
// searching 32 bytes a step (the route kernels beside the WAF scan, held to GM_ROUTE_WPE waves,
// leave both out: they spilled them / cost them a wave)
template <bool FAST = false, bool LONGHOST = true>
__device__ __forceinline__ void route_one(const uint8_t *A, uint64_t alen, const gm_req *rp, const Rec &r, const RoutePre &pre,
                          const GTab &t, const HotTabs h, RouteOut &o, const uint32_t *rkb, int32_t rk_in = RK_INLINE,
                          bool *pend = nullptr) {
    o.server = GM_NONE; o.loc = GM_NONE; o.ups = GM_NONE; o.status = 0;
    o.action = GM_ACT_NO_LISTENER; o.kind = GM_ROUTE_NONE; o.bucket = 0xFF; o.match = 0xFF; o.waf = GM_WAF_OFF;
    o.slow = 0;
    o.pend_best = -1;
    const uint64_t f_uri = r.base, f_host = r.base + r.uri_len + r.args_len + r.hdr_len + r.body_len;
    // ---- listen port
    uint32_t pi = GM_NONE;
    for (uint32_t i = 0; i < t.n_ports; i++) if (h.ports[i].port == r.port) { pi = i; break; }
    if (pi == GM_NONE) return;
    const DPort P = h.ports[pi];
    const bool https = r.flags & GM_REQ_HTTPS;
    if (https && !P.ssl) return;
    uint32_t sid = P.default_server;
    if (r.flags & GM_REQ_INVALID) {   // rejected by the wire parser: its status, from the port's default server
        o.server = sid; o.action = GM_ACT_BAD_REQUEST; o.status = r.bad_status;
        return;
    }
    // ---- host -> server (exact > *.x/.x > x.*)
    bool bad = false;
    if (r.host_len) {
        uint32_t s = GM_NONE;
        int hl;
        if (r.host_len <= 32) {
            hl = host_fast<FAST>(pre.hw, r.host_len, t, h, pi, s);
            if (FAST && hl == -2) {   // an IPv6 literal: the arena-byte path
                hl = validate_host(A + f_host, r.host_len);
                if (hl >= 0) s = name_probe(h.names, t.names_mask, h.name_bytes, A + f_host, 0, (uint32_t)hl, pi);
            }
        } else if (LONGHOST && r.host_len <= 64) {   // 33..64 bytes: the same SWAR over 16 words
            uint32_t hw16[16], lo[8], hi[8];
            load_span_n(A, f_host, alen, 32, lo);
            load_span_n(A, f_host + 32, alen, r.host_len - 32, hi);
#pragma unroll
            for (int k = 0; k < 8; k++) { hw16[k] = lo[k]; hw16[8 + k] = hi[k]; }
            hl = host_fast<true, 16>(hw16, r.host_len, t, h, pi, s);
            if (hl == -2) {   // an IPv6 literal: the arena-byte path
                hl = validate_host(A + f_host, r.host_len);
                if (hl >= 0) s = name_probe(h.names, t.names_mask, h.name_bytes, A + f_host, 0, (uint32_t)hl, pi);
            }
        } else {
            hl = validate_host(A + f_host, r.host_len);
            if (hl >= 0) s = name_probe(h.names, t.names_mask, h.name_bytes, A + f_host, 0, (uint32_t)hl, pi);
        }
        if (hl < 0) bad = true;
        else {
            if (s == GM_NONE && t.n_wild) {   // (no wildcard names: the port's default server)
                if (FAST) s = host_wildcards_body<true>(A + f_host, hl, t, pi);
                else s = host_wildcards(A + f_host, hl, *t.self, pi);
            }
            if (s != GM_NONE) sid = s;
        }
    }
    o.server = sid;
    if (bad || (P.ssl && !https)) { o.action = GM_ACT_BAD_REQUEST; o.status = 400; return; }
    const DServer S = h.servers[sid];
    // ---- server rewrite phase
    for (uint32_t i = 0; i < S.n_if; i++) {
        const DServerIf f = h.server_ifs[S.first_if + i];
        bool hit;
        if (f.op == SIF_RETURN) hit = true;
        else if (f.op == SIF_FLAGS) hit = (f.tt >> (r.flags & 3)) & 1u;
        else if (f.op == 0xFF) { o.action = GM_ACT_UNSUPPORTED; o.status = 0; return; }
        else {
            if (FAST) { o.slow = 1; return; }
            const int g = server_if_generic(A, rp, *t.self, S.first_if + i, S.realip);
            if (g < 0) { o.action = GM_ACT_UNSUPPORTED; o.status = 0; return; }
            hit = g != 0;
        }
        if (hit) { o.action = is_redirect(f.code) ? GM_ACT_REDIRECT : GM_ACT_RETURN; o.status = f.code; return; }
    }
    route_locphase<FAST, LONGHOST>(A, rp, r, pre, t, h, o, rkb, rk_in, pend, S, sid);
}

// route_one's location phase: trie walk (exact, longest prefix, auto_redirect), then regex
// locations, then route_loc.  The first 32 URI bytes come from registers (a window shifted one
// dword per 4 bytes).
template <bool FAST, bool LONGHOST>
__device__ __forceinline__ void route_locphase(const uint8_t *A, const gm_req *rp, const Rec &r, const RoutePre &pre,
                                               const GTab &t, const HotTabs h, RouteOut &o, const uint32_t *rkb,
                                               int32_t rk_in, bool *pend, const DServer &S, uint32_t sid) {
    const uint64_t f_uri = r.base;
    const uint8_t *u = A + f_uri;
    uint32_t uw[8];
#pragma unroll
    for (int k = 0; k < 8; k++) uw[k] = pre.uw[k];
    int32_t best = -1, fexact = -1, far = -1;
    bool full = false;   // a location-trie node spells the whole URI
    if (S.sl_n) {
        // small server: compare the URI's first 16 bytes with every location-carrying node
        uint32_t bestlen = 0;
        for (uint32_t j = 0; j < S.sl_n; j++) {
            const DSmallLoc E = h.small[S.sl_first + j];
            if (E.len > r.uri_len) continue;
            uint32_t diff = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int rem = (int)E.len - 4 * k;
                const uint32_t m = rem >= 4 ? 0xFFFFFFFFu : rem > 0 ? (1u << (8 * rem)) - 1 : 0u;
                diff |= (uw[k] ^ E.path[k]) & m;
            }
            if (diff) continue;
            if (E.len == r.uri_len) { full = true; fexact = E.exact_loc; far = E.ar_loc; }
            if (E.prefix_loc >= 0 && (best < 0 || E.len > bestlen)) { best = E.prefix_loc; bestlen = E.len; }
        }
    } else {
        uint32_t node = S.trie_root;
        best = t.nodes[node].prefix_loc;
        uint32_t i = 0;
        for (;; i++) {
            if (i == r.uri_len) break;
            uint32_t b;
            if (i < 32) {
                b = uw[0] & 0xFF;
                uw[0] >>= 8;
                if ((i & 3) == 3) {
    #pragma unroll
                    for (int k = 0; k < 7; k++) uw[k] = uw[k + 1];
                    uw[7] = 0;
                }
            } else {
                b = u[i];
            }
            const uint32_t key = node * 256u + b + 1u;
            uint32_t slot = edge_hash(key) & t.edges_mask, child = GM_NONE;
            int32_t cpref = -1;
            for (;; slot = (slot + 1) & t.edges_mask) {
                const DEdge e = t.edges[slot];
                if (e.key == 0) break;
                if (e.key == key) { child = e.child; cpref = e.child_prefix; break; }
            }
            if (child == GM_NONE) break;
            node = child;
            if (cpref >= 0) best = cpref;
        }
        if (i == r.uri_len) {
            const DNode nd = t.nodes[node];
            full = true; fexact = nd.exact_loc; far = nd.ar_loc;
        }
    }
    int32_t loc = -1;
    if (full) {
        if (fexact >= 0) loc = fexact;
        else if (far >= 0) {
            // (the location found is the redirect's target: its client_max_body_size is checked
            // before the redirect, ngx_http_core_find_config_phase)
            o.loc = (uint32_t)far;
            if (!req_chunked(rp) && req_body_len(rp) > h.locs[far].body_max) too_large(o);
            else { o.action = GM_ACT_AUTO_301; o.status = 301; }
            return;
        }
    }
    if (loc < 0) {
        if (best >= 0 && h.locs[best].noregex) loc = best;
        else {
            if (S.rk_on && rk_in >= -1) loc = rk_in;
            else if (S.rk_on && rk_in == RK_DEFER &&
                     (S.rsl_n || (r.uri_len <= RLOC_URI_CAP && S.n_rloc <= RLOC_BM_BITS))) {
                *pend = true;
                o.pend_best = best;
                return;
            } else if (FAST) {   // (a server without regex locations: none matches)
                if (S.rk_on || S.n_rloc) { o.slow = 1; return; }
            } else loc = rloc_first_match(*t.self, S, sid, u, r.uri_len, rkb);
            if (loc < 0) loc = best;
        }
    }
    route_loc<FAST, LONGHOST>(A, rp, t, h, loc, o);
}

// The rest of route_one once the location is known (loc < 0: none): location kinds, rules and
// split routes, return / proxy.  The regex-location tail pass starts here with k_rloc's answer
// (or the request's longest prefix match) instead of routing the request again.
// client_max_body_size: a Content-Length body is checked against the location found (the
// server's limit when none) before that location's rewrite phase (ngx_http_core_find_config_phase);
// a chunked body only when it is read -- by the proxying location, the final one after an
// internal redirect (the chunked body filter)
// ngx_http_access_module's handler (nginx 1.17.3, satisfy all) for the address the request's
// connection has after the realip module: 0 allowed (no rule matched, or an allow), 1 denied (403),
// 2 unknown to the engine (realip from a header it cannot read, an unparseable $remote_addr).
// An IPv4 client is tested against the IPv4 list; an IPv6 one that maps an IPv4 address against
// the IPv4 list when there is one (and only it), else against the IPv6 list.
__device__ __noinline__ int access_eval(const uint8_t *A, const gm_req *rp, const GTab &t, uint32_t list, uint32_t rip) {
    const Rec r = load_rec(rp);
    InetAddr a;
    a.fam = 0;
    if (rip != GM_NONE) {
        Ctx c;
        ctx_init(c, A, r, &t, rip);
        if (c.rip_state == RIPS_UNKNOWN) return 2;
        a = c.ra;   // (realip_eval parsed the connection address into it first)
    } else {
        const uint64_t ra = r.base + r.uri_len + r.args_len + r.hdr_len + r.body_len + r.host_len + r.method_len + r.ruri_len;
        a.fam = r.raddr_len <= 45 ? d_parse_addr(A + ra, r.raddr_len, a.b) : 0u;
    }
    if (a.fam == 0) return 2;
    const DAccList L = t.acc_lists[list];
    uint32_t fam = a.fam, first = L.first4, nr = L.n4;
    const uint8_t *b = a.b;
    if (fam == 6) {
        bool mapped = b[10] == 0xFF && b[11] == 0xFF;
        for (int i = 0; i < 10; i++) mapped = mapped && b[i] == 0;
        if (mapped && L.n4) b += 12, fam = 4;
        else { first = L.first6; nr = L.n6; }
    }
    const uint32_t nb = fam == 4 ? 4u : 16u;
    for (uint32_t k = 0; k < nr; k++) {
        const DAccRule R = t.acc_rules[first + k];
        const uint8_t *ad = reinterpret_cast<const uint8_t *>(R.c.addr), *mk = reinterpret_cast<const uint8_t *>(R.c.mask);
        bool hit = true;
        for (uint32_t i = 0; i < nb; i++) hit = hit && (b[i] & mk[i]) == ad[i];
        if (hit) return R.deny ? 1 : 0;
    }
    return 0;
}

template <bool FAST, bool LONGHOST>
__device__ __forceinline__ void route_loc(const uint8_t *A, const gm_req *rp, const GTab &t, const HotTabs h, int32_t loc,
                          RouteOut &o) {
    const uint32_t blen = req_body_len(rp);
    const bool chunked = req_chunked(rp);
    if (loc < 0) {
        if (!chunked && blen > h.servers[o.server].body_max) { too_large(o); return; }
        const uint32_t sa = h.servers[o.server].access;   // (the server block's own conf: its access phase)
        if (sa != GM_NONE) {
            if (FAST) { o.slow = 1; return; }
            const int a = access_eval(A, rp, *t.self, sa, h.servers[o.server].realip);
            if (a == 1) { o.action = GM_ACT_FORBIDDEN; o.status = 403; return; }
            if (a == 2) { o.action = GM_ACT_UNSUPPORTED; return; }
        }
        o.action = GM_ACT_NOT_FOUND; o.status = 404; return;
    }
    o.loc = (uint32_t)loc;
    DLoc L = h.locs[loc];
    if (!chunked && blen > L.body_max) { too_large(o); return; }
    uint32_t fin = (uint32_t)loc;
    // (2: stopped with the server and the location known -- k_route's SLOW pass resumes here)
    if (FAST && (L.kind == LK_IRL_RULES || L.kind == LK_IRL_SPLIT || L.access != GM_NONE)) { o.slow = 2; return; }
    if (L.kind == LK_IRL_RULES) {
        const DRules R = t.rules[L.route];
        const int idx = rules_generic<LONGHOST ? 2 : 1>(A, rp, *t.self, L.route, h.servers[o.server].realip);
        o.kind = GM_ROUTE_RULES;
        if (idx < 0) { o.action = GM_ACT_UNSUPPORTED; return; }
        o.match = (uint8_t)idx;
        fin = idx == 0xFF ? R.default_target : t.rtargets[R.first_target + idx];
    } else if (L.kind == LK_IRL_SPLIT) {
        o.kind = GM_ROUTE_SPLIT;
        const uint32_t k = split_generic(A, rp, *t.self, L.route, h.servers[o.server].realip);
        if (k == 0xFFFFFFFFu) { o.action = GM_ACT_UNSUPPORTED; return; }
        fin = GM_NONE;
        if (k != 0xFFu) { o.bucket = (uint8_t)k; fin = t.parts[t.splits[L.route].first_part + k].target; }
    } else if (L.kind == LK_UNSUPPORTED) {
        o.action = GM_ACT_UNSUPPORTED; return;
    }
    if (L.kind == LK_IRL_RULES || L.kind == LK_IRL_SPLIT) {
        if (fin == GM_NONE) { o.action = GM_ACT_ERRPAGE; o.status = 302; return; }
        L = h.locs[fin];
        if (L.kind != LK_PROXY && L.kind != LK_RETURN && L.kind != LK_NONE && L.kind != LK_STATUS) {
            o.action = GM_ACT_UNSUPPORTED; return;
        }
    }
    // (`return` answers in the rewrite phase, before the access phase)
    if (L.kind == LK_RETURN) { o.action = is_redirect(L.ret_code) ? GM_ACT_REDIRECT : GM_ACT_RETURN; o.status = L.ret_code; return; }
    if (fin == (uint32_t)loc && L.kind == LK_PROXY) o.kind = GM_ROUTE_PLAIN;   // (a 403 / 413 keeps the route)
    if (L.access != GM_NONE) {   // allow / deny (the FAST pass sent such locations here)
        const int a = access_eval(A, rp, *t.self, L.access, h.servers[o.server].realip);
        if (a == 1) { o.action = GM_ACT_FORBIDDEN; o.status = 403; return; }
        if (a == 2) { o.action = GM_ACT_UNSUPPORTED; return; }
    }
    if (L.kind == LK_STATUS) { o.action = GM_ACT_RETURN; o.status = 200; return; }
    if (L.kind != LK_PROXY) { o.action = GM_ACT_NOT_FOUND; o.status = 404; return; }
    if (chunked && blen > L.body_max) { too_large(o); return; }
    o.action = GM_ACT_PROXY; o.status = 0; o.ups = L.upstream; o.waf = L.waf_mode;
}

// the verdict's two 16-byte halves (n_hits and first_hit_off 0: the WAF stages fill them in)
__device__ __forceinline__ void write_verdict(gm_verdict *v, const GTab &t, const RouteOut &o) {
    uint4 w0, w1;
    w0.x = t.gen; w0.y = o.server; w0.z = o.loc; w0.w = o.ups;
    w1.x = (uint32_t)o.action | ((uint32_t)o.kind << 8) | ((uint32_t)o.bucket << 16) | ((uint32_t)o.match << 24);
    w1.y = (uint32_t)o.waf;   // n_hits = 0
    w1.z = 0;                 // first_hit_off
    w1.w = o.status;
    uint4 *dst = reinterpret_cast<uint4 *>(v);
    dst[0] = w0; dst[1] = w1;
}
// ============================================================================ kernels
constexpr int ROUTE_BLOCK = 256;
// register target (waves per SIMD) of the route beside the WAF scan: the scan's workgroup holds
// 4 waves per SIMD, and the route's waves share what registers they leave
#define GM_ROUTE_WPE_SHIPPED 5
#ifndef GM_ROUTE_WPE
#define GM_ROUTE_WPE GM_ROUTE_WPE_SHIPPED
#endif
// k_route's dynamic LDS: the hot route tables it stages (0 when they exceed ROUTE_STAGE_BYTES),
// then the per-block location histogram when the generation's locations fit it -- at most
// LDS_HIST_BESIDE entries beside the WAF scan (2 KiB: a route block fits beside the scan's Bloom
// filter and record stages in the CU's 160 KiB), LDS_HIST_ALONE otherwise (C3's ~1000 regex
// locations counted with one global atomic per request took most of the 3.5 ms tail pass)
constexpr uint32_t LDS_HIST_BESIDE = 512, LDS_HIST_ALONE = 8192;
inline uint32_t route_hot16(const GTab &t) { return (t.hot_len + 15u) & ~15u; }
inline uint32_t route_hist_n(const GTab &t, bool beside) {
    return t.n_locs <= (beside ? LDS_HIST_BESIDE : LDS_HIST_ALONE) ? t.n_locs : 0u;
}
inline uint32_t route_lds(const GTab &t, bool beside) { return route_hot16(t) + 4u * route_hist_n(t, beside); }

// WPE: waves per SIMD the register allocation targets (beside the scan's workgroup, a CU has
// room for route waves only when they are small)
// RK: the generation has prefiltered regex locations -- their step is deferred to k_rloc when
// q.list is set (requests appended to q.list as {index, server}); TAIL: the second pass over
// q.list, finishing each deferred request with k_rloc's location (q.loc).
// st: per deferred request {$uri base (lo, hi), $uri length, server} -- what a union-DFA slice
// pass needs, 16 B instead of the list entry plus the 64-B record (k_rloc_multi reads it once per
// slice, and only for requests the slice can still answer)
// best: the deferred request's longest prefix match (-1 none), where the tail pass starts when no
// regex location matched
// u: its $uri's first 32 bytes (two uint4; the slices' first two 16-byte steps read them instead
// of an arena line each)
struct RlocQ { uint2 *list; uint32_t *count; int32_t *loc; uint4 *st; int32_t *best; uint4 *u; };
// SLOW: the second pass over the requests a FAST pass listed (q.list / q.count): the whole route
// with its out-of-line steps, the verdict and the location counter (blk2rec and the hit counts
// were written by the first pass)
template <int WPE, bool RK = false, bool TAIL = false, bool SLOW = false>
__global__ __launch_bounds__(ROUTE_BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void k_route(const gm_req *__restrict__ reqs, uint32_t n,
                                                       const uint8_t *__restrict__ A, uint64_t arena_len,
                                                       GTab tg, gm_verdict *__restrict__ out,
                                                       unsigned long long *__restrict__ counters,
                                                       uint32_t *__restrict__ blk2rec, uint32_t nblk,
                                                       uint32_t *__restrict__ hcnt, int prio,
                                                       const uint64_t *__restrict__ dlen, uint32_t hist_n,
                                                       RlocQ q = RlocQ{}) {
    if (dlen) arena_len = *dlen;   // gm_batch.arena_len_dev: the length a producer wrote on the device
    // beside the WAF scan: issue priority over the scan's waves, so the route's short
    // latency-bound waves finish early instead of stretching past the scan (GM_ROUTE_PRIO)
    if (prio) __builtin_amdgcn_s_setprio(2);
    // the generation's hot tables in LDS (gm_tables.hpp ROUTE_STAGE_BYTES): every pointer into
    // the hot prefix is rebased onto the block's copy; generic (flat) loads then hit LDS
    // (dynamic LDS, route_lds(): the generation's hot_len rounded up to 16 B, so that a route block
    // beside the WAF scan takes only what this generation's tables need)
    extern __shared__ uint4 hot[];
    const GTab &t = tg;
    HotTabs h{tg.ports, tg.names, tg.servers, tg.server_ifs, tg.small, tg.locs, tg.name_bytes};
    if (tg.hot_len) {
        const uint4 *src = reinterpret_cast<const uint4 *>(tg.hot_base);
        for (uint32_t k = threadIdx.x; k < (tg.hot_len + 15) / 16; k += blockDim.x) hot[k] = src[k];
        const uint8_t *lb = reinterpret_cast<const uint8_t *>(hot);
        auto rb = [&](const void *p) { return lb + (reinterpret_cast<const uint8_t *>(p) - tg.hot_base); };
        h.ports = (const DPort *)rb(tg.ports);
        h.names = (const DName *)rb(tg.names);
        h.servers = (const DServer *)rb(tg.servers);
        h.server_ifs = (const DServerIf *)rb(tg.server_ifs);
        h.small = (const DSmallLoc *)rb(tg.small);
        h.locs = (const DLoc *)rb(tg.locs);
        h.name_bytes = rb(tg.name_bytes);
    }
    // the location histogram after the hot tables (hist_n = route_hist_n(): 0 = global atomics)
    uint32_t *hist = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(hot) + ((tg.hot_len + 15u) & ~15u));
    const bool use_hist = hist_n != 0;
    if (use_hist) for (uint32_t k = threadIdx.x; k < t.n_locs; k += blockDim.x) hist[k] = 0;
    // RK: servers with many regex locations -- the prefilter's key bit filter in LDS
    __shared__ uint32_t rkb[RK ? RK_BLOOM_WORDS : 1];
    if (RK) for (uint32_t k = threadIdx.x; k < RK_BLOOM_WORDS; k += blockDim.x) rkb[k] = t.rk_bloom[k];
    __syncthreads();
    const uint32_t nn = TAIL || SLOW ? *q.count : n;
    const uint32_t stride = gridDim.x * blockDim.x;
    // no out-of-line call in the first pass (the requests that need one go to q.list)
    constexpr bool FASTK = !RK && !TAIL && !SLOW;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < nn; x += stride) {
        uint32_t i = x;
        RouteOut o;
        bool pend = false;
        Rec r{};
        RoutePre pre;
        if (TAIL) {
            // a deferred request: its location is k_rloc's answer, else its longest prefix match
            // (saved by the first pass); only the location's own step runs again
            const uint2 e = q.list[x];
            i = e.x;
            int32_t loc = q.loc[x];
            if (loc < 0) loc = q.best[x];
            o.server = e.y; o.loc = GM_NONE; o.ups = GM_NONE; o.status = 0; o.action = GM_ACT_NO_LISTENER;
            o.kind = GM_ROUTE_NONE; o.bucket = 0xFF; o.match = 0xFF; o.waf = GM_WAF_OFF; o.pend_best = -1; o.slow = 0;
            route_loc<false, (WPE < GM_ROUTE_WPE_SHIPPED)>(A, reqs + i, t, h, loc, o);
        } else {
            uint32_t rsm = 0;
            if (SLOW) { const uint2 e = q.list[x]; i = e.x; rsm = e.y; }
            if (SLOW && rsm) {
                // the first pass stopped in route_loc (a rules / split location, an access list):
                // the server and location it found, only the location's own step again
                o.server = (rsm >> 16) & 0x7FFFu; o.loc = GM_NONE; o.ups = GM_NONE; o.status = 0;
                o.action = GM_ACT_NO_LISTENER; o.kind = GM_ROUTE_NONE; o.bucket = 0xFF; o.match = 0xFF;
                o.waf = GM_WAF_OFF; o.pend_best = -1; o.slow = 0;
                route_loc<false, (WPE < GM_ROUTE_WPE_SHIPPED)>(A, reqs + i, t, h, (int32_t)(rsm & 0xFFFFu), o);
            } else {
                r = load_rec(reqs + i);
                route_prefetch(A, arena_len, r, pre);
                route_one<FASTK, (WPE < GM_ROUTE_WPE_SHIPPED)>(A, arena_len, reqs + i, r, pre, t, h, o, RK ? rkb : nullptr,
                                 RK && q.list ? RK_DEFER : RK_INLINE, &pend);
            }
        }
        const bool slow = FASTK && o.slow;
        if (FASTK) {   // to the SLOW pass, one atomic per wave
            const unsigned long long sm = __ballot(slow);
            if (sm) {
                const uint32_t lane = threadIdx.x & 63;
                const int leader = __ffsll(sm) - 1;
                uint32_t b = 0;
                if (lane == (uint32_t)leader) b = atomicAdd(q.count, (uint32_t)__popcll(sm));
                b = __shfl(b, leader);
                // (server, location) | bit 31 when the SLOW pass can resume at route_loc, else 0
                const uint32_t rsm = o.slow == 2 && o.server < 0x8000u && o.loc < 0x10000u
                                         ? 0x80000000u | (o.server << 16) | o.loc : 0u;
                if (slow) q.list[b + (uint32_t)__popcll(sm & ((1ull << lane) - 1))] = make_uint2(i, rsm);
            }
        }
        const uint32_t cloc = slow ? GM_NONE : o.loc;   // (counted by the SLOW pass)
        if (RK && !TAIL) {   // deferred to k_rloc: appended, one atomic per wave
            const unsigned long long pm = __ballot(pend);
            if (pm) {
                const uint32_t lane = threadIdx.x & 63;
                const int leader = __ffsll(pm) - 1;
                uint32_t b = 0;
                if (lane == (uint32_t)leader) b = atomicAdd(q.count, (uint32_t)__popcll(pm));
                b = __shfl(b, leader);
                if (pend) {
                    const uint32_t slot = b + (uint32_t)__popcll(pm & ((1ull << lane) - 1));
                    q.list[slot] = make_uint2(i, o.server);
                    q.st[slot] = make_uint4((uint32_t)r.base, (uint32_t)(r.base >> 32), r.uri_len, o.server);
                    q.best[slot] = o.pend_best;
                    q.u[2 * slot] = make_uint4(pre.uw[0], pre.uw[1], pre.uw[2], pre.uw[3]);
                    q.u[2 * slot + 1] = make_uint4(pre.uw[4], pre.uw[5], pre.uw[6], pre.uw[7]);
                }
            }
        }
        if (!pend && !slow) write_verdict(out + i, t, o);
        // per-location counter: the wave's first few distinct locations in one atomic each for all
        // their lanes (most waves: one to three locations), any lane left after four rounds its
        // own atomic (C3's ~50 distinct locations per wave took a round each)
        {
            unsigned long long todo = __ballot(cloc != GM_NONE);
            for (int round = 0; todo && round < 4; round++) {
                const int leader = __ffsll(todo) - 1;
                const uint32_t lk = __shfl(cloc, leader);
                const unsigned long long same = __ballot(cloc == lk) & todo;
                if ((threadIdx.x & 63) == (uint32_t)leader) {
                    if (use_hist) atomicAdd(&hist[lk], (uint32_t)__popcll(same));
                    else atomicAdd(&counters[lk], (unsigned long long)__popcll(same));
                }
                todo &= ~same;
            }
            if ((todo >> (threadIdx.x & 63)) & 1ull) {
                if (use_hist) atomicAdd(&hist[cloc], 1u);
                else atomicAdd(&counters[cloc], 1ull);
            }
        }
        if (TAIL || SLOW) continue;
        if (hcnt) {   // the WAF stages' per-request hit counts start the batch at zero
            hcnt[i] = 0;
            if (i + 1 == n) hcnt[n] = 0;
        }
        if (blk2rec) {
            // blocks whose start lies in [base_i, base_{i+1}) belong to record i (base_{i+1}: the
            // next lane's record, which it holds; lane 63 and the last request read it)
            uint64_t b0 = (i == 0) ? 0 : r.base;
            const uint32_t nb_lo = (uint32_t)__shfl_down((int)(uint32_t)r.base, 1);
            const uint32_t nb_hi = (uint32_t)__shfl_down((int)(uint32_t)(r.base >> 32), 1);
            const bool nxt_lane = (threadIdx.x & 63) != 63 && x + 1 < nn;
            uint64_t b1 = (i + 1 < n) ? (nxt_lane ? ((uint64_t)nb_hi << 32 | nb_lo) : reqs[i + 1].base) : arena_len;
            uint64_t k0 = (b0 + (1u << BLK_SHIFT) - 1) >> BLK_SHIFT;
            uint64_t k1 = (b1 + (1u << BLK_SHIFT) - 1) >> BLK_SHIFT;
            if (i + 1 == n) k1 = nblk;
            for (uint64_t k = k0; k < k1 && k < nblk; k++) blk2rec[k] = i;
        }
    }
    if (use_hist) {
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < t.n_locs; k += blockDim.x)
            if (hist[k]) atomicAdd(&counters[k], (unsigned long long)hist[k]);
    }
}

#include "gm_waf.inc"
#include "gm_rloc.inc"
#include "gm_decode.inc"

}  // namespace

// ============================================================================ host runtime
// A generation owns its device image and its counters (the counter space is the generation's
// locations + signatures): gm_load_generation builds the next one beside the live one and swaps
// under an exclusive lock; batches read `gen` under a shared lock for as long as they enqueue.
struct Generation {
    uint8_t *d_image = nullptr;
    unsigned long long *d_counters = nullptr;       // this device's cumulative counters
    unsigned long long *d_counters_sum = nullptr;   // gm_counters_allreduce's out-of-place result
    GTab *d_gtab = nullptr;                         // tab in device memory (GTab::self)
    size_t n_counters = 0;
    TabHeader hdr{};
    GTab tab{};
    gm_stats_t stats{};
    std::vector<uint8_t> host_image;   // kept for host-side introspection (gpumatch_debug.h)
    std::vector<std::string> peer_addrs;   // gm_peer_address
    std::vector<uint32_t> peer_ups;
    std::vector<UpstreamMeta> ups_meta;     // gm_update_upstream
    std::vector<std::string> rejects;       // gm_rejects
    // gm_update_upstream -> gm_peers_migrate: new peer id -> the previous table's peer id (GM_NONE:
    // a new server), and the previous table's peer count
    uint32_t *d_peer_map = nullptr;
    uint32_t peer_map_old_n = GM_NONE;
    ~Generation() {
        for (void *p : {(void *)d_image, (void *)d_counters, (void *)d_counters_sum, (void *)d_gtab, (void *)d_peer_map})
            if (p) (void)hipFree(p);
    }
};


// batches a stream may hold before gm_sync (the next gm_match_batch completes them first)
constexpr uint32_t PENDING_MAX = 64;
// Everything one batch writes, per (ctx, stream): batches on different streams never share a
// buffer, so gm_match_batch is thread-safe per ctx + stream pair without a ctx-wide lock.
struct Scratch {
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;               // k_route beside the WAF scan
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // recorded on `stream` after every call that enqueues work reading a generation or its
    // counters: a generation swap or a counter read waits for these events (not for the device)
    hipEvent_t ev_done = nullptr;
    bool done_rec = false;
    hipEvent_t ev[5] = {}, ev_route[2] = {};  // GM_CREATE_PROFILE stage events
    bool ev_pending = false, route_side = false;
    int ev_used = 0;
    uint32_t *d_status = nullptr, *h_status = nullptr;
    uint32_t *d_blk2rec = nullptr; size_t cap_blk = 0;
    unsigned long long *d_cand = nullptr; size_t cap_cand = 0;
    uint4 *d_surv = nullptr; size_t cap_surv = 0;   // stage-2 survivors (gm_waf.inc surv_entry, 16 B)
    unsigned long long *d_pairs = nullptr; size_t cap_pairs = 0; // unique active (request, rule) pairs
    unsigned long long *d_jobs = nullptr; size_t cap_jobs = 0;   // unique (request, regex, zone) jobs
    unsigned long long *d_set = nullptr; size_t cap_set = 0;     // dedupe set (power of two)
    uint32_t epoch = 0;                                          // dedupe epoch of the last batch
    // capacity multipliers: a batch that overflowed a buffer (void, GM_E_OVERFLOW at gm_sync)
    // doubles it for the stream's next batches -- traffic that passes the prefilter far more
    // often than the default sizing assumes (e.g. the C4 stress variant) settles after a retry
    uint32_t cand_mult = 1, surv_mult = 1, list_mult = 1;
    uint32_t *d_cnt = nullptr, *d_start = nullptr; size_t cap_cnt = 0, cap_start = 0;
    uint32_t *d_ccnt = nullptr; size_t cap_ccnt = 0;
    uint8_t *d_temp = nullptr; size_t cap_temp = 0;
    uint8_t *d_stage = nullptr; size_t cap_stage = 0;            // GM_BATCH_HOST staging
    uint64_t *d_wsize = nullptr, *d_wbase = nullptr; size_t cap_wsize = 0, cap_wbase = 0;   // wire parser
    uint8_t *d_wtemp = nullptr; size_t cap_wtemp = 0;
    uint8_t *d_wscr = nullptr; size_t cap_wscr = 0;   // the wire parser's per-wave $uri scratch
    uint8_t *d_wsum = nullptr; size_t cap_wsum = 0;   // and its pass-1 summaries (WireSum, 80 B each)
    uint32_t *d_wfull = nullptr; size_t cap_wfull = 0;   // pass 1's per-wave lists of the requests pass 2
                                                         // writes one at a time, then their counts
    uint32_t *d_wblk = nullptr; size_t cap_wblk = 0;     // pass 2's output block map (k_wire_blk)
    uint2 *d_wpieces = nullptr; size_t cap_wpieces = 0;  // pass 1's chunked-body pieces (WIRE_PIECES each)
    gm_wire_msg *d_wmsg = nullptr; size_t cap_wmsg = 0;   // and the descriptors past their PROXY headers
    uint32_t *d_pk = nullptr; size_t cap_pk = 0;     // peer selection: keys, values (x2: sorted),
    uint32_t *d_pseg = nullptr; size_t cap_pseg = 0; // per-upstream ranges, periodic programs
    uint4 *d_pprog = nullptr; size_t cap_pprog = 0;
    uint32_t *d_ppat = nullptr; size_t cap_ppat = 0;
    uint8_t *d_ptemp = nullptr; size_t cap_ptemp = 0;
    uint64_t *d_usize = nullptr; size_t cap_usize = 0;   // upstream URIs: sizes
    gm_req *d_sreqs = nullptr; size_t cap_sreqs = 0;     // decoded views: shadow records, arena,
    uint8_t *d_sarena = nullptr; size_t cap_sarena = 0;  // block map, sizes / bases, scan temp
    uint32_t *d_sblk = nullptr; size_t cap_sblk = 0;
    uint64_t *d_ssize = nullptr, *d_sbase = nullptr; size_t cap_ssize = 0, cap_sbase = 0;
    uint8_t *d_stemp = nullptr; size_t cap_stemp = 0;
    uint8_t *d_utemp = nullptr; size_t cap_utemp = 0;
    uint2 *d_rq = nullptr; size_t cap_rq = 0;            // regex-location requests deferred to k_rloc
    int32_t *d_rql = nullptr; size_t cap_rql = 0;        // and k_rloc's locations
    uint4 *d_rqs = nullptr; size_t cap_rqs = 0;          // and each one's $uri span + server (k_rloc_multi)
    uint4 *d_rqu = nullptr; size_t cap_rqu = 0;          // and its $uri's first 32 bytes (+ a pad block)
    int32_t *d_rqb = nullptr; size_t cap_rqb = 0;        // and its longest prefix match (the tail pass)
    unsigned long long *d_rqm = nullptr; size_t cap_rqm = 0;   // and its prefiltered-slice mask
    uint32_t *d_hlist = nullptr; size_t cap_hlist = 0;         // the anchored slices' candidate lists
    uint32_t *d_along = nullptr; size_t cap_along = 0;         // the always-run slices' long zones + count
    uint4 *d_amlist = nullptr; size_t cap_amlist = 0;          // and their match list (AlwMatch)
    uint32_t *d_amcnt = nullptr; size_t cap_amcnt = 0;         // with a count per slice
    uint32_t *d_hcnt = nullptr; size_t cap_hcnt = 0;           // and their lengths (k_rloc_heads)
    unsigned long long *d_bctr = nullptr; size_t cap_bctr = 0; // this batch's counters (k_ctr_commit)
    uint2 *d_slow = nullptr; size_t cap_slow = 0;              // requests for k_route's SLOW pass
    unsigned long long *d_agree = nullptr, *h_agree = nullptr;  // gm_counters_allreduce's agreement words
    // gm_sync's continuation of an OV_SET batch: the requests to redo (bitmap, list), their sub-batch
    uint32_t *d_redo = nullptr; size_t cap_redo = 0;
    uint32_t *d_rlist = nullptr; size_t cap_rlist = 0;
    uint64_t *d_rsize = nullptr, *d_rbase = nullptr; size_t cap_rsize = 0, cap_rbase = 0;
    uint8_t *d_rtemp = nullptr; size_t cap_rtemp = 0;
    gm_req *d_rsreq = nullptr; size_t cap_rsreq = 0;
    uint8_t *d_rsarena = nullptr; size_t cap_rsarena = 0;
    gm_verdict *d_rsout = nullptr; size_t cap_rsout = 0;
    uint32_t *d_rsblk = nullptr; size_t cap_rsblk = 0;
    uint32_t *d_rscnt = nullptr; size_t cap_rscnt = 0;
    // the pairs a full dedupe set refused (Dedup::spill) and their sorted copy
    unsigned long long *d_spill = nullptr, *d_spill2 = nullptr; size_t cap_spill = 0, cap_spill2 = 0;
    // each pending batch's final overflow bits (k_ctr_commit), one word per batch since the last
    // gm_sync: later batches do not clear an earlier one's
    uint32_t *d_ovlog = nullptr, *h_ovlog = nullptr;
    // the batches enqueued since the last gm_sync, with their arguments: gm_sync completes a batch
    // whose dedupe set overflowed (OV_SET) -- only the caller's hit_cap voids a batch
    struct Replay {
        uint32_t slot = 0;   // its word of d_ovlog
        const void *gen = nullptr; uint64_t seq = 0;
        const gm_req *reqs = nullptr; const uint8_t *A = nullptr; uint64_t alen = 0; uint32_t n = 0;
        gm_verdict *out = nullptr; uint32_t *hits = nullptr; size_t hit_cap = 0; const uint64_t *dlen = nullptr;
        // GM_BATCH_HOST: the staged device copies and the caller's host buffers
        gm_verdict *h_out = nullptr; uint32_t *h_hits = nullptr; size_t h_hit_cap = 0;
    };
    std::vector<Replay> pending;
    // per-batch outcome (GM_OK / GM_E_OVERFLOW) of the batches completed since the last gm_sync /
    // gm_sync_batches, in enqueue order: appended by each completion (a forced one in gm_match_batch
    // too), handed out and cleared by the next explicit sync
    std::vector<int32_t> sync_log;
    bool last_is_batch = false;   // the stream's last call was a gm_match_batch (its scratch in place)
    ~Scratch() {
        for (void *p : {(void *)d_status, (void *)d_blk2rec, (void *)d_cand, (void *)d_surv, (void *)d_pairs,
                        (void *)d_jobs, (void *)d_set, (void *)d_cnt, (void *)d_start, (void *)d_ccnt,
                        (void *)d_temp, (void *)d_stage, (void *)d_wsize, (void *)d_wbase, (void *)d_wtemp, (void *)d_wscr, (void *)d_wsum, (void *)d_wfull, (void *)d_wblk, (void *)d_wpieces,
                        (void *)d_pk, (void *)d_pseg, (void *)d_pprog, (void *)d_ppat, (void *)d_ptemp,
                        (void *)d_usize, (void *)d_utemp, (void *)d_sreqs, (void *)d_sarena, (void *)d_sblk,
                        (void *)d_ssize, (void *)d_sbase, (void *)d_stemp, (void *)d_rq, (void *)d_rql, (void *)d_rqs, (void *)d_rqb, (void *)d_rqm, (void *)d_rqu, (void *)d_bctr, (void *)d_slow,
                        (void *)d_redo, (void *)d_rlist, (void *)d_rsize, (void *)d_rbase, (void *)d_rtemp, (void *)d_rsreq,
                        (void *)d_rsarena, (void *)d_rsout, (void *)d_rsblk, (void *)d_rscnt, (void *)d_ovlog, (void *)d_wmsg, (void *)d_spill, (void *)d_spill2,
                        (void *)d_hlist, (void *)d_hcnt, (void *)d_along, (void *)d_amlist, (void *)d_amcnt})
            if (p) (void)hipFree(p);
        if (h_status) (void)hipHostFree(h_status);
        if (h_ovlog) (void)hipHostFree(h_ovlog);
        if (h_agree) (void)hipHostFree(h_agree);
        if (d_agree) (void)hipFree(d_agree);
        for (auto &e : ev) if (e) (void)hipEventDestroy(e);
        for (auto &e : ev_route) if (e) (void)hipEventDestroy(e);
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (side) (void)hipStreamDestroy(side);
    }
};

// ---- gm_counters_allreduce's protocol: the agreement rides in the counter sum.
// Each rank contributes, beside its counters, a block of RED_WORDS u64 words {1, v, v^2 for the four
// 16-bit halves v of (gen, n_counters), 0} to one SUM: with N = the summed first word, the ranks
// hold one value v iff N * sum(v^2) == sum(v)^2 (Cauchy-Schwarz; exact in u64 for N < 2^20).  The
// collective's count is RED_WORDS + the agreed n on every rank (agreed by the same test, once,
// synchronously).  A call whose block shows the ranks apart, or on another n, has no valid totals,
// and the next call re-agrees synchronously; every rank reads the same block, so every rank takes
// the same branch at the same call and no collective of mismatched size is ever issued.
constexpr uint32_t RED_WORDS = 10;
struct RedBlock { unsigned long long w[RED_WORDS]; };
struct RedProto {
    bool agreed = false;      // (gen, n) agreed: the combined collective carries RED_WORDS + n words
    uint32_t gen = 0;
    uint64_t n = 0;
    bool last_valid = true;   // the last call's totals are every rank's counters of one space
    static void pack(uint32_t g, uint64_t cnt, unsigned long long *w) {
        const uint32_t v[4] = {g & 0xFFFFu, g >> 16, (uint32_t)(cnt & 0xFFFFu), (uint32_t)((cnt >> 16) & 0xFFFFu)};
        w[0] = 1;
        for (int i = 0; i < 4; i++) { w[1 + 2 * i] = v[i]; w[2 + 2 * i] = (unsigned long long)v[i] * v[i]; }
        w[9] = 0;
    }
    __host__ __device__ static bool all_equal(const unsigned long long *s, uint32_t &g, uint64_t &cnt) {
        const unsigned long long N = s[0];
        if (N == 0) return false;
        uint32_t v[4];
        for (int i = 0; i < 4; i++) {
            if (N * s[2 + 2 * i] != s[1 + 2 * i] * s[1 + 2 * i]) return false;
            v[i] = (uint32_t)(s[1 + 2 * i] / N);
        }
        g = v[0] | v[1] << 16;
        cnt = (uint64_t)v[2] | (uint64_t)v[3] << 16;
        return true;
    }
    // the block-only collective of a synchronous agreement
    bool agree(const unsigned long long *s) {
        uint32_t g; uint64_t m;
        agreed = all_equal(s, g, m);
        if (agreed) { gen = g; n = m; } else last_valid = false;
        return agreed;
    }
    // the summed block of a combined collective
    void finish(const unsigned long long *s) {
        uint32_t g; uint64_t m;
        last_valid = all_equal(s, g, m) && m == n;
        if (last_valid) gen = g; else agreed = false;
    }
};
// [block | the first na counters, zero-padded] -- the rank's contribution (n: its own count)
__global__ void k_red_stage(const unsigned long long *__restrict__ ctr, uint64_t n, uint64_t na, RedBlock b,
                            unsigned long long *__restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < RED_WORDS + na; i += (uint64_t)gridDim.x * blockDim.x) {
        unsigned long long v = 0;
        if (i < RED_WORDS) {
#pragma unroll
            for (uint32_t k = 0; k < RED_WORDS; k++) if (i == k) v = b.w[k];
        } else if (i - RED_WORDS < n) {
            v = ctr[i - RED_WORDS];
        }
        out[i] = v;
    }
}
// the totals to the generation's reduced buffer, only when the block shows every rank on this
// count (the same test the host applies to the block afterwards)
__global__ void k_red_finish(const unsigned long long *__restrict__ sum, uint64_t na, unsigned long long *__restrict__ dst,
                             uint64_t n) {
    uint32_t g;
    uint64_t m;
    if (!RedProto::all_equal(sum, g, m) || m != na || n != na) return;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < na; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = sum[RED_WORDS + i];
}

struct gm_ctx {
    int dev = 0;
    uint32_t flags = 0;
    int cu_count = 256;
    double cap_scale = 1.0;                   // GM_CREATE_SCRATCH_SHIFT (test hook): internal WAF capacities
    uint32_t set_shift = 0;                   // GM_CREATE_SET_SHIFT (test hook): the dedupe set
    uint32_t spill_shift = 0;                 // GM_CREATE_SPILL_SHIFT (test hook): the refused pairs' spill
    std::atomic<uint32_t> n_set_reruns{0};    // gm_sync re-runs of OV_SET batches
    std::atomic<uint32_t> last_redo{0};       // requests the last continuation redid
    std::atomic<uint32_t> last_spill{0};      // pairs the last spill continuation emitted from the spill
    std::shared_mutex gen_mu;                 // shared: enqueueing batches; exclusive: the swap
    Generation *gen = nullptr;
    uint64_t publish_seq = 0;                 // bumped under gen_mu (exclusive) by every publish
    std::mutex scr_mu;                        // the stream -> scratch map only
    std::map<hipStream_t, std::unique_ptr<Scratch>> scratch;
    ncclComm_t comm = nullptr;
    // gm_counters_allreduce's protocol state (RedProto) and buffers: [agreement block | counters] in
    // and out, the last call's summed block (pinned) and its completion event
    std::mutex red_mu;
    RedProto red;
    unsigned long long *d_red = nullptr; size_t cap_red = 0;
    unsigned long long *h_red = nullptr;
    hipEvent_t ev_red = nullptr;
    bool red_pending = false;
    // last completed batch (gm_sync), for gm_stats / gm_debug_status
    std::mutex last_mu;
    uint64_t last_candidates = 0, last_pairs = 0, last_hits = 0, last_ctx_pass = 0, last_jobs = 0;
    float last_ms[4] = {0, 0, 0, 0};
    uint32_t last_status[STATUS_WORDS] = {};
};

// gm_last_error() is thread-local (include/gpumatch.h): concurrent callers on one ctx never see
// each other's messages
static thread_local std::string t_err;
// gm_debug_update_hook: a test callback run by gm_update_upstream between reading the live tables
// and publishing (no lock held), e.g. a gm_load_generation racing the update
static void (*g_update_hook)(void *) = nullptr;
static void *g_update_hook_arg = nullptr;

static int fail(gm_ctx *, int code, const std::string &m) {
    t_err = m;
    return code;
}
#define HIPCHK(c, x)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return fail((c), GM_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

// grow a scratch buffer of stream s: work already enqueued on s may still read the old one, so
// the stream drains first (only when a batch outgrows the buffer, i.e. the first large batches)
template <class T>
static int grow(gm_ctx *c, hipStream_t s, T *&p, size_t &cap, size_t need) {
    if (need <= cap) return GM_OK;
    if (p) {
        HIPCHK(c, hipStreamSynchronize(s));
        HIPCHK(c, hipFree(p));
    }
    p = nullptr;
    cap = 0;
    const size_t nc = need + need / 4;
    HIPCHK(c, hipMalloc((void **)&p, nc * sizeof(T)));
    cap = nc;
    return GM_OK;
}

// the scratch of `stream`, created on first use (with its side stream, events and status words)
static Scratch *scratch_for(gm_ctx *c, hipStream_t stream) {
    std::lock_guard<std::mutex> lk(c->scr_mu);
    auto it = c->scratch.find(stream);
    if (it != c->scratch.end()) return it->second.get();
    std::unique_ptr<Scratch> s(new Scratch());
    s->stream = stream;
    if (hipMalloc((void **)&s->d_status, STATUS_WORDS * 4) != hipSuccess ||
        hipHostMalloc((void **)&s->h_status, STATUS_WORDS * 4, hipHostMallocDefault) != hipSuccess ||
        hipMemset(s->d_status, 0, STATUS_WORDS * 4) != hipSuccess ||
        hipMalloc((void **)&s->d_ovlog, PENDING_MAX * 4) != hipSuccess ||
        hipHostMalloc((void **)&s->h_ovlog, PENDING_MAX * 4, hipHostMallocDefault) != hipSuccess ||
        hipMemset(s->d_ovlog, 0, PENDING_MAX * 4) != hipSuccess ||
        hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming) != hipSuccess) {
        t_err = "scratch allocation failed";
        return nullptr;
    }
    memset(s->h_status, 0, STATUS_WORDS * 4);
    if (c->flags & GM_CREATE_PROFILE) {
        for (auto &e : s->ev) if (hipEventCreate(&e) != hipSuccess) { t_err = "event create failed"; return nullptr; }
        for (auto &e : s->ev_route) if (hipEventCreate(&e) != hipSuccess) { t_err = "event create failed"; return nullptr; }
    }
    Scratch *p = s.get();
    c->scratch.emplace(stream, std::move(s));
    return p;
}

// the call just enqueued on S's stream is the stream's last use of the live generation so far
static int mark_done(gm_ctx *c, Scratch *S) {
    HIPCHK(c, hipEventRecord(S->ev_done, S->stream));
    S->done_rec = true;
    return GM_OK;
}
// Scope guard of a call that enqueues work: done() records ev_done; an early (error) return drains
// the stream and its side stream instead, so nothing enqueued before the error is left in flight
// uncovered by an event (RCU retirement and counter reads wait only on ev_done).
struct DoneGuard {
    Scratch *S;
    bool armed = true;
    explicit DoneGuard(Scratch *s) : S(s) {}
    int done(gm_ctx *c) { armed = false; return mark_done(c, S); }
    ~DoneGuard() {
        if (armed && S) {
            (void)hipStreamSynchronize(S->side);
            (void)hipStreamSynchronize(S->stream);
        }
    }
};

// Wait until every call enqueued so far through this ctx has completed: the completion event of
// each stream's last call (RCU retirement of a swapped-out generation, counter reads).  Only this
// ctx's streams are waited for -- not the device (other work on it, other contexts).  Events are
// owned by the scratch, so a stream the caller has destroyed since is no hazard.
static int wait_done(gm_ctx *c) {
    std::vector<hipEvent_t> evs;
    {
        std::lock_guard<std::mutex> lk(c->scr_mu);
        for (auto &kv : c->scratch) if (kv.second->done_rec) evs.push_back(kv.second->ev_done);
    }
    for (hipEvent_t e : evs) HIPCHK(c, hipEventSynchronize(e));
    return GM_OK;
}

#ifdef GM_EXP_COUNT
extern "C" int gm_exp_read(unsigned long long *out) {
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_exp), sizeof(unsigned long long) * 8);
    unsigned long long z[8] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(g_exp), z, sizeof z);
    return 0;
}
#endif
extern "C" const char gm_csrc_hash_text[];   // gm_buildid.cpp (the Makefile's source hash)
static uint64_t csrc_hash_u64() {
    uint64_t v = 0;
    for (int k = 0; k < 16; k++) {
        const char ch = gm_csrc_hash_text[k];
        const int d = ch >= '0' && ch <= '9' ? ch - '0' : ch >= 'a' && ch <= 'f' ? ch - 'a' + 10 : -1;
        if (d < 0) return 0;
        v = v << 4 | (uint64_t)d;
    }
    return v;
}
extern "C" {

uint32_t gm_abi_version(void) { return GM_ABI_VERSION; }
const char *gm_build_hash(void) { return gm_csrc_hash_text; }

gm_ctx *gm_create(int hip_device, uint32_t flags) {
    gm_ctx *c = new gm_ctx();
    c->dev = hip_device;
    c->flags = flags;
    if (const uint32_t k = (flags >> 8) & 0xFFu) c->cap_scale = k < 32 ? 1.0 / (double)(1ull << k) : 1.0;
    if (const uint32_t k = (flags >> 16) & 0xFFu) c->set_shift = k < 24 ? k : 0;
    if (const uint32_t k = (flags >> 24) & 0xFFu) c->spill_shift = k < 24 ? k : 0;
    if (!(flags & GM_CREATE_COMPILE_ONLY)) {
        if (hipSetDevice(hip_device) != hipSuccess) { t_err = "hipSetDevice failed"; delete c; return nullptr; }
        // the WAF scan's Bloom filter is dynamic LDS beyond the 64 KiB default
        const void *scans[] = {(const void *)k_waf_scan<BLOOM_PK_PERM, SCAN_DEPTH>, (const void *)k_waf_scan<1, SCAN_DEPTH>,
                               (const void *)k_waf_scan<2, SCAN_DEPTH>, (const void *)k_waf_scan<3, SCAN_DEPTH>,
                               (const void *)k_waf_direct<BLOOM_PK_PERM>, (const void *)k_waf_direct<1>,
                               (const void *)k_waf_direct<2>, (const void *)k_waf_direct<3>};
        for (const void *f : scans)
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)SCAN_DYN_LDS) != hipSuccess) {
                t_err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; delete c; return nullptr;
            }
        const void *alws[] = {(const void *)k_waf_always_multi<1>, (const void *)k_waf_always_multi<2>,
                              (const void *)k_waf_always_multi<3>, (const void *)k_waf_always_multi<4>,
                              (const void *)k_waf_always_multi<5>, (const void *)k_waf_always_multi<6>,
                              (const void *)k_waf_always_multi<7>, (const void *)k_waf_always_multi<8>,
                              (const void *)k_rloc_multi<1>, (const void *)k_rloc_multi<2>,
                              (const void *)k_rloc_multi<3>, (const void *)k_rloc_multi<4>,
                              (const void *)k_rloc_multi<5>, (const void *)k_rloc_multi<6>,
                              (const void *)k_rloc_multi<7>, (const void *)k_rloc_multi<8>};
        for (const void *f : alws) {
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ALWAYS_LDS_BYTES) != hipSuccess) {
                t_err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; delete c; return nullptr;
            }
            // their chains address the slice by its LDS offset (alw_step): the dynamic LDS must start
            // at 0, i.e. the kernels hold no static __shared__
            hipFuncAttributes fa{};
            if (hipFuncGetAttributes(&fa, f) != hipSuccess || fa.sharedSizeBytes != 0) {
                t_err = "union-DFA kernel with static LDS (alw_step needs its slice at LDS offset 0)"; delete c; return nullptr;
            }
        }
        if (hipFuncSetAttribute((const void *)k_rloc_heads, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(HEADS_LDS_SLOTS * RSL_HEAD_WORDS * 4)) != hipSuccess) {
            t_err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; delete c; return nullptr;
        }
        if (hipFuncSetAttribute((const void *)k_rloc_pref, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)RLOC_PREF_LDS) != hipSuccess) {
            t_err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; delete c; return nullptr;
        }
        // the route's hot tables + location histogram (route_lds)
        const void *routes[] = {(const void *)k_route<3, true, true>, (const void *)k_route<3, true>,
                                (const void *)k_route<3>, (const void *)k_route<GM_ROUTE_WPE, true>, (const void *)k_route<GM_ROUTE_WPE>};
        for (const void *f : routes)
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(ROUTE_STAGE_BYTES + 4 * LDS_HIST_ALONE)) != hipSuccess) {
                t_err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; delete c; return nullptr;
            }
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, hip_device) == hipSuccess && cus > 0)
            c->cu_count = cus;
    }
    return c;
}

void gm_destroy(gm_ctx *c) {
    if (!c) return;
    if (!(c->flags & GM_CREATE_COMPILE_ONLY)) {
        (void)hipSetDevice(c->dev);
        (void)hipDeviceSynchronize();
        c->scratch.clear();
        if (c->comm) ncclCommDestroy(c->comm);
        if (c->d_red) (void)hipFree(c->d_red);
        if (c->h_red) (void)hipHostFree(c->h_red);
        if (c->ev_red) (void)hipEventDestroy(c->ev_red);
    }
    delete c->gen;
    delete c;
}

const char *gm_last_error(gm_ctx *) { return t_err.c_str(); }

// Publish compiled tables as the live generation: device copy-in beside the live one, swap under
// the exclusive lock, then RCU retirement -- every call that read the old generation finished
// enqueueing before the lock was granted, and its completion event is waited for before the old
// memory is freed.  `same_counters`: the new tables keep the live generation's counter space
// (gm_update_upstream: same locations and signatures), the counters move over unreset.
// `expect_seq` (same_counters only): the publish_seq the tables were derived under -- a load or
// another update published since fails GM_E_STALE instead of being overwritten (the reference's
// Plus update refuses a configVersion mismatch, verifyConfigVersion, manager.go:258).
static int publish(gm_ctx *c, CompileResult &R, uint32_t gen, bool same_counters, uint64_t expect_seq = 0) {
    if (R.stats.n_sigs >= (1u << 21) || R.stats.n_sig_regex >= (1u << 21))
        return fail(c, GM_E_INVAL, "more than 2^21 signatures");
    std::unique_ptr<Generation> g(new Generation());
    g->hdr = R.hdr;
    g->host_image = R.image;
    g->stats = R.stats;
    g->stats.gen = gen;
    g->peer_addrs = std::move(R.peer_addrs);
    g->peer_ups = std::move(R.peer_ups);
    g->ups_meta = std::move(R.ups_meta);
    g->rejects = std::move(R.rejects);
    g->n_counters = g->stats.n_counters;
    if (!(c->flags & GM_CREATE_COMPILE_ONLY)) {
        HIPCHK(c, hipSetDevice(c->dev));
        HIPCHK(c, hipMalloc((void **)&g->d_image, R.image.size()));
        HIPCHK(c, hipMemcpy(g->d_image, R.image.data(), R.image.size(), hipMemcpyHostToDevice));
        g->tab = make_gtab(g->hdr, g->d_image, gen);
        HIPCHK(c, hipMalloc((void **)&g->d_gtab, sizeof(GTab)));
        g->tab.self = g->d_gtab;
        HIPCHK(c, hipMemcpy(g->d_gtab, &g->tab, sizeof(GTab), hipMemcpyHostToDevice));
        if (!R.peer_map.empty()) {
            HIPCHK(c, hipMalloc((void **)&g->d_peer_map, R.peer_map.size() * 4));
            HIPCHK(c, hipMemcpy(g->d_peer_map, R.peer_map.data(), R.peer_map.size() * 4, hipMemcpyHostToDevice));
        }
        if (!same_counters) {
            const size_t cb = std::max<size_t>(g->n_counters, 1) * 8;
            HIPCHK(c, hipMalloc((void **)&g->d_counters, cb));
            HIPCHK(c, hipMalloc((void **)&g->d_counters_sum, cb));
            HIPCHK(c, hipMemset(g->d_counters, 0, cb));
            HIPCHK(c, hipMemset(g->d_counters_sum, 0, cb));
        }
    }
    Generation *old;
    {
        std::unique_lock<std::shared_mutex> lk(c->gen_mu);
        old = c->gen;
        if (same_counters) {
            if (c->publish_seq != expect_seq || !old)
                return fail(c, GM_E_STALE, "the live generation changed during the upstream update (a load or "
                                           "another update published first); nothing published");
            if (old->n_counters != g->n_counters) return fail(c, GM_E_INVAL, "counter space changed");
            g->d_counters = old->d_counters; g->d_counters_sum = old->d_counters_sum;
            old->d_counters = old->d_counters_sum = nullptr;
            g->peer_map_old_n = old->stats.n_peers;
        }
        c->gen = g.release();
        c->publish_seq++;
    }
    if (old && !(c->flags & GM_CREATE_COMPILE_ONLY)) {
        const int e = wait_done(c);
        if (e) { delete old; return e; }
    }
    delete old;
    return GM_OK;
}

int gm_load_generation(gm_ctx *c, const void *blob, size_t len, uint32_t gen) {
    if (!c || !blob) return fail(c, GM_E_INVAL, "null argument");
    CompileResult R = compile_generation((const uint8_t *)blob, len, gen);
    if (!R.ok) return fail(c, R.code, R.err);   // previous generation stays live
    return publish(c, R, gen, false);
}

int gm_update_upstream(gm_ctx *c, const char *upstream, const char *const *servers, uint32_t n) {
    if (!c || !upstream || (n && !servers)) return fail(c, GM_E_INVAL, "null argument");
    std::vector<std::string> addrs;
    for (uint32_t i = 0; i < n; i++) {
        if (!servers[i] || !servers[i][0]) return fail(c, GM_E_INVAL, "empty server address");
        addrs.emplace_back(servers[i]);
    }
    CompileResult live;
    uint32_t gen;
    uint64_t seq;
    {
        std::shared_lock<std::shared_mutex> lk(c->gen_mu);
        const Generation *g = c->gen;
        if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
        live.image = g->host_image; live.hdr = g->hdr; live.stats = g->stats;
        live.peer_addrs = g->peer_addrs; live.peer_ups = g->peer_ups; live.ups_meta = g->ups_meta;
        live.rejects = g->rejects;
        gen = g->stats.gen;
        seq = c->publish_seq;
    }
    CompileResult R = update_upstream(live, upstream, addrs);
    if (!R.ok) return fail(c, R.code, R.err);
    R.rejects = live.rejects;
    if (g_update_hook) g_update_hook(g_update_hook_arg);   // tests: a load between the read and the publish
    return publish(c, R, gen, true, seq);
}

static uint32_t build_flags();   // (defined at the end of the file: every tuning macro is set by then)


int gm_stats(gm_ctx *c, gm_stats_t *out) {
    if (!c || !out) return fail(c, GM_E_INVAL, "null argument");
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    if (!c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    *out = c->gen->stats;
    out->build_flags = build_flags();
    out->csrc_hash = csrc_hash_u64();
    out->scratch_scale = (float)c->cap_scale;
    out->n_set_reruns = c->n_set_reruns.load();
    out->last_redo = c->last_redo.load();
    out->last_spill = c->last_spill.load();
    out->set_shift = c->set_shift;
    std::lock_guard<std::mutex> l2(c->last_mu);
    out->last_candidates = c->last_candidates;
    out->last_pairs = c->last_pairs;
    out->last_hits = c->last_hits;
    out->last_ctx_pass = (uint32_t)c->last_ctx_pass;
    out->last_jobs = (uint32_t)c->last_jobs;
    out->last_ms_route = c->last_ms[0]; out->last_ms_scan = c->last_ms[1];
    out->last_ms_verify = c->last_ms[2]; out->last_ms_tail = c->last_ms[3];
    return GM_OK;
}

int gm_rejects(gm_ctx *c, char *buf, size_t cap) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    if (!c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    std::string t;
    for (const std::string &r : c->gen->rejects) { t += r; t += '\n'; }
    if (buf && cap) {
        const size_t k = std::min(cap - 1, t.size());
        memcpy(buf, t.data(), k);
        buf[k] = 0;
    }
    return (int)std::min<size_t>(t.size(), 0x7FFFFFFF);
}

// Enqueue one batch on stream s (device pointers).  No host synchronisation: every size a later
// stage needs is a device status word or a host-known capacity.
// the always-run regexes: the LDS-staged groups, then the groups read from the image, then the
// regexes no group could take (lane per (request, regex))
static int launch_always(gm_ctx *c, hipStream_t s, const Generation *g, const uint8_t *A, uint64_t alen,
                         const gm_req *reqs, uint32_t n, Scratch *S, const Dedup &dd, bool skip_empty,
                         const uint64_t *dlen) {
    const GTab &t = g->tab;
    const DAlwSlice *sls = reinterpret_cast<const DAlwSlice *>(g->host_image.data() + g->hdr.off_alw_slices);
    // the long zones first (k_alw_long): one list per WAF pass, one entry per request's long zone at
    // most on average (a longer list is not used)
    uint32_t n_slices = 0;
    for (uint32_t k = 0; k < t.n_alw_slices; k++) n_slices += sls[k].server == GM_NONE;
    const uint32_t lcap = std::max<uint32_t>(n, 1024);
    if (n_slices) {
        int e;
        if ((e = grow(c, s, S->d_along, S->cap_along, (size_t)lcap + 1))) return e;
        HIPCHK(c, hipMemsetAsync(S->d_along + lcap, 0, 4, s));
        k_alw_long<<<std::max<uint32_t>(1, std::min<uint32_t>((n + 1023) / 1024, (uint32_t)c->cu_count * 4)), 1024, 0, s>>>(
            reqs, n, dd.out, S->d_along, lcap, S->d_along + lcap);
        HIPCHK(c, hipGetLastError());
    }
    const uint32_t *LL = S->d_along, *LC = S->d_along + lcap;
    // the slices' match lists (AlwMatch): one region reused slice after slice, a count per slice;
    // k_alw_emit turns each slice's matches into pairs right after it
    AlwMatch am{};
    if (t.n_alw_slices) {
        int e;
        // (GM_CREATE_SCRATCH_SHIFT scales it, GM_CREATE_SPILL_SHIFT shrinks it: the test hooks of
        // the lists whose overflow gm_sync completes)
        const size_t mcap = std::max<size_t>(
            (size_t)((double)(((size_t)n / 4 + 65536) * S->list_mult) * c->cap_scale) >> c->spill_shift, 16);
        if ((e = grow(c, s, S->d_amlist, S->cap_amlist, mcap)) ||
            (e = grow(c, s, S->d_amcnt, S->cap_amcnt, (size_t)t.n_alw_slices)))
            return e;
        HIPCHK(c, hipMemsetAsync(S->d_amcnt, 0, (size_t)t.n_alw_slices * 4, s));
        am = AlwMatch{S->d_amlist, S->d_amcnt, (uint32_t)std::min<size_t>(std::min(mcap, S->cap_amlist), 0xFFFFFFFFu), dd.redo,
                      dd.status};
    }
    for (uint32_t k = 0; k < t.n_alw_slices; k++) {
        const DAlwSlice &sl = sls[k];
        const dim3 grid((uint32_t)c->cu_count), blk(1024);
        AlwMatch amk = am;
        amk.count = am.count + k;
        switch (sl.n_groups) {
        case 1: k_waf_always_multi<1><<<grid, blk, sl.len, s>>>(A, alen, reqs, n, t, dd.out, amk, skip_empty, dlen, k, LL, LC, lcap); break;
        case 2: k_waf_always_multi<2><<<grid, blk, sl.len, s>>>(A, alen, reqs, n, t, dd.out, amk, skip_empty, dlen, k, LL, LC, lcap); break;
        case 3: k_waf_always_multi<3><<<grid, blk, sl.len, s>>>(A, alen, reqs, n, t, dd.out, amk, skip_empty, dlen, k, LL, LC, lcap); break;
        case 4: k_waf_always_multi<4><<<grid, blk, sl.len, s>>>(A, alen, reqs, n, t, dd.out, amk, skip_empty, dlen, k, LL, LC, lcap); break;
        case 5: k_waf_always_multi<5><<<grid, blk, sl.len, s>>>(A, alen, reqs, n, t, dd.out, amk, skip_empty, dlen, k, LL, LC, lcap); break;
        case 6: k_waf_always_multi<6><<<grid, blk, sl.len, s>>>(A, alen, reqs, n, t, dd.out, amk, skip_empty, dlen, k, LL, LC, lcap); break;
        case 7: k_waf_always_multi<7><<<grid, blk, sl.len, s>>>(A, alen, reqs, n, t, dd.out, amk, skip_empty, dlen, k, LL, LC, lcap); break;
        default: k_waf_always_multi<8><<<grid, blk, sl.len, s>>>(A, alen, reqs, n, t, dd.out, amk, skip_empty, dlen, k, LL, LC, lcap); break;
        }
        HIPCHK(c, hipGetLastError());
        k_alw_emit<<<(uint32_t)c->cu_count * 2, 256, 0, s>>>(t, am.list, amk.count, am.cap, S->d_pairs, (uint32_t)S->cap_pairs, dd);
        HIPCHK(c, hipGetLastError());
    }
    if (t.n_always > t.n_always_lds) {
        k_waf_always<<<(uint32_t)c->cu_count * 8, 256, 0, s>>>(A, reqs, n, t, S->d_pairs, (uint32_t)S->cap_pairs, dd,
                                                               skip_empty, t.n_always_lds);
        HIPCHK(c, hipGetLastError());
    }
    return GM_OK;
}

// ---- the WAF stages of one pass, shared by a batch (beside its route) and gm_sync's dedupe-set
// continuation (a sub-batch of the requests to redo)
struct WafCaps {
    uint32_t scan_blocks, W, wcap, bcap, exact_blocks;
    size_t scan_tmp;
    uint32_t *xprof;
    u32x4 *cand;
};
struct WafIO {
    const uint8_t *A; uint64_t alen; const uint64_t *dlen;
    const gm_req *reqs; uint32_t n;
    const gm_verdict *out;     // verdicts (waf_active, the decoders' location)
    const uint32_t *blk2rec;   // arena block -> first record (the route writes the batch's)
    uint32_t nblk;
};
#ifndef GM_EXACT_BPC
#define GM_EXACT_BPC 6
#endif
// grow the pair list keeping its first `keep` entries (the continuation appends to the first pass's)
static int grow_keep(gm_ctx *c, hipStream_t s, unsigned long long *&p, size_t &cap, size_t need, size_t keep) {
    if (need <= cap) return GM_OK;
    unsigned long long *np = nullptr;
    const size_t nc = need + need / 4;
    HIPCHK(c, hipMalloc((void **)&np, nc * 8));
    if (p && keep) HIPCHK(c, hipMemcpyAsync(np, p, std::min(keep, cap) * 8, hipMemcpyDeviceToDevice, s));
    if (p) { HIPCHK(c, hipStreamSynchronize(s)); HIPCHK(c, hipFree(p)); }
    p = np; cap = nc;
    return GM_OK;
}
// capacities (host-known: the arena length and the request count, never a device count) and the
// buffers grown to them; keep_pairs: entries of the pair list to preserve across a growth
static int waf_buffers(gm_ctx *c, Scratch *S, uint64_t alen, uint32_t n, WafCaps &k, size_t keep_pairs = 0) {
    hipStream_t s = S->stream;
    int e;
    // candidate records: 32 B (4 x u64) each, room for one per 64 arena bytes; survivors; unique
    // pairs (2 per request on average) and jobs (1 per request); overflow is reported, never
    // truncated silently
    k.scan_blocks = (uint32_t)c->cu_count;
    k.W = k.scan_blocks * SCAN_WAVES;
    const uint32_t W = k.W;
    // (GM_CREATE_SCRATCH_SHIFT, a test hook: scales these defaults, so the overflow continuations run on
    // batches small enough for the oracle)
    const double sc = c->cap_scale;
    auto scaled = [sc](size_t x, size_t lo) { return std::max<size_t>(lo, (size_t)((double)x * sc)); };
    const size_t ccap = scaled(4 * (alen / 64 + 16384) * S->cand_mult, 4 * W);
    const size_t pcap0 = ((size_t)n * 2 + 65536) * S->list_mult, jcap0 = ((size_t)n + 65536) * S->list_mult;
    const size_t pcap = scaled(pcap0, 64) + keep_pairs, jcap = scaled(jcap0, 64);
    // the dedupe set holds every unique pair and job of the batch (the lists' fallback when they
    // overflow): sized from the unscaled list capacities
    size_t set_need = 1;
    while (set_need < 2 * (pcap0 + jcap0)) set_need <<= 1;
    set_need = std::max<size_t>(set_need >> c->set_shift, 1024);
    k.scan_tmp = 0;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, k.scan_tmp, S->d_cnt, S->d_start, (int)n + 1, s));
    if ((e = grow(c, s, S->d_cand, S->cap_cand, std::max<size_t>(ccap, scaled((size_t)W * 4096, 4 * W))))) return e;
    // scan-wave counts, ctx-block counts, scan-wave resume chunks, ctx-region resume records,
    // then k_waf_exact's per-workgroup profiling partials (4 words each)
    k.exact_blocks = (uint32_t)c->cu_count * GM_EXACT_BPC;
    if ((e = grow(c, s, S->d_ccnt, S->cap_ccnt, 3 * (size_t)W + k.scan_blocks + 4 * (size_t)k.exact_blocks))) return e;
    k.xprof = S->d_ccnt + 3 * (size_t)W + k.scan_blocks;
    if ((e = grow(c, s, S->d_surv, S->cap_surv, std::min<size_t>(scaled((alen / 256 + 65536) * S->surv_mult, k.scan_blocks),
                                                                 0xFFFFFFFFu)))) return e;
    if ((e = grow_keep(c, s, S->d_pairs, S->cap_pairs, pcap, keep_pairs))) return e;
    if ((e = grow(c, s, S->d_spill, S->cap_spill, pcap))) return e;
    if ((e = grow(c, s, S->d_jobs, S->cap_jobs, jcap))) return e;
    if ((e = grow(c, s, S->d_cnt, S->cap_cnt, (size_t)n + 1))) return e;
    if ((e = grow(c, s, S->d_start, S->cap_start, (size_t)n + 1))) return e;
    if ((e = grow(c, s, S->d_temp, S->cap_temp, k.scan_tmp))) return e;
    if (set_need > S->cap_set) {
        if ((e = grow(c, s, S->d_set, S->cap_set, set_need))) return e;
        S->cap_set = set_need;   // exactly a power of two: the probe mask
        S->epoch = 0;
        HIPCHK(c, hipMemsetAsync(S->d_set, 0, S->cap_set * 8, s));
    }
    k.wcap = (uint32_t)std::min<size_t>(S->cap_cand / 4 / W, 0xFFFFFFFFu);   // records per wave
    k.bcap = (uint32_t)std::min<size_t>(S->cap_surv / k.scan_blocks, 0xFFFFFFFFu);   // survivors per workgroup
    k.cand = reinterpret_cast<u32x4 *>(S->d_cand);
    return GM_OK;
}
// one epoch per pass over the set (two with decoders: the decoded pass's jobs take epoch + 1)
static int next_epoch(gm_ctx *c, Scratch *S, const GTab &t) {
    S->epoch += t.decoders ? 2 : 1;
    if (S->epoch + (t.decoders ? 1 : 0) > 255) {   // epoch wrap: every slot becomes free again
        S->epoch = 1;
        HIPCHK(c, hipMemsetAsync(S->d_set, 0, S->cap_set * 8, S->stream));
    }
    return GM_OK;
}

static int launch_scan(gm_ctx *c, Scratch *S, const GTab &t, const WafCaps &k, const uint8_t *A, uint64_t alen,
                       const uint64_t *dlen) {
    hipStream_t s = S->stream;
    const uint32_t W = k.W;
#define GM_SCAN(PKV) k_waf_scan<PKV, SCAN_DEPTH><<<k.scan_blocks, SCAN_BLOCK, SCAN_DYN_LDS, s>>>(A, alen, t, k.cand, k.wcap, \
        S->d_ccnt, dlen, S->d_ccnt + W + k.scan_blocks)
    if (t.bloom_pk == BLOOM_PK_PERM) GM_SCAN(BLOOM_PK_PERM);
    else if (t.bloom_pk == 1) GM_SCAN(1);
    else if (t.bloom_pk == 2) GM_SCAN(2);
    else GM_SCAN(3);
#undef GM_SCAN
    HIPCHK(c, hipGetLastError());
    return GM_OK;
}

// scan -> (route_hook: the route beside it) -> context filter -> (join: the route's outputs) ->
// exact check -> overflow continuation -> regex jobs -> always-run regexes, then the same stages
// over the decoded views when the signature set declares parsers
static int waf_stages(gm_ctx *c, Scratch *S, const Generation *g, const WafCaps &k, const WafIO &io, const Dedup &dd,
                      const std::function<int()> &route_hook, bool join, const std::function<int(int)> &mark) {
    hipStream_t s = S->stream;
    const GTab &t = g->tab;
    const uint32_t W = k.W, scan_blocks = k.scan_blocks, n = io.n;
    int e;
    // persistent scan grid: one 1024-thread workgroup per CU (128 KiB LDS prefilter); every wave
    // owns a contiguous arena range and a private candidate region of wcap records
    if ((e = launch_scan(c, S, t, k, io.A, io.alen, io.dlen))) return e;
    if (route_hook && (e = route_hook())) return e;
    if (mark(2)) return GM_E_HIP;
    // the continuation of overflowed candidate / survivor regions (a no-op launch otherwise)
    auto launch_direct = [&](const uint8_t *DA, uint64_t dl, const gm_req *DR, const uint32_t *b2r, const Dedup &d,
                             const uint64_t *dlp) -> int {
        uint32_t *res = S->d_ccnt + W + scan_blocks, *cres = S->d_ccnt + 2 * W + scan_blocks;
#define GM_DIRECT(PKV) k_waf_direct<PKV><<<scan_blocks, SCAN_BLOCK, SCAN_LDS_BYTES, s>>>(DA, dl, DR, n, b2r, t, k.cand, k.wcap, \
            S->d_ccnt, res, cres, S->d_pairs, (uint32_t)S->cap_pairs, S->d_jobs, (uint32_t)S->cap_jobs, S->d_status, d, dlp)
        if (t.bloom_pk == BLOOM_PK_PERM) GM_DIRECT(BLOOM_PK_PERM);
        else if (t.bloom_pk == 1) GM_DIRECT(1);
        else if (t.bloom_pk == 2) GM_DIRECT(2);
        else GM_DIRECT(3);
#undef GM_DIRECT
        HIPCHK(c, hipGetLastError());
        return GM_OK;
    };
    auto launch_ctx = [&]() -> int {
        k_waf_ctx<<<scan_blocks, VER_BLOCK, 0, s>>>(k.cand, k.wcap, S->d_ccnt, W, t, S->d_surv, k.bcap, S->d_ccnt + W,
                                                    S->d_status, S->d_ccnt + 2 * W + scan_blocks);
        HIPCHK(c, hipGetLastError());
        return GM_OK;
    };
    auto launch_exact = [&](const uint8_t *XA, uint64_t xl, const gm_req *XR, const uint32_t *b2r, const Dedup &d,
                            const uint64_t *xlp) -> int {
        // persistent exact check: EXACT_BPC workgroups per CU, all resident
        k_waf_exact<<<k.exact_blocks, EXACT_BLOCK, 0, s>>>(XA, xl, XR, n, b2r, t, S->d_surv, k.bcap,
                                                           S->d_ccnt + W, scan_blocks, S->d_pairs, (uint32_t)S->cap_pairs,
                                                           S->d_jobs, (uint32_t)S->cap_jobs, S->d_status, d, xlp, k.xprof);
        HIPCHK(c, hipGetLastError());
        k_exact_prof<<<1, 256, 0, s>>>(k.xprof, k.exact_blocks, S->d_status);
        HIPCHK(c, hipGetLastError());
        return GM_OK;
    };
    if ((e = launch_ctx())) return e;
    // join: blk2rec, the verdicts and the zeroed counts are complete before the exact check
    if (join) HIPCHK(c, hipStreamWaitEvent(s, S->ev_join, 0));
    if ((e = launch_exact(io.A, io.alen, io.reqs, io.blk2rec, dd, io.dlen))) return e;
    if ((e = launch_direct(io.A, io.alen, io.reqs, io.blk2rec, dd, io.dlen))) return e;
    if (mark(3)) return GM_E_HIP;
    if (t.n_sig_regex) {
        k_waf_regex<<<(uint32_t)c->cu_count * 4, 256, 0, s>>>(io.A, io.reqs, t, S->d_jobs, (uint32_t)S->cap_jobs, S->d_pairs,
                                                               (uint32_t)S->cap_pairs, dd);
        HIPCHK(c, hipGetLastError());
    }
    if ((e = launch_always(c, s, g, io.A, io.alen, io.reqs, n, S, dd, false, io.dlen))) return e;
    if (!t.decoders) return GM_OK;
    // ---- the request parsers' decoded views (gm_decode.inc): shadow records, same indices,
    // then the WAF stages once more over them; hits land in the same dedupe set and counts
    const size_t scap = 2 * (size_t)io.alen + 32 * (size_t)n + 4096;   // a view <= 2x its zones
    const uint32_t snblk = (uint32_t)((scap >> BLK_SHIFT) + 1);
    if ((e = grow(c, s, S->d_sreqs, S->cap_sreqs, (size_t)n))) return e;
    if ((e = grow(c, s, S->d_sarena, S->cap_sarena, scap))) return e;
    if ((e = grow(c, s, S->d_sblk, S->cap_sblk, snblk))) return e;
    if ((e = grow(c, s, S->d_ssize, S->cap_ssize, (size_t)n + 2))) return e;
    if ((e = grow(c, s, S->d_sbase, S->cap_sbase, (size_t)n + 2))) return e;
    size_t dtmp = 0;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, dtmp, S->d_ssize, S->d_sbase, (int)n + 1, s));
    if ((e = grow(c, s, S->d_stemp, S->cap_stemp, dtmp))) return e;
    const uint32_t dblocks = (n + 255) / 256;
    k_dec_size<<<dblocks, 256, 0, s>>>(io.reqs, io.A, n, t, io.out, S->d_ssize);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(S->d_stemp, dtmp, S->d_ssize, S->d_sbase, (int)n + 1, s));
    uint64_t *slen = S->d_sbase + n + 1;   // the shadow arena's length, on the device
    k_dec_emit<<<dblocks, 256, 0, s>>>(io.reqs, io.A, n, t, io.out, S->d_sbase, S->d_sreqs, S->d_sarena, scap,
                                       S->d_sblk, snblk, slen, S->d_status);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemsetAsync(S->d_status + 2, 0, 4, s));   // the job list restarts (pairs continue)
    k_status_pass<<<1, 64, 0, s>>>(S->d_status);   // the continuations restart too
    HIPCHK(c, hipGetLastError());
    Dedup dd2 = dd;
    dd2.jepoch = dd.epoch + 1;
    const uint8_t *SA = S->d_sarena;
    const gm_req *SR = S->d_sreqs;
    if ((e = launch_scan(c, S, t, k, SA, scap, slen))) return e;
    if ((e = launch_ctx())) return e;
    if ((e = launch_exact(SA, scap, SR, S->d_sblk, dd2, slen))) return e;
    if ((e = launch_direct(SA, scap, SR, S->d_sblk, dd2, slen))) return e;
    if (t.n_sig_regex) {
        k_waf_regex<<<(uint32_t)c->cu_count * 4, 256, 0, s>>>(SA, SR, t, S->d_jobs, (uint32_t)S->cap_jobs, S->d_pairs,
                                                               (uint32_t)S->cap_pairs, dd2);
        HIPCHK(c, hipGetLastError());
    }
    return launch_always(c, s, g, SA, scap, SR, n, S, dd2, true, slen);
}

// hit emission: offsets by an exclusive scan of the per-request counts (request order), the
// pairs into their slots, each request's ids sorted (continuation: remap / redo / np1, see
// k_hits_scatter)
// the stream's per-request bitmaps: redo bits, then hold bits (Dedup::redo, Dedup::hold)
static size_t redo_words(uint32_t n) { return ((size_t)n + 31) / 32; }
static int emit_hits(gm_ctx *c, Scratch *S, const Generation *g, uint32_t n, gm_verdict *out, uint32_t *hit_ids,
                     size_t hit_cap, unsigned long long *ctr, const Dedup &dd, const uint32_t *redo, uint32_t np1,
                     const uint32_t *remap, const unsigned long long *spill = nullptr, uint32_t nspill = 0,
                     bool cont = false) {
    hipStream_t s = S->stream;
    size_t scan_tmp = 0;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, S->d_cnt, S->d_start, (int)n + 1, s));
    if (int e = grow(c, s, S->d_temp, S->cap_temp, scan_tmp)) return e;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(S->d_temp, scan_tmp, S->d_cnt, S->d_start, (int)n + 1, s));
    k_hits_scatter<<<(uint32_t)c->cu_count * 4, 256, 0, s>>>(S->d_pairs, (uint32_t)S->cap_pairs, S->d_cnt, S->d_start,
                                                              hit_ids, hit_cap, ctr, g->tab.n_locs, S->d_status, dd,
                                                              redo, np1, remap, spill, nspill);
    HIPCHK(c, hipGetLastError());
    k_hits_finalize<<<std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, (uint32_t)c->cu_count * 8)), 256, 0, s>>>(
        S->d_start, n, out, hit_ids, hit_cap, S->d_status, S->d_redo, S->d_redo + redo_words(n), cont ? 1u : 0u);
    HIPCHK(c, hipGetLastError());
    return GM_OK;
}

// the entries of the spill a batch may fill (the whole buffer, or 2^-k of it under the
// GM_CREATE_SPILL_SHIFT(k) test hook): the count word can run past it, the entries cannot
static size_t spill_cap_of(const gm_ctx *c, const Scratch *S) {
    return c->spill_shift ? std::min<size_t>(std::max<size_t>(S->cap_spill >> c->spill_shift, 16), S->cap_spill)
                          : S->cap_spill;
}

static int run_batch(gm_ctx *c, Scratch *S, const Generation *g, const gm_req *reqs, const uint8_t *A, uint64_t alen,
                     uint32_t n, gm_verdict *out, uint32_t *hit_ids, size_t hit_cap, const uint64_t *dlen, uint32_t slot) {
    hipStream_t s = S->stream;
    const GTab &t = g->tab;
    const bool waf = t.n_sigs > 0 && (t.n_lits > 0 || t.n_sig_regex > 0);
    const uint32_t nblk = (uint32_t)((alen >> BLK_SHIFT) + 1);
#define GM_ROUTE_LAUNCH(W, RKV, TAILV, GRID, LDS, STRM, ...) \
    k_route<W, RKV, TAILV><<<GRID, ROUTE_BLOCK, LDS, STRM>>>(__VA_ARGS__)
    const bool prof = c->flags & GM_CREATE_PROFILE;
    auto mark = [&](int k) -> int {
        if (prof) { HIPCHK(c, hipEventRecord(S->ev[k], s)); S->ev_used = k + 1; S->ev_pending = true; }
        return GM_OK;
    };
    S->ev_used = 0;
    S->route_side = false;
    HIPCHK(c, hipMemsetAsync(S->d_status, 0, BATCH_STATUS_WORDS * 4, s));
    // the batch's counters accumulate apart and are committed by k_ctr_commit at the end
    const size_t nctr = std::max<size_t>(g->n_counters, 1);
    if (int e0 = grow(c, s, S->d_bctr, S->cap_bctr, nctr)) return e0;
    HIPCHK(c, hipMemsetAsync(S->d_bctr, 0, nctr * 8, s));
    auto commit = [&]() -> int {
        k_ctr_commit<<<std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)((nctr + 255) / 256), (uint32_t)c->cu_count)), 256, 0, s>>>(
            S->d_bctr, g->d_counters, (uint32_t)g->n_counters, S->d_status, S->d_ovlog + slot);
        HIPCHK(c, hipGetLastError());
        return GM_OK;
    };
    if (mark(0)) return GM_E_HIP;
#ifndef GM_SLOW_WPE
#define GM_SLOW_WPE 3   // the SLOW route pass's waves per SIMD target (its header walks are latency-bound)
#endif
#ifndef GM_SOLO_WPE
// the FAST route pass's waves per SIMD target without a WAF phase (C1 / C2 / C5).  Measured (round 6,
// ms per 10M): 4 -> C2 4.89 / C1 0.490 / C5 1.317 against 4.90 / 0.491 / 1.331 at 3 (noise); 5 -> C1
// 0.477 but C2 5.28 (no 16-word long-host path at 5) and C5 1.348
#define GM_SOLO_WPE 3
#endif
    const uint32_t route_blocks = std::max<uint32_t>(1, std::min<uint32_t>((n + ROUTE_BLOCK - 1) / ROUTE_BLOCK,
                                                                           (uint32_t)c->cu_count * GM_EXP_GRIDMUL));
    unsigned long long *ctr = S->d_bctr;
    // prefiltered regex locations: k_route defers their step to k_rloc (a tile of requests per
    // workgroup, gm_rloc.inc) and a second k_route pass over the deferred list finishes them
    RlocQ q{};
    const bool rk = t.rk_keys || t.n_rsl;
    if (rk) {
        int e2;
        if ((e2 = grow(c, s, S->d_rq, S->cap_rq, n)) || (e2 = grow(c, s, S->d_rql, S->cap_rql, n)) ||
            (e2 = grow(c, s, S->d_rqs, S->cap_rqs, n)) || (e2 = grow(c, s, S->d_rqb, S->cap_rqb, n)) ||
            (e2 = grow(c, s, S->d_rqm, S->cap_rqm, n)) || (e2 = grow(c, s, S->d_rqu, S->cap_rqu, 2 * (size_t)n + 1))) return e2;
        q = RlocQ{S->d_rq, S->d_status + RLOC_STATUS_WORD, S->d_rql, S->d_rqs, S->d_rqb, S->d_rqu};
    }
    // the first (FAST) route pass lists the requests that need an out-of-line step; the SLOW pass
    // routes them (the RK passes keep their calls in line)
    RlocQ qs{};
    if (!rk) {
        if (int e2 = grow(c, s, S->d_slow, S->cap_slow, n)) return e2;
        qs.list = S->d_slow; qs.count = S->d_status + SLOW_STATUS_WORD;
    }
    auto launch_rloc = [&](hipStream_t rs, uint32_t tail_blocks) -> int {
        // union-DFA slices of the servers that have them (config order: a request answered by one
        // slice skips the later ones), then the factor prefilter for the others
        if (t.n_rsl) {
            HIPCHK(c, hipMemsetAsync(q.loc, 0xFF, (size_t)n * 4, rs));
            // the factor masks of the prefiltered slices' requests (gm_rloc.inc k_rloc_pref)
            const unsigned long long *pm = nullptr;
            const size_t pref_lds = 4u * RK_BLOOM_WORDS + sizeof(DRlocKey) * ((size_t)t.rk_mask + 1) +
                                    sizeof(PrefEnt) * (size_t)g->hdr.n_rk_ents_n;
            if (GM_RLOC_PREF && g->stats.n_rsl_pref && pref_lds <= RLOC_PREF_LDS) {
                k_rloc_pref<<<(uint32_t)c->cu_count, 1024, pref_lds, rs>>>(A, alen, t, q.st, q.count, S->d_rqm,
                                                                              dlen, g->hdr.n_rk_ents_n);
                HIPCHK(c, hipGetLastError());
                pm = S->d_rqm;
            }
            const DAlwSlice *sls = reinterpret_cast<const DAlwSlice *>(g->host_image.data() + g->hdr.off_alw_slices);
            // the anchored slices' candidate lists (k_rloc_heads): each such slice runs over its list
            const uint32_t nh = g->hdr.n_rsl_heads;
            if (nh) {
                int e5;
                if ((e5 = grow(c, rs, S->d_hlist, S->cap_hlist, (size_t)nh * n)) ||
                    (e5 = grow(c, rs, S->d_hcnt, S->cap_hcnt, (size_t)RSL_HEADS_MAX))) return e5;
                HIPCHK(c, hipMemsetAsync(S->d_hcnt, 0, (size_t)nh * 4, rs));
                for (uint32_t h0 = 0; h0 < nh; h0 += HEADS_LDS_SLOTS) {
                    const uint32_t k = std::min<uint32_t>(HEADS_LDS_SLOTS, nh - h0);
                    k_rloc_heads<<<(uint32_t)c->cu_count, 1024, k * RSL_HEAD_WORDS * 4, rs>>>(
                        A, t, q.st, q.u, q.count, t.rsl_head_slice, h0, k, S->d_hlist, n, S->d_hcnt);
                    HIPCHK(c, hipGetLastError());
                }
                static const bool trace_heads = getenv("GM_TRACE_HEADS") != nullptr;
                if (trace_heads) {   // (diagnostics, GM_TRACE_HEADS=1: the candidate lists' lengths)
                    std::vector<uint32_t> hc(nh);
                    HIPCHK(c, hipMemcpyAsync(hc.data(), S->d_hcnt, nh * 4, hipMemcpyDeviceToHost, rs));
                    HIPCHK(c, hipStreamSynchronize(rs));
                    fprintf(stderr, "[heads] n=%u:", n);
                    for (uint32_t h = 0; h < nh; h++) fprintf(stderr, " %u", hc[h]);
                    fprintf(stderr, "\n");
                }
            }
            for (uint32_t k = t.n_alw_slices; k < t.n_alw_slices + t.n_rsl; k++) {
                const dim3 grid((uint32_t)c->cu_count), blk(1024);
                const bool hl = nh && (sls[k].flags & ALW_SLICE_HEADS);
                const uint32_t slot = (sls[k].flags >> 16) & 0xFFu;
                const uint32_t *L = hl ? S->d_hlist + (size_t)slot * n : nullptr;
                const uint32_t *LC = hl ? S->d_hcnt + slot : nullptr;
                switch (sls[k].n_groups) {
                case 1: k_rloc_multi<1><<<grid, blk, sls[k].len, rs>>>(A, alen, t, q.st, q.u, q.count, q.loc, dlen, k, pm, L, LC); break;
                case 2: k_rloc_multi<2><<<grid, blk, sls[k].len, rs>>>(A, alen, t, q.st, q.u, q.count, q.loc, dlen, k, pm, L, LC); break;
                case 3: k_rloc_multi<3><<<grid, blk, sls[k].len, rs>>>(A, alen, t, q.st, q.u, q.count, q.loc, dlen, k, pm, L, LC); break;
                case 4: k_rloc_multi<4><<<grid, blk, sls[k].len, rs>>>(A, alen, t, q.st, q.u, q.count, q.loc, dlen, k, pm, L, LC); break;
                case 5: k_rloc_multi<5><<<grid, blk, sls[k].len, rs>>>(A, alen, t, q.st, q.u, q.count, q.loc, dlen, k, pm, L, LC); break;
                case 6: k_rloc_multi<6><<<grid, blk, sls[k].len, rs>>>(A, alen, t, q.st, q.u, q.count, q.loc, dlen, k, pm, L, LC); break;
                case 7: k_rloc_multi<7><<<grid, blk, sls[k].len, rs>>>(A, alen, t, q.st, q.u, q.count, q.loc, dlen, k, pm, L, LC); break;
                default: k_rloc_multi<8><<<grid, blk, sls[k].len, rs>>>(A, alen, t, q.st, q.u, q.count, q.loc, dlen, k, pm, L, LC); break;
                }
                HIPCHK(c, hipGetLastError());
            }
            k_rloc_fin<<<(uint32_t)c->cu_count * 4, 256, 0, rs>>>(t, q.list, q.count, q.loc);
            HIPCHK(c, hipGetLastError());
        }
        if (t.n_rk_prefilter)
            k_rloc<<<(uint32_t)c->cu_count * 4, RLOC_BLOCK, 0, rs>>>(reqs, A, alen, t, q.list, q.count, q.loc, dlen);
        GM_ROUTE_LAUNCH(3, true, true, tail_blocks, route_lds(t, false), rs, reqs, n, A, alen, t, out, ctr, nullptr, nblk,
                        nullptr, 0, dlen, route_hist_n(t, false), q);
        HIPCHK(c, hipGetLastError());
        return GM_OK;
    };
    if (!waf) {
        if (rk) GM_ROUTE_LAUNCH(3, true, false, route_blocks, route_lds(t, false), s, reqs, n, A, alen, t, out, ctr, nullptr, nblk, nullptr, 0, dlen, route_hist_n(t, false), q);
        else {
            GM_ROUTE_LAUNCH(GM_SOLO_WPE, false, false, route_blocks, route_lds(t, false), s, reqs, n, A, alen, t, out, ctr, nullptr, nblk, nullptr, 0, dlen, route_hist_n(t, false), qs);
            HIPCHK(c, hipGetLastError());
            k_route<GM_SLOW_WPE, false, false, true><<<route_blocks, ROUTE_BLOCK, route_lds(t, false), s>>>(
                reqs, n, A, alen, t, out, ctr, nullptr, nblk, nullptr, 0, dlen, route_hist_n(t, false), qs);
        }
        HIPCHK(c, hipGetLastError());
        if (rk) {
            const int e4 = launch_rloc(s, route_blocks);
            if (e4) return e4;
        }
        if (int e5 = commit()) return e5;
        return mark(1) ? GM_E_HIP : GM_OK;
    }
    int e;
    WafCaps k{};
    if ((e = waf_buffers(c, S, alen, n, k))) return e;
    if ((e = grow(c, s, S->d_blk2rec, S->cap_blk, nblk))) return e;
    if ((e = grow(c, s, S->d_redo, S->cap_redo, 2 * redo_words(n)))) return e;
    HIPCHK(c, hipMemsetAsync(S->d_redo, 0, 2 * redo_words(n) * 4, s));
    // one epoch per batch (two with decoders: the decoded pass's jobs take epoch + 1)
    if ((e = next_epoch(c, S, t))) return e;
    const size_t spill_cap = spill_cap_of(c, S);
    Dedup dd{S->d_set, (uint32_t)(S->cap_set - 1), S->epoch, S->epoch, out, S->d_cnt, S->d_status, S->d_redo,
             S->d_spill, (uint32_t)std::min<size_t>(spill_cap, 0xFFFFFFFFu), S->d_redo + redo_words(n)};

    // ---- fork: k_route on the side stream, beside the WAF scan (independent inputs; its waves
    // fit beside the scan's one workgroup per CU; issued after the scan so the scan claims the
    // CUs first).  It writes the verdicts, the location counters, blk2rec and zeroes the counts.
    // GM_CREATE_SERIAL (measurement): the route alone first, on the caller's stream.
    const bool serial = c->flags & GM_CREATE_SERIAL;
    hipStream_t rs = serial ? s : S->side;
#ifndef GM_ROUTE_BPC
#define GM_ROUTE_BPC 1   // route blocks per CU beside the scan (round 4, the call-free route: 1: 4.91,
                         // 2: 5.09 ms per C4 step; before it, 1: 5.86, 2: 5.41, 3: 5.60)
#endif
#ifndef GM_ROUTE_PRIO
#define GM_ROUTE_PRIO 0  // 1: the route at raised issue priority beside the scan (5.32 vs 5.06 ms per C4 step)
#endif
    if (!serial) {
        HIPCHK(c, hipEventRecord(S->ev_fork, s));
        HIPCHK(c, hipStreamWaitEvent(S->side, S->ev_fork, 0));
    }
    auto launch_route = [&]() -> int {
        // beside the scan, GM_ROUTE_BPC route blocks per CU (more steal issue slots from the scan)
        const uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>((n + ROUTE_BLOCK - 1) / ROUTE_BLOCK,
                                                                     (uint32_t)c->cu_count * (serial ? 8 : GM_ROUTE_BPC)));
        if (prof) HIPCHK(c, hipEventRecord(S->ev_route[0], rs));
        if (rk)
            GM_ROUTE_LAUNCH(GM_ROUTE_WPE, true, false, nb, route_lds(t, !serial), rs, reqs, n, A, alen, t, out, ctr, S->d_blk2rec, nblk, S->d_cnt, GM_ROUTE_PRIO, dlen, route_hist_n(t, !serial), q);
        else {
            GM_ROUTE_LAUNCH(GM_ROUTE_WPE, false, false, nb, route_lds(t, !serial), rs, reqs, n, A, alen, t, out, ctr, S->d_blk2rec, nblk, S->d_cnt, GM_ROUTE_PRIO, dlen, route_hist_n(t, !serial), qs);
            HIPCHK(c, hipGetLastError());
            k_route<GM_ROUTE_WPE, false, false, true><<<nb, ROUTE_BLOCK, route_lds(t, !serial), rs>>>(
                reqs, n, A, alen, t, out, ctr, S->d_blk2rec, nblk, S->d_cnt, GM_ROUTE_PRIO, dlen, route_hist_n(t, !serial), qs);
        }
        HIPCHK(c, hipGetLastError());
        int e3;
        if (rk && (e3 = launch_rloc(rs, nb))) return e3;
        if (prof) HIPCHK(c, hipEventRecord(S->ev_route[1], rs));
        if (!serial) HIPCHK(c, hipEventRecord(S->ev_join, rs));
        S->route_side = true;
        return GM_OK;
    };
    if (serial && (e = launch_route())) return e;
    if (mark(1)) return GM_E_HIP;
    const WafIO io{A, alen, dlen, reqs, n, out, S->d_blk2rec, nblk};
    if ((e = waf_stages(c, S, g, k, io, dd, serial ? std::function<int()>() : std::function<int()>(launch_route), !serial,
                        mark))) return e;
    // ---- hit emission: offsets by an exclusive scan of the per-request counts (request order)
    if ((e = emit_hits(c, S, g, n, out, hit_ids, hit_cap, ctr, dd, nullptr, 0, nullptr))) return e;
    if ((e = commit())) return e;
    if (mark(4)) return GM_E_HIP;
    return GM_OK;
}

// A batch's record on its stream until gm_sync completes it: the arguments, for the dedupe set's
// continuation (the stream's last batch: only the requests with a refused insert are redone) or a
// whole re-run (an earlier batch of the stream, whose scratch later batches have reused)
static int enqueue_batch(gm_ctx *c, Scratch *S, const Generation *g, const Scratch::Replay &rp) {
    return run_batch(c, S, g, rp.reqs, rp.A, rp.alen, rp.n, rp.out, rp.hits, rp.hit_cap, rp.dlen, rp.slot);
}

// GM_TRACE_SYNC=1 (environment): gm_sync's phases with host timestamps on stderr (diagnostics)
static bool trace_sync() {
    static const bool on = getenv("GM_TRACE_SYNC") != nullptr;
    return on;
}
static void trace(const char *what) {
    if (!trace_sync()) return;
    static auto t0 = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "[gm_sync %10.3f ms] %s\n", ms, what);
}

// GM_BATCH_HOST: the staged verdicts and hits back to the caller's host buffers
static int copy_back(gm_ctx *c, Scratch *S, const Scratch::Replay &rp) {
    if (!rp.h_out) return GM_OK;
    HIPCHK(c, hipMemcpyAsync(rp.h_out, rp.out, (size_t)rp.n * sizeof(gm_verdict), hipMemcpyDeviceToHost, S->stream));
    if (rp.h_hits && rp.h_hit_cap)
        HIPCHK(c, hipMemcpyAsync(rp.h_hits, rp.hits, rp.h_hit_cap * 4, hipMemcpyDeviceToHost, S->stream));
    return GM_OK;
}

// read the stream's status words (and the pending batches' overflow words) to the host
static int read_status(gm_ctx *c, Scratch *S) {
    HIPCHK(c, hipMemcpyAsync(S->h_status, S->d_status, STATUS_WORDS * 4, hipMemcpyDeviceToHost, S->stream));
    HIPCHK(c, hipMemcpyAsync(S->h_ovlog, S->d_ovlog, PENDING_MAX * 4, hipMemcpyDeviceToHost, S->stream));
    HIPCHK(c, hipStreamSynchronize(S->stream));
    return GM_OK;
}

// a batch whose dedupe set overflowed, re-run whole with the set doubled until it fits (a stream's
// earlier batch, or the rare case a continuation cannot take): ov = its final overflow bits
static int rerun_whole(gm_ctx *c, Scratch *S, const Scratch::Replay &rp0, uint32_t &ov) {
    Scratch::Replay rp = rp0;
    rp.slot = 0;
    for (;;) {
        if (S->list_mult >= 64) return GM_OK;   // at its largest: ov keeps OV_SET, reported by the caller
        S->list_mult *= 2;
        std::shared_lock<std::shared_mutex> lk(c->gen_mu);
        if (c->gen != rp.gen || c->publish_seq != rp.seq)
            return fail(c, GM_E_OVERFLOW, "WAF dedupe set full and the generation changed before the batch could be "
                                          "re-run: retry it");
        c->n_set_reruns++;
        DoneGuard G(S);
        int e = enqueue_batch(c, S, c->gen, rp);
        if (e || (e = copy_back(c, S, rp)) || (e = G.done(c))) return e;
        lk.unlock();
        if ((e = read_status(c, S))) return e;
        ov = S->h_ovlog[0];
        if (!ov_held(ov)) return GM_OK;
    }
}

// the first nspill spilled pairs sorted into d_spill2 and each distinct one counted for its request
// (those of a redone request, redo's bits, skipped): out = the sorted array
static int sort_spill(gm_ctx *c, Scratch *S, uint32_t nspill, const uint32_t *redo, const Dedup &dd,
                      unsigned long long *&out) {
    hipStream_t s = S->stream;
    int e;
    if ((e = grow(c, s, S->d_spill2, S->cap_spill2, (size_t)nspill))) return e;
    size_t tmp = 0;
    HIPCHK(c, hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, S->d_spill, S->d_spill2, (int)nspill, 0, 64, s));
    if ((e = grow(c, s, S->d_rtemp, S->cap_rtemp, tmp))) return e;
    HIPCHK(c, hipcub::DeviceRadixSort::SortKeys(S->d_rtemp, tmp, S->d_spill, S->d_spill2, (int)nspill, 0, 64, s));
    k_spill_count<<<std::min<uint32_t>((nspill + 255) / 256, (uint32_t)c->cu_count * 4), 256, 0, s>>>(S->d_spill2, nspill,
                                                                                                        redo, S->d_cnt, dd);
    HIPCHK(c, hipGetLastError());
    out = S->d_spill2;
    return GM_OK;
}

// The dedupe set of the stream's last batch refused pairs, and the spill took them all (OV_SET
// without OV_SPILL; no refused job lost to an overflowing job list): the batch's answer is exact
// with the spill's distinct pairs added -- sorted, counted, emitted after the pair list.  No WAF
// stage runs again.
static int spill_continuation(gm_ctx *c, Scratch *S, const Scratch::Replay &rp, uint32_t &ov, bool &done) {
    done = false;
    hipStream_t s = S->stream;
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    if (c->gen != rp.gen || c->publish_seq != rp.seq)
        return fail(c, GM_E_OVERFLOW, "WAF dedupe set full and the generation changed before the batch could be "
                                      "completed: retry it");
    const Generation *g = c->gen;
    const uint32_t nspill = (uint32_t)std::min<size_t>(S->h_status[SPILL_WORD], spill_cap_of(c, S));
    int e;
    DoneGuard G(S);
    unsigned long long *sp = nullptr;
    const Dedup dd0{S->d_set, (uint32_t)(S->cap_set - 1), S->epoch, S->epoch + 1, rp.out, S->d_cnt, S->d_status, nullptr,
                    nullptr, 0u};
    if (nspill && (e = sort_spill(c, S, nspill, nullptr, dd0, sp))) return e;
    k_clear_held<<<1, 64, 0, s>>>(S->d_status);
    HIPCHK(c, hipGetLastError());
    if ((e = emit_hits(c, S, g, rp.n, rp.out, rp.hits, rp.hit_cap, S->d_bctr, dd0, nullptr, 0, nullptr, sp, nspill, true)))
        return e;
    const size_t nctr = std::max<size_t>(g->n_counters, 1);
    k_ctr_commit<<<std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)((nctr + 255) / 256), (uint32_t)c->cu_count)), 256, 0, s>>>(
        S->d_bctr, g->d_counters, (uint32_t)g->n_counters, S->d_status, S->d_ovlog + rp.slot);
    HIPCHK(c, hipGetLastError());
    if ((e = copy_back(c, S, rp))) return e;
    if ((e = G.done(c))) return e;
    lk.unlock();
    if ((e = read_status(c, S))) return e;
    trace("spill continuation: emitted");
    c->last_spill = nspill;
    ov = S->h_ovlog[rp.slot];
    done = true;
    return GM_OK;
}

// The dedupe set of the stream's last batch overflowed (OV_SET): only the requests with a refused
// insert are redone (k_redo_*), as a sub-batch of their WAF zones through the same stages with a
// set twice as large (doubled again while it overflows), and the emission merges both passes.
// The first pass left its pairs in [0, np1), its counts, the route's verdicts and location counters
// (k_hits_scatter / k_hits_finalize / k_ctr_commit held back on OV_SET).  done = false: the
// continuation does not apply (the caller re-runs the batch whole).
static int set_continuation(gm_ctx *c, Scratch *S, const Scratch::Replay &rp, uint32_t ov1, uint32_t &ov, bool &done) {
    done = false;
    hipStream_t s = S->stream;
    if (ov1 & (OV_PAIRS | OV_HITS | OV_DEC)) return GM_OK;   // the first pass's lists are incomplete / void
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    if (c->gen != rp.gen || c->publish_seq != rp.seq)
        return fail(c, GM_E_OVERFLOW, "WAF dedupe set full and the generation changed before the batch could be "
                                      "completed: retry it");
    const Generation *g = c->gen;
    const GTab &t = g->tab;
    const uint32_t n = rp.n;
    const uint32_t np1 = S->h_status[1];
    const uint32_t nspill = (uint32_t)std::min<size_t>(S->h_status[SPILL_WORD], spill_cap_of(c, S));
    int e;
    DoneGuard G(S);
    // the requests to redo
    if ((e = grow(c, s, S->d_rlist, S->cap_rlist, (size_t)n))) return e;
    HIPCHK(c, hipMemsetAsync(S->d_status + REDO_STATUS_WORD, 0, 4, s));
    k_redo_list<<<(uint32_t)c->cu_count * 4, 256, 0, s>>>(S->d_redo, n, S->d_rlist, S->d_cnt, S->d_status + REDO_STATUS_WORD);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(S->h_status + REDO_STATUS_WORD, S->d_status + REDO_STATUS_WORD, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const uint32_t m = S->h_status[REDO_STATUS_WORD];
    trace("continuation: requests listed");
    if (m == 0 || m > n) { G.armed = false; return mark_done(c, S); }
    c->last_redo = m;
    // their zones gathered into a sub-batch
    if ((e = grow(c, s, S->d_rsize, S->cap_rsize, (size_t)m + 1)) || (e = grow(c, s, S->d_rbase, S->cap_rbase, (size_t)m + 1)))
        return e;
    size_t tmp = 0;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, S->d_rsize, S->d_rbase, (int)m + 1, s));
    if ((e = grow(c, s, S->d_rtemp, S->cap_rtemp, tmp))) return e;
    k_redo_size<<<(m + 255) / 256, 256, 0, s>>>(rp.reqs, S->d_rlist, m, S->d_rsize);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(S->d_rtemp, tmp, S->d_rsize, S->d_rbase, (int)m + 1, s));
    uint64_t sub_len = 0;
    HIPCHK(c, hipMemcpyAsync(&sub_len, S->d_rbase + m, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    trace("continuation: sub-batch sized");
    const uint32_t snblk = (uint32_t)((sub_len >> BLK_SHIFT) + 1);
    if ((e = grow(c, s, S->d_rsreq, S->cap_rsreq, (size_t)m)) || (e = grow(c, s, S->d_rsarena, S->cap_rsarena, sub_len + 1024)) ||
        (e = grow(c, s, S->d_rsout, S->cap_rsout, (size_t)m)) || (e = grow(c, s, S->d_rsblk, S->cap_rsblk, snblk)) ||
        (e = grow(c, s, S->d_rscnt, S->cap_rscnt, (size_t)m + 1)))
        return e;
    HIPCHK(c, hipMemsetAsync(S->d_rsarena + sub_len, 0, 1024, s));
    k_redo_emit<<<(m + 255) / 256, 256, 0, s>>>(rp.reqs, rp.A, rp.out, S->d_rlist, m, S->d_rbase, sub_len, S->d_rsreq,
                                                S->d_rsarena, S->d_rsout, S->d_rsblk, snblk);
    HIPCHK(c, hipGetLastError());
    // the first pass's spilled pairs of the requests not redone, sorted and counted now: the
    // sub-batch's buffers may reallocate the spill (waf_buffers), not its sorted copy
    unsigned long long *sp = nullptr;
    if (nspill) {
        // (the first pass's set: the pair epoch, its jobs' epochs taken as in use)
        const Dedup dd1{S->d_set, (uint32_t)(S->cap_set - 1), S->epoch, S->epoch + 1, rp.out, S->d_cnt, S->d_status,
                        nullptr, nullptr, 0u};
        if ((e = sort_spill(c, S, nspill, S->d_redo, dd1, sp))) return e;
    }
    const WafIO io{S->d_rsarena, sub_len, nullptr, S->d_rsreq, m, S->d_rsout, S->d_rsblk, snblk};
    const std::function<int(int)> nomark = [](int) { return GM_OK; };
    for (;;) {
        // a set twice the size that overflowed, fresh; the sub-batch's pairs follow the first pass's
        if (S->list_mult >= 64) { ov = OV_SET; G.armed = false; return mark_done(c, S); }
        S->list_mult *= 2;
        if ((e = grow(c, s, S->d_set, S->cap_set, 2 * S->cap_set))) return e;
        S->cap_set = (size_t)1 << (63 - __builtin_clzll(S->cap_set));   // (grow pads; the mask needs a power of two)
        S->epoch = 0;
        HIPCHK(c, hipMemsetAsync(S->d_set, 0, S->cap_set * 8, s));
        WafCaps k{};
        if ((e = waf_buffers(c, S, sub_len, m, k, np1))) return e;
        if ((e = next_epoch(c, S, t))) return e;
        k_redo_status<<<1, 64, 0, s>>>(S->d_status, np1);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemsetAsync(S->d_rscnt, 0, ((size_t)m + 1) * 4, s));
        c->n_set_reruns++;
        // (no spill in a redo pass: a refusal there is an overflow, and the pass re-runs larger)
        const Dedup dd{S->d_set, (uint32_t)(S->cap_set - 1), S->epoch, S->epoch, S->d_rsout, S->d_rscnt, S->d_status, nullptr,
                       nullptr, 0u};
        trace("continuation: sub-batch enqueued");
        if ((e = waf_stages(c, S, g, k, io, dd, std::function<int()>(), false, nomark))) return e;
        if ((e = read_status(c, S))) return e;
        trace("continuation: sub-batch done");
        const uint32_t ov2 = S->h_status[3] | S->h_status[PASS1_OV_WORD];
        if (ov2 & (OV_PAIRS | OV_DEC)) { G.armed = false; return mark_done(c, S); }   // whole re-run instead
        if (!ov_held(ov2)) break;
    }
    // merge: the sub-requests' counts, then the emission over the whole batch and the commit
    k_redo_merge<<<(m + 255) / 256, 256, 0, s>>>(S->d_rlist, m, S->d_rscnt, S->d_cnt);
    HIPCHK(c, hipGetLastError());
    const Dedup dd0{S->d_set, (uint32_t)(S->cap_set - 1), S->epoch, S->epoch, rp.out, S->d_cnt, S->d_status, nullptr,
                    nullptr, 0u};
    if ((e = emit_hits(c, S, g, n, rp.out, rp.hits, rp.hit_cap, S->d_bctr, dd0, S->d_redo, np1, S->d_rlist, sp,
                       nspill, true))) return e;
    const size_t nctr = std::max<size_t>(g->n_counters, 1);
    k_ctr_commit<<<std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)((nctr + 255) / 256), (uint32_t)c->cu_count)), 256, 0, s>>>(
        S->d_bctr, g->d_counters, (uint32_t)g->n_counters, S->d_status, S->d_ovlog + rp.slot);
    HIPCHK(c, hipGetLastError());
    if ((e = copy_back(c, S, rp))) return e;
    if ((e = G.done(c))) return e;
    lk.unlock();
    if ((e = read_status(c, S))) return e;
    trace("continuation: emitted");
    ov = S->h_ovlog[rp.slot];
    done = true;
    return GM_OK;
}

// Complete the stream's pending batches (gm_sync): overflow bits per batch, OV_SET batches
// completed (the last by the continuation, earlier ones re-run whole), errors reported.
static int sync_pending(gm_ctx *c, Scratch *S) {
    int e;
    trace("sync: start");
    if ((e = read_status(c, S))) return e;
    trace("sync: pending batches done");
    {
        std::lock_guard<std::mutex> lk(c->last_mu);
        memcpy(c->last_status, S->h_status, STATUS_WORDS * 4);
        c->last_candidates = S->h_status[6];
        c->last_ctx_pass = S->h_status[7];
        c->last_jobs = S->h_status[2];
        c->last_pairs = S->h_status[1];
        c->last_hits = S->h_status[4];
        if (S->ev_pending) {
            for (int k = 0; k < 4; k++) {
                c->last_ms[k] = 0;
                if (k + 1 < S->ev_used) (void)hipEventElapsedTime(&c->last_ms[k], S->ev[k], S->ev[k + 1]);
            }
            // stage 0 = the route on the side stream (its own time); stage 1 = the scan
            if (S->route_side) (void)hipEventElapsedTime(&c->last_ms[0], S->ev_route[0], S->ev_route[1]);
            S->ev_pending = false;
        }
    }
    const uint32_t parse_ov = S->h_status[PARSE_STATUS_WORD + 3], upuri_ov = S->h_status[UPURI_STATUS_WORD];
    std::vector<Scratch::Replay> pend;
    pend.swap(S->pending);
    const bool last_in_place = S->last_is_batch;
    S->last_is_batch = false;
    uint32_t any = 0;
    for (const auto &rp : pend) any |= S->h_ovlog[rp.slot];
    // the next batch on this stream gets twice the buffer that overflowed (bounded)
    if ((any & OV_CAND) && S->cand_mult < 64) S->cand_mult *= 2;
    if ((any & OV_SURV) && S->surv_mult < 64) S->surv_mult *= 2;
    if ((any & (OV_PAIRS | OV_JOBS)) && S->list_mult < 64) S->list_mult *= 2;
    std::vector<uint32_t> ovs(pend.size());
    for (size_t i = 0; i < pend.size(); i++) ovs[i] = S->h_ovlog[pend[i].slot];
    uint32_t err = 0;
    // the last batch first: its scratch (pairs, counts, redo bits) is still in place
    for (size_t i = pend.size(); i-- > 0;) {
        uint32_t ov = ovs[i];
        if (ov_held(ov)) {
            bool done = false;
            if (i + 1 == pend.size() && last_in_place) {
                // refused pairs all in the spill: emitted from it; else the requests whose pairs the
                // spill missed, or whose refused jobs a full job list lost, are redone
                const bool redo = (ov & OV_SPILL) || ((ov & OV_JSET) && (ov & OV_JOBS));
                e = redo ? set_continuation(c, S, pend[i], ov, ov, done) : spill_continuation(c, S, pend[i], ov, done);
                if (e) return e;
            }
            if (!done && (e = rerun_whole(c, S, pend[i], ov))) return e;
            if (i + 1 == pend.size()) {
                std::lock_guard<std::mutex> lk(c->last_mu);
                c->last_hits = S->h_status[4];
            }
        }
        ovs[i] = ov;
        err |= ov;
    }
    // (the same conditions as the batch-void errors below, per batch)
    for (uint32_t ov : ovs) S->sync_log.push_back((ov & (OV_HITS | OV_DEC)) || ov_held(ov) ? GM_E_OVERFLOW : GM_OK);
    if (parse_ov) return fail(c, GM_E_OVERFLOW, "gm_parse_requests: arena capacity exceeded");
    if (upuri_ov) return fail(c, GM_E_OVERFLOW, "gm_upstream_uris: output capacity exceeded");
    if (err & OV_HITS) return fail(c, GM_E_OVERFLOW, "hit_ids capacity exceeded (the batch's counters were not committed)");
    // candidate / survivor / pair / job overflows were completed on the device (k_waf_direct, the
    // set-based scatter and regex runs): the batch is whole, the buffers grow for speed
    if (ov_held(err)) return fail(c, GM_E_OVERFLOW, "WAF dedupe set full at its largest size (64x: > ~380 unique hits + "
                                                    "regex jobs per request); the batch's counters were not committed");
    if (err & OV_DEC) return fail(c, GM_E_OVERFLOW, "decoded-view arena capacity exceeded");
    return GM_OK;
}

int gm_match_batch(gm_ctx *c, const gm_batch *in, gm_verdict *out, uint32_t *hit_ids, size_t hit_cap, void *stream) {
    if (!c || !in || !out) return fail(c, GM_E_INVAL, "null argument");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    HIPCHK(c, hipSetDevice(c->dev));
    hipStream_t s = (hipStream_t)stream;
    Scratch *S = scratch_for(c, s);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    // the stream's pending batches are recorded until gm_sync; past PENDING_MAX unsynced batches the
    // oldest are completed here first (synchronously), so no batch's overflow goes unreported
    if (S->pending.size() >= PENDING_MAX) {
        const int e0 = sync_pending(c, S);
        if (e0 == GM_E_OVERFLOW)
            return fail(c, GM_E_EARLIER, "an earlier batch of this stream completed void in the forced sync (" +
                                         t_err + "); this batch was not enqueued");
        if (e0) return e0;
    }
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    const Generation *g = c->gen;
    if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
    S->last_is_batch = false;
    if (in->n == 0) { HIPCHK(c, hipMemsetAsync(S->d_status, 0, BATCH_STATUS_WORDS * 4, s)); S->ev_pending = false; return GM_OK; }
    if (((uintptr_t)in->arena & 15) || ((uintptr_t)in->reqs & 15) || ((uintptr_t)out & 15))
        return fail(c, GM_E_INVAL, "reqs / arena / out must be 16-byte aligned");
    if (in->arena_len >> SURV_POS_BITS) return fail(c, GM_E_INVAL, "arena_len must be below 512 GiB");
    if (hit_cap > 0xFFFFFFFFull) hit_cap = 0xFFFFFFFFull;   // hit offsets are u32
    DoneGuard G(S);
    Scratch::Replay rp;
    rp.gen = g; rp.seq = c->publish_seq; rp.n = in->n; rp.alen = in->arena_len;
    rp.slot = (uint32_t)S->pending.size();
    if (!(in->flags & GM_BATCH_HOST)) {
        rp.reqs = in->reqs; rp.A = in->arena; rp.out = out; rp.hits = hit_ids; rp.hit_cap = hit_ids ? hit_cap : 0;
        rp.dlen = in->arena_len_dev;
        const int e = enqueue_batch(c, S, g, rp);
        if (e) return e;
        S->pending.push_back(rp);
        S->last_is_batch = true;
        return G.done(c);
    }
    // host buffers: stage reqs + arena + verdicts + hits through HBM (PCIe both ways); a stream
    // holds one staged batch at a time (the staging buffer is reused), so earlier ones complete first
    if (!S->pending.empty()) {
        const int e0 = sync_pending(c, S);
        if (e0 == GM_E_OVERFLOW)
            return fail(c, GM_E_EARLIER, "an earlier batch of this stream completed void before the staged batch (" +
                                         t_err + "); this batch was not enqueued");
        if (e0) return e0;
        rp.slot = 0;
    }
    size_t rq = (size_t)in->n * sizeof(gm_req), ar = (in->arena_len + 255) & ~255ull;
    size_t vo = (size_t)in->n * sizeof(gm_verdict), ho = hit_cap * 4;
    size_t tot = rq + ar + vo + ho + 1024;
    int e = grow(c, s, S->d_stage, S->cap_stage, tot);
    if (e) return e;
    uint8_t *p = S->d_stage;
    gm_req *dr = (gm_req *)p; p += (rq + 255) & ~255ull;
    uint8_t *da = p; p += ar;
    gm_verdict *dv = (gm_verdict *)p; p += (vo + 255) & ~255ull;
    uint32_t *dh = (uint32_t *)p;
    if (in->arena_len_dev) return fail(c, GM_E_INVAL, "arena_len_dev with GM_BATCH_HOST");
    HIPCHK(c, hipMemcpyAsync(dr, in->reqs, rq, hipMemcpyHostToDevice, s));
    if (in->arena_len) HIPCHK(c, hipMemcpyAsync(da, in->arena, in->arena_len, hipMemcpyHostToDevice, s));
    rp.reqs = dr; rp.A = da; rp.out = dv; rp.hits = dh; rp.hit_cap = hit_ids ? hit_cap : 0; rp.dlen = nullptr;
    rp.h_out = out; rp.h_hits = hit_ids; rp.h_hit_cap = hit_ids ? hit_cap : 0;
    e = enqueue_batch(c, S, g, rp);
    if (e) return e;
    if ((e = copy_back(c, S, rp))) return e;
    S->pending.push_back(rp);
    S->last_is_batch = true;
    return G.done(c);
}

int gm_sync(gm_ctx *c, void *stream) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return GM_OK;
    HIPCHK(c, hipSetDevice(c->dev));
    hipStream_t s = (hipStream_t)stream;
    Scratch *S = scratch_for(c, s);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    const int e = sync_pending(c, S);
    S->sync_log.clear();
    return e;
}

int gm_sync_batches(gm_ctx *c, void *stream, int32_t *status, size_t cap) {
    if (!c || (!status && cap)) return fail(c, GM_E_INVAL, "null argument");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return 0;
    HIPCHK(c, hipSetDevice(c->dev));
    hipStream_t s = (hipStream_t)stream;
    Scratch *S = scratch_for(c, s);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    const int e = sync_pending(c, S);
    if (e && e != GM_E_OVERFLOW) return e;   // (a HIP error: the log stays for the next call)
    const uint32_t parse_ov = S->h_status[PARSE_STATUS_WORD + 3], upuri_ov = S->h_status[UPURI_STATUS_WORD];
    if (e && (parse_ov || upuri_ov)) return e;   // not a gm_match_batch's: reported as gm_sync does
    const size_t n = S->sync_log.size();
    for (size_t i = 0; i < n && i < cap; i++) status[i] = S->sync_log[i];
    S->sync_log.clear();
    return n > 0x7FFFFFFFu ? 0x7FFFFFFF : (int)n;
}

int gm_counters(gm_ctx *c, uint64_t *out, size_t n) {
    if (!c || !out) return fail(c, GM_E_INVAL, "null argument");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    if (!c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    HIPCHK(c, hipSetDevice(c->dev));
    if (int e = wait_done(c)) return e;
    HIPCHK(c, hipMemcpy(out, c->gen->d_counters, std::min(n, c->gen->n_counters) * 8, hipMemcpyDeviceToHost));
    return GM_OK;
}

int gm_counters_global(gm_ctx *c, uint64_t *out, size_t n) {
    if (!c || !out) return fail(c, GM_E_INVAL, "null argument");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    if (!c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    HIPCHK(c, hipSetDevice(c->dev));
    if (int e = wait_done(c)) return e;
    {
        std::lock_guard<std::mutex> rl(c->red_mu);
        if (c->red_pending) {
            HIPCHK(c, hipEventSynchronize(c->ev_red));
            c->red_pending = false;
            c->red.finish(c->h_red);
        }
        if (!c->red.last_valid)
            return fail(c, GM_E_COMM, "the last gm_counters_allreduce found the ranks on different generations or "
                                      "counter spaces: no totals (the next call re-agrees)");
    }
    HIPCHK(c, hipMemcpy(out, c->gen->d_counters_sum, std::min(n, c->gen->n_counters) * 8, hipMemcpyDeviceToHost));
    return GM_OK;
}

int gm_counters_reset(gm_ctx *c) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return GM_OK;
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    if (!c->gen) return GM_OK;
    HIPCHK(c, hipSetDevice(c->dev));
    if (int e = wait_done(c)) return e;
    const size_t cb = std::max<size_t>(c->gen->n_counters, 1) * 8;
    HIPCHK(c, hipMemset(c->gen->d_counters, 0, cb));
    HIPCHK(c, hipMemset(c->gen->d_counters_sum, 0, cb));
    return GM_OK;
}

int gm_comm_unique_id(void *out) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return fail(nullptr, GM_E_COMM, "ncclGetUniqueId failed");
    memcpy(out, &id, sizeof id);
    return GM_OK;
}

int gm_comm_init(gm_ctx *c, const void *uid, int nranks, int rank) {
    if (!c || !uid) return fail(c, GM_E_INVAL, "null argument");
    HIPCHK(c, hipSetDevice(c->dev));
    ncclUniqueId id;
    memcpy(&id, uid, sizeof id);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) return fail(c, GM_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    return GM_OK;
}

// Out of place: the cumulative local counters stay this device's own; their sum over the ranks
// goes to the generation's reduced buffer (gm_counters_global).  Any number of calls give the
// true totals (an in-place reduction of cumulative counters would add them up again each time).
// The ranks' agreement on (gen, n_counters) rides in the same collective (RedProto): in steady
// state a call enqueues one staging kernel, ONE ncclAllReduce and one check kernel, with no host
// synchronisation (the 4-word agreement was a host round trip in front of every sum).
// The call evaluates the previous call's agreement first (its event, normally long complete); a
// failed one makes this call re-agree synchronously, and GM_E_COMM reaches every rank at the same
// call, since every rank reads the same summed block.
int gm_counters_allreduce(gm_ctx *c, void *stream) {
    if (!c || !c->comm) return fail(c, GM_E_COMM, "gm_comm_init not called");
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    if (!c->gen || !c->gen->d_counters) return fail(c, GM_E_NOGEN, "no counters");
    HIPCHK(c, hipSetDevice(c->dev));
    hipStream_t s = (hipStream_t)stream;
    Scratch *S = scratch_for(c, s);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    std::lock_guard<std::mutex> rl(c->red_mu);
    if (!c->h_red) {
        HIPCHK(c, hipHostMalloc((void **)&c->h_red, RED_WORDS * 8, hipHostMallocDefault));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_red, hipEventDisableTiming));
    }
    // the previous call's verdict, before anything of this call is issued (lockstep over the ranks)
    if (c->red_pending) {
        HIPCHK(c, hipEventSynchronize(c->ev_red));
        c->red_pending = false;
        c->red.finish(c->h_red);
    }
    DoneGuard G(S);
    const uint32_t gen = c->gen->stats.gen;
    const uint64_t n = c->gen->n_counters;
    unsigned long long blk[RED_WORDS];
    RedProto::pack(gen, n, blk);
    if (!c->red.agreed) {
        // synchronous: the agreement block alone (count RED_WORDS on every rank)
        if (int e = grow(c, s, c->d_red, c->cap_red, 2 * RED_WORDS)) return e;
        memcpy(c->h_red, blk, sizeof blk);
        HIPCHK(c, hipMemcpyAsync(c->d_red, c->h_red, RED_WORDS * 8, hipMemcpyHostToDevice, s));
        ncclResult_t r = ncclAllReduce(c->d_red, c->d_red + RED_WORDS, RED_WORDS, ncclUint64, ncclSum, c->comm, s);
        if (r != ncclSuccess) return fail(c, GM_E_COMM, std::string("ncclAllReduce (agreement): ") + ncclGetErrorString(r));
        HIPCHK(c, hipMemcpyAsync(c->h_red, c->d_red + RED_WORDS, RED_WORDS * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        if (!c->red.agree(c->h_red))
            return fail(c, GM_E_COMM, "ranks disagree on the generation or its counter space: no reduction issued");
    }
    // the block and the counters in one collective of RED_WORDS + the agreed count on every rank
    const uint64_t na = c->red.n;
    if (int e = grow(c, s, c->d_red, c->cap_red, 2 * (RED_WORDS + na))) return e;
    unsigned long long *din = c->d_red, *dout = c->d_red + RED_WORDS + na;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((RED_WORDS + na + 255) / 256, (uint64_t)c->cu_count * 4);
    RedBlock rb;
    memcpy(rb.w, blk, sizeof blk);
    k_red_stage<<<blocks, 256, 0, s>>>(c->gen->d_counters, n, na, rb, din);
    HIPCHK(c, hipGetLastError());
    ncclResult_t r = ncclAllReduce(din, dout, RED_WORDS + na, ncclUint64, ncclSum, c->comm, s);
    if (r != ncclSuccess) return fail(c, GM_E_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    k_red_finish<<<blocks, 256, 0, s>>>(dout, na, c->gen->d_counters_sum, n);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->h_red, dout, RED_WORDS * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipEventRecord(c->ev_red, s));
    c->red_pending = true;
    return G.done(c);
}

}  // extern "C"

// ============================================================================ debug (gpumatch_debug.h)
extern "C" int gm_debug_waf_keys(gm_ctx *c, uint32_t *out, size_t cap) {
    if (!c || !c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    const TabHeader &h = c->gen->hdr;
    const DLitBucket *b = (const DLitBucket *)(c->gen->host_image.data() + h.off_lit_buckets);
    size_t k = 0;
    for (uint32_t i = 0; i < h.n_lit_buckets_cap; i++)
        if (b[i].count) { if (k < cap) out[k] = b[i].key; k++; }
    return (int)k;
}

// The always-run union DFAs on the host over a batch (host buffers): per (group, request, zone it
// scans) step counts -- out[0] transitions, out[1] those taken in the start state that stay in
// it, out[2] those taken in the start state, out[3] (group, request, zone) tasks
extern "C" int gm_debug_alw_profile(gm_ctx *c, const gm_req *reqs, const uint8_t *arena, uint32_t n, uint64_t *out) {
    if (!c || !out) return fail(c, GM_E_INVAL, "null argument");
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    const Generation *g = c->gen;
    if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
    const uint8_t *img = g->host_image.data();
    const TabHeader &h = g->hdr;
    const DAlwSlice *sls = reinterpret_cast<const DAlwSlice *>(img + h.off_alw_slices);
    const DAlwGroup *grs = reinterpret_cast<const DAlwGroup *>(img + h.off_alw);
    uint64_t tot = 0, stay = 0, at = 0, tasks = 0;
    for (uint32_t si = 0; si < h.n_alw_slices; si++) {
        const DAlwSlice &sl = sls[si];
        if (sl.server != GM_NONE) continue;
        const uint8_t *P = img + h.off_alw_pack + sl.off;
        const uint8_t *clsa = P + ALW_DEAD_BYTES;
        const uint32_t ngb = alw_cls_ngb(sl.n_groups);
        for (uint32_t j = 0; j < sl.n_groups; j++) {
            const DAlwGroup &gr = grs[sl.first_group + j];
            for (uint32_t r = 0; r < n; r++) {
                const gm_req &q = reqs[r];
                const uint32_t lens[4] = {q.uri_len, q.args_len, q.hdr_len, q.body_len};
                uint64_t o = q.base;
                for (uint32_t z = 0; z < 4; z++) {
                    if ((gr.zones >> z) & 1u) {
                        tasks++;
                        uint32_t row = gr.start_row;
                        for (uint32_t i = 0; i < lens[z] && row; i++) {
                            const uint32_t b = arena[o + i];
                            uint16_t nx;
                            memcpy(&nx, P + 4 * row + clsa[b * ngb + j], 2);   // (rows: slice offset / 4)
                            tot++;
                            if (row == gr.start_row) { at++; if (nx == gr.start_row) stay++; }
                            row = nx;
                        }
                    }
                    o += lens[z];
                }
            }
        }
    }
    out[0] = tot; out[1] = stay; out[2] = at; out[3] = tasks;
    return GM_OK;
}

// gm_counters_allreduce's agreement protocol, exposed for the world-size-2 gloo test
// gm_counters_allreduce's protocol (RedProto) with the caller as the transport: pack the block a
// rank contributes, and drive one state machine per rank (new / begin / agree / finish)
extern "C" void gm_debug_red_pack(uint64_t gen, uint64_t n, uint64_t *words) {
    unsigned long long w[RED_WORDS];
    RedProto::pack((uint32_t)gen, n, w);
    for (uint32_t k = 0; k < RED_WORDS; k++) words[k] = w[k];
}
extern "C" uint32_t gm_debug_red_words(void) { return RED_WORDS; }
extern "C" void *gm_debug_red_new(void) { return new RedProto(); }
extern "C" void gm_debug_red_free(void *p) { delete static_cast<RedProto *>(p); }
// 1: this call must agree synchronously first (a block-only collective); 0: it issues the
// combined collective at once, of RED_WORDS + *count words
extern "C" int gm_debug_red_begin(void *p, uint64_t *count) {
    const RedProto *r = static_cast<RedProto *>(p);
    *count = r->agreed ? r->n : 0;
    return r->agreed ? 0 : 1;
}
extern "C" int gm_debug_red_agree(void *p, const uint64_t *sum) {
    unsigned long long w[RED_WORDS];
    for (uint32_t k = 0; k < RED_WORDS; k++) w[k] = sum[k];
    return static_cast<RedProto *>(p)->agree(w) ? GM_OK : GM_E_COMM;
}
// the summed block of a combined collective: GM_OK when its totals are valid (and the next call
// needs no agreement), GM_E_COMM otherwise
extern "C" int gm_debug_red_finish(void *p, const uint64_t *sum) {
    unsigned long long w[RED_WORDS];
    for (uint32_t k = 0; k < RED_WORDS; k++) w[k] = sum[k];
    RedProto *r = static_cast<RedProto *>(p);
    r->finish(w);
    return r->last_valid ? GM_OK : GM_E_COMM;
}

extern "C" void gm_debug_update_hook(void (*fn)(void *), void *arg) {
    g_update_hook = fn;
    g_update_hook_arg = arg;
}

extern "C" int gm_debug_inet(const uint8_t *text, size_t n, char *out, size_t cap) {
    InetAddr a;
    if (!text || !out || n > 0xFFFF || !ngx_parse_addr_port(text, (uint32_t)n, a)) return -1;
    uint8_t t[48];
    const uint32_t k = ngx_addr_text(a, t);
    const int w = snprintf(out, cap, "%.*s %u", (int)k, (const char *)t, a.port);
    return w;
}

// The last batch's device status words (gm_waf.inc STATUS_WORDS: counts and profiling counters),
// as of the last gm_sync.
extern "C" int gm_debug_status(gm_ctx *c, uint32_t *out, size_t n) {
    if (!c || !out) return fail(c, GM_E_INVAL, "null argument");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    std::lock_guard<std::mutex> lk(c->last_mu);
    memcpy(out, c->last_status, std::min<size_t>(n, STATUS_WORDS) * 4);
    return (int)std::min<size_t>(n, STATUS_WORDS);
}

extern "C" int gm_debug_waf_lits(gm_ctx *c, uint32_t *out, size_t cap) {
    if (!c || !c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    const TabHeader &h = c->gen->hdr;
    const DLitBucket *b = (const DLitBucket *)(c->gen->host_image.data() + h.off_lit_buckets);
    const DLit *l = (const DLit *)(c->gen->host_image.data() + h.off_lits);
    size_t k = 0;
    for (uint32_t i = 0; i < h.n_lit_buckets_cap; i++)
        for (uint32_t j = 0; j < b[i].count; j++, k++) {
            if (k >= cap) continue;
            const DLit &d = l[b[i].first + j];
            out[4 * k] = b[i].key; out[4 * k + 1] = d.id;
            out[4 * k + 2] = (uint32_t)(uint16_t)d.key_off | (uint32_t)d.len << 16;
            out[4 * k + 3] = (uint32_t)d.flags | (uint32_t)d.zones << 8;
        }
    return (int)k;
}

extern "C" int gm_debug_waf_lit_bytes(gm_ctx *c, uint32_t row, uint8_t *out, size_t cap) {
    if (!c || !c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    const TabHeader &h = c->gen->hdr;
    const uint8_t *img = c->gen->host_image.data();
    const DLitBucket *b = (const DLitBucket *)(img + h.off_lit_buckets);
    const DLit *l = (const DLit *)(img + h.off_lits);
    uint32_t k = 0;
    for (uint32_t i = 0; i < h.n_lit_buckets_cap; i++) {
        if (row >= k + b[i].count) { k += b[i].count; continue; }
        const DLit &d = l[b[i].first + (row - k)];
        memcpy(out, img + h.off_bytes + d.bytes_off, std::min<size_t>(cap, d.len));
        return d.len;
    }
    return fail(c, GM_E_INVAL, "row out of range");
}

// Host restatement of k_waf_scan's candidate rule over `len` arena bytes (same tables, same
// hashes): the CPU tests use it to check that every literal occurrence is a candidate and to
// measure the prefilter's false-positive rate without a GPU.
extern "C" int64_t gm_debug_waf_prefilter(gm_ctx *c, const uint8_t *A, size_t len, uint64_t *out, size_t cap) {
    if (!c || !c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    const TabHeader &h = c->gen->hdr;
    const uint32_t *bloom = (const uint32_t *)(c->gen->host_image.data() + h.off_waf_a);
    int64_t k = 0;
    for (size_t p = 0; p + 3 <= len; p += 2) {   // even offsets only (stride-2 scan); the window's
        uint32_t w = 0;                              // bytes past the arena read as 0
        memcpy(&w, A + p, std::min<size_t>(4, len - p));
        const BloomProbe b = scan_probe(fold4(w), h.bloom_mul, h.bloom_pk);
        if ((bloom[b.block] & b.mask) == b.mask) { if ((size_t)k < cap && out) out[k] = p; k++; }
    }
    return k;
}

// Host restatement of both filter stages: k_waf_scan's candidate rule, then k_waf_verify's
// stage-2 context filter (bytes outside the arena read as the fold of 0, like the kernels).
extern "C" int64_t gm_debug_waf_prefilter2(gm_ctx *c, const uint8_t *A, size_t len, uint64_t *out, size_t cap) {
    if (!c || !c->gen) return fail(c, GM_E_NOGEN, "no generation loaded");
    const TabHeader &h = c->gen->hdr;
    const uint32_t *bloom = (const uint32_t *)(c->gen->host_image.data() + h.off_waf_a);
    const uint32_t *ctxb = (const uint32_t *)(c->gen->host_image.data() + h.off_waf_b);
    auto fb = [&](int64_t i) -> uint32_t { return (i >= 0 && (size_t)i < len ? A[i] : 0u) | 0x20u; };
    int64_t k = 0;
    for (size_t p = 0; p + 3 <= len; p += 2) {
        uint32_t w = 0;
        memcpy(&w, A + p, std::min<size_t>(4, len - p));
        w = fold4(w);
        const BloomProbe b = scan_probe(w, h.bloom_mul, h.bloom_pk);
        if ((bloom[b.block] & b.mask) != b.mask) continue;
        const int64_t q = (int64_t)p;
        const uint32_t l2 = fb(q - 2) | fb(q - 1) << 8, r2 = fb(q + 4) | fb(q + 5) << 8;
        bool hit = false;
        for (int i = 0; i < CTX_SHAPES && !hit; i++) {
            const uint32_t nl = ctx_shape_nl(i), nr = ctx_shape_nr(i);
            const BloomProbe b2 = bloom_probe(ctx_key(w, l2 & ctx_lmask(nl), r2 & ctx_rmask(nr), nl * 3 + nr),
                                              h.ctx_mul, CTX_PK);
            hit = (ctxb[b2.block] & b2.mask) == b2.mask;
        }
        if (hit) { if ((size_t)k < cap && out) out[k] = p; k++; }
    }
    return k;
}

// Server `sid` of the current generation as u32 words (DServer), followed by its regex
// locations (dfa, loc) pairs; returns the number of words written.
// The union-DFA slices (always-run, then regex-location): per slice 8 u32 (len, n_groups, zones,
// server, min_member, flags, states, classes summed over its groups) -- diagnostics
extern "C" int gm_debug_alw_slices(gm_ctx *c, uint32_t *out, size_t cap) {
    if (!c || !c->gen || !out) return -1;
    const TabHeader &h = c->gen->hdr;
    const uint8_t *b = c->gen->host_image.data();
    const DAlwSlice *sls = reinterpret_cast<const DAlwSlice *>(b + h.off_alw_slices);
    const DAlwGroup *grs = reinterpret_cast<const DAlwGroup *>(b + h.off_alw);
    const uint32_t ns = h.n_alw_slices + h.n_rsl;
    size_t k = 0;
    for (uint32_t i = 0; i < ns && k + 8 <= cap; i++) {
        const DAlwSlice &sl = sls[i];
        uint32_t st = 0, cl = 0;
        for (uint32_t g = sl.first_group; g < sl.first_group + sl.n_groups; g++) { st += grs[g].n_states; cl += grs[g].n_classes; }
        const uint32_t v[8] = {sl.len, sl.n_groups, sl.zones, sl.server, sl.min_member, sl.flags, st, cl};
        for (uint32_t q = 0; q < 8; q++) out[k++] = v[q];
    }
    return (int)k;
}

extern "C" int gm_debug_server(gm_ctx *c, uint32_t sid, uint32_t *out, size_t cap) {
    if (!c || !c->gen || !out) return -1;
    const TabHeader &h = c->gen->hdr;
    if (sid >= h.n_servers) return -1;
    const uint8_t *b = c->gen->host_image.data();
    const DServer S = reinterpret_cast<const DServer *>(b + h.off_servers)[sid];
    const DRegexLoc *rl = reinterpret_cast<const DRegexLoc *>(b + h.off_rlocs);
    size_t k = 0;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(&S);
    for (size_t i = 0; i < sizeof(DServer) / 4 && k < cap; i++) out[k++] = w[i];
    for (uint32_t i = 0; i < S.n_rloc && k + 2 <= cap; i++) { out[k++] = rl[S.first_rloc + i].dfa; out[k++] = rl[S.first_rloc + i].loc; }
    return (int)k;
}

// ---------------------------------------------------------------------------------------------
// $uri normalisation: nginx's ngx_http_parse_complex_uri with merge_slashes on,
// restated as a byte state machine -- percent-decoding (a decoded byte re-enters the state that
// saw its '%', so %2F acts as '/' and %2E as '.', except decoded '%', '#' and '?', which are
// kept literally), merged slashes, "." and ".." segments; '?' or '#' ends the path; a bad escape,
// a NUL or ".." above the root is a 400 (GM_NONE).  Lane per path; the output never outgrows
// the input, so path i is written at its own arena offset.  Bound: HBM, algorithmic bytes per
// path = its length read + its normalised length written + 16 B of (offset, length, out_len).
namespace {
enum : uint32_t { UN_USUAL, UN_SLASH, UN_DOT, UN_DOTDOT, UN_Q1, UN_Q2 };

__device__ __forceinline__ int un_hex(uint32_t c) {
    if (c - '0' < 10u) return (int)(c - '0');
    c |= 0x20;
    return c - 'a' < 6u ? (int)(c - 'a' + 10) : -1;
}

// out[0 .. u) holds "<...>/.."; drop it and the segment before it; false if that leaves the root
__device__ __forceinline__ bool un_up(const uint8_t *out, uint32_t &u) {
    if (u < 4) return false;
    for (int64_t k = (int64_t)u - 4; k >= 0; k--)
        if (out[k] == '/') { u = (uint32_t)k + 1; return true; }
    return false;
}

// (no __restrict__: out may alias in -- the write position never passes the read position)
__device__ uint32_t un_one(const uint8_t *in, uint32_t n, uint8_t *out) {
    uint32_t st = UN_USUAL, qst = UN_USUAL, dec = 0, u = 0, i = 0, ch = 0;
    bool again = false;
    for (;;) {
        if (!again) {
            if (i >= n) break;
            ch = in[i++];
        }
        again = false;
        if (st == UN_Q1) {
            const int v = un_hex(ch);
            if (v < 0) return GM_NONE;
            dec = (uint32_t)v; st = UN_Q2;
            continue;
        }
        if (st == UN_Q2) {
            const int v = un_hex(ch);
            if (v < 0) return GM_NONE;
            ch = dec << 4 | (uint32_t)v;
            if (v < 10 ? (ch == '%' || ch == '#') : ch == '?') { out[u++] = (uint8_t)ch; st = UN_USUAL; continue; }
            if (ch == 0) return GM_NONE;
            st = qst; again = true;
            continue;
        }
        if (ch == 0) return GM_NONE;
        if (ch == '?' || ch == '#') break;
        if (ch == '%') { qst = st; st = UN_Q1; continue; }
        switch (st) {
        case UN_USUAL:
            out[u++] = (uint8_t)ch;
            if (ch == '/') st = UN_SLASH;
            break;
        case UN_SLASH:
            if (ch == '/') break;
            out[u++] = (uint8_t)ch;
            st = ch == '.' ? UN_DOT : UN_USUAL;
            break;
        case UN_DOT:
            if (ch == '/') { u--; st = UN_SLASH; break; }
            out[u++] = (uint8_t)ch;
            st = ch == '.' ? UN_DOTDOT : UN_USUAL;
            break;
        default:   // UN_DOTDOT
            if (ch == '/') {
                if (!un_up(out, u)) return GM_NONE;
                st = UN_SLASH;
                break;
            }
            out[u++] = (uint8_t)ch;
            st = UN_USUAL;
            break;
        }
    }
    if (st == UN_Q1 || st == UN_Q2) return GM_NONE;
    if (st == UN_DOT) u--;
    else if (st == UN_DOTDOT && !un_up(out, u)) return GM_NONE;
    return u;
}

__global__ __launch_bounds__(256) void k_uri_normalize(const uint8_t *A, const uint64_t *__restrict__ off,
                                                        const uint32_t *__restrict__ len, uint32_t n,
                                                        uint8_t *out, uint32_t *__restrict__ out_len) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out_len[i] = un_one(A + off[i], len[i], out + off[i]);
}

#include "gm_wire.inc"
#include "gm_peers.inc"
#include "gm_upuri.inc"
}  // namespace

extern "C" int gm_normalize_uris(gm_ctx *c, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                                 uint32_t n, uint8_t *out, uint32_t *out_len, void *stream) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    if (n == 0) return GM_OK;
    if (!arena || !off || !len || !out || !out_len) return fail(c, GM_E_INVAL, "null argument");
    HIPCHK(c, hipSetDevice(c->dev));
    // the call is this stream's last enqueued work: its status words start clean, so a gm_sync
    // after it reports OK (no stale match-batch overflow)
    Scratch *S = scratch_for(c, (hipStream_t)stream);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    S->last_is_batch = false;   // (the batch status words are cleared: a pending batch's continuation
                                //  becomes a whole re-run)
    HIPCHK(c, hipMemsetAsync(S->d_status, 0, STATUS_WORDS * 4, (hipStream_t)stream));
    S->ev_pending = false;
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, (uint32_t)c->cu_count * 16));
    k_uri_normalize<<<blocks, 256, 0, (hipStream_t)stream>>>(arena, off, len, n, out, out_len);
    HIPCHK(c, hipGetLastError());
    return GM_OK;
}

extern "C" int gm_parse_requests(gm_ctx *c, const uint8_t *wire, const gm_wire_msg *msgs, uint32_t n, gm_req *reqs,
                      uint8_t *arena, uint64_t arena_cap, uint64_t *arena_len_dev, void *stream) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    if (!arena_len_dev || (n && (!wire || !msgs || !reqs || !arena))) return fail(c, GM_E_INVAL, "null argument");
    if (((uintptr_t)reqs & 15) || ((uintptr_t)arena & 15)) return fail(c, GM_E_INVAL, "reqs / arena must be 16-byte aligned");
    HIPCHK(c, hipSetDevice(c->dev));
    hipStream_t s = (hipStream_t)stream;
    Scratch *S = scratch_for(c, s);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    HIPCHK(c, hipMemsetAsync(S->d_status + PARSE_STATUS_WORD, 0, (UPURI_STATUS_WORD - PARSE_STATUS_WORD) * 4, s));
    if (n == 0) { HIPCHK(c, hipMemsetAsync(arena_len_dev, 0, 8, s)); return GM_OK; }
    size_t tmp = 0;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, S->d_wsize, S->d_wbase, (int)n + 1, s));
    int e;
    if ((e = grow(c, s, S->d_wsize, S->cap_wsize, (size_t)n + 1))) return e;
    if ((e = grow(c, s, S->d_wbase, S->cap_wbase, (size_t)n + 1))) return e;
    if ((e = grow(c, s, S->d_wtemp, S->cap_wtemp, tmp))) return e;
    // the parser's waves are persistent (grid-stride): GM_WIRE_WPE waves per SIMD are resident (WIRE_OCC),
    // i.e. GM_WIRE_WPE blocks per CU -- a larger grid would only queue, and its per-wave $uri scratch
    // (WIRE_SCR each) would hold memory no resident wave uses
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((n + WIRE_WAVES - 1) / WIRE_WAVES,
                                                                     (uint32_t)c->cu_count * GM_WIRE_WPE));
    if ((e = grow(c, s, S->d_wscr, S->cap_wscr, (size_t)blocks * WIRE_WAVES * WIRE_SCR))) return e;
    if ((e = grow(c, s, S->d_wsum, S->cap_wsum, (size_t)n * sizeof(WireSum)))) return e;
    WireSum *wsum = reinterpret_cast<WireSum *>(S->d_wsum);
    // PROXY protocol: on a generation with a `listen ... proxy_protocol` port the descriptors go
    // through k_wire_proxy first (their headers read, the messages advanced past them); the parse
    // passes read the copies.  The generation's port table decides (shared lock: the copy of the
    // flags is taken before the launch, the kernel reads the image the lock keeps alive until the
    // stream's completion event)
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    DoneGuard G(S);
    const Generation *g = c->gen;
    bool proxy = false;
    if (g) {
        const DPort *ports = reinterpret_cast<const DPort *>(g->host_image.data() + g->hdr.off_ports);
        for (uint32_t k = 0; k < g->hdr.n_ports; k++) proxy |= ports[k].proxy != 0;
    }
    if (proxy) {
        if ((e = grow(c, s, S->d_wmsg, S->cap_wmsg, (size_t)n))) return e;
        k_wire_proxy<<<std::min<uint32_t>((n + 255) / 256, (uint32_t)c->cu_count * 8), 256, 0, s>>>(wire, msgs, n, g->tab,
                                                                                                   S->d_wmsg);
        HIPCHK(c, hipGetLastError());
        msgs = S->d_wmsg;
    }
    const uint32_t fmask = proxy ? WIRE_FMASK_PROXY : WIRE_FMASK_PLAIN;
    // pass 1's per-wave lists: a wave sizes requests gw, gw + W, ... -- at most `per` of them
    const uint32_t W = blocks * WIRE_WAVES, per = (n + W - 1) / W;
    if ((e = grow(c, s, S->d_wfull, S->cap_wfull, (size_t)W * per + W))) return e;
    uint32_t *fcnt = S->d_wfull + (size_t)W * per;
    const uint32_t nblk = (uint32_t)std::min<uint64_t>((arena_cap >> 10) + 1, 0xFFFFFFFFull);
    if ((e = grow(c, s, S->d_wblk, S->cap_wblk, (size_t)nblk))) return e;
    if ((e = grow(c, s, S->d_wpieces, S->cap_wpieces, (size_t)n * WIRE_PIECES))) return e;
    k_wire_size<<<blocks, 64 * WIRE_WAVES, 0, s>>>(wire, msgs, n, S->d_wsize, S->d_wscr, wsum, fmask, S->d_wfull, per, fcnt,
                                                   S->d_wpieces);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(S->d_wtemp, tmp, S->d_wsize, S->d_wbase, (int)n + 1, s));
    // pass 2: the block map, the flat gather of nearly every slot (a lane per 16-byte chunk), the
    // void batch's records, the full lists
    const uint32_t lb = std::min<uint32_t>((n + 255) / 256, (uint32_t)c->cu_count * 8);
    k_wire_blk<<<lb, 256, 0, s>>>(S->d_wbase, n, S->d_wblk, nblk);
    HIPCHK(c, hipGetLastError());
    k_wire_gather<<<(uint32_t)c->cu_count * 16, 256, 0, s>>>(wire, msgs, n, S->d_wsize, S->d_wbase, reqs, arena, arena_cap,
                                                           arena_len_dev, S->d_status + PARSE_STATUS_WORD, wsum, S->d_wblk,
                                                           fmask, S->d_wpieces);
    HIPCHK(c, hipGetLastError());
    k_wire_void<<<lb, 256, 0, s>>>(msgs, n, S->d_wsize, S->d_wbase, reqs, arena_cap);
    HIPCHK(c, hipGetLastError());
    k_wire_emit_full<<<blocks, 64 * WIRE_WAVES, 0, s>>>(wire, msgs, n, S->d_wsize, S->d_wbase, reqs, arena, arena_cap,
                                                        S->d_wscr, wsum, fmask, S->d_wfull, per, fcnt);
    HIPCHK(c, hipGetLastError());
    return G.done(c);
}

// The last gm_parse_requests' per-request slot sizes on `stream` (size pass), for debugging.
extern "C" int gm_debug_wire_sizes(gm_ctx *c, void *stream, uint64_t *out, size_t n) {
    if (!c || !out) return fail(c, GM_E_INVAL, "null argument");
    Scratch *S = scratch_for(c, (hipStream_t)stream);
    if (!S || !S->d_wsize) return fail(c, GM_E_INVAL, "no parse on this stream");
    HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
    HIPCHK(c, hipMemcpy(out, S->d_wsize, std::min(n, S->cap_wsize) * 8, hipMemcpyDeviceToHost));
    return GM_OK;
}

// ---------------------------------------------------------------- upstream peer selection (§8 f3)
extern "C" int gm_peers_init(gm_ctx *c, gm_peer_state *state, uint32_t n_peers, void *stream) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    HIPCHK(c, hipSetDevice(c->dev));
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    const Generation *g = c->gen;
    if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
    if (n_peers != g->tab.n_peers) return fail(c, GM_E_INVAL, "n_peers differs from the generation's peer count");
    if (n_peers == 0) return GM_OK;
    if (!state) return fail(c, GM_E_INVAL, "null state");
    Scratch *S = scratch_for(c, (hipStream_t)stream);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    DoneGuard G(S);
    k_peers_init<<<std::min<uint32_t>((n_peers + 255) / 256, 1024), 256, 0, (hipStream_t)stream>>>(g->tab, state);
    HIPCHK(c, hipGetLastError());
    return G.done(c);
}

// NGINX Plus keeps a kept server's runtime state across an API update: new_state[j] = the state
// of the previous table's peer it came from (gm_update_upstream's map), else the initial state.
__global__ void k_peers_migrate(const gm_peer_state *__restrict__ old_st, const uint32_t *__restrict__ map,
                                const uint32_t *__restrict__ init, uint32_t n, gm_peer_state *__restrict__ new_st) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const uint32_t from = map[j];
        gm_peer_state v{0u, 0, init[j], 0u};
        if (from != GM_NONE) v = old_st[from];
        new_st[j] = v;
    }
}

extern "C" int gm_peers_migrate(gm_ctx *c, const gm_peer_state *old_state, uint32_t old_n, gm_peer_state *new_state,
                                uint32_t new_n, void *stream) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    HIPCHK(c, hipSetDevice(c->dev));
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    const Generation *g = c->gen;
    if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
    if (!g->d_peer_map && g->tab.n_peers) return fail(c, GM_E_INVAL, "the live tables did not come from gm_update_upstream");
    if (old_n != g->peer_map_old_n) return fail(c, GM_E_INVAL, "old_n differs from the previous table's peer count");
    if (new_n != g->tab.n_peers) return fail(c, GM_E_INVAL, "new_n differs from the generation's peer count");
    if (new_n == 0) return GM_OK;
    if (!new_state || (old_n && !old_state)) return fail(c, GM_E_INVAL, "null state");
    if ((const void *)old_state == (const void *)new_state) return fail(c, GM_E_INVAL, "migrate in place");
    Scratch *S = scratch_for(c, (hipStream_t)stream);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    DoneGuard G(S);
    k_peers_migrate<<<std::min<uint32_t>((new_n + 255) / 256, 1024), 256, 0, (hipStream_t)stream>>>(
        old_state, g->d_peer_map, g->tab.peer_init, new_n, new_state);
    HIPCHK(c, hipGetLastError());
    return G.done(c);
}

extern "C" int gm_select_peers(gm_ctx *c, const gm_batch *in, const gm_verdict *verdicts, gm_peer_state *state,
                               uint32_t n_peers, uint32_t *peer_out, void *stream) {
    if (!c || !in) return fail(c, GM_E_INVAL, "null argument");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    if (in->flags & GM_BATCH_HOST) return fail(c, GM_E_INVAL, "gm_select_peers takes device buffers");
    const uint32_t n = in->n;
    if (n && (!verdicts || !peer_out || !in->reqs)) return fail(c, GM_E_INVAL, "null argument");
    if (((uintptr_t)verdicts & 15) || ((uintptr_t)in->reqs & 15)) return fail(c, GM_E_INVAL, "verdicts / reqs must be 16-byte aligned");
    HIPCHK(c, hipSetDevice(c->dev));
    hipStream_t s = (hipStream_t)stream;
    Scratch *S = scratch_for(c, s);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    DoneGuard G(S);
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    const Generation *g = c->gen;
    if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
    const GTab &t = g->tab;
    if (n_peers != t.n_peers) return fail(c, GM_E_INVAL, "n_peers differs from the generation's peer count");
    if (t.n_peers && !state) return fail(c, GM_E_INVAL, "null state");
    if (n == 0) return GM_OK;
    const uint32_t nu = std::max<uint32_t>(t.n_ups, 1);
    int e;
    if ((e = grow(c, s, S->d_pk, S->cap_pk, (size_t)n * 4))) return e;
    if ((e = grow(c, s, S->d_pseg, S->cap_pseg, (size_t)nu * 2))) return e;
    if ((e = grow(c, s, S->d_pprog, S->cap_pprog, (size_t)nu))) return e;
    if ((e = grow(c, s, S->d_ppat, S->cap_ppat, (size_t)std::max<uint32_t>(t.n_peers, 1) * 2))) return e;
    uint32_t *keys = S->d_pk, *vals = keys + n, *ks = vals + n, *vs = ks + n;
    const int bits = t.n_ups ? 32 - __builtin_clz(t.n_ups) : 1;   // keys <= n_ups (the sentinel)
    size_t tb = 0;
    HIPCHK(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, ks, vals, vs, (int)n, 0, bits, s));
    if ((e = grow(c, s, S->d_ptemp, S->cap_ptemp, tb))) return e;
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, (uint32_t)c->cu_count * 8));
    // one lane per request, no grid-stride loop: every request's dependent loads (verdict ->
    // record -> draws -> peer state) in flight at once
    k_peer_pick<<<(n + 255) / 256, 256, 0, s>>>(in->reqs, in->arena, verdicts, n, t, state, peer_out, keys, vals);
    HIPCHK(c, hipGetLastError());
    if (t.n_ups) {
        HIPCHK(c, hipcub::DeviceRadixSort::SortPairs(S->d_ptemp, tb, keys, ks, vals, vs, (int)n, 0, bits, s));
        HIPCHK(c, hipMemsetAsync(S->d_pseg, 0, (size_t)nu * 2 * 4, s));
        k_peer_segs<<<blocks, 256, 0, s>>>(ks, n, t.n_ups, S->d_pseg, S->d_pseg + nu);
        HIPCHK(c, hipGetLastError());
        k_peer_seq<<<t.n_ups, 64, 0, s>>>(t, state, S->d_pseg, S->d_pseg + nu, vs, peer_out, S->d_ppat, S->d_pprog);
        HIPCHK(c, hipGetLastError());
        k_peer_fill<<<blocks, 256, 0, s>>>(ks, vs, n, t, S->d_pseg, S->d_pprog, S->d_ppat, peer_out);
        HIPCHK(c, hipGetLastError());
    }
    if (t.n_peers) {
        // histogram blocks: enough to stream the picks, few enough that the flush stays small
        k_peer_count<<<std::max<uint32_t>(1, std::min<uint32_t>((n + 4095) / 4096, (uint32_t)c->cu_count * 2)), 256, 0, s>>>(
            peer_out, n, state, t.n_peers, 1);
        HIPCHK(c, hipGetLastError());
    }
    return G.done(c);
}

extern "C" int gm_release_peers(gm_ctx *c, const uint32_t *peer_ids, uint32_t n, gm_peer_state *state,
                                uint32_t n_peers, void *stream) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    HIPCHK(c, hipSetDevice(c->dev));
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    const Generation *g = c->gen;
    if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
    if (n_peers != g->tab.n_peers) return fail(c, GM_E_INVAL, "n_peers differs from the generation's peer count");
    if (n == 0 || n_peers == 0) return GM_OK;
    if (!peer_ids || !state) return fail(c, GM_E_INVAL, "null argument");
    Scratch *S = scratch_for(c, (hipStream_t)stream);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    DoneGuard G(S);
    k_peer_count<<<std::max<uint32_t>(1, std::min<uint32_t>((n + 4095) / 4096, (uint32_t)c->cu_count * 2)), 256, 0,
                   (hipStream_t)stream>>>(peer_ids, n, state, n_peers, -1);
    HIPCHK(c, hipGetLastError());
    return G.done(c);
}

extern "C" int gm_peer_address(gm_ctx *c, uint32_t peer, char *buf, size_t cap, uint32_t *upstream_id) {
    if (!c) return fail(c, GM_E_INVAL, "null ctx");
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    const Generation *g = c->gen;
    if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
    if (peer >= g->peer_addrs.size()) return fail(c, GM_E_INVAL, "peer id out of range");
    const std::string &a = g->peer_addrs[peer];
    if (buf && cap) {
        const size_t m = std::min(cap - 1, a.size());
        memcpy(buf, a.data(), m);
        buf[m] = 0;
    }
    if (upstream_id) *upstream_id = g->peer_ups[peer];
    return (int)a.size();
}

// ---------------------------------------------------------------- upstream request URIs (§8 f1)
extern "C" int gm_upstream_uris(gm_ctx *c, const gm_batch *in, const gm_verdict *verdicts, uint8_t *out,
                                uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, void *stream) {
    if (!c || !in) return fail(c, GM_E_INVAL, "null argument");
    if (c->flags & GM_CREATE_COMPILE_ONLY) return fail(c, GM_E_NODEVICE, "compile-only context");
    if (in->flags & GM_BATCH_HOST) return fail(c, GM_E_INVAL, "gm_upstream_uris takes device buffers");
    const uint32_t n = in->n;
    if (n && (!verdicts || !out_off || !out_len || !in->reqs || !in->arena || (!out && out_cap)))
        return fail(c, GM_E_INVAL, "null argument");
    if (((uintptr_t)verdicts & 15) || ((uintptr_t)in->reqs & 15)) return fail(c, GM_E_INVAL, "verdicts / reqs must be 16-byte aligned");
    HIPCHK(c, hipSetDevice(c->dev));
    hipStream_t s = (hipStream_t)stream;
    Scratch *S = scratch_for(c, s);
    if (!S) return fail(c, GM_E_NOMEM, t_err);
    DoneGuard G(S);
    std::shared_lock<std::shared_mutex> lk(c->gen_mu);
    const Generation *g = c->gen;
    if (!g) return fail(c, GM_E_NOGEN, "no generation loaded");
    HIPCHK(c, hipMemsetAsync(S->d_status + UPURI_STATUS_WORD, 0, 4, s));
    if (n == 0) return GM_OK;
    int e;
    if ((e = grow(c, s, S->d_usize, S->cap_usize, (size_t)n))) return e;
    size_t tb = 0;
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, S->d_usize, out_off, (int)n, s));
    if ((e = grow(c, s, S->d_utemp, S->cap_utemp, tb))) return e;
    const uint32_t blocks = (n + 255) / 256;
    k_upuri_size<<<blocks, 256, 0, s>>>(in->reqs, in->arena, verdicts, n, g->tab, S->d_usize);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(S->d_utemp, tb, S->d_usize, out_off, (int)n, s));
    k_upuri_emit<<<blocks, 256, 0, s>>>(in->reqs, in->arena, verdicts, n, g->tab, out_off, out, out_cap, out_len,
                                        S->d_status + UPURI_STATUS_WORD);
    HIPCHK(c, hipGetLastError());
    return G.done(c);
}

// The measurement / tuning variants compiled in (gm_stats_t.build_flags): a bench line can show it
// came from the product build.  Every GM_EXP_* macro is a measurement (timing) variant; the
// tuning macros count when they differ from the shipped values.
static constexpr uint32_t kBuildFlags =
#if defined(GM_EXP_COUNT) || defined(GM_EXP_RLOC_NOREC) || defined(GM_EXP_RLOC_NOSB) || defined(GM_EXP_ALW_NOEMIT) || \
    defined(GM_EXP_NO_RULES) || defined(GM_EXP_NO_SPLIT) || defined(GM_EXP_RULES_NOSPAN) || defined(GM_EXP_RULES_NOVAR) || \
    defined(GM_EXP_ALW_COUNT)
    GM_BUILD_EXPERIMENT |
#endif
#if GM_SCAN_BLOCK != 1024 || GM_SCAN_CPOL != 2 || GM_SCAN_DEPTH != 6 || GM_SCAN_STG != 32 || \
    GM_ROUTE_BPC != 1 || GM_ROUTE_PRIO != 0 || GM_ROUTE_WPE != GM_ROUTE_WPE_SHIPPED || GM_EXP_GRIDMUL != 8 || \
    GM_EXP_WPE != 3 || GM_RLOC_CTX != 1 || GM_RLOC_PREF != 0 || GM_ALW_SLICE_GROUPS != 8 || GM_WIRE_WPE != 6 || \
    GM_WIRE_WPE_EMIT != GM_WIRE_WPE || GM_WIRE_CANON != 1 || GM_EXACT_BPC != 6 || !defined(GM_DFA_INL_SHIPPED) || \
    GM_SLOW_WPE != 3 || GM_SOLO_WPE != 3
    GM_BUILD_TUNING |
#endif
    0u;
static uint32_t build_flags() { return kBuildFlags; }
