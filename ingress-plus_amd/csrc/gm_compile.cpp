// gm_compile.cpp -- generation compiler (host C++, part of libgpumatch.so).
//
// Input: the GMB1 blob the Manager wrapper builds from what the Configurator handed to
// nginx.Manager (internal/nginx/manager.go:34-50): the main nginx.conf (version1/nginx.tmpl),
// the conf.d files (version1/nginx.ingress.tmpl, version2/nginx.virtualserver.tmpl) in include
// order, and the build-defined WAF signature set.  Output: one flat table image (gm_tables.hpp).
//
// The text is parsed with nginx's token rules (ngx_conf_read_token) and the directives that
// decide a request's verdict are compiled; everything else (timeouts, headers, buffers) is
// ignored.  Constructs the device path cannot express are counted in gm_stats_t and the
// affected location answers GM_ACT_UNSUPPORTED; they never fail the load (SURVEY §8 b).
#include "gm_compile.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <thread>
#include <unordered_map>

#include "gm_inet.hpp"
#include "gm_regex.hpp"

namespace gm {
namespace {

// ============================================================================ tokens
struct Dir {
    std::vector<std::string> a;
    std::vector<Dir> body;
    bool block = false;
};

class Tokenizer {
  public:
    Tokenizer(const char *s, size_t n) : s_(s), n_(n) {}
    enum Ev { WORD, SEMI, OPEN, CLOSE, END, BAD };
    Ev next(std::string &w) {
        for (;;) {
            while (i_ < n_ && is_ws(s_[i_])) i_++;
            if (i_ >= n_) return END;
            char c = s_[i_];
            if (c == '#') { while (i_ < n_ && s_[i_] != '\n') i_++; continue; }
            if (c == ';') { i_++; return SEMI; }
            if (c == '{') { i_++; return OPEN; }
            if (c == '}') { i_++; return CLOSE; }
            w.clear();
            if (c == '"' || c == '\'') {
                size_t j = i_ + 1;
                while (j < n_ && s_[j] != c) j += (s_[j] == '\\') ? 2 : 1;
                if (j >= n_) return BAD;
                unescape(i_ + 1, j, w);
                i_ = j + 1;
                if (i_ < n_ && s_[i_] == ')') pending_paren_ = true;   // "...") -> extra ")" token
                else if (i_ < n_ && !is_ws(s_[i_]) && s_[i_] != ';' && s_[i_] != '{') return BAD;
                return WORD;
            }
            size_t j = i_;
            bool dollar = false;
            while (j < n_) {
                char ch = s_[j];
                if (ch == '{' && dollar) { j++; continue; }
                dollar = false;
                if (ch == '\\' && j + 1 < n_) { j += 2; continue; }
                if (ch == '$') { dollar = true; j++; continue; }
                if (is_ws(ch) || ch == ';' || ch == '{') break;
                j++;
            }
            unescape(i_, j, w);
            i_ = j;
            return WORD;
        }
    }
    bool take_paren() { if (pending_paren_) { pending_paren_ = false; i_++; return true; } return false; }

  private:
    static bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
    void unescape(size_t a, size_t b, std::string &w) {
        for (size_t k = a; k < b; k++) {
            if (s_[k] == '\\' && k + 1 < b) {
                char e = s_[k + 1];
                const char *m = strchr("\"'\\", e);
                if (m) { w.push_back(e); k++; continue; }
                if (e == 't') { w.push_back('\t'); k++; continue; }
                if (e == 'r') { w.push_back('\r'); k++; continue; }
                if (e == 'n') { w.push_back('\n'); k++; continue; }
            }
            w.push_back(s_[k]);
        }
    }
    const char *s_;
    size_t n_, i_ = 0;
    bool pending_paren_ = false;
};

bool parse_body(Tokenizer &T, std::vector<Dir> &out, bool nested) {
    Dir cur;
    std::string w;
    for (;;) {
        auto ev = T.next(w);
        switch (ev) {
        case Tokenizer::WORD:
            cur.a.push_back(w);
            if (T.take_paren()) cur.a.push_back(")");
            break;
        case Tokenizer::SEMI:
            if (cur.a.empty()) return false;
            out.push_back(std::move(cur)); cur = Dir();
            break;
        case Tokenizer::OPEN:
            cur.block = true;
            if (!parse_body(T, cur.body, true)) return false;
            out.push_back(std::move(cur)); cur = Dir();
            break;
        case Tokenizer::CLOSE:
            return nested && cur.a.empty();
        case Tokenizer::END:
            return !nested && cur.a.empty();
        case Tokenizer::BAD:
            return false;
        }
    }
}

// ============================================================================ IR
enum LocKind { PFX, EXACT, NOREGEX, RX, RXI, NAMED };
// Wallarm parser names (wallarm_parser_disable, annotations.go:320-329) -> DEC_* bits
uint32_t decoder_bit(const std::string &name) {
    if (name == "percent") return DEC_PERCENT;
    if (name == "urlenc") return DEC_URLENC;
    if (name == "json_doc" || name == "json") return DEC_JSON;
    if (name == "base64") return DEC_BASE64;
    return 0;
}

struct Loc {
    int id = 0, server = 0;
    LocKind kind = PFX;
    std::string path;
    bool has_proxy = false, has_return = false, nested = false;
    bool unknown = false;        // a directive outside the known-neutral set (default-deny)
    std::string cmbs;            // client_max_body_size given here ("" inherit)
    std::string ups, err418;
    std::string pass_uri;        // the URI part of proxy_pass (nginx.org/rewrites), "" none
    uint32_t parser_off = 0;     // wallarm_parser_disable in the location (DEC_* bits)
    bool has_pd = false;
    bool pass_vars = false, grpc = false;
    bool stub = false;           // stub_status (a content handler answering 200)
    std::vector<std::pair<bool, std::string>> access;   // allow (false) / deny (true) rules here
    int code = 0;
    int waf = -1;
};
// nocount: an http-level deferral repeated in every server (counted once, at the http block)
struct SIf { std::string var; int op = 0; std::string val; int code = 0; bool ret_only = false; bool nocount = false; };
// realip settings of a server (or the http block, which servers inherit, ngx_http_realip_merge_loc_conf)
struct RealIpIR {
    std::vector<std::string> from;   // set_real_ip_from values, config order
    std::string header;              // real_ip_header value ("" unset)
    int recursive = -1;              // real_ip_recursive (-1 unset)
    bool bad = false;                // a value the engine does not model (a duplicate header)
};
struct Server {
    int id = 0, waf = GM_WAF_OFF;
    uint32_t parser_off = 0;     // server-level wallarm_parser_disable (DEC_* bits)
    std::string cmbs;            // server-level client_max_body_size ("" inherit)
    RealIpIR rip;
    std::vector<std::pair<bool, std::string>> access;   // server-level allow / deny
    std::vector<std::pair<int, int>> listens;   // port, flags (1 ssl, 2 default)
    std::vector<std::string> names;
    std::vector<SIf> ifs;
    std::vector<int> locs;
};
struct MapIR {
    std::string src, var;
    struct P { std::string key; bool rx = false, rxi = false; std::string val; };
    std::vector<P> params;
    bool has_default = false;
    std::string def;
};
struct SplitIR { std::string src, var; std::vector<std::pair<std::string, std::string>> parts; };

// an `upstream` block (version1/nginx.ingress.tmpl:2-8, version2/nginx.virtualserver.tmpl:2-10)
struct UpstreamIR {
    std::string name;
    uint32_t method = UM_RR;
    std::string key;                 // hash / hash consistent key (complex value)
    bool defer = false;              // a construct the engine does not model
    std::string sticky;              // NGINX Plus `sticky cookie <name> ...`: the cookie's name
    struct Peer { std::string addr; bool down = false; };
    std::vector<Peer> peers;
};

struct Model {
    std::vector<Server> servers;
    std::vector<UpstreamIR> upstream_defs;
    std::vector<Loc> locs;
    std::map<std::string, MapIR> maps;
    std::map<std::string, SplitIR> splits;
    std::vector<std::string> upstreams;
    int http_waf = GM_WAF_OFF;
    uint32_t rejected_other = 0, rejected_pcre = 0;
    std::string http_cmbs;       // http-level client_max_body_size ("" = nginx's default 1m)
    RealIpIR http_rip;
    std::vector<std::pair<bool, std::string>> http_access;   // http-level allow / deny
    bool http_unknown = false;   // an http-level directive outside the known set: every server defers
    std::vector<std::string> reject_log;   // "context: directive" of every construct rejected
};

// ---- default-deny.  The directives the compile knows to leave a request's
// verdict alone: what goes upstream (proxy_* / grpc_*), TLS, logging, response headers, timeouts,
// buffers, Wallarm tuning -- everything the reference templates emit besides the directives the
// engine models (version1/nginx.ingress.tmpl, version2/nginx.virtualserver.tmpl, version1/nginx.tmpl
// and their Plus variants).  Any other directive reaching a request (snippets: `deny all;`,
// `auth_basic`, `limit_except`, `internal`, `root` ...) makes it GM_ACT_UNSUPPORTED, counted in
// n_rejected_other and listed by gm_rejects.  Restated in oracle/gm_oracle.c (neutral_directive).
bool neutral_directive(const std::string &n, int ctx /* 0 http, 1 server, 2 location */) {
    static const char *pre[] = {"proxy_", "grpc_", "ssl_", "gzip", "http2_", "open_file_cache", "sub_filter",
                                "keepalive_", "wallarm_"};
    for (const char *p : pre) if (n.rfind(p, 0) == 0) return true;
    static const std::set<std::string> any = {
        "add_header", "add_trailer", "access_log", "error_log", "log_not_found", "log_subrequest",
        "default_type", "charset", "charset_types", "source_charset", "override_charset", "expires", "etag",
        "send_timeout", "client_body_timeout", "client_body_buffer_size", "client_body_temp_path",
        "client_header_timeout", "sendfile", "sendfile_max_chunk", "tcp_nodelay", "tcp_nopush",
        "server_tokens", "status_zone", "chunked_transfer_encoding", "output_buffers", "postpone_output",
        "lingering_close", "lingering_time", "lingering_timeout", "reset_timedout_connection", "resolver",
        "resolver_timeout", "auth_jwt_key_file", "auth_jwt_leeway", "port_in_redirect",
        "server_name_in_redirect", "absolute_redirect", "msie_padding", "msie_refresh"};
    if (any.count(n)) return true;
    if (ctx == 2) return n == "health_check";
    static const std::set<std::string> http = {
        "log_format", "server_names_hash_max_size", "server_names_hash_bucket_size", "variables_hash_max_size",
        "variables_hash_bucket_size", "types_hash_max_size", "types_hash_bucket_size", "map_hash_max_size",
        "map_hash_bucket_size", "limit_req_zone", "limit_conn_zone", "proxy_cache_path", "geo", "match",
        "js_include", "js_import", "keyval_zone", "types"};
    return ctx == 0 && http.count(n);
}

int waf_mode(const std::string &s) {
    if (s == "monitoring") return GM_WAF_MONITORING;
    if (s == "safe_blocking") return GM_WAF_SAFE_BLOCKING;
    if (s == "block") return GM_WAF_BLOCK;
    return GM_WAF_OFF;
}

std::string lower(std::string s) { for (auto &c : s) if (c >= 'A' && c <= 'Z') c |= 0x20; return s; }

bool parse_cidr(const std::string &t, DCidr &c);
// an allow / deny argument the engine reads (ngx_http_access_rule): `all`, `unix:`, an address or
// CIDR; anything else (a host name nginx would refuse) is deferred like an unknown directive
static bool access_arg_ok(const std::string &a) {
    DCidr c;
    return a == "all" || a == "unix:" || parse_cidr(a, c);
}

struct Builder {
    Model &M;
    const std::vector<std::vector<Dir>> &confd;
    explicit Builder(Model &m, const std::vector<std::vector<Dir>> &c) : M(m), confd(c) {}

    // a rejected construct: counted (n_rejected_other) and listed for the Manager's log (gm_rejects)
    void reject(const std::string &where, const Dir &k) {
        std::string t = where + ": ";
        for (size_t q = 0; q < k.a.size() && q < 3; q++) t += (q ? " " : "") + k.a[q];
        M.reject_log.push_back(t);
    }

    void location(Server &S, const Dir &d) {
        Loc L;
        L.id = (int)M.locs.size(); L.server = S.id;
        if (d.a.size() == 3) {
            const std::string &m = d.a[1];
            L.kind = m == "=" ? EXACT : m == "^~" ? NOREGEX : m == "~" ? RX : m == "~*" ? RXI : PFX;
            if (L.kind == PFX) { M.rejected_other++; reject("location", d); }
            L.path = d.a[2];
        } else if (d.a.size() == 2) {
            L.path = d.a[1];
            L.kind = (!L.path.empty() && L.path[0] == '@') ? NAMED : PFX;
        }
        const std::string where = "location " + L.path;
        for (const Dir &k : d.body) {
            if (k.a.empty()) continue;
            const std::string &n = k.a[0];
            // grpc_pass (nginx.org/grpc-services, version1/nginx.ingress.tmpl:154-158) proxies like
            // proxy_pass, auto_redirect included (ngx_http_grpc_module sets clcf->auto_redirect)
            if ((n == "proxy_pass" || n == "grpc_pass") && k.a.size() == 2) {
                std::string u = k.a[1];
                size_t p = u.find("://");
                u = p == std::string::npos ? u : u.substr(p + 3);
                size_t e = u.find_first_of("/$");
                L.ups = u.substr(0, e); L.has_proxy = true;
                L.pass_vars = u.find('$') != std::string::npos;
                L.pass_uri = e != std::string::npos && u[e] == '/' ? u.substr(e) : std::string();
                L.grpc = n == "grpc_pass";
            } else if (n == "return" && k.a.size() >= 2) {
                L.has_return = true;
                L.code = isdigit((unsigned char)k.a[1][0]) ? atoi(k.a[1].c_str()) : 302;
            } else if (n == "error_page" && k.a.size() == 4 && k.a[1] == "418" && k.a[2] == "=") {
                L.err418 = k.a[3];
            } else if (n == "error_page" && k.a.size() >= 3 && k.a.back().rfind("@grpcerror", 0) == 0) {
                // the gRPC error pages (version1/nginx.ingress.tmpl:121-133): a named location that
                // answers the same status, so the verdict does not change
            } else if (n == "wallarm_mode" && k.a.size() == 2) {
                L.waf = waf_mode(k.a[1]);
            } else if (n == "wallarm_parser_disable" && k.a.size() == 2) {
                L.parser_off |= decoder_bit(k.a[1]); L.has_pd = true;
            } else if (n == "client_max_body_size" && k.a.size() == 2) {
                L.cmbs = k.a[1];
            } else if ((n == "allow" || n == "deny") && k.a.size() == 2 && access_arg_ok(k.a[1])) {
                L.access.push_back({n == "deny", k.a[1]});
            } else if (n == "stub_status" && (k.a.size() == 1 || (k.a.size() == 2 && k.a[1] == "on"))) {
                L.stub = true;   // (nginx.tmpl:104-115: the status server's only location)
            } else if (n == "location" || n == "if" || n == "rewrite") {
                L.nested = true;
                reject(where, k);
            } else if (n == "auth_jwt" && k.a.size() == 2 && k.a[1] == "off") {
            } else if (!neutral_directive(n, 2)) {
                L.unknown = true;
                reject(where, k);
            }
        }
        if (L.nested || L.unknown) M.rejected_other++;
        M.locs.push_back(L);
        S.locs.push_back(L.id);
    }

    // realip directives of a server or the http block; false: not one
    static bool realip_dir(RealIpIR &R, const Dir &k) {
        const std::string &n = k.a[0];
        if (n == "set_real_ip_from" && k.a.size() == 2) { R.from.push_back(k.a[1]); return true; }
        if (n == "real_ip_header" && k.a.size() == 2) {
            if (!R.header.empty()) R.bad = true;   // nginx: "is duplicate" (a config error)
            R.header = k.a[1];
            return true;
        }
        if (n == "real_ip_recursive" && k.a.size() == 2) { R.recursive = k.a[1] == "on" ? 1 : 0; return true; }
        return false;
    }

    void server(const Dir &d) {
        Server S;
        S.id = (int)M.servers.size();
        S.waf = M.http_waf;
        for (const Dir &k : d.body) {
            if (k.a.size() == 2 && k.a[0] == "wallarm_mode") S.waf = waf_mode(k.a[1]);
            if (k.a.size() == 2 && k.a[0] == "wallarm_parser_disable") S.parser_off |= decoder_bit(k.a[1]);
        }
        auto defer_here = [&](const Dir &k) {
            // a construct outside the modelled subset: a request that reaches it in the server's
            // directive order defers to nginx (GM_ACT_UNSUPPORTED), counted
            SIf f; f.var = "$uri"; f.op = -1;
            S.ifs.push_back(f);
            reject("server", k);
        };
        for (const Dir &k : d.body) {
            if (k.a.empty()) continue;
            const std::string &n = k.a[0];
            if (n == "listen" && k.a.size() >= 2) {
                const std::string &a = k.a[1];
                if (a.rfind("unix:", 0) == 0) continue;
                size_t c = a.rfind(':');
                int port = atoi((c == std::string::npos ? a : a.substr(c + 1)).c_str());
                int fl = 0;
                for (size_t q = 2; q < k.a.size(); q++) {
                    if (k.a[q] == "ssl") fl |= 1;
                    if (k.a[q] == "default_server" || k.a[q] == "default") fl |= 2;
                    if (k.a[q] == "proxy_protocol") fl |= 4;
                }
                S.listens.push_back({port, fl});
            } else if (n == "server_name") {
                for (size_t q = 1; q < k.a.size(); q++) S.names.push_back(k.a[q][0] == '~' ? k.a[q] : lower(k.a[q]));
            } else if (n == "if" && k.block) {
                std::vector<std::string> a(k.a.begin() + 1, k.a.end());
                if (!a.empty() && !a[0].empty() && a[0][0] == '(') {
                    if (a[0].size() == 1) a.erase(a.begin()); else a[0] = a[0].substr(1);
                }
                if (!a.empty() && !a.back().empty() && a.back().back() == ')') {
                    if (a.back().size() == 1) a.pop_back(); else a.back().pop_back();
                }
                SIf f;
                bool has_ret = false, other = false;
                for (const Dir &r : k.body) {
                    if (r.a.size() >= 2 && r.a[0] == "return") {
                        has_ret = true;
                        f.code = isdigit((unsigned char)r.a[1][0]) ? atoi(r.a[1].c_str()) : 302;
                    } else if (!(r.a.size() >= 2 && r.a[0] == "set" && r.a[1] == "$hsts_header_val")) {
                        other = true;
                    }
                }
                if (other) { defer_here(k); continue; }
                if (!has_ret) continue;   // the HSTS `if` (nginx.ingress.tmpl:66-71) only sets a header value
                if (a.size() == 1) { f.var = a[0]; f.op = 0; }
                else if (a.size() == 3) {
                    f.var = a[0]; f.val = a[2];
                    const std::string &op = a[1];
                    f.op = op == "=" ? 1 : op == "!=" ? 2 : op == "~" ? 3 : op == "~*" ? 4 : op == "!~" ? 5 : op == "!~*" ? 6 : -1;
                } else f.op = -1;
                S.ifs.push_back(f);
            } else if (n == "return" && k.a.size() >= 2) {
                SIf f; f.ret_only = true;
                f.code = isdigit((unsigned char)k.a[1][0]) ? atoi(k.a[1].c_str()) : 302;
                S.ifs.push_back(f);
            } else if (n == "location" && k.block) {
                location(S, k);
            } else if (n == "client_max_body_size" && k.a.size() == 2) {
                S.cmbs = k.a[1];
            } else if ((n == "allow" || n == "deny") && k.a.size() == 2 && access_arg_ok(k.a[1])) {
                S.access.push_back({n == "deny", k.a[1]});
            } else if (realip_dir(S.rip, k)) {
            } else if (n == "set" && k.a.size() >= 2 && k.a[1] == "$hsts_header_val") {
            } else if (n == "error_page" && k.a.size() >= 3 && k.a.back().rfind("@grpcerror", 0) == 0) {
            } else if (n == "auth_jwt" && k.a.size() == 2 && k.a[1] == "off") {
            } else if (n == "rewrite" || !neutral_directive(n, 1)) {
                // (a server-level rewrite, server snippets: not compiled either)
                defer_here(k);
            }
        }
        M.servers.push_back(std::move(S));
    }

    // Balancing method and peers of an upstream block.  The method directive nginx applies is
    // the last one (a second one only warns "load balancing method redefined"); `server`
    // parameters other than the ones the templates emit (max_fails, fail_timeout; slow_start is
    // Plus) and an explicit weight=1 / max_conns=0 make the upstream UM_DEFER.
    void upstream(const Dir &d) {
        UpstreamIR U;
        U.name = d.a[1];
        for (const Dir &k : d.body) {
            if (k.a.empty()) continue;
            const std::string &m = k.a[0];
            if (m == "server" && k.a.size() >= 2) {
                UpstreamIR::Peer p;
                p.addr = k.a[1];
                for (size_t q = 2; q < k.a.size(); q++) {
                    const std::string &a = k.a[q];
                    if (a == "down") p.down = true;
                    else if (a.rfind("max_fails=", 0) == 0 || a.rfind("fail_timeout=", 0) == 0 ||
                             a.rfind("slow_start=", 0) == 0 || a == "weight=1" || a == "max_conns=0") {}
                    else U.defer = true;   // weight, backup, max_conns, resolve, service, route
                }
                U.peers.push_back(p);
            } else if (m == "least_conn" && k.a.size() == 1) U.method = UM_LEAST_CONN;
            else if (m == "ip_hash" && k.a.size() == 1) U.method = UM_IP_HASH;
            else if (m == "hash" && (k.a.size() == 2 || (k.a.size() == 3 && k.a[2] == "consistent"))) {
                U.method = k.a.size() == 3 ? UM_CHASH : UM_HASH;
                U.key = k.a[1];
            } else if (m == "random") {
                if (k.a.size() == 1) U.method = UM_RANDOM;
                else if (k.a[1] == "two" && (k.a.size() == 2 || (k.a.size() == 3 && k.a[2] == "least_conn")))
                    U.method = UM_RANDOM2;
                else U.defer = true;   // random two least_time=... (Plus)
            } else if (m == "sticky" && k.a.size() >= 3 && k.a[1] == "cookie") {
                // NGINX Plus session persistence (nginx-plus.ingress.tmpl:10, nginx.com/sticky-cookie-
                // services, annotations.go:390-395): expires / domain / path / httponly / secure only
                // shape the Set-Cookie of the response, not the choice
                U.sticky = k.a[2];
            } else if (m == "least_time" || m == "sticky" || m == "queue" || m == "ntlm" || m == "hash") {
                U.defer = true;   // sticky route / learn, ...
            }
            // keepalive, zone, keepalive_timeout / _requests: connection reuse, not the choice
        }
        M.upstream_defs.push_back(std::move(U));
    }

    void http(const std::vector<Dir> &body) {
        for (const Dir &d : body) {
            if (d.a.empty()) continue;
            const std::string &n = d.a[0];
            if (n == "include" && d.a.size() == 2 && d.a[1].find("conf.d/") != std::string::npos) {
                for (auto &f : confd) http(f);
            } else if (n == "include" && d.a.size() == 2 &&
                       (d.a[1] == "/etc/nginx/mime.types" || d.a[1] == "mime.types" ||
                        d.a[1] == "/etc/nginx/config-version.conf")) {
                // MIME types; the config-version server (verify.go:81-92, a unix-socket listener)
            } else if (n == "client_max_body_size" && d.a.size() == 2) {
                M.http_cmbs = d.a[1];
            } else if ((n == "allow" || n == "deny") && d.a.size() == 2 && access_arg_ok(d.a[1])) {
                M.http_access.push_back({n == "deny", d.a[1]});
            } else if (realip_dir(M.http_rip, d)) {
            } else if (n == "wallarm_mode" && d.a.size() == 2) {
                M.http_waf = waf_mode(d.a[1]);
            } else if (n == "upstream" && d.block && d.a.size() == 2) {
                M.upstreams.push_back(d.a[1]);
                upstream(d);
            } else if (n == "map" && d.block && d.a.size() == 3) {
                MapIR m;
                m.src = d.a[1]; m.var = lower(d.a[2].substr(1));
                for (const Dir &p : d.body) {
                    if (p.a.size() == 1 && (p.a[0] == "hostnames" || p.a[0] == "volatile")) continue;
                    if (p.a.size() != 2) continue;
                    if (p.a[0] == "default") { m.has_default = true; m.def = p.a[1]; continue; }
                    if (p.a[0] == "include") continue;
                    MapIR::P q;
                    q.val = p.a[1];
                    std::string k = p.a[0];
                    if (!k.empty() && k[0] == '~') {
                        q.rx = true;
                        if (k.size() > 1 && k[1] == '*') { q.rxi = true; q.key = k.substr(2); }
                        else q.key = k.substr(1);
                    } else {
                        if (!k.empty() && k[0] == '\\') k = k.substr(1);
                        q.key = lower(k);
                    }
                    m.params.push_back(q);
                }
                M.maps[m.var] = m;
            } else if (n == "split_clients" && d.block && d.a.size() == 3) {
                SplitIR s;
                s.src = d.a[1]; s.var = lower(d.a[2].substr(1));
                for (const Dir &p : d.body) if (p.a.size() == 2) s.parts.push_back({p.a[0], p.a[1]});
                M.splits[s.var] = s;
            } else if (n == "server" && d.block) {
                server(d);
            } else if (!neutral_directive(n, 0)) {
                // applies to every server (access-phase directives, http snippets): every request
                // defers after its server's rewrite phase
                if (!M.http_unknown) M.rejected_other++;
                M.http_unknown = true;
                reject("http", d);
            }
        }
    }
};

// ============================================================================ image writer
struct Image {
    std::vector<uint8_t> buf;
    template <class T> uint64_t put(const std::vector<T> &v) {
        size_t off = (buf.size() + 15) & ~size_t(15);
        buf.resize(off + v.size() * sizeof(T) + 16, 0);
        if (!v.empty()) memcpy(buf.data() + off, v.data(), v.size() * sizeof(T));
        buf.resize(off + v.size() * sizeof(T));
        return off;
    }
};

// A superset of a PCRE-only regex in the RE2 subset, or "" when there is none here: lookaround
// groups dropped, atomic groups made plain, possessive quantifiers made greedy, \K dropped,
// backreferences widened to (?:.|\n)*.  Every subject the original matches, the relaxed
// pattern matches too, so a regex location whose relaxed DFA does not match a URI is skipped
// exactly; one that matches is deferred (GM_ACT_UNSUPPORTED).  Restated in oracle/gm_oracle.c
// (orc_relax).
static std::string relax_pcre_only(const std::string &p) {
    std::string o;
    const size_t n = p.size();
    bool cls = false;
    for (size_t i = 0; i < n; i++) {
        const char ch = p[i];
        if (ch == '\\' && i + 1 < n) {
            const char e = p[i + 1];
            if (!cls && e >= '1' && e <= '9') { o += "(?:.|\\n)*"; i++; continue; }
            if (!cls && e == 'K') { i++; continue; }
            if (!cls && (e == 'g' || e == 'k')) return "";
            o += ch; o += e; i++;
            continue;
        }
        if (cls) { o += ch; if (ch == ']') cls = false; continue; }
        if (ch == '[') {
            cls = true; o += ch;
            if (i + 1 < n && p[i + 1] == '^') o += p[++i];
            if (i + 1 < n && p[i + 1] == ']') o += p[++i];
            continue;
        }
        if (ch == '(' && i + 2 < n && p[i + 1] == '?') {
            const char a = p[i + 2];
            const bool look = a == '=' || a == '!' || (a == '<' && i + 3 < n && (p[i + 3] == '=' || p[i + 3] == '!'));
            if (look) {   // skip to the matching ')'
                int depth = 0;
                bool c2 = false;
                size_t j = i;
                for (; j < n; j++) {
                    if (p[j] == '\\') { j++; continue; }
                    if (c2) { if (p[j] == ']') c2 = false; continue; }
                    if (p[j] == '[') { c2 = true; if (j + 1 < n && p[j + 1] == '^') j++; if (j + 1 < n && p[j + 1] == ']') j++; continue; }
                    if (p[j] == '(') depth++;
                    else if (p[j] == ')' && --depth == 0) break;
                }
                if (j >= n) return "";
                i = j;
                if (i + 1 < n && (p[i + 1] == '*' || p[i + 1] == '+' || p[i + 1] == '?' || p[i + 1] == '{')) return "";
                continue;
            }
            if (a == '>') { o += "(?:"; i += 2; continue; }
            if (a == 'R' || a == '(' || a == 'C' || a == 'P' || a == '&' || a == '|' || (a >= '0' && a <= '9')) return "";
        }
        if ((ch == '*' || ch == '+' || ch == '?' || ch == '}') && i + 1 < n && p[i + 1] == '+' &&
            !(ch == '?' && i > 0 && p[i - 1] == '(')) { o += ch; i++; continue; }
        o += ch;
    }
    return o;
}

uint32_t pow2_at_least(size_t n) { uint32_t c = 16; while (c < n) c <<= 1; return c; }

// client_max_body_size (ngx_parse_offset): decimal digits with an optional k / m / g suffix;
// 0 = no limit.  BODY_UNLIMITED for 0 and for limits no u32 body length can pass; -1: not a size
int64_t parse_body_max(const std::string &v) {
    if (v.empty()) return -1;
    size_t n = v.size();
    uint64_t scale = 1;
    const char u = v[n - 1];
    if (u == 'k' || u == 'K') { scale = 1024; n--; }
    else if (u == 'm' || u == 'M') { scale = 1024 * 1024; n--; }
    else if (u == 'g' || u == 'G') { scale = 1024ull * 1024 * 1024; n--; }
    if (n == 0) return -1;
    uint64_t x = 0;
    for (size_t i = 0; i < n; i++) {
        if (v[i] < '0' || v[i] > '9') return -1;
        x = x * 10 + (uint64_t)(v[i] - '0');
        if (x > (1ull << 40)) return BODY_UNLIMITED;   // past any u32 body length either way
    }
    x *= scale;
    return x == 0 || x >= BODY_UNLIMITED ? (int64_t)BODY_UNLIMITED : (int64_t)x;
}

// ngx_ptocidr: "addr[/bits]" -> family + masked network-order bytes; false: not an address
// (nginx would resolve a host name here: the engine does not)
bool parse_cidr(const std::string &t, DCidr &c) {
    memset(&c, 0, sizeof c);
    const size_t sl = t.find('/');
    const std::string a = sl == std::string::npos ? t : t.substr(0, sl);
    uint8_t b[16] = {0}, m[16] = {0};
    const uint32_t fam = ngx_parse_addr((const uint8_t *)a.data(), (uint32_t)a.size(), b);
    if (!fam) return false;
    const uint32_t nb = fam == 4 ? 4 : 16;
    int64_t bits = (int64_t)nb * 8;
    if (sl != std::string::npos) {
        bits = ngx_atoi_dec((const uint8_t *)t.data() + sl + 1, (uint32_t)(t.size() - sl - 1));
        if (bits < 0 || bits > (int64_t)nb * 8) return false;
    }
    for (uint32_t i = 0; i < nb; i++) {
        const int64_t k = bits - 8 * (int64_t)i;
        m[i] = k >= 8 ? 0xFF : k <= 0 ? 0 : (uint8_t)(0xFF << (8 - k));
        b[i] &= m[i];   // nginx warns "low address bits are meaningless" and clears them
    }
    c.family = fam;
    memcpy(c.addr, b, 16);
    memcpy(c.mask, m, 16);
    return true;
}

struct Compiler {
    Model &M;
    gm_stats_t &st;
    std::vector<uint8_t> bytes;                  // shared byte pool
    std::vector<DSrc> srcs;
    std::map<std::string, uint32_t> src_ids;
    std::vector<DCond> conds;
    std::vector<uint32_t> chain_heads;
    std::vector<DRules> rules;
    std::vector<uint8_t> rtab;
    std::vector<uint32_t> rtargets;
    std::vector<DSplit> splits;
    std::vector<DPart> parts;
    std::vector<DDfa> dfas;
    std::vector<uint16_t> dfa_trans;
    std::vector<uint8_t> dfa_acc, dfa_cls;

    Compiler(Model &m, gm_stats_t &s) : M(m), st(s) {}

    uint32_t put_bytes(const std::string &s) {
        uint32_t o = (uint32_t)bytes.size();
        bytes.insert(bytes.end(), s.begin(), s.end());
        return o;
    }

    int add_dfa(const Dfa &d) {
        DDfa x{};
        x.trans_off = (uint32_t)dfa_trans.size();
        x.acc_off = (uint32_t)dfa_acc.size();
        x.cls_off = (uint32_t)dfa_cls.size();
        x.n_states = (uint16_t)d.n_states; x.n_classes = (uint16_t)d.n_classes;
        x.flags = d.anchored_start ? DFA_ANCHOR_START : 0;
        // entries carry the target's accept flags in bits 14-15 (DFA_TRANS_STATE_MASK): the
        // device step is one dependent load per byte, not a transition load then a flags load
        for (uint16_t e : d.trans) dfa_trans.push_back((uint16_t)(e | (uint16_t)((d.acc[e] & 3u) << 14)));
        dfa_acc.insert(dfa_acc.end(), d.acc.begin(), d.acc.end());
        dfa_cls.insert(dfa_cls.end(), d.cls, d.cls + 256);
        dfas.push_back(x);
        st.n_dfa_states += d.n_states;
        return (int)dfas.size() - 1;
    }

    // regex -> dfa id, or -1 (counted)
    // superset: for a PCRE-only pattern, compile relax_pcre_only(pat) instead (still counted as
    // rejected) and report it through *superset
    int regex(const std::string &pat, bool ci, Dfa *keep = nullptr, std::vector<std::string> *factors = nullptr,
              bool *superset = nullptr) {
        RegexInfo ri = compile_regex(pat, ci);
        if (superset) *superset = false;
        if (ri.status == RX_PCRE_ONLY && superset) {
            st.n_rejected_pcre++;
            const std::string rp = relax_pcre_only(pat);
            if (rp.empty()) return -1;
            ri = compile_regex(rp, ci);
            if (ri.status != RX_OK) return -1;
            *superset = true;
        } else if (ri.status != RX_OK) {
            if (ri.status == RX_PCRE_ONLY) st.n_rejected_pcre++; else st.n_rejected_other++;
            return -1;
        }
        if (keep) *keep = ri.dfa;
        if (factors) { factors->clear(); if (ri.min_factor >= 4) *factors = ri.factors; }
        return add_dfa(ri.dfa);
    }

    // request variable "$name" -> DSrc id, or -1
    int src(const std::string &var) {
        if (var.size() < 2 || var[0] != '$') return -1;
        std::string n = lower(var.substr(1));
        if (n.size() > 2 && n[0] == '{' && n.back() == '}') n = n.substr(1, n.size() - 2);
        auto it = src_ids.find(n);
        if (it != src_ids.end()) return (int)it->second;
        DSrc s{};
        static const std::map<std::string, uint8_t> vars = {
            {"scheme", V_SCHEME}, {"https", V_HTTPS}, {"http2", V_HTTP2}, {"request_method", V_METHOD},
            {"args", V_ARGS}, {"query_string", V_ARGS}, {"uri", V_URI}, {"document_uri", V_URI},
            {"request_uri", V_REQUEST_URI}, {"request", V_REQUEST}, {"request_body", V_REQUEST_BODY},
            {"remote_addr", V_REMOTE_ADDR}, {"remote_port", V_REMOTE_PORT}, {"server_port", V_SERVER_PORT},
            {"request_id", V_REQUEST_ID}, {"host", V_HOST}};
        auto v = vars.find(n);
        if (v != vars.end()) { s.kind = SRC_VAR; s.var = v->second; }
        else if (n.rfind("http_", 0) == 0 && n.size() > 5) {
            s.kind = SRC_HTTP;
            std::string h = n.substr(5);
            s.join = h == "cookie" ? ';' : h == "x_forwarded_for" ? ',' : 0;
            s.name_off = put_bytes(h); s.name_len = (uint32_t)h.size();
        } else if (n.rfind("cookie_", 0) == 0 && n.size() > 7) {
            s.kind = SRC_COOKIE; std::string h = n.substr(7);
            s.name_off = put_bytes(h); s.name_len = (uint32_t)h.size();
        } else if (n.rfind("arg_", 0) == 0 && n.size() > 4) {
            s.kind = SRC_ARG; std::string h = n.substr(4);
            s.name_off = put_bytes(h); s.name_len = (uint32_t)h.size();
        } else return -1;
        srcs.push_back(s);
        src_ids[n] = (uint32_t)srcs.size() - 1;
        return (int)srcs.size() - 1;
    }

    // split a complex value into $var parts; returns false if literal text is mixed in
    static bool var_list(const std::string &v, std::vector<std::string> &out) {
        size_t i = 0;
        while (i < v.size()) {
            if (v[i] != '$') return false;
            size_t j = i + 1;
            if (j < v.size() && v[j] == '{') {
                size_t e = v.find('}', j);
                if (e == std::string::npos) return false;
                out.push_back(lower(v.substr(j + 1, e - j - 1))); i = e + 1; continue;
            }
            while (j < v.size() && (isalnum((unsigned char)v[j]) || v[j] == '_')) j++;
            if (j == i + 1) return false;
            out.push_back(lower(v.substr(i + 1, j - i - 1)));
            i = j;
        }
        return !out.empty();
    }

    // chain map var -> node id (NEXT_0 / NEXT_1 for constants); INT32_MIN = unsupported
    std::map<std::string, int32_t> chain_memo;
    int32_t chain(const std::string &var, int depth) {
        if (depth > 64) return INT32_MIN;
        auto it = chain_memo.find(var);
        if (it != chain_memo.end()) return it->second;
        auto mit = M.maps.find(var);
        if (mit == M.maps.end()) return INT32_MIN;
        const MapIR &m = mit->second;
        std::vector<std::string> sv;
        if (!var_list(m.src, sv) || sv.size() != 1) return INT32_MIN;
        int s = src("$" + sv[0]);
        if (s < 0 || m.params.size() > 1) return INT32_MIN;
        auto res = [&](const std::string &r) -> int32_t {
            if (r == "0") return NEXT_0;
            if (r == "1") return NEXT_1;
            std::vector<std::string> rv;
            if (var_list(r, rv) && rv.size() == 1) return chain(rv[0], depth + 1);
            return INT32_MIN;
        };
        int32_t f = res(m.has_default ? m.def : std::string(""));
        if (m.params.empty()) { chain_memo[var] = f; return f; }
        const MapIR::P &p = m.params[0];
        int32_t t = res(p.val);
        if (t == INT32_MIN || f == INT32_MIN) return INT32_MIN;
        DCond c{};
        c.src = (uint32_t)s;
        if (p.rx) {
            int d = regex(p.key, p.rxi);
            if (d < 0) return INT32_MIN;
            c.is_regex = 1; c.dfa = (uint32_t)d;
        } else {
            c.key_off = put_bytes(p.key); c.key_len = (uint32_t)p.key.size();
        }
        c.next_true = t; c.next_false = f;
        conds.push_back(c);
        int32_t id = (int32_t)conds.size() - 1;
        chain_memo[var] = id;
        return id;
    }

    // IRL target "@name" -> named location id in server S; GM_NONE for empty; -2 unsupported
    int64_t target(const Server &S, const std::string &v) {
        if (v.empty()) return GM_NONE;
        if (v.find('$') != std::string::npos || v[0] != '@') return -2;
        for (int l : S.locs) if (M.locs[l].kind == NAMED && M.locs[l].path == v) return l;
        return -2;
    }

    // rules route for IRL in server S referencing map `var`; returns DRules index or -1
    int rules_route(const Server &S, const std::string &var) {
        const MapIR &m = M.maps.at(var);
        std::vector<std::string> chains;
        if (!var_list(m.src, chains) || chains.size() > RULES_CHAINS_MAX) return -1;
        DRules r{};
        r.first_chain = (uint32_t)chain_heads.size();
        r.n_chains = (uint32_t)chains.size();
        std::vector<uint32_t> heads;
        for (auto &c : chains) {
            int32_t h = chain(c, 0);
            if (h == INT32_MIN) return -1;
            heads.push_back((uint32_t)h);
        }
        // result of each param: literal "@name"
        std::vector<uint32_t> tg;
        std::vector<Dfa> rx(m.params.size());
        for (size_t k = 0; k < m.params.size(); k++) {
            int64_t t = target(S, m.params[k].val);
            if (t == -2) return -1;
            tg.push_back((uint32_t)t);
            if (m.params[k].rx) {
                RegexInfo ri = compile_regex(m.params[k].key, m.params[k].rxi);
                if (ri.status != RX_OK) {
                    if (ri.status == RX_PCRE_ONLY) st.n_rejected_pcre++; else st.n_rejected_other++;
                    return -1;
                }
                rx[k] = ri.dfa;
            }
        }
        int64_t dt = m.has_default ? target(S, m.def) : (int64_t)GM_NONE;
        if (dt == -2) return -1;
        if (chains.size() > RULES_TABLE_MAX) {
            // too many chains for a 2^n truth table: the map's params as conditions over the
            // chains' '0'/'1' string, evaluated on the device in ngx_http_map_find's order (the
            // exact keys, then the regexes in config order); DRules.pad[0] = the first
            r.table_off = GM_NONE;
            r.pad[0] = (uint32_t)conds.size();
            std::vector<DCond> pc;
            for (size_t k = 0; k < m.params.size(); k++) {
                DCond c{};
                if (m.params[k].rx) {
                    const int d = regex(m.params[k].key, m.params[k].rxi);
                    if (d < 0) return -1;
                    c.is_regex = 1; c.dfa = (uint32_t)d;
                } else {
                    c.key_off = put_bytes(m.params[k].key); c.key_len = (uint32_t)m.params[k].key.size();
                }
                pc.push_back(c);
            }
            conds.insert(conds.end(), pc.begin(), pc.end());
        } else {
        // truth table over the chains' 0/1 outcomes (ngx_http_map_find: hash, then regexes)
        r.table_off = (uint32_t)rtab.size();
        for (uint32_t b = 0; b < (1u << chains.size()); b++) {
            std::string s;
            for (size_t c = 0; c < chains.size(); c++) s.push_back((b >> c) & 1 ? '1' : '0');
            int res = -1;
            for (size_t k = 0; k < m.params.size() && res < 0; k++)
                if (!m.params[k].rx && m.params[k].key == s) res = (int)k;
            for (size_t k = 0; k < m.params.size() && res < 0; k++)
                if (m.params[k].rx && !s.empty() && dfa_search(rx[k], (const uint8_t *)s.data(), s.size())) res = (int)k;
            rtab.push_back(res < 0 ? 0xFF : (uint8_t)res);
        }
        }
        for (auto h : heads) chain_heads.push_back(h);
        r.first_target = (uint32_t)rtargets.size();
        r.n_targets = (uint32_t)tg.size();
        for (auto t : tg) rtargets.push_back(t);
        r.default_target = (uint32_t)dt;
        rules.push_back(r);
        return (int)rules.size() - 1;
    }

    int split_route(const Server &S, const std::string &var) {
        const SplitIR &sp = M.splits.at(var);
        std::vector<std::string> sv;
        if (!var_list(sp.src, sv) || sv.size() != 1) return -1;
        int s = src("$" + sv[0]);
        if (s < 0) return -1;
        DSplit d{};
        d.first_part = (uint32_t)parts.size(); d.src = (uint32_t)s;
        uint64_t last = 0;
        std::vector<DPart> ps;
        for (auto &p : sp.parts) {
            DPart q{};
            int64_t t = target(S, p.second);
            if (t == -2) return -1;
            q.target = (uint32_t)t;
            if (p.first == "*") { q.star = 1; }
            else {
                // ngx_atofp(value, len - 1, 2)
                const std::string &w = p.first;
                if (w.empty() || w.back() != '%') return -1;
                uint32_t pc = 0; int dec = -1;
                for (size_t k = 0; k + 1 < w.size(); k++) {
                    char c = w[k];
                    if (c == '.') { if (dec >= 0) return -1; dec = 0; continue; }
                    if (!isdigit((unsigned char)c)) return -1;
                    if (dec >= 0) { if (dec < 2) { pc = pc * 10 + (c - '0'); dec++; } }
                    else pc = pc * 10 + (c - '0');
                }
                for (int k = dec < 0 ? 0 : dec; k < 2; k++) pc *= 10;
                last += (uint64_t)pc * 0xffffffffull / 10000;
                q.bound = (uint32_t)last;
            }
            ps.push_back(q);
        }
        d.n_parts = (uint32_t)ps.size();
        for (auto &q : ps) parts.push_back(q);
        splits.push_back(d);
        return (int)splits.size() - 1;
    }
};

// ============================================================================ signatures
struct SigRule { bool lit; bool nocase; int zones; std::string pat; };

static int hexv(char c) {
    return c >= '0' && c <= '9' ? c - '0' : (c | 0x20) >= 'a' && (c | 0x20) <= 'f' ? (c | 0x20) - 'a' + 10 : -1;
}

// One rule per line: "lit|re <i|-> <zones> <hex literal | regex>"; "@decoders a,b,..." names the
// request parsers whose decoded views the set's rules are written against (DEC_*).
bool parse_sigs(const char *t, size_t n, std::vector<SigRule> &out, uint32_t &decoders) {
    size_t i = 0;
    while (i < n) {
        size_t e = i;
        while (e < n && t[e] != '\n') e++;
        std::string line(t + i, e - i);
        i = e + 1;
        while (!line.empty() && (line.back() == '\r' || line.back() == ' ' || line.back() == '\t')) line.pop_back();
        size_t s = line.find_first_not_of(" \t");
        if (s == std::string::npos || line[s] == '#') continue;
        line = line.substr(s);
        if (line.rfind("@decoders", 0) == 0) {
            std::string v = line.substr(9);
            size_t a = 0;
            while (a < v.size()) {
                size_t b = v.find(',', a);
                if (b == std::string::npos) b = v.size();
                std::string nm = v.substr(a, b - a);
                nm.erase(0, nm.find_first_not_of(" \t"));
                nm.erase(nm.find_last_not_of(" \t") + 1);
                decoders |= decoder_bit(nm);
                a = b + 1;
            }
            continue;
        }
        std::string f[3];
        size_t p = 0;
        for (int k = 0; k < 3; k++) {
            size_t q = line.find(' ', p);
            if (q == std::string::npos) return false;
            f[k] = line.substr(p, q - p);
            p = line.find_first_not_of(' ', q);
            if (p == std::string::npos) return false;
        }
        SigRule r;
        r.lit = f[0] == "lit";
        if (!r.lit && f[0] != "re") return false;
        r.nocase = f[1] == "i";
        r.zones = 0;
        for (char z : f[2]) r.zones |= z == 'u' ? 1 : z == 'a' ? 2 : z == 'h' ? 4 : z == 'b' ? 8 : 0;
        std::string pat = line.substr(p);
        if (r.lit) {
            if (pat.size() % 2) return false;
            for (size_t k = 0; k < pat.size(); k += 2) {
                const int hi = hexv(pat[k]), lo = hexv(pat[k + 1]);
                if (hi < 0 || lo < 0) return false;
                r.pat.push_back((char)(hi * 16 + lo));
            }
        } else r.pat = pat;
        out.push_back(r);
    }
    return true;
}

uint32_t load4(const std::string &s, size_t o = 0) {
    return (uint32_t)(uint8_t)s[o] | (uint32_t)(uint8_t)s[o + 1] << 8 | (uint32_t)(uint8_t)s[o + 2] << 16 |
           (uint32_t)(uint8_t)s[o + 3] << 24;
}

// Key window choice: the prefilter's candidate rate is dominated by 4-grams that benign
// traffic really contains ("from", "into", "inse", "form"...), so each literal is keyed on its
// least probable window under a unigram English/HTTP byte-frequency model (any window is
// correct: verification re-checks the whole literal at pos - key_off).
double byte_logfreq(uint8_t c) {
    static const double letters[26] = {8.2, 1.5, 2.8, 4.3, 12.7, 2.2, 2.0, 6.1, 7.0, 0.15, 0.8, 4.0, 2.4,
                                       6.7, 7.5, 1.9, 0.1, 6.0, 6.3, 9.1, 2.8, 1.0, 2.4, 0.15, 2.0, 0.07};
    double f;
    if (c >= 'A' && c <= 'Z') c |= 0x20;
    if (c >= 'a' && c <= 'z') f = letters[c - 'a'] * 0.8;
    else if (c == ' ') f = 15.0;
    else if (c >= '0' && c <= '9') f = 1.5;                  // ids, timestamps, addresses
    else if (strchr("/.-_=&:,;\r\n", c) && c) f = 2.0;       // URL / form / header punctuation
    else if (c >= 0x20 && c < 0x7f) f = 0.2;
    else f = 0.05;
    return std::log2(f);
}

// Background model: 4-grams of frequent English words and HTTP header tokens.  A window that
// occurs in ordinary text is a bad prefilter key however rare its letters are ("from", "kind").
const char *kBackground =
    "the of and to in is it you that he was for on are with as his they be at one have this from or had "
    "by hot word but what some we can out other were all there when up use your how said an each she "
    "which do their time if will way about many then them write would like so these her long make thing "
    "see him two has look more day could go come did number sound no most people my over know water "
    "than call first who may down side been now find any new work part take get place made live where "
    "after back little only round man year came show every good me give our under name very through "
    "just form sentence great think say help low line differ turn cause much mean before move right boy "
    "old too same tell does set three want air well also play small end put home read hand port large "
    "spell add even land here must big high such follow act why ask men change went light kind off need "
    "house picture try us again animal point mother world near build self earth father head stand own "
    "page should country found answer school grow study still learn plant cover food sun four between "
    "state keep eye never last let thought city tree cross farm hard start might story saw far sea draw "
    "left late run don't while press close night real life few north open seem together next white "
    "children begin got walk example ease paper group always music those both mark often letter until "
    "mile river car feet care second book carry took science eat room friend began idea fish mountain "
    "stop once base hear horse cut sure watch color face wood main enough plain girl usual young ready "
    "above ever red list though feel talk bird soon body dog family direct pose leave song measure door "
    "product black short numeral class wind question happen complete ship area half rock order fire "
    "south problem piece told knew pass since top whole king space heard best hour better true during "
    "hundred five remember step early hold west ground interest reach fast verb sing listen six table "
    "travel less morning ten simple several vowel toward war lay against pattern slow center love person "
    "money serve appear road map rain rule govern pull cold notice voice unit power town fine certain fly "
    "fall lead cry dark machine note wait plan figure star box noun field rest correct able pound done "
    "beauty drive stood contain front teach week final gave green quick develop ocean warm free minute "
    "strong special mind behind clear tail produce fact street inch multiply nothing course stay wheel "
    "full force blue object decide surface deep moon island foot system busy test record boat common "
    "gold possible plane stead dry wonder laugh thousand ago ran check game shape equate miss brought "
    "heat snow tire bring yes distant fill east paint language among customer price cart checkout "
    "account login session token user email address phone item items quantity total shipping billing "
    "status created updated update insert delete select value values content information schema "
    "mozilla windows linux x86_64 applewebkit khtml like gecko chrome safari firefox text/html "
    "application/json application/xml application/xhtml+xml image/webp accept language encoding gzip "
    "deflate keep-alive connection cache-control no-cache max-age referer origin cookie set-cookie "
    "authorization bearer content-type content-length user-agent host http https www. .com .org .net "
    "navigate same-origin cors upgrade-insecure-requests x-forwarded-for x-request x-trace-id "
    "if-none-match etag utf-8 charset boundary multipart form-data urlencoded";

// Standard request header lines as they sit in a header block (CRLF-separated): every request
// carries a dozen of them, so their folded 4-grams ("\r\nUs" -> "-*us") are the most frequent
// windows a scan sees and must not test positive in the prefilter.
const char *kHeaderLines[] = {
    "Host: ", "User-Agent: Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko)",
    "Accept: text/html,application/xhtml+xml,application/xml;q=0.9,image/webp,*/*;q=0.8",
    "Accept-Language: en-US,en;q=0.9", "Accept-Encoding: gzip, deflate, br", "Connection: keep-alive",
    "Referer: https://www.", "Cache-Control: no-cache, max-age=0", "Upgrade-Insecure-Requests: 1",
    "X-Forwarded-For: ", "X-Forwarded-Proto: https", "X-Real-IP: ", "X-Request-ID: ", "X-Requested-With: ",
    "Sec-Fetch-Mode: navigate", "Sec-Fetch-Site: same-origin", "Sec-Fetch-Dest: document", "DNT: 1",
    "Pragma: no-cache", "Origin: https://", "Content-Type: application/json", "Content-Length: ",
    "Authorization: Bearer ", "If-None-Match: W/\"", "If-Modified-Since: ", "Cookie: session=",
    "X-Client-Version: ", "X-Trace-Id: ", "X-Request-Start: t="};
// separators words meet in URIs, query strings, JSON, form data and text
const char *kSeps[] = {" ", "\n", "\r\n", "_", "-", "/", ":", "=", "&", ".", ",", "\"", "\": \"", ", ", ". "};

// folded 4-gram -> relative weight (header-line grams 16, word/separator grams by word rank)
const std::unordered_map<uint32_t, double> &background_weights() {
    static std::unordered_map<uint32_t, double> g = [] {
        std::unordered_map<uint32_t, double> m;
        auto add = [&](const std::string &t, double wt) {
            for (size_t i = 0; i + 4 <= t.size(); i++) {
                uint32_t w;
                memcpy(&w, t.data() + i, 4);
                double &x = m[fold4(w)];
                x = std::max(x, wt);
            }
        };
        add(std::string(kBackground), 0.05);
        std::vector<std::string> words;
        {
            std::string t(kBackground), cur;
            for (char ch : t) { if (ch == ' ') { if (!cur.empty()) words.push_back(cur); cur.clear(); } else cur += ch; }
            if (!cur.empty()) words.push_back(cur);
        }
        // kBackground lists the English words by frequency: Zipf weights by rank
        for (size_t r = 0; r < words.size(); r++)
            for (const char *a : kSeps)
                for (const char *b : kSeps) add(std::string(a) + words[r] + b, 50.0 / (double)(r + 10));
        std::string hb;
        for (const char *h : kHeaderLines) hb += std::string("\r\n") + h + "\r\n";
        add(hb, 16.0);
        return m;
    }();
    return g;
}

const std::set<uint32_t> &background_grams() {
    static std::set<uint32_t> g = [] {
        std::set<uint32_t> s;
        for (auto &kv : background_weights()) s.insert(kv.first);
        return s;
    }();
    return g;
}

// folded 3-grams of the background corpus, including word boundaries seen as separators
// ("lay" of "play_" / "delay="): a window containing one is only somewhat rarer than the word
const std::set<uint32_t> &background_grams3() {
    static std::set<uint32_t> g = [] {
        std::set<uint32_t> s;
        std::string t(kBackground);
        for (size_t i = 0; i + 3 <= t.size(); i++)
            s.insert(fold4((uint8_t)t[i] | (uint32_t)(uint8_t)t[i + 1] << 8 | (uint32_t)(uint8_t)t[i + 2] << 16) &
                     0xFFFFFFu);
        return s;
    }();
    return g;
}

// model score of a folded window: log2 of a relative frequency, +40 for background 4-grams,
// +6 per background 3-gram (word-internal)
double window_score_w(uint32_t w) {
    double s = 0;
    for (int k = 0; k < 4; k++) s += byte_logfreq((uint8_t)(w >> (8 * k)));
    if (background_grams().count(w)) s += 40.0;
    for (int k = 0; k < 2; k++) {
        const uint32_t g3 = (w >> (8 * k)) & 0xFFFFFFu;
        if ((g3 & 0xFF) != ' ' && (g3 >> 16) != ' ' && background_grams3().count(g3)) s += 6.0;
    }
    return s;
}

// Expected benign occurrences of a folded 4-gram key window.  With a traffic sample in the
// generation blob (GM_ENTRY_SAMPLE: bytes of benign requests, as a deployment would sample its
// own traffic) the count in the sample decides; the byte/background model above only ranks
// windows the sample does not contain.  Without a sample the model alone decides.
struct KeyModel {
    std::unordered_map<uint32_t, uint32_t> cnt;
    double n = 0;
    void add_sample(const uint8_t *b, size_t len) {
        for (size_t i = 0; i + 4 <= len; i++) {
            uint32_t w;
            memcpy(&w, b + i, 4);
            cnt[fold4(w)]++;
        }
        n += len >= 4 ? (double)(len - 3) : 0.0;
    }
    double cost(uint32_t w) const {
        const double prior = std::exp2(window_score_w(w));
        if (n == 0) return prior;
        auto it = cnt.find(w);
        // the model's term is squashed into (0, 1): it ranks the windows the sample does not hold
        // and never outweighs one observed occurrence (round 6: unsquashed, an unseen window could
        // score ~350 and lose to one the sample held ~1800 times once the context penalty applied)
        const double m = n * prior * std::exp2(-28.0);
        return (it == cnt.end() ? 0.0 : (double)it->second) + m / (1.0 + m);
    }
};

// A prefix-mode regex's anchored DFA after its prefix literal f (k_waf_exact starts the run there:
// the literal is already verified), as a transition entry (state | accept flags << 14); 0 = run
// from the start.  Valid only when the arena's bytes take the same path as f's: the literal is
// matched case-insensitively, so a case-sensitive regex qualifies only if f has no letters.  A
// state on the way that accepts makes the entry accepting (the run would have stopped there); a
// '\n' in f keeps the full run (PCRE's "$ before a final newline" looks at the subject's last byte).
uint16_t prefix_entry(const Dfa &d, const std::string &f, bool nocase) {
    if (d.n_states == 0 || d.n_states > (int)DFA_TRANS_STATE_MASK) return 0;
    uint32_t s = 1, fl = d.acc[1] & 3u;
    for (unsigned char c : f) {
        if (c == '\n' || (!nocase && ((c | 0x20) >= 'a' && (c | 0x20) <= 'z'))) return 0;
        if (fl & 1u) break;
        s = d.trans[(size_t)s * d.n_classes + d.cls[c]];
        if (s == 0) return 0;
        fl = d.acc[s] & 3u;
    }
    return (uint16_t)(s | (fl << 14));
}

// The scan probes only even arena offsets (k_waf_scan), so every pattern is keyed on a set of
// windows that catches an occurrence at either parity: an occurrence at an even arena offset is
// probed at the pattern's even offsets, one at an odd arena offset at its odd offsets, so the keys
// are one EVEN-offset choice plus one ODD-offset choice, each either
//   a window inside the pattern (o, o + 4 <= L), or
//   a family: the window one byte past either end, for each of the 128 folded values of that byte
//   ("Zabc", key_off -1: odd; "xyzY", key_off L - 3) -- the only choice of a 4-byte pattern's odd
//   class, and what a 5- or 6-byte pattern takes when its few inside windows are frequent text.
// Round 6: the two choices are independent (they were an adjacent pair (o, o + 1)): a 5-byte
// pattern "hipp?" had to key on "hipp", 15 % of the C4 pool's key-window hits.
struct KeyChoice { std::vector<std::pair<uint32_t, int16_t>> keys; };
// follow: the bytes that can come right after the pattern (regex prefix / factor strings;
// nullptr = any byte) -- a right-hand family then only needs those
// use: how many patterns already key on a window.  A window's cost is (benign cost + a floor for
// attack traffic) x (1 + patterns sharing the key: each is one more literal compare per hit in
// k_waf_exact) x 8 per missing byte of stage-2 context (the k_waf_ctx filter checks up to two
// pattern bytes either side of the window); a family adds, per key, the Bloom fill it costs every
// probed window (kKeyLoad, in the same units).
KeyChoice choose_keys(const std::string &pat, const KeyModel &M, std::unordered_map<uint32_t, uint32_t> &use,
                      const std::bitset<256> *follow = nullptr) {
    KeyChoice r;
    const int L = (int)pat.size();
    // one key's share of the Bloom false positives per probed window (4 bits of a 2^20-bit filter
    // at ~17 % fill: d(f^4)/dn = 16 f^3 / m), scaled like M.cost (sample counts, or a probability)
    const double kKeyLoad = 3.5e-8 * (M.n > 0 ? M.n : 1.0);
    auto share = [&](uint32_t w) {
        auto it = use.find(w);
        return 1.0 + (it == use.end() ? 0.0 : (double)it->second);
    };
    auto ctx_miss = [&](int o) {   // stage-2 context bytes the pattern lacks around window o
        return (2 - std::max(0, std::min(2, o))) + (2 - std::max(0, std::min(2, L - o - 4)));
    };
    auto wcost = [&](int o) {
        const uint32_t w = fold4(load4(pat, (size_t)o));
        return (M.cost(w) + std::exp2(-30.0)) * share(w) * std::exp2(3.0 * ctx_miss(o));
    };
    std::bitset<256> ys;   // folded right-hand bytes
    for (uint32_t z = 0; z < 256; z++) if (!follow || (*follow)[z]) ys[z | 0x20u] = true;
    ys[0x20] = true;   // a pattern that ends the arena: the scan reads the byte past it as 0, folded ' '
                       // (k_waf_scan probes windows of >= 3 arena bytes)
    // the family of window o (o = -1: the byte before the pattern varies; o = L - 3: the byte after):
    // its keys, and its expected candidates -- benign occurrences of its windows plus the Bloom
    // load of its keys (kKeyLoad each)
    auto family = [&](int o, std::vector<uint32_t> *out) {
        double c = 0;
        const bool left = o < 0;
        for (uint32_t z = 0; z < 256; z++) {
            if ((z | 0x20u) != z || (!left && !ys[z])) continue;
            const uint32_t w = left ? (z | (fold4(load4(pat, 0)) << 8)) : ((fold4(load4(pat, (size_t)L - 4)) >> 8) | (z << 24));
            if (out) out->push_back(w);
            else c += M.cost(w) + kKeyLoad;
        }
        return c;
    };
    if (L >= 5) {
        double best[2] = {1e300, 1e300};
        int bo[2] = {0, 1};
        for (int o = 0; o + 4 <= L; o++) {
            const double c = wcost(o);
            if (c < best[o & 1] * (1 - 1e-12)) { best[o & 1] = c; bo[o & 1] = o; }
        }
        // a class whose best inside window is frequent benign text (more expected candidates than a
        // whole family's Bloom load) takes a family instead when that family expects 4x fewer
        // candidates: the left one serves the odd class, the right one the class of L - 3
        int fam[2] = {0, 0};   // 0: inside window; -1: left family; 1: right family
        for (int cls = 0; cls < 2; cls++) {
            const double cin = M.cost(fold4(load4(pat, (size_t)bo[cls])));
            if (cin <= 128 * kKeyLoad) continue;
            double fb = 1e300;
            if (cls == 1) { const double f = family(-1, nullptr); if (4 * f < cin && f < fb) { fb = f; fam[cls] = -1; } }
            if (((L - 3) & 1) == cls) { const double f = family(L - 3, nullptr); if (4 * f < cin && f < fb) { fb = f; fam[cls] = 1; } }
        }
        for (int cls = 0; cls < 2; cls++) {
            if (fam[cls]) {
                const int o = fam[cls] < 0 ? -1 : L - 3;
                std::vector<uint32_t> ws;
                family(o, &ws);
                for (uint32_t w : ws) { r.keys.push_back({w, (int16_t)o}); use[w]++; }
            } else {
                const uint32_t w = fold4(load4(pat, (size_t)bo[cls]));
                r.keys.push_back({w, (int16_t)bo[cls]});
                use[w]++;
            }
        }
        return r;
    }
    const uint32_t w = fold4(load4(pat, 0));
    double cl = 0, cr = 0;
    for (uint32_t z = 0; z < 256; z++) {
        if ((z | 0x20u) != z) continue;
        cl += M.cost(z | (w << 8));
        if (ys[z]) cr += M.cost((w >> 8) | (z << 24));
    }
    // every key also costs prefilter precision (Bloom load): a right-hand family restricted by a
    // follow set of at most 32 bytes wins unless it is far costlier in benign traffic
    const size_t nr = ys.count();
    const bool left = nr <= 32 ? cl * 8 < cr : cl <= cr;
    r.keys.push_back({w, 0});
    for (uint32_t z = 0; z < 256; z++) {
        if ((z | 0x20u) != z) continue;
        if (left) r.keys.push_back({z | (w << 8), -1});
        else if (ys[z]) r.keys.push_back({(w >> 8) | (z << 24), 1});
    }
    return r;
}

// Bloom multiplier and probe count per generation: a Bloom filter's false-positive rate is an
// average; on real traffic what matters is whether the frequent benign 4-grams collide.  Each
// candidate multiplier builds the filter and is scored by the benign non-key windows that test
// positive (weighted by their sample counts; without a sample: the background corpus).
const uint32_t kBloomMuls[] = {0x9E3779B1u, 0x85EBCA77u, 0xC2B2AE3Du, 0x27D4EB2Fu, 0x165667B1u, 0xD3A2646Cu | 1u,
                               0xFD7046C5u, 0xB55A4F09u, 0x7FEB352Du, 0x846CA68Bu, 0x2C1B3C6Du, 0x297A2D39u,
                               0xE6546B64u | 1u, 0x1B873593u, 0xCC9E2D51u, 0x5BD1E995u};

// the 16 fixed multipliers plus more odd ones from a fixed-seed splitmix sequence, GM_BLOOM_NMUL in
// all: 1024 scored 12 % fewer scan candidates on the C4 traffic than 64 (0.372 vs 0.422 % of the
// windows), and the C4 step ran 4.63 vs 4.71 ms (A/B on one box)
const std::vector<uint32_t> &bloom_mul_candidates() {
    static std::vector<uint32_t> v = [] {
        std::vector<uint32_t> r(std::begin(kBloomMuls), std::end(kBloomMuls));
        uint64_t x = 0x243F6A8885A308D3ull;
#ifndef GM_BLOOM_NMUL
#define GM_BLOOM_NMUL 1024
#endif
        while (r.size() < GM_BLOOM_NMUL) {
            x += 0x9E3779B97F4A7C15ull;
            uint64_t z = x;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            r.push_back((uint32_t)z | 1u);
        }
        return r;
    }();
    return v;
}

struct BloomChoice { uint32_t mul = 0; double fp = 0; };   // fp: weighted false positives per window
BloomChoice choose_bloom_mul(const std::vector<uint32_t> &keys, uint32_t pk, const KeyModel &M,
                             std::vector<uint32_t> &filter, size_t max_cands = SIZE_MAX) {
    std::set<uint32_t> kset(keys.begin(), keys.end());
    std::vector<std::pair<uint32_t, double>> test;   // benign non-key windows, weight
    if (M.n > 0) {
        for (auto &kv : M.cnt) if (!kset.count(kv.first)) test.push_back({kv.first, kv.second / M.n});
    } else {
        for (auto &kv : background_weights()) if (!kset.count(kv.first)) test.push_back({kv.first, kv.second / 65536});
    }
    // the candidates are scored on up to 8 host threads (each its own filter); the lowest score
    // wins, ties to the earlier candidate, so the choice does not depend on the thread count
    const std::vector<uint32_t> &all = bloom_mul_candidates();
    const std::vector<uint32_t> cands(all.begin(), all.begin() + std::min(max_cands, all.size()));
    std::vector<double> score(cands.size(), 1e300);
    auto run = [&](size_t t0, size_t step) {
        std::vector<uint32_t> f(filter.size());
        for (size_t c = t0; c < cands.size(); c += step) {
            std::fill(f.begin(), f.end(), 0u);
            for (uint32_t k : keys) { const BloomProbe b = scan_probe(k, cands[c], pk); f[b.block] |= b.mask; }
            double fp = 0;
            for (auto &t : test) {
                const BloomProbe b = scan_probe(t.first, cands[c], pk);
                if ((f[b.block] & b.mask) == b.mask) fp += t.second;
            }
            score[c] = fp;
        }
    };
    const size_t nt = std::max<size_t>(1, std::min<size_t>(8, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (size_t q = 1; q < nt; q++) pool.emplace_back(run, q, nt);
    run(0, nt);
    for (auto &th : pool) th.join();
    BloomChoice best{kBloomMuls[0], 1e300};
    for (size_t c = 0; c < cands.size(); c++)
        if (score[c] < best.fp) best = BloomChoice{cands[c], score[c]};
    std::fill(filter.begin(), filter.end(), 0u);
    for (uint32_t k : keys) { const BloomProbe b = scan_probe(k, best.mul, pk); filter[b.block] |= b.mask; }
    return best;
}

}  // namespace

// ngx_http_upstream_update_chash: per server, 160 * weight points; the base CRC over host, one NUL
// byte and port (split at the last ':' followed by digits only; "unix:" paths have no port), each
// point = final(base + the previous point's 4 LE bytes).  Sorted by hash; equal hashes keep one
// point (nginx keeps the first after an unstable sort -- here the lowest peer index).  Appends
// the ring to `points` (peer = index within the upstream).
void chash_ring(const std::vector<std::string> &addrs, std::vector<DPoint> &points) {
    static constexpr Crc32Table T = make_crc32_table();
    auto upd = [&](uint32_t c, const uint8_t *p, size_t n) {
        for (size_t q = 0; q < n; q++) c = T.t[(c ^ p[q]) & 0xFF] ^ (c >> 8);
        return c;
    };
    std::vector<DPoint> ring;
    for (uint32_t j = 0; j < addrs.size(); j++) {
        const std::string &sv = addrs[j];
        std::string host = sv, port;
        if (sv.size() >= 5 && lower(sv.substr(0, 5)) == "unix:") host = sv.substr(5);
        else {
            for (size_t q = 0; q < sv.size(); q++) {
                const char c = sv[sv.size() - q - 1];
                if (c == ':') { host = sv.substr(0, sv.size() - q - 1); port = sv.substr(sv.size() - q); break; }
                if (c < '0' || c > '9') break;
            }
        }
        uint32_t base = 0xFFFFFFFFu;
        base = upd(base, (const uint8_t *)host.data(), host.size());
        const uint8_t nul = 0;
        base = upd(base, &nul, 1);
        base = upd(base, (const uint8_t *)port.data(), port.size());
        uint32_t prev = 0;
        for (int q = 0; q < 160; q++) {
            const uint8_t pb[4] = {(uint8_t)prev, (uint8_t)(prev >> 8), (uint8_t)(prev >> 16), (uint8_t)(prev >> 24)};
            const uint32_t h = upd(base, pb, 4) ^ 0xFFFFFFFFu;
            ring.push_back(DPoint{h, j});
            prev = h;
        }
    }
    std::sort(ring.begin(), ring.end(), [](const DPoint &a, const DPoint &b) {
        return a.hash != b.hash ? a.hash < b.hash : a.peer < b.peer;
    });
    for (size_t q = 0; q < ring.size(); q++)
        if (q == 0 || ring[q].hash != ring[q - 1].hash) points.push_back(ring[q]);
}

// ============================================================================ entry

// RFC 1321 MD5 (the NGINX Plus sticky cookie's value is the hex MD5 of the peer's address text)
static void md5_digest(const std::string &msg, uint32_t out[4]) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9, 14, 20, 5, 9, 14, 20, 5, 9, 14, 20, 5, 9, 14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    std::vector<uint8_t> m(msg.begin(), msg.end());
    const uint64_t bits = (uint64_t)msg.size() * 8;
    m.push_back(0x80);
    while (m.size() % 64 != 56) m.push_back(0);
    for (int i = 0; i < 8; i++) m.push_back((uint8_t)(bits >> (8 * i)));
    uint32_t h[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
    for (size_t o = 0; o < m.size(); o += 64) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++)
            w[i] = m[o + 4 * i] | m[o + 4 * i + 1] << 8 | m[o + 4 * i + 2] << 16 | (uint32_t)m[o + 4 * i + 3] << 24;
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
        for (int i = 0; i < 64; i++) {
            uint32_t f, g;
            if (i < 16) { f = (b & c) | (~b & d); g = i; }
            else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) % 16; }
            else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) % 16; }
            else { f = c ^ (b | ~d); g = (7 * i) % 16; }
            const uint32_t x = a + f + K[i] + w[g];
            a = d; d = c; c = b;
            b = b + (x << R[i] | x >> (32 - R[i]));
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d;
    }
    for (int i = 0; i < 4; i++) out[i] = h[i];   // little-endian words: bytes in digest order
}
static void put_md5(std::vector<uint32_t> &v, const std::string &addr) {
    uint32_t d[4];
    md5_digest(addr, d);
    v.insert(v.end(), d, d + 4);
}


// The heads of an anchored DFA (state 1 = start, 0 = dead; acc bit0 match, bit1 match at the
// subject's end): bit rsl_head_key(b0, b1, b2) of `bits` (RSL_HEAD_WORDS u32) for every three-byte
// start b0 b1 b2 of a subject it can match (a 0 stands for "no byte": rsl_head_key(b0, b1, 0) is
// the two-byte subject b0 b1, and so on; a $uri with a NUL in its first three bytes joins every
// list, k_rloc_heads); a DFA that matches at its start state sets every bit.  A final '\n' may
// satisfy a `$` (PCRE), so an end-accepting state also sets its subject + '\n'.  Past
// RSL_HEAD_PAIRS live two-byte starts the map is full (a superset: the slice runs on every request).
static void dfa_heads(const Dfa &d, std::vector<uint32_t> &bits) {
    auto set = [&](uint32_t key) { bits[key >> 5] |= 1u << (key & 31); };
    auto step = [&](uint32_t st, int b) { return (uint32_t)(d.trans[(size_t)st * d.n_classes + d.cls[b]] & DFA_TRANS_STATE_MASK); };
    auto fill = [&]() { std::fill(bits.begin(), bits.end(), 0xFFFFFFFFu); };
    if (d.n_states < 2 || (d.acc[1] & 1)) { fill(); return; }
    if (d.acc[1] & 2) { set(rsl_head_key(0, 0, 0)); set(rsl_head_key('\n', 0, 0)); }
    uint32_t pairs = 0;
    for (uint32_t b0 = 1; b0 < 256; b0++) {
        const uint32_t s1 = step(1, (int)b0);
        if (!s1) continue;
        if (d.acc[s1] & 1) {
            for (uint32_t b1 = 0; b1 < 256; b1++)
                for (uint32_t b2 = 0; b2 < 256; b2++) set(rsl_head_key(b0, b1, b2));
            continue;
        }
        if (d.acc[s1] & 2) { set(rsl_head_key(b0, 0, 0)); set(rsl_head_key(b0, '\n', 0)); }
        for (uint32_t b1 = 1; b1 < 256; b1++) {
            const uint32_t s2 = step(s1, (int)b1);
            if (!s2) continue;
            if (++pairs > RSL_HEAD_PAIRS) { fill(); return; }
            if (d.acc[s2] & 1) {
                for (uint32_t b2 = 0; b2 < 256; b2++) set(rsl_head_key(b0, b1, b2));
                continue;
            }
            if (d.acc[s2] & 2) { set(rsl_head_key(b0, b1, 0)); set(rsl_head_key(b0, b1, '\n')); }
            for (uint32_t b2 = 1; b2 < 256; b2++)
                if (step(s2, (int)b2)) set(rsl_head_key(b0, b1, b2));
        }
    }
}

CompileResult compile_generation(const uint8_t *blob, size_t len, uint32_t gen) {
    CompileResult R;
    gm_stats_t &st = R.stats;
    memset(&st, 0, sizeof st);
    st.gen = gen;
    if (!blob || len < 8) { R.code = GM_E_INVAL; R.err = "short blob"; return R; }
    uint32_t magic, n;
    memcpy(&magic, blob, 4); memcpy(&n, blob + 4, 4);
    if (magic != GM_BLOB_MAGIC) { R.code = GM_E_INVAL; R.err = "bad blob magic"; return R; }
    size_t off = 8;
    std::vector<Dir> main_body;
    bool have_main = false;
    std::vector<std::vector<Dir>> confd;
    const char *sig_text = nullptr; size_t sig_len = 0;
    KeyModel KM;
    for (uint32_t e = 0; e < n; e++) {
        if (off + 12 > len) { R.code = GM_E_INVAL; R.err = "truncated blob"; return R; }
        uint32_t kind, nl, dl;
        memcpy(&kind, blob + off, 4); memcpy(&nl, blob + off + 4, 4); memcpy(&dl, blob + off + 8, 4);
        off += 12;
        if (off + (uint64_t)nl + dl > len) { R.code = GM_E_INVAL; R.err = "truncated blob entry"; return R; }
        const char *data = (const char *)blob + off + nl;
        off += nl + dl;
        if (kind == GM_ENTRY_SIGS) { sig_text = data; sig_len = dl; continue; }
        if (kind == GM_ENTRY_SAMPLE) { KM.add_sample((const uint8_t *)data, dl); continue; }
        Tokenizer T(data, dl);
        std::vector<Dir> body;
        if (!parse_body(T, body, false)) {
            R.code = GM_E_PARSE;
            R.err = "nginx config parse error in " + std::string((const char *)blob + off - dl - nl, nl);
            return R;
        }
        if (kind == GM_ENTRY_MAIN) { main_body = std::move(body); have_main = true; }
        else confd.push_back(std::move(body));
    }

    std::vector<SigRule> sig;
    uint32_t decoders = 0;
    if (sig_text && !parse_sigs(sig_text, sig_len, sig, decoders)) { R.code = GM_E_PARSE; R.err = "signature set parse error"; return R; }
    st.decoders = decoders;

    Model M;
    Builder B(M, confd);
    if (have_main) {
        for (const Dir &d : main_body)
            if (!d.a.empty() && d.a[0] == "http" && d.block) B.http(d.body);
    } else {
        for (auto &f : confd) B.http(f);
    }

    Compiler C(M, st);
    st.n_rejected_other += M.rejected_other;
    R.rejects = M.reject_log;

    // ---- upstreams: sorted unique name table
    std::vector<std::string> ups = M.upstreams;
    std::sort(ups.begin(), ups.end());
    ups.erase(std::unique(ups.begin(), ups.end()), ups.end());
    st.n_upstreams = (uint32_t)ups.size();

    // ---- upstream peers (§8 f3): one DUpstream per sorted name (first block of a name wins;
    // nginx rejects a duplicate upstream outright)
    std::vector<DUpstream> dups(ups.size());
    std::vector<DKeyPart> key_parts;
    std::vector<DPoint> points;
    std::vector<uint32_t> peer_init;
    R.peer_addrs.clear(); R.peer_ups.clear();
    R.ups_meta.assign(ups.size(), UpstreamMeta{});
    for (size_t u = 0; u < ups.size(); u++) R.ups_meta[u].name = ups[u];
    {
        std::map<std::string, const UpstreamIR *> defs;
        for (const UpstreamIR &U : M.upstream_defs) defs.emplace(U.name, &U);
        for (size_t u = 0; u < ups.size(); u++) {
            DUpstream &D = dups[u];
            memset(&D, 0, sizeof D);
            D.first_peer = (uint32_t)peer_init.size();
            const UpstreamIR *U = defs.count(ups[u]) ? defs[ups[u]] : nullptr;
            if (!U) { D.method = UM_DEFER; st.n_upstreams_deferred++; continue; }
            D.method = U->method;
            D.n_peers = (uint32_t)U->peers.size();
            for (const auto &p : U->peers) {
                peer_init.push_back(p.down ? GM_PEER_DOWN : 0u);
                R.peer_addrs.push_back(p.addr);
                R.peer_ups.push_back((uint32_t)u);
            }
            bool defer = U->defer;
            if (!U->sticky.empty()) {
                const int sid = C.src("$cookie_" + U->sticky);
                if (sid < 0) defer = true; else D.sticky = 1u + (uint32_t)sid;
            }
            UpstreamMeta &um = R.ups_meta[u];
            um.has_block = true;
            um.method = U->method;
            if ((D.method == UM_RR || D.method == UM_LEAST_CONN) && D.n_peers > SEQ_PEERS_MAX) defer = true;
            if (D.method == UM_HASH || D.method == UM_CHASH) {
                // key = literal text and $variables; the engine's variables except $host (nginx's
                // $host is the validated name or the server_name, not the raw header)
                D.first_part = (uint32_t)key_parts.size();
                const std::string &k = U->key;
                size_t i = 0;
                while (i < k.size() && !defer) {
                    if (k[i] == '$') {
                        size_t j = i + 1, e;
                        std::string nm;
                        if (j < k.size() && k[j] == '{') {
                            e = k.find('}', j);
                            if (e == std::string::npos) { defer = true; break; }
                            nm = k.substr(j + 1, e - j - 1); e++;
                        } else {
                            e = j;
                            while (e < k.size() && (isalnum((unsigned char)k[e]) || k[e] == '_')) e++;
                            nm = k.substr(j, e - j);
                        }
                        const int sid = lower(nm) == "host" ? -1 : C.src("$" + nm);
                        if (sid < 0) { defer = true; break; }
                        key_parts.push_back(DKeyPart{(uint32_t)sid, KEY_PART_VAR});
                        i = e;
                    } else {
                        size_t e = k.find('$', i);
                        if (e == std::string::npos) e = k.size();
                        key_parts.push_back(DKeyPart{C.put_bytes(k.substr(i, e - i)), (uint32_t)(e - i)});
                        i = e;
                    }
                }
                D.n_parts = (uint32_t)key_parts.size() - D.first_part;
                // chash: two server lines with one address would share ring points (nginx then
                // round-robins between them): not modelled
                um.defer_fixed = U->defer || defer;   // the key's shape, not the servers
                std::set<std::string> seen;
                for (const auto &p : U->peers) if (!seen.insert(p.addr).second && D.method == UM_CHASH) defer = true;
            } else {
                um.defer_fixed = U->defer;
            }
            if (D.method == UM_CHASH && !defer) {
                std::vector<std::string> addrs;
                for (const auto &p : U->peers) addrs.push_back(p.addr);
                D.first_point = (uint32_t)points.size();
                chash_ring(addrs, points);
                D.n_points = (uint32_t)points.size() - D.first_point;
            }
            if (defer) { D.method = UM_DEFER; st.n_upstreams_deferred++; }
        }
    }
    st.n_peers = (uint32_t)peer_init.size();

    // ---- ports
    std::vector<DPort> ports;
    std::map<int, int> port_idx;
    std::set<int> def_seen;   // ports whose default_server is set (the first `default_server` wins)
    for (auto &S : M.servers)
        for (auto &l : S.listens) {
            auto it = port_idx.find(l.first);
            if (it == port_idx.end()) {
                port_idx[l.first] = (int)ports.size();
                ports.push_back(DPort{(uint32_t)l.first, 0, (uint32_t)S.id, 0u});
                it = port_idx.find(l.first);
            }
            DPort &P = ports[it->second];
            if (l.second & 1) P.ssl = 1;
            if (l.second & 4) P.proxy = 1;   // proxy_protocol: ORed over the port's listens (ngx_http_add_addresses)
            if ((l.second & 2) && !def_seen.count(l.first)) { P.default_server = (uint32_t)S.id; def_seen.insert(l.first); }
        }

    // ---- server names: exact / wildcard-head / wildcard-tail hash tables, first wins
    struct NameKey { std::string name; int port; uint32_t server; };
    std::vector<NameKey> exact, head, tail;
    for (auto &S : M.servers) {
        std::set<int> sp;
        for (auto &l : S.listens) sp.insert(port_idx[l.first]);
        for (auto &nm : S.names) {
            if (nm.empty()) continue;
            if (nm[0] == '~') { st.n_rejected_other++; continue; }
            for (int p : sp) {
                if (nm.size() > 2 && nm[0] == '*' && nm[1] == '.') head.push_back({nm.substr(2), p, (uint32_t)S.id});
                else if (nm.size() > 1 && nm[0] == '.') head.push_back({nm.substr(1), p, (uint32_t)S.id | 0x80000000u});
                else if (nm.size() > 2 && nm.back() == '*' && nm[nm.size() - 2] == '.')
                    tail.push_back({nm.substr(0, nm.size() - 2), p, (uint32_t)S.id});
                else if (nm.find('*') == std::string::npos) exact.push_back({nm, p, (uint32_t)S.id});
                else st.n_rejected_other++;
            }
        }
    }
    std::vector<uint8_t> name_bytes;   // server-name strings (their own hot section, see off_hot_end)
    auto put_name = [&](const std::string &nm) {
        const uint32_t off = (uint32_t)name_bytes.size();
        name_bytes.insert(name_bytes.end(), nm.begin(), nm.end());
        return off;
    };
    auto build_names = [&](std::vector<NameKey> &keys, uint32_t &mask) {
        uint32_t cap = pow2_at_least(keys.size() * 2 + 1);
        std::vector<DName> tab(cap);
        for (auto &k : keys) {
            uint32_t h = name_hash_init((uint32_t)k.name.size());
            for (size_t o = 0; o < k.name.size(); o += 4) {
                uint32_t w = 0;
                for (size_t q = 0; q < 4 && o + q < k.name.size(); q++) w |= (uint32_t)(uint8_t)k.name[o + q] << (8 * q);
                h = name_hash_word(h, w);
            }
            h = name_hash_fin(h, (uint32_t)k.port);
            uint32_t i = h & (cap - 1);
            bool dup = false;
            while (tab[i].hash) {
                const DName &e = tab[i];
                if (e.hash == h && e.port_idx == k.port && e.name_len == k.name.size() &&
                    !memcmp(name_bytes.data() + e.name_off, k.name.data(), k.name.size())) { dup = true; break; }
                i = (i + 1) & (cap - 1);
            }
            if (dup) continue;   // duplicate name on this port: first definition wins
            tab[i].hash = h; tab[i].name_off = put_name(k.name); tab[i].name_len = (uint16_t)k.name.size();
            tab[i].port_idx = (uint16_t)k.port; tab[i].server = k.server;
        }
        mask = cap - 1;
        return tab;
    };
    uint32_t names_mask, head_mask, tail_mask;
    auto tab_exact = build_names(exact, names_mask);
    auto tab_head = build_names(head, head_mask);
    auto tab_tail = build_names(tail, tail_mask);

    // ---- locations, tries, regex locations, server ifs
    std::vector<DLoc> dlocs(M.locs.size());
    for (DLoc &d : dlocs) d.access = GM_NONE;
    std::vector<DLocUri> dluri(M.locs.size());
    std::vector<DNode> nodes;
    std::vector<std::pair<uint32_t, uint32_t>> edge_list;   // key, child
    std::map<std::pair<uint32_t, uint8_t>, uint32_t> edge_map;
    std::vector<DServer> dservers(M.servers.size());
    std::vector<DServerIf> sifs;
    std::vector<DRegexLoc> rlocs;
    std::vector<std::vector<std::string>> rloc_factors;   // parallel to rlocs: >= 4-byte factors
    std::vector<uint8_t> rsl_pbit;   // parallel to rlocs (filled below): k_rloc_pref's mask bit, 0xFF none
    std::vector<uint32_t> rsl_heads; // anchored slices' head maps (ALW_SLICE_HEADS), RSL_HEAD_WORDS each
    std::vector<uint32_t> rsl_head_slice;   // and each map's slice
    // parallel to rlocs: the DFA of ^(\n)?rev(X) for an unanchored X$ (n_states 0: none) --
    // union-DFA slices of these run backwards from the URI's end (gm_regex.hpp
    // compile_regex_reversed) and die within a few bytes, where the forward search reads it all
    std::vector<Dfa> rloc_rev;
    auto new_node = [&]() { nodes.push_back(DNode{-1, -1, -1, 0}); return (uint32_t)nodes.size() - 1; };
    auto walk = [&](uint32_t root, const std::string &p) {
        uint32_t cur = root;
        for (unsigned char c : p) {
            auto key = std::make_pair(cur, c);
            auto it = edge_map.find(key);
            if (it == edge_map.end()) {
                uint32_t nn = new_node();
                edge_map[key] = nn;
                edge_list.push_back({cur * 256u + c + 1u, nn});
                cur = nn;
            } else cur = it->second;
        }
        return cur;
    };
    auto is_redirect = [](int code) { return code == 301 || code == 302 || code == 303 || code == 307 || code == 308; };
    (void)is_redirect;
    std::vector<DRealIp> realips;
    std::vector<DCidr> cidrs;
    std::vector<DAccRule> acc_rules;
    std::vector<DAccList> acc_lists;
    std::map<std::vector<std::pair<bool, std::string>>, uint32_t> acc_index;   // one list per distinct rule set
    // the allow / deny rules in effect -> a DAccList index (GM_NONE: none), ngx_http_access_rule:
    // `all` goes to both lists, an IPv4 CIDR to the first, an IPv6 one to the second; `unix:` rules
    // never see a TCP client.  bad: a rule the engine does not read (a host name, a bad prefix).
    auto access_list = [&](const std::vector<std::pair<bool, std::string>> &rules, bool &bad) -> uint32_t {
        bad = false;
        if (rules.empty()) return GM_NONE;
        auto it = acc_index.find(rules);
        if (it != acc_index.end()) return it->second;
        std::vector<DAccRule> r4, r6;
        for (const auto &r : rules) {
            if (r.second == "unix:") continue;
            DAccRule a{};
            a.deny = r.first ? 1u : 0u;
            if (r.second == "all") { r4.push_back(a); r6.push_back(a); continue; }
            if (!parse_cidr(r.second, a.c)) { bad = true; continue; }
            (a.c.family == 4 ? r4 : r6).push_back(a);
        }
        DAccList L{(uint32_t)acc_rules.size(), (uint32_t)r4.size(), 0, (uint32_t)r6.size()};
        acc_rules.insert(acc_rules.end(), r4.begin(), r4.end());
        L.first6 = (uint32_t)acc_rules.size();
        acc_rules.insert(acc_rules.end(), r6.begin(), r6.end());
        const uint32_t idx = (uint32_t)acc_lists.size();
        acc_lists.push_back(L);
        acc_index[rules] = idx;
        return idx;
    };
    auto body_of = [&](const std::string &own, const Server &S, bool &bad) -> uint32_t {
        // client_max_body_size in effect: the location's, else the server's, else the http
        // block's, else nginx's default 1m (ngx_http_core_merge_loc_conf)
        const std::string &v = !own.empty() ? own : !S.cmbs.empty() ? S.cmbs : !M.http_cmbs.empty() ? M.http_cmbs
                                                                                                         : std::string("1m");
        const int64_t x = parse_body_max(v);
        bad = x < 0;
        return x < 0 ? BODY_UNLIMITED : (uint32_t)x;
    };
    for (auto &S : M.servers) {
        DServer &D = dservers[S.id];
        D.trie_root = new_node();
        D.waf_mode = (uint32_t)S.waf;
        bool sbad = false;
        D.body_max = body_of("", S, sbad);
        if (sbad) { S.ifs.insert(S.ifs.begin(), SIf{"$uri", -1}); R.rejects.push_back("server: client_max_body_size " + S.cmbs); }
        // realip in effect (ngx_http_realip_merge_loc_conf: the server's set_real_ip_from list,
        // else the http block's; header and recursion merged one by one)
        {   // allow / deny for a request that matches no location: the server block's own rules
            bool abad = false;
            D.access = access_list(!S.access.empty() ? S.access : M.http_access, abad);
        }
        D.realip = GM_NONE;
        {
            const RealIpIR &a = S.rip, &h = M.http_rip;
            const std::vector<std::string> &from = !a.from.empty() ? a.from : h.from;
            const std::string hdr = !a.header.empty() ? a.header : !h.header.empty() ? h.header : std::string("X-Real-IP");
            const int rec = a.recursive >= 0 ? a.recursive : h.recursive >= 0 ? h.recursive : 0;
            if (!from.empty()) {
                DRealIp ri{};
                ri.recursive = (uint32_t)rec;
                ri.first_cidr = (uint32_t)cidrs.size();
                bool bad = a.bad || h.bad;
                for (const std::string &f : from) {
                    if (f.rfind("unix:", 0) == 0) continue;   // never a TCP client
                    DCidr c;
                    if (!parse_cidr(f, c)) { bad = true; continue; }
                    cidrs.push_back(c);
                }
                ri.n_cidr = (uint32_t)cidrs.size() - ri.first_cidr;
                // (strcmp, case-sensitive: ngx_http_realip)
                if (hdr == "X-Real-IP") ri.type = RIP_XREALIP;
                else if (hdr == "X-Forwarded-For") ri.type = RIP_XFWD;
                else if (hdr == "proxy_protocol") ri.type = RIP_PROXY;
                else { ri.type = RIP_HEADER; ri.hdr_off = C.put_bytes(lower(hdr)); ri.hdr_len = (uint32_t)hdr.size(); }
                // the address nginx would use is unknown to the engine: a hostname in
                // set_real_ip_from -- requests whose verdict reads $remote_addr / $remote_port
                // defer (proxy_protocol reads the record's PROXY address, gm_parse_requests)
                if (bad) { ri.type = RIP_UNKNOWN; st.n_rejected_other++; R.rejects.push_back("server: set_real_ip_from (not an address)"); }
                D.realip = (uint32_t)realips.size();
                realips.push_back(ri);
            }
        }
        if (M.http_unknown) { SIf f; f.var = "$uri"; f.op = -1; f.nocount = true; S.ifs.push_back(f); }
        D.first_if = (uint32_t)sifs.size();
        for (auto &f : S.ifs) {
            DServerIf x{};
            x.code = (uint32_t)f.code;
            if (f.ret_only) x.op = SIF_RETURN;
            else {
                int s = C.src(f.var);
                if (s < 0 || f.op < 0) { x.op = 0xFF; if (!f.nocount) st.n_rejected_other++; }
                else {
                    x.src = (uint32_t)s;
                    if (f.op == 0) x.op = 4;   // truthy: non-empty and not "0"
                    else if (f.op == 1 || f.op == 2) { x.op = f.op == 1 ? SIF_EQ : SIF_NE; x.val_off = C.put_bytes(f.val); x.val_len = (uint32_t)f.val.size(); }
                    else {
                        int d = C.regex(f.val, f.op == 4 || f.op == 6);
                        if (d < 0) x.op = 0xFF;
                        else { x.op = (f.op == 3 || f.op == 4) ? 5 : 6; x.val_off = (uint32_t)d; }
                    }
                    const DSrc &ds = C.srcs[s];
                    if (ds.kind == SRC_VAR && (ds.var == V_SCHEME || ds.var == V_HTTPS || ds.var == V_HTTP2) &&
                        (x.op == 4 || x.op == SIF_EQ || x.op == SIF_NE)) {
                        // value per (https, http2) -- get_var's V_SCHEME / V_HTTPS / V_HTTP2 cases
                        uint32_t tt = 0;
                        for (uint32_t fl = 0; fl < 4; fl++) {
                            const bool https = fl & GM_REQ_HTTPS, h2 = fl & GM_REQ_HTTP2;
                            const std::string v = ds.var == V_SCHEME ? (https ? "https" : "http")
                                                  : ds.var == V_HTTPS ? (https ? "on" : "") : (h2 ? "h2" : "");
                            const bool hit = x.op == 4 ? (!v.empty() && v != "0")
                                             : x.op == SIF_EQ ? v == f.val : v != f.val;
                            if (hit) tt |= 1u << fl;
                        }
                        x.op = SIF_FLAGS; x.tt = tt;
                    }
                }
            }
            sifs.push_back(x);
        }
        D.n_if = (uint32_t)sifs.size() - D.first_if;
        D.first_rloc = (uint32_t)rlocs.size();
        for (int lid : S.locs) {
            Loc &L = M.locs[lid];
            DLoc &dl = dlocs[lid];
            dl.waf_mode = (uint8_t)(L.waf >= 0 ? L.waf : S.waf);
            // the request parsers this location runs: the signature set's, minus
            // wallarm_parser_disable (a location's own list replaces the server's, nginx's array merge)
            dluri[lid].flags |= (decoders & ~(L.has_pd ? L.parser_off : S.parser_off)) << LOCURI_DEC_SHIFT;
            dl.upstream = GM_NONE;
            {   // allow / deny in effect: the location's own, else the server's, else the http block's
                const auto &acc = !L.access.empty() ? L.access : !S.access.empty() ? S.access : M.http_access;
                bool abad = false;
                dl.access = access_list(acc, abad);
                if (abad) {
                    L.unknown = true; st.n_rejected_other++;
                    R.rejects.push_back("location " + L.path + ": allow / deny with an address the engine does not read");
                }
            }
            dl.noregex = L.kind == NOREGEX;
            dl.is_named = L.kind == NAMED;
            bool lbad = false;
            dl.body_max = body_of(L.cmbs, S, lbad);
            if (lbad) { L.unknown = true; st.n_rejected_other++; R.rejects.push_back("location " + L.path + ": client_max_body_size " + L.cmbs); }
            // a nested `location` can change which location's limit applies: no 413 decided here
            if (L.nested) dl.body_max = BODY_UNLIMITED;
            if (L.nested || L.unknown) dl.kind = LK_UNSUPPORTED;
            else if (L.has_return && L.code == 418 && !L.err418.empty()) {
                std::vector<std::string> vv;
                int route = -1;
                uint8_t kind = LK_UNSUPPORTED;
                if (Compiler::var_list(L.err418, vv) && vv.size() == 1) {
                    if (M.splits.count(vv[0])) { route = C.split_route(S, vv[0]); kind = LK_IRL_SPLIT; }
                    else if (M.maps.count(vv[0])) { route = C.rules_route(S, vv[0]); kind = LK_IRL_RULES; }
                }
                if (route < 0) {
                    dl.kind = LK_UNSUPPORTED; st.n_rejected_other++;
                    R.rejects.push_back("location " + L.path + ": error_page 418 = " + L.err418 + " (map / split not modelled)");
                }
                else { dl.kind = kind; dl.route = (uint32_t)route; }
                if (kind == LK_IRL_SPLIT && route >= 0) st.n_routes_split++;
                if (kind == LK_IRL_RULES && route >= 0) st.n_routes_rules++;
            } else if (L.has_return) { dl.kind = LK_RETURN; dl.ret_code = (uint32_t)L.code; }
            else if (L.has_proxy) {
                dl.kind = LK_PROXY;
                auto it = std::lower_bound(ups.begin(), ups.end(), L.ups);
                if (it != ups.end() && *it == L.ups) dl.upstream = (uint32_t)(it - ups.begin());
                // the upstream request URI (ngx_http_proxy_create_request): a URI part replaces
                // the matched location prefix of $uri; variables, a URI part under a regex / named
                // location (a config error in nginx) or on grpc_pass are left to nginx
                DLocUri &du = dluri[lid];
                du.flags &= ~(LOCURI_REWRITE | LOCURI_DEFER);
                if (L.pass_vars || (!L.pass_uri.empty() && (L.grpc || L.kind == RX || L.kind == RXI || L.kind == NAMED)))
                    du.flags |= LOCURI_DEFER;
                else if (!L.pass_uri.empty()) {
                    du.flags |= LOCURI_REWRITE;
                    du.off = C.put_bytes(L.pass_uri);
                    du.len = (uint32_t)L.pass_uri.size();
                    du.loc_len = (uint32_t)L.path.size();
                }
            } else if (L.stub) dl.kind = LK_STATUS;
            else dl.kind = LK_NONE;
            // the access phase beside the Wallarm module's (both in NGX_HTTP_ACCESS_PHASE, in an
            // order the reference does not fix): a location with both defers
            if (dl.access != GM_NONE && dl.waf_mode != GM_WAF_OFF && dl.kind != LK_RETURN && dl.kind != LK_UNSUPPORTED) {
                dl.kind = LK_UNSUPPORTED; st.n_rejected_other++;
                R.rejects.push_back("location " + L.path + ": allow / deny beside wallarm_mode");
            }

            if (L.kind == PFX || L.kind == NOREGEX || L.kind == EXACT) {
                D.trie_depth = std::max<uint32_t>(D.trie_depth, (uint32_t)L.path.size());
                uint32_t nd = walk(D.trie_root, L.path);
                int32_t &slot = (L.kind == EXACT) ? nodes[nd].exact_loc : nodes[nd].prefix_loc;
                if (slot >= 0) st.n_rejected_other++;   // duplicate location: nginx refuses; keep first
                else slot = lid;
            } else if (L.kind == RX || L.kind == RXI) {
                // a rejected (PCRE-only) regex stays in config order with the DFA of a superset
                // pattern (relax_pcre_only), or dfa GM_NONE when there is none: a URI that
                // reaches it and matches the superset gets GM_ACT_UNSUPPORTED -- nginx's answer
                // depends on PCRE there, so the request is the data plane's to defer
                std::vector<std::string> fac;
                bool sup = false;
                int d = C.regex(L.path, L.kind == RXI, nullptr, &fac, &sup);
                // sup: the DFA is a superset -- the location is reached only maybe, so its limit
                // is not applied either
                if (d < 0 || sup) { dl.kind = LK_UNSUPPORTED; dl.body_max = BODY_UNLIMITED; }
                rlocs.push_back(DRegexLoc{d >= 0 ? (uint32_t)d : GM_NONE, (uint32_t)lid});
                rloc_factors.push_back(std::move(fac));
                Dfa rv;
                if (d >= 0 && !sup && !(C.dfas[d].flags & DFA_ANCHOR_START) &&
                    compile_regex_reversed(L.path, L.kind == RXI, 4096, rv))
                    rloc_rev.push_back(std::move(rv));
                else rloc_rev.push_back(Dfa{});
            }
        }
        D.n_rloc = (uint32_t)rlocs.size() - D.first_rloc;
        D.rk_on = D.n_rloc > RLOC_SEQ_MAX;
        // auto_redirect: location "<p>/" with proxy_pass -> node for "<p>" if nothing ends there
        for (int lid : S.locs) {
            Loc &L = M.locs[lid];
            if (!(L.kind == PFX || L.kind == NOREGEX || L.kind == EXACT)) continue;
            if (!L.has_proxy || L.path.empty() || L.path.back() != '/') continue;
            uint32_t nd = walk(D.trie_root, L.path.substr(0, L.path.size() - 1));
            if (nodes[nd].prefix_loc < 0 && nodes[nd].exact_loc < 0 && nodes[nd].ar_loc < 0) nodes[nd].ar_loc = lid;
        }
    }
    // second pass: an ar_loc whose node later got a location is void
    for (auto &nd : nodes) if (nd.prefix_loc >= 0 || nd.exact_loc >= 0) nd.ar_loc = -1;

    // small servers: the trie nodes that carry a location, as a flat list (DSmallLoc)
    std::vector<DSmallLoc> smalls;
    std::unordered_map<uint32_t, std::vector<std::pair<uint8_t, uint32_t>>> kids;
    for (auto &kv : edge_map) kids[kv.first.first].push_back({kv.first.second, kv.second});
    for (auto &S : M.servers) {
        DServer &D = dservers[S.id];
        if (D.trie_depth > 16) continue;
        std::vector<std::pair<std::string, uint32_t>> todo{{"", D.trie_root}}, marked;
        bool ok = true;
        while (!todo.empty() && ok) {
            auto [path, nd] = todo.back();
            todo.pop_back();
            const DNode &N = nodes[nd];
            if (N.prefix_loc >= 0 || N.exact_loc >= 0 || N.ar_loc >= 0) marked.push_back({path, nd});
            if (marked.size() > SMALL_LOCS_MAX) ok = false;
            for (auto &c : kids[nd]) todo.push_back({path + (char)c.first, c.second});
        }
        if (!ok) continue;
        D.sl_first = (uint32_t)smalls.size(); D.sl_n = (uint32_t)marked.size();
        if (D.sl_n == 0) { D.sl_first = 0; continue; }   // no location at all: the walk finds none either
        for (auto &m : marked) {
            DSmallLoc e{};
            memcpy(e.path, m.first.data(), m.first.size());
            e.len = (uint32_t)m.first.size();
            e.prefix_loc = nodes[m.second].prefix_loc; e.exact_loc = nodes[m.second].exact_loc;
            e.ar_loc = nodes[m.second].ar_loc;
            smalls.push_back(e);
        }
    }

    uint32_t ecap = pow2_at_least(edge_list.size() * 2 + 1);
    std::vector<DEdge> edges(ecap, DEdge{0, 0, -1, 0});
    for (auto &e : edge_list) {
        uint32_t i = edge_hash(e.first) & (ecap - 1);
        while (edges[i].key) i = (i + 1) & (ecap - 1);
        edges[i] = DEdge{e.first, e.second, nodes[e.second].prefix_loc, 0};
    }

    // ---- regex-location factor prefilter (servers with rk_on).  Each regex is keyed on one
    // folded 4-byte window per factor (every match contains one of its factors); the window is
    // the one shared by the fewest regexes so far, preferring windows that span a '/' (a path
    // segment boundary: rarer in URIs than a window inside one word).
    std::map<std::pair<uint32_t, uint32_t>, std::vector<DRlocEnt>> rk_lists;   // (server, key) -> entries
    std::vector<DRlocEnt> rk_ents;
    std::vector<uint32_t> rk_ids;
    for (auto &S : M.servers) {
        DServer &D = dservers[S.id];
        if (!D.rk_on) continue;
        std::vector<uint32_t> alw;
        std::map<uint32_t, uint32_t> use;
        for (uint32_t k = 0; k < D.n_rloc; k++) {
            const DRegexLoc &rl = rlocs[D.first_rloc + k];
            const auto &fac = rloc_factors[D.first_rloc + k];
            if (rl.dfa == GM_NONE || fac.empty()) { alw.push_back(k); continue; }
            std::vector<std::pair<uint32_t, DRlocEnt>> keys;   // a factor each (two may share a window)
            for (const std::string &f : fac) {
                uint32_t best = 0; int best_cost = INT32_MAX, best_o = 0;
                for (size_t o = 0; o + 4 <= f.size(); o++) {
                    uint32_t w = 0;
                    for (int b = 0; b < 4; b++) w |= (uint32_t)(uint8_t)f[o + b] << (8 * b);
                    w = fold4(w);
                    bool span = f[o + 1] == '/' || f[o + 2] == '/' || f[o + 3] == '/';
                    int cost = 2 * (int)use[w] + (span ? 0 : 1);
                    if (cost < best_cost) { best_cost = cost; best = w; best_o = (int)o; }
                }
                std::string ff = f.substr(0, 0x7FFF);   // a prefix of a factor is a factor
                for (char &ch : ff) ch = (char)((uint8_t)ch | 0x20);
                keys.push_back({best, DRlocEnt{k, C.put_bytes(ff), (uint16_t)ff.size(), (int16_t)best_o}});
            }
            for (auto &kv : keys) { use[kv.first]++; rk_lists[{(uint32_t)S.id, kv.first}].push_back(kv.second); }
        }
        D.first_ralw = (uint32_t)rk_ids.size(); D.n_ralw = (uint32_t)alw.size();
        rk_ids.insert(rk_ids.end(), alw.begin(), alw.end());
    }
    const uint32_t rkcap = pow2_at_least(rk_lists.size() * 2 + 1);
    std::vector<DRlocKey> rk(rkcap, DRlocKey{0, 0, 0, 0});
    std::vector<uint32_t> rk_bloom(RK_BLOOM_WORDS, 0u);
    for (auto &kv : rk_lists) {
        const uint32_t sv = kv.first.first, w = kv.first.second;
        const uint32_t bb = rk_bloom_bit(rk_hash(w, sv));
        rk_bloom[bb >> 5] |= 1u << (bb & 31);
        uint32_t i = rk_hash(w, sv) & (rkcap - 1);
        while (rk[i].key) i = (i + 1) & (rkcap - 1);
        rk[i] = DRlocKey{w, (uint32_t)rk_ents.size(), (uint32_t)kv.second.size(), sv};
        rk_ents.insert(rk_ents.end(), kv.second.begin(), kv.second.end());   // ascending k: pushed in k order
    }

    // ---- signatures (parsed up front: the set's decoders shape the location tables)

    struct LitE { uint32_t key; DLit lit; std::string bytes; };
    std::vector<LitE> lits;
    std::vector<DSigRegex> sregex;
    std::vector<uint32_t> always;
    std::vector<Dfa> always_dfa;   // the always regexes' search DFAs (union groups, below)
    std::vector<std::string> always_pat;
    // one prefilter pattern -> its key windows (stride-2 scan, see choose_keys)
    std::unordered_map<uint32_t, uint32_t> key_use;
    auto add_lit = [&](const std::string &pat, const std::string &bytes, uint32_t id, uint8_t flags, uint8_t zones,
                       const std::bitset<256> *follow = nullptr, uint16_t dfa_entry = 0) {
        const DLit d{id, 0, (uint16_t)bytes.size(), flags, zones, 0, dfa_entry};
        for (auto &k : choose_keys(pat, KM, key_use, follow).keys) {
            LitE e{k.first, d, bytes};
            e.lit.key_off = k.second;
            lits.push_back(e);
        }
    };
    for (size_t r = 0; r < sig.size(); r++) {
        const SigRule &g = sig[r];
        if (g.lit) {
            if (g.pat.size() < 4 || g.pat.size() > 0xFFFF) { st.n_rejected_other++; continue; }
            std::string b = g.nocase ? lower(g.pat) : g.pat;
            add_lit(g.pat, b, (uint32_t)r, (uint8_t)(g.nocase ? LIT_NOCASE : 0), (uint8_t)g.zones);
            st.n_sig_literals++;
        } else {
            RegexInfo ri = compile_regex(g.pat, g.nocase);
            if (ri.status != RX_OK) {
                if (ri.status == RX_PCRE_ONLY) st.n_rejected_pcre++; else st.n_rejected_other++;
                continue;
            }
            int d = C.add_dfa(ri.dfa);
            uint32_t ridx = (uint32_t)sregex.size();
            DSigRegex sr{(uint32_t)d, 0, (uint32_t)r, (uint16_t)g.zones, (uint16_t)RXM_TRIGGER};
            st.n_sig_regex++;
            if (ri.prefix_mode) {
                sr.mode = RXM_PREFIX;
                sr.adfa = (uint32_t)C.add_dfa(ri.anchored);
                for (auto &f : ri.prefix)
                    add_lit(f, f, ridx, (uint8_t)(LIT_NOCASE | LIT_TRIGGER | LIT_PREFIX), (uint8_t)g.zones,
                            ri.has_prefix_follow ? &ri.prefix_follow : nullptr, prefix_entry(ri.anchored, f, g.nocase));
            } else if (ri.min_factor < 4) {
                sr.mode = RXM_ALWAYS;
                always.push_back(ridx);
                always_dfa.push_back(ri.dfa);
                always_pat.push_back(g.pat);
                st.n_sig_regex_always++;
            } else {
                for (auto &f : ri.factors)
                    add_lit(f, f, ridx, (uint8_t)(LIT_NOCASE | LIT_TRIGGER), (uint8_t)g.zones,
                            ri.has_factor_follow ? &ri.factor_follow : nullptr);
            }
            sregex.push_back(sr);
        }
    }
    st.n_sigs = (uint32_t)sig.size();
    std::sort(lits.begin(), lits.end(), [](const LitE &a, const LitE &b) {
        return a.key != b.key ? a.key < b.key : a.lit.id < b.lit.id;
    });
    std::vector<DLit> dlits;
    std::vector<DLitChk> dchk;
    std::vector<uint32_t> waf_a(BLOOM_WORDS, 0);   // LDS Bloom image
    // stage-2 context filter: each entry's key window plus the pattern bytes around it
    std::vector<uint32_t> waf_b(BLOOM_WORDS, 0);
    for (const LitE &e : lits) {
        const int k = e.lit.key_off, L = (int)e.bytes.size();
        auto cb = [&](int i) { return (uint32_t)(uint8_t)e.bytes[i] | 0x20u; };
        uint32_t nl = k <= 0 ? 0u : (uint32_t)std::min(2, k);
        uint32_t nr = (uint32_t)std::max(0, std::min(2, L - (k + 4)));
        ctx_canon(nl, nr);
        const uint32_t l2 = (nl >= 2 ? cb(k - 2) : 0u) | (nl >= 1 ? cb(k - 1) << 8 : 0u);
        const uint32_t r2 = (nr >= 1 ? cb(k + 4) : 0u) | (nr >= 2 ? cb(k + 5) << 8 : 0u);
        const BloomProbe b = bloom_probe(ctx_key(e.key, l2, r2, nl * 3 + nr), CTX_MUL_DEFAULT, CTX_PK);
        waf_b[b.block] |= b.mask;
    }
    std::vector<std::pair<uint32_t, std::pair<uint32_t, uint32_t>>> buckets;
    std::vector<uint32_t> keys;
    for (size_t i = 0; i < lits.size(); i++) {
        LitE &e = lits[i];
        e.lit.bytes_off = C.put_bytes(e.bytes);
        dlits.push_back(e.lit);
        {   // the pattern bytes in the 4 arena bytes either side of the key window, folded
            const int k = e.lit.key_off, L = (int)e.bytes.size();
            DLitChk c{0, 0, 0, 0};
            for (int j = 0; j < 4; j++) {
                const int ib = k - 4 + j, ia = k + 4 + j;
                if (ib >= 0 && ib < L) { c.b |= ((uint32_t)(uint8_t)e.bytes[ib] | 0x20u) << (8 * j); c.bmask |= 0xFFu << (8 * j); }
                if (ia >= 0 && ia < L) { c.a |= ((uint32_t)(uint8_t)e.bytes[ia] | 0x20u) << (8 * j); c.amask |= 0xFFu << (8 * j); }
            }
            dchk.push_back(c);
        }
        if (i == 0 || lits[i - 1].key != e.key) {
            buckets.push_back({e.key, {(uint32_t)i, 0}});
            keys.push_back(e.key);
        }
        buckets.back().second.second++;
    }
    // probes per window: K = 4 bits as one bit per byte (BLOOM_PK_PERM: 2 VALU ops per probe on
    // the device), or pk = 3 packed shifts (K = 6, 4 ops) when that cuts the modelled false
    // positives enough: a false positive costs ~20 probes' worth (its 32-byte record and the
    // stage-2 context test)
    uint32_t bloom_pk = BLOOM_PK_DEFAULT, bloom_mul = kBloomMuls[0];
    if (!keys.empty()) {
        BloomChoice b = choose_bloom_mul(keys, bloom_pk, KM, waf_a);
        {
            std::vector<uint32_t> f3(BLOOM_WORDS, 0);
            BloomChoice b3 = choose_bloom_mul(keys, 3, KM, f3, 64);   // (the rarer kind: fewer candidates)
            if (0.4 + 20.0 * b3.fp < 20.0 * b.fp) { b = b3; bloom_pk = 3; waf_a.swap(f3); }
        }
        bloom_mul = b.mul;
        st.bloom_fp_ppm = (uint32_t)std::min(1e9, b.fp * 1e6);
    }
    st.n_waf_keys = (uint32_t)keys.size();
    st.bloom_pk = bloom_pk;
    uint32_t lcap = pow2_at_least(buckets.size() * 2 + 1);
    std::vector<DLitBucket> ltab(lcap, DLitBucket{0, 0, 0, 0});
    for (auto &b : buckets) {
        uint32_t i = lit_bucket_hash(b.first) & (lcap - 1);
        while (ltab[i].count) i = (i + 1) & (lcap - 1);
        ltab[i] = DLitBucket{b.first, b.second.first, b.second.second, 0};
    }

    // ---- stats
    st.n_servers = (uint32_t)M.servers.size();
    st.n_locations = (uint32_t)M.locs.size();
    st.n_counters = st.n_locations + st.n_sigs;
    st.lds_bytes_scan = SCAN_LDS_BYTES;

    // ---- image
    Image I;
    TabHeader &h = R.hdr;
    memset(&h, 0, sizeof h);
    I.buf.resize(sizeof(TabHeader));
    h.magic = 0x47544142u; h.version = 1;
    h.n_ports = (uint32_t)ports.size();
    h.n_names_cap = names_mask + 1; h.n_wild_head_cap = head_mask + 1; h.n_wild_tail_cap = tail_mask + 1;
    h.n_wild = (uint32_t)(head.size() + tail.size());
    h.n_servers = (uint32_t)dservers.size(); h.n_server_ifs = (uint32_t)sifs.size(); h.n_rlocs = (uint32_t)rlocs.size();
    h.n_nodes = (uint32_t)nodes.size(); h.n_edges_cap = ecap; h.n_locs = (uint32_t)dlocs.size();
    h.n_srcs = (uint32_t)C.srcs.size(); h.n_conds = (uint32_t)C.conds.size(); h.n_chain_heads = (uint32_t)C.chain_heads.size();
    h.n_rules = (uint32_t)C.rules.size(); h.n_splits = (uint32_t)C.splits.size(); h.n_parts = (uint32_t)C.parts.size();
    h.n_dfas = (uint32_t)C.dfas.size();
    // k_waf_exact's rings carry a literal index in 24 bits (gm_waf.inc XPOS_MASK)
    if (dlits.size() >= (1u << 24)) { R.code = GM_E_INVAL; R.err = "signature set too large: >= 2^24 prefilter literal rows"; return R; }
    h.n_lit_buckets_cap = lcap; h.n_lits = (uint32_t)dlits.size(); h.n_sig_regex = (uint32_t)sregex.size();
    h.n_always = (uint32_t)always.size(); h.n_sigs = st.n_sigs;
    // ---- union-DFA groups (gm_regex.hpp MultiDfa) packed into LDS slices (gm_tables.hpp
    // DAlwSlice): the always-run signature regexes, then the regex locations of rk_on servers
    std::vector<DAlwGroup> alw;
    std::vector<DAlwSlice> alw_slices;
    std::vector<uint8_t> alw_pack;
    std::vector<uint32_t> alw_rule, always_grouped, always_single;
    // always-run groups: member k's rules are alw_rl[alw_rule[first + k] .. alw_rule[first + k + 1]),
    // each zones << 24 | rule id -- one member per distinct (pattern, nocase), however many rules
    // and zone sets share it (the location slices keep one value per member in alw_rule)
    std::vector<uint32_t> alw_rl;
    auto tab_bytes = [](const MultiDfa &m) {   // the group's rows (gm_tables.hpp DAlwGroup)
        return (size_t)m.n_states * ((size_t)alw_row_cols((uint32_t)m.n_classes) + 4) * 2;
    };
    // greedy: in `order`, a component joins the open group while joinable(first member, it), the
    // group has < ALW_GROUP_MAX members and the minimised union's rows stay within
    // ALW_GROUP_BYTES; a component that cannot form a group even alone goes to `single`
    auto form_groups = [&](const std::vector<const Dfa *> &comps, const std::vector<uint32_t> &order, auto joinable,
                           std::vector<std::vector<uint32_t>> &gmem, std::vector<MultiDfa> &gdfa,
                           std::vector<uint32_t> &single) {
        std::vector<uint32_t> cur;
        MultiDfa cur_m;
        auto close = [&]() {
            if (!cur.empty()) { gmem.push_back(cur); gdfa.push_back(std::move(cur_m)); }
            cur.clear();
        };
        for (uint32_t x : order) {
            if (!cur.empty() && joinable(cur[0], x) && cur.size() < ALW_GROUP_MAX) {
                std::vector<const Dfa *> cs;
                for (uint32_t y : cur) cs.push_back(comps[y]);
                cs.push_back(comps[x]);
                MultiDfa m;
                if (build_multi(cs, (int)ALW_BUILD_STATES, m) && tab_bytes(m) <= ALW_GROUP_BYTES &&
                    m.n_classes <= ALW_CLASSES_MAX) {
                    cur.push_back(x); cur_m = std::move(m); continue;
                }
            }
            close();
            MultiDfa m;
            if (build_multi({comps[x]}, (int)ALW_BUILD_STATES, m) && tab_bytes(m) <= ALW_GROUP_BYTES &&
                m.n_classes <= ALW_CLASSES_MAX) {
                cur.push_back(x); cur_m = std::move(m);
            } else single.push_back(x);
        }
        close();
    };
    // slices: consecutive groups, <= ALW_SLICE_GROUPS of them within ALWAYS_LDS_BYTES; member k of
    // group g stores val(g, k) in alw_rule and scans the zones zones(g, k)
    bool alw_layout_err = false;   // (an internal invariant: the class table's offsets are the rows')
    auto pack_slices = [&](const std::vector<std::vector<uint32_t>> &gmem, const std::vector<MultiDfa> &gdfa,
                           auto val, auto zones, uint32_t server, const std::vector<std::vector<uint32_t>> *mrules = nullptr) {
        auto pad16 = [&]() { alw_pack.resize((alw_pack.size() + 15) & ~size_t(15), 0); };
        for (size_t g0 = 0; g0 < gmem.size();) {
            // the class table's size grows at the fifth group (alw_cls_bytes)
            size_t g1 = g0, rows_bytes = 0;
            while (g1 < gmem.size() && g1 - g0 < ALW_SLICE_GROUPS &&
                   alw_cls_bytes((uint32_t)(g1 - g0 + 1)) + rows_bytes + tab_bytes(gdfa[g1]) + 16 <= ALWAYS_LDS_BYTES)
                rows_bytes += ((tab_bytes(gdfa[g1++]) + 15) & ~size_t(15));
            DAlwSlice sl{};
            sl.off = (uint32_t)alw_pack.size();
            sl.first_group = (uint32_t)alw.size();
            sl.n_groups = (uint32_t)(g1 - g0);
            sl.server = server;
            // the dead row (zeros), then clsa[b * NGB + j] = 2 x byte b's class in group j: the byte
            // offset of b's column within group j's rows (alw_cls_bytes; NGB = 4 or 8 bytes per byte)
            const uint32_t ngb = alw_cls_ngb(sl.n_groups), hdr = alw_cls_bytes(sl.n_groups);
            std::vector<uint32_t> tro(g1 - g0, 0);
            {
                uint32_t o = hdr;
                for (size_t j = g0; j < g1; j++) { tro[j - g0] = o; o += (uint32_t)((tab_bytes(gdfa[j]) + 15) & ~size_t(15)); }
                if (o > 4u * 65535u) alw_layout_err = true;   // (rows / 4 fit a u16: never past the LDS)
            }
            std::vector<uint8_t> clsa(hdr, 0);
            for (size_t j = g0; j < g1; j++) {
                for (int b = 0; b < 256; b++)
                    clsa[ALW_DEAD_BYTES + (size_t)b * ngb + (j - g0)] = (uint8_t)(2u * gdfa[j].cls[b]);
                clsa[ALW_DEAD_BYTES + (size_t)ALW_CLS_IDENTITY * ngb + (j - g0)] = (uint8_t)(2u * (uint32_t)gdfa[j].n_classes);
            }
            const uint8_t *cb = reinterpret_cast<const uint8_t *>(clsa.data());
            alw_pack.insert(alw_pack.end(), cb, cb + hdr);
            for (size_t j = g0; j < g1; j++) {
                const MultiDfa &m = gdfa[j];
                const size_t S = (size_t)m.n_states, Cn = (size_t)m.n_classes, Cp = alw_row_cols((uint32_t)Cn), R = Cp + 4;
                DAlwGroup g{};
                g.tr_off = (uint32_t)(alw_pack.size() - sl.off);
                if (g.tr_off != tro[j - g0]) alw_layout_err = true;
                g.mask_off = (uint32_t)(2 * Cp);
                // states renumbered: the dead state 0, the others, then the emitting ones (an emit
                // mask, or the target of a transition flagged MDFA_EMIT) from row emit_row on
                std::vector<uint8_t> emits(S, 0);
                for (size_t q = 1; q < S; q++) {
                    if (m.emit[q]) emits[q] = 1;
                    for (size_t c = 0; c < Cn; c++)
                        if (m.trans[q * Cn + c] & MDFA_EMIT) emits[m.trans[q * Cn + c] & 0x3FFF] = 1;
                }
                emits[0] = 0;
                std::vector<uint32_t> perm(S, 0);
                uint32_t nid = 1;
                for (size_t q = 1; q < S; q++) if (!emits[q]) perm[q] = nid++;
                // a state's row: its byte offset in the slice / 4; the dead state 0 (the shared dead row)
                const uint32_t gb = tro[j - g0];
                auto row4 = [&](uint32_t id) -> uint16_t { return id ? (uint16_t)((gb + 2 * R * id) >> 2) : (uint16_t)0; };
                g.emit_row = row4(nid);
                for (size_t q = 1; q < S; q++) if (emits[q]) perm[q] = nid++;
                g.start_row = row4(perm[1]);
                std::vector<uint16_t> rows(S * R, 0);
                for (size_t q = 1; q < S; q++) {
                    const size_t o = (size_t)perm[q] * R;
                    for (size_t c = 0; c < Cn; c++)
                        rows[o + c] = row4(perm[m.trans[q * Cn + c] & 0x3FFF]);
                    rows[o + Cn] = row4(perm[q]);   // the identity column
                    rows[o + Cp] = (uint16_t)m.emit[q]; rows[o + Cp + 1] = (uint16_t)(m.emit[q] >> 16);
                    rows[o + Cp + 2] = (uint16_t)m.endm[q]; rows[o + Cp + 3] = (uint16_t)(m.endm[q] >> 16);
                }
                const uint8_t *rb = reinterpret_cast<const uint8_t *>(rows.data());
                alw_pack.insert(alw_pack.end(), rb, rb + rows.size() * 2);
                pad16();
                g.n_classes = (uint32_t)Cn; g.n_states = (uint32_t)S;
                g.first = (uint32_t)alw_rule.size();
                for (size_t k = 0; k < gmem[j].size(); k++) {
                    if (mrules) {   // the member's rule list (val: its entries, zones << 24 | rule)
                        alw_rule.push_back((uint32_t)alw_rl.size());
                        for (uint32_t e : (*mrules)[gmem[j][k]]) alw_rl.push_back(e);
                    } else {
                        alw_rule.push_back(val(j, k));
                    }
                    const uint32_t zk = zones(j, k);
                    for (uint32_t z = 0; z < 4; z++)
                        if (zk & (1u << z)) g.zone_mask[z] |= 1u << k;
                    g.zones |= zk;
                }
                if (mrules) alw_rule.push_back((uint32_t)alw_rl.size());   // the last member's end
                sl.zones |= g.zones;
                st.n_alw_states += (uint32_t)S;
                alw.push_back(g);
            }
            sl.len = (uint32_t)(alw_pack.size() - sl.off);
            alw_slices.push_back(sl);
            g0 = g1;
        }
    };
    // the always-run regexes, ordered by (zone set, pattern text) -- the same shapes side by side,
    // whose unions stay small; a group holds one zone set.  `always` is reordered: the grouped
    // regexes first (group order), then those left to the per-regex kernel.
    {
        // members: one per distinct (pattern, nocase) -- the same search DFA -- with every rule
        // that uses it (its zones the union of theirs); a match of member k in zone z emits the
        // member's rules that scan z
        std::map<std::string, uint32_t> ukey;
        std::vector<uint32_t> urep;                      // member -> its first always index
        std::vector<std::vector<uint32_t>> uall, mrules;  // member -> always indices / rule entries
        std::vector<uint32_t> uzones;
        for (uint32_t x = 0; x < always.size(); x++) {
            const DSigRegex &sr = sregex[always[x]];
            const std::string key = always_pat[x] + (sig[sr.rule].nocase ? std::string("\x01i") : std::string("\x01c"));
            auto it = ukey.find(key);
            uint32_t m;
            if (it == ukey.end()) {
                m = (uint32_t)urep.size();
                ukey.emplace(key, m);
                urep.push_back(x); uall.emplace_back(); mrules.emplace_back(); uzones.push_back(0);
            } else m = it->second;
            uall[m].push_back(x);
            mrules[m].push_back((uint32_t)(sr.zones & 15u) << 24 | sr.rule);
            uzones[m] |= sr.zones & 15u;
        }
        st.n_alw_members = (uint32_t)urep.size();
        std::vector<const Dfa *> comps;
        for (uint32_t m = 0; m < urep.size(); m++) comps.push_back(&always_dfa[urep[m]]);
        std::vector<uint32_t> ord(urep.size());
        for (uint32_t i = 0; i < ord.size(); i++) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
            return uzones[x] != uzones[y] ? uzones[x] < uzones[y] : always_pat[urep[x]] < always_pat[urep[y]];
        });
        std::vector<std::vector<uint32_t>> gmem;
        std::vector<MultiDfa> gdfa;
        std::vector<uint32_t> single;
        form_groups(comps, ord, [&](uint32_t a, uint32_t b) { return uzones[a] == uzones[b]; }, gmem, gdfa, single);
        pack_slices(gmem, gdfa, [](size_t, size_t) { return 0u; },
                    [&](size_t j, size_t k) { return uzones[gmem[j][k]]; }, GM_NONE, &mrules);
        for (auto &gm : gmem) for (uint32_t m : gm) for (uint32_t x : uall[m]) always_grouped.push_back(always[x]);
        for (uint32_t m : single) for (uint32_t x : uall[m]) always_single.push_back(always[x]);
    }
    const uint32_t n_alw_slices = (uint32_t)alw_slices.size();
    // the regex locations of every rk_on server, in config order (consecutive groups, so the
    // first group with a match holds the first matching regex); a PCRE-only location carries its
    // superset DFA, one without any DFA matches at once (a DFA whose start state accepts).  A
    // server with a regex no group can hold keeps the factor prefilter.
    {
        rsl_pbit.assign(rlocs.size(), 0xFF);
        Dfa match_all;
        match_all.n_states = 2; match_all.n_classes = 1;
        match_all.trans.assign(2, 0); match_all.trans[1] = 1;
        match_all.acc = {0, 1};
        match_all.anchored_start = true;
        memset(match_all.cls, 0, sizeof match_all.cls);
        for (auto &Sv : M.servers) {
            DServer &D = dservers[Sv.id];
            if (!D.rk_on) continue;
            std::vector<Dfa> own(D.n_rloc);
            std::vector<const Dfa *> comps(D.n_rloc);
            for (uint32_t k = 0; k < D.n_rloc; k++) {
                const DRegexLoc &rl = rlocs[D.first_rloc + k];
                if (rl.dfa == GM_NONE) { comps[k] = &match_all; continue; }
                const DDfa &dd = C.dfas[rl.dfa];
                Dfa &o = own[k];
                o.n_states = dd.n_states; o.n_classes = dd.n_classes;
                o.anchored_start = (dd.flags & DFA_ANCHOR_START) != 0;
                o.trans.resize((size_t)dd.n_states * dd.n_classes);
                for (size_t i = 0; i < o.trans.size(); i++) o.trans[i] = C.dfa_trans[dd.trans_off + i] & DFA_TRANS_STATE_MASK;
                o.acc.assign(C.dfa_acc.begin() + dd.acc_off, C.dfa_acc.begin() + dd.acc_off + dd.n_states);
                for (int b2 = 0; b2 < 256; b2++) o.cls[b2] = C.dfa_cls[dd.cls_off + b2];
                comps[k] = &o;
            }
            // anchored (^) and unanchored regexes in separate groups, each in config order: a
            // union of anchored regexes dies within a few bytes of most URIs; the groups are then
            // ordered by their first (lowest) member
            // X$ regexes with a reversed DFA form groups of their own (run backwards: slices
            // flagged ALW_SLICE_REVERSED, packed first -- they are cheap, and the matches they
            // find let later slices skip requests)
            // The slices, in this order: reversed (X$), anchored, unanchored without a factor,
            // unanchored with factors (prefiltered, below) -- cheap slices first, so that the
            // matches they find let the costly ones skip requests; within a kind, config order
            std::vector<uint32_t> ord_a, ord_un, ord_uf, ord_r;
            std::vector<const Dfa *> rcomps(D.n_rloc, nullptr);
            std::vector<std::vector<uint32_t>> heads(D.n_rloc);
            for (uint32_t k = 0; k < D.n_rloc; k++) {
                const Dfa &rv = rloc_rev[D.first_rloc + k];
                if (rv.n_states > 0) {
                    rcomps[k] = &rv;
                    ord_r.push_back(k);
                    // (a reversed DFA reads the $uri from its end: its heads are the last bytes)
                    heads[k].assign(RSL_HEAD_WORDS, 0u);
                    dfa_heads(rv, heads[k]);
                }
                else if (comps[k]->anchored_start) {
                    ord_a.push_back(k);
                    heads[k].assign(RSL_HEAD_WORDS, 0u);
                    dfa_heads(*comps[k], heads[k]);
                }
                else if (rlocs[D.first_rloc + k].dfa != GM_NONE && !rloc_factors[D.first_rloc + k].empty())
                    ord_uf.push_back(k);
                else ord_un.push_back(k);
            }
            // anchored regexes by their lowest head (config order among equal ones): a group then
            // holds regexes that start alike, so each anchored slice's head map is narrow and a
            // $uri's first two bytes pick few slices (the first match in config order is the
            // lowest index any slice finds, whatever the slices' order)
            auto head0 = [&](uint32_t k) {
                for (uint32_t w = 0; w < RSL_HEAD_WORDS; w++)
                    if (heads[k][w]) return w * 32 + (uint32_t)__builtin_ctz(heads[k][w]);
                return 0xFFFFFFFFu;
            };
            // (narrow maps first -- a few starts each, grouped by their lowest -- then the broader
            // ones, which select most requests wherever they go)
            auto breadth = [&](uint32_t k) {
                uint32_t c = 0;
                for (uint32_t w = 0; w < RSL_HEAD_WORDS; w++) c += (uint32_t)__builtin_popcount(heads[k][w]);
                return c <= 16 ? 0u : c <= 1024 ? 1u : 2u;
            };
            std::vector<uint32_t> hb(rcomps.size(), 0), h0(rcomps.size(), 0);
            for (uint32_t k : ord_a) { hb[k] = breadth(k); h0[k] = head0(k); }
            for (uint32_t k : ord_r) { hb[k] = breadth(k); h0[k] = head0(k); }
            auto by_heads = [&](uint32_t a, uint32_t b) { return hb[a] != hb[b] ? hb[a] < hb[b] : h0[a] < h0[b]; };
            std::stable_sort(ord_a.begin(), ord_a.end(), by_heads);
            std::stable_sort(ord_r.begin(), ord_r.end(), by_heads);
            std::vector<std::vector<uint32_t>> gm_a, gm_un, gm_uf, gm_r;
            std::vector<MultiDfa> gd_a, gd_un, gd_uf, gd_r;
            std::vector<uint32_t> single;
            auto all = [](uint32_t, uint32_t) { return true; };
            form_groups(comps, ord_a, all, gm_a, gd_a, single);
            form_groups(comps, ord_un, all, gm_un, gd_un, single);
            form_groups(comps, ord_uf, all, gm_uf, gd_uf, single);
            form_groups(rcomps, ord_r, all, gm_r, gd_r, single);
            if (!single.empty()) { h.n_rk_prefilter++; st.n_rk_prefilter++; continue; }
            D.rsl_first = (uint32_t)alw_slices.size();
            const uint32_t fr = D.first_rloc;
            auto pack_kind = [&](std::vector<std::vector<uint32_t>> &gmk, std::vector<MultiDfa> &gdk, uint32_t flags) {
                const size_t s0 = alw_slices.size();
                if (!gmk.empty())
                    pack_slices(gmk, gdk, [&](size_t j, size_t k) { return fr + gmk[j][k]; },
                                [](size_t, size_t) { return 1u; }, (uint32_t)Sv.id);
                for (size_t k = s0; k < alw_slices.size(); k++) alw_slices[k].flags |= flags;
                return (uint32_t)(alw_slices.size() - s0);
            };
            // each anchored or reversed slice's head map: the OR of its members'
            auto assign_heads = [&](size_t a0) {
            for (size_t k = a0; k < alw_slices.size(); k++) {
                const uint32_t slot = (uint32_t)(rsl_heads.size() / RSL_HEAD_WORDS);
                if (slot >= RSL_HEADS_MAX) break;
                rsl_heads.resize(rsl_heads.size() + RSL_HEAD_WORDS, 0u);
                uint32_t *hb = rsl_heads.data() + (size_t)slot * RSL_HEAD_WORDS;
                const DAlwSlice &sl = alw_slices[k];
                for (uint32_t g = sl.first_group; g < sl.first_group + sl.n_groups; g++)
                    for (uint32_t q = 0; q < (uint32_t)__builtin_popcount(alw[g].zone_mask[0]); q++) {
                        const uint32_t m = alw_rule[alw[g].first + q] - fr;
                        for (uint32_t w = 0; w < RSL_HEAD_WORDS; w++) hb[w] |= heads[m][w];
                    }
                alw_slices[k].flags |= ALW_SLICE_HEADS | slot << 16;
                rsl_head_slice.push_back((uint32_t)k);
            }
            };
            const size_t r0 = alw_slices.size();
            st.n_rsl_reversed += pack_kind(gm_r, gd_r, ALW_SLICE_REVERSED);
            assign_heads(r0);
            const size_t a0 = alw_slices.size();
            pack_kind(gm_a, gd_a, 0);
            assign_heads(a0);
            pack_kind(gm_un, gd_un, 0);
            pack_kind(gm_uf, gd_uf, 0);
            D.rsl_n = (uint32_t)alw_slices.size() - D.rsl_first;
            // the lowest regex-location index a slice holds (members of a head-ordered anchored group
            // are not in config order: the minimum over all of them)
            for (uint32_t k = D.rsl_first; k < D.rsl_first + D.rsl_n; k++) {
                const DAlwSlice &sl = alw_slices[k];
                uint32_t mn = 0xFFFFFFFFu;
                for (uint32_t g = sl.first_group; g < sl.first_group + sl.n_groups; g++)
                    for (uint32_t q = 0; q < (uint32_t)__builtin_popcount(alw[g].zone_mask[0]); q++)
                        mn = std::min(mn, alw_rule[alw[g].first + q]);
                alw_slices[k].min_member = mn;
            }
            st.n_rsl_slices += D.rsl_n;
            // forward slices of unanchored regexes that all have >= 4-byte factors run only for
            // the requests whose $uri holds a factor of one of them: k_rloc_pref sets bit
            // (slice - rsl_first) & 63 of a request's mask per factor found (the rk tables above)
            for (uint32_t s2 = D.rsl_first; s2 < D.rsl_first + D.rsl_n; s2++) {
                DAlwSlice &sl = alw_slices[s2];
                if (sl.flags & ALW_SLICE_REVERSED) continue;
                std::vector<uint32_t> mem;
                for (uint32_t g = sl.first_group; g < sl.first_group + sl.n_groups; g++)
                    for (uint32_t k = 0; k < (uint32_t)__builtin_popcount(alw[g].zone_mask[0]); k++)
                        mem.push_back(alw_rule[alw[g].first + k]);
                bool pref = !mem.empty();
                for (uint32_t m : mem)
                    if (rlocs[m].dfa == GM_NONE || rloc_factors[m].empty() || comps[m - fr]->anchored_start) pref = false;
                if (!pref) continue;
                const uint32_t bit = (s2 - D.rsl_first) & 63u;
                sl.flags |= ALW_SLICE_PREF | bit << 8;
                for (uint32_t m : mem) rsl_pbit[m] = (uint8_t)bit;
                st.n_rsl_pref++;
            }
        }
    }
    h.n_always_lds = (uint32_t)always_grouped.size();
    h.n_alw_groups = (uint32_t)alw.size();
    h.n_alw_slices = n_alw_slices;
    h.n_rsl = (uint32_t)alw_slices.size() - n_alw_slices;
    h.alw_pack_len = (uint32_t)alw_pack.size();
    st.n_alw_groups = h.n_alw_groups; st.n_alw_slices = h.n_alw_slices;
    st.n_alw_single = (uint32_t)always_single.size();
    always = always_grouped;
    always.insert(always.end(), always_single.begin(), always_single.end());
    // the route's hot tables first, contiguous (k_route stages them into LDS when they fit)
    h.off_ports = I.put(ports);
    h.off_names = I.put(tab_exact); h.off_wild_head = I.put(tab_head); h.off_wild_tail = I.put(tab_tail);
    h.off_servers = I.put(dservers); h.off_server_ifs = I.put(sifs);
    h.off_small = I.put(smalls); h.off_locs = I.put(dlocs);
    name_bytes.resize(name_bytes.size() + 64, 0);   // slack: 16-B block loads may over-read
    h.off_name_bytes = I.put(name_bytes);
    h.off_hot_end = (I.buf.size() + 15) & ~size_t(15);
    h.off_rlocs = I.put(rlocs);
    h.off_nodes = I.put(nodes); h.off_edges = I.put(edges);
    h.off_srcs = I.put(C.srcs); h.off_conds = I.put(C.conds); h.off_chain_heads = I.put(C.chain_heads);
    h.off_rules = I.put(C.rules); h.off_rtab = I.put(C.rtab); h.off_rtargets = I.put(C.rtargets);
    h.off_splits = I.put(C.splits); h.off_parts = I.put(C.parts);
    h.off_dfas = I.put(C.dfas); h.off_dfa_trans = I.put(C.dfa_trans); h.off_dfa_acc = I.put(C.dfa_acc);
    h.off_dfa_cls = I.put(C.dfa_cls);
    h.off_waf_a = I.put(waf_a); h.off_waf_b = I.put(waf_b);
    h.off_lit_buckets = I.put(ltab); h.off_lits = I.put(dlits); h.off_sig_regex = I.put(sregex);
    h.off_always = I.put(always);
    h.off_alw = I.put(alw); h.off_alw_slices = I.put(alw_slices); h.off_alw_pack = I.put(alw_pack);
    h.off_alw_rule = I.put(alw_rule);
    h.off_alw_rl = I.put(alw_rl);
    h.off_lit_chk = I.put(dchk);
    rsl_pbit.resize((rsl_pbit.size() + 3) & ~size_t(3), 0xFF);
    h.off_rsl_pbit = I.put(rsl_pbit);
    if (rsl_heads.empty()) rsl_heads.assign(1, 0u);
    h.n_rsl_heads = (uint32_t)(rsl_heads.size() / RSL_HEAD_WORDS);
    if (alw_layout_err) { R.code = GM_E_INVAL; R.err = "internal: union-DFA slice layout"; return R; }
    st.n_rsl_heads = (uint32_t)rsl_head_slice.size();
    h.off_rsl_heads = I.put(rsl_heads);
    rsl_head_slice.resize(std::max<size_t>(rsl_head_slice.size(), 1), 0u);
    h.off_rsl_head_slice = I.put(rsl_head_slice);
    // (before the upstream section: gm_update_upstream copies everything before it unchanged)
    h.n_realip = (uint32_t)realips.size(); h.n_cidrs = (uint32_t)cidrs.size();
    st.n_realip = h.n_realip;
    h.off_realip = I.put(realips); h.off_cidrs = I.put(cidrs);
    h.n_acc_rules = (uint32_t)acc_rules.size(); h.n_acc_lists = (uint32_t)acc_lists.size();
    h.off_acc_rules = I.put(acc_rules); h.off_acc_lists = I.put(acc_lists);
    h.n_rk_cap = rkcap; h.n_rk_ids = (uint32_t)rk_ids.size(); h.n_rk_ents_keys = (uint32_t)rk_lists.size();
    h.off_rk = I.put(rk); h.off_rk_ids = I.put(rk_ids); h.off_rk_ents = I.put(rk_ents); h.off_rk_bloom = I.put(rk_bloom);
    h.n_rk_ents_n = (uint32_t)rk_ents.size();
    h.n_ups = (uint32_t)dups.size(); h.n_peers = (uint32_t)peer_init.size();
    h.n_key_parts = (uint32_t)key_parts.size(); h.n_points = (uint32_t)points.size();
    h.off_ups = I.put(dups); h.off_key_parts = I.put(key_parts); h.off_points = I.put(points);
    h.off_peer_init = I.put(peer_init);
    {
        std::vector<uint32_t> peer_md5;
        for (const std::string &a : R.peer_addrs) put_md5(peer_md5, a);
        h.off_peer_md5 = I.put(peer_md5);
    }
    h.off_loc_uri = I.put(dluri);
    h.decoders = decoders;
    C.bytes.resize(C.bytes.size() + 64, 0);   // slack: vector compares may over-read
    h.off_bytes = I.put(C.bytes);
    I.buf.resize((I.buf.size() + 255) & ~size_t(255), 0);
    h.total = I.buf.size();
    h.bloom_log2 = BLOOM_LOG2; h.bloom_mul = bloom_mul; h.bloom_pk = bloom_pk; h.ctx_mul = CTX_MUL_DEFAULT;
    memcpy(I.buf.data(), &h, sizeof h);
    st.table_bytes = h.total;
    R.image = std::move(I.buf);
    R.ok = true;
    return R;
}

CompileResult update_upstream(const CompileResult &live, const std::string &name, const std::vector<std::string> &addrs) {
    CompileResult R;
    const TabHeader &h0 = live.hdr;
    const uint8_t *b = live.image.data();
    const uint32_t nu = h0.n_ups;
    uint32_t uu = GM_NONE;
    for (uint32_t u = 0; u < nu && u < live.ups_meta.size(); u++)
        if (live.ups_meta[u].name == name) { uu = u; break; }
    if (uu == GM_NONE) { R.code = GM_E_INVAL; R.err = "no upstream named '" + name + "'"; return R; }
    const DUpstream *ou = (const DUpstream *)(b + h0.off_ups);
    const DPoint *opt = (const DPoint *)(b + h0.off_points);
    const uint32_t *oinit = (const uint32_t *)(b + h0.off_peer_init);
    std::vector<DUpstream> dups(ou, ou + nu);
    std::vector<DPoint> points;
    std::vector<uint32_t> peer_init;
    R.stats = live.stats;
    R.stats.n_upstreams_deferred = 0;
    R.ups_meta = live.ups_meta;
    for (uint32_t u = 0; u < nu; u++) {
        DUpstream &D = dups[u];
        const DUpstream &O = ou[u];
        D.first_peer = (uint32_t)peer_init.size();
        if (u != uu) {
            for (uint32_t j = 0; j < O.n_peers; j++) {
                peer_init.push_back(oinit[O.first_peer + j]);
                R.peer_addrs.push_back(live.peer_addrs[O.first_peer + j]);
                R.peer_ups.push_back(u);
                R.peer_map.push_back(O.first_peer + j);
            }
            D.first_point = (uint32_t)points.size();
            points.insert(points.end(), opt + O.first_point, opt + O.first_point + O.n_points);
            if (D.method == UM_DEFER) R.stats.n_upstreams_deferred++;
            continue;
        }
        // the updated upstream in NGINX Plus's order after UpdateHTTPServers (the API client deletes
        // the servers not listed and POSTs the new ones, each appended to the upstream's peer list):
        // the kept servers in their previous relative order, then the added ones in the order given.
        // A kept address keeps its state (gm_peers_migrate).  (The order of a live Plus upstream is
        // parity-unpinned: no reference fixture covers it; the tests check this rule.)
        const UpstreamMeta &M = live.ups_meta[u];
        std::vector<bool> taken(addrs.size(), false);
        std::vector<std::string> order;
        auto put = [&](const std::string &a, uint32_t from) {
            peer_init.push_back(0u);   // Plus API servers: none `down`
            R.peer_addrs.push_back(a);
            R.peer_ups.push_back(u);
            R.peer_map.push_back(from);
            order.push_back(a);
        };
        for (uint32_t j = 0; j < O.n_peers; j++) {
            const std::string &old_a = live.peer_addrs[O.first_peer + j];
            for (size_t i = 0; i < addrs.size(); i++)
                if (!taken[i] && addrs[i] == old_a) { taken[i] = true; put(old_a, O.first_peer + j); break; }
        }
        for (size_t i = 0; i < addrs.size(); i++)
            if (!taken[i]) put(addrs[i], GM_NONE);
        D.n_peers = (uint32_t)addrs.size();
        D.method = M.has_block ? M.method : UM_DEFER;
        bool defer = !M.has_block || M.defer_fixed;
        if ((D.method == UM_RR || D.method == UM_LEAST_CONN) && D.n_peers > SEQ_PEERS_MAX) defer = true;
        D.first_point = (uint32_t)points.size();
        D.n_points = 0;
        if (D.method == UM_CHASH && !defer) {
            std::set<std::string> seen;
            for (const std::string &a : order) if (!seen.insert(a).second) defer = true;
            if (!defer) chash_ring(order, points);
            D.n_points = (uint32_t)points.size() - D.first_point;
        }
        if (defer) { D.method = UM_DEFER; R.stats.n_upstreams_deferred++; }
    }
    R.stats.n_peers = (uint32_t)peer_init.size();
    // the image: everything before the upstream section as it is, then the rebuilt section, then
    // the sections after it (DLocUri, the byte pool) moved along -- their contents are offsets into
    // the byte pool, relative to its own base, so they move unchanged
    Image I;
    I.buf.assign(b, b + h0.off_ups);
    TabHeader h = h0;
    h.n_peers = R.stats.n_peers;
    h.n_points = (uint32_t)points.size();
    std::vector<DKeyPart> key_parts((const DKeyPart *)(b + h0.off_key_parts),
                                    (const DKeyPart *)(b + h0.off_key_parts) + h0.n_key_parts);
    std::vector<DLocUri> dluri((const DLocUri *)(b + h0.off_loc_uri), (const DLocUri *)(b + h0.off_loc_uri) + h0.n_locs);
    std::vector<uint8_t> bytes(b + h0.off_bytes, b + h0.total);
    h.off_ups = I.put(dups); h.off_key_parts = I.put(key_parts); h.off_points = I.put(points);
    h.off_peer_init = I.put(peer_init);
    {
        std::vector<uint32_t> peer_md5;
        for (const std::string &a : R.peer_addrs) put_md5(peer_md5, a);
        h.off_peer_md5 = I.put(peer_md5);
    }
    h.off_loc_uri = I.put(dluri);
    h.off_bytes = I.put(bytes);
    I.buf.resize((I.buf.size() + 255) & ~size_t(255), 0);
    h.total = I.buf.size();
    memcpy(I.buf.data(), &h, sizeof h);
    R.stats.table_bytes = h.total;
    R.hdr = h;
    R.image = std::move(I.buf);
    R.ok = true;
    return R;
}

GTab make_gtab(const TabHeader &h, const uint8_t *b, uint32_t gen) {
    GTab t{};
    t.ports = (const DPort *)(b + h.off_ports);
    t.names = (const DName *)(b + h.off_names);
    t.wild_head = (const DName *)(b + h.off_wild_head);
    t.wild_tail = (const DName *)(b + h.off_wild_tail);
    t.servers = (const DServer *)(b + h.off_servers);
    t.server_ifs = (const DServerIf *)(b + h.off_server_ifs);
    t.rlocs = (const DRegexLoc *)(b + h.off_rlocs);
    t.nodes = (const DNode *)(b + h.off_nodes);
    t.edges = (const DEdge *)(b + h.off_edges);
    t.locs = (const DLoc *)(b + h.off_locs);
    t.srcs = (const DSrc *)(b + h.off_srcs);
    t.conds = (const DCond *)(b + h.off_conds);
    t.chain_heads = (const uint32_t *)(b + h.off_chain_heads);
    t.rules = (const DRules *)(b + h.off_rules);
    t.rtab = b + h.off_rtab;
    t.rtargets = (const uint32_t *)(b + h.off_rtargets);
    t.splits = (const DSplit *)(b + h.off_splits);
    t.parts = (const DPart *)(b + h.off_parts);
    t.dfas = (const DDfa *)(b + h.off_dfas);
    t.dfa_trans = (const uint16_t *)(b + h.off_dfa_trans);
    t.dfa_acc = b + h.off_dfa_acc;
    t.dfa_cls = b + h.off_dfa_cls;
    t.bytes = b + h.off_bytes;
    t.waf_a = (const uint32_t *)(b + h.off_waf_a);
    t.waf_b = (const uint32_t *)(b + h.off_waf_b);
    t.lit_buckets = (const DLitBucket *)(b + h.off_lit_buckets);
    t.lits = (const DLit *)(b + h.off_lits);
    t.sig_regex = (const DSigRegex *)(b + h.off_sig_regex);
    t.always = (const uint32_t *)(b + h.off_always);
    t.rk = (const DRlocKey *)(b + h.off_rk);
    t.rk_ids = (const uint32_t *)(b + h.off_rk_ids);
    t.rk_mask = h.n_rk_cap - 1;
    t.small = (const DSmallLoc *)(b + h.off_small);
    t.rk_ents = (const DRlocEnt *)(b + h.off_rk_ents);
    t.rk_bloom = (const uint32_t *)(b + h.off_rk_bloom);
    t.rk_keys = h.n_rk_ents_keys;
    t.name_bytes = b + h.off_name_bytes;
    t.hot_base = b + h.off_ports;
    t.hot_len = h.off_hot_end - h.off_ports <= ROUTE_STAGE_BYTES ? (uint32_t)(h.off_hot_end - h.off_ports) : 0u;
    t.ups = (const DUpstream *)(b + h.off_ups);
    t.key_parts = (const DKeyPart *)(b + h.off_key_parts);
    t.points = (const DPoint *)(b + h.off_points);
    t.peer_init = (const uint32_t *)(b + h.off_peer_init);
    t.peer_md5 = (const uint32_t *)(b + h.off_peer_md5);
    t.n_ups = h.n_ups; t.n_peers = h.n_peers; t.n_servers = h.n_servers;
    t.loc_uri = (const DLocUri *)(b + h.off_loc_uri);
    t.decoders = h.decoders;
    t.alw = (const DAlwGroup *)(b + h.off_alw);
    t.alw_slices = (const DAlwSlice *)(b + h.off_alw_slices);
    t.alw_pack = b + h.off_alw_pack;
    t.alw_rule = (const uint32_t *)(b + h.off_alw_rule);
    t.alw_rl = (const uint32_t *)(b + h.off_alw_rl);
    t.lit_chk = (const DLitChk *)(b + h.off_lit_chk);
    t.rsl_pbit = b + h.off_rsl_pbit;
    t.rsl_heads = (const uint32_t *)(b + h.off_rsl_heads);
    t.n_rsl_heads = h.n_rsl_heads;
    t.rsl_head_slice = (const uint32_t *)(b + h.off_rsl_head_slice);
    t.realip = (const DRealIp *)(b + h.off_realip);
    t.cidrs = (const DCidr *)(b + h.off_cidrs);
    t.acc_rules = (const DAccRule *)(b + h.off_acc_rules);
    t.acc_lists = (const DAccList *)(b + h.off_acc_lists);
    t.n_always_lds = h.n_always_lds; t.n_alw_groups = h.n_alw_groups; t.n_alw_slices = h.n_alw_slices;
    t.n_rsl = h.n_rsl; t.n_rk_prefilter = h.n_rk_prefilter;
    t.n_ports = h.n_ports;
    t.names_mask = h.n_names_cap - 1; t.wild_head_mask = h.n_wild_head_cap - 1; t.wild_tail_mask = h.n_wild_tail_cap - 1;
    t.n_wild = h.n_wild;
    t.edges_mask = h.n_edges_cap - 1; t.lit_mask = h.n_lit_buckets_cap - 1;
    t.n_locs = h.n_locs; t.n_sigs = h.n_sigs; t.n_sig_regex = h.n_sig_regex; t.n_always = h.n_always;
    t.n_lits = h.n_lits;
    t.bloom_log2 = h.bloom_log2; t.bloom_mul = h.bloom_mul; t.bloom_pk = h.bloom_pk; t.ctx_mul = h.ctx_mul;
    t.gen = gen;
    return t;
}

}  // namespace gm
