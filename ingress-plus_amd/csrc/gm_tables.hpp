// gm_tables.hpp -- device-resident table generation: layout shared by the host compiler
// (gm_compile.cpp) and the gfx950 kernels (gm_device.hip).
//
// One generation = one contiguous image in HBM (copy-in at gm_load_generation).  Every section
// is an array of plain structs at a 16-byte aligned offset; `GTab` carries the device pointers
// by value into every kernel launch.  Sizes are small (KB..MB) and read-mostly, so after first
// touch they live in L2 / Infinity Cache; the hot WAF bitmap is staged into LDS per workgroup.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace gm {

// ---- servers / hosts -----------------------------------------------------------------
struct DPort {               // one entry per distinct listen port
    uint32_t port;
    uint32_t ssl;            // any `listen <port> ssl`
    uint32_t default_server; // `default_server` or first server listening on the port
    uint32_t proxy;          // any `listen <port> ... proxy_protocol` (nginx ORs the option per port)
};

// open-addressing hash: exact names and wildcard keys, keyed by (port index, lowercase name)
struct DName {
    uint32_t hash;           // 0 = empty slot
    uint32_t name_off;       // into bytes pool
    uint16_t name_len;
    uint16_t port_idx;
    uint32_t server;
};

// SIF_FLAGS: the variable depends only on (https, http2) -- $scheme, $https, $http2 -- so the
// compiler evaluates the condition for the 4 flag combinations: hit = tt >> (flags & 3) & 1.
enum : uint32_t { SIF_EQ = 1, SIF_NE = 2, SIF_RETURN = 3, SIF_FLAGS = 7 };
struct DServer {
    uint32_t trie_root;      // node index of this server's location trie
    uint32_t first_if, n_if; // server rewrite-phase `if (...) { return }` list (DServerIf)
    uint32_t first_rloc, n_rloc;  // regex locations (DRegexLoc), config order
    uint32_t waf_mode;
    uint32_t trie_depth;     // longest exact / prefix location name: URI bytes the trie walk reads
    uint32_t rk_on;          // regex locations behind the factor prefilter (n_rloc > RLOC_SEQ_MAX)
    uint32_t first_ralw, n_ralw;  // rk_ids slice: regex locations evaluated for every URI (no
                                  // >= 4-byte factor, or PCRE-only), ascending
    uint32_t sl_first, sl_n;      // small-server location list (DSmallLoc), sl_n = 0: trie walk
    uint32_t rsl_first, rsl_n;    // rk_on servers: union-DFA slices of the regex locations
                                  // (DAlwSlice, config order; rsl_n = 0: the factor prefilter)
    uint32_t realip;              // DRealIp index (set_real_ip_from ...), GM_NONE: none
    uint32_t body_max;            // client_max_body_size of the server level (a request that
                                  // matches no location), BODY_UNLIMITED: none
    uint32_t access;              // DAccList of the server level's allow / deny (a request that
                                  // matches no location), GM_NONE: none
};
// client_max_body_size (version1/nginx.ingress.tmpl:175, version2/nginx.virtualserver.tmpl:93):
// a body longer than this gets 413; 0 (nginx's "no limit") and limits >= 4 GiB never trigger
constexpr uint32_t BODY_UNLIMITED = 0xFFFFFFFFu;
// ngx_http_realip_module (set_real_ip_from / real_ip_header / real_ip_recursive,
// version1/nginx.ingress.tmpl:46-49, version2/nginx.virtualserver.tmpl:64-72, ConfigMap keys
// configmaps.go:153-169): the header the client address is taken from, and the trusted proxies
// RIP_PROXY: real_ip_header proxy_protocol (the record's paddr, from the PROXY header);
// RIP_UNKNOWN: a set_real_ip_from value that is not an address (nginx resolves host names)
enum : uint32_t { RIP_XREALIP = 1, RIP_XFWD = 2, RIP_PROXY = 3, RIP_HEADER = 4, RIP_UNKNOWN = 5 };
struct DRealIp {
    uint32_t type;           // RIP_*
    uint32_t recursive;      // real_ip_recursive on
    uint32_t first_cidr, n_cidr;   // DCidr list (set_real_ip_from, config order)
    uint32_t hdr_off, hdr_len;     // RIP_HEADER: the lowercased header name (bytes pool)
    uint32_t pad[2];
};
struct DCidr {
    uint32_t family;         // 4 or 6
    uint32_t addr[4];        // network-order bytes, packed little-endian per dword (masked)
    uint32_t mask[4];
    uint32_t pad[3];
};
// A server whose location names all fit 16 bytes and whose trie has at most SMALL_LOCS_MAX
// nodes carrying a location gets those nodes as a flat list: the route compares the URI's
// first 16 bytes (registers) with every entry -- independent loads instead of one dependent
// edge probe per URI byte.  Same answers as the trie walk (exact, longest prefix, auto_redirect).
constexpr uint32_t SMALL_LOCS_MAX = 8;
struct DSmallLoc {
    uint32_t path[4];        // name bytes, zero padded
    uint32_t len;
    int32_t prefix_loc, exact_loc, ar_loc;   // as DNode
};
// A server with more regex locations than this evaluates them behind a factor prefilter: every
// match of regex k contains one of its factors, so k is a candidate only if one of its key
// windows (a folded 4-byte window of a factor) occurs in the URI.  Candidates run in config
// order, merged with the always list; the first match wins (ngx_http_core_find_location).
constexpr uint32_t RLOC_SEQ_MAX = 8;
struct DRlocKey { uint32_t key; uint32_t first, count; uint32_t server; };   // key 0 = empty slot; DRlocEnt slice
// one keyed regex: the folded factor whose window the key is, checked in full at the window
// before the regex becomes a candidate
// bit filter over the prefilter keys, staged into LDS by k_route: a URI window whose bit is
// clear skips the key-table probe in L2
constexpr uint32_t RK_BLOOM_WORDS = 1024;
__host__ __device__ inline uint32_t rk_bloom_bit(uint32_t h) { return h >> 17; }   // 15 bits
struct DRlocEnt { uint32_t k; uint32_t fac_off; uint16_t fac_len; int16_t key_off; };
struct DServerIf {
    uint32_t op;             // SIF_*
    uint32_t src;            // DSrc index (variable), unused for SIF_RETURN
    uint32_t val_off, val_len;  // literal (case-sensitive compare, ngx_http_script_equal_code)
    uint32_t code;           // return code
    uint32_t tt;             // SIF_FLAGS truth table
    uint32_t pad[2];
};
struct DRegexLoc { uint32_t dfa; uint32_t loc; };

// ---- location trie ---------------------------------------------------------------------
struct DNode {
    int32_t prefix_loc;      // prefix / ^~ location whose name ends here, -1 none
    int32_t exact_loc;       // `location = ...` ending here
    int32_t ar_loc;          // auto_redirect target: location named <this>/ (only if nothing ends here)
    uint32_t pad;
};
// key = node*256 + byte + 1 (0 = empty); child_prefix = the child's prefix_loc, so the walk reads
// one 16-byte edge per URI byte instead of an edge and then the child node
struct DEdge { uint32_t key; uint32_t child; int32_t child_prefix; uint32_t pad; };

// ---- locations -------------------------------------------------------------------------
enum : uint8_t { LK_PROXY = 0, LK_RETURN = 1, LK_IRL_SPLIT = 2, LK_IRL_RULES = 3, LK_UNSUPPORTED = 4,
                 LK_NONE = 5, LK_IRL_EMPTY = 6, LK_STATUS = 7 /* stub_status: a 200 content handler */ };
struct DLoc {
    uint8_t  kind;           // LK_*
    uint8_t  noregex;        // ^~
    uint8_t  waf_mode;
    uint8_t  is_named;
    uint32_t upstream;       // GM_NONE if not a known upstream
    uint32_t ret_code;
    uint32_t route;          // DSplit / DRules index for IRLs
    uint32_t body_max;       // client_max_body_size in effect here (BODY_UNLIMITED: none, or a
                             // location whose own identity is uncertain: nested / PCRE-only)
    uint32_t access;         // DAccList of the allow / deny rules in effect here, GM_NONE: none
};
// ngx_http_access_module (nginx 1.17.3) rules in effect at a location -- its own, else its
// server's, else the http block's (ngx_http_access_merge_loc_conf): the IPv4 list (IPv4 and `all`
// rules, config order: alcf->rules) and the IPv6 list (IPv6 and `all`: alcf->rules6).  A rule is
// a DCidr (family 0 for `all`: mask 0) and its verdict.
struct DAccRule { DCidr c; uint32_t deny; uint32_t pad[2]; };
struct DAccList { uint32_t first4, n4, first6, n6; };

// The upstream request URI of a proxying location (§8 f1, nginx.org/rewrites: the URI part of
// proxy_pass, annotations.go:347-361, version1/nginx.ingress.tmpl:194-196), indexed like DLoc.
enum : uint32_t { LOCURI_REWRITE = 1, LOCURI_DEFER = 2 };
// flags bits 8..11: the request parsers (Wallarm's, §8 f4) the location runs before the WAF
// stages -- the signature set's "@decoders" minus wallarm_parser_disable
constexpr uint32_t LOCURI_DEC_SHIFT = 8;
enum : uint32_t { DEC_PERCENT = 1, DEC_URLENC = 2, DEC_JSON = 4, DEC_BASE64 = 8 };
struct DLocUri {
    uint32_t off, len;       // the URI part (bytes pool)
    uint32_t loc_len;        // the location's prefix length: $uri[loc_len:] follows the URI part
    uint32_t flags;          // 0: the request's own $request_uri goes upstream unchanged
};

// ---- request variables ---------------------------------------------------------------
enum : uint8_t { SRC_HTTP = 1, SRC_COOKIE = 2, SRC_ARG = 3, SRC_VAR = 4 };
enum : uint8_t { V_SCHEME = 1, V_HTTPS, V_HTTP2, V_METHOD, V_ARGS, V_URI, V_REQUEST_URI, V_REQUEST,
                 V_REQUEST_BODY, V_REMOTE_ADDR, V_REMOTE_PORT, V_SERVER_PORT, V_REQUEST_ID, V_HOST };
struct DSrc {
    uint8_t  kind;           // SRC_*
    uint8_t  var;            // V_* for SRC_VAR
    uint8_t  join;           // $http_cookie -> ';', $http_x_forwarded_for -> ','
    uint8_t  pad;
    uint32_t name_off, name_len;   // lowercase header name with '_' / cookie / arg name
};

// ---- rules routes (compiled map chains) ----------------------------------------------
// A condition node evaluates one map: value(src) vs one key (lowercase literal, or a DFA on
// the raw value that is only run for a non-empty value, ngx_http_map_find), then branches.
// next_* >= 0: another node; NEXT_0 / NEXT_1: the chain's constant result.
enum : int32_t { NEXT_0 = -1, NEXT_1 = -2 };
struct DCond {
    uint32_t src;            // DSrc index
    uint32_t is_regex;
    uint32_t key_off, key_len;   // literal (lowercased)
    uint32_t dfa;
    int32_t  next_true, next_false;
    uint32_t pad;
};
// a rules map of <= RULES_TABLE_MAX chains is a 2^n truth table; up to RULES_CHAINS_MAX its
// params are conditions over the chains' '0'/'1' string (table_off = GM_NONE, pad[0]: first DCond)
constexpr uint32_t RULES_TABLE_MAX = 8, RULES_CHAINS_MAX = 32;
struct DRules {
    uint32_t first_chain, n_chains;  // chain head node ids in DChainHead[]
    uint32_t table_off;              // 2^n_chains entries (uint8 result index, 0xFF = default)
    uint32_t first_target, n_targets;// n_targets = #params (result index -> named location)
    uint32_t default_target;         // named location id, GM_NONE -> empty (302)
    uint32_t pad[2];
};
struct DSplit {
    uint32_t first_part, n_parts;    // DPart
    uint32_t src;                    // DSrc (normally $request_id)
    uint32_t pad;
};
struct DPart { uint32_t bound; uint32_t star; uint32_t target; uint32_t pad; };  // target GM_NONE -> empty

// ---- DFAs (regex) ----------------------------------------------------------------------
enum : uint32_t { DFA_ANCHOR_START = 1, DFA_ANCHOR_END = 2 };
// dfa_trans entry = target state | accept flags of the target << 14 (states < 16384: the regex
// compiler caps DFAs at 8192 states)
constexpr uint32_t DFA_TRANS_STATE_MASK = 0x3FFFu;
struct DDfa {
    uint32_t trans_off;      // uint16 [n_states][n_classes] into dfa_trans; state 0 = dead, 1 = start
    uint32_t acc_off;        // uint8 [n_states] accept flags into dfa_acc
    uint32_t cls_off;        // uint8 [256] byte -> class into dfa_cls
    uint16_t n_states, n_classes;
    uint32_t flags;          // DFA_ANCHOR_*
    uint32_t pad[3];
};

// ---- WAF signatures ----------------------------------------------------------------------
// WAF prefilter: a blocked Bloom filter of the folded 4-byte key windows (one window per
// literal), resident in LDS for the whole scan -- 2^BLOOM_LOG2 32-bit blocks = 128 KiB, one
// 1024-thread workgroup per CU.  Every arena offset is probed: one ds_read_b32 and pk
// packed 16-bit shifts (2 bits each) per byte position.
constexpr int BLOOM_LOG2 = 15;
constexpr int BLOOM_PK_DEFAULT = 4;  // BLOOM_PK_PERM: K = 4 bits, one per byte (else K = 2 * pk, pk = 1..3)
constexpr uint32_t BLOOM_PK_PERM = 4;
constexpr uint32_t BLOOM_WORDS = 1u << BLOOM_LOG2;
constexpr uint32_t SCAN_LDS_BYTES = 4u * BLOOM_WORDS;
constexpr int CAND_SHARDS = 64;      // candidate-list shards (one atomic tail per shard)
constexpr int BLK_SHIFT = 10;        // arena block (1 KiB) -> first record index (blk2rec)

enum : uint8_t { LIT_NOCASE = 1, LIT_TRIGGER = 2, LIT_PREFIX = 4 };
struct DLitBucket { uint32_t key; uint32_t first; uint32_t count; uint32_t pad; };  // key = folded 4-gram + 1? see kWafEmpty
struct DLit {
    uint32_t id;             // signature rule id (LIT) or regex index (TRIGGER)
    uint32_t bytes_off;      // pattern bytes (folded if NOCASE)
    uint16_t len;
    uint8_t  flags;          // LIT_*
    uint8_t  zones;          // bit0 uri, bit1 args, bit2 hdrs, bit3 body
    int16_t  key_off;        // offset of the 4-byte key window inside the pattern; -1 = the window
                             // starts one byte before the pattern (4-byte patterns, gm_compile.cpp)
    uint16_t dfa_entry;      // LIT_PREFIX: the anchored DFA's state after the whole literal, with
                             // its accept flags in bits 14-15 (a transition entry), so the run
                             // starts after the literal; 0 = run from the start state
};
// k_waf_exact's first test of a literal at a key hit, before any pattern byte is read: the folded
// pattern bytes in the 4 arena bytes before (b) and after (a) the key window, each with the mask
// of the bytes that lie inside the pattern (parallel to the DLit array)
struct DLitChk { uint32_t b, bmask, a, amask; };
enum : uint32_t { RXM_TRIGGER = 0, RXM_ALWAYS = 1, RXM_PREFIX = 2 };
struct DSigRegex {
    uint32_t dfa;            // search DFA (whole zone)
    uint32_t adfa;           // anchored DFA (RXM_PREFIX: run from each prefix occurrence)
    uint32_t rule;           // signature rule id
    uint16_t zones;
    uint16_t mode;           // RXM_*: TRIGGER = factor hit -> zone job; ALWAYS = no >= 4-byte
                             // factor, every request; PREFIX = verified inline in k_waf_verify
};

// ---- upstream peer selection ---------------------------------------------
// One DUpstream per entry of the sorted upstream-name table (the verdict's upstream_id), its
// `server` lines as peers [first_peer, first_peer + n_peers) in config order (global peer ids).
// Methods follow the upstream block the templates render (version1/nginx.ingress.tmpl:2-8,
// version2/nginx.virtualserver.tmpl:2-10) from LBMethod (config_params.go:123, ParseLBMethod
// parsing_helpers.go:89-161).  UM_DEFER: a construct the engine does not model (weights, backup,
// max_conns, Plus-only methods, hash keys over unsupported variables) -- the data plane asks nginx.
enum : uint32_t { UM_RR = 0, UM_LEAST_CONN = 1, UM_IP_HASH = 2, UM_HASH = 3, UM_CHASH = 4, UM_RANDOM = 5,
                  UM_RANDOM2 = 6, UM_DEFER = 7 };
struct DUpstream {
    uint32_t first_peer, n_peers;
    uint32_t method;         // UM_*
    uint32_t first_part, n_parts;    // hash key: DKeyPart list (literal text and variables)
    uint32_t first_point, n_points;  // UM_CHASH: sorted, de-duplicated DPoint ring
    uint32_t sticky;         // NGINX Plus `sticky cookie <name>`: 1 + the DSrc index of $cookie_<name>; 0 none
};
constexpr uint32_t KEY_PART_VAR = 0xFFFFFFFFu;
struct DKeyPart { uint32_t off; uint32_t len; };   // len KEY_PART_VAR: off = DSrc index
struct DPoint { uint32_t hash; uint32_t peer; };    // peer: index within the upstream
// the sequential methods (RR, least_conn) hold an upstream's peer state in LDS on the device
constexpr uint32_t SEQ_PEERS_MAX = 1024;

// nginx ngx_crc32 (CRC-32/IEEE, reflected 0xEDB88320): hash keys and the consistent-hash ring
struct Crc32Table { uint32_t t[256]; };
constexpr Crc32Table make_crc32_table() {
    Crc32Table r{};
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        r.t[i] = c;
    }
    return r;
}
// $request_id-keyed draw j for `random` / `random two` (nginx draws ngx_random(); the engine
// draws reproducibly from the request's own random id): splitmix64 finaliser
__host__ __device__ inline uint32_t peer_draw(uint64_t lo, uint64_t hi, uint32_t j) {
    uint64_t x = lo ^ (hi * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(j + 1) * 0xD1B54A32D192ED03ull);
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return (uint32_t)(x >> 32);
}

// Always-run signature regexes (RXM_ALWAYS, no >= 4-byte factor): grouped into union DFAs
// (gm_regex.hpp MultiDfa, <= ALW_GROUP_MAX regexes and ALW_GROUP_BYTES of rows a group), so one
// pass over a zone answers a whole group.  Groups are packed into slices of <= ALW_SLICE_GROUPS
// groups that fit ALWAYS_LDS_BYTES together; k_waf_always_multi stages one slice in LDS and runs a
// transition chain per group of the slice.
// Slice pack (16-B aligned): the shared dead row (ALW_DEAD_BYTES of zeros at offset 0) | clsa
// u8[257 * NGB] (NGB = 4 for up to four groups, else 8; entry b * NGB + j = 2 x byte b's class in
// group j: the byte offset of b's column within a row of group j, so the class columns of a byte
// for every group of the slice are one 4- or 8-byte LDS read, and the read's lanes spread over the
// banks as the bytes do -- a 16-byte entry per byte took ~9 LDS cycles per wave-byte on C4 stress
// text against ~4 for these; entry 256 the identity columns) | per group, its rows.  A row (state)
// is Cp + 4 u16: the transitions of the C classes, the identity column (the row's own value),
// padded to Cp = alw_row_cols(C), then the state's emit mask and end mask (u32 each).  A
// transition, and a chain's row, is the target row's byte offset IN THE SLICE / 4 (rows are 4-byte
// aligned; u16 reaches 256 KiB): a step is one shift-add (row << 2) + column and one u16 read, with
// no per-group base, and the value 0 -- the dead state of every group -- reads the shared dead row.
// The emitting states are numbered last, from row emit_row on: a chain entered one within a chunk
// iff the largest row it took there is >= emit_row (one max per step, no flag bit to strip).
constexpr uint32_t ALWAYS_LDS_BYTES = 160 * 1024;
constexpr uint32_t ALW_GROUP_BYTES = 64 * 1024 - 64;
constexpr uint32_t ALW_GROUP_MAX = 32;
constexpr uint32_t ALW_CLASSES_MAX = 127;   // (2 x the identity class fits the u8 column)
// the shared dead row: zeros over every group's columns and masks (2 x 128 + 8 bytes)
constexpr uint32_t ALW_DEAD_BYTES = 272;
__host__ __device__ constexpr uint32_t alw_cls_ngb(uint32_t n_groups) { return n_groups <= 4 ? 4u : 8u; }
// entries 0..255: the bytes; entry 256: every group's identity column (a row's own value: a step
// that changes nothing, for the bytes past a chunk's end)
constexpr uint32_t ALW_CLS_IDENTITY = 256;
__host__ __device__ constexpr uint32_t alw_cls_bytes(uint32_t n_groups) {
    return ALW_DEAD_BYTES + ((257u * alw_cls_ngb(n_groups) + 15u) & ~15u);
}
// a group's row: its classes, the identity column (class n_classes), padded to even, then the emit
// and end masks (u32 each)
__host__ __device__ constexpr uint32_t alw_row_cols(uint32_t n_classes) { return (n_classes + 2) & ~1u; }
#ifndef GM_ALW_SLICE_GROUPS
#define GM_ALW_SLICE_GROUPS 8
#endif
constexpr uint32_t ALW_SLICE_GROUPS = GM_ALW_SLICE_GROUPS;
constexpr uint32_t ALW_BUILD_STATES = 8192;   // product states before minimisation
struct DAlwGroup {
    uint32_t tr_off;         // byte offset of the group's rows from the slice start
    uint32_t mask_off;       // byte offset of the emit mask within a row (2 Cp); the end mask follows
    uint32_t start_row;      // the start state's row (its byte offset in the slice / 4)
    uint32_t n_classes, n_states;
    uint32_t zone_mask[4];   // members (bit k) that scan zone z
    uint32_t first;          // member k: a location slice's value alw_rule[first + k]; an always-run
                             // group's rule list alw_rl[alw_rule[first + k] .. alw_rule[first + k + 1])
    uint32_t zones;          // zones some member scans
    uint32_t emit_row;       // the first emitting state's row (slice offset / 4; rows past it emit too)
};
struct DAlwSlice {
    uint32_t off, len;       // bytes of the pack
    uint32_t first_group, n_groups;
    uint32_t zones;          // zones some group scans
    uint32_t server;         // regex-location slices: the server (GM_NONE: always-run regexes)
    uint32_t min_member;     // regex-location slices: the lowest regex-location index it holds
    uint32_t flags;          // ALW_SLICE_REVERSED: X$ regexes run backwards (compile_regex_reversed)
};
constexpr uint32_t ALW_SLICE_REVERSED = 1;
// a forward slice of unanchored regexes that all have factors: it runs only for requests whose
// k_rloc_pref mask has bit (flags >> 8) & 63
constexpr uint32_t ALW_SLICE_PREF = 2;
// an anchored regex-location slice with a head map (flags >> 16: its slot in rsl_heads): bit
// rsl_head_key(b0, b1, b2) is set if a member can match a $uri whose first three bytes are b0 b1
// b2 (0: no byte -- a shorter $uri); k_rloc_heads lists each slice's candidate requests, the slice
// runs only those
constexpr uint32_t ALW_SLICE_HEADS = 4;
constexpr uint32_t RSL_HEAD_WORDS = 65536 / 32;
// the key of a $uri's first three bytes in a head map: the second and third bytes, XOR-ed with a
// hash of the first (nearly always '/': a $uri's first byte says little)
__host__ __device__ constexpr uint32_t rsl_head_key(uint32_t b0, uint32_t b1, uint32_t b2) {
    return ((b1 << 8) | b2) ^ ((b0 * 0x9E37u) & 0xFFFFu);
}
constexpr uint32_t RSL_HEAD_PAIRS = 4096;   // live two-byte starts past which a head map is full
constexpr uint32_t RSL_HEADS_MAX = 64;

struct TabHeader {
    uint32_t magic, version;
    uint32_t n_ports, n_names_cap, n_wild_head_cap, n_wild_tail_cap;
    uint32_t n_servers, n_server_ifs, n_rlocs, n_nodes, n_edges_cap, n_locs;
    uint32_t n_srcs, n_conds, n_chain_heads, n_rules, n_splits, n_parts, n_dfas;
    uint32_t n_lit_buckets_cap, n_lits, n_sig_regex, n_always, n_sigs;
    uint64_t off_ports, off_names, off_wild_head, off_wild_tail, off_servers, off_server_ifs, off_rlocs,
             off_nodes, off_edges, off_locs, off_srcs, off_conds, off_chain_heads, off_rules, off_rtab,
             off_rtargets, off_splits, off_parts, off_dfas, off_dfa_trans, off_dfa_acc, off_dfa_cls,
             off_bytes, off_waf_a, off_waf_b, off_lit_buckets, off_lits, off_sig_regex, off_always;
    uint64_t total;
    uint32_t bloom_log2;     // BLOOM_LOG2 the image was built for
    uint32_t bloom_mul;      // Bloom hash multiplier (chosen per generation, see gm_compile.cpp)
    uint32_t bloom_pk;       // probe kind: BLOOM_PK_PERM (4 bits, one per byte) or pk packed shifts (K = 2 pk)
    uint32_t ctx_mul;        // stage-2 context filter multiplier (waf_b, see ctx_key)
    uint32_t n_rk_cap, n_rk_ids;   // regex-location prefilter: key table (pow2) and id lists
    uint32_t n_rk_ents_keys, pad_rk;   // distinct (server, key) pairs
    uint64_t off_rk, off_rk_ids;
    uint64_t off_small;            // DSmallLoc lists
    uint64_t off_rk_ents;          // DRlocEnt lists
    uint64_t off_rk_bloom;         // RK_BLOOM_WORDS: one bit per (server, key), top bits of rk_hash
    uint64_t off_name_bytes;       // server-name strings (DName.name_off), 64 B of slack
    uint64_t off_hot_end;          // [off_ports, off_hot_end): the route's hot tables, contiguous
    uint32_t n_ups, n_peers, n_key_parts, n_points;
    uint64_t off_ups, off_key_parts, off_points, off_peer_init;   // peer_init: u32 GM_PEER_DOWN per peer
    uint64_t off_peer_md5;   // 16-byte MD5 of each peer's address text ("ip:port"): NGINX Plus sticky cookie
    uint64_t off_loc_uri;          // DLocUri per location
    uint32_t decoders, pad_dec;    // the signature set's request parsers (DEC_*)
    uint32_t n_always_lds;         // always[0, n_always_lds) are in union-DFA groups
    uint32_t n_alw_groups, n_alw_slices, alw_pack_len, n_rsl;   // n_rsl: regex-location slices
                                                                 // after the n_alw_slices
    uint32_t n_rk_prefilter, pad_rkp;   // rk_on servers left to the factor prefilter (rsl_n 0)
    uint64_t off_alw, off_alw_slices, off_alw_pack, off_alw_rule;
    uint64_t off_rsl_pbit;         // u8 per regex location: its prefiltered slice's mask bit (0xFF none)
    uint64_t off_rsl_heads;        // anchored regex-location slices: a 65536-bit head map each (RSL_HEAD_WORDS u32)
    uint64_t off_rsl_head_slice;   // and each map's slice index (u32)
    uint32_t n_rsl_heads, pad_heads;
    uint32_t n_rk_ents_n, pad_rke; // DRlocEnt entries (k_rloc_pref stages them in LDS)
    uint32_t n_realip, n_cidrs;    // realip configurations and their set_real_ip_from entries
    uint64_t off_realip, off_cidrs;
    uint64_t off_alw_rl;           // always-run members' rule lists (zones << 24 | rule)
    uint64_t off_lit_chk;          // DLitChk per DLit
    uint32_t n_wild, pad_wild;     // wildcard server names (both tables)
    uint32_t n_acc_rules, n_acc_lists;   // allow / deny rules and the lists locations point at
    uint64_t off_acc_rules, off_acc_lists;
};
// The route's hot tables -- ports, the three name tables, servers, server ifs, small-location
// lists, locations and the name strings -- are laid out first and contiguously in the image;
// k_route copies them into LDS when they fit ROUTE_STAGE_BYTES (small configs: the cafe Ingress,
// VirtualServers), so its per-request chain of dependent table reads hits LDS, not L2.
constexpr uint32_t ROUTE_STAGE_BYTES = 8192;

struct GTab {                // device pointers, built on host from the image base
    const DPort *ports; const DName *names; const DName *wild_head; const DName *wild_tail;
    const DServer *servers; const DServerIf *server_ifs; const DRegexLoc *rlocs;
    const DNode *nodes; const DEdge *edges; const DLoc *locs;
    const DSrc *srcs; const DCond *conds; const uint32_t *chain_heads; const DRules *rules;
    const uint8_t *rtab; const uint32_t *rtargets; const DSplit *splits; const DPart *parts;
    const DDfa *dfas; const uint16_t *dfa_trans; const uint8_t *dfa_acc; const uint8_t *dfa_cls;
    const uint8_t *bytes; const uint32_t *waf_a; const uint32_t *waf_b;
    const DLitBucket *lit_buckets; const DLit *lits; const DSigRegex *sig_regex; const uint32_t *always;
    const DRlocKey *rk; const uint32_t *rk_ids; uint32_t rk_mask; const DSmallLoc *small; const DRlocEnt *rk_ents;
    const uint32_t *rk_bloom; uint32_t rk_keys;
    const uint8_t *name_bytes;
    const uint8_t *hot_base; uint32_t hot_len;   // the hot prefix (hot_len 0: larger than ROUTE_STAGE_BYTES)
    const DUpstream *ups; const DKeyPart *key_parts; const DPoint *points; const uint32_t *peer_init;
    const uint32_t *peer_md5;   // 4 words per peer (off_peer_md5)
    uint32_t n_ups, n_peers, n_servers;
    const DLocUri *loc_uri;
    uint32_t decoders;
    const DAlwGroup *alw; const DAlwSlice *alw_slices; const uint8_t *alw_pack; const uint32_t *alw_rule;
    const uint8_t *rsl_pbit;
    const uint32_t *rsl_heads; uint32_t n_rsl_heads; const uint32_t *rsl_head_slice;
    const DRealIp *realip; const DCidr *cidrs;
    const DAccRule *acc_rules; const DAccList *acc_lists;
    const uint32_t *alw_rl;
    const DLitChk *lit_chk;
    uint32_t n_always_lds, n_alw_groups, n_alw_slices, n_rsl, n_rk_prefilter;
    uint32_t n_ports, names_mask, wild_head_mask, wild_tail_mask, edges_mask, lit_mask;
    uint32_t n_wild;             // wildcard server names (0: k_route skips the wildcard step)
    uint32_t n_locs, n_sigs, n_sig_regex, n_always, n_lits, bloom_log2, bloom_mul, bloom_pk, ctx_mul;
    uint32_t gen;
    // this struct's copy in device memory: a kernel hands *self (not its kernel argument) to
    // out-of-line device functions, so the ~600-byte argument is not copied to scratch
    const GTab *self;
};

// hashing shared by compiler and kernels
// server-name hash: 4-byte little-endian words of the lowercased name (the last one zero padded),
// so the device hashes a host held in registers a word per step (SWAR), not a byte per step
__host__ __device__ inline uint32_t name_hash_word(uint32_t h, uint32_t w) {
    h ^= w; h *= 0x9E3779B1u; return h ^ (h >> 15);
}
__host__ __device__ inline uint32_t name_hash_init(uint32_t len) { return 2166136261u ^ (len * 0x85EBCA77u); }
__host__ __device__ inline uint32_t name_hash_fin(uint32_t h, uint32_t port_idx) {
    h ^= port_idx * 0x9E3779B9u; h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13;
    return h | 1u;           // never 0 (0 marks an empty slot)
}
__host__ __device__ inline uint32_t edge_hash(uint32_t key) {
    uint32_t h = key * 0x9E3779B1u; return h ^ (h >> 15);
}
// Bloom probe of a folded 4-gram w: p = w * mul (32x32 -> 64 bit).  Block = top BLOOM_LOG2 bits
// of the low word (multiplicative hashing keeps the TOP bits); the bit positions come from the
// high word, whose bits all depend on every input bit: pk packed shifts 1 << (hi >> 4q),
// each setting one bit in each 16-bit half (v_pk_lshlrev_b16: bits [0..3] and [16..19]).
struct BloomProbe { uint32_t block, mask; };
__host__ __device__ inline uint32_t pk_bits(uint32_t x) {
    return (1u << (x & 15)) | (1u << (16 + ((x >> 16) & 15)));
}
// BLOOM_PK_PERM: one bit in each byte of the block, at bit (hi >> 8k) & 7 of byte k -- on the
// device one v_and_b32 and one v_perm_b32 that reads the byte table {1, 2, 4, ..., 128}
// (0x80402010'08040201) with those four selectors: 2 VALU ops for 4 bits (pk_bits: 3 ops).
__host__ __device__ inline uint32_t perm_bits(uint32_t hi) {
    uint32_t m = 0;
    for (uint32_t k = 0; k < 4; k++) m |= 1u << (8 * k + ((hi >> (8 * k)) & 7));
    return m;
}
__host__ __device__ inline BloomProbe bloom_probe(uint32_t w, uint32_t mul, uint32_t pk) {
    const uint64_t p = (uint64_t)w * mul;
    const uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
    uint32_t m = 0;
    if (pk == BLOOM_PK_PERM) m = perm_bits(hi);
    else for (uint32_t q = 0; q < pk; q++) m |= pk_bits(hi >> (4 * q));
    return BloomProbe{lo >> (32 - BLOOM_LOG2), m};
}
// The scan filter's probe (waf_a, k_waf_scan).  Measured, not kept: the block from bits 2 .. 16
// of hi (its LDS byte address one v_and, 8 fewer VALU ops per KiB chunk) with the bit positions
// from hi ^ lo -- 15 % more scan candidates, C4 step 4.79 vs 4.65 ms; and K = 8 bits as two per
// byte (perm_bits of hi and of hi rotated by 3): as many candidates as K = 4 (most are windows
// that are keys, not filter collisions).
__host__ __device__ inline BloomProbe scan_probe(uint32_t w, uint32_t mul, uint32_t pk) {
    return bloom_probe(w, mul, pk);
}
// Stage-2 context filter (waf_b, same size as the scan Bloom filter; staged into LDS by
// k_waf_ctx).  A scan candidate window w at arena offset p survives only if waf_b holds w
// together with the folded bytes around it that its pattern fixes: up to two on the left
// (l2 = A[p-2] | A[p-1] << 8) and two on the right (r2 = A[p+4] | A[p+5] << 8).  Each key entry
// inserts one shape (nl, nr = context bytes used on each side): the bytes its pattern has,
// canonicalised to one of the CTX_SHAPES shapes (ctx_canon); a window is probed with all of
// them.  Bytes outside the arena read as the fold of 0 (0x20).
constexpr uint32_t CTX_PK = 3;
constexpr uint32_t CTX_MUL_DEFAULT = 0x7FEB352Du;
__host__ __device__ inline uint32_t ctx_lmask(uint32_t nl) { return nl == 0 ? 0u : nl == 1 ? 0xFF00u : 0xFFFFu; }
__host__ __device__ inline uint32_t ctx_rmask(uint32_t nr) { return nr == 0 ? 0u : nr == 1 ? 0x00FFu : 0xFFFFu; }
// the probed shapes, as nl * 3 + nr: (2,2) (1,1) (1,0) (0,1) (0,0)
constexpr int CTX_SHAPES = 5;
__host__ __device__ inline uint32_t ctx_shape_nl(int i) { return i == 0 ? 2u : i <= 2 ? 1u : 0u; }
__host__ __device__ inline uint32_t ctx_shape_nr(int i) { return i == 0 ? 2u : (i == 1 || i == 3) ? 1u : 0u; }
// the largest probed shape within the context (nl, nr) a pattern has
__host__ __device__ inline void ctx_canon(uint32_t &nl, uint32_t &nr) {
    if (nl == 2 && nr == 2) return;
    if (nl >= 1 && nr >= 1) { nl = nr = 1; return; }
    nl = nl ? 1u : 0u; nr = nr ? 1u : 0u;
}
__host__ __device__ inline uint32_t ctx_key(uint32_t w, uint32_t l2, uint32_t r2, uint32_t shape) {
    uint32_t c = (l2 * 0x9E3779B1u) ^ (r2 * 0x85EBCA77u) ^ ((shape + 1u) * 0xC2B2AE3Du);
    c ^= c >> 15;
    return w ^ c;
}
__host__ __device__ inline uint32_t lit_bucket_hash(uint32_t w) { uint32_t h = w * 0xC2B2AE3Du; return h ^ (h >> 16); }
__host__ __device__ inline uint32_t rk_hash(uint32_t w, uint32_t server) { return lit_bucket_hash(w ^ (server * 0x9E3779B9u)); }
// Prefilter fold: OR 0x20 into every byte.  Maps A-Z onto a-z (so case-insensitive keys match)
// and merges a few other byte pairs (0x40/0x60, 0x00-0x1F/0x20-0x3F, ...); the merge only adds
// prefilter candidates -- k_waf_verify compares the literal bytes exactly (lc() for nocase).
__host__ __device__ inline uint32_t fold4(uint32_t w) { return w | 0x20202020u; }
// exact ASCII lowercase (A-Z only) of four packed bytes, SWAR
__host__ __device__ inline uint32_t lower4(uint32_t w) {
    const uint32_t x = w & 0x7F7F7F7Fu;
    const uint32_t ge_a = (x + 0x3F3F3F3Fu) & 0x80808080u;   // byte >= 'A'
    const uint32_t gt_z = (x + 0x25252525u) & 0x80808080u;   // byte >  'Z'
    return w | ((ge_a & ~gt_z & ~w & 0x80808080u) >> 2);
}

}  // namespace gm
