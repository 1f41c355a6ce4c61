// gm_regex.cpp -- regex (RE2-compatible subset, PCRE 8.x semantics) -> byte-class DFA + factors.
// See gm_regex.hpp for the supported language.
#include "gm_regex.hpp"

#include <algorithm>
#include <cstring>
#include <bitset>
#include <map>
#include <unordered_map>

namespace gm {
namespace {

using CSet = std::bitset<256>;

struct Node {
    enum K { EMPTY, SET, CAT, ALT, REP, BOL, EOL } k = EMPTY;
    CSet set;
    std::vector<int> kids;
    int mn = 0, mx = 0;  // REP: mx < 0 = unbounded
};

struct Parser {
    const std::string &p;
    size_t i = 0;
    bool icase = false, dotall = false;
    RegexStatus st = RX_OK;
    std::string err;
    std::vector<Node> nodes;

    explicit Parser(const std::string &s) : p(s) {}

    int add(Node n) { nodes.push_back(std::move(n)); return (int)nodes.size() - 1; }
    bool fail(RegexStatus s, const char *m) { if (st == RX_OK) { st = s; err = m; } return false; }
    bool eof() const { return i >= p.size(); }

    void fold(CSet &s) const {
        if (!icase) return;
        for (int c = 'a'; c <= 'z'; c++) {
            if (s[c] || s[c - 32]) { s[c] = true; s[c - 32] = true; }
        }
    }
    static CSet digit() { CSet s; for (int c = '0'; c <= '9'; c++) s[c] = true; return s; }
    static CSet word() {
        CSet s = digit();
        for (int c = 'a'; c <= 'z'; c++) { s[c] = true; s[c - 32] = true; }
        s['_'] = true; return s;
    }
    static CSet space() { CSet s; for (int c : {' ', '\t', '\n', '\v', '\f', '\r'}) s[c] = true; return s; }

    int hexv(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }

    // escape after '\\' (i points past the backslash). Returns true and fills `out`.
    bool escape(CSet &out, bool in_class) {
        if (eof()) return fail(RX_SYNTAX, "trailing backslash");
        char c = p[i++];
        out.reset();
        switch (c) {
        case 'd': out = digit(); return true;
        case 'D': out = ~digit(); return true;
        case 'w': out = word(); return true;
        case 'W': out = ~word(); return true;
        case 's': out = space(); return true;
        case 'S': out = ~space(); return true;
        case 't': out['\t'] = true; return true;
        case 'n': out['\n'] = true; return true;
        case 'r': out['\r'] = true; return true;
        case 'f': out['\f'] = true; return true;
        case 'e': out[0x1b] = true; return true;
        case 'a': out[0x07] = true; return true;
        case 'x': {
            int v = 0, n = 0;
            if (!eof() && p[i] == '{') return fail(RX_UNSUPPORTED, "\\x{...}");
            while (n < 2 && !eof() && hexv(p[i]) >= 0) { v = v * 16 + hexv(p[i++]); n++; }
            out[v] = true; return true;
        }
        case 'b':
            if (in_class) { out[0x08] = true; return true; }
            return fail(RX_UNSUPPORTED, "\\b word boundary");
        case '0': {
            int v = 0, n = 0;
            while (n < 2 && !eof() && p[i] >= '0' && p[i] <= '7') { v = v * 8 + (p[i++] - '0'); n++; }
            out[v & 0xff] = true; return true;
        }
        default: break;
        }
        if (c >= '1' && c <= '9') return fail(RX_PCRE_ONLY, "backreference");
        if (c == 'K') return fail(RX_PCRE_ONLY, "\\K");
        if (c == 'G' || c == 'R' || c == 'X' || c == 'C' || c == 'g' || c == 'k') return fail(RX_PCRE_ONLY, "PCRE escape");
        if (c == 'B' || c == 'A' || c == 'z' || c == 'Z') return fail(RX_UNSUPPORTED, "assertion escape");
        if (c == 'p' || c == 'P' || c == 'h' || c == 'H' || c == 'v' || c == 'V' || c == 'N' || c == 'Q' ||
            c == 'E' || c == 'c' || c == 'o' || c == 'u' || c == 'U' || c == 'l' || c == 'L')
            return fail(RX_UNSUPPORTED, "escape");
        if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) return fail(RX_UNSUPPORTED, "unknown escape");
        out[(unsigned char)c] = true;
        return true;
    }

    int parse_class() {   // after '['
        CSet s;
        bool neg = false;
        if (!eof() && p[i] == '^') { neg = true; i++; }
        bool first = true;
        for (;;) {
            if (eof()) { fail(RX_SYNTAX, "unterminated class"); return -1; }
            char c = p[i];
            if (c == ']' && !first) { i++; break; }
            first = false;
            if (c == '[' && i + 1 < p.size() && (p[i + 1] == ':' || p[i + 1] == '=' || p[i + 1] == '.')) {
                fail(RX_UNSUPPORTED, "POSIX class"); return -1;
            }
            CSet lo; int lo_ch = -1;
            i++;
            if (c == '\\') {
                if (!escape(lo, true)) return -1;
                if (lo.count() == 1) for (int k = 0; k < 256; k++) if (lo[k]) lo_ch = k;
            } else { lo[(unsigned char)c] = true; lo_ch = (unsigned char)c; }
            if (lo_ch >= 0 && i + 1 < p.size() && p[i] == '-' && p[i + 1] != ']') {
                i++;
                char d = p[i++]; int hi_ch;
                if (d == '\\') {
                    CSet h; if (!escape(h, true)) return -1;
                    if (h.count() != 1) { fail(RX_SYNTAX, "bad range"); return -1; }
                    hi_ch = 0; for (int k = 0; k < 256; k++) if (h[k]) hi_ch = k;
                } else hi_ch = (unsigned char)d;
                if (hi_ch < lo_ch) { fail(RX_SYNTAX, "range out of order"); return -1; }
                for (int k = lo_ch; k <= hi_ch; k++) s[k] = true;
            } else s |= lo;
        }
        fold(s);
        if (neg) s = ~s;   // PCRE: a negated class matches '\n' too
        Node n; n.k = Node::SET; n.set = s;
        return add(n);
    }

    int parse_atom() {
        char c = p[i];
        if (c == '(') {
            i++;
            if (!eof() && p[i] == '?') {
                i++;
                if (eof()) { fail(RX_SYNTAX, "bad group"); return -1; }
                char t = p[i];
                if (t == ':') i++;
                else if (t == 'P' || t == '<' || t == '\'') {
                    if (t == 'P') { i++; if (eof() || p[i] != '<') { fail(RX_PCRE_ONLY, "(?P"); return -1; } }
                    if (p[i] == '<' && i + 1 < p.size() && (p[i + 1] == '=' || p[i + 1] == '!')) {
                        fail(RX_PCRE_ONLY, "lookbehind"); return -1;
                    }
                    char close = p[i] == '\'' ? '\'' : '>';
                    while (!eof() && p[i] != close) i++;
                    if (eof()) { fail(RX_SYNTAX, "bad group name"); return -1; }
                    i++;
                } else if (t == '=' || t == '!' || t == '>' || t == '|' || t == '(' || t == 'R' ||
                           t == '&' || t == '#' || t == 'C' || (t >= '0' && t <= '9') || t == '+') {
                    fail(RX_PCRE_ONLY, "PCRE group construct"); return -1;
                } else { fail(RX_UNSUPPORTED, "inline flags inside pattern"); return -1; }
            }
            int r = parse_alt();
            if (r < 0) return -1;
            if (eof() || p[i] != ')') { fail(RX_SYNTAX, "missing )"); return -1; }
            i++;
            return r;
        }
        if (c == '[') { i++; return parse_class(); }
        if (c == '.') {
            i++; Node n; n.k = Node::SET; n.set.set(); if (!dotall) n.set['\n'] = false; return add(n);
        }
        if (c == '^') { i++; Node n; n.k = Node::BOL; return add(n); }
        if (c == '$') { i++; Node n; n.k = Node::EOL; return add(n); }
        if (c == '*' || c == '+' || c == '?') { fail(RX_SYNTAX, "nothing to repeat"); return -1; }
        i++;
        Node n; n.k = Node::SET;
        if (c == '\\') { if (!escape(n.set, false)) return -1; }
        else n.set[(unsigned char)c] = true;
        fold(n.set);
        return add(n);
    }

    bool quant(int &mn, int &mx) {   // at a possible quantifier; returns false if none
        if (eof()) return false;
        char c = p[i];
        if (c == '*') { i++; mn = 0; mx = -1; return true; }
        if (c == '+') { i++; mn = 1; mx = -1; return true; }
        if (c == '?') { i++; mn = 0; mx = 1; return true; }
        if (c == '{') {
            size_t j = i + 1; int a = 0, b = -1, da = 0, db = 0; bool comma = false;
            while (j < p.size() && isdigit((unsigned char)p[j])) { a = a * 10 + (p[j] - '0'); j++; da++; }
            if (j < p.size() && p[j] == ',') {
                comma = true; j++; b = 0;
                while (j < p.size() && isdigit((unsigned char)p[j])) { b = b * 10 + (p[j] - '0'); j++; db++; }
            }
            if (j >= p.size() || p[j] != '}' || da == 0) return false;   // literal '{'
            i = j + 1;
            mn = a; mx = comma ? (db ? b : -1) : a;
            if (mx >= 0 && mx < mn) { fail(RX_SYNTAX, "bad {n,m}"); return false; }
            if (mn > 1000 || mx > 1000) { fail(RX_TOO_BIG, "repeat count"); return false; }
            return true;
        }
        return false;
    }

    int parse_rep() {
        int a = parse_atom();
        if (a < 0) return -1;
        for (;;) {
            int mn, mx;
            if (!quant(mn, mx)) { if (st != RX_OK) return -1; return a; }
            if (nodes[a].k == Node::BOL || nodes[a].k == Node::EOL) { fail(RX_UNSUPPORTED, "quantified anchor"); return -1; }
            if (!eof() && p[i] == '+') { fail(RX_PCRE_ONLY, "possessive quantifier"); return -1; }
            if (!eof() && p[i] == '?') i++;   // lazy: same language
            Node n; n.k = Node::REP; n.kids = {a}; n.mn = mn; n.mx = mx;
            a = add(n);
            if (!eof() && (p[i] == '*' || p[i] == '+' || p[i] == '?')) { fail(RX_SYNTAX, "nothing to repeat"); return -1; }
        }
    }

    int parse_cat() {
        Node n; n.k = Node::CAT;
        while (!eof() && p[i] != '|' && p[i] != ')') {
            int r = parse_rep();
            if (r < 0) return -1;
            n.kids.push_back(r);
        }
        if (n.kids.empty()) { Node e; e.k = Node::EMPTY; return add(e); }
        if (n.kids.size() == 1) return n.kids[0];
        return add(n);
    }

    int parse_alt() {
        int a = parse_cat();
        if (a < 0) return -1;
        if (eof() || p[i] != '|') return a;
        Node n; n.k = Node::ALT; n.kids = {a};
        while (!eof() && p[i] == '|') {
            i++;
            int b = parse_cat();
            if (b < 0) return -1;
            n.kids.push_back(b);
        }
        return add(n);
    }

    int parse() {
        // leading inline flags (?i) (?s) (?is) ...
        while (i + 2 < p.size() && p[i] == '(' && p[i + 1] == '?') {
            size_t j = i + 2; bool ok = true, any = false; bool fi = icase, fs = dotall;
            while (j < p.size() && p[j] != ')') {
                if (p[j] == 'i') fi = true; else if (p[j] == 's') fs = true; else { ok = false; break; }
                j++; any = true;
            }
            if (!ok || !any || j >= p.size()) break;
            icase = fi; dotall = fs; i = j + 1;
        }
        int r = parse_alt();
        if (r >= 0 && !eof()) { fail(RX_SYNTAX, "unmatched )"); return -1; }
        return r;
    }
};

// anchors: ^ only in head position, $ only in tail position (else unsupported)
bool check_anchors(const std::vector<Node> &N, int n, bool head, bool tail) {
    const Node &x = N[n];
    switch (x.k) {
    case Node::BOL: return head;
    case Node::EOL: return tail;
    case Node::SET: case Node::EMPTY: return true;
    case Node::REP: return check_anchors(N, x.kids[0], false, false);
    case Node::ALT:
        for (int k : x.kids) if (!check_anchors(N, k, head, tail)) return false;
        return true;
    case Node::CAT: {
        // head position persists across leading anchors/empties
        size_t m = x.kids.size();
        for (size_t k = 0; k < m; k++) {
            bool h = head, t = tail;
            for (size_t q = 0; q < k; q++) { auto kk = N[x.kids[q]].k; if (kk != Node::BOL && kk != Node::EMPTY) h = false; }
            for (size_t q = k + 1; q < m; q++) { auto kk = N[x.kids[q]].k; if (kk != Node::EOL && kk != Node::EMPTY) t = false; }
            if (!check_anchors(N, x.kids[k], h, t)) return false;
        }
        return true;
    }
    }
    return true;
}

// ---------------------------------------------------------------- Thompson NFA
struct NS { enum T { SET, SPLIT, EPS, BOL, EOL, MATCH } t; int set; int out, out1; };

struct NfaBuilder {
    const std::vector<Node> &N;
    std::vector<NS> st;
    std::vector<CSet> sets;
    bool too_big = false;
    explicit NfaBuilder(const std::vector<Node> &n) : N(n) {}

    int mk(NS s) { st.push_back(s); if (st.size() > 200000) too_big = true; return (int)st.size() - 1; }
    struct Frag { int start; std::vector<int *> dummy; std::vector<std::pair<int, int>> outs; };  // (state, which)

    void patch(const std::vector<std::pair<int, int>> &outs, int to) {
        for (auto &o : outs) (o.second == 0 ? st[o.first].out : st[o.first].out1) = to;
    }

    Frag build(int n) {
        if (too_big) return Frag{mk({NS::EPS, -1, -1, -1}), {}, {}};
        const Node &x = N[n];
        switch (x.k) {
        case Node::EMPTY: { int s = mk({NS::EPS, -1, -1, -1}); return Frag{s, {}, {{s, 0}}}; }
        case Node::BOL: { int s = mk({NS::BOL, -1, -1, -1}); return Frag{s, {}, {{s, 0}}}; }
        case Node::EOL: { int s = mk({NS::EOL, -1, -1, -1}); return Frag{s, {}, {{s, 0}}}; }
        case Node::SET: {
            sets.push_back(x.set);
            int s = mk({NS::SET, (int)sets.size() - 1, -1, -1});
            return Frag{s, {}, {{s, 0}}};
        }
        case Node::CAT: {
            Frag f = build(x.kids[0]);
            for (size_t k = 1; k < x.kids.size(); k++) {
                Frag g = build(x.kids[k]);
                patch(f.outs, g.start);
                f.outs = g.outs;
            }
            return f;
        }
        case Node::ALT: {
            Frag f = build(x.kids[0]);
            for (size_t k = 1; k < x.kids.size(); k++) {
                Frag g = build(x.kids[k]);
                int s = mk({NS::SPLIT, -1, f.start, g.start});
                f.start = s;
                f.outs.insert(f.outs.end(), g.outs.begin(), g.outs.end());
            }
            return f;
        }
        case Node::REP: {
            int kid = x.kids[0];
            int mn = x.mn, mx = x.mx;
            int entry = mk({NS::EPS, -1, -1, -1});
            std::vector<std::pair<int, int>> outs = {{entry, 0}};
            for (int r = 0; r < mn; r++) {
                Frag g = build(kid);
                patch(outs, g.start); outs = g.outs;
            }
            if (mx < 0) {
                Frag g = build(kid);
                int sp = mk({NS::SPLIT, -1, g.start, -1});
                patch(outs, sp);
                patch(g.outs, sp);
                outs = {{sp, 1}};
            } else {
                std::vector<std::pair<int, int>> skips;
                for (int r = mn; r < mx; r++) {
                    Frag g = build(kid);
                    int sp = mk({NS::SPLIT, -1, g.start, -1});
                    patch(outs, sp);
                    skips.push_back({sp, 1});
                    outs = g.outs;
                }
                outs.insert(outs.end(), skips.begin(), skips.end());
            }
            return Frag{entry, {}, outs};
        }
        }
        return Frag{mk({NS::EPS, -1, -1, -1}), {}, {}};
    }
};

// ---------------------------------------------------------------- factors
// Follow set of a string set: the folded bytes that can come right after any of its strings
// (none = unknown).  The WAF scan probes only even offsets, and keys a 4-byte string at odd
// offsets through the windows one byte left or right of it (gm_compile.cpp choose_keys): with a
// known follow set the right-hand family has |follow| members instead of 128.
struct Follow { CSet set; bool ok = false; };
struct FI {
    bool exact_ok = false;
    std::vector<std::string> exact;
    std::vector<std::string> best;     // best OR-set found anywhere inside (empty = none)
    Follow best_follow;
    std::vector<std::string> prefix = {""};   // every match starts with one of these (folded)
    Follow prefix_follow;
};

bool small_set(const std::vector<std::string> &v) {
    if (v.size() > 16) return false;
    for (auto &s : v) if (s.size() > 32) return false;
    return true;
}
std::vector<std::string> cross(const std::vector<std::string> &a, const std::vector<std::string> &b) {
    std::vector<std::string> r;
    for (auto &x : a) for (auto &y : b) r.push_back(x + y);
    std::sort(r.begin(), r.end()); r.erase(std::unique(r.begin(), r.end()), r.end());
    return r;
}

int score_len(const std::vector<std::string> &s) {
    if (s.empty()) return -1;
    size_t m = SIZE_MAX;
    for (auto &x : s) m = std::min(m, x.size());
    return (int)m;
}
bool better(const std::vector<std::string> &a, const std::vector<std::string> &b) {   // a better than b
    int la = score_len(a), lb = score_len(b);
    if (la != lb) return la > lb;
    return !a.empty() && (b.empty() || a.size() < b.size());
}
void uniq(std::vector<std::string> &v) { std::sort(v.begin(), v.end()); v.erase(std::unique(v.begin(), v.end()), v.end()); }
void take_best(std::vector<std::string> &best, const std::vector<std::string> &cand) {
    if (score_len(cand) > 0 && better(cand, best)) best = cand;
}
void take_best(std::vector<std::string> &best, Follow &bf, const std::vector<std::string> &cand, const Follow &cf) {
    if (score_len(cand) > 0 && better(cand, best)) { best = cand; bf = cf; }
}

// FIRST set of a node (ASCII-folded: the factors are matched caseless) and whether it can match
// the empty string.  Used to extend 4-byte factors by the byte that must follow them: the WAF
// scan probes only even offsets, which a >= 5-byte key covers with two windows
// (gm_compile.cpp add_lit), while a 4-byte key needs 128 one-byte variants.
struct First { CSet set; bool nullable = true; };
First first_of(const std::vector<Node> &N, int n) {
    const Node &x = N[n];
    First r;
    switch (x.k) {
    case Node::EMPTY: case Node::BOL: case Node::EOL: return r;
    case Node::SET:
        for (int c = 0; c < 256; c++) if (x.set[c]) r.set[(c >= 'A' && c <= 'Z') ? c | 0x20 : c] = true;
        r.nullable = false;
        return r;
    case Node::CAT:
        for (int k : x.kids) {
            First g = first_of(N, k);
            r.set |= g.set;
            if (!g.nullable) { r.nullable = false; break; }
        }
        return r;
    case Node::ALT:
        r.nullable = false;
        for (int k : x.kids) { First g = first_of(N, k); r.set |= g.set; if (g.nullable) r.nullable = true; }
        return r;
    case Node::REP: {
        First g = first_of(N, x.kids[0]);
        r.set = g.set;
        r.nullable = x.mn == 0 || g.nullable;
        return r;
    }
    }
    return r;
}
// FIRST of the sequence kids[i..] of a CAT; nullable = the whole rest can be empty
First first_seq(const std::vector<Node> &N, const std::vector<int> &kids, size_t i) {
    First r;
    for (; i < kids.size(); i++) {
        First g = first_of(N, kids[i]);
        r.set |= g.set;
        if (!g.nullable) { r.nullable = false; return r; }
    }
    return r;
}
Follow follow_of(const First &f) {
    Follow r;
    if (!f.nullable && f.set.any()) { r.set = f.set; r.ok = true; }
    return r;
}

FI factors(const std::vector<Node> &N, int n) {
    const Node &x = N[n];
    FI r;
    switch (x.k) {
    case Node::EMPTY: case Node::BOL: case Node::EOL:
        r.exact_ok = true; r.exact = {""}; return r;
    case Node::SET: {
        std::vector<int> chars;
        CSet f;
        for (int c = 0; c < 256; c++) if (x.set[c]) f[(c >= 'A' && c <= 'Z') ? c | 0x20 : c] = true;
        if (f.count() <= 4) {
            r.exact_ok = true;
            for (int c = 0; c < 256; c++) if (f[c]) r.exact.push_back(std::string(1, (char)c));
            r.prefix = r.exact;
        }
        return r;
    }
    case Node::CAT: {
        std::vector<std::string> cur = {""};
        bool cur_ok = true, all_exact = true;
        std::vector<FI> gs;
        for (int k : x.kids) gs.push_back(factors(N, k));
        for (size_t gi = 0; gi < gs.size(); gi++) {
            const FI &g = gs[gi];
            take_best(r.best, r.best_follow, g.best, g.best_follow);
            if (g.exact_ok && cur_ok && cur.size() * g.exact.size() <= 16) {
                std::vector<std::string> nx;
                for (auto &a : cur) for (auto &b : g.exact) nx.push_back(a + b);
                uniq(nx);
                bool too_long = false; for (auto &s : nx) if (s.size() > 32) too_long = true;
                if (!too_long) { cur = nx; continue; }
            }
            // chain breaks here: cur is followed by FIRST(kids[gi..])
            all_exact = false;
            take_best(r.best, r.best_follow, cur, follow_of(first_seq(N, x.kids, gi)));
            if (g.exact_ok) { cur = g.exact; cur_ok = true; }
            else { cur = {""}; cur_ok = true; }
        }
        take_best(r.best, r.best_follow, cur, Follow{});
        if (all_exact) { r.exact_ok = true; r.exact = cur; }
        std::vector<std::string> pre = {""};
        Follow pf;   // follow set of pre
        for (size_t gi = 0; gi < gs.size(); gi++) {
            const FI &g = gs[gi];
            if (g.exact_ok) {
                auto nx = cross(pre, g.exact);
                if (small_set(nx)) { pre = nx; continue; }
                pf = follow_of(first_seq(N, x.kids, gi));
                break;
            }
            auto nx = cross(pre, g.prefix);
            if (small_set(nx) && g.prefix != std::vector<std::string>{""}) { pre = nx; pf = g.prefix_follow; }
            else pf = follow_of(first_seq(N, x.kids, gi));
            break;
        }
        r.prefix_follow = pf;
        r.prefix = pre;
        return r;
    }
    case Node::ALT: {
        bool all_exact = true, all_req = true;
        std::vector<std::string> ex, un, pu;
        Follow uf, pf;   // unions of the kids' follow sets (unknown if any kid's is)
        uf.ok = pf.ok = true;
        for (int k : x.kids) {
            FI g = factors(N, k);
            pu.insert(pu.end(), g.prefix.begin(), g.prefix.end());
            pf.ok = pf.ok && g.prefix_follow.ok; pf.set |= g.prefix_follow.set;
            if (g.exact_ok) ex.insert(ex.end(), g.exact.begin(), g.exact.end()); else all_exact = false;
            std::vector<std::string> b = g.best;
            Follow bf = g.best_follow;
            if (g.exact_ok) take_best(b, bf, g.exact, Follow{});
            uf.ok = uf.ok && bf.ok; uf.set |= bf.set;
            if (score_len(b) <= 0) all_req = false; else un.insert(un.end(), b.begin(), b.end());
        }
        uniq(ex); uniq(un);
        if (all_exact && ex.size() <= 16) { r.exact_ok = true; r.exact = ex; }
        if (all_req) { r.best = un; if (uf.ok) r.best_follow = uf; }
        uniq(pu);
        r.prefix = small_set(pu) ? pu : std::vector<std::string>{""};
        if (small_set(pu) && pf.ok) r.prefix_follow = pf;
        return r;
    }
    case Node::REP: {
        FI g = factors(N, x.kids[0]);
        if (x.mn >= 1) {
            r.prefix = g.prefix;
            r.prefix_follow = g.exact_ok ? Follow{} : g.prefix_follow;
            r.best = g.best;
            r.best_follow = g.best_follow;
            if (g.exact_ok) take_best(r.best, r.best_follow, g.exact, Follow{});
            if (x.mn == x.mx && g.exact_ok) {
                std::vector<std::string> cur = {""};
                bool ok = true;
                for (int q = 0; q < x.mn && ok; q++) {
                    std::vector<std::string> nx;
                    for (auto &a : cur) for (auto &b : g.exact) nx.push_back(a + b);
                    uniq(nx);
                    if (nx.size() > 16) ok = false;
                    for (auto &s : nx) if (s.size() > 32) ok = false;
                    cur = nx;
                }
                if (ok) { r.exact_ok = true; r.exact = cur; }
            }
        }
        return r;
    }
    }
    return r;
}

// ---------------------------------------------------------------- DFA construction
// Reversal of a pattern X$ (no '^', its only '$' the last item of the top-level sequence): the
// regex ^(\n)?rev(X) over the reversed subject.  X$ matches s (PCRE search: X ends at the end of
// s, or right before a final '\n') iff rev(X) matches a prefix of rev(s), or of rev(s) after its
// leading '\n' -- an anchored search that dies within a few bytes of most subjects.
int reverse_node(std::vector<Node> &N, int n) {
    Node x = N[n];
    if (x.k == Node::CAT) {
        std::vector<int> kids;
        for (auto it = x.kids.rbegin(); it != x.kids.rend(); ++it) kids.push_back(reverse_node(N, *it));
        x.kids = kids;
    } else if (x.k == Node::ALT || x.k == Node::REP) {
        for (int &k : x.kids) k = reverse_node(N, k);
    }
    N.push_back(x);
    return (int)N.size() - 1;
}
bool has_anchor(const std::vector<Node> &N, int n) {
    const Node &x = N[n];
    if (x.k == Node::BOL || x.k == Node::EOL) return true;
    for (int k : x.kids) if (has_anchor(N, k)) return true;
    return false;
}
int reverse_tail_anchored(std::vector<Node> &N, int root) {
    const Node r = N[root];
    if (r.k != Node::CAT || r.kids.empty() || N[r.kids.back()].k != Node::EOL) return -1;
    for (size_t q = 0; q + 1 < r.kids.size(); q++) if (has_anchor(N, r.kids[q])) return -1;
    Node body; body.k = Node::CAT;
    for (size_t q = 0; q + 1 < r.kids.size(); q++) body.kids.push_back(r.kids[q]);
    N.push_back(body);
    const int rb = reverse_node(N, (int)N.size() - 1);
    Node bol; bol.k = Node::BOL;
    N.push_back(bol);
    const int nb = (int)N.size() - 1;
    Node nl; nl.k = Node::SET; nl.set['\n'] = true;
    N.push_back(nl);
    Node opt; opt.k = Node::REP; opt.kids = {(int)N.size() - 1}; opt.mn = 0; opt.mx = 1;
    N.push_back(opt);
    const int no = (int)N.size() - 1;
    Node cat; cat.k = Node::CAT; cat.kids = {nb, no, rb};
    N.push_back(cat);
    return (int)N.size() - 1;
}

RegexInfo compile_impl(const std::string &pattern, bool caseless, int max_states, bool reversed);
}  // namespace

RegexInfo compile_regex(const std::string &pattern, bool caseless, int max_states) {
    return compile_impl(pattern, caseless, max_states, false);
}
bool compile_regex_reversed(const std::string &pattern, bool caseless, int max_states, Dfa &out) {
    RegexInfo r = compile_impl(pattern, caseless, max_states, true);
    if (r.status != RX_OK) return false;
    out = std::move(r.dfa);
    return true;
}

namespace {
RegexInfo compile_impl(const std::string &pattern, bool caseless, int max_states, bool reversed) {
    RegexInfo out;
    Parser P(pattern);
    P.icase = caseless;
    int root = P.parse();
    if (root < 0 || P.st != RX_OK) {
        out.status = P.st == RX_OK ? RX_SYNTAX : P.st;
        out.error = P.err;
        return out;
    }
    if (!check_anchors(P.nodes, root, true, true)) { out.status = RX_UNSUPPORTED; out.error = "anchor position"; return out; }
    if (reversed) {
        root = reverse_tail_anchored(P.nodes, root);
        if (root < 0) { out.status = RX_UNSUPPORTED; out.error = "not X$"; return out; }
    }

    NfaBuilder B(P.nodes);
    auto f = B.build(root);
    int match = B.mk({NS::MATCH, -1, -1, -1});
    B.patch(f.outs, match);
    int start = f.start;
    if (B.too_big) { out.status = RX_TOO_BIG; out.error = "nfa too big"; return out; }

    // byte classes: refine by membership in every set
    std::vector<int> cls(256, 0);
    {
        std::map<std::vector<bool>, int> sig;
        for (int b = 0; b < 256; b++) {
            std::vector<bool> v(B.sets.size());
            for (size_t s = 0; s < B.sets.size(); s++) v[s] = B.sets[s][b];
            auto it = sig.find(v);
            if (it == sig.end()) { int id = (int)sig.size(); sig[v] = id; cls[b] = id; }
            else cls[b] = it->second;
        }
        out.dfa.n_classes = (int)sig.size();
    }
    std::vector<int> rep(out.dfa.n_classes, 0);
    for (int b = 255; b >= 0; b--) rep[cls[b]] = b;

    const auto &S = B.st;
    auto closure = [&](std::vector<int> seeds, bool bol) {
        std::vector<char> seen(S.size(), 0);
        std::vector<int> stack = std::move(seeds), res;
        while (!stack.empty()) {
            int s = stack.back(); stack.pop_back();
            if (s < 0 || seen[s]) continue;
            seen[s] = 1;
            switch (S[s].t) {
            case NS::SPLIT: stack.push_back(S[s].out); stack.push_back(S[s].out1); break;
            case NS::EPS: stack.push_back(S[s].out); break;
            case NS::BOL: if (bol) stack.push_back(S[s].out); break;
            default: res.push_back(s); break;   // SET, EOL, MATCH kept
            }
        }
        std::sort(res.begin(), res.end());
        return res;
    };
    auto end_accept = [&](const std::vector<int> &set) {
        // follow EOL edges (and epsilons) to MATCH
        std::vector<int> seeds;
        for (int s : set) { if (S[s].t == NS::MATCH) return true; if (S[s].t == NS::EOL) seeds.push_back(S[s].out); }
        std::vector<char> seen(S.size(), 0);
        while (!seeds.empty()) {
            int s = seeds.back(); seeds.pop_back();
            if (s < 0 || seen[s]) continue;
            seen[s] = 1;
            if (S[s].t == NS::MATCH) return true;
            if (S[s].t == NS::SPLIT) { seeds.push_back(S[s].out); seeds.push_back(S[s].out1); }
            else if (S[s].t == NS::EPS || S[s].t == NS::EOL) seeds.push_back(S[s].out);
        }
        return false;
    };
    auto useful = [&](const std::vector<int> &set) {
        for (int s : set) if (S[s].t != NS::BOL) return true;
        return false;
    };

    std::vector<int> restart = closure({start}, false);
    bool can_restart = false;
    for (int s : restart) if (S[s].t == NS::SET || S[s].t == NS::MATCH || S[s].t == NS::EOL) can_restart = true;

    // search = true: unanchored PCRE search DFA (start set re-entered at every byte);
    // search = false: a DFA anchored at the first byte (prefix-trigger verification).
    auto build = [&](bool search, Dfa &D) -> bool {
        const bool has_restart = search && can_restart;
        D.anchored_start = !has_restart;
        D.n_classes = out.dfa.n_classes;
        std::map<std::vector<int>, int> ids;
        std::vector<std::vector<int>> sets;
        sets.push_back({});                       // 0 = dead
        std::vector<int> s0 = closure({start}, true);
        ids[s0] = 1; sets.push_back(s0);
        std::vector<uint16_t> trans;
        std::vector<uint8_t> acc;
        const int C = D.n_classes;
        for (size_t cur = 0; cur < sets.size(); cur++) {
            trans.resize((cur + 1) * C, 0);
            uint8_t a = 0;
            if (cur != 0) {
                for (int s : sets[cur]) if (S[s].t == NS::MATCH) a |= 1;
                if (end_accept(sets[cur])) a |= 2;
            }
            acc.push_back(a);
            if (cur == 0) continue;
            if (a & 1) {   // absorbing: a match already exists
                for (int c = 0; c < C; c++) trans[cur * C + c] = (uint16_t)cur;
                continue;
            }
            for (int c = 0; c < C; c++) {
                int b = rep[c];
                std::vector<int> seeds;
                for (int s : sets[cur]) if (S[s].t == NS::SET && B.sets[S[s].set][b]) seeds.push_back(S[s].out);
                if (has_restart) seeds.push_back(start);
                std::vector<int> nx = closure(seeds, false);
                int id;
                if (!useful(nx) || nx.empty()) id = 0;
                else {
                    auto it = ids.find(nx);
                    if (it == ids.end()) {
                        id = (int)sets.size();
                        if (id >= max_states) return false;
                        ids[nx] = id; sets.push_back(nx);
                    } else id = it->second;
                }
                trans[cur * C + c] = (uint16_t)id;
            }
        }
        D.trans = std::move(trans);
        D.acc = std::move(acc);
        D.n_states = (int)sets.size();
        for (int b = 0; b < 256; b++) D.cls[b] = (uint8_t)cls[b];
        return true;
    };
    if (!build(true, out.dfa)) { out.status = RX_TOO_BIG; out.error = "dfa too big"; return out; }
    if (reversed) { out.status = RX_OK; return out; }

    FI fi = factors(P.nodes, root);
    std::vector<std::string> best = fi.best;
    Follow bf = fi.best_follow;
    if (fi.exact_ok) take_best(best, bf, fi.exact, Follow{});
    if (score_len(best) > 0) {
        out.factors = best; out.min_factor = score_len(best);
        out.factor_follow = bf.set; out.has_factor_follow = bf.ok;
    }
    bool has_bol = false;
    for (auto &nd : P.nodes) if (nd.k == Node::BOL) has_bol = true;
    // prefix mode needs >= 4-byte prefixes (verified by an anchored DFA that dies within a few
    // bytes -- far cheaper than a factor job's search over the whole zone, so it always wins)
    if (!has_bol && score_len(fi.prefix) >= 4 && build(false, out.anchored)) {
        out.prefix = fi.prefix;
        out.prefix_follow = fi.prefix_follow.set; out.has_prefix_follow = fi.prefix_follow.ok;
        out.prefix_mode = true;
    }
    out.status = RX_OK;
    return out;
}
}  // namespace

bool dfa_search(const Dfa &d, const uint8_t *s, size_t n) {
    int st = 1;
    if (d.acc[st] & 1) return true;
    for (size_t i = 0; i < n; i++) {
        if ((d.acc[st] & 2) && i + 1 == n && s[i] == '\n') return true;
        st = d.trans[(size_t)st * d.n_classes + d.cls[s[i]]];
        if (st == 0) return false;
        if (d.acc[st] & 1) return true;
    }
    return (d.acc[st] & 2) != 0;
}

// ---------------------------------------------------------------- union DFA (always-run groups)
bool build_multi(const std::vector<const Dfa *> &comps, int max_states, MultiDfa &out) {
    const size_t k = comps.size();
    if (k == 0 || k > 32 || max_states > 0x3FFF) return false;
    // joint byte classes: bytes with the same class in every component
    int cls[256];
    std::vector<int> rep;
    {
        std::map<std::vector<uint8_t>, int> sig;
        for (int b = 0; b < 256; b++) {
            std::vector<uint8_t> v(k);
            for (size_t i = 0; i < k; i++) v[i] = comps[i]->cls[b];
            auto it = sig.emplace(v, (int)sig.size()).first;
            cls[b] = it->second;
            if (it->second == (int)rep.size()) rep.push_back(b);
        }
    }
    const int C = (int)rep.size();
    // state key: component states (u16 each) + the emitted mask
    std::unordered_map<std::string, int> ids;
    std::vector<std::vector<uint16_t>> tup;
    std::vector<uint32_t> emit;
    auto key_of = [&](const std::vector<uint16_t> &t, uint32_t e) {
        std::string s(reinterpret_cast<const char *>(t.data()), 2 * t.size());
        s.append(reinterpret_cast<const char *>(&e), 4);
        return s;
    };
    auto intern = [&](const std::vector<uint16_t> &t, uint32_t e) -> int {
        const std::string key = key_of(t, e);
        auto it = ids.find(key);
        if (it != ids.end()) return it->second;
        if ((int)tup.size() >= max_states) return -1;
        ids.emplace(key, (int)tup.size());
        tup.push_back(t);
        emit.push_back(e);
        return (int)tup.size() - 1;
    };
    intern(std::vector<uint16_t>(k, 0), 0);   // 0 = dead
    {
        std::vector<uint16_t> t(k, 1);
        uint32_t e = 0;
        for (size_t i = 0; i < k; i++)
            if (comps[i]->acc[1] & 1) { e |= 1u << i; t[i] = 0; }
        intern(t, e);
    }
    std::vector<uint16_t> trans;
    for (size_t cur = 0; cur < tup.size(); cur++) {
        trans.resize((cur + 1) * C, 0);
        if (cur == 0) continue;
        for (int c = 0; c < C; c++) {
            const int b = rep[c];
            std::vector<uint16_t> nt(k, 0);
            uint32_t e = 0;
            for (size_t i = 0; i < k; i++) {
                const uint16_t s = tup[cur][i];
                if (!s) continue;
                const Dfa &d = *comps[i];
                const uint16_t ns = d.trans[(size_t)s * d.n_classes + d.cls[b]];
                if (d.acc[ns] & 1) e |= 1u << i; else nt[i] = ns;
            }
            const int id = intern(nt, e);
            if (id < 0) return false;
            trans[cur * C + c] = (uint16_t)(id | (e ? MDFA_EMIT : 0));
        }
    }
    out.n_states = (int)tup.size();
    out.n_classes = C;
    out.trans = std::move(trans);
    out.emit = emit;
    out.endm.assign(tup.size(), 0);
    for (size_t s = 0; s < tup.size(); s++)
        for (size_t i = 0; i < k; i++)
            if (tup[s][i] && (comps[i]->acc[tup[s][i]] & 2)) out.endm[s] |= 1u << i;
    for (int b = 0; b < 256; b++) out.cls[b] = (uint8_t)cls[b];
    minimize_multi(out);
    return true;
}

// Moore partition refinement: states with the same emit / end masks whose transitions lead to
// equivalent states on every class merge (the product carries many: retired components, the
// same tuple reached with and without an emission).  Dead stays 0, start stays 1; the rest are
// numbered breadth-first from the start.
void minimize_multi(MultiDfa &m) {
    const int S = m.n_states, C = m.n_classes;
    if (S <= 2) return;
    std::vector<int> part(S), np(S);
    {
        std::map<std::pair<uint32_t, uint32_t>, int> ids;
        for (int s = 0; s < S; s++) part[s] = ids.emplace(std::make_pair(m.emit[s], m.endm[s]), (int)ids.size()).first->second;
    }
    int nparts = 0;
    for (;;) {
        std::unordered_map<std::string, int> ids;
        std::vector<int> sig(C + 1);
        for (int s = 0; s < S; s++) {
            sig[0] = part[s];
            for (int c = 0; c < C; c++) sig[c + 1] = part[m.trans[(size_t)s * C + c] & 0x3FFF];
            std::string key(reinterpret_cast<const char *>(sig.data()), sig.size() * sizeof(int));
            np[s] = ids.emplace(std::move(key), (int)ids.size()).first->second;
        }
        const int n = (int)ids.size();
        part.swap(np);
        if (n == nparts) break;
        nparts = n;
    }
    if (part[0] == part[1]) return;   // nothing can ever match: keep the product as built
    // renumber: dead 0, start 1, then BFS order
    std::vector<int> id(nparts, -1), rep;
    id[part[0]] = 0; rep.push_back(0);
    id[part[1]] = 1; rep.push_back(1);
    for (size_t q = 1; q < rep.size(); q++)
        for (int c = 0; c < C; c++) {
            const int t = m.trans[(size_t)rep[q] * C + c] & 0x3FFF;
            if (id[part[t]] < 0) { id[part[t]] = (int)rep.size(); rep.push_back(t); }
        }
    const int S2 = (int)rep.size();
    std::vector<uint16_t> tr((size_t)S2 * C, 0);
    std::vector<uint32_t> em(S2), en(S2);
    for (int q = 0; q < S2; q++) {
        em[q] = m.emit[rep[q]]; en[q] = m.endm[rep[q]];
        if (q == 0) continue;
        for (int c = 0; c < C; c++) {
            const uint16_t e = m.trans[(size_t)rep[q] * C + c];
            tr[(size_t)q * C + c] = (uint16_t)(id[part[e & 0x3FFF]] | (e & MDFA_EMIT));
        }
    }
    m.trans.swap(tr); m.emit.swap(em); m.endm.swap(en);
    m.n_states = S2;
}

uint32_t multi_search(const MultiDfa &m, const uint8_t *s, size_t n) {
    uint32_t st = 1, r = m.emit[1];
    for (size_t i = 0; i < n; i++) {
        if (i + 1 == n && s[i] == '\n') r |= m.endm[st];
        st = m.trans[(size_t)st * m.n_classes + m.cls[s[i]]] & 0x3FFF;
        r |= m.emit[st];
        if (st == 0) return r;
    }
    return r | m.endm[st];
}

}  // namespace gm

// ---------------------------------------------------------------- debug exports (gpumatch_debug.h)
extern "C" int gm_debug_regex(const char *pat, int caseless, const uint8_t *subj, size_t n) {
    gm::RegexInfo ri = gm::compile_regex(pat, caseless != 0);
    if (ri.status != gm::RX_OK) return -(int)ri.status;
    return gm::dfa_search(ri.dfa, subj, n) ? 1 : 0;
}

extern "C" int gm_debug_regex_rev(const char *pat, int caseless, const uint8_t *subj, size_t n) {
    gm::Dfa d;
    if (!gm::compile_regex_reversed(pat, caseless != 0, 4096, d)) return -1;
    std::vector<uint8_t> r(subj, subj + n);
    std::reverse(r.begin(), r.end());
    return gm::dfa_search(d, r.data(), r.size()) ? 1 : 0;
}
extern "C" int gm_debug_regex_factors(const char *pat, int caseless, char *out, size_t cap) {
    gm::RegexInfo ri = gm::compile_regex(pat, caseless != 0);
    if (ri.status != gm::RX_OK) return -(int)ri.status;
    size_t o = 0;
    for (auto &f : ri.factors) {
        if (o + f.size() + 1 > cap) break;
        memcpy(out + o, f.data(), f.size());
        o += f.size();
        out[o++] = '\n';
    }
    if (o < cap) out[o] = 0;
    return ri.min_factor;
}
