// gm_regex.hpp -- RE2-compatible regex subset -> byte-class DFA, plus required-literal factors.
//
// Semantics follow PCRE 8.x as nginx uses it (ngx_regex_compile, no PCRE_MULTILINE /
// PCRE_DOTALL; `~*` adds PCRE_CASELESS): `.` excludes '\n', `^` = subject start, `$` = subject
// end or before a final '\n', \s = [\t\n\v\f\r ], \w = [0-9A-Za-z_], ASCII case folding.
// PCRE-only constructs (backrefs, lookaround, atomic groups, possessive quantifiers, \K,
// recursion, conditionals, callouts) are rejected with RX_PCRE_ONLY and counted by the caller
// (SURVEY.md §8 A8).
#pragma once
#include <stdint.h>
#include <bitset>
#include <string>
#include <vector>

namespace gm {

enum RegexStatus { RX_OK = 0, RX_PCRE_ONLY = 1, RX_UNSUPPORTED = 2, RX_SYNTAX = 3, RX_TOO_BIG = 4 };

struct Dfa {
    // state 0 = dead, state 1 = start.  acc bit0: accepting (match found once reached),
    // bit1: accepting at end of subject ($ satisfied).
    std::vector<uint16_t> trans;   // [n_states * n_classes]
    std::vector<uint8_t> acc;
    uint8_t cls[256];
    int n_states = 0, n_classes = 0;
    bool anchored_start = false;   // every start path begins with ^ (no search prefix)
};

struct RegexInfo {
    RegexStatus status = RX_SYNTAX;
    std::string error;
    Dfa dfa;
    std::vector<std::string> factors;  // case-folded literals; every match contains one of them
    int min_factor = 0;                // shortest factor length (0 = no factor)
    // prefix mode: every match *starts* with one of `prefix` (case-folded, all >= 4 bytes) and the
    // pattern has no '^': a match exists iff `anchored` accepts from some occurrence of a prefix.
    bool prefix_mode = false;
    std::vector<std::string> prefix;
    Dfa anchored;
    // folded bytes that can follow a factor / prefix string (has_* false = unknown): the WAF key
    // chooser keys a 4-byte string at odd offsets on "its last three bytes + a follow byte"
    std::bitset<256> factor_follow, prefix_follow;
    bool has_factor_follow = false, has_prefix_follow = false;
};

RegexInfo compile_regex(const std::string &pattern, bool caseless, int max_states = 8192);
// X$ (no '^'; its only '$' ends the top-level sequence): the DFA of ^(\n)?rev(X), which run over
// the subject's bytes from the last one backwards answers "X$ matches" (PCRE search semantics) and
// dies within a few bytes of most subjects.  false: not of that form, or too big.
bool compile_regex_reversed(const std::string &pattern, bool caseless, int max_states, Dfa &out);

// Union of search DFAs (compile_regex().dfa each): one pass over a subject answers "which of
// them match".  A state is (every component's state, the components that matched on entering
// it); a component that reaches an accepting state is retired (its state becomes 0) and the
// target state emits its bit, so the union never carries a matched component further.
// trans entries: target state | MDFA_EMIT when the target emits; endm[s]: components whose state
// in s accepts at the end of the subject ($).  State 0 = dead, 1 = start.
constexpr uint16_t MDFA_EMIT = 0x4000;
struct MultiDfa {
    std::vector<uint16_t> trans;   // [n_states * n_classes]
    std::vector<uint32_t> emit, endm;
    uint8_t cls[256];
    int n_states = 0, n_classes = 0;
};
// false when the union needs more than max_states states (<= 0x3FFF) before minimisation, or
// more than 32 components; the result is minimised (minimize_multi)
bool build_multi(const std::vector<const Dfa *> &comps, int max_states, MultiDfa &out);
void minimize_multi(MultiDfa &m);
// Host evaluation: bit k set iff comps[k] matches s (dfa_search semantics per component)
uint32_t multi_search(const MultiDfa &m, const uint8_t *s, size_t n);

// Host evaluation with PCRE search semantics (used for compile-time map truth tables).
bool dfa_search(const Dfa &d, const uint8_t *s, size_t n);

}  // namespace gm
