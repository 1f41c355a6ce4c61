// sanitizer harness for the union DFAs (gm_regex.cpp build_multi / minimize_multi): regexes from
// argv[1] ("<caseless 0|1> <pattern>" a line), subjects from argv[2] (one a line, "\n" escapes
// kept as the bytes they stand for).  Groups of 1..32 consecutive regexes are unioned; for every
// subject the union's answer (multi_search) must equal each member's own search (dfa_search).
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>
#include "gm_regex.hpp"
using namespace gm;
static std::string unescape(const std::string &s) {
    std::string o;
    for (size_t i = 0; i < s.size(); i++) {
        if (s[i] == '\\' && i + 1 < s.size() && s[i + 1] == 'n') { o += '\n'; i++; }
        else o += s[i];
    }
    return o;
}
int main(int argc, char **argv) {
    if (argc < 3) return 2;
    std::ifstream fr(argv[1]), fs(argv[2]);
    std::vector<Dfa> D;
    std::string line;
    while (std::getline(fr, line)) {
        if (line.size() < 3) continue;
        RegexInfo ri = compile_regex(line.substr(2), line[0] == '1');
        if (ri.status == RX_OK) D.push_back(ri.dfa);
    }
    std::vector<std::string> S;
    while (std::getline(fs, line)) S.push_back(unescape(line));
    S.push_back("");
    size_t groups = 0, checks = 0;
    int bad = 0;
    for (size_t g0 = 0, sz = 1; g0 < D.size(); g0 += sz, sz = sz % 32 + 1) {
        std::vector<const Dfa *> comps;
        for (size_t i = g0; i < D.size() && i < g0 + sz; i++) comps.push_back(&D[i]);
        MultiDfa m;
        if (!build_multi(comps, 8192, m)) continue;   // too big: the compiler keeps such a regex apart
        groups++;
        for (const std::string &s : S) {
            uint32_t want = 0;
            for (size_t k = 0; k < comps.size(); k++)
                if (dfa_search(*comps[k], (const uint8_t *)s.data(), s.size())) want |= 1u << k;
            const uint32_t got = multi_search(m, (const uint8_t *)s.data(), s.size());
            checks++;
            if (got != want && bad++ < 10) fprintf(stderr, "group at %zu size %zu: subject %zu: got %x want %x\n",
                                                   g0, comps.size(), (size_t)(&s - &S[0]), got, want);
        }
    }
    printf("regexes %zu groups %zu checks %zu mismatches %d\n", D.size(), groups, checks, bad);
    return bad ? 1 : 0;
}
