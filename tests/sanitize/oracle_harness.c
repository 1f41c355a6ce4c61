/* Sanitizer harness (ASan + UBSan, CPU only) for the oracle: for each (blob, requests) pair on
 * the command line, build the oracle context and run the matcher, the balancers, the upstream
 * URIs and the $uri normaliser; then parse a wire file.  Inputs are written by
 * tests/test_sanitizers.py. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gpumatch.h"

typedef struct orc_ctx orc_ctx;
orc_ctx *orc_create(const void *blob, size_t len, uint32_t gen);
int64_t orc_match(orc_ctx *c, const gm_req *reqs, const uint8_t *arena, uint32_t n, gm_verdict *out,
                  uint32_t *hit_ids, size_t hit_cap, int nthreads);
int orc_n_peers(orc_ctx *c);
int orc_peers_init(orc_ctx *c, gm_peer_state *st, uint32_t n_peers);
int orc_select_peers(orc_ctx *c, const gm_req *reqs, const uint8_t *arena, const gm_verdict *v, uint32_t n,
                     gm_peer_state *st, uint32_t n_peers, uint32_t *out);
int64_t orc_upstream_uris(orc_ctx *c, const gm_req *reqs, const uint8_t *arena, const gm_verdict *v, uint32_t n,
                          uint8_t *out, uint64_t cap, uint64_t *out_off, uint32_t *out_len);
int orc_set_prefilter(orc_ctx *c, int on);
void orc_normalize_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t n,
                         uint8_t *out, uint32_t *out_len);
int64_t orc_parse_requests(const uint8_t *wire, const gm_wire_msg *msgs, uint32_t n, gm_req *reqs, uint8_t *arena,
                           uint64_t cap);

static uint8_t *slurp(const char *p, size_t *n) {
    FILE *f = fopen(p, "rb");
    if (!f) { perror(p); exit(2); }
    fseek(f, 0, SEEK_END); *n = (size_t)ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t *b = malloc(*n + 16);
    if (*n && fread(b, 1, *n, f) != *n) { perror(p); exit(2); }
    fclose(f);
    return b;
}

int main(int argc, char **argv) {
    /* argv: wire msgs  then triples: blob reqs arena */
    if (argc < 3) return 2;
    size_t wn, mn;
    uint8_t *w = slurp(argv[1], &wn), *m = slurp(argv[2], &mn);
    uint32_t nm = (uint32_t)(mn / sizeof(gm_wire_msg));
    uint64_t cap = 16;
    for (uint32_t i = 0; i < nm; i++) cap += ((2 * (uint64_t)((gm_wire_msg *)m)[i].len + 40 + 15) & ~15ull);
    gm_req *pr = calloc(nm + 1, sizeof(gm_req));
    uint8_t *pa = calloc(cap, 1);
    if (orc_parse_requests(w, (gm_wire_msg *)m, nm, pr, pa, cap) < 0) return 3;
    for (int a = 3; a + 2 < argc; a += 3) {
        size_t bn, rn, an;
        uint8_t *b = slurp(argv[a], &bn), *r = slurp(argv[a + 1], &rn), *ar = slurp(argv[a + 2], &an);
        uint32_t n = (uint32_t)(rn / sizeof(gm_req));
        orc_ctx *c = orc_create(b, bn, 1);
        if (!c) { printf("%s: rejected\n", argv[a]); continue; }
        gm_verdict *v = calloc(n + 1, sizeof(gm_verdict));
        size_t hc = 64 * (size_t)n + 1024;
        uint32_t *h = calloc(hc, 4);
        for (int pf = 0; pf < 2; pf++) {
            orc_set_prefilter(c, pf);
            if (orc_match(c, (gm_req *)r, ar, n, v, h, hc, 2) < 0) return 4;
        }
        int np = orc_n_peers(c);
        gm_peer_state *st = calloc(np + 1, sizeof(gm_peer_state));
        orc_peers_init(c, st, (uint32_t)np);
        uint32_t *po = calloc(n + 1, 4);
        orc_select_peers(c, (gm_req *)r, ar, v, n, st, (uint32_t)np, po);
        uint64_t ucap = 4 * an + 64 * (uint64_t)n + 64;
        uint8_t *uo = calloc(ucap, 1);
        uint64_t *off = calloc(n + 1, 8);
        uint32_t *ln = calloc(n + 1, 4);
        orc_upstream_uris(c, (gm_req *)r, ar, v, n, uo, ucap, off, ln);
        for (uint32_t i = 0; i < n; i++) { off[i] = ((gm_req *)r)[i].base; ln[i] = ((gm_req *)r)[i].uri_len; }
        uint8_t *no = calloc(an + 16, 1);
        uint32_t *nl = calloc(n + 1, 4);
        orc_normalize_batch(ar, off, ln, n, no, nl);
        printf("%s: %u requests ok\n", argv[a], n);
    }
    return 0;
}
