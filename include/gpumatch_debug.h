/*
 * gpumatch_debug.h -- host-only introspection exports of libgpumatch.so, used by the CPU test
 * suite to check the generation compiler without a GPU (no request classification here).
 */
#ifndef GPUMATCH_DEBUG_H
#define GPUMATCH_DEBUG_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* Compile `pat` with the engine's regex compiler and run the DFA on the host:
 * 1 match, 0 no match, < 0 rejected (-1 PCRE-only, -2 unsupported, -3 syntax, -4 too big). */
int gm_debug_regex(const char *pat, int caseless, const uint8_t *subject, size_t n);
/* The reversed DFA of an X$ pattern (compile_regex_reversed) run over the subject from its last
 * byte backwards: 1 match, 0 no match, -1 not of the X$ form (or too big). */
int gm_debug_regex_rev(const char *pat, int caseless, const uint8_t *subject, size_t n);
/* Required-literal factors ('\n'-separated, case-folded) the WAF prefilter uses for `pat`;
 * returns the shortest factor length (0 = none), < 0 if rejected. */
int gm_debug_regex_factors(const char *pat, int caseless, char *out, size_t cap);
/* The distinct case-folded 4-byte key windows of the loaded generation's WAF prefilter (all
 * literals + regex triggers); returns their number (writes at most `cap`). */
struct gm_ctx;
/* The last batch's device status words (counts, profiling counters) as of the last gm_sync;
 * returns the number copied. */
int gm_debug_status(struct gm_ctx *ctx, uint32_t *out, size_t n);
/* the last gm_parse_requests' per-request slot sizes (its size pass) on `stream` */
int gm_debug_wire_sizes(struct gm_ctx *ctx, void *stream, uint64_t *out, size_t n);
/* DServer words of server `sid`, then its (dfa, loc) regex-location pairs; returns words written. */
int gm_debug_server(struct gm_ctx *ctx, uint32_t sid, uint32_t *out, size_t cap);
/* The union-DFA slices: 8 u32 each (len, n_groups, zones, server, min_member, flags, states,
 * classes); returns the u32 count. */
int gm_debug_alw_slices(struct gm_ctx *ctx, uint32_t *out, size_t cap);
int gm_debug_waf_keys(struct gm_ctx *ctx, uint32_t *out, size_t cap);
/* The prefilter's literal table: one row of 4 x uint32 per (key window, pattern) entry --
 * {key, rule id or regex index, (uint16)key_off | len << 16, flags | zones << 8}; returns the
 * number of entries (writes at most `cap` rows). */
int gm_debug_waf_lits(struct gm_ctx *ctx, uint32_t *out, size_t cap);
/* Pattern bytes (folded if nocase) of row `row` of gm_debug_waf_lits; returns the length. */
int gm_debug_waf_lit_bytes(struct gm_ctx *ctx, uint32_t row, uint8_t *out, size_t cap);
/* Host restatement of the WAF scan kernel's candidate rule over arena bytes A[0, len): writes
 * the candidate positions (at most `cap`) and returns their number. */
int64_t gm_debug_waf_prefilter(struct gm_ctx *ctx, const uint8_t *A, size_t len, uint64_t *out, size_t cap);
/* The same followed by k_waf_verify's stage-2 context filter: the windows that reach the exact check. */
int64_t gm_debug_waf_prefilter2(struct gm_ctx *ctx, const uint8_t *A, size_t len, uint64_t *out, size_t cap);
/* The realip address rules on the host (gm_inet.hpp, the code the device runs): `text` parsed as
 * ngx_parse_addr_port -> "<ngx_sock_ntop text> <port>" into out; -1 if it is not an address. */
/* Host-side profile of the always-run union DFAs over a batch (host buffers): out[0] transitions,
 * out[1] transitions taken in a group's start state that stay there, out[2] transitions taken in
 * the start state, out[3] (group, request, zone) tasks. */
int gm_debug_alw_profile(gm_ctx *ctx, const gm_req *reqs, const uint8_t *arena, uint32_t n, uint64_t *out4);
/* gm_counters_allreduce's protocol (RedProto, gm_device.hip) with the caller as the transport:
 * the block of gm_debug_red_words() u64 words a rank contributes to the SUM, and one state machine
 * per rank.  begin: 1 = agree first (a block-only collective, then gm_debug_red_agree with its sum),
 * 0 = issue the combined collective of red_words + *count words at once; finish: the combined
 * collective's summed block -> GM_OK (valid totals) or GM_E_COMM. */
void     gm_debug_red_pack(uint64_t gen, uint64_t n_counters, uint64_t *words);
uint32_t gm_debug_red_words(void);
void    *gm_debug_red_new(void);
void     gm_debug_red_free(void *proto);
int      gm_debug_red_begin(void *proto, uint64_t *count);
int      gm_debug_red_agree(void *proto, const uint64_t *sum_words);
int      gm_debug_red_finish(void *proto, const uint64_t *sum_words);
/* Tests: fn(arg) runs inside every later gm_update_upstream between its read of the live tables and
 * its publish, with no lock held (a gm_load_generation there must make the update fail GM_E_STALE).
 * fn = NULL clears it. */
void gm_debug_update_hook(void (*fn)(void *), void *arg);
int gm_debug_inet(const uint8_t *text, size_t n, char *out, size_t cap);
#ifdef __cplusplus
}
#endif
#endif
