// gm_consumer -- a data-plane consumer of the C-ABI: raw HTTP/1.x requests in,
// one decision per request out, every step on the GPU through libgpumatch.so only
// (include/gpumatch.h; no Python, no torch):
//
//   gm_parse_requests -> gm_match_batch -> gm_select_peers -> gm_upstream_uris -> gm_sync
//
// Batches are double-buffered on two HIP streams: while batch k runs on one stream, batch k+1's
// bytes are copied in on the other (pinned host buffers), so the copies overlap the kernels.
// The balancer state (gm_peer_state per peer) lives on the device for the whole run and carries
// from batch to batch; completed requests release their peer (gm_release_peers) the way nginx
// ends a connection.
//
//   gm_consumer <generation.blob> <requests.bin> [batch] [gen]
//     requests.bin: records { u32 len; u16 port; u8 https; u8 pad; u8 rid[16]; u8 raddr_len;
//                             u8 raddr[raddr_len]; u8 bytes[len] } back to back
//   stdout, one line per request, in order:
//     proxy <peer address> <upstream URI>     (GM_ACT_PROXY)
//     block 403 | return <status> | redirect <status> | reject <status> | notfound 404
//     defer | drop
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gpumatch.h"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)
#define GM(ctx, x)                                                                   \
    do {                                                                             \
        int r_ = (x);                                                                \
        if (r_ != GM_OK) {                                                           \
            fprintf(stderr, "%s: %d %s\n", #x, r_, gm_last_error(ctx));              \
            exit(3);                                                                 \
        }                                                                            \
    } while (0)

static std::vector<uint8_t> slurp(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    std::vector<uint8_t> b;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + k);
    fclose(f);
    return b;
}

struct Msg { size_t off; uint32_t len; gm_wire_msg m; };

// one batch's device buffers and pinned host mirrors
struct Slot {
    hipStream_t s = nullptr;
    uint8_t *h_wire = nullptr, *d_wire = nullptr;
    gm_wire_msg *h_msgs = nullptr, *d_msgs = nullptr;
    gm_req *d_reqs = nullptr;
    uint8_t *d_arena = nullptr;
    uint64_t *d_alen = nullptr;
    gm_verdict *d_out = nullptr, *h_out = nullptr;
    uint32_t *d_hits = nullptr;
    uint32_t *d_peer = nullptr, *h_peer = nullptr;
    uint8_t *d_uri = nullptr, *h_uri = nullptr;
    uint64_t *d_uoff = nullptr, *h_uoff = nullptr;
    uint32_t *d_ulen = nullptr, *h_ulen = nullptr;
    size_t wire_cap = 0, arena_cap = 0, uri_cap = 0;
    uint32_t n = 0, first = 0;
};

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s generation.blob requests.bin [batch] [gen]\n", argv[0]);
        return 1;
    }
    const uint32_t B = argc > 3 ? (uint32_t)atoi(argv[3]) : 4096;
    const uint32_t gen = argc > 4 ? (uint32_t)atoi(argv[4]) : 1;
    std::vector<uint8_t> blob = slurp(argv[1]), rq = slurp(argv[2]);

    gm_ctx *ctx = gm_create(0, 0);
    if (!ctx) { fprintf(stderr, "gm_create: %s\n", gm_last_error(nullptr)); return 2; }
    GM(ctx, gm_load_generation(ctx, blob.data(), blob.size(), gen));
    gm_stats_t st;
    GM(ctx, gm_stats(ctx, &st));
    const uint32_t n_peers = st.n_peers;

    // requests file -> messages
    std::vector<Msg> msgs;
    for (size_t p = 0; p + 24 <= rq.size();) {
        Msg x{};
        memcpy(&x.len, &rq[p], 4);
        uint16_t port; memcpy(&port, &rq[p + 4], 2);
        const uint8_t https = rq[p + 6];
        memset(&x.m, 0, sizeof x.m);
        x.m.port = port;
        x.m.flags = https ? GM_REQ_HTTPS : 0;
        memcpy(x.m.rid, &rq[p + 8], 16);
        const uint8_t ral = rq[p + 24];
        x.m.raddr_len = ral > 40 ? 40 : ral;
        memcpy(x.m.raddr, &rq[p + 25], x.m.raddr_len);
        x.m.remote_port = 40000;
        x.off = p + 25 + ral;
        if (x.off + x.len > rq.size()) break;
        msgs.push_back(x);
        p = x.off + x.len;
    }
    const uint32_t N = (uint32_t)msgs.size();

    gm_peer_state *d_state = nullptr;
    CK(hipMalloc(&d_state, (size_t)(n_peers ? n_peers : 1) * sizeof(gm_peer_state)));
    Slot slots[2];
    for (auto &sl : slots) CK(hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
    GM(ctx, gm_peers_init(ctx, d_state, n_peers, slots[0].s));
    CK(hipStreamSynchronize(slots[0].s));

    auto stage = [&](Slot &sl, uint32_t first) {
        sl.first = first;
        sl.n = std::min<uint32_t>(B, N - first);
        size_t wire = 0;
        for (uint32_t i = 0; i < sl.n; i++) wire += msgs[first + i].len;
        size_t acap = 16;
        for (uint32_t i = 0; i < sl.n; i++) acap += (2 * (size_t)msgs[first + i].len + 40 + 15) & ~size_t(15);
        const size_t ucap = 4 * acap + 64;
        if (wire + 16 > sl.wire_cap) {
            if (sl.h_wire) { CK(hipHostFree(sl.h_wire)); CK(hipFree(sl.d_wire)); }
            sl.wire_cap = 2 * (wire + 16);
            CK(hipHostMalloc((void **)&sl.h_wire, sl.wire_cap, hipHostMallocDefault));
            CK(hipMalloc((void **)&sl.d_wire, sl.wire_cap));
        }
        if (!sl.h_msgs) {
            CK(hipHostMalloc((void **)&sl.h_msgs, B * sizeof(gm_wire_msg), hipHostMallocDefault));
            CK(hipMalloc((void **)&sl.d_msgs, B * sizeof(gm_wire_msg)));
            CK(hipMalloc((void **)&sl.d_reqs, B * sizeof(gm_req)));
            CK(hipMalloc((void **)&sl.d_alen, 8));
            CK(hipMalloc((void **)&sl.d_out, B * sizeof(gm_verdict)));
            CK(hipHostMalloc((void **)&sl.h_out, B * sizeof(gm_verdict), hipHostMallocDefault));
            CK(hipMalloc((void **)&sl.d_hits, (4 * (size_t)B + 1024) * 4));
            CK(hipMalloc((void **)&sl.d_peer, B * 4));
            CK(hipHostMalloc((void **)&sl.h_peer, B * 4, hipHostMallocDefault));
            CK(hipMalloc((void **)&sl.d_uoff, B * 8));
            CK(hipHostMalloc((void **)&sl.h_uoff, B * 8, hipHostMallocDefault));
            CK(hipMalloc((void **)&sl.d_ulen, B * 4));
            CK(hipHostMalloc((void **)&sl.h_ulen, B * 4, hipHostMallocDefault));
        }
        if (acap > sl.arena_cap) {
            if (sl.d_arena) CK(hipFree(sl.d_arena));
            sl.arena_cap = 2 * acap;
            CK(hipMalloc((void **)&sl.d_arena, sl.arena_cap));
        }
        if (ucap > sl.uri_cap) {
            if (sl.d_uri) { CK(hipFree(sl.d_uri)); CK(hipHostFree(sl.h_uri)); }
            sl.uri_cap = 2 * ucap;
            CK(hipMalloc((void **)&sl.d_uri, sl.uri_cap));
            CK(hipHostMalloc((void **)&sl.h_uri, sl.uri_cap, hipHostMallocDefault));
        }
        size_t o = 0;
        for (uint32_t i = 0; i < sl.n; i++) {
            const Msg &x = msgs[first + i];
            memcpy(sl.h_wire + o, &rq[x.off], x.len);
            sl.h_msgs[i] = x.m;
            sl.h_msgs[i].off = o;
            sl.h_msgs[i].len = x.len;
            o += x.len;
        }
        CK(hipMemcpyAsync(sl.d_wire, sl.h_wire, o ? o : 1, hipMemcpyHostToDevice, sl.s));
        CK(hipMemcpyAsync(sl.d_msgs, sl.h_msgs, sl.n * sizeof(gm_wire_msg), hipMemcpyHostToDevice, sl.s));
        // the device chain, first half: bytes -> records -> verdicts (no shared state)
        GM(ctx, gm_parse_requests(ctx, sl.d_wire, sl.d_msgs, sl.n, sl.d_reqs, sl.d_arena, sl.arena_cap, sl.d_alen, sl.s));
        gm_batch in{};
        in.reqs = sl.d_reqs; in.arena = sl.d_arena; in.arena_len = sl.arena_cap; in.n = sl.n;
        in.arena_len_dev = sl.d_alen;
        GM(ctx, gm_match_batch(ctx, &in, sl.d_out, sl.d_hits, 4 * (size_t)B + 1024, sl.s));
    };

    // second half: peers (the shared balancer state) -> upstream URIs -> copies out
    auto stage_back = [&](Slot &sl) {
        gm_batch in{};
        in.reqs = sl.d_reqs; in.arena = sl.d_arena; in.arena_len = sl.arena_cap; in.n = sl.n;
        in.arena_len_dev = sl.d_alen;
        GM(ctx, gm_select_peers(ctx, &in, sl.d_out, d_state, n_peers, sl.d_peer, sl.s));
        GM(ctx, gm_upstream_uris(ctx, &in, sl.d_out, sl.d_uri, sl.uri_cap, sl.d_uoff, sl.d_ulen, sl.s));
        CK(hipMemcpyAsync(sl.h_out, sl.d_out, sl.n * sizeof(gm_verdict), hipMemcpyDeviceToHost, sl.s));
        CK(hipMemcpyAsync(sl.h_peer, sl.d_peer, sl.n * 4, hipMemcpyDeviceToHost, sl.s));
        CK(hipMemcpyAsync(sl.h_uoff, sl.d_uoff, sl.n * 8, hipMemcpyDeviceToHost, sl.s));
        CK(hipMemcpyAsync(sl.h_ulen, sl.d_ulen, sl.n * 4, hipMemcpyDeviceToHost, sl.s));
    };

    auto finish = [&](Slot &sl) {
        GM(ctx, gm_sync(ctx, sl.s));   // completes the stream (and reports overflow)
        uint64_t ubytes = 0;           // the URI bytes this batch produced
        for (uint32_t i = 0; i < sl.n; i++)
            if (sl.h_ulen[i] < GM_PEER_DEFER) ubytes = std::max<uint64_t>(ubytes, sl.h_uoff[i] + sl.h_ulen[i]);
        if (ubytes) CK(hipMemcpy(sl.h_uri, sl.d_uri, ubytes, hipMemcpyDeviceToHost));
        char addr[512];
        for (uint32_t i = 0; i < sl.n; i++) {
            const gm_verdict &v = sl.h_out[i];
            switch (v.action) {
            case GM_ACT_PROXY: {
                const uint32_t p = sl.h_peer[i], ul = sl.h_ulen[i];
                if (p == GM_PEER_DEFER || ul == GM_PEER_DEFER) { printf("defer\n"); break; }
                if (p == GM_NONE) { printf("return 502\n"); break; }
                if (gm_peer_address(ctx, p, addr, sizeof addr, nullptr) < 0) { printf("defer\n"); break; }
                printf("proxy %s %.*s\n", addr, (int)ul, (const char *)sl.h_uri + sl.h_uoff[i]);
                break;
            }
            case GM_ACT_BLOCK: printf("block %u\n", v.status); break;
            case GM_ACT_REDIRECT:
            case GM_ACT_AUTO_301: printf("redirect %u\n", v.status); break;
            case GM_ACT_RETURN:
            case GM_ACT_ERRPAGE: printf("return %u\n", v.status); break;
            case GM_ACT_NOT_FOUND: printf("notfound %u\n", v.status); break;
            case GM_ACT_BAD_REQUEST: printf("reject %u\n", v.status); break;
            case GM_ACT_UNSUPPORTED: printf("defer\n"); break;
            default: printf("drop\n"); break;
            }
        }
        // the proxied requests' connections end: their peers are released for the next batch
        GM(ctx, gm_release_peers(ctx, sl.d_peer, sl.n, d_state, n_peers, sl.s));
    };

    // two batches in flight: batch k+1's copies, parse and match run while batch k finishes;
    // the balancer state is shared, so k+1's peer selection waits (an event) for k's release
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    uint32_t next = 0;
    int cur = 0;
    if (next < N) { stage(slots[0], next); stage_back(slots[0]); next += slots[0].n; }
    while (slots[cur].n) {
        Slot &a = slots[cur], &b = slots[cur ^ 1];
        b.n = 0;
        if (next < N) { stage(b, next); next += b.n; }
        finish(a);
        if (b.n) {
            CK(hipEventRecord(ev, a.s));
            CK(hipStreamWaitEvent(b.s, ev, 0));
            stage_back(b);
        }
        a.n = 0;
        cur ^= 1;
    }
    CK(hipEventDestroy(ev));
    CK(hipDeviceSynchronize());
    gm_destroy(ctx);
    return 0;
}
