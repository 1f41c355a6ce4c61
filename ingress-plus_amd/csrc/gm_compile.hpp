// gm_compile.hpp -- generation compiler: GMB1 blob (nginx config text + signature set) ->
// device table image (gm_tables.hpp layout) + gm_stats_t.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/gpumatch.h"
#include "gm_tables.hpp"

namespace gm {

// Per upstream (sorted-name order): what a runtime server update needs to rebuild its peers.
struct UpstreamMeta {
    std::string name;
    uint32_t method = UM_DEFER;   // the block's balancing method before any defer
    bool has_block = false;       // an `upstream` block of this name exists
    bool defer_fixed = false;     // deferred whatever its servers (parameters, Plus method, key)
};

struct CompileResult {
    bool ok = false;
    int code = GM_OK;
    std::string err;
    std::vector<uint8_t> image;   // TabHeader at offset 0, sections at hdr.off_*
    TabHeader hdr{};
    gm_stats_t stats{};
    std::vector<std::string> peer_addrs;   // per global peer id: the `server` address
    std::vector<uint32_t> peer_ups;        // per global peer id: its upstream id
    std::vector<UpstreamMeta> ups_meta;    // per upstream id
    std::vector<uint32_t> peer_map;        // update_upstream: new peer id -> old peer id or GM_NONE
    std::vector<std::string> rejects;      // every rejected construct, "context: directive" (gm_rejects)
};

CompileResult compile_generation(const uint8_t *blob, size_t len, uint32_t gen);

// NGINX Plus runtime server update (Manager.UpdateServersInPlus, manager.go:257-284): the live
// generation `live` with upstream `name`'s `server` lines replaced by `addrs` (no `down`; the
// Plus API's max_fails / fail_timeout / slow_start do not change a pick).  Only the upstream
// section is rebuilt (DUpstream, consistent-hash rings, peers' initial flags); every other
// table is the live one's.  R.peer_map maps each new peer to the live peer of the same upstream
// and address (first unused one) or GM_NONE.  !R.ok with GM_E_INVAL: no such upstream.
CompileResult update_upstream(const CompileResult &live, const std::string &name, const std::vector<std::string> &addrs);

// The consistent-hash ring of a server list (ngx_http_upstream_update_chash), appended to points.
void chash_ring(const std::vector<std::string> &addrs, std::vector<DPoint> &points);

// Resolve device pointers of an image placed at `base` (host or device address).
GTab make_gtab(const TabHeader &h, const uint8_t *base, uint32_t gen);

}  // namespace gm
