// gm_compile.hpp -- generation compiler: GMB1 blob (nginx config text + signature set) ->
// device table image (gm_tables.hpp layout) + gm_stats_t.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/gpumatch.h"
#include "gm_tables.hpp"

namespace gm {

struct CompileResult {
    bool ok = false;
    int code = GM_OK;
    std::string err;
    std::vector<uint8_t> image;   // TabHeader at offset 0, sections at hdr.off_*
    TabHeader hdr{};
    gm_stats_t stats{};
    std::vector<std::string> peer_addrs;   // per global peer id: the `server` address
    std::vector<uint32_t> peer_ups;        // per global peer id: its upstream id
};

CompileResult compile_generation(const uint8_t *blob, size_t len, uint32_t gen);

// Resolve device pointers of an image placed at `base` (host or device address).
GTab make_gtab(const TabHeader &h, const uint8_t *base, uint32_t gen);

}  // namespace gm
