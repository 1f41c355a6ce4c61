#!/bin/bash
# Wire-parser phase probes (measurement only, never shipped): exp/wpK/libgpumatch.so from a patched
# copy of csrc, the tree's sources untouched (their hash pairs the committed profiles).
#   wp0: the size pass stops after the LF scan and LDS stage     wp1: ... after the request line
#   wp2: ... after the header lines                              wp3: the whole size pass
# Every probe skips pass 2 (k_wire_emit / k_wire_emit_full), so wp3 = pass 1 + the size scan, and
# main - wp3 = pass 2.  Time them with: VARIANTS="main wp3 wp2 wp1 wp0" bash scripts/ab_wire.sh
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
mkdir -p "$W/ingress-plus_amd"
cp -r "$ROOT/ingress-plus_amd/csrc" "$W/ingress-plus_amd/"
cp -r "$ROOT/include" "$W/"
rm -f "$W"/ingress-plus_amd/csrc/*.o
cd "$W/ingress-plus_amd/csrc"
python3 - <<'EOF'
def put(path, anchor, text):
    s = open(path).read()
    assert s.count(anchor) == 1, anchor
    open(path, "w").write(s.replace(anchor, text + anchor))
put("gm_wire.inc", "    // the header as staged in LDS (the usual case: the line table ends inside the stage), else",
    "#if defined(GM_WIRE_PROBE) && GM_WIRE_PROBE == 0\n"
    "    if (!EMIT) return 16 + ((L + first_nul + status) & 16);\n#endif\n")
put("gm_wire.inc", "        // ---- header lines 1 .. L-1, a lane per line (rounds of 64)",
    "#if defined(GM_WIRE_PROBE) && GM_WIRE_PROBE == 1\n"
    "        if (!EMIT) return (uint64_t)(16 + ((status + uri_len + o.method_len + o.args_len) & 16));\n#endif\n")
put("gm_wire.inc", "        // ---- body: chunked (lane 0 walks the chunk lines) or Content-Length",
    "#if defined(GM_WIRE_PROBE) && GM_WIRE_PROBE == 2\n"
    "        if (!EMIT) return (uint64_t)(16 + ((status + hdrs_len + te_kind + (uint32_t)cl + uri_len) & 16));\n#endif\n")
put("gm_device.hip", "    k_wire_emit<<<blocks, 64 * WIRE_WAVES, 0, s>>>(wire, msgs, n, S->d_wsize, S->d_wbase, reqs, arena, arena_cap,",
    "#if defined(GM_WIRE_PROBE)\n    if (n) return G.done(c);\n#endif\n")
EOF
FL="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable"
make -s gm_compile.o gm_regex.o
for v in 0 1 2 3; do
  /opt/rocm/bin/hipcc $FL -DGM_WIRE_PROBE=$v --offload-arch=gfx950 -c gm_device.hip -o dev$v.o &
done
wait
for v in 0 1 2 3; do
  mkdir -p "$ROOT/exp/wp$v"
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/exp/wp$v/libgpumatch.so" dev$v.o gm_compile.o gm_regex.o \
    -L/opt/rocm/lib -lrccl -lamdhip64
done
rm -rf "$W"
