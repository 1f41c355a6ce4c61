// The source hash libgpumatch.so was built from (Makefile: -DGM_CSRC_HASH, scripts/scan_profile.py
// csrc_hash over this directory and include/gpumatch.h).  Rebuilt whenever any source changes, so a
// shipped library always names the sources it came from (gm_build_hash, gm_stats_t.csrc_hash).
#ifndef GM_CSRC_HASH
#define GM_CSRC_HASH "unknown"
#endif
extern "C" const char gm_csrc_hash_text[] = GM_CSRC_HASH;
