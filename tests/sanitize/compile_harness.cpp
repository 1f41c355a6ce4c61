// sanitizer harness: compile every blob given on the command line with the generation compiler
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gm_compile.hpp"
int main(int argc, char **argv) {
    int bad = 0;
    for (int i = 1; i < argc; i++) {
        FILE *f = fopen(argv[i], "rb");
        if (!f) { perror(argv[i]); return 2; }
        std::vector<uint8_t> b;
        uint8_t buf[65536]; size_t k;
        while ((k = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + k);
        fclose(f);
        gm::CompileResult r = gm::compile_generation(b.data(), b.size(), 1);
        printf("%s: ok=%d code=%d image=%zu\n", argv[i], (int)r.ok, r.code, r.image.size());
        if (!r.ok && r.code != GM_E_PARSE) bad++;
    }
    return bad ? 1 : 0;
}
