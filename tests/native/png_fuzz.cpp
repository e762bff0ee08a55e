// Host-only driver for the sanitizer test of the PNG keyframe decoder (csrc/ingest.cpp):
// decodes every file named on the command line at its IHDR size and at a wrong size,
// so AddressSanitizer / UndefinedBehaviorSanitizer see every parser path on hostile
// input.  Built and run by tests/test_ingest_sanitizers.py; never part of the product.
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../include/mlgate.h"

static std::vector<uint8_t> slurp(const char* path) {
    std::vector<uint8_t> b;
    if (FILE* f = std::fopen(path, "rb")) {
        int c;
        while ((c = std::fgetc(f)) != EOF) b.push_back((uint8_t)c);
        std::fclose(f);
    }
    return b;
}

int main(int argc, char** argv) {
    int ok = 0, bad = 0;
    for (int i = 1; i < argc; ++i) {
        std::vector<uint8_t> b = slurp(argv[i]);
        int32_t w = 0, h = 0, ct = 0, bd = 0;
        const uint8_t* p = b.empty() ? nullptr : b.data();
        if (!p || mlg_png_info(p, b.size(), &w, &h, &ct, &bd) != MLG_OK || (long)w * h > (1L << 22)) {
            w = 16;
            h = 16;
        }
        for (int pass = 0; pass < 2; ++pass) {
            const int H = pass ? h + 1 : h, W = w;
            std::vector<uint8_t> out((size_t)H * W * 3);
            const uint8_t* ptrs[1] = {p ? p : (const uint8_t*)""};
            const size_t lens[1] = {b.size()};
            int32_t st = 0;
            if (mlg_png_decode_bgr(ptrs, lens, 1, out.data(), H, W, 1, &st) != MLG_OK) return 2;
            (st == MLG_OK ? ok : bad) += 1;
        }
        const char* paths[1] = {argv[i]};
        std::vector<uint8_t> out((size_t)h * w * 3);
        int32_t st = 0;
        if (mlg_png_load_bgr(paths, 1, out.data(), h, w, 2, &st) != MLG_OK) return 3;
    }
    std::printf("decoded %d, rejected %d\n", ok, bad);
    return 0;
}
