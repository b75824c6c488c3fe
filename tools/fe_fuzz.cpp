// Mutation fuzzer for the native front-end (host only): build with ASan/UBSan and run over
// seed streams; every mutated stream must decode or fail with an error code, never crash.
//   g++ -O1 -g -fsanitize=address,undefined -std=c++17 -pthread -Iinclude \
//       tools/fe_fuzz.cpp p265_amd/csrc/fe/*.cpp -o /tmp/fe_fuzz && /tmp/fe_fuzz 2000 seeds/*.bin
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "p265fe.h"

int main(int argc, char** argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: fe_fuzz iters seed.bin...\n"); return 2; }
    int iters = std::atoi(argv[1]);
    std::mt19937 rng(265);
    int ok = 0, err = 0;
    for (int f = 2; f < argc; ++f) {
        FILE* fp = std::fopen(argv[f], "rb");
        if (!fp) return 2;
        std::vector<uint8_t> seed;
        int ch;
        while ((ch = std::fgetc(fp)) != EOF) seed.push_back((uint8_t)ch);
        std::fclose(fp);
        for (int it = 0; it < iters; ++it) {
            std::vector<uint8_t> d = seed;
            int kind = rng() % 4;
            int n = 1 + rng() % 8;
            for (int k = 0; k < n && !d.empty(); ++k) {
                size_t pos = rng() % d.size();
                if (kind == 0) d[pos] ^= (uint8_t)(1u << (rng() % 8));
                else if (kind == 1) d[pos] = (uint8_t)rng();
                else if (kind == 2) d.insert(d.begin() + pos, (uint8_t)rng());
                else d.resize(pos + 1);
            }
            p265fe_decoder* dec = nullptr;
            p265fe_create(&dec);
            int r = p265fe_decode(dec, d.data(), d.size(), 1 + (it & 1));
            if (r >= 0) {
                ++ok;
                p265fe_picture_info info;
                for (int i = 0; i < r; ++i) p265fe_picture(dec, i, &info);
            } else {
                ++err;
            }
            p265fe_destroy(dec);
        }
    }
    std::printf("fuzz done: %d decoded, %d rejected\n", ok, err);
    return 0;
}
