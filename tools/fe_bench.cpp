// Host benchmark of the native front-end: parse a stream `reps` times on `threads` threads.
//   g++ -O3 -std=c++17 -pthread -Iinclude tools/fe_bench.cpp p265_amd/csrc/fe/*.cpp -o /tmp/fe_bench
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "p265fe.h"

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: fe_bench stream.bin [reps] [threads]\n"); return 2; }
    int reps = argc > 2 ? std::atoi(argv[2]) : 5, threads = argc > 3 ? std::atoi(argv[3]) : 1;
    FILE* fp = std::fopen(argv[1], "rb");
    if (!fp) return 2;
    std::vector<uint8_t> d;
    int ch;
    while ((ch = std::fgetc(fp)) != EOF) d.push_back((uint8_t)ch);
    std::fclose(fp);
    p265fe_decoder* dec = nullptr;
    p265fe_create(&dec);
    double best = 1e30;
    int n = 0;
    long ctus = 0;
    for (int r = 0; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        n = p265fe_decode(dec, d.data(), d.size(), threads);
        auto t1 = std::chrono::steady_clock::now();
        if (n < 0) { std::fprintf(stderr, "error %d: %s\n", n, p265fe_last_error(dec)); return 1; }
        double s = std::chrono::duration<double>(t1 - t0).count();
        if (s < best) best = s;
    }
    ctus = 0;
    for (int i = 0; i < n; ++i) { p265fe_picture_info info; p265fe_picture(dec, i, &info); ctus += info.n_ctus; }
    std::printf("%d pictures, %ld CTUs, %zu bytes: best %.3f ms -> %.0f CTU/s, %.1f MB/s (%d threads)\n", n, ctus,
                d.size(), best * 1e3, ctus / best, d.size() / best / 1e6, threads);
    p265fe_destroy(dec);
    return 0;
}
