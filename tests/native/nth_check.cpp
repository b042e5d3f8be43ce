// Host check: orbsel::nth_element (csrc/nth_select.h) == libstdc++ std::nth_element on
// tie-heavy random arrays (element identity carried in the low bits, compared on the top 8).
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>
#include "../../orbslam_jpminipc_amd/csrc/nth_select.h"
int depth_check(int);
int main(int argc, char** argv) {
    int trials = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 rng(12345);
    auto comp = [](uint32_t a, uint32_t b) { return (a >> 24) > (b >> 24); };
    long bad = 0;
    for (int t = 0; t < trials; ++t) {
        int n = (int)(rng() % 600) + 1;
        int span = 1 + (int)(rng() % 40);           // few distinct scores -> many ties
        int keep = (int)(rng() % (n + 3));
        std::vector<uint32_t> a(n);
        for (int i = 0; i < n; ++i) a[i] = ((uint32_t)(20 + rng() % span) << 24) | (uint32_t)i;
        if (t % 7 == 0) std::sort(a.begin(), a.end(), [](uint32_t x, uint32_t y){ return (x>>24) < (y>>24); });
        if (t % 11 == 0) for (int i = 0; i < n; ++i) a[i] = (200u << 24) | (uint32_t)i;  // all equal
        std::vector<uint32_t> b = a;
        if (keep < n) std::nth_element(b.begin(), b.begin() + keep, b.end(), comp);
        std::vector<uint32_t> c = a;
        orbsel::nth_element(c.data(), keep < n ? keep : n, n, comp);
        if (b != c) ++bad;
    }
    printf("trials %d mismatches %ld\n", trials, bad);
    return (bad != 0) | depth_check(trials);
}
// depth-limited path (__heap_select at depth 0), driven through libstdc++'s internal
// std::__introselect with an explicit depth so both sides take the heap branch.
int depth_check(int trials) {
    std::mt19937_64 rng(777);
    auto comp = [](uint32_t a, uint32_t b) { return (a >> 24) > (b >> 24); };
    long bad = 0;
    for (int t = 0; t < trials; ++t) {
        int n = (int)(rng() % 300) + 5, keep = (int)(rng() % n), depth = (int)(rng() % 4);
        std::vector<uint32_t> a(n);
        for (int i = 0; i < n; ++i) a[i] = ((uint32_t)(rng() % 17) << 24) | (uint32_t)i;
        std::vector<uint32_t> b = a, c = a;
        std::__introselect(b.begin(), b.begin() + keep, b.end(), (long)depth,
                           __gnu_cxx::__ops::__iter_comp_iter(comp));
        orbsel::introselect(c.data(), keep, n, depth, comp);
        if (b != c) ++bad;
    }
    printf("depth trials %d mismatches %ld\n", trials, bad);
    return bad != 0;
}
