// CPU test of tools/interest_sets.hpp against std::set: random add/del streams
// over a few ranges (tables that grow, clusters that wrap, deletes that shift).
#include <cstdio>
#include <random>
#include <set>
#include <vector>

#include "../../tools/interest_sets.hpp"

int main() {
    std::mt19937_64 rng(12345);
    const uint32_t n = 300;
    std::vector<uint32_t> sizes(n);
    for (auto &s : sizes) s = (uint32_t)(rng() % 40);
    gwsets::Range r0, r1;
    r0.init(0, 150, sizes.data());
    r1.init(150, n, sizes.data() + 150);
    std::vector<std::set<uint32_t>> ref(n);
    auto R = [&](uint32_t s) -> gwsets::Range & { return s < 150 ? r0 : r1; };
    long ops = 0;
    for (int it = 0; it < 400000; ++it) {
        const uint32_t s = (uint32_t)(rng() % n);
        const uint32_t k = (uint32_t)(rng() % (s % 7 == 0 ? 5000 : 200));  // some sets get big
        const bool add = rng() % 3 != 0;
        const bool got = add ? R(s).add(s, k) : R(s).del(s, k);
        const bool want = add ? ref[s].insert(k).second : ref[s].erase(k) > 0;
        if (got != want) {
            std::printf("FAIL op %d: s=%u k=%u add=%d got=%d want=%d\n", it, s, k, add, got, want);
            return 1;
        }
        ++ops;
    }
    for (uint32_t s = 0; s < n; ++s) {
        const std::vector<uint32_t> m = R(s).members(s);
        if (m != std::vector<uint32_t>(ref[s].begin(), ref[s].end()) || R(s).size(s) != ref[s].size()) {
            std::printf("FAIL members of %u\n", s);
            return 1;
        }
        for (uint32_t k = 0; k < 300; ++k)
            if (R(s).has(s, k) != (ref[s].count(k) > 0)) {
                std::printf("FAIL has(%u, %u)\n", s, k);
                return 1;
            }
    }
    // replay_rows: rows of enters / leaves applied to In and By
    std::vector<uint32_t> off{0}, items;
    for (uint32_t s = 0; s < n; ++s) {
        for (uint32_t k = 0; k < 3; ++k) items.push_back((s + k + 1) % n | 0x80000000u);
        off.push_back((uint32_t)items.size());
    }
    gwsets::Range in, by;
    in.init(0, n, nullptr);
    by.init(0, n, nullptr);
    const uint64_t done = gwsets::replay_rows(in, by, off.data(), items.data(), 0x80000000u);
    if (done != 6ull * n || in.size(5) != 3 || !by.has(5, 6)) {
        std::printf("FAIL replay_rows\n");
        return 1;
    }
    std::printf("ok %ld ops\n", ops);
    return 0;
}
