// CPU test of tools/interest_sets.hpp against std::set: random add/del streams
// on the two sets of an entity (InterestedIn / InterestedBy bits of one table)
// over a few ranges (tables that grow, clusters that wrap, deletes that shift),
// and replay_rows on per-entity rows.
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
    std::vector<std::set<uint32_t>> ref[2] = {std::vector<std::set<uint32_t>>(n), std::vector<std::set<uint32_t>>(n)};
    auto R = [&](uint32_t s) -> gwsets::Range & { return s < 150 ? r0 : r1; };
    const uint32_t bitof[2] = {gwsets::IN, gwsets::BY};
    long ops = 0;
    for (int it = 0; it < 600000; ++it) {
        const uint32_t s = (uint32_t)(rng() % n);
        const uint32_t k = (uint32_t)(rng() % (s % 7 == 0 ? 5000 : 200));  // some sets get big
        const bool add = rng() % 3 != 0;
        const int which = (int)(rng() % 3);  // 0: In, 1: By, 2: both
        const uint32_t bits = which == 2 ? (gwsets::IN | gwsets::BY) : bitof[which];
        const bool got = add ? R(s).add(s, k, bits) : R(s).del(s, k, bits);
        bool want = false;
        for (int q = 0; q < 2; ++q)
            if (which == 2 || which == q) want |= add ? ref[q][s].insert(k).second : ref[q][s].erase(k) > 0;
        if (got != want) {
            std::printf("FAIL op %d: s=%u k=%u add=%d sets=%d got=%d want=%d\n", it, s, k, add, which, got, want);
            return 1;
        }
        ++ops;
    }
    for (uint32_t s = 0; s < n; ++s)
        for (int q = 0; q < 2; ++q) {
            const std::vector<uint32_t> m = R(s).members(s, bitof[q]);
            if (m != std::vector<uint32_t>(ref[q][s].begin(), ref[q][s].end()) || R(s).size(s, bitof[q]) != ref[q][s].size()) {
                std::printf("FAIL members of %u (set %d)\n", s, q);
                return 1;
            }
            for (uint32_t k = 0; k < 300; ++k)
                if (R(s).has(s, k, bitof[q]) != (ref[q][s].count(k) > 0)) {
                    std::printf("FAIL has(%u, %u, set %d)\n", s, k, q);
                    return 1;
                }
        }
    // replay_rows: rows of enters then leaves applied to In and By
    std::vector<uint32_t> off{0}, items;
    for (uint32_t s = 0; s < n; ++s) {
        for (uint32_t k = 0; k < 3; ++k) items.push_back((s + k + 1) % n | 0x80000000u);
        off.push_back((uint32_t)items.size());
    }
    gwsets::Range r;
    r.init(0, n, nullptr);
    const uint64_t done = gwsets::replay_rows(r, off.data(), items.data(), 0x80000000u);
    if (done != 6ull * n || r.size(5, gwsets::IN) != 3 || !r.has(5, 6, gwsets::BY)) {
        std::printf("FAIL replay_rows\n");
        return 1;
    }
    std::vector<uint32_t> off2{0}, items2;  // a leave of every other member
    for (uint32_t s = 0; s < n; ++s) {
        items2.push_back((s + 2) % n);
        off2.push_back((uint32_t)items2.size());
    }
    gwsets::replay_rows(r, off2.data(), items2.data(), 0x80000000u);
    if (r.size(5, gwsets::IN) != 2 || r.has(5, 7, gwsets::BY) || !r.has(5, 8, gwsets::IN)) {
        std::printf("FAIL replay_rows leaves\n");
        return 1;
    }
    std::printf("ok %ld ops\n", ops);
    return 0;
}
