// C++ host mirror (include/gwaoi_aoi.hpp) on the GPU: Appendix C KATs through
// the AOIManager interface, then a random Enter/Moved/Leave/space-change
// stream whose interest sets are checked after every flush against a
// brute-force evaluation of the closed form and for
// In == By symmetry.  Prints "ok" and exits 0 on success.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <set>
#include <vector>

#include "gwaoi_aoi.hpp"

namespace {

int failures = 0;
#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                  \
        }                                                                \
    } while (0)

struct Ent : gwaoi::AOICallback {
    int id = 0;
    gwaoi::AOI aoi;
    std::set<Ent *> in, by;
    void OnEnterAOI(gwaoi::AOI *o) override {
        Ent *e = static_cast<Ent *>(o->Data);
        in.insert(e);
        e->by.insert(this);
    }
    void OnLeaveAOI(gwaoi::AOI *o) override {
        Ent *e = static_cast<Ent *>(o->Data);
        in.erase(e);
        e->by.erase(this);
    }
};

float bits(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// P_W(L) of go-aoi: L inside W's float32 window
bool pred(float wx, float wz, float lx, float lz, float D) {
    return lx >= wx - D && lx <= wx + D && lz >= wz - D && lz <= wz + D;
}

void kats() {
    gwaoi::World w(16);
    auto m = w.NewXZListAOIManager(100.f);
    Ent a, b;
    a.id = 0;
    b.id = 1;
    gwaoi::InitAOI(&a.aoi, 100.f, &a, &a);
    gwaoi::InitAOI(&b.aoi, 100.f, &b, &b);
    // R1: A = 0xc57cc1a7, B = 0xc58180d4; whoever moved last decides
    m->Enter(&b.aoi, bits(0xC58180D4), 0.f);
    m->Enter(&a.aoi, bits(0xC57CC1A7), 0.f);
    auto r = w.Flush();
    CHECK(r.first == 2 && r.second == 0 && a.in.count(&b) && b.in.count(&a));
    m->Moved(&b.aoi, bits(0xC58180D4), 0.f);
    r = w.Flush();
    CHECK(r.first == 0 && r.second == 2 && a.in.empty() && b.in.empty());
    m->Leave(&a.aoi);
    m->Leave(&b.aoi);
    w.Flush();
    // T1: 10 co-located entities -> 90 directed enters; L1: leave -> 2k leaves
    std::vector<Ent> t(10);
    for (int i = 0; i < 10; ++i) {
        t[i].id = i;
        gwaoi::InitAOI(&t[i].aoi, 100.f, &t[i], &t[i]);
        m->Enter(&t[i].aoi, 0.f, 0.f);
    }
    r = w.Flush();
    CHECK(r.first == 90);
    m->Leave(&t[3].aoi);
    r = w.Flush();
    CHECK(r.second == 18 && t[3].in.empty() && t[3].by.empty());
    // misuse throws like the reference panics
    bool threw = false;
    try {
        m->Moved(&t[3].aoi, 1.f, 1.f);
    } catch (const gwaoi::Error &) {
        threw = true;
    }
    CHECK(threw);
    for (int i = 0; i < 10; ++i)
        if (i != 3) m->Leave(&t[i].aoi);
    w.Flush();
}

void random_stream() {
    const int n = 500, ns = 2;
    const float D[ns] = {100.f, 45.f};
    gwaoi::World w(n + 8, ns);
    std::unique_ptr<gwaoi::XZListAOIManager> mg[ns] = {w.NewXZListAOIManager(D[0]), w.NewXZListAOIManager(D[1])};
    std::vector<Ent> e(n);
    std::vector<int> where(n, -1);
    std::vector<uint64_t> seq(n, 0);
    std::vector<float> x(n), z(n);
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<float> U(-400.f, 400.f), S(-5.f, 5.f), P(0.f, 1.f);
    uint64_t next = 1;
    for (int i = 0; i < n; ++i) {
        e[i].id = i;
        gwaoi::InitAOI(&e[i].aoi, 100.f, &e[i], &e[i]);
        x[i] = U(rng);
        z[i] = U(rng);
    }
    for (int tick = 0; tick < 12; ++tick) {
        std::vector<int> order(n);
        for (int i = 0; i < n; ++i) order[i] = i;
        std::shuffle(order.begin(), order.end(), rng);
        for (int i : order) {
            const float r = P(rng);
            if (where[i] < 0) {
                if (tick == 0 || r < 0.6f) {
                    where[i] = (int)(rng() % ns);
                    mg[where[i]]->Enter(&e[i].aoi, x[i], z[i]);
                    seq[i] = next++;
                }
            } else if (r < 0.04f) {
                mg[where[i]]->Leave(&e[i].aoi);
                where[i] = -1;
            } else if (r < 0.07f) {  // change space inside the flush
                mg[where[i]]->Leave(&e[i].aoi);
                where[i] = 1 - where[i];
                mg[where[i]]->Enter(&e[i].aoi, x[i], z[i]);
                seq[i] = next++;
            } else if (r < 0.09f) {  // teleport
                x[i] = U(rng);
                z[i] = U(rng);
                mg[where[i]]->Moved(&e[i].aoi, x[i], z[i]);
                seq[i] = next++;
            } else {
                x[i] = x[i] + S(rng);
                z[i] = z[i] + S(rng);
                mg[where[i]]->Moved(&e[i].aoi, x[i], z[i]);
                seq[i] = next++;
            }
        }
        w.Flush();
        for (int a = 0; a < n; ++a) {
            CHECK(e[a].in == e[a].by);
            std::set<Ent *> want;
            if (where[a] >= 0)
                for (int b = 0; b < n; ++b) {
                    if (b == a || where[b] != where[a]) continue;
                    const bool aw = seq[a] > seq[b];
                    const int W = aw ? a : b, L = aw ? b : a;
                    if (pred(x[W], z[W], x[L], z[L], D[where[a]])) want.insert(&e[b]);
                }
            if (e[a].in != want) {
                std::fprintf(stderr, "tick %d entity %d: %zu interests, closed form %zu\n", tick, a, e[a].in.size(),
                             want.size());
                ++failures;
                return;
            }
        }
    }
}

}  // namespace

int main() {
    try {
        kats();
        random_stream();
    } catch (const gwaoi::Error &ex) {
        std::fprintf(stderr, "gwaoi error %d: %s\n", ex.status(), ex.what());
        return 2;
    }
    if (failures) {
        std::fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    std::printf("ok\n");
    return 0;
}
