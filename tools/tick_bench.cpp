// gwaoi_tick_bench -- SURVEY.md §8(d)'s end-to-end tick from a C++ host, the
// view a cgo caller has: config 3 (1M entities, 256 Gaussian crowd hotspots +
// uniform background, D = 100, every entity moves by U(-1,1) per axis per tick
// in a seeded random call order), host move arrays (the caller's pinned buffers,
// gwaoi_moved_batch_pinned: one H2D, checked on the device) -> flush -> events
// in pinned host memory,
// then the callback replay of Entity.go:236-246 (interest / uninterest: a.In
// += b, b.By += a per directed event) into per-entity InterestedIn /
// InterestedBy sets, the part SURVEY.md §7 (hard part 6) expects to dominate.
//
// Three measurements, one JSON line:
//   serial     gwaoi_moved_batch_pinned + gwaoi_tick per tick (latency p50 / p99)
//   pipelined  gwaoi_tick_begin(t); gwaoi_moved_batch_pinned(t+1) while the GPU runs;
//              gwaoi_tick_finish(t)  (period = host replay overlapped with the flush)
//   replay     the tick's events into the sets: the event pairs on one thread;
//              the per-entity rows of gwaoi_events_csr on one and on T threads
//              (each thread owns the sets of a slot range; persistent pool)
//
// The sets are flat open-addressing tables in slot order (tools/interest_sets.hpp),
// so a replay of the rows moves forward through memory, about one cache line per
// set operation.  At the end 1,000 sampled entities' InterestedIn sets are
// compared with gwaoi_neighbors (the replay is exact, not just timed).
//
// The workload mirrors goworld_amd/workload.py (SplitMix64, Box-Muller in
// double); only its shape matters here, not bit-identity with the Python one.
//
// usage: gwaoi_tick_bench [ticks=20] [threads=16] [n=1000000]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <thread>
#include <vector>

#include "gwaoi.h"
#include "interest_sets.hpp"

namespace {

constexpr uint64_t GAMMA = 0x9E3779B97F4A7C15ull;

uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t subseed(uint64_t seed, uint64_t a, uint64_t b = ~0ull) {
    uint64_t h = mix64(seed ^ (a * GAMMA));
    if (b != ~0ull) h = mix64(h ^ (b * GAMMA));
    return h;
}
struct Stream {  // consecutive SplitMix64 outputs of a seed
    uint64_t s;
    uint64_t next() { return mix64(s += GAMMA); }
    double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double pct(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    if (v.empty()) return 0;
    return v[std::min(v.size() - 1, (size_t)(p / 100.0 * (v.size() - 1) + 0.5))];
}

void check(int rc, const char *what, gwaoi_world *w) {
    if (rc) {
        std::fprintf(stderr, "%s: %s (%s)\n", what, gwaoi_strerror(rc), w ? gwaoi_last_error(w) : "");
        std::exit(1);
    }
}

// InterestedIn / InterestedBy of every entity (one table per entity, a bit per
// set: tools/interest_sets.hpp), split into T slot ranges (one owner thread each).
struct Sets {
    uint32_t n, T;
    std::vector<gwsets::Range> r;
    Sets(uint32_t n_, uint32_t T_, const uint32_t *sizes) : n(n_), T(T_), r(T_) {
        for (uint32_t k = 0; k < T; ++k) {
            const uint32_t lo = lo_of(k), hi = lo_of(k + 1);
            r[k].init(lo, hi, sizes ? sizes + lo : nullptr);
        }
    }
    uint32_t lo_of(uint32_t k) const { return (uint32_t)((uint64_t)n * k / T); }
    uint32_t owner(uint32_t s) const {  // range holding slot s
        uint32_t k = (uint32_t)((uint64_t)s * T / n);
        while (k + 1 < T && s >= lo_of(k + 1)) ++k;
        while (k > 0 && s < lo_of(k)) --k;
        return k;
    }
};

// Entity.go:236-246 for the flush's event pairs on one thread (leaves first, then
// enters): uninterest / interest = a.In -/+= b, b.By -/+= a.
void replay_pairs(Sets &S, const gwaoi_events &ev) {
    for (uint64_t k = 0; k < ev.n_leave; ++k) {
        const uint32_t a = ev.leave[2 * k], b = ev.leave[2 * k + 1];
        S.r[S.owner(a)].del(a, b, gwsets::IN);
        S.r[S.owner(b)].del(b, a, gwsets::BY);
    }
    for (uint64_t k = 0; k < ev.n_enter; ++k) {
        const uint32_t a = ev.enter[2 * k], b = ev.enter[2 * k + 1];
        S.r[S.owner(a)].add(a, b, gwsets::IN);
        S.r[S.owner(b)].add(b, a, gwsets::BY);
    }
}

// Persistent workers: run(f) calls f(k) for k = 0..T-1 (k = 0 on the caller) and waits.
class Pool {
  public:
    explicit Pool(unsigned T) : T_(T) {
        for (unsigned k = 1; k < T; ++k) th_.emplace_back([this, k] { loop(k); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    void run(const std::function<void(unsigned)> &f) {
        {
            std::lock_guard<std::mutex> g(m_);
            f_ = &f;
            left_ = T_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return left_ == 0; });
    }

  private:
    void loop(unsigned k) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)> *f;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                f = f_;
            }
            (*f)(k);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--left_ == 0) done_.notify_one();
            }
        }
    }
    unsigned T_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)> *f_ = nullptr;
    uint64_t gen_ = 0;
    unsigned left_ = 0;
    bool stop_ = false;
};

}  // namespace

int main(int argc, char **argv) {
    const int ticks = argc > 1 ? std::atoi(argv[1]) : 20;
    const unsigned T = argc > 2 ? (unsigned)std::atoi(argv[2]) : 16;
    const uint32_t n = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 1000000;
    const uint64_t seed = 0x5EED0003ull;
    const double L = std::sqrt((double)n * 1250.0);
    // ---- config 3 positions: half uniform, half in hotspots of ~1953 entities (sigma 250)
    std::vector<float> x(n), z(n);
    {
        const uint32_t nu = n / 2, nh = n - nu, hot = std::max(1u, (uint32_t)std::lround(256.0 * n / 1e6));
        Stream su{subseed(seed, 1)};
        for (uint32_t i = 0; i < nu; ++i) x[i] = (float)(su.unit() * L - L / 2);
        for (uint32_t i = 0; i < nu; ++i) z[i] = (float)(su.unit() * L - L / 2);
        std::vector<double> cx(hot), cz(hot);
        Stream sc{subseed(seed, 2)};
        for (auto &c : cx) c = (sc.unit() * 0.8 - 0.4) * L;
        for (auto &c : cz) c = (sc.unit() * 0.8 - 0.4) * L;
        Stream sh{subseed(seed, 3)};
        for (uint32_t i = 0; i < nh; ++i) {
            const uint32_t h = (uint32_t)(sh.next() % hot);
            const double u1 = 1.0 - sh.unit(), u2 = sh.unit(), u3 = 1.0 - sh.unit(), u4 = sh.unit();
            x[nu + i] = (float)(cx[h] + 250.0 * std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2));
            z[nu + i] = (float)(cz[h] + 250.0 * std::sqrt(-2.0 * std::log(u3)) * std::cos(2.0 * M_PI * u4));
        }
    }
    // ---- move batches: 2 * ticks + 2 of them (serial + pipelined legs, one warmup each)
    const int nb = 2 * ticks + 2;
    std::vector<std::vector<uint32_t>> bs(nb);
    std::vector<std::vector<float>> bx(nb), bz(nb);
    {
        std::vector<std::pair<uint64_t, uint32_t>> ord(n);
        for (int t = 0; t < nb; ++t) {
            Stream so{subseed(seed, 0x0D3, (uint64_t)t)}, sm{subseed(seed, 0x71C, (uint64_t)t)};
            for (uint32_t i = 0; i < n; ++i) ord[i] = {so.next(), i};
            std::sort(ord.begin(), ord.end());
            bs[t].resize(n);
            bx[t].resize(n);
            bz[t].resize(n);
            std::vector<float> sx(n), sz(n);
            for (uint32_t i = 0; i < n; ++i) sx[i] = (float)(2.0 * sm.unit() - 1.0);
            for (uint32_t i = 0; i < n; ++i) sz[i] = (float)(2.0 * sm.unit() - 1.0);
            for (uint32_t k = 0; k < n; ++k) {
                const uint32_t s = ord[k].second;
                x[s] = x[s] + sx[s];
                z[s] = z[s] + sz[s];
                bs[t][k] = s;
                bx[t][k] = x[s];
                bz[t][k] = z[s];
            }
        }
    }
    // Enter at batch 0's positions (in its order) and move from batch 1 on.
    gwaoi_config cfg{};
    cfg.max_slots = n;
    cfg.max_spaces = 1;
    cfg.device = 0;
    gwaoi_world *w = nullptr;
    check(gwaoi_world_create(&cfg, &w), "world_create", nullptr);
    uint32_t sp = 0;
    check(gwaoi_space_create(w, 100.0f, &sp), "space_create", w);
    check(gwaoi_enter_batch(w, sp, bs[0].data(), bx[0].data(), bz[0].data(), n), "enter_batch", w);
    // the caller's per-tick move buffers in pinned memory (gwaoi_pinned_alloc), filled before timing:
    // a game server appends the decoded moves there while the tick's packets arrive, and
    // gwaoi_moved_batch_pinned sends a buffer with one H2D (checked on the device)
    std::vector<uint32_t *> pin(nb, nullptr);
    for (int t = 1; t < nb; ++t) {
        void *p = nullptr;
        check(gwaoi_pinned_alloc(w, 12 * (size_t)n, &p), "pinned_alloc", w);
        pin[t] = static_cast<uint32_t *>(p);
        std::copy(bs[t].begin(), bs[t].end(), pin[t]);
        std::copy(bx[t].begin(), bx[t].end(), reinterpret_cast<float *>(pin[t] + n));
        std::copy(bz[t].begin(), bz[t].end(), reinterpret_cast<float *>(pin[t] + 2 * (size_t)n));
    }
    auto batch = [&](int t) {
        check(gwaoi_moved_batch_pinned(w, pin[t], reinterpret_cast<const float *>(pin[t] + n),
                                       reinterpret_cast<const float *>(pin[t] + 2 * (size_t)n), n),
              "moved_batch_pinned", w);
    };
    gwaoi_events ev{};
    check(gwaoi_tick(w, &ev), "populate", w);
    const uint64_t populate = ev.n_enter;
    // the sets start from the populate flush's rows (tables sized 2x the first relation)
    const uint32_t *coff = nullptr, *citems = nullptr;
    uint64_t cn = 0;
    check(gwaoi_events_csr(w, &coff, &citems, &cn), "events_csr (populate)", w);
    std::vector<uint32_t> sizes(n);
    for (uint32_t i = 0; i < n; ++i) sizes[i] = coff[i + 1] - coff[i];
    Sets S(n, T, sizes.data());
    Pool pool(T);
    pool.run([&](unsigned k) { gwsets::replay_rows(S.r[k], coff, citems, GWAOI_CSR_ENTER); });

    // ---- serial leg: moved_batch + tick, then replay (one thread); odd ticks replay the event
    // pairs, even ticks the per-entity rows (gwaoi_events_csr, built on the GPU and copied)
    std::vector<double> t_stage, t_tick, t_lat, t_rep1, t_csr, t_repc1;
    uint64_t events = 0;
    for (int t = 1; t <= ticks; ++t) {
        const double a = now();
        batch(t);
        const double b = now();
        check(gwaoi_tick(w, &ev), "tick", w);
        const double c = now();
        double d, e = 0;
        if (t % 2) {
            replay_pairs(S, ev);
            d = now();
        } else {
            check(gwaoi_events_csr(w, &coff, &citems, &cn), "events_csr", w);
            e = now();
            for (unsigned k = 0; k < T; ++k) gwsets::replay_rows(S.r[k], coff, citems, GWAOI_CSR_ENTER);
            d = now();
        }
        if (t > 2) {  // the first ticks size the pinned buffers
            t_stage.push_back(b - a);
            t_tick.push_back(c - b);
            t_lat.push_back(c - a);
            if (t % 2) {
                t_rep1.push_back(d - c);
            } else {
                t_csr.push_back(e - c);
                t_repc1.push_back(d - e);
            }
            events += ev.n_enter + ev.n_leave;
        }
    }
    // ---- pipelined leg: while the GPU runs the flush of tick t, the host stages the batch of
    // t+1 and replays the callbacks of t-1 on T threads (the events of t-1 stay in the pinned
    // buffer until gwaoi_tick_finish(t) replaces them)
    std::vector<double> p_lat, t_repT, p_host;
    auto replay_T = [&]() {  // the rows of the last gwaoi_events_csr, T pool threads over slot ranges
        const double r0 = now();
        pool.run([&](unsigned k) { gwsets::replay_rows(S.r[k], coff, citems, GWAOI_CSR_ENTER); });
        t_repT.push_back(now() - r0);
    };
    int t = ticks + 1;
    double t_issue = now();
    batch(t);
    const double p0 = now();
    int done = 0;
    bool have_prev = false;
    for (; t < nb; ++t) {
        check(gwaoi_tick_begin(w), "tick_begin", w);
        const double h0 = now(), issued_next = h0;
        if (t + 1 < nb) batch(t + 1);
        if (have_prev) replay_T();  // tick t-1's callbacks, overlapping the flush of t
        p_host.push_back(now() - h0);
        uint64_t ne_, nl_;
        check(gwaoi_tick_finish(w, 0u, &ne_, &nl_), "tick_end", w);
        check(gwaoi_events_csr(w, &coff, &citems, &cn), "events_csr", w);
        p_lat.push_back(now() - t_issue);  // from this tick's batch call to its rows in host memory
        have_prev = true;
        t_issue = issued_next;
        ++done;
    }
    replay_T();
    const double p_total = now() - p0;
    const double p_flush = p_total;
    // exactness: In == By in size, the sets hold the last flush's relation, and 1,000 sampled
    // InterestedIn sets equal the world's neighbour rows
    uint64_t sin = 0, sby = 0;
    for (uint32_t i = 0; i < n; ++i) {
        sin += S.r[S.owner(i)].size(i, gwsets::IN);
        sby += S.r[S.owner(i)].size(i, gwsets::BY);
    }
    uint32_t sample_bad = 0;
    {
        std::vector<uint32_t> nb(1 << 16);
        Stream sq{subseed(seed, 0x5A)};
        for (int q = 0; q < 1000; ++q) {
            const uint32_t s = (uint32_t)(sq.next() % n);
            size_t cnt = 0;
            check(gwaoi_neighbors(w, s, nb.data(), nb.size(), &cnt), "neighbors", w);
            std::vector<uint32_t> want(nb.begin(), nb.begin() + (long)std::min(cnt, nb.size()));
            std::sort(want.begin(), want.end());
            if (S.r[S.owner(s)].members(s, gwsets::IN) != want || S.r[S.owner(s)].members(s, gwsets::BY) != want) ++sample_bad;
        }
    }
    for (uint32_t *p : pin)
        if (p) gwaoi_pinned_free(w, p);
    gwaoi_world_destroy(w);
    const double ms = 1e3;
    std::printf(
        "{\"entities\": %u, \"ticks\": %d, \"populate_enters\": %llu, \"events_per_tick\": %.1f, "
        "\"serial\": {\"stage_ms_p50\": %.4f, \"tick_ms_p50\": %.4f, \"latency_ms_mean\": %.4f, "
        "\"latency_ms_p50\": %.4f, \"latency_ms_p99\": %.4f}, "
        "\"pipelined\": {\"ms_per_tick\": %.4f, \"moves_per_s\": %.4g, \"latency_ms_p50\": %.4f, "
        "\"latency_ms_p99\": %.4f, \"host_ms_p50\": %.4f, "
        "\"note\": \"per tick: staging of t+1 and the T-thread replay of t-1 (per-entity rows) overlap the flush "
        "of t; latency = batch call to the rows in pinned host memory\"}, "
        "\"replay\": {\"pairs_ms_1thread_p50\": %.4f, \"csr_build_copy_ms_p50\": %.4f, "
        "\"csr_ms_1thread_p50\": %.4f, \"csr_ms_%uthreads_p50\": %.4f, \"threads\": %u}, "
        "\"relation_pairs\": %llu, \"in_eq_by\": %s, \"sampled_sets_vs_neighbors_mismatches\": %u}\n",
        n, ticks, (unsigned long long)populate, (double)events / std::max<size_t>(1, t_lat.size()),
        pct(t_stage, 50) * ms, pct(t_tick, 50) * ms,
        std::accumulate(t_lat.begin(), t_lat.end(), 0.0) / std::max<size_t>(1, t_lat.size()) * ms,
        pct(t_lat, 50) * ms, pct(t_lat, 99) * ms, p_flush / done * ms, (double)n * done / p_flush,
        pct(p_lat, 50) * ms, pct(p_lat, 99) * ms, pct(p_host, 50) * ms, pct(t_rep1, 50) * ms,
        pct(t_csr, 50) * ms, pct(t_repc1, 50) * ms, T, pct(t_repT, 50) * ms, T,
        (unsigned long long)sin, sin == sby ? "true" : "false", sample_bad);
    return 0;
}
