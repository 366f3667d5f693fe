// Per-entity InterestedIn / InterestedBy sets for the callback replay of
// Entity.go:236-246 (interest: a.InterestedIn.Add(b), b.InterestedBy.Add(a);
// uninterest: the deletes), the host side a cgo caller of libgwaoi keeps.
//
// One flat arena of open-addressing tables (linear probing, backward-shift
// delete, no tombstones), one table per entity, laid out in slot order: a
// replay that walks the flush's per-entity rows (gwaoi_events_csr) in slot
// order touches about one cache line per set operation and moves forward
// through memory, instead of chasing one heap vector per entity and scanning
// it for every delete.  A table that fills past half is moved to a bigger one
// at the end of its owner's overflow arena (the sets of a slot range belong to
// one thread, so no locks).
//
// The event stream never adds a present member or removes an absent one (the
// flush reports net changes), but add/del here are exact
// set operations anyway and report whether they changed the set.
//
// An entity's two sets share one table: an entry is the member's slot (< 2^30)
// with a bit for InterestedIn and a bit for InterestedBy, so one probe serves
// both sets of a row item (interest(s, b) and the mirrored interest(b, s) both
// change row s) and an entry leaves the table when neither bit is left.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace gwsets {

constexpr uint32_t EMPTY = 0xFFFFFFFFu;

struct Table {  // one entity's set: keys at arena[off .. off + cap)
    uint64_t off;
    uint32_t cap;  // power of two (0: no table yet)
    uint32_t size;
};

inline uint32_t slot_hash(uint32_t k, uint32_t mask) { return (k * 0x9E3779B1u >> 7) & mask; }

constexpr uint32_t IN = 1u << 30, BY = 1u << 31, KEY = IN - 1;  // entry = slot | membership bits

// The sets of entities [lo, hi): one owner thread.
class Range {
  public:
    Range() = default;
    // sizes[s - lo] = expected members of s (a table of 2x that, at least 16 keys = one line)
    void init(uint32_t lo, uint32_t hi, const uint32_t *sizes) {
        lo_ = lo;
        hi_ = hi;
        t_.assign(hi - lo, Table{0, 0, 0});
        uint64_t total = 0;
        for (uint32_t s = lo; s < hi; ++s) {
            const uint32_t c = cap_for(sizes ? sizes[s - lo] : 0);
            t_[s - lo] = Table{total, c, 0};
            total += c;
        }
        arena_.assign(total, EMPTY);
    }
    // add k to the sets of s named by bits (IN, BY or both); true if some set changed
    bool add(uint32_t s, uint32_t k, uint32_t bits) {
        Table &t = t_[s - lo_];
        if (2 * (t.size + 1) > t.cap) grow(t);
        uint32_t *a = arena_.data() + t.off;
        const uint32_t mask = t.cap - 1;
        for (uint32_t h = slot_hash(k, mask);; h = (h + 1) & mask) {
            if (a[h] == EMPTY) {
                a[h] = k | bits;
                ++t.size;
                return true;
            }
            if ((a[h] & KEY) == k) {
                const bool changed = (a[h] & bits) != bits;
                a[h] |= bits;
                return changed;
            }
        }
    }
    // remove k from the sets of s named by bits; true if some set changed
    bool del(uint32_t s, uint32_t k, uint32_t bits) {
        Table &t = t_[s - lo_];
        if (!t.size) return false;
        uint32_t *a = arena_.data() + t.off;
        const uint32_t mask = t.cap - 1;
        uint32_t h = slot_hash(k, mask);
        for (;; h = (h + 1) & mask) {
            if (a[h] == EMPTY) return false;
            if ((a[h] & KEY) == k) break;
        }
        const bool changed = (a[h] & bits) != 0;
        a[h] &= ~bits;
        if (a[h] & (IN | BY)) return changed;
        // neither set holds k: backward-shift delete, pulling later members of the probe
        // cluster into the hole
        uint32_t hole = h;
        for (uint32_t j = (h + 1) & mask; a[j] != EMPTY; j = (j + 1) & mask) {
            const uint32_t home = slot_hash(a[j] & KEY, mask);
            // a[j] may move to the hole iff the hole lies on its probe path [home, j)
            if (((j - home) & mask) >= ((j - hole) & mask)) {
                a[hole] = a[j];
                hole = j;
            }
        }
        a[hole] = EMPTY;
        --t.size;
        return changed;
    }
    bool has(uint32_t s, uint32_t k, uint32_t bit) const {
        const Table &t = t_[s - lo_];
        if (!t.cap) return false;
        const uint32_t *a = arena_.data() + t.off;
        const uint32_t mask = t.cap - 1;
        for (uint32_t h = slot_hash(k, mask);; h = (h + 1) & mask) {
            if (a[h] == EMPTY) return false;
            if ((a[h] & KEY) == k) return (a[h] & bit) != 0;
        }
    }
    // the members of one set (IN or BY) of s, sorted
    std::vector<uint32_t> members(uint32_t s, uint32_t bit) const {
        const Table &t = t_[s - lo_];
        std::vector<uint32_t> m;
        for (uint32_t i = 0; i < t.cap; ++i) {
            const uint32_t e = arena_[t.off + i];
            if (e != EMPTY && (e & bit)) m.push_back(e & KEY);
        }
        std::sort(m.begin(), m.end());
        return m;
    }
    uint32_t size(uint32_t s, uint32_t bit) const {
        const Table &t = t_[s - lo_];
        uint32_t c = 0;
        for (uint32_t i = 0; i < t.cap; ++i) {
            const uint32_t e = arena_[t.off + i];
            c += e != EMPTY && (e & bit) ? 1u : 0u;
        }
        return c;
    }
    uint32_t lo() const { return lo_; }
    uint32_t hi() const { return hi_; }
    // prefetch the line where a lookup of k in s's table starts (the replay runs this some
    // rows ahead: one random line per operation is the whole cost, and it is latency)
    void prefetch(uint32_t s, uint32_t k) const {
        const Table &t = t_[s - lo_];
        if (t.cap) __builtin_prefetch(arena_.data() + t.off + slot_hash(k, t.cap - 1), 1, 1);
    }

  private:
    static uint32_t cap_for(uint32_t n) {
        uint32_t c = 16;
        while (c < 2 * n + 2) c <<= 1;
        return c;
    }
    void grow(Table &t) {
        const uint32_t nc = t.cap ? 2 * t.cap : 16;
        const uint64_t noff = arena_.size();
        arena_.resize(noff + nc, EMPTY);  // (the old table's space is left unused)
        uint32_t *na = arena_.data() + noff;
        const uint32_t mask = nc - 1;
        for (uint32_t i = 0; i < t.cap; ++i) {
            const uint32_t e = arena_[t.off + i];
            if (e == EMPTY) continue;
            uint32_t h = slot_hash(e & KEY, mask);
            while (na[h] != EMPTY) h = (h + 1) & mask;
            na[h] = e;
        }
        t.off = noff;
        t.cap = nc;
    }
    uint32_t lo_ = 0, hi_ = 0;
    std::vector<Table> t_;
    std::vector<uint32_t> arena_;
};

// The replay of one flush for the slots of one Range from the per-entity rows
// of gwaoi_events_csr (row s: items b | enter_bit for the events (s, b)).  The
// flush's events come in pairs (s, b) and (b, s), so row s holds every change
// of s.InterestedIn (event (s, b)) and of s.InterestedBy (event (b, s)): one
// probe per item updates both.  Returns the set operations done.
inline uint64_t replay_rows(Range &r, const uint32_t *off, const uint32_t *items, uint32_t enter_bit) {
    constexpr uint32_t AHEAD = 16;  // items prefetched ahead of the one applied
    uint64_t ops = 0;
    // the item stream of the range, with its row, runs AHEAD items in front of the replay
    uint32_t ps = r.lo(), pk = off[r.lo()];
    const uint32_t kend = off[r.hi()];
    auto advance = [&]() {
        if (pk >= kend) return;
        while (off[ps + 1] <= pk) ++ps;
        r.prefetch(ps, items[pk] & ~enter_bit);
        ++pk;
    };
    for (uint32_t q = 0; q < AHEAD; ++q) advance();
    for (uint32_t s = r.lo(); s < r.hi(); ++s) {
        const uint32_t e = off[s + 1];
        for (uint32_t k = off[s]; k < e; ++k) {
            advance();
            const uint32_t it = items[k], b = it & ~enter_bit;
            if (it & enter_bit) r.add(s, b, IN | BY);
            else r.del(s, b, IN | BY);
        }
        ops += 2ull * (e - off[s]);
    }
    return ops;
}

}  // namespace gwsets
