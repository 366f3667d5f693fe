/*
 * gwaoi_aoi.hpp -- C++ mirror of go-aoi's AOIManager interface over the C ABI
 * (gwaoi.h).  Header-only; link with -lgwaoi.
 *
 *   go-aoi (package aoi, v0.2.0)             here
 *   --------------------------------------   ------------------------------------
 *   type Coord float32                       gwaoi::Coord
 *   type AOI struct {..., Data interface{}}  gwaoi::AOI (Data = void*)
 *   InitAOI(aoi, dist, data, cb)             gwaoi::InitAOI     (Entity.go:210)
 *   AOICallback{OnEnterAOI, OnLeaveAOI}      gwaoi::AOICallback (Entity.go:227-233)
 *   AOIManager{Enter, Leave, Moved}          gwaoi::AOIManager  (Space.go:211,221,243,259)
 *   NewXZListAOIManager(dist)                World::NewXZListAOIManager (Space.go:105)
 *
 * Calls are queued in call order and handed to the GPU in batches at
 * World::Flush(), which replays the NET per-flush callbacks: all leaves, then
 * all enters, each pair as A->OnXxx(B), B->OnXxx(A).  Misuse go-aoi panics on
 * throws gwaoi::Error at the call.  One World per GPU and thread.
 */
#ifndef GWAOI_AOI_HPP
#define GWAOI_AOI_HPP

#include <cmath>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "gwaoi.h"

namespace gwaoi {

using Coord = float;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

class Error : public std::runtime_error {
  public:
    Error(int status, const std::string &what) : std::runtime_error(what), status_(status) {}
    int status() const { return status_; }

  private:
    int status_;
};

struct AOI;

struct AOICallback {
    virtual ~AOICallback() = default;
    virtual void OnEnterAOI(AOI *other) = 0;
    virtual void OnLeaveAOI(AOI *other) = 0;
};

class XZListAOIManager;

struct AOI {
    Coord x = 0, y = 0;  // y carries world Z, as GoWorld passes it
    Coord dist = 0;      // stored, not used by the XZ-list manager (as in go-aoi)
    void *Data = nullptr;
    AOICallback *callback = nullptr;
    // engine state
    uint32_t slot = kNoSlot;
    XZListAOIManager *mgr = nullptr;
};

inline void InitAOI(AOI *aoi, Coord dist, void *data, AOICallback *cb) {
    aoi->dist = dist;
    aoi->Data = data;
    aoi->callback = cb;
}

class AOIManager {
  public:
    virtual ~AOIManager() = default;
    virtual void Enter(AOI *aoi, Coord x, Coord y) = 0;
    virtual void Leave(AOI *aoi) = 0;
    virtual void Moved(AOI *aoi, Coord x, Coord y) = 0;
};

class World {
  public:
    explicit World(uint32_t max_entities, uint32_t max_spaces = 1, int device = -1, float cells_per_dist = 0.f)
        : by_slot_(max_entities, nullptr) {
        gwaoi_config cfg{};
        cfg.max_slots = max_entities;
        cfg.max_spaces = max_spaces;
        cfg.device = device;
        cfg.cells_per_dist = cells_per_dist;
        check(gwaoi_world_create(&cfg, &w_));
        free_.reserve(max_entities);
        for (uint32_t s = max_entities; s-- > 0;) free_.push_back(s);
    }
    ~World() {
        if (w_) gwaoi_world_destroy(w_);
    }
    World(const World &) = delete;
    World &operator=(const World &) = delete;

    inline std::unique_ptr<XZListAOIManager> NewXZListAOIManager(Coord dist);

    // Flush: GPU tick + callback replay.  Returns (directed enters, directed leaves).
    std::pair<uint64_t, uint64_t> Flush() {
        submit();
        gwaoi_events ev{};
        check(gwaoi_tick(w_, &ev));
        for (uint64_t i = 0; i < ev.n_leave; ++i) {
            AOI *a = by_slot_[ev.leave[2 * i]], *b = by_slot_[ev.leave[2 * i + 1]];
            a->callback->OnLeaveAOI(b);
        }
        for (uint64_t i = 0; i < ev.n_enter; ++i) {
            AOI *a = by_slot_[ev.enter[2 * i]], *b = by_slot_[ev.enter[2 * i + 1]];
            a->callback->OnEnterAOI(b);
        }
        for (uint32_t s : quarantine_) {
            AOI *a = by_slot_[s];
            if (a && !a->mgr && a->slot == s) {  // still out of every space: release
                a->slot = kNoSlot;
                by_slot_[s] = nullptr;
                free_.push_back(s);
            }
        }
        quarantine_.clear();
        return {ev.n_enter, ev.n_leave};
    }

    // Neighbour set as of the last flush (debug / parity).
    std::vector<AOI *> Neighbors(const AOI *aoi) {
        std::vector<AOI *> out;
        if (aoi->slot == kNoSlot || !aoi->mgr) return out;
        std::vector<uint32_t> buf(256);
        size_t n = 0;
        for (;;) {
            check(gwaoi_neighbors(w_, aoi->slot, buf.data(), buf.size(), &n));
            if (n <= buf.size()) break;
            buf.resize(n);
        }
        for (size_t i = 0; i < n; ++i) out.push_back(by_slot_[buf[i]]);
        return out;
    }

    gwaoi_world *handle() { return w_; }

  private:
    friend class XZListAOIManager;
    enum Kind : uint8_t { kMoved = 0, kEnter = 1, kLeave = 2 };

    void check(int rc) {
        if (rc != GWAOI_OK) {
            std::string m = gwaoi_strerror(rc);
            if (w_) {
                const char *l = gwaoi_last_error(w_);
                if (l && *l) m += std::string(" (") + l + ")";
            }
            throw Error(rc, m);
        }
    }
    void log(Kind k, uint32_t slot, Coord x, Coord z, uint32_t space) {
        kind_.push_back(k);
        slot_.push_back(slot);
        x_.push_back(x);
        z_.push_back(z);
        space_.push_back(space);
    }
    void submit() {  // runs of one kind (and one space for Enter) -> batch calls, in order
        const size_t n = kind_.size();
        for (size_t i = 0; i < n;) {
            size_t j = i + 1;
            while (j < n && kind_[j] == kind_[i] && (kind_[i] != kEnter || space_[j] == space_[i])) ++j;
            const size_t k = j - i;
            if (kind_[i] == kMoved)
                check(gwaoi_moved_batch(w_, &slot_[i], &x_[i], &z_[i], k));
            else if (kind_[i] == kEnter)
                check(gwaoi_enter_batch(w_, space_[i], &slot_[i], &x_[i], &z_[i], k));
            else
                check(gwaoi_leave_batch(w_, &slot_[i], k));
            i = j;
        }
        kind_.clear();
        slot_.clear();
        x_.clear();
        z_.clear();
        space_.clear();
    }

    gwaoi_world *w_ = nullptr;
    std::vector<AOI *> by_slot_;
    std::vector<uint32_t> free_, quarantine_;
    std::vector<uint8_t> kind_;
    std::vector<uint32_t> slot_, space_;
    std::vector<float> x_, z_;
};

// go-aoi XZListAOIManager for one space of a World.
class XZListAOIManager final : public AOIManager {
  public:
    XZListAOIManager(World *w, uint32_t space, Coord dist) : w_(w), space_(space), dist_(dist) {}
    ~XZListAOIManager() override { gwaoi_space_destroy(w_->w_, space_); }

    void Enter(AOI *aoi, Coord x, Coord y) override {  // Space.go:211,221
        if (aoi->mgr) throw Error(GWAOI_ESTATE, "Enter of an AOI that is already in a space");
        if (!std::isfinite(x) || !std::isfinite(y)) throw Error(GWAOI_ENONFINITE, "non-finite coordinate");
        if (aoi->slot == kNoSlot) {
            if (w_->free_.empty()) throw Error(GWAOI_EBADSLOT, "no free AOI slot");
            aoi->slot = w_->free_.back();
            w_->free_.pop_back();
            w_->by_slot_[aoi->slot] = aoi;
        }
        aoi->mgr = this;
        aoi->x = x;
        aoi->y = y;
        w_->log(World::kEnter, aoi->slot, x, y, space_);
    }
    void Leave(AOI *aoi) override {  // Space.go:243
        if (aoi->mgr != this) throw Error(GWAOI_ESTATE, "Leave of an AOI that is not in this space");
        aoi->mgr = nullptr;
        w_->log(World::kLeave, aoi->slot, 0.f, 0.f, space_);
        w_->quarantine_.push_back(aoi->slot);  // slot released after the flush replays its leaves
    }
    void Moved(AOI *aoi, Coord x, Coord y) override {  // Space.go:259
        if (aoi->mgr != this) throw Error(GWAOI_ESTATE, "Moved of an AOI that is not in this space");
        if (!std::isfinite(x) || !std::isfinite(y)) throw Error(GWAOI_ENONFINITE, "non-finite coordinate");
        aoi->x = x;
        aoi->y = y;
        w_->log(World::kMoved, aoi->slot, x, y, space_);
    }
    uint32_t space() const { return space_; }
    Coord dist() const { return dist_; }

  private:
    World *w_;
    uint32_t space_;
    Coord dist_;
};

inline std::unique_ptr<XZListAOIManager> World::NewXZListAOIManager(Coord dist) {
    if (!(dist > 0.f)) throw Error(GWAOI_EINVAL, "aoi distance must be > 0");  // Space.go:92
    uint32_t s = 0;
    check(gwaoi_space_create(w_, dist, &s));
    return std::make_unique<XZListAOIManager>(this, s, dist);
}

}  // namespace gwaoi

#endif
