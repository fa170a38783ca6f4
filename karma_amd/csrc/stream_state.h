// karma_amd/csrc/stream_state.h -- the C ABI's per-(device, stream) state and its lifetime
// (karma_crc32c_release_stream / _trim / _graph_hold, include/karma_crc32c.h).
//
// A batch call keeps, per device and stream, what its launches point at: the workspace (unit
// plan, combine levels, byte grid), the ragged plan's look-back words and the single-record
// combine's tagged words.  They are allocated by the first call that needs them and grown by
// later ones.  A buffer a stream outgrows is freed once the stream has drained -- unless a
// hipGraph was ever captured on that stream: its kernel arguments may point into the old buffer,
// so the buffer is kept (retired) until the caller trims with no graph hold.
//
// Templated on the operations it issues (Ops: alloc / free / zero / sync_stream / sync_device /
// capturing) so that tests/cpp/host_logic_test.cc drives the bookkeeping under ASan through a
// recording stub, as gather_p2p.h is tested; capi.cc instantiates it with the HIP calls.
// Not thread-safe: the caller holds the library lock.
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>
#include <utility>
#include <vector>

namespace karma::engine {

template <class Ops>
class StreamStates {
  public:
    struct Buf {
        void* p = nullptr;
        size_t bytes = 0;
    };
    struct State {
        void* stream = nullptr;      // the handle the calls were made on
        Buf ws;                      // workspace
        Buf lb;                      // look-back words (zeroed when allocated)
        Buf fused;                   // fused-combine words (zeroed when allocated)
        std::vector<void*> retired;  // outgrown buffers a captured graph may still use
        bool captured = false;       // a capture was seen on this stream
    };

    explicit StreamStates(Ops ops = Ops()) : ops_(ops) {}

    // The state of (dev, key), created empty on first use; notes a capture in progress.
    State& get(int dev, uintptr_t key, void* stream) {
        State& s = states_[{dev, key}];
        s.stream = stream;
        if (ops_.capturing(stream)) s.captured = true;
        return s;
    }

    // b grown to at least `need` bytes (allocating `alloc` >= need; zeroed on `stream` when
    // `zero`).  *fresh: a new buffer.  The old one is freed after the stream drains, or retired
    // when the stream was captured (a graph may hold its address).
    int grow(State& s, Buf& b, size_t need, size_t alloc, bool zero, bool* fresh = nullptr) {
        if (fresh) *fresh = false;
        if (b.p && b.bytes >= need) return 0;
        if (b.p) {
            if (s.captured) {
                s.retired.push_back(b.p);
            } else {
                if (const int rc = ops_.sync_stream(s.stream)) return rc;
                ops_.free(b.p);
            }
            b.p = nullptr;
            b.bytes = 0;
        }
        if (const int rc = ops_.alloc(&b.p, alloc)) {
            b.p = nullptr;
            return rc;
        }
        b.bytes = alloc;
        if (zero)
            if (const int rc = ops_.zero(b.p, alloc, s.stream)) return rc;
        if (fresh) *fresh = true;
        return 0;
    }

    // Waits for the stream and frees everything (dev, key) holds.  Absent: nothing to do.
    int release(int dev, uintptr_t key) {
        auto it = states_.find({dev, key});
        if (it == states_.end()) return 0;
        if (const int rc = ops_.sync_stream(it->second.stream)) return rc;
        free_state(it->second);
        states_.erase(it);
        return 0;
    }

    // The per-thread state of an exited thread (its stream is gone): moved aside whole, freed by
    // the next trim after the device has drained.
    void orphan(uintptr_t key) {
        for (auto it = states_.begin(); it != states_.end();) {
            if (it->first.second == key) {
                zombies_.push_back({it->first.first, std::move(it->second)});
                it = states_.erase(it);
            } else {
                ++it;
            }
        }
    }

    // Waits for the device, then frees what no live stream holds: the orphaned states, and --
    // unless a graph hold is active -- every retired buffer.  An orphaned state that saw a capture
    // is kept while a hold is active too (a graph captured on hipStreamPerThread by a thread that
    // has exited still points into it).
    int trim(int dev) {
        if (const int rc = ops_.sync_device(dev)) return rc;
        const bool held = holds(dev) > 0;
        for (auto it = zombies_.begin(); it != zombies_.end();) {
            if (it->first == dev && !(held && it->second.captured)) {
                free_state(it->second);
                it = zombies_.erase(it);
            } else {
                ++it;
            }
        }
        if (held) return 0;
        for (auto& kv : states_) {
            if (kv.first.first != dev) continue;
            for (void* p : kv.second.retired) ops_.free(p);
            kv.second.retired.clear();
        }
        return 0;
    }

    // Graphs a caller keeps on dev (retired buffers survive trim while > 0); returns the count.
    int hold(int dev, int delta) {
        int& h = holds_[dev];
        h += delta;
        if (h < 0) h = 0;
        return h;
    }
    int holds(int dev) const {
        auto it = holds_.find(dev);
        return it == holds_.end() ? 0 : it->second;
    }

    size_t states() const { return states_.size(); }
    size_t zombies() const { return zombies_.size(); }

  private:
    void free_state(State& s) {
        for (Buf* b : {&s.ws, &s.lb, &s.fused})
            if (b->p) ops_.free(b->p);
        for (void* p : s.retired) ops_.free(p);
        s = State{};
    }

    Ops ops_;
    std::map<std::pair<int, uintptr_t>, State> states_;
    std::vector<std::pair<int, State>> zombies_;
    std::map<int, int> holds_;
};

}  // namespace karma::engine
