// karma_amd/csrc/host_trace.h -- opt-in phase timing of the host-side batch
// layers (KARMA_TRACE_HOST=1 prints "phase: ms" lines to stderr).  Off by default.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace karma::engine {

inline bool host_trace_on() {
    static const bool on = std::getenv("KARMA_TRACE_HOST") != nullptr;
    return on;
}

struct PhaseTimer {
    const char* scope;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    explicit PhaseTimer(const char* s) : scope(s) {}
    void mark(const char* phase) {
        if (!host_trace_on()) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[karma %s] %s: %.3f ms\n", scope, phase,
                     std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

}  // namespace karma::engine
