// karma_amd/csrc/ab.h -- build-time A/B knobs.
//
// The shipped library (karma_amd/lib/libkarma_crc32c.so) is built WITHOUT
// KARMA_AB: it holds one kernel per plan shape, never reads the environment on
// a launch path, and every knob below is its compile-time default.  The tools
// build (tools/lib/libkarma_crc32c_ab.so, `make -C karma_amd/csrc ab`, linked
// only by tools/ and by the variant tests) adds the alternative kernels of
// DESIGN.md §4's measurements, selected per call from KARMA_* variables so one
// process can interleave them.  Some of those alternatives are timing
// experiments whose CRCs are wrong by design (KARMA_CRC_VARIANT=6); they exist
// only in that build.
#pragma once

#ifdef KARMA_AB
#include <cstdlib>
namespace karma::engine {
inline long ab_knob(const char* name, long dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::atol(e) : dflt;
}
}  // namespace karma::engine
#define KARMA_AB_KNOB(name, dflt) ::karma::engine::ab_knob(name, dflt)
#else
#define KARMA_AB_KNOB(name, dflt) (dflt)
#endif
