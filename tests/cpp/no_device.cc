// tests/cpp/no_device.cc -- link stand-ins for the device launchers (test infrastructure).
//
// The sanitizer build of the host side (karma_amd/csrc/Makefile `san`) links the library's
// host objects without the gfx950 kernels (hipcc objects carry device code that ASan does
// not instrument and that this container cannot run).  Every entry point checks for a device
// before it launches anything, so on a machine without a GPU none of these is reached; if
// one were, it refuses like a missing device.
#include <hip/hip_runtime_api.h>

#include "engine.h"

namespace karma::engine {

hipError_t launch_fixed(const FixedArgs&, int, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_segment_once(const FixedArgs&, int, hipStream_t, bool) { return hipErrorNoDevice; }
hipError_t launch_combine_fixed(const FixedArgs&, const uint32_t*, uint64_t, uint32_t*, uint64_t, const uint32_t*,
                                hipStream_t) {
    return hipErrorNoDevice;
}
hipError_t launch_combine_block(const FixedArgs&, const uint32_t*, uint64_t, uint64_t, const uint32_t*, hipStream_t) {
    return hipErrorNoDevice;
}
hipError_t launch_ragged_scan(const RaggedArgs&, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_ragged_main(const RaggedArgs&, int, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_ragged_direct(const RaggedArgs&, int, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_wal_walk(const WalArgs&, uint64_t, const WalWalkPlan&, hipStream_t, bool) { return hipErrorNoDevice; }
hipError_t launch_ragged_direct_dev(const RaggedArgs&, int, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_ragged_staged_dev(const RaggedArgs&, int, hipStream_t, bool) { return hipErrorNoDevice; }
hipError_t launch_wal_plan(const WalArgs&, uint64_t, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_wal_gather(const WalArgs&, uint64_t, bool, int, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_wal_resolve_gather(const WalArgs&, uint64_t, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_wal_compare(const WalArgs&, uint64_t, int, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_wal_publish(const WalSummary*, WalSummary*, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_ragged_staged_spec(const RaggedArgs&, int, hipStream_t, bool) { return hipErrorNoDevice; }
hipError_t launch_ragged_direct_spec(const RaggedArgs&, int, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_fill_splitmix(uint8_t*, uint64_t, uint64_t, uint64_t, hipStream_t) { return hipErrorNoDevice; }
hipError_t launch_stream_probe(const uint8_t*, uint64_t, uint32_t*, int, hipStream_t) { return hipErrorNoDevice; }

}  // namespace karma::engine
