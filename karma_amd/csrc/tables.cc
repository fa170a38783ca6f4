// karma_amd/csrc/tables.cc -- host builders of the kernels' table blobs (gf2.h).
#include "engine.h"
#include "gf2.h"

namespace karma {
namespace engine {

void build_stream_blob(uint32_t* out) {
    using gf2::Map;
    gf2::slicing_tables(Map::zero_bytes(kChunk), out + kBlobStride);
    gf2::slicing_tables(Map::zero_bytes(4), out + kBlobZ4);
    gf2::slicing_tables(Map::zero_bytes(16), out + kBlobZ16);
    gf2::slicing_tables(Map::zero_bytes(32), out + kBlobZ32);
    gf2::slicing_tables(Map::zero_bytes(64), out + kBlobZ64);
    gf2::byte_table(out + kBlobT8);
}

void build_lane_blob(uint32_t* out) {
    build_stream_blob(out);
    gf2::slicing_tables(gf2::Map::zero_bytes(16), out + kBlobStride);  // one lane's 4 word slots: stride 16
}

void build_quad_blob(uint32_t* out) {
    build_stream_blob(out);
    gf2::slicing_tables(gf2::Map::zero_bytes(64), out + kBlobStride);  // groups of 4 lanes: stride 64
}

void build_block_combine_blob(uint64_t unit_bytes, uint64_t per_thread, uint32_t* out) {
    using gf2::Map;
    gf2::slicing_tables(Map::zero_bytes(unit_bytes), out + kBcZD);
    Map m = Map::zero_bytes(unit_bytes * per_thread);
    for (int d = 0; d < 6; ++d) {
        gf2::slicing_tables(m, out + kBcTree + d * 1024);
        m = Map::compose(m, m);
    }
    gf2::slicing_tables(m, out + kBcWave);  // Z_{64 m D}
    gf2::slicing_tables(Map::zero_bytes(4), out + kBcZ4);
    gf2::byte_table(out + kBcT8);
}

void build_combine_blob(uint64_t unit_bytes, uint32_t* out) {
    using gf2::Map;
    Map m = Map::zero_bytes(unit_bytes);
    for (int k = 0; k < kCombMaps; ++k) {
        gf2::slicing_tables(m, out + k * 1024);
        m = Map::compose(m, m);  // Z_{D*2^(k+1)}
    }
    gf2::slicing_tables(Map::zero_bytes(4), out + kCombZ4);
    for (int i = 0; i < 1024; ++i) out[kCombT8 + i] = 0;
    gf2::byte_table(out + kCombT8);
    for (int i = 0; i < kCombSmallMaps; ++i) gf2::slicing_tables(Map::zero_bytes(16ull << i), out + kCombSmall + i * 1024);
    for (int i = 0; i < 4; ++i) gf2::slicing_tables(Map::inverse(Map::zero_bytes(1ull << i)), out + kCombInv + i * 1024);
}

}  // namespace engine
}  // namespace karma
