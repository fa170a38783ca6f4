// include/karma-util/crc32c.h
//
// Drop-in surface for Karma's WAL checksum (reference interface:
// /root/reference/karma-util/crc32c.h:11-39).  Karma's callers
//   karma-store/segment_file.cc:22      crc32c::Value   (WAL append)
//   karma-store/wal.cc:60               crc32c::Value   (WAL replay check)
//   karma-transport/frame.cc:56-57,119  crc32c::Value + crc32c::Extend (KFP frames)
// compile and link unchanged when this directory is first on the include
// path and libkarma_crc32c.so replaces karma-util/crc32c.cc.  The guard macro
// matches the reference so a stray include of the old header is a no-op.
//
// Extend() runs on the host (karma_amd/csrc/host_crc32c.cc): one record per
// call, synchronous, like the reference.  Batches of records are checksummed
// on MI355X through the C ABI in include/karma_crc32c.h.
#ifndef STORAGE_LEVELDB_UTIL_CRC32C_H_
#define STORAGE_LEVELDB_UTIL_CRC32C_H_

#include <cstddef>
#include <cstdint>

namespace crc32c {

// CRC-32C (Castagnoli) of A || data[0, n) given init_crc = CRC-32C of A.
// Total: no exceptions, no status; data may be nullptr when n == 0.
uint32_t Extend(uint32_t init_crc, const char* data, size_t n);

// CRC-32C of data[0, n)  ==  Extend(0, data, n).
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

// Masking for CRCs stored next to the data they cover (LevelDB convention).
static const uint32_t kMaskDelta = 0xa282ead8ul;

namespace detail {
inline uint32_t rotr32(uint32_t v, unsigned s) { return (v >> s) | (v << (32u - s)); }
}  // namespace detail

inline uint32_t Mask(uint32_t crc) { return detail::rotr32(crc, 15) + kMaskDelta; }

inline uint32_t Unmask(uint32_t masked_crc) { return detail::rotr32(masked_crc - kMaskDelta, 17); }

}  // namespace crc32c

#endif  // STORAGE_LEVELDB_UTIL_CRC32C_H_
