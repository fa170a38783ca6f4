// tests/cpp/dropin_test.cc -- the drop-in boundary, exercised the way Karma's callers use it.
//
// Built by tests/test_host.py with g++ against include/karma-util/crc32c.h and linked against
// libkarma_crc32c.so (not against karma-util/crc32c.cc).  The three call patterns are restated
// from the reference callers:
//   WAL append   karma-store/segment_file.cc:21-31  [crc = Value(payload)][len<<8|type][payload]
//   WAL footer   karma-store/segment_file.cc:33-49  type-1 padding record, crc field 0
//   WAL replay   karma-store/wal.cc:34-87           DecodeFixed32(stored) vs Value(payload)
//   KFP frames   karma-transport/frame.cc:56-57, 119-122  Extend(Value(header), payload)
// and the transport test's contracts (test/test-karma-transport/transport_test.cc:29-59):
// round trip, trailing garbage tolerated, a flipped CRC byte is detected.
#include <cassert>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "karma-util/crc32c.h"

namespace {

void put_fixed32(std::string* dst, uint32_t v) {
    char b[4] = {char(v), char(v >> 8), char(v >> 16), char(v >> 24)};
    dst->append(b, 4);
}

uint32_t decode_fixed32(const char* p) {
    const unsigned char* u = reinterpret_cast<const unsigned char*>(p);
    return uint32_t(u[0]) | uint32_t(u[1]) << 8 | uint32_t(u[2]) << 16 | uint32_t(u[3]) << 24;
}

// segment_file::append_record framing
void append_record(std::string* seg, const std::string& payload) {
    put_fixed32(seg, crc32c::Value(payload.data(), payload.size()));
    put_fixed32(seg, uint32_t(payload.size()) << 8 | 0u);
    seg->append(payload);
}

// segment_file::append_footer: pad to seg_size with a type-1 record (crc 0)
void append_footer(std::string* seg, size_t seg_size) {
    if (seg_size - seg->size() < 8) {
        seg->append(seg_size - seg->size(), '0');
        return;
    }
    size_t pad = seg_size - seg->size() - 8;
    put_fixed32(seg, 0);
    put_fixed32(seg, uint32_t(pad) << 8 | 1u);
    seg->append(pad, '0');
}

// wal::scan_record replay loop: returns records verified, -1 on "Corrupt record"
long replay(const std::string& seg) {
    size_t pos = 0;
    long n = 0;
    while (pos + 8 <= seg.size()) {
        uint32_t crc = decode_fixed32(seg.data() + pos);
        uint32_t st = decode_fixed32(seg.data() + pos + 4);
        uint32_t type = st & 0xffu, size = st >> 8;
        if (type == 1) break;
        if (pos + 8 + size > seg.size()) return -1;
        if (crc32c::Value(seg.data() + pos + 8, size) != crc) return -1;
        pos += 8 + size;
        ++n;
    }
    return n;
}

// frame::encode / frame::parse CRC chain
std::string encode_frame(const std::string& header, const std::string& body) {
    std::string f = header + body;
    uint32_t crc = crc32c::Extend(crc32c::Value(header.data(), header.size()), body.data(), body.size());
    put_fixed32(&f, crc);
    return f;
}

bool parse_frame(const std::string& f, size_t header_len, size_t body_len) {
    if (f.size() < header_len + body_len + 4) return false;
    uint32_t stored = decode_fixed32(f.data() + header_len + body_len);
    uint32_t crc = crc32c::Extend(crc32c::Value(f.data(), header_len), f.data() + header_len, body_len);
    return crc == stored;
}

}  // namespace

int main() {
    // known answers through the drop-in symbol
    assert(crc32c::Value("123456789", 9) == 0xE3069283u);
    assert(crc32c::Value(nullptr, 0) == 0u);
    assert(crc32c::Extend(0xDEADBEEFu, nullptr, 0) == 0xDEADBEEFu);
    assert(crc32c::Extend(crc32c::Value("hello ", 6), "world", 5) == crc32c::Value("hello world", 11));
    assert(crc32c::Mask(0xE3069283u) == 0xC78AB0E5u);
    assert(crc32c::Unmask(crc32c::Mask(0x12345678u)) == 0x12345678u);
    assert(crc32c::kMaskDelta == 0xa282ead8ul);

    // WAL append -> replay over a 1 MiB segment of ~180-byte records (sivir_benchmark.cc intent)
    std::string seg;
    const size_t seg_size = 1 << 20;
    uint64_t x = 42;
    long appended = 0;
    while (true) {
        std::string payload(176 + (x % 5), 'a');
        for (auto& c : payload) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            c = char('a' + (x >> 59) % 26);
        }
        if (seg.size() + 8 + payload.size() + 8 > seg_size) break;
        append_record(&seg, payload);
        ++appended;
    }
    append_footer(&seg, seg_size);
    assert(seg.size() == seg_size);
    assert(replay(seg) == appended);
    // a flipped payload byte is a "Corrupt record" (wal.cc:62-65)
    std::string bad = seg;
    bad[8 + 100] ^= 0x01;
    assert(replay(bad) == -1);

    // KFP frames (transport_test.cc:29-59)
    std::string header = "I am header", body = "I am body";
    std::string f = encode_frame(header, body);
    assert(parse_frame(f, header.size(), body.size()));
    assert(parse_frame(f + "I am an random string", header.size(), body.size()));
    std::string g = f;
    g.back() = 'F';
    assert(!parse_frame(g, header.size(), body.size()));

    std::printf("dropin_test: ok (%ld WAL records, frames, KATs)\n", appended);
    return 0;
}
