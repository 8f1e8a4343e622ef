// mh_gunzip.h -- whole-buffer gunzip (mh_gunzip.cpp).
#pragma once
#include <stdint.h>

#include <string>

namespace mh {

// Decode a whole gzip buffer (all concatenated members) into `out`.
// 0 on success; -3 (or -2 out of memory) with `why` set otherwise.
int gunzip_buffer(const uint8_t *src, int64_t len, std::string &out, std::string &why);
// true when the libdeflate decoder is in use
bool gunzip_fast_available();
// One gzip member of src[0 .. len) at `level` (libdeflate when present);
// 0, or -2 when compression fails.
int gzip_member(const char *src, size_t len, std::string &out, int level);
// crc32 (zlib's polynomial; libdeflate's PCLMUL code when present)
uint32_t crc32_update(uint32_t crc, const void *p, size_t n);
// crc32 of A then B from crc32(A), crc32(B) and the length of B
uint32_t crc32_join(uint32_t a, uint32_t b, int64_t len_b);
// true when src[0 ..) starts with a plausible gzip member header (RFC 1952)
bool gzip_header_at(const uint8_t *src, int64_t avail);
// true when a gzip member starting at src decodes without error through
// its first `probe` output bytes (or to its end, CRC and size checked): the
// test a sharded reader uses to find a member boundary in compressed data
bool gzip_member_probe(const uint8_t *src, int64_t len, size_t probe);

}  // namespace mh
