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

}  // namespace mh
