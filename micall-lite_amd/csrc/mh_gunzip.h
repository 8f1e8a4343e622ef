// mh_gunzip.h -- whole-buffer gunzip (mh_gunzip.cpp).
#pragma once
#include <stdint.h>

#include <string.h>

#include <algorithm>
#include <memory>
#include <string>

namespace mh {

// Large host buffers: anonymous mappings with transparent huge pages asked
// for (the box's THP mode is "madvise"), so filling and freeing a GB-sized
// text faults and frees 2 MiB pages instead of half a million 4 KiB ones.
// Small ones come from the heap.  Contents are not initialised.
char *big_alloc(size_t n);
void big_free(char *p, size_t n);

struct BigDeleter {
    size_t n = 0;
    void operator()(char *p) const { big_free(p, n); }
};

// A growable byte buffer whose new bytes are not zero-filled (a GB-sized
// std::string::resize is a serial memset before the threads that fill it
// can start; here the pages are first touched by the threads that write
// them).
class TextBuf {
  public:
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    char *data() { return p_.get(); }
    const char *data() const { return p_.get(); }
    char &operator[](size_t i) { return p_[i]; }
    const char &operator[](size_t i) const { return p_[i]; }
    void reserve(size_t k)
    {
        if (k <= cap_) return;
        std::unique_ptr<char[], BigDeleter> q(big_alloc(k), BigDeleter{k});
        if (n_) memcpy(q.get(), p_.get(), n_);
        p_.swap(q);
        cap_ = k;
    }
    void resize(size_t k)   // new bytes are left uninitialised
    {
        if (k > cap_) reserve(std::max(k, cap_ + cap_ / 2));
        n_ = k;
    }
    void append(const char *s, size_t k)
    {
        const size_t at = n_;
        resize(n_ + k);
        if (k) memcpy(p_.get() + at, s, k);
    }
    void assign(const char *s, size_t k) { n_ = 0; append(s, k); }
    void clear() { n_ = 0; }
    void release() { p_.reset(); n_ = cap_ = 0; }
    void swap(TextBuf &o) { p_.swap(o.p_); std::swap(n_, o.n_); std::swap(cap_, o.cap_); }

  private:
    std::unique_ptr<char[], BigDeleter> p_{nullptr, BigDeleter{}};
    size_t n_ = 0, cap_ = 0;
};

// Decode a whole gzip buffer (all concatenated members) into `out`.
// 0 on success; -3 (or -2 out of memory) with `why` set otherwise.
int gunzip_buffer(const uint8_t *src, int64_t len, std::string &out, std::string &why);
int gunzip_buffer(const uint8_t *src, int64_t len, TextBuf &out, std::string &why);
// true when the libdeflate decoder is in use
bool gunzip_fast_available();
// One gzip member of src[0 .. len) at `level` (libdeflate when present);
// 0, or -2 when compression fails.
int gzip_member(const char *src, size_t len, std::string &out, int level);
int gzip_member(const char *src, size_t len, TextBuf &out, int level);
// The whole regular file fd mapped read-only for a native parser: 0, 1
// when it holds '\r' (a text-mode read would translate it: the caller reads
// it itself; nothing stays mapped), or -3 (error set).  The '\r' scan runs
// on many threads, which also faults the mapping in in parallel.
int map_text_file(int fd, const char **text, size_t *len);
void unmap_text_file(const char *text, size_t len);

// One gzip member (the whole of src) inflated by `threads` host threads
// (mh_pinflate.cpp); -1 when it cannot be (the caller inflates serially).
template <class Buf>
int gunzip_single_parallel(const uint8_t *src, int64_t len, Buf &out, int threads);
// One part of one gzip member for a job of `parts` ranks (mh_pinflate.cpp):
// open finds the part's span starts (info: [0] its first block start bit or
// -1, [1] the deflate stream's end bit, [2] trailer CRC-32, [3] trailer size,
// [4] spans); decode inflates them up to end_bit (the next part's first
// start, or the stream's end), span 0 with an unknown window unless part 0;
// place lays the text out in `out` (window-derived bytes symbolic); tail
// resolves the last 32 KiB from the window (the previous part's last 32 KiB;
// NULL for part 0) and copies them out; finish resolves the rest and gives
// the CRC-32 of the part's text.  Each returns 0 or -1 (not decodable this
// way: the caller falls back).
struct MemberPart;
MemberPart *member_part_open(const uint8_t *src, int64_t len, int part, int parts, int threads,
                             int64_t *info);
int member_part_decode(MemberPart *m, int64_t end_bit, bool windowed, int threads);
template <class Buf>
int member_part_place(MemberPart *m, Buf &out, int threads);
template <class Buf>
int member_part_tail(MemberPart *m, Buf &out, const char *window, char *tail);
template <class Buf>
int member_part_finish(MemberPart *m, Buf &out, const char *window, int threads, uint32_t *crc);
void member_part_free(MemberPart *m);
// Raw DEFLATE (RFC 1951) through libdeflate: ld_raw_alloc() is nullptr when
// libdeflate is absent.  ld_raw_inflate decodes in[0 .. n) up to the end of
// its final block: 0 (*in_used, *out_used set), 1 bad data, 3 out of space.
void *ld_raw_alloc();
void ld_raw_free(void *d);
int ld_raw_inflate(void *d, const uint8_t *in, size_t n, char *out, size_t cap, size_t *in_used,
                   size_t *out_used);
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
