// mh_fastq.cpp -- staged FASTQ text for a sharded ingest (host code only).
//
// In a job of W ranks every rank must end up with the reads of its own
// contiguous block of FASTQ records without decoding the whole file.  The
// reference streams each file once per mapping pass (prelim_map.py:114-134,
// bowtie2 reading the FASTQ; censor_fastq.py:58-96 line by line); here a rank
// reads its 1/W share of the file:
//
//   * a gzip file of many members (as a parallel gzip, or this library's
//     censor, writes it): the members that start in the rank's byte range
//     [size * p / W, size * (p + 1) / W), the cuts moved to the nearest
//     member start (found by probing the header-shaped offsets either side:
//     a false one fails to decode), so the ranges of consecutive ranks meet
//     exactly;
//   * a plain file: the byte range itself;
//   * one gzip member (as bcl2fastq writes it; mh_fastq_scan_part finds no
//     member start in any rank's range): the deflate bits from the first
//     block start in the rank's share of the compressed bytes to the next
//     rank's (mh_fastq_member_*, mh_pinflate.cpp), decoded without the
//     window the rank before holds, which then arrives through the caller's
//     rank-order chain of 32 KiB messages (mode 3);
//   * anything else: the whole file (mode 0), and the rank keeps its records
//     by count.
//
// The text a rank holds then starts and ends mid-record.  mh_fastq_frame
// locates its record starts from the number of lines before it (a record is
// four lines); the caller moves the bytes before the first record start to
// the rank before (mh_fastq_splice), and exchanges whole records between
// ranks to align the mates of R1 and R2.  All of that exchange is the
// caller's (torch.distributed in micall_amd/ingest.py); this file only
// decodes, frames and splices host buffers.
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "mh_fastq.h"
#include "mh_gunzip.h"
#include "micall_hip.h"

namespace mh {
void set_error(const char *fmt, ...);
int s2a_threads();
}

using namespace mh;

namespace {

// a read-only view of a whole file (mmap, or read() for what cannot be mapped)
struct FileView {
    const uint8_t *p = nullptr;
    int64_t size = 0;
    void *map = nullptr;
    TextBuf copy;
    ~FileView() { if (map) munmap(map, (size_t)size); }
};

int view_file(const char *path, int fd_in, FileView &v)
{
    int fd = fd_in;
    if (path) {
        fd = open(path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) { set_error("cannot open FASTQ %s", path); return -3; }
    }
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) {
        if (path) close(fd);
        set_error("cannot stat FASTQ %s", path ? path : "(descriptor)");
        return -3;
    }
    v.size = (int64_t)st.st_size;
    int rc = 0;
    if (v.size > 0 && S_ISREG(st.st_mode)) {
        void *m = mmap(nullptr, (size_t)v.size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m != MAP_FAILED) {
            v.map = m;
            v.p = (const uint8_t *)m;
        }
    }
    if (!v.p && v.size > 0) {
        v.copy.resize((size_t)v.size);
        int64_t got = 0;
        while (got < v.size) {
            const ssize_t r = pread(fd, v.copy.data() + got, (size_t)(v.size - got), (off_t)got);
            if (r <= 0) { set_error("cannot read FASTQ %s", path ? path : "(descriptor)"); rc = -3; break; }
            got += r;
        }
        v.p = (const uint8_t *)v.copy.data();
    }
    if (path) close(fd);
    return rc;
}

// the first offset in [from, to) where a gzip member starts (probed), or
// v.size (to < 0: to the end of the file)
int64_t next_member(const FileView &v, int64_t from, int64_t to = -1)
{
    // candidates start before `to`; the probe may read on to the file's end
    const uint8_t *p = v.p + from, *e = v.p + (to < 0 ? v.size : std::min(to, v.size));
    const uint8_t *end = v.p + v.size;
    while (p < e) {
        p = (const uint8_t *)memchr(p, 0x1f, (size_t)(e - p));
        if (!p) break;
        if (gzip_header_at(p, end - p) && gzip_member_probe(p, end - p, 1 << 16)) return p - v.p;
        ++p;
    }
    return v.size;
}

// the last offset in [0, before) where a gzip member starts (probed); 0 if
// none is found (offset 0 starts the file's first member)
int64_t prev_member(const FileView &v, int64_t before)
{
    for (int64_t at = std::min(before, v.size) - 1; at > 0; --at) {
        const uint8_t *p = (const uint8_t *)memrchr(v.p, 0x1f, (size_t)at + 1);
        if (!p) break;
        at = p - v.p;
        if (at > 0 && gzip_header_at(p, v.size - at) && gzip_member_probe(p, v.size - at, 1 << 16))
            return at;
    }
    return 0;
}

// the member start nearest to x (the earlier one on a tie): the cut between
// parts, the same on both ranks that share it
int64_t cut_at(const FileView &v, int64_t x)
{
    const int64_t before = prev_member(v, x), after = next_member(v, x);
    return x - before <= after - x ? before : after;
}

double ms_since(std::chrono::steady_clock::time_point t)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

}  // namespace

struct mh_fastq {
    TextBuf data;                  // the held text
    std::vector<int64_t> rec;      // byte offsets of its record starts (mh_fastq_frame)
    bool framed = false;
    // one part of a single gzip member (mh_fastq_member_*): the file's view
    // and the part's decode state until mh_fastq_member_finish
    std::unique_ptr<FileView> view;
    MemberPart *member = nullptr;
    int part = 0, parts = 1;
    double member_ms = 0;
    ~mh_fastq() { if (member) member_part_free(member); }
};

namespace {

// newlines of d on host threads; info[3..6] of the open_part layout
void text_info(const TextBuf &d, int64_t *info)
{
    const int64_t n = (int64_t)d.size();
    const int nt = std::max(1, std::min(s2a_threads(), (int)(n >> 22) + 1));
    std::vector<int64_t> cnt(nt, 0);
    std::vector<std::thread> th;
    auto count = [&](int t) {
        const char *a = d.data() + n * t / nt, *b = d.data() + n * (t + 1) / nt;
        int64_t k = 0;
        while (a < b) {
            const char *q = (const char *)memchr(a, '\n', (size_t)(b - a));
            if (!q) break;
            ++k;
            a = q + 1;
        }
        cnt[t] = k;
    };
    try {
        for (int t = 1; t < nt; ++t) th.emplace_back(count, t);
    } catch (const std::system_error &) {   // no more threads: the rest run here
        for (int t = (int)th.size() + 1; t < nt; ++t) count(t);
    }
    count(0);
    for (auto &x : th) x.join();
    int64_t nl = 0;
    for (int64_t k : cnt) nl += k;
    info[3] = n;
    info[4] = nl;
    info[5] = n > 0 && d[n - 1] == '\n';
    info[6] = n > 0 && d[0] == '\n';
}

}  // namespace

extern "C" {

int mh_fastq_open_part(const char *path, int fd, int part, int parts, mh_fastq **out, int64_t *info)
{
    if (!out || !info || (!path && fd < 0) || parts < 1 || part < 0 || part >= parts) {
        set_error("mh_fastq_open_part: bad arguments");
        return -3;
    }
    *out = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        FileView v;
        if (int st = view_file(path, fd, v)) return st;
        std::unique_ptr<mh_fastq> fq(new mh_fastq());
        const bool gz = v.size >= 2 && v.p[0] == 0x1f && v.p[1] == 0x8b;
        int64_t mode = 0, c0 = 0, c1 = v.size;
        if (parts > 1 && !gz) {
            mode = 2;
            c0 = v.size * part / parts;
            c1 = v.size * (part + 1) / parts;
        } else if (parts > 1) {
            mode = 1;
            const int64_t lo = v.size * part / parts, hi = v.size * (part + 1) / parts;
            c0 = part == 0 ? 0 : cut_at(v, lo);
            c1 = part == parts - 1 ? v.size : std::max(c0, cut_at(v, hi));
            if (c0 >= c1) c0 = c1 = std::max(c0, c1);
        }
        std::string why;
        if (gz && c1 > c0) {
            if (gunzip_buffer(v.p + c0, c1 - c0, fq->data, why)) {
                set_error("gzip error reading %s: %s", path ? path : "(descriptor)", why.c_str());
                return -3;
            }
        } else if (c1 > c0) {
            fq->data.assign((const char *)v.p + c0, (size_t)(c1 - c0));
        }
        info[0] = mode;
        info[1] = c0;
        info[2] = c1;
        text_info(fq->data, info);
        info[7] = c1 - c0;
        info[8] = v.size;
        info[9] = (int64_t)(ms_since(t0) * 1000.0);   // microseconds
        *out = fq.release();
        return 0;
    } catch (const std::bad_alloc &) {
        set_error("mh_fastq_open_part: out of memory");
        return -2;
    } catch (const std::exception &e) {
        set_error("mh_fastq_open_part: %s", e.what());
        return -4;
    }
}

int mh_fastq_scan_part(const char *path, int fd, int part, int parts, int64_t *info)
{
    if (!info || (!path && fd < 0) || parts < 1 || part < 0 || part >= parts) {
        set_error("mh_fastq_scan_part: bad arguments");
        return -3;
    }
    try {
        FileView v;
        if (int st = view_file(path, fd, v)) return st;
        const bool gz = v.size >= 2 && v.p[0] == 0x1f && v.p[1] == 0x8b;
        const int64_t lo = v.size * part / parts, hi = v.size * (part + 1) / parts;
        info[0] = gz;
        info[1] = v.size;
        // a member start inside this part's byte range (past offset 0, the
        // file's first member): the scan covers 1/parts of the file
        info[2] = gz && hi > std::max<int64_t>(lo, 1) && next_member(v, std::max<int64_t>(lo, 1), hi) < hi;
        return 0;
    } catch (const std::bad_alloc &) {
        set_error("mh_fastq_scan_part: out of memory");
        return -2;
    } catch (const std::exception &e) {
        set_error("mh_fastq_scan_part: %s", e.what());
        return -4;
    }
}

int mh_fastq_member_open(const char *path, int fd, int part, int parts, mh_fastq **out, int64_t *info)
{
    if (!out || !info || (!path && fd < 0) || parts < 1 || part < 0 || part >= parts) {
        set_error("mh_fastq_member_open: bad arguments");
        return -3;
    }
    *out = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        std::unique_ptr<mh_fastq> fq(new mh_fastq());
        fq->view.reset(new FileView());
        if (int st = view_file(path, fd, *fq->view)) return st;
        const FileView &v = *fq->view;
        for (int k = 0; k < 5; ++k) info[k] = -1;
        info[5] = v.size;
        if (v.size >= 2 && v.p[0] == 0x1f && v.p[1] == 0x8b)
            fq->member = member_part_open(v.p, v.size, part, parts, s2a_threads(), info);
        if (!fq->member) info[0] = -1;
        fq->part = part;
        fq->parts = parts;
        fq->member_ms = ms_since(t0);
        info[6] = (int64_t)(fq->member_ms * 1000.0);
        *out = fq.release();
        return 0;
    } catch (const std::bad_alloc &) {
        set_error("mh_fastq_member_open: out of memory");
        return -2;
    } catch (const std::exception &e) {
        set_error("mh_fastq_member_open: %s", e.what());
        return -4;
    }
}

int mh_fastq_member_decode(mh_fastq *fq, int64_t end_bit, int64_t *info)
{
    if (!fq || !info || !fq->member) { set_error("mh_fastq_member_decode: bad arguments"); return -3; }
    const auto t0 = std::chrono::steady_clock::now();
    try {
        info[0] = -1;
        if (member_part_decode(fq->member, end_bit, fq->part > 0, s2a_threads()) == 0 &&
            member_part_place(fq->member, fq->data, s2a_threads()) == 0)
            info[0] = (int64_t)fq->data.size();
        fq->member_ms += ms_since(t0);
        info[1] = (int64_t)(ms_since(t0) * 1000.0);
        return 0;
    } catch (const std::bad_alloc &) {
        set_error("mh_fastq_member_decode: out of memory");
        return -2;
    } catch (const std::exception &e) {
        set_error("mh_fastq_member_decode: %s", e.what());
        return -4;
    }
}

int mh_fastq_member_tail(mh_fastq *fq, const char *window, char *tail)
{
    if (!fq || !tail || !fq->member || (fq->part > 0 && !window)) {
        set_error("mh_fastq_member_tail: bad arguments");
        return -3;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const int st = member_part_tail(fq->member, fq->data, window, tail);
    fq->member_ms += ms_since(t0);
    if (st) { set_error("mh_fastq_member_tail: the window does not resolve this part"); return -1; }
    return 0;
}

int mh_fastq_member_finish(mh_fastq *fq, const char *window, int64_t c0, int64_t c1, int64_t *info)
{
    if (!fq || !info || !fq->member || (fq->part > 0 && !window)) {
        set_error("mh_fastq_member_finish: bad arguments");
        return -3;
    }
    const auto t0 = std::chrono::steady_clock::now();
    try {
        uint32_t crc = 0;
        const int st = member_part_finish(fq->member, fq->data, window, s2a_threads(), &crc);
        member_part_free(fq->member);
        fq->member = nullptr;
        const int64_t size = fq->view ? fq->view->size : 0;
        fq->view.reset();
        if (st) { set_error("mh_fastq_member_finish: the window does not resolve this part"); return -1; }
        info[0] = 3;
        info[1] = c0;
        info[2] = c1;
        text_info(fq->data, info);
        info[7] = c1 - c0;
        info[8] = size;
        fq->member_ms += ms_since(t0);
        info[9] = (int64_t)(fq->member_ms * 1000.0);
        info[10] = crc;
        return 0;
    } catch (const std::bad_alloc &) {
        set_error("mh_fastq_member_finish: out of memory");
        return -2;
    } catch (const std::exception &e) {
        set_error("mh_fastq_member_finish: %s", e.what());
        return -4;
    }
}

int mh_fastq_frame(mh_fastq *fq, int64_t line0, int starts_line, int64_t *out)
{
    if (!fq || !out || line0 < 0) { set_error("mh_fastq_frame: bad arguments"); return -3; }
    try {
        const TextBuf &d = fq->data;
        const int64_t n = (int64_t)d.size();
        fq->rec.clear();
        int64_t first_line = -1;
        int64_t blank = 0, tail_cr = 0;
        // line starts: offset 0 when the text starts a line (its index is
        // line0), else the first byte continues line line0 and the next line
        // (line0 + 1) starts after the first '\n'
        int64_t at = 0, line = line0;
        if (!starts_line) {
            const char *q = (const char *)memchr(d.data(), '\n', (size_t)n);
            at = q ? (q - d.data()) + 1 : n;
            line = line0 + 1;
        }
        while (at < n) {
            const char *q = (const char *)memchr(d.data() + at, '\n', (size_t)(n - at));
            const int64_t end = q ? q - d.data() : n;
            if ((line & 3) == 0) {
                if (first_line < 0) first_line = line;
                fq->rec.push_back(at);
                int64_t e = end;
                if (e > at && d[e - 1] == '\r') --e;
                if (q && e == at) blank = 1;          // a blank line where a record starts
                if (!q && end - at == 1 && d[at] == '\r') tail_cr = 1;
            }
            at = end + 1;
            ++line;
        }
        fq->framed = true;
        out[0] = fq->rec.empty() ? n : fq->rec[0];
        out[1] = (int64_t)fq->rec.size();
        out[2] = first_line;
        out[3] = blank;
        out[4] = tail_cr;
        return 0;
    } catch (const std::bad_alloc &) {
        set_error("mh_fastq_frame: out of memory");
        return -2;
    }
}

int mh_fastq_record_offset(mh_fastq *fq, int64_t k, int64_t *off)
{
    if (!fq || !off || !fq->framed || k < 0 || k > (int64_t)fq->rec.size()) {
        set_error("mh_fastq_record_offset: bad arguments");
        return -3;
    }
    *off = k == (int64_t)fq->rec.size() ? (int64_t)fq->data.size() : fq->rec[k];
    return 0;
}

int mh_fastq_splice(mh_fastq *fq, int64_t lo, int64_t hi, const char *front, int64_t flen,
                    const char *back, int64_t blen)
{
    if (!fq || lo < 0 || hi < lo || hi > (int64_t)fq->data.size() || flen < 0 || blen < 0 ||
        (flen && !front) || (blen && !back)) {
        set_error("mh_fastq_splice: bad arguments");
        return -3;
    }
    try {
        TextBuf &d = fq->data;
        if (flen == 0) {
            if (lo > 0) memmove(d.data(), d.data() + lo, (size_t)(hi - lo));
            d.resize((size_t)(hi - lo));
        } else {
            TextBuf t;
            t.reserve((size_t)(flen + (hi - lo) + blen));
            t.append(front, (size_t)flen);
            t.append(d.data() + lo, (size_t)(hi - lo));
            d.swap(t);
        }
        if (blen) d.append(back, (size_t)blen);
        fq->rec.clear();
        fq->framed = false;
        return 0;
    } catch (const std::bad_alloc &) {
        set_error("mh_fastq_splice: out of memory");
        return -2;
    }
}

int mh_fastq_view(mh_fastq *fq, const char **data, int64_t *len)
{
    if (!fq || !data || !len) return -3;
    *data = fq->data.data();
    *len = (int64_t)fq->data.size();
    return 0;
}

int mh_fastq_close(mh_fastq *fq)
{
    delete fq;
    return 0;
}

}  // extern "C"

namespace mh {

const TextBuf &fastq_text(const mh_fastq *fq) { return fq->data; }

TextBuf take_fastq_text(mh_fastq *fq)
{
    TextBuf out;
    out.swap(fq->data);
    fq->rec.clear();
    fq->framed = false;
    return out;
}

}  // namespace mh
