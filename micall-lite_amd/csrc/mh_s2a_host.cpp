// mh_s2a_host.cpp -- host half of the sam2aln stage (see mh_sam2aln.hip):
//   s2a_parse   remap.csv as csv.DictReader reads it (sam2aln.py:298), in
//               parallel chunks split at record boundaries; matchmaker
//               (:291-312); parse_sam's row-level causes (:340-348) and the
//               apply_cigar checks that raise (:113-151)
//   s2a_format  aligned.csv (:459-478), insert.csv (:357-380, :446-447),
//               failed.csv (:387-389, :449-450) as DictWriter writes them
// Threads: min(16, hardware threads, OMP_NUM_THREADS); output is identical
// for any thread count.
#include <algorithm>
#include <memory>
#include <cerrno>
#include <unistd.h>
#include <atomic>
#include <charconv>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mh_sam2aln.h"
#include "mh_text.h"

namespace mh {

static const char *const S2A_CAUSE[] = {"", "unmatched", "badCigar", "2refs", "manyNs", ""};

int s2a_threads()
{
    int n = (int)std::thread::hardware_concurrency();
    if (const char *e = getenv("OMP_NUM_THREADS")) {
        const int v = atoi(e);
        if (v > 0 && v < n) n = v;
    }
    if (n < 1) n = 1;
    return n > 16 ? 16 : n;
}

// fn(t) on nt threads; the first exception a worker throws (an allocation
// failure) is rethrown here once every worker has ended
static void parallel_for(int nt, const std::function<void(int)> &fn)
{
    if (nt <= 1) { fn(0); return; }
    std::exception_ptr err;
    std::mutex mu;
    auto guarded = [&](int t) {
        try {
            fn(t);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    try {
        for (int t = 1; t < nt; ++t) th.emplace_back(guarded, t);
    } catch (const std::system_error &) {   // no more threads: the rest run here
        for (int t = (int)th.size() + 1; t < nt; ++t) guarded(t);
    }
    guarded(0);
    for (auto &x : th) x.join();
    if (err) std::rethrow_exception(err);
}

struct FieldRef {
    const char *p;
    size_t n;
};

constexpr int MAXCOLS = 64;

// one CSV record as views (quoted fields unescaped into scratch[k]); same
// dialect as csv_record (mh_text.h)
static bool record_views(const char *&p, const char *end, std::vector<FieldRef> &f,
                         std::vector<std::string> &scratch)
{
    f.clear();
    if (p >= end) return false;
    for (size_t k = 0;; ++k) {
        if (k >= (size_t)MAXCOLS) return false;
        if (p < end && *p == '"') {
            std::string &s = scratch[k];
            s.clear();
            ++p;
            while (p < end) {
                if (*p == '"') {
                    if (p + 1 < end && p[1] == '"') { s.push_back('"'); p += 2; continue; }
                    ++p;
                    break;
                }
                s.push_back(*p++);
            }
            while (p < end && *p != ',' && *p != '\n' && *p != '\r') s.push_back(*p++);
            f.push_back({s.data(), s.size()});
        } else {
            const char *q = p;
            while (p < end && *p != ',' && *p != '\n' && *p != '\r') ++p;
            f.push_back({q, (size_t)(p - q)});
        }
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == '\r') ++p;
        if (p < end && *p == '\n') ++p;
        return true;
    }
}

// Python int() on a CSV field: optional surrounding whitespace and sign
static bool py_int(const FieldRef &f, int32_t &v)
{
    const char *a = f.p, *b = f.p + f.n;
    while (a < b && (*a == ' ' || *a == '\t')) ++a;
    while (b > a && (b[-1] == ' ' || b[-1] == '\t')) --b;
    if (a < b && *a == '+') ++a;
    if (a == b) return false;
    long long x = 0;
    auto r = std::from_chars(a, b, x);
    if (r.ec != std::errc() || r.ptr != b || x < INT32_MIN || x > INT32_MAX) return false;
    v = (int32_t)x;
    return true;
}

static uint64_t hash_bytes(const char *p, size_t n)
{
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) { h ^= (uint8_t)p[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

// CIGAR -> ops + apply_cigar's verdict for a read of length L
static int8_t cigar_ops(const char *c, size_t n, int64_t L, std::vector<uint32_t> &ops)
{
    ops.clear();
    if (n == 1 && c[0] == '*') return CIG_STAR;
    for (size_t i = 0; i < n;) {
        size_t j = i;
        while (j < n && c[j] >= '0' && c[j] <= '9') ++j;
        if (j == i || j >= n || !strchr("MIDNSHPX=", c[j]) || c[j] == '\0') return CIG_INVALID;
        i = j + 1;
    }
    int64_t left = 0;
    for (size_t i = 0; i < n;) {
        uint64_t v = 0;
        size_t j = i;
        while (c[j] >= '0' && c[j] <= '9') { v = v * 10 + (uint64_t)(c[j] - '0'); ++j; }
        uint32_t code;
        switch (c[j]) {
        case 'M': code = MH_OP_M; left += (int64_t)v; break;
        case 'I': code = MH_OP_I; left += (int64_t)v; break;
        case 'S': code = MH_OP_S; left += (int64_t)v; break;
        case 'D': code = MH_OP_D; break;
        default: return CIG_UNSUPPORTED;
        }
        if (left > L) return CIG_LONG;
        ops.push_back(((uint32_t)v << 4) | code);
        i = j + 1;
    }
    return left < L ? CIG_SHORT : CIG_OK;
}

struct Part {
    const char *beg = nullptr, *end = nullptr;
    int64_t rows = 0;
    TextBuf qpool, cpool, seq, qual;
    std::vector<int64_t> qoff, coff, soff;
    std::vector<int32_t> qlen, clen, slen, flag, pos, cig_off, n_cig, rid;
    std::vector<uint64_t> qhash;
    std::vector<int8_t> cstate;
    std::vector<uint8_t> qshort;
    std::vector<uint32_t> cig;
    std::vector<std::string> rnames;
    int err = 0;
    int64_t err_row = 0;
    std::string err_msg;
};

static void parse_part(Part &P, const int *col)
{
    std::vector<FieldRef> f;
    std::vector<std::string> scratch(MAXCOLS);
    std::unordered_map<std::string, int> rmap;
    std::vector<uint32_t> ops;
    const char *p = P.beg;
    int need = 0;
    for (int k = 0; k < 11; ++k) need = std::max(need, col[k] + 1);
    {   // upper bounds from the part's bytes (a row's seq and qual are under
        // half its bytes each; C2 rows are ~600 bytes): no regrowth copies
        const size_t bytes = (size_t)(P.end - P.beg);
        P.seq.reserve(bytes / 2 + 64);
        P.qual.reserve(bytes / 2 + 64);
        P.qpool.reserve(bytes / 4 + 64);
        P.cpool.reserve(bytes / 8 + 64);
        const size_t rows = bytes / 256 + 16;
        P.qoff.reserve(rows); P.coff.reserve(rows); P.soff.reserve(rows); P.qlen.reserve(rows);
        P.clen.reserve(rows); P.slen.reserve(rows); P.flag.reserve(rows); P.pos.reserve(rows);
        P.cig_off.reserve(rows); P.n_cig.reserve(rows); P.rid.reserve(rows); P.qhash.reserve(rows);
        P.cstate.reserve(rows); P.qshort.reserve(rows);
    }
    while (p < P.end) {
        if (!record_views(p, P.end, f, scratch)) {
            P.err = 1; P.err_row = P.rows; P.err_msg = "more than 64 columns";
            return;
        }
        if (f.size() == 1 && f[0].n == 0) continue;          // blank line
        if ((int)f.size() < need) {
            P.err = 1; P.err_row = P.rows; P.err_msg = "short row";
            return;
        }
        const FieldRef &q = f[col[0]], &rn = f[col[2]], &cg = f[col[5]], &sq = f[col[9]],
                       &ql = f[col[10]];
        int32_t fl = 0, ps = 0;
        if (!py_int(f[col[1]], fl)) {
            P.err = 1; P.err_row = P.rows; P.err_msg = "flag is not an integer";
            return;
        }
        P.flag.push_back(fl);
        P.pos.push_back(py_int(f[col[3]], ps) ? ps : INT32_MIN);
        P.qoff.push_back((int64_t)P.qpool.size());
        P.qlen.push_back((int32_t)q.n);
        P.qpool.append(q.p, q.n);
        P.qhash.push_back(hash_bytes(q.p, q.n));
        auto it = rmap.find(std::string(rn.p, rn.n));
        if (it == rmap.end()) {
            it = rmap.emplace(std::string(rn.p, rn.n), (int)P.rnames.size()).first;
            P.rnames.emplace_back(rn.p, rn.n);
        }
        P.rid.push_back(it->second);
        P.coff.push_back((int64_t)P.cpool.size());
        P.clen.push_back((int32_t)cg.n);
        P.cpool.append(cg.p, cg.n);
        P.cstate.push_back(cigar_ops(cg.p, cg.n, (int64_t)sq.n, ops));
        P.cig_off.push_back((int32_t)P.cig.size());
        P.n_cig.push_back(P.cstate.back() == CIG_OK ? (int32_t)ops.size() : 0);
        if (P.cstate.back() == CIG_OK) P.cig.insert(P.cig.end(), ops.begin(), ops.end());
        P.soff.push_back((int64_t)P.seq.size());
        P.slen.push_back((int32_t)sq.n);
        P.seq.append(sq.p, sq.n);
        P.qshort.push_back(ql.n < sq.n);
        if (ql.n >= sq.n) P.qual.append(ql.p, sq.n);
        else {
            P.qual.append(ql.p, ql.n);
            const size_t at = P.qual.size();
            P.qual.resize(at + (sq.n - ql.n));
            memset(P.qual.data() + at, '!', sq.n - ql.n);
        }
        ++P.rows;
    }
}

static std::string cigar_text(const S2AState &S, int64_t r)
{
    return std::string(S.cpool.data() + S.coff[r], (size_t)S.clen[r]);
}

// the RuntimeError apply_cigar raises for row r, as the reference words it
static int row_error(const S2AState &S, int64_t r)
{
    const std::string cg = cigar_text(S, r);
    switch (S.cstate[r]) {
    case CIG_INVALID: set_error("Invalid CIGAR string: '%s'.", cg.c_str()); return -3;
    case CIG_UNSUPPORTED: {
        // the first token that is not M/I/D/S (sam2aln.py:141-143)
        size_t i = 0;
        while (i < cg.size()) {
            size_t j = i;
            while (cg[j] >= '0' && cg[j] <= '9') ++j;
            if (!strchr("MIDS", cg[j])) break;
            i = j + 1;
        }
        size_t j = i;
        while (j < cg.size() && cg[j] >= '0' && cg[j] <= '9') ++j;
        set_error("Unsupported CIGAR token: '%s'.", cg.substr(i, j + 1 - i).c_str());
        return -3;
    }
    case CIG_LONG: set_error("CIGAR string '%s' is too long for sequence.", cg.c_str()); return -3;
    case CIG_SHORT: set_error("CIGAR string '%s' is too short for sequence.", cg.c_str()); return -3;
    default: break;
    }
    if (S.pos[r] == INT32_MIN) { set_error("invalid literal for int() in pos of row %lld", (long long)r + 1); return -3; }
    if (S.qshort[r]) { set_error("string index out of range (qual shorter than seq, row %lld)", (long long)r + 1); return -3; }
    return 0;
}

// MH_S2A_TRACE=1: phase times of s2a_parse to stderr
static void s2a_mark(std::chrono::steady_clock::time_point t0, const char *what)
{
    static const bool on = getenv("MH_S2A_TRACE") && *getenv("MH_S2A_TRACE") == '1';
    if (on)
        fprintf(stderr, "s2a_parse %s %.1f ms\n", what,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

int s2a_parse(S2AState &S, const char *text, int64_t len, int64_t body_lo, int64_t body_hi)
{
    const auto tp = std::chrono::steady_clock::now();
    const char *p = text, *end = text + len;
    std::vector<std::string> head;
    if (!csv_record(p, end, head)) {
        set_error("remap csv: empty");
        return -3;
    }
    if (body_lo >= 0) {       // one part of the body: records [body_lo, body_hi)
        if (body_lo < p - text || body_hi < body_lo || body_hi > len) {
            set_error("remap csv: bad part bounds");
            return -3;
        }
        p = text + body_lo;
        end = text + body_hi;
    }
    const char *want[11] = {"qname", "flag", "rname", "pos", "mapq", "cigar", "rnext", "pnext",
                            "tlen", "seq", "qual"};
    int col[11];
    for (int k = 0; k < 11; ++k) {
        col[k] = -1;
        for (size_t z = 0; z < head.size(); ++z) if (head[z] == want[k]) col[k] = (int)z;
        if (col[k] < 0) {
            if (k == 4 || k == 6 || k == 7 || k == 8) { col[k] = 0; continue; }   // unused
            set_error("remap csv: missing column %s", want[k]);
            return -3;
        }
    }
    // ---- split the body at record boundaries: '\n' outside quotes ----
    const int64_t body = end - p;
    int nt = s2a_threads();
    if (body < (int64_t)nt * (1 << 20)) nt = (int)std::max<int64_t>(1, body >> 20);
    std::vector<const char *> cut(nt + 1, p);
    cut[nt] = end;
    for (int t = 1; t < nt; ++t) {
        const char *c = p + body * t / nt;
        while (c < end && *c != '\n') ++c;
        cut[t] = c < end ? c + 1 : end;
        if (cut[t] < cut[t - 1]) cut[t] = cut[t - 1];
    }
    std::vector<int64_t> quotes(nt, 0);
    parallel_for(nt, [&](int t) {
        int64_t n = 0;
        for (const char *c = cut[t]; c < cut[t + 1]; ++c) n += *c == '"';
        quotes[t] = n;
    });
    int64_t par = 0;
    for (int t = 0; t + 1 < nt; ++t) {
        par += quotes[t];
        if (par & 1) { nt = 1; cut.assign({p, end}); break; }   // a boundary inside quotes
    }
    std::vector<Part> parts(nt);
    for (int t = 0; t < nt; ++t) { parts[t].beg = cut[t]; parts[t].end = cut[t + 1]; }
    s2a_mark(tp, "split");
    parallel_for(nt, [&](int t) { parse_part(parts[t], col); });
    s2a_mark(tp, "parts");
    int64_t base = 0;
    for (auto &P : parts) {
        if (P.err) {
            set_error("remap csv: row %lld: %s", (long long)(base + P.err_row + 1), P.err_msg.c_str());
            return -3;
        }
        base += P.rows;
    }
    // ---- concatenate the parts ----
    const int64_t nr = base;
    S.n_rows = nr;
    std::vector<int64_t> r0(nt + 1, 0), q0(nt + 1, 0), c0(nt + 1, 0), s0(nt + 1, 0), g0(nt + 1, 0);
    for (int t = 0; t < nt; ++t) {
        r0[t + 1] = r0[t] + parts[t].rows;
        q0[t + 1] = q0[t] + (int64_t)parts[t].qpool.size();
        c0[t + 1] = c0[t] + (int64_t)parts[t].cpool.size();
        s0[t + 1] = s0[t] + (int64_t)parts[t].seq.size();
        g0[t + 1] = g0[t] + (int64_t)parts[t].cig.size();
    }
    // rnames: global ids in part order of first appearance
    std::unordered_map<std::string, int> gid;
    S.rnames.clear();
    std::vector<std::vector<int32_t>> remap_id(nt);
    for (int t = 0; t < nt; ++t)
        for (auto &n : parts[t].rnames) {
            auto it = gid.emplace(n, (int)S.rnames.size());
            if (it.second) S.rnames.push_back(n);
            remap_id[t].push_back(it.first->second);
        }
    S.qpool.resize((size_t)q0[nt]); S.cpool.resize((size_t)c0[nt]);
    S.seq.resize((size_t)s0[nt]); S.qual.resize((size_t)s0[nt]);
    S.qoff.resize(nr); S.qlen.resize(nr); S.coff.resize(nr); S.clen.resize(nr);
    S.cstate.resize(nr); S.rid.resize(nr); S.flag.resize(nr); S.pos.resize(nr);
    S.qshort.resize(nr); S.soff.resize(nr); S.slen.resize(nr); S.cig_off.resize(nr);
    S.n_cig.resize(nr); S.cig.resize((size_t)g0[nt]);
    std::vector<uint64_t> qhash(nr);
    parallel_for(nt, [&](int t) {
        const Part &P = parts[t];
        const int64_t b = r0[t];
        memcpy(&S.qpool[q0[t]], P.qpool.data(), P.qpool.size());
        memcpy(&S.cpool[c0[t]], P.cpool.data(), P.cpool.size());
        memcpy(&S.seq[s0[t]], P.seq.data(), P.seq.size());
        memcpy(&S.qual[s0[t]], P.qual.data(), P.qual.size());
        if (!P.cig.empty()) memcpy(&S.cig[g0[t]], P.cig.data(), 4 * P.cig.size());
        for (int64_t i = 0; i < P.rows; ++i) {
            S.qoff[b + i] = P.qoff[i] + q0[t];
            S.qlen[b + i] = P.qlen[i];
            S.coff[b + i] = P.coff[i] + c0[t];
            S.clen[b + i] = P.clen[i];
            S.cstate[b + i] = P.cstate[i];
            S.rid[b + i] = remap_id[t][P.rid[i]];
            S.flag[b + i] = P.flag[i];
            S.pos[b + i] = P.pos[i];
            S.qshort[b + i] = P.qshort[i];
            S.soff[b + i] = P.soff[i] + s0[t];
            S.slen[b + i] = P.slen[i];
            S.cig_off[b + i] = (int32_t)(P.cig_off[i] + g0[t]);
            S.n_cig[b + i] = P.n_cig[i];
            qhash[b + i] = P.qhash[i];
        }
    });
    {   // the parts' buffers freed off the clock (GB-sized frees take tens of ms)
        auto *old = new std::vector<Part>(std::move(parts));
        std::thread([old]() { delete old; }).detach();
    }
    s2a_mark(tp, "concat");
    // ---- matchmaker (sam2aln.py:291-312): open addressing on qname ----
    uint64_t cap = 1024;
    while (cap < (uint64_t)(2 * nr + 2)) cap <<= 1;
    std::vector<int64_t> slot_row(cap, -1);   // row waiting for its mate
    std::vector<int64_t> pend_of_row(nr, -1);
    std::vector<std::pair<int64_t, bool>> pend;
    pend.reserve((size_t)nr);
    S.u1.clear(); S.u2.clear();
    S.u1.reserve((size_t)nr / 2 + 1); S.u2.reserve((size_t)nr / 2 + 1);
    auto same = [&](int64_t a, int64_t b) {
        return S.qlen[a] == S.qlen[b] &&
               memcmp(S.qpool.data() + S.qoff[a], S.qpool.data() + S.qoff[b], (size_t)S.qlen[a]) == 0;
    };
    for (int64_t r = 0; r < nr; ++r) {
        uint64_t s = qhash[r] & (cap - 1);
        int64_t hit = -1;
        uint64_t tomb = ~0ull;
        while (slot_row[s] != -1) {
            const int64_t o = slot_row[s];
            if (o == -2) { if (tomb == ~0ull) tomb = s; }
            else if (qhash[o] == qhash[r] && same(o, r)) { hit = (int64_t)s; break; }
            s = (s + 1) & (cap - 1);
        }
        if (hit >= 0) {
            const int64_t o = slot_row[hit];
            pend[pend_of_row[o]].second = false;
            S.u1.push_back(o);
            S.u2.push_back(r);
            slot_row[hit] = -2;   // tombstone
        } else {
            slot_row[tomb != ~0ull ? tomb : s] = r;
            pend_of_row[r] = (int64_t)pend.size();
            pend.push_back({r, true});
        }
    }
    for (auto &o : pend) if (o.second) { S.u1.push_back(o.first); S.u2.push_back(-1); }
    s2a_mark(tp, "matchmaker");
    // ---- parse_sam's early causes and the rname order ----
    const int64_t nu = (int64_t)S.u1.size();
    S.ucause.assign(nu, -1);
    S.upaired.assign(nu, 0);
    S.merge_of_unit.assign(nu, -1);
    S.name_id.assign(nu, 0);
    S.names.clear();
    std::vector<int32_t> nid_of_rid(S.rnames.size(), -1);
    for (int64_t u = 0; u < nu; ++u) {
        const int64_t r1 = S.u1[u], r2 = S.u2[u];
        int32_t &n = nid_of_rid[S.rid[r1]];
        if (n < 0) { n = (int32_t)S.names.size(); S.names.push_back(S.rnames[S.rid[r1]]); }
        S.name_id[u] = n;
        const int paired = S.flag[r1] & 1;
        S.upaired[u] = (int8_t)paired;
        int cause = -1;
        if (paired && r2 < 0) cause = S2A_UNMATCHED;
        else if (S.cstate[r1] == CIG_STAR || (r2 >= 0 && S.cstate[r2] == CIG_STAR)) cause = S2A_BADCIGAR;
        else if (paired && S.rid[r1] != S.rid[r2]) cause = S2A_2REFS;
        S.ucause[u] = (int8_t)cause;
        if (cause < 0) {
            if (int st = row_error(S, r1)) return st;
            if (paired)
                if (int st = row_error(S, r2)) return st;
        }
    }
    s2a_mark(tp, "causes");
    return 0;
}

// ---------------------------------------------------------------------------
// output
// ---------------------------------------------------------------------------
static void put_int(std::string &out, long long v)
{
    char b[24];
    auto r = std::to_chars(b, b + sizeof b, v);
    out.append(b, (size_t)(r.ptr - b));
}

template <class Cmp>
static void parallel_sort(std::vector<int64_t> &v, Cmp cmp, int nt)
{
    const size_t n = v.size();
    if (nt <= 1 || n < 65536) { std::sort(v.begin(), v.end(), cmp); return; }
    std::vector<size_t> b(nt + 1);
    for (int t = 0; t <= nt; ++t) b[t] = n * (size_t)t / (size_t)nt;
    parallel_for(nt, [&](int t) { std::sort(v.begin() + b[t], v.begin() + b[t + 1], cmp); });
    for (int w = 1; w < nt; w *= 2) {
        std::vector<std::pair<int, int>> jobs;
        for (int t = 0; t + w < nt; t += 2 * w) jobs.push_back({t, std::min(t + 2 * w, nt)});
        parallel_for((int)jobs.size(), [&](int j) {
            const int a = jobs[j].first, m = a + w, z = jobs[j].second;
            std::inplace_merge(v.begin() + b[a], v.begin() + b[m], v.begin() + b[z], cmp);
        });
    }
}

// the pieces fn(t, range) writes for nt ranges of [0, n), appended in order
using Pieces = std::vector<std::string>;

// Where an output's text goes, in order: collected as pieces (out), or
// written to fd from pos (pwrite) as each piece is finished.
struct TextSink {
    Pieces *out = nullptr;
    int fd = -1;
    int64_t pos = 0;
    int err = 0;    // errno of a failed write
    void put(std::string &s)
    {
        if (out) {
            if (!s.empty()) out->push_back(std::move(s));
            return;
        }
        const char *p = s.data();
        size_t left = s.size();
        while (left > 0 && !err) {
            const ssize_t w = pwrite(fd, p, left, (off_t)pos);
            if (w <= 0) { err = errno ? errno : EIO; break; }
            p += (size_t)w;
            left -= (size_t)w;
            pos += w;
        }
        std::string().swap(s);
    }
};

// fn(text, a, b) formats items [a, b) of n.  Collected: one piece per
// thread.  Streamed: jobs of STREAM_ROWS items on nt - 1 formatting threads
// while this thread writes the finished jobs in order, so the writing of a
// GB-sized output overlaps its formatting.
constexpr int64_t STREAM_ROWS = 4096;
static void parallel_text(int64_t n, int nt, TextSink &sink,
                          const std::function<void(std::string &, int64_t, int64_t)> &fn)
{
    if (n < 4096) nt = 1;
    if (sink.out) {
        std::vector<std::string> piece(nt);
        parallel_for(nt, [&](int t) { fn(piece[t], n * t / nt, n * (t + 1) / nt); });
        for (auto &x : piece) sink.put(x);
        return;
    }
    const int64_t nj = (n + STREAM_ROWS - 1) / STREAM_ROWS;
    if (nt <= 1 || nj <= 1) {
        std::string one;
        fn(one, 0, n);
        sink.put(one);
        return;
    }
    std::vector<std::string> buf((size_t)nj);
    std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[(size_t)nj]);
    for (int64_t j = 0; j < nj; ++j) done[j].store(0);
    std::atomic<int64_t> next(0);
    std::atomic<int> failed(0);
    std::exception_ptr exc;
    std::mutex mu;
    auto work = [&]() {
        try {
            for (int64_t j; !failed && (j = next.fetch_add(1)) < nj;) {
                fn(buf[(size_t)j], j * STREAM_ROWS, std::min(n, (j + 1) * STREAM_ROWS));
                done[j].store(1, std::memory_order_release);
            }
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!exc) exc = std::current_exception();
            failed = 1;
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, nt - 1); ++t) th.emplace_back(work);
    for (int64_t j = 0; j < nj && !failed && !sink.err; ++j) {
        while (!done[j].load(std::memory_order_acquire) && !failed) std::this_thread::yield();
        if (failed) break;
        sink.put(buf[(size_t)j]);
    }
    failed = 1;   // a write error: the formatters stop at their next job
    for (auto &x : th) x.join();
    if (exc) std::rethrow_exception(exc);
}

// aligned.csv (sam2aln.py:459-478): per rname in first-seen order, the
// distinct merged sequences sorted by (count, gap prefix, sequence), all
// descending; seq written without its leading / trailing gaps
static void s2a_aligned(const S2AState &S, TextSink &out)
{
    const int nt = s2a_threads();
    {
        std::string head("refname,qcut,rank,count,offset,seq\n");
        out.put(head);
    }
    const int nn = (int)S.names.size();
    std::vector<int32_t> mref(S.n_merge);
    for (int64_t u = 0; u < (int64_t)S.u1.size(); ++u)
        if (S.merge_of_unit[u] >= 0) mref[S.merge_of_unit[u]] = S.name_id[u];
    std::vector<std::vector<int64_t>> by(nn);
    for (int64_t k = 0; k < S.n_unique; ++k) by[mref[S.uniq[2 * k]]].push_back(k);
    auto cmp = [&](int64_t x, int64_t y) {
        const int64_t rx = S.uniq[2 * x], ry = S.uniq[2 * y];
        const int cx = S.uniq[2 * x + 1], cy = S.uniq[2 * y + 1];
        if (cx != cy) return cx > cy;
        const int ox = S.res[4 * rx + 1], oy = S.res[4 * ry + 1];
        if (ox != oy) return ox > oy;
        const int64_t lx = S.uniq_off[x + 1] - S.uniq_off[x], ly = S.uniq_off[y + 1] - S.uniq_off[y];
        const int c = memcmp(S.gathered.data() + S.uniq_off[x], S.gathered.data() + S.uniq_off[y],
                             (size_t)std::min(lx, ly));
        if (c != 0) return c > 0;
        return lx > ly;
    };
    // the order of cmp in two passes: by (count, offset) -- one 64-bit key,
    // cheap to compare -- then each run of equal keys by its sequence, the
    // runs sorted in parallel (no serial merge of memcmp comparisons)
    std::vector<uint64_t> key((size_t)S.n_unique);
    parallel_for(nt, [&](int t) {
        for (int64_t k = S.n_unique * t / nt; k < S.n_unique * (t + 1) / nt; ++k)
            key[(size_t)k] = (uint64_t)(uint32_t)S.uniq[2 * k + 1] << 32 |
                             (uint32_t)(S.res[4 * S.uniq[2 * k] + 1] ^ (int32_t)0x80000000);
    });
    auto by_key = [&](int64_t x, int64_t y) { return key[(size_t)x] > key[(size_t)y]; };
    for (int r = 0; r < nn; ++r) {
        auto &v = by[r];
        if (v.empty()) continue;
        parallel_sort(v, by_key, nt);
        std::vector<size_t> runs{0};
        for (size_t i = 1; i < v.size(); ++i)
            if (key[(size_t)v[i]] != key[(size_t)v[i - 1]]) runs.push_back(i);
        runs.push_back(v.size());
        std::atomic<size_t> next_run(0);
        parallel_for(nt, [&](int) {
            for (size_t j; (j = next_run.fetch_add(1)) + 1 < runs.size();)
                if (runs[j + 1] - runs[j] > 1) std::sort(v.begin() + runs[j], v.begin() + runs[j + 1], cmp);
        });
        std::string ref;
        csv_field(ref, S.names[r].data(), S.names[r].size());
        const size_t row_guess = ref.size() + 40 + (S.n_unique ? (size_t)(S.gathered.size() / S.n_unique) : 0);
        parallel_text((int64_t)v.size(), nt, out, [&](std::string &o, int64_t a, int64_t b) {
            o.reserve(o.size() + (size_t)(b - a) * row_guess);
            for (int64_t rank = a; rank < b; ++rank) {
                const int64_t k = v[rank], rep = S.uniq[2 * k];
                o += ref;
                o.push_back(',');
                put_int(o, S.q_cutoff);
                o.push_back(',');
                put_int(o, rank);
                o.push_back(',');
                put_int(o, S.uniq[2 * k + 1]);
                o.push_back(',');
                put_int(o, S.res[4 * rep + 1]);
                o.push_back(',');
                o.append(S.gathered.data() + S.uniq_off[k], (size_t)S.res[4 * rep + 3]);
                o.push_back('\n');
            }
        });
    }
}

// insert.csv rows of parse_sam (sam2aln.py:357-380): every I op of the
// mates of a unit that reached apply_cigar, at pos - 1 + read offset
static void s2a_inserts(const S2AState &S, TextSink &out, int64_t u0, int64_t u1, bool head_row)
{
    if (head_row) {
        std::string head("qname,fwd_rev,refname,pos,insert,qual\n");
        out.put(head);
    }
    parallel_text(u1 - u0, s2a_threads(), out, [&](std::string &o, int64_t a, int64_t b) {
        for (int64_t u = u0 + a; u < u0 + b; ++u) {
            if (S.ucause[u] >= 0) continue;
            const int64_t r1 = S.u1[u];
            for (int k = 0; k < (S.upaired[u] ? 2 : 1); ++k) {
                const int64_t r = k ? S.u2[u] : r1;
                int64_t left = 0;
                for (int x = 0; x < S.n_cig[r]; ++x) {
                    const uint32_t op = S.cig[S.cig_off[r] + x];
                    const int n = (int)(op >> 4), t = (int)(op & 15);
                    if (t == MH_OP_I) {
                        csv_field(o, S.qpool.data() + S.qoff[r1], (size_t)S.qlen[r1]);
                        o += (S.flag[r] & 0x40) ? ",F," : ",R,";
                        const std::string &rn = S.rnames[S.rid[r1]];
                        csv_field(o, rn.data(), rn.size());
                        o.push_back(',');
                        put_int(o, (long long)S.pos[r] - 1 + left);
                        o.push_back(',');
                        csv_field(o, S.seq.data() + S.soff[r] + left, (size_t)n);
                        o.push_back(',');
                        csv_field(o, S.qual.data() + S.soff[r] + left, (size_t)n);
                        o.push_back('\n');
                    }
                    if (t == MH_OP_M || t == MH_OP_I || t == MH_OP_S) left += n;
                }
            }
        }
    });
}

static void s2a_failed(const S2AState &S, TextSink &out, int64_t u0, int64_t u1, bool head_row)
{
    if (head_row) {
        std::string head("qname,cause\n");
        out.put(head);
    }
    parallel_text(u1 - u0, s2a_threads(), out, [&](std::string &o, int64_t a, int64_t b) {
        for (int64_t u = u0 + a; u < u0 + b; ++u) {
            int cause = S.ucause[u];
            if (cause < 0 && S.res[4 * S.merge_of_unit[u]] == S2A_MANYNS) cause = S2A_MANYNS;
            if (cause < 0) continue;
            const int64_t r1 = S.u1[u];
            csv_field(o, S.qpool.data() + S.qoff[r1], (size_t)S.qlen[r1]);
            o.push_back(',');
            o += S2A_CAUSE[cause];
            o.push_back('\n');
        }
    });
}

static void s2a_emit(const S2AState &S, int which, TextSink &sink)
{
    const int64_t nu = (int64_t)S.u1.size();
    if (which == 0) s2a_aligned(S, sink);
    else if (which == 1) s2a_inserts(S, sink, 0, nu, true);
    else s2a_failed(S, sink, 0, nu, true);
}

int s2a_format_units(const S2AState &S, int which, int64_t u0, int64_t u1, bool head_row,
                     std::vector<std::string> &out)
{
    out.clear();
    TextSink sink;
    sink.out = &out;
    if (which == 1) s2a_inserts(S, sink, u0, u1, head_row);
    else s2a_failed(S, sink, u0, u1, head_row);
    return 0;
}

int s2a_format(const S2AState &S, int which, std::vector<std::string> &out)
{
    out.clear();
    TextSink sink;
    sink.out = &out;
    s2a_emit(S, which, sink);
    return 0;
}

int s2a_format_write(const S2AState &S, int which, int fd, int64_t offset, int64_t *written)
{
    TextSink sink;
    sink.fd = fd;
    sink.pos = offset;
    s2a_emit(S, which, sink);
    if (written) *written = sink.pos - offset;
    return sink.err;
}

}  // namespace mh
