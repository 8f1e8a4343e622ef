// mh_s2a_shard.cpp -- sam2aln split over the ranks of a job (host code; the
// merge itself is the device pass of mh_sam2aln.hip, per rank).
//
// The reference (micall/core/sam2aln.py:395-478) parses remap.csv once,
// pairs rows by qname (matchmaker), merges each pair (parse_sam, which its
// own pool runs in parallel over pairs, :411-424), counts identical merged
// sequences per reference (:446-452) and writes them sorted by count (:466-478).
// Here rank r of W:
//
//   part     parses the records in its share of remap.csv's bytes (cuts at
//            record starts, a cut between two rows of one qname moved past
//            the second) and merges its pairs on its GPU.  Its units are its
//            pairs in the order of their second rows, then its unmatched rows
//            in the order they came: in the reference's matchmaker order
//            these are a contiguous run of the pairs and one of the leftovers,
//            provided no qname has rows on two ranks (the caller checks the
//            leftovers' qname hashes across ranks and otherwise runs the
//            whole file on one rank).
//   export   its distinct merged sequences (reference name, count, gap
//            prefix, body) as records, each to the rank that owns its hash;
//   merge 0  the owner adds up the counts of identical records and sorts them
//            as aligned.csv lists them (name, then count, gap prefix and
//            sequence, all descending);
//   samples / splitters   evenly spaced records of every owner, gathered by
//            all, cut each name's order into W ranges;
//   export 1 / merge 1   records to the rank of their range, which sorts them:
//            rank r now holds a contiguous piece of each name's rows, and the
//            caller places it after the pieces of ranks 0 .. r-1 (the row
//            numbers, the "rank" column, start at their row counts);
//   text     insert.csv / failed.csv rows of its pair units and of its
//            leftover units: two segments the caller places segment-major.
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstring>
#include <exception>
#include <functional>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "mh_sam2aln.h"
#include "mh_text.h"

namespace mh {

namespace {

// one distinct merged sequence on the wire: this header, then body_len
// bytes of the merged sequence from its first non-gap character (trailing
// gaps included), padded to 8
struct S2ARec {
    uint64_t hash;
    int32_t gname, count, offset, body_len, strip_len, pad;
};
static_assert(sizeof(S2ARec) == 32, "record header");

inline const char *rec_body(const S2ARec *r) { return (const char *)(r + 1); }
inline size_t rec_size(int32_t body_len) { return sizeof(S2ARec) + (((size_t)body_len + 7) & ~(size_t)7); }

// aligned.csv order: name (global id), then count, gap prefix and sequence,
// all descending (sam2aln.py:466-470: intermed.sort(reverse=True) of
// (count, len_gap_prefix(s), s)); a longer sequence that the shorter one
// prefixes sorts first
bool rec_before(const S2ARec *x, const S2ARec *y)
{
    if (x->gname != y->gname) return x->gname < y->gname;
    if (x->count != y->count) return x->count > y->count;
    if (x->offset != y->offset) return x->offset > y->offset;
    const int c = memcmp(rec_body(x), rec_body(y), (size_t)std::min(x->body_len, y->body_len));
    if (c != 0) return c > 0;
    return x->body_len > y->body_len;
}

bool rec_same(const S2ARec *x, const S2ARec *y)
{
    return x->hash == y->hash && x->gname == y->gname && x->offset == y->offset &&
           x->body_len == y->body_len && memcmp(rec_body(x), rec_body(y), (size_t)x->body_len) == 0;
}

// identity order for the owner's merge of equal records
bool rec_ident_less(const S2ARec *x, const S2ARec *y)
{
    if (x->hash != y->hash) return x->hash < y->hash;
    if (x->gname != y->gname) return x->gname < y->gname;
    if (x->offset != y->offset) return x->offset < y->offset;
    if (x->body_len != y->body_len) return x->body_len < y->body_len;
    return memcmp(rec_body(x), rec_body(y), (size_t)x->body_len) < 0;
}

uint64_t mix64(uint64_t z)
{
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

uint64_t seq_hash(int32_t gname, int32_t offset, const char *p, int32_t n)
{
    uint64_t h = mix64(((uint64_t)(uint32_t)gname << 32) ^ (uint32_t)offset ^ ((uint64_t)n << 40));
    int32_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = mix64(h ^ w);
    }
    uint64_t w = 0;
    memcpy(&w, p + i, (size_t)(n - i));
    return mix64(h ^ w ^ 0x5bd1e995ull);
}

void run_threads(int nt, const std::function<void(int)> &fn)
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

template <class Cmp>
void par_sort(std::vector<const S2ARec *> &v, Cmp cmp)
{
    const int nt = s2a_threads();
    const size_t n = v.size();
    if (nt <= 1 || n < 65536) { std::sort(v.begin(), v.end(), cmp); return; }
    std::vector<size_t> b((size_t)nt + 1);
    for (int t = 0; t <= nt; ++t) b[(size_t)t] = n * (size_t)t / (size_t)nt;
    run_threads(nt, [&](int t) { std::sort(v.begin() + b[(size_t)t], v.begin() + b[(size_t)t + 1], cmp); });
    for (int w = 1; w < nt; w *= 2) {
        std::vector<std::pair<int, int>> jobs;
        for (int t = 0; t + w < nt; t += 2 * w) jobs.push_back({t, std::min(t + 2 * w, nt)});
        run_threads((int)jobs.size(), [&](int j) {
            const int a = jobs[(size_t)j].first, m = a + w, z = jobs[(size_t)j].second;
            std::inplace_merge(v.begin() + b[(size_t)a], v.begin() + b[(size_t)m], v.begin() + b[(size_t)z], cmp);
        });
    }
}

// records of a received buffer, in place (the buffer is kept by the caller)
bool parse_records(const uint8_t *p, int64_t len, std::vector<const S2ARec *> &out)
{
    int64_t at = 0;
    while (at < len) {
        if (len - at < (int64_t)sizeof(S2ARec)) return false;
        const S2ARec *r = (const S2ARec *)(p + at);
        if (r->body_len < 0) return false;
        const int64_t sz = (int64_t)rec_size(r->body_len);
        if (len - at < sz) return false;
        out.push_back(r);
        at += sz;
    }
    return true;
}

void put_rec(uint8_t *dst, const S2ARec &h, const char *body)
{
    memcpy(dst, &h, sizeof h);
    memcpy(dst + sizeof h, body, (size_t)h.body_len);
    const size_t padded = ((size_t)h.body_len + 7) & ~(size_t)7;
    if (padded > (size_t)h.body_len) memset(dst + sizeof h + h.body_len, 0, padded - (size_t)h.body_len);
}

void put_int(std::string &out, long long v)
{
    char b[24];
    const int n = snprintf(b, sizeof b, "%lld", v);
    out.append(b, (size_t)n);
}

}  // namespace

struct S2AShard {
    int part = 0, parts = 1;
    int64_t b0 = 0, b1 = 0;            // this rank's bytes of remap.csv
    int64_t n_pair_units = 0;
    std::vector<int32_t> gid;          // local name id -> global name id
    std::vector<uint8_t> held;         // received records (merge) and splitters
    std::vector<const S2ARec *> recs;  // the records this rank holds, sorted
    std::vector<uint8_t> split_pool;
    std::vector<std::vector<const S2ARec *>> split;   // per global name: splitters, sorted
    std::vector<uint8_t> out;          // the last export / samples / formatted text
    std::vector<int64_t> out_sizes;
};

void s2a_shard_free(S2AShard *sh) { delete sh; }

S2AShard &s2a_shard(S2AState &S)
{
    if (!S.shard) S.shard = new S2AShard();
    return *S.shard;
}

// the start of the record at or after byte x of the body [lo, hi) (a line
// start: the caller has checked that no field is quoted)
static int64_t line_start(const char *t, int64_t lo, int64_t hi, int64_t x)
{
    if (x <= lo) return lo;
    if (x >= hi) return hi;
    if (t[x - 1] == '\n') return x;
    const char *q = (const char *)memchr(t + x, '\n', (size_t)(hi - x));
    return q ? (q - t) + 1 : hi;
}

// the qname field of the record starting at a (the text before the first ',')
static std::pair<const char *, size_t> qname_at(const char *t, int64_t a, int64_t hi, int col)
{
    const char *p = t + a, *e = t + hi;
    const char *le = (const char *)memchr(p, '\n', (size_t)(e - p));
    if (!le) le = e;
    for (int k = 0; k < col; ++k) {
        const char *c = (const char *)memchr(p, ',', (size_t)(le - p));
        if (!c) return {p, 0};
        p = c + 1;
    }
    const char *c = (const char *)memchr(p, ',', (size_t)(le - p));
    return {p, (size_t)((c ? c : le) - p)};
}

// true when no line end of [a, e) lies inside quotes (and the quotes
// balance): every line holds an even number of '"'
static bool even_quote_lines(const char *a, const char *e)
{
    bool open = false;
    const char *q = a;
    for (const char *x = (const char *)memchr(a, '"', (size_t)(e - a)); x;
         x = (const char *)memchr(q, '"', (size_t)(e - q))) {
        if (open && memchr(q, '\n', (size_t)(x - q))) return false;
        open = !open;
        q = x + 1;
    }
    return !open;
}

// The cut between part k - 1 and part k: the record start at or after the
// even split of the body; when the rows either side of it have one qname
// (the two mates of a pair, written one after the other) it moves past the
// second.  Every rank computes every cut the same way.
int64_t s2a_cut(const char *t, int64_t lo, int64_t hi, int k, int parts, int qcol)
{
    if (k <= 0) return lo;
    if (k >= parts) return hi;
    int64_t c = line_start(t, lo, hi, lo + (hi - lo) * k / parts);
    if (c <= lo || c >= hi) return c;
    // the row before the cut starts after the last '\n' before c - 1
    int64_t a = c - 1;
    while (a > lo && t[a - 1] != '\n') --a;
    const auto q1 = qname_at(t, a, hi, qcol), q2 = qname_at(t, c, hi, qcol);
    if (q1.second == q2.second && memcmp(q1.first, q2.first, q1.second) == 0) {
        const char *q = (const char *)memchr(t + c, '\n', (size_t)(hi - c));
        c = q ? (q - t) + 1 : hi;
    }
    return c;
}

// ---- distinct records ------------------------------------------------------

// this rank's distinct sequences as records, each to its owner (hash % parts)
int s2a_export_owned(S2AState &S, int parts)
{
    S2AShard &H = s2a_shard(S);
    const int64_t n = S.n_unique;
    std::vector<int32_t> mref((size_t)S.n_merge);
    for (int64_t u = 0; u < (int64_t)S.u1.size(); ++u)
        if (S.merge_of_unit[u] >= 0) mref[(size_t)S.merge_of_unit[u]] = S.name_id[u];
    std::vector<S2ARec> hdr((size_t)n);
    std::vector<int32_t> dest((size_t)n);
    const int nt = std::max(1, std::min(s2a_threads(), (int)(n >> 12) + 1));
    run_threads(nt, [&](int t) {
        for (int64_t k = n * t / nt; k < n * (t + 1) / nt; ++k) {
            const int64_t rep = S.uniq[2 * k];
            S2ARec &h = hdr[(size_t)k];
            h.gname = H.gid[(size_t)mref[(size_t)rep]];
            h.count = S.uniq[2 * k + 1];
            h.offset = S.res[4 * rep + 1];
            h.body_len = S.res[4 * rep + 2];
            h.strip_len = S.res[4 * rep + 3];
            h.pad = 0;
            h.hash = seq_hash(h.gname, h.offset, S.gathered.data() + S.uniq_off[k], h.body_len);
            dest[(size_t)k] = (int32_t)(h.hash % (uint64_t)parts);
        }
    });
    std::vector<int64_t> size((size_t)parts, 0);
    for (int64_t k = 0; k < n; ++k) size[(size_t)dest[(size_t)k]] += (int64_t)rec_size(hdr[(size_t)k].body_len);
    std::vector<int64_t> base((size_t)parts + 1, 0);
    for (int p = 0; p < parts; ++p) base[(size_t)p + 1] = base[(size_t)p] + size[(size_t)p];
    std::vector<int64_t> at((size_t)n);
    {
        std::vector<int64_t> cur(base.begin(), base.end() - 1);
        for (int64_t k = 0; k < n; ++k) {
            at[(size_t)k] = cur[(size_t)dest[(size_t)k]];
            cur[(size_t)dest[(size_t)k]] += (int64_t)rec_size(hdr[(size_t)k].body_len);
        }
    }
    H.out.resize((size_t)base[(size_t)parts]);
    run_threads(nt, [&](int t) {
        for (int64_t k = n * t / nt; k < n * (t + 1) / nt; ++k)
            put_rec(H.out.data() + at[(size_t)k], hdr[(size_t)k], S.gathered.data() + S.uniq_off[k]);
    });
    H.out_sizes = size;
    H.parts = parts;
    return 0;
}

// stage 0: the owner's records -- equal ones added up -- sorted in
// aligned.csv order; stage 1: the records of this rank's ranges, sorted
int s2a_merge(S2AState &S, int stage, const uint8_t *data, int64_t len)
{
    S2AShard &H = s2a_shard(S);
    H.held.assign(data, data + len);
    H.recs.clear();
    if (!parse_records(H.held.data(), (int64_t)H.held.size(), H.recs)) {
        set_error("sam2aln: malformed records from another rank");
        return -3;
    }
    if (stage == 0 && !H.recs.empty()) {
        par_sort(H.recs, rec_ident_less);
        size_t w = 0;
        for (size_t i = 0; i < H.recs.size();) {
            size_t j = i + 1;
            int64_t cnt = H.recs[i]->count;
            while (j < H.recs.size() && rec_same(H.recs[i], H.recs[j])) cnt += H.recs[j++]->count;
            S2ARec *first = const_cast<S2ARec *>(H.recs[i]);
            if (cnt > INT32_MAX) { set_error("sam2aln: count overflow"); return -3; }
            first->count = (int32_t)cnt;
            H.recs[w++] = first;
            i = j;
        }
        H.recs.resize(w);
    }
    par_sort(H.recs, rec_before);
    return 0;
}

// up to per_name records of every name, evenly spaced in this rank's order
int s2a_samples(S2AState &S, int per_name)
{
    S2AShard &H = s2a_shard(S);
    H.out.clear();
    for (size_t i = 0; i < H.recs.size();) {
        size_t j = i;
        while (j < H.recs.size() && H.recs[j]->gname == H.recs[i]->gname) ++j;
        const size_t n = j - i;
        for (int s = 0; s < per_name && (size_t)s < n; ++s) {
            const S2ARec *r = H.recs[i + n * (size_t)(s + 1) / (size_t)(per_name + 1)];
            const size_t at = H.out.size();
            H.out.resize(at + rec_size(r->body_len));
            put_rec(H.out.data() + at, *r, rec_body(r));
        }
        i = j;
    }
    H.out_sizes.assign(1, (int64_t)H.out.size());
    return 0;
}

// every rank's samples: the splitters cutting each name's order into parts
// ranges (the same on every rank: the same samples, the same sort)
int s2a_splitters(S2AState &S, const uint8_t *data, int64_t len, int parts)
{
    S2AShard &H = s2a_shard(S);
    H.split_pool.assign(data, data + len);
    std::vector<const S2ARec *> all;
    if (!parse_records(H.split_pool.data(), (int64_t)H.split_pool.size(), all)) {
        set_error("sam2aln: malformed samples");
        return -3;
    }
    std::sort(all.begin(), all.end(), rec_before);
    int32_t top = -1;
    for (const S2ARec *r : all) top = std::max(top, r->gname);
    for (const S2ARec *r : H.recs) top = std::max(top, r->gname);
    H.split.assign((size_t)(top + 1), {});
    for (size_t i = 0; i < all.size();) {
        size_t j = i;
        while (j < all.size() && all[j]->gname == all[i]->gname) ++j;
        const size_t m = j - i;
        auto &sp = H.split[(size_t)all[i]->gname];
        for (int p = 1; p < parts; ++p) sp.push_back(all[i + std::min(m - 1, m * (size_t)p / (size_t)parts)]);
        i = j;
    }
    H.parts = parts;
    return 0;
}

// the owner's sorted records, each to the rank of its range
int s2a_export_ranges(S2AState &S)
{
    S2AShard &H = s2a_shard(S);
    const int parts = H.parts;
    const size_t n = H.recs.size();
    std::vector<int32_t> dest(n, 0);
    for (size_t k = 0; k < n; ++k) {
        const S2ARec *r = H.recs[k];
        if ((size_t)r->gname >= H.split.size()) continue;
        const auto &sp = H.split[(size_t)r->gname];
        dest[k] = (int32_t)(std::upper_bound(sp.begin(), sp.end(), r, rec_before) - sp.begin());
    }
    std::vector<int64_t> size((size_t)parts, 0), base((size_t)parts + 1, 0);
    for (size_t k = 0; k < n; ++k) size[(size_t)dest[k]] += (int64_t)rec_size(H.recs[k]->body_len);
    for (int p = 0; p < parts; ++p) base[(size_t)p + 1] = base[(size_t)p] + size[(size_t)p];
    std::vector<int64_t> at(n);
    {
        std::vector<int64_t> cur(base.begin(), base.end() - 1);
        for (size_t k = 0; k < n; ++k) {
            at[k] = cur[(size_t)dest[k]];
            cur[(size_t)dest[k]] += (int64_t)rec_size(H.recs[k]->body_len);
        }
    }
    std::vector<uint8_t> out((size_t)base[(size_t)parts]);
    const int nt = std::max(1, std::min(s2a_threads(), (int)(n >> 12) + 1));
    run_threads(nt, [&](int t) {
        for (size_t k = n * (size_t)t / (size_t)nt; k < n * (size_t)(t + 1) / (size_t)nt; ++k)
            put_rec(out.data() + at[k], *H.recs[k], rec_body(H.recs[k]));
    });
    H.out.swap(out);
    H.out_sizes = size;
    return 0;
}

// rows of this rank's range per global name
void s2a_range_counts(S2AState &S, int n_names, int64_t *counts)
{
    S2AShard &H = s2a_shard(S);
    for (int g = 0; g < n_names; ++g) counts[g] = 0;
    for (const S2ARec *r : H.recs)
        if (r->gname >= 0 && r->gname < n_names) ++counts[r->gname];
}

// aligned.csv rows of this rank's range (sam2aln.py:471-478), one segment
// per global name; row numbers from base[name]
int s2a_range_format(S2AState &S, int n_names, const char *const *names, const int64_t *base)
{
    S2AShard &H = s2a_shard(S);
    const int64_t n = (int64_t)H.recs.size();
    std::vector<std::string> ref((size_t)n_names);
    for (int g = 0; g < n_names; ++g) csv_field(ref[(size_t)g], names[g], strlen(names[g]));
    // each record's row number: base of its name + its place among the
    // name's records here
    std::vector<int64_t> rank((size_t)n);
    {
        int64_t k = 0;
        while (k < n) {
            const int32_t g = H.recs[(size_t)k]->gname;
            int64_t j = k;
            while (j < n && H.recs[(size_t)j]->gname == g) {
                rank[(size_t)j] = base[g] + (j - k);
                ++j;
            }
            k = j;
        }
    }
    const int nt = std::max(1, std::min(s2a_threads(), (int)(n >> 12) + 1));
    std::vector<std::string> piece((size_t)nt);
    std::vector<std::vector<int64_t>> seg((size_t)nt, std::vector<int64_t>((size_t)n_names, 0));
    run_threads(nt, [&](int t) {
        std::string &o = piece[(size_t)t];
        for (int64_t k = n * t / nt; k < n * (t + 1) / nt; ++k) {
            const S2ARec *r = H.recs[(size_t)k];
            const size_t before = o.size();
            o += ref[(size_t)r->gname];
            o.push_back(',');
            put_int(o, S.q_cutoff);
            o.push_back(',');
            put_int(o, rank[(size_t)k]);
            o.push_back(',');
            put_int(o, r->count);
            o.push_back(',');
            put_int(o, r->offset);
            o.push_back(',');
            o.append(rec_body(r), (size_t)r->strip_len);
            o.push_back('\n');
            seg[(size_t)t][(size_t)r->gname] += (int64_t)(o.size() - before);
        }
    });
    size_t total = 0;
    for (auto &p : piece) total += p.size();
    H.out.resize(total);
    size_t at = 0;
    for (auto &p : piece) {
        memcpy(H.out.data() + at, p.data(), p.size());
        at += p.size();
        std::string().swap(p);
    }
    H.out_sizes.assign((size_t)n_names, 0);
    for (int t = 0; t < nt; ++t)
        for (int g = 0; g < n_names; ++g) H.out_sizes[(size_t)g] += seg[(size_t)t][(size_t)g];
    return 0;
}

}  // namespace mh

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
using namespace mh;

namespace {

S2AState *state_of(mh_ctx *ctx)
{
    Ctx &c = *ctx_of(ctx);
    if (!c.s2a) c.s2a = new S2AState();
    return c.s2a;
}

// the last output of the shard (pointer, sizes)
void hand_out(S2AState &S, int64_t *sizes, int n, const uint8_t **data)
{
    S2AShard &H = s2a_shard(S);
    for (int k = 0; k < n; ++k) sizes[k] = k < (int)H.out_sizes.size() ? H.out_sizes[(size_t)k] : 0;
    *data = H.out.data();
}

template <class F>
int guarded(const char *what, F &&fn)
{
    try {
        return fn();
    } catch (const std::bad_alloc &) {
        set_error("%s: out of memory", what);
        return -2;
    } catch (const std::exception &e) {
        set_error("%s: %s", what, e.what());
        return -2;
    }
}

}  // namespace

extern "C" int mh_sam2aln_part(mh_ctx *ctx, int fd, int part, int parts, int q_cutoff, double max_prop_n,
                               int64_t *info)
{
    if (!ctx || fd < 0 || parts < 1 || part < 0 || part >= parts || !info || q_cutoff < 0 || q_cutoff > 93)
        return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    const char *text = nullptr;
    size_t len = 0;
    if (int st = map_text_file(fd, &text, &len)) return st;   // 1: '\r' in it (not split)
    S2AState &S = *state_of(ctx);
    const int rc = guarded("mh_sam2aln_part", [&]() -> int {
        S.q_cutoff = q_cutoff;
        S.n_merge = S.n_unique = 0;
        S.res.clear();
        for (auto &o : S.out_cache) std::vector<std::string>().swap(o);
        S.out_valid = 0;
        // the header row and the qname column
        const char *p = text, *end = text + len;
        std::vector<std::string> head;
        if (!csv_record(p, end, head)) { set_error("remap csv: empty"); return -3; }
        int qcol = -1;
        for (size_t k = 0; k < head.size(); ++k) if (head[k] == "qname") qcol = (int)k;
        if (qcol < 0) return 1;
        const int64_t lo = p - text, hi = (int64_t)len;
        S2AShard &H = s2a_shard(S);
        H.part = part;
        H.parts = parts;
        H.b0 = s2a_cut(text, lo, hi, part, parts, qcol);
        H.b1 = s2a_cut(text, lo, hi, part + 1, parts, qcol);
        // the cuts are record starts when no quoted field holds a line end
        // (csv quotes a quality string with '"' or ',' in it, never across
        // lines in remap.csv): every line of this part has an even number of
        // quote characters, else the part is not split (the caller's ranks
        // agree on it)
        if (!even_quote_lines(text + H.b0, text + H.b1)) return 1;
        const auto t0 = std::chrono::steady_clock::now();
        if (int st = s2a_parse(S, text, (int64_t)len, H.b0, H.b1)) return st;
        const auto t1 = std::chrono::steady_clock::now();
        if (int st = s2a_run(c, S, max_prop_n)) return st;
        const auto t2 = std::chrono::steady_clock::now();
        S.t_parse = std::chrono::duration<double, std::milli>(t1 - t0).count();
        S.t_device = std::chrono::duration<double, std::milli>(t2 - t1).count();
        int64_t pairs = 0;
        while (pairs < (int64_t)S.u2.size() && S.u2[(size_t)pairs] >= 0) ++pairs;
        H.n_pair_units = pairs;
        H.gid.assign(S.names.size(), -1);
        info[0] = (int64_t)S.u1.size();
        info[1] = pairs;
        info[2] = (int64_t)S.names.size();
        info[3] = S.n_unique;
        info[4] = H.b1 - H.b0;
        info[5] = (int64_t)len;
        return 0;
    });
    unmap_text_file(text, len);
    if (rc < 0) S.u1.clear();
    return rc;
}

extern "C" int mh_sam2aln_part_units(mh_ctx *ctx, uint64_t *qhash, uint8_t *leftover)
{
    if (!ctx || !qhash || !leftover) return -3;
    S2AState &S = *state_of(ctx);
    const int64_t nu = (int64_t)S.u1.size();
    for (int64_t u = 0; u < nu; ++u) {
        const int64_t r = S.u1[(size_t)u];
        qhash[u] = seq_hash(0, 0, S.qpool.data() + S.qoff[(size_t)r], S.qlen[(size_t)r]);
        leftover[u] = S.u2[(size_t)u] < 0;
    }
    return 0;
}

extern "C" int mh_sam2aln_part_names(mh_ctx *ctx, char *buf, size_t cap, size_t *used, int64_t *first_unit)
{
    if (!ctx || !used) return -3;
    S2AState &S = *state_of(ctx);
    size_t n = 0;
    for (const auto &x : S.names) n += x.size() + 1;
    *used = n;
    if (!buf) return 0;
    if (cap < n || !first_unit) { set_error("mh_sam2aln_part_names: buffer too small"); return -2; }
    for (const auto &x : S.names) { memcpy(buf, x.data(), x.size()); buf += x.size(); *buf++ = '\n'; }
    for (size_t k = 0; k < S.names.size(); ++k) first_unit[k] = -1;
    for (int64_t u = 0; u < (int64_t)S.u1.size(); ++u)
        if (first_unit[S.name_id[(size_t)u]] < 0) first_unit[S.name_id[(size_t)u]] = u;
    return 0;
}

extern "C" int mh_sam2aln_part_set_names(mh_ctx *ctx, const int32_t *gid, int n)
{
    if (!ctx || (!gid && n)) return -3;
    S2AState &S = *state_of(ctx);
    if (n != (int)S.names.size()) { set_error("mh_sam2aln_part_set_names: %d names, %zu held", n, S.names.size()); return -3; }
    s2a_shard(S).gid.assign(gid, gid + n);
    return 0;
}

extern "C" int mh_sam2aln_records(mh_ctx *ctx, int step, int parts, int per_name, int64_t *sizes,
                                  const uint8_t **data)
{
    if (!ctx || !sizes || !data || parts < 1) return -3;
    S2AState &S = *state_of(ctx);
    return guarded("mh_sam2aln_records", [&]() -> int {
        int st = 0;
        if (step == 0) st = s2a_export_owned(S, parts);
        else if (step == 1) st = s2a_samples(S, per_name);
        else if (step == 2) st = s2a_export_ranges(S);
        else return -3;
        if (st) return st;
        hand_out(S, sizes, step == 1 ? 1 : parts, data);
        return 0;
    });
}

extern "C" int mh_sam2aln_records_merge(mh_ctx *ctx, int stage, const uint8_t *data, int64_t len)
{
    if (!ctx || (!data && len) || len < 0) return -3;
    S2AState &S = *state_of(ctx);
    return guarded("mh_sam2aln_records_merge", [&]() { return s2a_merge(S, stage, data, len); });
}

extern "C" int mh_sam2aln_splitters(mh_ctx *ctx, const uint8_t *data, int64_t len, int parts)
{
    if (!ctx || (!data && len) || len < 0 || parts < 1) return -3;
    S2AState &S = *state_of(ctx);
    return guarded("mh_sam2aln_splitters", [&]() { return s2a_splitters(S, data, len, parts); });
}

extern "C" int mh_sam2aln_range_counts(mh_ctx *ctx, int n_names, int64_t *counts)
{
    if (!ctx || n_names < 0 || (!counts && n_names)) return -3;
    s2a_range_counts(*state_of(ctx), n_names, counts);
    return 0;
}

extern "C" int mh_sam2aln_range_text(mh_ctx *ctx, int n_names, const char *const *names, const int64_t *base,
                                     int64_t *seg_bytes, const uint8_t **data)
{
    if (!ctx || n_names < 0 || (n_names && (!names || !base || !seg_bytes)) || !data) return -3;
    S2AState &S = *state_of(ctx);
    return guarded("mh_sam2aln_range_text", [&]() -> int {
        if (int st = s2a_range_format(S, n_names, names, base)) return st;
        hand_out(S, seg_bytes, n_names, data);
        return 0;
    });
}

extern "C" int mh_sam2aln_part_text(mh_ctx *ctx, int which, int seg, int head, int64_t *bytes,
                                    const uint8_t **data)
{
    if (!ctx || (which != 1 && which != 2) || seg < 0 || seg > 1 || !bytes || !data) return -3;
    S2AState &S = *state_of(ctx);
    return guarded("mh_sam2aln_part_text", [&]() -> int {
        S2AShard &H = s2a_shard(S);
        const int64_t nu = (int64_t)S.u1.size();
        const int64_t u0 = seg ? H.n_pair_units : 0, u1 = seg ? nu : H.n_pair_units;
        std::vector<std::string> pieces;
        s2a_format_units(S, which, u0, u1, head != 0, pieces);
        size_t total = 0;
        for (auto &x : pieces) total += x.size();
        H.out.resize(total);
        size_t at = 0;
        for (auto &x : pieces) { memcpy(H.out.data() + at, x.data(), x.size()); at += x.size(); }
        H.out_sizes.assign(1, (int64_t)total);
        *bytes = (int64_t)total;
        *data = H.out.data();
        return 0;
    });
}
