// mh_text.h -- host-side text helpers shared by the C-ABI translation units:
// the csv-module dialect MiCall's files use (DictReader / DictWriter with
// QUOTE_MINIMAL) and CIGAR strings as sam2aln.apply_cigar accepts them.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "micall_hip.h"

namespace mh {

// One CSV record (quoted fields may hold ',', '"' doubled, and newlines).
inline bool csv_record(const char *&p, const char *end, std::vector<std::string> &f)
{
    f.clear();
    if (p >= end) return false;
    std::string cur;
    bool any = false;
    for (;;) {
        cur.clear();
        if (p < end && *p == '"') {
            ++p;
            while (p < end) {
                if (*p == '"') {
                    if (p + 1 < end && p[1] == '"') { cur.push_back('"'); p += 2; continue; }
                    ++p;
                    break;
                }
                cur.push_back(*p++);
            }
            while (p < end && *p != ',' && *p != '\n' && *p != '\r') cur.push_back(*p++);
        } else {
            while (p < end && *p != ',' && *p != '\n' && *p != '\r') cur.push_back(*p++);
        }
        f.push_back(cur);
        any = true;
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == '\r') ++p;
        if (p < end && *p == '\n') ++p;
        break;
    }
    return any;
}

inline bool parse_cigar_ops(const std::string &c, std::vector<uint32_t> &ops, int &maxm)
{
    // ^((\d+)([MIDNSHPX=]))*$ ; only M/I/D/S are usable (sam2aln.py:113-142)
    ops.clear();
    maxm = 0;
    size_t i = 0;
    bool ok = true;
    while (i < c.size()) {
        size_t j = i;
        uint64_t n = 0;
        while (j < c.size() && c[j] >= '0' && c[j] <= '9') { n = n * 10 + (c[j] - '0'); ++j; }
        if (j == i || j >= c.size()) return false;
        const char op = c[j];
        uint32_t code;
        switch (op) {
        case 'M': code = MH_OP_M; if ((int)n > maxm) maxm = (int)n; break;
        case 'I': code = MH_OP_I; break;
        case 'D': code = MH_OP_D; break;
        case 'S': code = MH_OP_S; break;
        case 'N': case 'H': case 'P': case 'X': case '=': code = 3; ok = false; break;  // unsupported
        default: return false;
        }
        ops.push_back(((uint32_t)n << 4) | code);
        i = j + 1;
    }
    (void)ok;
    return true;
}

// csv.writer QUOTE_MINIMAL: quote a field holding ',', '"', '\n' or '\r'.
inline void csv_field(std::string &out, const char *s, size_t n)
{
    bool quote = false;
    for (size_t i = 0; i < n; ++i)
        if (s[i] == ',' || s[i] == '"' || s[i] == '\n' || s[i] == '\r') { quote = true; break; }
    if (!quote) { out.append(s, n); return; }
    out.push_back('"');
    for (size_t i = 0; i < n; ++i) {
        if (s[i] == '"') out.push_back('"');
        out.push_back(s[i]);
    }
    out.push_back('"');
}


}  // namespace mh
