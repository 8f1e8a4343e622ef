// mh_sam2aln.h -- state of the sam2aln stage shared by its host half
// (mh_s2a_host.cpp: remap.csv parse, matchmaker, CSV output) and its device
// half (mh_sam2aln.hip: merge, grouping).  See mh_sam2aln.hip for the map
// onto micall/core/sam2aln.py.
#pragma once
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "mh_gunzip.h"
#include "mh_internal.h"

namespace mh {

enum { S2A_OK = 0, S2A_UNMATCHED = 1, S2A_BADCIGAR = 2, S2A_2REFS = 3, S2A_MANYNS = 4,
       S2A_EMPTY = 5 };

// apply_cigar's verdict on a row's CIGAR (sam2aln.py:113-151)
enum { CIG_OK = 0, CIG_STAR = 1, CIG_INVALID = 2, CIG_UNSUPPORTED = 3, CIG_LONG = 4,
       CIG_SHORT = 5 };

struct S2AShard;                 // sam2aln split over the ranks of a job (mh_s2a_shard.cpp)
void s2a_shard_free(S2AShard *sh);

struct S2AState {
    // ---- rows of the last remap.csv (host) ----
    int64_t n_rows = 0;
    TextBuf qpool;                      // qnames back to back (not zero-filled)
    std::vector<int64_t> qoff;
    std::vector<int32_t> qlen;
    TextBuf cpool;                      // CIGAR texts (for error messages)
    std::vector<int64_t> coff;
    std::vector<int32_t> clen;
    std::vector<int8_t> cstate;         // CIG_*
    std::vector<int32_t> rid;           // rname id into rnames
    std::vector<std::string> rnames;
    std::vector<int32_t> flag, pos;     // pos INT32_MIN: not an integer
    std::vector<uint8_t> qshort;        // qual shorter than seq
    TextBuf seq, qual;                  // concatenated, qual padded to seq length
    std::vector<int64_t> soff;
    std::vector<int32_t> slen;
    std::vector<int32_t> cig_off, n_cig;
    std::vector<uint32_t> cig;          // (len << 4) | op of usable CIGARs
    // ---- units in matchmaker order ----
    std::vector<int64_t> u1, u2;        // rows; u2 = -1 for None
    std::vector<int8_t> ucause;         // host-decided cause, -1 = merged on the device
    std::vector<int8_t> upaired;        // is_paired of row1
    std::vector<int64_t> merge_of_unit; // index into the device merge list, -1 if none
    std::vector<int32_t> name_id;       // per unit: index into names
    std::vector<std::string> names;     // rnames in first-seen order over units
    int q_cutoff = 15;
    // ---- device ----
    uint8_t *d_seq = nullptr, *d_qual = nullptr, *d_out = nullptr, *d_gather = nullptr;
    int64_t *d_soff = nullptr, *d_units = nullptr, *d_slot = nullptr, *d_goff = nullptr;
    int32_t *d_pos = nullptr, *d_cigoff = nullptr, *d_ncig = nullptr, *d_uref = nullptr,
            *d_res = nullptr, *d_tcnt = nullptr, *d_trep = nullptr, *d_uniq = nullptr,
            *d_ctr = nullptr;
    uint32_t *d_cig = nullptr;
    uint64_t *d_h = nullptr, *d_tkey = nullptr;
    std::unordered_map<const void *, size_t> dcap;   // bytes allocated behind each device pointer (grow-only)
    // ---- results of the device pass ----
    int64_t n_merge = 0, n_unique = 0;
    std::vector<int32_t> res;           // per merge unit: status, offset, body_len, strip_len
    std::vector<int32_t> uniq;          // rep merge unit, count
    std::vector<int64_t> uniq_off;      // offsets into gathered
    TextBuf gathered;                   // bodies of the distinct sequences (not zero-filled)
    // ---- formatted outputs (cached between the size query and the copy) ----
    std::vector<std::string> out_cache[3];   // the text as pieces, in order
    int out_valid = 0;
    // ---- host timings of the last call (ms) ----
    double t_parse = 0, t_device = 0, t_format[3] = {0, 0, 0};
    // ---- this rank's part of a sharded sam2aln ----
    S2AShard *shard = nullptr;
    ~S2AState() { if (shard) s2a_shard_free(shard); }
};

// host half: the header row of text, then its records (body_lo >= 0: only
// the records in bytes [body_lo, body_hi) of text, both record boundaries)
int s2a_parse(S2AState &S, const char *text, int64_t len, int64_t body_lo = -1, int64_t body_hi = -1);
// insert.csv (which 1) or failed.csv (2) rows of units [u0, u1)
int s2a_format_units(const S2AState &S, int which, int64_t u0, int64_t u1, bool head_row,
                     std::vector<std::string> &out);
int s2a_format(const S2AState &S, int which, std::vector<std::string> &out);
// the same text written to fd from offset while it is formatted; 0 or errno
int s2a_format_write(const S2AState &S, int which, int fd, int64_t offset, int64_t *written);
int s2a_threads();
// device half
int s2a_run(Ctx &c, S2AState &S, double max_prop_n);

}  // namespace mh
