/*
 * oracle/og_mapper.h -- TEST INFRASTRUCTURE ONLY (CPU oracle of the read
 * mapper).  See og_mapper.c for the specification and provenance.
 */
#ifndef OG_MAPPER_H
#define OG_MAPPER_H
#include <stdint.h>

#define OG_BAND 64            /* storage width of a DP row (>= 2 * OG_MAXHALF + 1) */
#define OG_MAXHALF 15         /* bowtie2's maxhalf: band = center +- min(15, max gaps) */
#define OG_MAXCAND 4          /* extension candidates per mate */
#define OG_MAXHITS_SEED 64    /* seeds with more exact hits are skipped */
#define OG_MAXHITS_MATE 512   /* hit budget per mate (seed order) */
#define OG_CLUSTER_GAP 8      /* diagonals closer than this join a cluster */
#define OG_MAXSEEDS 32        /* seeds per strand */
#define OG_MAXOPS 128         /* CIGAR capacity per alignment */
#define OG_MAXLEN 1024        /* longest read accepted */
#define OG_NEG (-(1 << 29))

enum { OG_E2E = 0, OG_LOCAL = 1 };
enum { OG_OP_M = 0, OG_OP_I = 1, OG_OP_D = 2, OG_OP_S = 4 };
enum { OG_YT_CP = 0, OG_YT_DP = 1, OG_YT_UP = 2, OG_YT_UU = 3 };
enum { OG_YF_NONE = 0, OG_YF_NS = 1, OG_YF_LN = 2 };

typedef struct {
    int mode;       /* OG_E2E (prelim_map) or OG_LOCAL (remap) */
    int rdg_open, rdg_ext;  /* --rdg (deletions, gap in read) */
    int rfg_open, rfg_ext;  /* --rfg (insertions, gap in reference) */
    int maxins;     /* -X */
} og_params;

/* One SAM record worth of alignment facts for one mate. */
typedef struct {
    int32_t ref;        /* reference index, -1 if unaligned */
    int32_t pos;        /* 0-based leftmost reference position (after trimming) */
    int32_t rev;        /* aligned to the reverse strand */
    int32_t score;      /* AS:i */
    int32_t secbest;    /* XS:i, INT32_MIN if none */
    int32_t flag;       /* SAM FLAG */
    int32_t mapq;
    int32_t rnext;      /* -2: '*', -1: '=', >=0: reference index */
    int32_t pnext;      /* 1-based, 0 if none */
    int32_t tlen;
    int32_t sam_ref;    /* RNAME index (-1: '*'); unaligned mates borrow the mate's */
    int32_t sam_pos;    /* POS, 1-based, 0 if none */
    int32_t xm, xo, xg, nm;
    int32_t ys;         /* mate's AS, INT32_MIN if mate unaligned */
    int32_t yt, yf;
    int32_t n_cigar;
    uint32_t cigar[OG_MAXOPS];  /* (len << 4) | op */
} og_aln;

typedef struct og_index og_index;

og_index *og_index_build(int n_refs, const char *const *seqs, int seedlen);
void og_index_free(og_index *ix);

/* Map n_reads reads (paired: reads 2p, 2p+1 are mates 1 and 2).  Reads are
 * stored back to back in seq/qual with offsets[r] and lens[r]. */
int og_map(const og_index *ix, const og_params *par, int64_t n_reads, int paired,
           const uint8_t *seq, const uint8_t *qual, const int64_t *offsets,
           const int32_t *lens, og_aln *out, int nthreads);

/* og_map plus two int32 per read: the cause (OG_CAUSE_*) and the number of
 * seed-hit clusters before the top-OG_MAXCAND cut.  Diagnostics only. */
enum { OG_CAUSE_ALIGNED = 0, OG_CAUSE_RESCUED = 1, OG_CAUSE_FILTERED = 2,
       OG_CAUSE_NO_CANDIDATE = 3, OG_CAUSE_SCORE_MIN = 4, OG_CAUSE_NCEIL = 5, OG_CAUSE_OTHER = 6 };
int og_map_diag(const og_index *ix, const og_params *par, int64_t n_reads, int paired,
                const uint8_t *seq, const uint8_t *qual, const int64_t *offsets,
                const int32_t *lens, og_aln *out, int nthreads, int32_t *diag);

/* Per-length tables shared with the device path (host-computed). */
int og_seed_interval(int mode, int len);
int og_min_score(int mode, int len);
int og_n_ceil(int len);
int og_band_half(const og_params *par, int len);
#endif
