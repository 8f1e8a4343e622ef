"""Throwaway k_pileup phase clock (like kdp_phases.py): copies
micall-lite_amd/csrc to variants/pphases/src, stamps s_memtime at the phase
boundaries of k_pileup's unit loop, sums the wave cycles per phase in a
device array and prints them to stderr after every pileup launch.

    python profiles/diag/pileup_phases.py && make -C variants/pphases/src -j8 \
        OUTDIR=.. OBJDIR=_obj
Phases: rows (unpack, ops, early exits), cigar (op scans), expand (op lookup,
base loads, LDS writes), ins (merge_inserts), prefix (merge starts), counts
(update_counts), tail (reductions, per-reference scalars), flush (block end).
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, 'micall-lite_amd', 'csrc')
DST = os.path.join(ROOT, 'variants', 'pphases', 'src')


def sub(text, old, new, count=1):
    if text.count(old) < 1:
        sys.exit('anchor not found: %r' % old[:70])
    return text.replace(old, new, count)


def main():
    if os.path.isdir(DST):
        shutil.rmtree(DST)
    shutil.copytree(SRC, DST, ignore=shutil.ignore_patterns('_obj*'))
    mk = open(os.path.join(DST, 'Makefile')).read()
    mk = mk.replace('-I../../include', '-I%s' % os.path.join(ROOT, 'include'))
    mk = mk.replace('../../include/micall_hip.h', os.path.join(ROOT, 'include', 'micall_hip.h'))
    open(os.path.join(DST, 'Makefile'), 'w').write(mk)
    p = os.path.join(DST, 'mh_pileup.hip')
    t = open(p).read()
    t = sub(t, 'template <int SRC>\n__global__ __launch_bounds__(1024, 6) void k_pileup(PileArgs A)\n{\n',
            '__device__ unsigned long long g_pph[8];\n'
            'template <int SRC>\n__global__ __launch_bounds__(1024, 6) void k_pileup(PileArgs A)\n{\n'
            '    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n'
            '    unsigned long long t0 = 0, t1;\n'
            '#define PH(k) do { __builtin_amdgcn_wave_barrier(); t1 = __builtin_readcyclecounter(); '
            'ph[k] += t1 - t0; t0 = t1; } while (0)\n')
    t = sub(t, '    if (u < A.n_units) npk = load_rows_packed<SRC>(A, u, lane);\n',
            '    if (u < A.n_units) npk = load_rows_packed<SRC>(A, u, lane);\n'
            '    t0 = __builtin_readcyclecounter();\n')
    t = sub(t, '        // ---- apply_cigar: op offsets by a lane-parallel prefix scan, then\n',
            '        PH(0);\n        // ---- apply_cigar: op offsets by a lane-parallel prefix scan, then\n')
    t = sub(t, '        const int spanA = lenA - padA, spanB = nm > 1 ? lenB - padB : 0;\n',
            '        PH(1);\n        const int spanA = lenA - padA, spanB = nm > 1 ? lenB - padB : 0;\n')
    t = sub(t, '        // ---- merge_inserts (only units with I ops): keys left + pad,\n',
            '        PH(2);\n        // ---- merge_inserts (only units with I ops): keys left + pad,\n')
    t = sub(t, '        // ---- merge_pairs positions: seq1 = shorter padded read ----\n',
            '        PH(3);\n        // ---- merge_pairs positions: seq1 = shorter padded read ----\n')
    t = sub(t, '        // ---- update_counts over mseq (remap.py:284-301) ----\n',
            '        PH(4);\n        // ---- update_counts over mseq (remap.py:284-301) ----\n')
    t = sub(t, '        mxp = wave_max_all(mxp);\n', '        PH(5);\n        mxp = wave_max_all(mxp);\n')
    t = sub(t, '    // ---- flush the block\'s windows (consecutive threads add to consecutive\n',
            '    PH(6);\n    // ---- flush the block\'s windows (consecutive threads add to consecutive\n')
    t = sub(t, '        if (rl[r].max_pos > 0) atomicMax(&A.max_pos[r], rl[r].max_pos);\n    }\n}\n',
            '        if (rl[r].max_pos > 0) atomicMax(&A.max_pos[r], rl[r].max_pos);\n    }\n'
            '    PH(7);\n'
            '    if (lane == 0) for (int k = 0; k < 8; ++k) atomicAdd(&g_pph[k], ph[k]);\n}\n')
    t = sub(t, '        if (ctr[3]) { set_error("mh_pileup: malformed alignment row (CIGAR/position)"); return -3; }\n',
            '        {\n'
            '            unsigned long long ph[8];\n'
            '            MH_HIP(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_pph), sizeof(ph)));\n'
            '            double tot = 0;\n'
            '            for (int k = 0; k < 8; ++k) tot += (double)ph[k];\n'
            '            fprintf(stderr, "PILE_PHASES src=%d units=%lld rows=%.4f cigar=%.4f expand=%.4f ins=%.4f '
            'prefix=%.4f counts=%.4f tail=%.4f flush=%.4f total_gcyc=%.3f wpb=%d blocks=%lld win_words=%d\\n",\n'
            '                    source, (long long)n_units, ph[0] / tot, ph[1] / tot, ph[2] / tot, ph[3] / tot,\n'
            '                    ph[4] / tot, ph[5] / tot, ph[6] / tot, ph[7] / tot, tot / 1e9, geo.wpb,\n'
            '                    (long long)geo.blocks, geo.win_words);\n'
            '            memset(ph, 0, sizeof(ph));\n'
            '            MH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_pph), ph, sizeof(ph)));\n'
            '        }\n'
            '        if (ctr[3]) { set_error("mh_pileup: malformed alignment row (CIGAR/position)"); return -3; }\n')
    open(p, 'w').write(t)
    print('patched', p)


if __name__ == '__main__':
    main()
