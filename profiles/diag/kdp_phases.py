"""Throwaway k_dp phase clock: copies micall-lite_amd/csrc to
_ab/phases/src, inserts s_memtime stamps around the phases of k_dp's
item loop (staging, fast-path attempt, DP rows, finish of fast items, finish
of DP pairs, the tail), sums the wave cycles per phase and mode in a device
array, and prints them to stderr after every mh_map pass.  Builds
_ab/phases/libmicall_hip.so; run with MICALL_HIP_LIB pointing at it.

    python profiles/diag/kdp_phases.py && make -C _ab/phases/src -j8 \
        OUTDIR=.. OBJDIR=_obj
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, 'micall-lite_amd', 'csrc')
DST = os.path.join(ROOT, '_ab', 'phases', 'src')


def sub(text, old, new, count=1):
    if text.count(old) < 1:
        sys.exit('anchor not found: %r' % old[:60])
    return text.replace(old, new, count)


def main():
    if os.path.isdir(DST):
        shutil.rmtree(DST)
    shutil.copytree(SRC, DST, ignore=shutil.ignore_patterns('_obj*'))
    # the Makefile includes ../../include relative to csrc
    mk = open(os.path.join(DST, 'Makefile')).read()
    mk = mk.replace('-I../../include', '-I%s' % os.path.join(ROOT, 'include'))
    mk = mk.replace('../../include/micall_hip.h', os.path.join(ROOT, 'include', 'micall_hip.h'))
    open(os.path.join(DST, 'Makefile'), 'w').write(mk)
    p = os.path.join(DST, 'mh_map.hip')
    t = open(p).read()
    t = sub(t, 'template <int LOCAL, int ROUND>\n__global__ __launch_bounds__(256) void k_dp(DpArgs A)',
            '__device__ unsigned long long g_ph[2][8];\n'
            'template <int LOCAL, int ROUND>\n__global__ __launch_bounds__(256) void k_dp(DpArgs A)')
    t = sub(t, '    bool pend = false;     // half 0 holds an item waiting for the DP\n',
            '    bool pend = false;     // half 0 holds an item waiting for the DP\n'
            '    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n'
            '    unsigned long long t0 = __builtin_readcyclecounter(), t1;\n'
            '#define PH(k) do { wave_sync(); t1 = __builtin_readcyclecounter(); ph[k] += t1 - t0; t0 = t1; } while (0)\n')
    t = sub(t, '        const XView X = h ? X1 : X0;\n',
            '        const XView X = h ? X1 : X0;\n        PH(6);\n')
    t = sub(t, '            stage_ext<LOCAL>(A, it, X, lane);\n        }\n        wave_sync();\n',
            '            stage_ext<LOCAL>(A, it, X, lane);\n        }\n        wave_sync();\n        PH(0);\n')
    t = sub(t, '        n_fast += fast;\n', '        n_fast += fast;\n        PH(1);\n')
    t = sub(t, '            finish_ext<LOCAL>(A, it, X, bits, 32 * h, best, bi, bl, lane, ck_base, ck_left, low);\n',
            '            finish_ext<LOCAL>(A, it, X, bits, 32 * h, best, bi, bl, lane, ck_base, ck_left, low);\n'
            '            PH(3);\n')
    t = sub(t, '            dp_pair<LOCAL>(A, X0, X1, P.m, it.m, P.hb, it.hb, bits, lane, b0, i0, l0, b1, i1, l1);\n'
               '            wave_sync();\n',
            '            dp_pair<LOCAL>(A, X0, X1, P.m, it.m, P.hb, it.hb, bits, lane, b0, i0, l0, b1, i1, l1);\n'
            '            wave_sync();\n            PH(2);\n')
    t = sub(t, '            finish_ext<LOCAL>(A, it, X1, bits, 32, b1, i1, l1, lane, ck_base, ck_left);\n'
               '            pend = false;\n',
            '            finish_ext<LOCAL>(A, it, X1, bits, 32, b1, i1, l1, lane, ck_base, ck_left);\n'
            '            pend = false;\n            PH(4);\n')
    t = sub(t, '    if (lane == 0 && n_fast) atomicAdd(&A.pool_ctr[2], n_fast);\n}',
            '    if (lane == 0 && n_fast) atomicAdd(&A.pool_ctr[2], n_fast);\n'
            '    PH(5);\n'
            '    if (lane == 0) for (int k = 0; k < 8; ++k) atomicAdd(&g_ph[LOCAL][k], ph[k]);\n}')
    # the traceback walk inside finish_ext, summed into ph[7]
    t = sub(t, 'int &ck_left, int fast_low = -2)\n{\n',
            'int &ck_left, unsigned long long &fw, int fast_low = -2)\n{\n'
            '    const unsigned long long f0 = __builtin_readcyclecounter();\n')
    t = sub(t, '    const WalkOut W = walk1<LOCAL>(A, it, X, bits, hcol, best, bi, bl, lane, fast_low);\n    wave_sync();\n',
            '    const WalkOut W = walk1<LOCAL>(A, it, X, bits, hcol, best, bi, bl, lane, fast_low);\n    wave_sync();\n'
            '    fw += __builtin_readcyclecounter() - f0;\n')
    t = t.replace('ck_base, ck_left, low);', 'ck_base, ck_left, ph[7], low);')
    t = t.replace('lane, ck_base, ck_left);', 'lane, ck_base, ck_left, ph[7]);')
    t = sub(t, '            M.last_fast = ctr[3];\n',
            '            M.last_fast = ctr[3];\n'
            '            {\n'
            '                unsigned long long ph[2][8];\n'
            '                MH_HIP(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_ph), sizeof(ph)));\n'
            '                const int L = par.mode == MH_LOCAL;\n'
            '                double tot = 0;\n'
            '                for (int k = 0; k < 7; ++k) tot += (double)ph[L][k];\n'
            '                fprintf(stderr, "KDP_PHASES mode=%s stage=%.4f fasttry=%.4f rows=%.4f '
            'finish_fast=%.4f finish_pair=%.4f tail=%.4f loopctl=%.4f walk=%.4f total_gcyc=%.3f work=%d fast=%d rescue=%d\\n",\n'
            '                        L ? "local" : "e2e", ph[L][0] / tot, ph[L][1] / tot, ph[L][2] / tot,\n'
            '                        ph[L][3] / tot, ph[L][4] / tot, ph[L][5] / tot, ph[L][6] / tot, ph[L][7] / tot, tot / 1e9,\n'
            '                        ctr[0], ctr[3], ctr[4]);\n'
            '                memset(ph, 0, sizeof(ph));\n'
            '                MH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ph), ph, sizeof(ph)));\n'
            '            }\n')
    open(p, 'w').write(t)
    print('patched', p)


if __name__ == '__main__':
    main()
