"""Throwaway k_rescue phase clock (like kdp_phases.py): copies
micall-lite_amd/csrc to variants/rphases/src, stamps s_memtime around the
phases of k_rescue (the per-pair test, the mate's staging, the window's
staging, the diagonal counts, the tail) and prints the shares after every
mapping pass.

    python profiles/diag/rescue_phases.py && make -C variants/rphases/src -j8 \
        OUTDIR=.. OBJDIR=_obj
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, 'micall-lite_amd', 'csrc')
DST = os.path.join(ROOT, 'variants', 'rphases', 'src')


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
    p = os.path.join(DST, 'mh_map.hip')
    t = open(p).read()
    t = sub(t, '__global__ __launch_bounds__(256) void k_rescue(RescueArgs A)\n{\n',
            '__device__ unsigned long long g_rph[8];\n'
            '__global__ __launch_bounds__(256) void k_rescue(RescueArgs A)\n{\n'
            '    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n'
            '    unsigned long long t0 = __builtin_readcyclecounter(), t1;\n'
            '#define RPH(k) do { wave_sync(); t1 = __builtin_readcyclecounter(); ph[k] += t1 - t0; t0 = t1; } while (0)\n')
    t = sub(t, '        uint64_t todo = __builtin_amdgcn_ballot_w64(need != 0);\n',
            '        uint64_t todo = __builtin_amdgcn_ballot_w64(need != 0);\n        RPH(0);\n')
    t = sub(t, '            const bool any_read_n = __builtin_amdgcn_ballot_w64(read_n) != 0;\n',
            '            const bool any_read_n = __builtin_amdgcn_ballot_w64(read_n) != 0;\n            RPH(1);\n')
    t = sub(t, '                    pl[w] = make_uint2(pl0, pl1);\n                }\n                wave_sync();\n',
            '                    pl[w] = make_uint2(pl0, pl1);\n                }\n                wave_sync();\n'
            '                RPH(2);\n')
    t = sub(t, '            const int mmax = wave_max(bestM);\n',
            '            RPH(3);\n            const int mmax = wave_max(bestM);\n')
    t = sub(t, '            if (lane < n_items) A.work[base + lane] = sh_items[wv][lane];\n        }\n        wave_sync();\n    }\n}',
            '            if (lane < n_items) A.work[base + lane] = sh_items[wv][lane];\n        }\n        wave_sync();\n'
            '        RPH(4);\n    }\n'
            '    if (lane == 0) for (int k = 0; k < 8; ++k) atomicAdd(&g_rph[k], ph[k]);\n}')
    t = sub(t, '                if (int st = launch_dp(M.rwork, M.counters + 4,',
            '                {\n'
            '                    unsigned long long ph[8];\n'
            '                    MH_HIP(hipStreamSynchronize(s));\n'
            '                    MH_HIP(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_rph), sizeof(ph)));\n'
            '                    double tot = 0;\n'
            '                    for (int k = 0; k < 8; ++k) tot += (double)ph[k];\n'
            '                    fprintf(stderr, "RESCUE_PHASES test=%.4f read=%.4f window=%.4f count=%.4f '
            'tail=%.4f total_gcyc=%.3f\\n", ph[0] / tot, ph[1] / tot, ph[2] / tot, ph[3] / tot, '
            'ph[4] / tot, tot / 1e9);\n'
            '                    memset(ph, 0, sizeof(ph));\n'
            '                    MH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_rph), ph, sizeof(ph)));\n'
            '                }\n'
            '                if (int st = launch_dp(M.rwork, M.counters + 4,')
    open(p, 'w').write(t)
    print('patched', p)


if __name__ == '__main__':
    main()
