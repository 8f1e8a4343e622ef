"""Throwaway k_dp census (like kdp_phases.py): copies micall-lite_amd/csrc to
variants/kfail/src and counts, per mode, the extensions whose best cell ends
below --score-min (no alignment) against all extensions, printed after every
mapping pass.

    python profiles/diag/kdp_fail.py && make -C variants/kfail/src -j8 \
        OUTDIR=.. OBJDIR=_obj
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, 'micall-lite_amd', 'csrc')
DST = os.path.join(ROOT, 'variants', 'kfail', 'src')


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
    t = sub(t, 'template <int LOCAL>\n__device__ WalkOut walk1(',
            '__device__ unsigned long long g_fail[2][3];\n'
            'template <int LOCAL>\n__device__ WalkOut walk1(')
    t = sub(t, '    fast_low = __builtin_amdgcn_readfirstlane(fast_low);\n',
            '    fast_low = __builtin_amdgcn_readfirstlane(fast_low);\n'
            '    if (lane == 0) {\n'
            '        atomicAdd(&g_fail[LOCAL][0], 1ull);\n'
            '        if (!(!(LOCAL && best <= 0) && best >= minsc)) atomicAdd(&g_fail[LOCAL][1], 1ull);\n'
            '        if (fast_low > -2) atomicAdd(&g_fail[LOCAL][2], 1ull);\n'
            '    }\n')
    # the end-to-end row bound: after each 8-row group inside both reads, the
    # half's best H of the row (no later row adds to an end-to-end score);
    # the first group where it is below --score-min, per half
    t = sub(t, 'template <int LOCAL>\n__device__ void dp_pair(',
            '__device__ unsigned long long g_bound[6];\n'
            'template <int LOCAL>\n__device__ void dp_pair(')
    t = sub(t, '    const int mlo = m0 < m1 ? m0 : m1, mhi = m0 < m1 ? m1 : m0;\n',
            '    const int mlo = m0 < m1 ? m0 : m1, mhi = m0 < m1 ? m1 : m0;\n'
            '    const int ms0 = A.len_tab[(MAXLEN + 1) + m0], ms1 = A.len_tab[(MAXLEN + 1) + m1];\n'
            '    int f0 = -1, f1 = -1;\n')
    t = sub(t, '        bits[(i0 >> 3) * 64 + lane] = acc;\n    }\n',
            '        bits[(i0 >> 3) * 64 + lane] = acc;\n'
            '        if (!LOCAL && i0 + 8 <= mlo) {\n'
            '            const int hv = live ? Hp - BIAS - A.exD * lane - 8 * (i0 + 8) : INT32_MIN;\n'
            '            const int s = half_scan_max(hv);\n'
            '            const int x0 = __builtin_amdgcn_readlane(s, 31), x1 = __builtin_amdgcn_readlane(s, 63);\n'
            '            if (f0 < 0 && x0 < ms0) f0 = i0 + 8;\n'
            '            if (f1 < 0 && x1 < ms1) f1 = i0 + 8;\n'
            '        }\n'
            '    }\n')
    t = sub(t, '    bl1 = (63 - (int)(k1 & 63)) & 31;\n}\n',
            '    bl1 = (63 - (int)(k1 & 63)) & 31;\n'
            '    if (!LOCAL && lane == 0) {\n'
            '        const bool same = X0.tab == X1.tab;\n'
            '        if (f0 >= 0) atomicAdd(&g_bound[0], 1ull);\n'
            '        if (f0 >= 0 && best0 >= ms0) atomicAdd(&g_bound[5], 1ull);\n'
            '        if (!same && f1 >= 0) atomicAdd(&g_bound[0], 1ull);\n'
            '        if (!same && f1 >= 0 && best1 >= ms1) atomicAdd(&g_bound[5], 1ull);\n'
            '        atomicAdd(&g_bound[1], same ? 1ull : 2ull);\n'
            '        if (f0 >= 0 && (same || f1 >= 0)) {\n'
            '            atomicAdd(&g_bound[2], 1ull);\n'
            '            const int f = same ? f0 : (f0 > f1 ? f0 : f1);\n'
            '            atomicAdd(&g_bound[3], (unsigned long long)(mhi - f));\n'
            '        }\n'
            '        atomicAdd(&g_bound[4], (unsigned long long)mhi);\n'
            '    }\n}\n')
    t = sub(t, '            M.last_fast = ctr[3];\n',
            '            M.last_fast = ctr[3];\n'
            '            {\n'
            '                unsigned long long b[6];\n'
            '                MH_HIP(hipMemcpyFromSymbol(b, HIP_SYMBOL(g_bound), sizeof(b)));\n'
            '                fprintf(stderr, "KDP_BOUND halves_below=%llu halves=%llu waves_both=%llu rows_saved=%llu rows=%llu wrong=%llu\\n",\n'
            '                        b[0], b[1], b[2], b[3], b[4], b[5]);\n'
            '                memset(b, 0, sizeof(b));\n'
            '                MH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_bound), b, sizeof(b)));\n'
            '            }\n')
    t = sub(t, '            M.last_fast = ctr[3];\n',
            '            M.last_fast = ctr[3];\n'
            '            {\n'
            '                unsigned long long f[2][3];\n'
            '                MH_HIP(hipMemcpyFromSymbol(f, HIP_SYMBOL(g_fail), sizeof(f)));\n'
            '                const int L = par.mode == MH_LOCAL;\n'
            '                fprintf(stderr, "KDP_FAIL mode=%s items=%llu below_min=%llu fast=%llu\\n",\n'
            '                        L ? "local" : "e2e", f[L][0], f[L][1], f[L][2]);\n'
            '                memset(f, 0, sizeof(f));\n'
            '                MH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_fail), f, sizeof(f)));\n'
            '            }\n')
    open(p, 'w').write(t)
    print('patched', p)


if __name__ == '__main__':
    main()
