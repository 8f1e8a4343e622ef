"""Throwaway k_seed phase clock (like kdp_phases.py): copies
micall-lite_amd/csrc to variants/sphases/src and stamps s_memtime in
seed_read around its phases (the seed windows and N count, the hash probes,
the hit loads, the clustering) plus the chunk loop around them; prints the
shares after every mapping pass.

    python profiles/diag/seed_phases.py && make -C variants/sphases/src -j8 \
        OUTDIR=.. OBJDIR=_obj
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, 'micall-lite_amd', 'csrc')
DST = os.path.join(ROOT, 'variants', 'sphases', 'src')


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
    t = sub(t, '__device__ int seed_read(const SeedArgs &A, int64_t r, int m, int64_t off, int lane, uint64_t *hits,\n'
               '                         Cand *best)\n{\n',
            '__device__ unsigned long long g_sph[2][8];\n'
            '#define SPH(k) do { wave_sync(); t1 = __builtin_readcyclecounter(); ph[k] += t1 - t0; t0 = t1; } while (0)\n'
            '__device__ int seed_read(const SeedArgs &A, int64_t r, int m, int64_t off, int lane, uint64_t *hits,\n'
            '                         Cand *best, unsigned long long *ph, unsigned long long &t0)\n{\n'
            '    unsigned long long t1;\n')
    t = sub(t, '    nn = wave_sum(nn);\n', '    nn = wave_sum(nn);\n    SPH(1);\n')
    t = sub(t, '    const int pre = wave_excl_scan(cnt, lane);\n',
            '    SPH(2);\n    const int pre = wave_excl_scan(cnt, lane);\n')
    t = sub(t, '    if (total == 0) {\n        if (lane == 0) A.n_cand[r] = 0;\n        return 0;\n    }\n',
            '    SPH(3);\n    if (total == 0) {\n        if (lane == 0) A.n_cand[r] = 0;\n        return 0;\n    }\n')
    t = sub(t, '    __shared__ int32_t sh_work[4][SEED_CHUNK * MAXCAND];\n',
            '    __shared__ int32_t sh_work[4][SEED_CHUNK * MAXCAND];\n'
            '    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n'
            '    unsigned long long t0 = __builtin_readcyclecounter(), t1;\n')
    t = sub(t, '            const int nc = seed_read(A, r, m, off, lane, sh_hits[wv], sh_best[wv]);\n',
            '            SPH(0);\n'
            '            const int nc = seed_read(A, r, m, off, lane, sh_hits[wv], sh_best[wv], ph, t0);\n'
            '            SPH(4);\n')
    t = sub(t, '        for (int x = lane; x < n_work; x += 64) A.work[base + x] = sh_work[wv][x];\n        wave_sync();\n    }\n}',
            '        for (int x = lane; x < n_work; x += 64) A.work[base + x] = sh_work[wv][x];\n        wave_sync();\n'
            '        SPH(5);\n    }\n'
            '    if (lane == 0) for (int k = 0; k < 8; ++k) atomicAdd(&g_sph[A.I.seedlen == 20][k], ph[k]);\n}')
    t = sub(t, '            M.last_fast = ctr[3];\n',
            '            M.last_fast = ctr[3];\n'
            '            {\n'
            '                unsigned long long ph[2][8];\n'
            '                MH_HIP(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_sph), sizeof(ph)));\n'
            '                for (int L = 0; L < 2; ++L) {\n'
            '                    double tot = 0;\n'
            '                    for (int k = 0; k < 8; ++k) tot += (double)ph[L][k];\n'
            '                    if (tot > 0) fprintf(stderr, "SEED_PHASES seedlen20=%d loop=%.4f windows=%.4f probe=%.4f hits=%.4f '
            'cluster=%.4f chunk=%.4f total_gcyc=%.3f\\n", L, ph[L][0] / tot, ph[L][1] / tot, ph[L][2] / tot, '
            'ph[L][3] / tot, ph[L][4] / tot, ph[L][5] / tot, tot / 1e9);\n'
            '                }\n'
            '                memset(ph, 0, sizeof(ph));\n'
            '                MH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sph), ph, sizeof(ph)));\n'
            '            }\n')
    open(p, 'w').write(t)
    print('patched', p)


if __name__ == '__main__':
    main()
