"""profiles/diag/e2e_profile.py -- cProfile of bench.end_to_end (prelim_map()
then remap() file to file on the C2 input) on the GPU box.
    python3 profiles/diag/e2e_profile.py [pairs]"""
import cProfile
import os
import pstats
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import bench  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
with tempfile.TemporaryDirectory(dir='/tmp') as d:
    prof = cProfile.Profile()
    real = bench.end_to_end

    # profile only prelim_map / remap (not the FASTQ writing)
    from micall_amd import prelim_map, remap
    for mod, name in ((prelim_map, 'prelim_map'), (remap, 'remap')):
        fn = getattr(mod, name)

        def wrap(*a, _fn=fn, **kw):
            prof.enable()
            try:
                return _fn(*a, **kw)
            finally:
                prof.disable()
        setattr(mod, name, wrap)
    out = real(pairs, d)
    print({k: out[k] for k in ('value', 'seconds', 'prelim_map_s', 'remap_s')})
    pstats.Stats(prof).sort_stats('tottime').print_stats(30)
