#!/usr/bin/env python3
"""
tests/golden/gen_regions.py -- derives the product's default region table
micall-lite_amd/micall_amd/data/micall_regions.json from the reference's
micall/projects.json (data, not code).  Dev container only.

Kept: every region's joined reference sequence and seed group (remap.py:450-454,
project_config.py:114-121) and, per project, its seed region names
(project_config.py:43-66).  The product also reads the reference's own
projects.json format directly when one is passed with json=/--projects.
"""
import json
import os
import sys

REF = os.environ.get('MICALL_REFERENCE', '/root/reference')
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, 'micall-lite_amd', 'micall_amd', 'data', 'micall_regions.json')


def main():
    with open(os.path.join(REF, 'micall', 'projects.json')) as f:
        cfg = json.load(f)
    regions = {name: {'seq': ''.join(r['reference']), 'seed_group': r['seed_group']}
               for name, r in cfg['regions'].items()}
    projects = {}
    for pname, p in cfg['projects'].items():
        seeds = set()
        for r in p['regions']:
            seeds.update(r['seed_region_names'])
        projects[pname] = sorted(seeds)
    out = {'source': 'derived from MiCall-Lite micall/projects.json by tests/golden/gen_regions.py',
           'project_seed_regions': projects, 'regions': regions}
    with open(OUT, 'w') as f:
        json.dump(out, f, indent=1, sort_keys=False)
    print('wrote', OUT, len(regions), 'regions')


if __name__ == '__main__':
    sys.exit(main())
