#!/usr/bin/env python3
"""
tests/golden/gen_regions.py -- derives the product's default region table
micall-lite_amd/micall_amd/data/micall_regions.json from the reference's
micall/projects.json (data, not code).  Dev container only.

Kept: every region's joined reference sequence and seed group (remap.py:450-454,
project_config.py:114-121), per project its seed region names
(project_config.py:43-66) and its (coordinate region, seed names) links
(project_config.py:72-85).  Also writes data/gotoh_models.json: the
EmpHIV25 and HYPHY_NUC score matrices of micall/alignment/models/ (data)
that aln2counts and remap align with.  The product also reads the reference's own
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
    projects, links = {}, {}
    for pname, p in cfg['projects'].items():
        seeds = set()
        for r in p['regions']:
            seeds.update(r['seed_region_names'])
        projects[pname] = sorted(seeds)
        links[pname] = [[r['coordinate_region'], list(r['seed_region_names'])] for r in p['regions']]
    out = {'source': 'derived from MiCall-Lite micall/projects.json by tests/golden/gen_regions.py',
           'project_seed_regions': projects, 'project_regions': links, 'regions': regions}
    with open(OUT, 'w') as f:
        json.dump(out, f, indent=1, sort_keys=False)
    print('wrote', OUT, len(regions), 'regions')
    models = {}
    for name in ('EmpHIV25', 'HYPHY_NUC'):
        with open(os.path.join(REF, 'micall', 'alignment', 'models', name + '.csv')) as f:
            lines = f.read().splitlines()
        models[name] = {'alphabet': ''.join(lines[0].split(',')),
                        'matrix': [int(v) for line in lines[1:] if line for v in line.split(',')]}
    path = os.path.join(os.path.dirname(OUT), 'gotoh_models.json')
    with open(path, 'w') as f:
        json.dump(models, f)
    print('wrote', path)


if __name__ == '__main__':
    sys.exit(main())
