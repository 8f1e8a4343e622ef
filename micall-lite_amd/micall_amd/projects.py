"""
Project / seed-reference configuration for the remap path.

Mirrors the parts of micall/core/project_config.py that prelim_map and remap
use: loadDefault / loadCustom (:28-41), writeSeedFasta (:43-66),
getReference (:68-70), getSeedGroup (:114-121), and the `seeds` dict remap
builds from every region (remap.py:450-454).  The default table is
data/micall_regions.json (derived from the reference's projects.json); a
custom file in the reference's own projects.json format is read as is.
"""
import json
import os

DEFAULT_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data',
                            'micall_regions.json')


class ProjectConfig(object):
    def __init__(self, regions, project_seed_regions, json_file=None):
        self.regions = regions                      # {name: {'seq', 'seed_group'}}
        self.project_seed_regions = project_seed_regions  # {project: [seed names]}
        self.json_file = json_file

    @classmethod
    def loadDefault(cls):
        return cls.loadCustom(DEFAULT_PATH)

    @classmethod
    def loadCustom(cls, json_path):
        try:
            with open(json_path) as f:
                cfg = json.load(f)
        except Exception as ex:
            raise RuntimeError('No project definitions found in {!r}'.format([json_path])) from ex
        if 'project_seed_regions' in cfg:
            return cls(cfg['regions'], cfg['project_seed_regions'], json_path)
        regions = {name: {'seq': ''.join(r['reference']), 'seed_group': r['seed_group']}
                   for name, r in cfg['regions'].items()}
        projects = {}
        for pname, p in cfg['projects'].items():
            seeds = set()
            for r in p['regions']:
                seeds.update(r['seed_region_names'])
            projects[pname] = sorted(seeds)
        return cls(regions, projects, json_path)

    def seed_names(self):
        """Sorted seed region names (project_config.py:48-55)."""
        names = set()
        for seeds in self.project_seed_regions.values():
            names.update(seeds)
        return sorted(names)

    def seed_sequences(self):
        """{seed name: sequence} in writeSeedFasta order; raises on duplicate
        sequences like the reference (project_config.py:57-64)."""
        out, by_seq = {}, {}
        for name in self.seed_names():
            seq = self.regions[name]['seq']
            dup = by_seq.get(seq)
            if dup is not None:
                raise RuntimeError('Duplicate references: {} and {}.'.format(dup, name))
            by_seq[seq] = name
            out[name] = seq
        return out

    def writeSeedFasta(self, fasta_file):
        for name, seq in self.seed_sequences().items():
            fasta_file.write('>{name}\n{ref}\n'.format(name=name, ref=seq))

    def getReference(self, region_name):
        return self.regions[region_name]['seq'].encode('utf-8')

    def getSeedGroup(self, seed_region):
        return self.regions[seed_region]['seed_group']

    def all_region_sequences(self):
        """remap's `seeds`: every region, in file order (remap.py:450-454)."""
        return {name: r['seq'] for name, r in self.regions.items()}


def load_default():
    return ProjectConfig.loadDefault()


def load(json_path=None):
    return ProjectConfig.loadDefault() if json_path is None else ProjectConfig.loadCustom(json_path)
