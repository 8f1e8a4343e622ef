"""
Project / seed-reference configuration for the remap path.

Mirrors the parts of micall/core/project_config.py that prelim_map, remap and
aln2counts use: loadDefault / loadCustom / load (:28-41), writeSeedFasta
(:43-66), getReference (:68-70), getCoordinateReferences (:72-85),
getSeedGroup (:114-121), and the `seeds` dict remap builds from every region
(remap.py:450-454).  The default table is
data/micall_regions.json (derived from the reference's projects.json); a
custom file in the reference's own projects.json format is read as is.
"""
import json
import os

DEFAULT_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data',
                            'micall_regions.json')


class ProjectConfig(object):
    def __init__(self, regions=None, project_seed_regions=None, json_file=None,
                 project_regions=None):
        self.regions = regions or {}                # {name: {'seq', 'seed_group'}}
        self.project_seed_regions = project_seed_regions or {}  # {project: [seed names]}
        # {project: [[coordinate region, [seed names]], ...]} in file order
        self.project_regions = project_regions or {}
        self.json_file = json_file

    @classmethod
    def from_config(cls, cfg, json_file=None):
        """From a parsed projects file: the reference's projects.json format
        or this package's data/micall_regions.json."""
        if 'project_seed_regions' in cfg:
            return cls(cfg['regions'], cfg['project_seed_regions'], json_file,
                       cfg.get('project_regions'))
        regions = {name: {'seq': ''.join(r['reference']), 'seed_group': r.get('seed_group')}
                   for name, r in cfg['regions'].items()}
        projects, links = {}, {}
        for pname, p in cfg['projects'].items():
            seeds = set()
            for r in p['regions']:
                seeds.update(r['seed_region_names'])
            projects[pname] = sorted(seeds)
            links[pname] = [[r['coordinate_region'], list(r['seed_region_names'])]
                            for r in p['regions']]
        return cls(regions, projects, json_file, links)

    def load(self, json_file):
        """project_config.ProjectConfig.load (:39-41) from an open file."""
        other = self.from_config(json.load(json_file), getattr(json_file, 'name', None))
        self.__dict__.update(other.__dict__)

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
        return cls.from_config(cfg, json_path)

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

    def getCoordinateReferences(self, seed_region):
        """{coordinate region: reference bytes} linked to a seed, in file
        order (project_config.py:72-85)."""
        coord_refs = {}
        for links in self.project_regions.values():
            for coord_region, seed_names in links:
                if seed_region in seed_names and coord_region:
                    coord_refs[coord_region] = self.getReference(coord_region)
        return coord_refs

    def getSeedGroup(self, seed_region):
        return self.regions[seed_region]['seed_group']

    def all_region_sequences(self):
        """remap's `seeds`: every region, in file order (remap.py:450-454)."""
        return {name: r['seq'] for name, r in self.regions.items()}


def load_default():
    return ProjectConfig.loadDefault()


def load(json_path=None):
    return ProjectConfig.loadDefault() if json_path is None else ProjectConfig.loadCustom(json_path)
