"""
Replays tests/golden/aln2counts_golden.json -- every call
micall/tests/aln2counts_test.py makes on SequenceReport, InsertionWriter,
SeedAmino and SeedNucleotide, recorded around the reference code by
tests/golden/gen_golden.py a2c with what each call wrote, returned or raised
-- against another implementation of those classes: the device drop-in
(micall_amd.aln2counts) or the oracle (oracle/og_aln2counts.py).
"""
import io
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden',
                      'aln2counts_golden.json')


def scripts():
    with open(GOLDEN) as f:
        return json.load(f)['scripts']


def _stubbed(report_cls):
    class Stubbed(report_cls):
        """StubbedSequenceReport (aln2counts_test.py:11-36): alignment overrides."""
        overrides = None

        def _pair_align(self, reference, query, *args, **kwargs):
            hit = (self.overrides or {}).get((reference, query))
            return hit if hit is not None else report_cls._pair_align(self, reference, query)
    return Stubbed


def replay(script, impl):
    """impl: dict(SequenceReport=, InsertionWriter=, SeedAmino=,
    SeedNucleotide=, projects=callable(config dict)).  Returns the list of
    mismatches (empty when every call wrote / returned / raised the same)."""
    objs, files, bad = {}, {}, []
    report_cls = _stubbed(impl['SequenceReport'])
    for k, c in enumerate(script['calls']):
        op = c['op']
        where = '{} #{} {}'.format(script['test'], k, op)
        f = n0 = None
        summary = None
        try:
            if op == 'InsertionWriter':
                f = files.setdefault(c['file'], io.StringIO())
                n0 = len(f.getvalue())
                w = objs[c['obj']] = impl['InsertionWriter'](f)
                w._replay_file = f
                got = None
            elif op == 'SequenceReport':
                objs[c['obj']] = report_cls(objs[c['writer']], None, c['cutoffs'])
                continue
            elif op == 'SeedAmino':
                a = objs[c['obj']] = impl['SeedAmino'](c['index'])
                for t, nuc in zip(c['nucs'], a.nucleotides):
                    objs[t] = nuc
                continue
            elif op == 'SeedNucleotide':
                objs[c['obj']] = impl['SeedNucleotide']()
                continue
            else:
                obj = objs[c['obj']]
                if op == 'read':
                    obj.projects = impl['projects'](c['config'])
                    obj.overrides = {(a, b): tuple(v) for a, b, v in c['overrides']}
                    got = obj.read(c['rows'])
                elif 'file' in c:
                    f = files.setdefault(c['file'], io.StringIO())
                    n0 = len(f.getvalue())
                    kwargs = {}
                    if 'summary_in' in c:
                        summary = dict(c['summary_in'])
                        kwargs['coverage_summary'] = summary
                    got = getattr(obj, op)(f, **kwargs)
                elif op in ('write_insertions', 'write'):
                    f = (obj.insert_writer if op == 'write_insertions' else obj)._replay_file
                    n0 = len(f.getvalue())
                    got = getattr(obj, op)(*c['args'], **c['kwargs'])
                else:
                    got = getattr(obj, op)(*c['args'], **c['kwargs'])
        except Exception as ex:
            if c.get('raises') != type(ex).__name__:
                bad.append('{}: raised {!r}'.format(where, ex))
            continue
        if 'raises' in c:
            bad.append('{}: expected {}'.format(where, c['raises']))
            continue
        if 'out' in c and f.getvalue()[n0:] != c['out']:
            bad.append('{}: wrote {!r}, want {!r}'.format(where, f.getvalue()[n0:], c['out']))
        if 'result' in c and got != c['result']:
            bad.append('{}: returned {!r}, want {!r}'.format(where, got, c['result']))
        if 'summary_out' in c and summary != c['summary_out']:
            bad.append('{}: summary {!r}, want {!r}'.format(where, summary, c['summary_out']))
    return bad
