#!/usr/bin/env python3
"""
oracle/bowtie2_shim.py -- TEST INFRASTRUCTURE ONLY.

A bowtie2 / bowtie2-build-s stand-in with the command-line contract the
reference uses (micall/utils/externals.py:161-203, prelim_map.py:106-134,
remap.py:695-734; observed contract in SURVEY.md 8(b)), backed by the CPU
oracle mapper.  It lets the stock reference pipeline (prelim_map -> remap ->
sam2aln) run in the dev container and produce the golden CSVs of
tests/golden/e2e/.  Invoked through oracle/shim_bin/{bowtie2,bowtie2-build-s}.

  bowtie2-build-s --version | [--wrapper W] [--quiet] -f FASTA TEMPLATE
      writes TEMPLATE.{1,2,3,4,rev.1,rev.2}.bt2 (the .1.bt2 holds the FASTA)
  bowtie2 --version | [--wrapper W] [--quiet] -x TEMPLATE (-1 R1 -2 R2 | -U R)
          [--rdg O,E] [--rfg O,E] [--local] [--no-hd] [-X N] [-p N]
      prints SAM records (input order) to stdout
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import oracle  # noqa: E402

SUFFIXES = ['1', '2', '3', '4', 'rev.1', 'rev.2']


def read_fasta(path):
    names, seqs = [], []
    with open(path) as f:
        for line in f:
            line = line.rstrip('\n')
            if line.startswith('>'):
                names.append(line[1:].split()[0])
                seqs.append([])
            elif names:
                seqs[-1].append(line.strip())
    return names, [''.join(s) for s in seqs]


def build(argv):
    if '--version' in argv:
        print('/usr/bin/bowtie2-build-s version 2.2.8 (oracle shim)')
        return 0
    args = [a for a in argv if a not in ('--quiet', '-f')]
    if '--wrapper' in args:
        i = args.index('--wrapper')
        del args[i:i + 2]
    fasta, template = args[-2], args[-1]
    names, seqs = read_fasta(fasta)
    with open(template + '.1.bt2', 'w') as f:
        for n, s in zip(names, seqs):
            f.write('>%s\n%s\n' % (n, s))
    for suffix in SUFFIXES[1:]:
        open('%s.%s.bt2' % (template, suffix), 'w').close()
    return 0


def align(argv):
    if '--version' in argv:
        print('/usr/bin/bowtie2-align-s version 2.2.8 (oracle shim)')
        return 0
    opts = {}
    flags = set()
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ('-x', '-1', '-2', '-U', '--rdg', '--rfg', '-X', '-p', '--wrapper'):
            opts[a] = argv[i + 1]
            i += 2
        else:
            flags.add(a)
            i += 1
    names, seqs = read_fasta(opts['-x'] + '.1.bt2')
    mode = oracle.LOCAL if '--local' in flags else oracle.E2E
    rdg = tuple(int(x) for x in opts.get('--rdg', '5,3').split(','))
    rfg = tuple(int(x) for x in opts.get('--rfg', '5,3').split(','))
    maxins = int(opts.get('-X', '500'))
    if '-1' in opts:
        lines = oracle.map_fastq_to_sam(names, seqs, mode, opts['-1'], opts['-2'], rdg, rfg, maxins)
    else:
        lines = oracle.map_fastq_to_sam(names, seqs, mode, opts['-U'], None, rdg, rfg, maxins)
    out = sys.stdout
    for line in lines:
        out.write(line)
    out.flush()
    return 0


def main():
    if sys.argv[1:2] == ['--shim-build']:
        return build(sys.argv[2:])
    return align(sys.argv[2:] if sys.argv[1:2] == ['--shim-align'] else sys.argv[1:])


if __name__ == '__main__':
    sys.exit(main())
