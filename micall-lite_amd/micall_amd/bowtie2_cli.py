"""
bowtie2 / bowtie2-build-s commands over the HIP mapper.

The reference runs its mapper as a subprocess (micall/utils/externals.py:
158-203) from prelim_map.py:106-134 and remap.py:695-734; SURVEY.md 8(b) is
the observed contract.  These commands keep it, so the stock pipeline runs
unchanged with --bt2 / --bt2build (bin/micall) pointed at micall-lite_amd/bin
and maps on the GPU:

    bowtie2-build-s --version      (the first line ends with the version:
                                    externals.py:164-165, :178 read its
                                    last token)
    bowtie2-build-s [--wrapper W] [--quiet] [-f] FASTA TEMPLATE
        The "index" is TEMPLATE.1.bt2, a copy of the reference FASTA; the
        other five names bowtie2-build creates (.2/.3/.4/.rev.1/.rev.2.bt2)
        are written empty, since the caller removes all six.  The device
        k-mer index is built when bowtie2 loads it (a few ms).
    bowtie2 --version
    bowtie2 [--wrapper W] [--quiet] -x TEMPLATE (-1 R1 -2 R2 | -U R)
            [--local] [--rdg O,E] [--rfg O,E] [--no-hd] [-X N] [-p N]
        FASTQ (plain or gzip) -> mh_reads_load_fastq, mh_index_build
        (seed 22 end-to-end, 20 local), mh_map, and the SAM records of
        every read in input order on stdout (mh_format_rows style 0: the
        eleven fields plus AS/XS/XN/XM/XO/XG/NM/YS/YF/YT tags).  Without
        --no-hd the @HD / @SQ / @PG header comes first.  -p is accepted and
        ignored (the device is the parallelism); MICALL_HIP_DEVICE picks
        the GPU, as for the drop-ins.

bowtie2's defaults apply to options left out (--rdg 5,3 --rfg 5,3 -X 500,
end-to-end).  Options the pipeline never passes are refused with exit
status 1, as bowtie2 refuses unknown ones.  Note what this route costs next
to the in-process drop-ins (prelim_map.py / remap.py here): every call
re-reads the FASTQ and the pipeline parses SAM text again, as it does with
bowtie2.
"""
import os
import sys

from . import _native

VERSION = '2.2.8'
BT2_SUFFIXES = ('1', '2', '3', '4', 'rev.1', 'rev.2')
TAKES_VALUE = ('-x', '-1', '-2', '-U', '--rdg', '--rfg', '-X', '-p', '--wrapper')
SWITCHES = ('--local', '--no-hd', '--quiet', '--end-to-end')


class UsageError(Exception):
    pass


def fasta_records(path):
    """(names, sequences) of a FASTA file; a name is its header up to the
    first whitespace, as bowtie2 names references."""
    names, parts = [], []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            if line[0] == '>':
                fields = line[1:].split()
                names.append(fields[0] if fields else '')
                parts.append([])
            elif parts:
                parts[-1].append(line)
    return names, [''.join(p) for p in parts]


def build_main(argv, out=sys.stdout):
    """bowtie2-build-s."""
    if '--version' in argv:
        out.write('bowtie2-build-s version {}\nmicall-lite_amd (HIP mapper)\n'.format(VERSION))
        return 0
    rest, i = [], 0
    while i < len(argv):
        a = argv[i]
        if a == '--wrapper':
            i += 2
            continue
        if a not in ('--quiet', '-f'):
            rest.append(a)
        i += 1
    if len(rest) != 2:
        raise UsageError('bowtie2-build-s: expected FASTA and TEMPLATE, got {!r}'.format(rest))
    fasta, template = rest
    names, seqs = fasta_records(fasta)
    with open(template + '.1.bt2', 'w') as f:
        for name, seq in zip(names, seqs):
            f.write('>{}\n{}\n'.format(name, seq))
    for suffix in BT2_SUFFIXES[1:]:
        open('{}.{}.bt2'.format(template, suffix), 'w').close()
    return 0


def parse_align_args(argv):
    opts, switches = {}, set()
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in TAKES_VALUE:
            if i + 1 >= len(argv):
                raise UsageError('bowtie2: option {} needs a value'.format(a))
            opts[a] = argv[i + 1]
            i += 2
        elif a in SWITCHES:
            switches.add(a)
            i += 1
        else:
            raise UsageError('bowtie2: unsupported option {!r}'.format(a))
    if '-x' not in opts:
        raise UsageError('bowtie2: -x TEMPLATE is required')
    if ('-1' in opts) != ('-2' in opts) or ('-1' in opts) == ('-U' in opts):
        raise UsageError('bowtie2: give either -1 R1 -2 R2 or -U R')
    return opts, switches


def pair_of(text):
    o, e = text.split(',')
    return int(o), int(e)


def sam_header(names, seqs, argv):
    lines = ['@HD\tVN:1.0\tSO:unsorted\n']
    lines += ['@SQ\tSN:{}\tLN:{}\n'.format(n, len(s)) for n, s in zip(names, seqs)]
    lines.append('@PG\tID:bowtie2\tPN:bowtie2\tVN:{}\tCL:"{}"\n'.format(VERSION, ' '.join(argv)))
    return ''.join(lines)


def align_main(argv, out=sys.stdout, device=None):
    """bowtie2 (bowtie2-align-s)."""
    if '--version' in argv:
        out.write('bowtie2-align-s version {}\nmicall-lite_amd (HIP mapper)\n'.format(VERSION))
        return 0
    opts, switches = parse_align_args(argv)
    names, seqs = fasta_records(opts['-x'] + '.1.bt2')
    mode = _native.LOCAL if '--local' in switches else _native.E2E
    par = _native.params(mode, rdg=pair_of(opts.get('--rdg', '5,3')),
                         rfg=pair_of(opts.get('--rfg', '5,3')), maxins=int(opts.get('-X', '500')))
    if device is None:   # the drop-ins' device choice (session.py)
        device = int(os.environ.get('MICALL_HIP_DEVICE', '0'))
    ctx = _native.Context(device)
    try:
        if '-1' in opts:
            ctx.reads_load_fastq(opts['-1'], opts['-2'])
        else:
            ctx.reads_load_fastq(opts['-U'])
        ctx.index_build(names, seqs, 20 if mode == _native.LOCAL else 22)
        ctx.map(par)
        if '--no-hd' not in switches:
            out.write(sam_header(names, seqs, argv))
        ctx.write_rows(out, 0)
        out.flush()
    finally:
        ctx.close()
    return 0


def main(which, argv=None):
    argv = sys.argv[1:] if argv is None else argv
    try:
        return build_main(argv) if which == 'build' else align_main(argv)
    except (UsageError, OSError, _native.NativeError, _native.NativeUnavailable) as e:
        sys.stderr.write('{}\n'.format(e))
        return 1


if __name__ == '__main__':
    sys.exit(main('align'))
