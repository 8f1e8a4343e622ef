"""
oracle/cpu_e2e.py -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline
end-to-end leg and tests/test_cpu_e2e.py).

The reference's file-to-file path restated on the CPU: prelim_map()
(prelim_map.py:96-161) and remap() (remap.py:381-658) with the reference's
own structure -- FASTQ re-read and parsed on every mapping pass, SAM text per
read, prelim.csv written with csv.DictWriter and read back with
csv.DictReader + itertools.groupby, sam_to_conseqs over SAM lines, the
remap loop and its stopping rules, MixedReferenceSplitter, unmapped FASTQs --
with the oracle's C mapper (og_map, OpenMP over read pairs on `nthreads`
threads) standing where bowtie2 -p N stood and the oracle pileup (og_pileup)
under sam_to_conseqs.  On the golden e2e cases it writes the reference's
files byte for byte (tests/test_cpu_e2e.py), so its wall time is an honest
CPU figure for the same work the drop-ins do.
"""
import csv
import gzip
import itertools
import os
from collections import Counter

import oracle

FIELDNAMES = ['qname', 'flag', 'rname', 'pos', 'mapq', 'cigar', 'rnext', 'pnext', 'tlen', 'seq',
              'qual']
COUNT_COLUMNS = 'type count filtered_count seed_dist other_dist other_seed'.split()
CONSENSUS_Q_CUTOFF = 20
MIN_MAPPING_EFFICIENCY = 0.95
MAX_REMAPS = 3
# micall/alignment/models/HYPHY_NUC.csv (remap.py:33's aligner model)
HYPHY_NUC = ([5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
              0, 0, 0, 0, 0], 'ACGT?')
_COMP = str.maketrans('ACGTWRKYSMBDHVN*-', 'TGCASYMRWKVHDBN*-')


def _sam(refnames, refseqs, mode, fastq1, fastq2, nthreads):
    """bowtie2 [--local] -p nthreads stand-in: SAM lines, FASTQ order."""
    return oracle.map_fastq_to_sam(refnames, refseqs, mode, fastq1, fastq2, nthreads=nthreads)


def prelim_map(fastq1, fastq2, prelim_csv, seeds, nthreads):
    """prelim_map.py:96-161: end-to-end over every seed, rows grouped by
    rname in first-seen order."""
    names = list(seeds)
    output = {}
    for line in _sam(names, [seeds[k] for k in names], oracle.E2E, fastq1, fastq2, nthreads):
        items = line.split('\t')
        output.setdefault(items[2], []).append(items[:11])
    writer = csv.DictWriter(prelim_csv, FIELDNAMES, lineterminator=os.linesep)
    writer.writeheader()
    for lines in output.values():
        for line in lines:
            writer.writerow(dict(zip(FIELDNAMES, line)))


def _lines(path):
    opener = gzip.open if path.endswith('.gz') else open
    with opener(path, 'rb') as f:
        return sum(chunk.count(b'\n') for chunk in iter(lambda: f.read(1 << 20), b''))


def _is_short(cigar, max_primer_length=50):
    import re
    return max(int(n) for n in re.findall(r'(\d+)M', cigar)) <= max_primer_length


def _header(refseqs):
    return (['@HD\tVN:1.0\tSO:unsorted\n'] +
            ['@SQ\tSN:%s\tLN:%d\n' % (k, len(v)) for k, v in refseqs.items()] +
            ['@PG\tID:bowtie2\tPN:bowtie2\tVN:2.2.3\tCL:""\n'])


def _map_to_reference(fastq1, fastq2, refseqs, unmapped1, unmapped2, new_counts, nthreads):
    """remap.py:661-761: --local pass; SAM lines (with header) and the
    unmapped count; unmapped reads appended to the FASTQ handles."""
    names = list(refseqs)
    body = _sam(names, [refseqs[k] for k in names], oracle.LOCAL, fastq1, fastq2, nthreads)
    new_counts.clear()
    unmapped = 0
    for line in body:
        qname, flag, rname, _, _, _, _, _, _, seq, qual = line.split('\t')[:11]
        if int(flag) & 4:
            handle = unmapped1 if int(flag) & 0x40 else unmapped2
            if handle:
                handle.write('@%s\n%s\n+\n%s\n' % (qname, seq, qual))
            unmapped += 1
            continue
        new_counts[rname] += 1
    return _header(refseqs) + body, unmapped


def _split(sam_lines, workdir):
    """MixedReferenceSplitter.split (remap.py:780-828): rows that stay,
    and {rname: (R1 path, R2 path)} of the pairs split off."""
    kept, unmatched, splits = [], {}, {}
    for line in sam_lines:
        if line.startswith('@'):
            continue
        fields = line.strip('\n').split('\t')
        if fields[6] in ('=', '*') or int(fields[1]) & 12:
            kept.append(fields[:11])
            continue
        match = unmatched.pop(fields[0], None)
        if match is None:
            unmatched[fields[0]] = fields
            continue
        if fields[4] != match[4]:
            rname = fields[2] if fields[4] > match[4] else match[2]
        else:
            score = [int(t[5:]) for t in fields[11:] if t.startswith('AS:i:')]
            mscore = [int(t[5:]) for t in match[11:] if t.startswith('AS:i:')]
            rname = fields[2] if score and mscore and score[0] > mscore[0] else match[2]
        if rname not in splits:
            splits[rname] = tuple(open(os.path.join(workdir, '%s_R%d.fastq' % (rname, k)), 'w')
                                  for k in (1, 2))
        fwd, rev = (fields, match) if int(fields[1]) & 0x40 else (match, fields)
        splits[rname][0].write('@{}\n{}\n+\n{}\n'.format(fwd[0], fwd[9], fwd[10]))
        splits[rname][1].write('@{}\n{}\n+\n{}\n'.format(rev[0], rev[9][::-1].translate(_COMP),
                                                         rev[10][::-1]))
    for f1, f2 in splits.values():
        f1.close()
        f2.close()
    return kept, {k: (v[0].name, v[1].name) for k, v in splits.items()}


def remap(fastq1, fastq2, prelim_csv, remap_csv, remap_counts_csv, remap_conseq_csv, unmapped1,
          unmapped2, seeds, seed_groups, workdir, nthreads, count_threshold=10):
    """remap.py:381-658.  seeds: every region's reference (projects.json
    'regions'); seed_groups: rname -> seed group."""
    conseqs = dict(seeds)
    raw_count = _lines(fastq1) / 2
    counts_writer = csv.DictWriter(remap_counts_csv, COUNT_COLUMNS, lineterminator=os.linesep)
    counts_writer.writeheader()
    counts_writer.writerow(dict(type='raw', count=raw_count))
    sam = _header(conseqs)
    refgroups = {}
    for refname, group in itertools.groupby(csv.DictReader(prelim_csv), lambda r: r['rname']):
        count = filtered = 0
        for row in group:
            count += 1
            sam.append('\t'.join(row[f] for f in FIELDNAMES) + '\n')
            if int(row['flag']) & 4 or _is_short(row['cigar']):
                continue
            filtered += 1
        counts_writer.writerow(dict(type='prelim %s' % refname, count=count, filtered_count=filtered))
        if refname == '*':
            continue
        threshold = 1 if refname == 'HIV1B-env-seed' else count_threshold
        _best, best = refgroups.get(seed_groups[refname], (None, threshold - 1))
        if filtered > best:
            refgroups[seed_groups[refname]] = (refname, filtered)
    seed_counts = {ref: n for ref, n in refgroups.values()}
    built = oracle.sam_to_conseqs(sam, CONSENSUS_Q_CUTOFF, seeds=seeds, nuc_model=HYPHY_NUC)
    conseqs, map_counts = {}, {}
    for rname, conseq in built.items():
        if rname in seed_counts:
            map_counts[rname] = seed_counts[rname]
            conseqs[rname] = conseq

    n_remaps = 0
    new_counts = Counter()
    unmapped_count = raw_count
    sam = []
    while conseqs:
        for handle in (unmapped1, unmapped2):
            handle.seek(0)
            handle.truncate()
        refseqs = conseqs
        sam, unmapped_count = _map_to_reference(fastq1, fastq2, refseqs, unmapped1, unmapped2,
                                                new_counts, nthreads)
        old_names = set(conseqs)
        report = {}
        conseqs = oracle.sam_to_conseqs(sam, CONSENSUS_Q_CUTOFF, seeds=seeds, is_filtered=True,
                                        filter_coverage=count_threshold / 2, distance_report=report,
                                        nuc_model=HYPHY_NUC)
        n_remaps += 1
        for name in sorted(new_counts):
            counts_writer.writerow(dict(report.get(name, {}), type='remap-%d %s' % (n_remaps, name),
                                        count=new_counts[name]))
        if set(conseqs) == old_names:
            if all(n <= map_counts[name] for name, n in new_counts.items()):
                break
            if sum(new_counts.values()) / float(raw_count) > MIN_MAPPING_EFFICIENCY:
                break
            if n_remaps >= MAX_REMAPS:
                break
        map_counts = dict(new_counts)

    writer = csv.DictWriter(remap_csv, FIELDNAMES, lineterminator=os.linesep)
    writer.writeheader()
    if new_counts:
        kept, splits = _split(sam, workdir)
        for fields in kept:
            writer.writerow(dict(zip(FIELDNAMES, fields)))
        split_counts = Counter()
        for rname, (f1, f2) in splits.items():
            lines, extra = _map_to_reference(f1, f2, {rname: conseqs[rname]}, unmapped1, unmapped2,
                                             split_counts, nthreads)
            unmapped_count += extra
            new_counts.update(split_counts)
            for line in lines:
                if not line.startswith('@'):
                    writer.writerow(dict(zip(FIELDNAMES, line.strip('\n').split('\t'))))
            os.remove(f1)
            os.remove(f2)
    remap_conseq_csv.write('region,sequence\n')
    for name in new_counts:
        remap_conseq_csv.write('%s,%s\n' % (name, conseqs.get(name) or seeds[name]))
    for name in sorted(new_counts):
        counts_writer.writerow(dict(type='remap-final %s' % name, count=new_counts[name]))
    counts_writer.writerow(dict(type='unmapped', count=unmapped_count))
