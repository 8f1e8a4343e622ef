"""
Run the reference's own bin/micall with the MI355X drop-ins in place of its
imports, on one GPU or as one sharded job under torchrun:

    python -m micall_amd.run_micall /path/to/MiCall-Lite/bin/micall R1.fastq.gz R2.fastq.gz ...
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m micall_amd.run_micall /path/to/MiCall-Lite/bin/micall R1.fastq.gz R2.fastq.gz -i ...

bin/micall imports (bin/micall:10-17)

    micall.core.parse_interop   read_errors, write_phix_csv
    micall.core.filter_quality  report_bad_cycles
    micall.core.censor_fastq    censor
    micall.core.prelim_map      prelim_map
    micall.core.remap           remap
    micall.core.sam2aln         sam2aln
    micall.core.aln2counts      aln2counts
    micall.utils.externals      Bowtie2

Each of these names is bound here to the drop-in module of this package
before the script runs (sys.modules), so the script's text is not changed.
Bowtie2 reports the mapper the drop-ins use instead of looking for a bowtie2
executable (bin/micall:200-207 only prints its path and version).

Under torchrun every rank runs the script: the drop-ins agree through
torch.distributed (micall_amd.session: the process group comes up over
MICALL_DIST_BACKEND, default nccl = RCCL, one GPU per LOCAL_RANK).  censor,
prelim_map and remap split their work by rank; the InterOp reports, sam2aln
and aln2counts run on rank 0 while the others wait.  bin/micall removes
prelim.csv and remap.csv after a sample unless --keep (:190-192); every rank
would remove the same two files, so on ranks other than 0 os.remove of a
file that is already gone is not an error.
"""
import os
import runpy
import sys
import types

from . import (aln2counts, censor_fastq, filter_quality, parse_interop, prelim_map, remap,
               sam2aln, session)
from .prelim_map import BOWTIE_VERSION


class Bowtie2:
    """bin/micall's `Bowtie2(execname=...)` check (externals.py:161-166):
    path and version of the mapper in use."""

    def __init__(self, execname='bowtie2', logger=None):
        self.path = 'libmicall_hip.so (MI355X mapper, in place of {})'.format(execname)
        self.version = BOWTIE_VERSION


def install():
    """Bind micall.core.* / micall.utils.externals to the drop-ins."""
    def package(name):
        mod = sys.modules.get(name)
        if mod is None:
            mod = types.ModuleType(name)
            mod.__path__ = []
            sys.modules[name] = mod
        return mod

    package('micall')
    core = package('micall.core')
    utils = package('micall.utils')
    for name, mod in (('parse_interop', parse_interop), ('filter_quality', filter_quality),
                      ('censor_fastq', censor_fastq), ('prelim_map', prelim_map),
                      ('remap', remap), ('sam2aln', sam2aln), ('aln2counts', aln2counts)):
        sys.modules['micall.core.' + name] = mod
        setattr(core, name, mod)
    externals = types.ModuleType('micall.utils.externals')
    externals.Bowtie2 = Bowtie2
    sys.modules['micall.utils.externals'] = externals
    utils.externals = externals


def _tolerant_remove():
    real = os.remove

    def remove(path, *a, **kw):
        try:
            real(path, *a, **kw)
        except FileNotFoundError:
            if session.is_writer():
                raise
    os.remove = remove


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    script, args = argv[0], argv[1:]
    install()
    if int(os.environ.get('WORLD_SIZE', '1')) > 1:
        session.shard()          # the process group, before the script's first call
        _tolerant_remove()
    sys.argv = [script] + args
    try:
        runpy.run_path(script, run_name='__main__')
    finally:
        sh = session.shard()
        if sh is not None:
            sh.barrier()
            sh.dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
