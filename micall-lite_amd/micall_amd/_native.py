"""
ctypes binding of libmicall_hip.so (include/micall_hip.h).

This is the only way the host package reaches the GPU path.  There is no CPU
fallback: if the library is missing, or no gfx950 device is visible,
constructing a Context raises NativeUnavailable.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('MICALL_HIP_LIB', os.path.join(HERE, 'libmicall_hip.so'))

E2E, LOCAL = 0, 1
MAXOPS = 128
INT32_MIN = -2 ** 31
OP_CHARS = 'MIDxS'
PILEUP_SLACK = 2048


class NativeUnavailable(RuntimeError):
    pass


class NativeError(RuntimeError):
    pass


class Params(ctypes.Structure):
    _fields_ = [('mode', ctypes.c_int), ('rdg_open', ctypes.c_int), ('rdg_ext', ctypes.c_int),
                ('rfg_open', ctypes.c_int), ('rfg_ext', ctypes.c_int), ('maxins', ctypes.c_int)]


ALN_FIELDS = ('ref', 'pos', 'rev', 'score', 'secbest', 'flag', 'mapq', 'rnext', 'pnext', 'tlen',
              'sam_ref', 'sam_pos', 'xm', 'xo', 'xg', 'nm', 'ys', 'yt', 'yf', 'n_cigar')


class Aln(ctypes.Structure):
    _fields_ = [(name, ctypes.c_int32) for name in ALN_FIELDS] + [('cigar', ctypes.c_uint32 * MAXOPS)]


ALN_DTYPE = np.dtype([(name, np.int32) for name in ALN_FIELDS] + [('cigar', np.uint32, MAXOPS)])
assert ALN_DTYPE.itemsize == ctypes.sizeof(Aln)

_lib = None

_P = ctypes.c_void_p
_I64P = ctypes.POINTER(ctypes.c_int64)
_I32P = ctypes.POINTER(ctypes.c_int32)


def _declare(L):
    sig = {
        'mh_version': ([], ctypes.c_int),
        'mh_last_error': ([ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
        'mh_device_count': ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        'mh_ctx_create': ([ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
        'mh_ctx_destroy': ([_P], ctypes.c_int),
        'mh_ctx_sync': ([_P], ctypes.c_int),
        'mh_ctx_stream': ([_P, ctypes.POINTER(_P)], ctypes.c_int),
        'mh_index_build': ([_P, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int], ctypes.c_int),
        'mh_reads_load': ([_P, ctypes.c_int64, ctypes.c_int, _P, _P, _P, _P], ctypes.c_int),
        'mh_reads_load_fastq': ([_P, ctypes.c_char_p, ctypes.c_char_p, _I64P], ctypes.c_int),
        'mh_reads_load_fastq_part': ([_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                      ctypes.c_int, _I64P, _I64P], ctypes.c_int),
        'mh_reads_count': ([_P, _I64P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        'mh_reads_set_names': ([_P, ctypes.c_int64, ctypes.POINTER(ctypes.c_char_p)], ctypes.c_int),
        'mh_map': ([_P, ctypes.POINTER(Params)], ctypes.c_int),
        'mh_probe_extend': ([_P, ctypes.POINTER(Params), ctypes.c_int, _P, _P], ctypes.c_int),
        'mh_conseqs_build': ([ctypes.c_int, _P, _P, _P, _P, ctypes.c_int32, _P, _P, _P, ctypes.c_int64,
                              _P, _P, _P, _P, _P, ctypes.c_char_p, _P, ctypes.c_int64, _P, _P],
                             ctypes.c_int),
        'mh_top_tokens': ([ctypes.c_int32, ctypes.c_int32, _P, _P, _P, ctypes.c_char_p, ctypes.c_int32, _P,
                           _P], ctypes.c_int),
        'mh_alns_fetch': ([_P, ctypes.c_int64, ctypes.c_int64, _P], ctypes.c_int),
        'mh_map_counts': ([_P, _P, _P, _P, _P, _P, _I64P, _I64P, _I64P], ctypes.c_int),
        'mh_map_stats': ([_P, _P], ctypes.c_int),
        'mh_recs_fetch_fields': ([_P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _P],
                                 ctypes.c_int),
        'mh_recs_fetch': ([_P, ctypes.c_int64, ctypes.c_int64, _P], ctypes.c_int),
        'mh_test_set_capacities': ([_P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int64], ctypes.c_int),
        'mh_retry_counts': ([_P, _P], ctypes.c_int),
        'mh_test_set_gotoh_wait': ([_P, ctypes.c_int64], ctypes.c_int),
        'mh_format_rows': ([_P, ctypes.c_int, _P, ctypes.c_int64, ctypes.c_int64,
                            ctypes.POINTER(ctypes.c_char_p), _P, ctypes.c_size_t,
                            ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        'mh_write_rows': ([_P, ctypes.c_int, _P, ctypes.c_int64, ctypes.c_int64,
                           ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int64, _I64P],
                          ctypes.c_int),
        'mh_write_rows_crc': ([_P, ctypes.c_int, _P, ctypes.c_int64, ctypes.c_int64,
                               ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int64, _I64P,
                               ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
        'mh_file_checksum': ([ctypes.c_int, _I64P, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
        'mh_rows_load': ([_P, ctypes.c_int64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                          ctypes.c_int64, _P], ctypes.c_int),
        'mh_rows_load_csv': ([_P, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int,
                              ctypes.POINTER(ctypes.c_char_p), _I64P, _I64P, _I32P], ctypes.c_int),
        'mh_rows_info': ([_P, _P, _P, ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
        'mh_reads_fastq_lines': ([_P, _I64P], ctypes.c_int),
        'mh_pileup': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P], ctypes.c_int),
        'mh_pileup_only': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, ctypes.c_int, _P], ctypes.c_int),
        'mh_pileup_dims': ([_P, ctypes.POINTER(ctypes.c_int), _I32P, _I64P, _I64P], ctypes.c_int),
        'mh_pileup_fetch': ([_P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
        'mh_pileup_fetch_ref': ([_P, ctypes.c_int, _P, _P, _P], ctypes.c_int),
        'mh_pileup_fetch_refs': ([_P, ctypes.c_int, _P, _P, _P, _P], ctypes.c_int),
        'mh_pileup_events': ([_P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
        'mh_pileup_exchange_bytes': ([_P, ctypes.c_int, _I64P, _I64P, _I64P], ctypes.c_int),
        'mh_pileup_export': ([_P, ctypes.c_int, _P, ctypes.c_int64, _P, _P, _P], ctypes.c_int),
        'mh_pileup_import': ([_P, ctypes.c_int, _P, _P, _P, _P], ctypes.c_int),
        'mh_gotoh_align': ([_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                            ctypes.c_int, ctypes.c_char_p, _P, ctypes.c_char_p, ctypes.c_char_p,
                            ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        'mh_levenshtein': ([ctypes.c_char_p, ctypes.c_char_p], ctypes.c_int),
        'mh_gotoh_align_batch': ([_P, ctypes.c_int, _P, _P, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_char_p, _P, _P, _P, _P, _P, _P],
                                 ctypes.c_int),
        'mh_gotoh_distance_batch': ([_P, ctypes.c_int, _P, _P, _P, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_char_p, _P, _P, _P, _P], ctypes.c_int),
        'mh_levenshtein_batch': ([ctypes.c_int, _P, _P, _P], ctypes.c_int),
        'mh_pileup_event_bytes': ([_P, _P, _P], ctypes.c_int),
        'mh_pileup_events_export': ([_P, _P, _P], ctypes.c_int),
        'mh_pileup_events_import': ([_P, ctypes.c_int, _P, _P, _P, ctypes.c_int64, _P,
                                     ctypes.c_int64], ctypes.c_int),
        'mh_sam2aln_csv': ([_P, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                            _I64P], ctypes.c_int),
        'mh_sam2aln_output': ([_P, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                               ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        'mh_sam2aln_file': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_double, _I64P], ctypes.c_int),
        'mh_sam2aln_write': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_int64, _I64P], ctypes.c_int),
        'mh_sam2aln_stats': ([_P, _P], ctypes.c_int),
        'mh_a2c_part_open': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                              _I64P], ctypes.c_int),
        'mh_a2c_part_groups': ([_P, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                ctypes.POINTER(ctypes.c_size_t), _I64P, _P, _I64P], ctypes.c_int),
        'mh_a2c_part_count': ([_P, ctypes.c_int, ctypes.c_int64, ctypes.c_char_p, _I64P, _P, _I64P, _I64P],
                              ctypes.c_int),
        'mh_a2c_part_counters': ([_P, ctypes.c_int, ctypes.c_int, _P, _P], ctypes.c_int),
        'mh_a2c_insert_export': ([_P, ctypes.c_int, _P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)],
                                 ctypes.c_int),
        'mh_a2c_insert_merge': ([_P, ctypes.c_int, _P, ctypes.c_int64, _I64P], ctypes.c_int),
        'mh_sam2aln_part': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                             _I64P], ctypes.c_int),
        'mh_sam2aln_part_units': ([_P, _P, _P], ctypes.c_int),
        'mh_sam2aln_part_names': ([_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                   _I64P], ctypes.c_int),
        'mh_sam2aln_part_set_names': ([_P, _P, ctypes.c_int], ctypes.c_int),
        'mh_sam2aln_records': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I64P, ctypes.POINTER(_P)],
                               ctypes.c_int),
        'mh_sam2aln_records_merge': ([_P, ctypes.c_int, _P, ctypes.c_int64], ctypes.c_int),
        'mh_sam2aln_splitters': ([_P, _P, ctypes.c_int64, ctypes.c_int], ctypes.c_int),
        'mh_sam2aln_range_counts': ([_P, ctypes.c_int, _I64P], ctypes.c_int),
        'mh_sam2aln_range_text': ([_P, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), _I64P, _I64P,
                                   ctypes.POINTER(_P)], ctypes.c_int),
        'mh_sam2aln_part_text': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I64P, ctypes.POINTER(_P)],
                                 ctypes.c_int),
        'mh_sam2aln_timing': ([_P, _P], ctypes.c_int),
        'mh_censor_fastq': ([_P, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                             ctypes.POINTER(ctypes.c_char_p), _P, ctypes.c_int, _I64P, _I64P],
                            ctypes.c_int),
        'mh_censor_staged': ([_P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), _P, ctypes.c_int,
                              _I64P, _I64P, _I64P], ctypes.c_int),
        'mh_censor_staged_write': ([_P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), _P, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int64, _I64P, _I64P, _I64P], ctypes.c_int),
        'mh_censor_output': ([_P, ctypes.c_char_p, ctypes.c_size_t,
                              ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        'mh_censor_write': ([_P, ctypes.c_int, ctypes.c_int64, _I64P], ctypes.c_int),
        'mh_censor_timing': ([_P, _P], ctypes.c_int),
        'mh_a2c_load_file': ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, _I64P], ctypes.c_int),
        'mh_a2c_insert_rows': ([_P, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, _P, _P, ctypes.c_char_p,
                                ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)],
                               ctypes.c_int),
        'mh_a2c_load_csv': ([_P, ctypes.c_int, ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p,
                             _I64P], ctypes.c_int),
        'mh_a2c_load_rows': ([_P, ctypes.c_int, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64,
                              _P, _P, _P, _P, ctypes.c_int64, _P, ctypes.c_char_p], ctypes.c_int),
        'mh_a2c_group': ([_P, ctypes.c_int, ctypes.c_int64, _P, ctypes.c_char_p, ctypes.c_size_t,
                          ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        'mh_a2c_counts': ([_P, ctypes.c_int, ctypes.c_int64, ctypes.c_int, _P, _P, _P, _P],
                          ctypes.c_int),
        'mh_a2c_inserts': ([_P, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _P, _P,
                            _I64P], ctypes.c_int),
        'mh_a2c_insert_entries': ([_P, ctypes.c_int, _P, _P, _P, ctypes.c_char_p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        'mh_a2c_timing': ([_P, ctypes.c_int, _P], ctypes.c_int),
        'mh_fastq_open_part': ([ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(_P), _I64P], ctypes.c_int),
        'mh_fastq_scan_part': ([ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I64P],
                               ctypes.c_int),
        'mh_fastq_member_open': ([ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(_P), _I64P], ctypes.c_int),
        'mh_fastq_member_decode': ([_P, ctypes.c_int64, _I64P], ctypes.c_int),
        'mh_fastq_member_tail': ([_P, _P, _P], ctypes.c_int),
        'mh_fastq_member_finish': ([_P, _P, ctypes.c_int64, ctypes.c_int64, _I64P], ctypes.c_int),
        'mh_fastq_frame': ([_P, ctypes.c_int64, ctypes.c_int, _I64P], ctypes.c_int),
        'mh_fastq_record_offset': ([_P, ctypes.c_int64, _I64P], ctypes.c_int),
        'mh_fastq_splice': ([_P, ctypes.c_int64, ctypes.c_int64, _P, ctypes.c_int64, _P,
                             ctypes.c_int64], ctypes.c_int),
        'mh_fastq_view': ([_P, ctypes.POINTER(_P), _I64P], ctypes.c_int),
        'mh_fastq_close': ([_P], ctypes.c_int),
        'mh_fastq_parse': ([_P, _P, ctypes.c_char_p, ctypes.c_size_t, _P, _P, ctypes.c_size_t, _P,
                            ctypes.c_int64, _I64P, _I64P, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        'mh_reads_load_staged': ([_P, _P, _P, _I64P, ctypes.c_int64, _I64P], ctypes.c_int),
        'mh_format_segments': ([_P, ctypes.c_int, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_char_p),
                                ctypes.c_int, _P, _P], ctypes.c_int),
        'mh_write_segments': ([_P, ctypes.c_int, _P, _P], ctypes.c_int),
        'mh_crc32_combine': ([ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64], ctypes.c_uint32),
        'mh_file_crc32': ([ctypes.c_int, _I64P, ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
        'mh_phase_times': ([_P, _P, ctypes.c_int], ctypes.c_int),
        'mh_profile': ([_P, ctypes.c_int], ctypes.c_int),
        'mh_profile_get': ([_P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), _I64P],
                           ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    return sig


EXPORTED = None


def lib():
    """The loaded library (raises NativeUnavailable if it was not built)."""
    global _lib, EXPORTED
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable('libmicall_hip.so not built at {} (run __graft_entry__.build() '
                                    'or make -C micall-lite_amd/csrc)'.format(LIB_PATH))
        _lib = ctypes.CDLL(LIB_PATH)
        EXPORTED = sorted(_declare(_lib))
    return _lib


def last_error():
    buf = ctypes.create_string_buffer(1024)
    lib().mh_last_error(buf, len(buf))
    return buf.value.decode(errors='replace')


def check(status, what):
    if status == 0:
        return
    msg = last_error()
    if status == -5:
        raise NativeUnavailable('{}: {}'.format(what, msg))
    if status == -1:
        raise RuntimeError(msg or 'Traceback failed, try local alignment')
    raise NativeError('{} failed ({}): {}'.format(what, status, msg))


def top_tokens(length, rows, dense, nflag, dflag, seed, tok):
    """mh_top_tokens: tok[:length] = the top base-like token of each
    position (host code of the library; dense (>= rows, 4) int32, flags
    uint8, seed bytes); returns whether any row holds a positive count."""
    pos = ctypes.c_int32()
    check(lib().mh_top_tokens(length, rows, _ptr(dense), _ptr(nflag), _ptr(dflag), seed, len(seed),
                              _ptr(tok), ctypes.byref(pos)), 'mh_top_tokens')
    return bool(pos.value)


def conseqs_build(rows_of, lengths, seeds, dense, nflag, dflag, ev_row, ev_pos, ev_off, ev_len, ev_cnt,
                  pool):
    """mh_conseqs_build: [(consensus bytes, present)] per selected row.
    dense (n, cap, 4) int32, flags (n, cap) uint8, all C-contiguous; seeds
    bytes per selected row; events as arrays (row, pos, token offset and
    length in `pool`, merged pairs)."""
    n = len(rows_of)
    cap = dense.shape[1] if dense.ndim == 3 else 0
    rows_of = np.ascontiguousarray(rows_of, dtype=np.int32)
    lengths = np.ascontiguousarray(lengths, dtype=np.int32)
    seed_bufs = [ctypes.create_string_buffer(sd, len(sd) + 1) for sd in seeds]
    seed_ptrs = (ctypes.c_char_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_char_p) for b in seed_bufs])
    seed_lens = np.ascontiguousarray([len(sd) for sd in seeds], dtype=np.int32)
    n_ev = len(ev_row)
    ev_row = np.ascontiguousarray(ev_row, dtype=np.int32)
    ev_pos = np.ascontiguousarray(ev_pos, dtype=np.int32)
    ev_off = np.ascontiguousarray(ev_off, dtype=np.int64)
    ev_len = np.ascontiguousarray(ev_len, dtype=np.int32)
    ev_cnt = np.ascontiguousarray(ev_cnt, dtype=np.int64)
    out_cap = int(lengths.sum()) + int(ev_len.sum()) + 1
    out = np.zeros(out_cap, dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.int64)
    present = np.zeros(max(n, 1), dtype=np.int32)
    check(lib().mh_conseqs_build(n, _ptr(rows_of), _ptr(lengths), seed_ptrs, _ptr(seed_lens), cap,
                                 _ptr(dense), _ptr(nflag), _ptr(dflag), n_ev, _ptr(ev_row),
                                 _ptr(ev_pos), _ptr(ev_off), _ptr(ev_len), _ptr(ev_cnt), bytes(pool) or b'\0',
                                 _ptr(out), out_cap, _ptr(off), _ptr(present)), 'mh_conseqs_build')
    raw = out.tobytes()
    return [(raw[off[k]:off[k + 1]], bool(present[k])) for k in range(n)]


def device_count():
    n = ctypes.c_int()
    if lib().mh_device_count(ctypes.byref(n)) != 0:
        return 0
    return n.value


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def params(mode, rdg=(10, 3), rfg=(10, 3), maxins=1200):
    return Params(mode, rdg[0], rdg[1], rfg[0], rfg[1], maxins)


class Context:
    """One device context (HIP stream, resident reads, index, results)."""

    def __init__(self, device=0):
        L = lib()
        h = ctypes.c_void_p()
        check(L.mh_ctx_create(device, ctypes.byref(h)), 'mh_ctx_create')
        self.h = h
        self.device = device
        # bumped whenever the resident reads or the mapping records change
        # (session.prelim_resident compares it)
        self.map_serial = 0
        self.n_refs = 0
        self.refnames = []
        self.reflens = []

    def close(self):
        if getattr(self, 'h', None):
            lib().mh_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(lib().mh_ctx_sync(self.h), 'mh_ctx_sync')

    # ---- sam2aln --------------------------------------------------------
    def sam2aln_csv(self, text, q_cutoff=15, max_prop_n=0.5):
        """mh_sam2aln_csv on remap.csv text (str or bytes); returns the
        number of matchmaker pairs."""
        data = text.encode() if isinstance(text, str) else bytes(text)
        n = ctypes.c_int64()
        check(lib().mh_sam2aln_csv(self.h, data, len(data), int(q_cutoff), float(max_prop_n),
                                   ctypes.byref(n)), 'mh_sam2aln_csv')
        return n.value

    def sam2aln_file(self, fd, q_cutoff=15, max_prop_n=0.5):
        """mh_sam2aln_file on the whole regular file fd (mmap'd): the number of
        matchmaker pairs, or None when the file holds '\r' (read it in text
        mode and use sam2aln_csv)."""
        n = ctypes.c_int64()
        st = lib().mh_sam2aln_file(self.h, int(fd), int(q_cutoff), float(max_prop_n), ctypes.byref(n))
        if st == 1:
            return None
        check(st, 'mh_sam2aln_file')
        return n.value

    # ---- sam2aln split over the ranks of a job (mh_s2a_shard.cpp) ----
    def sam2aln_part(self, fd, part, parts, q_cutoff=15, max_prop_n=0.5):
        """This rank's records of remap.csv (file fd) parsed and merged:
        dict(units, pair_units, names, distinct, bytes, file_bytes), or None
        when the file cannot be split by lines ('\r' or a quoted field)."""
        info = np.zeros(6, dtype=np.int64)
        st = lib().mh_sam2aln_part(self.h, int(fd), int(part), int(parts), int(q_cutoff),
                                   float(max_prop_n), info.ctypes.data_as(_I64P))
        if st == 1:
            return None
        check(st, 'mh_sam2aln_part')
        return dict(zip(('units', 'pair_units', 'names', 'distinct', 'bytes', 'file_bytes'),
                        (int(x) for x in info)))

    def sam2aln_part_units(self, n_units):
        """(qname hash, leftover?) of every unit of this rank's part."""
        h = np.zeros(max(n_units, 1), dtype=np.uint64)
        left = np.zeros(max(n_units, 1), dtype=np.uint8)
        check(lib().mh_sam2aln_part_units(self.h, _ptr(h), _ptr(left)), 'mh_sam2aln_part_units')
        return h[:n_units], left[:n_units].astype(bool)

    def sam2aln_part_names(self, n_names):
        """(reference names of this part in first-seen order, first unit of each)."""
        used = ctypes.c_size_t()
        check(lib().mh_sam2aln_part_names(self.h, None, 0, ctypes.byref(used), None),
              'mh_sam2aln_part_names')
        buf = ctypes.create_string_buffer(max(used.value, 1))
        first = np.zeros(max(n_names, 1), dtype=np.int64)
        check(lib().mh_sam2aln_part_names(self.h, buf, len(buf), ctypes.byref(used),
                                          first.ctypes.data_as(_I64P)), 'mh_sam2aln_part_names')
        names = buf.raw[:used.value].decode().split('\n')[:n_names]
        return names, first[:n_names]

    def sam2aln_part_set_names(self, gids):
        g = np.ascontiguousarray(gids, dtype=np.int32)
        check(lib().mh_sam2aln_part_set_names(self.h, _ptr(g), len(g)), 'mh_sam2aln_part_set_names')

    def _held_view(self, ptr, n):
        if n <= 0 or not ptr:
            return np.zeros(0, dtype=np.uint8)
        return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ptr))

    def sam2aln_records(self, step, parts, per_name=0):
        """step 0: this part's distinct sequences bucketed by owner rank;
        1: samples of the owner's sorted records; 2: the owner's records
        bucketed by range rank.  Returns (uint8 view of the library's buffer,
        valid until the next call, per-destination sizes)."""
        sizes = np.zeros(max(parts, 1), dtype=np.int64)
        ptr = ctypes.c_void_p()
        check(lib().mh_sam2aln_records(self.h, int(step), int(parts), int(per_name),
                                       sizes.ctypes.data_as(_I64P), ctypes.byref(ptr)), 'mh_sam2aln_records')
        n = int(sizes[0]) if step == 1 else int(sizes.sum())
        return self._held_view(ptr.value, n), (sizes[:1] if step == 1 else sizes)

    def sam2aln_records_merge(self, stage, data):
        d = np.ascontiguousarray(data, dtype=np.uint8)
        check(lib().mh_sam2aln_records_merge(self.h, int(stage), _ptr(d), len(d)), 'mh_sam2aln_records_merge')

    def sam2aln_splitters(self, data, parts):
        d = np.ascontiguousarray(data, dtype=np.uint8)
        check(lib().mh_sam2aln_splitters(self.h, _ptr(d), len(d), int(parts)), 'mh_sam2aln_splitters')

    def sam2aln_range_counts(self, n_names):
        out = np.zeros(max(n_names, 1), dtype=np.int64)
        check(lib().mh_sam2aln_range_counts(self.h, int(n_names), out.ctypes.data_as(_I64P)),
              'mh_sam2aln_range_counts')
        return out[:n_names]

    def sam2aln_range_text(self, names, base):
        """aligned.csv rows of this rank's ranges: (uint8 view, bytes per name)."""
        arr = (ctypes.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
        b = np.ascontiguousarray(base, dtype=np.int64)
        seg = np.zeros(max(len(names), 1), dtype=np.int64)
        ptr = ctypes.c_void_p()
        check(lib().mh_sam2aln_range_text(self.h, len(names), arr, b.ctypes.data_as(_I64P),
                                          seg.ctypes.data_as(_I64P), ctypes.byref(ptr)),
              'mh_sam2aln_range_text')
        seg = seg[:len(names)]
        return self._held_view(ptr.value, int(seg.sum())), seg

    def sam2aln_part_text(self, which, seg, head=False):
        """insert.csv ('insert') or failed.csv ('failed') rows of this part's
        pair units (seg 0) or leftover units (seg 1), as bytes."""
        w = {'insert': 1, 'failed': 2}[which]
        n = ctypes.c_int64()
        ptr = ctypes.c_void_p()
        check(lib().mh_sam2aln_part_text(self.h, w, int(seg), int(bool(head)), ctypes.byref(n),
                                         ctypes.byref(ptr)), 'mh_sam2aln_part_text')
        return self._held_view(ptr.value, n.value).tobytes()

    def sam2aln_size(self, which):
        """Bytes of output 'aligned' | 'insert' | 'failed' (formats it)."""
        w = {'aligned': 0, 'insert': 1, 'failed': 2}[which]
        used = ctypes.c_size_t()
        check(lib().mh_sam2aln_output(self.h, w, None, 0, ctypes.byref(used)), 'mh_sam2aln_output')
        return used.value

    def sam2aln_write(self, which, fd, offset):
        """Output `which` written to fd at offset (pwrite); bytes written."""
        w = {'aligned': 0, 'insert': 1, 'failed': 2}[which]
        n = ctypes.c_int64()
        check(lib().mh_sam2aln_write(self.h, w, int(fd), int(offset), ctypes.byref(n)), 'mh_sam2aln_write')
        return n.value

    def sam2aln_output(self, which):
        """'aligned' | 'insert' | 'failed' CSV text of the last sam2aln."""
        w = {'aligned': 0, 'insert': 1, 'failed': 2}[which]
        used = ctypes.c_size_t()
        check(lib().mh_sam2aln_output(self.h, w, None, 0, ctypes.byref(used)), 'mh_sam2aln_output')
        buf = bytearray(used.value)
        cbuf = (ctypes.c_char * max(len(buf), 1)).from_buffer(buf) if buf else None
        check(lib().mh_sam2aln_output(self.h, w, cbuf, len(buf), ctypes.byref(used)),
              'mh_sam2aln_output')
        del cbuf
        return buf.decode()

    @staticmethod
    def _bad_cycle_args(bad_cycles):
        tiles = (ctypes.c_char_p * max(len(bad_cycles), 1))(*[t.encode() for t, _ in bad_cycles])
        cycles = np.array([c for _, c in bad_cycles] or [0], dtype=np.int32)
        return tiles, cycles

    def censor_fastq(self, data, bad_cycles, src_gzip, dst_gzip):
        """mh_censor_fastq: (censored bytes, base_count, score_sum) for FASTQ
        bytes and [(tile, cycle)] bad cycles."""
        tiles, cycles = self._bad_cycle_args(bad_cycles)
        bc, ss = ctypes.c_int64(), ctypes.c_int64()
        src = data if isinstance(data, bytes) else bytes(data)
        check(lib().mh_censor_fastq(self.h, src, len(src), int(src_gzip), len(bad_cycles),
                                    tiles, _ptr(cycles), int(dst_gzip), ctypes.byref(bc),
                                    ctypes.byref(ss)), 'mh_censor_fastq')
        return self.censor_output(), bc.value, ss.value

    def censor_staged(self, fq, bad_cycles, dst_gzip):
        """mh_censor_staged on a staged FASTQ's text (taken from the handle):
        (output bytes held, base_count, score_sum)."""
        tiles, cycles = self._bad_cycle_args(bad_cycles)
        nb, bc, ss = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().mh_censor_staged(self.h, fq.h, len(bad_cycles), tiles, _ptr(cycles), int(dst_gzip),
                                     ctypes.byref(nb), ctypes.byref(bc), ctypes.byref(ss)),
              'mh_censor_staged')
        return nb.value, bc.value, ss.value

    def censor_staged_write(self, fq, bad_cycles, dst_gzip, fd, offset):
        """mh_censor_staged_write: the censored output written to fd from
        offset while it is made: (bytes written, base_count, score_sum)."""
        tiles, cycles = self._bad_cycle_args(bad_cycles)
        nw, bc, ss = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().mh_censor_staged_write(self.h, fq.h, len(bad_cycles), tiles, _ptr(cycles), int(dst_gzip),
                                           int(fd), int(offset), ctypes.byref(nw), ctypes.byref(bc),
                                           ctypes.byref(ss)),
              'mh_censor_staged_write')
        return nw.value, bc.value, ss.value

    def censor_output(self):
        """The held censored output as a bytearray (then released)."""
        used = ctypes.c_size_t()
        check(lib().mh_censor_output(self.h, None, 0, ctypes.byref(used)), 'mh_censor_output')
        buf = bytearray(used.value)
        cbuf = (ctypes.c_char * max(len(buf), 1)).from_buffer(buf) if buf else None
        check(lib().mh_censor_output(self.h, cbuf, len(buf), ctypes.byref(used)), 'mh_censor_output')
        del cbuf
        return buf

    def censor_write(self, fd, offset):
        """The held censored output written to fd at offset (then released)."""
        n = ctypes.c_int64()
        check(lib().mh_censor_write(self.h, int(fd), int(offset), ctypes.byref(n)), 'mh_censor_write')
        return n.value

    def censor_timing(self):
        out = np.zeros(3, dtype=np.float64)
        check(lib().mh_censor_timing(self.h, _ptr(out)), 'mh_censor_timing')
        return [float(x) for x in out]

    # ---- aln2counts -----------------------------------------------------
    def a2c_load_csv(self, slot, text, codon_chars):
        """mh_a2c_load_csv on aligned.csv text (str or bytes): number of
        (refname, qcut) groups."""
        data = text.encode() if isinstance(text, str) else bytes(text)
        n = ctypes.c_int64()
        check(lib().mh_a2c_load_csv(self.h, slot, data, len(data), codon_chars, ctypes.byref(n)),
              'mh_a2c_load_csv')
        return n.value

    def a2c_load_file(self, slot, fd, codon_chars):
        """mh_a2c_load_file on the whole regular file fd (mmap'd): number of
        groups, or None when it holds '\r' (read it in text mode instead)."""
        n = ctypes.c_int64()
        st = lib().mh_a2c_load_file(self.h, slot, int(fd), codon_chars, ctypes.byref(n))
        if st == 1:
            return None
        check(st, 'mh_a2c_load_file')
        return n.value

    def a2c_inserts_text(self, slot, g, frame, lefts, rights, lead, targets, eol):
        """mh_a2c_inserts then mh_a2c_insert_rows: the insertion report rows
        as text ('' when there are none)."""
        lo = np.array(list(lefts) or [0], dtype=np.int32)
        hi = np.array(list(rights) or [0], dtype=np.int32)
        n = ctypes.c_int64()
        check(lib().mh_a2c_inserts(self.h, slot, g, frame, len(lefts), _ptr(lo), _ptr(hi),
                                   ctypes.byref(n)), 'mh_a2c_inserts')
        if n.value == 0:
            return ''
        tg = np.array([INT32_MIN if t is None else t for t in targets] or [0], dtype=np.int32)
        used = ctypes.c_size_t()
        args = (self.h, slot, lead.encode(), len(lefts), _ptr(lo), _ptr(tg), eol.encode())
        check(lib().mh_a2c_insert_rows(*args, None, 0, ctypes.byref(used)), 'mh_a2c_insert_rows')
        buf = ctypes.create_string_buffer(max(used.value, 1))
        check(lib().mh_a2c_insert_rows(*args, buf, len(buf), ctypes.byref(used)), 'mh_a2c_insert_rows')
        return buf.raw[:used.value].decode()

    def _a2c_insert_rows(self, slot, lefts, lead, targets, eol):
        lo = np.array(list(lefts) or [0], dtype=np.int32)
        tg = np.array([INT32_MIN if t is None else t for t in targets] or [0], dtype=np.int32)
        used = ctypes.c_size_t()
        args = (self.h, slot, lead.encode(), len(lefts), _ptr(lo), _ptr(tg), eol.encode())
        check(lib().mh_a2c_insert_rows(*args, None, 0, ctypes.byref(used)), 'mh_a2c_insert_rows')
        buf = ctypes.create_string_buffer(max(used.value, 1))
        check(lib().mh_a2c_insert_rows(*args, buf, len(buf), ctypes.byref(used)), 'mh_a2c_insert_rows')
        return buf.raw[:used.value].decode()

    # ---- aln2counts split over the ranks of a job (mh_a2c_part_*) ----
    def a2c_part_open(self, slot, fd, part, parts, codon_chars):
        """Parse this rank's share of aligned.csv (file fd): dict(rows,
        groups, bytes), or None when the file is not split ('\r' or quotes)."""
        info = np.zeros(3, dtype=np.int64)
        st = lib().mh_a2c_part_open(self.h, slot, int(fd), int(part), int(parts), codon_chars,
                                    info.ctypes.data_as(_I64P))
        if st == 1:
            return None
        check(st, 'mh_a2c_part_open')
        return dict(rows=int(info[0]), groups=int(info[1]), bytes=int(info[2]))

    def a2c_part_groups(self, slot, n):
        """This part's runs of (refname, qcut): (key bytes 'ref\x1fqcut\n'
        joined, rows, codon extents [n, 3], count totals)."""
        used = ctypes.c_size_t()
        check(lib().mh_a2c_part_groups(self.h, slot, None, 0, ctypes.byref(used), None, None, None),
              'mh_a2c_part_groups')
        buf = ctypes.create_string_buffer(max(used.value, 1))
        rows = np.zeros(max(n, 1), dtype=np.int64)
        ncod = np.zeros((max(n, 1), 3), dtype=np.int32)
        total = np.zeros(max(n, 1), dtype=np.int64)
        check(lib().mh_a2c_part_groups(self.h, slot, buf, len(buf), ctypes.byref(used),
                                       rows.ctypes.data_as(_I64P), _ptr(ncod), total.ctypes.data_as(_I64P)),
              'mh_a2c_part_groups')
        return buf.raw[:used.value], rows[:n], ncod[:n], total[:n]

    def a2c_part_count(self, slot, keys, gid, ncod, row_base):
        """Count this part's rows into the job's groups (keys joined as
        a2c_part_groups gives them); returns the counter cells."""
        g = np.ascontiguousarray(gid, dtype=np.int64)
        nc = np.ascontiguousarray(ncod, dtype=np.int32)
        rb = np.ascontiguousarray(row_base, dtype=np.int64)
        cells = ctypes.c_int64()
        n_groups = keys.count(b'\n')
        check(lib().mh_a2c_part_count(self.h, slot, n_groups, keys, g.ctypes.data_as(_I64P), _ptr(nc),
                                      rb.ctypes.data_as(_I64P), ctypes.byref(cells)), 'mh_a2c_part_count')
        return cells.value

    def a2c_part_counters(self, slot, cells, values=None):
        """The counters (count, first row) of the slot, or set them."""
        if values is not None:
            c = np.ascontiguousarray(values[0], dtype=np.uint32)
            f = np.ascontiguousarray(values[1], dtype=np.uint32)
            check(lib().mh_a2c_part_counters(self.h, slot, 1, _ptr(c), _ptr(f)), 'mh_a2c_part_counters')
            return None
        c = np.zeros(max(cells, 1), dtype=np.uint32)
        f = np.zeros(max(cells, 1), dtype=np.uint32)
        check(lib().mh_a2c_part_counters(self.h, slot, 0, _ptr(c), _ptr(f)), 'mh_a2c_part_counters')
        return c[:cells], f[:cells]

    def a2c_inserts_local(self, slot, g, frame, lefts, rights):
        """mh_a2c_inserts over this rank's rows of group g, then the entries
        as bytes (mh_a2c_insert_export)."""
        lo = np.array(list(lefts) or [0], dtype=np.int32)
        hi = np.array(list(rights) or [0], dtype=np.int32)
        n = ctypes.c_int64()
        check(lib().mh_a2c_inserts(self.h, slot, g, frame, len(lefts), _ptr(lo), _ptr(hi),
                                   ctypes.byref(n)), 'mh_a2c_inserts')
        used = ctypes.c_size_t()
        check(lib().mh_a2c_insert_export(self.h, slot, None, 0, ctypes.byref(used)), 'mh_a2c_insert_export')
        buf = np.zeros(max(used.value, 1), dtype=np.uint8)
        check(lib().mh_a2c_insert_export(self.h, slot, _ptr(buf), len(buf), ctypes.byref(used)),
              'mh_a2c_insert_export')
        return buf[:used.value].tobytes()

    def a2c_inserts_merged_text(self, slot, entries, lefts, lead, targets, eol):
        """Every rank's entries merged (mh_a2c_insert_merge), then the rows
        as text ('' when there are none)."""
        d = np.frombuffer(entries, dtype=np.uint8) if entries else np.zeros(1, dtype=np.uint8)
        n = ctypes.c_int64()
        check(lib().mh_a2c_insert_merge(self.h, slot, _ptr(d), len(entries), ctypes.byref(n)),
              'mh_a2c_insert_merge')
        if n.value == 0:
            return ''
        return self._a2c_insert_rows(slot, lefts, lead, targets, eol)

    def a2c_load_rows(self, slot, seqs, offsets, counts, group_first, codon_chars):
        """mh_a2c_load_rows from lists: seq strings, offsets, counts and the
        first row of every group (plus the row count at the end)."""
        enc = [s.encode() for s in seqs]
        lens = np.array([len(s) for s in enc] or [0], dtype=np.int32)
        soff = np.zeros(max(len(enc), 1), dtype=np.int64)
        if len(enc) > 1:
            np.cumsum(lens[:-1], out=soff[1:])
        pool = b''.join(enc)
        off = np.array(list(offsets) or [0], dtype=np.int64)
        cnt = np.array(list(counts) or [0], dtype=np.int64)
        gf = np.array(group_first, dtype=np.int64)
        check(lib().mh_a2c_load_rows(self.h, slot, len(enc), pool, len(pool), _ptr(soff), _ptr(lens),
                                     _ptr(off), _ptr(cnt), len(gf) - 1, _ptr(gf), codon_chars),
              'mh_a2c_load_rows')

    def a2c_group(self, slot, g):
        info = np.zeros(5, dtype=np.int64)
        used = ctypes.c_size_t()
        check(lib().mh_a2c_group(self.h, slot, g, _ptr(info), None, 0, ctypes.byref(used)),
              'mh_a2c_group')
        buf = ctypes.create_string_buffer(used.value + 1)
        check(lib().mh_a2c_group(self.h, slot, g, _ptr(info), buf, len(buf), ctypes.byref(used)),
              'mh_a2c_group')
        ref, qcut = buf.raw[:used.value].split(b'\0', 1)
        return dict(first=int(info[0]), n_rows=int(info[1]), ncod=[int(x) for x in info[2:5]],
                    refname=ref.decode(), qcut=qcut.decode())

    def a2c_counts(self, slot, g, frame, ncod):
        """(aa_count, aa_first) [ncod, 21] and (nuc_count, nuc_first)
        [ncod, 18] uint32 of one group and frame."""
        n = max(ncod, 1)
        aa_c = np.zeros((n, 21), np.uint32)
        aa_f = np.zeros((n, 21), np.uint32)
        nt_c = np.zeros((n, 18), np.uint32)
        nt_f = np.zeros((n, 18), np.uint32)
        check(lib().mh_a2c_counts(self.h, slot, g, frame, _ptr(aa_c), _ptr(aa_f), _ptr(nt_c),
                                  _ptr(nt_f)), 'mh_a2c_counts')
        return aa_c[:ncod], aa_f[:ncod], nt_c[:ncod], nt_f[:ncod]

    def a2c_inserts(self, slot, g, frame, lefts, rights):
        """[(range index, count, first row, amino-acid string)] in
        (range, first row) order."""
        lo = np.array(list(lefts) or [0], dtype=np.int32)
        hi = np.array(list(rights) or [0], dtype=np.int32)
        n = ctypes.c_int64()
        check(lib().mh_a2c_inserts(self.h, slot, g, frame, len(lefts), _ptr(lo), _ptr(hi),
                                   ctypes.byref(n)), 'mh_a2c_inserts')
        k = n.value
        rng = np.zeros(max(k, 1), np.int32)
        cnt = np.zeros(max(k, 1), np.int64)
        first = np.zeros(max(k, 1), np.uint32)
        used = ctypes.c_size_t()
        check(lib().mh_a2c_insert_entries(self.h, slot, _ptr(rng), _ptr(cnt), _ptr(first), None, 0,
                                          ctypes.byref(used)), 'mh_a2c_insert_entries')
        buf = ctypes.create_string_buffer(max(used.value, 1))
        check(lib().mh_a2c_insert_entries(self.h, slot, None, None, None, buf, len(buf),
                                          ctypes.byref(used)), 'mh_a2c_insert_entries')
        aminos = buf.raw[:used.value].decode().split('\n')[:k]
        return [(int(rng[i]), int(cnt[i]), int(first[i]), aminos[i]) for i in range(k)]

    def a2c_timing(self, slot):
        out = np.zeros(3, dtype=np.float64)
        check(lib().mh_a2c_timing(self.h, slot, _ptr(out)), 'mh_a2c_timing')
        return [float(x) for x in out]

    def sam2aln_timing(self):
        """Host ms of the last sam2aln: parse, device, and formatting of
        aligned / insert / failed."""
        out = np.zeros(5, dtype=np.float64)
        check(lib().mh_sam2aln_timing(self.h, _ptr(out)), 'mh_sam2aln_timing')
        return [float(x) for x in out]

    def sam2aln_stats(self):
        """(pairs, merged on the device, distinct merged sequences, failed)."""
        out = np.zeros(4, dtype=np.int64)
        check(lib().mh_sam2aln_stats(self.h, _ptr(out)), 'mh_sam2aln_stats')
        return tuple(int(x) for x in out)

    # ---- reference set --------------------------------------------------
    def index_build(self, names, seqs, seedlen):
        seqs = list(seqs)
        # the same str objects again (the seed set of every prelim pass): reuse
        # their encoded buffers; the cache holds the objects, so ids stay theirs
        cached = getattr(self, '_index_enc', None)
        if cached is not None and len(cached[0]) == len(seqs) and all(
                a is b for a, b in zip(cached[0], seqs)):
            arr = cached[1]
        else:
            arr = (ctypes.c_char_p * max(len(seqs), 1))(*[s.encode() for s in seqs])
            self._index_enc = (seqs, arr)
        check(lib().mh_index_build(self.h, len(seqs), arr, seedlen), 'mh_index_build')
        self.refnames = list(names)
        self.reflens = [len(s) for s in seqs]
        self.n_refs = len(seqs)

    # ---- reads ----------------------------------------------------------
    def reads_load_arrays(self, seq, qual, offsets, lens, paired):
        """seq/qual: uint8 buffers; offsets int64, lens int32 per read."""
        seq = np.ascontiguousarray(seq, dtype=np.uint8)
        qual = np.ascontiguousarray(qual, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        check(lib().mh_reads_load(self.h, len(lens), int(paired), _ptr(seq), _ptr(qual),
                                  _ptr(offsets), _ptr(lens)), 'mh_reads_load')
        self.map_serial += 1

    def reads_load(self, seqs, quals, paired, names=None):
        lens = np.array([len(s) for s in seqs], dtype=np.int32)
        offsets = np.zeros(len(seqs), dtype=np.int64)
        if len(seqs):
            offsets[1:] = np.cumsum(lens[:-1])
        seq = np.frombuffer(''.join(seqs).encode(), dtype=np.uint8)
        qual = np.frombuffer(''.join(quals).encode(), dtype=np.uint8)
        self.reads_load_arrays(seq, qual, offsets, lens, paired)
        if names is not None:
            self.set_names(names)

    def reads_load_fixed(self, reads, quals, paired):
        """reads/quals: (n, L) uint8 arrays (mates interleaved when paired)."""
        n, L = reads.shape
        lens = np.full(n, L, dtype=np.int32)
        offsets = np.arange(n, dtype=np.int64) * L
        self.reads_load_arrays(reads.reshape(-1), quals.reshape(-1), offsets, lens, paired)

    def reads_load_fastq(self, path1, path2=None):
        n = ctypes.c_int64()
        check(lib().mh_reads_load_fastq(self.h, path1.encode(), path2.encode() if path2 else None,
                                        ctypes.byref(n)), 'mh_reads_load_fastq')
        self.map_serial += 1
        return n.value

    def reads_load_fastq_part(self, path1, path2, part, parts):
        """One rank's contiguous block of the FASTQ units: (reads loaded,
        first unit of the block)."""
        n = ctypes.c_int64()
        u0 = ctypes.c_int64()
        check(lib().mh_reads_load_fastq_part(self.h, path1.encode(),
                                             path2.encode() if path2 else None, part, parts,
                                             ctypes.byref(n), ctypes.byref(u0)),
              'mh_reads_load_fastq_part')
        self.map_serial += 1
        return n.value, u0.value

    def reads_load_staged(self, fq1, fq2, ranges, fastq_lines1):
        """Reads of staged FASTQ text (Fastq handles; their texts move into
        the context): ranges = (u0, u1, v0, v1) record ranges of fq1 / fq2,
        -1 for all."""
        r = np.ascontiguousarray(ranges, dtype=np.int64)
        n = ctypes.c_int64()
        check(lib().mh_reads_load_staged(self.h, fq1.h, fq2.h if fq2 is not None else None,
                                         r.ctypes.data_as(_I64P), int(fastq_lines1),
                                         ctypes.byref(n)), 'mh_reads_load_staged')
        self.map_serial += 1
        return n.value

    def phase_times(self, reset=False):
        """Host wall ms per phase of the file path (inflate, parse, upload,
        format, write) since the last reset."""
        out = np.zeros(5, dtype=np.float64)
        check(lib().mh_phase_times(self.h, _ptr(out), int(reset)), 'mh_phase_times')
        return dict(zip(('inflate', 'parse', 'upload', 'format', 'write'), (float(x) for x in out)))

    def format_segments(self, style, order, seg_rows):
        """Format rows order[0 ..] (None: every read) in segments
        [seg_rows[s], seg_rows[s + 1]); the text stays in the library for
        write_segments.  Returns the bytes per segment (int64 array)."""
        if order is not None:
            order = np.ascontiguousarray(order, dtype=np.int64)
            n = len(order)
        else:
            n = self.reads_count()[0]
        seg_rows = np.ascontiguousarray(seg_rows, dtype=np.int64)
        k = len(seg_rows) - 1
        out = np.zeros(max(k, 1), dtype=np.int64)
        names = (ctypes.c_char_p * max(self.n_refs, 1))(*[r.encode() for r in self.refnames])
        check(lib().mh_format_segments(self.h, style, None if order is None else _ptr(order), n,
                                       names, k, _ptr(seg_rows), _ptr(out)), 'mh_format_segments')
        return out[:k]

    def write_rows_at(self, fd, offset, style, order=None):
        """Rows order[...] (None: every read) formatted and written to
        descriptor fd at `offset` in one stream (formatting overlapped with
        the write); returns (bytes written, crc32)."""
        if order is not None:
            order = np.ascontiguousarray(order, dtype=np.int64)
            n = len(order)
        else:
            n = self.reads_count()[0]
        names = (ctypes.c_char_p * max(self.n_refs, 1))(*[r.encode() for r in self.refnames])
        written = ctypes.c_int64()
        crc = ctypes.c_uint32()
        check(lib().mh_write_rows_crc(self.h, style, None if order is None else _ptr(order), 0, n,
                                      names, int(fd), int(offset), ctypes.byref(written),
                                      ctypes.byref(crc)), 'mh_write_rows_crc')
        return written.value, crc.value

    def write_segments(self, fd, offsets, crc=True):
        """Write the last format_segments text, segment s at file offset
        offsets[s] of descriptor fd; returns the crc32 of every segment."""
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        out = np.zeros(max(len(offsets), 1), dtype=np.uint32)
        check(lib().mh_write_segments(self.h, int(fd), _ptr(offsets), _ptr(out) if crc else None),
              'mh_write_segments')
        return out[:len(offsets)]

    def reads_count(self):
        n = ctypes.c_int64()
        p = ctypes.c_int()
        check(lib().mh_reads_count(self.h, ctypes.byref(n), ctypes.byref(p)), 'mh_reads_count')
        return n.value, bool(p.value)

    def set_names(self, names):
        arr = (ctypes.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
        check(lib().mh_reads_set_names(self.h, len(names), arr), 'mh_reads_set_names')

    # ---- mapping --------------------------------------------------------
    def map(self, par):
        check(lib().mh_map(self.h, ctypes.byref(par)), 'mh_map')
        self.map_serial += 1

    def fetch(self, first=0, n=None):
        if n is None:
            n = self.reads_count()[0] - first
        out = np.zeros(max(n, 1), dtype=ALN_DTYPE)
        check(lib().mh_alns_fetch(self.h, first, n, _ptr(out)), 'mh_alns_fetch')
        return out[:n]

    def map_counts(self):
        k = max(self.n_refs, 1)
        lines, filt, mapped, first, firstm = (np.zeros(k, dtype=np.int64) for _ in range(5))
        unm = ctypes.c_int64()
        star = ctypes.c_int64()
        star_first = ctypes.c_int64()
        check(lib().mh_map_counts(self.h, _ptr(lines), _ptr(filt), _ptr(mapped), _ptr(first),
                                  _ptr(firstm), ctypes.byref(unm), ctypes.byref(star),
                                  ctypes.byref(star_first)), 'mh_map_counts')
        n = self.n_refs
        return dict(lines=lines[:n], filtered=filt[:n], mapped=mapped[:n], first_row=first[:n],
                    first_mapped=firstm[:n], unmapped=unm.value, star=star.value,
                    star_first=star_first.value)


    def map_stats(self):
        """(reads, banded extensions, CIGAR ops, ungapped fast-path extensions,
        mate-rescue extensions) of the last mapping pass."""
        out = np.zeros(5, dtype=np.int64)
        check(lib().mh_map_stats(self.h, _ptr(out)), 'mh_map_stats')
        return tuple(int(x) for x in out)

    def probe_extend(self, par, items):
        """Diagnostics: items = (n, 4) int32 (read, strand, ref, centre) of
        the loaded reads and built index; returns (n, 8) int32 rows (fast
        path taken, its score, row, lane; band half; the full DP's score,
        row, lane) -- mh_probe_extend."""
        items = np.ascontiguousarray(items, dtype=np.int32).reshape(-1, 4)
        out = np.zeros((max(len(items), 1), 8), dtype=np.int32)
        check(lib().mh_probe_extend(self.h, ctypes.byref(par), len(items), _ptr(items), _ptr(out)),
              'mh_probe_extend')
        return out[:len(items)]

    def test_set_capacities(self, cigar_pool_words=0, pileup_events=0, pileup_event_bytes=0,
                            token_bytes=0):
        """Test entry point: start the grow-and-retry buffers of every later
        call at these capacities (0 = the library's own sizing)."""
        check(lib().mh_test_set_capacities(self.h, cigar_pool_words, pileup_events,
                                           pileup_event_bytes, token_bytes),
              'mh_test_set_capacities')
        self.map_serial += 1

    def retry_counts(self):
        """Retries taken so far: dict(cigar_pool, pileup_events, token_bytes,
        gotoh_wait)."""
        out = np.zeros(4, dtype=np.int64)
        check(lib().mh_retry_counts(self.h, _ptr(out)), 'mh_retry_counts')
        return dict(cigar_pool=int(out[0]), pileup_events=int(out[1]), token_bytes=int(out[2]),
                    gotoh_wait=int(out[3]))

    def test_set_gotoh_wait(self, ticks):
        """Test entry point: the first attempt of every later Gotoh batch gives
        up a neighbour wait after `ticks` of the 100 MHz clock (0: default)."""
        check(lib().mh_test_set_gotoh_wait(self.h, int(ticks)), 'mh_test_set_gotoh_wait')

    def recs(self, first=0, n=None):
        """(n, 20) int32 SAM header fields (ALN_FIELDS order) without CIGARs."""
        if n is None:
            n = self.reads_count()[0] - first
        out = np.zeros((max(n, 1), 20), dtype=np.int32)
        check(lib().mh_recs_fetch(self.h, first, n, _ptr(out)), 'mh_recs_fetch')
        return out[:n]

    def rec_fields(self, names, first=0, n=None):
        """(n, len(names)) int32 of consecutive ALN_FIELDS columns of the
        records (one strided copy; names must be adjacent in ALN_FIELDS)."""
        if n is None:
            n = self.reads_count()[0] - first
        idx = [ALN_FIELDS.index(k) for k in names]
        if idx != list(range(idx[0], idx[0] + len(idx))):
            raise ValueError('rec_fields: columns must be adjacent')
        out = np.empty((max(n, 1), len(idx)), dtype=np.int32)
        check(lib().mh_recs_fetch_fields(self.h, first, n, idx[0], len(idx), _ptr(out)),
              'mh_recs_fetch_fields')
        return out[:n]

    def format_rows(self, style, first=0, n=None, order=None):
        """SAM (style 0) or CSV (style 1) text of reads [first, first+n), or
        of reads order[first:first+n] when an order is given."""
        if order is not None:
            order = np.ascontiguousarray(order, dtype=np.int64)
            if n is None:
                n = len(order) - first
        elif n is None:
            n = self.reads_count()[0] - first
        names = (ctypes.c_char_p * max(self.n_refs, 1))(*[r.encode() for r in self.refnames])
        used = ctypes.c_size_t()
        optr = None if order is None else _ptr(order)
        # a size query formats the rows (host threads) and keeps the text;
        # the second call copies it into a buffer of exactly that size
        check(lib().mh_format_rows(self.h, style, optr, first, n, names, None, 0,
                                   ctypes.byref(used)), 'mh_format_rows')
        buf = np.empty(max(used.value, 1), dtype=np.uint8)
        check(lib().mh_format_rows(self.h, style, optr, first, n, names, _ptr(buf), used.value,
                                   ctypes.byref(used)), 'mh_format_rows')
        return buf[:used.value].tobytes().decode()

    def write_rows(self, out, style, first=0, n=None, order=None):
        """format_rows(...) written to the text file `out`.  A seekable
        UTF-8 / ASCII file that writes '\n' as is (the text is ASCII) gets
        the rows straight from the formatting threads (mh_write_rows at its
        file position); another file gets them through its binary buffer, a
        non-file stream as str."""
        fd = _plain_fd(out)
        if fd is not None:
            if order is not None:
                order = np.ascontiguousarray(order, dtype=np.int64)
                if n is None:
                    n = len(order) - first
            elif n is None:
                n = self.reads_count()[0] - first
            names = (ctypes.c_char_p * max(self.n_refs, 1))(*[r.encode() for r in self.refnames])
            out.flush()
            off = os.lseek(fd, 0, os.SEEK_CUR)
            written = ctypes.c_int64()
            check(lib().mh_write_rows(self.h, style, None if order is None else _ptr(order), first, n,
                                      names, fd, off, ctypes.byref(written)), 'mh_write_rows')
            out.seek(off + written.value)
            return
        text = self.format_rows_bytes(style, first, n, order)
        raw = getattr(out, 'buffer', None)
        enc = (getattr(out, 'encoding', '') or '').lower().replace('-', '')
        if (raw is not None and enc in ('utf8', 'ascii') and os.linesep == '\n' and
                getattr(out, '_writenl', None) in (None, '\n')):
            out.flush()
            raw.write(text)
        else:
            out.write(bytes(text).decode())

    def format_rows_bytes(self, style, first=0, n=None, order=None):
        """format_rows as a uint8 array (no str)."""
        if order is not None:
            order = np.ascontiguousarray(order, dtype=np.int64)
            if n is None:
                n = len(order) - first
        elif n is None:
            n = self.reads_count()[0] - first
        names = (ctypes.c_char_p * max(self.n_refs, 1))(*[r.encode() for r in self.refnames])
        used = ctypes.c_size_t()
        optr = None if order is None else _ptr(order)
        check(lib().mh_format_rows(self.h, style, optr, first, n, names, None, 0,
                                   ctypes.byref(used)), 'mh_format_rows')
        buf = np.empty(max(used.value, 1), dtype=np.uint8)
        check(lib().mh_format_rows(self.h, style, optr, first, n, names, _ptr(buf), used.value,
                                   ctypes.byref(used)), 'mh_format_rows')
        return memoryview(buf[:used.value])

    # ---- pileup ---------------------------------------------------------
    def rows_load(self, flag, ref, pos, cig_off, n_cigar, cigar, seq, qual, offsets, lens, units):
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in (
            (flag, np.int32), (ref, np.int32), (pos, np.int32), (cig_off, np.int32),
            (n_cigar, np.int32), (cigar, np.uint32), (seq, np.uint8), (qual, np.uint8),
            (offsets, np.int64), (lens, np.int32), (units, np.int64))]
        self._rows_keep = arrs
        n_units = len(arrs[10]) // 2
        check(lib().mh_rows_load(self.h, len(arrs[0]), *[_ptr(a) for a in arrs[:10]], n_units,
                                 _ptr(arrs[10])), 'mh_rows_load')

    def rows_load_csv(self, text, refnames):
        """prelim.csv text -> device rows.  Returns dict(n_rows, n_units,
        info, present, unknown): info[:, 0..3] = name id (>= 0: index into
        refnames, < 0: unknown[-1 - id]), flag, longest M run, compact ref id;
        present[k] = refnames index of compact ref k."""
        data = text.encode() if isinstance(text, str) else text
        names = (ctypes.c_char_p * max(len(refnames), 1))(*[r.encode() for r in refnames])
        nr = ctypes.c_int64()
        nu = ctypes.c_int64()
        npres = ctypes.c_int32()
        check(lib().mh_rows_load_csv(self.h, data, len(data), len(refnames), names,
                                     ctypes.byref(nr), ctypes.byref(nu), ctypes.byref(npres)),
              'mh_rows_load_csv')
        info = np.zeros((max(nr.value, 1), 4), dtype=np.int32)
        present = np.zeros(max(npres.value, 1), dtype=np.int32)
        buf = ctypes.create_string_buffer(1 << 20)
        check(lib().mh_rows_info(self.h, _ptr(info), _ptr(present), buf, len(buf)), 'mh_rows_info')
        unknown = buf.value.decode().split('\n')[:-1]
        return dict(n_rows=nr.value, n_units=nu.value, info=info[:nr.value],
                    present=present[:npres.value], unknown=unknown)

    def fastq_lines(self):
        n = ctypes.c_int64()
        check(lib().mh_reads_fastq_lines(self.h, ctypes.byref(n)), 'mh_reads_fastq_lines')
        return n.value

    def pileup(self, source, q_cutoff, ref_lens, only=None):
        """Pile up the last mapping pass (source 0) or the loaded rows (1);
        `only` (reference indices): count just these (mh_pileup_only)."""
        rl = np.ascontiguousarray(ref_lens, dtype=np.int32)
        if only is None:
            check(lib().mh_pileup(self.h, source, q_cutoff, len(rl), _ptr(rl)), 'mh_pileup')
        else:
            sel = np.ascontiguousarray(list(only), dtype=np.int32)
            check(lib().mh_pileup_only(self.h, source, q_cutoff, len(rl), _ptr(rl), len(sel), _ptr(sel)),
                  'mh_pileup_only')

    def pileup_fetch(self, only=None, events=True):
        """The last pileup: every reference's scalars, the counter rows of
        those that received pairs (of `only`'s among them, when given),
        the insertion tokens as arrays (`ev_raw`) and, with events=True, as
        (ref, pos, token, merged pairs) tuples too."""
        n = ctypes.c_int()
        cap = ctypes.c_int32()
        ne = ctypes.c_int64()
        nb = ctypes.c_int64()
        check(lib().mh_pileup_dims(self.h, ctypes.byref(n), ctypes.byref(cap), ctypes.byref(ne),
                                   ctypes.byref(nb)), 'mh_pileup_dims')
        n, cap, ne, nb = n.value, cap.value, ne.value, nb.value
        dense = np.zeros((max(n, 1), cap, 4), dtype=np.int32)
        nflag = np.zeros((max(n, 1), cap), dtype=np.uint8)
        dflag = np.zeros((max(n, 1), cap), dtype=np.uint8)
        rc = np.zeros(max(n, 1), dtype=np.int64)
        fu = np.zeros(max(n, 1), dtype=np.int64)
        mp = np.zeros(max(n, 1), dtype=np.int32)
        # scalars first; then the counter rows of the references that received
        # pairs (np.zeros leaves the other rows as untouched zero pages)
        check(lib().mh_pileup_fetch(self.h, None, None, None, _ptr(rc), _ptr(fu), _ptr(mp)),
              'mh_pileup_fetch')
        sel = np.flatnonzero((fu[:n] >= 0) | (mp[:n] > 0)).astype(np.int32)
        if only is not None:
            sel = np.intersect1d(sel, np.asarray(only, dtype=np.int32)).astype(np.int32)
        if len(sel):   # their rows up to their last counted position, one call
            check(lib().mh_pileup_fetch_refs(self.h, len(sel), _ptr(sel), _ptr(dense), _ptr(nflag),
                                             _ptr(dflag)), 'mh_pileup_fetch_refs')
        eref = np.zeros(max(ne, 1), dtype=np.int32)
        epos = np.zeros(max(ne, 1), dtype=np.int32)
        eoff = np.zeros(max(ne, 1), dtype=np.int32)
        elen = np.zeros(max(ne, 1), dtype=np.int32)
        ecnt = np.zeros(max(ne, 1), dtype=np.int64)
        pool = ctypes.create_string_buffer(max(nb, 1))
        check(lib().mh_pileup_events(self.h, _ptr(eref), _ptr(epos), _ptr(eoff), _ptr(elen),
                                     _ptr(ecnt), pool), 'mh_pileup_events')
        raw = pool.raw[:max(nb, 0)]
        out = dict(dense=dense[:n], nflag=nflag[:n], dflag=dflag[:n], read_counts=rc[:n],
                   first_unit=fu[:n], max_pos=mp[:n], cap=cap,
                   ev_raw=dict(ref=eref[:ne].astype(np.int64), pos=epos[:ne].astype(np.int64),
                               off=eoff[:ne].astype(np.int64), len=elen[:ne].astype(np.int64),
                               count=ecnt[:ne], pool=raw))
        if events:
            # (ref, pos, token, number of merged pairs with that token); the
            # arrays as lists first (a numpy scalar per field costs ~100 ns)
            out['events'] = [(r, p, raw[o:o + ln].decode(), k) for r, p, o, ln, k in
                             zip(eref[:ne].tolist(), epos[:ne].tolist(), eoff[:ne].tolist(),
                                 elen[:ne].tolist(), ecnt[:ne].tolist())]
        return out

    def pileup_scalars(self):
        """read_counts, first_unit, max_pos of the last pileup (n_refs each)."""
        n = ctypes.c_int()
        check(lib().mh_pileup_dims(self.h, ctypes.byref(n), None, None, None), 'mh_pileup_dims')
        k = max(n.value, 1)
        rc = np.zeros(k, dtype=np.int64)
        fu = np.zeros(k, dtype=np.int64)
        mp = np.zeros(k, dtype=np.int32)
        check(lib().mh_pileup_fetch(self.h, None, None, None, _ptr(rc), _ptr(fu), _ptr(mp)),
              'mh_pileup_fetch')
        return rc[:n.value], fu[:n.value], mp[:n.value]

    def pileup_exchange_bytes(self, n_sel):
        s, m, f = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().mh_pileup_exchange_bytes(self.h, n_sel, ctypes.byref(s), ctypes.byref(m),
                                             ctypes.byref(f)), 'mh_pileup_exchange_bytes')
        return s.value, m.value, f.value

    def pileup_export(self, sel, unit_base, dev_sum_ptr, dev_max_ptr, dev_flags_ptr):
        sel = np.ascontiguousarray(sel, dtype=np.int32)
        check(lib().mh_pileup_export(self.h, len(sel), _ptr(sel), unit_base,
                                     ctypes.c_void_p(dev_sum_ptr), ctypes.c_void_p(dev_max_ptr),
                                     ctypes.c_void_p(dev_flags_ptr)), 'mh_pileup_export')

    def pileup_import(self, sel, dev_sum_ptr, dev_max_ptr, dev_flags_ptr):
        sel = np.ascontiguousarray(sel, dtype=np.int32)
        check(lib().mh_pileup_import(self.h, len(sel), _ptr(sel), ctypes.c_void_p(dev_sum_ptr),
                                     ctypes.c_void_p(dev_max_ptr), ctypes.c_void_p(dev_flags_ptr)),
              'mh_pileup_import')

    # ---- kernel timing ---------------------------------------------------
    def pileup_event_bytes(self):
        """(raw insertion-token events, pool bytes) of the last pileup."""
        n, b = ctypes.c_int64(), ctypes.c_int64()
        check(lib().mh_pileup_event_bytes(self.h, ctypes.byref(n), ctypes.byref(b)),
              'mh_pileup_event_bytes')
        return n.value, b.value

    def pileup_events_export(self, dev_events_ptr, dev_pool_ptr):
        check(lib().mh_pileup_events_export(self.h, ctypes.c_void_p(dev_events_ptr),
                                            ctypes.c_void_p(dev_pool_ptr)),
              'mh_pileup_events_export')

    def pileup_events_import(self, n_events, pool_bytes, dev_events_ptr, events_stride,
                             dev_pool_ptr, pool_stride):
        n = np.ascontiguousarray(n_events, dtype=np.int64)
        b = np.ascontiguousarray(pool_bytes, dtype=np.int64)
        check(lib().mh_pileup_events_import(self.h, len(n), _ptr(n), _ptr(b),
                                            ctypes.c_void_p(dev_events_ptr), int(events_stride),
                                            ctypes.c_void_p(dev_pool_ptr), int(pool_stride)),
              'mh_pileup_events_import')

    def profile(self, enable=True):
        check(lib().mh_profile(self.h, int(enable)), 'mh_profile')

    def profile_get(self, kernel):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(lib().mh_profile_get(self.h, kernel.encode(), ctypes.byref(ms), ctypes.byref(n)),
              'mh_profile_get')
        return ms.value, n.value

    # ---- gotoh ----------------------------------------------------------
    def gotoh_align(self, seq1, seq2, gop, gep, is_global, alphabet, matrix):
        cap = len(seq1) + len(seq2) + 1
        o1 = ctypes.create_string_buffer(cap)
        o2 = ctypes.create_string_buffer(cap)
        score = ctypes.c_int()
        mat = np.ascontiguousarray(matrix, dtype=np.int32)
        check(lib().mh_gotoh_align(self.h, seq1.encode(), seq2.encode(), gop, gep, int(is_global),
                                   alphabet.encode(), _ptr(mat), o1, o2, cap, ctypes.byref(score)),
              'mh_gotoh_align')
        return o1.value.decode(), o2.value.decode(), score.value


    def gotoh_align_many(self, pairs, gop, gep, is_global, alphabet, matrix):
        """[(aligned1, aligned2, score)] for [(seq1, seq2)], one launch; a
        pair whose traceback fails gives RuntimeError in its place."""
        n = len(pairs)
        if n == 0:
            return []
        enc = _encoder()
        s1 = (ctypes.c_char_p * n)(*[enc(a) for a, _ in pairs])
        s2 = (ctypes.c_char_p * n)(*[enc(b) for _, b in pairs])
        caps = np.array([len(a) + len(b) + 1 for a, b in pairs], dtype=np.int32)
        o1 = [ctypes.create_string_buffer(int(c)) for c in caps]
        o2 = [ctypes.create_string_buffer(int(c)) for c in caps]
        p1 = (ctypes.c_char_p * n)(*[ctypes.cast(b, ctypes.c_char_p) for b in o1])
        p2 = (ctypes.c_char_p * n)(*[ctypes.cast(b, ctypes.c_char_p) for b in o2])
        score = np.zeros(n, dtype=np.int32)
        status = np.zeros(n, dtype=np.int32)
        mat = np.ascontiguousarray(matrix, dtype=np.int32)
        check(lib().mh_gotoh_align_batch(self.h, n, ctypes.cast(s1, ctypes.c_void_p),
                                         ctypes.cast(s2, ctypes.c_void_p), gop, gep,
                                         int(is_global), alphabet.encode(), _ptr(mat),
                                         ctypes.cast(p1, ctypes.c_void_p),
                                         ctypes.cast(p2, ctypes.c_void_p), _ptr(caps),
                                         _ptr(score), _ptr(status)),
              'mh_gotoh_align_batch')
        return [RuntimeError('Traceback failed, try local alignment') if status[t] else
                (o1[t].value.decode(), o2[t].value.decode(), int(score[t])) for t in range(n)]

    def gotoh_distance_many(self, triples, gop, gep, is_global, alphabet, matrix):
        """The consensus-distance filter's edit distances (remap.py:249-251)
        for [(seq1, seq2, text)]: Levenshtein distance between text and the
        part of seq1 under seq2's aligned span (extract_relevant_seed), each
        alignment as gotoh_align_many's, all reduced on the device
        (mh_gotoh_distance_batch).  A pair whose traceback fails gives
        RuntimeError in its place; one whose aligned seq2 has no non-gap
        column AttributeError, as the reference's re.match gives None."""
        n = len(triples)
        if n == 0:
            return []
        enc = _encoder()
        s1 = (ctypes.c_char_p * n)(*[enc(a) for a, _, _ in triples])
        s2 = (ctypes.c_char_p * n)(*[enc(b) for _, b, _ in triples])
        tx = (ctypes.c_char_p * n)(*[enc(c) for _, _, c in triples])
        dist = np.zeros(n, dtype=np.int32)
        score = np.zeros(n, dtype=np.int32)
        status = np.zeros(n, dtype=np.int32)
        mat = np.ascontiguousarray(matrix, dtype=np.int32)
        check(lib().mh_gotoh_distance_batch(self.h, n, ctypes.cast(s1, ctypes.c_void_p),
                                            ctypes.cast(s2, ctypes.c_void_p),
                                            ctypes.cast(tx, ctypes.c_void_p), gop, gep, int(is_global),
                                            alphabet.encode(), _ptr(mat), _ptr(dist), _ptr(score),
                                            _ptr(status)),
              'mh_gotoh_distance_batch')
        out = []
        for t in range(n):
            if status[t] == -1:
                out.append(RuntimeError('Traceback failed, try local alignment'))
            elif status[t]:
                out.append(AttributeError("'NoneType' object has no attribute 'start'"))
            else:
                out.append(int(dist[t]))
        return out


def _encoder():
    """str -> bytes, one bytes object per distinct string of a batch, so the
    library sees one pointer per distinct sequence (mh_gotoh_align_batch
    uploads each distinct sequence once)."""
    seen = {}

    def enc(x):
        b = seen.get(x)
        if b is None:
            b = seen[x] = x.encode()
        return b
    return enc


def _plain_fd(handle):
    """The descriptor of an open text file the rows can be written to
    directly (seekable, not appending, UTF-8 / ASCII, '\n' written as is),
    else None."""
    try:
        enc = (getattr(handle, 'encoding', '') or '').lower().replace('-', '')
        if (enc not in ('utf8', 'ascii') or os.linesep != '\n' or
                getattr(handle, '_writenl', None) not in (None, '\n') or
                'a' in getattr(handle, 'mode', 'a') or not handle.seekable()):
            return None
        return handle.fileno()
    except (AttributeError, OSError, ValueError):
        return None


class Fastq:
    """A FASTQ file's text staged on the host for a sharded ingest
    (mh_fastq_*): this part's share of the file, framed into records,
    spliced as the ranks exchange boundary records.  Host memory only; no
    device needed."""
    INFO = ('mode', 'c0', 'c1', 'bytes', 'newlines', 'ends_nl', 'starts_nl', 'file_bytes_read',
            'file_size', 'decode_us')

    MEMBER_WINDOW = 32768
    MEMBER_INFO = ('first_bit', 'end_bit', 'crc', 'isize', 'spans', 'file_size', 'open_us')

    def __init__(self, path=None, fd=-1, part=0, parts=1, member=False):
        """member=False: mh_fastq_open_part (this part's text, decoded).
        member=True: mh_fastq_member_open -- part `part` of one gzip member,
        searched but not decoded yet; info holds MEMBER_INFO, and the text
        comes from member_decode / member_tail / member_finish."""
        h = ctypes.c_void_p()
        info = np.zeros(10, dtype=np.int64)
        fn = 'mh_fastq_member_open' if member else 'mh_fastq_open_part'
        check(getattr(lib(), fn)(path.encode() if path else None, int(fd), int(part), int(parts),
                                 ctypes.byref(h), info.ctypes.data_as(_I64P)), fn)
        self.h = h
        self.info = dict(zip(self.MEMBER_INFO if member else self.INFO, (int(x) for x in info)))
        self.info_member = self.info if member else None

    @staticmethod
    def scan_part(path=None, fd=-1, part=0, parts=1):
        """(is gzip, file size, a gzip member starts in this part's byte
        range past offset 0): mh_fastq_scan_part."""
        info = np.zeros(3, dtype=np.int64)
        check(lib().mh_fastq_scan_part(path.encode() if path else None, int(fd), int(part), int(parts),
                                       info.ctypes.data_as(_I64P)), 'mh_fastq_scan_part')
        return bool(info[0]), int(info[1]), bool(info[2])

    def member_decode(self, end_bit):
        """Decode this member part up to end_bit: its text bytes, or -1."""
        info = np.zeros(2, dtype=np.int64)
        check(lib().mh_fastq_member_decode(self.h, int(end_bit), info.ctypes.data_as(_I64P)),
              'mh_fastq_member_decode')
        self.info['decode_us'] = int(info[1])
        return int(info[0])

    def member_tail(self, window):
        """This part's last 32 KiB of text resolved from `window` (the part
        before's tail; None for part 0), or None when it does not resolve."""
        tail = np.zeros(self.MEMBER_WINDOW, dtype=np.uint8)
        w = None if window is None else np.frombuffer(bytes(window), dtype=np.uint8)
        st = lib().mh_fastq_member_tail(self.h, None if w is None else _ptr(w), _ptr(tail))
        if st == -1:
            return None
        check(st, 'mh_fastq_member_tail')
        return tail

    def member_finish(self, window, c0, c1):
        """Resolve the rest of the text; info becomes the open_part fields
        (mode 3) plus 'crc' of this part's text.  False when it does not
        resolve."""
        info = np.zeros(11, dtype=np.int64)
        w = None if window is None else np.frombuffer(bytes(window), dtype=np.uint8)
        st = lib().mh_fastq_member_finish(self.h, None if w is None else _ptr(w), int(c0), int(c1),
                                          info.ctypes.data_as(_I64P))
        if st == -1:
            return False
        check(st, 'mh_fastq_member_finish')
        self.info = dict(zip(self.INFO + ('crc',), (int(x) for x in info)))
        return True

    def frame(self, line0, starts_line):
        """(first record offset, record starts, first record's file line,
        blank record-start line, tail is a lone '\r')."""
        out = np.zeros(5, dtype=np.int64)
        check(lib().mh_fastq_frame(self.h, int(line0), int(bool(starts_line)),
                                   out.ctypes.data_as(_I64P)), 'mh_fastq_frame')
        return tuple(int(x) for x in out)

    def record_offset(self, k):
        off = ctypes.c_int64()
        check(lib().mh_fastq_record_offset(self.h, int(k), ctypes.byref(off)),
              'mh_fastq_record_offset')
        return off.value

    def view(self, lo=0, hi=None):
        """The held text [lo, hi) as a read-only numpy view (no copy; valid
        until the next splice)."""
        p = ctypes.c_void_p()
        n = ctypes.c_int64()
        check(lib().mh_fastq_view(self.h, ctypes.byref(p), ctypes.byref(n)), 'mh_fastq_view')
        hi = n.value if hi is None else hi
        if hi <= lo or not p.value:
            return np.zeros(0, dtype=np.uint8)
        buf = (ctypes.c_uint8 * (hi - lo)).from_address(p.value + lo)
        a = np.ctypeslib.as_array(buf)
        a.flags.writeable = False
        return a

    def size(self):
        p = ctypes.c_void_p()
        n = ctypes.c_int64()
        check(lib().mh_fastq_view(self.h, ctypes.byref(p), ctypes.byref(n)), 'mh_fastq_view')
        return n.value

    def splice(self, lo, hi, front=b'', back=b''):
        """The held text becomes front + text[lo, hi) + back."""
        f = np.frombuffer(bytes(front), dtype=np.uint8) if len(front) else None
        b = np.frombuffer(bytes(back), dtype=np.uint8) if len(back) else None
        check(lib().mh_fastq_splice(self.h, int(lo), int(hi), None if f is None else _ptr(f),
                                    0 if f is None else len(f), None if b is None else _ptr(b),
                                    0 if b is None else len(b)), 'mh_fastq_splice')

    def parse(self, mate=None):
        """The reads the loader would take from this text (and `mate`'s, the
        R2 text, interleaved): ([qname], [seq bytes], [qual bytes]).  Host
        only (tests of the ingest without a device)."""
        n, nb, nn = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_size_t()
        m = mate.h if mate is not None else None
        check(lib().mh_fastq_parse(self.h, m, None, 0, None, None, 0, None, 0, ctypes.byref(n),
                                   ctypes.byref(nb), ctypes.byref(nn)), 'mh_fastq_parse')
        names = ctypes.create_string_buffer(max(nn.value, 1))
        seq = np.zeros(max(nb.value, 1), dtype=np.uint8)
        qual = np.zeros(max(nb.value, 1), dtype=np.uint8)
        lens = np.zeros(max(n.value, 1), dtype=np.int32)
        check(lib().mh_fastq_parse(self.h, m, names, len(names), _ptr(seq), _ptr(qual), len(seq),
                                   _ptr(lens), len(lens), ctypes.byref(n), ctypes.byref(nb),
                                   ctypes.byref(nn)), 'mh_fastq_parse')
        qn = names.raw[:nn.value].decode().split('\n')[:n.value]
        out_s, out_q, at = [], [], 0
        for L in lens[:n.value].tolist():
            out_s.append(seq[at:at + L].tobytes())
            out_q.append(qual[at:at + L].tobytes())
            at += L
        return qn, out_s, out_q

    def close(self):
        if getattr(self, 'h', None):
            lib().mh_fastq_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def crc32_combine(a, b, len_b):
    return int(lib().mh_crc32_combine(int(a) & 0xffffffff, int(b) & 0xffffffff, int(len_b)))


def file_crc32(fd):
    """(size, crc32) of a whole open file."""
    size = ctypes.c_int64()
    crc = ctypes.c_uint32()
    check(lib().mh_file_crc32(fd, ctypes.byref(size), ctypes.byref(crc)), 'mh_file_crc32')
    return size.value, crc.value


def file_checksum(fd):
    """(size, checksum) of a whole open file: (crc32 << 32) | adler32."""
    size = ctypes.c_int64()
    sum_ = ctypes.c_uint64()
    check(lib().mh_file_checksum(fd, ctypes.byref(size), ctypes.byref(sum_)), 'mh_file_checksum')
    return size.value, sum_.value


def levenshtein(a, b):
    return lib().mh_levenshtein(a.encode(), b.encode())


def levenshtein_many(pairs):
    """[edit distance] for [(a, b)], pairs spread over host threads."""
    n = len(pairs)
    if n == 0:
        return []
    a = (ctypes.c_char_p * n)(*[x.encode() for x, _ in pairs])
    b = (ctypes.c_char_p * n)(*[y.encode() for _, y in pairs])
    out = np.zeros(n, dtype=np.int32)
    check(lib().mh_levenshtein_batch(n, ctypes.cast(a, ctypes.c_void_p),
                                     ctypes.cast(b, ctypes.c_void_p), _ptr(out)),
          'mh_levenshtein_batch')
    return [int(x) for x in out]


def cigar_text(aln):
    if aln['ref'] < 0:
        return '*'
    return ''.join('{}{}'.format(int(c) >> 4, OP_CHARS[int(c) & 7])
                   for c in aln['cigar'][:aln['n_cigar']])
