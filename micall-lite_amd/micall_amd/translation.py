"""
Codon translation for the aln2counts stage (host side).

Mirrors micall/utils/translation.py:40-142 for the arguments aln2counts uses
(`offset`, `ambig_char`; mixtures translated, nothing resolved or listed):

  * a codon with more than one '-' or any '?' is '-' when it is '---' and
    `ambig_char` otherwise (:86-93);
  * a codon of plain A/C/G/T is looked up (:98-101);
  * a codon with IUPAC mixtures (W R K Y S M B D H V N, and a single '-')
    is expanded to every plain codon; one amino acid -> that amino acid,
    several -> `ambig_char` (:107-141);
  * a trailing partial codon is dropped (:80-81).

`codon_chars()` folds all of that into the 6 x 6 x 6 table over the
aligned-read alphabet A C G T N - that the aln2counts kernels read
(micall-lite_amd/csrc/mh_a2c.hip); the device never translates anything else.
"""
import itertools

_BASES = 'TCAG'
_AMINOS = 'FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG'
CODON_DICT = {a + b + c: _AMINOS[16 * i + 4 * j + k]
              for i, a in enumerate(_BASES)
              for j, b in enumerate(_BASES)
              for k, c in enumerate(_BASES)}

MIXTURES = {'W': 'AT', 'R': 'AG', 'K': 'GT', 'Y': 'CT', 'S': 'CG', 'M': 'AC',
            'V': 'AGC', 'H': 'ATC', 'D': 'ATG', 'B': 'TGC', 'N': 'ATGC', '-': 'ATGC'}
# sorted resolution -> IUPAC letter (translation.py:27-29)
AMBIG = {''.join(sorted(v)): k for k, v in MIXTURES.items() if k != '-'}

# aligned-read alphabet of the device codon table, in class order
READ_ALPHABET = 'ACGTN-'


def translate_codon(codon, ambig_char='?'):
    """One upper-case 3-letter codon (translation.py:78-141)."""
    if codon.count('-') > 1 or '?' in codon:
        return '-' if codon == '---' else ambig_char
    if all(c in 'ACGT' for c in codon):
        return CODON_DICT[codon]
    choices = [MIXTURES.get(c, c) for c in codon]
    aminos = {CODON_DICT[''.join(p)] for p in itertools.product(*choices)}
    return aminos.pop() if len(aminos) == 1 else ambig_char


def translate(seq, offset=0, ambig_char='?'):
    """translation.translate(seq, offset, ambig_char=...) with the default
    mixture handling; accepts str or bytes like the reference (:66-67)."""
    if isinstance(seq, bytes):
        seq = seq.decode('utf-8')
    seq = '-' * offset + seq.upper()
    n = len(seq) - len(seq) % 3
    return ''.join(translate_codon(seq[i:i + 3], ambig_char) for i in range(0, n, 3))


def codon_chars(ambig_char='?'):
    """216 bytes: the translation of codon c0 c1 c2 over READ_ALPHABET at
    index 36*c0 + 6*c1 + c2 (the table the device kernels read)."""
    return ''.join(translate_codon(''.join(c), ambig_char)
                   for c in itertools.product(READ_ALPHABET, repeat=3)).encode()
