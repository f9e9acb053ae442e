"""Alphabets, quality characters and CLI defaults (semantics of src/constants.py:1-15)."""

NULL_NUCLEOTIDES_CHAR = "N"                 # k-mers containing it are not indexed (src/kmer.py:145)
NULL_NUCLEOTIDES = {NULL_NUCLEOTIDES_CHAR}
REAL_NUCLEOTIDES_CHARS = "ACGT"             # the only read bases the FASTQ grammar accepts
REAL_NUCLEOTIDES = set(REAL_NUCLEOTIDES_CHARS)
NUCLEOTIDES_CHARS = REAL_NUCLEOTIDES_CHARS + NULL_NUCLEOTIDES_CHAR
NUCLEOTIDES = set(NUCLEOTIDES_CHARS)

# PHRED+33 quality characters: every printable ASCII character from '!' (33) to '~' (126).
# The pseudo-alignment filters use the raw ASCII code, without the -33 offset (quirk 5).
PHRED33_SCORES = {chr(c): c for c in range(33, 127)}

DEFAULT_UNIQUE_THRESHOLD = 1
DEFAULT_AMBIGUOUS_THRESHOLD = 1
DEFAULT_SIMILARITY_THRESHOLD = 0.95
