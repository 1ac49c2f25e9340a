"""CPU restatement of the reference's FASTQ record encoding — the checker of the HIP
formatter (ganon_fastq_*, include/ganon.h).

TEST INFRASTRUCTURE ONLY: used by tests/ (and through ``OracleEngine.format_fastq`` by the
CPU pipeline tests, which pin it against the reference's own FASTQ files in tests/golden),
never by the product.

Follows, per record:
* ``AnonymizedRead.set_original_sequence`` — the sequence upper-cased (anonymizer_methods.py:163);
  the nt16 decode "=ACMGRSVTWYHKDBN" is already upper case;
* ``reverse_complement`` (anonymizer_methods.py:205-213): ``np.vectorize(reverses.get)`` over the
  bases with ``reverses`` = {A:T, C:G, G:C, T:A, N:N} (:22), flipped; a base outside ACGTN maps
  to None and the decode raises TypeError — reported here as ``BadRecord(i)``;
  the qualities are reversed in the same call, which undoes the forward orientation
  ``get_forward_qualities`` gave them: the caller says per record whether the
  stored qualities print reversed (``qual_rev``);
* ``get_anonymized_fastq_record`` (:215-243): name + '/1' or '/2', sequence, qualities
  ``chr(q + 33)``; ``write_pair`` (short_read_tumor_normal_anonymizer.py:134-165) adds the
  record's trailing newline: '@name/m\\nSEQ\\n+\\nQUAL\\n'.

The native formatters write one byte per quality, (q + 33) & 0xFF: identical to this for
phred <= 94 (SAM's printable range; BAM's 0xFF "missing" makes pysam return None and the
reference fail), which is what the tests use.
"""
from __future__ import annotations

NT16 = "=ACMGRSVTWYHKDBN"
REVERSES = {ord("A"): ord("T"), ord("C"): ord("G"), ord("G"): ord("C"), ord("T"): ord("A"), ord("N"): ord("N")}


class BadRecord(Exception):
    def __init__(self, index: int):
        super().__init__(f"record {index}: reverse read with a base outside ACGTN")
        self.index = index


def _nibbles(buf, nib0: int, n: int):
    out = []
    for k in range(n):
        i = nib0 + k
        b = int(buf[i >> 1])
        out.append(b & 0xF if i & 1 else b >> 4)
    return out


def format_record(recs: dict, i: int) -> bytes:
    sb = recs["seq_bufs"][int(recs["seq_sel"][i])]
    seq = [ord(NT16[c]) for c in _nibbles(sb, int(recs["seq_nib_off"][i]), int(recs["seq_len"][i]))]
    qb = recs["qual_bufs"][int(recs["qual_sel"][i])]
    q0, Q = int(recs["qual_off"][i]), int(recs["qual_len"][i])
    quals = [int(x) for x in qb[q0:q0 + Q]]
    if recs["reverse"][i]:
        comp = [REVERSES.get(b) for b in seq]
        if any(c is None for c in comp):
            raise BadRecord(i)
        seq = comp[::-1]
    if recs["qual_rev"][i]:
        quals = quals[::-1]
    names = recs["names"]
    no, nl = int(recs["name_off"][i]), int(recs["name_len"][i])
    name = bytes(names[no:no + nl]).decode("latin-1")
    text = f"@{name}/{int(recs['mate'][i])}\n{bytes(seq).decode()}\n+\n{''.join(chr(q + 33) for q in quals)}\n"
    return text.encode()   # the reference's text files are UTF-8: chr(q + 33) > 127 takes two bytes


def format_records(recs: dict) -> bytes:
    return b"".join(format_record(recs, i) for i in range(len(recs["seq_len"])))
