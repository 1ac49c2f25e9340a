"""The reference's own plugin boundary, served by the GPU: a drop-in for
``CompleteGermlineAnonymizer`` (anonymizer_methods.py:422-556) that the reference's driver can call
once per scope exactly as it calls its own class (``anonymize_window``,
short_read_tumor_normal_anonymizer.py:289-293):

    anonymize(variant_to_keep, tumor_normal_pileup, ref_genome, stats_recorder=None)
        -> Generator[[AnonymizedRead | None, AnonymizedRead | None]]

Per call:
1. the pileup generator (pileup_io.iter_pileups, pileup_io.pyx:8-41: (tumor column | None,
   normal column | None) in position order) is consumed once and kept;
2. its distinct alignments become a one-scope ``ganon_batch`` (BAM nt16 bases of
   ``query_sequence``, BAM CIGAR words, dataset, every read written by the scope, the scope's
   reference slice from ``ref_genome.fetch``, the kept SNV) masked by libganon_hip.so
   (``HipMasker.mask(..., indels=True)``): the SNV tally, the tumor/normal state machine and the
   masking (variation_classifier.py:144-215, variants.py:33-39, AM:537-556) and the germline indel
   tally (variation_classifier.py:52-141) run on the device;
3. the columns are replayed through the reference's control flow with the device's decisions:
   read objects are created and merged as ``add_anonymized_read_pair_to_collection_from_alignment``
   does (AM:320-349), at each normal column the masked calls of that position are applied to
   their supporting reads — base overwrite, or a left-over for supplementary reads and indels —
   and counted (``mask_germline_variants``, AM:537-556), complete pairs whose rightmost end lies
   left of the column are yielded (AM:472-514), the rest at the end (AM:515-533).

The yielded objects are the reference's ``AnonymizedRead`` when the reference package is
importable (the adapter living in the reference tree); otherwise the restated
``AnonymizedRead`` of this module, which produces the same FASTQ record
(``get_anonymized_fastq_record``, AM:215-243).

Batching: one scope per call is what the reference's driver offers; the kernels are built for many
scopes per batch (genomeanonymizer_amd/anonymizer_methods.py), so this path trades throughput for a
zero-change integration.
"""
from __future__ import annotations

import array
import dataclasses
from typing import Dict, Generator, List, Optional, Tuple

import numpy as np

from .variants import VariantType

NT16 = "=ACMGRSVTWYHKDBN"
_NT16_OF = {c: i for i, c in enumerate(NT16)}
PAIR_1_IDX, PAIR_2_IDX = 0, 1
_CIGAR_OPS = "MIDNSHP=X"
_COMPLEMENT = {ord("A"): ord("T"), ord("C"): ord("G"), ord("G"): ord("C"), ord("T"): ord("A"), ord("N"): ord("N")}


# ---- the reference's object model, restated (used when the reference is not importable) ------

@dataclasses.dataclass(eq=False)
class CalledVariant:
    """The fields of CalledGenomicVariant (variants.py:42-56) the masking path reads; equality is
    the reference's call identity (variants.py:83-96)."""
    seq_name: str
    pos: int
    end: int
    variant_type: VariantType
    length: int
    allele: str
    ref_allele: str

    def __eq__(self, other):
        return (other is not None and self.seq_name == other.seq_name and self.variant_type == other.variant_type
                and self.pos == other.pos and self.end == other.end and self.length == other.length
                and self.allele == other.allele)


def supplementary_hash(aln) -> str:
    """get_supplementary_hash_from_aln (AM:63-64)."""
    return (f"{aln.reference_name};{aln.reference_start};{aln.cigarstring};{aln.query_sequence};"
            f"{aln.query_qualities};{aln.flag}")


class AnonymizedRead:
    """The per-read state the reference yields (AM:84-288): ASCII bases (upper-cased), forward
    qualities, pair index, supplementary bookkeeping, left-over edits."""

    def __init__(self, aln, dataset_idx: int, variant_type=VariantType):
        self._vt = variant_type
        self.query_name = aln.query_name
        self.is_read1, self.is_read2, self.is_reverse = aln.is_read1, aln.is_read2, aln.is_reverse
        self.dataset_idx = dataset_idx
        self._set_from(aln)
        self.is_supplementary = aln.is_supplementary
        self.has_supplementary = aln.has_tag("SA")
        self.supplementary_hashes = set()
        self.n_supplementaries = 0
        if self.has_supplementary:
            self.n_supplementaries = len(aln.get_tag("SA").rstrip(";").split(";"))
            if self.is_supplementary:
                self.record_supplementary_aln(supplementary_hash(aln))
        self.left_over_variants_to_mask: List[Tuple[int, object]] = []
        self.has_left_overs_to_mask = False

    def _set_from(self, aln):
        self.anonymized_sequence_array = np.frombuffer(bytearray(aln.query_sequence.upper().encode()), np.uint8)
        self.anonymized_qualities_array = aln.get_forward_qualities()

    def get_pair_idx(self):
        if self.is_read1:
            return PAIR_1_IDX
        if self.is_read2:
            return PAIR_2_IDX

    def anonymized_read_is_complete(self) -> bool:
        if self.is_supplementary:
            return False
        return not (self.has_supplementary and len(self.supplementary_hashes) < self.n_supplementaries)

    def record_supplementary_aln(self, h: str) -> None:
        self.supplementary_hashes.add(h)

    def update_from_primary_mapping(self, aln) -> None:
        if aln.is_supplementary:
            raise ValueError("update_from_primary_mapping got a supplementary alignment (only the primary "
                             "record may supply the sequence and qualities)")
        self._set_from(aln)
        self.is_supplementary = False

    def update_anonymized_read_from_other(self, other) -> None:
        if other.has_left_overs_to_mask:
            self.left_over_variants_to_mask.extend(other.left_over_variants_to_mask)
        if self.left_over_variants_to_mask:
            self.has_left_overs_to_mask = True
        for h in other.supplementary_hashes:
            self.record_supplementary_aln(h)

    def mask_or_modify_base_pair(self, pos_in_read: int, new_base: str) -> None:
        np.put(self.anonymized_sequence_array, pos_in_read, ord(new_base), mode="raise")

    def mask_or_modify_indel(self, irp: int, v) -> None:
        seq, qual = self.anonymized_sequence_array, self.anonymized_qualities_array
        if v.variant_type == self._vt.INS:
            seq = np.concatenate((seq[:irp], seq[irp + v.length:]))
            qual = qual[:irp] + qual[irp + v.length:]
        elif v.variant_type == self._vt.DEL:
            ref = np.frombuffer(bytearray(v.ref_allele.encode()), np.uint8)
            seq = np.concatenate((seq[:irp], ref, seq[irp:]))
            qual = qual[:irp] + array.array("B", [int(np.mean(qual))] * v.length) + qual[irp:]
        if len(seq) != len(qual):
            raise ValueError(f"left-over edits left {len(seq)} bases but {len(qual)} qualities")
        self.anonymized_sequence_array, self.anonymized_qualities_array = seq, qual

    def add_left_over_variant(self, irp: int, v) -> None:
        if not self.is_supplementary and v.variant_type == self._vt.SNV:
            raise ValueError(f"{self.query_name}: an SNV left-over on a read that holds its primary record "
                             f"(its SNVs are masked directly)")
        self.left_over_variants_to_mask.append((irp, v))
        self.has_left_overs_to_mask = True

    def mask_or_anonymize_left_over_variants(self) -> None:
        if self.is_supplementary:
            raise ValueError(f"{self.query_name}: left-over edits applied before the primary record was met")
        self.left_over_variants_to_mask.sort(key=lambda x: x[1].variant_type.value)
        for irp, v in self.left_over_variants_to_mask:
            if v.variant_type == self._vt.SNV:
                self.mask_or_modify_base_pair(irp, v.ref_allele)
            if v.variant_type in (self._vt.DEL, self._vt.INS):
                self.mask_or_modify_indel(irp, v)
        self.has_left_overs_to_mask = False

    def get_anonymized_fastq_record(self) -> str:
        if self.is_reverse:
            self.anonymized_sequence_array = np.flip(np.vectorize(_COMPLEMENT.get)(self.anonymized_sequence_array))
            self.anonymized_qualities_array = reversed(self.anonymized_qualities_array)
        name = f"{self.query_name}/{PAIR_1_IDX + 1}" if self.is_read1 else f"{self.query_name}/{PAIR_2_IDX + 1}"
        seq = "".join(map(chr, self.anonymized_sequence_array))
        qual = "".join(chr(x + 33) for x in self.anonymized_qualities_array)
        return f"@{name}\n{seq}\n+\n{qual}"


@dataclasses.dataclass
class ObjectModel:
    """The classes the yielded objects are built from."""
    anonymized_read: type
    called_variant: type        # ctor(seq_name, pos, end, var_type, length, allele, ref_allele)
    variant_type: type


def default_model() -> ObjectModel:
    """The reference's classes when its package is importable (the adapter inside the reference
    tree), else this module's restatement."""
    try:  # pragma: no cover - only inside the reference tree
        from src.GenomeAnonymizer.anonymizer_methods import AnonymizedRead as RefRead
        from src.GenomeAnonymizer.variants import CalledGenomicVariant
        from variant_extractor.variants import VariantType as RefVT
        return ObjectModel(RefRead, CalledGenomicVariant, RefVT)
    except Exception:
        return ObjectModel(lambda aln, ds: AnonymizedRead(aln, ds), CalledVariant, VariantType)


# ---- the adapter ----------------------------------------------------------------------------

def _pack_nt16(codes: np.ndarray) -> np.ndarray:
    if len(codes) & 1:
        codes = np.concatenate([codes, np.zeros(1, np.uint8)])
    return ((codes[0::2] << 4) | codes[1::2]).astype(np.uint8)


def _nt16_codes(s: str) -> np.ndarray:
    return np.fromiter((_NT16_OF.get(c, 15) for c in s.upper()), np.uint8, len(s))


class GpuCompleteGermlineAnonymizer:
    """Drop-in for the reference's CompleteGermlineAnonymizer: the same ``anonymize`` generator
    contract and ``reset``. ``engine``: anything with ``HipMasker.mask``'s signature (default: a
    HipMasker on ``device``)."""

    def __init__(self, device: int = 0, engine=None, model: Optional[ObjectModel] = None):
        self.device = device
        self._engine = engine
        self.model = model or default_model()
        self.anonymized_reads: Dict[str, List[Optional[object]]] = {}
        self._built: set = set()      # alignments whose AnonymizedRead was built once this scope

    @property
    def engine(self):
        if self._engine is None:
            from . import native
            self._engine = native.HipMasker(self.device)
        return self._engine

    def reset(self) -> None:
        self.anonymized_reads = {}
        self._built = set()

    # -- 1 + 2: the scope as a device batch ------------------------------------------------------
    def _device_calls(self, columns, variant_to_keep, ref_genome):
        """Mask the scope's reads on the device. Returns (contig, SNV masks by normal column,
        indel calls by normal column): {pos: [(call, [(dataset, aln_key, query_pos)])]}."""
        alns: Dict[tuple, Tuple[int, object]] = {}
        contig = None
        for pair in columns:
            for ds, col in enumerate(pair):
                if col is None:
                    continue
                contig = col.reference_name
                for pr in col.pileups:
                    a = pr.alignment
                    alns.setdefault(self._key(ds, a), (ds, a))
        if not alns:
            return contig, {}, {}
        keys = list(alns)
        reads = [alns[k] for k in keys]
        starts = np.array([a.reference_start for _, a in reads], np.int64)
        ends = np.array([a.reference_end if a.reference_end is not None else a.reference_start + 1
                         for _, a in reads], np.int64)
        s0, s1 = int(starts.min()), int(max(ends.max(), starts.min() + 1))
        ref = ref_genome.fetch(contig, s0, s1).upper()
        seq_parts, seq_off, cig, cig_off, n_cig, L = [], [], [], [], [], []
        off = 0
        for _, a in reads:
            codes = _nt16_codes(a.query_sequence)
            p = _pack_nt16(codes)
            seq_parts.append(p)
            seq_off.append(off)
            off += len(p)
            cig_off.append(len(cig))
            ct = a.cigartuples or []
            cig.extend((n << 4) | op for op, n in ct)
            n_cig.append(len(ct))
            L.append(len(codes))
        n = len(reads)
        keep_pos, keep_code = -1, 0
        v = variant_to_keep
        if v is not None and v.variant_type == self.model.variant_type.SNV and v.pos == v.end and v.length == 1 \
                and len(v.allele) == 1 and v.allele in _NT16_OF and v.allele != "N" and v.seq_name == contig:
            keep_pos, keep_code = int(v.pos), _NT16_OF[v.allele]
        arrays = {
            "ref_start": starts.astype(np.int32), "read_len": np.array(L, np.int32),
            "seq_off": np.array(seq_off, np.int64),
            "seq_nt16": np.concatenate(seq_parts) if seq_parts else np.zeros(0, np.uint8),
            "cig_off": np.array(cig_off, np.int64), "n_cig": np.array(n_cig, np.int32),
            "cigar": np.array(cig, np.uint32), "dataset": np.array([ds for ds, _ in reads], np.uint8),
            "write_scope": np.zeros(n, np.int32), "scope_incid_off": np.array([0, n], np.int64),
            "incid_read": self._incidence_order(reads), "scope_span_start": np.array([s0], np.int32),
            "scope_span_len": np.array([s1 - s0], np.int32), "scope_ref_off": np.array([0], np.int64),
            "ref_nt16": _pack_nt16(_nt16_codes(ref)), "keep_pos": np.array([keep_pos], np.int32),
            "keep_code": np.array([keep_code], np.uint8),
        }
        out, calls, bases, totals, irecs = self.engine.mask(arrays, indels=True)
        VT = self.model.variant_type
        snv: Dict[int, Dict[str, list]] = {}
        for r, (ds, a) in enumerate(reads):
            o, Lr = int(arrays["seq_off"][r]), L[r]
            if Lr == 0:
                continue
            nib_in = self._nibbles(arrays["seq_nt16"], o, Lr)
            nib_out = self._nibbles(out, o, Lr)
            for q in np.nonzero(nib_in != nib_out)[0].tolist():
                p = self._ref_pos(a, q)
                snv.setdefault(p, {}).setdefault(NT16[nib_in[q]], []).append((ds, keys[r], q, NT16[nib_out[q]]))
        snv_calls: Dict[int, list] = {}
        for p, by_allele in snv.items():
            for allele, sup in by_allele.items():
                call = self.model.called_variant(contig, p, p, VT.SNV, 1, allele, sup[0][3])
                snv_calls.setdefault(p, []).append((call, [(ds, k, q) for ds, k, q, _ in sup]))
        n_snv = sum(len(v) for v in snv_calls.values())
        if n_snv != int(calls[0]):
            raise RuntimeError(f"device masked {int(calls[0])} SNV calls, {n_snv} recovered from the bytes")
        indel_calls: Dict[int, list] = {}
        live: Dict[tuple, object] = {}
        for rec in irecs.tolist():
            _, pos, length, vtype, rank, kind, read, irp = rec
            ds, a = reads[read]
            if kind == 0:   # INDEL_CALL: identity from the first registered support
                vt = VT.INS if vtype == VariantType.INS.value else VT.DEL
                end = pos + 1 if vt == VT.INS else pos + length - 1
                allele = a.query_sequence[irp:irp + (length if vt == VT.INS else 2)]
                call = self.model.called_variant(contig, pos, end, vt, length, allele,
                                                 ref_genome.fetch(contig, pos, end + 1).upper())
                live[(pos, rank)] = call
                indel_calls.setdefault(pos, []).append((rank, call, []))
            else:
                for rk, call, sup in indel_calls[pos]:
                    if rk == rank:
                        sup.append((ds, keys[read], irp))
        for pos in indel_calls:
            indel_calls[pos] = [(c, s) for _, c, s in sorted(indel_calls[pos], key=lambda x: x[0])]
        return contig, snv_calls, indel_calls

    @staticmethod
    def _key(ds, a) -> tuple:
        return (ds, a.query_name, a.flag, a.reference_start, a.cigarstring)

    @staticmethod
    def _incidence_order(reads) -> np.ndarray:
        """The indel tally's registration order (include/ganon.h): tumor reads in file order, then
        normal reads — file order is reference_start order within a dataset."""
        order = sorted(range(len(reads)), key=lambda r: (reads[r][0], reads[r][1].reference_start, r))
        return np.array(order, np.int32)

    @staticmethod
    def _nibbles(buf: np.ndarray, byte_off: int, n: int) -> np.ndarray:
        b = buf[byte_off:byte_off + (n + 1) // 2]
        nib = np.empty(2 * len(b), np.uint8)
        nib[0::2] = b >> 4
        nib[1::2] = b & 0xF
        return nib[:n]

    @staticmethod
    def _ref_pos(a, q: int) -> int:
        p, qq = a.reference_start, 0
        for op, n in a.cigartuples:
            if op in (0, 7, 8):
                if qq <= q < qq + n:
                    return p + (q - qq)
                qq += n
                p += n
            elif op in (1, 4):
                qq += n
            elif op in (2, 3):
                p += n
        raise RuntimeError("masked base outside the aligned part of its read")

    # -- 3: the reference's per-scope control flow ---------------------------------------------
    def _add_from_alignment(self, aln, ds: int) -> None:
        """add_anonymized_read_pair_to_collection_from_alignment (AM:320-349). The reference builds
        a new AnonymizedRead at every column (Q13) and keeps it only when the pair slot is empty;
        here it is built when it is kept, or the first time an alignment is met (so that whatever
        the constructor would raise is raised at the same column) — a long read meets ~10^4
        columns."""
        pair = self.anonymized_reads.get(aln.query_name)
        key = self._key(ds, aln)
        idx = PAIR_1_IDX if aln.flag & 0x40 else PAIR_2_IDX if aln.flag & 0x80 else None
        new = None
        if key not in self._built or pair is None or pair[idx] is None:
            self._built.add(key)
            new = self.model.anonymized_read(aln, ds)
            idx = new.get_pair_idx()
        if pair is None:
            pair = self.anonymized_reads[aln.query_name] = [None, None]
            pair[idx] = new
            return
        if pair[idx] is None:
            pair[idx] = new
        cur = pair[idx]
        if not aln.is_supplementary and cur.is_supplementary:
            cur.update_from_primary_mapping(aln)
        if aln.is_supplementary:
            cur.record_supplementary_aln(_supplementary_hash(aln, self.model))

    @staticmethod
    def _writeable(p1, p2) -> bool:
        return p1 is not None and p2 is not None and p1.anonymized_read_is_complete() and \
            p2.anonymized_read_is_complete()

    @staticmethod
    def _mask_left_overs(p1, p2) -> None:
        for p in (p1, p2):
            if p is not None and not p.is_supplementary and p.has_left_overs_to_mask:
                p.mask_or_anonymize_left_over_variants()

    def _mask_column(self, pos: int, snv_calls, indel_calls, stats_recorder) -> None:
        """mask_germline_variants (AM:537-556) with the device's calls at this normal column."""
        VT = self.model.variant_type
        for group in (snv_calls.get(pos, ()), indel_calls.get(pos, ())):
            for call, supports in group:
                for ds, key, q in supports:
                    read = self.anonymized_reads.get(key[1])[self._pair_of(key)]
                    if read.is_supplementary or call.variant_type != VT.SNV:
                        read.add_left_over_variant(q, call)
                        continue
                    read.mask_or_modify_base_pair(q, call.ref_allele)
                if stats_recorder is not None:
                    stats_recorder.count_variant(call)

    @staticmethod
    def _pair_of(key) -> int:
        flag = key[2]
        return PAIR_1_IDX if flag & 0x40 else PAIR_2_IDX

    def anonymize(self, variant_to_keep, tumor_normal_pileup, ref_genome,
                  stats_recorder=None) -> Generator[list, None, None]:
        # pysam columns are views of the pileup engine's live buffer (the next step of the iterator
        # overwrites them): every column is copied while it is current, its reads as
        # (alignment, query_position) — pysam's PileupRead.alignment is a copy of the record
        columns = [tuple(None if c is None else _ColumnSnapshot(c) for c in p) for p in tumor_normal_pileup]
        _, snv_calls, indel_calls = self._device_calls(columns, variant_to_keep, ref_genome)
        # the kept window variant is never masked nor counted (AM:546-547): SNVs on the device,
        # indels here (their identity includes the allele)
        if variant_to_keep is not None:
            for pos in list(indel_calls):
                indel_calls[pos] = [(c, s) for c, s in indel_calls[pos] if c != variant_to_keep]
        to_yield: Dict[str, int] = {}
        for pair in columns:
            for ds, col in enumerate(pair):
                if col is None:
                    continue
                for pr in col.pileups:
                    a = pr.alignment
                    self._add_from_alignment(a, ds)
                    end = a.reference_end
                    to_yield[a.query_name] = end if a.query_name not in to_yield else max(to_yield[a.query_name], end)
                if ds != 1:
                    continue
                pos = col.reference_pos
                self._mask_column(pos, snv_calls, indel_calls, stats_recorder)
                done = []
                for rid, right in to_yield.items():
                    cand = self.anonymized_reads.get(rid)
                    if right < pos and self._writeable(cand[PAIR_1_IDX], cand[PAIR_2_IDX]):
                        self._mask_left_overs(cand[PAIR_1_IDX], cand[PAIR_2_IDX])
                        yield cand
                        self.anonymized_reads.pop(rid)
                        done.append(rid)
                for rid in done:
                    to_yield.pop(rid)
        for rid, pair in self.anonymized_reads.items():
            self._mask_left_overs(pair[PAIR_1_IDX], pair[PAIR_2_IDX])
            yield pair
        self.reset()


class _ReadSnapshot:
    __slots__ = ("alignment", "query_position")

    def __init__(self, pr):
        self.alignment = pr.alignment
        self.query_position = pr.query_position


class _ColumnSnapshot:
    """The parts of a pysam PileupColumn the adapter reads, copied while the column is current."""
    __slots__ = ("reference_pos", "reference_name", "pileups")

    def __init__(self, col):
        self.reference_pos = col.reference_pos
        self.reference_name = col.reference_name
        self.pileups = [_ReadSnapshot(pr) for pr in col.pileups]


def _supplementary_hash(aln, model) -> str:
    return supplementary_hash(aln)
