/*
 * ganon_host.h — native host helpers around the masking path (libganon_host.so):
 * a BGZF/BAM decoder into structure-of-arrays columns and the FASTQ record formatter.
 *
 * These replace, for this path only, what the reference gets from pysam/htslib
 * (BAM decode behind AlignmentFile.fetch/pileup, pileup_io.pyx:8-41, :124-298) and the
 * per-read FASTQ encoding of AnonymizedRead (anonymizer_methods.py:205-243, with the
 * quality-orientation quirk SURVEY Q1), plus write_pair's record framing
 * (short_read_tumor_normal_anonymizer.py:134-165). Pure CPU code: no device calls.
 */
#ifndef GANON_HOST_H
#define GANON_HOST_H

#include <stdint.h>

#ifdef __cplusplus
#define GANON_HOST_API extern "C" __attribute__((visibility("default")))
#else
#define GANON_HOST_API __attribute__((visibility("default")))
#endif

typedef struct ganon_bam ganon_bam;

/* Column view of a decoded BAM. Record order = file order. All arrays owned by the
 * ganon_bam handle and valid until ganon_bam_close. */
typedef struct ganon_bam_view {
  int64_t n_records;
  int32_t n_ref;
  const char *ref_names;        /* NUL-separated */
  const int64_t *ref_name_off;  /* [n_ref] */
  const int64_t *ref_len;       /* [n_ref] */
  /* per record */
  const int32_t *tid, *pos, *end;   /* end = htslib bam_endpos (pos + ref len, >= pos + 1) */
  const int32_t *flag, *mapq, *l_seq, *n_cigar;
  const int32_t *mate_tid, *mate_pos, *tlen;
  const int64_t *name_off;          /* into names, NUL-terminated */
  const int32_t *name_len;
  const int64_t *cig_off;           /* into cigar (u32 ops) */
  const int64_t *seq_off;           /* byte offset into seq (packed nt16, BAM layout) */
  const int64_t *qual_off;          /* into qual (raw phred, BAM order) */
  const int64_t *aux_off;           /* into aux (raw BAM aux bytes) */
  const int32_t *aux_len;
  /* blobs */
  const char *names;
  int64_t names_bytes;
  const uint32_t *cigar;
  int64_t cigar_ops;
  const uint8_t *seq;
  int64_t seq_bytes;
  const uint8_t *qual;
  int64_t qual_bytes;
  const uint8_t *aux;
  int64_t aux_bytes;
} ganon_bam_view;

/* Decode the whole file (BGZF inflate on `threads` threads). Returns 0 or <0. */
GANON_HOST_API int ganon_bam_open(const char *path, int threads, ganon_bam **out);
GANON_HOST_API int ganon_bam_view_get(ganon_bam *bam, ganon_bam_view *view);
GANON_HOST_API const char *ganon_bam_error(ganon_bam *bam);
GANON_HOST_API void ganon_bam_close(ganon_bam *bam);
GANON_HOST_API const char *ganon_host_last_error(void);

/* FASTQ formatter. For record i:
 *   '@' name '/' mate '\n' SEQ '\n' '+' '\n' QUAL '\n'
 * SEQ: seq_len[i] nt16 nibbles starting at nibble seq_nib_off[i] of seq_buf[seq_sel[i]],
 *      printed as "=ACMGRSVTWYHKDBN"; when reverse[i], reverse-complemented with the
 *      reference's table {A<->T, C<->G, N->N} (any other code is an error).
 * QUAL: qual_len[i] bytes at qual_off[i] of qual_buf[qual_sel[i]], +33, printed in
 *      stored order when qual_rev[i] == 0 and reversed otherwise.
 * Returns the number of bytes written, or -(index+1) of the first bad record, or
 * INT64_MIN when `cap` is too small. */
GANON_HOST_API int64_t ganon_fastq_format(int64_t n, const uint8_t *const *seq_buf, const uint8_t *seq_sel,
                                          const int64_t *seq_nib_off, const int32_t *seq_len,
                                          const uint8_t *reverse, const uint8_t *const *qual_buf,
                                          const uint8_t *qual_sel, const int64_t *qual_off,
                                          const int32_t *qual_len, const uint8_t *qual_rev,
                                          const char *names, const int64_t *name_off, const int32_t *name_len,
                                          const uint8_t *mate, char *out, int64_t cap);

/* Upper-case a FASTA slice and pack it to nt16 nibbles (2 per byte, high first). Bytes
 * outside "=ACMGRSVTWYHKDBN" (after upper-casing) become N (15). `out` has (n+1)/2 bytes. */
GANON_HOST_API void ganon_pack_nt16(const char *ascii, int64_t n, uint8_t *out);

#endif /* GANON_HOST_H */
