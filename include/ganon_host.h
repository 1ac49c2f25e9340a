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
/* The host BGZF inflater in use: "libdeflate" (the system libdeflate.so.0, loaded at run time) or
 * "zlib" (no libdeflate, or GANON_INFLATE=zlib in the environment at the first decode). */
GANON_HOST_API const char *ganon_host_inflate_backend(void);

/* Contig reader: bounded-memory decode of one reference sequence at a time (the records of BAM tid
 * `tid`, file order). Seeks through the BAM index (<path>.bai or <path minus .bam>.bai) when one
 * is present and valid, otherwise streams forward (a request for an earlier tid rescans from the
 * first record). The returned ganon_bam carries the full reference list and is released with
 * ganon_bam_close. The reader header view has n_records = 0. */
typedef struct ganon_bam_reader ganon_bam_reader;
/* entries of each record's SA tag (len(tag.rstrip(';').split(';')), anonymizer_methods.py:103-106),
 * -1 without one, from the aux blob of a ganon_bam_view */
GANON_HOST_API int ganon_aux_sa_count(const uint8_t *aux, const int64_t *aux_off, const int32_t *aux_len, int64_t n,
                                      int32_t *out);
GANON_HOST_API int ganon_bam_reader_open(const char *path, int threads, ganon_bam_reader **out);
GANON_HOST_API int ganon_bam_reader_has_index(const ganon_bam_reader *reader);
/* Compressed bytes read and inflated per step (default 32 MiB, at least 128 KiB). */
GANON_HOST_API int ganon_bam_reader_set_window(ganon_bam_reader *reader, int64_t bytes);
/* Block inflater for the reader's windows: inflates n_blocks raw DEFLATE payloads at
 * comp[in_off[i], + in_len[i]) to out[out_off[i], + out_len[i]); 0 on success. The signature of
 * ganon_inflate_hostcb (include/ganon.h: the GPU inflate, user = a ganon_ctx). Windows of at least
 * min_blocks blocks go to it, smaller ones to the reader's zlib threads; fn NULL restores zlib for
 * all. The reader is not thread-safe; neither need fn be for one reader. */
typedef int (*ganon_inflate_fn)(void *user, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                                const int32_t *in_len, const int64_t *out_off, const int32_t *out_len,
                                int64_t n_blocks, uint8_t *out, int64_t out_total);
GANON_HOST_API int ganon_bam_reader_set_inflater(ganon_bam_reader *reader, ganon_inflate_fn fn, void *user,
                                                 int64_t min_blocks);
/* Where the reader's scans put their inflated bytes: a buffer from alloc (grown through it, freed
 * through free_fn, kept across the reader's scans) instead of fresh pageable memory — with
 * ganon_pinned_alloc / ganon_pinned_free (include/ganon.h) the GPU inflater's device-to-host copies
 * go by DMA. alloc returns 0 on success. NULL, NULL restores fresh buffers. */
typedef int (*ganon_buf_alloc_fn)(int64_t bytes, void **out);
typedef int (*ganon_buf_free_fn)(void *p);
GANON_HOST_API int ganon_bam_reader_set_buffer_alloc(ganon_bam_reader *reader, ganon_buf_alloc_fn alloc,
                                                     ganon_buf_free_fn free_fn);
/* Region decoder (ganon_region_decode of include/ganon.h, user = a ganon_ctx): a region read's
 * first window of at least min_blocks blocks goes to it whole — inflated, walked and filtered on the
 * device, the kept records' columns back in one block the returned table owns (release(block) at
 * ganon_bam_close). It returns 1 with *cols / *block when the region ends inside the window, 0 after
 * writing the inflated window to out (the reader's walk goes on from there), -1 on an inflate error.
 * The window is then sized to the region's index span (up to 16x the reader's window). fn NULL
 * turns it off. */
typedef int (*ganon_region_fn)(void *user, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                               const int32_t *in_len, const int64_t *out_off, const int32_t *out_len,
                               int64_t n_blocks, uint8_t *out, int64_t out_total, int64_t p0, int32_t tid,
                               int64_t beg, int64_t end, int at_eof, ganon_bam_view *cols, void **block);
GANON_HOST_API int ganon_bam_reader_set_region_decoder(ganon_bam_reader *reader, ganon_region_fn fn, void *user,
                                                       int64_t min_blocks, ganon_buf_free_fn release);
GANON_HOST_API int ganon_bam_reader_header(ganon_bam_reader *reader, ganon_bam_view *view);
GANON_HOST_API int ganon_bam_reader_contig(ganon_bam_reader *reader, int32_t tid, ganon_bam **out);
/* The records of tid overlapping [beg, end) (0-based; htslib's region semantics: pos < end and
 * bam_endpos > beg, placed unmapped records at [pos, pos + 1)), file order, through the index's
 * linear offsets (an index is required): what the reference's fetch(contig, beg, end) returns
 * (pileup_io.pyx:138-139, short_read_tumor_normal_anonymizer.py:570-573). */
GANON_HOST_API int ganon_bam_reader_region(ganon_bam_reader *reader, int32_t tid, int64_t beg, int64_t end,
                                           ganon_bam **out);
GANON_HOST_API void ganon_bam_reader_close(ganon_bam_reader *reader);

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

/* Indel left-overs applied to formatted records (replaces the per-record host loop of
 * AnonymizedRead.mask_or_anonymize_left_over_variants, anonymizer_methods.py:254-270, and
 * mask_or_modify_indel, :178-203, then get_anonymized_fastq_record, :205-243). Record i is
 * rec[rec_off[i] .. rec_off[i+1]) as ganon_fastq_format wrote it without edits; reverse[i] its
 * BAM strand; its edits e in [edit_off[i], edit_off[i+1]) are (edits[3e] read position,
 * edits[3e+1] VariantType value: 2 DEL, 3 INS, others only length-checked, edits[3e+2] length),
 * a DEL inserting alleles[allele_off[e] .. allele_off[e+1]); stably sorted by type and applied
 * times[i] times to the stored-orientation sequence and the forward-oriented
 * qualities (Q1, Q6). Writes the edited records back to back into `out` (cap bytes), lengths in
 * out_len. Returns 0; 1 = reverse read with a base outside ACGTN after its edits (Q7, the
 * reference's KeyError), 2 = sequence and quality lengths diverge (ValueError), 3 = a DEL on a
 * read without qualities (int(nan), ValueError), with *bad = the record; -1 bad arguments or
 * malformed record, -2 `cap` too small. */
GANON_HOST_API int ganon_fastq_edit(int64_t n, const char *recs, const int64_t *rec_off, const uint8_t *reverse,
                                    const int32_t *times, const int64_t *edit_off, const int64_t *edits,
                                    const char *alleles, const int64_t *allele_off, char *out, int64_t cap,
                                    int64_t *out_len, int64_t *bad);

/* Copy the byte ranges src[off[i] .. off[i] + len[i]) back to back into dst (cap bytes): the
 * output stage slicing records out of a job's pre-formatted FASTQ blob. Returns the bytes
 * written, or -1 for a range outside src_len or a too-small cap. */
GANON_HOST_API int64_t ganon_gather_ranges(const char *src, int64_t src_len, int64_t n, const int64_t *off,
                                           const int64_t *len, char *dst, int64_t cap);

/* The same from two sources: range i is src0[off[i] ..) when sel[i] == 0, src1[off[i] ..) when 1 (the
 * output stage splicing a job's few indel-edited records in among its pre-formatted ones with one
 * copy). Returns the bytes written, or -1 for a bad selector, a range outside its source or a
 * too-small cap. */
GANON_HOST_API int64_t ganon_gather_ranges2(const char *src0, int64_t len0, const char *src1, int64_t len1, int64_t n,
                                            const uint8_t *sel, const int64_t *off, const int64_t *len, char *dst,
                                            int64_t cap);

/* Decoder phase clocks: wall seconds the reader's calling threads spent per phase since the last
 * reset (parse of BGZF headers, inflate, record walk of the region scan, copies of kept runs, the
 * columns' record walk, sizes pass, columns pass), summed over calls and threads; out[0..n). Returns
 * the number of phases. Diagnostics (tools/e2e_bench.py). */
GANON_HOST_API int ganon_host_phase_times(double *out, int n, int reset);

/* Upper-case a FASTA slice and pack it to nt16 nibbles (2 per byte, high first). Bytes
 * outside "=ACMGRSVTWYHKDBN" (after upper-casing) become N (15). `out` has (n+1)/2 bytes. */
GANON_HOST_API void ganon_pack_nt16(const char *ascii, int64_t n, uint8_t *out);

/* ---- Scope planner -------------------------------------------------------
 * Replaces, for one tumor/normal pair, the control flow of anonymize_genome
 * (short_read_tumor_normal_anonymizer.py:625-760) that decides which reads meet in which pileup
 * scope and which scope's masked copy of each read is written, in which order: sections
 * (SR:245-276), anonymize_window (SR:279-372), anonymize_inter_window_region + iter_fetch_pair
 * (SR:498-558, pileup_io.pyx:124-298), the yield order of CompleteGermlineAnonymizer.anonymize
 * (anonymizer_methods.py:472-532), write_pair / to_pair_anonymized_reads / unmapped-mate pairing /
 * single ends (SR:134-165, :375-406, :561-622, AM:320-389) and the statistics recorder's events.
 * Same results as genomeanonymizer_amd/planner.py (SamplePlanner.run). */
enum {
  GANON_PLAN_OK = 0,
  GANON_PLAN_E_ARG = -1,
  GANON_PLAN_E_NOMEM = -3,
  GANON_PLAN_E_VALUE = -10,        /* the reference raises ValueError (region errors Q4, Q10, ...) */
  GANON_PLAN_E_TYPE = -11,         /* the reference raises TypeError (Q8, reads without SEQ, ...)  */
  GANON_PLAN_E_UNSUPPORTED = -12,  /* input this build does not restate                           */
  GANON_PLAN_E_INDEX = -13         /* the reference raises IndexError (np.put out of range)        */
};
typedef struct ganon_plan_table {  /* one sample, file order (columns of a ganon_bam_view) */
  int64_t n;
  const int32_t *tid, *pos, *end, *flag, *l_seq, *n_cigar;
  const char *names;
  const int64_t *name_off;
  const int32_t *name_len;
  int32_t n_ref;
  const int64_t *ref_len;          /* [n_ref] BAM header lengths                            */
  const int32_t *tid_of_contig;    /* [n_contigs] this BAM's tid of each FASTA contig, -1 none */
  const int32_t *mate_tid;         /* per record; read only in contig mode                    */
  const int32_t *mate_pos;         /* per record; read only in job mode (ganon_plan_input.sec_hi) */
  const int32_t *n_sa;             /* per record: entries of its SA tag, -1 without one; NULL = none.
                                      Records with an SA tag or the SECONDARY / SUPPLEMENTARY flag make
                                      their name "complex" (contig mode only; see ganon_plan_view.objs) */
} ganon_plan_table;
typedef struct ganon_plan_input {
  ganon_plan_table tables[2];      /* 0 tumor, 1 normal                                      */
  int32_t n_contigs;               /* FASTA contigs, FASTA order                              */
  const int64_t *contig_len;
  const char *contig_names;        /* NUL-terminated names at contig_name_off (messages)      */
  const int64_t *contig_name_off;
  int32_t n_windows;               /* variant windows in get_windows order (SR:71-131)        */
  const int32_t *win_contig;
  const int64_t *win_first, *win_last;
  /* Contig mode (contig_mode != 0): plan FASTA contig only_contig alone from tables holding that
   * contig's records (ganon_bam_reader_contig). Names with a record whose mate is on another
   * reference sequence or unplaced (mate_tid != tid) are "cross" names: every operation of the
   * reference's pairing state on them (write_pair of a complete pair, the to_pair store of an
   * incomplete one, a pass-through) becomes a placeholder event (kinds 3 / 4 / 5) that
   * ganon_resolver_contig decides with the state of the contigs before; the other names are planned
   * here exactly. Their pairs still unwritten at the contig's end are exported (view.left), and so
   * are the placed-unmapped records of the contig's windows that pair_unmapped_mates may need
   * (view.cand). */
  int32_t contig_mode;
  int32_t only_contig;
  /* Contig mode: names planned as cross names although every record of theirs on this contig says
   * otherwise (n_force names at force_off / force_len; NULL / 0 = none). The caller lists the names of
   * secondary alignments on earlier contigs whose mate is on this one: the reference's pairing state
   * for such a name may hold that alignment's object when this contig's records arrive. */
  int64_t n_force;
  const char *force_names;
  const int64_t *force_off;
  const int32_t *force_len;
  /* Job mode (contig mode with sec_hi >= 0): plan only sections [sec_lo, sec_hi) of the contig (its
   * sections in get_genome_sections order, SR:245-276) from tables holding the records overlapping
   * [reg_lo, reg_hi), the union of those sections' region queries (the jobs of a contig tile it, so
   * a record overlapping another job's range is in both tables). Names with a record reaching outside
   * the range, or whose mate starts outside it, are cross names too; the candidates are the windows
   * of these sections only. */
  int32_t sec_lo, sec_hi;
  int64_t reg_lo, reg_hi;
} ganon_plan_input;
typedef struct ganon_plan ganon_plan;
typedef struct ganon_plan_view {
  int32_t n_scopes;
  const int32_t *scope_contig, *scope_window;      /* window -1: a gap cluster scope      */
  const int64_t *scope_first, *scope_last, *scope_span_start, *scope_span_end;
  const int64_t *scope_t_off, *scope_n_off;        /* [n_scopes + 1] CSR into t_rows/n_rows */
  const int64_t *t_rows, *n_rows;                  /* mapped pileup reads, file order      */
  int64_t n_events;                                /* I/O log                              */
  const int32_t *events;     /* 7 per event: kind (0 open, 1 write, 2 close), handle, file dataset,
                                file mate slot, instance dataset, instance scope (-1 unmasked),
                                reapply: 1 when the written object's left-overs are applied a second
                                time (its left-over flag re-set by update_anonymized_read_from_other,
                                AM:281-287) */
  const int64_t *event_rows; /* instance row of a write event, -1 otherwise                 */
  int64_t n_stats;
  const int32_t *stats;      /* 2 per event: kind (0 window -> window index, 1 outside, 2 scope id) */
  int64_t n_single[2];
  const int64_t *single[2];  /* per dataset: (row, scope, reapply) of the single-end records  */
  int32_t write_single_end;
  /* contig mode: events may also hold kind 3 (a complete pair of a cross name: two consecutive events,
   * slot 0 then 1), 4 (store in to_pair, write and drop when complete: anonymize_window SR:313-360),
   * 5 (pass-through store, write when complete: SR:375-406); the 7th int is the event's clock. */
  int64_t n_left;
  const int64_t *left;       /* 11 per unwritten pair: clock, has0, ds0, scope0, row0, has1, ds1, scope1, row1,
                                reapply0, reapply1 */
  int64_t n_cand;
  const int64_t *cand;       /* 6 per record: window, dataset (-1: this window's fetch raises), row,
                                slot (-1: no READ1/READ2 flag), 1 if the record has no SEQ, object info
                                of the record (bit 0 supplementary, bit 1 has an SA tag, bits 8.. SA
                                entries: the AnonymizedRead it creates, AM:98-108) */
  /* contig mode, complex names (a record with an SA tag, or a secondary / supplementary alignment):
   * the reference's AnonymizedRead objects (anonymizer_methods.py:84-287) of such a name are planned
   * here and resolved sample-wide. objs: 10 int64 per object: scope (-1: created by a pass-through),
   * dataset, slot, creator row (the alignment that created it: orientation, SA count), base row (the
   * first non-supplementary alignment, whose sequence it holds; -1: still supplementary), offset and
   * count in obj_rows of its alignments in the scope (registration order), offset and count in
   * obj_rows of the supplementary records it recorded, creator info (bit 0 supplementary, bit 1 has an
   * SA tag, bits 8.. SA entries). Events kind 6: the objects of one yield of a complex name (e[2] bit 0
   * first event of the group, bits 1..2 objects in the group; e[3] slot, e[4] dataset, e[5] scope,
   * e[6] clock, row = object index); kind 7: a pass-through record of a complex name (row = object).
   * skip: 3 per incidence (scope, dataset, row) left out of the indel tally (a later alignment of a
   * read already met in the scope: seen_read_alns, variation_classifier.py:196-207). */
  int64_t n_objs;
  const int64_t *objs;
  int64_t n_obj_rows;
  const int64_t *obj_rows;
  int64_t n_skip;
  const int64_t *skip;
} ganon_plan_view;
/* Returns GANON_PLAN_OK or a GANON_PLAN_E_* code (message: ganon_plan_last_error()). */
GANON_HOST_API int ganon_plan_run(const ganon_plan_input *in, ganon_plan **out);
GANON_HOST_API int ganon_plan_view_get(const ganon_plan *plan, ganon_plan_view *view);
GANON_HOST_API void ganon_plan_free(ganon_plan *plan);
GANON_HOST_API const char *ganon_plan_last_error(void);
/* ---- Cross-contig resolution (contig mode) -------------------------------------------------------
 * Replays, contig after contig in FASTA order, the placeholder events of the contig plans against the
 * sample-wide pairing state (to_pair_anonymized_reads / written_read_ids, SR:134-165, :304-406,
 * AM:351-389), then the end of the sample: pair_unmapped_mates (SR:561-600) over the exported
 * candidates and the single ends (SR:603-622). Instances are (job, dataset, scope, row), job = the
 * contig plan they come from. A write is 7 int64: file dataset, file slot, job, dataset, scope, row,
 * reapply (see ganon_plan_view.events). */
typedef struct ganon_resolver ganon_resolver;
GANON_HOST_API int ganon_resolver_create(ganon_resolver **out);
GANON_HOST_API void ganon_resolver_free(ganon_resolver *r);
/* ops: the placeholder events of job's plan (7 int32 each, plan layout) with their rows and read
 * names; left: the plan's unwritten pairs (11 int64 each) with names. obj_ids (NULL, or one per
 * obj_rows entry, -1 = none): content identities of the objects' records, for the supplementary
 * records an object recorded (get_supplementary_hash_from_aln, AM:61-62): a record the tables of two
 * jobs both hold (job mode) is one record. out_n[i] receives the number of writes op i makes (0 or
 * 2), out_w 14 int64 per op. */
GANON_HOST_API int ganon_resolver_contig(ganon_resolver *r, int32_t job, int64_t n_ops, const int32_t *ops,
                                         const int64_t *op_rows, const char *op_names, const int64_t *op_name_off,
                                         const int32_t *op_name_len, int64_t n_left, const int64_t *left,
                                         const char *left_names, const int64_t *left_name_off,
                                         const int32_t *left_name_len, int64_t n_objs, const int64_t *objs,
                                         const int64_t *obj_rows, const int64_t *obj_ids, int32_t *out_n,
                                         int64_t *out_w);
/* Complex names (ganon_plan_view.objs): an object is identified by (job << 32) | index for the plan's
 * objects, or 1 << 62 | k for a plain instance the resolver had to follow as an object. A write of an
 * object is (file dataset, slot, -1, dataset, -2, serial, 0); what it writes follows from the object
 * log, 8 int64 per entry, in order: (1, id, job, dataset, scope, row, reapply, 0) a plain instance
 * becomes object id; (2, dst, src) update_anonymized_read_from_other(dst, src) (AM:281-287);
 * (3, id) mask_or_anonymize_left_over_variants if flagged (AM:254-270); (4, id, job, dataset, row)
 * update_from_primary_mapping with that record (AM:142-149); (5, id, serial) the object is written.
 * ganon_resolver_take_log copies the entries made since the last call and returns their count (all of
 * them, and clears the log, when cap >= count). */
GANON_HOST_API int64_t ganon_resolver_take_log(ganon_resolver *r, int64_t *out, int64_t cap);
/* Pending instances (4 int64 each: job, dataset, scope, row; an object: -1, dataset, -2, id); returns
 * the count (all of them when cap >= count, else only the count). */
GANON_HOST_API int64_t ganon_resolver_pending(ganon_resolver *r, int64_t *out, int64_t cap);
/* Names written on an earlier contig by a plan that did not treat them as cross names (an off-contig
 * secondary alignment met later names one: its name's other records said nothing of it). Every name
 * the resolver has no state for is marked written; returns how many were marked. */
GANON_HOST_API int64_t ganon_resolver_mark_written(ganon_resolver *r, int64_t n, const char *names,
                                                   const int64_t *name_off, const int32_t *name_len);
/* cand: 8 int64 per record (job, window, dataset, row, slot, no-SEQ flag, object info as in
 * ganon_plan_view.cand, content identity or -1) in window order, with names. tail (14 int64 per candidate) receives the writes of pair_unmapped_mates (count n_tail);
 * single[d] (5 int64 per record: job, dataset, scope, row, reapply; capacity = ganon_resolver_pending
 * count) the single ends in dictionary order (counts n_single[2]). Returns GANON_PLAN_OK or GANON_PLAN_E_VALUE / _TYPE with the
 * reference's error (message: ganon_plan_last_error). */
GANON_HOST_API int ganon_resolver_finish(ganon_resolver *r, int64_t n_cand, const int64_t *cand, const char *names,
                                         const int64_t *name_off, const int32_t *name_len, int64_t *tail,
                                         int64_t *n_tail, int64_t *single0, int64_t *single1, int64_t *n_single,
                                         int32_t *write_single_end);

/* ---- Objects of complex names (the content side of the resolver log) ---------------------------
 * AnonymizedRead content (anonymizer_methods.py:84-287): sequence and forward qualities of the base
 * record, SNV masks written at the query position of the alignment that found them (directly once
 * the object holds a primary mapping, else as left-overs), left-over lists applied stable by variant
 * type, update_anonymized_read_from_other, update_from_primary_mapping, the FASTQ record with the
 * creator's orientation (genomeanonymizer_amd/objects.py is the Python restatement the tests compare).
 *
 * ganon_objects_pack: what one contig plan's objects need, as one self-contained blob (it travels
 * between ranks): the plan objects, their records (name, flag, position, CIGAR, bases, qualities),
 * the bases the device changed in every (alignment, scope) copy (with their reference columns) and
 * the indel left-overs. */
typedef struct ganon_objects_table {   /* one sample's records of the contig (ReadTable columns) */
  int64_t n;
  const int32_t *flag, *pos, *l_seq, *n_cigar, *name_len;
  const int64_t *seq_off, *qual_off, *name_off, *cig_off;
  const uint8_t *seq;                  /* nt16, 2 per byte, BAM layout                            */
  const uint8_t *qual;                 /* BAM order; first byte 0xFF = missing                    */
  const char *names;
  const uint32_t *cigar;
} ganon_objects_table;
typedef struct ganon_objects_src {
  ganon_objects_table tables[2];
  int64_t n_objs;
  const int64_t *objs;                 /* ganon_plan_view.objs (10 per object)                    */
  int64_t n_obj_rows;
  const int64_t *obj_rows;
  int64_t n_inc;
  const int64_t *inc;                  /* (dataset, row, scope) per masked copy                   */
  const int64_t *inc_nib;              /* nibble index of that copy in masked                     */
  const uint8_t *masked;               /* the device output                                       */
  int64_t n_ind;
  const int64_t *ind;                  /* 6 per left-over: dataset, row, scope, in_read_pos, type
                                          (2 DEL, 3 INS), length                                  */
  const char *ind_ref;                 /* reference allele of each (ind_ref_off / ind_ref_len)    */
  const int64_t *ind_ref_off;
  const int32_t *ind_ref_len;
} ganon_objects_src;
typedef struct ganon_blob ganon_blob;
GANON_HOST_API int ganon_objects_pack(const ganon_objects_src *src, ganon_blob **out);
GANON_HOST_API int64_t ganon_blob_size(const ganon_blob *b);
GANON_HOST_API const uint8_t *ganon_blob_data(const ganon_blob *b);
GANON_HOST_API void ganon_blob_free(ganon_blob *b);
typedef struct ganon_objects ganon_objects;
GANON_HOST_API int ganon_objects_create(ganon_objects **out);
GANON_HOST_API void ganon_objects_free(ganon_objects *o);
/* a packed job (its object ids are job << 32 | index) */
GANON_HOST_API int ganon_objects_add_job(ganon_objects *o, int32_t job, const uint8_t *blob, int64_t size);
/* a plain instance's content for log entries 1 / 4: its formatted record (writer.py), BAM flag and
 * indel left-overs (n_ind entries of 3: in_read_pos, type, length, with reference alleles) */
GANON_HOST_API int ganon_objects_add_plain(ganon_objects *o, int64_t job, int64_t ds, int64_t scope, int64_t row,
                                           int32_t flag, const char *fastq, int64_t len, int64_t n_ind,
                                           const int64_t *ind, const char *ind_ref, const int64_t *ind_ref_off,
                                           const int32_t *ind_ref_len);
/* replay resolver log entries (ganon_resolver_take_log); GANON_PLAN_OK or the reference's error
 * (E_INDEX / E_TYPE / E_VALUE / E_UNSUPPORTED, message: ganon_objects_last_error) */
GANON_HOST_API int ganon_objects_run(ganon_objects *o, int64_t n, const int64_t *log);
/* bytes of written object `serial` (returns the size; copies and forgets it when cap >= size; -1:
 * unknown serial) */
GANON_HOST_API int64_t ganon_objects_take(ganon_objects *o, int64_t serial, char *out, int64_t cap);
/* after a round: create the pending objects of the added jobs, drop every other state and the jobs */
/* every written object at once: returns their count, *total their bytes; fills serials / lens / buf
 * (and forgets them) when cap >= *total */
GANON_HOST_API int64_t ganon_objects_take_all(ganon_objects *o, int64_t *serials, int64_t *lens, char *buf,
                                              int64_t cap, int64_t *total);
GANON_HOST_API int ganon_objects_settle(ganon_objects *o, int64_t n_live, const int64_t *live_ids);
GANON_HOST_API const char *ganon_objects_last_error(void);

/* Order in which the write events of an I/O log (ganon_plan_view.events layout, 7 ints each)
 * reach the four FASTQ files (tumor .1, tumor .2, normal .1, normal .2 = file dataset * 2 + slot):
 * every "open" creates four CPython append-mode text handles (8 KiB TextIOWrapper chunks over a
 * BufferedWriter of `block` bytes), records become visible when a flush reaches the raw layer
 * (SR:297-299, 516-518, 564-566). rec_len[i]: byte length of write event i's record.
 * order (>= number of write events) receives event indices, file by file; file_count[4] their
 * counts. Returns the number written or GANON_PLAN_E_ARG (unbalanced log). */
GANON_HOST_API int64_t ganon_io_replay(int64_t n_events, const int32_t *events, const int64_t *rec_len,
                                       int64_t block, int64_t *order, int64_t *file_count);

#endif /* GANON_HOST_H */
