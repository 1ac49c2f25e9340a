/*
 * ganon.h — C ABI of the MI355X germline-variant masking path (libganon_hip.so).
 *
 * Drop-in boundary for the reference's per-scope anonymizer plugin:
 *   CompleteGermlineAnonymizer.anonymize(variant_to_keep, tumor_normal_pileup, ref_genome,
 *                                        stats_recorder)      anonymizer_methods.py:431-535
 * called once per scope by anonymize_window (short_read_tumor_normal_anonymizer.py:289-293).
 * Inside one call the reference classifies every aligned base of every tumor/normal read
 * of the scope (variation_classifier.py:144-215, SomaticVariationType state machine
 * variants.py:33-39) and overwrites, in every supporting read, each SNV seen in >=1 tumor
 * AND >=1 normal read with the reference base (mask_germline_variants,
 * anonymizer_methods.py:537-556 -> mask_or_modify_base_pair :170-176), except the window's
 * own VCF variant (:546-547). This ABI processes MANY scopes per call: the host scheduler
 * (genomeanonymizer_amd/planner.py) lays the scopes of a contig out as one batch.
 *
 * Conventions
 *  - Plain pointers and sizes only; all coordinates are 0-based and contig-relative.
 *  - Bases are BAM nt16 codes ("=ACMGRSVTWYHKDBN"), packed two per byte, high nibble
 *    first, exactly as stored in a BAM record; every read starts at a byte boundary.
 *  - CIGAR ops are BAM u32 words (len << 4 | op), op in MIDNSHP=X.
 *  - Return value 0 on success, a negative GANON_E* code otherwise; the message is in
 *    ganon_last_error(ctx). No C++ exception or abort crosses the ABI.
 *  - One ctx per GPU per host thread; a ctx is not thread-safe.
 *  - There is no CPU implementation behind this ABI: without a usable gfx950 device
 *    ganon_ctx_create fails with GANON_E_DEVICE.
 */
#ifndef GANON_H
#define GANON_H

#include <stdint.h>

#ifdef __cplusplus
#define GANON_API extern "C" __attribute__((visibility("default")))
#else
#define GANON_API __attribute__((visibility("default")))
#endif

#define GANON_ABI_VERSION 5

enum {
  GANON_OK = 0,
  GANON_E_ARG = -1,      /* invalid argument / inconsistent batch (message says which) */
  GANON_E_DEVICE = -2,   /* no device, wrong architecture, HIP runtime error */
  GANON_E_NOMEM = -3,    /* device or host allocation failed */
  GANON_E_STATE = -4     /* call out of order (e.g. download before run) */
};

/* Totals written by ganon_batch_download / ganon_mask_batch (int64 each). */
enum {
  GANON_T_MASKED_SNV_CALLS = 0, /* TN SNV calls masked, summed over scopes (stats #SNV) */
  GANON_T_MASKED_BASES = 1,     /* bases overwritten in written reads                   */
  GANON_T_READS_IN = 2,         /* reads presented to the kernels                      */
  GANON_T_READS_WRITTEN = 3,    /* reads with write_scope >= 0                          */
  GANON_T_SCOPES = 4,           /* scopes in the batch                                  */
  GANON_T_RARE_SCOPES = 5,      /* scopes re-run on the 16-code tally (non-ACGTN bases) */
  GANON_T_LARGE_TILES = 6,      /* position tiles of scopes wider than the LDS cap      */
  GANON_N_TOTALS = 8
};

typedef struct ganon_ctx ganon_ctx;
typedef struct ganon_dbatch ganon_dbatch;
typedef struct ganon_ref ganon_ref;

typedef struct ganon_batch {
  int32_t n_reads;
  int32_t n_scopes;
  int64_t n_incid;
  int64_t seq_bytes;              /* size of seq_nt16 (and of the output buffer)          */
  int64_t n_cigar_ops;            /* size of cigar                                        */
  int64_t ref_bytes;              /* size of ref_nt16                                     */
  /* reads (BAM order) */
  const int32_t *ref_start;       /* [n_reads] BAM pos                                    */
  const int32_t *read_len;        /* [n_reads] l_seq                                      */
  const int64_t *seq_off;         /* [n_reads] byte offset of the read in seq_nt16        */
  const uint8_t *seq_nt16;        /* [seq_bytes]                                          */
  const int64_t *cig_off;         /* [n_reads] first op of the read in cigar              */
  const int32_t *n_cig;           /* [n_reads]                                            */
  const uint32_t *cigar;          /* [n_cigar_ops]                                        */
  const uint8_t *dataset;         /* [n_reads] 0 tumor, 1 normal                          */
  const int32_t *write_scope;     /* [n_reads] scope whose tally masks this read, -1 none */
  /* scopes: CSR over incidences (a read may belong to several scopes) */
  const int64_t *scope_incid_off; /* [n_scopes + 1]                                       */
  const int32_t *incid_read;      /* [n_incid]                                            */
  const int32_t *scope_span_start;/* [n_scopes] first position covered by the scope reads */
  const int32_t *scope_span_len;  /* [n_scopes] covered extent (max end - span_start)     */
  const int64_t *scope_ref_off;   /* [n_scopes] nibble index of span_start in ref_nt16    */
  const uint8_t *ref_nt16;        /* [ref_bytes] upper-cased reference, nt16, 2 per byte  */
  const int32_t *keep_pos;        /* [n_scopes] kept SNV position, -1 none (AM:546-547)   */
  const uint8_t *keep_code;       /* [n_scopes] nt16 code of the kept alt allele          */
} ganon_batch;

/* Context: one device, one HIP stream, device scratch. */
GANON_API int ganon_ctx_create(int device, ganon_ctx **out);
GANON_API int ganon_ctx_destroy(ganon_ctx *ctx);
GANON_API const char *ganon_last_error(ganon_ctx *ctx);
/* Page-locked host memory (hipHostMalloc) for the host side of large device copies: the FASTQ
 * records a job formats on the device land in it by DMA, with no staging copy on the host's cores.
 * Returns GANON_OK or GANON_E_NOMEM. */
GANON_API int ganon_pinned_alloc(int64_t bytes, void **out);
GANON_API int ganon_pinned_free(void *p);
/* The process's page-locked block counters since it started: out4 = {blocks pinned anew, their bytes,
 * nanoseconds spent pinning them (hipHostMalloc), requests served from the cache}. */
GANON_API int ganon_pinned_stats(int64_t *out4);
GANON_API int ganon_abi_version(void);
/* Use an external hipStream_t (e.g. torch's current stream); NULL = the ctx's own. */
GANON_API int ganon_ctx_set_stream(ganon_ctx *ctx, void *hip_stream);
/* Group kernel selection. Since ABI 3 the fused group kernel (one workgroup per group of
 * consecutive scopes copies its line-aligned pieces of the output and masks with byte stores) is
 * the only one: GANON_VARIANT_DEFAULT and GANON_VARIANT_GROUP_FUSED both select it; any other value
 * (the round-1 A/B kernels 1-4 and 6 were retired) is rejected with GANON_E_ARG. */
enum {
  GANON_VARIANT_DEFAULT = 0,
  GANON_VARIANT_GROUP_FUSED = 5
};
GANON_API int ganon_ctx_set_variant(ganon_ctx *ctx, int variant);
/* Tuning knobs (results never depend on them). GANON_PARAM_GROUP_UNROLL: 16-base chunks each
 * thread of the group kernels loads at once (chunk = 16 x value bases): 1, 2, 4 or 8; 0 (default)
 * = 1 in long-read prep mode, else 2.
 * GANON_PARAM_GROUP_SKIP is for phase timing only and DOES change results: bit 0 leaves out
 * the classification, bit 1 the chunk scan, bit 2 the partition copy of the group kernels, bit 3
 * the per-scope count stores.
 * Keep it 0 in production. GANON_PARAM_GROUP_TARGET: segments per scope group (read at
 * upload, in cost units: segments plus 3 per scope; 0 (default) = 1408 in long-read prep mode, else 704). GANON_PARAM_NT_COPY: non-temporal stores for the fused partition copy
 * (default 1). GANON_PARAM_REF2: group kernels read a 2-bit copy of the reference for segments
 * whose reference range is all ACGT (1, default) or the nt16 reference only (0).
 * GANON_PARAM_FASTQ_KD: FASTQ formatter kernel: 0 (default) = 16-byte units with per-span window
 *   setup, 3 per lane in one load round; 13 / 14 = the same, 2 per lane, one / two 8 KiB tiles per
 *   workgroup; 16 / 9 / 10 = 16-byte units with per-unit setup (the default up to round 4), 2 / 1 / 3
 *   per lane; 11 = 16-byte units, 2 per lane, bases windows selected per output dword (A/B instance);
 *   12 = record rows; 1-6 or 8 = the dword kernel with that many output dwords per lane at once.
 * GANON_PARAM_FASTQ_SKIP (phase timing only, changes results): bit 0 leaves out the
 * formatter's source loads, bit 1 its stores; bits 3-6 stop after the descriptor scan / after the
 * dword map / leave out the interior pass / leave out the edge and constant bytes.
 * GANON_PARAM_INDEL_SORT: the indel tally keeps only observations at positions where two or more
 * reads have an I/D op and sorts them per scope (0, default: segmented, 32-bit position keys), or
 * sorts every observation in one global sort of 64-bit scope|position keys (1). Same records.
 * GANON_PARAM_PREP_LONG (read at upload): which device prep builds the segment records. -1 (default):
 * the long-read prep (groups cut on the prefix of aligned segments per scope, one wave per incidence
 * walking its CIGAR) when a read of the batch has more than one segment and reads are longer than
 * 1000 bases; the one-segment prep (one record per incidence at its own index) when no read has more
 * than one segment; else (short reads with indels) the two-pass per-group emit; 1: always the
 * long-read prep; 2: the one-segment prep when it applies; 0: the two-pass per-group emit. Same
 * results. */
enum { GANON_PARAM_GROUP_UNROLL = 1, GANON_PARAM_GROUP_SKIP = 2, GANON_PARAM_GROUP_TARGET = 3,
       GANON_PARAM_NT_COPY = 4, GANON_PARAM_REF2 = 5, GANON_PARAM_FASTQ_SKIP = 6, GANON_PARAM_FASTQ_KD = 7,
       GANON_PARAM_INDEL_SORT = 8, GANON_PARAM_PREP_LONG = 9, GANON_PARAM_GROUP_OBS = 10,
       GANON_PARAM_PREP_UNROLL = 11, GANON_PARAM_FAR_INIT = 12, GANON_PARAM_SPEC_PLAN = 13,
       GANON_PARAM_FUSED_FLAT = 14, GANON_PARAM_XREC_INIT = 15 };
/* GANON_PARAM_XREC_INIT: first capacity of a batch's extras list (the fused mode's records of reads
 * with 2-8 aligned segments; 0 = auto, n_reads / 8 but at least 65536). A plan that needs more grows
 * it to the count and scans again; a speculative run that needs more is gated (testing knob: 1
 * forces both paths). */
/* GANON_PARAM_FUSED_FLAT: 1 (default) a batch of short reads (no read of more than 8 aligned segments,
 * none of more than 48 CIGAR ops) builds no segment records in HBM — the plan's scan writes a 16-byte
 * descriptor per read (and the segments of reads with several: short reads with I/D/N ops, round 5)
 * and the partition candidates, and the group kernel makes each incidence's records in LDS; 0 the
 * record pass (the one-segment prep emit; the two-pass emit for reads of several segments). Same
 * results. */
/* GANON_PARAM_SPEC_PLAN: 1 (default) speculative replans (ganon_batch_replan), 0 every plan
 * synchronizes for the scan's result, 2 (testing knob) reloads speculate too — their caller must
 * not read the shape before the download. Same results. */
/* GANON_PARAM_FAR_INIT: first capacity of a batch's far-mask list (entries; 0 = auto, n_reads / 8 but
 * at least 65536). A run that needs more is run again by ganon_batch_download with the list grown
 * to the count it needed (testing knob: 1 forces that path). */
/* GANON_PARAM_PREP_UNROLL: incidences each thread of the one-segment prep emit takes per trip (1, 2,
 * 4; 0 = default). */
/* GANON_PARAM_GROUP_OBS: observations a group keeps in LDS before its list overflows into the global
 * region: 512 (0, default) or 1024 (fewer resident workgroups; slower on every measured config). */
GANON_API int ganon_ctx_set_param(ganon_ctx *ctx, int param, int value);
/* When on, ganon_batch_run records a HIP event pair around each kernel it launches. */
GANON_API int ganon_ctx_set_profiling(ganon_ctx *ctx, int enabled);

/* One-shot: upload, run, download, free (synchronous). seq_out has seq_bytes bytes;
 * scope_calls_out / scope_bases_out ([n_scopes] each) and totals_out ([GANON_N_TOTALS])
 * may be NULL. */
GANON_API int ganon_mask_batch(ganon_ctx *ctx, const ganon_batch *batch, uint8_t *seq_out_nt16,
                               int32_t *scope_calls_out, int32_t *scope_bases_out,
                               int64_t *totals_out);

/* Resident reference: the genome (upper-cased nt16, 2 per byte, contigs concatenated) copied
 * to HBM once, with a 2-bit copy and a non-ACGT block map built on the device. Batches uploaded
 * with ganon_batch_upload_ref read it in place (their ref_nt16 / ref_bytes are ignored; scope_ref_off
 * indexes this reference). It must outlive those batches. */
GANON_API int ganon_ref_upload(ganon_ctx *ctx, const uint8_t *ref_nt16, int64_t ref_bytes, ganon_ref **out);
GANON_API int ganon_ref_free(ganon_ctx *ctx, ganon_ref *ref);

/* Device-resident path (streaming, benchmarks, multi-GPU shards). Upload copies only the raw
 * ganon_batch arrays to HBM and plans them on the device: one scan validates every read and scope
 * and sizes the derived layer (one synchronization). Every ganon_batch_run rebuilds the derived
 * layer (per-incidence CIGAR walk into aligned segments, output partitions) from those raw arrays
 * on the device, then masks. The incidence checks (read index, read inside its scope's span) and
 * the write-scope check run inside the run; their errors (GANON_E_ARG) are returned by
 * ganon_batch_download. ganon_batch_upload uploads the batch's own reference;
 * ganon_batch_upload_ref uses a resident one. ganon_batch_reload replaces the contents of an
 * uploaded batch with another host batch, reusing its device buffers (grow-only) and its
 * reference (resident, or the new batch's own) — the double-buffered streaming path.
 * ganon_batch_replan plans the batch's device arrays again from scratch, exactly as a fresh upload
 * of the same contents would (for arrays another stream or kernel wrote in place, and for timing
 * what a fresh batch costs: replan + run). Since ABI 4. A replan is speculative (no
 * synchronization: the scan and the run are enqueued back to back) when the batch's previous plan
 * found every read with at most one aligned segment (at most 8 short-read segments in the fused
 * mode, GANON_PARAM_FUSED_FLAT: short reads with I/D/N ops) and no scope wider than 2^20 positions, for
 * the same read / scope / incidence counts, or — a batch of other counts — when the context's last
 * full plan found that shape (the new batch is assumed to have it: its buffers are sized on the host
 * from its counts, the overflow regions for reads no longer than that plan's) (GANON_PARAM_SPEC_PLAN
 * 0 turns this off): the scan's reduction checks that the new contents fit that plan and gates the
 * run's kernels; a batch that
 * does not fit (or fails validation) runs nothing, and ganon_batch_download then plans it in full
 * and runs it again (or returns the validation error) — the results are those of a full plan
 * either way. After a speculative replan, ganon_batch_info / ganon_batch_shape report the previous
 * full plan until the next download. */
GANON_API int ganon_batch_upload(ganon_ctx *ctx, const ganon_batch *batch, ganon_dbatch **out);
GANON_API int ganon_batch_upload_ref(ganon_ctx *ctx, const ganon_batch *batch, const ganon_ref *ref,
                                     ganon_dbatch **out);
GANON_API int ganon_batch_reload(ganon_ctx *ctx, ganon_dbatch *db, const ganon_batch *batch);
GANON_API int ganon_batch_replan(ganon_ctx *ctx, ganon_dbatch *db);
GANON_API int ganon_batch_run(ganon_ctx *ctx, ganon_dbatch *db);      /* async on the stream */
GANON_API int ganon_batch_sync(ganon_ctx *ctx);
GANON_API int ganon_batch_download(ganon_ctx *ctx, ganon_dbatch *db, uint8_t *seq_out_nt16,
                                   int32_t *scope_calls_out, int32_t *scope_bases_out,
                                   int64_t *totals_out);
GANON_API int ganon_batch_free(ganon_ctx *ctx, ganon_dbatch *db);
/* Device pointer of the device-side totals ([GANON_N_TOTALS] int64), valid after run. */
GANON_API int ganon_batch_device_totals(ganon_dbatch *db, void **dev_ptr);
/* Enqueue a device-to-device copy of the totals into dev_dst (e.g. an RCCL buffer). */
GANON_API int ganon_batch_copy_totals(ganon_ctx *ctx, ganon_dbatch *db, void *dev_dst);

/* Kernel timing of the last profiled run: up to max_k entries of
 * (name, launches, total milliseconds). Returns the number of distinct kernels. */
typedef struct ganon_kernel_time {
  char name[48];
  int32_t launches;
  float ms;
} ganon_kernel_time;
GANON_API int ganon_last_kernel_times(ganon_ctx *ctx, ganon_kernel_time *out, int max_k);

/* Plan of an uploaded batch: [scope groups, segment records, huge scopes (> 2^20 positions, tile
 * path), huge-scope tiles, far-mask capacity (nibbles), reads written by huge scopes, overflow-region
 * entries, written reads]. */
GANON_API int ganon_batch_info(ganon_dbatch *db, int64_t *info8);
/* Shape of the planned batch, from the device scan: [I/D CIGAR ops (0: the indel tally has nothing
 * to do), longest read, most aligned segments of one read, prep mode (0 two-pass, 1 long-read,
 * 2 one-segment, 3 one-segment fused: GANON_PARAM_FUSED_FLAT, 4 the same with reads of 2-8 aligned
 * segments, the fused mode's multi-segment records (a full plan; a speculative one reports 3))].
 * Since ABI 4. */
GANON_API int ganon_batch_shape(ganon_dbatch *db, int64_t *shape4);
/* How often the group kernel took its rarer paths since upload (synchronous): [lists of more than
 * 256 observations classified after an LDS sort, lists of more than 512 (overflowing into the
 * group's global region), key-range splits of an overflowing region, overflowing lists the Bloom
 * filter brought back into LDS (no region pass)]. */
GANON_API int ganon_batch_path_counts(ganon_ctx *ctx, ganon_dbatch *db, int64_t *out4);
/* Runs since upload whose speculative plan the batch did not fit (their kernels ran nothing; the
 * next ganon_batch_download planned and ran the batch in full). Synchronous. Since ABI 4. */
GANON_API int ganon_batch_gated_runs(ganon_ctx *ctx, ganon_dbatch *db, int64_t *out);

/* ---- FASTQ record formatter ------------------------------------------
 * Replaces, for many reads at once, AnonymizedRead.get_anonymized_fastq_record
 * (anonymizer_methods.py:215-243, with reverse_complement :205-213) and write_pair's record
 * framing (short_read_tumor_normal_anonymizer.py:134-165). Record i is
 *   '@' name '/' ('0' + mate) '\n' SEQ '\n' '+' '\n' QUAL '\n'
 * SEQ: seq_len[i] nt16 nibbles from nibble seq_nib_off[i] of sequence buffer seq_sel[i], printed
 *      as "=ACMGRSVTWYHKDBN"; when reverse[i], reverse-complemented with the reference's table
 *      {A<->T, C<->G, N->N} — any other code is the reference's KeyError.
 * QUAL: qual_len[i] bytes from qual_off[i] of quality buffer qual_sel[i], each + 33, in stored
 *      order (qual_rev[i] == 0; the reference's output for every read) or reversed.
 * Byte-identical to the host formatter ganon_fastq_format (include/ganon_host.h). */
#define GANON_FASTQ_MAX_BUFS 4
#define GANON_FASTQ_FAILED (INT64_MIN + 1)   /* device/argument failure, see ganon_last_error */
typedef struct ganon_fastq ganon_fastq;   /* device-resident record batch */
typedef struct ganon_fastq_records {
  int64_t n;
  int32_t n_seq_bufs, n_qual_bufs;           /* 1..GANON_FASTQ_MAX_BUFS each */
  const uint8_t *const *seq_buf;             /* host nt16 buffers (ignored with seq_batch) */
  const ganon_dbatch *seq_batch;             /* or: buffer 0 = the batch's masked output,
                                                buffer 1 = its input, no copy */
  const uint8_t *seq_sel;
  const int64_t *seq_nib_off;
  const int32_t *seq_len;
  const uint8_t *reverse;
  const uint8_t *const *qual_buf;            /* host raw phred buffers */
  const uint8_t *qual_sel;
  const int64_t *qual_off;
  const int32_t *qual_len;
  const uint8_t *qual_rev;
  const char *names;                         /* host name blob */
  const int64_t *name_off;
  const int32_t *name_len;                   /* <= 65535 */
  const uint8_t *mate;
} ganon_fastq_records;
/* Upload the records (and the used slices of the host buffers); synchronous. */
GANON_API int ganon_fastq_upload(ganon_ctx *ctx, const ganon_fastq_records *records, ganon_fastq **out);
/* Format on the device (async on the stream): offsets scan + one workgroup per 16 KiB tile. */
GANON_API int ganon_fastq_run(ganon_ctx *ctx, ganon_fastq *f);
/* Output size in bytes (sum of 8 + name + seq + qual lengths). */
GANON_API int64_t ganon_fastq_bytes(const ganon_fastq *f);
/* Device pointer of the formatted bytes (valid after run). */
GANON_API int ganon_fastq_device_output(const ganon_fastq *f, void **dev_ptr);
/* Synchronize and copy the output: returns the byte count, -(i+1) for the first bad record i
 * (Q7), INT64_MIN when cap is too small, GANON_FASTQ_FAILED on other errors. */
GANON_API int64_t ganon_fastq_download(ganon_ctx *ctx, ganon_fastq *f, char *out, int64_t cap);
GANON_API int ganon_fastq_free(ganon_ctx *ctx, ganon_fastq *f);
/* One-shot with exactly the arguments of the host formatter ganon_fastq_format
 * (include/ganon_host.h): upload, run, download, free. Same return convention as
 * ganon_fastq_download. */
GANON_API int64_t ganon_fastq_format_hip(ganon_ctx *ctx, int64_t n, const uint8_t *const *seq_buf,
                                         const uint8_t *seq_sel, const int64_t *seq_nib_off,
                                         const int32_t *seq_len, const uint8_t *reverse,
                                         const uint8_t *const *qual_buf, const uint8_t *qual_sel,
                                         const int64_t *qual_off, const int32_t *qual_len,
                                         const uint8_t *qual_rev, const char *names,
                                         const int64_t *name_off, const int32_t *name_len,
                                         const uint8_t *mate, char *out, int64_t cap);

/* ---- Germline indel tally ----------------------------------------------
 * Replaces, for every scope of an uploaded batch at once, process_indels
 * (variation_classifier.py:52-141: every I/D CIGAR op of every scope read is a call keyed by
 * (pos, type, length, allele) with the reference's read-offset arithmetic), the
 * tumor/normal state machine (variants.py:33-39) and the indel half of mask_germline_variants
 * (anonymizer_methods.py:537-556 -> add_left_over_variant :245-252): a call seen in >=1 tumor and
 * >=1 normal read of the scope, at a position some normal read of the scope covers (a normal
 * pileup column exists there), is a masked TN indel call. The variable-length edits themselves
 * (mask_or_modify_indel, anonymizer_methods.py:178-203) are applied by the host when the record
 * is formatted, as the reference applies left-overs when a pair is yielded.
 *   pos          = ref_start + sum of M/D/N/=/X lengths before the op
 *   in_read_pos  = sum of M/N/=/X/S/H/I lengths before the op (the reference's counter adds S/H/I
 *                  and subtracts D from a sum that includes D and N)
 *   allele       = read bases [in_read_pos, in_read_pos + (INS ? length : 2)) clipped to the read
 * Registration order (which call at a position came first, needed for the order of a read's
 * left-overs) assumes each scope's incidences list its tumor reads in file order, then its normal
 * reads in file order (the reference meets reads column by column, tumor before normal).
 * Output: one record per masked TN call (kind GANON_INDEL_CALL: read/in_read_pos = its first
 * registered support, for the host's kept-variant check) and one per support by a read whose
 * write_scope is that scope (kind GANON_INDEL_SUPPORT; a read supporting a call twice keeps its
 * last offset, like the reference's supporting_reads dict). Records are in device order; a call
 * is identified by (scope, pos, rank), rank = its registration order among the calls at pos. */
enum { GANON_INDEL_DEL = 2, GANON_INDEL_INS = 3 };          /* VariantType values */
enum { GANON_INDEL_CALL = 0, GANON_INDEL_SUPPORT = 1 };
typedef struct ganon_indel_rec {
  int32_t scope;        /* batch scope                                   */
  int32_t pos;          /* contig position of the call                   */
  int32_t length;       /* CIGAR op length                               */
  int32_t type;         /* GANON_INDEL_DEL / GANON_INDEL_INS             */
  int32_t rank;         /* registration order among the calls at pos     */
  int32_t kind;         /* GANON_INDEL_CALL / GANON_INDEL_SUPPORT        */
  int32_t read;         /* batch read                                    */
  int32_t in_read_pos;  /* offset of the op in the read (see above)      */
} ganon_indel_rec;
typedef struct ganon_indels ganon_indels;
/* Plan the tally of an uploaded batch: b must be the host batch db was uploaded from (CIGARs are
 * scanned on the host to size the observation buffers). db must outlive the handle. */
GANON_API int ganon_indel_upload(ganon_ctx *ctx, const ganon_batch *b, const ganon_dbatch *db,
                                 ganon_indels **out);
/* Observation emission, sort and classification on the device (async on the stream). */
GANON_API int ganon_indel_run(ganon_ctx *ctx, ganon_indels *t);
/* Synchronize and copy the records: returns their count; copies only when out != NULL and
 * cap >= count (call again with a larger buffer otherwise); negative GANON_E* on failure. */
GANON_API int64_t ganon_indel_download(ganon_ctx *ctx, ganon_indels *t, ganon_indel_rec *out, int64_t cap);
/* [observations, incidences with an I/D op, sort key bits, records (after download, else -1),
 *  observations emitted by the last run (after download, else -1: the candidate filter keeps only
 *  positions where two or more reads have an I/D op), reads with an I/D op, sort strategy, 0] */
GANON_API int ganon_indel_info(const ganon_indels *t, int64_t *info8);
GANON_API int ganon_indel_free(ganon_ctx *ctx, ganon_indels *t);

/* ---- BGZF inflate (input decode offload) ---------------------------------
 * Replaces the zlib inflate behind AlignmentFile.fetch / pileup (pileup_io.pyx:12-17 via htslib's
 * bgzf_read): n_blocks raw DEFLATE payloads (RFC 1951; BGZF blocks, at most 64 KiB in and out each)
 * at comp[in_off[i], + in_len[i]) inflate to out[out_off[i], + out_len[i]) (out_len = the block's
 * ISIZE). Host buffers in and out (synchronous: H2D, one workgroup per block, D2H); the device
 * buffers are kept by the context. GANON_E_ARG with *first_bad = the block when a stream is invalid
 * or does not inflate to its ISIZE. ganon_inflate_hostcb has the host BAM reader's inflater
 * signature (include/ganon_host.h ganon_bam_reader_set_inflater, user = the context). Since ABI 4. */
GANON_API int ganon_inflate(ganon_ctx *ctx, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                            const int32_t *in_len, const int64_t *out_off, const int32_t *out_len,
                            int64_t n_blocks, uint8_t *out, int64_t out_total, int64_t *first_bad);
GANON_API int ganon_inflate_hostcb(void *ctx, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                                   const int32_t *in_len, const int64_t *out_off, const int32_t *out_len,
                                   int64_t n_blocks, uint8_t *out, int64_t out_total);

/* The device copy of the last successful ganon_inflate's output on this context (out_total bytes,
 * block i at out_off[i]): valid until the context's next ganon_inflate. Lets the record walk below
 * run on the inflated stream where it already lies. */
GANON_API int ganon_inflate_device_output(ganon_ctx *ctx, const uint8_t **out, int64_t *bytes);

/* ---- BAM records -> columns on the device (the record walk after the inflate) ----
 * Replaces, for a stream the device holds, libganon_host.so's record walk (records_to_columns in
 * csrc/ganon_host.cpp, the ganon_bam_view of include/ganon_host.h) — what the reference gets from
 * htslib's bam_read1 behind AlignmentFile.fetch / pileup (pileup_io.pyx:12-17). The records lie back
 * to back at stream[p, n) (p: the first record, after the BAM header); stream is a 4-byte aligned
 * device pointer, or a host pointer with on_host = 1 (copied to the device first). The columns are those of
 * ganon_bam_view, same values and blob layout (record order = stream order; name blob with one NUL
 * per name; bam_endpos in `end`), plus rec_off = each record's offset in the stream; they stay in
 * device memory, owned by the handle. Errors as the host decoder's: GANON_E_ARG on a bad record size
 * or fields that exceed a record's block size. Since ABI 4 (round 5). */
typedef struct ganon_bam_cols {
  int64_t n_records;
  int32_t *tid, *pos, *end, *flag, *mapq, *l_seq, *n_cigar, *mate_tid, *mate_pos, *tlen, *name_len, *aux_len;
  int64_t *name_off, *cig_off, *seq_off, *qual_off, *aux_off, *rec_off;
  char *names;
  int64_t names_bytes;
  uint32_t *cigar;
  int64_t cigar_ops;
  uint8_t *seq;
  int64_t seq_bytes;
  uint8_t *qual;
  int64_t qual_bytes;
  uint8_t *aux;
  int64_t aux_bytes;
} ganon_bam_cols;
typedef struct ganon_bam_dcols ganon_bam_dcols;
GANON_API int ganon_bam_columns(ganon_ctx *ctx, const uint8_t *stream, int64_t p, int64_t n, int on_host,
                                ganon_bam_dcols **out);
/* The device pointers and sizes; *fixes = the stream chunks whose first record start was guessed wrong. */
GANON_API int ganon_bam_dcols_get(const ganon_bam_dcols *c, ganon_bam_cols *device_view, int64_t *fixes);
/* Copy the columns to host arrays sized from ganon_bam_dcols_get's counts (NULL members skipped). */
GANON_API int ganon_bam_dcols_download(ganon_ctx *ctx, const ganon_bam_dcols *c, const ganon_bam_cols *host);
/* (with the context that made it: its device blocks return to that context's cache) */
GANON_API int ganon_bam_dcols_free(ganon_ctx *ctx, ganon_bam_dcols *c);

/* A region read's window decoded on the device: the reader's region decoder (ganon_region_fn of
 * include/ganon_host.h, user = a ganon_ctx; libganon_host.so's ganon_bam_reader_region, the
 * reference's AlignmentFile.fetch(contig, beg, end), short_read_tumor_normal_anonymizer.py:570-573).
 * Inflates the window's BGZF blocks (as ganon_inflate) and keeps them in device memory; walks the
 * records from byte p0 (the window may end inside a record); the region ends at the first record of
 * another sequence or with pos >= end; records with bam_endpos > beg are kept. Returns 1 when the
 * region ends inside the window: *cols = the kept records' columns (ganon_bam_view's record fields
 * and blobs, same values and layout as the host decoder's) in one page-locked block *block, freed
 * with ganon_pinned_free. Returns 0 when the region goes on past the window, or the window holds
 * what the host decoder must report (a malformed record, an index that points before the
 * sequence): out[0, out_total) then holds the inflated window for the host's walk. -1: the inflate
 * failed. Since ABI 5 (round 6). */
struct ganon_bam_view;
GANON_API int ganon_region_decode(void *user, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                                  const int32_t *in_len, const int64_t *out_off, const int32_t *out_len,
                                  int64_t n_blocks, uint8_t *out, int64_t out_total, int64_t p0, int32_t tid,
                                  int64_t beg, int64_t end, int at_eof, struct ganon_bam_view *cols, void **block);

#endif /* GANON_H */
