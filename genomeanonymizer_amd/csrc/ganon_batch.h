// ganon_batch.h — internal to libganon_hip.so: the device batch (ganon_dbatch), the resident
// reference (ganon_ref), the layouts the device prep kernels (ganon_prep.hip) write and the
// masking kernels (ganon_hip.hip) read. Not part of the C ABI (include/ganon.h is).
//
// A batch lives in HBM in two layers:
//   raw      the ganon_batch SoA exactly as the host hands it over (BAM nt16 bases, BAM CIGAR
//            words, per-read/per-scope metadata, the scope->read incidence CSR) — the only
//            bytes that cross PCIe;
//   derived  everything the masking kernels need beyond that — per-read segment counts and
//            read ends, scope groups, 16-byte segment records (one per aligned M/=/X run of a
//            read in a scope), output partition pieces, overflow regions — rebuilt from the raw
//            layer by the prep kernels on every ganon_batch_run.
#ifndef GANON_BATCH_H
#define GANON_BATCH_H

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/ganon.h"
#include "ganon_ctx.h"

namespace ganon_dev {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kTile = 16384;           // positions per tile of a huge scope (tile path)

// ---- group kernels (ganon_hip.hip k_group) -----------------------------------------------
constexpr int kGrpRec = 5;             // int4 records per group (layout below)
constexpr int kGrpObs = 512;           // observations per LDS list
constexpr int kGrpMaxScopes = 256;     // scopes per group (8-bit LDS counters index, 12-bit field)
constexpr int kGrpMaxSpan = 1 << 20;   // widest scope of the group kernels (20-bit position field)
constexpr int64_t kPartAlign = 128;    // partition boundaries fall on whole lines
constexpr int kSegMaxLen = (1 << 14) - 1;   // longer aligned runs are cut into pieces
constexpr uint32_t kSegMine = 1u << 31;     // the segment's read is written by this scope
// segment record (int4, 16 bytes): x = query nibble bits 0-31, y = reference nibble bits 0-31,
// z = query nibble bits 32-39 | reference nibble bits 32-39 << 8 | length << 16 (14 bits) |
// dataset << 30 | mine << 31, w = scope_local | (pos - span_start) << 12.
// group record (kGrpRec x int4), one per group in launch order:
//   [0] {s_begin, s_end, seg_begin lo, hi}      [1] {seg_end lo, hi, seg_mid lo, hi}
//   [2] {piece A begin lo, hi, end lo, hi}       [3] {overflow region lo, hi, capacity, 0}
//   [4] {piece B begin lo, hi, end lo, hi}
// segments [seg_begin, seg_mid) have an all-ACGT reference range (2-bit reference).
// read descriptor (int4, 16 bytes; k_prep_scan writes one per read of at most kScanLongCigar CIGAR
// ops that passed its checks): everything the fused one-segment group kernel gathers per incidence.
//   x = query nibble of the read's first aligned segment, bits 0-31 (2 seq_off + q),
//   y = its contig position p (ref_start when the read has no segment),
//   z = query nibble bits 32-39 | length << 8 (14 bits; 0: no segment) | dataset << 22 | wide << 23 |
//       (p - ref_start) << 24 (4 bits) | (read_end - p - length) << 28 (4 bits),
//   w = write scope.
// wide: one of the two deltas did not fit (the span check then reads ref_start and read_end).
// A read of 2..kFusedMaxSeg aligned segments (a short read with an I/D/N op, round 5) is described the
// same way by its FIRST segment, with kDescMulti (bit 7: query nibbles are below 2^39, so bit 7 of the
// high byte is free) and its further segment count in bits 28-30 instead of the end delta (its span
// end is checked when its further segments are expanded). Its further segments are in the extras
// list (k_prep_scan) at xidx[read]: a header {ref_start, read_end, 0, 0}, then one record per further
// segment (int4: x = query nibble bits 0-31, y = contig position, z = query nibble bits 32-38 |
// length << 8, w = 0). Round 5's first layout pointed the descriptor at the extras list, and every
// tile waited for one more dependent load round (c2id k_group 0.56 vs c2 0.49 ms).
constexpr uint32_t kDescWide = 1u << 23;
constexpr uint32_t kDescMulti = 1u << 7;
constexpr int kFusedMaxSeg = 8;   // most aligned segments of a read the fused one-segment mode takes
// long-read mode: read record (int4; k_prep_read_recs, at b_rbase[read] + k for the read's k-th
// aligned-segment piece, in CIGAR order): x = query nibble bits 0-31, y = contig position,
// z = query nibble bits 32-39 | length << 16 (14 bits) | dataset << 30, w = 0 — a segment record
// without its scope's fields. incidence record (int4; k_prep_long_groups): x = the incidence's
// first slot in its group's slot space (its read's records follow), y = scope local | mine << 31,
// z / w = b_rbase of its read (lo, hi). (The reference copy is chosen per tile from the scopes'
// flags: a per-segment flag moved nothing on C5, profiles/r04/c5_ab.) The group kernel's slot t of a group: the incidence with the
// largest first slot <= t, its read record t - x. Long-read group records: [0] seg_begin = 0,
// [1] seg_end = the group's slot count, seg_mid = its first incidence; [3].w = its incidence count.

// Device view of a batch (all pointers device-resident).
struct DevBatch {
  const int32_t *ref_start, *read_len, *read_end, *n_cig, *write_scope;
  const int64_t *seq_off, *cig_off;
  const uint8_t *seq, *dataset;
  const uint32_t *cigar;
  const int64_t *incid_off;
  const int32_t *incid_read;
  const int32_t *span_start, *span_len, *keep_pos;
  const int64_t *ref_off;
  const uint8_t *ref, *keep_code;
  const uint32_t *ref2;   // 2-bit reference (k_ref2), null = nt16 only
};

struct Tile {
  int32_t scope;
  int32_t a;      // tile covers [a, b) (contig positions)
  int32_t b;
  int32_t pad;
  int64_t lo;     // candidate range in large_incid
  int64_t hi;
};

// First error the device validation found: per-read and per-scope checks at plan time, incidence
// and write-scope checks during the run (reported by ganon_batch_download).
struct PrepErr {
  int code;         // 0 none, else a PrepErrKind
  int pad;
  long long index;  // read / scope / incidence
  long long a, b;
};

// Rarely used outputs and scratch of the group kernels, read through one pointer (device
// memory) so that their addresses do not occupy scalar registers for the whole kernel.
struct GrpAux {
  int32_t *scope_calls, *scope_bases, *part;   // per-scope counts; per-workgroup partial totals
  unsigned long long *far;                      // masks of bytes outside the masking group's pieces
  unsigned long long *far_count;                // 64-bit: a whole sample may be one batch
  int64_t far_cap;
  unsigned long long *paths;                    // [0] sorted lists, [1] region passes, [2] key-range splits
  unsigned long long *okey, *opay, *tkey;       // overflow regions
  unsigned int *tflag;
  // fused one-segment mode: the group kernel makes its segment records from the incidences and the
  // read descriptors itself (incidence checks, write-scope hash sums per group)
  const int32_t *incid_read, *ref_start, *read_end;
  const int4 *desc;
  const int64_t *incid_off, *ref_off;
  const uint8_t *sdirty;                        // per scope: its reference span holds a non-ACGT block
  const int4 *inc4, *rrec;                      // long-read mode: incidence and read records
  // fused mode, multi-segment reads: the extras records (k_prep_scan) and, per group, the entries of
  // its incidences with further segments (k_group's first pass, at the group's first incidence:
  // x = the read's extras index, y = scope local | further segments << 12 | dataset << 15 | mine << 31)
  const int4 *xrec;
  const int32_t *xidx;                          // per multi-segment read: its extras header's index
  int2 *xlist;
  int32_t n_reads, pad_;
  PrepErr *err;
  unsigned long long *ws_part;
};
enum PrepErrKind {
  kErrReadSeq = 1, kErrReadCigar, kErrReadDataset, kErrReadWriteScope, kErrReadLong, kErrCigarOp, kErrReadPos,
  kErrScopeOff, kErrScopeSpan, kErrScopeRef, kErrScopeKeep, kErrIncidRead, kErrIncidSpan, kErrWriteScopeMissing
};

// ---- device helpers shared by the prep kernels (ganon_prep.hip) and the group kernels
#ifdef __HIPCC__
__device__ __forceinline__ void report(PrepErr *err, int kind, long long index, long long a = 0, long long b = 0) {
  if (atomicCAS(&err->code, 0, kind) == 0) {
    err->index = index;
    err->a = a;
    err->b = b;
  }
}

__device__ __forceinline__ bool is_aligned_op(int op) { return op == 0 || op == 7 || op == 8; }

// Aligned runs of a read (M/=/X ops, cut at kSegMaxLen, clipped to the read length): f(q, p, n)
// with query offset q, contig position p, length n — the host planner's segments_of, round 1.
template <typename F>
__device__ __forceinline__ void walk_segments(const uint32_t *__restrict__ cig, int nc, int L, int ref_start, uint32_t w0,
                                              F &&f) {
  int q = 0, p = ref_start;
  for (int k = 0; k < nc && q < L; ++k) {
    const uint32_t w = k == 0 ? w0 : cig[k];   // (the first word is loaded early by the caller)
    const int op = (int)(w & 0xF);
    const int len = (int)(w >> 4);
    if (is_aligned_op(op)) {
      const int n = min(len, L - q);
      for (int o = 0; o < n; o += kSegMaxLen) f(q + o, p + o, min(kSegMaxLen, n - o));
      q += len;
      p += len;
    } else if (op == 1 || op == 4) {
      q += len;
    } else if (op == 2 || op == 3) {
      p += len;
    }
  }
}

// Is the reference range [rnib, rnib + n) free of non-ACGT codes (every 64-base block clean)?
__device__ __forceinline__ bool ref_clean(const uint64_t *__restrict__ bad, int64_t n_blk, int64_t rnib, int n) {
  const int64_t k0 = rnib >> 6, k1 = (rnib + n - 1) >> 6;
  if (k1 >= n_blk) return false;
  for (int64_t wd = k0 >> 6; wd <= (k1 >> 6); ++wd) {
    const int lo = wd == (k0 >> 6) ? (int)(k0 & 63) : 0;
    const int hi = wd == (k1 >> 6) ? (int)(k1 & 63) : 63;
    const uint64_t mask = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & ~((1ull << lo) - 1);
    if (bad[wd] & mask) return false;
  }
  return true;
}


__device__ __forceinline__ unsigned long long ws_hash(int r) {
  unsigned long long z = (unsigned long long)(uint32_t)r + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

#endif

// Grow-only device buffer (+128 bytes of padding: the group kernels load up to 68 bytes past a
// chunk start, the patch atomics touch whole dwords).
struct DBuf {
  void *p = nullptr;
  size_t bytes = 0;
};

}  // namespace ganon_dev

// Resident reference: uploaded once, shared by every batch of a context (a whole genome).
struct ganon_ref {
  uint8_t *nt16 = nullptr;     // upper-cased reference, nt16, 2 per byte (+ padding)
  uint32_t *ref2 = nullptr;    // 2-bit copy (A0 C1 G2 T3), 16 bases per word
  uint64_t *bad = nullptr;     // bit k: 64-base block k holds a non-ACGT code (N, IUPAC, '=')
  int64_t bytes = 0, n_blk = 0;
  bool owned_by_batch = false;
};

struct ganon_dbatch {
  ganon_dev::DevBatch B{};
  // sizes of the current contents
  int32_t n_reads = 0, n_scopes = 0;
  int64_t n_incid = 0, seq_bytes = 0, n_cigar_ops = 0;
  const ganon_ref *ref = nullptr;
  ganon_ref *own_ref = nullptr;          // a batch uploaded without a resident reference
  // raw layer (grow-only)
  ganon_dev::DBuf b_ref_start, b_read_len, b_seq_off, b_cig_off, b_n_cig, b_dataset, b_write_scope, b_seq, b_cigar,
      b_incid_off, b_incid_read, b_span_start, b_span_len, b_ref_off, b_keep_pos, b_keep_code;
  // derived layer
  ganon_dev::DBuf b_part;                                          // k_prep_scan per-block partials
  ganon_dev::DBuf b_long;                                          // k_prep_scan's list of long-CIGAR reads
  ganon_dev::DBuf b_nseg, b_scost, b_scan_tmp, b_slots, b_slot0;   // segments per read; long-read mode: group
                                                                  // costs, dirty flags, first slot per incidence
  ganon_dev::DBuf b_wspart;                                        // per-group write-scope hash sums
  ganon_dev::DBuf b_order;                                         // group launch order (k_prep_order_*), then per-block class counts
  int64_t max_scope_incid = 0;                                     // most incidences of one scope (host, at load)
  bool ordered = false;                                            // the run launches groups in b_order's order
  ganon_dev::DBuf b_read_end, b_cursor, b_gs0, b_lo, b_linemap, b_groups, b_seg4, b_grp_part, b_far, b_gokey, b_gopay, b_gtkey, b_gtflag, b_out,
      b_scope_calls, b_scope_bases, b_small;   // b_small: totals, static totals, counters, acc, status, errors
  uint8_t *out = nullptr;
  int32_t *scope_calls = nullptr, *scope_bases = nullptr;
  unsigned long long *totals = nullptr, *static_totals = nullptr, *acc = nullptr, *far_count = nullptr;
  int32_t *counters = nullptr;          // [0] rare small (unused), [1] rare tiles
  int32_t *status = nullptr;            // device status bits of the run (1: far-mask list overflow, 2: write-scope
                                        // sums, 4: gated by the plan); cleared with the other flags per plan
  unsigned int *long_count = nullptr;   // reads the scan left to k_prep_scan_long
  unsigned long long *far_need = nullptr;   // far masks a run needed (k_finish)
  size_t flags_bytes = 0;               // err .. far_need: one memset per plan
  ganon_dev::PrepErr *err = nullptr;
  unsigned long long *plan_info = nullptr;   // [0] I/D ops, [1] huge scopes, [2] written reads, [3] longest read,
                                             // [4] most segments of one read, [5] short-read groups,
                                             // [6] write-scope hash sum (k_finish compares)
  unsigned long long *paths = nullptr;       // GrpAux::paths (since upload)
  unsigned long long *gated = nullptr;       // runs stopped by a speculative plan's gate (since upload)
  unsigned long long *cursor = nullptr;      // k_prep_emit allocation counters and their bases (b_cursor)
  ganon_dev::GrpAux *aux = nullptr;
  // plan of the current contents (device prep, sized at upload)
  int32_t n_groups = 0, group_target = 512;
  // speculative replan (GANON_PARAM_SPEC_PLAN): the last full plan was one-segment mode without huge
  // scopes for these sizes, so a replan of the same sizes launches its run without waiting for the
  // scan; the device checks the assumption (plan_info[7]) and ganon_batch_download plans and runs
  // again when it failed
  bool spec = false, spec_ready = false;
  bool spec_sized = false;   // the speculation sized this plan's buffers for new counts (ctx->spec_*)
  int64_t spec_sizes[4] = {-1, -1, -1, -1};   // reads, scopes, incidences, group target of that plan
  // long-read mode (a read with more than one aligned segment): groups cut on the prefix of segments
  // per scope (scost, upload) instead of the CSR offsets, and emitted one wave per incidence
  bool long_mode = false;
  bool flat_mode = false;   // every read has at most one aligned segment: one record per incidence, in place
  // fused one-segment mode (GANON_PARAM_FUSED_FLAT, default on): no record pass — the scan writes a
  // descriptor per read (b_desc) and the partition candidates (b_cand: per group and dataset, the
  // complement of the lowest buffer offset written, atomicMax), the group kernel makes each
  // incidence's record in LDS. Off for batches with long-CIGAR reads (the scan does not describe them).
  bool fused = false;
  ganon_dev::DBuf b_desc, b_cand, b_sdirty;
  // ... and reads of several aligned segments (at most kFusedMaxSeg): their segments as extras records
  // (b_xrec, allocated by the scan with a counter, capacity xcap records: a plan that needs more grows
  // it and scans again, a speculative one is gated), the group kernel's per-group entries (b_xlist)
  ganon_dev::DBuf b_xrec, b_xlist, b_xcnt, b_xidx;
  int64_t xcap = 0;
  unsigned int *xcount = nullptr;       // the scan's allocation counters (b_xcnt: one stripe of xcap / 64
                                        // records per counter, one 128-byte line each; cleared per plan)
  // long-read mode: segment records once per read (b_rrec at b_rbase[read]) and per incidence its
  // first slot in its group, scope and write mark (b_inc4); the group kernel reads the read's
  // records for every scope that lists it
  ganon_dev::DBuf b_inc4, b_rbase, b_rrec;
  int64_t n_rrec = 0, n_long_seg = 0;
  unsigned long long *cand = nullptr;   // the scan's candidates of this plan (null: the emit marks them)
  int64_t *scost = nullptr;
  int64_t n_seg = 0, region = 0, far_cap = 0, n_written = 0, region_per_incid = 0, n_id_ops = 0;
  int64_t max_len = 0, max_seg = 0;         // longest read, most aligned segments of one read (plan)
  int64_t far_cap_alloc = 0;                 // capacity of b_far (kept across batches, grown on overflow)
  std::vector<unsigned long long> cursor_h;  // emit sub-counter bases (host copy of an async upload)
  ganon_dev::GrpAux aux_h{};                 // host copies of the async uploads of a plan
  unsigned long long static_h[GANON_N_TOTALS] = {0};
  // huge scopes (> kGrpMaxSpan positions): tile path, planned on the host at upload
  std::vector<void *> huge_allocs;
  ganon_dev::Tile *tiles_h = nullptr;
  int32_t *large_incid = nullptr, *large_written_h = nullptr, *large_ids = nullptr;
  int64_t *tab_off = nullptr;
  uint16_t *tn_tab = nullptr;
  int64_t tn_entries = 0;
  int32_t n_tiles_h = 0, n_large_written_h = 0, n_huge_scopes = 0;
  int32_t *rare_tile_list = nullptr;
  bool ran = false;
};

namespace ganon_prep {

// Validate the raw layer on the device and plan the derived layer (prep mode, group count, segment
// count, overflow regions) from it: one scan over the raw arrays and one synchronization (two more
// in the two-pass and long-read modes). Everything a freshly arrived raw batch needs before its
// first run (upload, reload, ganon_batch_replan).
int plan(ganon_ctx *ctx, ganon_dbatch *db, bool allow_spec);
// Rebuild every derived array from the raw layer (async on the stream): the first half of
// every ganon_batch_run.
int run(ganon_ctx *ctx, ganon_dbatch *db);
// The write-scope sums disagreed (k_finish status bit 2): find the read (async; then batch_error).
int ws_diag(ganon_ctx *ctx, ganon_dbatch *db);
// Synchronize and report the first error the device checks recorded (GANON_E_ARG) or GANON_OK.
int batch_error(ganon_ctx *ctx, ganon_dbatch *db);
// Grow-only allocation of count elements of T.
int grow(ganon_ctx *ctx, ganon_dev::DBuf &b, size_t bytes);
template <typename T>
inline int grow_n(ganon_ctx *ctx, ganon_dev::DBuf &b, size_t count, T **out) {
  int rc = grow(ctx, b, count * sizeof(T));
  *out = static_cast<T *>(b.p);
  return rc;
}

}  // namespace ganon_prep

// Non-ACGT block bitmap of a resident reference (ganon_prep.hip), async on the stream.
int ganon_ref_blocks(ganon_ctx *ctx, ganon_ref *ref);

#endif  // GANON_BATCH_H
