// ganon_indel.hip — germline indel tally on MI355X (gfx950); C ABI in
// include/ganon.h (ganon_indel_*), part of libganon_hip.so.
//
// Reference semantics, per scope (= one CompleteGermlineAnonymizer.anonymize call):
//   process_indels (variation_classifier.py:52-141) registers every I/D CIGAR op of every read
//   the scope's pileup meets, once per read (seen_read_alns, :208-215), as a call keyed by
//   (pos, end, type, length, allele) (CalledGenomicVariant.__eq__, variants.py:83-96; end is a
//   function of pos/type/length); the tumor/normal state machine (variants.py:33-39) makes it
//   TUMORAL_NORMAL once a tumor AND a normal read support it; at the normal pileup column `pos`
//   every TN call other than the kept window variant is counted and handed to each supporting
//   read as a left-over edit (anonymizer_methods.py:537-556, :245-252).
//
// Design: integer work, no MFMA. Observations are rare in short-read batches and
// dense in long-read ones (5 % indel errors: ~10^8 per C5 batch), so the tally is a sort rather
// than an LDS table:
//   candidates        (default) k_indel_mark sets a tumor / normal bit per genome position of every
//                     read's I/D ops; k_indel_rcount + k_indel_remit walk each read once (a wave per
//                     block of 256 CIGAR ops: lanes take 64 ops at a time, wave prefix sums give each
//                     op its reference position and read offset) and list its ops at positions
//                     with both bits (ballot-compacted, read-major);
//   k_indel_expand    one wave per (scope, read) incidence: its read's candidates as 16-byte
//                     observations with a 32-bit sort key (pos - span_start, plus the scope
//                     segment's parity in bit 31), scope-major (GANON_PARAM_INDEL_SORT 1:
//                     k_indel_emit walks every incidence and writes all its ops at the host's slots);
//   radix sort        rocPRIM segmented pairs (key, observation index), one segment per scope
//                     with observations, position bits only (GANON_PARAM_INDEL_SORT 1: one
//                     global sort of 64-bit scope|position keys instead);
//   k_indel_classify  the first thread of each (scope, pos) run resolves the run — singletons
//                     leave at once: exact allele comparison groups observations into calls,
//                     tumor+normal presence, normal coverage of pos (the scope's normal reads),
//                     registration rank among the calls at pos, the observations that become
//                     output records, one atomic add of the record count per run;
//   k_indel_write     (download) records at atomic slots; results do not depend on slot order
//                     (a call is (scope, pos, rank); the host sorts the records).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ganon.h"
#include "ganon_ctx.h"

using ganon_detail::check_launch;
using ganon_detail::fail;
using ganon_detail::KernelScope;

namespace {

// Work items are blocks of kWalkOps CIGAR ops (long-read CIGARs hold thousands of ops), each with
// the reference's running offsets at its first op computed on the host, so that every block is an
// independent wave.
constexpr int kWalkJ = 4;
constexpr int kWalkOps = 64 * kWalkJ;

struct IndelInc {       // one block of one incidence with an I/D op (host plan)
  int32_t read;
  uint32_t scope_par;   // scope | (index of the scope among scopes with observations & 1) << 31
  int32_t k0;           // first CIGAR op of the block
  int32_t pos0, irp0;   // reference position / in_read_pos at op k0
  int32_t pad;
  int64_t obs_off;      // slot of the block's first I/D op (unfiltered numbering = registration order)
  int64_t cbase;        // genome nibble index of the read's contig start (candidate map)
};

struct IndelRead {      // one block of one read with an I/D op (candidate marking, per-read candidates)
  int32_t read, k0, pos0, irp0;
  int32_t nid0, pad;    // I/D ops of the read before the block
  int64_t cbase;
};

struct IndelIncR {      // one (scope, read) incidence with an I/D op (the filtered path, per incidence)
  int32_t read;
  uint32_t scope_par;   // scope | segment parity << 31
  int32_t rfirst, rnb;  // the read's blocks in the read list (its candidates: rcand[roff[rfirst]..roff[rfirst + rnb]])
  int64_t obs_base;     // the incidence's first unfiltered slot (registration order)
};

struct IndelCand {      // one candidate I/D op of a read (scope-free part of an observation)
  int32_t pos, irp, type_len, ord;   // ord: the op's index among the read's I/D ops
};

struct IndelObs {       // one I/D op of one incidence
  int32_t read;
  int32_t irp;          // in_read_pos (reference arithmetic)
  int32_t scope;
  int32_t type_len;     // length << 1 | is_insertion
  uint32_t ord;         // unfiltered slot: incidence order, then op order (registration order)
};

// Candidate map: 2 bits per genome position (bit 0: a tumor read has an I/D op there, bit 1: a
// normal read has) — or, when the batch has far fewer I/D ops than the genome has positions (a
// short-read batch: ~3e5 ops on 3 Gb), 2 bits per cell of a hashed map of at least 64 cells per
// op (map_cell): cleared per run in microseconds instead of a 750 MB memset. A collision can only
// add a position (its observations are then emitted and classified, and it holds no TN call: one of
// its datasets had no op there); no position with both bits is ever lost. A TN call at (scope, pos) needs a tumor and a normal read with an op at pos, so
// a position missing either bit has no TN call in any scope; the other calls at such a position
// only matter as the rank of a TN call there (registration order among the calls at pos), and
// there is none. Its observations are not emitted (GANON_PARAM_INDEL_SORT 0); every observation
// at a position with both bits is, so the ranks are those of the full tally. (Round 3 kept every
// position two reads of any dataset shared: at C5's 5 % indel errors about twice as many.)


// Sort keys. Segmented (default): one segment per scope, 32-bit key = segment parity << 31 |
// (pos - span_start), sorted on the position bits only — the parity bit still tells adjacent
// scopes apart in the sorted array. Global (A/B): 64-bit key = scope << pos_bits | (pos - span_start).
template <typename KeyT>
__device__ __forceinline__ KeyT make_key(uint32_t scope_par, int pos_bits, uint32_t rel) {
  if constexpr (sizeof(KeyT) == 4) return (scope_par & 0x80000000u) | rel;
  else return ((unsigned long long)(scope_par & 0x7FFFFFFFu) << pos_bits) | rel;
}

// Map cell of genome nibble g: g itself (dense map, shift 0) or the top bits of a multiplicative
// hash (hashed map of 2^(64 - shift) cells).
__device__ __forceinline__ uint64_t map_cell(int64_t g, int shift) {
  return shift ? ((uint64_t)g * 0x9E3779B97F4A7C15ull) >> shift : (uint64_t)g;
}

constexpr int kIndelWaves = 4;
constexpr int kIndelThreads = 64 * kIndelWaves;

// Bounds-checked builds (tools/build_variant.py ichk -DGANON_INDEL_CHECK=1; verdict r05 item 2): every
// index a kernel of the tally dereferences is checked against its buffer's capacity first; a failing
// check records its source line in g_indel_chk (first one wins) and the thread leaves instead of
// touching memory, and ganon_indel_download reports the line. Default builds compile the checks away.
#ifndef GANON_INDEL_CHECK
#define GANON_INDEL_CHECK 0
#endif
// capacities the checks compare against: [0] observations, [1] read candidates, [2] records,
// [3] reads, [4] scopes, [5] incidence blocks (list), [6] filtered incidences (ilist), [7] read blocks
__device__ long long g_indel_cap[8];
__device__ unsigned int g_indel_chk[2];   // [0] first failing line, [1] failures
#if GANON_INDEL_CHECK
#define ICHK_RET(cond, ...)                                   \
  do {                                                        \
    if (!(cond)) {                                            \
      atomicCAS(&g_indel_chk[0], 0u, (unsigned int)__LINE__); \
      atomicAdd(&g_indel_chk[1], 1u);                         \
      return __VA_ARGS__;                                     \
    }                                                         \
  } while (0)
#else
#define ICHK_RET(cond, ...) \
  do {                      \
  } while (0)
#endif
#define ICHK(cond) ICHK_RET(cond)
#define IN_CAP(i, k) ((long long)(i) >= 0 && (long long)(i) < g_indel_cap[k])

__device__ __forceinline__ int nib(const uint8_t *__restrict__ seq, int64_t byte_off, int i) {
  const uint8_t b = seq[byte_off + (i >> 1)];
  return (i & 1) ? (b & 0xF) : (b >> 4);
}

__device__ __forceinline__ int wave_excl_scan(int v, int lane) {
  (void)lane;
  return ganon_wave::incl_sum(v) - v;
}

// The reference's offsets of a read's ops, 64 CIGAR ops per step of one wave: pos = reference
// start + M/D/N/=/X lengths before the op; irp = M/N/=/X/S/H/I lengths before it.
struct CigarStep {
  int op, len, pos, irp;
  bool is_id;
};

// One block: every lane loads kWalkJ CIGAR words before any is used, and the callback gets the
// kWalkJ steps of 64 ops together so that it can issue its own loads (the candidate map) for all of
// them at once.
template <typename F>
__device__ __forceinline__ void walk_block(const GanonReadView &V, int r, int k0, int pos0, int irp0, int lane, F &&f) {
  const int nc = min(V.n_cig[r], k0 + kWalkOps);
  const uint32_t *__restrict__ cig = V.cigar + V.cig_off[r];
  int rcarry = pos0, qcarry = irp0;
  uint32_t word[kWalkJ];
#pragma unroll
  for (int j = 0; j < kWalkJ; ++j) {
    const int k = k0 + 64 * j + lane;
    word[j] = k < nc ? cig[k] : 0u;
  }
  CigarStep c[kWalkJ];
#pragma unroll
  for (int j = 0; j < kWalkJ; ++j) {
    const int k = k0 + 64 * j + lane;
    c[j].op = (int)(word[j] & 0xF);
    c[j].len = (int)(word[j] >> 4);
    const int op = c[j].op, len = c[j].len;
    const int radv = (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) ? len : 0;
    const int qadv = (op == 0 || op == 1 || op == 3 || op == 4 || op == 5 || op == 7 || op == 8) ? len : 0;
    c[j].is_id = k < nc && (op == 1 || op == 2);
    c[j].pos = rcarry + wave_excl_scan(radv, lane);
    c[j].irp = qcarry + wave_excl_scan(qadv, lane);
    rcarry = ganon_wave::last(c[j].pos + radv);
    qcarry = ganon_wave::last(c[j].irp + qadv);
  }
  f(c);
}

// Candidate marking: one wave per block of a read with an I/D op (each read once, whatever its
// scopes): its dataset's bit at every op position (no-return atomics, nothing waits on them).
__global__ void __launch_bounds__(kIndelThreads) k_indel_mark(const GanonReadView V, const IndelRead *__restrict__ reads,
                                                              int64_t n_reads, uint32_t *__restrict__ map, int shift) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * kIndelWaves + (threadIdx.x >> 6);
  if (w >= n_reads) return;
  const IndelRead e = reads[w];
  ICHK(IN_CAP(e.read, 3));
  const uint32_t ds = V.dataset[e.read] & 1u;
  walk_block(V, e.read, e.k0, e.pos0, 0, lane, [&](const CigarStep (&c)[kWalkJ]) {
#pragma unroll
    for (int j = 0; j < kWalkJ; ++j) {
      const uint64_t g = map_cell(e.cbase + c[j].pos, shift);
      if (c[j].is_id) atomicOr(map + (g >> 4), 1u << (2 * (g & 15) + ds));
    }
  });
}

// Candidate bits of kWalkJ steps, their map words loaded together.
__device__ __forceinline__ void cand_bits(const uint32_t *__restrict__ map, int shift, int64_t cbase,
                                          const CigarStep (&c)[kWalkJ], bool (&hit)[kWalkJ]) {
  uint32_t mw[kWalkJ];
  uint64_t g[kWalkJ];
#pragma unroll
  for (int j = 0; j < kWalkJ; ++j) {
    g[j] = map_cell(cbase + c[j].pos, shift);
    mw[j] = c[j].is_id ? map[g[j] >> 4] : 0u;
  }
#pragma unroll
  for (int j = 0; j < kWalkJ; ++j)
    hit[j] = c[j].is_id && ((mw[j] >> (2 * (g[j] & 15))) & 3) == 3;   // tumor and normal
}

// The unfiltered path (GANON_PARAM_INDEL_SORT 1, one global sort): every I/D op of every listed
// incidence block at the host's slots.
template <typename KeyT>
__global__ void __launch_bounds__(kIndelThreads) k_indel_emit(const GanonReadView V, const IndelInc *__restrict__ list,
                                                              int64_t n_list, int pos_bits, IndelObs *__restrict__ obs,
                                                              KeyT *__restrict__ keys, uint32_t *__restrict__ vals) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * kIndelWaves + (threadIdx.x >> 6);
  if (w >= n_list) return;
  const IndelInc e = list[w];
  const int scope = (int)(e.scope_par & 0x7FFFFFFFu);
  ICHK(IN_CAP(e.read, 3) && IN_CAP(scope, 4));
  const int span0 = V.span_start[scope];
  int64_t slot = e.obs_off;
  const unsigned long long below = (1ull << lane) - 1ull;
  walk_block(V, e.read, e.k0, e.pos0, e.irp0, lane, [&](const CigarStep (&c)[kWalkJ]) {
#pragma unroll
    for (int j = 0; j < kWalkJ; ++j) {
      const unsigned long long m = __ballot(c[j].is_id);
      if (c[j].is_id) {
        const int64_t o = slot + __popcll(m & below);
        ICHK(IN_CAP(o, 0));
        IndelObs ob;
        ob.read = e.read;
        ob.irp = c[j].irp;
        ob.scope = scope;
        ob.type_len = (c[j].len << 1) | (c[j].op == 1 ? 1 : 0);
        ob.ord = (uint32_t)o;
        obs[o] = ob;
        keys[o] = make_key<KeyT>(e.scope_par, pos_bits, (uint32_t)(c[j].pos - span0));
        vals[o] = (uint32_t)o;
      }
      slot += __popcll(m);
    }
  });
}

// ---- filtered path, per read (round 4) -------------------------------------------------------
// A read's candidate ops (those at positions where a tumor and a normal read have an I/D op) do not
// depend on the scope: they are found once per read block (k_indel_rcount / k_indel_remit, the
// CIGAR walked twice per read instead of twice per (scope, read) incidence, ~4 per C5 read) into a
// read-major candidate list, and every incidence's observations are a coalesced copy of its read's
// entries with the scope's key (k_indel_expand).
__global__ void __launch_bounds__(kIndelThreads) k_indel_rcount(const GanonReadView V, const IndelRead *__restrict__ reads,
                                                                int64_t n_reads, const uint32_t *__restrict__ map,
                                                                int shift, int32_t *__restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * kIndelWaves + (threadIdx.x >> 6);
  if (w >= n_reads) return;
  const IndelRead e = reads[w];
  ICHK(IN_CAP(e.read, 3));
  int total = 0;
  walk_block(V, e.read, e.k0, e.pos0, e.irp0, lane, [&](const CigarStep (&c)[kWalkJ]) {
    bool hit[kWalkJ];
    cand_bits(map, shift, e.cbase, c, hit);
#pragma unroll
    for (int j = 0; j < kWalkJ; ++j) total += __popcll(__ballot(hit[j]));
  });
  if (lane == 0) cnt[w] = total;
}

__global__ void __launch_bounds__(kIndelThreads) k_indel_remit(const GanonReadView V, const IndelRead *__restrict__ reads,
                                                               int64_t n_reads, const uint32_t *__restrict__ map,
                                                               int shift, const int32_t *__restrict__ roff,
                                                               IndelCand *__restrict__ rcand) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * kIndelWaves + (threadIdx.x >> 6);
  if (w >= n_reads) return;
  const IndelRead e = reads[w];
  int64_t slot = roff[w];
  int ord = e.nid0;
  const unsigned long long below = (1ull << lane) - 1ull;
  walk_block(V, e.read, e.k0, e.pos0, e.irp0, lane, [&](const CigarStep (&c)[kWalkJ]) {
    bool keep[kWalkJ];
    cand_bits(map, shift, e.cbase, c, keep);
#pragma unroll
    for (int j = 0; j < kWalkJ; ++j) {
      const unsigned long long m_all = __ballot(c[j].is_id);
      const unsigned long long m = __ballot(keep[j]);
      ICHK(!keep[j] || IN_CAP(slot + __popcll(m & below), 1));
      if (keep[j])
        rcand[slot + __popcll(m & below)] = IndelCand{c[j].pos, c[j].irp, (c[j].len << 1) | (c[j].op == 1 ? 1 : 0),
                                                      ord + (int)__popcll(m_all & below)};
      slot += __popcll(m);
      ord += __popcll(m_all);
    }
  });
}

// Observations per incidence: its read's candidates (thread per incidence).
__global__ void k_indel_icount(const IndelIncR *__restrict__ inc, int64_t n_inc, const int32_t *__restrict__ roff,
                               int32_t *__restrict__ cnt) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n_inc) return;
  const IndelIncR e = inc[i];
  ICHK(e.rfirst >= 0 && e.rnb >= 0 && (long long)e.rfirst + e.rnb <= g_indel_cap[7]);
  cnt[i] = roff[e.rfirst + e.rnb] - roff[e.rfirst];
}

// One wave per incidence: its read's candidate entries with the scope's key, 64 at a time.
template <typename KeyT>
__global__ void __launch_bounds__(kIndelThreads) k_indel_expand(const GanonReadView V, const IndelIncR *__restrict__ inc,
                                                                int64_t n_inc, int pos_bits,
                                                                const int32_t *__restrict__ roff,
                                                                const IndelCand *__restrict__ rcand,
                                                                const int32_t *__restrict__ off, IndelObs *__restrict__ obs,
                                                                KeyT *__restrict__ keys, uint32_t *__restrict__ vals) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * kIndelWaves + (threadIdx.x >> 6);
  if (w >= n_inc) return;
  const IndelIncR e = inc[w];
  const int scope = (int)(e.scope_par & 0x7FFFFFFFu);
  ICHK(IN_CAP(scope, 4) && IN_CAP(e.read, 3) && e.rfirst >= 0 && (long long)e.rfirst + e.rnb <= g_indel_cap[7]);
  const int span0 = V.span_start[scope];
  const int64_t a = roff[e.rfirst], n = roff[e.rfirst + e.rnb] - a, o0 = off[w];
  for (int64_t k = lane; k < n; k += 64) {
    ICHK(IN_CAP(a + k, 1) && IN_CAP(o0 + k, 0));
    const IndelCand c = rcand[a + k];
    const int64_t o = o0 + k;
    IndelObs ob;
    ob.read = e.read;
    ob.irp = c.irp;
    ob.scope = scope;
    ob.type_len = c.type_len;
    ob.ord = (uint32_t)(e.obs_base + c.ord);
    obs[o] = ob;
    keys[o] = make_key<KeyT>(e.scope_par, pos_bits, (uint32_t)(c.pos - span0));
    vals[o] = (uint32_t)o;
  }
}

// ---- short reads (round 5): a thread per read and per incidence ---------------------------------
// A 150 bp read with an indel has 3 CIGAR ops: a wave per read block (above) left 61 of its 64 lanes
// idle, and the ~3e5 indel reads of a c2id batch cost ~0.09 ms per walk kernel in wave launches
// alone. Batches whose reads with I/D ops all have at most kThreadWalkOps ops walk them a thread
// each; the same op order, positions and counts as walk_block.
constexpr int kThreadWalkOps = 32;
constexpr int64_t kTsortMax = 4096;   // (k_indel_tsort) most observations of one scope

template <typename F>
__device__ __forceinline__ void thread_walk(const GanonReadView &V, const IndelRead &e, F &&f) {
  const int nc = V.n_cig[e.read];
  const uint32_t *__restrict__ cig = V.cigar + V.cig_off[e.read];
  int pos = e.pos0, irp = e.irp0;
  for (int k = e.k0; k < nc; ++k) {
    const uint32_t w = cig[k];
    const int op = (int)(w & 0xF), len = (int)(w >> 4);
    if (op == 1 || op == 2) f(pos, irp, op, len);
    pos += (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) ? len : 0;
    irp += (op == 0 || op == 1 || op == 3 || op == 4 || op == 5 || op == 7 || op == 8) ? len : 0;
  }
}

__global__ void __launch_bounds__(256) k_indel_mark_t(const GanonReadView V, const IndelRead *__restrict__ reads,
                                                      int64_t n_reads, uint32_t *__restrict__ map, int shift) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= n_reads) return;
  const IndelRead e = reads[w];
  ICHK(IN_CAP(e.read, 3));
  const uint32_t ds = V.dataset[e.read] & 1u;
  thread_walk(V, e, [&](int pos, int, int, int) {
    const uint64_t g = map_cell(e.cbase + pos, shift);
    atomicOr(map + (g >> 4), 1u << (2 * (g & 15) + ds));
  });
}

__device__ __forceinline__ bool cand_bit(const uint32_t *__restrict__ map, int shift, int64_t gpos) {
  const uint64_t g = map_cell(gpos, shift);
  return ((map[g >> 4] >> (2 * (g & 15))) & 3) == 3;
}

// Count, place and list in one kernel (thread walks): each read's candidates at a block-aggregated
// allocation (one atomic per block) instead of a count kernel, a device scan and a list kernel;
// rstart / rcnt per read (the list is read-major within a block, blocks in any order: a read's
// candidates stay contiguous and in op order, which is all the expansion needs).
__global__ void __launch_bounds__(256) k_indel_rlist_t(const GanonReadView V, const IndelRead *__restrict__ reads,
                                                       int64_t n_reads, const uint32_t *__restrict__ map, int shift,
                                                       int32_t *__restrict__ rstart, int32_t *__restrict__ rcnt,
                                                       unsigned int *__restrict__ total, IndelCand *__restrict__ rcand) {
  __shared__ int wsum[4];
  __shared__ unsigned int base;
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  IndelRead e{};
  int cnt = 0;
  if (w < n_reads) {
    e = reads[w];
    thread_walk(V, e, [&](int pos, int, int, int) { cnt += cand_bit(map, shift, e.cbase + pos) ? 1 : 0; });
  }
  const int incl = ganon_wave::incl_sum(cnt);
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int wbase = 0, btot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    wbase += k < wave ? wsum[k] : 0;
    btot += wsum[k];
  }
  if (threadIdx.x == 0) base = btot ? atomicAdd(total, (unsigned int)btot) : 0u;
  __syncthreads();
  if (w >= n_reads) return;
  int64_t slot = (int64_t)base + wbase + incl - cnt;
  rstart[w] = (int32_t)slot;
  rcnt[w] = cnt;
  if (!cnt) return;
  int ord = e.nid0;
  thread_walk(V, e, [&](int pos, int irp, int op, int len) {
    if (cand_bit(map, shift, e.cbase + pos)) {
      ICHK(IN_CAP(slot, 1));
      rcand[slot++] = IndelCand{pos, irp, (len << 1) | (op == 1 ? 1 : 0), ord};
    }
    ++ord;
  });
}

// Observations per incidence from the thread walks' per-read counts (every short read is one block).
__global__ void k_indel_icount_t(const IndelIncR *__restrict__ inc, int64_t n_inc, const int32_t *__restrict__ rcnt,
                                 int32_t *__restrict__ cnt) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n_inc) return;
  ICHK(IN_CAP(inc[i].rfirst, 7));
  cnt[i] = rcnt[inc[i].rfirst];
}

template <typename KeyT>
__global__ void __launch_bounds__(256) k_indel_expand_t(const GanonReadView V, const IndelIncR *__restrict__ inc,
                                                        int64_t n_inc, int pos_bits, const int32_t *__restrict__ roff,
                                                        const int32_t *__restrict__ rcnt,
                                                        const IndelCand *__restrict__ rcand,
                                                        const int32_t *__restrict__ off, IndelObs *__restrict__ obs,
                                                        KeyT *__restrict__ keys, uint32_t *__restrict__ vals) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= n_inc) return;
  const IndelIncR e = inc[w];
  ICHK(IN_CAP(e.rfirst, 7) && IN_CAP(e.read, 3));
  // (roff: the read's start; rcnt: its count — k_indel_rlist_t, every short read one block)
  const int64_t a = roff[e.rfirst], n = rcnt[e.rfirst];
  if (!n) return;
  const int scope = (int)(e.scope_par & 0x7FFFFFFFu);
  const int span0 = V.span_start[scope];
  const int64_t o0 = off[w];
  ICHK(IN_CAP(scope, 4) && (n == 0 || (IN_CAP(a, 1) && IN_CAP(a + n - 1, 1) && IN_CAP(o0, 0) && IN_CAP(o0 + n - 1, 0))));
  for (int64_t k = 0; k < n; ++k) {
    const IndelCand c = rcand[a + k];
    IndelObs ob;
    ob.read = e.read;
    ob.irp = c.irp;
    ob.scope = scope;
    ob.type_len = c.type_len;
    ob.ord = (uint32_t)(e.obs_base + c.ord);
    obs[o0 + k] = ob;
    keys[o0 + k] = make_key<KeyT>(e.scope_par, pos_bits, (uint32_t)(c.pos - span0));
    vals[o0 + k] = (uint32_t)(o0 + k);
  }
}

// Segment offsets of the filtered observations: seg_off[k] = off[first listed incidence of k].
// Also marks every segment's first element in segbits: a run of equal keys never crosses a segment
// boundary. (The 32-bit key's parity bit alone told adjacent segments apart, but the filter empties
// segments, and two segments of one parity with one empty between them met in one run when the last
// key of the first equalled the first of the second: a missed TN call or a wrong rank — found by
// tools/indel_ab.py on a 10 M-read c2id batch, round 5.)
__global__ void k_indel_segs(const int32_t *__restrict__ seg_first, int32_t n_seg, const int32_t *__restrict__ off,
                             int32_t *__restrict__ seg_off, uint32_t *__restrict__ segbits) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k <= n_seg) {
    ICHK(seg_first[k] >= 0 && seg_first[k] <= g_indel_cap[6]);
    const int32_t o = off[seg_first[k]];
    ICHK(o >= 0 && o <= g_indel_cap[0]);
    seg_off[k] = o;
    // (non-empty segments only: the empty ones share their successor's start, and thousands of
    // atomics on one word serialised the kernel — 0.3 ms on c2id)
    if (k < n_seg && off[seg_first[k + 1]] > o) atomicOr(segbits + (o >> 5), 1u << (o & 31));
  }
}

// Short-read batches (round 5): the filtered observations are already scope-major in registration
// order (incidence, then op order), so sorting each scope's few observations by position in place — a
// stable insertion sort, a thread per segment — is the whole sort. (rocPRIM's segmented sort cost
// 0.17 ms on c2id's ~2e5 mostly empty segments, a global 64-bit radix sort of the capacity 0.09 ms.)
template <typename KeyT>
__global__ void __launch_bounds__(256) k_indel_tsort(KeyT *__restrict__ keys, uint32_t *__restrict__ vals,
                                                     const int32_t *__restrict__ seg_off, int32_t n_seg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_seg) return;
  const int32_t a = seg_off[k], b = seg_off[k + 1];
  ICHK(a >= 0 && a <= b && b <= g_indel_cap[0]);
  for (int32_t i = a + 1; i < b; ++i) {
    const KeyT kk = keys[i];
    const uint32_t vv = vals[i];
    int32_t j = i - 1;
    while (j >= a && keys[j] > kk) {
      keys[j + 1] = keys[j];
      vals[j + 1] = vals[j];
      --j;
    }
    keys[j + 1] = kk;
    vals[j + 1] = vv;
  }
}

__device__ __forceinline__ bool seg_start(const uint32_t *__restrict__ segbits, int64_t j) {
  return segbits && ((segbits[j >> 5] >> (j & 31)) & 1u);
}

// Exact call identity of two observations at the same (scope, pos): type, length, allele.
__device__ bool same_call(const GanonReadView &V, const IndelObs &a, const IndelObs &b) {
  if (a.type_len != b.type_len) return false;
  const int len = a.type_len >> 1;
  const int alen = (a.type_len & 1) ? len : 2;
  ICHK_RET(IN_CAP(a.read, 3) && IN_CAP(b.read, 3) && a.irp >= 0 && b.irp >= 0, false);
  const int La = V.read_len[a.read], Lb = V.read_len[b.read];
  // python slice [irp, irp + alen) clipped to the read
  const int na = max(0, min(La, a.irp + alen) - a.irp);
  const int nb = max(0, min(Lb, b.irp + alen) - b.irp);
  if (na != nb) return false;
  const int64_t oa = V.seq_off[a.read], ob = V.seq_off[b.read];
  for (int i = 0; i < na; ++i)
    if (nib(V.seq, oa, a.irp + i) != nib(V.seq, ob, b.irp + i)) return false;
  return true;
}

// Registration order key of an observation: the reference meets reads by first pileup column
// (ref_start), tumor before normal, file order — the incidence order of the scope — and a read's
// ops in CIGAR order; observation slots follow incidence then op order.
__device__ __forceinline__ unsigned long long reg_key(const GanonReadView &V, const IndelObs &o) {
  return ((unsigned long long)(uint32_t)V.ref_start[o.read] << 32) | o.ord;
}

#ifndef GANON_CLS_DIAG
#define GANON_CLS_DIAG 0   // phase timing builds only (tools/build_variant.py): 1 no normal-column check,
#endif                     // 2 no pass 2, 3 run extents only — all change results
// Does a normal read of the scope cover pos? Eight incidences per round, their loads issued together
// (one incidence per round was a chain of dependent gathers per TN run).
__device__ bool normal_covers(const GanonReadView &V, int scope, int pos) {
  constexpr int kU = 8;
  const int64_t i1 = V.incid_off[scope + 1];
  for (int64_t i = V.incid_off[scope]; i < i1; i += kU) {
    int r[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) r[u] = i + u < i1 ? V.incid_read[i + u] : -1;
#pragma unroll
    for (int u = 0; u < kU; ++u) ICHK_RET(r[u] < 0 || IN_CAP(r[u], 3), false);
    bool hit = false;
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (r[u] >= 0) hit |= V.dataset[r[u]] == 1 && V.ref_start[r[u]] <= pos && pos < V.read_end[r[u]];
    if (hit) return true;
  }
  return false;
}

// One run (a thread each): call heads, TN state, first registered support; the normal pileup column;
// ranks and records of the masked calls. (Round 5 tried the column check a wave per TN run: no gain
// on c2id, and long-read runs lost the thread-per-run parallelism of their second pass: c5 classify
// 0.72 -> 3.8 ms. Not kept.)
template <typename KeyT>
__device__ void classify_run(const GanonReadView &V, const KeyT *__restrict__ keys, const uint32_t *__restrict__ vals,
                             int64_t n, int pos_bits, const IndelObs *__restrict__ obs, uint8_t *__restrict__ flags,
                             int32_t *__restrict__ rank, unsigned long long *__restrict__ repk, int64_t j0,
                             unsigned long long *__restrict__ n_rec, const uint32_t *__restrict__ segbits) {
  ICHK(j0 >= 0 && j0 < n && n <= g_indel_cap[0]);
  const KeyT key = keys[j0];
  int64_t j1 = j0 + 1;
  while (j1 < n && keys[j1] == key && !seg_start(segbits, j1)) ++j1;
#if GANON_INDEL_CHECK
  for (int64_t a = j0; a < j1; ++a) {
    ICHK(IN_CAP(vals[a], 0));
    const IndelObs o = obs[vals[a]];
    ICHK(IN_CAP(o.read, 3) && IN_CAP(o.scope, 4) && o.irp >= 0);
  }
#endif
#if GANON_CLS_DIAG == 3
  if (j1 > j0) return;   // (phase timing builds only: results change)
#endif
  const int scope = obs[vals[j0]].scope;
  const unsigned long long kNone = ~0ull;
  bool any_tn = false;
  // pass 1: call heads (first element of each distinct call, in sorted = slot order), TN state,
  // first registered support
  for (int64_t a = j0; a < j1; ++a) {
    flags[a] = 0;
    repk[a] = kNone;
    const IndelObs oa = obs[vals[a]];
    bool head = true;
    for (int64_t b = j0; b < a && head; ++b)
      if (same_call(V, obs[vals[b]], oa)) head = false;
    if (!head) continue;
    bool t = false, nn = false;
    unsigned long long best = kNone;
    for (int64_t c = a; c < j1; ++c) {
      const uint32_t ic = vals[c];
      const IndelObs oc = obs[ic];
      if (c != a && !same_call(V, oa, oc)) continue;
      if (V.dataset[oc.read] == 0) t = true; else nn = true;
      best = min(best, reg_key(V, oc));
    }
    repk[a] = best;
    if (t && nn) {
      flags[a] = 0x80;         // TN call head; the normal column is checked once per run below
      any_tn = true;
    }
  }
  if (!any_tn) return;
#if GANON_CLS_DIAG == 2
  return;
#endif
  const int pos = V.span_start[scope] + (int)((unsigned long long)key & ((1ull << pos_bits) - 1ull));
  if (GANON_CLS_DIAG != 1 && !normal_covers(V, scope, pos)) {
    for (int64_t a = j0; a < j1; ++a) flags[a] = 0;
    return;
  }
  // pass 2: ranks and records of the masked calls
  unsigned long long recs = 0;
  for (int64_t a = j0; a < j1; ++a) {
    if (!(flags[a] & 0x80)) continue;
    const unsigned long long ka = repk[a];
    int rk = 0;
    for (int64_t b = j0; b < j1; ++b)
      if (repk[b] < ka) ++rk;   // every call head has a distinct first support
    const IndelObs oa = obs[vals[a]];
    for (int64_t c = a; c < j1; ++c) {
      const uint32_t ic = vals[c];
      const IndelObs oc = obs[ic];
      if (c != a && !same_call(V, oa, oc)) continue;
      uint8_t f = (reg_key(V, oc) == ka) ? 1 : 0;
      if (V.write_scope[oc.read] == scope) {
        // a read supporting the call twice keeps its last offset (dict assignment)
        bool last = true;
        for (int64_t d = c + 1; d < j1 && last; ++d) {
          const IndelObs od = obs[vals[d]];
          if (od.read == oc.read && same_call(V, oa, od)) last = false;
        }
        if (last) f |= 2;
      }
      if (f) {
        flags[c] = (uint8_t)((flags[c] & 0x80) | f);
        rank[c] = rk;
        recs += (f & 1) + (f >> 1);
      }
    }
  }
  for (int64_t a = j0; a < j1; ++a) flags[a] &= 3;
  if (recs) atomicAdd(n_rec, recs);
}

// Runs of equal keys = observations at one (scope, pos). Every element's flags start at 0; the
// first element of each run with more than one observation goes to run_list. A workgroup covers
// kRunChunk elements (coalesced, kRunPer per thread) and takes its list slots with ONE atomic add:
// a single global counter hit once per wave serialises (~10 ns per add at the L2).
constexpr int kRunPer = 16;
constexpr int kRunChunk = 256 * kRunPer;

template <typename KeyT>
__global__ void __launch_bounds__(256) k_indel_runs(const KeyT *__restrict__ keys, const int32_t *__restrict__ n_dev,
                                                    uint8_t *__restrict__ flags, int32_t *__restrict__ run_list,
                                                    unsigned int *__restrict__ run_count,
                                                    const uint32_t *__restrict__ segbits) {
  const int64_t n = *n_dev;
  ICHK(n >= 0 && n <= g_indel_cap[0]);
  __shared__ unsigned int wsum[4];
  __shared__ unsigned int base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * kRunChunk;
  unsigned int heads = 0;   // bit i: element c0 + i * 256 + tid is a run head
#pragma unroll
  for (int i = 0; i < kRunPer; ++i) {
    const int64_t j = c0 + (int64_t)i * 256 + threadIdx.x;
    if (j < n) {
      flags[j] = 0;
      const KeyT k = keys[j];
      if ((j == 0 || keys[j - 1] != k || seg_start(segbits, j)) && j + 1 < n && keys[j + 1] == k &&
          !seg_start(segbits, j + 1))
        heads |= 1u << i;
    }
  }
  const unsigned int cnt = __popc(heads);
  // block exclusive scan of cnt
  unsigned int x = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  unsigned int wbase = 0, total = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    wbase += (w < wave) ? wsum[w] : 0u;
    total += wsum[w];
  }
  if (threadIdx.x == 0) base = total ? atomicAdd(run_count, total) : 0u;
  __syncthreads();
  unsigned int o = base + wbase + x - cnt;
#pragma unroll
  for (int i = 0; i < kRunPer; ++i)
    if (heads & (1u << i)) run_list[o++] = (int32_t)(c0 + (int64_t)i * 256 + threadIdx.x);
}

// One thread per run of k_indel_runs (grid-stride over the device-side count). flags per element:
// bit 0 = call record (first registered support of a masked TN call), bit 1 = support record (a
// read the scope writes); rank = the call's registration rank at pos. repk: scratch, registration
// key of each call's first support (UINT64_MAX = not a call head). n_rec: records of the whole
// batch (one atomic add per run that has any).
template <typename KeyT>
__global__ void __launch_bounds__(256) k_indel_classify(const GanonReadView V, const KeyT *__restrict__ keys,
                                                        const uint32_t *__restrict__ vals, const int32_t *__restrict__ n_dev,
                                                        int pos_bits, const IndelObs *__restrict__ obs,
                                                        uint8_t *__restrict__ flags, int32_t *__restrict__ rank,
                                                        unsigned long long *__restrict__ repk,
                                                        const int32_t *__restrict__ run_list,
                                                        const unsigned int *__restrict__ run_count,
                                                        unsigned long long *__restrict__ n_rec,
                                                        const uint32_t *__restrict__ segbits) {
  const int64_t n = *n_dev;
  const unsigned int n_runs = *run_count;
  for (unsigned int ri = blockIdx.x * blockDim.x + threadIdx.x; ri < n_runs; ri += gridDim.x * blockDim.x)
    classify_run<KeyT>(V, keys, vals, n, pos_bits, obs, flags, rank, repk, run_list[ri], n_rec, segbits);
}

// Records in device order (slots from an atomic counter; the host sorts them).
template <typename KeyT>
__global__ void __launch_bounds__(256) k_indel_write(const GanonReadView V, const KeyT *__restrict__ keys,
                                                     const uint32_t *__restrict__ vals, const int32_t *__restrict__ n_dev,
                                                     int pos_bits, const IndelObs *__restrict__ obs,
                                                     const uint8_t *__restrict__ flags, const int32_t *__restrict__ rank,
                                                     unsigned long long *__restrict__ slot,
                                                     ganon_indel_rec *__restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= *n_dev) return;
  const uint8_t f = flags[j];
  if (!f) return;
  ICHK(IN_CAP(vals[j], 0));
  const IndelObs o = obs[vals[j]];
  ICHK(IN_CAP(o.scope, 4));
  ganon_indel_rec rec;
  rec.scope = o.scope;
  rec.pos = V.span_start[o.scope] + (int)((unsigned long long)keys[j] & ((1ull << pos_bits) - 1ull));
  rec.length = o.type_len >> 1;
  rec.type = (o.type_len & 1) ? GANON_INDEL_INS : GANON_INDEL_DEL;
  rec.rank = rank[j];
  rec.read = o.read;
  rec.in_read_pos = o.irp;
  unsigned long long w = atomicAdd(slot, (unsigned long long)((f & 1) + (f >> 1)));
  ICHK(IN_CAP(w + (f & 1) + (f >> 1) - 1, 2));
  if (f & 1) {
    rec.kind = GANON_INDEL_CALL;
    out[w++] = rec;
  }
  if (f & 2) {
    rec.kind = GANON_INDEL_SUPPORT;
    out[w] = rec;
  }
}

// Checked builds: a failed bounds check of any tally kernel so far (its source line), else GANON_OK.
int indel_check_result(ganon_ctx *ctx) {
#if GANON_INDEL_CHECK
  unsigned int chk[2] = {0, 0};
  if (hipMemcpyFromSymbol(chk, HIP_SYMBOL(g_indel_chk), sizeof chk, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(ctx, GANON_E_DEVICE, "indel check: reading the check word failed");
  if (chk[0])
    return fail(ctx, GANON_E_DEVICE, "indel bounds check failed at ganon_indel.hip:%u (%u failures)", chk[0], chk[1]);
#else
  (void)ctx;
#endif
  return GANON_OK;
}

int bits_for(int64_t v) {   // bits to hold 0..v
  int b = 1;
  while (b < 62 && (v >> b) != 0) ++b;
  return b;
}

}  // namespace

struct ganon_indels {
  std::vector<void *> allocs;
  GanonReadView V{};
  const void *db = nullptr;           // the device batch it tallies (the fork point, ctx->fork_db)
  int64_t n_obs = 0, n_list = 0, n_rdist = 0, n_records = -1, n_candidates = -1;
  int32_t n_seg = 0;                  // scopes with observations (segments of the sort)
  int pos_bits = 1, key_bits = 2;
  bool global = false;                // strategy of the last run (GANON_PARAM_INDEL_SORT 1)
  // the filtered observations sorted by one global radix sort of 64-bit (scope, position) keys (the
  // short-read batches, round 5) instead of rocPRIM's segmented sort, whose partitioning copies the
  // segment counts to the host and SYNCHRONIZES the stream: the host waited ~1 ms per c2id step for
  // every queued kernel of its context, so the pipelined contexts ran one after another
  bool gsort = false;
  bool tsort = false;                 // short reads: the in-place segment sort (k_indel_tsort), 32-bit keys
  bool key64 = false;                 // the last run's keys are 64-bit (global or gsort)
  IndelInc *list = nullptr;
  IndelRead *rdist = nullptr;         // distinct reads with an I/D op (candidate marking)
  uint32_t *map = nullptr;            // candidate map, 2 bits per genome position or hashed cell
  int64_t map_words = 0;
  int map_shift = 0;                  // 0: dense (a cell per genome position), else hashed (map_cell)
  bool thread_walk = false;           // every read with an I/D op has at most kThreadWalkOps CIGAR ops
  int32_t *cnt = nullptr;             // [n_list + 1] candidate observations per incidence (ilist)
  int32_t *off = nullptr;             // [n_list + 1] their exclusive scan; off[n_ilist] = count
  IndelIncR *ilist = nullptr;         // incidences with an I/D op (filtered path)
  int64_t n_ilist = 0;
  int32_t *rcnt = nullptr;            // [n_rdist + 1] candidates per read block, then their scan (roff)
  int32_t *roff = nullptr;
  IndelCand *rcand = nullptr;         // the reads' candidate ops, read-major
  int64_t n_rcand_cap = 0;
  int32_t *seg_first = nullptr;       // [n_seg + 1] first ilist incidence of each segment
  int32_t *seg_off = nullptr;         // [n_seg + 1] observation offsets of the segments
  int32_t *nval = nullptr;            // [1] n_obs (unfiltered runs)
  IndelObs *obs = nullptr;
  void *keys[2] = {nullptr, nullptr}; // 8 bytes per observation (either key width)
  uint32_t *vals[2] = {nullptr, nullptr};
  int sorted_sel = 0;                 // which half of the double buffers holds the sorted pairs
  uint8_t *flags = nullptr;
  int32_t *rank = nullptr;
  unsigned long long *repk = nullptr;
  unsigned long long *counters = nullptr;   // [0] records (classify), [1] write slots
  int32_t *run_list = nullptr;        // first element of each run of >1 observations
  unsigned int *run_count = nullptr;
  uint32_t *segbits = nullptr;        // (segmented sort) bit j: element j starts a segment
  void *temp = nullptr;
  size_t temp_bytes = 0;
  ganon_indel_rec *recs = nullptr;
  int64_t recs_cap = 0;
  bool ran = false;
  const int32_t *n_dev() const { return global ? nval : off + n_ilist; }
};

namespace {

template <typename T>
int ind_alloc(ganon_ctx *ctx, ganon_indels *t, T **p, size_t count) {
  *p = nullptr;
  const size_t bytes = std::max<size_t>(count, 1) * sizeof(T) + 128;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(p), bytes);
  if (e != hipSuccess) return fail(ctx, GANON_E_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  t->allocs.push_back(*p);
  return GANON_OK;
}

void ind_release(ganon_indels *t) {
  for (void *p : t->allocs) hipFree(p);
  t->allocs.clear();
}

// rocPRIM's default segmented config partitions the segments by size once there are 3,000 or more,
// and the partitioning copies the small / medium / large counts to the host with a stream
// synchronization: every segmented sort waited for its context's whole queue (the host ~1 ms per c2id
// step, round 5). This config never partitions (the threshold is out of reach) and still sorts short
// segments a warp each (unpartitioned warp sort).
using SegSortConfig = rocprim::segmented_radix_sort_config<7, rocprim::kernel_config<256, 16>,
                                                           rocprim::WarpSortConfig<32, 4, 256, 0xFFFFFFFFu>, true>;

// Segmented (filtered observations, device segment offsets) or one global sort (all observations).
// num_items is the capacity: the filtered count stays on the device, the segments bound the work.
template <typename KeyT>
hipError_t sort_pairs(ganon_indels *t, void *temp, size_t &bytes, bool global, hipStream_t st, int *sel) {
  rocprim::double_buffer<KeyT> K(static_cast<KeyT *>(t->keys[0]), static_cast<KeyT *>(t->keys[1]));
  rocprim::double_buffer<uint32_t> Vb(t->vals[0], t->vals[1]);
  hipError_t e;
  if (global)
    e = rocprim::radix_sort_pairs(temp, bytes, K, Vb, (unsigned int)t->n_obs, 0u, (unsigned int)t->key_bits, st);
  else
    e = rocprim::segmented_radix_sort_pairs<SegSortConfig>(temp, bytes, K, Vb, (unsigned int)t->n_obs, (unsigned int)t->n_seg,
                                            t->seg_off, t->seg_off + 1, 0u, (unsigned int)t->pos_bits, st);
  if (sel) {
    const int ks = K.current() == static_cast<KeyT *>(t->keys[0]) ? 0 : 1;
    const int vs = Vb.current() == t->vals[0] ? 0 : 1;
    *sel = ks == vs ? ks : -1;
  }
  return e;
}

hipError_t scan_counts(ganon_indels *t, void *temp, size_t &bytes, hipStream_t st) {
  return rocprim::exclusive_scan(temp, bytes, t->cnt, t->off, 0, (size_t)(t->n_ilist + 1), rocprim::plus<int32_t>(),
                                 st);
}

hipError_t scan_read_counts(ganon_indels *t, void *temp, size_t &bytes, hipStream_t st) {
  return rocprim::exclusive_scan(temp, bytes, t->rcnt, t->roff, 0, (size_t)(t->n_rdist + 1), rocprim::plus<int32_t>(),
                                 st);
}

template <typename KeyT>
int run_tally(ganon_ctx *ctx, ganon_indels *t) {
  int rc;
  const int64_t n = t->n_obs;   // capacity
  const bool filter = !t->global;
  const unsigned lgrid = (unsigned)((t->n_list + kIndelWaves - 1) / kIndelWaves);
  if (filter && t->key64)   // (one global sort of the capacity: the slots past the filtered count sort last)
    HIP_OR_FAIL(hipMemsetAsync(t->keys[0], 0xFF, (size_t)t->n_obs * sizeof(unsigned long long), ctx->stream));
  HIP_OR_FAIL(hipMemsetAsync(t->counters, 0, 2 * sizeof(unsigned long long), ctx->stream));
  HIP_OR_FAIL(hipMemsetAsync(t->run_count, 0, sizeof(unsigned int), ctx->stream));
#if GANON_INDEL_CHECK   // (checked builds: the capacities every index is checked against; one context at a time)
  {
    const long long caps[8] = {t->n_obs, t->n_rcand_cap, t->recs_cap, t->V.n_reads, t->V.n_scopes, t->n_list, t->n_ilist,
                               t->n_rdist};
    HIP_OR_FAIL(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_indel_cap), caps, sizeof caps, 0, hipMemcpyHostToDevice, ctx->stream));
    HIP_OR_FAIL(ganon_detail::sync_stream(ctx->stream));   // (caps is a stack array)
  }
#endif
  const unsigned rgrid = (unsigned)((t->n_rdist + kIndelWaves - 1) / kIndelWaves);
  if (filter) {
    // per read block: the map, then its candidate ops (count, scan, list); per incidence: counts
    // from the read's, their scan, the segments
    KernelScope ks(ctx, "indel_candidates");
    HIP_OR_FAIL(hipMemsetAsync(t->map, 0, (size_t)t->map_words * 4, ctx->stream));
    const unsigned tgrid = (unsigned)((t->n_rdist + 255) / 256);
    if (t->thread_walk) {
      hipLaunchKernelGGL(k_indel_mark_t, dim3(tgrid), dim3(256), 0, ctx->stream, t->V, t->rdist, t->n_rdist, t->map,
                         t->map_shift);
      // count + place + list in one kernel (its allocation counter: counters[1], idle until download)
      hipLaunchKernelGGL(k_indel_rlist_t, dim3(tgrid), dim3(256), 0, ctx->stream, t->V, t->rdist, t->n_rdist, t->map,
                         t->map_shift, t->roff, t->rcnt, reinterpret_cast<unsigned int *>(t->counters + 1), t->rcand);
      hipLaunchKernelGGL(k_indel_icount_t, dim3((unsigned)((t->n_ilist + 255) / 256)), dim3(256), 0, ctx->stream,
                         t->ilist, t->n_ilist, t->rcnt, t->cnt);
    } else {
      hipLaunchKernelGGL(k_indel_mark, dim3(rgrid), dim3(kIndelThreads), 0, ctx->stream, t->V, t->rdist, t->n_rdist,
                         t->map, t->map_shift);
      hipLaunchKernelGGL(k_indel_rcount, dim3(rgrid), dim3(kIndelThreads), 0, ctx->stream, t->V, t->rdist, t->n_rdist,
                         t->map, t->map_shift, t->rcnt);
      size_t rb = t->temp_bytes;
      if (scan_read_counts(t, t->temp, rb, ctx->stream) != hipSuccess)
        return fail(ctx, GANON_E_DEVICE, "indel read scan failed");
      hipLaunchKernelGGL(k_indel_remit, dim3(rgrid), dim3(kIndelThreads), 0, ctx->stream, t->V, t->rdist, t->n_rdist,
                         t->map, t->map_shift, t->roff, t->rcand);
      hipLaunchKernelGGL(k_indel_icount, dim3((unsigned)((t->n_ilist + 255) / 256)), dim3(256), 0, ctx->stream,
                         t->ilist, t->n_ilist, t->roff, t->cnt);
    }
    size_t bytes = t->temp_bytes;
    if (scan_counts(t, t->temp, bytes, ctx->stream) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "indel scan failed");
    if (!t->key64) {
      HIP_OR_FAIL(hipMemsetAsync(t->segbits, 0, ((size_t)t->n_obs / 32 + 2) * sizeof(uint32_t), ctx->stream));
      hipLaunchKernelGGL(k_indel_segs, dim3((unsigned)((t->n_seg + 256) / 256)), dim3(256), 0, ctx->stream,
                         t->seg_first, t->n_seg, t->off, t->seg_off, t->segbits);
    }
    if ((rc = check_launch(ctx, "indel_candidates"))) return rc;
  }
  {
    KernelScope ks(ctx, "k_indel_emit");
    if (filter && t->thread_walk)
      hipLaunchKernelGGL(k_indel_expand_t<KeyT>, dim3((unsigned)((t->n_ilist + 255) / 256)), dim3(256), 0, ctx->stream,
                         t->V, t->ilist, t->n_ilist, t->pos_bits, t->roff, t->rcnt, t->rcand, t->off, t->obs,
                         static_cast<KeyT *>(t->keys[0]), t->vals[0]);
    else if (filter)
      hipLaunchKernelGGL(k_indel_expand<KeyT>, dim3((unsigned)((t->n_ilist + kIndelWaves - 1) / kIndelWaves)),
                         dim3(kIndelThreads), 0, ctx->stream, t->V, t->ilist, t->n_ilist, t->pos_bits, t->roff, t->rcand,
                         t->off, t->obs, static_cast<KeyT *>(t->keys[0]), t->vals[0]);
    else
      hipLaunchKernelGGL(k_indel_emit<KeyT>, dim3(lgrid), dim3(kIndelThreads), 0, ctx->stream, t->V, t->list, t->n_list,
                         t->pos_bits, t->obs, static_cast<KeyT *>(t->keys[0]), t->vals[0]);
    if ((rc = check_launch(ctx, "k_indel_emit"))) return rc;
  }
  {
    KernelScope ks(ctx, "indel_sort");
    if (filter && t->tsort) {
      hipLaunchKernelGGL(k_indel_tsort<KeyT>, dim3((unsigned)((t->n_seg + 255) / 256)), dim3(256), 0, ctx->stream,
                         static_cast<KeyT *>(t->keys[0]), t->vals[0], t->seg_off, t->n_seg);
      if ((rc = check_launch(ctx, "k_indel_tsort"))) return rc;
      t->sorted_sel = 0;
    } else {
      size_t bytes = t->temp_bytes;
      int sel = 0;
      if (sort_pairs<KeyT>(t, t->temp, bytes, t->key64, ctx->stream, &sel) != hipSuccess)
        return fail(ctx, GANON_E_DEVICE, "indel radix sort failed");
      if (sel < 0) return fail(ctx, GANON_E_DEVICE, "indel radix sort: key/value buffers diverged");
      t->sorted_sel = sel;
    }
  }
  {
    KernelScope ks(ctx, "k_indel_classify");
    const KeyT *keys = static_cast<const KeyT *>(t->keys[t->sorted_sel]);
    // (segment starts: the segmented sort's filtered path only; 64-bit keys hold the whole scope)
    const uint32_t *segbits = filter && !t->key64 ? t->segbits : nullptr;
    hipLaunchKernelGGL(k_indel_runs<KeyT>, dim3((unsigned)((n + kRunChunk - 1) / kRunChunk)), dim3(256), 0,
                       ctx->stream, keys, t->n_dev(), t->flags, t->run_list, t->run_count, segbits);
    // runs <= n / 2 (the counts stay on the device): one thread per possible run, the threads past
    // the count leave at once
    const unsigned grid = (unsigned)std::max<int64_t>(1, (n / 2 + 255) / 256);   // (n = 1: one idle workgroup)
    hipLaunchKernelGGL(k_indel_classify<KeyT>, dim3(grid), dim3(256), 0, ctx->stream, t->V, keys,
                       t->vals[t->sorted_sel], t->n_dev(), t->pos_bits, t->obs, t->flags, t->rank, t->repk,
                       t->run_list, t->run_count, t->counters, segbits);
    if ((rc = check_launch(ctx, "k_indel_classify"))) return rc;
  }
  return GANON_OK;
}

}  // namespace

GANON_API int ganon_indel_upload(ganon_ctx *ctx, const ganon_batch *b, const ganon_dbatch *db, ganon_indels **out) {
  if (!ctx || !b || !db || !out) return fail(ctx, GANON_E_ARG, "null argument");
  *out = nullptr;
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  GanonReadView V{};
  if (ganon_dbatch_read_view(db, &V) || V.n_reads != b->n_reads || V.n_scopes != b->n_scopes)
    return fail(ctx, GANON_E_ARG, "indel upload: host batch does not match the device batch");
  // per read: I/D ops (the host CIGARs were validated by ganon_batch_upload)
  std::vector<int32_t> nid(b->n_reads, 0);
  int32_t max_nc_id = 0;   // most CIGAR ops of a read with an I/D op (the thread-walk kernels' bound)
  for (int32_t r = 0; r < b->n_reads; ++r) {
    const uint32_t *c = b->cigar + b->cig_off[r];
    int32_t k = 0;
    for (int32_t i = 0; i < b->n_cig[r]; ++i) {
      const uint32_t op = c[i] & 0xF;
      k += (op == 1 || op == 2);
    }
    nid[r] = k;
    if (k) max_nc_id = std::max(max_nc_id, b->n_cig[r]);
  }
  // per read with an I/D op: the reference's running offsets at every kWalkOps-th op, and the I/D
  // ops before it (process_indels arithmetic, variation_classifier.py:52-141)
  struct Blk {
    int32_t k0, pos0, irp0, nid0;
  };
  std::vector<int64_t> blk_of(b->n_reads, -1);
  std::vector<Blk> blks;
  for (int32_t r = 0; r < b->n_reads; ++r) {
    if (!nid[r]) continue;
    blk_of[r] = (int64_t)blks.size();
    const uint32_t *c = b->cigar + b->cig_off[r];
    int64_t pos = b->ref_start[r], irp = 0;
    int32_t k_id = 0;
    for (int32_t k = 0; k < b->n_cig[r]; ++k) {
      if (k % kWalkOps == 0) blks.push_back(Blk{k, (int32_t)pos, (int32_t)irp, k_id});
      const uint32_t op = c[k] & 0xF, len = c[k] >> 4;
      if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) pos += len;
      if (op == 0 || op == 1 || op == 3 || op == 4 || op == 5 || op == 7 || op == 8) irp += len;
      k_id += (op == 1 || op == 2);
    }
    if (pos > INT32_MAX || irp > INT32_MAX) return fail(ctx, GANON_E_ARG, "indel upload: read %d offsets over 2^31", r);
  }
  auto n_blk = [&](int32_t r) { return (b->n_cig[r] + kWalkOps - 1) / kWalkOps; };
  auto blk_ids = [&](int32_t r, int i) {   // I/D ops in block i of read r
    const Blk &x = blks[(size_t)(blk_of[r] + i)];
    return (i + 1 < n_blk(r) ? blks[(size_t)(blk_of[r] + i + 1)].nid0 : nid[r]) - x.nid0;
  };
  std::vector<IndelInc> list;            // per incidence block (the unfiltered global-sort path)
  std::vector<IndelIncR> ilist;          // per incidence (the filtered path)
  std::vector<IndelRead> rdist;          // each read with an I/D op once (first incidence's contig)
  std::vector<int32_t> rfirst(b->n_reads, -1), rnb(b->n_reads, 0);   // a read's blocks in rdist
  std::vector<int32_t> seg_first;        // first ilist entry of each segment, then the list size
  int64_t n_obs = 0, n_rcand = 0;
  int32_t max_span = 0;
  int64_t max_seg_obs = 0;   // most observations of one scope before the filter (k_indel_tsort's bound)
  for (int32_t s = 0; s < b->n_scopes; ++s) {
    max_span = std::max(max_span, b->scope_span_len[s]);
    const int64_t obs_before = n_obs;
    const uint32_t par = (uint32_t)(seg_first.size() & 1) << 31;
    const int64_t cbase = b->scope_ref_off[s] - b->scope_span_start[s];   // contig start, genome nibbles
    const size_t before = ilist.size();
    for (int64_t i = b->scope_incid_off[s]; i < b->scope_incid_off[s + 1]; ++i) {
      const int32_t r = b->incid_read[i];
      if (!nid[r]) continue;
      const bool first = rfirst[r] < 0;
      if (first) rfirst[r] = (int32_t)rdist.size();
      for (int k = 0; k < n_blk(r); ++k) {
        const int ids = blk_ids(r, k);
        if (!ids) continue;
        const Blk &x = blks[(size_t)(blk_of[r] + k)];
        list.push_back(IndelInc{r, (uint32_t)s | par, x.k0, x.pos0, x.irp0, 0, n_obs + x.nid0, cbase});
        if (first) {
          rdist.push_back(IndelRead{r, x.k0, x.pos0, x.irp0, x.nid0, 0, cbase});
          ++rnb[r];
        }
      }
      if (first) n_rcand += nid[r];
      ilist.push_back(IndelIncR{r, (uint32_t)s | par, rfirst[r], rnb[r], n_obs});
      n_obs += nid[r];
    }
    if (ilist.size() > before) seg_first.push_back((int32_t)before);
    max_seg_obs = std::max(max_seg_obs, n_obs - obs_before);
  }
  seg_first.push_back((int32_t)ilist.size());
  if (n_obs >= (int64_t)INT32_MAX) return fail(ctx, GANON_E_ARG, "indel upload: %lld observations (max 2^31-1)", (long long)n_obs);
  ganon_indels *t = new ganon_indels();
  t->V = V;
  t->db = db;
  t->n_obs = n_obs;
  t->n_list = (int64_t)list.size();
  t->n_ilist = (int64_t)ilist.size();
  t->n_rdist = (int64_t)rdist.size();
  t->n_rcand_cap = n_rcand;
  t->n_seg = (int32_t)seg_first.size() - 1;
  t->pos_bits = bits_for((int64_t)max_span);
  t->key_bits = t->pos_bits + bits_for(std::max<int64_t>((int64_t)b->n_scopes - 1, 1));
  t->map_words = (2 * b->ref_bytes + 64) / 16 + 1;
  {
    const char *tw = getenv("GANON_INDEL_WAVE_WALK");   // (A/B: 1 keeps the wave-per-block walks)
    t->thread_walk = max_nc_id <= kThreadWalkOps && !(tw && tw[0] == '1');
    // short reads: the in-place segment sort while no scope has more than kTsortMax observations
    // before the filter (its worst case is quadratic); GANON_INDEL_SORTMODE (A/B): seg = rocPRIM's
    // segmented sort, global = one 64-bit radix sort of the capacity
    const char *sm = getenv("GANON_INDEL_SORTMODE");
    const std::string mode = sm ? sm : "";
    t->tsort = t->thread_walk && max_seg_obs <= kTsortMax && mode.empty();
    t->gsort = t->thread_walk && !t->tsort && mode != "seg";
    // hashed map: 2^k cells, at least 64 per candidate-marking op, when that is smaller than the
    // genome's positions (env GANON_INDEL_DENSE_MAP=1: always dense, A/B)
    int k = 12;
    while (k < 40 && (int64_t(1) << k) < 64 * std::max<int64_t>(n_rcand, 1)) ++k;
    const char *dense = getenv("GANON_INDEL_DENSE_MAP");
    if ((int64_t(1) << k) / 16 + 1 < t->map_words && !(dense && dense[0] == '1')) {
      t->map_words = (int64_t(1) << k) / 16;
      t->map_shift = 64 - k;
    }
  }
  int rc = GANON_OK;
  auto bail = [&](int code) {
    ind_release(t);
    delete t;
    return code;
  };
  if (t->pos_bits > 31 || t->key_bits > 64) return bail(fail(ctx, GANON_E_ARG, "indel upload: sort key needs %d bits", t->key_bits));
  if (n_obs > 0) {
    if ((rc = ind_alloc(ctx, t, &t->list, list.size()))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->rdist, rdist.size()))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->map, (size_t)t->map_words))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->cnt, list.size() + 1))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->off, list.size() + 1))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->ilist, ilist.size()))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->rcnt, rdist.size() + 1))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->roff, rdist.size() + 1))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->rcand, (size_t)n_rcand))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->seg_first, seg_first.size()))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->seg_off, seg_first.size()))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->nval, 1))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->obs, (size_t)n_obs))) return bail(rc);
    for (int h = 0; h < 2; ++h) {
      if ((rc = ind_alloc(ctx, t, reinterpret_cast<unsigned long long **>(&t->keys[h]), (size_t)n_obs))) return bail(rc);
      if ((rc = ind_alloc(ctx, t, &t->vals[h], (size_t)n_obs))) return bail(rc);
    }
    if ((rc = ind_alloc(ctx, t, &t->flags, (size_t)n_obs))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->rank, (size_t)n_obs))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->repk, (size_t)n_obs))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->counters, 2))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->run_list, (size_t)n_obs / 2 + 1))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->run_count, 1))) return bail(rc);
    if ((rc = ind_alloc(ctx, t, &t->segbits, (size_t)n_obs / 32 + 2))) return bail(rc);
    // temp storage: the largest of the two sorts and the count scan
    size_t seg_bytes = 0, glob_bytes = 0, scan_bytes = 0, rscan_bytes = 0;
    if (sort_pairs<uint32_t>(t, nullptr, seg_bytes, false, ctx->stream, nullptr) != hipSuccess ||
        sort_pairs<unsigned long long>(t, nullptr, glob_bytes, true, ctx->stream, nullptr) != hipSuccess ||
        scan_counts(t, nullptr, scan_bytes, ctx->stream) != hipSuccess ||
        scan_read_counts(t, nullptr, rscan_bytes, ctx->stream) != hipSuccess)
      return bail(fail(ctx, GANON_E_DEVICE, "indel upload: radix sort / scan sizing failed"));
    t->temp_bytes = std::max(std::max(seg_bytes, glob_bytes), std::max(scan_bytes, rscan_bytes));
    if ((rc = ind_alloc(ctx, t, reinterpret_cast<uint8_t **>(&t->temp), t->temp_bytes))) return bail(rc);
    const int32_t nv = (int32_t)n_obs;
    hipError_t e = hipMemcpyAsync(t->list, list.data(), list.size() * sizeof(IndelInc), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(t->rdist, rdist.data(), rdist.size() * sizeof(IndelRead), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(t->ilist, ilist.data(), ilist.size() * sizeof(IndelIncR), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(t->seg_first, seg_first.data(), seg_first.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                         ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(t->nval, &nv, sizeof nv, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(t->cnt + ilist.size(), 0, sizeof(int32_t), ctx->stream);   // scan tails
    if (e == hipSuccess) e = hipMemsetAsync(t->rcnt + rdist.size(), 0, sizeof(int32_t), ctx->stream);
    if (e == hipSuccess) e = ganon_detail::sync_stream(ctx->stream);
    if (e != hipSuccess) return bail(fail(ctx, GANON_E_DEVICE, "indel upload copy failed: %s", hipGetErrorString(e)));
  }
  *out = t;
  return GANON_OK;
}

GANON_API int ganon_indel_run(ganon_ctx *ctx, ganon_indels *t) {
  if (!ctx || !t) return fail(ctx, GANON_E_ARG, "null argument");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  t->ran = true;
  t->n_records = -1;
  t->n_candidates = -1;
  if (t->n_obs == 0) return GANON_OK;
  t->global = ctx->indel_sort != 0;
  t->key64 = t->global || t->gsort;
  if (!(ctx->indel_fork > 0 && ctx->fork_db && ctx->fork_db == t->db))
    return t->key64 ? run_tally<unsigned long long>(ctx, t) : run_tally<uint32_t>(ctx, t);
  // on the side stream from the batch's fork point, joined back into the context's stream (every
  // later operation of the context — downloads, the next plan — waits for the tally)
  ctx->fork_db = nullptr;
  if (!ctx->side) HIP_OR_FAIL(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
  if (!ctx->join_ev) HIP_OR_FAIL(hipEventCreateWithFlags(&ctx->join_ev, hipEventDisableTiming));
  const hipStream_t main = ctx->stream;
  HIP_OR_FAIL(hipStreamWaitEvent(ctx->side, ctx->fork_ev, 0));
  ctx->stream = ctx->side;
  const int rc = t->key64 ? run_tally<unsigned long long>(ctx, t) : run_tally<uint32_t>(ctx, t);
  ctx->stream = main;
  HIP_OR_FAIL(hipEventRecord(ctx->join_ev, ctx->side));
  HIP_OR_FAIL(hipStreamWaitEvent(main, ctx->join_ev, 0));
  return rc;
}

GANON_API int64_t ganon_indel_download(ganon_ctx *ctx, ganon_indels *t, ganon_indel_rec *out, int64_t cap) {
  if (!ctx || !t) return fail(ctx, GANON_E_ARG, "null argument");
  if (!t->ran) return fail(ctx, GANON_E_STATE, "indel download before run");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipSetDevice failed");
  if (t->n_obs == 0) {
    t->n_records = 0;
    return 0;
  }
  unsigned long long total = 0;
  int32_t cand = 0;
  hipError_t e = ganon_detail::readback(&total, t->counters, sizeof total, ctx->stream);
  if (e == hipSuccess) e = ganon_detail::readback(&cand, t->n_dev(), sizeof cand, ctx->stream);
  if (e == hipSuccess) e = ganon_detail::sync_stream(ctx->stream);
  t->n_candidates = cand;
  if (e != hipSuccess) return fail(ctx, GANON_E_DEVICE, "indel download: %s", hipGetErrorString(e));
  if (int crc = indel_check_result(ctx)) return crc;
  t->n_records = (int64_t)total;
  if (!out || cap < (int64_t)total || total == 0) return (int64_t)total;
  if (t->recs_cap < (int64_t)total) {
    int rc = ind_alloc(ctx, t, &t->recs, (size_t)total);
    if (rc) return rc;
    t->recs_cap = (int64_t)total;
  }
  const int64_t n = t->n_obs;
  const unsigned grid = (unsigned)((n + 255) / 256);
  e = hipMemsetAsync(t->counters + 1, 0, sizeof(unsigned long long), ctx->stream);
  if (e != hipSuccess) return fail(ctx, GANON_E_DEVICE, "indel download: %s", hipGetErrorString(e));
#if GANON_INDEL_CHECK
  {
    const long long rcap = t->recs_cap;
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_indel_cap), &rcap, sizeof rcap, 2 * sizeof(long long), hipMemcpyHostToDevice,
                               ctx->stream);
    if (e == hipSuccess) e = ganon_detail::sync_stream(ctx->stream);
    if (e != hipSuccess) return fail(ctx, GANON_E_DEVICE, "indel download: %s", hipGetErrorString(e));
  }
#endif
  if (t->key64)
    hipLaunchKernelGGL(k_indel_write<unsigned long long>, dim3(grid), dim3(256), 0, ctx->stream, t->V,
                       static_cast<const unsigned long long *>(t->keys[t->sorted_sel]), t->vals[t->sorted_sel],
                       t->n_dev(), t->pos_bits, t->obs, t->flags, t->rank, t->counters + 1, t->recs);
  else
    hipLaunchKernelGGL(k_indel_write<uint32_t>, dim3(grid), dim3(256), 0, ctx->stream, t->V,
                       static_cast<const uint32_t *>(t->keys[t->sorted_sel]), t->vals[t->sorted_sel], t->n_dev(),
                       t->pos_bits, t->obs, t->flags, t->rank, t->counters + 1, t->recs);
  int rc = check_launch(ctx, "k_indel_write");
  if (rc) return rc;
  e = hipMemcpyAsync(out, t->recs, (size_t)total * sizeof(ganon_indel_rec), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = ganon_detail::sync_stream(ctx->stream);
  if (e != hipSuccess) return fail(ctx, GANON_E_DEVICE, "indel download: %s", hipGetErrorString(e));
  if ((rc = indel_check_result(ctx))) return rc;
  return (int64_t)total;
}

GANON_API int ganon_indel_info(const ganon_indels *t, int64_t *info8) {
  if (!t || !info8) return GANON_E_ARG;
  info8[0] = t->n_obs;
  info8[1] = t->n_list;
  info8[2] = t->key64 ? t->key_bits : t->pos_bits;
  info8[3] = t->n_records;
  info8[4] = t->n_candidates;
  info8[5] = t->n_rdist;
  info8[6] = t->global ? 1 : 0;
  info8[7] = 0;
  return GANON_OK;
}

GANON_API int ganon_indel_free(ganon_ctx *ctx, ganon_indels *t) {
  if (!t) return GANON_OK;
  if (ctx) {
    hipSetDevice(ctx->device);
    ganon_detail::sync_stream(ctx->stream);
  }
  ind_release(t);
  delete t;
  return GANON_OK;
}
