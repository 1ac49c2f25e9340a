// ganon_hip.hip — MI355X (gfx950) germline-variant masking kernels + the C ABI of
// include/ganon.h (libganon_hip.so).
//
// Reference semantics (per scope = one CompleteGermlineAnonymizer.anonymize call,
// anonymizer_methods.py:431-535):
//   tally     process_snv for every aligned base of every scope read
//             (variation_classifier.py:144-182, :185-215): base != 'N', base != ref,
//             ref in ACGT -> observation (pos, allele, tumor|normal);
//   classify  SomaticVariationType state machine (variants.py:33-39): a call ends in
//             TUMORAL_NORMAL_VARIANT iff it was observed in >=1 tumor AND >=1 normal read;
//   mask      at the normal column: every supporting read of a TN call other than the
//             kept window variant gets the reference base (anonymizer_methods.py:537-556,
//             :170-176); the call is counted for the statistics (:555-556).
//
// Design: integer/byte work, HBM-bound — no MFMA. A run is
//   device prep (ganon_prep.hip): the raw SoA -> segment records, scope groups, partitions;
//   k_group<2, true>: one 256-thread workgroup per scope group copies its partition pieces of
//             the output and streams every aligned base of its scopes in 32-base chunks;
//             mismatches become LDS observations, classified per (scope, position, allele);
//   k_tile_large + k_mask_large: scopes wider than 1 Mi positions (16 Ki-position LDS tiles);
//   k_finish: far masks, totals.
// The reference genome is resident (ganon_ref): nt16 + a 2-bit copy + a non-ACGT block map.
#include <hip/hip_runtime.h>
#include <map>
#include <mutex>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/ganon.h"
#include "ganon_batch.h"
#include "ganon_ctx.h"

using namespace ganon_dev;

namespace {

// Buffers reached through GrpAux (device memory holding pointers) as address-space-1 pointers:
// global_* memory ops instead of flat_* on the overflow, far-list and per-scope-count paths.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T *gp(T *p) {
  return (__attribute__((address_space(1))) T *)(uintptr_t)p;
}
typedef __attribute__((address_space(1))) unsigned long long GU64;
typedef __attribute__((address_space(1))) unsigned int GU32;

__device__ __forceinline__ int nib_at(const uint8_t *__restrict__ buf, int64_t i) {
  const uint8_t b = buf[i >> 1];
  return (i & 1) ? (b & 0xF) : (b >> 4);
}

__device__ __forceinline__ bool is_acgt(int c) { return c != 0 && (c & (c - 1)) == 0 && c <= 8; }

// Per-lane monotone walk over a read's CIGAR: query positions visited in increasing order.
struct CigarCursor {
  const uint32_t *cig;
  int n, k;
  int q0;        // first query position of op k
  int r0;        // first reference position of op k
  int qlen, rlen, op;

  __device__ __forceinline__ void load() {
    if (k < n) {
      const uint32_t w = cig[k];
      op = w & 0xF;
      const int len = (int)(w >> 4);
      qlen = (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) ? len : 0;
      rlen = (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) ? len : 0;
    }
  }
  __device__ __forceinline__ void init(const uint32_t *c, int nc, int ref_start) {
    cig = c; n = nc; k = 0; q0 = 0; r0 = ref_start; qlen = rlen = 0; op = 0;
    load();
  }
  // Returns the reference position aligned to query position q (M/=/X), or -1 when q sits
  // in an I/S op or beyond the CIGAR. q must not decrease between calls.
  __device__ __forceinline__ int ref_of(int q) {
    while (k < n && q >= q0 + qlen) {
      q0 += qlen; r0 += rlen; ++k;
      load();
    }
    if (k >= n) return -1;
    if (op == 0 || op == 7 || op == 8) return r0 + (q - q0);
    return -1;
  }
};

__device__ __forceinline__ int block_sum(int v, int *scratch) {
  // wave reduction then LDS across waves; scratch holds kWaves ints.
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wave] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) t += scratch[w];
  return t;
}

// ---- tally of one read into the LDS table covering [a, b) ------------------------------
// TB = bytes per position: 1 (ACGT nibbles) or 4 (16-code masks). Returns true when a
// non-ACGTN base that would be a call was seen (only meaningful for TB == 1).
// Reference nibble of contig position p: staged in LDS (nibble 0 = position a) ...
struct LdsRef {
  const uint8_t *refb;
  int a;
  __device__ __forceinline__ int operator()(int p) const {
    const int off = p - a;
    return (refb[off >> 1] >> ((off & 1) ? 0 : 4)) & 0xF;
  }
};
// ... or read straight from the packed genome (nib0 = nibble index of position 0).
struct GlobalRef {
  const uint8_t *ref;
  int64_t nib0;
  __device__ __forceinline__ int operator()(int p) const { return nib_at(ref, nib0 + p); }
};

template <int TB, typename RefFn>
__device__ __forceinline__ bool tally_read(const DevBatch &B, int r, int a, int b,
                                           uint32_t *tab, const RefFn &refn, int lane) {
  const int L = B.read_len[r];
  const int ds = B.dataset[r];
  const int64_t sq = B.seq_off[r] * 2;
  CigarCursor cur;
  cur.init(B.cigar + B.cig_off[r], B.n_cig[r], B.ref_start[r]);
  bool rare = false;
  for (int q = lane; q < L; q += 64) {
    const int p = cur.ref_of(q);
    if (p < a || p >= b) continue;
    const int c = nib_at(B.seq, sq + q);
    const int off = p - a;
    const int rc = refn(p);
    if (c == 15 || c == rc || !is_acgt(rc)) continue;
    if (TB == 1) {
      if (is_acgt(c)) atomicOr(&tab[off >> 2], (uint32_t)c << (ds * 4 + (off & 3) * 8));
      else rare = true;
    } else {
      atomicOr(&tab[off], (1u << c) << (16 * ds));
    }
  }
  return rare;
}

template <int TB>
__device__ __forceinline__ uint32_t tn_mask(const uint32_t *tab, int off) {
  if (TB == 1) {
    const uint32_t byte = (tab[off >> 2] >> ((off & 3) * 8)) & 0xFF;
    return byte & (byte >> 4) & 0xF;                  // ACGT one-hot codes
  } else {
    const uint32_t w = tab[off];
    return w & (w >> 16) & 0xFFFF;                    // bit c = code c
  }
}

template <int TB>
__device__ __forceinline__ bool tn_hit(uint32_t tn, int c) {
  if (TB == 1) return is_acgt(c) && (tn & (uint32_t)c);
  return (tn >> c) & 1u;
}

template <int TB>
__device__ __forceinline__ int tn_count(uint32_t tn) { return __popc(tn); }

// Stage the reference nibbles of [a, a + span) into LDS (packed, nibble 0 = position a).
__device__ __forceinline__ void stage_ref(const DevBatch &B, int64_t nib0, int span, uint8_t *refb) {
  const int nbytes = (span + 1) >> 1;
  for (int j = threadIdx.x; j < nbytes; j += kBlock) {
    const int64_t n0 = nib0 + 2 * (int64_t)j;
    const int hi = nib_at(B.ref, n0);
    const int lo = (2 * j + 1 < span) ? nib_at(B.ref, n0 + 1) : 0;
    refb[j] = (uint8_t)((hi << 4) | lo);
  }
}

// Clear the tumor bit of the kept allele so the kept call is neither masked nor counted.
template <int TB>
__device__ __forceinline__ void clear_keep(const DevBatch &B, int s, int a, int b, uint32_t *tab) {
  if (threadIdx.x != 0) return;
  const int kp = B.keep_pos[s];
  if (kp < a || kp >= b) return;
  const int kc = B.keep_code[s];
  const int off = kp - a;
  if (TB == 1) {
    if (is_acgt(kc)) atomicAnd(&tab[off >> 2], ~((uint32_t)kc << ((off & 3) * 8)));
  } else {
    atomicAnd(&tab[off], ~(1u << kc));
  }
}

// Write the masked copy of read r (all bytes) using the LDS tally of [a, b).
template <int TB, typename RefFn>
__device__ __forceinline__ int mask_read_lds(const DevBatch &B, int r, int a, const uint32_t *tab,
                                             const RefFn &refn, uint8_t *__restrict__ out, int lane) {
  const int L = B.read_len[r];
  const int64_t so = B.seq_off[r];
  CigarCursor cur;
  cur.init(B.cigar + B.cig_off[r], B.n_cig[r], B.ref_start[r]);
  int masked = 0;
  const int nbytes = (L + 1) >> 1;
  for (int j = lane; j < nbytes; j += 64) {
    const uint8_t in = B.seq[so + j];
    int nb[2] = {in >> 4, in & 0xF};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = 2 * j + h;
      if (q >= L) break;
      const int p = cur.ref_of(q);
      if (p < 0) continue;
      const int off = p - a;
      const uint32_t tn = tn_mask<TB>(tab, off);
      if (tn && tn_hit<TB>(tn, nb[h])) {
        nb[h] = refn(p);
        ++masked;
      }
    }
    out[so + j] = (uint8_t)((nb[0] << 4) | nb[1]);
  }
  return masked;
}

// ---- nibble helpers ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t nib_swap(uint32_t d) { return ((d >> 4) & 0x0F0F0F0Fu) | ((d & 0x0F0F0F0Fu) << 4); }

// 16 consecutive nibbles starting at nibble index n of a packed buffer (padded by 12 bytes):
// nibble k of the result at bits [4k, 4k+4).
__device__ __forceinline__ uint64_t load16(const uint8_t *__restrict__ buf, int64_t n) {
  const uint32_t *p = reinterpret_cast<const uint32_t *>(buf) + (n >> 3);
  const uint32_t d0 = nib_swap(p[0]), d1 = nib_swap(p[1]), d2 = nib_swap(p[2]);
  const uint64_t x0 = (uint64_t)d0 | ((uint64_t)d1 << 32);
  const uint64_t x1 = (uint64_t)d1 | ((uint64_t)d2 << 32);
  const int sh = 4 * (int)(n & 7);
  return (uint64_t)(uint32_t)(x0 >> sh) | ((uint64_t)(uint32_t)(x1 >> sh) << 32);
}

__device__ __forceinline__ void patch_nibble(uint8_t *out, int64_t nib_index, int from, int to) {
  const int64_t byte = nib_index >> 1;
  const int sh = 8 * (int)(byte & 3) + ((nib_index & 1) ? 0 : 4);
  atomicXor(reinterpret_cast<uint32_t *>(out) + (byte >> 2), (uint32_t)(from ^ to) << sh);
}

__device__ __forceinline__ int64_t i64_of(int lo, int hi) {
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// ---- 2-bit reference ----------------------------------------------------------------------
// Word w = bases [16w, 16w + 16) of ref_nt16 as 2-bit codes (A0 C1 G2 T3; base i at bits
// 2 * (i & 15)). Non-ACGT bases get code 0: only segments whose reference range is all ACGT
// (ordered first in their group at upload) read this copy — half the bytes, fewer lines.
__global__ void __launch_bounds__(kBlock) k_ref2(const uint8_t *__restrict__ ref, int64_t n_words,
                                                 uint32_t *__restrict__ ref2) {
  for (int64_t w = blockIdx.x * (int64_t)kBlock + threadIdx.x; w < n_words; w += (int64_t)gridDim.x * kBlock) {
    const uint64_t v = load16(ref, 16 * w);
    uint32_t code = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int c = (int)((v >> (4 * k)) & 15);
      if (is_acgt(c)) code |= (uint32_t)__builtin_ctz(c) << (2 * k);
    }
    ref2[w] = code;
  }
}

// 16 codes of a 2-bit window (code k at bits 2k) as one-hot nt16 nibbles (nibble k).
__device__ __forceinline__ uint64_t expand2(uint32_t x) {
  uint64_t y = x;
  y = (y | (y << 16)) & 0x0000FFFF0000FFFFull;
  y = (y | (y << 8)) & 0x00FF00FF00FF00FFull;
  y = (y | (y << 4)) & 0x0F0F0F0F0F0F0F0Full;
  y = (y | (y << 2)) & 0x3333333333333333ull;        // code k in nibble k
  const uint64_t lo = y & 0x1111111111111111ull, hi = (y >> 1) & 0x1111111111111111ull;
  const uint64_t v = lo + 0x1111111111111111ull;     // 1 (A) or 2 (C) ...
  const uint64_t m = hi * 15;                         // ... shifted to 4 (G) or 8 (T)
  return (v & ~m) | ((v << 2) & m);
}


// ---- group kernels: scope groups, observation lists ---------------------------------------
// No per-scope table and no per-scope serialization. At upload every read of a small scope is
// cut into segments (one per aligned M/=/X run: query nibble index, reference nibble index,
// length) and consecutive scopes are packed into groups of ~kGrpTarget segments. One 256-thread
// workgroup streams all 16-base chunks of all segments of its group at once (memory-level
// parallelism across scopes instead of one scope at a time), and every base that differs from
// an ACGT reference base becomes an observation in LDS:
//   key = scope_local:12 | (pos - span_start):48 | allele:4
//   payload = nibble index:48 | ref:4 | dataset:1 | mine:1
// A set of equal keys is one call (pos, allele) of one scope, TN iff it holds a tumor and a
// normal observation — the end state of the reference's per-position state machine
// (variants.py:33-39) — and not the window's kept variant. TN calls are counted
// and their observations in reads the scope writes are masked. All 16 codes are handled
// alike (no re-run). A group whose observations overflow the LDS list (deep coverage, long
// reads) is re-scanned once into its own global observation region (sized at upload, L2-hot),
// aggregated in a global hash table of distinct keys (workgroup-scope atomics: only this
// workgroup touches it), classified, and masked from the observation region — the reads are
// not scanned again. A region that overflows too is split over halves of its key range.
//
// Output. GROUP: a device copy of seq precedes the kernel, masks are atomic XORs. GROUP_FUSED:
// groups are launched in the order of their reads in the sequence buffer and each workgroup
// owns a 128-byte-aligned partition [p0, p1) of the output, which it copies with whole-line
// 16-byte stores before scanning (its reads' bases are then L2-hot for the scan). Masks inside
// the partition are plain byte stores seq[b] ^ mask after the copy has drained; masks of
// bytes in another workgroup's partition (a read crossing a partition boundary) go to a
// global list applied by k_finish after the kernel. Partial-line stores from different
// workgroups cost ~4x whole-line stores on MI355X (tools/membench.hip), hence partitions.
constexpr int kGrpThreads = 256;
#ifndef GANON_K2_BLOCKS
#define GANON_K2_BLOCKS 6   // resident workgroups per CU the K = 2 instance is compiled for
#endif
constexpr int kGrpTile = 256;        // segment records staged per tile
constexpr int kGrpStack = 80;        // key ranges pending (bisection depth <= 64)
constexpr int kGrpMap = 4096;        // chunk -> segment map entries (larger tiles binary-search)
constexpr int kGrpQuad = 256;        // lists up to this size are matched without sorting
constexpr unsigned long long kEmpty = ~0ull;
constexpr unsigned long long kNibMask = (1ull << 48) - 1;
// key-range pass: observations to the LDS list, overflow to the group's global region
enum { kModeCollect = 0 };
// GANON_PARAM_GROUP_SKIP (profiling only, results invalid): phases left out
enum { kSkipClassify = 1, kSkipChunks = 2, kSkipCopy = 4, kSkipCounts = 8 };
static_assert(kGrpTile == kGrpThreads && kGrpTile <= 256, "one staged record per thread, 8-bit map");

// The few batch arrays the group kernels read (a slim kernel argument keeps SGPRs free).
struct GrpBatch {
  const uint8_t *seq, *ref, *keep_code;
  const uint32_t *ref2;
  const int32_t *keep_pos, *span_start, *span_len;
};

// OBS: observations held in LDS before a list overflows into the group's global region (512; 1024
// for deep-coverage batches, ganon_batch_run picks it); the in-partition mask list has the same size.
template <int OBS>
struct GrpSharedT {
  static constexpr int kObs = OBS;
  int4 rec[kGrpTile];               // segment records (layout at kSegMine)
  int pre[kGrpTile];
  uint8_t cmap[kGrpMap];            // staged segment of each chunk (tiles of <= kGrpMap chunks)
  int wsum[kGrpThreads / 64];
  unsigned long long key[OBS];      // observation list
  unsigned long long pay[OBS];
  unsigned long long patch[OBS];    // nibble index << 4 | (from ^ to)
  unsigned long long stk_lo[kGrpStack], stk_hi[kGrpStack];
  int stk_mode[kGrpStack];
  unsigned long long kmin, kmax;
  int top, n_obs, n_patch, n_filt;
  int blk_calls, blk_bases;         // this workgroup's contribution to the totals
  int cnt_calls[kGrpMaxScopes];     // per-scope counts, written out once at the end
  int cnt_bases[kGrpMaxScopes];
  int wdirty[kGrpThreads / 64];     // fused one-segment mode: a wave's records need the nt16 reference
  unsigned long long hsum;          // ... and the write-scope hash sum of the group's mine incidences
  int n_xent, n_xrec, n_xtile;      // ... and its incidences with further segments (entries), their records, an
                                    // extras tile's records
};

struct GrpRange {
  unsigned long long lo, hi;
  int mode;
};

struct PatchSink {
  uint8_t *out;
  int64_t p0, p1, q0, q1;           // fused: this workgroup's partition pieces of out (bytes)
  const GrpAux *aux;                // far-mask list
  bool fused;
  bool lds;                         // fused: in-partition masks into the LDS list
  __device__ bool inside(int64_t byte) const { return (byte >= p0 && byte < p1) || (byte >= q0 && byte < q1); }
};

template <class SH>
__device__ __forceinline__ void sink_patch(SH &sh, const PatchSink &k, int64_t nib, int c, int rc) {
  const unsigned long long e = ((unsigned long long)nib << 4) | (unsigned long long)(c ^ rc);
  if (k.fused) {
    const int64_t byte = nib >> 1;
    if (!k.inside(byte)) {
      const unsigned long long i = __hip_atomic_fetch_add(gp(k.aux->far_count), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (i < (unsigned long long)k.aux->far_cap) gp(k.aux->far)[i] = e;
      return;
    }
    if (k.lds) {
      const int i = atomicAdd(&sh.n_patch, 1);
      if (i < SH::kObs) sh.patch[i] = e;
      return;
    }
  }
  patch_nibble(k.out, nib, c, rc);
}

// A group's global observation region (overflow path): cap observations (key, payload) at
// obs + off, and a hash table of up to 2 * cap distinct keys (key, 2-bit tumor/normal flags)
// at tkey/tflag + 2 * off. Only the owning workgroup touches it.
struct GrpGlobal {
  const GrpAux *aux;
  int64_t off;
  int cap;
};

__device__ __forceinline__ unsigned long long ld_l2(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1: past the CU's L1
}
__device__ __forceinline__ unsigned int ld_l2(const unsigned int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_l2(const GU64 *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned int ld_l2(const GU32 *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// threadIdx.x the compiler cannot hoist out of a loop: address arithmetic of the rare overflow
// paths is then recomputed where it is used instead of being kept live (spilled to scratch)
// across the whole kernel.
__device__ __forceinline__ int opaque_tid() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

__device__ __forceinline__ unsigned gtab_home(unsigned long long key, int tsize) {
  const unsigned long long h = key * 0x9E3779B97F4A7C15ull;
  return (unsigned)(((h >> 32) * (unsigned long long)tsize) >> 32);
}

template <class SH>
__device__ __forceinline__ void grp_count(SH &sh, int s_local, int calls, int bases);

// Per-dataset Bloom bitmaps of an overflowing pass's observation keys, built from the stored
// observations in the patch list's LDS (unused until the classification): a key seen in only one
// dataset can never be a TN call, so a list that overflows the LDS list is first filtered by them
// (grp_filter) — a 60x scope's sequencing errors, almost all single-dataset, then mostly drop out
// and the rest fits in LDS. Passes that do not overflow (every configs[1] group) pay nothing.
#ifndef GANON_GRP_BLOOM
#define GANON_GRP_BLOOM 1   // 0: no Bloom filtering (A/B builds)
#endif
constexpr int kBloomBits = 16384;   // per dataset: the two take the 4 KiB of the 512-entry patch list
__device__ __forceinline__ uint32_t bloom_hash(unsigned long long key) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 40);
}
template <class SH>
__device__ __forceinline__ uint32_t *bloom_of(SH &sh) {
  static_assert(sizeof(sh.patch) * 8 >= 2 * kBloomBits, "Bloom bitmaps live in the patch list");
  return reinterpret_cast<uint32_t *>(sh.patch);
}
template <class SH>
__device__ __forceinline__ bool bloom_both(SH &sh, unsigned long long key) {
  const uint32_t h = bloom_hash(key) & (kBloomBits - 1), *b = bloom_of(sh);
  return ((b[h >> 5] & b[(kBloomBits + h) >> 5]) >> (h & 31)) & 1u;
}

// payload: nibble index:48 | ref:4 | dataset:1 | mine:1
template <class SH>
__device__ __forceinline__ void grp_observe(SH &sh, const GrpRange &R, const GrpGlobal &gg,
                                            unsigned long long key, int64_t nib, int rc, int ds, uint32_t mine) {
  if (key < R.lo || key >= R.hi) return;
  const unsigned long long pay = (unsigned long long)nib | ((unsigned long long)rc << 48) |
                                 ((unsigned long long)ds << 52) | ((unsigned long long)mine << 53);
  const int k = atomicAdd(&sh.n_obs, 1);
  if (k < SH::kObs) {
    sh.key[k] = key;
    sh.pay[k] = pay;
  } else {
    // past the LDS list: straight into the group's global region (no second scan)
    if (k - SH::kObs < gg.cap - SH::kObs) {
      gp(gg.aux->okey)[gg.off + (k - SH::kObs)] = key;
      gp(gg.aux->opay)[gg.off + (k - SH::kObs)] = pay;
    }
  }
}

// Is (scope s, pos_off, allele c) the window's kept variant? (clear_keep's rule)
__device__ __forceinline__ bool grp_kept(const GrpBatch &B, int s, int64_t pos_off, int c) {
  const int kp = B.keep_pos[s];
  return kp >= 0 && B.keep_code[s] == c && (int64_t)kp - B.span_start[s] == pos_off;
}

// Fused partition copy: bytes [p0, p1) of src to dst in 16-byte windows (p0 16-byte aligned; a
// window may end past p1 only at the end of the buffer, which is padded), 8 windows in flight
// per thread: all loads issue before the first store waits on them.
__device__ __forceinline__ void copy_windows(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, int64_t p0,
                                             int64_t p1, int nt) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int kCopyUnroll = 8;
  for (int64_t D0 = p0 + 16 * (int)threadIdx.x; D0 < p1; D0 += 16 * kGrpThreads * kCopyUnroll) {
    u32x4 v[kCopyUnroll];
#pragma unroll
    for (int k = 0; k < kCopyUnroll; ++k) {
      const int64_t D = D0 + 16 * kGrpThreads * k;
      if (D < p1) v[k] = *reinterpret_cast<const u32x4 *>(src + D);
    }
#pragma unroll
    for (int k = 0; k < kCopyUnroll; ++k) {
      const int64_t D = D0 + 16 * kGrpThreads * k;
      if (D >= p1) break;
      if (nt) __builtin_nontemporal_store(v[k], reinterpret_cast<u32x4 *>(dst + D));
      else *reinterpret_cast<u32x4 *>(dst + D) = v[k];
    }
  }
}

// The staged tile's chunk map: the exclusive prefix of the records' chunk counts (nck: this
// thread's record) and the chunk -> record map; returns the tile's chunk total.
template <class SH>
__device__ __forceinline__ int grp_tile_map(SH &sh, int nck) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // wave inclusive scan: DPP row_shr within each 16-lane row, then the row totals (no lane-index
  // registers: shuffle index arithmetic hoisted out of the tile loop cost 9 VGPRs and spills)
  int incl = nck;
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xF, 0xF, false);   // row_shr:1
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xF, 0xF, false);   // row_shr:2
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xF, 0xF, false);   // row_shr:4
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xF, 0xF, false);   // row_shr:8
  {
    const int r0 = __builtin_amdgcn_readlane(incl, 15), r1 = __builtin_amdgcn_readlane(incl, 31),
              r2 = __builtin_amdgcn_readlane(incl, 47);
    const int row = lane >> 4;
    incl += (row >= 1 ? r0 : 0) + (row >= 2 ? r1 : 0) + (row >= 3 ? r2 : 0);
  }
  if (lane == 63) sh.wsum[wave] = incl;
  __syncthreads();
  int wbase = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kGrpThreads / 64; ++w) {
    const int v = sh.wsum[w];
    wbase += w < wave ? v : 0;
    total += v;
  }
  const int pre = wbase + incl - nck;
  sh.pre[tid] = pre;
  if (total <= kGrpMap)
    for (int k = 0; k < nck; ++k) sh.cmap[pre + k] = (uint8_t)tid;
  __syncthreads();
  return total;
}

// Stage records [c0, c0 + nh) in LDS with the exclusive prefix of their chunk counts;
// returns the tile's chunk total.
template <class SH>
__device__ __forceinline__ int grp_tile(SH &sh, const int4 *__restrict__ rec4, int64_t c0, int nh, int chunk) {
  const int tid = threadIdx.x;
  const int4 r = rec4[c0 + (tid < nh ? tid : nh - 1)];
  int nck = 0;
  if (tid < nh) {
    sh.rec[tid] = r;
    nck = ((((uint32_t)r.z >> 16) & kSegMaxLen) + chunk - 1) / chunk;
  }
  return grp_tile_map(sh, nck);
}

// ---- fused one-segment mode: records made in LDS ------------------------------------------
// A one-segment batch (every read at most one aligned segment) needs no record pass over HBM:
// k_prep_scan wrote a 16-byte descriptor per read (its segment's query nibble, contig position and
// length, dataset, write scope, ganon_batch.h), and each tile here turns incidences [c0, c0 + nh)
// into the records k_prep_emit_flat used to write — scope by binary search in the staged scope
// table, the span check, the write-scope mark (and, on the group's first pass, the incidence checks
// and the write-scope hash sum). The group's scopes sit in the patch list's LDS (unused while chunks
// stream; staged again before every pass, the classification reuses it), 16 bytes each. A tile reads
// the 2-bit reference unless one of its records lies in a scope whose reference span holds a
// non-ACGT block (the record pass decided this per group; both copies give the same bases where
// the 2-bit one is read).
struct FlatScope {
  int off;                  // first incidence, relative to the group's
  int sstart;               // span start
  unsigned long long pk;    // ref_off - span_start (42-bit signed) | min(span_len, 2^20 + 1) << 42 | dirty << 63
};
static_assert(sizeof(FlatScope) * kGrpMaxScopes <= sizeof(unsigned long long) * kGrpObs,
              "the scope table fits the patch list");

template <class SH>
__device__ __forceinline__ FlatScope *flat_scopes(SH &sh) {
  return reinterpret_cast<FlatScope *>(sh.patch);
}

// Scope s of a group whose incidences start at i_begin (a thread per scope: at most kGrpMaxScopes,
// the group's workgroup size).
static_assert(kGrpMaxScopes <= kGrpThreads, "one staging thread per scope of a group");
__device__ __forceinline__ FlatScope flat_load(const GrpBatch &B, const GrpAux *__restrict__ aux, int s, int64_t i_begin) {
  const int64_t off = aux->incid_off[s], ro = aux->ref_off[s];
  const int ss = B.span_start[s], sl = B.span_len[s];
  const bool dirty = aux->sdirty[s] != 0;   // (k_prep_scan)
  FlatScope f;
  f.off = (int)(off - i_begin);
  f.sstart = ss;
  f.pk = ((unsigned long long)(ro - ss) & ((1ull << 42) - 1)) | ((unsigned long long)min(sl, kGrpMaxSpan + 1) << 42) |
         ((unsigned long long)dirty << 63);
  return f;
}

template <class SH>
__device__ __forceinline__ int blk_excl_sum(SH &sh, int v, int *total);
template <class SH>
__device__ __attribute__((noinline)) int grp_xexpand(SH &sh, const GrpAux *__restrict__ aux, int64_t i_begin, int e0, int n_e,
                                           int base, int *n_rec, int s_begin, bool first);

// r: incidence c0 + tid's read (loaded a tile ahead by grp_scan_flat). last: the group's last
// incidence tile — when the further segments of the group's multi-segment reads fit in its free
// slots, they join it (merged: no extras tile after it); nh grows by their records.
template <class SH>
__device__ __forceinline__ int grp_tile_flat(SH &sh, const GrpBatch &B, const GrpAux *__restrict__ aux, int64_t c0,
                                             int &nh, int chunk, int s_begin, int ns, int64_t i_begin, bool first,
                                             int r, bool &clean, bool last, bool &merged) {
  const int tid = threadIdx.x;
  const FlatScope *sc = flat_scopes(sh);
  int nck = 0;
  bool dirty = false;
  unsigned long long hsum = 0;
  if (tid < nh) {
    const int64_t i = c0 + tid;
    const int il = (int)(i - i_begin);
    int lo = 0, hi = ns - 1;   // the incidence's scope: largest j with off[j] <= il
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sc[mid].off <= il) lo = mid;
      else hi = mid - 1;
    }
    const int j = lo;
    int4 rec = make_int4(0, 0, 0, j);   // zero length: no chunks
    if (r < 0 || r >= aux->n_reads) {
      if (first) report(aux->err, kErrIncidRead, i, r);
    } else {
      const int4 d = aux->desc[r];
      const FlatScope S = sc[j];
      const uint32_t z = (uint32_t)d.z;
      const int n = (int)((z >> 8) & kSegMaxLen), p = d.y;
      // (a multi-segment read: the first segment's end here, the read's end when its further
      // segments are expanded)
      const bool multi = (z & kDescMulti) != 0;
      const int nx = multi ? (int)((z >> 28) & 7) : 0;
      const uint64_t sq = (uint64_t)(uint32_t)d.x | ((uint64_t)(z & 0x7F) << 32);
      int rs, re;
      if (z & kDescWide) {
        rs = aux->ref_start[r];
        re = multi ? p + n : aux->read_end[r];
      } else {
        rs = p - (int)((z >> 24) & 15);
        re = p + n + (multi ? 0 : (int)(z >> 28));
      }
      int sl = (int)((S.pk >> 42) & ((1ull << 21) - 1));
      const bool huge = sl > kGrpMaxSpan;
      if (huge) sl = B.span_len[s_begin + j];
      if (rs < S.sstart || (int64_t)re > (int64_t)S.sstart + sl) {
        if (first) report(aux->err, kErrIncidSpan, s_begin + j, r);
      } else {
        const bool mine = d.w == s_begin + j;
        if (first && mine) hsum += ws_hash(r);
        if (!huge && n > 0) {
          const int64_t r0 = (int64_t)(S.pk << 22) >> 22;
          const uint64_t rf = (uint64_t)(r0 + p);
          if (first && nx) {   // its further segments: an entry in the group's list (streamed after the incidences)
            const int k = atomicAdd(&sh.n_xent, 1);
            atomicAdd(&sh.n_xrec, nx);
            aux->xlist[i_begin + k] = make_int2(r, (int)((uint32_t)j | ((uint32_t)nx << 12) | (((z >> 22) & 1u) << 15) |
                                                        (mine ? 0x80000000u : 0u)));
          }
          const uint32_t rz = (uint32_t)((sq >> 32) & 0x7F) | ((uint32_t)((rf >> 32) & 0xFF) << 8) |
                              ((uint32_t)n << 16) | (((z >> 22) & 1u) << 30) | (mine ? kSegMine : 0u);
          rec = make_int4((int)(uint32_t)sq, (int)(uint32_t)rf, (int)rz,
                          (int)((uint32_t)j | ((uint32_t)(p - S.sstart) << 12)));
          dirty = (S.pk >> 63) != 0;
          nck = (n + chunk - 1) / chunk;
        }
      }
    }
    sh.rec[tid] = rec;
  }
  if (first) {   // the tile's write-scope hashes into the group's sum (uniform branch)
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)hsum, o), hi = __shfl_xor((uint32_t)(hsum >> 32), o);
      hsum += ((unsigned long long)hi << 32) | lo;
    }
    if ((tid & 63) == 0 && hsum) atomicAdd(&sh.hsum, hsum);
  }
  if (last) {   // (uniform) the group's further segments into this tile's free slots when they fit
    if (first) __builtin_amdgcn_s_waitcnt(0);   // (this tile's entries at L2 before the barrier)
    __syncthreads();
    const int ne = sh.n_xent, nr = sh.n_xrec;
    if (ne && nh + nr <= kGrpTile) {
      int got;
      grp_xexpand(sh, aux, i_begin, 0, ne, nh, &got, s_begin, first);   // (every entry fits: ends on a barrier)
      if (tid >= nh && tid < nh + nr) {
        const int4 x = sh.rec[tid];
        nck = ((((uint32_t)x.z >> 16) & kSegMaxLen) + chunk - 1) / chunk;
        dirty = (flat_scopes(sh)[x.w & 0xFFF].pk >> 63) != 0;
      }
      nh += nr;
      merged = true;
    }
  }
  const unsigned long long dm = __ballot(dirty);
  if ((tid & 63) == 0) sh.wdirty[tid >> 6] = dm != 0ull;
  const int total = grp_tile_map(sh, nck);
  int any = 0;
#pragma unroll
  for (int w = 0; w < kGrpThreads / 64; ++w) any |= sh.wdirty[w];
  clean = any == 0;
  return total;
}

// The staged segment owning chunk t (largest j with pre[j] <= t).
template <class SH>
__device__ __forceinline__ int grp_find(const SH &sh, int nh, int total, int t) {
  if (total <= kGrpMap) return sh.cmap[t];
  int lo = 0, hi = nh - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (sh.pre[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// One chunk (16 * K bases) of staged record j: each thread loads the 2K + 1 sequence dwords and
// the K + 1 (2-bit) or 2K + 1 (nt16) reference dwords covering it at once (one memory round trip
// per chunk), then takes the K 16-base windows out of registers with static indices.
template <int K, bool REF2, class SH>
__device__ __forceinline__ void grp_chunk(const GrpBatch &B, SH &sh, const GrpRange &R, const GrpGlobal &gg, int t,
                                          int j) {
  {
    {
      const int4 r = sh.rec[j];
      const uint32_t rz = (uint32_t)r.z;
      const int L = (int)((rz >> 16) & kSegMaxLen);
      const int q0 = 16 * K * (t - sh.pre[j]);
      const int64_t sn = (int64_t)((uint64_t)(uint32_t)r.x | ((uint64_t)(rz & 0xFF) << 32)) + q0;
      const int64_t rn = (int64_t)((uint64_t)(uint32_t)r.y | ((uint64_t)((rz >> 8) & 0xFF) << 32)) + q0;
      const uint32_t *ps = reinterpret_cast<const uint32_t *>(B.seq) + (sn >> 3);
      const uint32_t *pr = REF2 ? B.ref2 + (rn >> 4) : reinterpret_cast<const uint32_t *>(B.ref) + (rn >> 3);
      constexpr int NR = REF2 ? K + 1 : 2 * K + 1;   // reference words covering the chunk
      uint32_t ds[2 * K + 1], dr[NR];
#pragma unroll
      for (int i = 0; i < 2 * K + 1; ++i) ds[i] = ps[i];
#pragma unroll
      for (int i = 0; i < NR; ++i) dr[i] = pr[i];
#pragma unroll
      for (int i = 0; i < 2 * K + 1; ++i) ds[i] = nib_swap(ds[i]);
      if (!REF2) {
#pragma unroll
        for (int i = 0; i < NR; ++i) dr[i] = nib_swap(dr[i]);
      }
      const int shs = 4 * (int)(sn & 7), shr = REF2 ? 2 * (int)(rn & 15) : 4 * (int)(rn & 7);
      const int ds_ = (int)((rz >> 30) & 1);
      const unsigned long long sk = (unsigned long long)(r.w & 0xFFF) << 52;
      const int pos_seg = (int)((uint32_t)r.w >> 12);
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int qi = q0 + 16 * i;
        if (qi >= L) break;
        const uint64_t xs0 = (uint64_t)ds[2 * i] | ((uint64_t)ds[2 * i + 1] << 32);
        const uint64_t xs1 = (uint64_t)ds[2 * i + 1] | ((uint64_t)ds[2 * i + 2] << 32);
        const uint64_t sv = (uint64_t)(uint32_t)(xs0 >> shs) | ((uint64_t)(uint32_t)(xs1 >> shs) << 32);
        uint64_t rv;
        if (REF2) {
          rv = expand2((uint32_t)((((uint64_t)dr[i]) | ((uint64_t)dr[i + 1] << 32)) >> shr));
        } else {
          const uint64_t xr0 = (uint64_t)dr[2 * i] | ((uint64_t)dr[2 * i + 1] << 32);
          const uint64_t xr1 = (uint64_t)dr[2 * i + 1] | ((uint64_t)dr[2 * i + 2] << 32);
          rv = (uint64_t)(uint32_t)(xr0 >> shr) | ((uint64_t)(uint32_t)(xr1 >> shr) << 32);
        }
        const int nb = (L - qi) < 16 ? (L - qi) : 16;
        uint64_t diff = sv ^ rv;
        diff = (diff | (diff >> 1) | (diff >> 2) | (diff >> 3)) & 0x1111111111111111ull;
        if (nb < 16) diff &= (1ull << (4 * nb)) - 1;
        while (diff) {
          const int k = __builtin_ctzll(diff) >> 2;
          diff &= diff - 1;
          const int c = (int)((sv >> (4 * k)) & 15);
          const int rc = (int)((rv >> (4 * k)) & 15);
          if (c == 15 || !is_acgt(rc)) continue;
          const unsigned long long key = sk | ((unsigned long long)(pos_seg + qi + k) << 4) | (unsigned long long)c;
          grp_observe(sh, R, gg, key, sn + 16 * i + k, rc, ds_, rz >> 31);
        }
      }
    }
  }
}

// Stream every chunk of every segment of the group, feeding observations in range R.
template <int K, bool REF2, class SH>
__device__ __forceinline__ void grp_scan(const GrpBatch &B, SH &sh, const GrpRange &R, const GrpGlobal &gg,
                                         int64_t i_begin, int64_t i_end, const int4 *__restrict__ rec4, int skip) {
  const int tid = threadIdx.x;
  for (int64_t c0 = i_begin; c0 < i_end; c0 += kGrpTile) {
    const int nh = (int)((i_end - c0) < kGrpTile ? (i_end - c0) : kGrpTile);
    int total = grp_tile(sh, rec4, c0, nh, 16 * K);
    if (skip & kSkipChunks) total = 0;
    for (int t = tid; t < total; t += kGrpThreads) {
      const int j = grp_find(sh, nh, total, t);
      grp_chunk<K, REF2>(B, sh, R, gg, t, j);
    }
    __syncthreads();
  }
}

// Long-read mode: slots [c0, c0 + nh) of a group whose incidences are [inc0, inc0 + n_inc): the
// incidence owning slot t (largest first slot <= t: incidences without records share their
// successor's first slot and lose to it), its read's record t - first slot, completed with the
// scope's fields from the staged scope table (reference offset, span start, reference flag) and
// the incidence's write mark. A tile of a 10-100 kb read's incidence reads 256 consecutive read
// records (one coalesced load). long_fetch issues a tile's loads; grp_scan_long issues the next
// tile's before it streams the current one, so their latency overlaps the chunk loads.
// itab: the group's incidence records staged in LDS after the scope table (ns + n_inc <= the
// table's 256 entries: every C5 group), else null (looked up in global memory).
struct LongFetch {
  int4 rr;   // the read record
  int iy;    // the incidence record's y: scope local | mine << 31
};

__device__ __forceinline__ LongFetch long_fetch(const GrpAux *__restrict__ aux, int64_t c0, int nh, int64_t inc0,
                                                int n_inc, const int4 *itab) {
  LongFetch f{make_int4(0, 0, 0, 0), 0};
  const int tid = threadIdx.x;
  if (tid < nh) {
    const int64_t t = c0 + tid;
    const int4 *it = itab ? itab : aux->inc4 + inc0;
    int lo = 0, hi = n_inc - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int64_t)it[mid].x <= t) lo = mid;
      else hi = mid - 1;
    }
    const int4 I = it[lo];
    const int64_t rb = (int64_t)((uint64_t)(uint32_t)I.z | ((uint64_t)(uint32_t)I.w << 32));
    f.rr = aux->rrec[rb + (t - (int64_t)(uint32_t)I.x)];
    f.iy = I.y;
  }
  return f;
}

template <class SH>
__device__ __forceinline__ int grp_tile_long(SH &sh, const LongFetch &F, int nh, int chunk, bool &clean) {
  const int tid = threadIdx.x;
  const FlatScope *sc = flat_scopes(sh);
  int nck = 0;
  bool dirty = false;
  if (tid < nh) {
    const int j = F.iy & 0xFFF;
    const FlatScope S = sc[j];
    const uint32_t z = (uint32_t)F.rr.z;
    const int n = (int)((z >> 16) & kSegMaxLen), p = F.rr.y;
    const int64_t r0 = (int64_t)(S.pk << 22) >> 22;
    const uint64_t rf = (uint64_t)(r0 + p);
    const uint32_t rz = (z & 0xFFu) | ((uint32_t)((rf >> 32) & 0xFF) << 8) | ((uint32_t)n << 16) | (z & (1u << 30)) |
                        ((uint32_t)F.iy & kSegMine);
    sh.rec[tid] = make_int4(F.rr.x, (int)(uint32_t)rf, (int)rz, (int)((uint32_t)j | ((uint32_t)(p - S.sstart) << 12)));
    dirty = (S.pk >> 63) != 0;
    nck = (n + chunk - 1) / chunk;
  }
  const unsigned long long dm = __ballot(dirty);
  if ((tid & 63) == 0) sh.wdirty[tid >> 6] = dm != 0ull;
  const int total = grp_tile_map(sh, nck);
  int any = 0;
#pragma unroll
  for (int w = 0; w < kGrpThreads / 64; ++w) any |= sh.wdirty[w];
  clean = any == 0;
  return total;
}

template <int K, class SH>
__device__ __forceinline__ void grp_scan_long(const GrpBatch &B, SH &sh, const GrpRange &R, const GrpGlobal &gg,
                                              const GrpAux *__restrict__ aux, int64_t i_begin, int64_t i_end,
                                              int64_t inc0, int n_inc, const int4 *itab, int skip) {
  const int tid = threadIdx.x;
  const auto tile_n = [&](int64_t c0) { return (int)((i_end - c0) < kGrpTile ? (i_end - c0) : kGrpTile); };
  LongFetch next = i_begin < i_end ? long_fetch(aux, i_begin, tile_n(i_begin), inc0, n_inc, itab) : LongFetch{};
  for (int64_t c0 = i_begin; c0 < i_end; c0 += kGrpTile) {
    const int nh = tile_n(c0);
    const LongFetch cur = next;
    if (c0 + kGrpTile < i_end) next = long_fetch(aux, c0 + kGrpTile, tile_n(c0 + kGrpTile), inc0, n_inc, itab);
    bool clean;
    int total = grp_tile_long(sh, cur, nh, 16 * K, clean);
    if (skip & kSkipChunks) total = 0;
    if (clean && B.ref2) {
      for (int t = tid; t < total; t += kGrpThreads) grp_chunk<K, true>(B, sh, R, gg, t, grp_find(sh, nh, total, t));
    } else {
      for (int t = tid; t < total; t += kGrpThreads) grp_chunk<K, false>(B, sh, R, gg, t, grp_find(sh, nh, total, t));
    }
    __syncthreads();
  }
}

template <int K, class SH>
__device__ __forceinline__ void grp_scan_extra(const GrpBatch &B, SH &sh, const GrpRange &R,
                                                         const GrpGlobal &gg, const GrpAux *__restrict__ aux,
                                                         int64_t i_begin, int n_e, int skip, int s_begin, bool first);

// Fused one-segment mode: the same stream over records made from incidences [i_begin, i_end) tile
// by tile (grp_tile_flat), each tile through the 2-bit reference when all of its records allow.
template <int K, class SH>
__device__ __forceinline__ void grp_scan_flat(const GrpBatch &B, SH &sh, const GrpRange &R, const GrpGlobal &gg,
                                              const GrpAux *__restrict__ aux, int64_t i_begin, int64_t i_end,
                                              int s_begin, int ns, bool first, int skip) {
  const int tid = threadIdx.x;
  // each tile's incidence reads are loaded while the previous tile streams (one dependent load,
  // the descriptor, left per tile); the first tile's by the caller (staged in sh.rec[tid].x)
  int r_next = sh.rec[tid].x;
  bool merged = false;
  for (int64_t c0 = i_begin; c0 < i_end; c0 += kGrpTile) {
    const int nh = (int)((i_end - c0) < kGrpTile ? (i_end - c0) : kGrpTile);
    const int r = r_next;
    const int64_t in = c0 + kGrpTile + tid;
    r_next = in < i_end ? aux->incid_read[in] : -1;
    bool clean;
    int nt = nh;   // (the last tile may take the extras records too)
    int total = grp_tile_flat(sh, B, aux, c0, nt, 16 * K, s_begin, ns, i_begin, first, r, clean, c0 + kGrpTile >= i_end,
                              merged);
    if (skip & kSkipChunks) total = 0;
    if (clean && B.ref2) {
      for (int t = tid; t < total; t += kGrpThreads) grp_chunk<K, true>(B, sh, R, gg, t, grp_find(sh, nt, total, t));
    } else {
      for (int t = tid; t < total; t += kGrpThreads) grp_chunk<K, false>(B, sh, R, gg, t, grp_find(sh, nt, total, t));
    }
    __syncthreads();
  }
  // multi-segment reads (short reads with an I/D/N op): their further segments, from the entries the
  // first pass listed — a segment's observations are those of any other record of its scope, so they
  // may come after the incidences: in the last tile's free slots (merged), else in extras tiles
  if (merged) return;
  if (first) {   // (the entries' stores at L2 before any thread reads them back)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  const int n_e = sh.n_xent;
  if (n_e) grp_scan_extra<K>(B, sh, R, gg, aux, i_begin, n_e, skip, s_begin, first);
}

// Block-wide exclusive prefix sum of v (every thread calls; ends on a barrier); *total = the sum.
template <class SH>
__device__ __forceinline__ int blk_excl_sum(SH &sh, int v, int *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int incl = ganon_wave::incl_sum(v);
  if (lane == 63) sh.wsum[wave] = incl;
  __syncthreads();
  int base = 0, t = 0;
#pragma unroll
  for (int w = 0; w < kGrpThreads / 64; ++w) {
    const int x = sh.wsum[w];
    base += w < wave ? x : 0;
    t += x;
  }
  *total = t;
  __syncthreads();   // (sh.wsum is free again)
  return base + incl - v;
}

// The fused mode's extras tiles: the group's n_e entries (an incidence of a multi-segment read each:
// its read's extras index, scope, further segments, dataset, write mark) expanded into the records
// of their further segments, as many whole entries per tile as fit its kGrpTile records (an entry
// has at most kFusedMaxSeg - 1), then streamed like any tile.
// Entries [e0, e0 + min(n_e - e0, kGrpTile)) of the group's list expanded into the records of their
// further segments at sh.rec[base + ...]: as many whole entries as fit the tile (every entry has 1 to
// kFusedMaxSeg - 1 records, so the fitting ones are a prefix). Returns the entries taken; *n_rec = the
// records written. Every thread calls; ends on a barrier.
template <class SH>
__device__ __attribute__((noinline)) int grp_xexpand(SH &sh, const GrpAux *__restrict__ aux, int64_t i_begin, int e0, int n_e,
                                           int base, int *n_rec, int s_begin, bool first) {
  const int tid = opaque_tid();
  const FlatScope *sc = flat_scopes(sh);
  const unsigned long long *xl = reinterpret_cast<const unsigned long long *>(aux->xlist) + i_begin;
  const int m = min(n_e - e0, kGrpTile);
  unsigned long long ent = 0;
  if (tid < m) ent = ld_l2(xl + e0 + tid);   // (written by this workgroup's first pass: read past L1)
  const uint32_t ey = (uint32_t)(ent >> 32);
  const int nx = tid < m ? (int)((ey >> 12) & 7) : 0;
  int total;
  const int pre = base + blk_excl_sum(sh, nx, &total);
  const bool fit = tid < m && pre + nx <= kGrpTile;
  if (fit) {
    const int j = (int)(ey & 0xFFF);
    const FlatScope S = sc[j];
    const int64_t r0 = (int64_t)(S.pk << 22) >> 22;
    const int r = (int)(uint32_t)ent;
    const uint32_t xi = (uint32_t)aux->xidx[r];
    const uint32_t hi = (((ey >> 15) & 1u) << 30) | (ey & kSegMine);
    // the read's span check (the tile checked its first segment's end only): a read reaching past
    // its scope's span is the batch's error, and its further segments stream nothing
    const int4 h = aux->xrec[xi];
    const int sl = (int)((S.pk >> 42) & ((1ull << 21) - 1));   // (entries are never made in huge scopes)
    const bool in_span = h.x >= S.sstart && (int64_t)h.y <= (int64_t)S.sstart + sl;
    if (!in_span && first) report(aux->err, kErrIncidSpan, s_begin + j, r);
    for (int k = 0; k < nx; ++k) {
      const int4 e = aux->xrec[xi + 1 + k];
      const uint32_t z = (uint32_t)e.z;
      const int n = in_span ? (int)((z >> 8) & kSegMaxLen) : 0, p = e.y;
      const uint64_t rf = (uint64_t)(r0 + p);
      const uint32_t rz = (z & 0x7Fu) | ((uint32_t)((rf >> 32) & 0xFF) << 8) | ((uint32_t)n << 16) | hi;
      sh.rec[pre + k] = make_int4(e.x, (int)(uint32_t)rf, (int)rz, (int)((uint32_t)j | ((uint32_t)(p - S.sstart) << 12)));
    }
  }
  const int used = __syncthreads_count(fit);
  if (fit && tid == used - 1) sh.n_xtile = pre + nx - base;
  __syncthreads();
  *n_rec = sh.n_xtile;
  return used;
}

// The fused mode's extras tiles (the further segments that did not fit the group's last tile): the
// group's n_e entries (an incidence of a multi-segment read each: its read's extras index, scope,
// further segments, dataset, write mark) expanded tile by tile, then streamed like any tile.
template <int K, class SH>
__device__ __forceinline__ void grp_scan_extra(const GrpBatch &B, SH &sh, const GrpRange &R,
                                                         const GrpGlobal &gg, const GrpAux *__restrict__ aux,
                                                         int64_t i_begin, int n_e, int skip, int s_begin, bool first) {
  const int tid = opaque_tid();
  const FlatScope *sc = flat_scopes(sh);
  for (int e0 = 0; e0 < n_e;) {
    int nh;
    const int used = grp_xexpand(sh, aux, i_begin, e0, n_e, 0, &nh, s_begin, first);
    int nck = 0;
    bool dirty = false;
    if (tid < nh) {
      const int4 r = sh.rec[tid];
      nck = ((((uint32_t)r.z >> 16) & kSegMaxLen) + 16 * K - 1) / (16 * K);
      dirty = (sc[r.w & 0xFFF].pk >> 63) != 0;
    }
    const bool clean = !__syncthreads_or(dirty);
    int tot = grp_tile_map(sh, nck);
    if (skip & kSkipChunks) tot = 0;
    if (clean && B.ref2) {
      for (int t = tid; t < tot; t += kGrpThreads) grp_chunk<K, true>(B, sh, R, gg, t, grp_find(sh, nh, tot, t));
    } else {
      for (int t = tid; t < tot; t += kGrpThreads) grp_chunk<K, false>(B, sh, R, gg, t, grp_find(sh, nh, tot, t));
    }
    __syncthreads();
    e0 += used;
  }
}

// In-LDS bitonic sort of n keys (n <= capacity rounded to a power of two); optional payload.
__device__ __forceinline__ void lds_bitonic(unsigned long long *key, unsigned long long *pay, int n) {
  const int tid = threadIdx.x;
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (int i = n + tid; i < n2; i += kGrpThreads) key[i] = ~0ull;
  __syncthreads();
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < n2; i += kGrpThreads) {
        const int ixj = i ^ j;
        if (ixj <= i) continue;
        const unsigned long long a = key[i], b = key[ixj];
        if ((a > b) == ((i & k) == 0)) {
          key[i] = b;
          key[ixj] = a;
          if (pay) {
            const unsigned long long p = pay[i];
            pay[i] = pay[ixj];
            pay[ixj] = p;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Observation list -> calls. Up to kGrpQuad observations every thread matches its own
// observation against the whole list (no sort, no barrier); longer lists are sorted and one
// thread takes each run of equal keys. count: add calls/bases to the per-scope and workgroup
// totals (off for a re-run that only re-applies masks).
template <class SH>
__device__ __forceinline__ void grp_count(SH &sh, int s_local, int calls, int bases) {
  if (calls) {
    atomicAdd(&sh.cnt_calls[s_local], calls);
    atomicAdd(&sh.blk_calls, calls);
  }
  if (bases) {
    atomicAdd(&sh.cnt_bases[s_local], bases);
    atomicAdd(&sh.blk_bases, bases);
  }
}

template <class SH>
__device__ __forceinline__ void grp_classify(const GrpBatch &B, SH &sh, int n, int s_begin,
                                             const PatchSink &sink, bool count) {
  const int tid = threadIdx.x;
  if (n <= kGrpQuad) {
    if (tid >= n) return;
    const unsigned long long key = sh.key[tid];
    int seen = 0;
    bool head = true;
    for (int j = 0; j < n; ++j) {
      if (sh.key[j] != key) continue;
      seen |= 1 << ((sh.pay[j] >> 52) & 1);
      head &= j >= tid;
    }
    if (seen != 3) return;
    const int s = s_begin + (int)(key >> 52);
    const int c = (int)(key & 15);
    if (grp_kept(B, s, (int64_t)((key >> 4) & kNibMask), c)) return;
    const unsigned long long p = sh.pay[tid];
    const int mine = (int)((p >> 53) & 1);
    if (mine) sink_patch(sh, sink, (int64_t)(p & kNibMask), c, (int)((p >> 48) & 15));
    if (count) grp_count(sh, s - s_begin, head ? 1 : 0, mine);
    return;
  }
  lds_bitonic(sh.key, sh.pay, n);
  for (int i = tid; i < n; i += kGrpThreads) {
    const unsigned long long key = sh.key[i];
    if (i > 0 && sh.key[i - 1] == key) continue;
    int e = i, seen = 0;
    while (e < n && sh.key[e] == key) seen |= 1 << ((sh.pay[e++] >> 52) & 1);
    if (seen != 3) continue;
    const int s = s_begin + (int)(key >> 52);
    const int c = (int)(key & 15);
    if (grp_kept(B, s, (int64_t)((key >> 4) & kNibMask), c)) continue;
    int masked = 0;
    for (int x = i; x < e; ++x) {
      const unsigned long long p = sh.pay[x];
      if (!((p >> 53) & 1)) continue;
      sink_patch(sh, sink, (int64_t)(p & kNibMask), c, (int)((p >> 48) & 15));
      ++masked;
    }
    if (count) grp_count(sh, s - s_begin, 1, masked);
  }
}

// An overflowing list (n > OBS: OBS in LDS, the rest in the group's global region) filtered by the
// pass's Bloom bitmaps: the LDS list is compacted in place to its keys seen in both datasets (a key
// seen in one can never be a TN call; the bitmaps have no false negatives), the region's surviving
// observations are appended after it as far as OBS. Returns all survivors; sh.n_obs = the LDS
// list's. The region itself is left as it was.
template <class SH>
__device__ __attribute__((noinline)) int grp_filter(SH &sh, const GrpGlobal &gg, int n) {
  constexpr int kPer = SH::kObs / kGrpThreads;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  GU64 *okey = gp(gg.aux->okey) + gg.off, *opay = gp(gg.aux->opay) + gg.off;
  uint32_t *bloom = bloom_of(sh);
  for (int i = tid; i < 2 * kBloomBits / 32; i += kGrpThreads) bloom[i] = 0u;
  __builtin_amdgcn_s_waitcnt(0);   // the scan's region stores at L2
  __syncthreads();
  // the bitmaps: every stored observation's key, by dataset (payload bit 52)
  for (int i = opaque_tid(); i < n; i += kGrpThreads) {
    const unsigned long long key = i < SH::kObs ? sh.key[i] : ld_l2(okey + (i - SH::kObs));
    const unsigned long long pay = i < SH::kObs ? sh.pay[i] : ld_l2(opay + (i - SH::kObs));
    const uint32_t h = (bloom_hash(key) & (kBloomBits - 1)) + (uint32_t)((pay >> 52) & 1) * kBloomBits;
    atomicOr(bloom + (h >> 5), 1u << (h & 31));
  }
  __syncthreads();
  unsigned long long k[kPer], p[kPer];
  bool keep[kPer];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int i = tid + j * kGrpThreads;
    k[j] = sh.key[i];
    p[j] = sh.pay[i];
    keep[j] = bloom_both(sh, k[j]);
    cnt += keep[j] ? 1 : 0;
  }
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int x = __shfl_up(incl, o);
    if (lane >= o) incl += x;
  }
  if (lane == 63) sh.wsum[wave] = incl;
  if (tid == 0) sh.n_filt = 0;
  __syncthreads();   // (every thread holds its entries: the list can be rewritten)
  int base = incl - cnt, total = 0;
#pragma unroll
  for (int w = 0; w < kGrpThreads / 64; ++w) {
    const int v = sh.wsum[w];
    base += w < wave ? v : 0;
    total += v;
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if (keep[j]) {
      sh.key[base] = k[j];
      sh.pay[base] = p[j];
      ++base;
    }
  if (tid == 0) sh.n_obs = total;
  for (int i = opaque_tid(); i < n - SH::kObs; i += kGrpThreads) {
    const unsigned long long key = ld_l2(okey + i);
    if (!bloom_both(sh, key)) continue;
    const int slot = total + atomicAdd(&sh.n_filt, 1);
    if (slot < SH::kObs) {
      sh.key[slot] = key;
      sh.pay[slot] = ld_l2(opay + i);
    }
  }
  __syncthreads();
  return total + sh.n_filt;
}

// Overflow path: n observations of one key range sit in the group's global region. Aggregate
// them in a hash table of distinct keys (workgroup-scope atomics in L2), count the TN calls
// (minus the kept variant), and mask the observations of reads the scopes write.
template <class SH>
__device__ __forceinline__ void grp_global(const GrpBatch &B, SH &sh, const GrpGlobal &gg, int n,
                                           int s_begin, const PatchSink &sink) {
  const int tid = opaque_tid();
  const int tsize = max(2 * n, 64);
  GU64 *tk = gp(gg.aux->tkey) + 2 * gg.off;
  GU32 *tf = gp(gg.aux->tflag) + 2 * gg.off;
  GU64 *okey = gp(gg.aux->okey) + gg.off, *opay = gp(gg.aux->opay) + gg.off;
  for (int i = tid; i < tsize; i += kGrpThreads) {
    tk[i] = kEmpty;
    tf[i] = 0;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = tid; i < n; i += kGrpThreads) {
    const unsigned long long key = ld_l2(okey + i);
    const int ds = (int)((ld_l2(opay + i) >> 52) & 1);
    unsigned slot = gtab_home(key, tsize);
    for (int probe = 0; probe < tsize; ++probe) {
      unsigned long long expected = kEmpty;
      __hip_atomic_compare_exchange_strong(tk + slot, &expected, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
      if (expected == kEmpty || expected == key) {
        __hip_atomic_fetch_or(tf + slot, 1u << ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      if (++slot == (unsigned)tsize) slot = 0;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  // calls: one per TN slot
  for (int i = tid; i < tsize; i += kGrpThreads) {
    const unsigned long long key = ld_l2(tk + i);
    if (key == kEmpty || ld_l2(tf + i) != 3) continue;
    const int c = (int)(key & 15);
    if (grp_kept(B, s_begin + (int)(key >> 52), (int64_t)((key >> 4) & kNibMask), c)) continue;
    grp_count(sh, (int)(key >> 52), 1, 0);
  }
  // masks: every observation of a read the scope writes whose key is TN
  for (int i = tid; i < n; i += kGrpThreads) {
    const unsigned long long pay = ld_l2(opay + i);
    if (!((pay >> 53) & 1)) continue;
    const unsigned long long key = ld_l2(okey + i);
    unsigned slot = gtab_home(key, tsize);
    unsigned int f = 0;
    for (int probe = 0; probe < tsize; ++probe) {
      const unsigned long long k = ld_l2(tk + slot);
      if (k == key) {
        f = ld_l2(tf + slot);
        break;
      }
      if (k == kEmpty) break;
      if (++slot == (unsigned)tsize) slot = 0;
    }
    if (f != 3) continue;
    const int c = (int)(key & 15);
    if (grp_kept(B, s_begin + (int)(key >> 52), (int64_t)((key >> 4) & kNibMask), c)) continue;
    grp_count(sh, (int)(key >> 52), 0, 1);
    const int64_t nib = (int64_t)(pay & kNibMask);
    const int rc = (int)((pay >> 48) & 15);
    if (!sink.fused || !sink.inside(nib >> 1)) {
      PatchSink direct = sink;
      direct.lds = false;
      sink_patch(sh, direct, nib, c, rc);
      continue;
    }
    okey[i] = ((unsigned long long)nib << 4) | (unsigned long long)(c ^ rc);   // in-partition mask
    opay[i] = pay | (1ull << 54);
  }
  if (!sink.fused) return;
  // fused: merge the in-partition masks per byte (the table area again, keyed by byte) and
  // apply each byte once, out[b] ^= mask — only this workgroup writes its partition
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = tid; i < tsize; i += kGrpThreads) {
    tk[i] = kEmpty;
    tf[i] = 0;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = tid; i < n; i += kGrpThreads) {
    const unsigned long long e = ld_l2(okey + i);
    const unsigned long long pay = ld_l2(opay + i);
    if (!((pay >> 54) & 1)) continue;                       // no in-partition mask
    const unsigned long long byte = e >> 5;
    unsigned slot = gtab_home(byte, tsize);
    for (int probe = 0; probe < tsize; ++probe) {
      unsigned long long expected = kEmpty;
      __hip_atomic_compare_exchange_strong(tk + slot, &expected, byte, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
      if (expected == kEmpty || expected == byte) {
        __hip_atomic_fetch_xor(tf + slot, (unsigned)(e & 15) << (((e >> 4) & 1) ? 0 : 4), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      if (++slot == (unsigned)tsize) slot = 0;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = tid; i < tsize; i += kGrpThreads) {
    const unsigned long long byte = ld_l2(tk + i);
    if (byte == kEmpty) continue;
    const unsigned w = ld_l2(reinterpret_cast<const unsigned int *>(sink.out) + (byte >> 2));
    sink.out[byte] = (uint8_t)((w >> (8 * (byte & 3))) ^ ld_l2(tf + i));
  }
  __builtin_amdgcn_s_waitcnt(0);
}

// Fused: apply the sorted in-partition list (nibble << 4 | from ^ to) with one plain byte store
// per masked byte, out[b] ^ mask — the partition copy and earlier masks of that byte were
// stored by this workgroup and have drained (read back from L2).
template <class SH>
__device__ __forceinline__ void grp_patch_bytes(const GrpBatch &B, SH &sh, int np, uint8_t *out) {
  for (int i = threadIdx.x; i < np; i += kGrpThreads) {
    const unsigned long long e = sh.patch[i];
    const int64_t byte = (int64_t)(e >> 5);
    if (i > 0 && (int64_t)(sh.patch[i - 1] >> 5) == byte) continue;
    uint32_t x = 0;
    for (int k = i; k < np && (int64_t)(sh.patch[k] >> 5) == byte; ++k) {
      const unsigned long long f = sh.patch[k];
      x ^= (uint32_t)(f & 15) << (((f >> 4) & 1) ? 0 : 4);
    }
    const unsigned w = ld_l2(reinterpret_cast<const unsigned int *>(out) + (byte >> 2));
    out[byte] = (uint8_t)((w >> (8 * (byte & 3))) ^ x);
  }
}

// groups: kGrpRec x int4 per group, in launch order: {s_begin, s_end, seg_begin lo, hi},
// {seg_end lo, hi, seg_mid lo, hi}, {partition piece A begin lo, hi, end lo, hi} (bytes; fused
// only), {global region offset lo, hi, capacity, 0}, {piece B begin lo, hi, end lo, hi};
// segments [seg_begin, seg_mid) have an all-ACGT reference range (2-bit reference).
// FLAT: fused one-segment mode (records from incidences and read descriptors, grp_tile_flat; rec4
// unused; group record 1's mid ignored). LONG: long-read mode (records from the read records and
// incidence records, grp_tile_long; rec4 unused).
template <int U, bool FUSED, int OBS, bool FLAT, bool LONG = false>
__global__ void __launch_bounds__(kGrpThreads, (OBS > 512 ? 4 : U == 1 ? 6 : U == 2 ? GANON_K2_BLOCKS : U == 4 ? 5 : 4)) k_group(const GrpBatch B, const int4 *__restrict__ groups,
                                                       const int4 *__restrict__ rec4,
                                                       uint8_t *__restrict__ out, const GrpAux *__restrict__ aux,
                                                       int skip, int nt_copy, const unsigned long long *__restrict__ gate,
                                                       const int32_t *__restrict__ order) {
  __shared__ GrpSharedT<OBS> sh;
  const int tid = threadIdx.x;
  // the group this block runs: order[] (k_prep_order, longest first) when the batch has groups of
  // very unequal cost, else blockIdx (order[0] = -1); partials stay at the block's own slot
  int gid = blockIdx.x;
  if (order) {
    const int o0 = order[0];
    if (o0 >= 0) gid = blockIdx.x ? order[blockIdx.x] : o0;
  }
  // one-segment mode launches for the group bound: blocks past the scan's count (gate[5]) add
  // nothing; no block runs on a batch the scan rejected (gate[7])
  if (gate && (gate[7] || (unsigned long long)gid >= gate[5])) {
    if (tid == 0) {
      gp(aux->part)[2 * blockIdx.x] = 0;
      gp(aux->part)[2 * blockIdx.x + 1] = 0;
    }
    return;
  }
  const int4 g0 = groups[kGrpRec * gid];
  const int4 g1 = groups[kGrpRec * gid + 1];
  const int4 g2 = groups[kGrpRec * gid + 2];
  const int4 g3 = groups[kGrpRec * gid + 3];
  const int4 g4 = groups[kGrpRec * gid + 4];
  const GrpGlobal gg{aux, i64_of(g3.x, g3.y), g3.z};
  const int s_begin = g0.x, s_end = g0.y;
  const int64_t i_begin = i64_of(g0.z, g0.w), i_end = i64_of(g1.x, g1.y), i_mid = i64_of(g1.z, g1.w);
  const PatchSink sink{out, i64_of(g2.x, g2.y), i64_of(g2.z, g2.w), i64_of(g4.x, g4.y), i64_of(g4.z, g4.w),
                       aux, FUSED, FUSED};
  // the partition pieces, whole 16-byte windows (the buffers are padded past seq_bytes); the
  // stores drain while the scan runs (s_waitcnt before the mask stores). (Copying tile by tile,
  // each time up to the tile's written reads so that the scan's loads hit L2, read 0.34 GB less
  // per c2 launch but took 0.55 instead of 0.54 ms in the same build: DESIGN 5. Round 4 tried it
  // again in the fused one-segment kernel, each tile first copying the piece up to its last segment
  // byte: 0.665-0.679 vs 0.618 ms per pipelined c2 step, profiles/r04/tile_copy_ab.)
  // (FLAT: the first pass's scope table and first tile's reads are loaded before the copy, which
  // hides their latency)
  FlatScope fs{};
  int r_first = -1;
  int4 inc_rec{};   // (LONG) this thread's incidence record, staged after the scope table
  const bool inc_lds = LONG && (s_end - s_begin) + g3.w <= kGrpMaxScopes;
  if constexpr (FLAT || LONG) {
    if (tid < s_end - s_begin) fs = flat_load(B, aux, s_begin + tid, i_begin);
  }
  if constexpr (LONG) {
    if (inc_lds && tid < g3.w) inc_rec = aux->inc4[i_mid + tid];
  }
  if constexpr (FLAT) {
    if (i_begin + tid < i_end) r_first = aux->incid_read[i_begin + tid];
  }
  if (FUSED && !(skip & kSkipCopy)) {
    copy_windows(B.seq, out, sink.p0, sink.p1, nt_copy);
    copy_windows(B.seq, out, sink.q0, sink.q1, nt_copy);
  }
  // (staged for the first pass now: registers carried into the pass loop would stay live through
  // the classification and spill)
  if constexpr (FLAT || LONG) {
    if (tid < s_end - s_begin) flat_scopes(sh)[tid] = fs;
  }
  if constexpr (LONG) {
    if (inc_lds && tid < g3.w) reinterpret_cast<int4 *>(flat_scopes(sh) + (s_end - s_begin))[tid] = inc_rec;
  }
  if constexpr (FLAT) sh.rec[tid].x = r_first;   // (read by the first tile before it writes sh.rec)
  if (tid == 0) {
    sh.top = 0;
    sh.stk_lo[0] = 0ull;
    sh.stk_hi[0] = ~0ull;
    sh.stk_mode[0] = kModeCollect;
    sh.n_patch = 0;
    sh.blk_calls = 0;
    sh.blk_bases = 0;
    sh.hsum = 0;
    sh.n_xent = 0;
    sh.n_xrec = 0;
  }
  for (int i = tid; i < kGrpMaxScopes; i += kGrpThreads) {
    sh.cnt_calls[i] = 0;
    sh.cnt_bases[i] = 0;
  }
  bool first = true;   // (FLAT) the group's first pass makes the incidence checks and the hash sum
  for (;;) {
    __syncthreads();
    const int top = sh.top;
    if (top < 0) {
      // per-scope counts (wide scopes in the id range belong to the tile path) and the
      // workgroup's partial totals (k_finish sums them)
      for (int i = opaque_tid(); i < ((skip & kSkipCounts) ? 0 : s_end - s_begin); i += kGrpThreads) {
        if (B.span_len[s_begin + i] > kGrpMaxSpan) continue;
        gp(aux->scope_calls)[s_begin + i] = sh.cnt_calls[i];
        gp(aux->scope_bases)[s_begin + i] = sh.cnt_bases[i];
      }
      if (tid == 0) {
        gp(aux->part)[2 * blockIdx.x] = sh.blk_calls;
        gp(aux->part)[2 * blockIdx.x + 1] = sh.blk_bases;
        if (FLAT) gp(aux->ws_part)[gid] = sh.hsum;
      }
      break;
    }
    const GrpRange R{sh.stk_lo[top], sh.stk_hi[top], sh.stk_mode[top]};
    __syncthreads();
    if (tid == 0) {
      sh.top = top - 1;
      sh.n_obs = 0;
      sh.kmin = ~0ull;
      sh.kmax = 0ull;
    }
    __syncthreads();
    if constexpr (FLAT) {
      // the scope table (patch list space: the previous pass's classification is done with it)
      if (!first) {   // (staged again: a pass after a key-range split)
        if (tid < s_end - s_begin) flat_scopes(sh)[tid] = flat_load(B, aux, s_begin + opaque_tid(), i_begin);
        sh.rec[tid].x = i_begin + tid < i_end ? aux->incid_read[i_begin + opaque_tid()] : -1;
      }
      __syncthreads();
      grp_scan_flat<U>(B, sh, R, gg, aux, i_begin, i_end, s_begin, s_end - s_begin, first, skip);
      first = false;
    } else if constexpr (LONG) {
      const int ns = s_end - s_begin;
      int4 *itab = reinterpret_cast<int4 *>(flat_scopes(sh) + ns);
      if (!first) {   // (staged again: a pass after a key-range split)
        if (tid < ns) flat_scopes(sh)[tid] = flat_load(B, aux, s_begin + opaque_tid(), i_begin);
        if (inc_lds && tid < g3.w) itab[tid] = aux->inc4[i_mid + opaque_tid()];
      }
      __syncthreads();
      // (i_mid: the group's first incidence, g3.w: its incidence count)
      grp_scan_long<U>(B, sh, R, gg, aux, i_begin, i_end, i_mid, g3.w, inc_lds ? itab : nullptr, skip);
      first = false;
    } else if (B.ref2) {
      grp_scan<U, true>(B, sh, R, gg, i_begin, i_mid, rec4, skip);
      grp_scan<U, false>(B, sh, R, gg, i_mid, i_end, rec4, skip);
    } else {
      grp_scan<U, false>(B, sh, R, gg, i_begin, i_end, rec4, skip);
    }
    // (grp_scan ends on a barrier)
    if (skip & kSkipClassify) continue;
    int n = sh.n_obs;
    if (tid == 0 && n > kGrpQuad)   // path counters (ganon_batch_path_counts): sorted list, region, split
      __hip_atomic_fetch_add(gp(aux->paths) + (n <= OBS ? 0 : n <= gg.cap ? 1 : 2), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n > OBS) {
      if (n <= gg.cap) {
        // drop the observations whose key was not seen in both datasets (Bloom bitmaps): when the
        // rest fits in the LDS list, it is classified there like a short list
        const int m = GANON_GRP_BLOOM ? grp_filter(sh, gg, n) : OBS + 1;
        if (m <= OBS) {
          if (tid == 0)   // (counted as a region pass above too)
            __hip_atomic_fetch_add(gp(aux->paths) + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          grp_classify(B, sh, m, s_begin, sink, true);
          if (sink.lds) {
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            const int np = sh.n_patch;
            if (np) {
              lds_bitonic(sh.patch, nullptr, np);
              grp_patch_bytes(B, sh, np, out);
              __builtin_amdgcn_s_waitcnt(0);
            }
            if (tid == 0) sh.n_patch = 0;
          }
          continue;
        }
        // the list (its kept part: m - survivors of the region beyond it) joins the region's
        // tail: the region's own entries are untouched
        const int ml = GANON_GRP_BLOOM ? sh.n_obs : OBS;   // (grp_filter: the kept part of the LDS list)
        n = (n - OBS) + ml;
        for (int i = opaque_tid(); i < ml; i += kGrpThreads) {
          gp(aux->okey)[gg.off + (n - ml) + i] = sh.key[i];
          gp(aux->opay)[gg.off + (n - ml) + i] = sh.pay[i];
        }
        __builtin_amdgcn_s_waitcnt(0);   // region stores at L2 before the barrier
        __syncthreads();
        grp_global(B, sh, gg, n, s_begin, sink);
        continue;
      }
      // the region overflowed too (more than ~2 % of the bases mismatch): split [R.lo, R.hi)
      // at the middle of the stored keys' range — both halves keep stored keys, and a single key
      // never fills a region (capacity > 3 x the group's reads)
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      for (int i = opaque_tid(); i < gg.cap; i += kGrpThreads) {
        const unsigned long long k = i < OBS ? sh.key[i] : ld_l2(gp(aux->okey) + gg.off + (i - OBS));
        atomicMin(&sh.kmin, k);
        atomicMax(&sh.kmax, k);
      }
      __syncthreads();
      if (tid == 0) {
        const unsigned long long a = sh.kmin, b = sh.kmax, mid = a + (b - a) / 2 + 1;
        int t = sh.top;
        if (a < b && t + 2 < kGrpStack) {
          ++t;
          sh.stk_lo[t] = mid;
          sh.stk_hi[t] = R.hi;
          sh.stk_mode[t] = kModeCollect;
          ++t;
          sh.stk_lo[t] = R.lo;
          sh.stk_hi[t] = mid;
          sh.stk_mode[t] = kModeCollect;
        }
        sh.top = t;
      }
      continue;
    }
    grp_classify(B, sh, n, s_begin, sink, true);
    if (!sink.lds) continue;
    // fused: in-partition masks (at most one per observation of this list) as byte stores, after
    // every wave's earlier stores have drained
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const int np = sh.n_patch;
    if (np) {
      lds_bitonic(sh.patch, nullptr, np);
      grp_patch_bytes(B, sh, np, out);
      __builtin_amdgcn_s_waitcnt(0);
    }
    if (tid == 0) sh.n_patch = 0;
  }
}

// Last kernel of a group-variant run. (1) Fused: masks of bytes outside the masking
// workgroup's partition (every partition is written by now). (2) Totals: the group
// workgroups' partials plus the wide scopes' counts, reduced per workgroup into acc; the last
// workgroup to finish (ticket acc[2]) writes totals = static values + sums + rare counts and
// resets acc and counters for the next run — no memset or copy is launched per run.
// counters: [0] rare small scopes (unused), [1] rare tiles; far_count: far masks.
__global__ void __launch_bounds__(kBlock) k_finish(const unsigned long long *__restrict__ far, int64_t far_cap,
                                                   uint8_t *__restrict__ out, const int32_t *__restrict__ grp_part,
                                                   int n_groups, const int32_t *__restrict__ large_ids, int n_large,
                                                   const int32_t *__restrict__ scope_calls,
                                                   const int32_t *__restrict__ scope_bases,
                                                   const unsigned long long *__restrict__ static_totals,
                                                   int32_t *counters, unsigned long long *far_count,
                                                   int32_t *status, unsigned long long *acc,
                                                   unsigned long long *far_need,
                                                   unsigned long long *totals,
                                                   const unsigned long long *__restrict__ ws_part,
                                                   const unsigned long long *__restrict__ plan_info,
                                                   unsigned long long *gated) {
  const int64_t gtid = blockIdx.x * (int64_t)kBlock + threadIdx.x, gstride = (int64_t)gridDim.x * kBlock;
  const unsigned long long far_n = *far_count;
  const int64_t n_far = far_n < (unsigned long long)far_cap ? (int64_t)far_n : far_cap;
  for (int64_t i = gtid; i < n_far; i += gstride) {
    const unsigned long long e = far[i];
    const int64_t nib = (int64_t)(e >> 4);
    const int64_t byte = nib >> 1;
    const int sh = 8 * (int)(byte & 3) + ((nib & 1) ? 0 : 4);
    atomicXor(reinterpret_cast<uint32_t *>(out) + (byte >> 2), (uint32_t)(e & 15) << sh);
  }
  long long c = 0, b = 0;
  unsigned long long h = 0;   // write-scope hash sums of the emit paths (one per group)
  for (int64_t i = gtid; i < n_groups; i += gstride) {
    c += grp_part[2 * i];
    b += grp_part[2 * i + 1];
    h += ws_part[i];
  }
  for (int64_t i = gtid; i < n_large; i += gstride) {
    c += scope_calls[large_ids[i]];
    b += scope_bases[large_ids[i]];
  }
  __shared__ long long part[3][kWaves];
  __shared__ int last;
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    b += __shfl_xor(b, o);
    h += __shfl_xor(h, o);
  }
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = c;
    part[1][threadIdx.x >> 6] = b;
    part[2][threadIdx.x >> 6] = (long long)h;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    c = b = 0;
    h = 0;
    for (int w = 0; w < kWaves; ++w) {
      c += part[0][w];
      b += part[1][w];
      h += (unsigned long long)part[2][w];
    }
    if (c) atomicAdd(&acc[0], (unsigned long long)c);
    if (b) atomicAdd(&acc[1], (unsigned long long)b);
    if (h) atomicAdd(&acc[4], h);
    __threadfence();
    last = atomicAdd(&acc[2], 1ull) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __threadfence();
  const unsigned long long sc = atomicExch(&acc[0], 0ull), sb = atomicExch(&acc[1], 0ull);
  atomicExch(&acc[2], 0ull);
  // every written read met once in its write scope (k_prep_scan's sum vs the emit paths'); a gated
  // run (plan_info[7]: a speculative plan the batch did not fit, or an invalid batch) ran no
  // one-segment kernel: ganon_batch_download plans and runs it again (or reports the error)
  const unsigned long long hs = atomicExch(&acc[4], 0ull);
  if (plan_info[7]) {
    atomicOr(status, 4);
    atomicAdd(gated, 1ull);   // (cumulative since upload: ganon_batch_gated_runs)
  } else if (hs != plan_info[6]) {
    atomicOr(status, 2);
  }
  for (int k = 0; k < GANON_N_TOTALS; ++k) totals[k] = static_totals[k];
  totals[GANON_T_READS_WRITTEN] = plan_info[2];
  totals[GANON_T_MASKED_SNV_CALLS] += sc;
  totals[GANON_T_MASKED_BASES] += sb;
  totals[GANON_T_RARE_SCOPES] += (unsigned long long)(atomicExch(&counters[0], 0) + atomicExch(&counters[1], 0));
  // more far masks than the list holds: the masks past it were dropped — ganon_batch_download grows
  // the list to the count kept in far_need and runs the batch again
  const unsigned long long n_far_all = atomicExch(far_count, 0ull);
  if (n_far_all > (unsigned long long)far_cap) {
    atomicOr(status, 1);
    atomicMax(far_need, n_far_all);
  }
}
// One workgroup per 16 Ki-position tile of a large scope: tally -> TN table (global).
template <int TB>
__global__ void __launch_bounds__(kBlock) k_tile_large(const DevBatch B, const Tile *__restrict__ tiles,
                                                       const int32_t *__restrict__ tile_list, int n_static,
                                                       const int32_t *count_ptr, const int32_t *__restrict__ large_incid,
                                                       const int64_t *__restrict__ tab_off, uint16_t *__restrict__ tn_tab,
                                                       int32_t *scope_calls, int32_t *rare_list, int32_t *rare_count) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int tab_words = kTile * TB / 4;
  uint32_t *tab = smem;
  uint8_t *refb = reinterpret_cast<uint8_t *>(smem + tab_words);
  int *scratch = reinterpret_cast<int *>(refb + kTile / 2);
  const int n = count_ptr ? *count_ptr : n_static;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int li = blockIdx.x; li < n; li += gridDim.x) {
    const int ti = tile_list ? tile_list[li] : li;
    const Tile t = tiles[ti];
    const int s = t.scope;
    const int span = t.b - t.a;
    const int words = (span * TB + 3) >> 2;
    for (int w = threadIdx.x; w < words; w += kBlock) tab[w] = 0;
    stage_ref(B, B.ref_off[s] + (t.a - B.span_start[s]), span, refb);
    if (threadIdx.x == 0) scratch[kWaves] = 0;
    __syncthreads();
    bool rare = false;
    for (int64_t i = t.lo + wave; i < t.hi; i += kWaves) {
      const int r = large_incid[i];
      if (B.read_end[r] <= t.a || B.ref_start[r] >= t.b) continue;
      rare |= tally_read<TB>(B, r, t.a, t.b, tab, LdsRef{refb, t.a}, lane);
    }
    if (TB == 1 && rare) scratch[kWaves] = 1;
    __syncthreads();
    clear_keep<TB>(B, s, t.a, t.b, tab);
    __syncthreads();
    int calls = 0;
    uint16_t *dst = tn_tab + tab_off[s] + (t.a - B.span_start[s]);
    for (int off = threadIdx.x; off < span; off += kBlock) {
      const uint32_t tn = tn_mask<TB>(tab, off);
      uint32_t m16;
      if (TB == 1) m16 = ((tn & 1u) << 1) | ((tn & 2u) << 1) | ((tn & 4u) << 2) | ((tn & 8u) << 5);
      else m16 = tn;
      dst[off] = (uint16_t)m16;
      calls += tn_count<TB>(tn);
    }
    calls = block_sum(calls, scratch);
    if (threadIdx.x == 0) {
      const bool is_rare = (TB == 1) && scratch[kWaves];
      if (is_rare) rare_list[atomicAdd(rare_count, 1)] = ti;
      else if (calls) atomicAdd(&scope_calls[s], calls);
    }
    __syncthreads();
  }
}

// Reads written from large scopes: one wave per read, TN table lookups in global memory.
__global__ void __launch_bounds__(kBlock) k_mask_large(const DevBatch B, const int32_t *__restrict__ list, int n,
                                                       const int64_t *__restrict__ tab_off,
                                                       const uint16_t *__restrict__ tn_tab,
                                                       uint8_t *__restrict__ out, int32_t *scope_bases) {
  const int lane = threadIdx.x & 63;
  const int gw = (blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int nw = (gridDim.x * kBlock) >> 6;
  for (int i = gw; i < n; i += nw) {
    const int r = list[i];
    const int s = B.write_scope[r];
    const int a = B.span_start[s];
    const int64_t to = tab_off[s];
    const int64_t rnib = B.ref_off[s];
    const int L = B.read_len[r];
    const int64_t so = B.seq_off[r];
    CigarCursor cur;
    cur.init(B.cigar + B.cig_off[r], B.n_cig[r], B.ref_start[r]);
    int masked = 0;
    for (int j = lane; j < ((L + 1) >> 1); j += 64) {
      const uint8_t in = B.seq[so + j];
      int nb[2] = {in >> 4, in & 0xF};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int q = 2 * j + h;
        if (q >= L) break;
        const int p = cur.ref_of(q);
        if (p < 0) continue;
        const uint32_t tn = tn_tab[to + (p - a)];
        if ((tn >> nb[h]) & 1u) {
          nb[h] = nib_at(B.ref, rnib + (p - a));
          ++masked;
        }
      }
      out[so + j] = (uint8_t)((nb[0] << 4) | nb[1]);
    }
    for (int o = 32; o > 0; o >>= 1) masked += __shfl_xor(masked, o);
    if (lane == 0 && masked) atomicAdd(&scope_bases[s], masked);
  }
}

}  // namespace
// ---- host side ---------------------------------------------------------------------------

using ganon_detail::check_launch;
using ganon_detail::fail;
using ganon_detail::KernelScope;

namespace {

constexpr int64_t kFarMaxEntries = int64_t(1) << 30;   // far-mask list entries at most (8 GiB)

size_t tile_lds_bytes(int tb) { return (size_t)kTile * tb + kTile / 2 + 16 * sizeof(int); }

void free_buf(DBuf &b) {
  if (b.p) hipFree(b.p);
  b = DBuf{};
}

void free_ref(ganon_ref *r) {
  if (!r) return;
  if (r->nt16) hipFree(r->nt16);
  if (r->ref2) hipFree(r->ref2);
  if (r->bad) hipFree(r->bad);
  delete r;
}

void free_huge(ganon_dbatch *db) {
  for (void *p : db->huge_allocs) hipFree(p);
  db->huge_allocs.clear();
  db->tiles_h = nullptr;
  db->large_incid = db->large_written_h = db->large_ids = db->rare_tile_list = nullptr;
  db->tab_off = nullptr;
  db->tn_tab = nullptr;
  db->n_tiles_h = db->n_large_written_h = 0;
  db->tn_entries = 0;
}

void free_batch(ganon_dbatch *db) {
  DBuf *bufs[] = {&db->b_ref_start, &db->b_read_len, &db->b_seq_off, &db->b_cig_off, &db->b_n_cig, &db->b_dataset,
                  &db->b_write_scope, &db->b_seq, &db->b_cigar, &db->b_incid_off, &db->b_incid_read,
                  &db->b_span_start, &db->b_span_len, &db->b_ref_off, &db->b_keep_pos, &db->b_keep_code,
                  &db->b_read_end, &db->b_wspart, &db->b_cursor, &db->b_gs0, &db->b_lo, &db->b_linemap, &db->b_groups,
                  &db->b_seg4, &db->b_grp_part, &db->b_far, &db->b_gokey, &db->b_gopay, &db->b_gtkey, &db->b_gtflag,
                  &db->b_out, &db->b_scope_calls, &db->b_scope_bases, &db->b_small, &db->b_part, &db->b_long, &db->b_nseg,
                  &db->b_scost, &db->b_scan_tmp, &db->b_slots, &db->b_slot0, &db->b_order, &db->b_desc, &db->b_cand,
                  &db->b_sdirty, &db->b_inc4, &db->b_rbase, &db->b_rrec, &db->b_xrec, &db->b_xlist, &db->b_xcnt, &db->b_xidx};
  for (DBuf *b : bufs) free_buf(*b);
  free_huge(db);
  free_ref(db->own_ref);
  db->own_ref = nullptr;
}

// Grow b to count elements and enqueue the copy of src (async on the stream).
template <typename T>
int h2d(ganon_ctx *ctx, DBuf &b, const T *src, size_t count, const T **field) {
  T *p = nullptr;
  int rc = ganon_prep::grow_n(ctx, b, count, &p);
  if (rc) return rc;
  if (count) {
    hipError_t e = hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipMemcpyAsync H2D failed: %s", hipGetErrorString(e));
  }
  *field = p;
  return GANON_OK;
}

template <typename T>
int dmalloc(ganon_ctx *ctx, std::vector<void *> &allocs, T **p, size_t count) {
  *p = nullptr;
  const size_t bytes = std::max<size_t>(count, 1) * sizeof(T) + 128;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(p), bytes);
  if (e != hipSuccess) return fail(ctx, GANON_E_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  allocs.push_back(*p);
  return GANON_OK;
}

int ref_create(ganon_ctx *ctx, const uint8_t *nt16, int64_t bytes, ganon_ref **out) {
  *out = nullptr;
  if (bytes < 0 || (bytes > 0 && !nt16)) return fail(ctx, GANON_E_ARG, "bad reference buffer");
  if (2 * bytes >= (int64_t(1) << 40)) return fail(ctx, GANON_E_ARG, "reference over 2^40 bases");
  ganon_ref *r = new ganon_ref();
  r->bytes = bytes;
  r->n_blk = (bytes + 31) / 32;
  const int64_t n_words = (2 * bytes + 15) / 16;
  const int64_t n_bad = (r->n_blk + 63) / 64 + 1;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(&r->nt16), (size_t)bytes + 128);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&r->ref2), (size_t)(n_words + 2) * 4 + 128);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&r->bad), (size_t)n_bad * 8 + 128);
  if (e != hipSuccess) {
    free_ref(r);
    return fail(ctx, GANON_E_NOMEM, "reference allocation failed: %s", hipGetErrorString(e));
  }
  if (bytes) e = hipMemcpyAsync(r->nt16, nt16, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(r->nt16 + bytes, 0, 128, ctx->stream);
  if (e != hipSuccess) {
    free_ref(r);
    return fail(ctx, GANON_E_DEVICE, "reference copy failed: %s", hipGetErrorString(e));
  }
  int rc = GANON_OK;
  if (n_words) {
    k_ref2<<<(int)std::min<int64_t>((n_words + kBlock - 1) / kBlock, 16384), kBlock, 0, ctx->stream>>>(r->nt16, n_words,
                                                                                                    r->ref2);
    rc = check_launch(ctx, "k_ref2");
  }
  if (!rc) rc = ganon_ref_blocks(ctx, r);
  if (!rc && ganon_detail::sync_stream(ctx->stream) != hipSuccess) rc = fail(ctx, GANON_E_DEVICE, "reference upload sync failed");
  if (rc) {
    free_ref(r);
    return rc;
  }
  *out = r;
  return GANON_OK;
}

// bam_endpos of read r from the host batch (huge-scope planning only).
int32_t host_read_end(const ganon_batch *b, int32_t r) {
  int64_t rl = 0;
  for (int k = 0; k < b->n_cig[r]; ++k) {
    const uint32_t w = b->cigar[b->cig_off[r] + k];
    const int op = w & 0xF;
    if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += w >> 4;
  }
  return (int32_t)(b->ref_start[r] + (rl > 0 ? rl : 1));
}

// Scopes wider than kGrpMaxSpan (whole-contig union scopes of very deep samples; none in the
// benchmark configs): 16 Ki-position tiles planned on the host from the scopes' incidences.
int plan_huge(ganon_ctx *ctx, ganon_dbatch *db, const ganon_batch *b) {
  free_huge(db);
  if (!db->n_huge_scopes) return GANON_OK;
  std::vector<int32_t> large_incid, ids, written;
  std::vector<int64_t> tab_off((size_t)b->n_scopes, -1);
  std::vector<Tile> tiles;
  int64_t tn_entries = 0;
  for (int32_t s = 0; s < b->n_scopes; ++s) {
    const int32_t sl = b->scope_span_len[s];
    if (sl <= kGrpMaxSpan) continue;
    ids.push_back(s);
    tab_off[s] = tn_entries;
    tn_entries += sl;
    const int64_t base = (int64_t)large_incid.size();
    for (int64_t i = b->scope_incid_off[s]; i < b->scope_incid_off[s + 1]; ++i) large_incid.push_back(b->incid_read[i]);
    std::stable_sort(large_incid.begin() + base, large_incid.end(),
                     [&](int32_t x, int32_t y) { return b->ref_start[x] < b->ref_start[y]; });
    int32_t maxspan = 1;
    for (int64_t i = base; i < (int64_t)large_incid.size(); ++i) {
      const int32_t r = large_incid[i];
      maxspan = std::max(maxspan, host_read_end(b, r) - b->ref_start[r]);
    }
    const int32_t ss = b->scope_span_start[s];
    for (int64_t a = ss; a < (int64_t)ss + sl; a += kTile) {
      Tile t{};
      t.scope = s;
      t.a = (int32_t)a;
      t.b = (int32_t)std::min<int64_t>(a + kTile, (int64_t)ss + sl);
      auto first = large_incid.begin() + base;
      auto last = large_incid.end();
      t.lo = std::lower_bound(first, last, (int64_t)t.a - maxspan,
                              [&](int32_t r, int64_t key) { return (int64_t)b->ref_start[r] < key; }) -
             large_incid.begin();
      t.hi = std::lower_bound(first, last, (int64_t)t.b,
                              [&](int32_t r, int64_t key) { return (int64_t)b->ref_start[r] < key; }) -
             large_incid.begin();
      tiles.push_back(t);
    }
  }
  for (int32_t r = 0; r < b->n_reads; ++r) {
    const int32_t ws = b->write_scope[r];
    if (ws >= 0 && b->scope_span_len[ws] > kGrpMaxSpan) written.push_back(r);
  }
  int rc;
  auto up = [&](auto **p, const auto &v) -> int {
    using T = std::remove_const_t<std::remove_reference_t<decltype(v[0])>>;
    T *q = nullptr;
    int c = dmalloc(ctx, db->huge_allocs, &q, v.size());
    if (c) return c;
    if (!v.empty() && hipMemcpyAsync(q, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
      return fail(ctx, GANON_E_DEVICE, "huge-scope plan copy failed");
    *p = q;
    return GANON_OK;
  };
  if ((rc = up(&db->tiles_h, tiles)) || (rc = up(&db->large_incid, large_incid)) || (rc = up(&db->tab_off, tab_off)) ||
      (rc = up(&db->large_written_h, written)) || (rc = up(&db->large_ids, ids)))
    return rc;
  if ((rc = dmalloc(ctx, db->huge_allocs, &db->rare_tile_list, tiles.size()))) return rc;
  db->n_tiles_h = (int32_t)tiles.size();
  db->n_large_written_h = (int32_t)written.size();
  db->tn_entries = tn_entries;
  return GANON_OK;
}

// Host copies of the arrays plan_huge reads, for a batch planned from its device arrays alone
// (ganon_batch_replan of a batch with scopes wider than the group kernels': rare).
struct HostCopy {
  std::vector<int32_t> ref_start, n_cig, write_scope, incid_read, span_start, span_len;
  std::vector<int64_t> cig_off, incid_off;
  std::vector<uint32_t> cigar;
  ganon_batch b{};
};

template <typename T>
int d2h_vec(ganon_ctx *ctx, std::vector<T> &v, const T *src, size_t n) {
  v.resize(n);
  if (n) HIP_OR_FAIL(ganon_detail::readback(v.data(), src, n * sizeof(T), ctx->stream));
  return GANON_OK;
}

int host_copy(ganon_ctx *ctx, const ganon_dbatch *db, HostCopy &h) {
  const DevBatch &B = db->B;
  int rc;
  if ((rc = d2h_vec(ctx, h.ref_start, B.ref_start, (size_t)db->n_reads)) ||
      (rc = d2h_vec(ctx, h.n_cig, B.n_cig, (size_t)db->n_reads)) ||
      (rc = d2h_vec(ctx, h.write_scope, B.write_scope, (size_t)db->n_reads)) ||
      (rc = d2h_vec(ctx, h.cig_off, B.cig_off, (size_t)db->n_reads)) ||
      (rc = d2h_vec(ctx, h.cigar, B.cigar, (size_t)db->n_cigar_ops)) ||
      (rc = d2h_vec(ctx, h.incid_off, B.incid_off, (size_t)db->n_scopes + 1)) ||
      (rc = d2h_vec(ctx, h.incid_read, B.incid_read, (size_t)db->n_incid)) ||
      (rc = d2h_vec(ctx, h.span_start, B.span_start, (size_t)db->n_scopes)) ||
      (rc = d2h_vec(ctx, h.span_len, B.span_len, (size_t)db->n_scopes)))
    return rc;
  HIP_OR_FAIL(ganon_detail::sync_stream(ctx->stream));
  ganon_batch &b = h.b;
  b.n_reads = db->n_reads;
  b.n_scopes = db->n_scopes;
  b.n_incid = db->n_incid;
  b.n_cigar_ops = db->n_cigar_ops;
  b.ref_start = h.ref_start.data();
  b.n_cig = h.n_cig.data();
  b.write_scope = h.write_scope.data();
  b.cig_off = h.cig_off.data();
  b.cigar = h.cigar.data();
  b.scope_incid_off = h.incid_off.data();
  b.incid_read = h.incid_read.data();
  b.scope_span_start = h.span_start.data();
  b.scope_span_len = h.span_len.data();
  return GANON_OK;
}

// Plan a batch whose raw arrays are on the device (ganon_prep::plan: validation, prep mode, sizes),
// the huge-scope tiles (from `host`, or host copies), and upload the group kernels' aux pointers
// and the static totals (async).
int prepare(ganon_ctx *ctx, ganon_dbatch *db, const ganon_batch *host, bool allow_spec = false) {
  int rc;
  if ((rc = ganon_prep::plan(ctx, db, allow_spec))) return rc;   // (it clears the step's flags first)
  if (db->spec && !db->spec_sized) {
    // the previous plan's tiles (none), aux pointers and static totals, unchanged on the host; copied
    // again (a reload clears the device's small state)
    HIP_OR_FAIL(hipMemcpyAsync(db->aux, &db->aux_h, sizeof db->aux_h, hipMemcpyHostToDevice, ctx->stream));
    HIP_OR_FAIL(hipMemcpyAsync(db->static_totals, db->static_h, GANON_N_TOTALS * sizeof(unsigned long long),
                               hipMemcpyHostToDevice, ctx->stream));
    return GANON_OK;
  }
  if (db->n_huge_scopes && !host) {
    HostCopy h;
    if ((rc = host_copy(ctx, db, h)) || (rc = plan_huge(ctx, db, &h.b))) return rc;
  } else if ((rc = plan_huge(ctx, db, host))) {
    return rc;
  }
  GrpAux &a = db->aux_h;
  a = GrpAux{};
  a.scope_calls = db->scope_calls;
  a.scope_bases = db->scope_bases;
  a.part = static_cast<int32_t *>(db->b_grp_part.p);
  a.far = static_cast<unsigned long long *>(db->b_far.p);
  a.far_count = db->far_count;
  a.far_cap = db->far_cap;
  a.paths = db->paths;
  a.okey = static_cast<unsigned long long *>(db->b_gokey.p);
  a.opay = static_cast<unsigned long long *>(db->b_gopay.p);
  a.tkey = static_cast<unsigned long long *>(db->b_gtkey.p);
  a.tflag = static_cast<unsigned int *>(db->b_gtflag.p);
  a.incid_read = db->B.incid_read;
  a.ref_start = db->B.ref_start;
  a.read_end = db->B.read_end;
  a.desc = static_cast<const int4 *>(db->b_desc.p);
  a.incid_off = db->B.incid_off;
  a.ref_off = db->B.ref_off;
  a.sdirty = static_cast<const uint8_t *>(db->b_sdirty.p);
  a.inc4 = static_cast<const int4 *>(db->b_inc4.p);
  a.rrec = static_cast<const int4 *>(db->b_rrec.p);
  a.xrec = static_cast<const int4 *>(db->b_xrec.p);
  a.xidx = static_cast<const int32_t *>(db->b_xidx.p);
  a.xlist = static_cast<int2 *>(db->b_xlist.p);
  a.n_reads = db->n_reads;
  a.err = db->err;
  a.ws_part = static_cast<unsigned long long *>(db->b_wspart.p);
  unsigned long long *st = db->static_h;
  std::fill(st, st + GANON_N_TOTALS, 0ull);
  st[GANON_T_READS_IN] = (unsigned long long)db->n_reads;
  st[GANON_T_READS_WRITTEN] = (unsigned long long)db->n_written;
  st[GANON_T_SCOPES] = (unsigned long long)db->n_scopes;
  st[GANON_T_LARGE_TILES] = (unsigned long long)db->n_tiles_h;
  // (from db-resident host copies: the next plan of db synchronizes before it rewrites them)
  HIP_OR_FAIL(hipMemcpyAsync(db->aux, &db->aux_h, sizeof db->aux_h, hipMemcpyHostToDevice, ctx->stream));
  HIP_OR_FAIL(hipMemcpyAsync(db->static_totals, st, GANON_N_TOTALS * sizeof(unsigned long long), hipMemcpyHostToDevice,
                             ctx->stream));
  return GANON_OK;
}

// Copy a host batch into db (grow-only buffers), validate and plan it on the device.
int load_batch(ganon_ctx *ctx, ganon_dbatch *db, const ganon_batch *b, const ganon_ref *shared) {
  if (b->n_reads < 0 || b->n_scopes < 0 || b->n_incid < 0 || b->seq_bytes < 0 || b->n_cigar_ops < 0 || b->ref_bytes < 0)
    return fail(ctx, GANON_E_ARG, "negative size in batch");
  if (b->n_reads > 0 && (!b->ref_start || !b->read_len || !b->seq_off || !b->cig_off || !b->n_cig || !b->dataset ||
                         !b->write_scope))
    return fail(ctx, GANON_E_ARG, "null read array");
  if (b->seq_bytes > 0 && !b->seq_nt16) return fail(ctx, GANON_E_ARG, "null seq_nt16");
  if (b->n_cigar_ops > 0 && !b->cigar) return fail(ctx, GANON_E_ARG, "null cigar");
  if (!b->scope_incid_off) return fail(ctx, GANON_E_ARG, "null scope_incid_off");
  if (b->n_scopes > 0 && (!b->scope_span_start || !b->scope_span_len || !b->scope_ref_off || !b->keep_pos ||
                          !b->keep_code))
    return fail(ctx, GANON_E_ARG, "null scope array");
  if (b->n_incid > 0 && !b->incid_read) return fail(ctx, GANON_E_ARG, "null incid_read");
  if (!shared && b->ref_bytes > 0 && !b->ref_nt16) return fail(ctx, GANON_E_ARG, "null ref_nt16");
  if (b->scope_incid_off[0] != 0 || b->scope_incid_off[b->n_scopes] != b->n_incid)
    return fail(ctx, GANON_E_ARG, "scope_incid_off must start at 0 and end at n_incid");
  if (2 * b->seq_bytes >= (int64_t(1) << 39)) return fail(ctx, GANON_E_ARG, "sequence over 2^39 bases");
  int64_t max_si = 0;   // (the group kernel's launch order: ganon_prep launch_pieces)
  for (int32_t s = 0; s < b->n_scopes; ++s) max_si = std::max(max_si, b->scope_incid_off[s + 1] - b->scope_incid_off[s]);
  if (b->n_incid >= INT32_MAX) return fail(ctx, GANON_E_ARG, "more than 2^31-1 incidences");
  int rc;
  HIP_OR_FAIL(ganon_detail::sync_stream(ctx->stream));   // a previous run of db may still read its buffers
  db->ran = false;
  db->max_scope_incid = max_si;
  if (shared) {
    db->ref = shared;
  } else {
    free_ref(db->own_ref);
    db->own_ref = nullptr;
    if ((rc = ref_create(ctx, b->ref_nt16, b->ref_bytes, &db->own_ref))) return rc;
    db->ref = db->own_ref;
  }
  db->n_reads = b->n_reads;
  db->n_scopes = b->n_scopes;
  db->n_incid = b->n_incid;
  db->seq_bytes = b->seq_bytes;
  db->n_cigar_ops = b->n_cigar_ops;
  db->group_target = ctx->group_target;
  DevBatch &D = db->B;
  if ((rc = h2d(ctx, db->b_ref_start, b->ref_start, b->n_reads, &D.ref_start)) ||
      (rc = h2d(ctx, db->b_read_len, b->read_len, b->n_reads, &D.read_len)) ||
      (rc = h2d(ctx, db->b_seq_off, b->seq_off, b->n_reads, &D.seq_off)) ||
      (rc = h2d(ctx, db->b_cig_off, b->cig_off, b->n_reads, &D.cig_off)) ||
      (rc = h2d(ctx, db->b_n_cig, b->n_cig, b->n_reads, &D.n_cig)) ||
      (rc = h2d(ctx, db->b_dataset, b->dataset, b->n_reads, &D.dataset)) ||
      (rc = h2d(ctx, db->b_write_scope, b->write_scope, b->n_reads, &D.write_scope)) ||
      (rc = h2d(ctx, db->b_seq, b->seq_nt16, b->seq_bytes, &D.seq)) ||
      (rc = h2d(ctx, db->b_cigar, b->cigar, b->n_cigar_ops, &D.cigar)) ||
      (rc = h2d(ctx, db->b_incid_off, b->scope_incid_off, (size_t)b->n_scopes + 1, &D.incid_off)) ||
      (rc = h2d(ctx, db->b_incid_read, b->incid_read, b->n_incid, &D.incid_read)) ||
      (rc = h2d(ctx, db->b_span_start, b->scope_span_start, b->n_scopes, &D.span_start)) ||
      (rc = h2d(ctx, db->b_span_len, b->scope_span_len, b->n_scopes, &D.span_len)) ||
      (rc = h2d(ctx, db->b_ref_off, b->scope_ref_off, b->n_scopes, &D.ref_off)) ||
      (rc = h2d(ctx, db->b_keep_pos, b->keep_pos, b->n_scopes, &D.keep_pos)) ||
      (rc = h2d(ctx, db->b_keep_code, b->keep_code, b->n_scopes, &D.keep_code)))
    return rc;
  D.ref = db->ref->nt16;
  D.ref2 = db->ref->ref2;
  // small device state: totals, static totals, acc, far count, plan info (u64); counters, status;
  // the first validation error; the group kernels' aux pointers
  constexpr size_t kU64 = 8 + 8 + 5 + 1 + 8 + 4 + 1;
  // the per-plan flags (first error, status bits, long-read count, far masks needed) are adjacent:
  // one memset clears them at the start of every plan
  constexpr size_t kFlags = sizeof(PrepErr) + 16;
  constexpr size_t kSmallBytes = kU64 * 8 + 8 * 4 + kFlags + sizeof(GrpAux) + 64;
  uint8_t *sm = nullptr;
  if ((rc = ganon_prep::grow_n(ctx, db->b_small, kSmallBytes, &sm))) return rc;
  auto *u = reinterpret_cast<unsigned long long *>(sm);
  db->totals = u;
  db->static_totals = u + 8;
  db->acc = u + 16;        // [0] calls, [1] bases, [2] ticket, [3] far masks needed, [4] write-scope sum
  db->far_count = u + 21;
  db->plan_info = u + 22;
  db->paths = u + 30;
  db->gated = u + 34;      // runs a speculative plan's gate stopped (cumulative)
  db->counters = reinterpret_cast<int32_t *>(u + kU64);
  db->err = reinterpret_cast<PrepErr *>(sm + kU64 * 8 + 8 * 4);
  db->status = reinterpret_cast<int32_t *>(db->err + 1);
  db->long_count = reinterpret_cast<unsigned int *>(db->status + 1);
  db->far_need = reinterpret_cast<unsigned long long *>(db->long_count + 1);
  db->flags_bytes = kFlags;
  db->aux = reinterpret_cast<GrpAux *>(sm + kU64 * 8 + 8 * 4 + kFlags);
  HIP_OR_FAIL(hipMemsetAsync(sm, 0, kSmallBytes, ctx->stream));
  if ((rc = ganon_prep::grow_n(ctx, db->b_scope_calls, b->n_scopes, &db->scope_calls)) ||
      (rc = ganon_prep::grow_n(ctx, db->b_scope_bases, b->n_scopes, &db->scope_bases)) ||
      (rc = ganon_prep::grow_n(ctx, db->b_out, b->seq_bytes, &db->out)))
    return rc;
  // bytes outside every read are never written by the masking kernels: make them defined
  HIP_OR_FAIL(hipMemsetAsync(db->out, 0, (size_t)b->seq_bytes + 16, ctx->stream));
  if ((rc = prepare(ctx, db, b, ctx->spec_plan == 2))) return rc;   // (2: testing knob)
  HIP_OR_FAIL(ganon_detail::sync_stream(ctx->stream));
  return GANON_OK;
}

int upload_common(ganon_ctx *ctx, const ganon_batch *b, const ganon_ref *ref, ganon_dbatch **out) {
  if (!ctx || !b || !out) return fail(ctx, GANON_E_ARG, "null argument");
  *out = nullptr;
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  ganon_dbatch *db = new ganon_dbatch();
  int rc = load_batch(ctx, db, b, ref);
  if (rc) {
    ganon_detail::sync_stream(ctx->stream);
    free_batch(db);
    delete db;
    return rc;
  }
  *out = db;
  return GANON_OK;
}

}  // namespace

GANON_API int ganon_abi_version(void) { return GANON_ABI_VERSION; }

GANON_API int ganon_ctx_create(int device, ganon_ctx **out) {
  if (!out) return GANON_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return GANON_E_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return GANON_E_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return GANON_E_DEVICE;
  if (hipSetDevice(device) != hipSuccess) return GANON_E_DEVICE;
  ganon_ctx *ctx = new ganon_ctx();
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return GANON_E_DEVICE;
  }
  ctx->stream = ctx->own;
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_tile_large<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)tile_lds_bytes(1));
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_tile_large<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)tile_lds_bytes(4));
  *out = ctx;
  return GANON_OK;
}

GANON_API int ganon_ctx_destroy(ganon_ctx *ctx) {
  if (!ctx) return GANON_E_ARG;
  hipSetDevice(ctx->device);
  if (ctx->own) {
    ganon_detail::sync_stream(ctx->own);
    hipStreamDestroy(ctx->own);
  }
  for (auto &r : ctx->recs) {
    hipEventDestroy(r.e0);
    hipEventDestroy(r.e1);
  }
  for (auto e : ctx->pool) hipEventDestroy(e);
  if (ctx->side) {
    ganon_detail::sync_stream(ctx->side);
    hipStreamDestroy(ctx->side);
  }
  if (ctx->fork_ev) hipEventDestroy(ctx->fork_ev);
  if (ctx->join_ev) hipEventDestroy(ctx->join_ev);
  for (auto &b : ctx->dcache) hipFree(b.second);
  ganon_inflate_free(ctx->inflate);
  delete ctx;
  return GANON_OK;
}

GANON_API const char *ganon_last_error(ganon_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// Page-locked blocks are cached per process (up to 8 GiB): pinning and unpinning hundreds of MB per
// reader and run (the readers' scan buffers, the FASTQ blobs) cost more than the copies they save.
namespace {
std::mutex g_pin_mu;
std::multimap<size_t, void *> g_pin_free;   // capacity -> block
std::map<void *, size_t> g_pin_cap;         // every live or cached block's capacity
size_t g_pin_cached = 0;
constexpr size_t kPinCacheMax = size_t(8) << 30;
int64_t g_pin_stats[4] = {0, 0, 0, 0};      // blocks pinned anew, their bytes, seconds in hipHostMalloc, cache hits
}  // namespace

GANON_API int ganon_pinned_alloc(int64_t bytes, void **out) {
  if (!out || bytes < 0) return GANON_E_ARG;
  *out = nullptr;
  const size_t want = (size_t)std::max<int64_t>(bytes, 1);
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pin_free.lower_bound(want);
    if (it != g_pin_free.end() && it->first <= 2 * want + (size_t(16) << 20)) {
      g_pin_stats[3] += 1;
      *out = it->second;
      g_pin_cached -= it->first;
      g_pin_free.erase(it);
      return GANON_OK;
    }
  }
  const size_t cap = (want + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
  const auto t0 = std::chrono::steady_clock::now();
  if (hipHostMalloc(out, cap, hipHostMallocDefault) != hipSuccess) {
    *out = nullptr;
    return GANON_E_NOMEM;
  }
  const int64_t ns = (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pin_cap[*out] = cap;
  g_pin_stats[0] += 1;
  g_pin_stats[1] += (int64_t)cap;
  g_pin_stats[2] += ns;
  return GANON_OK;
}

GANON_API int ganon_pinned_stats(int64_t *out4) {
  if (!out4) return GANON_E_ARG;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  for (int k = 0; k < 4; ++k) out4[k] = g_pin_stats[k];
  return GANON_OK;
}

GANON_API int ganon_pinned_free(void *p) {
  if (!p) return GANON_OK;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pin_cap.find(p);
  if (it == g_pin_cap.end()) return GANON_E_ARG;
  if (g_pin_cached + it->second <= kPinCacheMax) {
    g_pin_free.emplace(it->second, p);
    g_pin_cached += it->second;
  } else {
    g_pin_cap.erase(it);
    hipHostFree(p);
  }
  return GANON_OK;
}

GANON_API int ganon_ctx_set_stream(ganon_ctx *ctx, void *hip_stream) {
  if (!ctx) return GANON_E_ARG;
  ctx->stream = hip_stream ? reinterpret_cast<hipStream_t>(hip_stream) : ctx->own;
  return GANON_OK;
}

GANON_API int ganon_ctx_set_variant(ganon_ctx *ctx, int variant) {
  if (!ctx) return GANON_E_ARG;
  if (variant != GANON_VARIANT_DEFAULT && variant != GANON_VARIANT_GROUP_FUSED)
    return fail(ctx, GANON_E_ARG, "kernel variant %d was retired: the fused group kernel is the only small-scope path",
                variant);
  ctx->variant = variant;
  return GANON_OK;
}

GANON_API int ganon_ctx_set_param(ganon_ctx *ctx, int param, int value) {
  if (!ctx) return GANON_E_ARG;
  if (param == GANON_PARAM_GROUP_UNROLL) {
    if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8)
      return fail(ctx, GANON_E_ARG, "group unroll must be 0 (auto), 1, 2, 4 or 8 (got %d)", value);
    ctx->group_unroll = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_GROUP_TARGET) {
    if (value != 0 && (value < 16 || value > 65536))
      return fail(ctx, GANON_E_ARG, "group target must be 0 (auto) or in [16, 65536] (got %d)", value);
    ctx->group_target = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_REF2) {
    ctx->ref2 = value != 0;
    return GANON_OK;
  }
  if (param == GANON_PARAM_FASTQ_SKIP) {
    ctx->fq_skip = value & 127;
    return GANON_OK;
  }
  if (param == GANON_PARAM_INDEL_SORT) {
    if (value != 0 && value != 1) return fail(ctx, GANON_E_ARG, "indel sort: 0 (segmented) or 1 (global)");
    ctx->indel_sort = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_FASTQ_KD) {
    if (value < 0 || value > 17 || value == 7)
      return fail(ctx, GANON_E_ARG,
                  "FASTQ kernel: 0 (spans, 3 units per lane), 13 / 14 (spans, 2 per lane, 8 / 16 KiB tiles), "
                  "15 / 17 (as 0, span found by binary search / from a map entry per 8 units), "
                  "16 / 9 / 10 (quads, 2 / 1 / 3 per lane), 11 (quads, per-dword base select), "
                  "12 (record rows), dwords per lane 1-6 or 8");
    ctx->fq_kd = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_PREP_LONG) {
    if (value < -1 || value > 2) return fail(ctx, GANON_E_ARG, "prep mode: -1 (auto), 0 (two-pass), 1 (long), 2 (one-segment)");
    ctx->prep_long = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_PREP_UNROLL) {
    if (value != 0 && value != 1 && value != 2 && value != 4)
      return fail(ctx, GANON_E_ARG, "prep unroll: 0 (auto), 1, 2 or 4 (got %d)", value);
    ctx->prep_unroll = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_GROUP_OBS) {
    if (value != 0 && value != 512 && value != 1024)
      return fail(ctx, GANON_E_ARG, "group observation list: 0 (auto), 512 or 1024 (got %d)", value);
    ctx->group_obs = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_NT_COPY) {
    ctx->nt_copy = value != 0;
    return GANON_OK;
  }
  if (param == GANON_PARAM_SPEC_PLAN) {
    if (value < 0 || value > 2) return fail(ctx, GANON_E_ARG, "speculative plans: 0, 1 or 2 (got %d)", value);
    ctx->spec_plan = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_FUSED_FLAT) {
    if (value != 0 && value != 1) return fail(ctx, GANON_E_ARG, "fused one-segment mode: 0 or 1 (got %d)", value);
    ctx->fused_flat = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_XREC_INIT) {
    if (value < 0) return fail(ctx, GANON_E_ARG, "extras list capacity must be >= 0");
    ctx->xrec_init = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_FAR_INIT) {
    if (value < 0) return fail(ctx, GANON_E_ARG, "far-mask list capacity must be >= 0");
    ctx->far_init = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_GROUP_SKIP) {
    ctx->group_skip = value & (kSkipClassify | kSkipChunks | kSkipCopy | kSkipCounts);
    return GANON_OK;
  }
  return fail(ctx, GANON_E_ARG, "unknown parameter %d", param);
}

GANON_API int ganon_ctx_set_profiling(ganon_ctx *ctx, int enabled) {
  if (!ctx) return GANON_E_ARG;
  ctx->profiling = enabled != 0;
  return GANON_OK;
}

GANON_API int ganon_ref_upload(ganon_ctx *ctx, const uint8_t *ref_nt16, int64_t ref_bytes, ganon_ref **out) {
  if (!ctx || !out) return fail(ctx, GANON_E_ARG, "null argument");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  return ref_create(ctx, ref_nt16, ref_bytes, out);
}

GANON_API int ganon_ref_free(ganon_ctx *ctx, ganon_ref *ref) {
  if (!ref) return GANON_E_ARG;
  if (ctx) {
    hipSetDevice(ctx->device);
    ganon_detail::sync_stream(ctx->stream);
  }
  free_ref(ref);
  return GANON_OK;
}

GANON_API int ganon_batch_upload(ganon_ctx *ctx, const ganon_batch *b, ganon_dbatch **out) {
  return upload_common(ctx, b, nullptr, out);
}

GANON_API int ganon_batch_upload_ref(ganon_ctx *ctx, const ganon_batch *b, const ganon_ref *ref, ganon_dbatch **out) {
  if (!ref) return fail(ctx, GANON_E_ARG, "null reference");
  return upload_common(ctx, b, ref, out);
}

GANON_API int ganon_batch_reload(ganon_ctx *ctx, ganon_dbatch *db, const ganon_batch *b) {
  if (!ctx || !db || !b) return fail(ctx, GANON_E_ARG, "null argument");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  const ganon_ref *shared = db->own_ref ? nullptr : db->ref;
  int rc = load_batch(ctx, db, b, shared);
  if (rc) {
    // the device batch holds a partial load: only free or reload is valid now
    db->n_groups = 0;
    db->ran = false;
  }
  return rc;
}

namespace {
// A new profiled step: the event pairs of the previous one go back to the pool.
void new_step(ganon_ctx *ctx) {
  for (auto &r : ctx->recs) {
    ctx->pool.push_back(r.e0);
    ctx->pool.push_back(r.e1);
  }
  ctx->recs.clear();
}
}  // namespace

GANON_API int ganon_batch_replan(ganon_ctx *ctx, ganon_dbatch *db) {
  if (!ctx || !db) return fail(ctx, GANON_E_ARG, "null argument");
  if (!db->b_small.p) return fail(ctx, GANON_E_STATE, "replan of a batch that was never loaded");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  new_step(ctx);
  ctx->step_open = true;   // the next run's kernels join this step's timings
  // (speculative: an upload or reload plans in full — its caller reads the shape at once, e.g. the
  // I/D op count that decides the indel tally)
  int rc = prepare(ctx, db, nullptr, true);
  if (rc) {
    db->n_groups = 0;
    db->ran = false;
  }
  return rc;
}

GANON_API int ganon_batch_run(ganon_ctx *ctx, ganon_dbatch *db) {
  if (!ctx || !db) return fail(ctx, GANON_E_ARG, "null argument");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  if (!ctx->step_open) new_step(ctx);
  ctx->step_open = false;
  hipStream_t st = ctx->stream;
  DevBatch B = db->B;
  if (!ctx->ref2) B.ref2 = nullptr;   // group kernels then read the nt16 reference only
  int rc;
  // 16-base chunks per thread: long reads (short segments between indels) waste less with one
  // (profiles/r02/sweep_c5.jsonl); short reads run best with two (sweep_c3.jsonl)
  const int u = ctx->group_unroll ? ctx->group_unroll : db->long_mode ? 1 : 2;
  // 1. derived layer from the raw SoA
  if ((rc = ganon_prep::run(ctx, db))) return rc;
  if (ctx->indel_fork < 0) {
    const char *v = std::getenv("GANON_INDEL_FORK");
    ctx->indel_fork = v && v[0] == '1' ? 1 : 0;
  }
  if (ctx->indel_fork) {   // (the fork point of this batch's indel tally: its inputs are final here)
    if (!ctx->fork_ev) HIP_OR_FAIL(hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming));
    HIP_OR_FAIL(hipEventRecord(ctx->fork_ev, st));
    ctx->fork_db = db;
  }
  if (db->n_huge_scopes) {
    // huge scopes are counted with atomics (tiles)
    HIP_OR_FAIL(hipMemsetAsync(db->scope_calls, 0, (size_t)db->n_scopes * sizeof(int32_t), st));
    HIP_OR_FAIL(hipMemsetAsync(db->scope_bases, 0, (size_t)db->n_scopes * sizeof(int32_t), st));
  }
  // 2. masking: the fused group kernel writes every byte of out (its pieces tile [0, seq_bytes))
  if (db->n_groups) {
    KernelScope ks(ctx, "k_group_fused");
    // 512 unless forced: the 1024-entry list (4 workgroups per CU instead of 6) measured slower on
    // c3 too (3.19 vs 2.84 ms, profiles/r02/sweep_c3_obs.jsonl) — occupancy outweighs the region path
    const int obs = ctx->group_obs ? ctx->group_obs : 512;
    auto kern = db->fused
                    ? (obs == 1024 ? (u == 1 ? k_group<1, true, 1024, true> : k_group<2, true, 1024, true>)
                                   : u == 2 ? k_group<2, true, 512, true> : u == 4 ? k_group<4, true, 512, true>
                                   : u == 8 ? k_group<8, true, 512, true> : k_group<1, true, 512, true>)
                : db->long_mode
                    ? (obs == 1024 ? (u == 1 ? k_group<1, true, 1024, false, true> : k_group<2, true, 1024, false, true>)
                                   : u == 2 ? k_group<2, true, 512, false, true> : u == 4 ? k_group<4, true, 512, false, true>
                                   : u == 8 ? k_group<8, true, 512, false, true> : k_group<1, true, 512, false, true>)
                    : (obs == 1024 ? (u == 1 ? k_group<1, true, 1024, false> : k_group<2, true, 1024, false>)
                                   : u == 2 ? k_group<2, true, 512, false> : u == 4 ? k_group<4, true, 512, false>
                                   : u == 8 ? k_group<8, true, 512, false> : k_group<1, true, 512, false>);
    const GrpBatch GB{B.seq, B.ref, B.keep_code, B.ref2, B.keep_pos, B.span_start, B.span_len};
    kern<<<db->n_groups, kGrpThreads, 0, st>>>(GB, static_cast<const int4 *>(db->b_groups.p),
                                               static_cast<const int4 *>(db->b_seg4.p), db->out, db->aux,
                                               ctx->group_skip, ctx->nt_copy, db->flat_mode ? db->plan_info : nullptr,
                                               db->ordered ? static_cast<const int32_t *>(db->b_order.p) : nullptr);
    if ((rc = check_launch(ctx, "k_group"))) return rc;
  } else if (db->seq_bytes) {
    KernelScope ks(ctx, "copy_seq");
    HIP_OR_FAIL(hipMemcpyAsync(db->out, B.seq, (size_t)db->seq_bytes, hipMemcpyDeviceToDevice, st));
  }
  if (db->n_tiles_h) {
    if (!db->tn_tab && (rc = dmalloc(ctx, db->huge_allocs, &db->tn_tab, (size_t)db->tn_entries))) return rc;
    {
      KernelScope ks(ctx, "k_tile_large<1>");
      k_tile_large<1><<<db->n_tiles_h, kBlock, tile_lds_bytes(1), st>>>(
          B, db->tiles_h, nullptr, db->n_tiles_h, nullptr, db->large_incid, db->tab_off, db->tn_tab, db->scope_calls,
          db->rare_tile_list, db->counters + 1);
      if ((rc = check_launch(ctx, "k_tile_large<1>"))) return rc;
    }
    {
      // tiles that met a non-ACGTN base: re-run on the 16-code tally (count stays on the device)
      KernelScope ks(ctx, "k_tile_large<4>/rare");
      k_tile_large<4><<<std::min<int>(db->n_tiles_h, 1024), kBlock, tile_lds_bytes(4), st>>>(
          B, db->tiles_h, db->rare_tile_list, 0, db->counters + 1, db->large_incid, db->tab_off, db->tn_tab,
          db->scope_calls, nullptr, nullptr);
      if ((rc = check_launch(ctx, "k_tile_large<4>"))) return rc;
    }
    if (db->n_large_written_h) {
      KernelScope ks(ctx, "k_mask_large");
      const int grid = std::min<int>((db->n_large_written_h + kWaves - 1) / kWaves, 8192);
      k_mask_large<<<grid, kBlock, 0, st>>>(B, db->large_written_h, db->n_large_written_h, db->tab_off, db->tn_tab,
                                            db->out, db->scope_bases);
      if ((rc = check_launch(ctx, "k_mask_large"))) return rc;
    }
  }
  {
    // far masks, totals from the group partials and the huge scopes, counter reset
    KernelScope ks(ctx, "k_finish");
    k_finish<<<64, kBlock, 0, st>>>(static_cast<const unsigned long long *>(db->b_far.p), db->n_groups ? db->far_cap : 0,
                                    db->out, static_cast<const int32_t *>(db->b_grp_part.p), db->n_groups,
                                    db->large_ids, db->n_huge_scopes, db->scope_calls, db->scope_bases,
                                    db->static_totals, db->counters, db->far_count, db->status, db->acc, db->far_need,
                                    db->totals,
                                    static_cast<const unsigned long long *>(db->b_wspart.p), db->plan_info, db->gated);
    if ((rc = check_launch(ctx, "k_finish"))) return rc;
  }
  db->ran = true;
  return GANON_OK;
}

GANON_API int ganon_batch_sync(ganon_ctx *ctx) {
  if (!ctx) return GANON_E_ARG;
  HIP_OR_FAIL(ganon_detail::sync_stream(ctx->stream));
  if (ctx->profiling) {
    ctx->last_times.clear();
    for (auto &r : ctx->recs) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, r.e0, r.e1);
      auto it = std::find_if(ctx->last_times.begin(), ctx->last_times.end(),
                             [&](const ganon_kernel_time &t) { return r.name == t.name; });
      if (it == ctx->last_times.end()) {
        ganon_kernel_time t{};
        std::snprintf(t.name, sizeof t.name, "%s", r.name.c_str());
        t.launches = 1;
        t.ms = ms;
        ctx->last_times.push_back(t);
      } else {
        it->launches += 1;
        it->ms += ms;
      }
    }
  }
  return GANON_OK;
}

GANON_API int ganon_last_kernel_times(ganon_ctx *ctx, ganon_kernel_time *out, int max_k) {
  if (!ctx) return GANON_E_ARG;
  const int n = (int)ctx->last_times.size();
  for (int i = 0; i < n && i < max_k && out; ++i) out[i] = ctx->last_times[i];
  return n;
}

GANON_API int ganon_batch_download(ganon_ctx *ctx, ganon_dbatch *db, uint8_t *seq_out, int32_t *scope_calls_out,
                                   int32_t *scope_bases_out, int64_t *totals_out) {
  if (!ctx || !db) return fail(ctx, GANON_E_ARG, "null argument");
  if (!db->ran) return fail(ctx, GANON_E_STATE, "download before run");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  int rc;
  // the checks made during the run (incidences, write scopes)
  if ((rc = ganon_prep::batch_error(ctx, db))) return rc;
  int32_t status = 0;
  unsigned long long far_need = 0;
  HIP_OR_FAIL(ganon_detail::readback(&status, db->status, sizeof status, st));
  HIP_OR_FAIL(ganon_detail::readback(&far_need, db->far_need, sizeof far_need, st));
  HIP_OR_FAIL(ganon_detail::sync_stream(st));
  if (status & 4) {
    // a speculative replan the batch did not fit (a read with several segments, a longer read, a
    // huge scope): plan it in full and run it again
    const int sp = ctx->spec_plan;
    const bool prof = ctx->profiling;
    ctx->spec_plan = 0;
    ctx->profiling = false;
    rc = prepare(ctx, db, nullptr);
    if (!rc) rc = ganon_batch_run(ctx, db);
    ctx->spec_plan = sp;
    ctx->profiling = prof;
    if (rc) return rc;
    if ((rc = ganon_prep::batch_error(ctx, db))) return rc;
    HIP_OR_FAIL(ganon_detail::readback(&status, db->status, sizeof status, st));
    HIP_OR_FAIL(ganon_detail::readback(&far_need, db->far_need, sizeof far_need, st));
    HIP_OR_FAIL(ganon_detail::sync_stream(st));
  }
  if (status & 2) {
    // a written read its write scope does not list (or lists twice): name it
    if ((rc = ganon_prep::ws_diag(ctx, db)) || (rc = ganon_prep::batch_error(ctx, db))) return rc;
    return fail(ctx, GANON_E_ARG, "a written read is not listed exactly once by its write scope");
  }
  if (status & 1) {
    // the far-mask list overflowed: grow it to the count the run needed and run again (the list
    // keeps its capacity for later batches)
    if ((int64_t)far_need > kFarMaxEntries)
      return fail(ctx, GANON_E_NOMEM, "far-mask list: %llu entries needed (max %lld)", far_need, (long long)kFarMaxEntries);
    unsigned long long *far = nullptr;
    const int64_t cap = std::min<int64_t>(kFarMaxEntries, (int64_t)far_need + (int64_t)far_need / 4 + 1024);
    if ((rc = ganon_prep::grow_n(ctx, db->b_far, (size_t)cap, &far))) return rc;
    db->far_cap = db->far_cap_alloc = cap;
    db->aux_h.far = far;
    db->aux_h.far_cap = cap;
    HIP_OR_FAIL(hipMemcpyAsync(db->aux, &db->aux_h, sizeof db->aux_h, hipMemcpyHostToDevice, st));
    HIP_OR_FAIL(hipMemsetAsync(db->status, 0, sizeof(int32_t), st));
    HIP_OR_FAIL(hipMemsetAsync(db->far_need, 0, sizeof(unsigned long long), st));
    const bool prof = ctx->profiling;
    ctx->profiling = false;
    rc = ganon_batch_run(ctx, db);
    ctx->profiling = prof;
    if (rc) return rc;
    HIP_OR_FAIL(ganon_detail::readback(&status, db->status, sizeof status, st));
  }
  if (seq_out && db->seq_bytes)
    HIP_OR_FAIL(hipMemcpyAsync(seq_out, db->out, (size_t)db->seq_bytes, hipMemcpyDeviceToHost, st));
  if (scope_calls_out && db->n_scopes)
    HIP_OR_FAIL(hipMemcpyAsync(scope_calls_out, db->scope_calls, (size_t)db->n_scopes * 4, hipMemcpyDeviceToHost, st));
  if (scope_bases_out && db->n_scopes)
    HIP_OR_FAIL(hipMemcpyAsync(scope_bases_out, db->scope_bases, (size_t)db->n_scopes * 4, hipMemcpyDeviceToHost, st));
  if (totals_out)
    HIP_OR_FAIL(hipMemcpyAsync(totals_out, db->totals, GANON_N_TOTALS * 8, hipMemcpyDeviceToHost, st));
  HIP_OR_FAIL(ganon_detail::sync_stream(st));
  if (status & 1) return fail(ctx, GANON_E_STATE, "far-mask list overflowed after growing: output invalid");
  return GANON_OK;
}

GANON_API int ganon_batch_free(ganon_ctx *ctx, ganon_dbatch *db) {
  if (!db) return GANON_E_ARG;
  if (ctx) {
    hipSetDevice(ctx->device);
    ganon_detail::sync_stream(ctx->stream);
  }
  free_batch(db);
  delete db;
  return GANON_OK;
}

GANON_API int ganon_batch_device_totals(ganon_dbatch *db, void **dev_ptr) {
  if (!db || !dev_ptr) return GANON_E_ARG;
  *dev_ptr = db->totals;
  return GANON_OK;
}

GANON_API int ganon_batch_copy_totals(ganon_ctx *ctx, ganon_dbatch *db, void *dev_dst) {
  if (!ctx || !db || !dev_dst) return fail(ctx, GANON_E_ARG, "null argument");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  HIP_OR_FAIL(hipMemcpyAsync(dev_dst, db->totals, GANON_N_TOTALS * sizeof(int64_t), hipMemcpyDeviceToDevice,
                             ctx->stream));
  return GANON_OK;
}

GANON_API int ganon_batch_gated_runs(ganon_ctx *ctx, ganon_dbatch *db, int64_t *out) {
  if (!ctx || !db || !out) return fail(ctx, GANON_E_ARG, "null argument");
  if (!db->gated) return fail(ctx, GANON_E_STATE, "batch never loaded");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  unsigned long long g = 0;
  HIP_OR_FAIL(ganon_detail::readback(&g, db->gated, sizeof g, ctx->stream));
  HIP_OR_FAIL(ganon_detail::sync_stream(ctx->stream));
  *out = (int64_t)g;
  return GANON_OK;
}

GANON_API int ganon_batch_path_counts(ganon_ctx *ctx, ganon_dbatch *db, int64_t *out4) {
  if (!ctx || !db || !out4) return fail(ctx, GANON_E_ARG, "null argument");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  HIP_OR_FAIL(ganon_detail::readback(out4, db->paths, 4 * sizeof(int64_t), ctx->stream));
  HIP_OR_FAIL(ganon_detail::sync_stream(ctx->stream));
  return GANON_OK;
}

GANON_API int ganon_batch_info(ganon_dbatch *db, int64_t *info) {
  if (!db || !info) return GANON_E_ARG;
  info[0] = db->n_groups;
  info[1] = db->n_seg;
  info[2] = db->n_huge_scopes;
  info[3] = db->n_tiles_h;
  info[4] = db->far_cap;
  info[5] = db->n_large_written_h;
  info[6] = db->region;
  info[7] = db->n_written;
  return GANON_OK;
}

GANON_API int ganon_batch_shape(ganon_dbatch *db, int64_t *shape) {
  if (!db || !shape) return GANON_E_ARG;
  shape[0] = db->n_id_ops;
  shape[1] = db->max_len;
  shape[2] = db->max_seg;
  // (4: fused with multi-segment reads, found by a full plan; a speculative plan reports 3)
  shape[3] = db->long_mode ? 1 : db->flat_mode ? (db->fused ? (db->max_seg > 1 && !db->spec ? 4 : 3) : 2) : 0;
  return GANON_OK;
}

int ganon_dbatch_seq_buffers(const ganon_dbatch *db, const uint8_t **in, const uint8_t **out, int64_t *bytes) {
  if (!db) return GANON_E_ARG;
  *in = db->B.seq;
  *out = db->out;
  *bytes = db->seq_bytes;
  return GANON_OK;
}

int ganon_dbatch_read_view(const ganon_dbatch *db, GanonReadView *v) {
  if (!db || !v) return GANON_E_ARG;
  const DevBatch &B = db->B;
  v->ref_start = B.ref_start;
  v->read_len = B.read_len;
  v->read_end = B.read_end;
  v->n_cig = B.n_cig;
  v->write_scope = B.write_scope;
  v->seq_off = B.seq_off;
  v->cig_off = B.cig_off;
  v->seq = B.seq;
  v->dataset = B.dataset;
  v->cigar = B.cigar;
  v->incid_off = B.incid_off;
  v->incid_read = B.incid_read;
  v->span_start = B.span_start;
  v->span_len = B.span_len;
  v->n_reads = db->n_reads;
  v->n_scopes = db->n_scopes;
  return GANON_OK;
}

GANON_API int ganon_mask_batch(ganon_ctx *ctx, const ganon_batch *batch, uint8_t *seq_out, int32_t *scope_calls_out,
                               int32_t *scope_bases_out, int64_t *totals_out) {
  if (!ctx || !batch || (!seq_out && batch->seq_bytes)) return fail(ctx, GANON_E_ARG, "null argument");
  ganon_dbatch *db = nullptr;
  int rc = ganon_batch_upload(ctx, batch, &db);
  if (rc) return rc;
  rc = ganon_batch_run(ctx, db);
  if (!rc) rc = ganon_batch_sync(ctx);
  if (!rc) rc = ganon_batch_download(ctx, db, seq_out, scope_calls_out, scope_bases_out, totals_out);
  ganon_batch_free(ctx, db);
  return rc;
}
