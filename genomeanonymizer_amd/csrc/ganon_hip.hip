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
// Design: integer/byte work, HBM-bound — no MFMA. One workgroup owns one
// scope (or a 16 Ki-position tile of a wide scope). The scope's reference slice and a
// per-position tally live in LDS: 1 byte per position (tumor ACGT nibble | normal ACGT
// nibble, updated with ds_or_b32 on the containing dword). nt16 codes of A, C, G, T are
// one-hot (1, 2, 4, 8), so a nibble IS the allele set and TN = tumor & normal.
// Non-ACGTN read bases ("=" and IUPAC codes) are rare; a scope that meets one is re-run
// on a 16-code tally (4 bytes per position: tumor code mask | normal code mask << 16).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <type_traits>
#include <thread>
#include <vector>

#include "../../include/ganon.h"
#include "ganon_ctx.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kSmallCap0 = 2560;    // positions, class 0 (window scopes: 2001 + read overhang)
constexpr int kSmallCap1 = 16384;   // positions, class 1 (= wide cap)
constexpr int kTile = 16384;        // positions per tile of a large scope
constexpr int kPersistGrid = 1024;  // grid of the device-counted (rare) re-run kernels

struct Tile {
  int32_t scope;
  int32_t a;      // tile covers [a, b) (contig positions)
  int32_t b;
  int32_t pad;
  int64_t lo;     // candidate range in large_incid
  int64_t hi;
};

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
  const uint32_t *ref2;   // 2-bit reference (k_ref2) for the group kernels, null = nt16 only
};

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

// ---- kernels ---------------------------------------------------------------------------

// Reads written unmasked (write_scope == -1): plain copy.
__global__ void __launch_bounds__(kBlock) k_passthrough(const DevBatch B, const int32_t *__restrict__ list,
                                                        int n, uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int gw = (blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int nw = (gridDim.x * kBlock) >> 6;
  for (int i = gw; i < n; i += nw) {
    const int r = list[i];
    const int64_t so = B.seq_off[r];
    const int nbytes = (B.read_len[r] + 1) >> 1;
    for (int j = lane; j < nbytes; j += 64) out[so + j] = B.seq[so + j];
  }
}

// One workgroup per small scope (span <= cap): tally -> classify -> mask, all in LDS.
// count_ptr != nullptr: the list length lives on the device (re-run of rare scopes).
template <int TB>
__global__ void __launch_bounds__(kBlock) k_scope_small(const DevBatch B, const int32_t *__restrict__ list,
                                                        int n_static, const int32_t *count_ptr, int cap,
                                                        uint8_t *__restrict__ out, int32_t *scope_calls,
                                                        int32_t *scope_bases, int32_t *rare_list,
                                                        int32_t *rare_count) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int tab_words = cap * TB / 4;
  uint32_t *tab = smem;
  uint8_t *refb = reinterpret_cast<uint8_t *>(smem + tab_words);
  int *scratch = reinterpret_cast<int *>(refb + ((cap / 2 + 15) & ~15));
  const int n = count_ptr ? *count_ptr : n_static;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int li = blockIdx.x; li < n; li += gridDim.x) {
    const int s = list[li];
    const int a = B.span_start[s];
    const int span = B.span_len[s];
    const int b = a + span;
    const int words = (span * TB + 3) >> 2;
    for (int w = threadIdx.x; w < words; w += kBlock) tab[w] = 0;
    stage_ref(B, B.ref_off[s], span, refb);
    if (threadIdx.x == 0) scratch[kWaves] = 0;
    __syncthreads();
    const int64_t i0 = B.incid_off[s], i1 = B.incid_off[s + 1];
    bool rare = false;
    const LdsRef refn{refb, a};
    for (int64_t i = i0 + wave; i < i1; i += kWaves) rare |= tally_read<TB>(B, B.incid_read[i], a, b, tab, refn, lane);
    if (TB == 1 && rare) scratch[kWaves] = 1;
    __syncthreads();
    clear_keep<TB>(B, s, a, b, tab);
    __syncthreads();
    int calls = 0;
    for (int off = threadIdx.x; off < span; off += kBlock) calls += tn_count<TB>(tn_mask<TB>(tab, off));
    calls = block_sum(calls, scratch);
    int bases = 0;
    for (int64_t i = i0 + wave; i < i1; i += kWaves) {
      const int r = B.incid_read[i];
      if (B.write_scope[r] != s) continue;
      bases += mask_read_lds<TB>(B, r, a, tab, refn, out, lane);
    }
    bases = block_sum(bases, scratch);
    if (threadIdx.x == 0) {
      scope_calls[s] = calls;
      scope_bases[s] = bases;
      if (TB == 1 && scratch[kWaves]) rare_list[atomicAdd(rare_count, 1)] = s;
    }
    __syncthreads();
  }
}

// One WAVE per small scope (the common case: ~2.3 kb spans, a handful to a few hundred
// reads). Reads are taken 64 at a time: each lane loads one read's metadata, reads with a
// single M/=/X op covering the whole sequence ("simple", ~all short reads) are compacted
// into LDS and processed four at a time by 16-lane groups (one packed byte = two bases
// per lane step); reads with any other CIGAR go through the per-read cursor walk. The
// reference nibbles come straight from the packed genome (no staging), the tally is the
// 1-byte-per-position LDS table. Same results as k_scope_small<1>.
constexpr int kMetaLds = 64 * (4 * 4 + 8);

__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__global__ void __launch_bounds__(64) k_scope_wave(const DevBatch B, const int32_t *__restrict__ list, int n,
                                                   int cap, uint8_t *__restrict__ out, int32_t *scope_calls,
                                                   int32_t *scope_bases, int32_t *rare_list, int32_t *rare_count) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t *tab = smem;
  int *m_start = reinterpret_cast<int *>(smem + cap / 4);
  int *m_len = m_start + 64;
  int *m_ds = m_len + 64;
  int64_t *m_off = reinterpret_cast<int64_t *>(m_ds + 128);
  const int lane = threadIdx.x;
  for (int li = blockIdx.x; li < n; li += gridDim.x) {
    const int s = list[li];
    const int a = B.span_start[s];
    const int span = B.span_len[s];
    const int b = a + span;
    const GlobalRef refn{B.ref, B.ref_off[s] - a};
    uint4 *t4 = reinterpret_cast<uint4 *>(tab);
    for (int k = lane; k < ((span + 15) >> 4); k += 64) t4[k] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const int64_t i0 = B.incid_off[s], i1 = B.incid_off[s + 1];
    bool rare = false;
    // ---- tally ------------------------------------------------------------------------
    for (int64_t c0 = i0; c0 < i1; c0 += 64) {
      const int nh = (int)((i1 - c0) < 64 ? (i1 - c0) : 64);
      int r = 0;
      bool simple = false, cplx = false;
      if (lane < nh) {
        r = B.incid_read[c0 + lane];
        const int L = B.read_len[r];
        const int nc = B.n_cig[r];
        if (nc == 1) {
          const uint32_t w = B.cigar[B.cig_off[r]];
          const int op = w & 15;
          simple = (op == 0 || op == 7 || op == 8) && (int)(w >> 4) == L && L > 0;
        }
        cplx = !simple && nc > 0 && L > 0;
      }
      const uint64_t sm = __ballot(simple);
      if (simple) {
        const int idx = __popcll(sm & lanes_below(lane));
        m_start[idx] = B.ref_start[r];
        m_len[idx] = B.read_len[r];
        m_ds[idx] = B.dataset[r];
        m_off[idx] = B.seq_off[r];
      }
      __syncthreads();
      const int ns = __popcll(sm);
      for (int j0 = 0; j0 < ns; j0 += 4) {
        const int j = j0 + (lane >> 4);
        if (j >= ns) continue;
        const int st = m_start[j], L = m_len[j], d = m_ds[j];
        const int64_t so = m_off[j];
        const int nb = (L + 1) >> 1;
        for (int bi = lane & 15; bi < nb; bi += 16) {
          const uint32_t byte = B.seq[so + bi];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int q = 2 * bi + h;
            if (q >= L) break;
            const int c = h ? (byte & 15) : (byte >> 4);
            const int p = st + q;
            const int rc = refn(p);
            if (c == 15 || c == rc || !is_acgt(rc)) continue;
            if (is_acgt(c)) {
              const int off = p - a;
              atomicOr(&tab[off >> 2], (uint32_t)c << (d * 4 + (off & 3) * 8));
            } else {
              rare = true;
            }
          }
        }
      }
      uint64_t cm = __ballot(cplx);
      while (cm) {
        const int l = __ffsll((unsigned long long)cm) - 1;
        cm &= cm - 1;
        const int rr = __shfl(r, l);
        rare |= tally_read<1>(B, rr, a, b, tab, refn, lane);
      }
      __syncthreads();
    }
    // ---- classify: kept allele out, count TN calls --------------------------------------
    clear_keep<1>(B, s, a, b, tab);
    __syncthreads();
    int calls = 0;
    for (int k = lane; k < ((span + 3) >> 2); k += 64) {
      const uint32_t w = tab[k];
      calls += __popc(w & (w >> 4) & 0x0F0F0F0Fu);
    }
    // ---- mask the reads this scope writes -------------------------------------------------
    int bases = 0;
    for (int64_t c0 = i0; c0 < i1; c0 += 64) {
      const int nh = (int)((i1 - c0) < 64 ? (i1 - c0) : 64);
      int r = 0;
      bool simple = false, cplx = false;
      if (lane < nh) {
        r = B.incid_read[c0 + lane];
        if (B.write_scope[r] == s) {
          const int L = B.read_len[r];
          const int nc = B.n_cig[r];
          if (nc == 1) {
            const uint32_t w = B.cigar[B.cig_off[r]];
            const int op = w & 15;
            simple = (op == 0 || op == 7 || op == 8) && (int)(w >> 4) == L && L > 0;
          }
          cplx = !simple && L > 0;
        }
      }
      const uint64_t sm = __ballot(simple);
      if (simple) {
        const int idx = __popcll(sm & lanes_below(lane));
        m_start[idx] = B.ref_start[r];
        m_len[idx] = B.read_len[r];
        m_off[idx] = B.seq_off[r];
      }
      __syncthreads();
      const int ns = __popcll(sm);
      for (int j0 = 0; j0 < ns; j0 += 4) {
        const int j = j0 + (lane >> 4);
        if (j >= ns) continue;
        const int st = m_start[j], L = m_len[j];
        const int64_t so = m_off[j];
        const int nb = (L + 1) >> 1;
        for (int bi = lane & 15; bi < nb; bi += 16) {
          const uint32_t byte = B.seq[so + bi];
          int nib[2] = {(int)(byte >> 4), (int)(byte & 15)};
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int q = 2 * bi + h;
            if (q >= L) break;
            const int off = st + q - a;
            const uint32_t t = (tab[off >> 2] >> ((off & 3) * 8)) & 0xFF;
            const uint32_t tn = t & (t >> 4) & 15;
            if (tn && is_acgt(nib[h]) && (tn & (uint32_t)nib[h])) {
              nib[h] = refn(st + q);
              ++bases;
            }
          }
          out[so + bi] = (uint8_t)((nib[0] << 4) | nib[1]);
        }
      }
      uint64_t cm = __ballot(cplx);
      while (cm) {
        const int l = __ffsll((unsigned long long)cm) - 1;
        cm &= cm - 1;
        const int rr = __shfl(r, l);
        bases += mask_read_lds<1>(B, rr, a, tab, refn, out, lane);
      }
      __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) {
      calls += __shfl_xor(calls, o);
      bases += __shfl_xor(bases, o);
    }
    const bool any_rare = __ballot(rare) != 0;
    if (lane == 0) {
      scope_calls[s] = calls;
      scope_bases[s] = bases;
      if (any_rare) rare_list[atomicAdd(rare_count, 1)] = s;
    }
    __syncthreads();
  }
}

// ---- v2: copy-then-patch ----------------------------------------------------------------
// The output starts as a device copy of the input bases (one streaming memcpy); the scope
// kernel only reads. Per incidence a 16-byte record (built at upload, scope-major, so a
// scope's records are one coalesced load) says where the read is and whether this scope
// writes it. Simple reads are taken 16 nibbles per lane (three aligned dword loads each for
// the read and the reference, nibble-swapped so nibble k sits at bits 4k), mismatches go
// to the LDS tally AND to a short LDS observation list; after classification only the
// observations that hit a TN call in a read this scope writes are patched in place
// (atomicXor on the containing dword: neighbouring reads' bytes are untouched).
constexpr int kObsCap = 256;
constexpr uint32_t kRecSimple = 1u << 25, kRecMine = 1u << 26, kRecCplx = 1u << 27;

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

struct ObsList {
  uint32_t *meta;   // off | c << 16 | ds << 20 | mine << 21
  int64_t *nib;     // nibble index of the base in the sequence buffer
  int *count;       // [0] entries, [1] overflow flag
  int cap = kObsCap;
  __device__ __forceinline__ void add(int off, int c, int ds, bool mine, int64_t nib_index) {
    const int k = atomicAdd(count, 1);
    if (k < cap) {
      meta[k] = (uint32_t)off | ((uint32_t)c << 16) | ((uint32_t)ds << 20) | ((uint32_t)mine << 21);
      nib[k] = nib_index;
    } else {
      count[1] = 1;
    }
  }
};

__device__ __forceinline__ void patch_nibble(uint8_t *out, int64_t nib_index, int from, int to) {
  const int64_t byte = nib_index >> 1;
  const int sh = 8 * (int)(byte & 3) + ((nib_index & 1) ? 0 : 4);
  atomicXor(reinterpret_cast<uint32_t *>(out) + (byte >> 2), (uint32_t)(from ^ to) << sh);
}

// One observation of base c at position p (offset off in the table) of dataset ds.
__device__ __forceinline__ bool observe(uint32_t *tab, ObsList &obs, int off, int c, int rc, int ds, bool mine,
                                        int64_t nib_index) {
  if (c == 15 || c == rc || !is_acgt(rc)) return false;
  if (!is_acgt(c)) return true;                       // rare: 16-code re-run
  atomicOr(&tab[off >> 2], (uint32_t)c << (ds * 4 + (off & 3) * 8));
  obs.add(off, c, ds, mine, nib_index);
  return false;
}

__global__ void __launch_bounds__(64) k_scope_v2(const DevBatch B, const int4 *__restrict__ inc_rec,
                                                 const int32_t *__restrict__ list, int n, int cap,
                                                 uint8_t *__restrict__ out, int32_t *scope_calls,
                                                 int32_t *scope_bases, int32_t *rare_list, int32_t *rare_count) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t *tab = smem;
  int *m_start = reinterpret_cast<int *>(smem + cap / 4);
  int *m_len = m_start + 64;
  int *m_ds = m_len + 64;
  int *m_mine = m_ds + 64;
  int64_t *m_off = reinterpret_cast<int64_t *>(m_mine + 64);
  ObsList obs;
  obs.meta = reinterpret_cast<uint32_t *>(m_off + 64);
  obs.nib = reinterpret_cast<int64_t *>(obs.meta + kObsCap);
  obs.count = reinterpret_cast<int *>(obs.nib + kObsCap);
  const int lane = threadIdx.x;
  for (int li = blockIdx.x; li < n; li += gridDim.x) {
    const int s = list[li];
    const int a = B.span_start[s];
    const int span = B.span_len[s];
    const int b = a + span;
    const int64_t rnib0 = B.ref_off[s] - a;            // nibble index of contig position 0
    const GlobalRef refn{B.ref, rnib0};
    uint4 *t4 = reinterpret_cast<uint4 *>(tab);
    for (int k = lane; k < ((span + 15) >> 4); k += 64) t4[k] = make_uint4(0u, 0u, 0u, 0u);
    if (lane < 2) obs.count[lane] = 0;
    __syncthreads();
    const int64_t i0 = B.incid_off[s], i1 = B.incid_off[s + 1];
    bool rare = false;
    for (int64_t c0 = i0; c0 < i1; c0 += 64) {
      const int nh = (int)((i1 - c0) < 64 ? (i1 - c0) : 64);
      int4 rec = make_int4(0, 0, 0, 0);
      if (lane < nh) rec = inc_rec[c0 + lane];
      const uint32_t fl = (uint32_t)rec.y;
      const bool simple = (fl & kRecSimple) != 0;
      const bool cplx = (fl & kRecCplx) != 0;
      const uint64_t sm = __ballot(simple);
      if (simple) {
        const int idx = __popcll(sm & lanes_below(lane));
        m_start[idx] = rec.x;
        m_len[idx] = (int)(fl & 0xFFFFFF);
        m_ds[idx] = (int)((fl >> 24) & 1);
        m_mine[idx] = (fl & kRecMine) ? 1 : 0;
        m_off[idx] = (int64_t)(((uint64_t)(uint32_t)rec.w << 32) | (uint32_t)rec.z);
      }
      __syncthreads();
      const int ns = __popcll(sm);
      for (int j0 = 0; j0 < ns; j0 += 4) {
        const int j = j0 + (lane >> 4);
        if (j >= ns) continue;
        const int st = m_start[j], L = m_len[j], d = m_ds[j];
        const bool mine = m_mine[j] != 0;
        const int64_t snib = 2 * m_off[j];
        for (int q0 = 16 * (lane & 15); q0 < L; q0 += 256) {
          const uint64_t sv = load16(B.seq, snib + q0);
          const uint64_t rv = load16(B.ref, rnib0 + st + q0);
          const int nb = (L - q0) < 16 ? (L - q0) : 16;
          // nibbles that differ from the reference (cheap pre-filter: usually none)
          uint64_t diff = sv ^ rv;
          diff = (diff | (diff >> 1) | (diff >> 2) | (diff >> 3)) & 0x1111111111111111ull;
          if (nb < 16) diff &= (1ull << (4 * nb)) - 1;
          while (diff) {
            const int k = __builtin_ctzll(diff) >> 2;
            diff &= diff - 1;
            const int c = (int)((sv >> (4 * k)) & 15);
            const int rc = (int)((rv >> (4 * k)) & 15);
            rare |= observe(tab, obs, st + q0 + k - a, c, rc, d, mine, snib + q0 + k);
          }
        }
      }
      uint64_t cm = __ballot(cplx);
      while (cm) {
        const int l = __ffsll((unsigned long long)cm) - 1;
        cm &= cm - 1;
        const int r = __shfl(rec.x, l);
        const bool mine = (__shfl((int)fl, l) & kRecMine) != 0;
        const int L = B.read_len[r];
        const int ds = B.dataset[r];
        const int64_t snib = 2 * B.seq_off[r];
        CigarCursor cur;
        cur.init(B.cigar + B.cig_off[r], B.n_cig[r], B.ref_start[r]);
        for (int q = lane; q < L; q += 64) {
          const int p = cur.ref_of(q);
          if (p < a || p >= b) continue;
          rare |= observe(tab, obs, p - a, nib_at(B.seq, snib + q), refn(p), ds, mine, snib + q);
        }
      }
      __syncthreads();
    }
    clear_keep<1>(B, s, a, b, tab);
    __syncthreads();
    int calls = 0;
    for (int k = lane; k < ((span + 3) >> 2); k += 64) {
      const uint32_t w = tab[k];
      calls += __popc(w & (w >> 4) & 0x0F0F0F0Fu);
    }
    int bases = 0;
    const int n_obs = obs.count[0] < kObsCap ? obs.count[0] : kObsCap;
    if (!obs.count[1]) {
      for (int e = lane; e < n_obs; e += 64) {
        const uint32_t m = obs.meta[e];
        if (!(m & (1u << 21))) continue;
        const int off = (int)(m & 0xFFFF), c = (int)((m >> 16) & 15);
        const uint32_t t = (tab[off >> 2] >> ((off & 3) * 8)) & 0xFF;
        if (t & (t >> 4) & (uint32_t)c) {
          patch_nibble(out, obs.nib[e], c, refn(a + off));
          ++bases;
        }
      }
    } else {
      // more mismatches than the list holds: walk the reads this scope writes again
      for (int64_t i = i0; i < i1; ++i) {
        const int4 rec = inc_rec[i];
        if (!(rec.y & kRecMine)) continue;
        const int r = B.incid_read[i];
        const int L = B.read_len[r];
        const int64_t snib = 2 * B.seq_off[r];
        CigarCursor cur;
        cur.init(B.cigar + B.cig_off[r], B.n_cig[r], B.ref_start[r]);
        for (int q = lane; q < L; q += 64) {
          const int p = cur.ref_of(q);
          if (p < a || p >= b) continue;
          const int c = nib_at(B.seq, snib + q);
          const int off = p - a;
          const uint32_t t = (tab[off >> 2] >> ((off & 3) * 8)) & 0xFF;
          if (is_acgt(c) && (t & (t >> 4) & (uint32_t)c)) {
            patch_nibble(out, snib + q, c, refn(p));
            ++bases;
          }
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      calls += __shfl_xor(calls, o);
      bases += __shfl_xor(bases, o);
    }
    const bool any_rare = __ballot(rare) != 0;
    if (lane == 0) {
      scope_calls[s] = calls;
      scope_bases[s] = bases;
      if (any_rare) rare_list[atomicAdd(rare_count, 1)] = s;
    }
    __syncthreads();
  }
}

size_t v2_lds_bytes(int cap) {
  return (size_t)cap + 64 * (4 * 4 + 8) + kObsCap * (4 + 8) + 16;
}

// ---- v3: persistent waves ------------------------------------------------------------------
// v2's algorithm with the latency chain cut down: 256-thread workgroups whose four waves
// work independently (wave-level sync only), a persistent grid in which every wave walks
// its own stream of scopes and prefetches the next scope's 48-byte record while it works
// on the current one, and simple reads spread over the lanes chunk by chunk (16 bases per
// lane, chunk -> read by binary search over an LDS prefix array) so six 150 bp reads fill
// one 64-lane pass. LDS per wave stays under 5 KB for the 2.5 K class (32 waves per CU).
constexpr int kV3Obs = 96;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__host__ __device__ inline size_t v3_wave_lds_bytes(int cap) {
  return (size_t)cap + 64 * 16 + 68 * 4 + kV3Obs * (4 + 8) + 16;
}

__device__ __forceinline__ int64_t i64_of(int lo, int hi) {
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__global__ void __launch_bounds__(256) k_scope_v3(const DevBatch B, const int4 *__restrict__ srec, int n, int cap,
                                                  const int4 *__restrict__ inc_rec, uint8_t *__restrict__ out,
                                                  int32_t *scope_calls, int32_t *scope_bases, int32_t *rare_list,
                                                  int32_t *rare_count) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  // wave index made provably wave-uniform: scope records then live in SGPRs (s_load)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t *base = smem + wave * (v3_wave_lds_bytes(cap) / 4);
  uint32_t *tab = base;
  int4 *mrec = reinterpret_cast<int4 *>(base + cap / 4);
  int *mcs = reinterpret_cast<int *>(mrec + 64);
  ObsList obs;
  obs.meta = reinterpret_cast<uint32_t *>(mcs + 68);
  obs.nib = reinterpret_cast<int64_t *>(obs.meta + kV3Obs);
  obs.count = reinterpret_cast<int *>(obs.nib + kV3Obs);
  obs.cap = kV3Obs;
  const int nw = gridDim.x * 4;
  int li = blockIdx.x * 4 + wave;
  int4 ra = make_int4(0, 0, 0, 0), rb = ra, rc = ra;
  if (li < n) {
    ra = srec[3 * li];
    rb = srec[3 * li + 1];
    rc = srec[3 * li + 2];
  }
  while (li < n) {
    const int nli = li + nw;
    int4 na = make_int4(0, 0, 0, 0), nb = na, nc = na;
    if (nli < n) {                                   // prefetch the next scope's record
      na = srec[3 * nli];
      nb = srec[3 * nli + 1];
      nc = srec[3 * nli + 2];
    }
    const int s = ra.x, a = ra.y, span = ra.z, keep_pos = ra.w;
    const int64_t i0 = i64_of(rb.x, rb.y);
    const int ninc = rb.z, keep_code = rb.w;
    const int64_t rnib0 = i64_of(rc.x, rc.y);      // nibble index of contig position 0
    const int b = a + span;
    const GlobalRef refn{B.ref, rnib0};
    uint4 *t4 = reinterpret_cast<uint4 *>(tab);
    for (int k = lane; k < ((span + 15) >> 4); k += 64) t4[k] = make_uint4(0u, 0u, 0u, 0u);
    if (lane < 2) obs.count[lane] = 0;
    wave_sync();
    bool rare = false;
    for (int c0 = 0; c0 < ninc; c0 += 64) {
      const int nh = (ninc - c0) < 64 ? (ninc - c0) : 64;
      int4 rec = make_int4(0, 0, 0, 0);
      if (lane < nh) rec = inc_rec[i0 + c0 + lane];
      const uint32_t fl = (uint32_t)rec.y;
      const bool simple = (fl & kRecSimple) != 0;
      const bool cplx = (fl & kRecCplx) != 0;
      const int nck = simple ? (int)(((fl & 0xFFFFFF) + 15) >> 4) : 0;
      int incl = nck;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
      }
      const int total = __shfl(incl, 63);
      mrec[lane] = rec;
      mcs[lane] = incl - nck;
      wave_sync();
      for (int t = lane; t < total; t += 64) {
        int lo = 0, hi = 63;                         // largest j with mcs[j] <= t
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (mcs[mid] <= t) lo = mid;
          else hi = mid - 1;
        }
        const int4 r = mrec[lo];
        const int q0 = 16 * (t - mcs[lo]);
        const uint32_t rf = (uint32_t)r.y;
        const int L = (int)(rf & 0xFFFFFF), d = (int)((rf >> 24) & 1);
        const bool mine = (rf & kRecMine) != 0;
        const int64_t snib = 2 * i64_of(r.z, r.w);
        const uint64_t sv = load16(B.seq, snib + q0);
        const uint64_t rv = load16(B.ref, rnib0 + r.x + q0);
        const int nbase = (L - q0) < 16 ? (L - q0) : 16;
        uint64_t diff = sv ^ rv;
        diff = (diff | (diff >> 1) | (diff >> 2) | (diff >> 3)) & 0x1111111111111111ull;
        if (nbase < 16) diff &= (1ull << (4 * nbase)) - 1;
        while (diff) {
          const int k = __builtin_ctzll(diff) >> 2;
          diff &= diff - 1;
          rare |= observe(tab, obs, r.x + q0 + k - a, (int)((sv >> (4 * k)) & 15), (int)((rv >> (4 * k)) & 15), d,
                          mine, snib + q0 + k);
        }
      }
      uint64_t cm = __ballot(cplx);
      while (cm) {
        const int l = __ffsll((unsigned long long)cm) - 1;
        cm &= cm - 1;
        const int r = __shfl(rec.x, l);
        const bool mine = (__shfl((int)fl, l) & kRecMine) != 0;
        const int L = B.read_len[r];
        const int ds = B.dataset[r];
        const int64_t snib = 2 * B.seq_off[r];
        CigarCursor cur;
        cur.init(B.cigar + B.cig_off[r], B.n_cig[r], B.ref_start[r]);
        for (int q = lane; q < L; q += 64) {
          const int p = cur.ref_of(q);
          if (p < a || p >= b) continue;
          rare |= observe(tab, obs, p - a, nib_at(B.seq, snib + q), refn(p), ds, mine, snib + q);
        }
      }
      wave_sync();
    }
    if (lane == 0 && keep_pos >= a && keep_pos < b && is_acgt(keep_code)) {
      const int off = keep_pos - a;
      atomicAnd(&tab[off >> 2], ~((uint32_t)keep_code << ((off & 3) * 8)));
    }
    wave_sync();
    int calls = 0;
    for (int k = lane; k < ((span + 3) >> 2); k += 64) {
      const uint32_t w = tab[k];
      calls += __popc(w & (w >> 4) & 0x0F0F0F0Fu);
    }
    int bases = 0;
    const int n_obs = obs.count[0] < kV3Obs ? obs.count[0] : kV3Obs;
    if (obs.count[0] <= kV3Obs) {
      for (int e = lane; e < n_obs; e += 64) {
        const uint32_t m = obs.meta[e];
        if (!(m & (1u << 21))) continue;
        const int off = (int)(m & 0xFFFF), c = (int)((m >> 16) & 15);
        const uint32_t t = (tab[off >> 2] >> ((off & 3) * 8)) & 0xFF;
        if (t & (t >> 4) & (uint32_t)c) {
          patch_nibble(out, obs.nib[e], c, refn(a + off));
          ++bases;
        }
      }
    } else {
      // more mismatches than the list holds: walk the reads this scope writes again
      for (int64_t i = i0; i < i0 + ninc; ++i) {
        const int4 rec = inc_rec[i];
        if (!(rec.y & kRecMine)) continue;
        const int r = B.incid_read[i];
        const int L = B.read_len[r];
        const int64_t snib = 2 * B.seq_off[r];
        CigarCursor cur;
        cur.init(B.cigar + B.cig_off[r], B.n_cig[r], B.ref_start[r]);
        for (int q = lane; q < L; q += 64) {
          const int p = cur.ref_of(q);
          if (p < a || p >= b) continue;
          const int c = nib_at(B.seq, snib + q);
          const int off = p - a;
          const uint32_t t = (tab[off >> 2] >> ((off & 3) * 8)) & 0xFF;
          if (is_acgt(c) && (t & (t >> 4) & (uint32_t)c)) {
            patch_nibble(out, snib + q, c, refn(p));
            ++bases;
          }
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      calls += __shfl_xor(calls, o);
      bases += __shfl_xor(bases, o);
    }
    const bool any_rare = __ballot(rare) != 0;
    if (lane == 0) {
      scope_calls[s] = calls;
      scope_bases[s] = bases;
      if (any_rare) rare_list[atomicAdd(rare_count, 1)] = s;
    }
    wave_sync();
    ra = na;
    rb = nb;
    rc = nc;
    li = nli;
  }
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
constexpr int kGrpTarget = 256;      // segments per group (a larger scope forms its own group)
constexpr int kGrpObs = 512;         // observations per LDS list
constexpr int kGrpMaxScopes = 256;   // scopes per group (12-bit local index field)
constexpr int kGrpStack = 80;        // key ranges pending (bisection depth <= 64)
constexpr int kGrpPatch = 512;       // in-partition masks of one list pass (<= its observations)
constexpr int kGrpMap = 4096;        // chunk -> segment map entries (larger tiles binary-search)
constexpr int kGrpQuad = 256;        // lists up to this size are matched without sorting
constexpr int kGrpMaxSpan = 1 << 20; // widest scope of the group kernels (20-bit position field)
constexpr unsigned long long kEmpty = ~0ull;
constexpr int64_t kPartAlign = 128;  // partition boundaries fall on whole lines
constexpr int kGrpRec = 5;           // int4 records per group (layout at k_group)
// segment record (int4, 16 bytes): x = query nibble bits 0-31, y = reference nibble bits 0-31,
// z = query nibble bits 32-39 | reference nibble bits 32-39 << 8 | length << 16 (14 bits) |
// dataset << 30 | mine << 31, w = scope_local | (pos - span_start) << 12
constexpr int kSegMaxLen = (1 << 14) - 1;   // longer aligned runs are cut into pieces at upload
constexpr uint32_t kSegMine = 1u << 31;     // the segment's read is written by this scope
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

struct GrpShared {
  int4 rec[kGrpTile];               // segment records (layout at kSegMine)
  int pre[kGrpTile];
  uint8_t cmap[kGrpMap];            // staged segment of each chunk (tiles of <= kGrpMap chunks)
  int wsum[kGrpThreads / 64];
  unsigned long long key[kGrpObs];   // observation list
  unsigned long long pay[kGrpObs];
  unsigned long long patch[kGrpPatch];   // nibble index << 4 | (from ^ to)
  unsigned long long stk_lo[kGrpStack], stk_hi[kGrpStack];
  int stk_mode[kGrpStack];
  unsigned long long kmin, kmax;
  int top, n_obs, n_patch;
  int blk_calls, blk_bases;         // this workgroup's contribution to the totals
  int cnt_calls[kGrpMaxScopes];     // per-scope counts, written out once at the end
  int cnt_bases[kGrpMaxScopes];
};

struct GrpRange {
  unsigned long long lo, hi;
  int mode;
};

// Where a masked base goes.
// Rarely used outputs and scratch of the group kernels, read through one pointer (device
// memory) so that their addresses do not occupy scalar registers for the whole kernel.
struct GrpAux {
  int32_t *scope_calls, *scope_bases, *part;   // per-scope counts; per-workgroup partial totals
  unsigned long long *far;                      // fused: masks of bytes outside the partition
  int *far_count;
  int64_t far_cap;
  unsigned long long *okey, *opay, *tkey;       // overflow regions (GrpGlobal)
  unsigned int *tflag;
};

struct PatchSink {
  uint8_t *out;
  int64_t p0, p1, q0, q1;           // fused: this workgroup's partition pieces of out (bytes)
  const GrpAux *aux;                // far-mask list
  bool fused;
  bool lds;                         // fused: in-partition masks into the LDS list
  __device__ bool inside(int64_t byte) const { return (byte >= p0 && byte < p1) || (byte >= q0 && byte < q1); }
};

__device__ __forceinline__ void sink_patch(GrpShared &sh, const PatchSink &k, int64_t nib, int c, int rc) {
  const unsigned long long e = ((unsigned long long)nib << 4) | (unsigned long long)(c ^ rc);
  if (k.fused) {
    const int64_t byte = nib >> 1;
    if (!k.inside(byte)) {
      const int i = atomicAdd(k.aux->far_count, 1);
      if (i < k.aux->far_cap) k.aux->far[i] = e;
      return;
    }
    if (k.lds) {
      const int i = atomicAdd(&sh.n_patch, 1);
      if (i < kGrpPatch) sh.patch[i] = e;
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

__device__ __forceinline__ void grp_count(GrpShared &sh, int s_local, int calls, int bases);

// payload: nibble index:48 | ref:4 | dataset:1 | mine:1
__device__ __forceinline__ void grp_observe(GrpShared &sh, const GrpRange &R, const GrpGlobal &gg,
                                            unsigned long long key, int64_t nib, int rc, int ds, uint32_t mine) {
  if (key < R.lo || key >= R.hi) return;
  const unsigned long long pay = (unsigned long long)nib | ((unsigned long long)rc << 48) |
                                 ((unsigned long long)ds << 52) | ((unsigned long long)mine << 53);
  const int k = atomicAdd(&sh.n_obs, 1);
  if (k < kGrpObs) {
    sh.key[k] = key;
    sh.pay[k] = pay;
  } else {
    // past the LDS list: straight into the group's global region (no second scan)
    if (k - kGrpObs < gg.cap - kGrpObs) {
      gg.aux->okey[gg.off + (k - kGrpObs)] = key;
      gg.aux->opay[gg.off + (k - kGrpObs)] = pay;
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

// Stage records [c0, c0 + nh) in LDS with the exclusive prefix of their chunk counts;
// returns the tile's chunk total.
__device__ __forceinline__ int grp_tile(GrpShared &sh, const int4 *__restrict__ rec4, int64_t c0, int nh,
                                        int chunk) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t ix = c0 + (tid < nh ? tid : nh - 1);
  const int4 r = rec4[ix];
  int nck = 0;
  if (tid < nh) {
    sh.rec[tid] = r;
    nck = ((((uint32_t)r.z >> 16) & kSegMaxLen) + chunk - 1) / chunk;
  }
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

// The staged segment owning chunk t (largest j with pre[j] <= t).
__device__ __forceinline__ int grp_find(const GrpShared &sh, int nh, int total, int t) {
  if (total <= kGrpMap) return sh.cmap[t];
  int lo = 0, hi = nh - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (sh.pre[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Stream every chunk of every segment of the group, feeding observations in range R. A chunk
// is 16 * K bases: each thread loads the 2K + 1 sequence dwords and 2K + 1 reference dwords
// covering its chunk at once (one memory round trip per chunk), then takes the K 16-base
// windows out of registers with static indices.
template <int K, bool REF2>
__device__ __forceinline__ void grp_scan(const GrpBatch &B, GrpShared &sh, const GrpRange &R, const GrpGlobal &gg,
                                         int64_t i_begin, int64_t i_end, const int4 *__restrict__ rec4, int skip) {
  const int tid = threadIdx.x;
  for (int64_t c0 = i_begin; c0 < i_end; c0 += kGrpTile) {
    const int nh = (int)((i_end - c0) < kGrpTile ? (i_end - c0) : kGrpTile);
    int total = grp_tile(sh, rec4, c0, nh, 16 * K);
    if (skip & kSkipChunks) total = 0;
    for (int t = tid; t < total; t += kGrpThreads) {
      const int j = grp_find(sh, nh, total, t);
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
    __syncthreads();
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
__device__ __forceinline__ void grp_count(GrpShared &sh, int s_local, int calls, int bases) {
  if (calls) {
    atomicAdd(&sh.cnt_calls[s_local], calls);
    atomicAdd(&sh.blk_calls, calls);
  }
  if (bases) {
    atomicAdd(&sh.cnt_bases[s_local], bases);
    atomicAdd(&sh.blk_bases, bases);
  }
}

__device__ __forceinline__ void grp_classify(const GrpBatch &B, GrpShared &sh, int n, int s_begin,
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

// Overflow path: n observations of one key range sit in the group's global region. Aggregate
// them in a hash table of distinct keys (workgroup-scope atomics in L2), count the TN calls
// (minus the kept variant), and mask the observations of reads the scopes write.
__device__ __forceinline__ void grp_global(const GrpBatch &B, GrpShared &sh, const GrpGlobal &gg, int n,
                                           int s_begin, const PatchSink &sink) {
  const int tid = opaque_tid();
  const int tsize = max(2 * n, 64);
  unsigned long long *tk = gg.aux->tkey + 2 * gg.off;
  unsigned int *tf = gg.aux->tflag + 2 * gg.off;
  unsigned long long *okey = gg.aux->okey + gg.off, *opay = gg.aux->opay + gg.off;
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
__device__ __forceinline__ void grp_patch_bytes(const GrpBatch &B, GrpShared &sh, int np, uint8_t *out) {
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
template <int U, bool FUSED>
__global__ void __launch_bounds__(kGrpThreads, (U == 1 ? 6 : U == 2 ? GANON_K2_BLOCKS : U == 4 ? 5 : 4)) k_group(const GrpBatch B, const int4 *__restrict__ groups,
                                                       const int4 *__restrict__ rec4,
                                                       uint8_t *__restrict__ out, const GrpAux *__restrict__ aux,
                                                       int skip, int nt_copy) {
  __shared__ GrpShared sh;
  const int tid = threadIdx.x;
  const int4 g0 = groups[kGrpRec * blockIdx.x];
  const int4 g1 = groups[kGrpRec * blockIdx.x + 1];
  const int4 g2 = groups[kGrpRec * blockIdx.x + 2];
  const int4 g3 = groups[kGrpRec * blockIdx.x + 3];
  const int4 g4 = groups[kGrpRec * blockIdx.x + 4];
  const GrpGlobal gg{aux, i64_of(g3.x, g3.y), g3.z};
  const int s_begin = g0.x, s_end = g0.y;
  const int64_t i_begin = i64_of(g0.z, g0.w), i_end = i64_of(g1.x, g1.y), i_mid = i64_of(g1.z, g1.w);
  const PatchSink sink{out, i64_of(g2.x, g2.y), i64_of(g2.z, g2.w), i64_of(g4.x, g4.y), i64_of(g4.z, g4.w),
                       aux, FUSED, FUSED};
  // the partition pieces, whole 16-byte windows (the buffers are padded past seq_bytes); the
  // stores drain while the scan runs (s_waitcnt before the mask stores). (Copying tile by tile,
  // each time up to the tile's written reads so that the scan's loads hit L2, read 0.34 GB less
  // per c2 launch but took 0.55 instead of 0.54 ms in the same build: DESIGN 5.)
  if (FUSED && !(skip & kSkipCopy)) {
    copy_windows(B.seq, out, sink.p0, sink.p1, nt_copy);
    copy_windows(B.seq, out, sink.q0, sink.q1, nt_copy);
  }
  if (tid == 0) {
    sh.top = 0;
    sh.stk_lo[0] = 0ull;
    sh.stk_hi[0] = ~0ull;
    sh.stk_mode[0] = kModeCollect;
    sh.n_patch = 0;
    sh.blk_calls = 0;
    sh.blk_bases = 0;
  }
  for (int i = tid; i < kGrpMaxScopes; i += kGrpThreads) {
    sh.cnt_calls[i] = 0;
    sh.cnt_bases[i] = 0;
  }
  for (;;) {
    __syncthreads();
    const int top = sh.top;
    if (top < 0) {
      // per-scope counts (wide scopes in the id range belong to the tile path) and the
      // workgroup's partial totals (k_finish sums them)
      for (int i = opaque_tid(); i < ((skip & kSkipCounts) ? 0 : s_end - s_begin); i += kGrpThreads) {
        if (B.span_len[s_begin + i] > kGrpMaxSpan) continue;
        aux->scope_calls[s_begin + i] = sh.cnt_calls[i];
        aux->scope_bases[s_begin + i] = sh.cnt_bases[i];
      }
      if (tid == 0) {
        aux->part[2 * blockIdx.x] = sh.blk_calls;
        aux->part[2 * blockIdx.x + 1] = sh.blk_bases;
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
    if (B.ref2) {
      grp_scan<U, true>(B, sh, R, gg, i_begin, i_mid, rec4, skip);
      grp_scan<U, false>(B, sh, R, gg, i_mid, i_end, rec4, skip);
    } else {
      grp_scan<U, false>(B, sh, R, gg, i_begin, i_end, rec4, skip);
    }
    // (grp_scan ends on a barrier)
    if (skip & kSkipClassify) continue;
    const int n = sh.n_obs;
    if (n > kGrpObs) {
      if (n <= gg.cap) {
        // the list joins the region's tail: n observations contiguous in the region
        for (int i = opaque_tid(); i < kGrpObs; i += kGrpThreads) {
          aux->okey[gg.off + (n - kGrpObs) + i] = sh.key[i];
          aux->opay[gg.off + (n - kGrpObs) + i] = sh.pay[i];
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
        const unsigned long long k = i < kGrpObs ? sh.key[i] : ld_l2(aux->okey + gg.off + (i - kGrpObs));
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
// counters: [0] rare small scopes, [1] rare tiles, [2] far masks.
__global__ void __launch_bounds__(kBlock) k_finish(const unsigned long long *__restrict__ far, int64_t far_cap,
                                                   uint8_t *__restrict__ out, const int32_t *__restrict__ grp_part,
                                                   int n_groups, const int32_t *__restrict__ large_ids, int n_large,
                                                   const int32_t *__restrict__ scope_calls,
                                                   const int32_t *__restrict__ scope_bases,
                                                   const unsigned long long *__restrict__ static_totals,
                                                   int32_t *counters, unsigned long long *acc,
                                                   unsigned long long *totals) {
  const int64_t gtid = blockIdx.x * (int64_t)kBlock + threadIdx.x, gstride = (int64_t)gridDim.x * kBlock;
  const int64_t n_far = min((int64_t)counters[2], far_cap);
  for (int64_t i = gtid; i < n_far; i += gstride) {
    const unsigned long long e = far[i];
    const int64_t nib = (int64_t)(e >> 4);
    const int64_t byte = nib >> 1;
    const int sh = 8 * (int)(byte & 3) + ((nib & 1) ? 0 : 4);
    atomicXor(reinterpret_cast<uint32_t *>(out) + (byte >> 2), (uint32_t)(e & 15) << sh);
  }
  long long c = 0, b = 0;
  for (int64_t i = gtid; i < n_groups; i += gstride) {
    c += grp_part[2 * i];
    b += grp_part[2 * i + 1];
  }
  for (int64_t i = gtid; i < n_large; i += gstride) {
    c += scope_calls[large_ids[i]];
    b += scope_bases[large_ids[i]];
  }
  __shared__ long long part[2][kWaves];
  __shared__ int last;
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    b += __shfl_xor(b, o);
  }
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = c;
    part[1][threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    c = b = 0;
    for (int w = 0; w < kWaves; ++w) {
      c += part[0][w];
      b += part[1][w];
    }
    if (c) atomicAdd(&acc[0], (unsigned long long)c);
    if (b) atomicAdd(&acc[1], (unsigned long long)b);
    __threadfence();
    last = atomicAdd(&acc[2], 1ull) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __threadfence();
  const unsigned long long sc = atomicExch(&acc[0], 0ull), sb = atomicExch(&acc[1], 0ull);
  atomicExch(&acc[2], 0ull);
  for (int k = 0; k < GANON_N_TOTALS; ++k) totals[k] = static_totals[k];
  totals[GANON_T_MASKED_SNV_CALLS] += sc;
  totals[GANON_T_MASKED_BASES] += sb;
  totals[GANON_T_RARE_SCOPES] += (unsigned long long)(atomicExch(&counters[0], 0) + atomicExch(&counters[1], 0));
  atomicExch(&counters[2], 0);
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

// Totals: per-scope counts of the scopes in ids (all n scopes when ids is null) plus the
// (calls, bases) partials of the group kernel's workgroups.
__global__ void __launch_bounds__(kBlock) k_totals(const int32_t *__restrict__ calls, const int32_t *__restrict__ bases,
                                                   const int32_t *__restrict__ ids, int n,
                                                   const int32_t *__restrict__ grp_part, int n_part,
                                                   const int32_t *rare_small, const int32_t *rare_tiles,
                                                   unsigned long long *totals) {
  long long c = 0, b = 0;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const int s = ids ? ids[i] : i;
    c += calls[s];
    b += bases[s];
  }
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n_part; i += gridDim.x * kBlock) {
    c += grp_part[2 * i];
    b += grp_part[2 * i + 1];
  }
  // one same-address atomic per workgroup: they serialize at the memory side
  __shared__ long long part[2][kWaves];
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    b += __shfl_xor(b, o);
  }
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = c;
    part[1][threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    c = b = 0;
    for (int w = 0; w < kWaves; ++w) {
      c += part[0][w];
      b += part[1][w];
    }
    if (c) atomicAdd(&totals[GANON_T_MASKED_SNV_CALLS], (unsigned long long)c);
    if (b) atomicAdd(&totals[GANON_T_MASKED_BASES], (unsigned long long)b);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    atomicAdd(&totals[GANON_T_RARE_SCOPES], (unsigned long long)(*rare_small + *rare_tiles));
}

}  // namespace

// ---- host side ---------------------------------------------------------------------------

using ganon_detail::check_launch;
using ganon_detail::fail;
using ganon_detail::KernelScope;

struct ganon_dbatch {
  DevBatch B{};
  std::vector<void *> allocs;
  int32_t n_reads = 0, n_scopes = 0;
  int64_t seq_bytes = 0;
  uint8_t *out = nullptr;
  int32_t *scope_calls = nullptr, *scope_bases = nullptr;
  unsigned long long *totals = nullptr, *static_totals = nullptr;
  int32_t *counters = nullptr;  // [0] rare small count, [1] rare tile count
  int32_t *small_list[2] = {nullptr, nullptr};
  int32_t n_small[2] = {0, 0};
  int32_t *pt_list = nullptr;
  int32_t n_pt = 0;
  Tile *tiles = nullptr;
  int32_t n_tiles = 0;
  int32_t *large_incid = nullptr;
  int64_t *tab_off = nullptr;
  uint16_t *tn_tab = nullptr;
  int64_t tn_entries = 0;
  int32_t *large_written = nullptr;
  int32_t n_large_written = 0;
  int32_t n_large_scopes = 0;
  int32_t *rare_small_list = nullptr, *rare_tile_list = nullptr;
  int32_t max_small_span = 0;
  int4 *inc_rec = nullptr;      // per incidence, scope-major: {start|read, len|flags, seq_off lo, hi}
  int4 *srec[2] = {nullptr, nullptr};   // per small scope of each class: 3 x int4 (k_scope_v3)
  int4 *groups = nullptr;               // k_group: 2 x int4 per group
  int4 *seg4 = nullptr;                 // k_group: segment records (16 bytes, layout at kSegMine)
  int32_t n_groups = 0;
  int64_t n_seg = 0;
  unsigned long long *acc = nullptr;    // k_finish: calls, bases, workgroup ticket
  uint32_t *ref2 = nullptr;             // 2-bit reference (k_ref2)
  unsigned long long *far = nullptr;    // fused: masks outside the masking group's partition
  int64_t far_cap = 0;
  int32_t *grp_part = nullptr;          // k_group: (calls, bases) per workgroup
  int32_t *large_ids = nullptr;         // scopes of the tile path under the group variants (huge)
  GrpAux *aux = nullptr;                // k_group's rarely used pointers (device copy)
  unsigned long long *gokey = nullptr, *gopay = nullptr, *gtkey = nullptr;   // group overflow regions
  unsigned int *gtflag = nullptr;
  Tile *tiles_h = nullptr;              // tiles / written reads of huge scopes (group variants)
  int32_t *large_written_h = nullptr;
  int32_t n_tiles_h = 0, n_large_written_h = 0, n_huge_scopes = 0;
  bool ran = false;
};

namespace {


template <typename T>
int dev_alloc(ganon_ctx *ctx, ganon_dbatch *db, T **p, size_t count) {
  *p = nullptr;
  // +128 bytes: the group kernels load up to 68 bytes from a chunk start past a buffer's last nibble,
  // and the patch
  // atomics touch whole dwords
  size_t bytes = std::max<size_t>(count, 1) * sizeof(T) + 128;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(p), bytes);
  if (e != hipSuccess) return fail(ctx, GANON_E_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  db->allocs.push_back(*p);
  return GANON_OK;
}

template <typename T>
int dev_copy(ganon_ctx *ctx, ganon_dbatch *db, T **p, const T *src, size_t count) {
  int rc = dev_alloc(ctx, db, p, count);
  if (rc) return rc;
  if (count) {
    hipError_t e = hipMemcpyAsync(*p, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipMemcpyAsync H2D failed: %s", hipGetErrorString(e));
  }
  return GANON_OK;
}

void free_batch(ganon_dbatch *db) {
  for (void *p : db->allocs) hipFree(p);
  db->allocs.clear();
}

size_t small_lds_bytes(int tb, int cap) {
  return (size_t)cap * tb + (((size_t)cap / 2 + 15) & ~(size_t)15) + 16 * sizeof(int);
}

size_t tile_lds_bytes(int tb) { return (size_t)kTile * tb + kTile / 2 + 16 * sizeof(int); }

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
  // Every kernel gets the LDS its worst class needs.
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_scope_small<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)small_lds_bytes(1, kSmallCap1));
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_scope_small<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)small_lds_bytes(4, kSmallCap1));
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_tile_large<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)tile_lds_bytes(1));
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_tile_large<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)tile_lds_bytes(4));
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_scope_v3), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)(4 * v3_wave_lds_bytes(kSmallCap1)));
  // persistent grid of k_scope_v3: every resident workgroup slot, no more
  const int caps[2] = {kSmallCap0, kSmallCap1};
  for (int k = 0; k < 2; ++k) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_scope_v3, kBlock, 4 * v3_wave_lds_bytes(caps[k])) !=
            hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    ctx->v3_blocks[k] = per_cu * prop.multiProcessorCount;
  }
  *out = ctx;
  return GANON_OK;
}

GANON_API int ganon_ctx_destroy(ganon_ctx *ctx) {
  if (!ctx) return GANON_E_ARG;
  hipSetDevice(ctx->device);
  if (ctx->own) {
    hipStreamSynchronize(ctx->own);
    hipStreamDestroy(ctx->own);
  }
  for (auto &r : ctx->recs) {
    hipEventDestroy(r.e0);
    hipEventDestroy(r.e1);
  }
  for (auto e : ctx->pool) hipEventDestroy(e);
  delete ctx;
  return GANON_OK;
}

GANON_API const char *ganon_last_error(ganon_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

GANON_API int ganon_ctx_set_stream(ganon_ctx *ctx, void *hip_stream) {
  if (!ctx) return GANON_E_ARG;
  ctx->stream = hip_stream ? reinterpret_cast<hipStream_t>(hip_stream) : ctx->own;
  return GANON_OK;
}

GANON_API int ganon_ctx_set_variant(ganon_ctx *ctx, int variant) {
  if (!ctx || variant < GANON_VARIANT_DEFAULT || variant > GANON_VARIANT_PERSIST)
    return fail(ctx, GANON_E_ARG, "unknown kernel variant %d", variant);
  ctx->variant = variant;
  return GANON_OK;
}

GANON_API int ganon_ctx_set_param(ganon_ctx *ctx, int param, int value) {
  if (!ctx) return GANON_E_ARG;
  if (param == GANON_PARAM_GROUP_UNROLL) {
    if (value != 1 && value != 2 && value != 4 && value != 8)
      return fail(ctx, GANON_E_ARG, "group unroll must be 1, 2, 4 or 8 (got %d)", value);
    ctx->group_unroll = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_GROUP_TARGET) {
    if (value < 16 || value > 65536) return fail(ctx, GANON_E_ARG, "group target must be in [16, 65536] (got %d)", value);
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
    if (value < 1 || value > 8 || value == 7) return fail(ctx, GANON_E_ARG, "FASTQ dwords per lane: 1-6 or 8");
    ctx->fq_kd = value;
    return GANON_OK;
  }
  if (param == GANON_PARAM_NT_COPY) {
    ctx->nt_copy = value != 0;
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

static int validate(ganon_ctx *ctx, const ganon_batch *b, std::vector<int32_t> &read_end) {
  if (b->n_reads < 0 || b->n_scopes < 0 || b->n_incid < 0 || b->seq_bytes < 0 || b->n_cigar_ops < 0 ||
      b->ref_bytes < 0)
    return fail(ctx, GANON_E_ARG, "negative size in batch");
  if (b->n_reads > 0 && (!b->ref_start || !b->read_len || !b->seq_off || !b->cig_off || !b->n_cig ||
                         !b->dataset || !b->write_scope))
    return fail(ctx, GANON_E_ARG, "null read array");
  if (b->seq_bytes > 0 && !b->seq_nt16) return fail(ctx, GANON_E_ARG, "null seq_nt16");
  if (b->n_cigar_ops > 0 && !b->cigar) return fail(ctx, GANON_E_ARG, "null cigar");
  if (!b->scope_incid_off) return fail(ctx, GANON_E_ARG, "null scope_incid_off");
  if (b->n_scopes > 0 && (!b->scope_span_start || !b->scope_span_len || !b->scope_ref_off || !b->keep_pos ||
                          !b->keep_code))
    return fail(ctx, GANON_E_ARG, "null scope array");
  if (b->n_incid > 0 && !b->incid_read) return fail(ctx, GANON_E_ARG, "null incid_read");
  if (b->ref_bytes > 0 && !b->ref_nt16) return fail(ctx, GANON_E_ARG, "null ref_nt16");
  read_end.assign(b->n_reads, 0);
  for (int32_t r = 0; r < b->n_reads; ++r) {
    const int64_t L = b->read_len[r];
    if (L < 0 || b->seq_off[r] < 0 || b->seq_off[r] + (L + 1) / 2 > b->seq_bytes)
      return fail(ctx, GANON_E_ARG, "read %d: sequence out of range", r);
    if (b->n_cig[r] < 0 || b->cig_off[r] < 0 || b->cig_off[r] + b->n_cig[r] > b->n_cigar_ops)
      return fail(ctx, GANON_E_ARG, "read %d: cigar out of range", r);
    if (b->dataset[r] > 1) return fail(ctx, GANON_E_ARG, "read %d: dataset must be 0 or 1", r);
    if (b->write_scope[r] < -1 || b->write_scope[r] >= b->n_scopes)
      return fail(ctx, GANON_E_ARG, "read %d: write_scope out of range", r);
    int64_t rl = 0;
    for (int k = 0; k < b->n_cig[r]; ++k) {
      const uint32_t w = b->cigar[b->cig_off[r] + k];
      const int op = w & 0xF;
      if (op > 8) return fail(ctx, GANON_E_ARG, "read %d: bad cigar op %d", r, op);
      if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += w >> 4;
    }
    if (b->ref_start[r] < 0 || b->ref_start[r] + rl > INT32_MAX) return fail(ctx, GANON_E_ARG, "read %d: bad position", r);
    read_end[r] = (int32_t)(b->ref_start[r] + (rl > 0 ? rl : 1));
  }
  if (b->scope_incid_off[0] != 0 || b->scope_incid_off[b->n_scopes] != b->n_incid)
    return fail(ctx, GANON_E_ARG, "scope_incid_off must start at 0 and end at n_incid");
  std::vector<uint8_t> seen(b->n_reads, 0);
  for (int32_t s = 0; s < b->n_scopes; ++s) {
    const int64_t i0 = b->scope_incid_off[s], i1 = b->scope_incid_off[s + 1];
    if (i1 < i0) return fail(ctx, GANON_E_ARG, "scope %d: decreasing incidence offsets", s);
    const int64_t ss = b->scope_span_start[s], sl = b->scope_span_len[s];
    if (sl < 0 || ss < 0) return fail(ctx, GANON_E_ARG, "scope %d: bad span", s);
    if (b->scope_ref_off[s] < 0 || b->scope_ref_off[s] + sl > 2 * b->ref_bytes)
      return fail(ctx, GANON_E_ARG, "scope %d: reference slice out of range", s);
    if (b->keep_code[s] > 15) return fail(ctx, GANON_E_ARG, "scope %d: keep_code > 15", s);
    for (int64_t i = i0; i < i1; ++i) {
      const int32_t r = b->incid_read[i];
      if (r < 0 || r >= b->n_reads) return fail(ctx, GANON_E_ARG, "incidence %lld: read out of range", (long long)i);
      if (b->ref_start[r] < ss || read_end[r] > ss + sl)
        return fail(ctx, GANON_E_ARG, "scope %d: read %d [%d,%d) outside span [%lld,%lld)", s, r, b->ref_start[r],
                    read_end[r], (long long)ss, (long long)(ss + sl));
      if (b->write_scope[r] == s) seen[r] = 1;
    }
  }
  for (int32_t r = 0; r < b->n_reads; ++r)
    if (b->write_scope[r] >= 0 && !seen[r])
      return fail(ctx, GANON_E_ARG, "read %d: write_scope %d does not contain it", r, b->write_scope[r]);
  return GANON_OK;
}

GANON_API int ganon_batch_upload(ganon_ctx *ctx, const ganon_batch *b, ganon_dbatch **out) {
  if (!ctx || !b || !out) return fail(ctx, GANON_E_ARG, "null argument");
  *out = nullptr;
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  std::vector<int32_t> read_end;
  int rc = validate(ctx, b, read_end);
  if (rc) return rc;
  ganon_dbatch *db = new ganon_dbatch();
  db->n_reads = b->n_reads;
  db->n_scopes = b->n_scopes;
  db->seq_bytes = b->seq_bytes;
  auto bail = [&](int code) {
    hipStreamSynchronize(ctx->stream);
    free_batch(db);
    delete db;
    return code;
  };
  // ---- work lists (host) ----
  std::vector<int32_t> small[2], pt, large_written, large_incid, large_scopes;
  std::vector<int64_t> tab_off(b->n_scopes, -1);
  std::vector<Tile> tiles;
  int64_t tn_entries = 0;
  for (int32_t s = 0; s < b->n_scopes; ++s) {
    const int32_t sl = b->scope_span_len[s];
    if (sl <= kSmallCap0) small[0].push_back(s);
    else if (sl <= kSmallCap1) small[1].push_back(s);
    else {
      large_scopes.push_back(s);
      tab_off[s] = tn_entries;
      tn_entries += sl;
      const int64_t i0 = b->scope_incid_off[s], i1 = b->scope_incid_off[s + 1];
      const int64_t base = (int64_t)large_incid.size();
      for (int64_t i = i0; i < i1; ++i) large_incid.push_back(b->incid_read[i]);
      std::stable_sort(large_incid.begin() + base, large_incid.end(),
                       [&](int32_t x, int32_t y) { return b->ref_start[x] < b->ref_start[y]; });
      int32_t maxspan = 1;
      for (int64_t i = base; i < (int64_t)large_incid.size(); ++i) {
        const int32_t r = large_incid[i];
        maxspan = std::max(maxspan, read_end[r] - b->ref_start[r]);
      }
      const int32_t ss = b->scope_span_start[s];
      for (int64_t a = ss; a < (int64_t)ss + sl; a += kTile) {
        Tile t{};
        t.scope = s;
        t.a = (int32_t)a;
        t.b = (int32_t)std::min<int64_t>(a + kTile, (int64_t)ss + sl);
        auto first = large_incid.begin() + base;
        auto last = large_incid.end();
        const int64_t lo_key = (int64_t)t.a - maxspan;
        t.lo = std::lower_bound(first, last, lo_key,
                                [&](int32_t r, int64_t key) { return (int64_t)b->ref_start[r] < key; }) -
               large_incid.begin();
        t.hi = std::lower_bound(first, last, (int64_t)t.b,
                                [&](int32_t r, int64_t key) { return (int64_t)b->ref_start[r] < key; }) -
               large_incid.begin();
        tiles.push_back(t);
      }
    }
  }
  for (int32_t r = 0; r < b->n_reads; ++r) {
    const int32_t ws = b->write_scope[r];
    if (ws < 0) pt.push_back(r);
    else if (tab_off[ws] >= 0) large_written.push_back(r);
  }
  int32_t max_small = 0;
  for (auto s : small[0]) max_small = std::max(max_small, b->scope_span_len[s]);
  for (auto s : small[1]) max_small = std::max(max_small, b->scope_span_len[s]);
  // ---- device copies ----
  DevBatch &D = db->B;
#define COPY(field, src, n)                                                                       \
  do {                                                                                            \
    using T_ = std::remove_const_t<std::remove_pointer_t<decltype(D.field)>>;                     \
    T_ *q_ = nullptr;                                                                             \
    if ((rc = dev_copy(ctx, db, &q_, reinterpret_cast<const T_ *>(src), (size_t)(n)))) return bail(rc); \
    D.field = q_;                                                                                 \
  } while (0)
  COPY(ref_start, b->ref_start, b->n_reads);
  COPY(read_len, b->read_len, b->n_reads);
  COPY(read_end, read_end.data(), b->n_reads);
  COPY(n_cig, b->n_cig, b->n_reads);
  COPY(write_scope, b->write_scope, b->n_reads);
  COPY(seq_off, b->seq_off, b->n_reads);
  COPY(cig_off, b->cig_off, b->n_reads);
  COPY(seq, b->seq_nt16, b->seq_bytes);
  COPY(dataset, b->dataset, b->n_reads);
  COPY(cigar, b->cigar, b->n_cigar_ops);
  COPY(incid_off, b->scope_incid_off, (size_t)b->n_scopes + 1);
  COPY(incid_read, b->incid_read, b->n_incid);
  COPY(span_start, b->scope_span_start, b->n_scopes);
  COPY(span_len, b->scope_span_len, b->n_scopes);
  COPY(keep_pos, b->keep_pos, b->n_scopes);
  COPY(ref_off, b->scope_ref_off, b->n_scopes);
  COPY(ref, b->ref_nt16, b->ref_bytes);
  COPY(keep_code, b->keep_code, b->n_scopes);
#undef COPY
  for (int k = 0; k < 2; ++k) {
    if ((rc = dev_copy(ctx, db, &db->small_list[k], small[k].data(), small[k].size()))) return bail(rc);
    db->n_small[k] = (int32_t)small[k].size();
  }
  if ((rc = dev_copy(ctx, db, &db->pt_list, pt.data(), pt.size()))) return bail(rc);
  db->n_pt = (int32_t)pt.size();
  if ((rc = dev_copy(ctx, db, &db->tiles, tiles.data(), tiles.size()))) return bail(rc);
  db->n_tiles = (int32_t)tiles.size();
  if ((rc = dev_copy(ctx, db, &db->large_incid, large_incid.data(), large_incid.size()))) return bail(rc);
  if ((rc = dev_copy(ctx, db, &db->tab_off, tab_off.data(), tab_off.size()))) return bail(rc);
  // the tile path's TN table (2 bytes per position of every wide scope) is allocated on the
  // first run that uses it: under the group variants only scopes over kGrpMaxSpan tile
  db->tn_entries = tn_entries;
  if ((rc = dev_copy(ctx, db, &db->large_written, large_written.data(), large_written.size()))) return bail(rc);
  db->n_large_written = (int32_t)large_written.size();
  db->n_large_scopes = (int32_t)large_scopes.size();
  {
    // the group kernels take every scope up to kGrpMaxSpan positions; only wider ("huge")
    // scopes keep the tile path under the group variants
    std::vector<Tile> tiles_h;
    std::vector<int32_t> written_h, ids_h;
    for (const Tile &t : tiles)
      if (b->scope_span_len[t.scope] > kGrpMaxSpan) tiles_h.push_back(t);
    for (int32_t r : large_written)
      if (b->scope_span_len[b->write_scope[r]] > kGrpMaxSpan) written_h.push_back(r);
    for (int32_t x : large_scopes)
      if (b->scope_span_len[x] > kGrpMaxSpan) ids_h.push_back(x);
    if ((rc = dev_copy(ctx, db, &db->tiles_h, tiles_h.data(), tiles_h.size()))) return bail(rc);
    if ((rc = dev_copy(ctx, db, &db->large_written_h, written_h.data(), written_h.size()))) return bail(rc);
    if ((rc = dev_copy(ctx, db, &db->large_ids, ids_h.data(), ids_h.size()))) return bail(rc);
    db->n_tiles_h = (int32_t)tiles_h.size();
    db->n_large_written_h = (int32_t)written_h.size();
    db->n_huge_scopes = (int32_t)ids_h.size();
  }
  db->max_small_span = max_small;
  {
    // per-incidence records for the v2 scope kernel (scope-major, one int4 each)
    std::vector<int4> rec((size_t)b->n_incid);
    for (int32_t s = 0; s < b->n_scopes; ++s) {
      for (int64_t i = b->scope_incid_off[s]; i < b->scope_incid_off[s + 1]; ++i) {
        const int32_t r = b->incid_read[i];
        const int32_t L = b->read_len[r];
        bool simple = false;
        if (b->n_cig[r] == 1) {
          const uint32_t w = b->cigar[b->cig_off[r]];
          const int op = w & 0xF;
          simple = (op == 0 || op == 7 || op == 8) && (int64_t)(w >> 4) == L && L > 0;
        }
        const bool cplx = !simple && b->n_cig[r] > 0 && L > 0;
        if (L >= (1 << 24)) return bail(fail(ctx, GANON_E_ARG, "read %d longer than 16 Mb", r));
        uint32_t fl = (uint32_t)L | ((uint32_t)b->dataset[r] << 24);
        if (simple) fl |= kRecSimple;
        if (cplx) fl |= kRecCplx;
        if (b->write_scope[r] == s) fl |= kRecMine;
        const uint64_t so = (uint64_t)b->seq_off[r];
        rec[i] = make_int4(simple ? b->ref_start[r] : r, (int)fl, (int)(uint32_t)so, (int)(uint32_t)(so >> 32));
      }
    }
    if ((rc = dev_copy(ctx, db, &db->inc_rec, rec.data(), rec.size()))) return bail(rc);
    for (int k = 0; k < 2; ++k) {
      std::vector<int4> sr(3 * small[k].size());
      for (size_t j = 0; j < small[k].size(); ++j) {
        const int32_t s = small[k][j];
        const int64_t i0 = b->scope_incid_off[s];
        const int64_t ni = b->scope_incid_off[s + 1] - i0;
        if (ni >= INT32_MAX) return bail(fail(ctx, GANON_E_ARG, "scope %d has too many reads", s));
        const int64_t nib0 = b->scope_ref_off[s] - b->scope_span_start[s];
        sr[3 * j] = make_int4(s, b->scope_span_start[s], b->scope_span_len[s], b->keep_pos[s]);
        sr[3 * j + 1] = make_int4((int)(uint32_t)i0, (int)(uint32_t)((uint64_t)i0 >> 32), (int)ni, b->keep_code[s]);
        sr[3 * j + 2] = make_int4((int)(uint32_t)nib0, (int)(uint32_t)((uint64_t)nib0 >> 32), 0, 0);
      }
      if ((rc = dev_copy(ctx, db, &db->srec[k], sr.data(), sr.size()))) return bail(rc);
    }
  }
  {
    // group kernels: aligned segments of every read of every small scope, scope-major, packed
    // into groups of consecutive scopes; groups launch in the order of their written reads in
    // the sequence buffer, each owning the 128-byte-aligned partition of out from its first
    // written read to the next group's (fused variant)
    if (2 * b->seq_bytes >= (int64_t(1) << 40) || 2 * b->ref_bytes >= (int64_t(1) << 40))
      return bail(fail(ctx, GANON_E_ARG, "sequence or reference over 2^40 bases"));
    std::vector<int4> s4;
    s4.reserve((size_t)b->n_incid);
    auto lo32 = [](int64_t v) { return (int)(uint32_t)(uint64_t)v; };
    auto hi32 = [](int64_t v) { return (int)(uint32_t)((uint64_t)v >> 32); };
    struct G {
      int32_t s0, s1;
      int64_t i0, i1, first;   // first: lowest seq_off of a read the group writes
      int64_t mid;             // segments [i0, mid) have an all-ACGT reference range
      int64_t bases;           // aligned bases of its segments (sizes the overflow region)
    };
    std::vector<G> gs;
    int32_t g_s0 = -1;
    int64_t g_i0 = 0, g_first = INT64_MAX;
    // 64-base reference blocks holding a non-ACGT code (N, IUPAC, '='), for the clean/dirty split
    const int64_t n_blk = (b->ref_bytes + 31) / 32;
    std::vector<uint8_t> bad_blk((size_t)n_blk, 0);
    {
      uint8_t ok[256];
      for (int v = 0; v < 256; ++v) ok[v] = ((0x116 >> (v >> 4)) & 1) && ((0x116 >> (v & 15)) & 1);
      const int nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
      std::vector<std::thread> th;
      for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
          for (int64_t k = t; k < n_blk; k += nt) {
            const int64_t e = std::min<int64_t>(32 * k + 32, b->ref_bytes);
            uint8_t bad = 0;
            for (int64_t x = 32 * k; x < e; ++x) bad |= !ok[b->ref_nt16[x]];
            bad_blk[k] = bad;
          }
        });
      for (auto &x : th) x.join();
    }
    auto ref_clean = [&](int64_t rnib, int64_t n) {
      for (int64_t k = rnib >> 6; k <= (rnib + n - 1) >> 6; ++k)
        if (k >= n_blk || bad_blk[k]) return false;
      return true;
    };
    std::vector<int4> c4, d4;   // the open group's segments: clean, dirty reference
    auto close_group = [&](int32_t s_end) {
      if (g_s0 < 0) return;
      int64_t bases = 0;
      for (const int4 &x : c4) bases += ((uint32_t)x.z >> 16) & kSegMaxLen;
      for (const int4 &x : d4) bases += ((uint32_t)x.z >> 16) & kSegMaxLen;
      s4.insert(s4.end(), c4.begin(), c4.end());
      const int64_t mid = (int64_t)s4.size();
      s4.insert(s4.end(), d4.begin(), d4.end());
      c4.clear();
      d4.clear();
      gs.push_back(G{g_s0, s_end, g_i0, (int64_t)s4.size(), g_first, mid, bases});
      g_s0 = -1;
      g_first = INT64_MAX;
    };
    auto segments_of = [&](int32_t r, auto &&emit) {
      const int64_t L = b->read_len[r];
      int64_t q = 0, p = b->ref_start[r];
      for (int k = 0; k < b->n_cig[r] && q < L; ++k) {
        const uint32_t w = b->cigar[b->cig_off[r] + k];
        const int op = w & 0xF;
        const int64_t len = w >> 4;
        if (op == 0 || op == 7 || op == 8) {
          const int64_t n = std::min(len, L - q);
          for (int64_t o = 0; o < n; o += kSegMaxLen) emit(q + o, p + o, std::min<int64_t>(kSegMaxLen, n - o));
          q += len;
          p += len;
        } else if (op == 1 || op == 4) {
          q += len;
        } else if (op == 2 || op == 3) {
          p += len;
        }
      }
    };
    for (int32_t s = 0; s < b->n_scopes; ++s) {
      if (b->scope_span_len[s] > kGrpMaxSpan) continue;   // huge scope: tile path
      const int64_t i0 = b->scope_incid_off[s], i1 = b->scope_incid_off[s + 1];
      int64_t nseg = 0;
      for (int64_t i = i0; i < i1; ++i) segments_of(b->incid_read[i], [&](int64_t, int64_t, int64_t) { ++nseg; });
      if (g_s0 >= 0 && ((int64_t)(c4.size() + d4.size()) + nseg > ctx->group_target || s - g_s0 >= kGrpMaxScopes))
        close_group(s);
      if (g_s0 < 0) {
        g_s0 = s;
        g_i0 = (int64_t)s4.size();
      }
      const int64_t ref0 = b->scope_ref_off[s] - b->scope_span_start[s];
      for (int64_t i = i0; i < i1; ++i) {
        const int32_t r = b->incid_read[i];
        if (b->read_len[r] >= (1 << 24)) return bail(fail(ctx, GANON_E_ARG, "read %d longer than 16 Mb", r));
        uint32_t fl = (uint32_t)b->dataset[r] << 30;
        if (b->write_scope[r] == s) {
          fl |= kSegMine;
          g_first = std::min(g_first, b->seq_off[r]);
        }
        const int64_t qnib = 2 * b->seq_off[r];
        segments_of(r, [&](int64_t q, int64_t p, int64_t n) {
          const bool clean = ref_clean(ref0 + p, n);
          const uint64_t sq = (uint64_t)(qnib + q), rf = (uint64_t)(ref0 + p);
          const uint32_t z = (uint32_t)((sq >> 32) & 0xFF) | ((uint32_t)((rf >> 32) & 0xFF) << 8) |
                             ((uint32_t)n << 16) | fl;
          // scope span <= kGrpMaxSpan = 2^20 positions
          const uint32_t pos_off = (uint32_t)(p - b->scope_span_start[s]);
          (clean ? c4 : d4).push_back(make_int4((int)(uint32_t)sq, (int)(uint32_t)rf, (int)z,
                                                (int)((uint32_t)(s - g_s0) | (pos_off << 12))));
        });
      }
    }
    close_group(b->n_scopes);
    const int32_t ng = (int32_t)gs.size();
    // partition pieces: the sequence buffer in byte order is a sequence of runs of written reads
    // owned by one group (a group's written reads are contiguous per dataset when each dataset's
    // reads are stored in position order — the product layout is every tumor read, then every
    // normal read, so a group has one run per dataset). Each group keeps its two largest runs as
    // pieces; any other run (a read at a group boundary) joins the piece before it. The pieces
    // tile [0, seq_bytes) at 128-byte boundaries; bytes of a read outside its group's pieces
    // are masked through the far list.
    std::vector<int32_t> scope_grp((size_t)b->n_scopes, -1);
    for (int32_t k = 0; k < ng; ++k)
      for (int32_t s = gs[k].s0; s < gs[k].s1; ++s)
        if (b->scope_span_len[s] <= kGrpMaxSpan) scope_grp[s] = k;
    auto owner_of = [&](int32_t r) -> int32_t {
      const int32_t ws = b->write_scope[r];
      return (ws < 0 || b->read_len[r] == 0) ? -1 : scope_grp[ws];
    };
    std::vector<int32_t> byoff;
    byoff.reserve((size_t)b->n_reads);
    bool sorted = true;
    for (int32_t r = 0; r < b->n_reads; ++r) {
      if (owner_of(r) < 0) continue;
      if (!byoff.empty() && b->seq_off[r] < b->seq_off[byoff.back()]) sorted = false;
      byoff.push_back(r);
    }
    if (!sorted)
      std::stable_sort(byoff.begin(), byoff.end(), [&](int32_t x, int32_t y) { return b->seq_off[x] < b->seq_off[y]; });
    struct Run {
      int64_t start;
      int32_t owner;
    };
    std::vector<Run> runs;
    for (int32_t r : byoff) {
      const int32_t g = owner_of(r);
      if (runs.empty() || runs.back().owner != g) runs.push_back(Run{b->seq_off[r], g});
    }
    // each group's two largest runs (bytes up to the next run)
    auto run_len = [&](int64_t i) {
      return ((size_t)i + 1 < runs.size() ? runs[(size_t)i + 1].start : b->seq_bytes) - runs[(size_t)i].start;
    };
    std::vector<int64_t> best((size_t)ng * 2, -1);
    for (int64_t i = 0; i < (int64_t)runs.size(); ++i) {
      int64_t *bb = &best[2 * (size_t)runs[(size_t)i].owner];
      const int64_t len = run_len(i);
      if (bb[0] < 0 || len > run_len(bb[0])) {
        bb[1] = bb[0];
        bb[0] = i;
      } else if (bb[1] < 0 || len > run_len(bb[1])) {
        bb[1] = i;
      }
    }
    std::vector<Run> pieces;
    for (int64_t i = 0; i < (int64_t)runs.size(); ++i) {
      const int32_t g = runs[(size_t)i].owner;
      if (best[2 * (size_t)g] != i && best[2 * (size_t)g + 1] != i) continue;
      const int64_t c = pieces.empty() ? 0 : std::min(runs[(size_t)i].start, b->seq_bytes) / kPartAlign * kPartAlign;
      if (!pieces.empty() && c <= pieces.back().start) pieces.back().owner = g;   // the previous piece is empty
      else pieces.push_back(Run{c, g});
    }
    std::vector<int64_t> pc((size_t)ng * 4, 0);   // per group: piece A [0], [1); piece B [2], [3)
    std::vector<int64_t> first((size_t)ng, INT64_MAX);
    for (size_t i = 0; i < pieces.size(); ++i) {
      const int32_t g = pieces[i].owner;
      const int64_t e = i + 1 < pieces.size() ? pieces[i + 1].start : b->seq_bytes;
      int64_t *q = &pc[4 * (size_t)g];
      const int slot = first[g] == INT64_MAX ? 0 : 2;   // at most two pieces per group
      q[slot] = pieces[i].start;
      q[slot + 1] = e;
      first[g] = std::min(first[g], pieces[i].start);
    }
    if (pieces.empty() && ng) {   // no written read in a small scope: the first group copies it all
      pc[0] = 0;
      pc[1] = b->seq_bytes;
      first[0] = 0;
    }
    std::vector<int32_t> order(ng);
    for (int32_t k = 0; k < ng; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return first[x] < first[y]; });
    // exact bound on masks landing outside the masking group's pieces: every nibble of a
    // written read that lies outside them
    int64_t far_cap = 0;
    for (int32_t r : byoff) {
      const int64_t *q = &pc[4 * (size_t)owner_of(r)];
      const int64_t r0 = b->seq_off[r], r1 = r0 + ((int64_t)b->read_len[r] + 1) / 2;
      const int64_t in = std::max<int64_t>(0, std::min(r1, q[1]) - std::max(r0, q[0])) +
                         std::max<int64_t>(0, std::min(r1, q[3]) - std::max(r0, q[2]));
      far_cap += 2 * ((r1 - r0) - in);
    }
    // overflow regions: (bases / 48 + kGrpObs) observations per group, i.e. up to ~2 % of its
    // aligned bases mismatching (more: key-range halving)
    std::vector<int4> grp(kGrpRec * (size_t)ng);
    int64_t region = 0;
    for (int32_t k = 0; k < ng; ++k) {
      const G &g = gs[order[k]];
      const int64_t *q = &pc[4 * (size_t)order[k]];
      const int64_t cap = std::min<int64_t>(g.bases / 48 + kGrpObs, INT32_MAX / 2);
      grp[kGrpRec * k] = make_int4(g.s0, g.s1, lo32(g.i0), hi32(g.i0));
      grp[kGrpRec * k + 1] = make_int4(lo32(g.i1), hi32(g.i1), lo32(g.mid), hi32(g.mid));
      grp[kGrpRec * k + 2] = make_int4(lo32(q[0]), hi32(q[0]), lo32(q[1]), hi32(q[1]));
      grp[kGrpRec * k + 3] = make_int4(lo32(region), hi32(region), (int)cap, 0);
      grp[kGrpRec * k + 4] = make_int4(lo32(q[2]), hi32(q[2]), lo32(q[3]), hi32(q[3]));
      region += cap;
    }
    if ((rc = dev_alloc(ctx, db, &db->gokey, (size_t)region))) return bail(rc);
    if ((rc = dev_alloc(ctx, db, &db->gopay, (size_t)region))) return bail(rc);
    if ((rc = dev_alloc(ctx, db, &db->gtkey, 2 * (size_t)region + 64))) return bail(rc);
    if ((rc = dev_alloc(ctx, db, &db->gtflag, 2 * (size_t)region + 64))) return bail(rc);
    if ((rc = dev_copy(ctx, db, &db->groups, grp.data(), grp.size()))) return bail(rc);
    if ((rc = dev_copy(ctx, db, &db->seg4, s4.data(), s4.size()))) return bail(rc);
    db->n_groups = ng;
    if ((rc = dev_alloc(ctx, db, &db->grp_part, 2 * (size_t)ng))) return bail(rc);
    db->n_seg = (int64_t)s4.size();
    db->far_cap = far_cap;
    if ((rc = dev_alloc(ctx, db, &db->far, (size_t)far_cap))) return bail(rc);
    const int64_t n_words = (2 * b->ref_bytes + 15) / 16;
    if ((rc = dev_alloc(ctx, db, &db->ref2, (size_t)n_words + 2))) return bail(rc);
    if (n_words) {
      k_ref2<<<(int)std::min<int64_t>((n_words + kBlock - 1) / kBlock, 16384), kBlock, 0, ctx->stream>>>(
          D.ref, n_words, db->ref2);
      if ((rc = check_launch(ctx, "k_ref2"))) return bail(rc);
    }
    D.ref2 = db->ref2;
  }
  if ((rc = dev_alloc(ctx, db, &db->out, (size_t)b->seq_bytes))) return bail(rc);
  // bytes outside every read are never written by the fused variant: make them defined
  if (hipMemsetAsync(db->out, 0, (size_t)b->seq_bytes + 16, ctx->stream) != hipSuccess)
    return bail(fail(ctx, GANON_E_DEVICE, "hipMemsetAsync(out) failed"));
  if ((rc = dev_alloc(ctx, db, &db->scope_calls, (size_t)b->n_scopes))) return bail(rc);
  if ((rc = dev_alloc(ctx, db, &db->scope_bases, (size_t)b->n_scopes))) return bail(rc);
  if ((rc = dev_alloc(ctx, db, &db->totals, GANON_N_TOTALS))) return bail(rc);
  if ((rc = dev_alloc(ctx, db, &db->counters, 4))) return bail(rc);
  if ((rc = dev_alloc(ctx, db, &db->acc, 3))) return bail(rc);
  {
    const GrpAux a{db->scope_calls, db->scope_bases, db->grp_part, db->far, db->counters + 2, db->far_cap,
                   db->gokey, db->gopay, db->gtkey, db->gtflag};
    if ((rc = dev_copy(ctx, db, &db->aux, &a, 1))) return bail(rc);
  }
  // k_finish keeps these zero between runs
  if (hipMemsetAsync(db->counters, 0, 4 * sizeof(int32_t), ctx->stream) != hipSuccess ||
      hipMemsetAsync(db->acc, 0, 3 * sizeof(unsigned long long), ctx->stream) != hipSuccess)
    return bail(fail(ctx, GANON_E_DEVICE, "hipMemsetAsync(counters) failed"));
  if ((rc = dev_alloc(ctx, db, &db->rare_small_list, small[0].size() + small[1].size()))) return bail(rc);
  if ((rc = dev_alloc(ctx, db, &db->rare_tile_list, tiles.size()))) return bail(rc);
  unsigned long long st[GANON_N_TOTALS] = {0};
  int64_t written = 0;
  for (int32_t r = 0; r < b->n_reads; ++r) written += b->write_scope[r] >= 0;
  st[GANON_T_READS_IN] = (unsigned long long)b->n_reads;
  st[GANON_T_READS_WRITTEN] = (unsigned long long)written;
  st[GANON_T_SCOPES] = (unsigned long long)b->n_scopes;
  st[GANON_T_LARGE_TILES] = (unsigned long long)tiles.size();
  if ((rc = dev_copy(ctx, db, &db->static_totals, st, GANON_N_TOTALS))) return bail(rc);
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    fail(ctx, GANON_E_DEVICE, "upload sync failed: %s", hipGetErrorString(e));
    return bail(GANON_E_DEVICE);
  }
  *out = db;
  return GANON_OK;
}

GANON_API int ganon_batch_run(ganon_ctx *ctx, ganon_dbatch *db) {
  if (!ctx || !db) return fail(ctx, GANON_E_ARG, "null argument");
  HIP_OR_FAIL(hipSetDevice(ctx->device));
  for (auto &r : ctx->recs) {
    ctx->pool.push_back(r.e0);
    ctx->pool.push_back(r.e1);
  }
  ctx->recs.clear();
  hipStream_t st = ctx->stream;
  DevBatch B = db->B;
  if (!ctx->ref2) B.ref2 = nullptr;   // group kernels then read the nt16 reference only
  int rc;
  const bool v3 = ctx->variant == GANON_VARIANT_PERSIST;
  const bool v2 = ctx->variant == GANON_VARIANT_COPYPATCH;
  const bool v5 = ctx->variant == GANON_VARIANT_DEFAULT || ctx->variant == GANON_VARIANT_GROUP_FUSED;
  const bool v4 = ctx->variant == GANON_VARIANT_GROUP || v5;   // group kernels
  if (!v4) {
    // group variants leave counters zero and write totals in k_finish
    HIP_OR_FAIL(hipMemsetAsync(db->counters, 0, 4 * sizeof(int32_t), st));
    HIP_OR_FAIL(hipMemcpyAsync(db->totals, db->static_totals, GANON_N_TOTALS * sizeof(unsigned long long),
                               hipMemcpyDeviceToDevice, st));
  }
  const Tile *tiles = v4 ? db->tiles_h : db->tiles;
  const int32_t n_tiles = v4 ? db->n_tiles_h : db->n_tiles;
  const int32_t *large_written = v4 ? db->large_written_h : db->large_written;
  const int32_t n_large_written = v4 ? db->n_large_written_h : db->n_large_written;
  if (v4 ? db->n_huge_scopes : db->n_large_scopes) {
    // wide scopes are counted with atomics (tiles)
    HIP_OR_FAIL(hipMemsetAsync(db->scope_calls, 0, (size_t)db->n_scopes * sizeof(int32_t), st));
    HIP_OR_FAIL(hipMemsetAsync(db->scope_bases, 0, (size_t)db->n_scopes * sizeof(int32_t), st));
  }
  if (v5 && db->n_groups) {
    // the fused group kernel writes every byte of out (its partitions tile [0, seq_bytes))
  } else if (v2 || v3 || v4) {
    // copy-then-patch: every read's bytes first, the scope kernels patch masked nibbles
    KernelScope ks(ctx, "copy_seq");
    if (db->seq_bytes) HIP_OR_FAIL(hipMemcpyAsync(db->out, B.seq, (size_t)db->seq_bytes, hipMemcpyDeviceToDevice, st));
  } else if (db->n_pt) {
    KernelScope ks(ctx, "k_passthrough");
    const int grid = std::min<int>((db->n_pt + kWaves - 1) / kWaves, 8192);
    k_passthrough<<<grid, kBlock, 0, st>>>(B, db->pt_list, db->n_pt, db->out);
    if ((rc = check_launch(ctx, "k_passthrough"))) return rc;
  }
  if (v4 && db->n_groups) {
    KernelScope ks(ctx, v5 ? "k_group_fused" : "k_group");
    const int u = ctx->group_unroll;
    auto kern = v5 ? (u == 2 ? k_group<2, true> : u == 4 ? k_group<4, true> : u == 8 ? k_group<8, true>
                                                                                     : k_group<1, true>)
                   : (u == 2 ? k_group<2, false> : u == 4 ? k_group<4, false> : u == 8 ? k_group<8, false>
                                                                                       : k_group<1, false>);
    const GrpBatch GB{B.seq, B.ref, B.keep_code, B.ref2, B.keep_pos, B.span_start, B.span_len};
    kern<<<db->n_groups, kGrpThreads, 0, st>>>(GB, db->groups, db->seg4, db->out, db->aux, ctx->group_skip,
                                               ctx->nt_copy);
    if ((rc = check_launch(ctx, "k_group"))) return rc;
  }
  const int caps[2] = {kSmallCap0, kSmallCap1};
  for (int k = 0; k < 2 && !v4; ++k) {
    if (!db->n_small[k]) continue;
    if (v3) {
      KernelScope ks(ctx, k == 0 ? "k_scope_v3/2.5K" : "k_scope_v3/16K");
      const size_t lds = 4 * v3_wave_lds_bytes(caps[k]);
      const int grid = std::max(1, std::min((db->n_small[k] + 3) / 4, ctx->v3_blocks[k]));
      k_scope_v3<<<grid, kBlock, lds, st>>>(B, db->srec[k], db->n_small[k], caps[k], db->inc_rec, db->out,
                                            db->scope_calls, db->scope_bases, db->rare_small_list,
                                            db->counters + 0);
      if ((rc = check_launch(ctx, "k_scope_v3"))) return rc;
    } else if (v2) {
      KernelScope ks(ctx, k == 0 ? "k_scope_v2/2.5K" : "k_scope_v2/16K");
      k_scope_v2<<<db->n_small[k], 64, v2_lds_bytes(caps[k]), st>>>(
          B, db->inc_rec, db->small_list[k], db->n_small[k], caps[k], db->out, db->scope_calls, db->scope_bases,
          db->rare_small_list, db->counters + 0);
      if ((rc = check_launch(ctx, "k_scope_v2"))) return rc;
    } else if (ctx->variant == GANON_VARIANT_BLOCK) {
      KernelScope ks(ctx, k == 0 ? "k_scope_small<1>/2.5K" : "k_scope_small<1>/16K");
      k_scope_small<1><<<db->n_small[k], kBlock, small_lds_bytes(1, caps[k]), st>>>(
          B, db->small_list[k], db->n_small[k], nullptr, caps[k], db->out, db->scope_calls, db->scope_bases,
          db->rare_small_list, db->counters + 0);
      if ((rc = check_launch(ctx, "k_scope_small<1>"))) return rc;
    } else {
      KernelScope ks(ctx, k == 0 ? "k_scope_wave/2.5K" : "k_scope_wave/16K");
      k_scope_wave<<<db->n_small[k], 64, (size_t)caps[k] + kMetaLds, st>>>(
          B, db->small_list[k], db->n_small[k], caps[k], db->out, db->scope_calls, db->scope_bases,
          db->rare_small_list, db->counters + 0);
      if ((rc = check_launch(ctx, "k_scope_wave"))) return rc;
    }
  }
  if (n_tiles && !db->tn_tab && (rc = dev_alloc(ctx, db, &db->tn_tab, (size_t)db->tn_entries))) return rc;
  if (n_tiles) {
    KernelScope ks(ctx, "k_tile_large<1>");
    k_tile_large<1><<<n_tiles, kBlock, tile_lds_bytes(1), st>>>(
        B, tiles, nullptr, n_tiles, nullptr, db->large_incid, db->tab_off, db->tn_tab, db->scope_calls,
        db->rare_tile_list, db->counters + 1);
    if ((rc = check_launch(ctx, "k_tile_large<1>"))) return rc;
  }
  // Re-runs on the 16-code tally; list lengths stay on the device (no host sync).
  if (db->n_small[0] + db->n_small[1] && !v4) {
    KernelScope ks(ctx, "k_scope_small<4>/rare");
    const int grid = std::min<int>(db->n_small[0] + db->n_small[1], kPersistGrid);
    k_scope_small<4><<<grid, kBlock, small_lds_bytes(4, kSmallCap1), st>>>(
        B, db->rare_small_list, 0, db->counters + 0, kSmallCap1, db->out, db->scope_calls, db->scope_bases,
        nullptr, nullptr);
    if ((rc = check_launch(ctx, "k_scope_small<4>"))) return rc;
  }
  if (n_tiles) {
    KernelScope ks(ctx, "k_tile_large<4>/rare");
    const int grid = std::min<int>(n_tiles, kPersistGrid);
    k_tile_large<4><<<grid, kBlock, tile_lds_bytes(4), st>>>(
        B, tiles, db->rare_tile_list, 0, db->counters + 1, db->large_incid, db->tab_off, db->tn_tab,
        db->scope_calls, nullptr, nullptr);
    if ((rc = check_launch(ctx, "k_tile_large<4>"))) return rc;
  }
  if (n_large_written) {
    KernelScope ks(ctx, "k_mask_large");
    const int grid = std::min<int>((n_large_written + kWaves - 1) / kWaves, 8192);
    k_mask_large<<<grid, kBlock, 0, st>>>(B, large_written, n_large_written, db->tab_off, db->tn_tab,
                                          db->out, db->scope_bases);
    if ((rc = check_launch(ctx, "k_mask_large"))) return rc;
  }
  {
    if (v4) {
      // far masks (fused), totals from the group partials and the wide scopes, counter reset
      KernelScope ks(ctx, "k_finish");
      k_finish<<<64, kBlock, 0, st>>>(db->far, v5 && db->n_groups ? db->far_cap : 0, db->out, db->grp_part,
                                      db->n_groups, db->large_ids, db->n_huge_scopes, db->scope_calls,
                                      db->scope_bases, db->static_totals, db->counters, db->acc, db->totals);
      if ((rc = check_launch(ctx, "k_finish"))) return rc;
    } else {
      KernelScope ks(ctx, "k_totals");
      const int grid = std::max(1, std::min<int>((db->n_scopes + kBlock - 1) / kBlock, 128));
      k_totals<<<grid, kBlock, 0, st>>>(db->scope_calls, db->scope_bases, nullptr, db->n_scopes, nullptr, 0,
                                        db->counters + 0, db->counters + 1, db->totals);
      if ((rc = check_launch(ctx, "k_totals"))) return rc;
    }
  }
  db->ran = true;
  return GANON_OK;
}

GANON_API int ganon_batch_sync(ganon_ctx *ctx) {
  if (!ctx) return GANON_E_ARG;
  HIP_OR_FAIL(hipStreamSynchronize(ctx->stream));
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
  if (seq_out && db->seq_bytes)
    HIP_OR_FAIL(hipMemcpyAsync(seq_out, db->out, (size_t)db->seq_bytes, hipMemcpyDeviceToHost, st));
  if (scope_calls_out && db->n_scopes)
    HIP_OR_FAIL(hipMemcpyAsync(scope_calls_out, db->scope_calls, (size_t)db->n_scopes * 4, hipMemcpyDeviceToHost, st));
  if (scope_bases_out && db->n_scopes)
    HIP_OR_FAIL(hipMemcpyAsync(scope_bases_out, db->scope_bases, (size_t)db->n_scopes * 4, hipMemcpyDeviceToHost, st));
  if (totals_out)
    HIP_OR_FAIL(hipMemcpyAsync(totals_out, db->totals, GANON_N_TOTALS * 8, hipMemcpyDeviceToHost, st));
  HIP_OR_FAIL(hipStreamSynchronize(st));
  return GANON_OK;
}

GANON_API int ganon_batch_free(ganon_ctx *ctx, ganon_dbatch *db) {
  if (!db) return GANON_E_ARG;
  if (ctx) {
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
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

GANON_API int ganon_batch_info(ganon_dbatch *db, int64_t *info) {
  if (!db || !info) return GANON_E_ARG;
  info[0] = db->n_small[0];
  info[1] = db->n_small[1];
  info[2] = db->n_large_scopes;
  info[3] = db->n_tiles;
  info[4] = db->n_pt;
  info[5] = db->n_large_written;
  info[6] = db->max_small_span;
  info[7] = db->tn_entries;
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
