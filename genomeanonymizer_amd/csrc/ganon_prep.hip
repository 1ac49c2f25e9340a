// ganon_prep.hip — device prep of a masking batch on MI355X (gfx950): the derived layer of
// ganon_batch.h rebuilt from the raw SoA on every ganon_batch_run, so that a step processes the
// batch exactly as the host hands it over (BAM nt16 bases + BAM CIGAR words + scope incidences).
//
// Reference semantics being prepared: the reference's pileup
// (pileup_io.pyx:8-41, htslib truncate=False) visits every aligned base (CIGAR M/=/X) of every
// read of a scope at reference position p, query position q; insertions and soft clips consume
// the read only, deletions and skips the reference only (variation_classifier.py:185-215 walks
// those columns). Here each read's CIGAR is walked once per (scope, read) incidence into segment
// records — one per aligned run: (query nibble, reference nibble, length, dataset, whether this
// scope writes the read) — that k_group (ganon_hip.hip) streams in 16-base chunks.
//
// Kernels (integer work, HBM/latency bound, no MFMA), in launch order:
//   k_prep_reads    thread per read: CIGAR walk -> segments, aligned bases, bam_endpos; at upload
//                   also every per-read check of the old host validation (no host loop remains);
//   k_prep_scopes   workgroup per 256 consecutive scopes: their incidences are one contiguous
//                   CSR range, scope of an incidence by binary search in LDS; per-scope cost
//                   (segments + a per-scope weight that caps a group at 256 scopes) and overflow
//                   region size, LDS 64-bit atomics;
//   scans           rocPRIM device scans: exclusive prefix of (cost, region) over scopes, then
//                   the group index (a group = scopes whose cost prefix falls in one bucket of
//                   group_target units);
//   k_prep_emit     workgroup per group: scope metadata staged in LDS, each thread walks one
//                   incidence's CIGAR (segments of short CIGARs kept in registers, longer ones
//                   walked again) around a block scan; segments whose reference range is all
//                   ACGT fill the group's records from the front, the others from the back (the
//                   group kernel reads the front half through the 2-bit reference); the lowest
//                   buffer offset of the reads the group writes, per dataset (LDS atomicMin);
//   k_prep_pieces   rocPRIM radix sort of those 2 x groups candidates; the sorted candidates,
//                   aligned down to 128-byte lines, tile the output buffer — each group copies
//                   at most two pieces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "ganon_batch.h"

using namespace ganon_dev;
using ganon_detail::check_launch;
using ganon_detail::fail;
using ganon_detail::KernelScope;

namespace {

constexpr int kPrepThreads = 256;
constexpr int kScopeChunk = 256;      // scopes per k_prep_scopes workgroup
constexpr unsigned long long kNone = ~0ull;
constexpr int64_t kFarMax = int64_t(1) << 28;   // far-mask list entries at most

struct Pair {
  long long a, b;   // a: scope cost (segments + weight), b: overflow-region observations
};
struct PairPlus {
  __host__ __device__ Pair operator()(const Pair &x, const Pair &y) const { return Pair{x.a + y.a, x.b + y.b}; }
};

// The raw arrays and sizes every prep kernel reads.
struct Raw {
  const int32_t *ref_start, *read_len, *n_cig, *write_scope;
  const int64_t *seq_off, *cig_off;
  const uint8_t *dataset;
  const uint32_t *cigar;
  const int64_t *incid_off;
  const int32_t *incid_read;
  const int32_t *span_start, *span_len;
  const int64_t *ref_off;
  const uint8_t *keep_code;
  int32_t n_reads, n_scopes;
  int64_t n_incid, seq_bytes, n_cigar_ops, ref_nibs;
};

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
__device__ __forceinline__ void walk_segments(const uint32_t *__restrict__ cig, int nc, int L, int ref_start, F &&f) {
  int q = 0, p = ref_start;
  for (int k = 0; k < nc && q < L; ++k) {
    const uint32_t w = cig[k];
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

// ---- reference blocks -----------------------------------------------------------------------
// Bit k of bad: 64-base block k (32 bytes of nt16) holds a code other than A, C, G, T.
__global__ void __launch_bounds__(kPrepThreads) k_ref_blocks(const uint8_t *__restrict__ ref, int64_t bytes,
                                                             int64_t n_blk, uint64_t *__restrict__ bad) {
  const int64_t stride = (int64_t)gridDim.x * kPrepThreads;
  // n_blk rounded up to whole waves so that every lane reaches the ballot
  const int64_t n_round = (n_blk + 63) & ~(int64_t)63;
  for (int64_t k = blockIdx.x * (int64_t)kPrepThreads + threadIdx.x; k < n_round; k += stride) {
    bool b = false;
    if (k < n_blk) {
      const int64_t e = min(32 * k + 32, bytes);
      for (int64_t x = 32 * k; x < e; ++x) {
        const int v = ref[x];
        const int hi = v >> 4, lo = v & 15;
        b |= !((0x116 >> hi) & 1) || !((0x116 >> lo) & 1);
      }
    }
    const uint64_t m = __ballot(b);
    if ((threadIdx.x & 63) == 0) bad[k >> 6] = m;
  }
}

// ---- per read ------------------------------------------------------------------------------
__global__ void __launch_bounds__(kPrepThreads) k_prep_reads(const Raw R, int validate, PrepErr *err,
                                                             int32_t *__restrict__ rseg, int32_t *__restrict__ rbase,
                                                             int32_t *__restrict__ read_end,
                                                             unsigned long long *written) {
  int n_written = 0;
  for (int64_t r = blockIdx.x * (int64_t)kPrepThreads + threadIdx.x; r < R.n_reads;
       r += (int64_t)gridDim.x * kPrepThreads) {
    const int L = R.read_len[r];
    const int nc = R.n_cig[r];
    const int64_t co = R.cig_off[r];
    const int rs = R.ref_start[r];
    if (validate) {
      const int64_t so = R.seq_off[r];
      const int ws = R.write_scope[r];
      if (L < 0 || so < 0 || so + ((int64_t)L + 1) / 2 > R.seq_bytes) { report(err, kErrReadSeq, r); continue; }
      if (nc < 0 || co < 0 || co + nc > R.n_cigar_ops) { report(err, kErrReadCigar, r); continue; }
      if (R.dataset[r] > 1) report(err, kErrReadDataset, r);
      if (ws < -1 || ws >= R.n_scopes) report(err, kErrReadWriteScope, r, ws);
      if (L >= (1 << 24)) report(err, kErrReadLong, r);
      n_written += ws >= 0;
    }
    int q = 0, nseg = 0, bases = 0;
    int64_t rl = 0;
    for (int k = 0; k < nc; ++k) {
      const uint32_t w = R.cigar[co + k];
      const int op = (int)(w & 0xF);
      const int len = (int)(w >> 4);
      if (validate && op > 8) { report(err, kErrCigarOp, r, op); break; }
      if (is_aligned_op(op)) {
        if (q < L) {
          const int n = min(len, L - q);
          nseg += (n + kSegMaxLen - 1) / kSegMaxLen;
          bases += n;
        }
        q += len;
        rl += len;
      } else if (op == 1 || op == 4) {
        q += len;
      } else if (op == 2 || op == 3) {
        rl += len;
      }
      if (q > L) q = L;   // (the host walk stops emitting once q reaches L; clamp keeps q in int)
    }
    if (validate && (rs < 0 || rs + rl > INT32_MAX)) { report(err, kErrReadPos, r); continue; }
    rseg[r] = nseg;
    rbase[r] = bases;
    read_end[r] = (int32_t)(rs + (rl > 0 ? rl : 1));
  }
  if (validate) {
    for (int o = 32; o > 0; o >>= 1) n_written += __shfl_xor(n_written, o);
    if ((threadIdx.x & 63) == 0 && n_written) atomicAdd(written, (unsigned long long)n_written);
  }
}

// ---- per scope (validation only) -----------------------------------------------------------
__global__ void __launch_bounds__(kPrepThreads) k_prep_scope_check(const Raw R, PrepErr *err,
                                                                   unsigned long long *huge) {
  int n_huge = 0;
  for (int64_t s = blockIdx.x * (int64_t)kPrepThreads + threadIdx.x; s < R.n_scopes;
       s += (int64_t)gridDim.x * kPrepThreads) {
    const int64_t i0 = R.incid_off[s], i1 = R.incid_off[s + 1];
    if (i0 < 0 || i1 < i0 || i1 > R.n_incid) report(err, kErrScopeOff, s);
    const int64_t ss = R.span_start[s], sl = R.span_len[s];
    if (ss < 0 || sl < 0) report(err, kErrScopeSpan, s);
    if (R.ref_off[s] < 0 || R.ref_off[s] + sl > R.ref_nibs) report(err, kErrScopeRef, s);
    if (R.keep_code[s] > 15) report(err, kErrScopeKeep, s);
    n_huge += sl > kGrpMaxSpan;
  }
  for (int o = 32; o > 0; o >>= 1) n_huge += __shfl_xor(n_huge, o);
  if ((threadIdx.x & 63) == 0 && n_huge) atomicAdd(huge, (unsigned long long)n_huge);
}

// Largest j in [0, n) with off[j] <= i (off nondecreasing, off[0] <= i).
__device__ __forceinline__ int lds_upper(const long long *off, int n, long long i) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// ---- per scope: cost and region size; at upload also the incidence checks --------------------
__global__ void __launch_bounds__(kPrepThreads) k_prep_scopes(const Raw R, int validate, PrepErr *err,
                                                              const int32_t *__restrict__ rseg,
                                                              const int32_t *__restrict__ rbase,
                                                              const int32_t *__restrict__ read_end,
                                                              uint8_t *__restrict__ seen, long long weight,
                                                              Pair *__restrict__ cost) {
  __shared__ long long off[kScopeChunk + 1];
  __shared__ unsigned long long lseg[kScopeChunk], lbase[kScopeChunk];
  __shared__ int lss[kScopeChunk], lse[kScopeChunk];
  __shared__ uint8_t lhuge[kScopeChunk];
  const int tid = threadIdx.x;
  const int s0 = blockIdx.x * kScopeChunk;
  const int ns = min(kScopeChunk, R.n_scopes - s0);
  for (int t = tid; t <= ns; t += kPrepThreads) off[t] = R.incid_off[s0 + t];
  for (int t = tid; t < ns; t += kPrepThreads) {
    lseg[t] = 0;
    lbase[t] = 0;
    lss[t] = R.span_start[s0 + t];
    lse[t] = R.span_start[s0 + t] + R.span_len[s0 + t];
    lhuge[t] = R.span_len[s0 + t] > kGrpMaxSpan;
  }
  __syncthreads();
  const long long i0 = off[0], i1 = off[ns];
  for (long long i = i0 + tid; i < i1; i += kPrepThreads) {
    const int j = lds_upper(off, ns, i);
    const int r = R.incid_read[i];
    if (validate) {
      if (r < 0 || r >= R.n_reads) { report(err, kErrIncidRead, i, r); continue; }
      if (R.ref_start[r] < lss[j] || read_end[r] > lse[j]) { report(err, kErrIncidSpan, s0 + j, r); continue; }
      if (R.write_scope[r] == s0 + j) seen[r] = 1;
    }
    if (!lhuge[j]) {
      atomicAdd(&lseg[j], (unsigned long long)rseg[r]);
      atomicAdd(&lbase[j], (unsigned long long)rbase[r]);
    }
  }
  __syncthreads();
  for (int t = tid; t < ns; t += kPrepThreads)
    cost[s0 + t] = Pair{(long long)lseg[t] + weight, (long long)((lbase[t] + 47) / 48)};
}

__global__ void __launch_bounds__(kPrepThreads) k_prep_seen_check(const Raw R, const uint8_t *__restrict__ seen,
                                                                  PrepErr *err) {
  for (int64_t r = blockIdx.x * (int64_t)kPrepThreads + threadIdx.x; r < R.n_reads;
       r += (int64_t)gridDim.x * kPrepThreads)
    if (R.write_scope[r] >= 0 && !seen[r]) report(err, kErrWriteScopeMissing, r, R.write_scope[r]);
}

// Group head flag of scope s: its cost prefix starts a new bucket of `target` units.
struct HeadOp {
  const Pair *P;
  long long target;
  __host__ __device__ int operator()(int s) const { return s == 0 || (P[s].a / target) != (P[s - 1].a / target); }
};

// gs0[g] = first scope of group g.
__global__ void __launch_bounds__(kPrepThreads) k_prep_groups(const Pair *__restrict__ P, const int32_t *__restrict__ gid,
                                                              int n_scopes, long long target, int32_t *__restrict__ gs0) {
  for (int64_t s = blockIdx.x * (int64_t)kPrepThreads + threadIdx.x; s < n_scopes; s += (int64_t)gridDim.x * kPrepThreads)
    if (s == 0 || (P[s].a / target) != (P[s - 1].a / target)) gs0[gid[s] - 1] = (int32_t)s;
}

__device__ __forceinline__ int4 piece(int64_t a, int64_t b) {
  return make_int4((int)(uint32_t)a, (int)(uint32_t)((uint64_t)a >> 32), (int)(uint32_t)b,
                   (int)(uint32_t)((uint64_t)b >> 32));
}

// Partition pieces from the sorted candidates: candidate i starts at its offset aligned down to
// a line (the first at 0) and ends where the next candidate starts (the last at the end of the
// buffer); a candidate whose next one starts on the same line is empty. Slot d of group g holds
// the piece of its dataset-d candidate. No written read at all: one group copies everything.
__global__ void __launch_bounds__(kPrepThreads) k_prep_pieces(const unsigned long long *__restrict__ key,
                                                              const uint32_t *__restrict__ idx, int n_cand,
                                                              int64_t seq_bytes, int4 *__restrict__ groups) {
  for (int64_t i = blockIdx.x * (int64_t)kPrepThreads + threadIdx.x; i < n_cand;
       i += (int64_t)gridDim.x * kPrepThreads) {
    const unsigned long long k = key[i];
    const uint32_t v = idx[i];
    int4 pc = piece(0, 0);
    if (k != kNone) {
      const int64_t c = i == 0 ? 0 : (int64_t)(k & ~(unsigned long long)(kPartAlign - 1));
      const unsigned long long kn = i + 1 < n_cand ? key[i + 1] : kNone;
      const int64_t e = kn != kNone ? (int64_t)(kn & ~(unsigned long long)(kPartAlign - 1)) : seq_bytes;
      if (e > c) pc = piece(c, e);
    } else if (i == 0) {
      pc = piece(0, seq_bytes);
    }
    groups[kGrpRec * (int64_t)(v >> 1) + 2 + 2 * (v & 1)] = pc;
  }
}

__device__ __forceinline__ int64_t rec_lo(const int4 &x) { return (int64_t)(((uint64_t)(uint32_t)x.y << 32) | (uint32_t)x.x); }
__device__ __forceinline__ int64_t rec_hi(const int4 &x) { return (int64_t)(((uint64_t)(uint32_t)x.w << 32) | (uint32_t)x.z); }

// Upload only: nibbles of written reads outside their group's pieces (the far-mask capacity).
__global__ void __launch_bounds__(kPrepThreads) k_prep_farcap(const Raw R, const int32_t *__restrict__ gid,
                                                              const int4 *__restrict__ groups,
                                                              unsigned long long *far_nibs) {
  unsigned long long acc = 0;
  for (int64_t r = blockIdx.x * (int64_t)kPrepThreads + threadIdx.x; r < R.n_reads;
       r += (int64_t)gridDim.x * kPrepThreads) {
    const int ws = R.write_scope[r];
    if (ws < 0 || R.read_len[r] == 0 || R.span_len[ws] > kGrpMaxSpan) continue;
    const int64_t g = gid[ws] - 1;
    const int4 A = groups[kGrpRec * g + 2], Bp = groups[kGrpRec * g + 4];
    const int64_t r0 = R.seq_off[r], r1 = r0 + ((int64_t)R.read_len[r] + 1) / 2;
    const int64_t in = max((int64_t)0, min(r1, rec_hi(A)) - max(r0, rec_lo(A))) +
                       max((int64_t)0, min(r1, rec_hi(Bp)) - max(r0, rec_lo(Bp)));
    acc += (unsigned long long)(2 * ((r1 - r0) - in));
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(far_nibs, acc);
}

// Block-wide exclusive scan of two counters (256 threads).
__device__ __forceinline__ void block_scan2(int a, int b, int &ea, int &eb, int &ta, int &tb, int *ws) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int ia = a, ib = b;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int xa = __shfl_up(ia, o), xb = __shfl_up(ib, o);
    if (lane >= o) {
      ia += xa;
      ib += xb;
    }
  }
  if (lane == 63) {
    ws[wave] = ia;
    ws[kWaves + wave] = ib;
  }
  __syncthreads();
  int ba = 0, bb = 0;
  ta = tb = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    const int va = ws[w], vb = ws[kWaves + w];
    if (w < wave) {
      ba += va;
      bb += vb;
    }
    ta += va;
    tb += vb;
  }
  ea = ba + ia - a;
  eb = bb + ib - b;
  __syncthreads();
}

// Segment records, group records 0, 1, 3 and the partition candidates of group g: the lowest
// buffer offset of the reads the group writes, per dataset (lo[2g + d], kNone if none; every
// written read is "mine" in exactly one incidence, its write scope's).
constexpr int kRegSegs = 2;   // segments of an incidence kept in registers between count and write
__global__ void __launch_bounds__(kPrepThreads) k_prep_emit(const Raw R, const Pair *__restrict__ P,
                                                            const int32_t *__restrict__ gs0, int n_groups,
                                                            long long weight, const uint64_t *__restrict__ bad,
                                                            int64_t n_blk, int4 *__restrict__ seg4,
                                                            int4 *__restrict__ groups, unsigned long long *__restrict__ lo,
                                                            uint32_t *__restrict__ lo_idx) {
  __shared__ long long off[kGrpMaxScopes + 1];
  __shared__ long long ref0[kGrpMaxScopes];
  __shared__ int sstart[kGrpMaxScopes];
  __shared__ uint8_t huge[kGrpMaxScopes];
  __shared__ int ws[2 * kWaves];
  __shared__ unsigned long long lmin[2];
  const int tid = threadIdx.x;
  const int g = blockIdx.x;
  const int s0 = gs0[g];
  const int s1 = g + 1 < n_groups ? gs0[g + 1] : R.n_scopes;
  const int ns = s1 - s0;   // <= kGrpMaxScopes (the cost weight bounds a bucket)
  for (int t = tid; t <= ns; t += kPrepThreads) off[t] = R.incid_off[s0 + t];
  for (int t = tid; t < ns; t += kPrepThreads) {
    sstart[t] = R.span_start[s0 + t];
    ref0[t] = R.ref_off[s0 + t] - R.span_start[s0 + t];
    huge[t] = R.span_len[s0 + t] > kGrpMaxSpan;
  }
  if (tid < 2) lmin[tid] = kNone;
  const Pair p0 = P[s0], p1 = P[s1];
  const int64_t seg_b = p0.a - weight * s0, seg_e = p1.a - weight * s1;
  __syncthreads();
  const long long i0 = off[0], i1 = off[ns];
  int64_t run_c = 0, run_d = 0;   // records placed so far (clean from the front, dirty from the back)
  for (long long base = i0; base < i1; base += kPrepThreads) {
    const long long i = base + tid;
    int j = 0, r = -1;
    if (i < i1) {
      j = lds_upper(off, ns, i);
      r = huge[j] ? -1 : R.incid_read[i];
    }
    const uint32_t *cig = nullptr;
    int ncig = 0, L = 0, rs = 0, nc = 0, nd = 0, ds = 0;
    bool mine = false;
    int64_t so = 0;
    int4 keep[kRegSegs];
    bool kclean[kRegSegs];
    const int64_t r0 = ref0[j];
    const int ss = sstart[j];
    if (r >= 0) {
      cig = R.cigar + R.cig_off[r];
      ncig = R.n_cig[r];
      L = R.read_len[r];
      rs = R.ref_start[r];
      so = R.seq_off[r];
      ds = R.dataset[r];
      mine = R.write_scope[r] == s0 + j;
      if (mine && L > 0) atomicMin(&lmin[ds], (unsigned long long)so);
      const uint32_t fl = ((uint32_t)ds << 30) | (mine ? kSegMine : 0u);
      const int64_t qnib = 2 * so;
      walk_segments(cig, ncig, L, rs, [&](int q, int p, int n) {
        const uint64_t sq = (uint64_t)(qnib + q), rf = (uint64_t)(r0 + p);
        const bool clean = ref_clean(bad, n_blk, (int64_t)rf, n);
        const int k = nc + nd;
        if (k < kRegSegs) {
          const uint32_t z = (uint32_t)((sq >> 32) & 0xFF) | ((uint32_t)((rf >> 32) & 0xFF) << 8) | ((uint32_t)n << 16) | fl;
          keep[k] = make_int4((int)(uint32_t)sq, (int)(uint32_t)rf, (int)z, (int)((uint32_t)j | ((uint32_t)(p - ss) << 12)));
          kclean[k] = clean;
        }
        if (clean) ++nc;
        else ++nd;
      });
    }
    int ec, ed, tc, td;
    block_scan2(nc, nd, ec, ed, tc, td, ws);
    if (r >= 0 && nc + nd) {
      int64_t pc = seg_b + run_c + ec, pd = seg_e - 1 - (run_d + ed);
      if (nc + nd <= kRegSegs) {
#pragma unroll
        for (int k = 0; k < kRegSegs; ++k) {
          if (k >= nc + nd) break;
          if (kclean[k]) seg4[pc++] = keep[k];
          else seg4[pd--] = keep[k];
        }
      } else {
        const uint32_t fl = ((uint32_t)ds << 30) | (mine ? kSegMine : 0u);
        const int64_t qnib = 2 * so;
        walk_segments(cig, ncig, L, rs, [&](int q, int p, int n) {
          const uint64_t sq = (uint64_t)(qnib + q), rf = (uint64_t)(r0 + p);
          const uint32_t z = (uint32_t)((sq >> 32) & 0xFF) | ((uint32_t)((rf >> 32) & 0xFF) << 8) | ((uint32_t)n << 16) | fl;
          const int4 rec = make_int4((int)(uint32_t)sq, (int)(uint32_t)rf, (int)z,
                                     (int)((uint32_t)j | ((uint32_t)(p - ss) << 12)));
          if (ref_clean(bad, n_blk, (int64_t)rf, n)) seg4[pc++] = rec;
          else seg4[pd--] = rec;
        });
      }
    }
    run_c += tc;
    run_d += td;
  }
  __syncthreads();
  if (tid < 2) {
    lo[2 * (int64_t)g + tid] = lmin[tid];
    lo_idx[2 * (int64_t)g + tid] = (uint32_t)(2 * g + tid);
  }
  if (tid == 0) {
    const int64_t mid = seg_b + run_c;
    const int64_t region = p0.b + (int64_t)kGrpObs * g;
    const int64_t cap = min<int64_t>(p1.b - p0.b + kGrpObs, INT32_MAX / 2);
    groups[kGrpRec * (int64_t)g] = make_int4(s0, s1, (int)(uint32_t)seg_b, (int)(uint32_t)((uint64_t)seg_b >> 32));
    groups[kGrpRec * (int64_t)g + 1] = make_int4((int)(uint32_t)seg_e, (int)(uint32_t)((uint64_t)seg_e >> 32),
                                                 (int)(uint32_t)mid, (int)(uint32_t)((uint64_t)mid >> 32));
    groups[kGrpRec * (int64_t)g + 3] = make_int4((int)(uint32_t)region, (int)(uint32_t)((uint64_t)region >> 32),
                                                 (int)cap, 0);
  }
}

Raw raw_of(const ganon_dbatch *db) {
  const DevBatch &B = db->B;
  Raw R;
  R.ref_start = B.ref_start;
  R.read_len = B.read_len;
  R.n_cig = B.n_cig;
  R.write_scope = B.write_scope;
  R.seq_off = B.seq_off;
  R.cig_off = B.cig_off;
  R.dataset = B.dataset;
  R.cigar = B.cigar;
  R.incid_off = B.incid_off;
  R.incid_read = B.incid_read;
  R.span_start = B.span_start;
  R.span_len = B.span_len;
  R.ref_off = B.ref_off;
  R.keep_code = B.keep_code;
  R.n_reads = db->n_reads;
  R.n_scopes = db->n_scopes;
  R.n_incid = db->n_incid;
  R.seq_bytes = db->seq_bytes;
  R.n_cigar_ops = db->n_cigar_ops;
  R.ref_nibs = 2 * db->ref->bytes;
  return R;
}

unsigned grid_for(int64_t n, int64_t cap = 16384) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + kPrepThreads - 1) / kPrepThreads, cap));
}

long long weight_of(int target) { return (target + kGrpMaxScopes - 2) / (kGrpMaxScopes - 1); }

const char *err_text(int kind) {
  switch (kind) {
    case kErrReadSeq: return "read %lld: sequence out of range";
    case kErrReadCigar: return "read %lld: cigar out of range";
    case kErrReadDataset: return "read %lld: dataset must be 0 or 1";
    case kErrReadWriteScope: return "read %lld: write_scope %lld out of range";
    case kErrReadLong: return "read %lld longer than 16 Mb";
    case kErrCigarOp: return "read %lld: bad cigar op %lld";
    case kErrReadPos: return "read %lld: bad position";
    case kErrScopeOff: return "scope %lld: incidence offsets decreasing or out of range";
    case kErrScopeSpan: return "scope %lld: bad span";
    case kErrScopeRef: return "scope %lld: reference slice out of range";
    case kErrScopeKeep: return "scope %lld: keep_code > 15";
    case kErrIncidRead: return "incidence %lld: read %lld out of range";
    case kErrIncidSpan: return "scope %lld: read %lld outside its span";
    case kErrWriteScopeMissing: return "read %lld: write_scope %lld does not contain it";
    default: return "invalid batch (%lld)";
  }
}

int check_err(ganon_ctx *ctx, ganon_dbatch *db) {
  PrepErr e{};
  HIP_OR_FAIL(hipMemcpyAsync(&e, db->err, sizeof e, hipMemcpyDeviceToHost, ctx->stream));
  HIP_OR_FAIL(hipStreamSynchronize(ctx->stream));
  if (e.code) return fail(ctx, GANON_E_ARG, err_text(e.code), e.index, e.a, e.b);
  return GANON_OK;
}

// Temp storage of the three rocPRIM calls for n scopes and c candidates.
hipError_t scan_bytes(int64_t n, int64_t c, size_t &bytes) {
  size_t a = 0, b = 0, d = 0;
  hipError_t e = rocprim::exclusive_scan(nullptr, a, (Pair *)nullptr, (Pair *)nullptr, Pair{0, 0}, (size_t)n + 1,
                                         PairPlus{}, 0);
  if (e != hipSuccess) return e;
  e = rocprim::inclusive_scan(nullptr, b, rocprim::make_transform_iterator(rocprim::make_counting_iterator<int>(0),
                                                                          HeadOp{nullptr, 1}),
                              (int32_t *)nullptr, (size_t)n, rocprim::plus<int32_t>(), 0);
  if (e != hipSuccess) return e;
  e = rocprim::radix_sort_pairs(nullptr, d, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)c, 0, 40, 0);
  bytes = std::max(std::max(a, b), d);
  return e;
}

// The planning kernels shared by plan() and run(): scopes -> scans -> groups -> pieces.
int launch_scopes_groups(ganon_ctx *ctx, ganon_dbatch *db, const Raw &R, int validate) {
  hipStream_t st = ctx->stream;
  const long long w = weight_of(db->group_target);
  Pair *cost = static_cast<Pair *>(db->b_cost.p);
  Pair *P = static_cast<Pair *>(db->b_cost_scan.p);
  int32_t *gid = static_cast<int32_t *>(db->b_gid.p);
  {
    KernelScope ks(ctx, "prep_scopes");
    if (db->n_scopes) {
      hipLaunchKernelGGL(k_prep_scopes, dim3((unsigned)((db->n_scopes + kScopeChunk - 1) / kScopeChunk)),
                         dim3(kPrepThreads), 0, st, R, validate, db->err, static_cast<const int32_t *>(db->b_rseg.p),
                         static_cast<const int32_t *>(db->b_rbase.p), db->B.read_end,
                         static_cast<uint8_t *>(db->b_seen.p), w, cost);
      int rc = check_launch(ctx, "k_prep_scopes");
      if (rc) return rc;
    }
    HIP_OR_FAIL(hipMemsetAsync(cost + db->n_scopes, 0, sizeof(Pair), st));
  }
  if (validate) {
    hipLaunchKernelGGL(k_prep_seen_check, dim3(grid_for(db->n_reads)), dim3(kPrepThreads), 0, st, R,
                       static_cast<const uint8_t *>(db->b_seen.p), db->err);
    int rc = check_err(ctx, db);
    if (rc) return rc;
  }
  {
    KernelScope ks(ctx, "prep_scan");
    size_t bytes = db->scan_tmp_bytes;
    if (rocprim::exclusive_scan(db->b_scan_tmp.p, bytes, cost, P, Pair{0, 0}, (size_t)db->n_scopes + 1, PairPlus{},
                                st) != hipSuccess)
      return fail(ctx, GANON_E_DEVICE, "prep: scope scan failed");
    if (db->n_scopes) {
      bytes = db->scan_tmp_bytes;
      if (rocprim::inclusive_scan(db->b_scan_tmp.p, bytes,
                                  rocprim::make_transform_iterator(rocprim::make_counting_iterator<int>(0),
                                                                   HeadOp{P, (long long)db->group_target}),
                                  gid, (size_t)db->n_scopes, rocprim::plus<int32_t>(), st) != hipSuccess)
        return fail(ctx, GANON_E_DEVICE, "prep: group scan failed");
    }
  }
  return GANON_OK;
}

// Group starts, then (after the emit kernel wrote the candidates) sort + pieces.
int launch_groups(ganon_ctx *ctx, ganon_dbatch *db) {
  if (!db->n_groups) return GANON_OK;
  KernelScope ks(ctx, "prep_groups");
  hipLaunchKernelGGL(k_prep_groups, dim3(grid_for(db->n_scopes)), dim3(kPrepThreads), 0, ctx->stream,
                     static_cast<const Pair *>(db->b_cost_scan.p), static_cast<const int32_t *>(db->b_gid.p),
                     db->n_scopes, (long long)db->group_target, static_cast<int32_t *>(db->b_gs0.p));
  return check_launch(ctx, "k_prep_groups");
}

int launch_pieces(ganon_ctx *ctx, ganon_dbatch *db) {
  hipStream_t st = ctx->stream;
  const int n_cand = 2 * db->n_groups;
  if (!db->n_groups) return GANON_OK;
  KernelScope ks(ctx, "prep_pieces");
  auto *lo = static_cast<unsigned long long *>(db->b_lo.p);
  auto *lo_idx = static_cast<uint32_t *>(db->b_lo_idx.p);
  auto *lo_s = static_cast<unsigned long long *>(db->b_lo_sorted.p);
  auto *idx_s = static_cast<uint32_t *>(db->b_lo_idx_sorted.p);
  size_t bytes = db->scan_tmp_bytes;
  if (rocprim::radix_sort_pairs(db->b_scan_tmp.p, bytes, lo, lo_s, lo_idx, idx_s, (size_t)n_cand, 0, 40, st) !=
      hipSuccess)
    return fail(ctx, GANON_E_DEVICE, "prep: candidate sort failed");
  hipLaunchKernelGGL(k_prep_pieces, dim3(grid_for(n_cand)), dim3(kPrepThreads), 0, st, lo_s, idx_s, n_cand,
                     db->seq_bytes, static_cast<int4 *>(db->b_groups.p));
  return check_launch(ctx, "k_prep_pieces");
}

int launch_reads(ganon_ctx *ctx, ganon_dbatch *db, const Raw &R, int validate) {
  KernelScope ks(ctx, "prep_reads");
  if (!db->n_reads) return GANON_OK;
  hipLaunchKernelGGL(k_prep_reads, dim3(grid_for(db->n_reads)), dim3(kPrepThreads), 0, ctx->stream, R, validate,
                     db->err, static_cast<int32_t *>(db->b_rseg.p), static_cast<int32_t *>(db->b_rbase.p),
                     const_cast<int32_t *>(db->B.read_end), db->plan_info + 2);
  return check_launch(ctx, "k_prep_reads");
}

int launch_emit(ganon_ctx *ctx, ganon_dbatch *db, const Raw &R) {
  if (!db->n_groups) return GANON_OK;
  KernelScope ks(ctx, "prep_emit");
  hipLaunchKernelGGL(k_prep_emit, dim3((unsigned)db->n_groups), dim3(kPrepThreads), 0, ctx->stream, R,
                     static_cast<const Pair *>(db->b_cost_scan.p), static_cast<const int32_t *>(db->b_gs0.p),
                     db->n_groups, weight_of(db->group_target), db->ref->bad, db->ref->n_blk,
                     static_cast<int4 *>(db->b_seg4.p), static_cast<int4 *>(db->b_groups.p),
                     static_cast<unsigned long long *>(db->b_lo.p), static_cast<uint32_t *>(db->b_lo_idx.p));
  return check_launch(ctx, "k_prep_emit");
}

}  // namespace

namespace ganon_prep {

int grow(ganon_ctx *ctx, DBuf &b, size_t bytes) {
  const size_t need = bytes + 128;
  if (b.p && b.bytes >= need) return GANON_OK;
  if (b.p) {
    hipStreamSynchronize(ctx->stream);   // a previous run may still read it
    hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
  }
  const size_t alloc = std::max(need, b.bytes + b.bytes / 4);   // some headroom for reloads
  hipError_t e = hipMalloc(&b.p, alloc);
  if (e != hipSuccess) {
    b.p = nullptr;
    return fail(ctx, GANON_E_NOMEM, "hipMalloc(%zu) failed: %s", alloc, hipGetErrorString(e));
  }
  b.bytes = alloc;
  return GANON_OK;
}

int plan(ganon_ctx *ctx, ganon_dbatch *db) {
  hipStream_t st = ctx->stream;
  int rc;
  const int64_t nr = db->n_reads, ns = db->n_scopes;
  int32_t *p32 = nullptr;
  if ((rc = grow_n(ctx, db->b_read_end, nr, &p32))) return rc;
  db->B.read_end = p32;
  if ((rc = grow_n(ctx, db->b_rseg, nr, &p32)) || (rc = grow_n(ctx, db->b_rbase, nr, &p32))) return rc;
  uint8_t *seen = nullptr;
  if ((rc = grow_n(ctx, db->b_seen, nr, &seen))) return rc;
  Pair *pp = nullptr;
  if ((rc = grow_n(ctx, db->b_cost, ns + 1, &pp)) || (rc = grow_n(ctx, db->b_cost_scan, ns + 1, &pp))) return rc;
  if ((rc = grow_n(ctx, db->b_gid, ns, &p32))) return rc;
  // temp storage for the scans (candidates: at most one group per scope, two per group)
  size_t tmp = 0;
  if (scan_bytes(ns, 2 * ns, tmp) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "prep: rocPRIM sizing failed");
  uint8_t *t8 = nullptr;
  if ((rc = grow_n(ctx, db->b_scan_tmp, tmp, &t8))) return rc;
  db->scan_tmp_bytes = tmp;
  const Raw R = raw_of(db);
  HIP_OR_FAIL(hipMemsetAsync(db->err, 0, sizeof(PrepErr), st));
  HIP_OR_FAIL(hipMemsetAsync(db->plan_info, 0, 4 * sizeof(unsigned long long), st));
  HIP_OR_FAIL(hipMemsetAsync(seen, 0, (size_t)std::max<int64_t>(nr, 1), st));
  // 1. per-read and per-scope checks (every later kernel relies on them)
  if ((rc = launch_reads(ctx, db, R, 1))) return rc;
  if (ns) hipLaunchKernelGGL(k_prep_scope_check, dim3(grid_for(ns)), dim3(kPrepThreads), 0, st, R, db->err,
                             db->plan_info + 1);
  if ((rc = check_launch(ctx, "k_prep_scope_check")) || (rc = check_err(ctx, db))) return rc;
  // 2. incidences (checked inside), scans
  if ((rc = launch_scopes_groups(ctx, db, R, 1))) return rc;
  int32_t ng = 0;
  Pair total{0, 0};
  if (ns) HIP_OR_FAIL(hipMemcpyAsync(&ng, static_cast<int32_t *>(db->b_gid.p) + ns - 1, 4, hipMemcpyDeviceToHost, st));
  HIP_OR_FAIL(hipMemcpyAsync(&total, static_cast<Pair *>(db->b_cost_scan.p) + ns, sizeof total, hipMemcpyDeviceToHost, st));
  HIP_OR_FAIL(hipStreamSynchronize(st));
  db->n_groups = ng;
  db->n_seg = total.a - weight_of(db->group_target) * ns;
  db->region = total.b + (int64_t)kGrpObs * ng;
  // 3. derived buffers sized by the scans; groups, segments, pieces, far-mask capacity
  int4 *grp = nullptr;
  if ((rc = grow_n(ctx, db->b_groups, (size_t)kGrpRec * ng, &grp))) return rc;
  if ((rc = grow_n(ctx, db->b_gs0, ng, &p32))) return rc;
  unsigned long long *u64 = nullptr;
  uint32_t *u32 = nullptr;
  if ((rc = grow_n(ctx, db->b_lo, 2 * (size_t)ng, &u64)) || (rc = grow_n(ctx, db->b_lo_sorted, 2 * (size_t)ng, &u64)) ||
      (rc = grow_n(ctx, db->b_lo_idx, 2 * (size_t)ng, &u32)) ||
      (rc = grow_n(ctx, db->b_lo_idx_sorted, 2 * (size_t)ng, &u32)))
    return rc;
  int4 *s4 = nullptr;
  if ((rc = grow_n(ctx, db->b_seg4, (size_t)db->n_seg, &s4))) return rc;
  if ((rc = grow_n(ctx, db->b_grp_part, 2 * (size_t)ng, &p32))) return rc;
  if ((rc = launch_groups(ctx, db)) || (rc = launch_emit(ctx, db, R)) || (rc = launch_pieces(ctx, db))) return rc;
  if (ng && nr)
    hipLaunchKernelGGL(k_prep_farcap, dim3(grid_for(nr)), dim3(kPrepThreads), 0, st, R,
                       static_cast<const int32_t *>(db->b_gid.p), static_cast<const int4 *>(db->b_groups.p),
                       db->plan_info);
  if ((rc = check_launch(ctx, "k_prep_farcap"))) return rc;
  unsigned long long info[4] = {0, 0, 0, 0};
  HIP_OR_FAIL(hipMemcpyAsync(info, db->plan_info, sizeof info, hipMemcpyDeviceToHost, st));
  HIP_OR_FAIL(hipStreamSynchronize(st));
  // far masks: at most one per nibble of a written read outside its group's pieces. That bound is
  // exact but loose (masks are the TN-mismatching nibbles only), and a batch whose scopes are not
  // in genome order can put most written bytes outside their pieces: the list is capped at 2^28
  // entries (2 GiB); a run that needs more reports it (k_finish status) instead of dropping masks
  db->far_cap = std::min<int64_t>((int64_t)info[0], kFarMax);
  db->n_huge_scopes = (int32_t)info[1];
  db->n_written = (int64_t)info[2];
  if ((rc = grow_n(ctx, db->b_far, (size_t)db->far_cap, &u64))) return rc;
  if ((rc = grow_n(ctx, db->b_gokey, (size_t)db->region, &u64)) || (rc = grow_n(ctx, db->b_gopay, (size_t)db->region, &u64)) ||
      (rc = grow_n(ctx, db->b_gtkey, 2 * (size_t)db->region + 64, &u64)) ||
      (rc = grow_n(ctx, db->b_gtflag, 2 * (size_t)db->region + 64, &u32)))
    return rc;
  return GANON_OK;
}

int run(ganon_ctx *ctx, ganon_dbatch *db) {
  const Raw R = raw_of(db);
  int rc;
  if ((rc = launch_reads(ctx, db, R, 0))) return rc;
  if ((rc = launch_scopes_groups(ctx, db, R, 0))) return rc;
  if ((rc = launch_groups(ctx, db)) || (rc = launch_emit(ctx, db, R))) return rc;
  return launch_pieces(ctx, db);
}

}  // namespace ganon_prep

// Reference blocks of a resident reference (ganon_hip.hip ganon_ref_upload).
int ganon_ref_blocks(ganon_ctx *ctx, ganon_ref *ref) {
  if (!ref->n_blk) return GANON_OK;
  const int64_t n_round = (ref->n_blk + 63) & ~(int64_t)63;
  hipLaunchKernelGGL(k_ref_blocks, dim3(grid_for(n_round)), dim3(kPrepThreads), 0, ctx->stream, ref->nt16, ref->bytes,
                     ref->n_blk, ref->bad);
  return check_launch(ctx, "k_ref_blocks");
}
