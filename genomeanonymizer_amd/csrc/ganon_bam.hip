// ganon_bam.hip — BAM records to column arrays on MI355X (gfx950), part of libganon_hip.so; C ABI in
// include/ganon.h (ganon_bam_columns). SURVEY §8(f)4, its second half: the record walk after the
// inflate, which libganon_host.so does on the host (records_to_columns, csrc/ganon_host.cpp; the
// column view ganon_bam_view of include/ganon_host.h) and the reference gets from htslib's bam_read1
// behind AlignmentFile.fetch / pileup (pileup_io.pyx:12-17). The input is the inflated stream in
// device memory — k_inflate's output where the inflate ran on the device (ganon_inflate_device_output)
// — so the decoded records never cross PCIe.
//
// Record boundaries. Record k + 1 starts 4 + block_size(k) bytes after record k: a chain that one
// thread would walk at one dependent load per record. The stream [p, n) is cut into kChunk-byte
// chunks; chunk c holds the records that start in [p + c kChunk, p + (c + 1) kChunk). A wave per
// chunk guesses the chunk's first record start (the first offset from which kProbe chained records
// look like BAM records: sizes, reference ids, name terminator, read length against the block size)
// and one lane walks the chain to the chunk's end: its record count and exit (the first start at or past the
// chunk's end). The guesses are then proven: chunk 0 starts at p, and a chunk whose guess equals its
// predecessor's exit holds exactly the true records when its predecessor does — so by induction every
// chunk before the first failing one is exact. A failing chunk whose predecessor passed is walked
// again from that predecessor's exit, and the host repeats check and fix until no chunk fails (each
// round fixes at least the first failing run of chunks; `fixes` counts the failing chunks met).
// The exact walk checks what the host decoder checks (block_size >= 32, the record inside the
// stream), the per-record pass the rest (read length and CIGAR inside the block): same errors.
//
// Columns. Per-record sizes (name bytes kept with a NUL, CIGAR ops, packed sequence bytes, quality
// bytes, aux bytes), five exclusive scans (rocPRIM) for the blob offsets, then a wave per record:
// lanes 0-35 load the record's size and fixed fields once (broadcast by readlane), lane 0 writes the
// scalar columns, the wave copies name / CIGAR / sequence / quality / aux bytes lane-strided and sums
// the reference length of its CIGAR ops for bam_endpos. Bytes are copied as bytes: BAM fields are
// not aligned in the stream.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/ganon.h"
#include "../../include/ganon_host.h"
#include "ganon_ctx.h"

using ganon_detail::check_launch;
using ganon_detail::fail;

namespace {

constexpr int kBamThreads = 256;
constexpr int64_t kChunk = 2048;     // stream bytes per chunk (~6 short-read records)
constexpr int kProbe = 2;            // chained plausible records that make a guess (4: 0.23 vs 0.18 ms per 254 MB,
                                     // 506 vs 610 wrong guesses: each one costs a re-walk of a chunk, not a result)
constexpr int64_t kGuessSpan = 2 * kChunk;   // guess search window from the chunk start

__device__ __forceinline__ uint32_t rd32(const uint8_t *__restrict__ d, int64_t o) {
  return (uint32_t)d[o] | ((uint32_t)d[o + 1] << 8) | ((uint32_t)d[o + 2] << 16) | ((uint32_t)d[o + 3] << 24);
}

// 32 bits at any byte offset o of the stream [0, n) from the two aligned dwords that hold them
// (alignbyte): half the load instructions of four byte loads — the guess and the walk are bound
// by the texture path's per-instruction cost, not by bytes. Bytes near the stream's end, where the
// second dword would pass it, are read one by one.
__device__ __forceinline__ uint32_t ld32(const uint8_t *__restrict__ d, int64_t o, int64_t n) {
  const int64_t a = o & ~(int64_t)3;
  if (a + 8 > n) return rd32(d, o);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(d + a);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(o & 3));
}

// Does a BAM record plausibly start at o? (guesses only: a wrong guess is caught by the check)
__device__ __forceinline__ bool plausible(const uint8_t *__restrict__ d, int64_t o, int64_t n, int64_t &next) {
  if (o + 40 > n) {   // (the stream's last bytes: byte loads)
    if (o + 36 > n) return false;
  }
  uint32_t h[9];   // block_size and the fixed fields, [o, o + 36)
  if (o + 40 <= n) {
    const int64_t a = o & ~(int64_t)3;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(d + a);
    uint32_t x[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) x[k] = w[k];
    const uint32_t sh = (uint32_t)(o & 3);
#pragma unroll
    for (int k = 0; k < 9; ++k) h[k] = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) h[k] = rd32(d, o + 4 * k);
  }
  const int32_t bs = (int32_t)h[0];
  if (bs < 32 || o + 4 + (int64_t)bs > n) return false;
  const int32_t tid = (int32_t)h[1], pos = (int32_t)h[2];
  const int l_rn = (int)(h[3] & 0xFF);
  const int ncig = (int)(h[4] & 0xFFFF);
  const int32_t lseq = (int32_t)h[5];
  const int32_t mtid = (int32_t)h[6], mpos = (int32_t)h[7];
  if (tid < -1 || pos < -1 || mtid < -1 || mpos < -1 || l_rn < 1 || lseq < 0) return false;
  if (32 + (int64_t)l_rn + 4LL * ncig + ((int64_t)lseq + 1) / 2 + lseq > bs) return false;
  if (d[o + 4 + 32 + l_rn - 1] != 0) return false;
  next = o + 4 + bs;
  return true;
}

__device__ __forceinline__ bool chain_plausible(const uint8_t *__restrict__ d, int64_t o, int64_t n) {
  for (int k = 0; k < kProbe && o < n; ++k) {
    int64_t next;
    if (!plausible(d, o, n, next)) return false;
    o = next;
  }
  return true;
}

struct Chunks {
  int64_t *entry, *exitp, *cnt;
  int32_t *bad;     // 1: truncated size field, 2: bad block_size (the walk stopped there)
  uint8_t *flag;    // the chunk's entry is not its predecessor's exit
  unsigned long long *info;   // [failing chunks, first failing chunk, first bad chunk, first cut record]
  int64_t *tailp;   // (cut mode) the start of the record the stream's end cuts, -1 none
  bool cut;         // cut mode: the stream may end inside a record (a window of a region read); that
                    // record and the bytes after it are not records — the chain ends at its start
};

// Walk chunk c's chain from e (a record start, or < 0 for none): count and exit.
__device__ __forceinline__ void walk(const uint8_t *__restrict__ d, int64_t p, int64_t n, int64_t c, int64_t e,
                                     const Chunks &K) {
  const int64_t ce = min(n, p + (c + 1) * kChunk);
  int64_t s = e, k = 0, t = -1;
  int b = 0;
  if (s >= 0) {
    while (s < ce) {
      if (s + 4 > n) {
        if (K.cut) {   // (the chain ends here: every later chunk holds no record, entry = exit = n)
          t = s;
          s = n;
          break;
        }
        b = 1;
        break;
      }
      const int32_t bs = (int32_t)ld32(d, s, n);
      if (bs >= 32 && s + 4 + (int64_t)bs > n && K.cut) {
        t = s;
        s = n;
        break;
      }
      if (bs < 32 || s + 4 + (int64_t)bs > n) {
        b = 2;
        break;
      }
      s += 4 + (int64_t)bs;
      ++k;
    }
  }
  if (K.cut) K.tailp[c] = t;
  K.entry[c] = e;
  K.exitp[c] = b ? -2 : (e >= 0 ? s : -1);
  K.cnt[c] = k;
  K.bad[c] = b;
}

// Every chunk's guess and walk, a wave per chunk: the lanes test 64 consecutive candidate offsets at
// once (their first loads coalesced: a thread per chunk testing one offset after another made the
// byte loads of 64 lanes touch 64 cache lines apiece, 2.5 ms per 254 MB), the first plausible one
// (ballot) is the guess, and lane 0 walks the chain.
__global__ void __launch_bounds__(kBamThreads) k_bam_guess(const uint8_t *__restrict__ d, int64_t p, int64_t n,
                                                           int64_t n_chunks, Chunks K) {
  const int lane = threadIdx.x & 63;
  const int64_t c = ((int64_t)blockIdx.x * kBamThreads + threadIdx.x) >> 6;
  if (c >= n_chunks) return;   // (wave-uniform)
  int64_t e = -1;
  if (c == 0) {
    e = p;
  } else {
    const int64_t cs = p + c * kChunk, lim = min(n, cs + kGuessSpan);
    for (int64_t o0 = cs; o0 < lim; o0 += 64) {
      const int64_t o = o0 + lane;
      const unsigned long long m = __ballot(o < lim && chain_plausible(d, o, n));
      if (m) {
        e = o0 + __builtin_ctzll(m);
        break;
      }
    }
    if (e < 0 && lim == n) e = n;   // (no record starts in the rest of the stream: a guess too)
  }
  if (lane == 0) walk(d, p, n, c, e, K);
}

// A run of failing chunks whose predecessor passed, walked again from the predecessor's exit chunk
// after chunk by one thread (a long read's record covers several chunks that found no start: one
// round for the run).
__global__ void __launch_bounds__(kBamThreads) k_bam_fix(const uint8_t *__restrict__ d, int64_t p, int64_t n,
                                                         int64_t n_chunks, Chunks K) {
  const int64_t c = (int64_t)blockIdx.x * kBamThreads + threadIdx.x;
  if (c >= n_chunks || c == 0 || !K.flag[c] || K.flag[c - 1]) return;
  for (int64_t cc = c; cc < n_chunks && (cc == c || K.flag[cc]); ++cc) walk(d, p, n, cc, K.exitp[cc - 1], K);
}

__global__ void __launch_bounds__(kBamThreads) k_bam_check(int64_t n_chunks, Chunks K) {
  const int64_t c = (int64_t)blockIdx.x * kBamThreads + threadIdx.x;
  if (c >= n_chunks) return;
  const int64_t e = K.entry[c];
  const bool f = c > 0 && (e < 0 || e != K.exitp[c - 1]);
  K.flag[c] = f ? 1 : 0;
  if (f) {
    __hip_atomic_fetch_add(K.info, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_min(K.info + 1, (unsigned long long)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (K.bad[c]) __hip_atomic_fetch_min(K.info + 2, (unsigned long long)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // (read once no chunk fails: then every chunk is exact and at most one ends the chain at a cut)
  if (K.cut && K.tailp[c] >= 0)
    __hip_atomic_fetch_min(K.info + 3, (unsigned long long)K.tailp[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The record offsets: each chunk's chain again, from its proven entry, at its records' base index.
__global__ void __launch_bounds__(kBamThreads) k_bam_offsets(const uint8_t *__restrict__ d, int64_t p, int64_t n,
                                                             int64_t n_chunks, const int64_t *__restrict__ entry,
                                                             const int64_t *__restrict__ base,
                                                             int64_t *__restrict__ rec) {
  const int64_t c = (int64_t)blockIdx.x * kBamThreads + threadIdx.x;
  if (c >= n_chunks) return;
  const int64_t ce = min(n, p + (c + 1) * kChunk);
  int64_t s = entry[c], i = base[c];
  if (s < 0) return;
  while (s < ce) {
    if (s + 4 > n) break;   // (cut mode: the record the stream's end cuts is not one)
    const int64_t bs = (int64_t)(int32_t)ld32(d, s, n);
    if (s + 4 + bs > n) break;
    rec[i++] = s;
    s += 4 + bs;
  }
}

inline __device__ int64_t tid_order_d(int32_t t) { return t < 0 ? (int64_t)INT32_MAX : (int64_t)t; }

// A region read's records (ganon_bam_reader_region's scan_region, csrc/ganon_host.cpp): the window's
// records run from the region's first candidate; the region ends at the first record of another
// sequence or at pos >= end (info[0] = its index; info[1] = the same when that record's sequence
// comes before the region's: the index pointed before its sequence); a record before it is kept when
// bam_endpos > beg (htslib's overlap test). info[2] = 1: a record's CIGAR passes its block (the host
// decoder reports it).
__global__ void __launch_bounds__(kBamThreads) k_region_keep(const uint8_t *__restrict__ d, int64_t n,
                                                             const int64_t *__restrict__ rec, int64_t nr, int32_t tid,
                                                             int64_t beg, int64_t end, uint8_t *__restrict__ keep,
                                                             unsigned long long *__restrict__ info) {
  const int64_t i = (int64_t)blockIdx.x * kBamThreads + threadIdx.x;
  if (i >= nr) return;
  const int64_t o = rec[i];
  const int32_t bs = (int32_t)rd32(d, o), rtid = (int32_t)rd32(d, o + 4), rpos = (int32_t)rd32(d, o + 8);
  if (rtid != tid || (int64_t)rpos >= end) {
    keep[i] = 0;
    __hip_atomic_fetch_min(info, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid_order_d(rtid) < tid_order_d(tid))
      __hip_atomic_fetch_min(info + 1, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const int l_rn = d[o + 12];
  const int nc = (int)(d[o + 16] | (d[o + 17] << 8));
  const int flag = (int)(d[o + 18] | (d[o + 19] << 8));
  if (36 + (int64_t)l_rn + 4LL * nc > 4 + (int64_t)bs) {
    keep[i] = 1;
    info[2] = 1;   // (plain store of a constant: any writer's value is the same)
    return;
  }
  int64_t rl = 0;
  if (!(flag & 4))
    for (int k = 0; k < nc; ++k) {
      const uint32_t w = rd32(d, o + 36 + l_rn + 4LL * k);
      const int op = (int)(w & 0xF);
      if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += w >> 4;
    }
  keep[i] = (int64_t)rpos + (rl > 0 ? rl : 1) > beg ? 1 : 0;
}

struct Sizes {
  int64_t *name, *cig, *seq, *qual, *aux;   // [nr + 1] each (the last entry 0: the scan's total)
};

// Per record: the blob bytes it takes (records_to_columns' first pass), or the first bad record.
__global__ void __launch_bounds__(kBamThreads) k_bam_sizes(const uint8_t *__restrict__ d, const int64_t *__restrict__ rec,
                                                           int64_t nr, Sizes S, unsigned long long *__restrict__ first_bad) {
  const int64_t i = (int64_t)blockIdx.x * kBamThreads + threadIdx.x;
  if (i >= nr) return;
  const int64_t o = rec[i];
  const int32_t bs = (int32_t)rd32(d, o);
  const uint8_t *r = d + o + 4;
  const int l_rn = r[8];
  const int ncig = (int)(r[12] | (r[13] << 8));
  const int32_t lseq = (int32_t)rd32(r, 16);
  const int64_t need = 32 + (int64_t)l_rn + 4LL * ncig + ((int64_t)lseq + 1) / 2 + lseq;
  if (lseq < 0 || need > bs) {
    __hip_atomic_fetch_min(first_bad, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    S.name[i] = S.cig[i] = S.seq[i] = S.qual[i] = S.aux[i] = 0;
    return;
  }
  S.name[i] = l_rn + ((l_rn == 0 || r[32 + l_rn - 1] != 0) ? 1 : 0);
  S.cig[i] = ncig;
  S.seq[i] = ((int64_t)lseq + 1) / 2;
  S.qual[i] = lseq;
  S.aux[i] = bs - need;
}

}  // namespace

struct ganon_bam_dcols {
  ganon_bam_cols v{};          // device pointers
  void *block = nullptr;        // one block for the per-record columns
  void *blobs = nullptr;        // one block for the blobs
  uint8_t *stream = nullptr;    // the device copy of a host stream (on_host)
  size_t block_bytes = 0, blobs_bytes = 0, stream_bytes = 0;   // (context cache blocks)
  int64_t blobs_used = 0;       // bytes of the blob block the carve uses
  int64_t fixes = 0;            // failing chunks met by the checks (summed over the rounds)
};

namespace {

// Record i's columns and blob bytes, by one wave; src(k) = byte k of the record (its block_size
// field first), from global memory or from the block's LDS copy.
template <class Src>
__device__ __forceinline__ void scatter_record(const ganon_bam_cols &V, int64_t i, int lane, Src src) {
  uint8_t *cig8 = reinterpret_cast<uint8_t *>(V.cigar);
  const int hb = lane < 36 ? (int)src(lane) : 0;   // block_size + the fixed fields
  auto b = [&](int k) { return (uint32_t)__builtin_amdgcn_readlane(hb, k) & 0xFFu; };
  auto w32 = [&](int k) { return b(k) | (b(k + 1) << 8) | (b(k + 2) << 16) | (b(k + 3) << 24); };
  const int32_t bs = (int32_t)w32(0);
  const int l_rn = (int)b(12);
  const int ncig = (int)(b(16) | (b(17) << 8));
  const int flag = (int)(b(18) | (b(19) << 8));
  const int32_t lseq = (int32_t)w32(20);
  const int32_t pos = (int32_t)w32(8);
  const int64_t o_name = V.name_off[i], o_cig = V.cig_off[i], o_seq = V.seq_off[i], o_qual = V.qual_off[i],
                o_aux = V.aux_off[i];
  const int nseq = (int)(((int64_t)lseq + 1) / 2);
  const int e_name = l_rn, e_cig = e_name + 4 * ncig, e_seq = e_cig + nseq, e_qual = e_seq + lseq;
  const int body = bs - 32, na = body - e_qual;   // name .. aux: one byte stream, five blobs
  // each blob's destination less its first body index (wave-uniform): a byte's destination is
  // base[segment] + its body index
  uint8_t *const d_name = reinterpret_cast<uint8_t *>(V.names) + o_name, *const d_cig = cig8 + 4 * o_cig - e_name,
                 *const d_seq = V.seq + o_seq - e_cig, *const d_qual = V.qual + o_qual - e_seq,
                 *const d_aux = V.aux + o_aux - e_qual;
  // the body bytes, four loads in flight per lane before their stores
  for (int k0 = 0; k0 < body; k0 += 4 * 64) {
    uint8_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + 64 * u + lane;
      v[u] = k < body ? src(36 + k) : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + 64 * u + lane;
      if (k < body) {
        uint8_t *base = k < e_name ? d_name : k < e_cig ? d_cig : k < e_seq ? d_seq : k < e_qual ? d_qual : d_aux;
        base[k] = v[u];
      }
    }
  }
  if (lane == 0 && V.name_off[i + 1] - o_name > l_rn) V.names[o_name + l_rn] = 0;   // (a name without its NUL)
  // the reference length of the M / D / N / = / X ops (bam_endpos)
  unsigned long long rl = 0;
  for (int k = lane; k < ncig; k += 64) {
    const int64_t q = 36 + e_name + 4LL * k;
    const uint32_t w = (uint32_t)src(q) | ((uint32_t)src(q + 1) << 8) | ((uint32_t)src(q + 2) << 16) | ((uint32_t)src(q + 3) << 24);
    const int op = (int)(w & 0xF);
    if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += w >> 4;
  }
  for (int s = 32; s > 0; s >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)rl, s), hi = (uint32_t)__shfl_xor((int)(uint32_t)(rl >> 32), s);
    rl += ((unsigned long long)hi << 32) | lo;
  }
  if (lane == 0) {
    const int64_t rlen = (flag & 4) ? 0 : (int64_t)rl;
    V.tid[i] = (int32_t)w32(4);
    V.pos[i] = pos;
    V.end[i] = (int32_t)(pos + (rlen > 0 ? rlen : 1));
    V.flag[i] = flag;
    V.mapq[i] = (int)b(13);
    V.l_seq[i] = lseq;
    V.n_cigar[i] = ncig;
    V.mate_tid[i] = (int32_t)w32(24);
    V.mate_pos[i] = (int32_t)w32(28);
    V.tlen[i] = (int32_t)w32(32);
    V.name_len[i] = l_rn > 0 ? l_rn - 1 : 0;
    V.aux_len[i] = (int32_t)na;
  }
}

#ifndef GANON_SCAT_RECS
#define GANON_SCAT_RECS 32         // (profiles/r06/bam_sr: 8 0.643, 16 0.615, 32 0.598, 64 0.836 ms)
#endif
#ifndef GANON_SCAT_STAGE
#define GANON_SCAT_STAGE 16384
#endif
constexpr int kScatRecs = GANON_SCAT_RECS;    // records per workgroup (eight per wave)
constexpr int kStage = GANON_SCAT_STAGE;      // LDS bytes staged per workgroup

// A wave per record. The workgroup's run of kScatRecs records (back to back in the stream) is first
// copied to LDS with coalesced aligned dword loads, then each wave reads its record's bytes from
// there (a byte per lane per instruction from global memory, BAM fields being unaligned, cost the
// texture path as much as the stores); a run longer than the LDS copy reads global memory.
__global__ void __launch_bounds__(kBamThreads) k_bam_scatter(const uint8_t *__restrict__ d, int64_t n,
                                                             const int64_t *__restrict__ rec, int64_t nr,
                                                             ganon_bam_cols V) {
  __shared__ uint32_t stage[kStage / 4];
  const int64_t i0 = (int64_t)blockIdx.x * kScatRecs;
  if (i0 >= nr) return;
  const int64_t i1 = min(nr, i0 + kScatRecs);
  const int64_t s0 = rec[i0], s1 = i1 < nr ? rec[i1] : n;   // (records lie back to back up to n)
  const int64_t a0 = s0 & ~(int64_t)3;
  const bool fits = s1 - a0 <= kStage;
  if (fits) {
    const int nw = (int)((s1 - a0 + 3) >> 2);
    for (int w = threadIdx.x; w < nw; w += kBamThreads) {
      const int64_t a = a0 + 4LL * w;
      uint32_t v;
      if (a + 4 <= n) {
        v = *reinterpret_cast<const uint32_t *>(d + a);
      } else {
        v = 0;
        for (int k = 0; k < 4; ++k)
          if (a + k < n) v |= (uint32_t)d[a + k] << (8 * k);
      }
      stage[w] = v;
    }
  }
  __syncthreads();
  const uint8_t *sb = reinterpret_cast<const uint8_t *>(stage);
  const int lane = threadIdx.x & 63;
  for (int64_t i = i0 + (threadIdx.x >> 6); i < i1; i += kBamThreads / 64) {
    const int64_t o = rec[i];
    if (fits) {
      const int base = (int)(o - a0);
      scatter_record(V, i, lane, [&](int64_t k) { return sb[base + k]; });
    } else {
      scatter_record(V, i, lane, [&](int64_t k) { return d[o + k]; });
    }
  }
}

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + kBamThreads - 1) / kBamThreads); }

template <typename T>
T *carve(uint8_t *&at, int64_t count) {
  T *p = reinterpret_cast<T *>(at);
  at += ((count * (int64_t)sizeof(T) + 255) / 256) * 256;
  return p;
}

// A region read's request (ganon_region_decode): the records of sequence tid overlapping [beg, end)
// from the window's first record on. status out: 1 the region ends inside the window (the columns
// are its records'), 0 it goes on past the window, 2 declined — the window holds a malformed record
// or the index pointed before the sequence: the host's walk reports those.
struct RegionReq {
  int32_t tid;
  int64_t beg, end;
  bool at_eof;   // the window ends at the end of the file
  int status;
};

int columns(ganon_ctx *ctx, const uint8_t *d, int64_t p, int64_t n, ganon_bam_dcols *H, RegionReq *rg = nullptr) {
  hipStream_t s = ctx->stream;
  const int64_t n_chunks = n > p ? (n - p + kChunk - 1) / kChunk : 0;
  int rc;
  // chunk arrays and the scans' temporary space from the context's block cache (stream-ordered
  // reuse: no hipMalloc / hipFree, which synchronize, once a call of this size has run)
  std::vector<std::pair<void *, size_t>> tmp;
  auto dalloc = [&](size_t bytes) -> void * {
    void *q = nullptr;
    size_t got = 0;
    if (ctx_dmalloc(ctx, &q, std::max<size_t>(bytes, 256), &got) != hipSuccess) return nullptr;
    tmp.emplace_back(q, got);
    return q;
  };
  struct Free {
    ganon_ctx *ctx;
    std::vector<std::pair<void *, size_t>> &t;
    ~Free() {
      for (auto &q : t) ctx_dfree(ctx, q.first, q.second);
    }
  } free_tmp{ctx, tmp};
  Chunks K{};
  int64_t *base = nullptr;
  unsigned long long tail = ~0ull;   // (cut mode) the record the window's end cuts
  if (n_chunks) {
    const int64_t nc = n_chunks;
    K.entry = static_cast<int64_t *>(dalloc(nc * 8));
    K.exitp = static_cast<int64_t *>(dalloc(nc * 8));
    K.cnt = static_cast<int64_t *>(dalloc((nc + 1) * 8));
    base = static_cast<int64_t *>(dalloc((nc + 1) * 8));
    K.bad = static_cast<int32_t *>(dalloc(nc * 4));
    K.flag = static_cast<uint8_t *>(dalloc(nc));
    K.info = static_cast<unsigned long long *>(dalloc(4 * 8));
    K.cut = rg != nullptr;
    K.tailp = rg ? static_cast<int64_t *>(dalloc(nc * 8)) : nullptr;
    if (!K.entry || !K.exitp || !K.cnt || !base || !K.bad || !K.flag || !K.info || (rg && !K.tailp))
      return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: device allocation failed");
    {
      ganon_detail::KernelScope ks(ctx, "k_bam_guess");
      hipLaunchKernelGGL(k_bam_guess, dim3(grid_of(64 * nc)), dim3(kBamThreads), 0, s, d, p, n, nc, K);
    }
    if ((rc = check_launch(ctx, "k_bam_guess"))) return rc;
    for (int64_t round = 0;; ++round) {
      const unsigned long long init[4] = {0ull, ~0ull, ~0ull, ~0ull};
      unsigned long long info[4];
      HIP_OR_FAIL(hipMemcpyAsync(K.info, init, sizeof init, hipMemcpyHostToDevice, s));
      {
        ganon_detail::KernelScope ks(ctx, "k_bam_check");
        hipLaunchKernelGGL(k_bam_check, dim3(grid_of(nc)), dim3(kBamThreads), 0, s, nc, K);
      }
      if ((rc = check_launch(ctx, "k_bam_check"))) return rc;
      HIP_OR_FAIL(ganon_detail::readback(info, K.info, sizeof info, s));
      HIP_OR_FAIL(ganon_detail::sync_stream(s));
      // every chunk before the first failing one is exact: a bad walk there is the stream's error
      if (info[2] != ~0ull && info[2] < info[1]) {
        if (rg) {
          rg->status = 2;
          return GANON_OK;
        }
        return fail(ctx, GANON_E_ARG, "ganon_bam_columns: bad record size (chunk %lld)", (long long)info[2]);
      }
      if (info[0] == 0) {
        tail = info[3];
        break;
      }
      if (round > nc) return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: record chain did not settle");
      H->fixes += (int64_t)info[0];
      {
        ganon_detail::KernelScope ks(ctx, "k_bam_fix");
        hipLaunchKernelGGL(k_bam_fix, dim3(grid_of(nc)), dim3(kBamThreads), 0, s, d, p, n, nc, K);
      }
      if ((rc = check_launch(ctx, "k_bam_fix"))) return rc;
    }
    HIP_OR_FAIL(hipMemsetAsync(K.cnt + nc, 0, 8, s));
    size_t tb = 0;
    HIP_OR_FAIL(rocprim::exclusive_scan(nullptr, tb, K.cnt, base, (int64_t)0, (size_t)(nc + 1), rocprim::plus<int64_t>(), s));
    void *tsc = dalloc(tb);
    if (!tsc) return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: device allocation failed");
    HIP_OR_FAIL(rocprim::exclusive_scan(tsc, tb, K.cnt, base, (int64_t)0, (size_t)(nc + 1), rocprim::plus<int64_t>(), s));
  }
  int64_t nr = 0;
  if (n_chunks) {
    HIP_OR_FAIL(ganon_detail::readback(&nr, base + n_chunks, 8, s));
    HIP_OR_FAIL(ganon_detail::sync_stream(s));
  }
  // A region read: the window's records up to the region's end, those overlapping [beg, end) kept
  // (a stream compaction of their offsets); the columns below are built for those alone.
  int64_t *sel = nullptr;
  if (rg) {
    if (rg->at_eof && tail != ~0ull) {   // the file ends inside a record: the host's error
      rg->status = 2;
      return GANON_OK;
    }
    int64_t *all = static_cast<int64_t *>(dalloc((size_t)(nr + 1) * 8));
    uint8_t *keep = static_cast<uint8_t *>(dalloc((size_t)nr + 1));
    unsigned long long *ri = static_cast<unsigned long long *>(dalloc(3 * 8));
    sel = static_cast<int64_t *>(dalloc((size_t)(nr + 1) * 8));
    int64_t *cnt = static_cast<int64_t *>(dalloc(8));
    if (!all || !keep || !ri || !sel || !cnt) return fail(ctx, GANON_E_DEVICE, "ganon_region_decode: device allocation failed");
    const unsigned long long init[3] = {~0ull, ~0ull, 0ull};
    unsigned long long info[3] = {~0ull, ~0ull, 0ull};
    HIP_OR_FAIL(hipMemcpyAsync(ri, init, sizeof init, hipMemcpyHostToDevice, s));
    if (nr) {
      {
        ganon_detail::KernelScope ks(ctx, "k_bam_offsets");
        hipLaunchKernelGGL(k_bam_offsets, dim3(grid_of(n_chunks)), dim3(kBamThreads), 0, s, d, p, n, n_chunks, K.entry,
                           base, all);
      }
      if ((rc = check_launch(ctx, "k_bam_offsets"))) return rc;
      {
        ganon_detail::KernelScope ks(ctx, "k_region_keep");
        hipLaunchKernelGGL(k_region_keep, dim3(grid_of(nr)), dim3(kBamThreads), 0, s, d, n, all, nr, rg->tid, rg->beg,
                           rg->end, keep, ri);
      }
      if ((rc = check_launch(ctx, "k_region_keep"))) return rc;
      HIP_OR_FAIL(ganon_detail::readback(info, ri, sizeof info, s));
      HIP_OR_FAIL(ganon_detail::sync_stream(s));
    }
    if (info[2] || (info[1] != ~0ull && info[1] == info[0])) {
      rg->status = 2;
      return GANON_OK;
    }
    if (info[0] == ~0ull && (!rg->at_eof || tail != ~0ull)) {   // the region goes on past the window
      rg->status = 0;
      return GANON_OK;
    }
    const int64_t cut = info[0] == ~0ull ? nr : (int64_t)info[0];
    int64_t nk = 0;
    if (cut > 0) {
      size_t tb = 0;
      HIP_OR_FAIL(rocprim::select(nullptr, tb, all, keep, sel, cnt, (size_t)cut, s));
      void *tsel = dalloc(tb);
      if (!tsel) return fail(ctx, GANON_E_DEVICE, "ganon_region_decode: device allocation failed");
      HIP_OR_FAIL(rocprim::select(tsel, tb, all, keep, sel, cnt, (size_t)cut, s));
      HIP_OR_FAIL(ganon_detail::readback(&nk, cnt, 8, s));
      HIP_OR_FAIL(ganon_detail::sync_stream(s));
    }
    nr = nk;
    rg->status = 1;
  }
  // per-record columns: 12 int32 + 6 int64 (5 offsets of nr + 1, the record offsets) + the sizes
  ganon_bam_cols &V = H->v;
  V.n_records = nr;
  {
    const int64_t m = nr + 1;
    const int64_t bytes = 12 * (((m * 4) + 255) / 256 * 256) + 11 * (((m * 8) + 255) / 256 * 256);
    if (ctx_dmalloc(ctx, &H->block, (size_t)std::max<int64_t>(bytes, 256), &H->block_bytes) != hipSuccess)
      return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: device allocation of %lld bytes failed", (long long)bytes);
    uint8_t *at = static_cast<uint8_t *>(H->block);
    for (int32_t **f : {&V.tid, &V.pos, &V.end, &V.flag, &V.mapq, &V.l_seq, &V.n_cigar, &V.mate_tid, &V.mate_pos, &V.tlen,
                        &V.name_len, &V.aux_len})
      *f = carve<int32_t>(at, m);
    for (int64_t **f : {&V.name_off, &V.cig_off, &V.seq_off, &V.qual_off, &V.aux_off, &V.rec_off}) *f = carve<int64_t>(at, m);
    Sizes S{carve<int64_t>(at, m), carve<int64_t>(at, m), carve<int64_t>(at, m), carve<int64_t>(at, m),
            carve<int64_t>(at, m)};
    unsigned long long *first_bad = static_cast<unsigned long long *>(dalloc(8));
    if (!first_bad) return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: device allocation failed");
    const unsigned long long none = ~0ull;
    HIP_OR_FAIL(hipMemcpyAsync(first_bad, &none, 8, hipMemcpyHostToDevice, s));
    if (sel) {
      if (nr) HIP_OR_FAIL(hipMemcpyAsync(V.rec_off, sel, (size_t)nr * 8, hipMemcpyDeviceToDevice, s));
    } else {
      if (nr) {
        ganon_detail::KernelScope ks(ctx, "k_bam_offsets");
        hipLaunchKernelGGL(k_bam_offsets, dim3(grid_of(n_chunks)), dim3(kBamThreads), 0, s, d, p, n, n_chunks, K.entry,
                           base, V.rec_off);
      }
      if ((rc = check_launch(ctx, "k_bam_offsets"))) return rc;
    }
    for (int64_t *z : {S.name, S.cig, S.seq, S.qual, S.aux}) HIP_OR_FAIL(hipMemsetAsync(z + nr, 0, 8, s));
    if (nr) {
      ganon_detail::KernelScope ks(ctx, "k_bam_sizes");
      hipLaunchKernelGGL(k_bam_sizes, dim3(grid_of(nr)), dim3(kBamThreads), 0, s, d, V.rec_off, nr, S, first_bad);
    }
    if ((rc = check_launch(ctx, "k_bam_sizes"))) return rc;
    size_t tb = 0;
    HIP_OR_FAIL(rocprim::exclusive_scan(nullptr, tb, S.name, V.name_off, (int64_t)0, (size_t)m, rocprim::plus<int64_t>(), s));
    void *tsc = dalloc(tb);
    if (!tsc) return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: device allocation failed");
    {
      ganon_detail::KernelScope ks(ctx, "bam_scans");
      const std::pair<int64_t *, int64_t *> io[5] = {{S.name, V.name_off}, {S.cig, V.cig_off}, {S.seq, V.seq_off},
                                                     {S.qual, V.qual_off}, {S.aux, V.aux_off}};
      for (const auto &x : io)
        HIP_OR_FAIL(rocprim::exclusive_scan(tsc, tb, x.first, x.second, (int64_t)0, (size_t)m, rocprim::plus<int64_t>(), s));
    }
    unsigned long long bad_rec = ~0ull;
    int64_t tot[5];
    HIP_OR_FAIL(ganon_detail::readback(&bad_rec, first_bad, 8, s));
    int64_t *offs[5] = {V.name_off, V.cig_off, V.seq_off, V.qual_off, V.aux_off};
    for (int k = 0; k < 5; ++k) HIP_OR_FAIL(ganon_detail::readback(&tot[k], offs[k] + nr, 8, s));
    HIP_OR_FAIL(ganon_detail::sync_stream(s));
    if (bad_rec != ~0ull) {
      if (rg) {
        rg->status = 2;
        return GANON_OK;
      }
      return fail(ctx, GANON_E_ARG, "ganon_bam_columns: record %lld: fields exceed block size", (long long)bad_rec);
    }
    V.names_bytes = tot[0];
    V.cigar_ops = tot[1];
    V.seq_bytes = tot[2];
    V.qual_bytes = tot[3];
    V.aux_bytes = tot[4];
  }
  {
    const int64_t rb = ((V.names_bytes + 255) / 256 + (4 * V.cigar_ops + 255) / 256 + (V.seq_bytes + 255) / 256 +
                        (V.qual_bytes + 255) / 256 + (V.aux_bytes + 255) / 256) * 256;
    if (ctx_dmalloc(ctx, &H->blobs, (size_t)std::max<int64_t>(rb, 256), &H->blobs_bytes) != hipSuccess)
      return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: device allocation of %lld bytes failed", (long long)rb);
    uint8_t *at = static_cast<uint8_t *>(H->blobs);
    V.names = carve<char>(at, V.names_bytes);
    V.cigar = carve<uint32_t>(at, V.cigar_ops);
    V.seq = carve<uint8_t>(at, V.seq_bytes);
    V.qual = carve<uint8_t>(at, V.qual_bytes);
    V.aux = carve<uint8_t>(at, V.aux_bytes);
    H->blobs_used = rb;
  }
  if (nr) {
    ganon_detail::KernelScope ks(ctx, "k_bam_scatter");
    const unsigned grid = (unsigned)((nr + kScatRecs - 1) / kScatRecs);
    hipLaunchKernelGGL(k_bam_scatter, dim3(grid), dim3(kBamThreads), 0, s, d, n, V.rec_off, nr, V);
  }
  if ((rc = check_launch(ctx, "k_bam_scatter"))) return rc;
  return ganon_batch_sync(ctx);   // (collects the kernel times when profiling)
}

void release(ganon_ctx *ctx, ganon_bam_dcols *H) {
  if (!H) return;
  ctx_dfree(ctx, H->block, H->block_bytes);
  ctx_dfree(ctx, H->blobs, H->blobs_bytes);
  ctx_dfree(ctx, H->stream, H->stream_bytes);
  delete H;
}

}  // namespace

GANON_API int ganon_bam_columns(ganon_ctx *ctx, const uint8_t *stream, int64_t p, int64_t n, int on_host,
                                ganon_bam_dcols **out) {
  if (!ctx || !out || p < 0 || n < p || (n > 0 && !stream))
    return fail(ctx, GANON_E_ARG, "ganon_bam_columns: bad arguments");
  if (!on_host && (reinterpret_cast<uintptr_t>(stream) & 3))   // (the walks read aligned dwords)
    return fail(ctx, GANON_E_ARG, "ganon_bam_columns: a device stream must be 4-byte aligned");
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipSetDevice failed");
  if (ctx->profiling) {   // a profiled call: ganon_last_kernel_times reports this call's kernels alone
    ganon_detail::sync_stream(ctx->stream);
    for (auto &r : ctx->recs) {
      ctx->pool.push_back(r.e0);
      ctx->pool.push_back(r.e1);
    }
    ctx->recs.clear();
  }
  auto *H = new ganon_bam_dcols();
  const uint8_t *d = stream;
  if (on_host && n > 0) {
    if (ctx_dmalloc(ctx, reinterpret_cast<void **>(&H->stream), (size_t)n, &H->stream_bytes) != hipSuccess) {
      release(ctx, H);
      return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: device allocation of %lld bytes failed", (long long)n);
    }
    // (waited for: the kernel events that follow time the record walk, not the copy)
    if (hipMemcpyAsync(H->stream, stream, (size_t)n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
        ganon_detail::sync_stream(ctx->stream) != hipSuccess) {
      ganon_detail::sync_stream(ctx->stream);
      release(ctx, H);
      return fail(ctx, GANON_E_DEVICE, "ganon_bam_columns: stream copy failed");
    }
    d = H->stream;
  }
  const int rc = columns(ctx, d, p, n, H);
  if (rc) {
    ganon_detail::sync_stream(ctx->stream);
    release(ctx, H);
    return rc;
  }
  *out = H;
  return GANON_OK;
}

GANON_API int ganon_bam_dcols_get(const ganon_bam_dcols *c, ganon_bam_cols *device_view, int64_t *fixes) {
  if (!c || !device_view) return GANON_E_ARG;
  *device_view = c->v;
  if (fixes) *fixes = c->fixes;
  return GANON_OK;
}

GANON_API int ganon_bam_dcols_download(ganon_ctx *ctx, const ganon_bam_dcols *c, const ganon_bam_cols *host) {
  if (!ctx || !c || !host) return fail(ctx, GANON_E_ARG, "ganon_bam_dcols_download: bad arguments");
  const ganon_bam_cols &V = c->v;
  const int64_t nr = V.n_records;
  hipStream_t s = ctx->stream;
  auto cp = [&](void *dst, const void *src, int64_t bytes) {
    return !dst || bytes <= 0 || hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, s) == hipSuccess;
  };
  bool ok = true;
  const std::pair<int32_t *, const int32_t *> i32[12] = {
      {host->tid, V.tid}, {host->pos, V.pos}, {host->end, V.end}, {host->flag, V.flag}, {host->mapq, V.mapq},
      {host->l_seq, V.l_seq}, {host->n_cigar, V.n_cigar}, {host->mate_tid, V.mate_tid}, {host->mate_pos, V.mate_pos},
      {host->tlen, V.tlen}, {host->name_len, V.name_len}, {host->aux_len, V.aux_len}};
  for (const auto &x : i32) ok = ok && cp(x.first, x.second, nr * 4);
  const std::pair<int64_t *, const int64_t *> i64[6] = {{host->name_off, V.name_off}, {host->cig_off, V.cig_off},
                                                        {host->seq_off, V.seq_off},   {host->qual_off, V.qual_off},
                                                        {host->aux_off, V.aux_off},   {host->rec_off, V.rec_off}};
  for (const auto &x : i64) ok = ok && cp(x.first, x.second, nr * 8);
  ok = ok && cp(host->names, V.names, V.names_bytes) && cp(host->cigar, V.cigar, 4 * V.cigar_ops) &&
       cp(host->seq, V.seq, V.seq_bytes) && cp(host->qual, V.qual, V.qual_bytes) && cp(host->aux, V.aux, V.aux_bytes);
  if (!ok || ganon_detail::sync_stream(s) != hipSuccess) {
    ganon_detail::sync_stream(s);
    return fail(ctx, GANON_E_DEVICE, "ganon_bam_dcols_download: copy failed");
  }
  return GANON_OK;
}

GANON_API int ganon_bam_dcols_free(ganon_ctx *ctx, ganon_bam_dcols *c) {
  if (ctx) ganon_detail::sync_stream(ctx->stream);
  release(ctx, c);
  return GANON_OK;
}

// ---- a region read decoded on the device (the reader's region decoder, ganon_bam_reader_region) ----
GANON_API int ganon_region_decode(void *user, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                                  const int32_t *in_len, const int64_t *out_off, const int32_t *out_len,
                                  int64_t n_blocks, uint8_t *out, int64_t out_total, int64_t p0, int32_t tid,
                                  int64_t beg, int64_t end, int at_eof, ganon_bam_view *cols, void **block) {
  ganon_ctx *ctx = static_cast<ganon_ctx *>(user);
  if (!ctx || !cols || !block || (out_total > 0 && !out) || p0 < 0) return -1;
  *block = nullptr;
  if (ganon_inflate_impl(ctx, comp, comp_len, in_off, in_len, out_off, out_len, n_blocks, nullptr, out_total, nullptr))
    return -1;   // (the inflate failed: ctx->err)
  const uint8_t *dout = nullptr;
  int64_t bytes = 0;
  if (ganon_inflate_device_output(ctx, &dout, &bytes) || bytes != out_total) return -1;
  hipStream_t s = ctx->stream;
  // the host's walk goes on from the inflated window: its bytes to `out`
  auto raw = [&]() -> int {
    if (out_total > 0 && (hipMemcpyAsync(out, dout, (size_t)out_total, hipMemcpyDeviceToHost, s) != hipSuccess ||
                          ganon_detail::sync_stream(s) != hipSuccess)) {
      ganon_detail::sync_stream(s);
      return fail(ctx, -1, "ganon_region_decode: copy failed");
    }
    return 0;
  };
  if (p0 > out_total) return raw();
  auto *H = new ganon_bam_dcols();
  RegionReq rq{tid, beg, end, at_eof != 0, 0};
  const int rc = columns(ctx, dout, p0, out_total, H, &rq);
  if (rc || rq.status != 1) {   // (a device failure, too, leaves the window to the host)
    ganon_detail::sync_stream(s);
    release(ctx, H);
    return raw();
  }
  // the columns to one page-locked block, laid out as the device block's first 17 columns and the
  // blob block: two copies by DMA
  const ganon_bam_cols &V = H->v;
  const int64_t m = V.n_records + 1;
  const int64_t prefix = 12 * (((m * 4) + 255) / 256 * 256) + 5 * (((m * 8) + 255) / 256 * 256);
  void *hb = nullptr;
  if (ganon_pinned_alloc(prefix + H->blobs_used + 256, &hb) != 0 || !hb) {
    release(ctx, H);
    return raw();
  }
  uint8_t *h8 = static_cast<uint8_t *>(hb);
  if (hipMemcpyAsync(h8, H->block, (size_t)prefix, hipMemcpyDeviceToHost, s) != hipSuccess ||
      (H->blobs_used > 0 &&
       hipMemcpyAsync(h8 + prefix, H->blobs, (size_t)H->blobs_used, hipMemcpyDeviceToHost, s) != hipSuccess) ||
      ganon_detail::sync_stream(s) != hipSuccess) {
    ganon_detail::sync_stream(s);
    release(ctx, H);
    ganon_pinned_free(hb);
    return raw();
  }
  ganon_bam_cols hv{};
  uint8_t *at = h8;
  for (int32_t **f : {&hv.tid, &hv.pos, &hv.end, &hv.flag, &hv.mapq, &hv.l_seq, &hv.n_cigar, &hv.mate_tid, &hv.mate_pos,
                      &hv.tlen, &hv.name_len, &hv.aux_len})
    *f = carve<int32_t>(at, m);
  for (int64_t **f : {&hv.name_off, &hv.cig_off, &hv.seq_off, &hv.qual_off, &hv.aux_off}) *f = carve<int64_t>(at, m);
  at = h8 + prefix;
  hv.names = carve<char>(at, V.names_bytes);
  hv.cigar = carve<uint32_t>(at, V.cigar_ops);
  hv.seq = carve<uint8_t>(at, V.seq_bytes);
  hv.qual = carve<uint8_t>(at, V.qual_bytes);
  hv.aux = carve<uint8_t>(at, V.aux_bytes);
  *cols = ganon_bam_view{};
  cols->n_records = V.n_records;
  cols->tid = hv.tid, cols->pos = hv.pos, cols->end = hv.end, cols->flag = hv.flag, cols->mapq = hv.mapq;
  cols->l_seq = hv.l_seq, cols->n_cigar = hv.n_cigar, cols->mate_tid = hv.mate_tid, cols->mate_pos = hv.mate_pos;
  cols->tlen = hv.tlen, cols->name_len = hv.name_len, cols->aux_len = hv.aux_len;
  cols->name_off = hv.name_off, cols->cig_off = hv.cig_off, cols->seq_off = hv.seq_off, cols->qual_off = hv.qual_off;
  cols->aux_off = hv.aux_off;
  cols->names = hv.names, cols->names_bytes = V.names_bytes;
  cols->cigar = hv.cigar, cols->cigar_ops = V.cigar_ops;
  cols->seq = hv.seq, cols->seq_bytes = V.seq_bytes;
  cols->qual = hv.qual, cols->qual_bytes = V.qual_bytes;
  cols->aux = hv.aux, cols->aux_bytes = V.aux_bytes;
  release(ctx, H);
  *block = hb;
  return 1;
}
