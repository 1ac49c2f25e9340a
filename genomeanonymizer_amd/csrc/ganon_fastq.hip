// ganon_fastq.hip — MI355X (gfx950) FASTQ record formatter, part of
// libganon_hip.so; C ABI in include/ganon.h (ganon_fastq_*).
//
// Reference: AnonymizedRead.get_anonymized_fastq_record (anonymizer_methods.py:215-243) with
// reverse_complement (:205-213; table `reverses`, :22: A<->T, C<->G, N->N, any other base a
// KeyError — SURVEY Q7) and write_pair's record framing (short_read_tumor_normal_anonymizer.py
// :134-165): '@' name '/' mate '\n' SEQ '\n' '+' '\n' QUAL '\n', qualities printed in the order
// they are stored in the BAM for every read. Same contract as the host formatter
// ganon_fastq_format (include/ganon_host.h), which the parity tests compare byte for byte.
//
// Design: byte work, HBM-bound. A run is four launches:
//   k_fq_bsum   record-length sums per block of 2048 records
//   k_fq_bscan  one workgroup: exclusive scan of the block sums (also resets the error slot)
//   k_fq_off    record output offsets (u64) + for every 8 KiB output tile the record that
//               holds its first byte
//   k_fq_span   (default) one workgroup per 8 KiB output tile, assembled in LDS and stored
//               with full-line 16-byte stores: per record its three field spans (staged once by
//               the record's thread), a virtual map of 16-byte units filled forward, then every
//               unit's source dwords loaded in one round (3 units per lane), transformed (names
//               as they are, qualities + 33 per byte, bases as nibbles through two v_perm table
//               lookups, reverse complement with a zero-byte test for the Q7 error) and written.
//   k_fq_quad / k_fq_rows / k_fq_format: earlier designs kept as A/B instances
//               (GANON_PARAM_FASTQ_KD); k_fq_dense takes tiles with more than 64 records.
#include "ganon_ctx.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <thread>
#include <vector>

namespace {

using ganon_detail::check_launch;
using ganon_detail::fail;
using ganon_detail::KernelScope;

constexpr int kFqThreads = 256;
constexpr int kFqTile = 8192;                                 // output bytes per workgroup
constexpr int kFqStage = 64;                                  // records per tile of the main kernel (more: k_fq_dense)
constexpr int kFqDenseGrid = 512;                             // workgroups of k_fq_dense
constexpr int kFqScanPer = 8;                                 // records per thread in the offset scan
constexpr int kFqScanBlock = kFqThreads * kFqScanPer;         // 2048 records per scan block
constexpr int kFqScanThreads = 1024;
constexpr int kFqMaxBufs = GANON_FASTQ_MAX_BUFS;

constexpr uint64_t kOff56 = (1ull << 56) - 1;
constexpr uint64_t kOff48 = (1ull << 48) - 1;

// One record, 32 bytes:
//   seq  = nibble offset (56 bits) | seq buffer << 56 (2 bits) | reverse << 58 | qual_rev << 59
//   qual = byte offset (48 bits) | mate byte << 48 | qual buffer << 56 (2 bits)
//   name = byte offset (48 bits) | name length << 48 (16 bits)
struct FqRec {
  uint64_t seq, qual, name;
  uint32_t len, qlen;
};
static_assert(sizeof(FqRec) == 32, "FqRec is two 16-byte words");

struct FqBufs {
  const uint8_t *seq[kFqMaxBufs];
  const uint8_t *qual[kFqMaxBufs];
  const uint8_t *names;
};

// "=ACMGRSVTWYHKDBN" and its reverse complement per reverse_complement (0 = no mapping).
constexpr uint64_t kFwdLo = 0x565352474D43413Dull;   // = A C M G R S V   (codes 0..7)
constexpr uint64_t kFwdHi = 0x4E42444B48595754ull;   // T W Y H K D B N   (codes 8..15)
constexpr uint64_t kRevLo = 0x0000004300475400ull;   // A->T, C->G, G->C  (codes 1, 2, 4)
constexpr uint64_t kRevHi = 0x4E00000000000041ull;   // T->A (8), N->N (15)

__device__ __forceinline__ uint32_t tab16(uint64_t lo, uint64_t hi, uint32_t c) {
  const uint64_t w = c < 8 ? lo : hi;
  return (uint32_t)(w >> (8 * (c & 7))) & 0xFF;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v) {
  const int lane = threadIdx.x & 63;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

__global__ void __launch_bounds__(kFqThreads) k_fq_bsum(const uint32_t *__restrict__ len,
                                                        unsigned long long *__restrict__ bsum) {
  __shared__ unsigned long long s[kFqThreads / 64];
  const uint4 *p = reinterpret_cast<const uint4 *>(len + (int64_t)blockIdx.x * kFqScanBlock) + 2 * threadIdx.x;
  const uint4 a = p[0], b = p[1];
  unsigned long long v = (unsigned long long)a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ void __launch_bounds__(kFqScanThreads) k_fq_bscan(unsigned long long *__restrict__ bsum, int64_t nb,
                                                             unsigned long long *__restrict__ err,
                                                             unsigned int *__restrict__ dense_count) {
  __shared__ unsigned long long s[kFqScanThreads / 64];
  __shared__ unsigned long long s_carry;
  if (threadIdx.x == 0) {
    s_carry = 0;
    *err = ~0ull;
    *dense_count = 0;
  }
  __syncthreads();
  for (int64_t base = 0; base < nb; base += kFqScanThreads) {
    const int64_t i = base + threadIdx.x;
    const unsigned long long v = i < nb ? bsum[i] : 0;
    const unsigned long long w = wave_incl_scan(v);
    if ((threadIdx.x & 63) == 63) s[threadIdx.x >> 6] = w;
    __syncthreads();
    unsigned long long pre = s_carry;
    for (int k = 0; k < (int)(threadIdx.x >> 6); ++k) pre += s[k];
    if (i < nb) bsum[i] = pre + w - v;   // exclusive
    __syncthreads();
    if (threadIdx.x == kFqScanThreads - 1) s_carry = pre + w;
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kFqThreads) k_fq_off(const uint32_t *__restrict__ len,
                                                       const unsigned long long *__restrict__ boff, int64_t n,
                                                       uint64_t *__restrict__ off, int64_t *__restrict__ tile_first) {
  __shared__ unsigned long long s[kFqThreads / 64];
  const int64_t r0 = (int64_t)blockIdx.x * kFqScanBlock + kFqScanPer * threadIdx.x;
  const uint4 *p = reinterpret_cast<const uint4 *>(len + r0);
  const uint4 a = p[0], b = p[1];
  const uint32_t l[kFqScanPer] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  unsigned long long v = 0;
#pragma unroll
  for (int k = 0; k < kFqScanPer; ++k) v += l[k];
  const unsigned long long w = wave_incl_scan(v);
  if ((threadIdx.x & 63) == 63) s[threadIdx.x >> 6] = w;
  __syncthreads();
  unsigned long long o = boff[blockIdx.x] + w - v;
  for (int k = 0; k < (int)(threadIdx.x >> 6); ++k) o += s[k];
#pragma unroll
  for (int k = 0; k < kFqScanPer; ++k) {
    const int64_t r = r0 + k;
    if (r >= n) break;
    const unsigned long long e = o + l[k];
    off[r] = o;
    // tiles whose first byte lies in [o, e)
    for (unsigned long long t = (o + kFqTile - 1) / kFqTile; t * kFqTile < e; ++t) tile_first[t] = r;
    if (r == n - 1) off[n] = e;
    o = e;
  }
}

__device__ __forceinline__ const uint8_t *pick4(const uint8_t *const (&p)[kFqMaxBufs], uint32_t sel) {
  // per-lane choice among kernel-argument pointers without indexing the argument block
  const uint8_t *a = (sel & 1) ? p[1] : p[0];
  const uint8_t *b = (sel & 1) ? p[3] : p[2];
  return (sel & 2) ? b : a;
}

// Per output byte (record offset o of record R): its source and how it is transformed.
// info = constant value | kind << 8 (0 const, 1 raw name byte, 2 nt16 nibble, 3 quality) |
//        low nibble << 10 | reverse << 11
struct FqSrc {
  const uint8_t *addr;
  uint32_t info;
};

__device__ __forceinline__ FqSrc fq_src(const FqRec &R, uint32_t o, const FqBufs &bufs) {
  const uint32_t NL = (uint32_t)(R.name >> 48), L = R.len, Q = R.qlen;
  FqSrc s{bufs.names, 0u};
  if (o == 0) {
    s.info = '@';
    return s;
  }
  o -= 1;
  if (o < NL) {
    s.addr = bufs.names + (R.name & kOff48) + o;
    s.info = 1u << 8;
    return s;
  }
  o -= NL;
  if (o < 3) {
    s.info = o == 0 ? '/' : o == 1 ? (((uint32_t)(R.qual >> 48) & 0xFF) + '0') & 0xFF : '\n';
    return s;
  }
  o -= 3;
  if (o < L) {
    const uint32_t rev = (uint32_t)(R.seq >> 58) & 1;
    const uint64_t nib = (R.seq & kOff56) + (rev ? L - 1 - o : o);
    s.addr = pick4(bufs.seq, (uint32_t)(R.seq >> 56) & 3) + (nib >> 1);
    s.info = (2u << 8) | ((uint32_t)(nib & 1) << 10) | (rev << 11);
    return s;
  }
  o -= L;
  if (o < 3) {
    s.info = o == 1 ? '+' : '\n';
    return s;
  }
  o -= 3;
  if (o < Q) {
    const uint32_t qrev = (uint32_t)(R.seq >> 59) & 1;
    s.addr = pick4(bufs.qual, (uint32_t)(R.qual >> 56) & 3) + (R.qual & kOff48) + (qrev ? Q - 1 - o : o);
    s.info = 3u << 8;
    return s;
  }
  s.info = '\n';
  return s;
}

__device__ __forceinline__ uint32_t fq_val(uint32_t info, uint32_t byte, bool &bad) {
  const uint32_t kind = (info >> 8) & 3;
  if (kind == 1) return byte;
  if (kind == 3) return (byte + 33) & 0xFF;
  if (kind == 2) {
    const uint32_t c = (info >> 10) & 1 ? (byte & 0xF) : (byte >> 4);
    if ((info >> 11) & 1) {
      const uint32_t x = tab16(kRevLo, kRevHi, c);
      bad |= x == 0;
      return x;
    }
    return tab16(kFwdLo, kFwdHi, c);
  }
  return info & 0xFF;
}

// nt16 codes (one per byte of c, 0..15) -> table bytes, two v_perm over the 16-byte table.
__device__ __forceinline__ uint32_t nt16_lut(uint32_t c, uint64_t lo, uint64_t hi) {
  const uint32_t sel = c & 0x07070707u;
  const uint32_t a = __builtin_amdgcn_perm((uint32_t)(lo >> 32), (uint32_t)lo, sel);
  const uint32_t b = __builtin_amdgcn_perm((uint32_t)(hi >> 32), (uint32_t)hi, sel);
  const uint32_t m = ((c >> 3) & 0x01010101u) * 0xFFu;
  return (b & m) | (a & ~m);
}

__device__ __forceinline__ uint32_t add33(uint32_t x) {   // per byte (x + 33) & 0xFF
  return ((x & 0x7F7F7F7Fu) + 0x21212121u) ^ (x & 0x80808080u);
}

// Field f of a record (0 name, 1 bases, 2 qualities) clipped to the tile, in tile bytes:
// [a, b); aligned interior dwords [ia, ib) (empty when ia >= ib: then every byte is an edge).
struct FqField {
  int a, b, ia, ib;
};

// int64 clamps written out: HIP's min/max templates on int64_t compile to f64 conversions here
__device__ __forceinline__ int64_t lo64(int64_t a, int64_t b) { return a < b ? a : b; }
__device__ __forceinline__ int64_t hi64(int64_t a, int64_t b) { return a < b ? b : a; }

__device__ __forceinline__ FqField fq_field(int64_t P0, uint32_t fa, uint32_t len) {
  FqField F;
  const int64_t a = hi64(P0 + fa, 0), b = lo64(P0 + fa + len, kFqTile);
  F.a = (int)lo64(a, kFqTile);
  F.b = (int)hi64(b, (int64_t)F.a);
  F.ia = (F.a + 3) & ~3;
  F.ib = F.b & ~3;
  return F;
}

// Edge byte e (0..5) of a field: tile position, or -1.
__device__ __forceinline__ int fq_edge(const FqField &F, int e) {
  if (F.ia >= F.ib) return F.a + e < F.b ? F.a + e : -1;
  if (e < 3) return F.a + e < F.ia ? F.a + e : -1;
  return F.ib + (e - 3) < F.b ? F.ib + (e - 3) : -1;
}

// One record into the tile image by one wave, in three phases so that a wave can keep the
// loads of several records in flight (k_fq_format batches NB records): prep computes every
// source address, load issues the loads, finish transforms and writes. Every branch is
// wave-uniform except the lane-range guards: name / base / quality interiors as aligned dwords
// (two dword loads, a v_perm or SWAR transform, ds_write_b32), the <= 6 edge bytes of each
// field and the 8 constant bytes on lanes 0..25 (one byte load each, ds_write_b8). Fields
// longer than 256 bytes take several passes (ps); edges and constants go with pass 0.
struct FqWork {
  int64_t r;
  const uint32_t *an, *as, *aq;
  const uint8_t *eaddr;
  int tn, ts, tq, et;
  uint32_t shn, shs, shq, par, flags;   // flags: hn | hs << 1 | hq << 2 | rev << 3 | qrev << 4 | ekind << 5 | elow << 8
  uint32_t econst;
  uint32_t n0, n1, s0w, s1w, q0, q1, ev;
};

__device__ __forceinline__ int fq_passes(const FqRec &R, int64_t P0) {
  const uint32_t NL = (uint32_t)(R.name >> 48), L = R.len, Q = R.qlen;
  const FqField Fn = fq_field(P0, 1, NL), Fs = fq_field(P0, NL + 4, L), Fq = fq_field(P0, NL + 7 + L, Q);
  const int nmax = max(max(Fn.ib - Fn.ia, Fs.ib - Fs.ia), Fq.ib - Fq.ia) >> 2;
  return max(1, (nmax + 63) >> 6);
}

__device__ __forceinline__ void fq_prep(FqWork &w, const FqRec &R, int64_t r, int64_t P0, int ps,
                                        const FqBufs &bufs, int lane) {
  const uint32_t NL = (uint32_t)(R.name >> 48), L = R.len, Q = R.qlen;
  const FqField Fn = fq_field(P0, 1, NL), Fs = fq_field(P0, NL + 4, L), Fq = fq_field(P0, NL + 7 + L, Q);
  const uint8_t *nm = bufs.names + (R.name & kOff48);
  const uint32_t rev = (uint32_t)(R.seq >> 58) & 1, qrev = (uint32_t)(R.seq >> 59) & 1;
  const uint8_t *sb = pick4(bufs.seq, (uint32_t)(R.seq >> 56) & 3);
  const uint64_t s0 = R.seq & kOff56;
  const uint8_t *qb = pick4(bufs.qual, (uint32_t)(R.qual >> 56) & 3) + (R.qual & kOff48);
  const int64_t bn = P0 + 1, bs = P0 + NL + 4, bq = P0 + NL + 7 + L;   // tile position of each field's byte 0
  w.r = r;
  // interiors
  const int d = 64 * ps + lane;
  const uint32_t hn = d < ((Fn.ib - Fn.ia) >> 2), hs = d < ((Fs.ib - Fs.ia) >> 2), hq = d < ((Fq.ib - Fq.ia) >> 2);
  w.tn = Fn.ia + 4 * d;
  w.ts = Fs.ia + 4 * d;
  w.tq = Fq.ia + 4 * d;
  const uint8_t *pn = nm + (uint32_t)(w.tn - bn);
  const uint32_t js = (uint32_t)(w.ts - bs);
  const uint64_t nbs = s0 + (rev ? L - 4 - js : js);
  const uint8_t *psq = sb + (nbs >> 1);
  const uint32_t jq = (uint32_t)(w.tq - bq);
  const uint8_t *pq = qb + (qrev ? Q - 4 - jq : jq);
  w.an = reinterpret_cast<const uint32_t *>((uintptr_t)pn & ~(uintptr_t)3);
  w.as = reinterpret_cast<const uint32_t *>((uintptr_t)psq & ~(uintptr_t)3);
  w.aq = reinterpret_cast<const uint32_t *>((uintptr_t)pq & ~(uintptr_t)3);
  w.shn = (uint32_t)(uintptr_t)pn & 3;
  w.shs = (uint32_t)(uintptr_t)psq & 3;
  w.shq = (uint32_t)(uintptr_t)pq & 3;
  w.par = (uint32_t)(nbs & 1);
  // edge / constant lane: one byte (pass 0 only)
  int et = -1;
  uint32_t ekind = 0, elow = 0;
  w.econst = 0;
  w.eaddr = nm;
  if (ps == 0 && lane < 18) {
    const int f = lane / 6, e = lane - 6 * f;
    const FqField &F = f == 0 ? Fn : f == 1 ? Fs : Fq;
    et = fq_edge(F, e);
    if (et >= 0) {
      const uint32_t j = (uint32_t)(et - (f == 0 ? bn : f == 1 ? bs : bq));
      ekind = f + 1;
      if (f == 0) {
        w.eaddr = nm + j;
      } else if (f == 1) {
        const uint64_t nib = s0 + (rev ? L - 1 - j : j);
        w.eaddr = sb + (nib >> 1);
        elow = (uint32_t)(nib & 1);
      } else {
        w.eaddr = qb + (qrev ? Q - 1 - j : j);
      }
    }
  } else if (ps == 0 && lane < 26) {
    int64_t o;
    switch (lane - 18) {
      case 0: o = 0; w.econst = '@'; break;
      case 1: o = NL + 1; w.econst = '/'; break;
      case 2: o = NL + 2; w.econst = ((uint32_t)(R.qual >> 48) + '0') & 0xFF; break;
      case 3: o = NL + 3; w.econst = '\n'; break;
      case 4: o = NL + 4 + L; w.econst = '\n'; break;
      case 5: o = NL + 5 + L; w.econst = '+'; break;
      case 6: o = NL + 6 + L; w.econst = '\n'; break;
      default: o = NL + 7 + L + Q; w.econst = '\n'; break;
    }
    const int64_t t = P0 + o;
    et = (t >= 0 && t < kFqTile) ? (int)t : -1;
  }
  w.et = et;
  w.flags = hn | (hs << 1) | (hq << 2) | (rev << 3) | (qrev << 4) | (ekind << 5) | (elow << 8);
}

__device__ __forceinline__ void fq_load(FqWork &w) {
  w.n0 = w.n1 = w.s0w = w.s1w = w.q0 = w.q1 = w.ev = 0;
  if (w.flags & 1) { w.n0 = w.an[0]; w.n1 = w.an[1]; }
  if (w.flags & 2) { w.s0w = w.as[0]; w.s1w = w.as[1]; }
  if (w.flags & 4) { w.q0 = w.aq[0]; w.q1 = w.aq[1]; }
  if (w.et >= 0 && (w.flags >> 5) & 3) w.ev = *w.eaddr;
}

__device__ __forceinline__ void fq_finish(const FqWork &w, uint8_t *tile, unsigned long long &bad) {
  uint32_t *tile32 = reinterpret_cast<uint32_t *>(tile);
  const bool rev = (w.flags >> 3) & 1, qrev = (w.flags >> 4) & 1;
  if (w.flags & 1) tile32[w.tn >> 2] = __builtin_amdgcn_alignbyte(w.n1, w.n0, w.shn);
  if (w.flags & 2) {
    const uint32_t x0 = __builtin_amdgcn_alignbyte(w.s1w, w.s0w, w.shs);
    const uint32_t hiN = (x0 >> 4) & 0x0F0F0F0Fu, loN = x0 & 0x0F0F0F0Fu;
    // codes in output order: forward [H0 L0 H1 L1] / [L0 H1 L1 H2], reverse the mirror
    const uint32_t sel = rev ? (w.par ? 0x04010502u : 0x00040105u) : (w.par ? 0x02050104u : 0x05010400u);
    const uint32_t cc = __builtin_amdgcn_perm(loN, hiN, sel);
    const uint32_t x = rev ? nt16_lut(cc, kRevLo, kRevHi) : nt16_lut(cc, kFwdLo, kFwdHi);
    if (rev && ((x - 0x01010101u) & ~x & 0x80808080u)) bad = min(bad, (unsigned long long)w.r);
    tile32[w.ts >> 2] = x;
  }
  if (w.flags & 4) {
    const uint32_t x0 = __builtin_amdgcn_alignbyte(w.q1, w.q0, w.shq);
    tile32[w.tq >> 2] = add33(qrev ? __builtin_bswap32(x0) : x0);
  }
  if (w.et >= 0) {
    const uint32_t ekind = (w.flags >> 5) & 3;
    uint32_t x = w.econst;
    if (ekind == 1) {
      x = w.ev;
    } else if (ekind == 2) {
      const uint32_t c = (w.flags >> 8) & 1 ? (w.ev & 0xF) : (w.ev >> 4);
      x = rev ? tab16(kRevLo, kRevHi, c) : tab16(kFwdLo, kFwdHi, c);
      if (x == 0) bad = min(bad, (unsigned long long)w.r);
    } else if (ekind == 3) {
      x = (w.ev + 33) & 0xFF;
    }
    tile[w.et] = (uint8_t)x;
  }
}

// Tile image of a dense tile (k_fq_dense): built in LDS record by record, one wave per record.
__device__ __forceinline__ void fq_tile_by_records(uint8_t *smem, const FqBufs &bufs, const FqRec *__restrict__ recs,
                                                   const uint64_t *__restrict__ off, int64_t r0, int64_t rl,
                                                   uint64_t t0, unsigned long long &bad) {
  uint8_t *tile = smem;
  FqRec *s_rec = reinterpret_cast<FqRec *>(smem + kFqTile);
  uint64_t *s_off = reinterpret_cast<uint64_t *>(smem + kFqTile + kFqStage * sizeof(FqRec));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t sb = r0; sb <= rl; sb += kFqStage) {
    const int ns = (int)lo64(kFqStage, rl - sb + 1);
    if (sb != r0) __syncthreads();   // the previous batch of staged records is done
    for (int k = threadIdx.x; k < ns; k += kFqThreads) s_rec[k] = recs[sb + k];
    for (int k = threadIdx.x; k <= ns; k += kFqThreads) s_off[k] = off[sb + k];
    __syncthreads();
    for (int k = wave; k < ns; k += kFqThreads / 64) {
      const FqRec R = s_rec[k];
      const int64_t P0 = (int64_t)s_off[k] - (int64_t)t0;
      const int np = fq_passes(R, P0);
      for (int ps = 0; ps < np; ++ps) {
        FqWork w;
        fq_prep(w, R, sb + k, P0, ps, bufs, lane);
        fq_load(w);
        fq_finish(w, tile, bad);
      }
    }
  }
}

// Per-tile field spans (LDS): field f (0 bases, 1 qualities, 2 name) of staged record k is
// span f * kFqStage + k, written once by the record's thread.
struct FqSpan {
  uint64_t src;    // name / qualities: address of field byte 0; bases: 2 * buffer address + first nibble
  int32_t j0;      // field index of byte 0 of the span's first tile dword (-3..)
  uint32_t len;    // field length
  uint16_t td0;    // first tile dword
  uint16_t vs;     // first virtual dword
  uint32_t flags;  // reverse | f << 1
};
static_assert(sizeof(FqSpan) == 24, "FqSpan layout");
constexpr int kFqDw = kFqTile / 4;   // dwords per tile
constexpr int kFqMap = 4096;         // virtual dwords: tile dwords + up to 3 shared edge dwords per record
static_assert(kFqMap >= kFqDw + 3 * kFqStage, "virtual dword map");
constexpr size_t kFqSmemA = kFqTile + kFqStage * sizeof(FqRec) + (kFqStage + 1) * sizeof(uint64_t);
constexpr size_t kFqSmemB = kFqTile + kFqMap * sizeof(uint16_t) + 3 * kFqStage * sizeof(FqSpan);

// Block-wide exclusive scan of a u64 (packed counters), 256 threads; returns the total too.
__device__ __forceinline__ unsigned long long block_excl_scan(unsigned long long v, unsigned long long *s_w,
                                                              unsigned long long &total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  unsigned long long pre = inc - v;
  total = 0;
  for (int k = 0; k < kFqThreads / 64; ++k) {
    if (k < w) pre += s_w[k];
    total += s_w[k];
  }
  return pre;
}

template <int KD>
__global__ void __launch_bounds__(kFqThreads) k_fq_format(const FqBufs bufs, const FqRec *__restrict__ recs,
                                                          const uint64_t *__restrict__ off,
                                                          const int64_t *__restrict__ tile_first, int64_t n,
                                                          uint64_t total, uint8_t *__restrict__ out,
                                                          unsigned long long *__restrict__ err, int skip,
                                                          int *__restrict__ dense_list,
                                                          unsigned int *__restrict__ dense_count) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kFqSmemB];
  __shared__ unsigned long long s_w[kFqThreads / 64];
  const uint64_t t0 = (uint64_t)blockIdx.x * kFqTile;
  const int64_t r0 = tile_first[blockIdx.x];
  const int64_t rl = (t0 + kFqTile < total) ? tile_first[blockIdx.x + 1] : n - 1;   // last record touching the tile
  const int t = threadIdx.x;
  unsigned long long bad = ~0ull;
  uint8_t *tile = smem;
  uint32_t *tile32 = reinterpret_cast<uint32_t *>(smem);
  if (rl - r0 + 1 > kFqStage) {   // left to k_fq_dense
    if (t == 0) dense_list[atomicAdd(dense_count, 1u)] = (int)blockIdx.x;
    return;
  }
  {
    const int ns = (int)(rl - r0 + 1);
    uint16_t *map = reinterpret_cast<uint16_t *>(smem + kFqTile);   // virtual dword -> span
    FqSpan *spans = reinterpret_cast<FqSpan *>(smem + kFqTile + kFqMap * sizeof(uint16_t));
    // 1. zero tile and map; one thread per record: its three field spans (the tile dwords each
    //    field touches — neighbouring fields share edge dwords, OR-ed together) and, once the
    //    tile is zero, its 8 constant bytes
    reinterpret_cast<uint4 *>(tile)[t] = make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4 *>(tile)[t + kFqThreads] = make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4 *>(map)[t] = make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4 *>(map)[t + kFqThreads] = make_uint4(0, 0, 0, 0);
    unsigned long long cnt = 0;   // dwords touched: bases | qualities << 16 | name << 32
    FqSpan sp[3];
    int64_t P0 = 0;
    uint32_t NL = 0, L = 0, Q = 0, mate = 0;
    if (t < ns) {
      const FqRec R = recs[r0 + t];
      P0 = (int64_t)off[r0 + t] - (int64_t)t0;
      NL = (uint32_t)(R.name >> 48);
      L = R.len;
      Q = R.qlen;
      mate = (uint32_t)((R.qual >> 48) & 0xFF);
      const uint32_t fa[3] = {NL + 4, NL + 7 + L, 1u}, len[3] = {L, Q, NL};
      const uint32_t rev[3] = {(uint32_t)(R.seq >> 58) & 1, (uint32_t)(R.seq >> 59) & 1, 0u};
      const uint64_t src[3] = {2 * (uint64_t)(uintptr_t)pick4(bufs.seq, (uint32_t)(R.seq >> 56) & 3) + (R.seq & kOff56),
                               (uint64_t)(uintptr_t)(pick4(bufs.qual, (uint32_t)(R.qual >> 56) & 3) + (R.qual & kOff48)),
                               (uint64_t)(uintptr_t)(bufs.names + (R.name & kOff48))};
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const FqField F = fq_field(P0, fa[f], len[f]);
        const int d0 = F.a >> 2, d1 = (F.b + 3) >> 2;
        sp[f].src = src[f];
        sp[f].j0 = (int)(4 * (int64_t)d0 - (P0 + fa[f]));
        sp[f].len = len[f];
        sp[f].td0 = (uint16_t)d0;
        sp[f].flags = rev[f] | (f << 1);
        cnt |= (unsigned long long)(F.b > F.a ? d1 - d0 : 0) << (16 * f);
      }
    }
    unsigned long long tot;
    const unsigned long long pre = block_excl_scan(cnt, s_w, tot);   // (its barrier: tile and map are zero)
    if (skip & 8) return;
    const int V0 = (int)(tot & 0xFFFF), V1 = V0 + (int)((tot >> 16) & 0xFFFF), V = V1 + (int)((tot >> 32) & 0xFFFF);
    if (t < ns) {
      const int base[3] = {0, V0, V1};
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const int c = (int)((cnt >> (16 * f)) & 0xFFFF);
        const int v = base[f] + (int)((pre >> (16 * f)) & 0xFFFF);
        sp[f].vs = (uint16_t)v;
        spans[f * kFqStage + t] = sp[f];
        if (c > 0) map[v] = (uint16_t)(f * kFqStage + t);
      }
      if (!(skip & 64)) {
        const int64_t o[8] = {0, NL + 1, NL + 2, NL + 3, NL + 4 + L, NL + 5 + L, NL + 6 + L, NL + 7 + L + Q};
        const uint32_t x[8] = {'@', '/', (mate + '0') & 0xFF, '\n', '\n', '+', '\n', '\n'};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int64_t p = P0 + o[e];
          if (p >= 0 && p < kFqTile) atomicOr(&tile32[p >> 2], x[e] << (8 * (p & 3)));
        }
      }
    }
    __syncthreads();
    // 2. fill forward (prefix max over f << 8 | record, increasing along the virtual dwords):
    //    thread t owns map[16t, 16t + 16)
    {
      static_assert(kFqMap == 16 * kFqThreads, "two uint4 of the map per thread");
      uint4 *m4 = reinterpret_cast<uint4 *>(map) + 2 * t;
      const uint4 a = m4[0], b = m4[1];
      uint32_t v[16] = {a.x & 0xFFFF, a.x >> 16, a.y & 0xFFFF, a.y >> 16, a.z & 0xFFFF, a.z >> 16, a.w & 0xFFFF, a.w >> 16,
                        b.x & 0xFFFF, b.x >> 16, b.y & 0xFFFF, b.y >> 16, b.z & 0xFFFF, b.z >> 16, b.w & 0xFFFF, b.w >> 16};
      uint32_t mx = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = max(mx, v[i]);
      uint32_t inc = mx;
      const int lane = t & 63;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o);
        if (lane >= o) inc = max(inc, u);
      }
      __syncthreads();   // s_w reused
      if (lane == 63) s_w[t >> 6] = inc;
      __syncthreads();
      uint32_t pm = __shfl_up(inc, 1);
      if (lane == 0) pm = 0;
      for (int w = 0; w < (t >> 6); ++w) pm = max(pm, (uint32_t)s_w[w]);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        pm = max(pm, v[i]);
        v[i] = pm;
      }
      m4[0] = make_uint4(v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16);
      m4[1] = make_uint4(v[8] | v[9] << 16, v[10] | v[11] << 16, v[12] | v[13] << 16, v[14] | v[15] << 16);
    }
    __syncthreads();
    if (skip & 16) return;
    // 3. field dwords: virtual dwords on consecutive lanes (one field type per wave but at the
    //    two type changes), KD per lane at a time. The 4-byte source window is clamped inside the
    //    field (never before a buffer's start), shifted into place and masked to the field's
    //    bytes; whole dwords are written, edge dwords OR-ed into the zeroed tile.
#pragma unroll 1
    for (int vb = 0; vb < ((skip & 32) ? 0 : V); vb += kFqThreads * KD) {
      uint32_t key[KD], sh[KD], par[KD], v0[KD], v1[KD], flg[KD];
      int td_[KD], dsh[KD];   // dsh: byte shift from the clamped window to the wanted one
      uint32_t msk[KD];
      const uint32_t *a0[KD];
#pragma unroll
      for (int j = 0; j < KD; ++j) {
        const int v = vb + j * kFqThreads + t;
        key[j] = 0xFFFFu;
        a0[j] = reinterpret_cast<const uint32_t *>(bufs.names);
        sh[j] = par[j] = 0;
        td_[j] = 0;
        dsh[j] = 0;
        msk[j] = 0;
        flg[j] = 0;
        if (v >= V) continue;
        const uint32_t kf = map[v];
        key[j] = kf;
        const FqSpan S = spans[kf];
        const int i = v - S.vs;
        td_[j] = S.td0 + i;
        const int j0 = S.j0 + 4 * i;   // field index of the dword's byte 0
        const int len = (int)S.len;
        // bytes i with 0 <= j0 + i < len
        const int lo = max(0, -j0), hi = min(4, len - j0);
        msk[j] = hi > lo ? (0xFFFFFFFFu >> (8 * (4 - (hi - lo)))) << (8 * lo) : 0u;
        const bool rev = S.flags & 1;
        // wanted source window start m (ascending source order), clamped into [0, max(0, len - 4)]
        const int m = rev ? len - 4 - j0 : j0;
        const int c = min(max(m, 0), max(0, len - 4));
        dsh[j] = rev ? c - m : m - c;   // > 0: shift right, < 0: shift left (bytes)
        const uint8_t *src;
        if ((S.flags >> 1) == 0) {
          const uint64_t nb = S.src + (uint64_t)c;
          src = reinterpret_cast<const uint8_t *>(nb >> 1);
          par[j] = (uint32_t)(nb & 1);
        } else {
          src = reinterpret_cast<const uint8_t *>(S.src + (uint64_t)c);
        }
        flg[j] = S.flags;
        sh[j] = (uint32_t)((uintptr_t)src & 3);
        a0[j] = reinterpret_cast<const uint32_t *>((uintptr_t)src & ~(uintptr_t)3);
      }
      if (!(skip & 1)) {
#pragma unroll
        for (int j = 0; j < KD; ++j) {
          v0[j] = __builtin_nontemporal_load(a0[j]);
          v1[j] = __builtin_nontemporal_load(a0[j] + 1);
        }
      } else {
#pragma unroll
        for (int j = 0; j < KD; ++j) v0[j] = v1[j] = 0x11111111u;
      }
#pragma unroll
      for (int j = 0; j < KD; ++j) {
        if (key[j] == 0xFFFFu || msk[j] == 0) continue;
        const int f = flg[j] >> 1, k = key[j] % kFqStage;
        const bool rev = flg[j] & 1;
        const uint32_t w = __builtin_amdgcn_alignbyte(v1[j], v0[j], sh[j]);
        const int ds = dsh[j];
        auto place = [&](uint32_t y) {   // clamped window -> wanted window
          return ds >= 0 ? y >> (8 * ds) : y << (8 * -ds);
        };
        uint32_t x;
        if (f == 0) {
          const uint32_t hiN = (w >> 4) & 0x0F0F0F0Fu, loN = w & 0x0F0F0F0Fu;
          // codes in output order: forward [H0 L0 H1 L1] / [L0 H1 L1 H2], reverse the mirror
          const uint32_t sel = rev ? (par[j] ? 0x04010502u : 0x00040105u) : (par[j] ? 0x02050104u : 0x05010400u);
          const uint32_t cc = place(__builtin_amdgcn_perm(loN, hiN, sel));
          x = rev ? nt16_lut(cc, kRevLo, kRevHi) : nt16_lut(cc, kFwdLo, kFwdHi);
          const uint32_t y = x | ~msk[j];
          if (rev && ((y - 0x01010101u) & ~y & 0x80808080u)) bad = min(bad, (unsigned long long)(r0 + k));
        } else if (f == 1) {
          x = add33(place(rev ? __builtin_bswap32(w) : w));
        } else {
          x = place(w);
        }
        if (msk[j] == 0xFFFFFFFFu) tile32[td_[j]] = x;
        else atomicOr(&tile32[td_[j]], x & msk[j]);
      }
    }
  }
  if (bad != ~0ull && !(skip & 1)) atomicMin(err, bad);
  __syncthreads();
  if (skip & 2) return;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int q = 0; q < kFqTile / (16 * kFqThreads); ++q) {
    const int p = (q * kFqThreads + t) * 16;
    if (t0 + p >= total) break;
    __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(tile + p), reinterpret_cast<u32x4 *>(out + t0 + p));
  }
}

// ---- quad variant (GANON_PARAM_FASTQ_KD 16 / 9 / 10; the default up to round 4) --------------------
// The same tile design with 16-byte units: a virtual unit is one 16-byte-aligned tile quad of one
// field, so the map / span lookup and the address arithmetic are paid once per 16 output bytes
// instead of once per 4 (the dword kernel above is VALU-bound: without loads and stores it still
// takes 2.2 of its 2.6 ms on configs[1]'s 10 M records). Each unit loads the aligned dwords under its
// 16-byte source window (3 for bases: 16 nibbles; 5 for names / qualities), every dword address
// clamped into the field's own aligned extent (bytes outside the field are masked off anyway, so a
// clamped dword never matters and no load leaves the field's allocation), builds the four output
// dwords with the dword kernel's transforms and writes them with one ds_write_b128 when the quad
// lies inside the field, else per dword (whole dwords stored, edge dwords OR-ed). The virtual map is
// 4x smaller, so the fill-forward scan is too.
constexpr int kFqQMap = 1024;        // virtual quads: 512 tile quads + up to 3 shared per record
static_assert(kFqQMap >= kFqTile / 16 + 3 * kFqStage, "virtual quad map");
constexpr size_t kFqSmemQ = kFqTile + kFqQMap * sizeof(uint16_t) + 3 * kFqStage * sizeof(FqSpan);

__device__ __forceinline__ uint32_t fq_dmask(int jd, int len) {   // bytes of dword jd..jd+3 inside [0, len)
  const int lo = max(0, -jd), hi = min(4, len - jd);
  return hi > lo ? (0xFFFFFFFFu >> (8 * (4 - (hi - lo)))) << (8 * lo) : 0u;
}

__device__ __forceinline__ const uint32_t *fq_clamp(uintptr_t a, uintptr_t lo, uintptr_t hi) {
  return reinterpret_cast<const uint32_t *>(a < lo ? lo : a > hi ? hi : a);
}

typedef __attribute__((address_space(1))) const uint32_t GU32;

template <int KQ, bool ALIGN5 = true>
__global__ void __launch_bounds__(kFqThreads) k_fq_quad(const FqBufs bufs, const FqRec *__restrict__ recs,
                                                        const uint64_t *__restrict__ off,
                                                        const int64_t *__restrict__ tile_first, int64_t n,
                                                        uint64_t total, uint8_t *__restrict__ out,
                                                        unsigned long long *__restrict__ err, int skip,
                                                        int *__restrict__ dense_list,
                                                        unsigned int *__restrict__ dense_count) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kFqSmemQ];
  __shared__ unsigned long long s_w[kFqThreads / 64];
  const uint64_t t0 = (uint64_t)blockIdx.x * kFqTile;
  const int64_t r0 = tile_first[blockIdx.x];
  const int64_t rl = (t0 + kFqTile < total) ? tile_first[blockIdx.x + 1] : n - 1;
  const int t = threadIdx.x;
  unsigned long long bad = ~0ull;
  uint8_t *tile = smem;
  uint32_t *tile32 = reinterpret_cast<uint32_t *>(smem);
  if (rl - r0 + 1 > kFqStage) {   // left to k_fq_dense
    if (t == 0) dense_list[atomicAdd(dense_count, 1u)] = (int)blockIdx.x;
    return;
  }
  const int ns = (int)(rl - r0 + 1);
  uint16_t *map = reinterpret_cast<uint16_t *>(smem + kFqTile);
  FqSpan *spans = reinterpret_cast<FqSpan *>(smem + kFqTile + kFqQMap * sizeof(uint16_t));
  // 1. zero tile and map; one thread per record: its three field spans in tile quads
  reinterpret_cast<uint4 *>(tile)[t] = make_uint4(0, 0, 0, 0);
  reinterpret_cast<uint4 *>(tile)[t + kFqThreads] = make_uint4(0, 0, 0, 0);
  static_assert(kFqQMap * sizeof(uint16_t) == 8 * kFqThreads, "one uint2 of the map per thread");
  reinterpret_cast<uint2 *>(map)[t] = make_uint2(0, 0);
  unsigned long long cnt = 0;   // quads touched: bases | qualities << 16 | name << 32
  FqSpan sp[3];
  int64_t P0 = 0;
  uint32_t NL = 0, L = 0, Q = 0, mate = 0;
  if (t < ns) {
    const FqRec R = recs[r0 + t];
    P0 = (int64_t)off[r0 + t] - (int64_t)t0;
    NL = (uint32_t)(R.name >> 48);
    L = R.len;
    Q = R.qlen;
    mate = (uint32_t)((R.qual >> 48) & 0xFF);
    const uint32_t fa[3] = {NL + 4, NL + 7 + L, 1u}, len[3] = {L, Q, NL};
    const uint32_t rev[3] = {(uint32_t)(R.seq >> 58) & 1, (uint32_t)(R.seq >> 59) & 1, 0u};
    const uint64_t src[3] = {2 * (uint64_t)(uintptr_t)pick4(bufs.seq, (uint32_t)(R.seq >> 56) & 3) + (R.seq & kOff56),
                             (uint64_t)(uintptr_t)(pick4(bufs.qual, (uint32_t)(R.qual >> 56) & 3) + (R.qual & kOff48)),
                             (uint64_t)(uintptr_t)(bufs.names + (R.name & kOff48))};
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const FqField F = fq_field(P0, fa[f], len[f]);
      const int q0 = F.a >> 4, q1 = (F.b + 15) >> 4;
      sp[f].src = src[f];
      sp[f].j0 = (int)(16 * (int64_t)q0 - (P0 + fa[f]));
      sp[f].len = len[f];
      sp[f].td0 = (uint16_t)q0;
      sp[f].flags = rev[f] | (f << 1);
      cnt |= (unsigned long long)(F.b > F.a ? q1 - q0 : 0) << (16 * f);
    }
  }
  unsigned long long tot;
  const unsigned long long pre = block_excl_scan(cnt, s_w, tot);   // (its barrier: tile and map are zero)
  if (skip & 8) return;
  const int V0 = (int)(tot & 0xFFFF), V1 = V0 + (int)((tot >> 16) & 0xFFFF), V = V1 + (int)((tot >> 32) & 0xFFFF);
  if (t < ns) {
    const int base[3] = {0, V0, V1};
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const int c = (int)((cnt >> (16 * f)) & 0xFFFF);
      const int v = base[f] + (int)((pre >> (16 * f)) & 0xFFFF);
      sp[f].vs = (uint16_t)v;
      spans[f * kFqStage + t] = sp[f];
      if (c > 0) map[v] = (uint16_t)(f * kFqStage + t);
    }
    const int64_t o[8] = {0, NL + 1, NL + 2, NL + 3, NL + 4 + L, NL + 5 + L, NL + 6 + L, NL + 7 + L + Q};
    const uint32_t x[8] = {'@', '/', (mate + '0') & 0xFF, '\n', '\n', '+', '\n', '\n'};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t p = P0 + o[e];
      if (p >= 0 && p < kFqTile) atomicOr(&tile32[p >> 2], x[e] << (8 * (p & 3)));
    }
  }
  __syncthreads();
  // 2. fill forward (prefix max over the virtual quads): thread t owns map[4t, 4t + 4)
  {
    uint2 *m2 = reinterpret_cast<uint2 *>(map) + t;
    const uint2 a = *m2;
    uint32_t v[4] = {a.x & 0xFFFF, a.x >> 16, a.y & 0xFFFF, a.y >> 16};
    const uint32_t mx = max(max(v[0], v[1]), max(v[2], v[3]));
    uint32_t inc = mx;
    const int lane = t & 63;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o);
      if (lane >= o) inc = max(inc, u);
    }
    __syncthreads();   // s_w reused
    if (lane == 63) s_w[t >> 6] = inc;
    __syncthreads();
    uint32_t pm = __shfl_up(inc, 1);
    if (lane == 0) pm = 0;
    for (int w = 0; w < (t >> 6); ++w) pm = max(pm, (uint32_t)s_w[w]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pm = max(pm, v[i]);
      v[i] = pm;
    }
    *m2 = make_uint2(v[0] | v[1] << 16, v[2] | v[3] << 16);
  }
  __syncthreads();
  if (skip & 16) return;
  // 3. units: KQ virtual quads per lane at a time
#pragma unroll 1
  for (int vb = 0; vb < ((skip & 32) ? 0 : V); vb += kFqThreads * KQ) {
    uint32_t key[KQ], dw[KQ][5], sh[KQ], par[KQ], flg[KQ];
    int tq[KQ], J[KQ], len[KQ];
    const GU32 *ad[KQ][5];   // global address space: global_load, not flat (no LDS wait coupling)
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
      const int v = vb + j * kFqThreads + t;
      key[j] = 0xFFFFu;
      sh[j] = par[j] = flg[j] = 0;
      tq[j] = J[j] = len[j] = 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) ad[j][k] = reinterpret_cast<const GU32 *>((uintptr_t)bufs.names);
      if (v >= V) continue;
      const uint32_t kf = map[v];
      key[j] = kf;
      const FqSpan S = spans[kf];
      const int i = v - S.vs;
      tq[j] = S.td0 + i;
      J[j] = S.j0 + 16 * i;
      len[j] = (int)S.len;
      flg[j] = S.flags;
      const int rel = (S.flags & 1) ? len[j] - 16 - J[j] : J[j];   // window start in field units
      // 32-bit offsets from the field's aligned base A0: the window's aligned dwords, each clamped
      // into the field's aligned extent [0, hi]
      int start, hi;
      uint64_t A0;
      if ((S.flags >> 1) == 0) {   // bases: nibble units (S.src = 2 * byte address + first nibble)
        const int n_off = (int)(S.src & 7) + rel;
        par[j] = (uint32_t)(n_off & 1);
        start = n_off >> 1;
        hi = (((int)(S.src & 7) + len[j] - 1) >> 1) & ~3;
        A0 = (S.src >> 1) & ~(uint64_t)3;
      } else {
        start = (int)(S.src & 3) + rel;
        hi = ((int)(S.src & 3) + len[j] - 1) & ~3;
        A0 = S.src & ~(uint64_t)3;
      }
      sh[j] = (uint32_t)(start & 3);
      const int a = start - (start & 3);
#pragma unroll
      for (int k = 0; k < 5; ++k)
        ad[j][k] = reinterpret_cast<const GU32 *>(A0 + (uint64_t)(uint32_t)min(max(a + 4 * k, 0), hi));
    }
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
      if (skip & 1) {
        dw[j][0] = dw[j][1] = dw[j][2] = dw[j][3] = dw[j][4] = 0x11111111u;
        continue;
      }
      dw[j][0] = __builtin_nontemporal_load(ad[j][0]);
      dw[j][1] = __builtin_nontemporal_load(ad[j][1]);
      dw[j][2] = __builtin_nontemporal_load(ad[j][2]);
      if ((flg[j] >> 1) != 0) {
        dw[j][3] = __builtin_nontemporal_load(ad[j][3]);
        dw[j][4] = __builtin_nontemporal_load(ad[j][4]);
      } else {
        dw[j][3] = dw[j][4] = 0;
      }
    }
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
      if (key[j] == 0xFFFFu) continue;
      const int f = flg[j] >> 1, k = key[j] % kFqStage;
      const bool rev = flg[j] & 1;
      uint32_t x[4], m[4];
      const bool full = J[j] >= 0 && J[j] + 16 <= len[j];
#pragma unroll
      for (int d = 0; d < 4; ++d) m[d] = full ? 0xFFFFFFFFu : fq_dmask(J[j] + 4 * d, len[j]);
      if (f == 0) {
        const uint32_t sel = rev ? (par[j] ? 0x04010502u : 0x00040105u) : (par[j] ? 0x02050104u : 0x05010400u);
        const uint64_t tlo = rev ? kRevLo : kFwdLo, thi = rev ? kRevHi : kFwdHi;
        // window bytes [sh + 2d, sh + 2d + 4) for d = 0..3 (reversed: sh + 6 - 2d) from five byte
        // alignments instead of a 3-way dword select per output dword
        const uint32_t w0 = __builtin_amdgcn_alignbyte(dw[j][1], dw[j][0], sh[j]);
        const uint32_t w1 = __builtin_amdgcn_alignbyte(dw[j][2], dw[j][1], sh[j]);
        const uint32_t w2 = __builtin_amdgcn_alignbyte(dw[j][3], dw[j][2], sh[j]);
        const uint32_t h0 = __builtin_amdgcn_alignbyte(w1, w0, 2), h1 = __builtin_amdgcn_alignbyte(w2, w1, 2);
        const uint32_t win[4] = {rev ? h1 : w0, rev ? w1 : h0, rev ? h0 : w1, rev ? w0 : h1};
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          uint32_t w = win[d];
          if constexpr (!ALIGN5) {   // round-1 select per output dword (A/B: GANON_PARAM_FASTQ_KD 11)
            const uint32_t o = sh[j] + (rev ? 6 - 2 * d : 2 * d);
            const uint32_t kk = o >> 2;
            const uint32_t lo_w = kk == 0 ? dw[j][0] : kk == 1 ? dw[j][1] : dw[j][2];
            const uint32_t hi_w = kk == 0 ? dw[j][1] : kk == 1 ? dw[j][2] : dw[j][3];
            w = __builtin_amdgcn_alignbyte(hi_w, lo_w, o & 3);
          }
          const uint32_t hiN = (w >> 4) & 0x0F0F0F0Fu, loN = w & 0x0F0F0F0Fu;
          const uint32_t cc = __builtin_amdgcn_perm(loN, hiN, sel);
          x[d] = nt16_lut(cc, tlo, thi);
          const uint32_t y = x[d] | ~m[d];
          if (rev && ((y - 0x01010101u) & ~y & 0x80808080u)) bad = min(bad, (unsigned long long)(r0 + k));
        }
      } else {
        uint32_t we[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) we[e] = __builtin_amdgcn_alignbyte(dw[j][e + 1], dw[j][e], sh[j]);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t y = rev ? __builtin_bswap32(we[3 - d]) : we[d];
          x[d] = f == 1 ? add33(y) : y;
        }
      }
      if (full) {
        reinterpret_cast<uint4 *>(tile)[tq[j]] = make_uint4(x[0], x[1], x[2], x[3]);
      } else {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (m[d] == 0xFFFFFFFFu) tile32[4 * tq[j] + d] = x[d];
          else if (m[d]) atomicOr(&tile32[4 * tq[j] + d], x[d] & m[d]);
        }
      }
    }
  }
  if (bad != ~0ull) atomicMin(err, bad);
  __syncthreads();
  if (skip & 2) return;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int q = 0; q < kFqTile / (16 * kFqThreads); ++q) {
    const int p = (q * kFqThreads + t) * 16;
    if (t0 + p >= total) break;
    __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(tile + p), reinterpret_cast<u32x4 *>(out + t0 + p));
  }
}

// ---- span variant (GANON_PARAM_FASTQ_KD 0, the default / 13 / 14) ------------------------------
// The quad kernel's units with their per-unit setup moved into the descriptor phase. Within one
// field span every unit's source window moves by a fixed step (16 bytes, 8 for the nt16 bases,
// negative on reversed fields), so the byte shift, the nibble parity and the aligned window start
// of unit 0 are computed once per span by the record's thread; a unit adds i * step and clamps its
// five dword offsets with one v_med3 each. Partial units (a field's first and last) build their byte
// masks from two thresholds; the reverse-complement error test is folded over the unit's four
// dwords; the nt16 table blend takes its byte mask from v_perm's constant selectors. The kernel is
// latency-bound (eight 4-wave workgroups per CU, each a chain of dependent rounds: tile_first ->
// records -> spans -> source loads -> tile stores), so a unit's loads are issued as soon as its
// addresses exist and, with LEAN, only the loaded dwords stay live across the wait (the span fields
// are re-read from LDS after it): 3 units per lane fit 64 VGPRs and cover a c2 tile's ~600 units in
// one load round. TM base tiles (8 KiB each) per workgroup (TM = 2 measured slower:
// fewer resident workgroups); a workgroup with more than 64 * TM records lists its base tiles for
// k_fq_dense.
struct FqSpanS {
  uint64_t base;   // 4-byte-aligned address of the field's first source byte (bases: of its first nibble)
  int32_t a0;      // offset (from base) of unit 0's first aligned source dword
  int32_t hi;      // offset of the field's last aligned source dword
  int32_t j0;      // field index of unit 0's first byte (-15..0, or the bytes before the tile)
  int32_t len;     // field length
  uint16_t td0;    // first tile quad
  uint16_t vs;     // first virtual quad
  uint32_t info;   // byte shift | parity << 2 | reverse << 3 | field << 4 (0 bases, 1 qualities, 2 name) |
                   // window step per unit (int8) << 8
};
static_assert(sizeof(FqSpanS) == 32, "FqSpanS layout");

template <int TM>
struct FqSpanCfg {
  static constexpr int kTile = TM * kFqTile;
  static constexpr int kStage = TM * kFqStage;
  static constexpr int kMap = TM * kFqQMap;
  static constexpr size_t kSmem = kTile + kMap * sizeof(uint16_t) + 3 * kStage * sizeof(FqSpanS);
  static_assert(kMap >= kTile / 16 + 3 * kStage, "virtual quad map");
  static_assert(kMap * sizeof(uint16_t) == 8 * TM * kFqThreads, "TM uint2 of the map per thread");
};

__device__ __forceinline__ int med3i(int x, int lo, int hi) { return min(max(x, lo), hi); }   // v_med3_i32

// bytes [4d, 4d + 4) of a unit, as a dword mask, that lie in [lo, hi) (unit byte positions)
__device__ __forceinline__ uint32_t fq_rmask(int lo, int hi, int d) {
  const uint32_t ge = (uint32_t)(~0ull << med3i(8 * (lo - 4 * d), 0, 32));
  const uint32_t lt = ~(uint32_t)(~0ull << med3i(8 * (hi - 4 * d), 0, 32));
  return ge & lt;
}

// nt16 codes (one per byte, 0..15) -> table bytes; the bit-3 blend mask from v_perm selectors
// 0x0C (byte 0x00) / 0x0D (byte 0xFF)
__device__ __forceinline__ uint32_t nt16_lut2(uint32_t c, uint64_t lo, uint64_t hi) {
  const uint32_t sel = c & 0x07070707u;
  const uint32_t a = __builtin_amdgcn_perm((uint32_t)(lo >> 32), (uint32_t)lo, sel);
  const uint32_t b = __builtin_amdgcn_perm((uint32_t)(hi >> 32), (uint32_t)hi, sel);
  const uint32_t m = __builtin_amdgcn_perm(0u, 0u, ((c >> 3) & 0x01010101u) | 0x0C0C0C0Cu);
  return (b & m) | (a & ~m);
}

template <int KQ, int TM, bool LEAN = false, int MAP = 0>   // MAP: 0 filled map, 1 binary search, 2 coarse map
__global__ void __launch_bounds__(kFqThreads, TM == 1 ? 8 : 4) k_fq_span(const FqBufs bufs, const FqRec *__restrict__ recs,
                                                        const uint64_t *__restrict__ off,
                                                        const int64_t *__restrict__ tile_first, int64_t n,
                                                        uint64_t total, uint8_t *__restrict__ out,
                                                        unsigned long long *__restrict__ err, int skip,
                                                        int *__restrict__ dense_list,
                                                        unsigned int *__restrict__ dense_count,
                                                        int64_t n_tiles) {
  using C = FqSpanCfg<TM>;
  constexpr int TT = C::kTile;
  __shared__ __attribute__((aligned(16))) uint8_t smem[C::kSmem];
  __shared__ unsigned long long s_w[kFqThreads / 64];
  __shared__ uint32_t s_m[kFqThreads / 64];   // fill-forward wave maxima (s_w is still being read)
  const int64_t tb = (int64_t)blockIdx.x * TM;   // first base tile
  const uint64_t t0 = (uint64_t)tb * kFqTile;
  const int64_t r0 = tile_first[tb];
  const int64_t rl = (t0 + TT < total) ? tile_first[tb + TM] : n - 1;
  const int t = threadIdx.x;
  unsigned long long bad = ~0ull;
  uint8_t *tile = smem;
  uint32_t *tile32 = reinterpret_cast<uint32_t *>(smem);
  if (rl - r0 + 1 > C::kStage) {   // left to k_fq_dense, base tile by base tile
    if (t < TM && tb + t < n_tiles) dense_list[atomicAdd(dense_count, 1u)] = (int)(tb + t);
    return;
  }
  const int ns = (int)(rl - r0 + 1);
  uint16_t *map = reinterpret_cast<uint16_t *>(smem + TT);
  FqSpanS *spans = reinterpret_cast<FqSpanS *>(smem + TT + C::kMap * sizeof(uint16_t));
  // 1. zero tile and map; one thread per record: its three field spans in tile quads
#pragma unroll
  for (int k = 0; k < 2 * TM; ++k) reinterpret_cast<uint4 *>(tile)[t + k * kFqThreads] = make_uint4(0, 0, 0, 0);
  if (MAP == 0) {
#pragma unroll
    for (int k = 0; k < TM; ++k) reinterpret_cast<uint2 *>(map)[t + k * kFqThreads] = make_uint2(0, 0);
  }
  unsigned long long cnt = 0;   // quads touched: bases | qualities << 16 | name << 32
  FqSpanS sp[3];
  int64_t P0 = 0;
  uint32_t NL = 0, L = 0, Q = 0, mate = 0;
  if (t < ns) {
    const FqRec R = recs[r0 + t];
    P0 = (int64_t)off[r0 + t] - (int64_t)t0;
    NL = (uint32_t)(R.name >> 48);
    L = R.len;
    Q = R.qlen;
    mate = (uint32_t)((R.qual >> 48) & 0xFF);
    const uint32_t fa[3] = {NL + 4, NL + 7 + L, 1u}, len[3] = {L, Q, NL};
    const uint32_t rev[3] = {(uint32_t)(R.seq >> 58) & 1, (uint32_t)(R.seq >> 59) & 1, 0u};
    const uint64_t src[3] = {2 * (uint64_t)(uintptr_t)pick4(bufs.seq, (uint32_t)(R.seq >> 56) & 3) + (R.seq & kOff56),
                             (uint64_t)(uintptr_t)(pick4(bufs.qual, (uint32_t)(R.qual >> 56) & 3) + (R.qual & kOff48)),
                             (uint64_t)(uintptr_t)(bufs.names + (R.name & kOff48))};
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const int64_t fs = P0 + fa[f];
      const int a = (int)lo64(hi64(fs, 0), TT), b = (int)hi64(lo64(fs + len[f], TT), (int64_t)a);
      const int q0 = a >> 4, q1 = (b + 15) >> 4;
      const int j0 = (int)(16 * (int64_t)q0 - fs);
      const int L_ = (int)len[f];
      const int rel0 = rev[f] ? L_ - 16 - j0 : j0;   // unit 0's window start in field units
      int start0, hi;
      uint64_t base;
      uint32_t par = 0;
      if (f == 0) {   // nibble units: src = 2 * byte address + first nibble
        const int n_off = (int)(src[0] & 7) + rel0;
        par = (uint32_t)(n_off & 1);
        start0 = n_off >> 1;
        hi = (((int)(src[0] & 7) + L_ - 1) >> 1) & ~3;
        base = (src[0] >> 1) & ~(uint64_t)3;
      } else {
        start0 = (int)(src[f] & 3) + rel0;
        hi = ((int)(src[f] & 3) + L_ - 1) & ~3;
        base = src[f] & ~(uint64_t)3;
      }
      const uint32_t sh = (uint32_t)start0 & 3;
      sp[f].base = base;
      sp[f].a0 = start0 - (int)sh;
      sp[f].hi = hi;
      sp[f].j0 = j0;
      sp[f].len = L_;
      sp[f].td0 = (uint16_t)q0;
      const int step = (f == 0 ? 8 : 16) * (rev[f] ? -1 : 1);   // window move per unit (bytes)
      sp[f].info = sh | (par << 2) | (rev[f] << 3) | ((uint32_t)f << 4) | (((uint32_t)step & 0xFF) << 8);
      cnt |= (unsigned long long)(b > a ? q1 - q0 : 0) << (16 * f);
    }
  }
  unsigned long long tot;
  const unsigned long long pre = block_excl_scan(cnt, s_w, tot);   // (its barrier: tile and map are zero)
  if (skip & 8) return;
  const int V0 = (int)(tot & 0xFFFF), V1 = V0 + (int)((tot >> 16) & 0xFFFF), V = V1 + (int)((tot >> 32) & 0xFFFF);
  if (t < ns) {
    const int base[3] = {0, V0, V1};
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const int c = (int)((cnt >> (16 * f)) & 0xFFFF);
      const int v = base[f] + (int)((pre >> (16 * f)) & 0xFFFF);
      sp[f].vs = (uint16_t)v;
      spans[f * C::kStage + t] = sp[f];
      if (MAP == 0 && c > 0) map[v] = (uint16_t)(f * C::kStage + t);
      if (MAP == 2)   // coarse map: the span holding unit 8b, for the blocks b whose first unit is ours
        for (int b = (v + 7) >> 3; 8 * b < v + c; ++b) map[b] = (uint16_t)(f * C::kStage + t);
    }
    const int64_t o[8] = {0, NL + 1, NL + 2, NL + 3, NL + 4 + L, NL + 5 + L, NL + 6 + L, NL + 7 + L + Q};
    const uint32_t x[8] = {'@', '/', (mate + '0') & 0xFF, '\n', '\n', '+', '\n', '\n'};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t p = P0 + o[e];
      if (p >= 0 && p < TT) atomicOr(&tile32[p >> 2], x[e] << (8 * (p & 3)));
    }
  }
  __syncthreads();
  // 2. fill forward (prefix max over the virtual quads): thread t owns map[4TM t, 4TM t + 4TM).
  //    MAP 1: no map; a unit finds its span by a binary search over the field's span starts.
  //    MAP 2: one entry per 8 units (written per record above); a unit walks forward from it
  if (MAP == 0) {
    uint32_t *mw = reinterpret_cast<uint32_t *>(map) + 2 * TM * t;
    uint32_t v[4 * TM];
#pragma unroll
    for (int k = 0; k < 2 * TM; ++k) {
      const uint32_t w = mw[k];
      v[2 * k] = w & 0xFFFF;
      v[2 * k + 1] = w >> 16;
    }
    uint32_t mx = 0;
#pragma unroll
    for (int i = 0; i < 4 * TM; ++i) mx = max(mx, v[i]);
    uint32_t inc = mx;
    const int lane = t & 63;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o);
      if (lane >= o) inc = max(inc, u);
    }
    if (lane == 63) s_m[t >> 6] = inc;
    __syncthreads();
    uint32_t pm = __shfl_up(inc, 1);
    if (lane == 0) pm = 0;
    for (int w = 0; w < (t >> 6); ++w) pm = max(pm, s_m[w]);
#pragma unroll
    for (int i = 0; i < 4 * TM; ++i) {
      pm = max(pm, v[i]);
      v[i] = pm;
    }
#pragma unroll
    for (int k = 0; k < 2 * TM; ++k) mw[k] = v[2 * k] | v[2 * k + 1] << 16;
    __syncthreads();
  }
  if (skip & 16) return;
  // 3. units: KQ virtual quads per lane at a time
#pragma unroll 1
  for (int vb = 0; vb < ((skip & 32) ? 0 : V); vb += kFqThreads * KQ) {
    uint32_t key[KQ], dw[KQ][5], info[KQ];
    int tq[KQ], J[KQ], len[KQ];
#pragma unroll
    for (int j = 0; j < KQ; ++j) {   // each unit's loads issued as soon as its addresses exist
      const int v = vb + j * kFqThreads + t;
      key[j] = 0xFFFFu;
      info[j] = 0;
      tq[j] = J[j] = len[j] = 0;
      dw[j][0] = dw[j][1] = dw[j][2] = dw[j][3] = dw[j][4] = 0;
      if (v >= V) continue;
      uint32_t kf;
      if (MAP == 2) {   // from the span of unit 8 * (v / 8), forward over the spans starting <= v
        kf = map[v >> 3];
        for (;;) {
          const uint32_t kt = kf % C::kStage;
          const uint32_t nx = (int)kt + 1 < ns ? kf + 1 : (kf - kt) + C::kStage;
          if (nx >= 3u * C::kStage || (int)spans[nx].vs > v) break;
          kf = nx;
        }
      } else if (MAP == 1) {   // the last record of the unit's field whose span starts at or before v
        const int f = v < V0 ? 0 : v < V1 ? 1 : 2;
        const FqSpanS *fs = spans + f * C::kStage;
        int k = 0;
#pragma unroll
        for (int st = C::kStage / 2; st > 0; st >>= 1) {
          const int c = k + st;
          if (c < ns && (int)fs[c].vs <= v) k = c;
        }
        kf = (uint32_t)(f * C::kStage + k);
      } else {
        kf = map[v];
      }
      key[j] = kf;
      const FqSpanS S = spans[kf];
      const int i = v - S.vs;
      tq[j] = S.td0 + i;
      J[j] = S.j0 + 16 * i;
      len[j] = S.len;
      info[j] = S.info;
      const int a = S.a0 + __mul24(((int)(S.info << 16)) >> 24, i);   // + i * step
      const int nd = ((S.info >> 4) & 3) != 0 ? 5 : 3;
      if (skip & 1) {
        dw[j][0] = dw[j][1] = dw[j][2] = dw[j][3] = dw[j][4] = 0x11111111u;
        continue;
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        if (k >= nd) break;
        int o;
        asm("v_med3_i32 %0, %1, 0, %2" : "=v"(o) : "v"(a + 4 * k), "v"(S.hi));
        dw[j][k] = __builtin_nontemporal_load(reinterpret_cast<const GU32 *>(S.base + (uint64_t)(uint32_t)o));
      }
    }
    if (LEAN) {   // only the loaded dwords live across the load wait: the unit's span fields again
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < KQ; ++j) {
        const int v = vb + j * kFqThreads + t;
        if (v >= V) continue;
        const FqSpanS &S = spans[key[j]];
        const int i = v - S.vs;
        tq[j] = S.td0 + i;
        J[j] = S.j0 + 16 * i;
        len[j] = S.len;
        info[j] = S.info;
      }
    }
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
      if (key[j] == 0xFFFFu) continue;
      const int f = (info[j] >> 4) & 3, k = key[j] % C::kStage;
      const uint32_t sh = info[j] & 3, par = (info[j] >> 2) & 1;
      const bool rev = (info[j] >> 3) & 1;
      const bool full = J[j] >= 0 && J[j] + 16 <= len[j];
      uint32_t x[4];
      if (f == 0) {
        const uint32_t sel = rev ? (par ? 0x04010502u : 0x00040105u) : (par ? 0x02050104u : 0x05010400u);
        const uint64_t tlo = rev ? kRevLo : kFwdLo, thi = rev ? kRevHi : kFwdHi;
        const uint32_t w0 = __builtin_amdgcn_alignbyte(dw[j][1], dw[j][0], sh);
        const uint32_t w1 = __builtin_amdgcn_alignbyte(dw[j][2], dw[j][1], sh);
        const uint32_t w2 = __builtin_amdgcn_alignbyte(dw[j][3], dw[j][2], sh);
        const uint32_t h0 = __builtin_amdgcn_alignbyte(w1, w0, 2), h1 = __builtin_amdgcn_alignbyte(w2, w1, 2);
        const uint32_t win[4] = {rev ? h1 : w0, rev ? w1 : h0, rev ? h0 : w1, rev ? w0 : h1};
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t w = win[d];
          const uint32_t hiN = (w >> 4) & 0x0F0F0F0Fu, loN = w & 0x0F0F0F0Fu;
          x[d] = nt16_lut2(__builtin_amdgcn_perm(loN, hiN, sel), tlo, thi);
        }
        if (rev) {   // a zero byte (no complement) inside the field: the reference's KeyError (Q7)
          uint32_t z = 0;
          const int lo = -J[j], hb = len[j] - J[j];
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const uint32_t y = full ? x[d] : x[d] | ~fq_rmask(lo, hb, d);
            z |= (y - 0x01010101u) & ~y & 0x80808080u;
          }
          if (z) bad = min(bad, (unsigned long long)(r0 + k));
        }
      } else {
        uint32_t we[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) we[e] = __builtin_amdgcn_alignbyte(dw[j][e + 1], dw[j][e], sh);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t y = rev ? __builtin_bswap32(we[3 - d]) : we[d];
          x[d] = f == 1 ? add33(y) : y;
        }
      }
      if (full) {
        reinterpret_cast<uint4 *>(tile)[tq[j]] = make_uint4(x[0], x[1], x[2], x[3]);
      } else {
        const int lo = -J[j], hb = len[j] - J[j];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t m = fq_rmask(lo, hb, d);
          if (m == 0xFFFFFFFFu) tile32[4 * tq[j] + d] = x[d];
          else if (m) atomicOr(&tile32[4 * tq[j] + d], x[d] & m);
        }
      }
    }
  }
  if (bad != ~0ull) atomicMin(err, bad);
  __syncthreads();
  if (skip & 2) return;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int q = 0; q < TT / (16 * kFqThreads); ++q) {
    const int p = (q * kFqThreads + t) * 16;
    if (t0 + p >= total) break;
    __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(tile + p), reinterpret_cast<u32x4 *>(out + t0 + p));
  }
}

// ---- row variant (GANON_PARAM_FASTQ_KD 12) -----------------------------------------------------
// No virtual map: one thread per record stages its three field extents (tile offset, source,
// length) and its constant bytes; then each field is formatted in one flat pass over (record,
// 8-byte unit) pairs — a record's units are G consecutive lanes, G the tile's widest extent of that
// field rounded up to a power of two (20 of 32 lanes carry a 150-byte field, 5-7 of 8 a read
// name). A unit is two tile dwords: three aligned source dwords (clamped into the field's own
// aligned extent: bytes outside the field are masked off anyway), two v_alignbyte, the transform
// (+33 per byte for qualities, two v_perm nibble selects and the 16-entry table for bases, byte
// reversal for reversed fields) and two LDS stores — plain for dwords inside the field, masked OR
// for the dwords it shares with a neighbour or a constant. Per unit that is ~1/3 of the quad
// variant's address and map work.
struct FqRow {
  uint64_t src[3];   // bases: 2 * byte address + first nibble; qualities / name: address of byte 0
  int32_t fo[3];     // tile offset of the field's first byte (< 0: it starts in an earlier tile)
  uint32_t len[3];
  uint32_t rev;      // bit 0 bases reversed, bit 1 qualities reversed
  uint32_t pad;
};
static_assert(sizeof(FqRow) == 56, "FqRow layout");

__device__ __forceinline__ uint32_t fq_bmask(int j, int len) {   // bytes j..j+3 of a field inside [0, len)
  const int lo = max(0, -j), hi = min(4, len - j);
  return hi > lo ? (0xFFFFFFFFu >> (8 * (4 - (hi - lo)))) << (8 * lo) : 0u;
}

// Field f (0 bases, 1 qualities, 2 name) of every staged record: units u of record k.
template <int F>
__device__ __forceinline__ void fq_rows_field(const FqRow *rows, int ns, int lg, uint32_t *tile32, int64_t r0,
                                              unsigned long long &bad) {
  const int G = 1 << lg;
  for (int vl = threadIdx.x; vl < (ns << lg); vl += kFqThreads) {
    const int k = vl >> lg, u = vl & (G - 1);
    const int fo = rows[k].fo[F];
    const int len = (int)rows[k].len[F];
    const int T = ((fo >> 3) + u) * 8;           // tile byte of the unit (8-aligned)
    if (T < 0 || T >= kFqTile || T >= fo + len || len == 0) continue;
    const int i0 = T - fo;                       // field byte of the unit's first byte (>= -7)
    const bool rev = F == 0 ? (rows[k].rev & 1) : F == 1 ? ((rows[k].rev >> 1) & 1) : false;
    const uint64_t src = rows[k].src[F];
    uint32_t x0, x1;
    if (F == 0) {
      // nibbles of the 8 bases, ascending: [n_lo, n_lo + 8)
      const int64_t nlo = (int64_t)src + (rev ? (int64_t)(len - 8 - i0) : (int64_t)i0);
      const uint64_t fb0 = src >> 1, fb1 = ((uint64_t)src + len - 1) >> 1;   // the field's bytes
      const uint64_t A0 = fb0 & ~(uint64_t)3;
      const int hi = (int)((fb1 - A0) >> 2);
      const int64_t B = nlo >> 1;                                            // first byte (may precede the field)
      const int64_t rel = B - (int64_t)A0;                                   // >= -4
      const int di = (int)((rel + 8) >> 2) - 2, sh = (int)((rel + 8) & 3);
      const GU32 *base = reinterpret_cast<const GU32 *>(A0);
      const uint32_t d0 = __builtin_nontemporal_load(base + min(max(di, 0), hi));
      const uint32_t d1 = __builtin_nontemporal_load(base + min(max(di + 1, 0), hi));
      const uint32_t d2 = __builtin_nontemporal_load(base + min(max(di + 2, 0), hi));
      const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
      const uint32_t h0 = __builtin_amdgcn_alignbyte(w1, w0, 2);   // bytes B + 2 .. B + 5
      const uint32_t par = (uint32_t)(nlo & 1);
      const uint32_t sel = rev ? (par ? 0x04010502u : 0x00040105u) : (par ? 0x02050104u : 0x05010400u);
      const uint64_t tlo = rev ? kRevLo : kFwdLo, thi = rev ? kRevHi : kFwdHi;
      const uint32_t a = rev ? h0 : w0, b = rev ? w0 : h0;   // reversed: the upper nibbles first
      const uint32_t ca = __builtin_amdgcn_perm(a & 0x0F0F0F0Fu, (a >> 4) & 0x0F0F0F0Fu, sel);
      const uint32_t cb = __builtin_amdgcn_perm(b & 0x0F0F0F0Fu, (b >> 4) & 0x0F0F0F0Fu, sel);
      x0 = nt16_lut(ca, tlo, thi);
      x1 = nt16_lut(cb, tlo, thi);
      if (rev) {
        const uint32_t y0 = x0 | ~fq_bmask(i0, len), y1 = x1 | ~fq_bmask(i0 + 4, len);
        if (((y0 - 0x01010101u) & ~y0 & 0x80808080u) | ((y1 - 0x01010101u) & ~y1 & 0x80808080u))
          bad = min(bad, (unsigned long long)(r0 + k));
      }
    } else {
      // bytes [j_lo, j_lo + 8) of the field, ascending (reversed qualities: read backwards)
      const int jlo = rev ? len - 8 - i0 : i0;
      const uint64_t A0 = src & ~(uint64_t)3;
      const int hi = (int)(((src & 3) + (uint64_t)len - 1) >> 2);
      const int rel = (int)(src & 3) + jlo;                                  // >= -7
      const int di = ((rel + 8) >> 2) - 2, sh = (rel + 8) & 3;
      const GU32 *base = reinterpret_cast<const GU32 *>(A0);
      const uint32_t d0 = __builtin_nontemporal_load(base + min(max(di, 0), hi));
      const uint32_t d1 = __builtin_nontemporal_load(base + min(max(di + 1, 0), hi));
      const uint32_t d2 = __builtin_nontemporal_load(base + min(max(di + 2, 0), hi));
      uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
      if (rev) {
        const uint32_t t = __builtin_bswap32(w1);
        w1 = __builtin_bswap32(w0);
        w0 = t;
      }
      x0 = F == 1 ? add33(w0) : w0;
      x1 = F == 1 ? add33(w1) : w1;
    }
    const uint32_t m0 = fq_bmask(i0, len), m1 = fq_bmask(i0 + 4, len);
    uint32_t *t32 = tile32 + (T >> 2);
    if (m0 == 0xFFFFFFFFu) t32[0] = x0;
    else if (m0) atomicOr(t32, x0 & m0);
    if (m1 == 0xFFFFFFFFu) t32[1] = x1;
    else if (m1) atomicOr(t32 + 1, x1 & m1);
  }
}

__global__ void __launch_bounds__(kFqThreads) k_fq_rows(const FqBufs bufs, const FqRec *__restrict__ recs,
                                                        const uint64_t *__restrict__ off,
                                                        const int64_t *__restrict__ tile_first, int64_t n,
                                                        uint64_t total, uint8_t *__restrict__ out,
                                                        unsigned long long *__restrict__ err, int skip,
                                                        int *__restrict__ dense_list,
                                                        unsigned int *__restrict__ dense_count) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kFqTile];
  __shared__ FqRow rows[kFqStage];
  __shared__ int s_lg[3];
  const uint64_t t0 = (uint64_t)blockIdx.x * kFqTile;
  const int64_t r0 = tile_first[blockIdx.x];
  const int64_t rl = (t0 + kFqTile < total) ? tile_first[blockIdx.x + 1] : n - 1;
  const int t = threadIdx.x;
  uint32_t *tile32 = reinterpret_cast<uint32_t *>(tile);
  if (rl - r0 + 1 > kFqStage) {   // left to k_fq_dense
    if (t == 0) dense_list[atomicAdd(dense_count, 1u)] = (int)blockIdx.x;
    return;
  }
  const int ns = (int)(rl - r0 + 1);
  // 1. zero the tile; one thread per record: its row, its constant bytes, the field widths
  reinterpret_cast<uint4 *>(tile)[t] = make_uint4(0, 0, 0, 0);
  reinterpret_cast<uint4 *>(tile)[t + kFqThreads] = make_uint4(0, 0, 0, 0);
  if (t < 3) s_lg[t] = 0;
  __syncthreads();
  if (t < ns) {
    const FqRec R = recs[r0 + t];
    const int64_t P0 = (int64_t)off[r0 + t] - (int64_t)t0;   // > -2^31: a record is < 2^31 bytes
    const uint32_t NL = (uint32_t)(R.name >> 48), L = R.len, Q = R.qlen;
    const uint32_t mate = (uint32_t)((R.qual >> 48) & 0xFF);
    FqRow w;
    w.src[0] = 2 * (uint64_t)(uintptr_t)pick4(bufs.seq, (uint32_t)(R.seq >> 56) & 3) + (R.seq & kOff56);
    w.src[1] = (uint64_t)(uintptr_t)(pick4(bufs.qual, (uint32_t)(R.qual >> 56) & 3) + (R.qual & kOff48));
    w.src[2] = (uint64_t)(uintptr_t)(bufs.names + (R.name & kOff48));
    w.fo[0] = (int32_t)(P0 + NL + 4);
    w.fo[1] = (int32_t)(P0 + NL + 7 + L);
    w.fo[2] = (int32_t)(P0 + 1);
    w.len[0] = L;
    w.len[1] = Q;
    w.len[2] = NL;
    w.rev = (uint32_t)((R.seq >> 58) & 1) | ((uint32_t)((R.seq >> 59) & 1) << 1);
    w.pad = 0;
    rows[t] = w;
#pragma unroll
    for (int f = 0; f < 3; ++f) {   // units (8-byte) the field spans, as a power-of-two exponent
      const int units = w.len[f] ? ((w.fo[f] + (int)w.len[f] + 7) >> 3) - (w.fo[f] >> 3) : 0;
      int lg = 0;
      while ((1 << lg) < units) ++lg;
      atomicMax(&s_lg[f], lg);
    }
    const int64_t o[8] = {0, NL + 1, NL + 2, NL + 3, NL + 4 + L, NL + 5 + L, NL + 6 + L, NL + 7 + L + Q};
    const uint32_t x[8] = {'@', '/', (mate + '0') & 0xFF, '\n', '\n', '+', '\n', '\n'};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t p = P0 + o[e];
      if (p >= 0 && p < kFqTile) atomicOr(&tile32[p >> 2], x[e] << (8 * (p & 3)));
    }
  }
  __syncthreads();
  unsigned long long bad = ~0ull;
  if (!(skip & 32)) {
    fq_rows_field<0>(rows, ns, s_lg[0], tile32, r0, bad);
    fq_rows_field<1>(rows, ns, s_lg[1], tile32, r0, bad);
    fq_rows_field<2>(rows, ns, s_lg[2], tile32, r0, bad);
  }
  if (bad != ~0ull) atomicMin(err, bad);
  __syncthreads();
  if (skip & 2) return;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int q = 0; q < kFqTile / (16 * kFqThreads); ++q) {
    const int p = (q * kFqThreads + t) * 16;
    if (t0 + p >= total) break;
    __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(tile + p), reinterpret_cast<u32x4 *>(out + t0 + p));
  }
}

// Tiles touched by more than kFqStage records (records of a few dozen bytes), listed by
// k_fq_format: built in LDS record by record (one wave per record), a fixed grid looping over
// the list.
__global__ void __launch_bounds__(kFqThreads) k_fq_dense(const FqBufs bufs, const FqRec *__restrict__ recs,
                                                         const uint64_t *__restrict__ off,
                                                         const int64_t *__restrict__ tile_first, int64_t n,
                                                         uint64_t total, uint8_t *__restrict__ out,
                                                         unsigned long long *__restrict__ err,
                                                         const int *__restrict__ dense_list,
                                                         const unsigned int *__restrict__ dense_count) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kFqSmemA];
  const unsigned int cnt = *dense_count;
  unsigned long long bad = ~0ull;
  for (unsigned int i = blockIdx.x; i < cnt; i += gridDim.x) {
    const int tl = dense_list[i];
    const uint64_t t0 = (uint64_t)tl * kFqTile;
    const int64_t r0 = tile_first[tl];
    const int64_t rl = (t0 + kFqTile < total) ? tile_first[tl + 1] : n - 1;
    __syncthreads();   // the previous tile's image has been stored
    fq_tile_by_records(smem, bufs, recs, off, r0, rl, t0, bad);
    __syncthreads();
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int q = 0; q < kFqTile / (16 * kFqThreads); ++q) {
      const int p = (q * kFqThreads + threadIdx.x) * 16;
      if (t0 + p >= total) break;
      __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(smem + p), reinterpret_cast<u32x4 *>(out + t0 + p));
    }
  }
  if (bad != ~0ull) atomicMin(err, bad);
}

}  // namespace

// ---- host side ---------------------------------------------------------------------------

struct ganon_fastq {
  std::vector<std::pair<void *, size_t>> allocs;
  int64_t n = 0, nb = 0, n_tiles = 0;
  uint64_t total = 0;
  FqBufs bufs{};
  FqRec *recs = nullptr;
  uint32_t *len = nullptr;
  uint64_t *off = nullptr;
  int64_t *tile_first = nullptr;
  unsigned long long *bsum = nullptr, *err = nullptr;
  int *dense_list = nullptr;          // tiles left to k_fq_dense
  unsigned int *dense_count = nullptr;
  uint8_t *out = nullptr;
};

namespace {

template <typename T>
int fq_alloc(ganon_ctx *ctx, ganon_fastq *f, T **p, size_t count) {
  *p = nullptr;
  const size_t bytes = std::max<size_t>(count, 1) * sizeof(T) + 128;
  size_t got = 0;
  hipError_t e = ctx_dmalloc(ctx, reinterpret_cast<void **>(p), bytes, &got);
  if (e != hipSuccess) return fail(ctx, GANON_E_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  f->allocs.emplace_back(*p, got);
  return GANON_OK;
}

void fq_release(ganon_ctx *ctx, ganon_fastq *f) {
  for (auto &a : f->allocs) ctx_dfree(ctx, a.first, a.second);
  f->allocs.clear();
}

// Parallel loop over [0, n) in contiguous slices (host packing of the record array).
template <typename F>
void host_parallel(int64_t n, F fn) {
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(std::thread::hardware_concurrency(),
                                                               std::min<int64_t>(16, n / 65536 + 1)));
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t)
    pool.emplace_back([&, t] { fn(n * t / nt, n * (t + 1) / nt); });
  for (auto &th : pool) th.join();
}

}  // namespace

GANON_API int ganon_fastq_upload(ganon_ctx *ctx, const ganon_fastq_records *in, ganon_fastq **out) {
  if (!ctx || !in || !out) return GANON_E_ARG;
  *out = nullptr;
  const int64_t n = in->n;
  if (n < 0 || n > (int64_t)INT32_MAX * 64) return fail(ctx, GANON_E_ARG, "bad record count %lld", (long long)n);
  const int nsb = in->n_seq_bufs, nqb = in->n_qual_bufs;
  if (nsb < 1 || nsb > kFqMaxBufs || nqb < 1 || nqb > kFqMaxBufs)
    return fail(ctx, GANON_E_ARG, "1..%d sequence and quality buffers", kFqMaxBufs);
  if (n && (!in->seq_sel || !in->seq_nib_off || !in->seq_len || !in->reverse || !in->qual_sel || !in->qual_off ||
            !in->qual_len || !in->qual_rev || !in->name_off || !in->name_len || !in->mate))
    return fail(ctx, GANON_E_ARG, "null record array");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipSetDevice failed");
  ganon_fastq *f = new ganon_fastq();
  f->n = n;
  auto bail = [&](int rc) {
    fq_release(ctx, f);
    delete f;
    return rc;
  };
  // extents of every source buffer the records use
  struct Ext { int64_t lo = INT64_MAX, hi = 0; };
  std::vector<Ext> se(kFqMaxBufs), qe(kFqMaxBufs);
  Ext ne;
  uint64_t total = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int s = in->seq_sel[i], q = in->qual_sel[i];
    const int64_t L = in->seq_len[i], Q = in->qual_len[i], NL = in->name_len[i];
    if (s >= nsb || q >= nqb || L < 0 || Q < 0 || NL < 0 || NL > 0xFFFF || in->seq_nib_off[i] < 0 ||
        in->qual_off[i] < 0 || in->name_off[i] < 0)
      return bail(fail(ctx, GANON_E_ARG, "record %lld: bad buffer, length or offset", (long long)i));
    if (L) {
      se[s].lo = std::min(se[s].lo, in->seq_nib_off[i] >> 1);
      se[s].hi = std::max(se[s].hi, (in->seq_nib_off[i] + L + 1) >> 1);
    }
    if (Q) {
      qe[q].lo = std::min(qe[q].lo, in->qual_off[i]);
      qe[q].hi = std::max(qe[q].hi, in->qual_off[i] + Q);
    }
    if (NL) {
      ne.lo = std::min(ne.lo, in->name_off[i]);
      ne.hi = std::max(ne.hi, in->name_off[i] + NL);
    }
    const uint64_t rl = (uint64_t)(8 + NL + L + Q);
    if (rl > UINT32_MAX) return bail(fail(ctx, GANON_E_ARG, "record %lld longer than 4 GiB", (long long)i));
    total += rl;
  }
  if (ne.lo == INT64_MAX) ne.lo = ne.hi = 0;
  for (auto &e : se) if (e.lo == INT64_MAX) e.lo = e.hi = 0;
  for (auto &e : qe) if (e.lo == INT64_MAX) e.lo = e.hi = 0;
  int rc;
  // sources: device batch buffers (no copy) or the used slice of each host buffer
  int64_t seq_base[kFqMaxBufs] = {0, 0, 0, 0};
  if (in->seq_batch) {
    const uint8_t *din = nullptr, *dout = nullptr;
    int64_t bytes = 0;
    if ((rc = ganon_dbatch_seq_buffers(in->seq_batch, &din, &dout, &bytes))) return bail(fail(ctx, rc, "bad batch"));
    if (nsb > 2) return bail(fail(ctx, GANON_E_ARG, "a device batch provides two sequence buffers"));
    for (int s = 0; s < nsb; ++s)
      if (se[s].hi > bytes) return bail(fail(ctx, GANON_E_ARG, "sequence offset past the batch buffer"));
    f->bufs.seq[0] = dout;
    f->bufs.seq[1] = din;
  } else {
    if (!in->seq_buf) return bail(fail(ctx, GANON_E_ARG, "no sequence buffers"));
    for (int s = 0; s < nsb; ++s) {
      uint8_t *d = nullptr;
      const int64_t sz = se[s].hi - se[s].lo;
      if (sz && !in->seq_buf[s]) return bail(fail(ctx, GANON_E_ARG, "null sequence buffer %d", s));
      if ((rc = fq_alloc(ctx, f, &d, (size_t)sz))) return bail(rc);
      if (sz) HIP_OR_FAIL(hipMemcpyAsync(d, in->seq_buf[s] + se[s].lo, sz, hipMemcpyHostToDevice, ctx->stream));
      f->bufs.seq[s] = d;
      seq_base[s] = se[s].lo;
    }
  }
  if (!in->qual_buf) return bail(fail(ctx, GANON_E_ARG, "no quality buffers"));
  for (int q = 0; q < nqb; ++q) {
    uint8_t *d = nullptr;
    const int64_t sz = qe[q].hi - qe[q].lo;
    if (sz && !in->qual_buf[q]) return bail(fail(ctx, GANON_E_ARG, "null quality buffer %d", q));
    if ((rc = fq_alloc(ctx, f, &d, (size_t)sz))) return bail(rc);
    if (sz) HIP_OR_FAIL(hipMemcpyAsync(d, in->qual_buf[q] + qe[q].lo, sz, hipMemcpyHostToDevice, ctx->stream));
    f->bufs.qual[q] = d;
  }
  {
    uint8_t *d = nullptr;
    const int64_t sz = ne.hi - ne.lo;
    if (sz && !in->names) return bail(fail(ctx, GANON_E_ARG, "null name blob"));
    if ((rc = fq_alloc(ctx, f, &d, (size_t)sz))) return bail(rc);
    if (sz) HIP_OR_FAIL(hipMemcpyAsync(d, in->names + ne.lo, sz, hipMemcpyHostToDevice, ctx->stream));
    f->bufs.names = d;
  }
  for (int s = nsb; s < kFqMaxBufs; ++s) f->bufs.seq[s] = f->bufs.seq[0];
  for (int q = nqb; q < kFqMaxBufs; ++q) f->bufs.qual[q] = f->bufs.qual[0];
  // packed records and lengths (lengths padded to whole scan blocks with zeros)
  f->nb = (n + kFqScanBlock - 1) / kFqScanBlock;
  f->total = total;
  f->n_tiles = (int64_t)((total + kFqTile - 1) / kFqTile);
  std::vector<FqRec> rec((size_t)n);
  std::vector<uint32_t> len((size_t)(f->nb * kFqScanBlock), 0u);
  host_parallel(n, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      const int s = in->seq_sel[i], q = in->qual_sel[i];
      FqRec &R = rec[i];
      R.seq = (uint64_t)(in->seq_nib_off[i] - 2 * seq_base[s]) | ((uint64_t)s << 56) |
              ((uint64_t)(in->reverse[i] != 0) << 58) | ((uint64_t)(in->qual_rev[i] != 0) << 59);
      R.qual = (uint64_t)(in->qual_off[i] - qe[q].lo) | ((uint64_t)in->mate[i] << 48) | ((uint64_t)q << 56);
      R.name = (uint64_t)(in->name_len[i] ? in->name_off[i] - ne.lo : 0) | ((uint64_t)in->name_len[i] << 48);
      R.len = (uint32_t)in->seq_len[i];
      R.qlen = (uint32_t)in->qual_len[i];
      len[i] = (uint32_t)(8 + in->name_len[i] + in->seq_len[i] + in->qual_len[i]);
    }
  });
  if ((rc = fq_alloc(ctx, f, &f->recs, (size_t)n))) return bail(rc);
  if ((rc = fq_alloc(ctx, f, &f->len, len.size()))) return bail(rc);
  if ((rc = fq_alloc(ctx, f, &f->off, (size_t)n + 1))) return bail(rc);
  if ((rc = fq_alloc(ctx, f, &f->tile_first, (size_t)f->n_tiles + 1))) return bail(rc);
  if ((rc = fq_alloc(ctx, f, &f->bsum, (size_t)f->nb))) return bail(rc);
  if ((rc = fq_alloc(ctx, f, &f->err, 1))) return bail(rc);
  if ((rc = fq_alloc(ctx, f, &f->dense_list, (size_t)f->n_tiles))) return bail(rc);
  if ((rc = fq_alloc(ctx, f, &f->dense_count, 1))) return bail(rc);
  if ((rc = fq_alloc(ctx, f, &f->out, (size_t)f->n_tiles * kFqTile))) return bail(rc);
  if (n) {
    HIP_OR_FAIL(hipMemcpyAsync(f->recs, rec.data(), rec.size() * sizeof(FqRec), hipMemcpyHostToDevice, ctx->stream));
    HIP_OR_FAIL(hipMemcpyAsync(f->len, len.data(), len.size() * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
  }
  HIP_OR_FAIL(hipMemsetAsync(f->err, 0xFF, sizeof(unsigned long long), ctx->stream));
  HIP_OR_FAIL(ganon_detail::sync_stream(ctx->stream));   // the host staging vectors die here
  *out = f;
  return GANON_OK;
}

GANON_API int ganon_fastq_run(ganon_ctx *ctx, ganon_fastq *f) {
  if (!ctx || !f) return GANON_E_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipSetDevice failed");
  if (ctx->profiling) {
    for (auto &r : ctx->recs) {
      ctx->pool.push_back(r.e0);
      ctx->pool.push_back(r.e1);
    }
    ctx->recs.clear();
  }
  if (f->n == 0) return GANON_OK;
  int rc;
  {
    KernelScope ks(ctx, "k_fq_scan");
    hipLaunchKernelGGL(k_fq_bsum, dim3((unsigned)f->nb), dim3(kFqThreads), 0, ctx->stream, f->len, f->bsum);
    hipLaunchKernelGGL(k_fq_bscan, dim3(1), dim3(kFqScanThreads), 0, ctx->stream, f->bsum, f->nb, f->err,
                       f->dense_count);
    hipLaunchKernelGGL(k_fq_off, dim3((unsigned)f->nb), dim3(kFqThreads), 0, ctx->stream, f->len, f->bsum, f->n,
                       f->off, f->tile_first);
    if ((rc = check_launch(ctx, "k_fq_scan"))) return rc;
  }
  {
    KernelScope ks(ctx, "k_fq_format");
    // virtual dwords per lane per round: a tile holds ~2,100 of them (2,048 tile dwords plus the
    // dwords neighbouring fields share), so the width sets the number of dependent load rounds
    const int kd = ctx->fq_kd;
    auto kern = kd == 16 ? k_fq_quad<2> : kd == 12 ? k_fq_rows : kd == 9 ? k_fq_quad<1> : kd == 10 ? k_fq_quad<3>
              : kd == 11 ? k_fq_quad<2, false>
              : kd == 1 ? k_fq_format<1> : kd == 2 ? k_fq_format<2> : kd == 3 ? k_fq_format<3>
              : kd == 5 ? k_fq_format<5> : kd == 6 ? k_fq_format<6> : kd == 8 ? k_fq_format<8> : k_fq_format<4>;
    if (kd == 0 || (kd >= 13 && kd <= 15) || kd == 17) {   // span kernels (default: 3 units per lane, one 8 KiB tile)
      const int tm = kd == 14 ? 2 : 1;
      auto sk = kd == 0 ? k_fq_span<3, 1, true> : kd == 13 ? k_fq_span<2, 1> : kd == 14 ? k_fq_span<2, 2>
              : kd == 15 ? k_fq_span<3, 1, true, 1> : k_fq_span<3, 1, true, 2>;
      hipLaunchKernelGGL(sk, dim3((unsigned)((f->n_tiles + tm - 1) / tm)), dim3(kFqThreads), 0, ctx->stream, f->bufs,
                         f->recs, f->off, f->tile_first, f->n, f->total, f->out, f->err, ctx->fq_skip, f->dense_list,
                         f->dense_count, f->n_tiles);
    } else {
      hipLaunchKernelGGL(kern, dim3((unsigned)f->n_tiles), dim3(kFqThreads), 0, ctx->stream, f->bufs, f->recs,
                         f->off, f->tile_first, f->n, f->total, f->out, f->err, ctx->fq_skip, f->dense_list,
                         f->dense_count);
    }
    hipLaunchKernelGGL(k_fq_dense, dim3(kFqDenseGrid), dim3(kFqThreads), 0, ctx->stream, f->bufs, f->recs, f->off,
                       f->tile_first, f->n, f->total, f->out, f->err, f->dense_list, f->dense_count);
    if ((rc = check_launch(ctx, "k_fq_format"))) return rc;
  }
  return GANON_OK;
}

GANON_API int64_t ganon_fastq_bytes(const ganon_fastq *f) { return f ? (int64_t)f->total : -1; }

GANON_API int ganon_fastq_device_output(const ganon_fastq *f, void **dev_ptr) {
  if (!f || !dev_ptr) return GANON_E_ARG;
  *dev_ptr = f->out;
  return GANON_OK;
}

GANON_API int64_t ganon_fastq_download(ganon_ctx *ctx, ganon_fastq *f, char *out, int64_t cap) {
  constexpr int64_t kFailed = GANON_FASTQ_FAILED;
  if (!ctx || !f || (!out && f->total)) return kFailed;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipSetDevice failed"), kFailed;
  unsigned long long bad = ~0ull;
  if (f->n && ganon_detail::readback(&bad, f->err, sizeof bad, ctx->stream) != hipSuccess)
    return fail(ctx, GANON_E_DEVICE, "error-slot copy failed"), kFailed;
  if (ganon_detail::sync_stream(ctx->stream) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "formatter run failed"), kFailed;
  if (bad != ~0ull) {
    fail(ctx, GANON_E_ARG, "record %llu: reverse read with a base outside ACGTN (SURVEY Q7)", bad);
    return -(int64_t)bad - 1;
  }
  if ((int64_t)f->total > cap) {
    fail(ctx, GANON_E_ARG, "output buffer too small (%llu bytes needed)", (unsigned long long)f->total);
    return INT64_MIN;
  }
  if (f->total && (hipMemcpyAsync(out, f->out, f->total, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                   ganon_detail::sync_stream(ctx->stream) != hipSuccess))
    return fail(ctx, GANON_E_DEVICE, "output copy failed"), kFailed;
  return (int64_t)f->total;
}

GANON_API int ganon_fastq_free(ganon_ctx *ctx, ganon_fastq *f) {
  if (!f) return GANON_E_ARG;
  if (ctx) hipSetDevice(ctx->device);
  fq_release(ctx, f);
  delete f;
  return GANON_OK;
}

GANON_API int64_t ganon_fastq_format_hip(ganon_ctx *ctx, int64_t n, const uint8_t *const *seq_buf,
                                         const uint8_t *seq_sel, const int64_t *seq_nib_off, const int32_t *seq_len,
                                         const uint8_t *reverse, const uint8_t *const *qual_buf,
                                         const uint8_t *qual_sel, const int64_t *qual_off, const int32_t *qual_len,
                                         const uint8_t *qual_rev, const char *names, const int64_t *name_off,
                                         const int32_t *name_len, const uint8_t *mate, char *out, int64_t cap) {
  if (!ctx || n < 0) return GANON_FASTQ_FAILED;
  ganon_fastq_records r{};
  r.n = n;
  int ms = 0, mq = 0;
  for (int64_t i = 0; i < n; ++i) {
    ms = std::max<int>(ms, seq_sel[i]);
    mq = std::max<int>(mq, qual_sel[i]);
  }
  r.n_seq_bufs = ms + 1;
  r.n_qual_bufs = mq + 1;
  r.seq_buf = seq_buf;
  r.seq_sel = seq_sel;
  r.seq_nib_off = seq_nib_off;
  r.seq_len = seq_len;
  r.reverse = reverse;
  r.qual_buf = qual_buf;
  r.qual_sel = qual_sel;
  r.qual_off = qual_off;
  r.qual_len = qual_len;
  r.qual_rev = qual_rev;
  r.names = names;
  r.name_off = name_off;
  r.name_len = name_len;
  r.mate = mate;
  ganon_fastq *f = nullptr;
  if (ganon_fastq_upload(ctx, &r, &f)) return GANON_FASTQ_FAILED;
  const int64_t w = ganon_fastq_run(ctx, f) ? GANON_FASTQ_FAILED : ganon_fastq_download(ctx, f, out, cap);
  ganon_fastq_free(ctx, f);
  return w;
}
