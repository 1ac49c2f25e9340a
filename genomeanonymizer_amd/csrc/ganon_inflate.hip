// ganon_inflate.hip — BGZF block inflate on MI355X (gfx950), part of libganon_hip.so; C ABI in
// include/ganon.h (ganon_inflate). SURVEY §8(f)4: the input decode offload.
//
// The host BAM reader (ganon_host.cpp) cuts a window of the compressed file into BGZF blocks —
// independent raw DEFLATE streams (RFC 1951) of at most 64 KiB of output each — and hands their
// payloads here instead of to zlib on its threads (ganon_bam_reader_set_inflater).
//
// One 64-lane workgroup per block, and the wave decodes it as ONE decoder: Huffman decoding is a
// serial bit stream. Token rounds (round 5, below): every lane decodes the token that would start
// at one of the next 256 bit offsets, a scalar chain through them (readlane) finds the true token
// boundaries, the literals are written by their lanes at once and the matches copied in stream
// order by all lanes (periodic source index w - dist + (j mod dist): even an overlapping match has
// no intra-copy dependence); tokens the tables cannot finish go through the scalar symbol loop.
// The payload comes through a 2 KiB LDS ring; the output through an 8 KiB LDS ring written out to
// the block's output every completed 1 KiB, and matches further back than 4 KiB read the written
// output from global memory. ~16 KiB of LDS per decoder: ten blocks decode per CU. Stored, fixed-
// and dynamic-Huffman blocks. Every read and write is range-checked (output against the block's
// ISIZE): a malformed stream sets the block's status and stops it, never faults.
// Written from RFC 1951 and the BGZF section of the SAM specification.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ganon_ctx.h"

namespace {

using ganon_detail::check_launch;
using ganon_detail::fail;

constexpr int kInfThreads = 64;
constexpr int kWin = 65536;          // BGZF: at most 64 KiB of output per block
constexpr int kRing = 2048;          // payload ring (LDS), refilled kRing/2 bytes at a time
constexpr int kRingHalf = kRing / 2;
// Output: an 8 KiB LDS ring of the latest output, written out to the block's output every
// completed kFlush bytes; a match reaching further back than kNear reads the block's output in
// global memory (written out and fenced by then). Round 5: the ring held DEFLATE's whole 32 KiB
// window (40 KiB of LDS per decoder, 4 decoders per CU, one wave per SIMD: every dependent
// instruction of the serial decoder waited out its latency alone); 16 KiB per decoder fits 10.
constexpr int kOutRing = 8192;
constexpr int kFlush = 1024;
constexpr int kNear = 4096;
#ifndef INF_FAST_BITS
#define INF_FAST_BITS 10
#endif
constexpr int kFastBits = INF_FAST_BITS;   // Huffman lookup table width
constexpr uint32_t kFastMask = (1u << kFastBits) - 1;

// Canonical Huffman code: counts per length, symbols by (length, value), a kFastBits lookup table
// of (symbol | length << 9) for codes of at most kFastBits bits (0: longer code or none).
struct Huff {
  uint16_t count[16];
  uint16_t symbol[288];
  uint16_t fast[1 << kFastBits];
};

constexpr int kRoundK = 4;        // token rounds: kRoundK x 64 bit offsets decoded at once
constexpr int kRoundMaxM = 8;     // ... at most this many matches per round
constexpr int kRoundOut = 2048;   // ... and about this many output bytes (+ one match)

struct InfShared {
  uint8_t out[kOutRing];
  uint8_t ring[kRing];
  Huff lit, dist;
  uint16_t lens[19 + 288 + 32];   // code-length code, then literal/length + distance lengths
  int4 mrec[kRoundMaxM];          // a round's matches: bit offset, output offset, length, distance
};

constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum { kInfOk = 0, kInfBadBlock = 1, kInfBadCode = 2, kInfOverrun = 3, kInfBadDist = 4, kInfSize = 5 };

// The decoder below is host-callable too (NL = 1 lane, no barriers): tools/inflate_host_check.cpp
// runs the same code against zlib without a GPU.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (uint64_t)(uint32_t)uni((int)(uint32_t)v) | ((uint64_t)(uint32_t)uni((int)(uint32_t)(v >> 32)) << 32);
}
// LDS operations of one wave complete in issue order, so a lane reading what another lane of the
// same (single-wave) workgroup stored earlier needs only the compiler kept from reordering them
#define INF_WAVE_ORDER() __asm__ __volatile__("" ::: "memory")
#else
inline int uni(int v) { return v; }
inline uint64_t uni64(uint64_t v) { return v; }
#define INF_WAVE_ORDER() ((void)0)
#endif
#define INF_FN __host__ __device__
// (the decoder state must stay in registers: a helper left out of line takes its reference arguments
// to the stack, and every access of the bit reader becomes a scratch round trip)
#define INF_INL __host__ __device__ __attribute__((always_inline)) inline

// LSB-first bit reader. Payload bytes [filled - kRing, filled) are in the LDS ring (index & mask);
// top_up (wave-uniform: every lane calls it together) keeps at least kRingHalf bytes ahead of pos.
template <int NL>
struct Bits {
  const uint8_t *g;   // the block's payload in global memory
  uint8_t *ring;
  int n, pos, filled, lane;
  uint64_t buf;
  int cnt;
  INF_INL void top_up() {
    // (refilled 64 bytes early: a token round rewinds pos by up to 8 bytes of the bit buffer, and
    // those must still be in the ring)
    if (filled < n && filled - pos < kRingHalf - 64) {
      INF_WAVE_ORDER();   // earlier ring reads are issued before their slots are overwritten
      const int e = filled + kRingHalf < n ? filled + kRingHalf : n;
      // kRingHalf / NL consecutive bytes per lane, all loads issued before the first store
      constexpr int kPer = kRingHalf / NL;
      const int k0 = filled + lane * kPer;
      uint8_t v[kPer];
#pragma unroll
      for (int i = 0; i < kPer; ++i) v[i] = k0 + i < e ? g[k0 + i] : 0;
#pragma unroll
      for (int i = 0; i < kPer; ++i)
        if (k0 + i < e) ring[(k0 + i) & (kRing - 1)] = v[i];
      filled = e;
      INF_WAVE_ORDER();
    }
  }
  // Tops the bit buffer up to 57..64 bits (or the end of the payload) with one LDS round trip:
  // the three aligned ring dwords under the next 8 bytes.
  INF_INL void refill() {
    if (cnt > 56 || pos >= n) return;
    top_up();
    const uint32_t *rw = reinterpret_cast<const uint32_t *>(ring);
    constexpr int kWm = kRing / 4 - 1;
    const int w = pos >> 2;
    const uint32_t w0 = (uint32_t)uni((int)rw[w & kWm]), w1 = (uint32_t)uni((int)rw[(w + 1) & kWm]),
                   w2 = (uint32_t)uni((int)rw[(w + 2) & kWm]);
    const int sh = 8 * (pos & 3);
    const uint64_t lo = (uint64_t)w0 | ((uint64_t)w1 << 32), hi = (uint64_t)w2;
    const uint64_t v = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;   // payload bytes pos .. pos + 7
    int nb = (64 - cnt) >> 3;
    if (nb > n - pos) nb = n - pos;
    buf |= (nb == 8 ? v : v & ((1ull << (8 * nb)) - 1)) << cnt;
    cnt += 8 * nb;
    pos += nb;
  }
  INF_INL bool need(int k) {
    if (cnt < k) refill();
    return cnt >= k;
  }
  // the decoder state is wave-uniform: say so to the compiler (scalar registers, scalar branches)
  INF_INL void uniform() {
    pos = uni(pos);
    filled = uni(filled);
    cnt = uni(cnt);
    buf = uni64(buf);
  }
  INF_INL uint32_t take(int k) {   // (need(k) checked by the caller)
    const uint32_t v = k ? (uint32_t)(buf & ((1ull << k) - 1)) : 0u;
    buf >>= k;
    cnt -= k;
    return v;
  }
};

INF_FN inline uint32_t rev_bits(uint32_t v, int n) { return __builtin_bitreverse32(v) >> (32 - n); }

// Build h from n code lengths; false on an over-subscribed code (an incomplete one is allowed:
// RFC 1951 permits a single distance code). Counts and symbols: every lane writes the same values;
// the lookup table: split over the lanes.
template <int NL>
__attribute__((noinline)) INF_FN bool huff_build(Huff &h, const uint16_t *len, int n, int lane) {
  uint32_t cnt[16];
  for (int l = 0; l < 16; ++l) cnt[l] = 0;
  for (int s = 0; s < n; ++s) {
    const int l = uni(len[s]);
    if (l >= 16) return false;
    cnt[l]++;
  }
  cnt[0] = 0;
  int left = 1;
  for (int l = 1; l < 16; ++l) {
    left <<= 1;
    left -= (int)cnt[l];
    if (left < 0) return false;
  }
  uint32_t offs[16];
  offs[0] = offs[1] = 0;
  for (int l = 1; l < 15; ++l) offs[l + 1] = offs[l] + cnt[l];
  for (int l = 0; l < 16; ++l) h.count[l] = (uint16_t)cnt[l];
  for (int s = 0; s < n; ++s) {
    const int l = uni(len[s]);
    if (l) h.symbol[offs[l]++] = (uint16_t)s;
  }
  for (int i = lane; i < (1 << kFastBits); i += NL) h.fast[i] = 0;
  INF_WAVE_ORDER();
  // canonical codes of lengths <= kFastBits into the table (bit-reversed: the stream's bit order);
  // the 2^(kFastBits - l) entries of a code are split over the lanes
  int code = 0, idx = 0;
  for (int l = 1; l <= kFastBits; ++l) {
    for (uint32_t k = 0; k < cnt[l]; ++k, ++idx, ++code) {
      const uint32_t r = rev_bits((uint32_t)code, l);
      const uint16_t e = (uint16_t)(uni(h.symbol[idx]) | (l << 9));
      for (uint32_t f = r + ((uint32_t)lane << l); f < (1u << kFastBits); f += (uint32_t)NL << l) h.fast[f] = e;
    }
    code <<= 1;
  }
  INF_WAVE_ORDER();
  return true;
}

// One symbol through the table (header code-length codes); -1 on an invalid code or a stream
// that ends inside it.
template <int NL>
INF_INL int huff_decode(const Huff &h, Bits<NL> &b) {
  b.refill();
  if (b.cnt >= kFastBits || b.pos >= b.n) {
    const int e = uni(h.fast[b.buf & kFastMask]);
    const int l = e >> 9;
    if (l && l <= b.cnt) {
      b.take(l);
      return e & 511;
    }
  }
  // longer codes: the canonical walk, one bit at a time (RFC 1951 3.2.2)
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; ++l) {
    if (!b.need(1)) return -1;
    code |= (int)b.take(1);
    const int count = uni(h.count[l]);
    if (code - count < first) return uni(h.symbol[index + (code - first)]);
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

// A code the kFastBits table does not finish (longer, or near the end of the payload): the
// canonical walk (RFC 1951 3.2.2) over the cnt valid bits of buf. Returns sym | length << 16, -1.
__attribute__((noinline)) INF_FN int huff_slow(const Huff &h, uint64_t buf, int cnt) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16 && l <= cnt; ++l) {
    code |= (int)((buf >> (l - 1)) & 1);
    const int count = uni(h.count[l]);
    if (code - count < first) return uni(h.symbol[index + (code - first)]) | (l << 16);
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

// Output bytes [from, to) of the ring to dst (the block's output), by the lanes.
template <int NL>
INF_INL void flush_out(const uint8_t *ring, uint8_t *dst, int from, int to, int lane) {
  INF_WAVE_ORDER();   // the ring bytes (lane 0's literals, every lane's copies) are issued
  // dword stores over the aligned middle when the chunk does not wrap the ring
  int a = from;
  const int a4 = (from + 3) & ~3, b4 = to & ~3;
  const bool words = (((uintptr_t)(dst + a4)) & 3) == 0 && a4 < b4 &&
                     (a4 & (kOutRing - 1)) + (b4 - a4) <= kOutRing;
  if (words) {
    for (int k0 = from; k0 < a4; k0 += NL) {
      const int k = k0 + lane;
      if (k < a4) dst[k] = ring[k & (kOutRing - 1)];
    }
    const uint32_t *rw = reinterpret_cast<const uint32_t *>(ring + (a4 & (kOutRing - 1)));
    uint32_t *dw = reinterpret_cast<uint32_t *>(dst + a4);
    const int nw = (b4 - a4) >> 2;
    for (int k0 = 0; k0 < nw; k0 += NL) {
      const int k = k0 + lane;
      if (k < nw) dw[k] = rw[k];
    }
    a = b4;
  }
  for (int k0 = a; k0 < to; k0 += NL) {
    const int k = k0 + lane;
    if (k < to) dst[k] = ring[k & (kOutRing - 1)];
  }
  // far matches read these bytes back from global memory (other lanes of this wave): the stores
  // complete before any later load
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#endif
}


// Copy of a match: out[w + j] = out[w - dist + j], j < len, by all lanes at once (a periodic source
// index for an overlapping match: out[w + j] = out[w - dist + (j mod dist)]).
template <int NL>
INF_INL void copy_match(InfShared &S, const uint8_t *dst, int w, int len, int dist, int lane) {
  constexpr int M = kOutRing - 1;
  INF_WAVE_ORDER();   // the literals and the last copy are read by every lane
  if (dist > kNear) {   // (far: its source is written out; dist > kNear >= len, no overlap)
    for (int j0 = 0; j0 < len; j0 += NL) {
      const int j = j0 + lane;
      if (j < len) S.out[(w + j) & M] = dst[w - dist + j];
    }
  } else if (dist >= len) {
    for (int j0 = 0; j0 < len; j0 += NL) {
      const int j = j0 + lane;
      if (j < len) S.out[(w + j) & M] = S.out[(w - dist + j) & M];
    }
  } else {
    // lane mod dist, lane < 64 (exact: (lane + 1/2) / dist is >= 1/(2 dist) from an integer)
    const int q = (int)(((float)lane + 0.5f) / (float)dist);
    int r = lane - q * dist;
    const int step = NL % dist;
    for (int j0 = 0; j0 < len; j0 += NL) {
      if (j0 + lane < len) S.out[(w + j0 + lane) & M] = S.out[(w - dist + r) & M];
      r += step;
      if (r >= dist) r -= dist;
    }
  }
}

// ---- token rounds ------------------------------------------------------------------------------
// The scalar symbol loop pays one dependent LDS lookup and ~20 scalar instructions per code, and a
// wave issues one instruction per 4 cycles: ~400 cycles per literal. A round instead decodes, on
// every lane, the token (literal, or length + distance with their extra bits) that WOULD start at
// each of the next kRoundK x 64 bit offsets — independent lookups, issued together. The true token
// boundaries are then a scalar chain through those lanes (readlane: offset -> offset + the token's
// bit length), a handful of scalar instructions per token; the round's literals are written by
// their lanes at once, its matches copied in stream order. A token the tables cannot finish (a
// code longer than kFastBits, the end-of-block code, bits past the payload, an invalid code) stops
// the chain: the scalar loop decodes that one token, with every check, and rounds resume.
constexpr uint32_t kTokMatch = 1u << 15, kTokStop = 1u << 16;
// (tuning build, -DINF_PROF: cycles of each part of a round, summed per wave, tools/inflate_prof.py)
#if defined(INF_PROF)
__device__ unsigned long long g_inf_prof[6];
#endif
#if defined(INF_PROF) && defined(__HIP_DEVICE_COMPILE__)
#define INF_T() ((uint64_t)__builtin_amdgcn_s_memtime())
#define INF_ACC(i, t0) (prof[i] += INF_T() - (t0))
#else
#define INF_T() ((uint64_t)0)
#define INF_ACC(i, t0) ((void)(t0))
#endif
#ifdef INF_STATS
long long inf_stats[8];
#endif

// The tokens at bits B0 + 64 k (k < kRoundK) of the payload (the ring holds them): bits 0-5 the
// token's length in bits, 6-14 its output length, kTokMatch, kTokStop, 24-31 a literal's byte;
// d[k] a match's distance. Branch-free, so that the LDS reads of every k are in flight together:
// the ring words (the same shift for every k), then the literal/length codes, then the distance
// codes (looked up for literals too, and ignored).
INF_INL void lane_tokens(const InfShared &S, uint32_t B0, uint32_t nbits, uint32_t *t, uint32_t *d) {
  const uint32_t *rw = reinterpret_cast<const uint32_t *>(S.ring);
  constexpr int kWm = kRing / 4 - 1;
  const uint32_t wd = B0 >> 5;
  const int sh = (int)(B0 & 31);
  uint32_t wv[2 * kRoundK + 1];
#pragma unroll
  for (int i = 0; i < 2 * kRoundK + 1; ++i) wv[i] = rw[(wd + (uint32_t)i) & kWm];
  uint64_t bits[kRoundK];
  int e[kRoundK];
#pragma unroll
  for (int k = 0; k < kRoundK; ++k) {
    const uint64_t lo = (uint64_t)wv[2 * k] | ((uint64_t)wv[2 * k + 1] << 32);
    bits[k] = (lo >> sh) | (((uint64_t)wv[2 * k + 2] << 1) << (63 - sh));   // (sh = 0: no high word)
    e[k] = S.lit.fast[bits[k] & kFastMask];
  }
  int len[kRoundK], lbits[kRoundK], dd[kRoundK];
  uint64_t b2[kRoundK];
#pragma unroll
  for (int k = 0; k < kRoundK; ++k) {
    const int l = e[k] >> 9, sym = e[k] & 511;
    const int li = sym > 256 ? sym - 257 : 0;   // RFC 1951 3.2.5 length codes
    const int le = li < 8 || li >= 28 ? 0 : (li - 4) >> 2;
    const int lb = li < 8 ? 3 + li : li == 28 ? 258 : ((4 + (li & 3)) << le) + 3;
    len[k] = lb + (int)((bits[k] >> l) & ((1u << le) - 1));
    lbits[k] = l + le;
    b2[k] = bits[k] >> lbits[k];
    dd[k] = S.dist.fast[b2[k] & kFastMask];
  }
#pragma unroll
  for (int k = 0; k < kRoundK; ++k) {
    const int l = e[k] >> 9, sym = e[k] & 511;
    const int dl = dd[k] >> 9, ds = dd[k] & 511;
    const int de = ds < 4 ? 0 : (ds - 2) >> 1;
    const uint32_t dv = (uint32_t)(ds < 4 ? 1 + ds : ((2 + (ds & 1)) << de) + 1) +
                        (uint32_t)((b2[k] >> dl) & ((1u << de) - 1));
    const bool lit = l && sym < 256;
    const bool match = l && sym > 256 && sym < 257 + 29 && dl && ds < 30;
    uint32_t tok = lit ? (uint32_t)l | (1u << 6) | ((uint32_t)sym << 24)
                 : match ? (uint32_t)(lbits[k] + dl + de) | ((uint32_t)len[k] << 6) | kTokMatch : kTokStop;
    if ((uint64_t)B0 + 64 * k + (tok & 63) > nbits) tok = kTokStop;
    t[k] = tok;
    d[k] = dv;
  }
}

// The tokens of one round. On the device each lane holds its kRoundK offsets in registers, the
// chain reads them with readlane and writes each literal's output offset back with writelane; the
// host build (NL = 1) keeps all kRoundK x 64 in arrays.
template <int NL>
struct RoundToks {
  uint32_t t[kRoundK][64], d[kRoundK][64];
  int pos[kRoundK][64];
  INF_FN void fill(const InfShared &S, uint32_t P, uint32_t nbits, int) {
    for (int l = 0; l < 64; ++l) {
      uint32_t tt[kRoundK], dd[kRoundK];
      lane_tokens(S, P + (uint32_t)l, nbits, tt, dd);
      for (int k = 0; k < kRoundK; ++k) {
        t[k][l] = tt[k];
        d[k][l] = dd[k];
      }
    }
  }
  // The chain through the literals of k from offset xk: each one's output offset recorded, its bit
  // set in m. Stops at offset 64, at `lim` bytes of output, or at a match / stop token (returned).
  INF_FN uint32_t chain(int k, int &xk, int &out, int lim, uint64_t &m) {
    uint32_t tk = 0;
    while (xk < 64 && out < lim) {
      tk = t[k][xk];
      if (tk & (kTokStop | kTokMatch)) break;
      pos[k][xk] = out;
      m |= 1ull << xk;
      ++out;
      xk += (int)(tk & 63);
    }
    return tk;
  }
  INF_FN uint32_t dist(int k, int l) const { return d[k][l]; }
  template <class F>
  INF_FN void each_literal(const uint64_t (&lm)[kRoundK], int, F &&f) const {
    for (int k = 0; k < kRoundK; ++k)
      for (int l = 0; l < 64; ++l)
        if ((lm[k] >> l) & 1) f(64 * k + l, pos[k][l], (uint8_t)(t[k][l] >> 24));
  }
};
#if defined(__HIP_DEVICE_COMPILE__)
template <>
struct RoundToks<64> {
  uint32_t t[kRoundK], d[kRoundK];
  int pos[kRoundK];
  __device__ void fill(const InfShared &S, uint32_t P, uint32_t nbits, int lane) {
    lane_tokens(S, P + (uint32_t)lane, nbits, t, d);
  }
  // (the literal loop in scalar instructions: a readlane, a test, a writelane, a bit set, three adds)
  __device__ uint32_t chain(int k, int &xk, int &out, int lim, uint64_t &m) {
    uint32_t tk, tmp;
    int p = pos[k];
    xk = uni(xk);   // (wave-uniform: the compiler must see scalars for the asm's SGPR operands)
    out = uni(out);
    lim = uni(lim);
    m = uni64(m);
    // (the offset lives in m0 inside the loop: writelane may take m0 as its lane select beside an
    // SGPR value, where a second SGPR would break the one-SGPR operand limit)
    // (with room for a whole k of literals — at most 64 — the output limit is not tested per
    // literal, and the loop takes two literals per branch back)
    __asm__ __volatile__(
        "s_mov_b32 %[tk], 0\n\t"
        "s_mov_b32 m0, %[xk]\n\t"
        "s_sub_i32 %[tmp], %[lim], %[out]\n\t"
        "s_cmp_lt_i32 %[tmp], 64\n\t"
        "s_cbranch_scc1 3f\n"
        "1:\n\t"
        "s_cmp_lt_i32 m0, 64\n\t"
        "s_cbranch_scc0 2f\n\t"
        "v_readlane_b32 %[tk], %[tv], m0\n\t"
        "s_and_b32 %[tmp], %[tk], 0x18000\n\t"
        "s_cbranch_scc1 2f\n\t"
        "v_writelane_b32 %[p], %[out], m0\n\t"
        "s_bitset1_b64 %[m], m0\n\t"
        "s_and_b32 %[tmp], %[tk], 63\n\t"
        "s_add_i32 %[out], %[out], 1\n\t"
        "s_add_i32 m0, m0, %[tmp]\n\t"
        "s_cmp_lt_i32 m0, 64\n\t"
        "s_cbranch_scc0 2f\n\t"
        "v_readlane_b32 %[tk], %[tv], m0\n\t"
        "s_and_b32 %[tmp], %[tk], 0x18000\n\t"
        "s_cbranch_scc1 2f\n\t"
        "v_writelane_b32 %[p], %[out], m0\n\t"
        "s_bitset1_b64 %[m], m0\n\t"
        "s_and_b32 %[tmp], %[tk], 63\n\t"
        "s_add_i32 %[out], %[out], 1\n\t"
        "s_add_i32 m0, m0, %[tmp]\n\t"
        "s_branch 1b\n"
        "3:\n\t"
        "s_cmp_lt_i32 m0, 64\n\t"
        "s_cbranch_scc0 2f\n\t"
        "s_cmp_lt_i32 %[out], %[lim]\n\t"
        "s_cbranch_scc0 2f\n\t"
        "v_readlane_b32 %[tk], %[tv], m0\n\t"
        "s_and_b32 %[tmp], %[tk], 0x18000\n\t"
        "s_cbranch_scc1 2f\n\t"
        "v_writelane_b32 %[p], %[out], m0\n\t"
        "s_bitset1_b64 %[m], m0\n\t"
        "s_and_b32 %[tmp], %[tk], 63\n\t"
        "s_add_i32 %[out], %[out], 1\n\t"
        "s_add_i32 m0, m0, %[tmp]\n\t"
        "s_branch 3b\n"
        "2:\n\t"
        "s_mov_b32 %[xk], m0"
        : [tk] "=&s"(tk), [tmp] "=&s"(tmp), [xk] "+s"(xk), [out] "+s"(out), [m] "+s"(m), [p] "+v"(p)
        : [tv] "v"(t[k]), [lim] "s"(lim)
        : "scc", "m0");
    pos[k] = p;
    return tk;
  }
  __device__ uint32_t dist(int k, int l) const { return (uint32_t)__builtin_amdgcn_readlane((int)d[k], l); }
  template <class F>
  __device__ void each_literal(const uint64_t (&lm)[kRoundK], int lane, F &&f) const {
#pragma unroll
    for (int k = 0; k < kRoundK; ++k)
      if ((lm[k] >> lane) & 1) f(64 * k + lane, pos[k], (uint8_t)(t[k] >> 24));
  }
};
#endif

// Rounds from bit P until a token needs the scalar loop (returned true) or the round limits end
// them (false: another round). Advances P and w; flushes completed output chunks.
template <int NL>
INF_INL bool inflate_round(InfShared &S, RoundToks<NL> &R, uint32_t &P, int &w, int &flushed, uint32_t nbits,
                          int cap, uint8_t *dst, int lane, uint64_t *prof) {
  constexpr int M = kOutRing - 1;
  uint64_t t0 = INF_T();
  R.fill(S, P, nbits, lane);
  INF_ACC(0, t0);
#if defined(INF_PROF) && defined(__HIP_DEVICE_COMPILE__)
  prof[4] += 1;
#endif
  t0 = INF_T();
  uint64_t lm[kRoundK];
  int nm = 0, out = 0, x = 0, maxd = 0;
  bool need_scalar = false, stop = false;
  // output this round may produce: kRoundOut (+ one match), never past the block's ISIZE
  const int room = cap - w, lim = room < kRoundOut ? room : kRoundOut;
#pragma unroll
  for (int k = 0; k < kRoundK; ++k) {
    lm[k] = 0;
    if (stop) continue;
    int xk = x - 64 * k;
    uint64_t m = 0;
    for (;;) {
      const uint32_t t = R.chain(k, xk, out, lim, m);
      if (!(t & (kTokStop | kTokMatch))) break;   // offset 64 or the output limit
      const int ol = (int)((t >> 6) & 511);
      const int dv = (int)R.dist(k, xk);
      // a token for the scalar loop (a code the tables cannot finish, end of block, an invalid
      // code, bits past the payload, a bad distance, output past ISIZE), or a full record list
      if ((t & kTokStop) || dv > w + out || out + ol > room || nm == kRoundMaxM) {
        need_scalar = (t & kTokStop) || dv > w + out || out + ol > room;
        stop = true;
        break;
      }
      if (lane == 0) S.mrec[nm] = make_int4(xk + 64 * k, out, ol, dv);
      ++nm;
      if (dv <= kNear && dv > maxd) maxd = dv;   // (far matches read global memory)
      out += ol;
      xk += (int)(t & 63);
    }
    lm[k] = m;
    x = xk + 64 * k;
    if (out >= lim) stop = true;
  }
  INF_WAVE_ORDER();   // the match records are read by every lane
  INF_ACC(1, t0);
  t0 = INF_T();
#if defined(INF_STATS) && !defined(__HIP_DEVICE_COMPILE__)
  inf_stats[0]++; inf_stats[1] += out; inf_stats[2] += nm; inf_stats[3] += need_scalar; inf_stats[4] += x;
#endif
  if (nm == 0 || maxd + out <= kOutRing) {
    // no match reads a ring slot a later literal of the round overwrites: literals first
    R.each_literal(lm, lane, [&](int, int pos, uint8_t v) { S.out[(w + pos) & M] = v; });
    for (int j = 0; j < nm; ++j) {
      const int4 mr = S.mrec[j];
      copy_match<NL>(S, dst, w + mr.y, mr.z, mr.w, lane);
    }
  } else {   // stream order: the literals before each match, then the match
    int xprev = -1;
    for (int j = 0; j <= nm; ++j) {
      const int4 mr = j < nm ? S.mrec[j] : make_int4(1 << 30, 0, 0, 0);
      R.each_literal(lm, lane, [&](int xl, int pos, uint8_t v) {
        if (xl > xprev && xl < mr.x) S.out[(w + pos) & M] = v;
      });
      if (j < nm) copy_match<NL>(S, dst, w + mr.y, mr.z, mr.w, lane);
      xprev = mr.x;
    }
  }
  w += out;
  P += (uint32_t)x;
  if (w - flushed >= kFlush) {
    const int to = w & ~(kFlush - 1);
    flush_out<NL>(S.out, dst, flushed, to, lane);
    flushed = to;
  }
  INF_ACC(2, t0);
  return need_scalar || x == 0;
}

// Decode one block's payload (n bytes at g) into dst (cap = the block's ISIZE bytes, never more);
// returns the bytes decoded or -status. Wave-uniform: all 64 lanes run it together.
template <int NL, bool ROUNDS = true>
INF_FN int inflate_wave(InfShared &S, const uint8_t *g, int n, uint8_t *dst, int cap, int lane) {
  // the block's arguments are wave-uniform: say so (an out-of-line call passes them in vector
  // registers, and every branch on them would run under exec masks)
  n = uni(n);
  cap = uni(cap);
  g = reinterpret_cast<const uint8_t *>(uni64(reinterpret_cast<uint64_t>(g)));
  dst = reinterpret_cast<uint8_t *>(uni64(reinterpret_cast<uint64_t>(dst)));
  Bits<NL> b{g, S.ring, n, 0, 0, lane, 0ull, 0};
  constexpr int M = kOutRing - 1;
  int w = 0, flushed = 0;
  uint64_t prof[6] = {0, 0, 0, 0, 0, 0};
  const uint64_t t_block = INF_T();
  for (;;) {
    if (!b.need(3)) return -kInfOverrun;
    const int final_ = (int)b.take(1);
    const int type = (int)b.take(2);
    if (type == 0) {   // stored: byte-aligned LEN, NLEN, LEN bytes
      b.take(b.cnt & 7);
      if (!b.need(32)) return -kInfOverrun;
      const int ln = (int)b.take(16), nl = (int)b.take(16);
      if ((ln ^ 0xFFFF) != nl) return -kInfBadBlock;
      if (w + ln > cap) return -kInfSize;
      int k = 0;
      for (; k < ln && b.cnt >= 8; ++k, ++w) {   // bytes already in the bit buffer
        const uint8_t v = (uint8_t)b.take(8);
        if (lane == 0) S.out[w & M] = v;
      }
      int rest = ln - k;
      if (b.pos + rest > n) return -kInfOverrun;
      while (rest > 0) {   // the rest from global memory, a flush chunk at a time
        const int piece = rest < kFlush ? rest : kFlush;
        for (int j0 = 0; j0 < piece; j0 += NL) {
          const int j = j0 + lane;
          if (j < piece) S.out[(w + j) & M] = g[b.pos + j];
        }
        w += piece;
        b.pos += piece;
        rest -= piece;
        if (w - flushed >= kFlush) {
          const int to = w & ~(kFlush - 1);
          flush_out<NL>(S.out, dst, flushed, to, lane);
          flushed = to;
        }
      }
      if (b.filled < b.pos) b.filled = b.pos;
    } else if (type == 1 || type == 2) {
      if (type == 1) {   // fixed codes
        for (int s = 0; s < 288; ++s) S.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
        for (int s = 0; s < 30; ++s) S.lens[288 + s] = 5;
        huff_build<NL>(S.lit, S.lens, 288, lane);
        huff_build<NL>(S.dist, S.lens + 288, 30, lane);
      } else {           // dynamic codes
        if (!b.need(14)) return -kInfOverrun;
        const int nlen = (int)b.take(5) + 257, ndist = (int)b.take(5) + 1, ncode = (int)b.take(4) + 4;
        if (nlen > 286 || ndist > 30) return -kInfBadBlock;
        for (int i = 0; i < 19; ++i) S.lens[i] = 0;
        for (int i = 0; i < ncode; ++i) {
          if (!b.need(3)) return -kInfOverrun;
          S.lens[kClOrder[i]] = (uint16_t)b.take(3);
        }
        if (!huff_build<NL>(S.dist, S.lens, 19, lane)) return -kInfBadCode;   // (the code-length code, in dist)
        // the literal/length and distance code lengths, after the code-length code's 19 slots
        uint16_t *ll = S.lens + 19;
        int k = 0;
        while (k < nlen + ndist) {
          const int sym = huff_decode(S.dist, b);
          if (sym < 0) return -kInfBadCode;
          if (sym < 16) {
            ll[k++] = (uint16_t)sym;
            continue;
          }
          int rep, val = 0;
          if (sym == 16) {
            if (k == 0 || !b.need(2)) return -kInfBadCode;
            val = uni(ll[k - 1]);
            rep = 3 + (int)b.take(2);
          } else if (sym == 17) {
            if (!b.need(3)) return -kInfOverrun;
            rep = 3 + (int)b.take(3);
          } else {
            if (!b.need(7)) return -kInfOverrun;
            rep = 11 + (int)b.take(7);
          }
          if (k + rep > nlen + ndist) return -kInfBadCode;
          while (rep--) ll[k++] = (uint16_t)val;
        }
        if (uni(ll[256]) == 0) return -kInfBadCode;   // no end-of-block code
        if (!huff_build<NL>(S.lit, ll, nlen, lane)) return -kInfBadCode;
        if (!huff_build<NL>(S.dist, ll + nlen, ndist, lane)) return -kInfBadCode;
      }
      // the symbol loop: errors leave it through `err` (a single exit, and only uniform inner
      // loops, keep the control flow and so the state scalar)
      const uint16_t *lfast = S.lit.fast, *dfast = S.dist.fast;
      int err = 0;
      for (;;) {
        b.uniform();
        w = uni(w);
        flushed = uni(flushed);
        if (ROUNDS) {   // token rounds up to the next token the scalar code below must decode
          uint32_t P = (uint32_t)(8 * b.pos - b.cnt);
          for (;;) {
            b.pos = (int)(P >> 3);
            b.top_up();
            RoundToks<NL> R;
            const bool sc = inflate_round<NL>(S, R, P, w, flushed, 8u * (uint32_t)n, cap, dst, lane, prof);
            P = (uint32_t)uni((int)P);
            w = uni(w);
            flushed = uni(flushed);
            if (sc) break;
          }
          // the bit reader at P again
          b.pos = (int)(P >> 3);
          b.buf = 0;
          b.cnt = 0;
          b.top_up();
          b.refill();
          b.take((int)(P & 7));
          b.uniform();
        }
        if (b.cnt < 15) b.refill();
        int e = uni(lfast[b.buf & kFastMask]);
        int l = e >> 9;
#if defined(INF_STATS) && !defined(__HIP_DEVICE_COMPILE__)
        if (ROUNDS) {
          if (l == 0) inf_stats[5]++;
          else if ((e & 511) == 256) inf_stats[6]++;
          else inf_stats[7]++;
        }
#endif
        if (l == 0 || l > b.cnt) {
          e = uni(huff_slow(S.lit, b.buf, b.cnt));
          if (e < 0) {
            err = kInfBadCode;
            break;
          }
          l = e >> 16;
        }
        const int sym = e & 511;
        b.buf >>= l;
        b.cnt -= l;
        if (sym < 256) {
          if (w >= cap) {
            err = kInfSize;
            break;
          }
#ifdef INF_MARK
          __asm__ volatile("; MARK_LITERAL");
#endif
          if (lane == 0) S.out[w & M] = (uint8_t)sym;
          ++w;
          // a second literal in the same iteration when its code is in the table and the bits
          // are there (literal runs: half the loop overhead)
          const int e2 = uni(lfast[b.buf & kFastMask]);
          const int l2 = e2 >> 9, s2 = e2 & 511;
          if (l2 && l2 <= b.cnt && s2 < 256 && w < cap) {
            if (lane == 0) S.out[w & M] = (uint8_t)s2;
            ++w;
            b.buf >>= l2;
            b.cnt -= l2;
          }
        } else {
          if (sym == 256) break;
          const int li = sym - 257;
          if (li >= 29) {
            err = kInfBadCode;
            break;
          }
          if (b.cnt < 33) b.refill();   // length extra (<= 5) + distance code (<= 15) + extra (<= 13)
          // RFC 1951 3.2.5 length codes: base 3 + li below 8, then 4..7 << extra (+ 3); 258 alone
          const int le = li < 8 || li == 28 ? 0 : (li - 4) >> 2;
          const int lb = li < 8 ? 3 + li : li == 28 ? 258 : ((4 + (li & 3)) << le) + 3;
          int d = uni(dfast[(b.buf >> le) & kFastMask]);
          int dl = d >> 9;
          if (b.cnt < le) {
            err = kInfOverrun;
            break;
          }
          const int len = lb + (int)(b.buf & ((1u << le) - 1));
          b.buf >>= le;
          b.cnt -= le;
          if (dl == 0 || dl > b.cnt) {
            d = uni(huff_slow(S.dist, b.buf, b.cnt));
            if (d < 0) {
              err = kInfBadCode;
              break;
            }
            dl = d >> 16;
          }
          const int ds = d & 511;
          b.buf >>= dl;
          b.cnt -= dl;
          // distance codes: base 1 + ds below 4, then 2..3 << extra (+ 1)
          const int de = ds < 4 ? 0 : (ds - 2) >> 1;
          if (ds >= 30 || b.cnt < de) {
            err = ds >= 30 ? kInfBadCode : kInfOverrun;
            break;
          }
          const int dist = (ds < 4 ? 1 + ds : ((2 + (ds & 1)) << de) + 1) + (int)(b.buf & ((1u << de) - 1));
          b.buf >>= de;
          b.cnt -= de;
          if (dist > w || w + len > cap) {
            err = dist > w ? kInfBadDist : kInfSize;
            break;
          }
          copy_match<NL>(S, dst, w, len, dist, lane);
          w += len;
        }
        if (w - flushed >= kFlush) {   // (at most kFlush + 257 bytes are ever unflushed)
          const int to = w & ~(kFlush - 1);
          flush_out<NL>(S.out, dst, flushed, to, lane);
          flushed = to;
        }
      }
      if (err) return -err;
    } else {
      return -kInfBadBlock;
    }
    if (final_) {
      flush_out<NL>(S.out, dst, flushed, w, lane);
#if defined(INF_PROF) && defined(__HIP_DEVICE_COMPILE__)
      prof[3] += INF_T() - t_block;
      if (lane == 0)
        for (int i = 0; i < 6; ++i) atomicAdd(&g_inf_prof[i], (unsigned long long)prof[i]);
#endif
      return w;
    }
  }
}

// Block i: payload comp[in_off[i], + in_len[i]) -> out[out_off[i], + out_len[i]) (its ISIZE);
// status[i] = 0 or the failure (a length other than ISIZE included).
template <bool ROUNDS>
__global__ void __launch_bounds__(kInfThreads) k_inflate(const uint8_t *__restrict__ comp, int64_t comp_len,
                                                         const int64_t *__restrict__ in_off,
                                                         const int32_t *__restrict__ in_len,
                                                         const int64_t *__restrict__ out_off,
                                                         const int32_t *__restrict__ out_len, int64_t n_blocks,
                                                         uint8_t *__restrict__ out, int64_t out_total,
                                                         int32_t *__restrict__ status) {
  __shared__ InfShared S;
  const int t = threadIdx.x;
  for (int64_t i = blockIdx.x; i < n_blocks; i += gridDim.x) {
    const int64_t io = in_off[i], oo = out_off[i];
    const int il = in_len[i], ol = out_len[i];
    const bool ok = io >= 0 && il >= 0 && io + il <= comp_len && oo >= 0 && ol >= 0 && ol <= kWin &&
                    oo + ol <= out_total;
    if (!ok) {
      if (t == 0) status[i] = kInfSize;
      continue;
    }
    const int r = inflate_wave<kInfThreads, ROUNDS>(S, comp + io, il, out + oo, ol, t);
    if (t == 0) status[i] = r < 0 ? -r : (r == ol ? kInfOk : kInfSize);
    __syncthreads();   // (S is reused by the next block)
  }
}

}  // namespace

struct ganon_inflate_state {
  uint8_t *comp = nullptr, *out = nullptr;
  int64_t *in_off = nullptr, *out_off = nullptr;
  int32_t *in_len = nullptr, *out_len = nullptr, *status = nullptr;
  size_t comp_cap = 0, out_cap = 0, blk_cap = 0;
  int64_t last_out = -1;                // out_total of the last successful call (ganon_inflate_device_output)
  hipStream_t copy = nullptr;           // copies of a chunked call (the kernels run on ctx->stream)
  std::vector<hipEvent_t> ev;           // two per chunk
};

namespace {

template <typename T>
int grow_dev(ganon_ctx *ctx, T **p, size_t &cap, size_t need) {
  if (*p && cap >= need) return GANON_OK;
  if (*p) {
    ganon_detail::sync_stream(ctx->stream);
    hipFree(*p);
    *p = nullptr;
  }
  const size_t n = std::max(need, cap + cap / 2);
  if (hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
    *p = nullptr;
    cap = 0;
    return fail(ctx, GANON_E_NOMEM, "hipMalloc for the inflate buffers failed");
  }
  cap = n;
  return GANON_OK;
}

}  // namespace

// ganon_inflate; out == nullptr keeps the output in device memory only (ganon_inflate_device_output:
// the device region decode of ganon_bam.hip walks it there)
int ganon_inflate_impl(ganon_ctx *ctx, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                       const int32_t *in_len, const int64_t *out_off, const int32_t *out_len, int64_t n_blocks,
                       uint8_t *out, int64_t out_total, int64_t *first_bad) {
  if (!ctx) return GANON_E_ARG;
  if (first_bad) *first_bad = -1;
  if (n_blocks < 0 || comp_len < 0 || out_total < 0 || (n_blocks && (!comp || !in_off || !in_len || !out_off ||
                                                                      !out_len)))
    return fail(ctx, GANON_E_ARG, "ganon_inflate: bad arguments");
  if (!n_blocks) return GANON_OK;
  // every block inside both buffers before any span is computed from them: the host copies of a
  // chunk are sized from its first and last block only
  for (int64_t i = 0; i < n_blocks; ++i)
    if (in_off[i] < 0 || in_len[i] < 0 || out_off[i] < 0 || out_len[i] < 0 || in_off[i] + in_len[i] > comp_len ||
        out_off[i] + out_len[i] > out_total) {
      if (first_bad) *first_bad = i;
      return fail(ctx, GANON_E_ARG, "ganon_inflate: block %lld lies outside the buffers", (long long)i);
    }
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipSetDevice failed");
  if (!ctx->inflate) ctx->inflate = new ganon_inflate_state();
  ganon_inflate_state *st = ctx->inflate;
  const size_t nb = (size_t)n_blocks;
  size_t cap_blk = st->blk_cap;
  int rc;
  st->last_out = -1;
  if ((rc = grow_dev(ctx, &st->comp, st->comp_cap, (size_t)comp_len)) ||
      (rc = grow_dev(ctx, &st->out, st->out_cap, (size_t)out_total)))
    return rc;
  {
    size_t c1 = cap_blk, c2 = cap_blk, c3 = cap_blk, c4 = cap_blk, c5 = cap_blk;
    if ((rc = grow_dev(ctx, &st->in_off, c1, nb)) || (rc = grow_dev(ctx, &st->out_off, c2, nb)) ||
        (rc = grow_dev(ctx, &st->in_len, c3, nb)) || (rc = grow_dev(ctx, &st->out_len, c4, nb)) ||
        (rc = grow_dev(ctx, &st->status, c5, nb)))
      return rc;
    st->blk_cap = c1;
  }
  hipStream_t s = ctx->stream;
  if (ctx->profiling) {   // a profiled call: ganon_last_kernel_times reports k_inflate alone
    for (auto &r : ctx->recs) {
      ctx->pool.push_back(r.e0);
      ctx->pool.push_back(r.e1);
    }
    ctx->recs.clear();
  }
  // Chunks of kChunk blocks (about one round of decoders on the chip: 10 per CU) when the blocks lie in file
  // order: the payload of chunk c + 1 goes up and the output of chunk c - 1 comes down on a copy
  // stream while chunk c decodes; otherwise one chunk.
  constexpr int64_t kChunk = 2560;
  bool ordered = true;
  for (size_t i = 1; i < nb && ordered; ++i)
    ordered = in_off[i] >= in_off[i - 1] + in_len[i - 1] && out_off[i] >= out_off[i - 1] + out_len[i - 1];
  const int64_t n_chunks = ordered ? (n_blocks + kChunk - 1) / kChunk : 1;
  auto span_in = [&](int64_t b0, int64_t b1, int64_t &lo, int64_t &hi) {
    lo = ordered ? in_off[b0] : 0;
    hi = ordered ? in_off[b1 - 1] + in_len[b1 - 1] : comp_len;
  };
  auto span_out = [&](int64_t b0, int64_t b1, int64_t &lo, int64_t &hi) {
    lo = ordered ? out_off[b0] : 0;
    hi = ordered ? out_off[b1 - 1] + out_len[b1 - 1] : out_total;
  };
  if (ordered && (in_off[0] < 0 || in_off[nb - 1] + in_len[nb - 1] > comp_len || out_off[0] < 0 ||
                  out_off[nb - 1] + out_len[nb - 1] > out_total))
    return fail(ctx, GANON_E_ARG, "ganon_inflate: block ranges outside the buffers");
  if (!st->copy && hipStreamCreateWithFlags(&st->copy, hipStreamNonBlocking) != hipSuccess)
    return fail(ctx, GANON_E_DEVICE, "ganon_inflate: stream creation failed");
  while ((int64_t)st->ev.size() < 2 * n_chunks) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      return fail(ctx, GANON_E_DEVICE, "ganon_inflate: event creation failed");
    st->ev.push_back(e);
  }
  hipStream_t cs = st->copy;
  bool okc = hipMemcpyAsync(st->in_off, in_off, nb * 8, hipMemcpyHostToDevice, cs) == hipSuccess &&
             hipMemcpyAsync(st->out_off, out_off, nb * 8, hipMemcpyHostToDevice, cs) == hipSuccess &&
             hipMemcpyAsync(st->in_len, in_len, nb * 4, hipMemcpyHostToDevice, cs) == hipSuccess &&
             hipMemcpyAsync(st->out_len, out_len, nb * 4, hipMemcpyHostToDevice, cs) == hipSuccess;
  auto d2h = [&](int64_t c) {
    const int64_t b0 = c * kChunk, b1 = std::min(n_blocks, b0 + kChunk);
    int64_t lo, hi;
    span_out(b0, b1, lo, hi);
    return hipStreamWaitEvent(cs, st->ev[2 * c + 1], 0) == hipSuccess &&
           (!out || hi <= lo ||
            hipMemcpyAsync(out + lo, st->out + lo, (size_t)(hi - lo), hipMemcpyDeviceToHost, cs) == hipSuccess);
  };
  for (int64_t c = 0; c < n_chunks && okc; ++c) {
    const int64_t b0 = c * kChunk, b1 = std::min(n_blocks, b0 + kChunk);
    int64_t lo, hi;
    span_in(b0, b1, lo, hi);
    okc = (hi <= lo || hipMemcpyAsync(st->comp + lo, comp + lo, (size_t)(hi - lo), hipMemcpyHostToDevice, cs) == hipSuccess) &&
          hipEventRecord(st->ev[2 * c], cs) == hipSuccess && hipStreamWaitEvent(s, st->ev[2 * c], 0) == hipSuccess;
    if (!okc) break;
    {
      ganon_detail::KernelScope ks(ctx, "k_inflate");
      const unsigned grid = (unsigned)std::min<int64_t>(b1 - b0, 1 << 16);
      // (GANON_INFLATE_ROUNDS=0: the scalar symbol loop alone, A/B)
      static const bool rounds = !(std::getenv("GANON_INFLATE_ROUNDS") && std::getenv("GANON_INFLATE_ROUNDS")[0] == '0');
      hipLaunchKernelGGL(rounds ? k_inflate<true> : k_inflate<false>, dim3(grid), dim3(kInfThreads), 0, s, st->comp, comp_len, st->in_off + b0,
                         st->in_len + b0, st->out_off + b0, st->out_len + b0, b1 - b0, st->out, out_total,
                         st->status + b0);
    }
    if ((rc = check_launch(ctx, "k_inflate"))) {
      // copies from / into the caller's buffers may still be queued: they end before it gets them back
      ganon_detail::sync_stream(cs);
      ganon_detail::sync_stream(s);
      return rc;
    }
    okc = hipEventRecord(st->ev[2 * c + 1], s) == hipSuccess && (c == 0 || d2h(c - 1));
  }
  std::vector<int32_t> stat(nb);
  okc = okc && d2h(n_chunks - 1) &&
        ganon_detail::readback(stat.data(), st->status, nb * 4, cs) == hipSuccess &&
        ganon_detail::sync_stream(cs) == hipSuccess;
  if (!okc) {
    ganon_detail::sync_stream(cs);
    ganon_detail::sync_stream(s);
    return fail(ctx, GANON_E_DEVICE, "ganon_inflate: copy failed");
  }
  if ((rc = ganon_batch_sync(ctx))) return rc;   // (collects the kernel times when profiling)
  for (size_t i = 0; i < nb; ++i)
    if (stat[i]) {
      if (first_bad) *first_bad = (int64_t)i;
      return fail(ctx, GANON_E_ARG, "BGZF block %lld: invalid DEFLATE stream (code %d)", (long long)i, stat[i]);
    }
  st->last_out = out_total;
  return GANON_OK;
}

GANON_API int ganon_inflate(ganon_ctx *ctx, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                            const int32_t *in_len, const int64_t *out_off, const int32_t *out_len, int64_t n_blocks,
                            uint8_t *out, int64_t out_total, int64_t *first_bad) {
  if (ctx && n_blocks > 0 && !out) return fail(ctx, GANON_E_ARG, "ganon_inflate: bad arguments");
  return ganon_inflate_impl(ctx, comp, comp_len, in_off, in_len, out_off, out_len, n_blocks, out, out_total, first_bad);
}

GANON_API int ganon_inflate_device_output(ganon_ctx *ctx, const uint8_t **out, int64_t *bytes) {
  if (!ctx || !out || !bytes) return fail(ctx, GANON_E_ARG, "ganon_inflate_device_output: bad arguments");
  if (!ctx->inflate || ctx->inflate->last_out < 0)
    return fail(ctx, GANON_E_ARG, "ganon_inflate_device_output: no successful inflate on this context");
  *out = ctx->inflate->out;
  *bytes = ctx->inflate->last_out;
  return GANON_OK;
}

GANON_API int ganon_inflate_hostcb(void *ctx, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                                   const int32_t *in_len, const int64_t *out_off, const int32_t *out_len,
                                   int64_t n_blocks, uint8_t *out, int64_t out_total) {
  return ganon_inflate(static_cast<ganon_ctx *>(ctx), comp, comp_len, in_off, in_len, out_off, out_len, n_blocks, out,
                       out_total, nullptr);
}

void ganon_inflate_free(ganon_inflate_state *st) {
  if (!st) return;
  if (st->copy) {
    ganon_detail::sync_stream(st->copy);
    hipStreamDestroy(st->copy);
  }
  for (hipEvent_t e : st->ev) hipEventDestroy(e);
  for (void *p : {(void *)st->comp, (void *)st->out, (void *)st->in_off, (void *)st->out_off, (void *)st->in_len,
                  (void *)st->out_len, (void *)st->status})
    if (p) hipFree(p);
  delete st;
}

#if defined(INF_PROF)
// (tuning build only) the summed round cycles since the last call: fill, chain, emit, block total,
// rounds; then zeroed
GANON_API int ganon_inflate_prof_read(unsigned long long *out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_inf_prof), sizeof(unsigned long long) * 6) != hipSuccess) return -1;
  unsigned long long z[6] = {0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_inf_prof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
