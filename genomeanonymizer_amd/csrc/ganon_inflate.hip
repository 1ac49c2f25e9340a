// ganon_inflate.hip — BGZF block inflate on MI355X (gfx950), part of libganon_hip.so; C ABI in
// include/ganon.h (ganon_inflate). SURVEY §8(f)4: the input decode offload.
//
// The host BAM reader (ganon_host.cpp) cuts a window of the compressed file into BGZF blocks —
// independent raw DEFLATE streams (RFC 1951) of at most 64 KiB of output each — and hands their
// payloads here instead of to zlib on its threads (ganon_bam_reader_set_inflater).
//
// One 64-lane workgroup per block, and the wave decodes it as ONE decoder: Huffman decoding is a
// serial bit stream, so every lane runs the same symbol loop on the same (wave-uniform, mostly
// scalar) state, and the lanes split only the byte work — the payload is pulled into an 8 KiB LDS
// ring 4 KiB at a time, an LZ77 match of length L is copied by all 64 lanes at once (periodic
// source index w - dist + (j mod dist), so even an overlapping match has no intra-copy dependence)
// and a stored block is copied straight from global memory. The 64 KiB output window stays in LDS
// and is written out coalesced at the end. 76 KiB of LDS: two blocks decode per CU, 512 on the
// chip. Stored, fixed- and dynamic-Huffman blocks; canonical codes through a 9-bit lookup table
// with a bit-by-bit canonical walk for longer codes. Every read and write is range-checked: a
// malformed stream sets the block's status and stops it, never faults.
// Written from RFC 1951 and the BGZF section of the SAM specification.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "ganon_ctx.h"

namespace {

using ganon_detail::check_launch;
using ganon_detail::fail;

constexpr int kInfThreads = 64;
constexpr int kWin = 65536;          // BGZF: at most 64 KiB of output and of payload per block
constexpr int kRing = 8192;          // payload ring (LDS), refilled kRing/2 bytes at a time
constexpr int kRingHalf = kRing / 2;
constexpr int kFastBits = 9;         // Huffman lookup table width

// Canonical Huffman code: counts per length, symbols by (length, value), a kFastBits lookup table
// of (symbol | length << 9) for codes of at most kFastBits bits (0: longer code or none).
struct Huff {
  uint16_t count[16];
  uint16_t symbol[288];
  uint16_t fast[1 << kFastBits];
};

struct InfShared {
  uint8_t out[kWin];
  uint8_t ring[kRing];
  Huff lit, dist;
  uint16_t lens[19 + 288 + 32];   // code-length code, then literal/length + distance lengths
};

constexpr uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99,
                                   115, 131, 163, 195, 227, 258};
constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                    1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11,
                                    12, 12, 13, 13};
constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum { kInfOk = 0, kInfBadBlock = 1, kInfBadCode = 2, kInfOverrun = 3, kInfBadDist = 4, kInfSize = 5 };

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// LSB-first bit reader. Payload bytes [filled - kRing, filled) are in the LDS ring (index & mask);
// top_up (wave-uniform: every lane calls it together) keeps at least kRingHalf bytes ahead of pos.
struct Bits {
  const uint8_t *g;   // the block's payload in global memory
  uint8_t *ring;
  int n, pos, filled, lane;
  uint64_t buf;
  int cnt;
  __device__ void top_up() {
    if (filled < n && filled - pos < kRingHalf) {
      __syncthreads();   // earlier ring reads are done before their slots are overwritten
      const int e = min(filled + kRingHalf, n);
      for (int k = filled + lane; k < e; k += kInfThreads) ring[k & (kRing - 1)] = g[k];
      filled = e;
      __syncthreads();
    }
  }
  __device__ void refill() {
    if (cnt > 56) return;
    top_up();
    while (cnt <= 56 && pos < n) {
      buf |= (uint64_t)(uint32_t)uni(ring[pos & (kRing - 1)]) << cnt;
      ++pos;
      cnt += 8;
    }
  }
  __device__ bool need(int k) {
    if (cnt < k) refill();
    return cnt >= k;
  }
  __device__ uint32_t take(int k) {   // (need(k) checked by the caller)
    const uint32_t v = k ? (uint32_t)(buf & ((1ull << k) - 1)) : 0u;
    buf >>= k;
    cnt -= k;
    return v;
  }
};

__device__ __forceinline__ uint32_t rev_bits(uint32_t v, int n) { return __builtin_bitreverse32(v) >> (32 - n); }

// Build h from n code lengths; false on an over-subscribed code (an incomplete one is allowed:
// RFC 1951 permits a single distance code). Wave-uniform: every lane writes the same values.
__device__ bool huff_build(Huff &h, const uint16_t *len, int n) {
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
  for (int i = 0; i < (1 << kFastBits); ++i) h.fast[i] = 0;
  // canonical codes of lengths <= kFastBits into the table (bit-reversed: the stream's bit order)
  int code = 0, idx = 0;
  for (int l = 1; l <= kFastBits; ++l) {
    for (uint32_t k = 0; k < cnt[l]; ++k, ++idx, ++code) {
      const uint32_t r = rev_bits((uint32_t)code, l);
      const uint16_t e = (uint16_t)(uni(h.symbol[idx]) | (l << 9));
      for (uint32_t f = r; f < (1u << kFastBits); f += 1u << l) h.fast[f] = e;
    }
    code <<= 1;
  }
  return true;
}

// One symbol; -1 on an invalid code or a stream that ends inside it.
__device__ int huff_decode(const Huff &h, Bits &b) {
  b.refill();
  if (b.cnt >= kFastBits || b.pos >= b.n) {
    const int e = uni(h.fast[b.buf & ((1u << kFastBits) - 1)]);
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

// Decode one block's payload (n bytes at g) into S.out; returns the bytes written or -status.
// Wave-uniform: all 64 lanes run it together.
__device__ int inflate_wave(InfShared &S, const uint8_t *g, int n, int lane) {
  Bits b{g, S.ring, n, 0, 0, lane, 0ull, 0};
  int w = 0;
  for (;;) {
    if (!b.need(3)) return -kInfOverrun;
    const int final_ = (int)b.take(1);
    const int type = (int)b.take(2);
    if (type == 0) {   // stored: byte-aligned LEN, NLEN, LEN bytes
      b.take(b.cnt & 7);
      if (!b.need(32)) return -kInfOverrun;
      const int ln = (int)b.take(16), nl = (int)b.take(16);
      if ((ln ^ 0xFFFF) != nl) return -kInfBadBlock;
      if (w + ln > kWin) return -kInfSize;
      int k = 0;
      for (; k < ln && b.cnt >= 8; ++k, ++w) {   // bytes already in the bit buffer
        const uint8_t v = (uint8_t)b.take(8);
        if (lane == 0) S.out[w] = v;
      }
      const int rest = ln - k;
      if (b.pos + rest > n) return -kInfOverrun;
      for (int j = lane; j < rest; j += kInfThreads) S.out[w + j] = g[b.pos + j];
      w += rest;
      b.pos += rest;
      if (b.filled < b.pos) b.filled = b.pos;
    } else if (type == 1 || type == 2) {
      if (type == 1) {   // fixed codes
        for (int s = 0; s < 288; ++s) S.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
        for (int s = 0; s < 30; ++s) S.lens[288 + s] = 5;
        huff_build(S.lit, S.lens, 288);
        huff_build(S.dist, S.lens + 288, 30);
      } else {           // dynamic codes
        if (!b.need(14)) return -kInfOverrun;
        const int nlen = (int)b.take(5) + 257, ndist = (int)b.take(5) + 1, ncode = (int)b.take(4) + 4;
        if (nlen > 286 || ndist > 30) return -kInfBadBlock;
        for (int i = 0; i < 19; ++i) S.lens[i] = 0;
        for (int i = 0; i < ncode; ++i) {
          if (!b.need(3)) return -kInfOverrun;
          S.lens[kClOrder[i]] = (uint16_t)b.take(3);
        }
        if (!huff_build(S.dist, S.lens, 19)) return -kInfBadCode;   // (the code-length code, in dist)
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
        if (!huff_build(S.lit, ll, nlen)) return -kInfBadCode;
        if (!huff_build(S.dist, ll + nlen, ndist)) return -kInfBadCode;
      }
      for (;;) {
        const int sym = huff_decode(S.lit, b);
        if (sym < 0) return -kInfBadCode;
        if (sym < 256) {
          if (w >= kWin) return -kInfSize;
          if (lane == 0) S.out[w] = (uint8_t)sym;
          ++w;
          continue;
        }
        if (sym == 256) break;
        const int li = sym - 257;
        if (li >= 29) return -kInfBadCode;
        if (!b.need(kLenExtra[li])) return -kInfOverrun;
        const int len = kLenBase[li] + (int)b.take(kLenExtra[li]);
        const int ds = huff_decode(S.dist, b);
        if (ds < 0 || ds >= 30) return -kInfBadCode;
        if (!b.need(kDistExtra[ds])) return -kInfOverrun;
        const int dist = kDistBase[ds] + (int)b.take(kDistExtra[ds]);
        if (dist > w) return -kInfBadDist;
        if (w + len > kWin) return -kInfSize;
        __syncthreads();   // lane 0's literals and the last copy are visible to every lane
        const uint8_t *src = S.out + (w - dist);
        if (dist >= len) {
          for (int j = lane; j < len; j += kInfThreads) S.out[w + j] = src[j];
        } else {           // overlapping: out[w + j] = out[w - dist + j mod dist]
          int r = lane % dist;
          const int step = kInfThreads % dist;
          for (int j = lane; j < len; j += kInfThreads) {
            S.out[w + j] = src[r];
            r += step;
            if (r >= dist) r -= dist;
          }
        }
        w += len;
      }
    } else {
      return -kInfBadBlock;
    }
    if (final_) return w;
  }
}

// Block i: payload comp[in_off[i], + in_len[i]) -> out[out_off[i], + out_len[i]) (its ISIZE);
// status[i] = 0 or the failure (a length other than ISIZE included).
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
    const bool ok = io >= 0 && il >= 0 && il <= kWin && io + il <= comp_len && oo >= 0 && ol >= 0 && ol <= kWin &&
                    oo + ol <= out_total;
    if (!ok) {
      if (t == 0) status[i] = kInfSize;
      continue;
    }
    const int r = inflate_wave(S, comp + io, il, t);
    if (t == 0) status[i] = r < 0 ? -r : (r == ol ? kInfOk : kInfSize);
    __syncthreads();
    if (r == ol) {
      uint8_t *o = out + oo;
      int k0 = 0;
      if ((oo & 3) == 0) {   // aligned: dword stores
        const int n4 = ol >> 2;
        for (int k = t; k < n4; k += kInfThreads)
          reinterpret_cast<uint32_t *>(o)[k] = reinterpret_cast<const uint32_t *>(S.out)[k];
        k0 = n4 << 2;
      }
      for (int k = k0 + t; k < ol; k += kInfThreads) o[k] = S.out[k];
    }
    __syncthreads();   // (S is reused by the next block)
  }
}

}  // namespace

struct ganon_inflate_state {
  uint8_t *comp = nullptr, *out = nullptr;
  int64_t *in_off = nullptr, *out_off = nullptr;
  int32_t *in_len = nullptr, *out_len = nullptr, *status = nullptr;
  size_t comp_cap = 0, out_cap = 0, blk_cap = 0;
};

namespace {

template <typename T>
int grow_dev(ganon_ctx *ctx, T **p, size_t &cap, size_t need) {
  if (*p && cap >= need) return GANON_OK;
  if (*p) {
    hipStreamSynchronize(ctx->stream);
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

GANON_API int ganon_inflate(ganon_ctx *ctx, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                            const int32_t *in_len, const int64_t *out_off, const int32_t *out_len, int64_t n_blocks,
                            uint8_t *out, int64_t out_total, int64_t *first_bad) {
  if (!ctx) return GANON_E_ARG;
  if (first_bad) *first_bad = -1;
  if (n_blocks < 0 || comp_len < 0 || out_total < 0 || (n_blocks && (!comp || !in_off || !in_len || !out_off ||
                                                                      !out_len || !out)))
    return fail(ctx, GANON_E_ARG, "ganon_inflate: bad arguments");
  if (!n_blocks) return GANON_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GANON_E_DEVICE, "hipSetDevice failed");
  if (!ctx->inflate) ctx->inflate = new ganon_inflate_state();
  ganon_inflate_state *st = ctx->inflate;
  const size_t nb = (size_t)n_blocks;
  size_t cap_blk = st->blk_cap;
  int rc;
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
  if (hipMemcpyAsync(st->comp, comp, (size_t)comp_len, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(st->in_off, in_off, nb * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(st->out_off, out_off, nb * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(st->in_len, in_len, nb * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(st->out_len, out_len, nb * 4, hipMemcpyHostToDevice, s) != hipSuccess)
    return fail(ctx, GANON_E_DEVICE, "ganon_inflate: host-to-device copy failed");
  const unsigned grid = (unsigned)std::min<int64_t>(n_blocks, 1 << 16);
  hipLaunchKernelGGL(k_inflate, dim3(grid), dim3(kInfThreads), 0, s, st->comp, comp_len, st->in_off, st->in_len,
                     st->out_off, st->out_len, n_blocks, st->out, out_total, st->status);
  if ((rc = check_launch(ctx, "k_inflate"))) return rc;
  std::vector<int32_t> stat(nb);
  if (hipMemcpyAsync(out, st->out, (size_t)out_total, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(stat.data(), st->status, nb * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(ctx, GANON_E_DEVICE, "ganon_inflate: device-to-host copy failed");
  for (size_t i = 0; i < nb; ++i)
    if (stat[i]) {
      if (first_bad) *first_bad = (int64_t)i;
      return fail(ctx, GANON_E_ARG, "BGZF block %lld: invalid DEFLATE stream (code %d)", (long long)i, stat[i]);
    }
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
  for (void *p : {(void *)st->comp, (void *)st->out, (void *)st->in_off, (void *)st->out_off, (void *)st->in_len,
                  (void *)st->out_len, (void *)st->status})
    if (p) hipFree(p);
  delete st;
}
