// ganon_host.cpp — BGZF/BAM decoder to SoA columns and FASTQ formatter (libganon_host.so).
// See include/ganon_host.h. Written from the SAM/BAM v1 specification.
#include <dlfcn.h>
#include <sys/mman.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <memory>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/ganon_host.h"

namespace {

thread_local std::string g_err;

// memcpy of n bytes; n == 0 (an empty blob's data() may be null) copies nothing
inline void copy_bytes(void *dst, const void *src, size_t n) {
  if (n) std::memcpy(dst, src, n);
}

// A vector whose resize / sized construction leaves new elements uninitialised: the decoder's
// buffers are written in full before they are read (zero-filling them was one more serial pass over
// every inflated byte).
template <class T>
struct NoInit : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInit<U>;
  };
  NoInit() = default;
  template <class U>
  NoInit(const NoInit<U> &) noexcept {}
  template <class U>
  void construct(U *p) noexcept {
    ::new (static_cast<void *>(p)) U;
  }
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
  }
};
template <class T>
using RawVec = std::vector<T, NoInit<T>>;

// Large decoder buffers are first touched by the decoder itself: ask for transparent huge pages on
// them (THP "madvise" mode) so that a chromosome-sized contig does not take a 4 KiB page fault per
// page of every buffer it fills (measured: a 1 GB contig spent more time faulting its buffers in
// than inflating). No effect on small buffers or where THP is off.
inline void huge_advise(void *p, size_t bytes) {
  constexpr uintptr_t kHuge = 2u << 20;
  if (bytes < 4 * kHuge) return;
  const uintptr_t a = ((uintptr_t)p + kHuge - 1) & ~(kHuge - 1), e = ((uintptr_t)p + bytes) & ~(kHuge - 1);
  if (e > a) madvise(reinterpret_cast<void *>(a), e - a, MADV_HUGEPAGE);
}

template <class T>
void huge_resize(RawVec<T> &v, size_t n) {
  const bool grow = n > v.capacity();
  v.resize(n);
  if (grow) huge_advise(v.data(), v.capacity() * sizeof(T));
}

template <class T>
void huge_reserve(RawVec<T> &v, size_t n) {
  if (n <= v.capacity()) return;
  v.reserve(n);
  huge_advise(v.data(), v.capacity() * sizeof(T));
}

// Decoder phase clocks (ganon_host_phase_times): wall nanoseconds of the calling threads, summed over
// calls and threads — where a reader's decode time goes (tools/e2e_bench.py reports them per rank).
enum { kPhParse, kPhInflate, kPhWalk, kPhCopy, kPhRecWalk, kPhSizes, kPhColumns, kPhDevice, kPhRead, kPhDeviceCpu,
       kPhN };
std::atomic<long long> g_phase_ns[kPhN];
// region reads the device decoder finished, and those it handed back to the host's walk
std::atomic<long long> g_dev_regions{0}, g_dev_fallbacks{0};
using PhClock = std::chrono::steady_clock;
// charge the time since t to phase ph and restart t
inline void lap(int ph, PhClock::time_point &t) {
  const auto now = PhClock::now();
  g_phase_ns[ph].fetch_add((long long)std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count(),
                           std::memory_order_relaxed);
  t = now;
}

struct Block {
  int64_t in_off;   // compressed payload offset in the file buffer
  int32_t in_len;   // compressed payload length
  int32_t out_len;  // ISIZE
  int64_t out_off;  // offset in the inflated stream
};

// Raw DEFLATE of one BGZF block. The system's libdeflate (whole-buffer decoder, libdeflate0 in
// the image) is resolved at run time and used when present: ~3x zlib's inflate per core on BAM
// blocks, no per-block state allocation. zlib 1.2.11 otherwise, or with GANON_INFLATE=zlib (A/B);
// both are exact decoders, so the inflated bytes are the same.
struct LibDeflate {
  void *(*alloc)(void);
  int (*decompress)(void *, const void *, size_t, void *, size_t, size_t *);   // 0 = LIBDEFLATE_SUCCESS
  void (*release)(void *);
};

const LibDeflate *libdeflate() {
  static LibDeflate d{};
  static const bool ok = [] {
    const char *e = std::getenv("GANON_INFLATE");
    if (e && std::strcmp(e, "zlib") == 0) return false;
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return false;
    d.alloc = reinterpret_cast<void *(*)(void)>(dlsym(h, "libdeflate_alloc_decompressor"));
    d.decompress = reinterpret_cast<int (*)(void *, const void *, size_t, void *, size_t, size_t *)>(
        dlsym(h, "libdeflate_deflate_decompress"));
    d.release = reinterpret_cast<void (*)(void *)>(dlsym(h, "libdeflate_free_decompressor"));
    return d.alloc && d.decompress && d.release;
  }();
  return ok ? &d : nullptr;
}

// One decoder per thread, kept for the thread's life (the reader's pools are short-lived threads).
struct ThreadInflater {
  void *ld = nullptr;
  z_stream zs{};
  bool z_ready = false;
  ~ThreadInflater() {
    if (ld) libdeflate()->release(ld);
    if (z_ready) inflateEnd(&zs);
  }
};
thread_local ThreadInflater t_inflater;

bool inflate_raw(const uint8_t *in, int32_t in_len, uint8_t *out, int32_t out_len) {
  ThreadInflater &T = t_inflater;
  if (const LibDeflate *L = libdeflate()) {
    if (!T.ld && !(T.ld = L->alloc())) return false;
    // a null actual-size pointer: success only when exactly out_len bytes come out
    return L->decompress(T.ld, in, (size_t)in_len, out, (size_t)out_len, nullptr) == 0;
  }
  if (!T.z_ready) {
    if (inflateInit2(&T.zs, -15) != Z_OK) return false;
    T.z_ready = true;
  } else if (inflateReset(&T.zs) != Z_OK) {
    return false;
  }
  T.zs.next_in = const_cast<Bytef *>(in);
  T.zs.avail_in = (uInt)in_len;
  T.zs.next_out = out;
  T.zs.avail_out = (uInt)out_len;
  const int rc = inflate(&T.zs, Z_FINISH);
  return rc == Z_STREAM_END && T.zs.total_out == (uLong)out_len;
}

}  // namespace

struct ganon_bam {
  std::string err;
  std::vector<char> ref_names;
  std::vector<int64_t> ref_name_off, ref_len;
  RawVec<int32_t> tid, pos, end, flag, mapq, l_seq, n_cigar, mate_tid, mate_pos, tlen, name_len, aux_len;
  RawVec<int64_t> name_off, cig_off, seq_off, qual_off, aux_off;
  RawVec<char> names;
  RawVec<uint32_t> cigar;
  RawVec<uint8_t> seq, qual, aux;
  // (a region decoded on the device, ganon_bam_reader_set_region_decoder) the record columns lie in
  // one block from the decoder, freed with ext_free; the vectors above stay empty
  void *ext_block = nullptr;
  ganon_buf_free_fn ext_free = nullptr;
  ganon_bam_view ext{};
  ganon_bam() = default;
  ganon_bam(const ganon_bam &) = delete;
  ganon_bam &operator=(const ganon_bam &) = delete;
  ~ganon_bam() {
    if (ext_block && ext_free) ext_free(ext_block);
  }
};

static int set_err(const std::string &m) {
  g_err = m;
  return -1;
}

GANON_HOST_API const char *ganon_host_last_error(void) { return g_err.c_str(); }

namespace {

// One BGZF block at h (avail bytes from h to the end of the buffer). Returns 1 with the block's
// total length, payload position/length and ISIZE; 0 when the buffer ends inside the block; -1 on a
// malformed block (message set). Untrusted input: every field is checked before it is used.
int parse_block(const uint8_t *h, int64_t avail, int64_t &blen, int64_t &in_rel, int32_t &in_len, int32_t &isize) {
  if (avail < 18) return 0;
  if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return set_err("not a BGZF file");
  const int xlen = h[10] | (h[11] << 8);
  if (12 + xlen + 8 > avail) return 0;   // the extra field and the CRC32/ISIZE trailer
  int bsize = -1;
  for (int x = 12; x < 12 + xlen;) {
    if (x + 4 > 12 + xlen) return set_err("malformed BGZF extra subfield");
    const int slen = h[x + 2] | (h[x + 3] << 8);
    if (x + 4 + slen > 12 + xlen) return set_err("malformed BGZF extra subfield");
    if (h[x] == 66 && h[x + 1] == 67 && slen == 2) bsize = h[x + 4] | (h[x + 5] << 8);
    x += 4 + slen;
  }
  if (bsize < 0) return set_err("BGZF block without BC subfield");
  blen = (int64_t)bsize + 1;
  if (blen > avail) return 0;
  const int64_t il = blen - 12 - xlen - 8;
  if (il < 0) return set_err("BGZF block size smaller than its header");
  uint32_t is;
  std::memcpy(&is, h + blen - 4, 4);
  if (is > 65536) return set_err("BGZF block ISIZE over 64 KiB");
  in_rel = 12 + xlen;
  in_len = (int32_t)il;
  isize = (int32_t)is;
  return 1;
}

// Inflates blocks[b0, b1) of `file` into data (block out_off relative to blocks[b0].out_off).
bool inflate_blocks(const uint8_t *file, const std::vector<Block> &blocks, size_t b0, size_t b1, uint8_t *data,
                    int threads) {
  std::atomic<size_t> next{b0};
  std::atomic<bool> bad{false};
  const int64_t base = b0 < b1 ? blocks[b0].out_off : 0;
  const int nt = std::max(1, std::min(threads, 64));
  auto worker = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= b1 || bad.load()) return;
      const Block &b = blocks[i];
      if (!inflate_raw(file + b.in_off, b.in_len, data + (b.out_off - base), b.out_len)) bad = true;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt && (size_t)t < b1 - b0; ++t) pool.emplace_back(worker);
  worker();
  for (auto &t : pool) t.join();
  return !bad;
}

// BAM header (magic, text, reference list) at d[0, n). Returns 1 with p = first record offset, 0
// when n ends inside the header, -1 on a malformed header.
int parse_header(const uint8_t *d, int64_t n, ganon_bam *bam, int64_t &p) {
  if (n < 12) return 0;
  if (std::memcmp(d, "BAM\1", 4) != 0) return set_err("not a BAM stream");
  int32_t l_text, n_ref;
  std::memcpy(&l_text, d + 4, 4);
  if (l_text < 0) return set_err("negative header text length");
  p = 8 + (int64_t)l_text;
  if (p + 4 > n) return 0;
  std::memcpy(&n_ref, d + p, 4);
  p += 4;
  if (n_ref < 0) return set_err("negative reference count");
  bam->ref_names.clear();
  bam->ref_name_off.clear();
  bam->ref_len.clear();
  for (int32_t i = 0; i < n_ref; ++i) {
    int32_t l_name, l_ref;
    if (p + 4 > n) return 0;
    std::memcpy(&l_name, d + p, 4);
    p += 4;
    if (l_name <= 0) return set_err("bad reference name");
    if (p + l_name + 4 > n) return 0;
    bam->ref_name_off.push_back((int64_t)bam->ref_names.size());
    bam->ref_names.insert(bam->ref_names.end(), d + p, d + p + l_name);
    bam->ref_names.back() = '\0';
    p += l_name;
    std::memcpy(&l_ref, d + p, 4);
    p += 4;
    bam->ref_len.push_back(l_ref);
  }
  return 1;
}

// Column arrays of the records packed back to back in d[p, n) (each: block_size + body), or, with
// `known`, of the records at those offsets of d (the reader's scans walked and checked them already:
// their records stay in place in the scan's buffer, no boundary walk and no copy of the kept runs).
int records_to_columns(const uint8_t *d, int64_t p, int64_t n, ganon_bam *bam, int threads,
                       const std::vector<int64_t> *known = nullptr) {
  const int nt = std::max(1, std::min(threads, 64));
  // ---- records: boundaries (sequential), sizes + offsets, then columns in parallel ----
  std::vector<int64_t> own;   // offset of each record's block_size field
  auto tph = PhClock::now();
  if (!known) {
    while (p < n) {
      int32_t bs;
      if (p + 4 > n) return set_err("truncated record size");
      std::memcpy(&bs, d + p, 4);
      if (bs < 32 || p + 4 + bs > n) return set_err("bad record size");
      own.push_back(p);
      p += 4 + bs;
    }
  }
  const std::vector<int64_t> &rec = known ? *known : own;
  const int64_t nr = (int64_t)rec.size();
  // per record: name bytes kept, CIGAR ops, sequence length, aux bytes
  std::vector<int64_t> o_name(nr + 1), o_cig(nr + 1), o_seq(nr + 1), o_qual(nr + 1), o_aux(nr + 1);
  std::atomic<int64_t> first_bad{INT64_MAX};
  lap(kPhRecWalk, tph);
  auto run_chunks = [&](auto &&fn) {
    std::vector<std::thread> ts;
    const int64_t per = (nr + nt - 1) / std::max(nt, 1);
    for (int t = 1; t < nt; ++t) ts.emplace_back([&, t] { fn(std::min(nr, t * per), std::min(nr, (t + 1) * per)); });
    fn((int64_t)0, std::min(nr, per));
    for (auto &th : ts) th.join();
  };
  run_chunks([&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const uint8_t *r = d + rec[i] + 4;
      int32_t bs, lseq;
      uint16_t ncig;
      std::memcpy(&bs, d + rec[i], 4);
      std::memcpy(&ncig, r + 12, 2);
      std::memcpy(&lseq, r + 16, 4);
      const uint8_t l_rn = r[8];
      const int64_t need = 32 + (int64_t)l_rn + 4LL * ncig + (lseq + 1) / 2 + lseq;
      if (lseq < 0 || need > bs) {
        int64_t cur = first_bad.load();
        while (i < cur && !first_bad.compare_exchange_weak(cur, i)) {
        }
        o_name[i + 1] = o_cig[i + 1] = o_seq[i + 1] = o_qual[i + 1] = o_aux[i + 1] = 0;
        continue;
      }
      o_name[i + 1] = l_rn + ((l_rn == 0 || r[32 + l_rn - 1] != 0) ? 1 : 0);
      o_cig[i + 1] = ncig;
      o_seq[i + 1] = (lseq + 1) / 2;
      o_qual[i + 1] = lseq;
      o_aux[i + 1] = bs - need;
    }
  });
  if (first_bad.load() != INT64_MAX) return set_err("record fields exceed block size");
  for (int64_t i = 0; i < nr; ++i) {
    o_name[i + 1] += o_name[i];
    o_cig[i + 1] += o_cig[i];
    o_seq[i + 1] += o_seq[i];
    o_qual[i + 1] += o_qual[i];
    o_aux[i + 1] += o_aux[i];
  }
  for (auto *v : {&bam->tid, &bam->pos, &bam->end, &bam->flag, &bam->mapq, &bam->l_seq, &bam->n_cigar, &bam->mate_tid,
                  &bam->mate_pos, &bam->tlen, &bam->name_len, &bam->aux_len})
    huge_resize(*v, (size_t)nr);
  for (auto *v : {&bam->name_off, &bam->cig_off, &bam->seq_off, &bam->qual_off, &bam->aux_off}) huge_resize(*v, (size_t)nr);
  huge_resize(bam->names, (size_t)o_name[nr]);
  huge_resize(bam->cigar, (size_t)o_cig[nr]);
  huge_resize(bam->seq, (size_t)o_seq[nr]);
  huge_resize(bam->qual, (size_t)o_qual[nr]);
  huge_resize(bam->aux, (size_t)o_aux[nr]);
  lap(kPhSizes, tph);
  run_chunks([&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const uint8_t *r = d + rec[i] + 4;
      int32_t bs, rtid, rpos, mtid, mpos, rtlen, lseq;
      uint16_t ncig, rflag;
      std::memcpy(&bs, d + rec[i], 4);
      std::memcpy(&rtid, r + 0, 4);
      std::memcpy(&rpos, r + 4, 4);
      const uint8_t l_rn = r[8], rmapq = r[9];
      std::memcpy(&ncig, r + 12, 2);
      std::memcpy(&rflag, r + 14, 2);
      std::memcpy(&lseq, r + 16, 4);
      std::memcpy(&mtid, r + 20, 4);
      std::memcpy(&mpos, r + 24, 4);
      std::memcpy(&rtlen, r + 28, 4);
      bam->tid[i] = rtid;
      bam->pos[i] = rpos;
      bam->flag[i] = rflag;
      bam->mapq[i] = rmapq;
      bam->l_seq[i] = lseq;
      bam->n_cigar[i] = ncig;
      bam->mate_tid[i] = mtid;
      bam->mate_pos[i] = mpos;
      bam->tlen[i] = rtlen;
      int64_t q = 32;
      bam->name_off[i] = o_name[i];
      bam->name_len[i] = l_rn > 0 ? l_rn - 1 : 0;
      char *nm = bam->names.data() + o_name[i];
      copy_bytes(nm, r + q, l_rn);
      if (o_name[i + 1] - o_name[i] > l_rn) nm[l_rn] = '\0';
      q += l_rn;
      bam->cig_off[i] = o_cig[i];
      int64_t rlen = 0;
      uint32_t *cg = bam->cigar.data() + o_cig[i];
      copy_bytes(cg, r + q, 4LL * ncig);
      for (int k = 0; k < ncig; ++k) {
        const uint32_t w = cg[k];
        const int op = w & 0xF;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rlen += w >> 4;
      }
      q += 4LL * ncig;
      if (rflag & 4) rlen = 0;
      bam->end[i] = (int32_t)(rpos + (rlen > 0 ? rlen : 1));
      bam->seq_off[i] = o_seq[i];
      copy_bytes(bam->seq.data() + o_seq[i], r + q, (size_t)((lseq + 1) / 2));
      q += (lseq + 1) / 2;
      bam->qual_off[i] = o_qual[i];
      copy_bytes(bam->qual.data() + o_qual[i], r + q, (size_t)lseq);
      q += lseq;
      bam->aux_off[i] = o_aux[i];
      bam->aux_len[i] = (int32_t)(bs - q);
      copy_bytes(bam->aux.data() + o_aux[i], r + q, (size_t)(bs - q));
    }
  });
  lap(kPhColumns, tph);
  return 0;
}


}  // namespace

static int bam_open_impl(const char *path, int threads, ganon_bam **out) {
  FILE *fh = std::fopen(path, "rb");
  if (!fh) return set_err(std::string("cannot open ") + path);
  std::fseek(fh, 0, SEEK_END);
  const long fsize = std::ftell(fh);
  std::fseek(fh, 0, SEEK_SET);
  RawVec<uint8_t> file((size_t)std::max(0L, fsize));
  if (fsize > 0 && std::fread(file.data(), 1, (size_t)fsize, fh) != (size_t)fsize) {
    std::fclose(fh);
    return set_err("short read");
  }
  std::fclose(fh);
  std::vector<Block> blocks;
  int64_t off = 0, total = 0;
  const int64_t fsz = (int64_t)file.size();
  while (off < fsz) {
    int64_t blen, in_rel;
    int32_t in_len, isize;
    const int rc = parse_block(&file[off], fsz - off, blen, in_rel, in_len, isize);
    if (rc < 0) return -1;
    if (rc == 0) return set_err("truncated BGZF block");
    if (isize > 0) blocks.push_back(Block{off + in_rel, in_len, isize, total});
    total += isize;
    off += blen;
  }
  RawVec<uint8_t> data((size_t)total);
  if (!inflate_blocks(file.data(), blocks, 0, blocks.size(), data.data(), threads))
    return set_err("BGZF inflate failed");
  file.clear();
  file.shrink_to_fit();
  auto *bam = new ganon_bam();
  int64_t p = 0;
  const int hr = parse_header(data.data(), (int64_t)data.size(), bam, p);
  if (hr <= 0) {
    delete bam;
    return hr < 0 ? -1 : set_err("truncated header");
  }
  if (records_to_columns(data.data(), p, (int64_t)data.size(), bam, threads) != 0) {
    delete bam;
    return -1;
  }
  *out = bam;
  return 0;
}

// No C++ exception crosses the C ABI: allocation failures (a huge ISIZE total, a corrupt record
// count) become an error code.
GANON_HOST_API int ganon_bam_open(const char *path, int threads, ganon_bam **out) {
  if (!path || !out) return set_err("null argument");
  *out = nullptr;
  try {
    return bam_open_impl(path, threads, out);
  } catch (const std::bad_alloc &) {
    return set_err("out of memory decoding the BAM file");
  } catch (const std::exception &e) {
    return set_err(std::string("BAM decode failed: ") + e.what());
  }
}

GANON_HOST_API int ganon_bam_view_get(ganon_bam *b, ganon_bam_view *v) {
  if (!b || !v) return set_err("null argument");
  if (b->ext_block) {
    *v = b->ext;
    v->n_ref = (int32_t)b->ref_len.size();
    v->ref_names = b->ref_names.data();
    v->ref_name_off = b->ref_name_off.data();
    v->ref_len = b->ref_len.data();
    return 0;
  }
  v->n_records = (int64_t)b->tid.size();
  v->n_ref = (int32_t)b->ref_len.size();
  v->ref_names = b->ref_names.data();
  v->ref_name_off = b->ref_name_off.data();
  v->ref_len = b->ref_len.data();
  v->tid = b->tid.data();
  v->pos = b->pos.data();
  v->end = b->end.data();
  v->flag = b->flag.data();
  v->mapq = b->mapq.data();
  v->l_seq = b->l_seq.data();
  v->n_cigar = b->n_cigar.data();
  v->mate_tid = b->mate_tid.data();
  v->mate_pos = b->mate_pos.data();
  v->tlen = b->tlen.data();
  v->name_off = b->name_off.data();
  v->name_len = b->name_len.data();
  v->cig_off = b->cig_off.data();
  v->seq_off = b->seq_off.data();
  v->qual_off = b->qual_off.data();
  v->aux_off = b->aux_off.data();
  v->aux_len = b->aux_len.data();
  v->names = b->names.data();
  v->names_bytes = (int64_t)b->names.size();
  v->cigar = b->cigar.data();
  v->cigar_ops = (int64_t)b->cigar.size();
  v->seq = b->seq.data();
  v->seq_bytes = (int64_t)b->seq.size();
  v->qual = b->qual.data();
  v->qual_bytes = (int64_t)b->qual.size();
  v->aux = b->aux.data();
  v->aux_bytes = (int64_t)b->aux.size();
  return 0;
}

GANON_HOST_API const char *ganon_bam_error(ganon_bam *) { return g_err.c_str(); }

GANON_HOST_API void ganon_bam_close(ganon_bam *b) { delete b; }

// ---- contig reader (bounded-memory streaming decode) ------------------------------------------
// The reference reads a sample through region queries (AlignmentFile.fetch / pileup per section,
// short_read_tumor_normal_anonymizer.py:498-558, pileup_io.pyx:8-41), never the whole file at once.
// The reader decodes the records of one reference sequence at a time: it seeks to the sequence's
// first record through the BAM index (.bai: pseudo-bin 37450 or the smallest chunk start of its
// bins) or, without one, streams forward from the previous sequence's end; it inflates a bounded
// window of BGZF blocks at a time on `threads` threads and keeps only the sequence's records.
struct ganon_bam_reader {
  FILE *fh = nullptr;
  int64_t fsize = 0;
  const uint8_t *map = nullptr;      // the whole file mapped read-only (nullptr: fread per window)
  int threads = 8;
  int64_t chunk = 32 << 20;          // compressed bytes read per step
  ganon_bam header;                  // reference list only
  int64_t data_voff = 0;             // virtual offset of the first record
  bool has_index = false;
  std::vector<int64_t> index_beg;    // per tid: virtual offset of its first record, -1 = no records
  std::vector<int64_t> index_end;    // per tid: virtual offset past its last record (-1 unknown)
  std::vector<std::vector<int64_t>> linear;   // per tid: the linear index (first record of each 16 kb window)
  int64_t cur_voff = -1;             // forward cursor: the first record not yet consumed
  int32_t cur_tid = 0;
  ganon_buf_alloc_fn balloc = nullptr;   // ganon_bam_reader_set_buffer_alloc: the scans' inflated bytes in
  ganon_buf_free_fn bfree = nullptr;     // a page-locked buffer kept across scans (pbuf, pcap)
  uint8_t *pbuf = nullptr;
  int64_t pcap = 0;
  uint8_t *cbuf = nullptr;               // (with balloc) the compressed windows for the GPU inflater,
  int64_t ccap = 0;                      // read by pread into page-locked memory
  ganon_inflate_fn inflater = nullptr;   // ganon_bam_reader_set_inflater: block windows inflated by it
  void *inflater_user = nullptr;
  int64_t inflater_min = 64;             // ... when they hold at least this many blocks
  ganon_region_fn rdec = nullptr;        // ganon_bam_reader_set_region_decoder: a region read's first
  void *rdec_user = nullptr;             // window decoded whole by it (at least rdec_min blocks)
  int64_t rdec_min = 64;
  ganon_buf_free_fn rdec_release = nullptr;
};

namespace {

// The inflated bytes of one scan: the reader's page-locked buffer when it has a buffer allocator
// (the GPU inflater's device-to-host copies then land by DMA, with no staging copy on the host's
// cores; the buffer is reused by the reader's next scan: the columns are copied out of it), else a
// fresh huge-page buffer.
struct ScanBuf {
  ganon_bam_reader *R;
  RawVec<uint8_t> own;
  size_t n = 0;
  bool pinned;
  explicit ScanBuf(ganon_bam_reader *r) : R(r), pinned(r->balloc != nullptr) {}
  uint8_t *data() { return pinned ? R->pbuf : own.data(); }
  size_t size() const { return pinned ? n : own.size(); }
  bool empty() const { return size() == 0; }
  void clear() {
    if (pinned) n = 0;
    else own.clear();
  }
  uint8_t &operator[](size_t i) { return data()[i]; }
  bool grow(size_t m) {   // (pinned) capacity for m bytes, contents kept
    if ((int64_t)m <= R->pcap) return true;
    const size_t cap = std::max(m, (size_t)(2 * R->pcap));
    void *p = nullptr;
    if (R->balloc((int64_t)cap, &p) != 0 || !p) return false;
    if (n) std::memcpy(p, R->pbuf, n);
    if (R->pbuf) R->bfree(R->pbuf);
    R->pbuf = static_cast<uint8_t *>(p);
    R->pcap = (int64_t)cap;
    return true;
  }
  void reserve(size_t c) {
    if (pinned) {
      if (!grow(c)) throw std::bad_alloc();
    } else {
      huge_reserve(own, c);
    }
  }
  void resize(size_t m) {
    if (pinned) {
      if (!grow(m)) throw std::bad_alloc();
      n = m;
    } else {
      huge_resize(own, m);
    }
  }
};
inline void buf_resize(RawVec<uint8_t> &v, size_t m) { huge_resize(v, m); }
inline void buf_resize(ScanBuf &v, size_t m) { v.resize(m); }

constexpr int32_t kTidEnd = INT32_MAX;
inline int64_t tid_order(int32_t t) { return t < 0 ? (int64_t)INT32_MAX : (int64_t)t; }   // unplaced last

// A region read's first window offered to the reader's region decoder: the records from byte p0 of
// the window's inflated bytes; done = the decoder returned the region's columns (cols, block).
struct RegionCall {
  int32_t tid;
  int64_t beg, end, p0;
  bool done = false;
  ganon_bam_view cols{};
  void *block = nullptr;
};

// Reads and inflates complete BGZF blocks starting at file offset coff (at most R->chunk compressed
// bytes). Appends the inflated bytes to data and one (data offset, file offset) pair per non-empty
// block to bmap. Returns the file offset after the last complete block, or -1 on error. With rq and
// a region decoder, a window of enough blocks goes to the decoder (rq->done: the region is decoded,
// data holds nothing of it).
template <class Buf>
int64_t read_blocks(ganon_bam_reader *R, int64_t coff, int64_t step, Buf &data,
                    std::vector<std::pair<int64_t, int64_t>> &bmap, RegionCall *rq = nullptr) {
  auto tph = PhClock::now();
  const int64_t want = std::min<int64_t>(std::max<int64_t>(step, 1 << 17), R->fsize - coff);
  const bool dev = rq && R->rdec;   // (then the decoder inflates the window if it holds enough blocks)
  // the window's compressed bytes: in place in the file mapping (the inflate threads read the page
  // cache directly; no serial copy, no fresh buffer to fault in per window), else read into a buffer
  RawVec<uint8_t> buf;
  const uint8_t *comp;
  if (R->balloc && ((R->inflater && want >= R->inflater_min * 16384) || (dev && want >= R->rdec_min * 16384))) {
    // a window for the GPU inflater: read into the reader's page-locked buffer (its upload then goes
    // by DMA; through the file mapping, every page faulted into this process and was copied again
    // by the runtime's staging, and unmapping the touched pages was most of the readers' close)
    if (want > R->ccap) {
      void *p = nullptr;
      const int64_t cap = std::max<int64_t>(want, 2 * R->ccap);
      if (R->balloc(cap, &p) != 0 || !p) return set_err("page-locked window allocation failed");
      if (R->cbuf) R->bfree(R->cbuf);
      R->cbuf = static_cast<uint8_t *>(p);
      R->ccap = cap;
    }
    const int fd = fileno(R->fh);
    int64_t got = 0;
    while (got < want) {
      const ssize_t r = pread(fd, R->cbuf + got, (size_t)(want - got), (off_t)(coff + got));
      if (r <= 0) return set_err("short read");
      got += r;
    }
    comp = R->cbuf;
    lap(kPhRead, tph);
  } else if (R->map) {
    comp = R->map + coff;
    const uintptr_t pg = 4096, a = (uintptr_t)comp & ~(pg - 1);
    madvise(reinterpret_cast<void *>(a), (size_t)((uintptr_t)comp + want - a), MADV_WILLNEED);
  } else {
    buf.resize((size_t)want);
    if (std::fseek(R->fh, (long)coff, SEEK_SET) != 0 || std::fread(buf.data(), 1, (size_t)want, R->fh) != (size_t)want)
      return set_err("short read");
    comp = buf.data();
  }
  std::vector<Block> blocks;
  std::vector<int64_t> bcoff;
  int64_t off = 0, total = 0;
  while (off < want) {
    int64_t blen, in_rel;
    int32_t in_len, isize;
    const int rc = parse_block(comp + off, want - off, blen, in_rel, in_len, isize);
    if (rc < 0) return -1;
    if (rc == 0) break;
    if (isize > 0) {
      blocks.push_back(Block{off + in_rel, in_len, isize, total});
      bcoff.push_back(coff + off);
    }
    total += isize;
    off += blen;
  }
  if (off == 0) return set_err("truncated BGZF block");
  const size_t base = data.size();
  buf_resize(data, base + (size_t)total);
  lap(kPhParse, tph);
  if (dev && (int64_t)blocks.size() >= R->rdec_min) {
    const size_t nb = blocks.size();
    std::vector<int64_t> in_off(nb), out_off(nb);
    std::vector<int32_t> in_len(nb), out_len(nb);
    for (size_t i = 0; i < nb; ++i) {
      in_off[i] = blocks[i].in_off;
      in_len[i] = blocks[i].in_len;
      out_off[i] = blocks[i].out_off;
      out_len[i] = blocks[i].out_len;
    }
    const int at_eof = coff + off >= R->fsize ? 1 : 0;
    timespec c0{}, c1{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
    const int r = R->rdec(R->rdec_user, comp, off, in_off.data(), in_len.data(), out_off.data(), out_len.data(),
                          (int64_t)nb, data.data() + base, total, rq->p0 + (int64_t)base, rq->tid, rq->beg, rq->end,
                          at_eof, &rq->cols, &rq->block);
    lap(kPhDevice, tph);
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
    g_phase_ns[kPhDeviceCpu].fetch_add((c1.tv_sec - c0.tv_sec) * 1000000000LL + (c1.tv_nsec - c0.tv_nsec),
                                       std::memory_order_relaxed);
    if (r < 0) return set_err("BGZF inflate failed (region decoder)");
    if (r == 1) {
      rq->done = true;
      g_dev_regions.fetch_add(1, std::memory_order_relaxed);
      return coff + off;
    }
    g_dev_fallbacks.fetch_add(1, std::memory_order_relaxed);
  } else if (R->inflater && (int64_t)blocks.size() >= R->inflater_min) {
    const size_t nb = blocks.size();
    std::vector<int64_t> in_off(nb), out_off(nb);
    std::vector<int32_t> in_len(nb), out_len(nb);
    for (size_t i = 0; i < nb; ++i) {
      in_off[i] = blocks[i].in_off;
      in_len[i] = blocks[i].in_len;
      out_off[i] = blocks[i].out_off;
      out_len[i] = blocks[i].out_len;
    }
    if (R->inflater(R->inflater_user, comp, off, in_off.data(), in_len.data(), out_off.data(), out_len.data(),
                    (int64_t)nb, data.data() + base, total) != 0)
      return set_err("BGZF inflate failed (inflater)");
  } else if (!inflate_blocks(comp, blocks, 0, blocks.size(), data.data() + base, R->threads)) {
    return set_err("BGZF inflate failed");
  }
  lap(kPhInflate, tph);
  for (size_t i = 0; i < blocks.size(); ++i) bmap.emplace_back((int64_t)base + blocks[i].out_off, bcoff[i]);
  return coff + off;
}

int64_t voff_at(const std::vector<std::pair<int64_t, int64_t>> &bmap, int64_t x) {
  auto it = std::upper_bound(bmap.begin(), bmap.end(), std::make_pair(x, INT64_MAX));
  if (it == bmap.begin()) return -1;
  --it;
  return (it->second << 16) | (x - it->first);
}

// Streams from virtual offset voff: keeps the records of `tid`, stops at the first record after them
// (each tid's records are contiguous in a coordinate-sorted file). first_tid: tid of the first
// record met (kTidEnd when none) so that an index start can be validated. hint: expected compressed
// bytes of the sequence (index span) or 0; the step read and inflated at a time starts there (or at
// 1 MiB) and doubles up to the reader's window, so a small sequence never inflates a whole window.
int scan_tid(ganon_bam_reader *R, int64_t voff, int32_t tid, int64_t hint, ScanBuf &data,
             std::vector<int64_t> &recs, int64_t &next_voff, int32_t &next_tid, int32_t &first_tid) {
  // (the records stay where they were inflated: `data` grows by every window and only the offsets of
  // the sequence's records are kept — round 6; the windows' consumed bytes used to be dropped and the
  // kept runs copied into a second buffer, then walked again to find their boundaries)
  int64_t step = std::min<int64_t>(hint > 0 ? hint + (1 << 16) : (1 << 20), R->chunk);
  int64_t coff = voff >> 16;
  std::vector<std::pair<int64_t, int64_t>> bmap;
  data.clear();
  recs.clear();
  int64_t dpos = (int64_t)(voff & 0xFFFF);
  bool seen = false;
  first_tid = kTidEnd;
  for (;;) {
    if (coff >= R->fsize) {
      if (dpos != (int64_t)data.size()) return set_err("truncated BAM record");
      next_voff = -1;
      next_tid = kTidEnd;
      return 0;
    }
    coff = read_blocks(R, coff, step, data, bmap);
    if (coff < 0) return -1;
    step = std::min<int64_t>(2 * step, R->chunk);
    auto tw = PhClock::now();
    for (;;) {
      if (dpos + 4 > (int64_t)data.size()) break;
      int32_t bs, rtid;
      std::memcpy(&bs, &data[(size_t)dpos], 4);
      if (bs < 32) return set_err("bad record size");
      if (dpos + 4 + bs > (int64_t)data.size()) break;
      std::memcpy(&rtid, &data[(size_t)dpos + 4], 4);
      if (first_tid == kTidEnd) first_tid = rtid;
      if (rtid == tid) {
        recs.push_back(dpos);
        seen = true;
      } else if (seen || tid_order(rtid) > tid_order(tid)) {
        next_voff = voff_at(bmap, dpos);
        next_tid = rtid;
        lap(kPhWalk, tw);
        return 0;
      }
      dpos += 4 + bs;
    }
    lap(kPhWalk, tw);
  }
}

// Record end (bam_endpos: pos + reference length, pos + 1 without one or when unmapped) of the
// record at d (block_size first).
int64_t record_end(const uint8_t *d) {
  int32_t pos, l_rn_mq_bin, flag_nc;
  std::memcpy(&pos, d + 8, 4);
  std::memcpy(&l_rn_mq_bin, d + 12, 4);
  std::memcpy(&flag_nc, d + 16, 4);
  const int l_rn = l_rn_mq_bin & 0xFF, nc = flag_nc & 0xFFFF, flag = (int)((uint32_t)flag_nc >> 16);
  int64_t rl = 0;
  if (!(flag & 4)) {
    const uint8_t *cg = d + 36 + l_rn;
    for (int k = 0; k < nc; ++k) {
      uint32_t w;
      std::memcpy(&w, cg + 4 * k, 4);
      const int op = w & 0xF;
      if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += w >> 4;
    }
  }
  return (int64_t)pos + (rl > 0 ? rl : 1);
}

// Streams from virtual offset voff: keeps the records of `tid` overlapping [beg, end) (htslib's
// region semantics: pos < end and bam_endpos > beg), in file order; stops at the first record of
// another sequence or at pos >= end. Runs of kept records are copied to kept at once.
int scan_region(ganon_bam_reader *R, int64_t voff, int32_t tid, int64_t beg, int64_t end, int64_t hint,
                ScanBuf &data, std::vector<int64_t> &recs, RegionCall *rq = nullptr, int64_t dev_step = 0) {
  // (records stay in place in `data`, their offsets in recs: as scan_tid)
  int64_t step = std::min<int64_t>(hint > 0 ? hint + (1 << 16) : (1 << 20), R->chunk);
  int64_t coff = voff >> 16;
  std::vector<std::pair<int64_t, int64_t>> bmap;
  data.clear();
  recs.clear();
  int64_t dpos = (int64_t)(voff & 0xFFFF);
  if (rq) {
    rq->p0 = dpos;
    if (dev_step > 0) step = dev_step;
  }
  for (;;) {
    if (coff >= R->fsize) {
      if (dpos < (int64_t)data.size()) return set_err("truncated BAM record");
      return 0;
    }
    coff = read_blocks(R, coff, step, data, bmap, rq);
    if (coff < 0) return -1;
    if (rq && rq->done) return 0;
    rq = nullptr;   // (the first window only)
    step = std::min<int64_t>(2 * step, R->chunk);
    auto tw = PhClock::now();
    for (;;) {
      if (dpos + 4 > (int64_t)data.size()) break;
      int32_t bs, rtid, rpos;
      std::memcpy(&bs, &data[(size_t)dpos], 4);
      if (bs < 32) return set_err("bad record size");
      if (dpos + 4 + bs > (int64_t)data.size()) break;
      std::memcpy(&rtid, &data[(size_t)dpos + 4], 4);
      std::memcpy(&rpos, &data[(size_t)dpos + 8], 4);
      if (rtid != tid || rpos >= end) {
        if (tid_order(rtid) < tid_order(tid)) return set_err("BAM index points before its sequence");
        lap(kPhWalk, tw);
        return 0;
      }
      if (record_end(&data[(size_t)dpos]) > beg) recs.push_back(dpos);
      dpos += 4 + bs;
    }
    lap(kPhWalk, tw);
  }
}

void load_index(ganon_bam_reader *R, const std::string &bam_path) {
  std::vector<std::string> cands{bam_path + ".bai"};
  if (bam_path.size() > 4 && bam_path.compare(bam_path.size() - 4, 4, ".bam") == 0)
    cands.push_back(bam_path.substr(0, bam_path.size() - 4) + ".bai");
  for (const std::string &ip : cands) {
    FILE *f = std::fopen(ip.c_str(), "rb");
    if (!f) continue;
    std::vector<uint8_t> b;
    uint8_t tmp[65536];
    size_t k;
    while ((k = std::fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + k);
    std::fclose(f);
    size_t p = 0;
    auto rd = [&](void *dst, size_t n) {
      if (p + n > b.size()) return false;
      std::memcpy(dst, &b[p], n);
      p += n;
      return true;
    };
    char magic[4];
    int32_t n_ref;
    if (!rd(magic, 4) || std::memcmp(magic, "BAI\1", 4) != 0 || !rd(&n_ref, 4) ||
        n_ref != (int32_t)R->header.ref_len.size())
      continue;
    std::vector<int64_t> beg((size_t)n_ref, -1), end((size_t)n_ref, -1);
    std::vector<std::vector<int64_t>> lin((size_t)n_ref);
    bool ok = true;
    for (int32_t r = 0; r < n_ref && ok; ++r) {
      int32_t n_bin;
      if (!rd(&n_bin, 4) || n_bin < 0) { ok = false; break; }
      int64_t pseudo = -1, pseudo_end = -1, lo = -1, hi = -1;
      for (int32_t i = 0; i < n_bin && ok; ++i) {
        uint32_t bin;
        int32_t n_chunk;
        if (!rd(&bin, 4) || !rd(&n_chunk, 4) || n_chunk < 0) { ok = false; break; }
        for (int32_t c = 0; c < n_chunk; ++c) {
          uint64_t cb, ce;
          if (!rd(&cb, 8) || !rd(&ce, 8)) { ok = false; break; }
          if (bin == 37450) {
            if (c == 0) {
              pseudo = (int64_t)cb;
              pseudo_end = (int64_t)ce;
            }
          } else {
            if (lo < 0 || (int64_t)cb < lo) lo = (int64_t)cb;
            if ((int64_t)ce > hi) hi = (int64_t)ce;
          }
        }
      }
      int32_t n_intv;
      if (!ok || !rd(&n_intv, 4) || n_intv < 0 || p + 8ull * (size_t)n_intv > b.size()) { ok = false; break; }
      lin[(size_t)r].resize((size_t)n_intv);
      if (n_intv) std::memcpy(lin[(size_t)r].data(), &b[p], 8ull * (size_t)n_intv);
      p += 8ull * (size_t)n_intv;
      beg[(size_t)r] = pseudo >= 0 ? pseudo : lo;
      end[(size_t)r] = pseudo >= 0 ? pseudo_end : hi;
    }
    if (!ok) continue;
    R->index_beg = std::move(beg);
    R->index_end = std::move(end);
    R->linear = std::move(lin);
    R->has_index = true;
    return;
  }
}

int reader_open_impl(const char *path, int threads, ganon_bam_reader **out) {
  auto *R = new ganon_bam_reader();
  R->threads = std::max(1, std::min(threads, 64));
  R->fh = std::fopen(path, "rb");
  if (!R->fh) {
    delete R;
    return set_err(std::string("cannot open ") + path);
  }
  std::fseek(R->fh, 0, SEEK_END);
  R->fsize = (int64_t)std::ftell(R->fh);
  if (R->fsize > 0 && !std::getenv("GANON_NO_MMAP")) {   // (GANON_NO_MMAP=1: fread per window, A/B)
    void *m = mmap(nullptr, (size_t)R->fsize, PROT_READ, MAP_PRIVATE, fileno(R->fh), 0);
    if (m != MAP_FAILED) R->map = static_cast<const uint8_t *>(m);
  }
  // header: inflate block windows until it is complete
  RawVec<uint8_t> data;
  std::vector<std::pair<int64_t, int64_t>> bmap;
  int64_t coff = 0, p = 0;
  for (;;) {
    if (coff >= R->fsize) {
      ganon_bam_reader_close(R);
      return set_err("truncated header");
    }
    coff = read_blocks(R, coff, 1 << 20, data, bmap);
    if (coff < 0) {
      ganon_bam_reader_close(R);
      return -1;
    }
    const int hr = parse_header(data.data(), (int64_t)data.size(), &R->header, p);
    if (hr < 0) {
      ganon_bam_reader_close(R);
      return -1;
    }
    if (hr > 0) break;
  }
  R->data_voff = p == (int64_t)data.size() ? (coff << 16) : voff_at(bmap, p);
  R->cur_voff = R->data_voff;
  R->cur_tid = 0;
  load_index(R, path);
  *out = R;
  return 0;
}

}  // namespace

GANON_HOST_API int ganon_bam_reader_open(const char *path, int threads, ganon_bam_reader **out) {
  if (!path || !out) return set_err("null argument");
  *out = nullptr;
  try {
    return reader_open_impl(path, threads, out);
  } catch (const std::bad_alloc &) {
    return set_err("out of memory reading the BAM header");
  }
}

GANON_HOST_API int ganon_bam_reader_set_window(ganon_bam_reader *R, int64_t bytes) {
  if (!R) return set_err("null argument");
  R->chunk = std::max<int64_t>(bytes, 1 << 17);   // at least two maximal BGZF blocks
  return 0;
}

GANON_HOST_API int ganon_bam_reader_set_buffer_alloc(ganon_bam_reader *R, ganon_buf_alloc_fn alloc,
                                                     ganon_buf_free_fn free_fn) {
  if (!R || (!alloc) != (!free_fn)) return set_err("ganon_bam_reader_set_buffer_alloc: bad arguments");
  if (R->pbuf) R->bfree(R->pbuf);
  if (R->cbuf) R->bfree(R->cbuf);
  R->pbuf = R->cbuf = nullptr;
  R->pcap = R->ccap = 0;
  R->balloc = alloc;
  R->bfree = free_fn;
  return 0;
}

GANON_HOST_API int ganon_bam_reader_set_inflater(ganon_bam_reader *R, ganon_inflate_fn fn, void *user,
                                                 int64_t min_blocks) {
  if (!R || min_blocks < 1) return set_err("ganon_bam_reader_set_inflater: bad arguments");
  R->inflater = fn;
  R->inflater_user = fn ? user : nullptr;
  R->inflater_min = min_blocks;
  return 0;
}

GANON_HOST_API int ganon_bam_reader_set_region_decoder(ganon_bam_reader *R, ganon_region_fn fn, void *user,
                                                       int64_t min_blocks, ganon_buf_free_fn release) {
  if (!R || min_blocks < 1 || (fn && !release)) return set_err("ganon_bam_reader_set_region_decoder: bad arguments");
  R->rdec = fn;
  R->rdec_user = fn ? user : nullptr;
  R->rdec_min = min_blocks;
  R->rdec_release = fn ? release : nullptr;
  return 0;
}

GANON_HOST_API int ganon_bam_reader_has_index(const ganon_bam_reader *R) { return R && R->has_index ? 1 : 0; }

GANON_HOST_API int ganon_bam_reader_header(ganon_bam_reader *R, ganon_bam_view *v) {
  if (!R) return set_err("null argument");
  return ganon_bam_view_get(&R->header, v);
}

GANON_HOST_API int ganon_bam_reader_contig(ganon_bam_reader *R, int32_t tid, ganon_bam **out) {
  if (!R || !out) return set_err("null argument");
  *out = nullptr;
  if (tid < 0 || tid >= (int32_t)R->header.ref_len.size()) return set_err("tid out of range");
  try {
    ScanBuf data(R);
    std::vector<int64_t> recs;
    int64_t next_voff = -1;
    int32_t next_tid = kTidEnd, first_tid = kTidEnd;
    bool done = false;
    if (R->has_index) {
      const int64_t beg = R->index_beg[(size_t)tid];
      if (beg < 0) {
        done = true;   // the index lists no record of this sequence
      } else {
        const int64_t e = R->index_end[(size_t)tid];
        const int64_t hint = e > beg ? (e >> 16) - (beg >> 16) : 0;
        // the sequence's blocks, inflated, at ~3.5x their compressed span (address space only: an
        // underestimate just grows the buffer)
        data.reserve((size_t)hint * 7 / 2 + (4 << 20));
        if (scan_tid(R, beg, tid, hint, data, recs, next_voff, next_tid, first_tid) != 0) return -1;
        done = first_tid == tid;   // a stale index falls back to the forward scan
        if (!done) recs.clear();
      }
    }
    if (!done) {
      const bool forward = R->cur_voff >= 0 && tid_order(R->cur_tid) <= tid_order(tid);
      if (scan_tid(R, forward ? R->cur_voff : R->data_voff, tid, 0, data, recs, next_voff, next_tid, first_tid) != 0)
        return -1;
      R->cur_voff = next_voff;
      R->cur_tid = next_tid;
    }
    auto *bam = new ganon_bam();
    bam->ref_names = R->header.ref_names;
    bam->ref_name_off = R->header.ref_name_off;
    bam->ref_len = R->header.ref_len;
    if (records_to_columns(data.data(), 0, (int64_t)data.size(), bam, R->threads, &recs) != 0) {
      delete bam;
      return -1;
    }
    *out = bam;
    return 0;
  } catch (const std::bad_alloc &) {
    return set_err("out of memory decoding a BAM sequence");
  }
}

GANON_HOST_API int ganon_bam_reader_region(ganon_bam_reader *R, int32_t tid, int64_t beg, int64_t end,
                                           ganon_bam **out) {
  if (!R || !out) return set_err("null argument");
  *out = nullptr;
  if (tid < 0 || tid >= (int32_t)R->header.ref_len.size()) return set_err("tid out of range");
  if (!R->has_index) return set_err("region reads need the BAM index");
  if (beg < 0 || end < beg) return set_err("bad region");
  try {
    ScanBuf data(R);
    std::vector<int64_t> recs;
    RegionCall rq{tid, beg, end, 0};
    const int64_t first = R->index_beg[(size_t)tid];
    if (first >= 0 && end > beg) {
      // the first record that can overlap beg: the linear index entry of its 16 kb window (the
      // nearest filled one before it), never before the sequence's first record
      int64_t voff = first;
      const std::vector<int64_t> &lin = R->linear[(size_t)tid];
      for (int64_t w = std::min<int64_t>(beg >> 14, (int64_t)lin.size() - 1); w >= 0; --w)
        if (lin[(size_t)w] > 0) {
          voff = std::max(voff, lin[(size_t)w]);
          break;
        }
      const int64_t e = R->index_end[(size_t)tid];
      const int64_t span = e > voff ? (e >> 16) - (voff >> 16) : 0;
      const int64_t len = R->header.ref_len[(size_t)tid];
      const int64_t hint = len > 0 ? std::min<int64_t>(span, span * (end - beg) / len + (1 << 20)) : 0;
      // (with a region decoder the first window is the whole region's estimated span: the span from
      // voff covers [beg, len) — plus 1/32 and 1 MiB of margin, and two blocks past a sequence's end
      // for the next record that ends the region)
      int64_t dev_step = 0;
      if (R->rdec) {
        const int64_t rest = std::max<int64_t>(1, len - beg);
        dev_step = std::min<int64_t>({span + (1 << 17), span * std::min<int64_t>(end - beg, rest) / rest * 33 / 32 + (1 << 20),
                                      16 * R->chunk});
      }
      if (!R->rdec) data.reserve((size_t)hint * 7 / 2 + (4 << 20));
      if (scan_region(R, voff, tid, beg, end, hint, data, recs, R->rdec ? &rq : nullptr, dev_step) != 0) return -1;
    }
    auto *bam = new ganon_bam();
    bam->ref_names = R->header.ref_names;
    bam->ref_name_off = R->header.ref_name_off;
    bam->ref_len = R->header.ref_len;
    if (rq.done) {
      bam->ext = rq.cols;
      bam->ext_block = rq.block;
      bam->ext_free = R->rdec_release;
      *out = bam;
      return 0;
    }
    if (records_to_columns(data.data(), 0, (int64_t)data.size(), bam, R->threads, &recs) != 0) {
      delete bam;
      return -1;
    }
    *out = bam;
    return 0;
  } catch (const std::bad_alloc &) {
    return set_err("out of memory decoding a BAM region");
  }
}

GANON_HOST_API void ganon_bam_reader_close(ganon_bam_reader *R) {
  if (!R) return;
  if (R->map) munmap(const_cast<uint8_t *>(R->map), (size_t)R->fsize);
  if (R->pbuf) R->bfree(R->pbuf);
  if (R->cbuf) R->bfree(R->cbuf);
  if (R->fh) std::fclose(R->fh);
  delete R;
}

GANON_HOST_API int64_t ganon_fastq_format(int64_t n, const uint8_t *const *seq_buf, const uint8_t *seq_sel,
                                          const int64_t *seq_nib_off, const int32_t *seq_len,
                                          const uint8_t *reverse, const uint8_t *const *qual_buf,
                                          const uint8_t *qual_sel, const int64_t *qual_off,
                                          const int32_t *qual_len, const uint8_t *qual_rev,
                                          const char *names, const int64_t *name_off, const int32_t *name_len,
                                          const uint8_t *mate, char *out, int64_t cap) {
  static const char kNt16[] = "=ACMGRSVTWYHKDBN";
  // reverses (anonymizer_methods.py:22): A<->T, C<->G, N->N; others are unmapped (-> error)
  static const int8_t kComp[16] = {-1, 8, 4, -1, 2, -1, -1, -1, 1, -1, -1, -1, -1, -1, -1, 15};
  int64_t w = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t L = seq_len[i], Q = qual_len[i], NL = name_len[i];
    const int64_t need = 1 + NL + 3 + L + 3 + Q + 1;
    if (w + need > cap) return INT64_MIN;
    char *o = out + w;
    *o++ = '@';
    std::memcpy(o, names + name_off[i], (size_t)NL);
    o += NL;
    *o++ = '/';
    *o++ = (char)('0' + mate[i]);
    *o++ = '\n';
    const uint8_t *sb = seq_buf[seq_sel[i]];
    const int64_t s0 = seq_nib_off[i];
    if (!reverse[i]) {
      for (int32_t k = 0; k < L; ++k) {
        const int64_t ni = s0 + k;
        const int c = (ni & 1) ? (sb[ni >> 1] & 0xF) : (sb[ni >> 1] >> 4);
        *o++ = kNt16[c];
      }
    } else {
      for (int32_t k = L - 1; k >= 0; --k) {
        const int64_t ni = s0 + k;
        const int c = (ni & 1) ? (sb[ni >> 1] & 0xF) : (sb[ni >> 1] >> 4);
        const int rc = kComp[c];
        if (rc < 0) return -(i + 1);
        *o++ = kNt16[rc];
      }
    }
    *o++ = '\n';
    *o++ = '+';
    *o++ = '\n';
    const uint8_t *qb = qual_buf[qual_sel[i]] + qual_off[i];
    if (!qual_rev[i]) {
      for (int32_t k = 0; k < Q; ++k) *o++ = (char)(qb[k] + 33);
    } else {
      for (int32_t k = Q - 1; k >= 0; --k) *o++ = (char)(qb[k] + 33);
    }
    *o++ = '\n';
    w += need;
  }
  return w;
}

GANON_HOST_API void ganon_pack_nt16(const char *ascii, int64_t n, uint8_t *out) {
  int8_t lut[256];
  std::memset(lut, 15, sizeof lut);
  const char *codes = "=ACMGRSVTWYHKDBN";
  for (int i = 0; i < 16; ++i) {
    lut[(uint8_t)codes[i]] = (int8_t)i;
    if (codes[i] >= 'A' && codes[i] <= 'Z') lut[(uint8_t)(codes[i] - 'A' + 'a')] = (int8_t)i;
  }
  for (int64_t i = 0; i + 1 < n; i += 2)
    out[i >> 1] = (uint8_t)((lut[(uint8_t)ascii[i]] << 4) | lut[(uint8_t)ascii[i + 1]]);
  if (n & 1) out[n >> 1] = (uint8_t)(lut[(uint8_t)ascii[n - 1]] << 4);
}

// ---- SA tag entries per record (the object model's n_supplementaries, AM:103-106) ----
GANON_HOST_API int ganon_aux_sa_count(const uint8_t *aux, const int64_t *aux_off, const int32_t *aux_len, int64_t n,
                                      int32_t *out) {
  if (n < 0 || (n > 0 && (!aux_off || !aux_len || !out))) return -1;
  auto size_of = [](uint8_t t) -> int {
    switch (t) {
      case 'A': case 'c': case 'C': return 1;
      case 's': case 'S': return 2;
      case 'i': case 'I': case 'f': return 4;
      default: return 0;
    }
  };
  for (int64_t r = 0; r < n; ++r) {
    out[r] = -1;
    const uint8_t *a = aux + aux_off[r];
    const int64_t len = aux_len[r];
    int64_t j = 0;
    while (j + 3 <= len) {
      const uint8_t t0 = a[j], t1 = a[j + 1], ty = a[j + 2];
      j += 3;
      if (ty == 'Z' || ty == 'H') {
        int64_t k = j;
        while (k < len && a[k]) ++k;
        if (t0 == 'S' && t1 == 'A' && ty == 'Z') {
          // len(value.rstrip(';').split(';'))
          int64_t e = k;
          while (e > j && a[e - 1] == ';') --e;
          int32_t c = 1;
          for (int64_t x = j; x < e; ++x) c += a[x] == ';';
          out[r] = c;
        }
        j = k + 1;
      } else if (ty == 'B') {
        if (j + 5 > len) break;
        const int sz = size_of(a[j]);
        int32_t cnt;
        std::memcpy(&cnt, a + j + 1, 4);
        j += 5 + (int64_t)sz * cnt;
      } else {
        const int sz = size_of(ty);
        if (!sz) break;   // malformed: leave the rest
        j += sz;
      }
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Indel left-overs on formatted records: mask_or_anonymize_left_over_variants (AM:254-270, edits
// stably sorted by VariantType value, offsets not shifted between edits) and
// mask_or_modify_indel (AM:178-203) on the stored-orientation sequence and the *forward-oriented*
// qualities, then get_anonymized_fastq_record (AM:205-243) again. The input record is
// the unedited one the formatter wrote, so the stored sequence and qualities are recovered from it.
GANON_HOST_API int ganon_fastq_edit(int64_t n, const char *recs, const int64_t *rec_off, const uint8_t *reverse,
                                    const int32_t *times, const int64_t *edit_off, const int64_t *edits,
                                    const char *alleles, const int64_t *allele_off, char *out, int64_t cap,
                                    int64_t *out_len, int64_t *bad) {
  if (n < 0 || (n > 0 && (!recs || !rec_off || !reverse || !times || !edit_off || !out_len || !bad)) ||
      (n > 0 && edit_off[n] > edit_off[0] && (!edits || !allele_off)))
    return -1;
  *bad = -1;
  uint8_t kComp[256] = {};
  kComp['A'] = 'T', kComp['C'] = 'G', kComp['G'] = 'C', kComp['T'] = 'A', kComp['N'] = 'N';
  std::string seq, s2;
  std::vector<int64_t> qual, q2;
  std::vector<int64_t> order;
  int64_t w = 0;
  for (int64_t i = 0; i < n; ++i) {
    const char *r = recs + rec_off[i];
    const int64_t rl = rec_off[i + 1] - rec_off[i];
    const char *e1 = (const char *)memchr(r, '\n', (size_t)rl);
    if (!e1) return -1;
    const int64_t hl = e1 - r + 1;                      // "@name/m\n"
    const int64_t L = (rl - hl - 4) / 2;                // seq \n + \n qual \n
    if (L < 0 || hl + 2 * L + 4 != rl) return -1;
    const char *ps = r + hl, *pq = ps + L + 3;
    const bool rev = reverse[i] != 0;
    seq.assign(ps, (size_t)L);
    qual.resize((size_t)L);
    for (int64_t k = 0; k < L; ++k) qual[k] = (uint8_t)(pq[k] - 33);
    if (rev) {                                          // printed = revcomp(stored), qualities stored order
      std::reverse(seq.begin(), seq.end());
      for (auto &c : seq) c = (char)kComp[(uint8_t)c];
      std::reverse(qual.begin(), qual.end());           // forward-oriented qualities (Q1)
    }
    order.clear();
    for (int64_t e = edit_off[i]; e < edit_off[i + 1]; ++e) order.push_back(e);
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return edits[3 * a + 1] < edits[3 * b + 1]; });
    for (int t = 0; t < times[i]; ++t) {
      for (int64_t e : order) {
        const int64_t type = edits[3 * e + 1], len = edits[3 * e + 2];
        const int64_t S = (int64_t)seq.size(), Q = (int64_t)qual.size();
        auto clampp = [](int64_t p, int64_t size) { return p < 0 ? std::max<int64_t>(0, p + size) : std::min(p, size); };
        const int64_t irp = edits[3 * e];
        if (type == 3) {                                // INS: seq[:irp] + seq[irp + len:]
          const int64_t a = clampp(irp, S), b = clampp(irp + len, S);
          s2.assign(seq, 0, (size_t)a);
          s2.append(seq, (size_t)b, std::string::npos);
          const int64_t qa = clampp(irp, Q), qb = clampp(irp + len, Q);
          q2.assign(qual.begin(), qual.begin() + qa);
          q2.insert(q2.end(), qual.begin() + qb, qual.end());
          seq.swap(s2);
          qual.swap(q2);
        } else if (type == 2) {                         // DEL: ref allele and `len` average qualities at irp
          if (Q == 0) {
            *bad = i;
            return 3;                                   // int(nan): ValueError
          }
          int64_t sum = 0;
          for (int64_t v : qual) sum += v;
          const int64_t avg = (int64_t)((double)sum / (double)Q);
          const int64_t a = clampp(irp, S), qa = clampp(irp, Q);
          seq.insert((size_t)a, alleles + allele_off[e], (size_t)(allele_off[e + 1] - allele_off[e]));
          qual.insert(qual.begin() + qa, (size_t)std::max<int64_t>(0, len), avg);
        }
        if (seq.size() != qual.size()) {
          *bad = i;
          return 2;                                     // lengths diverge: ValueError
        }
      }
    }
    const int64_t L2 = (int64_t)seq.size();
    for (int64_t v : qual)
      if (v < 0 || v > 255) {                           // bytes(qual) refuses it
        *bad = i;
        return 2;
      }
    if (rev) {
      for (auto c : seq)
        if (!kComp[(uint8_t)c]) {
          *bad = i;
          return 1;                                     // reverse complement of a non-ACGTN base (Q7)
        }
      std::reverse(seq.begin(), seq.end());
      for (auto &c : seq) c = (char)kComp[(uint8_t)c];
      std::reverse(qual.begin(), qual.end());
    }
    const int64_t need = hl + 2 * L2 + 4;
    if (w + need > cap) return -2;
    char *o = out + w;
    memcpy(o, r, (size_t)hl);
    o += hl;
    memcpy(o, seq.data(), (size_t)L2);
    o += L2;
    memcpy(o, "\n+\n", 3);
    o += 3;
    for (int64_t k = 0; k < L2; ++k) o[k] = (char)((qual[k] + 33) & 0xFF);
    o += L2;
    *o = '\n';
    out_len[i] = need;
    w += need;
  }
  return 0;
}

// Byte ranges of `src` back to back into `dst` (the output stage's splice of pre-formatted
// records); threads for large copies. Returns the bytes written, -1 on bad arguments.
static int64_t gather_impl(const char *const *src, const int64_t *src_len, int n_src, int64_t n, const uint8_t *sel,
                           const int64_t *off, const int64_t *len, char *dst, int64_t cap) {
  if (n < 0 || (n > 0 && (!off || !len || !dst))) return -1;
  for (int k = 0; k < n_src; ++k)
    if (n > 0 && !src[k] && src_len[k] > 0) return -1;
  std::vector<int64_t> at((size_t)n + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int k = sel ? sel[i] : 0;
    if (k >= n_src || off[i] < 0 || len[i] < 0 || off[i] + len[i] > src_len[k]) return -1;
    at[i + 1] = at[i] + len[i];
  }
  if (at[n] > cap) return -1;
  auto work = [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i)
      if (len[i]) memcpy(dst + at[i], src[sel ? sel[i] : 0] + off[i], (size_t)len[i]);
  };
  const int nt = (int)std::min<int64_t>(8, std::max<int64_t>(1, at[n] >> 23));   // one thread per 8 MiB
  if (nt == 1) {
    work(0, n);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(work, n * t / nt, n * (t + 1) / nt);
    for (auto &th : pool) th.join();
  }
  return at[n];
}

GANON_HOST_API int64_t ganon_gather_ranges(const char *src, int64_t src_len, int64_t n, const int64_t *off,
                                           const int64_t *len, char *dst, int64_t cap) {
  if (n > 0 && !src) return -1;
  return gather_impl(&src, &src_len, 1, n, nullptr, off, len, dst, cap);
}

GANON_HOST_API int64_t ganon_gather_ranges2(const char *src0, int64_t len0, const char *src1, int64_t len1, int64_t n,
                                            const uint8_t *sel, const int64_t *off, const int64_t *len, char *dst,
                                            int64_t cap) {
  if (n > 0 && !sel) return -1;
  const char *src[2] = {src0, src1};
  const int64_t sl[2] = {len0, len1};
  return gather_impl(src, sl, 2, n, sel, off, len, dst, cap);
}

GANON_HOST_API int ganon_host_phase_times(double *out, int n, int reset) {
  const int k = std::min(n, (int)kPhN);
  for (int i = 0; i < k; ++i)
    out[i] = (reset ? g_phase_ns[i].exchange(0) : g_phase_ns[i].load()) * 1e-9;
  // then two counts: region reads the device decoder finished / handed back to the host's walk
  if (n > kPhN) out[kPhN] = (double)(reset ? g_dev_regions.exchange(0) : g_dev_regions.load());
  if (n > kPhN + 1) out[kPhN + 1] = (double)(reset ? g_dev_fallbacks.exchange(0) : g_dev_fallbacks.load());
  return (int)kPhN + 2;
}

GANON_HOST_API const char *ganon_host_inflate_backend(void) { return libdeflate() ? "libdeflate" : "zlib"; }
