// ganon_host.cpp — BGZF/BAM decoder to SoA columns and FASTQ formatter (libganon_host.so).
// See include/ganon_host.h. Written from the SAM/BAM v1 specification.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ganon_host.h"

namespace {

thread_local std::string g_err;

// memcpy of n bytes; n == 0 (an empty blob's data() may be null) copies nothing
inline void copy_bytes(void *dst, const void *src, size_t n) {
  if (n) std::memcpy(dst, src, n);
}

struct Block {
  int64_t in_off;   // compressed payload offset in the file buffer
  int32_t in_len;   // compressed payload length
  int32_t out_len;  // ISIZE
  int64_t out_off;  // offset in the inflated stream
};

bool inflate_raw(const uint8_t *in, int32_t in_len, uint8_t *out, int32_t out_len) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, -15) != Z_OK) return false;
  zs.next_in = const_cast<Bytef *>(in);
  zs.avail_in = (uInt)in_len;
  zs.next_out = out;
  zs.avail_out = (uInt)out_len;
  int rc = inflate(&zs, Z_FINISH);
  const bool ok = (rc == Z_STREAM_END) && zs.total_out == (uLong)out_len;
  inflateEnd(&zs);
  return ok;
}

}  // namespace

struct ganon_bam {
  std::string err;
  std::vector<char> ref_names;
  std::vector<int64_t> ref_name_off, ref_len;
  std::vector<int32_t> tid, pos, end, flag, mapq, l_seq, n_cigar, mate_tid, mate_pos, tlen, name_len, aux_len;
  std::vector<int64_t> name_off, cig_off, seq_off, qual_off, aux_off;
  std::vector<char> names;
  std::vector<uint32_t> cigar;
  std::vector<uint8_t> seq, qual, aux;
};

static int set_err(const std::string &m) {
  g_err = m;
  return -1;
}

GANON_HOST_API const char *ganon_host_last_error(void) { return g_err.c_str(); }

static int bam_open_impl(const char *path, int threads, ganon_bam **out) {
  FILE *fh = std::fopen(path, "rb");
  if (!fh) return set_err(std::string("cannot open ") + path);
  std::fseek(fh, 0, SEEK_END);
  const long fsize = std::ftell(fh);
  std::fseek(fh, 0, SEEK_SET);
  std::vector<uint8_t> file((size_t)std::max(0L, fsize));
  if (fsize > 0 && std::fread(file.data(), 1, (size_t)fsize, fh) != (size_t)fsize) {
    std::fclose(fh);
    return set_err("short read");
  }
  std::fclose(fh);
  // ---- BGZF block table (untrusted input: every field is checked before it is used) ----
  std::vector<Block> blocks;
  int64_t off = 0, total = 0;
  const int64_t fsz = (int64_t)file.size();
  while (off < fsz) {
    if (off + 18 > fsz) return set_err("truncated BGZF header");
    const uint8_t *h = &file[off];
    if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return set_err("not a BGZF file");
    const int xlen = h[10] | (h[11] << 8);
    // the extra field and the 8-byte CRC32/ISIZE trailer must lie inside the file
    if (off + 12 + xlen + 8 > fsz) return set_err("truncated BGZF extra field");
    int bsize = -1;
    for (int x = 12; x < 12 + xlen;) {
      if (x + 4 > 12 + xlen) return set_err("malformed BGZF extra subfield");
      const int slen = h[x + 2] | (h[x + 3] << 8);
      if (x + 4 + slen > 12 + xlen) return set_err("malformed BGZF extra subfield");
      if (h[x] == 66 && h[x + 1] == 67 && slen == 2) bsize = h[x + 4] | (h[x + 5] << 8);
      x += 4 + slen;
    }
    if (bsize < 0) return set_err("BGZF block without BC subfield");
    const int64_t blen = (int64_t)bsize + 1;
    if (off + blen > fsz) return set_err("truncated BGZF block");
    const int64_t in_len = blen - 12 - xlen - 8;
    if (in_len < 0) return set_err("BGZF block size smaller than its header");
    Block b;
    b.in_off = off + 12 + xlen;
    b.in_len = (int32_t)in_len;
    uint32_t isize;
    std::memcpy(&isize, &file[off + blen - 4], 4);
    if (isize > 65536) return set_err("BGZF block ISIZE over 64 KiB");
    b.out_len = (int32_t)isize;
    b.out_off = total;
    total += isize;
    if (b.out_len > 0) blocks.push_back(b);
    off += blen;
  }
  std::vector<uint8_t> data((size_t)total);
  std::atomic<int64_t> next{0};
  std::atomic<bool> bad{false};
  const int nt = std::max(1, std::min(threads, 64));
  auto worker = [&]() {
    for (;;) {
      const int64_t i = next.fetch_add(1);
      if (i >= (int64_t)blocks.size() || bad.load()) return;
      const Block &b = blocks[i];
      if (!inflate_raw(&file[b.in_off], b.in_len, &data[b.out_off], b.out_len)) bad = true;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(worker);
  worker();
  for (auto &t : pool) t.join();
  if (bad) return set_err("BGZF inflate failed");
  file.clear();
  file.shrink_to_fit();
  // ---- BAM header ----
  auto *bam = new ganon_bam();
  auto die = [&](const char *m) {
    delete bam;
    return set_err(m);
  };
  const uint8_t *d = data.data();
  const int64_t n = (int64_t)data.size();
  if (n < 12 || std::memcmp(d, "BAM\1", 4) != 0) return die("not a BAM stream");
  int32_t l_text, n_ref;
  std::memcpy(&l_text, d + 4, 4);
  if (l_text < 0) return die("negative header text length");
  int64_t p = 8 + (int64_t)l_text;
  if (p + 4 > n) return die("truncated header");
  std::memcpy(&n_ref, d + p, 4);
  p += 4;
  if (n_ref < 0) return die("negative reference count");
  for (int32_t i = 0; i < n_ref; ++i) {
    int32_t l_name, l_ref;
    if (p + 4 > n) return die("truncated reference list");
    std::memcpy(&l_name, d + p, 4);
    p += 4;
    if (l_name <= 0 || p + l_name + 4 > n) return die("bad reference name");
    bam->ref_name_off.push_back((int64_t)bam->ref_names.size());
    bam->ref_names.insert(bam->ref_names.end(), d + p, d + p + l_name);
    bam->ref_names.back() = '\0';
    p += l_name;
    std::memcpy(&l_ref, d + p, 4);
    p += 4;
    bam->ref_len.push_back(l_ref);
  }
  // ---- records: boundaries (sequential), sizes + offsets, then columns in parallel ----
  std::vector<int64_t> rec;   // offset of each record's block_size field
  while (p < n) {
    int32_t bs;
    if (p + 4 > n) return die("truncated record size");
    std::memcpy(&bs, d + p, 4);
    if (bs < 32 || p + 4 + bs > n) return die("bad record size");
    rec.push_back(p);
    p += 4 + bs;
  }
  const int64_t nr = (int64_t)rec.size();
  // per record: name bytes kept, CIGAR ops, sequence length, aux bytes
  std::vector<int64_t> o_name(nr + 1), o_cig(nr + 1), o_seq(nr + 1), o_qual(nr + 1), o_aux(nr + 1);
  std::atomic<int64_t> first_bad{INT64_MAX};
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
  if (first_bad.load() != INT64_MAX) return die("record fields exceed block size");
  for (int64_t i = 0; i < nr; ++i) {
    o_name[i + 1] += o_name[i];
    o_cig[i + 1] += o_cig[i];
    o_seq[i + 1] += o_seq[i];
    o_qual[i + 1] += o_qual[i];
    o_aux[i + 1] += o_aux[i];
  }
  for (auto *v : {&bam->tid, &bam->pos, &bam->end, &bam->flag, &bam->mapq, &bam->l_seq, &bam->n_cigar, &bam->mate_tid,
                  &bam->mate_pos, &bam->tlen, &bam->name_len, &bam->aux_len})
    v->resize((size_t)nr);
  for (auto *v : {&bam->name_off, &bam->cig_off, &bam->seq_off, &bam->qual_off, &bam->aux_off}) v->resize((size_t)nr);
  bam->names.resize((size_t)o_name[nr]);
  bam->cigar.resize((size_t)o_cig[nr]);
  bam->seq.resize((size_t)o_seq[nr]);
  bam->qual.resize((size_t)o_qual[nr]);
  bam->aux.resize((size_t)o_aux[nr]);
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
