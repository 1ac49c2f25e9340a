// sanitize_driver.cpp — TEST INFRASTRUCTURE: runs the host-side C/C++ code that parses untrusted
// input or walks untrusted indices — the BGZF/BAM decoder and FASTQ formatter
// (genomeanonymizer_amd/csrc/ganon_host.cpp), the scope planner (csrc/ganon_plan.cpp) and the C
// oracle (oracle/ganon_oracle.c) — in one executable built with -fsanitize=address,undefined
// (tests/test_sanitizers.py). Any sanitizer report aborts with a non-zero status.
//
//   sanitize_driver bam FILE...                 decode each file (malformed ones must fail cleanly)
//   sanitize_driver plan T.bam N.bam SPEC       plan a pair, replay its I/O log, format every record
//   sanitize_driver oracle SEED                 mask a random batch (single- and multi-threaded)
//   sanitize_driver edit SEED                   indel left-overs on random (and malformed) records, range gathers
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/ganon.h"
#include "../../include/ganon_host.h"

extern "C" int oracle_mask_batch(const ganon_batch *b, uint8_t *seq_out, int32_t *scope_calls, int32_t *scope_bases,
                                 int64_t *totals);
extern "C" int oracle_mask_batch_mt(const ganon_batch *b, uint8_t *seq_out, int32_t *scope_calls,
                                    int32_t *scope_bases, int64_t *totals, int threads);

static uint64_t touch(const ganon_bam_view &v) {
  uint64_t h = 0;
  for (int64_t i = 0; i < v.n_records; ++i) {
    h += (uint64_t)v.tid[i] + v.pos[i] + v.end[i] + v.flag[i] + v.l_seq[i] + v.n_cigar[i] + v.mate_tid[i];
    h += (uint64_t)v.names[v.name_off[i]] + v.name_len[i];
    for (int k = 0; k < v.n_cigar[i]; ++k) h += v.cigar[v.cig_off[i] + k];
    for (int k = 0; k < (v.l_seq[i] + 1) / 2; ++k) h += v.seq[v.seq_off[i] + k];
    for (int k = 0; k < v.l_seq[i]; ++k) h += v.qual[v.qual_off[i] + k];
    for (int k = 0; k < v.aux_len[i]; ++k) h += v.aux[v.aux_off[i] + k];
  }
  return h;
}

static int run_bam(int argc, char **argv) {
  int ok = 0, bad = 0;
  for (int a = 0; a < argc; ++a) {
    ganon_bam *b = nullptr;
    if (ganon_bam_open(argv[a], 4, &b) != 0) {
      ++bad;
      continue;
    }
    ganon_bam_view v;
    if (ganon_bam_view_get(b, &v) == 0) std::printf("%s %lld records %llu\n", argv[a], (long long)v.n_records,
                                                  (unsigned long long)touch(v));
    ganon_bam_close(b);
    ++ok;
  }
  std::printf("decoded %d rejected %d\n", ok, bad);
  return 0;
}

// SPEC: n_contigs, then "name length" lines, then n_windows, then "contig first last" lines.
static int run_plan(char **argv) {
  ganon_bam *bam[2] = {nullptr, nullptr};
  ganon_bam_view v[2];
  for (int d = 0; d < 2; ++d) {
    if (ganon_bam_open(argv[d], 4, &bam[d]) != 0 || ganon_bam_view_get(bam[d], &v[d]) != 0) {
      std::fprintf(stderr, "cannot decode %s: %s\n", argv[d], ganon_host_last_error());
      return 2;
    }
  }
  FILE *fh = std::fopen(argv[2], "r");
  if (!fh) return 2;
  int nc = 0, nw = 0;
  if (std::fscanf(fh, "%d", &nc) != 1) return 2;
  std::vector<std::string> names(nc);
  std::vector<int64_t> len(nc), name_off(nc);
  std::string blob;
  for (int c = 0; c < nc; ++c) {
    char buf[256];
    long long l;
    if (std::fscanf(fh, "%255s %lld", buf, &l) != 2) return 2;
    names[c] = buf;
    len[c] = l;
    name_off[c] = (int64_t)blob.size();
    blob += names[c];
    blob.push_back('\0');
  }
  if (std::fscanf(fh, "%d", &nw) != 1) return 2;
  std::vector<int32_t> wc(nw);
  std::vector<int64_t> wf(nw), wl(nw);
  for (int w = 0; w < nw; ++w) {
    long long f, l;
    if (std::fscanf(fh, "%d %lld %lld", &wc[w], &f, &l) != 3) return 2;
    wf[w] = f;
    wl[w] = l;
  }
  std::fclose(fh);
  ganon_plan_input in{};
  std::vector<int32_t> tid_of[2];
  for (int d = 0; d < 2; ++d) {
    tid_of[d].assign(nc, -1);
    for (int c = 0; c < nc; ++c)
      for (int t = 0; t < v[d].n_ref; ++t)
        if (names[c] == std::string(v[d].ref_names + v[d].ref_name_off[t])) tid_of[d][c] = t;
    ganon_plan_table &t = in.tables[d];
    t.n = v[d].n_records;
    t.tid = v[d].tid;
    t.pos = v[d].pos;
    t.end = v[d].end;
    t.flag = v[d].flag;
    t.l_seq = v[d].l_seq;
    t.n_cigar = v[d].n_cigar;
    t.names = v[d].names;
    t.name_off = v[d].name_off;
    t.name_len = v[d].name_len;
    t.n_ref = v[d].n_ref;
    t.ref_len = v[d].ref_len;
    t.tid_of_contig = tid_of[d].data();
  }
  in.n_contigs = nc;
  in.contig_len = len.data();
  in.contig_names = blob.c_str();
  in.contig_name_off = name_off.data();
  in.n_windows = nw;
  in.win_contig = wc.data();
  in.win_first = wf.data();
  in.win_last = wl.data();
  ganon_plan *plan = nullptr;
  if (ganon_plan_run(&in, &plan) != 0) {
    std::printf("plan rejected: %s\n", ganon_plan_last_error());
  } else {
    ganon_plan_view pv;
    ganon_plan_view_get(plan, &pv);
    std::vector<int64_t> rec_len((size_t)pv.n_events, 0), order((size_t)pv.n_events + 1, 0), file_count(4, 0);
    for (int64_t e = 0; e < pv.n_events; ++e)
      if (pv.events[7 * e] == 1) rec_len[e] = 300 + (e % 37);
    const int64_t w = ganon_io_replay(pv.n_events, pv.events, rec_len.data(), 4096, order.data(), file_count.data());
    std::printf("plan: %d scopes, %lld events, replay %lld\n", pv.n_scopes, (long long)pv.n_events, (long long)w);
    ganon_plan_free(plan);
  }
  // FASTQ records of every read of both samples, half of them reverse-complemented
  for (int d = 0; d < 2; ++d) {
    const int64_t n = v[d].n_records;
    std::vector<uint8_t> sel(n, 0), rev(n), qrev(n, 0), mate(n);
    std::vector<int64_t> nib(n);
    for (int64_t i = 0; i < n; ++i) {
      nib[i] = 2 * v[d].seq_off[i];
      rev[i] = (uint8_t)(i & 1);
      mate[i] = (uint8_t)(1 + (i & 1));
    }
    const uint8_t *sb[1] = {v[d].seq}, *qb[1] = {v[d].qual};
    int64_t bytes = 0;
    for (int64_t i = 0; i < n; ++i) bytes += 8 + v[d].name_len[i] + 2 * (int64_t)v[d].l_seq[i];
    std::vector<char> out((size_t)bytes + 1);
    const int64_t w = ganon_fastq_format(n, sb, sel.data(), nib.data(), v[d].l_seq, rev.data(), qb, sel.data(),
                                         v[d].qual_off, v[d].l_seq, qrev.data(), v[d].names, v[d].name_off,
                                         v[d].name_len, mate.data(), out.data(), bytes);
    std::printf("fastq %d: %lld bytes\n", d, (long long)w);
  }
  ganon_bam_close(bam[0]);
  ganon_bam_close(bam[1]);
  return 0;
}

// A random batch: scopes of reads with random CIGARs (M/I/D/N/S/H/=/X), bases over all 16 codes.
static int run_oracle(int seed) {
  std::mt19937_64 rng((uint64_t)seed);
  auto U = [&](int a, int b) { return (int)(a + rng() % (uint64_t)(b - a + 1)); };
  const int n_scopes = 40;
  std::vector<int32_t> ref_start, read_len, n_cig, write_scope, span_start, span_len, keep_pos, incid;
  std::vector<int64_t> seq_off, cig_off, incid_off{0}, ref_off;
  std::vector<uint8_t> seq, dataset, keep_code, ref;
  std::vector<uint32_t> cigar;
  const int region = 5000;
  for (int s = 0; s < n_scopes; ++s)
    for (int k = 0; k < region / 2; ++k) ref.push_back((uint8_t)((1 << U(0, 3)) << 4 | (1 << U(0, 3))));
  for (int s = 0; s < n_scopes; ++s) {
    const int nr = U(0, 30);
    int lo = 1 << 30, hi = 0;
    const size_t first = ref_start.size();
    for (int k = 0; k < nr; ++k) {
      const int pos = U(100, region - 1200);
      int q = 0, p = pos, L = 0;
      cig_off.push_back((int64_t)cigar.size());
      const int nops = U(1, 6);
      for (int o = 0; o < nops; ++o) {
        const int op = (int[]){0, 0, 0, 1, 2, 3, 4, 5, 7, 8}[U(0, 9)];
        const int len = U(0, 60);
        cigar.push_back((uint32_t)len << 4 | (uint32_t)op);
        if (op == 0 || op == 7 || op == 8) { q += len; p += len; }
        else if (op == 1 || op == 4) q += len;
        else if (op == 2 || op == 3) p += len;
      }
      L = q;
      n_cig.push_back(nops);
      ref_start.push_back(pos);
      read_len.push_back(L);
      seq_off.push_back((int64_t)seq.size());
      for (int b = 0; b < (L + 1) / 2; ++b) seq.push_back((uint8_t)rng());
      dataset.push_back((uint8_t)U(0, 1));
      write_scope.push_back(U(0, 9) < 8 ? s : -1);
      lo = std::min(lo, pos);
      hi = std::max(hi, std::max(p, pos + 1));
      incid.push_back((int32_t)(ref_start.size() - 1));
    }
    if (ref_start.size() == first) lo = hi = 0;
    incid_off.push_back((int64_t)incid.size());
    span_start.push_back(lo);
    span_len.push_back(hi - lo);
    ref_off.push_back((int64_t)s * region + lo);
    keep_pos.push_back(U(0, 1) ? lo + U(0, 50) : -1);
    keep_code.push_back((uint8_t)(1 << U(0, 3)));
  }
  ganon_batch b{};
  b.n_reads = (int32_t)ref_start.size();
  b.n_scopes = n_scopes;
  b.n_incid = (int64_t)incid.size();
  b.seq_bytes = (int64_t)seq.size();
  b.n_cigar_ops = (int64_t)cigar.size();
  b.ref_bytes = (int64_t)ref.size();
  b.ref_start = ref_start.data();
  b.read_len = read_len.data();
  b.seq_off = seq_off.data();
  b.seq_nt16 = seq.data();
  b.cig_off = cig_off.data();
  b.n_cig = n_cig.data();
  b.cigar = cigar.data();
  b.dataset = dataset.data();
  b.write_scope = write_scope.data();
  b.scope_incid_off = incid_off.data();
  b.incid_read = incid.data();
  b.scope_span_start = span_start.data();
  b.scope_span_len = span_len.data();
  b.scope_ref_off = ref_off.data();
  b.ref_nt16 = ref.data();
  b.keep_pos = keep_pos.data();
  b.keep_code = keep_code.data();
  std::vector<uint8_t> out(seq.size() + 1), out2(seq.size() + 1);
  std::vector<int32_t> calls(n_scopes), bases(n_scopes), calls2(n_scopes), bases2(n_scopes);
  int64_t tot[GANON_N_TOTALS], tot2[GANON_N_TOTALS];
  if (oracle_mask_batch(&b, out.data(), calls.data(), bases.data(), tot) != 0) return 3;
  if (oracle_mask_batch_mt(&b, out2.data(), calls2.data(), bases2.data(), tot2, 4) != 0) return 3;
  if (out != out2 || calls != calls2 || bases != bases2) return 4;
  std::printf("oracle seed %d: %lld calls %lld bases\n", seed, (long long)tot[0], (long long)tot[1]);
  return 0;
}

// Random records (some truncated or with a missing newline) and edits (positions past the read,
// negative lengths, empty reads) through ganon_fastq_edit; range gathers in and out of bounds.
static int run_edit(int seed) {
  std::mt19937_64 rng((uint64_t)seed);
  const char *bases = "ACGTNMR=";
  int ok = 0, refused = 0;
  for (int it = 0; it < 3000; ++it) {
    const int L = (int)(rng() % 40);
    const bool rev = rng() & 1;
    std::string rec = "@r" + std::to_string(it) + "/1\n";
    for (int k = 0; k < L; ++k) rec += bases[rng() % (rev ? 5 : 8)];
    rec += "\n+\n";
    for (int k = 0; k < L; ++k) rec += (char)(33 + rng() % 60);
    rec += "\n";
    if (rng() % 10 == 0) rec.resize(rng() % (rec.size() + 1));   // malformed: truncated
    const int ne = 1 + (int)(rng() % 3);
    std::vector<int64_t> edits, aoff{0};
    std::string alleles;
    for (int e = 0; e < ne; ++e) {
      const int64_t type = 2 + (int64_t)(rng() % 2), len = (int64_t)(rng() % 7) - 1;
      edits.push_back((int64_t)(rng() % (L + 6)) - 1);
      edits.push_back(type);
      edits.push_back(len);
      const int al = type == 2 ? (int)std::max<int64_t>(0, len + (int64_t)(rng() % 2)) : 0;
      for (int k = 0; k < al; ++k) alleles += bases[rng() % 4];
      aoff.push_back((int64_t)alleles.size());
    }
    const int64_t rec_off[2] = {0, (int64_t)rec.size()}, edit_off[2] = {0, ne};
    const uint8_t r8 = rev;
    const int32_t times = 1 + (int32_t)(rng() % 2);
    std::vector<char> out(rec.size() + 2 * (alleles.size() + 8 * ne) + 64);
    int64_t out_len = 0, bad = -1;
    const int rc = ganon_fastq_edit(1, rec.data(), rec_off, &r8, &times, edit_off, edits.data(), alleles.data(),
                                    aoff.data(), out.data(), (int64_t)out.size(), &out_len, &bad);
    if (rc == 0) {
      if (out_len < 0 || out_len > (int64_t)out.size()) return 1;
      ++ok;
    } else {
      ++refused;
    }
  }
  std::string src(1000, 'x');
  std::vector<int64_t> off{0, 10, 990}, len{5, 20, 10};
  std::vector<char> dst(64);
  if (ganon_gather_ranges(src.data(), (int64_t)src.size(), 3, off.data(), len.data(), dst.data(), 64) != 35) return 1;
  len[2] = 11;   // one byte past the source
  if (ganon_gather_ranges(src.data(), (int64_t)src.size(), 3, off.data(), len.data(), dst.data(), 64) != -1) return 1;
  std::printf("edit ok=%d refused=%d\n", ok, refused);
  return 0;
}

int main(int argc, char **argv) {
  if (argc >= 2 && !std::strcmp(argv[1], "bam")) return run_bam(argc - 2, argv + 2);
  if (argc >= 5 && !std::strcmp(argv[1], "plan")) return run_plan(argv + 2);
  if (argc >= 3 && !std::strcmp(argv[1], "oracle")) return run_oracle(std::atoi(argv[2]));
  if (argc >= 3 && !std::strcmp(argv[1], "edit")) return run_edit(std::atoi(argv[2]));
  std::fprintf(stderr, "usage: sanitize_driver bam FILE... | plan T.bam N.bam SPEC | oracle SEED\n");
  return 2;
}
