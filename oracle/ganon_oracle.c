/*
 * ganon_oracle.c — CPU restatement of the reference's per-scope SNV classification and
 * masking, over the same batch layout as include/ganon.h.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline. The product (genomeanonymizer_amd) never links or calls it.
 *
 * What it restates, per scope (one CompleteGermlineAnonymizer.anonymize call):
 *  - pileup column order: ascending reference position, tumor column before normal
 *    column at a tie (pileup_io.pyx:21-41, anonymizer_methods.py:440-451);
 *  - process_snv (variation_classifier.py:144-182): for each aligned base with
 *    query_position != None, skip if base == 'N', base == ref, or ref not in ACGT; else
 *    find-or-create the call (pos, allele) and advance the SomaticVariationType state
 *    machine (variants.py:33-39) with the read's dataset;
 *  - at every normal column, mask_germline_variants (anonymizer_methods.py:537-556):
 *    each call at that position in state TUMORAL_NORMAL_VARIANT that is not the kept
 *    variant has every supporting read's base at var_read_pos set to the reference base
 *    (mask_or_modify_base_pair :170-176) and is counted for the statistics (:555-556).
 * The masked sequence that reaches the output is the one of the AnonymizedRead object of
 * the scope given by write_scope (the object the host writer emits).
 *
 * Build: make -C oracle  (plain gcc, no dependencies).
 */
#include <stdint.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ganon.h"

enum { UNCLASSIFIED = 0, NORMAL_SINGLE = 1, TUMORAL_SINGLE = 2, NORMAL_ONLY = 3,
       TUMORAL_ONLY = 4, TUMORAL_NORMAL = 5 };

typedef struct {
  int32_t pos;
  int32_t read;   /* read index (the supporting_reads key: name;pair, unique per read) */
  int32_t qpos;
  uint8_t allele; /* nt16 code */
  uint8_t dataset;
} obs_t;

static int nib(const uint8_t *buf, int64_t nibble_index) {
  uint8_t b = buf[nibble_index >> 1];
  return (nibble_index & 1) ? (b & 0xF) : (b >> 4);
}

static void set_nib(uint8_t *buf, int64_t nibble_index, int v) {
  uint8_t *b = &buf[nibble_index >> 1];
  if (nibble_index & 1) *b = (uint8_t)((*b & 0xF0) | v);
  else *b = (uint8_t)((*b & 0x0F) | (v << 4));
}

static int is_acgt(int code) { return code == 1 || code == 2 || code == 4 || code == 8; }

static int cmp_obs(const void *a, const void *b) {
  const obs_t *x = (const obs_t *)a, *y = (const obs_t *)b;
  if (x->pos != y->pos) return x->pos < y->pos ? -1 : 1;
  if (x->dataset != y->dataset) return x->dataset < y->dataset ? -1 : 1; /* T column first */
  if (x->allele != y->allele) return x->allele < y->allele ? -1 : 1;
  return x->read < y->read ? -1 : (x->read > y->read);
}

static int advance(int state, int dataset) {
  /* variation_classifier.py:163-182 */
  if (state == UNCLASSIFIED) return dataset == 0 ? TUMORAL_SINGLE : NORMAL_SINGLE;
  if (dataset == 0) {
    if (state == NORMAL_SINGLE || state == NORMAL_ONLY) return TUMORAL_NORMAL;
    if (state == TUMORAL_SINGLE) return TUMORAL_ONLY;
  } else {
    if (state == TUMORAL_SINGLE || state == TUMORAL_ONLY) return TUMORAL_NORMAL;
    if (state == NORMAL_SINGLE) return NORMAL_ONLY;
  }
  return state;
}

/* Aligned (M/=/X) bases of read r: calls emit(p, q). */
static int64_t collect_obs(const ganon_batch *b, int32_t s, int32_t r, obs_t *out) {
  const int64_t ss = b->scope_span_start[s];
  const int64_t se = ss + b->scope_span_len[s];
  int64_t n = 0;
  int64_t p = b->ref_start[r];
  int64_t q = 0;
  const int64_t sq0 = b->seq_off[r] * 2;
  const uint32_t *cig = b->cigar + b->cig_off[r];
  for (int k = 0; k < b->n_cig[r]; ++k) {
    int op = cig[k] & 0xF;
    int64_t len = cig[k] >> 4;
    if (op == 0 || op == 7 || op == 8) {
      for (int64_t i = 0; i < len; ++i) {
        int64_t pp = p + i, qq = q + i;
        if (qq >= b->read_len[r] || pp < ss || pp >= se) continue;
        int c = nib(b->seq_nt16, sq0 + qq);
        int rc = nib(b->ref_nt16, b->scope_ref_off[s] + (pp - ss));
        if (c == 15 || c == rc || !is_acgt(rc)) continue;
        out[n].pos = (int32_t)pp; out[n].read = r; out[n].qpos = (int32_t)qq;
        out[n].allele = (uint8_t)c; out[n].dataset = b->dataset[r];
        ++n;
      }
      p += len; q += len;
    } else if (op == 1 || op == 4) {
      q += len;
    } else if (op == 2 || op == 3) {
      p += len;
    }
  }
  return n;
}

/* Scopes [s0, s1): classify and mask (seq_out already holds the input copy). A read is masked
 * only by its write scope and every read starts on a byte boundary, so disjoint scope ranges
 * write disjoint bytes (the multi-threaded baseline relies on it). */
static int mask_scopes(const ganon_batch *b, int32_t s0, int32_t s1, uint8_t *seq_out, int32_t *scope_calls,
                       int32_t *scope_bases, int64_t *tot) {
  int64_t cap = 0;
  obs_t *obs = NULL;
  for (int32_t s = s0; s < s1; ++s) {
    int64_t need = 0;
    for (int64_t i = b->scope_incid_off[s]; i < b->scope_incid_off[s + 1]; ++i)
      need += b->read_len[b->incid_read[i]];
    if (need > cap) {
      free(obs);
      cap = need + 1024;
      obs = (obs_t *)malloc(sizeof(obs_t) * (size_t)cap);
      if (!obs) return GANON_E_NOMEM;
    }
    int64_t n = 0;
    for (int64_t i = b->scope_incid_off[s]; i < b->scope_incid_off[s + 1]; ++i)
      n += collect_obs(b, s, b->incid_read[i], obs + n);
    qsort(obs, (size_t)n, sizeof(obs_t), cmp_obs);
    int32_t calls = 0, bases = 0;
    /* walk positions; per position the calls are the distinct alleles observed there */
    for (int64_t i = 0; i < n;) {
      int64_t j = i;
      while (j < n && obs[j].pos == obs[i].pos) ++j;
      /* state machine per allele in column order (T observations then N observations) */
      int state[16];
      memset(state, 0, sizeof(state));
      for (int64_t k = i; k < j; ++k) state[obs[k].allele] = advance(state[obs[k].allele], obs[k].dataset);
      int has_normal = 0;
      for (int64_t k = i; k < j; ++k) has_normal |= obs[k].dataset == 1;
      /* masking happens at the normal column of this position; TN needs a normal
       * observation so the column exists whenever a call can be TN */
      if (has_normal) {
        for (int a = 0; a < 16; ++a) {
          if (state[a] != TUMORAL_NORMAL) continue;
          if (b->keep_pos[s] == obs[i].pos && b->keep_code[s] == a) continue;
          ++calls;
          int rc = nib(b->ref_nt16, b->scope_ref_off[s] + (obs[i].pos - b->scope_span_start[s]));
          for (int64_t k = i; k < j; ++k) {
            if (obs[k].allele != a) continue;
            int32_t r = obs[k].read;
            if (b->write_scope[r] != s) continue; /* another scope's AnonymizedRead object */
            set_nib(seq_out, b->seq_off[r] * 2 + obs[k].qpos, rc);
            ++bases;
          }
        }
      }
      i = j;
    }
    if (scope_calls) scope_calls[s] = calls;
    if (scope_bases) scope_bases[s] = bases;
    tot[GANON_T_MASKED_SNV_CALLS] += calls;
    tot[GANON_T_MASKED_BASES] += bases;
  }
  free(obs);
  return GANON_OK;
}

static void static_totals(const ganon_batch *b, int64_t *tot) {
  memset(tot, 0, sizeof(int64_t) * GANON_N_TOTALS);
  tot[GANON_T_READS_IN] = b->n_reads;
  tot[GANON_T_SCOPES] = b->n_scopes;
  for (int32_t r = 0; r < b->n_reads; ++r) tot[GANON_T_READS_WRITTEN] += b->write_scope[r] >= 0;
}

int oracle_mask_batch(const ganon_batch *b, uint8_t *seq_out, int32_t *scope_calls,
                      int32_t *scope_bases, int64_t *totals) {
  if (!b || !seq_out) return GANON_E_ARG;
  memcpy(seq_out, b->seq_nt16, (size_t)b->seq_bytes);
  int64_t tot[GANON_N_TOTALS];
  static_totals(b, tot);
  const int rc = mask_scopes(b, 0, b->n_scopes, seq_out, scope_calls, scope_bases, tot);
  if (rc) return rc;
  if (totals) memcpy(totals, tot, sizeof(tot));
  return GANON_OK;
}

typedef struct {
  const ganon_batch *b;
  int32_t s0, s1;
  uint8_t *seq_out;
  int32_t *calls, *bases;
  int64_t tot[GANON_N_TOTALS];
  int rc;
} shard_t;

static void *shard_main(void *arg) {
  shard_t *w = (shard_t *)arg;
  memset(w->tot, 0, sizeof(w->tot));
  w->rc = mask_scopes(w->b, w->s0, w->s1, w->seq_out, w->calls, w->bases, w->tot);
  return NULL;
}

/* The same results on `threads` POSIX threads, each over a contiguous range of scopes (SURVEY
 * §8(d) "ref-cpu-N": the CPU path on all of a host's cores). */
int oracle_mask_batch_mt(const ganon_batch *b, uint8_t *seq_out, int32_t *scope_calls, int32_t *scope_bases,
                         int64_t *totals, int threads) {
  if (!b || !seq_out || threads < 1) return GANON_E_ARG;
  if (threads > 256) threads = 256;
  memcpy(seq_out, b->seq_nt16, (size_t)b->seq_bytes);
  int64_t tot[GANON_N_TOTALS];
  static_totals(b, tot);
  shard_t w[256];
  pthread_t th[256];
  for (int t = 0; t < threads; ++t) {
    w[t].b = b;
    w[t].s0 = (int32_t)((int64_t)b->n_scopes * t / threads);
    w[t].s1 = (int32_t)((int64_t)b->n_scopes * (t + 1) / threads);
    w[t].seq_out = seq_out;
    w[t].calls = scope_calls;
    w[t].bases = scope_bases;
    if (pthread_create(&th[t], NULL, shard_main, &w[t]) != 0) return GANON_E_NOMEM;
  }
  int rc = GANON_OK;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    if (w[t].rc) rc = w[t].rc;
    tot[GANON_T_MASKED_SNV_CALLS] += w[t].tot[GANON_T_MASKED_SNV_CALLS];
    tot[GANON_T_MASKED_BASES] += w[t].tot[GANON_T_MASKED_BASES];
  }
  if (rc) return rc;
  if (totals) memcpy(totals, tot, sizeof(tot));
  return GANON_OK;
}
