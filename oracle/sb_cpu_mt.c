/*
 * sb_cpu_mt.c -- multi-threaded CPU baseline over the oracle's page decoders.
 *
 * TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline legs): the reference's
 * src/read decoders are single-threaded per column (read/batch_read.rs:
 * 190-209 appends page after page); the all-cores leg shards a column's pages
 * into contiguous ranges, one per std::thread-like worker (pthreads here),
 * each running the oracle's restatement of the page reader
 * (orc_read_flat_page / orc_read_binary_page / orc_read_list_page /
 * orc_read_bool_page) into its share of the output, then merges what depends
 * on earlier shards (Utf8 value bases, list leaf bases, bitmaps at unaligned
 * bit offsets).  n_threads = 1 is the reference's single-threaded shape.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sb_oracle.h"

static void put_bits(uint8_t* dst, size_t at, const uint8_t* src, size_t n) {
  if ((at & 7) == 0) {
    memcpy(dst + at / 8, src, n / 8);
    for (size_t i = n & ~(size_t)7; i < n; i++) {
      size_t r = at + i;
      if ((src[i >> 3] >> (i & 7)) & 1) dst[r >> 3] |= (uint8_t)(1u << (r & 7));
      else dst[r >> 3] &= (uint8_t)~(1u << (r & 7));
    }
    return;
  }
  for (size_t i = 0; i < n; i++) {
    size_t r = at + i;
    if ((src[i >> 3] >> (i & 7)) & 1) dst[r >> 3] |= (uint8_t)(1u << (r & 7));
    else dst[r >> 3] &= (uint8_t)~(1u << (r & 7));
  }
}

/* contiguous page ranges balanced by bytes; for byte-aligned bitmaps a cut
 * only falls on a page whose first row is a multiple of 8 */
static size_t shard(const uint64_t* metas, size_t n_pages, int nt, int need_align, size_t* cut) {
  uint64_t total = 0;
  for (size_t p = 0; p < n_pages; p++) total += metas[2 * p];
  size_t k = 0, p = 0;
  uint64_t acc = 0, row = 0;
  cut[k++] = 0;
  for (int t = 1; t < nt; t++) {
    const uint64_t target = total * (uint64_t)t / (uint64_t)nt;
    while (p < n_pages && acc < target) {
      acc += metas[2 * p];
      row += metas[2 * p + 1];
      p++;
    }
    while (need_align && p < n_pages && (row & 7)) {
      acc += metas[2 * p];
      row += metas[2 * p + 1];
      p++;
    }
    if (p > cut[k - 1] && p < n_pages) cut[k++] = p;
  }
  cut[k] = n_pages;
  return k;
}

typedef struct {
  const uint8_t* chunk;
  const uint64_t* metas;
  size_t p0, p1;
  uint64_t byte0, row0;
  int kind, width, nullable, ow, ln, in;
  uint8_t* out_values;
  uint8_t* out_bits;
  /* binary */
  orc_binvec bv;
  uint8_t* tbits;
  /* list */
  int64_t* loffs;
  uint8_t* lbits;
  uint8_t* lvals;
  uint8_t* fbits;
  size_t rows, leaves;
  int rc;
} job_t;

static void* flat_worker(void* arg) {
  job_t* j = (job_t*)arg;
  uint64_t pos = j->byte0, row = j->row0;
  uint8_t* tmp = NULL;
  for (size_t p = j->p0; p < j->p1 && !j->rc; p++) {
    const uint64_t len = j->metas[2 * p], nv = j->metas[2 * p + 1];
    if (j->nullable) tmp = (uint8_t*)realloc(tmp, (nv + 7) / 8 + 1);
    j->rc = orc_read_flat_page(j->chunk + pos, len, nv, j->kind, j->width, j->nullable,
                               j->out_values + row * (uint64_t)j->width, tmp);
    if (!j->rc && j->nullable) put_bits(j->out_bits, row, tmp, nv);
    pos += len;
    row += nv;
  }
  free(tmp);
  return NULL;
}

static void run(job_t* jobs, size_t k, void* (*fn)(void*)) {
  pthread_t th[256];
  for (size_t t = 1; t < k; t++) pthread_create(&th[t], NULL, fn, &jobs[t]);
  fn(&jobs[0]);
  for (size_t t = 1; t < k; t++) pthread_join(th[t], NULL);
}

static size_t setup(job_t* jobs, const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int nt, int align) {
  size_t cut[257];
  if (nt < 1) nt = 1;
  if (nt > 256) nt = 256;
  size_t k = shard(metas, n_pages, nt, align, cut);
  uint64_t byte = 0, row = 0;
  size_t p = 0;
  for (size_t t = 0; t < k; t++) {
    memset(&jobs[t], 0, sizeof(job_t));
    jobs[t].chunk = chunk;
    jobs[t].metas = metas;
    jobs[t].p0 = cut[t];
    jobs[t].p1 = cut[t + 1];
    for (; p < cut[t]; p++) {
      byte += metas[2 * p];
      row += metas[2 * p + 1];
    }
    jobs[t].byte0 = byte;
    jobs[t].row0 = row;
  }
  return k;
}

/* read_integer / read_double over a column chunk, pages sharded over threads */
int orc_mt_read_column(const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int kind, int width, int nullable,
                       uint8_t* out_values, uint8_t* out_bits, int n_threads) {
  job_t jobs[256];
  size_t k = setup(jobs, chunk, metas, n_pages, n_threads, nullable);
  for (size_t t = 0; t < k; t++) {
    jobs[t].kind = kind;
    jobs[t].width = width;
    jobs[t].nullable = nullable;
    jobs[t].out_values = out_values;
    jobs[t].out_bits = out_bits;
  }
  run(jobs, k, flat_worker);
  for (size_t t = 0; t < k; t++)
    if (jobs[t].rc) return jobs[t].rc;
  return ORC_OK;
}

static void* bin_worker(void* arg) {
  job_t* j = (job_t*)arg;
  uint64_t pos = j->byte0, row = 0;
  for (size_t p = j->p0; p < j->p1 && !j->rc; p++) {
    const uint64_t len = j->metas[2 * p], nv = j->metas[2 * p + 1];
    uint8_t tmp[8192 / 8 + 8];
    uint8_t* bits = nv <= 8192 ? tmp : (uint8_t*)malloc((nv + 7) / 8 + 1);
    j->rc = orc_read_binary_page(j->chunk + pos, len, nv, j->nullable, j->ow, &j->bv, bits);
    if (!j->rc && j->nullable) put_bits(j->tbits, row, bits, nv);
    if (bits != tmp) free(bits);
    pos += len;
    row += nv;
  }
  j->rows = row;
  return NULL;
}

/* read_binary (read/array/binary.rs:223-265): offsets (ow bytes each, rows + 1)
 * and values; *values_len = bytes written.  values_cap bounds out_values. */
int orc_mt_read_binary_column(const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int nullable, int ow,
                              uint8_t* out_offsets, uint8_t* out_values, uint64_t values_cap, uint8_t* out_bits,
                              int n_threads, uint64_t* values_len) {
  job_t jobs[256];
  size_t k = setup(jobs, chunk, metas, n_pages, n_threads, 0);
  for (size_t t = 0; t < k; t++) {
    jobs[t].nullable = nullable;
    jobs[t].ow = ow;
    uint64_t rows = 0;
    for (size_t p = jobs[t].p0; p < jobs[t].p1; p++) rows += metas[2 * p + 1];
    jobs[t].tbits = nullable ? (uint8_t*)calloc(rows / 8 + 2, 1) : NULL;
  }
  run(jobs, k, bin_worker);
  int rc = ORC_OK;
  uint64_t vbase = 0;
  for (size_t t = 0; t < k && !rc; t++) {
    job_t* j = &jobs[t];
    if (j->rc) { rc = j->rc; break; }
    if (vbase + j->bv.n_val > values_cap) { rc = ORC_E_ARG; break; }
    memcpy(out_values + vbase, j->bv.values, j->bv.n_val);
    const size_t first = t == 0 ? 0 : 1;  /* later shards drop their leading 0 */
    for (size_t i = first; i < j->bv.n_off; i++) {
      const int64_t v = j->bv.offsets[i] + (int64_t)vbase;
      const uint64_t r = j->row0 + i;
      if (ow == 8) memcpy(out_offsets + r * 8, &v, 8);
      else { int32_t w = (int32_t)v; memcpy(out_offsets + r * 4, &w, 4); }
    }
    if (nullable) put_bits(out_bits, j->row0, j->tbits, j->rows);
    vbase += j->bv.n_val;
  }
  for (size_t t = 0; t < k; t++) {
    orc_binvec_free(&jobs[t].bv);
    free(jobs[t].tbits);
  }
  *values_len = vbase;
  return rc;
}

static void* list_worker(void* arg) {
  job_t* j = (job_t*)arg;
  uint64_t pos = j->byte0;
  size_t rows = 0, leaves = 0, cap_r = 0, cap_l = 0;
  for (size_t p = j->p0; p < j->p1 && !j->rc; p++) {
    const uint64_t len = j->metas[2 * p], nlev = j->metas[2 * p + 1];
    if (rows + nlev + 1 > cap_r) {
      cap_r = 2 * (rows + nlev + 1);
      j->loffs = (int64_t*)realloc(j->loffs, cap_r * 8);
      j->lbits = (uint8_t*)realloc(j->lbits, cap_r / 8 + 2);
    }
    if (leaves + nlev + 1 > cap_l) {
      cap_l = 2 * (leaves + nlev + 1);
      j->lvals = (uint8_t*)realloc(j->lvals, cap_l * (size_t)j->width);
      j->fbits = (uint8_t*)realloc(j->fbits, cap_l / 8 + 2);
    }
    int64_t* po = (int64_t*)malloc((nlev + 1) * 8);
    uint8_t* pl = (uint8_t*)calloc(nlev / 8 + 2, 1);
    uint8_t* pf = (uint8_t*)calloc(nlev / 8 + 2, 1);
    size_t r = 0, v = 0;
    j->rc = orc_read_list_page(j->chunk + pos, len, nlev, j->ln, j->in, j->kind, j->width, po, pl,
                               j->lvals + leaves * (size_t)j->width, pf, &r, &v);
    if (!j->rc) {
      for (size_t i = 0; i < r; i++) j->loffs[rows + i] = po[i] + (int64_t)leaves;
      if (j->ln) put_bits(j->lbits, rows, pl, r);
      if (j->in) put_bits(j->fbits, leaves, pf, v);
      rows += r;
      leaves += v;
    }
    free(po);
    free(pl);
    free(pf);
    pos += len;
  }
  j->rows = rows;
  j->leaves = leaves;
  return NULL;
}

/* batch read of a List<T> leaf (read_validity_nested + create_list, pages
 * appended): offsets int64 rows + 1, list bits, values, leaf bits. */
int orc_mt_read_list_column(const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int list_nullable,
                            int item_nullable, int kind, int width, int64_t* out_offsets, uint8_t* out_list_bits,
                            uint8_t* out_values, uint8_t* out_leaf_bits, int n_threads, uint64_t* rows_out,
                            uint64_t* leaves_out) {
  job_t jobs[256];
  size_t k = setup(jobs, chunk, metas, n_pages, n_threads, 0);
  for (size_t t = 0; t < k; t++) {
    jobs[t].ln = list_nullable;
    jobs[t].in = item_nullable;
    jobs[t].kind = kind;
    jobs[t].width = width;
  }
  run(jobs, k, list_worker);
  int rc = ORC_OK;
  uint64_t rb = 0, lb = 0;
  for (size_t t = 0; t < k; t++) {
    job_t* j = &jobs[t];
    if (!rc && j->rc) rc = j->rc;
    if (!rc) {
      for (size_t i = 0; i < j->rows; i++) out_offsets[rb + i] = j->loffs[i] + (int64_t)lb;
      if (j->leaves) memcpy(out_values + lb * (size_t)width, j->lvals, j->leaves * (size_t)width);
      if (list_nullable) put_bits(out_list_bits, rb, j->lbits, j->rows);
      if (item_nullable) put_bits(out_leaf_bits, lb, j->fbits, j->leaves);
      rb += j->rows;
      lb += j->leaves;
    }
    free(j->loffs);
    free(j->lbits);
    free(j->lvals);
    free(j->fbits);
  }
  out_offsets[rb] = (int64_t)lb;
  *rows_out = rb;
  *leaves_out = lb;
  return rc;
}

static void* bool_worker(void* arg) {
  job_t* j = (job_t*)arg;
  uint64_t pos = j->byte0, row = j->row0;
  for (size_t p = j->p0; p < j->p1 && !j->rc; p++) {
    const uint64_t len = j->metas[2 * p], nv = j->metas[2 * p + 1];
    uint8_t* vb = (uint8_t*)calloc(nv / 8 + 2, 1);
    uint8_t* mb = (uint8_t*)calloc(nv / 8 + 2, 1);
    j->rc = orc_read_bool_page(j->chunk + pos, len, nv, j->nullable, vb, mb);
    if (!j->rc) {
      put_bits(j->out_values, row, vb, nv);
      if (j->nullable) put_bits(j->out_bits, row, mb, nv);
    }
    free(vb);
    free(mb);
    pos += len;
    row += nv;
  }
  return NULL;
}

/* read_boolean (read/array/boolean.rs:191-219) */
int orc_mt_read_bool_column(const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int nullable,
                            uint8_t* out_bits, uint8_t* out_valid, int n_threads) {
  job_t jobs[256];
  size_t k = setup(jobs, chunk, metas, n_pages, n_threads, 1);
  for (size_t t = 0; t < k; t++) {
    jobs[t].nullable = nullable;
    jobs[t].out_values = out_bits;
    jobs[t].out_bits = out_valid;
  }
  run(jobs, k, bool_worker);
  for (size_t t = 0; t < k; t++)
    if (jobs[t].rc) return jobs[t].rc;
  return ORC_OK;
}
