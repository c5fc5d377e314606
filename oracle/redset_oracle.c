/*
 * redset_oracle.c -- TEST INFRASTRUCTURE ONLY (see redset_oracle.h).
 *
 * Plain C99 restatement of the reference's Reed-Solomon / XOR codec as
 * single-process, whole-set operations. Written from the reference's
 * behaviour; each function names the reference lines it follows.
 */
#define _GNU_SOURCE
#include "redset_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------ */
/* GF(2^8) arithmetic                                                  */
/* ------------------------------------------------------------------ */

/* carry-less multiply then reduce by x^8 + 0x1D.
 * follows gf_mult(8, 0x1D, a, b), src/redset_reedsolomon_common.c:41-75 */
static unsigned int shift_mult(unsigned int a, unsigned int b)
{
  unsigned int acc = 0;
  for (int k = 0; k < 8 && a; k++, a >>= 1) {
    if (a & 1u) acc ^= (b << k);
  }
  /* reduce bits 14..8 (mask starts at 1<<(2m-2)), :64-72 */
  for (int k = 6; k >= 0; k--) {
    unsigned int top = 1u << (k + 8);
    if (acc & top) {
      acc &= ~top;
      acc ^= (0x1Du << k);
    }
  }
  return acc;
}

/* gf_build_tables(state, 8), src/redset_reedsolomon_common.c:79-150:
 * exp[i] = 2^i for i < 255, exp[255] = 0, log[0] = 0, log[1] = 0,
 * imult by exhaustive search. */
void ro_gf_tables(unsigned int* lg, unsigned int* ex, unsigned int* im)
{
  lg[0] = 0;
  ex[255] = 0;
  lg[1] = 0;
  ex[0] = 1;
  unsigned int v = 2;
  for (int i = 1; i < 255; i++) {
    ex[i] = v;
    lg[v] = (unsigned int) i;
    v = shift_mult(v, 2);
  }
  im[0] = 0;
  for (unsigned int a = 1; a < 256; a++) {
    for (unsigned int b = 1; b < 256; b++) {
      if (shift_mult(a, b) == 1) { im[a] = b; break; }
    }
  }
}

/* gf_mult_table, src/redset_reedsolomon_common.c:153-179 */
unsigned int ro_gf_mult(const ro_rs* st, unsigned int a, unsigned int b)
{
  if (a == 0 || b == 0) return 0;
  unsigned int s = st->log[a] + st->log[b];
  if (s >= 255) s -= 255;
  return st->exp[s];
}

/* gf_premult_table, src/redset_reedsolomon_common.c:184-233 */
void ro_rs_premult_table(const ro_rs* st, unsigned int v, uint8_t* prods)
{
  if (v == 0) { memset(prods, 0, 256); return; }
  for (unsigned int x = 0; x < 256; x++) {
    prods[x] = (uint8_t) ro_gf_mult(st, v, x);
  }
}

/* ------------------------------------------------------------------ */
/* encoding matrix                                                     */
/* ------------------------------------------------------------------ */

/* swap_columns, src/redset_reedsolomon_common.c:250-264 */
static void col_swap(unsigned int* m, int rows, int cols, int a, int b)
{
  if (a == b) return;
  for (int r = 0; r < rows; r++) {
    unsigned int t = m[r * cols + a];
    m[r * cols + a] = m[r * cols + b];
    m[r * cols + b] = t;
  }
}

/* build_vandermonde + normalize_vandermonde,
 * src/redset_reedsolomon_common.c:634-725: element (row, col) = row^col,
 * then column elimination so the top p x p block is the identity. */
static void make_matrix(ro_rs* st)
{
  const int n = st->ranks, k = st->encoding, rows = n + k;
  unsigned int* m = st->mat;
  for (int r = 0; r < rows; r++) {
    m[r * n] = 1;
    unsigned int pw = (unsigned int) r;
    for (int c = 1; c < n; c++) {
      m[r * n + c] = pw;
      pw = ro_gf_mult(st, pw, (unsigned int) r);
    }
  }
  for (int r = 0; r < n; r++) {
    int nz = -1;
    for (int c = r; c < n; c++) {
      if (m[r * n + c] != 0) { nz = c; break; }
    }
    col_swap(m, rows, n, r, nz);
    unsigned int inv = st->imult[m[r * n + r]];
    for (int r2 = r; r2 < rows; r2++) {
      m[r2 * n + r] = ro_gf_mult(st, m[r2 * n + r], inv);
    }
    for (int c = 0; c < n; c++) {
      if (c == r) continue;
      unsigned int f = m[r * n + c];
      if (f == 0) continue;
      for (int r2 = r; r2 < rows; r2++) {
        m[r2 * n + c] ^= ro_gf_mult(st, f, m[r2 * n + r]);
      }
    }
  }
}

/* redset_rs_gf_alloc, src/redset_reedsolomon_common.c:727-757 */
int ro_rs_init(ro_rs* st, int ranks, int encoding)
{
  if (ranks < 2 || encoding < 1 || encoding >= ranks || ranks + encoding > 256) return 1;
  st->ranks = ranks;
  st->encoding = encoding;
  ro_gf_tables(st->log, st->exp, st->imult);
  st->mat = (unsigned int*) malloc(sizeof(unsigned int) * (size_t)(ranks + encoding) * ranks);
  if (!st->mat) return 1;
  make_matrix(st);
  return 0;
}

void ro_rs_free(ro_rs* st)
{
  free(st->mat);
  st->mat = NULL;
}

ro_rs* ro_rs_new(int ranks, int encoding)
{
  ro_rs* st = (ro_rs*) calloc(1, sizeof(ro_rs));
  if (st && ro_rs_init(st, ranks, encoding) != 0) { free(st); st = NULL; }
  return st;
}

void ro_rs_delete(ro_rs* st)
{
  if (st) { ro_rs_free(st); free(st); }
}

const unsigned int* ro_rs_matrix(const ro_rs* st) { return st->mat; }

/* ------------------------------------------------------------------ */
/* stripe layout                                                       */
/* ------------------------------------------------------------------ */

/* redset_rs_get_encoding_id, src/redset_reedsolomon_common.c:822-833 */
int ro_rs_get_encoding_id(int ranks, int encoding, int rank, int chunk_id)
{
  int d = ranks - encoding;
  int id = (d - rank + ranks + chunk_id) % ranks;
  return (id < d) ? rank : ranks + (id - d);
}

/* redset_rs_get_data_id, src/redset_reedsolomon_common.c:836-853 */
int ro_rs_get_data_id(int ranks, int encoding, int rank, int chunk_id)
{
  int id = chunk_id;
  if (id > rank) id -= encoding;
  int lead = rank + encoding - ranks;
  if (lead > 0) id -= lead;
  return id;
}

/* ------------------------------------------------------------------ */
/* buffer kernels                                                      */
/* ------------------------------------------------------------------ */

/* redset_rs_reduce_buffer_multadd, src/redset_reedsolomon_common.c:786-819 */
void ro_rs_multadd(const ro_rs* st, size_t count, uint8_t* buf, unsigned int coeff, const uint8_t* data)
{
  uint8_t t[256];
  ro_rs_premult_table(st, coeff, t);
  for (size_t j = 0; j < count; j++) buf[j] ^= t[data[j]];
}

/* reduce_buffer_add (:772-783) and reduce_xor (src/redset_xor.c:35-42) */
static void xor_into(size_t count, uint8_t* buf, const uint8_t* data)
{
  for (size_t j = 0; j < count; j++) buf[j] ^= data[j];
}

/* scale_row, src/redset_reedsolomon_common.c:268-319 */
static void row_scale(const ro_rs* st, unsigned int* m, int cols, unsigned int v, int r,
                      size_t count, uint8_t* buf)
{
  uint8_t t[256];
  ro_rs_premult_table(st, v, t);
  for (int c = 0; c < cols; c++) m[r * cols + c] = t[m[r * cols + c]];
  for (size_t j = 0; j < count; j++) buf[j] = t[buf[j]];
}

/* mult_add_row (+ add_row), src/redset_reedsolomon_common.c:323-415 */
static void row_madd(const ro_rs* st, unsigned int* m, int cols, unsigned int v, int a, int b,
                     size_t count, const uint8_t* bufa, uint8_t* bufb)
{
  if (v == 0) return;
  uint8_t t[256];
  ro_rs_premult_table(st, v, t);
  for (int c = 0; c < cols; c++) m[b * cols + c] ^= t[m[a * cols + c]];
  for (size_t j = 0; j < count; j++) bufb[j] ^= t[bufa[j]];
}

/* redset_rs_gaussian_solve_identify_rows, src/redset_reedsolomon_common.c:425-564 */
void ro_rs_identify_rows(const ro_rs* st, int missing, const int* unknowns,
                         unsigned int* m, int* rows)
{
  const int n = st->ranks, k = st->encoding;
  int numk[256];
  int taken[256];
  for (int r = 0; r < k; r++) {
    numk[r] = 0;
    taken[r] = 0;
    for (int i = 0; i < missing; i++) {
      int u = unknowns[i];
      if (u < n) { if (st->mat[(r + n) * n + u] != 0) numk[r]++; }
      else if (u == r + n) numk[r]++;
    }
  }
  for (int i = 0; i < missing; i++) {
    int best = -1, lo = missing + 1, u = unknowns[i];
    for (int r = 0; r < k; r++) {
      if (taken[r]) continue;
      int defined = (u < n) ? (st->mat[(r + n) * n + u] != 0) : (u == r + n);
      if (defined && numk[r] < lo) { lo = numk[r]; best = r; }
    }
    rows[i] = best;
    taken[best] = 1;
    for (int j = 0; j < missing; j++) {
      int uj = unknowns[j];
      if (uj < n) m[i * missing + j] = st->mat[(best + n) * n + uj];
      else m[i * missing + j] = (uj == best + n) ? 1u : 0u;
    }
  }
}

/* redset_rs_gaussian_solve, src/redset_reedsolomon_common.c:570-630.
 * Column swaps permute the coefficient matrix only, never the buffers,
 * exactly as the reference does. */
void ro_rs_gaussian_solve(const ro_rs* st, unsigned int* m, int missing, size_t count, uint8_t** bufs)
{
  for (int r = 0; r < missing; r++) {
    int nz = r;
    for (int c = r; c < missing; c++) {
      if (m[r * missing + c] > 0) { nz = c; break; }
    }
    col_swap(m, missing, missing, r, nz);
    unsigned int v = m[r * missing + r];
    if (v != 0) row_scale(st, m, missing, st->imult[v], r, count, bufs[r]);
    for (int r2 = r + 1; r2 < missing; r2++) {
      row_madd(st, m, missing, m[r2 * missing + r], r, r2, count, bufs[r], bufs[r2]);
    }
  }
  for (int r = missing - 1; r > 0; r--) {
    for (int r2 = r - 1; r2 >= 0; r2--) {
      row_madd(st, m, missing, m[r2 * missing + r], r, r2, count, bufs[r], bufs[r2]);
    }
  }
}

/* redset_rs_reduce_decode, src/redset_reedsolomon_common.c:855-899 */
static void reduce_decode(const ro_rs* st, int chunk_id, int sender, int missing, const int* rows,
                          size_t count, const uint8_t* cell, uint8_t** acc)
{
  const int n = st->ranks;
  int enc = ro_rs_get_encoding_id(n, st->encoding, sender, chunk_id);
  for (int i = 0; i < missing; i++) {
    int row = rows[i] + n;
    if (enc < n) ro_rs_multadd(st, count, acc[i], st->mat[row * n + sender], cell);
    else if (row == enc) xor_into(count, acc[i], cell);
  }
}

/* ------------------------------------------------------------------ */
/* whole-set RS                                                        */
/* ------------------------------------------------------------------ */

static const uint8_t* data_cell(const ro_rs* st, uint8_t* const* lofi, size_t C, int rank, int chunk)
{
  int seg = ro_rs_get_data_id(st->ranks, st->encoding, rank, chunk);
  return lofi[rank] + (size_t) seg * C;
}

/* redset_reedsolomon_encode, src/redset_reedsolomon.c:280-402, with the ring
 * (:346-363) resolved in one address space: at ring step `chunk_step`, member
 * r's slot i receives from s = r + (p - chunk_step + i) the cell s sends,
 * i.e. s's data cell of stripe (r + i) mod p, weighted by mat[(p+i)*p + s]. */
void ro_rs_encode_set(const ro_rs* st, size_t C, uint8_t* const* lofi, uint8_t* const* parity, size_t slice)
{
  const int p = st->ranks, e = st->encoding;
  if (slice == 0) slice = C;
  for (size_t nread = 0; nread < C; nread += slice) {
    size_t count = (C - nread < slice) ? C - nread : slice;
    for (int r = 0; r < p; r++) {
      for (int i = 0; i < e; i++) memset(parity[r] + (size_t) i * C + nread, 0, count);
      for (int step = p - 1; step >= e; step--) {
        for (int i = 0; i < e; i++) {
          int s = (r + p - step + i) % p;
          int chunk = (s + step) % p;           /* == (r + i) % p */
          unsigned int coeff = st->mat[(p + i) * p + s];
          ro_rs_multadd(st, count, parity[r] + (size_t) i * C + nread, coeff,
                        data_cell(st, lofi, C, s, chunk) + nread);
        }
      }
    }
  }
}

/* redset_reedsolomon_decode, src/redset_reedsolomon.c:570-785: member r
 * solves stripe r from every member's cell of that stripe (ring order
 * :646-703, erased members contribute zeros), runs the elimination
 * (:707-708) and hands unknown i to rebuild_ranks[i] (:713-765). */
int ro_rs_rebuild_set(const ro_rs* st, size_t C, int missing, const int* rebuild_ranks,
                      uint8_t* const* lofi, uint8_t* const* parity, size_t slice)
{
  const int p = st->ranks, e = st->encoding;
  if (missing > e) return 1;
  if (missing == 0) return 0;
  if (slice == 0) slice = C;
  int erased[256] = {0};
  for (int i = 0; i < missing; i++) erased[rebuild_ranks[i]] = 1;

  uint8_t** acc = (uint8_t**) malloc(sizeof(uint8_t*) * (size_t) missing);
  uint8_t* zero = (uint8_t*) calloc(slice, 1);
  for (int i = 0; i < missing; i++) acc[i] = (uint8_t*) malloc(slice);
  unsigned int* m = (unsigned int*) malloc(sizeof(unsigned int) * (size_t) missing * missing);
  unsigned int* mcopy = (unsigned int*) malloc(sizeof(unsigned int) * (size_t) missing * missing);
  int* rows = (int*) malloc(sizeof(int) * (size_t) missing);
  int* unknowns = (int*) malloc(sizeof(int) * (size_t) missing);
  /* results are staged per stripe, then scattered, because the scatter
   * overwrites cells other stripes' solves still read */
  uint8_t** out = (uint8_t**) malloc(sizeof(uint8_t*) * (size_t) p * missing);
  for (int i = 0; i < p * missing; i++) out[i] = (uint8_t*) malloc(C);

  for (int r = 0; r < p; r++) {
    for (int i = 0; i < missing; i++) {
      unknowns[i] = ro_rs_get_encoding_id(p, e, rebuild_ranks[i], r);
    }
    ro_rs_identify_rows(st, missing, unknowns, m, rows);
    for (size_t nread = 0; nread < C; nread += slice) {
      size_t count = (C - nread < slice) ? C - nread : slice;
      for (int i = 0; i < missing; i++) memset(acc[i], 0, count);
      for (int step = 0; step < p; step++) {
        int sender = (r - step + p) % p;
        const uint8_t* cell;
        if (erased[sender]) {
          cell = zero;
        } else {
          int enc = ro_rs_get_encoding_id(p, e, sender, r);
          cell = (enc < p) ? data_cell(st, lofi, C, sender, r) + nread
                           : parity[sender] + (size_t)(enc - p) * C + nread;
        }
        reduce_decode(st, r, sender, missing, rows, count, cell, acc);
      }
      memcpy(mcopy, m, sizeof(unsigned int) * (size_t) missing * missing);
      ro_rs_gaussian_solve(st, mcopy, missing, count, acc);
      for (int i = 0; i < missing; i++) memcpy(out[r * missing + i] + nread, acc[i], count);
    }
  }
  for (int r = 0; r < p; r++) {
    for (int i = 0; i < missing; i++) {
      int dst = rebuild_ranks[i];
      int enc = ro_rs_get_encoding_id(p, e, dst, r);
      uint8_t* where = (enc < p) ? lofi[dst] + (size_t) ro_rs_get_data_id(p, e, dst, r) * C
                                 : parity[dst] + (size_t)(enc - p) * C;
      memcpy(where, out[r * missing + i], C);
    }
  }
  for (int i = 0; i < p * missing; i++) free(out[i]);
  free(out);
  for (int i = 0; i < missing; i++) free(acc[i]);
  free(acc);
  free(zero);
  free(m);
  free(mcopy);
  free(rows);
  free(unknowns);
  return 0;
}

/* ------------------------------------------------------------------ */
/* whole-set XOR                                                       */
/* ------------------------------------------------------------------ */

/* segment of member s holding stripe c (s != c):
 * src/redset_xor.c:255-258, src/redset_xor_serial.c:216-227 */
static size_t xor_seg(int s, int c) { return (size_t)(c < s ? c : c - 1); }

/* redset_xor_encode, src/redset_xor.c:220-295: the pipelined ring leaves
 * member r with the XOR of every other member's cell of stripe r. The
 * accumulation order (r-1, r-2, ...) does not change XOR's result. */
void ro_xor_encode_set(int p, size_t C, uint8_t* const* lofi, uint8_t* const* xorc, size_t slice)
{
  if (slice == 0) slice = C;
  for (int r = 0; r < p; r++) {
    for (size_t nread = 0; nread < C; nread += slice) {
      size_t count = (C - nread < slice) ? C - nread : slice;
      memset(xorc[r] + nread, 0, count);
      for (int t = 1; t < p; t++) {
        int s = (r - t + p) % p;
        xor_into(count, xorc[r] + nread, lofi[s] + xor_seg(s, r) * C + nread);
      }
    }
  }
}

/* redset_recover_xor_rebuild_serial, src/redset_xor_serial.c:161-275 */
void ro_xor_rebuild_set(int p, size_t C, int root, uint8_t* const* lofi, uint8_t* const* xorc, size_t slice)
{
  if (slice == 0) slice = C;
  uint8_t* a = (uint8_t*) malloc(slice);
  for (int c = 0; c < p; c++) {
    for (size_t nread = 0; nread < C; nread += slice) {
      size_t count = (C - nread < slice) ? C - nread : slice;
      memset(a, 0, count);
      for (int s = 0; s < p; s++) {
        if (s == root) continue;
        const uint8_t* src = (c != s) ? lofi[s] + xor_seg(s, c) * C : xorc[s];
        xor_into(count, a, src + nread);
      }
      uint8_t* dst = (c != root) ? lofi[root] + xor_seg(root, c) * C : xorc[root];
      memcpy(dst + nread, a, count);
    }
  }
  free(a);
}

/* ------------------------------------------------------------------ */
/* pthreads CPU baselines                                              */
/* ------------------------------------------------------------------ */

/* One job = one contiguous piece of one multadd (or XOR), as in
 * reduce_rs_pthread_launch3 (src/redset_reedsolomon_pthreads.c:447-504). */
typedef struct {
  uint8_t* a;
  const uint8_t* b;
  size_t n;
  unsigned int coeff;   /* 0x100 marks a plain XOR job */
} ro_job;

typedef struct {
  const ro_rs* st;
  pthread_mutex_t mu;
  pthread_cond_t work_cv, done_cv;
  ro_job* jobs;
  int njobs, next, done, quit;
} ro_pool;

static void* pool_worker(void* arg)
{
  ro_pool* P = (ro_pool*) arg;
  uint8_t premult[256];   /* private table, src/redset_reedsolomon_pthreads.c:30, :200 */
  pthread_mutex_lock(&P->mu);
  for (;;) {
    while (!P->quit && P->next >= P->njobs) pthread_cond_wait(&P->work_cv, &P->mu);
    if (P->quit) break;
    ro_job* j = &P->jobs[P->next++];
    pthread_mutex_unlock(&P->mu);
    if (j->coeff == 0x100u) {
      for (size_t x = 0; x < j->n; x++) j->a[x] ^= j->b[x];
    } else {
      ro_rs_premult_table(P->st, j->coeff, premult);
      for (size_t x = 0; x < j->n; x++) j->a[x] ^= premult[j->b[x]];
    }
    pthread_mutex_lock(&P->mu);
    if (++P->done == P->njobs) pthread_cond_signal(&P->done_cv);
  }
  pthread_mutex_unlock(&P->mu);
  return NULL;
}

/* post the job list and wait for it: reduce_rs_pthread_sync3, :507-519 */
static void pool_run(ro_pool* P, ro_job* jobs, int njobs)
{
  pthread_mutex_lock(&P->mu);
  P->jobs = jobs;
  P->njobs = njobs;
  P->next = 0;
  P->done = 0;
  pthread_cond_broadcast(&P->work_cv);
  while (P->done < P->njobs) pthread_cond_wait(&P->done_cv, &P->mu);
  pthread_mutex_unlock(&P->mu);
}

static int default_threads(int cap)
{
  long n = sysconf(_SC_NPROCESSORS_ONLN);   /* redset_get_nprocs, src/redset_util.c:454-471 */
  if (n < 1) n = 1;
  return (int)(n > cap ? cap : n);
}

/* split one buffer op into nthreads contiguous jobs, :459-499 */
static int split_jobs(ro_job* out, int nthreads, uint8_t* a, const uint8_t* b, size_t count, unsigned int coeff)
{
  size_t piece = count / (size_t) nthreads;
  if (piece * (size_t) nthreads < count) piece++;
  int nj = 0;
  for (size_t off = 0; off < count; off += piece) {
    size_t amt = (count - off < piece) ? count - off : piece;
    out[nj].a = a + off;
    out[nj].b = b + off;
    out[nj].n = amt;
    out[nj].coeff = coeff;
    nj++;
  }
  return nj;
}

static void pool_start(ro_pool* P, const ro_rs* st, int nthreads, pthread_t* tids)
{
  memset(P, 0, sizeof(*P));
  P->st = st;
  pthread_mutex_init(&P->mu, NULL);
  pthread_cond_init(&P->work_cv, NULL);
  pthread_cond_init(&P->done_cv, NULL);
  for (int t = 0; t < nthreads; t++) pthread_create(&tids[t], NULL, pool_worker, P);
}

static void pool_stop(ro_pool* P, int nthreads, pthread_t* tids)
{
  pthread_mutex_lock(&P->mu);
  P->quit = 1;
  pthread_cond_broadcast(&P->work_cv);
  pthread_mutex_unlock(&P->mu);
  for (int t = 0; t < nthreads; t++) pthread_join(tids[t], NULL);
  pthread_mutex_destroy(&P->mu);
  pthread_cond_destroy(&P->work_cv);
  pthread_cond_destroy(&P->done_cv);
}

/* redset_reedsolomon_encode_pthreads, src/redset_reedsolomon_pthreads.c:567-699 */
int ro_rs_encode_pthreads(const ro_rs* st, size_t C, uint8_t* const* lofi, uint8_t* const* parity,
                          size_t slice, int nthreads, int rank_lo, int rank_hi)
{
  const int p = st->ranks, e = st->encoding;
  if (nthreads <= 0) nthreads = default_threads(10);   /* max_threads = 10, :393-397 */
  if (slice == 0) slice = C;
  pthread_t tids[64];
  if (nthreads > 64) nthreads = 64;
  ro_pool P;
  pool_start(&P, st, nthreads, tids);
  ro_job* jobs = (ro_job*) malloc(sizeof(ro_job) * (size_t) e * nthreads);
  for (int r = rank_lo; r < rank_hi; r++) {
    for (size_t nread = 0; nread < C; nread += slice) {
      size_t count = (C - nread < slice) ? C - nread : slice;
      for (int i = 0; i < e; i++) memset(parity[r] + (size_t) i * C + nread, 0, count);
      for (int step = p - 1; step >= e; step--) {
        int nj = 0;
        for (int i = 0; i < e; i++) {
          int s = (r + p - step + i) % p;
          int chunk = (s + step) % p;
          nj += split_jobs(jobs + nj, nthreads, parity[r] + (size_t) i * C + nread,
                           data_cell(st, lofi, C, s, chunk) + nread, count,
                           st->mat[(p + i) * p + s]);
        }
        pool_run(&P, jobs, nj);   /* sync3 after every step, :670 */
      }
    }
  }
  free(jobs);
  pool_stop(&P, nthreads, tids);
  return nthreads;
}

/* redset_xor_encode_pthreads, src/redset_xor_pthreads.c:311-392 (≤16 threads, :170-173) */
int ro_xor_encode_pthreads(int p, size_t C, uint8_t* const* lofi, uint8_t* const* xorc,
                           size_t slice, int nthreads, int rank_lo, int rank_hi)
{
  if (nthreads <= 0) nthreads = default_threads(16);
  if (slice == 0) slice = C;
  pthread_t tids[64];
  if (nthreads > 64) nthreads = 64;
  ro_pool P;
  ro_rs dummy;
  memset(&dummy, 0, sizeof(dummy));
  pool_start(&P, &dummy, nthreads, tids);
  ro_job* jobs = (ro_job*) malloc(sizeof(ro_job) * (size_t) nthreads);
  for (int r = rank_lo; r < rank_hi; r++) {
    for (size_t nread = 0; nread < C; nread += slice) {
      size_t count = (C - nread < slice) ? C - nread : slice;
      memset(xorc[r] + nread, 0, count);
      for (int t = 1; t < p; t++) {
        int s = (r - t + p) % p;
        int nj = split_jobs(jobs, nthreads, xorc[r] + nread, lofi[s] + xor_seg(s, r) * C + nread,
                            count, 0x100u);
        pool_run(&P, jobs, nj);
      }
    }
  }
  free(jobs);
  pool_stop(&P, nthreads, tids);
  return nthreads;
}

/* ------------------------------------------------------------------ */
/* CRC32 (zlib, reflected 0xEDB88320)                                  */
/* ------------------------------------------------------------------ */
uint32_t ro_crc32(uint32_t crc, const uint8_t* buf, size_t len)
{
  static uint32_t table[256];
  static int ready = 0;
  if (!ready) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    ready = 1;
  }
  crc = ~crc;
  for (size_t i = 0; i < len; i++) crc = table[(crc ^ buf[i]) & 0xFFu] ^ (crc >> 8);
  return ~crc;
}
