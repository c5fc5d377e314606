/*
 * sharded.c -- sets sharded over the GPUs of a node (include/redset_hip.h,
 * "sets sharded over the GPUs of a node"). Host code in C over the codec's
 * own C ABI; the exchanges go through a caller-chosen transport (RCCL over
 * xGMI in production, transport_rccl.c; MPI host buffers, rank_mpi.c; a test
 * callback) and the arithmetic through the HIP plans or a compute callback.
 *
 * Replaces, for the multi-rank rebuild, the decode ring of
 * redset_reedsolomon_decode (src/redset_reedsolomon.c:646-703: p-1 steps,
 * one cell per step per rank) with one grouped gather of column slices, and
 * its gather of solved cells to the failed ranks (:713-733) with one grouped
 * return; for encode, the ring of redset_reedsolomon_encode (:329-377).
 * Stripe ownership differs on purpose: the reference has rank r solve stripe
 * r whole (:606-611); here every GPU solves its column slice of every stripe,
 * so the work splits evenly whatever p and the number of GPUs. XOR sets
 * (redset_hip_xor_sharded_plan) work the same way: the rebuild replaces the
 * pipelined reduce to the lost member (src/redset_xor.c:466-524), whose root
 * receives every survivor's every cell, with slices gathered onto every GPU.
 */
#include <hip/hip_runtime_api.h>
#include <limits.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "redset_hip.h"

#define MAX_RANKS 256

static int sfail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
static int sfail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return redset_hip_record_error(buf);
}

/* ---- transfer lists ---------------------------------------------------- */

typedef struct {
  redset_hip_xfer* v;
  int n, cap;
} xlist;

static int xl_push(xlist* L, redset_hip_xfer x) {
  if (L->n == L->cap) {
    int cap = L->cap ? 2 * L->cap : 64;
    redset_hip_xfer* v = realloc(L->v, sizeof(*v) * (size_t) cap);
    if (!v) return sfail("out of host memory");
    L->v = v;
    L->cap = cap;
  }
  L->v[L->n++] = x;
  return 0;
}

/* Per-peer message lists of one exchange. Rows appended to a peer's send (or
 * receive) list merge with the previous one when contiguous in local memory.
 * Both processes of a pair walk the same rows in the same order, and a row's
 * offset on one side differs from its offset on the other by a constant of
 * the pair (the buffers share one layout), so they merge alike and the
 * message lengths match. Nothing moves within a process: its own slice of
 * the members it hosts is computed in place (plan_sets). */
typedef struct {
  int world, rank;
  xlist* send;   /* [world] */
  xlist* recv;   /* [world] */
} exch;

static int ex_init(exch* X, int world, int rank) {
  memset(X, 0, sizeof(*X));
  X->world = world;
  X->rank = rank;
  X->send = calloc((size_t) world, sizeof(xlist));
  X->recv = calloc((size_t) world, sizeof(xlist));
  return (X->send && X->recv) ? 0 : sfail("out of host memory");
}

static void ex_free(exch* X) {
  for (int g = 0; X->send && g < X->world; ++g) free(X->send[g].v);
  for (int g = 0; X->recv && g < X->world; ++g) free(X->recv[g].v);
  free(X->send);
  free(X->recv);
  memset(X, 0, sizeof(*X));
}

static int ex_row(xlist* L, int peer, int send, unsigned char* buf, size_t len) {
  if (L->n > 0) {
    redset_hip_xfer* t = &L->v[L->n - 1];
    if ((unsigned char*) t->buf + t->len == buf) {
      t->len += len;
      return 0;
    }
  }
  redset_hip_xfer x = {peer, send, buf, len};
  return xl_push(L, x);
}

static int ex_send(exch* X, int peer, unsigned char* buf, size_t len) { return ex_row(&X->send[peer], peer, 1, buf, len); }
static int ex_recv(exch* X, int peer, unsigned char* buf, size_t len) { return ex_row(&X->recv[peer], peer, 0, buf, len); }

/* message statistics of one phase (the info block) */
typedef struct {
  int *messages, *recv_messages;
  unsigned long long *sent, *recvd, *max_msg, *min_msg;
} xstats;

/* flatten into one list for the transport: per peer its sends and
 * receives; byte counts and message sizes for the info block */
static int ex_flatten(exch* X, xlist* out, const xstats* st) {
  for (int g = 0; g < X->world; ++g) {
    for (int i = 0; i < X->send[g].n; ++i) {
      const unsigned long long len = X->send[g].v[i].len;
      if (xl_push(out, X->send[g].v[i])) return REDSET_FAILURE;
      *st->sent += len;
      ++*st->messages;
      if (len > *st->max_msg) *st->max_msg = len;
      if (*st->min_msg == 0 || len < *st->min_msg) *st->min_msg = len;
    }
    for (int i = 0; i < X->recv[g].n; ++i) {
      if (xl_push(out, X->recv[g].v[i])) return REDSET_FAILURE;
      *st->recvd += X->recv[g].v[i].len;
      ++*st->recv_messages;
    }
  }
  return 0;
}

/* ---- combine job lists (the partial-sum shape) -------------------------- */

/* jobs with their pointer and coefficient arrays in growing pools; the jobs
 * keep pool offsets until cs_finish points them at the pools */
typedef struct {
  redset_hip_combine_job* v;
  int n, cap;
  unsigned char** ptr;             /* inputs then outputs of every job */
  size_t np, pcap;
  unsigned char* coef;
  size_t nc, ccap;
  unsigned long long bytes;        /* HBM bytes the jobs move (reads + writes) */
} cset;

static void cs_free(cset* S) {
  free(S->v);
  free(S->ptr);
  free(S->coef);
  memset(S, 0, sizeof(*S));
}

/* one job: nin inputs, nout outputs, coef nout x nin, over n cell bytes */
static int cs_add(cset* S, int nin, unsigned char* const* in, int nout, unsigned char* const* out,
                  const unsigned char* coef, int accumulate, size_t n) {
  if (S->n == S->cap) {
    int cap = S->cap ? 2 * S->cap : 32;
    redset_hip_combine_job* v = realloc(S->v, sizeof(*v) * (size_t) cap);
    if (!v) return sfail("out of host memory");
    S->v = v;
    S->cap = cap;
  }
  const size_t k = (size_t) nin + (size_t) nout, kc = (size_t) nin * (size_t) nout;
  if (S->np + k > S->pcap) {
    size_t cap = S->pcap ? 2 * S->pcap : 256;
    while (cap < S->np + k) cap *= 2;
    unsigned char** v = realloc(S->ptr, sizeof(*v) * cap);
    if (!v) return sfail("out of host memory");
    S->ptr = v;
    S->pcap = cap;
  }
  if (S->nc + kc > S->ccap) {
    size_t cap = S->ccap ? 2 * S->ccap : 1024;
    while (cap < S->nc + kc) cap *= 2;
    unsigned char* v = realloc(S->coef, cap);
    if (!v) return sfail("out of host memory");
    S->coef = v;
    S->ccap = cap;
  }
  redset_hip_combine_job J;
  J.nin = nin;
  J.nout = nout;
  J.in = (const unsigned char* const*) (uintptr_t) S->np; /* offsets until cs_finish */
  J.out = (unsigned char* const*) (uintptr_t) (S->np + (size_t) nin);
  J.coef = (const unsigned char*) (uintptr_t) S->nc;
  J.accumulate = accumulate;
  memcpy(S->ptr + S->np, in, sizeof(*in) * (size_t) nin);
  memcpy(S->ptr + S->np + nin, out, sizeof(*out) * (size_t) nout);
  memcpy(S->coef + S->nc, coef, kc);
  S->np += k;
  S->nc += kc;
  S->v[S->n++] = J;
  S->bytes += (unsigned long long) (nin + nout + (accumulate ? nout : 0)) * n;
  return 0;
}

static void cs_finish(cset* S) {
  for (int i = 0; i < S->n; ++i) {
    redset_hip_combine_job* J = &S->v[i];
    J->in = (const unsigned char* const*) (S->ptr + (uintptr_t) J->in);
    J->out = S->ptr + (uintptr_t) J->out;
    J->coef = S->coef + (uintptr_t) J->coef;
  }
}

/* ---- the plan ---------------------------------------------------------- */

struct redset_hip_sharded {
  redset_hip_sharded_info info;
  redset_hip_transport tr;
  redset_hip_compute comp;
  int p, e, missing;
  int lost[MAX_RANKS];
  size_t W;
  /* the exchanges, set by set: set k's transfers are gather.v[goff[k] ..
   * goff[k+1]) and ret.v[roff[k] .. roff[k+1]); a phase runs all of them */
  xlist gather, ret;
  int* goff;                       /* [nsets + 1] */
  int* roff;                       /* [nsets + 1] */
  /* pipelined execute (HIP compute): a stream for the exchanges, two events */
  hipStream_t xstream;
  hipEvent_t ev_x;                 /* exchange stream -> caller's stream */
  hipEvent_t* ev_c;                /* [nsets] set k's compute done */
  /* compute per set: HIP plans, or the member pointers for the callback */
  redset_hip_plan** plans;         /* [nsets] (NULL entries when my slice is empty) */
  unsigned char** lofi;            /* [nsets * p] */
  unsigned char** parity;          /* [nsets * p] */
  /* the partial-sum shape (REDSET_HIP_SHAPE_REDUCE): per set, the combines
   * of the COMPUTE phase (partial sums, and outputs only my inputs feed) and
   * of the ACCUMULATE phase (outputs partials arrived for); the partial
   * exchange is `ret` */
  int shape;
  cset* part;                      /* [nsets] */
  cset* acc;                       /* [nsets] */
  redset_hip_plan** part_plans;    /* [nsets] (HIP compute; NULL: no job) */
  redset_hip_plan** acc_plans;     /* [nsets] */
  hipEvent_t* ev_r;                /* [nsets] set k's partials arrived */
  int (*combine)(void*, const redset_hip_combine_job*, int, size_t, void*);
  void* combine_ctx;
  redset_hip_sharded_shape_info shape_info;
};

size_t redset_hip_shard_slice_bytes(size_t chunk_size, int world) {
  if (world < 1) world = 1;
  size_t w = (chunk_size + (size_t) world - 1) / (size_t) world;
  return (w + 255) & ~(size_t) 255;
}

static int is_encode(int kind) { return kind == REDSET_HIP_PLAN_RS_ENCODE || kind == REDSET_HIP_PLAN_XOR_ENCODE; }
static int is_xor(int kind) { return kind == REDSET_HIP_PLAN_XOR_ENCODE || kind == REDSET_HIP_PLAN_XOR_REBUILD; }

/* Which cells of each member some stripe's decode reads: need[r*p + c] for
 * member r's cell in stripe c (data or parity, whichever it is). Encode
 * reads every data cell; an XOR rebuild every cell of every survivor
 * (src/redset_xor_serial.c:202-273). */
static int plan_inputs(const redset_hip_rs* rs, int p, int e, int kind, int missing, const int* lost,
                       unsigned char* need) {
  memset(need, 0, (size_t) p * p);
  if (kind == REDSET_HIP_PLAN_RS_ENCODE) {
    for (int r = 0; r < p; ++r)
      for (int c = 0; c < p; ++c) need[r * p + c] = redset_hip_rs_get_encoding_id(p, e, r, c) < p;
    return 0;
  }
  if (kind == REDSET_HIP_PLAN_XOR_ENCODE) {
    for (int r = 0; r < p; ++r)
      for (int c = 0; c < p; ++c) need[r * p + c] = c != r; /* member r's parity is stripe r */
    return 0;
  }
  if (kind == REDSET_HIP_PLAN_XOR_REBUILD) {
    for (int r = 0; r < p; ++r)
      for (int c = 0; c < p; ++c) need[r * p + c] = r != lost[0];
    return 0;
  }
  unsigned char* D = malloc((size_t) missing * p);
  if (!D) return sfail("out of host memory");
  for (int c = 0; c < p; ++c) {
    if (redset_hip_rs_decode_matrix(rs, missing, lost, c, D)) {
      free(D);
      return REDSET_FAILURE;
    }
    for (int r = 0; r < p; ++r)
      for (int i = 0; i < missing; ++i)
        if (D[(size_t) i * p + r]) need[r * p + c] = 1;
  }
  free(D);
  return 0;
}

/* member r's cell in stripe c: data cell index, or -(1 + parity slot).
 * XOR: stripe r is member r's parity, stripe c != r its logical-file
 * segment c or c - 1 (src/redset_xor.c:251-266). */
static int cell_of(int p, int e, int kind, int r, int c) {
  if (is_xor(kind)) return c == r ? -1 : (c < r ? c : c - 1);
  const int enc = redset_hip_rs_get_encoding_id(p, e, r, c);
  return enc < p ? redset_hip_rs_get_data_id(p, e, r, c) : -(1 + (enc - p));
}

/* planning context: the layout and what this process is */
typedef struct {
  const redset_hip_shard_layout* L;
  const int* by_slot;         /* (h, j) -> member, or -1 */
  const unsigned char* need;  /* [p * p] member r's cell in stripe c is read */
  int p, e, d, mh, world, me, kind, missing;
  const int* lost;
  size_t W;
  const int* sidx;            /* [world] the column slice a process computes, or -1 */
  int me_s;                   /* mine */
} pctx;

/* addresses in this process's buffers (include/redset_hip.h layout) */
static unsigned char* hd(const pctx* C, int q, int j, int s) {
  return C->L->hosted_data + (((size_t) q * C->mh + j) * C->d + s) * C->W;
}
static unsigned char* hp(const pctx* C, int q, int j, int i) {
  return C->L->hosted_parity + (((size_t) q * C->mh + j) * C->e + i) * C->W;
}
static unsigned char* gd(const pctx* C, int h, int j, int s) {
  return C->L->gathered_data + (((size_t) h * C->mh + j) * C->d + s) * C->W;
}
static unsigned char* gp(const pctx* C, int h, int j, int i) {
  return C->L->gathered_parity + (((size_t) h * C->mh + j) * C->e + i) * C->W;
}

/* does some stripe read member r's data cell x (pass 0) / parity slot x (pass 1)? */
static int wanted(const pctx* C, int r, int pass, int x) {
  for (int c = 0; c < C->p; ++c)
    if (C->need[r * C->p + c] && cell_of(C->p, C->e, C->kind, r, c) == (pass == 0 ? x : -(1 + x))) return 1;
  return 0;
}

/* set k's gather: slice sidx[g] of every needed cell of every surviving
 * member of the set goes from its host to each computing process g; data
 * rows then parity rows, members in slot order (both ends of a pair walk the
 * same rows). My own slice of the members I host stays where it is: the
 * compute reads it in the hosted slabs (plan_sets), so nothing is copied
 * within the process */
static int plan_gather(const pctx* C, int k, exch* G) {
  const int me = C->me;
  int rc = 0;
  for (int g = 0; g < C->world && !rc; ++g) {
    if (g == me) continue;
    for (int pass = 0; pass < 2 && !rc; ++pass) {
      const int ncell = pass == 0 ? C->d : C->e;
      for (int j = 0; j < C->mh && !rc && C->sidx[g] >= 0; ++j) { /* what I send to g */
        const int m = C->by_slot[(size_t) me * C->mh + j];
        if (m < 0 || m / C->p != k) continue;
        for (int x = 0; x < ncell && !rc; ++x) {
          if (!wanted(C, m % C->p, pass, x)) continue;
          rc = ex_send(G, g, pass == 0 ? hd(C, C->sidx[g], j, x) : hp(C, C->sidx[g], j, x), C->W);
        }
      }
      for (int j = 0; j < C->mh && !rc && C->me_s >= 0; ++j) { /* my slice of g's members' needed cells */
        const int m = C->by_slot[(size_t) g * C->mh + j];
        if (m < 0 || m / C->p != k) continue;
        for (int x = 0; x < ncell && !rc; ++x)
          if (wanted(C, m % C->p, pass, x)) rc = ex_recv(G, g, pass == 0 ? gd(C, g, j, x) : gp(C, g, j, x), C->W);
      }
    }
  }
  return rc;
}

/* set k's return: the outputs (encode: every member's parity; rebuild: every
 * cell of the lost members) go from each computing process's gathered slots
 * to the member's host: data rows, then parity rows, members in set order. A
 * member I host got my slice in place (the compute wrote its hosted slab) */
static int plan_return(const pctx* C, int k, exch* R) {
  int rc = 0;
  for (int pass = 0; pass < 2 && !rc; ++pass) {
    if (pass == 0 && is_encode(C->kind)) continue; /* encode returns parity only */
    for (int m = k * C->p; m < (k + 1) * C->p && !rc; ++m) {
      int is_out = is_encode(C->kind);
      for (int i = 0; i < C->missing; ++i) is_out |= C->lost[i] == m % C->p;
      if (!is_out) continue;
      const int h = C->L->host[m], j = C->L->slot[m];
      const size_t len = (size_t) (pass == 0 ? C->d : C->e) * C->W;
      if (h != C->me) {
        if (C->me_s >= 0) rc = ex_send(R, h, pass == 0 ? gd(C, h, j, 0) : gp(C, h, j, 0), len);
        continue;
      }
      for (int g = 0; g < C->world && !rc; ++g)
        if (g != C->me && C->sidx[g] >= 0)
          rc = ex_recv(R, g, pass == 0 ? hd(C, C->sidx[g], j, 0) : hp(C, C->sidx[g], j, 0), len);
    }
  }
  return rc;
}

/* ---- the partial-sum shape (REDSET_HIP_SHAPE_REDUCE) ------------------- */
/*
 * Every output cell O of a stripe (a lost member's cell; encode: a parity
 * cell) is a linear combination of the stripe's input cells. The processes
 * hosting some input with a nonzero coefficient for O are O's contributors;
 * each one other than O's host combines ITS inputs into a partial cell and
 * sends it to O's host, which XORs the partials and its own inputs' share
 * into O. GF(2^8) addition is XOR, so the bytes equal the whole combination's
 * (the reference's multadd, src/redset_reedsolomon_common.c:786-819, sums in
 * another order to the same bytes).
 *
 * Slice by slice: a member's cells are stored as `world` column slabs, so
 * every combine works on one slice q of its cells (W bytes; the last slice's
 * padding is computed and sent too, and lands in padding). A partial's slice
 * q is a row of W bytes: in the sender's scratch (the gathered slabs, which
 * this shape does not otherwise use), and at the receiver either straight in
 * the output (the first remote contributor's, in rank order) or in the
 * receiver's scratch (the others'), from where the ACCUMULATE combine XORs
 * it in.
 *
 * Every process computes the same row allocation for every process, so a
 * pair's messages merge rows alike on both sides: a sender's rows for
 * receiver h, set k, lie in its scratch in the order (q, output); a
 * receiver's rows from sender g, set k, likewise; rows merge into one
 * message where both sides are contiguous.
 */
#define REDUCE_MAX_WORLD 64

typedef struct {
  int r, pass, x, c; /* member of the set, 0: data cell x / 1: parity slot x, stripe */
} ocell;

/* every output cell of a set (the same in every set) and its stripe's
 * coefficients over the p members, coef[o * p + s] */
static int set_outputs(const redset_hip_rs* rs, int p, int e, int kind, int missing, const int* lost, ocell** oc_out,
                       unsigned char** coef_out, int* nout_out) {
  const int per = is_encode(kind) ? e : missing;
  const int n = p * per;
  ocell* oc = malloc(sizeof(*oc) * (size_t) n);
  unsigned char* coef = calloc((size_t) n * p, 1);
  unsigned char* mat = rs ? malloc((size_t) (p + e) * p) : NULL;
  unsigned char* D = malloc((size_t) (missing > 0 ? missing : 1) * p);
  int rc = (!oc || !coef || !D || (rs && !mat)) ? sfail("out of host memory") : 0;
  if (!rc && rs) rc = redset_hip_rs_matrix(rs, mat);
  int o = 0;
  for (int c = 0; c < p && !rc; ++c) {
    if (kind == REDSET_HIP_PLAN_RS_REBUILD && (rc = redset_hip_rs_decode_matrix(rs, missing, lost, c, D))) break;
    for (int i = 0; i < p && o < n; ++i) {
      int r = -1;
      if (kind == REDSET_HIP_PLAN_RS_ENCODE) {
        if (redset_hip_rs_get_encoding_id(p, e, i, c) >= p) r = i;
      } else if (kind == REDSET_HIP_PLAN_XOR_ENCODE) {
        if (i == c) r = c;
      } else if (i < missing) {
        r = lost[i];
      }
      if (r < 0) continue;
      const int x = cell_of(p, e, kind, r, c);
      ocell O = {r, x >= 0 ? 0 : 1, x >= 0 ? x : -(1 + x), c};
      oc[o] = O;
      unsigned char* row = coef + (size_t) o * p;
      for (int t = 0; t < p; ++t) {
        if (kind == REDSET_HIP_PLAN_RS_ENCODE) {
          const int enc = redset_hip_rs_get_encoding_id(p, e, r, c);
          row[t] = redset_hip_rs_get_encoding_id(p, e, t, c) < p ? mat[(size_t) enc * p + t] : 0;
        } else if (kind == REDSET_HIP_PLAN_RS_REBUILD) {
          row[t] = D[(size_t) i * p + t];
        } else {
          row[t] = t != r;
        }
      }
      ++o;
    }
  }
  free(mat);
  free(D);
  if (!rc && o != n) rc = sfail("sharded plan: %d outputs per set, expected %d", o, n);
  if (rc) {
    free(oc);
    free(coef);
    return REDSET_FAILURE;
  }
  *oc_out = oc;
  *coef_out = coef;
  *nout_out = n;
  return 0;
}

/* the row allocation of the partial-sum shape for every process */
typedef struct {
  int world, nsets, nout, p, d, e, mh;
  size_t W, C;
  int nslices;              /* slices with cell bytes */
  const int *host, *slot;   /* layout placement */
  ocell* oc;
  unsigned char* coef;
  int* ord;                 /* [nsets][nout] set k's outputs by (pass, slot, cell) */
  uint64_t* mask;           /* [nsets][nout] contributing processes */
  int* srow;                /* [k][o][q][g] row of sender g's scratch, or -1 */
  int* rrow;                /* [k][o][q][g] row of the receiver's scratch, -1 (direct) */
  int* byhost;              /* [nsets][nout] set k's outputs in `ord` order, grouped by host */
  int* hoff;                /* [nsets][world + 1] host h's outputs: byhost[hoff[h] .. hoff[h + 1]) */
  long *S, *R;              /* [world] scratch rows sent / received into scratch */
  unsigned long long *sent, *recvd; /* [world] rows sent / received */
  long rows;                /* scratch rows per process (the gathered slabs) */
  int ok;                   /* fits, and every output has a contributor */
  int fused;                /* 1: an output's host folds its own inputs in with the partials it
                               makes (COMPUTE), and receives every partial into scratch; 0: the
                               first remote partial lands in the output and the host's own
                               inputs are combined again in ACCUMULATE (less scratch) */
} reduce_alloc;

static void ra_free(reduce_alloc* A) {
  free(A->oc);
  free(A->coef);
  free(A->ord);
  free(A->byhost);
  free(A->hoff);
  free(A->mask);
  free(A->srow);
  free(A->rrow);
  free(A->S);
  free(A->R);
  free(A->sent);
  free(A->recvd);
  memset(A, 0, sizeof(*A));
}

static size_t ra_key(const reduce_alloc* A, int k, int o, int q, int g) {
  return (((size_t) k * A->nout + o) * (size_t) A->world + (size_t) q) * (size_t) A->world + (size_t) g;
}
static int ra_host(const reduce_alloc* A, int k, int o) { return A->host[(size_t) k * A->p + A->oc[o].r]; }
static int ra_slot(const reduce_alloc* A, int k, int o) { return A->slot[(size_t) k * A->p + A->oc[o].r]; }
/* O's contributors other than its host */
static uint64_t ra_remote(const reduce_alloc* A, int k, int o) {
  return A->mask[(size_t) k * A->nout + o] & ~((uint64_t) 1 << ra_host(A, k, o));
}

/* where host h's outputs start among set k's outputs grouped by host */
static int ra_lo(const reduce_alloc* A, int k, int h) { return A->hoff[(size_t) k * (size_t) (A->world + 1) + (size_t) h]; }

/* set k's outputs by (pass, the host's slot, cell): the order of a pair's rows */
static int ra_before(const reduce_alloc* A, int k, int oa, int ob) {
  const ocell *x = &A->oc[oa], *y = &A->oc[ob];
  if (x->pass != y->pass) return x->pass < y->pass;
  const int sa = ra_slot(A, k, oa), sb = ra_slot(A, k, ob);
  if (sa != sb) return sa < sb;
  return x->x < y->x;
}
static void ra_sort(const reduce_alloc* A, int k, int* v, int n) {
  for (int i = 1; i < n; ++i) {
    const int t = v[i];
    int j = i;
    for (; j > 0 && ra_before(A, k, t, v[j - 1]); --j) v[j] = v[j - 1];
    v[j] = t;
  }
}

static int ra_build(reduce_alloc* A, const redset_hip_rs* rs, int p, int e, int kind, int missing, const int* lost,
                    const redset_hip_shard_layout* L, int world) {
  memset(A, 0, sizeof(*A));
  A->world = world;
  A->nsets = L->nsets;
  A->p = p;
  A->e = e;
  A->d = p - e;
  A->mh = L->max_hosted;
  A->W = L->slice_bytes;
  A->C = L->chunk_size;
  A->host = L->host;
  A->slot = L->slot;
  if (world < 2 || world > REDUCE_MAX_WORLD) return 0; /* not ok: nothing to reduce, or too wide */
  for (int q = 0; q < world; ++q)
    if ((size_t) q * A->W < A->C) A->nslices = q + 1;
  if (set_outputs(rs, p, e, kind, missing, lost, &A->oc, &A->coef, &A->nout)) return REDSET_FAILURE;
  const size_t nk = (size_t) A->nsets * A->nout, nkey = nk * (size_t) world * (size_t) world;
  if (nkey > ((size_t) 1 << 23)) return 0; /* too many rows to plan this way */
  A->ord = malloc(sizeof(int) * nk);
  A->byhost = malloc(sizeof(int) * nk);
  A->hoff = calloc((size_t) A->nsets * (size_t) (world + 1), sizeof(int));
  A->mask = calloc(nk, sizeof(uint64_t));
  A->srow = malloc(sizeof(int) * nkey);
  A->rrow = malloc(sizeof(int) * nkey);
  A->S = calloc((size_t) world, sizeof(long));
  A->R = calloc((size_t) world, sizeof(long));
  A->sent = calloc((size_t) world, sizeof(unsigned long long));
  A->recvd = calloc((size_t) world, sizeof(unsigned long long));
  if (!A->ord || !A->byhost || !A->hoff || !A->mask || !A->srow || !A->rrow || !A->S || !A->R || !A->sent ||
      !A->recvd)
    return sfail("out of host memory");
  for (size_t i = 0; i < nkey; ++i) A->srow[i] = A->rrow[i] = -1;
  A->ok = 1;
  for (int k = 0; k < A->nsets; ++k) {
    for (int o = 0; o < A->nout; ++o) {
      uint64_t m = 0;
      for (int t = 0; t < p; ++t)
        if (A->coef[(size_t) o * p + t]) m |= (uint64_t) 1 << A->host[(size_t) k * p + t];
      A->mask[(size_t) k * A->nout + o] = m;
      if (!m) A->ok = 0; /* an output nothing feeds: not this shape's business */
      A->ord[(size_t) k * A->nout + o] = o;
    }
    ra_sort(A, k, A->ord + (size_t) k * A->nout, A->nout);
    /* the sorted outputs bucketed by host, order kept */
    int* off = A->hoff + (size_t) k * (size_t) (world + 1);
    for (int o = 0; o < A->nout; ++o) ++off[ra_host(A, k, o) + 1];
    for (int h = 0; h < world; ++h) off[h + 1] += off[h];
    int* fill = calloc((size_t) world, sizeof(int));
    if (!fill) return sfail("out of host memory");
    for (int i = 0; i < A->nout; ++i) {
      const int o = A->ord[(size_t) k * A->nout + i], h = ra_host(A, k, o);
      A->byhost[(size_t) k * A->nout + (size_t) (off[h] + fill[h]++)] = o;
    }
    free(fill);
  }
  /* sender g's rows, in the order (set, receiver, slice, output) */
  for (int k = 0; k < A->nsets; ++k)
    for (int h = 0; h < world; ++h)
      for (int q = 0; q < A->nslices; ++q)
        for (int i = ra_lo(A, k, h); i < ra_lo(A, k, h + 1); ++i) {
          const int o = A->byhost[(size_t) k * A->nout + i];
          const uint64_t rem = ra_remote(A, k, o);
          for (int g = 0; g < world; ++g)
            if (rem >> g & 1) {
              A->srow[ra_key(A, k, o, q, g)] = A->S[g]++;
              ++A->sent[g];
              ++A->recvd[h];
            }
        }
  /* receiver h's scratch rows (after its sent ones), in the order (set,
   * sender, slice, output). The first remote contributor's row goes
   * straight into the output when the output's host has no share of its
   * own to write there first (fused), or always (direct); the fused
   * allocation is tried first, the direct one if that does not fit */
  A->rows = (long) world * A->mh * (A->d + A->e);
  for (int g = 0; g < world; ++g)
    if (A->S[g] > A->rows || A->S[g] > INT_MAX / 2) A->ok = 0;
  int first = 1;
#if REDSET_HIP_TEST_KNOBS
  /* test builds: the direct allocation even where the fused one fits, so
   * small test sets run it (tests/test_mpi_sharded.py) */
  if (getenv("REDSET_HIP_TEST_REDUCE_DIRECT")) first = 0;
#endif
  for (int fused = first; fused >= 0 && A->ok; --fused) {
    int fits = 1;
    for (int h = 0; h < world; ++h) A->R[h] = 0;
    for (int k = 0; k < A->nsets; ++k)
      for (int h = 0; h < world; ++h)
        for (int g = 0; g < world; ++g)
          for (int q = 0; q < A->nslices; ++q)
            for (int i = ra_lo(A, k, h); i < ra_lo(A, k, h + 1); ++i) {
              const int o = A->byhost[(size_t) k * A->nout + i];
              const uint64_t rem = ra_remote(A, k, o);
              const int own = (int) (A->mask[(size_t) k * A->nout + o] >> h & 1);
              const size_t key = ra_key(A, k, o, q, g);
              A->rrow[key] = -1;
              if (!(rem >> g & 1)) continue;
              if ((rem & (~rem + 1)) == ((uint64_t) 1 << g) && !(fused && own)) continue; /* direct */
              A->rrow[key] = (int) (A->S[h] + A->R[h]++);
            }
    for (int g = 0; g < world; ++g)
      if (A->S[g] + A->R[g] > A->rows) fits = 0;
    if (fits) {
      A->fused = fused;
      return 0;
    }
  }
  A->ok = 0;
  return 0;
}

/* a row's place in process memory: buffer (0 hosted data, 1 hosted parity,
 * 2 gathered data, 3 gathered parity) and offset */
typedef struct {
  int buf;
  size_t off;
} rloc;

static rloc ra_scratch(const reduce_alloc* A, long row) {  /* row >= 0 */
  const long nD = (long) A->world * A->mh * A->d;
  rloc l = {row < nD ? 2 : 3, (size_t) (row < nD ? row : row - nD) * A->W};
  return l;
}
static rloc ra_output(const reduce_alloc* A, int k, int o, int q) {
  const ocell* O = &A->oc[o];
  const int j = ra_slot(A, k, o);
  rloc l = {O->pass, (((size_t) q * A->mh + (size_t) j) * (size_t) (O->pass ? A->e : A->d) + (size_t) O->x) * A->W};
  return l;
}
/* where sender g's row of (k, o, q) lands at the receiver */
static rloc ra_dest(const reduce_alloc* A, int k, int o, int q, int g) {
  const int r = A->rrow[ra_key(A, k, o, q, g)];
  return r < 0 ? ra_output(A, k, o, q) : ra_scratch(A, r);
}

static unsigned char* ra_ptr(const redset_hip_shard_layout* L, rloc l) {
  unsigned char* base[4] = {L->hosted_data, L->hosted_parity, L->gathered_data, L->gathered_parity};
  return base[l.buf] + l.off;
}

/* member t of set k's cell in stripe c, slice q, in my hosted slabs */
static unsigned char* ra_input(const reduce_alloc* A, const redset_hip_shard_layout* L, int kind, int k, int t, int c,
                               int q) {
  const int j = A->slot[(size_t) k * A->p + t], x = cell_of(A->p, A->e, kind, t, c);
  rloc l = {x >= 0 ? 0 : 1, 0};
  l.off = (((size_t) q * A->mh + (size_t) j) * (size_t) (x >= 0 ? A->d : A->e) + (size_t) (x >= 0 ? x : -(1 + x))) * A->W;
  return ra_ptr(L, l);
}

/* one direction of a pair's rows in set k as merged messages: the rows of
 * outputs hosted by `h` that `g` contributes to, (slice, output) order;
 * g == me: my sends to h, else my receives from g (h == me) */
static int ra_messages(const reduce_alloc* A, const redset_hip_shard_layout* L, int k, int g, int h, int me,
                       xlist* out, int* nmsg, unsigned long long* bytes) {
  int have = 0;
  rloc s0 = {0, 0}, r0 = {0, 0};
  size_t len = 0;
  for (int q = 0; q < A->nslices; ++q)
    for (int i = ra_lo(A, k, h); i < ra_lo(A, k, h + 1); ++i) {
      const int o = A->byhost[(size_t) k * A->nout + i];
      if (!(ra_remote(A, k, o) >> g & 1)) continue;
      const rloc sl = ra_scratch(A, A->srow[ra_key(A, k, o, q, g)]), rl = ra_dest(A, k, o, q, g);
      if (have && sl.buf == s0.buf && sl.off == s0.off + len && rl.buf == r0.buf && rl.off == r0.off + len) {
        len += A->W;
        continue;
      }
      if (have) {
        redset_hip_xfer x = {g == me ? h : g, g == me, ra_ptr(L, g == me ? s0 : r0), len};
        if (xl_push(out, x)) return REDSET_FAILURE;
        ++*nmsg;
        *bytes += len;
      }
      have = 1;
      s0 = sl;
      r0 = rl;
      len = A->W;
    }
  if (have) {
    redset_hip_xfer x = {g == me ? h : g, g == me, ra_ptr(L, g == me ? s0 : r0), len};
    if (xl_push(out, x)) return REDSET_FAILURE;
    ++*nmsg;
    *bytes += len;
  }
  return 0;
}

/* does some partial of output o, slice q, land in its host's scratch? */
static int ra_has_scratch(const reduce_alloc* A, int k, int o, int q) {
  for (int g = 0; g < A->world; ++g)
    if (A->rrow[ra_key(A, k, o, q, g)] >= 0) return 1;
  return 0;
}

/* my combines and exchanges of the partial-sum shape (A->ok) */
static int plan_reduce(redset_hip_sharded* P, const reduce_alloc* A, const redset_hip_shard_layout* L, int kind,
                       int me) {
  const int world = A->world, p = A->p, nout = A->nout;
  int rc = 0;
  P->part = calloc((size_t) A->nsets, sizeof(cset));
  P->acc = calloc((size_t) A->nsets, sizeof(cset));
  P->goff = calloc((size_t) A->nsets + 1, sizeof(int));
  P->roff = calloc((size_t) A->nsets + 1, sizeof(int));
  int* sel = malloc(sizeof(int) * (size_t) nout);
  int* ins = malloc(sizeof(int) * (size_t) p);
  const size_t maxin = (size_t) p + (size_t) nout * (size_t) world;
  unsigned char** ip = malloc(sizeof(*ip) * maxin);
  unsigned char** op = malloc(sizeof(*op) * (size_t) nout);
  unsigned char* cf = malloc(maxin * (size_t) nout);
  if (!P->part || !P->acc || !P->goff || !P->roff || !sel || !ins || !ip || !op || !cf) rc = sfail("out of host memory");
  for (int k = 0; k < A->nsets && !rc; ++k) {
    /* combines: stripe by stripe, slice by slice, the outputs grouped by host */
    for (int c = 0; c < p && !rc; ++c)
      for (int q = 0; q < A->nslices && !rc; ++q) {
        const size_t n = A->C - (size_t) q * A->W < A->W ? A->C - (size_t) q * A->W : A->W;
        /* the jobs: (h, grp) = (host, 0) the partials for that host (h ==
         * me: the outputs only my inputs feed); (me, 1) my outputs that
         * partials arrive for (ACCUMULATE). Fused: (-1, 0) one job making
         * every output my inputs feed -- partials for other hosts and my own
         * outputs' shares -- so my inputs are read once, and (me, 1) XORs
         * the partials in my scratch into my outputs */
        for (int h = A->fused ? -1 : 0; h < world && !rc; ++h)
          for (int grp = 0; grp < (h == me ? 2 : 1) && !rc; ++grp) {
            if (A->fused && h >= 0 && !(h == me && grp == 1)) continue;
            int ns = 0;
            for (int o = 0; o < nout; ++o) {
              if (A->oc[o].c != c || (h >= 0 && ra_host(A, k, o) != h)) continue;
              const uint64_t rem = ra_remote(A, k, o);
              const int own = (int) (A->mask[(size_t) k * A->nout + o] >> me & 1);
              int take;
              if (h < 0) take = own;  /* fused COMPUTE */
              else if (h != me) take = (int) (rem >> me & 1);
              else if (A->fused) take = ra_has_scratch(A, k, o, q);
              else take = grp == 0 ? rem == 0 : rem != 0;
              if (take) sel[ns++] = o;
            }
            if (ns == 0) continue;
            /* my inputs with a coefficient for one of them (fused
             * accumulate: none, the partials only) */
            int ni = 0;
            for (int t = 0; t < p && !(A->fused && grp == 1); ++t) {
              if (A->host[(size_t) k * p + t] != me) continue;
              int used = 0;
              for (int a = 0; a < ns && !used; ++a) used = A->coef[(size_t) sel[a] * p + t] != 0;
              if (used) ins[ni++] = t;
            }
            int nin = ni;
            for (int a = 0; a < ni; ++a) ip[a] = ra_input(A, L, kind, k, ins[a], c, q);
            /* the accumulate's extra inputs: partials in my scratch */
            const int extra0 = nin;
            for (int a = 0; grp == 1 && a < ns; ++a)
              for (int g = 0; g < world; ++g) {
                const int r = A->rrow[ra_key(A, k, sel[a], q, g)];
                if (ra_remote(A, k, sel[a]) >> g & 1 && r >= 0) ip[nin++] = ra_ptr(L, ra_scratch(A, r));
              }
            if (nin == 0) {
              if (grp == 0 && h == me) rc = sfail("sharded plan: an output with no input");
              continue; /* grp 1 (direct): the one partial that arrived is the output */
            }
            memset(cf, 0, (size_t) nin * (size_t) ns);
            int ex = extra0;
            for (int a = 0; a < ns; ++a) {
              const int o = sel[a];
              for (int b = 0; b < ni; ++b) cf[(size_t) a * nin + b] = A->coef[(size_t) o * p + ins[b]];
              op[a] = ra_host(A, k, o) == me ? ra_ptr(L, ra_output(A, k, o, q))
                                             : ra_ptr(L, ra_scratch(A, A->srow[ra_key(A, k, o, q, me)]));
              for (int g = 0; grp == 1 && g < world; ++g)
                if (ra_remote(A, k, o) >> g & 1 && A->rrow[ra_key(A, k, o, q, g)] >= 0) cf[(size_t) a * nin + ex++] = 1;
            }
            rc = cs_add(grp == 1 ? &P->acc[k] : &P->part[k], nin, ip, ns, op, cf, grp == 1, n);
          }
      }
    /* the partial exchange: per peer my sends, then my receives */
    xlist X;
    memset(&X, 0, sizeof(X));
    for (int g = 0; g < world && !rc; ++g) {
      if (g == me) continue;
      rc = ra_messages(A, L, k, me, g, me, &X, &P->info.return_messages, &P->info.return_bytes_sent);
      if (!rc) rc = ra_messages(A, L, k, g, me, me, &X, &P->info.return_recv_messages, &P->info.return_bytes_recv);
    }
    for (int i = 0; i < X.n && !rc; ++i) {
      if (X.v[i].send) {
        if (X.v[i].len > P->info.return_msg_max) P->info.return_msg_max = X.v[i].len;
        if (!P->info.return_msg_min || X.v[i].len < P->info.return_msg_min) P->info.return_msg_min = X.v[i].len;
      }
      rc = xl_push(&P->ret, X.v[i]);
    }
    free(X.v);
    P->goff[k + 1] = 0;
    P->roff[k + 1] = P->ret.n;
    cs_finish(&P->part[k]);
    cs_finish(&P->acc[k]);
    P->info.compute_bytes += P->part[k].bytes + P->acc[k].bytes;
  }
  free(sel);
  free(ins);
  free(ip);
  free(op);
  free(cf);
  return rc;
}

/* the gather shape's bytes sent / received by every process, from the
 * placement alone (the planner's lists carry the same totals; merging rows
 * into messages does not change them): every wanted cell of a member goes,
 * one W-byte slice each, to every computing process but its host, and every
 * output cell of a member comes back from every computing process but its
 * host. O(members x processes), so AUTO can weigh every process's counts
 * at any world size */
static int gather_counts_all(const pctx* C, unsigned long long* sent, unsigned long long* recvd) {
  const int p = C->p, world = C->world;
  int* wc = calloc((size_t) p, sizeof(int)); /* member r's wanted cells */
  if (!wc) return sfail("out of host memory");
  for (int r = 0; r < p; ++r) {
    for (int x = 0; x < C->d; ++x) wc[r] += wanted(C, r, 0, x);
    for (int x = 0; x < C->e; ++x) wc[r] += wanted(C, r, 1, x);
  }
  int K = 0;
  for (int g = 0; g < world; ++g) K += C->sidx[g] >= 0;
  memset(sent, 0, sizeof(*sent) * (size_t) world);
  memset(recvd, 0, sizeof(*recvd) * (size_t) world);
  const unsigned long long W = C->W;
  for (int k = 0; k < C->L->nsets; ++k)
    for (int r = 0; r < p; ++r) {
      const int h = C->L->host[(size_t) k * p + r], hc = C->sidx[h] >= 0;
      /* the gather: my wanted cells to every other computing process */
      sent[h] += (unsigned long long) wc[r] * W * (unsigned long long) (K - hc);
      for (int g = 0; g < world && wc[r]; ++g)
        if (g != h && C->sidx[g] >= 0) recvd[g] += (unsigned long long) wc[r] * W;
      /* the return: an output member's cells from every other computing process */
      int is_out = is_encode(C->kind);
      for (int i = 0; i < C->missing; ++i) is_out |= C->lost[i] == r;
      if (!is_out) continue;
      const unsigned long long len = (unsigned long long) (is_encode(C->kind) ? C->e : C->d + C->e) * W;
      recvd[h] += len * (unsigned long long) (K - hc);
      for (int g = 0; g < world; ++g)
        if (g != h && C->sidx[g] >= 0) sent[g] += len;
    }
  free(wc);
  return 0;
}

/* what the _ex entry points pass down; the legacy ones plan GATHER and
 * compare nothing */
typedef struct {
  int shape;       /* REDSET_HIP_SHAPE_* */
  int compare;     /* count both shapes (the _ex entry points) */
  int (*combine)(void*, const redset_hip_combine_job*, int, size_t, void*);
  void* combine_ctx;
} shape_req;

/* the plan of either scheme: rs (RS kinds) or NULL (XOR kinds, e = 1);
 * compute: which processes compute a column slice (NULL: all) */
static int plan_sets(const redset_hip_rs* rs, int p, int e, int kind, int missing, const int* rebuild_ranks,
                     const redset_hip_shard_layout* L, const int* compute, const redset_hip_transport* tr,
                     const redset_hip_compute* comp, const shape_req* want, redset_hip_sharded** out) {
  if (is_encode(kind)) missing = 0;
  if (!is_encode(kind)) {
    if (missing < 1 || missing > e) return sfail("cannot rebuild %d members with %d parity chunks", missing, e);
    if (!rebuild_ranks) return sfail("null rebuild_ranks");
    for (int i = 0; i < missing; ++i)
      if (rebuild_ranks[i] < 0 || rebuild_ranks[i] >= p || (i && rebuild_ranks[i] <= rebuild_ranks[i - 1]))
        return sfail("rebuild ranks must be ascending members of 0..%d", p - 1);
  }
  const int world = tr->world, me = tr->rank, d = p - e;
  if (world < 1 || me < 0 || me >= world) return sfail("transport world %d / rank %d invalid", world, me);
  if (L->nsets < 1 || !L->host || !L->slot || L->max_hosted < 1) return sfail("sharded layout: bad placement");
  /* the column slice each process computes: the K computing processes in
   * rank order take slices 0 .. K - 1 */
  int* sidx = malloc(sizeof(int) * (size_t) world);
  if (!sidx) return sfail("out of host memory");
  int K = 0;
  for (int g = 0; g < world; ++g) sidx[g] = (!compute || compute[g]) ? K++ : -1;
  const size_t W = L->slice_bytes;
  if (K == 0 || W == 0 || W * (size_t) K < L->chunk_size) {
    free(sidx);
    return K == 0 ? sfail("sharded plan: no process computes")
                  : sfail("slice_bytes %zu too small for %zu over %d", W, L->chunk_size, K);
  }
  if (!L->hosted_data || !L->hosted_parity || !L->gathered_data || !L->gathered_parity) {
    free(sidx);
    return sfail("sharded layout: null buffer");
  }
  const int nm = L->nsets * p, mh = L->max_hosted;
  {
    /* every (host, slot) at most once */
    unsigned char* used = calloc((size_t) world * mh, 1);
    if (!used) {
      free(sidx);
      return sfail("out of host memory");
    }
    for (int m = 0; m < nm; ++m) {
      const int h = L->host[m], j = L->slot[m];
      if (h < 0 || h >= world || j < 0 || j >= mh || used[(size_t) h * mh + j]) {
        free(used);
        free(sidx);
        return sfail("sharded layout: member %d placed at (%d, %d) invalid or twice", m, h, j);
      }
      used[(size_t) h * mh + j] = 1;
    }
    free(used);
  }

  redset_hip_sharded* P = calloc(1, sizeof(*P));
  unsigned char* need = malloc((size_t) p * p);
  int* by_slot = malloc(sizeof(int) * (size_t) world * mh); /* (h, j) -> member, or -1 */
  exch G, R;
  reduce_alloc A;
  memset(&G, 0, sizeof(G));
  memset(&R, 0, sizeof(R));
  memset(&A, 0, sizeof(A));
  int rc = (!P || !need || !by_slot) ? sfail("out of host memory") : 0;
  if (!rc) rc = ex_init(&G, world, me);
  if (!rc) rc = ex_init(&R, world, me);
  if (rc) goto done;
  P->tr = *tr;
  if (comp) P->comp = *comp;
  P->p = p;
  P->e = e;
  P->missing = missing;
  for (int i = 0; i < missing; ++i) P->lost[i] = rebuild_ranks[i];
  P->W = W;
  P->info.kind = kind;
  P->info.world = world;
  P->info.rank = me;
  P->info.nsets = L->nsets;
  P->info.missing = missing;
  P->shape = REDSET_HIP_SHAPE_GATHER;
  P->shape_info.struct_size = sizeof(P->shape_info);
  P->shape_info.scratch_bytes = (unsigned long long) world * mh * p * W;
  if (sidx[me] >= 0) {
    const size_t lo = (size_t) sidx[me] * W;
    P->info.my_slice_len = lo >= L->chunk_size ? 0 : (L->chunk_size - lo < W ? L->chunk_size - lo : W);
  }
  for (int i = 0; i < world * mh; ++i) by_slot[i] = -1;
  for (int m = 0; m < nm; ++m) by_slot[(size_t) L->host[m] * mh + L->slot[m]] = m;
  if ((rc = plan_inputs(rs, p, e, kind, missing, rebuild_ranks, need))) goto done;

  pctx C = {L, by_slot, need, p, e, d, mh, world, me, kind, missing, P->lost, W, sidx, sidx[me]};

  /* the shape: both counted (the _ex entry points), the one asked for or
   * the one whose busiest process moves fewer bytes */
  if (want && want->compare) {
    redset_hip_sharded_shape_info* S = &P->shape_info;
    unsigned long long* gs = calloc((size_t) world * 2, sizeof(unsigned long long));
    rc = gs ? gather_counts_all(&C, gs, gs + world) : sfail("out of host memory");
    for (int g = 0; g < world && !rc; ++g) {
      const unsigned long long b = gs[g] > gs[world + g] ? gs[g] : gs[world + g];
      if (b > S->gather_busiest_bytes) S->gather_busiest_bytes = b;
    }
    if (!rc) S->gather_bytes_sent = gs[me], S->gather_bytes_recv = gs[world + me];
    free(gs);
    /* the partial sums need every process computing, and either the HIP
     * plans or a combine callback (a whole-set callback cannot run them) */
    const int can = !compute && (!comp || !comp->run || want->combine);
    if (!rc && can) rc = ra_build(&A, rs, p, e, kind, missing, rebuild_ranks, L, world);
    if (!rc && A.ok) {
      S->reduce_possible = 1;
      for (int g = 0; g < world; ++g) {
        const unsigned long long b = (A.sent[g] > A.recvd[g] ? A.sent[g] : A.recvd[g]) * W;
        if (b > S->reduce_busiest_bytes) S->reduce_busiest_bytes = b;
      }
      S->reduce_bytes_sent = A.sent[me] * W;
      S->reduce_bytes_recv = A.recvd[me] * W;
      S->scratch_bytes_needed = (unsigned long long) (A.S[me] + A.R[me]) * W;
      S->reduce_fused = A.fused;
    }
    if (!rc && want->shape == REDSET_HIP_SHAPE_REDUCE && !A.ok)
      rc = sfail(world < 2 ? "sharded plan: the partial-sum shape needs at least 2 processes"
                 : !can   ? "sharded plan: the partial-sum shape needs every process computing and HIP or combine compute"
                          : "sharded plan: the partial sums do not fit the gathered slabs (or over 64 processes)");
    if (!rc && A.ok &&
        (want->shape == REDSET_HIP_SHAPE_REDUCE ||
         (want->shape == REDSET_HIP_SHAPE_AUTO && S->reduce_busiest_bytes < S->gather_busiest_bytes)))
      P->shape = REDSET_HIP_SHAPE_REDUCE;
  }
  P->shape_info.shape = P->shape;
  if (rc) goto done;

  if (P->shape == REDSET_HIP_SHAPE_REDUCE) {
    P->combine = want->combine;
    P->combine_ctx = want->combine_ctx;
    P->info.my_slice_len = L->chunk_size; /* every process combines whole cells' worth of its inputs */
    rc = plan_reduce(P, &A, L, kind, me);
    P->shape_info.reduce_messages = P->info.return_messages;
    P->shape_info.reduce_recv_messages = P->info.return_recv_messages;
    if (!rc && !P->combine) {
      P->part_plans = calloc((size_t) L->nsets, sizeof(*P->part_plans));
      P->acc_plans = calloc((size_t) L->nsets, sizeof(*P->acc_plans));
      if (!P->part_plans || !P->acc_plans) rc = sfail("out of host memory");
      for (int k = 0; k < L->nsets && !rc; ++k) {
        if (P->part[k].n) rc = redset_hip_plan_combine(P->part[k].v, P->part[k].n, W, &P->part_plans[k]);
        if (!rc && P->acc[k].n) rc = redset_hip_plan_combine(P->acc[k].v, P->acc[k].n, W, &P->acc_plans[k]);
      }
    }
    goto done;
  }

  P->goff = calloc((size_t) L->nsets + 1, sizeof(int));
  P->roff = calloc((size_t) L->nsets + 1, sizeof(int));
  if (!P->goff || !P->roff) {
    rc = sfail("out of host memory");
    goto done;
  }
  /* set by set, so a set's exchanges can run on their own (pipelined execute) */
  for (int k = 0; k < L->nsets && !rc; ++k) {
    rc = plan_gather(&C, k, &G);
    const xstats gs = {&P->info.gather_messages, &P->info.gather_recv_messages, &P->info.gather_bytes_sent,
                       &P->info.gather_bytes_recv, &P->info.gather_msg_max, &P->info.gather_msg_min};
    const xstats rs_ = {&P->info.return_messages, &P->info.return_recv_messages, &P->info.return_bytes_sent,
                        &P->info.return_bytes_recv, &P->info.return_msg_max, &P->info.return_msg_min};
    if (!rc) rc = ex_flatten(&G, &P->gather, &gs);
    if (!rc) rc = plan_return(&C, k, &R);
    if (!rc) rc = ex_flatten(&R, &P->ret, &rs_);
    P->goff[k + 1] = P->gather.n;
    P->roff[k + 1] = P->ret.n;
    ex_free(&G);
    ex_free(&R);
    if (!rc) rc = ex_init(&G, world, me);
    if (!rc) rc = ex_init(&R, world, me);
  }
  if (rc) goto done;

  /* compute: every set over my slices, cell stride W: a member hosted
   * elsewhere in the gathered layout, a member I host in place in its
   * hosted slabs (my slice q = sidx[me] is [d][W] / [e][W] there too); a
   * process that computes nothing keeps no pointers */
  P->plans = calloc((size_t) L->nsets, sizeof(*P->plans));
  P->lofi = malloc(sizeof(*P->lofi) * (size_t) nm);
  P->parity = malloc(sizeof(*P->parity) * (size_t) nm);
  if (!P->plans || !P->lofi || !P->parity) {
    rc = sfail("out of host memory");
    goto done;
  }
  for (int m = 0; m < nm; ++m) {
    const int local = L->host[m] == me, q = C.me_s < 0 ? 0 : C.me_s;
    P->lofi[m] = local ? hd(&C, q, L->slot[m], 0) : gd(&C, L->host[m], L->slot[m], 0);
    P->parity[m] = local ? hp(&C, q, L->slot[m], 0) : gp(&C, L->host[m], L->slot[m], 0);
  }
  const size_t n = P->info.my_slice_len;
  P->info.compute_bytes = (unsigned long long) L->nsets * p * (d + (is_encode(kind) ? e : missing)) * n;
  for (int k = 0; k < L->nsets && !rc && n > 0 && !P->comp.run; ++k) {
    unsigned char* const* lf = P->lofi + (size_t) k * p;
    unsigned char* const* pr = P->parity + (size_t) k * p;
    switch (kind) {
      case REDSET_HIP_PLAN_RS_ENCODE: rc = redset_hip_rs_plan_encode(rs, lf, pr, n, W, &P->plans[k]); break;
      case REDSET_HIP_PLAN_RS_REBUILD:
        rc = redset_hip_rs_plan_rebuild(rs, missing, P->lost, lf, pr, n, W, &P->plans[k]);
        break;
      case REDSET_HIP_PLAN_XOR_ENCODE: rc = redset_hip_xor_plan_encode(p, lf, pr, n, W, &P->plans[k]); break;
      default: rc = redset_hip_xor_plan_rebuild(p, P->lost[0], lf, pr, n, W, &P->plans[k]); break;
    }
  }
done:
  ex_free(&G);
  ex_free(&R);
  ra_free(&A);
  free(need);
  free(by_slot);
  free(sidx);
  if (rc) {
    redset_hip_sharded_destroy(P);
    return REDSET_FAILURE;
  }
  *out = P;
  return REDSET_SUCCESS;
}

int redset_hip_rs_sharded_plan_on(const redset_hip_rs* rs, int kind, int missing, const int* rebuild_ranks,
                                  const redset_hip_shard_layout* L, const int* compute,
                                  const redset_hip_transport* tr, const redset_hip_compute* comp,
                                  redset_hip_sharded** out) {
  int p, e;
  if (!out) return sfail("sharded_plan: null out-pointer");
  *out = NULL;
  if (!rs || !L || !tr || !tr->exchange) return sfail("sharded_plan: null argument");
  if (redset_hip_rs_shape(rs, &p, &e)) return REDSET_FAILURE;
  if (kind != REDSET_HIP_PLAN_RS_ENCODE && kind != REDSET_HIP_PLAN_RS_REBUILD)
    return sfail("sharded_plan: kind %d is not RS encode or rebuild", kind);
  return plan_sets(rs, p, e, kind, missing, rebuild_ranks, L, compute, tr, comp, NULL, out);
}

int redset_hip_rs_sharded_plan(const redset_hip_rs* rs, int kind, int missing, const int* rebuild_ranks,
                               const redset_hip_shard_layout* L, const redset_hip_transport* tr,
                               const redset_hip_compute* comp, redset_hip_sharded** out) {
  return redset_hip_rs_sharded_plan_on(rs, kind, missing, rebuild_ranks, L, NULL, tr, comp, out);
}

int redset_hip_xor_sharded_plan_on(int ranks, int kind, int root, const redset_hip_shard_layout* L,
                                   const int* compute, const redset_hip_transport* tr,
                                   const redset_hip_compute* comp, redset_hip_sharded** out) {
  if (!out) return sfail("xor_sharded_plan: null out-pointer");
  *out = NULL;
  if (!L || !tr || !tr->exchange) return sfail("xor_sharded_plan: null argument");
  if (ranks < 2 || ranks > MAX_RANKS) return sfail("XOR needs 2..%d ranks, got %d", MAX_RANKS, ranks);
  if (kind != REDSET_HIP_PLAN_XOR_ENCODE && kind != REDSET_HIP_PLAN_XOR_REBUILD)
    return sfail("xor_sharded_plan: kind %d is not XOR encode or rebuild", kind);
  if (kind == REDSET_HIP_PLAN_XOR_REBUILD && (root < 0 || root >= ranks))
    return sfail("root %d out of range", root);
  return plan_sets(NULL, ranks, 1, kind, kind == REDSET_HIP_PLAN_XOR_REBUILD ? 1 : 0, &root, L, compute, tr, comp,
                   NULL, out);
}

int redset_hip_xor_sharded_plan(int ranks, int kind, int root, const redset_hip_shard_layout* L,
                                const redset_hip_transport* tr, const redset_hip_compute* comp,
                                redset_hip_sharded** out) {
  return redset_hip_xor_sharded_plan_on(ranks, kind, root, L, NULL, tr, comp, out);
}

static int opts_req(const redset_hip_sharded_opts* o, shape_req* w) {
  memset(w, 0, sizeof(*w));
  w->compare = 1;
  if (!o) return 0;
  if (o->struct_size != sizeof(*o))
    return sfail("sharded_plan_ex: opts.struct_size %zu, this library's is %zu", o->struct_size, sizeof(*o));
  if (o->shape < REDSET_HIP_SHAPE_AUTO || o->shape > REDSET_HIP_SHAPE_REDUCE)
    return sfail("sharded_plan_ex: unknown shape %d", o->shape);
  w->shape = o->shape;
  w->combine = o->combine;
  w->combine_ctx = o->combine_ctx;
  return 0;
}

int redset_hip_rs_sharded_plan_ex(const redset_hip_rs* rs, int kind, int missing, const int* rebuild_ranks,
                                  const redset_hip_shard_layout* L, const redset_hip_transport* tr,
                                  const redset_hip_sharded_opts* opts, redset_hip_sharded** out) {
  int p, e;
  shape_req w;
  if (!out) return sfail("sharded_plan_ex: null out-pointer");
  *out = NULL;
  if (!rs || !L || !tr || !tr->exchange) return sfail("sharded_plan_ex: null argument");
  if (opts_req(opts, &w)) return REDSET_FAILURE;
  if (redset_hip_rs_shape(rs, &p, &e)) return REDSET_FAILURE;
  if (kind != REDSET_HIP_PLAN_RS_ENCODE && kind != REDSET_HIP_PLAN_RS_REBUILD)
    return sfail("sharded_plan_ex: kind %d is not RS encode or rebuild", kind);
  return plan_sets(rs, p, e, kind, missing, rebuild_ranks, L, opts ? opts->compute_on : NULL, tr,
                   opts ? opts->compute : NULL, &w, out);
}

int redset_hip_xor_sharded_plan_ex(int ranks, int kind, int root, const redset_hip_shard_layout* L,
                                   const redset_hip_transport* tr, const redset_hip_sharded_opts* opts,
                                   redset_hip_sharded** out) {
  shape_req w;
  if (!out) return sfail("xor_sharded_plan_ex: null out-pointer");
  *out = NULL;
  if (!L || !tr || !tr->exchange) return sfail("xor_sharded_plan_ex: null argument");
  if (opts_req(opts, &w)) return REDSET_FAILURE;
  if (ranks < 2 || ranks > MAX_RANKS) return sfail("XOR needs 2..%d ranks, got %d", MAX_RANKS, ranks);
  if (kind != REDSET_HIP_PLAN_XOR_ENCODE && kind != REDSET_HIP_PLAN_XOR_REBUILD)
    return sfail("xor_sharded_plan_ex: kind %d is not XOR encode or rebuild", kind);
  if (kind == REDSET_HIP_PLAN_XOR_REBUILD && (root < 0 || root >= ranks))
    return sfail("root %d out of range", root);
  return plan_sets(NULL, ranks, 1, kind, kind == REDSET_HIP_PLAN_XOR_REBUILD ? 1 : 0, &root, L,
                   opts ? opts->compute_on : NULL, tr, opts ? opts->compute : NULL, &w, out);
}

int redset_hip_sharded_get_shape(const redset_hip_sharded* P, redset_hip_sharded_shape_info* info, size_t size) {
  if (!P || !info) return sfail("null argument");
  memcpy(info, &P->shape_info, size < sizeof(P->shape_info) ? size : sizeof(P->shape_info));
  return REDSET_SUCCESS;
}

static int compute_set(redset_hip_sharded* P, int k, void* stream) {
  const size_t n = P->info.my_slice_len;
  if (n == 0) return REDSET_SUCCESS;
  if (P->comp.run) {
    if (P->comp.run(P->comp.ctx, P->info.kind, P->missing, P->lost, P->lofi + (size_t) k * P->p,
                    P->parity + (size_t) k * P->p, n, P->W, stream) != 0)
      return sfail("sharded compute callback failed (set %d)", k);
    return REDSET_SUCCESS;
  }
  return redset_hip_plan_execute(P->plans[k], stream);
}

/* transfers [lo, hi) of list L as one exchange */
static int exchange(redset_hip_sharded* P, const xlist* L, int lo, int hi, void* stream, const char* what) {
  if (hi > lo && P->tr.exchange(P->tr.ctx, L->v + lo, hi - lo, stream) != 0)
    return sfail("sharded %s: transport exchange failed", what);
  return REDSET_SUCCESS;
}

/* the partial-sum shape's combines of set k: COMPUTE (partials, outputs
 * only my inputs feed) or ACCUMULATE (outputs partials arrived for) */
static int reduce_set(redset_hip_sharded* P, int k, int acc, void* stream) {
  const cset* S = acc ? &P->acc[k] : &P->part[k];
  if (S->n == 0) return REDSET_SUCCESS;
  if (P->combine) {
    if (P->combine(P->combine_ctx, S->v, S->n, P->W, stream) != 0)
      return sfail("sharded combine callback failed (set %d)", k);
    return REDSET_SUCCESS;
  }
  return redset_hip_plan_execute(acc ? P->acc_plans[k] : P->part_plans[k], stream);
}

int redset_hip_sharded_execute_phase(redset_hip_sharded* P, int phase, void* stream) {
  if (!P) return sfail("null sharded plan");
  const int reduce = P->shape == REDSET_HIP_SHAPE_REDUCE;
  switch (phase) {
    case REDSET_HIP_PHASE_GATHER:
      return reduce ? REDSET_SUCCESS : exchange(P, &P->gather, 0, P->gather.n, stream, "gather");
    case REDSET_HIP_PHASE_COMPUTE:
      for (int k = 0; k < P->info.nsets; ++k)
        if (reduce ? reduce_set(P, k, 0, stream) : compute_set(P, k, stream)) return REDSET_FAILURE;
      return REDSET_SUCCESS;
    case REDSET_HIP_PHASE_RETURN:
      return exchange(P, &P->ret, 0, P->ret.n, stream, reduce ? "partial sums" : "return");
    case REDSET_HIP_PHASE_ACCUMULATE:
      for (int k = 0; k < P->info.nsets && reduce; ++k)
        if (reduce_set(P, k, 1, stream)) return REDSET_FAILURE;
      return REDSET_SUCCESS;
    default:
      return sfail("unknown sharded phase %d", phase);
  }
}

static int hfail(const char* what, hipError_t e) { return sfail("sharded execute: %s: %s", what, hipGetErrorString(e)); }

/* Sets pipelined over two streams: set k+1's gather runs on the plan's
 * exchange stream while set k's gf_mac runs on the caller's, and the returns
 * follow the gathers there, each after its own set's compute (so the last
 * compute overlaps the first returns). Exchange stream: G0 .. G(n-1) R0 ..
 * R(n-1); caller's stream: C0 .. C(n-1), each after its gather. Both start
 * after the work already on `stream`, and `stream` resumes after the last
 * return. A transport that completes its exchange before returning (MPI)
 * overlaps the same way: the host runs gather k+1 while the GPU computes k.
 * After a local HIP or compute error every exchange still runs (the other
 * members are in them and would wait forever, src/redset_reedsolomon.c:
 * 338-342): the bytes this member sends are then unspecified, and the error
 * is returned at the end. */
/* the plan's exchange stream and events, made on the first execute */
static int pipe_setup(redset_hip_sharded* P) {
  hipError_t e;
  int rc = 0;
  const int n = P->info.nsets;
  if (!P->xstream && !P->ev_c) {
    P->ev_c = calloc((size_t) n, sizeof(hipEvent_t));
    P->ev_r = calloc((size_t) n, sizeof(hipEvent_t));
    if (!P->ev_c || !P->ev_r) rc = sfail("out of host memory");
    if (!rc && (e = hipStreamCreateWithFlags(&P->xstream, hipStreamNonBlocking)) != hipSuccess) rc = hfail("stream", e);
    if (!rc && (e = hipEventCreateWithFlags(&P->ev_x, hipEventDisableTiming)) != hipSuccess) rc = hfail("event", e);
    for (int k = 0; k < n && !rc; ++k)
      if ((e = hipEventCreateWithFlags(&P->ev_c[k], hipEventDisableTiming)) != hipSuccess ||
          (e = hipEventCreateWithFlags(&P->ev_r[k], hipEventDisableTiming)) != hipSuccess)
        rc = hfail("event", e);
  } else if (!P->xstream || !P->ev_x) {
    rc = sfail("sharded execute: the plan's stream or events were not created");
  }
  return rc;
}

/* The partial-sum shape pipelined: every set's partial sums on the caller's
 * stream, one after another; set k's exchange on the exchange stream as soon
 * as its partials are made (so it overlaps set k+1's); set k's accumulate on
 * the caller's stream once its exchange is done. Host order: all partial
 * combines enqueued first, then per set its exchange and accumulate, so a
 * transport that completes its exchange before returning (MPI) overlaps the
 * same way. Every exchange runs after a local error (the peers are in it). */
static int execute_reduce(redset_hip_sharded* P, hipStream_t s) {
  hipError_t e;
  const int n = P->info.nsets;
  if (P->ret.n == 0) {
    int rc = 0;
    for (int k = 0; k < n && !rc; ++k) rc = reduce_set(P, k, 0, s);
    for (int k = 0; k < n && !rc; ++k) rc = reduce_set(P, k, 1, s);
    return rc;
  }
  int rc = pipe_setup(P);
  hipStream_t x = P->xstream ? P->xstream : s;
  if (!rc && ((e = hipEventRecord(P->ev_x, s)) != hipSuccess || (e = hipStreamWaitEvent(x, P->ev_x, 0)) != hipSuccess))
    rc = hfail("order after the caller's stream", e);
  for (int k = 0; k < n; ++k) {
    if (!rc && reduce_set(P, k, 0, s)) rc = REDSET_FAILURE;
    if (!rc && (e = hipEventRecord(P->ev_c[k], s)) != hipSuccess) rc = hfail("partials event", e);
  }
  for (int k = 0; k < n; ++k) {
    if (!rc && (e = hipStreamWaitEvent(x, P->ev_c[k], 0)) != hipSuccess) rc = hfail("partials -> exchange", e);
    if (exchange(P, &P->ret, P->roff[k], P->roff[k + 1], x, "partial sums") && !rc) rc = REDSET_FAILURE;
    if (!rc && ((e = hipEventRecord(P->ev_r[k], x)) != hipSuccess || (e = hipStreamWaitEvent(s, P->ev_r[k], 0)) != hipSuccess))
      rc = hfail("exchange -> accumulate", e);
    if (!rc && reduce_set(P, k, 1, s)) rc = REDSET_FAILURE;
  }
  return rc;
}

static int execute_pipelined(redset_hip_sharded* P, hipStream_t s) {
  hipError_t e;
  int rc = 0;
  const int n = P->info.nsets;
  if (P->gather.n == 0 && P->ret.n == 0) {
    /* nothing to exchange (one process, or only its own slices): the
     * computes alone, on the caller's stream, with no second stream to
     * order against */
    for (int k = 0; k < n && !rc; ++k) rc = compute_set(P, k, s);
    return rc;
  }
  rc = pipe_setup(P);
  /* without its own stream (a failed setup) the exchanges go on `s` */
  hipStream_t x = P->xstream ? P->xstream : s;
  /* the exchange stream starts after the caller's work (ev_c[0] is free until
   * compute 0 records it) */
  if (!rc && ((e = hipEventRecord(P->ev_c[0], s)) != hipSuccess || (e = hipStreamWaitEvent(x, P->ev_c[0], 0)) != hipSuccess))
    rc = hfail("order after the caller's stream", e);
  for (int k = 0; k < n; ++k) {
    if (exchange(P, &P->gather, P->goff[k], P->goff[k + 1], x, "gather") && !rc) rc = REDSET_FAILURE;
    if (!rc && ((e = hipEventRecord(P->ev_x, x)) != hipSuccess || (e = hipStreamWaitEvent(s, P->ev_x, 0)) != hipSuccess))
      rc = hfail("gather -> compute", e);
    if (!rc && compute_set(P, k, s)) rc = REDSET_FAILURE;
    if (!rc && (e = hipEventRecord(P->ev_c[k], s)) != hipSuccess) rc = hfail("compute event", e);
  }
  for (int k = 0; k < n; ++k) {
    if (P->roff[k + 1] == P->roff[k]) continue;
    if (!rc && (e = hipStreamWaitEvent(x, P->ev_c[k], 0)) != hipSuccess) rc = hfail("compute -> return", e);
    if (exchange(P, &P->ret, P->roff[k], P->roff[k + 1], x, "return") && !rc) rc = REDSET_FAILURE;
  }
  if (!rc && ((e = hipEventRecord(P->ev_x, x)) != hipSuccess || (e = hipStreamWaitEvent(s, P->ev_x, 0)) != hipSuccess))
    rc = hfail("order the caller's stream after the returns", e);
  return rc;
}

int redset_hip_sharded_execute(redset_hip_sharded* P, void* stream) {
  if (!P) return sfail("null sharded plan");
  const int reduce = P->shape == REDSET_HIP_SHAPE_REDUCE;
  if ((!reduce && P->comp.run) || (reduce && P->combine)) {
    /* every phase runs after a failed one (see execute_pipelined) */
    int rc = 0;
    for (int ph = REDSET_HIP_PHASE_GATHER; ph <= REDSET_HIP_PHASE_ACCUMULATE; ++ph)
      if (redset_hip_sharded_execute_phase(P, ph, stream) && !rc) rc = REDSET_FAILURE;
    return rc;
  }
  return reduce ? execute_reduce(P, (hipStream_t) stream) : execute_pipelined(P, (hipStream_t) stream);
}

int redset_hip_sharded_get_info(const redset_hip_sharded* P, redset_hip_sharded_info* info) {
  if (!P || !info) return sfail("null argument");
  *info = P->info;
  return REDSET_SUCCESS;
}

void redset_hip_sharded_destroy(redset_hip_sharded* P) {
  if (!P) return;
  for (int k = 0; P->plans && k < P->info.nsets; ++k) redset_hip_plan_destroy(P->plans[k]);
  free(P->plans);
  for (int k = 0; k < P->info.nsets; ++k) {
    if (P->part_plans) redset_hip_plan_destroy(P->part_plans[k]);
    if (P->acc_plans) redset_hip_plan_destroy(P->acc_plans[k]);
    if (P->part) cs_free(&P->part[k]);
    if (P->acc) cs_free(&P->acc[k]);
  }
  free(P->part_plans);
  free(P->acc_plans);
  free(P->part);
  free(P->acc);
  if (P->xstream) (void) hipStreamSynchronize(P->xstream);
  for (int k = 0; P->ev_c && k < P->info.nsets; ++k)
    if (P->ev_c[k]) (void) hipEventDestroy(P->ev_c[k]);
  for (int k = 0; P->ev_r && k < P->info.nsets; ++k)
    if (P->ev_r[k]) (void) hipEventDestroy(P->ev_r[k]);
  free(P->ev_c);
  free(P->ev_r);
  if (P->ev_x) (void) hipEventDestroy(P->ev_x);
  if (P->xstream) (void) hipStreamDestroy(P->xstream);
  free(P->goff);
  free(P->roff);
  free(P->lofi);
  free(P->parity);
  free(P->gather.v);
  free(P->ret.v);
  free(P);
}
