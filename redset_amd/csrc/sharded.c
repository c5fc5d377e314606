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

/* the plan of either scheme: rs (RS kinds) or NULL (XOR kinds, e = 1);
 * compute: which processes compute a column slice (NULL: all) */
static int plan_sets(const redset_hip_rs* rs, int p, int e, int kind, int missing, const int* rebuild_ranks,
                     const redset_hip_shard_layout* L, const int* compute, const redset_hip_transport* tr,
                     const redset_hip_compute* comp, redset_hip_sharded** out) {
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
  memset(&G, 0, sizeof(G));
  memset(&R, 0, sizeof(R));
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
  if (sidx[me] >= 0) {
    const size_t lo = (size_t) sidx[me] * W;
    P->info.my_slice_len = lo >= L->chunk_size ? 0 : (L->chunk_size - lo < W ? L->chunk_size - lo : W);
  }
  for (int i = 0; i < world * mh; ++i) by_slot[i] = -1;
  for (int m = 0; m < nm; ++m) by_slot[(size_t) L->host[m] * mh + L->slot[m]] = m;
  if ((rc = plan_inputs(rs, p, e, kind, missing, rebuild_ranks, need))) goto done;

  pctx C = {L, by_slot, need, p, e, d, mh, world, me, kind, missing, P->lost, W, sidx, sidx[me]};
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
  return plan_sets(rs, p, e, kind, missing, rebuild_ranks, L, compute, tr, comp, out);
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
                   out);
}

int redset_hip_xor_sharded_plan(int ranks, int kind, int root, const redset_hip_shard_layout* L,
                                const redset_hip_transport* tr, const redset_hip_compute* comp,
                                redset_hip_sharded** out) {
  return redset_hip_xor_sharded_plan_on(ranks, kind, root, L, NULL, tr, comp, out);
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

int redset_hip_sharded_execute_phase(redset_hip_sharded* P, int phase, void* stream) {
  if (!P) return sfail("null sharded plan");
  switch (phase) {
    case REDSET_HIP_PHASE_GATHER:
      return exchange(P, &P->gather, 0, P->gather.n, stream, "gather");
    case REDSET_HIP_PHASE_COMPUTE:
      for (int k = 0; k < P->info.nsets; ++k)
        if (compute_set(P, k, stream)) return REDSET_FAILURE;
      return REDSET_SUCCESS;
    case REDSET_HIP_PHASE_RETURN:
      return exchange(P, &P->ret, 0, P->ret.n, stream, "return");
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
  if (!P->xstream && !P->ev_c) {
    P->ev_c = calloc((size_t) n, sizeof(hipEvent_t));
    if (!P->ev_c) rc = sfail("out of host memory");
    if (!rc && (e = hipStreamCreateWithFlags(&P->xstream, hipStreamNonBlocking)) != hipSuccess) rc = hfail("stream", e);
    if (!rc && (e = hipEventCreateWithFlags(&P->ev_x, hipEventDisableTiming)) != hipSuccess) rc = hfail("event", e);
    for (int k = 0; k < n && !rc; ++k)
      if ((e = hipEventCreateWithFlags(&P->ev_c[k], hipEventDisableTiming)) != hipSuccess) rc = hfail("event", e);
  } else if (!P->xstream || !P->ev_x) {
    rc = sfail("sharded execute: the plan's stream or events were not created");
  }
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
  if (P->comp.run) {
    /* every phase runs after a failed one (see execute_pipelined) */
    int rc = 0;
    for (int ph = REDSET_HIP_PHASE_GATHER; ph <= REDSET_HIP_PHASE_RETURN; ++ph)
      if (redset_hip_sharded_execute_phase(P, ph, stream) && !rc) rc = REDSET_FAILURE;
    return rc;
  }
  return execute_pipelined(P, (hipStream_t) stream);
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
  if (P->xstream) (void) hipStreamSynchronize(P->xstream);
  for (int k = 0; P->ev_c && k < P->info.nsets; ++k)
    if (P->ev_c[k]) (void) hipEventDestroy(P->ev_c[k]);
  free(P->ev_c);
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
