/*
 * sharded_test.c -- the sharded encode / rebuild of include/redset_hip.h
 * under mpirun on CPU: every MPI process is one "GPU" of the node, the C
 * planner (redset_hip_rs_sharded_plan) moves column slices through the MPI
 * transport (redset_hip_mpi_transport_*, host buffers) and the compute is a
 * callback into the CPU oracle (test infrastructure), so the placement, the
 * slicing and both exchanges are checked against the oracle's whole-set
 * encode / rebuild without a GPU.
 *
 * usage: sharded_test [--gpu | --gpu-host | --gpu-host-null] <p> <e> <chunk> [lost ranks...]   (world = MPI size)
 * SHARDED_TEST_SCHEME=xor: an XOR set (redset_hip_xor_sharded_plan; e must be
 * 1 and the one lost rank is the root), checked against the oracle's XOR.
 * SHARDED_TEST_REPS=<n> (--gpu): after the checks, time n rebuilds with the
 * pipelined execute and n with the three phases one after another (slowest
 * process, ms per rebuild).
 * --gpu: the slabs live in HBM, the compute is the HIP gf_mac plans and the
 * MPI transport stages through pinned host memory (every process may share
 * one GPU) -- the whole sharded path with the real kernels at world > 1.
 * --gpu-host: the slabs live in page-locked host memory, the compute is the
 * HIP gf_mac plans reading and writing them in place, and the MPI transport
 * works on the host buffers directly -- it must wait for the kernels that
 * wrote a return exchange's slices before it sends them.
 * --gpu-host-null: the same on the null stream (the transport is
 * created for HIP-written host buffers, device_buffers = 2, and must wait for
 * the null stream too).
 * SHARDED_TEST_IDLE=<r,r,...>: those processes compute no column slice
 * (redset_hip_*_sharded_plan_on with the complementary mask; the others take
 * slices 0 .. K - 1 of W = ceil(C / K)); they still host members, send their
 * cells and receive their outputs.
 * SHARDED_TEST_SHAPE=gather|reduce|auto: plan through redset_hip_*_sharded_plan_ex
 * with that exchange shape (REDSET_HIP_SHAPE_*; CPU mode: the partial sums'
 * combines go to the oracle's multadd); every process prints the shape it
 * planned and both shapes' byte counts.
 * SHARDED_TEST_TRANSPORT=rccl: the RCCL transport (transport_rccl.c) instead
 * of MPI's; the unique id goes out by MPI_Bcast. On the one-GPU test box and
 * on the CPU this runs against tests/rcclstub (LD_LIBRARY_PATH), which
 * accepts any number of ranks per GPU.
 * Placement: `world` sets of p members, member m on process (m * 7 + 3) %
 * world (SHARDED_TEST_SEED=<s>: on a pseudo-random process), hosted slots in
 * ascending member order. Exit 0 iff every process
 * found its hosted parity (after encode) and its lost members' cells (after
 * rebuild) equal to the oracle's.
 */
#include <hip/hip_runtime_api.h>
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "redset_hip.h"
#include "redset_hip_mpi.h"
#include "redset_oracle.h"

static int P, E, D, XOR;
static ro_rs* ORACLE;
/* SHARDED_TEST_FAIL_COMPUTE=<rank>: that process's compute callback fails in
 * the encode (the plan must still run every exchange, or its peers hang) */
static int ME, FAIL_COMPUTE = -1;

static uint8_t byte_of(int k, int r, size_t i) { /* member (k, r)'s logical-file byte i */
  uint64_t z = ((uint64_t) k << 48) ^ ((uint64_t) r << 32) ^ (uint64_t) i ^ 0x5EEDULL;
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return (uint8_t) (z ^ (z >> 31));
}

/* slab copies: hipMemcpy / hipMemset for HBM slabs, plain memory ops for
 * page-locked host slabs (after the stream's kernels are done with them) */
static int HOST_SLABS;
static int to_slab(void* dst, const void* src, size_t n) {
  if (HOST_SLABS) return memcpy(dst, src, n), 0;
  return hipMemcpy(dst, src, n, hipMemcpyHostToDevice) != hipSuccess;
}
static int from_slab(void* dst, const void* src, size_t n) {
  if (HOST_SLABS) return memcpy(dst, src, n), 0;
  return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) != hipSuccess;
}
static int fill_slab(void* dst, int v, size_t n) {
  if (HOST_SLABS) return memset(dst, v, n), 0;
  return hipMemset(dst, v, n) != hipSuccess;
}

/* compute callback: the oracle on compacted copies of the slices */
static int oracle_run(void* ctx, int kind, int missing, const int* lost, unsigned char* const* lofi,
                      unsigned char* const* parity, size_t n, size_t W, void* stream) {
  if (ME == FAIL_COMPUTE && (kind == REDSET_HIP_PLAN_RS_ENCODE || kind == REDSET_HIP_PLAN_XOR_ENCODE)) return 1;
  uint8_t** lf = malloc(sizeof(*lf) * P);
  uint8_t** pr = malloc(sizeof(*pr) * P);
  for (int r = 0; r < P; ++r) {
    lf[r] = malloc((size_t) D * n + 1);
    pr[r] = malloc((size_t) E * n + 1);
    for (int s = 0; s < D; ++s) memcpy(lf[r] + (size_t) s * n, lofi[r] + (size_t) s * W, n);
    for (int i = 0; i < E; ++i) memcpy(pr[r] + (size_t) i * n, parity[r] + (size_t) i * W, n);
  }
  int rc = 0;
  if (kind == REDSET_HIP_PLAN_RS_ENCODE) ro_rs_encode_set(ORACLE, n, lf, pr, 1 << 20);
  else if (kind == REDSET_HIP_PLAN_RS_REBUILD) rc = ro_rs_rebuild_set(ORACLE, n, missing, lost, lf, pr, 1 << 20);
  else if (kind == REDSET_HIP_PLAN_XOR_ENCODE) ro_xor_encode_set(P, n, lf, pr, 1 << 20);
  else if (missing == 1) ro_xor_rebuild_set(P, n, lost[0], lf, pr, 1 << 20);
  else rc = 1;
  for (int r = 0; r < P; ++r) {
    for (int s = 0; s < D; ++s) memcpy(lofi[r] + (size_t) s * W, lf[r] + (size_t) s * n, n);
    for (int i = 0; i < E; ++i) memcpy(parity[r] + (size_t) i * W, pr[r] + (size_t) i * n, n);
    free(lf[r]);
    free(pr[r]);
  }
  free(lf);
  free(pr);
  return rc;
}

/* the partial-sum shape's combines on the CPU: the oracle's multadd
 * (src/redset_reedsolomon_common.c:786-819) per output and input */
static int oracle_combine(void* ctx, const redset_hip_combine_job* jobs, int njobs, size_t n, void* stream) {
  (void) ctx;
  (void) stream;
  if (ME == FAIL_COMPUTE) return 1; /* SHARDED_TEST_FAIL_COMPUTE: the encode's first combine fails */
  for (int k = 0; k < njobs; ++k) {
    const redset_hip_combine_job* J = &jobs[k];
    for (int j = 0; j < J->nout; ++j) {
      if (!J->accumulate) memset(J->out[j], 0, n);
      for (int i = 0; i < J->nin; ++i)
        if (J->coef[j * J->nin + i]) ro_rs_multadd(ORACLE, n, J->out[j], J->coef[j * J->nin + i], J->in[i]);
    }
  }
  return 0;
}

static const char* shape_name(int s) {
  return s == REDSET_HIP_SHAPE_REDUCE ? "reduce" : s == REDSET_HIP_SHAPE_GATHER ? "gather" : "auto";
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int world, me;
  MPI_Comm_size(MPI_COMM_WORLD, &world);
  MPI_Comm_rank(MPI_COMM_WORLD, &me);
  ME = me;
  if (getenv("SHARDED_TEST_FAIL_COMPUTE")) FAIL_COMPUTE = atoi(getenv("SHARDED_TEST_FAIL_COMPUTE"));
  const int null_stream = argc > 1 && strcmp(argv[1], "--gpu-host-null") == 0;
  const int host_slabs = null_stream || (argc > 1 && strcmp(argv[1], "--gpu-host") == 0);
  const int gpu = host_slabs || (argc > 1 && strcmp(argv[1], "--gpu") == 0);
  HOST_SLABS = host_slabs;
  if (gpu) {
    --argc;
    ++argv;
  }
  if (argc < 4) MPI_Abort(MPI_COMM_WORLD, 2);
  P = atoi(argv[1]);
  E = atoi(argv[2]);
  D = P - E;
  XOR = getenv("SHARDED_TEST_SCHEME") && strcmp(getenv("SHARDED_TEST_SCHEME"), "xor") == 0;
  if (XOR && E != 1) MPI_Abort(MPI_COMM_WORLD, 2);
  const size_t C = (size_t) atoll(argv[3]);
  const int missing = argc - 4;
  int lost[64];
  for (int i = 0; i < missing; ++i) lost[i] = atoi(argv[4 + i]);
  ORACLE = ro_rs_new(P, E);

  const int nsets = world, nm = nsets * P;
  int* host = malloc(sizeof(int) * nm);
  int* slot = malloc(sizeof(int) * nm);
  int* count = calloc(world, sizeof(int));
  int mh = 0;
  const char* seed_env = getenv("SHARDED_TEST_SEED");
  for (int m = 0; m < nm; ++m) {
    /* SHARDED_TEST_SEED: members on random processes (unbalanced allowed) */
    host[m] = seed_env ? (int) (byte_of(0x7FFF, atoi(seed_env), (size_t) m) % world) : (m * 7 + 3) % world;
    slot[m] = count[host[m]]++;
    if (count[host[m]] > mh) mh = count[host[m]];
  }
  /* the processes that compute: all, or all but SHARDED_TEST_IDLE's */
  int* on = malloc(sizeof(int) * world);
  int NS = 0; /* column slices */
  for (int g = 0; g < world; ++g) on[g] = 1;
  if (getenv("SHARDED_TEST_IDLE")) {
    char* list = strdup(getenv("SHARDED_TEST_IDLE"));
    for (char* t = strtok(list, ","); t; t = strtok(NULL, ","))
      if (atoi(t) >= 0 && atoi(t) < world) on[atoi(t)] = 0;
    free(list);
  }
  for (int g = 0; g < world; ++g) NS += on[g];
  if (NS == 0) MPI_Abort(MPI_COMM_WORLD, 2);
  const size_t W = redset_hip_shard_slice_bytes(C, NS);
  const size_t hd = (size_t) world * mh * D * W, hp = (size_t) world * mh * E * W;
  uint8_t* HD = calloc(hd, 1);
  uint8_t* HP = calloc(hp, 1);
  uint8_t* GD = calloc(hd, 1);
  uint8_t* GP = calloc(hp, 1);
  /* my hosted members' slabs: slice q of data cell s */
  for (int m = 0; m < nm; ++m) {
    if (host[m] != me) continue;
    for (int q = 0; q < NS; ++q)
      for (int s = 0; s < D; ++s)
        for (size_t b = 0; b < W && q * W + b < C; ++b)
          HD[(((size_t) q * mh + slot[m]) * D + s) * W + b] = byte_of(m / P, m % P, s * C + q * W + b);
  }
  /* the oracle's whole-set answer for every set */
  uint8_t** want_l = malloc(sizeof(uint8_t*) * nm);
  uint8_t** want_p = malloc(sizeof(uint8_t*) * nm);
  for (int m = 0; m < nm; ++m) {
    want_l[m] = malloc((size_t) D * C);
    want_p[m] = calloc((size_t) E * C, 1);
    for (size_t i = 0; i < (size_t) D * C; ++i) want_l[m][i] = byte_of(m / P, m % P, i);
  }
  for (int k = 0; k < nsets; ++k) {
    if (XOR) ro_xor_encode_set(P, C, want_l + k * P, want_p + k * P, 1 << 20);
    else ro_rs_encode_set(ORACLE, C, want_l + k * P, want_p + k * P, 1 << 20);
  }

  redset_hip_rs* rs = NULL;
  redset_hip_transport tr;
  redset_hip_mpi_transport* th = NULL;
  redset_hip_compute comp = {oracle_run, NULL};
  redset_hip_shard_layout L = {nsets, host, slot, mh, C, W, HD, HP, GD, GP};
  uint8_t *dHD = NULL, *dHP = NULL, *dGD = NULL, *dGP = NULL;
  hipStream_t stream = NULL;
  if (host_slabs) {
    /* every slab page-locked; kernels and MPI use the same addresses */
    if (hipHostMalloc((void**) &dHD, hd, 0) || hipHostMalloc((void**) &dHP, hp, 0) ||
        hipHostMalloc((void**) &dGD, hd, 0) || hipHostMalloc((void**) &dGP, hp, 0) ||
        (!null_stream && hipStreamCreate(&stream))) {
      fprintf(stderr, "rank %d: pinned setup failed\n", me);
      MPI_Abort(MPI_COMM_WORLD, 3);
    }
    memcpy(dHD, HD, hd);
    memset(dHP, 0, hp);
    memset(dGD, 0, hd);
    memset(dGP, 0, hp);
    L.hosted_data = dHD;
    L.hosted_parity = dHP;
    L.gathered_data = dGD;
    L.gathered_parity = dGP;
  } else if (gpu) {
    if (hipMalloc((void**) &dHD, hd) || hipMalloc((void**) &dHP, hp) || hipMalloc((void**) &dGD, hd) ||
        hipMalloc((void**) &dGP, hp) || hipStreamCreate(&stream) || hipMemcpy(dHD, HD, hd, hipMemcpyHostToDevice) ||
        hipMemset(dHP, 0, hp) || hipMemset(dGD, 0, hd) || hipMemset(dGP, 0, hp)) {
      fprintf(stderr, "rank %d: device setup failed\n", me);
      MPI_Abort(MPI_COMM_WORLD, 3);
    }
    L.hosted_data = dHD;
    L.hosted_parity = dHP;
    L.gathered_data = dGD;
    L.gathered_parity = dGP;
  }
  redset_hip_sharded *enc = NULL, *reb = NULL;
  const redset_hip_compute* cp = gpu ? NULL : &comp;
  const char* tenv = getenv("SHARDED_TEST_TRANSPORT");
  const int use_rccl = tenv && strcmp(tenv, "rccl") == 0;
  redset_hip_rccl* rh = NULL;
  int ok = XOR || redset_hip_rs_create(P, E, &rs) == 0;
  if (ok && use_rccl) {
    unsigned char uid[128];
    memset(uid, 0, sizeof(uid));
    int got = me != 0 || redset_hip_rccl_unique_id(uid) == 0, all_got = 0;
    MPI_Allreduce(&got, &all_got, 1, MPI_INT, MPI_LAND, MPI_COMM_WORLD);
    MPI_Bcast(uid, 128, MPI_BYTE, 0, MPI_COMM_WORLD);
    ok = all_got && redset_hip_rccl_transport_create(uid, world, me, &tr, &rh) == 0;
  } else if (ok) {
    ok = redset_hip_mpi_transport_create(MPI_COMM_WORLD, host_slabs ? 2 : gpu ? 1 : 0, &tr, &th) == 0;
  }
  const char* shape_env = getenv("SHARDED_TEST_SHAPE");
  redset_hip_sharded_opts opts;
  memset(&opts, 0, sizeof(opts));
  opts.struct_size = sizeof(opts);
  opts.shape = !shape_env ? REDSET_HIP_SHAPE_AUTO
               : strcmp(shape_env, "reduce") == 0 ? REDSET_HIP_SHAPE_REDUCE
               : strcmp(shape_env, "gather") == 0 ? REDSET_HIP_SHAPE_GATHER
                                                  : REDSET_HIP_SHAPE_AUTO;
  opts.compute_on = getenv("SHARDED_TEST_IDLE") ? on : NULL;
  opts.compute = cp;
  opts.combine = gpu ? NULL : oracle_combine;
  if (ok && shape_env && XOR)
    ok = redset_hip_xor_sharded_plan_ex(P, REDSET_HIP_PLAN_XOR_ENCODE, 0, &L, &tr, &opts, &enc) == 0 &&
         (missing == 0 ||
          (missing == 1 && redset_hip_xor_sharded_plan_ex(P, REDSET_HIP_PLAN_XOR_REBUILD, lost[0], &L, &tr, &opts, &reb) == 0));
  else if (ok && shape_env)
    ok = redset_hip_rs_sharded_plan_ex(rs, REDSET_HIP_PLAN_RS_ENCODE, 0, NULL, &L, &tr, &opts, &enc) == 0 &&
         (missing == 0 || redset_hip_rs_sharded_plan_ex(rs, REDSET_HIP_PLAN_RS_REBUILD, missing, lost, &L, &tr, &opts, &reb) == 0);
  else if (ok && XOR)
    ok = redset_hip_xor_sharded_plan_on(P, REDSET_HIP_PLAN_XOR_ENCODE, 0, &L, on, &tr, cp, &enc) == 0 &&
         (missing == 0 || (missing == 1 && redset_hip_xor_sharded_plan_on(P, REDSET_HIP_PLAN_XOR_REBUILD, lost[0], &L, on,
                                                                            &tr, cp, &reb) == 0));
  else if (ok)
    ok = redset_hip_rs_sharded_plan_on(rs, REDSET_HIP_PLAN_RS_ENCODE, 0, NULL, &L, on, &tr, cp, &enc) == 0 &&
         (missing == 0 ||
          redset_hip_rs_sharded_plan_on(rs, REDSET_HIP_PLAN_RS_REBUILD, missing, lost, &L, on, &tr, cp, &reb) == 0);
  if (!ok) fprintf(stderr, "rank %d: setup: %s\n", me, redset_hip_last_error());
  for (int i = 0; ok && shape_env && i < 2; ++i) {
    redset_hip_sharded* pl = i == 0 ? enc : reb;
    redset_hip_sharded_shape_info si;
    if (!pl || redset_hip_sharded_get_shape(pl, &si, sizeof(si)) != 0) continue;
    printf("rank %d: %s shape %s (asked %s): gather busiest %llu B, reduce busiest %llu B (possible %d), "
           "sent %llu / %llu B, scratch %llu of %llu B, fused %d\n",
           me, i == 0 ? "encode" : "rebuild", shape_name(si.shape), shape_name(opts.shape), si.gather_busiest_bytes,
           si.reduce_busiest_bytes, si.reduce_possible, si.gather_bytes_sent, si.reduce_bytes_sent,
           si.scratch_bytes_needed, si.scratch_bytes, si.reduce_fused);
    /* the shape counts (computed from the placement) against the planned
     * lists' own totals */
    redset_hip_sharded_info inf;
    if (redset_hip_sharded_get_info(pl, &inf) == 0) {
      const unsigned long long ls = inf.gather_bytes_sent + inf.return_bytes_sent;
      const unsigned long long lr = inf.gather_bytes_recv + inf.return_bytes_recv;
      const unsigned long long ws = si.shape == REDSET_HIP_SHAPE_REDUCE ? si.reduce_bytes_sent : si.gather_bytes_sent;
      const unsigned long long wr = si.shape == REDSET_HIP_SHAPE_REDUCE ? si.reduce_bytes_recv : si.gather_bytes_recv;
      if (ls != ws || lr != wr) {
        fprintf(stderr, "rank %d: %s: the shape info counts %llu / %llu B, the plan's lists %llu / %llu B\n", me,
                i == 0 ? "encode" : "rebuild", ws, wr, ls, lr);
        ok = 0;
      }
    }
  }
  int bad = 0;
  if (ok && redset_hip_sharded_execute(enc, stream) != 0) {
    fprintf(stderr, "rank %d: encode: %s\n", me, redset_hip_last_error());
    ok = 0;
  }
  if (gpu && (hipStreamSynchronize(stream) || from_slab(HP, dHP, hp))) ok = 0;
  /* compare my hosted members' parity slabs with the oracle */
  for (int m = 0; ok && m < nm; ++m) {
    if (host[m] != me) continue;
    for (int q = 0; q < NS; ++q)
      for (int i = 0; i < E; ++i)
        for (size_t b = 0; b < W && q * W + b < C; ++b)
          bad += HP[(((size_t) q * mh + slot[m]) * E + i) * W + b] != want_p[m][i * C + q * W + b];
  }
  if (bad) fprintf(stderr, "rank %d: %d parity bytes differ from the oracle\n", me, bad);
  /* the rebuild is collective: every member runs it or none (as the
   * backends agree before an exchange) */
  int enc_ok = ok, all_enc = 0;
  MPI_Allreduce(&enc_ok, &all_enc, 1, MPI_INT, MPI_LAND, MPI_COMM_WORLD);
  if (ok && reb && all_enc) {
    /* lose the members, scribble on the gathered slots, rebuild */
    for (int m = 0; m < nm; ++m) {
      int is_lost = 0;
      for (int i = 0; i < missing; ++i) is_lost |= lost[i] == m % P;
      if (!is_lost || host[m] != me) continue;
      for (int q = 0; q < NS; ++q) {
        memset(HD + (((size_t) q * mh + slot[m]) * D) * W, 0xEE, (size_t) D * W);
        memset(HP + (((size_t) q * mh + slot[m]) * E) * W, 0xEE, (size_t) E * W);
      }
    }
    memset(GD, 0xA5, hd);
    memset(GP, 0x5A, hp);
    if (gpu && (to_slab(dHD, HD, hd) || to_slab(dHP, HP, hp) || fill_slab(dGD, 0xA5, hd) || fill_slab(dGP, 0x5A, hp)))
      ok = 0;
    if (ok && redset_hip_sharded_execute(reb, stream) != 0) {
      fprintf(stderr, "rank %d: rebuild: %s\n", me, redset_hip_last_error());
      ok = 0;
    }
    if (gpu && (hipStreamSynchronize(stream) || from_slab(HD, dHD, hd) || from_slab(HP, dHP, hp)))
      ok = 0;
    int rbad = 0;
    for (int m = 0; ok && m < nm; ++m) {
      if (host[m] != me) continue;
      for (int q = 0; q < NS; ++q)
        for (size_t b = 0; b < W && q * W + b < C; ++b) {
          for (int s = 0; s < D; ++s)
            rbad += HD[(((size_t) q * mh + slot[m]) * D + s) * W + b] != want_l[m][s * C + q * W + b];
          for (int i = 0; i < E; ++i)
            rbad += HP[(((size_t) q * mh + slot[m]) * E + i) * W + b] != want_p[m][i * C + q * W + b];
        }
    }
    if (rbad) fprintf(stderr, "rank %d: %d bytes differ after the rebuild\n", me, rbad);
    bad += rbad;
    const char* reps_env = getenv("SHARDED_TEST_REPS");
    const int reps = gpu && reps_env ? atoi(reps_env) : 0;
    for (int mode = 0; ok && !rbad && reps > 0 && mode < 2; ++mode) {
      /* repeated rebuilds rewrite the same bytes; mode 0 pipelined, 1 phased */
      MPI_Barrier(MPI_COMM_WORLD);
      double t0 = MPI_Wtime();
      for (int i = 0; ok && i < reps; ++i) {
        if (mode == 0) ok = redset_hip_sharded_execute(reb, stream) == 0;
        for (int ph = REDSET_HIP_PHASE_GATHER; ok && mode == 1 && ph <= REDSET_HIP_PHASE_ACCUMULATE; ++ph)
          ok = redset_hip_sharded_execute_phase(reb, ph, stream) == 0;
      }
      ok = ok && hipStreamSynchronize(stream) == hipSuccess;
      double dt = (MPI_Wtime() - t0) * 1e3 / reps, dmax = 0;
      MPI_Allreduce(&dt, &dmax, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
      if (me == 0) printf("timing: %s rebuild %.3f ms\n", mode == 0 ? "pipelined" : "phased", dmax);
    }
    redset_hip_sharded_info info;
    if (ok && redset_hip_sharded_get_info(reb, &info) == 0)
      printf("rank %d: rebuild gather %llu B sent in %d messages (%llu..%llu B), return %llu B sent in %d messages, "
             "local %llu B\n",
             me, info.gather_bytes_sent, info.gather_messages, info.gather_msg_min, info.gather_msg_max,
             info.return_bytes_sent, info.return_messages, info.local_bytes);
  }
  int mine = ok && !bad, all = 0;
  MPI_Allreduce(&mine, &all, 1, MPI_INT, MPI_LAND, MPI_COMM_WORLD);
  redset_hip_sharded_destroy(enc);
  redset_hip_sharded_destroy(reb);
  redset_hip_mpi_transport_destroy(th);
  redset_hip_rccl_transport_destroy(rh);
  redset_hip_rs_destroy(rs);
  if (host_slabs) {
    (void) hipHostFree(dHD);
    (void) hipHostFree(dHP);
    (void) hipHostFree(dGD);
    (void) hipHostFree(dGP);
    (void) hipStreamDestroy(stream);
  } else if (gpu) {
    (void) hipFree(dHD);
    (void) hipFree(dHP);
    (void) hipFree(dGD);
    (void) hipFree(dGP);
    (void) hipStreamDestroy(stream);
  }
  ro_rs_delete(ORACLE);
  for (int m = 0; m < nm; ++m) {
    free(want_l[m]);
    free(want_p[m]);
  }
  free(want_l);
  free(want_p);
  free(HD);
  free(HP);
  free(GD);
  free(GP);
  free(host);
  free(slot);
  free(on);
  free(count);
  MPI_Finalize();
  return all ? 0 : 1;
}
