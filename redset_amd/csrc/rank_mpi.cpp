// rank_mpi.cpp -- per-rank MPI backends (include/redset_hip_mpi.h): the
// reference's backend-slot functions with the arithmetic on the GPU.
//
// Each function keeps the reference's slice loop and exchange pattern and
// replaces the per-step host multadds with one gf_mac / xor launch per slice
// over all inputs that slice gathered. Host buffers are page-locked so the
// H2D / D2H copies run at PCIe rate; MPI sees host memory (no GPU-aware MPI
// needed).
#include "redset_hip_mpi.h"

#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <vector>

#include "gf256.h"
#include "stripe_map.h"

using redset_hip::CellRef;
using redset_hip::fail;
using redset_hip::StripeMap;

namespace {

constexpr size_t kDefaultBuf = 1u << 20;  // redset_mpi_buf_size default, src/redset.c:45

// page-locked host + device scratch, released on scope exit
struct Scratch {
  std::vector<void*> host, dev;
  hipStream_t stream = nullptr;
  int rc = 0;
  Scratch() {
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) rc = fail("hipStreamCreate failed");
  }
  ~Scratch() {
    if (stream) (void) hipStreamSynchronize(stream);
    for (void* p : host) (void) hipHostFree(p);
    for (void* p : dev) (void) hipFree(p);
    if (stream) (void) hipStreamDestroy(stream);
  }
  uint8_t* h(size_t n) {
    void* p = nullptr;
    if (rc == 0 && hipHostMalloc(&p, n ? n : 1, hipHostMallocDefault) != hipSuccess) rc = fail("hipHostMalloc(%zu) failed", n);
    if (p) host.push_back(p);
    return static_cast<uint8_t*>(p);
  }
  uint8_t* d(size_t n) {
    void* p = nullptr;
    if (rc == 0 && hipMalloc(&p, n ? n : 1) != hipSuccess) rc = fail("hipMalloc(%zu) failed", n);
    if (p) dev.push_back(p);
    return static_cast<uint8_t*>(p);
  }
  int sync() { return hipStreamSynchronize(stream) == hipSuccess ? 0 : fail("hipStreamSynchronize failed"); }
  int h2d(void* dst, const void* src, size_t n) {
    return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, stream) == hipSuccess ? 0 : fail("H2D failed");
  }
  int d2h(void* dst, const void* src, size_t n) {
    return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, stream) == hipSuccess ? 0 : fail("D2H failed");
  }
};

// full pread / pwrite (redset_read_attempt / redset_write_attempt,
// src/redset_io.c:234-310)
int pread_full(int fd, void* buf, size_t n, off_t off) {
  char* p = static_cast<char*>(buf);
  while (n) {
    ssize_t k = ::pread(fd, p, n, off);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    p += k;
    n -= static_cast<size_t>(k);
    off += k;
  }
  return 0;
}

int pwrite_full(int fd, const void* buf, size_t n, off_t off) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t k = ::pwrite(fd, p, n, off);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    p += k;
    n -= static_cast<size_t>(k);
    off += k;
  }
  return 0;
}

int comm_geometry(MPI_Comm comm, int& ranks, int& rank) {
  if (MPI_Comm_size(comm, &ranks) != MPI_SUCCESS || MPI_Comm_rank(comm, &rank) != MPI_SUCCESS)
    return fail("MPI_Comm_size/rank failed");
  return 0;
}

// a map whose inputs/outputs are positions in scratch arrays (cells are
// addressed by the caller); coef is nout x nin
StripeMap scratch_map(int nin, int nout, const std::vector<uint8_t>& coef, bool xor_only) {
  StripeMap m;
  for (int i = 0; i < nin; ++i) m.in.push_back(CellRef{i, redset_hip::kData, 0});
  for (int j = 0; j < nout; ++j) m.out.push_back(CellRef{j, redset_hip::kData, 0});
  m.coef = coef;
  m.xor_only = xor_only;
  return m;
}

}  // namespace

extern "C" {

int redset_hip_rs_encode_rank(const redset_hip_rs* rs, MPI_Comm comm, const redset_hip_io* lofi,
                              const char* chunk_file, int fd_chunk, size_t chunk_size, size_t buf_size) {
  (void) chunk_file;
  if (!rs || !lofi || !lofi->read) return fail("rs_encode_rank: null argument");
  int p, r;
  if (int rc = comm_geometry(comm, p, r)) return rc;
  if (p != rs->ranks) return fail("communicator has %d ranks, codec %d", p, rs->ranks);
  const int e = rs->encoding, d = p - e;
  const size_t B = buf_size ? buf_size : kDefaultBuf;
  const off_t header = ::lseek(fd_chunk, 0, SEEK_CUR);  // src/redset_reedsolomon.c:295
  if (header < 0) return fail("lseek(%s) failed", chunk_file ? chunk_file : "chunk file");

  Scratch S;
  uint8_t* h_send = S.h(B);
  uint8_t* h_recv = S.h(static_cast<size_t>(d) * e * B);  // [step s][slot i]
  uint8_t* h_par = S.h(static_cast<size_t>(e) * B);
  uint8_t* d_recv = S.d(static_cast<size_t>(d) * e * B);
  uint8_t* d_par = S.d(static_cast<size_t>(e) * B);
  if (S.rc) return S.rc;

  // slot i's coefficients over the d slices received for it, in ring-step
  // order: at step s (chunk_step p-1-s) slot i receives from r + (p - chunk_step + i)
  std::vector<StripeMap> maps(e);
  for (int i = 0; i < e; ++i) {
    std::vector<uint8_t> coef(d);
    for (int s = 0; s < d; ++s) {
      const int step = p - 1 - s;
      const int sender = (r + (p - step + i)) % p;
      coef[s] = rs->mat[static_cast<size_t>(p + i) * p + sender];
    }
    maps[i] = scratch_map(d, 1, coef, false);
  }
  std::vector<MPI_Request> req(2 * e);
  std::vector<const uint8_t*> ins(d);
  int rc = 0;
  for (size_t nread = 0; nread < chunk_size; nread += B) {
    const size_t count = std::min(B, chunk_size - nread);
    for (int s = 0; s < d; ++s) {  // chunk_step = p-1 .. e, src/redset_reedsolomon.c:329-377
      const int step = p - 1 - s;
      const int chunk_id = (r + step) % p;
      const int seg = redset_hip::data_id(p, e, r, chunk_id);
      if (lofi->read(lofi->ctx, 0, REDSET_HIP_CELL_DATA, seg, nread, count, h_send) != 0) rc = fail("lofi read failed");
      int k = 0;
      for (int i = 0; i < e; ++i) {
        const int dist = p - step + i;
        MPI_Irecv(h_recv + (static_cast<size_t>(s) * e + i) * B, static_cast<int>(count), MPI_BYTE, (r + dist) % p, 0,
                  comm, &req[k++]);
        MPI_Isend(h_send, static_cast<int>(count), MPI_BYTE, (r - dist + p) % p, 0, comm, &req[k++]);
      }
      MPI_Waitall(k, req.data(), MPI_STATUSES_IGNORE);
    }
    // all d*e slices of this slice window: one H2D, one kernel per slot, one D2H
    int grc = S.h2d(d_recv, h_recv, static_cast<size_t>(d) * e * B);
    for (int i = 0; i < e && grc == 0; ++i) {
      for (int s = 0; s < d; ++s) ins[s] = d_recv + (static_cast<size_t>(s) * e + i) * B;
      uint8_t* out = d_par + static_cast<size_t>(i) * B;
      grc = redset_hip::run_stripe(maps[i], ins.data(), &out, count, S.stream, 0);
    }
    if (grc == 0) grc = S.d2h(h_par, d_par, static_cast<size_t>(e) * B);
    if (grc == 0) grc = S.sync();
    if (grc) return grc;  // a device failure is not recoverable mid-collective
    for (int i = 0; i < e; ++i) {  // :379-388
      const off_t off = header + static_cast<off_t>(i) * static_cast<off_t>(chunk_size) + static_cast<off_t>(nread);
      if (pwrite_full(fd_chunk, h_par + static_cast<size_t>(i) * B, count, off) != 0) rc = fail("write %s failed", chunk_file);
    }
  }
  return rc;
}

int redset_hip_rs_decode_rank(const redset_hip_rs* rs, MPI_Comm comm, int missing, const int* rebuild_ranks,
                              int need_rebuild, const redset_hip_io* lofi, const char* chunk_file, int fd_chunk,
                              size_t chunk_size, size_t buf_size) {
  if (!rs || !lofi || !rebuild_ranks) return fail("rs_decode_rank: null argument");
  int p, r;
  if (int rc = comm_geometry(comm, p, r)) return rc;
  if (p != rs->ranks) return fail("communicator has %d ranks, codec %d", p, rs->ranks);
  const int e = rs->encoding;
  const size_t B = buf_size ? buf_size : kDefaultBuf;
  const off_t header = ::lseek(fd_chunk, 0, SEEK_CUR);  // :588
  if (header < 0) return fail("lseek(%s) failed", chunk_file ? chunk_file : "chunk file");

  // member r solves stripe r (decode_chunk_id = rank, :607-611)
  std::vector<uint8_t> D;
  if (int rc = redset_hip::rs_decode_matrix(rs, missing, rebuild_ranks, r, D)) return rc;
  std::vector<int> cols;
  for (int s = 0; s < p; ++s) {
    bool used = false;
    for (int i = 0; i < missing; ++i) used = used || D[static_cast<size_t>(i) * p + s] != 0;
    if (used) cols.push_back(s);
  }
  std::vector<uint8_t> coef;
  for (int i = 0; i < missing; ++i)
    for (int s : cols) coef.push_back(D[static_cast<size_t>(i) * p + s]);
  const StripeMap map = scratch_map(static_cast<int>(cols.size()), missing, coef, false);

  Scratch S;
  uint8_t* h_send = S.h(B);
  uint8_t* h_cells = S.h(static_cast<size_t>(p) * B);   // member s's cell of stripe r
  uint8_t* h_out = S.h(static_cast<size_t>(missing) * B);
  uint8_t* h_gather = S.h(static_cast<size_t>(p) * B);  // rebuilt cells received from every solver
  uint8_t* d_cells = S.d(static_cast<size_t>(p) * B);
  uint8_t* d_out = S.d(static_cast<size_t>(missing) * B);
  if (S.rc) return S.rc;
  std::vector<const uint8_t*> ins(cols.size());
  std::vector<uint8_t*> outs(missing);
  for (size_t k = 0; k < cols.size(); ++k) ins[k] = d_cells + static_cast<size_t>(cols[k]) * B;
  for (int i = 0; i < missing; ++i) outs[i] = d_out + static_cast<size_t>(i) * B;
  std::vector<MPI_Request> req(2 * p + missing + 2);
  int rc = 0;
  for (size_t nread = 0; nread < chunk_size; nread += B) {
    const size_t count = std::min(B, chunk_size - nread);
    for (int step = 0; step < p; ++step) {  // :646-703
      const int lhs = (r - step + p) % p, rhs = (r + step) % p;
      const int chunk_id = (r + step) % p;
      const int enc = redset_hip::encoding_id(p, e, r, chunk_id);
      if (!need_rebuild) {
        if (enc < p) {
          const int seg = redset_hip::data_id(p, e, r, chunk_id);
          if (lofi->read(lofi->ctx, 0, REDSET_HIP_CELL_DATA, seg, nread, count, h_send) != 0) rc = fail("lofi read failed");
        } else {
          const off_t off = header + static_cast<off_t>(enc - p) * static_cast<off_t>(chunk_size) + static_cast<off_t>(nread);
          if (pread_full(fd_chunk, h_send, count, off) != 0) rc = fail("read %s failed", chunk_file);
        }
      } else {
        std::memset(h_send, 0, count);  // an erased member contributes nothing
      }
      if (step > 0) {
        MPI_Irecv(h_cells + static_cast<size_t>(lhs) * B, static_cast<int>(count), MPI_BYTE, lhs, 0, comm, &req[0]);
        MPI_Isend(h_send, static_cast<int>(count), MPI_BYTE, rhs, 0, comm, &req[1]);
        MPI_Waitall(2, req.data(), MPI_STATUSES_IGNORE);
      } else {
        std::memcpy(h_cells + static_cast<size_t>(r) * B, h_send, count);
      }
    }
    int grc = S.h2d(d_cells, h_cells, static_cast<size_t>(p) * B);
    if (grc == 0 && !cols.empty()) grc = redset_hip::run_stripe(map, ins.data(), outs.data(), count, S.stream, 0);
    if (grc == 0) grc = S.d2h(h_out, d_out, static_cast<size_t>(missing) * B);
    if (grc == 0) grc = S.sync();
    if (grc) return grc;
    // gather rebuilt cells to the erased members, :713-733
    int k = 0;
    if (need_rebuild) {
      for (int step = 0; step < p; ++step) {
        const int lhs = (r - step + p) % p;
        MPI_Irecv(h_gather + static_cast<size_t>(lhs) * B, static_cast<int>(count), MPI_BYTE, lhs, 0, comm, &req[k++]);
      }
    }
    for (int i = 0; i < missing; ++i)
      MPI_Isend(h_out + static_cast<size_t>(i) * B, static_cast<int>(count), MPI_BYTE, rebuild_ranks[i], 0, comm,
                &req[k++]);
    MPI_Waitall(k, req.data(), MPI_STATUSES_IGNORE);
    if (need_rebuild) {  // :736-765
      for (int step = 0; step < p; ++step) {
        const int lhs = (r - step + p) % p;
        const int enc = redset_hip::encoding_id(p, e, r, lhs);
        const uint8_t* cell = h_gather + static_cast<size_t>(lhs) * B;
        if (enc < p) {
          const int seg = redset_hip::data_id(p, e, r, lhs);
          if (!lofi->write || lofi->write(lofi->ctx, 0, REDSET_HIP_CELL_DATA, seg, nread, count, cell) != 0)
            rc = fail("lofi write failed");
        } else {
          const off_t off = header + static_cast<off_t>(enc - p) * static_cast<off_t>(chunk_size) + static_cast<off_t>(nread);
          if (pwrite_full(fd_chunk, cell, count, off) != 0) rc = fail("write %s failed", chunk_file);
        }
      }
    }
  }
  return rc;
}

int redset_hip_xor_encode_rank(MPI_Comm comm, const redset_hip_io* lofi, const char* chunk_file, int fd_chunk,
                               size_t chunk_size, size_t buf_size) {
  if (!lofi || !lofi->read) return fail("xor_encode_rank: null argument");
  int p, r;
  if (int rc = comm_geometry(comm, p, r)) return rc;
  if (p < 2) return fail("XOR needs at least 2 ranks");
  const size_t B = buf_size ? buf_size : kDefaultBuf;
  const off_t header = ::lseek(fd_chunk, 0, SEEK_CUR);
  if (header < 0) return fail("lseek(%s) failed", chunk_file ? chunk_file : "chunk file");
  Scratch S;
  uint8_t* h_send = S.h(static_cast<size_t>(p) * B);  // my cell of stripe t, for t != r
  uint8_t* h_recv = S.h(static_cast<size_t>(p) * B);  // member t's cell of stripe r
  uint8_t* h_out = S.h(B);
  uint8_t* d_recv = S.d(static_cast<size_t>(p) * B);
  uint8_t* d_out = S.d(B);
  if (S.rc) return S.rc;
  const StripeMap map = scratch_map(p - 1, 1, std::vector<uint8_t>(p - 1, 1), true);
  std::vector<const uint8_t*> ins;
  for (int t = 0; t < p; ++t)
    if (t != r) ins.push_back(d_recv + static_cast<size_t>(t) * B);
  std::vector<MPI_Request> req(2 * p);
  int rc = 0;
  for (size_t nread = 0; nread < chunk_size; nread += B) {
    const size_t count = std::min(B, chunk_size - nread);
    int k = 0;
    // the ring of src/redset_xor.c:251-285 leaves member r with the XOR of
    // every other member's cell of stripe r; exchange those cells directly
    for (int t = 0; t < p; ++t) {
      if (t == r) continue;
      const int seg = redset_hip::xor_segment(r, t);
      if (lofi->read(lofi->ctx, 0, REDSET_HIP_CELL_DATA, seg, nread, count, h_send + static_cast<size_t>(t) * B) != 0)
        rc = fail("lofi read failed");
      MPI_Irecv(h_recv + static_cast<size_t>(t) * B, static_cast<int>(count), MPI_BYTE, t, 0, comm, &req[k++]);
      MPI_Isend(h_send + static_cast<size_t>(t) * B, static_cast<int>(count), MPI_BYTE, t, 0, comm, &req[k++]);
    }
    MPI_Waitall(k, req.data(), MPI_STATUSES_IGNORE);
    int grc = S.h2d(d_recv, h_recv, static_cast<size_t>(p) * B);
    if (grc == 0) grc = redset_hip::run_stripe(map, ins.data(), &d_out, count, S.stream, 0);
    if (grc == 0) grc = S.d2h(h_out, d_out, count);
    if (grc == 0) grc = S.sync();
    if (grc) return grc;
    if (pwrite_full(fd_chunk, h_out, count, header + static_cast<off_t>(nread)) != 0)  // :280-284
      rc = fail("write %s failed", chunk_file);
  }
  return rc;
}

int redset_hip_xor_decode_rank(MPI_Comm comm, int root, const redset_hip_io* lofi, const char* chunk_file,
                               int fd_chunk, size_t chunk_size, size_t buf_size) {
  if (!lofi || !lofi->read) return fail("xor_decode_rank: null argument");
  int p, r;
  if (int rc = comm_geometry(comm, p, r)) return rc;
  if (root < 0 || root >= p) return fail("root %d out of range", root);
  const size_t B = buf_size ? buf_size : kDefaultBuf;
  const off_t header = ::lseek(fd_chunk, 0, SEEK_CUR);
  if (header < 0) return fail("lseek(%s) failed", chunk_file ? chunk_file : "chunk file");
  Scratch S;
  uint8_t* h_cells = S.h(static_cast<size_t>(p) * B);
  uint8_t* h_out = S.h(B);
  uint8_t* d_cells = S.d(static_cast<size_t>(p) * B);
  uint8_t* d_out = S.d(B);
  if (S.rc) return S.rc;
  const StripeMap map = scratch_map(p - 1, 1, std::vector<uint8_t>(p - 1, 1), true);
  std::vector<const uint8_t*> ins;
  for (int t = 0; t < p; ++t)
    if (t != root) ins.push_back(d_cells + static_cast<size_t>(t) * B);
  std::vector<MPI_Request> req(p);
  int rc = 0;
  // stripe by stripe, as the reference's pipelined reduce to the root
  // (src/redset_xor.c:466-524): every survivor sends its cell of stripe c,
  // the root XORs them on the GPU and writes its own cell of stripe c
  for (int c = 0; c < p; ++c) {
    for (size_t nread = 0; nread < chunk_size; nread += B) {
      const size_t count = std::min(B, chunk_size - nread);
      if (r != root) {
        uint8_t* mine = h_cells + static_cast<size_t>(r) * B;
        if (c != r) {
          if (lofi->read(lofi->ctx, 0, REDSET_HIP_CELL_DATA, redset_hip::xor_segment(r, c), nread, count, mine) != 0)
            rc = fail("lofi read failed");
        } else if (pread_full(fd_chunk, mine, count, header + static_cast<off_t>(nread)) != 0) {
          rc = fail("read %s failed", chunk_file);
        }
        MPI_Send(mine, static_cast<int>(count), MPI_BYTE, root, 0, comm);
        continue;
      }
      int k = 0;
      for (int t = 0; t < p; ++t)
        if (t != root)
          MPI_Irecv(h_cells + static_cast<size_t>(t) * B, static_cast<int>(count), MPI_BYTE, t, 0, comm, &req[k++]);
      MPI_Waitall(k, req.data(), MPI_STATUSES_IGNORE);
      int grc = S.h2d(d_cells, h_cells, static_cast<size_t>(p) * B);
      if (grc == 0) grc = redset_hip::run_stripe(map, ins.data(), &d_out, count, S.stream, 0);
      if (grc == 0) grc = S.d2h(h_out, d_out, count);
      if (grc == 0) grc = S.sync();
      if (grc) return grc;
      if (c != root) {
        if (!lofi->write ||
            lofi->write(lofi->ctx, 0, REDSET_HIP_CELL_DATA, redset_hip::xor_segment(root, c), nread, count, h_out) != 0)
          rc = fail("lofi write failed");
      } else if (pwrite_full(fd_chunk, h_out, count, header + static_cast<off_t>(nread)) != 0) {
        rc = fail("write %s failed", chunk_file);
      }
    }
  }
  return rc;
}

}  // extern "C"
