// stream_pipeline.cpp -- host-resident encode / rebuild through pinned
// staging buffers and HBM (include/redset_hip.h, "streaming pipeline").
//
// The reference runs its codec slice by slice: read a 1 MiB slice of each
// input (redset_lofi_pread), combine, write the parity slice after the
// header (src/redset_reedsolomon.c:309-391, src/redset_reedsolomon_serial.c:
// 226-325). Here a (stripe, slice) *unit* flows through four overlapped
// stages on NSLOT rotating slots:
//   read    I/O threads fill the slot's pinned input buffer (io->read)
//   H2D     hipMemcpyAsync on the copy-in stream
//   compute gf_mac / xor kernel on the compute stream (run_stripe)
//   D2H     hipMemcpyAsync on the copy-out stream, then I/O threads drain
//           the pinned output buffer (io->write)
// so PCIe in, PCIe out, the kernel and host I/O of different units run at
// the same time. A slot returns to the reader only after its writes finish.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "codec_kernels.h"
#include "redset_hip.h"
#include "stripe_map.h"

using redset_hip::CellRef;
using redset_hip::fail;
using redset_hip::StripeMap;

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Streams and staging buffers kept across calls. Creating and destroying a
// stream costs ~2.7 ms and pinning ~0.15 ms per MiB each way
// (profiles/r02_alloc_probe.jsonl): for a small set that was a third of the
// call. A successful call hands its three streams and (within the limits)
// its slot buffers back; REDSET_HIP_SCRATCH_CACHE=0 allocates and frees per
// call; redset_hip_release_scratch() empties the cache.
class ResourceCache {
 public:
  static ResourceCache& get() {
    static ResourceCache c;
    return c;
  }
  static bool enabled() {
    const char* v = std::getenv("REDSET_HIP_SCRATCH_CACHE");
    return !v || std::atoi(v) != 0;
  }
  // Everything cached belongs to the device that was current when it was
  // made, and is handed out again only while that device is current.
  static int device() {
    int d = -1;
    return hipGetDevice(&d) == hipSuccess ? d : -1;
  }
  hipStream_t take_stream() {
    if (enabled()) {
      const int dev = device();
      std::lock_guard<std::mutex> g(mu_);
      for (size_t i = 0; i < streams_.size(); ++i)
        if (streams_[i].device == dev) {
          hipStream_t s = streams_[i].s;
          streams_.erase(streams_.begin() + static_cast<long>(i));
          return s;
        }
    }
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    return s;
  }
  void give_stream(hipStream_t s, bool ok) {
    if (!s) return;
    if (ok && enabled()) {
      const int dev = device();
      std::lock_guard<std::mutex> g(mu_);
      if (streams_.size() < 6) {
        streams_.push_back(CachedStream{s, dev});
        return;
      }
    }
    (void) hipStreamDestroy(s);
  }
  // the smallest cached buffer of the kind holding n bytes, or a new one;
  // *have = its size
  void* take_buf(size_t n, bool dev, size_t* have) {
    if (n == 0) n = 1;
    if (enabled()) {
      const int cur = device();
      std::lock_guard<std::mutex> g(mu_);
      int best = -1;
      for (int i = 0; i < static_cast<int>(bufs_.size()); ++i)
        if (bufs_[i].dev == dev && bufs_[i].device == cur && bufs_[i].n >= n && (best < 0 || bufs_[i].n < bufs_[best].n))
          best = i;
      if (best >= 0) {
        Buf b = bufs_[best];
        bufs_.erase(bufs_.begin() + best);
        bytes_[dev] -= b.n;
        *have = b.n;
        return b.p;
      }
    }
    void* p = nullptr;
    if ((dev ? hipMalloc(&p, n) : hipHostMalloc(&p, n, hipHostMallocDefault)) != hipSuccess) return nullptr;
    *have = n;
    return p;
  }
  void give_buf(void* p, size_t n, bool dev, bool ok) {
    if (!p) return;
    if (ok && enabled()) {
      const int cur = device();
      std::lock_guard<std::mutex> g(mu_);
      const size_t limit = dev ? (size_t(1) << 30) : (size_t(256) << 20);
      if (bufs_.size() < 32 && bytes_[dev] + n <= limit) {
        bufs_.push_back(Buf{p, n, dev, cur});
        bytes_[dev] += n;
        return;
      }
    }
    free_buf(p, dev);
  }
  void release() {
    std::lock_guard<std::mutex> g(mu_);
    for (const Buf& b : bufs_) free_buf(b.p, b.dev);
    bufs_.clear();
    bytes_[0] = bytes_[1] = 0;
    for (const CachedStream& c : streams_) (void) hipStreamDestroy(c.s);
    streams_.clear();
  }

 private:
  struct Buf {
    void* p;
    size_t n;
    bool dev;    // device memory (else pinned host)
    int device;  // current device when it was allocated
  };
  struct CachedStream {
    hipStream_t s;
    int device;
  };
  static void free_buf(void* p, bool dev) {
    if (dev) (void) hipFree(p);
    else (void) hipHostFree(p);
  }
  std::mutex mu_;
  std::vector<Buf> bufs_;
  size_t bytes_[2] = {0, 0};
  std::vector<CachedStream> streams_;
};

// Fixed pool of I/O workers; run() executes a batch and waits for it.
class IoPool {
 public:
  explicit IoPool(int n) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~IoPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  // run every task, return when all are done. The completion count lives
  // under `dmu`: a worker decrements and notifies while holding it, so the
  // caller cannot see zero, return and destroy dmu/dcv before the last
  // worker has finished touching them.
  void run(std::vector<std::function<void()>>& tasks) {
    int left = static_cast<int>(tasks.size());
    std::mutex dmu;
    std::condition_variable dcv;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& t : tasks) {
        q_.push([&t, &left, &dmu, &dcv] {
          t();
          std::lock_guard<std::mutex> g2(dmu);
          if (--left == 0) dcv.notify_all();
        });
      }
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lk(dmu);
    dcv.wait(lk, [&] { return left == 0; });
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return quit_ || !q_.empty(); });
        if (quit_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop();
      }
      f();
    }
  }
  std::vector<std::thread> workers_;
  std::queue<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool quit_ = false;
};

struct Unit {
  int map;      // index into maps
  size_t off;   // byte offset within each cell
  size_t len;
};

enum SlotState { kFree, kRead, kOnGpu };

struct Slot {
  uint8_t* h_in = nullptr;
  uint8_t* h_out = nullptr;
  uint8_t* d_in = nullptr;
  uint8_t* d_out = nullptr;
  size_t n_h_in = 0, n_h_out = 0, n_d_in = 0, n_d_out = 0;  // sizes as allocated (cached ones may be larger)
  hipEvent_t ev_in = nullptr, ev_comp = nullptr, ev_done = nullptr, ev_start = nullptr;
  SlotState state = kFree;
  size_t unit = 0;
  std::vector<void*> src, dst;  // mapped (page-locked) host cells, or null
};

constexpr int kSlots = 4;

int hip_ok(hipError_t e, const char* what) { return e == hipSuccess ? 0 : fail("%s: %s", what, hipGetErrorString(e)); }

// The kernels' hang word (include/redset_hip.h redset_hip_hang_faults), read
// in order on `s`: at the start of a call, and after its last sync, where a
// count that moved fails the call -- a wait with no fallback gave up, so
// some launch's outputs are wrong and the call must not report success.
int hang_mark(hipStream_t s, unsigned* v) {
  return hip_ok(static_cast<hipError_t>(redset_hip::read_hang_faults(s, v, 0)), "hang-fault read");
}
int hang_check(hipStream_t s, unsigned before) {
  unsigned now = before;
  if (int rc = hang_mark(s, &now)) return rc;
  return now == before ? 0 : fail("a kernel wait hit its hang cap (%u since the call began): outputs not trusted", now - before);
}

// Zero copy: when every cell of every stripe is page-locked host memory
// (io->map gives its address, contiguous over the whole cell), the gf_mac /
// xor kernel reads its inputs and writes its outputs over PCIe directly --
// no staging buffers, no SDMA copies, one launch per stripe. Measured on
// MI355X (tools/zerocopy_probe.py): a kernel's host reads run at the SDMA
// H2D rate (55-56 GB/s) while its host writes use the other direction at the
// same time, 75.5 GB/s of PCIe bytes for an 8-in / 3-out stripe against the
// staged pipeline's ~60. Test builds (REDSET_HIP_TEST_KNOBS):
// REDSET_HIP_ZERO_COPY=0 forces the staged pipeline over mapped cells.
// Returns 1 (not applicable) without side effects when a cell is not mapped.
int try_zero_copy(const std::vector<StripeMap>& maps, size_t chunk, const redset_hip_io* io,
                  redset_hip_stream_stats* st, int* rc_out) {
#if REDSET_HIP_TEST_KNOBS
  const char* env = std::getenv("REDSET_HIP_ZERO_COPY");
  if (env && env[0] == '0') return 1;
#endif
  if (!io->map || chunk == 0) return 1;
  std::vector<std::vector<const uint8_t*>> ins(maps.size());
  std::vector<std::vector<uint8_t*>> outs(maps.size());
  auto dev = [&](const CellRef& c) -> void* {
    void* h0 = io->map(io->ctx, c.rank, c.kind, c.index, 0);
    void* h1 = io->map(io->ctx, c.rank, c.kind, c.index, chunk - 1);
    if (!h0 || static_cast<char*>(h1) != static_cast<char*>(h0) + (chunk - 1)) return nullptr;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h0, 0) != hipSuccess) {
      (void) hipGetLastError();
      return nullptr;
    }
    return d;
  };
  for (size_t k = 0; k < maps.size(); ++k) {
    for (const CellRef& c : maps[k].in) {
      void* d = dev(c);
      if (!d) return 1;
      ins[k].push_back(static_cast<const uint8_t*>(d));
    }
    for (const CellRef& c : maps[k].out) {
      void* d = dev(c);
      if (!d) return 1;
      outs[k].push_back(static_cast<uint8_t*>(d));
    }
  }
  const double t0 = now_s();
  ResourceCache& cache = ResourceCache::get();
  hipStream_t s = cache.take_stream();
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = s ? 0 : fail("hipStreamCreate failed");
  unsigned hang0 = 0;
  rc = rc ? rc : hang_mark(s, &hang0);
  rc = rc ? rc : hip_ok(hipEventCreate(&e0), "event");
  rc = rc ? rc : hip_ok(hipEventCreate(&e1), "event");
  rc = rc ? rc : hip_ok(hipEventRecord(e0, s), "event record");
  for (size_t k = 0; k < maps.size() && rc == 0; ++k) {
    if (maps[k].out.empty()) continue;
    rc = redset_hip::run_stripe(maps[k], ins[k].data(), outs[k].data(), chunk, s, 0);
    st->bytes_read += maps[k].in.size() * chunk;
    st->bytes_written += maps[k].out.size() * chunk;
    st->units += 1;
  }
  rc = rc ? rc : hip_ok(hipEventRecord(e1, s), "event record");
  rc = rc ? rc : hip_ok(hipStreamSynchronize(s), "stream synchronize");
  rc = rc ? rc : hang_check(s, hang0);
  float ms = 0;
  if (rc == 0 && hipEventElapsedTime(&ms, e0, e1) == hipSuccess) st->gpu_seconds = ms * 1e-3;
  const bool synced = s && hipStreamSynchronize(s) == hipSuccess;
  if (e0) (void) hipEventDestroy(e0);
  if (e1) (void) hipEventDestroy(e1);
  cache.give_stream(s, rc == 0 && synced);
  st->seconds = now_s() - t0;
  *rc_out = rc;
  return 0;
}

int run_pipeline(const std::vector<StripeMap>& maps, size_t chunk, size_t slice, int io_threads,
                 const redset_hip_io* io, redset_hip_stream_stats* stats) {
  if (!io || !io->read || !io->write) return fail("null redset_hip_io");
  {
    redset_hip_stream_stats zst;
    std::memset(&zst, 0, sizeof(zst));
    int zrc = 0;
    if (try_zero_copy(maps, chunk, io, &zst, &zrc) == 0) {
      if (stats) *stats = zst;
      return zrc;
    }
  }
  // default slice: 8 MiB; a chunk that would fit one slice is cut into ~16
  // slices of >= 256 KiB instead, so small sets pipeline and pin less
  // (configs[0]'s 5.6 MB chunks: apply 58 -> 29 ms, profiles/r01_config1_headers_e2e.jsonl)
  if (slice == 0) slice = chunk > (8u << 20) ? (8u << 20) : std::max<size_t>(256u << 10, chunk / 16);
  slice = std::min(slice, std::max<size_t>(chunk, 1));
  slice = (slice + 255) & ~static_cast<size_t>(255);
  if (io_threads <= 0) io_threads = 8;
  const double t0 = now_s();
  size_t max_in = 0, max_out = 0;
  for (const StripeMap& m : maps) {
    max_in = std::max(max_in, m.in.size());
    max_out = std::max(max_out, m.out.size());
  }
  std::vector<Unit> units;
  for (size_t k = 0; k < maps.size(); ++k)
    for (size_t off = 0; off < chunk; off += slice) units.push_back(Unit{static_cast<int>(k), off, std::min(slice, chunk - off)});
  redset_hip_stream_stats st;
  std::memset(&st, 0, sizeof(st));
  if (units.empty() || max_out == 0) {
    if (stats) *stats = st;
    return REDSET_SUCCESS;
  }

  Slot slots[kSlots];
  ResourceCache& cache = ResourceCache::get();
  hipStream_t s_in = cache.take_stream(), s_comp = cache.take_stream(), s_out = cache.take_stream();
  int rc = (s_in && s_comp && s_out) ? 0 : fail("hipStreamCreate failed");
  unsigned hang0 = 0;
  rc = rc ? rc : hang_mark(s_comp, &hang0);
  auto buf = [&](uint8_t** p, size_t* have, size_t n, bool dev) {
    if (rc) return;
    *p = static_cast<uint8_t*>(cache.take_buf(n, dev, have));
    if (!*p) rc = fail("%s(%zu) failed", dev ? "hipMalloc" : "hipHostMalloc", n);
  };
  for (Slot& S : slots) {
    buf(&S.h_in, &S.n_h_in, max_in * slice, false);
    buf(&S.h_out, &S.n_h_out, max_out * slice, false);
    buf(&S.d_in, &S.n_d_in, max_in * slice, true);
    buf(&S.d_out, &S.n_d_out, max_out * slice, true);
    rc = rc ? rc : hip_ok(hipEventCreateWithFlags(&S.ev_in, hipEventDisableTiming), "event");
    rc = rc ? rc : hip_ok(hipEventCreateWithFlags(&S.ev_comp, hipEventDisableTiming), "event");
    rc = rc ? rc : hip_ok(hipEventCreate(&S.ev_start), "event");
    rc = rc ? rc : hip_ok(hipEventCreate(&S.ev_done), "event");
  }

  std::mutex mu;
  std::condition_variable cv;
  std::atomic<int> io_err(0);
  std::atomic<long long> read_ns(0), write_ns(0);
  double gpu_s = 0;
  const size_t nunits = units.size();

  if (rc == 0) {
    IoPool rpool(io_threads), wpool(std::max(1, io_threads / 2));

    std::atomic<bool> abort(false);
    // false if the pipeline was aborted while waiting
    auto wait_state = [&](Slot& S, SlotState want) {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return S.state == want || abort.load(); });
      return !abort.load();
    };
    // wake every stage and make it return (a HIP failure anywhere)
    auto stop = [&] {
      {
        std::lock_guard<std::mutex> g(mu);
        abort = true;
      }
      cv.notify_all();
    };
    auto set_state = [&](Slot& S, SlotState s) {
      {
        std::lock_guard<std::mutex> g(mu);
        S.state = s;
      }
      cv.notify_all();
    };

    // reader: fills slots ahead of the GPU
    std::thread reader([&] {
      for (size_t u = 0; u < nunits; ++u) {
        Slot& S = slots[u % kSlots];
        if (!wait_state(S, kFree)) return;
        const Unit& U = units[u];
        const StripeMap& m = maps[U.map];
        S.src.assign(m.in.size(), nullptr);
        S.dst.assign(m.out.size(), nullptr);
        if (io->map) {
          for (size_t i = 0; i < m.in.size(); ++i)
            S.src[i] = io->map(io->ctx, m.in[i].rank, m.in[i].kind, m.in[i].index, U.off);
          for (size_t j = 0; j < m.out.size(); ++j)
            S.dst[j] = io->map(io->ctx, m.out[j].rank, m.out[j].kind, m.out[j].index, U.off);
        }
        std::vector<std::function<void()>> tasks;
        for (size_t i = 0; i < m.in.size(); ++i) {
          if (S.src[i]) continue;  // DMAed straight from mapped host memory
          tasks.push_back([&, i, U] {
            const CellRef& c = maps[U.map].in[i];
            const double a = now_s();
            if (io->read(io->ctx, c.rank, c.kind, c.index, U.off, U.len, S.h_in + i * slice) != 0) io_err = 1;
            read_ns += static_cast<long long>((now_s() - a) * 1e9);
          });
        }
        rpool.run(tasks);
        S.unit = u;
        set_state(S, kRead);
      }
    });

    // writer: drains slots after D2H
    std::thread writer([&] {
      for (size_t u = 0; u < nunits; ++u) {
        Slot& S = slots[u % kSlots];
        if (!wait_state(S, kOnGpu)) return;
        if (hipEventSynchronize(S.ev_done) != hipSuccess) {
          io_err = 2;
          stop();
          return;
        }
        // the pipeline failed after this unit was published: do not write
        // bytes that may belong to no finished computation
        if (abort.load()) return;
        float ms = 0;
        if (hipEventElapsedTime(&ms, S.ev_start, S.ev_done) == hipSuccess) gpu_s += ms * 1e-3;
        const Unit& U = units[u];
        const StripeMap& m = maps[U.map];
        std::vector<std::function<void()>> tasks;
        for (size_t j = 0; j < m.out.size(); ++j) {
          if (S.dst[j]) continue;  // D2H went straight to mapped host memory
          tasks.push_back([&, j, U] {
            const CellRef& c = maps[U.map].out[j];
            const double a = now_s();
            if (io->write(io->ctx, c.rank, c.kind, c.index, U.off, U.len, S.h_out + j * slice) != 0) io_err = 1;
            write_ns += static_cast<long long>((now_s() - a) * 1e9);
          });
        }
        wpool.run(tasks);
        set_state(S, kFree);
      }
    });

    // GPU feeder (this thread)
    std::vector<const uint8_t*> ins;
    std::vector<uint8_t*> outs;
    for (size_t u = 0; u < nunits && rc == 0; ++u) {
      Slot& S = slots[u % kSlots];
      if (!wait_state(S, kRead)) break;
      const Unit& U = units[u];
      const StripeMap& m = maps[U.map];
      const size_t nin = m.in.size(), nout = m.out.size();
      rc = rc ? rc : hip_ok(hipEventRecord(S.ev_start, s_in), "event record");
      for (size_t i = 0; i < nin && rc == 0; ++i) {
        const void* from = S.src[i] ? S.src[i] : S.h_in + i * slice;
        rc = hip_ok(hipMemcpyAsync(S.d_in + i * slice, from, U.len, hipMemcpyHostToDevice, s_in), "H2D");
      }
      rc = rc ? rc : hip_ok(hipEventRecord(S.ev_in, s_in), "event record");
      rc = rc ? rc : hip_ok(hipStreamWaitEvent(s_comp, S.ev_in, 0), "stream wait");
      ins.resize(nin);
      outs.resize(nout);
      for (size_t i = 0; i < nin; ++i) ins[i] = S.d_in + i * slice;
      for (size_t j = 0; j < nout; ++j) outs[j] = S.d_out + j * slice;
      if (rc == 0) rc = redset_hip::run_stripe(m, ins.data(), outs.data(), U.len, s_comp, 0);
      rc = rc ? rc : hip_ok(hipEventRecord(S.ev_comp, s_comp), "event record");
      rc = rc ? rc : hip_ok(hipStreamWaitEvent(s_out, S.ev_comp, 0), "stream wait");
      for (size_t j = 0; j < nout && rc == 0; ++j) {
        void* to = S.dst[j] ? S.dst[j] : S.h_out + j * slice;
        rc = hip_ok(hipMemcpyAsync(to, S.d_out + j * slice, U.len, hipMemcpyDeviceToHost, s_out), "D2H");
      }
      rc = rc ? rc : hip_ok(hipEventRecord(S.ev_done, s_out), "event record");
      // a failed unit is never handed to the writer (its ev_done may not be
      // recorded and h_out would hold another unit's bytes): abort below
      if (rc != 0) break;
      st.bytes_read += nin * U.len;
      st.bytes_written += nout * U.len;
      st.units += 1;
      set_state(S, kOnGpu);
    }
    if (rc != 0) stop();  // a HIP failure: stop the reader and writer wherever they wait
    reader.join();
    writer.join();
  }
  bool ok = rc == 0 && io_err.load() != 2;
  for (hipStream_t s : {s_in, s_comp, s_out})
    if (s && hipStreamSynchronize(s) != hipSuccess) ok = false;
  if (ok) rc = hang_check(s_comp, hang0);
  for (Slot& S : slots) {
    cache.give_buf(S.h_in, S.n_h_in, false, ok);
    cache.give_buf(S.h_out, S.n_h_out, false, ok);
    cache.give_buf(S.d_in, S.n_d_in, true, ok);
    cache.give_buf(S.d_out, S.n_d_out, true, ok);
    if (S.ev_in) (void) hipEventDestroy(S.ev_in);
    if (S.ev_comp) (void) hipEventDestroy(S.ev_comp);
    if (S.ev_start) (void) hipEventDestroy(S.ev_start);
    if (S.ev_done) (void) hipEventDestroy(S.ev_done);
  }
  cache.give_stream(s_in, ok);
  cache.give_stream(s_comp, ok);
  cache.give_stream(s_out, ok);
  st.seconds = now_s() - t0;
  st.read_seconds = read_ns.load() * 1e-9;
  st.write_seconds = write_ns.load() * 1e-9;
  st.gpu_seconds = gpu_s;
  if (stats) *stats = st;
  if (rc) return rc;
  if (io_err.load() == 2) return fail("stream pipeline: device-to-host copy failed");
  if (io_err.load()) return fail("stream I/O callback failed");
  return REDSET_SUCCESS;
}

int stripe_range(int ranks, int first, int n, int& lo, int& hi) {
  if (n <= 0) {
    first = 0;
    n = ranks;
  }
  if (first < 0 || first + n > ranks) return fail("stripe range [%d, %d) outside 0..%d", first, first + n, ranks);
  lo = first;
  hi = first + n;
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// built-in I/O: host memory
// ---------------------------------------------------------------------------

struct redset_hip_hostio {
  std::vector<unsigned char*> lofi, parity;
  size_t stride;
};

namespace {
void* hostio_map(void* ctx, int rank, int kind, int index, unsigned long long off) {
  auto* h = static_cast<redset_hip_hostio*>(ctx);
  unsigned char* base = kind == REDSET_HIP_CELL_DATA ? h->lofi[rank] : h->parity[rank];
  return base + static_cast<size_t>(index) * h->stride + off;
}
}  // namespace

namespace {
int hostio_read(void* ctx, int rank, int kind, int index, unsigned long long off, size_t len, void* dst) {
  auto* h = static_cast<redset_hip_hostio*>(ctx);
  const unsigned char* base = kind == REDSET_HIP_CELL_DATA ? h->lofi[rank] : h->parity[rank];
  std::memcpy(dst, base + static_cast<size_t>(index) * h->stride + off, len);
  return 0;
}
int hostio_write(void* ctx, int rank, int kind, int index, unsigned long long off, size_t len, const void* src) {
  auto* h = static_cast<redset_hip_hostio*>(ctx);
  unsigned char* base = kind == REDSET_HIP_CELL_DATA ? h->lofi[rank] : h->parity[rank];
  std::memcpy(base + static_cast<size_t>(index) * h->stride + off, src, len);
  return 0;
}
}  // namespace

// ---------------------------------------------------------------------------
// built-in I/O: files with redset logical-file semantics
// ---------------------------------------------------------------------------

struct redset_hip_fileio {
  struct File {
    std::string path;
    unsigned long long size;
    int fd;
    bool writable;
  };
  std::vector<std::vector<File>> data;  // member -> its files, in logical order
  std::vector<int> red_fd;
  std::vector<unsigned long long> header;
  size_t chunk;
};

namespace {

// pread/pwrite of a full range, retrying short transfers and EINTR
// (redset_read_attempt / redset_write_attempt, src/redset_io.c:234-310).
// EOF inside the range is a failure, as a short redset_read_attempt is to
// its callers (src/redset_lofi.c:74-77, src/redset_reedsolomon.c:678-681):
// a data or redundancy file shorter than recorded must not read as zeros.
// Zero padding exists only past a member's last file (lofi_rw).
int full_pread(int fd, void* buf, size_t len, off_t off) {
  char* p = static_cast<char*>(buf);
  while (len > 0) {
    ssize_t n = ::pread(fd, p, len, off);
    if (n < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    if (n == 0) return -1;  // EOF before the end of the recorded range
    p += n;
    len -= static_cast<size_t>(n);
    off += n;
  }
  return 0;
}

int full_pwrite(int fd, const void* buf, size_t len, off_t off) {
  const char* p = static_cast<const char*>(buf);
  while (len > 0) {
    ssize_t n = ::pwrite(fd, p, len, off);
    if (n < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    p += n;
    len -= static_cast<size_t>(n);
    off += n;
  }
  return 0;
}

// redset_read_pad_n / redset_write_pad_n (src/redset_lofi.c:30-173): walk the
// member's files over the logical range [pos, pos+len)
int lofi_rw(redset_hip_fileio* f, int rank, unsigned long long pos, size_t len, char* buf, bool write) {
  unsigned long long start = 0;
  for (const auto& F : f->data[rank]) {
    const unsigned long long end = start + F.size;
    if (pos < end && len > 0) {
      const size_t n = static_cast<size_t>(std::min<unsigned long long>(len, end - pos));
      const off_t off = static_cast<off_t>(pos - start);
      const int r = write ? full_pwrite(F.fd, buf, n, off) : full_pread(F.fd, buf, n, off);
      if (r != 0) return -1;
      pos += n;
      buf += n;
      len -= n;
    }
    start = end;
  }
  if (len > 0 && !write) std::memset(buf, 0, len);  // past the last file: zeros
  return 0;
}

int fileio_read(void* ctx, int rank, int kind, int index, unsigned long long off, size_t len, void* dst) {
  auto* f = static_cast<redset_hip_fileio*>(ctx);
  if (kind == REDSET_HIP_CELL_DATA)
    return lofi_rw(f, rank, static_cast<unsigned long long>(index) * f->chunk + off, len, static_cast<char*>(dst), false);
  if (f->red_fd[rank] < 0) return -1;
  return full_pread(f->red_fd[rank], dst, len, static_cast<off_t>(f->header[rank] + index * f->chunk + off));
}

int fileio_write(void* ctx, int rank, int kind, int index, unsigned long long off, size_t len, const void* src) {
  auto* f = static_cast<redset_hip_fileio*>(ctx);
  if (kind == REDSET_HIP_CELL_DATA)
    return lofi_rw(f, rank, static_cast<unsigned long long>(index) * f->chunk + off, len,
                   const_cast<char*>(static_cast<const char*>(src)), true);
  if (f->red_fd[rank] < 0) return -1;
  return full_pwrite(f->red_fd[rank], src, len, static_cast<off_t>(f->header[rank] + index * f->chunk + off));
}

}  // namespace

extern "C" {

void redset_hip_release_scratch(void) { ResourceCache::get().release(); }


int redset_hip_rs_encode_stream(const redset_hip_rs* rs, size_t chunk_size, int first_stripe, int nstripes,
                                size_t slice_bytes, int io_threads, const redset_hip_io* io,
                                redset_hip_stream_stats* stats) {
  if (!rs) return fail("null rs state");
  int lo, hi;
  if (int rc = stripe_range(rs->ranks, first_stripe, nstripes, lo, hi)) return rc;
  std::vector<StripeMap> maps(hi - lo);
  for (int c = lo; c < hi; ++c) redset_hip::rs_encode_map(rs, c, maps[c - lo]);
  return run_pipeline(maps, chunk_size, slice_bytes, io_threads, io, stats);
}

int redset_hip_rs_rebuild_stream(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, size_t chunk_size,
                                 int first_stripe, int nstripes, size_t slice_bytes, int io_threads,
                                 const redset_hip_io* io, redset_hip_stream_stats* stats) {
  if (!rs || !rebuild_ranks) return fail("null argument");
  int lo, hi;
  if (int rc = stripe_range(rs->ranks, first_stripe, nstripes, lo, hi)) return rc;
  std::vector<StripeMap> maps(hi - lo);
  for (int c = lo; c < hi; ++c)
    if (int rc = redset_hip::rs_rebuild_map(rs, missing, rebuild_ranks, c, maps[c - lo])) return rc;
  return run_pipeline(maps, chunk_size, slice_bytes, io_threads, io, stats);
}

int redset_hip_xor_encode_stream(int ranks, size_t chunk_size, int first_stripe, int nstripes, size_t slice_bytes,
                                 int io_threads, const redset_hip_io* io, redset_hip_stream_stats* stats) {
  if (ranks < 2) return fail("XOR needs at least 2 ranks, got %d", ranks);
  int lo, hi;
  if (int rc = stripe_range(ranks, first_stripe, nstripes, lo, hi)) return rc;
  std::vector<StripeMap> maps(hi - lo);
  for (int c = lo; c < hi; ++c) redset_hip::xor_encode_map(ranks, c, maps[c - lo]);
  return run_pipeline(maps, chunk_size, slice_bytes, io_threads, io, stats);
}

int redset_hip_xor_rebuild_stream(int ranks, int root, size_t chunk_size, int first_stripe, int nstripes,
                                  size_t slice_bytes, int io_threads, const redset_hip_io* io,
                                  redset_hip_stream_stats* stats) {
  if (ranks < 2) return fail("XOR needs at least 2 ranks, got %d", ranks);
  int lo, hi;
  if (int rc = stripe_range(ranks, first_stripe, nstripes, lo, hi)) return rc;
  std::vector<StripeMap> maps(hi - lo);
  for (int c = lo; c < hi; ++c)
    if (int rc = redset_hip::xor_rebuild_map(ranks, root, c, maps[c - lo])) return rc;
  return run_pipeline(maps, chunk_size, slice_bytes, io_threads, io, stats);
}

int redset_hip_hostio_create(int ranks, unsigned char* const* lofi, unsigned char* const* parity, size_t cell_stride,
                             int pinned, redset_hip_io* io_out, redset_hip_hostio** out) {
  if (!out || !io_out || !lofi || !parity || ranks < 1) return fail("hostio_create: bad argument");
  auto* h = new (std::nothrow) redset_hip_hostio;
  if (!h) return fail("out of host memory");
  h->lofi.assign(lofi, lofi + ranks);
  h->parity.assign(parity, parity + ranks);
  h->stride = cell_stride;
  io_out->read = hostio_read;
  io_out->write = hostio_write;
  io_out->map = pinned ? hostio_map : nullptr;
  io_out->ctx = h;
  *out = h;
  return REDSET_SUCCESS;
}

void redset_hip_hostio_destroy(redset_hip_hostio* h) { delete h; }

int redset_hip_fileio_create(int ranks, const int* nfiles, const char* const* paths, const unsigned long long* sizes,
                             const char* const* redundancy_paths, const unsigned long long* header_sizes,
                             size_t chunk_size, const int* writable, redset_hip_io* io_out,
                             redset_hip_fileio** out) {
  if (!out || !io_out || !nfiles || !paths || !sizes || ranks < 1) return fail("fileio_create: bad argument");
  auto* f = new (std::nothrow) redset_hip_fileio;
  if (!f) return fail("out of host memory");
  f->chunk = chunk_size;
  f->data.resize(ranks);
  f->red_fd.assign(ranks, -1);
  f->header.assign(ranks, 0);
  size_t k = 0;
  int rc = 0;
  for (int r = 0; r < ranks && rc == 0; ++r) {
    const bool w = writable && writable[r];
    for (int i = 0; i < nfiles[r] && rc == 0; ++i, ++k) {
      int fd = w ? ::open(paths[k], O_RDWR | O_CREAT, 0600) : ::open(paths[k], O_RDONLY);
      if (fd < 0) {
        rc = fail("open(%s): %s", paths[k], strerror(errno));
        break;
      }
      if (w && ::ftruncate(fd, static_cast<off_t>(sizes[k])) != 0) rc = fail("ftruncate(%s): %s", paths[k], strerror(errno));
      f->data[r].push_back(redset_hip_fileio::File{paths[k], sizes[k], fd, w});
    }
    if (rc) break;
    f->header[r] = header_sizes ? header_sizes[r] : 0;
    if (!redundancy_paths || !redundancy_paths[r]) continue;  // data-only I/O (per-rank backends)
    f->red_fd[r] = ::open(redundancy_paths[r], O_RDWR | O_CREAT, 0600);
    if (f->red_fd[r] < 0) rc = fail("open(%s): %s", redundancy_paths[r], strerror(errno));
  }
  if (rc) {
    redset_hip_fileio_destroy(f);
    return rc;
  }
  io_out->read = fileio_read;
  io_out->write = fileio_write;
  io_out->map = nullptr;
  io_out->ctx = f;
  *out = f;
  return REDSET_SUCCESS;
}

void redset_hip_fileio_destroy(redset_hip_fileio* f) {
  if (!f) return;
  // fsync what we may have written before closing, as redset_close does
  // (src/redset_io.c:119-139)
  for (auto& files : f->data)
    for (auto& F : files)
      if (F.fd >= 0) {
        if (F.writable) (void) ::fsync(F.fd);
        ::close(F.fd);
      }
  for (int fd : f->red_fd)
    if (fd >= 0) {
      (void) ::fsync(fd);
      ::close(fd);
    }
  delete f;
}

}  // extern "C"
