// cpk_api.cpp -- the C ABI (include/cpk.h) over the HIP kernels.  Host side only: argument
// checks, scratch management, launch sequencing.  No C++ exception crosses the boundary.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <chrono>
#include <new>
#include <utility>
#include <vector>

#include "../../include/cpk.h"
#include "cpk_kernels.h"

struct cpk_ctx {
  int device = 0;
  void* scratch = nullptr;       // device scratch (descriptors, bitmaps, tile tables)
  size_t scratch_size = 0;
  uint32_t* err = nullptr;       // device error word (first batch-level error)
  // (host entry points, small batches) where a single-launch kernel copies the error word at its
  // end -- a pinned host word, device view -- so that no download is needed; else NULL
  uint32_t* err_host = nullptr;
  bool fused_last = false;  // the last call was one launch that copied its error word there
  // device staging: [0..2] the *_host entry points, [3] cpk_pack_segments (segment list, flat
  // message, chunk offsets), [4] cpk_split_packed_stream (call state, record-head map)
  void* stage[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  size_t stage_size[5] = {0, 0, 0, 0, 0};
  // the stream split's record-head map (in stage[4]) as last laid out: its memory and extent
  // (a reallocation always changes the size: a new allocation at the old address is caught)
  void* split_map = nullptr;
  size_t split_map_size = 0;
  uint64_t split_map_words = 0;
  // measurement hooks: [0] pack (tile, scan, placement), [1] unpack (the tile kernel after the
  // header launch), [2] the unpack tile kernel alone
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[CPK_TIMERS];
  std::vector<hipEvent_t> pool;
  // cpk_pack_segments: pinned host staging for the segment list, free again once `meta_ev`
  // (recorded after its upload) has completed
  void* pinned = nullptr;
  size_t pinned_size = 0;
  hipEvent_t meta_ev = nullptr;
  // calls on different streams share the scratch and the device staging: a call on a stream
  // other than the previous call's waits for everything enqueued on that stream (order_ev)
  hipStream_t last_stream = nullptr;
  bool used = false;
  hipEvent_t order_ev = nullptr;
  // state that is zero at rest (each call that dirties it clears it again on the device): the
  // unpack header launch's scan descriptors (cleared by the tile kernel of the same call)
  uint64_t* hdr_desc = nullptr;
  size_t hdr_desc_n = 0;
  // the pack's chunk-start bitmap and per-tile start bits (set by the framing launch, cleared
  // by the tile kernel that reads them)
  uint64_t* pack_bits = nullptr;
  size_t pack_bits_n = 0;
  // the host entry points' staging for batches up to kHostIoMax bytes: one pinned host buffer
  // and one device buffer, so a call is one upload, the kernels, one download of every result
  // and one synchronisation (per-call latency of small messages)
  void* hio = nullptr;
  uint8_t* hio_dev = nullptr;  // its device view
  size_t hio_size = 0;
  void* dio = nullptr;
  size_t dio_size = 0;
};

namespace cpk {
uint32_t debug_skip() {
  static const uint32_t v = getenv("CPK_DEBUG_SKIP") ? (uint32_t)atoi(getenv("CPK_DEBUG_SKIP")) : 0;
  return v;
}
unsigned long long* debug_stamps(int which) {
  static unsigned long long* bufs[4] = {nullptr, nullptr, nullptr, nullptr};
  static const bool on = getenv("CPK_STAMPS") && atoi(getenv("CPK_STAMPS")) != 0;
  if (!on) return nullptr;
  if (!bufs[which]) {
    const size_t bytes = (size_t)cpk::kStampSlots * cpk::kStampRows * 8;
    if (hipMalloc((void**)&bufs[which], bytes) != hipSuccess) return nullptr;
    if (hipMemset(bufs[which], 0, bytes) != hipSuccess) return nullptr;
  }
  return bufs[which];
}
}  // namespace cpk

namespace {

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

cpk_status hip_status(hipError_t e) { return e == hipSuccess ? CPK_OK : CPK_ERR_HIP; }

cpk_status ensure(void** p, size_t* size, size_t need) {
  if (need <= *size) return CPK_OK;
  if (*p) {
    if (hipFree(*p) != hipSuccess) return CPK_ERR_HIP;
    *p = nullptr;
    *size = 0;
  }
  size_t sz = need + need / 8 + 4096;
  if (hipMalloc(p, sz) != hipSuccess) return CPK_ERR_HIP;
  *size = sz;
  return CPK_OK;
}

// Pinned host staging of the host entry points (grown on demand, never shrunk).
cpk_status ensure_pinned(void** p, size_t* size, size_t need) {
  if (need <= *size) return CPK_OK;
  if (*p) {
    if (hipHostFree(*p) != hipSuccess) return CPK_ERR_HIP;
    *p = nullptr;
    *size = 0;
  }
  const size_t sz = need + need / 8 + 4096;
  if (hipHostMalloc(p, sz, 0) != hipSuccess) return CPK_ERR_HIP;
  *size = sz;
  return CPK_OK;
}

// Host entry points stage through one pinned buffer and one device buffer when the whole call
// fits in this many bytes each way (larger batches keep the per-buffer copies).
constexpr size_t kHostIoMax = 64ull << 20;
// Inputs up to this size are read by the kernels straight from the pinned buffer (no upload);
// CPK_HOST_ZERO_COPY (bytes) overrides it.
size_t zero_copy_max() {
  static const size_t v = [] {
    const char* e = getenv("CPK_HOST_ZERO_COPY");
    return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)(256 << 10);
  }();
  return v;
}

// Staging of one host call.  Device buffer: [error word, 16 B][results][inputs (uploaded)]; the
// error word is zero at rest and stands in for the context's for the call, so one download
// brings back the error and the results together.  Pinned buffer: [inputs][error][results].
struct HostIo {
  uint8_t* hin;   // pinned inputs
  uint8_t* din;   // the kernels' view of the inputs (the pinned buffer itself when small)
  uint8_t* dres;  // device results
  uint8_t* hres;  // pinned results
  uint32_t* derr;
  const uint32_t* herr;
  uint32_t* dherr;  // device view of herr (small batches), else NULL
  bool upload;
};

cpk_status host_io(cpk_ctx* ctx, size_t in_bytes, size_t out_bytes, HostIo* io) {
  cpk_status st;
  void* const hbefore = ctx->hio;
  if ((st = ensure_pinned(&ctx->hio, &ctx->hio_size, in_bytes + 16 + out_bytes)) != CPK_OK)
    return st;
  // (the device view of the pinned buffer, looked up once per allocation)
  if ((ctx->hio != hbefore || !ctx->hio_dev) &&
      hipHostGetDevicePointer((void**)&ctx->hio_dev, ctx->hio, 0) != hipSuccess)
    return CPK_ERR_HIP;
  void* const before = ctx->dio;
  if ((st = ensure(&ctx->dio, &ctx->dio_size, 16 + out_bytes + in_bytes)) != CPK_OK) return st;
  if (ctx->dio != before && (hipMemset(ctx->dio, 0, 16) != hipSuccess ||
                             hipDeviceSynchronize() != hipSuccess))
    return CPK_ERR_HIP;
  uint8_t* const hb = (uint8_t*)ctx->hio;
  uint8_t* const db = (uint8_t*)ctx->dio;
  io->hin = hb;
  io->upload = in_bytes > zero_copy_max();
  io->din = io->upload ? db + 16 + out_bytes : ctx->hio_dev;
  io->derr = (uint32_t*)db;
  io->dres = db + 16;
  io->herr = (const uint32_t*)(hb + in_bytes);
  io->hres = hb + in_bytes + 16;
  io->dherr = nullptr;
  if (!io->upload) {
    // small batches: the kernels also write their results straight to the pinned buffer, and a
    // single-launch kernel its error word (nothing to download then)
    io->dres = ctx->hio_dev + in_bytes + 16;
    io->dherr = (uint32_t*)(ctx->hio_dev + in_bytes);
  }
  return CPK_OK;
}

// Runs fn (the device entry point) on the staged inputs with the call's error word, then brings
// back error and results (out_bytes) with one download and one synchronisation.
template <class F>
cpk_status host_io_run(cpk_ctx* ctx, const HostIo& io, size_t in_bytes, size_t out_bytes,
                       bool* downloaded, F fn) {
  hipStream_t s = nullptr;
  *downloaded = false;
  if (io.upload && hipMemcpyAsync(io.din, io.hin, in_bytes, hipMemcpyHostToDevice, s) != hipSuccess)
    return CPK_ERR_HIP;
  constexpr uint32_t kUnset = 0xffffffffu;  // (no cpk_status)
  if (io.dherr) *(volatile uint32_t*)io.herr = kUnset;
  uint32_t* const saved = ctx->err;
  ctx->err = io.derr;
  ctx->err_host = io.dherr;
  ctx->fused_last = false;
  cpk_status st = fn(s);
  ctx->err = saved;
  ctx->err_host = nullptr;
  if (st != CPK_OK) {
    // kernels of this call may still be running (reading the pinned inputs, raising the call's
    // error word): let them finish and reset the word before the next call reuses both
    (void)hipStreamSynchronize(s);
    (void)hipMemset(io.derr, 0, 4);
    return st;
  }
  if (io.dherr) {
    // results are in place; the error word too when one launch did the call, written last (after
    // a system-scope release): spinning on it returns as soon as the kernel is done, a stream
    // synchronisation only some microseconds later
    bool seen = false;
    if (ctx->fused_last) {
      const auto t0 = std::chrono::steady_clock::now();
      for (uint32_t i = 0;; i++) {
        if (*(volatile const uint32_t*)io.herr != kUnset) {
          seen = true;
          break;
        }
        if ((i & 1023) == 1023 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2))
          break;  // (long call or a fault: the runtime's synchronisation tells)
        _mm_pause();
      }
      std::atomic_thread_fence(std::memory_order_acquire);
    }
    if (!seen) {
      if (hipStreamSynchronize(s) != hipSuccess) return CPK_ERR_HIP;
      if (*(volatile const uint32_t*)io.herr == kUnset &&
          hipMemcpy((void*)io.herr, io.derr, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return CPK_ERR_HIP;
    }
  } else if (hipMemcpyAsync((void*)io.herr, io.derr, 16 + out_bytes, hipMemcpyDeviceToHost, s) !=
                 hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess) {
    return CPK_ERR_HIP;
  }
  *downloaded = true;
  if (*io.herr) {
    st = (cpk_status)*io.herr;
    return hipMemset(io.derr, 0, 4) != hipSuccess ? CPK_ERR_HIP : st;
  }
  return CPK_OK;
}

// Carves aligned sub-buffers out of the context scratch.
struct Carve {
  char* base;
  size_t off = 0;
  explicit Carve(void* b) : base((char*)b) {}
  template <class T>
  T* take(size_t count) {
    T* p = (T*)(base + off);
    off = align16(off + count * sizeof(T));
    return p;
  }
};

hipEvent_t take_event(cpk_ctx* ctx) {
  if (!ctx->pool.empty()) {
    hipEvent_t e = ctx->pool.back();
    ctx->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Brackets one launch with events when timing is on.
struct TimedLaunch {
  cpk_ctx* ctx;
  int which;
  hipStream_t stream;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  TimedLaunch(cpk_ctx* c, int w, hipStream_t s) : ctx(c), which(w), stream(s) {
    if (!ctx->timing) return;
    e0 = take_event(ctx);
    e1 = take_event(ctx);
    if (e0) (void)hipEventRecord(e0, stream);
  }
  void done() {
    if (!ctx->timing || !e0 || !e1) return;
    (void)hipEventRecord(e1, stream);
    ctx->ev[which].emplace_back(e0, e1);
  }
};

// Orders this call after the context's previous call when they come on different streams: the
// scratch, the tile tables and stage[] belong to the context, not to a stream.  (Inside a graph
// capture the previous stream's work is outside the graph: captured sequences use one stream.)
//
// And no two of the codec's waiting launches (tile look-backs, the header scan), from any context
// of the process, run at the same time on one device.  Within one launch a tile waits only on
// tiles dealt earlier to the per-XCD dispatchers, which dispatch in order, so the lowest unfinished
// tile is always resident; two such launches side by side could each fill the XCDs the other's
// next workgroup needs (forward progress).  Kernels of other libraries never wait on
// a codec tile: they only delay it.  So a call that launches waiting kernels (DeviceTurn::waiting)
// records the device's order event behind them, and a call on another stream waits (on the host)
// until they are done before it launches; DeviceTurn holds the device's order lock for the whole
// call, so the event covers the launches.
struct DeviceOrder {
  std::recursive_mutex m;
  hipStream_t last = nullptr;
  bool has = false;
  hipEvent_t ev = nullptr;
};
DeviceOrder& device_order(int device) {
  static DeviceOrder orders[64];
  return orders[device & 63];
}
bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
}
struct DeviceTurn {
  DeviceOrder& o;
  std::unique_lock<std::recursive_mutex> lk;
  hipStream_t stream = nullptr;
  bool waiting = false;  // this call launched waiting kernels on `stream`
  explicit DeviceTurn(cpk_ctx* ctx) : o(device_order(ctx ? ctx->device : 0)), lk(o.m) {}
  ~DeviceTurn() {
    if (!waiting || capturing(stream)) return;
    if (!o.ev && hipEventCreateWithFlags(&o.ev, hipEventDisableTiming) != hipSuccess) return;
    if (hipEventRecord(o.ev, stream) == hipSuccess) {
      o.last = stream;
      o.has = true;
    }
  }
};

cpk_status order_streams(cpk_ctx* ctx, hipStream_t s) {
  if (ctx->used && s != ctx->last_stream) {
    // an event recorded on (or waited for by) a capturing stream would join the other stream to
    // the graph or invalidate the capture: skip the ordering when either stream is capturing
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone, cl = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) return CPK_ERR_HIP;
    if (hipStreamIsCapturing(ctx->last_stream, &cl) != hipSuccess) cl = hipStreamCaptureStatusNone;
    if (cs == hipStreamCaptureStatusNone && cl == hipStreamCaptureStatusNone) {
      if (!ctx->order_ev &&
          hipEventCreateWithFlags(&ctx->order_ev, hipEventDisableTiming) != hipSuccess)
        return CPK_ERR_HIP;
      if (hipEventRecord(ctx->order_ev, ctx->last_stream) != hipSuccess ||
          hipStreamWaitEvent(s, ctx->order_ev, 0) != hipSuccess)
        return CPK_ERR_HIP;
    }
  }
  ctx->used = true;
  ctx->last_stream = s;
  // the device's last waiting launches, when on another stream (of any context): waited for on
  // the host -- a stream-side wait on another stream's event puts a barrier into a hardware queue
  // the two streams may share, and the pipelined host path (bench.py host_inclusive: one stream
  // per chunk, each its own context) then ran its copies one after another (C2 host-inclusive
  // 24.9 -> 13.3 GiB/s)
  DeviceOrder& o = device_order(ctx->device);
  if (o.has && o.last != s && !capturing(s)) {
    if (hipEventSynchronize(o.ev) != hipSuccess) return CPK_ERR_HIP;
    o.has = false;
  }
  return CPK_OK;
}

struct PackScratch {
  uint32_t* state;
  unsigned long long* arena_next;
  uint64_t* desc;
  uint64_t* gdesc;
  size_t zero_bytes;
  uint64_t* tile_first;
  uint64_t* tile_bytes;
  uint32_t* thole;
  uint32_t* tpatch;
  uint64_t* tpiece;
  uint8_t* arena;
  uint64_t arena_cap;
  size_t total;
};

// Byte arena of a pack of `ntiles` tiles: the packed bytes of the tiles whose offset is not known
// in time wait there for the placement launch, each in a piece of exactly its size (rounded to 16
// bytes).  Only a tile of at most kPackArenaTile packed bytes takes a piece, so ntiles pieces of
// that size are all any batch can use (2 bytes per word; at most 8 GiB, past which a tile finding
// it full waits for its offset instead).
uint64_t pack_arena_bytes(uint64_t ntiles) {
  uint64_t cap = ntiles * (uint64_t)cpk::kPackArenaTile;
  if (cap > (8ull << 30)) cap = 8ull << 30;
  return cap;
}

// Pack scratch: the zeroed part (exit budgets polled by the next tile, the arena's fill counter,
// the tiles' look-back descriptors and the placement groups'; zeroed by the framing launch), then
// per tile the first requested position, byte count, count-byte patch and arena piece, then the
// arena.  (The chunk-start bitmap is zero at rest in its own buffer, ctx->pack_bits.)
PackScratch carve_pack(void* base, uint64_t N, uint64_t ntiles) {
  Carve c(base);
  PackScratch s;
  s.state = c.take<uint32_t>(ntiles);
  s.arena_next = c.take<unsigned long long>(2);
  s.desc = c.take<uint64_t>(ntiles);
  s.gdesc = c.take<uint64_t>(cpk::pack_place_groups(ntiles));
  s.zero_bytes = c.off;
  s.tile_first = c.take<uint64_t>(ntiles);
  s.tile_bytes = c.take<uint64_t>(ntiles);
  s.thole = c.take<uint32_t>(ntiles);
  s.tpatch = c.take<uint32_t>(ntiles);
  s.tpiece = c.take<uint64_t>(ntiles);
  s.arena_cap = ntiles > 1 ? pack_arena_bytes(ntiles) : 0;
  s.arena = c.take<uint8_t>(s.arena_cap + 16);
  s.total = c.off;
  return s;
}

size_t pack_scratch_bytes(uint64_t N, uint64_t ntiles) {
  return carve_pack(nullptr, N, ntiles).total + 64;
}

cpk_status ensure_pack_bits(cpk_ctx* ctx, uint64_t N, uint64_t ntiles);
size_t pack_bits_words(uint64_t N, uint64_t ntiles);

cpk_status pack_common(cpk_ctx* ctx, const uint64_t* d_words, uint64_t N, const uint64_t* d_off,
                       uint64_t n, bool messages, uint8_t* d_out, uint64_t cap,
                       uint64_t* d_out_off, int32_t* d_status, hipStream_t stream) {
  if (!ctx || (!d_off && n) || (!d_words && N) || (!d_out && cap)) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  DeviceTurn turn(ctx);  // (for the rest of the call)
  if (order_streams(ctx, stream) != CPK_OK) return CPK_ERR_HIP;
  const uint64_t T = cpk::kPackTileWords;
  const uint64_t ntiles = (N + T - 1) / T;
  // a batch of one tile (a single small message): one launch, the tile kernel framing the batch
  // itself and writing its bytes at offset 0 (no framing or placement launch)
  const bool single = ntiles == 1;
  cpk_status st = ensure(&ctx->scratch, &ctx->scratch_size, carve_pack(nullptr, N, ntiles).total + 64);
  if (st != CPK_OK) return st;
  PackScratch s = carve_pack(ctx->scratch, N, ntiles);
  if ((st = ensure_pack_bits(ctx, N, ntiles)) != CPK_OK) return st;
  uint64_t* const bits = ctx->pack_bits;
  uint8_t* const tstarts = (uint8_t*)(bits + (N + 63) / 64 + 1);
  cpk::TileFirstJob tf;  // tile_first for the requested output positions, in the same launch
  tf.pos = d_off;
  tf.npos = n;
  tf.ntiles = (d_out_off && n && N) ? ntiles : 0;
  tf.T = T;
  tf.out = s.tile_first;
  tf.zero = (uint64_t*)ctx->scratch;  // and the zeroing of the tile kernel's scratch
  tf.zero_words = (s.zero_bytes + 7) / 8;
  if (N == 0) {
    if (d_out_off && cpk::launch_fill(d_out_off, (n + 1) * 8, 0, stream) != hipSuccess)
      return CPK_ERR_HIP;
    tf.zero = nullptr;
    tf.zero_words = 0;
    if (messages && n)
      return hip_status(
          cpk::launch_message_bits(d_words, d_off, n, N, bits, tstarts, d_status, tf, stream));
    return CPK_OK;
  }
  if (messages && n == 0) return CPK_ERR_INVALID_ARGUMENT;  // words outside any message
  hipError_t e = hipSuccess;
  if (!single)
    e = messages ? cpk::launch_message_bits(d_words, d_off, n, N, bits, tstarts, d_status, tf, stream)
                 : cpk::launch_chunk_bits(d_off, n, N, bits, tstarts, tf, stream);
  // the bitmap is zero at rest only if the tile kernel runs and clears it: after any failure
  // from here on it is cleared here
  auto clear_bits = [&]() {
    // (on the call's stream, behind the framing launch: the null stream would not order against
    // a non-blocking stream)
    (void)cpk::launch_fill(bits, pack_bits_words(N, ntiles) * 8, 0, stream);
  };
  if (e != hipSuccess) {
    clear_bits();
    return CPK_ERR_HIP;
  }
  cpk::PackTileArgs a;
  a.words = d_words;
  a.nwords = N;
  a.chunk_bits = bits;
  a.tile_starts = tstarts;
  a.ntiles = ntiles;
  a.out = d_out;
  a.out_capacity = cap;
  a.pos = (d_out_off && n) ? d_off : nullptr;
  a.npos = n;
  a.tile_first = s.tile_first;
  a.pos_out = d_out_off;
  a.total_out = nullptr;
  a.state = s.state;
  a.tile_bytes = s.tile_bytes;
  a.arena = s.arena;
  a.arena_cap = s.arena_cap;
  a.arena_next = s.arena_next;
  a.tpiece = s.tpiece;
  a.gdesc = s.gdesc;
  a.thole = s.thole;
  a.tpatch = s.tpatch;
  a.err = ctx->err;
  a.desc = s.desc;
  a.err_host = single ? ctx->err_host : nullptr;
  ctx->fused_last = a.err_host != nullptr;
  a.frame_mode = single ? (messages ? 1u : 2u) : 0u;
  a.frame_off = d_off;
  a.frame_n = n;
  a.frame_status = d_status;
  turn.stream = stream;
  turn.waiting = !single;  // (the tile kernel's waits, the placement's look-back)
  TimedLaunch tl(ctx, 0, stream);
  // tiles -> output (offset known in time) or arena pieces, placed by the placement launch
  e = cpk::launch_pack_tiles(a, stream);
  if (e != hipSuccess) clear_bits();
  if (e == hipSuccess && !single) e = cpk::launch_pack_place(a, stream);
  tl.done();
  return hip_status(e);
}

// Zero-at-rest header-scan descriptors for n messages (allocated and zeroed once, grown when n
// grows; never part of the re-carved scratch).
cpk_status ensure_hdr_desc(cpk_ctx* ctx, uint64_t n) {
  const size_t need = cpk::header_scan_blocks(n) + 1;
  if (need <= ctx->hdr_desc_n) return CPK_OK;
  if (ctx->hdr_desc && hipFree(ctx->hdr_desc) != hipSuccess) return CPK_ERR_HIP;
  ctx->hdr_desc = nullptr;
  ctx->hdr_desc_n = 0;
  const size_t sz = need + need / 4 + 64;
  if (hipMalloc((void**)&ctx->hdr_desc, sz * 8) != hipSuccess) return CPK_ERR_HIP;
  // (the null stream does not order against non-blocking streams: wait for the zeroing here)
  if (hipMemset(ctx->hdr_desc, 0, sz * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return CPK_ERR_HIP;
  ctx->hdr_desc_n = sz;
  return CPK_OK;
}

// Zero-at-rest chunk-start bitmap of a pack of N words (+ one bit per tile).
size_t pack_bits_words(uint64_t N, uint64_t ntiles) { return (N + 63) / 64 + 1 + (ntiles + 16) / 8; }
cpk_status ensure_pack_bits(cpk_ctx* ctx, uint64_t N, uint64_t ntiles) {
  const size_t need = pack_bits_words(N, ntiles);
  if (need <= ctx->pack_bits_n) return CPK_OK;
  if (ctx->pack_bits && hipFree(ctx->pack_bits) != hipSuccess) return CPK_ERR_HIP;
  ctx->pack_bits = nullptr;
  ctx->pack_bits_n = 0;
  const size_t sz = need + need / 8 + 64;
  if (hipMalloc((void**)&ctx->pack_bits, sz * 8) != hipSuccess) return CPK_ERR_HIP;
  if (hipMemset(ctx->pack_bits, 0, sz * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return CPK_ERR_HIP;
  ctx->pack_bits_n = sz;
  return CPK_OK;
}

struct UnpackScratch {
  uint64_t* desc;
  uint32_t* x0p;
  uint64_t* desc2;
  uint64_t* gdesc;
  uint32_t* gate;
  unsigned int* ticket;
  size_t zero_bytes;
  uint64_t* tile_first;
  uint64_t* tile_firstpos;
  int32_t* hdr_status;
  uint64_t* tbits;
  uint32_t* tegs;
  uint64_t* texcl;
  size_t total;
};

// Unpack scratch: per message 4 B (header status), per 4 KiB tile 28 B (descriptor, chain-0
// exit, first message and its start), and for a flat stream decode 8 B more (second-candidate
// descriptor).  The split message decode adds per tile 524 B (chain 0's record-start bits, the
// guessed entry, the words before the tile) and per 64-tile group 8 B (zeroed).  The tile
// descriptors and exits are zeroed (in the header / init launch).
UnpackScratch carve_unpack(void* base, uint64_t ntiles, uint64_t n, bool flat = false,
                           bool split = false) {
  Carve c(base);
  UnpackScratch s;
  s.desc = c.take<uint64_t>(ntiles);
  s.x0p = c.take<uint32_t>(ntiles);
  s.desc2 = flat ? c.take<uint64_t>(ntiles) : nullptr;
  s.gdesc = split ? c.take<uint64_t>(cpk::resolve_groups(ntiles)) : nullptr;
  s.gate = split ? c.take<uint32_t>(4) : nullptr;
  s.ticket = split ? (unsigned int*)(s.gate + 1) : nullptr;  // the resolve launch's group tickets
  s.zero_bytes = c.off;
  s.tile_first = c.take<uint64_t>(ntiles);
  s.tile_firstpos = c.take<uint64_t>(ntiles);
  s.hdr_status = c.take<int32_t>(n);
  s.tbits = split ? c.take<uint64_t>(ntiles * 64) : nullptr;
  s.tegs = split ? c.take<uint32_t>(ntiles) : nullptr;
  s.texcl = split ? c.take<uint64_t>(ntiles) : nullptr;
  s.total = c.off;
  return s;
}

// The split message decode (index, resolve, expand launches: cpk_unpack.hip) for message batches
// of more than one tile, with CPK_UNPACK_SPLIT=1 (A/B; measured slower than the one-pass kernel,
// DESIGN.md 3.2).
// The stream split's flat decode in two launches (cpk_unpack.hip, FLAT with PHASE 1 / 2): the
// default; CPK_FLAT_SPLIT=0 selects the one-pass flat decode (the measured alternative).
bool flat_split_enabled() {
  static const bool v = !(getenv("CPK_FLAT_SPLIT") && atoi(getenv("CPK_FLAT_SPLIT")) == 0);
  return v;
}
bool unpack_split_enabled() {
  static const bool v = getenv("CPK_UNPACK_SPLIT") && atoi(getenv("CPK_UNPACK_SPLIT")) != 0;
  return v;
}

cpk_status unpack_common(cpk_ctx* ctx, uint32_t mode, const uint8_t* d_packed, uint64_t P,
                         const uint64_t* d_in_off, uint64_t n, const uint64_t* d_word_off_in,
                         uint64_t* d_words, uint64_t cap, uint64_t* d_word_off_out,
                         int32_t* d_status, uint64_t* d_size_out, uint64_t limit,
                         hipStream_t stream, uint64_t* d_in_end = nullptr,
                         uint64_t* d_rec_pos = nullptr, bool store_free = false,
                         const uint64_t* d_rec_gen = nullptr) {
  if (!ctx || (!d_in_off && n) || (!d_packed && P) || (!d_status && n) || (d_rec_pos && !d_rec_gen))
    return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  DeviceTurn turn(ctx);  // (for the rest of the call)
  if (order_streams(ctx, stream) != CPK_OK) return CPK_ERR_HIP;
  const uint64_t B = cpk::kUnpackTileBytes;
  const uint64_t ntiles = (P + B - 1) / B;
  // a flat stream decode (the stream split) carries second-candidate tile descriptors
  const bool flat = d_rec_pos != nullptr;
  // a message batch of several tiles decodes in three launches, no tile waiting on another (the
  // stream readers' message ends, skips and the flat decode keep the one-pass kernel)
  const bool split = mode == 0 && ntiles > 1 && !flat && !d_in_end && !store_free && d_words &&
                     unpack_split_enabled();
  // the flat decode in two launches (index, then decode over published descriptors; the index
  // launch leaves the base chain's record-start bits for the second)
  const bool flat_split = flat && ntiles > 1 && flat_split_enabled();
  UnpackScratch probe = carve_unpack(nullptr, ntiles, n, flat, split || flat_split);
  cpk_status st = ensure(&ctx->scratch, &ctx->scratch_size, probe.total + 64);
  if (st != CPK_OK) return st;
  UnpackScratch s = carve_unpack(ctx->scratch, ntiles, n, flat, split || flat_split);
  const uint64_t* word_off = d_word_off_in;
  hipError_t e = hipSuccess;
  cpk::TileFirstJob tf;  // each tile's first message, in the same launch as the headers
  tf.pos = d_in_off;
  tf.npos = n;
  tf.ntiles = ntiles;
  tf.T = B;
  tf.out = s.tile_first;
  tf.outpos = s.tile_firstpos;
  tf.zero = (uint64_t*)ctx->scratch;  // zeroed in the header / init launch
  tf.zero_words = s.zero_bytes / 8;
  // a single-tile batch of few messages: one launch, the tile kernel reading the headers itself
  const bool fuse = mode == 0 && ntiles == 1 && n <= cpk::kUnpackFuseMsgs;
  // (waiting launches: the tile kernel's look-back, the header launch's scan)
  turn.stream = stream;
  turn.waiting = ntiles > 1 || (mode == 0 && !fuse && cpk::header_scan_blocks(n) > 1);
  if (mode == 0) {
    if (!d_word_off_out) return CPK_ERR_INVALID_ARGUMENT;
    if (n == 0) return hip_status(cpk::launch_fill(d_word_off_out, 8, 0, stream));
    if ((st = ensure_hdr_desc(ctx, n)) != CPK_OK) return st;
    if (!fuse) {
      e = cpk::launch_unpack_header(d_packed, P, d_in_off, n, limit, d_word_off_out, s.hdr_status,
                                    d_status, ctx->hdr_desc, ctx->err, tf, stream);
      if (e != hipSuccess) return CPK_ERR_HIP;
    }
    word_off = d_word_off_out;
    if (ntiles == 0)  // no tile kernel to clear the header launch's descriptors
      return hip_status(cpk::launch_fill(ctx->hdr_desc, 8 * cpk::header_scan_blocks(n), 0, stream));
  } else {
    if (n == 0) return CPK_OK;
    e = cpk::launch_unpack_init(mode, d_in_off, word_off, n, d_status, d_size_out, tf, stream);
    if (e != hipSuccess) return CPK_ERR_HIP;
  }
  if (ntiles == 0) return CPK_OK;
  cpk::UnpackArgs a;
  a.packed = d_packed;
  a.nbytes = P;
  a.in_off = d_in_off;
  a.nmsgs = n;
  a.tile_first = s.tile_first;
  a.tile_firstpos = s.tile_firstpos;
  a.word_off = mode == 2 ? nullptr : word_off;
  a.hdr_status = mode == 0 ? s.hdr_status : nullptr;
  a.words = d_words;
  // a store-free parse (PackedInputStream::skip) decodes against no output at all
  a.words_capacity = store_free ? ~0ull : (d_words ? cap : 0);
  a.status = d_status;
  a.size_out = d_size_out;
  a.in_end = d_in_end;
  a.rec_pos = d_rec_pos;
  a.rec_gen = d_rec_gen;
  a.mode = mode;
  a.ntiles = ntiles;
  a.desc = s.desc;
  a.x0p = s.x0p;
  a.err = ctx->err;
  a.stamps = cpk::debug_stamps(1);  // diagnostic counters (CPK_STAMPS=1), else NULL
  a.debug_skip = cpk::debug_skip();
  a.hdr_desc = ctx->hdr_desc;
  a.hdr_nblocks = mode == 0 && !fuse ? cpk::header_scan_blocks(n) : 0;
  a.desc2 = s.desc2;
  a.hdr_fuse = fuse ? 1u : 0u;
  // messages of >= 4 tiles on average: most tiles look back over AGGs (no message start of their
  // own), and the waves ahead of the expansions in the issue arbitration publish sooner (C2
  // unpack_tiles 225.9 -> 222.6 us, C4 unchanged; on every batch: C5 9.36 -> 9.72 ms)
  a.prio = (mode != 2 && n && P / n >= 4 * B) ? 1u : 0u;
  a.err_host = fuse ? ctx->err_host : nullptr;
  ctx->fused_last = a.err_host != nullptr;
  a.hdr_limit = limit;
  a.hdr_word_off = d_word_off_out;
  a.hdr_status_out = s.hdr_status;
  a.phase = 0;
  a.tbits = s.tbits;
  a.tegs = s.tegs;
  a.texcl = s.texcl;
  a.gate = s.gate;
  TimedLaunch tl(ctx, 1, stream);
  if (split) {
    cpk::ResolveArgs r;
    r.packed = d_packed;
    r.nbytes = P;
    r.ntiles = ntiles;
    r.desc = s.desc;
    r.x0p = s.x0p;
    r.tbits = s.tbits;
    r.tile_firstpos = s.tile_firstpos;
    r.gdesc = s.gdesc;
    r.ticket = s.ticket;
    r.texcl = s.texcl;
    r.gate = s.gate;
    r.err = ctx->err;
    TimedLaunch tk(ctx, 2, stream);
    a.phase = 1;
    e = cpk::launch_unpack_stage(cpk::kUnpackIndex, a, stream);
    if (e == hipSuccess) e = cpk::launch_unpack_resolve(r, stream);
    a.phase = 2;
    a.hdr_nblocks = 0;  // (cleared by the index launch)
    if (e == hipSuccess) e = cpk::launch_unpack_stage(cpk::kUnpackExpand, a, stream);
    tk.done();
    if (e != hipSuccess) {
      (void)cpk::launch_fill(ctx->hdr_desc, 8 * cpk::header_scan_blocks(n), 0, stream);
      return CPK_ERR_HIP;
    }
    tl.done();
    return CPK_OK;
  }
  const int first_stage = flat_split ? cpk::kUnpackIndex : cpk::kUnpackTiles;
  const int last_stage = flat_split ? cpk::kUnpackExpand : cpk::kUnpackTiles;
  for (int stage = first_stage; stage <= last_stage; stage++) {
    TimedLaunch tk(ctx, 2 + stage, stream);
    e = cpk::launch_unpack_stage(stage, a, stream);
    tk.done();
    if (e != hipSuccess) {
      // the header launch ran: its look-back descriptors are zero at rest only if the tile
      // kernel clears them
      if (a.hdr_nblocks) (void)cpk::launch_fill(ctx->hdr_desc, 8 * a.hdr_nblocks, 0, stream);
      return CPK_ERR_HIP;
    }
  }
  tl.done();
  return CPK_OK;
}

}  // namespace

extern "C" {

const char* cpk_status_string(int32_t status) {
  switch (status) {
    case CPK_OK: return "";
    case CPK_ERR_PREMATURE_EOF: return "Premature end of packed input.";
    case CPK_ERR_RUN_OVERSHOOT: return "Packed input did not end cleanly on a segment boundary.";
    case CPK_ERR_TOO_MANY_SEGMENTS: return "Message has too many segments.";
    case CPK_ERR_MESSAGE_TOO_LARGE:
      return "Message is too large.  To increase the limit on the receiving end, see "
             "capnp::ReaderOptions.";
    case CPK_ERR_INVALID_PACKED: return "invalid packed data";
    case CPK_ERR_BAD_FRAMING: return "Segment table does not match the message size.";
    case CPK_ERR_TRAILING_BYTES: return "Packed input holds bytes past the end of the message.";
    case CPK_ERR_CAPACITY: return "backing array was not large enough for the data";
    case CPK_ERR_INVALID_ARGUMENT: return "invalid argument";
    case CPK_ERR_HIP: return "HIP runtime error";
    case CPK_ERR_EMPTY_MESSAGE: return "Tried to serialize uninitialized message.";
    case CPK_ERR_INTERNAL: return "internal error (device wait timed out)";
    case CPK_ERR_NO_DEVICE: return "no HIP device";
    default: return "unknown status";
  }
}

int cpk_abi_version(void) { return CPK_ABI_VERSION; }

uint64_t cpk_packed_bound(uint64_t words, uint64_t chunks) {
  return words * 8 + (words + 1) / 2 + 2 * chunks;
}

cpk_status cpk_init(int device, cpk_ctx** out) {
  if (!out) return CPK_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return CPK_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(device) != hipSuccess) return CPK_ERR_HIP;
  cpk_ctx* c = new (std::nothrow) cpk_ctx();
  if (!c) return CPK_ERR_INTERNAL;
  c->device = device;
  if (hipMalloc((void**)&c->err, 16) != hipSuccess || hipMemset(c->err, 0, 16) != hipSuccess) {
    delete c;
    return CPK_ERR_HIP;
  }
  *out = c;
  return CPK_OK;
}

cpk_status cpk_destroy(cpk_ctx* ctx) {
  if (!ctx) return CPK_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->err) (void)hipFree(ctx->err);
  for (int w = 0; w < CPK_TIMERS; w++)
    for (auto& p : ctx->ev[w]) {
      (void)hipEventDestroy(p.first);
      (void)hipEventDestroy(p.second);
    }
  for (hipEvent_t e : ctx->pool) (void)hipEventDestroy(e);
  for (int i = 0; i < 5; i++)
    if (ctx->stage[i]) (void)hipFree(ctx->stage[i]);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  if (ctx->meta_ev) (void)hipEventDestroy(ctx->meta_ev);
  if (ctx->order_ev) (void)hipEventDestroy(ctx->order_ev);
  if (ctx->hdr_desc) (void)hipFree(ctx->hdr_desc);
  if (ctx->pack_bits) (void)hipFree(ctx->pack_bits);
  if (ctx->hio) (void)hipHostFree(ctx->hio);
  if (ctx->dio) (void)hipFree(ctx->dio);
  delete ctx;
  return CPK_OK;
}

cpk_status cpk_reserve(cpk_ctx* ctx, uint64_t max_words, uint64_t max_packed_bytes,
                       uint64_t max_items) {
  if (!ctx) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  const uint64_t pt = (max_words + cpk::kPackTileWords - 1) / cpk::kPackTileWords;
  size_t need = pack_scratch_bytes(max_words, pt);
  const uint64_t ut = (max_packed_bytes + cpk::kUnpackTileBytes - 1) / cpk::kUnpackTileBytes;
  // (the flat stream decode's second-candidate descriptors included)
  // (the flat decode's second descriptors and, when the split decode is on, its bits and prefixes)
  const size_t un =
      carve_unpack(nullptr, ut, max_items, true, unpack_split_enabled() || flat_split_enabled())
          .total + 64;
  if (un > need) need = un;
  cpk_status st = ensure(&ctx->scratch, &ctx->scratch_size, need);
  if (st != CPK_OK) return st;
  // the zero-at-rest buffers too: a first call at a new size inside a stream capture would
  // otherwise allocate and synchronise the device while the stream is capturing
  if ((st = ensure_pack_bits(ctx, max_words, pt)) != CPK_OK) return st;
  return ensure_hdr_desc(ctx, max_items);
}

cpk_status cpk_copy_ranges(cpk_ctx* ctx, const uint8_t* d_src, const uint64_t* d_src_off,
                           const uint64_t* d_dst_off, const uint64_t* d_len, uint64_t n,
                           uint8_t* d_dst, void* stream) {
  if (!ctx || (n && (!d_src || !d_src_off || !d_dst_off || !d_len || !d_dst)))
    return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  return hip_status(cpk::launch_copy_ranges(d_src, d_src_off, d_dst_off, d_len, n, d_dst,
                                            (hipStream_t)stream));
}

cpk_status cpk_sync(cpk_ctx* ctx, void* stream) {
  if (!ctx) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return CPK_ERR_HIP;
  uint32_t e = 0;
  if (hipMemcpy(&e, ctx->err, 4, hipMemcpyDeviceToHost) != hipSuccess) return CPK_ERR_HIP;
  if (e) {
    if (hipMemset(ctx->err, 0, 4) != hipSuccess) return CPK_ERR_HIP;
  }
  return (cpk_status)e;
}

cpk_status cpk_pack_chunks(cpk_ctx* ctx, const uint64_t* d_words, uint64_t total_words,
                           const uint64_t* d_chunk_word_off, uint64_t nchunks, uint8_t* d_out,
                           uint64_t out_capacity, uint64_t* d_chunk_out_off, void* stream) {
  return pack_common(ctx, d_words, total_words, d_chunk_word_off, nchunks, false, d_out,
                     out_capacity, d_chunk_out_off, nullptr, (hipStream_t)stream);
}

cpk_status cpk_pack_messages(cpk_ctx* ctx, const uint64_t* d_words, uint64_t total_words,
                             const uint64_t* d_msg_word_off, uint64_t nmsgs, uint8_t* d_out,
                             uint64_t out_capacity, uint64_t* d_msg_out_off, int32_t* d_status,
                             void* stream) {
  return pack_common(ctx, d_words, total_words, d_msg_word_off, nmsgs, true, d_out, out_capacity,
                     d_msg_out_off, d_status, (hipStream_t)stream);
}

cpk_status cpk_pack_segments(cpk_ctx* ctx, const uint64_t* const* h_seg_ptrs,
                             const uint64_t* h_seg_words, uint64_t nseg, uint8_t* d_out,
                             uint64_t out_capacity, uint64_t* d_out_bytes, void* stream) {
  if (!ctx || (nseg && (!h_seg_ptrs || !h_seg_words)) || !d_out_bytes)
    return CPK_ERR_INVALID_ARGUMENT;
  if (nseg == 0) return CPK_ERR_EMPTY_MESSAGE;  // serialize.c++:333
  if (nseg > (1u << 20)) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  DeviceTurn turn(ctx);  // (for the rest of the call)
  if (order_streams(ctx, s) != CPK_OK) return CPK_ERR_HIP;
  const uint64_t tw = nseg / 2 + 1;
  // meta: seg_ptr[nseg], chunk_off[nseg + 2], table[tw]
  const uint64_t nmeta = nseg + (nseg + 2) + tw;
  std::vector<uint64_t> chunk_off(nseg + 2);
  chunk_off[0] = 0;
  chunk_off[1] = tw;
  for (uint64_t i = 0; i < nseg; i++) {
    if (h_seg_words[i] > 0xffffffffull || (h_seg_words[i] && !h_seg_ptrs[i]))
      return CPK_ERR_INVALID_ARGUMENT;
    chunk_off[i + 2] = chunk_off[i + 1] + h_seg_words[i];
  }
  const uint64_t total = chunk_off[nseg + 1];
  cpk_status st;
  // the previous call's upload must have left the pinned buffer before it is refilled
  if (ctx->meta_ev && hipEventSynchronize(ctx->meta_ev) != hipSuccess) return CPK_ERR_HIP;
  if (ctx->pinned_size < nmeta * 8) {
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    ctx->pinned = nullptr;
    ctx->pinned_size = 0;
    if (hipHostMalloc(&ctx->pinned, nmeta * 8 + 4096, 0) != hipSuccess) return CPK_ERR_HIP;
    ctx->pinned_size = nmeta * 8 + 4096;
  }
  if (!ctx->meta_ev && hipEventCreateWithFlags(&ctx->meta_ev, hipEventDisableTiming) != hipSuccess)
    return CPK_ERR_HIP;
  uint64_t* h = (uint64_t*)ctx->pinned;
  for (uint64_t i = 0; i < nseg; i++) h[i] = (uint64_t)(uintptr_t)h_seg_ptrs[i];
  memcpy(h + nseg, chunk_off.data(), (nseg + 2) * 8);
  uint32_t* t32 = (uint32_t*)(h + nseg + nseg + 2);  // serializeSegmentTable, serialize.c++:311-330
  memset(t32, 0, tw * 8);
  t32[0] = (uint32_t)(nseg - 1);
  for (uint64_t i = 0; i < nseg; i++) t32[i + 1] = (uint32_t)h_seg_words[i];
  // device: meta, then the flat message, then the chunk output offsets
  const size_t need = align16(nmeta * 8) + align16(total * 8) + (nseg + 2) * 8 + 64;
  if ((st = ensure(&ctx->stage[3], &ctx->stage_size[3], need)) != CPK_OK) return st;
  uint64_t* d_meta = (uint64_t*)ctx->stage[3];
  uint64_t* d_flat = (uint64_t*)((char*)d_meta + align16(nmeta * 8));
  uint64_t* d_chunk_out = (uint64_t*)((char*)d_flat + align16(total * 8));
  if (hipMemcpyAsync(d_meta, h, nmeta * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipEventRecord(ctx->meta_ev, s) != hipSuccess)
    return CPK_ERR_HIP;
  if (cpk::launch_gather_segments(d_meta, (uint32_t)nseg, total, d_flat, s) != hipSuccess)
    return CPK_ERR_HIP;
  st = pack_common(ctx, d_flat, total, d_meta + nseg, nseg + 1, false, d_out, out_capacity,
                   d_chunk_out, nullptr, s);
  if (st != CPK_OK) return st;
  return hip_status(hipMemcpyAsync(d_out_bytes, d_chunk_out + nseg + 1, 8,
                                   hipMemcpyDeviceToDevice, s));
}

cpk_status cpk_pack_messages_host(cpk_ctx* ctx, const uint64_t* h_words, uint64_t total_words,
                                  const uint64_t* h_msg_word_off, uint64_t nmsgs, uint8_t* h_out,
                                  uint64_t out_capacity, uint64_t* h_msg_out_off,
                                  int32_t* h_status) {
  if (!ctx || !h_msg_word_off) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  const size_t wbytes = total_words * 8, obytes = (nmsgs + 1) * 8;
  cpk_status st;
  const size_t in_bytes = align16(wbytes) + align16(obytes);
  const size_t out_bytes = align16(obytes) + align16(4 * nmsgs) + align16(out_capacity);
  if (in_bytes + out_bytes <= kHostIoMax) {
    // inputs read in place (or one upload), the kernels, one download (error word, offsets,
    // statuses, packed bytes), one synchronisation
    HostIo io;
    if ((st = host_io(ctx, in_bytes, out_bytes, &io)) != CPK_OK) return st;
    if (wbytes) memcpy(io.hin, h_words, wbytes);
    memcpy(io.hin + align16(wbytes), h_msg_word_off, obytes);
    const uint64_t* d_words = (const uint64_t*)io.din;
    const uint64_t* d_off = (const uint64_t*)(io.din + align16(wbytes));
    uint64_t* d_out_off = (uint64_t*)io.dres;  // results: out_off | status | packed bytes
    int32_t* d_status = (int32_t*)(io.dres + align16(obytes));
    uint8_t* d_out = io.dres + align16(obytes) + align16(4 * nmsgs);
    bool got = false;
    st = host_io_run(ctx, io, in_bytes, out_bytes, &got, [&](hipStream_t s) {
      return cpk_pack_messages(ctx, d_words, total_words, d_off, nmsgs, d_out, out_capacity,
                               d_out_off, d_status, s);
    });
    const uint64_t* ho = (const uint64_t*)io.hres;
    if (got) {
      if (h_msg_out_off) memcpy(h_msg_out_off, ho, obytes);
      if (h_status && nmsgs) memcpy(h_status, io.hres + align16(obytes), 4 * nmsgs);
    }
    if (st != CPK_OK) return st;
    const uint64_t total = ho[nmsgs];
    if (total > out_capacity) return CPK_ERR_CAPACITY;
    if (total) memcpy(h_out, io.hres + align16(obytes) + align16(4 * nmsgs), total);
    return CPK_OK;
  }
  if ((st = ensure(&ctx->stage[0], &ctx->stage_size[0], wbytes + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[1], &ctx->stage_size[1], out_capacity + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[2], &ctx->stage_size[2], 2 * obytes + 4 * nmsgs + 64)) != CPK_OK)
    return st;
  uint64_t* d_words = (uint64_t*)ctx->stage[0];
  uint8_t* d_out = (uint8_t*)ctx->stage[1];
  uint64_t* d_off = (uint64_t*)ctx->stage[2];
  uint64_t* d_out_off = d_off + (nmsgs + 1);
  int32_t* d_status = (int32_t*)(d_out_off + (nmsgs + 1));
  hipStream_t s = nullptr;
  if (hipMemcpyAsync(d_words, h_words, wbytes, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_off, h_msg_word_off, obytes, hipMemcpyHostToDevice, s) != hipSuccess)
    return CPK_ERR_HIP;
  st = cpk_pack_messages(ctx, d_words, total_words, d_off, nmsgs, d_out, out_capacity, d_out_off,
                         d_status, s);
  if (st != CPK_OK) return st;
  st = cpk_sync(ctx, s);
  uint64_t total = 0;
  if (hipMemcpy(&total, d_out_off + nmsgs, 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  if (h_msg_out_off && hipMemcpy(h_msg_out_off, d_out_off, obytes, hipMemcpyDeviceToHost))
    return CPK_ERR_HIP;
  if (h_status && nmsgs && hipMemcpy(h_status, d_status, 4 * nmsgs, hipMemcpyDeviceToHost))
    return CPK_ERR_HIP;
  if (st != CPK_OK) return st;
  if (total > out_capacity) return CPK_ERR_CAPACITY;
  if (total && hipMemcpy(h_out, d_out, total, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  return CPK_OK;
}

cpk_status cpk_unpack_messages(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t total_bytes,
                               const uint64_t* d_msg_in_off, uint64_t nmsgs, uint64_t* d_words,
                               uint64_t words_capacity, uint64_t* d_msg_word_off,
                               int32_t* d_status, const cpk_limits* limits, void* stream) {
  const uint64_t limit = limits ? limits->traversal_limit_words : 8ull * 1024 * 1024;
  return unpack_common(ctx, 0, d_packed, total_bytes, d_msg_in_off, nmsgs, nullptr, d_words,
                       words_capacity, d_msg_word_off, d_status, nullptr, limit,
                       (hipStream_t)stream);
}

cpk_status cpk_read_packed_messages(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t total_bytes,
                                   const uint64_t* d_msg_in_off, uint64_t nmsgs,
                                   uint64_t* d_words, uint64_t words_capacity,
                                   uint64_t* d_msg_word_off, int32_t* d_status,
                                   uint64_t* d_msg_in_end, const cpk_limits* limits,
                                   void* stream) {
  if (!d_msg_in_end && nmsgs) return CPK_ERR_INVALID_ARGUMENT;
  const uint64_t limit = limits ? limits->traversal_limit_words : 8ull * 1024 * 1024;
  return unpack_common(ctx, 0, d_packed, total_bytes, d_msg_in_off, nmsgs, nullptr, d_words,
                       words_capacity, d_msg_word_off, d_status, nullptr, limit,
                       (hipStream_t)stream, d_msg_in_end);
}

cpk_status cpk_split_packed_stream(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t nbytes,
                                   uint64_t* d_words, uint64_t words_capacity, uint64_t max_msgs,
                                   uint64_t* d_msg_word_off, uint64_t* d_msg_in_off,
                                   int32_t* d_status, uint64_t* d_nmsgs, const cpk_limits* limits,
                                   void* stream) {
  if (!ctx || (!d_packed && nbytes) || !d_msg_word_off || !d_msg_in_off || !d_status || !d_nmsgs ||
      (!d_words && words_capacity) || (words_capacity == 0 && nbytes))
    return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  const uint64_t limit = limits ? limits->traversal_limit_words : 8ull * 1024 * 1024;
  hipStream_t s = (hipStream_t)stream;
  DeviceTurn turn(ctx);  // (for the rest of the call)
  if (order_streams(ctx, s) != CPK_OK) return CPK_ERR_HIP;
  // (record positions share their u64 with the call's generation: kRecGenShift bits)
  if (nbytes >> cpk::kRecGenShift) return CPK_ERR_INVALID_ARGUMENT;
  // the record-head map (one u64 per output word) after 16 words of state: in_off[2],
  // word_off[2], meta[4] (stop byte, stop word, decode status), the map's generation and fill
  // flag (kept from call to call)
  const uint64_t rp_bytes = align16(words_capacity * 8 + 128);
  cpk_status st = ensure(&ctx->stage[4], &ctx->stage_size[4],
                         rp_bytes + cpk::split_scratch_bytes(words_capacity));
  if (st != CPK_OK) return st;
  uint64_t* state = (uint64_t*)ctx->stage[4];
  uint64_t* meta = state + 4;
  uint64_t* genw = state + 8;
  uint32_t* fillw = (uint32_t*)(state + 9);
  uint64_t* rec_pos = state + 16;
  void* split_scr = (char*)ctx->stage[4] + rp_bytes;
  // the map is filled when its memory or extent is new to it (the scratch after it moves with
  // the extent) or the generation wraps; otherwise the generation moves on and old entries stop
  // counting
  const bool fresh = ctx->split_map != ctx->stage[4] || ctx->split_map_size != ctx->stage_size[4] ||
                     ctx->split_map_words != words_capacity;
  hipError_t e = cpk::launch_set_u64x4(state, 0, nbytes, 0, words_capacity, s);
  if (e == hipSuccess) e = cpk::launch_set_u64x4(meta, 0, 0, CPK_ERR_PREMATURE_EOF, 0, s);
  if (e == hipSuccess) e = cpk::launch_split_gen(genw, fillw, fresh, rec_pos, words_capacity * 8, s);
  if (e != hipSuccess) return CPK_ERR_HIP;
  ctx->split_map = ctx->stage[4];
  ctx->split_map_size = ctx->stage_size[4];
  ctx->split_map_words = words_capacity;
  if (nbytes) {
    // the whole stream as one flat chunk of up to words_capacity words, stopping at the first
    // record the input cuts (prefix mode: meta[0..1] = where it stopped)
    st = unpack_common(ctx, 1, d_packed, nbytes, state, 1, state + 2, d_words, words_capacity,
                       nullptr, (int32_t*)(meta + 2), meta + 1, 0, s, meta, rec_pos, false, genw);
    if (st != CPK_OK) return st;
  }
  return hip_status(cpk::launch_split_walk(d_packed, nbytes, d_words, rec_pos, genw, meta, max_msgs,
                                           limit, words_capacity, split_scr, d_msg_word_off,
                                           d_msg_in_off, d_status, d_nmsgs, s));
}

cpk_status cpk_unpacked_size(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t total_bytes,
                             const uint64_t* d_in_off, uint64_t n, uint64_t* d_words_out,
                             int32_t* d_status, void* stream) {
  if (!d_words_out && n) return CPK_ERR_INVALID_ARGUMENT;
  return unpack_common(ctx, 2, d_packed, total_bytes, d_in_off, n, nullptr, nullptr, 0, nullptr,
                       d_status, d_words_out, 0, (hipStream_t)stream);
}

cpk_status cpk_unpack_chunks(cpk_ctx* ctx, const uint8_t* d_packed, uint64_t total_bytes,
                             const uint64_t* d_in_off, const uint64_t* d_word_off, uint64_t n,
                             uint64_t* d_words, uint64_t words_capacity, int32_t* d_status,
                             void* stream) {
  if (!d_word_off && n) return CPK_ERR_INVALID_ARGUMENT;
  return unpack_common(ctx, 1, d_packed, total_bytes, d_in_off, n, d_word_off, d_words,
                       words_capacity, nullptr, d_status, nullptr, 0, (hipStream_t)stream);
}

cpk_status cpk_unpack_messages_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t total_bytes,
                                    const uint64_t* h_msg_in_off, uint64_t nmsgs,
                                    uint64_t* h_words, uint64_t words_capacity,
                                    uint64_t* h_msg_word_off, int32_t* h_status,
                                    const cpk_limits* limits) {
  if (!ctx || !h_msg_in_off || (!h_words && words_capacity)) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  const size_t obytes = (nmsgs + 1) * 8;
  cpk_status st;
  const size_t in_bytes = align16(total_bytes) + align16(obytes);
  const size_t out_bytes = align16(obytes) + align16(4 * nmsgs) + align16(words_capacity * 8);
  if (in_bytes + out_bytes <= kHostIoMax) {
    // inputs read in place (or one upload), the kernels, one download (error word, word
    // offsets, statuses, words), one synchronisation
    HostIo io;
    if ((st = host_io(ctx, in_bytes, out_bytes, &io)) != CPK_OK) return st;
    if (total_bytes) memcpy(io.hin, h_packed, total_bytes);
    memcpy(io.hin + align16(total_bytes), h_msg_in_off, obytes);
    const uint8_t* d_packed = io.din;
    const uint64_t* d_in_off = (const uint64_t*)(io.din + align16(total_bytes));
    uint64_t* d_word_off = (uint64_t*)io.dres;  // results: word offsets | status | words
    int32_t* d_status = (int32_t*)(io.dres + align16(obytes));
    uint64_t* d_words = (uint64_t*)(io.dres + align16(obytes) + align16(4 * nmsgs));
    bool got = false;
    st = host_io_run(ctx, io, in_bytes, out_bytes, &got, [&](hipStream_t s) {
      return cpk_unpack_messages(ctx, d_packed, total_bytes, d_in_off, nmsgs, d_words,
                                 words_capacity, d_word_off, d_status, limits, s);
    });
    const uint64_t* hw = (const uint64_t*)io.hres;
    if (got) {
      if (h_msg_word_off) memcpy(h_msg_word_off, hw, obytes);
      if (h_status && nmsgs) memcpy(h_status, io.hres + align16(obytes), 4 * nmsgs);
    }
    if (st != CPK_OK) return st;
    const uint64_t total = hw[nmsgs];
    const uint64_t n = total < words_capacity ? total : words_capacity;
    if (n) memcpy(h_words, io.hres + align16(obytes) + align16(4 * nmsgs), n * 8);
    return CPK_OK;
  }
  if ((st = ensure(&ctx->stage[0], &ctx->stage_size[0], words_capacity * 8 + 16)) != CPK_OK)
    return st;
  if ((st = ensure(&ctx->stage[1], &ctx->stage_size[1], total_bytes + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[2], &ctx->stage_size[2], 2 * obytes + 4 * nmsgs + 64)) != CPK_OK)
    return st;
  uint64_t* d_words = (uint64_t*)ctx->stage[0];
  uint8_t* d_packed = (uint8_t*)ctx->stage[1];
  uint64_t* d_in_off = (uint64_t*)ctx->stage[2];
  uint64_t* d_word_off = d_in_off + (nmsgs + 1);
  int32_t* d_status = (int32_t*)(d_word_off + (nmsgs + 1));
  hipStream_t s = nullptr;
  if ((total_bytes &&
       hipMemcpyAsync(d_packed, h_packed, total_bytes, hipMemcpyHostToDevice, s) != hipSuccess) ||
      hipMemcpyAsync(d_in_off, h_msg_in_off, obytes, hipMemcpyHostToDevice, s) != hipSuccess)
    return CPK_ERR_HIP;
  st = cpk_unpack_messages(ctx, d_packed, total_bytes, d_in_off, nmsgs, d_words, words_capacity,
                           d_word_off, d_status, limits, s);
  if (st != CPK_OK) return st;
  st = cpk_sync(ctx, s);
  uint64_t total = 0;
  if (hipMemcpy(&total, d_word_off + nmsgs, 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  if (h_msg_word_off && hipMemcpy(h_msg_word_off, d_word_off, obytes, hipMemcpyDeviceToHost))
    return CPK_ERR_HIP;
  if (h_status && nmsgs && hipMemcpy(h_status, d_status, 4 * nmsgs, hipMemcpyDeviceToHost))
    return CPK_ERR_HIP;
  if (st != CPK_OK) return st;
  const uint64_t n = total < words_capacity ? total : words_capacity;
  if (n && hipMemcpy(h_words, d_words, n * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  return CPK_OK;
}

cpk_status cpk_read_packed_message_host(cpk_ctx* ctx, const uint8_t* h_packed,
                                       uint64_t avail_bytes, uint64_t* h_words,
                                       uint64_t words_capacity, uint64_t* words_out,
                                       uint64_t* consumed_out, const cpk_limits* limits) {
  if (!ctx || (!h_packed && avail_bytes) || (!h_words && words_capacity))
    return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  if (words_out) *words_out = 0;
  if (consumed_out) *consumed_out = 0;
  if (avail_bytes == 0) return CPK_ERR_PREMATURE_EOF;
  cpk_status st;
  if ((st = ensure(&ctx->stage[0], &ctx->stage_size[0], words_capacity * 8 + 16)) != CPK_OK)
    return st;
  if ((st = ensure(&ctx->stage[1], &ctx->stage_size[1], avail_bytes + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[2], &ctx->stage_size[2], 64)) != CPK_OK) return st;
  uint64_t* d_words = (uint64_t*)ctx->stage[0];
  uint8_t* d_packed = (uint8_t*)ctx->stage[1];
  uint64_t* d_in_off = (uint64_t*)ctx->stage[2];  // [2]
  uint64_t* d_word_off = d_in_off + 2;            // [2]
  uint64_t* d_in_end = d_word_off + 2;            // [1]
  int32_t* d_status = (int32_t*)(d_in_end + 1);
  const uint64_t in_off[2] = {0, avail_bytes};
  hipStream_t s = nullptr;
  if (hipMemcpyAsync(d_packed, h_packed, avail_bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_in_off, in_off, 16, hipMemcpyHostToDevice, s) != hipSuccess)
    return CPK_ERR_HIP;
  st = cpk_read_packed_messages(ctx, d_packed, avail_bytes, d_in_off, 1, d_words, words_capacity,
                                d_word_off, d_status, d_in_end, limits, s);
  if (st != CPK_OK) return st;
  if ((st = cpk_sync(ctx, s)) != CPK_OK) return st;
  uint64_t wo[2] = {0, 0}, end = 0;
  int32_t ms = 0;
  if (hipMemcpy(wo, d_word_off, 16, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&end, d_in_end, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&ms, d_status, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  // more bytes in the buffer than the message uses: the rest is the next message's
  if (ms == CPK_ERR_TRAILING_BYTES) ms = CPK_OK;
  if (words_out) *words_out = wo[1];
  if (ms != CPK_OK) return (cpk_status)ms;
  if (consumed_out) *consumed_out = end;
  if (wo[1] > words_capacity) return CPK_ERR_CAPACITY;
  if (wo[1] && hipMemcpy(h_words, d_words, wo[1] * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  return CPK_OK;
}

cpk_status cpk_pack_chunks_host(cpk_ctx* ctx, const uint64_t* h_words, uint64_t total_words,
                                const uint64_t* h_chunk_word_off, uint64_t nchunks, uint8_t* h_out,
                                uint64_t out_capacity, uint64_t* h_chunk_out_off) {
  if (!ctx || (!h_chunk_word_off && nchunks) || (!h_words && total_words))
    return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  const size_t wbytes = total_words * 8, obytes = (nchunks + 1) * 8;
  cpk_status st;
  if ((st = ensure(&ctx->stage[0], &ctx->stage_size[0], wbytes + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[1], &ctx->stage_size[1], out_capacity + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[2], &ctx->stage_size[2], 2 * obytes + 64)) != CPK_OK) return st;
  uint64_t* d_words = (uint64_t*)ctx->stage[0];
  uint8_t* d_out = (uint8_t*)ctx->stage[1];
  uint64_t* d_off = (uint64_t*)ctx->stage[2];
  uint64_t* d_out_off = d_off + (nchunks + 1);
  hipStream_t s = nullptr;
  if ((wbytes && hipMemcpyAsync(d_words, h_words, wbytes, hipMemcpyHostToDevice, s)) ||
      hipMemcpyAsync(d_off, h_chunk_word_off, obytes, hipMemcpyHostToDevice, s) != hipSuccess)
    return CPK_ERR_HIP;
  st = cpk_pack_chunks(ctx, d_words, total_words, d_off, nchunks, d_out, out_capacity, d_out_off,
                       s);
  if (st != CPK_OK) return st;
  st = cpk_sync(ctx, s);
  uint64_t total = 0;
  if (hipMemcpy(&total, d_out_off + nchunks, 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  if (h_chunk_out_off && hipMemcpy(h_chunk_out_off, d_out_off, obytes, hipMemcpyDeviceToHost))
    return CPK_ERR_HIP;
  if (st != CPK_OK) return st;
  if (total > out_capacity) return CPK_ERR_CAPACITY;
  if (total && hipMemcpy(h_out, d_out, total, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  return CPK_OK;
}

cpk_status cpk_unpack_words_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t avail_bytes,
                                 uint64_t* h_words, uint64_t nwords, uint64_t* consumed_out) {
  if (!ctx || (!h_packed && avail_bytes) || (!h_words && nwords) || !consumed_out)
    return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  *consumed_out = 0;
  if (nwords == 0) return CPK_OK;
  if (avail_bytes == 0) return CPK_ERR_PREMATURE_EOF;
  cpk_status st;
  if ((st = ensure(&ctx->stage[0], &ctx->stage_size[0], nwords * 8 + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[1], &ctx->stage_size[1], avail_bytes + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[2], &ctx->stage_size[2], 64)) != CPK_OK) return st;
  uint64_t* d_words = (uint64_t*)ctx->stage[0];
  uint8_t* d_packed = (uint8_t*)ctx->stage[1];
  uint64_t* d_in_off = (uint64_t*)ctx->stage[2];  // [2]
  uint64_t* d_word_off = d_in_off + 2;            // [2]
  uint64_t* d_in_end = d_word_off + 2;            // [1]
  int32_t* d_status = (int32_t*)(d_in_end + 1);
  const uint64_t offs[4] = {0, avail_bytes, 0, nwords};
  hipStream_t s = nullptr;
  if (hipMemcpyAsync(d_packed, h_packed, avail_bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_in_off, offs, 32, hipMemcpyHostToDevice, s) != hipSuccess)
    return CPK_ERR_HIP;
  // one exact-size chunk (the flat-packed mode) with the end of its last record reported
  st = unpack_common(ctx, 1, d_packed, avail_bytes, d_in_off, 1, d_word_off, d_words, nwords,
                     nullptr, d_status, nullptr, 0, s, d_in_end);
  if (st != CPK_OK) return st;
  if ((st = cpk_sync(ctx, s)) != CPK_OK) return st;
  uint64_t end = 0;
  int32_t ms = 0;
  if (hipMemcpy(&end, d_in_end, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&ms, d_status, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  if (ms == CPK_ERR_TRAILING_BYTES) ms = CPK_OK;  // the rest of the buffer is not ours
  if (ms != CPK_OK) return (cpk_status)ms;
  *consumed_out = end;
  if (hipMemcpy(h_words, d_words, nwords * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  return CPK_OK;
}

cpk_status cpk_unpack_prefix_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t avail_bytes,
                                  uint64_t* h_words, uint64_t max_words, uint64_t* words_out,
                                  uint64_t* consumed_out) {
  if (!ctx || (!h_packed && avail_bytes) || !words_out || !consumed_out)
    return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  *words_out = 0;
  *consumed_out = 0;
  if (max_words == 0) return CPK_OK;
  if (avail_bytes == 0) return CPK_ERR_PREMATURE_EOF;
  // a record of b bytes yields at most 128 b words (a 2-byte zero run: 256 words), so the
  // device never writes past min(max_words, 128 * avail + 256) words
  const uint64_t room = std::min<uint64_t>(max_words, 128 * avail_bytes + 256);
  cpk_status st;
  // h_words NULL: a skip (serialize-packed.c++:185-299) -- parsed with nothing stored at all
  const bool store_free = h_words == nullptr;
  if (!store_free &&
      (st = ensure(&ctx->stage[0], &ctx->stage_size[0], room * 8 + 16)) != CPK_OK)
    return st;
  if ((st = ensure(&ctx->stage[1], &ctx->stage_size[1], avail_bytes + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[2], &ctx->stage_size[2], 80)) != CPK_OK) return st;
  uint64_t* d_words = store_free ? nullptr : (uint64_t*)ctx->stage[0];
  uint8_t* d_packed = (uint8_t*)ctx->stage[1];
  uint64_t* d_in_off = (uint64_t*)ctx->stage[2];  // [2]
  uint64_t* d_word_off = d_in_off + 2;            // [2]
  uint64_t* d_in_end = d_word_off + 2;            // [1]
  uint64_t* d_at = d_in_end + 1;                  // [1]
  int32_t* d_status = (int32_t*)(d_at + 1);
  const uint64_t offs[4] = {0, avail_bytes, 0, max_words};
  hipStream_t s = nullptr;
  if (hipMemcpyAsync(d_packed, h_packed, avail_bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_in_off, offs, 32, hipMemcpyHostToDevice, s) != hipSuccess ||
      cpk::launch_fill(d_in_end, 16, 0, s) != hipSuccess)
    return CPK_ERR_HIP;
  // one exact-size chunk of max_words words (the flat-packed mode); with d_at given the
  // terminal record also reports where a short or overshooting read stops
  st = unpack_common(ctx, 1, d_packed, avail_bytes, d_in_off, 1, d_word_off, d_words, max_words,
                     nullptr, d_status, d_at, 0, s, d_in_end, nullptr, store_free);
  if (st != CPK_OK) return st;
  if ((st = cpk_sync(ctx, s)) != CPK_OK) return st;
  uint64_t at[2] = {0, 0};  // in_end, words
  int32_t ms = 0;
  if (hipMemcpy(at, d_in_end, 16, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&ms, d_status, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  if (ms == CPK_ERR_TRAILING_BYTES) ms = CPK_OK;  // the rest of the buffer is not ours
  if (ms != CPK_OK && ms != CPK_ERR_PREMATURE_EOF && ms != CPK_ERR_RUN_OVERSHOOT)
    return (cpk_status)ms;
  if (ms == CPK_OK) at[1] = max_words;
  if (at[0] > avail_bytes || at[1] > room) return CPK_ERR_INTERNAL;
  *words_out = at[1];
  *consumed_out = at[0];
  if (h_words && at[1] &&
      hipMemcpy(h_words, d_words, at[1] * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  return (cpk_status)ms;
}

cpk_status cpk_unpacked_size_host(cpk_ctx* ctx, const uint8_t* h_packed, uint64_t nbytes,
                                  uint64_t* words_out) {
  if (!ctx || (!h_packed && nbytes) || !words_out) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  *words_out = 0;
  if (nbytes == 0) return CPK_OK;
  cpk_status st;
  if ((st = ensure(&ctx->stage[1], &ctx->stage_size[1], nbytes + 16)) != CPK_OK) return st;
  if ((st = ensure(&ctx->stage[2], &ctx->stage_size[2], 64)) != CPK_OK) return st;
  uint8_t* d_packed = (uint8_t*)ctx->stage[1];
  uint64_t* d_in_off = (uint64_t*)ctx->stage[2];
  uint64_t* d_size = d_in_off + 2;
  int32_t* d_status = (int32_t*)(d_size + 1);
  const uint64_t in_off[2] = {0, nbytes};
  hipStream_t s = nullptr;
  if (hipMemcpyAsync(d_packed, h_packed, nbytes, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_in_off, in_off, 16, hipMemcpyHostToDevice, s) != hipSuccess)
    return CPK_ERR_HIP;
  st = cpk_unpacked_size(ctx, d_packed, nbytes, d_in_off, 1, d_size, d_status, s);
  if (st != CPK_OK) return st;
  if ((st = cpk_sync(ctx, s)) != CPK_OK) return st;
  int32_t ms = 0;
  if (hipMemcpy(words_out, d_size, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&ms, d_status, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  return (cpk_status)ms;
}

// Diagnostic (not in include/cpk.h): the last pack call's per-tile tables (two-pass kernels).
extern "C" cpk_status cpk_debug_stamps(int which, uint64_t* out16) {
  unsigned long long* b = cpk::debug_stamps(which);
  if (!b || !out16) return CPK_ERR_INVALID_ARGUMENT;
  if (hipDeviceSynchronize() != hipSuccess) return CPK_ERR_HIP;
  // rows of kStampSlots slots (spread by block), summed here
  std::vector<uint64_t> rows((size_t)cpk::kStampSlots * cpk::kStampRows);
  if (hipMemcpy(rows.data(), b, rows.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CPK_ERR_HIP;
  for (int i = 0; i < 16; i++) out16[i] = 0;
  for (size_t r = 0; r < rows.size(); r++) out16[r % cpk::kStampSlots] += rows[r];
  if (hipMemset(b, 0, rows.size() * 8) != hipSuccess) return CPK_ERR_HIP;
  return CPK_OK;
}

// Diagnostic (not in include/cpk.h): raw copy of a stamp buffer.
extern "C" cpk_status cpk_debug_dump(int which, uint64_t* out, uint64_t n) {
  unsigned long long* b = cpk::debug_stamps(which);
  if (!b || !out || n > (uint64_t)cpk::kStampSlots * cpk::kStampRows) return CPK_ERR_INVALID_ARGUMENT;
  if (hipDeviceSynchronize() != hipSuccess) return CPK_ERR_HIP;
  if (hipMemcpy(out, b, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return CPK_ERR_HIP;
  return CPK_OK;
}

// Diagnostic (not in include/cpk.h): the streaming copy kernel bench.py measures the HBM ceiling
// with (16 B per lane; dst, src and nbytes 16-byte aligned).
extern "C" cpk_status cpk_debug_copy(void* dst, const void* src, uint64_t nbytes, uint32_t blocks,
                                     void* stream) {
  return hip_status(cpk::launch_copy(dst, src, nbytes, blocks, (hipStream_t)stream));
}

cpk_status cpk_timing_enable(cpk_ctx* ctx, int on) {
  if (!ctx) return CPK_ERR_INVALID_ARGUMENT;
  ctx->timing = on != 0;
  return CPK_OK;
}

cpk_status cpk_timing_read_all(cpk_ctx* ctx, double* ms_out, uint64_t* launches) {
  if (!ctx) return CPK_ERR_INVALID_ARGUMENT;
  double ms[CPK_TIMERS] = {0};
  for (int w = 0; w < CPK_TIMERS; w++) {
    for (auto& p : ctx->ev[w]) {
      float t = 0;
      if (hipEventSynchronize(p.second) != hipSuccess ||
          hipEventElapsedTime(&t, p.first, p.second) != hipSuccess)
        return CPK_ERR_HIP;
      ms[w] += t;
    }
  }
  for (int w = 0; w < CPK_TIMERS; w++) {
    if (ms_out) ms_out[w] = ms[w];
    if (launches) launches[w] = ctx->ev[w].size();
    for (auto& p : ctx->ev[w]) {
      ctx->pool.push_back(p.first);
      ctx->pool.push_back(p.second);
    }
    ctx->ev[w].clear();
  }
  return CPK_OK;
}

cpk_status cpk_timing_read(cpk_ctx* ctx, double* pack_ms, uint64_t* pack_launches,
                           double* unpack_ms, uint64_t* unpack_launches) {
  double ms[CPK_TIMERS];
  uint64_t n[CPK_TIMERS];
  const cpk_status st = cpk_timing_read_all(ctx, ms, n);
  if (st != CPK_OK) return st;
  if (pack_ms) *pack_ms = ms[0];
  if (unpack_ms) *unpack_ms = ms[1];
  if (pack_launches) *pack_launches = n[0];
  if (unpack_launches) *unpack_launches = n[1];
  return CPK_OK;
}

cpk_status cpk_gen_messages(cpk_ctx* ctx, int profile, uint64_t seed, uint64_t first_msg,
                            uint64_t msg_stride, uint64_t nmsgs, uint32_t nseg,
                            const uint64_t* d_msg_word_off, uint64_t* d_words, void* stream) {
  if (!ctx || profile < 0 || profile > 3 || nseg == 0) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  return hip_status(cpk::launch_gen(profile, seed, first_msg, msg_stride ? msg_stride : 1, nmsgs, nseg, d_msg_word_off,
                                    d_words, (hipStream_t)stream));
}

cpk_status cpk_gen_offsets(cpk_ctx* ctx, uint64_t seed, uint64_t first_msg,
                           uint64_t msg_stride, uint64_t nmsgs, uint32_t nseg, uint64_t seg_words, uint64_t* d_msg_word_off,
                           uint64_t* total_words_out, void* stream) {
  if (!ctx || nseg == 0 || (seg_words == 0 && nseg != 1)) return CPK_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(ctx->device) != hipSuccess) return CPK_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  const uint64_t nt = cpk::scan_tiles(nmsgs);
  const size_t need = 16 + align16(8 * nt) + align16(8 * (nmsgs + 1)) + 64;
  cpk_status st = ensure(&ctx->scratch, &ctx->scratch_size, need);
  if (st != CPK_OK) return st;
  Carve c(ctx->scratch);
  uint32_t* counter = c.take<uint32_t>(4);
  uint64_t* desc = c.take<uint64_t>(nt);
  const size_t zero = c.off;
  uint64_t* sizes = c.take<uint64_t>(nmsgs + 1);
  if (cpk::launch_fill(ctx->scratch, zero, 0, s) != hipSuccess) return CPK_ERR_HIP;
  if (cpk::launch_gen_sizes(seed, first_msg, msg_stride ? msg_stride : 1, nmsgs, nseg, seg_words, sizes, s) != hipSuccess)
    return CPK_ERR_HIP;
  if (cpk::launch_exclusive_scan(sizes, nmsgs, d_msg_word_off, counter, desc, ctx->err, s) !=
      hipSuccess)
    return CPK_ERR_HIP;
  if (total_words_out) {
    if (hipMemcpyAsync(total_words_out, d_msg_word_off + nmsgs, 8, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return CPK_ERR_HIP;
  }
  return CPK_OK;
}

}  // extern "C"
