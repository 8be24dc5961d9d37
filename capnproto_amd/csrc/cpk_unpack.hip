// cpk_unpack.hip -- MI355X (gfx950) kernels for Cap'n Proto's packed decoding.
//
// Functional spec: PackedInputStream::tryRead (capnproto c++/src/capnp/serialize-packed.c++:
// 34-183) driven by InputStreamMessageReader (serialize.c++:202-302): read the first word, check
// the segment count (< 512), read the rest of the table, check the traversal limit, then read
// all segments.  A record is a tag byte, its non-zero bytes, and for tags 0x00 / 0xff a count
// byte (plus 8*count raw bytes for 0xff); a run may not overshoot the words being read.
//
// Three launches per batch:
//   1. header_kernel    one thread per message: decodes the first word and the rest of the
//                       segment table with the reference's checks; yields the flat size.
//   2. scan             message word offsets (cpk_scan.hip).
//   3. body_kernel      one wave per 4 KiB tile of the packed batch.  Record starts are a chain
//                       (next = p + record length) that restarts at every message start.  Each
//                       lane walks its 64-byte sub-tile speculatively from the sub-tile start;
//                       lanes then agree on their true entries by a fixed-point iteration of
//                       "entry = max(previous exits)", re-walking only where an entry misses the
//                       speculative chain.  Across tiles the same idea runs optimistically: a
//                       tile publishes the exit of the chain entered at its own first byte, the
//                       successor uses it as its entry, and every tile verifies that its true
//                       entry (its predecessor's published exit) leads to the exit it published.
//                       A tile whose chains do not merge flags the message; flagged messages are
//                       re-decoded serially by fallback_kernel (never seen on canonical input).
//                       Word offsets come from a segmented (per message) decoupled look-back.
//                       Records are then expanded one lane per record, 64 consecutive records at
//                       a time, so output stores are coalesced; zero and raw runs are written
//                       cooperatively by the whole wave.
#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {

namespace {

constexpr int kB = (int)kUnpackTileBytes;  // 4096
constexpr int kPad = 16;
constexpr int kDead = 1 << 24;  // chain ran into the end of the batch
constexpr uint64_t kSegBit = 1ull << 61;

// status codes (include/cpk.h)
constexpr int32_t kOK = 0, kEOF = 1, kOvershoot = 2, kTooMany = 3, kTooLarge = 4, kInvalid = 5;
constexpr int32_t kTrailing = 7, kCap = 8;
constexpr int32_t kSizeDone = 100;  // mode 2: last record of the buffer

__device__ __forceinline__ uint64_t load_u64_unaligned(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

// PackedInputStream::read of exactly n words from b[p..end) (serialize-packed.c++:65-177 with
// minBytes == maxBytes); f(index, word) receives every word.  Same failure order as the
// reference: missing bytes -> PREMATURE_EOF, run past n -> RUN_OVERSHOOT (checked once the count
// byte is present, before the raw bytes).
template <class F>
__device__ int32_t decode_exact(const uint8_t* b, uint64_t& p, uint64_t end, uint64_t n, F f) {
  uint64_t o = 0;
  while (o < n) {
    if (p >= end) return kEOF;
    const uint32_t tag = b[p++];
    uint64_t w = 0;
    for (int i = 0; i < 8; i++) {
      if ((tag >> i) & 1) {
        if (p >= end) return kEOF;
        w |= (uint64_t)b[p++] << (8 * i);
      }
    }
    f(o, w);
    o++;
    if (tag == 0 || tag == 0xff) {
      if (p >= end) return kEOF;
      const uint64_t c = b[p++];
      if (c > n - o) return kOvershoot;
      if (tag == 0) {
        for (uint64_t k = 0; k < c; k++) f(o + k, 0);
      } else {
        if (end - p < 8 * c) return kEOF;
        for (uint64_t k = 0; k < c; k++) f(o + k, load_u64_unaligned(b + p + 8 * k));
        p += 8 * c;
      }
      o += c;
    }
  }
  return kOK;
}

// 1. Message headers (serialize.c++:202-242).
__global__ void header_kernel(const uint8_t* __restrict__ packed,
                              const uint64_t* __restrict__ in_off, uint64_t n, uint64_t limit,
                              uint64_t* __restrict__ flat, int32_t* __restrict__ hdr_status,
                              int32_t* __restrict__ status) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  uint64_t p = in_off[m];
  const uint64_t end = in_off[m + 1];
  uint64_t first = 0;
  int32_t st = decode_exact(packed, p, end, 1, [&](uint64_t, uint64_t w) { first = w; });
  uint64_t words = 0;
  if (st == kOK) {
    const uint32_t segm1 = (uint32_t)first;
    if (segm1 >= 511) {
      st = kTooMany;
    } else {
      const uint32_t nseg = segm1 + 1;
      uint64_t total = first >> 32;
      if (nseg > 1) {
        st = decode_exact(packed, p, end, (nseg & ~1u) / 2, [&](uint64_t i, uint64_t w) {
          if (2 + 2 * i <= nseg) total += (uint32_t)w;
          if (3 + 2 * i <= nseg) total += (uint32_t)(w >> 32);
        });
      }
      if (st == kOK) {
        if (total > limit) st = kTooLarge;
        else words = nseg / 2 + 1 + total;
      }
    }
  }
  flat[m] = words;
  hdr_status[m] = st;
  status[m] = st;
}

// Record length at tile position p given the staged bytes (no clipping).
__device__ __forceinline__ int record_len(const uint8_t* d, int p) {
  const uint32_t tag = d[p];
  int len = 1 + __popc(tag);
  if (tag == 0) len += 1;
  else if (tag == 0xff) len += 1 + 8 * (int)d[p + 9];
  return len;
}

struct SubTile {
  int s, end, vend;  // sub-tile [s, end); walks stop at vend = min(end, batch end)
  uint64_t msw;      // message-start bits of the sub-tile
  int nms_after;     // first message start >= end (tile-relative; may be >= kB)
  int pend;          // batch end, tile-relative
};

// Next chain position after a record at p: the record end, clipped at the next message start.
__device__ __forceinline__ int next_pos(const uint8_t* d, const SubTile& st, int p) {
  int np = p + record_len(d, p);
  const int k = p - st.s + 1;
  const uint64_t after = k < 64 ? (st.msw >> k) : 0;
  const int nm = after ? p + 1 + lowest_bit(after) : st.nms_after;
  return np < nm ? np : nm;
}

// Walks from p (inside the sub-tile) marking record starts until the chain leaves the sub-tile
// or reaches a position of `stop`.  Returns the position reached.
__device__ __forceinline__ int walk(const uint8_t* d, const SubTile& st, int p, uint64_t stop,
                                    uint64_t* marks, uint64_t* runs = nullptr) {
  uint64_t m = 0, rm = 0;
  while (p < st.vend) {
    const uint64_t bit = 1ull << (p - st.s);
    m |= bit;
    const uint32_t tag = d[p];
    if (tag == 0 || tag == 0xff) rm |= bit;
    p = next_pos(d, st, p);
    if (p < st.vend && ((stop >> (p - st.s)) & 1)) break;
  }
  *marks = m;
  if (runs) *runs = rm;
  if (p >= st.pend) return kDead;
  return p;
}

// Lane-entry fixed point for a tile entry E.  In: spec chain (chain, sx).  In/out: e (entries).
// Out: true record-start mask of the lane and its exit.
__device__ __forceinline__ void resolve(const uint8_t* d, const SubTile& st, uint64_t chain,
                                        int sx, int E, int& e, uint64_t& tm, int& out,
                                        uint64_t& runm) {
  const int l = lane_id();
  for (int iter = 0; iter < 80; iter++) {
    if (e >= st.end || e >= st.pend) {
      out = e >= st.pend ? kDead : e;
      tm = 0;
    } else if ((chain >> (e - st.s)) & 1) {
      out = sx;
      tm = chain & ~mask_lt(e - st.s);
    } else {
      uint64_t wm, wr;
      const int p = walk(d, st, e, chain, &wm, &wr);
      runm |= wr;
      if (p != kDead && p < st.vend) {
        out = sx;
        tm = wm | (chain & ~mask_lt(p - st.s));
      } else {
        out = p;
        tm = wm;
      }
    }
    const uint32_t incl = wave_incl_max32((uint32_t)out);
    const int prev = (int)shfl32(incl, l > 0 ? l - 1 : 0);
    const int en = l == 0 ? E : (prev > E ? prev : E);
    if (!ballot(en != e)) break;
    e = en;
  }
}

// Position of the k-th set bit of m (k < popcount(m)).
__device__ __forceinline__ int select_bit(uint64_t m, int k) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t low = m & ((1ull << w) - 1);
    const int c = __popcll(low);
    if (k >= c) {
      k -= c;
      m >>= w;
      pos += w;
    } else {
      m = low;
    }
  }
  return pos;
}

// Record r's tile position from the per-lane true masks (R = exclusive record prefix by lane).
__device__ __forceinline__ int record_pos(uint32_t R, uint64_t tm, uint32_t r) {
  int j = 0;
#pragma unroll
  for (int step = 32; step >= 1; step >>= 1) {
    const int c = j + step;
    const uint32_t Rc = shfl32(R, c <= 63 ? c : 63);
    if (c <= 63 && Rc <= r) j = c;
  }
  const uint32_t Rj = shfl32(R, j);
  const uint64_t mj = shfl64(tm, j);
  return 64 * j + select_bit(mj, (int)(r - Rj));
}

struct Rec {
  uint32_t tag;
  int hb;       // tag + data bytes
  uint32_t cnt; // run count (0 unless tag 0x00 / 0xff and the count byte is in range)
  bool run;
};

__device__ __forceinline__ Rec read_rec(const uint8_t* d, int p) {
  Rec r;
  r.tag = d[p];
  r.hb = 1 + __popc(r.tag);
  r.run = r.tag == 0 || r.tag == 0xff;
  r.cnt = r.run ? d[p + r.hb] : 0;
  return r;
}

// 8 bytes at any LDS offset q: three aligned dword reads + byte funnel shifts.
__device__ __forceinline__ uint64_t read8(const uint8_t* d, int q) {
  const uint32_t* w = (const uint32_t*)(d + (q & ~3));
  const uint32_t sh = q & 3;
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
  return ((uint64_t)hi << 32) | lo;
}

// v_perm selector that deposits the first popc(n) bytes of its source into the byte lanes of
// nibble n (byte i <- source byte rank_i when bit i is set, else 0): the inverse of the tag
// compaction (serialize-packed.c++:105-119).
__device__ __forceinline__ uint32_t deposit_sel(uint32_t n) {
  uint32_t sel = 0, r = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const bool b = (n >> i) & 1;
    sel |= (b ? r : 0x0cu) << (8 * i);
    r += b;
  }
  return sel;
}

// Expands a record's word from the staged bytes following its tag (two v_perm_b32).
__device__ __forceinline__ uint64_t expand_word(const uint8_t* d, int p, uint32_t tag,
                                                uint32_t lut) {
  const uint64_t data = read8(d, p + 1);
  const uint32_t tl = tag & 15, th = tag >> 4;
  const uint32_t sl = shfl32(lut, (int)tl), sh = shfl32(lut, (int)th);
  const uint32_t lo = __builtin_amdgcn_perm((uint32_t)(data >> 32), (uint32_t)data, sl);
  const uint64_t d2 = data >> (8 * __popc(tl));
  const uint32_t hi = __builtin_amdgcn_perm((uint32_t)(d2 >> 32), (uint32_t)d2, sh);
  return ((uint64_t)hi << 32) | lo;
}

struct MsgInfo {
  uint64_t base, total, end;  // word offset, flat words, packed end (absolute byte)
  bool ok, fits;
};

__device__ __forceinline__ MsgInfo msg_info(const UnpackArgs& a, uint64_t m) {
  MsgInfo mi;
  if (!a.word_off) {  // size-only mode
    mi.base = 0;
    mi.total = ~0ull >> 2;
    mi.end = a.in_off[m + 1];
    mi.ok = true;
    mi.fits = false;
    return mi;
  }
  mi.base = a.word_off[m];
  mi.total = a.word_off[m + 1] - mi.base;
  mi.end = a.in_off[m + 1];
  mi.ok = a.hdr_status ? a.hdr_status[m] == kOK : true;
  mi.fits = mi.base + mi.total <= a.words_capacity;
  return mi;
}

// Checks + main word for one record (lane).  wb = words of the message before this record.
// Returns the record's terminal status (or -1), and the run still to be written (run_n words
// at run_dst, raw source run_src or zeros).
struct RunJob {
  uint64_t dst, src;
  uint32_t n;
  bool raw;
  uint64_t end;  // absolute packed byte after this record (terminal records: message end)
};

__device__ __forceinline__ int32_t handle_record(const UnpackArgs& a, const uint8_t* d, int p,
                                                 uint64_t pabs, uint64_t wb, const MsgInfo& mi,
                                                 RunJob* job, uint64_t word) {
  job->n = 0;
  job->dst = job->src = 0;
  job->raw = false;
  const Rec r = read_rec(d, p);
  const uint64_t mend = mi.end;
  if (a.mode == 2) {
    // computeUnpackedSizeInWords (serialize-packed.c++:487-505) bounds checks, incl. its
    // `end - ptr >= count` test that admits a record whose last data byte is missing.
    if (mend - pabs < (uint64_t)(r.hb - 1)) return kInvalid;
    uint64_t ptr = pabs + r.hb;
    if (r.run) {
      if (!(ptr < mend)) return kInvalid;
      ptr += 1;
      if (r.tag == 0xff) {
        if (mend - ptr < 8ull * r.cnt) return kInvalid;
        ptr += 8ull * r.cnt;
      }
    }
    return ptr >= mend ? kSizeDone : -1;  // terminal: words = wb + 1 + count (caller)
  }
  if (!mi.ok || wb >= mi.total) return -1;
  int32_t st = -1;
  const bool trunc1 = pabs + r.hb > mend;
  const bool trunc2 = !trunc1 && r.run && pabs + r.hb >= mend;
  uint64_t end = pabs + r.hb;
  uint32_t cnt = (trunc1 || trunc2) ? 0 : r.cnt;
  bool trunc3 = false, over = false;
  if (trunc1 || trunc2) {
    st = kEOF;
  } else if (r.run) {
    end += 1;
    if (wb + 1 + cnt > mi.total) {
      over = true;
      st = kOvershoot;
    } else if (r.tag == 0xff) {
      end += 8ull * cnt;
      if (end > mend) {
        trunc3 = true;
        st = kEOF;
      }
    }
  }
  job->end = end;
  if (st < 0) {
    if (wb + 1 + cnt == mi.total) st = end < mend ? kTrailing : kOK;
    else if (end >= mend) st = kEOF;
  }
  if (st == kOK && !mi.fits) st = kCap;
  if (mi.fits && !trunc1) {
    a.words[mi.base + wb] = word;
    uint64_t n = cnt;
    if (over) n = mi.total - wb - 1;
    if (trunc3) {
      const uint64_t avail = (mend - (pabs + r.hb + 1)) / 8;
      n = n < avail ? n : avail;
    }
    if (n) {
      job->n = (uint32_t)n;
      job->dst = mi.base + wb + 1;
      job->raw = r.tag == 0xff;
      job->src = pabs + r.hb + 1;
    }
  }
  return st;
}

// Writes the pending runs of a batch with the whole wave (coalesced).
__device__ __forceinline__ void run_jobs(const UnpackArgs& a, const RunJob& job) {
  uint64_t pend = ballot(job.n != 0);
  const int l = lane_id();
  while (pend) {
    const int j = lowest_bit(pend);
    pend &= pend - 1;
    const uint32_t n = readlane32(job.n, j);
    const uint64_t dst = readlane64(job.dst, j);
    const uint64_t src = readlane64(job.src, j);
    const bool raw = readlane32(job.raw, j);
    for (uint32_t k = l; k < n; k += 64) {
      uint64_t v = 0;
      if (raw) {
        const uint64_t s = src + 8ull * k;
        const uint64_t al = s & ~7ull;
        const uint32_t sh = (uint32_t)(s & 7);
        if (al + 16 <= a.nbytes) {
          const uint64_t v0 = *(const uint64_t*)(a.packed + al);
          const uint64_t v1 = *(const uint64_t*)(a.packed + al + 8);
          v = sh ? (v0 >> (8 * sh)) | (v1 << (64 - 8 * sh)) : v0;
        } else {
          v = load_u64_unaligned(a.packed + s);
        }
      }
      a.words[dst + k] = v;
    }
  }
}

__device__ __forceinline__ void flag_message(const UnpackArgs& a, uint64_t m) {
  if (atomicExch(a.fail_flag + m, 1u) == 0) {
    const uint32_t i = atomicAdd(a.fail_count, 1u);
    a.fail_list[i] = (uint32_t)m;
  }
}

// Per-tile window of message metadata: lane i describes message mw + i.
struct MsgWin {
  int64_t mw;        // message of lane 0 (may be -1 / past the end: empty entries)
  uint64_t start;    // in_off[m]          (~0 for missing entries)
  uint64_t end;      // in_off[m + 1]
  uint64_t base;     // word_off[m]
  uint64_t total;    // word_off[m + 1] - word_off[m]
  uint32_t ok;       // header accepted
};

__device__ __forceinline__ void load_win(const UnpackArgs& a, int64_t mw, MsgWin& w) {
  const int64_t m = mw + lane_id();
  w.mw = mw;
  if (m >= 0 && (uint64_t)m < a.nmsgs) {
    w.start = a.in_off[m];
    w.end = a.in_off[m + 1];
    if (a.word_off) {
      w.base = a.word_off[m];
      w.total = a.word_off[m + 1] - w.base;
    } else {
      w.base = 0;
      w.total = ~0ull >> 2;
    }
    w.ok = a.hdr_status ? a.hdr_status[m] == kOK : 1;
  } else {
    w.start = ~0ull;
    w.end = ~0ull;
    w.base = 0;
    w.total = 0;
    w.ok = 0;
  }
}

// Stages packed bytes [A, A + kB + kPad) of the batch into d (zero past the end).
__device__ __forceinline__ void stage_tile(const UnpackArgs& a, uint64_t A, uint8_t* d) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const int l = lane_id();
  const uint64_t P = a.nbytes;
  const bool aligned = ((uintptr_t)a.packed & 15) == 0;
#pragma unroll
  for (int k = 0; k < (kB + kPad) / 1024 + 1; k++) {
    const int o = 16 * (64 * k + l);
    if (o < kB + kPad) {
      u32x4 v = {0, 0, 0, 0};
      if (aligned && A + o + 16 <= P) {
        v = *(const u32x4*)(a.packed + A + o);
      } else {
        uint8_t tmp[16];
        for (int i = 0; i < 16; i++) tmp[i] = (A + o + i < P) ? a.packed[A + o + i] : 0;
        v = *(const u32x4*)tmp;
      }
      *(u32x4*)(d + o) = v;
    }
  }
}

// v_perm selectors depositing the bytes that follow a tag into the word: byte i <- data byte
// rank_i when bit i of the tag is set, else 0 (the inverse of serialize-packed.c++:332-350).
__device__ __forceinline__ uint64_t make_dep(uint32_t tag) {
  uint64_t sel = 0;
  uint32_t r = 0;
  for (int i = 0; i < 8; i++) {
    const bool b = (tag >> i) & 1;
    sel |= (uint64_t)(b ? r : 0x0cu) << (8 * i);
    r += b;
  }
  return sel;
}

// A tile whose look-back and expansion are deferred (see body_kernel).
struct PendTile {
  uint64_t t, A, mfirst, mlast, agg;
  bool on, tile_has_start;
};

// 3. Body: one wave per 4 KiB tile, persistent waves over a static strided tile order.
//   phase 1  stage, message starts, speculative walks, entries (published spec exit, the
//            predecessor's exit), per-lane record masks, the tile's word count -> publish
//   phase 2  (deferred until the wave's next tile has done phase 1, so the look-back has a
//            whole phase to resolve) look-back, re-stage (L2), record list, expansion.
template <bool STAMPS>
__global__ __launch_bounds__(256) void body_kernel(UnpackArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_data[4][kB + kPad];
  __shared__ uint64_t lds_ms[4][64];
  __shared__ uint16_t lds_list[4][kB / 4];  // record positions of half a tile (<= 1024)
  __shared__ uint64_t dep_tab[256];
  const int l = lane_id();
  const int wv = (int)uniform32(threadIdx.x >> 6);  // wave-uniform (keeps tile math scalar)
  uint8_t* d = lds_data[wv];
  uint16_t* list = lds_list[wv];
  dep_tab[threadIdx.x] = make_dep(threadIdx.x);
  __syncthreads();
  const uint32_t lut = deposit_sel((uint32_t)l & 15);
  const uint64_t P = a.nbytes;

  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  Stamps<STAMPS> stm;
  PendTile pend;
  pend.on = false;
  uint64_t ptm = 0, pmsw = 0;  // pending tile: this lane's record-start and message-start bits

  // ---------------------------------------------------------------- phase 2 of a pending tile
  auto finish = [&](const PendTile& pt, uint64_t tm, uint64_t msw) {
    const uint64_t A = pt.A;
    uint64_t excl = 0;
    if (!(a.debug_skip & 1)) {
      excl = lookback2(a.desc, a.gdesc, pt.t, kSegBit, a.err);
      publish_incl(a.desc, a.gdesc, pt.t, a.ntiles, pt.tile_has_start ? pt.agg : excl + pt.agg);
    }
    stage_tile(a, A, d);
    lds_ms[wv][l] = msw;
    MsgWin win;
    load_win(a, (int64_t)pt.mfirst - 1, win);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    // Fast expansion when every message touching the tile is in the window, has a valid
    // header, fits the output, and no two messages start at the same byte.
    bool fast = a.mode == 0 && pt.mlast - (pt.mfirst - 1) <= 63 && a.word_off;
    if (fast) {
      const int64_t m = win.mw + l;
      const bool inrange = m >= 0 && (uint64_t)m < pt.mlast;
      const bool bad = inrange && (!win.ok || win.base + win.total > a.words_capacity);
      const uint64_t nxs = shfl64(win.start, l < 63 ? l + 1 : 63);
      const bool dup = inrange && l < 63 && (uint64_t)(m + 1) < pt.mlast && nxs == win.start;
      fast = ballot(bad || dup) == 0;
    }
    const uint32_t cnt_all = __popcll(tm);
    const uint32_t Rall_incl = wave_incl_sum32(cnt_all);
    const uint32_t nrec = readlane32(Rall_incl, 63);
    const uint32_t nfirst = readlane32(Rall_incl, 31);
    if (nfirst > kB / 4 || nrec - nfirst > kB / 4) fast = false;  // list capacity (1-byte records)
    if (!fast) {
      // general path: one lane per record, record positions by binary search, message of each
      // record from the window (see handle_record for the reference checks)
      const uint32_t R = Rall_incl - cnt_all;
      const uint64_t* msw_all = lds_ms[wv];
      int64_t mcur = (int64_t)pt.mfirst - 1;
      uint64_t nxt_start = readlane64(win.start, 1);
      uint64_t sum = 0;
      uint32_t base_key = 0;
      for (uint32_t b0 = 0; b0 < nrec; b0 += 64) {
        const uint32_t r = b0 + l;
        const bool act = r < nrec;
        const int rp = record_pos(R, tm, act ? r : 0);
        const int p = act ? rp : 0;
        const uint64_t pabs = A + p;
        const Rec rc = read_rec(d, p);
        const uint32_t w = act ? 1 + rc.cnt : 0;
        const bool is_ms = act && ((msw_all[p >> 6] >> (p & 63)) & 1);
        const uint32_t inc = wave_incl_sum32(w);
        const uint64_t Sx = sum + inc - w;
        const uint32_t key = is_ms ? (uint32_t)(Sx + 1) : 0;
        uint32_t km = wave_incl_max32(key);
        if (km < base_key) km = base_key;
        const uint64_t wb = km ? Sx - (km - 1) : excl + Sx;
        const uint32_t lastl = (nrec - b0 < 64 ? nrec - b0 : 64) - 1;
        const uint64_t maxp = readlane64(pabs, (int)lastl);
        int64_t m = mcur;
        if (maxp >= nxt_start) {
          bool found = false;
          for (;;) {
            int c = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1) {
              const uint64_t probe = shfl64(win.start, c + step <= 63 ? c + step : 63);
              if (c + step <= 63 && probe <= pabs) c += step;
            }
            const bool beyond = act && c == 63 && readlane64(win.start, 63) <= pabs;
            if (!found && !beyond) m = win.mw + c;
            found = found || !beyond;
            if (!ballot(beyond)) break;
            load_win(a, win.mw + 63, win);
          }
          mcur = (int64_t)readlane64((uint64_t)m, (int)lastl);
          if (mcur - win.mw >= 63) load_win(a, mcur, win);
          nxt_start = readlane64(win.start, (int)(mcur - win.mw) + 1);
        }
        const int64_t wl64 = m - win.mw;
        const bool inwin = wl64 >= 0 && wl64 < 64;
        const int wl = inwin ? (int)wl64 : 0;
        MsgInfo mi;
        mi.base = shfl64(win.base, wl);
        mi.total = shfl64(win.total, wl);
        mi.end = shfl64(win.end, wl);
        mi.ok = shfl32(win.ok, wl) != 0;
        if (!inwin && act && m >= 0 && (uint64_t)m < a.nmsgs) mi = msg_info(a, (uint64_t)m);
        mi.fits = a.word_off ? (mi.base + mi.total <= a.words_capacity) : false;
        const uint64_t word = expand_word(d, p, rc.tag, lut);
        RunJob job;
        job.n = 0;
        if (act && m >= 0 && (uint64_t)m < a.nmsgs) {
          const int32_t st = handle_record(a, d, p, pabs, wb, mi, &job, word);
          if (a.mode == 2) {
            if (st == kInvalid) {
              a.status[m] = kInvalid;
              a.size_out[m] = 0;
            } else if (st == kSizeDone) {
              a.status[m] = kOK;
              a.size_out[m] = wb + 1 + (rc.run ? rc.cnt : 0);
            }
          } else if (st >= 0) {
            a.status[m] = st;
            if (a.in_end && (st == kOK || st == kTrailing || st == kCap)) a.in_end[m] = job.end;
          }
        }
        run_jobs(a, job);
        base_key = readlane32(km, 63);
        sum += readlane32(inc, 63);
      }
      return;
    }
    // fast path: record list per half tile (lanes 0-31, then 32-63), 64 records per batch
    uint64_t sum = 0;        // words of the tile's records so far
    uint32_t base_key = 0;   // key of the latest message start so far (key-max reset)
    uint32_t mcount = 0;     // message starts so far
    for (int h = 0; h < 2; h++) {
      const bool mine = (l >> 5) == h;
      uint64_t bits = mine ? tm : 0;
      const uint32_t c = __popcll(bits);
      const uint32_t Rin = wave_incl_sum32(c);
      const uint32_t nh = readlane32(Rin, 63);
      uint32_t r = Rin - c;
      while (bits) {
        const int b = lowest_bit(bits);
        bits &= bits - 1;
        const uint32_t ms = (uint32_t)((msw >> b) & 1);
        list[r++] = (uint16_t)((64 * l + b) | (ms << 12));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (uint32_t b0 = 0; b0 < nh; b0 += 64) {
        const uint32_t rr = b0 + l;
        const bool act = rr < nh;
        const uint32_t e = act ? list[rr] : 0;
        const int p = (int)(e & 0xfff);
        const bool is_ms = act && ((e >> 12) & 1);
        // bytes p .. p + 12: tag, up to 8 data bytes, count byte
        const uint32_t* dw = (const uint32_t*)(d + (p & ~3));
        const uint32_t sh = (uint32_t)p & 3;
        const uint32_t q0 = dw[0], q1 = dw[1], q2 = dw[2], q3 = dw[3];
        const uint32_t b0w = __builtin_amdgcn_alignbyte(q1, q0, sh);  // bytes p .. p+3
        const uint32_t b1w = __builtin_amdgcn_alignbyte(q2, q1, sh);  // p+4 .. p+7
        const uint32_t b2w = __builtin_amdgcn_alignbyte(q3, q2, sh);  // p+8 .. p+11
        const uint32_t tag = b0w & 0xff;
        const uint32_t dlo = __builtin_amdgcn_alignbyte(b1w, b0w, 1);  // data bytes 0..3
        const uint32_t dhi = __builtin_amdgcn_alignbyte(b2w, b1w, 1);  // data bytes 4..7
        const uint32_t nz = __popc(tag);
        const bool z = tag == 0, f = tag == 0xff;
        const uint32_t cnt = act ? (z ? ((b0w >> 8) & 0xff) : (f ? ((b2w >> 8) & 0xff) : 0u)) : 0u;
        const uint32_t w = act ? 1 + cnt : 0;
        const uint32_t inc = wave_incl_sum32(w);
        const uint64_t Sx = sum + inc - w;
        const uint32_t key = is_ms ? (uint32_t)(Sx + 1) : 0;
        uint32_t km = wave_incl_max32(key);
        if (km < base_key) km = base_key;
        const uint64_t wb = km ? Sx - (km - 1) : excl + Sx;
        const uint64_t msb = ballot(is_ms);
        const int wl = (int)(mcount + (uint32_t)__popcll(msb & mask_le(l)));  // window lane
        const uint64_t mbase = shfl64(win.base, wl);
        const uint64_t mtotal = shfl64(win.total, wl);
        const uint64_t mend = shfl64(win.end, wl);
        const uint64_t sel = dep_tab[tag];
        const uint32_t wlo = __builtin_amdgcn_perm(dhi, dlo, (uint32_t)sel);
        const uint32_t whi = __builtin_amdgcn_perm(dhi, dlo, (uint32_t)(sel >> 32));
        const uint64_t word = ((uint64_t)whi << 32) | wlo;
        const uint32_t len = 1 + nz + ((z || f) ? 1 + (f ? 8 * cnt : 0) : 0);
        const uint64_t pabs = A + p;
        // records that end a message (or break it) go through the reference checks
        const bool special = act && (wb + w >= mtotal || pabs + len >= mend);
        RunJob job;
        job.n = 0;
        if (act && !special) {
          a.words[mbase + wb] = word;
          if (cnt) {
            job.n = cnt;
            job.dst = mbase + wb + 1;
            job.raw = f;
            job.src = pabs + 10;
          }
        } else if (special) {
          MsgInfo mi;
          mi.base = mbase;
          mi.total = mtotal;
          mi.end = mend;
          mi.ok = true;
          mi.fits = true;
          const int64_t m = win.mw + wl;
          const int32_t st = handle_record(a, d, p, pabs, wb, mi, &job, word);
          if (st >= 0) {
            a.status[m] = st;
            if (a.in_end && (st == kOK || st == kTrailing || st == kCap)) a.in_end[m] = job.end;
          }
        }
        run_jobs(a, job);
        base_key = readlane32(km, 63);
        sum += readlane32(inc, 63);
        mcount += (uint32_t)__popcll(msb);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };

  for (uint64_t t = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv; t < a.ntiles; t += nwaves) {
  stm.start(a.stamps);
  const uint64_t A = t * kB;

  // ---- stage bytes [A, A + kB + kPad) -------------------------------------------------------
  stage_tile(a, A, d);
  // ---- message window (lane 0 = message holding byte A) and message-start bitmap --------------
  const uint64_t mfirst = a.tile_first[t];
  MsgWin win;
  load_win(a, (int64_t)mfirst - 1, win);
  lds_ms[wv][l] = 0;
  uint64_t mlast;                     // one past the last message starting in [A, A + kB)
  int nms_tile_after;                 // first message start >= A + kB (tile-relative)
  {
    MsgWin w2 = win;
    for (;;) {
      const bool in = l > 0 && w2.start >= A && w2.start < A + kB;
      if (in) {
        const uint64_t r = w2.start - A;
        atomicOr((unsigned long long*)&lds_ms[wv][r >> 6], 1ull << (r & 63));
      }
      const uint64_t inm = ballot(in);
      if (inm != (~0ull << 1)) {
        const int c = __popcll(inm);
        mlast = (uint64_t)(w2.mw + 1 + c);
        const uint64_t nx = mlast < a.nmsgs ? uniform64(a.in_off[mlast]) : P;
        nms_tile_after = (int)((nx < P ? nx : P) - A);
        break;
      }
      load_win(a, w2.mw + 63, w2);  // 63 starts in this window: continue with the next
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (P - A < (uint64_t)kB) {
    const int pe = (int)(P - A);
    atomicOr((unsigned long long*)&lds_ms[wv][pe >> 6], 1ull << (pe & 63));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  stm.mark(0);  // staging + message window
  SubTile st;
  st.s = 64 * l;
  st.end = st.s + 64;
  st.pend = (int)(P - A) < kDead ? (int)(P - A) : kDead;
  st.vend = st.end < st.pend ? st.end : st.pend;
  st.msw = lds_ms[wv][l];
  {
    // first message start in a later sub-tile (suffix min over lanes)
    const int fs = st.msw ? st.s + lowest_bit(st.msw) : 0x7fffffff;
    int v = fs;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
      const int o = (int)shfl32((uint32_t)v, l + dd <= 63 ? l + dd : l);
      if (l + dd <= 63) v = o < v ? o : v;
    }
    const int nxt = (int)shfl32((uint32_t)v, l < 63 ? l + 1 : 63);
    st.nms_after = (l < 63 && nxt != 0x7fffffff) ? nxt : nms_tile_after;
  }

  // ---- speculative chains per sub-tile -------------------------------------------------------
  uint64_t chain = 0, runm = 0;
  int sx = kDead;
  if (st.s < st.pend) sx = walk(d, st, st.s, 0, &chain, &runm);

  stm.mark(1);  // speculative walks
  // ---- tile entry: speculative (first byte) then true (predecessor's published exit) ---------
  const bool a_is_start = lds_ms[wv][0] & 1;
  int e = l == 0 ? 0 : st.s;
  uint64_t tm = 0;
  int out = 0;
  resolve(d, st, chain, sx, 0, e, tm, out, runm);
  const int spec_exit = (int)readlane32((uint32_t)out, 63);
  if (l == 0) {
    const uint32_t enc = spec_exit >= kDead ? 0xffffu : (uint32_t)(spec_exit - kB);
    store_agent32(a.state + t, 0x80000000u | enc);
  }
  stm.mark(2);  // spec resolve + publish
  if (!a_is_start && t > 0) {
    const uint32_t v = wait_nonzero32(a.state + t - 1, a.err);
    const int E = (v & 0xffffu) == 0xffffu ? kDead : (int)(v & 0xffffu);
    if (E != 0) {
      if (l == 0) e = E;
      resolve(d, st, chain, sx, E, e, tm, out, runm);
    }
  }
  {
    // the exit published above must be the true one whenever the successor starts mid-message
    const int true_exit = (int)readlane32((uint32_t)out, 63);
    const bool next_is_start = nms_tile_after == kB;
    if (true_exit != spec_exit && !next_is_start && A + kB < P) {
      if (l == 0) flag_message(a, mlast - 1);
    }
  }

  stm.mark(3);  // entry wait + true resolve
  // ---- tile aggregate: words per lane, segmented by message starts ---------------------------
  const uint32_t cnt = __popcll(tm);
  uint64_t w_all = cnt, w_post = 0;
  bool has_ms = false;
  {
    uint64_t rr = tm & runm;
    const uint64_t msin = tm & st.msw;  // message starts that are records of this lane
    const int lastms = highest_bit(msin);
    has_ms = lastms >= 0;
    if (has_ms) w_post = __popcll(tm & ~mask_lt(lastms));
    while (rr) {
      const int b = lowest_bit(rr);
      rr &= rr - 1;
      const int p = st.s + b;
      const uint32_t tag = d[p];
      const uint32_t c = d[p + 1 + __popc(tag)];
      w_all += c;
      if (has_ms && b >= lastms) w_post += c;
    }
  }
  uint64_t agg;
  bool tile_has_start;
  {
    const uint64_t hm = ballot(has_ms);
    tile_has_start = hm != 0;
    const int lm = highest_bit(hm);
    // words after the last message start = w_post of that lane + w_all of later lanes
    const uint64_t contrib = (!tile_has_start || l > lm) ? w_all : (l == lm ? w_post : 0);
    agg = wave_sum64(contrib);
  }
  const uint64_t agg_desc = tile_has_start ? (kSegBit | agg) : agg;
  if (!(a.debug_skip & 1))
    publish_agg(a.desc, a.gdesc, a.gcnt, t, a.ntiles, agg_desc, kSegBit, a.err);
  stm.mark(4);  // aggregate

  // ---- phase 2 of the previous tile, then this tile becomes the pending one ----------------
  if (pend.on) finish(pend, ptm, pmsw);
  pend.t = t;
  pend.A = A;
  pend.mfirst = mfirst;
  pend.mlast = mlast;
  pend.agg = agg;
  pend.tile_has_start = tile_has_start;
  pend.on = true;
  ptm = tm;
  pmsw = st.msw;
  stm.mark(5);  // deferred look-back + expansion
  if (STAMPS && l == 0 && a.stamps) atomicAdd(a.stamps + 15, 1ull);
  }  // tile loop
  if (pend.on) finish(pend, ptm, pmsw);
}

// Serial re-decode of flagged messages: lane 0 walks the records of a 4 KiB window, then the
// wave expands them with the same record handler as body_kernel.
__global__ __launch_bounds__(64) void fallback_kernel(UnpackArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t d[kB + kPad];
  __shared__ uint16_t rpos[kB];
  __shared__ uint64_t rwb[kB];
  __shared__ int sh_n, sh_adv;
  const int l = lane_id();
  const uint32_t lut = deposit_sel((uint32_t)l & 15);
  const uint32_t nfail = *a.fail_count;
  for (uint32_t fi = blockIdx.x; fi < nfail; fi += gridDim.x) {
    const uint64_t m = a.fail_list[fi];
    const MsgInfo mi = msg_info(a, m);
    if (!mi.ok) continue;
    uint64_t pos = a.in_off[m];
    const uint64_t mend = mi.end;
    uint64_t wb = 0;
    bool done = false;
    while (!done && pos < mend) {
      for (int o = l; o < kB + kPad; o += 64) d[o] = (pos + o < mend) ? a.packed[pos + o] : 0;
      __syncthreads();
      if (l == 0) {
        int p = 0, n = 0;
        uint64_t w = wb;
        while (p < kB && pos + p < mend) {
          rpos[n] = (uint16_t)p;
          rwb[n] = w;
          n++;
          const Rec rc = read_rec(d, p);
          w += 1 + rc.cnt;
          p += rc.hb + (rc.run ? 1 : 0) + (rc.tag == 0xff ? 8 * (int)rc.cnt : 0);
          if (w >= mi.total) break;
        }
        sh_n = n;
        sh_adv = p;
      }
      __syncthreads();
      const int n = sh_n;
      for (int b0 = 0; b0 < n; b0 += 64) {
        const int r = b0 + l;
        RunJob job;
        job.n = 0;
        const int pp = r < n ? rpos[r] : 0;
        const uint64_t word = expand_word(d, pp, d[pp], lut);
        if (r < n) {
          const int p = pp;
          const uint64_t w0 = rwb[r];
          if (a.mode == 2) {
            const int32_t s = handle_record(a, d, p, pos + p, w0, mi, &job, word);
            if (s == kInvalid) {
              a.status[m] = kInvalid;
              a.size_out[m] = 0;
              done = true;
            } else if (s == kSizeDone) {
              const Rec rc = read_rec(d, p);
              a.status[m] = kOK;
              a.size_out[m] = w0 + 1 + (rc.run ? rc.cnt : 0);
              done = true;
            }
          } else {
            const int32_t s = handle_record(a, d, p, pos + p, w0, mi, &job, word);
            if (s >= 0) {
              a.status[m] = s;
              if (a.in_end && (s == kOK || s == kTrailing || s == kCap)) a.in_end[m] = job.end;
              done = true;
            }
          }
        }
        run_jobs(a, job);
      }
      done = ballot(done) != 0;
      if (n > 0) {
        const Rec rc = read_rec(d, rpos[n - 1]);
        wb = rwb[n - 1] + 1 + rc.cnt;
      }
      pos += (uint64_t)sh_adv;
      __syncthreads();
    }
  }
}

// Status before any record is seen (buffers with no records keep it): flat-packed chunks read
// exactly word_off[m+1]-word_off[m] words; size-only buffers start at 0 words.
__global__ void init_kernel(uint32_t mode, const uint64_t* __restrict__ in_off,
                            const uint64_t* __restrict__ word_off, uint64_t n,
                            int32_t* __restrict__ status, uint64_t* __restrict__ size_out) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const bool empty = in_off[m + 1] == in_off[m];
  if (mode == 2) {
    status[m] = kOK;
    size_out[m] = 0;
  } else {
    const bool zero = word_off[m + 1] == word_off[m];
    status[m] = zero ? (empty ? kOK : kTrailing) : kEOF;
  }
}

}  // namespace

hipError_t launch_unpack_init(uint32_t mode, const uint64_t* in_off, const uint64_t* word_off,
                              uint64_t n, int32_t* status, uint64_t* size_out,
                              hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, mode,
                     in_off, word_off, n, status, size_out);
  return hipGetLastError();
}

hipError_t launch_unpack_header(const uint8_t* packed, const uint64_t* in_off, uint64_t n,
                                uint64_t limit, uint64_t* flat, int32_t* hdr_status,
                                int32_t* status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(header_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     packed, in_off, n, limit, flat, hdr_status, status);
  return hipGetLastError();
}

hipError_t launch_unpack_body(const UnpackArgs& a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  static const unsigned cap = resident_blocks((const void*)body_kernel<false>, 256, 0);
  const uint64_t want = (a.ntiles + 3) / 4;
  const unsigned blocks = (unsigned)(want < cap ? want : cap);
  if (a.stamps)
    hipLaunchKernelGGL(body_kernel<true>, dim3(blocks), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(body_kernel<false>, dim3(blocks), dim3(256), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fallback_kernel, dim3(256), dim3(64), 0, stream, a);
  return hipGetLastError();
}

}  // namespace cpk
