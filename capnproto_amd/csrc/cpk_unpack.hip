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
                                    uint64_t* marks) {
  uint64_t m = 0;
  while (p < st.vend) {
    m |= 1ull << (p - st.s);
    p = next_pos(d, st, p);
    if (p < st.vend && ((stop >> (p - st.s)) & 1)) break;
  }
  *marks = m;
  if (p >= st.pend) return kDead;
  return p;
}

// Lane-entry fixed point for a tile entry E.  In: spec chain (chain, sx).  In/out: e (entries).
// Out: true record-start mask of the lane and its exit.
__device__ __forceinline__ void resolve(const uint8_t* d, const SubTile& st, uint64_t chain,
                                        int sx, int E, int& e, uint64_t& tm, int& out) {
  const int l = lane_id();
  for (int iter = 0; iter < 80; iter++) {
    if (e >= st.end || e >= st.pend) {
      out = e >= st.pend ? kDead : e;
      tm = 0;
    } else if ((chain >> (e - st.s)) & 1) {
      out = sx;
      tm = chain & ~mask_lt(e - st.s);
    } else {
      uint64_t wm;
      const int p = walk(d, st, e, chain, &wm);
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

// Expands a record's word from the staged bytes following its tag.
__device__ __forceinline__ uint64_t expand_word(const uint8_t* d, int p, uint32_t tag) {
  uint64_t w = 0;
  int k = p + 1;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t bit = (tag >> i) & 1;
    const uint64_t v = d[k];
    w |= bit ? (v << (8 * i)) : 0;
    k += (int)bit;
  }
  return w;
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
};

__device__ __forceinline__ int32_t handle_record(const UnpackArgs& a, const uint8_t* d, int p,
                                                 uint64_t pabs, uint64_t wb, const MsgInfo& mi,
                                                 RunJob* job) {
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
  if (st < 0) {
    if (wb + 1 + cnt == mi.total) st = end < mend ? kTrailing : kOK;
    else if (end >= mend) st = kEOF;
  }
  if (st == kOK && !mi.fits) st = kCap;
  if (mi.fits && !trunc1) {
    a.words[mi.base + wb] = expand_word(d, p, r.tag);
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

// 3. Body: one wave per 4 KiB tile.
__global__ __launch_bounds__(256) void body_kernel(UnpackArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_data[4][kB + kPad];
  __shared__ uint64_t lds_ms[4][64];
  const int l = lane_id();
  const int wv = threadIdx.x >> 6;
  uint8_t* d = lds_data[wv];

  uint32_t t32 = 0;
  if (l == 0) t32 = atomicAdd(a.tile_counter, 1u);
  const uint64_t t = uniform32(t32);
  if (t >= a.ntiles) return;
  const uint64_t A = t * kB;
  const uint64_t P = a.nbytes;
  const int pend = (int)((P - A) < (uint64_t)kB + 64 ? (P - A) : (uint64_t)kB + 64);

  // ---- stage bytes [A, A + kB + kPad) -------------------------------------------------------
  {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
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
  // ---- message starts inside the tile (+ batch end as a sentinel) ---------------------------
  const uint64_t mfirst = a.tile_first[t];
  lds_ms[wv][l] = 0;
  uint64_t mlast = mfirst;  // one past the last message starting in [A, A + kB)
  int nms_tile_after = (int)(P - A);  // first message start >= A + kB (tile-relative)
  {
    uint64_t m = mfirst;
    for (;;) {
      const uint64_t i = m + l;
      const uint64_t s = i <= a.nmsgs ? a.in_off[i] : ~0ull;
      const bool in = s < A + kB;
      if (in) atomicOr((unsigned long long*)&lds_ms[wv][(s - A) >> 6], 1ull << ((s - A) & 63));
      const uint64_t inm = ballot(in);
      const int c = __popcll(inm);
      m += c;
      if (c < 64) {
        const uint64_t nx = m <= a.nmsgs ? uniform64(a.in_off[m]) : P;
        nms_tile_after = (int)((nx < P ? nx : P) - A);
        break;
      }
    }
    mlast = m;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (P - A < (uint64_t)kB) {
    const int pe = (int)(P - A);
    atomicOr((unsigned long long*)&lds_ms[wv][pe >> 6], 1ull << (pe & 63));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  SubTile st;
  st.s = 64 * l;
  st.end = st.s + 64;
  st.pend = (int)(P - A) < kDead ? (int)(P - A) : kDead;
  st.vend = st.end < st.pend ? st.end : st.pend;
  st.msw = lds_ms[wv][l];
  {
    // first message start at or after the next sub-tile (suffix min over lanes)
    const int fs = st.msw ? st.s + lowest_bit(st.msw) : 0x7fffffff;
    int v = fs;
    // suffix min: reverse inclusive scan
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
      const int o = (int)shfl32((uint32_t)v, l + dd <= 63 ? l + dd : l);
      if (l + dd <= 63) v = o < v ? o : v;
    }
    const int nxt = (int)shfl32((uint32_t)v, l < 63 ? l + 1 : 63);
    st.nms_after = (l < 63 && nxt != 0x7fffffff) ? nxt : nms_tile_after;
  }
  (void)pend;

  // ---- speculative chains per sub-tile -------------------------------------------------------
  uint64_t chain = 0;
  int sx = kDead;
  if (st.s < st.pend) {
    sx = walk(d, st, st.s, 0, &chain);
  }

  // ---- tile entry: speculative (first byte) then true (predecessor's published exit) ---------
  const bool a_is_start = lds_ms[wv][0] & 1;
  int e = l == 0 ? 0 : st.s;
  uint64_t tm = 0;
  int out = 0;
  resolve(d, st, chain, sx, 0, e, tm, out);
  const int spec_exit = (int)readlane32((uint32_t)out, 63);
  if (l == 0) {
    const uint32_t enc = spec_exit >= kDead ? 0xffffu : (uint32_t)(spec_exit - kB);
    store_agent32(a.state + t, 0x80000000u | enc);
  }
  int E = 0;
  if (!a_is_start && t > 0) {
    const uint32_t v = wait_nonzero32(a.state + t - 1, a.err);
    E = (v & 0xffffu) == 0xffffu ? kDead : (int)(v & 0xffffu);
    if (E != 0) {
      if (l == 0) e = E;
      resolve(d, st, chain, sx, E, e, tm, out);
    }
  }
  // verification of the exit this tile published (matters only if the successor starts
  // mid-message)
  {
    const int true_exit = (int)readlane32((uint32_t)out, 63);
    const bool next_is_start = (uint64_t)nms_tile_after == (uint64_t)kB;
    if (true_exit != spec_exit && !next_is_start && A + kB < P) {
      // message containing byte A + kB
      if (l == 0) flag_message(a, mlast - 1);
    }
  }

  // ---- records: counts, segmented word sums (pass 1) ----------------------------------------
  const uint32_t cnt = __popcll(tm);
  const uint32_t Rincl = wave_incl_sum32(cnt);
  const uint32_t R = Rincl - cnt;
  const uint32_t nrec = readlane32(Rincl, 63);
  const uint64_t* msw_all = lds_ms[wv];

  uint64_t sum = 0;       // words of all previous records in the tile
  uint64_t base_key = 0;  // 1 + word sum at the last message start so far (0 = none)
  for (uint32_t b0 = 0; b0 < nrec; b0 += 64) {
    const uint32_t r = b0 + l;
    const bool act = r < nrec;
    const int rp = record_pos(R, tm, act ? r : 0);  // uniform shuffles
    const int p = act ? rp : 0;
    const Rec rc = read_rec(d, p);
    const uint32_t w = act ? 1 + rc.cnt : 0;
    const bool is_ms = act && ((msw_all[p >> 6] >> (p & 63)) & 1);
    const uint32_t inc = wave_incl_sum32(w);
    const uint64_t Sx = sum + inc - w;  // exclusive word sum at this record
    const uint32_t key = is_ms ? (uint32_t)(Sx + 1) : 0;
    const uint32_t km = wave_incl_max32(key);
    const uint64_t last_key = readlane32(km, 63);
    if (last_key) base_key = last_key;
    sum += readlane32(inc, 63);
  }
  const bool has_start = base_key != 0;
  const uint64_t agg = has_start ? (kSegBit | (sum - (base_key - 1))) : sum;

  // ---- segmented decoupled look-back ---------------------------------------------------------
  uint64_t excl = 0;
  if (t == 0) {
    if (l == 0) store_agent(a.desc, kDescIncl | agg);
  } else {
    if (l == 0) store_agent(a.desc + t, kDescAgg | agg);
    excl = lookback(a.desc, t, a.err, kSegBit);
    const uint64_t incl = has_start ? (agg & ~kSegBit) : excl + agg;
    if (l == 0) store_agent(a.desc + t, kDescIncl | incl);
  }

  // ---- pass 2: expansion ---------------------------------------------------------------------
  int64_t mcur = (int64_t)mfirst - 1;  // message of the previous record
  uint64_t nxt_start = uniform64(a.in_off[mfirst <= a.nmsgs ? mfirst : a.nmsgs]);
  sum = 0;
  base_key = 0;
  for (uint32_t b0 = 0; b0 < nrec; b0 += 64) {
    const uint32_t r = b0 + l;
    const bool act = r < nrec;
    const int rp = record_pos(R, tm, act ? r : 0);  // uniform shuffles
    const int p = act ? rp : 0;
    const uint64_t pabs = A + p;
    const Rec rc = read_rec(d, p);
    const uint32_t w = act ? 1 + rc.cnt : 0;
    const bool is_ms = act && ((msw_all[p >> 6] >> (p & 63)) & 1);
    const uint32_t inc = wave_incl_sum32(w);
    const uint64_t Sx = sum + inc - w;
    const uint32_t key = is_ms ? (uint32_t)(Sx + 1) : 0;
    uint32_t km = wave_incl_max32(key);
    if (km < base_key) km = (uint32_t)base_key;
    const uint64_t wb = km ? Sx - (km - 1) : excl + Sx;
    // message of each record: last m with in_off[m] <= pabs
    const uint32_t lastl = (nrec - b0 < 64 ? nrec - b0 : 64) - 1;
    const uint64_t maxp = readlane64(pabs, (int)lastl);
    int64_t m = mcur;
    if (maxp >= nxt_start) {
      uint64_t rank = 0;
      int64_t wbase = mcur;
      for (;;) {
        const int64_t i = wbase + 1 + l;
        const uint64_t sv = (uint64_t)i <= a.nmsgs ? a.in_off[i] : ~0ull;
        // count of window entries <= pabs (window sorted): binary search by shuffles
        int c = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1) {
          const uint64_t probe = shfl64(sv, c + step - 1);
          if (probe <= pabs) c += step;
        }
        if (shfl64(sv, c) <= pabs) c += 1;  // c <= 63 here; reaches 64 when all entries <= pabs
        rank += act ? c : 0;
        if (!ballot(act && c == 64)) break;
        wbase += 64;
      }
      m = mcur + (int64_t)rank;
      mcur = (int64_t)readlane64((uint64_t)m, (int)lastl);
      const uint64_t nm = (uint64_t)(mcur + 1);
      nxt_start = uniform64(nm <= a.nmsgs ? a.in_off[nm] : ~0ull);
    }
    RunJob job;
    job.n = 0;
    if (act && m >= 0 && (uint64_t)m < a.nmsgs) {
      const MsgInfo mi = msg_info(a, (uint64_t)m);
      if (a.mode == 2) {
        // size only
        const int32_t s = handle_record(a, d, p, pabs, wb, mi, &job);
        if (s == kInvalid) {
          a.status[m] = kInvalid;
          a.size_out[m] = 0;
        } else if (s == kSizeDone) {
          a.status[m] = kOK;
          a.size_out[m] = wb + 1 + (rc.run ? rc.cnt : 0);
        }
      } else {
        const int32_t s = handle_record(a, d, p, pabs, wb, mi, &job);
        if (s >= 0) a.status[m] = s;
      }
    }
    run_jobs(a, job);
    base_key = readlane32(km, 63);
    sum += readlane32(inc, 63);
  }
}

// Serial re-decode of flagged messages: lane 0 walks the records of a 4 KiB window, then the
// wave expands them with the same record handler as body_kernel.
__global__ __launch_bounds__(64) void fallback_kernel(UnpackArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t d[kB + kPad];
  __shared__ uint16_t rpos[kB];
  __shared__ uint64_t rwb[kB];
  __shared__ int sh_n, sh_adv;
  const int l = lane_id();
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
        if (r < n) {
          const int p = rpos[r];
          const uint64_t w0 = rwb[r];
          if (a.mode == 2) {
            const int32_t s = handle_record(a, d, p, pos + p, w0, mi, &job);
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
            const int32_t s = handle_record(a, d, p, pos + p, w0, mi, &job);
            if (s >= 0) {
              a.status[m] = s;
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
  hipLaunchKernelGGL(body_kernel, dim3((unsigned)((a.ntiles + 3) / 4)), dim3(256), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fallback_kernel, dim3(256), dim3(64), 0, stream, a);
  return hipGetLastError();
}

}  // namespace cpk
