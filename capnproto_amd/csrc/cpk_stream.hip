// cpk_stream.hip -- stream boundary discovery.
//
// A packed stream holds messages back to back with no index (a file or socket buffer written by
// repeated writePackedMessage; serialize-packed-test.c++:348-371 reads two of them from one
// stream).  Records never cross a message, so decoding the whole stream as one flat sequence of
// words (the unpack pipeline, with the byte of every record head kept in rec_pos) yields the
// messages' flat words back to back.  What is left is sequential by nature: message k+1 starts
// where the segment table of message k says message k ends (serialize.c++:202-242).  One wave
// follows that chain over the decoded words:
//   * a stretch of same-size single-segment messages (the common batch shape) is confirmed 64
//     messages per step -- lane j checks the header and both read boundaries of message k+j;
//   * any other message costs two dependent loads (its first word, then its end's record head).
// Each message is checked the way InputStreamMessageReader reads it from a PackedInputStream:
// the first word (a run may not cross word 1), the rest of the table (nor its end), the
// segment-count and traversal limits, then the segments (nor the message end).
#include "cpk_device.h"
#include "cpk_kernels.h"

namespace cpk {
namespace {

constexpr uint64_t kNone = ~0ull;
constexpr int32_t sOK = 0, sEOF = 1, sOver = 2, sTooMany = 3, sTooLarge = 4, sCap = 8;

__global__ void set4_kernel(uint64_t* d, uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3) {
  if (threadIdx.x == 0) {
    d[0] = v0;
    d[1] = v1;
    d[2] = v2;
    d[3] = v3;
  }
}

// Scratch zeroing as a kernel: every buffer the codec fills is 8-byte aligned.  (Inside a
// captured hipGraph, memset nodes that share a destination -- the pack and the unpack scratch
// are one buffer -- were observed to replay with the wrong extent; a kernel node is a kernel.)
__global__ void fill_kernel(uint8_t* __restrict__ p, uint64_t n, uint8_t value) {
  const uint64_t v8 = 0x0101010101010101ull * value;
  const uint64_t nw = n / 8;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw;
       i += (uint64_t)gridDim.x * blockDim.x)
    ((uint64_t*)p)[i] = v8;
  if (blockIdx.x == 0 && threadIdx.x < n - 8 * nw) p[8 * nw + threadIdx.x] = value;
}

// Streaming device-to-device copy, 16 bytes per lane with U loads in flight per lane before their
// stores: the measured HBM ceiling bench.py quotes beside the 8 TB/s spec (MI355X_MICROARCH.md:
// 6.29 TB/s for a float4 copy).  Diagnostic, not on the codec path.
typedef uint32_t cu32x4 __attribute__((ext_vector_type(4)));
template <int U, bool NT, bool CONTIG>
__global__ __launch_bounds__(256) void copy_kernel(const cu32x4* __restrict__ src,
                                                   cu32x4* __restrict__ dst, uint64_t n16) {
  // CONTIG: block b copies its own contiguous share of the buffer (256 lanes x U blocks of 16 B
  // per step); else grid-strided.  NT: non-temporal loads and stores (no cache allocation).
  uint64_t i, stride, end;
  if (CONTIG) {
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per;
    end = b0 + per < n16 ? b0 + per : n16;
    i = b0 + threadIdx.x;
    stride = 256;
  } else {
    end = n16;
    stride = (uint64_t)gridDim.x * 256;
    i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  }
  for (; i + (U - 1) * stride < end; i += U * stride) {
    cu32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; k++)
      v[k] = NT ? __builtin_nontemporal_load(src + i + k * stride) : src[i + k * stride];
#pragma unroll
    for (int k = 0; k < U; k++) {
      if (NT) __builtin_nontemporal_store(v[k], dst + i + k * stride);
      else dst[i + k * stride] = v[k];
    }
  }
  for (; i < end; i += stride) dst[i] = src[i];
}

// The same copy through CDNA4's LDS-DMA: each wave stages U KiB of its block's contiguous share
// with global_load_lds_dwordx4 (no VGPR destination: the bytes land in the wave's LDS, lane-linear),
// waits for them, and stores them from LDS.  (The bench's copy ceiling: MI355X_MICROARCH.md
// measures LDS-DMA streams at 6.4-6.8 TB/s chip-wide, read side.)
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_lds_kernel(const cu32x4* __restrict__ src,
                                                       cu32x4* __restrict__ dst, uint64_t n16) {
  __shared__ __attribute__((aligned(16))) cu32x4 buf[4][U * 64];
  const int w = (int)(threadIdx.x >> 6), l = (int)(threadIdx.x & 63);
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * per;
  const uint64_t end = b0 + per < n16 ? b0 + per : n16;
  constexpr uint64_t kChunk = (uint64_t)U * 64;
  // (every wave of the block the same trip count: the barrier below is block-wide)
  uint64_t base = b0;
  for (; base + 4 * kChunk <= end; base += 4 * kChunk) {
    const uint64_t i = base + (uint64_t)w * kChunk;
#pragma unroll
    for (int k = 0; k < U; k++)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src + i + 64 * k + l),
          (__attribute__((address_space(3))) void*)&buf[w][64 * k], 16, 0, NT ? 2 : 0);
    // LDS-DMA bytes are ordered for a ds_read by the issuing wave's vmcnt and then a barrier
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int k = 0; k < U; k++) {
      const cu32x4 v = buf[w][64 * k + l];
      if (NT) __builtin_nontemporal_store(v, dst + i + 64 * k + l);
      else dst[i + 64 * k + l] = v;
    }
  }
  // (less than one round of chunks left: plain copies)
  for (uint64_t j = base + threadIdx.x; j < end; j += 256) dst[j] = src[j];
}

struct Flat {
  const uint8_t* packed;
  uint64_t nbytes;
  const uint64_t* rec_pos;
  const uint64_t* rec_gen;  // (device) the call's generation: rec_pos entries of other calls
                            // (or of none) do not count
  const uint64_t* meta;  // (device) where the flat decode stopped: packed byte, word, status
  uint64_t Bc, Tc;  // packed byte / word where the flat decode stopped
  uint64_t gen;
  bool capped;      // ... because the output was full, not because the input ended

  __device__ void load() {
    Bc = meta[0];
    Tc = meta[1];
    gen = *rec_gen;
    capped = (int32_t)meta[2] != sEOF && Bc < nbytes;
  }

  // packed byte of the record whose head is word x (x <= Tc); kNone inside a run
  __device__ uint64_t head(uint64_t x) const {
    if (x == Tc) return Bc;
    const uint64_t v = rec_pos[x];
    return (v >> kRecGenShift) == gen ? (v & kRecPosMask) : kNone;
  }

  // A read that has to end at word x > Tc meets the record at Bc first: the reference checks a
  // raw run's count against the read before it needs the run's bytes (serialize-packed.c++:
  // 138-143), every other cut record is the end of the input.
  __device__ int32_t past_end(uint64_t x) const {
    if (capped) return sCap;
    if (Bc < nbytes && packed[Bc] == 0xff && Bc + 9 < nbytes && Tc + 1 + packed[Bc + 9] > x)
      return sOver;
    return sEOF;
  }
  // a read from a record head up to word x, given head(x) when x <= Tc
  __device__ int32_t read_to(uint64_t x, uint64_t hx) const {
    if (x > Tc) return past_end(x);
    return hx == kNone ? sOver : sOK;
  }
};

// One message of the chain at word s (s < Tc; hs = head(s)), checked the way
// InputStreamMessageReader reads it from a PackedInputStream (serialize.c++:207-269): the first
// word (no run may cross word 1), the rest of the table (nor its end), the segment-count and
// traversal limits, the segments (nor the message end).  Single lane.  Returns the status; on
// success *end / *he are the next message's first word and its record head, *single the
// message's size when it has one segment (0 otherwise).
__device__ int32_t message_at(const Flat& F, const uint64_t* __restrict__ words, uint64_t s,
                              uint64_t limit, uint64_t* end, uint64_t* he, uint64_t* single) {
  const uint64_t w0 = words[s];
  const uint64_t h1 = F.head(s + 1);  // s < Tc, so s + 1 <= Tc
  int32_t e = F.read_to(s + 1, h1);
  if (e) return e;
  const uint32_t nm1 = (uint32_t)w0;
  if (nm1 >= 511) return sTooMany;  // :217
  const uint32_t nseg = nm1 + 1;
  const uint64_t tw = nseg / 2 + 1;
  uint64_t total = w0 >> 32;
  if (nseg > 1) {
    // the other sizes ((nseg & ~1) u32 entries) in one read that ends with the table
    e = F.read_to(s + tw, s + tw <= F.Tc ? F.head(s + tw) : kNone);
    if (e) return e;
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(words + s);
    for (uint32_t i = 1; i < nseg; i++) total += t32[i + 1];
  }
  if (total > limit) return sTooLarge;  // :235
  const uint64_t x = s + tw + total;
  const uint64_t hx = x <= F.Tc ? F.head(x) : kNone;
  e = F.read_to(x, hx);  // the segments: no run may cross the message end
  if (e) return e;
  *end = x;
  *he = hx;
  *single = nseg == 1 ? tw + total : 0;
  return sOK;
}

// Where a walk stopped: k messages from its start, the next message's first word s and record
// head hs, and why (kRunOn: it reached its word limit wend and the stream goes on).
constexpr int32_t kRunOn = -1;
struct WalkEnd {
  uint64_t k, s, hs;
  int32_t stop;
};

// The message chain from word s (head hs) by one wave, until a message would start at or past
// word wend, kmax messages are out, the decoded words end, or a message fails its checks.
// emit(i, s_i, hs_i) receives message i of the walk (on the lane that found it).  A stretch of
// same-size single-segment messages (the common batch shape) is confirmed 64 messages per step:
// lane j checks the header and both read boundaries of message k + j; any other message costs a
// few dependent loads.
// meet(s) (optional): true when the walk should stop at message start s (kMet), before it.
constexpr int32_t kMet = -2;
struct NoMeet {
  __device__ bool operator()(uint64_t) const { return false; }
  static constexpr bool kActive = false;
};
template <class Emit, class Meet = NoMeet>
__device__ WalkEnd walk_messages(const Flat& F, const uint64_t* __restrict__ words, uint64_t s,
                                 uint64_t hs, uint64_t kmax, uint64_t limit, uint64_t wend,
                                 Emit emit, Meet meet = Meet()) {
  const int l = lane_id();
  uint64_t k = 0;
  uint64_t L = 0, prevL = 0;  // the last two message sizes (a stride is tried when they agree)
  bool exact = false;         // the next message goes through message_at
  WalkEnd r;
  r.stop = kRunOn;
  while (k < kmax && s < wend) {
    if (Meet::kActive && meet(s)) {
      r.stop = kMet;
      break;
    }
    if (s == F.Tc) {
      // the next message's first word lies past what decoded: end of input (clean when no bytes
      // are left), a cut record, or a full output
      r.stop = (F.Bc < F.nbytes || F.capped) ? F.read_to(s + 1, kNone) : sOK;
      break;
    }
    if (!Meet::kActive && L != 0 && L == prevL) {
      // ---- a stretch of messages of L words (single segment): 64 per step ----
      const uint64_t p = s + (uint64_t)l * L;
      bool ok = k + (uint64_t)l < kmax && p < wend && p + L <= F.Tc;
      uint64_t w0 = 0, h1 = kNone, hL = kNone;
      if (ok) {
        w0 = words[p];
        h1 = F.head(p + 1);
        hL = F.head(p + L);
      }
      ok = ok && w0 == ((L - 1) << 32) && L - 1 <= limit && h1 != kNone && hL != kNone;
      const uint64_t bad = ballot(!ok);
      const int n = bad ? lowest_bit(bad) : 64;
      const uint64_t hprev = shfl64(hL, l > 0 ? l - 1 : 0);
      if (l < n) emit(k + l, p, l == 0 ? hs : hprev);
      if (n > 0) {
        hs = readlane64(hL, n - 1);
        s += (uint64_t)n * L;
        k += (uint64_t)n;
        if (n == 64) continue;
      }
      prevL = 0;  // the stretch ended: the next message goes the serial way
      continue;
    }
    if (!Meet::kActive && !exact) {
      // ---- up to 64 messages followed on their first words alone, checked together ----
      // Lane 0 follows the chain through each message's first words only (one dependent load per
      // message: the sizes of up to 7 segments share the first four words); every lane then
      // checks one message's reads against the record heads as message_at does, in its order
      // (first word, table, segments).  A message whose table is longer, ends past the decoded
      // words or exceeds the limit goes through message_at next (`exact`).
      __shared__ uint64_t b_s[64], b_x[64];
      __shared__ uint32_t b_tw[64];
      uint32_t nb = 0, fall = 0;
      if (l == 0) {
        uint64_t cs = s;
        while (nb < 64 && k + nb < kmax && cs < wend && cs < F.Tc) {
          const uint64_t w0 = words[cs];
          const uint32_t nm1 = (uint32_t)w0;
          const uint64_t tw = (nm1 + 1) / 2 + 1;
          if (nm1 > 6 || cs + tw > F.Tc) {
            fall = 1;
            break;
          }
          uint64_t total = w0 >> 32;
          if (nm1) {
            const uint32_t* t32 = reinterpret_cast<const uint32_t*>(words + cs);
            for (uint32_t i = 1; i <= nm1; i++) total += t32[i + 1];
          }
          const uint64_t x = cs + tw + total;
          if (total > limit || x > F.Tc) {
            fall = 1;
            break;
          }
          b_s[nb] = cs;
          b_x[nb] = x;
          b_tw[nb] = (uint32_t)tw | (nm1 ? 0x80000000u : 0u);
          nb++;
          cs = x;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      nb = readlane32(nb, 0);
      fall = readlane32(fall, 0);
      if (nb) {
        const bool act = (uint32_t)l < nb;
        const uint32_t j = act ? (uint32_t)l : 0u;
        const uint64_t sj = b_s[j], xj = b_x[j];
        const uint32_t twj = b_tw[j];
        int32_t e = F.read_to(sj + 1, F.head(sj + 1));
        const uint64_t st = sj + (twj & 0x7fffffffu);
        if (!e && (twj >> 31)) e = F.read_to(st, F.head(st));
        const uint64_t hxj = F.head(xj);  // (xj <= Tc)
        if (!e) e = F.read_to(xj, hxj);
        const uint64_t bad = ballot(act && e != 0);
        const uint32_t n = bad ? (uint32_t)lowest_bit(bad) : nb;
        const uint64_t hprev = shfl64(hxj, l > 0 ? l - 1 : 0);
        const uint64_t hsj = l == 0 ? hs : hprev;
        if ((uint32_t)l < n) emit(k + (uint64_t)l, sj, hsj);
        if (bad) {
          r.stop = (int32_t)readlane32((uint32_t)e, (int)n);
          k += n;
          s = readlane64(sj, (int)n);
          hs = readlane64(hsj, (int)n);
          break;
        }
        const uint64_t single = (twj >> 31) ? 0ull : xj - sj;
        prevL = nb >= 2 ? readlane64(single, (int)nb - 2) : L;
        L = readlane64(single, (int)nb - 1);
        k += nb;
        s = readlane64(xj, (int)nb - 1);
        hs = readlane64(hxj, (int)nb - 1);
      }
      exact = fall != 0;
      continue;
    }
    exact = false;
    uint64_t x = 0, hx = kNone, single = 0;
    int32_t e = 0;
    if (l == 0) e = message_at(F, words, s, limit, &x, &hx, &single);
    e = (int32_t)readlane32((uint32_t)e, 0);
    if (e) {
      r.stop = e;
      break;
    }
    if (l == 0) emit(k, s, hs);
    k++;
    prevL = L;
    L = readlane64(single, 0);
    s = readlane64(x, 0);
    hs = readlane64(hx, 0);
  }
  r.k = k;
  r.s = s;
  r.hs = hs;
  return r;
}

// ---- block-parallel split ------------------------------------------------------------------
// The decoded words are cut into blocks of kSplitBlock words.  Every block guesses where the
// chain first enters it -- the first record head from which two messages in a row pass their
// checks (a guess is only a guess: a wrong one is caught below) -- and walks the chain from
// there to the block end, keeping up to kSplitList message starts.  One wave then runs over the
// blocks in order: a block whose true entry (the previous block's exit) is its guess keeps its
// walk; any other block is walked again from its true entry.  A last pass writes every block's
// messages at their global index.
#ifndef CPK_SPLIT_BLOCK_LOG
#define CPK_SPLIT_BLOCK_LOG 16  // log2 words per block (20: C5-shaped split 4.1 ms guess walks)
#endif
// Blocks are the unit of parallelism of the guess, meet and write walks (one wave each, a few
// dependent loads per message): 64 Ki-word blocks give a C5-shaped stream ~7 k waves where 1 Mi
// gave 456, each walking ~150 messages instead of ~2300.
constexpr uint64_t kSplitBlock = 1ull << CPK_SPLIT_BLOCK_LOG;  // words per block
constexpr uint32_t kSplitList = CPK_SPLIT_BLOCK_LOG >= 20 ? 4096 : 2048;  // starts a block keeps
constexpr uint64_t kSplitScan = 1ull << 16;    // words a block searches for its guess

// in-order pass counters (diagnostic, read by cpk_debug_split): windows resolved in parallel,
// blocks they resolved, then serial blocks by path -- guess, se, se2, walked, passed over
__device__ unsigned long long g_split_dbg[8];

struct SplitBlock {
  uint64_t g, x, hx, k;  // guess (kNone: none), exit word / head, messages
  int32_t stop;          // kRunOn, or why the walk from the guess ended inside the block
  uint32_t over;         // more messages than the list holds
  uint64_t entry, kbase, kend;  // resolved: true entry (kNone: none), first / end global index
  // the block walked from the previous block's guess exit (se; kNone: not done) -- its true
  // entry whenever the previous block's true chain met its guess: messages, exit, stop
  uint64_t se, sk, sx, shx;
  int32_t sst;
  // the same from the previous block's se walk's exit, when that walk did not meet its guess
  // chain (a guess off the chain: the next block's se then is not its entry)
  uint64_t se2, sk2, sx2, shx2;
  int32_t sst2;
};

__global__ __launch_bounds__(64) void split_spec_kernel(Flat F, const uint64_t* __restrict__ words,
                                                        uint64_t limit, SplitBlock* blocks,
                                                        uint64_t* lists) {
  F.load();
  const int l = lane_id();
  const uint64_t b = blockIdx.x;
  const uint64_t w0 = b * kSplitBlock;
  const uint64_t w1 = w0 + kSplitBlock;
  SplitBlock r;
  r.g = kNone;
  r.x = kNone;
  r.hx = kNone;
  r.k = 0;
  r.stop = kRunOn;
  r.over = 0;
  uint64_t* const list = lists + b * kSplitList;
  auto walk_from = [&](uint64_t g, uint64_t hg) {
    const WalkEnd we = walk_messages(F, words, g, hg, ~0ull, limit, w1,
                                     [&](uint64_t i, uint64_t s, uint64_t) {
                                       if (i < kSplitList) list[i] = s;
                                     });
    r.g = g;
    r.x = we.s;
    r.hx = we.hs;
    r.k = we.k;
    r.stop = we.stop;
    r.over = we.k > kSplitList ? 1u : 0u;
  };
  if (b == 0) {
    walk_from(0, F.head(0));
  } else {
    // the first record head from which two messages in a row pass their checks and whose chain
    // then runs to the block end without failing (the true chain of a readable stream never
    // fails inside it; a chain through words that only look like segment tables soon does)
    const uint64_t lim = min(min(w1, F.Tc), w0 + kSplitScan);
    for (uint64_t base = w0; base < lim;) {
      const uint64_t p = base + (uint64_t)l;
      bool cand = false;
      uint64_t hp = kNone;
      if (p < lim) {
        hp = F.head(p);  // (p < Tc)
        if (hp != kNone && (uint32_t)words[p] < 511) {
          uint64_t x = 0, hx = 0, single = 0;
          if (message_at(F, words, p, limit, &x, &hx, &single) == sOK) {
            uint64_t x2 = 0, hx2 = 0;
            cand = x == F.Tc || message_at(F, words, x, limit, &x2, &hx2, &single) == sOK;
          }
        }
      }
      const uint64_t cb = ballot(cand);
      if (!cb) {
        base += 64;
        continue;
      }
      const int j = lowest_bit(cb);
      walk_from(base + (uint64_t)j, readlane64(hp, j));
      if (r.stop == kRunOn || r.stop == sOK) break;  // ran to the block end (or the stream's)
      r.g = kNone;  // failed inside the block: not the chain; the next candidate
      base += (uint64_t)j + 1;
    }
  }
  if (l == 0) {
    r.entry = kNone;
    r.kbase = r.kend = 0;
    r.se = kNone;
    r.sk = r.sx = r.shx = 0;
    r.sst = kRunOn;
    r.se2 = kNone;
    r.sk2 = r.sx2 = r.shx2 = 0;
    r.sst2 = kRunOn;
    blocks[b] = r;
  }
}

// Meets a block's listed starts (ascending) -- lane 0 keeps the list position.
struct Meet2 {
  const uint64_t* list;
  uint64_t n;
  uint64_t* j;
  static constexpr bool kActive = true;
  __device__ bool operator()(uint64_t s) const {
    bool met = false;
    if (lane_id() == 0) {
      while (*j < n && list[*j] < s) (*j)++;
      met = *j < n && list[*j] == s;
    }
    return readlane32(met ? 1u : 0u, 0) != 0;
  }
};

// Every block b > 0 walked, in parallel, from where block b - 1's guess chain leaves it until the
// chain meets block b's guess chain (a few messages): block b's entry whenever block b - 1's true
// chain met its guess, which the in-order pass below then only has to confirm.
__global__ __launch_bounds__(64) void split_meet_kernel(Flat F, const uint64_t* __restrict__ words,
                                                        uint64_t limit, SplitBlock* blocks,
                                                        const uint64_t* __restrict__ lists,
                                                        uint64_t nblocks) {
  F.load();
  const uint64_t b = (uint64_t)blockIdx.x + 1;
  if (b >= nblocks) return;
  const uint64_t pg = blocks[b - 1].g, E = blocks[b - 1].x, hE = blocks[b - 1].hx;
  const int32_t pst = blocks[b - 1].stop;
  const uint64_t g = blocks[b].g, gk = blocks[b].k;
  const uint64_t w1 = (b + 1) * kSplitBlock;
  uint64_t se = kNone, sk = 0, sx = 0, shx = 0;
  int32_t sst = kRunOn;
  if (pg != kNone && pst == kRunOn && E < w1 && E != g) {
    const bool listed = g != kNone && gk <= kSplitList;
    uint64_t jl = 0;
    Meet2 mt{lists + b * kSplitList, listed ? gk : 0, &jl};
    const WalkEnd we = walk_messages(F, words, E, hE, ~0ull, limit, w1,
                                     [&](uint64_t, uint64_t, uint64_t) {}, mt);
    jl = readlane64(jl, 0);
    se = E;
    if (we.stop == kMet) {
      sk = we.k + (gk - jl);
      sx = blocks[b].x;
      shx = blocks[b].hx;
      sst = blocks[b].stop;
    } else {
      sk = we.k;
      sx = we.s;
      shx = we.hs;
      sst = we.stop;
    }
  }
  if (lane_id() == 0) {
    SplitBlock* const B = blocks + b;
    B->se = se;
    B->sk = sk;
    B->sx = sx;
    B->shx = shx;
    B->sst = sst;
  }
}

// Every block b > 1 whose predecessor's se walk ran past its guess chain without meeting it (the
// predecessor's guess was off the chain, so its exit is not where the true chain leaves it):
// walked from that walk's exit until it meets block b's guess chain -- a third candidate entry
// the in-order pass takes without walking.
__global__ __launch_bounds__(64) void split_meet2_kernel(Flat F, const uint64_t* __restrict__ words,
                                                         uint64_t limit, SplitBlock* blocks,
                                                         const uint64_t* __restrict__ lists,
                                                         uint64_t nblocks) {
  F.load();
  const uint64_t b = (uint64_t)blockIdx.x + 2;
  if (b >= nblocks) return;
  const SplitBlock& P = blocks[b - 1];
  const uint64_t E = P.sx, hE = P.shx;
  const uint64_t g = blocks[b].g, gk = blocks[b].k, se = blocks[b].se;
  const uint64_t w1 = (b + 1) * kSplitBlock;
  if (P.se == kNone || P.sst != kRunOn || E == P.x || E >= w1 || E == g || E == se) return;
  const bool listed = g != kNone && gk <= kSplitList;
  uint64_t jl = 0;
  Meet2 mt{lists + b * kSplitList, listed ? gk : 0, &jl};
  const WalkEnd we = walk_messages(F, words, E, hE, ~0ull, limit, w1,
                                   [&](uint64_t, uint64_t, uint64_t) {}, mt);
  jl = readlane64(jl, 0);
  if (lane_id() == 0) {
    SplitBlock* const B = blocks + b;
    B->se2 = E;
    if (we.stop == kMet) {
      B->sk2 = we.k + (gk - jl);
      B->sx2 = blocks[b].x;
      B->shx2 = blocks[b].hx;
      B->sst2 = blocks[b].stop;
    } else {
      B->sk2 = we.k;
      B->sx2 = we.s;
      B->shx2 = we.hs;
      B->sst2 = we.stop;
    }
  }
}

// A full window of 64 blocks resolved in parallel.  Block b's entry is, nearly always, one of two
// known candidates: its guess g (state a: then its walk gives exit x, k messages, stop) or the
// entry the previous block's guess chain leaves it at, se (state b: split_meet_kernel's walk
// gives sx, sk, sst).  So each block maps the state of its entry to the state its exit gives the
// next block (a, b; 2: neither; 3: the chain stopped) plus messages, these maps compose, and six
// shuffle steps give every block its entry state and message base.  Returns the blocks resolved:
// up to the first whose entry matches neither candidate (a block passed over by a long message,
// a wrong guess), which the serial pass then takes.
__device__ int resolve_window(SplitBlock* blocks, uint64_t base, const SplitBlock& mine,
                              uint64_t max_msgs, uint64_t& E, uint64_t& hE, uint64_t& K,
                              int32_t& stop) {
  const int l = lane_id();
  const uint64_t g0 = readlane64(mine.g, 0), se0 = readlane64(mine.se, 0);
  const uint32_t sin = (g0 != kNone && E == g0) ? 0u : ((se0 != kNone && E == se0) ? 1u : 2u);
  if (sin == 2u) return 0;
  // the next block's candidates (lane 63: not needed -- the window's exit is carried as a word)
  const uint64_t ng = shfl64(mine.g, l < 63 ? l + 1 : 63);
  const uint64_t nse = shfl64(mine.se, l < 63 ? l + 1 : 63);
  auto cls = [&](uint64_t X) -> uint32_t {
    if (l == 63) return 0u;
    return (ng != kNone && X == ng) ? 0u : ((nse != kNone && X == nse) ? 1u : 2u);
  };
  const uint32_t fa = mine.g == kNone ? 2u : (mine.stop != kRunOn ? 3u : cls(mine.x));
  const uint32_t fb = mine.se == kNone ? 2u : (mine.sst != kRunOn ? 3u : cls(mine.sx));
  const uint64_t ka = mine.k, kb = mine.sk;
  // inclusive composition toward higher lanes (the earlier block applied first)
  uint32_t sa = fa, sb = fb;
  uint64_t wa = ka, wb = kb;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int q = l >= o ? l - o : 0;
    const uint32_t psa = shfl32(sa, q), psb = shfl32(sb, q);
    const uint64_t pwa = shfl64(wa, q), pwb = shfl64(wb, q);
    if (l >= o) {
      const uint32_t na = psa >= 2u ? psa : (psa == 0u ? sa : sb);
      const uint64_t nwa = pwa + (psa >= 2u ? 0ull : (psa == 0u ? wa : wb));
      const uint32_t nb = psb >= 2u ? psb : (psb == 0u ? sa : sb);
      const uint64_t nwb = pwb + (psb >= 2u ? 0ull : (psb == 0u ? wa : wb));
      sa = na;
      wa = nwa;
      sb = nb;
      wb = nwb;
    }
  }
  // the state entering each block, and the messages before it
  const int q = l > 0 ? l - 1 : 0;
  const uint32_t pa = shfl32(sa, q), pb = shfl32(sb, q);
  const uint64_t pwa = shfl64(wa, q), pwb = shfl64(wb, q);
  const uint32_t in = l == 0 ? sin : (sin == 0u ? pa : pb);
  const uint64_t kin = K + (l == 0 ? 0ull : (sin == 0u ? pwa : pwb));
  const uint64_t fb2 = ballot(in == 2u);
  const int f = fb2 ? lowest_bit(fb2) : 64;  // the first block that matches neither
  if (f == 0) return 0;
  const bool reached = in < 2u && l < f;
  const uint64_t kk = in == 0u ? mine.k : mine.sk;
  const uint64_t kend = kin + kk;
  // the message limit: the first block it falls in is cut there (the writer walks it)
  const uint64_t cb = ballot(reached && kend >= max_msgs);
  const int cut = cb ? lowest_bit(cb) : 64;
  if (reached && l <= cut) {
    SplitBlock* const B = blocks + base + l;
    B->entry = in == 0u ? mine.g : mine.se;
    B->kbase = kin;
    B->kend = l == cut ? max_msgs : kend;
    B->over = (l == cut || in == 1u || mine.over) ? 1u : 0u;
  }
  if (cut < 64) {
    K = max_msgs;
    stop = sOK;
    return 64;
  }
  // the last block reached: its exit goes on, or the chain stopped in it
  const int last = 63 - __builtin_clzll(ballot(reached));
  const uint32_t il = readlane32(in, last);
  E = readlane64(il == 0u ? mine.x : mine.sx, last);
  hE = readlane64(il == 0u ? mine.hx : mine.shx, last);
  K = readlane64(kend, last);
  const int32_t st = (int32_t)readlane32((uint32_t)(il == 0u ? mine.stop : mine.sst), last);
  if (st != kRunOn) stop = st;
  return f;
}

// One wave over the blocks in order: each block's true entry, global message range and the
// stream's stop.  A block whose entry is its guess (or that the chain passes over) costs a load;
// any other block is walked again here.
__global__ __launch_bounds__(64) void split_resolve_kernel(Flat F, const uint64_t* __restrict__ words,
                                                           uint64_t limit, uint64_t max_msgs,
                                                           SplitBlock* blocks,
                                                           const uint64_t* __restrict__ lists,
                                                           uint64_t nblocks,
                                                           uint64_t* __restrict__ msg_word_off,
                                                           uint64_t* __restrict__ msg_in_off,
                                                           int32_t* __restrict__ status,
                                                           uint64_t* __restrict__ nmsgs) {
  F.load();
  const int l = lane_id();
  uint64_t E = 0, hE = F.head(0), K = 0;
  int32_t stop = kRunOn;
  for (uint64_t base = 0; base < nblocks && stop == kRunOn;) {
    // the next 64 blocks' walks in one round trip (lane j: block base + j)
    SplitBlock mine = {};
    if (base + l < nblocks) mine = blocks[base + l];
    // in parallel up to the first block whose entry matches neither candidate; that block
    // serially; then the next window from the block after it (the last, partial window: serially)
    const bool full = base + 64 <= nblocks;
    const int done = full ? resolve_window(blocks, base, mine, max_msgs, E, hE, K, stop) : 0;
    if (l == 0 && done) {
      atomicAdd(&g_split_dbg[0], 1ull);
      atomicAdd(&g_split_dbg[1], (unsigned long long)done);
    }
    const int jend = full ? (done < 64 ? done + 1 : 64) : 64;
    for (int j = done; j < jend && base + j < nblocks && stop == kRunOn; j++) {
      const uint64_t b = base + j;
      const uint64_t w1 = (b + 1) * kSplitBlock;
      if (E >= w1) {  // the chain passes over the block (a message longer than it)
        if (l == 0) atomicAdd(&g_split_dbg[6], 1ull);
        continue;
      }
      const uint64_t g = readlane64(mine.g, j);
      uint64_t x, hx, k;
      int32_t st;
      bool redo = readlane32(mine.over, j) != 0;
      if (g == E) {
        if (l == 0) atomicAdd(&g_split_dbg[2], 1ull);
        x = readlane64(mine.x, j);
        hx = readlane64(mine.hx, j);
        k = readlane64(mine.k, j);
        st = (int32_t)readlane32((uint32_t)mine.stop, j);
      } else if (readlane64(mine.se, j) == E) {
        // walked in parallel from this very entry (split_meet_kernel)
        if (l == 0) atomicAdd(&g_split_dbg[3], 1ull);
        x = readlane64(mine.sx, j);
        hx = readlane64(mine.shx, j);
        k = readlane64(mine.sk, j);
        st = (int32_t)readlane32((uint32_t)mine.sst, j);
        redo = true;
      } else if (readlane64(mine.se2, j) == E) {
        // or from this one (split_meet2_kernel)
        if (l == 0) atomicAdd(&g_split_dbg[4], 1ull);
        x = readlane64(mine.sx2, j);
        hx = readlane64(mine.shx2, j);
        k = readlane64(mine.sk2, j);
        st = (int32_t)readlane32((uint32_t)mine.sst2, j);
        redo = true;
      } else {
        // the guess was not the entry: walk the block from its true entry until the chain meets
        // the guess's chain (a guess whose chain ran to the block end without failing nearly
        // always joined the true chain early: a few messages here), then take the rest from it
        const uint64_t gk = readlane64(mine.k, j);
        if (l == 0) atomicAdd(&g_split_dbg[5], 1ull);
        const bool listed = g != kNone && gk <= kSplitList;
        const uint64_t* const list = lists + b * kSplitList;
        uint64_t jl = 0;  // next listed start to compare with (both chains ascend)
        Meet2 mt{list, listed ? gk : 0, &jl};
        const WalkEnd we = walk_messages(F, words, E, hE, ~0ull, limit, w1,
                                         [&](uint64_t, uint64_t, uint64_t) {}, mt);
        jl = readlane64(jl, 0);
        if (we.stop == kMet) {
          x = readlane64(mine.x, j);
          hx = readlane64(mine.hx, j);
          k = we.k + (gk - jl);
          st = (int32_t)readlane32((uint32_t)mine.stop, j);
        } else {
          x = we.s;
          hx = we.hs;
          k = we.k;
          st = we.stop;
        }
        redo = true;
      }
      uint64_t kend = K + k;
      if (kend >= max_msgs) {
        // the message limit falls in this block: the writer walks it and stops there
        kend = max_msgs;
        redo = true;
        st = kRunOn;
      }
      if (l == 0) {
        SplitBlock* const B = blocks + b;
        B->entry = E;
        B->kbase = K;
        B->kend = kend;
        B->over = redo ? 1u : 0u;  // the writer walks the block itself
      }
      K = kend;
      if (K >= max_msgs) {
        stop = sOK;  // max_msgs messages; the next one starts where the writer stops
        break;
      }
      E = x;
      hE = hx;
      stop = st;
    }
    base += (uint64_t)jend;
  }
  if (stop == kRunOn) stop = sOK;  // (nblocks covers every decoded word)
  if (l == 0) {
    *nmsgs = K;
    status[K] = stop;
    if (K < max_msgs || max_msgs == 0) {
      msg_word_off[K] = E;
      msg_in_off[K] = hE;
    }
  }
}

// Every block's messages at their global index: copied from the block's list, or walked again
// when the list did not hold them (or the guess was off the chain, or the limit cuts the block).
__global__ __launch_bounds__(64) void split_write_kernel(Flat F, const uint64_t* __restrict__ words,
                                                         uint64_t limit, const SplitBlock* blocks,
                                                         const uint64_t* lists,
                                                         uint64_t* __restrict__ msg_word_off,
                                                         uint64_t* __restrict__ msg_in_off,
                                                         int32_t* __restrict__ status,
                                                         uint64_t max_msgs) {
  F.load();
  const int l = lane_id();
  const uint64_t b = blockIdx.x;
  const SplitBlock B = blocks[b];
  if (B.entry == kNone || B.kend <= B.kbase) return;
  const uint64_t n = B.kend - B.kbase;
  if (!B.over) {
    const uint64_t* const list = lists + b * kSplitList;
    for (uint64_t i = l; i < n; i += 64) {
      const uint64_t s = list[i];
      msg_word_off[B.kbase + i] = s;
      msg_in_off[B.kbase + i] = F.head(s);
      status[B.kbase + i] = sOK;
    }
    return;
  }
  const WalkEnd we = walk_messages(F, words, B.entry, F.head(B.entry), n, limit,
                                   (b + 1) * kSplitBlock, [&](uint64_t i, uint64_t s, uint64_t hs) {
                                     msg_word_off[B.kbase + i] = s;
                                     msg_in_off[B.kbase + i] = hs;
                                     status[B.kbase + i] = sOK;
                                   });
  // the message limit cut this block: the entry after the last message
  if (B.kend == max_msgs && l == 0) {
    msg_word_off[max_msgs] = we.s;
    msg_in_off[max_msgs] = we.hs;
  }
}

// ---- framing without a host gather ----------------------------------------------------------
// writePackedMessage(getSegmentsForOutput()) with the segments where the builder keeps them
// (serialize-packed.h:92-98, arena.c++:300-329): the segment table and every segment are copied
// into one flat message in HBM (coalesced: each block takes 2048 consecutive output words and
// finds its segment once), which the pack kernels then take as nseg + 1 chunks.
// meta: seg_ptr[nseg], chunk_off[nseg + 2] (0, table words, then each segment's end), table[tw].
__global__ __launch_bounds__(256) void gather_kernel(const uint64_t* __restrict__ meta,
                                                     uint32_t nseg, uint64_t* __restrict__ out) {
  const uint64_t* const* seg_ptr = reinterpret_cast<const uint64_t* const*>(meta);
  const uint64_t* chunk_off = meta + nseg;
  const uint64_t* table = chunk_off + nseg + 2;
  const uint64_t tw = chunk_off[1], total = chunk_off[nseg + 1];
  const uint64_t base = (uint64_t)blockIdx.x * 2048;
  if (base >= total) return;
  // the chunk holding the block's first word: last c with chunk_off[c] <= base
  uint32_t lo = 0, hi = nseg + 1;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (chunk_off[mid] <= base) lo = mid;
    else hi = mid;
  }
  uint32_t c = lo;
  for (uint64_t i = base + threadIdx.x; i < base + 2048 && i < total; i += 256) {
    while (chunk_off[c + 1] <= i) c++;
    out[i] = c == 0 ? table[i] : seg_ptr[c - 1][i - chunk_off[c]];
  }
  (void)tw;
}

// ---- message placement for the batch exchange ------------------------------------------------
// n byte ranges src[src_off[i], +len[i]) -> dst[dst_off[i], ...): one wave per range (the waves
// of a capped grid stride over the ranges, so any n launches), the body as 16-byte stores aligned
// on the destination, each from five aligned source dwords shifted by v_alignbyte (the head and
// tail bytes one per lane).  Used by the multi-GPU gather to put round-robin shards' messages at
// their global positions (capnproto_amd/shard.py).
constexpr uint64_t kCopyRangesMaxBlocks = 1u << 16;
__device__ __forceinline__ void copy_range(const uint8_t* __restrict__ s0, uint8_t* __restrict__ o0,
                                           uint64_t nb, uint32_t l) {
  const uint64_t A0 = (uint64_t)(uintptr_t)o0, A1 = A0 + nb;
  const uint64_t al = (A0 + 15) & ~15ull;
  const uint64_t head = (al < A1 ? al : A1) - A0;  // bytes before 16-byte alignment
  if (l < head) o0[l] = s0[l];
  if (A1 <= al) return;
  const uint64_t body = (A1 & ~15ull) - A0;
  const uint64_t nblk = (body - head) >> 4;
  // output block k = source bytes [head + 16k, +16): aligned source dwords from there, shifted
  const uint64_t sb = (uint64_t)(uintptr_t)(s0 + head);
  const uint32_t* const s32 = (const uint32_t*)(sb & ~3ull);
  const uint32_t rr = (uint32_t)(sb & 3u);
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4* const ob = (u32x4*)(o0 + head);
  for (uint64_t k = l; k < nblk; k += 64) {
    const uint32_t* const q = s32 + 4 * k;
    // (the fifth dword is read only when the shift needs it: it may lie past the range)
    const uint32_t v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3], v4 = rr ? q[4] : 0u;
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(v1, v0, rr);
    v.y = __builtin_amdgcn_alignbyte(v2, v1, rr);
    v.z = __builtin_amdgcn_alignbyte(v3, v2, rr);
    v.w = __builtin_amdgcn_alignbyte(v4, v3, rr);
    ob[k] = v;
  }
  if (body + l < nb) o0[body + l] = s0[body + l];
}

__global__ __launch_bounds__(256) void copy_ranges_kernel(const uint8_t* __restrict__ src,
                                                          const uint64_t* __restrict__ src_off,
                                                          const uint64_t* __restrict__ dst_off,
                                                          const uint64_t* __restrict__ len,
                                                          uint64_t n, uint8_t* __restrict__ dst) {
  const uint32_t l = threadIdx.x & 63u;
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += stride) {
    const uint64_t nb = len[i];
    if (nb) copy_range(src + src_off[i], dst + dst_off[i], nb, l);
  }
}

}  // namespace

hipError_t launch_copy_ranges(const uint8_t* src, const uint64_t* src_off,
                              const uint64_t* dst_off, const uint64_t* len, uint64_t n,
                              uint8_t* dst, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 3) / 4 < kCopyRangesMaxBlocks ? (n + 3) / 4 : kCopyRangesMaxBlocks;
  copy_ranges_kernel<<<(unsigned)blocks, 256, 0, stream>>>(src, src_off, dst_off, len, n, dst);
  return hipGetLastError();
}

hipError_t launch_gather_segments(const uint64_t* meta, uint32_t nseg, uint64_t total,
                                  uint64_t* out, hipStream_t stream) {
  if (total == 0) return hipSuccess;
  gather_kernel<<<(unsigned)((total + 2047) / 2048), 256, 0, stream>>>(meta, nseg, out);
  return hipGetLastError();
}

hipError_t launch_fill(void* p, uint64_t nbytes, uint8_t value, hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  if ((uintptr_t)p & 7) return hipErrorInvalidValue;
  const uint64_t nw = nbytes / 8;
  uint64_t blocks = (nw + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  fill_kernel<<<(unsigned)blocks, 256, 0, stream>>>((uint8_t*)p, nbytes, value);
  return hipGetLastError();
}

hipError_t launch_copy(void* dst, const void* src, uint64_t nbytes, uint32_t blocks,
                       hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  if (((uintptr_t)dst | (uintptr_t)src | nbytes) & 15) return hipErrorInvalidValue;
  // blocks: low 24 bits the grid; bits 24-25 the loads in flight per lane (4, 8, 16), bit 26
  // non-temporal loads and stores, bit 27 contiguous per-block shares instead of grid strides;
  // bit 28: LDS-DMA staging (copy_lds_kernel, contiguous shares) of 2 / 4 / 8 KiB per wave
  const unsigned g = (blocks & 0xffffffu) ? (blocks & 0xffffffu) : 4096u;
  const auto* s16 = (const cu32x4*)src;
  auto* d16 = (cu32x4*)dst;
  const uint64_t n = nbytes / 16;
  const unsigned form = (blocks >> 24) & 31u;
  if (form & 16u) {
    switch (form & 7u) {
      case 0: copy_lds_kernel<2, false><<<g, 256, 0, stream>>>(s16, d16, n); break;
      case 1: copy_lds_kernel<4, false><<<g, 256, 0, stream>>>(s16, d16, n); break;
      case 2: copy_lds_kernel<8, false><<<g, 256, 0, stream>>>(s16, d16, n); break;
      case 4: copy_lds_kernel<2, true><<<g, 256, 0, stream>>>(s16, d16, n); break;
      case 5: copy_lds_kernel<4, true><<<g, 256, 0, stream>>>(s16, d16, n); break;
      case 6: copy_lds_kernel<8, true><<<g, 256, 0, stream>>>(s16, d16, n); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
#define CPK_COPY_CASE(F, U, NT, C) \
  case F: copy_kernel<U, NT, C><<<g, 256, 0, stream>>>(s16, d16, n); break;
  switch (form) {
    CPK_COPY_CASE(0, 4, false, false)
    CPK_COPY_CASE(1, 8, false, false)
    CPK_COPY_CASE(2, 16, false, false)
    CPK_COPY_CASE(4, 4, true, false)
    CPK_COPY_CASE(5, 8, true, false)
    CPK_COPY_CASE(6, 16, true, false)
    CPK_COPY_CASE(8, 4, false, true)
    CPK_COPY_CASE(9, 8, false, true)
    CPK_COPY_CASE(10, 16, false, true)
    CPK_COPY_CASE(12, 4, true, true)
    CPK_COPY_CASE(13, 8, true, true)
    CPK_COPY_CASE(14, 16, true, true)
    default: return hipErrorInvalidValue;
  }
#undef CPK_COPY_CASE
  return hipGetLastError();
}

hipError_t launch_set_u64x4(uint64_t* dst, uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3,
                            hipStream_t stream) {
  set4_kernel<<<1, 64, 0, stream>>>(dst, v0, v1, v2, v3);
  return hipGetLastError();
}

uint64_t split_scratch_bytes(uint64_t words_capacity) {
  const uint64_t nb = words_capacity / kSplitBlock + 1;
  return nb * (sizeof(SplitBlock) + 8ull * kSplitList) + 64;
}

__global__ void split_gen_kernel(uint64_t* genw, uint32_t* fill, int force) {
  uint64_t g = force ? 1 : *genw + 1;
  if (g >= kRecGenMax) {
    g = 1;
    force = 1;
  }
  *genw = g;
  *fill = force ? 1u : 0u;
}

// the map fill when split_gen_kernel asks for it (a grid of 4096 blocks that exit at once
// otherwise)
__global__ void fill_if_kernel(uint64_t* __restrict__ p, uint64_t nw, const uint32_t* fill) {
  if (!*fill) return;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw;
       i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = ~0ull;
}

hipError_t launch_split_gen(uint64_t* genw, uint32_t* fill, bool force, uint64_t* rec_pos,
                            uint64_t nbytes, hipStream_t stream) {
  split_gen_kernel<<<1, 1, 0, stream>>>(genw, fill, force ? 1 : 0);
  const uint64_t nw = nbytes / 8;
  if (nw) {
    uint64_t blocks = (nw + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    fill_if_kernel<<<(unsigned)blocks, 256, 0, stream>>>(rec_pos, nw, fill);
  }
  return hipGetLastError();
}

hipError_t launch_split_walk(const uint8_t* packed, uint64_t nbytes, const uint64_t* words,
                             const uint64_t* rec_pos, const uint64_t* rec_gen,
                             const uint64_t* meta, uint64_t max_msgs,
                             uint64_t limit, uint64_t words_capacity, void* scratch,
                             uint64_t* msg_word_off, uint64_t* msg_in_off, int32_t* status,
                             uint64_t* nmsgs, hipStream_t stream) {
  Flat F;
  F.packed = packed;
  F.nbytes = nbytes;
  F.rec_pos = rec_pos;
  F.rec_gen = rec_gen;
  F.meta = meta;
  const uint64_t nb = words_capacity / kSplitBlock + 1;
  SplitBlock* blocks = (SplitBlock*)scratch;
  uint64_t* lists = (uint64_t*)((char*)scratch + ((nb * sizeof(SplitBlock) + 15) & ~15ull));
  split_spec_kernel<<<(unsigned)nb, 64, 0, stream>>>(F, words, limit, blocks, lists);
  if (nb > 1) split_meet_kernel<<<(unsigned)(nb - 1), 64, 0, stream>>>(F, words, limit, blocks, lists, nb);
  if (nb > 2) split_meet2_kernel<<<(unsigned)(nb - 2), 64, 0, stream>>>(F, words, limit, blocks, lists, nb);
  split_resolve_kernel<<<1, 64, 0, stream>>>(F, words, limit, max_msgs, blocks, lists, nb,
                                             msg_word_off, msg_in_off, status, nmsgs);
  split_write_kernel<<<(unsigned)nb, 64, 0, stream>>>(F, words, limit, blocks, lists,
                                                      msg_word_off, msg_in_off, status, max_msgs);
  return hipGetLastError();
}

}  // namespace cpk

// diagnostic: copies out and zeroes the split's in-order pass counters (8 u64)
extern "C" int cpk_debug_split(uint64_t* out) {
  if (hipDeviceSynchronize() != hipSuccess) return 10;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cpk::g_split_dbg), 64) != hipSuccess) return 10;
  const uint64_t z[8] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(cpk::g_split_dbg), z, 64) != hipSuccess) return 10;
  return 0;
}
