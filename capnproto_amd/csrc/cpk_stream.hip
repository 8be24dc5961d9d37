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

struct Flat {
  const uint8_t* packed;
  uint64_t nbytes;
  const uint64_t* rec_pos;
  uint64_t Bc, Tc;  // packed byte / word where the flat decode stopped
  bool capped;      // ... because the output was full, not because the input ended

  // packed byte of the record whose head is word x (x <= Tc); kNone inside a run
  __device__ uint64_t head(uint64_t x) const { return x == Tc ? Bc : rec_pos[x]; }

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

__global__ __launch_bounds__(64) void split_walk_kernel(Flat F, const uint64_t* __restrict__ words,
                                                        const uint64_t* __restrict__ meta,
                                                        uint64_t max_msgs, uint64_t limit,
                                                        uint64_t* __restrict__ msg_word_off,
                                                        uint64_t* __restrict__ msg_in_off,
                                                        int32_t* __restrict__ status,
                                                        uint64_t* __restrict__ nmsgs) {
  const int l = lane_id();
  F.Bc = meta[0];
  F.Tc = meta[1];
  F.capped = (int32_t)meta[2] != sEOF && F.Bc < F.nbytes;
  uint64_t s = 0, k = 0, hs = F.head(0);
  uint64_t L = 0, prevL = 0;  // the last two message sizes (a stride is tried when they agree)
  int32_t stop = sOK;
  while (k < max_msgs) {
    if (s == F.Tc) {
      // the next message's first word lies past what decoded: end of input (clean when no
      // bytes are left), a cut record, or a full output
      if (F.Bc < F.nbytes || F.capped) stop = F.read_to(s + 1, kNone);
      break;
    }
    if (L != 0 && L == prevL) {
      // ---- a stretch of messages of L words (single segment): 64 per step ----
      const uint64_t p = s + (uint64_t)l * L;
      bool ok = k + (uint64_t)l < max_msgs && p + L <= F.Tc;
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
      if (l < n) {
        msg_word_off[k + l] = p;
        msg_in_off[k + l] = l == 0 ? hs : hprev;
        status[k + l] = sOK;
      }
      if (n > 0) {
        hs = readlane64(hL, n - 1);
        s += (uint64_t)n * L;
        k += (uint64_t)n;
        if (n == 64) continue;
      }
      prevL = 0;  // the stretch ended: the next message goes the serial way
      continue;
    }
    // ---- one message (serialize.c++:207-269) ----
    const uint64_t w0 = words[s];
    const uint64_t h1 = F.head(s + 1);  // s < Tc, so s + 1 <= Tc
    int32_t e = F.read_to(s + 1, h1);   // the first word: no run may cross word 1
    if (e) {
      stop = e;
      break;
    }
    const uint32_t nm1 = (uint32_t)w0;
    if (nm1 >= 511) {  // :217
      stop = sTooMany;
      break;
    }
    const uint32_t nseg = nm1 + 1;
    const uint64_t tw = nseg / 2 + 1;
    uint64_t total = w0 >> 32;
    if (nseg > 1) {
      // the other sizes ((nseg & ~1) u32 entries) in one read that ends with the table
      e = F.read_to(s + tw, s + tw <= F.Tc ? F.head(s + tw) : kNone);
      if (e) {
        stop = e;
        break;
      }
      const uint32_t* t32 = reinterpret_cast<const uint32_t*>(words + s);
      uint64_t part = 0;
      for (uint32_t i = 1 + (uint32_t)l; i < nseg; i += 64) part += t32[i + 1];
      total += wave_sum64(part);
    }
    if (total > limit) {  // :235
      stop = sTooLarge;
      break;
    }
    const uint64_t end = s + tw + total;
    const uint64_t he = end <= F.Tc ? F.head(end) : kNone;
    e = F.read_to(end, he);  // the segments: no run may cross the message end
    if (e) {
      stop = e;
      break;
    }
    if (l == 0) {
      msg_word_off[k] = s;
      msg_in_off[k] = hs;
      status[k] = sOK;
    }
    k++;
    prevL = L;
    L = nseg == 1 ? tw + total : 0;
    s = end;
    hs = he;
  }
  if (l == 0) {
    msg_word_off[k] = s;
    msg_in_off[k] = hs;
    status[k] = stop;
    *nmsgs = k;
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

}  // namespace

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

hipError_t launch_set_u64x4(uint64_t* dst, uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3,
                            hipStream_t stream) {
  set4_kernel<<<1, 64, 0, stream>>>(dst, v0, v1, v2, v3);
  return hipGetLastError();
}

hipError_t launch_split_walk(const uint8_t* packed, uint64_t nbytes, const uint64_t* words,
                             const uint64_t* rec_pos, const uint64_t* meta, uint64_t max_msgs,
                             uint64_t limit, uint64_t* msg_word_off, uint64_t* msg_in_off,
                             int32_t* status, uint64_t* nmsgs, hipStream_t stream) {
  Flat F;
  F.packed = packed;
  F.nbytes = nbytes;
  F.rec_pos = rec_pos;
  F.Bc = F.Tc = 0;
  F.capped = false;
  split_walk_kernel<<<1, 64, 0, stream>>>(F, words, meta, max_msgs, limit, msg_word_off,
                                          msg_in_off, status, nmsgs);
  return hipGetLastError();
}

}  // namespace cpk
