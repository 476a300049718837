// sz4_dict.hip -- dictionary mode on the whole GPU (smallz4.h:544-571 prepends the dictionary, the
// match loop at smallz4.h:603-760 is the usual one).
//
// With a dictionary every block starts at 65535 mod 65536, so the reference writes a chain entry at
// the block-relative slot i & 65535 (smallz4.h:656) and reads it back at the absolute slot
// pos & 65535 (smallz4.h:190, 200, 694): a read finds the entry of the neighbouring position, and the
// chains stop being runs of one key.  They are still a pure function of the insertion order:
//   * previousHash of an inserted position is the distance to the last earlier inserted position with
//     the same getHash32 (smallz4.h:648-666) -- a sort by (hash, position);
//   * the value a read of slot s sees at insertion step t is the one the latest insertion at or
//     before t with block-relative index == s (mod 65536) wrote (read_slot below): O(1) per read, from
//     the arrays of every position's previousHash / previousExact;
//   * previousExact (smallz4.h:668-720) is the hash-chain walk over those snapshot reads, and
//     findLongestMatch (smallz4.h:173-255) the exact-chain walk over them: one lane per position.
// The same-letter shortcut (smallz4.h:631-643) makes the set of inserted positions depend on the
// matches: a position after a distance-1 match longer than MaxSameLetter is neither inserted nor
// searched and copies that match one byte shorter.  The kernels take an ASSUMED set of shortcut
// intervals per block (the plan's interval lists), and k_dict_sc_bits / k_dict_sc derive from the
// results the intervals the reference's loop would take; where they differ the host runs the chunk
// again from its saved tables with the derived set.  Up to the first disagreement both sets are equal,
// and at it the derived one is right (its prefix was computed from the reference's state), so every
// round confirms a longer prefix and the rounds end (tools/dict_model.py model-checks this).
// Legacy frames (smallz4.h:806-817 resets the tables after every block, and nothing is inserted before
// a block, lookback 0) are the same computation with independent blocks.
//
//   k_dict_begin    the carried tables: reset (first chunk) or shifted with the staged coordinates
//   k_dict_keys     per block: (hash << 23 | position) of its own insertions (shortcut positions last)
//   (rocPRIM radix sort of the keys)
//   k_dict_ph       previousHash of every insertion: its predecessor in the sorted run of its hash
//   k_dict_last     the hash table's final positions (lastHash, smallz4.h:650-652)
//   k_dict_pe       previousExact of every insertion: the hash-chain walk over snapshot reads
//   k_dict_search   findLongestMatch of every linked position of every block; shortcut positions copy
//   k_dict_lz_*     greedy/lazy levels: the reference's skip bookkeeping (smallz4.h:726-744), walked
//                   speculatively per 4096-position sub-segment and repaired per block
//   k_dict_carry    the final chain tables, for the next chunk
//   k_dict_sc_bits, k_dict_sc   the shortcut intervals the results imply, compared with the assumed ones
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

#include "sz4_device.h"
#include "sz4_internal.h"

namespace sz4 {

constexpr uint32_t kDictNoPos = 0xFFFFFFFFu;
constexpr uint32_t kDictPosBits = 23;  // a block's insertions and the 64 KiB below them: < 2^23 positions
constexpr uint64_t kDictPosMask = (1ull << kDictPosBits) - 1;
constexpr uint32_t kDictSkipKey = 1u << kHashBits;  // k_dict_keys: a shortcut position (sorts after every hash)
constexpr uint32_t kDictSortBits = kHashBits + 1 + kDictPosBits;

// the insertion steps of one chunk: block b inserts block-relative i = back(b) .. size - 12
// (smallz4.h:612-625, 627) minus its shortcut intervals; every block but the stream's first re-inserts
// the previous block's last 12 positions, and the first of them (i = -12) was that block's last
// insertion: a duplicate whose entries are both EndOfChain (its lastHash is itself, distance 0).
// Legacy frames insert nothing before a block (lookback 0) and start every block from empty tables.
struct DictPlan {
  const Block* blocks;
  uint32_t nb;
  uint32_t cont;      // the first block continues the previous chunk's stream
  uint32_t dictBack;  // first chunk: insertions start this far before block 0
  uint32_t low0;      // reference dataZero at the first block (cont only)
  uint32_t legacy;    // independent blocks (tables reset per block, lookback 0)
  const Interval* iv;        // assumed shortcut intervals: block b's at iv[b * kMaxIv], ivCount[b] of them
  const uint32_t* ivCount;
  const uint2* runTab;       // runs covering whole 64-byte chunks (k_dict_runs), from runBase
  uint64_t runBase, runChunks;

  __host__ __device__ __forceinline__ int64_t back(uint32_t b) const
  {
    if (legacy) return 0;
    return (b == 0 && !cont) ? -(int64_t)dictBack : -(int64_t)kTailNoMatch;
  }
  __host__ __device__ __forceinline__ bool dup_block(uint32_t b) const { return !legacy && (b != 0 || cont); }
  // first position whose entries block b computes (the duplicate excluded), given its start
  __host__ __device__ __forceinline__ int64_t own_lo_at(uint32_t b, uint64_t start) const
  {
    return (int64_t)start + (dup_block(b) ? -(int64_t)kTailNoMatch + 1 : back(b));
  }
  __device__ __forceinline__ int64_t own_lo(uint32_t b) const { return own_lo_at(b, blocks[b].start); }
  __device__ __forceinline__ int64_t own_hi(uint32_t b) const { return (int64_t)blocks[b].end - kTailNoMatch; }
  // reference dataZero while block b is compressed (smallz4.h:799-804 keeps the last 64 KiB - 1)
  __device__ __forceinline__ uint64_t low(uint32_t b) const
  {
    if (legacy) return blocks[b].start;  // only the block's own positions are in the tables
    const int64_t l0 = cont ? (int64_t)low0 : 0;
    if (b == 0) return (uint64_t)l0;
    const int64_t l = (int64_t)blocks[b - 1].end - (int64_t)kWindow;
    return (uint64_t)(l > l0 ? l : l0);
  }
  // is absolute position pos inside an assumed shortcut interval of block b
  __device__ __forceinline__ bool skipped(uint32_t b, uint64_t pos) const
  {
    const uint32_t n = ivCount[b];
    const Interval* v = iv + (uint64_t)b * kMaxIv;
    for (uint32_t k = 0; k < n; k++)
      if (pos >= v[k].lo && pos < v[k].hi) return true;
    return false;
  }
  // the latest block-relative index <= iw of block b that is == iw (mod 65536) and was inserted: a
  // shortcut position writes no chain entry, so its slot still holds the one from 65536 indices back
  __device__ __forceinline__ int64_t inserted_at_or_below(uint32_t b, uint64_t start, int64_t iw) const
  {
    const uint32_t n = ivCount[b];
    if (!n) return iw;
    const Interval* v = iv + (uint64_t)b * kMaxIv;
    int64_t pos = (int64_t)start + iw;
    for (int32_t k = (int32_t)n - 1; k >= 0; k--)  // intervals ascend: a jump only lands lower
      if (pos >= (int64_t)v[k].lo && pos < (int64_t)v[k].hi)
        pos -= (((pos - (int64_t)v[k].lo) >> 16) + 1) << 16;
    return pos - (int64_t)start;
  }
};

// the entry slot s holds at insertion step (b, it) of the chunk: written by the latest insertion at or
// before it with block-relative index == s (mod 65536), or carried from the previous chunk (legacy:
// nothing before the block, the tables start empty).  `tab` holds every non-duplicate insertion's entry
// at its staged position.
__device__ __forceinline__ uint32_t read_slot(const DictPlan& P, const uint16_t* __restrict__ tab,
                                              const uint16_t* __restrict__ carried, uint32_t s, uint32_t b, int64_t it,
                                              uint64_t start, int64_t lo)
{
  int64_t iw = P.inserted_at_or_below(b, start, it - ((it - (int64_t)s) & (int64_t)kWindow));
  if (iw >= lo) {  // in the current block (the common case)
    if (iw == -(int64_t)kTailNoMatch && P.dup_block(b)) return 0u;
    return tab[start + iw];
  }
  if (P.legacy) return 0u;
  for (int32_t bb = (int32_t)b - 1; bb >= 0; bb--) {
    const Block B = P.blocks[bb];
    const int64_t hi = (int64_t)(B.end - B.start) - kTailNoMatch;
    iw = P.inserted_at_or_below((uint32_t)bb, B.start, hi - ((hi - (int64_t)s) & (int64_t)kWindow));
    if (iw >= P.back((uint32_t)bb)) {
      if (iw == -(int64_t)kTailNoMatch && P.dup_block((uint32_t)bb)) return 0u;
      return tab[B.start + iw];
    }
  }
  return carried[s];
}

// ---- runs of one byte value (the chains' 1-hop stretches) ------------------------------------------
// runTab[k] for the 64-byte chunk k of the chunk's staged range (from base, 64-aligned): {first, end} of
// the run of one byte value that covers the whole chunk, {0, 0} when the chunk is not uniform
__global__ __launch_bounds__(256) void k_dict_run_flags(const uint8_t* __restrict__ in, uint64_t base, uint64_t nchunks,
                                                        uint32_t* __restrict__ flag)
{
  const uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (k >= nchunks) return;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in + base + k * 64);
  const uint32_t v = w[0] & 0xFFu, all = v * 0x01010101u;
  bool u = true;
#pragma unroll
  for (int j = 0; j < 16; j++) u &= w[j] == all;
  flag[k] = u ? v + 1u : 0u;
}

// one wavefront per 64 chunks: every run head among them (a uniform chunk whose predecessor is not the
// same byte) measures its run -- back to its first byte (>= lo), forward over the uniform chunks, then
// into the chunk after them (< hi) -- and writes it to all its chunks
// The first round's guess of the same-letter shortcut intervals, from a run [first, end) of more than
// MaxSameLetter + 1 bytes: in a block it starts at the run, the first position whose chain begins with
// the distance-1 candidate is first + 2 (the chain of p starts at the entry of p - 1, and the run's first
// position has no distance-1 predecessor); a run that comes in from the previous block is met at the
// block start (its last position before the block is a lookback insertion; legacy frames have none).
// Appended to the block's list; k_dict_sc checks every guess like any assumed interval.
__device__ __forceinline__ void dict_guess(const Block* __restrict__ blocks, uint32_t nb, uint32_t legacy, uint64_t first,
                                           uint64_t end, Interval* __restrict__ ivAll, uint32_t* __restrict__ ivCount)
{
  if (end - first <= (uint64_t)kSameLetter + 1) return;
  for (uint32_t b = 0; b < nb; b++) {
    const Block B = blocks[b];
    if (B.end <= first || B.start >= end) continue;
    const uint64_t a = (first < B.start && !legacy) ? B.start : (first > B.start ? first : B.start) + 2;
    const uint64_t lim = end < B.end - kTailLiterals ? end : B.end - kTailLiterals;
    if (lim <= a || lim - a <= (uint64_t)kSameLetter || a + kTailNoMatch > B.end) continue;
    const uint64_t La = lim - a;
    const uint32_t k = atomicAdd(&ivCount[b], 1u);
    if (k >= kMaxIv) continue;  // k_dict_sc clamps the count
    Interval x;
    x.a = a;
    x.La = La;
    x.lo = a + 1;
    x.hi = a + 1 + (La - kSameLetter);
    ivAll[(uint64_t)b * kMaxIv + k] = x;
  }
}

// the guessed intervals of each block in position order (few: one thread per block)
__global__ __launch_bounds__(64) void k_dict_guess_sort(uint32_t nb, Interval* __restrict__ ivAll, uint32_t* __restrict__ ivCount)
{
  const uint32_t b = blockIdx.x * 64 + threadIdx.x;
  if (b >= nb) return;
  const uint32_t n = ivCount[b] < kMaxIv ? ivCount[b] : kMaxIv;
  ivCount[b] = n;
  Interval* v = ivAll + (uint64_t)b * kMaxIv;
  for (uint32_t i = 1; i < n; i++) {
    const Interval x = v[i];
    uint32_t j = i;
    while (j > 0 && v[j - 1].lo > x.lo) {
      v[j] = v[j - 1];
      j--;
    }
    v[j] = x;
  }
}

__global__ __launch_bounds__(64) void k_dict_runs(const uint8_t* __restrict__ in, uint64_t base, uint64_t nchunks, uint64_t lo,
                                                  uint64_t hi, const uint32_t* __restrict__ flag, uint2* __restrict__ runTab,
                                                  const Block* __restrict__ blocks, uint32_t nb, uint32_t legacy,
                                                  Interval* __restrict__ ivAll, uint32_t* __restrict__ ivCount)
{
  const uint32_t lane = threadIdx.x;
  const uint64_t k = (uint64_t)blockIdx.x * 64 + lane;
  const uint32_t f = k < nchunks ? flag[k] : 0u;
  const uint32_t fp = k < nchunks && k > 0 ? flag[k - 1] : 0u;
  if (k < nchunks && f == 0u) runTab[k] = make_uint2(0u, 0u);
  uint64_t heads = __ballot(f != 0u && fp != f);
  while (heads) {
    const uint32_t l = (uint32_t)__builtin_ctzll(heads);
    heads &= heads - 1;
    const uint64_t h = (uint64_t)blockIdx.x * 64 + l;
    const uint32_t v = rdlane(f, l) - 1u;
    // first byte: the last non-v byte in the 64 before the chunk, + 1
    const uint64_t c0 = base + h * 64;
    const int64_t q = (int64_t)c0 - 64 + (int64_t)lane;
    const uint64_t om = __ballot(q < (int64_t)lo || in[q] != v);  // bytes before lo count as "not v"
    uint64_t first = om ? c0 - 64 + (uint64_t)(63 - __builtin_clzll(om)) + 1 : c0 - 64;
    if (first < lo) first = lo;
    // the uniform chunks of the run, 64 at a time
    uint64_t j = h + 1;
    while (true) {
      const uint64_t jj = j + lane;
      const bool same = jj < nchunks && flag[jj] == v + 1u;
      const uint64_t stop = __ballot(!same);
      if (stop) {
        j += (uint64_t)__builtin_ctzll(stop);
        break;
      }
      j += 64;
    }
    // into chunk j (not uniform v): its leading v bytes
    const uint64_t e0 = base + j * 64, e = e0 + lane;
    const uint64_t nm = __ballot(e >= hi || in[e] != v);
    const uint64_t end = nm ? e0 + (uint64_t)__builtin_ctzll(nm) : e0 + 64;
    for (uint64_t t = h + lane; t < j; t += 64) runTab[t] = make_uint2((uint32_t)first, (uint32_t)(end < hi ? end : hi));
    if (ivAll && lane == 0) dict_guess(blocks, nb, legacy, first, end < hi ? end : hi, ivAll, ivCount);
  }
}

__global__ __launch_bounds__(256) void k_dict_begin(uint32_t* __restrict__ last, uint16_t* __restrict__ prevH,
                                                    uint16_t* __restrict__ prevX, uint32_t cont, uint32_t shift)
{
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  if (j >= (1u << kHashBits)) return;
  if (!cont) {
    last[j] = kDictNoPos;
    if (j < 65536u) {
      prevH[j] = 0;
      prevX[j] = 0;
    }
  } else {
    // chain slots are absolute positions mod 65536, unchanged by a shift that is a multiple of
    // 65536; positions below the carried bytes become "no entry" (more than MaxDistance away)
    const uint32_t v = last[j];
    last[j] = (v == kDictNoPos || v < shift) ? kDictNoPos : v - shift;
  }
}

// block b's own insertions [ownLo, ownLo + n): (hash << kDictPosBits | index); a shortcut position
// gets kDictSkipKey and sorts after every hash (never a predecessor, never in the hash table)
__global__ __launch_bounds__(256) void k_dict_keys(const uint8_t* __restrict__ in, DictPlan P, uint32_t b, uint64_t ownLo,
                                                   uint32_t n, uint64_t* __restrict__ keys)
{
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  if (j >= n) return;
  const uint64_t p = ownLo + j;
  const uint32_t h = P.skipped(b, p) ? kDictSkipKey : ref_hash(gload4(in, p));
  keys[j] = ((uint64_t)h << kDictPosBits) | j;
}

// previousHash (smallz4.h:648-666): the predecessor in the sorted run of the hash, else the hash
// table left by the earlier blocks and chunks (legacy: empty before every block)
__global__ __launch_bounds__(256) void k_dict_ph(const uint64_t* __restrict__ keys, uint32_t n, uint64_t ownLo,
                                                 const uint32_t* __restrict__ last, uint16_t* __restrict__ ph,
                                                 uint32_t legacy)
{
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  if (j >= n) return;
  const uint64_t k = keys[j];
  const uint32_t h = (uint32_t)(k >> kDictPosBits);
  if (h == kDictSkipKey) return;
  const uint64_t p = ownLo + (k & kDictPosMask);
  uint64_t d = kNone;
  if (j > 0 && (uint32_t)(keys[j - 1] >> kDictPosBits) == h) {
    d = p - (ownLo + (keys[j - 1] & kDictPosMask));
  } else if (!legacy) {
    const uint32_t q = last[h];  // the previous chunk's (or an earlier block's) lastHash
    if (q != kDictNoPos && q < p) d = p - q;
  }
  ph[p] = d <= kWindow ? (uint16_t)d : (uint16_t)0;
}

__global__ __launch_bounds__(256) void k_dict_last(const uint64_t* __restrict__ keys, uint32_t n, uint64_t ownLo,
                                                   uint32_t* __restrict__ last)
{
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  if (j >= n) return;
  const uint64_t k = keys[j];
  const uint32_t h = (uint32_t)(k >> kDictPosBits);
  if (h != kDictSkipKey && (j + 1 == n || (uint32_t)(keys[j + 1] >> kDictPosBits) != h))
    last[h] = (uint32_t)(ownLo + (k & kDictPosMask));
}

// previousExact (smallz4.h:668-720): from the previousHash candidate, follow the hash chain through
// snapshot reads while the hash still matches; grid (positions, blocks)
__global__ __launch_bounds__(256) void k_dict_pe(const uint8_t* __restrict__ in, DictPlan P,
                                                 const uint16_t* __restrict__ ph, const uint16_t* __restrict__ prevH0,
                                                 uint16_t* __restrict__ pe)
{
  const uint32_t b = blockIdx.y;
  const int64_t lo = P.own_lo(b), hi = P.own_hi(b);
  const int64_t p = lo + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p > hi) return;
  if (P.skipped(b, (uint64_t)p)) {  // a shortcut position: not inserted, not linked
    pe[p] = 0;
    return;
  }
  const uint64_t start = P.blocks[b].start;
  const int64_t it = p - (int64_t)start, back = P.back(b);
  const uint64_t low = P.low(b);
  const uint32_t first = ph[p];
  uint32_t exact = 0;
  if (first) {
    const uint32_t four = gload4(in, (uint64_t)p), h = ref_hash(four);
    uint64_t cand = (uint64_t)p - first, dist = first;
    bool ok = true;
    while (true) {
      if (cand < low) {  // the reference would read before its buffer
        ok = false;
        break;
      }
      const uint32_t seen = gload4(in, cand);
      if (seen == four) break;
      if (ref_hash(seen) != h) {
        ok = false;
        break;
      }
      const uint32_t step = read_slot(P, ph, prevH0, (uint32_t)(cand & kWindow), b, it, start, back);
      if (!step) {
        ok = false;
        break;
      }
      dist += step;
      if (dist > kWindow) {
        ok = false;
        break;
      }
      cand -= step;
    }
    exact = ok ? (uint32_t)dist : 0u;
  }
  pe[p] = (uint16_t)exact;
}

// findLongestMatch (smallz4.h:173-255) of every linked position (previousExact set) of every block,
// over snapshot reads of the exact chains: strictly longer replaces, maxChain counts replacements.
// Every other position gets (0, 0): not searched.  Grid (position ranges, blocks).
// The chains' lengths are skewed (text: 76 hops on average, 1350 at the 99th percentile), so a wavefront
// takes kDictSearchPer * 64 consecutive positions as a queue: a lane takes the next one whenever its
// walk ends, one hop per loop turn, and the wavefront runs for about the mean, not 64 maxima.
// (8 waves per SIMD: the chain walks are latency-bound)
constexpr uint32_t kDictSearchPer = 8;
constexpr uint32_t kDictSearchSpan = 64 * kDictSearchPer;  // positions per wavefront
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8), amdgpu_num_sgpr(80))) void k_dict_search(const uint8_t* __restrict__ in, DictPlan P, uint32_t maxChain,
                                                     const uint16_t* __restrict__ pe, const uint16_t* __restrict__ prevX0,
                                                     uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist,
                                                     uint32_t* __restrict__ sel, uint32_t* __restrict__ longFlag)
{
  const uint32_t b = blockIdx.y;
  const Block B = P.blocks[b];
  const uint32_t size = (uint32_t)(B.end - B.start);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t first = (blockIdx.x * 4u + (threadIdx.x >> 6)) * kDictSearchSpan;
  if (first >= size) return;
  const uint32_t last = first + kDictSearchSpan < size ? first + kDictSearchSpan : size;
  const int64_t back = P.back(b);
  const uint64_t stop = B.end - kTailLiterals;
  const bool hasIv = P.ivCount[b] != 0;
  uint32_t cursor = first;  // the wavefront's next untaken position (uniform)
  uint32_t i = 0, bestLen = 0, bestDist = 0, steps = 0, hop = 0;
  uint64_t pos = 0, backDist = 0;
  int64_t room = 0, twAt = -1;  // tw: the target's word at twAt (phase 1's first compare)
  uint32_t tw = 0;
  bool walking = false, live = false, rmq = false;
  while (true) {
    // lanes without a position take the next ones, in lane order
    const uint64_t want = __ballot(!walking);
    if (want) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
      if (!walking) {
        i = cursor + rank;
        live = i < last;
      }
      cursor += (uint32_t)__builtin_popcountll(want);
      if (!walking && live) {
        pos = B.start + i;
        if (maxChain > (uint32_t)kGreedyMax && i + kTailLiterals >= size) sel[pos] = 0;
        bestLen = 0;
        bestDist = 0;
        if (hasIv && P.skipped(b, pos)) {
          // same-letter shortcut (smallz4.h:636-641): the interval's distance-1 match, one byte shorter per step
          const Interval* v = P.iv + (uint64_t)b * kMaxIv;
          uint32_t k = 0;
          while (!(pos >= v[k].lo && pos < v[k].hi)) k++;
          bestLen = (uint32_t)(v[k].La - (pos - v[k].a));
          bestDist = 1;
        } else if (i + kTailNoMatch <= size && pe[pos] != 0) {
          bestLen = 1;
          steps = maxChain;
          hop = read_slot(P, pe, prevX0, (uint32_t)(pos & kWindow), b, (int64_t)i, B.start, back);
          backDist = 0;
          room = (int64_t)(stop - pos);
          twAt = -1;
          walking = true;
        }
        if (!walking) {
          mlen[pos] = bestLen;
          mdist[pos] = (uint16_t)bestDist;
          rmq |= bestLen >= kRmqLen && !(bestDist == 1u && bestLen >= kSameLetter);
        }
      }
    }
    if (!__ballot(walking)) {
      if (cursor >= last) break;
      continue;
    }
    if (walking) {
      // one candidate of the walk
      bool done = hop == 0;
      if (!done) {
        backDist += hop;
        done = backDist > kWindow;
      }
      if (!done) {
        hop = read_slot(P, pe, prevX0, (uint32_t)((pos - backDist) & kWindow), b, (int64_t)i, B.start, back);
        const int64_t need = (int64_t)bestLen + 1;
        done = need > room;
        if (!done) {
          uint64_t c = pos - backDist;
          if (hop == 1u && bestLen >= 4u) {
            // In a run of one byte value v every inserted position's exact predecessor is the one before it,
            // so the chain steps down the run one position at a time.  Once p holds a match of bestLen and
            // its byte at bestLen is not v, a candidate c' of the run with c' + need <= run end fails the
            // first word of phase 1 (bytes need-4 .. need-1: p's differ from v at bestLen, c''s are all v):
            // the whole stretch is rejected, and the walk continues at its bottom c_j with the hop read there.
            // Stretch: read at y gives 1 for y in (c_j, c] when y - 1 and y - 2 are inserted positions of
            // the run's interior (first + 1 .. end - 4) of this block (no shortcut interval among them).
            const uint64_t rk = (c - P.runBase) >> 6;
            const uint2 rt = c >= P.runBase && rk < P.runChunks ? P.runTab[rk] : make_uint2(0u, 0u);
            if (rt.y != 0u && c + (uint64_t)need <= rt.y && c + 3 <= rt.y && in[pos + bestLen] != in[c]) {
              uint64_t cj = max((uint64_t)rt.x + 2, B.start + 2);
              const uint32_t niv = P.ivCount[b];
              const Interval* v = P.iv + (uint64_t)b * kMaxIv;
              bool inside = false;
              for (uint32_t k = 0; k < niv; k++) {
                if (c >= v[k].lo && c < v[k].hi) inside = true;
                if (v[k].hi <= c && v[k].hi + 2 > cj) cj = v[k].hi + 2;
              }
              if (!inside && cj < c && pos - cj <= kWindow) {
                c = cj;
                backDist = pos - cj;
                hop = read_slot(P, pe, prevX0, (uint32_t)(cj & kWindow), b, (int64_t)i, B.start, back);
              }
            }
          }
          // phase 1: the bytes between the first one and the first new one, backwards (never bytes 0-3); the
          // target's first word of it changes only with bestLen: kept in a register (one load per hop fewer)
          int64_t lo = need - 4;
          if (lo > 0) {
            if (twAt != lo) {
              tw = gload4(in, pos + lo);
              twAt = lo;
            }
            if (tw == gload4(in, c + lo)) {
              lo -= 4;
              while (lo > 0 && gload4(in, pos + lo) == gload4(in, c + lo)) lo -= 4;
            }
          }
          if (lo <= 0) {
            // phase 2: forward from the first new byte; 32 bytes per step while they all agree (the loads of
            // a step are independent: one latency per 32 bytes in a long run instead of one per 4)
            int64_t hi = need;
            while (hi + 32 <= room) {
              uint32_t x = 0;
#pragma unroll
              for (int k = 0; k < 32; k += 4) x |= gload4(in, pos + hi + k) ^ gload4(in, c + hi + k);
              if (x) break;
              hi += 32;
            }
            while (hi + 4 <= room && gload4(in, pos + hi) == gload4(in, c + hi)) hi += 4;
            while (hi < room && in[pos + hi] == in[c + hi]) hi++;
            bestLen = (uint32_t)hi;
            bestDist = (uint32_t)backDist;
            done = --steps == 0;
          }
        }
      }
      if (done) {
        mlen[pos] = bestLen;
        mdist[pos] = (uint16_t)bestDist;
        rmq |= bestLen >= kRmqLen && !(bestDist == 1u && bestLen >= kSameLetter);
        walking = false;
      }
    }
  }
  // optimal levels search every linked position: the parse's range-minimum flag is set here
  if (maxChain > (uint32_t)kLazyMax && __ballot(rmq) && lane == 0) atomicOr(longFlag + b, kFlagRmq);
}

// Greedy/lazy levels: the skip bookkeeping (smallz4.h:726-744) over the linked positions of a block
// (previousExact set, i >= 0).  Between searches the reference's state is (next searched position,
// mode, carry):
//   fresh search at q (skip 0), length L:  L == 1 -> the next linked position is searched fresh;
//                                          else   -> the next one is searched lazily, carry = L - 1;
//   lazy search at q, length L2:           the next (L2 != 1 ? L2 : carry) linked positions are
//                                          skipped, the one after is searched fresh.
// (A search that finds nothing, length 1, is possible here: the snapshot chains need not lead to a
// match.)  A fresh position fixes the whole future, so the chain is walked speculatively per
// kWalkSeg sub-segment from its first linked position (k_dict_lz_walk: searched and fresh positions as
// bit masks), k_dict_lz_fix walks a block's sub-segments in order and re-walks from the true entry until
// it reaches a position the speculative walk searched fresh, and k_dict_lz_clear clears the linked
// positions nobody searched.  Masks: kWalkSeg bits each, [fresh | kept] per sub-segment.
constexpr uint32_t kLzWords = kWalkSeg / 32;
// per sub-segment: [fresh | kept | the join's re-walked positions] bit masks, then the join's record (4 words)
constexpr uint32_t kLzStride = 3 * kLzWords + 4;
constexpr uint32_t kLzEnd = 0x7FFFFFFFu;

// the need-th (0-based) linked position at or after pos over a register window of 64 positions
// (loads three windows ahead, unconditional with a clamped index as in k_walk)
struct DictWalker {
  const uint32_t* L;
  const uint16_t* E;
  uint32_t last;  // inclusive
  uint32_t wbase, wL, wE, xL1, xE1, xL2, xE2, xL3, xE3;
  __device__ __forceinline__ void ld(uint32_t b, uint32_t& l, uint32_t& e) const
  {
    const uint32_t i = b + lane_id();
    const uint32_t j = i <= last ? i : last;
    l = L[j];
    e = E[j];
  }
  __device__ __forceinline__ void start(uint32_t pos)
  {
    wbase = pos & ~63u;
    ld(wbase, wL, wE);
    ld(wbase + 64, xL1, xE1);
    ld(wbase + 128, xL2, xE2);
    ld(wbase + 192, xL3, xE3);
  }
  __device__ __forceinline__ uint32_t next(uint32_t pos, uint32_t need)
  {
    while (pos <= last) {
      while (pos >= wbase + 64) {
        if (pos < wbase + 256) {
          wbase += 64;
          wL = xL1;
          wE = xE1;
          xL1 = xL2;
          xE1 = xE2;
          xL2 = xL3;
          xE2 = xE3;
          ld(wbase + 192, xL3, xE3);
        } else {
          start(pos);
        }
      }
      const uint64_t mask = __ballot(wE != 0u && wbase + lane_id() <= last) & (~0ull << (pos - wbase));
      const uint32_t pc = (uint32_t)__popcll(mask);
      if (need < pc) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        const uint64_t hit = __ballot(((mask >> lane_id()) & 1ull) && below == need);
        return wbase + (uint32_t)__builtin_ctzll(hit);
      }
      need -= pc;
      pos = wbase + 64;
    }
    return kLzEnd;
  }
  __device__ __forceinline__ uint32_t len(uint32_t q) const { return rdlane(wL, q - wbase); }
};

// one step of the chain from the searched position q (mode md: 0 fresh, 1 lazy; carry: see above)
__device__ __forceinline__ uint32_t lz_step(DictWalker& w, uint32_t q, uint32_t& md, uint32_t& carry)
{
  const uint32_t L = w.len(q);
  if (md == 0u) {
    if (L != 1u) {
      carry = L - 1u;
      md = 1u;
    }
    return w.next(q + 1, 0u);
  }
  md = 0u;
  return w.next(q + 1, L != 1u ? L : carry);
}

__device__ __forceinline__ void lz_setbit(uint32_t* m, uint32_t i)
{
  if (lane_id() == 0) m[i >> 5] |= 1u << (i & 31);
}

__global__ __launch_bounds__(64 * 4) void k_dict_lz_walk(const Block* __restrict__ blocks, const uint2* __restrict__ walkSegs,
                                                         uint32_t nwalk, const uint32_t* __restrict__ mlen,
                                                         const uint16_t* __restrict__ pe, uint32_t* __restrict__ masks,
                                                         uint4* __restrict__ state)
{
  __shared__ uint32_t bits[4][2 * kLzWords];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * 4 + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch) return;
  uint32_t* fresh = bits[wave];
  uint32_t* kept = fresh + kLzWords;
  for (uint32_t t = lane; t < 2 * kLzWords; t += 64) fresh[t] = 0;
  const uint32_t a = ws.y * kWalkSeg, aNext = a + kWalkSeg < n ? a + kWalkSeg : n;
  DictWalker w;
  w.L = mlen + B.start;
  w.E = pe + B.start;
  w.last = n - kTailNoMatch;
  w.start(a);
  uint32_t md = 0, carry = 0;
  uint32_t q = w.next(a, 0u);  // assumed: the sub-segment's first linked position, searched fresh
  __builtin_amdgcn_wave_barrier();
  while (q < aNext) {
    lz_setbit(kept, q - a);
    if (md == 0u) lz_setbit(fresh, q - a);
    q = lz_step(w, q, md, carry);
  }
  __builtin_amdgcn_wave_barrier();
  uint32_t* out = masks + (uint64_t)idx * kLzStride;
  for (uint32_t t = lane; t < 2 * kLzWords; t += 64) out[t] = fresh[t];
  if (lane == 0) state[idx] = make_uint4(q, md, carry, 0u);
}

// every sub-segment k >= 1 joined at once from an ASSUMED entry, sub-segment k - 1's speculative exit (the
// true one whenever k - 1's true walk reached a position its speculative walk searched fresh): re-walked
// from there until it reaches such a position of its own walk (merged) or leaves the sub-segment.  The
// re-walked positions go to the third mask, the record (exit q, mode, carry, 1 | merged << 1 | from << 2)
// after it; k_dict_lz_fix keeps the joins whose assumption holds.
__global__ __launch_bounds__(64 * 4) void k_dict_lz_join(const Block* __restrict__ blocks, const uint2* __restrict__ walkSegs,
                                                         uint32_t nwalk, const uint32_t* __restrict__ mlen,
                                                         const uint16_t* __restrict__ pe, uint32_t* __restrict__ masks,
                                                         const uint4* __restrict__ state)
{
  __shared__ uint32_t bits[4][2 * kLzWords];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * 4 + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  if (ws.y == 0) return;
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch) return;
  uint32_t* m = masks + (uint64_t)idx * kLzStride;
  const uint4 ex = state[idx - 1];
  const uint32_t a = ws.y * kWalkSeg, aNext = a + kWalkSeg < n ? a + kWalkSeg : n;
  uint32_t q = ex.x, md = ex.y, carry = ex.z;
  if (q >= aNext) {  // nothing searched here: k_dict_lz_fix's own loop (cheap)
    if (lane == 0) m[3 * kLzWords + 3] = 0u;
    return;
  }
  uint32_t* fresh = bits[wave];
  uint32_t* rep = fresh + kLzWords;
  for (uint32_t t = lane; t < kLzWords; t += 64) {
    fresh[t] = m[t];
    rep[t] = 0;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  auto is_fresh = [&](uint32_t p) { return (fresh[(p - a) >> 5] >> ((p - a) & 31)) & 1u; };
  bool merged = md == 0u && is_fresh(q);
  if (!merged) {
    DictWalker w;
    w.L = mlen + B.start;
    w.E = pe + B.start;
    w.last = n - kTailNoMatch;
    w.start(q);
    (void)w.next(q, 0u);
    while (q < aNext) {
      if (md == 0u && is_fresh(q)) {
        merged = true;
        break;
      }
      lz_setbit(rep, q - a);
      q = lz_step(w, q, md, carry);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  for (uint32_t t = lane; t < kLzWords; t += 64) m[2 * kLzWords + t] = rep[t];
  const uint32_t from = merged ? q - a : kWalkSeg;
  if (lane == 0) {
    const uint4 sp = state[idx];
    const uint4 rec = merged ? make_uint4(sp.x, sp.y, sp.z, 1u | 2u | (from << 2)) : make_uint4(q, md, carry, 1u | (from << 2));
    m[3 * kLzWords + 0] = rec.x;
    m[3 * kLzWords + 1] = rec.y;
    m[3 * kLzWords + 2] = rec.z;
    m[3 * kLzWords + 3] = rec.w;
  }
}

__global__ __launch_bounds__(64) void k_dict_lz_fix(const Block* __restrict__ blocks, const uint32_t* __restrict__ mlen,
                                                    const uint16_t* __restrict__ pe, uint32_t* __restrict__ masks,
                                                    uint4* __restrict__ state)
{
  __shared__ uint32_t fresh[kLzWords], rep[kLzWords];
  const Block B = blocks[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch || B.walkCount < 2) return;
  DictWalker w;
  w.L = mlen + B.start;
  w.E = pe + B.start;
  w.last = n - kTailNoMatch;
  w.wbase = 0xFFFFFFC0u;  // no window loaded yet
  uint4 ex = state[B.walkFirst];  // sub-segment 0 was walked from the block start: exact
  uint4 prevSpec = ex;            // the speculative exit of the sub-segment before k (k_dict_lz_join's assumption)
  auto same = [](const uint4& x, const uint4& y) { return x.x == y.x && x.y == y.y && x.z == y.z; };
  for (uint32_t k = 1; k < B.walkCount;) {
    {
      // sub-segments k .. k + 63: lane j's join holds when its assumed entry (the speculative exit of
      // k + j - 1) is the true one: for j = 0 when it is ex, for j > 0 when lane j - 1's holds and its
      // join's exit is its speculative exit.  Up to the first that does not hold, all at once
      const uint32_t kj = k + lane;
      const bool in = kj < B.walkCount;
      const uint32_t idxj = B.walkFirst + (in ? kj : k);
      uint32_t* mj = masks + (uint64_t)idxj * kLzStride;
      const uint4 sj = state[idxj];
      const uint4 jr = in ? make_uint4(mj[3 * kLzWords], mj[3 * kLzWords + 1], mj[3 * kLzWords + 2], mj[3 * kLzWords + 3])
                          : make_uint4(0u, 0u, 0u, 0u);
      // this lane's join exit equals its speculative exit (then the next sub-segment's assumption holds)
      const bool exitIsSpec = (jr.w & 2u) != 0u;
      const bool prevOk = (__ballot(exitIsSpec) << 1 >> lane) & 1ull;  // lane j - 1's
      const bool holds = in && (jr.w & 1u) && (lane == 0 ? same(ex, prevSpec) : prevOk);
      const uint64_t notHeld = ~__ballot(holds);
      const uint32_t nOk = notHeld ? (uint32_t)__builtin_ctzll(notHeld) : 64u;
      for (uint32_t j = 0; j < nOk; j++) {
        // kept = the re-walked positions, then the speculative ones from the merge point on
        uint32_t* mm = masks + (uint64_t)(B.walkFirst + k + j) * kLzStride;
        const uint32_t from = rdlane(jr.w, j) >> 2;
        for (uint32_t t = lane; t < kLzWords; t += 64) {
          const uint32_t lo = t * 32;
          const uint32_t keepSpec = from <= lo ? 0xFFFFFFFFu : (from >= lo + 32 ? 0u : ~0u << (from - lo));
          mm[kLzWords + t] = mm[2 * kLzWords + t] | (mm[kLzWords + t] & keepSpec);
        }
      }
      if (nOk) {
        ex = make_uint4(rdlane(jr.x, nOk - 1u), rdlane(jr.y, nOk - 1u), rdlane(jr.z, nOk - 1u), 0u);
        prevSpec = make_uint4(rdlane(sj.x, nOk - 1u), rdlane(sj.y, nOk - 1u), rdlane(sj.z, nOk - 1u), 0u);
        k += nOk;
        if (nOk == 64u) continue;
      }
      if (k >= B.walkCount) break;
    }
    const uint32_t kc = k++;
    const uint32_t idx = B.walkFirst + kc;
    const uint4 spec = state[idx];
    prevSpec = spec;
    const uint32_t a = kc * kWalkSeg, aNext = a + kWalkSeg < n ? a + kWalkSeg : n;
    uint32_t* m = masks + (uint64_t)idx * kLzStride;
    uint32_t q = ex.x, md = ex.y, carry = ex.z;
    if (q >= aNext) {  // nothing searched in this sub-segment
      for (uint32_t t = lane; t < kLzWords; t += 64) m[kLzWords + t] = 0;
      continue;  // ex unchanged: the entry of the next sub-segment
    }
    for (uint32_t t = lane; t < kLzWords; t += 64) {
      fresh[t] = m[t];
      rep[t] = 0;
    }
    __syncthreads();
    auto is_fresh = [&](uint32_t p) { return (fresh[(p - a) >> 5] >> ((p - a) & 31)) & 1u; };
    // the speculative walk is right from its first fresh position at or after the true entry on;
    // before it, re-walk from the true entry
    bool merged = md == 0u && is_fresh(q);
    if (!merged) {
      if (w.wbase == 0xFFFFFFC0u || q < w.wbase || q >= w.wbase + 256) w.start(q);
      (void)w.next(q, 0u);  // q is linked: brings its window in
      while (q < aNext) {
        if (md == 0u && is_fresh(q)) {
          merged = true;
          break;
        }
        lz_setbit(rep, q - a);
        q = lz_step(w, q, md, carry);
      }
    }
    __syncthreads();
    // kept = the re-walked positions, then the speculative ones from the merge point on
    const uint32_t from = merged ? q - a : kWalkSeg;
    for (uint32_t t = lane; t < kLzWords; t += 64) {
      const uint32_t lo = t * 32;
      const uint32_t keepSpec = from <= lo ? 0xFFFFFFFFu : (from >= lo + 32 ? 0u : ~0u << (from - lo));
      m[kLzWords + t] = rep[t] | (m[kLzWords + t] & keepSpec);
    }
    ex = merged ? spec : make_uint4(q, md, carry, 0u);
    __syncthreads();
  }
}

// linked positions no walk searched get (0, 0); the parse's range-minimum flag over the searched ones
__global__ __launch_bounds__(64 * 4) void k_dict_lz_clear(const Block* __restrict__ blocks, const uint2* __restrict__ walkSegs,
                                                          uint32_t nwalk, uint32_t* __restrict__ mlen,
                                                          uint16_t* __restrict__ mdist, const uint16_t* __restrict__ pe,
                                                          const uint32_t* __restrict__ masks, uint32_t* __restrict__ longFlag)
{
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * 4 + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch) return;
  const uint32_t last = n - kTailNoMatch;
  const uint32_t a = ws.y * kWalkSeg;
  const uint32_t hi = a + kWalkSeg - 1 < last ? a + kWalkSeg - 1 : last;  // inclusive
  const uint32_t* kept = masks + (uint64_t)idx * kLzStride + kLzWords;
  bool rmq = false;
  for (uint32_t x0 = a; x0 <= hi; x0 += 64) {
    const uint32_t x = x0 + lane;
    if (x > hi) break;
    const uint64_t p = B.start + x;
    const bool keep = (kept[(x - a) >> 5] >> ((x - a) & 31)) & 1u;
    if (!keep) {
      if (pe[p] != 0u) {
        mlen[p] = 0;
        mdist[p] = 0;
      }
    } else {
      const uint32_t L = mlen[p];
      if (L >= kRmqLen) rmq |= !(mdist[p] == 1u && L >= kSameLetter);
    }
  }
  if (__ballot(rmq) && lane == 0) atomicOr(longFlag + ws.x, kFlagRmq);
}

// the chain tables after the chunk's last insertion, in place (slot s reads only its own carried value)
__global__ __launch_bounds__(256) void k_dict_carry(DictPlan P, const uint16_t* __restrict__ ph,
                                                    const uint16_t* __restrict__ pe, uint16_t* __restrict__ prevH,
                                                    uint16_t* __restrict__ prevX)
{
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= 65536u) return;
  const uint32_t b = P.nb - 1;
  const Block B = P.blocks[b];
  const int64_t it = (int64_t)(B.end - B.start) - kTailNoMatch, back = P.back(b);
  if (it < back) return;  // no insertion in the chunk (not reached: every block inserts)
  const uint16_t h = (uint16_t)read_slot(P, ph, prevH, s, b, it, B.start, back);
  const uint16_t x = (uint16_t)read_slot(P, pe, prevX, s, b, it, B.start, back);
  prevH[s] = h;
  prevX[s] = x;
}


// ---- the shortcut intervals the results imply (smallz4.h:631-643) --------------------------------
// bit a of a block: block-relative a is searched (not assumed skipped) and found a distance-1 match
// longer than MaxSameLetter, so the reference's loop would skip a + 1 .. a + La - MaxSameLetter.
// Positions assumed skipped have no search result, so they start nothing (the next round searches them).
__global__ __launch_bounds__(256) void k_dict_sc_bits(DictPlan P, const uint32_t* __restrict__ mlen,
                                                      const uint16_t* __restrict__ mdist, uint64_t* __restrict__ bits,
                                                      uint64_t wordsPerBlock)
{
  const uint32_t b = blockIdx.y;
  const Block B = P.blocks[b];
  const uint64_t n = B.end - B.start;
  const uint64_t a = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (a >= ((n + 63) & ~63ull)) return;
  const uint64_t pos = B.start + a;
  // a + 1 must be a position of the loop: a + 1 + 12 <= n
  const bool q = a + 1 + kTailNoMatch <= n && mdist[pos] == 1u && mlen[pos] > kSameLetter && !P.skipped(b, pos);
  const uint64_t m = __ballot(q);
  if (lane_id() == 0) bits[(uint64_t)b * wordsPerBlock + (a >> 6)] = m;
}

// one wavefront per block: the intervals in the order the reference's loop meets them (a start inside an
// interval already taken is not a start), compared with the assumed ones; a difference replaces them
// and raises kStPrepRound
__global__ __launch_bounds__(64) void k_dict_sc(const Block* __restrict__ blocks, const uint64_t* __restrict__ bits,
                                                uint64_t wordsPerBlock, const uint32_t* __restrict__ mlen,
                                                Interval* __restrict__ ivAll, uint32_t* __restrict__ ivCount,
                                                int* __restrict__ status)
{
  __shared__ Interval ys[kMaxIv];
  const uint32_t b = blockIdx.x, lane = threadIdx.x;
  const Block B = blocks[b];
  const uint64_t n = B.end - B.start;
  const uint64_t* w = bits + (uint64_t)b * wordsPerBlock;
  const uint64_t words = (n + 63) / 64;
  uint32_t ny = 0;
  bool overflow = false;
  uint64_t from = 0;  // block-relative: the next position that may start an interval
  for (uint64_t w0 = 0; w0 < words; w0 += 64) {
    uint64_t mine = w0 + lane < words ? w[w0 + lane] : 0ull;
    while (true) {
      // clear the bits below `from`
      const uint64_t base = (w0 + lane) * 64;
      if (base + 64 <= from) mine = 0;
      else if (base < from) mine &= ~0ull << (from - base);
      const uint64_t any = __ballot(mine != 0);
      if (!any) break;
      const uint32_t l = (uint32_t)__builtin_ctzll(any);
      const uint64_t word = ((uint64_t)rdlane((uint32_t)(mine >> 32), l) << 32) | rdlane((uint32_t)mine, l);
      const uint64_t a = (w0 + l) * 64 + (uint64_t)__builtin_ctzll(word);
      const uint32_t La = mlen[B.start + a];
      if (ny < kMaxIv) {
        if (lane == 0) {
          Interval x;
          x.a = B.start + a;
          x.La = La;
          x.lo = x.a + 1;
          x.hi = x.lo + (La - kSameLetter);
          ys[ny] = x;
        }
        ny++;
      } else {
        overflow = true;
      }
      from = a + 1 + (La - kSameLetter);
    }
  }
  __syncthreads();
  if (overflow) {
    if (lane == 0) atomicOr(status, kStInvariant);
    return;
  }
  Interval* xs = ivAll + (uint64_t)b * kMaxIv;
  const uint32_t nx = ivCount[b];
  bool same = nx == ny;
  if (same) {
    bool diff = false;
    for (uint32_t k = lane; k < ny; k += 64)
      diff |= xs[k].lo != ys[k].lo || xs[k].hi != ys[k].hi || xs[k].La != ys[k].La;
    same = __ballot(diff) == 0;
  }
  if (same) return;
  for (uint32_t k = lane; k < ny; k += 64) xs[k] = ys[k];
  if (lane == 0) {
    ivCount[b] = ny;
    atomicOr(status, kStPrepRound);
  }
}

uint64_t dict_lz_mask_bytes_per_walk() { return kLzStride * 4; }

uint64_t dict_sort_keys_max() { return kBlockMaxLegacy + 64; }

uint64_t dict_sort_temp_bytes()
{
  size_t bytes = 0;
  if (rocprim::radix_sort_keys(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)dict_sort_keys_max(), 0,
                               kDictSortBits, (hipStream_t)0) != hipSuccess)
    return 0;
  return bytes;
}

int launch_dict_parallel(const DictArgs& A, hipStream_t s)
{
  const uint32_t nb = A.nb;
  if (!nb) return 0;
  const uint64_t runLo = A.hBlocks[0].start, runHi = A.hBlocks[nb - 1].end;
  const uint64_t runBase = runLo & ~63ull, runChunks = (runHi - runBase) / 64;
  DictPlan P{A.dBlocks, nb, A.cont, A.dictBack, A.low0, A.legacy ? 1u : 0u, A.iv, A.ivCount, A.runTab, runBase, runChunks};
  if (A.buildRuns && runChunks) {
    hipLaunchKernelGGL(k_dict_run_flags, dim3((uint32_t)((runChunks + 255) / 256)), dim3(256), 0, s, A.in, runBase, runChunks,
                       A.runFlag);
    hipLaunchKernelGGL(k_dict_runs, dim3((uint32_t)((runChunks + 63) / 64)), dim3(64), 0, s, A.in, runBase, runChunks, runLo,
                       runHi, A.runFlag, A.runTab, A.dBlocks, nb, A.legacy ? 1u : 0u, A.guess ? A.iv : nullptr, A.ivCount);
    if (A.guess) hipLaunchKernelGGL(k_dict_guess_sort, dim3((nb + 63) / 64), dim3(64), 0, s, nb, A.iv, A.ivCount);
  }
  if (!A.legacy)
    hipLaunchKernelGGL(k_dict_begin, dim3((1u << kHashBits) / 256), dim3(256), 0, s, A.last, A.prevH, A.prevX, A.cont,
                       A.shift);
  // previousHash: per block, a sort of its own insertions (earlier ones through the hash table)
  uint32_t maxOwn = 0, maxSize = 0;
  for (uint32_t b = 0; b < nb; b++) {
    const Block& B = A.hBlocks[b];
    const int64_t ownLo = P.own_lo_at(b, B.start);
    const int64_t ownHi = (int64_t)B.end - kTailNoMatch;
    maxSize = std::max<uint32_t>(maxSize, (uint32_t)(B.end - B.start));
    if (ownHi < ownLo) continue;
    const uint32_t n = (uint32_t)(ownHi - ownLo + 1);
    maxOwn = std::max<uint32_t>(maxOwn, n);
    if ((uint64_t)n > dict_sort_keys_max()) return -1;
    const uint32_t g = (n + 255) / 256;
    hipLaunchKernelGGL(k_dict_keys, dim3(g), dim3(256), 0, s, A.in, P, b, (uint64_t)ownLo, n, A.keysA);
    size_t tb = A.tempBytes;
    if (rocprim::radix_sort_keys(A.temp, tb, A.keysA, A.keysB, (size_t)n, 0, kDictSortBits, s)) return -1;
    hipLaunchKernelGGL(k_dict_ph, dim3(g), dim3(256), 0, s, A.keysB, n, (uint64_t)ownLo, A.last, A.ph,
                       A.legacy ? 1u : 0u);
    if (!A.legacy) hipLaunchKernelGGL(k_dict_last, dim3(g), dim3(256), 0, s, A.keysB, n, (uint64_t)ownLo, A.last);
  }
  if (maxOwn)
    hipLaunchKernelGGL(k_dict_pe, dim3((maxOwn + 255) / 256, nb), dim3(256), 0, s, A.in, P, A.ph, A.prevH, A.pe);
  hipLaunchKernelGGL(k_dict_search, dim3((maxSize + 4 * kDictSearchSpan - 1) / (4 * kDictSearchSpan), nb), dim3(256), 0, s, A.in, P, A.maxChain, A.pe, A.prevX,
                     A.mlen, A.mdist, A.sel, A.longFlag);
  if (A.maxChain <= (uint32_t)kLazyMax && A.nwalk) {
    hipLaunchKernelGGL(k_dict_lz_walk, dim3((A.nwalk + 3) / 4), dim3(256), 0, s, A.dBlocks, A.walkSegs, A.nwalk, A.mlen,
                       A.pe, A.lzMasks, A.lzState);
    hipLaunchKernelGGL(k_dict_lz_join, dim3((A.nwalk + 3) / 4), dim3(256), 0, s, A.dBlocks, A.walkSegs, A.nwalk, A.mlen,
                       A.pe, A.lzMasks, A.lzState);
    hipLaunchKernelGGL(k_dict_lz_fix, dim3(nb), dim3(64), 0, s, A.dBlocks, A.mlen, A.pe, A.lzMasks, A.lzState);
    hipLaunchKernelGGL(k_dict_lz_clear, dim3((A.nwalk + 3) / 4), dim3(256), 0, s, A.dBlocks, A.walkSegs, A.nwalk, A.mlen,
                       A.mdist, A.pe, A.lzMasks, A.longFlag);
  }
  if (!A.legacy) hipLaunchKernelGGL(k_dict_carry, dim3(65536 / 256), dim3(256), 0, s, P, A.ph, A.pe, A.prevH, A.prevX);
  // the intervals these results imply (the host runs the chunk again if they differ)
  const uint64_t wpb = (maxSize + 63) / 64;
  hipLaunchKernelGGL(k_dict_sc_bits, dim3((uint32_t)((wpb * 64 + 255) / 256), nb), dim3(256), 0, s, P, A.mlen, A.mdist,
                     A.scBits, wpb);
  hipLaunchKernelGGL(k_dict_sc, dim3(nb), dim3(64), 0, s, A.dBlocks, A.scBits, wpb, A.mlen, A.iv, A.ivCount, A.status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

uint64_t dict_sc_bits_bytes(uint32_t nb, uint64_t maxBlock) { return (uint64_t)nb * ((maxBlock + 63) / 64) * 8 + 64; }

uint64_t dict_run_table_bytes(uint64_t staged) { return (staged / 64 + 2) * (sizeof(uint2) + 4) + 64; }

}  // namespace sz4
