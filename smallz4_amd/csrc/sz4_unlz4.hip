// sz4_unlz4.hip -- gfx950 decoder for LZ4 frames with the semantics of the reference's decoder
// smallz4cat (unlz4_userPtr, smallz4cat.c:112-360) as the oracle restates it (oz_unlz4 in
// oracle/smallz4_oracle.c): modern and legacy frames, stored blocks, block and content checksums
// skipped, content-size and dictionary-ID fields skipped, an optional dictionary whose last 64 KiB
// precede the output (smallz4cat.c:168-187), legacy decoding ending after the first block shorter
// than 8 MiB (smallz4cat.c:325-327).
//
//   k_unlz4_ix_*    the block index (the chain of size words, smallz4cat.c:189-205): every frame offset
//                   classified as a possible size word, the candidates listed, linked and walked by one
//                   wavefront 64 at a time; k_unlz4_index (one lane walks the size words) is the in-launch
//                   fallback for what the candidates cannot settle
//   k_unlz4_sizes   one wavefront per block: token headers only -> decoded length, validation, and
//                   the block's sequence list (literal run, match length, offset, frame offset of
//                   the literals), recorded 64 at a time as coalesced 16-byte entries
//   (host)          output offset of every block, legacy truncation, capacity check
//   k_unlz4_blocks  one wavefront per block replays its sequence list, 64 sequences per step: their
//                   output offsets by one wavefront scan, their literal bytes prefetched into
//                   registers (a 512-byte frame window) and picked with ds_bpermute, then per
//                   sequence the literals and the match 64 bytes per step through the block's last
//                   64 KiB of output in an LDS ring (the reference's history[], smallz4cat.c:161-166).
//                   No header parsing and no global load on the sequence chain.  A match reaching
//                   below the block start waits for the blocks it reads: blocks are claimed in order
//                   through a ticket (placement independent), each publishes a done flag (agent
//                   release), a waiter polls relaxed, then acquires; every spin is bounded.
//
//   split mode (blocks of >= 256 KiB payload): k_unlz4_spec walks every 8 KiB sub-segment from its first
//                   byte, k_unlz4_join joins each to the true token chain from an assumed entry, k_unlz4_fix
//                   checks the assumptions per block (re-joining the wrong ones), k_unlz4_sub decodes every
//                   sub-segment into a value-or-reference image, k_unlz4_pack resolves the references
//
// Byte work only: decoding one block is a chain of sequences (each match may read the bytes the one
// before it wrote), so the parallelism is one wavefront per block (or per sub-segment in split mode) and
// 64 bytes per copy step.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "sz4_internal.h"

namespace sz4 {
#ifndef SZ4_DIAG
#define SZ4_DIAG 0
#endif
#if SZ4_DIAG == 8
// diagnostic build 8: k_unlz4_fix's serial re-joins (tools/diag_unlz4.py)
__device__ uint64_t sz4_udiag[16];
#define SZ4_D8(...) __VA_ARGS__
#else
#define SZ4_D8(...)
#endif

namespace {

__device__ __forceinline__ uint32_t un_rdlane(uint32_t v, uint32_t l)
{
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// 256 frame bytes [base, base + 256) held by the 64 lanes, 4 each; the cursor is wave-uniform
struct Window {
  const uint8_t* f;
  uint64_t n;  // frame length: bytes past it read as 0
  uint64_t base;
  uint32_t w;
  __device__ __forceinline__ void fill(uint64_t at, uint32_t lane)
  {
    base = at & ~3ull;
    const uint64_t o = base + 4ull * lane;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) v |= (o + k < n ? (uint32_t)f[o + k] : 0u) << (8 * k);
    w = v;
  }
  // byte at the uniform offset c; refills when c is not in the window's first 192 bytes
  __device__ __forceinline__ uint32_t byte(uint64_t c, uint32_t lane)
  {
    if (c < base || c >= base + 192) fill(c, lane);
    const uint32_t r = (uint32_t)(c - base);
    return (un_rdlane(w, r >> 2) >> (8 * (r & 3))) & 0xFFu;
  }
};

constexpr uint64_t kWaitLimit = 100000000ull * 60;  // 60 s of s_memrealtime (100 MHz)

// The LDS ring holds the last kRing output bytes (16 KiB: ten 64-lane workgroups per CU instead of two
// with the reference's full 64 KiB history).  Bytes further back are read from `out` itself: the wave
// drains its stores (s_waitcnt vmcnt(0) + workgroup acquire) whenever it has written kSync bytes since
// the last drain, so every byte below the ring's reach has been written and is visible to all lanes
// (kSync <= kRing - 64: a read below cur + 64 - kRing is then below the drained position).
constexpr uint32_t kRing = 16384;
constexpr uint32_t kSync = kRing / 2;

// v_writelane (the LLVM intrinsic by name): lane `l` of v becomes the uniform `x`
extern "C" __device__ int sz4_un_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t un_wrlane(uint32_t v, uint32_t x, uint32_t l)
{
  return (uint32_t)sz4_un_writelane((int)x, (int)l, (int)v);
}

// inclusive add-scan over the 64 lanes by DPP (row shifts 1, 2, 4, 8, then the row broadcasts): six
// dependent VALU steps instead of six ds_bpermute round trips
__device__ __forceinline__ uint32_t un_incl_scan_add(uint32_t v, uint32_t lane)
{
  (void)lane;
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return v;
}

// Sequence list of block bi: at most len/3 + 2 entries (a sequence with a match takes >= 3 frame
// bytes), at seqAll + src/3 + 2 * bi -- disjoint from every other block's, no host prefix needed.
__device__ __forceinline__ uint4* seq_base(uint4* seqAll, const UnBlock& B, uint32_t bi)
{
  return seqAll + B.src / 3 + 2ull * bi;
}
__device__ __forceinline__ uint32_t seq_cap(const UnBlock& B) { return B.len / 3 + 2; }

// Header walk of one block (smallz4cat.c:212-323) from block-relative frame offset r0: its decoded
// length, or kNone when it is malformed the way oz_unlz4 rejects it (a length byte, literal run or
// offset running past the block, offset 0).  Every sequence is recorded as (literals, match length,
// offset, frame offset of the literals from B.src): lane l holds entry (count & ~63) + l until 64 are
// complete, then one coalesced store.  The whole block: r0 = 0, stop = B.len.  A split block's
// sub-segment (below): the walk stops at its first token start >= stop (W.exit) and, with kMark, sets
// bit (token start - mb) of the LDS mask for every sequence it parsed; with kMerge, it stops before a
// token start whose bit is set in that LDS mask (W.merged: the speculative walk of the sub-segment
// parsed from there on already).  With kMark, cum (when given) receives each recorded sequence's output
// offset from r0 (the bytes the sequences before it decode), stored like seq.
struct WalkEnd {
  uint32_t exit;    // block-relative frame offset where the walk stopped
  uint32_t ns;      // sequences recorded
  uint32_t merged;  // 1: stopped at a merge bit (exit is that token start)
  uint32_t end;     // 1: reached the block end
};
template <bool kMark, bool kMerge>
__device__ uint64_t unlz4_walk(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, uint32_t lane, uint32_t r0,
                               uint32_t stop, uint4* __restrict__ seq, uint32_t cap, uint32_t* maskLds, uint32_t mb,
                               WalkEnd& W, uint32_t* __restrict__ cum = nullptr)
{
  W = WalkEnd{r0, 0u, 0u, 0u};
  if (B.stored) {  // uncompressed block (smallz4cat.c:329-343)
    W.exit = B.len;
    W.end = 1;
    return B.len;
  }
  const uint64_t end = B.src + B.len;
  uint64_t r = B.src + r0, w = 0;  // frame cursor; bytes decoded so far
  uint32_t ns = 0;
  uint4 buf = make_uint4(0u, 0u, 0u, 0u);
  uint32_t bufc = 0;
  // before: the bytes decoded from r0 up to this sequence
  auto push = [&](uint32_t tok, uint32_t lits, uint32_t ml, uint32_t off, uint32_t frel, uint32_t before) {
    const uint32_t l = ns & 63u;
    if constexpr (kMark) {
      if (lane == 0) atomicOr(&maskLds[(tok - mb) >> 5], 1u << ((tok - mb) & 31));
      bufc = un_wrlane(bufc, before, l);
    }
    buf.x = un_wrlane(buf.x, lits, l);
    buf.y = un_wrlane(buf.y, ml, l);
    buf.z = un_wrlane(buf.z, off, l);
    buf.w = un_wrlane(buf.w, frel, l);
    ns++;
    if ((ns & 63u) == 0u) {
      seq[ns - 64u + lane] = buf;
      if (kMark && cum) cum[ns - 64u + lane] = bufc;
    }
  };
  auto merge_at = [&](uint32_t tok) -> bool {
    if constexpr (kMerge) return (maskLds[(tok - mb) >> 5] >> ((tok - mb) & 31)) & 1u;
    return false;
  };
  Window win{f, n, 0, 0};
  // One sequence byte by byte through the window (smallz4cat.c:212-323): 0 next, 1 block done, 2 malformed.
  // Taken for what the pre-decoded headers below do not cover: extended literal runs, match lengths
  // with more than one extension byte, headers reaching past the register window.
  auto one_seq = [&]() -> int {
    const uint32_t tokAt = (uint32_t)(r - B.src);
    const uint32_t tok = win.byte(r++, lane);
    uint64_t lits = tok >> 4;
    if (lits == 15) {
      uint32_t x;
      do {
        if (r >= end) return 2;
        x = win.byte(r++, lane);
        lits += x;
      } while (x == 255);
    }
    if (r + lits > end) return 2;
    const uint32_t frel = (uint32_t)(r - B.src);
    w += lits;
    r += lits;
    if (r == end) {  // the last sequence has literals only
      push(tokAt, (uint32_t)lits, 0u, 0u, frel, (uint32_t)(w - lits));
      return 1;
    }
    if (r + 2 > end) return 2;
    const uint32_t off = win.byte(r, lane) | (win.byte(r + 1, lane) << 8);
    r += 2;
    if (off == 0) return 2;  // "invalid offset" (smallz4cat.c:265-267)
    uint64_t ml = kMinMatch + (tok & 15);
    if (ml == kMinMatch + 15) {
      uint32_t x;
      do {
        if (r >= end) return 2;
        x = win.byte(r++, lane);
        ml += x;
      } while (x == 255);
    }
    push(tokAt, (uint32_t)lits, (uint32_t)ml, off, frel, (uint32_t)(w - lits));
    w += ml;
    return 0;
  };
  // A sequence starting 20 or more bytes before the block end passes every bounds check of one_seq
  // (its header reads at most 18 bytes past the token, its literals end before the block does), so the
  // walk below checks nothing but a zero offset and runs on block-relative 32-bit cursors.
  const uint32_t fastEnd = min(B.len > 20u ? B.len - 20u : 0u, stop);
  while (r < end && (uint32_t)(r - B.src) < stop) {
    if (kMerge && merge_at((uint32_t)(r - B.src))) {
      W.merged = 1;
      break;
    }
    // Pre-decode a header at every window position q = 4 lane + k: token | offset << 8 | extension
    // byte << 24, or ~0 when the header needs the byte-wise path (literal run >= 15, a second match
    // extension byte, or bytes past the register window).  The walk costs one readlane per sequence.
    win.fill(r, lane);
    // kMerge: the mask words this window can reach, one per lane (a token start's merge bit by readlane, not
    // one dependent LDS read per sequence); the mask is read-only while a join walks
    uint32_t mw = 0, mw0 = 0;
    if constexpr (kMerge) {
      mw0 = (uint32_t)(r - B.src - mb) >> 5;
      const uint32_t wi = mw0 + lane;
      mw = lane < 8u && wi < kUnSub / 32u ? maskLds[wi] : 0u;
    }
    uint32_t cand[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t tok = (win.w >> (8 * k)) & 0xFFu;
      const uint32_t a = 4u * lane + (uint32_t)k + 1u + (tok >> 4);  // window index of the offset
      const uint32_t ia = (a >> 2) << 2;
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)ia, (int)win.w);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ia + 4u), (int)win.w);
      const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (a & 3u)));
      const bool ext = (tok & 15u) == 15u;
      const uint32_t last = a + 1u + (ext ? 1u : 0u);  // last window byte the header reads
      const bool ok = (tok >> 4) != 15u && last < 256u && !(ext && ((v >> 16) & 0xFFu) == 255u);
      cand[k] = ok ? (tok | (v << 8)) : 0xFFFFFFFFu;  // v's bytes 0-2: offset, extension byte
    }
    const uint32_t wb = (uint32_t)(win.base - B.src);  // window base, block-relative (r >= B.src >= base - 3)
    uint32_t rr = (uint32_t)(r - B.src);
    bool slow = false, stopped = false;
    while (rr < fastEnd) {
      if (kMerge && rr != (uint32_t)(r - B.src) &&
          ((un_rdlane(mw, ((rr - mb) >> 5) - mw0) >> ((rr - mb) & 31u)) & 1u)) {
        stopped = true;
        break;
      }
      const uint32_t q = rr - wb;
      if (q >= 192u) break;
      const uint32_t ql = q >> 2;
      const uint32_t c0 = un_rdlane(cand[0], ql), c1 = un_rdlane(cand[1], ql);
      const uint32_t c2 = un_rdlane(cand[2], ql), c3 = un_rdlane(cand[3], ql);
      const uint32_t pk = (q & 2u) ? ((q & 1u) ? c3 : c2) : ((q & 1u) ? c1 : c0);
      if (pk == 0xFFFFFFFFu) {
        slow = q < 64u;  // else refill at rr first: the header may fit the next window
        break;
      }
      const uint32_t off = (pk >> 8) & 0xFFFFu;
      if (off == 0) {  // "invalid offset" (smallz4cat.c:265-267)
        W.exit = rr;
        return kNone;
      }
      const uint32_t lits = (pk >> 4) & 15u, nib = pk & 15u;
      const uint32_t ml = kMinMatch + nib + (nib == 15u ? pk >> 24 : 0u);
      push(rr, lits, ml, off, rr + 1u, (uint32_t)w);
      w += lits + ml;
      rr += 3u + lits + (nib == 15u ? 1u : 0u);
    }
    r = B.src + rr;
    if (stopped) continue;  // the loop head sees the merge bit
    if (rr < fastEnd && !slow) continue;  // refill
    // byte-wise: a header the window could not pre-decode, or the block's last 20 bytes
    if (r >= end || rr >= stop) break;
    if (kMerge && merge_at(rr)) {
      W.merged = 1;
      break;
    }
    if (ns >= cap) {  // cannot happen in a well-formed block
      W.exit = rr;
      return kNone;
    }
    const int e = one_seq();
    if (e == 2) {
      W.exit = rr;
      return kNone;
    }
    if (e == 1) break;
  }
  if (ns & 63u) {
    const uint32_t b = ns & ~63u;
    if (lane < (ns & 63u)) {
      seq[b + lane] = buf;
      if (kMark && cum) cum[b + lane] = bufc;
    }
  }
  W.exit = (uint32_t)(r - B.src);
  W.ns = ns;
  W.end = r >= end ? 1u : 0u;
  return w;
}


// every lane receives the sum of its 16-lane row
__device__ __forceinline__ uint32_t un_row_sum(uint32_t v)
{
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  return v;
}

// unlz4_walk over a whole block (k_unlz4_sizes) with the token chain followed 64 window positions at a
// time on the vector unit: lane l takes the pre-decoded header at window position 64 s + l, steps to
// l + 3 + literals (+ 1 for a match-length byte) -- F1, 64 = out of the sub-window, or 64 where the
// header needs the byte-wise path --, F2 .. F32 by doubling (ds_bpermute), and every lane finds the last
// token start at or below itself by binary lifting from the entry.  The lanes that find themselves are
// the block's sequences in this sub-window: stored by mbcnt rank, their decoded bytes summed by a row
// reduction.  Whatever the pre-decoded headers do not cover goes through the same byte-wise sequence
// as unlz4_walk, so the two agree on every frame, malformed ones included.
__device__ uint64_t unlz4_walk_vec(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, uint32_t lane,
                                   uint4* __restrict__ seq, uint32_t cap, WalkEnd& W)
{
  W = WalkEnd{0u, 0u, 0u, 0u};
  if (B.stored) {
    W.exit = B.len;
    W.end = 1;
    return B.len;
  }
  const uint64_t end = B.src + B.len;
  uint64_t r = B.src, w = 0;
  uint32_t ns = 0;
  auto push = [&](uint32_t lits, uint32_t ml, uint32_t off, uint32_t frel) {
    if (lane == 0) seq[ns] = make_uint4(lits, ml, off, frel);
    ns++;
  };
  Window win{f, n, 0, 0};
  auto one_seq = [&]() -> int {
    const uint32_t tok = win.byte(r++, lane);
    uint64_t lits = tok >> 4;
    if (lits == 15) {
      uint32_t x;
      do {
        if (r >= end) return 2;
        x = win.byte(r++, lane);
        lits += x;
      } while (x == 255);
    }
    if (r + lits > end) return 2;
    const uint32_t frel = (uint32_t)(r - B.src);
    w += lits;
    r += lits;
    if (r == end) {  // the last sequence has literals only
      push((uint32_t)lits, 0u, 0u, frel);
      return 1;
    }
    if (r + 2 > end) return 2;
    const uint32_t off = win.byte(r, lane) | (win.byte(r + 1, lane) << 8);
    r += 2;
    if (off == 0) return 2;  // "invalid offset" (smallz4cat.c:265-267)
    uint64_t ml = kMinMatch + (tok & 15);
    if (ml == kMinMatch + 15) {
      uint32_t x;
      do {
        if (r >= end) return 2;
        x = win.byte(r++, lane);
        ml += x;
      } while (x == 255);
    }
    push((uint32_t)lits, (uint32_t)ml, off, frel);
    w += ml;
    return 0;
  };
  const uint32_t fastEnd = B.len > 20u ? B.len - 20u : 0u;
  while (r < end) {
    win.fill(r, lane);
    uint32_t cand[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t tok = (win.w >> (8 * k)) & 0xFFu;
      const uint32_t a = 4u * lane + (uint32_t)k + 1u + (tok >> 4);  // window index of the offset
      const uint32_t ia = (a >> 2) << 2;
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)ia, (int)win.w);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ia + 4u), (int)win.w);
      const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (a & 3u)));
      const bool ext = (tok & 15u) == 15u;
      const uint32_t last = a + 1u + (ext ? 1u : 0u);  // last window byte the header reads
      const bool ok = (tok >> 4) != 15u && last < 256u && !(ext && ((v >> 16) & 0xFFu) == 255u) && (v & 0xFFFFu) != 0u;
      cand[k] = ok ? (tok | (v << 8)) : 0xFFFFFFFFu;  // v's bytes 0-2: offset, extension byte
    }
    const uint32_t wb = (uint32_t)(win.base - B.src);  // window base, block-relative
    uint32_t rr = (uint32_t)(r - B.src);
    bool slow = false, bad = false;
    while (rr < fastEnd) {
      const uint32_t q0 = rr - wb;
      if (q0 >= 192u) break;  // refill
      const uint32_t sb = q0 & ~63u, e = q0 & 63u;
      const int src = (int)(((sb >> 2) + (lane >> 2)) << 2);
      const uint32_t g0 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cand[0]);
      const uint32_t g1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cand[1]);
      const uint32_t g2 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cand[2]);
      const uint32_t g3 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cand[3]);
      const uint32_t c = (lane & 2u) ? ((lane & 1u) ? g3 : g2) : ((lane & 1u) ? g1 : g0);
      const uint32_t pos = wb + sb + lane;  // block-relative frame offset of this lane's token
      const bool ok = c != 0xFFFFFFFFu && pos < fastEnd;
      const uint32_t lits = (c >> 4) & 15u, nib = c & 15u;
      const uint32_t step = 3u + lits + (nib == 15u ? 1u : 0u);
      uint32_t F[6];
      F[0] = ok && lane + step < 64u ? lane + step : 64u;
#pragma unroll
      for (int k = 1; k < 6; k++) {
        const uint32_t g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(F[k - 1] << 2), (int)F[k - 1]);
        F[k] = F[k - 1] >= 64u ? 64u : g;
      }
      uint32_t x = e;
      {
        const uint32_t y = un_rdlane(F[5], e);
        x = y <= lane ? y : x;
      }
#pragma unroll
      for (int k = 4; k >= 0; k--) {
        const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(x << 2), (int)F[k]);
        x = y <= lane ? y : x;
      }
      const bool tok = x == lane && ok;
      const uint64_t tb = __ballot(tok);
      const uint32_t cnt = (uint32_t)__builtin_popcountll(tb);
      if (ns + cnt > cap) {  // cannot happen in a well-formed block
        bad = true;
        break;
      }
      const uint32_t ml = kMinMatch + nib + (nib == 15u ? c >> 24 : 0u);
      if (tok) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(tb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tb, 0u));
        seq[ns + rank] = make_uint4(lits, ml, (c >> 8) & 0xFFFFu, pos + 1u);
      }
      ns += cnt;
      const uint32_t rs = un_row_sum(tok ? lits + ml : 0u);
      w += (uint64_t)(un_rdlane(rs, 0) + un_rdlane(rs, 16) + un_rdlane(rs, 32) + un_rdlane(rs, 48));
      const uint32_t p = un_rdlane(x, 63);  // the last token start of the path in this sub-window
      if (!((__ballot(ok) >> p) & 1ull)) {
        // a header the window did not pre-decode: from a refilled window, or byte-wise at the window start
        rr = wb + sb + p;
        slow = sb + p < 64u;
        break;
      }
      rr = wb + sb + p + un_rdlane(step, p);
    }
    if (bad) {
      W.exit = rr;
      return kNone;
    }
    r = B.src + rr;
    if (rr < fastEnd && !slow) continue;  // refill
    if (r >= end) break;
    if (ns >= cap) {
      W.exit = rr;
      return kNone;
    }
    const int e = one_seq();
    if (e == 2) {
      W.exit = (uint32_t)(r - B.src);
      return kNone;
    }
    if (e == 1) break;
  }
  W.exit = (uint32_t)(r - B.src);
  W.ns = ns;
  W.end = r >= end ? 1u : 0u;
  return w;
}

// unlz4_walk<kMark, kMerge> of a sub-segment on the vector unit, as unlz4_walk_vec: the path through 64
// window positions at a time by binary lifting.  kMerge (a join): its first token start at or past stop or
// with its bit set in the read-only LDS mask ends the walk there (W.merged).  kMark (the speculative walk):
// the path's token starts are OR-ed into the mask 64 window positions at a time (one ballot), and cum
// receives each sequence's output offset from r0.  Whatever the pre-decoded headers do not cover goes
// byte-wise, as in unlz4_walk, so the two agree on every frame.
template <bool kMark, bool kMerge>
__device__ uint64_t unlz4_walk_v(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, uint32_t lane,
                                 uint32_t r0, uint32_t stop, uint4* __restrict__ seq, uint32_t cap, uint32_t* maskLds,
                                 uint32_t mb, WalkEnd& W, uint32_t* __restrict__ cum = nullptr)
{
  W = WalkEnd{r0, 0u, 0u, 0u};
  if (B.stored) {
    W.exit = B.len;
    W.end = 1;
    return B.len;
  }
  const uint64_t end = B.src + B.len;
  uint64_t r = B.src + r0, w = 0;
  uint32_t ns = 0;
  auto push = [&](uint32_t tokAt, uint32_t lits, uint32_t ml, uint32_t off, uint32_t frel, uint32_t before) {
    if (lane == 0) {
      seq[ns] = make_uint4(lits, ml, off, frel);
      if constexpr (kMark) {
        atomicOr(&maskLds[(tokAt - mb) >> 5], 1u << ((tokAt - mb) & 31));
        if (cum) cum[ns] = before;
      }
    }
    ns++;
  };
  auto merge_at = [&](uint32_t tok) -> bool {
    if constexpr (kMerge) return (maskLds[(tok - mb) >> 5] >> ((tok - mb) & 31)) & 1u;
    return false;
  };
  Window win{f, n, 0, 0};
  auto one_seq = [&]() -> int {
    const uint32_t tokAt = (uint32_t)(r - B.src);
    const uint32_t tok = win.byte(r++, lane);
    uint64_t lits = tok >> 4;
    if (lits == 15) {
      uint32_t x;
      do {
        if (r >= end) return 2;
        x = win.byte(r++, lane);
        lits += x;
      } while (x == 255);
    }
    if (r + lits > end) return 2;
    const uint32_t frel = (uint32_t)(r - B.src);
    w += lits;
    r += lits;
    if (r == end) {  // the last sequence has literals only
      push(tokAt, (uint32_t)lits, 0u, 0u, frel, (uint32_t)(w - lits));
      return 1;
    }
    if (r + 2 > end) return 2;
    const uint32_t off = win.byte(r, lane) | (win.byte(r + 1, lane) << 8);
    r += 2;
    if (off == 0) return 2;  // "invalid offset" (smallz4cat.c:265-267)
    uint64_t ml = kMinMatch + (tok & 15);
    if (ml == kMinMatch + 15) {
      uint32_t x;
      do {
        if (r >= end) return 2;
        x = win.byte(r++, lane);
        ml += x;
      } while (x == 255);
    }
    push(tokAt, (uint32_t)lits, (uint32_t)ml, off, frel, (uint32_t)(w - lits));
    w += ml;
    return 0;
  };
  const uint32_t fastEnd = min(B.len > 20u ? B.len - 20u : 0u, stop);
  bool done = false;
  while (r < end && (uint32_t)(r - B.src) < stop) {
    if (kMerge && merge_at((uint32_t)(r - B.src))) {
      W.merged = 1;
      break;
    }
    win.fill(r, lane);
    uint32_t cand[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t tok = (win.w >> (8 * k)) & 0xFFu;
      const uint32_t a = 4u * lane + (uint32_t)k + 1u + (tok >> 4);  // window index of the offset
      const uint32_t ia = (a >> 2) << 2;
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)ia, (int)win.w);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ia + 4u), (int)win.w);
      const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (a & 3u)));
      const bool ext = (tok & 15u) == 15u;
      const uint32_t last = a + 1u + (ext ? 1u : 0u);  // last window byte the header reads
      const bool ok = (tok >> 4) != 15u && last < 256u && !(ext && ((v >> 16) & 0xFFu) == 255u) && (v & 0xFFFFu) != 0u;
      cand[k] = ok ? (tok | (v << 8)) : 0xFFFFFFFFu;  // v's bytes 0-2: offset, extension byte
    }
    const uint32_t wb = (uint32_t)(win.base - B.src);  // window base, block-relative
    uint32_t rr = (uint32_t)(r - B.src);
    bool slow = false, bad = false;
    while (rr < fastEnd) {
      const uint32_t q0 = rr - wb;
      if (q0 >= 192u) break;  // refill
      const uint32_t sb = q0 & ~63u, e = q0 & 63u;
      const int src = (int)(((sb >> 2) + (lane >> 2)) << 2);
      const uint32_t g0 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cand[0]);
      const uint32_t g1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cand[1]);
      const uint32_t g2 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cand[2]);
      const uint32_t g3 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cand[3]);
      const uint32_t c = (lane & 2u) ? ((lane & 1u) ? g3 : g2) : ((lane & 1u) ? g1 : g0);
      const uint32_t pos = wb + sb + lane;  // block-relative frame offset of this lane's token
      const bool ok = c != 0xFFFFFFFFu && pos < fastEnd;
      const uint32_t lits = (c >> 4) & 15u, nib = c & 15u;
      const uint32_t step = 3u + lits + (nib == 15u ? 1u : 0u);
      uint32_t F[6];
      F[0] = ok && lane + step < 64u ? lane + step : 64u;
#pragma unroll
      for (int k = 1; k < 6; k++) {
        const uint32_t g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(F[k - 1] << 2), (int)F[k - 1]);
        F[k] = F[k - 1] >= 64u ? 64u : g;
      }
      uint32_t x = e;
      {
        const uint32_t y = un_rdlane(F[5], e);
        x = y <= lane ? y : x;
      }
#pragma unroll
      for (int k = 4; k >= 0; k--) {
        const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(x << 2), (int)F[k]);
        x = y <= lane ? y : x;
      }
      // the path's token starts in this sub-window (its last one may need the byte-wise path); the first of
      // them at or past stop, or with its merge bit set, ends the walk (positions >= stop are not ok, so
      // such a token is the path's last)
      const bool onPath = x == lane && lane >= e;
      const uint32_t mrel = pos - mb;
      const bool mbit = kMerge && pos < stop && mrel < kUnSub && ((maskLds[mrel >> 5] >> (mrel & 31u)) & 1u);
      const uint64_t term = __ballot(onPath && (pos >= stop || mbit));
      const uint32_t T = term ? (uint32_t)__builtin_ctzll(term) : 64u;
      const bool tok = onPath && ok && lane < T;
      const uint64_t tb = __ballot(tok);
      const uint32_t cnt = (uint32_t)__builtin_popcountll(tb);
      if (ns + cnt > cap) {  // cannot happen in a well-formed block
        bad = true;
        break;
      }
      const uint32_t ml = kMinMatch + nib + (nib == 15u ? c >> 24 : 0u);
      const uint32_t dec = tok ? lits + ml : 0u;
      uint32_t incl = 0;
      if constexpr (kMark) incl = un_incl_scan_add(dec, lane);
      if (tok) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(tb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tb, 0u));
        seq[ns + rank] = make_uint4(lits, ml, (c >> 8) & 0xFFFFu, pos + 1u);
        if (kMark && cum) cum[ns + rank] = (uint32_t)w + incl - dec;
      }
      if constexpr (kMark) {
        // the recorded token starts' bits: 64 consecutive positions from wb + sb (those below mb are none)
        if (tb && lane == 0) {
          int32_t m0 = (int32_t)(wb + sb) - (int32_t)mb;
          uint64_t bits = tb;
          if (m0 < 0) {
            bits >>= (uint32_t)(-m0);
            m0 = 0;
          }
          const uint32_t j0 = (uint32_t)m0 >> 5, sh = (uint32_t)m0 & 31u;
          const uint32_t b0 = (uint32_t)(bits << sh), b1 = (uint32_t)(bits >> (32u - sh));
          const uint32_t b2 = sh ? (uint32_t)(bits >> (64u - sh)) : 0u;
          if (b0) atomicOr(&maskLds[j0], b0);
          if (b1) atomicOr(&maskLds[j0 + 1u], b1);
          if (b2) atomicOr(&maskLds[j0 + 2u], b2);
        }
      }
      ns += cnt;
      if constexpr (kMark) {
        w += un_rdlane(incl, 63);
      } else {
        const uint32_t rs = un_row_sum(dec);
        w += (uint64_t)(un_rdlane(rs, 0) + un_rdlane(rs, 16) + un_rdlane(rs, 32) + un_rdlane(rs, 48));
      }
      if (term) {
        rr = wb + sb + T;
        W.merged = rr < stop ? 1u : 0u;
        done = true;
        break;
      }
      const uint32_t p = un_rdlane(x, 63);  // the last token start of the path in this sub-window
      if (!((__ballot(ok) >> p) & 1ull)) {
        // a header the window did not pre-decode: from a refilled window, or byte-wise at the window start
        rr = wb + sb + p;
        slow = sb + p < 64u;
        break;
      }
      rr = wb + sb + p + un_rdlane(step, p);
    }
    if (bad) {
      W.exit = rr;
      return kNone;
    }
    r = B.src + rr;
    if (done) break;
    if (rr < fastEnd && !slow) continue;  // refill
    if (r >= end || rr >= stop) break;
    if (kMerge && merge_at(rr)) {
      W.merged = 1;
      break;
    }
    if (ns >= cap) {
      W.exit = rr;
      return kNone;
    }
    const int e = one_seq();
    if (e == 2) {
      W.exit = (uint32_t)(r - B.src);
      return kNone;
    }
    if (e == 1) break;
  }
  W.exit = (uint32_t)(r - B.src);
  W.ns = ns;
  W.end = r >= end ? 1u : 0u;
  return w;
}

// Replays block bi's sequence list into `out` (and the ring); returns the decoded length.
// From sequence b0Start on, with wStart bytes of the block already decoded (and drained): how the vector
// decoder below hands a block over when a match reads below the block start.
__device__ uint64_t unlz4_decode(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, uint32_t bi, uint32_t lane,
                                 const uint4* __restrict__ seq, uint8_t* __restrict__ out, uint8_t* __restrict__ ring,
                                 const uint8_t* __restrict__ dict, uint64_t dl, const UnBlock* __restrict__ blk,
                                 uint32_t* __restrict__ done, uint32_t* __restrict__ status, uint32_t b0Start = 0,
                                 uint64_t wStart = 0)
{
  if (B.stored) {
    // later blocks read it from `out`
    for (uint64_t k = lane; k < B.len; k += 64) out[B.dst + k] = f[B.src + k];
    return B.len;
  }
  uint64_t floorPos = B.dst;  // output below this is read only after its blocks are done
  uint32_t waitIdx = bi;
  uint64_t w = wStart;             // bytes decoded so far
  uint64_t synced = B.dst + wStart;  // this block's output below it is drained and readable from `out`
  for (uint32_t b0 = b0Start; b0 < B.nseq; b0 += 64) {
    const uint32_t cnt = B.nseq - b0 < 64u ? B.nseq - b0 : 64u;
    const uint4 q = lane < cnt ? seq[b0 + lane] : make_uint4(0u, 0u, 0u, 0u);
    // output offset of every sequence's literals (a wavefront scan of literals + match length)
    const uint32_t tot = q.x + q.y;
    const uint32_t incl = un_incl_scan_add(tot, lane);
    const uint64_t pos = w + (incl - tot);
    // the frame bytes of the 64 sequences' literals in registers when they span <= 512 bytes: lane l
    // holds [fb + 8l, fb + 8l + 8)
    const uint64_t fb = (B.src + un_rdlane(q.w, 0)) & ~7ull;
    const uint64_t fe = B.src + un_rdlane(q.w + q.x, cnt - 1u);
    const bool inWin = fe - fb <= 512u;
    uint32_t w0 = 0, w1 = 0;
    if (inWin) {
      const uint64_t o = fb + 8ull * lane;
      if (o + 8 <= n && (reinterpret_cast<uintptr_t>(f) & 7u) == 0u) {
        const uint2 v = *reinterpret_cast<const uint2*>(f + o);
        w0 = v.x;
        w1 = v.y;
      } else {
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const uint32_t b = o + k < n ? (uint32_t)f[o + k] : 0u;
          if (k < 4) w0 |= b << (8 * k);
          else w1 |= b << (8 * (k - 4));
        }
      }
    }
    for (uint32_t j = 0; j < cnt; j++) {
      const uint32_t L = un_rdlane(q.x, j), M = un_rdlane(q.y, j), off = un_rdlane(q.z, j), fr = un_rdlane(q.w, j);
      const uint64_t P = B.dst + (uint64_t)un_rdlane((uint32_t)pos, j);  // a block decodes to < 2^32 bytes
      if (L) {
        if (inWin && L <= 64u) {
          // lane k takes byte k out of the register window
          const uint32_t rel = (uint32_t)(B.src + fr - fb) + lane;
          const int addr = (int)((rel >> 3) << 2);
          const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)w0);
          const uint32_t c = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)w1);
          const uint8_t v = (uint8_t)(((rel & 4u) ? c : a) >> (8 * (rel & 3u)));
          if (lane < L) {
            out[P + lane] = v;
            ring[(P + lane) & (kRing - 1u)] = v;
          }
        } else {
          for (uint64_t k = lane; k < L; k += 64) {
            const uint8_t v = f[B.src + fr + k];
            out[P + k] = v;
            ring[(P + k) & (kRing - 1u)] = v;
          }
        }
      }
      if (M) {
        const uint64_t Q = P + L;                     // the match's first output byte
        const int64_t lo = (int64_t)Q - (int64_t)off;  // lowest byte it reads
        if (lo < (int64_t)floorPos && floorPos > 0 && waitIdx > 0) {
          // the blocks holding output in [max(lo, 0), floorPos) must be finished
          while (waitIdx > 0 && (int64_t)floorPos > lo && floorPos > 0) {
            waitIdx--;
            if (lane == 0) {
              const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
              while (__hip_atomic_load(&done[waitIdx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                __builtin_amdgcn_s_sleep(8);
                if (__builtin_amdgcn_s_memrealtime() - t0 > kWaitLimit) {
                  atomicOr(status, 2u);  // give up: the result is flagged, the grid still drains
                  break;
                }
              }
            }
            floorPos = blk[waitIdx].dst;
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // output Q + j = output Q + j - off.  First step: lane j reads Q - off + (j mod off), all
        // written before the match.  Later steps read Q + j - q with q the smallest multiple of off
        // that is >= 64: the previous step's bytes (period off), so the ring never needs more than
        // 64 KiB even for matches longer than that.
        const uint32_t qq = off >= 64u ? off : off * ((64u + off - 1u) / off);
        for (uint64_t k = 0; k < M; k += 64) {
          const uint64_t cur = Q + k;  // every output byte below it has been stored
          if (cur - synced >= kSync) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            synced = cur;
          }
          // ring slots of this step's reads are still intact above cur + 64 - kRing
          const int64_t ringLo = (int64_t)cur + 64 - (int64_t)kRing;
          const uint64_t jj = k + lane;
          const int64_t s = k == 0 ? lo + (int64_t)(off >= 64u ? lane : lane % off) : (int64_t)(Q + jj) - (int64_t)qq;
          uint8_t v = 0;
          if (jj < M) {
            if (s >= (int64_t)B.dst && s >= ringLo) v = ring[(uint64_t)s & (kRing - 1u)];
            else if (s >= 0) v = out[s];  // drained output of this block, or an earlier (finished) block
            else if ((uint64_t)(-s) <= dl) v = dict[dl - (uint64_t)(-s)];  // the dictionary's tail
            // else 0: before the history (oz_unlz4's zero-initialised history)
          }
          if (jj < M) {
            out[Q + jj] = v;
            ring[(Q + jj) & (kRing - 1u)] = v;
          }
        }
      }
    }
    w += un_rdlane(incl, cnt - 1u);
  }
  return w;
}


// inclusive max-scan over the 64 lanes (rows by DPP shifts, then the row broadcasts)
__device__ __forceinline__ uint32_t un_scan_max(uint32_t v)
{
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));  // row_shr:1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));  // row_shr:2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));  // row_shr:4
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));  // row_shr:8
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}

// Block bi's sequence list replayed 64 OUTPUT bytes per step instead of one sequence per step: for an
// output window [W, W + 64) the sequences starting in it mark their first byte (an LDS slot per byte),
// a max-scan gives every lane its sequence, four ds_bpermutes its fields; a literal byte comes from the
// frame, a match byte from `out` / the LDS ring when its source lies before the window, and from an
// earlier lane of the window otherwise (resolved by pointer jumping: src -> src - offset until a known
// byte, at most log2(64) rounds per distinct offset).  Blocks whose matches stay inside the block
// (independent blocks: every frame bench.py decodes); the first batch with a match reaching below the
// block start (linked blocks, a dictionary) or an empty sequence continues in unlz4_decode.
__device__ uint64_t unlz4_decode_vec(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, uint32_t bi,
                                     uint32_t lane, const uint4* __restrict__ seq, uint8_t* __restrict__ out,
                                     uint8_t* __restrict__ ring, uint32_t* __restrict__ slot,
                                     const uint8_t* __restrict__ dict, uint64_t dl, const UnBlock* __restrict__ blk,
                                     uint32_t* __restrict__ done, uint32_t* __restrict__ status)
{
  if (B.stored) {
    for (uint64_t k = lane; k < B.len; k += 64) out[B.dst + k] = f[B.src + k];
    return B.len;
  }
  uint64_t w = 0;            // block-relative output of the batches done
  uint64_t synced = 0;       // block-relative: output below it is drained and readable from `out`
  slot[lane] = 0;
  for (uint32_t b0 = 0; b0 < B.nseq; b0 += 64) {
    const uint32_t cnt = B.nseq - b0 < 64u ? B.nseq - b0 : 64u;
    const uint4 q = lane < cnt ? seq[b0 + lane] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t tot = q.x + q.y;
    const uint32_t incl = un_incl_scan_add(tot, lane);
    const uint32_t pj = incl - tot;  // batch-relative output offset of sequence `lane`
    const uint32_t blen = un_rdlane(incl, cnt - 1u);
    // a match reading below the block start, or a sequence of no bytes: the sequence-wise decoder
    const bool far = lane < cnt && q.y != 0u && w + pj + q.x < (uint64_t)q.z;
    if (__ballot(far || (lane < cnt && tot == 0u))) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      return unlz4_decode(f, n, B, bi, lane, seq, out, ring, dict, dl, blk, done, status, b0, w);
    }
    uint32_t jc = 0;  // 1 + the sequence covering the byte before the window
    for (uint32_t W = 0; W < blen; W += 64) {
      const uint64_t cur = w + W;  // block-relative first byte of the window
      if (cur - synced >= kSync) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        synced = cur;
      }
      if (lane < cnt && pj >= W && pj - W < 64u) slot[pj - W] = lane + 1u;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint32_t mark = slot[lane];
      slot[lane] = 0;
      const uint32_t sc = un_scan_max(mark);
      const uint32_t jj = (sc ? sc : jc) - 1u;  // this lane's sequence
      jc = un_rdlane(sc ? sc : jc, 63);
      const uint32_t o = W + lane;  // batch-relative output byte
      const bool valid = o < blen;
      const int addr = (int)(jj << 2);
      const uint32_t P = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)pj);
      const uint32_t L = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)q.x);
      const uint32_t off = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)q.z);
      const uint32_t fr = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)q.w);
      const uint32_t k = o - P;
      const bool lit = k < L;
      const uint64_t ob = w + o;    // block-relative
      const uint64_t src = ob - off;  // a match's source (>= 0: checked per batch)
      const bool inWin = valid && !lit && src >= cur;
      uint32_t val = 0;
      if (valid && lit) val = f[B.src + fr + k];
      // the ring holds [cur - kRing, cur) until this window's stores; further back is drained in `out`
      else if (valid && !inWin) val = src + kRing >= cur ? ring[(B.dst + src) & (kRing - 1u)] : out[B.dst + src];
      bool known = !inWin;
      uint32_t ref = inWin ? (uint32_t)(src - cur) : lane;
      while (__ballot(!known)) {
        const uint32_t kv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ref << 2), known ? 1 : 0);
        const uint32_t vv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ref << 2), (int)val);
        const uint32_t rv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ref << 2), (int)ref);
        if (!known) {
          if (kv) {
            val = vv;
            known = true;
          } else {
            ref = rv;
          }
        }
      }
      if (valid) {
        out[B.dst + ob] = (uint8_t)val;
        ring[(B.dst + ob) & (kRing - 1u)] = (uint8_t)val;
      }
    }
    w += blen;
  }
  return w;
}

}  // namespace

// ---- frame index: the chain of block size words (smallz4cat.c:114-159 header, 189-205 blocks) ------
// A 4-byte read at any frame offset: two aligned dwords when the frame is 4-byte aligned and they lie
// inside it, else byte by byte
__device__ __forceinline__ uint32_t un_rd32(const uint8_t* f, uint64_t n, uint64_t o)
{
  const uint64_t a = o & ~3ull;
  if ((reinterpret_cast<uintptr_t>(f) & 3u) == 0 && a + 8 <= n) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(f + a);
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(o & 3));
  }
  return (uint32_t)f[o] | ((uint32_t)f[o + 1] << 8) | ((uint32_t)f[o + 2] << 16) | ((uint32_t)f[o + 3] << 24);
}

// signature and frame descriptor: the offset of the first size word, or st = 1 (smallz4cat.c:114-159)
struct UnHeader {
  uint64_t r0;
  bool legacy, blockSum;
  uint32_t st;
};
__device__ __forceinline__ UnHeader un_header(const uint8_t* f, uint64_t n)
{
  UnHeader h{4, false, false, 0};
  if (n < 4) {
    h.st = 1;
    return h;
  }
  const uint32_t magic = un_rd32(f, n, 0);
  const bool modern = magic == 0x184D2204u;
  h.legacy = magic == 0x184C2102u;
  if (!modern && !h.legacy) {
    h.st = 1;
  } else if (modern) {
    if (h.r0 + 1 > n) {
      h.st = 1;
    } else {
      const uint32_t flg = f[h.r0];
      if ((flg >> 6) != 1u) h.st = 1;
      h.blockSum = (flg & 16u) != 0;
      const uint64_t skip = 1 + ((flg & 8u) ? 8 : 0) + ((flg & 1u) ? 4 : 0) + 1;
      if (h.r0 + 1 + skip > n) h.st = 1;
      else h.r0 += 1 + skip;
    }
  }
  return h;
}

// the walk in order, one lane: meta[0] = blocks found, meta[1] = 0 (frame end reached), 1 (malformed
// after meta[0] blocks) or 2 (more than maxBlocks), meta[2] = legacy frame, meta[3] = 1 when the parallel
// index decided (0: the serial walk), meta[4] = the longest payload (the host's split decision)
__device__ void unlz4_index_serial(const uint8_t* __restrict__ f, uint64_t n, UnBlock* __restrict__ blk, uint64_t maxBlocks,
                                   uint64_t* __restrict__ meta)
{
  const UnHeader h = un_header(f, n);
  uint64_t nb = 0, st = h.st, r = h.r0, maxLen = 0;
  // blocks until the end mark (smallz4cat.c:189-205, 345-349)
  while (st == 0) {
    if (r == n && h.legacy) break;
    if (r + 4 > n) { st = 1; break; }
    uint32_t word = un_rd32(f, n, r);
    r += 4;
    const bool packed = h.legacy || (word & 0x80000000u) == 0;
    if (!h.legacy) word &= 0x7FFFFFFFu;
    if (word == 0) break;
    if (r + word > n) { st = 1; break; }
    if (nb == maxBlocks) { st = 2; break; }
    UnBlock b;
    b.src = r;
    b.dst = 0;
    b.size = 0;
    b.len = word;
    b.stored = packed ? 0u : 1u;
    blk[nb++] = b;
    maxLen = word > maxLen ? word : maxLen;
    r += word;
    if (h.blockSum) {
      if (r + 4 > n) { st = 1; break; }
      r += 4;
    }
  }
  meta[0] = nb;
  meta[1] = st;
  meta[2] = h.legacy ? 1 : 0;
  meta[3] = 0;  // the serial walk decided
  meta[4] = maxLen;
}

__global__ __launch_bounds__(64) void k_unlz4_index(const uint8_t* __restrict__ f, uint64_t n, UnBlock* __restrict__ blk,
                                                    uint64_t maxBlocks, uint64_t* __restrict__ meta)
{
  if (threadIdx.x == 0) unlz4_index_serial(f, n, blk, maxBlocks, meta);
}

// The parallel index.  Every frame offset r >= r0 is classified as if a size word started there:
//   END    the chain stops cleanly (a zero word; a legacy frame's end, r == n)
//   BLOCK  a size word whose payload (and block checksum) fits: next(r) = r + 4 + len (+ 4)
//   BAD    anything else
// A *candidate* is an offset whose chain stays END/BLOCK for kIxHops hops.  Every size word of a frame
// the reference reads to its end mark is a candidate, and a random offset almost never is (its "word"
// must point exactly inside the frame, kIxHops times over), so the true chain is the walk from r0 over
// the candidates: k_unlz4_ix_cand (a bit per offset, a count per workgroup) -> k_unlz4_ix_scan (workgroup
// offsets) -> k_unlz4_ix_list (candidates in order, the rank of every bitmap word) -> k_unlz4_ix_link
// (each candidate's successor by rank) -> k_unlz4_ix_walk (one wavefront takes the successors 64 at a time,
// finds the path through them by binary lifting, and the workgroup writes the blocks).  Whatever the
// candidates cannot settle -- a bad header, r0 not a candidate, a successor that is not one (a frame
// that ends malformed), too many candidates -- falls back to the serial walk, so meta is exactly
// unlz4_index_serial's.
constexpr uint32_t kIxHops = 5;       // a false candidate needs five words in a row that point inside the frame
constexpr uint32_t kIxWgWords = 256;  // bitmap words (32 offsets each) per 1024-thread workgroup: 8 offsets a thread
constexpr uint32_t kIxEnd = 0xFFFFFFFFu, kIxBad = 0xFFFFFFFEu;
constexpr uint32_t kIxLds = 16384;  // successors k_unlz4_ix_walk stages in LDS (64 KiB)

__device__ __forceinline__ uint32_t ix_kind(const uint8_t* f, uint64_t n, const UnHeader& h, uint64_t r, uint32_t word,
                                            uint64_t& next)
{
  if (r == n && h.legacy) return kIxEnd;
  if (r + 4 > n) return kIxBad;
  if (!h.legacy) word &= 0x7FFFFFFFu;
  if (word == 0) return kIxEnd;
  next = r + 4 + word + (h.blockSum ? 4 : 0);
  return r + 4 + word <= n && next <= n ? 0u : kIxBad;
}

// offsets b0 + 32 w + j (j < 32, b0 = r0 rounded down to 4, offsets below r0 left out) of bitmap word w;
// the span ends at n inclusive (a legacy frame's end).  Four threads per word, 8 offsets each.  An END
// offset is a candidate at once; a BLOCK offset (its word points inside the frame: a few percent of the
// offsets of compressed data, almost none of text) follows its chain -- breadth-first over the thread's 8
// offsets, so each hop's loads go out together and a wavefront waits once per hop, not once per offset
__global__ __launch_bounds__(1024) void k_unlz4_ix_cand(const uint8_t* __restrict__ f, uint64_t n, uint64_t nWords,
                                                        uint32_t* __restrict__ bits, uint32_t* __restrict__ wgCount)
{
  __shared__ uint32_t s_sum[16];
  const UnHeader h = un_header(f, n);
  const uint32_t tid = threadIdx.x, q = tid & 3u;
  const uint64_t w = (uint64_t)blockIdx.x * kIxWgWords + (tid >> 2);
  uint32_t ok = 0, live = 0;  // offset j: a candidate / its chain still to follow
  uint64_t cur[8];
  if (w < nWords && h.st == 0) {
    const uint64_t p0 = (h.r0 & ~3ull) + 32 * w + 8 * q;
    if ((reinterpret_cast<uintptr_t>(f + p0) & 3u) == 0 && p0 + 16 <= n && p0 >= h.r0) {
      // 12 bytes as three aligned dwords, the 8 words by alignbyte, the first hop in 32-bit arithmetic
      const uint32_t* a = reinterpret_cast<const uint32_t*>(f + p0);
      const uint32_t d0 = a[0], d1 = a[1], d2 = a[2];
      const uint64_t rem64 = n - p0;
      const uint32_t rem = rem64 > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)rem64;
      const uint32_t bs = h.blockSum ? 4u : 0u;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint32_t lo = j < 4 ? d0 : d1, hi = j < 4 ? d1 : d2;
        const uint32_t word = (j & 3) ? __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(j & 3)) : lo;
        const uint32_t len = h.legacy ? word : word & 0x7FFFFFFFu;
        const uint32_t room = rem - (uint32_t)j - 4u;  // rem >= 16 > j + 4
        if (len == 0u) ok |= 1u << j;
        else if (len <= room && len + bs <= room) live |= 1u << j;
        cur[j] = p0 + (uint64_t)j + 4u + len + bs;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint64_t r = p0 + j;
        uint64_t next = 0;
        const uint32_t k = r >= h.r0 && r <= n ? ix_kind(f, n, h, r, r + 4 <= n ? un_rd32(f, n, r) : 0u, next) : kIxBad;
        cur[j] = next;
        if (k == kIxEnd) ok |= 1u << j;
        else if (k == 0u) live |= 1u << j;
      }
    }
  }
  for (uint32_t hop = 1; hop < kIxHops && __any(live != 0u); hop++) {
    uint32_t wd[8];
#pragma unroll
    for (int j = 0; j < 8; j++) wd[j] = ((live >> j) & 1u) && cur[j] + 4 <= n ? un_rd32(f, n, cur[j]) : 0u;
#pragma unroll
    for (int j = 0; j < 8; j++)
      if ((live >> j) & 1u) {
        uint64_t next = 0;
        const uint32_t k = ix_kind(f, n, h, cur[j], wd[j], next);
        cur[j] = next;
        if (k == kIxEnd) ok |= 1u << j;
        if (k != 0u) live &= ~(1u << j);
      }
  }
  uint32_t m = ok | live;  // chains still BLOCK after kIxHops hops
  // the word from its four threads (consecutive lanes)
  m <<= 8 * q;
  m |= (uint32_t)__shfl_xor((int)m, 1);
  m |= (uint32_t)__shfl_xor((int)m, 2);
  if (w < nWords && h.st == 0 && q == 0) bits[w] = m;
  // the workgroup's candidate count
  uint32_t c = q == 0 ? (uint32_t)__popc(m) : 0u;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
  if ((tid & 63) == 0) s_sum[tid >> 6] = c;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
    for (int k = 0; k < 16; k++) t += s_sum[k];
    wgCount[blockIdx.x] = t;
  }
}

// exclusive scan of the per-workgroup counts (one workgroup); wgOff[nWg] = the number of candidates
__global__ __launch_bounds__(1024) void k_unlz4_ix_scan(const uint32_t* __restrict__ wgCount, uint32_t nWg,
                                                        uint32_t* __restrict__ wgOff)
{
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t b = 0; b < nWg; b += 1024) {
    const uint32_t i = b + tid;
    const uint32_t v = i < nWg ? wgCount[i] : 0u;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint32_t before = s_carry;
    for (uint32_t k = 0; k < wv; k++) before += s_w[k];
    if (i < nWg) wgOff[i] = before + x - v;
    __syncthreads();
    if (tid == 1023) s_carry = before + x;
    __syncthreads();
  }
  if (tid == 0) wgOff[nWg] = s_carry;
}

// candidates in offset order (list[rank] = offset) and every bitmap word's first rank; nothing is listed
// beyond `cap` (the walk then falls back)
__global__ __launch_bounds__(256) void k_unlz4_ix_list(const uint8_t* __restrict__ f, uint64_t n, uint64_t nWords,
                                                       const uint32_t* __restrict__ bits, const uint32_t* __restrict__ wgOff,
                                                       uint32_t nWg, uint64_t cap, uint32_t* __restrict__ wordPre,
                                                       uint64_t* __restrict__ list)
{
  __shared__ uint32_t s_w[4];
  const UnHeader h = un_header(f, n);
  if (h.st != 0 || (uint64_t)wgOff[nWg] > cap) return;
  const uint64_t w = (uint64_t)blockIdx.x * kIxWgWords + threadIdx.x;
  const bool mine = threadIdx.x < kIxWgWords && w < nWords;
  const uint32_t m = mine ? bits[w] : 0u;
  const uint32_t v = (uint32_t)__popc(m), lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  uint32_t rank = wgOff[blockIdx.x] + x - v;
  for (uint32_t k = 0; k < wv; k++) rank += s_w[k];
  if (mine) wordPre[w] = rank;
  uint32_t mm = m;
  while (mm) {
    const uint32_t j = (uint32_t)__builtin_ctz(mm);
    mm &= mm - 1u;
    list[rank++] = (h.r0 & ~3ull) + 32 * w + j;
  }
}

// the rank of offset q among the candidates, or kIxBad when q is not one
__device__ __forceinline__ uint32_t ix_rank(const UnHeader& h, uint64_t nWords, const uint32_t* __restrict__ bits,
                                            const uint32_t* __restrict__ wordPre, uint64_t q)
{
  if (q < h.r0) return kIxBad;
  const uint64_t rel = q - (h.r0 & ~3ull), w = rel >> 5;
  if (w >= nWords) return kIxBad;
  const uint32_t m = bits[w], b = (uint32_t)(rel & 31);
  if (!((m >> b) & 1u)) return kIxBad;
  return wordPre[w] + (uint32_t)__popc(m & ((1u << b) - 1u));
}

// every candidate's successor (kIxEnd: the chain ends there, kIxBad: the next offset is no candidate),
// workgroup b taking the candidates k_unlz4_ix_list listed for its offsets
__global__ __launch_bounds__(64) void k_unlz4_ix_link(const uint8_t* __restrict__ f, uint64_t n, uint64_t nWords,
                                                      const uint32_t* __restrict__ bits, const uint32_t* __restrict__ wgOff,
                                                      uint32_t nWg, uint64_t cap, const uint32_t* __restrict__ wordPre,
                                                      const uint64_t* __restrict__ list, uint32_t* __restrict__ link)
{
  const UnHeader h = un_header(f, n);
  if (h.st != 0 || (uint64_t)wgOff[nWg] > cap) return;
  const uint32_t a = wgOff[blockIdx.x], b = wgOff[blockIdx.x + 1];
  for (uint32_t i = a + threadIdx.x; i < b; i += 64) {
    const uint64_t r = list[i];
    uint64_t next = 0;
    const uint32_t k = ix_kind(f, n, h, r, r + 4 <= n ? un_rd32(f, n, r) : 0u, next);
    link[i] = k ? k : ix_rank(h, nWords, bits, wordPre, next);
  }
}

__global__ __launch_bounds__(1024) void k_unlz4_ix_walk(const uint8_t* __restrict__ f, uint64_t n, uint64_t nWords,
                                                        const uint32_t* __restrict__ bits, const uint32_t* __restrict__ wgOff,
                                                        uint32_t nWg, uint64_t cap, const uint32_t* __restrict__ wordPre,
                                                        const uint64_t* __restrict__ list, uint32_t* __restrict__ link,
                                                        uint32_t* __restrict__ chain, UnBlock* __restrict__ blk,
                                                        uint64_t maxBlocks, uint64_t* __restrict__ meta)
{
  __shared__ uint32_t s_nb, s_st, s_max;
  __shared__ uint32_t s_link[kIxLds];  // the successors, when they fit: the walk then reads no HBM
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const UnHeader h = un_header(f, n);
  const uint64_t M = wgOff[nWg];
  const bool usable = h.st == 0 && M <= cap && M < (uint64_t)kIxBad;
  const bool inLds = usable && M <= kIxLds;
  if (inLds)
    for (uint32_t i = tid; i < (uint32_t)M; i += 1024) s_link[i] = link[i];
  if (tid == 0) s_max = 0;
  __syncthreads();
  if (tid < 64) {
    // one wavefront follows the successors from r0, 64 candidates per step: lane l holds candidate e + l
    // (e: the entry), its local successor in the window (64: it leaves the window, ends or is BAD), the
    // doubling tables J1..J32 by ds_bpermute, and every lane finds the last path node at or below itself by
    // binary lifting from lane 0 -- the lanes that find themselves are the path (as k_walk does for the
    // parse).  The path's last node leads to the next window's entry.
    uint32_t st = 1, nb = 0;
    uint32_t e = usable ? ix_rank(h, nWords, bits, wordPre, h.r0) : kIxBad;
    e = (uint32_t)__builtin_amdgcn_readfirstlane((int)e);
    // table T at per-lane index x (x = 64: "outside", stays 64)
    auto at = [&](uint32_t T, uint32_t x) -> uint32_t {
      const uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((x < 64u ? x : 63u) << 2), (int)T);
      return x < 64u ? r : 64u;
    };
    while (e != kIxBad) {
      const uint64_t ci = (uint64_t)e + lane;
      const uint32_t val = ci < M ? (inLds ? s_link[ci] : link[ci]) : kIxBad;
      const uint32_t nl = val < (uint32_t)M && (uint64_t)val < (uint64_t)e + 64 ? val - e : 64u;
      uint32_t J[6];
      J[0] = nl;
#pragma unroll
      for (int k = 1; k < 6; k++) J[k] = at(J[k - 1], J[k - 1]);
      uint32_t pos = 0;
#pragma unroll
      for (int k = 5; k >= 0; k--) {
        const uint32_t c = at(J[k], pos);
        if (c <= lane) pos = c;
      }
      const uint64_t path = __ballot(pos == lane);  // lane 0 is on it
      const uint32_t last = 63u - (uint32_t)__builtin_clzll(path);
      const uint32_t exitv = un_rdlane(val, last);
      // the path's nodes are blocks, except a last node that ends the chain (END) or cannot be followed (BAD)
      const uint64_t blocks = exitv == kIxEnd || exitv == kIxBad ? path & ~(1ull << last) : path;
      const uint32_t cnt = (uint32_t)__builtin_popcountll(blocks);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(blocks >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)blocks, 0u));
      const bool take = ((blocks >> lane) & 1ull) && (uint64_t)nb + below < maxBlocks;
      if (take) chain[nb + below] = e + lane;
      if ((uint64_t)nb + cnt > maxBlocks) {
        nb = (uint32_t)maxBlocks;
        st = 2;
        break;
      }
      nb += cnt;
      if (exitv == kIxEnd) {
        st = 0;
        break;
      }
      if (exitv == kIxBad) break;  // the serial walk decides
      e = exitv;  // >= e + 64: the next window
    }
    if (lane == 0) {
      s_nb = nb;
      s_st = st;
    }
  }
  __syncthreads();
  const uint32_t nb = s_nb, st = s_st;
  if (st == 1) {
    if (tid == 0) unlz4_index_serial(f, n, blk, maxBlocks, meta);
    return;
  }
  uint32_t myMax = 0;
  for (uint32_t k = tid; k < nb; k += 1024) {
    const uint64_t r = list[chain[k]];
    uint32_t word = un_rd32(f, n, r);
    const bool packed = h.legacy || (word & 0x80000000u) == 0;
    if (!h.legacy) word &= 0x7FFFFFFFu;
    UnBlock b;
    b.src = r + 4;
    b.dst = 0;
    b.size = 0;
    b.len = word;
    b.stored = packed ? 0u : 1u;
    blk[k] = b;
    myMax = word > myMax ? word : myMax;
  }
  if (myMax) atomicMax(&s_max, myMax);
  __syncthreads();
  if (tid == 0) {
    meta[0] = nb;
    meta[1] = st;
    meta[2] = h.legacy ? 1 : 0;
    meta[3] = 1;  // the parallel index decided
    meta[4] = s_max;
  }
}

__global__ __launch_bounds__(64) void k_unlz4_sizes(const uint8_t* __restrict__ f, uint64_t n, UnBlock* __restrict__ blk,
                                                    uint32_t nb, uint4* __restrict__ seqAll)
{
  const uint32_t bi = blockIdx.x, lane = threadIdx.x;
  if (bi >= nb) return;
  const UnBlock B = blk[bi];
  WalkEnd W;
  const uint64_t size = unlz4_walk_vec(f, n, B, lane, seq_base(seqAll, B, bi), seq_cap(B), W);
  if (lane == 0) {
    blk[bi].size = size;
    blk[bi].nseq = W.ns;
  }
}

// flags[0..nb) done flags, flags[nb] status bits, flags[nb + 1] ticket (all zeroed before the launch)
__global__ __launch_bounds__(64) void k_unlz4_blocks(const uint8_t* __restrict__ f, uint64_t n, const UnBlock* __restrict__ blk,
                                                     uint32_t nb, const uint4* __restrict__ seqAll, uint8_t* __restrict__ out,
                                                     const uint8_t* __restrict__ dict, uint64_t dl, uint32_t* __restrict__ flags)
{
  __shared__ uint8_t ring[kRing];
  const uint32_t lane = threadIdx.x;
  uint32_t* done = flags;
  uint32_t* status = flags + nb;
  // blocks are claimed in order by running workgroups: every block a claim can wait for has been
  // claimed by a workgroup that is already running (no dispatch-order assumption)
  uint32_t t = 0;
  if (lane == 0) t = atomicAdd(&flags[nb + 1], 1u);
  const uint32_t bi = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
  if (bi >= nb) return;
  const UnBlock B = blk[bi];
  __shared__ uint32_t slot[64];
  const uint64_t got = unlz4_decode_vec(f, n, B, bi, lane, seq_base(const_cast<uint4*>(seqAll), B, bi), out, ring, slot,
                                        dict, dl, blk, done, status);
  if (lane == 0 && got != B.size) atomicOr(status, 1u);
  // publish: this wave's stores drained, written back (agent release), then the flag
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(&done[bi], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ================================================================================================
// Split mode: blocks decoded by many wavefronts at once (frames of large blocks, e.g. the 4 MiB
// dependent blocks smallz4::lz4 writes).
// ================================================================================================
constexpr uint32_t kSubWords = kUnSub / 32;

__device__ __forceinline__ uint4* sub_pre(uint4* seq, uint32_t g) { return seq + (uint64_t)g * 2 * kUnSubCap; }
__device__ __forceinline__ uint4* sub_spec(uint4* seq, uint32_t g) { return seq + (uint64_t)g * 2 * kUnSubCap + kUnSubCap; }

// one wavefront per sub-segment: the token chain as if a token started at its first byte, every token
// start it parsed as a bit.  Wherever the true chain meets one of those starts, the two are the same
// chain from there on (k_unlz4_fix).  Side tables for k_unlz4_fix (kUnAuxWords per sub-segment): the
// mask, its prefix bit counts per word, and every speculative sequence's output offset, so that the
// rank of a token start and the bytes from it to the sub-segment's end are two loads.
__device__ __forceinline__ uint32_t* sub_mask(uint32_t* aux, uint32_t g) { return aux + (uint64_t)g * kUnAuxWords; }
__device__ __forceinline__ uint16_t* sub_mpre(uint32_t* aux, uint32_t g)
{
  return reinterpret_cast<uint16_t*>(aux + (uint64_t)g * kUnAuxWords + kSubWords);
}
__device__ __forceinline__ uint32_t* sub_cum(uint32_t* aux, uint32_t g)
{
  return aux + (uint64_t)g * kUnAuxWords + kSubWords + kSubWords / 2;
}

__global__ __launch_bounds__(64) void k_unlz4_spec(const uint8_t* __restrict__ f, uint64_t n, const UnBlock* __restrict__ blk,
                                                   UnSub* __restrict__ subs, uint32_t nsub, uint4* __restrict__ seq,
                                                   uint32_t* __restrict__ aux)
{
  __shared__ uint32_t mask[kSubWords];
  const uint32_t g = blockIdx.x, lane = threadIdx.x;
  if (g >= nsub) return;
  for (uint32_t w = lane; w < kSubWords; w += 64) mask[w] = 0;
  __syncthreads();
  const UnSub U = subs[g];
  const UnBlock B = blk[U.block];
  const uint32_t s0 = U.k * kUnSub, s1 = min(s0 + kUnSub, B.len);
  WalkEnd W{s0, 0u, 0u, 0u};
  const uint64_t sz = B.stored ? 0ull
                               : unlz4_walk_v<true, false>(f, n, B, lane, s0, s1, sub_spec(seq, g), kUnSubCap, mask, s0,
                                                           W, sub_cum(aux, g));
  __syncthreads();
  // the mask (4 words per lane) and its exclusive prefix bit counts per word
  static_assert(kSubWords == 256, "four mask words per lane");
  uint32_t m[4], c = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    m[k] = mask[4 * lane + k];
    c += __popc(m[k]);
  }
  uint32_t pre = un_incl_scan_add(c, lane) - c;
  uint32_t* gm = sub_mask(aux, g);
  uint16_t* gp = sub_mpre(aux, g);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    gm[4 * lane + k] = m[k];
    gp[4 * lane + k] = (uint16_t)pre;
    pre += __popc(m[k]);
  }
  if (lane == 0) {
    subs[g].specN = B.stored ? 0u : W.ns;
    subs[g].specExit = B.stored ? s1 : W.exit;
    subs[g].specFlags = B.stored ? 0u : ((sz == kNone ? 1u : 0u) | (W.end ? 2u : 0u));
    subs[g].specBytes = sz == kNone ? 0u : (uint32_t)sz;
  }
}

// The join of sub-segment g (block-relative payload [a0, a1)) from an entry t of the true token chain:
// where the speculative walk of g parsed that token start, its list is the true one from there; else the
// chain is re-parsed from t until it meets a speculative start (a wrong start falls into the true chain
// within a few tokens) or leaves the sub-segment.  Output: the re-parsed prefix (preN, in sub_pre), the
// first speculative sequence kept, the bytes decoded, the exit and whether the block ended.
struct Join {
  uint32_t preN, specFrom, outLen, exit;
  bool ended, ok;
};
__device__ Join un_join(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, const UnSub& U, uint32_t g,
                        uint32_t lane, uint32_t t, bool ended, uint4* __restrict__ seq, uint32_t* __restrict__ aux,
                        uint32_t* mask)
{
  const uint32_t a0 = U.k * kUnSub, a1 = min(a0 + kUnSub, B.len);
  Join J{0u, U.specN, 0u, t, ended, true};
  if (B.stored) {  // an uncompressed block: its bytes as they are
    J.specFrom = 0;
    J.outLen = a1 - a0;
    J.exit = a1;
    J.ended = a1 == B.len;
    return J;
  }
  if (ended || t >= a1) return J;  // nothing of the chain starts here
  for (uint32_t w = lane; w < kSubWords; w += 64) mask[w] = sub_mask(aux, g)[w];
  __syncthreads();
  bool merged = (mask[(t - a0) >> 5] >> ((t - a0) & 31)) & 1u;
  if (!merged) {
    WalkEnd W;
    const uint64_t sz = unlz4_walk_v<false, true>(f, n, B, lane, t, a1, sub_pre(seq, g), kUnSubCap, mask, a0, W);
    if (sz == kNone) {
      J.ok = false;
    } else {
      J.preN = W.ns;
      J.outLen = (uint32_t)sz;
      merged = W.merged != 0;
      J.exit = W.exit;
      J.ended = W.end != 0;
    }
  }
  if (J.ok && merged) {
    if (U.specFlags & 1u) {  // the true chain runs into the malformed sequence the walk met
      J.ok = false;
    } else {
      const uint32_t x = J.exit - a0;
      J.specFrom = (uint32_t)sub_mpre(aux, g)[x >> 5] + (uint32_t)__popc(mask[x >> 5] & ((1u << (x & 31)) - 1u));
      J.outLen += U.specBytes - (J.specFrom < U.specN ? sub_cum(aux, g)[J.specFrom] : U.specBytes);
      J.exit = U.specExit;
      J.ended = (U.specFlags & 2u) != 0;
    }
  }
  __syncthreads();
  return J;
}

constexpr uint32_t kJoinRounds = 1;

__device__ __forceinline__ void un_store_join(UnSub* __restrict__ subs, uint32_t g, const Join& J, uint32_t entry,
                                              bool assumedEnded)
{
  subs[g].preN = J.preN;
  subs[g].specFrom = J.specFrom;
  subs[g].outLen = J.outLen;
  subs[g].joinEntry = entry;
  // (read by the next sub-segment's wavefront while a join round runs)
  __hip_atomic_store(&subs[g].joinExit, J.exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&subs[g].joinFlags, (assumedEnded ? 1u : 0u) | (J.ok ? 0u : 2u) | (J.ended ? 4u : 0u),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one wavefront per sub-segment: its join from an ASSUMED entry.  Round 0 assumes the true chain enters
// where the previous sub-segment's speculative walk left (it does whenever the chain met that walk within
// the previous sub-segment: then it leaves where the walk left -- about 85 % of Silesia's 8 KiB pieces);
// a later round assumes the exit of the previous sub-segment's latest join, and joins again only where
// that changed the assumption: after r rounds every sub-segment is right whose chain of wrong guesses is
// shorter than r.  A round may read the previous sub-segment's record while its own wavefront rewrites it;
// whatever it reads is only an assumption, which k_unlz4_fix checks against the true chain.
__global__ __launch_bounds__(64) void k_unlz4_join(const uint8_t* __restrict__ f, uint64_t n, const UnBlock* __restrict__ blk,
                                                   UnSub* __restrict__ subs, uint32_t nsub, uint4* __restrict__ seq,
                                                   uint32_t* __restrict__ aux, uint32_t round)
{
  __shared__ uint32_t mask[kSubWords];
  const uint32_t g = blockIdx.x, lane = threadIdx.x;
  if (g >= nsub) return;
  const UnSub U = subs[g];
  uint32_t t = 0;
  bool ended = false;
  if (U.k != 0) {
    if (round == 0) {
      t = subs[g - 1].specExit;
      ended = (subs[g - 1].specFlags & 2u) != 0;
    } else {
      t = __hip_atomic_load(&subs[g - 1].joinExit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ended = (__hip_atomic_load(&subs[g - 1].joinFlags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 4u) != 0;
      if (t == U.joinEntry && ended == ((U.joinFlags & 1u) != 0)) return;  // the same assumption as before
    }
  } else if (round != 0) {
    return;  // the first sub-segment's entry is known
  }
  const UnBlock B = blk[U.block];
  const Join J = un_join(f, n, B, U, g, lane, t, ended, seq, aux, mask);
  if (lane == 0) un_store_join(subs, g, J, t, ended);
}

// one wavefront per block: the true chain enters sub-segment k where k - 1's join left.  Sub-segments are
// taken 64 at a time: lane j's join (k_unlz4_join) holds if its assumed entry is the true one, which by
// induction is the recorded exit of lane j - 1; up to the first that does not hold, every output offset is
// one prefix sum; that one is joined again from its true entry, and the next batch starts after it.
// Per block: the decoded length, or kNone when the block is malformed (as the whole-block walk finds).
__global__ __launch_bounds__(64) void k_unlz4_fix(const uint8_t* __restrict__ f, uint64_t n, UnBlock* __restrict__ blk,
                                                  uint32_t nb, UnSub* __restrict__ subs, uint4* __restrict__ seq,
                                                  uint32_t* __restrict__ aux)
{
  __shared__ uint32_t mask[kSubWords];
  const uint32_t bi = blockIdx.x, lane = threadIdx.x;
  if (bi >= nb) return;
  const UnBlock B = blk[bi];
  if (B.subCount == 0) return;  // an empty block (not split)
  uint32_t t = 0, outRel = 0;
  bool ok = true, ended = false;
  uint32_t k = 0;
  SZ4_D8(const uint64_t d8t0 = __builtin_readcyclecounter(); uint64_t d8Re = 0, d8Quick = 0, d8Tok = 0, d8Tk = 0, d8Merged = 0, d8Batch = 0;)
  while (k < B.subCount && ok) {
    SZ4_D8(d8Batch++;)
    const uint32_t kj = k + lane;
    const bool in = kj < B.subCount;
    const uint32_t g = B.subFirst + (in ? kj : k);
    const uint32_t entry = in ? subs[g].joinEntry : 0u, exit = in ? subs[g].joinExit : 0u;
    const uint32_t flags = in ? subs[g].joinFlags : 2u, outLen = in ? subs[g].outLen : 0u;
    // the true entry and end state of lane j: lane j - 1's join (lane 0: the batch's)
    uint32_t tEntry = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - 1u) & 63u) << 2), (int)exit);
    uint32_t pFlags = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - 1u) & 63u) << 2), (int)flags);
    bool tEnded = (pFlags & 4u) != 0;
    if (lane == 0) {
      tEntry = t;
      tEnded = ended;
    }
    const bool holds = in && entry == tEntry && ((flags & 1u) != 0) == tEnded;
    const uint64_t notHeld = ~__ballot(holds);
    const uint32_t nOk = notHeld ? (uint32_t)__builtin_ctzll(notHeld) : 64u;
    const uint64_t bad = __ballot(lane < nOk && (flags & 2u));
    if (bad) {  // a held join met a malformed sequence: the block is malformed
      ok = false;
      break;
    }
    if (nOk) {
      const bool mine = lane < nOk;
      const uint32_t incl = un_incl_scan_add(mine ? outLen : 0u, lane);
      if (mine) subs[g].outRel = outRel + incl - outLen;
      outRel += un_rdlane(incl, nOk - 1u);
      t = un_rdlane(exit, nOk - 1u);
      ended = (un_rdlane(flags, nOk - 1u) & 4u) != 0;
      k += nOk;
      if (nOk == 64u) continue;
    }
    if (k >= B.subCount) break;
    // sub-segment k again, from its true entry
    const uint32_t gk = B.subFirst + k;
    const UnSub U = subs[gk];
    SZ4_D8(const uint64_t d8c0 = __builtin_readcyclecounter(); d8Re++;
           if (ended || t >= min(U.k * kUnSub + kUnSub, B.len)) d8Quick++;)
    const Join J = un_join(f, n, B, U, gk, lane, t, ended, seq, aux, mask);
    SZ4_D8(d8Tk += __builtin_readcyclecounter() - d8c0; d8Tok += J.preN; if (J.exit == U.specExit) d8Merged++;)
    if (!J.ok) {
      ok = false;
      break;
    }
    if (lane == 0) {
      un_store_join(subs, gk, J, t, ended);
      subs[gk].outRel = outRel;
    }
    outRel += J.outLen;
    t = J.exit;
    ended = J.ended;
    k++;
  }
  if (lane == 0) blk[bi].size = ok && ended && t == B.len ? (uint64_t)outRel : kNone;
  SZ4_D8(if (lane == 0) {
    const uint64_t dt = __builtin_readcyclecounter() - d8t0;
    atomicAdd((unsigned long long*)&sz4_udiag[0], 1ull);
    atomicAdd((unsigned long long*)&sz4_udiag[1], (unsigned long long)B.subCount);
    atomicAdd((unsigned long long*)&sz4_udiag[2], (unsigned long long)d8Batch);
    atomicAdd((unsigned long long*)&sz4_udiag[3], (unsigned long long)d8Re);
    atomicAdd((unsigned long long*)&sz4_udiag[4], (unsigned long long)d8Quick);
    atomicAdd((unsigned long long*)&sz4_udiag[5], (unsigned long long)d8Tok);
    atomicAdd((unsigned long long*)&sz4_udiag[6], (unsigned long long)d8Merged);
    atomicAdd((unsigned long long*)&sz4_udiag[7], (unsigned long long)d8Tk);
    atomicAdd((unsigned long long*)&sz4_udiag[8], (unsigned long long)dt);
    atomicMax((unsigned long long*)&sz4_udiag[9], (unsigned long long)dt);
    atomicMax((unsigned long long*)&sz4_udiag[10], (unsigned long long)d8Re);
  })
}

// The decode image: one u32 per output byte, the byte's value (< 256) or kUnRef | p: "the same byte as
// output position p", for a match byte whose source lies before the sub-segment's own output (another
// wavefront writes it).  A sub-segment's own earlier bytes are copied as they are (values or
// references): recent ones through an LDS ring of the last kRingU words, older ones from the image after
// the wave drained its stores, as in unlz4_decode.
// 8 KiB of LDS per one-wave workgroup: 20 per CU (5 waves per SIMD; 4096 words held it to 2.5, and the
// latency-bound copy loop needs the waves: Silesia at 4 MiB blocks 16.4 -> 14.9 ms, profiles/r06/r06aa)
constexpr uint32_t kRingU = 2048;
constexpr uint32_t kSyncU = kRingU / 2;

__global__ __launch_bounds__(64) void k_unlz4_sub(const uint8_t* __restrict__ f, uint64_t n, const UnBlock* __restrict__ blk,
                                                  const UnSub* __restrict__ subs, uint32_t nsub, const uint4* __restrict__ seqAll,
                                                  uint32_t* __restrict__ img, const uint8_t* __restrict__ dict, uint64_t dl)
{
  __shared__ uint32_t ring[kRingU];
  const uint32_t g = blockIdx.x, lane = threadIdx.x;
  if (g >= nsub) return;
  const UnSub U = subs[g];
  const UnBlock B = blk[U.block];
  const uint64_t D0 = B.dst + U.outRel;  // this sub-segment's first output byte
  if (B.stored) {
    const uint64_t s0 = (uint64_t)U.k * kUnSub;
    for (uint64_t j = lane; j < U.outLen; j += 64) img[D0 + j] = f[B.src + s0 + j];
    return;
  }
  uint64_t P = D0, synced = D0;
  // the sequences: the re-parsed prefix, then the speculative list from specFrom
  const uint4* lists[2] = {seqAll + (uint64_t)g * 2 * kUnSubCap, seqAll + (uint64_t)g * 2 * kUnSubCap + kUnSubCap};
  const uint32_t from[2] = {0u, U.specFrom}, to[2] = {U.preN, U.specN};
  for (int li = 0; li < 2; li++) {
    const uint4* seq = lists[li];
    for (uint32_t b0 = from[li]; b0 < to[li]; b0 += 64) {
      const uint32_t cnt = to[li] - b0 < 64u ? to[li] - b0 : 64u;
      const uint4 q = lane < cnt ? seq[b0 + lane] : make_uint4(0u, 0u, 0u, 0u);
      const uint32_t tot = q.x + q.y;
      const uint32_t incl = un_incl_scan_add(tot, lane);
      const uint32_t rel = incl - tot;  // output offset of the literals from P
      for (uint32_t j = 0; j < cnt; j++) {
        const uint32_t L = un_rdlane(q.x, j), M = un_rdlane(q.y, j), off = un_rdlane(q.z, j), fr = un_rdlane(q.w, j);
        const uint64_t Pj = P + un_rdlane(rel, j);
        for (uint64_t k = lane; k < L; k += 64) {
          const uint32_t v = f[B.src + fr + k];
          img[Pj + k] = v;
          ring[(Pj + k) & (kRingU - 1u)] = v;
        }
        if (!M) continue;
        const uint64_t Q = Pj + L;
        const int64_t lo = (int64_t)Q - (int64_t)off;
        const uint32_t qq = off >= 64u ? off : off * ((64u + off - 1u) / off);
        for (uint64_t k = 0; k < M; k += 64) {
          const uint64_t cur = Q + k;
          if (cur - synced >= kSyncU) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            synced = cur;
          }
          const int64_t ringLo = (int64_t)cur + 64 - (int64_t)kRingU;
          const uint64_t jj = k + lane;
          const int64_t src = k == 0 ? lo + (int64_t)(off >= 64u ? lane : lane % off) : (int64_t)(Q + jj) - (int64_t)qq;
          uint32_t v = 0;
          if (jj < M) {
            if (src >= (int64_t)D0 && src >= ringLo) v = ring[(uint64_t)src & (kRingU - 1u)];
            else if (src >= (int64_t)D0) v = img[src];              // own, drained
            else if (src >= 0) v = kUnRef | (uint32_t)src;            // another wavefront's byte
            else if ((uint64_t)(-src) <= dl) v = dict[dl - (uint64_t)(-src)];  // the dictionary's tail
            // else 0: before the history (oz_unlz4's zero-initialised history)
            img[Q + jj] = v;
            ring[(Q + jj) & (kRingU - 1u)] = v;
          }
        }
      }
      P += un_rdlane(incl, cnt - 1u);
    }
  }
}

// image -> bytes, references resolved on the way: a word kUnRef | p is "the same byte as output position
// p", and p's word is a value or a reference to an earlier byte (each hop lands in an earlier
// sub-segment), so following it ends.  A resolved word is written back, which shortens the chains other
// lanes follow through it; a lane may read a word before or after another lane's write-back, and both are
// the same byte.  hops: the longest chain followed (atomic max).
__global__ __launch_bounds__(256) void k_unlz4_pack(uint32_t* __restrict__ img, uint64_t total, uint8_t* __restrict__ out,
                                                    uint32_t* __restrict__ hops)
{
  uint32_t most = 0;
  auto resolve = [&](uint64_t o, uint32_t v) -> uint32_t {
    if (!(v & kUnRef)) return v;
    uint32_t h = 0, w = v;
    while (w & kUnRef) {
      w = __hip_atomic_load(&img[w & ~kUnRef], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      h++;
    }
    __hip_atomic_store(&img[o], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    most = h > most ? h : most;
    return w;
  };
  for (uint64_t o = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4; o < total; o += (uint64_t)gridDim.x * 1024) {
    if (o + 4 <= total && ((reinterpret_cast<uintptr_t>(out + o) & 3u) == 0)) {
      const uint4 v = *reinterpret_cast<const uint4*>(img + o);
      const uint32_t a = resolve(o, v.x), b = resolve(o + 1, v.y), c = resolve(o + 2, v.z), d = resolve(o + 3, v.w);
      *reinterpret_cast<uint32_t*>(out + o) = (a & 0xFFu) | ((b & 0xFFu) << 8) | ((c & 0xFFu) << 16) | (d << 24);
    } else {
      for (uint64_t j = o; j < o + 4 && j < total; j++) out[j] = (uint8_t)resolve(j, img[j]);
    }
  }
  const uint32_t m = __reduce_max_sync(~0ull, most);
  if ((threadIdx.x & 63u) == 0 && m) atomicMax(hops, m);
}

void launch_unlz4_split_sizes(const uint8_t* f, uint64_t n, UnBlock* blk, uint32_t nb, UnSub* subs, uint32_t nsub,
                              uint4* seq, uint32_t* masks, hipStream_t s)
{
  if (nsub) hipLaunchKernelGGL(k_unlz4_spec, dim3(nsub), dim3(64), 0, s, f, n, blk, subs, nsub, seq, masks);
  for (uint32_t round = 0; round < kJoinRounds && nsub; round++)
    hipLaunchKernelGGL(k_unlz4_join, dim3(nsub), dim3(64), 0, s, f, n, blk, subs, nsub, seq, masks, round);
  if (nb) hipLaunchKernelGGL(k_unlz4_fix, dim3(nb), dim3(64), 0, s, f, n, blk, nb, subs, seq, masks);
}

void launch_unlz4_split_decode(const uint8_t* f, uint64_t n, const UnBlock* blk, const UnSub* subs, uint32_t nsub,
                               const uint4* seq, uint32_t* image, const uint8_t* dict, uint64_t dl, hipStream_t s)
{
  if (nsub) hipLaunchKernelGGL(k_unlz4_sub, dim3(nsub), dim3(64), 0, s, f, n, blk, subs, nsub, seq, image, dict, dl);
}

void launch_unlz4_pack(uint32_t* image, uint64_t total, uint8_t* out, uint32_t* hops, hipStream_t s)
{
  const uint64_t g = std::min<uint64_t>((total + 1023) / 1024, 8192);
  if (total) hipLaunchKernelGGL(k_unlz4_pack, dim3((uint32_t)g), dim3(256), 0, s, image, total, out, hops);
}

void launch_unlz4_index(const uint8_t* f, uint64_t n, UnBlock* blk, uint64_t maxBlocks, uint64_t* meta, hipStream_t s)
{
  hipLaunchKernelGGL(k_unlz4_index, dim3(1), dim3(64), 0, s, f, n, blk, maxBlocks, meta);
}

// the parallel index's scratch for a frame of n bytes, carved in this order
struct IxLayout {
  uint64_t words, nWg, cap, off[7], total;
  explicit IxLayout(uint64_t n)
  {
    words = n / 32 + 2;  // offsets from r0 rounded down to 4 up to n inclusive
    nWg = (words + kIxWgWords - 1) / kIxWgWords;
    cap = unlz4_ix_cap(n);
    const uint64_t bytes[7] = {4 * words, 4 * words, 4 * (nWg + 1), 4 * (nWg + 1), 8 * cap, 4 * cap, 4 * cap};
    total = 0;
    for (int k = 0; k < 7; k++) {
      off[k] = total;
      total += (bytes[k] + 255) & ~255ull;
    }
  }
};

uint64_t unlz4_ix_cap(uint64_t n) { return n / 128 + 65536; }

uint64_t unlz4_ix_scratch_bytes(uint64_t n) { return IxLayout(n).total; }

void launch_unlz4_index_par(const uint8_t* f, uint64_t n, void* scratch, UnBlock* blk, uint64_t maxBlocks, uint64_t* meta,
                            hipStream_t s)
{
  const IxLayout L(n);
  uint8_t* p = static_cast<uint8_t*>(scratch);
  const uint64_t words = L.words, cap = L.cap;
  const uint32_t nWg = (uint32_t)L.nWg;
  uint32_t* bits = reinterpret_cast<uint32_t*>(p + L.off[0]);
  uint32_t* wordPre = reinterpret_cast<uint32_t*>(p + L.off[1]);
  uint32_t* wgCount = reinterpret_cast<uint32_t*>(p + L.off[2]);
  uint32_t* wgOff = reinterpret_cast<uint32_t*>(p + L.off[3]);
  uint64_t* list = reinterpret_cast<uint64_t*>(p + L.off[4]);
  uint32_t* link = reinterpret_cast<uint32_t*>(p + L.off[5]);
  uint32_t* chain = reinterpret_cast<uint32_t*>(p + L.off[6]);
  hipLaunchKernelGGL(k_unlz4_ix_cand, dim3(nWg), dim3(1024), 0, s, f, n, words, bits, wgCount);
  hipLaunchKernelGGL(k_unlz4_ix_scan, dim3(1), dim3(1024), 0, s, wgCount, nWg, wgOff);
  hipLaunchKernelGGL(k_unlz4_ix_list, dim3(nWg), dim3(256), 0, s, f, n, words, bits, wgOff, nWg, cap, wordPre, list);
  hipLaunchKernelGGL(k_unlz4_ix_link, dim3(nWg), dim3(64), 0, s, f, n, words, bits, wgOff, nWg, cap, wordPre, list, link);
  hipLaunchKernelGGL(k_unlz4_ix_walk, dim3(1), dim3(1024), 0, s, f, n, words, bits, wgOff, nWg, cap, wordPre, list, link,
                     chain, blk, maxBlocks, meta);
}

uint64_t unlz4_seq_entries(uint64_t frameLen, uint32_t nb) { return frameLen / 3 + 2ull * nb + 2; }

void launch_unlz4_sizes(const uint8_t* f, uint64_t n, UnBlock* blk, uint32_t nb, uint4* seq, hipStream_t s)
{
  if (nb) hipLaunchKernelGGL(k_unlz4_sizes, dim3(nb), dim3(64), 0, s, f, n, blk, nb, seq);
}

void launch_unlz4_blocks(const uint8_t* f, uint64_t n, const UnBlock* blk, uint32_t nb, const uint4* seq, uint8_t* out,
                         const uint8_t* dict, uint64_t dl, uint32_t* flags, hipStream_t s)
{
  if (nb) hipLaunchKernelGGL(k_unlz4_blocks, dim3(nb), dim3(64), 0, s, f, n, blk, nb, seq, out, dict, dl, flags);
}

}  // namespace sz4
#if SZ4_DIAG == 8
extern "C" int sz4_udiag_read(uint64_t* out, uint64_t n)
{
  if (n > 16) n = 16;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sz4::sz4_udiag), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int sz4_udiag_clear()
{
  uint64_t z[16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(sz4::sz4_udiag), z, sizeof z, 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
#endif
