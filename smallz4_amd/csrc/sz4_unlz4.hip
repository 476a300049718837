// sz4_unlz4.hip -- gfx950 decoder for LZ4 frames with the semantics of the reference's decoder
// smallz4cat (unlz4_userPtr, smallz4cat.c:112-360) as the oracle restates it (oz_unlz4 in
// oracle/smallz4_oracle.c): modern and legacy frames, stored blocks, block and content checksums
// skipped, content-size and dictionary-ID fields skipped, an optional dictionary whose last 64 KiB
// precede the output (smallz4cat.c:168-187), legacy decoding ending after the first block shorter
// than 8 MiB (smallz4cat.c:325-327).
//
//   k_unlz4_index   one lane walks the block size words (a dependent chain, smallz4cat.c:189-205)
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
// Byte work only: decoding one block is a chain of sequences (each match may read the bytes the one
// before it wrote), so the parallelism is one wavefront per block and 64 bytes per copy step.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sz4_internal.h"

namespace sz4 {

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

__device__ __forceinline__ uint32_t un_incl_scan_add(uint32_t v, uint32_t lane)
{
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += o;
  }
  return v;
}

// Sequence list of block bi: at most len/3 + 2 entries (a sequence with a match takes >= 3 frame
// bytes), at seqAll + src/3 + 2 * bi -- disjoint from every other block's, no host prefix needed.
__device__ __forceinline__ uint4* seq_base(uint4* seqAll, const UnBlock& B, uint32_t bi)
{
  return seqAll + B.src / 3 + 2ull * bi;
}
__device__ __forceinline__ uint32_t seq_cap(const UnBlock& B) { return B.len / 3 + 2; }

// Header walk of one block (smallz4cat.c:212-323): its decoded length, or kNone when it is malformed
// the way oz_unlz4 rejects it (a length byte, literal run or offset running past the block, offset 0).
// Every sequence is recorded as (literals, match length, offset, frame offset of the literals from
// B.src): lane l holds entry (count & ~63) + l until 64 are complete, then one coalesced store.
__device__ uint64_t unlz4_parse(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, uint32_t lane,
                                uint4* __restrict__ seq, uint32_t* nseq)
{
  *nseq = 0;
  if (B.stored) return B.len;  // uncompressed block (smallz4cat.c:329-343)
  const uint64_t end = B.src + B.len;
  const uint32_t cap = seq_cap(B);
  uint64_t r = B.src, w = 0;  // frame cursor; bytes decoded so far
  uint32_t ns = 0;
  uint4 buf = make_uint4(0u, 0u, 0u, 0u);
  auto push = [&](uint32_t lits, uint32_t ml, uint32_t off, uint32_t frel) {
    const uint32_t l = ns & 63u;
    buf.x = un_wrlane(buf.x, lits, l);
    buf.y = un_wrlane(buf.y, ml, l);
    buf.z = un_wrlane(buf.z, off, l);
    buf.w = un_wrlane(buf.w, frel, l);
    ns++;
    if ((ns & 63u) == 0u) seq[ns - 64u + lane] = buf;
  };
  Window win{f, n, 0, 0};
  // One sequence byte by byte through the window (smallz4cat.c:212-323): 0 next, 1 block done, 2 malformed.
  // Taken for what the pre-decoded headers below do not cover: extended literal runs, match lengths
  // with more than one extension byte, headers reaching past the register window.
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
  // A sequence starting 20 or more bytes before the block end passes every bounds check of one_seq
  // (its header reads at most 18 bytes past the token, its literals end before the block does), so the
  // walk below checks nothing but a zero offset and runs on block-relative 32-bit cursors.
  const uint32_t fastEnd = B.len > 20u ? B.len - 20u : 0u;
  while (r < end) {
    // Pre-decode a header at every window position q = 4 lane + k: token | offset << 8 | extension
    // byte << 24, or ~0 when the header needs the byte-wise path (literal run >= 15, a second match
    // extension byte, or bytes past the register window).  The walk costs one readlane per sequence.
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
      const bool ok = (tok >> 4) != 15u && last < 256u && !(ext && ((v >> 16) & 0xFFu) == 255u);
      cand[k] = ok ? (tok | (v << 8)) : 0xFFFFFFFFu;  // v's bytes 0-2: offset, extension byte
    }
    const uint32_t wb = (uint32_t)(win.base - B.src);  // window base, block-relative (r >= B.src >= base - 3)
    uint32_t rr = (uint32_t)(r - B.src);
    bool slow = false;
    while (rr < fastEnd) {
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
      if (off == 0) return kNone;  // "invalid offset" (smallz4cat.c:265-267)
      const uint32_t lits = (pk >> 4) & 15u, nib = pk & 15u;
      const uint32_t ml = kMinMatch + nib + (nib == 15u ? pk >> 24 : 0u);
      push(lits, ml, off, rr + 1u);
      w += lits + ml;
      rr += 3u + lits + (nib == 15u ? 1u : 0u);
    }
    r = B.src + rr;
    if (rr < fastEnd && !slow) continue;  // refill
    // byte-wise: a header the window could not pre-decode, or the block's last 20 bytes
    if (r >= end) break;
    if (ns >= cap) return kNone;  // cannot happen in a well-formed block
    const int e = one_seq();
    if (e == 2) return kNone;
    if (e == 1) break;
  }
  if (ns & 63u) {
    const uint32_t b = ns & ~63u;
    if (lane < (ns & 63u)) seq[b + lane] = buf;
  }
  *nseq = ns;
  return w;
}

// Replays block bi's sequence list into `out` (and the ring); returns the decoded length.
__device__ uint64_t unlz4_decode(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, uint32_t bi, uint32_t lane,
                                 const uint4* __restrict__ seq, uint8_t* __restrict__ out, uint8_t* __restrict__ ring,
                                 const uint8_t* __restrict__ dict, uint64_t dl, const UnBlock* __restrict__ blk,
                                 uint32_t* __restrict__ done, uint32_t* __restrict__ status)
{
  if (B.stored) {
    // later blocks read it from `out`
    for (uint64_t k = lane; k < B.len; k += 64) out[B.dst + k] = f[B.src + k];
    return B.len;
  }
  uint64_t floorPos = B.dst;  // output below this is read only after its blocks are done
  uint32_t waitIdx = bi;
  uint64_t w = 0;             // bytes decoded so far
  uint64_t synced = B.dst;    // this block's output below it is drained and readable from `out`
  for (uint32_t b0 = 0; b0 < B.nseq; b0 += 64) {
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

}  // namespace

// one lane walks the size words: meta[0] = blocks found, meta[1] = 0 (frame end reached),
// 1 (malformed after meta[0] blocks) or 2 (more than maxBlocks), meta[2] = legacy frame
__global__ __launch_bounds__(64) void k_unlz4_index(const uint8_t* __restrict__ f, uint64_t n, UnBlock* __restrict__ blk,
                                                    uint64_t maxBlocks, uint64_t* __restrict__ meta)
{
  if (threadIdx.x != 0) return;
  auto rd32 = [&](uint64_t o) {
    return (uint32_t)f[o] | ((uint32_t)f[o + 1] << 8) | ((uint32_t)f[o + 2] << 16) | ((uint32_t)f[o + 3] << 24);
  };
  uint64_t nb = 0, st = 0, r = 4;
  bool legacy = false, blockSum = false;
  if (n < 4) {
    st = 1;
  } else {
    // signature and frame descriptor (smallz4cat.c:114-159)
    const uint32_t magic = rd32(0);
    const bool modern = magic == 0x184D2204u;
    legacy = magic == 0x184C2102u;
    if (!modern && !legacy) {
      st = 1;
    } else if (modern) {
      if (r + 1 > n) {
        st = 1;
      } else {
        const uint32_t flg = f[r++];
        if ((flg >> 6) != 1u) st = 1;
        blockSum = (flg & 16u) != 0;
        const uint64_t skip = 1 + ((flg & 8u) ? 8 : 0) + ((flg & 1u) ? 4 : 0) + 1;
        if (r + skip > n) st = 1;
        else r += skip;
      }
    }
  }
  // blocks until the end mark (smallz4cat.c:189-205, 345-349)
  while (st == 0) {
    if (r == n && legacy) break;
    if (r + 4 > n) { st = 1; break; }
    uint32_t word = rd32(r);
    r += 4;
    const bool packed = legacy || (word & 0x80000000u) == 0;
    if (!legacy) word &= 0x7FFFFFFFu;
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
    r += word;
    if (blockSum) {
      if (r + 4 > n) { st = 1; break; }
      r += 4;
    }
  }
  meta[0] = nb;
  meta[1] = st;
  meta[2] = legacy ? 1 : 0;
}

__global__ __launch_bounds__(64) void k_unlz4_sizes(const uint8_t* __restrict__ f, uint64_t n, UnBlock* __restrict__ blk,
                                                    uint32_t nb, uint4* __restrict__ seqAll)
{
  const uint32_t bi = blockIdx.x, lane = threadIdx.x;
  if (bi >= nb) return;
  const UnBlock B = blk[bi];
  uint32_t ns = 0;
  const uint64_t size = unlz4_parse(f, n, B, lane, seq_base(seqAll, B, bi), &ns);
  if (lane == 0) {
    blk[bi].size = size;
    blk[bi].nseq = ns;
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
  const uint64_t got = unlz4_decode(f, n, B, bi, lane, seq_base(const_cast<uint4*>(seqAll), B, bi), out, ring, dict, dl, blk,
                                    done, status);
  if (lane == 0 && got != B.size) atomicOr(status, 1u);
  // publish: this wave's stores drained, written back (agent release), then the flag
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(&done[bi], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

void launch_unlz4_index(const uint8_t* f, uint64_t n, UnBlock* blk, uint64_t maxBlocks, uint64_t* meta, hipStream_t s)
{
  hipLaunchKernelGGL(k_unlz4_index, dim3(1), dim3(64), 0, s, f, n, blk, maxBlocks, meta);
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
