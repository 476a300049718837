// sz4_unlz4.hip -- gfx950 decoder for LZ4 frames with the semantics of the reference's decoder
// smallz4cat (unlz4_userPtr, smallz4cat.c:112-360) as the oracle restates it (oz_unlz4 in
// oracle/smallz4_oracle.c): modern and legacy frames, stored blocks, block and content checksums
// skipped, content-size and dictionary-ID fields skipped, an optional dictionary whose last 64 KiB
// precede the output (smallz4cat.c:168-187), legacy decoding ending after the first block shorter
// than 8 MiB (smallz4cat.c:325-327).
//
//   k_unlz4_index   one lane walks the block size words (a dependent chain, smallz4cat.c:189-205)
//   k_unlz4_sizes   one wavefront per block: token headers only -> decoded length, validation
//   (host)          output offset of every block, legacy truncation, capacity check
//   k_unlz4_blocks  one wavefront per block: token headers from a 256-byte register window, literal
//                   and match bytes 64 per step, the block's last 64 KiB of output in an LDS ring
//                   (the reference's history[], smallz4cat.c:161-166).  A match reaching below the
//                   block start waits for the blocks it reads: blocks are claimed in order through
//                   a ticket (placement independent), each publishes a done flag (agent release),
//                   a waiter polls relaxed, then acquires; every spin is bounded.
//
// Byte work only: decoding one block is a chain of token headers, so the parallelism is one
// wavefront per block and 64 bytes per copy step.
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

// Decode (kWrite) or measure (!kWrite) one block.  Returns its decoded length, or kNone when it is
// malformed the way oz_unlz4 rejects it: a length byte, literal run or offset running past the
// block, or offset 0 (smallz4cat.c:212-323).
template <bool kWrite>
__device__ uint64_t unlz4_block(const uint8_t* __restrict__ f, uint64_t n, const UnBlock& B, uint32_t bi, uint32_t lane,
                                uint8_t* __restrict__ out, uint8_t* __restrict__ ring, const uint8_t* __restrict__ dict,
                                uint64_t dl, const UnBlock* __restrict__ blk, uint32_t* __restrict__ done,
                                uint32_t* __restrict__ status)
{
  if (B.stored) {
    // uncompressed block (smallz4cat.c:329-343): later blocks read it from `out`
    if (kWrite)
      for (uint64_t k = lane; k < B.len; k += 64) out[B.dst + k] = f[B.src + k];
    return B.len;
  }
  const uint64_t end = B.src + B.len;
  uint64_t r = B.src, w = 0;  // frame cursor; bytes decoded so far (output position B.dst + w)
  uint64_t floorPos = B.dst;  // output below this is read only after its blocks are done
  uint32_t waitIdx = bi;
  Window win{f, n, 0, 0};
  win.fill(r, lane);
  while (r < end) {
    const uint32_t tok = win.byte(r++, lane);
    uint64_t lits = tok >> 4;
    if (lits == 15) {
      uint32_t x;
      do {
        if (r >= end) return kNone;
        x = win.byte(r++, lane);
        lits += x;
      } while (x == 255);
    }
    if (r + lits > end) return kNone;
    if (kWrite && lits) {
      const uint64_t P = B.dst + w;
      if (lits <= 64) {
        // lane j takes byte r + j out of the register window
        if (r + lits > win.base + 256) win.fill(r, lane);
        const uint32_t rel = (uint32_t)(r - win.base) + lane;
        const uint32_t word = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((rel >> 2) << 2), (int)win.w);
        const uint8_t v = (uint8_t)(word >> (8 * (rel & 3)));
        if (lane < lits) {
          out[P + lane] = v;
          ring[(P + lane) & 0xFFFFu] = v;
        }
      } else {
        for (uint64_t k = lane; k < lits; k += 64) {
          const uint8_t v = f[r + k];
          out[P + k] = v;
          ring[(P + k) & 0xFFFFu] = v;
        }
      }
    }
    w += lits;
    r += lits;
    if (r == end) break;  // the last sequence has literals only
    if (r + 2 > end) return kNone;
    const uint32_t off = win.byte(r, lane) | (win.byte(r + 1, lane) << 8);
    r += 2;
    if (off == 0) return kNone;  // "invalid offset" (smallz4cat.c:265-267)
    uint64_t ml = kMinMatch + (tok & 15);
    if (ml == kMinMatch + 15) {
      uint32_t x;
      do {
        if (r >= end) return kNone;
        x = win.byte(r++, lane);
        ml += x;
      } while (x == 255);
    }
    if (kWrite) {
      const uint64_t P = B.dst + w;
      const int64_t lo = (int64_t)P - (int64_t)off;  // lowest byte this match reads
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
      // output P + j = output P + j - off.  First step: lane j reads P - off + (j mod off), all
      // written before the match.  Later steps read P + j - q with q the smallest multiple of off
      // that is >= 64: the previous step's bytes (period off), so the ring never needs more than
      // 64 KiB even for matches longer than that.
      const uint32_t q = off >= 64u ? off : off * ((64u + off - 1u) / off);
      for (uint64_t k = 0; k < ml; k += 64) {
        const uint64_t j = k + lane;
        const int64_t s = k == 0 ? lo + (int64_t)(off >= 64u ? lane : lane % off) : (int64_t)(P + j) - (int64_t)q;
        uint8_t v = 0;
        if (j < ml) {
          if (s >= (int64_t)B.dst) v = ring[(uint64_t)s & 0xFFFFu];
          else if (s >= 0) v = out[s];                                   // an earlier block (finished)
          else if ((uint64_t)(-s) <= dl) v = dict[dl - (uint64_t)(-s)];  // the dictionary's tail
          // else 0: before the history (oz_unlz4's zero-initialised history)
        }
        if (j < ml) {
          out[P + j] = v;
          ring[(P + j) & 0xFFFFu] = v;
        }
      }
    }
    w += ml;
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
                                                    uint32_t nb)
{
  const uint32_t bi = blockIdx.x, lane = threadIdx.x;
  if (bi >= nb) return;
  const UnBlock B = blk[bi];
  const uint64_t size = unlz4_block<false>(f, n, B, bi, lane, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr);
  if (lane == 0) blk[bi].size = size;
}

// flags[0..nb) done flags, flags[nb] status bits, flags[nb + 1] ticket (all zeroed before the launch)
__global__ __launch_bounds__(64) void k_unlz4_blocks(const uint8_t* __restrict__ f, uint64_t n, const UnBlock* __restrict__ blk,
                                                     uint32_t nb, uint8_t* __restrict__ out, const uint8_t* __restrict__ dict,
                                                     uint64_t dl, uint32_t* __restrict__ flags)
{
  __shared__ uint8_t ring[65536];
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
  const uint64_t got = unlz4_block<true>(f, n, B, bi, lane, out, ring, dict, dl, blk, done, status);
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

void launch_unlz4_sizes(const uint8_t* f, uint64_t n, UnBlock* blk, uint32_t nb, hipStream_t s)
{
  if (nb) hipLaunchKernelGGL(k_unlz4_sizes, dim3(nb), dim3(64), 0, s, f, n, blk, nb);
}

void launch_unlz4_blocks(const uint8_t* f, uint64_t n, const UnBlock* blk, uint32_t nb, uint8_t* out, const uint8_t* dict,
                         uint64_t dl, uint32_t* flags, hipStream_t s)
{
  if (nb) hipLaunchKernelGGL(k_unlz4_blocks, dim3(nb), dim3(64), 0, s, f, n, blk, nb, out, dict, dl, flags);
}

}  // namespace sz4
