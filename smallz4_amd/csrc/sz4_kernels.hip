// sz4_kernels.hip -- gfx950 kernels of the LZ4 optimal-parse compressor.
//
// Pipeline per batch of blocks (all data resident in HBM):
//   k_runs         same-letter runs -> shortcut intervals              (smallz4.h:631-643)
//   k_find_sorted  per segment, first the sort of its positions by (4-byte key hash, position), which
//                  replaces the previousHash/previousExact chains      (smallz4.h:645-720)
//                  then pass 1, lane = target in sorted order: longest match over its key group
//                                                                      (smallz4.h:173-255)
//   k_find_big / k_find_long9 / k_find   pass 2: big groups, long matches, shortcut intervals
//   k_prep         never-searched tail positions
//   k_lazy_*       greedy/lazy skip bookkeeping in parallel, shortcut intervals checked
//                                                                      (smallz4.h:631-643, 726-744)
//   k_dp_spec / k_dp_fix    backward optimal parse as speculative segments + repair
//                                                                      (smallz4.h:376-472)
//   k_walk / k_walk_fix     forward walk of the parse choices          (smallz4.h:259-300)
//   k_seg_scan, k_seg_tokens, k_block_bytes, k_scan, k_write_seg
//                  tokens, sizes, stored/compressed decision, frame    (smallz4.h:300-371, 762-813)
//   k_dict_matches dictionary mode: the reference's match loop replayed by one wavefront
//
// Integer/byte work only: no MFMA.  The reference semantics each kernel must
// reproduce are restated in DESIGN.md section 3.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "sz4_internal.h"
#include "sz4_device.h"

#ifndef SZ4_SKIP_SHIFT  // timing experiments only (results wrong): leave out a phase of k_find_sorted
#define SZ4_SKIP_SHIFT 0
#endif
#ifndef SZ4_SKIP_BCAST
#define SZ4_SKIP_BCAST 0
#endif
#ifndef SZ4_SKIP_SEARCH
#define SZ4_SKIP_SEARCH 0
#endif
#ifndef SZ4_DIAG
#define SZ4_DIAG 0  // diagnostic builds only: 3 = per-wave timeline of k_find_sorted in sz4_diag[]
#endif
// SZ4_Dn(statements): the statements in the SZ4_DIAG == n build only (tools/build_diag.sh n; 3: k_find_sorted's
// per-wave counters, 5: k_find_long9's, 6: k_find_big's phase clocks, 7: k_dp_fix's repair counters)
#if SZ4_DIAG == 3
#define SZ4_D3(...) __VA_ARGS__
#else
#define SZ4_D3(...)
#endif
#if SZ4_DIAG == 5
#define SZ4_D5(...) __VA_ARGS__
#else
#define SZ4_D5(...)
#endif
#if SZ4_DIAG == 7
#define SZ4_D7(...) __VA_ARGS__
#else
#define SZ4_D7(...)
#endif

namespace sz4 {

// ------------------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------------------

__device__ __forceinline__ uint32_t lload4(const uint32_t* w, uint32_t off)
{
  const uint32_t lo = w[off >> 2], hi = w[(off >> 2) + 1];
  return __builtin_amdgcn_alignbyte(hi, lo, off & 3);
}


// v_ffbl_b32: index of the lowest set bit, ~0u for 0 (defined, unlike __builtin_ctz)
__device__ __forceinline__ uint32_t ffbl(uint32_t x)
{
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v)
{
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t o = __shfl_xor(v, m, 64);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ int32_t wave_max_i32(int32_t v)
{
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const int32_t o = __shfl_xor(v, m, 64);
    v = o > v ? o : v;
  }
  return v;
}

// clears bit idx of `bits` for the lanes where `pred` holds: one atomic per distinct word (lanes with
// nearby indices share words; 64 atomics on one address serialise in L2)
__device__ __forceinline__ void wave_clear_bits(uint32_t* bits, uint64_t idx, bool pred)
{
  uint64_t rest = __ballot(pred);
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint64_t w = idx >> 5;
  while (rest) {
    const uint32_t l = (uint32_t)__builtin_ctzll(rest);
    const uint64_t wl = ((uint64_t)__builtin_amdgcn_readlane((int)(w >> 32), l) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w, l);
    const bool mine = pred && w == wl;
    uint32_t m = mine ? 1u << (idx & 31) : 0u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m |= (uint32_t)__shfl_xor((int)m, d, 64);
    if (lane == l) atomicAnd(&bits[wl], ~m);
    rest &= ~__ballot(mine);
  }
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint32_t o = __shfl_xor(v, m, 64);
    v = o < v ? o : v;
  }
  return v;
}


// DPP row (16-lane) permutations
#if SZ4_DIAG >= 3
__device__ uint64_t sz4_diag[1 << 20];
extern "C" int sz4_diag_read(uint64_t* out, uint64_t n)
{
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sz4_diag), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int sz4_diag_clear()
{
  static uint64_t zero[64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(sz4_diag), zero, sizeof zero, 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
#endif

// v_writelane (no clang builtin on this toolchain; the LLVM intrinsic by name): lane `l` of v
// becomes the uniform `x`
extern "C" __device__ int sz4_llvm_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wrlane(uint32_t v, uint32_t x, uint32_t l)
{
  return (uint32_t)sz4_llvm_writelane((int)x, (int)l, (int)v);
}

template <int kCtrl>
__device__ __forceinline__ uint32_t dpp(uint32_t v)
{
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
}
constexpr int kQuadSwap1 = 0xB1;      // quad_perm [1,0,3,2]
constexpr int kQuadSwap2 = 0x4E;      // quad_perm [2,3,0,1]
constexpr int kRowHalfMirror = 0x141;
constexpr int kRowMirror = 0x140;
constexpr int kRowShr = 0x110;        // + n
constexpr int kWaveShr1 = 0x138;      // wave_shr:1 (whole 64-lane wavefront)
constexpr int kRowBcast15 = 0x142;    // lane 15 of each row to the next row
constexpr int kRowBcast31 = 0x143;    // lane 31 to rows 2 and 3

// DPP into the rows of kRowMask only; the other rows (and lanes without a source) keep `old`
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_rows(uint32_t old, uint32_t v)
{
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kCtrl, kRowMask, 0xF, false);
}


// every lane receives the min / max of its 16-lane row
__device__ __forceinline__ uint32_t row_min(uint32_t v)
{
  v = min(v, dpp<kQuadSwap1>(v));
  v = min(v, dpp<kQuadSwap2>(v));
  v = min(v, dpp<kRowHalfMirror>(v));
  v = min(v, dpp<kRowMirror>(v));
  return v;
}
__device__ __forceinline__ uint32_t row_max(uint32_t v)
{
  v = max(v, dpp<kQuadSwap1>(v));
  v = max(v, dpp<kQuadSwap2>(v));
  v = max(v, dpp<kRowHalfMirror>(v));
  v = max(v, dpp<kRowMirror>(v));
  return v;
}
// inclusive max-scan inside each 16-lane row (lanes below the row start contribute 0)
__device__ __forceinline__ uint32_t row_scan_max(uint32_t v)
{
  v = max(v, dpp<kRowShr + 1>(v));
  v = max(v, dpp<kRowShr + 2>(v));
  v = max(v, dpp<kRowShr + 4>(v));
  v = max(v, dpp<kRowShr + 8>(v));
  return v;
}
// wave-wide min delivered to EVERY lane (no SGPR round trip): rows, then row pairs, then halves
__device__ __forceinline__ uint32_t wave_min_all(uint32_t v)
{
  v = row_min(v);
  auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = min(a[0], a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return min(b[0], b[1]);
}

// four wave-wide minima, interleaved so that no DPP step waits on the one before (no s_nop), rows
// joined with permlane swaps; results uniform
__device__ __forceinline__ void wave_min4(uint32_t (&v)[4])
{
#pragma unroll
  for (int r = 0; r < 4; r++) v[r] = min(v[r], dpp<kQuadSwap1>(v[r]));
#pragma unroll
  for (int r = 0; r < 4; r++) v[r] = min(v[r], dpp<kQuadSwap2>(v[r]));
#pragma unroll
  for (int r = 0; r < 4; r++) v[r] = min(v[r], dpp<kRowHalfMirror>(v[r]));
#pragma unroll
  for (int r = 0; r < 4; r++) v[r] = min(v[r], dpp<kRowMirror>(v[r]));
#pragma unroll
  for (int r = 0; r < 4; r++) {
    auto a = __builtin_amdgcn_permlane16_swap(v[r], v[r], false, false);
    v[r] = min(a[0], a[1]);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    auto b = __builtin_amdgcn_permlane32_swap(v[r], v[r], false, false);
    v[r] = (uint32_t)__builtin_amdgcn_readfirstlane((int)min(b[0], b[1]));
  }
}

// wave-wide max, result uniform
__device__ __forceinline__ uint32_t wave_max_fast(uint32_t v)
{
  v = row_max(v);
  const uint32_t a = rdlane(v, 0), b = rdlane(v, 16), c = rdlane(v, 32), d = rdlane(v, 48);
  return max(max(a, b), max(c, d));
}

// wave-wide min, result uniform
__device__ __forceinline__ uint32_t wave_min_fast(uint32_t v)
{
  v = row_min(v);
  const uint32_t a = rdlane(v, 0), b = rdlane(v, 16), c = rdlane(v, 32), d = rdlane(v, 48);
  return min(min(a, b), min(c, d));
}

// inclusive wavefront scans by DPP: row shifts 1, 2, 4, 8, then lane 15 of each row into the next row and
// lane 31 into rows 2-3, lanes without a source taking the identity (0 for + and unsigned max) -- six
// dependent VALU steps instead of six ds_bpermute round trips
__device__ __forceinline__ uint32_t wave_incl_scan_add(uint32_t v)
{
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowShr + 1, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowShr + 2, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowShr + 4, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowShr + 8, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowBcast15, 0xA, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowBcast31, 0xC, 0xF, false);
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan_max(uint32_t v)
{
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowShr + 1, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowShr + 2, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowShr + 4, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowShr + 8, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowBcast15, 0xA, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRowBcast31, 0xC, 0xF, false));
  return v;
}

// load that bypasses the vector L1 (sc1): for data this wavefront itself rewrote earlier in the
// same kernel -- a plain load may hit the stale L1 line
__device__ __forceinline__ uint32_t ld_fresh(const uint32_t* p)
{
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// is position q inside one of `cnt` intervals of list `iv`
__device__ __forceinline__ bool in_iv(const Interval* iv, uint32_t cnt, uint64_t q)
{
  for (uint32_t k = 0; k < cnt; k++)
    if (q >= iv[k].lo && q < iv[k].hi) return true;
  return false;
}

// ================================================================================================
// k_runs: one workgroup per block.  A run of one byte value longer than ~65300 bytes is where the
// reference's same-letter shortcut (smallz4.h:631-643) stops inserting positions.  For levels that
// search every position (maxChain > 6) the shortcut is fully determined by the run:
//   a  = first searched position of the run whose predecessor is in the run
//        (run start + 1, or the block start when the run began in the previous block),
//   La = min(run end, block end - 5) - a         (its distance-1 match, capped by the block),
//   skipped positions = [a + 1, a + La - MaxSameLetter]  when La > MaxSameLetter.
// ================================================================================================
__global__ __launch_bounds__(256) void k_runs(const uint8_t* __restrict__ in, const Block* __restrict__ blocks,
                                              Interval* __restrict__ ivOut, uint32_t* __restrict__ ivCount)
{
  const Block B = blocks[blockIdx.x];
  const uint32_t tid = threadIdx.x;
  Interval* iv = ivOut + (uint64_t)blockIdx.x * kMaxIv;
  __shared__ uint32_t s_count;
  __shared__ uint64_t s_hit;  // first probe position (relative) that may sit inside a long run
  __shared__ uint64_t s_edge;
  if (tid == 0) s_count = 0;
  const uint64_t n = B.end - B.start;
  if (n < (uint64_t)kSameLetter + kTailNoMatch + 2) {
    if (tid == 0) ivCount[blockIdx.x] = 0;
    return;
  }
  const uint64_t stopAbs = B.end - kTailLiterals;
  // a run longer than MaxSameLetter (65299) covers three consecutive multiples of 16384
  const uint64_t nprobe = (n + 16383) / 16384;
  uint64_t from = 0;  // relative position from which to look for the next run
  __syncthreads();
  while (true) {
    if (tid == 0) s_hit = kNone;
    __syncthreads();
    for (uint64_t k = tid; k + 2 < nprobe; k += blockDim.x) {
      const uint64_t p = k * 16384;
      if (p < from) continue;
      const uint8_t v = in[B.start + p];
      if (in[B.start + p + 16384] == v && in[B.start + p + 32768] == v) atomicMin((unsigned long long*)&s_hit, p);
    }
    __syncthreads();
    const uint64_t hit = s_hit;
    if (hit == kNone) break;
    const uint8_t v = in[B.start + hit];
    // run end e: first position > hit with a different byte (or block end)
    if (tid == 0) s_edge = n;
    __syncthreads();
    for (uint64_t base = hit; base < n; base += blockDim.x * 16) {
      bool found = false;
      for (uint32_t j = 0; j < 16; j++) {
        const uint64_t q = base + (uint64_t)tid * 16 + j;
        if (q < n && in[B.start + q] != v) { atomicMin((unsigned long long*)&s_edge, q); found = true; break; }
      }
      (void)found;
      __syncthreads();
      if (s_edge != n) break;
      __syncthreads();
    }
    __syncthreads();
    const uint64_t eRel = s_edge;
    __syncthreads();
    // run start r: scan left; may continue into the previous block when the block has lookback
    const bool canLookLeft = B.prev != kNoBlock;
    if (tid == 0) s_edge = kNone;  // holds (hit - r) once found
    __syncthreads();
    const uint64_t leftLimit = canLookLeft ? (hit + 1) : hit;  // how far left we may step from hit
    for (uint64_t base = 1; base <= leftLimit; base += blockDim.x * 16) {
      for (uint32_t j = 0; j < 16; j++) {
        const uint64_t back = base + (uint64_t)tid * 16 + j;
        if (back <= leftLimit && in[B.start + hit - back] != v) {
          atomicMin((unsigned long long*)&s_edge, back);
          break;
        }
      }
      __syncthreads();
      if (s_edge != kNone) break;
      __syncthreads();
    }
    __syncthreads();
    const uint64_t backHit = s_edge;  // first step left that leaves the run (kNone: none within limit)
    __syncthreads();
    if (tid == 0) {
      // run start r (relative); only whether it precedes the block start matters beyond that
      const bool beforeStart = canLookLeft && backHit == kNone;
      const uint64_t rRel = backHit == kNone ? 0 : hit - backHit + 1;
      const uint64_t a = beforeStart ? B.start : B.start + rRel + 1;
      const uint64_t eAbs = B.start + eRel;
      const uint64_t lim = eAbs < stopAbs ? eAbs : stopAbs;
      if (a + kTailNoMatch <= B.end && lim > a) {
        const uint64_t La = lim - a;
        if (La > kSameLetter && s_count < kMaxIv) {
          Interval t;
          t.lo = a + 1;
          t.hi = a + 1 + (La - kSameLetter);
          t.a = a;
          t.La = La;
          iv[s_count] = t;
          s_count = s_count + 1;
        }
      }
    }
    __syncthreads();
    from = eRel;  // continue after this run
    if (from >= n) break;
  }
  __syncthreads();
  if (tid == 0) ivCount[blockIdx.x] = s_count;
}

// ================================================================================================
// The sort (sort_segment, at the start of k_find_sorted): one 1024-thread workgroup per segment groups
// the inserted positions of the window [w0, s1) by their four key bytes, positions ascending inside a
// group.  Elements are packed 32-bit (hash << posBits | position - w0) with a 15/16-bit hash of the key;
// different keys that share a hash land in the same group and the searches compare the four key bytes
// themselves, so the candidate sets stay exact.  After the sort the candidates of target p are the
// same-key entries just below p's slot -- the reference's previousExact chain of p, nearest first.
// Stable MSD radix sort: one pass by the hash's high 8 bits through LDS, a tile of kSortTile elements at
// a time (the tile ranked by ballot, reordered by digit in LDS, written out as one contiguous run per
// digit: whole cache lines), its keys read straight from the text; then every high-digit bucket is sorted
// by its low digit by one wavefront taken from a counter: low-digit counts by LDS atomics, whose exclusive
// prefix is each hash group's start, and the elements ranked stably by ballot straight to their slots.
// Outputs (in bufB): per slot the window position and the slot where its hash group starts (u16 each when
// the window fits 16 bits, u32 otherwise).  The slot of a target is written by k_find_sorted for the
// targets it hands to pass 2 only.
// ================================================================================================
constexpr int kSortThreads = 1024;
constexpr int kSortWaves = kSortThreads / 64;
constexpr uint32_t kSortBatch = 8;                          // elements per lane per tile
constexpr uint32_t kSortTile = kSortThreads * kSortBatch;   // 8192 elements staged per tile
constexpr uint32_t kCoopBucket = 4096;  // a high-digit bucket larger than this is sorted by the whole workgroup

__device__ __forceinline__ uint32_t pos_bits(uint32_t W) { return W <= 65536u ? 16u : 17u; }
__device__ __forceinline__ uint32_t key_hash(uint32_t key, uint32_t posBits)
{
  return (key * 2654435761u) >> posBits;  // top (32 - posBits) bits of a multiplicative hash
}

constexpr uint32_t kKeyNone = 0xFFFFFF00u;  // an invalid parse key that survives a +192 bias

// The sort's shared memory (57 KB): k_find_sorted sorts its segment with it in the window buffer, which
// is loaded only after the sort
struct SortLds {
  uint32_t tile[kSortTile];        // a tile in digit order; the histogram pass's second table; the scan
  uint32_t cnt[kSortWaves][256];   // per wave and digit: count, then offset inside the tile
  uint32_t gOff[256];              // per high digit: next output slot
  uint32_t tileStart[256], tileCnt[256];
  uint64_t exLo[2 * kMaxIv], exHi[2 * kMaxIv];
  uint32_t wsum[kSortWaves];
  uint32_t nEx;
  uint32_t bstart[257];            // MSD: first slot of every high-digit bucket
  uint32_t bnext;                  // MSD: the next bucket a wave takes
  uint32_t nCoop;                  // buckets of more than kCoopBucket elements (step 4)
};

static_assert(sizeof(SortLds) <= 65536, "k_find_sorted sorts its segment inside the 64 KiB window buffer");

// exclusive prefix sum over the 256 digits of v (threads 0..255 hold one digit each), result in out
__device__ __forceinline__ void digit_scan(uint32_t v, uint32_t* out, uint32_t* wsum)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t incl = 0;
  if (tid < 256) {
    incl = wave_incl_scan_add(v);
    if (lane == 63) wsum[wave] = incl;
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t base = 0;
    for (uint32_t w = 0; w < wave; w++) base += wsum[w];
    out[tid] = base + incl - v;
  }
  __syncthreads();
}

__device__ __forceinline__ void sort_segment(const uint8_t* __restrict__ in, const Segment& S, const Block& B,
                                             const Interval* __restrict__ ivAll, const uint32_t* __restrict__ ivCount,
                                             uint2* bufA, uint2* bufB, SortLds& L)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));

  // positions excluded from insertion: shortcut intervals of this block and of the previous one
  if (tid == 0) {
    uint32_t k = 0;
    const uint32_t blkIds[2] = {B.prev, S.block};
    for (int t = 0; t < 2; t++) {
      if (blkIds[t] == kNoBlock) continue;
      const Interval* iv = ivAll + (uint64_t)blkIds[t] * kMaxIv;
      for (uint32_t j = 0; j < ivCount[blkIds[t]]; j++) {
        uint64_t lo = iv[j].lo > S.w0 ? iv[j].lo : S.w0;
        uint64_t hi = iv[j].hi < S.s1 ? iv[j].hi : S.s1;
        if (lo < hi) { L.exLo[k] = lo; L.exHi[k] = hi; k++; }
      }
    }
    L.nEx = k;
  }
  __syncthreads();
  const uint32_t ne = L.nEx;
  uint64_t excluded = 0;
  for (uint32_t j = 0; j < ne; j++) excluded += L.exHi[j] - L.exLo[j];

  const uint32_t W = (uint32_t)(S.s1 - S.w0);
  const uint32_t E = W - (uint32_t)excluded;
  const uint32_t pb = pos_bits(W);
  const uint32_t posMask = (1u << pb) - 1u;
  // element i of the compacted window: its position (intervals skipped; they are ordered and disjoint)
  auto elem_at = [&](uint32_t i) -> uint32_t {
    uint64_t q = S.w0 + i;
    for (uint32_t j = 0; j < ne; j++)
      if (q >= L.exLo[j]) q += L.exHi[j] - L.exLo[j];
    const uint32_t r = (uint32_t)(q - S.w0);
    return (key_hash(gload4(in, q), pb) << pb) | r;
  };

  // 1. the high digit's totals: per-wave histograms, then every digit's first slot (its bucket's start)
  const uint32_t sh = pb + 8u;
  for (uint32_t i = tid; i < kSortWaves * 256; i += kSortThreads) L.tile[i] = 0;
  __syncthreads();
  for (uint32_t i0 = tid; i0 < E; i0 += kSortThreads * kSortBatch) {
    uint32_t e[kSortBatch];
#pragma unroll
    for (uint32_t u = 0; u < kSortBatch; u++) e[u] = i0 + u * kSortThreads < E ? elem_at(i0 + u * kSortThreads) : 0u;
#pragma unroll
    for (uint32_t u = 0; u < kSortBatch; u++)
      if (i0 + u * kSortThreads < E) atomicAdd(&L.tile[wave * 256 + ((e[u] >> sh) & 255u)], 1u);
  }
  __syncthreads();
  {
    uint32_t h = 0;
    if (tid < 256)
      for (uint32_t w = 0; w < kSortWaves; w++) h += L.tile[w * 256 + tid];
    digit_scan(h, L.gOff, L.wsum);
  }
  if (tid < 256) L.bstart[tid] = L.gOff[tid];
  if (tid == 0) {
    L.bstart[256] = E;
    L.bnext = 0;
    L.nCoop = 0;
  }
  __syncthreads();
  if (tid < 256 && L.bstart[tid + 1] - L.bstart[tid] > kCoopBucket) atomicAdd(&L.nCoop, 1u);

  // 2. the stable pass by the high digit (buckets of equal high digit, positions ascending), keys from the
  //    text, a tile at a time ranked and reordered in LDS; every bucket is then sorted by its low digit by
  //    one wavefront (step 3)
  uint32_t* src = reinterpret_cast<uint32_t*>(bufA + S.elemOff);
  for (uint32_t t0 = 0; t0 < E; t0 += kSortTile) {
    const uint32_t tn = E - t0 < kSortTile ? E - t0 : kSortTile;
    for (uint32_t d = tid; d < kSortWaves * 256; d += kSortThreads) (&L.cnt[0][0])[d] = 0;
    __syncthreads();
    // wave w ranks elements [t0 + w * 512, +512), 64 per batch; (element, digit, rank in the wave)
    uint32_t e[kSortBatch], rk[kSortBatch];
    const uint32_t wb = t0 + wave * (64 * kSortBatch);
#pragma unroll
    for (uint32_t u = 0; u < kSortBatch; u++) {
      const uint32_t i = wb + 64 * u + lane;
      e[u] = i < t0 + tn ? elem_at(i) : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < kSortBatch; u++) {
      const uint32_t i = wb + 64 * u + lane;
      const bool valid = i < t0 + tn;
      const uint32_t d = (e[u] >> sh) & 255u;
      uint64_t peers = __ballot(valid);
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const uint64_t m = __ballot((d >> b) & 1);
        peers &= ((d >> b) & 1) ? m : ~m;
      }
      rk[u] = 0;
      if (valid) {
        const uint32_t below = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        rk[u] = L.cnt[wave][d] + below;
      }
      // the lowest lane of each digit advances the wave's count (after every lane has read it)
      const bool leader = valid && (peers & ((1ull << lane) - 1ull)) == 0;
      if (leader) L.cnt[wave][d] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // tile layout: digit-major, waves in order inside a digit
    uint32_t tc = 0;
    if (tid < 256)
      for (uint32_t w = 0; w < kSortWaves; w++) {
        const uint32_t c = L.cnt[w][tid];
        L.cnt[w][tid] = tc;
        tc += c;
      }
    digit_scan(tc, L.tileStart, L.wsum);
    if (tid < 256) {
      L.tileCnt[tid] = tc;
      const uint32_t st = L.tileStart[tid];
      for (uint32_t w = 0; w < kSortWaves; w++) L.cnt[w][tid] += st;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < kSortBatch; u++) {
      const uint32_t i = wb + 64 * u + lane;
      if (i < t0 + tn) L.tile[L.cnt[wave][(e[u] >> sh) & 255u] + rk[u]] = e[u];
    }
    __syncthreads();
    // one contiguous run per digit
    for (uint32_t i = tid; i < tn; i += kSortThreads) {
      const uint32_t v = L.tile[i];
      const uint32_t d = (v >> sh) & 255u;
      src[L.gOff[d] + (i - L.tileStart[d])] = v;
    }
    __syncthreads();
    if (tid < 256) L.gOff[tid] += L.tileCnt[tid];
    __syncthreads();
  }
  // the sorted elements are in bufA; bufB receives the per-slot arrays
  const bool small = W <= 65536u;  // == compact_small(S)
  uint16_t* pos16 = reinterpret_cast<uint16_t*>(bufB + S.elemOff);
  uint16_t* gs16 = pos16 + E;
  uint32_t* pos32 = reinterpret_cast<uint32_t*>(bufB + S.elemOff);
  uint32_t* gs32 = pos32 + E;
  // 3. every high-digit bucket by one wavefront, taken from a counter: its low digits counted, their
  //    exclusive prefix is each hash group's start (no scan over the segment), and the elements (in
  //    position order) are ranked stably by ballot, 64 at a time, straight to their final slots.
  //    A bucket of more than kCoopBucket elements (one frequent key: a run of one byte value, zero pages)
  //    is left to step 4, where the whole workgroup sorts it
  const uint32_t lowMask = 255u;
  // element e of the bucket starting at b0 to its slot g + r (g: its hash group's first slot)
  auto place = [&](uint32_t e, uint32_t g, uint32_t r) {
    const uint32_t rel = e & posMask;
    if (small) {
      pos16[g + r] = (uint16_t)rel;
      gs16[g + r] = (uint16_t)g;
    } else {
      pos32[g + r] = rel;
      gs32[g + r] = g;
    }
  };
  // the lanes of one 64-element batch with the same low digit as this lane's: (all of them, those below)
  auto peers_of = [&](bool valid, uint32_t x, uint64_t& below) -> uint64_t {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t m = __ballot((x >> b) & 1);
      peers &= ((x >> b) & 1) ? m : ~m;
    }
    below = peers & ((1ull << lane) - 1ull);
    return peers;
  };
  {
    uint32_t* run = L.cnt[wave];                 // per low digit: elements placed so far
    uint32_t* pre = L.tile + wave * 512u;        // per low digit: first slot inside the bucket
    while (true) {
      uint32_t d = 0;
      if (lane == 0) d = atomicAdd(&L.bnext, 1u);
      d = rdlane(d, 0);
      if (d >= 256u) break;
      const uint32_t b0 = L.bstart[d], b1 = L.bstart[d + 1];
      if (b0 == b1 || b1 - b0 > kCoopBucket) continue;
      for (uint32_t x = lane; x < 256u; x += 64) run[x] = 0;
      __builtin_amdgcn_wave_barrier();
      for (uint32_t i = b0 + lane; i < b1; i += 64) atomicAdd(&run[(src[i] >> pb) & lowMask], 1u);
      __builtin_amdgcn_wave_barrier();
      {
        // exclusive prefix of the 256 counts: lane l holds digits 4l .. 4l + 3
        uint32_t c[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          c[k] = run[4 * lane + k];
          sum += c[k];
        }
        const uint32_t incl = wave_incl_scan_add(sum);
        uint32_t acc = incl - sum;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          pre[4 * lane + k] = acc;
          run[4 * lane + k] = 0;
          acc += c[k];
        }
      }
      __builtin_amdgcn_wave_barrier();
      for (uint32_t i0 = b0; i0 < b1; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool valid = i < b1;
        const uint32_t e = valid ? src[i] : 0u;
        const uint32_t x = (e >> pb) & lowMask;
        uint64_t below;
        const uint64_t peers = peers_of(valid, x, below);
        if (valid) place(e, b0 + pre[x], run[x] + (uint32_t)__popcll(below));
        __builtin_amdgcn_wave_barrier();
        if (valid && below == 0) run[x] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  __syncthreads();
  // 4. the big buckets, each by the whole workgroup: wave w counts the low digits of the w-th sixteenth
  //    of it, every (digit, wave) gets its first slot (digit-major, waves in position order: stable), and
  //    each wave ranks its part by ballot as in step 3
  for (uint32_t d = 0; d < 256u && L.nCoop; d++) {
    const uint32_t b0 = L.bstart[d], b1 = L.bstart[d + 1];
    if (b1 - b0 <= kCoopBucket) continue;  // uniform
    const uint32_t per = (b1 - b0 + kSortWaves - 1) / kSortWaves;
    const uint32_t c0 = b0 + wave * per, c1 = min(c0 + per, b1);
    uint32_t* run = L.cnt[wave];
    for (uint32_t x = lane; x < 256u; x += 64) run[x] = 0;
    __syncthreads();
    for (uint32_t i = c0 + lane; i < c1; i += 64) atomicAdd(&run[(src[i] >> pb) & lowMask], 1u);
    __syncthreads();
    if (tid < 256) {  // digit tid: the waves' exclusive offsets inside it, its total
      uint32_t acc = 0;
      for (uint32_t w = 0; w < kSortWaves; w++) {
        const uint32_t c = L.cnt[w][tid];
        L.cnt[w][tid] = acc;
        acc += c;
      }
      L.tileCnt[tid] = acc;
    }
    __syncthreads();
    digit_scan(tid < 256 ? L.tileCnt[tid] : 0u, L.tileStart, L.wsum);  // every hash group's start
    for (uint32_t i0 = c0; i0 < c1; i0 += 64) {
      const uint32_t i = i0 + lane;
      const bool valid = i < c1;
      const uint32_t e = valid ? src[i] : 0u;
      const uint32_t x = (e >> pb) & lowMask;
      uint64_t below;
      const uint64_t peers = peers_of(valid, x, below);
      if (valid) place(e, b0 + L.tileStart[x], run[x] + (uint32_t)__popcll(below));
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) run[x] += (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
  }
}


// ================================================================================================
// k_find: longest match per target position.  One workgroup per segment; wavefronts take chunks
// of 64 consecutive positions and walk them in order.  For each position the wavefront scores
// 64 candidates of the sorted key group per step (nearest first), lanes reject a candidate with a
// single 4-byte compare at the length it would have to reach (the reference's phase 1), and the
// survivors compute their exact common prefix.
//
//  maxChain >= 65535 ("-9"): result = longest common prefix over all candidates, nearest on ties
//      (equivalent to the reference's strictly-improving walk).  Position p+1 starts from the
//      known match (dist d, len L-1) of position p, so long repeats are not re-extended.
//  maxChain <  65535: the reference's step limit counts strict improvements ("records") along the
//      chain; each 64-candidate step resolves its records with a wavefront prefix-max.
// ================================================================================================
constexpr int kFindThreads = 1024;  // 16 wavefronts (2 workgroups = 32 per CU with the 64 KiB window)

template <bool kLds>
struct Bytes;

template <>
struct Bytes<true> {
  const uint32_t* w;
  uint64_t base;
  __device__ __forceinline__ uint32_t ld4(uint64_t pos) const { return lload4(w, (uint32_t)(pos - base)); }
  // bytes pos .. pos + 11 as three little-endian words
  __device__ __forceinline__ void ld12(uint64_t pos, uint32_t& a, uint32_t& b, uint32_t& c) const
  {
    a = ld4(pos);
    b = ld4(pos + 4);
    c = ld4(pos + 8);
  }
  // bytes pos .. pos + 15 (reads up to pos + 19)
  __device__ __forceinline__ void ld16(uint64_t pos, uint32_t (&v)[4]) const
  {
    const uint32_t off = (uint32_t)(pos - base), i = off >> 2, sh = off & 3;
    const uint32_t w0 = w[i], w1 = w[i + 1], w2 = w[i + 2], w3 = w[i + 3], w4 = w[i + 4];
    v[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
    v[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
    v[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
    v[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
  }
};

template <>
struct Bytes<false> {
  const uint8_t* in;
  __device__ __forceinline__ uint32_t ld4(uint64_t pos) const { return gload4(in, pos); }
  // one 16-byte load (dword aligned; the staged input is padded) instead of three 8-byte ones: a third of
  // the memory instructions and L2 requests for a candidate's or target's first 12 bytes
  __device__ __forceinline__ void ld12(uint64_t pos, uint32_t& a, uint32_t& b, uint32_t& c) const
  {
    typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
    const u32x4a4 q = *reinterpret_cast<const u32x4a4*>(in + (pos & ~3ull));
    const uint32_t sh = (uint32_t)(pos & 3);
    a = __builtin_amdgcn_alignbyte(q.y, q.x, sh);
    b = __builtin_amdgcn_alignbyte(q.z, q.y, sh);
    c = __builtin_amdgcn_alignbyte(q.w, q.z, sh);
  }
  // bytes pos .. pos + 15: a 16-byte and a 4-byte load (reads up to pos + 19)
  __device__ __forceinline__ void ld16(uint64_t pos, uint32_t (&v)[4]) const
  {
    typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
    const uint8_t* a = in + (pos & ~3ull);
    const u32x4a4 q = *reinterpret_cast<const u32x4a4*>(a);
    const uint32_t w4 = *reinterpret_cast<const uint32_t*>(a + 16);
    const uint32_t sh = (uint32_t)(pos & 3);
    v[0] = __builtin_amdgcn_alignbyte(q.y, q.x, sh);
    v[1] = __builtin_amdgcn_alignbyte(q.z, q.y, sh);
    v[2] = __builtin_amdgcn_alignbyte(q.w, q.z, sh);
    v[3] = __builtin_amdgcn_alignbyte(w4, q.w, sh);
  }
};

// common prefix of the texts at x and y from byte k on (the first k known equal), at most cap: 16 bytes per
// step -- the loads of a step are independent, one latency per 16 bytes of a long match instead of one per 4
// -- while a whole step lies below cap, then 4 bytes per step (reading at most 3 bytes past cap, as before)
template <class Src>
__device__ __forceinline__ uint32_t ext_prefix(const Src& src, uint64_t x, uint64_t y, uint32_t k, uint32_t cap)
{
  while (k + 16 <= cap) {
    uint32_t a[4], b[4];
    src.ld16(x + k, a);
    src.ld16(y + k, b);
    const uint32_t d0 = a[0] ^ b[0], d1 = a[1] ^ b[1], d2 = a[2] ^ b[2], d3 = a[3] ^ b[3];
    if (d0 | d1 | d2 | d3) {
      const uint32_t j = d0 ? 0u : d1 ? 4u : d2 ? 8u : 12u;
      const uint32_t d = d0 ? d0 : d1 ? d1 : d2 ? d2 : d3;
      return k + j + ((uint32_t)__builtin_ctz(d) >> 3);
    }
    k += 16;
  }
  while (k < cap) {
    const uint32_t d = src.ld4(x + k) ^ src.ld4(y + k);
    if (d) {
      k += (uint32_t)__builtin_ctz(d) >> 3;
      break;
    }
    k += 4;
  }
  return k < cap ? k : cap;
}

// [base, base + span) in LDS, every other byte from HBM/L2 (positions below base included)
struct BytesTail {
  const uint32_t* w;
  uint64_t base, span;
  const uint8_t* in;
  __device__ __forceinline__ uint32_t ld4(uint64_t pos) const
  {
    const uint64_t d = pos - base;  // wraps below base (so d + 8 could wrap too: compare d itself)
    return d <= span - 8 ? lload4(w, (uint32_t)d) : gload4(in, pos);
  }
};

// exact common prefix of p and c (capped at room) if it reaches `need`, else 0
template <class Src>
__device__ __forceinline__ uint32_t prefix_if_at_least(const Src& src, uint64_t p, uint64_t c, uint32_t need, uint32_t room)
{
  if (need > room) return 0;
  if (need > 4) {
    if (src.ld4(p + need - 4) != src.ld4(c + need - 4)) return 0;
    for (uint32_t k = 4; k + 4 < need; k += 4)
      if (src.ld4(p + k) != src.ld4(c + k)) return 0;
  }
  uint32_t k = need > 4 ? need : 4;
  while (k < room) {
    const uint32_t x = src.ld4(p + k) ^ src.ld4(c + k);
    if (x) {
      k += (uint32_t)__builtin_ctz(x) >> 3;
      break;
    }
    k += 4;
  }
  return k < room ? k : room;
}

// prefix_if_at_least with a same-letter run [rLo, rHi) known around p (rHi capped at the block's last
// searchable byte): a candidate inside the run matches exactly up to the run's end, so no byte loop
// (O(1) instead of O(run) per candidate: greedy/lazy levels on long runs were quadratic)
template <class Src>
__device__ __forceinline__ uint32_t prefix_run(const Src& src, uint64_t p, uint64_t c, uint32_t need, uint32_t room,
                                               uint64_t rLo, uint64_t rHi)
{
  if (p >= rLo && p < rHi && c >= rLo) {
    const uint64_t e = rHi - p;
    const uint32_t pr = e < (uint64_t)room ? (uint32_t)e : room;
    return pr >= need ? pr : 0u;
  }
  return prefix_if_at_least(src, p, c, need, room);
}

// ================================================================================================
// k_find_sorted (pass 1): a wavefront takes 64 consecutive SORTED slots (lane = target).  A
// target's candidates are the slots below it in its hash group, nearest first, and each is checked
// on its first 12 bytes, which every lane keeps in registers for its own slot:
//   1. candidates inside the chunk come through a shift register (DPP wave_shr:1): after s shifts
//      lane l holds slot first + l - s, so every lane sees its own candidates in order;
//   2. candidates below the chunk can only belong to the group that started before it, so they
//      are the same for all of its lanes: 64 at a time into registers, one v_readlane each.
// -9 takes the maximum of (prefix << 17 | position): the reference's nearest-first strict-improvement
// walk (smallz4.h:190-252) ends on the nearest candidate of maximal prefix, so no order is needed;
// candidates whose 12 bytes all match are queued per wavefront and extended from the text 64 at a
// time.  Bounded chains keep the ordered walk (masked "first bestLen+1 bytes" test, strict
// improvement, step limit).  Prefixes are capped at kLongCap: a target reaching it keeps the marker
// kLongMatch and is finished by k_find (pass 2), which walks long repeats in text order.
// ================================================================================================
// bounded chains: prefixes >= this are finished by pass 2 (32 sent 4x more targets to k_find's second chain walk:
// -3/-6/-8 on configs[1] 10191/7742/9444 -> 11347/8925/11334 MB/s at 256, frames identical)
constexpr uint32_t kLongCap = 256;
constexpr uint32_t kLongCap9 = 256;  // -9: pass 1 extends exactly up to this
constexpr uint32_t kSatQ = 128;  // saturated-candidate queue per wavefront (flushed at 64)
// broadcast chunk list: >= slots / 64 + number of groups of >= 64 slots (64 Ki slots with the LDS
// window, 128 Ki otherwise)
template <bool kLds>
constexpr uint32_t kBigChunks = kLds ? 2048 : 4096;
constexpr uint32_t kLongMatch = 0xFFFFFFFFu;
constexpr uint32_t kBigGroup = 8192;  // -9: targets with more candidates go to k_find_big / k_find_long9
constexpr uint32_t kBigRun = 2048;    // the same for a run key (vvvv) in blocks k_find_big takes
constexpr uint32_t kBigRunL = 32;   // ... in blocks above 64 KiB (k_find_big's run table is exact and cheap)
constexpr uint32_t kLpfMin = 256;   // ... and for an LPF target (below)
constexpr uint64_t kLpfBlockMin = 65536;  // LPF targets go to k_find_big only in blocks larger than this
__device__ __forceinline__ bool run_key(uint32_t k) { return k == (k & 0xFFu) * 0x01010101u; }
// k_find_sorted's results leave in text order, tiles of kOutTile positions staged in LDS
constexpr uint32_t kOutTileBits = 14;
constexpr uint32_t kOutTile = 1u << kOutTileBits;    // 64 KiB of LDS as u32
constexpr uint32_t kOutTiles = 65536u / kOutTile;    // a segment has at most 65536 targets
constexpr uint32_t kOutLong = 0xFFFFu;               // packed length: long, finished by pass 2
constexpr uint32_t kOutUnsearched = 0xFFFEu;         // not a sorted target (shortcut interval)

// per-slot arrays written by the sort: u16 when the segment's window fits 16 bits (same predicate there)
__device__ __forceinline__ bool compact_small(const Segment& S) { return S.s1 - S.w0 <= 65536u; }
__device__ __forceinline__ uint32_t slot_pos(const void* base, bool small, uint32_t s)
{
  return small ? (uint32_t)reinterpret_cast<const uint16_t*>(base)[s] : reinterpret_cast<const uint32_t*>(base)[s];
}
__device__ __forceinline__ uint32_t slot_gs(const void* base, bool small, uint32_t E, uint32_t s)
{
  return small ? (uint32_t)reinterpret_cast<const uint16_t*>(base)[E + s] : reinterpret_cast<const uint32_t*>(base)[E + s];
}


template <bool kLds>
__device__ __forceinline__ void find_sorted_body(const uint8_t* __restrict__ in, const Segment* __restrict__ segs,
                                const Block* __restrict__ blocks, const Interval* __restrict__ ivAll,
                                const uint32_t* __restrict__ ivCount, uint2* compactAll, uint32_t maxChain,
                                uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist, uint64_t matchBase,
                                uint32_t* __restrict__ longBits, uint32_t* __restrict__ segLong, uint2* sortA,
                                uint32_t* rankOut)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t win[];
  __shared__ uint32_t s_next;
  __shared__ uint32_t s_long;
  __shared__ uint32_t s_tileCnt[kOutTiles];
  // -9: per wavefront, candidates whose first 12 bytes match (lane << 17 | position) and the best
  // exact key of each lane among them
  __shared__ uint32_t s_satQ[kFindThreads / 64][kSatQ];
  __shared__ uint32_t s_satBest[kFindThreads / 64][64];
  SZ4_D3(const uint64_t tEntry = __builtin_readcyclecounter();)
  // blocks above 64 KiB: consecutive segments of a block share 64 KiB of window and their text comes
  // from HBM/L2 -- give each XCD a contiguous run of segments (workgroups are dealt round-robin over
  // the 8 XCDs, MI355X_MICROARCH.md "Workgroup dispatch"), so the runs stay in that XCD's L2
  const uint32_t segIdx = blockIdx.x;
  const Segment S = segs[segIdx];
  const Block B = blocks[S.block];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t waveId = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
  uint32_t* satQ = s_satQ[waveId];
  uint32_t* satBest = s_satBest[waveId];
  const void* compact = compactAll + S.elemOff;
  // number of sorted slots: window positions minus shortcut-interval positions
  const uint32_t W = (uint32_t)(S.s1 - S.w0);
  uint32_t excluded = 0;
  {
    const uint32_t ids[2] = {B.prev, S.block};
    for (int t = 0; t < 2; t++) {
      if (ids[t] == kNoBlock) continue;
      const Interval* iv = ivAll + (uint64_t)ids[t] * kMaxIv;
      for (uint32_t j = 0; j < ivCount[ids[t]]; j++) {
        const uint64_t lo = iv[j].lo > S.w0 ? iv[j].lo : S.w0, hi = iv[j].hi < S.s1 ? iv[j].hi : S.s1;
        if (lo < hi) excluded += (uint32_t)(hi - lo);
      }
    }
  }
  const uint32_t E = W - excluded;
  const bool small = compact_small(S);
  {
    // the sort of this segment first, its shared memory in the (not yet loaded) window
    // buffer: the latency-bound sort of one workgroup overlaps the issue-bound search of the other
    // workgroup on the CU, and the sorted slots it writes are read back while L2-warm
    sort_segment(in, S, B, ivAll, ivCount, sortA, compactAll, *reinterpret_cast<SortLds*>(win));
    __syncthreads();
  }
  // results go out in text order through LDS (section at the end): during the search every target's
  // (position, result) is appended to the bucket of its 16 Ki-position tile, in the sort's scratch
  // (free now); s_tileCnt counts the entries per tile
  uint2* bucket = sortA + S.elemOff;
  const uint32_t nTargets = (uint32_t)(S.s1 - S.s0);
  if (tid < kOutTiles) s_tileCnt[tid] = 0;

  SZ4_D3(
  const uint64_t t0 = __builtin_readcyclecounter();
  uint64_t dB = 0, dL = 0, dBi = 0, dLi = 0;
  )
  if (tid == 0) {
    s_next = 0;
    // bounded chains: k_find (pass 2) visits a segment only if it has a long target or an unsearched
    // (shortcut-interval) one
    uint32_t sl = 0;
    if (maxChain < 65535u) {
      const Interval* iv = ivAll + (uint64_t)S.block * kMaxIv;
      for (uint32_t j = 0; j < ivCount[S.block]; j++)
        if (iv[j].lo < S.s1 && iv[j].hi > S.s0) sl = 1;
    }
    s_long = sl;
  }
  // kLds: the block's whole window in LDS; otherwise (1) every byte from HBM/L2, so that
  // the LDS holds only the sort and the result tiles and two workgroups share a CU -- the candidates'
  // first 12 bytes live in registers, so text reads are per chunk and per extension, not per
  // candidate -- or [w0, s1 + 64) in LDS and the rest from HBM
  typename std::conditional<kLds, Bytes<true>, Bytes<false>>::type src;
  if constexpr (kLds) {
    const uint64_t end = kLds ? B.end + 8 : (S.s1 + 64 < B.end + 8 ? S.s1 + 64 : B.end + 8);
    const uint32_t words = (uint32_t)((end - S.w0 + 3) / 4);
    for (uint32_t i = tid; i < words; i += kFindThreads) win[i] = gload4(in, S.w0 + 4ull * i);
    src.w = win;
    src.base = S.w0;
    if constexpr (!kLds) {
      src.lim = S.w0 + 4ull * words;
      src.in = in;
    }
  }
  if constexpr (!kLds) src.in = in;
  __syncthreads();

  uint64_t cut = B.cut;
  uint32_t cutHash = 0;
  if (cut != kNone) {
    const Interval* pv = ivAll + (uint64_t)B.prev * kMaxIv;
    if (in_iv(pv, ivCount[B.prev], cut)) cut = kNone;
    else cutHash = ref_hash(gload4(in, cut));
  }
  const uint64_t stopAbs = B.end - kTailLiterals;
  const bool unlimited = maxChain >= 65535u;
  // every distance inside a segment of at most 64 KiB is in the window, unless the lookback cut applies
  const bool needWin = (S.s1 - S.w0 > 65536u) || cut != kNone;
  const uint32_t nChunks = SZ4_SKIP_SEARCH ? 0u : (E + 63) / 64;

  while (true) {
    uint32_t item = 0;
    if (lane == 0) item = atomicAdd(&s_next, 1u);
    item = rdlane(item, 0);
    if (item >= nChunks) break;
    const uint32_t first = item * 64;
    const uint32_t count = E - first < 64 ? E - first : 64;
    const uint32_t slot = first + lane;
    // every lane's slot is a candidate for the lanes above it: its data is loaded even when the
    // slot itself is not a target (window-only positions)
    const bool inChunk = lane < count;
    const uint32_t myRel = inChunk ? slot_pos(compact, small, slot) : 0u;
    // the first block of candidates below the chunk (slots first - 1 - lane), loaded with the chunk's own
    // slots: a load issued later, before the in-chunk walk, made the compiler wait for it right there
    const uint32_t belowPre = slot_pos(compact, small, first > lane ? first - 1u - lane : 0u);
    const uint32_t gs = inChunk ? slot_gs(compact, small, E, slot) : slot;
    const uint64_t p = S.w0 + myRel;
    uint32_t me0, me1, me2;
    src.ld12(p, me0, me1, me2);
    if (!inChunk) me0 = me1 = me2 = 0u;
    const bool active = inChunk && p >= S.s0;  // window-only positions are candidates, not targets
    uint32_t room = 0, lbRel = 0, limit = 0;
    if (active) {
      room = (uint32_t)(stopAbs - p);
      uint64_t lb = p > kWindow ? p - kWindow : 0;
      if (cut != kNone && ref_hash(me0) == cutHash && cut > lb) lb = cut;
      lbRel = lb > S.w0 ? (uint32_t)(lb - S.w0) : 0u;
      const uint32_t cap = unlimited ? kLongCap9 : kLongCap;
      limit = room < cap ? room : cap;
    }
    uint32_t bestLen = 1, bestDist = 0, steps = unlimited ? 0xFFFFFFFFu : maxChain;
    // -9, a target with more than kBigGroup candidates (runs, periodic data): left to k_find_long9,
    // which walks in text order and prunes with the previous target's result
    // In blocks without a lookback (k_find_big takes those; shortcut intervals are fine) also run-key
    // targets and LPF targets go there; k_find_big takes exactly the targets marked here (distance 0)
    const bool lpfOk = B.cut == kNone && B.low == B.start;
    const uint64_t predLoF = S.w0 > B.low ? S.w0 : B.low;
    // LPF targets in blocks above 64 KiB only: a 64 KiB block's groups are small, and text gains nothing
    // there that would pay for k_find_big's pass over the segment
    const bool lpfBlock = B.end - B.start > kLpfBlockMin;
    // the LPF decision from the chunk itself: a target of the group that began before the chunk (more than
    // kLpfMin members below it) whose preceding byte at least 3/4 of that group's lanes in the chunk share
    // (their positions are the group's nearest to the target) -- no probes into the group below
    bool lpfLocal = false;
    if (unlimited && cut == kNone && lpfOk && lpfBlock) {
      const bool cand = active && slot - gs > kLpfMin && p > predLoF;
      const bool inGroup = inChunk && gs == rdlane(gs, 0) && gs < first;
      const uint32_t cls = cand ? (src.ld4(p - 1) & 0xFFu) : 0x100u;
      uint64_t peers = __ballot(inGroup && cand);
      const uint32_t nGroup = (uint32_t)__popcll(__ballot(inGroup));
#pragma unroll
      for (int b = 0; b < 9; b++) {
        const uint64_t m = __ballot((cls >> b) & 1u);
        peers &= ((cls >> b) & 1u) ? m : ~m;
      }
      lpfLocal = cand && inGroup && nGroup >= 16u && (uint32_t)__popcll(peers) * 4u >= 3u * nGroup;
    }
    const bool big = unlimited && cut == kNone && active &&
                     (slot - gs > kBigGroup ||
                      (lpfOk && ((run_key(me0) && slot - gs > (lpfBlock ? kBigRunL : kBigRun)) ||
                                 lpfLocal)));
    bool isLong = big, run = active && !big && bestLen < room && gs < slot;
    // a candidate improves iff its first need = bestLen + 1 bytes match: masks over bytes 4..11
    uint32_t m1 = 0, m2 = 0;
    // the candidate at cpos passed the mask test: its exact prefix (extended past 12 from the text)
    auto improve = [&](uint64_t cpos, uint32_t k1, uint32_t k2) {
      SZ4_D3(dBi++;)
      const uint32_t x1 = k1 ^ me1, x2 = k2 ^ me2;
      uint32_t kk = x1 ? 4u + ((uint32_t)__builtin_ctz(x1) >> 3) : x2 ? 8u + ((uint32_t)__builtin_ctz(x2) >> 3) : 12u;
      // 12 bytes equal and bestLen >= 12: it improves only if bytes bestLen - 3 .. bestLen match too (one
      // 4-byte test before the extension; inside a same-letter run every candidate passes the 12-byte mask)
      if (kk == 12u && bestLen >= 12u && src.ld4(p + bestLen - 3) != src.ld4(cpos + bestLen - 3)) kk = 0;
      if (kk == 12u) {
        bool open = true;
        while (open && kk < limit) {
          SZ4_D3(dLi++;)
          const uint32_t x = src.ld4(p + kk) ^ src.ld4(cpos + kk);
          if (x) {
            kk += (uint32_t)__builtin_ctz(x) >> 3;
            open = false;
          } else {
            kk += 4;
          }
        }
      }
      if (kk > limit) kk = limit;
      if (kk > bestLen) {
        bestLen = kk;
        bestDist = (uint32_t)(p - cpos);
        if (kk >= limit && limit < room) {
          isLong = true;
          run = false;
        } else if (--steps == 0 || bestLen >= room) {
          run = false;
        }
        const uint32_t nb = bestLen + 1;
        m1 = nb <= 4 ? 0u : nb >= 8 ? 0xFFFFFFFFu : (1u << (8 * (nb - 4))) - 1u;
        m2 = nb <= 8 ? 0u : nb >= 12 ? 0xFFFFFFFFu : (1u << (8 * (nb - 8))) - 1u;
      }
    };
    auto test = [&](uint32_t k0, uint32_t k1, uint32_t k2) -> uint32_t {
      return (k0 ^ me0) | ((k1 ^ me1) & m1) | ((k2 ^ me2) & m2);
    };
    if (unlimited) {
      // -9: the reference's nearest-first strict-improvement walk over every candidate ends on
      // the nearest candidate of maximal common prefix, so the result is the maximum of
      // key = prefix << 17 | position (window-relative), order-free and branch-free.  Prefixes are exact
      // up to 12 bytes; candidates reaching 12 are queued and
      // extended from the text in batches of 64 (one per lane).
      uint32_t bestKey = 3u << 17;  // length 3: no match yet
      uint32_t qn = 0;
      bool walk = false;  // phase 1: this lane still takes candidates inside the chunk
      satBest[lane] = 0;
      const uint32_t cap12 = limit < 12u ? limit : 12u;
      // keys and queue entries carry the candidate's window-relative POSITION (17 bits): inside one key
      // group positions ascend with the slots, so the maximum is the same, and no slot array is read to
      // turn a key into a distance (a global load in the flush would make the compiler wait on the
      // below-chunk prefetch at every step after it).  Shift-register step sh: the candidate is lane
      // (lane - sh)'s own position; broadcast candidate k: lane k's fRel
      auto spos = [&](uint32_t sh) -> uint32_t {
        return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - sh) & 63u) << 2), (int)myRel);
      };
      auto flush = [&]() {
        // lane t extends queue entry base + t: target = lane (e >> 17), candidate position e & 0x1FFFF
        for (uint32_t base = 0; base < qn; base += 64) {
        SZ4_D3(dLi += 1ull << 30;)  // flush rounds
        const uint32_t e = base + lane < qn ? satQ[base + lane] : 0u;
        const uint32_t tl = e >> 17, cs = e & 0x1FFFFu;
        const uint32_t tRel = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(tl << 2), (int)myRel);
        const uint32_t tLim = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(tl << 2), (int)limit);
        if (base + lane < qn) {
          const uint64_t tp = S.w0 + tRel, cp = S.w0 + cs;
          uint32_t kk = 12;
          bool open = true;
          // queued after the target's best so far (nearest first), so it only counts if longer: it
          // must match byte `cur` (one 4-byte test) before it is extended
          const uint32_t cur = satBest[tl] >> 17;
          if (cur >= 12u && (cur >= tLim || src.ld4(tp + cur - 3) != src.ld4(cp + cur - 3))) {
            open = false;
            kk = 0;
          }
          if constexpr (!kLds) {
            // text from HBM/L2: 16 bytes per step (one load latency per step, not per 4 bytes)
            if (open) kk = ext_prefix(src, tp, cp, 12u, tLim);
          } else {
            // the window in LDS: 4 bytes per step (the 16-byte step costs the LDS kernel spilled registers)
            while (open && kk < tLim) {
              SZ4_D3(dLi++;)  // lane-steps of the saturated extension
              const uint32_t x = src.ld4(tp + kk) ^ src.ld4(cp + kk);
              if (x) {
                kk += (uint32_t)__builtin_ctz(x) >> 3;
                open = false;
              } else {
                kk += 4;
              }
            }
            if (kk > tLim) kk = tLim;
          }
          if (kk) atomicMax(&satBest[tl], (kk << 17) | cs);
        }
        }
        qn = 0;
        // candidates arrive nearest first: a lane whose match reached its cap is finished
        if (satBest[lane] >= (limit << 17)) walk = run = false;
      };
      // lanes whose match can still grow past 12 bytes
      const uint64_t satOk = __ballot(limit > 12u);
      const uint32_t noGrow = limit > 12u ? 0u : 1u;
      // the same for a candidate every lane takes: its key, and x0 | x1 | x2 (0: all 12 bytes equal)
      auto score = [&](uint32_t cs, uint32_t k0, uint32_t k1, uint32_t k2) -> uint32_t {
        const uint32_t x0 = k0 ^ me0, x1 = k1 ^ me1, x2 = k2 ^ me2;
        const uint32_t z1 = (uint32_t)(__ffs(x1) - 1), z2 = (uint32_t)(__ffs(x2) - 1);  // ~0u when zero
        const uint32_t z = min(z1, 32u + min(z2, 32u));
        const uint32_t lcp = min(4u + (z >> 3), cap12);
        const uint32_t key = x0 == 0u ? (lcp << 17) | cs : 0u;
        bestKey = key > bestKey ? key : bestKey;
        return x0 | x1 | x2;
      };
      // score() for the lanes where `mine` holds (nonzero for the others)
      auto scoreIf = [&](bool mine, uint32_t cs, uint32_t k0, uint32_t k1, uint32_t k2) -> uint32_t {
        const uint32_t x0 = k0 ^ me0, x1 = k1 ^ me1, x2 = k2 ^ me2;
        const uint32_t z1 = (uint32_t)(__ffs(x1) - 1), z2 = (uint32_t)(__ffs(x2) - 1);
        const uint32_t z = min(z1, 32u + min(z2, 32u));
        const uint32_t lcp = min(4u + (z >> 3), cap12);
        const uint32_t key = (mine && x0 == 0u) ? (lcp << 17) | cs : 0u;
        bestKey = key > bestKey ? key : bestKey;
        return mine ? x0 | x1 | x2 : 1u;
      };
      // queue the lanes of `sat` (12 bytes equal, may grow past them) with candidate slot cs
      auto enqueue = [&](uint64_t sat, uint32_t cs) {
        if (sat) {
          const uint32_t at = qn + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(sat >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)sat, 0u));
          if ((sat >> lane) & 1ull) satQ[at] = (lane << 17) | cs;
          qn += (uint32_t)__builtin_popcountll(sat);
          if (qn >= 64) flush();
        }
      };
      // one candidate for this lane: slot cs with first 12 bytes k0..k2.  The common prefix is
      // 4 + (trailing zero bits of x2:x1) / 8; a candidate from another hash group never has x0 = 0
      auto visit = [&](bool mine, uint32_t cs, uint32_t k0, uint32_t k1, uint32_t k2) {
        const uint32_t x0 = k0 ^ me0, x1 = k1 ^ me1, x2 = k2 ^ me2;
        const uint32_t z1 = (uint32_t)(__ffs(x1) - 1), z2 = (uint32_t)(__ffs(x2) - 1);  // ~0u when zero
        const uint32_t z = min(z1, 32u + min(z2, 32u));
        const uint32_t lcp = min(4u + (z >> 3), cap12);
        const uint32_t key = (mine && x0 == 0u) ? (lcp << 17) | cs : 0u;
        bestKey = key > bestKey ? key : bestKey;
        const uint64_t sat = __ballot(mine && (x0 | x1 | x2) == 0u) & satOk;
        if (sat) {
          const uint32_t at = qn + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(sat >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)sat, 0u));
          if ((sat >> lane) & 1ull) satQ[at] = (lane << 17) | cs;
          qn += (uint32_t)__builtin_popcountll(sat);
          if (qn >= 64) flush();
        }
      };
      // candidates arrive nearest first (slots descend), so one can raise bestKey only with a longer
      // prefix: it must match the first bestLen + 1 bytes (all 12 once a lane holds 12 or its cap).
      // m1 / m2 mask bytes 4..11 of that need; the exact prefix is computed on a hit only
      // bestKey starts at length 3 (no match): the bytes to test past the first four are 8 (len - 3),
      // all of them once len reaches the cap -- as 63 mask bits: bit 63 of x2:x1 untested, which only
      // lets a rare candidate through the filter whose exact prefix then does not count
      auto setMasks = [&]() {
        const uint32_t len = bestKey >> 17;
        const uint32_t bits = len >= cap12 ? 63u : min(8u * len - 24u, 63u);
        const uint64_t mk = (1ull << bits) - 1ull;
        m1 = (uint32_t)mk;
        m2 = (uint32_t)(mk >> 32);
      };
      auto filt = [&](uint32_t k0, uint32_t k1, uint32_t k2) -> uint32_t {
        return (k0 ^ me0) | ((k1 ^ me1) & m1) | ((k2 ^ me2) & m2);
      };
      // the hit, from the candidate's words already xor-ed with the lane's own (x0 = 0: same first word)
      auto hitx = [&](bool mine, uint32_t cs, uint32_t x0, uint32_t x1, uint32_t x2) {
        SZ4_D3(dBi++;)  // hit branches (wave-level)
        // v_ffbl_b32 gives ~0u for 0, so min() takes x2 when x1 is 0 (no compare and select)
        const uint32_t z = min(ffbl(x1), 32u + min(ffbl(x2), 32u));
        const uint32_t lcp = min(4u + (z >> 3), cap12);
        const uint32_t key = (mine && x0 == 0u) ? (lcp << 17) | cs : 0u;
        bestKey = key > bestKey ? key : bestKey;
        setMasks();
        // queued: 12 bytes equal, and the match may grow past them (the lane's own bit of the ballot, not
        // the predicate again: one compare instead of a materialised bool compared twice)
        const uint64_t sat = __ballot(mine && (x0 | x1 | x2 | noGrow) == 0u);
        if (sat) {
          const uint32_t at = qn + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(sat >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)sat, 0u));
          if ((sat >> lane) & 1ull) satQ[at] = (lane << 17) | cs;
          qn += (uint32_t)__builtin_popcountll(sat);
          if (qn >= 64) flush();
        }
      };
      auto hit = [&](bool mine, uint32_t cs, uint32_t k0, uint32_t k1, uint32_t k2) {
        hitx(mine, cs, k0 ^ me0, k1 ^ me1, k2 ^ me2);
      };
      setMasks();
      // 1. inside the chunk: shift register (after s shifts lane l holds slot first + l - s)
      {
        // lane l has slot - max(gs, first) candidates inside the chunk (lanes below it), so the walk is a
        // uniform trip count (the longest of them) with a per-lane bound -- no per-step walk flags.  With a
        // window test the bound starts at the lowest of those lanes inside the window (positions ascend
        // with the lane inside a group: a binary search over the chunk), and a lane cut by the window has
        // nothing left below the chunk
        const int32_t lo1 = (int32_t)(gs > first ? gs : first);
        uint32_t jLo = run && (int32_t)slot > lo1 ? (uint32_t)(lo1 - (int32_t)first) : lane;
        if (needWin) {
          uint32_t a = jLo, b = lane;  // the first lane j in [a, b) with myRel(j) >= lbRel, else b
#pragma unroll
          for (int it = 0; it < 6; it++) {
            const uint32_t mid = (a + b) >> 1;
            const uint32_t rj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mid << 2), (int)myRel);
            const bool go = a < b;
            if (go && rj < lbRel) a = mid + 1u;
            else if (go) b = mid;
          }
          if (a > jLo) run = false;
          jLo = a;
        }
        const uint32_t myCnt = lane - jLo;
        const uint32_t rm = row_max(myCnt);
        const uint32_t trips = SZ4_SKIP_SHIFT ? 0u : max(max(rdlane(rm, 0), rdlane(rm, 16)), max(rdlane(rm, 32), rdlane(rm, 48)));
        uint32_t r0 = me0, r1 = me1, r2 = me2;
        uint32_t s = 1;
        // wave shift right by one, zero into lane 0 (bound_ctrl: no old value to set up)
        auto shr1 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kWaveShr1, 0xF, 0xF, true); };
        if (!needWin) {
          // a source lane below the target's group holds another key (x0 != 0), so only the lanes that do
          // not run need a mask, folded into the first word's test
          const uint32_t dead = run ? 0u : ~0u;
          for (; s <= trips; s++) {
            SZ4_D3(dL++;)
            r0 = shr1(r0);
            r1 = shr1(r1);
            r2 = shr1(r2);
            const uint32_t y = ((r0 ^ me0) | dead) | ((r1 ^ me1) & m1) | ((r2 ^ me2) & m2);
            if (__ballot(y == 0u)) hit(s <= myCnt, spos(s), r0, r1, r2);
          }
        } else {
          for (; s <= trips; s++) {
            SZ4_D3(dL++;)
            r0 = shr1(r0);
            r1 = shr1(r1);
            r2 = shr1(r2);
            const uint32_t dead = s <= myCnt ? 0u : ~0u;
            const uint32_t y = ((r0 ^ me0) | dead) | ((r1 ^ me1) & m1) | ((r2 ^ me2) & m2);
            if (__ballot(y == 0u)) hit(s <= myCnt, spos(s), r0, r1, r2);
          }
        }
        for (; s <= trips; s++) {
          SZ4_D3(dL++;)
          r0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r0, kWaveShr1, 0xF, 0xF, false);
          r1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r1, kWaveShr1, 0xF, 0xF, false);
          r2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r2, kWaveShr1, 0xF, 0xF, false);
          visit(s <= myCnt, spos(s), r0, r1, r2);
        }
        run = run && (int32_t)gs < (int32_t)first;
      }
      // 2. below the chunk: the group that started before it, one uniform candidate per step
      if (!SZ4_SKIP_BCAST && __ballot(run)) {
        const int32_t gsB = (int32_t)rdlane(gs, 0);
        // a chunk whose 64 targets share their first word (inside one wide key group)
        const uint32_t me0u = rdlane(me0, 0);
        // (the LDS-window kernel only: in k_find_sorted_hbm the loop costs the registers of a second workgroup per CU)
        const bool sameMe0 = 1 && kLds && __ballot(me0 == me0u) == ~0ull;
        int32_t cBase = (int32_t)first - 1;
        uint32_t nextBlk = cBase - (int32_t)lane >= gsB ? belowPre : 0u;
        while (cBase >= gsB && __ballot(run)) {
          uint32_t fRel;
          asm volatile("v_mov_b32 %0, %1" : "=v"(fRel) : "v"(nextBlk));
          const int32_t cn = cBase - 64 - (int32_t)lane;
          nextBlk = cn >= gsB ? slot_pos(compact, small, (uint32_t)cn) : 0u;
          const uint64_t fp = S.w0 + fRel;
          uint32_t f0, f1, f2;
          src.ld12(fp, f0, f1, f2);
          const int32_t n = cBase - gsB + 1 < 64 ? cBase - gsB + 1 : 64;
          SZ4_D3(dLi += 1ull << 46;)  // broadcast blocks
          if (needWin) {
            // the block's candidates inside this lane's window: positions descend with k, so they are
            // the first kc (a binary search over the block); a lane whose window ends here is done
            uint32_t a = 0, b = (uint32_t)n;  // up to 64 candidates: 7 halvings
#pragma unroll
            for (int it = 0; it < 7; it++) {
              const uint32_t mid = (a + b) >> 1;
              const uint32_t fk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mid << 2), (int)fRel);
              const bool go = a < b;
              if (go && fk >= lbRel) a = mid + 1u;
              else if (go) b = mid;
            }
            const uint32_t kc = run ? a : 0u;
            int32_t k = 0;
            // 16 candidates per register, every row a copy (lane l: candidate q0 + (l & 15)); step K takes
            // candidate q0 + K to every lane by DPP row_newbcast:K folded into the xor with the lane's word
            for (int32_t q0 = 0; q0 < n; q0 += 16) {
              const int src = (int)((uint32_t)(q0 + (int32_t)(lane & 15u)) << 2);
              const uint32_t g0 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)f0);
              const uint32_t g1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)f1);
              const uint32_t g2 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)f2);
              const int32_t cnt = n - q0 < 16 ? n - q0 : 16;
              const uint32_t kcRel = kc > (uint32_t)q0 ? kc - (uint32_t)q0 : 0u;
#define SZ4_BSTEP_W(K)                                                                                          \
              if ((K) < cnt) {                                                                                  \
                const uint32_t x0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g0, 0x150 + (K), 0xF, 0xF, true) ^ me0; \
                const uint32_t x1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g1, 0x150 + (K), 0xF, 0xF, true) ^ me1; \
                const uint32_t x2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g2, 0x150 + (K), 0xF, 0xF, true) ^ me2; \
                if (__ballot((K) < kcRel && (x0 | (x1 & m1) | (x2 & m2)) == 0u))                                 \
                  hitx((K) < kcRel, rdlane(fRel, (uint32_t)(q0 + (K))), x0, x1, x2);                                    \
              }
              SZ4_BSTEP_W(0) SZ4_BSTEP_W(1) SZ4_BSTEP_W(2) SZ4_BSTEP_W(3) SZ4_BSTEP_W(4) SZ4_BSTEP_W(5)
              SZ4_BSTEP_W(6) SZ4_BSTEP_W(7) SZ4_BSTEP_W(8) SZ4_BSTEP_W(9) SZ4_BSTEP_W(10) SZ4_BSTEP_W(11)
              SZ4_BSTEP_W(12) SZ4_BSTEP_W(13) SZ4_BSTEP_W(14) SZ4_BSTEP_W(15)
#undef SZ4_BSTEP_W
            }
            k = n;
            for (; k + 1 < n; k += 2) {
              const uint32_t xa = scoreIf((uint32_t)k < kc, rdlane(fRel, (uint32_t)k), rdlane(f0, k), rdlane(f1, k), rdlane(f2, k));
              const uint32_t xb = scoreIf((uint32_t)k + 1u < kc, rdlane(fRel, (uint32_t)k + 1u), rdlane(f0, k + 1),
                                          rdlane(f1, k + 1), rdlane(f2, k + 1));
              if (__ballot(min(xa, xb) == 0u) & satOk) {
                enqueue(__ballot(xa == 0u) & satOk, rdlane(fRel, (uint32_t)k));
                enqueue(__ballot(xb == 0u) & satOk, rdlane(fRel, (uint32_t)k + 1u));
              }
            }
            if (k < n)
              visit((uint32_t)k < kc, rdlane(fRel, (uint32_t)k), rdlane(f0, k), rdlane(f1, k), rdlane(f2, k));
            if (kc < (uint32_t)n) run = false;
          } else {
            // no window test: every lane may take the candidate (only the group's lanes can match; a
            // lane finished at its cap cannot move: its queued candidates never beat the one it has)
            int32_t k = 0;
            {
              // 16 candidates per register, every row a copy (lane l: candidate q0 + (l & 15)); step K takes
              // candidate q0 + K to every lane by DPP row_newbcast:K folded into the xor with the lane's word.
              // A chunk whose 64 targets share their first word tests only the candidates with that word
              // (the others cannot pass): one scalar bit test per candidate, x0 = 0
              const bool same = 1 && kLds && sameMe0;
              const uint64_t todo64 = same ? __ballot((int32_t)lane < n && f0 == me0u) : 0ull;
              for (int32_t q0 = 0; q0 < n; q0 += 16) {
                const uint32_t todo = (uint32_t)(todo64 >> q0) & 0xFFFFu;
                if (same && !todo) continue;
                const int src = (int)((uint32_t)(q0 + (int32_t)(lane & 15u)) << 2);
                const uint32_t g1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)f1);
                const uint32_t g2 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)f2);
                const int32_t cnt = n - q0 < 16 ? n - q0 : 16;
                if (same) {
#define SZ4_BSTEP_S(K)                                                                                          \
                  if ((todo >> (K)) & 1u) {                                                                     \
                    const uint32_t x1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g1, 0x150 + (K), 0xF, 0xF, true) ^ me1; \
                    const uint32_t x2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g2, 0x150 + (K), 0xF, 0xF, true) ^ me2; \
                    if (__ballot(((x1 & m1) | (x2 & m2)) == 0u)) hitx(true, rdlane(fRel, (uint32_t)(q0 + (K))), 0u, x1, x2); \
                  }
                  SZ4_BSTEP_S(0) SZ4_BSTEP_S(1) SZ4_BSTEP_S(2) SZ4_BSTEP_S(3) SZ4_BSTEP_S(4) SZ4_BSTEP_S(5)
                  SZ4_BSTEP_S(6) SZ4_BSTEP_S(7) SZ4_BSTEP_S(8) SZ4_BSTEP_S(9) SZ4_BSTEP_S(10) SZ4_BSTEP_S(11)
                  SZ4_BSTEP_S(12) SZ4_BSTEP_S(13) SZ4_BSTEP_S(14) SZ4_BSTEP_S(15)
#undef SZ4_BSTEP_S
                } else {
                  const uint32_t g0 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)f0);
#define SZ4_BSTEP_N(K)                                                                                          \
                  if ((K) < cnt) {                                                                              \
                    const uint32_t x0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g0, 0x150 + (K), 0xF, 0xF, true) ^ me0; \
                    const uint32_t x1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g1, 0x150 + (K), 0xF, 0xF, true) ^ me1; \
                    const uint32_t x2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g2, 0x150 + (K), 0xF, 0xF, true) ^ me2; \
                    if (__ballot((x0 | (x1 & m1) | (x2 & m2)) == 0u)) hitx(true, rdlane(fRel, (uint32_t)(q0 + (K))), x0, x1, x2); \
                  }
                  SZ4_BSTEP_N(0) SZ4_BSTEP_N(1) SZ4_BSTEP_N(2) SZ4_BSTEP_N(3) SZ4_BSTEP_N(4) SZ4_BSTEP_N(5)
                  SZ4_BSTEP_N(6) SZ4_BSTEP_N(7) SZ4_BSTEP_N(8) SZ4_BSTEP_N(9) SZ4_BSTEP_N(10) SZ4_BSTEP_N(11)
                  SZ4_BSTEP_N(12) SZ4_BSTEP_N(13) SZ4_BSTEP_N(14) SZ4_BSTEP_N(15)
#undef SZ4_BSTEP_N
                }
              }
              k = n;
            }
            if (kLds && sameMe0 && k < n) {
              // every lane holds the same first word: only the block's candidates with that word can pass,
              // visited nearest first by bit scan, two readlanes each
              uint64_t todo = __ballot((int32_t)lane < n && f0 == me0u);
              while (todo) {
                const uint32_t kk = (uint32_t)__builtin_ctzll(todo);
                todo &= todo - 1ull;
                SZ4_D3(dB++;)
                const uint32_t k1 = rdlane(f1, kk), k2 = rdlane(f2, kk);
                if (__ballot((((k1 ^ me1) & m1) | ((k2 ^ me2) & m2)) == 0u)) hit(true, rdlane(fRel, kk), me0u, k1, k2);
              }
              k = n;
            }
            for (; k < n; k++) {
              SZ4_D3(dB++;)
              const uint32_t k0 = rdlane(f0, k), k1 = rdlane(f1, k), k2 = rdlane(f2, k);
              if (__ballot(filt(k0, k1, k2) == 0u)) hit(true, rdlane(fRel, (uint32_t)k), k0, k1, k2);
            }
            for (; k + 1 < n; k += 2) {
              SZ4_D3(dB += 2;)
              const uint32_t xa = score(rdlane(fRel, (uint32_t)k), rdlane(f0, k), rdlane(f1, k), rdlane(f2, k));
              const uint32_t xb = score(rdlane(fRel, (uint32_t)k + 1u), rdlane(f0, k + 1), rdlane(f1, k + 1), rdlane(f2, k + 1));
              if (__ballot(min(xa, xb) == 0u) & satOk) {
                enqueue(__ballot(xa == 0u) & satOk, rdlane(fRel, (uint32_t)k));
                enqueue(__ballot(xb == 0u) & satOk, rdlane(fRel, (uint32_t)k + 1u));
              }
            }
            for (; k < n; k++) {
              SZ4_D3(dB++;)
              visit(true, rdlane(fRel, (uint32_t)k), rdlane(f0, k), rdlane(f1, k), rdlane(f2, k));
            }
          }
          // settle queued candidates every 256: a lane whose match reached its cap stops there
          if (qn && ((uint32_t)(first - 1 - cBase) & 0xC0u) == 0xC0u) flush();
          cBase -= 64;
        }
      }
      if (qn) flush();
      const uint32_t sb = satBest[lane];
      bestKey = sb > bestKey ? sb : bestKey;
      const uint32_t bl = bestKey >> 17;
      // a big target stays handed on: the below-chunk loop lets every lane take its candidates (no
      // window test), so it may hold a partial maximum here
      if (bl >= 4u && !big) {
        bestLen = bl;
        bestDist = (uint32_t)(p - (S.w0 + (bestKey & 0x1FFFFu)));
        isLong = bl >= limit && limit < room;
      }
    } else {
    // 1. candidates inside the chunk, nearest first: a shift register -- after s shifts lane l holds
      //    slot first + l - s.  As at -9: a uniform trip count (the longest lane's) with a per-lane bound,
      //    the lane's window start found by a binary search over the chunk (positions ascend with the lane
      //    inside a group); a lane cut by its window has nothing left below the chunk.  Candidates stay in
      //    order per lane, so the step count (strict improvements) is the reference's.
      {
        const int32_t lo1 = (int32_t)(gs > first ? gs : first);
        uint32_t jLo = run && (int32_t)slot > lo1 ? (uint32_t)(lo1 - (int32_t)first) : lane;
        bool cutHere = false;
        if (needWin) {
          uint32_t a = jLo, b = lane;  // the first lane j in [a, b) with myRel(j) >= lbRel, else b
#pragma unroll
          for (int it = 0; it < 6; it++) {
            const uint32_t mid = (a + b) >> 1;
            const uint32_t rj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mid << 2), (int)myRel);
            const bool go = a < b;
            if (go && rj < lbRel) a = mid + 1u;
            else if (go) b = mid;
          }
          cutHere = a > jLo;
          jLo = a;
        }
        const uint32_t myCnt = lane - jLo;
        const uint32_t rm = row_max(myCnt);
        const uint32_t trips = max(max(rdlane(rm, 0), rdlane(rm, 16)), max(rdlane(rm, 32), rdlane(rm, 48)));
        uint32_t r0 = me0, r1 = me1, r2 = me2;
        auto shr1 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kWaveShr1, 0xF, 0xF, true); };
        for (uint32_t sft = 1; sft <= trips; sft++) {
          SZ4_D3(dL++;)
          r0 = shr1(r0);
          r1 = shr1(r1);
          r2 = shr1(r2);
          const bool h = run && sft <= myCnt && test(r0, r1, r2) == 0u;
          if (__ballot(h)) {
            const uint32_t cRel = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - sft) & 63u) << 2), (int)myRel);
            if (h) improve(S.w0 + cRel, r1, r2);
          }
          // lanes whose step count ran out stop early: leave when none is left with candidates
          if ((sft & 7u) == 0u && !__ballot(run && sft < myCnt)) break;
        }
        if (cutHere) run = false;
        // a lane whose group starts inside the chunk has seen all its candidates
        run = run && (int32_t)gs < (int32_t)first;
      }
      // 2. below the chunk: only the group that started before it (lanes 0..) is left, and every
      //    one of its lanes takes the same candidate -- 64 at a time (lane k: slot cBase - k, its
      //    position prefetched one block ahead, its first 12 bytes from the window), four per test
      if (__ballot(run)) {
        const int32_t gsB = (int32_t)rdlane(gs, 0);
        int32_t cBase = (int32_t)first - 1;
        uint32_t nextBlk = cBase - (int32_t)lane >= gsB ? belowPre : 0u;
        while (cBase >= gsB && __ballot(run)) {
          uint32_t fRel;
          asm volatile("v_mov_b32 %0, %1" : "=v"(fRel) : "v"(nextBlk));
          const int32_t cn = cBase - 64 - (int32_t)lane;
          nextBlk = cn >= gsB ? slot_pos(compact, small, (uint32_t)cn) : 0u;
          const uint64_t fp = S.w0 + fRel;
          uint32_t f0, f1, f2;
          src.ld12(fp, f0, f1, f2);
          const int32_t n = cBase - gsB + 1 < 64 ? cBase - gsB + 1 : 64;
          int32_t k = 0;
          {
            // as at -9: 16 candidates per register, every row a copy, candidate q0 + K to every lane by DPP
            // row_newbcast:K folded into the xor -- in order, nearest first, as the step count needs; with a
            // window test, a lane takes the first kc candidates of the block (positions descend with k)
            uint32_t kc = (uint32_t)n;
            if (needWin) {
              uint32_t a = 0, b = (uint32_t)n;
#pragma unroll
              for (int it = 0; it < 7; it++) {
                const uint32_t mid = (a + b) >> 1;
                const uint32_t fk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mid << 2), (int)fRel);
                const bool go = a < b;
                if (go && fk >= lbRel) a = mid + 1u;
                else if (go) b = mid;
              }
              kc = a;
            }
            for (int32_t q0 = 0; q0 < n && __ballot(run); q0 += 16) {
              const int srcl = (int)((uint32_t)(q0 + (int32_t)(lane & 15u)) << 2);
              const uint32_t g0 = (uint32_t)__builtin_amdgcn_ds_bpermute(srcl, (int)f0);
              const uint32_t g1 = (uint32_t)__builtin_amdgcn_ds_bpermute(srcl, (int)f1);
              const uint32_t g2 = (uint32_t)__builtin_amdgcn_ds_bpermute(srcl, (int)f2);
              const int32_t cnt = n - q0 < 16 ? n - q0 : 16;
              const uint32_t kcRel = kc > (uint32_t)q0 ? kc - (uint32_t)q0 : 0u;
#define SZ4_BSTEP_B(K)                                                                                          \
              if ((K) < cnt) {                                                                                  \
                const uint32_t x0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g0, 0x150 + (K), 0xF, 0xF, true) ^ me0; \
                const uint32_t x1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g1, 0x150 + (K), 0xF, 0xF, true) ^ me1; \
                const uint32_t x2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g2, 0x150 + (K), 0xF, 0xF, true) ^ me2; \
                const bool h = run && (K) < kcRel && (x0 | (x1 & m1) | (x2 & m2)) == 0u;                          \
                if (__ballot(h) && h) improve(S.w0 + rdlane(fRel, (uint32_t)(q0 + (K))), x1 ^ me1, x2 ^ me2);    \
              }
              SZ4_BSTEP_B(0) SZ4_BSTEP_B(1) SZ4_BSTEP_B(2) SZ4_BSTEP_B(3) SZ4_BSTEP_B(4) SZ4_BSTEP_B(5)
              SZ4_BSTEP_B(6) SZ4_BSTEP_B(7) SZ4_BSTEP_B(8) SZ4_BSTEP_B(9) SZ4_BSTEP_B(10) SZ4_BSTEP_B(11)
              SZ4_BSTEP_B(12) SZ4_BSTEP_B(13) SZ4_BSTEP_B(14) SZ4_BSTEP_B(15)
#undef SZ4_BSTEP_B
            }
            if (kc < (uint32_t)n) run = false;
            k = n;
          }
          if (!needWin) {
            for (; k + 4 <= n; k += 4) {
              SZ4_D3(dB += 4;)
              uint32_t a0[4], a1[4], a2[4], t[4];
#pragma unroll
              for (int u = 0; u < 4; u++) {
                a0[u] = rdlane(f0, k + u);
                a1[u] = rdlane(f1, k + u);
                a2[u] = rdlane(f2, k + u);
                t[u] = test(a0[u], a1[u], a2[u]);
              }
              if (__ballot(run && min(min(t[0], t[1]), min(t[2], t[3])) == 0u)) {
#pragma unroll
                for (int u = 0; u < 4; u++)
                  if (run && test(a0[u], a1[u], a2[u]) == 0u) improve(S.w0 + rdlane(fRel, k + u), a1[u], a2[u]);
              }
              if (!__ballot(run)) break;
            }
          }
          for (; k < n && __ballot(run); k++) {
            SZ4_D3(dB++;)
            const uint32_t k0 = rdlane(f0, k), k1 = rdlane(f1, k), k2 = rdlane(f2, k), crel = rdlane(fRel, k);
            if (needWin && run && crel < lbRel) run = false;
            if (run && test(k0, k1, k2) == 0u) improve(S.w0 + crel, k1, k2);
          }
          cBase -= 64;
        }
      }
    }
    // the result, packed: length (or kOutLong: pass 2 finishes it) << 16 | distance (for a long
    // target pass 2's seed: the nearest candidate at the cap), appended to its tile's bucket
    {
      const uint32_t rel = active ? (uint32_t)(p - S.s0) : 0u;
      // a run-key target whose match reached the cap goes to k_find_big as well (blocks above 64 KiB):
      // its run table gives the exact length, where pass 2 would compare the whole run per candidate
      const bool lateBig = unlimited && cut == kNone && active && isLong && !big && lpfOk && lpfBlock && run_key(me0);
      const uint32_t packed = ((isLong ? kOutLong : (bestDist ? bestLen : 0u)) << 16) | (big || lateBig ? 0u : (bestDist & 0xFFFFu));
#pragma unroll
      for (uint32_t k = 0; k < kOutTiles; k++) {
        const uint64_t m = __ballot(active && (rel >> kOutTileBits) == k);
        if (m) {
          uint32_t at = 0;
          if (lane == (uint32_t)__builtin_ctzll(m)) at = atomicAdd(&s_tileCnt[k], (uint32_t)__popcll(m));
          at = (uint32_t)__builtin_amdgcn_readlane((int)at, (int)__builtin_ctzll(m));
          if ((m >> lane) & 1ull) {
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            bucket[(k << kOutTileBits) + at + below] = make_uint2(rel, packed);
          }
        }
      }
      // pass 2 finds a long target's candidates from its slot
      if (active && isLong) rankOut[S.rankOff + rel] = slot;
    }
    if (__ballot(active && isLong) && lane == 0) s_long = 1;
  }
  SZ4_D3(const uint64_t tSearch = __builtin_readcyclecounter();)
  __syncthreads();
  if (tid == 0) segLong[segIdx] = s_long;

  // results in text order: tile by tile, the bucket is scattered into LDS (the window is free now)
  // and written out coalesced -- mlen u32, mdist u16 and pass 2's marker bits.  Targets no bucket
  // holds (shortcut intervals, never sorted) stay unresolved for pass 2.
  uint32_t* otile = win;
  for (uint32_t k = 0; k * kOutTile < nTargets; k++) {
    const uint32_t t0 = k * kOutTile, tn = nTargets - t0 < kOutTile ? nTargets - t0 : kOutTile;
    for (uint32_t i = tid; i < tn; i += kFindThreads) otile[i] = kOutUnsearched << 16;
    __syncthreads();
    const uint32_t cnt = s_tileCnt[k];
    const uint2* bk = bucket + t0;
    for (uint32_t i = tid; i < cnt; i += kFindThreads) {
      const uint2 v = bk[i];
      otile[v.x - t0] = v.y;
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < tn; i0 += kFindThreads) {
      const uint32_t i = i0 + tid;
      const bool in = i < tn;
      const uint32_t v = in ? otile[i] : 0u;
      const uint32_t len = v >> 16;
      const uint64_t idx = S.s0 + t0 + i - matchBase;
      if (in) {
        mlen[idx] = len >= kOutUnsearched ? kLongMatch : len;
        mdist[idx] = (uint16_t)(v & 0xFFFFu);
      }
      // marker bits of long pass-1 targets (-9): 64 consecutive positions per wave
      const uint64_t m = __ballot(in && unlimited && len == kOutLong);
      if (m && lane == 0) {
        const uint64_t b0 = S.s0 + t0 + (i0 + (tid & ~63u)) - matchBase;
        const uint32_t sh = (uint32_t)(b0 & 31);
        uint32_t* w = longBits + (b0 >> 5);
        const uint64_t lo = m << sh;  // bits b0 .. b0 + 63 over words w[0..2]
        if ((uint32_t)lo) atomicOr(&w[0], (uint32_t)lo);
        if ((uint32_t)(lo >> 32)) atomicOr(&w[1], (uint32_t)(lo >> 32));
        if (sh && (uint32_t)(m >> (64 - sh))) atomicOr(&w[2], (uint32_t)(m >> (64 - sh)));
      }
    }
    __syncthreads();
  }
  SZ4_D3(
  const uint64_t t2 = __builtin_readcyclecounter();
  const uint64_t w = (uint64_t)blockIdx.x * (kFindThreads / 64) + (tid >> 6);
  {
    uint64_t sLo = 0;
    for (int l = 0; l < 64; l++) sLo += (uint64_t)__shfl((long long)(dLi & 0x3FFFFFFFull), l);
    dLi = (dLi & ~0x3FFFFFFFull) | sLo;
  }
  if (lane == 0 && w * 8 + 8 <= (1u << 20)) {
    uint64_t* d = sz4_diag + w * 8;
    d[0] = t0; d[1] = t2; d[2] = dB; d[3] = dL; d[4] = dBi; d[5] = dLi; d[6] = tEntry; d[7] = tSearch;
  }
  )
}

// two 16-wave workgroups per CU need 8 waves per SIMD: .sgpr_count <= 80 (800 SGPRs per SIMD, a wave takes
// ceil(sgpr / 16) * 16 + 16; 82..96 admits 7 and so only one such workgroup).  Without the whole window
// in LDS a workgroup stages up to 128 KiB and runs alone on its CU: there the spills would only cost
__global__ __launch_bounds__(kFindThreads, 2) __attribute__((amdgpu_num_sgpr(80))) void k_find_sorted_lds(const uint8_t* __restrict__ in, const Segment* __restrict__ segs,
                                const Block* __restrict__ blocks, const Interval* __restrict__ ivAll,
                                const uint32_t* __restrict__ ivCount, uint2* compactAll, uint32_t maxChain,
                                uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist, uint64_t matchBase,
                                uint32_t* __restrict__ longBits, uint32_t* __restrict__ segLong, uint2* sortA,
                                uint32_t* rankOut)
{
  find_sorted_body<true>(in, segs, blocks, ivAll, ivCount, compactAll, maxChain, mlen, mdist, matchBase, longBits, segLong, sortA, rankOut);
}
__global__ __launch_bounds__(kFindThreads) __attribute__((amdgpu_waves_per_eu(8), amdgpu_num_sgpr(80))) void k_find_sorted_hbm(const uint8_t* __restrict__ in, const Segment* __restrict__ segs,
                                const Block* __restrict__ blocks, const Interval* __restrict__ ivAll,
                                const uint32_t* __restrict__ ivCount, uint2* compactAll, uint32_t maxChain,
                                uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist, uint64_t matchBase,
                                uint32_t* __restrict__ longBits, uint32_t* __restrict__ segLong, uint2* sortA,
                                uint32_t* rankOut)
{
  find_sorted_body<false>(in, segs, blocks, ivAll, ivCount, compactAll, maxChain, mlen, mdist, matchBase, longBits, segLong, sortA, rankOut);
}

// (1: two workgroups per CU when the window fits LDS -- <= 64 VGPRs, <= 80 SGPRs)
template <bool kLds>
__global__ __launch_bounds__(kFindThreads) __attribute__((amdgpu_waves_per_eu(8), amdgpu_num_sgpr(80))) void k_find(const uint8_t* __restrict__ in, const Segment* __restrict__ segs,
                                                       const Block* __restrict__ blocks, const Interval* __restrict__ ivAll,
                                                       const uint32_t* __restrict__ ivCount, const uint2* __restrict__ compactAll,
                                                       const uint32_t* __restrict__ rankAll, uint32_t maxChain,
                                                       uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist,
                                                       uint64_t matchBase, uint32_t* __restrict__ longFlag,
                                                       const uint32_t* __restrict__ segLong)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t win[];
  __shared__ uint32_t s_next;
  if (!segLong[blockIdx.x]) return;  // pass 1 left nothing here (uniform)
  const Segment S = segs[blockIdx.x];
  const Block B = blocks[S.block];
  const uint32_t tid = threadIdx.x, lane = tid & 63, row = lane >> 4, li = lane & 15;
  const void* compact = compactAll + S.elemOff;
  const uint32_t* rank = rankAll + S.rankOff;
  const Interval* iv = ivAll + (uint64_t)S.block * kMaxIv;
  const uint32_t niv = ivCount[S.block];
  // number of sorted slots (window minus shortcut-interval positions), as in the sort
  uint32_t E = (uint32_t)(S.s1 - S.w0);
  {
    const uint32_t ids[2] = {B.prev, S.block};
    for (int t = 0; t < 2; t++) {
      if (ids[t] == kNoBlock) continue;
      const Interval* ivb = ivAll + (uint64_t)ids[t] * kMaxIv;
      for (uint32_t j = 0; j < ivCount[ids[t]]; j++) {
        const uint64_t lo = ivb[j].lo > S.w0 ? ivb[j].lo : S.w0, hi = ivb[j].hi < S.s1 ? ivb[j].hi : S.s1;
        if (lo < hi) E -= (uint32_t)(hi - lo);
      }
    }
  }
  const bool small = compact_small(S);

  if (tid == 0) s_next = 0;
  Bytes<kLds> src;
  if constexpr (kLds) {
    const uint32_t words = (uint32_t)((B.end - S.w0 + 8 + 3) / 4);
    for (uint32_t i = tid; i < words; i += kFindThreads) win[i] = gload4(in, S.w0 + 4ull * i);
    src.w = win;
    src.base = S.w0;
  } else {
    src.in = in;
  }
  __syncthreads();

  // chain cut (lookback re-insertion of B.cut, smallz4.h:614-624): applies only if the previous
  // block inserted that position (it is not inside one of its shortcut intervals)
  uint64_t cut = B.cut;
  uint32_t cutHash = 0;
  if (cut != kNone) {
    const Interval* pv = ivAll + (uint64_t)B.prev * kMaxIv;
    if (in_iv(pv, ivCount[B.prev], cut)) cut = kNone;
    else cutHash = ref_hash(gload4(in, cut));
  }
  const Interval* pvIv = B.prev != kNoBlock ? ivAll + (uint64_t)B.prev * kMaxIv : iv;
  const uint32_t pvN = B.prev != kNoBlock ? ivCount[B.prev] : 0u;
  const uint64_t stopAbs = B.end - kTailLiterals;
  const bool unlimited = maxChain >= 65535u;
  const uint32_t nTargets = (uint32_t)(S.s1 - S.s0);
  const uint32_t rowBase = row << 4;

  while (true) {
    uint32_t chunkIdx = 0;
    if (lane == 0) chunkIdx = atomicAdd(&s_next, 1u);
    chunkIdx = rdlane(chunkIdx, 0);
    const uint32_t first = chunkIdx * 64;
    if (first >= nTargets) break;
    const uint32_t cnt = nTargets - first < 64 ? nTargets - first : 64;
    // pass 2: only targets pass 1 left marked (long matches, shortcut intervals) are searched here
    const uint64_t myIdx = S.s0 + first + lane - matchBase;
    const uint32_t pass1Len = lane < cnt ? mlen[myIdx] : 0u;
    const uint32_t pass1Dist = lane < cnt ? (uint32_t)mdist[myIdx] : 0u;
    if (__ballot(pass1Len == kLongMatch) == 0) continue;
    const uint32_t myRank = lane < cnt ? rank[first + lane] : 0u;
    const uint32_t rowCnt = cnt > rowBase ? (cnt - rowBase < 16 ? cnt - rowBase : 16) : 0;

    // per-row state (replicated over the row's 16 lanes)
    uint32_t j = 0;  // target index inside the row
    bool needInit = true, done = false, isIv = false;
    uint64_t p = 0, lb = 0;
    uint32_t key = 0, room = 0, bestLen = 0, bestDist = 0, steps = 0, gsCur = 0;
    int64_t slot = 0;
    uint32_t carryLen = 0, carryDist = 0;
    uint32_t resLen = pass1Len, resDist = pass1Dist;  // lane rowBase+t holds the result of target first+rowBase+t
    uint64_t runLo = 0, runHi = 0;  // the row's last same-letter run (1)
    bool wantRun = false;
    int64_t runJump = -1;            // the highest slot of the row's group below runLo, for (jumpLo, jumpGs)
    uint64_t jumpLo = ~0ull;
    uint32_t jumpGs = 0;
    // after a target's first step inside a run, the rest of the group's candidates inside the run match
    // exactly as far as the nearest one (the run's end): none can win, the walk jumps below the run
    auto run_jump = [&]() {
      if (!(1 && p >= runLo && p < runHi && slot >= (int64_t)gsCur)) return;
      if (S.w0 + slot_pos(compact, small, (uint32_t)slot) < runLo) return;
      if (jumpLo != runLo || jumpGs != gsCur) {
        int64_t a = (int64_t)gsCur, b = slot;  // largest s in [a, b] with position < runLo, else a - 1
        if (S.w0 + slot_pos(compact, small, (uint32_t)a) >= runLo) {
          b = a - 1;
        } else {
          while (a < b) {
            const int64_t mid = (a + b + 1) >> 1;
            if (S.w0 + slot_pos(compact, small, (uint32_t)mid) < runLo) a = mid;
            else b = mid - 1;
          }
          b = a;
        }
        runJump = b;
        jumpLo = runLo;
        jumpGs = gsCur;
      }
      if (runJump < slot) slot = runJump;
    };

    while (true) {
      const bool live = j < rowCnt;
      if (__ballot(live) == 0) break;
      const uint32_t rCur = __shfl(myRank, (int)(rowBase + (j & 15)), 64);
      const uint32_t curP1Len = __shfl(pass1Len, (int)(rowBase + (j & 15)), 64);
      const uint32_t curP1Dist = __shfl(pass1Dist, (int)(rowBase + (j & 15)), 64);
      if (live && needInit) {
        needInit = false;
        done = false;
        isIv = false;
        p = S.s0 + first + rowBase + j;
        if (curP1Len != kLongMatch) {
          // finished by pass 1: keep its result; it is also the carry for the next target
          bestLen = curP1Len;
          bestDist = curP1Dist;
          done = true;
        }
        for (uint32_t k = 0; !done && k < niv; k++)
          if (p >= iv[k].lo && p < iv[k].hi) {
            // shortcut interval: the reference copies the predecessor's match, minus one
            isIv = true;
            bestLen = (uint32_t)(iv[k].La - (p - iv[k].a));
            bestDist = 1;
          }
        if (isIv) {
          done = true;
        } else if (!done) {
          key = src.ld4(p);
          room = (uint32_t)(stopAbs - p);
          wantRun = 1 && key == (key & 0xFFu) * 0x01010101u && !(p >= runLo && p < runHi);
          lb = p > kWindow ? p - kWindow : 0;
          if (cut != kNone && ref_hash(key) == cutHash && cut > lb) lb = cut;
          slot = (int64_t)rCur - 1;
          gsCur = slot_gs(compact, small, E, rCur);
          if (unlimited) {
            bestLen = 0;
            bestDist = 0;
            // the candidate at the previous target's best distance matches exactly one byte less
            if (carryLen >= 5) {
              const uint64_t c = p - carryDist;
              if (c >= lb && !(niv && in_iv(iv, niv, c)) && !(pvN && in_iv(pvIv, pvN, c))) {
                bestLen = carryLen - 1;
                bestDist = carryDist;
              }
            }
            // pass 1 left the nearest candidate that reached its cap: its exact prefix, 64 bytes
            // per step over the row's 16 lanes, is a lower bound that ends most walks at once
            if (curP1Dist != 0u && (curP1Dist < bestDist || bestDist == 0u || bestLen < room)) {
              const uint64_t c = p - curP1Dist;
              uint32_t k = 0, lcp = 0;
              while (true) {
                const uint32_t off = k + 4u * li;
                const uint32_t x = off < room ? (src.ld4(p + off) ^ src.ld4(c + off)) : 0xFFFFFFFFu;
                const uint32_t mis = (uint32_t)(__ballot(x != 0u) >> rowBase) & 0xFFFFu;
                if (mis) {
                  const uint32_t f = (uint32_t)__builtin_ctz(mis);
                  const uint32_t xf = (uint32_t)__shfl(x, (int)(rowBase + f), 64);
                  lcp = k + 4u * f + ((uint32_t)__builtin_ctz(xf) >> 3);
                  break;
                }
                k += 64;
              }
              lcp = lcp < room ? lcp : room;
              if (lcp > bestLen || (lcp == bestLen && curP1Dist < bestDist)) {
                bestLen = lcp;
                bestDist = curP1Dist;
              }
            }
          } else {
            bestLen = 1;
            bestDist = 0;
            steps = maxChain;
          }
        }
      }
      // a target that starts four equal bytes outside the row's cached run: the run's extent, forward to
      // the block's last searchable byte and backward to the window base, 64 bytes per step over the
      // row's 16 lanes (once per run and row)
      if (__ballot(wantRun)) {
        const bool want = wantRun;
        wantRun = false;
        const uint32_t pat = (key & 0xFFu) * 0x01010101u;
        bool go = want;
        uint64_t hiF = p;
        for (uint64_t k = 0; __ballot(go); k += 64) {
          const uint64_t q = p + k + 4u * li;
          const uint32_t x = go && q < stopAbs ? (src.ld4(q) ^ pat) : 0xFFFFFFFFu;
          const uint32_t mis = (uint32_t)(__ballot(go && x != 0u) >> rowBase) & 0xFFFFu;
          if (go && mis) {
            const uint32_t f = (uint32_t)__builtin_ctz(mis);
            const uint32_t xf = (uint32_t)__shfl(x, (int)(rowBase + f), 64);
            hiF = p + k + 4u * f + ((uint32_t)__builtin_ctz(xf) >> 3);
            go = false;
          }
        }
        go = want;
        uint64_t loF = p;
        for (uint64_t k = 0; __ballot(go); k += 64) {
          const int64_t q = (int64_t)p - (int64_t)k - 4 * (int64_t)(li + 1u);  // bytes q .. q + 3
          uint32_t hm = 0;                                                     // 1 + highest mismatching byte
          bool m = false;
          if (go) {
            if (q < (int64_t)S.w0) {
              m = true;
              hm = 4u;  // not in the window: the run is only known down to the word above it
            } else {
              const uint32_t x = src.ld4((uint64_t)q) ^ pat;
              m = x != 0u;
              hm = m ? (uint32_t)(31 - __builtin_clz(x)) / 8u + 1u : 0u;
            }
          }
          const uint32_t mis = (uint32_t)(__ballot(go && m) >> rowBase) & 0xFFFFu;
          if (go && mis) {
            const uint32_t f = (uint32_t)__builtin_ctz(mis);  // nearest word below p with a mismatch
            const int64_t qf = (int64_t)p - (int64_t)k - 4 * (int64_t)(f + 1u);
            const uint32_t hf = (uint32_t)__shfl(hm, (int)(rowBase + f), 64);
            loF = (uint64_t)(qf + (int64_t)hf);  // bytes [loF, p) verified equal (>= S.w0: see hm)
            go = false;
          }
        }
        if (want) {
          runLo = loF;
          runHi = hiF < stopAbs ? hiF : stopAbs;
        }
      }
      // one step: 16 candidates of the row's key group, nearest first
      const bool act = live && !done;
      bool valid = false, exhausted = true;
      uint32_t got = 0, dist = 0;
      if (act) {
        const int64_t sl = slot - (int64_t)li;
        if (sl >= (int64_t)gsCur) {
          const uint64_t c = S.w0 + slot_pos(compact, small, (uint32_t)sl);
          exhausted = c < lb;  // positions descend inside the group: everything further is older
          dist = (uint32_t)(p - c);
          valid = !exhausted && src.ld4(c) == key;  // same hash, same four bytes
          if (valid) {
            if (unlimited) {
              if (dist != bestDist) {
                const uint32_t need = dist < bestDist ? bestLen : bestLen + 1;
                got = prefix_run(src, p, c, need < 4 ? 4 : need, room, runLo, runHi);
                if (got < need) got = 0;
              }
            } else {
              got = prefix_run(src, p, c, bestLen + 1 < 4 ? 4 : bestLen + 1, room, runLo, runHi);
              if (got <= bestLen) got = 0;
            }
          }
        }
      }
      const uint32_t rowExhausted = (uint32_t)(__ballot(exhausted) >> rowBase) & 0xFFFFu;
      if (unlimited) {
        // longest, then nearest (lower lane = nearer candidate)
        const uint32_t top = row_max(got ? (got << 4) | (15u - li) : 0u);
        const uint32_t wdist = __shfl(dist, (int)(rowBase + 15u - (top & 15u)), 64);
        const uint32_t farDist = __shfl(dist, (int)(rowBase + 15u), 64);
        if (act) {
          if (top) {
            const uint32_t tl = top >> 4;
            if (tl > bestLen || (tl == bestLen && wdist < bestDist)) {
              bestLen = tl;
              bestDist = wdist;
            }
          }
          if (rowExhausted != 0u) done = true;                           // key group / window exhausted
          else if (bestLen >= room && farDist >= bestDist) done = true;   // nothing left can win
          slot -= 16;
          if (!done) run_jump();
        }
      } else {
        // strict improvements in chain order ("records"); the reference stops after maxChain of them
        const uint32_t incl = row_scan_max(got);
        const uint32_t excl = dpp<kRowShr + 1>(incl);  // row lane 0 reads outside its row: 0 (keep unconditional: DPP must not read a masked-off lane)
        const bool rec = got > bestLen && got > excl;
        const uint32_t rowRec = (uint32_t)(__ballot(rec) >> rowBase) & 0xFFFFu;
        const uint32_t nrec = (uint32_t)__popc(rowRec);
        uint32_t sel = 0;
        if (nrec) {
          if (nrec >= steps) {
            uint32_t m = rowRec;
            for (uint32_t k = 1; k < steps; k++) m &= m - 1;
            sel = (uint32_t)__builtin_ctz(m);
          } else {
            sel = 31u - (uint32_t)__builtin_clz(rowRec);
          }
        }
        const uint32_t selGot = __shfl(got, (int)(rowBase + sel), 64);
        const uint32_t selDist = __shfl(dist, (int)(rowBase + sel), 64);
        if (act) {
          if (nrec) {
            bestLen = selGot;
            bestDist = selDist;
            if (nrec >= steps) done = true;
            else steps -= nrec;
          }
          if (rowExhausted != 0u || bestLen >= room) done = true;
          slot -= 16;
          if (!done) run_jump();
        }
      }
      if (live && done) {
        if (!isIv && bestDist == 0) bestLen = 0;  // no candidate: the reference never searched here
        if (li == j) {
          resLen = bestLen;
          resDist = bestDist;
        }
        carryLen = isIv ? 0u : bestLen;
        carryDist = bestDist;
        j++;
        needInit = true;
      }
    }
    if (lane < cnt && pass1Len == kLongMatch) {
      mlen[myIdx] = resLen;
      mdist[myIdx] = (uint16_t)resDist;
    }
    // the parse keeps range minima for blocks with matches of kRmqLen+ (other than same-letter runs)
    const bool rmqLen = lane < cnt && pass1Len == kLongMatch && resLen >= kRmqLen && !(resDist == 1u && resLen >= kSameLetter);
    if (__ballot(rmqLen) && lane == 0) atomicOr(&longFlag[S.block], kFlagRmq);
    // a distance-1 match beyond MaxSameLetter: the next position may take the same-letter shortcut
    // (smallz4.h:631-643): at greedy/lazy levels k_lazy_check compares the block's searches with its intervals
    const bool runLen = lane < cnt && pass1Len == kLongMatch && resDist == 1u && resLen > kSameLetter;
    if (__ballot(runLen) && lane == 0) atomicOr(&longFlag[S.block], kFlagRun);
  }
}

// ================================================================================================
// k_find_long9 (pass 2 at -9): the targets pass 1 left marked -- matches of kLongCap9+ bytes and
// targets of groups larger than kBigGroup -- walked in text order.  A wavefront takes a chunk of 64
// targets; every "stretch" of consecutive marked targets is walked by one wavefront from its head,
// 64 candidates (nearest first) per step.  Two facts bound the walk:
//   carry   if target p-1 has best match (d, L), candidate p - d has exactly L - 1 in common with p;
//   pruning any candidate c' whose preceding byte equals data[p-1] (c' - 1 then being a candidate of
//           p-1 with one more byte in common) has at most L - 1 in common with p, and if exactly
//           L - 1 it is not nearer than d: it cannot win (the longest-previous-factor argument).
//           Inside runs and periodic data such candidates form contiguous runs of sorted slots, and
//           skip[s] (the slot below the run of s) jumps over them in one step.
// Pruning needs p-1's result to be the reference's exact maximum (pass 1 / this pass), the carry to
// be a valid candidate of p, and no lookback cut (stream blocks keep the plain walk).
// ================================================================================================
constexpr uint32_t kPiece = 1024;  // stretch pieces walked one after the other by one wavefront

template <class Src>
__device__ __forceinline__ uint32_t wave_exact_prefix(const Src& src, uint64_t p, uint64_t c, uint32_t room)
{
  const uint32_t lane = lane_id();
  uint32_t k = 0;
  while (true) {
    const uint32_t off = k + 4u * lane;
    const uint32_t x = off < room ? (src.ld4(p + off) ^ src.ld4(c + off)) : 0xFFFFFFFFu;
    const uint64_t mis = __ballot(x != 0u);
    if (mis) {
      const uint32_t f = (uint32_t)__builtin_ctzll(mis);
      const uint32_t xf = rdlane(x, f);
      const uint32_t l = k + 4u * f + ((uint32_t)__builtin_ctz(xf) >> 3);
      return l < room ? l : room;
    }
    k += 256;
  }
}

template <bool kLds>
__device__ __forceinline__ void find_long9_body(const uint8_t* __restrict__ in, const Segment* __restrict__ segs,
                                                             const Block* __restrict__ blocks, const Interval* __restrict__ ivAll,
                                                             const uint32_t* __restrict__ ivCount, const uint2* __restrict__ compactAll,
                                                             uint2* __restrict__ skipAll, const uint32_t* __restrict__ rankAll,
                                                             const uint32_t* __restrict__ longBits, const uint32_t* __restrict__ segLong,
                                                             uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist,
                                                             uint64_t matchBase, uint32_t* __restrict__ longFlag,
                                                             uint32_t* __restrict__ specLen, uint32_t* __restrict__ specDist,
                                                             int fixMode)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t win[];
  __shared__ uint32_t s_next;
  __shared__ uint64_t exLo[2 * kMaxIv], exHi[2 * kMaxIv];
  __shared__ uint32_t nEx;
  __shared__ uint32_t s_scan[kFindThreads / 64];
  const Segment S = segs[blockIdx.x];
  const Block B = blocks[S.block];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const void* compact = compactAll + S.elemOff;
  const uint32_t* rank = rankAll + S.rankOff;
  int32_t* skip = reinterpret_cast<int32_t*>(skipAll + S.elemOff);
  const Interval* iv = ivAll + (uint64_t)S.block * kMaxIv;
  const uint32_t niv = ivCount[S.block];
  if (fixMode) {
    // the repair pass has work only where a piece head's speculative carry differs from its
    // predecessor's final result (the same test as below): otherwise leave before staging the window
    bool any = false;
    if (segLong[blockIdx.x] != 0u) {
      for (uint64_t q0 = S.s0 + kPiece * (1u + tid); q0 < S.s1; q0 += (uint64_t)kPiece * kFindThreads) {
        const uint64_t i0 = q0 - matchBase, i1 = q0 - 1 - matchBase;
        if (!((longBits[i0 >> 5] >> (i0 & 31)) & 1u) || !((longBits[i1 >> 5] >> (i1 & 31)) & 1u)) continue;
        const uint32_t sd = specDist[q0 - matchBase];
        if (sd == 0u) continue;
        if (mlen[q0 - 1 - matchBase] == specLen[q0 - matchBase] && mdist[q0 - 1 - matchBase] == sd) continue;
        any = true;
      }
    }
    if (__syncthreads_or(any ? 1 : 0) == 0) return;
  }

  // positions not inserted into the chains: shortcut intervals of this block and the previous one
  if (tid == 0) {
    uint32_t k = 0;
    const uint32_t ids[2] = {B.prev, S.block};
    for (int t = 0; t < 2; t++) {
      if (ids[t] == kNoBlock) continue;
      const Interval* ivb = ivAll + (uint64_t)ids[t] * kMaxIv;
      for (uint32_t j = 0; j < ivCount[ids[t]]; j++) {
        const uint64_t lo = ivb[j].lo > S.w0 ? ivb[j].lo : S.w0, hi = ivb[j].hi < S.s1 ? ivb[j].hi : S.s1;
        if (lo < hi) {
          exLo[k] = lo;
          exHi[k] = hi;
          k++;
        }
      }
    }
    nEx = k;
    s_next = 0;
  }
  // kLds: the block's whole window in LDS; otherwise [w0, s1 + 64) in LDS and the rest from HBM, or
  // (1) only the segment's own [s0, s1 + 64): 64 KiB, two workgroups per CU
  typename std::conditional<kLds, Bytes<true>, BytesTail>::type src;
  {
    const uint64_t lo = kLds ? S.w0 : S.s0;
    const uint64_t end = kLds ? B.end + 8 : (S.s1 + 64 < B.end + 8 ? S.s1 + 64 : B.end + 8);
    const uint32_t words = (uint32_t)((end - lo + 3) / 4);
    for (uint32_t i = tid; i < words; i += kFindThreads) win[i] = gload4(in, lo + 4ull * i);
    src.w = win;
    src.base = lo;
    if constexpr (!kLds) {
      src.span = 4ull * words;
      src.in = in;
    }
  }
  __syncthreads();
  const uint32_t ne = nEx;
  uint32_t E = (uint32_t)(S.s1 - S.w0);
  for (uint32_t j = 0; j < ne; j++) E -= (uint32_t)(exHi[j] - exLo[j]);
  const bool small = compact_small(S);
  auto excluded = [&](uint64_t q) -> bool {
    for (uint32_t j = 0; j < ne; j++)
      if (q >= exLo[j] && q < exHi[j]) return true;
    return false;
  };
  // preceding byte of candidate position q, or 256 when q - 1 is not a chain position
  auto pred_class = [&](uint64_t q) -> uint32_t {
    if (q <= S.w0 || excluded(q - 1)) return 256u;
    return src.ld4(q - 1) & 0xFFu;
  };
  auto long_bit = [&](uint64_t q) -> bool {
    const uint64_t idx = q - matchBase;
    return (longBits[idx >> 5] >> (idx & 31)) & 1u;
  };

  uint64_t cut = B.cut;
  uint32_t cutHash = 0;
  if (cut != kNone) {
    const Interval* pv = ivAll + (uint64_t)B.prev * kMaxIv;
    if (in_iv(pv, ivCount[B.prev], cut)) cut = kNone;
    else cutHash = ref_hash(gload4(in, cut));
  }
  const uint64_t stopAbs = B.end - kTailLiterals;
  const bool searched = segLong[blockIdx.x] != 0u;

  // 1. skip[s] = the slot just below the run of equal preceding bytes that holds s (runs end at
  //    group starts): an inclusive max-scan of run starts, tiles of 1024 slots
  if (searched && !fixMode) {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < E; base += kFindThreads) {
      const uint32_t sl = base + tid;
      const bool valid = sl < E;
      bool start = true;
      if (valid) {
        const uint32_t g = slot_gs(compact, small, E, sl);
        if (sl > g)
          start = pred_class(S.w0 + slot_pos(compact, small, sl)) != pred_class(S.w0 + slot_pos(compact, small, sl - 1));
      }
      uint32_t v = wave_incl_scan_max(valid && start ? sl + 1 : 0u);
      if (lane == 63) s_scan[wave] = v;
      __syncthreads();
      uint32_t pre = carry;
      for (uint32_t w = 0; w < wave; w++) pre = s_scan[w] > pre ? s_scan[w] : pre;
      v = v > pre ? v : pre;
      if (valid) skip[sl] = (int32_t)v - 2;  // (run start) - 1
      for (uint32_t w = wave; w < kFindThreads / 64; w++) pre = s_scan[w] > pre ? s_scan[w] : pre;
      carry = pre;
      __syncthreads();
    }
    __syncthreads();
  }

  // same-letter runs (1): the wave's last run [runLo, runHi) of a target's byte (runHi capped
  // at the block's last searchable byte).  A candidate inside the target's run matches exactly up to the
  // run's end, so after the nearest such candidate none of the others can win: the walk jumps below the
  // run (the slot, cached per run and key group).  Without it a run makes the walk quadratic.
  uint64_t runLo = 0, runHi = 0, jumpLo = ~0ull;
  int32_t jumpSlot = -1, jumpGs = -1;
  auto run_of = [&](uint64_t p, uint32_t key) {  // wave-uniform
    if (!1 || key != (key & 0xFFu) * 0x01010101u || (p >= runLo && p < runHi)) return;
    const uint32_t pat = key;
    uint64_t hi = p;
    for (uint64_t k = 0;; k += 256) {
      const uint64_t q = p + k + 4u * lane;
      const uint32_t x = q < stopAbs ? (src.ld4(q) ^ pat) : 0xFFFFFFFFu;
      const uint64_t mis = __ballot(x != 0u);
      if (mis) {
        const uint32_t f = (uint32_t)__builtin_ctzll(mis);
        hi = p + k + 4u * f + ((uint32_t)__builtin_ctz(rdlane(x, f)) >> 3);
        break;
      }
    }
    uint64_t lo = p;
    for (uint64_t k = 0;; k += 256) {
      const int64_t q = (int64_t)p - (int64_t)k - 4 * (int64_t)(lane + 1u);
      uint32_t hm = 4u;  // below the window: the run is only known down to the word above
      bool m = true;
      if (q >= (int64_t)S.w0) {
        const uint32_t x = src.ld4((uint64_t)q) ^ pat;
        m = x != 0u;
        hm = m ? (uint32_t)(31 - __builtin_clz(x)) / 8u + 1u : 0u;
      }
      const uint64_t mis = __ballot(m);
      if (mis) {
        const uint32_t f = (uint32_t)__builtin_ctzll(mis);
        lo = (uint64_t)((int64_t)p - (int64_t)k - 4 * (int64_t)(f + 1u) + (int64_t)rdlane(hm, f));
        break;
      }
    }
    runLo = lo;
    runHi = hi < stopAbs ? hi : stopAbs;
  };
  auto run_prefix = [&](uint64_t p, uint64_t c, uint32_t room, bool& known) -> uint32_t {
    known = 1 && p >= runLo && p < runHi && c >= runLo;
    const uint64_t e = runHi - p;
    return e < (uint64_t)room ? (uint32_t)e : room;
  };
  // the highest slot of key group [gs, s] whose position is below runLo (gs - 1: none)
  auto run_jump_slot = [&](int32_t gs, int32_t s) -> int32_t {
    if (jumpLo == runLo && jumpGs == gs) return jumpSlot;
    int32_t a = gs, b = s;
    if (S.w0 + slot_pos(compact, small, (uint32_t)a) >= runLo) {
      b = a - 1;
    } else {
      while (a < b) {
        const int32_t mid = (a + b + 1) >> 1;
        if (S.w0 + slot_pos(compact, small, (uint32_t)mid) < runLo) a = mid;
        else b = mid - 1;
      }
      b = a;
    }
    jumpLo = runLo;
    jumpGs = gs;
    jumpSlot = b;
    return b;
  };

  // best match of target p (wave-uniform): carry (cLen, cDist), exact = the carry is p-1's maximum
  auto best_of = [&](uint64_t p, uint32_t cLen, uint32_t cDist, bool exact, uint32_t& bLen, uint32_t& bDist) {
    SZ4_D5(if (lane_id() == 0) atomicAdd((unsigned long long*)&sz4_diag[0], 1ull);)
    const uint32_t key = src.ld4(p);
    const uint32_t room = (uint32_t)(stopAbs - p);
    uint64_t lb = p > kWindow ? p - kWindow : 0;
    if (cut != kNone && ref_hash(key) == cutHash && cut > lb) lb = cut;
    uint32_t bestLen = 0, bestDist = 0;
    bool carryOk = false;
    run_of(p, key);
    if (cDist != 0u && cLen >= 5u) {
      const uint64_t c = p - cDist;
      if (c >= lb && !excluded(c)) {
        bestLen = cLen - 1;
        bestDist = cDist;
        carryOk = true;
      }
    }
    if (carryOk && bestLen >= room && bestDist == 1u) {
      bLen = bestLen;  // as long as possible, and no candidate is nearer
      bDist = 1;
      return;
    }
    const uint32_t slot = rank[p - S.s0];
    const int32_t gs = (int32_t)slot_gs(compact, small, E, slot);
    const bool prune = exact && cut == kNone && (carryOk || cLen < 5u);
    const uint32_t pc = prune ? (src.ld4(p - 1) & 0xFFu) : 0xFFFFu;
    // pass 1's nearest candidate at its cap
    const uint32_t seed = mdist[p - matchBase];
    if (seed != 0u && (bestLen < room || seed < bestDist)) {
      bool rk;
      const uint32_t rl = run_prefix(p, p - seed, room, rk);
      const uint32_t l = rk ? rl : wave_exact_prefix(src, p, p - seed, room);
      if (l > bestLen || (l == bestLen && seed < bestDist)) {
        bestLen = l;
        bestDist = seed;
      }
    }
    int32_t s = (int32_t)slot - 1;
    if (bestDist == 0u && s >= gs) {
      // nothing known yet: the nearest candidate's exact prefix, 256 bytes per step, so that the walk
      // below rejects the others at a glance
      const uint64_t c = S.w0 + slot_pos(compact, small, (uint32_t)s);
      if (c >= lb && src.ld4(c) == key) {
        bool rk;
        const uint32_t rl = run_prefix(p, c, room, rk);
        bestLen = rk ? rl : wave_exact_prefix(src, p, c, room);
        bestDist = (uint32_t)(p - c);
        s--;
      }
    }
    // inside a run: the nearest unvisited candidate, when it lies in the run, is the best of the run's
    // candidates (all match up to the run's end; it is the nearest); the walk goes on below the run
    if (1 && key == (key & 0xFFu) * 0x01010101u && p >= runLo && p < runHi && s >= gs) {
      const uint64_t c0 = S.w0 + slot_pos(compact, small, (uint32_t)s);
      if (c0 >= runLo) {
        if (c0 >= lb) {
          bool rk;
          const uint32_t rl = run_prefix(p, c0, room, rk);
          const uint32_t d0 = (uint32_t)(p - c0);
          if (bestDist == 0u || rl > bestLen || (rl == bestLen && d0 < bestDist)) {
            bestLen = rl;
            bestDist = d0;
          }
        }
        const int32_t js = run_jump_slot(gs, s);
        if (js < s) s = js;
      }
    }
    while (s >= gs) {
      SZ4_D5(if (lane_id() == 0) atomicAdd((unsigned long long*)&sz4_diag[1], 1ull);)
      const int32_t sl = s - (int32_t)lane;
      const bool inG = sl >= gs;
      const uint64_t c = inG ? S.w0 + slot_pos(compact, small, (uint32_t)sl) : 0u;
      const bool below = inG && c < lb;  // positions descend: everything farther is out of the window
      const bool valid = inG && !below;
      const bool pruned = valid && prune && pred_class(c) == pc;
      const uint64_t inMask = __ballot(inG);
      if (!__ballot(below) && __ballot(pruned) == inMask && inMask == ~0ull) {
        s = skip[s - 63];  // the whole step is one run of pruned candidates: below that run
        continue;
      }
      const uint32_t dist = (uint32_t)(p - c);
      uint32_t got = 0;
      if (valid && !pruned && src.ld4(c) == key) {
        const uint32_t need = bestDist == 0u ? 4u : (dist < bestDist ? bestLen : bestLen + 1u);
        got = prefix_if_at_least(src, p, c, need < 4u ? 4u : need, room);
        if (got < need) got = 0;
      }
      // longest, then nearest (lower lane); got <= room < 2^26, so the key fits 32 bits: a DPP row
      // maximum and four readlanes instead of a 64-bit shuffle butterfly
      const uint32_t top = wave_max_fast(got ? (got << 6) | (63u - lane) : 0u);
      if (top) {
        const uint32_t tl = top >> 6, wl = 63u - (top & 63u);
        const uint32_t wd = rdlane(dist, wl);
        if (tl > bestLen || (tl == bestLen && wd < bestDist)) {
          bestLen = tl;
          bestDist = wd;
        }
      }
      if (__ballot(below)) break;
      const uint32_t lastLane = (uint32_t)(63 - __builtin_clzll(inMask));
      const uint32_t farDist = rdlane(dist, lastLane);
      if (bestDist != 0u && bestLen >= room && farDist >= bestDist) break;  // only nearer ties could win
      s -= 64;
    }
    if (bestDist == 0u) bestLen = 0;
    bLen = bestLen;
    bDist = bestDist;
  };

  // a stretch from q: best matches one after the other, each carrying into the next; ends at the
  // piece boundary or the first target pass 1 finished
  // one target per lane (a speculative batch): the same result as best_of under the same carry,
  // each lane walking its own candidates (class runs jumped with skip pointers)
  auto best_lane = [&](uint64_t p, uint32_t cLen, uint32_t cDist, uint32_t& bLen, uint32_t& bDist) {
    SZ4_D5(atomicAdd((unsigned long long*)&sz4_diag[2], 1ull);)
    const uint32_t key = src.ld4(p);
    const uint32_t room = (uint32_t)(stopAbs - p);
    const uint64_t lb = p > kWindow ? p - kWindow : 0;  // no lookback cut on this path
    uint32_t bestLen = 0, bestDist = 0;
    bool carryOk = false;
    if (cDist != 0u && cLen >= 5u) {
      const uint64_t c = p - cDist;
      if (c >= lb && !excluded(c)) {
        bestLen = cLen - 1;
        bestDist = cDist;
        carryOk = true;
      }
    }
    if (!(carryOk && bestLen >= room && bestDist == 1u)) {
      const bool prune = carryOk || cLen < 5u;
      const uint32_t pc = prune ? (src.ld4(p - 1) & 0xFFu) : 0xFFFFu;
      const uint32_t slot = rank[p - S.s0];
      const int32_t gs = (int32_t)slot_gs(compact, small, E, slot);
      int32_t sl = (int32_t)slot - 1;
      while (sl >= gs) {
        SZ4_D5(atomicAdd((unsigned long long*)&sz4_diag[3], 1ull);)
        const uint64_t c = S.w0 + slot_pos(compact, small, (uint32_t)sl);
        if (c < lb) break;  // positions descend: everything farther is out of the window
        if (prune && pred_class(c) == pc) {
          sl = skip[sl];  // a run of pruned candidates
          continue;
        }
        const uint32_t dist = (uint32_t)(p - c);
        if (bestDist != 0u && bestLen >= room && dist >= bestDist) break;  // only nearer ties could win
        if (src.ld4(c) == key) {
          const uint32_t need = bestDist == 0u ? 4u : (dist < bestDist ? bestLen : bestLen + 1u);
          const uint32_t got = prefix_if_at_least(src, p, c, need < 4u ? 4u : need, room);
          SZ4_D5(atomicAdd((unsigned long long*)&sz4_diag[7], (unsigned long long)((need > got ? need : got) / 4u + 1u));)
          if (got >= need && got != 0u && (got > bestLen || dist < bestDist)) {
            bestLen = got;
            bestDist = dist;
          }
        }
        sl--;
      }
    }
    bLen = bestDist ? bestLen : 0u;
    bDist = bestDist;
  };

  // a stretch from q: best matches in order, each carrying into the next; ends at the piece boundary
  // or the first target pass 1 finished.  With an exact carry (cLen, cDist) the next targets are
  // taken 64 at a time, one per lane, on the hypothesis that the carried match goes on: lane t
  // assumes best(q + t - 1) = (cLen - t, cDist).  Lane 0's carry is exact, and the first lane whose
  // result breaks the chain is exact too (its predecessor kept the hypothesis); the batch is taken up
  // to that lane and the next one starts after it with its result as the carry.
  auto walk_stretch = [&](uint64_t q, uint32_t cLen, uint32_t cDist, bool exact) {
    bool rmqLen = false;
    // stretch end: piece boundary, segment end or first unmarked target
    const uint64_t pieceEnd = S.s0 + (((q - S.s0) / kPiece) + 1) * kPiece;
    const uint64_t lim = pieceEnd < S.s1 ? pieceEnd : S.s1;
    uint64_t qEnd = q;
    while (qEnd < lim) {
      const uint64_t qi = qEnd - matchBase;
      const uint32_t w = longBits[qi >> 5] >> (qi & 31);  // the word's bits from qEnd on
      const uint32_t ones = (uint32_t)__builtin_ctzll(~(uint64_t)w);  // <= 32 - (qi & 31)
      qEnd += ones;
      if (ones < 32u - (uint32_t)(qi & 31)) break;
    }
    if (qEnd > lim) qEnd = lim;
    while (q < qEnd) {
      uint32_t bLen, bDist;
      const uint64_t left = qEnd - q;
      const uint32_t spec = exact && cut == kNone && cDist != 0u && cLen >= 6u
                                ? (uint32_t)min<uint64_t>(min<uint64_t>(64, left), cLen - 5u) : 0u;
      if (spec >= 2) {
        const bool mine = lane < spec;
        uint32_t rL = 0, rD = 0;
        if (mine) best_lane(q + lane, cLen - lane, cDist, rL, rD);
        const bool keeps = rL == cLen - 1u - lane && rD == cDist;
        const uint64_t breaks = __ballot(mine && !keeps);
        const uint32_t f = breaks ? (uint32_t)__builtin_ctzll(breaks) : spec - 1u;  // last lane taken
        if (lane <= f) {
          mlen[q + lane - matchBase] = rL;
          mdist[q + lane - matchBase] = (uint16_t)rD;
        }
        rmqLen |= __ballot(lane <= f && rL >= kRmqLen && !(rD == 1u && rL >= kSameLetter)) != 0;
        bLen = rdlane(rL, f);
        bDist = rdlane(rD, f);
        q += f + 1;
      } else {
        best_of(q, cLen, cDist, exact, bLen, bDist);
        if (lane == 0) {
          mlen[q - matchBase] = bLen;
          mdist[q - matchBase] = (uint16_t)bDist;
        }
        rmqLen |= bLen >= kRmqLen && !(bDist == 1u && bLen >= kSameLetter);
        q++;
      }
      cLen = bLen;
      cDist = bDist;
      exact = true;
    }
    if (rmqLen && lane == 0) atomicOr(&longFlag[S.block], kFlagRmq);
  };

  if (fixMode) {
    // repair pass: piece heads whose predecessor was still unknown walked with a speculative carry
    // (specLen, specDist).  In text order, a head whose predecessor's final result differs is walked
    // again with the true carry (which may change the next head's predecessor in turn).
    if (wave != 0 || !searched) return;
    for (uint64_t q0 = S.s0 + kPiece; q0 < S.s1; q0 += kPiece) {
      if (!long_bit(q0) || !long_bit(q0 - 1)) continue;
      const uint32_t sd = specDist[q0 - matchBase];
      if (sd == 0u) continue;  // walked without a carry: exact
      const uint32_t aLen = mlen[q0 - 1 - matchBase], aDist = mdist[q0 - 1 - matchBase];
      if (aLen == specLen[q0 - matchBase] && aDist == sd) continue;
      walk_stretch(q0, aLen, aDist, true);
      SZ4_D5(if (lane_id() == 0) atomicAdd((unsigned long long*)&sz4_diag[4], 1ull);)
    }
    return;
  }

  const uint32_t nTargets = (uint32_t)(S.s1 - S.s0);
  while (true) {
    uint32_t chunkIdx = 0;
    if (lane == 0) chunkIdx = atomicAdd(&s_next, 1u);
    chunkIdx = rdlane(chunkIdx, 0);
    const uint32_t first = chunkIdx * 64;
    if (first >= nTargets) break;
    const uint32_t cnt = nTargets - first < 64 ? nTargets - first : 64;
    const uint64_t p = S.s0 + first + lane;
    const uint64_t myIdx = p - matchBase;
    const uint32_t p1 = lane < cnt ? mlen[myIdx] : 0u;
    if (__ballot(p1 == kLongMatch) == 0) continue;
    const bool lg = lane < cnt && long_bit(p);
    SZ4_D5(
    {
      const uint32_t nl = (uint32_t)__builtin_popcountll(__ballot(lane < cnt && p1 == kLongMatch && lg));
      const uint32_t ni = (uint32_t)__builtin_popcountll(__ballot(lane < cnt && p1 == kLongMatch && !lg));
      if (lane == 0 && nl) atomicAdd((unsigned long long*)&sz4_diag[5], (unsigned long long)nl);
      if (lane == 0 && ni) atomicAdd((unsigned long long*)&sz4_diag[6], (unsigned long long)ni);
      if (lane < cnt && p1 == kLongMatch && lg) {
        const uint64_t k = atomicAdd((unsigned long long*)&sz4_diag[15], 1ull);
        if (k < 512) {
          sz4_diag[64 + 3 * k] = p - B.start;
          sz4_diag[65 + 3 * k] = src.ld4(p) | ((uint64_t)src.ld4(p + 4) << 32);
          sz4_diag[66 + 3 * k] = (uint64_t)mdist[myIdx] | ((uint64_t)(B.end - B.start) << 32);
        }
      }
    }
    )
    // marked but never sorted: shortcut-interval targets copy the predecessor's match, minus one
    if (lane < cnt && p1 == kLongMatch && !lg) {
      for (uint32_t k = 0; k < niv; k++)
        if (p >= iv[k].lo && p < iv[k].hi) {
          mlen[myIdx] = (uint32_t)(iv[k].La - (p - iv[k].a));
          mdist[myIdx] = 1;
        }
    }
    // stretch heads: marked targets whose predecessor is not (or lies before the segment); long
    // stretches are cut every kPiece targets so that they run in parallel
    const bool head = lg && (p == S.s0 || ((p - S.s0) & (kPiece - 1)) == 0 || !long_bit(p - 1));
    uint64_t heads = __ballot(head);
    while (heads) {
      const uint32_t h = (uint32_t)__builtin_ctzll(heads);
      heads &= heads - 1;
      const uint64_t q = S.s0 + first + h;
      // p-1's result: final when it is a target of this block that pass 1 finished
      uint32_t cLen = 0, cDist = 0;
      bool exact = false;
      if (q > B.start && !long_bit(q - 1) && !(niv && in_iv(iv, niv, q - 1))) {
        cLen = mlen[q - 1 - matchBase];
        cDist = mdist[q - 1 - matchBase];
        exact = true;
      } else if (q != S.s0 && long_bit(q - 1) && cut == kNone) {
        // a piece head inside a stretch: speculate that its predecessor's best match is the one
        // that makes the nearest candidate its carry (checked and repaired by the fixMode pass)
        const uint32_t key = src.ld4(q);
        const uint32_t slot = rank[q - S.s0];
        const int32_t gs = (int32_t)slot_gs(compact, small, E, slot);
        if ((int32_t)slot - 1 >= gs) {
          const uint64_t c = S.w0 + slot_pos(compact, small, slot - 1);
          if (c + kWindow >= q && src.ld4(c) == key && !excluded(c)) {
            cLen = wave_exact_prefix(src, q, c, (uint32_t)(stopAbs - q)) + 1u;
            cDist = (uint32_t)(q - c);
            exact = true;
          }
        }
      }
      if (lane == 0 && q != S.s0 && long_bit(q - 1)) {
        specLen[q - matchBase] = cLen;
        specDist[q - matchBase] = exact ? cDist : 0u;
      }
      walk_stretch(q, cLen, cDist, exact);
    }
  }
}

// k_find_long9_lds (the whole window in LDS, 64 KiB + 16 B) at <= 80 SGPRs: two 16-wave workgroups per
// CU (8 waves per SIMD) instead of one at 106; <false> stages up to 128 KiB and runs alone on its CU anyway.
#define SZ4_LONG9_ARGS                                                                                        \
  const uint8_t *__restrict__ in, const Segment *__restrict__ segs, const Block *__restrict__ blocks,         \
      const Interval *__restrict__ ivAll, const uint32_t *__restrict__ ivCount,                               \
      const uint2 *__restrict__ compactAll, uint2 *__restrict__ skipAll, const uint32_t *__restrict__ rankAll, \
      const uint32_t *__restrict__ longBits, const uint32_t *__restrict__ segLong, uint32_t *__restrict__ mlen, \
      uint16_t *__restrict__ mdist, uint64_t matchBase, uint32_t *__restrict__ longFlag,                      \
      uint32_t *__restrict__ specLen, uint32_t *__restrict__ specDist, int fixMode
#define SZ4_LONG9_PASS in, segs, blocks, ivAll, ivCount, compactAll, skipAll, rankAll, longBits, segLong, mlen, mdist, \
                       matchBase, longFlag, specLen, specDist, fixMode
__global__ __launch_bounds__(kFindThreads) __attribute__((amdgpu_num_sgpr(80))) void k_find_long9_lds(SZ4_LONG9_ARGS)
{
  find_long9_body<true>(SZ4_LONG9_PASS);
}
__global__ __launch_bounds__(kFindThreads) __attribute__((amdgpu_num_sgpr(80))) void k_find_long9_hbm(SZ4_LONG9_ARGS)
{
  find_long9_body<false>(SZ4_LONG9_PASS);
}
#undef SZ4_LONG9_ARGS
#undef SZ4_LONG9_PASS

// ================================================================================================
// k_find_big (-9, between pass 1 and pass 2): the targets pass 1 handed on because their key group
// holds more than kBigGroup candidates (structured records, tables, padding).  Walking such a group
// once per target is quadratic; instead the maximum is split (the longest-previous-factor identity):
//   best(p) = better of  LM(p)                  -- over the LEFT-MAXIMAL candidates c of p only:
//                                                  data[c-1] != data[p-1], or c-1 not a chain position
//            and         (L(p-1) - 1, D(p-1))    -- every other candidate c has c-1 as a candidate of
//                                                  p-1 with one byte more in common, and the nearest of
//                                                  the longest of those is p-1's own result
// ("better": longer, then nearer -- the reference's strict-improvement walk, smallz4.h:190-252).
// Unrolled along the text this is a prefix maximum of  key(q) = (q + len(q)) << 16 | (0xFFFF - dist(q))
// from the last target whose result is already exact (pass 1), and it needs LM(p) only.
//   1. the segment's big groups are regrouped by the candidates' preceding byte (class 256: no
//      predecessor), so a wavefront of 64 targets of one class scans every candidate EXCEPT its own
//      class in one broadcast pass (mixed-class wavefronts scan all and filter per lane);
//   2. LM(p) -> lm[p] (specLen, free until pass 2);
//   3. the prefix maximum in text order (16 wavefronts, carries through LDS) resolves every big target
//      that follows an exact target of this segment; the rest (a segment start inside a run of big
//      targets, a result at the pass-1 cap) stay marked for pass 2.
// Only blocks without a lookback cut or shortcut intervals (independent blocks): the identity needs
// every candidate position to be a chain position.
// ================================================================================================
constexpr uint32_t kMaxBigGroups = 256;  // big, run-key and LPF groups of one segment (> 128 Ki / 512)
constexpr uint32_t kClsNone = 256;      // preceding byte class of a position without a chain predecessor
constexpr uint32_t kBins = kClsNone + 1;
constexpr uint32_t kAEnd = 256;         // run table: a run that reaches the block end has no next byte
constexpr uint32_t kMaxSlotWords = (65536 + 65535 + 31) / 32;  // a window's slots as bits
constexpr uint32_t kNoScan = 0xFFFFFFFFu;
constexpr uint32_t kLmUnknown = 0xFFFFu;  // LM length: at pass 1's cap (longer possible): pass 2 decides

// exclusive prefix sums of v over the workgroup's threads (thread i: bin i); total in *tot
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* tot)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t incl = wave_incl_scan_add(v);
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (uint32_t w = 0; w < kFindThreads / 64; w++) {
    const uint32_t x = wsum[w];
    base += w < wave ? x : 0u;
    all += x;
  }
  __syncthreads();
  if (tot) *tot = all;
  return base + incl - v;
}

#if SZ4_DIAG == 6
#define SZ4_D6(k)                                                                                   \
  do {                                                                                            \
    if (threadIdx.x == 0) {                                                                       \
      const uint64_t now = __builtin_readcyclecounter();                                          \
      atomicAdd((unsigned long long*)&sz4_diag[k], (unsigned long long)(now - d6t));              \
      d6t = now;                                                                                  \
    }                                                                                             \
  } while (0)
#define SZ4_D6C(k, v) atomicAdd((unsigned long long*)&sz4_diag[k], (unsigned long long)(v))
#define SZ4_D6X(...) __VA_ARGS__
#else
#define SZ4_D6X(...)
#define SZ4_D6(k) \
  do {            \
  } while (0)
#define SZ4_D6C(k, v) \
  do {                \
  } while (0)
#endif
template <bool kLds>
__global__ __launch_bounds__(kFindThreads) __attribute__((amdgpu_waves_per_eu(8), amdgpu_num_sgpr(80))) void k_find_big(const uint8_t* __restrict__ in, const Segment* __restrict__ segs,
                                                           const Block* __restrict__ blocks, const Interval* __restrict__ ivAll,
                                                           const uint32_t* __restrict__ ivCount,
                                                           const uint2* __restrict__ compactAll, uint2* __restrict__ scratchAll,
                                                           uint32_t* __restrict__ longBits, const uint32_t* __restrict__ segLong,
                                                           uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist,
                                                           uint64_t matchBase, uint32_t* __restrict__ lm, uint64_t* __restrict__ segTail,
                                                           uint32_t* __restrict__ runBkt, const uint32_t* __restrict__ rankAll,
                                                           uint32_t* __restrict__ longFlag, uint32_t resolveOnly)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t win[];
  __shared__ uint32_t s_groups[2 * kMaxBigGroups];
  __shared__ uint32_t s_ng, s_next, s_mixed, s_nRuns, s_scanRun, s_niv;
  __shared__ uint64_t s_ivLo[kMaxIv], s_ivHi[kMaxIv], s_ivA[kMaxIv], s_ivLa[kMaxIv];  // this block's intervals
  __shared__ uint32_t s_cls[kBins + 1], s_tcls[kBins + 1];  // bin starts (candidates, targets); run buckets
  __shared__ uint32_t s_cur[2][kBins];                      // counts, then scatter cursors
  __shared__ uint32_t s_wsum[kFindThreads / 64];
  __shared__ uint32_t s_hasHead[kFindThreads / 64], s_outValid[kFindThreads / 64];
  __shared__ uint64_t s_outKey[kFindThreads / 64];
  const Segment S = segs[blockIdx.x];
  const Block B = blocks[S.block];
  if (B.cut != kNone || B.low != B.start)
    return;  // uniform over the workgroup (the resolve launch returns here for every segment of the block)
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  // the block's shortcut intervals (smallz4.h:631-643): their positions are neither inserted nor searched
  if (tid == 0) s_niv = ivCount[S.block] < kMaxIv ? ivCount[S.block] : kMaxIv;
  __syncthreads();
  const uint32_t niv = s_niv;
  for (uint32_t j = tid; j < niv; j += kFindThreads) {
    const Interval x = ivAll[(uint64_t)S.block * kMaxIv + j];
    s_ivLo[j] = x.lo;
    s_ivHi[j] = x.hi;
    s_ivA[j] = x.a;
    s_ivLa[j] = x.La;
  }
  __syncthreads();
  auto excluded = [&](uint64_t q) -> bool {
    for (uint32_t j = 0; j < niv; j++)
      if (q >= s_ivLo[j] && q < s_ivHi[j]) return true;
    return false;
  };
  auto iv_starting_at = [&](uint64_t q) -> int32_t {
    for (uint32_t j = 0; j < niv; j++)
      if (s_ivLo[j] == q) return (int32_t)j;
    return -1;
  };
  if (!resolveOnly && tid == 0) {
    // the state after this segment's last target for the next segment's resolve launch, as it stands
    // when no target here is left to this kernel (no big group, or more than fit): the last target's
    // own result when pass 1 finished it, else unknown.  Phase 3 below overwrites it.
    const uint32_t nTg = (uint32_t)(S.s1 - S.s0);
    const uint64_t idx = S.s1 - 1 - matchBase;
    const uint32_t ml = mlen[idx], md = mdist[idx];
    uint64_t t = 0;
    if (ml != kLongMatch) {
      const uint64_t e = (uint64_t)(nTg - 1) + ml;  // match end relative to s0
      t = (1ull << 63) | (ml >= (uint32_t)kMinMatch && e > (uint64_t)nTg + kMinMatch - 1u
                              ? ((e - nTg) << 16) | (0xFFFFu - md) : 0ull);
    }
    segTail[blockIdx.x] = t;
  }
  if (!segLong[blockIdx.x]) return;  // uniform
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
  const void* compact = compactAll + S.elemOff;
  uint32_t E = (uint32_t)(S.s1 - S.w0);  // window positions minus interval positions: the slots
  for (uint32_t j = 0; j < niv; j++) {
    const uint64_t lo = s_ivLo[j] > S.w0 ? s_ivLo[j] : S.w0, hi = s_ivHi[j] < S.s1 ? s_ivHi[j] : S.s1;
    if (lo < hi) E -= (uint32_t)(hi - lo);
  }
  const bool small = compact_small(S);

  SZ4_D6X(
  uint64_t d6t = __builtin_readcyclecounter();
  if (tid == 0 && !resolveOnly) SZ4_D6C(15, 1);
  )
  // 1. big groups: the groups of the targets pass 1 handed on (marked, distance 0), found through their
  //    slots (rank): their starts as a bitmap over the window's slots, collected in slot order, each
  //    group's end by a binary search over the group starts
  const uint32_t nTg = (uint32_t)(S.s1 - S.s0);
  const uint32_t* rank = rankAll + S.rankOff;
  auto handed = [&](uint64_t q) -> bool {  // q: a target of this segment
    const uint64_t idx = q - matchBase;
    return ((longBits[idx >> 5] >> (idx & 31)) & 1u) && mlen[idx] == kLongMatch && mdist[idx] == 0u;
  };
  const uint32_t gWords = (E + 31) / 32;
  uint32_t* s_gmap = win;  // (the window is loaded only after this: its buffer holds E bits many times over)
  for (uint32_t w = tid; w < gWords; w += kFindThreads) s_gmap[w] = 0;
  __syncthreads();
  for (uint32_t i = tid; i < nTg; i += kFindThreads)
    if (handed(S.s0 + i)) {
      const uint32_t g = slot_gs(compact, small, E, rank[i]);
      atomicOr(&s_gmap[g >> 5], 1u << (g & 31));
    }
  __syncthreads();
  uint32_t ng = 0;
  {
    // words per thread: ceil(4096 / 1024) = 4
    constexpr uint32_t kPer = (kMaxSlotWords + kFindThreads - 1) / kFindThreads;
    uint32_t cnt = 0;
    for (uint32_t k = 0; k < kPer; k++) {
      const uint32_t w = tid * kPer + k;
      cnt += w < gWords ? (uint32_t)__builtin_popcount(s_gmap[w]) : 0u;
    }
    uint32_t at = block_excl_scan(cnt, s_wsum, &ng);
    for (uint32_t k = 0; k < kPer; k++) {
      const uint32_t w = tid * kPer + k;
      uint32_t bits = w < gWords ? s_gmap[w] : 0u;
      while (bits) {
        const uint32_t b = (uint32_t)__builtin_ctz(bits);
        bits &= bits - 1;
        if (at < kMaxBigGroups) s_groups[2 * at] = w * 32 + b;
        at++;
      }
    }
    __syncthreads();
    if (tid < ng && tid < kMaxBigGroups) {
      const uint32_t g = s_groups[2 * tid];
      uint32_t lo = g, hi = E - 1;  // the group's last slot: the last s with gs(s) == g
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (slot_gs(compact, small, E, mid) == g) lo = mid;
        else hi = mid - 1;
      }
      s_groups[2 * tid + 1] = lo + 1;
    }
    __syncthreads();
  }
  SZ4_D6X(
  if (tid == 0 && ng == 0) SZ4_D6C(24, 1);
  if (tid == 0 && ng > kMaxBigGroups) SZ4_D6C(25, 1);
  )
  if (ng == 0 || ng > kMaxBigGroups) return;  // (more cannot fit a window; pass 2 would take them)
  const uint64_t stopAbs = B.end - kTailLiterals;

  if (!resolveOnly) SZ4_D6(0);
  // the second launch only resolves: a segment's first big targets need its predecessor segment's
  // last results, final after the first launch
  if (!resolveOnly) {
  // two workgroups per CU (<= 64 VGPRs): blocks above 64 KiB stage only the segment's own targets
  // [s0, s1 + 64) in LDS, the 64 KiB below them come from HBM/L2
  typename std::conditional<kLds, Bytes<true>, BytesTail>::type src;
  {
    const uint64_t lo = kLds ? S.w0 : S.s0;
    const uint64_t end = kLds ? B.end + 8 : (S.s1 + 64 < B.end + 8 ? S.s1 + 64 : B.end + 8);
    const uint32_t words = (uint32_t)((end - lo + 3) / 4);
    for (uint32_t i = tid; i < words; i += kFindThreads) win[i] = gload4(in, lo + 4ull * i);
    src.w = win;
    src.base = lo;
    if constexpr (!kLds) {
      src.span = 4ull * words;
      src.in = in;
    }
  }
  const uint64_t predLo = S.w0 > B.low ? S.w0 : B.low;  // a predecessor below this is not known here
  // class of a window position: its preceding byte, or kClsNone when that is not a chain position
  // (then the position is always left-maximal)
  auto cls_of = [&](uint64_t q) -> uint32_t {
    return q <= predLo || excluded(q - 1) ? kClsNone : (src.ld4(q - 1) & 0xFFu);
  };
  // a member k_find_sorted handed on
  auto is_target = [&](uint64_t q) { return q >= S.s0 && handed(q); };
  // common prefix of the texts at x and y, at most `cap` bytes (both readable that far)
  auto ext_len = [&](uint64_t x, uint64_t y, uint32_t cap) -> uint32_t {
    uint32_t k = 0;
    while (k < cap) {
      const uint32_t d = src.ld4(x + k) ^ src.ld4(y + k);
      if (d) {
        k += (uint32_t)__builtin_ctz(d) >> 3;
        break;
      }
      k += 4;
    }
    return k < cap ? k : cap;
  };
  uint32_t* C = reinterpret_cast<uint32_t*>(scratchAll + S.elemOff);  // candidates: cls << 17 | rel
  uint32_t* T = C + E;                                                 // targets: rel
  uint32_t* BK = runBkt + (S.s0 - matchBase);                          // run table: runs by next byte
  __syncthreads();

  SZ4_D6(1);
  for (uint32_t gi = 0; gi < ng; gi++) {
    const uint32_t ga = s_groups[2 * gi], gb = s_groups[2 * gi + 1];
    // the group's run key, if it has one (its first or last member's; other keys in the group are
    // 16-bit hash collisions, handled one by one below)
    // (the first and last members can both be collisions -- a random position that hashes like the
    // run key -- so members spread over the group are sampled too; s_mixed below weighs the rest)
    uint32_t gKey = gload4(in, S.w0 + slot_pos(compact, small, ga));
    for (uint32_t k = 1; k <= 8 && !run_key(gKey); k++) {
      const uint32_t at = k == 8 ? gb - 1 : ga + (uint32_t)((uint64_t)(gb - ga) * k / 8);
      gKey = gload4(in, S.w0 + slot_pos(compact, small, at));
    }
    if (tid == 0) s_mixed = 0;
    __syncthreads();
    if (run_key(gKey)) {
      uint32_t other = 0;
      for (uint32_t s = ga + tid; s < gb; s += kFindThreads)
        other += src.ld4(S.w0 + slot_pos(compact, small, s)) != gKey ? 1u : 0u;
      if (other) atomicAdd(&s_mixed, other);
      __syncthreads();
      SZ4_D6X(if (tid == 0 && s_mixed) SZ4_D6C(17, 1);)
    }
    // (a group of mostly other keys goes to the class path)
    const bool runGroup = run_key(gKey) && s_mixed * 4u <= gb - ga;
    __syncthreads();
    if (tid == 0) s_mixed = 0;
    __syncthreads();
    if (runGroup) {
      // ---- a run-key group: its members are the chain positions with at
      // least 4 bytes of a run of v left.  A "piece" is a maximal stretch of consecutive member
      // positions: a whole run, or the part of one before / after the positions the same-letter
      // shortcut left out (an interval), or the part inside the window.  Piece table (position
      // order): C[ga + k] = first rel | next byte a << 17 (the byte after the RUN, kAEnd at the block
      // end); T[ga + k] = R(first) (bytes of v from it, exact) | extra << 24 | kind << 30, kind 0: the
      // piece ends with its run (last = end - 4), 1: an interval follows (last = first + extra),
      // 2: the window ends inside it (last = s1 - 1).  BK: piece indices by a.  Every target's result is
      // exact by itself (all its candidates are considered), so it is written as final.
      const uint32_t v = gKey & 0xFFu;
      SZ4_D6(6);
      if (tid == 0) SZ4_D6C(14, 1);
      // A. pieces: a member whose predecessor position is not a member starts one (block-wide scan);
      //    C[ga + k] = its first, T[ga + k] = its first slot; a target member keeps its piece in lm.
      //    Members of other keys (hash collisions) go to a list of their own, in position order from
      //    the top: C[gb - 1 - j] = the j-th one (rel); a target among them keeps its j in lm.
      auto is_run = [&](uint32_t t) { return src.ld4(S.w0 + slot_pos(compact, small, t)) == gKey; };
      uint32_t base = 0, nColl = 0;
      for (uint32_t t0 = ga; t0 < gb; t0 += kFindThreads) {
        const uint32_t s = t0 + tid;
        const bool inG = s < gb && is_run(s);
        const bool isColl = s < gb && !inG;
        {
          uint32_t tc = 0;
          const uint32_t j = nColl + block_excl_scan(isColl ? 1u : 0u, s_wsum, &tc);
          if (isColl) {
            const uint32_t rc = slot_pos(compact, small, s);
            C[gb - 1u - j] = rc;
            if (is_target(S.w0 + rc)) lm[S.w0 + rc - matchBase] = j;
          }
          nColl += tc;
        }
        const uint32_t r = inG ? slot_pos(compact, small, s) : 0u;
        bool first = inG;
        if (inG) {
          int32_t t = (int32_t)s - 1;
          while (t >= (int32_t)ga && !is_run((uint32_t)t)) t--;
          first = t < (int32_t)ga || slot_pos(compact, small, (uint32_t)t) + 1u != r;
        }
        uint32_t tot = 0;
        const uint32_t k = base + block_excl_scan(first ? 1u : 0u, s_wsum, &tot);
        if (first) {
          C[ga + k] = r;
          T[ga + k] = s;
        }
        if (inG && is_target(S.w0 + r)) lm[S.w0 + r - matchBase] = first ? k : k - 1u;
        base += tot;
      }
      if (tid == 0) {
        s_nRuns = base;
        s_scanRun = kNoScan;
      }
      for (uint32_t k = tid; k <= kAEnd; k += kFindThreads) s_cur[0][k] = 0;
      __threadfence_block();
      __syncthreads();
      const uint32_t nRuns = s_nRuns;
      //    each piece's run end e: 4 bytes after its last member, unless the run goes on past it --
      //    into an interval (then to a + La, the interval's run end, and a few bytes more up to the
      //    block end) or past the window's last position (then a scan, below)
      bool bad = false;
      for (uint32_t k0 = 0; k0 < nRuns; k0 += kFindThreads) {
        const uint32_t k = k0 + tid;
        uint32_t r = 0, sFirst = 0, sNext = 0;
        if (k < nRuns) {
          r = C[ga + k];
          sFirst = T[ga + k];
          sNext = k + 1 < nRuns ? T[ga + k + 1] : gb;
        }
        __syncthreads();
        if (k < nRuns) {
          uint32_t tl = sNext - 1u;  // the piece's last member: the last run member before the next piece
          while (tl > sFirst && !is_run(tl)) tl--;
          const uint32_t lastRel = slot_pos(compact, small, tl);
          uint64_t e = S.w0 + lastRel + 4;
          uint32_t kind = 0, extra = 0;
          if ((src.ld4(e) & 0xFFu) == v) {
            if (S.w0 + lastRel + 1 == S.s1) {
              kind = 2;
              s_scanRun = k;  // at most one piece holds the window's last position
            } else {
              kind = 1;
              extra = lastRel - r;
              const int32_t j = iv_starting_at(S.w0 + lastRel + 1);
              if (j < 0 || extra > 63u) bad = true;
              else {
                e = s_ivA[j] + s_ivLa[j];
                while (e < B.end && (src.ld4(e) & 0xFFu) == v) e++;
              }
            }
          }
          if (e > B.end) e = B.end;
          C[ga + k] = r | ((e < B.end ? (src.ld4(e) & 0xFFu) : kAEnd) << 17);
          T[ga + k] = (uint32_t)(e - (S.w0 + r)) | (extra << 24) | (kind << 30);
        }
        __syncthreads();
      }
      if (bad) s_mixed = 1;
      SZ4_D6X(if (bad) SZ4_D6C(16, 1);)
      __threadfence_block();
      __syncthreads();
      //    the piece at the window's end: its run's end by wave 0, 256 bytes per step, jumping intervals
      if (s_scanRun != kNoScan && wave == 0) {
        const uint32_t k = s_scanRun;
        const uint32_t r = C[ga + k] & 0x1FFFFu;
        uint64_t e = S.s1 + 3;  // the window's last position is a member: its 4 bytes are v
        while (e < B.end) {
          const int32_t j = iv_starting_at(e);
          if (j >= 0) {
            e = s_ivA[j] + s_ivLa[j];
            continue;
          }
          const uint64_t q = e + 4ull * lane;
          const uint32_t x = q + 4 <= B.end ? src.ld4(q) ^ gKey : 0xFFFFFFFFu;
          const uint64_t mis = __ballot(x != 0u);
          if (mis) {
            const uint32_t f = (uint32_t)__builtin_ctzll(mis);
            const uint32_t xf = rdlane(x, f);
            const uint64_t qf = e + 4ull * f;
            e = qf + 4 <= B.end ? qf + ((uint32_t)__builtin_ctz(xf) >> 3) : qf;
            if (qf + 4 > B.end)
              while (e < B.end && (src.ld4(e) & 0xFFu) == v) e++;
            break;
          }
          e += 256;
        }
        if (e > B.end) e = B.end;
        if (lane == 0) {
          C[ga + k] = r | ((e < B.end ? (src.ld4(e) & 0xFFu) : kAEnd) << 17);
          T[ga + k] = (uint32_t)(e - (S.w0 + r)) | (2u << 30);
        }
      }
      __threadfence_block();
      __syncthreads();
      SZ4_D6(2);
      if (tid == 0) SZ4_D6C(12, nRuns);
      SZ4_D6X(if (tid == 0 && !s_mixed && nRuns > (uint32_t)(S.s1 - S.s0)) SZ4_D6C(18, 1);)
      if (!s_mixed && nRuns <= (uint32_t)(S.s1 - S.s0)) {  // (BK holds one word per target position of the segment)
      // with at most half as many pieces, BK's upper half maps a piece to its place in its bucket
      const bool invBk = 1 && nRuns <= nTg / 2;
      // B. buckets by next byte
      for (uint32_t k = tid; k < nRuns; k += kFindThreads) atomicAdd(&s_cur[0][C[ga + k] >> 17], 1u);
      __syncthreads();
      {
        const uint32_t c0 = tid <= kAEnd ? s_cur[0][tid] : 0u;
        const uint32_t o0 = block_excl_scan(c0, s_wsum, nullptr);
        if (tid <= kAEnd) {
          s_cls[tid] = o0;
          s_cur[0][tid] = o0;
        }
        if (tid == 0) {
          s_cls[kAEnd + 1] = nRuns;
          s_next = 0;
        }
      }
      __syncthreads();
      // (in piece order inside a bucket: one wavefront, 64 pieces at a time, one counter update per
      // distinct byte)
      if (wave == 0) {
        const uint64_t below = (1ull << lane) - 1ull;
        for (uint32_t k0 = 0; k0 < nRuns; k0 += 64) {
          const uint32_t k = k0 + lane;
          const uint32_t a = k < nRuns ? C[ga + k] >> 17 : 0xFFFFFFFFu;
          uint64_t rest = __ballot(k < nRuns);
          while (rest) {
            const uint32_t l = (uint32_t)__builtin_ctzll(rest);
            const uint32_t al = rdlane(a, l);
            const uint64_t m = __ballot(a == al);
            const uint32_t at = s_cur[0][al];
            if (a == al) {
              const uint32_t q = at + (uint32_t)__builtin_popcountll(m & below);
              BK[q] = k;
              if (invBk) BK[nTg / 2 + k] = q;  // the piece's place in its bucket
            }
            if (lane == 0) s_cur[0][al] = at + (uint32_t)__builtin_popcountll(m);
            rest &= ~m;
          }
        }
      }
      __threadfence_block();
      __syncthreads();
      // a piece's first, run end and last member (rel)
      auto piece = [&](uint32_t j, uint32_t& fj, uint32_t& ej, uint32_t& lj) {
        const uint32_t cj = C[ga + j], tj = T[ga + j];
        fj = cj & 0x1FFFFu;
        ej = fj + (tj & 0xFFFFFFu);
        const uint32_t kind = tj >> 30;
        lj = kind == 0 ? ej - 4u : kind == 1 ? fj + ((tj >> 24) & 63u) : (uint32_t)(S.s1 - 1 - S.w0);
      };
      SZ4_D6(3);
      // C. every target member, 64 slots per step
      const uint32_t nChunks = (gb - ga + 63) / 64;
      bool rmq = false;
      while (true) {
        uint32_t item = 0;
        if (lane == 0) item = atomicAdd(&s_next, 1u);
        item = rdlane(item, 0);
        if (item >= nChunks) break;
        const uint32_t s = ga + item * 64 + lane;
        const uint32_t pRel = s < gb ? slot_pos(compact, small, s) : 0u;
        const uint64_t p = S.w0 + pRel;
        const bool tgt = s < gb && is_target(p);
        const uint32_t pKey = tgt ? src.ld4(p) : 0u;
        const bool coll = tgt && pKey != gKey;  // a collision member: searched one by one, below
        const bool act = tgt && !coll;
        const uint32_t lo = tgt ? lm[p - matchBase] : 0u;  // its piece (a collision member: its list index)
        if (act) SZ4_D6C(8, 1);
        uint32_t fi = 0, eiRel = 0, li = 0;
        if (act) piece(lo, fi, eiRel, li);
        const uint32_t ai = act ? C[ga + lo] >> 17 : 0u;
        const uint64_t ei = S.w0 + eiRel;  // p's run ends here
        const uint32_t R = act ? eiRel - pRel : 0u;
        const uint32_t room = tgt ? (uint32_t)(stopAbs - p) : 0u;
        const uint32_t limit = room;  // exact lengths (no pass-1 cap; the result goes to mlen, u32)
        const uint32_t lbRel = p > S.w0 + kWindow ? (uint32_t)(p - kWindow - S.w0) : 0u;
        uint32_t bl = 0, bc = 0;  // best length, its candidate (rel)
        auto offer = [&](uint32_t l, uint32_t c) {
          if (l > bl || (l == bl && c > bc)) {
            bl = l;
            bc = c;
          }
        };
        // the pieces before p's that hold a position with exactly R bytes of v left (R(c) = R(p)), and
        // whose run is followed by the same byte: R bytes + the common prefix after the two runs
        //   (the bucket is in piece order: from p's own piece down, nearest first, to the window's start)
        auto same_r = [&](uint32_t Rp) {
          if (Rp >= limit || ai == kAEnd) return;
          const uint32_t b0 = s_cls[ai];
          uint32_t bLo = b0, bHi = s_cls[ai + 1];  // p's piece in it
          if (invBk) {
            bLo = BK[nTg / 2 + lo];
          } else {
            while (bLo < bHi) {
              const uint32_t mid = (bLo + bHi) >> 1;
              if (BK[mid] < lo) bLo = mid + 1;
              else bHi = mid;
            }
          }
          // the next piece index is loaded while this one's piece is read (clamped, unconditional)
          uint32_t jNext = BK[bLo > b0 ? bLo - 1u : b0];
          for (uint32_t b = bLo; b-- > b0;) {
            SZ4_D6C(9, 1);
            uint32_t j;
            asm volatile("v_mov_b32 %0, %1" : "=v"(j) : "v"(jNext));
            jNext = BK[b > b0 ? b - 1u : b0];
            uint32_t fj, ej, lj;
            piece(j, fj, ej, lj);
            if (lj < lbRel) break;     // it and every earlier piece lie below the window
            const uint32_t c = ej - Rp;  // its position with R(c) = Rp
            if (c < fj || c > lj || c < lbRel) continue;
            const uint32_t l = Rp + ext_len(S.w0 + ej, ei, limit - Rp);
            offer(l, c);
            if (l >= limit) break;  // the longest there is; the nearer ones came first
          }
        };
        SZ4_D6X(uint64_t w6 = __builtin_readcyclecounter();)
        auto W6 = [&](int k) {
          (void)k;
          SZ4_D6X(const uint64_t now = __builtin_readcyclecounter(); if (lane == 0) SZ4_D6C(k, now - w6); w6 = now;)
        };
        const uint32_t need = R < limit ? R : limit;
        int32_t wj = -1;       // a piece start's walk: next piece to look at when still open
        bool open = false;
        if (act && pRel > fi) {
          // interior (p-1 is a member of its piece): p-1 gives R bytes at distance 1; a candidate with
          // R(c) != R(p) has min(R(p), R(c)) in common, so only those with R(c) = R(p) can do better
          offer(need, pRel - 1u);
          same_r(R);
        } else if (act) {
          // piece start: the same, and the nearest piece holding a position with >= need bytes of v
          // left (lcp need), or failing any, the longest stretch the window holds
          same_r(R);
          wj = (int32_t)lo - 1;
          open = true;
          for (int it = 0; it < 16 && open; it++) {
            SZ4_D6C(10, 1);
            if (wj < 0) {
              open = false;
              break;
            }
            uint32_t fj, ej, lj;
            piece((uint32_t)wj, fj, ej, lj);
            if (lj < lbRel) {  // no member of this piece (or an earlier one) in the window
              open = false;
              break;
            }
            const uint32_t rHi = ej - (fj > lbRel ? fj : lbRel);
            if (rHi >= need) {
              offer(need, ej - need < lj ? ej - need : lj);
              open = false;
              break;
            }
            offer(rHi, ej - rHi);
            wj--;
          }
        }
        W6(21);
        // ... and the rare long walks by the whole wavefront, 64 pieces per step
        uint64_t pend = __ballot(open);
        while (pend) {
          const uint32_t t = (uint32_t)__builtin_ctzll(pend);
          pend &= pend - 1;
          int32_t jj = (int32_t)rdlane((uint32_t)wj, t);
          const uint32_t nd = rdlane(need, t), lb = rdlane(lbRel, t);
          uint64_t best = 0;  // len << 17 | candidate
          while (jj >= 0) {
            if (lane == 0) SZ4_D6C(11, 1);
            const int32_t k = jj - (int32_t)lane;
            const bool ok = k >= 0;
            uint32_t fj = 0, ej = 0, lj = 0;
            if (ok) piece((uint32_t)k, fj, ej, lj);
            const bool inW = ok && lj >= lb;
            const uint32_t rHi = inW ? ej - (fj > lb ? fj : lb) : 0u;
            const uint64_t hit = __ballot(inW && rHi >= nd);
            const uint64_t stop = hit | __ballot(!inW);
            const uint32_t f = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;  // nearest stop
            uint64_t key = 0;
            if (inW && lane < f) key = ((uint64_t)rHi << 17) | (ej - rHi);
            if (inW && lane == f && rHi >= nd) key = ((uint64_t)nd << 17) | (ej - nd < lj ? ej - nd : lj);
            key = wave_max_u64(key);
            best = key > best ? key : best;
            if (stop) break;
            jj -= 64;
          }
          if (lane == t) offer((uint32_t)(best >> 17), (uint32_t)(best & 0x1FFFFu));
        }
        W6(22);
        // collision members: the list entries of the same key below, by the whole wavefront
        uint64_t cm = __ballot(coll);
        while (cm) {
          const uint32_t t = (uint32_t)__builtin_ctzll(cm);
          cm &= cm - 1;
          if (lane == 0) SZ4_D6C(19, 1);
          const uint32_t jt = rdlane(lo, t), pr = rdlane(pRel, t), kt = rdlane(pKey, t);
          const uint32_t rm = rdlane(room, t), lb = rdlane(lbRel, t);
          uint64_t best = 0;
          for (uint32_t b0 = 0; b0 < jt; b0 += 64) {  // the list entries below it
            if (lane == 0) SZ4_D6C(20, 1);
            const uint32_t j = b0 + lane;
            const uint32_t cr = j < jt ? C[gb - 1u - j] : 0u;
            uint32_t l = 0;
            if (j < jt && cr >= lb && src.ld4(S.w0 + cr) == kt) {
              l = 4;
              while (l < rm) {
                const uint32_t x = src.ld4(S.w0 + pr + l) ^ src.ld4(S.w0 + cr + l);
                if (x) {
                  l += (uint32_t)__builtin_ctz(x) >> 3;
                  break;
                }
                l += 4;
              }
              l = l < rm ? l : rm;
            }
            const uint64_t key = l ? ((uint64_t)l << 17) | cr : 0ull;
            const uint64_t wm = wave_max_u64(key);
            best = wm > best ? wm : best;
          }
          if (lane == t) offer((uint32_t)(best >> 17), (uint32_t)(best & 0x1FFFFu));
        }
        W6(23);
        if (tgt) {
          // final: pass 1 and the prefix maximum below read it as an exact target
          const uint64_t idx = p - matchBase;
          const bool m = bl >= (uint32_t)kMinMatch;
          mlen[idx] = m ? bl : 0u;
          mdist[idx] = m ? (uint16_t)(pRel - bc) : (uint16_t)0;
          rmq |= m && bl >= kRmqLen && !(pRel - bc == 1u && bl >= kSameLetter);
        }
        wave_clear_bits(longBits, p - matchBase, tgt);
      }
      if (__ballot(rmq) && lane == 0) atomicOr(&longFlag[S.block], kFlagRmq);
      __syncthreads();
      SZ4_D6(5);
      continue;
      }
    }

    // ---- any other group: regrouped by class
    if (tid == 0) SZ4_D6C(13, 1);
    for (uint32_t k = tid; k < 2 * kBins; k += kFindThreads) (&s_cur[0][0])[k] = 0;
    __syncthreads();
    // counts per class (candidates: the whole group; targets: pass 1's big ones)
    for (uint32_t s = ga + tid; s < gb; s += kFindThreads) {
      const uint32_t r = slot_pos(compact, small, s);
      const uint64_t q = S.w0 + r;
      const uint32_t c = cls_of(q);
      atomicAdd(&s_cur[0][c], 1u);
      if (is_target(q)) atomicAdd(&s_cur[1][c], 1u);
    }
    __syncthreads();
    {
      uint32_t tc = 0, tt = 0;
      const uint32_t c0 = tid < kBins ? s_cur[0][tid] : 0u, c1 = tid < kBins ? s_cur[1][tid] : 0u;
      const uint32_t o0 = block_excl_scan(c0, s_wsum, &tc);
      const uint32_t o1 = block_excl_scan(c1, s_wsum, &tt);
      if (tid < kBins) {
        s_cls[tid] = o0;
        s_tcls[tid] = o1;
        s_cur[0][tid] = o0;
        s_cur[1][tid] = o1;
      }
      if (tid == 0) {
        s_cls[kBins] = tc;
        s_tcls[kBins] = tt;
        s_next = 0;
      }
    }
    __syncthreads();
    for (uint32_t s = ga + tid; s < gb; s += kFindThreads) {
      const uint32_t r = slot_pos(compact, small, s);
      const uint64_t q = S.w0 + r;
      const uint32_t c = cls_of(q);
      C[ga + atomicAdd(&s_cur[0][c], 1u)] = (c << 17) | r;
      if (is_target(q)) T[ga + atomicAdd(&s_cur[1][c], 1u)] = r;
    }
    __threadfence_block();
    __syncthreads();

    // 2. LM of every big target: chunks of up to 64 targets, taken class by class; a class's last,
    //    partial chunk is filled up with the next classes' first targets (mixed: scan all, filter)
    const uint32_t nT = s_tcls[kBins];
    const uint32_t nChunks = (nT + 63) / 64;
    while (true) {
      uint32_t item = 0;
      if (lane == 0) item = atomicAdd(&s_next, 1u);
      item = rdlane(item, 0);
      if (item >= nChunks) break;
      const uint32_t t = item * 64 + lane;
      const bool act = t < nT;
      const uint32_t pRel = act ? T[ga + t] : 0u;
      const uint64_t p = S.w0 + pRel;
      const uint32_t myCls = act ? cls_of(p) : kClsNone + 1;
      // p's own class is excluded only when p-1 is a target of this block (its result carries to p)
      const uint32_t exCls = act && p > B.start && myCls < kClsNone ? myCls : kClsNone + 1;
      const uint32_t me0 = act ? src.ld4(p) : 0u, me1 = act ? src.ld4(p + 4) : 0u, me2 = act ? src.ld4(p + 8) : 0u;
      const uint32_t room = act ? (uint32_t)(stopAbs - p) : 0u;
      const uint32_t limit = room < kLongCap9 ? room : kLongCap9;
      const uint32_t cap12 = limit < 12u ? limit : 12u;
      const uint32_t lbRel = p > S.w0 + kWindow ? (uint32_t)(p - kWindow - S.w0) : 0u;
      // candidate ranges of C: one class for the whole wavefront -> skip it; else scan everything
      const uint32_t e0 = rdlane(exCls, 0);
      const bool one = __ballot(act && exCls != e0) == 0 && e0 < kClsNone;
      uint32_t r0a = ga, r0b = gb, r1a = gb, r1b = gb;
      if (one) {
        r0b = ga + s_cls[e0];
        r1a = ga + s_cls[e0 + 1];
      }
      uint32_t bestKey = 0;
      // candidates arrive in no particular order (class by class), so the filter lets through those that
      // reach the current best length (ties are decided by position in the key), all 12 bytes once the
      // best has 12 or the cap
      uint32_t m1 = 0, m2 = 0;
      auto setMasksBig = [&]() {
        const uint32_t len = bestKey >> 17;
        const uint32_t bits = len >= cap12 ? 64u : len > 4u ? 8u * (len - 4u) : 0u;
        const uint64_t mk = bits >= 64u ? ~0ull : (1ull << bits) - 1ull;
        m1 = (uint32_t)mk;
        m2 = (uint32_t)(mk >> 32);
      };
      {
        // both candidate ranges as one sequence, 64 per step; the next step's entries of C are loaded
        // while this step's are scanned (unconditionally, at a clamped index: a load under a branch would
        // be waited for at once)
        const uint32_t len0 = r0b - r0a, tot = len0 + (r1b - r1a);
        auto cidx = [&](uint32_t j) -> uint32_t {
          const uint32_t jj = j < tot ? j : (tot ? tot - 1u : 0u);
          return jj < len0 ? r0a + jj : r1a + (jj - len0);
        };
        uint32_t ceNext = tot ? C[cidx(lane)] : 0u;
        for (uint32_t base = 0; base < tot; base += 64) {
          uint32_t ce;
          asm volatile("v_mov_b32 %0, %1" : "=v"(ce) : "v"(ceNext));
          ceNext = C[cidx(base + 64u + lane)];
          const bool inR = base + lane < tot;
          ce = inR ? ce : 0xFFFFFFFFu;
          const uint32_t cr = ce & 0x1FFFFu;
          const uint64_t cp = S.w0 + (inR ? cr : 0u);
          const uint32_t f0 = src.ld4(cp), f1 = src.ld4(cp + 4), f2 = src.ld4(cp + 8);
          const uint32_t n = tot - base < 64u ? tot - base : 64u;
          // 16 candidates per register, every row a copy; step K takes candidate q0 + K to every lane by DPP
          // row_newbcast:K (VGPR operands only), the exact prefix only when the filter lets it through
          for (uint32_t q0 = 0; q0 < n; q0 += 16) {
            const int sl = (int)((q0 + (lane & 15u)) << 2);
            const uint32_t gce = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)ce);
            const uint32_t g0 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)f0);
            const uint32_t g1 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)f1);
            const uint32_t g2 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)f2);
            const uint32_t cnt = n - q0 < 16u ? n - q0 : 16u;
            setMasksBig();
#define SZ4_BIGSTEP(K)                                                                                          \
            if ((K) < cnt) {                                                                                    \
              const uint32_t ej = (uint32_t)__builtin_amdgcn_mov_dpp((int)gce, 0x150 + (K), 0xF, 0xF, true);    \
              const uint32_t x0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g0, 0x150 + (K), 0xF, 0xF, true) ^ me0; \
              const uint32_t x1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g1, 0x150 + (K), 0xF, 0xF, true) ^ me1; \
              const uint32_t x2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)g2, 0x150 + (K), 0xF, 0xF, true) ^ me2; \
              const uint32_t c = ej & 0x1FFFFu;                                                                 \
              const bool ok = act && c < pRel && c >= lbRel && (ej >> 17) != exCls;                             \
              if (__ballot(ok && (x0 | (x1 & m1) | (x2 & m2)) == 0u)) {                                         \
                const uint32_t z = min(ffbl(x1), 32u + min(ffbl(x2), 32u));                                     \
                uint32_t lcp = min(4u + (z >> 3), cap12);                                                       \
                if (ok && x0 == 0u && lcp == 12u && limit > 12u) {                                              \
                  const uint64_t cc = S.w0 + c;                                                                 \
                  const uint32_t bl = bestKey >> 17;                                                            \
                  bool open = !(bl > 12u && src.ld4(p + bl - 4u) != src.ld4(cc + bl - 4u));                     \
                  while (open && lcp < limit) {                                                                 \
                    const uint32_t x = src.ld4(p + lcp) ^ src.ld4(cc + lcp);                                    \
                    if (x) {                                                                                    \
                      lcp += (uint32_t)__builtin_ctz(x) >> 3;                                                   \
                      open = false;                                                                             \
                    } else {                                                                                    \
                      lcp += 4;                                                                                 \
                    }                                                                                           \
                  }                                                                                             \
                  if (lcp > limit) lcp = limit;                                                                 \
                }                                                                                               \
                const uint32_t key = ok && x0 == 0u ? (lcp << 17) | c : 0u;                                     \
                bestKey = key > bestKey ? key : bestKey;                                                        \
                setMasksBig();                                                                                  \
              }                                                                                                 \
            }
            SZ4_BIGSTEP(0) SZ4_BIGSTEP(1) SZ4_BIGSTEP(2) SZ4_BIGSTEP(3) SZ4_BIGSTEP(4) SZ4_BIGSTEP(5)
            SZ4_BIGSTEP(6) SZ4_BIGSTEP(7) SZ4_BIGSTEP(8) SZ4_BIGSTEP(9) SZ4_BIGSTEP(10) SZ4_BIGSTEP(11)
            SZ4_BIGSTEP(12) SZ4_BIGSTEP(13) SZ4_BIGSTEP(14) SZ4_BIGSTEP(15)
#undef SZ4_BIGSTEP
          }
        }
      }
      if (act) {
        const uint32_t bl = bestKey >> 17;
        lm[p - matchBase] = bl >= kLongCap9 && room > kLongCap9 ? kLmUnknown << 16
                            : bl >= (uint32_t)kMinMatch ? (bl << 16) | (uint32_t)(pRel - (bestKey & 0x1FFFFu)) : 0u;
      }
    }
    __syncthreads();
    SZ4_D6(7);
  }
  }
  __threadfence_block();
  __syncthreads();

  SZ4_D6(4);
  // 3. prefix maximum in text order.  Per target: E (exact: pass 1 finished it) resets the state to
  //    its own key, U (unknown: a pass-1 long match, or LM at the cap) invalidates it, B (big) takes
  //    the maximum of the state and its LM.  16 wavefronts take consecutive ranges; a range's carry-in
  //    comes from the ranges before it (phase 0 summarises, phase 1 resolves).
  const uint32_t waves = kFindThreads / 64;
  const uint32_t span = ((nTg + waves - 1) / waves + 63) / 64 * 64;
  const uint32_t r0 = wave * span, r1 = r0 + span < nTg ? r0 + span : nTg;
  auto classify = [&](uint32_t i, uint32_t& kind, uint64_t& key) {
    // kind 0 = B, 1 = E, 2 = U
    const uint64_t p = S.s0 + i, idx = p - matchBase;
    const uint32_t ml = mlen[idx], md = mdist[idx];
    key = 0;
    if (ml != kLongMatch) {
      kind = 1;
      if (ml >= (uint32_t)kMinMatch) key = ((uint64_t)(i + ml) << 16) | (0xFFFFu - md);
      return;
    }
    const bool bit = (longBits[idx >> 5] >> (idx & 31)) & 1u;
    if (!bit || md != 0u) {
      kind = 2;
      return;
    }
    const uint32_t v = lm[idx];
    const uint32_t vl = v >> 16;
    if (vl == kLmUnknown) {
      kind = 2;
      return;
    }
    kind = 0;
    if (vl >= (uint32_t)kMinMatch) key = ((uint64_t)(i + vl) << 16) | (0xFFFFu - (v & 0xFFFFu));
  };
  // inclusive segmented scan over the wavefront; returns (head seen, valid, key) per lane
  auto scan = [&](uint32_t kind, uint64_t key, bool inRange, bool& head, bool& valid) -> uint64_t {
    head = inRange && kind != 0u;
    valid = kind == 1u;
    uint64_t v = inRange ? key : 0ull;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t vo = __shfl_up(v, d, 64);
      const bool ho = __shfl_up((int)head, d, 64) != 0, va = __shfl_up((int)valid, d, 64) != 0;
      if (lane >= (uint32_t)d && !head) {
        v = vo > v ? vo : v;
        valid = va;
        head = ho;
      }
    }
    return v;
  };
  for (int phase = 0; phase < 2; phase++) {
    bool cValid = false;
    uint64_t cKey = 0;
    if (phase == 1) {
      // carry-in: the block's first target has no predecessor (exact state, nothing to carry); a later
      // segment's first target takes its predecessor's result once that is final (not marked)
      cValid = S.s0 == B.start;
      if (!cValid && resolveOnly && blockIdx.x > 0 && segs[blockIdx.x - 1].block == S.block) {
        // the resolve launch: the state after the predecessor segment's last target, as the first
        // launch left it (final then: no launch writes it afterwards)
        const uint64_t t = segTail[blockIdx.x - 1];
        cValid = (t >> 63) != 0u;
        cKey = t & ~(1ull << 63);
      }
      for (uint32_t w = 0; w < wave; w++) {
        if (s_hasHead[w]) {
          cValid = s_outValid[w] != 0u;
          cKey = s_outKey[w];
        } else {
          cKey = s_outKey[w] > cKey ? s_outKey[w] : cKey;
        }
      }
    }
    bool anyHead = false;
    for (uint32_t i0 = r0; i0 < r1; i0 += 64) {
      const uint32_t i = i0 + lane;
      const bool inR = i < r1;
      uint32_t kind = 2;
      uint64_t key = 0;
      if (inR) classify(i, kind, key);
      bool head, valid;
      uint64_t v = scan(kind, key, inR, head, valid);
      if (!head) {
        v = cKey > v ? cKey : v;
        valid = cValid;
      }
      anyHead |= __ballot(inR && kind != 0u) != 0;
      bool rmq = false;
      SZ4_D6X(
      if (phase == 1 && resolveOnly) {
        const uint32_t nb = (uint32_t)__builtin_popcountll(__ballot(inR && kind == 0u && !valid));
        if (lane == 0 && nb) SZ4_D6C(26, nb);
        const uint32_t nu = (uint32_t)__builtin_popcountll(__ballot(inR && kind == 2u));
        if (lane == 0 && nu) SZ4_D6C(27, nu);
      }
      )
      if (phase == 1 && inR && kind == 0u && valid) {
        const uint64_t p = S.s0 + i, idx = p - matchBase;
        const uint32_t len = (uint32_t)(v >> 16) > i ? (uint32_t)(v >> 16) - i : 0u;
        const bool m = v != 0ull && len >= (uint32_t)kMinMatch;
        const uint32_t d = 0xFFFFu - (uint32_t)(v & 0xFFFFu);
        mlen[idx] = m ? len : 0u;
        mdist[idx] = m ? (uint16_t)d : (uint16_t)0;
        rmq = m && len >= kRmqLen && !(d == 1u && len >= kSameLetter);  // (a run target's exact length)
      }
      wave_clear_bits(longBits, S.s0 + i - matchBase, phase == 1 && inR && kind == 0u && valid);
      if (__ballot(rmq) && lane == 0) atomicOr(&longFlag[S.block], kFlagRmq);
      // carry to the next 64: the last lane in range
      const uint32_t last = (r1 - i0 < 64u ? r1 - i0 : 64u) - 1u;
      cKey = ((uint64_t)rdlane((uint32_t)(v >> 32), last) << 32) | rdlane((uint32_t)v, last);
      cValid = rdlane(valid ? 1u : 0u, last) != 0u;
    }
    if (phase == 0 && lane == 0) {
      // summary with carry-in "nothing": valid/key after the range, or (no head) the max of its B keys
      s_hasHead[wave] = anyHead ? 1u : 0u;
      s_outValid[wave] = cValid ? 1u : 0u;
      s_outKey[wave] = cKey;
    }
    if (phase == 1 && !resolveOnly && lane == 0 && r1 == nTg && r0 < r1) {
      // the state after the segment's last target, as a carry into the next segment (its s0 is our s1):
      // ends E = i + len are relative to our s0, so the next segment's are E - nTg
      const uint64_t e = cKey >> 16;
      const uint64_t k = e > (uint64_t)nTg + kMinMatch - 1u ? ((e - nTg) << 16) | (cKey & 0xFFFFu) : 0ull;
      segTail[blockIdx.x] = cValid ? (1ull << 63) | k : 0ull;
    }
    __syncthreads();
  }
}

// ================================================================================================
// The parse, after the matches are known.
//   k_prep    one wavefront per block: clears the positions the reference never searched (the
//             greedy/lazy skip bookkeeping runs before it in k_lazy_*, smallz4.h:726-744);
//   k_dp_spec one wavefront per DpSeg: the backward optimal parse (estimateCosts,
//             smallz4.h:376-472) of B.dpSize positions.  The top segment of a block starts from the
//             block end exactly; every other segment starts from a guessed boundary (costs 0 above
//             it).  Also writes reach[i] = max(q + len[q]) over the segment's positions q < i.
//   k_dp_fix  one wavefront per block: walks the segment boundaries top-down.  Segment k is parsed
//             again from the true state above it until the exact and the speculative parse agree:
//             both choose a match at i (so the literal counters agree) and exact - speculative
//             costs are one constant over every position [i, reach[i]] the rest of the segment can
//             reference.  Choices depend on cost differences only, so below i the speculative
//             choices are the exact ones and exact costs are speculative costs + that constant.
// Costs of recent positions sit in a register window (lane j & 63 holds cost[j]) and an LDS ring;
// older ones are read back from HBM.
// ================================================================================================
constexpr int kRing = 1024;

__device__ __forceinline__ uint32_t len_extra(uint32_t len)
{
  return len < 19 ? 3u : 4u + (len - 19) / 255;
}

// ------------------------------------------------------------------------------------------------
// Long lengths of the optimal parse.  A position with match length Lk > 64 takes
//   min over l in (64, Lk] of cost[i + l] + extra(l),  ties to the longest,
// with extra(l) = 4 + (l - 19) / 255, constant on pieces l in [19 + 255k, 273 + 255k].  The reference
// scans every l (smallz4.h:421-448); here:
//   A  l in [65, 273]: one wavefront step, four consecutive lengths per lane;
//   B  pieces k >= 1: a piece is a window of 255 positions, so it spans at most two 256-position
//      "rmq blocks" (aligned on the block's last parsed position `top`), and its minimum is
//      min(UP[a], DOWN[b]): UP[j] = min key over [j, top of j's rmq block], DOWN[j] = min key over
//      [bottom of j's rmq block, j], key = cost << 8 | (top - j) & 255 (ties: highest position).
//      One lane per piece;
//   C  a last partial piece inside one rmq block and aligned to neither end: scanned directly.
// Positions above `above` cost 0 (the guess above a speculative segment; the block tail).
// UP/DOWN exist only for blocks whose matches reach 274 bytes (longFlag, set by k_find); without
// them the pieces are scanned (never taken when the flag is right).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rmq_key(uint32_t cost, int32_t top, int32_t j)
{
  return (cost << 8) | ((uint32_t)(top - j) & 255u);
}

// inclusive min-scan over the wavefront by DPP: row shifts 1, 2, 4, 8, then lane 15 of each row into the
// next and lane 31 into rows 2-3 (lanes without a source take the identity) -- six dependent VALU steps
// instead of six ds_bpermute round trips (the parse's range-minimum stores are latency-exposed)
__device__ __forceinline__ uint32_t wave_incl_scan_min(uint32_t v)
{
  constexpr int kId = (int)0xFFFFFFFFu;
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)v, kRowShr + 1, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)v, kRowShr + 2, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)v, kRowShr + 4, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)v, kRowShr + 8, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)v, kRowBcast15, 0xA, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(kId, (int)v, kRowBcast31, 0xC, 0xF, false));
  return v;
}

// UP of the chunk [hi - cnt + 1, hi] (lane t = position hi - t, key kt).  The chunk lies inside one
// rmq block; upCarry = UP[hi + 1] when hi + 1 is in the same block.
__device__ __forceinline__ void rmq_store_up(uint32_t* up, int32_t top, int32_t hi, uint32_t cnt, uint32_t kt,
                                             uint32_t& upCarry)
{
  const uint32_t lane = lane_id();
  const bool blockTop = ((uint32_t)(top - hi) & 255u) == 0u;
  uint32_t v = wave_incl_scan_min(lane < cnt ? kt : 0xFFFFFFFFu);
  if (!blockTop) v = min(v, upCarry);
  if (lane < cnt) up[hi - (int32_t)lane] = v;
  upCarry = rdlane(v, 63);
}

// top of the rmq block holding position j
__device__ __forceinline__ int32_t rmq_block_top(int32_t top, int32_t j)
{
  return top - (int32_t)(((uint32_t)(top - j) >> 8) << 8);
}

// DOWN of the rmq block [jb, its top] (every position final); cost_of(j) is the exact cost
template <class CostOf>
__device__ __forceinline__ void rmq_store_down(uint32_t* down, int32_t top, int32_t jb, CostOf cost_of)
{
  const uint32_t lane = lane_id();
  const int32_t jt = rmq_block_top(top, jb);
  uint32_t carry = 0xFFFFFFFFu;
  for (int32_t j0 = jb; j0 <= jt; j0 += 64) {
    const int32_t j = j0 + (int32_t)lane;
    uint32_t v = j <= jt ? rmq_key(cost_of(j), top, j) : 0xFFFFFFFFu;
    v = min(wave_incl_scan_min(v), carry);
    if (j <= jt) down[j] = v;
    carry = rdlane(v, 63);
  }
}

// UP of a whole rmq block [jb, jt]
template <class CostOf>
__device__ __forceinline__ void rmq_store_up_block(uint32_t* up, int32_t top, int32_t jb, int32_t jt, CostOf cost_of)
{
  const uint32_t lane = lane_id();
  uint32_t carry = 0xFFFFFFFFu;
  for (int32_t j0 = jt; j0 >= jb; j0 -= 64) {
    const int32_t j = j0 - (int32_t)lane;
    uint32_t v = j >= jb ? rmq_key(cost_of(j), top, j) : 0xFFFFFFFFu;
    v = min(wave_incl_scan_min(v), carry);
    if (j >= jb) up[j] = v;
    carry = rdlane(v, 63);
  }
}

// minimum of cost_at(i + l) + extra over l in [l0, l1] (l1 - l0 < 256), four lengths per lane,
// folded into (minCost, best) with ties to the longest
template <class CostAt>
__device__ __forceinline__ void scan_lengths(int32_t i, uint32_t l0, uint32_t l1, uint32_t extra, int32_t above,
                                             CostAt cost_at, uint32_t& minCost, uint32_t& best)
{
  const uint32_t lane = lane_id();
  uint32_t c = 0xFFFFFFFFu, lb = 0;
#pragma unroll
  for (uint32_t u = 0; u < 4; u++) {
    const uint32_t l = l0 + 4u * lane + u;
    if (l <= l1) {
      const int32_t j = i + (int32_t)l;
      const uint32_t cj = j > above ? 0u : cost_at(j);
      if (cj <= c) {
        c = cj;
        lb = l;
      }
    }
  }
  const uint32_t key = c == 0xFFFFFFFFu ? 0xFFFFFFFFu : ((c + extra) << 8) | (255u - lane);
  const uint32_t km = wave_min_fast(key);
  if (km != 0xFFFFFFFFu && (km >> 8) <= minCost) {
    minCost = km >> 8;
    best = rdlane(lb, 255u - (km & 255u));
  }
}

// cost_at(j): exact cost of a position j in (i, above]; key_cost(j, key): exact cost encoded by an
// UP/DOWN key stored at position j.  Folds lengths 65 .. Lk into (minCost, best).
template <class CostAt, class KeyCost>
__device__ __forceinline__ void long_lengths(int32_t i, uint32_t Lk, int32_t top, int32_t above, bool rmq,
                                             const uint32_t* up, const uint32_t* down, CostAt cost_at,
                                             KeyCost key_cost, uint32_t& minCost, uint32_t& best)
{
  const uint32_t lane = lane_id();
  // A: lengths 65 .. 273 (piece 0)
  scan_lengths(i, 65u, Lk < 273u ? Lk : 273u, 4u, above, cost_at, minCost, best);
  if (Lk < kRmqLen) return;
  const uint32_t K = (Lk - 19u) / 255u;  // pieces 1 .. K
  if (!rmq) {
    for (uint32_t k = 1; k <= K; k++) {
      const uint32_t l0 = 19u + 255u * k, l1 = 273u + 255u * k < Lk ? 273u + 255u * k : Lk;
      scan_lengths(i, l0, l1, 4u + k, above, cost_at, minCost, best);
    }
    return;
  }
  // B: lane t takes piece kb + t
  bool direct = false;  // the last piece needs part C
  for (uint32_t kb = 1; kb <= K; kb += 64) {
    const uint32_t k = kb + lane;
    uint32_t key = 0xFFFFFFFFu, lsel = 0;
    if (k <= K) {
      const uint32_t la = 19u + 255u * k, lbnd = 273u + 255u * k < Lk ? 273u + 255u * k : Lk;
      const int32_t a = i + (int32_t)la, b = i + (int32_t)lbnd;
      uint32_t c = 0xFFFFFFFFu;
      if (b > above) {
        c = 0;  // zero costs above: the longest length of the piece
        lsel = lbnd;
      } else {
        const uint32_t ra = (uint32_t)(top - a), rb = (uint32_t)(top - b);
        const bool sameBlock = (ra >> 8) == (rb >> 8);
        const bool useUp = !sameBlock || (rb & 255u) == 0u;      // [a, top of a's block] inside the piece
        const bool useDown = !sameBlock || (ra & 255u) == 255u;  // [bottom of b's block, b] inside it
        if (!useUp && !useDown) {
          direct = true;  // only the last piece can be this short
        } else {
          uint32_t cu = 0xFFFFFFFFu, cd = 0xFFFFFFFFu;
          int32_t ju = 0, jd = 0;
          if (useUp) {
            const uint32_t kU = ld_fresh(&up[a]);
            ju = top - (int32_t)(((ra >> 8) << 8) + (kU & 255u));
            cu = key_cost(a, kU);
          }
          if (useDown) {
            const uint32_t kD = ld_fresh(&down[b]);
            jd = top - (int32_t)(((rb >> 8) << 8) + (kD & 255u));
            cd = key_cost(b, kD);
          }
          // the DOWN side holds the higher positions: it wins ties
          if (cd <= cu) {
            c = cd;
            lsel = (uint32_t)(jd - i);
          } else {
            c = cu;
            lsel = (uint32_t)(ju - i);
          }
        }
      }
      if (c != 0xFFFFFFFFu) key = ((c + 4u + k) << 8) | (255u - lane);
    }
    const uint32_t km = wave_min_fast(key);
    if (km != 0xFFFFFFFFu && (km >> 8) <= minCost) {
      minCost = km >> 8;
      best = rdlane(lsel, 255u - (km & 255u));
    }
  }
  // C: the last piece, scanned
  if (__ballot(direct)) scan_lengths(i, 19u + 255u * K, Lk, 4u + K, above, cost_at, minCost, best);
}

// ------------------------------------------------------------------------------------------------
// Long carried matches.  Along a repeat, consecutive positions share the end E = i + Lk of their
// match (a run of zeros: every position).  Since extra(a) + extra(b) >= extra(a + b) + 2 for any
// a >= 4, b >= 1 (extra(x) = 3 for x < 19), if every j in (i, E) has
//     cost[j] - extra(E - j) >= cost[E] - 2                                   (margin test)
// then every length l < Lk costs cost[i+l] + extra(l) >= cost[E] + extra(E - i): the full length is
// optimal among the matches (and wins ties, being the longest).  With costs flat above a speculative
// segment (the guess 0), E is the first position above it and the best length is the longest one of
// extra(E - i).  The running minimum `margin` of cost[j] - extra(E - j) is kept per position; it is
// established once per chain with range minima (end_margin), so a chain costs O(1) per position.
// ------------------------------------------------------------------------------------------------
constexpr int32_t kMarginBias = 1 << 30;

// minimum cost over [a, b] (b - a < 255) from UP/DOWN, or 0xFFFFFFFF when the range lies inside one
// rmq block aligned to neither end (the caller scans it)
template <class KeyCost>
__device__ __forceinline__ uint32_t rmq_range_cost(int32_t a, int32_t b, int32_t top, const uint32_t* up,
                                                   const uint32_t* down, KeyCost key_cost)
{
  const uint32_t ra = (uint32_t)(top - a), rb = (uint32_t)(top - b);
  const bool sameBlock = (ra >> 8) == (rb >> 8);
  const bool useUp = !sameBlock || (rb & 255u) == 0u;
  const bool useDown = !sameBlock || (ra & 255u) == 255u;
  if (!useUp && !useDown) return 0xFFFFFFFFu;
  uint32_t c = 0xFFFFFFFFu;
  if (useUp) c = key_cost(a, ld_fresh(&up[a]));
  if (useDown) {
    const uint32_t cd = key_cost(b, ld_fresh(&down[b]));
    c = cd < c ? cd : c;
  }
  return c;
}

// min over j in [i + 1, E - 1] of cost[j] - extra(E - j), + kMarginBias (wave-uniform)
template <class CostAt, class KeyCost>
__device__ __forceinline__ uint32_t end_margin(int32_t i, int32_t E, int32_t top, const uint32_t* up,
                                               const uint32_t* down, CostAt cost_at, KeyCost key_cost)
{
  const uint32_t lane = lane_id();
  uint32_t m = 0xFFFFFFFFu;
  // distances 1 .. 273 from E (pieces of extra 3 and 4): scanned, five per lane
#pragma unroll
  for (uint32_t u = 0; u < 5; u++) {
    const uint32_t D = 1u + 5u * lane + u;
    const int32_t j = E - (int32_t)D;
    if (D <= 273u && j > i) {
      const uint32_t v = cost_at(j) + kMarginBias - len_extra(D);
      m = v < m ? v : m;
    }
  }
  const uint32_t Dmax = (uint32_t)(E - i - 1);
  if (Dmax >= kRmqLen) {
    const uint32_t K = (Dmax - 19u) / 255u;  // pieces 1 .. K (the last one clipped at i + 1)
    bool direct = false;
    for (uint32_t kb = 1; kb <= K; kb += 64) {
      const uint32_t k = kb + lane;
      if (k <= K) {
        const int32_t b = E - 19 - 255 * (int32_t)k;
        const int32_t a0 = E - 273 - 255 * (int32_t)k;
        const int32_t a = a0 > i + 1 ? a0 : i + 1;
        const uint32_t c = rmq_range_cost(a, b, top, up, down, key_cost);
        if (c == 0xFFFFFFFFu) {
          direct = true;
        } else {
          const uint32_t v = c + kMarginBias - (4u + k);
          m = v < m ? v : m;
        }
      }
    }
    if (__ballot(direct)) {
      const int32_t b = E - 19 - 255 * (int32_t)K;
      const int32_t a0 = E - 273 - 255 * (int32_t)K;
      const int32_t a = a0 > i + 1 ? a0 : i + 1;
#pragma unroll
      for (int32_t u = 0; u < 4; u++) {
        const int32_t j = a + 4 * (int32_t)lane + u;
        if (j <= b) {
          const uint32_t v = cost_at(j) + kMarginBias - (4u + K);
          m = v < m ? v : m;
        }
      }
    }
  }
  return wave_min_fast(m);
}

// longest length with extra(len) == extra(x)
__device__ __forceinline__ uint32_t piece_end(uint32_t x)
{
  return x < 19u ? 18u : 273u + 255u * ((x - 19u) / 255u);
}

// chain state of the carried-match shortcut (wave-uniform)
// A chain is established at the first long position whose end differs (pending) and becomes valid at
// the chunk flush, once every position above the next one is stored with its UP/DOWN keys.
struct RunEnd {
  int32_t E = -1;
  uint32_t costE = 0;
  uint32_t margin = 0;  // + kMarginBias
  bool valid = false;
  bool pending = false;
  __device__ __forceinline__ void add(int32_t j, uint32_t c)
  {
    if (!valid) return;
    const uint32_t v = c + kMarginBias - len_extra((uint32_t)(E - j));
    margin = v < margin ? v : margin;
  }
};

// ================================================================================================
// k_dict_matches: dictionary mode (smallz4.h:541-760 with a dictionary).  The reference writes chain
// entries at block-relative slots (smallz4.h:656) but reads them at absolute ones (smallz4.h:190, 200,
// 694); with a dictionary every block starts at 65535 mod 65536, so a read finds the neighbour's
// entry and the chains are no longer same-key runs: the candidates follow a
// pointer chase the sorted-group model cannot express.  One wavefront replays the reference's loop
// exactly -- insertions in order, the chain walks, the same-letter shortcut and the greedy/lazy skip
// -- and writes the same match arrays the data-parallel finders write; the parse and the frame
// assembly then run as for any stream.  Sequential by nature (and slow): this mode exists for parity.
// Staged coordinates are the reference's data coordinates: a 65535-byte prefix (dictionary tail,
// zero-padded in front), then the input.
// ================================================================================================
constexpr uint32_t kNoPos = 0xFFFFFFFFu;

__global__ __launch_bounds__(64) void k_dict_matches(const uint8_t* __restrict__ in, const Block* __restrict__ blocks,
                                                     uint32_t nblocks, uint32_t maxChain, uint32_t dictBack, int legacy,
                                                     uint32_t* __restrict__ last, uint16_t* __restrict__ prevH,
                                                     uint16_t* __restrict__ prevXg, uint32_t cont, uint32_t shift,
                                                     uint32_t low0, uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist,
                                                     uint32_t* __restrict__ sel, uint32_t* __restrict__ longFlag)
{
  __shared__ uint16_t prevX[65536];
  const uint32_t lane = threadIdx.x;
  auto reset = [&]() {
    for (uint32_t j = lane; j < 65536; j += 64) {
      prevX[j] = 0;
      prevH[j] = 0;
    }
    for (uint32_t j = lane; j < (1u << kHashBits); j += 64) last[j] = kNoPos;
  };
  if (!cont) {
    reset();
  } else {
    // the previous chunk's tables: chain slots are absolute positions mod 65536, unchanged by a shift
    // that is a multiple of 65536; positions that fall below the carried bytes become "no entry" (the
    // reference finds them more than MaxDistance away)
    for (uint32_t j = lane; j < 65536; j += 64) prevX[j] = prevXg[j];
    for (uint32_t j = lane; j < (1u << kHashBits); j += 64) {
      const uint32_t v = last[j];
      last[j] = (v == kNoPos || v < shift) ? kNoPos : v - shift;
    }
  }
  for (uint32_t b = 0; b < nblocks; b++) {
    const Block B = blocks[b];
    for (uint64_t i = B.start + lane; i < B.end; i += 64) {
      mlen[i] = 0;
      mdist[i] = 0;
      if (maxChain > (uint32_t)kGreedyMax && i + kTailLiterals >= B.end) sel[i] = 0;
    }
  }
  __threadfence_block();
  __syncthreads();
  if (lane != 0) return;

  const bool greedy = maxChain <= (uint32_t)kGreedyMax, lazy = !greedy && maxChain <= (uint32_t)kLazyMax;
  uint64_t low = cont ? low0 : 0;  // reference dataZero
  bool withDict = !cont;
  for (uint32_t b = 0; b < nblocks; b++) {
    const Block B = blocks[b];
    const uint64_t start = B.start, size = B.end - B.start, stop = B.end - kTailLiterals;
    // the first block inserts the dictionary; every later one re-inserts the last 12 positions before
    // it (dataZero > BlockEndNoMatch from the second block on, smallz4.h:612-620)
    int64_t back = withDict ? -(int64_t)dictBack : -(int64_t)kTailNoMatch;
    if (legacy) back = 0;
    uint64_t skip = 0;
    bool lazyEval = false, rmq = false;
    for (int64_t i = back; i + kTailNoMatch <= (int64_t)size; i++) {
      const uint64_t pos = start + (uint64_t)i;
      // self-matching (smallz4.h:631-643)
      if (i > 0 && in[pos] == in[pos - 1] && mdist[pos - 1] == 1 && mlen[pos - 1] > kSameLetter) {
        mdist[pos] = 1;
        mlen[pos] = mlen[pos - 1] - 1;
        continue;
      }
      // insertion into both chains (smallz4.h:645-720): written at the block-relative slot
      const uint32_t slot = (uint32_t)((uint64_t)i & kWindow);
      const uint32_t four = gload4(in, pos);
      const uint32_t h = ref_hash(four);
      uint64_t cand = last[h] == kNoPos ? kNone : (uint64_t)last[h];
      last[h] = (uint32_t)pos;
      bool linked = false;
      if (cand == kNone || pos - cand > kWindow) {
        prevH[slot] = 0;
        prevX[slot] = 0;
      } else {
        uint64_t dist = pos - cand;
        prevH[slot] = (uint16_t)dist;
        bool ok = true;
        while (true) {
          if (cand < low) { ok = false; break; }  // the reference would read before its buffer
          const uint32_t seen = gload4(in, cand);
          if (seen == four) break;
          if (ref_hash(seen) != h) { ok = false; break; }
          const uint16_t step = prevH[cand & kWindow];  // read at the absolute slot
          if (step == 0) { ok = false; break; }
          dist += step;
          if (dist > kWindow) { ok = false; break; }
          cand -= step;
          if (cand < low) { ok = false; break; }
        }
        prevX[slot] = ok ? (uint16_t)dist : (uint16_t)0;
        linked = ok && dist != 0;
      }
      if (!linked || i < 0) continue;
      if (skip > 0) {
        skip--;
        if (!lazyEval) continue;
        lazyEval = false;
      }
      // findLongestMatch (smallz4.h:173-255): strictly longer replaces, maxChain counts replacements
      uint64_t bestLen = 1;
      uint32_t bestDist = 0, steps = maxChain;
      uint32_t hop = prevX[pos & kWindow];
      uint64_t backDist = 0;
      const int64_t room = (int64_t)(stop - pos);
      while (hop != 0) {
        backDist += hop;
        if (backDist > kWindow) break;
        hop = prevX[(pos - backDist) & kWindow];
        const int64_t need = (int64_t)bestLen + 1;
        if (need > room) break;
        const uint64_t c = pos - backDist;
        int64_t lo = need - 4;
        while (lo > 0 && gload4(in, pos + lo) == gload4(in, c + lo)) lo -= 4;
        if (lo > 0) continue;
        int64_t hi = need;
        while (hi + 4 <= room && gload4(in, pos + hi) == gload4(in, c + hi)) hi += 4;
        while (hi < room && in[pos + hi] == in[c + hi]) hi++;
        bestLen = (uint64_t)hi;
        bestDist = (uint32_t)backDist;
        if (--steps == 0) break;
      }
      mlen[pos] = (uint32_t)bestLen;
      mdist[pos] = (uint16_t)bestDist;
      rmq |= bestLen >= kRmqLen && !(bestDist == 1u && bestLen >= kSameLetter);
      if ((lazy || greedy) && bestLen != 1) {
        lazyEval = skip == 0;
        skip = bestLen;
      }
    }
    // positions the reference searched and found nothing keep (1, 0): the parse reads them as literals
    longFlag[b] = rmq ? 1u : 0u;
    withDict = false;
    if (legacy) {
      low = B.end;
      for (uint32_t j = 0; j < 65536; j++) {
        prevX[j] = 0;
        prevH[j] = 0;
      }
      for (uint32_t j = 0; j < (1u << kHashBits); j++) last[j] = kNoPos;
    } else if (B.end - low > kWindow) {
      low = B.end - kWindow;  // the reference keeps only the last 64 KiB - 1 (smallz4.h:799-804)
    }
  }
  for (uint32_t j = 0; j < 65536; j++) prevXg[j] = prevX[j];  // carried to the next chunk
}

void launch_dict(const uint8_t* in, const Block* blocks, uint32_t nblocks, uint32_t maxChain, uint32_t dictBack, int legacy,
                 uint32_t* last, uint16_t* prevH, uint16_t* prevX, uint32_t cont, uint32_t shift, uint32_t low0,
                 uint32_t* mlen, uint16_t* mdist, uint32_t* sel, uint32_t* longFlag, hipStream_t s)
{
  if (nblocks)
    hipLaunchKernelGGL(k_dict_matches, dim3(1), dim3(64), 0, s, in, blocks, nblocks, maxChain, dictBack, legacy, last, prevH,
                       prevX, cont, shift, low0, mlen, mdist, sel, longFlag);
}

// k_prep: the positions the reference never searches -- the last 12 of a block keep length 0, the parse's
// choices of the last 5 are literals.  (Greedy/lazy levels then replay the reference's skip bookkeeping in
// parallel: k_lazy_walk / k_lazy_fix / k_lazy_clear, checked against the assumed shortcut intervals by
// k_lazy_check / k_lazy_correct.)
__global__ __launch_bounds__(64) void k_prep(const uint8_t* __restrict__ in, const Block* __restrict__ blocks,
                                             Interval* __restrict__ ivAll, uint32_t* __restrict__ ivCount,
                                             uint32_t maxChain, uint32_t* __restrict__ mlen, uint16_t* __restrict__ mdist,
                                             uint64_t matchBase, uint32_t* __restrict__ sel, const uint32_t* __restrict__ longFlag,
                                             int* __restrict__ status)
{
  const Block B = blocks[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const uint64_t n = B.end - B.start;
  uint32_t* L = mlen + (B.start - matchBase);
  uint16_t* D = mdist + (B.start - matchBase);
  uint32_t* S = sel + (B.start - matchBase);
  if (maxChain == 0) return;
  const uint64_t lastSearch = n >= (uint64_t)kTailNoMatch ? n - kTailNoMatch : 0;  // inclusive, relative

  // positions the reference never searched keep length 0 (it leaves them default-constructed)
  for (uint64_t i = (n >= (uint64_t)kTailNoMatch ? lastSearch + 1 : 0) + lane; i < n; i += 64) L[i] = 0;
  if (maxChain > (uint32_t)kGreedyMax) {
    // the parse writes positions [0, n - 6]; the block ends with literals
    const uint64_t from = n > (uint64_t)kTailNoMatch ? n - kTailLiterals : 0;
    for (uint64_t i = from + lane; i < n; i += 64) S[i] = 0;
  }
}

// ================================================================================================
// Greedy/lazy levels in parallel.  The reference's bookkeeping (smallz4.h:726-744) touches only positions
// that have an exact predecessor ("linked": a match of >= 4 bytes) and are not same-letter shortcut copies
// (smallz4.h:631-643: the block's assumed intervals, masked out of the walk), and it is a chain of searched
// positions that alternates:
// k_lazy_walk walks this chain per 4096-position sub-segment from an assumed start (the
// sub-segment's first linked position, fresh); k_lazy_fix walks the sub-segments of a block in order
// and re-walks from the true entry until it meets the speculative walk at the same position in the
// same mode (from there both are the same walk); k_lazy_clear zeroes the linked positions no walk
// searched; k_lazy_check / k_lazy_correct compare the shortcut intervals the walk assumed with the ones its
// searches imply.
// ================================================================================================
constexpr int kWalkWaves = 4;         // sub-segments per k_walk / k_lazy_* workgroup
constexpr uint32_t kLazyCap = 1400;   // searched positions per sub-segment: <= 2 per 6 linked + 2
constexpr uint32_t kLazyEnd = 0x7FFFFFFFu;

// the searched-position chain over a register window of lengths: four 64-position windows in
// registers, loads three windows ahead (as k_walk); wave-uniform state
struct LazyWalker {
  const uint32_t* L;
  uint32_t lastSearch;  // inclusive
  uint32_t wbase, wL, xL1, xL2, xL3;
  // the block's assumed same-letter shortcut intervals (absolute positions, ascending): their positions copy
  // their predecessor's match and do no bookkeeping (smallz4.h:631-643), so the walk does not count them
  const Interval* iv = nullptr;
  uint32_t niv = 0, k0 = 0;
  uint64_t bstart = 0;
  uint64_t wIv = 0;  // lanes of the current window inside an interval
  __device__ __forceinline__ uint32_t ldw(uint32_t b) const
  {
    // unconditional load (clamped index; masked in next()): see k_walk
    const uint32_t i = b + lane_id();
    return L[i <= lastSearch ? i : lastSearch];
  }
  // lanes of the window [base, base + 64) inside an interval (intervals lie >= 65 299 positions apart, so
  // at most two can touch a window); k0 moves forward with the windows
  __device__ __forceinline__ uint64_t ivmask(uint32_t base)
  {
    while (k0 < niv && iv[k0].hi - bstart <= (uint64_t)base) k0++;
    uint64_t m = 0;
    for (uint32_t k = k0; k < niv && k < k0 + 2; k++) {
      const uint64_t lo = iv[k].lo - bstart, hi = iv[k].hi - bstart;
      if (lo >= (uint64_t)base + 64) break;
      const uint32_t a = lo > base ? (uint32_t)(lo - base) : 0u, b = hi < (uint64_t)base + 64 ? (uint32_t)(hi - base) : 64u;
      if (a < b) m |= (b - a == 64u ? ~0ull : ((1ull << (b - a)) - 1ull)) << a;
    }
    return m;
  }
  __device__ __forceinline__ void start(uint32_t pos)
  {
    wbase = pos & ~63u;
    wL = ldw(wbase);
    xL1 = ldw(wbase + 64);
    xL2 = ldw(wbase + 128);
    xL3 = ldw(wbase + 192);
    k0 = 0;
    wIv = niv ? ivmask(wbase) : 0ull;
  }
  // the need-th (0-based) linked position at or after pos, kLazyEnd when there is none
  __device__ __forceinline__ uint32_t next(uint32_t pos, uint32_t need)
  {
    while (pos <= lastSearch) {
      while (pos >= wbase + 64) {
        if (pos < wbase + 256) {
          wbase += 64;
          wL = xL1;
          xL1 = xL2;
          xL2 = xL3;
          xL3 = ldw(wbase + 192);
          wIv = niv ? ivmask(wbase) : 0ull;
        } else {
          start(pos);
        }
      }
      const uint64_t mask = __ballot(wL >= (uint32_t)kMinMatch && wbase + lane_id() <= lastSearch) & (~0ull << (pos - wbase)) & ~wIv;
      const uint32_t pc = (uint32_t)__popcll(mask);
      if (need < pc) {
        // the set bit with exactly `need` set bits below it: each lane counts its own (mbcnt)
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        const uint64_t hit = __ballot(((mask >> lane_id()) & 1ull) && below == need);
        return wbase + (uint32_t)__builtin_ctzll(hit);
      }
      need -= pc;
      pos = wbase + 64;
    }
    return kLazyEnd;
  }
  // length at q (q inside the current window: the position next() just returned)
  __device__ __forceinline__ uint32_t len(uint32_t q) const { return rdlane(wL, q - wbase); }
};

__global__ __launch_bounds__(64 * kWalkWaves) void k_lazy_walk(const Block* __restrict__ blocks,
                                                               const uint2* __restrict__ walkSegs, uint32_t nwalk,
                                                               const Interval* __restrict__ ivAll,
                                                               const uint32_t* __restrict__ ivCount,
                                                               const uint32_t* __restrict__ mlen, uint64_t matchBase,
                                                               uint32_t* __restrict__ slotsAll, uint4* __restrict__ state)
{
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * kWalkWaves + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch) return;
  uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kLazyCap) + kLazyCap;
  const uint32_t a = ws.y * kWalkSeg;
  const uint32_t aNext = a + kWalkSeg < n ? a + kWalkSeg : n;
  LazyWalker w;
  w.L = mlen + (B.start - matchBase);
  w.lastSearch = n - kTailNoMatch;
  w.iv = ivAll + (uint64_t)ws.x * kMaxIv;
  w.niv = ivCount[ws.x];
  w.bstart = B.start;
  w.start(a);
  // Fresh searches alternate with lazy ones: fresh q -> lazy q2 = the next linked position -> fresh = the
  // next linked position after skipping len(q2) more.  So the fresh positions form a functional graph, and
  // inside one 64-position window the walk's fresh positions are found at once (as k_walk does): every
  // linked lane computes its successor from the window's linked ranks (64 when it leaves the window), F2 ..
  // F32 by doubling, binary lifting from the entry.  The last fresh position of the window (its successor
  // elsewhere) and everything across windows go one step at a time through LazyWalker.
  uint32_t mode = 0, m = 0;  // mode 0: fresh, 1: lazy
  uint32_t q = w.next(a, 0);
  while (true) {
    if (q >= aNext) break;  // fresh, mode 0
    if (q >= w.wbase && q < w.wbase + 64) {
      const uint64_t M = __ballot(w.wL >= (uint32_t)kMinMatch && w.wbase + lane <= w.lastSearch) & ~w.wIv;
      const uint32_t pc = (uint32_t)__popcll(M);
      const bool lk = (M >> lane) & 1ull;
      const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
      // lane k: the lane of the k-th linked position of the window (k < pc)
      const uint32_t sel = (uint32_t)__builtin_amdgcn_ds_permute((int)((lk ? rk : 63u) << 2), (int)lane);
      // a fresh search at this lane: its lazy search is the next linked lane, which skips its length more
      const uint32_t r2 = rk + 1u;
      const uint32_t l2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((r2 < pc ? r2 : 0u) << 2), (int)sel);
      const uint32_t len2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(l2 << 2), (int)w.wL);
      const uint32_t r3 = r2 + 1u + len2;
      const uint32_t l3 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((r3 < pc ? r3 : 0u) << 2), (int)sel);
      const bool in = lk && r2 < pc && r3 < pc;
      uint32_t F[6];
      F[0] = in ? l3 : 64u;
#pragma unroll
      for (int k = 1; k < 6; k++) {
        const uint32_t g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((F[k - 1] & 63u) << 2), (int)F[k - 1]);
        F[k] = F[k - 1] >= 64u ? 64u : g;
      }
      const uint32_t e = q - w.wbase;
      uint32_t x = e;
      {
        const uint32_t y = rdlane(F[5], e);
        x = y <= lane ? y : x;
      }
#pragma unroll
      for (int k = 4; k >= 0; k--) {
        const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((x & 63u) << 2), (int)F[k]);
        x = y <= lane ? y : x;
      }
      const uint32_t pLast = rdlane(x, 63);  // the window's last fresh position of the walk
      const bool rec = x == lane && lane >= e && lane != pLast;  // fresh positions with both searches inside
      const uint64_t rb = __ballot(rec);
      const uint32_t cnt = (uint32_t)__popcll(rb);
      if (m + 2u * cnt + 2u > kLazyCap) {  // cannot happen (see kLazyCap); stop rather than overrun
        q = kLazyEnd;
        break;
      }
      if (rec) {
        const uint32_t j = m + 2u * __builtin_amdgcn_mbcnt_hi((uint32_t)(rb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rb, 0u));
        slots[j] = w.wbase + lane;
        slots[j + 1u] = w.wbase + l2;
      }
      m += 2u * cnt;
      q = w.wbase + pLast;
    }
    // the fresh search at q, its lazy one, the next fresh one -- one step at a time
    if (m + 2u > kLazyCap) {
      q = kLazyEnd;
      break;
    }
    if (lane == 0) slots[m] = q;
    m++;
    const uint32_t q2 = w.next(q + 1, 0);
    if (q2 >= aNext) {
      q = q2;
      mode = 1;
      break;
    }
    if (lane == 0) slots[m] = q2;
    m++;
    q = w.next(q2 + 1, w.len(q2));
  }
  if (lane == 0) state[idx] = make_uint4(kLazyCap, kLazyCap + m, q | (mode << 31), 0u);
}

// The join of sub-segment idx to the true walk from entry ex (q | mode << 31): the first speculative search
// at or after it; if that is the entry in the same mode, the speculative walk is the true one from there,
// else the walk is redone from the entry until it meets the speculative walk (same position, same mode) or
// leaves the sub-segment.  The redone searches go to fix[0, f); returns (merged, f, the speculative index it
// met: m when it did not, the exit); *bad: more than kLazyCap searches (cannot happen).
struct LazyJoin {
  uint32_t f, iMerge, exit;
  bool merged;
};
__device__ LazyJoin lazy_join(LazyWalker& w, const uint32_t* spec, uint32_t m, uint32_t* fix, uint32_t ex, uint32_t aNext,
                              uint32_t specExit, bool& bad)
{
  const uint32_t lane = lane_id();
  const uint32_t entry = ex & 0x7FFFFFFFu, emode = ex >> 31;
  auto first_at = [&](uint32_t from, uint32_t p) -> uint32_t {
    for (uint32_t b = from; b < m; b += 64) {
      const uint64_t ge = __ballot(b + lane < m && spec[b + lane] >= p);
      if (ge) return b + (uint32_t)__builtin_ctzll(ge);
    }
    return m;
  };
  auto visited = [&](uint32_t i, uint32_t p, uint32_t md) -> bool { return i < m && spec[i] == p && (i & 1u) == md; };
  uint32_t i = first_at(0, entry);
  if (visited(i, entry, emode)) return LazyJoin{0u, i, specExit, true};
  uint32_t q = entry, md = emode, f = 0;
  bool merged = false;
  if (w.wbase == 0xFFFFFFC0u || q < w.wbase || q >= w.wbase + 256) w.start(q);
  (void)w.next(q, 0);  // q is linked: brings its window in
  while (q < aNext) {
    if (f >= kLazyCap) {
      bad = true;
      break;
    }
    if (lane == 0) fix[f] = q;
    f++;
    const uint32_t need = md == 0 ? 0u : w.len(q);
    md ^= 1u;
    q = w.next(q + 1, need);
    if (q >= aNext) break;
    i = first_at(i, q);
    if (visited(i, q, md)) {
      merged = true;
      break;
    }
  }
  return LazyJoin{f, merged ? i : m, merged ? specExit : (q | (md << 31)), merged};
}

// every sub-segment k >= 1 joined at once from an ASSUMED entry, sub-segment k - 1's speculative exit (the
// true one whenever k - 1's true walk met its speculative walk: it then leaves where that one left).  The
// redone searches go just below the speculative list (slots [kLazyCap - f, kLazyCap), the list itself is
// kept for k_lazy_fix should the assumption fail); state.x = the join's exit, state.w = 1 << 31 | f << 11 |
// the speculative index it met (m when none).  k_lazy_fix keeps the joins whose assumption holds.
__global__ __launch_bounds__(64 * kWalkWaves) void k_lazy_join(const Block* __restrict__ blocks,
                                                               const uint2* __restrict__ walkSegs, uint32_t nwalk,
                                                               const Interval* __restrict__ ivAll,
                                                               const uint32_t* __restrict__ ivCount,
                                                               const uint32_t* __restrict__ mlen, uint64_t matchBase,
                                                               uint32_t* __restrict__ slotsAll, uint4* __restrict__ state)
{
  __shared__ uint32_t specAll[kWalkWaves][kLazyCap];
  __shared__ uint32_t fixAll[kWalkWaves][kLazyCap];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * kWalkWaves + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  if (ws.y == 0) return;
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch) return;
  const uint32_t ex = state[idx - 1].z;
  const uint4 st = state[idx];
  const uint32_t a = ws.y * kWalkSeg, aNext = a + kWalkSeg < n ? a + kWalkSeg : n;
  if ((ex & 0x7FFFFFFFu) >= aNext) {
    if (lane == 0) state[idx].w = 0;  // nothing searched here: k_lazy_fix's own loop (cheap)
    return;
  }
  const uint32_t m = st.y - kLazyCap;
  uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kLazyCap);
  uint32_t* spec = specAll[wave];
  uint32_t* fix = fixAll[wave];
  for (uint32_t t = lane; t < m; t += 64) spec[t] = slots[kLazyCap + t];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  LazyWalker w;
  w.L = mlen + (B.start - matchBase);
  w.lastSearch = n - kTailNoMatch;
  w.iv = ivAll + (uint64_t)ws.x * kMaxIv;
  w.niv = ivCount[ws.x];
  w.bstart = B.start;
  w.wbase = 0xFFFFFFC0u;
  bool bad = false;
  const LazyJoin J = lazy_join(w, spec, m, fix, ex, aNext, st.z, bad);
  __builtin_amdgcn_wave_barrier();
  for (uint32_t t = lane; t < J.f; t += 64) slots[kLazyCap - J.f + t] = fix[t];
  if (lane == 0) {
    state[idx].x = J.exit;
    state[idx].w = bad ? 0u : (0x80000000u | (J.f << 11) | J.iMerge);
  }
}

__global__ __launch_bounds__(64) void k_lazy_fix(const Block* __restrict__ blocks, const Interval* __restrict__ ivAll,
                                                 const uint32_t* __restrict__ ivCount, const uint32_t* __restrict__ mlen,
                                                 uint64_t matchBase, uint32_t* __restrict__ slotsAll,
                                                 uint4* __restrict__ state, int* __restrict__ status)
{
  __shared__ uint32_t spec[kLazyCap];  // the sub-segment's speculative searches
  __shared__ uint32_t fix[kLazyCap];   // the repaired ones in front of them
  const Block B = blocks[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch || B.walkCount < 2) return;
  LazyWalker w;
  w.L = mlen + (B.start - matchBase);
  w.lastSearch = n - kTailNoMatch;
  w.iv = ivAll + (uint64_t)blockIdx.x * kMaxIv;
  w.niv = ivCount[blockIdx.x];
  w.bstart = B.start;
  w.wbase = 0xFFFFFFC0u;  // no window loaded yet
  uint32_t ex = state[B.walkFirst].z;  // exact exit of sub-segment 0 (walked from the block start)
  uint32_t prevSpec = ex;               // the speculative exit of the sub-segment before k (k_lazy_join's assumption)
  for (uint32_t k = 1; k < B.walkCount;) {
    {
      // sub-segments k .. k + 63: lane j's join (k_lazy_join) holds when its assumed entry -- the speculative
      // exit of k + j - 1 -- is the true one: for j = 0 when it is ex, for j > 0 when lane j - 1's holds and
      // its join met its speculative walk (then it left where that walk left).  Up to the first that does not
      // hold, all at once: the redone searches moved in front of the speculative index the join met
      const uint32_t kj = k + lane;
      const bool in = kj < B.walkCount;
      const uint4 sj = in ? state[B.walkFirst + kj] : make_uint4(0u, 0u, 0u, 0u);
      const uint32_t pExit = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - 1u) & 63u) << 2), (int)sj.x);
      const uint32_t pSpec = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - 1u) & 63u) << 2), (int)sj.z);
      const bool holds = in && (sj.w >> 31) && (lane == 0 ? ex == prevSpec : pExit == pSpec);
      const uint64_t notHeld = ~__ballot(holds);
      const uint32_t nOk = notHeld ? (uint32_t)__builtin_ctzll(notHeld) : 64u;
      if (lane < nOk) {
        const uint32_t f = (sj.w >> 11) & 0x7FFu, iM = sj.w & 0x7FFu;
        const uint32_t start = kLazyCap + iM - f;
        uint32_t* sl = slotsAll + (uint64_t)(B.walkFirst + kj) * (2 * kLazyCap);
        if (iM) for (uint32_t t = f; t-- > 0;) sl[start + t] = sl[kLazyCap - f + t];  // (a few; moves up: descending)
        state[B.walkFirst + kj] = make_uint4(start, sj.y, sj.x, 0u);
      }
      if (nOk) {
        ex = rdlane(sj.x, nOk - 1u);
        prevSpec = rdlane(sj.z, nOk - 1u);
        k += nOk;
        if (nOk == 64u) continue;
      }
      if (k >= B.walkCount) break;
    }
    // sub-segment k on its own, from its true entry
    const uint32_t kc = k++;
    const uint32_t idx = B.walkFirst + kc;
    const uint4 st = state[idx];
    prevSpec = st.z;
    const uint32_t entry = ex & 0x7FFFFFFFu, emode = ex >> 31;
    const uint32_t a = kc * kWalkSeg, aNext = a + kWalkSeg < n ? a + kWalkSeg : n;
    uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kLazyCap);
    const uint32_t m = st.y - kLazyCap;
    if (entry >= aNext) {
      if (lane == 0) state[idx] = make_uint4(st.y, st.y, ex, 0u);  // nothing searched here
      continue;  // ex unchanged: the entry of the next sub-segment
    }
    for (uint32_t t = lane; t < m; t += 64) spec[t] = slots[kLazyCap + t];
    __syncthreads();
    // first speculative entry at or after p (64 slots per step); the speculative walk's i-th search
    // is in mode i & 1
    auto first_at = [&](uint32_t from, uint32_t p) -> uint32_t {
      for (uint32_t b = from; b < m; b += 64) {
        const uint64_t ge = __ballot(b + lane < m && spec[b + lane] >= p);
        if (ge) return b + (uint32_t)__builtin_ctzll(ge);
      }
      return m;
    };
    auto visited = [&](uint32_t i, uint32_t p, uint32_t md) -> bool { return i < m && spec[i] == p && (i & 1u) == md; };
    uint32_t i = first_at(0, entry);
    if (visited(i, entry, emode)) {
      if (lane == 0) state[idx] = make_uint4(kLazyCap + i, st.y, st.z, 0u);
      ex = st.z;
      __syncthreads();
      continue;
    }
    // re-walk from the true entry until it meets the speculative walk
    uint32_t q = entry, md = emode, f = 0;
    bool merged = false;
    if (w.wbase == 0xFFFFFFC0u || q < w.wbase || q >= w.wbase + 256) w.start(q);
    (void)w.next(q, 0);  // q is linked: brings its window in
    while (q < aNext) {
      if (f >= kLazyCap) {
        if (lane == 0) atomicOr(status, kStInvariant);
        break;
      }
      if (lane == 0) fix[f] = q;
      f++;
      const uint32_t need = md == 0 ? 0u : w.len(q);
      md ^= 1u;
      q = w.next(q + 1, need);
      if (q >= aNext) break;
      i = first_at(i, q);
      if (visited(i, q, md)) {
        merged = true;
        break;
      }
    }
    __syncthreads();
    const uint32_t iMerge = merged ? i : m;
    const uint32_t start = kLazyCap + iMerge - f;
    for (uint32_t t = lane; t < f; t += 64) slots[start + t] = fix[t];
    ex = merged ? st.z : (q | (md << 31));
    if (lane == 0) state[idx] = make_uint4(start, st.y, ex, 0u);
    __syncthreads();
  }
}

// the linked positions of a sub-segment that no walk searched get length 0
__global__ __launch_bounds__(64 * kWalkWaves) void k_lazy_clear(const Block* __restrict__ blocks,
                                                                const uint2* __restrict__ walkSegs, uint32_t nwalk,
                                                                const Interval* __restrict__ ivAll,
                                                                const uint32_t* __restrict__ ivCount,
                                                                uint32_t* __restrict__ mlen, uint64_t matchBase,
                                                                const uint32_t* __restrict__ slotsAll,
                                                                const uint4* __restrict__ state)
{
  __shared__ uint32_t bits[kWalkWaves][kWalkSeg / 32];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * kWalkWaves + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch) return;
  const uint32_t lastSearch = n - kTailNoMatch;
  uint32_t* L = mlen + (B.start - matchBase);
  const uint32_t a = ws.y * kWalkSeg;
  const uint32_t hi = a + kWalkSeg - 1 < lastSearch ? a + kWalkSeg - 1 : lastSearch;  // inclusive
  if (a > hi) return;
  uint32_t* bw = bits[wave];
  for (uint32_t t = lane; t < kWalkSeg / 32; t += 64) bw[t] = 0;
  const uint4 st = state[idx];
  const uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kLazyCap);
  for (uint32_t t = st.x + lane; t < st.y; t += 64) {
    const uint32_t q = slots[t] - a;
    atomicOr(&bw[q >> 5], 1u << (q & 31));
  }
  // positions inside a shortcut interval keep their copied match (written by k_find)
  LazyWalker w;
  w.iv = ivAll + (uint64_t)ws.x * kMaxIv;
  w.niv = ivCount[ws.x];
  w.bstart = B.start;
  // eight windows' lengths loaded together (unconditional, clamped index), then cleared
  for (uint32_t x00 = a; x00 <= hi; x00 += 512) {
    uint32_t lv[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) {
      const uint32_t x = x00 + 64u * u + lane;
      lv[u] = L[x <= hi ? x : hi];
    }
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) {
      const uint32_t x0 = x00 + 64u * u;
      if (x0 > hi) break;
      const uint32_t x = x0 + lane;
      const uint64_t inIv = w.niv ? w.ivmask(x0) : 0ull;
      if (x <= hi && lv[u] >= (uint32_t)kMinMatch && !((bw[(x - a) >> 5] >> ((x - a) & 31)) & 1u) && !((inIv >> lane) & 1ull))
        L[x] = 0;
    }
  }
}

// The same-letter shortcut intervals the walk ASSUMED (k_runs: from each long run's start, as at -9) against
// the ones the reference's loop would take given the walk's searches (smallz4.h:631-643): a searched position
// q whose match is (distance 1, length > MaxSameLetter) with data[q + 1] == data[q] starts one at q + 1.
// Both sets agree up to their first difference, and so does the walk (it only differs after a position the
// two treat differently), so the first difference of a block is the reference's: k_lazy_correct edits it
// into the block's list and the host runs the sort/find/walk round again -- each round settles a longer
// prefix.  firstBad[b] = block-relative position << 1 | (1: an assumed interval
// that does not start, 0: one that starts unassumed), ~0u when the block agrees.
__global__ __launch_bounds__(64 * kWalkWaves) void k_lazy_check(const uint8_t* __restrict__ in, const Block* __restrict__ blocks,
                                                                const uint2* __restrict__ walkSegs, uint32_t nwalk,
                                                                const Interval* __restrict__ ivAll,
                                                                const uint32_t* __restrict__ ivCount,
                                                                const uint32_t* __restrict__ longFlag,
                                                                const uint32_t* __restrict__ mlen, const uint16_t* __restrict__ mdist,
                                                                uint64_t matchBase, const uint32_t* __restrict__ slotsAll,
                                                                const uint4* __restrict__ state, uint32_t* __restrict__ firstBad)
{
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * kWalkWaves + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  const uint32_t niv = ivCount[ws.x];
  if (niv == 0u && (longFlag[ws.x] & kFlagRun) == 0u) return;  // no distance-1 match above MaxSameLetter
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  if (n < (uint32_t)kTailNoMatch) return;
  const uint32_t lastSearch = n - kTailNoMatch;
  const uint32_t* L = mlen + (B.start - matchBase);
  const uint16_t* D = mdist + (B.start - matchBase);
  const uint8_t* data = in + B.start;
  const Interval* iv = ivAll + (uint64_t)ws.x * kMaxIv;
  const uint4 st = state[idx];
  const uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kLazyCap);
  auto shortcut = [&](uint32_t q) {
    return D[q] == 1u && L[q] > kSameLetter && q + 1 <= lastSearch && data[q + 1] == data[q];
  };
  uint32_t bad = ~0u;
  // searched positions that start a shortcut: each must be an assumed interval's a
  for (uint32_t t = st.x + lane; t < st.y; t += 64) {
    const uint32_t q = slots[t];
    if (!shortcut(q)) continue;
    bool assumed = false;
    for (uint32_t j = 0; j < niv && !assumed; j++) assumed = iv[j].lo - B.start == (uint64_t)q + 1;
    if (!assumed) bad = min(bad, (q + 1) << 1);
  }
  // assumed intervals whose a lies in this sub-segment: a must be searched (binary search in the slot list)
  // and start a shortcut
  const uint32_t a0 = ws.y * kWalkSeg, a1 = a0 + kWalkSeg;
  for (uint32_t j = lane; j < niv; j += 64) {
    const uint32_t lo = (uint32_t)(iv[j].lo - B.start);
    if (lo == 0 || lo - 1 < a0 || lo - 1 >= a1) continue;
    const uint32_t q = lo - 1;
    uint32_t x = st.x, y = st.y;  // the first slot >= q
    while (x < y) {
      const uint32_t mid = (x + y) >> 1;
      if (slots[mid] < q) x = mid + 1;
      else y = mid;
    }
    if (!(x < st.y && slots[x] == q && shortcut(q))) bad = min(bad, (lo << 1) | 1u);
  }
  bad = wave_min_u32(bad);
  if (lane == 0 && bad != ~0u) atomicMin(&firstBad[ws.x], bad);
}

// one lane per block: the block's first difference edited into its interval list (as k_prep's serial replay
// did), and the host asked for another round
__global__ __launch_bounds__(64) void k_lazy_correct(const Block* __restrict__ blocks, Interval* __restrict__ ivAll,
                                                     uint32_t* __restrict__ ivCount, const uint32_t* __restrict__ mlen,
                                                     uint64_t matchBase, const uint32_t* __restrict__ firstBad,
                                                     int* __restrict__ status)
{
  const uint32_t b = blockIdx.x;
  const uint32_t v = firstBad[b];
  if (v == ~0u || threadIdx.x != 0) return;
  const Block B = blocks[b];
  Interval* iv = ivAll + (uint64_t)b * kMaxIv;
  const uint32_t niv = ivCount[b];
  const uint64_t lo = B.start + (v >> 1);
  uint32_t k0 = 0;  // intervals before this position are confirmed
  while (k0 < niv && iv[k0].lo < lo) k0++;
  uint32_t m;
  if (v & 1u) {
    // an assumed shortcut that does not happen here: dropped (a later position of the run may start the real
    // one, found in the next round)
    for (uint32_t j = k0; j + 1 < niv; j++) iv[j] = iv[j + 1];
    m = niv - 1;
  } else {
    // a shortcut nobody assumed: it runs while the copied length stays above MaxSameLetter; it replaces the
    // assumed intervals it overlaps
    const uint32_t La = mlen[lo - 1 - matchBase];
    Interval x;
    x.lo = lo;
    x.hi = lo + (La - kSameLetter);
    x.a = lo - 1;
    x.La = La;
    uint32_t r = k0;
    while (r < niv && iv[r].lo < x.hi) r++;
    if (r == k0) {
      for (uint32_t j = niv < kMaxIv ? niv : kMaxIv - 1; j > k0; j--) iv[j] = iv[j - 1];
      m = niv < kMaxIv ? niv + 1 : kMaxIv;
    } else {
      for (uint32_t j = 0; j < niv - r; j++) iv[k0 + 1 + j] = iv[r + j];
      m = k0 + 1 + (niv - r);
    }
    iv[k0] = x;
  }
  ivCount[b] = m;
  atomicOr(status, kStPrepRound);
}

constexpr int kSpecWaves = 4;  // independent segments per workgroup (workgroup slots, not LDS, bound occupancy)

template <bool kRmq>
__device__ __forceinline__ void dp_spec_body(const Block* __restrict__ blocks,
                                                             const DpSeg* __restrict__ dpSegs, uint32_t ndp,
                                                             const uint32_t* __restrict__ mlen,
                                                             const uint16_t* __restrict__ mdist, uint64_t matchBase,
                                                             uint32_t* __restrict__ costAll, uint32_t* __restrict__ sel,
                                                             uint32_t* __restrict__ reach, uint4* __restrict__ segState,
                                                             const uint32_t* __restrict__ longFlag,
                                                             uint32_t* __restrict__ upAll, uint32_t* __restrict__ downAll)
{
  __shared__ uint32_t rings[kSpecWaves][kRing];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // uniform
  const uint32_t segIdx = blockIdx.x * kSpecWaves + wave;
  if (segIdx >= ndp) return;  // whole wavefronts only; the waves never synchronize
  uint32_t* ring = rings[wave];
  const DpSeg G = dpSegs[segIdx];
  const Block B = blocks[G.block];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t base = B.start - matchBase;
  const uint32_t* L = mlen + base;
  const uint16_t* D = mdist + base;
  uint32_t* cost = costAll + base;
  uint32_t* S = sel + base;
  const int32_t segLo = (int32_t)G.lo, segHi = (int32_t)G.hi;
  // long lengths (> 273): UP/DOWN range minima over rmq blocks aligned on the block's last parsed position
  const int32_t top = (int32_t)(B.end - B.start) - 1 - kTailLiterals;
  // blocks with matches of kRmqLen+ run in the kRmq instantiation (range minima, carried chains);
  // the others in the lean one
  const bool rmq = (longFlag[G.block] & kFlagRmq) != 0u;
  if (rmq != kRmq) return;
  uint32_t* up = upAll + base;
  uint32_t* down = downAll + base;
  uint32_t upCarry = 0xFFFFFFFFu;

  // reach[i] = max over q in [lo, i) of q + len[q]: the highest cost a position below i reads
  if (G.k > 0) {
    uint32_t* R = reach + base;
    uint32_t carry = 0;
    // lengths one chunk ahead (opaque copy: the scan must not wait for the next load)
    uint32_t nxt = segLo + (int32_t)lane <= segHi ? L[segLo + (int32_t)lane] : 0u;
    for (int32_t c0 = segLo; c0 <= segHi; c0 += 64) {
      const int32_t q = c0 + (int32_t)lane;
      uint32_t Lq;
      asm volatile("v_mov_b32 %0, %1" : "=v"(Lq) : "v"(nxt));
      nxt = q + 64 <= segHi ? L[q + 64] : 0u;
      const uint32_t v = q <= segHi ? (uint32_t)q + Lq : 0u;
      const uint32_t incl = wave_incl_scan_max(v);
      // exclusive: wave_shr:1 by DPP, lane 0 takes the carry (the DPP's old value)
      uint32_t excl = (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)incl, kWaveShr1, 0xF, 0xF, false);
      excl = excl > carry ? excl : carry;
      if (q <= segHi) R[q] = excl;
      const uint32_t top = rdlane(incl, 63);
      carry = top > carry ? top : carry;
    }
  }

  // win: lane l holds cost[i0 + 1 + l] << 6 for the batch start i0.  For position i0 - r lane l
  // is match length l + 1 + r, so a candidate key is win + kLen[r] (a per-lane constant).
  // Above the segment the costs are the guess 0 (exact for k = 0).
  uint32_t kLen[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t len = lane + 1u + (uint32_t)r;
    // key = (cost + 3 [+1 from length 19]) << 6 | (64 - len): minimum = cheapest, then longest
    kLen[r] = len < (uint32_t)kMinMatch ? 0x80000000u : (((3u + (len >= 19u ? 1u : 0u)) << 6) + (64u - len));
  }
  uint32_t win = 0;
  // decision state (uniform, scalar)
  uint32_t lits = G.k == 0 ? (uint32_t)kTailLiterals : 0u;
  uint32_t litBump = 15;  // literal-run length at which a literal costs one more byte (15, 270, ...)
  uint32_t costNext = 0;  // cost[i + 1]
  uint32_t nextL = segHi - (int32_t)lane >= segLo ? L[segHi - lane] : 0u;
  auto key_cost = [&](int32_t, uint32_t key) -> uint32_t { return key >> 8; };
  RunEnd chain;
  bool noMatch = true;  // no position of the segment has a match: k_dp_fix repairs it in closed form
  int32_t runE = -1;    // the last same-letter run end read, and its cost
  uint32_t runC = 0;

  for (int32_t hi = segHi; hi >= segLo; hi -= 64) {
    const int32_t lo = hi - 63 > segLo ? hi - 63 : segLo;
    // opaque copy: the loop below must not wait for the prefetch issued right after
    uint32_t myL;
    asm volatile("v_mov_b32 %0, %1" : "=v"(myL) : "v"(nextL));
    const int32_t iN = hi - 64 - (int32_t)lane;
    nextL = iN >= segLo ? L[iN] : 0u;  // prefetch the next chunk
    // per position hi - t in lane t: its best key (0 = slow path, see bestBuf), its cost, its choice
    uint32_t kvBuf = 0xFFFFFFFFu, mcBuf = 0, bestBuf = 1;
    const uint32_t cnt = (uint32_t)(hi - lo + 1);
    const bool litChunk = __ballot(lane < cnt && myL >= (uint32_t)kMinMatch) == 0;
    noMatch = noMatch && litChunk;
    if (litChunk) {
      // no match anywhere in the chunk: every position is a literal, costs in closed form
      const uint32_t t = lane, run = lits + t + 1u;
      const uint32_t nb = run >= litBump ? 1u + (run - litBump) / 255u : 0u;
      mcBuf = costNext + t + 1u + nb;
      const uint32_t nbLast = rdlane(nb, cnt - 1u);
      costNext = rdlane(mcBuf, cnt - 1u);
      lits += cnt;
      litBump += 255u * nbLast;
      // next window: lane l = cost[lo + l] (position lo + l is lane cnt - 1 - l; only a full chunk has a next)
      win = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((63u - lane) << 2), (int)mcBuf) << 6;
      chain.valid = chain.pending = false;
    } else if (__ballot(lane < cnt && myL >= kSameLetter) == (cnt == 64u ? ~0ull : ((1ull << cnt) - 1ull)) &&
               [&]() -> bool {
                 const int32_t i = hi - (int32_t)lane;
                 const int32_t E0 = hi + (int32_t)rdlane(myL, 0);
                 const bool ok = lane >= cnt || (D[i] == 1u && i + (int32_t)myL == E0);
                 return __ballot(!ok) == 0;
               }()) {
      // a same-letter run: every position takes its distance-1 match unconditionally (smallz4.h:413-419)
      const int32_t i = hi - (int32_t)lane;
      const int32_t E0 = hi + (int32_t)rdlane(myL, 0);
      if (E0 != runE) {  // every chunk of a run shares its end: one load per run
        runE = E0;
        runC = E0 > segHi ? 0u : (E0 - hi < kRing - 64 ? ring[E0 & (kRing - 1)] : ld_fresh(&cost[E0]));
      }
      const uint32_t cE = runC;
      mcBuf = cE + 4u + (myL - 19u) / 255u;
      kvBuf = 0;
      bestBuf = myL;
      (void)i;
      costNext = rdlane(mcBuf, cnt - 1u);
      lits = 0;
      litBump = 15;
      if constexpr (kRmq) {
        if (E0 != chain.E || E0 > segHi) chain.valid = chain.pending = false;
      }
      win = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((63u - lane) << 2), (int)mcBuf) << 6;
    } else if (kRmq && chain.valid && chain.margin + 2u >= chain.costE + kMarginBias &&
               [&]() -> bool {
                 // every position continues the chain (a same-letter run position only when its end
                 // is the chain's end inside the segment: its length is not the flat optimum)
                 const int32_t i = hi - (int32_t)lane;
                 const bool in = lane < cnt;
                 const uint32_t Dl = in && myL >= kSameLetter ? (uint32_t)D[i] : 0u;
                 const int32_t Ei = i + (int32_t)myL > segHi ? segHi + 1 : i + (int32_t)myL;
                 const bool ok = !in || (myL >= (uint32_t)kMinMatch &&
                                         (Dl == 1u ? (i + (int32_t)myL == chain.E && chain.E <= segHi) : Ei == chain.E));
                 return __ballot(!ok) == 0;
               }() &&
               chain.costE + len_extra((uint32_t)(chain.E - hi)) <= costNext + 1u + (lits + 1u == litBump ? 1u : 0u)) {
      // chain chunk: every position takes its full length (the longest of its extra when flat above)
      const int32_t i = hi - (int32_t)lane;
      const uint32_t x = (uint32_t)(chain.E - i);
      mcBuf = chain.costE + len_extra(x);
      kvBuf = 0;
      bestBuf = i + (int32_t)myL > chain.E ? min(myL, piece_end(x)) : myL;
      costNext = rdlane(mcBuf, cnt - 1u);
      lits = 0;
      litBump = 15;
      const uint32_t mE = chain.costE + kMarginBias;
      chain.margin = mE < chain.margin ? mE : chain.margin;
      win = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((63u - lane) << 2), (int)mcBuf) << 6;
    } else {
    // a whole chunk whose match lengths are all <= 64: its batches unrolled (lane indices become
    // immediates, no per-batch bounds), as long as no literal-length bump is reachable; the first batch
    // that could reach one continues in the general loop below
    uint32_t tFast = 0;
    if (cnt == 64u) {
      if (__ballot(myL > 64u) == 0) {  // every length <= 64
        // Row-transposed batches.  The window is held as lane 16q + j = cost[i0 + 4j + 4 - q] << 6, so the
        // next batch's window is one DPP row shift with the four new costs entering lane 0 of their own
        // row.  The four positions' candidate keys (64 lanes each) are folded into one register by two
        // permlane32 swaps and one permlane16 swap (row r = position i0 - r), reduced inside the rows, and
        // the literal chain c_r = min(c_{r-1} + 1, mc_r) is a prefix minimum over the rows of mc_r - r
        // (two row broadcasts).  A batch's keys shift into their rows like the window, its costs stay in the window;
        // the scalar unit keeps only the literal-run length.
        const uint32_t q = lane >> 4, j = lane & 15u, o = 4u * j + 4u - q;  // o = cost offset in this lane
        uint32_t kP[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const uint32_t len = o + (uint32_t)r;
          // biased by -r << 6 so that (key >> 6) is mc_r - r; len < 4: far above every valid key
          kP[r] = len < (uint32_t)kMinMatch ? 0x80000000u
                                            : (((3u + (len >= 19u ? 1u : 0u)) << 6) + (64u - len) - ((uint32_t)r << 6));
        }
        // natural -> transposed window: lane 16q + j reads natural lane 4j + 3 - q
        uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((o - 1u) << 2), (int)win);
        const uint32_t rowBias = q << 6;
        // four lengths per lane (lane t: positions hi - t .. hi - t - 3), one readlane per batch
        const uint32_t pk = myL | (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane + 1u) << 2), (int)myL) << 8 |
                            (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane + 2u) << 2), (int)myL) << 16 |
                            (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane + 3u) << 2), (int)myL) << 24;
        uint32_t kRec = 0;  // lane 16 r + j: the key of position i0 - r of the j-th batch before the last
        auto batch = [&](uint32_t t) {
          const uint32_t P = rdlane(pk, t);
          uint32_t kv[4];
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int32_t Lr = (int32_t)((P >> (8 * r)) & 0xFFu);
            kv[r] = (int32_t)o <= Lr - r ? w + kP[r] : kKeyNone;
          }
          // fold: rows 0, 1 of X = position 0, rows 2, 3 = position 2; Y likewise positions 1, 3
          auto x = __builtin_amdgcn_permlane32_swap(kv[0], kv[2], false, false);
          auto y = __builtin_amdgcn_permlane32_swap(kv[1], kv[3], false, false);
          const uint32_t X = min(x[0], x[1]), Y = min(y[0], y[1]);
          auto z = __builtin_amdgcn_permlane16_swap(X, Y, false, false);
          const uint32_t key = row_min(min(z[0], z[1]));  // row r: position i0 - r, biased
          const uint32_t a = key >> 6;                    // mc_r - r
          uint32_t pm = min(a, dpp_rows<kRowBcast15, 0xA>(0xFFFFFFFFu, a));
          pm = min(pm, dpp_rows<kRowBcast31, 0xC>(0xFFFFFFFFu, pm));
          const uint32_t cp = min(pm, costNext + 1u);     // c_r - r
          const uint64_t use = __ballot(cp == a) & 0x0001000100010001ull;
          kRec = (uint32_t)__builtin_amdgcn_update_dpp((int)key, (int)kRec, kRowShr + 1, 0xF, 0xF, false);
          costNext = rdlane(cp, 48) + 3u;
          if (use) {
            lits = 3u - ((63u - (uint32_t)__builtin_clzll(use)) >> 4);
            litBump = 15u;
          } else {
            lits += 4u;
          }
          // next window: rows shift by one lane, lane 0 of row r takes c_r << 6
          w = (uint32_t)__builtin_amdgcn_update_dpp((int)((cp << 6) + rowBias), (int)w, kRowShr + 1, 0xF, 0xF, false);
        };
        uint32_t t = 0;
        // (a literal run that reaches its next length byte within the first batch starts in the loop below:
        // the sparse matches of the greedy/lazy levels leave long literal runs)
        if (lits + 4u < litBump) {
#pragma unroll
          for (uint32_t tb = 0; tb < 64; tb += 4) {
            batch(tb);
            t = tb + 4u;
            if (tb + 4u < 64u && lits + 4u >= litBump) break;
          }
        }
        // the rest of the chunk with a literal-length bump reachable: the literal term of the prefix minimum
        // costs one more from the position whose run length reaches litBump on (only the all-literal path
        // from the batch start can reach it: after a match the run restarts below 4 < 15)
        for (; t < 64u; t += 4u) {
          const uint32_t P = rdlane(pk, t);
          uint32_t kv[4];
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int32_t Lr = (int32_t)((P >> (8 * r)) & 0xFFu);
            kv[r] = (int32_t)o <= Lr - r ? w + kP[r] : kKeyNone;
          }
          auto x = __builtin_amdgcn_permlane32_swap(kv[0], kv[2], false, false);
          auto y = __builtin_amdgcn_permlane32_swap(kv[1], kv[3], false, false);
          const uint32_t X = min(x[0], x[1]), Y = min(y[0], y[1]);
          auto z = __builtin_amdgcn_permlane16_swap(X, Y, false, false);
          const uint32_t key = row_min(min(z[0], z[1]));
          const uint32_t a = key >> 6;
          uint32_t pm = min(a, dpp_rows<kRowBcast15, 0xA>(0xFFFFFFFFu, a));
          pm = min(pm, dpp_rows<kRowBcast31, 0xC>(0xFFFFFFFFu, pm));
          const uint32_t rStar = litBump - lits - 1u;  // the position whose literal is the bumped one
          const uint32_t cp = min(pm, costNext + 1u + (q >= rStar ? 1u : 0u));
          const uint64_t use = __ballot(cp == a) & 0x0001000100010001ull;
          kRec = (uint32_t)__builtin_amdgcn_update_dpp((int)key, (int)kRec, kRowShr + 1, 0xF, 0xF, false);
          costNext = rdlane(cp, 48) + 3u;
          if (use) {
            lits = 3u - ((63u - (uint32_t)__builtin_clzll(use)) >> 4);
            litBump = 15u;
          } else {
            lits += 4u;
            if (rStar < 4u) litBump += 255u;
          }
          w = (uint32_t)__builtin_amdgcn_update_dpp((int)((cp << 6) + rowBias), (int)w, kRowShr + 1, 0xF, 0xF, false);
        }
        tFast = t;
        // transposed -> natural: lane l = cost[i0 + 1 + l] is transposed lane 16 (3 - (l & 3)) + (l >> 2)
        win = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((16u * (3u - (lane & 3u))) + (lane >> 2)) << 2), (int)w);
        // position hi - l (l < tFast): its cost is in the window at offset tFast - l, its key in kRec
        const uint32_t oc = tFast - lane - 1u;
        const uint32_t rc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((16u * (3u - (oc & 3u))) + ((oc >> 2) & 15u)) << 2), (int)w);
        const uint32_t jb = (tFast >> 2) - 1u - (lane >> 2);
        const uint32_t rk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((16u * (lane & 3u)) + (jb & 15u)) << 2), (int)kRec);
        if (lane < tFast) {
          kvBuf = rk + ((lane & 3u) << 6);
          mcBuf = rc >> 6;
        }
        chain.valid = chain.pending = false;  // lengths <= 64: no chain continues through here
      }
    }
    for (uint32_t t = tFast; t < 64; t += 4) {
      const int32_t i0 = hi - (int32_t)t;
      if (i0 < lo) break;
      // next batch's window, shifted by four lanes (lanes 0-3 are refilled below)
      uint32_t nwin = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - 4u) << 2), (int)win);
      uint32_t Lr[4], kv[4], mcost[4];
      uint32_t maxL = 0;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        Lr[r] = i0 - r >= lo ? rdlane(myL, t + r) : 0u;
        maxL = Lr[r] > maxL ? Lr[r] : maxL;
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        // valid candidates: lengths 4 .. min(Lr[r], 64) (length l + 1 + r); longer ones are the slow path's
        const uint32_t top = Lr[r] < 64u ? Lr[r] : 64u;
        kv[r] = lane + 1u + (uint32_t)r <= top ? win + kLen[r] : 0xFFFFFFFFu;
      }
      if (maxL <= 16u) {
        // every candidate sits in row 0
#pragma unroll
        for (int r = 0; r < 4; r++) kv[r] = rdlane(row_min(kv[r]), 0);
      } else {
        wave_min4(kv);
      }
      // fast batch: four whole positions, no literal-length bump reachable, no length beyond 64
      if (i0 - 3 >= lo && maxL <= 64u && lits + 4u < litBump) {
        bool anyMatch = false;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          // a match wins ties; invalid keys decode to costs no literal path reaches
          const uint32_t mc = kv[r] >> 6;
          const uint32_t c = min(costNext + 1u, mc);
          const bool use = c == mc;
          lits = use ? 0u : lits + 1u;
          anyMatch |= use;
          costNext = c;
          mcost[r] = c;
          kvBuf = wrlane(kvBuf, kv[r], t + (uint32_t)r);
          mcBuf = wrlane(mcBuf, c, t + (uint32_t)r);
        }
        litBump = anyMatch ? 15u : litBump;
        chain.valid = chain.pending = false;  // lengths <= 64: no chain continues through here
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++) {
          mcost[r] = 0;
          const int32_t i = i0 - r;
          if (i < lo) break;
          const uint32_t Lk = Lr[r];
          lits++;
          uint32_t minCost = costNext + 1;
          if (lits == litBump) {
            minCost++;
            litBump += 255;
          }
          uint32_t best = 1;
          if (Lk >= (uint32_t)kMinMatch) {
            if (Lk >= kSameLetter && D[i] == 1) {
              best = Lk;
              const int32_t j = i + (int32_t)Lk;  // far back: spilled
              minCost = (j > segHi ? 0u : ld_fresh(&cost[j])) + 4 + (Lk - 19) / 255;
            } else {
              auto cost_at = [&](int32_t j) -> uint32_t {
                return j - i < kRing - 64 ? ring[j & (kRing - 1)] : ld_fresh(&cost[j]);
              };
              const int32_t Ei = i + (int32_t)Lk > segHi ? segHi + 1 : i + (int32_t)Lk;
              if (kRmq && Lk >= kRmqLen && chain.valid && chain.E == Ei && chain.margin + 2u >= chain.costE + kMarginBias) {
                // carried match, margin test passed: the full length (longest of its extra when flat above)
                const uint32_t x = (uint32_t)(Ei - i);
                const uint32_t l = i + (int32_t)Lk > Ei ? min(Lk, piece_end(x)) : Lk;
                const uint32_t mc = chain.costE + len_extra(x);
                if (mc <= minCost) {
                  minCost = mc;
                  best = l;
                }
              } else {
                const uint32_t kmin = kv[r];
                if ((kmin >> 6) <= minCost) {
                  minCost = kmin >> 6;
                  best = 64u - (kmin & 63u);
                }
                // lengths beyond 64: LDS ring (flushed every 64 positions), the HBM spill, UP/DOWN
                if (Lk > 64u) {
                  if constexpr (kRmq) {
                    long_lengths(i, Lk, top, segHi, true, up, down, cost_at, key_cost, minCost, best);
                  } else {
                    // no length reaches kRmqLen here: at most four steps
                    for (uint32_t b = 65; b <= Lk; b += 64) {
                      const uint32_t ln = b + lane;
                      uint32_t k2 = 0xFFFFFFFFu;
                      if (ln <= Lk) k2 = ((i + (int32_t)ln > segHi ? 0u : cost_at(i + (int32_t)ln)) + len_extra(ln)) << 6 | (63u - lane);
                      const uint32_t km = wave_min_fast(k2);
                      if (km != 0xFFFFFFFFu && (km >> 6) <= minCost) {
                        minCost = km >> 6;
                        best = b + (63u - (km & 63u));
                      }
                    }
                  }
                }
                if (kRmq && Lk >= kRmqLen) {
                  chain.E = Ei;
                  chain.costE = Ei > segHi ? 0u : cost_at(Ei);
                  // at the chunk top every position above is stored: the margin right away
                  chain.valid = i == hi;
                  chain.pending = i != hi;
                  if (i == hi) chain.margin = end_margin(i, Ei, top, up, down, cost_at, key_cost);
                }
              }
            }
          }
          if constexpr (kRmq) {
            if (Lk >= (uint32_t)kMinMatch && (i + (int32_t)Lk > segHi ? segHi + 1 : i + (int32_t)Lk) == chain.E) chain.add(i, minCost);
            else chain.valid = chain.pending = false;  // chains are contiguous
          }
          mcost[r] = minCost;
          costNext = minCost;
          if (best != 1) {
            lits = 0;
            litBump = 15;
          }
          kvBuf = wrlane(kvBuf, 0u, t + (uint32_t)r);
          mcBuf = wrlane(mcBuf, minCost, t + (uint32_t)r);
          bestBuf = wrlane(bestBuf, best, t + (uint32_t)r);
        }
      }
      // lanes 0-3 of the next window are positions i0-3 .. i0
#pragma unroll
      for (int r = 0; r < 4; r++) nwin = wrlane(nwin, mcost[r] << 6, 3u - (uint32_t)r);
      win = nwin;
    }
    }
    // flush: choices (a position took its best key iff its cost is that key's), costs to ring and HBM
    const int32_t iMine = hi - (int32_t)lane;
    if (iMine >= lo) {
      const uint32_t best = kvBuf == 0u ? bestBuf : ((kvBuf >> 6) == mcBuf ? 64u - (kvBuf & 63u) : 1u);
      S[iMine] = best;
      ring[iMine & (kRing - 1)] = mcBuf;
      cost[iMine] = mcBuf;  // read back (sc1) only >= kRing-64 positions later: no fence needed here
    }
    if constexpr (kRmq) {
      rmq_store_up(up, top, hi, cnt, rmq_key(mcBuf, top, iMine), upCarry);
      if (lo == 0 || ((uint32_t)(top - lo) & 255u) == 255u)
        rmq_store_down(down, top, lo, [&](int32_t j) -> uint32_t { return ring[j & (kRing - 1)]; });
      if (chain.pending) {
        const int32_t i = lo - 1;
        auto cost_at = [&](int32_t j) -> uint32_t {
          return j - i < kRing - 64 ? ring[j & (kRing - 1)] : ld_fresh(&cost[j]);
        };
        chain.margin = end_margin(i, chain.E, top, up, down, cost_at, key_cost);
        chain.valid = true;
        chain.pending = false;
      }
    }
  }
  if (lane == 0) segState[segIdx] = make_uint4(lits, litBump, noMatch ? 1u : 0u, 0u);
}

// The lean parse at <= 80 SGPRs: a wave takes ceil(sgpr / 16) * 16 + 16 of the SIMD's 800, so its natural
// 99 admit 6 waves per SIMD and 80 admit 8 (23 SGPRs spill to VGPR lanes).  The range-minimum variant
// would spill 133 and keeps its registers.
#define SZ4_DP_SPEC_ARGS                                                                                   \
  const Block *__restrict__ blocks, const DpSeg *__restrict__ dpSegs, uint32_t ndp,                        \
      const uint32_t *__restrict__ mlen, const uint16_t *__restrict__ mdist, uint64_t matchBase,           \
      uint32_t *__restrict__ costAll, uint32_t *__restrict__ sel, uint32_t *__restrict__ reach,            \
      uint4 *__restrict__ segState, const uint32_t *__restrict__ longFlag, uint32_t *__restrict__ upAll,   \
      uint32_t *__restrict__ downAll
__global__ __launch_bounds__(64 * kSpecWaves) __attribute__((amdgpu_num_sgpr(80))) void k_dp_spec_lean(SZ4_DP_SPEC_ARGS)
{
  dp_spec_body<false>(blocks, dpSegs, ndp, mlen, mdist, matchBase, costAll, sel, reach, segState, longFlag, upAll, downAll);
}
__global__ __launch_bounds__(64 * kSpecWaves) __attribute__((amdgpu_num_sgpr(80))) void k_dp_spec_rmq(SZ4_DP_SPEC_ARGS)
{
  dp_spec_body<true>(blocks, dpSegs, ndp, mlen, mdist, matchBase, costAll, sel, reach, segState, longFlag, upAll, downAll);
}
#undef SZ4_DP_SPEC_ARGS

// k_dp_fix<true>: the repair of every segment k >= 1 of a block without range minima at once, each from
// the SPECULATIVE costs and state of segment k - 1 (one wavefront per segment).  Choices depend on cost
// differences only, so the result is exact whenever everything it read lies in the part of k - 1 that
// k - 1's own (true) repair left speculative -- below k - 1's convergence point -- and k - 1 converged:
// its costs are then the exact ones minus that part's offset.  It saves the speculative values it
// overwrites (side, kDpSide positions at most, or it gives up) and records (conv or lowest position
// written, cost delta at conv, highest position read above the segment, converged) in dpRec.
// k_dp_fix<false> (one wavefront per block) then walks the boundaries: a segment whose record is exact
// only enters the offset tables; the others get their speculative values back and are repaired
// serially as before.
constexpr uint32_t kDpSide = 512;
// range-minimum blocks: k_dp_fix<true> also saves the UP/DOWN keys it overwrites, down to the bottom
// of its convergence point's rmq block (kDpSide + 255 positions at most), after the cost side
constexpr uint32_t kDpSideKeys = kDpSide + 256;
constexpr uint32_t kDpSideStride = kDpSide + kDpSideKeys;
// ... but only in blocks of more than this many parse segments: in a short block the serial walk is
// short too, while a range-minimum block's parallel repair reads long match ranges at every position it
// takes (zeros/urandom, 256 KiB blocks: parse 36.3 ms per 268 MB with it, 10.9 ms without)
constexpr uint32_t kParRmqMinSegs = 64;

template <bool kPar>
__global__ __launch_bounds__(64) void k_dp_fix(
const Block* __restrict__ blocks, const DpSeg* __restrict__ dpSegs,
                                               uint32_t ndp, const uint32_t* __restrict__ mlen,
                                               const uint16_t* __restrict__ mdist,
                                               uint64_t matchBase, uint32_t* __restrict__ costAll,
                                               uint32_t* __restrict__ sel, const uint32_t* __restrict__ reach,
                                               uint4* __restrict__ segState, const uint32_t* __restrict__ longFlag,
                                               uint32_t* __restrict__ upAll, uint32_t* __restrict__ downAll,
                                               uint2* __restrict__ side, uint4* __restrict__ dpRec, uint32_t tabStride)
{
  __shared__ uint32_t ring[kRing];
  // k_dp_fix<false>: four tables of tabStride (the launch's largest dpCount) words in dynamic LDS -- sized
  // for kMaxDpSegs they held 32 KiB and let only four of these one-wave workgroups share a CU
  extern __shared__ __attribute__((aligned(16))) uint32_t dpTab[];
  uint32_t* const convTab = dpTab;                   // positions >= convTab[k] of segment k: exact = stored + aboveTab[k]
  uint32_t* const deltaTab = dpTab + tabStride;      // below it: exact = stored + deltaTab[k]
  uint32_t* const convBlk = dpTab + 2 * tabStride;   // UP/DOWN keys of positions below it: exact = key cost + deltaTab[k]
  uint32_t* const aboveTab = dpTab + 3 * tabStride;  // 0, or the offset of the segment above when k_dp_fix<true> repaired it
  uint32_t bIdx, kFirst, kEnd;
  if constexpr (kPar) {
    if (blockIdx.x >= ndp) return;
    const DpSeg G0 = dpSegs[blockIdx.x];
    if (G0.k == 0 || ((longFlag[G0.block] & kFlagRmq) && blocks[G0.block].dpCount <= kParRmqMinSegs)) return;
    bIdx = G0.block;
    kFirst = G0.k;
    kEnd = G0.k + 1;
  } else {
    bIdx = blockIdx.x;
    kFirst = 1;
    kEnd = blocks[bIdx].dpCount;
  }
  const Block B = blocks[bIdx];
  if (B.dpCount <= 1) return;
  const uint32_t lane = threadIdx.x;
  SZ4_D7(
  // k_dp_fix<false> per block: serial positions, closed-form chunks, literal chunks, segments walked
  uint64_t d7Serial = 0, d7Closed = 0, d7Lit = 0, d7Segs = 0;
  uint64_t d7Tk[4] = {0, 0, 0, 0};  // ticks in literal / closed / serial chunks, and in the rmq stores
  const uint64_t d7t0 = __builtin_readcyclecounter();
  )
  if constexpr (kPar) {
    // a segment without any match cannot converge (that needs a match): nothing written, k_dp_fix<false>
    // repairs it in closed form
    if (segState[blockIdx.x].z != 0u) {
      if (lane == 0) dpRec[blockIdx.x] = make_uint4(dpSegs[blockIdx.x].hi + 1u, 0u, 0u, 2u);
      return;
    }
  }
  const uint64_t base = B.start - matchBase;
  const uint32_t* L = mlen + base;
  const uint16_t* D = mdist + base;
  const uint32_t* R = reach + base;
  uint32_t* cost = costAll + base;
  uint32_t* S = sel + base;
  const uint32_t first = dpSegs[B.dpFirst].hi;  // n - 6: the last parsed position
  const int32_t top = (int32_t)first;
  const bool rmq = (longFlag[bIdx] & kFlagRmq) != 0u;
  uint32_t* up = upAll + base;
  uint32_t* down = downAll + base;
  if (!kPar && lane == 0) {
    convTab[0] = 0;  // the top segment was parsed exactly
    deltaTab[0] = 0;
    convBlk[0] = 0;
    aboveTab[0] = 0;
  }
  __syncthreads();
  // exact cost of a position above the segment being repaired (0 past the parsed range); k_dp_fix<true>
  // takes the stored (speculative) costs, exact up to one offset where its result is used
  int32_t readTop = 0, keyTop = -1;  // k_dp_fix<true>: highest position above the segment read (costs, keys)
  auto exact_above = [&](uint32_t j) -> uint32_t {
    if (j > first) return 0u;
    if constexpr (kPar) {
      readTop = (int32_t)j > readTop ? (int32_t)j : readTop;
      return cost[j];
    } else {
      const uint32_t k = (first - j) / B.dpSize;
      const uint32_t v = ld_fresh(&cost[j]);
      return v + (j < convTab[k] ? deltaTab[k] : aboveTab[k]);
    }
  };
  // k_dp_fix<false> over blocks that k_dp_fix<true> repaired: the records 64 segments at a time
  const bool par = !kPar && (!rmq || B.dpCount > kParRmqMinSegs);
  uint32_t prevKeyLim = 0;  // convBlk of segment k - 1
  uint4 recV = make_uint4(0u, 0u, 0u, 0u);
  uint32_t prevV = 0, prevConv = 0;  // offset below segment k - 1's convergence point, that point
  bool prevDone = true;              // segment k - 1's repair converged (segment 0 is exact)
  bool recNoMatch = false;           // k_dp_fix<true>'s record: the segment has no match (flag 2)

  for (uint32_t k = kFirst; k < kEnd; k++) {
    const DpSeg G = dpSegs[B.dpFirst + k];
    const int32_t lo = (int32_t)G.lo, hi = (int32_t)G.hi;
    if (par) {
      if (((k - 1u) & 63u) == 0u) {
        const uint32_t kk = k + lane;
        recV = kk < B.dpCount ? dpRec[B.dpFirst + kk] : make_uint4(0u, 0u, 0u, 0u);
      }
      const uint32_t t = (k - 1u) & 63u;
      const uint32_t rConv = rdlane(recV.x, t), rDelta = rdlane(recV.y, t);
      const uint32_t rReach = rdlane(recV.z, t), rFlag = rdlane(recV.w, t);
      recNoMatch = (rFlag & 2u) != 0u;
      const uint32_t rKeyTop = rFlag >> 2;  // highest key position read + 1, 0: none
      // the bottom of the rmq block of its convergence point: keys at and above it were rewritten
      const uint32_t rKeyLim = rmq && (rFlag & 1u) ? max((uint32_t)rmq_block_top(top, (int32_t)rConv) - 255u, (uint32_t)lo)
                                                   : rConv;
      if ((rFlag & 1u) && (k == 1u || (prevDone && rReach < prevConv && (rKeyTop == 0u || rKeyTop - 1u < prevKeyLim)))) {
        // everything it read was exact - prevV: its costs are exact - prevV
        if (lane == 0) {
          convTab[k] = rConv;
          convBlk[k] = rKeyLim;
          aboveTab[k] = prevV;
          deltaTab[k] = prevV + rDelta;
        }
        prevV += rDelta;
        prevConv = rConv;
        prevKeyLim = rKeyLim;
        prevDone = true;
        __syncthreads();
        continue;
      }
      // repaired from a wrong state: the speculative values back, then the serial repair
      uint2* sd = side + (uint64_t)(B.dpFirst + k) * kDpSideStride;
      for (int32_t t2 = (int32_t)lane; hi - t2 >= (int32_t)rConv; t2 += 64) {  // rConv = hi + 1: nothing written
        const uint2 v = sd[t2];
        cost[hi - t2] = v.x;
        S[hi - t2] = v.y;
      }
      if (rmq)
        for (int32_t t2 = (int32_t)lane; hi - t2 >= (int32_t)rKeyLim; t2 += 64) {
          const uint2 v = sd[kDpSide + t2];
          up[hi - t2] = v.x;
          down[hi - t2] = v.y;
        }
      // the stores complete before the reloads below; only this wavefront reads them (same CU), so a
      // workgroup-scope fence does -- __threadfence() would write back and invalidate the XCD's whole L2
      // (buffer_wbl2 sc1 + buffer_inv sc1 on gfx950) once per restored segment
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    }
    const uint4 st = segState[B.dpFirst + k - 1];  // exact state below the segment above
    uint32_t lits = st.x, litBump = st.y;
    // no match in the segment (k_dp_spec): every chunk is closed-form literals and none converges, so
    // nothing needs loading (this segment's own state record is overwritten only at its end)
    // (blocks k_dp_fix<true> ran over carry the flag in their records, already in registers)
    const bool noMatch = !kPar && (par ? recNoMatch : segState[B.dpFirst + k].z != 0u);
    uint32_t costNext = exact_above((uint32_t)hi + 1);
    uint32_t cbuf = exact_above((uint32_t)hi + 1 + ((lane - (uint32_t)hi - 1u) & 63u));
    // exact cost of j > i: this pass's own results (ring / HBM) inside the segment, above it the table
    auto cost_at = [&](int32_t i, int32_t j) -> uint32_t {
      if (j > hi) return exact_above((uint32_t)j);
      return j - i < kRing ? ring[j & (kRing - 1)] : ld_fresh(&cost[j]);
    };
    // exact cost encoded by an UP/DOWN key at j: this pass's own inside the segment, the tables above
    auto key_cost = [&](int32_t j, uint32_t key) -> uint32_t {
      uint32_t c = key >> 8;
      if (j > hi) {
        if constexpr (kPar) {
          keyTop = j > keyTop ? j : keyTop;
        } else {
          const uint32_t kk = (first - (uint32_t)j) / B.dpSize;
          c += (uint32_t)j < convBlk[kk] ? deltaTab[kk] : aboveTab[kk];
        }
      }
      return c;
    };
    uint32_t prevDelta = 0;
    int32_t runTop = hi;
    int32_t conv = lo;
    uint32_t convDelta = 0;
    uint32_t upCarry = 0xFFFFFFFFu;
    RunEnd chain;
    uint32_t closedCost = 0;  // closed-form chunk: cost at its end closedE
    int32_t closedE = 0;
    bool closedRun = false;   // the closed-form chunk is a same-letter run (not a carried chain)
    int32_t runE = -1;        // the last same-letter run end read, and its exact cost
    uint32_t runC = 0;
    int32_t forcedE = -1;     // the run end forced_below was asked about, and its answer
    bool forcedOk = false;
    // positions [lo, top] all take the distance-1 match of a run ending at E unconditionally: 512 per
    // step, 8 loads in flight per lane
    auto forced_below = [&](int32_t top, int32_t E) -> bool {
      for (int32_t b = top; b >= lo; b -= 512) {
        bool bad = false;
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int32_t i = b - 64 * u - (int32_t)lane;
          const int32_t ic = i >= lo ? i : lo;  // unconditional (clamped) loads
          const uint32_t l = L[ic];
          const uint32_t d = (uint32_t)D[ic];
          bad |= i >= lo && !(l >= kSameLetter && d == 1u && ic + (int32_t)l == E);
        }
        if (__ballot(bad)) return false;
      }
      return true;
    };
    bool done = false;
    int32_t maxReach = hi + 64;  // k_dp_fix<true>: highest position read above the segment
    int32_t lowW = hi;           // k_dp_fix<true>: lowest position written
    // the chunk's inputs are loaded one chunk ahead (positions below are not rewritten before)
    // two chunks ahead: a block's repair is one wavefront per SIMD, nothing else hides the latency
    uint32_t nL, nD, nS, nC, nR, mL, mD, mS, mC, mR;
    auto load_chunk = [&](int32_t h, uint32_t& xL, uint32_t& xD, uint32_t& xS, uint32_t& xC, uint32_t& xR) {
      const int32_t ip = h - (int32_t)lane;
      const bool in = ip >= lo;
      xL = in ? L[ip] : 0u;
      xD = in ? (uint32_t)D[ip] : 0u;
      xS = in ? S[ip] : 0u;
      xC = in ? cost[ip] : 0u;
      xR = in ? R[ip] : 0u;
    };
    nL = nD = nS = nC = nR = mL = mD = mS = mC = mR = 0u;
    if (!noMatch) {
      load_chunk(hi, nL, nD, nS, nC, nR);
      if (hi - 64 >= lo) load_chunk(hi - 64, mL, mD, mS, mC, mR);
    }
    for (int32_t h = hi; h >= lo && !done; h -= 64) {
      const int32_t ip = h - (int32_t)lane;
      const bool in = ip >= lo;
      uint32_t cL, cD, cS, cC, cR;
      // opaque copies: the loop below must not wait for the prefetches issued right after
      asm volatile("v_mov_b32 %0, %1" : "=v"(cL) : "v"(nL));
      asm volatile("v_mov_b32 %0, %1" : "=v"(cD) : "v"(nD));
      asm volatile("v_mov_b32 %0, %1" : "=v"(cS) : "v"(nS));
      asm volatile("v_mov_b32 %0, %1" : "=v"(cC) : "v"(nC));
      asm volatile("v_mov_b32 %0, %1" : "=v"(cR) : "v"(nR));
      nL = mL;
      nD = mD;
      nS = mS;
      nC = mC;
      nR = mR;
      if (h - 128 >= lo && !noMatch) load_chunk(h - 128, mL, mD, mS, mC, mR);
      const int32_t cl = h - 63 > lo ? h - 63 : lo;
      const uint32_t cnt = (uint32_t)(h - cl + 1);
      if constexpr (kPar) {
        if ((uint32_t)(hi - h) >= kDpSide) break;  // gives up: k_dp_fix<false> repairs it
        if (in) {
          uint2* sd = side + (uint64_t)blockIdx.x * kDpSideStride;
          sd[(uint32_t)(hi - ip)] = make_uint2(cC, cS);
          if (rmq) sd[kDpSide + (uint32_t)(hi - ip)] = make_uint2(up[ip], down[ip]);
        }
        lowW = cl;
      }
      closedRun = false;
      SZ4_D7(if (h == hi) d7Segs++;)
      SZ4_D7(const uint64_t d7c0 = __builtin_readcyclecounter(); const uint64_t d7l0 = d7Lit, d7k0 = d7Closed;)
      if (noMatch || __ballot(in && cL >= (uint32_t)kMinMatch) == 0) {
        SZ4_D7(d7Lit++;)
        // no match anywhere in the chunk: all literals, costs in closed form (lane t = position h - t)
        auto lit_cost = [&](uint32_t t, uint32_t& nb) -> uint32_t {
          const uint32_t run = lits + t + 1u;
          nb = run >= litBump ? 1u + (run - litBump) / 255u : 0u;
          return costNext + t + 1u + nb;
        };
        uint32_t nb = 0, nb2 = 0;
        const uint32_t cT = lit_cost(lane, nb);
        if (lane < cnt) {
          S[ip] = 1;
          cost[ip] = cT;
          ring[ip & (kRing - 1)] = cT;
        }
        // register window: lane l holds the cost of the position congruent to l mod 64
        const uint32_t tl = ((uint32_t)h - lane) & 63u;
        if (tl < cnt) cbuf = lit_cost(tl, nb2);
        chain.valid = chain.pending = false;
        if (!noMatch) {  // convergence bookkeeping (a segment without matches never converges)
          const uint32_t delta = cT - cC;
          // the previous position's delta: wave_shr:1, lane 0 takes the carried one (the DPP's old value)
          const uint32_t dPrev = (uint32_t)__builtin_amdgcn_update_dpp((int)prevDelta, (int)delta, kWaveShr1, 0xF, 0xF, false);
          const uint64_t chg = __ballot(lane < cnt && (ip == hi || delta != dPrev));
          if (chg) runTop = h - (63 - (int32_t)__builtin_clzll(chg));
          prevDelta = rdlane(delta, cnt - 1u);
        }
        lits += cnt;
        litBump += 255u * rdlane(nb, cnt - 1u);
        costNext = rdlane(cT, cnt - 1u);
      } else if ([&]() -> bool {
                   // closed-form chunks: (a) a same-letter run, every position taking its distance-1
                   // match unconditionally (smallz4.h:413-419); (b) a carried chain whose full lengths
                   // are optimal (the first one beats its literal, the others beat theirs since
                   // extra(x + 1) <= extra(x) + 1)
                   const int32_t E0 = h + (int32_t)rdlane(cL, 0);
                   if (__ballot(in && !(cL >= kSameLetter && cD == 1u && ip + (int32_t)cL == E0)) == 0) {
                     // every chunk of a run shares its end: one (dependent, uncached) load per run
                     if (E0 != runE) {
                       runC = cost_at(h, E0);
                       runE = E0;
                     }
                     closedCost = runC;
                     closedE = E0;
                     closedRun = true;
                     return true;
                   }
                   if (rmq && chain.valid && chain.margin + 2u >= chain.costE + kMarginBias &&
                       __ballot(in && !(cL >= (uint32_t)kMinMatch && ip + (int32_t)cL == chain.E)) == 0 &&
                       chain.costE + len_extra((uint32_t)(chain.E - h)) <= costNext + 1u + (lits + 1u == litBump ? 1u : 0u)) {
                     closedCost = chain.costE;
                     closedE = chain.E;
                     return true;
                   }
                   return false;
                 }()) {
        const uint32_t cT = closedCost + len_extra((uint32_t)(closedE - ip));
        SZ4_D7(d7Closed++;)
        if (closedE > maxReach) maxReach = closedE;
        if (closedE != chain.E) chain.valid = chain.pending = false;
        const uint32_t delta = cT - cC;
        const uint32_t dPrev = (uint32_t)__builtin_amdgcn_update_dpp((int)prevDelta, (int)delta, kWaveShr1, 0xF, 0xF, false);
        const uint64_t chg = __ballot(lane < cnt && (ip == hi || delta != dPrev));
        const uint64_t upTo = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
        const int32_t rt = (chg & upTo) ? h - (63 - (int32_t)__builtin_clzll(chg & upTo)) : runTop;
        const int32_t need = (int32_t)cR > ip ? (int32_t)cR : ip;
        uint64_t cv = __ballot(lane < cnt && cS != 1u && rt >= need);
        // every position from here down to the segment's bottom takes the same run's match unconditionally
        // (smallz4.h:409-415: length >= MaxSameLetter, distance 1, the same end): its choice is the stored
        // one and its cost the stored one plus this chunk's (constant) offset -- converged right here
        if (cv == 0u && closedRun) {
          if (forcedE != closedE) {
            forcedE = closedE;
            forcedOk = forced_below(h - 64, closedE);
          }
          if (forcedOk) cv = 1ull;  // lane 0: position h
        }
        const uint32_t last = cv ? (uint32_t)__builtin_ctzll(cv) : cnt - 1u;  // last position processed
        if (lane <= last) {
          S[ip] = cL;
          cost[ip] = cT;
          ring[ip & (kRing - 1)] = cT;
        }
        const uint32_t tl = ((uint32_t)h - lane) & 63u;
        if (tl <= last) cbuf = closedCost + len_extra((uint32_t)(closedE - (h - (int32_t)tl)));
        const uint32_t mE = closedCost + kMarginBias;
        if (chain.valid) chain.margin = mE < chain.margin ? mE : chain.margin;
        runTop = rdlane((uint32_t)rt, last);
        prevDelta = rdlane(delta, last);
        costNext = rdlane(cT, last);
        lits = 0;
        litBump = 15;
        if (cv) {
          conv = h - (int32_t)last;
          convDelta = prevDelta;
          done = true;
        }
      } else
      for (uint32_t t = 0; t < 64; t++) {
        const int32_t i = h - (int32_t)t;
        if (i < lo) break;
        SZ4_D7(d7Serial++;)
        const uint32_t Lk = rdlane(cL, t), Dk = rdlane(cD, t);
        if (Lk >= (uint32_t)kMinMatch && i + (int32_t)Lk > maxReach) maxReach = i + (int32_t)Lk;
        lits++;
        uint32_t minCost = costNext + 1;
        if (lits == litBump) {
          minCost++;
          litBump += 255;
        }
        uint32_t best = 1;
        if (Lk >= (uint32_t)kMinMatch) {
          if (Lk >= kSameLetter && Dk == 1) {
            best = Lk;
            // positions of one run share its end: one (dependent, uncached) load per run, as in the
            // closed-form chunks
            const int32_t E = i + (int32_t)Lk;
            if (E != runE) {
              runC = cost_at(i, E);
              runE = E;
            }
            minCost = runC + 4 + (Lk - 19) / 255;
          } else {
            auto cost_j = [&](int32_t j) -> uint32_t { return cost_at(i, j); };
            const int32_t Ei = i + (int32_t)Lk;  // <= top + 1
            if (rmq && Lk >= kRmqLen && chain.valid && chain.E == Ei && chain.margin + 2u >= chain.costE + kMarginBias) {
              const uint32_t mc = chain.costE + len_extra(Lk);  // carried match: the full length
              if (mc <= minCost) {
                minCost = mc;
                best = Lk;
              }
            } else {
              const uint32_t len = ((lane - (uint32_t)i - 1u) & 63u) + 1u;
              const uint32_t lim64 = Lk < 64 ? Lk : 64u;
              const uint32_t key = ((cbuf + 3u + ((len + 45u) >> 6)) << 6) + (64u - len);
              const uint32_t kmin = wave_min_fast(len - 4u <= lim64 - 4u ? key : 0xFFFFFFFFu);
              if ((kmin >> 6) <= minCost) {
                minCost = kmin >> 6;
                best = 64u - (kmin & 63u);
              }
              if (Lk > 64u) long_lengths(i, Lk, top, top, rmq, up, down, cost_j, key_cost, minCost, best);
              if (rmq && Lk >= kRmqLen) {
                chain.E = Ei;
                chain.costE = Ei > top ? 0u : cost_j(Ei);
                chain.valid = i == h;
                chain.pending = i != h;
                if (i == h) chain.margin = end_margin(i, Ei, top, up, down, cost_j, key_cost);
              }
            }
          }
        }
        if (Lk >= (uint32_t)kMinMatch && i + (int32_t)Lk == chain.E) chain.add(i, minCost);
        else chain.valid = chain.pending = false;  // chains are contiguous
        const uint32_t specBest = rdlane(cS, t), specCost = rdlane(cC, t), rch = rdlane(cR, t);
        if (lane == 0) {
          S[i] = best;
          cost[i] = minCost;
          ring[i & (kRing - 1)] = minCost;
        }
        cbuf = lane == ((uint32_t)i & 63u) ? minCost : cbuf;
        costNext = minCost;
        const uint32_t delta = minCost - specCost;
        if (i == hi || delta != prevDelta) runTop = i;
        prevDelta = delta;
        if (best != 1) {
          lits = 0;
          litBump = 15;
          const int32_t need = (int32_t)rch > i ? (int32_t)rch : i;
          if (specBest != 1 && runTop >= need) {
            conv = i;
            convDelta = delta;
            done = true;
            break;
          }
        }
      }
      SZ4_D7(const uint64_t d7c1 = __builtin_readcyclecounter();
             d7Tk[d7Lit != d7l0 ? 0 : d7Closed != d7k0 ? 1 : 2] += d7c1 - d7c0;)
      if (rmq) {
        if (!done) {
          // UP of the chunk, DOWN of a finished rmq block
          const uint32_t kt = lane < cnt ? rmq_key(ring[ip & (kRing - 1)], top, ip) : 0xFFFFFFFFu;
          rmq_store_up(up, top, h, cnt, kt, upCarry);
          if (cl == 0 || ((uint32_t)(top - cl) & 255u) == 255u)
            rmq_store_down(down, top, cl, [&](int32_t j) -> uint32_t { return ring[j & (kRing - 1)]; });
          if (chain.pending) {
            const int32_t i = cl - 1;
            auto cost_j = [&](int32_t j) -> uint32_t { return cost_at(i, j); };
            chain.margin = end_margin(i, chain.E, top, up, down, cost_j, key_cost);
            chain.valid = true;
            chain.pending = false;
          }
        } else {
          // converged inside conv's rmq block: its keys again, exact (below conv: stored + delta)
          const int32_t jt = rmq_block_top(top, conv);
          const int32_t jb0 = jt - 255;
          const int32_t jb = jb0 > lo ? jb0 : lo;
          if constexpr (kPar) {  // the keys below the chunks it went through: saved before rewritten
            uint2* sd = side + (uint64_t)blockIdx.x * kDpSideStride + kDpSide;
            for (int32_t j = jb + (int32_t)lane; j < lowW; j += 64) sd[(uint32_t)(hi - j)] = make_uint2(up[j], down[j]);
          }
          auto exact = [&](int32_t j) -> uint32_t {
            return j >= conv ? ring[j & (kRing - 1)] : ld_fresh(&cost[j]) + convDelta;
          };
          rmq_store_up_block(up, top, jb, jt, exact);
          rmq_store_down(down, top, jb, exact);
          if (!kPar && lane == 0) convBlk[k] = (uint32_t)jb;  // (k_dp_fix<true> has no tables)
        }
      }
      SZ4_D7(d7Tk[3] += __builtin_readcyclecounter() - d7c1;)
    }
    if constexpr (kPar) {
      const int32_t rd = wave_max_i32(readTop > maxReach ? readTop : maxReach);
      const uint32_t kt = (uint32_t)(wave_max_i32(keyTop) + 1);
      if (lane == 0)
        dpRec[blockIdx.x] = make_uint4(done ? (uint32_t)conv : (uint32_t)lowW, convDelta, (uint32_t)rd, (done ? 1u : 0u) | kt << 2);
    } else {
      if (lane == 0) {
        if (!done || !rmq) convBlk[k] = (uint32_t)conv;
        convTab[k] = (uint32_t)conv;
        deltaTab[k] = convDelta;
        aboveTab[k] = 0;
        // not converged: the state below the segment is this pass's own
        if (!done) segState[B.dpFirst + k] = make_uint4(lits, litBump, 0u, 0u);
      }
      prevV = convDelta;
      prevConv = (uint32_t)conv;
      prevDone = done;
      __syncthreads();
      prevKeyLim = convBlk[k];
    }
  }
  SZ4_D7(
  if (!kPar && lane == 0) {
    const uint64_t dt = __builtin_readcyclecounter() - d7t0;
    atomicAdd((unsigned long long*)&sz4_diag[0], (unsigned long long)d7Serial);
    atomicAdd((unsigned long long*)&sz4_diag[1], (unsigned long long)d7Closed);
    atomicAdd((unsigned long long*)&sz4_diag[2], (unsigned long long)d7Lit);
    atomicAdd((unsigned long long*)&sz4_diag[3], (unsigned long long)d7Segs);
    atomicMax((unsigned long long*)&sz4_diag[4], (unsigned long long)d7Serial);
    atomicAdd((unsigned long long*)&sz4_diag[5], (unsigned long long)dt);
    atomicMax((unsigned long long*)&sz4_diag[6], (unsigned long long)dt);
    atomicAdd((unsigned long long*)&sz4_diag[7], 1ull);
    if (rmq) atomicAdd((unsigned long long*)&sz4_diag[8], 1ull);
    for (int q = 0; q < 4; q++) atomicAdd((unsigned long long*)&sz4_diag[9 + q], (unsigned long long)d7Tk[q]);
  }
  )
}

// ================================================================================================
// Sequences.  The reference walks the parse forward (selectBestMatches, smallz4.h:259-371): a
// position with a chosen length > 1 starts a match, others are literals.  The walk is split into
// sub-segments of kWalkSeg positions walked at once (k_walk), repaired where a speculative start
// was wrong (k_walk_fix), and turned into 16-byte tokens (literal run, match) by k_seg_tokens.
// ================================================================================================


// k_walk: one wavefront per sub-segment walks the parse forward from the sub-segment's first
// position as if a sequence started there, and records the positions of the matches it takes
// until the walk reaches the next sub-segment.  Four 64-position windows of chosen lengths sit in
// registers (loads run three windows ahead); literal stretches are skipped with one ballot.
__global__ __launch_bounds__(64 * kWalkWaves) void k_walk(const Block* __restrict__ blocks,
                                                          const uint2* __restrict__ walkSegs, uint32_t nwalk,
                                                          const uint32_t* __restrict__ chosen, uint64_t matchBase,
                                                          uint32_t* __restrict__ slotsAll, uint4* __restrict__ state,
                                                          int* __restrict__ status)
{
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * kWalkWaves + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  const uint32_t* L = chosen + (B.start - matchBase);
  uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kWalkCap) + kWalkCap;
  const uint32_t a = ws.y * kWalkSeg;
  const uint32_t aNext = a + kWalkSeg < n ? a + kWalkSeg : n;

  // A window of 64 positions at a time, on the vector unit: lane l steps to l + max(1, chosen[l])
  // (F1, 64 = out of the window), F2 .. F32 by doubling (ds_bpermute), and every lane finds the last
  // path position at or below itself by binary lifting from the entry; the lanes that find themselves
  // are the path, its matches go to the slots compacted by mbcnt.  A window without a match from the
  // entry on is skipped with one ballot.
  auto ldw = [&](uint32_t b) -> uint32_t {
    const uint32_t i = b + lane;
    return L[i < n ? i : n - 1u];
  };
  uint32_t wbase = a, e = 0, m = 0, exitPos = aNext;
  uint32_t wL = ldw(a), nL = ldw(a + 64);
  while (true) {
    const uint32_t lim = aNext - wbase < 64u ? aNext - wbase : 64u;  // window positions before aNext
    const uint32_t len = wbase + lane < n && wL > 1u ? wL : 1u;
    const uint64_t mm = __ballot(len > 1u && lane >= e && lane < lim);
    uint32_t next, lastLen = 1;
    if (mm == 0) {
      next = wbase + lim;  // literals carry the path out of the window (or to aNext)
    } else {
      uint32_t F[6];
      F[0] = lane + len < 64u ? lane + len : 64u;
#pragma unroll
      for (int k = 1; k < 6; k++) {
        const uint32_t g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(F[k - 1] << 2), (int)F[k - 1]);
        F[k] = F[k - 1] >= 64u ? 64u : g;
      }
      uint32_t x = e;
      {
        const uint32_t y = rdlane(F[5], e);
        x = y <= lane ? y : x;
      }
#pragma unroll
      for (int k = 4; k >= 0; k--) {
        const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(x << 2), (int)F[k]);
        x = y <= lane ? y : x;
      }
      const bool rec = x == lane && len > 1u && lane < lim;
      const uint64_t rb = __ballot(rec);
      const uint32_t cnt = (uint32_t)__builtin_popcountll(rb);
      if (m + cnt > kWalkCap) {
        if (lane == 0) atomicOr(status, kStInvariant);
        break;
      }
      if (rec) slots[m + __builtin_amdgcn_mbcnt_hi((uint32_t)(rb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rb, 0u))] = wbase + lane;
      m += cnt;
      const uint32_t p = rdlane(x, lim - 1u);  // the last path position before lim
      lastLen = rdlane(len, p);
      next = wbase + p + lastLen;
    }
    if (next >= aNext) {
      exitPos = lastLen > 1u ? next : aNext;
      break;
    }
    const uint32_t nb = next & ~63u;
    wL = nb == wbase + 64u ? nL : ldw(nb);
    nL = ldw(nb + 64u);
    wbase = nb;
    e = next & 63u;
  }
  if (lane == 0) state[idx] = make_uint4(kWalkCap, kWalkCap + m, exitPos, 0u);
}

// Sub-segment repair.  Sub-segment k's walk is exact when the true path enters it at a position the
// speculative walk also visits; otherwise the path is walked again from its true entry until it meets
// the speculative path, and the repaired matches go in front of the speculative matches that survive.
// The true entry of k is the true exit of k - 1, which is the speculative exit of k - 1 whenever k - 1
// needed no repair or its repaired path met the speculative one (almost always).  So:
//   k_walk_fix_spec   one wavefront per sub-segment k >= 1 repairs k from k - 1's SPECULATIVE exit, all
//                     at once; the repaired matches go to the free lower half of k's slots and a
//                     record (final start, count, exit, the entry assumed) to `rec`;
//   k_walk_fix_commit one wavefront per block checks the assumed entries against the true exits 64
//                     sub-segments at a time, moves the repaired matches of every sub-segment whose
//                     assumption held into place, and repairs the others again serially
//                     (walk_repair) from their true entry.
// walk_repair: the repair of sub-segment idx from `entry` (wave-uniform).  Returns the record; the
// repaired matches are in fix[0, rec.y) (LDS).
struct WalkRepair {
  const uint32_t* L;
  const uint32_t* slots;  // the sub-segment's 2 * kWalkCap slots
  uint32_t lane;
  __device__ __forceinline__ uint4 run(uint32_t* fix, uint32_t a, uint32_t aNext, uint4 st, uint32_t entry, int* status) const
  {
    const uint32_t m = st.y - kWalkCap;
    if (entry == a) return make_uint4(st.x, 0u, st.z, entry);
    if (entry >= aNext) return make_uint4(st.y, 0u, entry, entry);
    // i = first speculative match at or after p (wave-parallel over 64 slots at a time)
    auto first_at = [&](uint32_t from, uint32_t p) -> uint32_t {
      for (uint32_t b = from; b < m; b += 64) {
        const uint64_t ge = __ballot(b + lane < m && slots[kWalkCap + b + lane] >= p);
        if (ge) return b + (uint32_t)__builtin_ctzll(ge);
      }
      return m;
    };
    // q lies strictly inside speculative match i - 1
    auto inside = [&](uint32_t i, uint32_t q) -> bool {
      if (i == 0) return false;
      const uint32_t pj = slots[kWalkCap + i - 1];
      return pj + L[pj] > q;
    };
    uint32_t i = first_at(0, entry);
    if (!inside(i, entry)) return make_uint4(kWalkCap + i, 0u, st.z, entry);
    uint32_t q = entry, f = 0;
    bool merged = false;
    while (q < aNext) {
      const uint32_t lq = L[q];
      if (lq > 1u) {
        if (f >= kWalkCap) {
          if (lane == 0) atomicOr(status, kStInvariant);
          break;
        }
        if (lane == 0) fix[f] = q;
        f++;
        q += lq;
      } else {
        q++;
      }
      i = first_at(i, q);
      if (q < aNext && !inside(i, q)) {
        merged = true;
        break;
      }
    }
    const uint32_t iMerge = merged ? i : m;
    return make_uint4(kWalkCap + iMerge - f, f, merged ? st.z : q, entry);
  }
};

__global__ __launch_bounds__(64 * kWalkWaves) void k_walk_fix_spec(const Block* __restrict__ blocks,
                                                                   const uint2* __restrict__ walkSegs, uint32_t nwalk,
                                                                   const uint32_t* __restrict__ chosen, uint64_t matchBase,
                                                                   uint32_t* __restrict__ slotsAll,
                                                                   const uint4* __restrict__ state, uint4* __restrict__ rec,
                                                                   int* __restrict__ status)
{
  __shared__ uint32_t fixAll[kWalkWaves][kWalkCap];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * kWalkWaves + wave;
  if (idx >= nwalk) return;
  const uint2 ws = walkSegs[idx];
  if (ws.y == 0) return;
  const uint32_t lane = threadIdx.x & 63;
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  const uint32_t a = ws.y * kWalkSeg, aNext = a + kWalkSeg < n ? a + kWalkSeg : n;
  uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kWalkCap);
  const WalkRepair W{chosen + (B.start - matchBase), slots, lane};
  uint32_t* fix = fixAll[wave];
  // k_walk's exit of k - 1 (this kernel writes no state)
  const uint4 r = W.run(fix, a, aNext, state[idx], state[idx - 1].z, status);
  __builtin_amdgcn_wave_barrier();  // lane 0's fix[] stores before the other lanes read them
  // repaired matches to the lower half [0, f): it holds nothing k_walk wrote
  for (uint32_t t = lane; t < r.y; t += 64) slots[t] = fix[t];
  if (lane == 0) rec[idx] = r;
}

__global__ __launch_bounds__(64) void k_walk_fix_commit(const Block* __restrict__ blocks, const uint32_t* __restrict__ chosen,
                                                        uint64_t matchBase, uint32_t* __restrict__ slotsAll,
                                                        uint4* __restrict__ state, const uint4* __restrict__ rec,
                                                        int* __restrict__ status)
{
  __shared__ uint32_t fix[kWalkCap];
  const Block B = blocks[blockIdx.x];
  if (B.walkCount < 2) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = (uint32_t)(B.end - B.start);
  const uint32_t* L = chosen + (B.start - matchBase);
  uint32_t T = state[B.walkFirst].z;  // true exit of sub-segment 0 (walked from the block start)
  for (uint32_t k0 = 1; k0 < B.walkCount; k0 += 64) {
    const uint32_t cnt = B.walkCount - k0 < 64u ? B.walkCount - k0 : 64u;
    const uint32_t idxL = B.walkFirst + k0 + lane;
    const uint4 r = lane < cnt ? rec[idxL] : make_uint4(0, 0, 0, 0);
    uint32_t cur = 0;
    while (cur < cnt) {
      // lane j assumed entry r.w; its true entry is the exit of lane j - 1 (T for the first open lane)
      uint32_t prevExit = __shfl_up(r.z, 1, 64);
      if (lane == cur) prevExit = T;
      const uint64_t bad = __ballot(lane >= cur && lane < cnt && r.w != prevExit);
      const uint32_t js = bad ? (uint32_t)__builtin_ctzll(bad) : cnt;
      if (lane >= cur && lane < js) {
        // the assumption held: move the repaired matches in place (destination above the source)
        uint32_t* slots = slotsAll + (uint64_t)idxL * (2 * kWalkCap);
        for (uint32_t t = r.y; t-- > 0;) slots[r.x + t] = slots[t];
        uint32_t* s32 = reinterpret_cast<uint32_t*>(state + idxL);
        s32[0] = r.x;
        s32[2] = r.z;
      }
      if (js == cnt) {
        T = rdlane(r.z, cnt - 1u);
        break;
      }
      // sub-segment k0 + js entered elsewhere: repaired again from its true entry
      const uint32_t idx = B.walkFirst + k0 + js;
      const uint32_t a = (k0 + js) * kWalkSeg, aNext = a + kWalkSeg < n ? a + kWalkSeg : n;
      uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kWalkCap);
      const WalkRepair W{L, slots, lane};
      const uint4 st = state[idx];
      const uint4 rr = W.run(fix, a, aNext, st, rdlane(prevExit, js), status);
      __syncthreads();
      for (uint32_t t = lane; t < rr.y; t += 64) slots[rr.x + t] = fix[t];
      if (lane == 0) state[idx] = make_uint4(rr.x, st.y, rr.z, 0u);
      __syncthreads();
      T = rr.z;
      cur = js + 1;
    }
  }
}

__device__ __forceinline__ uint64_t token_bytes(uint64_t lits, uint32_t mlen, bool last)
{
  uint64_t b = 1 + lits + (lits >= 15 ? (lits - 15) / 255 + 1 : 0);
  if (!last) {
    const int64_t mcode = (int64_t)mlen - kMinMatch;
    b += 2 + (mcode >= 15 ? (uint64_t)(mcode - 15) / 255 + 1 : 0);
  }
  return b;
}

// ================================================================================================
// k_scan: block offsets in the frame (header, then each block's word + payload, then the end mark)
// ================================================================================================
__global__ __launch_bounds__(1024) void k_scan(const uint32_t* __restrict__ blockBytes, uint32_t nblocks,
                                               uint64_t* __restrict__ offsets)
{
  __shared__ uint64_t s_carry;
  __shared__ uint32_t s_w[16];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nblocks; base += 1024) {
    const uint32_t i = base + tid;
    const uint32_t v = i < nblocks ? (blockBytes[i] & 0x7FFFFFFFu) : 0u;
    const uint32_t incl = wave_incl_scan_add(v);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint64_t pre = s_carry;
    for (uint32_t w = 0; w < wave; w++) pre += s_w[w];
    if (i < nblocks) offsets[i] = pre + incl - v;
    __syncthreads();
    if (tid == 1023) s_carry = pre + incl;
    __syncthreads();
  }
  if (tid == 0) offsets[nblocks] = s_carry;
}

constexpr uint64_t kOwnLits = 64;  // longer literal runs are copied by the whole workgroup

// ================================================================================================
// Frame assembly by walk sub-segment (kWalkSeg positions), so that large blocks fill the GPU too:
//   k_seg_scan    per block: exclusive scans over its sub-segments of the match counts (token base)
//                 and of the match ends (the end of the last match before the sub-segment)
//   k_seg_tokens  per sub-segment: its tokens (literal run + match, smallz4.h:259-371), their byte
//                 sizes summed; the block's last sub-segment adds the closing literal run
//   k_block_bytes per block: byte offsets of the sub-segments, encoded size, stored/compressed
//                 decision (smallz4.h:764-771)
//   k_scan        block offsets in the frame
//   k_write_seg   per sub-segment: its tokens (or its raw bytes) at their place in the frame
// ================================================================================================
constexpr int kAsmThreads = 1024;
constexpr int kSegWaves = 4;  // sub-segments per k_seg_tokens / k_write_seg workgroup

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// info[idx] = (token base, end of the last match before, byte size, byte offset) per sub-segment
__global__ __launch_bounds__(kAsmThreads) void k_seg_scan(const Block* __restrict__ blocks, const uint32_t* __restrict__ chosen,
                                                          uint64_t matchBase, const uint32_t* __restrict__ slotsAll,
                                                          const uint4* __restrict__ state, uint4* __restrict__ info)
{
  __shared__ uint32_t s_sum[kAsmThreads / 64], s_max[kAsmThreads / 64];
  const Block B = blocks[blockIdx.x];
  const uint32_t* L = chosen + (B.start - matchBase);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t carrySum = 0, carryMax = 0;
  for (uint32_t k0 = 0; k0 < B.walkCount; k0 += kAsmThreads) {
    const uint32_t k = k0 + tid;
    const bool valid = k < B.walkCount;
    const uint32_t idx = B.walkFirst + k;
    uint32_t cnt = 0, lastEnd = 0;
    if (valid) {
      const uint4 st = state[idx];
      cnt = st.y - st.x;
      if (cnt) {
        const uint32_t p = slotsAll[(uint64_t)idx * (2 * kWalkCap) + st.y - 1];
        lastEnd = p + L[p];
      }
    }
    const uint32_t incS = wave_incl_scan_add(cnt), incM = wave_incl_scan_max(lastEnd);
    uint32_t prevM = __shfl_up(incM, 1, 64);
    if (lane == 0) prevM = 0;
    if (lane == 63) {
      s_sum[wave] = incS;
      s_max[wave] = incM;
    }
    __syncthreads();
    uint32_t preS = carrySum, preM = carryMax;
    for (uint32_t w = 0; w < wave; w++) {
      preS += s_sum[w];
      preM = s_max[w] > preM ? s_max[w] : preM;
    }
    if (valid) info[idx] = make_uint4(preS + incS - cnt, prevM > preM ? prevM : preM, 0u, 0u);
    for (uint32_t w = 0; w < kAsmThreads / 64; w++) {
      carrySum += s_sum[w];
      carryMax = s_max[w] > carryMax ? s_max[w] : carryMax;
    }
    __syncthreads();
  }
}

// tokens of one sub-segment; blockTail[b] = (matches of the block, bytes of its closing literal run)
__global__ __launch_bounds__(64 * kSegWaves) void k_seg_tokens(const Block* __restrict__ blocks, const uint2* __restrict__ walkSegs,
                                                              uint32_t nwalk, const uint32_t* __restrict__ chosen,
                                                              const uint16_t* __restrict__ mdist, uint64_t matchBase,
                                                              const uint32_t* __restrict__ slotsAll, const uint4* __restrict__ state,
                                                              uint4* __restrict__ info, Token* __restrict__ tokAll,
                                                              uint2* __restrict__ blockTail)
{
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * kSegWaves + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  const Block B = blocks[ws.x];
  const uint32_t n = (uint32_t)(B.end - B.start);
  const uint32_t* L = chosen + (B.start - matchBase);
  const uint16_t* D = mdist + (B.start - matchBase);
  const uint4 st = state[idx];
  const uint4 inf = info[idx];
  const uint32_t m = st.y - st.x;
  const uint32_t* slots = slotsAll + (uint64_t)idx * (2 * kWalkCap);
  Token* tok = tokAll + B.tokOff + inf.x;
  uint32_t carryEnd = inf.y, bytes = 0;
  // loads run ahead: the next batch's match positions, then their lengths and distances
  uint32_t pN = lane < m ? slots[st.x + lane] : 0u;
  uint32_t LN = lane < m ? L[pN] : 0u, DN = lane < m ? (uint32_t)D[pN] : 0u;
  uint32_t pNN = 64u + lane < m ? slots[st.x + 64u + lane] : 0u;
  for (uint32_t c0 = 0; c0 < m; c0 += 64) {
    const uint32_t t = c0 + lane;
    const bool valid = t < m;
    uint32_t p, Lm, Dm;
    asm volatile("v_mov_b32 %0, %1" : "=v"(p) : "v"(pN));
    asm volatile("v_mov_b32 %0, %1" : "=v"(Lm) : "v"(LN));
    asm volatile("v_mov_b32 %0, %1" : "=v"(Dm) : "v"(DN));
    pN = pNN;
    LN = t + 64u < m ? L[pN] : 0u;
    DN = t + 64u < m ? (uint32_t)D[pN] : 0u;
    pNN = t + 128u < m ? slots[st.x + t + 128u] : 0u;
    const uint32_t end = p + Lm;
    uint32_t prev = __shfl_up(end, 1, 64);
    if (lane == 0) prev = carryEnd;
    uint32_t sz = 0;
    if (valid) {
      const uint32_t lits = p - prev;
      tok[t] = Token{lits ? prev : 0u, lits, Lm, Dm};
      sz = (uint32_t)token_bytes(lits, Lm, false);
    }
    bytes += wave_sum_u32(sz);
    carryEnd = rdlane(end, m - c0 < 64 ? m - c0 - 1 : 63);
  }
  if (lane == 0) info[idx].z = bytes;
  if (ws.y + 1 == B.walkCount && lane == 0) {
    // the closing literal run (kTokLast)
    const uint32_t M = inf.x + m;
    tokAll[B.tokOff + M] = Token{carryEnd, n - carryEnd, 0u, kTokLast};
    blockTail[ws.x] = make_uint2(M, (uint32_t)token_bytes(n - carryEnd, 0, true));
  }
}

// per block: byte offsets of its sub-segments, its encoded size and the stored/compressed decision
__global__ __launch_bounds__(kAsmThreads) void k_block_bytes(const Block* __restrict__ blocks, uint32_t maxChain,
                                                             uint4* __restrict__ info, const uint2* __restrict__ blockTail,
                                                             uint32_t* __restrict__ ntokOut, uint32_t* __restrict__ blockBytes,
                                                             int* __restrict__ status)
{
  __shared__ uint32_t s_sum[kAsmThreads / 64];
  const Block B = blocks[blockIdx.x];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t n = B.end - B.start;
  const bool stored = maxChain == 0;
  const bool legacy = (B.flags & kBlkLegacy) != 0;
  uint64_t enc = 0;
  uint32_t ntok = 0;
  if (!stored) {
    uint32_t carry = 0;
    for (uint32_t k0 = 0; k0 < B.walkCount; k0 += kAsmThreads) {
      const uint32_t k = k0 + tid;
      const bool valid = k < B.walkCount;
      const uint32_t idx = B.walkFirst + k;
      const uint32_t b = valid ? info[idx].z : 0u;
      const uint32_t inc = wave_incl_scan_add(b);
      if (lane == 63) s_sum[wave] = inc;
      __syncthreads();
      uint32_t pre = carry;
      for (uint32_t w = 0; w < wave; w++) pre += s_sum[w];
      if (valid) info[idx].w = pre + inc - b;
      for (uint32_t w = 0; w < kAsmThreads / 64; w++) carry += s_sum[w];
      __syncthreads();
    }
    const uint2 tail = blockTail[blockIdx.x];
    enc = (uint64_t)carry + tail.y;
    ntok = tail.x + 1;
  }
  const bool useEnc = (enc < n && !stored) || legacy;
  const uint32_t bytes = (uint32_t)(useEnc ? enc : n);
  // a block's tokens fit its Token slots ((n / 2 + 4), one match per >= 4 bytes) and its size word
  if (tid == 0 && (ntok > n / 2 + 4 || (useEnc ? enc : n) >= 0x7FFFFFFBull)) atomicOr(status, kStInvariant);
  if (tid == 0) {
    ntokOut[blockIdx.x] = useEnc ? ntok : 0u;
    blockBytes[blockIdx.x] = (useEnc ? 0u : 0x80000000u) | (bytes + 4u);
  }
}

// one wavefront per sub-segment writes its tokens (or its raw bytes) into the frame
__global__ __launch_bounds__(64 * kSegWaves) void k_write_seg(const uint8_t* __restrict__ in, const Block* __restrict__ blocks,
                                                             const uint2* __restrict__ walkSegs, uint32_t nwalk,
                                                             const uint4* __restrict__ state, const uint4* __restrict__ info,
                                                             const Token* __restrict__ tokAll, const uint32_t* __restrict__ ntokAll,
                                                             const uint32_t* __restrict__ blockBytes,
                                                             const uint64_t* __restrict__ offsets, uint8_t* __restrict__ out,
                                                             uint64_t headerLen)
{
  __shared__ uint32_t s_ld[kSegWaves][64], s_ls[kSegWaves][64], s_ll[kSegWaves][64];  // long literal runs
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t idx = blockIdx.x * kSegWaves + wave;
  if (idx >= nwalk) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint2 ws = walkSegs[idx];
  const Block B = blocks[ws.x];
  const uint64_t n = B.end - B.start;
  const uint32_t bb = blockBytes[ws.x];
  const bool raw = (bb & 0x80000000u) != 0;
  uint8_t* dst = out + headerLen + offsets[ws.x];
  if (ws.y == 0 && lane == 0) {
    const uint32_t word = ((bb & 0x7FFFFFFFu) - 4u) | (raw ? 0x80000000u : 0u);
    dst[0] = (uint8_t)word;
    dst[1] = (uint8_t)(word >> 8);
    dst[2] = (uint8_t)(word >> 16);
    dst[3] = (uint8_t)(word >> 24);
  }
  dst += 4;
  const uint8_t* src = in + B.start;
  if (raw) {
    const uint64_t lo = (uint64_t)ws.y * kWalkSeg, hi = lo + kWalkSeg < n ? lo + kWalkSeg : n;
    for (uint64_t j = lo + lane; j < hi; j += 64) dst[j] = src[j];
    return;
  }
  if (ntokAll[ws.x] == 0) return;  // legacy frame at level 0: an empty compressed block
  const uint4 st = state[idx], inf = info[idx];
  const uint32_t count = (st.y - st.x) + (ws.y + 1 == B.walkCount ? 1u : 0u);
  const Token* tok = tokAll + B.tokOff + inf.x;
  uint64_t carry = inf.w;
  for (uint32_t c0 = 0; c0 < count; c0 += 64) {
    const uint32_t t = c0 + lane;
    const bool valid = t < count;
    Token T{0, 0, 0, 0};
    uint64_t sz = 0;
    bool last = false;
    if (valid) {
      T = tok[t];
      last = (T.dist & kTokLast) != 0;
      sz = token_bytes(T.lits, T.mlen, last);
    }
    uint64_t incl = sz;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t o = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += o;
    }
    const uint64_t off = carry + incl - sz;
    carry += __shfl(incl, 63, 64);
    bool isLong = false;
    if (valid) {
      uint8_t* o = dst + off;
      const int64_t mcode = last ? 0 : (int64_t)T.mlen - kMinMatch;
      const uint8_t tk = (uint8_t)(mcode < 15 ? mcode : 15);
      const uint64_t lits = T.lits;
      if (lits < 15) {
        *o++ = (uint8_t)(tk | (lits << 4));
      } else {
        *o++ = (uint8_t)(tk | 0xF0);
        uint64_t v = lits - 15;
        while (v >= 255) { *o++ = 255; v -= 255; }
        *o++ = (uint8_t)v;
      }
      if (lits <= kOwnLits) {
        // 8 bytes per round: three aligned dwords loaded together, then byte stores (one load latency
        // per 8 literals instead of one per literal)
        // (the three dwords lie inside the block, the input buffer's alignment taken into account)
        for (uint32_t k = 0; k < (uint32_t)lits; k += 8) {
          const uint64_t a = (uint64_t)T.litFrom + k;
          const uint32_t nk = (uint32_t)lits - k < 8u ? (uint32_t)lits - k : 8u;
          const uintptr_t ab = reinterpret_cast<uintptr_t>(src + a);
          if (a >= 4u && a + 12u <= n) {
            const uint32_t* wp = reinterpret_cast<const uint32_t*>(ab & ~(uintptr_t)3);
            const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2];
            const uint32_t sh = (uint32_t)(ab & 3u);
            const uint32_t v0 = __builtin_amdgcn_alignbyte(w1, w0, sh), v1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
#pragma unroll
            for (uint32_t b = 0; b < 8; b++)
              if (b < nk) o[k + b] = (uint8_t)((b < 4 ? v0 : v1) >> (8 * (b & 3)));
          } else {
            for (uint32_t b = 0; b < nk; b++) o[k + b] = src[a + b];
          }
        }
      } else {
        isLong = true;  // copied by the whole wavefront below
        s_ld[wave][lane] = (uint32_t)(o - dst);
        s_ls[wave][lane] = T.litFrom;
        s_ll[wave][lane] = (uint32_t)lits;
      }
      o += lits;
      if (!last) {
        const uint32_t dd = T.dist & 0xFFFFu;
        o[0] = (uint8_t)(dd & 0xFF);
        o[1] = (uint8_t)(dd >> 8);
        o += 2;
        if (mcode >= 15) {
          uint64_t v = (uint64_t)(mcode - 15);
          while (v >= 255) { *o++ = 255; v -= 255; }
          *o++ = (uint8_t)v;
        }
      }
    }
    uint64_t longs = __ballot(isLong);
    while (longs) {
      const uint32_t l = (uint32_t)__builtin_ctzll(longs);
      longs &= longs - 1;
      uint8_t* d = dst + s_ld[wave][l];
      const uint8_t* ls = src + s_ls[wave][l];
      const uint32_t len = s_ll[wave][l];
      for (uint32_t k = lane; k < len; k += 64) d[k] = ls[k];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
void launch_runs(const uint8_t* in, const Block* blocks, uint32_t nblocks, Interval* iv, uint32_t* ivCount, hipStream_t s)
{
  if (nblocks) hipLaunchKernelGGL(k_runs, dim3(nblocks), dim3(256), 0, s, in, blocks, iv, ivCount);
}


uint32_t dp_side_positions() { return kDpSideStride; }

uint32_t find_lds_bytes() { return 65536 + 16; }

void launch_find(int pass, const uint8_t* in, const Segment* segs, uint32_t nsegs, const Block* blocks, const Interval* iv,
                 const uint32_t* ivCount, uint2* compact, uint2* scratch, uint32_t* rank, uint32_t maxChain,
                 uint32_t* mlen, uint16_t* mdist, uint64_t matchBase, uint32_t* longBits, uint32_t* segLong,
                 uint32_t* longFlag, uint32_t* specLen, uint32_t* specDist, uint64_t* segTail, bool ldsWindow,
                 hipStream_t s)
{
  static_assert(sizeof(SortLds) <= 65536, "the fused sort's shared memory must fit the window buffer");
  static_assert(kOutTile * 4u <= 65536u + 16u, "a result tile must fit the window buffer");
  if (!nsegs) return;
  const bool unlimited = maxChain >= 65535u;
  if (ldsWindow) {
    // dynamic-LDS limits are per function and device: set them on every launch (a host-side call,
    // no synchronisation) rather than caching them process-wide
    const void* fn = pass == 1 ? (const void*)k_find_sorted_lds
                     : unlimited ? (const void*)k_find_long9_lds : (const void*)k_find<true>;
    hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)find_lds_bytes());
    if (pass == 1)
      hipLaunchKernelGGL(k_find_sorted_lds, dim3(nsegs), dim3(kFindThreads), find_lds_bytes(), s, in, segs, blocks, iv,
                         ivCount, compact, maxChain, mlen, mdist, matchBase, longBits, segLong, scratch, rank);
    else if (unlimited) {
      // big key groups first (left-maximal candidates + text-order prefix maximum), then pass 2
      hipFuncSetAttribute((const void*)k_find_big<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)find_lds_bytes());
      for (uint32_t resolve = 0; resolve < 2; resolve++)
        hipLaunchKernelGGL(k_find_big<true>, dim3(nsegs), dim3(kFindThreads), find_lds_bytes(), s, in, segs, blocks, iv, ivCount,
                           compact, scratch, longBits, segLong, mlen, mdist, matchBase, specLen, segTail, specDist, rank, longFlag, resolve);
      for (int fix = 0; fix < 2; fix++)
        hipLaunchKernelGGL(k_find_long9_lds, dim3(nsegs), dim3(kFindThreads), find_lds_bytes(), s, in, segs, blocks, iv,
                           ivCount, compact, scratch, rank, longBits, segLong, mlen, mdist, matchBase, longFlag, specLen,
                           specDist, fix);
    } else
      hipLaunchKernelGGL(k_find<true>, dim3(nsegs), dim3(kFindThreads), find_lds_bytes(), s, in, segs, blocks, iv, ivCount,
                         compact, rank, maxChain, mlen, mdist, matchBase, longFlag, segLong);
  } else {
    if (pass == 1) {
      // the sort and the text-order result tiles use the same buffer: at least 64 KiB
      const uint32_t lds = kOutTile * 4u;
      hipFuncSetAttribute((const void*)k_find_sorted_hbm, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(k_find_sorted_hbm, dim3(nsegs), dim3(kFindThreads), lds, s, in, segs, blocks, iv, ivCount,
                         compact, maxChain, mlen, mdist, matchBase, longBits, segLong, scratch, rank);
    }
    else if (unlimited) {
      // (the segment's own 64 Ki targets and 64 bytes more)
      const uint32_t bigLds = 65536u + 256u;
      hipFuncSetAttribute((const void*)k_find_big<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bigLds);
      for (uint32_t resolve = 0; resolve < 2; resolve++)
        hipLaunchKernelGGL(k_find_big<false>, dim3(nsegs), dim3(kFindThreads), bigLds, s, in, segs, blocks, iv, ivCount,
                           compact, scratch, longBits, segLong, mlen, mdist, matchBase, specLen, segTail, specDist, rank, longFlag, resolve);
      // (the segment's own 64 Ki targets and 64 bytes more)
      const uint32_t l9Lds = 65536u + 256u;
      hipFuncSetAttribute((const void*)k_find_long9_hbm, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l9Lds);
      for (int fix = 0; fix < 2; fix++)
        hipLaunchKernelGGL(k_find_long9_hbm, dim3(nsegs), dim3(kFindThreads), l9Lds, s, in, segs, blocks, iv, ivCount,
                           compact, scratch, rank, longBits, segLong, mlen, mdist, matchBase, longFlag, specLen, specDist,
                           fix);
    }
    else
      hipLaunchKernelGGL(k_find<false>, dim3(nsegs), dim3(kFindThreads), 0, s, in, segs, blocks, iv, ivCount, compact, rank,
                         maxChain, mlen, mdist, matchBase, longFlag, segLong);
  }
}

void launch_prep(const uint8_t* in, const Block* blocks, uint32_t nblocks, Interval* iv, uint32_t* ivCount, uint32_t maxChain,
                 uint32_t* mlen, uint16_t* mdist, uint64_t matchBase, uint32_t* sel, const uint32_t* longFlag, int* status,
                 hipStream_t s)
{
  if (nblocks)
    hipLaunchKernelGGL(k_prep, dim3(nblocks), dim3(64), 0, s, in, blocks, iv, ivCount, maxChain, mlen, mdist, matchBase, sel,
                       longFlag, status);
}

void launch_lazy(const uint8_t* in, const Block* blocks, uint32_t nblocks, const uint2* walkSegs, uint32_t nwalk,
                 Interval* iv, uint32_t* ivCount, const uint32_t* longFlag, uint32_t* mlen, const uint16_t* mdist,
                 uint64_t matchBase, uint32_t* slots, uint4* state, uint32_t* firstBad, int* status, hipStream_t s)
{
  if (!nblocks || !nwalk) return;
  const uint32_t grid = (nwalk + kWalkWaves - 1) / kWalkWaves;
  hipLaunchKernelGGL(k_lazy_walk, dim3(grid), dim3(64 * kWalkWaves), 0, s, blocks, walkSegs, nwalk, iv, ivCount, mlen,
                     matchBase, slots, state);
  hipLaunchKernelGGL(k_lazy_join, dim3(grid), dim3(64 * kWalkWaves), 0, s, blocks, walkSegs, nwalk, iv, ivCount, mlen,
                     matchBase, slots, state);
  hipLaunchKernelGGL(k_lazy_fix, dim3(nblocks), dim3(64), 0, s, blocks, iv, ivCount, mlen, matchBase, slots, state, status);
  hipLaunchKernelGGL(k_lazy_clear, dim3(grid), dim3(64 * kWalkWaves), 0, s, blocks, walkSegs, nwalk, iv, ivCount, mlen,
                     matchBase, slots, state);
  hipMemsetAsync(firstBad, 0xFF, (size_t)nblocks * 4, s);
  hipLaunchKernelGGL(k_lazy_check, dim3(grid), dim3(64 * kWalkWaves), 0, s, in, blocks, walkSegs, nwalk, iv, ivCount, longFlag,
                     mlen, mdist, matchBase, slots, state, firstBad);
  hipLaunchKernelGGL(k_lazy_correct, dim3(nblocks), dim3(64), 0, s, blocks, iv, ivCount, mlen, matchBase, firstBad, status);
}

uint32_t lazy_slots_per_walk() { return 2 * kLazyCap; }

void launch_parse(const uint8_t* in, const Block* blocks, uint32_t nblocks, const DpSeg* dpSegs, uint32_t ndp,
                  uint32_t maxDpCount, const uint32_t* ivCount, uint32_t maxChain, uint32_t* mlen, const uint16_t* mdist, uint64_t matchBase,
                  uint32_t* cost, uint32_t* sel, uint32_t* reach, uint4* segState, const uint32_t* longFlag, uint32_t* rmqUp,
                  uint32_t* rmqDown, uint2* dpSide, uint4* dpRec, int* status, hipStream_t s)
{
  (void)in;
  if (!nblocks) return;
  if (maxChain <= (uint32_t)kGreedyMax || !ndp) return;
  // every segment is parsed by exactly one of the two instantiations (by its block's longFlag)
  hipLaunchKernelGGL(k_dp_spec_lean, dim3((ndp + kSpecWaves - 1) / kSpecWaves), dim3(64 * kSpecWaves), 0, s, blocks, dpSegs,
                     ndp, mlen, mdist, matchBase, cost, sel, reach, segState, longFlag, rmqUp, rmqDown);
  hipLaunchKernelGGL(k_dp_spec_rmq, dim3((ndp + kSpecWaves - 1) / kSpecWaves), dim3(64 * kSpecWaves), 0, s, blocks, dpSegs,
                     ndp, mlen, mdist, matchBase, cost, sel, reach, segState, longFlag, rmqUp, rmqDown);
  hipLaunchKernelGGL(k_dp_fix<true>, dim3(ndp), dim3(64), 0, s, blocks, dpSegs, ndp, mlen, mdist, matchBase, cost, sel,
                     reach, segState, longFlag, rmqUp, rmqDown, dpSide, dpRec, 0u);
  const uint32_t tab = maxDpCount < 1u ? 1u : maxDpCount > kMaxDpSegs ? kMaxDpSegs : maxDpCount;
  hipLaunchKernelGGL(k_dp_fix<false>, dim3(nblocks), dim3(64), 4 * tab * sizeof(uint32_t), s, blocks, dpSegs, ndp, mlen, mdist,
                     matchBase, cost, sel, reach, segState, longFlag, rmqUp, rmqDown, dpSide, dpRec, tab);
}

void launch_emit(const uint8_t* in, const Block* blocks, uint32_t nblocks, const uint2* walkSegs, uint32_t nwalk,
                 uint32_t maxChain, const uint32_t* chosen, const uint16_t* mdist, uint64_t matchBase, uint32_t* walkSlots,
                 uint4* walkState, uint32_t* posList, Token* tokens, uint32_t* ntok, uint32_t* blockBytes,
                 uint64_t* offsets, uint8_t* out, uint64_t headerLen, int* status, hipStream_t s)
{
  if (!nblocks) return;
  if (maxChain > 0 && nwalk) {
    hipLaunchKernelGGL(k_walk, dim3((nwalk + kWalkWaves - 1) / kWalkWaves), dim3(64 * kWalkWaves), 0, s, blocks, walkSegs,
                       nwalk, chosen, matchBase, walkSlots, walkState, status);
  }
  // per-sub-segment scratch in posList (the parse's reach array, free by now): the repair records,
  // then the token counts
  uint4* info = reinterpret_cast<uint4*>(posList);
  if (maxChain > 0 && nwalk) {
    hipLaunchKernelGGL(k_walk_fix_spec, dim3((nwalk + kWalkWaves - 1) / kWalkWaves), dim3(64 * kWalkWaves), 0, s, blocks,
                       walkSegs, nwalk, chosen, matchBase, walkSlots, walkState, info, status);
    hipLaunchKernelGGL(k_walk_fix_commit, dim3(nblocks), dim3(64), 0, s, blocks, chosen, matchBase, walkSlots, walkState, info,
                       status);
  }
  uint2* blockTail = reinterpret_cast<uint2*>(info + nwalk);
  const uint32_t segGrid = (nwalk + kSegWaves - 1) / kSegWaves;
  if (maxChain > 0 && nwalk) {
    hipLaunchKernelGGL(k_seg_scan, dim3(nblocks), dim3(kAsmThreads), 0, s, blocks, chosen, matchBase, walkSlots, walkState, info);
    hipLaunchKernelGGL(k_seg_tokens, dim3(segGrid), dim3(64 * kSegWaves), 0, s, blocks, walkSegs, nwalk, chosen, mdist, matchBase,
                       walkSlots, walkState, info, tokens, blockTail);
  }
  hipLaunchKernelGGL(k_block_bytes, dim3(nblocks), dim3(kAsmThreads), 0, s, blocks, maxChain, info, blockTail, ntok, blockBytes,
                     status);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, blockBytes, nblocks, offsets);
  if (nwalk)
    hipLaunchKernelGGL(k_write_seg, dim3(segGrid), dim3(64 * kSegWaves), 0, s, in, blocks, walkSegs, nwalk, walkState, info, tokens,
                       ntok, blockBytes, offsets, out, headerLen);
}

}  // namespace sz4
