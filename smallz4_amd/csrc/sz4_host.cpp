// sz4_host.cpp -- host driver behind the C ABI in include/smallz4_amd.h.
//
// Builds the block / segment plan for a job, keeps device scratch resident in
// HBM (grow-only, so repeated calls allocate nothing), launches the kernel
// pipeline of sz4_kernels.hip on one HIP stream and assembles the frame.
//
// Two job shapes:
//   * independent blocks (sz4_compress_blocks_device): every block compressed
//     as the reference compresses a stand-alone input -- the data-parallel
//     shape that fills the GPU (BASELINE configs 1-4);
//   * one reference stream (sz4_lz4): the exact block structure of
//     smallz4::compress (smallz4.h:476-813): 4 MiB blocks that see the previous
//     64 KiB, or 8 MiB independent legacy blocks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/smallz4_amd.h"
#include "sz4_internal.h"

using namespace sz4;

namespace {

constexpr uint64_t kPad = 64;                 // bytes of slack after every staged input
constexpr uint64_t kSegTargets = 65536;       // target positions per segment
constexpr uint64_t kBlockMax = 4ull << 20;    // MaxBlockSize (smallz4.h:124)
constexpr uint64_t kBlockMaxLegacy = 8ull << 20;

uint64_t token_capacity(uint64_t n) { return n / 2 + 4; }

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t bytes)
  {
    if (bytes <= cap) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 8 + 4096;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release()
  {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// pinned host memory (the stream path's chunk buffers), grow-only
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t bytes)
  {
    if (bytes <= cap) return hipSuccess;
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release()
  {
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// makes the context's device current for the duration of a call and restores the caller's
struct DeviceGuard {
  int saved = -1;
  explicit DeviceGuard(int device)
  {
    if (hipGetDevice(&saved) != hipSuccess) saved = -1;
    if (saved != device) hipSetDevice(device);
  }
  ~DeviceGuard()
  {
    int now = -1;
    if (saved >= 0 && hipGetDevice(&now) == hipSuccess && now != saved) hipSetDevice(saved);
  }
};

uint32_t xxh32_small(const uint8_t* d, size_t n)
{
  const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P5 = 374761393u;
  uint32_t h = P5 + (uint32_t)n;
  for (size_t i = 0; i < n; i++) {
    h += d[i] * P5;
    h = ((h << 11) | (h >> 21)) * P1;
  }
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

}  // namespace

struct sz4_ctx {
  int device = 0;
  std::string err;
  bool timing = false;
  hipEvent_t ev[kStages + 1] = {};
  float stageMs[kStages] = {};
  uint32_t lastBlocks = 0;
  int stopAfter = 0;
  uint32_t lastChain = 0;
  bool separateSort = false;  // k_sort runs inside k_find_sorted; SZ4_SEPARATE_SORT=1: its own launch

  DevBuf staged, blocks, segs, iv, ivCount, elemA, elemB, rank, mlen, mdist, cost, tokens, ntok, blockBytes, offsets, status;
  DevBuf dpSegs, sel, reach, segState, walkSegs, walkSlots, walkState, longFlag, rmqUp, rmqDown, longBits, segLong, segTail;
  DevBuf dpSide, dpRec;        // the parallel parse-boundary repair: saved speculative values, records
  DevBuf dictLast, dictPrevH, dictPrevX;  // dictionary mode: the reference's hash table and both chains
  DevBuf chunkOut;             // stream path: one chunk's blocks
  DevBuf lazySlots;            // greedy/lazy levels: searched positions per walk sub-segment
  HostBuf hostIn[2], hostOut[2];
  uint64_t streamChunk = 64ull << 20;  // stream path: input bytes per chunk (rounded to whole blocks)
  // stream path, chunk continuation: the previous chunk's last block's final shortcut intervals
  // (ghost slot nblocks of iv/ivCount, B.prev of the first block) and dictionary-mode state
  std::vector<Interval> ghostIv;
  bool ghost = false;
  uint32_t dictCont = 0, dictShift = 0, dictLow0 = 0;
  DevBuf unBlk, unMeta, unFlags, unFrame, unDict, unOut, unSeq;  // decoder (sz4_unlz4*)
  std::vector<UnBlock> hUn;
  int64_t dictBack = -1;       // >= 0: dictionary mode, first insertion this far before the first block
  int dictLegacy = 0;

  std::vector<Block> hBlocks;
  std::vector<Segment> hSegs;
  std::vector<DpSeg> hDp;
  std::vector<uint2> hWalk;
  uint64_t elemTotal = 0, rankTotal = 0, tokTotal = 0;
  bool ldsWindow = false;
  // the plan's device copy (blocks, segments, parse segments, walk sub-segments) is uploaded once per
  // plan: repeated calls on the same shape skip the uploads
  uint64_t planVersion = 0, uploadedVersion = ~0ull;
  const void* uploadedAt[4] = {};
  uint32_t hybridLds = 0;  // k_find_long9's LDS staging when the window is not LDS-resident
  // plan cache for sz4_compress_blocks_device
  uint64_t planN = ~0ull;
  uint32_t planBS = 0;
  std::vector<uint32_t> hostBytes;

  hipStream_t stream = nullptr;  // the stream path's own stream
  bool pooled = false;           // handed out by sz4_acquire
  std::mutex* poolMu = nullptr;
  std::vector<sz4_ctx*>* poolIdle = nullptr;

  std::vector<DevBuf*> all_buffers()
  {
    return {&staged, &blocks, &segs, &iv, &ivCount, &elemA, &elemB, &rank, &mlen, &mdist, &cost, &tokens, &ntok,
            &blockBytes, &offsets, &status, &dpSegs, &sel, &reach, &segState, &walkSegs, &walkSlots, &walkState,
            &longFlag, &rmqUp, &rmqDown, &longBits, &segLong, &segTail, &dpSide, &dpRec, &dictLast, &dictPrevH, &dictPrevX, &chunkOut, &lazySlots,
            &unBlk, &unMeta, &unFlags, &unFrame, &unDict, &unOut, &unSeq};
  }

  int fail(int code, const char* what, hipError_t e = hipSuccess)
  {
    char buf[512];
    if (e != hipSuccess) snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else snprintf(buf, sizeof buf, "%s", what);
    err = buf;
    return code;
  }
};

namespace {

// Targets of block B are positions [start, end - 11) (smallz4.h:629); the window of a segment
// reaches back 64 KiB - 1 but never below the block's lowest visible byte.
void add_segments(sz4_ctx* c, uint32_t bi)
{
  const Block& B = c->hBlocks[bi];
  if (B.end - B.start < (uint64_t)kTailNoMatch) return;
  const uint64_t t1 = B.end - kTailNoMatch + 1;
  for (uint64_t s0 = B.start; s0 < t1; s0 += kSegTargets) {
    Segment S{};
    S.s0 = s0;
    S.s1 = std::min(s0 + kSegTargets, t1);
    S.w0 = std::max(B.low, s0 >= kWindow ? s0 - kWindow : 0);
    S.block = bi;
    S.elemOff = c->elemTotal;
    S.rankOff = c->rankTotal;
    c->elemTotal += S.s1 - S.w0;
    c->rankTotal += S.s1 - S.s0;
    c->hSegs.push_back(S);
  }
}

void finish_plan(sz4_ctx* c)
{
  c->planVersion++;
  c->tokTotal = 0;
  for (Block& B : c->hBlocks) {
    B.tokOff = c->tokTotal;
    c->tokTotal += token_capacity(B.end - B.start);
  }
  c->hSegs.clear();
  c->elemTotal = c->rankTotal = 0;
  for (uint32_t b = 0; b < c->hBlocks.size(); b++) add_segments(c, b);
  // token-walk sub-segments: kWalkSeg positions each
  c->hWalk.clear();
  for (uint32_t b = 0; b < c->hBlocks.size(); b++) {
    Block& B = c->hBlocks[b];
    const uint64_t n = B.end - B.start;
    B.walkFirst = (uint32_t)c->hWalk.size();
    B.walkCount = (uint32_t)((n + kWalkSeg - 1) / kWalkSeg);
    for (uint32_t k = 0; k < B.walkCount; k++) c->hWalk.push_back(make_uint2(b, k));
  }
  // parse segments: positions [0, n - 6] of every block longer than 12 bytes, top segment first
  c->hDp.clear();
  for (uint32_t b = 0; b < c->hBlocks.size(); b++) {
    Block& B = c->hBlocks[b];
    const uint64_t n = B.end - B.start;
    B.dpFirst = (uint32_t)c->hDp.size();
    B.dpCount = 0;
    if (n <= (uint64_t)kTailNoMatch) continue;
    const uint64_t top = n - 1 - kTailLiterals;
    uint64_t seg = dp_segment_size(n);
    if (n > 65536) {
      // tuning knob for blocks above 64 KiB: a multiple of 256 (the parse's range-minimum blocks)
      if (const char* e = getenv("SZ4_DP_SIZE")) {
        const uint64_t v = strtoull(e, nullptr, 10);
        if (v >= 1024 && v % 256 == 0 && (n + v - 1) / v <= kMaxDpSegs) seg = v;
      }
    }
    B.dpSize = (uint32_t)seg;
    for (uint64_t hi = top, k = 0;; hi -= seg, k++) {
      const uint64_t lo = hi + 1 >= seg ? hi + 1 - seg : 0;
      c->hDp.push_back(DpSeg{b, (uint32_t)k, (uint32_t)lo, (uint32_t)hi});
      B.dpCount++;
      if (lo == 0) break;
    }
  }
  c->ldsWindow = true;
  c->hybridLds = 0;
  for (const Segment& S : c->hSegs) {
    const Block& B = c->hBlocks[S.block];
    if ((B.end - S.w0 + 8 + 3) / 4 * 4 > find_lds_bytes()) c->ldsWindow = false;
    const uint64_t end = std::min<uint64_t>(S.s1 + 64, B.end + 8);
    c->hybridLds = std::max<uint32_t>(c->hybridLds, (uint32_t)((end - S.w0 + 3) / 4 * 4));
  }
}

int reserve_all(sz4_ctx* c, uint64_t stagedBytes)
{
  const uint64_t nb = c->hBlocks.size();
  hipError_t e = hipSuccess;
  if ((e = c->blocks.reserve(nb * sizeof(Block) + 64)) ||
      (e = c->segs.reserve(c->hSegs.size() * sizeof(Segment) + 64)) ||
      (e = c->iv.reserve((nb + 1) * kMaxIv * sizeof(Interval) + 64)) ||
      (e = c->ivCount.reserve((nb + 1) * 4 + 64)) ||
      (e = c->elemA.reserve(c->elemTotal * sizeof(uint2) + 64)) ||
      (e = c->elemB.reserve(c->elemTotal * sizeof(uint2) + 64)) ||
      (e = c->rank.reserve(c->rankTotal * 4 + 64)) ||
      (e = c->mlen.reserve(stagedBytes * 4 + 64)) ||
      (e = c->mdist.reserve(stagedBytes * 2 + 64)) ||
      (e = c->cost.reserve((stagedBytes + nb + 8) * 4)) ||
      (e = c->tokens.reserve(c->tokTotal * sizeof(Token) + 64)) ||
      (e = c->ntok.reserve(nb * 4 + 64)) ||
      (e = c->blockBytes.reserve(nb * 4 + 64)) ||
      (e = c->offsets.reserve((nb + 1) * 8 + 64)) ||
      (e = c->status.reserve(64)) ||
      (e = c->dpSegs.reserve(c->hDp.size() * sizeof(DpSeg) + 64)) ||
      (e = c->sel.reserve(stagedBytes * 4 + 64)) ||
      (e = c->reach.reserve(stagedBytes * 4 + 64)) ||
      (e = c->segState.reserve(c->hDp.size() * sizeof(uint4) + 64)) ||
      (e = c->dpSide.reserve(c->hDp.size() * dp_side_positions() * sizeof(uint2) + 64)) ||
      (e = c->dpRec.reserve(c->hDp.size() * sizeof(uint4) + 64)) ||
      (e = c->walkSegs.reserve(c->hWalk.size() * sizeof(uint2) + 64)) ||
      (e = c->walkSlots.reserve(c->hWalk.size() * 2 * kWalkCap * 4 + 64)) ||
      (e = c->walkState.reserve(c->hWalk.size() * sizeof(uint4) + 64)) ||
      (e = c->longFlag.reserve(nb * 4 + 64)) ||
      (e = c->longBits.reserve(stagedBytes / 8 + 64)) ||
      (e = c->segLong.reserve(c->hSegs.size() * 4 + 64)) ||
      (e = c->segTail.reserve(c->hSegs.size() * 8 + 64)) ||
      (e = c->rmqUp.reserve((stagedBytes + nb + 8) * 4)) ||
      (e = c->rmqDown.reserve((stagedBytes + nb + 8) * 4)))
    return c->fail(SZ4_E_NOMEM, "device allocation", e);
  return SZ4_OK;
}

void mark(sz4_ctx* c, int i, hipStream_t s)
{
  if (c->timing) hipEventRecord(c->ev[i], s);
}

// run the kernel pipeline over the planned blocks of c->staged; frame goes to `out`
int run_pipeline(sz4_ctx* c, uint32_t maxChain, const uint8_t* hdr, uint64_t hdrLen, bool endMark, uint8_t* out,
                 uint64_t outCap, uint64_t* outSize, hipStream_t s)
{
  const uint32_t nb = (uint32_t)c->hBlocks.size();
  const uint8_t* in = c->staged.as<uint8_t>();
  c->lastChain = maxChain;
  hipError_t e;
  const void* at[4] = {c->blocks.p, c->segs.p, c->dpSegs.p, c->walkSegs.p};
  const bool fresh = c->uploadedVersion == c->planVersion && memcmp(at, c->uploadedAt, sizeof at) == 0;
  if (!fresh &&
      ((e = hipMemcpyAsync(c->blocks.p, c->hBlocks.data(), nb * sizeof(Block), hipMemcpyHostToDevice, s)) ||
       (e = hipMemcpyAsync(c->segs.p, c->hSegs.data(), c->hSegs.size() * sizeof(Segment), hipMemcpyHostToDevice, s)) ||
       (e = hipMemcpyAsync(c->dpSegs.p, c->hDp.data(), c->hDp.size() * sizeof(DpSeg), hipMemcpyHostToDevice, s)) ||
       (e = hipMemcpyAsync(c->walkSegs.p, c->hWalk.data(), c->hWalk.size() * sizeof(uint2), hipMemcpyHostToDevice, s))))
    return c->fail(SZ4_E_DEVICE, "upload plan", e);
  c->uploadedVersion = c->planVersion;
  memcpy(c->uploadedAt, at, sizeof at);
  if ((e = hipMemsetAsync(c->status.p, 0, 4, s)) || (e = hipMemsetAsync(c->longFlag.p, 0, nb * 4, s)))
    return c->fail(SZ4_E_DEVICE, "upload plan", e);
  // ghost slot nb: the previous chunk's last block (only its intervals are read, through B.prev)
  const uint32_t ghostN = c->ghost ? (uint32_t)c->ghostIv.size() : 0u;
  if ((ghostN && (e = hipMemcpyAsync(c->iv.as<Interval>() + (uint64_t)nb * kMaxIv, c->ghostIv.data(),
                                     ghostN * sizeof(Interval), hipMemcpyHostToDevice, s))) ||
      (e = hipMemcpyAsync(c->ivCount.as<uint32_t>() + nb, &ghostN, 4, hipMemcpyHostToDevice, s)))
    return c->fail(SZ4_E_DEVICE, "upload intervals", e);
  const uint32_t ns = (uint32_t)c->hSegs.size();
  Block* dB = c->blocks.as<Block>();
  Segment* dS = c->segs.as<Segment>();
  Interval* dIv = c->iv.as<Interval>();
  uint32_t* dIvN = c->ivCount.as<uint32_t>();

  mark(c, 0, s);
  if (c->dictBack < 0) launch_runs(in, dB, nb, dIv, dIvN, s);
  mark(c, 1, s);
  if (c->dictBack >= 0 && maxChain > 0) {
    // dictionary mode: the reference's sequential match loop (k_dict_matches), then the usual parse
    if ((e = c->dictLast.reserve(sizeof(uint32_t) << 20)) || (e = c->dictPrevH.reserve(2 * 65536)) ||
        (e = c->dictPrevX.reserve(2 * 65536)))
      return c->fail(SZ4_E_NOMEM, "dictionary tables", e);
    launch_dict(in, dB, nb, maxChain, (uint32_t)c->dictBack, c->dictLegacy, c->dictLast.as<uint32_t>(),
                c->dictPrevH.as<uint16_t>(), c->dictPrevX.as<uint16_t>(), c->dictCont, c->dictShift, c->dictLow0,
                c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), c->sel.as<uint32_t>(), c->longFlag.as<uint32_t>(), s);
    mark(c, 2, s);
    mark(c, 3, s);
    mark(c, 4, s);
    if (c->stopAfter == 3) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
  }
  // greedy/lazy levels: k_prep verifies the shortcut intervals k_runs assumed; a corrected block needs
  // another sort/find/prep round (each round checks a longer prefix of it)
  for (uint32_t round = 0; c->dictBack < 0; round++) {
    if (maxChain > 0) {
      // k_find_sorted writes every target (shortcut-interval targets "unresolved", for pass 2); its
      // marker bits are OR-ed in
      if ((e = hipMemsetAsync(c->longBits.p, 0, c->hBlocks.back().end / 8 + 8, s)))
        return c->fail(SZ4_E_DEVICE, "clear matches", e);
      // k_find_sorted sorts its own segment first unless SZ4_SEPARATE_SORT=1
      if (c->separateSort)
        launch_sort(in, dS, ns, dB, dIv, dIvN, c->elemA.as<uint2>(), c->elemB.as<uint2>(), c->rank.as<uint32_t>(), s);
    }
    mark(c, 2, s);
    if (maxChain > 0)
      launch_find(1, in, dS, ns, dB, dIv, dIvN, c->elemB.as<uint2>(), c->elemA.as<uint2>(), c->rank.as<uint32_t>(), maxChain,
                  c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->longBits.as<uint32_t>(), c->segLong.as<uint32_t>(),
                  nullptr, nullptr, nullptr, nullptr, c->ldsWindow, c->hybridLds, !c->separateSort, s);
    mark(c, 3, s);
    if (c->stopAfter == 2) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
    if (maxChain > 0)
      launch_find(2, in, dS, ns, dB, dIv, dIvN, c->elemB.as<uint2>(), c->elemA.as<uint2>(), c->rank.as<uint32_t>(), maxChain,
                  c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->longBits.as<uint32_t>(), c->segLong.as<uint32_t>(),
                  c->longFlag.as<uint32_t>(), c->cost.as<uint32_t>(), c->reach.as<uint32_t>(), c->segTail.as<uint64_t>(),
                  c->ldsWindow, c->hybridLds, false, s);
    mark(c, 4, s);
    if (c->stopAfter == 3) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
    launch_prep(in, dB, nb, dIv, dIvN, maxChain, c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->sel.as<uint32_t>(),
                c->longFlag.as<uint32_t>(), c->status.as<int>(), s);
    if (maxChain == 0 || maxChain > (uint32_t)kLazyMax) break;
    int st = 0;
    if ((e = hipMemcpyAsync(&st, c->status.p, 4, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
      return c->fail(SZ4_E_DEVICE, "prep", e);
    if (!(st & 2)) break;
    if (round > 2 * kMaxIv + 2) return c->fail(SZ4_E_DEVICE, "shortcut intervals did not settle");
    if ((e = hipMemsetAsync(c->status.p, 0, 4, s)) || (e = hipMemsetAsync(c->longFlag.p, 0, nb * 4, s)))
      return c->fail(SZ4_E_DEVICE, "prep", e);
  }
  if (maxChain > 0 && maxChain <= (uint32_t)kLazyMax && c->dictBack < 0) {
    // greedy/lazy: the reference's skip bookkeeping, in parallel for blocks without shortcut intervals
    // (the others were replayed by k_prep); the token walk's state array is free until k_walk
    if ((e = c->lazySlots.reserve(c->hWalk.size() * lazy_slots_per_walk() * 4ull + 64)))
      return c->fail(SZ4_E_NOMEM, "lazy replay slots", e);
    launch_lazy(dB, nb, c->walkSegs.as<uint2>(), (uint32_t)c->hWalk.size(), dIvN, c->longFlag.as<uint32_t>(),
                c->mlen.as<uint32_t>(), 0, c->lazySlots.as<uint32_t>(), c->walkState.as<uint4>(), c->status.as<int>(), s);
  }
  launch_parse(in, dB, nb, c->dpSegs.as<DpSeg>(), (uint32_t)c->hDp.size(), dIvN, maxChain, c->mlen.as<uint32_t>(),
               c->mdist.as<uint16_t>(), 0, c->cost.as<uint32_t>(), c->sel.as<uint32_t>(), c->reach.as<uint32_t>(),
               c->segState.as<uint4>(), c->longFlag.as<uint32_t>(), c->rmqUp.as<uint32_t>(), c->rmqDown.as<uint32_t>(),
               c->dpSide.as<uint2>(), c->dpRec.as<uint4>(),
               c->status.as<int>(), s);
  mark(c, 5, s);
  if (c->stopAfter == 4) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
  // optimal levels tokenize the parse's choices, greedy/lazy levels the (skip-filtered) matches
  const uint32_t* chosen = maxChain > (uint32_t)kGreedyMax ? c->sel.as<uint32_t>() : c->mlen.as<uint32_t>();
  // the parse's reach array is free by now: it holds each block's concatenated match positions
  launch_emit(in, dB, nb, c->walkSegs.as<uint2>(), (uint32_t)c->hWalk.size(), maxChain, chosen, c->mdist.as<uint16_t>(), 0,
              c->walkSlots.as<uint32_t>(), c->walkState.as<uint4>(), c->reach.as<uint32_t>(), c->tokens.as<Token>(),
              c->ntok.as<uint32_t>(), c->blockBytes.as<uint32_t>(), c->offsets.as<uint64_t>(), out, hdrLen,
              c->status.as<int>(), s);
  mark(c, 6, s);
  if ((e = hipGetLastError())) return c->fail(SZ4_E_DEVICE, "kernel launch", e);

  uint64_t total = 0;
  int status = 0;
  if ((e = hipMemcpyAsync(&total, c->offsets.as<uint64_t>() + nb, 8, hipMemcpyDeviceToHost, s)) ||
      (e = hipMemcpyAsync(&status, c->status.p, 4, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
    return c->fail(SZ4_E_DEVICE, "pipeline", e);
  if (status & kStInvariant) return c->fail(SZ4_E_DEVICE, "device invariant failed (walk slots / token capacity)");
  const uint64_t size = hdrLen + total + (endMark ? 4 : 0);
  if (size > outCap) return c->fail(SZ4_E_CAPACITY, "output buffer too small");
  if (hdrLen && (e = hipMemcpyAsync(out, hdr, hdrLen, hipMemcpyHostToDevice, s)))
    return c->fail(SZ4_E_DEVICE, "header", e);
  if (endMark && (e = hipMemsetAsync(out + hdrLen + total, 0, 4, s))) return c->fail(SZ4_E_DEVICE, "end mark", e);
  if ((e = hipStreamSynchronize(s))) return c->fail(SZ4_E_DEVICE, "finish", e);
  if (c->timing)
    for (int i = 0; i < kStages; i++) hipEventElapsedTime(&c->stageMs[i], c->ev[i], c->ev[i + 1]);
  c->lastBlocks = nb;
  *outSize = size;
  return SZ4_OK;
}

// ---- decoder (the reference's smallz4cat) ----------------------------------------------------
// Index and sizes passes: every block's output offset.  A legacy frame ends after its first block
// shorter than 8 MiB (smallz4cat.c:325-327), so a malformed tail after that block does not matter.
// *keep = blocks to decode, *total = decoded bytes.
int unlz4_plan(sz4_ctx* c, const uint8_t* f, uint64_t n, uint64_t* total, uint32_t* keep, hipStream_t s)
{
  hipError_t e;
  uint64_t maxBlocks = std::min<uint64_t>(n / 5 + 2, 1u << 16);  // a block takes >= 5 frame bytes
  uint64_t meta[3] = {0, 0, 0};
  for (;;) {
    if ((e = c->unBlk.reserve(maxBlocks * sizeof(UnBlock) + 64)) || (e = c->unMeta.reserve(64)))
      return c->fail(SZ4_E_NOMEM, "decoder scratch", e);
    launch_unlz4_index(f, n, c->unBlk.as<UnBlock>(), maxBlocks, c->unMeta.as<uint64_t>(), s);
    if ((e = hipMemcpyAsync(meta, c->unMeta.p, sizeof meta, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
      return c->fail(SZ4_E_DEVICE, "frame index", e);
    if (meta[1] != 2) break;
    maxBlocks = n / 5 + 2;
  }
  const uint32_t nb = (uint32_t)meta[0];
  c->hUn.resize(nb);
  if (nb) {
    if ((e = c->unSeq.reserve(unlz4_seq_entries(n, nb) * sizeof(uint4) + 64)))
      return c->fail(SZ4_E_NOMEM, "decoder sequences", e);
    launch_unlz4_sizes(f, n, c->unBlk.as<UnBlock>(), nb, c->unSeq.as<uint4>(), s);
    if ((e = hipMemcpyAsync(c->hUn.data(), c->unBlk.p, nb * sizeof(UnBlock), hipMemcpyDeviceToHost, s)) ||
        (e = hipStreamSynchronize(s)))
      return c->fail(SZ4_E_DEVICE, "block sizes", e);
  }
  uint64_t w = 0;
  uint32_t k = 0;
  bool ended = false;
  while (k < nb) {
    UnBlock& b = c->hUn[k++];
    if (b.size == kNone) return c->fail(SZ4_E_CORRUPT, "malformed LZ4 block");
    b.dst = w;
    w += b.size;
    if (meta[2] && b.size < kBlockMaxLegacy) {
      ended = true;
      break;
    }
  }
  if (meta[1] != 0 && !ended) return c->fail(SZ4_E_CORRUPT, "invalid or truncated LZ4 frame");
  *total = w;
  *keep = k;
  return SZ4_OK;
}

int unlz4_decode(sz4_ctx* c, const uint8_t* f, uint64_t n, const uint8_t* dict, uint64_t dl, uint8_t* out, uint32_t keep,
                 hipStream_t s)
{
  if (!keep) return SZ4_OK;
  hipError_t e;
  const uint64_t flagBytes = ((uint64_t)keep + 2) * 4;
  if ((e = c->unFlags.reserve(flagBytes + 64))) return c->fail(SZ4_E_NOMEM, "decoder flags", e);
  uint32_t* flags = c->unFlags.as<uint32_t>();
  uint32_t status = 0;
  if ((e = hipMemcpyAsync(c->unBlk.p, c->hUn.data(), keep * sizeof(UnBlock), hipMemcpyHostToDevice, s)) ||
      (e = hipMemsetAsync(flags, 0, flagBytes, s)))
    return c->fail(SZ4_E_DEVICE, "decoder plan", e);
  launch_unlz4_blocks(f, n, c->unBlk.as<UnBlock>(), keep, c->unSeq.as<uint4>(), out, dict, dl, flags, s);
  if ((e = hipGetLastError()) || (e = hipMemcpyAsync(&status, flags + keep, 4, hipMemcpyDeviceToHost, s)) ||
      (e = hipStreamSynchronize(s)))
    return c->fail(SZ4_E_DEVICE, "decode", e);
  if (status & 2u) return c->fail(SZ4_E_DEVICE, "decoder wait timed out");
  if (status) return c->fail(SZ4_E_DEVICE, "decoded length differs from the size pass");
  return SZ4_OK;
}


// ---- stream path: smallz4::lz4 over GET_BYTES / SEND_BYTES in bounded memory --------------------
// The input is compressed in chunks of whole blocks (4 MiB, legacy 8 MiB; c->streamChunk bytes per
// chunk).  A chunk is staged as [carried bytes | new bytes]: the carried bytes are the previous
// chunk's last 64..128 KiB (the reference keeps the last MaxDistance bytes, smallz4.h:798-805), so
// the chunk's first block sees exactly the window the reference's does.  The state a block takes
// from its predecessor -- the lookback cut (smallz4.h:614-624) and the positions the same-letter
// shortcut left out of the chains -- comes along as the previous block's final intervals in the
// ghost slot; dictionary mode carries the reference's hash table and chains.  The device footprint
// is fixed by the chunk size, whatever the input length.  While the GPU compresses chunk i on a
// worker thread, the caller's thread hands chunk i-1's blocks to sendBytes and pulls chunk i+1
// through getBytes (both callbacks always run on the caller's thread).
constexpr uint64_t kCarryMax = 2 * 65536;

struct MemSource {
  const uint8_t* p;
  uint64_t n, at;
};
struct MemSink {
  uint8_t* p;
  uint64_t cap, n;
};
size_t mem_get(void* data, size_t want, void* user)
{
  MemSource* m = static_cast<MemSource*>(user);
  const uint64_t k = std::min<uint64_t>(want, m->n - m->at);
  if (k) memcpy(data, m->p + m->at, k);
  m->at += k;
  return (size_t)k;
}
void mem_send(const void* data, size_t n, void* user)
{
  MemSink* m = static_cast<MemSink*>(user);
  if (n && m->n + n <= m->cap) memcpy(m->p + m->n, data, n);
  m->n += n;
}

struct ChunkJob {
  const uint8_t* host;  // pinned: the chunk's new bytes
  uint64_t pre, n;      // carried bytes already staged, new bytes
  bool first;           // the stream's first chunk
  bool more;            // another chunk follows: prepare the carry
  uint8_t* out;         // pinned: the chunk's blocks
  uint64_t outSize;
  uint64_t nextPre;
  int rc;
};

// compresses one chunk (worker thread); on success the carry for the next chunk is in place
int compress_chunk(sz4_ctx* c, uint32_t maxChain, int legacy, bool dictMode, ChunkJob& j)
{
  DeviceGuard guard(c->device);
  hipStream_t s = c->stream;
  const uint64_t bs = legacy ? kBlockMaxLegacy : kBlockMax;
  c->hBlocks.clear();
  for (uint64_t st = 0; st < j.n; st += bs) {
    Block B{};
    B.start = j.pre + st;
    B.end = j.pre + std::min(st + bs, j.n);
    if (legacy || (st == 0 && j.first)) {
      B.low = B.start;
      B.cut = kNone;
      B.prev = kNoBlock;
    } else {
      B.low = B.start - kWindow;
      B.cut = B.start - kTailNoMatch;  // re-inserted by the lookback of the next block
      B.prev = st == 0 ? kNoBlock - 1 : (uint32_t)c->hBlocks.size() - 1;  // first: the ghost slot, below
    }
    B.flags = legacy ? kBlkLegacy : 0;
    c->hBlocks.push_back(B);
  }
  const uint32_t nb = (uint32_t)c->hBlocks.size();
  if (c->hBlocks[0].prev == kNoBlock - 1) c->hBlocks[0].prev = nb;
  c->ghost = !legacy && !j.first && !dictMode;
  finish_plan(c);
  c->planN = ~0ull;  // invalidate the independent-block plan cache
  if (int r = reserve_all(c, j.pre + j.n + kPad)) return r;
  hipError_t e;
  const uint64_t cap = sz4_lz4_bound(j.n, legacy);
  if ((e = c->chunkOut.reserve(cap))) return c->fail(SZ4_E_NOMEM, "chunk output", e);
  uint8_t* staged = c->staged.as<uint8_t>();
  if ((e = hipMemcpyAsync(staged + j.pre, j.host, j.n, hipMemcpyHostToDevice, s)) ||
      (e = hipMemsetAsync(staged + j.pre + j.n, 0, kPad, s)))
    return c->fail(SZ4_E_DEVICE, "upload", e);
  uint64_t size = 0;
  if (int r = run_pipeline(c, maxChain, nullptr, 0, false, c->chunkOut.as<uint8_t>(), cap, &size, s)) return r;
  if ((e = hipMemcpyAsync(j.out, c->chunkOut.p, size, hipMemcpyDeviceToHost, s))) return c->fail(SZ4_E_DEVICE, "download", e);
  j.outSize = size;
  if (j.more) {
    // carry: the last (pre + n - shift) bytes, shift a multiple of 65536 so that dictionary mode's
    // absolute chain slots (pos & 65535) stay put; at least 65536 bytes precede the next chunk
    const uint64_t end = j.pre + j.n;
    const uint64_t shift = (end - 65536) / 65536 * 65536;
    j.nextPre = end - shift;
    if (!legacy && !dictMode) {
      // the last block's final shortcut intervals become the next chunk's ghost slot
      uint32_t cnt = 0;
      if ((e = hipMemcpyAsync(&cnt, c->ivCount.as<uint32_t>() + (nb - 1), 4, hipMemcpyDeviceToHost, s)) ||
          (e = hipStreamSynchronize(s)))
        return c->fail(SZ4_E_DEVICE, "intervals", e);
      std::vector<Interval> iv(cnt);
      if (cnt && ((e = hipMemcpyAsync(iv.data(), c->iv.as<Interval>() + (uint64_t)(nb - 1) * kMaxIv, cnt * sizeof(Interval),
                                      hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s))))
        return c->fail(SZ4_E_DEVICE, "intervals", e);
      c->ghostIv.clear();
      for (Interval x : iv) {
        if (x.hi <= shift) continue;
        x.lo = std::max(x.lo, shift) - shift;
        x.hi -= shift;
        x.a = x.a >= shift ? x.a - shift : 0;
        c->ghostIv.push_back(x);
      }
    }
    if (dictMode) {
      c->dictCont = legacy ? 0u : 1u;
      c->dictShift = (uint32_t)shift;
      c->dictLow0 = (uint32_t)(j.nextPre - kWindow);
    }
    // the source [shift, end) and the destination [0, end - shift) do not overlap: end - shift <= 2 * 65536 <= shift
    if ((e = hipMemcpyAsync(staged, staged + shift, j.nextPre, hipMemcpyDeviceToDevice, s))) return c->fail(SZ4_E_DEVICE, "carry", e);
  }
  if ((e = hipStreamSynchronize(s))) return c->fail(SZ4_E_DEVICE, "chunk", e);
  return SZ4_OK;
}

// the reference's output call pattern for a run of blocks: four 1-byte calls for the size word, then
// the payload, also when it is empty (smallz4.h:770-780)
void send_blocks(const uint8_t* f, uint64_t n, sz4_send_bytes send, void* user)
{
  uint64_t pos = 0;
  while (pos + 4 <= n) {
    uint32_t word = 0;
    memcpy(&word, f + pos, 4);
    for (int k = 0; k < 4; k++) send(f + pos + k, 1, user);
    pos += 4;
    const uint32_t bytes = word & 0x7FFFFFFFu;
    send(f + pos, bytes, user);
    pos += bytes;
  }
}

// reads up to `want` bytes through getBytes, 64 KiB per call (the reference's BufferSize); *eof is
// set once getBytes has returned 0
uint64_t pull(sz4_get_bytes get, void* user, uint8_t* dst, uint64_t want, bool* eof)
{
  uint64_t got = 0;
  while (got < want && !*eof) {
    const size_t k = get(dst + got, (size_t)std::min<uint64_t>(65536, want - got), user);
    if (k == 0) *eof = true;
    got += k;
  }
  return got;
}

int stream_compress(sz4_ctx* c, sz4_get_bytes get, sz4_send_bytes send, uint32_t maxChain, const uint8_t* dict,
                    uint64_t dictLen, int legacy, void* user, void* sinkUser = nullptr)
{
  void* out = sinkUser ? sinkUser : user;
  hipError_t e;
  if (!c->stream && (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)))
    return c->fail(SZ4_E_DEVICE, "stream", e);
  const uint64_t bs = legacy ? kBlockMaxLegacy : kBlockMax;
  const uint64_t chunk = std::max<uint64_t>(bs, c->streamChunk / bs * bs);
  const bool dictMode = dictLen != 0;
  // header (smallz4.h:478-496)
  const uint8_t hm[7] = {0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF};
  const uint8_t hl[4] = {0x02, 0x21, 0x4C, 0x18};
  send(legacy ? hl : hm, legacy ? 4 : 7, out);
  if ((e = c->hostIn[0].reserve(chunk)) || (e = c->hostIn[1].reserve(chunk)) ||
      (e = c->hostOut[0].reserve(sz4_lz4_bound(chunk, legacy))) || (e = c->hostOut[1].reserve(sz4_lz4_bound(chunk, legacy))))
    return c->fail(SZ4_E_NOMEM, "pinned host buffers", e);
  // fixed device footprint: the staged buffer is sized once for the largest chunk (the carry lives in it)
  if ((e = c->staged.reserve(kCarryMax + chunk + kPad))) return c->fail(SZ4_E_NOMEM, "staging", e);
  bool eof = false;
  uint64_t n = pull(get, user, c->hostIn[0].as<uint8_t>(), chunk, &eof);
  // dictionary: the staged stream starts with the reference's data buffer, a 65535-byte prefix (the
  // dictionary's last bytes, zero-padded in front) (smallz4.h:554-571)
  uint64_t pre = 0;
  c->dictBack = dictMode ? (int64_t)std::min<uint64_t>(dictLen, kWindow) : -1;
  c->dictLegacy = legacy;
  c->dictCont = 0;
  c->ghost = false;
  if (dictMode && n) {
    pre = kWindow;
    std::vector<uint8_t> prefix(pre, 0);
    const uint64_t k = std::min<uint64_t>(dictLen, pre);
    memcpy(prefix.data() + pre - k, dict + dictLen - k, k);
    if ((e = hipMemcpy(c->staged.p, prefix.data(), pre, hipMemcpyHostToDevice))) return c->fail(SZ4_E_DEVICE, "upload", e);
  }
  ChunkJob prevJob{};
  bool havePrev = false;
  for (uint32_t i = 0; n; i++) {
    ChunkJob j{};
    j.host = c->hostIn[i & 1].as<uint8_t>();
    j.pre = pre;
    j.n = n;
    j.first = i == 0;
    j.more = n == chunk && !eof;
    j.out = c->hostOut[i & 1].as<uint8_t>();
    j.rc = SZ4_OK;
    std::thread worker([&]() { j.rc = compress_chunk(c, maxChain, legacy, dictMode, j); });
    // meanwhile, on the caller's thread: the previous chunk's blocks out, the next chunk's bytes in
    if (havePrev) send_blocks(prevJob.out, prevJob.outSize, send, out);
    const uint64_t next = j.more ? pull(get, user, c->hostIn[(i + 1) & 1].as<uint8_t>(), chunk, &eof) : 0;
    worker.join();
    if (j.rc != SZ4_OK) return j.rc;
    prevJob = j;
    havePrev = true;
    pre = j.nextPre;
    n = next;
  }
  if (havePrev) send_blocks(prevJob.out, prevJob.outSize, send, out);
  if (!legacy) {
    static const uint8_t zero[4] = {0, 0, 0, 0};
    send(zero, 4, out);  // end mark (smallz4.h:807-812)
  }
  return SZ4_OK;
}

// ---- decoder stream path: unlz4_userPtr over GET_BYTE / SEND_BYTES in bounded memory -----------
// getByte is called exactly where the reference calls it on a valid frame (header, size words,
// payloads, checksums; a legacy frame ends after its first block that decodes to less than 8 MiB,
// smallz4cat.c:325-327).  Blocks are pulled until about c->streamChunk / 2 frame bytes are queued,
// rewrapped as a plain frame (smallz4's header, the blocks, an end mark; checksums dropped) and
// decoded on the GPU with the last 64 KiB of output (at first the dictionary's) as its history.
// sendBytes receives the output in 64 KiB pieces and the remainder at the end -- the reference's
// flush points (smallz4cat.c:249-253, 358-359).
uint64_t legacy_block_length(const uint8_t* p, uint64_t len)
{
  uint64_t r = 0, w = 0;
  while (r < len) {
    const uint8_t tok = p[r++];
    uint64_t lits = tok >> 4, ml = 4 + (tok & 15);
    uint8_t x;
    if (lits == 15) do { if (r >= len) return w; x = p[r++]; lits += x; } while (x == 255);
    r += lits;
    w += lits;
    if (r >= len) break;
    r += 2;
    if (ml == 19) do { if (r >= len) return w; x = p[r++]; ml += x; } while (x == 255);
    w += ml;
  }
  return w;
}

int stream_decompress(sz4_ctx* c, sz4_get_byte get, sz4_send_out send, const uint8_t* dict, uint64_t dictLen, void* user)
{
  uint32_t sig = 0;
  for (int k = 0; k < 4; k++) sig |= (uint32_t)get(user) << (8 * k);
  const bool modern = sig == 0x184D2204u, legacy = sig == 0x184C2102u;
  if (!modern && !legacy) return c->fail(SZ4_E_CORRUPT, "invalid signature");
  bool blockSum = false, contentSum = false;
  if (modern) {
    const uint8_t flags = get(user);
    if ((flags >> 6) != 1) return c->fail(SZ4_E_CORRUPT, "only LZ4 file format version 1 supported");
    blockSum = (flags & 16) != 0;
    contentSum = (flags & 4) != 0;
    int skip = 1 + ((flags & 8) ? 8 : 0) + ((flags & 1) ? 4 : 0) + 1;
    while (skip--) get(user);
  }
  std::vector<uint8_t> hist;  // the last <= 64 KiB before the next chunk's output
  if (dictLen) hist.assign(dict + (dictLen - std::min<uint64_t>(dictLen, 65536)), dict + dictLen);
  std::vector<uint8_t> frame, out, pend;  // pend: output not yet flushed (< 64 KiB)
  const uint8_t hdr[7] = {0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF};
  const uint64_t budget = std::max<uint64_t>(c->streamChunk / 2, 1u << 20);
  auto decode = [&]() -> int {
    if (frame.size() <= 7) return SZ4_OK;
    for (int k = 0; k < 4; k++) frame.push_back(0);  // end mark
    uint64_t size = 0;
    int r = sz4_unlz4(c, frame.data(), frame.size(), hist.empty() ? nullptr : hist.data(), hist.size(), nullptr, 0, &size);
    if (r == SZ4_E_CAPACITY) {
      out.resize(size);
      r = sz4_unlz4(c, frame.data(), frame.size(), hist.empty() ? nullptr : hist.data(), hist.size(), out.data(), size, &size);
    } else {
      out.clear();
    }
    if (r != SZ4_OK) return r;
    out.resize(size);
    // new history: the last 64 KiB of (history, output)
    if (size >= 65536) {
      hist.assign(out.end() - 65536, out.end());
    } else {
      hist.insert(hist.end(), out.begin(), out.end());
      if (hist.size() > 65536) hist.erase(hist.begin(), hist.end() - 65536);
    }
    // flush in 64 KiB pieces
    uint64_t at = 0;
    if (!pend.empty()) {
      const uint64_t k = std::min<uint64_t>(65536 - pend.size(), size);
      pend.insert(pend.end(), out.begin(), out.begin() + k);
      at = k;
      if (pend.size() == 65536) {
        send(pend.data(), 65536, user);
        pend.clear();
      }
    }
    for (; at + 65536 <= size; at += 65536) send(out.data() + at, 65536, user);
    pend.insert(pend.end(), out.begin() + at, out.begin() + size);
    frame.assign(hdr, hdr + 7);
    return SZ4_OK;
  };
  frame.assign(hdr, hdr + 7);
  for (;;) {
    uint32_t word = 0;
    for (int k = 0; k < 4; k++) word |= (uint32_t)get(user) << (8 * k);
    const bool packed = legacy || (word & 0x80000000u) == 0;
    if (modern) word &= 0x7FFFFFFFu;
    if (word == 0) break;
    if (legacy && (word & 0x80000000u)) return c->fail(SZ4_E_CORRUPT, "invalid or truncated LZ4 frame");
    const uint64_t at = frame.size();
    frame.resize(at + 4 + word);
    const uint32_t tagged = word | (packed ? 0u : 0x80000000u);
    memcpy(frame.data() + at, &tagged, 4);
    for (uint32_t k = 0; k < word; k++) frame[at + 4 + k] = get(user);
    if (legacy && packed && legacy_block_length(frame.data() + at + 4, word) < kBlockMaxLegacy) break;
    if (blockSum)
      for (int k = 0; k < 4; k++) get(user);
    if (frame.size() >= budget)
      if (int r = decode()) return r;
  }
  if (contentSum)
    for (int k = 0; k < 4; k++) get(user);
  if (int r = decode()) return r;
  send(pend.data(), (unsigned int)pend.size(), user);
  return SZ4_OK;
}
}  // namespace

extern "C" {

const char* sz4_version(void) { return "1.5"; }

int sz4_create(sz4_ctx** ctx, int device, uint64_t reserve_bytes)
{
  if (!ctx) return SZ4_E_ARG;
  *ctx = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return SZ4_E_DEVICE;
  DeviceGuard guard(device);
  sz4_ctx* c = new sz4_ctx();
  c->device = device;
  const char* sep = getenv("SZ4_SEPARATE_SORT");
  c->separateSort = sep && sep[0] == '1';
  for (auto& e : c->ev) hipEventCreate(&e);
  if (reserve_bytes && c->staged.reserve(reserve_bytes + kPad) != hipSuccess) {
    sz4_destroy(c);
    return SZ4_E_NOMEM;
  }
  *ctx = c;
  return SZ4_OK;
}

void sz4_destroy(sz4_ctx* c)
{
  if (!c) return;
  DeviceGuard guard(c->device);
  for (DevBuf* b : c->all_buffers()) b->release();
  for (HostBuf* b : {&c->hostIn[0], &c->hostIn[1], &c->hostOut[0], &c->hostOut[1]}) b->release();
  if (c->stream) hipStreamDestroy(c->stream);
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  delete c;
}

int sz4_acquire(sz4_ctx** ctx, int device)
{
  if (!ctx) return SZ4_E_ARG;
  static std::mutex mu;
  static std::vector<sz4_ctx*>* idle = new std::vector<sz4_ctx*>();  // never destroyed: contexts outlive exit order
  {
    std::lock_guard<std::mutex> lock(mu);
    for (size_t i = 0; i < idle->size(); i++)
      if ((*idle)[i]->device == device) {
        *ctx = (*idle)[i];
        idle->erase(idle->begin() + (long)i);
        (*ctx)->pooled = true;
        return SZ4_OK;
      }
  }
  const int r = sz4_create(ctx, device, 0);
  if (r == SZ4_OK) {
    (*ctx)->pooled = true;
    (*ctx)->poolMu = &mu;
    (*ctx)->poolIdle = idle;
  }
  return r;
}

void sz4_release(sz4_ctx* c)
{
  if (!c || !c->pooled || !c->poolMu) return;
  std::lock_guard<std::mutex> lock(*c->poolMu);
  c->poolIdle->push_back(c);
}

uint64_t sz4_bound(uint64_t n, uint32_t block_size)
{
  if (block_size == 0) return 0;
  const uint64_t nb = (n + block_size - 1) / block_size;
  return 16 + n + nb * 4 + 4;  // stored blocks are never larger than their input
}

uint64_t sz4_lz4_bound(uint64_t n, int legacy)
{
  const uint64_t bs = legacy ? kBlockMaxLegacy : kBlockMax;
  const uint64_t nb = n / bs + 2;
  return n + n / 255 + nb * 24 + 64;
}

int sz4_compress_blocks_device(sz4_ctx* c, const void* d_in, uint64_t n, uint32_t block_size, uint32_t max_chain,
                               int header, void* d_out, uint64_t out_cap, uint64_t* out_size, void* stream)
{
  if (!c || !out_size || (!d_in && n) || !d_out || block_size == 0 || block_size > kBlockMax || max_chain > 65535 ||
      header < SZ4_HEADER_SMALLZ4 || header > SZ4_HEADER_NONE)
    return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->err.clear();
  // the kernels write the frame in place: refuse a buffer that could be overrun
  if (out_cap < sz4_bound(n, block_size)) return c->fail(SZ4_E_CAPACITY, "out_cap < sz4_bound(n, block_size)");
  DeviceGuard guard(c->device);
  c->ghost = false;
  hipStream_t s = (hipStream_t)stream;
  c->dictBack = -1;
  if (c->planN != n || c->planBS != block_size) {
    c->hBlocks.clear();
    for (uint64_t st = 0; st < n; st += block_size) {
      Block B{};
      B.start = st;
      B.end = std::min<uint64_t>(st + block_size, n);
      B.low = st;
      B.cut = kNone;
      B.prev = kNoBlock;
      B.flags = 0;
      c->hBlocks.push_back(B);
    }
    finish_plan(c);
    c->planN = n;
    c->planBS = block_size;
  }
  if (int r = reserve_all(c, n + kPad)) return r;
  hipError_t e;
  if ((e = c->staged.reserve(n + kPad))) return c->fail(SZ4_E_NOMEM, "staging", e);
  // private padded copy: kernels read 4-byte windows that may run past the caller's buffer
  if (n && (e = hipMemcpyAsync(c->staged.p, d_in, n, hipMemcpyDeviceToDevice, s)))
    return c->fail(SZ4_E_DEVICE, "stage input", e);
  if ((e = hipMemsetAsync(c->staged.as<uint8_t>() + n, 0, kPad, s))) return c->fail(SZ4_E_DEVICE, "stage pad", e);

  uint8_t hdr[8];
  uint64_t hl = 0;
  bool endMark = true;
  if (header == SZ4_HEADER_SMALLZ4) {
    const uint8_t h[7] = {0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF};
    memcpy(hdr, h, 7);
    hl = 7;
  } else if (header == SZ4_HEADER_INDEPENDENT) {
    uint8_t bd = 4;
    while (bd < 7 && (1ull << (8 + 2 * bd)) < block_size) bd++;
    const uint8_t desc[2] = {0x60, (uint8_t)(bd << 4)};
    const uint8_t h[7] = {0x04, 0x22, 0x4D, 0x18, desc[0], desc[1], (uint8_t)((xxh32_small(desc, 2) >> 8) & 0xFF)};
    memcpy(hdr, h, 7);
    hl = 7;
  } else {
    endMark = false;
  }
  if (n == 0) {
    if (out_cap < hl + (endMark ? 4 : 0)) return c->fail(SZ4_E_CAPACITY, "output buffer too small");
    if (hl) hipMemcpyAsync(d_out, hdr, hl, hipMemcpyHostToDevice, s);
    if (endMark) hipMemsetAsync((uint8_t*)d_out + hl, 0, 4, s);
    hipStreamSynchronize(s);
    c->lastBlocks = 0;
    *out_size = hl + (endMark ? 4 : 0);
    return SZ4_OK;
  }
  return run_pipeline(c, max_chain, hdr, hl, endMark, (uint8_t*)d_out, out_cap, out_size, s);
}

int64_t sz4_last_block_sizes(sz4_ctx* c, uint32_t* sizes, uint64_t max_blocks)
{
  if (!c || !sizes) return SZ4_E_ARG;
  const uint64_t nb = std::min<uint64_t>(c->lastBlocks, max_blocks);
  if (nb && hipMemcpy(sizes, c->blockBytes.p, nb * 4, hipMemcpyDeviceToHost) != hipSuccess) return SZ4_E_DEVICE;
  for (uint64_t i = 0; i < nb; i++) sizes[i] &= 0x7FFFFFFFu;
  return (int64_t)nb;
}

int sz4_lz4_stream(sz4_ctx* c, sz4_get_bytes get_bytes, sz4_send_bytes send_bytes, uint32_t max_chain, const void* dict,
                   uint64_t dict_len, int legacy, void* user)
{
  if (!c || !get_bytes || !send_bytes || max_chain > 65535 || (dict_len && !dict))
    return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->err.clear();
  DeviceGuard guard(c->device);
  return stream_compress(c, get_bytes, send_bytes, max_chain, (const uint8_t*)dict, dict_len, legacy, user);
}

int sz4_lz4(sz4_ctx* c, const void* in, uint64_t n, uint32_t max_chain, const void* dict, uint64_t dict_len, int legacy,
            void* out, uint64_t out_cap, uint64_t* out_size)
{
  if (!c || !out_size || (!in && n) || !out || max_chain > 65535 || (dict_len && !dict))
    return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->err.clear();
  DeviceGuard guard(c->device);
  // the stream path over memory: the source hands out 64 KiB pieces, the sink appends
  MemSource src{(const uint8_t*)in, n, 0};
  MemSink dst{(uint8_t*)out, out_cap, 0};
  const int r = stream_compress(c, mem_get, mem_send, max_chain, (const uint8_t*)dict, dict_len, legacy, &src, &dst);
  if (r != SZ4_OK) return r;
  if (dst.n > out_cap) return c->fail(SZ4_E_CAPACITY, "output buffer too small");
  *out_size = dst.n;
  return SZ4_OK;
}

void sz4_set_stream_chunk(sz4_ctx* c, uint64_t bytes)
{
  if (c) c->streamChunk = bytes ? bytes : (64ull << 20);
}

int sz4_last_stage_ms(sz4_ctx* c, float* stage_ms, int n)
{
  if (!c || !stage_ms) return SZ4_E_ARG;
  const int k = std::min(n, kStages);
  for (int i = 0; i < k; i++) stage_ms[i] = c->stageMs[i];
  return kStages;
}

void sz4_set_timing(sz4_ctx* c, int on)
{
  if (c) c->timing = on != 0;
}

void sz4_debug_stop_after(sz4_ctx* c, int stop_after)
{
  if (c) c->stopAfter = stop_after;
}

int sz4_debug_matches(sz4_ctx* c, uint32_t* len, uint16_t* dist, uint64_t n)
{
  if (!c || !len || !dist) return SZ4_E_ARG;
  if (n * 4 > c->mlen.cap || n * 2 > c->mdist.cap) return SZ4_E_ARG;
  // after the parse at optimal levels the lengths are the parse's choices
  const DevBuf& lens = c->stopAfter == 4 && c->lastChain > (uint32_t)kGreedyMax ? c->sel : c->mlen;
  if (hipMemcpy(len, lens.p, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(dist, c->mdist.p, n * 2, hipMemcpyDeviceToHost) != hipSuccess)
    return SZ4_E_DEVICE;
  return SZ4_OK;
}

int sz4_unlz4_device(sz4_ctx* c, const void* d_frame, uint64_t frame_len, const void* d_dict, uint64_t dict_len,
                     void* d_out, uint64_t out_cap, uint64_t* out_size, void* stream)
{
  if (!c || !out_size || (!d_frame && frame_len) || (dict_len && !d_dict))
    return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->err.clear();
  DeviceGuard guard(c->device);
  hipStream_t s = (hipStream_t)stream;
  uint64_t total = 0;
  uint32_t keep = 0;
  if (int r = unlz4_plan(c, (const uint8_t*)d_frame, frame_len, &total, &keep, s)) return r;
  *out_size = total;
  if (total > out_cap || (total && !d_out)) return c->fail(SZ4_E_CAPACITY, "output buffer too small");
  // the dictionary's last 64 KiB precede the output (smallz4cat.c:168-187)
  const uint64_t dl = std::min<uint64_t>(dict_len, 65536);
  const uint8_t* dict = dl ? (const uint8_t*)d_dict + (dict_len - dl) : nullptr;
  return unlz4_decode(c, (const uint8_t*)d_frame, frame_len, dict, dl, (uint8_t*)d_out, keep, s);
}

int sz4_unlz4(sz4_ctx* c, const void* frame, uint64_t frame_len, const void* dict, uint64_t dict_len, void* out,
              uint64_t out_cap, uint64_t* out_size)
{
  if (!c || !out_size || (!frame && frame_len) || (dict_len && !dict))
    return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->err.clear();
  DeviceGuard guard(c->device);
  hipError_t e;
  const uint64_t dl = std::min<uint64_t>(dict_len, 65536);
  if ((e = c->unFrame.reserve(frame_len + 64)) || (e = c->unDict.reserve(dl + 64)))
    return c->fail(SZ4_E_NOMEM, "staging", e);
  if ((frame_len && (e = hipMemcpy(c->unFrame.p, frame, frame_len, hipMemcpyHostToDevice))) ||
      (dl && (e = hipMemcpy(c->unDict.p, (const uint8_t*)dict + (dict_len - dl), dl, hipMemcpyHostToDevice))))
    return c->fail(SZ4_E_DEVICE, "upload", e);
  uint64_t total = 0;
  uint32_t keep = 0;
  if (int r = unlz4_plan(c, c->unFrame.as<uint8_t>(), frame_len, &total, &keep, nullptr)) return r;
  *out_size = total;
  if (total > out_cap || (total && !out)) return c->fail(SZ4_E_CAPACITY, "output buffer too small");
  if (!total) return SZ4_OK;
  if ((e = c->unOut.reserve(total))) return c->fail(SZ4_E_NOMEM, "output", e);
  if (int r = unlz4_decode(c, c->unFrame.as<uint8_t>(), frame_len, dl ? c->unDict.as<uint8_t>() : nullptr, dl,
                           c->unOut.as<uint8_t>(), keep, nullptr))
    return r;
  if ((e = hipMemcpy(out, c->unOut.p, total, hipMemcpyDeviceToHost))) return c->fail(SZ4_E_DEVICE, "download", e);
  return SZ4_OK;
}

int sz4_unlz4_stream(sz4_ctx* c, sz4_get_byte get_byte, sz4_send_out send_bytes, const void* dict, uint64_t dict_len,
                     void* user)
{
  if (!c || !get_byte || !send_bytes || (dict_len && !dict)) return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->err.clear();
  DeviceGuard guard(c->device);
  return stream_decompress(c, get_byte, send_bytes, (const uint8_t*)dict, dict_len, user);
}

uint64_t sz4_device_bytes(sz4_ctx* c)
{
  if (!c) return 0;
  uint64_t t = 0;
  for (const DevBuf* b : c->all_buffers()) t += b->cap;
  return t;
}

const char* sz4_last_error(sz4_ctx* c) { return c ? c->err.c_str() : "no context"; }

}  // extern "C"
