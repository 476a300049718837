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
#include <cstdio>
#include <cstring>
#include <string>
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
  DevBuf dpSegs, sel, reach, segState, walkSegs, walkSlots, walkState, longFlag, rmqUp, rmqDown, longBits, segLong;
  DevBuf dictLast, dictPrevH;  // dictionary mode: the reference's hash table and hash chain
  DevBuf unBlk, unMeta, unFlags, unFrame, unDict, unOut;  // decoder (sz4_unlz4*)
  std::vector<UnBlock> hUn;
  int64_t dictBack = -1;       // >= 0: dictionary mode, first insertion this far before the first block
  int dictLegacy = 0;

  std::vector<Block> hBlocks;
  std::vector<Segment> hSegs;
  std::vector<DpSeg> hDp;
  std::vector<uint2> hWalk;
  uint64_t elemTotal = 0, rankTotal = 0, tokTotal = 0;
  bool ldsWindow = false;
  uint32_t hybridLds = 0;  // k_find_long9's LDS staging when the window is not LDS-resident
  // plan cache for sz4_compress_blocks_device
  uint64_t planN = ~0ull;
  uint32_t planBS = 0;
  std::vector<uint32_t> hostBytes;

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
    const uint64_t seg = dp_segment_size(n);
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
      (e = c->iv.reserve(nb * kMaxIv * sizeof(Interval) + 64)) ||
      (e = c->ivCount.reserve(nb * 4 + 64)) ||
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
      (e = c->walkSegs.reserve(c->hWalk.size() * sizeof(uint2) + 64)) ||
      (e = c->walkSlots.reserve(c->hWalk.size() * 2 * kWalkCap * 4 + 64)) ||
      (e = c->walkState.reserve(c->hWalk.size() * sizeof(uint4) + 64)) ||
      (e = c->longFlag.reserve(nb * 4 + 64)) ||
      (e = c->longBits.reserve(stagedBytes / 8 + 64)) ||
      (e = c->segLong.reserve(c->hSegs.size() * 4 + 64)) ||
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
  if ((e = hipMemcpyAsync(c->blocks.p, c->hBlocks.data(), nb * sizeof(Block), hipMemcpyHostToDevice, s)) ||
      (e = hipMemcpyAsync(c->segs.p, c->hSegs.data(), c->hSegs.size() * sizeof(Segment), hipMemcpyHostToDevice, s)) ||
      (e = hipMemcpyAsync(c->dpSegs.p, c->hDp.data(), c->hDp.size() * sizeof(DpSeg), hipMemcpyHostToDevice, s)) ||
      (e = hipMemcpyAsync(c->walkSegs.p, c->hWalk.data(), c->hWalk.size() * sizeof(uint2), hipMemcpyHostToDevice, s)) ||
      (e = hipMemsetAsync(c->status.p, 0, 4, s)) || (e = hipMemsetAsync(c->longFlag.p, 0, nb * 4, s)))
    return c->fail(SZ4_E_DEVICE, "upload plan", e);
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
    if ((e = c->dictLast.reserve(sizeof(uint32_t) << 20)) || (e = c->dictPrevH.reserve(2 * 65536)))
      return c->fail(SZ4_E_NOMEM, "dictionary tables", e);
    launch_dict(in, dB, nb, maxChain, (uint32_t)c->dictBack, c->dictLegacy, c->dictLast.as<uint32_t>(),
                c->dictPrevH.as<uint16_t>(), c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), c->sel.as<uint32_t>(),
                c->longFlag.as<uint32_t>(), s);
    mark(c, 2, s);
    mark(c, 3, s);
    mark(c, 4, s);
    if (c->stopAfter == 3) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
  }
  // greedy/lazy levels: k_prep verifies the shortcut intervals k_runs assumed; a corrected block needs
  // another sort/find/prep round (each round checks a longer prefix of it)
  for (uint32_t round = 0; c->dictBack < 0; round++) {
    if (maxChain > 0) {
      // every target starts "unresolved" (pass 2 picks up what pass 1 does not write: shortcut intervals)
      if ((e = hipMemsetAsync(c->mlen.p, 0xFF, c->hBlocks.back().end * 4, s)) ||
          (e = hipMemsetAsync(c->longBits.p, 0, c->hBlocks.back().end / 8 + 8, s)))
        return c->fail(SZ4_E_DEVICE, "clear matches", e);
      // k_find_sorted sorts its own segment first unless SZ4_SEPARATE_SORT=1
      if (c->separateSort)
        launch_sort(in, dS, ns, dB, dIv, dIvN, c->elemA.as<uint2>(), c->elemB.as<uint2>(), c->rank.as<uint32_t>(), s);
    }
    mark(c, 2, s);
    if (maxChain > 0)
      launch_find(1, in, dS, ns, dB, dIv, dIvN, c->elemB.as<uint2>(), c->elemA.as<uint2>(), c->rank.as<uint32_t>(), maxChain,
                  c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->longBits.as<uint32_t>(), c->segLong.as<uint32_t>(),
                  nullptr, nullptr, nullptr, c->ldsWindow, c->hybridLds, !c->separateSort, s);
    mark(c, 3, s);
    if (maxChain > 0)
      launch_find(2, in, dS, ns, dB, dIv, dIvN, c->elemB.as<uint2>(), c->elemA.as<uint2>(), c->rank.as<uint32_t>(), maxChain,
                  c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->longBits.as<uint32_t>(), c->segLong.as<uint32_t>(),
                  c->longFlag.as<uint32_t>(), c->cost.as<uint32_t>(), c->reach.as<uint32_t>(), c->ldsWindow, c->hybridLds,
                  false, s);
    mark(c, 4, s);
    if (c->stopAfter == 3) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
    launch_prep(in, dB, nb, dIv, dIvN, maxChain, c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->sel.as<uint32_t>(),
                c->status.as<int>(), s);
    if (maxChain == 0 || maxChain > (uint32_t)kLazyMax) break;
    int st = 0;
    if ((e = hipMemcpyAsync(&st, c->status.p, 4, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
      return c->fail(SZ4_E_DEVICE, "prep", e);
    if (!(st & 2)) break;
    if (round > 2 * kMaxIv + 2) return c->fail(SZ4_E_DEVICE, "shortcut intervals did not settle");
    if ((e = hipMemsetAsync(c->status.p, 0, 4, s)) || (e = hipMemsetAsync(c->longFlag.p, 0, nb * 4, s)))
      return c->fail(SZ4_E_DEVICE, "prep", e);
  }
  launch_parse(in, dB, nb, c->dpSegs.as<DpSeg>(), (uint32_t)c->hDp.size(), dIvN, maxChain, c->mlen.as<uint32_t>(),
               c->mdist.as<uint16_t>(), 0, c->cost.as<uint32_t>(), c->sel.as<uint32_t>(), c->reach.as<uint32_t>(),
               c->segState.as<uint4>(), c->longFlag.as<uint32_t>(), c->rmqUp.as<uint32_t>(), c->rmqDown.as<uint32_t>(),
               c->status.as<int>(), s);
  mark(c, 5, s);
  if (c->stopAfter == 4) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
  // optimal levels tokenize the parse's choices, greedy/lazy levels the (skip-filtered) matches
  const uint32_t* chosen = maxChain > (uint32_t)kGreedyMax ? c->sel.as<uint32_t>() : c->mlen.as<uint32_t>();
  // the parse's reach array is free by now: it holds each block's concatenated match positions
  launch_emit(in, dB, nb, c->walkSegs.as<uint2>(), (uint32_t)c->hWalk.size(), maxChain, chosen, c->mdist.as<uint16_t>(), 0,
              c->walkSlots.as<uint32_t>(), c->walkState.as<uint4>(), c->reach.as<uint32_t>(), c->tokens.as<Token>(),
              c->ntok.as<uint32_t>(), c->blockBytes.as<uint32_t>(), c->offsets.as<uint64_t>(), out, hdrLen, s);
  mark(c, 6, s);
  if ((e = hipGetLastError())) return c->fail(SZ4_E_DEVICE, "kernel launch", e);

  uint64_t total = 0;
  int status = 0;
  if ((e = hipMemcpyAsync(&total, c->offsets.as<uint64_t>() + nb, 8, hipMemcpyDeviceToHost, s)) ||
      (e = hipMemcpyAsync(&status, c->status.p, 4, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
    return c->fail(SZ4_E_DEVICE, "pipeline", e);
  (void)status;
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
    launch_unlz4_sizes(f, n, c->unBlk.as<UnBlock>(), nb, s);
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
  launch_unlz4_blocks(f, n, c->unBlk.as<UnBlock>(), keep, out, dict, dl, flags, s);
  if ((e = hipGetLastError()) || (e = hipMemcpyAsync(&status, flags + keep, 4, hipMemcpyDeviceToHost, s)) ||
      (e = hipStreamSynchronize(s)))
    return c->fail(SZ4_E_DEVICE, "decode", e);
  if (status & 2u) return c->fail(SZ4_E_DEVICE, "decoder wait timed out");
  if (status) return c->fail(SZ4_E_DEVICE, "decoded length differs from the size pass");
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
  if (hipSetDevice(device) != hipSuccess) return SZ4_E_DEVICE;
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
  hipSetDevice(c->device);
  for (DevBuf* b : {&c->staged, &c->blocks, &c->segs, &c->iv, &c->ivCount, &c->elemA, &c->elemB, &c->rank, &c->mlen,
                    &c->mdist, &c->cost, &c->tokens, &c->ntok, &c->blockBytes, &c->offsets, &c->status, &c->dpSegs,
                    &c->sel, &c->reach, &c->segState, &c->walkSegs, &c->walkSlots, &c->walkState, &c->longFlag,
                    &c->rmqUp, &c->rmqDown, &c->longBits, &c->segLong, &c->dictLast, &c->dictPrevH, &c->unBlk,
                    &c->unMeta, &c->unFlags, &c->unFrame, &c->unDict, &c->unOut})
    b->release();
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  delete c;
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
  hipSetDevice(c->device);
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

int sz4_lz4(sz4_ctx* c, const void* in, uint64_t n, uint32_t max_chain, const void* dict, uint64_t dict_len, int legacy,
            void* out, uint64_t out_cap, uint64_t* out_size)
{
  if (!c || !out_size || (!in && n) || !out || max_chain > 65535 || (dict_len && !dict))
    return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->err.clear();
  hipSetDevice(c->device);
  hipStream_t s = nullptr;
  // dictionary: the staged stream is the reference's data buffer, a 65535-byte prefix (the dictionary's
  // last bytes, zero-padded in front) and then the input (smallz4.h:554-571)
  const uint64_t pre = dict_len ? kWindow : 0;
  c->dictBack = dict_len ? (int64_t)std::min<uint64_t>(dict_len, kWindow) : -1;
  c->dictLegacy = legacy;
  // block structure of smallz4::compress (smallz4.h:541-606, 614-624, 782-805)
  const uint64_t bs = legacy ? kBlockMaxLegacy : kBlockMax;
  c->hBlocks.clear();
  for (uint64_t st = 0; st < n; st += bs) {
    Block B{};
    B.start = pre + st;
    B.end = pre + std::min(st + bs, n);
    const bool first = st == 0;
    if (legacy || first) {
      B.low = B.start;
      B.cut = kNone;
      B.prev = kNoBlock;
    } else {
      B.low = B.start - kWindow;
      B.cut = B.start - kTailNoMatch;  // re-inserted by the lookback of the next block
      B.prev = (uint32_t)c->hBlocks.size() - 1;
    }
    B.flags = legacy ? kBlkLegacy : 0;
    c->hBlocks.push_back(B);
  }
  finish_plan(c);
  c->planN = ~0ull;  // invalidate the independent-block plan cache
  if (int r = reserve_all(c, pre + n + kPad)) return r;
  hipError_t e;
  if ((e = c->staged.reserve(pre + n + kPad))) return c->fail(SZ4_E_NOMEM, "staging", e);
  DevBuf dout;
  const uint64_t cap = sz4_lz4_bound(n, legacy);
  if ((e = dout.reserve(cap))) return c->fail(SZ4_E_NOMEM, "output", e);
  if (pre) {
    std::vector<uint8_t> prefix(pre, 0);
    const uint64_t k = std::min<uint64_t>(dict_len, pre);
    memcpy(prefix.data() + pre - k, (const uint8_t*)dict + dict_len - k, k);
    if ((e = hipMemcpy(c->staged.p, prefix.data(), pre, hipMemcpyHostToDevice))) {
      dout.release();
      return c->fail(SZ4_E_DEVICE, "upload", e);
    }
  }
  if (n && (e = hipMemcpy(c->staged.as<uint8_t>() + pre, in, n, hipMemcpyHostToDevice))) {
    dout.release();
    return c->fail(SZ4_E_DEVICE, "upload", e);
  }
  hipMemset(c->staged.as<uint8_t>() + pre + n, 0, kPad);
  const uint8_t hm[7] = {0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF};
  const uint8_t hl[4] = {0x02, 0x21, 0x4C, 0x18};
  uint64_t size = 0;
  int r;
  if (n == 0) {
    size = legacy ? 4 : 11;
    if (size > out_cap) r = c->fail(SZ4_E_CAPACITY, "output buffer too small");
    else {
      memcpy(out, legacy ? hl : hm, legacy ? 4 : 7);
      if (!legacy) memset((uint8_t*)out + 7, 0, 4);
      r = SZ4_OK;
    }
  } else {
    r = run_pipeline(c, max_chain, legacy ? hl : hm, legacy ? 4 : 7, !legacy, dout.as<uint8_t>(), cap, &size, s);
    if (r == SZ4_OK) {
      if (size > out_cap) r = c->fail(SZ4_E_CAPACITY, "output buffer too small");
      else if ((e = hipMemcpy(out, dout.p, size, hipMemcpyDeviceToHost))) r = c->fail(SZ4_E_DEVICE, "download", e);
    }
  }
  dout.release();
  if (r == SZ4_OK) *out_size = size;
  return r;
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
  hipSetDevice(c->device);
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
  hipSetDevice(c->device);
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

const char* sz4_last_error(sz4_ctx* c) { return c ? c->err.c_str() : "no context"; }

}  // extern "C"
