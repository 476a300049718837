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
#include <chrono>
#include <mutex>
#include <cstdio>
#include <atomic>
#include <cstring>
#include <string>
#include <new>
#include <vector>

#include "../../include/smallz4_amd.h"
#include "sz4_internal.h"

using namespace sz4;

namespace {

constexpr uint64_t kPad = 64;                 // bytes of slack after every staged input
constexpr uint64_t kSegTargets = 65536;       // target positions per segment
// batch API pieces: at most 448 MiB of input, split evenly (a rank's 1.25 GiB slice of configs[4]: three
// pieces of 427 MiB), so that the scratch (48.6 B per piece byte at 256 KiB blocks) stays under ~21 GiB.
// Round 5's 1.5 GiB pieces took ~61 GiB for +14 % on configs[4]: the slice in ONE piece runs the per-block
// parse repair wavefronts of its 5120 blocks together, one latency-bound launch instead of one per piece
constexpr uint64_t kBatchChunkDefault = 448ull << 20;
constexpr uint64_t kScratchPerByte = 50;     // device scratch per piece byte, upper bound (36-49 measured)
constexpr uint64_t kPieceFloor = 16ull << 20;  // smallest batch piece the out-of-memory retry goes down to
constexpr uint64_t kBlockMax = kBlockMaxDict;  // MaxBlockSize (smallz4.h:124)
// dictionary rounds before the in-order replay takes the chunk: each round confirms a longer prefix of every
// block; a wrongly assumed interval may take two rounds (dropped in one, its real start inserted in the
// next: ADVICE r05), so a chunk needs at most 2 x (intervals per block) + 1 rounds, and a block holds at
// most one interval per MaxSameLetter + 1 bytes; a chunk that needs more than that (the old
// cap was 4 x kMaxIv = 544 rounds) goes to the replay
uint32_t dict_round_cap(uint64_t maxBlock) { return 2u * (uint32_t)(maxBlock / (kSameLetter + 1)) + 3u; }

uint64_t token_capacity(uint64_t n) { return n / 2 + 4; }

// Device scratch accounting of one context: the bytes it holds, an optional limit, and a call counter.
// A buffer records the call that last reserved it; buffers of earlier calls (another kind of call: the
// stream path's staging, dictionary tables, decoder images) are the ones a growing call may release.
struct DevBuf;
struct Budget {
  uint64_t used = 0;   // bytes held by the context's DevBufs
  uint64_t limit = 0;  // 0: none (sz4_set_device_limit)
  uint64_t gen = 1;    // the current call
  std::vector<DevBuf*> bufs;
  uint64_t shedCount = 0;  // buffers released by shed()
  void (*onShed)(void*) = nullptr;
  void* owner = nullptr;
  uint64_t shed();  // releases every buffer the current call has not reserved; returns the bytes freed
};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  Budget* bud = nullptr;
  uint64_t lastGen = 0;
  hipError_t reserve(size_t bytes)
  {
    if (bud) lastGen = bud->gen;
    if (bytes <= cap) return hipSuccess;
    size_t want = bytes + bytes / 32 + 4096;  // slack: a slightly larger next call does not reallocate
    if (bud && bud->limit) {
      if (bud->used - cap + want > bud->limit) want = bytes;
      if (bud->used - cap + want > bud->limit) bud->shed();
      if (bud->used - cap + want > bud->limit) return hipErrorOutOfMemory;
    }
    release();
    hipError_t e = hipMalloc(&p, want);
    if (e == hipErrorOutOfMemory && bud && bud->shed()) {
      (void)hipGetLastError();
      e = hipMalloc(&p, want);
    }
    if (e == hipSuccess) {
      cap = want;
      if (bud) bud->used += want;
    } else {
      p = nullptr;
      (void)hipGetLastError();  // the failure is returned, not left sticky for the next runtime call
    }
    return e;
  }
  void release()
  {
    if (p) hipFree(p);
    if (bud) bud->used -= cap;
    p = nullptr;
    cap = 0;
  }
  // the context could grow this buffer to `bytes` without releasing any other buffer
  bool fits(size_t bytes) const
  {
    return bytes <= cap || !bud || !bud->limit || bud->used - cap + bytes <= bud->limit;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

uint64_t Budget::shed()
{
  uint64_t freed = 0;
  for (DevBuf* b : bufs)
    if (b->p && b->lastGen != gen) {
      freed += b->cap;
      b->release();
      shedCount++;
    }
  if (freed && onShed) onShed(owner);
  return freed;
}

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

  DevBuf staged, blocks, segs, iv, ivCount, rank, mlen, mdist, cost, ntok, blockBytes, offsets, status;
  DevBuf dpSegs, reach, segState, walkSegs, walkState, longFlag, longBits, segLong, segTail;
  DevBuf dpRec;                // the parallel parse-boundary repair's records
  // One region for the arrays whose lifetimes do not overlap (reserve_all lays it out):
  //   match search   sort elements A | B  (dead once the search has finished)
  //   after it       parse choices (sel) | greedy/lazy replay slots, or the parse's range minima UP | DOWN and
  //                  k_dp_fix's saved speculative values, or the frame tokens | token-walk slots
  // sel stays live from k_prep (its tail) through the parse to the token walk; the rest are per stage.
  DevBuf work;
  uint64_t offElemB = 0, offRmqUp = 0, offRmqDown = 0, offSide = 0, offLazy = 0, offTok = 0, offWalk = 0;
  uint2* elemA() const { return work.as<uint2>(); }
  uint2* elemB() const { return reinterpret_cast<uint2*>(work.as<uint8_t>() + offElemB); }
  uint32_t* sel() const { return work.as<uint32_t>(); }
  uint32_t* rmqUp() const { return reinterpret_cast<uint32_t*>(work.as<uint8_t>() + offRmqUp); }
  uint32_t* rmqDown() const { return reinterpret_cast<uint32_t*>(work.as<uint8_t>() + offRmqDown); }
  uint2* dpSide() const { return reinterpret_cast<uint2*>(work.as<uint8_t>() + offSide); }
  uint32_t* lazySlots() const { return reinterpret_cast<uint32_t*>(work.as<uint8_t>() + offLazy); }
  Token* tokens() const { return reinterpret_cast<Token*>(work.as<uint8_t>() + offTok); }
  uint32_t* walkSlots() const { return reinterpret_cast<uint32_t*>(work.as<uint8_t>() + offWalk); }
  DevBuf dictLast, dictPrevH, dictPrevX;  // dictionary mode: the reference's hash table and both chains
  DevBuf dictPH, dictPE, dictKeys, dictTemp, dictSc, dictSnap, dictRuns, dictLz;  // dictionary mode on the whole GPU (sz4_dict.hip)
  uint32_t dictRounds = 0;  // most rounds a dictionary chunk of the last call took (~0u: one fell back to the in-order replay)
  uint32_t dictMaxRounds = getenv("SZ4_DICT_MAX_ROUNDS") && atoi(getenv("SZ4_DICT_MAX_ROUNDS")) > 0
                               ? (uint32_t)atoi(getenv("SZ4_DICT_MAX_ROUNDS")) : 0u;  // tests: force the replay (0: dict_round_cap)
  bool dictNoGuess = getenv("SZ4_DICT_NO_GUESS") != nullptr;  // A/B: the first round assumes no shortcut interval
  uint64_t dictTempBytes = 0;  // rocPRIM radix sort scratch for dictKeys (queried on first use)
  DevBuf chunkOut[2];          // stream path: two chunks' blocks (chunk i+1 computes while chunk i downloads)
  DevBuf stagedS[2];           // stream path: two chunks' staged input (chunk i+1 uploads while chunk i computes)
  HostBuf hostIn[2], hostOut[2];
  uint64_t streamChunk = 64ull << 20;  // stream path: input bytes per chunk (rounded to whole blocks)
  uint64_t batchChunk = kBatchChunkDefault;  // sz4_compress_blocks_device: input bytes per internal pipeline run
  bool batchChunkSet = false;          // set explicitly (sz4_set_batch_chunk, SZ4_BATCH_CHUNK): no free-memory cap
  bool batchChunked = false;           // the last sz4_compress_blocks_device call ran in several pieces
  uint64_t streamPlanKey[5] = {~0ull, 0, 0, 0, 0};  // stream path: the chunk shape the current plan is for
  // stream path, chunk continuation: the previous chunk's last block's final shortcut intervals
  // (ghost slot nblocks of iv/ivCount, B.prev of the first block) and dictionary-mode state
  std::vector<Interval> ghostIv;
  uint32_t ghostN = 0;
  bool ghost = false;
  uint32_t dictCont = 0, dictShift = 0, dictLow0 = 0;
  DevBuf unBlk, unMeta, unFlags, unFrame, unDict, unOut, unSeq;  // decoder (sz4_unlz4*)
  DevBuf unSubs, unMasks, unImage;  // decoder split mode: sub-segments, their token-start masks, the u32 image
  DevBuf unIx;                       // decoder: the parallel frame index's candidates and successors
  bool unIndexSerial = getenv("SZ4_UNLZ4_INDEX") && atoi(getenv("SZ4_UNLZ4_INDEX")) == 0;  // A/B: the one-lane walk
  std::vector<UnBlock> hUn;
  std::vector<UnSub> hSub;
  bool unSplit = false;  // the last planned frame decodes in split mode
  uint32_t unResolvePasses = 0;  // the longest reference chain the last split-mode decode's pack followed
  bool unIndexParallel = false;  // the last frame index came from the parallel index (not the serial walk)
  int unSplitMode = getenv("SZ4_UNLZ4_SPLIT") ? atoi(getenv("SZ4_UNLZ4_SPLIT")) : -1;  // -1 auto, 0 never, 1 always
  int64_t dictBack = -1;       // >= 0: dictionary mode, first insertion this far before the first block
  int dictLegacy = 0;
  bool dictSerial = getenv("SZ4_DICT_SERIAL") != nullptr;  // A/B and tests: the in-order replay for every chunk

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
  // plan cache for sz4_compress_blocks_device
  uint64_t planN = ~0ull;
  uint32_t planBS = 0;
  std::vector<uint32_t> hostBytes;

  hipStream_t stream = nullptr;  // the stream path's compute stream
  hipStream_t upStream = nullptr, downStream = nullptr;  // its upload and download streams
  hipEvent_t evUp[2] = {}, evDone[2] = {};  // per staging slot: upload complete, chunk computed
  bool pooled = false;           // handed out by sz4_acquire
  std::mutex* poolMu = nullptr;
  std::vector<sz4_ctx*>* poolIdle = nullptr;

  Budget budget;
  // a new call: later reserves record it, and a growing call may release what earlier calls left
  void begin_call()
  {
    err.clear();
    budget.gen++;
  }

  std::vector<DevBuf*> all_buffers()
  {
    return {&staged, &blocks, &segs, &iv, &ivCount, &rank, &mlen, &mdist, &cost, &ntok, &blockBytes, &offsets, &status,
            &dpSegs, &reach, &segState, &walkSegs, &walkState, &longFlag, &longBits, &segLong, &segTail, &dpRec, &work,
            &dictLast, &dictPrevH, &dictPrevX, &dictPH, &dictPE, &dictKeys, &dictTemp, &dictSc, &dictSnap, &dictRuns, &dictLz,
            &chunkOut[0], &chunkOut[1], &stagedS[0], &stagedS[1], &unBlk, &unMeta, &unFlags, &unFrame, &unDict,
            &unOut, &unSeq, &unSubs, &unMasks, &unImage, &unIx};
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
  // the finders' LDS-window kernels take the launch when every block's window fits their LDS
  c->ldsWindow = true;
  for (const Segment& S : c->hSegs) {
    const Block& B = c->hBlocks[S.block];
    if ((B.end - S.w0 + 8 + 3) / 4 * 4 > find_lds_bytes()) c->ldsWindow = false;
  }
}

// the shared region's layout for the current plan (sz4_ctx::work); returns its size in bytes
uint64_t work_layout(sz4_ctx* c, uint64_t stagedBytes)
{
  auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
  const uint64_t nb = c->hBlocks.size();
  const uint64_t elem = al(c->elemTotal * sizeof(uint2) + 64);
  c->offElemB = elem;
  const uint64_t findEnd = 2 * elem;
  const uint64_t selBytes = al(stagedBytes * 4 + 64), rmq = al((stagedBytes + nb + 8) * 4);
  c->offRmqUp = selBytes;
  c->offRmqDown = selBytes + rmq;
  c->offSide = selBytes + 2 * rmq;
  const uint64_t parseEnd = c->offSide + al(c->hDp.size() * dp_side_positions() * sizeof(uint2) + 64);
  c->offLazy = selBytes;
  const uint64_t lazyEnd = c->offLazy + al(c->hWalk.size() * lazy_slots_per_walk() * 4ull + 64);
  c->offTok = selBytes;
  c->offWalk = c->offTok + al(c->tokTotal * sizeof(Token) + 64);
  const uint64_t emitEnd = c->offWalk + al(c->hWalk.size() * 2 * kWalkCap * 4 + 64);
  return std::max(std::max(findEnd, parseEnd), std::max(lazyEnd, emitEnd));
}

int reserve_all(sz4_ctx* c, uint64_t stagedBytes)
{
  const uint64_t nb = c->hBlocks.size();
  hipError_t e = hipSuccess;
  if ((e = c->blocks.reserve(nb * sizeof(Block) + 64)) ||
      (e = c->segs.reserve(c->hSegs.size() * sizeof(Segment) + 64)) ||
      (e = c->iv.reserve((nb + 1) * kMaxIv * sizeof(Interval) + 64)) ||
      (e = c->ivCount.reserve((nb + 1) * 4 + 64)) ||
      (e = c->rank.reserve(c->rankTotal * 4 + 64)) ||
      (e = c->mlen.reserve(stagedBytes * 4 + 64)) ||
      (e = c->mdist.reserve(stagedBytes * 2 + 64)) ||
      (e = c->cost.reserve((stagedBytes + nb + 8) * 4)) ||
      (e = c->ntok.reserve(nb * 4 + 64)) ||
      (e = c->blockBytes.reserve(nb * 4 + 64)) ||
      (e = c->offsets.reserve((nb + 1) * 8 + 64)) ||
      (e = c->status.reserve(64)) ||
      (e = c->dpSegs.reserve(c->hDp.size() * sizeof(DpSeg) + 64)) ||
      (e = c->reach.reserve(stagedBytes * 4 + 64)) ||
      (e = c->segState.reserve(c->hDp.size() * sizeof(uint4) + 64)) ||
      (e = c->dpRec.reserve(c->hDp.size() * sizeof(uint4) + 64)) ||
      (e = c->walkSegs.reserve(c->hWalk.size() * sizeof(uint2) + 64)) ||
      (e = c->walkState.reserve(c->hWalk.size() * sizeof(uint4) + 64)) ||
      (e = c->longFlag.reserve(nb * 4 + 64)) ||
      (e = c->longBits.reserve(stagedBytes / 8 + 64)) ||
      (e = c->segLong.reserve(c->hSegs.size() * 4 + 64)) ||
      (e = c->segTail.reserve(c->hSegs.size() * 8 + 64)) ||
      (e = c->work.reserve(work_layout(c, stagedBytes))))
    return c->fail(SZ4_E_NOMEM, "device allocation", e);
  return SZ4_OK;
}

void mark(sz4_ctx* c, int i, hipStream_t s)
{
  if (c->timing) hipEventRecord(c->ev[i], s);
}

int pipeline_finish(sz4_ctx* c, const uint8_t* hdr, uint64_t hdrLen, bool endMark, uint8_t* out, uint64_t outCap,
                    uint64_t* outSize, hipStream_t s);

// run the kernel pipeline over the planned blocks of the staged input `in`; frame goes to `out`.
// finish = false: return once every kernel is enqueued (pipeline_finish collects the result)
int run_pipeline(sz4_ctx* c, uint32_t maxChain, const uint8_t* in, const uint8_t* hdr, uint64_t hdrLen, bool endMark,
                 uint8_t* out, uint64_t outCap, uint64_t* outSize, hipStream_t s, bool finish = true)
{
  const uint32_t nb = (uint32_t)c->hBlocks.size();
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
  // ghost slot nb: the previous chunk's last block (only its intervals are read, through B.prev).  The
  // sources of these asynchronous copies live in the context: the stream path returns before they run
  c->ghostN = c->ghost ? (uint32_t)c->ghostIv.size() : 0u;
  if ((c->ghostN && (e = hipMemcpyAsync(c->iv.as<Interval>() + (uint64_t)nb * kMaxIv, c->ghostIv.data(),
                                        c->ghostN * sizeof(Interval), hipMemcpyHostToDevice, s))) ||
      (e = hipMemcpyAsync(c->ivCount.as<uint32_t>() + nb, &c->ghostN, 4, hipMemcpyHostToDevice, s)))
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
    // dictionary mode (modern and legacy frames): the data-parallel match finder of sz4_dict.hip, in
    // rounds until its assumed same-letter shortcut intervals are the ones its results imply; then the
    // usual parse
    if ((e = c->dictLast.reserve(sizeof(uint32_t) << 20)) || (e = c->dictPrevH.reserve(2 * 65536)) ||
        (e = c->dictPrevX.reserve(2 * 65536)))
      return c->fail(SZ4_E_NOMEM, "dictionary tables", e);
    auto serial = [&]() {
      launch_dict(in, dB, nb, maxChain, (uint32_t)c->dictBack, c->dictLegacy, c->dictLast.as<uint32_t>(),
                  c->dictPrevH.as<uint16_t>(), c->dictPrevX.as<uint16_t>(), c->dictCont, c->dictShift, c->dictLow0,
                  c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), c->sel(), c->longFlag.as<uint32_t>(), s);
    };
    if (c->dictSerial) {
      serial();  // A/B and tests: the reference's loop replayed in order by one wavefront
    } else {
      const uint64_t staged = c->hBlocks.back().end + 64;
      uint64_t maxBlock = 0;
      for (const Block& B : c->hBlocks) maxBlock = std::max<uint64_t>(maxBlock, B.end - B.start);
      // rocPRIM's scratch size, queried once per context on its own device (0: the query failed)
      if (!c->dictTempBytes && !(c->dictTempBytes = dict_sort_temp_bytes()))
        return c->fail(SZ4_E_DEVICE, "dictionary sort: scratch size query");
      const uint64_t lastBytes = sizeof(uint32_t) << kHashBits, slotBytes = 2 * 65536;
      if ((e = c->dictPH.reserve(staged * 2)) || (e = c->dictPE.reserve(staged * 2)) ||
          (e = c->dictKeys.reserve(2 * dict_sort_keys_max() * 8)) || (e = c->dictTemp.reserve(c->dictTempBytes + 64)) ||
          (e = c->dictSc.reserve(dict_sc_bits_bytes(nb, maxBlock))) ||
          (e = c->dictSnap.reserve(lastBytes + 2 * slotBytes)) || (e = c->dictRuns.reserve(dict_run_table_bytes(staged))) ||
          (e = c->dictLz.reserve(c->hWalk.size() * dict_lz_mask_bytes_per_walk() + 64)))
        return c->fail(SZ4_E_NOMEM, "dictionary scratch", e);
      // the carried tables as this chunk found them: a round that finds other shortcut intervals starts
      // again from here (legacy frames carry nothing: every block starts from empty tables)
      uint8_t* snap = c->dictSnap.as<uint8_t>();
      auto tables = [&](bool save) -> hipError_t {
        hipError_t r;
        uint8_t* t[3] = {c->dictLast.as<uint8_t>(), c->dictPrevH.as<uint8_t>(), c->dictPrevX.as<uint8_t>()};
        const uint64_t off[3] = {0, lastBytes, lastBytes + slotBytes}, len[3] = {lastBytes, slotBytes, slotBytes};
        for (int k = 0; k < 3; k++)
          if ((r = hipMemcpyAsync(save ? snap + off[k] : t[k], save ? t[k] : snap + off[k], len[k],
                                  hipMemcpyDeviceToDevice, s)))
            return r;
        return hipSuccess;
      };
      if ((!c->dictLegacy && (e = tables(true))) || (e = hipMemsetAsync(dIvN, 0, nb * 4, s)))
        return c->fail(SZ4_E_DEVICE, "dictionary tables", e);
      DictArgs A{};
      A.in = in;
      A.dBlocks = dB;
      A.hBlocks = c->hBlocks.data();
      A.nb = nb;
      A.maxChain = maxChain;
      A.dictBack = (uint32_t)c->dictBack;
      A.cont = c->dictCont;
      A.shift = c->dictShift;
      A.low0 = c->dictLow0;
      A.legacy = c->dictLegacy;
      A.iv = dIv;
      A.ivCount = dIvN;
      A.last = c->dictLast.as<uint32_t>();
      A.prevH = c->dictPrevH.as<uint16_t>();
      A.prevX = c->dictPrevX.as<uint16_t>();
      A.ph = c->dictPH.as<uint16_t>();
      A.pe = c->dictPE.as<uint16_t>();
      A.keysA = c->dictKeys.as<uint64_t>();
      A.keysB = c->dictKeys.as<uint64_t>() + dict_sort_keys_max();
      A.temp = c->dictTemp.p;
      A.tempBytes = c->dictTempBytes;
      A.mlen = c->mlen.as<uint32_t>();
      A.mdist = c->mdist.as<uint16_t>();
      A.sel = c->sel();
      A.longFlag = c->longFlag.as<uint32_t>();
      A.walkSegs = c->walkSegs.as<uint2>();
      A.nwalk = (uint32_t)c->hWalk.size();
      A.lzMasks = c->dictLz.as<uint32_t>();
      A.lzState = c->walkState.as<uint4>();
      A.scBits = c->dictSc.as<uint64_t>();
      A.status = c->status.as<int>();
      A.runTab = c->dictRuns.as<uint2>();
      A.runFlag = reinterpret_cast<uint32_t*>(A.runTab + (staged / 64 + 2));
      for (uint32_t round = 0;; round++) {
        A.buildRuns = round == 0;
        A.guess = round == 0 && !c->dictNoGuess;
        if (round > 0 && ((!c->dictLegacy && (e = tables(false))) || (e = hipMemsetAsync(c->longFlag.p, 0, nb * 4, s))))
          return c->fail(SZ4_E_DEVICE, "dictionary tables", e);
        if (launch_dict_parallel(A, s)) return c->fail(SZ4_E_DEVICE, "dictionary kernels");
        int st = 0;
        if ((e = hipMemcpyAsync(&st, c->status.p, 4, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
          return c->fail(SZ4_E_DEVICE, "dictionary rounds", e);
        if (c->dictRounds != ~0u) c->dictRounds = std::max(c->dictRounds, round + 1);  // sticky over the call's chunks
        if (!(st & (kStPrepRound | kStInvariant))) break;
        if ((e = hipMemsetAsync(c->status.p, 0, 4, s))) return c->fail(SZ4_E_DEVICE, "dictionary rounds", e);
        // every round settles a longer prefix, so this is a safety net, not a path: the in-order replay
        if ((st & kStInvariant) || round + 1 >= (c->dictMaxRounds ? c->dictMaxRounds : dict_round_cap(maxBlock))) {
          if ((!c->dictLegacy && (e = tables(false))) || (e = hipMemsetAsync(c->longFlag.p, 0, nb * 4, s)))
            return c->fail(SZ4_E_DEVICE, "dictionary tables", e);
          serial();
          c->dictRounds = ~0u;
          break;
        }
      }
    }
    mark(c, 2, s);
    mark(c, 3, s);
    mark(c, 4, s);
    if (c->stopAfter == 3) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
  }
  // greedy/lazy levels: k_lazy_check verifies the shortcut intervals k_runs assumed; a corrected block
  // needs another sort/find/walk round (each round checks a longer prefix of it)
  for (uint32_t round = 0; c->dictBack < 0; round++) {
    if (maxChain > 0) {
      // k_find_sorted writes every target (shortcut-interval targets "unresolved", for pass 2); its
      // marker bits are OR-ed in
      if ((e = hipMemsetAsync(c->longBits.p, 0, c->hBlocks.back().end / 8 + 8, s)))
        return c->fail(SZ4_E_DEVICE, "clear matches", e);
    }
    mark(c, 2, s);
    if (maxChain > 0)
      launch_find(1, in, dS, ns, dB, dIv, dIvN, c->elemB(), c->elemA(), c->rank.as<uint32_t>(), maxChain,
                  c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->longBits.as<uint32_t>(), c->segLong.as<uint32_t>(),
                  nullptr, nullptr, nullptr, nullptr, c->ldsWindow, s);
    mark(c, 3, s);
    if (c->stopAfter == 2) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
    if (maxChain > 0)
      launch_find(2, in, dS, ns, dB, dIv, dIvN, c->elemB(), c->elemA(), c->rank.as<uint32_t>(), maxChain,
                  c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->longBits.as<uint32_t>(), c->segLong.as<uint32_t>(),
                  c->longFlag.as<uint32_t>(), c->cost.as<uint32_t>(), c->reach.as<uint32_t>(), c->segTail.as<uint64_t>(),
                  c->ldsWindow, s);
    mark(c, 4, s);
    if (c->stopAfter == 3) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
    launch_prep(in, dB, nb, dIv, dIvN, maxChain, c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->sel(),
                c->longFlag.as<uint32_t>(), c->status.as<int>(), s);
    if (maxChain == 0 || maxChain > (uint32_t)kLazyMax) break;
    // greedy/lazy: the reference's skip bookkeeping in parallel over the assumed shortcut intervals, which
    // k_lazy_check / k_lazy_correct then compare with the ones the searches imply (blockBytes is free until
    // the token walk: it holds each block's first difference)
    launch_lazy(in, dB, nb, c->walkSegs.as<uint2>(), (uint32_t)c->hWalk.size(), dIv, dIvN, c->longFlag.as<uint32_t>(),
                c->mlen.as<uint32_t>(), c->mdist.as<uint16_t>(), 0, c->lazySlots(), c->walkState.as<uint4>(),
                c->blockBytes.as<uint32_t>(), c->status.as<int>(), s);
    int st = 0;
    if ((e = hipMemcpyAsync(&st, c->status.p, 4, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
      return c->fail(SZ4_E_DEVICE, "prep", e);
    if (!(st & 2)) break;
    if (round > 2 * kMaxIv + 2) return c->fail(SZ4_E_DEVICE, "shortcut intervals did not settle");
    if ((e = hipMemsetAsync(c->status.p, 0, 4, s)) || (e = hipMemsetAsync(c->longFlag.p, 0, nb * 4, s)))
      return c->fail(SZ4_E_DEVICE, "prep", e);
  }
  uint32_t maxDpCount = 1;
  for (const Block& B : c->hBlocks) maxDpCount = std::max(maxDpCount, B.dpCount);
  launch_parse(in, dB, nb, c->dpSegs.as<DpSeg>(), (uint32_t)c->hDp.size(), maxDpCount, dIvN, maxChain, c->mlen.as<uint32_t>(),
               c->mdist.as<uint16_t>(), 0, c->cost.as<uint32_t>(), c->sel(), c->reach.as<uint32_t>(),
               c->segState.as<uint4>(), c->longFlag.as<uint32_t>(), c->rmqUp(), c->rmqDown(),
               c->dpSide(), c->dpRec.as<uint4>(),
               c->status.as<int>(), s);
  mark(c, 5, s);
  if (c->stopAfter == 4) return hipStreamSynchronize(s) == hipSuccess ? SZ4_OK : c->fail(SZ4_E_DEVICE, "pipeline");
  // optimal levels tokenize the parse's choices, greedy/lazy levels the (skip-filtered) matches
  const uint32_t* chosen = maxChain > (uint32_t)kGreedyMax ? c->sel() : c->mlen.as<uint32_t>();
  // the parse's reach array is free by now: it holds each block's concatenated match positions
  launch_emit(in, dB, nb, c->walkSegs.as<uint2>(), (uint32_t)c->hWalk.size(), maxChain, chosen, c->mdist.as<uint16_t>(), 0,
              c->walkSlots(), c->walkState.as<uint4>(), c->reach.as<uint32_t>(), c->tokens(),
              c->ntok.as<uint32_t>(), c->blockBytes.as<uint32_t>(), c->offsets.as<uint64_t>(), out, hdrLen,
              c->status.as<int>(), s);
  mark(c, 6, s);
  if ((e = hipGetLastError())) return c->fail(SZ4_E_DEVICE, "kernel launch", e);
  c->lastBlocks = nb;
  if (!finish) return SZ4_OK;
  return pipeline_finish(c, hdr, hdrLen, endMark, out, outCap, outSize, s);
}

// the frame size and device status of the pipeline enqueued last on s; header and end mark around it
int pipeline_finish(sz4_ctx* c, const uint8_t* hdr, uint64_t hdrLen, bool endMark, uint8_t* out, uint64_t outCap,
                    uint64_t* outSize, hipStream_t s)
{
  const uint32_t nb = (uint32_t)c->hBlocks.size();
  hipError_t e;
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
  uint64_t meta[5] = {0, 0, 0, 0, 0};
  for (;;) {
    if ((e = c->unBlk.reserve(maxBlocks * sizeof(UnBlock) + 64)) || (e = c->unMeta.reserve(64)))
      return c->fail(SZ4_E_NOMEM, "decoder scratch", e);
    // the parallel index (its scratch is about 3n / 8 bytes); the one-lane walk when that does not fit.  Under a
    // device bound it is tried only if it fits without releasing other buffers (it is optional: ADVICE r05)
    const uint64_t ixBytes = unlz4_ix_scratch_bytes(n);
    if (!c->unIndexSerial && c->unIx.fits(ixBytes) && c->unIx.reserve(ixBytes) == hipSuccess)
      launch_unlz4_index_par(f, n, c->unIx.p, c->unBlk.as<UnBlock>(), maxBlocks, c->unMeta.as<uint64_t>(), s);
    else
      launch_unlz4_index(f, n, c->unBlk.as<UnBlock>(), maxBlocks, c->unMeta.as<uint64_t>(), s);
    if ((e = hipMemcpyAsync(meta, c->unMeta.p, sizeof meta, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
      return c->fail(SZ4_E_DEVICE, "frame index", e);
    // the index scratch is dead once its result is read: kept for the next call, but releasable by a
    // growing reservation of this one (the split buffers, the output)
    c->unIx.lastGen = 0;
    if (meta[1] != 2) break;
    maxBlocks = n / 5 + 2;
  }
  const uint32_t nb = (uint32_t)meta[0];
  c->unIndexParallel = meta[3] == 1;
  c->hUn.resize(nb);
  c->unSplit = false;
  // split mode needs about twice the per-block decoder's scratch (the u32 image, the sub-segment lists):
  // when it does not fit, or its 31-bit image cannot address the output, the frame decodes block by block
  auto blockwise = [&]() {
    for (DevBuf* b : {&c->unSubs, &c->unMasks, &c->unImage}) b->release();
    const int mode = c->unSplitMode;
    c->unSplitMode = 0;
    const int r = unlz4_plan(c, f, n, total, keep, s);
    c->unSplitMode = mode;
    return r;
  };
  if (nb) {
    // split mode when a block is large (one wavefront per block would leave most of the chip idle); the
    // index reports the longest payload, so block-wise decoding reads the records back only after sizes
    const uint64_t maxLen = meta[4];
    c->unSplit = c->unSplitMode == 1 || (c->unSplitMode != 0 && maxLen >= kUnSplitMin);
    if (c->unSplit && ((e = hipMemcpyAsync(c->hUn.data(), c->unBlk.p, nb * sizeof(UnBlock), hipMemcpyDeviceToHost, s)) ||
                       (e = hipStreamSynchronize(s))))
      return c->fail(SZ4_E_DEVICE, "frame index", e);
  }
  if (nb && c->unSplit) {
    c->hSub.clear();
    for (uint32_t b = 0; b < nb; b++) {
      UnBlock& B = c->hUn[b];
      B.subFirst = (uint32_t)c->hSub.size();
      B.subCount = (B.len + kUnSub - 1) / kUnSub;
      for (uint32_t k = 0; k < B.subCount; k++) c->hSub.push_back(UnSub{b, k});
    }
    const uint32_t nsub = (uint32_t)c->hSub.size();
    if ((e = c->unSeq.reserve((uint64_t)nsub * 2 * kUnSubCap * sizeof(uint4) + 64)) ||
        (e = c->unSubs.reserve((uint64_t)nsub * sizeof(UnSub) + 64)) ||
        (e = c->unMasks.reserve((uint64_t)nsub * kUnAuxWords * 4 + 64))) {
      c->unSeq.release();
      return blockwise();
    }
    if ((e = hipMemcpyAsync(c->unBlk.p, c->hUn.data(), nb * sizeof(UnBlock), hipMemcpyHostToDevice, s)) ||
        (e = hipMemcpyAsync(c->unSubs.p, c->hSub.data(), nsub * sizeof(UnSub), hipMemcpyHostToDevice, s)))
      return c->fail(SZ4_E_DEVICE, "decoder plan", e);
    launch_unlz4_split_sizes(f, n, c->unBlk.as<UnBlock>(), nb, c->unSubs.as<UnSub>(), nsub, c->unSeq.as<uint4>(),
                             c->unMasks.as<uint32_t>(), s);
    if ((e = hipMemcpyAsync(c->hUn.data(), c->unBlk.p, nb * sizeof(UnBlock), hipMemcpyDeviceToHost, s)) ||
        (e = hipStreamSynchronize(s)))
      return c->fail(SZ4_E_DEVICE, "block sizes", e);
  } else if (nb) {
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
  // the split image addresses output bytes with 31 bits: a larger output decodes block by block
  if (c->unSplit && w >= (uint64_t)kUnRef) {
    c->unSeq.release();
    return blockwise();
  }
  if (c->unSplit && ((e = c->unImage.reserve(w * 4 + 64)) || (e = c->unFlags.reserve(64)))) {
    c->unSeq.release();
    return blockwise();
  }
  *total = w;
  *keep = k;
  return SZ4_OK;
}

// the device output buffer of the host-buffer decoders (sz4_unlz4, the stream decoder): when it does not fit
// beside a split-mode plan, the frame is planned again block by block (about half the scratch) and the
// reservation retried (the split plan's own check did not count this buffer)
int unlz4_reserve_out(sz4_ctx* c, const uint8_t* f, uint64_t n, uint64_t* total, uint32_t* keep)
{
  hipError_t e = c->unOut.reserve(*total);
  if (e == hipSuccess) return SZ4_OK;
  if (c->unSplit) {
    for (DevBuf* b : {&c->unSubs, &c->unMasks, &c->unImage, &c->unSeq, &c->unIx}) b->release();
    const int mode = c->unSplitMode;
    c->unSplitMode = 0;
    const int r = unlz4_plan(c, f, n, total, keep, nullptr);
    c->unSplitMode = mode;
    if (r) return r;
    e = c->unOut.reserve(*total);
    if (e == hipSuccess) return SZ4_OK;
  }
  return c->fail(SZ4_E_NOMEM, "output", e);
}

int unlz4_decode(sz4_ctx* c, const uint8_t* f, uint64_t n, const uint8_t* dict, uint64_t dl, uint8_t* out, uint32_t keep,
                 hipStream_t s)
{
  if (!keep) return SZ4_OK;
  hipError_t e;
  if (c->unSplit) {
    // split mode: the u32 image of the output, its references resolved, then packed into `out`
    const UnBlock& lastB = c->hUn[keep - 1];
    const uint64_t total = lastB.dst + lastB.size;
    const uint32_t nsub = lastB.subFirst + lastB.subCount;
    if (c->unImage.cap < total * 4 + 64 || c->unFlags.cap < 64) return c->fail(SZ4_E_NOMEM, "decoder image");
    uint32_t* flag = c->unFlags.as<uint32_t>();
    if ((e = hipMemcpyAsync(c->unBlk.p, c->hUn.data(), keep * sizeof(UnBlock), hipMemcpyHostToDevice, s)))
      return c->fail(SZ4_E_DEVICE, "decoder plan", e);
    launch_unlz4_split_decode(f, n, c->unBlk.as<UnBlock>(), c->unSubs.as<UnSub>(), nsub, c->unSeq.as<uint4>(),
                              c->unImage.as<uint32_t>(), dict, dl, s);
    // the pack follows every reference chain to its byte (each hop lands in an earlier sub-segment): no
    // host round trip between passes; unResolvePasses reports the longest chain
    if ((e = hipMemsetAsync(flag, 0, 4, s))) return c->fail(SZ4_E_DEVICE, "decoder resolve", e);
    launch_unlz4_pack(c->unImage.as<uint32_t>(), total, out, flag, s);
    uint32_t hops = 0;
    if ((e = hipGetLastError()) || (e = hipMemcpyAsync(&hops, flag, 4, hipMemcpyDeviceToHost, s)) ||
        (e = hipStreamSynchronize(s)))
      return c->fail(SZ4_E_DEVICE, "decode", e);
    c->unResolvePasses = hops;
    return SZ4_OK;
  }
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
// is fixed by the chunk size, whatever the input length.  Three streams overlap the chunks: while the
// compute stream runs chunk k+1, chunk k comes down on the download stream and goes to sendBytes, and
// chunk k+2 is pulled through getBytes and goes up on the upload stream (two staging and two output
// slots).  Both callbacks run on the caller's thread.
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

// grows pinned buffer b to at least `bytes`, keeping its first `keep` bytes
hipError_t grow_pinned(HostBuf& b, uint64_t bytes, uint64_t keep)
{
  if (bytes <= b.cap) return hipSuccess;
  void* p = nullptr;
  hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
  if (e != hipSuccess) return e;
  if (keep && b.p) memcpy(p, b.p, keep);
  if (b.p) hipHostFree(b.p);
  b.p = p;
  b.cap = bytes;
  return hipSuccess;
}

// reads up to `want` bytes through getBytes, 64 KiB per call (the reference's BufferSize), into pinned
// buffer b, which grows as it fills (a small input pins little); *eof is set once getBytes returns 0.
// A getBytes that returns more than it was asked for is an error (*bad)
uint64_t pull(HostBuf& b, sz4_get_bytes get, void* user, uint64_t want, bool* eof, hipError_t* err, bool* bad)
{
  uint64_t got = 0;
  while (got < want && !*eof) {
    if (got == b.cap && (*err = grow_pinned(b, std::min<uint64_t>(want, std::max<uint64_t>(4 * b.cap, 1u << 20)), got)))
      return got;
    const uint64_t ask = std::min<uint64_t>(65536, std::min<uint64_t>(want, b.cap) - got);
    const size_t k = get(b.as<uint8_t>() + got, (size_t)ask, user);
    if (k > ask) {
      *bad = true;
      *eof = true;
      return got;
    }
    if (k == 0) *eof = true;
    got += k;
  }
  return got;
}

// one chunk of the stream: [pre carried bytes | n new bytes] in stagedS[slot]
struct StreamChunk {
  uint64_t pre = 0, n = 0;
  bool first = false;
  uint64_t shift() const { return (pre + n - 65536) / 65536 * 65536; }  // carry: [shift, pre + n) moves to 0
  uint64_t nextPre() const { return pre + n - shift(); }
};

// the block plan of a chunk (smallz4.h:572-585: 4 MiB blocks seeing the previous 64 KiB, or 8 MiB
// independent legacy blocks); cached: equal-shaped chunks reuse the plan and its device copy
void plan_chunk(sz4_ctx* c, const StreamChunk& ch, int legacy, bool dictMode)
{
  const uint64_t key[5] = {ch.pre, ch.n, ch.first ? 1ull : 0ull, (uint64_t)legacy, dictMode ? 1ull : 0ull};
  if (memcmp(key, c->streamPlanKey, sizeof key) == 0) return;
  memcpy(c->streamPlanKey, key, sizeof key);
  const uint64_t bs = legacy ? kBlockMaxLegacy : kBlockMax;
  c->hBlocks.clear();
  for (uint64_t st = 0; st < ch.n; st += bs) {
    Block B{};
    B.start = ch.pre + st;
    B.end = ch.pre + std::min(st + bs, ch.n);
    if (legacy || (st == 0 && ch.first)) {
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
  if (nb && c->hBlocks[0].prev == kNoBlock - 1) c->hBlocks[0].prev = nb;
  finish_plan(c);
  c->planN = ~0ull;  // invalidate the independent-block plan cache
}

// drains the stream path's streams before an early return (nothing may still run on its buffers)
struct StreamDrain {
  sz4_ctx* c;
  ~StreamDrain()
  {
    for (hipStream_t x : {c->upStream, c->stream, c->downStream})
      if (x) hipStreamSynchronize(x);
  }
};

int stream_compress_body(sz4_ctx* c, sz4_get_bytes get, sz4_send_bytes send, uint32_t maxChain, const uint8_t* dict,
                         uint64_t dictLen, int legacy, void* user, void* out)
{
  hipError_t e;
  for (hipStream_t* x : {&c->stream, &c->upStream, &c->downStream})
    if (!*x && (e = hipStreamCreateWithFlags(x, hipStreamNonBlocking))) return c->fail(SZ4_E_DEVICE, "stream", e);
  for (int k = 0; k < 2; k++)
    for (hipEvent_t* x : {&c->evUp[k], &c->evDone[k]})
      if (!*x && (e = hipEventCreateWithFlags(x, hipEventDisableTiming))) return c->fail(SZ4_E_DEVICE, "event", e);
  const uint64_t bs = legacy ? kBlockMaxLegacy : kBlockMax;
  const uint64_t chunk = std::max<uint64_t>(bs, c->streamChunk / bs * bs);
  const bool dictMode = dictLen != 0;
  // header (smallz4.h:478-496)
  const uint8_t hm[7] = {0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF};
  const uint8_t hl[4] = {0x02, 0x21, 0x4C, 0x18};
  send(legacy ? hl : hm, legacy ? 4 : 7, out);
  StreamDrain drain{c};
  bool eof = false, bad = false;
  hipError_t he = hipSuccess;
  StreamChunk ch[2];
  ch[0].n = pull(c->hostIn[0], get, user, chunk, &eof, &he, &bad);
  if (he) return c->fail(SZ4_E_NOMEM, "pinned host buffers", he);
  if (bad) return c->fail(SZ4_E_ARG, "getBytes returned more bytes than asked for");
  // dictionary: the staged stream starts with the reference's data buffer, a 65535-byte prefix (the
  // dictionary's last bytes, zero-padded in front) (smallz4.h:554-571)
  c->dictBack = dictMode ? (int64_t)std::min<uint64_t>(dictLen, kWindow) : -1;
  c->dictLegacy = legacy;
  c->dictCont = 0;
  c->ghost = false;
  ch[0].pre = dictMode && ch[0].n ? kWindow : 0;
  ch[0].first = true;
  if (ch[0].n) {
    // device buffers fixed by the chunk size (by the input when it is shorter than a chunk); the
    // scratch is sized once for the steady-state chunk shape, so no buffer moves mid-stream
    const uint64_t span = eof ? ch[0].n : chunk;
    const uint64_t stage = (eof ? ch[0].pre : kCarryMax) + span + kPad;
    if ((e = c->stagedS[0].reserve(stage)) || (!eof && (e = c->stagedS[1].reserve(stage))) ||
        (e = c->chunkOut[0].reserve(sz4_lz4_bound(span, legacy))) ||
        (!eof && (e = c->chunkOut[1].reserve(sz4_lz4_bound(span, legacy)))))
      return c->fail(SZ4_E_NOMEM, "stream staging", e);
    StreamChunk worst;
    worst.pre = eof ? ch[0].pre : kCarryMax - 1;
    worst.n = span;
    worst.first = eof;
    plan_chunk(c, worst, legacy, dictMode);
    if (int r = reserve_all(c, worst.pre + worst.n + kPad)) return r;
  }
  if (dictMode && ch[0].n) {
    std::vector<uint8_t> prefix(kWindow, 0);
    const uint64_t k = std::min<uint64_t>(dictLen, kWindow);
    memcpy(prefix.data() + kWindow - k, dict + dictLen - k, k);
    if ((e = hipMemcpy(c->stagedS[0].p, prefix.data(), kWindow, hipMemcpyHostToDevice)))
      return c->fail(SZ4_E_DEVICE, "upload", e);
  }
  // chunk k -> slot k & 1: upload on the copy stream (after chunk k-2 let go of the slot), with the
  // previous chunk's carried bytes in front
  auto upload = [&](uint32_t k) -> int {
    const uint32_t sl = k & 1;
    const StreamChunk& x = ch[sl];
    uint8_t* dst = c->stagedS[sl].as<uint8_t>();
    if (k >= 2 && (e = hipStreamWaitEvent(c->upStream, c->evDone[sl], 0))) return c->fail(SZ4_E_DEVICE, "upload", e);
    if ((e = hipMemcpyAsync(dst + x.pre, c->hostIn[sl].p, x.n, hipMemcpyHostToDevice, c->upStream)) ||
        (k >= 1 && (e = hipMemcpyAsync(dst, c->stagedS[sl ^ 1].as<uint8_t>() + ch[sl ^ 1].shift(), x.pre,
                                       hipMemcpyDeviceToDevice, c->upStream))) ||
        (e = hipMemsetAsync(dst + x.pre + x.n, 0, kPad, c->upStream)) || (e = hipEventRecord(c->evUp[sl], c->upStream)))
      return c->fail(SZ4_E_DEVICE, "upload", e);
    return SZ4_OK;
  };
  // enqueue chunk k's pipeline on the compute stream (returns with the kernels in flight)
  auto compute = [&](uint32_t k) -> int {
    const uint32_t sl = k & 1;
    const StreamChunk& x = ch[sl];
    c->ghost = !legacy && !x.first && !dictMode;
    plan_chunk(c, x, legacy, dictMode);
    if (int r = reserve_all(c, x.pre + x.n + kPad)) return r;
    if ((e = hipStreamWaitEvent(c->stream, c->evUp[sl], 0))) return c->fail(SZ4_E_DEVICE, "chunk", e);
    uint64_t unused = 0;
    if (int r = run_pipeline(c, maxChain, c->stagedS[sl].as<uint8_t>(), nullptr, 0, false, c->chunkOut[sl].as<uint8_t>(),
                             c->chunkOut[sl].cap, &unused, c->stream, false))
      return r;
    if ((e = hipEventRecord(c->evDone[sl], c->stream))) return c->fail(SZ4_E_DEVICE, "chunk", e);
    return SZ4_OK;
  };
  // chunk k's frame size; the state its successor takes: the last block's final shortcut intervals
  // (the ghost slot) and dictionary mode's table position
  auto finish = [&](uint32_t k, uint64_t* size) -> int {
    const uint32_t sl = k & 1;
    const StreamChunk& x = ch[sl];
    if (int r = pipeline_finish(c, nullptr, 0, false, c->chunkOut[sl].as<uint8_t>(), c->chunkOut[sl].cap, size, c->stream))
      return r;
    const uint64_t shift = x.shift();
    const uint32_t nb = (uint32_t)c->hBlocks.size();
    if (!legacy && !dictMode) {
      uint32_t cnt = 0;
      if ((e = hipMemcpyAsync(&cnt, c->ivCount.as<uint32_t>() + (nb - 1), 4, hipMemcpyDeviceToHost, c->stream)) ||
          (e = hipStreamSynchronize(c->stream)))
        return c->fail(SZ4_E_DEVICE, "intervals", e);
      std::vector<Interval> iv(cnt);
      if (cnt && ((e = hipMemcpyAsync(iv.data(), c->iv.as<Interval>() + (uint64_t)(nb - 1) * kMaxIv, cnt * sizeof(Interval),
                                      hipMemcpyDeviceToHost, c->stream)) || (e = hipStreamSynchronize(c->stream))))
        return c->fail(SZ4_E_DEVICE, "intervals", e);
      c->ghostIv.clear();
      for (Interval y : iv) {
        if (y.hi <= shift) continue;
        y.lo = std::max(y.lo, shift) - shift;
        y.hi -= shift;
        y.a = y.a >= shift ? y.a - shift : 0;
        c->ghostIv.push_back(y);
      }
    }
    if (dictMode) {
      c->dictCont = legacy ? 0u : 1u;
      c->dictShift = (uint32_t)shift;
      c->dictLow0 = (uint32_t)(x.nextPre() - kWindow);
    }
    return SZ4_OK;
  };
  // the next chunk's bytes: [previous chunk's carry | new bytes]
  auto next_chunk = [&](uint32_t k) -> bool {
    const uint32_t sl = k & 1;
    if (eof) return false;
    if (k >= 2 && (e = hipEventSynchronize(c->evUp[sl]))) {  // the pinned buffer's previous upload
      c->fail(SZ4_E_DEVICE, "upload", e);
      return false;
    }
    ch[sl].n = pull(c->hostIn[sl], get, user, chunk, &eof, &he, &bad);
    ch[sl].pre = ch[sl ^ 1].nextPre();
    ch[sl].first = false;
    return ch[sl].n != 0 && !he && !bad;
  };
  if (!ch[0].n) {
    if (!legacy) {
      static const uint8_t zero[4] = {0, 0, 0, 0};
      send(zero, 4, out);  // end mark (smallz4.h:807-812)
    }
    return SZ4_OK;
  }
  if (int r = upload(0)) return r;
  if (int r = compute(0)) return r;
  bool have = next_chunk(1);
  if (he) return c->fail(SZ4_E_NOMEM, "pinned host buffers", he);
  if (bad) return c->fail(SZ4_E_ARG, "getBytes returned more bytes than asked for");
  if (have)
    if (int r = upload(1)) return r;
  // SZ4_STREAM_PROFILE=1: where the caller's thread spends its time, per phase, on stderr
  const bool prof = getenv("SZ4_STREAM_PROFILE") != nullptr;
  double tp[6] = {0, 0, 0, 0, 0, 0};
  auto now = []() { return std::chrono::steady_clock::now(); };
  auto lap = [&](std::chrono::steady_clock::time_point& t, int i) {
    const auto u = now();
    tp[i] += std::chrono::duration<double>(u - t).count();
    t = u;
  };
  for (uint32_t k = 0;; k++) {
    const uint32_t sl = k & 1;
    uint64_t size = 0;
    auto t = now();
    if (int r = finish(k, &size)) return r;
    lap(t, 0);
    if (have)
      if (int r = compute(k + 1)) return r;  // the GPU goes on with chunk k+1 ...
    lap(t, 1);
    // ... while chunk k comes down (its copy overlaps the read of chunk k+2) and goes out, and chunk
    // k+2 is read and goes up
    if ((e = grow_pinned(c->hostOut[sl], std::max<uint64_t>(size, 1), 0))) return c->fail(SZ4_E_NOMEM, "pinned host buffers", e);
    if ((e = hipMemcpyAsync(c->hostOut[sl].p, c->chunkOut[sl].p, size, hipMemcpyDeviceToHost, c->downStream)))
      return c->fail(SZ4_E_DEVICE, "download", e);
    const bool more = have;
    if (more) {
      have = next_chunk(k + 2);
      if (he) return c->fail(SZ4_E_NOMEM, "pinned host buffers", he);
      if (bad) return c->fail(SZ4_E_ARG, "getBytes returned more bytes than asked for");
      lap(t, 4);
      if (have)
        if (int r = upload(k + 2)) return r;
      lap(t, 5);
    }
    if ((e = hipStreamSynchronize(c->downStream))) return c->fail(SZ4_E_DEVICE, "download", e);
    lap(t, 2);
    send_blocks(c->hostOut[sl].as<uint8_t>(), size, send, out);
    lap(t, 3);
    if (!more) break;
  }
  if (prof)
    fprintf(stderr, "sz4 stream: finish-wait %.3f s, enqueue %.3f s, download %.3f s, sendBytes %.3f s, getBytes %.3f s, "
            "upload-enqueue %.3f s\n", tp[0], tp[1], tp[2], tp[3], tp[4], tp[5]);
  if (!legacy) {
    static const uint8_t zero[4] = {0, 0, 0, 0};
    send(zero, 4, out);  // end mark (smallz4.h:807-812)
  }
  return SZ4_OK;
}

// smallz4::lz4 over the callbacks.  A callback's exception (a C++ caller's sendBytes may throw) leaves
// through here after the streams have drained; an allocation failure becomes SZ4_E_NOMEM
int stream_compress(sz4_ctx* c, sz4_get_bytes get, sz4_send_bytes send, uint32_t maxChain, const uint8_t* dict,
                    uint64_t dictLen, int legacy, void* user, void* sinkUser = nullptr)
{
  c->dictRounds = 0;  // sz4_dict_rounds reports this call's chunks
  try {
    return stream_compress_body(c, get, send, maxChain, dict, dictLen, legacy, user, sinkUser ? sinkUser : user);
  } catch (const std::bad_alloc&) {
    return c->fail(SZ4_E_NOMEM, "host allocation");
  }
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

constexpr uint32_t kMaxFrameBlock = (uint32_t)(kBlockMaxLegacy + kBlockMaxLegacy / 255 + 16);  // LZ4 compress bound

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
    // one upload, one plan (its block sizes give the output length), one decode, one download
    hipError_t e;
    const uint64_t dl = hist.size(), fl = frame.size();
    if ((e = c->unFrame.reserve(fl + 64)) || (e = c->unDict.reserve(dl + 64))) return c->fail(SZ4_E_NOMEM, "staging", e);
    if ((e = hipMemcpy(c->unFrame.p, frame.data(), fl, hipMemcpyHostToDevice)) ||
        (dl && (e = hipMemcpy(c->unDict.p, hist.data(), dl, hipMemcpyHostToDevice))))
      return c->fail(SZ4_E_DEVICE, "upload", e);
    uint64_t size = 0;
    uint32_t keep = 0;
    if (int r = unlz4_plan(c, c->unFrame.as<uint8_t>(), fl, &size, &keep, nullptr)) return r;
    out.resize(size);
    if (size) {
      if (int r = unlz4_reserve_out(c, c->unFrame.as<uint8_t>(), fl, &size, &keep)) return r;
      if (int r = unlz4_decode(c, c->unFrame.as<uint8_t>(), fl, dl ? c->unDict.as<uint8_t>() : nullptr, dl,
                               c->unOut.as<uint8_t>(), keep, nullptr))
        return r;
      if ((e = hipMemcpy(out.data(), c->unOut.p, size, hipMemcpyDeviceToHost))) return c->fail(SZ4_E_DEVICE, "download", e);
    }
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
    // no LZ4 block is larger than a legacy 8 MiB block's worst case: a larger size word is corrupt
    // (the reference would read on until its input ends; this decoder must not reserve gigabytes first)
    if (word > kMaxFrameBlock) return c->fail(SZ4_E_CORRUPT, "block size word larger than any LZ4 block");
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
  // tuning knobs (A/B): the batch API's piece size and the stream path's chunk size in bytes
  // (sz4_set_batch_chunk / sz4_set_stream_chunk set them per context)
  if (const char* bc = getenv("SZ4_BATCH_CHUNK")) {
    const uint64_t v = strtoull(bc, nullptr, 10);
    if (v >= (1u << 20)) {
      c->batchChunk = v;
      c->batchChunkSet = true;
    }
  }
  if (const char* sc = getenv("SZ4_STREAM_CHUNK")) {
    const uint64_t v = strtoull(sc, nullptr, 10);
    if (v >= (1u << 20)) c->streamChunk = v;
  }
  for (auto& e : c->ev) hipEventCreate(&e);
  c->budget.bufs = c->all_buffers();
  for (DevBuf* b : c->budget.bufs) b->bud = &c->budget;
  c->budget.owner = c;
  // a released plan buffer may come back at the same address: upload the plan again
  c->budget.onShed = [](void* o) { static_cast<sz4_ctx*>(o)->uploadedVersion = ~0ull; };
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
  for (hipStream_t x : {c->stream, c->upStream, c->downStream})
    if (x) hipStreamDestroy(x);
  for (int k = 0; k < 2; k++)
    for (hipEvent_t x : {c->evUp[k], c->evDone[k]})
      if (x) hipEventDestroy(x);
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

// pooled contexts holding more device scratch than this are trimmed when they are returned
static std::atomic<uint64_t> g_poolCap{8ull << 30};

void sz4_release(sz4_ctx* c)
{
  if (!c || !c->pooled || !c->poolMu) return;
  if (c->budget.used > g_poolCap.load()) sz4_trim(c);
  std::lock_guard<std::mutex> lock(*c->poolMu);
  c->poolIdle->push_back(c);
}

void sz4_set_pool_cap(uint64_t bytes) { g_poolCap.store(bytes ? bytes : (8ull << 30)); }

void sz4_trim(sz4_ctx* c)
{
  if (!c) return;
  DeviceGuard guard(c->device);
  for (hipStream_t x : {c->stream, c->upStream, c->downStream})
    if (x) hipStreamSynchronize(x);
  for (DevBuf* b : c->all_buffers()) b->release();
  for (HostBuf* b : {&c->hostIn[0], &c->hostIn[1], &c->hostOut[0], &c->hostOut[1]}) b->release();
  c->uploadedVersion = ~0ull;
}

void sz4_set_device_limit(sz4_ctx* c, uint64_t bytes)
{
  if (c) c->budget.limit = bytes;
}

uint64_t sz4_released_buffers(sz4_ctx* c) { return c ? c->budget.shedCount : 0; }

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
  c->begin_call();
  // the kernels write the frame in place: refuse a buffer that could be overrun
  if (out_cap < sz4_bound(n, block_size)) return c->fail(SZ4_E_CAPACITY, "out_cap < sz4_bound(n, block_size)");
  DeviceGuard guard(c->device);
  try {
  c->ghost = false;
  hipStream_t s = (hipStream_t)stream;
  c->dictBack = -1;
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
  c->batchChunked = false;
  if (n == 0) {
    if (out_cap < hl + (endMark ? 4 : 0)) return c->fail(SZ4_E_CAPACITY, "output buffer too small");
    if (hl) hipMemcpyAsync(d_out, hdr, hl, hipMemcpyHostToDevice, s);
    if (endMark) hipMemsetAsync((uint8_t*)d_out + hl, 0, 4, s);
    hipStreamSynchronize(s);
    c->lastBlocks = 0;
    *out_size = hl + (endMark ? 4 : 0);
    return SZ4_OK;
  }
  // bounded memory: whole blocks in pieces of at most batchChunk input bytes, one pipeline run each
  // (the scratch is ~60-75 bytes per input byte), written one after the other into d_out
  // under a device bound the pieces shrink with it (the scratch is 36-60 bytes per piece byte)
  // Without a bound the default piece is capped so that its scratch (< kScratchPerByte per piece byte) takes at
  // most a quarter of the memory this context could use now (free + what it holds): a GPU shared with a
  // caching allocator gets smaller pieces instead of SZ4_E_NOMEM.  A piece whose reservation still fails is
  // halved and retried, down to kPieceFloor
  uint64_t chunk = c->batchChunk;
  if (c->budget.limit) {
    chunk = std::min<uint64_t>(chunk, std::max<uint64_t>(kPieceFloor, c->budget.limit / 64));
  } else if (!c->batchChunkSet) {
    size_t freeB = 0, totalB = 0;
    if (hipMemGetInfo(&freeB, &totalB) == hipSuccess)
      chunk = std::min<uint64_t>(chunk, std::max<uint64_t>(kPieceFloor, (freeB + c->budget.used) / (4 * kScratchPerByte)));
    else
      (void)hipGetLastError();
  }
  // equal pieces (the last one is not a small remainder): ceil(n / chunk) of them, whole blocks each
  const uint64_t nPieces = (n + chunk - 1) / std::max<uint64_t>(chunk, 1);
  const uint64_t even = (n + nPieces - 1) / nPieces;
  uint64_t piece = std::max<uint64_t>(block_size, (even + block_size - 1) / block_size * block_size);
  float stageSum[kStages] = {};
  uint64_t pos = 0;
  c->hostBytes.clear();
  for (uint64_t off = 0; off < n; off += piece) {
    const uint64_t len = std::min(piece, n - off);
    const bool firstPiece = off == 0, lastPiece = off + len == n;
    if (c->planN != len || c->planBS != block_size) {
      c->hBlocks.clear();
      for (uint64_t st = 0; st < len; st += block_size) {
        Block B{};
        B.start = st;
        B.end = std::min<uint64_t>(st + block_size, len);
        B.low = st;
        B.cut = kNone;
        B.prev = kNoBlock;
        B.flags = 0;
        c->hBlocks.push_back(B);
      }
      finish_plan(c);
      c->planN = len;
      c->planBS = block_size;
      c->streamPlanKey[0] = ~0ull;  // invalidate the stream path's plan cache
    }
    hipError_t e = hipSuccess;
    int rr = reserve_all(c, len + kPad);
    if (rr == SZ4_OK && (e = c->staged.reserve(len + kPad))) rr = c->fail(SZ4_E_NOMEM, "staging", e);
    if (rr == SZ4_E_NOMEM && piece > block_size && piece > kPieceFloor) {
      // smaller pieces: the next iteration re-plans this offset with half the piece
      piece = std::max<uint64_t>(block_size, std::max<uint64_t>(kPieceFloor, piece / 2) / block_size * block_size);
      c->planN = ~0ull;
      off -= piece;  // the loop adds it back
      continue;
    }
    if (rr) return rr;
    // private padded copy: kernels read 4-byte windows that may run past the caller's buffer
    if ((e = hipMemcpyAsync(c->staged.p, (const uint8_t*)d_in + off, len, hipMemcpyDeviceToDevice, s)))
      return c->fail(SZ4_E_DEVICE, "stage input", e);
    if ((e = hipMemsetAsync(c->staged.as<uint8_t>() + len, 0, kPad, s))) return c->fail(SZ4_E_DEVICE, "stage pad", e);
    uint64_t size = 0;
    if (int r = run_pipeline(c, max_chain, c->staged.as<uint8_t>(), hdr, firstPiece ? hl : 0, lastPiece && endMark,
                             (uint8_t*)d_out + pos, out_cap - pos, &size, s))
      return r;
    pos += size;
    for (int i = 0; i < kStages; i++) stageSum[i] += c->stageMs[i];
    if (!(firstPiece && lastPiece)) {
      // every piece's block sizes, for sz4_last_block_sizes
      const uint32_t nb = (uint32_t)c->hBlocks.size();
      const size_t at = c->hostBytes.size();
      c->hostBytes.resize(at + nb);
      if ((e = hipMemcpy(c->hostBytes.data() + at, c->blockBytes.p, nb * 4, hipMemcpyDeviceToHost)))
        return c->fail(SZ4_E_DEVICE, "block sizes", e);
    }
  }
  c->batchChunked = !c->hostBytes.empty();
  if (c->timing)
    for (int i = 0; i < kStages; i++) c->stageMs[i] = stageSum[i];
  *out_size = pos;
  return SZ4_OK;
  } catch (const std::bad_alloc&) {
    return c->fail(SZ4_E_NOMEM, "host allocation");
  }
}

int64_t sz4_last_block_sizes(sz4_ctx* c, uint32_t* sizes, uint64_t max_blocks)
{
  if (!c || !sizes) return SZ4_E_ARG;
  if (c->batchChunked) {
    const uint64_t nb = std::min<uint64_t>(c->hostBytes.size(), max_blocks);
    for (uint64_t i = 0; i < nb; i++) sizes[i] = c->hostBytes[i] & 0x7FFFFFFFu;
    return (int64_t)nb;
  }
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
  c->begin_call();
  DeviceGuard guard(c->device);
  return stream_compress(c, get_bytes, send_bytes, max_chain, (const uint8_t*)dict, dict_len, legacy, user);
}

int sz4_lz4(sz4_ctx* c, const void* in, uint64_t n, uint32_t max_chain, const void* dict, uint64_t dict_len, int legacy,
            void* out, uint64_t out_cap, uint64_t* out_size)
{
  if (!c || !out_size || (!in && n) || !out || max_chain > 65535 || (dict_len && !dict))
    return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->begin_call();
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

void sz4_set_batch_chunk(sz4_ctx* c, uint64_t bytes)
{
  if (c) {
    c->batchChunk = bytes ? bytes : kBatchChunkDefault;
    c->batchChunkSet = bytes != 0;
  }
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
  const uint32_t* lens = c->stopAfter == 4 && c->lastChain > (uint32_t)kGreedyMax ? c->sel() : c->mlen.as<uint32_t>();
  if (hipMemcpy(len, lens, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(dist, c->mdist.p, n * 2, hipMemcpyDeviceToHost) != hipSuccess)
    return SZ4_E_DEVICE;
  return SZ4_OK;
}

int sz4_unlz4_device(sz4_ctx* c, const void* d_frame, uint64_t frame_len, const void* d_dict, uint64_t dict_len,
                     void* d_out, uint64_t out_cap, uint64_t* out_size, void* stream)
{
  if (!c || !out_size || (!d_frame && frame_len) || (dict_len && !d_dict))
    return c ? c->fail(SZ4_E_ARG, "bad argument") : SZ4_E_ARG;
  c->begin_call();
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
  c->begin_call();
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
  if (int r = unlz4_reserve_out(c, c->unFrame.as<uint8_t>(), frame_len, &total, &keep)) return r;
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
  c->begin_call();
  DeviceGuard guard(c->device);
  try {
    return stream_decompress(c, get_byte, send_bytes, (const uint8_t*)dict, dict_len, user);
  } catch (const std::bad_alloc&) {
    return c->fail(SZ4_E_NOMEM, "host allocation");
  }
}

uint64_t sz4_device_bytes(sz4_ctx* c)
{
  if (!c) return 0;
  return c->budget.used;
}

uint32_t sz4_dict_rounds(sz4_ctx* c) { return c ? c->dictRounds : 0u; }

uint32_t sz4_unlz4_resolve_passes(sz4_ctx* c) { return c && c->unSplit ? c->unResolvePasses : 0u; }

int sz4_unlz4_index_parallel(sz4_ctx* c) { return c && c->unIndexParallel ? 1 : 0; }

const char* sz4_last_error(sz4_ctx* c) { return c ? c->err.c_str() : "no context"; }

}  // extern "C"
