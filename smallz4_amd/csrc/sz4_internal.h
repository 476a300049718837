// sz4_internal.h -- descriptors shared by the host driver (sz4_host.cpp) and the
// gfx950 kernels (sz4_kernels.hip).  Not part of the public ABI.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace sz4 {

// constants of the reference format (smallz4.h:92-131)
constexpr int kMinMatch = 4;             // MinMatch
constexpr int kTailNoMatch = 12;         // BlockEndNoMatch
constexpr int kTailLiterals = 5;         // BlockEndLiterals
constexpr uint32_t kWindow = 65535;      // MaxDistance
constexpr uint32_t kSameLetter = 19 + 255 * 256;  // MaxSameLetter
constexpr int kGreedyMax = 3;            // ShortChainsGreedy
constexpr int kLazyMax = 6;              // ShortChainsLazy
constexpr uint32_t kHashMul = 48271;     // getHash32 multiplier
constexpr int kHashBits = 20;
constexpr uint64_t kNone = ~0ull;
// the parse's per-block flags (longFlag), set by every match finder (sz4_kernels.hip, sz4_dict.hip)
constexpr uint32_t kRmqLen = 274;  // match lengths from here on use the parse's range minima
constexpr uint32_t kFlagRmq = 1;   // the block has matches of kRmqLen+ (other than same-letter runs)
constexpr uint32_t kFlagRun = 2;   // a distance-1 match longer than MaxSameLetter (bounded chains)
constexpr int kStages = 6;  // runs, sort, find (sorted pass), find (long pass), parse, assemble

// device status word bits (one int per pipeline run)
constexpr int kStPrepRound = 2;   // k_lazy_correct corrected a shortcut interval: run sort/find/walk again
constexpr int kStInvariant = 4;   // a capacity invariant of the walk/token kernels failed: the frame is invalid

// one LZ4 block (all positions absolute byte offsets in the staged input)
struct Block {
  uint64_t start, end;     // [start, end)
  uint64_t low;            // lowest position a match may reference (reference dataZero)
  uint64_t cut;            // start-12 when the block re-inserts the previous tail (lookback), else kNone
  uint64_t tokOff;         // first Token slot of this block (capacity (end-start)/2 + 4)
  uint32_t prev;           // index of the previous block of the same stream, or kNoBlock
  uint32_t flags;          // kBlk* below
  uint32_t dpFirst;        // first DpSeg of this block (top segment first)
  uint32_t dpCount;        // number of DpSegs (0 when the block is too short to parse)
  uint32_t walkFirst;      // first token-walk sub-segment of this block
  uint32_t walkCount;      // number of token-walk sub-segments (ceil(n / kWalkSeg))
  uint32_t dpSize;         // positions per parse segment (dp_segment_size(n))
  uint32_t pad;
};
constexpr uint32_t kNoBlock = 0xFFFFFFFFu;
constexpr uint32_t kBlkLegacy = 1;         // always emitted compressed (legacy frame)

// targets [s0, s1) of one block, searched against the window [w0, s1)
struct Segment {
  uint64_t w0, s0, s1;
  uint64_t elemOff;        // offset (elements) of this segment's sort scratch
  uint64_t rankOff;        // offset (u32) of this segment's rank array (s1 - s0 entries)
  uint32_t block;
  uint32_t pad;
};

// positions [lo, hi) are skipped by the reference's same-letter shortcut
// (smallz4.h:631-643): not inserted into the chains and given (dist 1, La - (p - a))
struct Interval {
  uint64_t lo, hi;
  uint64_t a;              // the position whose distance-1 match starts the shortcut
  uint64_t La;             // its match length
};
// block b owns iv[b * kMaxIv .. b * kMaxIv + ivCount[b]); slot nblocks holds the final intervals of the
// previous chunk's last block when a stream is compressed in chunks (the first block's B.prev)
constexpr uint32_t kMaxIv = 136;  // > 8 MiB / 65300

// the optimal parse of one block runs as independent segments of B.dpSize positions (top segment
// first, k = 0): every segment is parsed at once from a guessed boundary, then k_dp_fix walks the
// boundaries top-down and re-parses each segment until it agrees with the speculative parse.
struct DpSeg {
  uint32_t block;
  uint32_t k;              // 0 = the segment holding the block's last parsed position
  uint32_t lo, hi;         // block-relative positions [lo, hi], parsed from hi down
};
// short segments give more parallelism; the serial part of the repair (k_dp_fix<false>) walks a
// block's boundaries one after the other, so large blocks keep longer segments
inline uint32_t dp_segment_size(uint64_t n) { return n <= 65536 ? 4096u : 8192u; }
constexpr uint32_t kMaxDpSegs = 2048;  // 8 MiB legacy block / 4096 (SZ4_DP_SIZE)

// the token walk runs as sub-segments of kWalkSeg positions, each walked speculatively from its
// first position and repaired by k_walk_fix; a sub-segment's match positions live in 2 * kWalkCap
// u32 slots (speculative ones from kWalkCap on, repaired ones prepended below them)
constexpr uint32_t kWalkSeg = 4096;
constexpr uint32_t kWalkCap = kWalkSeg / 4 + 2;

// one LZ4 sequence: literal run [litFrom, litFrom+lits) (block-relative) then a match
struct Token {
  uint32_t litFrom, lits, mlen, dist;  // dist: low 16 bits; kTokLast marks the final literals-only token
};
constexpr uint32_t kTokLast = 0x80000000u;

// kernels (sz4_kernels.hip)
uint32_t find_lds_bytes();
void launch_runs(const uint8_t* in, const Block* blocks, uint32_t nblocks, Interval* iv, uint32_t* ivCount,
                 hipStream_t s);
// pass 1 = k_find_sorted (each segment sorted first inside it: compact = sorted slot arrays, scratch = sort
// buffer, rank written), pass 2 = k_find_big / k_find_long9 / k_find (long matches and shortcut intervals)
// scratch: per-slot words free after the sort (the skip pointers of k_find_long9); longBits: one bit per
// position marked for pass 2 (searched, not a shortcut interval); segLong: per segment, any such target;
// specLen/specDist: per position words free before the parse (k_find_big's left-maximal results, then the
// speculative carries of pass-2 piece heads); segTail: per segment, k_find_big's state after its last target
void launch_find(int pass, const uint8_t* in, const Segment* segs, uint32_t nsegs, const Block* blocks,
                 const Interval* iv, const uint32_t* ivCount, uint2* compact, uint2* scratch,
                 uint32_t* rank, uint32_t maxChain, uint32_t* mlen, uint16_t* mdist, uint64_t matchBase,
                 uint32_t* longBits, uint32_t* segLong, uint32_t* longFlag, uint32_t* specLen, uint32_t* specDist,
                 uint64_t* segTail, bool ldsWindow, hipStream_t s);
// dictionary mode: one wavefront replays the reference's match loop (dictBack = first insertion offset
// before the first block); last: 2^20 u32, prevH / prevX: 65536 u16 each -- the reference's tables,
// kept in HBM between the chunks of one stream.  cont: the first block continues the stream of the
// previous launch, whose staged positions were `shift` (a multiple of 65536) higher; low0 = its dataZero
void launch_dict(const uint8_t* in, const Block* blocks, uint32_t nblocks, uint32_t maxChain, uint32_t dictBack, int legacy,
                 uint32_t* last, uint16_t* prevH, uint16_t* prevX, uint32_t cont, uint32_t shift, uint32_t low0,
                 uint32_t* mlen, uint16_t* mdist, uint32_t* sel, uint32_t* longFlag, hipStream_t s);
// dictionary mode on the whole GPU (sz4_dict.hip), modern and legacy frames: hBlocks is the host copy of
// the plan, walkSegs the token walk's sub-segments; ph / pe: one u16 per staged position; keysA / keysB:
// dict_sort_keys_max() u64 each; temp: dict_sort_temp_bytes(); scBits: dict_sc_bits_bytes().  iv /
// ivCount: the assumed same-letter shortcut intervals per block (kMaxIv each); the launch replaces them
// with the ones its results imply and raises kStPrepRound in *status when they differ (then the chunk
// is run again from its saved tables).  Returns 0, or -1 on a launch failure
constexpr uint64_t kBlockMaxDict = 4ull << 20;     // MaxBlockSize (smallz4.h:124)
constexpr uint64_t kBlockMaxLegacy = 8ull << 20;   // MaxBlockSizeLegacy (smallz4.h:125)
struct DictArgs {
  const uint8_t* in;
  const Block* dBlocks;
  const Block* hBlocks;
  uint32_t nb, maxChain, dictBack, cont, shift, low0;
  int legacy;
  Interval* iv;
  uint32_t* ivCount;
  uint32_t* last;
  uint16_t *prevH, *prevX, *ph, *pe;
  uint64_t *keysA, *keysB;
  void* temp;
  uint64_t tempBytes;
  uint32_t* mlen;
  uint16_t* mdist;
  uint32_t *sel, *longFlag;
  const uint2* walkSegs;
  uint32_t nwalk;
  uint32_t* lzMasks;
  uint4* lzState;
  uint64_t* scBits;
  int* status;
  uint2* runTab;      // runs covering whole 64-byte chunks: dict_run_table_bytes(staged) with runFlag
  uint32_t* runFlag;
  bool buildRuns;     // the first round of a chunk builds the table (the input does not change)
  bool guess;         // ... and appends its guess of the shortcut intervals to iv / ivCount (zeroed before)
};
uint64_t dict_sort_keys_max();
uint64_t dict_sort_temp_bytes();  // rocPRIM's scratch for dict_sort_keys_max() keys; 0 if the query failed
uint64_t dict_sc_bits_bytes(uint32_t nb, uint64_t maxBlock);
uint64_t dict_run_table_bytes(uint64_t staged);
int launch_dict_parallel(const DictArgs& a, hipStream_t s);
// greedy/lazy levels: dict_lz_mask_bytes_per_walk() bytes per token-walk sub-segment (lzMasks), one
// uint4 per sub-segment (lzState)
uint64_t dict_lz_mask_bytes_per_walk();
// k_prep: the tail positions the reference never searches (lengths 0, literal choices)
void launch_prep(const uint8_t* in, const Block* blocks, uint32_t nblocks, Interval* iv, uint32_t* ivCount, uint32_t maxChain,
                 uint32_t* mlen, uint16_t* mdist, uint64_t matchBase, uint32_t* sel, const uint32_t* longFlag, int* status,
                 hipStream_t s);
// greedy/lazy levels: the parallel replay of the reference's skip bookkeeping (k_lazy_walk / k_lazy_fix /
// k_lazy_clear) over the assumed same-letter shortcut intervals, then their check (k_lazy_check /
// k_lazy_correct: status kStPrepRound = an interval list was corrected, run sort/find/walk again);
// slots: lazy_slots_per_walk() u32 per walk sub-segment, state: one uint4 per walk sub-segment,
// firstBad: one u32 per block
void launch_lazy(const uint8_t* in, const Block* blocks, uint32_t nblocks, const uint2* walkSegs, uint32_t nwalk,
                 Interval* iv, uint32_t* ivCount, const uint32_t* longFlag, uint32_t* mlen, const uint16_t* mdist,
                 uint64_t matchBase, uint32_t* slots, uint4* state, uint32_t* firstBad, int* status, hipStream_t s);
uint32_t lazy_slots_per_walk();
// maxDpCount: the largest dpCount of the launch's blocks (sizes k_dp_fix<false>'s LDS tables)
void launch_parse(const uint8_t* in, const Block* blocks, uint32_t nblocks, const DpSeg* dpSegs, uint32_t ndp,
                  uint32_t maxDpCount, const uint32_t* ivCount, uint32_t maxChain, uint32_t* mlen, const uint16_t* mdist,
                  uint64_t matchBase, uint32_t* cost, uint32_t* sel, uint32_t* reach, uint4* segState,
                  const uint32_t* longFlag, uint32_t* rmqUp, uint32_t* rmqDown, uint2* dpSide, uint4* dpRec, int* status,
                  hipStream_t s);
// k_dp_fix<true>'s saved speculative values: dp_side_positions() uint2 per DpSeg, and one uint4 record per DpSeg
uint32_t dp_side_positions();
void launch_emit(const uint8_t* in, const Block* blocks, uint32_t nblocks, const uint2* walkSegs, uint32_t nwalk,
                 uint32_t maxChain, const uint32_t* chosen, const uint16_t* mdist, uint64_t matchBase, uint32_t* walkSlots,
                 uint4* walkState, uint32_t* posList, Token* tokens, uint32_t* ntok, uint32_t* blockBytes,
                 uint64_t* offsets, uint8_t* out, uint64_t headerLen, int* status, hipStream_t s);

// decoder (sz4_unlz4.hip): one block of an LZ4 frame
struct UnBlock {
  uint64_t src;       // payload offset in the frame
  uint64_t dst;       // output offset (set by the host after the sizes pass)
  uint64_t size;      // decoded bytes (k_unlz4_sizes / k_unlz4_fix), kNone when malformed
  uint32_t len;       // payload bytes
  uint32_t stored;    // 1: uncompressed block
  uint32_t nseq;      // sequences recorded by k_unlz4_sizes
  uint32_t subFirst;  // split mode: first sub-segment of the block
  uint32_t subCount;  // split mode: its sub-segments (ceil(len / kUnSub))
  uint32_t pad;
};
// Split mode (frames with large blocks): every block is cut into sub-segments of kUnSub payload bytes,
// parsed speculatively from their first byte (k_unlz4_spec), joined to the true token chain per block
// (k_unlz4_fix), decoded into a u32 value-or-reference image one wavefront per sub-segment
// (k_unlz4_sub), whose references to earlier sub-segments are resolved by pointer jumping
// (k_unlz4_resolve) before the bytes are packed (k_unlz4_pack).
constexpr uint32_t kUnSub = 8192;
constexpr uint32_t kUnSubCap = kUnSub / 3 + 4;    // sequences one walk over a sub-segment records
constexpr uint32_t kUnSplitMin = 256u << 10;      // a block of at least this many payload bytes: split mode
constexpr uint32_t kUnRef = 0x80000000u;          // image word: "same byte as output position (w & ~kUnRef)"
struct UnSub {
  uint32_t block, k;        // plan: block index, sub-segment index in the block
  uint32_t specN, specExit;  // k_unlz4_spec: sequences recorded, block-relative frame offset where it stopped
  uint32_t specFlags;        // 1: the walk met a malformed sequence at specExit, 2: it reached the block end
  uint32_t preN, specFrom;   // k_unlz4_fix: sequences re-parsed from the true entry, first speculative one kept
  uint32_t outRel, outLen;   // k_unlz4_fix: block-relative output offset and decoded bytes
  uint32_t specBytes;        // k_unlz4_spec: bytes its speculative list decodes
  // k_unlz4_join: the join computed from an ASSUMED entry (the previous sub-segment's speculative exit):
  // that entry, the exit it leads to, and 1: the previous walk was assumed to end there / 2: the join met a
  // malformed sequence / 4: this sub-segment reaches the block end.  k_unlz4_fix keeps it where the
  // assumption was the true chain's, and joins the others again from their true entry
  uint32_t joinEntry, joinExit, joinFlags;
};
// per sub-segment, k_unlz4_spec's side tables (u32 words): the token-start mask (kUnSub / 32 words), the
// mask's prefix bit counts per word (u16, kUnSub / 64 words), and each speculative sequence's output offset
// from the sub-segment's first token (kUnSubCap words) -- k_unlz4_fix's rank and byte count in O(1)
constexpr uint32_t kUnAuxWords = (kUnSub / 32 + kUnSub / 64 + kUnSubCap + 63) / 64 * 64;
void launch_unlz4_index(const uint8_t* f, uint64_t n, UnBlock* blk, uint64_t maxBlocks, uint64_t* meta, hipStream_t s);
// the same result from the parallel index (candidate offsets, then one wavefront over their successors;
// falls back to the serial walk in the same launch when the candidates cannot settle the chain)
void launch_unlz4_index_par(const uint8_t* f, uint64_t n, void* scratch, UnBlock* blk, uint64_t maxBlocks, uint64_t* meta,
                            hipStream_t s);
uint64_t unlz4_ix_scratch_bytes(uint64_t n);
uint64_t unlz4_ix_cap(uint64_t n);
// sequence list: unlz4_seq_entries(frame length, blocks) uint4 entries (block bi's at src / 3 + 2 bi)
uint64_t unlz4_seq_entries(uint64_t frameLen, uint32_t nb);
void launch_unlz4_sizes(const uint8_t* f, uint64_t n, UnBlock* blk, uint32_t nb, uint4* seq, hipStream_t s);
// flags: nb done flags, then the status word, then the ticket (zeroed before the launch)
void launch_unlz4_blocks(const uint8_t* f, uint64_t n, const UnBlock* blk, uint32_t nb, const uint4* seq, uint8_t* out,
                         const uint8_t* dict, uint64_t dl, uint32_t* flags, hipStream_t s);
// split mode: seq holds 2 * kUnSubCap entries per sub-segment (re-parsed prefix, speculative list), masks
// kUnAuxWords words per sub-segment (the token-start mask and k_unlz4_spec's side tables)
void launch_unlz4_split_sizes(const uint8_t* f, uint64_t n, UnBlock* blk, uint32_t nb, UnSub* subs, uint32_t nsub,
                              uint4* seq, uint32_t* masks, hipStream_t s);
// image: one u32 per output byte; hops: one u32 (zeroed before k_unlz4_pack: the longest reference chain it followed)
void launch_unlz4_split_decode(const uint8_t* f, uint64_t n, const UnBlock* blk, const UnSub* subs, uint32_t nsub,
                               const uint4* seq, uint32_t* image, const uint8_t* dict, uint64_t dl, hipStream_t s);
void launch_unlz4_pack(uint32_t* image, uint64_t total, uint8_t* out, uint32_t* hops, hipStream_t s);

}  // namespace sz4
