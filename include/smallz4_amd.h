/* smallz4_amd.h -- C ABI of the MI355X (gfx950) LZ4 optimal-parse compressor.
 *
 * Drop-in boundary for the reference's compression entry point
 *   smallz4::lz4(GET_BYTES, SEND_BYTES, maxChainLength, dictionary,
 *                useLegacyFormat, userPtr)          reference smallz4.h:47-64
 * Everything here is plain C: pointers, sizes, integer status codes.  The C++
 * mirror of the reference class (include/smallz4_amd.hpp) and the Python
 * package (smallz4_amd/) are thin layers over these symbols.
 *
 * Compression levels are the reference's maxChainLength (smallz4.cpp:175-239):
 *   0 stored, 1..3 greedy, 4..6 lazy + optimal parse, 7..65534 optimal parse
 *   with a chain limit, 65535 ("-9") unlimited optimal parse.
 * Output is byte-identical to the reference at the same level.
 */
#ifndef SMALLZ4_AMD_H
#define SMALLZ4_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define SZ4_OK              0
#define SZ4_E_ARG          -1  /* bad argument                                  */
#define SZ4_E_DEVICE       -2  /* HIP runtime error                             */
#define SZ4_E_CAPACITY     -3  /* output buffer too small                       */
#define SZ4_E_NOMEM        -4  /* device/host allocation failed                 */
#define SZ4_E_UNSUPPORTED  -5  /* reserved: every level, format and dictionary is supported */
#define SZ4_E_CORRUPT      -6  /* decoder: a frame the reference decoder rejects           */

/* frame header written by sz4_compress_blocks_device */
#define SZ4_HEADER_SMALLZ4     0  /* exactly smallz4's header: 04 22 4D 18 40 70 DF  */
#define SZ4_HEADER_INDEPENDENT 1  /* LZ4 frame flagged block-independent, BD sized   */
#define SZ4_HEADER_NONE        2  /* no header and no end mark: bare blocks          */

typedef struct sz4_ctx sz4_ctx;

/* Version of the reference interface mirrored (smallz4.h:67-70). */
const char* sz4_version(void);

/* Create a compression context bound to HIP device `device`.  Scratch space is
 * allocated lazily and grown on demand; `reserve_bytes` pre-sizes it for that
 * much input (0 = on first use).  A context serves one call at a time: threads
 * that compress concurrently use a context each.  Every call makes the
 * context's device current and restores the caller's current device. */
int sz4_create(sz4_ctx** ctx, int device, uint64_t reserve_bytes);
void sz4_destroy(sz4_ctx* ctx);

/* Process-wide context pool (thread-safe): sz4_acquire hands out an idle context of `device` (creating
 * one when all are busy), sz4_release returns it.  Concurrent callers get different contexts, so
 * calls through the pool are reentrant -- the reference builds a fresh object per call
 * (smallz4.h:56-64).  Pooled contexts live until the process exits; one returned holding more device
 * memory than sz4_set_pool_cap is trimmed first. */
int sz4_acquire(sz4_ctx** ctx, int device);
void sz4_release(sz4_ctx* ctx);

/* Worst-case frame size for n input bytes cut into blocks of block_size. */
uint64_t sz4_bound(uint64_t n, uint32_t block_size);

/* Compress n bytes already resident in device memory as independent blocks of
 * block_size bytes (last block shorter).  Each block's bytes in the output
 * (4-byte size word + payload) are exactly what smallz4::lz4 emits for that
 * block compressed on its own (reference smallz4.h:476-813 with one block).
 * Any n in bounded memory: the blocks are compressed in pieces of at most
 * sz4_set_batch_chunk bytes (by default 448 MiB, split into equal pieces, and capped so that the scratch -- under 50 bytes
 * per piece byte -- takes at most a quarter of the device memory the context could use now;
 * under a sz4_set_device_limit bound about 1/64 of the bound).  A piece whose scratch cannot
 * be allocated is halved and retried, down to 16 MiB, before SZ4_E_NOMEM.
 *
 *   d_in, d_out   device pointers (d_out capacity out_cap bytes)
 *   block_size    1 .. 4 MiB
 *   max_chain     reference maxChainLength (0..65535)
 *   header        SZ4_HEADER_*
 *   out_size      host pointer, receives the frame size
 *   stream        hipStream_t (NULL = default stream); the call returns after
 *                 the stream has finished (out_size needs the result)
 */
int sz4_compress_blocks_device(sz4_ctx* ctx, const void* d_in, uint64_t n, uint32_t block_size,
                               uint32_t max_chain, int header, void* d_out, uint64_t out_cap,
                               uint64_t* out_size, void* stream);

/* Per-block result sizes of the last sz4_compress_blocks_device call
 * (4-byte word included), copied to host array sizes[0..nblocks).  Returns the
 * number of blocks, or a negative status. */
int64_t sz4_last_block_sizes(sz4_ctx* ctx, uint32_t* sizes, uint64_t max_blocks);

/* Whole-stream compression with the exact semantics of
 * smallz4::lz4(getBytes, sendBytes, maxChainLength, dictionary, useLegacyFormat)
 * (reference smallz4.h:47-64): 4 MiB dependent blocks (8 MiB independent
 * blocks in legacy format), optional dictionary, identical output bytes.
 * Host buffers; the device does all compression work, chunk by chunk as in
 * sz4_lz4_stream (fixed device footprint). */
int sz4_lz4(sz4_ctx* ctx, const void* in, uint64_t n, uint32_t max_chain, const void* dict,
            uint64_t dict_len, int legacy, void* out, uint64_t out_cap, uint64_t* out_size);

/* Worst-case size of sz4_lz4's output. */
uint64_t sz4_lz4_bound(uint64_t n, int legacy);

/* The reference's callback types (smallz4.h:41-44): read up to numBytes into data (0 = end of
 * input); write numBytes from data. */
typedef size_t (*sz4_get_bytes)(void* data, size_t numBytes, void* userPtr);
typedef void (*sz4_send_bytes)(const void* data, size_t numBytes, void* userPtr);

/* smallz4::lz4(getBytes, sendBytes, maxChainLength, dictionary, useLegacyFormat, userPtr)
 * (reference smallz4.h:47-64, 476-813) in bounded memory: the input is pulled through get_bytes
 * (64 KiB per call, as the reference's BufferSize) and compressed in chunks of whole 4 MiB blocks
 * (8 MiB legacy) -- sz4_set_stream_chunk bytes per chunk, 64 MiB by default -- each chunk carrying
 * the previous one's last 64 KiB and chain state, so the output is byte-identical to one pass over
 * the whole input and the device footprint does not grow with the input.  send_bytes receives the
 * header, then per block four 1-byte calls for the size word followed by the payload, then the end
 * mark: the reference's call pattern (smallz4.h:478-496, 770-780, 807-812).  Both callbacks run on
 * the calling thread; the GPU compresses chunk i+1 while chunk i is sent and chunk i+2 is read and
 * uploaded (three HIP streams).  Pinned host buffers grow with the input up to one chunk.
 * A context serves one call at a time (use one context per thread). */
int sz4_lz4_stream(sz4_ctx* ctx, sz4_get_bytes get_bytes, sz4_send_bytes send_bytes, uint32_t max_chain,
                   const void* dict, uint64_t dict_len, int legacy, void* user);

/* Input bytes per chunk of the stream paths (sz4_lz4_stream, sz4_lz4; sz4_unlz4_stream queues half
 * as many frame bytes); rounded down to whole blocks, at least one.  0 restores the 64 MiB default. */
void sz4_set_stream_chunk(sz4_ctx* ctx, uint64_t bytes);

/* Input bytes per internal piece of sz4_compress_blocks_device (whole blocks, at least one); the
 * device scratch is about 36-50 bytes per piece byte.  An explicit size is not capped by free memory.
 * 0 restores the default (448 MiB, capped by free memory). */
void sz4_set_batch_chunk(sz4_ctx* ctx, uint64_t bytes);

/* Device time (milliseconds) of each pipeline stage of the last call, measured
 * with HIP events on the call's stream.  stage_ms[0..n) receives
 * {runs, sort, find_sorted, find_long, parse, assemble} (find_sorted is the
 * k_find_sorted kernel alone); returns the number of stages. */
int sz4_last_stage_ms(sz4_ctx* ctx, float* stage_ms, int n);

/* Enable (1) or disable (0) per-stage event timing (default off). */
void sz4_set_timing(sz4_ctx* ctx, int on);

/* Diagnostics: stop the pipeline after stage `stop_after` (0 = run everything,
 * 3 = after the match search, 4 = after the parse) on subsequent calls, and copy
 * the per-position match arrays of the last call (length u32, distance u16, one
 * entry per input byte) to host memory.  After stage 4 at levels > 3 the lengths
 * are the parse's choices (1 = literal).  Used by the intermediate parity tests. */
void sz4_debug_stop_after(sz4_ctx* ctx, int stop_after);
int sz4_debug_matches(sz4_ctx* ctx, uint32_t* len, uint16_t* dist, uint64_t n);

/* ---- decoder: the reference's smallz4cat ------------------------------------------------------
 * Decompress an LZ4 frame with the semantics of the reference decoder
 *   unlz4_userPtr(GET_BYTE, SEND_BYTES, dictionary, userPtr)      smallz4cat.c:112-360
 * over memory: modern and legacy frames, stored blocks, skipped block / content checksums,
 * content size and dictionary ID, an optional dictionary (its last 64 KiB precede the output),
 * a legacy frame ending after its first block shorter than 8 MiB.  Every byte is decoded on the
 * GPU (one wavefront per block).
 *   out_size  receives the decoded size, also when out_cap is too small (SZ4_E_CAPACITY):
 *             call with out = NULL, out_cap = 0 to query it
 * Returns SZ4_E_CORRUPT for a frame the reference decoder rejects (signature, version, truncated
 * frame, offset 0) or would misread (a length, literal run or offset crossing its block). */
int sz4_unlz4(sz4_ctx* ctx, const void* frame, uint64_t frame_len, const void* dict, uint64_t dict_len,
              void* out, uint64_t out_cap, uint64_t* out_size);

/* The same on device memory (frame, dictionary and output are device pointers) and a HIP stream;
 * returns after the stream has finished. */
int sz4_unlz4_device(sz4_ctx* ctx, const void* d_frame, uint64_t frame_len, const void* d_dict,
                     uint64_t dict_len, void* d_out, uint64_t out_cap, uint64_t* out_size, void* stream);

/* The reference decoder's callback types (smallz4cat.c:62-65). */
typedef unsigned char (*sz4_get_byte)(void* userPtr);
typedef void (*sz4_send_out)(const unsigned char* data, unsigned int numBytes, void* userPtr);

/* unlz4_userPtr(getByte, sendBytes, dictionary, userPtr) (smallz4cat.c:112-360) in bounded memory:
 * get_byte is called where the reference calls it on a valid frame (header, size words, payloads,
 * checksums; a legacy frame ends after its first block that decodes to less than 8 MiB); blocks are
 * decoded on the GPU a chunk at a time with the last 64 KiB of output as history, and send_bytes
 * receives the output in 64 KiB pieces followed by the remainder (the reference's flush points).
 * dict: the dictionary's bytes (its last 64 KiB are used) or NULL. */
int sz4_unlz4_stream(sz4_ctx* ctx, sz4_get_byte get_byte, sz4_send_out send_bytes, const void* dict, uint64_t dict_len,
                     void* user);

/* Device memory (bytes) the context holds: its scratch, staging and output buffers.  Buffers grow on
 * demand and are kept for the next call of the same kind. */
uint64_t sz4_device_bytes(sz4_ctx* ctx);

/* Release every device buffer and pinned host buffer the context holds (after its last call has
 * finished); the next call allocates again.  The context stays valid. */
void sz4_trim(sz4_ctx* ctx);

/* Bound the context's device memory to `bytes` (0 = no bound, the default).  A call that would grow
 * past it first releases the buffers it does not use itself -- those kept from calls of another kind:
 * the stream path's staging, dictionary tables, the decoder's output image -- and fails with
 * SZ4_E_NOMEM if that is not enough (the decoder then takes its block-by-block mode, which needs about
 * half the memory of its split mode, before it gives up).  The same release happens, bound or not, when
 * the device itself runs out of memory. */
void sz4_set_device_limit(sz4_ctx* ctx, uint64_t bytes);

/* Buffers the context has released under a device bound or device memory pressure (diagnostics). */
uint64_t sz4_released_buffers(sz4_ctx* ctx);

/* Pooled contexts (sz4_acquire) that hold more than `bytes` of device memory when they are released
 * are trimmed (sz4_trim) before they go back to the pool.  0 restores the default, 8 GiB. */
void sz4_set_pool_cap(uint64_t bytes);

/* Dictionary mode: the most match-finder rounds any chunk of the last stream call took (the
 * data-parallel finder assumes the same-letter shortcut intervals and reruns a chunk whose results imply
 * others; 1 = none to correct, 0 = no dictionary chunk, UINT32_MAX = a chunk fell back to the in-order
 * replay: after (largest block / 65 300) + 3 rounds -- one more interval settles per round --, or
 * SZ4_DICT_MAX_ROUNDS in the environment when the context was created). */
uint32_t sz4_dict_rounds(sz4_ctx* ctx);

/* Decoder diagnostics: the longest reference chain (hops to earlier sub-segments) the last split-mode decode
 * followed while packing its output (frames with blocks of >= 256 KiB payload), 0 when it decoded block by
 * block or no byte referred to another sub-segment. */
uint32_t sz4_unlz4_resolve_passes(sz4_ctx* ctx);
/* 1 when the last decode's block index came from the parallel index, 0 when the serial size-word walk
 * decided (a malformed frame, too many candidates, or SZ4_UNLZ4_INDEX=0). */
int sz4_unlz4_index_parallel(sz4_ctx* ctx);

/* Last error message of the context ("" if none). */
const char* sz4_last_error(sz4_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* SMALLZ4_AMD_H */
