/* smallz4cat_amd.h -- drop-in for the reference decoder's interface (smallz4cat.c:62-65, 112-366),
 * decoding on the MI355X through the C ABI of smallz4_amd.h:
 *
 *   typedef unsigned char (*GET_BYTE)  (void* userPtr);
 *   typedef void          (*SEND_BYTES)(const unsigned char*, unsigned int, void* userPtr);
 *   void unlz4_userPtr(GET_BYTE, SEND_BYTES, const char* dictionary, void* userPtr);
 *   void unlz4        (GET_BYTE, SEND_BYTES, const char* dictionary);
 *
 * A program that carries smallz4cat.c's decoder includes this header instead and links
 * libsmallz4_amd.so.  getByte is called as often as the reference calls it on a valid frame: the
 * header, every size word, payload and checksum; in a legacy frame the decoded length of each
 * block (summed from its token headers, on the host) decides whether another size word is read
 * (smallz4cat.c:325-327).  The GPU then decodes the frame (sz4_unlz4) and sendBytes receives the
 * output in 64 KiB pieces followed by the remainder, the reference's flush pattern
 * (smallz4cat.c:249-253, 358-359).  Errors print "ERROR: <message>" and exit(1), as unlz4error
 * does (smallz4cat.c:49-56).  SMALLZ4_AMD_DEVICE=<n> selects the GPU.
 */
#ifndef SMALLZ4CAT_AMD_H
#define SMALLZ4CAT_AMD_H

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "smallz4_amd.h"

typedef unsigned char (*GET_BYTE)(void* userPtr);
typedef void (*SEND_BYTES)(const unsigned char*, unsigned int, void* userPtr);

static inline void sz4cat_error(const char* msg)
{
  fputs("ERROR: ", stderr);
  fputs(msg, stderr);
  fputc('\n', stderr);
  exit(1);
}

typedef struct {
  unsigned char* p;
  uint64_t n, cap;
} sz4cat_buf;

static inline unsigned char sz4cat_pull(sz4cat_buf* b, GET_BYTE getByte, void* userPtr)
{
  unsigned char c = getByte(userPtr);
  if (b->n == b->cap) {
    uint64_t cap = b->cap ? 2 * b->cap : (uint64_t)1 << 16;
    unsigned char* p = (unsigned char*)realloc(b->p, (size_t)cap);
    if (!p) sz4cat_error("out of memory");
    b->p = p;
    b->cap = cap;
  }
  b->p[b->n++] = c;
  return c;
}

/* decoded length of one compressed block, from its token headers only */
static inline uint64_t sz4cat_block_length(const unsigned char* p, uint64_t len)
{
  uint64_t r = 0, w = 0;
  while (r < len) {
    unsigned char tok = p[r++], x;
    uint64_t lits = tok >> 4, ml = 4 + (tok & 15);
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

static inline void unlz4_userPtr(GET_BYTE getByte, SEND_BYTES sendBytes, const char* dictionary, void* userPtr)
{
  static sz4_ctx* ctx = NULL;
  static unsigned char none[1];
  static unsigned char dict[65536];
  sz4cat_buf f = {NULL, 0, 0};
  uint64_t dictLen = 0, size = 0, k;
  uint32_t sig = 0;
  int modern, legacy, blockSum = 0, contentSum = 0, rc;
  unsigned char* out = NULL;

  /* signature and frame descriptor (smallz4cat.c:114-159) */
  for (k = 0; k < 4; k++) sig |= (uint32_t)sz4cat_pull(&f, getByte, userPtr) << (8 * k);
  modern = sig == 0x184D2204u;
  legacy = sig == 0x184C2102u;
  if (!modern && !legacy) sz4cat_error("invalid signature");
  if (modern) {
    unsigned char flags = sz4cat_pull(&f, getByte, userPtr);
    int skip = 1 + ((flags & 8) ? 8 : 0) + ((flags & 1) ? 4 : 0) + 1;
    blockSum = (flags & 16) != 0;
    contentSum = (flags & 4) != 0;
    if ((flags >> 6) != 1) sz4cat_error("only LZ4 file format version 1 supported");
    while (skip--) sz4cat_pull(&f, getByte, userPtr);
  }
  /* the dictionary's last 64 KiB (smallz4cat.c:168-187) */
  if (dictionary != NULL) {
    FILE* d = fopen(dictionary, "rb");
    long n, from;
    if (!d) sz4cat_error("cannot open dictionary");
    fseek(d, 0, SEEK_END);
    n = ftell(d);
    from = n < 65536 ? 0 : n - 65536;
    fseek(d, from, SEEK_SET);
    dictLen = (uint64_t)fread(dict, 1, (size_t)(n - from), d);
    fclose(d);
  }
  /* blocks until the end mark (smallz4cat.c:189-350) */
  for (;;) {
    uint32_t word = 0;
    uint64_t at;
    int packed;
    for (k = 0; k < 4; k++) word |= (uint32_t)sz4cat_pull(&f, getByte, userPtr) << (8 * k);
    packed = legacy || (word & 0x80000000u) == 0;
    if (modern) word &= 0x7FFFFFFFu;
    if (word == 0) break;
    at = f.n;
    for (k = 0; k < word; k++) sz4cat_pull(&f, getByte, userPtr);
    if (legacy && packed && sz4cat_block_length(f.p + at, word) < 8u * 1024 * 1024) break;
    if (blockSum) for (k = 0; k < 4; k++) sz4cat_pull(&f, getByte, userPtr);
  }
  if (contentSum) for (k = 0; k < 4; k++) sz4cat_pull(&f, getByte, userPtr);

  if (!ctx) {
    const char* dev = getenv("SMALLZ4_AMD_DEVICE");
    if (sz4_create(&ctx, dev ? atoi(dev) : 0, 0) != SZ4_OK) sz4cat_error("no usable HIP device");
  }
  rc = sz4_unlz4(ctx, f.p, f.n, dictLen ? dict : NULL, dictLen, NULL, 0, &size);
  if (rc == SZ4_E_CAPACITY) {
    out = (unsigned char*)malloc((size_t)size);
    if (!out) sz4cat_error("out of memory");
    rc = sz4_unlz4(ctx, f.p, f.n, dictLen ? dict : NULL, dictLen, out, size, &size);
  }
  if (rc != SZ4_OK) sz4cat_error(sz4_last_error(ctx));
  for (k = 0; k + 65536 <= size; k += 65536) sendBytes(out + k, 65536, userPtr);
  sendBytes(out ? out + k : none, (unsigned int)(size - k), userPtr);
  free(out);
  free(f.p);
}

static inline void unlz4(GET_BYTE getByte, SEND_BYTES sendBytes, const char* dictionary)
{
  unlz4_userPtr(getByte, sendBytes, dictionary, NULL);
}

#endif /* SMALLZ4CAT_AMD_H */
