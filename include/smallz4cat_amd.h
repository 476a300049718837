/* smallz4cat_amd.h -- drop-in for the reference decoder's interface (smallz4cat.c:62-65, 112-366),
 * decoding on the MI355X through the C ABI of smallz4_amd.h (sz4_unlz4_stream):
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
 * (smallz4cat.c:325-327).  Blocks are decoded on the GPU a chunk at a time, each chunk with the
 * previous 64 KiB of output as its history, so memory stays bounded on any frame length; sendBytes
 * receives the output in 64 KiB pieces followed by the remainder, the reference's flush pattern
 * (smallz4cat.c:249-253, 358-359).  Errors print "ERROR: <message>" and exit(1), as unlz4error
 * does (smallz4cat.c:49-56).  Calls are reentrant (each borrows a context from the library's pool).
 * SMALLZ4_AMD_DEVICE=<n> selects the GPU.
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

static inline void unlz4_userPtr(GET_BYTE getByte, SEND_BYTES sendBytes, const char* dictionary, void* userPtr)
{
  unsigned char* dict = NULL;  /* per call: reentrant */
  uint64_t dictLen = 0;
  sz4_ctx* ctx = NULL;
  const char* dev = getenv("SMALLZ4_AMD_DEVICE");
  int rc;
  /* the dictionary's last 64 KiB (smallz4cat.c:168-187) */
  if (dictionary != NULL) {
    FILE* d = fopen(dictionary, "rb");
    long n, from;
    if (!d) sz4cat_error("cannot open dictionary");
    fseek(d, 0, SEEK_END);
    n = ftell(d);
    from = n < 65536 ? 0 : n - 65536;
    fseek(d, from, SEEK_SET);
    dict = (unsigned char*)malloc(65536);
    if (!dict) sz4cat_error("out of memory");
    dictLen = (uint64_t)fread(dict, 1, (size_t)(n - from), d);
    fclose(d);
  }
  /* a context of the library's pool: concurrent calls from several threads do not share one */
  if (sz4_acquire(&ctx, dev ? atoi(dev) : 0) != SZ4_OK) sz4cat_error("no usable HIP device");
  rc = sz4_unlz4_stream(ctx, getByte, sendBytes, dictLen ? dict : NULL, dictLen, userPtr);
  if (rc != SZ4_OK) sz4cat_error(sz4_last_error(ctx));
  sz4_release(ctx);
  free(dict);
}

static inline void unlz4(GET_BYTE getByte, SEND_BYTES sendBytes, const char* dictionary)
{
  unlz4_userPtr(getByte, sendBytes, dictionary, NULL);
}

#endif /* SMALLZ4CAT_AMD_H */
