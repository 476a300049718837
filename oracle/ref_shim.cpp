// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// In-memory harness around the *unmodified* reference compressor
// (/root/reference/smallz4.h, included where it lies; nothing is copied).
// Built by oracle/Makefile into oracle/_ref/libsmallz4_ref.so and used to
// pin the C restatement (oracle/smallz4_oracle.c), to generate the golden
// vectors in tests/golden/, and as bench.py's cpu_baseline ("reference").
#include "smallz4.h"

#include <cstring>
#include <vector>

namespace {
struct MemIO {
  const unsigned char* in;
  size_t inLen, inPos;
  unsigned char* out;
  size_t cap, outPos;
  bool overflow;
};

// GET_BYTES (smallz4.h:42): full reads until the input is exhausted, like fread on a file.
size_t memGet(void* data, size_t numBytes, void* user)
{
  MemIO* io = static_cast<MemIO*>(user);
  size_t left = io->inLen - io->inPos;
  size_t k = numBytes < left ? numBytes : left;
  if (k) std::memcpy(data, io->in + io->inPos, k);
  io->inPos += k;
  return k;
}

// SEND_BYTES (smallz4.h:44)
void memSend(const void* data, size_t numBytes, void* user)
{
  MemIO* io = static_cast<MemIO*>(user);
  if (io->outPos + numBytes > io->cap) { io->overflow = true; return; }
  std::memcpy(io->out + io->outPos, data, numBytes);
  io->outPos += numBytes;
}
}  // namespace

extern "C" unsigned long long ref_lz4(const unsigned char* in, unsigned long long n, unsigned maxChain,
                                      const unsigned char* dict, unsigned long long dictLen, int legacy,
                                      unsigned char* out, unsigned long long cap)
{
  MemIO io{in, (size_t)n, 0, out, (size_t)cap, 0, false};
  std::vector<unsigned char> d;
  if (dict && dictLen) d.assign(dict, dict + dictLen);
  smallz4::lz4(memGet, memSend, (unsigned short)maxChain, d, legacy != 0, &io);
  return io.overflow ? 0ull : (unsigned long long)io.outPos;
}
