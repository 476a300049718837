// smallz4_amd.hpp -- drop-in for the reference's C++ interface (smallz4.h:38-80), backed by the
// MI355X library declared in smallz4_amd.h.
//
// A program written against the reference
//     #include "smallz4.h"
//     smallz4::lz4(getBytes, sendBytes, maxChainLength, dictionary, useLegacyFormat, userPtr);
// switches by including this header instead and linking libsmallz4_amd.so.  The class name,
// the callback typedefs, the overloads, getVersion() and the level thresholds are the
// reference's; the emitted byte stream is identical.  The callbacks are driven the way the
// reference drives them: getBytes is asked for 64 KiB at a time until it returns 0, and
// sendBytes receives the header, then per block four 1-byte calls for the size word followed
// by the payload, then the 4-byte end mark (smallz4.h:478-496, 770-780, 809-813).
//
// Memory is bounded as in the reference: the input is compressed in chunks of whole 4 MiB blocks
// (sz4_lz4_stream), so any input length runs in a fixed device and host footprint.  Calls are
// reentrant: each call borrows its own context from the library's pool (sz4_acquire), as the
// reference builds a fresh object per call (smallz4.h:56-64).
//
// Differences: errors from the device are reported as std::runtime_error (the reference has no
// error path); SMALLZ4_AMD_DEVICE=<n> selects the GPU (default 0).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "smallz4_amd.h"

class smallz4
{
public:
  // read  several bytes, see getBytesFromIn() in the reference's smallz4.cpp
  typedef size_t (*GET_BYTES)(void* data, size_t numBytes, void* userPtr);
  // write several bytes, see sendBytesToOut() in the reference's smallz4.cpp
  typedef void (*SEND_BYTES)(const void* data, size_t numBytes, void* userPtr);

  enum
  {
    /// greedy mode for short chains (compression level <= 3)
    ShortChainsGreedy = 3,
    /// lazy evaluation for medium-sized chains (compression level > 3 and <= 6)
    ShortChainsLazy = 6
  };

  /// compress everything in input stream (accessed via getBytes) and write to output stream (via sendBytes)
  static void lz4(GET_BYTES getBytes, SEND_BYTES sendBytes, unsigned short maxChainLength = 65535,
                  bool useLegacyFormat = false, void* userPtr = NULL)
  {
    lz4(getBytes, sendBytes, maxChainLength, std::vector<unsigned char>(), useLegacyFormat, userPtr);
  }

  /// same, with a predefined dictionary
  static void lz4(GET_BYTES getBytes, SEND_BYTES sendBytes, unsigned short maxChainLength,
                  const std::vector<unsigned char>& dictionary, bool useLegacyFormat = false, void* userPtr = NULL)
  {
    Lease ctx;
    const int rc = sz4_lz4_stream(ctx.c, getBytes, sendBytes, maxChainLength,
                                  dictionary.empty() ? NULL : dictionary.data(), dictionary.size(),
                                  useLegacyFormat ? 1 : 0, userPtr);
    if (rc != SZ4_OK) throw std::runtime_error(std::string("smallz4_amd: ") + sz4_last_error(ctx.c));
  }

  /// version string (smallz4.h:67-70)
  static const char* getVersion() { return sz4_version(); }

private:
  // a context of the library's pool for the duration of one call
  struct Lease
  {
    sz4_ctx* c;
    Lease() : c(NULL)
    {
      const char* dev = std::getenv("SMALLZ4_AMD_DEVICE");
      if (sz4_acquire(&c, dev ? std::atoi(dev) : 0) != SZ4_OK) throw std::runtime_error("smallz4_amd: no usable HIP device");
    }
    ~Lease() { sz4_release(c); }
    Lease(const Lease&);
    Lease& operator=(const Lease&);
  };
};
