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
// Differences: compression happens on the GPU after the whole input has been read (the
// reference interleaves reading and compressing 4 MiB at a time); errors from the device are
// reported as std::runtime_error (the reference has no error path).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <cstring>
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
    std::vector<unsigned char> input;
    std::vector<unsigned char> chunk(64 * 1024);
    for (;;) {
      size_t got = getBytes(chunk.data(), chunk.size(), userPtr);
      if (got == 0) break;
      input.insert(input.end(), chunk.begin(), chunk.begin() + got);
    }
    std::vector<unsigned char> frame(sz4_lz4_bound(input.size(), useLegacyFormat ? 1 : 0));
    uint64_t size = 0;
    int rc = sz4_lz4(context(), input.data(), input.size(), maxChainLength, dictionary.empty() ? NULL : dictionary.data(),
                     dictionary.size(), useLegacyFormat ? 1 : 0, frame.data(), frame.size(), &size);
    if (rc != SZ4_OK) throw std::runtime_error(std::string("smallz4_amd: ") + sz4_last_error(context()));
    replay(frame.data(), size, useLegacyFormat, sendBytes, userPtr);
  }

  /// version string (smallz4.h:67-70)
  static const char* getVersion() { return sz4_version(); }

private:
  static sz4_ctx* context()
  {
    static sz4_ctx* ctx = NULL;
    if (!ctx) {
      const char* dev = std::getenv("SMALLZ4_AMD_DEVICE");
      if (sz4_create(&ctx, dev ? std::atoi(dev) : 0, 0) != SZ4_OK)
        throw std::runtime_error("smallz4_amd: no usable HIP device");
    }
    return ctx;
  }

  // hand the frame to sendBytes in the reference's call pattern
  static void replay(const unsigned char* f, uint64_t n, bool legacy, SEND_BYTES sendBytes, void* userPtr)
  {
    uint64_t hdr = legacy ? 4 : 7;
    sendBytes(f, hdr, userPtr);
    uint64_t pos = hdr;
    const uint64_t tail = legacy ? 0 : 4;
    while (pos + tail < n) {
      uint32_t word = 0;
      std::memcpy(&word, f + pos, 4);
      for (int k = 0; k < 4; k++) sendBytes(f + pos + k, 1, userPtr);
      pos += 4;
      const uint32_t bytes = word & 0x7FFFFFFFu;
      sendBytes(f + pos, bytes, userPtr);  // the reference sends the payload even when empty
      pos += bytes;
    }
    if (!legacy) sendBytes(f + pos, 4, userPtr);
  }
};
