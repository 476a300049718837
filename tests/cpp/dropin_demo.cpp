// dropin_demo.cpp -- the reference's in-memory usage pattern (smallz4.cpp:50-117), compiled
// against include/smallz4_amd.hpp instead of the reference header.  Used by tests/test_abi.py
// (compiles) and tests/test_gpu.py (runs: stdin -> stdout).
//   usage: dropin_demo [level] [legacy] < input > output
#include <cstdio>
#include <cstdlib>

#include "smallz4_amd.hpp"

static size_t getBytesFromIn(void* data, size_t numBytes, void* userPtr)
{
  (void)userPtr;
  return fread(data, 1, numBytes, stdin);
}

static void sendBytesToOut(const void* data, size_t numBytes, void* userPtr)
{
  size_t* calls = static_cast<size_t*>(userPtr);
  ++*calls;
  if (numBytes) fwrite(data, 1, numBytes, stdout);
}

int main(int argc, char** argv)
{
  unsigned short level = argc > 1 ? (unsigned short)atoi(argv[1]) : 9;
  unsigned short chain = level >= 9 ? 65535 : level;
  bool legacy = argc > 2 && atoi(argv[2]) != 0;
  size_t calls = 0;
  smallz4::lz4(getBytesFromIn, sendBytesToOut, chain, legacy, &calls);
  fprintf(stderr, "smallz4_amd %s: %zu sendBytes calls\n", smallz4::getVersion(), calls);
  return 0;
}
