#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstring>
#include "../../root/repo/include/smallz4_amd.h"
#include "../../root/repo/smallz4_amd/csrc/sz4_internal.h"
using namespace sz4;
int main() {
  sz4_ctx* c; sz4_create(&c, 0, 0);
  const size_t n = 100000000;
  std::vector<uint8_t> in(n);
  uint32_t x = 1;
  for (size_t i = 0; i < n; i++) { x = x * 1103515245u + 12345u; in[i] = (i % 1000 < 700) ? 'a' + ((x >> 16) % 6) : (uint8_t)(x >> 16); }
  uint8_t *din, *dout; hipMalloc(&din, n); hipMalloc(&dout, n * 2);
  hipMemcpy(din, in.data(), n, hipMemcpyHostToDevice);
  uint64_t size = 0;
  int r = sz4_compress_blocks_device(c, din, n, 65536, 65535, SZ4_HEADER_SMALLZ4, dout, n * 2, &size, nullptr);
  printf("compress %d size %llu\n", r, (unsigned long long)size);
  uint64_t sb = unlz4_ix_scratch_bytes(size);
  void* scr; hipMalloc(&scr, sb); hipMemset(scr, 0, sb);
  UnBlock* blk; hipMalloc(&blk, 65536 * sizeof(UnBlock));
  uint64_t* meta; hipMalloc(&meta, 64);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 4; rep++) {
    hipEventRecord(e0);
    launch_unlz4_index_par(dout, size, scr, blk, 65536, meta, nullptr);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); printf("par %.3f ms\n", ms);
  }
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0);
    launch_unlz4_index(dout, size, blk, 65536, meta, nullptr);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); printf("serial %.3f ms\n", ms);
  }
  launch_unlz4_index_par(dout, size, scr, blk, 65536, meta, nullptr);
  hipDeviceSynchronize();
  uint64_t hm[4]; hipMemcpy(hm, meta, 32, hipMemcpyDeviceToHost);
  printf("meta nb %llu st %llu legacy %llu par %llu err %s\n", (unsigned long long)hm[0], (unsigned long long)hm[1], (unsigned long long)hm[2], (unsigned long long)hm[3], hipGetErrorString(hipGetLastError()));
  // scratch layout: bits, wordPre, wgCount, wgOff, list, link, chain (256-aligned)
  const uint64_t words = size / 32 + 2, nWg = (words + 255) / 256, cap = unlz4_ix_cap(size);
  auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
  uint64_t off[7], t = 0; uint64_t bytes[7] = {4 * words, 4 * words, 4 * (nWg + 1), 4 * (nWg + 1), 8 * cap, 4 * cap, 4 * cap};
  for (int k = 0; k < 7; k++) { off[k] = t; t += al(bytes[k]); }
  // the true chain (serial) and its bits
  launch_unlz4_index(dout, size, blk, 65536, meta, nullptr);
  hipDeviceSynchronize();
  std::vector<UnBlock> hb(1526); hipMemcpy(hb.data(), blk, 1526 * sizeof(UnBlock), hipMemcpyDeviceToHost);
  std::vector<uint32_t> bits2(words); hipMemcpy(bits2.data(), (uint8_t*)scr + off[0], 4 * words, hipMemcpyDeviceToHost);
  int miss = 0;
  for (int b = 0; b < 1526; b++) {
    const uint64_t r = hb[b].src - 4, rel = r - 4;
    const bool bit = (bits2[rel >> 5] >> (rel & 31)) & 1u;
    if (!bit && miss < 6) printf("missing block %d at %llu\n", b, (unsigned long long)r);
    miss += !bit;
  }
  printf("missing %d of 1526\n", miss);
  std::vector<uint32_t> wgOff(nWg + 1), bits(words);
  hipMemcpy(wgOff.data(), (uint8_t*)scr + off[3], 4 * (nWg + 1), hipMemcpyDeviceToHost);
  hipMemcpy(bits.data(), (uint8_t*)scr + off[0], 4 * words, hipMemcpyDeviceToHost);
  uint64_t M = wgOff[nWg];
  printf("words %llu nWg %llu M %llu bits0 %08x\n", (unsigned long long)words, (unsigned long long)nWg, (unsigned long long)M, bits[0]);
  std::vector<uint64_t> list(M); std::vector<uint32_t> link(M);
  hipMemcpy(list.data(), (uint8_t*)scr + off[4], 8 * M, hipMemcpyDeviceToHost);
  hipMemcpy(link.data(), (uint8_t*)scr + off[5], 4 * M, hipMemcpyDeviceToHost);
  for (uint64_t i = 0; i < M && i < 12; i++) printf("cand %llu pos %llu link %08x\n", (unsigned long long)i, (unsigned long long)list[i], link[i]);
  return 0;
}
