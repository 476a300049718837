// valu_ceiling.hip -- the integer VALU issue rate the MI355X sustains, measured at the clock it holds
// while doing it: the ceiling the finder and parse kernels are priced against in DESIGN.md (they are
// integer/byte kernels: no MFMA).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/valu_ceiling tools/valu_ceiling.hip
//   tools/bin/valu_ceiling            (prints one JSON line per variant)
//
// Every wave runs `iters` rounds of 16 v_add_u32 / v_xor_b32 in inline asm over kChains independent
// register chains (an instruction reads the result written kChains instructions before it, so with 8 or
// 16 chains one wave alone is not latency-bound), their second operand an SGPR or (mode 3) a VGPR,
// optionally with a DPP row shift or a v_readlane per round.  Grid: 256 CUs x `waves` waves of 64
// lanes, launched back to back for >= 2 s before the timed
// launch so that the clock has settled (MI355X_MICROARCH.md, DVFS give-back).
//
// The clock: lane 0 of every wave stamps s_memtime (shader clock) and s_memrealtime (100 MHz) around its
// loop; clock = median over waves of d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS
// item 6).  Reported: VALU wave-instructions per second, per SIMD per ns, and per SIMD per cycle at that
// clock (nominal: 0.5 -- a wave64 VALU instruction takes 2 cycles on a SIMD-32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

// 16 instructions over 4 chains: chain i's instruction k reads chain (i+1)'s value too (the round-4 loop)
#define SZ4_ROUND4(a, b, c, d)                                                                       \
  asm volatile("v_add_u32 %0, %0, %1\n\tv_add_u32 %1, %1, %2\n\tv_add_u32 %2, %2, %3\n\t"            \
               "v_add_u32 %3, %3, %0\n\tv_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %3\n\t"            \
               "v_xor_b32 %2, %2, %0\n\tv_xor_b32 %3, %3, %1\n\tv_add_u32 %0, %0, %1\n\t"            \
               "v_add_u32 %1, %1, %2\n\tv_add_u32 %2, %2, %3\n\tv_add_u32 %3, %3, %0\n\t"            \
               "v_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %3\n\tv_xor_b32 %2, %2, %0\n\t"            \
               "v_xor_b32 %3, %3, %1"                                                                \
               : "+v"(a), "+v"(b), "+v"(c), "+v"(d))
// 8 instructions, one per chain x0..x7, each reading only its own chain and one operand `s` that is a
// scalar register ("s") or a vector register ("v"): the finders' broadcast tests read v_readlane results
// (SGPRs), the shift-register tests only VGPRs
#define SZ4_ROUND8(op, x, s, c)                                                                      \
  asm volatile(op " %0, %0, %8\n\t" op " %1, %1, %8\n\t" op " %2, %2, %8\n\t" op " %3, %3, %8\n\t"  \
                  op " %4, %4, %8\n\t" op " %5, %5, %8\n\t" op " %6, %6, %8\n\t" op " %7, %7, %8"    \
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),   \
                 "+v"(x[7])                                                                          \
               : c(s))

template <int kChains, int kMode>
__global__ __launch_bounds__(256) void k_valu(unsigned* out, unsigned long long* stamps, int iters, unsigned s)
{
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  unsigned x[16];
  const unsigned vs = s ^ threadIdx.x;  // a per-lane operand: kept in a VGPR
#pragma unroll
  for (int k = 0; k < 16; k++) x[k] = threadIdx.x * (2u * k + 1u);
  for (int i = 0; i < iters; i++) {
    if constexpr (kChains == 4) {
      SZ4_ROUND4(x[0], x[1], x[2], x[3]);
    } else if constexpr (kChains == 8 && kMode == 3) {
      SZ4_ROUND8("v_add_u32", x, vs, "v");
      SZ4_ROUND8("v_xor_b32", x, vs, "v");
    } else if constexpr (kChains == 8) {
      SZ4_ROUND8("v_add_u32", x, s, "s");
      SZ4_ROUND8("v_xor_b32", x, s, "s");
    } else {
      SZ4_ROUND8("v_add_u32", x, s, "s");
      SZ4_ROUND8("v_add_u32", (x + 8), s, "s");
    }
    if constexpr (kMode == 1) {
      // one DPP row shift per round (the parse's window shift)
      x[0] = (unsigned)__builtin_amdgcn_update_dpp((int)x[1], (int)x[0], 0x111, 0xF, 0xF, false);
    } else if constexpr (kMode == 2) {
      // one readlane into the scalar unit and back per round (the finders' broadcast)
      x[1] += (unsigned)__builtin_amdgcn_readlane((int)x[2], i & 63);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  unsigned v = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) v ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
  if ((threadIdx.x & 63) == 0) {
    const unsigned w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    stamps[2 * w] = t1 - t0;
    stamps[2 * w + 1] = r1 - r0;
  }
}

template <int kChains, int kMode>
static void run(const char* name, int wavesPerCu, int iters, unsigned* out, unsigned long long* stamps)
{
  const int cus = 256, wavesPerWg = 4;
  const int grid = cus * wavesPerCu / wavesPerWg;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // back-to-back launches for >= 2 s: the clock the chip holds under this load
  CHECK(hipEventRecord(e0));
  int warm = 0;
  for (float el = 0; el < 2000.0f; warm++) {
    hipLaunchKernelGGL((k_valu<kChains, kMode>), dim3(grid), dim3(64 * wavesPerWg), 0, 0, out, stamps, iters, 0x9E3779B9u);
    if (warm % 8 == 7) {
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&el, e0, e1));
    }
  }
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((k_valu<kChains, kMode>), dim3(grid), dim3(64 * wavesPerWg), 0, 0, out, stamps, iters, 0x9E3779B9u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const int waves = grid * wavesPerWg;
  std::vector<unsigned long long> h(2 * (size_t)waves);
  CHECK(hipMemcpy(h.data(), stamps, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  std::vector<double> clk, loopNs;
  for (int w = 0; w < waves; w++) {
    if (h[2 * w + 1] == 0) continue;
    clk.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 0.1);  // GHz: memtime ticks per 10 ns
    loopNs.push_back((double)h[2 * w + 1] * 10.0);
  }
  std::sort(clk.begin(), clk.end());
  std::sort(loopNs.begin(), loopNs.end());
  const double ghz = clk[clk.size() / 2];
  const double perRound = 16.0 + (kMode == 1 || kMode == 2 ? 1.0 : 0.0);  // the loop counter lives in the scalar unit
  const double instr = (double)waves * iters * perRound;
  const double perSimdNs = instr / (ms * 1e-3) / 1024.0 / 1e9;
  // one wave's own issue rate: its instructions over its own loop time, in cycles at the clock
  const double perWaveCyc = (double)iters * perRound / (loopNs[loopNs.size() / 2] * ghz);
  std::printf("{\"variant\": \"%s\", \"chains\": %d, \"waves_per_cu\": %d, \"waves_per_simd\": %d, \"warm_launches\": %d, "
              "\"ms\": %.3f, \"clock_ghz_median\": %.3f, \"clock_ghz_min\": %.3f, \"clock_ghz_max\": %.3f, "
              "\"valu_instr_per_s\": %.4g, \"per_simd_per_ns\": %.4f, \"per_simd_per_cycle\": %.4f, "
              "\"per_simd_per_cycle_at_2p4\": %.4f, \"one_wave_per_cycle\": %.4f}\n",
              name, kChains, wavesPerCu, wavesPerCu / 4, warm, ms, ghz, clk.front(), clk.back(), instr / (ms * 1e-3),
              perSimdNs, perSimdNs / ghz, perSimdNs / 2.4, perWaveCyc);
  std::fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main()
{
  unsigned* out = nullptr;
  unsigned long long* stamps = nullptr;
  CHECK(hipMalloc(&out, 256 * 32 * 64 * sizeof(unsigned)));
  CHECK(hipMalloc(&stamps, 256 * 32 * 2 * sizeof(unsigned long long)));
  const int iters = 20000;
  run<4, 0>("add_xor_4chains_r04", 32, iters, out, stamps);
  for (int w : {4, 8, 16, 32}) run<8, 0>("add_xor_8chains", w, iters, out, stamps);
  run<16, 0>("add_16chains", 32, iters, out, stamps);
  run<8, 1>("add_xor_8chains+dpp", 32, iters, out, stamps);
  run<8, 2>("add_xor_8chains+readlane", 32, iters, out, stamps);
  for (int w : {8, 32}) run<8, 3>("add_xor_8chains_vgpr_operand", w, iters, out, stamps);
  CHECK(hipFree(out));
  CHECK(hipFree(stamps));
  return 0;
}
