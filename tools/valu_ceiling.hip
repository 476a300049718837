// valu_ceiling.hip -- measures the VALU issue rate the MI355X sustains on integer work, the ceiling the
// finder and parse kernels are priced against in DESIGN.md (they are integer/byte kernels: no MFMA).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/valu_ceiling tools/valu_ceiling.hip
//   tools/bin/valu_ceiling            (prints one JSON line per variant)
//
// Every wave runs `iters` rounds of 16 v_add_u32 / v_xor_b32 in inline asm: 4 independent chains of 4
// (so one wave alone is not latency-bound), optionally with a DPP row shift or a v_readlane in every
// round.  Grid: 256 CUs x `waves` waves of 64 lanes.  Rate = VALU instructions issued (64-lane waves)
// per second, per SIMD per clock at the measured effective clock is left to the reader (rocprofv3
// GRBM_GUI_ACTIVE); the number compared with a kernel is instructions per second, both from the same
// counters (SQ_INSTS_VALU / kernel time).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

template <int kMode>
__global__ __launch_bounds__(256) void k_valu(unsigned* out, int iters)
{
  unsigned a = threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u;
  for (int i = 0; i < iters; i++) {
    asm volatile(
        "v_add_u32 %0, %0, %1\n\t"
        "v_add_u32 %1, %1, %2\n\t"
        "v_add_u32 %2, %2, %3\n\t"
        "v_add_u32 %3, %3, %0\n\t"
        "v_xor_b32 %0, %0, %2\n\t"
        "v_xor_b32 %1, %1, %3\n\t"
        "v_xor_b32 %2, %2, %0\n\t"
        "v_xor_b32 %3, %3, %1\n\t"
        "v_add_u32 %0, %0, %1\n\t"
        "v_add_u32 %1, %1, %2\n\t"
        "v_add_u32 %2, %2, %3\n\t"
        "v_add_u32 %3, %3, %0\n\t"
        "v_xor_b32 %0, %0, %2\n\t"
        "v_xor_b32 %1, %1, %3\n\t"
        "v_xor_b32 %2, %2, %0\n\t"
        "v_xor_b32 %3, %3, %1\n\t"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    if constexpr (kMode == 1) {
      // one DPP row shift per round (the parse's window shift)
      a = (unsigned)__builtin_amdgcn_update_dpp((int)b, (int)a, 0x111, 0xF, 0xF, false);
    } else if constexpr (kMode == 2) {
      // one readlane into the scalar unit and back per round (the walks' pattern)
      b += (unsigned)__builtin_amdgcn_readlane((int)c, i & 63);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}

template <int kMode>
static void run(const char* name, int wavesPerCu, int iters, unsigned* out)
{
  const int cus = 256, wavesPerWg = 4;
  const int grid = cus * wavesPerCu / wavesPerWg;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_valu<kMode>, dim3(grid), dim3(64 * wavesPerWg), 0, 0, out, iters);  // warm-up
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_valu<kMode>, dim3(grid), dim3(64 * wavesPerWg), 0, 0, out, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double waves = (double)grid * wavesPerWg;
  const double perRound = 16.0 + (double)kMode;  // the loop counter lives in the scalar unit
  const double instr = waves * iters * perRound;
  std::printf("{\"variant\": \"%s\", \"waves_per_cu\": %d, \"ms\": %.3f, \"valu_instr_per_s\": %.4g, "
              "\"per_simd_per_ns\": %.4f}\n",
              name, wavesPerCu, ms, instr / (ms * 1e-3), instr / (ms * 1e-3) / 1024.0 / 1e9);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main()
{
  unsigned* out = nullptr;
  CHECK(hipMalloc(&out, 256 * 32 * 64 * sizeof(unsigned)));
  const int iters = 20000;
  for (int w : {8, 16, 32}) run<0>("add_xor", w, iters, out);
  run<1>("add_xor+dpp", 32, iters, out);
  run<2>("add_xor+readlane", 32, iters, out);
  CHECK(hipFree(out));
  return 0;
}
