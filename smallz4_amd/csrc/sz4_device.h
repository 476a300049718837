// sz4_device.h -- small device helpers shared by the gfx950 kernel files.  Not part of the public ABI.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "sz4_internal.h"

namespace sz4 {

// getHash32 (smallz4.h:163-168)
__device__ __forceinline__ uint32_t ref_hash(uint32_t four)
{
  return ((four * kHashMul) >> (32 - kHashBits)) & ((1u << kHashBits) - 1);
}

// four bytes at any offset of a buffer whose allocation is padded by >= 8 bytes and 4-aligned
__device__ __forceinline__ uint32_t gload4(const uint8_t* base, uint64_t off)
{
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (off & ~3ull));
  const uint32_t lo = w[0], hi = w[1];
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// value of a lane chosen by a wave-uniform index (v_readlane: no LDS round trip)
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane)
{
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

}  // namespace sz4
