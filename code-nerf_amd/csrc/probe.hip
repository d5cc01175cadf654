// Clock probe (measurement only; no reference counterpart).
//
// The MI355X lowers its shader clock under a dense bf16 MFMA load, by box and
// by data (MI355X_MICROARCH.md, "DVFS give-back"): the same binary measured
// 6.3 ms on one box and 6.8 ms on another (round 5).  bench.py runs this
// kernel before the warm-up and after the timed steps so a bench line records
// the clock its box held: every wave issues back-to-back
// v_mfma_f32_32x32x16_bf16 on hashed (non-zero, non-trivial) operands, and
// wave 0 of each workgroup stamps s_memtime (shader cycles) and s_memrealtime
// (100 MHz) around the loop.  clock = d(memtime) / d(memrealtime) x 100 MHz.
#pragma once
#include "cn_common.h"

namespace cn {

constexpr int kProbeWaves = 4;     // waves per workgroup

CN_DEV uint32_t probe_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// out[3 * blockIdx.x + {0, 1, 2}] = cycles, 100 MHz ticks, a checksum of the
// accumulators (keeps the MFMAs live)
__global__ __launch_bounds__(kProbeWaves * 64) void clock_probe_kernel(uint32_t* out, int iters, uint32_t seed) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    // random bf16 in [0.5, 1) x sign: exponent fixed, 7 random mantissa bits
    const uint32_t h = probe_hash(seed ^ (id * 8 + i));
    a[i] = __builtin_bit_cast(__bf16, (uint16_t)(0x3F00u | (h & 0x7Fu) | ((h >> 8) & 0x8000u)));
    b[i] = __builtin_bit_cast(__bf16, (uint16_t)(0x3F00u | ((h >> 16) & 0x7Fu) | ((h >> 24) & 0x80u) << 8));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c3, 0, 0, 0);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += c0[k] + c1[k] + c2[k] + c3[k];
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x + 0] = (uint32_t)(t1 - t0);
    out[3 * blockIdx.x + 1] = (uint32_t)(r1 - r0);
    out[3 * blockIdx.x + 2] = __builtin_bit_cast(uint32_t, s);
  }
}

}  // namespace cn
