// Micro-benchmark: what the weight stream costs an MFMA chain (gfx950).
//
// One persistent workgroup per CU runs the chain kernels' inner loop shape:
// per 16 KiB chunk of "weights" (16 x 1 KiB A fragments in an LDS ring),
// every wave reads each fragment (ds_read_b128) and issues its MFMAs
// (bf16: 1 x 32x32x16 per fragment, 8 waves = 2 per SIMD; x3: 3 MFMAs per
// two fragments, 4 waves = 1 per SIMD), one s_barrier per chunk.  The ring
// is refilled in different ways (MODE):
//   0  no refill (MFMA + LDS reads + barrier only)
//   1  LDS-DMA (buffer_load_dwordx4 ... lds), each wave's pieces right after
//      the barrier (the chain kernels' placement)
//   2  LDS-DMA, each wave's pieces spread over the chunk (wave-staggered)
//   3  buffer_load_dwordx4 to VGPRs after the barrier, ds_write_b128 at mid-chunk
//   4  no barrier, no refill (MFMA + LDS reads only)
// Prints cycles per MFMA (s_memtime, median over workgroups) per mode.
// Timing probe only: the LDS contents are never checked.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((address_space(3))) void lds_void;

template <int Begin, int End, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (Begin < End) {
    f(std::integral_constant<int, Begin>{});
    static_for<Begin + 1, End>(f);
  }
}

constexpr int kChunk = 16 * 1024, kNS = 5, kD = 3;

template <int MODE, int WAVES, bool X3>
__global__ __launch_bounds__(WAVES * 64, 1) void chain_probe(const char* src, float* out, long long* cyc, int nchunk) {
  __shared__ __attribute__((aligned(16))) char smem[kNS * kChunk];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int G = 16 / WAVES;           // pieces per wave per chunk
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), (short)0, -1, 0x00020000);
  f32x16 acc[8];
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  u32x4 bin[16], binl[16];
  for (int q = 0; q < 16; ++q) {
    bin[q] = u32x4{(unsigned)lane * 0x00010001u + q, 0x3f803f80u, 0x3f003f00u, (unsigned)q};
    binl[q] = bin[q] ^ u32x4{0x00800080u, 0, 0, 0};
  }
  for (int i = threadIdx.x; i < kNS * kChunk / 16; i += WAVES * 64) ((u32x4*)smem)[i] = u32x4{1u, 2u, 3u, (unsigned)i};
  __syncthreads();
  const uint32_t voffs = (uint32_t)(w * G * 1024 + lane * 16);
  u32x4 stage[G];
  auto dma_piece = [&](int c, int k) {
    char* dst = smem + ((c + kD) % kNS) * kChunk + (w * G + k) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, voffs, ((c + kD) & 63) * kChunk + k * 1024, 0, 0);
  };
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int c = 0; c < nchunk; ++c) {
    if constexpr (MODE != 4) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MODE == 1 || MODE == 2 ? (kD - 1) * G : 0) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if constexpr (MODE == 1)
      static_for<0, G>([&](auto k) { dma_piece(c, k); });
    if constexpr (MODE == 3)
      static_for<0, G>([&](auto k) {
        stage[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, voffs, ((c + kD) & 63) * kChunk + k * 1024, 0);
      });
    const char* slot = smem + (c % kNS) * kChunk + lane * 16;
    static_for<0, 16>([&](auto g) {
      if constexpr (MODE == 2) {
        // wave w's piece k after block (w * G + k) * 16 / 16... spread: block index b issues piece k when
        // b == (k * 16 / G + 2 * w) % 16
        static_for<0, G>([&](auto k) {
          if (g == (k * (16 / G) + 2 * w) % 16) dma_piece(c, k);
        });
      }
      if constexpr (MODE == 3 && g == 8) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        static_for<0, G>([&](auto k) {
          *(u32x4*)(smem + ((c + kD) % kNS) * kChunk + (w * G + k) * 1024 + lane * 16) = stage[k];
        });
      }
      const bf16x8 A = *(const bf16x8*)(slot + g * 1024);
      if constexpr (!X3) {
        acc[g / 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, __builtin_bit_cast(bf16x8, bin[g]), acc[g / 2], 0, 0, 0);
      } else {
        // fragments in (hi, lo) pairs: hi*hi + hi*lo, then lo*hi
        constexpr int kb = g / 2;
        if constexpr (g % 2 == 0) {
          acc[kb % 8] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, __builtin_bit_cast(bf16x8, bin[kb]), acc[kb % 8], 0, 0, 0);
          acc[kb % 8] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, __builtin_bit_cast(bf16x8, binl[kb]), acc[kb % 8], 0, 0, 0);
        } else {
          acc[kb % 8] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, __builtin_bit_cast(bf16x8, bin[kb]), acc[kb % 8], 0, 0, 0);
        }
      }
    });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int t = 0; t < 8; ++t)
    for (int r = 0; r < 16; ++r) s += acc[t][r];
  out[blockIdx.x * WAVES * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int WAVES, bool X3>
void run(const char* src, float* out, long long* cyc, int nwg, int nchunk, const char* name) {
  hipLaunchKernelGGL((chain_probe<MODE, WAVES, X3>), dim3(nwg), dim3(WAVES * 64), 0, 0, src, out, cyc, nchunk);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL((chain_probe<MODE, WAVES, X3>), dim3(nwg), dim3(WAVES * 64), 0, 0, src, out, cyc, nchunk);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  std::vector<long long> h(nwg);
  hipMemcpy(h.data(), cyc, nwg * sizeof(long long), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double mfma_per_wave = (double)nchunk * (X3 ? 24 : 16);
  const int waves_per_simd = WAVES / 4;
  // s_memtime ticks = shader clock cycles; per SIMD the waves share the MFMA pipe
  printf("%-28s %8.3f ms/launch  cycles/MFMA/SIMD %.2f (ideal 32)\n", name, ms / 5,
         (double)h[nwg / 2] / (mfma_per_wave * waves_per_simd));
}

int main(int argc, char** argv) {
  const int nwg = 256, nchunk = argc > 1 ? atoi(argv[1]) : 4000;
  char* src;
  float* out;
  long long* cyc;
  hipMalloc(&src, 64 * kChunk + 4096);
  hipMemset(src, 0, 64 * kChunk + 4096);
  hipMalloc(&out, nwg * 512 * sizeof(float));
  hipMalloc(&cyc, nwg * sizeof(long long));
  for (int rep = 0; rep < 2; ++rep) {
    printf("--- round %d\n", rep);
    run<4, 8, false>(src, out, cyc, nwg, nchunk, "bf16 8w: mfma+lds only");
    run<0, 8, false>(src, out, cyc, nwg, nchunk, "bf16 8w: + barrier");
    run<1, 8, false>(src, out, cyc, nwg, nchunk, "bf16 8w: + dma at barrier");
    run<2, 8, false>(src, out, cyc, nwg, nchunk, "bf16 8w: + dma staggered");
    run<3, 8, false>(src, out, cyc, nwg, nchunk, "bf16 8w: + vgpr stage");
    run<4, 4, true>(src, out, cyc, nwg, nchunk, "x3 4w: mfma+lds only");
    run<0, 4, true>(src, out, cyc, nwg, nchunk, "x3 4w: + barrier");
    run<1, 4, true>(src, out, cyc, nwg, nchunk, "x3 4w: + dma at barrier");
    run<2, 4, true>(src, out, cyc, nwg, nchunk, "x3 4w: + dma staggered");
    run<3, 4, true>(src, out, cyc, nwg, nchunk, "x3 4w: + vgpr stage");
  }
  return 0;
}
