// bf16 dX chain with TWO 32-sample groups per wave (CN_CHAIN_NG2, with
// CN_BWD_WAVES=4 and CN_CHAIN_TILEEPI): one wave per SIMD owns 64 samples and
// every A fragment read from the LDS ring feeds two MFMAs, halving the
// A-fragment reads, barriers and per-block issue work per MFMA (the fp32 chain
// amortises the same overhead over 4x the MFMA cycles and runs at 85%).
// Registers: bin[layer parity][group] + acc[tile parity][group] ~ 330 VGPRs,
// so one wave per SIMD (512).  Planes, masks and the slab numbering are those
// of the 8-wave kernel: group q of wave w is slab 2w + q of the workgroup.
// Reuses ChainT's schedule, epilogues and store bookkeeping.
#pragma once

namespace cn {

template <int P, int SB, int TB, int WAVES, int MODE>
struct ChainG {
  using C = Chain<P, SB, TB, true, WAVES, MODE>;
  using T = ChainT<P, SB, TB, true, WAVES, MODE>;
  using S = typename C::S;
  using N = typename C::N;
  using E = typename C::E;
  using BinT = typename C::BinT;
  static constexpr int NG = 2;
  static constexpr int kBin = C::kBin;
  static constexpr int kChunks = C::kChunks;
  static constexpr int D = C::D, NS = C::NS, kPF = C::kPF;
  static constexpr int kTiles = T::kTiles;
  static constexpr int kLdsBytes = C::kMaskOff + WAVES * NG * N::kMasks * 1024;
  static_assert(P == CN_P_BF16, "bf16 only");
  static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

  struct ChunkStores {
    int n[kChunks + 1] = {};
  };
  static constexpr ChunkStores chunk_stores() {
    ChunkStores cs{};
    for (int J = 0; J < kTiles; ++J)
      for (int half = 0; half < 3; ++half) {
        const int b = T::emit_block(J, half);
        if (b >= 0 && b < S::kBlocks) cs.n[b / kChunkBlocks] += NG * T::stores_of_part(J, half);
      }
    return cs;
  }
  static constexpr ChunkStores kChunkStores = chunk_stores();
  static constexpr int stores_in_chunk(int c) { return c < kChunks ? kChunkStores.n[c] : 0; }
  static constexpr int issued(int i) { return i < kChunks ? C::G : 0; }
  static constexpr int vm_wait(int c) {
    int n = 0;
    if (c < D) {
      for (int i = c + 1; i < D; ++i) n += issued(i);
      for (int i = 0; i < c; ++i) n += issued(i + D) + stores_in_chunk(i);
    } else {
      n += stores_in_chunk(c - D);
      for (int i = c - D + 1; i < c; ++i) n += issued(i + D) + stores_in_chunk(i);
    }
    return n;
  }

  __device__ static void run(const ChainArgs& a) {
    __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const int nslab = ((a.M + 255) & ~255) >> 5;
    int m[NG], mc[NG], wq[NG], wglob[NG];
    bool live[NG];
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      wq[q] = w * NG + q;
      wglob[q] = blockIdx.x * (WAVES * NG) + wq[q];
      m[q] = wglob[q] * 32 + (lane & 31);
      mc[q] = m[q] < a.M ? m[q] : a.M - 1;
      live[q] = wglob[q] < nslab;
    }
    float* prm = (float*)(smem + C::kRingBytes);
    uint32_t voff[6];
#pragma unroll
    for (int g = 0; g < 4; ++g) voff[g] = (uint32_t)slab_off(lane & 31, 8 * g + 4 * h, (int)sizeof(E));
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) voff[4 + gp] = (uint32_t)(bf16_pos(lane & 31, gp, h) * 16 + gp * 1024);
    for (int i = threadIdx.x; i < C::kBlobFloats / 4; i += WAVES * 64)
      ((f32x4*)prm)[i] = ((const f32x4*)a.bias)[i];

    BinT bin[2][NG][kBin];
    f32x16 acc[2][NG];
#pragma unroll
    for (int q = 0; q < NG; ++q) {
#pragma unroll
      for (int k = 0; k < kBin; ++k) bin[0][q][k] = bin[1][q][k] = BinT{};
      acc[0][q] = acc[1][q] = f32x16{};
    }
    float ds[NG];
#pragma unroll
    for (int q = 0; q < NG; ++q)
      ds[q] = C::prologue_bwd(a, bin[0][q], smem, h, lane, wq[q], m[q], mc[q], wglob[q], voff, live[q],
                              live[q] ? wglob[q] : nslab - 1);
    __syncthreads();

    static_for<0, D>([&](auto i) { C::template issue<i>(a, smem, w, lane); });

    auto emit = [&](auto Jc, auto Hc) {
      constexpr int J = Jc, HALF = Hc;
      constexpr int li = T::layer_of_tile(J);
      constexpr int t = J - T::tiles_before(li);
#pragma unroll
      for (int q = 0; q < NG; ++q)
        T::template tile_bwd<li, t, HALF>(a, bin[(li & 1) ^ 1][q], acc[J & 1][q], prm, smem, h, lane, wq[q], m[q],
                                          wglob[q], voff, ds[q], live[q]);
    };

    auto chunk = [&](auto cc) {
      constexpr int c = cc;
      const char* slot = smem + (c % NS) * kChunkBytes + lane * 16;
      bf16x8 Abuf[kPF + 1];
      static_for<0, kPF>([&](auto bb) {
        if constexpr (c * kChunkBlocks + bb < S::kBlocks) Abuf[bb] = *(const bf16x8*)(slot + bb * kBlockBytes);
      });
      static_for<0, kChunkBlocks>([&](auto bb) {
        constexpr int g = c * kChunkBlocks + bb;
        if constexpr (g < S::kBlocks) {
          constexpr int li = S::layer_of(g);
          constexpr int lb = g - S::first_block(li);
          constexpr int t = lb / S::bpt(li);
          constexpr int kb = lb % S::bpt(li);
          constexpr int J = T::tiles_before(li) + t;
          constexpr int cur = li & 1;
          const char* ap = slot + bb * kBlockBytes;
          if constexpr (bb + kPF < kChunkBlocks && g + kPF < S::kBlocks)
            Abuf[(bb + kPF) % (kPF + 1)] = *(const bf16x8*)(ap + kPF * kBlockBytes);
#pragma unroll
          for (int q = 0; q < NG; ++q)
            acc[J & 1][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                Abuf[bb % (kPF + 1)], __builtin_bit_cast(bf16x8, bin[cur][q][kb]), kb == 0 ? f32x16{} : acc[J & 1][q],
                0, 0, 0);
#if CN_CHAIN_SB
          __builtin_amdgcn_sched_barrier(CN_CHAIN_SB_MASK);
#endif
          if constexpr (!T::kDef) {
            if constexpr (kb == S::bpt(li) - 1) emit(std::integral_constant<int, J>{}, std::integral_constant<int, 2>{});
          } else if constexpr (J >= 1) {
            static_for<0, 2>([&](auto hh) {
              if constexpr (T::emit_block(J - 1, hh) == g)
                emit(std::integral_constant<int, J - 1>{}, std::integral_constant<int, (int)hh>{});
            });
          }
        }
      });
    };
    static_for<0, kChunks>([&](auto kk) {
      constexpr int k = kk;
      wait_vmcnt<vm_wait(k)>();
      block_barrier();
      if constexpr (k + D < kChunks) C::template issue<k + D>(a, smem, w, lane);
      chunk(std::integral_constant<int, k>{});
    });
    if constexpr (T::kDef) {
      emit(std::integral_constant<int, kTiles - 1>{}, std::integral_constant<int, 0>{});
      emit(std::integral_constant<int, kTiles - 1>{}, std::integral_constant<int, 1>{});
    }
  }
};

}  // namespace cn
