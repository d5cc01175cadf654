// Chain kernel body with PER-TILE epilogues (included by chain.hip).
//
// Same arithmetic, operand layouts, weight stream and stores as Chain (the
// prologues and constants are Chain's), but the epilogue of output tile t of
// a layer runs right after that tile's last MFMA instead of after the whole
// layer:
//   * the tile's bias/ReLU/pack/mask/store work overlaps the MFMAs of the next
//     tile, and the next layer's first MFMAs overlap the last tile's
//     epilogue -- with whole-layer epilogues every wave of a SIMD sat in the
//     same VALU burst at every layer boundary with the matrix core idle;
//   * accumulators ping-pong over two tiles (32 VGPRs instead of 128); the
//     packed B operand is double-buffered per layer parity (layer li reads
//     bin[li & 1], its epilogues write bin[(li + 1) & 1]);
//   * plane stores are issued by the tile epilogues (two 16-B stores per
//     bf16 tile), which spreads them over the layer without the deferred
//     store schedule.
#pragma once

namespace cn {

template <int P, int SB, int TB, bool BWD, int WAVES, int MODE>
struct ChainT {
  using C = Chain<P, SB, TB, BWD, WAVES, MODE>;
  using S = typename C::S;
  using N = typename C::N;
  using E = typename C::E;
  using BinT = typename C::BinT;
  static constexpr int kBin = C::kBin;
  static constexpr bool kBf16 = C::kBf16;
  static constexpr bool TRAIN = C::TRAIN;
  static constexpr int NL = C::NL;
  static constexpr int kChunks = C::kChunks;
  static constexpr int D = C::D, NS = C::NS, kPF = C::kPF;
  static constexpr int kRingBytes = C::kRingBytes;
  static constexpr int kWsOff = C::kWsOff, kMiscOff = C::kMiscOff;
  static constexpr int kDirOff = C::kDirOff, kDirStash = C::kDirStash, kMaskOff = C::kMaskOff;
  static constexpr int kLdsBytes = C::kLdsBytes;

  static constexpr bool plane_of(int i) { return C::plane_of(i); }
  static constexpr int tiles_before(int li) {
    int s = 0;
    for (int k = 0; k < li; ++k) s += S::L(k).T;
    return s;
  }
  static constexpr int kTiles = tiles_before(NL);
  static constexpr int layer_of_tile(int J) {
    int i = 0;
    while (i + 1 < NL && tiles_before(i + 1) <= J) ++i;
    return i;
  }

  // ---------------- epilogue placement
  // CN_CHAIN_DEFEPI: the epilogue of tile J is emitted in two halves (groups
  // 0-1, then 2-3 + the layer finalisation) between the MFMAs of tile J + 1,
  // after its k-blocks 1 and 3, so its VALU work issues while those MFMAs
  // execute (left to the scheduler, the epilogue ran as one VALU burst with
  // the matrix core idle: SQ_VALU_MFMA_COEXEC_CYCLES ~0.1 of the cycles);
  // the last tile's epilogue follows the loop.  Otherwise the whole epilogue
  // (half 2) follows the tile's last block.
  static constexpr bool kDef = CN_CHAIN_DEFEPI != 0;
  static constexpr int tile_first_block(int J) {
    const int li = layer_of_tile(J);
    return S::first_block(li) + (J - tiles_before(li)) * S::bpt(li);
  }
  static constexpr int tile_bpt(int J) { return S::bpt(layer_of_tile(J)); }
  // global block after which part `half` of tile J's epilogue is emitted
  // (kBlocks: after the loop)
  static constexpr int emit_block(int J, int half) {
    if (!kDef) return half == 2 ? tile_first_block(J) + tile_bpt(J) - 1 : -1;
    if (half == 2) return -1;
    if (J + 1 >= kTiles) return S::kBlocks;
    const int b = tile_bpt(J + 1);
    const int kb = half == 0 ? (b - 1 < 1 ? b - 1 : 1) : (b - 1 < 3 ? b - 1 : 3);
    return tile_first_block(J + 1) + kb;
  }
  // vector-memory stores issued by part `half` of tile J's epilogue
  static constexpr int stores_of_part(int J, int half) {
    const int li = layer_of_tile(J);
    const Layer l = S::L(li);
    const int t = J - tiles_before(li);
    if (!BWD && l.epi == EPI_RGB) return 0;     // after the last wait: not counted (safe)
    const int per_tile = plane_of(li) ? (kBf16 ? 2 : 4) : 0;
    int s = half == 2 ? per_tile : per_tile / 2;
    if (!BWD && half != 0 && t == l.T - 1) {
      if (TRAIN && l.mask >= 0) s += 1;
      if (l.epi == EPI_SHAPE) s += TRAIN ? 2 : 1;
    }
    return s;
  }
  // vector-memory stores a wave issues in each chunk (tile epilogues), built
  // once: one walk over the tiles' epilogue parts
  struct ChunkStores {
    int n[kChunks + 1] = {};
  };
  static constexpr ChunkStores chunk_stores() {
    ChunkStores cs{};
    for (int J = 0; J < kTiles; ++J)
      for (int half = 0; half < 3; ++half) {
        const int b = emit_block(J, half);
        if (b >= 0 && b < S::kBlocks) cs.n[b / kChunkBlocks] += stores_of_part(J, half);
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

  // accumulator of global tile J <- bias of its forward layer (rows 32t + 8g + 4h + i)
  template <int J>
  __device__ static void load_bias_tile(f32x16& acc, const float* prm, int h) {
    constexpr int li = layer_of_tile(J);
    constexpr int t = J - tiles_before(li);
    const float* b = prm + li * 256 + 32 * t + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *(const f32x4*)(b + 8 * g);
      acc[4 * g + 0] = v[0];
      acc[4 * g + 1] = v[1];
      acc[4 * g + 2] = v[2];
      acc[4 * g + 3] = v[3];
    }
  }

  __device__ static void run(const ChainArgs& a) {
    __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const int m = blockIdx.x * (WAVES * 32) + w * 32 + (lane & 31);
    const int mc = m < a.M ? m : a.M - 1;
    const int wglob = blockIdx.x * WAVES + w;
    // a workgroup of WAVES * 32 samples need not divide the 256-padded rows
    // (12-wave backward): waves past the end compute on clamped inputs and
    // store nothing (empty buffer ranges)
    const int nslab = ((a.M + 255) & ~255) >> 5;
    const bool live = wglob < nslab;
    float* prm = (float*)(smem + kRingBytes);
    uint32_t voff[6];   // [g]: 8-B stores of group g; [4 + gp]: bf16 16-B pair stores
#pragma unroll
    for (int g = 0; g < 4; ++g) voff[g] = (uint32_t)slab_off(lane & 31, 8 * g + 4 * h, (int)sizeof(E));
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) voff[4 + gp] = (uint32_t)(bf16_pos(lane & 31, gp, h) * 16 + gp * 1024);

    for (int i = threadIdx.x; i < C::kBlobFloats / 4; i += WAVES * 64)
      ((f32x4*)prm)[i] = ((const f32x4*)a.bias)[i];

    BinT bin[2][kBin];
    // [tile parity][k-block parity]: CN_CHAIN_2ACC splits each tile's
    // accumulation into two independent MFMA chains (even / odd k-blocks,
    // summed by the epilogue)
    f32x16 acc[2][2];
#pragma unroll
    for (int q = 0; q < kBin; ++q) bin[0][q] = bin[1][q] = BinT{};
    acc[0][0] = acc[1][0] = acc[0][1] = acc[1][1] = f32x16{};

    float ds = 0.f;
    if constexpr (!BWD) C::prologue_fwd(a, bin[0], smem, h, lane, w, m, mc, wglob, voff);
    else ds = C::prologue_bwd(a, bin[0], smem, h, lane, w, m, mc, wglob, voff, live, live ? wglob : nslab - 1);
    __syncthreads();
    if constexpr (!BWD) {
      load_bias_tile<0>(acc[0][0], prm, h);
      if constexpr (kTiles > 1) load_bias_tile<1>(acc[1][0], prm, h);
    }

    static_for<0, D>([&](auto i) { C::template issue<i>(a, smem, w, lane); });

    float sig_part = 0.f;
    uint32_t mlo[4] = {0u, 0u, 0u, 0u}, mhi[4] = {0u, 0u, 0u, 0u};

    // part `half` of global tile J's epilogue (0: groups 0-1, 1: groups 2-3 +
    // finalisation, 2: all)
    auto emit = [&](auto Jc, auto Hc) {
      constexpr int J = Jc, HALF = Hc;
      constexpr int li = layer_of_tile(J);
      constexpr int t = J - tiles_before(li);
      f32x16& a0 = acc[J & 1][0];
      if constexpr (HALF != 1 && kBf16 && CN_CHAIN_2ACC && S::bpt(li) > 1) a0 += acc[J & 1][1];
      if constexpr (!BWD) {
        tile_fwd<li, t, HALF>(a, bin[(li & 1) ^ 1], a0, prm, smem, h, lane, w, m, wglob, voff, sig_part, mlo, mhi);
        if constexpr (HALF != 0 && J + 2 < kTiles) load_bias_tile<J + 2>(a0, prm, h);
      } else {
        tile_bwd<li, t, HALF>(a, bin[(li & 1) ^ 1], a0, prm, smem, h, lane, w, m, wglob, voff, ds, live);
      }
    };

    auto chunk = [&](auto cc) {
      constexpr int c = cc;
      const char* slot = smem + (c % NS) * kChunkBytes + lane * 16;
      bf16x8 Abuf[kPF + 1];
      if constexpr (kBf16)
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
          constexpr int J = tiles_before(li) + t;
          constexpr int cur = li & 1;
          const char* ap = slot + bb * kBlockBytes;
          constexpr int kp = (kBf16 && CN_CHAIN_2ACC) ? (kb & 1) : 0;
          f32x16& ac = acc[J & 1][kp];
          // first MFMA of a chain: C = 0 (backward; forward odd chain), else the running sum
          constexpr bool zero_c = BWD ? kb <= kp : (kp == 1 && kb == 1);
          if constexpr (kBf16) {
            if constexpr (bb + kPF < kChunkBlocks && g + kPF < S::kBlocks)
              Abuf[(bb + kPF) % (kPF + 1)] = *(const bf16x8*)(ap + kPF * kBlockBytes);
            ac = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Abuf[bb % (kPF + 1)], __builtin_bit_cast(bf16x8, bin[cur][kb]),
                                                         zero_c ? f32x16{} : ac, 0, 0, 0);
#if CN_CHAIN_SB
            __builtin_amdgcn_sched_barrier(CN_CHAIN_SB_MASK);
#endif
          } else {
            const f32x4 A = *(const f32x4*)ap;
            ac = __builtin_amdgcn_mfma_f32_32x32x2f32(A[0], bin[cur][4 * kb + 0], zero_c ? f32x16{} : ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_32x32x2f32(A[1], bin[cur][4 * kb + 1], ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_32x32x2f32(A[2], bin[cur][4 * kb + 2], ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_32x32x2f32(A[3], bin[cur][4 * kb + 3], ac, 0, 0, 0);
          }
          if constexpr (!kDef) {
            if constexpr (kb == S::bpt(li) - 1) emit(std::integral_constant<int, J>{}, std::integral_constant<int, 2>{});
          } else if constexpr (J >= 1) {
            static_for<0, 2>([&](auto hh) {
              if constexpr (emit_block(J - 1, hh) == g)
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
    if constexpr (kDef) {
      emit(std::integral_constant<int, kTiles - 1>{}, std::integral_constant<int, 0>{});
      emit(std::integral_constant<int, kTiles - 1>{}, std::integral_constant<int, 1>{});
    }
  }

  // ---------------- forward tile epilogue: tile t of layer LI -> bin_next
  template <int LI, int T_, int HALF>
  __device__ static void tile_fwd(const ChainArgs& a, BinT* bin, const f32x16& acc, const float* prm, const char* smem,
                                  int h, int lane, int w, int m, int wglob, const uint32_t* voff, float& sig_part,
                                  uint32_t* mlo, uint32_t* mhi) {
    constexpr Layer l = S::L(LI);
    constexpr int t = T_;
    constexpr int g0 = HALF == 1 ? 2 : 0, g1 = HALF == 0 ? 2 : 4;
    constexpr bool fin = HALF != 0;
    if constexpr (l.epi == EPI_RGB) {
      if (fin && h == 0) {
        a.rgb[3 * m + 0] = acc[0];
        a.rgb[3 * m + 1] = acc[1];
        a.rgb[3 * m + 2] = acc[2];
      }
      return;
    } else {
      constexpr int yp = l.plane >= 0 ? l.plane : 0;
      constexpr int YF = N::plane_width(yp);
      const auto ry = slab_rsrc<E>(a.Y[yp], YF, wglob);
      const float* ws = prm + kWsOff + 4 * h;
      u32x2 pg[4];
#pragma unroll
      for (int g = g0; g < g1; ++g) {
        float v0 = acc[4 * g + 0], v1 = acc[4 * g + 1];
        float v2 = acc[4 * g + 2], v3 = acc[4 * g + 3];
        if constexpr (TRAIN && l.mask >= 0) {
          // elements 0 / 2 into the low half, 1 / 3 into the high half
          // (Chain::mask_pos): push order q = 8 (t & 1) + 2 g + i / 2
          mlo[t >> 1] = push_sign(push_sign(mlo[t >> 1], v0), v2);
          mhi[t >> 1] = push_sign(push_sign(mhi[t >> 1], v1), v3);
        }
        if constexpr (l.epi == EPI_SHAPE) {
          const f32x4 w4 = *(const f32x4*)(ws + 32 * t + 8 * g);
          sig_part = __builtin_fmaf(w4[0], v0, sig_part);
          sig_part = __builtin_fmaf(w4[1], v1, sig_part);
          sig_part = __builtin_fmaf(w4[2], v2, sig_part);
          sig_part = __builtin_fmaf(w4[3], v3, sig_part);
        }
        if constexpr (kBf16) {
          uint32_t p0 = pack_bf16x2(v0, v1), p1 = pack_bf16x2(v2, v3);
          if constexpr (l.epi == EPI_RELU) { p0 = relu_bf16x2(p0); p1 = relu_bf16x2(p1); }
          BinT& b = bin[2 * t + (g >> 1)];
          if ((g & 1) == 0) { b[0] = p0; b[1] = p1; } else { b[2] = p0; b[3] = p1; }
          pg[g] = u32x2{p0, p1};
          if constexpr (plane_of(LI))
            if (g & 1) plane_store_pair(ry, voff[4 + (g >> 1)], t, pg[g - 1], pg[g]);
        } else {
          if constexpr (l.epi == EPI_RELU) {
            v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
          }
          bin[16 * t + 4 * g + 0] = v0;
          bin[16 * t + 4 * g + 1] = v1;
          bin[16 * t + 4 * g + 2] = v2;
          bin[16 * t + 4 * g + 3] = v3;
          if constexpr (plane_of(LI)) plane_store<E>(ry, voff, t, g, v0, v1, v2, v3);
        }
      }
      if constexpr (fin && t == l.T - 1) {
        if constexpr (TRAIN && l.mask >= 0) {
          uint32_t mw[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            mw[k] = (mhi[k] << 16) | (mlo[k] & 0xFFFFu);
            mlo[k] = mhi[k] = 0u;
          }
          bstore128(mkrsrc(a.masks + (size_t)wglob * N::kMasks * 256), ((uint32_t)l.mask * 64 + lane) * 16,
                    u32x4{mw[0], mw[1], mw[2], mw[3]});
        }
        if constexpr (l.epi == EPI_SHAPE) {
          const float tot = sig_part + __shfl_xor(sig_part, 32);
          const float pre = tot + prm[kMiscOff];
          bstore32(mkrsrc(a.sigma), (uint32_t)m * 4, f2u(softplus20(pre)));
          if constexpr (TRAIN) bstore32(mkrsrc(a.spre), (uint32_t)m * 4, f2u(pre));
        }
        if constexpr (S::L(LI + 1).in_kind == IN_ACC_DIR) {
          const char* stash = smem + kDirOff + (w * 64 + lane) * kDirStash;
          if constexpr (kBf16) {
            bin[16] = ((const u32x4*)stash)[0];
            bin[17] = ((const u32x4*)stash)[1];
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f32x4 v = ((const f32x4*)stash)[q];
              bin[128 + 4 * q + 0] = v[0]; bin[128 + 4 * q + 1] = v[1];
              bin[128 + 4 * q + 2] = v[2]; bin[128 + 4 * q + 3] = v[3];
            }
          }
        }
      }
    }
  }

  // ---------------- backward tile epilogue: tile t of dX layer LI -> bin_next
  template <int LI, int T_, int HALF>
  __device__ static void tile_bwd(const ChainArgs& a, BinT* bin, const f32x16& acc, const float* prm,
                                  const char* smem, int h, int lane, int w, int m, int wglob, const uint32_t* voff,
                                  float ds, bool live) {
    constexpr Layer l = S::L(LI);
    constexpr int t = T_;
    constexpr int width = N::dplane_width(l.plane);
    const auto rdA = slab_rsrc<E>(a.dA[l.plane], width, wglob, live);
    uint32_t mword = 0u;
    if constexpr (l.epi == EPI_BMASK)
      mword = *(const uint32_t*)(smem + kMaskOff + (((size_t)w * N::kMasks + l.mask) * 64 + lane) * 16 + 4 * (t >> 1));
    const float* ws = prm + kWsOff + 4 * h;
    constexpr int g0 = HALF == 1 ? 2 : 0, g1 = HALF == 0 ? 2 : 4;
    u32x2 pg[4];
#pragma unroll
    for (int g = g0; g < g1; ++g) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc[4 * g + i];
        if constexpr (l.epi == EPI_BMASK && !kBf16) v[i] = relu_mask(v[i], mword, C::mask_pos(t, g, i));
      }
      if constexpr (l.epi == EPI_BSIGMA) {
        const f32x4 w4 = *(const f32x4*)(ws + 32 * t + 8 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fadd_rn(v[i], fmul_rn(ds, w4[i]));
      }
      if constexpr (kBf16) {
        uint32_t p0 = pack_bf16x2(v[0], v[1]), p1 = pack_bf16x2(v[2], v[3]);
        if constexpr (l.epi == EPI_BMASK) {
          static_for<0, 4>([&](auto gg) {
            if (gg == g) {
              p0 = relu_mask_bf16x2<C::mask_q(t, gg, 0)>(p0, mword);
              p1 = relu_mask_bf16x2<C::mask_q(t, gg, 2)>(p1, mword);
            }
          });
        }
        BinT& b = bin[2 * t + (g >> 1)];
        if ((g & 1) == 0) { b[0] = p0; b[1] = p1; } else { b[2] = p0; b[3] = p1; }
        pg[g] = u32x2{p0, p1};
        if constexpr (plane_of(LI))
          if (g & 1) plane_store_pair(rdA, voff[4 + (g >> 1)], t, pg[g - 1], pg[g]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) bin[16 * t + 4 * g + i] = v[i];
        if constexpr (plane_of(LI)) plane_store<E>(rdA, voff, t, g, v[0], v[1], v[2], v[3]);
      }
    }
  }
};

}  // namespace cn
