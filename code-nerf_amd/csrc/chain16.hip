// Fused CodeNeRF MLP chain kernels on v_mfma_f32_16x16x32_bf16 (forward and
// dX-backward) -- the layout of the bf16x3 precision (round 5).
//
// Same job as chain.hip (reference src/model.py:36-53 forward, the dX part of
// the backward of src/trainer.py:82), same HBM formats (activation planes,
// packed weight stream of 1 KiB blocks through a 16 KiB-slot LDS ring), but a
// wave owns 16 samples instead of 32:
//
//   * an MFMA computes Y^T[16 out features][16 samples] = W[16][32] X^T[32][16];
//     lane l holds sample l & 15, lane group q = l >> 4 holds output rows
//     4q .. 4q+3 of each 16-feature tile (C/D layout) and the input k-slots
//     8q .. 8q+7 of each 32-wide k-block (B layout);
//   * the accumulator of tiles 2u, 2u+1 IS the next layer's k-block u: k-slot
//     (q, j) <-> feature 32u + 16 (j >> 2) + 4q + (j & 3) (acc16_feature); the
//     packed weights absorb the permutation;
//   * registers per wave: 16 tiles x 4 accumulators (64) + the B operand
//     (9 k-blocks x 4, hi AND lo for bf16x3: 72) -- 136 against the 272 of a
//     32-sample wave, so bf16x3 runs TWO waves per SIMD (8-wave workgroups,
//     128 samples per weight stream) where chain.hip ran one: while one wave
//     converts a tile (ReLU, mask bits, hi / lo split, plane stores) or issues
//     its share of the weight stream's LDS-DMA, the other issues MFMAs;
//   * a lane's 4 features of a tile are 4 consecutive plane elements (8 B):
//     one buffer_store_dwordx2 per tile into the unchanged plane layout
//     (cn_layout.h slab_off), so the dW pass reads what it always read.
#include "cn_common.h"
#include "cn_sched.h"
#include "chain_args.h"

namespace cn {

// k-slot (k-block u, lane group q, element j) of an accumulator-fed input ->
// input feature
inline constexpr int acc16_feature(int u, int q, int j) { return 32 * u + 16 * (j >> 2) + 4 * q + (j & 3); }
// PE / dir planes: the same slot -> plane column (features of chain.hip's
// slot order: cn_layout.h pe_slot_feature / dir_slot_feature of col_half /
// col_slot), so the planes keep their layout
inline constexpr int col16(int u, int q, int j) { return acc16_feature(u, q, j); }

// Block schedule of a 16x16x32 chain: layer, output tile (16 rows), k-block
// (32), [W_hi, W_lo] fragment.
template <int P, int SB, int TB, bool BWD>
struct Sched16 {
  using N = Net<SB, TB>;
  static constexpr int NL = BWD ? N::kBwdLayers : N::kFwdLayers;
  static constexpr int kAmul = (P == CN_P_BF16X3) ? 2 : 1;
  static constexpr Layer L(int i) { return BWD ? N::bwd(i) : N::fwd(i); }
  // output tiles of 16 features (the rgb head: one tile, 3 real rows)
  static constexpr int tiles(int i) { return (!BWD && i == NL - 1) ? 1 : 2 * L(i).T; }
  // k-blocks of 32 (the drgb input of the first dX layer: one)
  static constexpr int kblocks(int i) { return (BWD && i == 0) ? 1 : L(i).K / 32; }
  static constexpr int bpt(int i) { return kblocks(i) * kAmul; }
  static constexpr int lblocks(int i) { return tiles(i) * bpt(i); }
  static constexpr int first_block(int i) {
    int s = 0;
    for (int k = 0; k < i; ++k) s += lblocks(k);
    return s;
  }
  static constexpr int kBlocks = first_block(NL);
  static constexpr int kChunks = (kBlocks + kChunkBlocks - 1) / kChunkBlocks;
  static constexpr int layer_of(int g) {
    int i = 0;
    while (i + 1 < NL && first_block(i + 1) <= g) ++i;
    return i;
  }
  static constexpr int last_block(int i) { return first_block(i) + lblocks(i) - 1; }
  static constexpr int packed_bytes() { return kChunks * kChunkBytes; }
};

template <int P, int SB, int TB, bool BWD, int WAVES, int MODE>
struct Chain16 {
  using S = Sched16<P, SB, TB, BWD>;
  using N = Net<SB, TB>;
  static_assert(P == CN_P_BF16 || P == CN_P_BF16X3, "16x16x32 chains are bf16-operand kernels");
  static constexpr bool kX3 = (P == CN_P_BF16X3);
  static constexpr bool TRAIN = MODE != CN_MODE_INFER;    // masks + sigma pre-activation
  static constexpr bool PLANES = MODE == CN_MODE_TRAIN;   // every operand plane of dW
  static constexpr bool kXlo = kX3 && PLANES && !BWD;     // + the lo parts of dW's X operands
  static constexpr int NL = S::NL;
  static constexpr int kChunks = S::kChunks;
  static constexpr int kSpw = 16;                          // samples per wave
  static_assert(kChunkBlocks % WAVES == 0, "every wave issues an equal share of a chunk");
  static constexpr int G = kChunkBlocks / WAVES;           // LDS-DMA instructions per wave per chunk
  // chunks in flight: a 16 KiB chunk feeds one wave 8 (bf16x3: 24) MFMAs of
  // 16 cycles, two waves per SIMD; ~1.1 us from LDS-DMA issue to landing
  static constexpr int D = kX3 ? 5 : 4;
  static constexpr int NS = D + 2;                         // ring slots (see chain.hip)
  static constexpr int kPF = 3;                            // A-fragment prefetch distance (blocks)
  static constexpr int kSbMask = 0x6;
  static constexpr int kRingBytes = NS * kChunkBytes;
  static constexpr int kBlobFloats = BiasBlob<SB, TB>::kFloats;
  static constexpr int kWsOff = BiasBlob<SB, TB>::kWs;
  static constexpr int kMiscOff = BiasBlob<SB, TB>::kMisc;
  static constexpr int kDirStash = kX3 ? 32 : 16;          // bytes per lane: the dir k-block (hi, lo)
  static constexpr int kDirOff = kRingBytes + kBlobFloats * 4;
  static constexpr int kMaskOff = kDirOff + (BWD ? 0 : WAVES * 64 * kDirStash);
  static constexpr int kMaskWave = N::kMasks * 64 * 8;     // mask bytes per wave (8 B per lane per layer)
  static constexpr int kLdsBytes = kMaskOff + (BWD ? WAVES * kMaskWave : 0);
  static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
  static_assert(kBlobFloats % 4 == 0, "blob alignment");
  static constexpr int kBin = 9;                           // k-blocks of the widest input (viewdir: 256 + 32)

  // ---------------- the plane stores of a layer
  static constexpr bool codes_plane(int p) { return MODE == CN_MODE_CODES && p >= 1 && N::fwd(p - 1).inj >= 0; }
  static constexpr bool plane_of(int i) {
    const int p = S::L(i).plane;
    return BWD ? ((PLANES && N::stored(p)) || codes_plane(p)) : (PLANES && p >= 0 && N::stored(p));
  }
  // ---------------- epilogue schedule ("diagonal", as chain.hip): tile t of
  // layer i feeds k-block t / 2 of layer i + 1.  Tiles 0-3 are converted at
  // the layer's last block, tile t >= 4 after k-block t / 2 - 2 of the next
  // layer's first tile (one k-block before the one that reads it), so the
  // conversion VALU issues between MFMAs instead of as one burst.
  static constexpr bool diag(int i) { return i + 1 < NL && S::L(i).epi != EPI_RGB; }
  static constexpr int conv_block(int i, int t) {
    return (!diag(i) || t < 4) ? S::last_block(i) : S::first_block(i + 1) + S::kAmul * ((t >> 1) - 1) - 1;
  }
  static constexpr int final_block(int i) { return conv_block(i, S::tiles(i) - 1); }
  static constexpr int conv_layer_at(int g) {
    for (int i = 0; i < NL; ++i)
      if (S::L(i).epi != EPI_RGB && g >= S::last_block(i) && g <= final_block(i))
        for (int t = 0; t < S::tiles(i); ++t)
          if (conv_block(i, t) == g) return i;
    return -1;
  }
  static constexpr int conv_first_tile(int i, int g) {
    for (int t = 0; t < S::tiles(i); ++t)
      if (conv_block(i, t) == g) return t;
    return 0;
  }
  static constexpr int conv_tiles(int i, int g) {
    int n = 0;
    for (int t = 0; t < S::tiles(i); ++t) n += conv_block(i, t) == g;
    return n;
  }
  // ---------------- compile-time vmcnt bookkeeping
  static constexpr int tile_stores(int i) { return plane_of(i) ? (kXlo ? 2 : 1) : 0; }
  static constexpr int final_stores(int i) {
    if (BWD) return 0;
    const Layer l = S::L(i);
    return (TRAIN && l.mask >= 0 ? 1 : 0) + (l.epi == EPI_SHAPE ? (TRAIN ? 2 : 1) : 0);
  }
  // VMEM stores issued right after block g's MFMAs (the rgb head's come after
  // the last wait point: not counted)
  static constexpr int stores_at_block(int g) {
    const int ci = conv_layer_at(g);
    if (ci < 0) return 0;
    return conv_tiles(ci, g) * tile_stores(ci) + (g == final_block(ci) ? final_stores(ci) : 0);
  }
  static constexpr int stores_between(int b0, int b1) {
    int s = 0;
    for (int g = b0; g < b1; ++g) s += stores_at_block(g);
    return s;
  }
  static constexpr int issued(int i) { return i < kChunks ? G : 0; }
  static constexpr int wp(int c) { return c == 0 ? 0 : c * kChunkBlocks - kPF; }
  static constexpr int wait_chunk_at(int g) {
    for (int c = 0; c < kChunks; ++c)
      if (wp(c) == g) return c;
    return -1;
  }
  static constexpr int vm_wait(int c) {
    int n = 0;
    if (c < D) {
      for (int i = c + 1; i < D; ++i) n += issued(i);
      for (int w = 0; w < c; ++w) n += issued(w + D);
      n += stores_between(0, wp(c));
    } else {
      for (int w = c - D + 1; w < c; ++w) n += issued(w + D);
      n += stores_between(wp(c - D), wp(c));
    }
    return n;
  }

  struct MaskAcc {
    uint32_t lo[2], hi[2];
  };

  // ---------------- kernel body
  __device__ static void run(const ChainArgs& a) {
    __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4;
    const int m = blockIdx.x * (WAVES * kSpw) + w * kSpw + (lane & 15);
    const int mc = m < a.M ? m : a.M - 1;
    const int wg = blockIdx.x * WAVES + w;       // global 16-sample wave index
    const int slab = wg >> 1;                    // its 32-sample plane slab
    const int s = 16 * (wg & 1) + (lane & 15);   // sample within the slab
    float* prm = (float*)(smem + kRingBytes);
    // per-lane byte offset of this lane's 4 features of a tile, by tile parity
    // (cn_layout.h slab_off(s, 16 t + 4 q); the 2 KiB per 32-feature pair of
    // tiles is a compile-time scalar offset)
    uint32_t voff[2];
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) voff[gp] = (uint32_t)slab_off(s, 16 * gp + 4 * q, 2);

    for (int i = threadIdx.x; i < kBlobFloats / 4; i += WAVES * 64)
      ((f32x4*)prm)[i] = ((const f32x4*)a.bias)[i];

    u32x4 bin[kBin];
    u32x4 binl[kX3 ? kBin : 1];
    f32x4 acc[16];
    if constexpr (!BWD)
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[t] = f32x4{};
#pragma unroll
    for (int u = 0; u < kBin; ++u) bin[u] = u32x4{};
    if constexpr (kX3)
#pragma unroll
      for (int u = 0; u < kBin; ++u) binl[u] = u32x4{};

    float ds = 0.f;
    if constexpr (!BWD) prologue_fwd(a, bin, binl, smem, q, lane, w, mc, slab, voff);
    else ds = prologue_bwd(a, bin, binl, smem, q, lane, w, m, mc, wg, slab, voff);
    __syncthreads();
    if constexpr (!BWD) static_for<0, S::tiles(0)>([&](auto t) { load_bias_tile<0>(acc[t], prm, q, t); });

    static_for<0, D>([&](auto i) { issue<i>(a, smem, w, lane); });

    float sig_part = 0.f;
    MaskAcc mk;
    bf16x8 Abuf[kPF + 1];
    const uint32_t lbase = lds_addr(smem) + lane * 16;
    auto block_off = [](int b) { return (b / kChunkBlocks % NS) * kChunkBytes + (b % kChunkBlocks) * kBlockBytes; };
    auto aread = [&](auto bbc) {
      constexpr int b = bbc;
      constexpr int off = block_off(b);
      u32x4 r;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(lbase + (off & ~0xFFFF)), "n"(off & 0xFFFF));
      Abuf[b % (kPF + 1)] = __builtin_bit_cast(bf16x8, r);
    };
    auto block = [&](auto gc) {
      constexpr int g = gc;
      constexpr int wc = wait_chunk_at(g);
      if constexpr (wc >= 0) {
        wait_vmcnt<vm_wait(wc)>();
        block_barrier_noread();
        if constexpr (wc + D < kChunks) issue<wc + D>(a, smem, w, lane);
        if constexpr (wc == 0)
          static_for<0, kPF>([&](auto bb) {
            if constexpr (bb < S::kBlocks) aread(bb);
          });
      }
      constexpr int li = S::layer_of(g);
      constexpr int lb = g - S::first_block(li);
      constexpr int t = lb / S::bpt(li);
      constexpr int kb = (lb % S::bpt(li)) / S::kAmul;
      constexpr int part = (lb % S::bpt(li)) % S::kAmul;     // bf16x3: 0 = W_hi, 1 = W_lo
      if constexpr (g + kPF < S::kBlocks) aread(std::integral_constant<int, g + kPF>{});
      // LDS reads return in order: wait for this block's fragment only
      constexpr int younger = (g + kPF < S::kBlocks ? g + kPF : S::kBlocks - 1) - g;
      asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(Abuf[g % (kPF + 1)]) : "n"(younger));
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Abuf[g % (kPF + 1)], __builtin_bit_cast(bf16x8, bin[kb]),
                                                      (BWD && kb == 0 && part == 0) ? f32x4{} : acc[t], 0, 0, 0);
      // bf16x3: W_hi x_lo after W_hi x_hi; the W_lo fragment multiplies x_hi
      if constexpr (kX3 && part == 0)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Abuf[g % (kPF + 1)], __builtin_bit_cast(bf16x8, binl[kb]),
                                                        acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(kSbMask);
      if constexpr (S::L(li).epi == EPI_RGB && g == S::last_block(li)) epilogue_rgb(a, acc, q, m);
      constexpr int ci = conv_layer_at(g);
      if constexpr (ci >= 0) {
        constexpr int t0 = conv_first_tile(ci, g);
        static_for<0, conv_tiles(ci, g)>([&](auto k) {
          constexpr int tt = t0 + k;
          if constexpr (!BWD) epi_tile_fwd<ci, tt>(a, bin, binl, acc, prm, q, slab, voff, sig_part, mk);
          else epi_tile_bwd<ci, tt>(a, bin, binl, acc, prm, smem, q, lane, w, slab, voff, ds);
        });
        if constexpr (!BWD && g == final_block(ci)) epi_final_fwd<ci>(a, bin, binl, prm, smem, lane, w, m, wg, sig_part, mk);
      }
    };
    static_for<0, kChunks>([&](auto cc) {
      static_for<0, kChunkBlocks>([&](auto bb) {
        constexpr int g = cc * kChunkBlocks + bb;
        if constexpr (g < S::kBlocks) block(std::integral_constant<int, g>{});
      });
    });
  }

  template <int C>
  __device__ static void issue(const ChainArgs& a, char* smem, int w, int lane) {
    const auto rs = mkrsrc(a.wpack);
    const uint32_t voffs = (uint32_t)(w * G * kBlockBytes + lane * 16);
    char* dst = smem + (C % NS) * kChunkBytes + w * G * kBlockBytes;
#pragma unroll
    for (int k = 0; k < G; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + k * kBlockBytes), 16, voffs,
                                               C * kChunkBytes + k * kBlockBytes, 0, 0);
  }

  // accumulator tile t <- bias of forward layer LI (rows 16 t + 4 q .. + 3)
  template <int LI>
  __device__ static void load_bias_tile(f32x4& acc, const float* prm, int q, int t) {
    acc = *(const f32x4*)(prm + LI * 256 + 16 * t + 4 * q);
  }

  // ---------------- prologues
  __device__ static void prologue_fwd(const ChainArgs& a, u32x4* bin, u32x4* binl, char* smem, int q, int lane,
                                      int w, int mc, int slab, const uint32_t* voff) {
    float x[3], d[3];
    if (a.mode == 0) {
      for (int k = 0; k < 3; ++k) { x[k] = a.xyz[3 * mc + k]; d[k] = a.vdir[3 * mc + k]; }
    } else {
      const int r = mc / a.nsamp;
      const int sm = mc - r * a.nsamp;
      const float z = a.zvals[r * a.z_stride + sm];
      for (int k = 0; k < 3; ++k) {
        d[k] = a.rays_d[3 * r + k];
        // xyz = ro + vd * z  (src/utils.py:30), no fused multiply-add
        x[k] = fadd_rn(a.rays_o[3 * r + k], fmul_rn(d[k], z));
      }
    }
    const int h = q & 1, qh = q >> 1;
    // this lane's PE columns: k-block u, jj -> 4 slots 4 mm .. 4 mm + 3 of
    // chain.hip's lane half h, mm = 4 u + 2 jj + qh (cn_layout.h
    // pe_slot_feature: slots 0 / 1 raw, then sin / cos pairs of argument
    // 15 h + k for slots 2 + 2k / 3 + 2k)
    auto arg = [&](const float* v, int p) { return (p % 3 == 0 ? v[0] : p % 3 == 1 ? v[1] : v[2]) * (float)(1 << (p / 3)); };
    auto scos = [&](float v, float& sn, float& cs) {
      if constexpr (kX3) sincosf(v, &sn, &cs);
      else sincos_turns(v, sn, cs);
    };
    float pe[2][2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int mm = 4 * u + 2 * jj;      // + qh (lane-dependent)
        float* o = pe[u][jj];
        if (mm == 0) {
          // qh = 0: slots 0-3 (raw pair + pair k = 0); qh = 1: slots 4-7 (pairs 1, 2)
          float sn0, cs0, sn1, cs1;
          scos(arg(x, 15 * h + (qh ? 1 : 0)), sn0, cs0);
          scos(arg(x, 15 * h + 2), sn1, cs1);
          const float r0 = h ? x[2] : x[0], r1 = h ? 0.f : x[1];
          o[0] = qh ? sn0 : r0;
          o[1] = qh ? cs0 : r1;
          o[2] = qh ? sn1 : sn0;
          o[3] = qh ? cs1 : cs0;
        } else {
          // slots 4 (mm + qh) .. +3: pairs k = 2 (mm + qh) - 1, 2 (mm + qh)
          const int k0 = 2 * (mm + qh) - 1;
          float sn0, cs0, sn1, cs1;
          scos(arg(x, 15 * h + k0), sn0, cs0);
          scos(arg(x, 15 * h + k0 + 1), sn1, cs1);
          o[0] = sn0; o[1] = cs0; o[2] = sn1; o[3] = cs1;
        }
      }
    // dir PE: slots 4 mm .. +3 of half h, mm = 2 jj + qh (dir_slot_feature:
    // half 0 args 0..6, half 1 args 7..11, the rest pad)
    float dp[2][4];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int mm = 2 * jj + qh;
      float* o = dp[jj];
      auto dpair = [&](int k, float& sn, float& cs) {
        const int p = h == 0 ? k : (k < 5 ? 7 + k : -1);
        sn = cs = 0.f;
        if (p >= 0) scos(arg(d, p), sn, cs);
      };
      if (mm == 0) {
        float sn, cs;
        dpair(0, sn, cs);
        o[0] = h ? d[2] : d[0];
        o[1] = h ? 0.f : d[1];
        o[2] = sn;
        o[3] = cs;
      } else {
        float sn0, cs0, sn1, cs1;
        dpair(2 * mm - 1, sn0, cs0);
        dpair(2 * mm, sn1, cs1);
        o[0] = sn0; o[1] = cs0; o[2] = sn1; o[3] = cs1;
      }
    }
    auto pk = [](const float* v0, const float* v1) {
      return u32x4{pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[0], v1[1]),
                   pack_bf16x2(v1[2], v1[3])};
    };
    auto lo4 = [](const float* v0, const float* v1, const u32x4& hi) {
      return u32x4{resid_bf16x2(v0[0], v0[1], hi[0]), resid_bf16x2(v0[2], v0[3], hi[1]),
                   resid_bf16x2(v1[0], v1[1], hi[2]), resid_bf16x2(v1[2], v1[3], hi[3])};
    };
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      bin[u] = pk(pe[u][0], pe[u][1]);
      if constexpr (kX3) binl[u] = lo4(pe[u][0], pe[u][1], bin[u]);
    }
    // the dir k-block is needed only by the viewdir layer: stash it in LDS
    char* stash = smem + kDirOff + (w * 64 + lane) * kDirStash;
    {
      const u32x4 dh = pk(dp[0], dp[1]);
      ((u32x4*)stash)[0] = dh;
      if constexpr (kX3) ((u32x4*)stash)[1] = lo4(dp[0], dp[1], dh);
    }
    if constexpr (PLANES) {
      const auto rp = slab_rsrc(a.pe, 64, slab);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) bstore64(rp, voff[jj], u32x2{bin[u][2 * jj], bin[u][2 * jj + 1]}, u * 2048);
      const auto rd = slab_rsrc(a.dir, 32, slab);
      const u32x4 dh = ((const u32x4*)stash)[0];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) bstore64(rd, voff[jj], u32x2{dh[2 * jj], dh[2 * jj + 1]});
      if constexpr (kXlo) {
        // the PE operand's lo parts (the dir-PE tile of encoding_viewdir's dW
        // stays hi only: dw.hip)
        const auto rpl = slab_rsrc(a.pelo, 64, slab);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            bstore64(rpl, voff[jj], u32x2{binl[u][2 * jj], binl[u][2 * jj + 1]}, u * 2048);
      }
    }
  }

  __device__ static float prologue_bwd(const ChainArgs& a, u32x4* bin, u32x4* binl, char* smem, int q, int lane,
                                       int w, int m, int mc, int wg, int slab, const uint32_t* voff) {
    // padding samples (m >= M) get zero upstream gradients, so every dA they
    // write is exactly 0 and the dW pass can sum whole 32-sample tiles
    const bool valid = m < a.M;
    const float g0 = valid ? a.drgb[3 * mc + 0] : 0.f;
    const float g1 = valid ? a.drgb[3 * mc + 1] : 0.f;
    const float g2 = valid ? a.drgb[3 * mc + 2] : 0.f;
    // Softplus backward exactly as torch: grad * (x > 20 ? 1 : e^x / (e^x + 1))
    const float sp = a.spre[mc];
    const float ex = expf(sp);
    const float ds = valid ? a.dsigma[mc] * (sp > 20.f ? 1.f : ex / (ex + 1.f)) : 0.f;
    // k-block 0: slots (q = 0, j = 0..2) = drgb components 0..2
    if (q == 0) {
      bin[0] = u32x4{pack_bf16x2(g0, g1), pack_bf16x2(g2, 0.f), 0u, 0u};
      if constexpr (kX3) binl[0] = u32x4{resid_bf16x2(g0, g1, bin[0][0]), resid_bf16x2(g2, 0.f, bin[0][1]), 0u, 0u};
    }
    if constexpr (PLANES) {
      // drgb as a padded 32-wide plane for the rgb-head weight gradient
      const auto r8 = slab_rsrc(a.d8, 32, slab);
      const uint32_t z0 = q == 0 ? pack_bf16x2(g0, g1) : 0u, z1 = q == 0 ? pack_bf16x2(g2, 0.f) : 0u;
      bstore64(r8, voff[0], u32x2{z0, z1});
      bstore64(r8, voff[1], u32x2{0u, 0u});
      // the sigma-head gradient rides in columns 256 (value) and 257 (its
      // rounding residual) of the viewdir dA plane (288 columns)
      const auto rv = slab_rsrc(a.dA[SB + 2], 288, slab);
      const float ds_hi = (float)(__bf16)ds;
      const uint32_t v0 = q == 0 ? pack_bf16x2(ds_hi, ds - ds_hi) : 0u;
      bstore64(rv, voff[0], u32x2{v0, 0u}, 8 * 2048);
      bstore64(rv, voff[1], u32x2{0u, 0u}, 8 * 2048);
    }
    // ReLU sign bits of this wave -> LDS (8 B per lane per layer)
    const u32x2* src = (const u32x2*)(a.masks) + (size_t)wg * N::kMasks * 64 + lane;
    u32x2* dst = (u32x2*)(smem + kMaskOff + w * kMaskWave) + lane;
#pragma unroll
    for (int k = 0; k < N::kMasks; ++k) dst[k * 64] = src[k * 64];
    return ds;
  }

  // buffer descriptor of a 32-sample slab of a bf16 plane of width F
  CN_DEV static __amdgpu_buffer_rsrc_t slab_rsrc(const void* plane, int F, int slab) {
    return mkrsrc((const char*)plane + (size_t)slab * (size_t)F * 64u);
  }

  // ---------------- epilogues
  // mask bits of a layer: tile t (value i) -> dword t >> 3; elements 0 / 2 in
  // the low half, 1 / 3 in the high half, pushed oldest-highest in the order
  // Q = 2 (t & 7) + i / 2, so that ONE shift by Q brings a pair's two bits
  // to 15 and 31 (relu_mask_bf16x2, chain.hip)
  template <int LI, int TT>
  __device__ static void epi_tile_fwd(const ChainArgs& a, u32x4* bin, u32x4* binl, f32x4* acc, const float* prm,
                                      int q, int slab, const uint32_t* voff, float& sig_part, MaskAcc& mk) {
    constexpr Layer l = S::L(LI);
    constexpr int t = TT;
    static_assert(LI + 1 >= NL || S::tiles(LI + 1) <= S::tiles(LI), "next layer wider than this one");
    if constexpr (t == 0) { mk.lo[0] = mk.hi[0] = mk.lo[1] = mk.hi[1] = 0u; }
    float v0 = acc[t][0], v1 = acc[t][1], v2 = acc[t][2], v3 = acc[t][3];
    if constexpr (TRAIN && l.mask >= 0) {
      mk.lo[t >> 3] = push_sign(push_sign(mk.lo[t >> 3], v0), v2);
      mk.hi[t >> 3] = push_sign(push_sign(mk.hi[t >> 3], v1), v3);
    }
    if constexpr (l.epi == EPI_SHAPE) {
      const f32x4 w4 = *(const f32x4*)(prm + kWsOff + 16 * t + 4 * q);
      sig_part = __builtin_fmaf(w4[0], v0, sig_part);
      sig_part = __builtin_fmaf(w4[1], v1, sig_part);
      sig_part = __builtin_fmaf(w4[2], v2, sig_part);
      sig_part = __builtin_fmaf(w4[3], v3, sig_part);
    }
    if constexpr (kX3 && l.epi == EPI_RELU) {
      v0 = relu_f32(v0); v1 = relu_f32(v1); v2 = relu_f32(v2); v3 = relu_f32(v3);
    }
    uint32_t p0 = pack_bf16x2(v0, v1), p1 = pack_bf16x2(v2, v3);
    if constexpr (!kX3 && l.epi == EPI_RELU) { p0 = relu_bf16x2(p0); p1 = relu_bf16x2(p1); }
    u32x4& b = bin[t >> 1];
    if constexpr ((t & 1) == 0) { b[0] = p0; b[1] = p1; } else { b[2] = p0; b[3] = p1; }
    uint32_t l0 = 0u, l1 = 0u;
    if constexpr (kX3) {
      l0 = resid_bf16x2(v0, v1, p0);
      l1 = resid_bf16x2(v2, v3, p1);
      u32x4& bl = binl[t >> 1];
      if constexpr ((t & 1) == 0) { bl[0] = l0; bl[1] = l1; } else { bl[2] = l0; bl[3] = l1; }
    }
    if constexpr (plane_of(LI)) {
      constexpr int yp = l.plane;
      bstore64(slab_rsrc(a.Y[yp], N::plane_width(yp), slab), voff[t & 1], u32x2{p0, p1}, (t >> 1) * 2048);
      if constexpr (kXlo)
        bstore64(slab_rsrc(a.Ylo[yp], N::plane_width(yp), slab), voff[t & 1], u32x2{l0, l1}, (t >> 1) * 2048);
    }
    // this tile's accumulator starts the next layer's tile t
    if constexpr (t < S::tiles(LI + 1)) load_bias_tile<LI + 1>(acc[t], prm, q, t);
  }

  template <int LI>
  __device__ static void epi_final_fwd(const ChainArgs& a, u32x4* bin, u32x4* binl, const float* prm,
                                       const char* smem, int lane, int w, int m, int wg, float& sig_part,
                                       MaskAcc& mk) {
    constexpr Layer l = S::L(LI);
    if constexpr (TRAIN && l.mask >= 0) {
      const uint32_t m0 = (mk.hi[0] << 16) | (mk.lo[0] & 0xFFFFu);
      const uint32_t m1 = (mk.hi[1] << 16) | (mk.lo[1] & 0xFFFFu);
      bstore64(mkrsrc(a.masks + (size_t)wg * N::kMasks * 128), ((uint32_t)l.mask * 64 + lane) * 8, u32x2{m0, m1});
    }
    if constexpr (l.epi == EPI_SHAPE) {
      float tot = sig_part + __shfl_xor(sig_part, 16);
      tot = tot + __shfl_xor(tot, 32);
      const float pre = tot + prm[kMiscOff];
      // all four lane groups hold the full sum: every lane stores (same value,
      // same address), so the store count per wave is fixed for vmcnt
      bstore32(mkrsrc(a.sigma), (uint32_t)m * 4, f2u(softplus20(pre)));
      if constexpr (TRAIN) bstore32(mkrsrc(a.spre), (uint32_t)m * 4, f2u(pre));
    }
    // the next layer (viewdir) takes the dir k-block from the LDS stash
    if constexpr (S::L(LI + 1).in_kind == IN_ACC_DIR) {
      const char* stash = smem + kDirOff + (w * 64 + lane) * kDirStash;
      bin[8] = ((const u32x4*)stash)[0];
      if constexpr (kX3) binl[8] = ((const u32x4*)stash)[1];
    }
  }

  __device__ static void epilogue_rgb(const ChainArgs& a, const f32x4* acc, int q, int m) {
    if (q == 0) {
      a.rgb[3 * m + 0] = acc[0][0];
      a.rgb[3 * m + 1] = acc[0][1];
      a.rgb[3 * m + 2] = acc[0][2];
    }
  }

  template <int LI, int TT>
  __device__ static void epi_tile_bwd(const ChainArgs& a, u32x4* bin, u32x4* binl, f32x4* acc, const float* prm,
                                      const char* smem, int q, int lane, int w, int slab, const uint32_t* voff,
                                      float ds) {
    constexpr Layer l = S::L(LI);
    constexpr int t = TT;
    float v0 = acc[t][0], v1 = acc[t][1], v2 = acc[t][2], v3 = acc[t][3];
    if constexpr (l.epi == EPI_BSIGMA) {
      const f32x4 w4 = *(const f32x4*)(prm + kWsOff + 16 * t + 4 * q);
      v0 = fadd_rn(v0, fmul_rn(ds, w4[0]));
      v1 = fadd_rn(v1, fmul_rn(ds, w4[1]));
      v2 = fadd_rn(v2, fmul_rn(ds, w4[2]));
      v3 = fadd_rn(v3, fmul_rn(ds, w4[3]));
    }
    uint32_t p0 = pack_bf16x2(v0, v1), p1 = pack_bf16x2(v2, v3);
    uint32_t l0 = 0u, l1 = 0u;
    if constexpr (kX3) { l0 = resid_bf16x2(v0, v1, p0); l1 = resid_bf16x2(v2, v3, p1); }
    if constexpr (l.epi == EPI_BMASK) {
      const uint32_t mw = *(const uint32_t*)(smem + kMaskOff + w * kMaskWave + (l.mask * 64 + lane) * 8 + 4 * (t >> 3));
      p0 = relu_mask_bf16x2<2 * (t & 7)>(p0, mw);
      p1 = relu_mask_bf16x2<2 * (t & 7) + 1>(p1, mw);
      if constexpr (kX3) {
        l0 = relu_mask_bf16x2<2 * (t & 7)>(l0, mw);
        l1 = relu_mask_bf16x2<2 * (t & 7) + 1>(l1, mw);
      }
    }
    u32x4& b = bin[t >> 1];
    if constexpr ((t & 1) == 0) { b[0] = p0; b[1] = p1; } else { b[2] = p0; b[3] = p1; }
    if constexpr (kX3) {
      u32x4& bl = binl[t >> 1];
      if constexpr ((t & 1) == 0) { bl[0] = l0; bl[1] = l1; } else { bl[2] = l0; bl[3] = l1; }
    }
    if constexpr (plane_of(LI)) {
      constexpr int p = l.plane;
      bstore64(slab_rsrc(a.dA[p], N::dplane_width(p), slab), voff[t & 1], u32x2{p0, p1}, (t >> 1) * 2048);
    }
  }
};

// 8-wave workgroups, two waves per SIMD (256 registers each)
template <int P, int SB, int TB, bool BWD, int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64, WAVES / 4) void chain16_kernel(ChainArgs a) {
  Chain16<P, SB, TB, BWD, WAVES, MODE>::run(a);
}

}  // namespace cn
