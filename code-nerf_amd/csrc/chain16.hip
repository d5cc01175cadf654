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
  // waves that issue the weight stream's LDS-DMA: all of them when WAVES
  // divides a chunk; of a 12-wave workgroup, waves 0-7 (2 blocks each)
  static constexpr int kIssuers = kChunkBlocks % WAVES == 0 ? WAVES : 8;
  static_assert(kChunkBlocks % kIssuers == 0, "issuing waves must divide a chunk");
  static constexpr int G = kChunkBlocks / kIssuers;        // LDS-DMA instructions per issuing wave per chunk
  // chunks in flight: a 16 KiB chunk feeds one wave 8 (bf16x3: 24) MFMAs of
  // 16 cycles, two or three waves per SIMD; ~1.1 us from LDS-DMA issue to
  // landing (a 12-wave backward keeps 4: its mask words take the LDS)
  static constexpr int D = (kX3 && !(BWD && WAVES > 8)) ? 5 : 4;
  static constexpr int NS = D + 2;                         // ring slots (see chain.hip)
  // A-fragment prefetch distance (blocks): 12-wave workgroups (three waves
  // per SIMD hide the LDS latency) read the forward's fragments in place and
  // the backward's one block ahead, which keeps them within the 168
  // registers of three waves
  static constexpr int kPF = WAVES > 8 ? (BWD ? 1 : 0) : 3;
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
  // ---------------- epilogue schedule: the tile pipeline (round 5).  Tile t
  // of layer i is converted (ReLU, mask bits, hi / lo split, plane stores)
  // after the SECOND block of tile t + 1 of the same layer -- the last tile
  // after the second block of the next layer's first tile -- so its VALU
  // issues among tile t + 1's MFMAs, evenly over the layer, instead of as
  // bursts at layer boundaries (a 16x16x32 MFMA leaves the vector issue free
  // for only 8 of its 16 cycles: the round-5 counters put the chains at
  // MFMA busy 0.65 with 0.02 MFMA / VALU co-execution when every tile of a
  // layer was converted inside the next layer's first tile).  A layer reads
  // its input k-blocks from one operand array and writes its output tiles
  // into the other (X[i & 1] -> X[(i & 1) ^ 1]); two accumulator tiles are
  // live (acc[t & 1]).
  static constexpr bool converts(int i) { return S::L(i).epi != EPI_RGB; }
  static constexpr int tile_first(int i, int t) { return S::first_block(i) + t * S::bpt(i); }
  // (the backward's last layer, with no next layer: its last tile at its own
  // last block)
  static constexpr int conv_block(int i, int t) {
    return t + 1 < S::tiles(i) ? tile_first(i, t + 1) + (S::bpt(i) > 1 ? 1 : 0)
           : i + 1 < NL        ? S::first_block(i + 1) + (S::bpt(i + 1) > 1 ? 1 : 0)
                               : S::last_block(i);
  }
  static constexpr int final_block(int i) { return conv_block(i, S::tiles(i) - 1); }
  static constexpr bool sched_ok() {
    for (int i = 0; i < NL; ++i) {
      if (!converts(i)) continue;
      const int T = S::tiles(i);
      if (T % 2) return false;                            // acc[t & 1] hand-over to the next layer
      // the last tile is converted before the next layer reads its k-block
      if (i + 1 < NL && final_block(i) >= S::first_block(i + 1) + ((T - 1) >> 1) * S::kAmul) return false;
      // and before tile t + 2 reuses its accumulator
      for (int t = 0; t < T; ++t) {
        if (t + 2 < T && conv_block(i, t) >= tile_first(i, t + 2)) return false;
        if (conv_at(conv_block(i, t)) != 64 * i + t) return false;      // conv_at inverts conv_block
      }
    }
    return true;
  }
  // (layer, tile) converted after block g: 64 layer + tile, or -1 (the
  // inverse of conv_block, cheap enough for the vmcnt bookkeeping's
  // compile-time loops)
  static constexpr int conv_at(int g) {
    const int li = S::layer_of(g), lb = g - S::first_block(li);
    const int tn = lb / S::bpt(li), r = lb % S::bpt(li), r1 = S::bpt(li) > 1 ? 1 : 0;
    if (r == r1 && tn >= 1 && converts(li)) return 64 * li + tn - 1;
    if (r == r1 && tn == 0 && li >= 1 && converts(li - 1)) return 64 * (li - 1) + S::tiles(li - 1) - 1;
    if (li == NL - 1 && g == S::last_block(li) && converts(li)) return 64 * li + S::tiles(li) - 1;
    return -1;
  }
  static_assert(sched_ok(), "tile pipeline schedule");

  // ---------------- LDS read groups.  Every LDS read inside the block loop is
  // an explicit ds_read whose lgkmcnt wait is counted at compile time, so the
  // compiler (which would wait lgkmcnt(0) behind a read it can see, draining
  // every fragment prefetch in flight) emits none.  Group x -- issued kPF
  // blocks before block x -- reads, in order: block x's A fragment; the bias
  // tile when x starts a forward output tile (the MFMA's C operand); the
  // sigma-head weights when the tile converted after block x needs them
  // (encoding_shape forward, encoding_viewdir backward); the mask word when a
  // backward tile converted after block x is masked.
  static constexpr int tile_of(int g) { return (g - S::first_block(S::layer_of(g))) / S::bpt(S::layer_of(g)); }
  static constexpr bool has_bias(int x) {
    return !BWD && (x - S::first_block(S::layer_of(x))) % S::bpt(S::layer_of(x)) == 0;
  }
  static constexpr bool has_ws(int x) {
    const int c = conv_at(x);
    return c >= 0 && S::L(c / 64).epi == (BWD ? EPI_BSIGMA : EPI_SHAPE);
  }
  static constexpr bool has_mask(int x) { const int c = conv_at(x); return BWD && c >= 0 && S::L(c / 64).epi == EPI_BMASK; }
  static constexpr int group_reads(int x) {
    return x < 0 || x >= S::kBlocks ? 0 : 1 + has_bias(x) + has_ws(x) + has_mask(x);
  }
  // reads issued after group g's last one, up to group g + kPF (issued by the
  // time block g runs)
  static constexpr int reads_after(int g) {
    int n = 0;
    for (int x = g + 1; x <= g + kPF; ++x) n += group_reads(x);
    return n;
  }
  // ---------------- compile-time vmcnt bookkeeping
  // a mask word (8 tiles' sign bits) is stored as soon as its last tile is
  // converted, so only one word's accumulators are live
  static constexpr bool mask_store_at(int i, int t) {
    return !BWD && TRAIN && S::L(i).mask >= 0 && ((t & 7) == 7 || t == S::tiles(i) - 1);
  }
  static constexpr int tile_stores(int i, int t) {
    return (plane_of(i) ? (kXlo ? 2 : 1) : 0) + (mask_store_at(i, t) ? 1 : 0);
  }
  static constexpr int final_stores(int i) {
    if (BWD) return 0;
    return S::L(i).epi == EPI_SHAPE ? (TRAIN ? 2 : 1) : 0;
  }
  // VMEM stores issued right after block g's MFMAs (the rgb head's come after
  // the last wait point: not counted)
  static constexpr int stores_at_block(int g) {
    const int c = conv_at(g);
    if (c < 0) return 0;
    const int ci = c / 64, t = c % 64;
    return tile_stores(ci, t) + (t == S::tiles(ci) - 1 ? final_stores(ci) : 0);
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
    uint32_t lo, hi;
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
    // its 32-sample plane slab, or -1 past the padded rows (a 12-wave
    // workgroup's 192 samples do not divide the 256-sample pad granule):
    // such a wave runs the schedule (barriers, weight DMA) but every store
    // of it is discarded (empty buffer range) and it reads clamped inputs
    const int nslab = ((a.M + 255) >> 8) << 3;
    const int slab = (wg >> 1) < nslab ? (wg >> 1) : -1;
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

    // the two operand arrays (hi; bf16x3 also lo) of the tile pipeline
    u32x4 X[2][kBin];
    u32x4 XL[2][kX3 ? kBin : 1];
    f32x4 acc[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      acc[k] = f32x4{};
#pragma unroll
      for (int u = 0; u < kBin; ++u) X[k][u] = u32x4{};
      if constexpr (kX3)
#pragma unroll
        for (int u = 0; u < kBin; ++u) XL[k][u] = u32x4{};
    }

    float ds = 0.f;
    if constexpr (!BWD) prologue_fwd(a, X[0], XL[0], smem, q, lane, w, mc, slab, voff);
    else ds = prologue_bwd(a, X[0], XL[0], smem, q, lane, w, m, mc, slab >= 0 ? wg : 2 * nslab - 1, slab, voff);
    __syncthreads();

    static_for<0, D>([&](auto i) { issue<i>(a, smem, w, lane); });

    float sig_part = 0.f;
    MaskAcc mk;
    bf16x8 Abuf[kPF + 1];
    f32x4 Bbuf[2], Wbuf[2];         // bias tiles (by tile parity), sigma-head weights (by converted tile parity)
    uint32_t Mbuf[2];               // mask words (by converted tile parity)
    const uint32_t lbase = lds_addr(smem) + lane * 16;
    const uint32_t pbase = lds_addr(prm) + q * 16;    // this lane group's 4 rows of a bias / weight tile
    const uint32_t mbase = lds_addr(smem + kMaskOff + w * kMaskWave) + lane * 8;
    auto block_off = [](int b) { return (b / kChunkBlocks % NS) * kChunkBytes + (b % kChunkBlocks) * kBlockBytes; };
    auto aread = [&](auto bbc) {
      constexpr int b = bbc;
      constexpr int off = block_off(b);
      u32x4 r;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(lbase + (off & ~0xFFFF)), "n"(off & 0xFFFF));
      Abuf[b % (kPF + 1)] = __builtin_bit_cast(bf16x8, r);
    };
    auto pread = [&](f32x4& dst, auto offc) {       // 16 B of the bias blob at float offset off (+ 4 q)
      constexpr int off = 4 * decltype(offc)::value;
      f32x4 r;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(pbase + (off & ~0xFFFF)), "n"(off & 0xFFFF));
      dst = r;
    };
    // the side reads of group x (after its A fragment: aread)
    auto side = [&](auto xc) {
      constexpr int x = xc;
      if constexpr (has_bias(x)) {
        constexpr int li = S::layer_of(x), t = tile_of(x);
        pread(Bbuf[t & 1], std::integral_constant<int, li * 256 + 16 * t>{});
      }
      constexpr int c = conv_at(x);
      if constexpr (has_ws(x))
        pread(Wbuf[(c % 64) & 1], std::integral_constant<int, kWsOff + 16 * (c % 64)>{});
      if constexpr (has_mask(x)) {
        constexpr int off = (S::L(c / 64).mask * 64) * 8 + 4 * ((c % 64) >> 3);
        uint32_t r;
        asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(mbase), "n"(off));
        Mbuf[(c % 64) & 1] = r;
      }
    };
    auto group = [&](auto xc) {
      aread(xc);
      side(xc);
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
            if constexpr (bb < S::kBlocks) group(bb);
          });
      }
      constexpr int li = S::layer_of(g);
      constexpr int lb = g - S::first_block(li);
      constexpr int t = lb / S::bpt(li);
      constexpr int kb = (lb % S::bpt(li)) / S::kAmul;
      constexpr int part = (lb % S::bpt(li)) % S::kAmul;     // bf16x3: 0 = W_hi, 1 = W_lo
      if constexpr (g + kPF < S::kBlocks) group(std::integral_constant<int, g + kPF>{});
      // LDS reads return in order: wait for this block's fragment (and bias)
      // only -- the reads of group g after them and of the later groups may
      // still be in flight
      constexpr int pin = li & 1;
      constexpr bool first = !BWD && kb == 0 && part == 0;
      constexpr int younger = reads_after(g) + has_ws(g) + has_mask(g);
      if constexpr (first)
        asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(Abuf[g % (kPF + 1)]), "+v"(Bbuf[t & 1]) : "n"(younger));
      else
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(Abuf[g % (kPF + 1)]) : "n"(younger));
      f32x4& ac = acc[t & 1];
      ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Abuf[g % (kPF + 1)], __builtin_bit_cast(bf16x8, X[pin][kb]),
                                                  (BWD && kb == 0 && part == 0) ? f32x4{} : first ? Bbuf[t & 1] : ac,
                                                  0, 0, 0);
      // bf16x3: W_hi x_lo after W_hi x_hi; the W_lo fragment multiplies x_hi
      if constexpr (kX3 && part == 0)
        ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Abuf[g % (kPF + 1)], __builtin_bit_cast(bf16x8, XL[pin][kb]),
                                                    ac, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(kSbMask);
      if constexpr (S::L(li).epi == EPI_RGB && g == S::last_block(li)) epilogue_rgb(a, acc[0], q, m, slab);
      constexpr int c = conv_at(g);
      if constexpr (c >= 0) {
        constexpr int ci = c / 64, tt = c % 64, po = (ci & 1) ^ 1;
        // the side reads of group g: every read of group g before them
        // returned, the later groups' may be in flight
        if constexpr (has_ws(g) && has_mask(g))
          asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(Wbuf[tt & 1]), "+v"(Mbuf[tt & 1]) : "n"(reads_after(g)));
        else if constexpr (has_ws(g))
          asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(Wbuf[tt & 1]) : "n"(reads_after(g)));
        else if constexpr (has_mask(g))
          asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(Mbuf[tt & 1]) : "n"(reads_after(g)));
        if constexpr (!BWD) {
          epi_tile_fwd<ci, tt>(a, X[po], XL[po], acc[tt & 1], Wbuf[tt & 1], q, lane, wg, slab, voff, sig_part, mk);
          if constexpr (tt == S::tiles(ci) - 1)
            epi_final_fwd<ci>(a, X[po], XL[po], prm, smem, lane, w, m, wg, slab, sig_part, mk);
        } else {
          epi_tile_bwd<ci, tt>(a, X[po], XL[po], acc[tt & 1], Wbuf[tt & 1], Mbuf[tt & 1], slab, voff, ds);
        }
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
    // (non-issuing waves have no LDS-DMA to wait for: their counted vmcnt
    // waits, sized for G DMAs per chunk, only relax towards their own stores)
    if (kIssuers < WAVES && w >= kIssuers) return;
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

  // buffer descriptor of a 32-sample slab of a bf16 plane of width F (slab
  // -1: an empty range, every store discarded)
  CN_DEV static __amdgpu_buffer_rsrc_t slab_rsrc(const void* plane, int F, int slab) {
    return mkrsrc((const char*)plane + (size_t)(slab >= 0 ? slab : 0) * (size_t)F * 64u, slab >= 0);
  }

  // ---------------- epilogues
  // mask bits of a layer: tile t (value i) -> dword t >> 3; elements 0 / 2 in
  // the low half, 1 / 3 in the high half, pushed oldest-highest in the order
  // Q = 2 (t & 7) + i / 2, so that ONE shift by Q brings a pair's two bits
  // to 15 and 31 (relu_mask_bf16x2, chain.hip)
  template <int LI, int TT>
  __device__ static void epi_tile_fwd(const ChainArgs& a, u32x4* bin, u32x4* binl, f32x4& ac, const f32x4& w4,
                                      int q, int lane, int wg, int slab, const uint32_t* voff, float& sig_part,
                                      MaskAcc& mk) {
    constexpr Layer l = S::L(LI);
    constexpr int t = TT;
    if constexpr ((t & 7) == 0) { mk.lo = mk.hi = 0u; }
    float v0 = ac[0], v1 = ac[1], v2 = ac[2], v3 = ac[3];
    if constexpr (TRAIN && l.mask >= 0) {
      mk.lo = push_sign(push_sign(mk.lo, v0), v2);
      mk.hi = push_sign(push_sign(mk.hi, v1), v3);
    }
    if constexpr (mask_store_at(LI, t)) {
      // word t >> 3 of this lane's 8 B per layer (a layer of <= 8 tiles: word
      // 1 written as 0, as one 8-B store)
      const uint32_t mw = (mk.hi << 16) | (mk.lo & 0xFFFFu);
      const auto rm = mkrsrc(a.masks + (size_t)wg * N::kMasks * 128, slab >= 0);
      const uint32_t off = ((uint32_t)l.mask * 64 + lane) * 8;
      if constexpr (S::tiles(LI) <= 8) bstore64(rm, off, u32x2{mw, 0u});
      else bstore32(rm, off + 4 * (t >> 3), mw);
    }
    if constexpr (l.epi == EPI_SHAPE) {
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
  }

  template <int LI>
  __device__ static void epi_final_fwd(const ChainArgs& a, u32x4* bin, u32x4* binl, const float* prm,
                                       const char* smem, int lane, int w, int m, int wg, int slab,
                                       float& sig_part, MaskAcc& mk) {
    constexpr Layer l = S::L(LI);
    if constexpr (l.epi == EPI_SHAPE) {
      float tot = sig_part + __shfl_xor(sig_part, 16);
      tot = tot + __shfl_xor(tot, 32);
      const float pre = tot + prm[kMiscOff];
      // all four lane groups hold the full sum: every lane stores (same value,
      // same address), so the store count per wave is fixed for vmcnt
      bstore32(mkrsrc(a.sigma, slab >= 0), (uint32_t)m * 4, f2u(softplus20(pre)));
      if constexpr (TRAIN) bstore32(mkrsrc(a.spre, slab >= 0), (uint32_t)m * 4, f2u(pre));
    }
    // the next layer (viewdir) takes the dir k-block from the LDS stash
    if constexpr (S::L(LI + 1).in_kind == IN_ACC_DIR) {
      const char* stash = smem + kDirOff + (w * 64 + lane) * kDirStash;
      bin[8] = ((const u32x4*)stash)[0];
      if constexpr (kX3) binl[8] = ((const u32x4*)stash)[1];
    }
  }

  __device__ static void epilogue_rgb(const ChainArgs& a, const f32x4& acc, int q, int m, int slab) {
    if (q == 0 && slab >= 0) {
      a.rgb[3 * m + 0] = acc[0];
      a.rgb[3 * m + 1] = acc[1];
      a.rgb[3 * m + 2] = acc[2];
    }
  }

  template <int LI, int TT>
  __device__ static void epi_tile_bwd(const ChainArgs& a, u32x4* bin, u32x4* binl, const f32x4& ac, const f32x4& w4,
                                      uint32_t mw, int slab, const uint32_t* voff, float ds) {
    constexpr Layer l = S::L(LI);
    constexpr int t = TT;
    float v0 = ac[0], v1 = ac[1], v2 = ac[2], v3 = ac[3];
    if constexpr (l.epi == EPI_BSIGMA) {
      v0 = fadd_rn(v0, fmul_rn(ds, w4[0]));
      v1 = fadd_rn(v1, fmul_rn(ds, w4[1]));
      v2 = fadd_rn(v2, fmul_rn(ds, w4[2]));
      v3 = fadd_rn(v3, fmul_rn(ds, w4[3]));
    }
    uint32_t p0 = pack_bf16x2(v0, v1), p1 = pack_bf16x2(v2, v3);
    uint32_t l0 = 0u, l1 = 0u;
    if constexpr (kX3) { l0 = resid_bf16x2(v0, v1, p0); l1 = resid_bf16x2(v2, v3, p1); }
    if constexpr (l.epi == EPI_BMASK) {
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
