// Fused CodeNeRF MLP chain kernels for gfx950 (forward and dX-backward).
//
// Replaces CodeNeRF.forward (reference src/model.py:36-53) and the dX part of
// its autograd backward (src/trainer.py:82) for a whole batch of samples in
// ONE launch each:
//
//   * a wave owns 32 samples for the whole chain; every activation lives in
//     registers (accumulator = next layer's B operand, see cn_layout.h);
//   * positional encoding (src/model.py:4-7) is computed in registers from the
//     sample position (or from ray origin/direction/z: src/utils.py:30);
//   * weights stream through a 4-slot LDS ring of 16 KiB chunks filled by
//     LDS-DMA (global_load_lds_dwordx4) 3 chunks ahead of use and shared by
//     all waves of the workgroup; one raw s_barrier per chunk and a counted
//     `s_waitcnt vmcnt(N)` whose N is computed at compile time from the static
//     schedule (including the epilogue stores issued in between);
//   * biases are the accumulators' initial value; the latent-code injection
//     y + z_j (src/model.py:41-43,49-51) is folded into a per-object bias
//     b_j + W_j z_j computed once per call (latent.hip);
//   * ReLU, the sigma head (Softplus, threshold 20) and the rgb head are fused
//     into the layer epilogues; for training the epilogues also write the
//     layer outputs (for dW) and one sign bit per pre-activation (ReLU mask
//     for the dX chain) with a single v_alignbit per value.
#pragma once
#include "cn_common.h"
#include "cn_sched.h"
#include "chain_args.h"

namespace cn {

template <int P> struct PT;
template <> struct PT<CN_P_BF16> {
  using E = __bf16;
  using BinT = u32x4;            // 8 bf16 packed in 4 dwords (one MFMA B operand)
  static constexpr int kBin = 18;
};
template <> struct PT<CN_P_BF16X3> : PT<CN_P_BF16> {};
template <> struct PT<CN_P_FP32> {
  using E = float;
  using BinT = float;            // one v_mfma_f32_32x32x2_f32 B operand
  static constexpr int kBin = 144;
};

// Two floats -> packed bf16 pair (round to nearest even) in ONE
// v_cvt_pk_bf16_f32: a vector conversion of a float2.  Built from two scalar
// conversions (bf16x2{(__bf16)lo, (__bf16)hi}) the compiler emitted, in the
// epilogues, one conversion per element against a zero plus a v_perm_b32
// (3 VALU instead of 1).
CN_DEV uint32_t pack_bf16x2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}
// bf16x3: the residual pair rn(lo - hi_lo), rn(hi - hi_hi) of a packed pair
// p = pack_bf16x2(lo, hi) -- the operand's lo part (x - rn(x) is exact in
// fp32, so x_hi + x_lo carries 16 significant bits)
CN_DEV uint32_t resid_bf16x2(float lo, float hi, uint32_t p) {
  const float rl = lo - __builtin_bit_cast(float, p << 16);
  const float rh = hi - __builtin_bit_cast(float, p & 0xFFFF0000u);
  return pack_bf16x2(rl, rh);
}
// ReLU of one fp32 as a signed-int32 max with 0 (one v_max_i32; fmaxf
// compiles to a canonicalising max plus the max)
CN_DEV float relu_f32(float v) {
  return __builtin_bit_cast(float, __builtin_elementwise_max(__builtin_bit_cast(int, v), 0));
}
// ReLU of two packed bf16: signed-int16 max with 0 (negative and -0 -> +0)
CN_DEV uint32_t relu_bf16x2(uint32_t x) {
  typedef __attribute__((ext_vector_type(2))) short s16x2;
  s16x2 v = __builtin_bit_cast(s16x2, x);
  v = __builtin_elementwise_max(v, s16x2{0, 0});
  return __builtin_bit_cast(uint32_t, v);
}
// ReLU backward from the stored sign bits (bit set -> pre-activation < 0 ->
// gradient 0).  fp32: one element.  bf16: a packed pair (elements at bit
// positions pa (low half) and pb (high half)) masked AFTER packing: the
// 16-bit halves of the mask are built with one v_bfi_b32 and applied with one
// v_and_b32 -- a plain AND on a packed word, which the compiler cannot turn
// into the v_cmp + v_cndmask (+ VCC hazard nop) it emits for a per-element
// masked select.  Masking before or after the bf16 rounding is the same.
CN_DEV float relu_mask(float v, uint32_t word, int pos) {
  const uint32_t off = (uint32_t)__builtin_amdgcn_sbfe((int)word, pos, 1);
  return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) & ~off);
}
// Mask word layout (written by the forward epilogue, mask_bit below): the two
// elements of a packed pair sit 16 bits apart, at bits 15 - q and 31 - q, so
// ONE shift by q brings them to bits 15 and 31, and ONE v_perm_b32 (byte
// selectors 8 / 9 replicate bits 15 / 31 of its low source) expands them into
// the pair's 16-bit halves: 3 VALU per pair with the AND-NOT, all
// compiler-visible.
template <int Q>
CN_DEV uint32_t relu_mask_bf16x2(uint32_t p, uint32_t word) {
  const uint32_t w = word << Q;
  const uint32_t m2 = __builtin_amdgcn_perm(w, w, 0x09090808u);
  return p & ~m2;
}
// sin and cos of v (radians) on the transcendental unit, for the bf16 path's
// positional encoding: v / 2 pi in turns with a two-term constant (the
// product's rounding error recovered by FMA), whole turns removed exactly by
// v_fract_f32, then v_sin_f32 / v_cos_f32 (input in turns).  Absolute error
// ~1e-6 at the largest argument (2^9 |x| ~ 1e3 rad), against the 2^-9
// relative rounding the bf16 operand applies next; the fp32 parity path and
// bf16x3 keep the correctly rounded sincosf (with the hardware sincos,
// bf16x3's one-object training trajectory left the fp32 replay by 0.093 dB
// at step 19 instead of 0.061 dB by step 26: tests/test_gpu_converge.py).
CN_DEV void sincos_turns(float v, float& s, float& c) {
  constexpr float kHi = 0.15915493667125702f, kLo = 6.4206382432985265e-09f;
  const float t = v * kHi;
  float e = __builtin_fmaf(v, kHi, -t);
  e = __builtin_fmaf(v, kLo, e);
  const float u = __builtin_amdgcn_fractf(t) + e;
  s = __builtin_amdgcn_sinf(u);
  c = __builtin_amdgcn_cosf(u);
}

// shift the sign bit of v into the running mask word (one v_alignbit_b32)
CN_DEV uint32_t push_sign(uint32_t bits, float v) {
  return __builtin_amdgcn_alignbit(bits, __builtin_bit_cast(uint32_t, v), 31);
}

// Store of 4 consecutive plane elements (group g of feature tile t) of this
// lane's sample into the wave-tiled plane layout (cn_layout.h): the per-lane
// part of the address is voff[g] (precomputed), the rest is wave-uniform.
template <class E>
CN_DEV void plane_store(__amdgpu_buffer_rsrc_t r, const uint32_t* voff, int t, int g,
                        float a, float b, float c, float d) {
  bstore4<E>(r, voff[g], t * (1024 * (int)sizeof(E)), a, b, c, d);
}
// groups 2gp and 2gp + 1 of feature tile t (8 consecutive values of a lane
// half's slots): bf16 one 16-B store (the pair-block layout puts the two
// quads side by side), fp32 two 16-B stores
template <class E>
CN_DEV void plane_store_oct(__amdgpu_buffer_rsrc_t r, const uint32_t* voff, int t, int gp, const float* v) {
  if constexpr (sizeof(E) == 2) {
    bstore128(r, voff[2 * gp],
              u32x4{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])},
              t * 2048);
  } else {
    plane_store<E>(r, voff, t, 2 * gp, v[0], v[1], v[2], v[3]);
    plane_store<E>(r, voff, t, 2 * gp + 1, v[4], v[5], v[6], v[7]);
  }
}
// Buffer descriptor of wave wglob's 32-sample slab of a plane of width F: the
// 64-bit slab base is wave-uniform (scalar arithmetic) and goes into the
// descriptor, so every per-store offset stays below one slab (<= 36 KiB).  No
// 4 GB descriptor range or 32-bit offset bounds the plane size.
template <class E>
CN_DEV __amdgpu_buffer_rsrc_t slab_rsrc(const void* plane, int F, int wglob, bool live = true) {
  return mkrsrc((const char*)plane + (size_t)wglob * (size_t)F * 32u * sizeof(E), live);
}
// bf16: groups 2gp and 2gp+1 of feature tile t (this lane: features 16gp +
// 4h .. +3 in a, 16gp + 8 + 4h .. +3 in b, as packed pairs) -> ONE 16-B store
// at voffa = slab_off(s, 16gp + 4h): the pair-block layout (cn_layout.h) puts
// exactly these two quads side by side, so the operand registers are stored
// as they are (no lane exchange, no register copies) and one store
// instruction writes the whole 1 KiB pair block (rounds 4-5: two 8-B
// stores of 512 B each; voffb = voffa + 8 is implied).
CN_DEV void plane_store_pair(__amdgpu_buffer_rsrc_t r, uint32_t voffa, uint32_t voffb, int t, u32x2 a, u32x2 b) {
  (void)voffb;
  bstore128(r, voffa, u32x4{a[0], a[1], b[0], b[1]}, t * 2048);
}

template <int P, int SB, int TB, bool BWD, int WAVES, int MODE>
struct Chain {
  using S = Sched<P, SB, TB, BWD>;
  using N = Net<SB, TB>;
  using E = typename PT<P>::E;
  using BinT = typename PT<P>::BinT;
  static constexpr int kBin = PT<P>::kBin;
  static constexpr bool kBf16 = (P != CN_P_FP32);
  static constexpr bool kX3 = (P == CN_P_BF16X3);    // hi + lo operands, three MFMAs per block
  static constexpr bool TRAIN = MODE != CN_MODE_INFER;    // masks + sigma pre-activation
  // every operand plane of dW (TRAIN_HI: the bf16x3 forward of a bf16x3f plan)
  static constexpr bool PLANES = MODE == CN_MODE_TRAIN || MODE == CN_MODE_TRAIN_HI;
  // bf16x3 training forward: also the lo parts of dW's X operands (PE and
  // every stored Y plane, from the binl registers the epilogues already
  // hold), so the weight gradients multiply hi + lo (dw.hip DwBody<..., LO>)
  static constexpr bool kXlo = kX3 && MODE == CN_MODE_TRAIN && !BWD;
  static_assert(MODE != CN_MODE_TRAIN_HI || (kX3 && !BWD), "TRAIN_HI is the bf16x3 forward of a bf16x3f plan");
  static constexpr int NL = S::NL;
  static constexpr int kChunks = S::kChunks;
  // waves that issue the weight stream's LDS-DMA (all of them when WAVES
  // divides a chunk; a 12-wave workgroup lets waves 0-3 issue 4 blocks each)
  static constexpr int kIssuers = kChunkBlocks % WAVES == 0 ? WAVES : 4;
  static constexpr int G = kChunkBlocks / kIssuers;   // LDS-DMA instructions per issuing wave per chunk
  // chunks in flight ahead of compute.  bf16x3 runs one wave per SIMD and
  // consumes a 16 KiB chunk in ~24 MFMAs (~0.37 us) against ~1.1 us from
  // LDS-DMA issue to landing, so it keeps twice as many chunks in flight
  static constexpr int D = kX3 ? 5 : (BWD ? 2 : 3);
  // ring slots: chunk c + D is issued at chunk c's wait point, which lies in
  // chunk c - 1's tail (cross-chunk A-fragment prefetch, below), so it refills
  // the slot of chunk c - 2 -- the last one every wave has finished with
  static constexpr int NS = D + 2;
  static constexpr int kPF = kX3 ? 3 : 2;   // A-fragment prefetch distance (blocks)
  // A fragments by explicit ds_read_b128 + counted lgkmcnt waits.  Left to
  // itself the compiler's waitcnt pass emits lgkmcnt(0) before every MFMA, so
  // each MFMA also waits for the prefetch issued just before it (its LDS
  // latency exposed once per block: with one wave per SIMD, bf16x3, nothing
  // hides it).  Sound because LDS reads return in order and no scalar load
  // is in flight inside the MFMA stream (every s_load of these kernels is in
  // the prologue, before the first barrier -- checked on the ISA); extra
  // compiler-issued LDS reads only make a counted wait stricter.
  // (bf16, two waves per SIMD: the other wave hides the latency, and the
  // counted waits measured no gain there)
  static constexpr bool kAsmLds = kX3;
  // kAsmLds backward: the ReLU mask words of a layer (4 words = one 16-B
  // read per lane) are read by an explicit ds_read_b128 issued with the A
  // fragment of the layer's last block, kPF blocks ahead, and counted like
  // the fragments -- a compiler-visible read there made it wait lgkmcnt(0)
  // (a drain of the fragment prefetch) before every tile pair's conversion
  static constexpr int mask_read_at(int x) {
    if (!(kAsmLds && BWD)) return -1;
    for (int i = 0; i < S::NL; ++i)
      if (S::L(i).epi == EPI_BMASK && S::L(i).mask >= 0 && x == S::last_block(i)) return i;
    return -1;
  }
  static constexpr int group_reads(int x) { return x < 0 || x >= S::kBlocks ? 0 : 1 + (mask_read_at(x) >= 0); }
  // One Mq register set serves every masked layer: layer j's read (issued
  // with block last_block(j) - kPF, before that block's conversions)
  // overwrites it, so every earlier masked layer must have finished its
  // conversions (final_block: its last diagonal tile) before that block.
  static constexpr bool mask_reads_ordered() {
    if (!(kAsmLds && BWD)) return true;
    for (int j = 0; j < S::NL; ++j) {
      if (mask_read_at(S::last_block(j)) != j) continue;
      for (int i = 0; i < j; ++i) {
        if (mask_read_at(S::last_block(i)) != i) continue;
        const int last_use = diag(i) ? final_block(i) : S::last_block(i);
        if (!(last_use < S::last_block(j) - kPF)) return false;
      }
    }
    return true;
  }
  static constexpr int reads_after(int g) {
    int n = 0;
    for (int x = g + 1; x <= g + kPF; ++x) n += group_reads(x);
    return n;
  }
  // sched_barrier mask after each block: VALU and SALU may cross; LDS
  // reads, MFMAs and VMEM stay in program order
  static constexpr int kSbMask = 0x6;
  static constexpr int kRingBytes = NS * kChunkBytes;
  static constexpr int kBlobFloats = BiasBlob<SB, TB>::kFloats;
  static constexpr int kBlobIters = (kBlobFloats / 4 + WAVES * 64 - 1) / (WAVES * 64);
  // the first D weight chunks are issued before the prologue (run())
  static constexpr bool kEarlyIssue = true;
  // VMEM stores of the prologue (forward: PE, dir and, bf16x3 training, PE
  // lo planes; backward: the drgb plane and the sigma-head columns), as
  // plane_store_oct instructions: issued after the early weight chunks, so
  // younger than them at their wait points
  static constexpr int kProStores =
      !PLANES ? 0 : !BWD ? (kBf16 ? 4 + 2 + (kXlo ? 4 : 0) : 8 + 4) : (kBf16 ? 4 : 8);
  static constexpr int kWsOff = BiasBlob<SB, TB>::kWs;
  static constexpr int kMiscOff = BiasBlob<SB, TB>::kMisc;
  static constexpr int kDirStash = (kBf16 && !kX3) ? 32 : 64;      // bytes per lane (bf16x3: hi, lo)
  static constexpr int kDirOff = kRingBytes + kBlobFloats * 4;
  static constexpr int kMaskOff = kDirOff + (BWD ? 0 : WAVES * 64 * kDirStash);
  static constexpr int kLdsBytes = kMaskOff + (BWD ? WAVES * N::kMasks * 1024 : 0);
  static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
  static_assert(kChunkBlocks % kIssuers == 0, "issuing waves must divide a chunk");
  static_assert(N::kPlanes <= kMaxPlanes, "too many planes");
  static_assert(kBlobFloats % 4 == 0, "blob alignment");

  // ---------------- deferred plane stores (bf16)
  // A layer's output plane (Y forward, dA backward) is exactly the packed B
  // operand `bin` of the NEXT layer, so its 16-B pair stores are issued
  // spread over the next layer's MFMA blocks instead of as one burst in the
  // epilogue (where every wave of the workgroup would stall on its store
  // queue at the same time).  Store j of layer li-1 follows block
  // first_block(li) + j * lblocks(li) / n.  The last layer's plane (backward:
  // dA of the first forward layer) has no next layer and is stored in place.
  static constexpr bool codes_plane(int p) { return MODE == CN_MODE_CODES && p >= 1 && N::fwd(p - 1).inj >= 0; }
  static constexpr bool plane_of(int i) {
    const int p = S::L(i).plane;
    return BWD ? ((PLANES && N::stored(p)) || codes_plane(p)) : (PLANES && p >= 0 && N::stored(p));
  }
  static constexpr bool defers(int i) { return kBf16 && plane_of(i) && i + 1 < NL; }
  static constexpr int deferred_count(int i) { return defers(i) ? 2 * S::L(i).T : 0; }
  // index j of the deferred store of layer li-1 issued after block g, or -1
  static constexpr int deferred_at(int g) {
    const int li = S::layer_of(g);
    if (li == 0) return -1;
    const int n = deferred_count(li - 1);
    if (n == 0) return -1;
    const int nb = S::lblocks(li), lb = g - S::first_block(li);
    for (int j = 0; j < n; ++j)
      if (j * nb / n == lb) return j;
    return -1;
  }

  // ---------------- compile-time vmcnt bookkeeping
  // plane store instructions per 32-feature tile: bf16 one 16-B store per
  // pair block (plane_store_pair), fp32 one 16-B store per 4-feature group
  static constexpr int kStoresPerTile = kBf16 ? 2 : 4;
  // Vector-memory instructions each wave issues in a layer epilogue.
  static constexpr int stores_of_layer(int i) {
    const Layer l = S::L(i);
    if (!BWD) {
      int s = 0;
      if (plane_of(i) && !defers(i)) s += l.T * kStoresPerTile;
      if (TRAIN && l.mask >= 0) s += 1;
      if (l.epi == EPI_SHAPE) s += TRAIN ? 2 : 1;
      return s;   // EPI_RGB stores come after the last wait: not counted (safe)
    }
    return plane_of(i) && !defers(i) ? l.T * kStoresPerTile : 0;
  }
  // ---------------- epilogue schedule (see the epilogues below)
  // layers whose epilogue is spread over the next layer's first tile
  static constexpr bool diag(int i) { return kBf16 && i + 1 < NL; }
  // block after whose MFMA(s) tile t of layer i is converted: tiles 0, 1 at
  // the layer's last block, tile t >= 2 after k-block 2t - 3 of the next
  // layer's first tile (two k-blocks before k-block 2t reads bin[2t])
  static constexpr int conv_block(int i, int t) {
    return (!diag(i) || t < 2) ? S::last_block(i) : S::first_block(i + 1) + S::kAmul * (2 * t - 2) - 1;
  }
  static constexpr int final_block(int i) { return conv_block(i, S::L(i).T - 1); }
  // the diag layer converting tiles at block g (at most one), its first tile, count
  static constexpr int conv_layer_at(int g) {
    for (int i = 0; i < NL; ++i)
      if (diag(i) && g >= S::last_block(i) && g <= final_block(i))
        for (int t = 0; t < S::L(i).T; ++t)
          if (conv_block(i, t) == g) return i;
    return -1;
  }
  static constexpr int conv_first_tile(int i, int g) {
    for (int t = 0; t < S::L(i).T; ++t)
      if (conv_block(i, t) == g) return t;
    return 0;
  }
  static constexpr int conv_tiles(int i, int g) {
    int n = 0;
    for (int t = 0; t < S::L(i).T; ++t) n += conv_block(i, t) == g;
    return n;
  }
  // the forward epilogue's final stores (mask words, sigma / pre-activation)
  static constexpr int final_stores(int i) {
    if (BWD) return 0;
    const Layer l = S::L(i);
    return (TRAIN && l.mask >= 0 ? 1 : 0) + (l.epi == EPI_SHAPE ? (TRAIN ? 2 : 1) : 0);
  }
  // VMEM stores issued right after block g's MFMA (an epilogue, a deferred
  // plane store).  A diag layer's plane stores are all deferred (defers()),
  // so its only epilogue stores are the final ones.
  static constexpr int stores_at_block(int g) {
    int s = 0;
    for (int i = 0; i < NL; ++i) {
      if (!diag(i) && S::last_block(i) == g) s += stores_of_layer(i);
      if (diag(i) && final_block(i) == g) s += final_stores(i);
    }
    if (deferred_at(g) >= 0) s += kXlo ? 2 : 1;     // one (or, with the lo plane, two) 16-B pair stores
    return s;
  }
  static constexpr int stores_between(int b0, int b1) {
    int s = 0;
    for (int g = b0; g < b1; ++g) s += stores_at_block(g);
    return s;
  }
  static constexpr int issued(int i) { return i < kChunks ? G : 0; }
  // bf16x3 (one wave per SIMD): piece k (of G) of chunk C >= D is issued at
  // the start of block wp(C - D) + k * kSpread (after that block's wait and
  // barrier when it is a wait point), one LDS-DMA instruction per kSpread
  // blocks instead of G back to back -- a piece issued among a burst of
  // pieces and LDS reads costs 100-185 cycles of issue, one among bare MFMAs
  // ~60 (MI355X_MICROARCH.md), and with one wave per SIMD nothing else
  // issues MFMAs meanwhile (r06h: bf16x3 fwd -2.1 %, dX -3.3 %; the bf16
  // chains, two waves per SIMD, neutral: they keep the burst, kSpread 0).
  // The window is the kChunkBlocks blocks to the next wait point (the first
  // one kChunkBlocks - kPFe).
  static constexpr int kSpread = kX3 ? kChunkBlocks / G : 0;
  static_assert((G - 1) * kSpread < kChunkBlocks - kPF, "a chunk's pieces must fit its issue window");
  // the chunk with a piece issued at the start of block g (-1: none), the
  // piece, and the number of pieces issued there (burst: G at a wait point)
  static constexpr int piece_chunk(int g) {
    if (g < 0 || g >= S::kBlocks) return -1;
    int c = (g + kPFe) / kChunkBlocks;           // the window g lies in: wp(c) <= g < wp(c + 1)
    if (c > 0 && g < wp(c)) --c;
    if (wp(c) > g || c + D >= kChunks) return -1;
    const int off = g - wp(c);
    if (kSpread == 0) return off == 0 ? c + D : -1;
    if (off % kSpread || off / kSpread >= G) return -1;
    return c + D;
  }
  static constexpr int piece_k(int g) { return kSpread == 0 ? 0 : (g - wp(piece_chunk(g) - D)) / kSpread; }
  static constexpr int pieces_at(int g) { return piece_chunk(g) < 0 ? 0 : kSpread == 0 ? G : 1; }
  // A-fragment read-ahead distance in blocks (fp32 reads each block in place)
  static constexpr int kPFe = kBf16 ? kPF : 0;
  // Wait point of chunk c: before block wp(c) -- kPFe blocks before the
  // chunk's first block, so the reads of its first fragments are issued while
  // the previous chunk's last MFMAs run.  There the wave waits for its own
  // LDS-DMA of chunk c (counted vmcnt), the workgroup barriers (every wave's
  // part of chunk c has landed; every wave is past chunk c - 2), and chunk
  // c + D is issued into chunk c - 2's slot.
  static constexpr int wp(int c) { return c == 0 ? 0 : c * kChunkBlocks - kPFe; }
  static constexpr int wait_chunk_at(int g) {
    for (int c = 0; c < kChunks; ++c)
      if (wp(c) == g) return c;
    return -1;
  }
  // Younger VMEM ops that may still be in flight at chunk c's wait point:
  // the LDS-DMAs issued after chunk c's and the stores issued since it.
  static constexpr int vm_wait(int c) {
    // issue order: the initial chunks 0 .. D-1 (G pieces each), the
    // prologue's stores, then per block g: [wait + barrier at a wait point]
    // the piece issued at g, the MFMAs, the stores after them
    int n = 0, b0;
    if (c < D) {
      for (int i = c + 1; i < D; ++i) n += issued(i);        // the initial issue, younger than c
      n += kProStores;                                       // the prologue's plane stores after it
      b0 = 0;
    } else {
      b0 = wp(c - D) + (G - 1) * kSpread;                    // block of chunk c's last piece
      n += stores_at_block(b0);                              // after it in its own block
      ++b0;
    }
    for (int g = b0; g < wp(c); ++g) n += pieces_at(g) + stores_at_block(g);
    return n;
  }

  // ---------------- kernel body
  __device__ static void run(const ChainArgs& a) {
    static_assert(mask_reads_ordered(), "a masked layer's mask read would overwrite Mq before an earlier layer's "
                                        "last conversion: double-buffer Mq or move the read");
    __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const int m = blockIdx.x * (WAVES * 32) + w * 32 + (lane & 31);
    const int mc = m < a.M ? m : a.M - 1;
    const int wglob = blockIdx.x * WAVES + w;
    float* prm = (float*)(smem + kRingBytes);
    uint32_t voff[4];   // [g]: the 8-B (bf16) / 16-B (fp32) stores of feature group g
#pragma unroll
    for (int g = 0; g < 4; ++g) voff[g] = (uint32_t)slab_off(lane & 31, 8 * g + 4 * h, (int)sizeof(E));

    // -- per-call bias blob (-> LDS below) and, forward, the sample inputs:
    // plain loads issued before the weight stream, so waiting for them does
    // not wait for its LDS-DMA (vmcnt counts in issue order)
    f32x4 blobv[kBlobIters];
#pragma unroll
    for (int j = 0; j < kBlobIters; ++j) {
      const int i = threadIdx.x + j * WAVES * 64;
      if (i < kBlobFloats / 4) blobv[j] = ((const f32x4*)a.bias)[i];
    }
    Inputs in{};
    BwdInputs bwd_in{};
    if constexpr (!BWD) in = load_inputs(a, mc);
    else bwd_in = load_bwd_inputs(a, m, mc, wglob, lane);
    // forward: the first D chunks of the weight stream are issued now and land
    // during the prologue (the positional encoding: 22 accurate sincosf per
    // lane in bf16x3), instead of after it
    if constexpr (kEarlyIssue) {
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, D>([&](auto i) { issue<i>(a, smem, w, lane); });
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < kBlobIters; ++j) {
      const int i = threadIdx.x + j * WAVES * 64;
      if (i < kBlobFloats / 4) ((f32x4*)prm)[i] = blobv[j];
    }

    BinT bin[kBin];
    BinT binl[kX3 ? kBin : 1];     // bf16x3: the operand's lo parts
    f32x16 acc[8];
    // backward: every tile's first MFMA takes C = 0 (no zeroing VALU)
    if constexpr (!BWD)
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
#pragma unroll
    for (int q = 0; q < kBin; ++q) bin[q] = BinT{};
    if constexpr (kX3)
#pragma unroll
      for (int q = 0; q < kBin; ++q) binl[q] = BinT{};

    float ds = 0.f;   // bwd: sigma-head pre-activation gradient of this sample
    if constexpr (!BWD) {
      prologue_fwd(a, bin, binl, smem, h, lane, w, m, mc, wglob, voff, in);
    } else {
      ds = prologue_bwd(a, bin, binl, smem, h, lane, w, wglob, voff, bwd_in);
    }
    __syncthreads();
    if constexpr (!BWD) load_bias<0>(acc, prm, h);

    if constexpr (!kEarlyIssue) static_for<0, D>([&](auto i) { issue<i>(a, smem, w, lane); });

    float sig_part = 0.f;
    MaskAcc mk;
    // bf16: A fragments are read kPF blocks ahead of their MFMA (rolling
    // register buffer) across chunk boundaries, so the LDS latency hides
    // behind earlier MFMAs everywhere, the first blocks of a chunk included
    u32x4 Abuf[kPF + 1];      // A fragments (8 bf16 each), as the asm reads write them
    const uint32_t lbase = lds_addr(smem) + lane * 16;
    u32x4 Mq = {};      // kAsmLds backward: the mask words of the layer being converted
    const uint32_t mbase = lds_addr(smem) + (uint32_t)(kMaskOff + ((size_t)w * N::kMasks * 64 + lane) * 16);
    auto block_off = [](int b) { return (b / kChunkBlocks % NS) * kChunkBytes + (b % kChunkBlocks) * kBlockBytes; };
    auto aread = [&](auto bbc) {
      constexpr int b = bbc;
      constexpr int off = block_off(b);
      // ds_read offsets are 16-bit: the ring's upper 64 KiB through a second base
      // (the asm reads write their consumer's registers directly: a copy of
      // a register whose LDS load is still in flight would read it early)
      if constexpr (kAsmLds) {
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(Abuf[b % (kPF + 1)]) : "v"(lbase + (off & ~0xFFFF)), "n"(off & 0xFFFF));
      } else {
        Abuf[b % (kPF + 1)] = *(const u32x4*)(smem + off + lane * 16);
      }
      if constexpr (mask_read_at(b) >= 0) {
        constexpr int moff = S::L(mask_read_at(b)).mask * 1024;
        // (named first: clang captures no variable of a generic lambda that
        // only an asm operand uses)
        u32x4& mq = Mq;
        const uint32_t mb = mbase;
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(mq) : "v"(mb), "n"(moff));
      }
    };
    auto block = [&](auto gc) {
      constexpr int g = gc;
      constexpr int wc = wait_chunk_at(g);
      if constexpr (wc >= 0) {
        wait_vmcnt<vm_wait(wc)>();
        block_barrier_noread();

        if constexpr (wc == 0 && kBf16)
          static_for<0, kPF>([&](auto bb) {
            if constexpr (bb < S::kBlocks) aread(bb);
          });
      }
      if constexpr (piece_chunk(g) >= 0) {
        if constexpr (kSpread == 0) issue<piece_chunk(g)>(a, smem, w, lane);   // the burst at a wait point
        else issue_piece<piece_chunk(g), piece_k(g)>(a, smem, w, lane);
      }
      constexpr int li = S::layer_of(g);
      constexpr int lb = g - S::first_block(li);
      constexpr int t = lb / S::bpt(li);
      constexpr int kb = (lb % S::bpt(li)) / S::kAmul;     // MFMA k-block
      constexpr int part = (lb % S::bpt(li)) % S::kAmul;   // bf16x3: 0 = W_hi, 1 = W_lo fragment
      if constexpr (kBf16) {
        if constexpr (g + kPF < S::kBlocks) aread(std::integral_constant<int, g + kPF>{});
        if constexpr (kAsmLds) {
          // the reads issued after block g's fragment: its mask read, the
          // groups g + 1 .. min(g + kPF, last)
          constexpr int younger = reads_after(g) + (mask_read_at(g) >= 0 ? 1 : 0);
          asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(Abuf[g % (kPF + 1)]) : "n"(younger));
        }
        const bf16x8 A = __builtin_bit_cast(bf16x8, Abuf[g % (kPF + 1)]);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            A, __builtin_bit_cast(bf16x8, bin[kb]), (BWD && kb == 0 && part == 0) ? f32x16{} : acc[t], 0, 0, 0);
        // bf16x3: W_hi x_lo after W_hi x_hi (same A fragment); the W_lo
        // fragment (part 1) multiplies x_hi only
        if constexpr (kX3 && part == 0)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, __builtin_bit_cast(bf16x8, binl[kb]), acc[t], 0, 0, 0);
        // pin the (A-fragment read, MFMA) order: left alone, the machine
        // scheduler sinks each LDS read next to its MFMA (2 buffers, a
        // lgkmcnt(0) every other MFMA), exposing the LDS latency kPF hides
        __builtin_amdgcn_sched_barrier(kSbMask);
      } else {
        const f32x4 A = *(const f32x4*)(smem + block_off(g) + lane * 16);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[0], bin[4 * kb + 0], (BWD && kb == 0) ? f32x16{} : acc[t],
                                                      0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[1], bin[4 * kb + 1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[2], bin[4 * kb + 2], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[3], bin[4 * kb + 3], acc[t], 0, 0, 0);
      }
      // this layer's mask words (read with group g) before its first conversion
      if constexpr (mask_read_at(g) >= 0)
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(Mq) : "n"(reads_after(g)));
      if constexpr (!diag(li) && g == S::last_block(li)) {
        if constexpr (!BWD)
          epilogue_fwd<li>(a, bin, binl, acc, prm, smem, h, lane, w, m, wglob, voff, sig_part, mk);
        else
          epilogue_bwd<li>(a, bin, binl, acc, prm, smem, h, lane, w, m, wglob, voff, ds, Mq);
      }
      constexpr int ci = conv_layer_at(g);       // diagonal schedule: this block's tile conversions
      if constexpr (ci >= 0) {
        constexpr int t0 = conv_first_tile(ci, g);
        static_for<0, conv_tiles(ci, g)>([&](auto k) {
          constexpr int tt = t0 + k;
          if constexpr (!BWD)
            epi_tile_fwd<ci, tt>(a, bin, binl, acc, prm, h, wglob, voff, sig_part, mk);
          else
            epi_tile_bwd<ci, tt>(a, bin, binl, acc, prm, smem, h, lane, w, wglob, voff, ds, Mq);
        });
        if constexpr (!BWD && g == final_block(ci))
          epi_final_fwd<ci>(a, bin, binl, prm, smem, lane, w, m, wglob, sig_part, mk);
      }
      if constexpr (deferred_at(g) >= 0) {
        constexpr int j = deferred_at(g);
        constexpr int pl = li - 1;                 // layer whose output bin holds
        constexpr int plane = S::L(pl).plane;
        constexpr int F = BWD ? N::dplane_width(plane) : N::plane_width(plane);
        const u32x4 b = bin[j];                    // tile j / 2, pair j % 2
        plane_store_pair(slab_rsrc<E>(BWD ? a.dA[plane] : a.Y[plane], F, wglob), voff[2 * (j & 1)],
                         voff[2 * (j & 1) + 1], j >> 1,
                         u32x2{b[0], b[1]}, u32x2{b[2], b[3]});
        if constexpr (kXlo) {
          const u32x4 bl = binl[j];
          plane_store_pair(slab_rsrc<E>(a.Ylo[plane], F, wglob), voff[2 * (j & 1)], voff[2 * (j & 1) + 1], j >> 1,
                           u32x2{bl[0], bl[1]},
                           u32x2{bl[2], bl[3]});
        }
      }
    };
    // (two nested loops: one static_for over ~300 blocks would exceed the
    // template instantiation depth)
    static_for<0, kChunks>([&](auto cc) {
      static_for<0, kChunkBlocks>([&](auto bb) {
        constexpr int g = cc * kChunkBlocks + bb;
        if constexpr (g < S::kBlocks) block(std::integral_constant<int, g>{});
      });
    });
  }

  // one piece (k of G) of chunk C
  template <int C, int K>
  __device__ static void issue_piece(const ChainArgs& a, char* smem, int w, int lane) {
    if (kIssuers < WAVES && w >= kIssuers) return;
    const auto rs = mkrsrc(a.wpack);
    const uint32_t voffs = (uint32_t)(w * G * kBlockBytes + lane * 16);
    char* dst = smem + (C % NS) * kChunkBytes + w * G * kBlockBytes;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + K * kBlockBytes), 16, voffs,
                                             C * kChunkBytes + K * kBlockBytes, 0, 0);
  }
  template <int C>
  __device__ static void issue(const ChainArgs& a, char* smem, int w, int lane) {
    // (non-issuing waves have no LDS-DMA to wait for: their counted vmcnt
    // waits, sized for G DMAs per chunk, only relax towards their own stores)
    if (kIssuers < WAVES && w >= kIssuers) return;
    // buffer_load ... lds: the per-lane part of the source address is one
    // fixed VGPR, the chunk / block part a compile-time scalar offset, so an
    // issue costs no VALU (a global_load_lds needs a 64-bit VGPR address
    // add per instruction: ~450 VALU per bf16x3 forward wave)
    const auto rs = mkrsrc(a.wpack);
    const uint32_t voffs = (uint32_t)(w * G * kBlockBytes + lane * 16);
    char* dst = smem + (C % NS) * kChunkBytes + w * G * kBlockBytes;
#pragma unroll
    for (int k = 0; k < G; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + k * kBlockBytes), 16, voffs,
                                               C * kChunkBytes + k * kBlockBytes, 0, 0);
  }

  // accumulator tile t <- bias of forward layer LI (rows 32t + 8g + 4h + i)
  template <int LI>
  __device__ static void load_bias_tile(f32x16& acc, const float* prm, int h, int t) {
    const float* b = prm + LI * 256 + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *(const f32x4*)(b + 32 * t + 8 * g);
      acc[4 * g + 0] = v[0];
      acc[4 * g + 1] = v[1];
      acc[4 * g + 2] = v[2];
      acc[4 * g + 3] = v[3];
    }
  }
  template <int LI>
  __device__ static void load_bias(f32x16* acc, const float* prm, int h) {
#pragma unroll
    for (int t = 0; t < S::L(LI).T; ++t) load_bias_tile<LI>(acc[t], prm, h, t);
  }

  // ---------------- prologues
  // The forward's per-sample inputs, loaded before the weight stream is
  // issued (run()): explicit points, or ray origin / direction and z
  struct Inputs {
    float o[3], d[3], z;
  };
  __device__ static Inputs load_inputs(const ChainArgs& a, int mc) {
    Inputs in;
    if (a.mode == 0) {
      for (int k = 0; k < 3; ++k) { in.o[k] = a.xyz[3 * mc + k]; in.d[k] = a.vdir[3 * mc + k]; }
      in.z = 0.f;
    } else {
      const int r = mc / a.nsamp;
      const int s = mc - r * a.nsamp;
      in.z = a.zvals[r * a.z_stride + s];
      for (int k = 0; k < 3; ++k) { in.o[k] = a.rays_o[3 * r + k]; in.d[k] = a.rays_d[3 * r + k]; }
    }
    return in;
  }
  __device__ static void prologue_fwd(const ChainArgs& a, BinT* bin, BinT* binl, char* smem, int h, int lane,
                                      int w, int m, int mc, int wglob, const uint32_t* voff, const Inputs& in) {
    float x[3], d[3];
    for (int k = 0; k < 3; ++k) {
      d[k] = in.d[k];
      // xyz = ro + vd * z  (src/utils.py:30), no fused multiply-add
      x[k] = a.mode == 0 ? in.o[k] : fadd_rn(in.o[k], fmul_rn(in.d[k], in.z));
    }
    // positional encodings: this lane half's 32 PE slots and 16 dir slots
    float pe[32], dp[16];
    pe[0] = h ? x[2] : x[0];
    pe[1] = h ? 0.f : x[1];
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const int p = 15 * h + k;
      const int comp = p % 3, oct = p / 3;
      const float v = (comp == 0 ? x[0] : comp == 1 ? x[1] : x[2]) * (float)(1 << oct);
      float sn, cs;
      if constexpr (kBf16 && !kX3) sincos_turns(v, sn, cs);
      else sincosf(v, &sn, &cs);
      pe[2 + 2 * k] = sn;
      pe[3 + 2 * k] = cs;
    }
    dp[0] = h ? d[2] : d[0];
    dp[1] = h ? 0.f : d[1];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int p = h ? (k < 5 ? 7 + k : -1) : k;
      float sn = 0.f, cs = 0.f;
      if (p >= 0) {
        const int comp = p % 3, oct = p / 3;
        const float v = (comp == 0 ? d[0] : comp == 1 ? d[1] : d[2]) * (float)(1 << oct);
        if constexpr (kBf16 && !kX3) sincos_turns(v, sn, cs);
        else sincosf(v, &sn, &cs);
      }
      dp[2 + 2 * k] = sn;
      dp[3 + 2 * k] = cs;
    }
    // dir operand is needed only by the viewdir layer: stash it in LDS
    char* stash = smem + kDirOff + (w * 64 + lane) * kDirStash;
    if constexpr (kBf16) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bin[q] = u32x4{pack_bf16x2(pe[8 * q + 0], pe[8 * q + 1]), pack_bf16x2(pe[8 * q + 2], pe[8 * q + 3]),
                       pack_bf16x2(pe[8 * q + 4], pe[8 * q + 5]), pack_bf16x2(pe[8 * q + 6], pe[8 * q + 7])};
#pragma unroll
      for (int q = 0; q < 2; ++q)
        ((u32x4*)stash)[q] = u32x4{pack_bf16x2(dp[8 * q + 0], dp[8 * q + 1]), pack_bf16x2(dp[8 * q + 2], dp[8 * q + 3]),
                                   pack_bf16x2(dp[8 * q + 4], dp[8 * q + 5]), pack_bf16x2(dp[8 * q + 6], dp[8 * q + 7])};
      if constexpr (kX3) {
        auto lo4 = [](const float* v, const u32x4& hi) {
          return u32x4{resid_bf16x2(v[0], v[1], hi[0]), resid_bf16x2(v[2], v[3], hi[1]),
                       resid_bf16x2(v[4], v[5], hi[2]), resid_bf16x2(v[6], v[7], hi[3])};
        };
#pragma unroll
        for (int q = 0; q < 4; ++q) binl[q] = lo4(pe + 8 * q, bin[q]);
#pragma unroll
        for (int q = 0; q < 2; ++q) ((u32x4*)stash)[2 + q] = lo4(dp + 8 * q, ((const u32x4*)stash)[q]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 32; ++q) bin[q] = pe[q];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        ((f32x4*)stash)[q] = f32x4{dp[4 * q], dp[4 * q + 1], dp[4 * q + 2], dp[4 * q + 3]};
    }
    if constexpr (PLANES) {
      // slot q of lane half h -> column slot_col(h, q): group k = q / 4 lands in
      // feature tile k / 4, group k % 4 (cn_layout.h); groups 2gp, 2gp + 1 of
      // a tile as one plane_store_oct (bf16: one 16-B store) -- explicit, so
      // kProStores counts exactly the store instructions issued here
      const auto rp = slab_rsrc<E>(a.pe, 64, wglob);
#pragma unroll
      for (int j = 0; j < 4; ++j) plane_store_oct<E>(rp, voff, j >> 1, j & 1, pe + 8 * j);
      const auto rd = slab_rsrc<E>(a.dir, 32, wglob);
#pragma unroll
      for (int j = 0; j < 2; ++j) plane_store_oct<E>(rd, voff, 0, j, dp + 8 * j);
      if constexpr (kXlo) {
        // the PE operand's lo parts (the dir-PE tile of encoding_viewdir's
        // dW stays hi only: its staged slab would not fit the LDS ring)
        float pl[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) pl[q] = pe[q] - (float)(__bf16)pe[q];
        const auto rpl = slab_rsrc<E>(a.pelo, 64, wglob);
#pragma unroll
        for (int j = 0; j < 4; ++j) plane_store_oct<E>(rpl, voff, j >> 1, j & 1, pl + 8 * j);
      }
    }
  }

  // The backward's per-sample inputs (upstream gradients, sigma-head
  // pre-activation, the wave's ReLU mask words), loaded before the weight
  // stream is issued (run())
  struct BwdInputs {
    float g0, g1, g2, dsig, spre;
    u32x4 mw[N::kMasks];
  };
  __device__ static BwdInputs load_bwd_inputs(const ChainArgs& a, int m, int mc, int wglob, int lane) {
    BwdInputs in;
    // padding samples (m >= M) get zero upstream gradients, so every dA they
    // write is exactly 0 and the dW pass can sum whole 32-sample tiles
    const bool valid = m < a.M;
    in.g0 = valid ? a.drgb[3 * mc + 0] : 0.f;
    in.g1 = valid ? a.drgb[3 * mc + 1] : 0.f;
    in.g2 = valid ? a.drgb[3 * mc + 2] : 0.f;
    in.dsig = valid ? a.dsigma[mc] : 0.f;
    in.spre = a.spre[mc];
    const u32x4* src = (const u32x4*)a.masks + (size_t)wglob * N::kMasks * 64 + lane;
#pragma unroll
    for (int k = 0; k < N::kMasks; ++k) in.mw[k] = src[k * 64];
    return in;
  }
  __device__ static float prologue_bwd(const ChainArgs& a, BinT* bin, BinT* binl, char* smem, int h, int lane,
                                       int w, int wglob, const uint32_t* voff, const BwdInputs& in) {
    const float g0 = in.g0, g1 = in.g1, g2 = in.g2;
    // Softplus backward exactly as torch: grad * (x > 20 ? 1 : e^x / (e^x + 1))
    const float s = in.spre;
    const float ex = expf(s);
    const float ds = in.dsig * (s > 20.f ? 1.f : ex / (ex + 1.f));
    if constexpr (kBf16) {
      // k-step 0, lane half h, element j -> drgb component 8h + j
      if (h == 0) {
        bin[0] = u32x4{pack_bf16x2(g0, g1), pack_bf16x2(g2, 0.f), 0u, 0u};
        if constexpr (kX3) binl[0] = u32x4{resid_bf16x2(g0, g1, bin[0][0]), resid_bf16x2(g2, 0.f, bin[0][1]), 0u, 0u};
      }
    } else {
      // k-step q, lane half h -> drgb component 2q + h
      bin[0] = h ? g1 : g0;
      bin[1] = h ? 0.f : g2;
    }
    if constexpr (PLANES) {
      // drgb as a padded 32-wide plane for the rgb-head weight gradient
      // (columns slot_col(0, 0..2) = 0..2); the sigma-head gradient rides in
      // columns 256 (value) and 257 (its rounding residual, so bf16 storage
      // keeps ~16 significant bits) of the viewdir dA plane (feature tile 8 of
      // its 288 columns).  Explicit 16-B stores: kProStores counts them.
      const float ds_hi = (float)(E)ds;
      const float z8[8] = {};
      const float d8v[8] = {h ? 0.f : g0, h ? 0.f : g1, h ? 0.f : g2, 0.f, 0.f, 0.f, 0.f, 0.f};
      const float dsv[8] = {h ? 0.f : ds_hi, h ? 0.f : ds - ds_hi, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const auto r8 = slab_rsrc<E>(a.d8, 32, wglob);
      plane_store_oct<E>(r8, voff, 0, 0, d8v);
      plane_store_oct<E>(r8, voff, 0, 1, z8);
      const auto rv = slab_rsrc<E>(a.dA[SB + 2], 288, wglob);
      plane_store_oct<E>(rv, voff, 8, 0, dsv);
      plane_store_oct<E>(rv, voff, 8, 1, z8);
    }
    // ReLU sign bits of this wave -> LDS
    u32x4* dst = (u32x4*)(smem + kMaskOff) + (size_t)w * N::kMasks * 64 + lane;
#pragma unroll
    for (int k = 0; k < N::kMasks; ++k) dst[k * 64] = in.mw[k];
    return ds;
  }

  // ---------------- epilogues
  // A layer's epilogue is split per output tile (epi_tile_*) plus a final
  // part (epi_final_fwd: mask words, sigma head, dir operand).  Run whole at
  // the layer's last block (fp32, the last layers), or -- bf16 -- spread over
  // the NEXT layer's first output tile ("diagonal" schedule, conv_block):
  // that tile's k-block 2u needs only bin[2u] / bin[2u + 1], i.e. this
  // layer's tile u, so tile u is converted two k-blocks ahead of its first
  // use and the epilogue's VALU work issues between the MFMAs of the next
  // layer instead of as a burst with the matrix core idle (one wave per
  // SIMD in bf16x3: nothing else would fill it).
  struct MaskAcc {
    uint32_t lo[4], hi[4];
  };
  template <int LI, int TT>
  __device__ static void epi_tile_fwd(const ChainArgs& a, BinT* bin, BinT* binl, f32x16* acc, const float* prm,
                                      int h, int wglob, const uint32_t* voff, float& sig_part, MaskAcc& mk) {
    constexpr Layer l = S::L(LI);
    constexpr int t = TT;
    // tile t of this layer starts tile t of the next one (bias, below): every
    // next-layer tile has a tile here only while the next layer is no wider
    static_assert(LI + 1 >= NL || S::L(LI + 1).T <= l.T, "next layer wider than this one: its extra tiles get no bias");
    if constexpr (t == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k) mk.lo[k] = mk.hi[k] = 0u;
    constexpr int yp = l.plane >= 0 ? l.plane : 0;
    constexpr int YF = N::plane_width(yp);
    const auto ry = slab_rsrc<E>(a.Y[yp], YF, wglob);
    const float* ws = prm + kWsOff + 4 * h;
    u32x2 pg[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v0 = acc[t][4 * g + 0], v1 = acc[t][4 * g + 1];
      float v2 = acc[t][4 * g + 2], v3 = acc[t][4 * g + 3];
      if constexpr (TRAIN && l.mask >= 0) {
        // elements 0 / 2 into the low half, 1 / 3 into the high half
        // (mask_bit): push order q = 8 (t & 1) + 2 g + i / 2
        mk.lo[t >> 1] = push_sign(push_sign(mk.lo[t >> 1], v0), v2);
        mk.hi[t >> 1] = push_sign(push_sign(mk.hi[t >> 1], v1), v3);
      }
      if constexpr (l.epi == EPI_SHAPE) {
        const f32x4 w4 = *(const f32x4*)(ws + 32 * t + 8 * g);
        sig_part = __builtin_fmaf(w4[0], v0, sig_part);
        sig_part = __builtin_fmaf(w4[1], v1, sig_part);
        sig_part = __builtin_fmaf(w4[2], v2, sig_part);
        sig_part = __builtin_fmaf(w4[3], v3, sig_part);
      }
      if constexpr (kBf16) {
        if constexpr (kX3 && l.epi == EPI_RELU) {
          v0 = relu_f32(v0); v1 = relu_f32(v1); v2 = relu_f32(v2); v3 = relu_f32(v3);
        }
        uint32_t p0 = pack_bf16x2(v0, v1), p1 = pack_bf16x2(v2, v3);
        if constexpr (!kX3 && l.epi == EPI_RELU) { p0 = relu_bf16x2(p0); p1 = relu_bf16x2(p1); }
        BinT& b = bin[2 * t + (g >> 1)];
        if ((g & 1) == 0) { b[0] = p0; b[1] = p1; } else { b[2] = p0; b[3] = p1; }
        if constexpr (kX3) {
          const uint32_t l0 = resid_bf16x2(v0, v1, p0), l1 = resid_bf16x2(v2, v3, p1);
          BinT& bl = binl[2 * t + (g >> 1)];
          if ((g & 1) == 0) { bl[0] = l0; bl[1] = l1; } else { bl[2] = l0; bl[3] = l1; }
        }
        pg[g] = u32x2{p0, p1};
        if constexpr (plane_of(LI) && !defers(LI))
          if (g & 1) plane_store_pair(ry, voff[g - 1], voff[g], t, pg[g - 1], pg[g]);
      } else {
        if constexpr (l.epi == EPI_RELU) {
          v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
        }
        bin[16 * t + 4 * g + 0] = v0;
        bin[16 * t + 4 * g + 1] = v1;
        bin[16 * t + 4 * g + 2] = v2;
        bin[16 * t + 4 * g + 3] = v3;
        if constexpr (plane_of(LI))
          plane_store<E>(ry, voff, t, g, v0, v1, v2, v3);
      }
    }
    // this tile's accumulator starts the next layer's tile t
    if constexpr (t < S::L(LI + 1).T) load_bias_tile<LI + 1>(acc[t], prm, h, t);
  }

  template <int LI>
  __device__ static void epi_final_fwd(const ChainArgs& a, BinT* bin, BinT* binl, const float* prm,
                                       const char* smem, int lane, int w, int m, int wglob, float& sig_part,
                                       MaskAcc& mk) {
    constexpr Layer l = S::L(LI);
    if constexpr (TRAIN && l.mask >= 0) {
      uint32_t mw[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) mw[k] = (mk.hi[k] << 16) | (mk.lo[k] & 0xFFFFu);
      bstore128(mkrsrc(a.masks + (size_t)wglob * N::kMasks * 256), ((uint32_t)l.mask * 64 + lane) * 16,
                u32x4{mw[0], mw[1], mw[2], mw[3]});
    }
    if constexpr (l.epi == EPI_SHAPE) {
      const float tot = sig_part + __shfl_xor(sig_part, 32);
      const float pre = tot + prm[kMiscOff];
      // both lane halves hold the full sum: every lane stores (same value,
      // same address), so the store count per wave is fixed for vmcnt
      bstore32(mkrsrc(a.sigma), (uint32_t)m * 4, f2u(softplus20(pre)));
      if constexpr (TRAIN) bstore32(mkrsrc(a.spre), (uint32_t)m * 4, f2u(pre));
    }
    // the next layer (viewdir) takes the dir operand from the LDS stash
    if constexpr (S::L(LI + 1).in_kind == IN_ACC_DIR) {
      const char* stash = smem + kDirOff + (w * 64 + lane) * kDirStash;
      if constexpr (kBf16) {
        bin[16] = ((const u32x4*)stash)[0];
        bin[17] = ((const u32x4*)stash)[1];
        if constexpr (kX3) {
          binl[16] = ((const u32x4*)stash)[2];
          binl[17] = ((const u32x4*)stash)[3];
        }
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

  // the whole forward epilogue at the layer's last block
  template <int LI>
  __device__ static void epilogue_fwd(const ChainArgs& a, BinT* bin, BinT* binl, f32x16* acc, const float* prm,
                                      const char* smem, int h, int lane, int w, int m, int wglob,
                                      const uint32_t* voff, float& sig_part, MaskAcc& mk) {
    constexpr Layer l = S::L(LI);
    if constexpr (l.epi == EPI_RGB) {
      if (h == 0) {
        a.rgb[3 * m + 0] = acc[0][0];
        a.rgb[3 * m + 1] = acc[0][1];
        a.rgb[3 * m + 2] = acc[0][2];
      }
    } else {
      static_for<0, l.T>([&](auto t) { epi_tile_fwd<LI, t>(a, bin, binl, acc, prm, h, wglob, voff, sig_part, mk); });
      epi_final_fwd<LI>(a, bin, binl, prm, smem, lane, w, m, wglob, sig_part, mk);
    }
  }

  // bit of the mask word holding the sign of element (tile t, group g, i):
  // the forward epilogue shifts elements 0 / 2 into the low half and 1 / 3
  // into the high half with v_alignbit, oldest highest, push order
  // q = 8 (t & 1) + 2 g + i / 2
  static constexpr int mask_q(int t, int g, int i) { return (t & 1) * 8 + 2 * g + (i >> 1); }
  static constexpr int mask_pos(int t, int g, int i) { return ((i & 1) ? 31 : 15) - mask_q(t, g, i); }

  template <int LI, int TT>
  __device__ static void epi_tile_bwd(const ChainArgs& a, BinT* bin, BinT* binl, f32x16* acc, const float* prm,
                                      const char* smem, int h, int lane, int w, int wglob, const uint32_t* voff,
                                      float ds, const u32x4& mq) {
    constexpr Layer l = S::L(LI);
    constexpr int t = TT;
    constexpr int width = N::dplane_width(l.plane);
    const auto rdA = slab_rsrc<E>(a.dA[l.plane], width, wglob);
    uint32_t mw = 0u;     // the mask word of this tile pair
    if constexpr (l.epi == EPI_BMASK) {
      if constexpr (kAsmLds) mw = mq[t >> 1];      // read with the layer's last block (mask_read_at)
      else mw = *(const uint32_t*)(smem + kMaskOff + (((size_t)w * N::kMasks + l.mask) * 64 + lane) * 16 + 4 * (t >> 1));
    }
    const float* ws = prm + kWsOff + 4 * h;
    u32x2 pg[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc[t][4 * g + i];
        if constexpr (l.epi == EPI_BMASK && !kBf16) v[i] = relu_mask(v[i], mw, mask_pos(t, g, i));
      }
      if constexpr (l.epi == EPI_BSIGMA) {
        const f32x4 w4 = *(const f32x4*)(ws + 32 * t + 8 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fadd_rn(v[i], fmul_rn(ds, w4[i]));
      }
      if constexpr (kBf16) {
        uint32_t p0 = pack_bf16x2(v[0], v[1]), p1 = pack_bf16x2(v[2], v[3]);
        uint32_t l0 = 0u, l1 = 0u;
        if constexpr (kX3) { l0 = resid_bf16x2(v[0], v[1], p0); l1 = resid_bf16x2(v[2], v[3], p1); }
        if constexpr (l.epi == EPI_BMASK) {
          static_for<0, 4>([&](auto gg) {
            if (gg == g) {
              p0 = relu_mask_bf16x2<mask_q(t & 1, gg, 0)>(p0, mw);
              p1 = relu_mask_bf16x2<mask_q(t & 1, gg, 2)>(p1, mw);
              if constexpr (kX3) {
                l0 = relu_mask_bf16x2<mask_q(t & 1, gg, 0)>(l0, mw);
                l1 = relu_mask_bf16x2<mask_q(t & 1, gg, 2)>(l1, mw);
              }
            }
          });
        }
        BinT& b = bin[2 * t + (g >> 1)];
        if ((g & 1) == 0) { b[0] = p0; b[1] = p1; } else { b[2] = p0; b[3] = p1; }
        if constexpr (kX3) {
          BinT& bl = binl[2 * t + (g >> 1)];
          if ((g & 1) == 0) { bl[0] = l0; bl[1] = l1; } else { bl[2] = l0; bl[3] = l1; }
        }
        pg[g] = u32x2{p0, p1};
        if constexpr (plane_of(LI) && !defers(LI))
          if (g & 1) plane_store_pair(rdA, voff[g - 1], voff[g], t, pg[g - 1], pg[g]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) bin[16 * t + 4 * g + i] = v[i];
        if constexpr (plane_of(LI)) plane_store<E>(rdA, voff, t, g, v[0], v[1], v[2], v[3]);
      }
    }
  }

  template <int LI>
  __device__ static void epilogue_bwd(const ChainArgs& a, BinT* bin, BinT* binl, f32x16* acc, const float* prm,
                                      const char* smem, int h, int lane, int w, int m, int wglob,
                                      const uint32_t* voff, float ds, const u32x4& mq) {
    static_for<0, S::L(LI).T>([&](auto t) {
      epi_tile_bwd<LI, t>(a, bin, binl, acc, prm, smem, h, lane, w, wglob, voff, ds, mq);
    });
  }
};

// min waves per SIMD: 8-wave workgroups -> 2 (one workgroup per CU); bf16
// 4-wave workgroups -> 2 (two workgroups per CU, so one's prologue and
// epilogues run beside the other's MFMAs); fp32 and bf16x3 4-wave -> 1
// (512 VGPRs)
template <int P, int SB, int TB, bool BWD, int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64, (WAVES >= 8 ? WAVES / 4 : (P == CN_P_BF16 ? 2 : 1))) void
chain_kernel(ChainArgs a) {
  Chain<P, SB, TB, BWD, WAVES, MODE>::run(a);
}

}  // namespace cn
