// Static description of the CodeNeRF MLP as a chain of MFMA layers.
//
// Shared by the host plan builder (packing / gradient-mapping tables) and the
// chain kernels (compile-time block schedule).  The network is the reference
// CodeNeRF (src/model.py:10-53) with W = latent_dim = 256, num_xyz_freq = 10,
// num_dir_freq = 4; shape_blocks (SB) and texture_blocks (TB) are template
// parameters.
//
// Orientation (both precisions): a wave owns 32 samples; an MFMA computes
// Y^T[32 out features][32 samples] = W[32][K] * X^T[K][32 samples].  The
// accumulator (32x32 f32: sample on the lane, features in 16 registers)
// therefore IS the next layer's B operand after bias/activation, with the k
// order permuted; the packed weights absorb that permutation.
#pragma once
#include <stdint.h>

namespace cn {

constexpr int kW = 256;
constexpr int kLatent = 256;
constexpr int kXyzFreq = 10;
constexpr int kDirFreq = 4;
constexpr int kPeSlots = 64;   // 63 PE features + 1 pad, 32 per lane half
constexpr int kDirSlots = 32;  // 27 dir-PE features + 5 pad, 16 per lane half
constexpr int kBlockBytes = 1024;        // one A-fragment block (64 lanes x 16 B)
constexpr int kChunkBlocks = 16;   // LDS ring slot = 16 blocks = 16 KiB (one barrier per slot)
constexpr int kChunkBytes = kBlockBytes * kChunkBlocks;

// Reference parameter tensor indices (state_dict order, oracle/params.py).
struct ParamIdx {
  int SB, TB;
  constexpr int enc_xyz_w() const { return 0; }
  constexpr int shape_latent_w(int j) const { return 2 + 4 * j; }      // j: 0-based block
  constexpr int shape_w(int j) const { return 4 + 4 * j; }
  constexpr int enc_shape_w() const { return 2 + 4 * SB; }
  constexpr int sigma_w() const { return 4 + 4 * SB; }
  constexpr int viewdir_w() const { return 6 + 4 * SB; }
  constexpr int tex_latent_w(int j) const { return 8 + 4 * SB + 4 * j; }
  constexpr int tex_w(int j) const { return 10 + 4 * SB + 4 * j; }
  constexpr int rgb0_w() const { return 8 + 4 * SB + 4 * TB; }
  constexpr int rgb2_w() const { return 10 + 4 * SB + 4 * TB; }
  constexpr int count() const { return 12 + 4 * (SB + TB); }
};

enum InKind : int { IN_PE = 0, IN_ACC = 1, IN_ACC_DIR = 2, IN_DRGB = 3 };
enum EpiKind : int {
  EPI_RELU = 0,      // fwd: + bias, ReLU, (store Y, mask), (+ injection)
  EPI_SHAPE = 1,     // fwd: + bias, no activation, sigma head (encoding_shape)
  EPI_RGB = 2,       // fwd: + bias, rgb output (last layer)
  EPI_BMASK = 3,     // bwd: dA = dY * mask, store dA
  EPI_BSIGMA = 4,    // bwd: dA = dY + w_sigma * ds (no activation), store dA
};

struct Layer {
  int T;          // output tiles of 32 features
  int K;          // input features incl. padding (multiple of 16 bf16 / 8 fp32)
  int in_kind;
  int epi;
  int w;          // weight tensor index (reference order)
  int b;          // bias tensor index, -1 none
  int inj;        // fwd: injection vector added to the output (next input), -1 none
  int mask;       // fwd: mask slot written; bwd: mask slot read; -1 none
  int plane;      // fwd: Y plane written; bwd: dA plane written; -1 none
  int t_in;       // input tiles from the previous accumulator (K_acc / 32)
};

template <int SB, int TB>
struct Net {
  static constexpr int kFwdLayers = SB + TB + 5;
  static constexpr int kBwdLayers = SB + TB + 4;
  static constexpr int kPlanes = SB + TB + 4;       // Y / dA planes (all but last layer)
  static constexpr int kMasks = SB + TB + 3;        // ReLU layers
  static constexpr int kInject = SB + TB;
  static constexpr ParamIdx P{SB, TB};

  // forward layer i (0-based)
  static constexpr Layer fwd(int i) {
    if (i == 0) return {8, kPeSlots, IN_PE, EPI_RELU, P.enc_xyz_w(), P.enc_xyz_w() + 1,
                        SB >= 1 ? 0 : -1, 0, 0, 0};
    if (i <= SB) return {8, 256, IN_ACC, EPI_RELU, P.shape_w(i - 1), P.shape_w(i - 1) + 1,
                         i < SB ? i : -1, i, i, 8};
    if (i == SB + 1) return {8, 256, IN_ACC, EPI_SHAPE, P.enc_shape_w(), P.enc_shape_w() + 1,
                             -1, -1, i, 8};
    if (i == SB + 2) return {8, 256 + kDirSlots, IN_ACC_DIR, EPI_RELU, P.viewdir_w(),
                             P.viewdir_w() + 1, TB >= 1 ? SB : -1, SB + 1, i, 8};
    if (i <= SB + 2 + TB) {
      int j = i - (SB + 3);
      return {8, 256, IN_ACC, EPI_RELU, P.tex_w(j), P.tex_w(j) + 1,
              j + 1 < TB ? SB + j + 1 : -1, i - 1, i, 8};
    }
    if (i == SB + TB + 3) return {4, 256, IN_ACC, EPI_RELU, P.rgb0_w(), P.rgb0_w() + 1, -1,
                                  SB + TB + 2, i, 8};
    return {1, 128, IN_ACC, EPI_RGB, P.rgb2_w(), P.rgb2_w() + 1, -1, -1, -1, 4};
  }

  // mask slot of forward layer f (or -1): ReLU layers in order
  static constexpr int mask_of(int f) { return fwd(f).mask; }

  // backward (dX) layer i in processing order; K in bf16 units (fp32 uses kdrgb8)
  static constexpr Layer bwd(int i) {
    const int last = SB + TB + 4;          // fwd index of rgb2
    if (i == 0) {   // rgb2^T: drgb -> d y_rgb0 ; dA(rgb0) = * mask(rgb0)
      return {4, 16, IN_DRGB, EPI_BMASK, P.rgb2_w(), -1, -1, mask_of(last - 1), last - 1, 0};
    }
    // i >= 1: transpose of forward layer f = last - i, producing dA of layer f - 1
    const int f = last - i;
    const Layer L = fwd(f);
    const int tin = fwd(f).T;              // input = dA of layer f (its T tiles)
    if (f == SB + 2) {   // viewdir^T (y part only) -> d y_shape (+ sigma head)
      return {8, tin * 32, IN_ACC, EPI_BSIGMA, L.w, -1, -1, -1, f - 1, tin};
    }
    return {8, tin * 32, IN_ACC, EPI_BMASK, L.w, -1, -1, mask_of(f - 1), f - 1, tin};
  }

  // encoding_shape (forward layer SB + 1) has no activation, so its output Y
  // and output gradient dA are linear in planes that ARE stored (Y of the last
  // shape layer; dA of encoding_viewdir + the sigma-head gradient).  The weight
  // gradients that would read them are folded through the layer instead
  // (dw_fold_kernel), and neither plane is written: 2 KB less HBM traffic per
  // bf16 training sample.
  static constexpr bool stored(int p) { return p != SB + 1; }
  static constexpr int plane_width(int p) { return p == SB + TB + 3 ? 128 : 256; }
  // dA plane widths: viewdir's carries the sigma-head gradient in column 256
  static constexpr int dplane_width(int p) {
    return p == SB + TB + 3 ? 128 : (p == SB + 2 ? 288 : 256);
  }
};

// ---- k-slot maps -------------------------------------------------------------
// PE slot (lane half h, index s in 0..31) -> reference PE feature (-1 = pad).
// Reference order (src/model.py:4-7): [x0 x1 x2, sin(a_0..a_29), cos(a_0..a_29)],
// a_p = 2^(p/3) * x_(p%3).  Each lane half computes sin AND cos of the same
// argument, so slots are (raw, raw, sin a_k, cos a_k, ...).
inline constexpr int pe_slot_feature(int h, int s) {
  if (s == 0) return h == 0 ? 0 : 2;
  if (s == 1) return h == 0 ? 1 : -1;
  int k = (s - 2) >> 1;                 // 0..14
  int p = 15 * h + k;                   // argument index 0..29
  return (s & 1) == 0 ? 3 + p : 33 + p;
}
// dir slot (h, s in 0..15) -> dir-PE feature (0..26) or -1
inline constexpr int dir_slot_feature(int h, int s) {
  if (s == 0) return h == 0 ? 0 : 2;
  if (s == 1) return h == 0 ? 1 : -1;
  int k = (s - 2) >> 1;
  int p = h == 0 ? k : 7 + k;           // half 0: args 0..6, half 1: 7..11
  if (h == 1 && k >= 5) return -1;
  return (s & 1) == 0 ? 3 + p : 15 + p;
}
// argument index for the sincos pair at slot pair k of half h (-1 none)
inline constexpr int pe_pair_arg(int h, int k) { return 15 * h + k; }
inline constexpr int dir_pair_arg(int h, int k) {
  return h == 0 ? k : (k < 5 ? 7 + k : -1);
}

// bf16 32x32x16: k-step q, lane half h, element j -> input index within K.
// For accumulator-fed inputs: feature 32u + 16s + 8(j>>2) + 4h + (j&3), q = 2u+s.
inline constexpr int bf16_acc_feature(int q, int h, int j) {
  return 32 * (q >> 1) + 16 * (q & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}
// fp32 32x32x2: k-step q (= 16u + r), lane half h -> feature 32u + (r&3) + 8(r>>2) + 4h
inline constexpr int f32_acc_feature(int q, int h) {
  return 32 * (q >> 4) + ((q & 15) & 3) + 8 * ((q & 15) >> 2) + 4 * h;
}
// accumulator register r of lane half h -> row within the 32-row tile
inline constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ---- activation planes in HBM: wave-tiled, bank-swizzled --------------------
// A plane of width F (multiple of 32) over Mp samples is stored slab by slab:
// a 32-sample slab is one contiguous run of F * 32 elements, made of 32-feature
// tiles.  Inside a tile the layout depends on the element size.
//
// fp32 (16 B = 4 features): per 8-feature group g, 64 "positions" of 4
// consecutive features; sample s, feature half hh = (f >> 2) & 1 sits at
//     pos = ((s + g + 4 hh) & 31) + 32 hh,
// so one epilogue store instruction (lane = s + 32 h writes features
// 32t + 8g + 4h .. +3) fills one contiguous 64 x 16 B block, and the fp32 dW
// pass's ds_read_b32 of one sample's 32 tile features (lane c: g = c >> 3,
// hh = (c >> 2) & 1) hits bank 4 ((s + g + 4 hh) mod 8) + (c & 3): all 32
// banks (a rotation by 8 g put the four groups on the same 8 banks: 4-way).
//
// bf16 (16 B = 8 features): per 16-feature pair block gp, 64 positions of 16
// B; position hh (lane half) of sample s holds the two feature quads a lane
// half hh owns after an MFMA (accumulator rows 4 hh .. +3 of both 8-row
// groups): features 16 gp + 4 hh .. +3 in its first 8 bytes and
// 16 gp + 8 + 4 hh .. +3 in its second, at
//     pos = 32 hh + ((s + 8 gp + 4 hh) & 31).
// So lane s + 32 hh stores its 8 features of a pair block as they sit in its
// registers with ONE 16-B store, and one store instruction fills the whole
// 1 KiB pair block (round 6; rounds 4-5: two 8-B stores per pair block, the
// quads of one 8-feature group side by side; round 3: a v_permlane32_swap
// lane exchange before a 16-B store).  The rotation by 8 gp + 4 hh makes the
// dW kernel's transposed LDS reads (ds_read_b64_tr_b16: 4 samples x 4
// features per lane, a 32-lane half spanning 4 samples x 32 features) hit 64
// distinct banks: bank pair 4 ((s + 8 gp + 4 hh) mod 16) + 2 gg.
inline constexpr int tile_pos(int s, int g, int hh) { return ((s + g + 4 * hh) & 31) + 32 * hh; }
inline constexpr int bf16_pos(int s, int gp, int hh) { return 32 * hh + ((s + 8 * gp + 4 * hh) & 31); }
// byte offset, inside a 32-sample slab, of features f .. f+3 (f % 4 == 0) of sample s
inline constexpr int slab_off(int s, int f, int es) {
  return es == 2 ? (f >> 5) * 2048 + ((f >> 4) & 1) * 1024 + bf16_pos(s, (f >> 4) & 1, (f >> 2) & 1) * 16 +
                       ((f >> 3) & 1) * 8
                 : (f >> 5) * 4096 + ((f >> 3) & 3) * 1024 + tile_pos(s, (f >> 3) & 3, (f >> 2) & 1) * 16;
}
// byte offset of features f .. f+3 of sample m in a plane of width F
inline constexpr uint64_t plane_off(uint64_t m, int f, int F, int es) {
  return (m >> 5) * (uint64_t)F * 32u * (uint64_t)es + (uint64_t)slab_off((int)(m & 31), f, es);
}
// prologue planes (PE, dir, drgb, sigma-head columns): the q-th value a lane
// half h holds goes to column 8 (q / 4) + 4 h + (q % 4), so it is written by the
// same store pattern as an epilogue group.
inline constexpr int slot_col(int h, int q) { return 8 * (q >> 2) + 4 * h + (q & 3); }
inline constexpr int col_half(int c) { return (c >> 2) & 1; }
inline constexpr int col_slot(int c) { return 4 * (c >> 3) + (c & 3); }

}  // namespace cn
