// Compile-time weight-stream schedule of a chain kernel (forward or dX).
//
// The packed weights of one chain are a sequence of 1 KiB fragment blocks
// (one A operand of one MFMA group for 64 lanes), layer after layer, output
// tile after output tile, k-block after k-block.  16 blocks form a 16 KiB
// chunk = one LDS ring slot; chunk c lives at byte offset c * 16 KiB of the
// packed blob, so the stream is a plain linear read.
//
//   bf16: one block = one v_mfma_f32_32x32x16_bf16 A fragment (8 bf16 / lane)
//   bf16x3: two blocks per k-block, the W_hi fragment then the W_lo one
//   fp32: one block = four v_mfma_f32_32x32x2_f32 A operands (4 f32 / lane)
#pragma once
#include "cn_layout.h"

namespace cn {

template <int P, int SB, int TB, bool BWD>
struct Sched {
  using N = Net<SB, TB>;
  static constexpr int NL = BWD ? N::kBwdLayers : N::kFwdLayers;
  static constexpr bool kBf16 = (P != 0);
  // fragment blocks per MFMA k-block: bf16x3 streams W_hi and W_lo
  // back to back (the A operand of the hi and lo MFMAs)
  static constexpr int kAmul = (P == 2) ? 2 : 1;
  static constexpr Layer L(int i) { return BWD ? N::bwd(i) : N::fwd(i); }
  // input width in MFMA-k units: drgb input is 16 (bf16) / 8 (fp32) wide
  static constexpr int kdim(int i) { return (BWD && i == 0) ? (kBf16 ? 16 : 8) : L(i).K; }
  static constexpr int kper_block() { return kBf16 ? 16 : 8; }
  static constexpr int bpt(int i) { return kdim(i) / kper_block() * kAmul; }
  static constexpr int lblocks(int i) { return L(i).T * bpt(i); }
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
  static constexpr int elems_per_lane() { return kBf16 ? 8 : 4; }
  static constexpr int packed_elems() { return kChunks * kChunkBlocks * 64 * elems_per_lane(); }
  static constexpr int packed_bytes() { return kChunks * kChunkBytes; }
};

// Where the weight element for (block g, lane, element e) comes from:
// returns the reference input-feature index k of row `row` (output feature of
// the forward layer for fwd, input feature for bwd), or -1 for zero padding.
// Filled by the host plan builder; see plan.cpp.
}  // namespace cn
