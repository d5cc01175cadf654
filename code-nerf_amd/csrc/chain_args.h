// Argument block and per-call bias blob layout of the chain kernels.
#pragma once
#include <stdint.h>
#include "cn_layout.h"

namespace cn {

constexpr int kMaxPlanes = 12;

// What a chain launch stores (template parameter MODE of chain_kernel).
enum ChainMode : int {
  CN_MODE_INFER = 0,   // outputs only
  CN_MODE_TRAIN = 1,   // + every plane the backward and the dW pass read
  CN_MODE_CODES = 2,   // codes-only optimisation (src/optimizer.py): forward stores
                       // ReLU masks + sigma pre-activations, backward only the dA
                       // planes of the layers fed by a code (the bias sums need them)
  CN_MODE_TRAIN_HI = 3,  // bf16x3 forward, training: every plane of CN_MODE_TRAIN but
                         // not the X lo planes (CN_P_BF16X3F: a bf16 dW reads hi only)
};

// Per-call bias blob (written by the latent kernel, read by the forward chain):
//   [kFwdLayers][256]  bias of every forward layer (code injection folded in)
//   [256]              sigma head weight (ws)
//   [4]                misc: [0] sigma head bias
template <int SB, int TB>
struct BiasBlob {
  static constexpr int kWs = Net<SB, TB>::kFwdLayers * 256;
  static constexpr int kMisc = kWs + 256;
  static constexpr int kFloats = kMisc + 4;
};

struct ChainArgs {
  const void* wpack;       // packed weight blocks of this chain
  const float* bias;       // per-call bias blob (BiasBlob layout)
  int M;
  // ---- forward inputs
  int mode;                // 0: explicit points, 1: rays x samples
  int nsamp;               // samples per ray (mode 1)
  int z_stride;            // 0: shared z (reference), nsamp: per-ray z
  const float* xyz;        // [M][3]            (mode 0)
  const float* vdir;       // [M][3]            (mode 0)
  const float* rays_o;     // [R][3]            (mode 1)
  const float* rays_d;     // [R][3]            (mode 1)
  const float* zvals;      // [z_stride ? R*nsamp : nsamp]
  // ---- forward outputs (sized to the padded sample count)
  float* sigma;            // [Mp]
  float* rgb;              // [Mp][3]
  // ---- activation workspace (training)
  void* pe;                // [Mp][64]
  void* dir;               // [Mp][32]
  void* Y[kMaxPlanes];     // forward layer outputs
  void* dA[kMaxPlanes];    // pre-activation gradients
  void* pelo;              // bf16x3: lo parts of pe       (or null)
  void* Ylo[kMaxPlanes];   // bf16x3: lo parts of every Y  (or null)
  void* d8;                // [Mp][32] drgb (padded)
  float* spre;             // [Mp] sigma-head pre-activation
  uint32_t* masks;         // [Mp/32][kMasks][64][4] pre-activation sign bits
  // ---- backward inputs
  const float* dsigma;     // [M]
  const float* drgb;       // [M][3]
};

}  // namespace cn
