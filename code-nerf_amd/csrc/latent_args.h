// Argument blocks of the latent-code kernels (latent.hip).
#pragma once

namespace cn {

constexpr int kLatentRowBlocks = 8;   // workgroups per latent weight-gradient update (latent_bwd_kernel)

struct LatentArgs {
  const float* const* params;   // device array of the reference parameters
  const float* shape_code;      // [256]
  const float* texture_code;    // [256]
  float* blob;                  // out: BiasBlob
  float* zvec;                  // out: [kInject][256]
};

struct LatentBwdArgs {
  const float* const* params;
  float* const* grads;          // device array of .grad pointers (accumulated)
  const float* shape_code;
  const float* texture_code;
  const float* zvec;            // [kInject][256]
  const float* dbuf;            // [kInject][256]: db of the layer each z feeds
  float* dpre;                  // scratch [kInject][256]
  float* d_shape_code;          // [256], accumulated
  float* d_texture_code;        // [256], accumulated
  float reg_coef;               // 0: no regulariser
  float* reg_out;               // [1]: reg_coef * (|s| + |t|)  (may be null)
};

}  // namespace cn
