// Per-configuration kernel sets (one translation unit per precision x net).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <vector>
#include "chain_args.h"

namespace cn {

struct DwArgs;
struct DwRedArgs;
struct DwFoldArgs;
struct DbArgs;
struct LatentArgs;
struct LatentBwdArgs;

struct ActLayout {
  size_t pe = 0, dir = 0, Y[kMaxPlanes] = {}, dA[kMaxPlanes] = {}, d8 = 0, spre = 0, masks = 0, bytes = 0;
  // bf16x3 only: the lo parts (rn(x - rn(x))) of the dW pass's X operands --
  // the PE plane and every stored Y plane -- so dW multiplies hi + lo
  // (0 = absent: the plane is not allocated)
  size_t pelo = 0, Ylo[kMaxPlanes] = {};
  size_t Yw[kMaxPlanes] = {}, dAw[kMaxPlanes] = {};   // plane widths (elements per sample)
  size_t mask_bytes_per_slab = 0;                     // per 32-sample slab
};

struct ChainSet {
  int prec = 0, SB = 0, TB = 0;      // prec: plane / dW element type (0 fp32, 1 bf16)
  int x3 = 0;                         // chain kernels in bf16x3 (CN_P_BF16X3)
  int waves_fwd = 0, waves_bwd = 0;   // waves per workgroup of the forward / backward chain kernels
  int tile = 0;                        // row alignment of a launch (the 256-sample pad granule)
  int n_params = 0, n_inject = 0, n_fwd_layers = 0;
  size_t pack_fwd_bytes = 0, pack_bwd_bytes = 0;
  int blob_floats = 0;
  void (*fwd_train)(ChainArgs) = nullptr;
  void (*fwd_infer)(ChainArgs) = nullptr;
  void (*bwd)(ChainArgs) = nullptr;
  void (*fwd_codes)(ChainArgs) = nullptr;   // codes-only optimisation (CN_MODE_CODES)
  void (*bwd_codes)(ChainArgs) = nullptr;
  void (*latent_fwd)(LatentArgs) = nullptr;
  void (*latent_bwd)(LatentBwdArgs) = nullptr;
  void (*code_grad)(LatentBwdArgs) = nullptr;
  std::vector<int32_t> (*fwd_table)() = nullptr;
  std::vector<int32_t> (*bwd_table)() = nullptr;
  ActLayout (*layout)(size_t Mp) = nullptr;
  // fills the dW / reduce argument blocks; returns the number of dW workgroups
  int (*dw_setup)(char* act, int act_M, int row0, int M, int nwg, const float* zvec, float* dbuf, char* ws,
                  DwArgs* dw, DwRedArgs* red) = nullptr;
  size_t (*dw_ws_bytes)(int M) = nullptr;
  // parameter indices of the encoding_shape fold (dw_fold_kernel)
  DwFoldArgs (*fold_args)() = nullptr;
  // fills the bias-only argument block (dbuf rows of the injection layers)
  int (*db_setup)(char* act, int act_M, int M, float* dbuf, char* ws, DbArgs* db) = nullptr;
};

ChainSet chain_set_fp32_3_1();
ChainSet chain_set_bf16_3_1();
ChainSet chain_set_fp32_2_1();
ChainSet chain_set_bf16_2_1();
ChainSet chain_set_bf16x3_3_1();
ChainSet chain_set_bf16x3_2_1();
ChainSet chain_set_bf16x3f_3_1();
ChainSet chain_set_bf16x3f_2_1();

}  // namespace cn
