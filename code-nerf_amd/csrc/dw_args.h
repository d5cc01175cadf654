// Argument blocks of the weight-gradient kernels (dw.hip).
#pragma once
#include <stdint.h>

namespace cn {

constexpr int kDwMaxProblems = 12;

struct DwProblem {
  const void* A;        // [Mp][lda] gradient plane (out features)
  int lda, a_valid;     // plane width, valid out features
  const void* X0;       // [Mp][ldx0] input plane for columns [0, x0_cols)
  int ldx0, x0_cols;
  const void* X1;       // [Mp][ldx1] input plane for columns [x0_cols, in_valid)
  int ldx1, in_valid;
  int out_tiles, in_tiles;
  float* part;          // [S][out_tiles*128][in_tiles*128]
  float* dbpart;        // [S][out_tiles*128]
};

struct DwArgs {
  DwProblem p[kDwMaxProblems];
  int nprob;
  int M;
  int slices;
  int mchunk;           // samples per slice (multiple of 32)
  int tile_prefix[kDwMaxProblems + 1];   // cumulative out_tiles*in_tiles
};

enum DwMap : int { MAP_PLAIN = 0, MAP_PE = 1, MAP_VIEWDIR = 2 };

struct DwRedProblem {
  const float* part;
  const float* dbpart;
  int ldp;              // in_tiles*128
  int rows_pad;         // out_tiles*128 (dbpart stride per slice)
  int out_real;         // rows mapped to the weight tensor
  int in_real;          // reference input width of the weight tensor
  int cols;             // columns to visit (in_valid)
  int map;              // DwMap
  int w, b;             // weight / bias tensor indices
  int w2, b2;           // viewdir: sigma-head weight / bias tensor indices
  const float* z;       // injection vector of the layer input (or null)
  float* dbout;         // this call's bias gradient (for the latent backward) or null
  int elems;            // work items: (out_real + extra rows) * cols
};

struct DwRedArgs {
  DwRedProblem p[kDwMaxProblems];
  int nprob;
  int slices;
  int prefix[kDwMaxProblems + 1];
  float* const* grads;
};

}  // namespace cn
