// Argument blocks of the weight-gradient kernels (dw.hip).
#pragma once
#include <stdint.h>

namespace cn {

constexpr int kDwMaxProblems = 12;

// One layer's weight gradient over one slice of the samples.  Operands are
// wave-tiled planes (cn_layout.h): a 32-sample slab of T feature tiles is one
// contiguous run of T * 1024 elements.
struct DwProblem {
  const void* A;        // gradient plane (rows of dW: out features)
  int a_width;          // plane width (elements)
  int a_tiles;          // 32-wide feature tiles of A staged per slab (<= 9)
  int out_tiles;        // row tiles computed by MFMA (<= 8)
  const void* X0;       // input plane, feature tiles [0, x0_tiles)
  int x0_width, x0_tiles;
  const void* X1;       // second input plane appended after X0 (dir PE), or null
  int x1_width, x1_tiles;
  const void* X0lo;     // bf16x3: lo parts of X0 (same layout), staged after X1; null: X0 only
  int lo;               // 1: X0lo given (dW multiplies A by X0 + X0lo)
  int sigma_head;       // viewdir: also sum ds (A column 256 + 257) x X columns 0..255
  int rows_pad, cols_pad;   // extent of the partial actually written (<= 288)
  int kind;             // DwKind: operand shape, selects the compile-time bf16 body
};

// The five operand shapes of the CodeNeRF weight gradients (tiles of 32
// features: A = gradient plane, X = input plane(s)).
enum DwKind : int {
  DW_FULL = 0,      // 256 x 256 hidden layers             A 8, X 8
  DW_PE = 1,        // encoding_xyz: 256 x 63 (PE input)   A 8, X 2
  DW_VIEWDIR = 2,   // encoding_viewdir (+ sigma head)     A 9, X 8 + 1 (dir PE)
  DW_RGB0 = 3,      // rgb.0: 128 x 256                    A 4, X 8
  DW_RGB2 = 4,      // rgb.2: 3 x 128                      A 1, X 4
};

// Persistent, byte-balanced schedule: the (problem, slab) stream -- problem
// after problem, slab after slab -- is cut into `nwg` equal shares of HBM
// bytes; workgroup g owns share g and so at most two consecutive problems
// ("segments"); it writes one partial per segment into slot (g, seg).
struct DwArgs {
  DwProblem p[kDwMaxProblems];
  int nprob;
  int total_tiles;              // slabs per problem (Mp / 32)
  int nwg;                      // workgroups (= partial slots / 2)
  long long wprefix[kDwMaxProblems + 1];   // cumulative bytes: problem p starts at wprefix[p]
  int pbytes[kDwMaxProblems];   // bytes per slab of problem p
  float* part;                  // [nwg][2][kPartRows][kPartCols]
  float* dbpart;                // [nwg][2][kPartRows]
};
constexpr int kPartRows = 288, kPartCols = 288;

#define CN_HD __host__ __device__ __forceinline__
// first byte of workgroup g's share
CN_HD long long dw_share_begin(int g, long long total, int nwg) { return total * g / nwg; }
// slabs [t0, t1) of problem p whose first byte lies in [b0, b1)
CN_HD void dw_slab_range(const long long* wprefix, const int* pbytes, int T, int p, long long b0, long long b1,
                         int& t0, int& t1) {
  const long long base = wprefix[p], pb = pbytes[p];
  auto cdiv = [&](long long x) -> int {
    if (x <= 0) return 0;
    const long long q = (x + pb - 1) / pb;
    return q > T ? T : (int)q;
  };
  t0 = cdiv(b0 - base);
  t1 = cdiv(b1 - base);
}

enum DwMap : int { MAP_PLAIN = 0, MAP_PE = 1, MAP_VIEWDIR = 2 };

struct DwRedProblem {
  int out_real;         // rows mapped to the weight tensor
  int in_real;          // reference input width of the weight tensor
  int cols;             // columns to visit
  int map;              // DwMap
  int w, b;             // weight / bias tensor indices
  int w2, b2;           // viewdir: sigma-head weight / bias tensor indices (row out_real)
  const float* z;       // injection vector of the layer input (or null)
  float* dbout;         // this call's bias gradient (for the latent backward) or null
  int elems;            // work items
  int pbytes;           // bytes per slab (schedule)
};

struct DwRedArgs {
  DwRedProblem p[kDwMaxProblems];
  int nprob;
  int prefix[kDwMaxProblems + 1];
  float* const* grads;
  int nwg;
  long long wprefix[kDwMaxProblems + 1];
  const float* part;            // DwArgs::part
  const float* dbpart;
  // workgroups holding slabs of problem p: gfirst[p] .. glast[p]; the first
  // one may hold it as its second segment (gseg[p]), the others as their first
  int gfirst[kDwMaxProblems], glast[kDwMaxProblems], gseg[kDwMaxProblems];
  int db_accum;                 // dbout += (a later row range of the same step) instead of =
  float* fold;                  // [kFoldRows][kFoldCols] Gx of the encoding_shape fold (viewdir problem)
};

// encoding_shape fold (chain_set.h fold_args): Gx = 257 rows (viewdir out
// features + sigma head) x 257 columns (last shape layer's features + bias sum)
constexpr int kFoldRows = 257, kFoldCols = 257;
struct DwFoldArgs {
  const float* fold;            // Gx, written by dw_reduce_kernel
  const float* const* params;   // reference parameter tensors (the weights the forward used)
  float* const* grads;          // their gradients (accumulated)
  int w_shape;                  // encoding_shape weight index (bias = +1)
  int w_view;                   // encoding_viewdir weight index ([256][view_cols])
  int view_cols;                // 256 + 27
  int w_sigma;                  // sigma head weight index (bias = +1)
};

// Bias gradients of the layers that follow a code injection only (codes-only
// optimisation: no weight gradients needed): db_j = sum over samples of dA.
constexpr int kDbMaxInject = 8;
constexpr int kDbBlocks = 256;               // sample-range blocks per layer
struct DbArgs {
  const void* A[kDbMaxInject];               // dA plane of the layer after injection j
  int a_width[kDbMaxInject];
  int ninj;
  int total_slabs;                           // Mp / 32
  int slabs_per_blk;
  float* part;                               // [ninj][kDbBlocks][256]
  float* dbout;                              // [ninj][256]
};

}  // namespace cn
