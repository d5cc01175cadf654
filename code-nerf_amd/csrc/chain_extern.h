// Every chain kernel the plans use, as (precision, shape_blocks,
// texture_blocks, backward, waves per workgroup, mode).  Each is instantiated
// in a translation unit of its own (chain_kernel_inst.hip, Makefile KERNELS:
// keep the two lists equal); the chain-set units declare them extern.
#pragma once
#include "chain.hip"

#define CN_CHAIN_KERNELS_NET(X, SB, TB)                                                                   \
  X(0, SB, TB, false, 4, 0) X(0, SB, TB, false, 4, 1) X(0, SB, TB, false, 4, 2)                           \
  X(0, SB, TB, true, 4, 1) X(0, SB, TB, true, 4, 2)                                                       \
  X(1, SB, TB, false, 8, 0) X(1, SB, TB, false, 8, 1) X(1, SB, TB, false, 8, 2)                           \
  X(1, SB, TB, true, 8, 1) X(1, SB, TB, true, 8, 2)                                                       \
  X(2, SB, TB, false, 4, 0) X(2, SB, TB, false, 4, 1) X(2, SB, TB, false, 4, 2) X(2, SB, TB, false, 4, 3) \
  X(2, SB, TB, true, 4, 1) X(2, SB, TB, true, 4, 2)
#define CN_CHAIN_KERNELS(X) CN_CHAIN_KERNELS_NET(X, 3, 1) CN_CHAIN_KERNELS_NET(X, 2, 1)

namespace cn {
#define CN_EXTERN_CHAIN(P, SB, TB, BWD, W, M) extern template __global__ void chain_kernel<P, SB, TB, BWD, W, M>(ChainArgs);
CN_CHAIN_KERNELS(CN_EXTERN_CHAIN)
#undef CN_EXTERN_CHAIN
}  // namespace cn
