// Kernel + table instantiation for the bf16x3f plan (bf16x3 forward, bf16
// backward), shape_blocks 3, texture_blocks 1.
#include "chain_set.h"
namespace cn {
ChainSet chain_set_bf16x3f_3_1() { return make_chain_set_x3f<3, 1>(); }
}  // namespace cn
