// Kernel + table instantiation for precision bf16x3, shape_blocks 2, texture_blocks 1.
#include "chain_set.h"
namespace cn {
ChainSet chain_set_bf16x3_2_1() { return make_chain_set<2, 2, 1>(); }
}  // namespace cn
