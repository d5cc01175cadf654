// Kernel + table instantiation for precision bf16x3, shape_blocks 3, texture_blocks 1.
#include "chain_set.h"
namespace cn {
ChainSet chain_set_bf16x3_3_1() { return make_chain_set<2, 3, 1>(); }
}  // namespace cn
