// Kernel + table instantiation for precision bf16, shape_blocks 3, texture_blocks 1.
#include "chain_set.h"
namespace cn {
ChainSet chain_set_bf16_3_1() { return make_chain_set<1, 3, 1>(); }
}  // namespace cn
