// Kernel + table instantiation for precision fp32, shape_blocks 2, texture_blocks 1.
#include "chain_set.h"
namespace cn {
ChainSet chain_set_fp32_2_1() { return make_chain_set<0, 2, 1>(); }
}  // namespace cn
