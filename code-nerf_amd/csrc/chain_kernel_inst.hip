// One chain kernel instantiation per translation unit (the Makefile compiles
// this file once per kernel with -DCN_KP/-DCN_KSB/-DCN_KTB/-DCN_KBWD/-DCN_KW/
// -DCN_KM): the unrolled chain schedules are the slowest code to compile, and
// one kernel per unit lets the build run them all in parallel.  The chain-set
// units (inst_*.hip) only reference them (chain_extern.h).
#include "chain.hip"
namespace cn {
template __global__ void chain_kernel<CN_KP, CN_KSB, CN_KTB, CN_KBWD, CN_KW, CN_KM>(ChainArgs);
}  // namespace cn
