# Timing instrumentation (results invalid): the forward chain's wave 0 of
# every workgroup stamps s_memtime at entry, before its first block and after
# its last block, with the CU's hardware ids, into sigma[128 b .. 128 b + 5]
# (tools/r06/wg_stamps.py reads them): how much of a workgroup's lifetime is
# prologue, and how long a CU sits between two workgroups -- the edges a
# persistent chain would cover.
import sys
p = sys.argv[1] + "/chain.hip"
s = open(p).read()


def sub(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


sub('''    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);''',
    '''    const uint64_t st0 = __builtin_amdgcn_s_memtime();
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);''')
sub('''    BinT bin[kBin];
    BinT binl[kX3 ? kBin : 1];     // bf16x3: the operand's lo parts''', '''    const uint64_t sta = __builtin_amdgcn_s_memtime();   // blob in LDS (its loads returned)
    BinT bin[kBin];
    BinT binl[kX3 ? kBin : 1];     // bf16x3: the operand's lo parts''')
sub('''    __syncthreads();
    if constexpr (!BWD) load_bias<0>(acc, prm, h);''', '''    const uint64_t stb = __builtin_amdgcn_s_memtime();   // prologue done (PE, its stores issued)
    __syncthreads();
    const uint64_t stc = __builtin_amdgcn_s_memtime();   // past the barrier
    if constexpr (!BWD) load_bias<0>(acc, prm, h);''')
sub('''    // (two nested loops: one static_for over ~300 blocks would exceed the
    // template instantiation depth)
    static_for<0, kChunks>([&](auto cc) {
      static_for<0, kChunkBlocks>([&](auto bb) {
        constexpr int g = cc * kChunkBlocks + bb;
        if constexpr (g < S::kBlocks) block(std::integral_constant<int, g>{});
      });
    });
  }''', '''    // (two nested loops: one static_for over ~300 blocks would exceed the
    // template instantiation depth)
    const uint64_t st1 = __builtin_amdgcn_s_memtime();
    static_for<0, kChunks>([&](auto cc) {
      static_for<0, kChunkBlocks>([&](auto bb) {
        constexpr int g = cc * kChunkBlocks + bb;
        if constexpr (g < S::kBlocks) block(std::integral_constant<int, g>{});
      });
    });
    const uint64_t st2 = __builtin_amdgcn_s_memtime();
    if constexpr (!BWD) {
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      if (w == 0 && lane == 0) {
        uint32_t* o = (uint32_t*)a.sigma + (size_t)blockIdx.x * (WAVES * 32);
        o[0] = (uint32_t)st0; o[1] = (uint32_t)st1; o[2] = (uint32_t)st2;
        o[3] = hw; o[4] = xcc; o[5] = 0x57a3u;
        o[6] = (uint32_t)sta; o[7] = (uint32_t)stb; o[8] = (uint32_t)stc;
      }
    }
  }''')
open(p, "w").write(s)
print("stamps")
