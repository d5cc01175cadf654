// Shared device/host definitions for the CodeNeRF gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <utility>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#define CN_DEV __device__ __forceinline__

// ---------------------------------------------------------------- precision
// CN_P_BF16X3: error-compensated bf16 ("bf16x3").  The chain kernels carry
// every weight AND every activation / upstream gradient as a bf16 hi + lo
// pair (x_hi = rn(x), x_lo = rn(x - x_hi)) and issue three MFMAs per block
// into one fp32 accumulator: A_hi B_hi + A_hi B_lo + A_lo B_hi (the lo x lo
// term, ~2^-16 relative, is dropped).  Activation planes (the dW operands)
// are stored as in CN_P_BF16.
// CN_P_BF16X3F (a plan, not a kernel arithmetic): the bf16x3 forward chain
// (rendered rgb at fp32 class) feeding the CN_P_BF16 backward -- dX chain and
// dW pass on bf16 operands; the forward stores the hi planes only
// (CN_MODE_TRAIN_HI), which are the CN_P_BF16 planes' format.
enum { CN_P_FP32 = 0, CN_P_BF16 = 1, CN_P_BF16X3 = 2, CN_P_BF16X3F = 3 };

// Compile-time for loop: f(std::integral_constant<int, I>) for I in [0, N).
// Recursive on purpose: every level is a forceinline function, so the chain
// kernels' register arrays captured by the loop bodies stay in registers (a
// fold-expression version left the bodies un-inlined and the arrays in
// scratch).  The deep instantiation needs a large compiler stack (Makefile).
template <int Begin, int End, class F>
CN_DEV void static_for(F&& f) {
  if constexpr (Begin < End) {
    f(std::integral_constant<int, Begin>{});
    static_for<Begin + 1, End>(f);
  }
}

// LDS pointer type for the LDS-DMA builtin.
typedef __attribute__((address_space(3))) void lds_void;

CN_DEV void glds16(const void* gsrc, lds_void* ldst) {
  // LDS-DMA: the wave writes 64 x 16 B contiguously at ldst (wave-uniform);
  // each lane supplies its own global source address.
  __builtin_amdgcn_global_load_lds(gsrc, ldst, 16, 0, 0);
}

// The same LDS-DMA as opaque asm.  The compiler then does not know the
// instruction writes LDS, so it does not drain every DMA in flight before
// each LDS read it cannot prove disjoint (it cannot, when the read comes from
// a ds_read_tr builtin, whose memory operand carries no alias scope); the
// caller owns the vmcnt bookkeeping (wait_vmcnt) entirely.
CN_DEV void glds16_opaque(const void* gsrc, uint32_t lds_byte) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "{m0}"(lds_byte) : "memory");
}
// The same with the non-temporal policy, for once-read streams.
CN_DEV void glds16_opaque_nt(const void* gsrc, uint32_t lds_byte) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(gsrc), "{m0}"(lds_byte) : "memory");
}
CN_DEV uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(lds_void*)p; }

template <int N>
CN_DEV void wait_vmcnt() {
  static_assert(N >= 0, "vmcnt");
  constexpr int n = N > 63 ? 63 : N;
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
}

CN_DEV void block_barrier() {
  // raw s_barrier: does not drain in-flight LDS-DMA (unlike __syncthreads).
  // lgkmcnt(0) first: this wave's LDS reads of the slot about to be refilled
  // must have returned before any wave issues the DMA into it.  The asm
  // memory clobbers stop the compiler moving LDS accesses across.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The same barrier without the lgkmcnt(0): for a ring whose refilled slot no
// wave can still be reading (the chain kernels refill chunk c - 2's slot, whose
// fragments every wave has already fed to its MFMAs), so the reads in flight
// ahead of the barrier keep hiding their latency behind it.
CN_DEV void block_barrier_noread() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

CN_DEV float bf2f(__bf16 x) { return (float)x; }

// Softplus(beta=1, threshold=20) as torch.nn.Softplus.
CN_DEV float softplus20(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// Exact (non-contracted) fp32 helpers so host-reference rounding is
// reproduced.  hipcc defaults to -ffp-contract=fast, which fuses a*b+c into an
// FMA even through __fmul_rn/__fadd_rn once inlined; the pragma keeps these
// operations un-fusable.
CN_DEV float fmul_rn(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
CN_DEV float fadd_rn(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}

// 4 consecutive elements of an activation plane (fp32 or bf16 storage)
template <class E> CN_DEV void store4(E* p, float a, float b, float c, float d);
template <> CN_DEV void store4<float>(float* p, float a, float b, float c, float d) {
  *(f32x4*)p = f32x4{a, b, c, d};
}
template <> CN_DEV void store4<__bf16>(__bf16* p, float a, float b, float c, float d) {
  *(bf16x4*)p = bf16x4{(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
}

// ---- buffer stores: descriptor in SGPRs, 32-bit per-lane offset, the
// compile-time part of the address folded into the instruction offset.
CN_DEV __amdgpu_buffer_rsrc_t mkrsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, -1, 0x00020000);
}
// the same, or an empty range (every access discarded by the hardware) for a
// wave past the end of the launch's rows
CN_DEV __amdgpu_buffer_rsrc_t mkrsrc(const void* p, bool live) {
  // `live` is wave-uniform; readfirstlane keeps the descriptor in SGPRs (a
  // VGPR descriptor costs a readfirstlane waterfall loop around every store)
  const int n = __builtin_amdgcn_readfirstlane(live ? -1 : 0);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, n, 0x00020000);
}
// `soff` is wave-uniform (an SGPR / inline constant), so compile-time
// address parts never cost a VGPR.
// Cache policy of the activation-plane stores (bits: 1 sc0, 2 nt, 16 sc1).
// The chain kernels stream GBs of activations that only the NEXT kernel
// reads; keeping them in the XCD's 4 MiB L2 would evict the weight pack that
// every workgroup re-reads from it.
constexpr int kStoreAux = 2;
CN_DEV void bstore32(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v, int soff = 0) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)off, soff, kStoreAux);
}
CN_DEV void bstore64(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x2 v, int soff = 0) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, soff, kStoreAux);
}
CN_DEV void bstore128(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v, int soff = 0) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, soff, kStoreAux);
}
CN_DEV uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
// 4 consecutive plane elements through a buffer descriptor
template <class E> CN_DEV void bstore4(__amdgpu_buffer_rsrc_t r, uint32_t off, int soff, float a, float b, float c, float d);
template <> CN_DEV void bstore4<float>(__amdgpu_buffer_rsrc_t r, uint32_t off, int soff, float a, float b, float c, float d) {
  bstore128(r, off, u32x4{f2u(a), f2u(b), f2u(c), f2u(d)}, soff);
}
template <> CN_DEV void bstore4<__bf16>(__amdgpu_buffer_rsrc_t r, uint32_t off, int soff, float a, float b, float c, float d) {
  bf16x4 v = bf16x4{(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  bstore64(r, off, __builtin_bit_cast(u32x2, v), soff);
}
