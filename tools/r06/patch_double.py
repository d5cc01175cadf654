# Power-neutral cost probes of the bf16x3 forward (variant name selects;
# timing only): the SAME work issued twice on the same data, so the operand
# values -- and with them the matrix cores' power and the clock -- stay real.
#   dbl_dma   every weight-stream LDS-DMA piece issued twice (same source,
#             same destination; the counted waits count both)
#   dbl_epi   every forward tile conversion computed twice (the first copy's
#             results consumed by an empty asm, so they are not dropped)
import os
import sys
d = sys.argv[1]
name = os.path.basename(os.path.dirname(os.path.abspath(d)))
p = d + "/chain.hip"
s = open(p).read()


def sub(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


X = "(kX3 && !BWD ? 2 : 1)"
if name == "dbl_dma":
    sub("static constexpr int issued(int i) { return i < kChunks ? G : 0; }",
        f"static constexpr int issued(int i) {{ return i < kChunks ? G * {X} : 0; }}")
    sub("static constexpr int pieces_at(int g) { return piece_chunk(g) < 0 ? 0 : kSpread == 0 ? G : 1; }",
        f"static constexpr int pieces_at(int g) {{ return piece_chunk(g) < 0 ? 0 : (kSpread == 0 ? G : 1) * {X}; }}")
    sub("""    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + K * kBlockBytes), 16, voffs,
                                             C * kChunkBytes + K * kBlockBytes, 0, 0);
""", """    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + K * kBlockBytes), 16, voffs,
                                             C * kChunkBytes + K * kBlockBytes, 0, 0);
    if constexpr (kX3 && !BWD)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + K * kBlockBytes), 16, voffs,
                                               C * kChunkBytes + K * kBlockBytes, 0, 0);
""")
    sub("""    for (int k = 0; k < G; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + k * kBlockBytes), 16, voffs,
                                               C * kChunkBytes + k * kBlockBytes, 0, 0);
""", """    for (int k = 0; k < G; ++k) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + k * kBlockBytes), 16, voffs,
                                               C * kChunkBytes + k * kBlockBytes, 0, 0);
      if constexpr (kX3 && !BWD)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + k * kBlockBytes), 16, voffs,
                                                 C * kChunkBytes + k * kBlockBytes, 0, 0);
    }
""")
if name == "dbl_epi":
    sub("""      if constexpr (kBf16) {
        if constexpr (kX3 && l.epi == EPI_RELU) {
          v0 = relu_f32(v0); v1 = relu_f32(v1); v2 = relu_f32(v2); v3 = relu_f32(v3);
        }""", """      if constexpr (kX3) {
        float w0 = v0, w1 = v1, w2 = v2, w3 = v3;
        asm volatile("" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
        if constexpr (l.epi == EPI_RELU) { w0 = relu_f32(w0); w1 = relu_f32(w1); w2 = relu_f32(w2); w3 = relu_f32(w3); }
        const uint32_t q0 = pack_bf16x2(w0, w1), q1 = pack_bf16x2(w2, w3);
        const uint32_t r0 = resid_bf16x2(w0, w1, q0), r1 = resid_bf16x2(w2, w3, q1);
        asm volatile("" :: "v"(q0), "v"(q1), "v"(r0), "v"(r1));
      }
      if constexpr (kBf16) {
        if constexpr (kX3 && l.epi == EPI_RELU) {
          v0 = relu_f32(v0); v1 = relu_f32(v1); v2 = relu_f32(v2); v3 = relu_f32(v3);
        }""")
open(p, "w").write(s)
print("double", name)
