# Timing ablations of the bf16x3 forward chain (results INVALID, timing only):
# the variant's name (variants/<name>/csrc) selects what is removed:
#   abl_nodma   no weight-stream LDS-DMA (MFMAs read whatever the ring holds)
#   abl_nobar   no LDS-DMA and no per-chunk barrier
#   abl_noepi   no forward tile epilogue (conversion, ReLU, masks, bias, stores)
#   abl_floor   no LDS-DMA, no barrier, no tile epilogue: MFMAs + A-fragment reads
#   abl_nowait  the LDS-DMA issued, its counted vmcnt waits dropped (barriers kept)
#   abl_bardma  the LDS-DMA and its waits, no per-chunk barrier
import os
import sys
d = sys.argv[1]
name = os.path.basename(os.path.dirname(os.path.abspath(d)))
p = d + "/chain.hip"
s = open(p).read()
X3 = "if constexpr (kX3 && !BWD) return;\n"


def sub(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


if name in ("abl_nodma", "abl_nobar", "abl_floor"):
    sub("""  __device__ static void issue_piece(const ChainArgs& a, char* smem, int w, int lane) {
""", """  __device__ static void issue_piece(const ChainArgs& a, char* smem, int w, int lane) {
    """ + X3)
    sub("""  __device__ static void issue(const ChainArgs& a, char* smem, int w, int lane) {
""", """  __device__ static void issue(const ChainArgs& a, char* smem, int w, int lane) {
    """ + X3)
if name == "abl_nowait":
    sub("""        wait_vmcnt<vm_wait(wc)>();
        block_barrier_noread();
""", """        if constexpr (!(kX3 && !BWD)) wait_vmcnt<vm_wait(wc)>();
        block_barrier_noread();
""")
if name == "abl_bardma":
    sub("""        wait_vmcnt<vm_wait(wc)>();
        block_barrier_noread();
""", """        wait_vmcnt<vm_wait(wc)>();
        if constexpr (!(kX3 && !BWD)) block_barrier_noread();
""")
if name in ("abl_nobar", "abl_floor"):
    sub("""        wait_vmcnt<vm_wait(wc)>();
        block_barrier_noread();
""", """        wait_vmcnt<vm_wait(wc)>();
        if constexpr (!(kX3 && !BWD)) block_barrier_noread();
""")
if name in ("abl_noepi", "abl_floor"):
    sub("""int h, int wglob, const uint32_t* voff, float& sig_part, MaskAcc& mk) {
    constexpr Layer l = S::L(LI);
""", """int h, int wglob, const uint32_t* voff, float& sig_part, MaskAcc& mk) {
    if constexpr (kX3) return;
    constexpr Layer l = S::L(LI);
""")
open(p, "w").write(s)
print("ablation", name)
