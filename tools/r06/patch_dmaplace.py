# Placement of the bf16x3 chains' weight-stream pieces inside their issue
# window (variant name selects; timing A/B, results unchanged):
#   dma_after       a piece issued after its block's MFMA(s) instead of before
#   dma_even        pieces at the part-0 blocks (two MFMAs: W_hi x_hi, W_hi x_lo)
#                   instead of the part-1 ones (one MFMA), windows c >= 1
#   dma_after_even  both
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


if "even" in name:
    sub("""    const int off = g - wp(c);""", """    const int off = g - wp(c) - kShift(c);
    if (off < 0) return -1;""")
    sub("""  static constexpr int piece_k(int g) { return kSpread == 0 ? 0 : (g - wp(piece_chunk(g) - D)) / kSpread; }""",
        """  static constexpr int kShift(int c) { return kSpread > 0 && c >= 1 ? 1 : 0; }
  static constexpr int piece_k(int g) {
    return kSpread == 0 ? 0 : (g - wp(piece_chunk(g) - D) - kShift(piece_chunk(g) - D)) / kSpread;
  }""")
    sub("""      b0 = wp(c - D) + (G - 1) * kSpread;""", """      b0 = wp(c - D) + (G - 1) * kSpread + kShift(c - D);""")
if "after" in name:
    sub("""      if constexpr (piece_chunk(g) >= 0) {
        if constexpr (kSpread == 0) issue<piece_chunk(g)>(a, smem, w, lane);   // the burst at a wait point
        else issue_piece<piece_chunk(g), piece_k(g)>(a, smem, w, lane);
      }
""", """      if constexpr (piece_chunk(g) >= 0 && kSpread == 0) issue<piece_chunk(g)>(a, smem, w, lane);
""")
    sub("""      // this layer's mask words (read with group g) before its first conversion""",
        """      if constexpr (piece_chunk(g) >= 0 && kSpread != 0) issue_piece<piece_chunk(g), piece_k(g)>(a, smem, w, lane);
      // this layer's mask words (read with group g) before its first conversion""")
open(p, "w").write(s)
print("dma placement", name)
