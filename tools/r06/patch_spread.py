# Spread the weight stream's LDS-DMA pieces of a chunk over the blocks of its
# issue window (piece k of chunk C at block wp(C - D) + k * kSpread) instead
# of issuing the G pieces back to back at the wait point; the counted vmcnt
# waits come from a compile-time walk of the issue order.
import sys

p = sys.argv[1] + "/chain.hip"
s = open(p).read()

old = '''  static constexpr int issued(int i) { return i < kChunks ? G : 0; }'''
new = '''  static constexpr int issued(int i) { return i < kChunks ? G : 0; }
  // Piece k (of G) of chunk C >= D is issued at the start of block
  // wp(C - D) + k * kSpread (after that block's wait and barrier when it is a
  // wait point): one LDS-DMA instruction per kSpread blocks instead of G back
  // to back -- a piece issued among a burst of pieces and LDS reads costs
  // 100-185 cycles of issue, one among bare MFMAs ~60 (MI355X_MICROARCH.md).
  // The window is the kChunkBlocks blocks to the next wait point (the first
  // one kChunkBlocks - kPFe).
  static constexpr int kSpread = kChunkBlocks / G;
  static_assert((G - 1) * kSpread < kChunkBlocks - kPF, "a chunk's pieces must fit its issue window");
  // the (chunk, piece) issued at the start of block g, or -1
  static constexpr int piece_chunk(int g) {
    if (g < 0 || g >= S::kBlocks) return -1;
    int c = (g + kPFe) / kChunkBlocks;           // the window g lies in: wp(c) <= g < wp(c + 1)
    if (c > 0 && g < wp(c)) --c;
    if (wp(c) > g) return -1;
    const int off = g - wp(c);
    if (off % kSpread || off / kSpread >= G || c + D >= kChunks) return -1;
    return c + D;
  }
  static constexpr int piece_k(int g) { return (g - wp(piece_chunk(g) - D)) / kSpread; }
  static constexpr int pieces_at(int g) { return piece_chunk(g) >= 0 ? 1 : 0; }'''
assert old in s
s = s.replace(old, new)

old = '''  static constexpr int vm_wait(int c) {
    int n = 0;
    if (c < D) {
      for (int i = c + 1; i < D; ++i) n += issued(i);        // the initial issue, younger than c
      n += kProStores;                                       // the prologue's plane stores after it
      for (int w = 0; w < c; ++w) n += issued(w + D);        // wait points 0 .. c-1
      n += stores_between(0, wp(c));
    } else {
      for (int w = c - D + 1; w < c; ++w) n += issued(w + D);
      n += stores_between(wp(c - D), wp(c));
    }
    return n;
  }'''
new = '''  static constexpr int vm_wait(int c) {
    // issue order: the initial chunks 0 .. D-1 (G pieces each), the
    // prologue's stores, then per block g: [wait + barrier at a wait point]
    // the piece issued at g, the MFMAs, the stores after them
    int n = 0, b0;
    if (c < D) {
      for (int i = c + 1; i < D; ++i) n += issued(i);        // the initial issue, younger than c
      n += kProStores;                                       // the prologue's plane stores after it
      b0 = 0;
    } else {
      b0 = wp(c - D) + (G - 1) * kSpread;                    // block of chunk c's last piece
      n += stores_at_block(b0);                              // after it in its own block
      ++b0;
    }
    for (int g = b0; g < wp(c); ++g) n += pieces_at(g) + stores_at_block(g);
    return n;
  }'''
assert old in s
s = s.replace(old, new)

old = '''        if constexpr (wc + D < kChunks) issue<wc + D>(a, smem, w, lane);'''
new = ''''''
assert old in s
s = s.replace(old, new)

old = '''      constexpr int li = S::layer_of(g);
      constexpr int lb = g - S::first_block(li);'''
new = '''      if constexpr (piece_chunk(g) >= 0) issue_piece<piece_chunk(g), piece_k(g)>(a, smem, w, lane);
      constexpr int li = S::layer_of(g);
      constexpr int lb = g - S::first_block(li);'''
assert old in s
s = s.replace(old, new)

old = '''  template <int C>
  __device__ static void issue(const ChainArgs& a, char* smem, int w, int lane) {'''
new = '''  // one piece (k of G) of chunk C
  template <int C, int K>
  __device__ static void issue_piece(const ChainArgs& a, char* smem, int w, int lane) {
    if (kIssuers < WAVES && w >= kIssuers) return;
    const auto rs = mkrsrc(a.wpack);
    const uint32_t voffs = (uint32_t)(w * G * kBlockBytes + lane * 16);
    char* dst = smem + (C % NS) * kChunkBytes + w * G * kBlockBytes;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + K * kBlockBytes), 16, voffs,
                                             C * kChunkBytes + K * kBlockBytes, 0, 0);
  }
  template <int C>
  __device__ static void issue(const ChainArgs& a, char* smem, int w, int lane) {'''
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
print("spread patch applied")
