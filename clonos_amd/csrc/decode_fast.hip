// decode_fast.hip -- the fast decode pipeline (gfx950): convergence points.
//
// For region l of a tile, start a parse at each of its first kCands offsets (every
// possible entry a fixed-layout record can leave behind) and advance the candidates in
// position order with a 64-bit frontier (paths that land on the same byte merge; paths
// that hit an invalid record die).  The first position through which every live
// candidate passes -- the region's convergence point -- is a record start on the true
// path whenever the true entry is one of the candidates.  Lanes then parse the segments
// between consecutive points; the chain of segments from a tile's entry point is checked
// (a lane that jumps over a point keeps going to the next one), so a wrong point costs
// extra parsing, never a wrong answer.  Spans whose chain breaks (no point reachable, a
// decode error, an overflowing Serializable table) are flagged and re-decoded by the DP
// pipeline in kernels.hip, which also reports exact error positions.
//
// Kernels:  k_fast_scan   stage tile -> points (BFS) -> filter -> segments -> chain
//           k_jser_fill   Serializable stream lengths for deferred tiles (walker)
//           k_fast_resolve  per span: tile entries/bases (regular: one scan)
//           k_fast_emit   stage tile -> record starts into LDS by output index ->
//                         decode + coalesced SoA stores
// The hot kernels are call-free: Serializable lengths come from per-tile tables, and
// tiles whose scan meets a magic-bearing tag-3 record before the tables exist are deferred.
//
// LDS image: dense (byte a of the tile's aligned coordinates at LDS byte a), followed by
// a halo of the span's next bytes.  Regions are 268 B = 67 dwords apart, an odd stride,
// so lanes scanning their own regions in step hit 64 distinct banks.
//
// Record layouts: SimpleDeterminantEncoder.java:124-323 (reference flink-runtime).
#include "dev_slow.h"

namespace clg {

#define CLG_JPHASE(i) \
  if (J.prof && lane == 0) J.prof[(uint64_t)t * 16 + (i)] = __builtin_amdgcn_s_memtime()

constexpr uint32_t kScanHalo = 1024;  // covers the next tile's first kFNext regions + BFS overrun
constexpr uint32_t kEmitHalo = 1024;  // the chain's last segment runs to a next-tile point (up to kFNext regions in)
constexpr int kScanImgDwords = (kTile + kScanHalo + 64) / 4;
constexpr int kEmitImgDwords = (kTile + kEmitHalo + 64) / 4;
constexpr uint32_t kNoFar = 0xFFFFFFFFu;
constexpr int kMaxPops = 96;          // give up early: an unknown point only lengthens a segment
constexpr uint32_t kMaxSegRecords = 1u << 20;
constexpr uint32_t kSerMagic = 0xACED0005u;
constexpr int kLenRare = -2;          // lean_len: use the general path
constexpr int kEmitCap = 1024;        // record starts staged per emit window (u16 start | u16 stream length)

// Region l of a tile with valid aligned coordinates [lo, hi).
__device__ __forceinline__ void fregion(uint32_t lo, uint32_t hi, int l, uint32_t* rs, uint32_t* re) {
  uint32_t s = (uint32_t)l * kFRegion;
  uint32_t e = (l + 1 == kFOwn) ? (uint32_t)kTile : (uint32_t)(l + 1) * kFRegion;
  *rs = s < lo ? lo : s;
  *re = e > hi ? hi : e;
}

// ---------------------------------------------------------------------------------
// Per-tile context.
// ---------------------------------------------------------------------------------
struct FastCtx {
  const uint32_t* T;  // LDS image
  uint32_t lo, hi, img_end;
  uint32_t end_a;     // aligned coordinate of the span end
  uint64_t so;        // span offset of coordinate lo
  const TileDesc* tiles;
  uint32_t t, t1;     // this tile, end of the span's tile range
  uint32_t tables;    // Serializable tables exist (scan mode 1, emit)
  JserTabs J;
  // the own tile's table staged in LDS (k_fast_scan mode 1, k_fast_emit; null: read J from
  // HBM).  A lookup was a binary search of dependent HBM loads per Serializable record, per
  // lane -- the robust emit took 10x the fast one on config 3
  const uint32_t* lpos = nullptr;
  const uint32_t* llen = nullptr;
  uint32_t ln = 0;
  // the next tile of the span (t + 1 < t1): its table in LDS too, and its geometry -- the
  // chain's last segment and the scan's next-tile points run through it, and each lookup there
  // was a tile search plus a binary search of dependent HBM loads (config 3's robust emit:
  // 6 ms, 9x the fast one)
  const uint32_t* npos = nullptr;
  const uint32_t* nlen = nullptr;
  uint32_t nn = 0;
  uint64_t n_off = 0;  // span offset of tile t + 1 (its first valid byte)
  uint32_t n_len = 0, n_delta = 0;
};
// The tile's table into LDS (every lane of the wave calls it; it holds a barrier).
__device__ __forceinline__ uint32_t stage_jtab(const JserTabs& J, uint32_t t, uint32_t* s_p, uint32_t* s_l,
                                               uint32_t lane) {
  const uint32_t n0 = J.n[t], n = n0 < (uint32_t)kJserCap ? n0 : (uint32_t)kJserCap;
  for (uint32_t i = lane; i < n; i += 64) {
    s_p[i] = J.pos[(uint64_t)t * kJserCap + i];
    s_l[i] = J.len[(uint64_t)t * kJserCap + i];
  }
  __syncthreads();
  return n;
}

// The next tile's geometry and (tables) its table into LDS.  Every lane calls it (a barrier).
__device__ __forceinline__ void stage_next(FastCtx& c, const JserTabs& J, bool tables, uint32_t* s_p, uint32_t* s_l,
                                           uint32_t lane) {
  if (c.t + 1 >= c.t1) return;
  const TileDesc nd = c.tiles[c.t + 1];
  c.n_off = nd.span_off;
  c.n_len = nd.len;
  c.n_delta = nd.delta;
  if (tables) {
    c.nn = stage_jtab(J, c.t + 1, s_p, s_l, lane);
    c.npos = s_p;
    c.nlen = s_l;
  }
}

// Span tile holding aligned coordinate a (a >= hi) and its local coordinate.
__device__ __forceinline__ uint32_t far_tile(const FastCtx& c, uint32_t a, uint32_t* local) {
  const uint64_t o = c.so + (a - c.lo);
  if (c.n_len && o - c.n_off < c.n_len) {  // (o >= n_off: a >= hi)
    *local = (uint32_t)(o - c.n_off) + c.n_delta;
    return c.t + 1;
  }
  uint32_t k = c.t + 1;
  while (k + 1 < c.t1 && o >= c.tiles[k].span_off + c.tiles[k].len) ++k;
  *local = (uint32_t)(o - c.tiles[k].span_off) + c.tiles[k].delta;
  return k;
}

// A byte of the span past the LDS image (tile t + 1 on), out of line: inlined at every byte
// access of the general parsers, the tile search bloated the scan and emit code.
__device__ __noinline__ int far_byte(const TileDesc* tiles, uint32_t t, uint32_t t1, uint64_t o) {
  uint32_t k = t + 1;
  while (k + 1 < t1 && o >= tiles[k].span_off + tiles[k].len) ++k;
  return tiles[k].abase[(uint32_t)(o - tiles[k].span_off) + tiles[k].delta];
}

__device__ __forceinline__ int fbyte(const FastCtx& c, uint32_t a) {
  if (a < c.img_end) return (int)d_u8(c.T, a);
  if (a >= c.end_a) return -1;
  return far_byte(c.tiles, c.t, c.t1, c.so + (a - c.lo));
}

__device__ __forceinline__ int64_t jfind(const uint32_t* pos, const uint32_t* len, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pos[mid] < key) lo = mid + 1; else hi = mid;
  }
  return (lo < n && pos[lo] == key) ? (int64_t)len[lo] : -1;
}

// Length of the Serializable record at a (magic already checked): from the owning
// tile's table; without tables the tile must be deferred.
__device__ __forceinline__ int64_t fser_lookup(const FastCtx& c, uint32_t a, bool* defer) {
  if (!c.tables) {
    *defer = true;
    return kLenErr;
  }
  uint32_t k = c.t, local = a;
  if (a >= c.hi) k = far_tile(c, a, &local);
  int64_t j;
  if (k == c.t && c.lpos) {
    j = jfind(c.lpos, c.llen, c.ln, local);
  } else if (k == c.t + 1 && c.npos) {
    j = jfind(c.npos, c.nlen, c.nn, local);
  } else {
    const uint32_t n = c.J.n[k];
    j = jfind(c.J.pos + (uint64_t)k * kJserCap, c.J.len + (uint64_t)k * kJserCap, n < kJserCap ? n : kJserCap, local);
  }
  if (j <= 0) return kLenErr;
  const int64_t L = 1 + j;
  return ((uint64_t)a + (uint64_t)L > c.end_a) ? kLenErr : L;
}

struct FarBytes {
  const FastCtx* c;
  uint32_t base;
  __device__ __forceinline__ int operator()(uint64_t k) const { return fbyte(*c, base + (uint32_t)k); }
};

// Lean length for the common case, branch-free: tag + the next 4 bytes from two LDS
// dwords.  Tags 0,1,2,6,7 resolve here, as do bad tags and a 3 without the stream magic;
// 4, 5, a magic-bearing 3 and anything near the image end return kLenRare.
__device__ __forceinline__ int lean_len(const FastCtx& c, uint32_t a, int* tag) {
  const bool in = a + 32u <= c.img_end;
  const uint32_t ac = in ? a : 0u;
  const uint32_t k = ac >> 2, sh = 8u * (ac & 3u);
  const uint32_t d0 = c.T[k], d1 = c.T[k + 1];
  const uint32_t x0 = __builtin_amdgcn_alignbit(d1, d0, sh);  // bytes a..a+3 (LE)
  const uint32_t b4 = (d1 >> sh) & 0xFFu;                       // byte a+4
  const uint32_t tg = x0 & 0xFFu;
  *tag = (int)tg;
  constexpr uint64_t lut = 2ull | 9ull << 4 | 5ull << 8 | 13ull << 24 | 5ull << 28;  // nibble per tag, 0 = special
  const uint32_t L = (uint32_t)(lut >> (4u * (tg & 15u))) & 0xFu;
  const bool magic = ((x0 >> 8) | (b4 << 24)) == 0x0500EDACu;  // LE of AC ED 00 05
  const bool rare = !in || tg == 4u || tg == 5u || (tg == 3u && magic);
  const bool err = tg > 7u || (tg == 3u && !magic) || a + L > c.end_a;
  return rare ? kLenRare : (err ? (int)kLenErr : (int)L);
}

// General length (any tag, any position): kLenErr on any decode error.
__device__ __forceinline__ int64_t full_len(const FastCtx& c, uint32_t a, int* tag, bool* defer) {
  if (a >= c.end_a) return kLenErr;
  if (a + 27u < c.img_end) {
    DenseBytes b{c.T, a};
    const int tg = b(0);
    *tag = tg;
    const int64_t L = len_fields(b, tg, (uint64_t)(c.end_a - a));
    if (L != kLenSlow) return L;
    if (d_be32(c.T, a + 1) != kSerMagic) return kLenErr;
    return fser_lookup(c, a, defer);
  }
  FarBytes b{&c, a};
  const int tg = b(0);
  *tag = tg;
  const int64_t L = len_fields(b, tg, (uint64_t)(c.end_a - a));
  if (L != kLenSlow) return L;
  if (rd_be32(b, 1) != kSerMagic) return kLenErr;
  return fser_lookup(c, a, defer);
}

__device__ __forceinline__ int64_t flen(const FastCtx& c, uint32_t a, int* tag, bool* defer) {
  const int L = lean_len(c, a, tag);
  if (L != kLenRare) return L;
  return full_len(c, a, tag, defer);
}

// Full record at a (a on the resolved path).
__device__ __forceinline__ bool fdecode(const FastCtx& c, uint32_t a, Rec& r) {
  int tag;
  bool defer = false;
  const int64_t L = flen(c, a, &tag, &defer);
  if (L <= 0) return false;
  r.tag = (uint8_t)tag;
  r.L = (uint32_t)L;
  r.wide = (uint8_t)is_wide(tag);
  if (a + 27u < c.img_end) {
    DenseBytes b{c.T, a};
    decode_fields(b, tag, L, r);
  } else {
    FarBytes b{&c, a};
    decode_fields(b, tag, L, r);
  }
  return true;
}

// Stage the tile (dense) plus up to `halo` bytes of the span that follow it.
__device__ __forceinline__ uint32_t stage_dense(uint32_t* T, const TileDesc& td, const TileDesc* tiles, uint32_t t1,
                                                uint32_t t, uint64_t span_len, uint32_t halo_cap, uint32_t lane) {
  const uint32_t words = (td.delta + td.len + 15) >> 4;
  uint4* T4 = reinterpret_cast<uint4*>(T);
  const uint4* src = reinterpret_cast<const uint4*>(td.abase);
  for (uint32_t w = lane; w < words; w += 64) T4[w] = src[w];
  const uint32_t hi = td.delta + td.len;
  const uint64_t after = td.span_off + td.len;
  const uint64_t avail = span_len > after ? span_len - after : 0;
  const uint32_t halo = (uint32_t)(avail < (uint64_t)halo_cap ? avail : (uint64_t)halo_cap);
  if (halo) {
    uint8_t* bb = reinterpret_cast<uint8_t*>(T);
    uint32_t k = t + 1, got = 0;  // the halo may span several (short) tiles
    while (got < halo && k < t1) {
      const TileDesc nt = tiles[k];
      const uint32_t take = nt.len < halo - got ? nt.len : halo - got;
      if (((hi + got) & 15u) == 0 && nt.delta == 0) {
        const uint4* ns = reinterpret_cast<const uint4*>(nt.abase);
        uint4* dst = reinterpret_cast<uint4*>(bb + hi + got);
        for (uint32_t w = lane; w < (take + 15) / 16; w += 64) dst[w] = ns[w];
      } else {
        for (uint32_t i = lane; i < take; i += 64) bb[hi + got + i] = nt.abase[nt.delta + i];
      }
      got += take;
      ++k;
    }
  }
  __syncthreads();
  return hi + halo;
}

// Serializable magic patterns starting in [rs, re) of the padded DP image (k_jser_fill).
__device__ __forceinline__ uint32_t count_magic(const uint32_t* T, uint32_t rs, uint32_t re) {
  uint32_t n = 0;
  for (uint32_t k = rs >> 2; k < (re + 3) >> 2; ++k) {
    const uint32_t w = t_dw(T, k) ^ 0x03030303u;
    if (!((w - 0x01010101u) & ~w & 0x80808080u)) continue;
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t a = 4 * k + i;
      if (a < rs || a >= re) continue;
      if (t_u8(T, a) == CLG_TAG_SERIALIZABLE && t_be32(T, a + 1) == kSerMagic) ++n;
    }
  }
  return n;
}

// ---------------------------------------------------------------------------------
// Convergence (64-bit frontier BFS over candidate record starts).
// ---------------------------------------------------------------------------------
// Candidate starts in [rs, rs + n) whose byte is a valid tag (0..7): bit i <-> rs + i.
__device__ __forceinline__ uint64_t cand_mask(const FastCtx& c, uint32_t rs, uint32_t n) {
  uint64_t m = 0;
  if (rs + 40u <= c.img_end) {
    const uint32_t k0 = rs >> 2, sh = rs & 3u;
    for (uint32_t j = 0; j < 9; ++j) {  // 36 bytes cover 32 candidates at any alignment
      const uint32_t y = c.T[k0 + j] & 0xF8F8F8F8u;
      const uint32_t z = (y - 0x01010101u) & ~y & 0x80808080u;  // exact: bytes of y are 0 or >= 8
      const uint64_t bits = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
      m |= bits << (4 * j);
    }
    m >>= sh;
  } else {
    for (uint32_t i = 0; i < n; ++i) {
      const int b = fbyte(c, rs + i);
      if (b >= 0 && b <= 7) m |= 1ull << i;
    }
  }
  return m & ((n >= 64) ? ~0ull : ((1ull << n) - 1ull));
}

// Invariant inside the loop: the frontier's lowest position is W (bit 0 of M), so the
// popped candidate is W itself and its successor lands at bit L.  F holds at most one
// position >= W + 64; `sink` marks a path that ended exactly at the span end.  The common
// path is straight-line (selects); only a rare record (or the image end) branches.
__device__ uint32_t converge(const FastCtx& c, uint32_t rs, uint32_t ncand, uint32_t* pops, bool* defer) {
  if (rs >= c.end_a) return kConvUnknown;
  if (ncand > c.end_a - rs) ncand = c.end_a - rs;
  uint64_t M = ncand ? cand_mask(c, rs, ncand) : 0;
  if (M == 0) return kConvUnknown;
  uint32_t W = rs + (uint32_t)__builtin_ctzll(M);
  M >>= __builtin_ctzll(M);
  uint32_t F = kNoFar;
  bool sink = false;
  uint32_t res = kConvUnknown;
  int np = 0;
  for (; np < kMaxPops; ++np) {
    const bool m0 = M == 0, hasF = F != kNoFar;
    // frontier empty apart from the far slot: jump the window there
    W = m0 && hasF ? F : W;
    M = m0 && hasF ? 1ull : M;
    F = m0 ? kNoFar : F;
    const bool dead = m0 && !hasF;                     // only the sink (or nothing) is left
    const bool one = M == 1ull && F == kNoFar && !sink;  // a single live candidate: converged
    if (dead || one) {
      res = one ? W : (sink ? c.end_a : kConvUnknown);
      break;
    }
    M ^= 1ull;  // pop W
    const bool at_end = W >= c.end_a;
    sink = sink || at_end;
    int tag;
    int L = lean_len(c, W, &tag);
    L = at_end ? (int)kLenErr : L;
    if (L == kLenRare) {
      const int64_t LL = full_len(c, W, &tag, defer);
      if (LL >= 64) {  // long record: its successor goes to the far slot
        const uint32_t q = W + (uint32_t)LL;
        if (F != kNoFar && F != q) {
          np |= 0x4000;  // two far candidates: not tracked
          break;
        }
        F = q;
        L = (int)kLenErr;
      } else {
        L = (int)LL;
      }
    }
    M |= L > 0 ? (1ull << (uint32_t)L) : 0ull;
    const bool fm = F != kNoFar && F - W < 64u;
    M |= fm ? (1ull << ((F - W) & 63u)) : 0ull;
    F = fm ? kNoFar : F;
    const uint32_t lo = (uint32_t)M, hi = (uint32_t)(M >> 32);
    const uint32_t s = lo ? (uint32_t)__builtin_ctz(lo) : (hi ? 32u + (uint32_t)__builtin_ctz(hi) : 0u);
    M >>= s;
    W += s;
  }
  *pops = (uint32_t)np;
  return res;
}

// ---------------------------------------------------------------------------------
// Segments between kept points.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ int next_kept(const uint32_t* s_c, int from) {
  while (from < kFPoints && s_c[from] == kConvUnknown) ++from;
  return from;
}

// Parse from point l until landing exactly on a later kept point (jumping over a point
// means it is off the path: aim at the next one).
__device__ LaneSeg parse_segment(const FastCtx& c, const uint32_t* s_c, int l, bool* defer) {
  LaneSeg seg{kEndFail, 0, 0, 0, 0};
  const uint32_t c0 = s_c[l];
  if (c0 == kConvUnknown) return seg;
  uint32_t pos = c0, cnt = 0, w = 0;
  int m = next_kept(s_c, l + 1);
  uint32_t target = m < kFPoints ? s_c[m] : kConvUnknown;
  for (uint32_t it = 0; it < kMaxSegRecords; ++it) {
    if (target < pos) {
      while (target < pos) {
        m = next_kept(s_c, m + 1);
        target = m < kFPoints ? s_c[m] : kConvUnknown;
      }
    }
    int tag;
    int L = lean_len(c, pos, &tag);
    if (L == kLenRare) {
      const int64_t LL = full_len(c, pos, &tag, defer);
      L = LL > 0x7FFFFFF0ll ? (int)kLenErr : (int)LL;
    }
    const bool hit = target == pos;
    if (hit || L <= 0 || m >= kFPoints) {
      if (hit) {
        seg.end = (uint8_t)m;
        seg.cnt = cnt;
        seg.wcnt = w;
      } else if (m >= kFPoints && pos >= c.hi && c.t + 1 < c.t1 && pos - c.hi < 0xFFFFu) {
        // every next-tile point passed: the chain's next start, in the next tile (kEndFar)
        seg.end = kEndFar;
        seg.far = (uint16_t)(pos - c.hi);
        seg.cnt = cnt;
        seg.wcnt = w;
      }
      return seg;
    }
    ++cnt;
    w += is_wide(tag);
    pos += (uint32_t)L;
  }
  return seg;
}

// Kept points: known, inside the tile they belong to ([.., bound)), and above every
// earlier kept point of the same tile (a running maximum, so the rule needs no later
// points and the previous tile evaluates the next tile's first points exactly as it does).
__device__ __forceinline__ uint32_t keep_points(uint32_t pt, uint32_t bound, uint32_t lane) {
  const uint32_t v = (pt != kConvUnknown && pt < bound) ? pt : kConvUnknown;
  uint32_t key = v == kConvUnknown ? 0u : v + 1u;
  const uint32_t seg0 = lane < (uint32_t)kFOwn ? 0u : (uint32_t)kFOwn;
  uint32_t incl = key;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off);
    if (lane >= seg0 + (uint32_t)off) incl = incl > y ? incl : y;
  }
  uint32_t excl = __shfl_up(incl, 1);
  if (lane == seg0) excl = 0;
  return (v != kConvUnknown && key > excl) ? v : kConvUnknown;
}

// ---- pass F1: fused scan --------------------------------------------------------------
__global__ __launch_bounds__(64) void k_fast_scan(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                  uint32_t* __restrict__ conv, JserTabs J, uint32_t mode,
                                                  LaneSeg* __restrict__ lanes, TileSum* __restrict__ sums,
                                                  uint32_t* __restrict__ dbg, uint64_t* __restrict__ prof) {
  __shared__ uint32_t s_img[kScanImgDwords];
#define CLG_PHASE(i) \
  if (prof && lane == 0) prof[(uint64_t)t * 8 + (i)] = __builtin_amdgcn_s_memtime()

  __shared__ uint32_t s_c[kFPoints];
  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  if (mode == 1 && !J.defer[t]) return;
  const TileDesc td = tiles[t];
  const SpanDesc sd = spans[td.span];
  const uint32_t t1 = sd.first_tile + sd.n_tiles;
  const bool last = t + 1 == t1;
  const uint32_t hi = td.delta + td.len;
  const uint64_t ea = sd.len - td.span_off + td.delta;
  const uint32_t end_a = ea > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)ea;
  CLG_PHASE(0);
  const uint32_t img_end = stage_dense(s_img, td, tiles, t1, t, sd.len, kScanHalo, lane);
  CLG_PHASE(1);
  uint32_t rs = 0, re = 0;
  if (lane < (uint32_t)kFOwn) fregion(td.delta, hi, (int)lane, &rs, &re);
  // No pre-scan for Serializable records: every record the BFS or the parse touches goes
  // through fser_lookup, which (mode 0, no tables yet) defers the tile.
  __shared__ uint32_t s_jp[kJserCap], s_jl[kJserCap];
  const uint32_t jn = mode == 1 ? stage_jtab(J, t, s_jp, s_jl, lane) : 0u;
  FastCtx c{s_img, td.delta, hi, img_end, end_a, td.span_off, tiles, t, t1, mode, J,
            mode == 1 ? s_jp : nullptr, mode == 1 ? s_jl : nullptr, jn};
  __shared__ uint32_t s_np[kJserCap], s_nl[kJserCap];
  stage_next(c, J, mode == 1, s_np, s_nl, lane);
  bool defer = false;
  CLG_PHASE(2);

  // ---- convergence points: own regions, then the next tile's first kFNext regions
  // (one call site for every lane: the wave runs a single BFS loop)
  uint32_t pt = kConvUnknown, pops = 0, bound = hi, brs = 0, bn = 0;
  if (lane < (uint32_t)kFOwn) {
    if (lane == 0 && t == sd.first_tile) pt = td.delta;  // a span starts on a record boundary
    else if (re > rs) {
      brs = rs;
      bn = re - rs;
    }
  } else if (!last) {
    const TileDesc nd = tiles[t + 1];
    uint32_t nrs, nre;
    fregion(nd.delta, nd.delta + nd.len, (int)lane - kFOwn, &nrs, &nre);
    bound = hi + nd.len;
    if (nre > nrs) {
      brs = hi + (nrs - nd.delta);
      bn = nre - nrs;
    }
  } else if (lane == (uint32_t)kFOwn) {
    pt = end_a;  // the span end closes the last tile
    bound = end_a + 1;
  }
  if (bn) pt = converge(c, brs, bn < (uint32_t)kCands ? bn : (uint32_t)kCands, &pops, &defer);
  if (mode == 0 && __any(defer)) {
    if (lane == 0) J.defer[t] = 1;
    return;
  }
  CLG_PHASE(3);
  const uint32_t kept = keep_points(pt, bound, lane);
  s_c[lane] = kept;
  conv[(uint64_t)t * kFPoints + lane] = kept;
  if (dbg) dbg[(uint64_t)t * kFPoints + lane] = pops | (pt == kConvUnknown ? 0x80000000u : 0u);
  __syncthreads();

  // ---- segments and the chain from the first kept point
  CLG_PHASE(4);
  LaneSeg seg{kEndFail, 0, 0, 0, 0};
  if (lane < (uint32_t)kFOwn) seg = parse_segment(c, s_c, (int)lane, &defer);
  CLG_PHASE(5);
  if (mode == 0 && __any(defer)) {
    if (lane == 0) J.defer[t] = 1;
    return;
  }
  if (mode == 0 && lane == 0) {
    J.defer[t] = 0;
    J.n[t] = 0;
  }
  lanes[(uint64_t)t * kFPoints + lane] = seg;
  const uint64_t own_kept = __ballot(lane < (uint32_t)kFOwn && kept != kConvUnknown);
  const int f = own_kept ? __builtin_ctzll(own_kept) : kFPoints;
  const uint32_t g_end = seg.end, g_cnt = seg.cnt, g_w = seg.wcnt, g_far = seg.far;
  uint64_t valid = 0;
  uint32_t cnt = 0, w = 0, far = 0;
  int v = f;
  while (v < kFOwn) {
    const uint32_t e = __builtin_amdgcn_readlane(g_end, v);
    if (e == kEndFail) break;
    valid |= 1ull << v;
    cnt += __builtin_amdgcn_readlane(g_cnt, v);
    w += __builtin_amdgcn_readlane(g_w, v);
    if (e == kEndFar) far = __builtin_amdgcn_readlane(g_far, v);
    v = (int)e;
  }
  if (lane == 0) {
    TileSum sm{};
    sm.f = f < kFOwn ? (uint8_t)f : kEndFail;
    sm.x = v == (int)kEndFar ? kEndFar : (v >= kFOwn && v < kFPoints) ? (uint8_t)(v - kFOwn) : kEndFail;
    sm.far = (uint16_t)far;
    sm.cnt = cnt;
    sm.wcnt = w;
    sm.valid = valid;
    sums[t] = sm;
  }
  CLG_PHASE(6);
#undef CLG_PHASE
}

// ---- Serializable stream-length tables for deferred tiles --------------------------------
// Record length of the candidate at a for the two common stream shapes, over a byte reader
// (the fused path's inline shapes, decode_fused.hip jser_inline_len / jser_flat_len): a
// TC_STRING, and one TC_OBJECT whose class and superclasses are fresh TC_CLASSDESCs with flags
// SC_SERIALIZABLE only, primitive fields only and an empty annotation.  *general: some other
// shape -- the grammar walker decides.  0 with *general clear: the stream runs past the span.
template <class R>
__device__ uint32_t jser_inline_len_r(R& r, uint32_t a, uint64_t avail, bool* general) {
  auto b = [&](uint32_t q) { return (uint32_t)r.at(q); };
  auto u16 = [&](uint32_t q) { return b(q) << 8 | b(q + 1); };
  *general = false;
  if (avail < 8) {
    *general = true;
    return 0u;
  }
  const uint32_t tc = b(a + 5);
  // bytes [q, q + n) as readUTF takes them (modified UTF-8, jser_flat.h jf_mutf; byte by byte:
  // the reader is not asked for bytes past them)
  auto mutf = [&](uint32_t q, uint32_t n) {
    for (uint32_t i = 0; i < n;) {
      const uint32_t b1 = b(q + i);
      if (b1 < 0x80u) {
        ++i;
        continue;
      }
      const uint32_t k = (b1 >> 5) == 6u ? 2u : (b1 >> 4) == 14u ? 3u : 0u;
      if (!k || n - i < k || (b(q + i + 1) & 0xC0u) != 0x80u || (k == 3u && (b(q + i + 2) & 0xC0u) != 0x80u))
        return false;
      i += k;
    }
    return true;
  };
  if (tc == jser::TC_STRING) {  // [03][AC ED 00 05][74][len u16][modified UTF-8]
    const uint64_t L = 8ull + u16(a + 6);
    return L <= avail && mutf(a + 8, (uint32_t)L - 8u) ? (uint32_t)L : 0u;
  }
  *general = true;
  if (tc != jser::TC_OBJECT) return 0u;
  const uint64_t lim = avail < 4096 ? avail : 4096;  // (longer: the walker)
  uint32_t p = a + 6, data = 0;
  for (int depth = 0;; ++depth) {
    if (p + 1 > a + lim || depth > 8) return 0u;
    const uint32_t c = b(p);  // [TC_CLASSDESC][className length u16] or [TC_NULL]
    if (c == jser::TC_NULL && depth > 0) {  // no (further) superclass (a null class of the object
      ++p;                                   // itself: the walker, which rejects it)
      break;
    }
    if (c != jser::TC_CLASSDESC || p + 3 > a + lim) return 0u;
    const uint32_t nq = p + 3, nl = u16(p + 1);
    p += 3 + nl + 8;  // className, serialVersionUID
    if (p + 3 > a + lim || !mutf(nq, nl)) return 0u;
    if (b(p) != jser::SC_SERIALIZABLE) return 0u;
    const uint32_t nf = u16(p + 1);
    if (nf & 0x8000u) return 0u;
    p += 3;
    for (uint32_t i = 0; i < nf; ++i) {
      if (p + 3 > a + lim) return 0u;
      const uint32_t ft = b(p);  // [typecode][fieldName length u16]
      const uint32_t sz = ft == 'B' || ft == 'Z' ? 1u : ft == 'C' || ft == 'S' ? 2u : ft == 'I' || ft == 'F' ? 4u
                          : ft == 'J' || ft == 'D' ? 8u : 0u;
      if (!sz) return 0u;
      data += sz;
      const uint32_t fq = p + 3, fl = u16(p + 1);
      p += 3 + fl;
      if (p > a + lim || !mutf(fq, fl)) return 0u;  // the field name
    }
    if (p + 1 > a + lim || b(p) != jser::TC_ENDBLOCKDATA) return 0u;
    ++p;
  }
  p += data;
  if (p > a + lim) return 0u;
  *general = false;
  return p - a;
}

// A tile's table from the write path's sidecar (kernels.h SideCar): its segment's entries
// inside the tile, taken when every one has a length the writer measured that ends inside the
// span (the record length; the table holds the stream's, one less), ranked by position when
// the list is out of order.  false: not applicable -- outside the pool, an overflowed list,
// a candidate of unknown length or cut by the span's end (the caller scans the tile).
// Block-uniform (one wave); s_a, s_c: kJserCap words of LDS each.
__device__ __forceinline__ bool jfill_side(const TileDesc& td, const SpanDesc& sd, uint32_t t, const JserTabs& J,
                                           uint32_t lane, uint32_t* s_a, uint32_t* s_c) {
  const SideCar& S = J.side;
  const uintptr_t ab = (uintptr_t)td.abase, pb = (uintptr_t)S.pool;
  if (!S.hdr || ab < pb || ab - pb >= S.pool_bytes) return false;
  const uint64_t off = ab - pb;
  const uint32_t seg = (uint32_t)(off / S.seg_bytes), so0 = (uint32_t)(off % S.seg_bytes);
  const uint32_t n = (uint32_t)S.hdr[seg];
  if (n > S.cap) return false;
  const uint32_t lo = so0 + td.delta, hi = lo + td.len;
  const uint64_t end_a = sd.len - td.span_off + td.delta;  // the span's end, image coordinate
  const uint32_t* ent = S.ent + (size_t)seg * S.cap;
  uint32_t kept = 0;
  bool bad = false;
  for (uint32_t k0 = 0; k0 < n; k0 += 64u) {
    const uint32_t k = k0 + lane;
    bool in = false;
    uint32_t a = 0, code = 0;
    if (k < n) {
      const uint32_t e = ent[k];
      const uint32_t pos = e & 0xFFFFu;
      code = e >> 16;
      in = pos >= lo && pos < hi;
      a = pos - so0;
      bad = bad || (in && (code == kSideUnknown || (uint64_t)a + code > end_a));
    }
    const uint64_t m = __ballot(in);
    if (in) {
      const uint32_t i = kept + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      if (i < (uint32_t)kJserCap) {
        s_a[i] = a;
        s_c[i] = code;
      }
    }
    kept += (uint32_t)__popcll(m);
  }
  if (__ballot(bad) || kept > (uint32_t)kJserCap) return false;
  __syncthreads();
  bool sorted = true;
  for (uint32_t i = lane; i < kept; i += 64u)
    if (i && s_a[i - 1] >= s_a[i]) sorted = false;
  sorted = __ballot(!sorted) == 0;
  for (uint32_t i = lane; i < kept; i += 64u) {
    const uint32_t a = s_a[i];
    uint32_t r = i;
    if (!sorted) {
      r = 0;
      for (uint32_t j = 0; j < kept; ++j) r += s_a[j] < a || (s_a[j] == a && j < i) ? 1u : 0u;
    }
    J.pos[(uint64_t)t * kJserCap + r] = a;
    J.len[(uint64_t)t * kJserCap + r] = s_c[i] - 1u;
  }
  if (lane == 0) J.n[t] = kept;
  return true;
}

__global__ __launch_bounds__(64) void k_jser_fill(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                  JserTabs J) {
  __shared__ uint32_t s_tile[kImageDwords];
  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const TileDesc td = tiles[t];
  const SpanDesc sd = spans[td.span];
  // deferred tiles, and the successor of a deferred tile (its segment crossing the tile
  // end, and its next-tile points, may land on Serializable records there)
  if (!J.defer[t] && !(t > sd.first_tile && J.defer[t - 1])) return;
  if (jfill_side(td, sd, t, J, lane, s_tile, s_tile + kJserCap)) return;
  __syncthreads();  // (the image's words were the sidecar path's scratch)
  CLG_JPHASE(0);
  SpanReader sr{tiles, sd.first_tile, sd.first_tile + sd.n_tiles, t, sd.len, J.ar};
  stage_tile(s_tile, td, sr, lane);
  CLG_JPHASE(1);
  const TileGeom g{td.delta, td.delta + td.len};
  const uint32_t rs = g.rs((int)lane), re = g.re((int)lane);
  const uint32_t nm = re > rs ? count_magic(s_tile, rs, re) : 0u;
  uint32_t ex = nm;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(ex, off);
    if ((int)lane >= off) ex += y;
  }
  const uint32_t total = __shfl(ex, 63);
  uint32_t idx = ex - nm;
  if (lane == 0) J.n[t] = total;
  CLG_JPHASE(2);
  if (total == 0) return;
  // pass 1: the candidates count_magic found, in position order, into LDS by table index:
  // dwords holding a 03 byte, then their bytes (a byte-by-byte pass over the region read every
  // byte from LDS)
  __shared__ uint32_t s_cand[kJserCap];
  if (nm) {
    for (uint32_t a = rs; a < re; ++a) {
      if ((a & 3u) == 0u || a == rs) {
        const uint32_t w = t_dw(s_tile, a >> 2) ^ 0x03030303u;
        if (!((w - 0x01010101u) & ~w & 0x80808080u)) {
          a |= 3u;  // no 03 byte in this dword: on to the next
          continue;
        }
      }
      if (t_u8(s_tile, a) != CLG_TAG_SERIALIZABLE || t_be32(s_tile, a + 1) != kSerMagic) continue;
      if (idx < (uint32_t)kJserCap) s_cand[idx] = a;
      ++idx;
    }
  }
  __syncthreads();
  // pass 2: one stream per lane.  Parsed where the scan found them, a lane's stream held the
  // wave at each candidate position any lane reached: config 3's fill took 290 k cycles a tile
  // for ~70 streams.  The parsers read the stream from the tile's LDS image (HBM only past the
  // tile): byte by byte from HBM it took config 3's 5 M streams 285 ms
  TileReader tr{reinterpret_cast<const uint8_t*>(s_tile), td.delta, td.delta + td.len, td.span_off, &sr};
  uint32_t ncand = 0, ngen = 0;
  const uint32_t nc = total < (uint32_t)kJserCap ? total : (uint32_t)kJserCap;
  for (uint32_t i = lane; i < nc; i += 64) {
    const uint32_t a = s_cand[i];
    const uint64_t avail = sd.len - (td.span_off + (a - td.delta));
    bool general = false;
    int64_t L = jser_inline_len_r(tr, a, avail, &general);  // the common shapes inline
    ncand += 1;
    ngen += general;
    if (general) {
      // the walker through copies: its reader's address escapes into the call, and an escaping
      // tr / sr would live in scratch for the whole kernel
      SpanReader sr2 = sr;
      TileReader tr2{tr.lds, tr.lo, tr.hi, tr.so, &sr2};
      AtTileSpan b{&tr2, a};
      L = rec_len_slow(b, avail);  // walker: 1 + stream length
    }
    J.pos[(uint64_t)t * kJserCap + i] = a;
    J.len[(uint64_t)t * kJserCap + i] = L > 1 ? (uint32_t)(L - 1) : 0u;
  }
  if (J.prof) {
    __syncthreads();
    CLG_JPHASE(3);
    uint32_t mx = ncand, sc = ncand, sg = ngen;
    for (int off = 32; off; off >>= 1) {
      mx = max(mx, (uint32_t)__shfl_xor(mx, off));
      sc += __shfl_xor(sc, off);
      sg += __shfl_xor(sg, off);
    }
    if (lane == 0) {
      J.prof[(uint64_t)t * 16 + 4] = sc;
      J.prof[(uint64_t)t * 16 + 5] = sg;
      J.prof[(uint64_t)t * 16 + 6] = mx;
    }
  }
}

// ---- pass F2: per-span resolution ------------------------------------------------------
// *exit_idx: the next tile's point index, or -1 - far (a kEndFar exit, `far` bytes past the
// tile end).
__device__ bool chain_from(const LaneSeg* lanes, uint32_t t, int e, uint64_t* valid, uint32_t* cnt, uint32_t* wcnt,
                           int* exit_idx) {
  uint64_t vm = 0;
  uint32_t c = 0, w = 0;
  int v = e;
  while (v < kFOwn) {
    const LaneSeg gs = lanes[(uint64_t)t * kFPoints + v];
    if (gs.end == kEndFail) return false;
    vm |= 1ull << v;
    c += gs.cnt;
    w += gs.wcnt;
    if (gs.end == kEndFar) {
      *valid = vm;
      *cnt = c;
      *wcnt = w;
      *exit_idx = -1 - (int)gs.far;
      return true;
    }
    v = gs.end;
  }
  if (v >= kFPoints) return false;
  *valid = vm;
  *cnt = c;
  *wcnt = w;
  *exit_idx = v - kFOwn;
  return true;
}

// A chain that enters tile t at aligned coordinate `entry` (a kEndFar exit of the tile
// before): walked record by record from HBM (exact lengths) to the first of the tile's own
// kept points it lands on, *m, over *c records (*w wide).  false: the walk fails or passes
// every own point (the span goes to the DP).  Reads only: far_apply makes the result visible.
__device__ bool far_walk(const TileDesc* tiles, const SpanDesc& sd, uint32_t t, uint32_t entry, const uint32_t* conv,
                         const JserTabs& J, int* m_out, uint32_t* c_out, uint32_t* w_out) {
  const JArena ar = J.ar;
  const uint32_t jn0 = J.n[t], jn = jn0 < (uint32_t)kJserCap ? jn0 : (uint32_t)kJserCap;
  const TileDesc td = tiles[t];
  SpanReader sr{tiles, sd.first_tile, sd.first_tile + sd.n_tiles, t, sd.len, ar};
  const uint32_t* cv = conv + (uint64_t)t * kFPoints;
  int m = next_kept(cv, 0);
  uint32_t pos = entry, c = 0, w = 0;
  for (uint32_t it = 0; it < kMaxSegRecords; ++it) {
    while (m < kFOwn && cv[m] < pos) m = next_kept(cv, m + 1);
    if (m >= kFOwn) return false;
    if (cv[m] == pos) {
      *m_out = m;
      *c_out = c;
      *w_out = w;
      return true;
    }
    const uint64_t so = td.span_off + (pos - td.delta);
    if (so >= sd.len) return false;
    AtSpan b{&sr, so};
    const int tag = (int)b(0);
    // a Serializable record's length from the tile's table when it has the record (the
    // grammar walker reads the stream byte by byte from HBM)
    int64_t L = tag == CLG_TAG_SERIALIZABLE && jn
                    ? jfind(J.pos + (uint64_t)t * kJserCap, J.len + (uint64_t)t * kJserCap, jn, pos) : -1;
    L = L > 0 && rd_be32(b, 1) == kSerMagic && (uint64_t)(L + 1) <= sd.len - so ? L + 1 : rec_len_slow(b, sd.len - so);
    if (L <= 0) return false;
    ++c;
    w += is_wide(tag);
    pos += (uint32_t)L;
  }
  return false;
}

// The chain goes on from own point *e: the landing point itself when the walk is empty;
// else point 0, rewritten to start at the entry with the walk as (the head of) its segment,
// so that the chain, the counts and the emit (which parses cnt records from conv[0]) go
// through it like any other.
__device__ int far_apply(uint32_t t, uint32_t entry, int m, uint32_t c, uint32_t w, uint32_t* conv, LaneSeg* lanes) {
  if (c == 0) return m;
  LaneSeg* ls = lanes + (uint64_t)t * kFPoints;
  LaneSeg head{(uint8_t)m, 0, 0, c, w};
  if (m == 0) {  // the walk ends on point 0: it heads point 0's own segment
    head = ls[0];
    head.cnt += c;
    head.wcnt += w;
  }
  ls[0] = head;
  conv[(uint64_t)t * kFPoints] = entry;
  return 0;
}

// Exit codes: the next tile's point index (>= 0), or -1 - far (a kEndFar exit).
__device__ __forceinline__ int sum_exit(const TileSum& sm) {
  return sm.x == kEndFar ? -1 - (int)sm.far : (int)sm.x;
}

// The chain from own point e of tile t (sm: its summary from the first kept point f).  A chain
// that reaches f is f's chain from there on (k_fast_scan summarised it): the walk stops there.
// *head_c / *head_w: records before f (for the far case, which also rewrites point 0).
__device__ bool chain_sum(const LaneSeg* lanes, uint32_t t, int e, const TileSum& sm, uint64_t* valid,
                          uint32_t* cnt, uint32_t* wcnt, int* exit_idx) {
  if (e == (int)sm.f && sm.f != kEndFail) {
    if (sm.x == kEndFail) return false;
    *valid = sm.valid;
    *cnt = sm.cnt;
    *wcnt = sm.wcnt;
    *exit_idx = sum_exit(sm);
    return true;
  }
  return chain_from(lanes, t, e, valid, cnt, wcnt, exit_idx);
}

// Speculative per-tile resolution (one thread per tile): the tile's entry is taken to be the
// exit of the previous tile's chain from its first kept point (sums), which it is whenever
// that tile was itself entered on its chain from f -- every tile of a span of short records,
// and the tiles after a long record (a kEndFar exit), whose far walk lands on f.  The serial
// pass accepts a tile's result when the true entry matches and redoes only the others.
struct SpecRes {
  uint64_t valid;
  uint32_t cnt, wcnt;
  int spec;     // the entry assumed (exit code of the tile before; 0 for the span's first tile)
  int exit;     // exit code
  int fm;       // far walk: the landing point (-1: none)
  uint32_t fc, fw;
  uint32_t ok;
};

__device__ SpecRes spec_tile(const TileDesc* tiles, const SpanDesc& sd, uint32_t i, const uint32_t* conv,
                             const LaneSeg* lanes, const TileSum* sums, const JserTabs& J) {
  const uint32_t t = sd.first_tile + i;
  const TileSum sm = sums[t];
  SpecRes r{};
  r.fm = -1;
  r.ok = 0;
  r.spec = i == 0 ? 0 : sum_exit(sums[t - 1]);
  if (i > 0 && sums[t - 1].x == kEndFail) return r;
  int e = r.spec;
  if (e < 0) {
    const uint32_t entry = tiles[t].delta + (uint32_t)(-1 - e);
    int m;
    uint32_t c, w;
    if (!far_walk(tiles, sd, t, entry, conv, J, &m, &c, &w)) return r;
    if (c == 0) {
      e = m;
    } else {
      r.fm = m;
      r.fc = c;
      r.fw = w;
      // the chain from point 0 (rewritten): the walk, then m's chain
      uint64_t vm;
      uint32_t cc, ww;
      int x;
      if (!chain_sum(lanes, t, m, sm, &vm, &cc, &ww, &x)) return r;
      if (m == 0) {  // point 0's own segment follows the walk: m's chain starts with it
        r.valid = vm;
      } else {
        r.valid = vm | 1ull;
      }
      r.cnt = cc + c;
      r.wcnt = ww + w;
      r.exit = x;
      r.ok = 1;
      return r;
    }
  }
  uint64_t vm;
  uint32_t cc, ww;
  int x;
  if (!chain_sum(lanes, t, e, sm, &vm, &cc, &ww, &x)) return r;
  r.valid = vm;
  r.cnt = cc;
  r.wcnt = ww;
  r.exit = x;
  r.ok = 1;
  return r;
}

__global__ __launch_bounds__(256) void k_fast_resolve(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                      uint32_t* __restrict__ conv, LaneSeg* __restrict__ lanes,
                                                      const TileSum* __restrict__ sums, JserTabs J,
                                                      FastRes* __restrict__ fres, SpanRes* __restrict__ sres,
                                                      uint32_t* __restrict__ span_flags) {
  const uint32_t* jn = J.n;
  __shared__ uint64_t s_r[256], s_w[256];
  __shared__ uint32_t s_irregular, s_overflow;
  __shared__ uint64_t s_carry_r, s_carry_w;
  const uint32_t s = blockIdx.x;
  const SpanDesc sd = spans[s];
  if (threadIdx.x == 0) {
    s_irregular = 0;
    s_overflow = 0;
    s_carry_r = 0;
    s_carry_w = 0;
  }
  __syncthreads();
  // regular: every tile's entry is its first kept point (point 0 for the span's first
  // tile), the previous tile's chain lands on exactly that point, and the last tile's
  // chain lands on the span end (its point kFOwn + 0).
  for (uint32_t i = threadIdx.x; i < sd.n_tiles; i += blockDim.x) {
    const uint32_t t = sd.first_tile + i;
    const TileSum sm = sums[t];
    bool bad = sm.x == kEndFail || sm.f == kEndFail;
    if (i == 0) bad |= sm.f != 0;
    else bad |= sums[t - 1].x != sm.f;
    if (i + 1 == sd.n_tiles) bad |= sm.x != 0;
    if (bad) atomicOr(&s_irregular, 1u);
    if (jn[t] > (uint32_t)kJserCap) atomicOr(&s_overflow, 1u);
  }
  __syncthreads();
  if (s_overflow) {
    if (threadIdx.x == 0) span_flags[s] = 2u;  // (2: a table overflowed, 1: a chain broke; diagnostics)
    return;
  }
  if (!s_irregular) {
    for (uint32_t base = 0; base < sd.n_tiles; base += blockDim.x) {
      const uint32_t i = base + threadIdx.x;
      const TileSum sm = i < sd.n_tiles ? sums[sd.first_tile + i] : TileSum{};
      const uint64_t r = i < sd.n_tiles ? sm.cnt : 0, w = i < sd.n_tiles ? sm.wcnt : 0;
      s_r[threadIdx.x] = r;
      s_w[threadIdx.x] = w;
      __syncthreads();
      for (uint32_t off = 1; off < blockDim.x; off <<= 1) {
        const uint64_t ar = threadIdx.x >= off ? s_r[threadIdx.x - off] : 0;
        const uint64_t aw = threadIdx.x >= off ? s_w[threadIdx.x - off] : 0;
        __syncthreads();
        s_r[threadIdx.x] += ar;
        s_w[threadIdx.x] += aw;
        __syncthreads();
      }
      if (i < sd.n_tiles) fres[sd.first_tile + i] = FastRes{sm.valid, s_carry_r + s_r[threadIdx.x] - r,
                                                            s_carry_w + s_w[threadIdx.x] - w};
      __syncthreads();
      if (threadIdx.x == 0) {
        s_carry_r += s_r[blockDim.x - 1];
        s_carry_w += s_w[blockDim.x - 1];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      SpanRes r{};
      r.n_rec = s_carry_r;
      r.n_wide = s_carry_w;
      r.status = CLG_OK;
      r.err_off = -1;
      sres[s] = r;
      span_flags[s] = 0;
    }
    return;
  }
  // irregular: every tile resolved speculatively in parallel (spec_tile), then a serial pass
  // over the results accepts those whose entry was right and walks the others; a break goes
  // to the DP pipeline.  (Serially from HBM, chain by chain, it was config 3's robust
  // resolve: 3.2 ms, its spans broken by long Serializable records.)
  __shared__ SpecRes s_spec[256];
  __shared__ uint32_t s_fallback;
  __shared__ int s_e;
  if (threadIdx.x == 0) {
    s_fallback = 0;
    s_e = 0;
  }
  __syncthreads();
  for (uint32_t base = 0; base < sd.n_tiles; base += blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    if (i < sd.n_tiles) s_spec[threadIdx.x] = spec_tile(tiles, sd, i, conv, lanes, sums, J);
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t n = sd.n_tiles - base < blockDim.x ? sd.n_tiles - base : blockDim.x;
      uint64_t rec = s_carry_r, wide = s_carry_w;
      int e = s_e;
      bool fallback = false;
      for (uint32_t j = 0; j < n; ++j) {
        const uint32_t t = sd.first_tile + base + j;
        SpecRes& r = s_spec[j];
        s_r[j] = rec;
        s_w[j] = wide;
        if (r.ok && r.spec == e) {  // accepted: point 0's rewrite (if any) is applied below
          rec += r.cnt;
          wide += r.wcnt;
          e = r.exit;
          continue;
        }
        r.fm = -1;
        if (e < 0) {  // the tile before left by a kEndFar exit: enter at that record start
          const uint32_t entry = tiles[t].delta + (uint32_t)(-1 - e);
          int m;
          uint32_t c, w;
          if (!far_walk(tiles, sd, t, entry, conv, J, &m, &c, &w)) {
            fallback = true;
            break;
          }
          e = far_apply(t, entry, m, c, w, conv, lanes);
        }
        uint64_t vm;
        uint32_t c, w;
        int x;
        if (!chain_from(lanes, t, e, &vm, &c, &w, &x)) {
          fallback = true;
          break;
        }
        r.valid = vm;
        rec += c;
        wide += w;
        e = x;
      }
      s_carry_r = rec;
      s_carry_w = wide;
      s_e = e;
      if (fallback) s_fallback = 1;
    }
    __syncthreads();
    if (s_fallback) break;
    if (i < sd.n_tiles) {
      const uint32_t t = sd.first_tile + i;
      const SpecRes& r = s_spec[threadIdx.x];
      if (r.fm >= 0) far_apply(t, tiles[t].delta + (uint32_t)(-1 - r.spec), r.fm, r.fc, r.fw, conv, lanes);
      fres[t] = FastRes{r.valid, s_r[threadIdx.x], s_w[threadIdx.x]};
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const bool fallback = s_fallback || (sd.n_tiles && s_e != 0);
    SpanRes r{};
    r.n_rec = s_carry_r;
    r.n_wide = s_carry_w;
    r.status = CLG_OK;
    r.err_off = -1;
    sres[s] = r;
    span_flags[s] = fallback ? 1u : 0u;
  }
}

// ---- pass F3: emit ---------------------------------------------------------------------
// Phase A: each chain lane walks its segment and drops every record start (u16 image
// coordinate; a Serializable record's length above it, which phase A looked up already) at
// its output index in LDS.  Phase B: lane i decodes the i-th record of the window from 8
// dwords of the image, every tag's fields as selects (no per-tag branches, no second length
// lookup), so every SoA store of the wave covers consecutive output elements.
constexpr uint32_t kEmitLenNone = 0xFFFFu;  // a Serializable record too long for the entry: fdecode

template <int O>
__device__ __forceinline__ uint32_t xw(const uint32_t (&x)[7]) {  // bytes O..O+3 (LE) of the record
  return (O & 3) == 0 ? x[O >> 2] : __builtin_amdgcn_alignbit(x[(O >> 2) + 1], x[O >> 2], 8 * (O & 3));
}
template <int O>
__device__ __forceinline__ uint32_t xbe32(const uint32_t (&x)[7]) { return __builtin_bswap32(xw<O>(x)); }
template <int O>
__device__ __forceinline__ uint64_t xbe64(const uint32_t (&x)[7]) {
  return (uint64_t)xbe32<O>(x) << 32 | xbe32<O + 4>(x);
}
template <int O>
__device__ __forceinline__ uint32_t xb(const uint32_t (&x)[7]) { return (x[O >> 2] >> (8 * (O & 3))) & 0xFFu; }

// Exact length of the record at a on the chain, from 8 dwords of the image: every tag's
// length rule as selects (SimpleDeterminantEncoder.java:124-323), and a Serializable record's
// from the own tile's table through the lane's cursor (its entries are in position order and
// the lane walks forward: one compare per record instead of a binary search).  kLenRare:
// near the image end, past the tile, or anything unexpected -- the general path decides.
__device__ __forceinline__ int emit_len(const FastCtx& c, uint32_t a, int* tag, uint32_t* cur) {
  // one round of LDS reads and every rule as selects: the lanes of a wave step through their
  // segments together, and a branch per tag ran each rule's reads in turn at every step
  const bool in = a + 32u <= c.img_end && a < c.hi;
  const uint32_t ac = in ? a : 0u;
  const uint32_t kk = ac >> 2, sh = 8u * (ac & 3u);
  uint32_t d[8], x[7];
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = c.T[kk + j];
#pragma unroll
  for (int j = 0; j < 7; ++j) x[j] = __builtin_amdgcn_alignbit(d[j + 1], d[j], sh);
  const uint32_t tg = x[0] & 0xFFu;
  *tag = (int)tg;
  constexpr uint64_t lut = 2ull | 9ull << 4 | 5ull << 8 | 13ull << 24 | 5ull << 28;
  const int ordT = (int)(int8_t)xb<13>(x), ordS = (int)(int8_t)xb<21>(x);
  const int32_t nl = (int32_t)xbe32<14>(x), rl = (int32_t)xbe32<23>(x);
  const bool var = xb<22>(x) != 0u;
  const bool isT = tg == CLG_TAG_TIMER_TRIGGER, isS = tg == CLG_TAG_SOURCE_CHECKPOINT;
  const bool isJ = tg == CLG_TAG_SERIALIZABLE;
  const int64_t LT = ordT != 6 ? 14 : 18 + (int64_t)nl, LS = var ? 27 + (int64_t)rl : 23;
  const bool okT = ordT >= 0 && ordT <= 6 && (ordT != 6 || nl >= 0);
  const bool okS = ordS >= 0 && ordS <= 1 && (!var || rl >= 0);
  int64_t L = isT ? LT : isS ? LS : (int64_t)((lut >> (4u * (tg & 15u))) & 0xFu);
  bool ok = in && tg <= 7u && (!isT || okT) && (!isS || okS);
  if (isJ) {
    ok = ok && xw<1>(x) == 0x0500EDACu;  // LE of AC ED 00 05
    uint32_t k = *cur;
    while (k < c.ln && c.lpos[k] < a) ++k;
    *cur = k;
    const int64_t j = k < c.ln && c.lpos[k] == a ? (int64_t)c.llen[k] : -1;
    ok = ok && j > 0;
    L = 1 + j;
  }
  if (!ok || (uint64_t)L > (uint64_t)(c.end_a - a)) return kLenRare;
  return (int)L;
}

__global__ __launch_bounds__(64) void k_fast_emit(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                  const uint32_t* __restrict__ conv, JserTabs J,
                                                  const LaneSeg* __restrict__ lanes, const FastRes* __restrict__ fres,
                                                  const SpanRes* __restrict__ sres, const uint32_t* __restrict__ span_flags,
                                                  DecodeOut out) {
  __shared__ uint32_t s_img[kEmitImgDwords];
  __shared__ uint32_t s_pos[kEmitCap];
  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const TileDesc td = tiles[t];
  if (span_flags[td.span]) return;  // decoded by the DP pipeline
  const FastRes fr = fres[t];
  if (fr.valid == 0) return;
  CLG_JPHASE(8);
  const SpanDesc sd = spans[td.span];
  const SpanRes sp = sres[td.span];
  const uint32_t t1 = sd.first_tile + sd.n_tiles;
  const uint64_t ea = sd.len - td.span_off + td.delta;
  const uint32_t end_a = ea > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)ea;
  const bool mine = (fr.valid >> lane) & 1ull;
  const LaneSeg seg = lanes[(uint64_t)t * kFPoints + lane];
  uint32_t pos = conv[(uint64_t)t * kFPoints + lane];
  const uint32_t img_end = stage_dense(s_img, td, tiles, t1, t, sd.len, kEmitHalo, lane);
  CLG_JPHASE(9);
  __shared__ uint32_t s_jp[kJserCap], s_jl[kJserCap];
  const uint32_t jn = stage_jtab(J, t, s_jp, s_jl, lane);
  FastCtx c{s_img, td.delta, td.delta + td.len, img_end, end_a, td.span_off, tiles, t, t1, 1u, J, s_jp, s_jl, jn};
  __shared__ uint32_t s_np[kJserCap], s_nl[kJserCap];
  stage_next(c, J, true, s_np, s_nl, lane);
  CLG_JPHASE(10);

  const uint32_t cn = mine ? seg.cnt : 0u;
  uint32_t ic = cn;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(ic, off);
    if ((int)lane >= off) ic += y;
  }
  const uint32_t total = __shfl(ic, 63);
  uint32_t idx = ic - cn, k = 0;
  const uint64_t rec0 = sp.rec_base + fr.rec_base;
  uint64_t wide = sp.wide_base + fr.wide_base;
  uint32_t nfar = 0, nrare = 0;
  // the lane's cursor into the own table: its first entry at or after the segment start
  uint32_t jcur = 0;
  if (cn) {
    uint32_t hi_i = jn;
    while (jcur < hi_i) {
      const uint32_t mid = (jcur + hi_i) >> 1;
      if (s_jp[mid] < pos) jcur = mid + 1; else hi_i = mid;
    }
  }
  for (uint32_t w0 = 0; w0 < total; w0 += kEmitCap) {
    const uint32_t wend = w0 + kEmitCap;
    while (k < cn && idx < wend) {  // phase A
      if (J.prof) {
        nfar += pos + 27u >= img_end;
        nrare += pos + 32u > img_end || (s_img[pos >> 2] >> (8 * (pos & 3)) & 0xFFu) - 3u <= 3u;
      }
      int tag;
      int L = emit_len(c, pos, &tag, &jcur);
      if (L == kLenRare) {
        bool defer = false;
        const int64_t LL = full_len(c, pos, &tag, &defer);
        L = LL > 0x7FFFFFF0ll ? (int)kLenErr : (int)LL;
      }
      const uint32_t jl = tag == CLG_TAG_SERIALIZABLE && L > 1 && L - 1 < (int)kEmitLenNone ? (uint32_t)(L - 1)
                                                                                             : kEmitLenNone;
      s_pos[idx - w0] = (pos & 0xFFFFu) | jl << 16;
      pos += L > 0 ? (uint32_t)L : 1u;
      ++k;
      ++idx;
    }
    __syncthreads();
    CLG_JPHASE(11);
    const uint32_t nw = total - w0 < (uint32_t)kEmitCap ? total - w0 : (uint32_t)kEmitCap;
    for (uint32_t i0 = 0; i0 < nw; i0 += 64) {  // phase B
      const uint32_t i = i0 + lane;
      const bool act = i < nw;
      const uint32_t ent = act ? s_pos[i] : td.delta;
      const uint32_t a = ent & 0xFFFFu, jl = ent >> 16;
      const bool in = a + 32u <= img_end;
      const uint32_t ac = in ? a : 0u;
      const uint32_t kk = ac >> 2, sh = 8u * (ac & 3u);
      uint32_t d[8], x[7];
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = s_img[kk + j];
#pragma unroll
      for (int j = 0; j < 7; ++j) x[j] = __builtin_amdgcn_alignbit(d[j + 1], d[j], sh);
      uint32_t tg = x[0] & 0xFFu;
      // every tag's fields (SimpleDeterminantEncoder readers :116-341), selected by tag
      const int64_t be64_1 = (int64_t)xbe64<1>(x), be64_5 = (int64_t)xbe64<5>(x);
      const int32_t be32_1 = (int32_t)xbe32<1>(x);
      const bool wide_t = tg >= 3u && tg <= 6u;
      int64_t v0 = tg == CLG_TAG_ORDER ? (int64_t)(int8_t)xb<1>(x)
                 : tg == CLG_TAG_TIMESTAMP ? be64_1
                 : tg == CLG_TAG_SERIALIZABLE ? (int64_t)jl
                 : wide_t ? be64_5 : (int64_t)be32_1;
      Rec r{};
      r.rc = wide_t && tg != CLG_TAG_SERIALIZABLE ? be32_1 : 0;
      r.v1 = tg == CLG_TAG_SOURCE_CHECKPOINT ? (int64_t)xbe64<13>(x) : 0;
      const uint32_t b13 = xb<13>(x), b21 = xb<21>(x), b22 = xb<22>(x);
      const bool tvar = tg == CLG_TAG_TIMER_TRIGGER && b13 == 6u;
      const bool svar = tg == CLG_TAG_SOURCE_CHECKPOINT && b22 != 0u;
      r.sub = (uint8_t)(tg == CLG_TAG_TIMER_TRIGGER ? b13 : tg == CLG_TAG_SOURCE_CHECKPOINT ? (b21 | (svar ? 0x80u : 0u)) : 0u);
      r.var_off = tg == CLG_TAG_SERIALIZABLE ? 1u : tvar ? 18u : svar ? 27u : 0u;
      r.var_len = tg == CLG_TAG_SERIALIZABLE ? jl : tvar ? xbe32<14>(x) : svar ? xbe32<23>(x) : 0u;
      bool wide_rec = wide_t;
      if (act && (!in || (tg == CLG_TAG_SERIALIZABLE && jl == kEmitLenNone))) {
        // near the image end, or a Serializable stream too long for the entry: the general decoder
        if (fdecode(c, a, r)) {
          tg = r.tag;
          v0 = r.v0;
          wide_rec = r.wide;
        }
      }
      const uint64_t wm = __ballot(act && wide_rec);
      const uint64_t g = rec0 + w0 + i;
      if (act) {
        const uint32_t so = (uint32_t)(td.span_off + (a - td.delta));
        if (g < out.cap) {
          out.off[g] = so;
          out.tag[g] = (uint8_t)tg;
          out.v0[g] = v0;
        }
        if (wide_rec) {
          const uint64_t wi = wide + (uint64_t)__popcll(wm & ((1ull << lane) - 1ull));
          if (wi < out.wcap) {
            out.w_idx[wi] = (uint32_t)g;
            out.w_rc[wi] = r.rc;
            out.w_v1[wi] = r.v1;
            out.w_var_off[wi] = r.var_off ? so + r.var_off : 0u;
            out.w_var_len[wi] = r.var_len;
            out.w_sub[wi] = r.sub;
          }
        }
      }
      wide += (uint64_t)__popcll(wm);
    }
    __syncthreads();
  }
  CLG_JPHASE(12);
  if (J.prof) {
    uint32_t mx = cn, sf = nfar, sr = nrare;
    for (int off = 32; off; off >>= 1) {
      mx = max(mx, (uint32_t)__shfl_xor(mx, off));
      sf += __shfl_xor(sf, off);
      sr += __shfl_xor(sr, off);
    }
    if (lane == 0) {
      J.prof[(uint64_t)t * 16 + 13] = sf;
      J.prof[(uint64_t)t * 16 + 14] = mx;
      J.prof[(uint64_t)t * 16 + 15] = (uint64_t)total | (uint64_t)sr << 32;
    }
  }
}

// ---------------------------------------------------------------------------------
// Launchers.
// ---------------------------------------------------------------------------------
static int ok(hipError_t e) { return launch_status(e); }

int launch_fast_scan(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, uint32_t* d_conv, JserTabs J,
                     uint32_t mode, LaneSeg* d_lanes, TileSum* d_sums, uint32_t* d_dbg, uint64_t* d_prof, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_fast_scan, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, d_conv, J, mode,
                     d_lanes, d_sums, d_dbg, d_prof);
  return ok(hipGetLastError());
}

int launch_jser_fill(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, JserTabs J, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_jser_fill, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, J);
  return ok(hipGetLastError());
}

int launch_fast_resolve(const TileDesc* d_tiles, const SpanDesc* d_spans, uint32_t n_spans, uint32_t* d_conv,
                        LaneSeg* d_lanes, const TileSum* d_sums, JserTabs J, FastRes* d_fres, SpanRes* d_sres,
                        uint32_t* d_span_flags, JArena ar, void* stream) {
  if (!n_spans) return CLG_OK;
  J.ar = ar;
  hipLaunchKernelGGL(k_fast_resolve, dim3(n_spans), dim3(256), 0, (hipStream_t)stream, d_tiles, d_spans, d_conv, d_lanes,
                     d_sums, J, d_fres, d_sres, d_span_flags);
  return ok(hipGetLastError());
}

int launch_fast_emit(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, const uint32_t* d_conv,
                     JserTabs J, const LaneSeg* d_lanes, const FastRes* d_fres, const SpanRes* d_sres,
                     const uint32_t* d_span_flags, DecodeOut out, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_fast_emit, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, d_conv, J, d_lanes,
                     d_fres, d_sres, d_span_flags, out);
  return ok(hipGetLastError());
}

}  // namespace clg
