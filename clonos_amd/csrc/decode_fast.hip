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
// Serializable records (tag 3) have no length prefix: their stream lengths come from a
// per-tile table filled by k_jser_fill (the only kernel here that calls the out-of-line
// grammar walker), so the hot kernels stay call-free.  k_fast_conv's first pass detects
// tiles holding a "03 AC ED 00 05" pattern and defers them until the table exists.
//
// Record layouts: SimpleDeterminantEncoder.java:124-323 (reference flink-runtime).
#include "dev_slow.h"

namespace clg {

constexpr int kFastRows = (kTile + kFastHalo) / kRegion + 1;
constexpr int kFastImageDwords = kFastRows * kPitch;
constexpr uint64_t kNoFar = ~0ull;
constexpr int kMaxPops = 192;          // give up early: an unknown point only lengthens a segment
constexpr int kMaxSegRecords = 1 << 15;
constexpr uint32_t kSerMagic = 0xACED0005u;

// ---------------------------------------------------------------------------------
// Per-tile context: LDS image + where everything else lives.
// ---------------------------------------------------------------------------------
struct FastCtx {
  const uint32_t* T;  // LDS image
  uint32_t lo, hi, img_end;
  uint64_t end_a;     // aligned coordinate of the span end
  uint64_t so;        // span offset of coordinate lo
  const TileDesc* tiles;
  uint32_t t, t1;     // this tile, end of the span's tile range
  const uint32_t* s_jpos;  // own Serializable table (LDS)
  const uint32_t* s_jlen;
  uint32_t s_jn;
  JserTabs J;         // all tables (global)
};

// Span tile holding aligned coordinate a (a >= hi) and its local coordinate.
__device__ __forceinline__ uint32_t far_tile(const FastCtx& c, uint32_t a, uint32_t* local) {
  const uint64_t o = c.so + (a - c.lo);
  uint32_t k = c.t + 1;
  while (k + 1 < c.t1 && o >= c.tiles[k].span_off + c.tiles[k].len) ++k;
  *local = (uint32_t)(o - c.tiles[k].span_off) + c.tiles[k].delta;
  return k;
}

__device__ __forceinline__ int fbyte(const FastCtx& c, uint32_t a) {
  if (a < c.img_end) return t_u8(c.T, a);
  if ((uint64_t)a >= c.end_a) return -1;
  uint32_t local;
  const uint32_t k = far_tile(c, a, &local);
  return c.tiles[k].abase[local];
}

__device__ __forceinline__ int64_t jfind(const uint32_t* pos, const uint32_t* len, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pos[mid] < key) lo = mid + 1; else hi = mid;
  }
  return (lo < n && pos[lo] == key) ? (int64_t)len[lo] : -1;
}

// Length of the Serializable record at a (magic already checked).
__device__ __forceinline__ int64_t fser(const FastCtx& c, uint32_t a) {
  int64_t j;
  if (a < c.hi) {
    j = jfind(c.s_jpos, c.s_jlen, c.s_jn, a);
  } else {
    uint32_t local;
    const uint32_t k = far_tile(c, a, &local);
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

// Record length at aligned coordinate a (< end_a); kLenErr for any decode error.
__device__ __forceinline__ int64_t flen(const FastCtx& c, uint32_t a, int* tag) {
  if (a + 27u < c.img_end) {
    const int tg = t_u8(c.T, a);
    *tag = tg;
    const int64_t L = len_inline(c.T, tg, a, c.end_a);
    return L == kLenSlow ? fser(c, a) : L;
  }
  FarBytes b{&c, a};
  const int tg = b(0);
  *tag = tg;
  const int64_t L = len_fields(b, tg, c.end_a - a);
  if (L != kLenSlow) return L;
  if (rd_be32(b, 1) != kSerMagic) return kLenErr;
  return fser(c, a);
}

// Full record at a (a on the resolved path).
__device__ __forceinline__ bool fdecode(const FastCtx& c, uint32_t a, Rec& r) {
  int tag;
  const int64_t L = flen(c, a, &tag);
  if (L <= 0) return false;
  r.tag = (uint8_t)tag;
  r.L = (uint32_t)L;
  r.wide = (uint8_t)is_wide(tag);
  if (a + 27u < c.img_end) {
    LdsBytes b{c.T, a};
    decode_fields(b, tag, L, r);
  } else {
    FarBytes b{&c, a};
    decode_fields(b, tag, L, r);
  }
  return true;
}

// Stage the tile plus up to kFastHalo bytes of the span that follow it.
__device__ __forceinline__ uint32_t stage_fast(uint32_t* s_tile, const TileDesc& td, const TileDesc* tiles,
                                               uint32_t t1, uint32_t t, uint64_t span_len, uint32_t lane) {
  const uint32_t words = (td.delta + td.len + 15) >> 4;
  for (uint32_t w = lane; w < words; w += 64) {
    const uint4 v = *reinterpret_cast<const uint4*>(td.abase + 16 * w);
    const uint32_t d = (w >> 4) * kPitch + ((w & 15u) << 2);
    s_tile[d + 0] = v.x;
    s_tile[d + 1] = v.y;
    s_tile[d + 2] = v.z;
    s_tile[d + 3] = v.w;
  }
  const uint32_t hi = td.delta + td.len;
  const uint64_t after = td.span_off + td.len;
  const uint64_t avail = span_len > after ? span_len - after : 0;
  const uint32_t halo = (uint32_t)(avail < (uint64_t)kFastHalo ? avail : (uint64_t)kFastHalo);
  __syncthreads();
  if (halo) {
    uint8_t* bb = reinterpret_cast<uint8_t*>(s_tile);
    uint32_t k = t + 1, got = 0;  // the halo may span several (short) tiles
    while (got < halo && k < t1) {
      const TileDesc nt = tiles[k];
      const uint32_t take = nt.len < halo - got ? nt.len : halo - got;
      if (((hi + got) & 15u) == 0 && nt.delta == 0) {
        for (uint32_t w = lane; w < (take + 15) / 16; w += 64) {
          const uint4 v = *reinterpret_cast<const uint4*>(nt.abase + 16 * w);
          const uint32_t a = hi + got + 16 * w;
          const uint32_t d = (a >> 8) * kPitch + ((a >> 2) & 63u);
          s_tile[d + 0] = v.x;
          s_tile[d + 1] = v.y;
          s_tile[d + 2] = v.z;
          s_tile[d + 3] = v.w;
        }
      } else {
        for (uint32_t i = lane; i < take; i += 64) {
          const uint32_t a = hi + got + i;
          bb[(a >> 8) * (kPitch * 4) + (a & 255u)] = nt.abase[nt.delta + i];
        }
      }
      got += take;
      ++k;
    }
    __syncthreads();
  }
  return hi + halo;
}

// Serializable magic positions in [rs, re): count (and optionally list via callback).
__device__ __forceinline__ uint32_t count_magic(const uint32_t* T, uint32_t rs, uint32_t re) {
  uint32_t n = 0;
  for (uint32_t k = rs >> 2; k < (re + 3) >> 2; ++k) {
    const uint32_t w = t_dw(T, k) ^ 0x03030303u;
    if (!((w - 0x01010101u) & ~w & 0x80808080u)) continue;  // no 0x03 byte in this dword
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
// Candidate starts whose tag byte is a valid tag (0..7): bit i <-> position rs + i.
__device__ __forceinline__ uint64_t valid_tag_mask(const uint32_t* T, uint32_t rs, uint32_t ncand) {
  uint64_t m = 0;
  const uint32_t k0 = rs >> 2, sh = rs & 3u;
  for (uint32_t j = 0; j < 10; ++j) {  // 40 bytes cover 32 candidates at any alignment
    const uint32_t y = t_dw(T, k0 + j) & 0xF8F8F8F8u;
    const uint32_t z = (y - 0x01010101u) & ~y & 0x80808080u;  // exact: bytes of y are 0 or >= 8
    const uint64_t bits = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
    m |= bits << (4 * j);
  }
  m >>= sh;
  const uint64_t want = ncand >= 64 ? ~0ull : ((1ull << ncand) - 1ull);
  return m & want;
}

__device__ uint32_t converge(const FastCtx& c, uint32_t rs, uint32_t ncand, uint32_t* pops) {
  if (ncand == 0) return kConvUnknown;
  uint64_t M = (rs + 40u + 4u < c.img_end) ? valid_tag_mask(c.T, rs, ncand)
                                            : (ncand >= 64 ? ~0ull : ((1ull << ncand) - 1ull));
  uint64_t W = rs;
  uint64_t F = kNoFar;
  bool sink = false;  // some candidate ended exactly at the span end
  int npop = 0;
  for (; npop < kMaxPops; ++npop) {
    const int n = __popcll(M) + (F != kNoFar ? 1 : 0) + (sink ? 1 : 0);
    if (n <= 1) {
      *pops = (uint32_t)npop | ((uint32_t)n << 16);
      if (n == 0) return kConvUnknown;
      if (M) return (uint32_t)(W + (uint64_t)(__ffsll((long long)M) - 1));
      if (F != kNoFar) return F > 0xFFFFFFF0ull ? kConvUnknown : (uint32_t)F;
      return c.end_a > 0xFFFFFFF0ull ? kConvUnknown : (uint32_t)c.end_a;
    }
    if (M == 0) {  // only the far slot (and maybe the sink) left: jump the window
      W = F;
      M = 1;
      F = kNoFar;
      continue;
    }
    const int b = __ffsll((long long)M) - 1;
    const uint64_t p = W + (uint64_t)b;
    M &= M - 1;
    if (p >= c.end_a) {
      sink = true;
    } else {
      int tag;
      const int64_t L = flen(c, (uint32_t)p, &tag);
      if (L > 0) {
        const uint64_t q = p + (uint64_t)L;
        if (q < W + 64) {
          M |= 1ull << (q - W);
        } else if (F == kNoFar || F == q) {
          F = q;
        } else {
          *pops = (uint32_t)npop | 0x80000000u;
          return kConvUnknown;  // two candidates far ahead: not tracked
        }
      }
    }
    if (M) {
      const int s = __ffsll((long long)M) - 1;
      if (s) {
        M >>= s;
        W += (uint64_t)s;
      }
    }
    if (F != kNoFar && F < W + 64) {
      M |= 1ull << (F - W);
      F = kNoFar;
    }
  }
  *pops = (uint32_t)npop;
  return kConvUnknown;
}

__device__ __forceinline__ void load_jtab(uint32_t* s_jpos, uint32_t* s_jlen, uint32_t* s_jn, const JserTabs& J,
                                          uint32_t t, uint32_t lane) {
  const uint32_t n = J.n[t];
  const uint32_t m = n < kJserCap ? n : kJserCap;
  for (uint32_t i = lane; i < m; i += 64) {
    s_jpos[i] = J.pos[(uint64_t)t * kJserCap + i];
    s_jlen[i] = J.len[(uint64_t)t * kJserCap + i];
  }
  if (lane == 0) *s_jn = m;
}

// ---- pass F1: convergence points (mode 0: every tile, tiles with Serializable
// records are deferred; mode 1: the deferred tiles, tables filled) -----------------------
__global__ __launch_bounds__(64) void k_fast_conv(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                  uint32_t* __restrict__ conv, JserTabs J, uint32_t mode,
                                                  uint32_t* __restrict__ dbg) {
  __shared__ uint32_t s_tile[kFastImageDwords];
  __shared__ uint32_t s_jpos[kJserCap], s_jlen[kJserCap];
  __shared__ uint32_t s_jn;
  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  if (mode == 1 && !J.defer[t]) return;
  const TileDesc td = tiles[t];
  const SpanDesc sd = spans[td.span];
  const uint32_t t1 = sd.first_tile + sd.n_tiles;
  if (mode == 1) {
    load_jtab(s_jpos, s_jlen, &s_jn, J, t, lane);
  } else if (lane == 0) {
    s_jn = 0;
  }
  const uint32_t img_end = stage_fast(s_tile, td, tiles, t1, t, sd.len, lane);
  const TileGeom g{td.delta, td.delta + td.len};
  const uint32_t rs = g.rs((int)lane), re = g.re((int)lane);
  if (mode == 0) {
    const uint32_t nm = re > rs ? count_magic(s_tile, rs, re) : 0u;
    if (__any(nm != 0)) {  // Serializable records here: wait for the stream-length table
      if (lane == 0) J.defer[t] = 1;
      return;
    }
    if (lane == 0) {
      J.defer[t] = 0;
      J.n[t] = 0;
    }
  }
  const FastCtx c{s_tile, td.delta, td.delta + td.len, img_end, sd.len - td.span_off + td.delta, td.span_off, tiles,
                  t, t1, s_jpos, s_jlen, s_jn, J};
  uint32_t pt, pops = 0;
  if (lane == 0 && t == sd.first_tile) {
    pt = td.delta;  // a span starts on a record boundary
  } else {
    const uint32_t RL = re > rs ? re - rs : 0;
    pt = converge(c, rs, RL < (uint32_t)kCands ? RL : (uint32_t)kCands, &pops);
  }
  conv[(uint64_t)t * kRegions + lane] = pt;
  if (dbg) dbg[(uint64_t)t * kRegions + lane] = pops;
}

// ---- Serializable stream-length tables for deferred tiles --------------------------------
__global__ __launch_bounds__(64) void k_jser_fill(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                  JserTabs J) {
  __shared__ uint32_t s_tile[kImageDwords];
  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  if (!J.defer[t]) return;
  const TileDesc td = tiles[t];
  const SpanDesc sd = spans[td.span];
  SpanReader sr{tiles, sd.first_tile, sd.first_tile + sd.n_tiles, t, sd.len};
  stage_tile(s_tile, td, sr, lane);
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
  if (!nm) return;
  for (uint32_t a = rs; a < re; ++a) {
    if (t_u8(s_tile, a) != CLG_TAG_SERIALIZABLE || t_be32(s_tile, a + 1) != kSerMagic) continue;
    const int64_t L = len_slow_span(&sr, td.span_off + (a - td.delta));  // walker: 1 + stream length
    if (idx < (uint32_t)kJserCap) {
      J.pos[(uint64_t)t * kJserCap + idx] = a;
      J.len[(uint64_t)t * kJserCap + idx] = L > 1 ? (uint32_t)(L - 1) : 0u;
    }
    ++idx;
  }
}

// ---- pass F2: segment counts -----------------------------------------------------------
__device__ __forceinline__ int next_known(const uint32_t* s_c, int from) {
  while (from < 2 * kRegions && s_c[from] == kConvUnknown) ++from;
  return from;
}

// Points of this tile (0..63) and of the span's next tile (64..127) in this tile's
// aligned coordinates; for the span's last tile the span end is point 64.  Both halves
// are then made monotonic by dropping points that lie beyond a later point (a dropped
// point only means a longer segment for the lane before it).  The next tile's half is
// filtered on its own, exactly as that tile filters it, so both tiles agree on where
// the chain crosses the boundary; this tile's half is filtered against everything after.
__device__ __forceinline__ void load_points(uint32_t* s_c, const uint32_t* conv, const TileDesc* tiles,
                                            const TileDesc& td, const SpanDesc& sd, uint32_t t, uint32_t lane,
                                            uint64_t end_a) {
  const uint32_t own0 = conv[(uint64_t)t * kRegions + lane];
  s_c[lane] = own0;
  const bool last = t + 1 == sd.first_tile + sd.n_tiles;
  uint32_t x = kConvUnknown;
  if (!last) {
    const uint32_t c = conv[(uint64_t)(t + 1) * kRegions + lane];
    if (c != kConvUnknown) {
      const uint64_t v = (uint64_t)(td.delta + td.len) + (uint64_t)(c - tiles[t + 1].delta);
      x = v > 0xFFFFFFF0ull ? kConvUnknown : (uint32_t)v;
    }
  } else if (lane == 0) {
    x = end_a > 0xFFFFFFF0ull ? kConvUnknown : (uint32_t)end_a;
  }
  // suffix minima over the known points (both halves in registers, wave-uniform loop)
  uint32_t own = s_c[lane];
  uint32_t lim = kConvUnknown;
  uint32_t keep_next = x;
  for (int l = kRegions - 1; l >= 0; --l) {  // next tile's half, filtered on its own
    const uint32_t c = __builtin_amdgcn_readlane(x, l);
    if (c == kConvUnknown) continue;
    if (c > lim) {
      if ((int)lane == l) keep_next = kConvUnknown;
    } else {
      lim = c;
    }
  }
  uint32_t keep_own = own;
  for (int l = kRegions - 1; l >= 0; --l) {  // this tile's half, filtered against everything after
    const uint32_t c = __builtin_amdgcn_readlane(own, l);
    if (c == kConvUnknown) continue;
    if (c > lim) {
      if ((int)lane == l) keep_own = kConvUnknown;
    } else {
      lim = c;
    }
  }
  s_c[lane] = keep_own;
  s_c[kRegions + lane] = keep_next;
  __syncthreads();
}

// Parse from point l until landing exactly on a later known point.
__device__ LaneSeg parse_segment(const FastCtx& c, const uint32_t* s_c, int l) {
  LaneSeg seg{kEndFail, 0, 0, 0, 0};
  const uint32_t c0 = s_c[l];
  if (c0 == kConvUnknown) return seg;
  uint32_t pos = c0, cnt = 0, w = 0;
  int m = next_known(s_c, l + 1);
  uint32_t target = m < 2 * kRegions ? s_c[m] : kConvUnknown;
  for (int it = 0; it < kMaxSegRecords; ++it) {
    while (target < pos) {  // jumped over a point: aim at the next one
      m = next_known(s_c, m + 1);
      target = m < 2 * kRegions ? s_c[m] : kConvUnknown;
    }
    if (m >= 2 * kRegions) return seg;
    if (target == pos) {
      seg.end = (uint8_t)m;
      seg.cnt = (uint16_t)cnt;
      seg.wcnt = (uint16_t)w;
      return seg;
    }
    if ((uint64_t)pos >= c.end_a) return seg;
    int tag;
    const int64_t L = flen(c, pos, &tag);
    if (L <= 0 || (uint64_t)pos + (uint64_t)L > 0xFFFFFFF0ull) return seg;
    ++cnt;
    w += is_wide(tag);
    pos += (uint32_t)L;
  }
  return seg;
}

__global__ __launch_bounds__(64) void k_fast_count(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                   const uint32_t* __restrict__ conv, JserTabs J,
                                                   LaneSeg* __restrict__ lanes, TileSum* __restrict__ sums) {
  __shared__ uint32_t s_tile[kFastImageDwords];
  __shared__ uint32_t s_c[2 * kRegions];
  __shared__ uint32_t s_jpos[kJserCap], s_jlen[kJserCap];
  __shared__ uint32_t s_jn;
  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const TileDesc td = tiles[t];
  const SpanDesc sd = spans[td.span];
  const uint32_t t1 = sd.first_tile + sd.n_tiles;
  const uint64_t end_a = sd.len - td.span_off + td.delta;
  load_jtab(s_jpos, s_jlen, &s_jn, J, t, lane);
  load_points(s_c, conv, tiles, td, sd, t, lane, end_a);
  const uint32_t img_end = stage_fast(s_tile, td, tiles, t1, t, sd.len, lane);
  const FastCtx c{s_tile, td.delta, td.delta + td.len, img_end, end_a, td.span_off, tiles, t, t1, s_jpos, s_jlen,
                  s_jn, J};

  const LaneSeg seg = parse_segment(c, s_c, (int)lane);
  lanes[(uint64_t)t * kRegions + lane] = seg;
  // chain of segments from the first known point (wave-uniform walk over registers)
  const uint32_t packed = (uint32_t)seg.end | ((uint32_t)seg.cnt << 8) | ((uint32_t)seg.wcnt << 20);
  const uint64_t known = __ballot(s_c[lane] != kConvUnknown);
  const int f = known ? __builtin_ctzll(known) : kRegions;
  uint64_t valid = 0;
  uint32_t cnt = 0, w = 0;
  int v = f;
  while (v < kRegions) {
    const uint32_t g = __builtin_amdgcn_readlane(packed, v);
    const uint32_t end = g & 0xFF;
    if (end == kEndFail) break;
    valid |= 1ull << v;
    cnt += (g >> 8) & 0xFFF;
    w += g >> 20;
    v = (int)end;
  }
  if (lane == 0) {
    TileSum sm{};
    sm.f = (uint8_t)f;
    sm.x = (v >= kRegions && v < 2 * kRegions) ? (uint8_t)(v - kRegions) : kEndFail;
    sm.cnt = cnt;
    sm.wcnt = w;
    sm.valid = valid;
    sums[t] = sm;
  }
}

// ---- pass F3: per-span resolution ------------------------------------------------------
__device__ bool chain_from(const LaneSeg* lanes, uint32_t t, int e, uint64_t* valid, uint32_t* cnt, uint32_t* wcnt,
                           int* exit_idx) {
  uint64_t vm = 0;
  uint32_t c = 0, w = 0;
  int v = e;
  while (v < kRegions) {
    const LaneSeg gs = lanes[(uint64_t)t * kRegions + v];
    if (gs.end == kEndFail) return false;
    vm |= 1ull << v;
    c += gs.cnt;
    w += gs.wcnt;
    v = gs.end;
  }
  if (v >= 2 * kRegions) return false;
  *valid = vm;
  *cnt = c;
  *wcnt = w;
  *exit_idx = v - kRegions;
  return true;
}

__global__ __launch_bounds__(256) void k_fast_resolve(const SpanDesc* __restrict__ spans, const LaneSeg* __restrict__ lanes,
                                                      const TileSum* __restrict__ sums, const uint32_t* __restrict__ jn,
                                                      FastRes* __restrict__ fres, SpanRes* __restrict__ sres,
                                                      uint32_t* __restrict__ span_flags) {
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
  // regular: every tile's entry point is its first known point (0 for the first tile)
  // and the previous tile's chain lands on it; the last tile lands on the span end.
  for (uint32_t i = threadIdx.x; i < sd.n_tiles; i += blockDim.x) {
    const uint32_t t = sd.first_tile + i;
    const TileSum sm = sums[t];
    bool bad = sm.x == kEndFail || sm.f >= kRegions;
    if (i == 0) bad |= sm.f != 0;
    else bad |= sums[t - 1].x != sm.f;
    if (i + 1 == sd.n_tiles) bad |= sm.x != 0;
    if (bad) atomicOr(&s_irregular, 1u);
    if (jn[t] > (uint32_t)kJserCap) atomicOr(&s_overflow, 1u);
  }
  __syncthreads();
  if (s_overflow) {
    if (threadIdx.x == 0) span_flags[s] = 1u;
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
  // irregular: serial walk with per-lane chains; give up to the DP pipeline on a break
  if (threadIdx.x == 0) {
    uint64_t rec = 0, wide = 0;
    int e = 0;
    bool fallback = false;
    for (uint32_t i = 0; i < sd.n_tiles; ++i) {
      const uint32_t t = sd.first_tile + i;
      uint64_t vm;
      uint32_t c, w;
      int x;
      if (!chain_from(lanes, t, e, &vm, &c, &w, &x)) {
        fallback = true;
        break;
      }
      fres[t] = FastRes{vm, rec, wide};
      rec += c;
      wide += w;
      e = x;
    }
    if (!fallback && sd.n_tiles && e != 0) fallback = true;
    SpanRes r{};
    r.n_rec = rec;
    r.n_wide = wide;
    r.status = CLG_OK;
    r.err_off = -1;
    sres[s] = r;
    span_flags[s] = fallback ? 1u : 0u;
  }
}

// ---- pass F4: emit ---------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_fast_emit(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                  const uint32_t* __restrict__ conv, JserTabs J,
                                                  const LaneSeg* __restrict__ lanes, const FastRes* __restrict__ fres,
                                                  const SpanRes* __restrict__ sres, const uint32_t* __restrict__ span_flags,
                                                  DecodeOut out) {
  __shared__ uint32_t s_tile[kFastImageDwords];
  __shared__ uint32_t s_c[2 * kRegions];
  __shared__ uint32_t s_jpos[kJserCap], s_jlen[kJserCap];
  __shared__ uint32_t s_jn;
  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const TileDesc td = tiles[t];
  if (span_flags[td.span]) return;  // decoded by the DP pipeline
  const FastRes fr = fres[t];
  if (fr.valid == 0) return;
  const SpanDesc sd = spans[td.span];
  const SpanRes sp = sres[td.span];
  const uint32_t t1 = sd.first_tile + sd.n_tiles;
  const uint64_t end_a = sd.len - td.span_off + td.delta;
  load_jtab(s_jpos, s_jlen, &s_jn, J, t, lane);
  load_points(s_c, conv, tiles, td, sd, t, lane, end_a);
  const uint32_t img_end = stage_fast(s_tile, td, tiles, t1, t, sd.len, lane);
  const FastCtx c{s_tile, td.delta, td.delta + td.len, img_end, end_a, td.span_off, tiles, t, t1, s_jpos, s_jlen,
                  s_jn, J};

  const bool mine = (fr.valid >> lane) & 1ull;
  const LaneSeg seg = lanes[(uint64_t)t * kRegions + lane];
  const uint32_t cn = mine ? seg.cnt : 0u, wn = mine ? seg.wcnt : 0u;
  uint32_t ic = cn, iw = wn;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t yc = __shfl_up(ic, off), yw = __shfl_up(iw, off);
    if ((int)lane >= off) {
      ic += yc;
      iw += yw;
    }
  }
  uint64_t rec = sp.rec_base + fr.rec_base + (ic - cn);
  uint64_t wide = sp.wide_base + fr.wide_base + (iw - wn);
  if (!mine) return;
  uint32_t a = s_c[lane];
  for (uint32_t k = 0; k < cn; ++k) {
    Rec r;
    if (!fdecode(c, a, r)) break;
    const uint32_t so = (uint32_t)(td.span_off + (a - td.delta));
    if (rec < out.cap) {
      out.off[rec] = so;
      out.tag[rec] = r.tag;
      out.v0[rec] = r.v0;
    }
    if (r.wide) {
      if (wide < out.wcap) {
        out.w_idx[wide] = (uint32_t)rec;
        out.w_rc[wide] = r.rc;
        out.w_v1[wide] = r.v1;
        out.w_var_off[wide] = r.var_off ? so + r.var_off : 0u;
        out.w_var_len[wide] = r.var_len;
        out.w_sub[wide] = r.sub;
      }
      ++wide;
    }
    ++rec;
    a += r.L;
  }
}

// ---------------------------------------------------------------------------------
// Launchers.
// ---------------------------------------------------------------------------------
static int ok(hipError_t e) { return e == hipSuccess ? CLG_OK : CLG_E_DEVICE; }

int launch_fast_conv(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, uint32_t* d_conv, JserTabs J,
                     uint32_t mode, uint32_t* d_dbg, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_fast_conv, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, d_conv, J, mode,
                     d_dbg);
  return ok(hipGetLastError());
}

int launch_jser_fill(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, JserTabs J, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_jser_fill, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, J);
  return ok(hipGetLastError());
}

int launch_fast_count(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, const uint32_t* d_conv,
                      JserTabs J, LaneSeg* d_lanes, TileSum* d_sums, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_fast_count, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, d_conv, J,
                     d_lanes, d_sums);
  return ok(hipGetLastError());
}

int launch_fast_resolve(const SpanDesc* d_spans, uint32_t n_spans, const LaneSeg* d_lanes, const TileSum* d_sums,
                        const uint32_t* d_jn, FastRes* d_fres, SpanRes* d_sres, uint32_t* d_span_flags, void* stream) {
  if (!n_spans) return CLG_OK;
  hipLaunchKernelGGL(k_fast_resolve, dim3(n_spans), dim3(256), 0, (hipStream_t)stream, d_spans, d_lanes, d_sums, d_jn,
                     d_fres, d_sres, d_span_flags);
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
