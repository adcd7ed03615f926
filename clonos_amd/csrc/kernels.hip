// kernels.hip -- gfx950 kernels of the causal-log engine.
//
//  * k_scatter           batched append: staged host bytes -> HBM segments
//  * k_gather            batched delta slice: segments -> packed per-consumer output
//  * k_dec_tables        decode pass 1: per-lane backward DP over 256-byte regions of a
//                        16 KiB tile -> per-region transfer tables -> tile aggregate
//  * k_dec_resolve       decode pass 2: per-span walk over tile aggregates -> tile entries
//  * k_dec_spanscan      decode pass 3: exclusive scan of per-span record counts
//  * k_dec_emit          decode pass 4: per-lane forward parse of each region -> SoA
//
// Record lengths follow SimpleDeterminantEncoder.decodeNext (reference:
// flink-runtime/.../causal/determinant/SimpleDeterminantEncoder.java:78-342).  The decode
// design (speculative per-byte length, transfer functions over entry offsets, converged
// region entries) is described in DESIGN.md section "Decode".
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/clonos_engine.h"
#include "dev_slow.h"
#include "jser_flat.h"

namespace clg {

// ==================================================================================
// Byte-range copies (gather pieces, scatter chunks): destination-aligned 16-byte chunks, the
// source realigned in registers with v_alignbyte (the shift is uniform per range).
// ==================================================================================
__device__ __forceinline__ uint32_t fsh(uint32_t hi, uint32_t lo, uint32_t s) {
  return s ? __builtin_amdgcn_alignbyte(hi, lo, s) : lo;
}
// 16 bytes starting m bytes into the 32-byte window lo:hi (m in 1..15, uniform).
__device__ __forceinline__ uint4 funnel16(const uint4 lo, const uint4 hi, uint32_t m) {
  const uint32_t s = m & 3;
  switch (m >> 2) {
    case 0: return make_uint4(fsh(lo.y, lo.x, s), fsh(lo.z, lo.y, s), fsh(lo.w, lo.z, s), fsh(hi.x, lo.w, s));
    case 1: return make_uint4(fsh(lo.z, lo.y, s), fsh(lo.w, lo.z, s), fsh(hi.x, lo.w, s), fsh(hi.y, hi.x, s));
    case 2: return make_uint4(fsh(lo.w, lo.z, s), fsh(hi.x, lo.w, s), fsh(hi.y, hi.x, s), fsh(hi.z, hi.y, s));
    default: return make_uint4(fsh(hi.x, lo.w, s), fsh(hi.y, hi.x, s), fsh(hi.z, hi.y, s), fsh(hi.w, hi.z, s));
  }
}

// [src, src + len) -> [dst, dst + len) by NT threads (tid 0..NT-1).  Each thread takes up to
// kCopyK destination chunks (NT apart) and issues all their source loads before any store.
// Chunks that straddle the range's ends are written byte by byte from the same registers (no
// dependent loads).  A source load is issued only for an aligned 16-byte word that holds a
// byte of the range, so it never leaves the pages the range lies on (a caller's buffer ending
// at an unmapped page is safe).
constexpr int kCopyK = 4;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <uint32_t NT>
__device__ __forceinline__ void copy_range(const uint8_t* src, uint8_t* dst, uint32_t len, uint32_t tid) {
  if (len == 0) return;
  const uintptr_t d0 = (uintptr_t)dst, d1 = d0 + len;
  const uintptr_t a0 = d0 & ~(uintptr_t)15;
  const uintptr_t sdelta = (uintptr_t)src - d0;  // src address = dst address + sdelta
  const uintptr_t s0 = (uintptr_t)src, s1 = s0 + len;
  const uint32_t m = (uint32_t)(sdelta & 15);
  const uint32_t nch = (uint32_t)((((d1 + 15) & ~(uintptr_t)15) - a0) >> 4);
  for (uint32_t j0 = 0; j0 < nch; j0 += kCopyK * NT) {
    uint4 lo[kCopyK], hi[kCopyK];
#pragma unroll
    for (int k = 0; k < kCopyK; ++k) {
      const uint32_t j = j0 + tid + NT * (uint32_t)k;
      lo[k] = hi[k] = make_uint4(0, 0, 0, 0);
      if (j < nch) {
        const uintptr_t sa = (a0 + 16u * (uintptr_t)j + sdelta) & ~(uintptr_t)15;
        if (sa + 16 > s0 && sa < s1) lo[k] = *reinterpret_cast<const uint4*>(sa);
        if (m && sa + 32 > s0 && sa + 16 < s1) hi[k] = *reinterpret_cast<const uint4*>(sa + 16);
      }
    }
#pragma unroll
    for (int k = 0; k < kCopyK; ++k) {
      const uint32_t j = j0 + tid + NT * (uint32_t)k;
      if (j < nch) {
        const uintptr_t c = a0 + 16u * (uintptr_t)j;
        const uint4 v = m ? funnel16(lo[k], hi[k], m) : lo[k];
        if (c >= d0 && c + 16 <= d1) {
          const u32x4 nv = {v.x, v.y, v.z, v.w};
          __builtin_nontemporal_store(nv, reinterpret_cast<u32x4*>(c));
        } else {  // range edge: the bytes inside [d0, d1)
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int x = 0; x < 16; ++x)
            if (c + x >= d0 && c + x < d1) *reinterpret_cast<uint8_t*>(c + x) = (uint8_t)(w[x >> 2] >> (8 * (x & 3)));
        }
      }
    }
  }
}

// ==================================================================================
// The write path's Serializable candidates (kernels.h SideCar): every "03 AC ED 00 05" of a
// chunk -- the tag of a Serializable record and the stream magic, SimpleDeterminantEncoder
// .java:316-341 -- with the record length where the stream's shape is one the decode measures
// inline and it ends inside the chunk; a prefix of the magic at the chunk's end is listed
// with an unknown length (the decode checks the magic against the bytes after it).
// ==================================================================================
constexpr uint64_t kMagic5 = 0x0500EDAC03ull;  // 03 AC ED 00 05, little-endian

// Bytes q .. q+7 of the chunk s[0, len) little-endian, zero at and past len (q < len).  Only
// aligned dwords holding a byte of the chunk are loaded, so no load leaves its pages.
__device__ __forceinline__ uint64_t chunk8(const uint8_t* s, uint32_t len, uint32_t q) {
  const uintptr_t b = (uintptr_t)s + q, a = b & ~(uintptr_t)3, e = (uintptr_t)s + len;
  uint32_t d[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) d[k] = a + 4u * k < e ? *reinterpret_cast<const uint32_t*>(a + 4u * k) : 0u;
  const uint32_t sh = (uint32_t)(b & 3) * 8u;
  const uint64_t lo = (uint64_t)d[0] | (uint64_t)d[1] << 32;
  uint64_t v = sh ? (lo >> sh) | ((uint64_t)d[2] << (64u - sh)) : lo;
  const uint32_t vb = len - q;
  if (vb < 8) v &= (1ull << (8u * vb)) - 1ull;
  return v;
}

// Record length of the full candidate at p (the decode's inline shapes: TC_STRING, flat
// objects), or kSideUnknown: another shape, or the stream runs past the chunk.
__device__ __forceinline__ uint32_t side_len(const uint8_t* s, uint32_t len, uint32_t p) {
  if (p + 8 > len) return kSideUnknown;
  auto rd4 = [s, len](uint32_t q) -> uint32_t { return q < len ? (uint32_t)chunk8(s, len, q) : 0u; };
  const uint32_t v = rd4(p + 5);
  uint32_t L = 0;
  if ((v & 0xFFu) == jser::TC_STRING) {  // [03][AC ED 00 05][74][len u16][modified UTF-8]
    L = 8u + jf_be16_12(v);
    if (p + L > len || !jf_mutf(rd4, p + 8u, L - 8u)) L = 0;  // (malformed: the decode's walker rejects it)
  } else if ((v & 0xFFu) == jser::TC_OBJECT) {
    L = jser_flat_len_t(rd4, p, len);
  }
  return L && L < kSideUnknown ? L : kSideUnknown;
}

// One wave records chunk ch's candidates in its segment's list.  One pass over the chunk's
// dwords (four dwords' loads in flight per lane; a dword and the next one hold every candidate
// starting in it) compacts the candidates' positions, in order, into the wave's LDS (`pos`,
// S.cap words); one reservation in the header (its life checked: a new life starts the list
// again); then a lane per candidate measures its stream and writes the entry.
// nx: the next chunk's descriptor when the request goes on into it (loaded by the caller
// before the copy), else len 0.
__device__ __forceinline__ void side_record(const ScatterChunk* __restrict__ chunks, uint32_t c, uint32_t n,
                                            const ScatterChunk& ch, const ScatterChunk& nx, const uint8_t* s,
                                            const SideCar& S, uint32_t lane, uint32_t* pos) {
  const uint64_t off = (uint64_t)(ch.dst - S.pool);
  const uint32_t seg = (uint32_t)(off / S.seg_bytes), so = (uint32_t)(off % S.seg_bytes), len = ch.len;
  const uint32_t life = ch.life & 0x7FFFFFFFu;
  // the request's bytes from this chunk through the next (contiguous in the source): enough to
  // see a magic the chunk's end cuts (the next chunk is a whole segment, at least 16 bytes, or
  // the request's last)
  uint32_t avail = len + nx.len;
  const uintptr_t A0 = (uintptr_t)s & ~(uintptr_t)3;
  const uint32_t lead = (uint32_t)((uintptr_t)s - A0);  // chunk bytes start at byte `lead` of dword 0
  const uint32_t nd = (lead + len + 3u) >> 2;    // dwords holding a byte of the chunk
  const uint32_t na = (lead + avail + 3u) >> 2;  // ... of the request's bytes from the chunk on
  constexpr int kU = 4;
  uint32_t total = 0;
  for (uint32_t d0 = 0; d0 < nd; d0 += 64u * kU) {
    uint32_t w[kU], x[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const uint32_t d = d0 + 64u * k + lane;
      const uint32_t* q = reinterpret_cast<const uint32_t*>(A0) + d;
      w[k] = d < nd ? q[0] : 0u;
      x[k] = d < nd && d + 1 < na ? q[1] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const uint32_t d = d0 + 64u * k + lane;
      // a magic starting in dword d has its ED byte in bytes 2-3 of d or 0-1 of d + 1; only a
      // prefix of it cut by the request's end ("03", "03 AC") has none: the exact test runs
      // only where one of those can be
      const uint32_t ed = ((w[k] >> 16) | (x[k] << 16)) ^ 0xEDEDEDEDu;
      const bool maybe = d < nd && (((ed - 0x01010101u) & ~ed & 0x80808080u) || 4u * d + 8u > lead + avail);
      if (!__ballot(maybe)) continue;
      const uint64_t v = (uint64_t)w[k] | (uint64_t)x[k] << 32;
      uint32_t c = 0;  // candidate's chunk position + 1 (at most one per dword: a second 03 within
                       // four bytes of a first would lie inside that one's magic)
#pragma unroll
      for (uint32_t sh = 0; sh < 4; ++sh) {
        const int64_t p = (int64_t)(4u * d + sh) - (int64_t)lead;
        if (!maybe || c || p < 0 || p >= (int64_t)len) continue;
        const uint32_t kb = avail - (uint32_t)p < 5u ? avail - (uint32_t)p : 5u;  // magic bytes written
        const uint64_t m = (1ull << (8u * kb)) - 1ull;
        if (((v >> (8u * sh)) & m) == (kMagic5 & m)) c = (uint32_t)p + 1u;
      }
      const uint64_t bm = __ballot(c != 0);
      if (c) {
        const uint32_t i = total + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
        if (i < S.cap) pos[i] = c - 1u;
      }
      total += (uint32_t)__popcll(bm);
    }
  }
  // A chunk that does not start its segment and holds no candidate has nothing to do: the
  // segment's first chunk of this life (at offset 0: segments fill from their start) stamps
  // the life; config 4's appends are mostly such chunks
  if (!total && so) return;
  uint32_t base = 0;
  if (lane == 0) {
    uint64_t* h = S.hdr + seg;
    uint64_t old = __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      const bool same = (uint32_t)(old >> 32) == life;
      if (same && !total) break;  // nothing to add, the life already stamped
      const uint64_t nw = same ? old + total : ((uint64_t)life << 32 | total);
      if (__hip_atomic_compare_exchange_strong(h, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        base = same ? (uint32_t)old : 0u;
        break;
      }
    }
  }
  if (!total) return;
  base = __shfl(base, 0);
  // for the lengths: the request's bytes up to 64 KiB past the chunk (at most four descriptors)
  {
    uint32_t more = nx.life >> 31, k = c + 2;
    while (more && k < n && k <= c + 4 && avail - len < 65536u) {
      const ScatterChunk nk = chunks[k++];
      avail += nk.len;
      more = nk.life >> 31;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the wave's LDS stores before its reads
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint32_t* ent = S.ent + (size_t)seg * S.cap;
  for (uint32_t i = lane; i < total && base + i < S.cap; i += 64u) {
    const uint32_t p = pos[i];
    ent[base + i] = (so + p) | (p + 5u <= avail ? side_len(s, avail, p) : kSideUnknown) << 16;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads done before the next chunk's stores
  __builtin_amdgcn_wave_barrier();
}

// ==================================================================================
// Append scatter: one wave per chunk (chunks are at most one segment; config 4's are
// mostly a few hundred bytes), 16-byte stores; causal-log chunks then record their
// Serializable candidates (S.hdr set).
// ==================================================================================
__global__ __launch_bounds__(256) void k_scatter(const ScatterChunk* __restrict__ chunks, uint32_t n,
                                                 const uint8_t* __restrict__ src, const SideCar S) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  extern __shared__ uint32_t s_pos[];  // per wave: its chunk's candidates, S.cap words (dynamic: 0 without S)
  for (uint32_t c = wave; c < n; c += nwaves) {
    const ScatterChunk ch = chunks[c];
    ScatterChunk nx{nullptr, 0, 0, 0};  // (loaded before the copy: its latency under the copy's)
    if (S.hdr && (ch.life >> 31) && c + 1 < n) nx = chunks[c + 1];
    copy_range<64>(src + ch.src, ch.dst, ch.len, lane);
    if (S.hdr) side_record(chunks, c, n, ch, nx, src + ch.src, S, lane, s_pos + (threadIdx.x >> 6) * S.cap);
  }
}

// ==================================================================================
// Gather (delta slice): one block per piece.
// ==================================================================================
__global__ __launch_bounds__(256) void k_gather(const GatherPiece* __restrict__ pieces, uint8_t* __restrict__ out) {
  // blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one; speed only, never
  // correctness): XCD x takes a contiguous range of pieces, so a request's consecutive
  // pieces (one source run, one destination run) stay in one L2
  const uint32_t nb = gridDim.x, b = blockIdx.x, q = nb >> 3, rm = nb & 7u, x = b & 7u;
  const GatherPiece p = pieces[x * q + (x < rm ? x : rm) + (b >> 3)];
  copy_range<256>(p.src, out + p.dst, p.len, threadIdx.x);
}

// ==================================================================================
// Device-side planning: item g -> its run (binary search over first) -> window.
// ==================================================================================
__device__ __forceinline__ uint32_t find_run(const SegSpan* spans, uint32_t n, uint32_t g) {
  uint32_t lo = 0, hi = n;  // last run with first <= g
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (spans[mid].first <= g) lo = mid; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_expand_pieces(const SegSpan* __restrict__ spans, uint32_t n_spans,
                                                       uint32_t n_pieces, const uint32_t* __restrict__ segtab,
                                                       const uint8_t* __restrict__ pool, uint32_t C,
                                                       GatherPiece* __restrict__ out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_pieces) return;
  const SegSpan r = spans[find_run(spans, n_spans, g)];
  const uint32_t w = r.phys / C + (g - r.first);
  const uint32_t s0 = w * C > r.phys ? w * C : r.phys;
  const uint32_t e1 = (w + 1) * C < r.phys + r.len ? (w + 1) * C : r.phys + r.len;
  out[g] = GatherPiece{pool + (size_t)segtab[r.segtab_off + w] * C + (s0 - w * C), r.dst + (s0 - r.phys), e1 - s0, 0};
}

__device__ __forceinline__ void expand_tile(const SegSpan* __restrict__ spans, uint32_t n_spans,
                                            const uint32_t* __restrict__ segtab, const uint8_t* __restrict__ pool,
                                            uint32_t C, uint32_t U, TileDesc* __restrict__ out, uint32_t g) {
  const SegSpan r = spans[find_run(spans, n_spans, g)];
  const uint32_t w = r.phys / U + (g - r.first);
  const uint32_t s0 = w * U > r.phys ? w * U : r.phys;
  const uint32_t e1 = (w + 1) * U < r.phys + r.len ? (w + 1) * U : r.phys + r.len;
  const uint32_t si = s0 / C, so = s0 % C;
  out[g] = TileDesc{pool + (size_t)segtab[r.segtab_off + si] * C + (so & ~15u), so & 15u, e1 - s0, (uint32_t)r.dst, 0,
                    (uint64_t)(s0 - r.phys)};
}
__global__ __launch_bounds__(256) void k_expand_tiles(const SegSpan* __restrict__ spans, uint32_t n_spans,
                                                      uint32_t n_tiles, const uint32_t* __restrict__ segtab,
                                                      const uint8_t* __restrict__ pool, uint32_t C, uint32_t U,
                                                      TileDesc* __restrict__ out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n_tiles) expand_tile(spans, n_spans, segtab, pool, C, U, out, g);
}

// The fast decode's set-up in one launch (it was a device copy, the tile expansion and four
// or five memsets, each a few microseconds of launch on the decode's critical path): item i
// < n_tiles expands tile i from the runs, the rest walk the word ranges in order (a copy
// where src is set, else a fill with val).
// A batch of few runs (config 2: 64 logs) searches them in LDS: from HBM the binary search
// was a chain of dependent loads, and beside the previous step's slice gather each took
// microseconds (the prep ran 30-95 us on the decode's critical path).
constexpr uint32_t kPrepLdsRuns = 256;
__global__ __launch_bounds__(256) void k_decode_prep(PrepArgs a) {
  __shared__ SegSpan s_runs[kPrepLdsRuns];
  const SegSpan* runs = a.runs;
  if (a.n_tiles && a.n_runs <= kPrepLdsRuns) {
    for (uint32_t i = threadIdx.x; i < a.n_runs; i += blockDim.x) s_runs[i] = a.runs[i];
    __syncthreads();
    runs = s_runs;
  }
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.total; i += stride) {
    uint64_t k = i;
    if (k < a.n_tiles) {
      expand_tile(runs, a.n_runs, a.segtab, a.pool, a.C, a.U, a.tiles, (uint32_t)k);
      continue;
    }
    k -= a.n_tiles;
#pragma unroll
    for (int r = 0; r < kPrepRanges; ++r) {
      if (k < a.r[r].n) {
        a.r[r].dst[k] = a.r[r].src ? a.r[r].src[k] : a.r[r].val;
        break;
      }
      k -= a.r[r].n;
    }
  }
}

// ==================================================================================
// Pass 1: transfer tables.  One wave per tile; lane l owns region l and runs a backward
// DP: ns(p) = (p + L(p) past the region end) ? that exit : ns(p + L(p)), with record
// and wide counts.  ns for the last 64 positions lives in an LDS ring; after the DP the
// ring holds the region's table for entries [0, 64).
// ==================================================================================
__global__ __launch_bounds__(64) void k_dec_tables(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                   uint64_t* __restrict__ agg, TileConv* __restrict__ conv,
                                                   const uint32_t* __restrict__ span_flags, JArena ar) {
  __shared__ uint32_t s_tile[kImageDwords];
  __shared__ uint32_t s_ring[kEntries * 64];  // [position mod 64][lane]
  __shared__ uint32_t s_conv_lane[kRegions];
  __shared__ uint32_t s_conv_cum[kRegions];
  __shared__ uint16_t s_conv_entry[kRegions];

  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const TileDesc td = tiles[t];
  if (span_flags && !span_flags[td.span]) return;
  const SpanDesc sd = spans[td.span];
  SpanReader sr{tiles, sd.first_tile, sd.first_tile + sd.n_tiles, t, sd.len, ar};
  stage_tile(s_tile, td, sr, lane);

  const TileGeom g{td.delta, td.delta + td.len};
  const uint64_t end_a = sd.len - td.span_off + td.delta;  // aligned coordinate of the span end

  // ---- backward DP over my region ----
  const uint32_t rs = g.rs(lane), re = g.re(lane);
  const uint32_t base = lane * kRegion;
  for (int j = kRegion - 4; j >= 0; j -= 4) {
    const uint32_t w4 = s_tile[lane * kPitch + (uint32_t)(j >> 2)];
#pragma unroll
    for (int k = 3; k >= 0; --k) {
      const uint32_t a = base + (uint32_t)(j + k);
      if (a < rs || a >= re) continue;
      const int tag = (int)((w4 >> (8 * k)) & 0xFFu);
      int64_t L = len_inline(s_tile, tag, a, end_a);
      if (L == kLenSlow) {
        L = len_slow_span(&sr, td.span_off + (a - td.delta));
        if (L <= 0) L = kLenErr;
      }
      uint32_t ns;
      if (L < 0) {
        ns = kNsErr;
      } else {
        const uint64_t t2 = (uint64_t)a + (uint64_t)L;
        const uint32_t inc = (1u << 16) | (is_wide(tag) << 24);
        if (t2 >= re) {
          const uint64_t rel = t2 - re;
          ns = (rel >= kNsFar ? kNsFar : (uint32_t)rel) | inc;
        } else if (L < kEntries) {
          const uint32_t x = s_ring[((uint32_t)t2 & 63u) * 64 + lane];
          const uint32_t xr = x & 0xFFFFu;
          ns = (xr >= kNsFar) ? xr : x + inc;
        } else {
          uint32_t ex, c, w;
          const int st = region_forward(s_tile, &sr, td.delta, td.span_off, end_a, (uint32_t)t2, re, &ex, &c, &w);
          if (st != CLG_OK) {
            ns = kNsErr;
          } else {
            const uint32_t rel = ex - re;
            ns = (rel >= kNsFar ? kNsFar : rel) | ((c + 1) << 16) | ((w + is_wide(tag)) << 24);
          }
        }
      }
      s_ring[(a & 63u) * 64 + lane] = ns;
    }
  }
  __syncthreads();

  // ---- candidate walk: lane i follows tile entry i through all regions ----
  uint32_t pos = td.delta + lane;  // aligned coordinate of the candidate's current record start
  uint32_t cnt = 0, wcnt = 0;
  uint32_t dead = 0;  // 0 live, 1 error, 2 far
  bool any_conv = false;
  for (int l = 0; l < kRegions; ++l) {
    const uint32_t rsl = g.rs(l), rel_ = g.re(l);
    if (rsl >= rel_) {
      if (lane == 0) s_conv_entry[l] = 0xFFFF;
      continue;
    }
    // convergence vote among live candidates
    const uint64_t live = __ballot(dead == 0);
    if (live) {
      const int first = __builtin_ctzll(live);
      const uint32_t p0 = __shfl(pos, first);
      const uint32_t c0 = __shfl(cnt | (wcnt << 16), first);
      const bool conv_here = __all(dead != 0 || pos == p0);
      if (lane == 0) {
        const bool ok = conv_here && p0 >= rsl && (p0 - rsl) < 0xFFFFu;
        s_conv_entry[l] = ok ? (uint16_t)(p0 - rsl) : (uint16_t)0xFFFF;
        s_conv_lane[l] = (uint32_t)first;
        s_conv_cum[l] = c0;
      }
      any_conv |= conv_here;
    } else if (lane == 0) {
      s_conv_entry[l] = 0xFFFF;
    }
    if (dead == 0 && pos < rel_) {
      const uint32_t e = pos - rsl;
      const uint32_t RLl = rel_ - rsl;
      if (e < (uint32_t)kEntries && e < RLl) {
        const uint32_t x = s_ring[(pos & 63u) * 64 + (uint32_t)l];
        const uint32_t xr = x & 0xFFFFu;
        if (xr == kNsErr) {
          dead = 1;
        } else if (xr == kNsFar) {
          dead = 2;
        } else {
          pos = rel_ + xr;
          cnt += (x >> 16) & 0xFF;
          wcnt += x >> 24;
        }
      } else {
        uint32_t ex, c, w;
        const int st = region_forward(s_tile, &sr, td.delta, td.span_off, end_a, pos, rel_, &ex, &c, &w);
        if (st != CLG_OK) {
          dead = 1;
        } else {
          pos = ex;
          cnt += c;
          wcnt += w;
        }
      }
    }
  }
  __syncthreads();

  const uint32_t tile_end = td.delta + td.len;
  uint64_t a64;
  if (dead == 1) {
    a64 = kExitErr;
  } else if (dead == 2) {
    a64 = kExitFar;
  } else {
    a64 = (uint64_t)(pos - tile_end) | ((uint64_t)cnt << 32) | ((uint64_t)wcnt << 48);
  }
  agg[(uint64_t)t * kEntries + lane] = a64;

  // ---- convergence info ----
  TileConv* cv = conv + t;
  const uint16_t ce = s_conv_entry[lane];
  cv->entry[lane] = ce;
  const uint32_t k_ref = (ce != 0xFFFF) ? s_conv_lane[lane] : 0u;
  const uint32_t tot = __shfl(cnt | (wcnt << 16), (int)k_ref);  // executed by every lane
  uint32_t suffix = 0;
  if (ce != 0xFFFF) {
    const uint32_t cum = s_conv_cum[lane];
    suffix = ((tot & 0xFFFF) - (cum & 0xFFFF)) | (((tot >> 16) - (cum >> 16)) << 16);
  }
  cv->suffix[lane] = suffix;
  const uint64_t live_end = __ballot(dead == 0);
  uint32_t ex = kExitErr;
  if (live_end) {
    const int first = __builtin_ctzll(live_end);
    const uint32_t p0 = __shfl(pos, first);
    const bool same = __all(dead != 0 || pos == p0);
    ex = same ? p0 - tile_end : kExitErr;
  }
  if (lane == 0) {
    cv->valid = any_conv ? 1u : 0u;
    cv->exit = ex;
  }
}

// ==================================================================================
// Pass 2: resolve tile entries per span.  One block per span; thread 0 walks the
// span's tiles over an LDS cache of their aggregates (loaded cooperatively), with the
// concrete walks made beforehand in parallel from guessed entries (k_dec_resolve).
// ==================================================================================
constexpr int kResolveChunk = 96;  // tiles cached in LDS per step (96*64*8 = 48 KiB)

// Concrete evaluation of one tile from entry `e` (tile-relative offset), serial, exact.
// Uses convergence info to short-cut once the path meets the shared path.
__device__ int tile_eval_concrete(const TileDesc* tiles, const SpanDesc& sd, uint32_t t, const TileConv& cv,
                                  uint32_t e, uint32_t* exit_rel, uint32_t* cnt, uint32_t* wcnt, int64_t* err_off,
                                  int* err_tag, uint32_t* limit, JArena ar) {
  const TileDesc td = tiles[t];
  SpanReader sr{tiles, sd.first_tile, sd.first_tile + sd.n_tiles, t, sd.len, ar};
  const uint32_t lo = td.delta, hi = td.delta + td.len;
  uint32_t a = lo + e;
  uint32_t c = 0, w = 0;
  int region = -1;
  while (a < hi) {
    const int l = (int)(a >> 8);
    if (l != region) {
      region = l;
      const uint32_t rsl = (uint32_t)l * kRegion < lo ? lo : (uint32_t)l * kRegion;
      const uint16_t ce = cv.entry[l];
      if (ce != 0xFFFF && rsl + ce == a && cv.exit != kExitErr) {
        // Joined the shared path: the rest of the tile is known.
        *exit_rel = cv.exit;
        *cnt = c + (cv.suffix[l] & 0xFFFF);
        *wcnt = w + (cv.suffix[l] >> 16);
        *limit = 0xFFFFFFFFu;
        return CLG_OK;
      }
    }
    const uint64_t so = td.span_off + (a - lo);
    AtSpan b{&sr, so};
    const int64_t L = rec_len_slow(b, sd.len - so);
    if (L < 0) {
      *err_off = (int64_t)so;
      *err_tag = (int8_t)sr.at(so);
      *cnt = c;
      *wcnt = w;
      *limit = a;
      return (int)L;
    }
    w += is_wide(sr.at(so));
    ++c;
    a += (uint32_t)L;
  }
  *exit_rel = a - hi;
  *cnt = c;
  *wcnt = w;
  *limit = 0xFFFFFFFFu;
  return CLG_OK;
}

// A tile's concrete evaluation from a guessed entry, made by its own thread before the
// serial walk reaches it.
struct PreEval {
  uint32_t entry;  // the guessed entry (0xFFFFFFFF: none made)
  uint32_t exit, c, w, lim;
  int32_t st, err_tag;
  int64_t err_off;
};

// One block per span.  The walk from tile to tile is serial (a tile's entry is its
// predecessor's exit), but a tile whose entry misses its table (a record from the previous
// tile reaching 64 B or more into it, or a dead table entry) needs a concrete walk over HBM,
// and those walks are what cost: one thread walking them one after another took config 3
// 77 ms.  So first every thread takes tiles of the chunk and, where the predecessor's
// candidates all left by one exit (TileConv.exit), walks its tile from that entry; then
// thread 0's serial walk takes the result wherever the actual entry is the guessed one, and
// walks concretely only where it is not.
__global__ __launch_bounds__(256) void k_dec_resolve(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                     const uint64_t* __restrict__ agg, const TileConv* __restrict__ conv,
                                                     TileRes* __restrict__ tres, SpanRes* __restrict__ sres,
                                                     const uint32_t* __restrict__ span_flags, JArena ar) {
  __shared__ uint64_t s_agg[kResolveChunk * kEntries];
  __shared__ uint32_t s_len[kResolveChunk];
  __shared__ PreEval s_pre[kResolveChunk];
  __shared__ uint64_t s_state[4];  // entry, rec, wide, done
  const uint32_t s = blockIdx.x;
  if (span_flags && !span_flags[s]) return;
  const SpanDesc sd = spans[s];
  if (threadIdx.x == 0) {
    s_state[0] = 0;
    s_state[1] = 0;
    s_state[2] = 0;
    s_state[3] = 0;
  }
  int status = CLG_OK;
  int64_t err_off = -1;
  int err_tag = 0;
  for (uint32_t base = 0; base < sd.n_tiles; base += kResolveChunk) {
    const uint32_t nt = min((uint32_t)kResolveChunk, sd.n_tiles - base);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nt * kEntries; i += blockDim.x)
      s_agg[i] = agg[(uint64_t)(sd.first_tile + base) * kEntries + i];
    for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) s_len[i] = tiles[sd.first_tile + base + i].len;
    __syncthreads();
    // the guessed entries' concrete walks, a thread per tile
    for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) {
      const uint32_t t = sd.first_tile + base + i;
      PreEval pe;
      pe.entry = 0xFFFFFFFFu;
      const uint32_t g = base + i == 0 ? 0u : conv[t - 1].exit;  // (the span's first tile: entry 0)
      if (g != kExitErr && g < s_len[i]) {
        const uint64_t x = g < (uint32_t)kEntries ? s_agg[i * kEntries + g] : (uint64_t)kExitFar;
        if ((uint32_t)x == kExitErr || (uint32_t)x == kExitFar) {
          pe.entry = g;
          pe.err_off = -1;
          pe.err_tag = 0;
          pe.st = tile_eval_concrete(tiles, sd, t, conv[t], g, &pe.exit, &pe.c, &pe.w, &pe.err_off, &pe.err_tag, &pe.lim, ar);
        }
      }
      s_pre[i] = pe;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t e = s_state[0], rec = s_state[1], wide = s_state[2];
      bool done = s_state[3] != 0;
      for (uint32_t i = 0; i < nt; ++i) {
        const uint32_t t = sd.first_tile + base + i;
        TileRes r;
        r.rec_base = rec;
        r.wide_base = wide;
        r.limit = 0xFFFFFFFFu;
        r.flags = 0;
        r.pad = 0;
        const uint32_t len = s_len[i];
        if (done) {
          r.entry = 0xFFFFFFFFu;
          tres[t] = r;
          continue;
        }
        r.entry = (uint32_t)min(e, (uint64_t)0xFFFFFFFFu);
        if (e >= len) {  // a record started earlier covers the whole tile
          e -= len;
          tres[t] = r;
          continue;
        }
        uint64_t x = (e < (uint64_t)kEntries) ? s_agg[i * kEntries + e] : (uint64_t)kExitFar;
        uint32_t xr = (uint32_t)x;
        uint32_t c, w;
        if (xr == kExitErr || xr == kExitFar) {
          uint32_t lim;
          int st;
          const PreEval& pe = s_pre[i];
          if (pe.entry == (uint32_t)e) {  // walked already, from this very entry
            xr = pe.exit;
            c = pe.c;
            w = pe.w;
            lim = pe.lim;
            st = pe.st;
            if (st != CLG_OK) {
              err_off = pe.err_off;
              err_tag = pe.err_tag;
            }
          } else {
            st = tile_eval_concrete(tiles, sd, t, conv[t], (uint32_t)e, &xr, &c, &w, &err_off, &err_tag, &lim, ar);
          }
          r.limit = lim;
          if (st != CLG_OK) {
            status = st;
            done = true;
            rec += c;
            wide += w;
            tres[t] = r;
            continue;
          }
        } else {
          c = (uint32_t)(x >> 32) & 0xFFFF;
          w = (uint32_t)(x >> 48);
          r.flags = kResTableLive;
        }
        rec += c;
        wide += w;
        e = xr;
        tres[t] = r;
      }
      s_state[0] = e;
      s_state[1] = rec;
      s_state[2] = wide;
      s_state[3] = done ? 1 : 0;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    SpanRes sr_;
    sr_.n_rec = s_state[1];
    sr_.n_wide = s_state[2];
    sr_.status = status;
    sr_.err_tag = err_tag;
    sr_.err_off = err_off;
    if (status == CLG_OK && s_state[0] != 0) {
      // The last record runs past the span end (cannot happen when tables flag
      // truncation, kept as a guard).
      sr_.status = CLG_E_TRUNCATED;
    }
    sr_.rec_base = 0;
    sr_.wide_base = 0;
    sres[s] = sr_;
  }
}

// ==================================================================================
// Pass 3: exclusive scan of span totals (single block).
// ==================================================================================
__global__ __launch_bounds__(1024) void k_dec_spanscan(SpanRes* __restrict__ sres, uint32_t n, uint64_t* __restrict__ totals) {
  __shared__ uint64_t s_r[1024], s_w[1024];
  __shared__ uint64_t carry_r, carry_w;
  if (threadIdx.x == 0) {
    carry_r = 0;
    carry_w = 0;
  }
  __syncthreads();
  for (uint32_t base = 0; base < n; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint64_t r = i < n ? sres[i].n_rec : 0, w = i < n ? sres[i].n_wide : 0;
    s_r[threadIdx.x] = r;
    s_w[threadIdx.x] = w;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
      const uint64_t ar = threadIdx.x >= off ? s_r[threadIdx.x - off] : 0;
      const uint64_t aw = threadIdx.x >= off ? s_w[threadIdx.x - off] : 0;
      __syncthreads();
      s_r[threadIdx.x] += ar;
      s_w[threadIdx.x] += aw;
      __syncthreads();
    }
    if (i < n) {
      sres[i].rec_base = carry_r + s_r[threadIdx.x] - r;
      sres[i].wide_base = carry_w + s_w[threadIdx.x] - w;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      carry_r += s_r[1023];
      carry_w += s_w[1023];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    totals[0] = carry_r;
    totals[1] = carry_w;
  }
}

// ==================================================================================
// Pass 4: emit.  One wave per tile; region entries from the convergence info (or a
// serial chain), then every lane parses its region forward twice (count, emit).
// ==================================================================================
// Decode one record at aligned coordinate a (a valid record start on the resolved path).
__device__ __forceinline__ int decode_at(const uint32_t* T, SpanReader* sr, uint32_t a, uint32_t lo, uint64_t tile_so,
                                         uint64_t end_a, Rec& r) {
  const int tag = t_u8(T, a);
  if (tag == CLG_TAG_SERIALIZABLE) {  // stream walk through the span reader
    const uint64_t so = tile_so + (a - lo);
    AtSpan b{sr, so};
    return decode_rec(b, sr->len - so, r);
  }
  const int64_t L = len_inline(T, tag, a, end_a);
  if (L <= 0) return CLG_E_STATE;
  r.tag = (uint8_t)tag;
  r.L = (uint32_t)L;
  r.wide = (uint8_t)is_wide(tag);
  r.v1 = 0;
  r.rc = 0;
  r.var_off = 0;
  r.var_len = 0;
  r.sub = 0;
  switch (tag) {
    case CLG_TAG_ORDER: r.v0 = (int8_t)t_u8(T, a + 1); break;
    case CLG_TAG_TIMESTAMP: r.v0 = (int64_t)t_be64(T, a + 1); break;
    case CLG_TAG_RNG:
    case CLG_TAG_BUFFER_BUILT: r.v0 = (int32_t)t_be32(T, a + 1); break;
    case CLG_TAG_IGNORE_CHECKPOINT:
      r.rc = (int32_t)t_be32(T, a + 1);
      r.v0 = (int64_t)t_be64(T, a + 5);
      break;
    case CLG_TAG_TIMER_TRIGGER:
      r.rc = (int32_t)t_be32(T, a + 1);
      r.v0 = (int64_t)t_be64(T, a + 5);
      r.sub = (uint8_t)t_u8(T, a + 13);
      if (r.sub == 6) {
        r.var_off = 18;
        r.var_len = (uint32_t)(L - 18);
      }
      break;
    default:  // SOURCE_CHECKPOINT
      r.rc = (int32_t)t_be32(T, a + 1);
      r.v0 = (int64_t)t_be64(T, a + 5);
      r.v1 = (int64_t)t_be64(T, a + 13);
      r.sub = (uint8_t)t_u8(T, a + 21);
      if (t_u8(T, a + 22) != 0) {
        r.sub |= 0x80;
        r.var_off = 27;
        r.var_len = (uint32_t)(L - 27);
      }
      break;
  }
  return CLG_OK;
}

__global__ __launch_bounds__(64) void k_dec_emit(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                 const TileConv* __restrict__ conv, const TileRes* __restrict__ tres,
                                                 const SpanRes* __restrict__ sres, const uint32_t* __restrict__ span_flags,
                                                 DecodeOut out, JArena ar) {
  __shared__ uint32_t s_tile[kImageDwords];
  __shared__ uint32_t s_entry[kRegions];
  __shared__ uint16_t s_ce[kRegions];
  const uint32_t t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const TileDesc td = tiles[t];
  if (span_flags && !span_flags[td.span]) return;
  const TileRes tr = tres[t];
  if (tr.entry >= td.len) return;  // no record starts in this tile (uniform)
  const SpanDesc sd = spans[td.span];
  const SpanRes sp = sres[td.span];
  SpanReader sr{tiles, sd.first_tile, sd.first_tile + sd.n_tiles, t, sd.len, ar};
  stage_tile(s_tile, td, sr, lane);

  const TileGeom g{td.delta, td.delta + td.len};
  const uint64_t end_a = sd.len - td.span_off + td.delta;
  s_ce[lane] = conv[t].entry[lane];
  __syncthreads();
  const uint32_t limit = tr.limit;  // emission stops at this aligned coordinate (error record)

  // ---- region entries (lane 0, serial until the path joins the shared path) ----
  // When the tile entry came from a live table path, that path is one of the candidates
  // whose convergence k_dec_tables recorded, so it reaches the converged position of
  // every later converged region: no serial parse is needed to get there.
  if (lane == 0) {
    const bool table_live = (tr.flags & kResTableLive) != 0;
    uint32_t cur = td.delta + tr.entry;
    bool joined = false;
    for (int l = 0; l < kRegions; ++l) {
      const uint32_t rsl = g.rs(l), rel_ = g.re(l);
      const uint16_t ce = s_ce[l];
      if (!joined && ce != 0xFFFF && (table_live || rsl + ce == cur)) joined = true;
      if (joined) {
        const uint32_t p = (ce != 0xFFFF) ? rsl + ce : 0xFFFFFFFFu;
        s_entry[l] = (rsl < rel_ && p < rel_ && p < limit) ? p : 0xFFFFFFFFu;
        continue;
      }
      if (rsl >= rel_ || cur >= rel_ || cur >= limit) {
        s_entry[l] = 0xFFFFFFFFu;
        continue;
      }
      s_entry[l] = cur;
      // Next region converged and our path is live: its entry is known, skip the parse.
      if (table_live && l + 1 < kRegions && s_ce[l + 1] != 0xFFFF) continue;
      uint32_t ex, c, w;
      const uint32_t stop = rel_ < limit ? rel_ : limit;
      const int st = region_forward(s_tile, &sr, td.delta, td.span_off, end_a, cur, stop, &ex, &c, &w);
      cur = (st == CLG_OK) ? ex : 0xFFFFFFFFu;
    }
  }
  __syncthreads();

  // ---- per-lane forward parse: count ----
  const uint32_t my_entry = s_entry[lane];
  const uint32_t my_re = g.re((int)lane);
  const uint32_t stop = my_re < limit ? my_re : limit;
  uint32_t c = 0, w = 0;
  if (my_entry != 0xFFFFFFFFu) {
    uint32_t a = my_entry;
    while (a < stop) {
      int tag;
      const int64_t L = rec_len_at(s_tile, &sr, a, td.delta, td.span_off, end_a, &tag);
      if (L <= 0) break;  // cannot happen before `limit` on a resolved path
      ++c;
      w += is_wide(tag);
      a += (uint32_t)L;
    }
  }
  // wave exclusive scan of (c, w)
  uint32_t ic = c, iw = w;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t yc = __shfl_up(ic, off), yw = __shfl_up(iw, off);
    if ((int)lane >= off) {
      ic += yc;
      iw += yw;
    }
  }
  uint64_t rec = sp.rec_base + tr.rec_base + (ic - c);
  uint64_t wide = sp.wide_base + tr.wide_base + (iw - w);

  // ---- emit ----
  if (my_entry != 0xFFFFFFFFu) {
    uint32_t a = my_entry;
    for (uint32_t k = 0; k < c; ++k) {
      Rec r;
      if (decode_at(s_tile, &sr, a, td.delta, td.span_off, end_a, r) != CLG_OK) break;
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
}

// ==================================================================================
// Launchers.
// ==================================================================================
namespace {
thread_local hipError_t g_launch_err = hipSuccess;
}
int launch_status(hipError_t e) {
  if (e == hipSuccess) return CLG_OK;
  g_launch_err = e;
  return CLG_E_DEVICE;
}
const char* take_launch_error() {
  const hipError_t e = g_launch_err;
  g_launch_err = hipSuccess;
  return e == hipSuccess ? nullptr : hipGetErrorString(e);
}

static int ok(hipError_t e) { return launch_status(e); }

int launch_scatter(const ScatterChunk* d_chunks, uint32_t n, const uint8_t* d_src, void* stream, const SideCar* side) {
  if (!n) return CLG_OK;
  const uint32_t blocks = min((n + 3) / 4, 4096u);
  SideCar S{};
  if (side && side->hdr) {
    if (!side->pool || !side->seg_bytes || side->seg_bytes > 65536u || !side->cap || side->cap > kSideCapMax)
      return CLG_E_INVALID_ARG;
    S = *side;
  }
  hipLaunchKernelGGL(k_scatter, dim3(blocks), dim3(256), S.hdr ? 4u * 4u * S.cap : 0u, (hipStream_t)stream, d_chunks, n,
                     d_src, S);
  return ok(hipGetLastError());
}

int launch_expand_pieces(const SegSpan* d_spans, uint32_t n_spans, uint32_t n_pieces, const uint32_t* d_segtab,
                         const uint8_t* pool, uint32_t seg_bytes, GatherPiece* d_out, void* stream) {
  if (!n_pieces) return CLG_OK;
  hipLaunchKernelGGL(k_expand_pieces, dim3((n_pieces + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_spans, n_spans,
                     n_pieces, d_segtab, pool, seg_bytes, d_out);
  return launch_status(hipGetLastError());
}

int launch_expand_tiles(const SegSpan* d_spans, uint32_t n_spans, uint32_t n_tiles, const uint32_t* d_segtab,
                        const uint8_t* pool, uint32_t seg_bytes, uint32_t unit, TileDesc* d_out, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_expand_tiles, dim3((n_tiles + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_spans, n_spans,
                     n_tiles, d_segtab, pool, seg_bytes, unit, d_out);
  return launch_status(hipGetLastError());
}

int launch_decode_prep(PrepArgs a, void* stream) {
  a.total = a.n_tiles;
  for (int r = 0; r < kPrepRanges; ++r) a.total += a.r[r].n;
  if (!a.total) return CLG_OK;
  const uint64_t want = (a.total + 255) / 256, blocks = want < 2048 ? want : 2048;
  hipLaunchKernelGGL(k_decode_prep, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, a);
  return launch_status(hipGetLastError());
}

int launch_gather(const GatherPiece* d_pieces, uint32_t n, uint8_t* d_out, void* stream) {
  if (!n) return CLG_OK;
  hipLaunchKernelGGL(k_gather, dim3(n), dim3(256), 0, (hipStream_t)stream, d_pieces, d_out);
  return ok(hipGetLastError());
}

int launch_decode_tables(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, uint64_t* d_agg,
                         TileConv* d_conv, const uint32_t* d_span_flags, JArena ar, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_dec_tables, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, d_agg, d_conv,
                     d_span_flags, ar);
  return ok(hipGetLastError());
}

// Kept decode errors (FusedCtl::span_err): one block per bad span.  Thread 0 reads the record
// at the recorded position by decodeNext's full rules (rec_len_slow over the span's tiles);
// an invalid record confirms the error (its status and tag out, the span's bad flag cleared,
// the counts of its tiles past the error zeroed -- the tile holding it counted the records
// before it already).  A valid record there, or a walker short of spill space, leaves the
// span bad: the robust pipeline decodes it as before.
__global__ __launch_bounds__(256) void k_err_classify(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                      const uint32_t* __restrict__ bad, FusedCtl ctl, int32_t* res,
                                                      JArena ar) {
  __shared__ int32_t s_st;
  const uint32_t i = blockIdx.x, s = bad[i];
  const SpanDesc sd = spans[s];
  const uint64_t E = ctl.span_err[s];
  if (threadIdx.x == 0) {
    int32_t st = 0, tag = 0;
    if (E < sd.len && sd.n_tiles) {
      SpanReader sr{tiles, sd.first_tile, sd.first_tile + sd.n_tiles, sd.first_tile, sd.len, ar};
      AtSpan b{&sr, E};
      const int64_t L = rec_len_slow(b, sd.len - E);
      if (L == CLG_E_CORRUPT_TAG || L == CLG_E_TRUNCATED || L == CLG_E_BAD_ENUM || L == CLG_E_NEG_LEN ||
          L == CLG_E_BAD_SERIAL) {
        st = (int32_t)L;
        tag = (int8_t)sr.at(E);
      }
    }
    res[2 * i] = st;
    res[2 * i + 1] = tag;
    s_st = st;
  }
  __syncthreads();
  if (s_st >= 0) return;
  for (uint32_t k = threadIdx.x; k < sd.n_tiles; k += 256)
    if (tiles[sd.first_tile + k].span_off > E) ctl.cnt[sd.first_tile + k] = 0;
  if (threadIdx.x == 0) ctl.span_bad[s] = 0;
}
int launch_err_classify(const TileDesc* d_tiles, const SpanDesc* d_spans, const uint32_t* d_bad, uint32_t n_bad,
                        FusedCtl ctl, int32_t* d_res, JArena ar, void* stream) {
  if (!n_bad) return CLG_OK;
  hipLaunchKernelGGL(k_err_classify, dim3(n_bad), dim3(256), 0, (hipStream_t)stream, d_tiles, d_spans, d_bad, ctl, d_res,
                     ar);
  return ok(hipGetLastError());
}

int launch_decode_resolve(const TileDesc* d_tiles, const SpanDesc* d_spans, uint32_t n_spans, const uint64_t* d_agg,
                          const TileConv* d_conv, TileRes* d_tres, SpanRes* d_sres, const uint32_t* d_span_flags,
                          JArena ar, void* stream) {
  if (!n_spans) return CLG_OK;
  hipLaunchKernelGGL(k_dec_resolve, dim3(n_spans), dim3(256), 0, (hipStream_t)stream, d_tiles, d_spans, d_agg, d_conv,
                     d_tres, d_sres, d_span_flags, ar);
  return ok(hipGetLastError());
}

int launch_decode_spanscan(SpanRes* d_sres, uint32_t n_spans, uint64_t* d_totals, void* stream) {
  hipLaunchKernelGGL(k_dec_spanscan, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_sres, n_spans, d_totals);
  return ok(hipGetLastError());
}

int launch_decode_emit(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, const TileConv* d_conv,
                       const TileRes* d_tres, const SpanRes* d_sres, const uint32_t* d_span_flags, DecodeOut out,
                       JArena ar, void* stream) {
  if (!n_tiles) return CLG_OK;
  hipLaunchKernelGGL(k_dec_emit, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, d_conv, d_tres,
                     d_sres, d_span_flags, out, ar);
  return ok(hipGetLastError());
}

}  // namespace clg
