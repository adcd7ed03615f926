// dev_common.h -- device helpers shared by the decode kernels (no Java serialization
// walker).  One out-of-line function: span_byte_at, the far byte read behind TileReader --
// a kernel that reads bytes past its tile's image makes that call.  It is static, so every
// translation unit has its own copy (no duplicate device symbols under -fgpu-rdc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/clonos_engine.h"
#include "kernels.h"

namespace clg {

// Global-address-space views of pointers that arrive inside structs: without them the
// compiler emits flat loads/stores, whose counters force a full wait before every LDS
// access and serialise staging and emission.
#define CLG_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ CLG_GLOBAL T* gp(T* p) {
  return (CLG_GLOBAL T*)(p);
}
template <class T>
__device__ __forceinline__ const CLG_GLOBAL T* gp(const T* p) {
  return (const CLG_GLOBAL T*)(p);
}

// ----------------------------------------------------------------------------------
// Packed region-table entry: exit offset past the region end (16 bits, 0xFFFF = error,
// 0xFFFE = far), record count (8 bits), wide-record count (8 bits).
// ----------------------------------------------------------------------------------
constexpr uint32_t kNsErr = 0xFFFFu;
constexpr uint32_t kNsFar = 0xFFFEu;
constexpr int kPitch = 65;  // dwords per region in the LDS tile image (64 + 1 pad)

__device__ __forceinline__ uint32_t lds_byte_addr(uint32_t a) {
  return ((a >> 8) * kPitch + ((a >> 2) & 63u)) * 4u + (a & 3u);
}

// Byte reader over a whole span (global memory, walks the span's tile list).
struct SpanReader {
  const TileDesc* tiles;
  uint32_t t0, t1, cur;
  uint64_t len;
  JArena ar;  // the stream walker's spill arena
  __device__ int at(uint64_t o) {
    if (o >= len) return -1;
    while (cur > t0 && o < tiles[cur].span_off) --cur;
    while (cur + 1 < t1 && o >= tiles[cur].span_off + tiles[cur].len) ++cur;
    const TileDesc& t = tiles[cur];
    return t.abase[t.delta + (o - t.span_off)];
  }
};

// A byte of the span through a fresh span reader, out of line: inlined at every byte the
// stream parsers read, the tile search made the table fill's code several times larger.  The
// search starts at the caller's tile hint `cur` (TileReader passes its reader's, which this
// call does not move: the search goes either way from it, so a stale hint costs steps only).
static __device__ __noinline__ int span_byte_at(const TileDesc* tiles, uint32_t t0, uint32_t t1, uint32_t cur, uint64_t len,
                                         uint64_t o) {
  SpanReader r{tiles, t0, t1, cur, len, JArena{}};
  return r.at(o);
}

// Byte reader for one tile: the LDS image for bytes inside the tile, the span reader
// beyond it.  Coordinates are the tile's aligned coordinates.
struct TileReader {
  const uint8_t* lds;
  uint32_t lo, hi;
  uint64_t so;  // span offset of aligned coordinate lo
  SpanReader* sr;
  __device__ __forceinline__ int at(uint32_t a) {
    if (a < hi) return lds[lds_byte_addr(a)];
    return span_byte_at(sr->tiles, sr->t0, sr->t1, sr->cur, sr->len, so + (a - lo));
  }
  __device__ __forceinline__ uint64_t span_off(uint32_t a) const { return so + (a - lo); }
};

// Bytes relative to a record start, for the length / value parsers.
template <class R>
struct At {
  R* r;
  uint32_t base;
  __device__ __forceinline__ int operator()(uint64_t k) { return r->at(base + (uint32_t)k); }
};
// A record through a tile reader (the LDS image inside the tile, HBM past it), with the
// span's spill arena: the stream walker reads a Serializable record from LDS.
struct AtTileSpan {
  TileReader* r;
  uint32_t base;
  __device__ __forceinline__ int operator()(uint64_t k) { return r->at(base + (uint32_t)k); }
  __device__ __forceinline__ JArena arena() const { return r->sr->ar; }
};
struct AtSpan {
  SpanReader* r;
  uint64_t base;
  __device__ __forceinline__ int operator()(uint64_t k) { return r->at(base + k); }
  __device__ __forceinline__ JArena arena() const { return r->ar; }
};

template <class F>
__device__ __forceinline__ uint32_t rd_be32(F& b, uint32_t k) {
  return (uint32_t)b(k) << 24 | (uint32_t)b(k + 1) << 16 | (uint32_t)b(k + 2) << 8 | (uint32_t)b(k + 3);
}
template <class F>
__device__ __forceinline__ uint64_t rd_be64(F& b, uint32_t k) {
  return (uint64_t)rd_be32(b, k) << 32 | rd_be32(b, k + 4);
}

// Fixed-length tags via a nibble LUT: 0->2, 1->9, 2->5, 6->13, 7->5; 0 = "slow" (3,4,5).
__device__ __forceinline__ int fast_len(int tag) {
  constexpr uint32_t lut = 2u | 9u << 4 | 5u << 8 | 0u << 12 | 0u << 16 | 0u << 20 | 13u << 24 | 5u << 28;
  return (tag >= 0 && tag < 8) ? (int)((lut >> (4 * tag)) & 0xF) : -1;
}
__device__ __forceinline__ uint32_t is_wide(int tag) { return (tag >= 3 && tag <= 6) ? 1u : 0u; }

// One decoded record (values + length), exact.
struct Rec {
  int64_t v0, v1;
  int32_t rc;
  uint32_t var_off, var_len;  // var_off relative to record start
  uint32_t L;
  uint8_t tag, sub, wide;
};

// ==================================================================================
// Decode, shared pieces.
//
// LDS tile image: 65 rows of 65 dwords.  Row r holds aligned coordinates
// [256 r, 256 r + 256) (one lane region) plus one pad dword, so that lanes reading
// their own regions at the same offset hit distinct banks.  Row 64 and the area past
// the tile's last valid byte hold a 32-byte halo copied from the span's next tile, so
// every fixed-layout field (at most 27 bytes into a record) is read from LDS.
// ==================================================================================
constexpr int kHalo = 32;
constexpr int kImageDwords = (kRegions + 1) * kPitch;
constexpr int64_t kLenErr = -1;   // any decode error (exact code from the slow path)
constexpr int64_t kLenSlow = 0;   // needs the slow path (Serializable stream walk)

struct TileGeom {
  uint32_t lo, hi;  // valid aligned coordinates
  __device__ __forceinline__ uint32_t rs(int l) const { uint32_t s = (uint32_t)l * kRegion; return s < lo ? lo : s; }
  __device__ __forceinline__ uint32_t re(int l) const { uint32_t e = (uint32_t)(l + 1) * kRegion; return e > hi ? hi : e; }
};

__device__ __forceinline__ uint32_t t_dw(const uint32_t* T, uint32_t k) { return T[(k >> 6) * kPitch + (k & 63u)]; }
__device__ __forceinline__ int t_u8(const uint32_t* T, uint32_t a) {
  return (int)((t_dw(T, a >> 2) >> (8 * (a & 3u))) & 0xFFu);
}
__device__ __forceinline__ uint32_t t_be32(const uint32_t* T, uint32_t a) {
  const uint32_t k = a >> 2, s = a & 3u;
  const uint32_t le = __builtin_amdgcn_alignbyte(t_dw(T, k + 1), t_dw(T, k), s);
  return __builtin_bswap32(le);
}
__device__ __forceinline__ uint64_t t_be64(const uint32_t* T, uint32_t a) {
  const uint32_t k = a >> 2, s = a & 3u;
  const uint32_t d0 = t_dw(T, k), d1 = t_dw(T, k + 1), d2 = t_dw(T, k + 2);
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, s), hi = __builtin_amdgcn_alignbyte(d2, d1, s);
  return __builtin_bswap64((uint64_t)hi << 32 | lo);
}

// Stage one tile (16-byte coalesced loads) plus its halo into the LDS image.
__device__ __forceinline__ void stage_tile(uint32_t* s_tile, const TileDesc& td, SpanReader& sr, uint32_t lane) {
  const uint32_t words = (td.delta + td.len + 15) >> 4;
  for (uint32_t w = lane; w < words; w += 64) {
    const uint4 v = *reinterpret_cast<const uint4*>(td.abase + 16 * w);
    const uint32_t d = (w >> 4) * kPitch + ((w & 15u) << 2);
    s_tile[d + 0] = v.x;
    s_tile[d + 1] = v.y;
    s_tile[d + 2] = v.z;
    s_tile[d + 3] = v.w;
  }
  __syncthreads();
  // halo: bytes [hi, hi + kHalo) of the span (zeros past the span end)
  if (lane < (uint32_t)kHalo) {
    const uint32_t a = td.delta + td.len + lane;
    const int b = sr.at(td.span_off + td.len + lane);
    reinterpret_cast<uint8_t*>(s_tile)[(a >> 8) * (kPitch * 4) + (a & 255u)] = (uint8_t)(b < 0 ? 0 : b);
  }
  __syncthreads();
}

// Record length at aligned coordinate a (a record start candidate, a < hi), using only
// the LDS image.  end_a = aligned coordinate of the span end.
__device__ __forceinline__ int64_t len_inline(const uint32_t* T, int tag, uint32_t a, uint64_t end_a) {
  constexpr uint32_t lut = 2u | 9u << 4 | 5u << 8 | 13u << 24 | 5u << 28;
  if ((uint32_t)tag > 7u) return kLenErr;
  int64_t L = (int64_t)((lut >> (4 * tag)) & 0xFu);
  if (L == 0) {
    if (tag == CLG_TAG_TIMER_TRIGGER) {
      const int ord = (int8_t)t_u8(T, a + 13);
      if (ord < 0 || ord > 6) return kLenErr;
      if (ord != 6) {
        L = 14;
      } else {
        const int32_t nl = (int32_t)t_be32(T, a + 14);
        if (nl < 0) return kLenErr;
        L = 18 + (int64_t)nl;
      }
    } else if (tag == CLG_TAG_SOURCE_CHECKPOINT) {
      const int ord = (int8_t)t_u8(T, a + 21);
      if (ord < 0 || ord > 1) return kLenErr;
      L = 23;
      if (t_u8(T, a + 22) != 0) {
        const int32_t rl = (int32_t)t_be32(T, a + 23);
        if (rl < 0) return kLenErr;
        L = 27 + (int64_t)rl;
      }
    } else {  // SERIALIZABLE: cheap magic check, the walk itself is out of line
      if (t_be32(T, a + 1) != 0xACED0005u) return kLenErr;
      return kLenSlow;
    }
  }
  return ((uint64_t)a + (uint64_t)L > end_a) ? kLenErr : L;
}

// LDS image bytes relative to a record start (for the accessor-generic helpers).
struct LdsBytes {
  const uint32_t* T;
  uint32_t base;
  __device__ __forceinline__ int operator()(uint64_t k) const { return t_u8(T, base + (uint32_t)k); }
};
template <class F>
__device__ __forceinline__ uint32_t fld_be32(const F& b, uint32_t k) {
  return (uint32_t)b(k) << 24 | (uint32_t)b(k + 1) << 16 | (uint32_t)b(k + 2) << 8 | (uint32_t)b(k + 3);
}
template <class F>
__device__ __forceinline__ uint64_t fld_be64(const F& b, uint32_t k) {
  return (uint64_t)fld_be32(b, k) << 32 | fld_be32(b, k + 4);
}
__device__ __forceinline__ uint32_t fld_be32(const LdsBytes& b, uint32_t k) { return t_be32(b.T, b.base + k); }
__device__ __forceinline__ uint64_t fld_be64(const LdsBytes& b, uint32_t k) { return t_be64(b.T, b.base + k); }

// ---------------------------------------------------------------------------------
// Dense LDS image accessors.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t d_u8(const uint32_t* T, uint32_t a) {
  return reinterpret_cast<const uint8_t*>(T)[a];
}
__device__ __forceinline__ uint32_t d_be32(const uint32_t* T, uint32_t a) {
  const uint32_t k = a >> 2;
  return __builtin_bswap32(__builtin_amdgcn_alignbyte(T[k + 1], T[k], a & 3u));
}
__device__ __forceinline__ uint64_t d_be64(const uint32_t* T, uint32_t a) {
  const uint32_t k = a >> 2, s = a & 3u;
  const uint32_t d0 = T[k], d1 = T[k + 1], d2 = T[k + 2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, s), hi = __builtin_amdgcn_alignbyte(d2, d1, s);
  return __builtin_bswap64((uint64_t)hi << 32 | lo);
}
struct DenseBytes {
  const uint32_t* T;
  uint32_t base;
  __device__ __forceinline__ int operator()(uint64_t k) const { return (int)d_u8(T, base + (uint32_t)k); }
};
__device__ __forceinline__ uint32_t fld_be32(const DenseBytes& b, uint32_t k) { return d_be32(b.T, b.base + k); }
__device__ __forceinline__ uint64_t fld_be64(const DenseBytes& b, uint32_t k) { return d_be64(b.T, b.base + k); }

// Exact length of a non-Serializable record through a byte accessor (inline, no calls):
// L > 0, kLenErr on any decode error (truncation, bad enum, negative length, bad tag),
// kLenSlow for a Serializable record (its length needs the stream walker).
template <class F>
__device__ __forceinline__ int64_t len_fields(const F& b, int tag, uint64_t avail) {
  constexpr uint32_t lut = 2u | 9u << 4 | 5u << 8 | 13u << 24 | 5u << 28;
  if ((uint32_t)tag > 7u) return kLenErr;
  int64_t L = (int64_t)((lut >> (4 * tag)) & 0xFu);
  if (L == 0) {
    if (tag == CLG_TAG_TIMER_TRIGGER) {
      if (avail < 14) return kLenErr;
      const int ord = (int8_t)b(13);
      if (ord < 0 || ord > 6) return kLenErr;
      if (ord != 6) {
        L = 14;
      } else {
        if (avail < 18) return kLenErr;
        const int32_t nl = (int32_t)fld_be32(b, 14);
        if (nl < 0) return kLenErr;
        L = 18 + (int64_t)nl;
      }
    } else if (tag == CLG_TAG_SOURCE_CHECKPOINT) {
      if (avail < 23) return kLenErr;
      L = 23;
      if (b(22) != 0) {
        if (avail < 27) return kLenErr;
        const int32_t rl = (int32_t)fld_be32(b, 23);
        if (rl < 0) return kLenErr;
        L = 27 + (int64_t)rl;
      }
      const int ord = (int8_t)b(21);
      if (ord < 0 || ord > 1) return kLenErr;
    } else {
      return kLenSlow;
    }
  }
  return (uint64_t)L > avail ? kLenErr : L;
}

// Values of a record whose tag and exact length are known (SimpleDeterminantEncoder
// readers :116-341; Serializable: the stream's position and length).
template <class F>
__device__ __forceinline__ void decode_fields(const F& b, int tag, int64_t L, Rec& r) {
  r.v1 = 0;
  r.rc = 0;
  r.var_off = 0;
  r.var_len = 0;
  r.sub = 0;
  switch (tag) {
    case CLG_TAG_ORDER: r.v0 = (int8_t)b(1); break;
    case CLG_TAG_TIMESTAMP: r.v0 = (int64_t)fld_be64(b, 1); break;
    case CLG_TAG_RNG:
    case CLG_TAG_BUFFER_BUILT: r.v0 = (int32_t)fld_be32(b, 1); break;
    case CLG_TAG_IGNORE_CHECKPOINT:
      r.rc = (int32_t)fld_be32(b, 1);
      r.v0 = (int64_t)fld_be64(b, 5);
      break;
    case CLG_TAG_TIMER_TRIGGER:
      r.rc = (int32_t)fld_be32(b, 1);
      r.v0 = (int64_t)fld_be64(b, 5);
      r.sub = (uint8_t)b(13);
      if (r.sub == 6) {
        r.var_off = 18;
        r.var_len = (uint32_t)(L - 18);
      }
      break;
    case CLG_TAG_SOURCE_CHECKPOINT:
      r.rc = (int32_t)fld_be32(b, 1);
      r.v0 = (int64_t)fld_be64(b, 5);
      r.v1 = (int64_t)fld_be64(b, 13);
      r.sub = (uint8_t)b(21);
      if (b(22) != 0) {
        r.sub |= 0x80;
        r.var_off = 27;
        r.var_len = (uint32_t)(L - 27);
      }
      break;
    default:  // SERIALIZABLE
      r.v0 = L - 1;
      r.var_off = 1;
      r.var_len = (uint32_t)(L - 1);
      break;
  }
}

}  // namespace clg
