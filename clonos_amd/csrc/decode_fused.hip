// decode_fused.hip -- single-pass batched decode (gfx950).
//
// SimpleDeterminantEncoder.decodeNext (reference flink-runtime
// causal/determinant/SimpleDeterminantEncoder.java:78-342) applied to whole spans.  Record
// starts form a chain p -> p + L(p) whose length function reads the tag byte (and, for
// TimerTrigger / SourceCheckpoint, a field at a fixed offset), so the stream is not
// self-synchronising.  One wave decodes one tile of kZTile bytes; lane l owns the kZRegion
// bytes of region l:
//
//   1. speculative walk: from the region's first byte, follow the chain, stepping one
//      byte past anything that is not a valid record (a 128-bit bitmap of the starts it
//      visits stays in registers);
//   2. merge: given the true entry e of the region, walk the true chain from e and the
//      speculative chain from the region start in lock-step (two pointers) until they
//      meet.  From the meeting point on the region's true starts ARE the speculative ones,
//      so the region's exit is the speculative exit and its starts are the true prefix
//      plus the speculative suffix.  Chains re-synchronise after a few records, so this
//      costs a few steps per region;
//   3. entries are the previous lane's exit; a lane whose entry changed re-merges
//      (wave-uniform loop, at most one pass per lane);
//   4. across tiles: every tile first computes its exit assuming the chain merges inside
//      it ("canonical" exit, independent of its entry) and publishes it, then reads its
//      predecessor's canonical exit as its entry, re-merges lane 0 and checks that its
//      true exit is the one it published.  Record and wide-record bases come from the
//      scan pass over the per-tile counts;
//   5. emit: record starts are dropped into LDS by output index and decoded by
//      consecutive lanes, so every SoA store of the wave is one contiguous run.
//
// Anything outside the fast path -- a decode error, a Serializable record (its length
// needs the Java-serialization walker), a record that jumps a whole tile, a tile whose
// true exit differs from the one it published -- raises the batch's abort flag; the
// host then re-decodes the batch with the robust pipeline (decode_fast.hip +
// kernels.hip), which also classifies errors exactly.  Abort never produces output the
// host keeps.
//
// Cross-workgroup hand-offs are single 8-byte words written and polled with agent-scope
// relaxed atomics (global_store/load ... sc1): the payload is the word itself.
// Record layouts: SimpleDeterminantEncoder.java:124-323.
#include "dev_common.h"
#include "jser_device.h"
#include "jser_flat.h"
#include "handoff.h"

namespace clg {

// LDS image: row r holds aligned bytes [kZRegion r, kZRegion (r + 1)), unpadded: the image
// is the bytes themselves (an address is the aligned coordinate).  Rows of 35 dwords with pad
// dwords repeating the next row's head spread the lanes' row walks over the banks, but cost
// two VALU per walk step; without them config-2 count took 0.179 -> 0.164 ms and config-3 emit
// 0.363 -> 0.335 ms (round 4), and round 5 measured it again (0.150 against 0.170 ms).  The
// warm-ups are staggered instead (warm_start), and build_lm reads column-wise.  Rows: the tile,
// then the halo + zero pad.
constexpr uint32_t kZRowDw = kZRegion / 4;  // 32
constexpr uint32_t kZPitch = kZRowDw;
constexpr uint32_t kZRows = kZTile / kZRegion + 2;
constexpr uint32_t kZImgDw = kZRows * kZPitch;
constexpr uint32_t kZWin = 1024;                       // emit: record starts staged per window (16-bit entries)
constexpr uint32_t kZEmitWin = 512;                    // emit: 32-bit entries, the same 2 KiB of LDS
constexpr int kZEmitPair = 1;  // emit: records per lane per pass (2, the loads hoisted: the same, round 4)
constexpr uint32_t kZCanon = 0xFFFFFFFFu;              // entry marker: not on the canonical chain
constexpr uint32_t kZCanonLanes = 16;                  // regions (2 KiB) the canonical chain spans
constexpr int kZSer = -2;                              // Serializable stream: walker needed
constexpr uint32_t kZTiny = kZTinySpan;                // small whole spans: a lane each (pass 0)

// ---------------------------------------------------------------------------------
// Wave-wide sums, scans and lane shifts through DPP (cross-lane moves inside the VALU): a
// __shfl is a ds_bpermute, an LDS round trip each, and the count pass's per-tile reductions
// were six of them in a row (the DPP forms: -2 % on count and emit, round 4).
// ---------------------------------------------------------------------------------
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtrl, 0xF, 0xF, false);
}
// inclusive scan over the 64 lanes (row_shr 1/2/4/8, then row_bcast 15 / 31)
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t v, uint32_t lane) {
  const uint32_t rl = lane & 15u;
  uint32_t t;
  t = dpp_mov<0x111>(v);
  if (rl >= 1u) v += t;
  t = dpp_mov<0x112>(v);
  if (rl >= 2u) v += t;
  t = dpp_mov<0x114>(v);
  if (rl >= 4u) v += t;
  t = dpp_mov<0x118>(v);
  if (rl >= 8u) v += t;
  t = dpp_mov<0x142>(v);
  if ((lane & 31u) >= 16u) v += t;
  t = dpp_mov<0x143>(v);
  if (lane >= 32u) v += t;
  return v;
}
// the sum over the 64 lanes, in every lane
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x124>(v);  // row_ror:4
  v += dpp_mov<0x128>(v);  // row_ror:8
  v += dpp_mov<0x142>(v);  // row_bcast:15
  v += dpp_mov<0x143>(v);  // row_bcast:31 (lane 63 holds the total)
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// lane l gets lane l - 1's value (lane 0: its own)
__device__ __forceinline__ uint32_t wave_prev_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ __forceinline__ uint32_t lane63(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

// ---------------------------------------------------------------------------------
// 128-bit region bitmaps (bit i <-> byte r0 + i of the lane's aligned region r0).
// ---------------------------------------------------------------------------------
struct Bits {
  uint64_t lo, hi;
};
__device__ __forceinline__ void bset(Bits& b, uint32_t i) {
  const uint64_t m = 1ull << (i & 63u);
  b.lo |= i < 64u ? m : 0ull;
  b.hi |= i < 64u ? 0ull : m;
}
// bits >= i
__device__ __forceinline__ Bits bge(const Bits& b, uint32_t i) {
  const uint64_t m = ~0ull << (i & 63u);
  return Bits{i < 64u ? b.lo & m : 0ull, i < 64u ? b.hi : b.hi & m};
}
__device__ __forceinline__ Bits bor(const Bits& a, const Bits& b) { return Bits{a.lo | b.lo, a.hi | b.hi}; }
__device__ __forceinline__ uint32_t bcount(const Bits& b) { return (uint32_t)(__popcll(b.lo) + __popcll(b.hi)); }

__device__ __forceinline__ uint32_t rk(uint32_t k) { return k; }  // dword k -> LDS dword
__device__ __forceinline__ uint32_t rb(uint32_t a) { return 4u * rk(a >> 2) + (a & 3u); }  // byte a -> LDS byte
__device__ __forceinline__ uint32_t zb(const uint32_t* T, uint32_t a) { return (T[rk(a >> 2)] >> (8u * (a & 3u))) & 0xFFu; }
__device__ __forceinline__ uint32_t zbe32(const uint32_t* T, uint32_t a) {
  const uint32_t p = rk(a >> 2);
  return __builtin_bswap32(__builtin_amdgcn_alignbyte(T[p + 1], T[p], a & 3u));
}
__device__ __forceinline__ uint64_t zbe64(const uint32_t* T, uint32_t a) {
  const uint32_t p = rk(a >> 2), sh = a & 3u;
  const uint32_t d0 = T[p], d1 = T[p + 1], d2 = T[p + 2];
  return __builtin_bswap64((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32 | __builtin_amdgcn_alignbyte(d1, d0, sh));
}
// Bytes relative to a record start, for len_fields / decode_fields (dev_common.h).
struct ZBytes {
  const uint32_t* T;
  uint32_t base;
  __device__ __forceinline__ int operator()(uint64_t k) const { return (int)zb(T, base + (uint32_t)k); }
};
__device__ __forceinline__ uint32_t fld_be32(const ZBytes& b, uint32_t k) { return zbe32(b.T, b.base + k); }
__device__ __forceinline__ uint64_t fld_be64(const ZBytes& b, uint32_t k) { return zbe64(b.T, b.base + k); }

// LDS byte offset of aligned coordinate a (the unpadded image: a itself).
__device__ __forceinline__ uint32_t zoff(uint32_t a) { return a; }
typedef const __attribute__((address_space(3))) uint8_t lds_u8;
typedef const __attribute__((address_space(3))) uint32_t lds_u32;
// Byte a of the LDS image: one ds_read_u8.
__device__ __forceinline__ uint32_t zb8(const uint32_t* T, uint32_t a) { return ((lds_u8*)(T))[zoff(a)]; }

// ---------------------------------------------------------------------------------
// Record length at aligned coordinate a (< tile end): L > 0, kLenErr (-1) for a record
// decodeNext rejects, kZSer for a Serializable record.  Reads only the LDS image (every
// field a valid record needs lies within 27 bytes of its start, inside tile + halo).
// Validity and length follow the SimpleDeterminantEncoder readers (:116-341; the same
// rules as len_fields in dev_common.h), all inline: the common tags cost one dword pair
// and a nibble table.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ int zlen_var(const uint32_t* T, uint32_t a, uint32_t end_a, uint32_t tg, uint32_t x0) {
  if (tg == CLG_TAG_SERIALIZABLE)
    return ((x0 >> 8) | (zb(T, a + 4) << 24)) == 0x0500EDACu ? kZSer : (int)kLenErr;  // AC ED 00 05
  // TimerTrigger / SourceCheckpoint, branch-free: the fields both need lie in bytes
  // a+13 .. a+26, read as five independent LDS dwords (one round trip) and selected by tag.
  //   TIMER_TRIGGER     [04][rc i32][ts i64][type u8]{[len i32][name]}        (:202-242)
  //   SOURCE_CHECKPOINT [05][rc][cp i64][ts i64][type u8][hasRef u8]{[len][ref]} (:244-287)
  const uint32_t avail = end_a - a;
  const uint32_t b0 = a + 13, k0 = b0 >> 2, sh = b0 & 3u;
  const uint32_t d0 = T[rk(k0)], d1 = T[rk(k0 + 1)], d2 = T[rk(k0 + 2)], d3 = T[rk(k0 + 3)], d4 = T[rk(k0 + 4)];
  const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);  // bytes a+13 .. a+16 (LE)
  const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);  // a+17 .. a+20
  const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);  // a+21 .. a+24
  const uint32_t w3 = __builtin_amdgcn_alignbyte(d4, d3, sh);  // a+25 .. a+28
  const int tt_ord = (int8_t)(w0 & 0xFFu);                                      // ProcessingTimeCallbackID.Type
  const int32_t tt_nl = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, 1));  // a+14 .. a+17
  const int sc_ord = (int8_t)(w2 & 0xFFu);                                      // CheckpointType (:27, :30)
  const bool sc_ref = ((w2 >> 8) & 0xFFu) != 0u;
  const int32_t sc_rl = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(w3, w2, 2));  // a+23 .. a+26
  uint64_t L;
  bool ok;
  if (tg == CLG_TAG_TIMER_TRIGGER) {
    ok = avail >= 14u && tt_ord >= 0 && tt_ord <= 6 && (tt_ord != 6 || (avail >= 18u && tt_nl >= 0));
    L = tt_ord == 6 ? 18ull + (uint64_t)(uint32_t)tt_nl : 14ull;
  } else {
    ok = avail >= 23u && sc_ord >= 0 && sc_ord <= 1 && (!sc_ref || (avail >= 27u && sc_rl >= 0));
    L = sc_ref ? 27ull + (uint64_t)(uint32_t)sc_rl : 23ull;
  }
  if (!ok) return (int)kLenErr;
  return (L > avail || L > 0x7FFFFFF0ull) ? (int)kLenErr : (int)L;
}
__device__ __forceinline__ int zlen(const uint32_t* T, uint32_t a, uint32_t end_a, uint32_t* tag) {
  lds_u32* d = (lds_u32*)((lds_u8*)(T) + (zoff(a) & ~3u));  // LDS dword rk(a >> 2)
  const uint32_t x0 = __builtin_amdgcn_alignbit(d[1], d[0], a << 3);  // bytes a..a+3 (LE); shift uses bits 0-4
  const uint32_t tg = x0 & 0xFFu;
  *tag = tg;
  constexpr uint32_t lut = 2u | 9u << 4 | 5u << 8 | 13u << 24 | 5u << 28;  // nibble per tag 0..7; 0: 3, 4, 5
  const uint32_t L = (lut >> ((tg & 7u) << 2)) & 0xFu;
  if (tg > 7u) return (int)kLenErr;
  if (L == 0) return zlen_var(T, a, end_a, tg, x0);  // TimerTrigger, SourceCheckpoint, Serializable
  return a + L > end_a ? (int)kLenErr : (int)L;
}

// ---------------------------------------------------------------------------------
// Walks.  Two step rules over the same length function:
//   true step  -- follow the record (any length); an invalid record is an error;
//   spec step  -- follow records of at most kZSpecMax bytes, step one byte past anything
//                 else.  Speculative chains start at arbitrary bytes, and a garbage
//                 TimerTrigger / SourceCheckpoint can claim a length of megabytes; the cap
//                 keeps such a chain local.  A skip is recorded (SpecR::bad) because from
//                 a skipped byte on the speculative chain no longer follows the true one.
// ---------------------------------------------------------------------------------
constexpr int kZSpecMax = 256;

// Serializable record lengths of the tile (phase 3 tables), staged in LDS: a candidate
// bitmap over aligned coordinates, the number of candidates before each bitmap dword, and
// the record length per candidate (0: the stream is invalid).
constexpr uint32_t kZJBitsDw = (kZTile + 16 + 31) / 32 + 3;  // 260
struct JL {
  const uint32_t* bits;
  const uint32_t* rank;
  const uint32_t* len;
  const uint32_t* lm = nullptr;  // count pass: the tile's step-code map (below), else null
  // count pass (load_jl_map): no bitmap or ranks, the entries' positions (sorted) instead
  const uint32_t* pos = nullptr;
  uint32_t n = 0;
  // a tile with more than kZJCap entries: the rest stay in HBM (the overflow arena), sorted
  // after the first kZJCap: on of them at opos / olen
  const uint32_t* opos = nullptr;
  const uint32_t* olen = nullptr;
  uint32_t on = 0;
};
// (The LDS table and the overflow entries are read by separate loads under a branch: a
// select between the two pointers compiles to a flat load.)
template <class P_>
__device__ __forceinline__ uint32_t jl_search(P_ P, uint32_t n, uint32_t a) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P[mid] < a) lo = mid + 1; else hi = mid;
  }
  return lo;
}
// Bitmap + ranks (load_jl).  j.on is wave-uniform (a scalar branch): a tile without overflow
// entries skips the HBM read, which -- predicated per lane, or waited for where the caller
// next wrote the register -- made every tile wait for its output stores at each wide record
// (config-3 emit 0.336 -> 0.386 ms).
__device__ __forceinline__ uint32_t jl_len_bits(const JL& j, uint32_t a) {
  const uint32_t w = j.bits[a >> 5], b = a & 31u;
  if (!((w >> b) & 1u)) return 0u;
  const uint32_t r = j.rank[a >> 5] + (uint32_t)__popc(w & ((1u << b) - 1u));
  if (j.on && r >= kZJCap) {
    const uint32_t L = gp(j.olen)[r - kZJCap];
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), inside the branch
    return L;
  }
  return ((const __attribute__((address_space(3))) uint32_t*)j.len)[r];
}
__device__ __forceinline__ uint32_t jl_len(const JL& j, uint32_t a) {
  if (!j.bits) {  // sorted positions: binary search (the count pass's rare slow path)
    const uint32_t k = jl_search(j.pos, j.n, a);
    return k < j.n && j.pos[k] == a ? j.len[k] : 0u;
  }
  return jl_len_bits(j, a);
}

struct Res {
  Bits bm, wb;     // true record starts in the region / wide ones (bad: those before the failing record)
  uint32_t exit;   // first true start >= re (bad: the speculative exit)
  uint32_t bad;    // true chain hits an invalid record (1) or, without tables, a Serializable one (2)
  uint32_t steps;  // true steps taken (diagnostics)
  uint32_t fail;   // bad: the failing record's start (aligned coordinate)
};

// True step lengths of the fixed-length tags (nibble per tag; 15: Serializable,
// TimerTrigger, SourceCheckpoint, IgnoreCheckpoint, the out-of-line case).
constexpr uint32_t kZLutTrue = 2u | 9u << 4 | 5u << 8 | 15u << 12 | 15u << 16 | 15u << 20 | 15u << 24 | 5u << 28;

struct SpecR {
  Bits sb, wb;     // followed starts in the region / wide ones (registers)
  uint32_t first;  // first position >= rs
  uint32_t exit;   // first position >= re
  uint32_t bad;    // 1 + last position skipped inside the region, 0 if none
};

// Speculative length of a TimerTrigger (tg 4) / SourceCheckpoint (tg 5) at q: only the
// bytes that decide the length are read (type / hasRef byte, then the name / reference
// length when there is one); 0 (step one byte) for an ordinal decodeNext would reject or a
// length past kZSpecMax or the span end.  Speculation only: the true chain re-checks every
// record with the full rules (zlen_var).
__device__ __forceinline__ uint32_t zspec_var(const uint32_t* T, uint32_t q, uint32_t end_a, uint32_t tg) {
  const bool tt = tg == CLG_TAG_TIMER_TRIGGER;
  const uint32_t b = zb8(T, q + (tt ? 13u : 22u));  // TT type ordinal / SC hasRef
  uint32_t L, var_at;
  bool var;
  if (tt) {
    L = b < 6u ? 14u : (b == 6u ? 18u : 0u);
    var = b == 6u;
    var_at = q + 14u;
  } else {
    const uint32_t ord = zb8(T, q + 21u);
    L = ord > 1u ? 0u : (b ? 27u : 23u);
    var = ord <= 1u && b;
    var_at = q + 23u;
  }
  if (var) {  // a name / reference follows: its big-endian length
    const uint32_t n = zbe32(T, var_at);
    L = n <= (uint32_t)kZSpecMax - L ? L + n : 0u;
  }
  return q + L <= end_a ? L : 0u;
}

template <bool J>
__device__ __forceinline__ uint32_t spec_len_fast(const uint32_t* T, uint32_t q, uint32_t end_a, bool safe, const JL& jl,
                                                  bool* wide) {
  constexpr uint32_t kLo = 2u | 9u << 8 | 5u << 16 | (J ? 0x40u : 0u) << 24;  // tags 0..3
  constexpr uint32_t kHi = 0x40u | 0x40u << 8 | 0x40u << 16 | 5u << 24;       // tags 4..7
  const uint32_t tg = zb8(T, q);
  const uint32_t c = __builtin_amdgcn_perm(kHi, kLo, min(tg, 12u)) & 0xFFu;
  uint32_t L = c;
  *wide = false;
  if (c >= 0x40u) {  // rare: the length needs fields of the record
    *wide = true;
    if (tg == CLG_TAG_IGNORE_CHECKPOINT) {
      L = 13;
    } else if (J && tg == CLG_TAG_SERIALIZABLE) {
      L = jl_len(jl, q);
      L = L <= (uint32_t)kZSpecMax ? L : 0u;
    } else {
      L = zspec_var(T, q, end_a, tg);
    }
  }
  if (!safe) L = q + L <= end_a ? L : 0u;
  return L;
}

// One speculative step in the region: the start bit of a followed record goes into sbw and,
// for a wide record, into wbw -- inside the rare branch, so the common path (fixed-length
// tags) pays nothing for the wide bitmap.  SAFE: the record's bytes cannot pass end_a.  A
// skipped byte's bit is set too; the skips are found from the bitmap afterwards (spec_bad).
template <bool J, bool SAFE>
__device__ __forceinline__ uint32_t spec_step(const uint32_t* T, uint32_t q, uint32_t end_a, const JL& jl,
                                              uint64_t& sbw, uint64_t& wbw) {
  constexpr uint32_t kLo = 2u | 9u << 8 | 5u << 16 | (J ? 0x40u : 0u) << 24;  // tags 0..3
  constexpr uint32_t kHi = 0x40u | 0x40u << 8 | 0x40u << 16 | 5u << 24;       // tags 4..7
  const uint32_t tg = zb8(T, q);
  const uint32_t c = __builtin_amdgcn_perm(kHi, kLo, min(tg, 12u)) & 0xFFu;
  uint32_t L = c;
  const uint64_t m = 1ull << (q & 63u);
  if (c >= 0x40u) {  // rare: the length needs fields of the record
    if (tg == CLG_TAG_IGNORE_CHECKPOINT) {
      L = 13;
    } else if (J && tg == CLG_TAG_SERIALIZABLE) {
      L = jl_len(jl, q);
      L = L <= (uint32_t)kZSpecMax ? L : 0u;
    } else {
      L = zspec_var(T, q, end_a, tg);
    }
    if (!SAFE) L = q + L <= end_a ? L : 0u;
    if (L) wbw |= m;
  } else if (!SAFE) {
    L = q + L <= end_a ? L : 0u;
  }
  sbw |= m;
  return q + (L > 1u ? L : 1u);
}

// 1 + the last position a speculative walk skipped in its region (0: none), from its start
// bitmap: every record is at least 2 bytes, so a start followed by a start one byte later
// was a skip, and so was the region's last start if the exit lies one byte past it.  (The
// merge walk uses only starts at or past it; the skipped bytes' own bits are never read.)
__device__ __forceinline__ uint32_t spec_bad(const SpecR& s, uint32_t r0) {
  const uint64_t klo = s.sb.lo & ((s.sb.lo >> 1) | (s.sb.hi << 63));
  const uint64_t khi = s.sb.hi & (s.sb.hi >> 1);
  uint32_t bad = khi ? r0 + 128u - (uint32_t)__clzll(khi) : (klo ? r0 + 64u - (uint32_t)__clzll(klo) : 0u);
  const uint32_t last1 = s.sb.hi ? r0 + 128u - (uint32_t)__clzll(s.sb.hi)
                                 : (s.sb.lo ? r0 + 64u - (uint32_t)__clzll(s.sb.lo) : 0u);  // 1 + last start
  return (last1 && s.exit == last1) ? last1 : bad;
}

template <bool J, bool SAFE>
__device__ __forceinline__ SpecR spec_walk_t(const uint32_t* T, uint32_t ws, uint32_t rs, uint32_t re, uint32_t end_a,
                                             uint32_t r0, const JL& jl) {
  SpecR s{{0, 0}, {0, 0}, rs, rs, 0};
  uint32_t q = ws;
  // warm-up: only where the chain enters the region matters, so any fixed rule will do;
  // this one steps one byte past wide tags (no branch, no field reads) and follows the
  // fixed-length ones
  {
    constexpr uint32_t kLo = 2u | 9u << 8 | 5u << 16;  // tags 0..3 (Serializable: 0)
    constexpr uint32_t kHi = 5u << 24;                  // tags 4..7 (wide: 0)
    while (q < rs) {
      const uint32_t L = __builtin_amdgcn_perm(kHi, kLo, min(zb8(T, q), 12u)) & 0xFFu;
      q += L > 1u ? L : 1u;
    }
  }
  s.first = q;
  const uint32_t mid = re < r0 + 64u ? re : r0 + 64u;
  while (q < mid) q = spec_step<J, SAFE>(T, q, end_a, jl, s.sb.lo, s.wb.lo);
  while (q < re) q = spec_step<J, SAFE>(T, q, end_a, jl, s.sb.hi, s.wb.hi);
  s.exit = q;
  s.bad = spec_bad(s, r0);
  return s;
}

// ---------------------------------------------------------------------------------
// Step-code map (count pass with Serializable tables).  Batches that hold Serializable
// records are dominated by wide records (config 3: 20 %), and a speculative walk that meets
// one takes a divergent branch with two or three dependent LDS reads; with 64 lanes some lane
// is in that branch at almost every step.  So before walking, the wave turns every byte of
// the tile into a step code, data-parallel, in place over the LDS image (same row layout):
//   0      no valid record starts here: the speculative walk steps 1
//   0x80   a valid wide record longer than kZLmMax: the speculative walk steps 1, the true
//          and canonical walks measure it from HBM / the table (lm_true_slow)
//   else   bits 0-6 the record length, bit 7 set for a wide record
// Fixed-length tags come from a byte-permute table over four tags at a time; TimerTrigger
// and SourceCheckpoint bytes (a few per region) get their length from their fields by the
// decodeNext rules (zlen_var); Serializable records get theirs from the phase-3 table
// (load_jl_map).  Every walk then costs one LDS read and no branch per step.  Every code
// was made by the full rules, so the true chain (merge_walk_lm) may follow codes too.
// ---------------------------------------------------------------------------------
constexpr uint32_t kZLmMax = 126;
// codes of tags 0..7: Order 2, Timestamp 9, RNG 5, Serializable 0 (table), TimerTrigger and
// SourceCheckpoint 0 (fields), IgnoreCheckpoint 13 (wide), BufferBuilt 5
constexpr uint32_t kLmLo = 2u | 9u << 8 | 5u << 16;
constexpr uint32_t kLmHi = (0x80u | 13u) << 16 | 5u << 24;
constexpr uint32_t kLmCand = 0x80u | 0x80u << 8;  // tags 4, 5 (the high table word)

__device__ __forceinline__ uint32_t lm8(const uint32_t* M, uint32_t a) { return ((lds_u8*)(M))[zoff(a)]; }
__device__ __forceinline__ void lm8_set(uint32_t* M, uint32_t a, uint32_t c) { ((uint8_t*)(M))[zoff(a)] = (uint8_t)c; }
// code 0x80 (wide, no length): a valid wide record longer than kZLmMax -- the speculative
// chains step one byte, the true and canonical chains measure it by the full rules
__device__ __forceinline__ uint32_t lm_code(int L, bool wide) {
  return (L > 0 && L <= (int)kZLmMax) ? (uint32_t)L | (wide ? 0x80u : 0u) : (L > 0 && wide ? 0x80u : 0u);
}

// One speculative step over the map (bits as spec_step; skips found by spec_bad).
__device__ __forceinline__ uint32_t lm_step(const uint32_t* M, uint32_t q, uint64_t& sbw, uint64_t& wbw) {
  const uint32_t c = lm8(M, q);
  const uint64_t m = 1ull << (q & 63u);
  sbw |= m;
  wbw |= (uint64_t)(c >> 7) << (q & 63u);  // bit 7: a wide record
  const uint32_t L = c & 0x7Fu;
  return q + (L > 1u ? L : 1u);
}
__device__ __forceinline__ SpecR lm_spec_walk(const uint32_t* M, uint32_t ws, uint32_t rs, uint32_t re, uint32_t r0) {
  SpecR s{{0, 0}, {0, 0}, rs, rs, 0};
  uint32_t q = ws;
  while (q < rs) {
    const uint32_t L = lm8(M, q) & 0x7Fu;
    q += L > 1u ? L : 1u;
  }
  s.first = q;
  const uint32_t mid = re < r0 + 64u ? re : r0 + 64u;
  while (q < mid) q = lm_step(M, q, s.sb.lo, s.wb.lo);
  while (q < re) q = lm_step(M, q, s.sb.hi, s.wb.hi);
  s.exit = q;
  s.bad = spec_bad(s, r0);
  return s;
}

// the lean warm-up step: fixed-length tags, one byte past wide ones
__device__ __forceinline__ uint32_t warm_len(uint32_t tg) {
  constexpr uint32_t kLo = 2u | 9u << 8 | 5u << 16;  // tags 0..3 (Serializable: 0)
  constexpr uint32_t kHi = 5u << 24;                  // tags 4..7 (wide: 0)
  const uint32_t L = __builtin_amdgcn_perm(kHi, kLo, min(tg, 12u)) & 0xFFu;
  return L > 1u ? L : 1u;
}

// ---------------------------------------------------------------------------------
// The lean speculative walk (FusedCtl::lean; batches without tables whose records are
// almost all fixed-length, as config 2's Order / Timestamp): the warm-up's rule in the
// region too -- fixed-length tags followed, anything else (wide tags included) one byte --
// so a step has no branch for wide records, and the starts go into four 32-bit words (a
// 32-bit shift and OR instead of a 64-bit shift and two ORs).  Its chain has no wide
// records: a wide record on it is a skip, which spec_bad puts before the merge's meeting
// point, so the true walk (full rules) crosses every wide record of the region itself and
// the result is the same; only its cost grows with wide records, which is why the host
// turns it off for batches that hold many (engine.cpp lean_hint).
// ---------------------------------------------------------------------------------
template <bool SAFE>
__device__ __forceinline__ SpecR lean_walk(const uint32_t* T, uint32_t ws, uint32_t rs, uint32_t re, uint32_t end_a,
                                           uint32_t r0) {
  SpecR s{{0, 0}, {0, 0}, rs, rs, 0};
  uint32_t q = ws;
  while (q < rs) q += warm_len(zb8(T, q));
  s.first = q;
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t lim = re < r0 + 32u * (uint32_t)(k + 1) ? re : r0 + 32u * (uint32_t)(k + 1);
    uint32_t b = 0;
    while (q < lim) {
      constexpr uint32_t kLo = 2u | 9u << 8 | 5u << 16;  // tags 0..3 (Serializable: 0)
      constexpr uint32_t kHi = 5u << 24;                  // tags 4..7 (wide: 0)
      uint32_t L = __builtin_amdgcn_perm(kHi, kLo, min(zb8(T, q), 12u)) & 0xFFu;
      if (!SAFE) L = q + L <= end_a ? L : 0u;
      b |= 1u << (q & 31u);
      q += L > 1u ? L : 1u;
    }
    w[k] = b;
  }
  s.sb.lo = (uint64_t)w[0] | (uint64_t)w[1] << 32;
  s.sb.hi = (uint64_t)w[2] | (uint64_t)w[3] << 32;
  s.exit = q;
  s.bad = spec_bad(s, r0);
  return s;
}

// The region's speculative walk: over the step-code map (batches with tables), the lean walk,
// or spec_walk_t.  (Two chains per lane in lockstep -- the region's halves walked at once --
// was measured slower, config-2 count 0.161 -> 0.209 ms: the walk is issue-bound, and the
// second chain's VALU cost more than its overlap saved; round 4.)  wsb is unused.
template <bool J>
__device__ __forceinline__ SpecR spec_walk_fast(const uint32_t* T, uint32_t ws, uint32_t wsb, uint32_t rs, uint32_t re,
                                                uint32_t end_a, uint32_t r0, const JL& jl, bool lean = false) {
  if (J && jl.lm) return lm_spec_walk(jl.lm, ws, rs, re, r0);
  if (!J && lean) return re + 16u <= end_a ? lean_walk<true>(T, ws, rs, re, end_a, r0) : lean_walk<false>(T, ws, rs, re, end_a, r0);
  // lanes whose records cannot run past the span end (all but the last tile's) skip the test
  if (re + 16u <= end_a) return spec_walk_t<J, true>(T, ws, rs, re, end_a, r0, jl);
  return spec_walk_t<J, false>(T, ws, rs, re, end_a, r0, jl);
}

// True chain from entry e (e >= rs) merged with the speculative chain: walk until the true
// chain lands on a speculative start past the speculative chain's last skip.  The walk runs
// over the region's two 64-bit bitmap halves in turn (as spec_walk_t), so a start costs one
// 64-bit shift and OR; `step(p, &L, &wide)` is the true length rule (false: decodeNext
// rejects the record, *why set).
template <class Step>
__device__ __forceinline__ Res merge_walk_h(uint32_t re, uint32_t end_a, uint32_t e, const SpecR& s, Step&& step) {
  Res r{{0, 0}, {0, 0}, e, 0, 0, 0};
  if (e >= re) return r;
  const uint32_t r0 = (re - 1u) & ~(kZRegion - 1u);
  uint32_t p = e, why = 0;
  Bits pb{0, 0}, pw{0, 0};
  // 0: reached lim, 1: met the speculative chain, 2: an invalid record
  auto run = [&](uint64_t sbw, uint64_t& pbw, uint64_t& pww, uint32_t lim) -> uint32_t {
    for (; p < lim; ++r.steps) {
      const uint32_t b = p & 63u;
      if (((sbw >> b) & 1ull) && p >= s.bad) return 1u;
      uint32_t L;
      bool w;
      if (!step(p, &L, &w, &why)) return 2u;
      if (p + L > end_a || p + L < p) {
        why = 1;
        return 2u;
      }
      const uint64_t m = 1ull << b;
      pbw |= m;
      if (w) pww |= m;
      p += L;
    }
    return 0u;
  };
  const uint32_t mid = re < r0 + 64u ? re : r0 + 64u;
  uint32_t st = run(s.sb.lo, pb.lo, pw.lo, mid);
  if (st == 0u) st = run(s.sb.hi, pb.hi, pw.hi, re);
  if (st == 1u) {
    const uint32_t i = p & 127u;
    r.bm = bor(pb, bge(s.sb, i));
    r.wb = bor(pw, bge(s.wb, i));
    r.exit = s.exit;
  } else if (st == 2u) {
    r.bad = why;
    r.exit = s.exit;
    r.bm = pb;  // the true starts before the failing record
    r.wb = pw;
    r.fail = p;
  } else {
    r.bm = pb;
    r.wb = pw;
    r.exit = p;
  }
  return r;
}

template <bool J>
__device__ __forceinline__ Res merge_walk_r(const uint32_t* T, uint32_t re, uint32_t end_a, uint32_t e, const SpecR& s,
                                            const JL& jl) {
  return merge_walk_h(re, end_a, e, s, [&](uint32_t p, uint32_t* Lp, bool* w, uint32_t* why) -> bool {
    const uint32_t tg = zb8(T, p);
    uint32_t L = __builtin_amdgcn_ubfe(kZLutTrue, tg << 2, 4);
    *w = false;
    if (L == 15u || tg >= 8u) {
      int v;
      uint32_t y = 1u;
      if (tg >= 8u) {
        v = (int)kLenErr;
      } else if (tg == CLG_TAG_SERIALIZABLE) {
        if (J) {
          const uint32_t jv = jl_len(jl, p);
          v = jv ? (int)jv : (int)kLenErr;
        } else {
          v = (int)kLenErr;
          y = zbe32(T, p + 1) == 0xACED0005u ? 2u : 1u;
        }
      } else {
        v = tg == CLG_TAG_IGNORE_CHECKPOINT ? 13 : zlen_var(T, p, end_a, tg, 0);
      }
      if (v <= 0) {
        *why = y;
        return false;
      }
      L = (uint32_t)v;
      *w = true;
    }
    *Lp = L;
    return true;
  });
}

// The true chain of a batch without tables (merge_walk_r<false>'s result) in a tight loop:
// the fixed-length tags (Order, Timestamp, RNG, BufferBuilt) by one byte-permute lookup, and
// ONE exit test per step for the three things that end the fast loop -- the chain met the
// speculative one (at or past its last skip), a tag that needs the full rule (wide, invalid,
// Serializable: length 0 in the table), a record past the span end.  The full rule then
// takes that one record (merge_walk_r's step) and the loop goes on.  merge_walk_r's nested
// rare branches cost about twice the VALU and SALU of this loop per step (the count pass's
// ISA), and the merges are the count pass's second-largest phase after the speculative walk.
__device__ __forceinline__ Res merge_walk_lean(const uint32_t* T, uint32_t re, uint32_t end_a, uint32_t e,
                                               const SpecR& s) {
  Res r{{0, 0}, {0, 0}, e, 0, 0, 0};
  if (e >= re) return r;
  const uint32_t r0 = (re - 1u) & ~(kZRegion - 1u);
  uint32_t p = e, why = 0;
  Bits pb{0, 0}, pw{0, 0};
  // 0: reached lim, 1: met the speculative chain, 2: an invalid record
  auto run = [&](uint64_t sbw, uint64_t& pbw, uint64_t& pww, uint32_t lim) -> uint32_t {
    while (p < lim) {
      constexpr uint32_t kLo = 2u | 9u << 8 | 5u << 16;  // tags 0..3 (Serializable: 0)
      constexpr uint32_t kHi = 5u << 24;                  // tags 4..7 (wide: 0)
      const uint32_t b = p & 63u;
      const uint64_t m = 1ull << b;
      const bool conv = (sbw & m) != 0ull && p >= s.bad;
      const uint32_t tg = zb8(T, p);
      const uint32_t L = __builtin_amdgcn_perm(kHi, kLo, min(tg, 12u)) & 0xFFu;
      if (conv || L == 0u || p + L > end_a) {
        if (conv) return 1u;
        // the full rule for this record (merge_walk_r's step)
        int v;
        uint32_t y = 1u;
        if (tg >= 8u) {
          v = (int)kLenErr;
        } else if (tg == CLG_TAG_SERIALIZABLE) {
          v = (int)kLenErr;
          y = zbe32(T, p + 1) == 0xACED0005u ? 2u : 1u;
        } else if (L) {  // a fixed-length record past the span end
          v = (int)kLenErr;
        } else {
          v = tg == CLG_TAG_IGNORE_CHECKPOINT ? 13 : zlen_var(T, p, end_a, tg, 0);
        }
        if (v <= 0 || p + (uint32_t)v > end_a || p + (uint32_t)v < p) {
          why = v <= 0 ? y : 1u;
          return 2u;
        }
        pbw |= m;
        pww |= m;
        p += (uint32_t)v;
        ++r.steps;
        continue;
      }
      pbw |= m;
      p += L;
      ++r.steps;
    }
    return 0u;
  };
  const uint32_t mid = re < r0 + 64u ? re : r0 + 64u;
  uint32_t st = run(s.sb.lo, pb.lo, pw.lo, mid);
  if (st == 0u) st = run(s.sb.hi, pb.hi, pw.hi, re);
  if (st == 1u) {
    const uint32_t i = p & 127u;
    r.bm = bor(pb, bge(s.sb, i));
    r.wb = bor(pw, bge(s.wb, i));
    r.exit = s.exit;
  } else if (st == 2u) {
    r.bad = why;
    r.exit = s.exit;
    r.bm = pb;  // the true starts before the failing record
    r.wb = pw;
    r.fail = p;
  } else {
    r.bm = pb;
    r.wb = pw;
    r.exit = p;
  }
  return r;
}

// ---------------------------------------------------------------------------------
// Hand-off words.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent32(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The words other blocks poll: pk_word / pk_state / pk_val (handoff.h).
// abort[0]: nonzero once any tile aborted (polled by waiting tiles); abort[r], r = 1..4:
// ~(lowest tile that aborted for reason r), for diagnostics.
// An invalid record at span offset so on a true chain of span `span` (the lowest one wins).
__device__ __forceinline__ void note_error(const FusedCtl& ctl, uint32_t span, uint64_t so) {
  if (ctl.span_err && so != ~0ull) atomicMin(reinterpret_cast<unsigned long long*>(ctl.span_err + span), (unsigned long long)so);
}
__device__ __forceinline__ void raise_abort(const FusedCtl& c, uint32_t reason, uint32_t t) {
  __hip_atomic_store(c.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_max(c.abort + reason, ~t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Polling backoff: every poll is an L2-bypassing load, and thousands of waves poll at
// once, so waiting waves sleep 0.1-3 us between polls (doubling) to leave the memory
// system to the waves that stage tiles.
constexpr uint64_t kZSpinLimit = 1ull << 29;  // ~0.2 s of shader clock: give up and abort
__device__ __forceinline__ bool backoff(uint32_t& n, uint64_t t0) {
  for (uint32_t i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(32);  // ~2k cycles each
  n = n < 16u ? n * 2u : 16u;
  return __builtin_amdgcn_s_memtime() - t0 < kZSpinLimit;
}

// Count words: [61:31] wide records | [30:0] records.
__device__ __forceinline__ uint64_t pack_cnt(uint32_t rec, uint32_t wide) { return (uint64_t)wide << 31 | rec; }

// Stage tile t into the padded row layout: the tile (16-byte loads, all in flight before
// any LDS store), a halo of the span's next bytes, a zero pad, then every row's pad dwords.
// kHaloMax bytes of halo (kZHalo for count / emit; phase 3 stages more so that whole
// Serializable streams near the tile end are in LDS); kRows rows of image.  n1: the next
// tile's descriptor when the caller has it.  If that tile continues the span and holds the
// whole halo (every tile but a span's last two, normally), the halo bytes are loaded
// together with the tile, so staging costs one memory latency; otherwise the halo is found
// by walking the span's tiles.
// A tile's words in registers between stage_issue (loads in flight) and stage_finish (LDS
// stores): the count pass issues the next tile's loads right after staging the current one,
// so their memory latency passes during the current tile's walk.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kZLoads = (int)(kZTile / 16 / 64);
struct StagePre {
  u32x4 v[kZLoads];
  u32x4 hv[2];
  uint32_t hb;
};
template <uint32_t kHaloMax = kZHalo>
struct StageGeom {
  uint32_t t1, halo, img_end;
  uint64_t after;
  bool near, far;
  __device__ __forceinline__ StageGeom(const TileDesc& td, const SpanDesc& sd, uint32_t t, uint32_t hi,
                                       const TileDesc* n1) {
    t1 = sd.first_tile + sd.n_tiles;
    after = td.span_off + td.len;
    const uint64_t rem = sd.len > after ? sd.len - after : 0;
    halo = rem < (uint64_t)kHaloMax ? (uint32_t)rem : kHaloMax;
    img_end = hi + halo;
    const bool next_ok = n1 && halo && t + 1 < t1 && n1->span_off == after && n1->len >= halo;
    near = kHaloMax <= 64u && next_ok;  // one byte per lane
    far = kHaloMax > 64u && next_ok;    // phase 3: up to 1 KiB, 16-byte words
  }
};
// Every lane issues its 8 loads (and its halo byte / words) -- the tile is at most 512 x 16 B.
template <uint32_t kHaloMax = kZHalo>
__device__ __forceinline__ void stage_issue(const TileDesc& td, const SpanDesc& sd, const uint32_t t, const uint32_t lane,
                                            const uint32_t hi, const TileDesc* n1, StagePre& P) {
  static_assert(kHaloMax <= 64u * 16u * 2u - 32u, "halo words: two per lane");
  const StageGeom<kHaloMax> G(td, sd, t, hi, n1);
  const uint32_t words = (hi + 15) >> 4;
  const CLG_GLOBAL u32x4* src = gp(reinterpret_cast<const u32x4*>(td.abase));
#pragma unroll
  for (int i = 0; i < kZLoads; ++i) {  // branch-free: lanes past the tile re-read its last word
    const uint32_t w = lane + 64u * (uint32_t)i;
    P.v[i] = src[w < words ? w : words - 1u];
  }
  P.hb = 0;
  if (G.near && lane < G.halo) P.hb = gp(n1->abase)[n1->delta + lane];
  if (G.far) {
    const uint32_t nw = (n1->delta + G.halo + 15u) >> 4;
    const CLG_GLOBAL u32x4* src1 = gp(reinterpret_cast<const u32x4*>(n1->abase));
    P.hv[0] = lane < nw ? src1[lane] : u32x4{0, 0, 0, 0};
    P.hv[1] = lane + 64u < nw ? src1[lane + 64u] : u32x4{0, 0, 0, 0};
  }
}

// Stage tile t into the padded row layout: the tile (16-byte loads, all in flight before
// any LDS store), a halo of the span's next bytes, a zero pad, then every row's pad dwords.
// kHaloMax bytes of halo (kZHalo for count / emit; phase 3 stages more so that whole
// Serializable streams near the tile end are in LDS); kRows rows of image.  n1: the next
// tile's descriptor when the caller has it.  If that tile continues the span and holds the
// whole halo (every tile but a span's last two, normally), the halo bytes are loaded
// together with the tile, so staging costs one memory latency; otherwise the halo is found
// by walking the span's tiles.  P: the words stage_issue loaded (same tile, same n1).
template <uint32_t kHaloMax = kZHalo, uint32_t kRows = kZRows>
__device__ __forceinline__ void stage_finish(const TileDesc& td, const SpanDesc& sd, const uint32_t t,
                                             const TileDesc* __restrict__ tiles, uint32_t* s_img, const uint32_t lane,
                                             const uint32_t hi, const TileDesc* n1, const StagePre& P) {
  static_assert((kZTile + 15 + kHaloMax + 64 + 127) / 128 <= kRows, "image rows: tile + halo + zero pad");
  const StageGeom<kHaloMax> G(td, sd, t, hi, n1);
  const uint32_t t1 = G.t1, halo = G.halo, img_end = G.img_end;
  const uint64_t after = G.after;
  const bool near = G.near, far = G.far;
  const uint32_t hb = P.hb;
  const u32x4* hv = P.hv;
  {
    const uint32_t words = (hi + 15) >> 4;
#pragma unroll
    for (int i = 0; i < kZLoads; ++i) {
      const uint32_t w = lane + 64u * (uint32_t)i;
      if (w < words) {
        uint32_t* d = s_img + (w >> 3) * kZPitch + 4u * (w & 7u);
        d[0] = P.v[i].x;
        d[1] = P.v[i].y;
        d[2] = P.v[i].z;
        d[3] = P.v[i].w;
      }
    }
  }
  __syncthreads();  // the tile's last word may run past hi: the halo overwrites it
  {
    uint8_t* bb = reinterpret_cast<uint8_t*>(s_img);
    if (near) {
      if (lane < halo) bb[rb(hi + lane)] = (uint8_t)hb;
    } else if (far && ((hi - n1->delta) & 15u) == 0u) {
      // the usual case: tiles split at 8 KiB inside a segment or at a segment's end, so the
      // next tile starts at this one's end in the same 16-byte alignment and its words land
      // on 16-byte image boundaries whole (bytes past the halo fall under the zero pad or
      // past the image's end; only the first word's bytes before the next tile are skipped)
      const uint32_t nw = (n1->delta + halo + 15u) >> 4;
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t c = lane + 64u * k;
        if (c >= nw) continue;
        const uint32_t at = hi - n1->delta + 16u * c;  // image position of the word's byte 0
        if (16u * c >= n1->delta) {
          uint32_t* d = s_img + rk(at >> 2);
          d[0] = hv[k].x;
          d[1] = hv[k].y;
          d[2] = hv[k].z;
          d[3] = hv[k].w;
        } else {
          const uint32_t w[4] = {hv[k].x, hv[k].y, hv[k].z, hv[k].w};
#pragma unroll
          for (uint32_t b = 0; b < 16; ++b)
            if (16u * c + b >= n1->delta) bb[rb(at + b)] = (uint8_t)(w[b >> 2] >> (8u * (b & 3u)));
        }
      }
    } else if (far) {
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t c = lane + 64u * k;
        const uint32_t w[4] = {hv[k].x, hv[k].y, hv[k].z, hv[k].w};
#pragma unroll
        for (uint32_t b = 0; b < 16; ++b) {
          const uint32_t x = 16u * c + b;  // byte of the next tile's aligned coordinates
          if (x >= n1->delta && x < n1->delta + halo) bb[rb(hi + x - n1->delta)] = (uint8_t)(w[b >> 2] >> (8u * (b & 3u)));
        }
      }
    } else {
      const TileDesc nn = halo ? tiles[t + 1] : td;
      if (kHaloMax > 64u && halo > 64u && nn.span_off == after && nn.len >= halo) {
        // the next tile holds the whole halo: 16-byte loads, byte stores
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        for (uint32_t c = lane; 16u * c < nn.delta + halo; c += 64) {
          const u32x4 v = gp(reinterpret_cast<const u32x4*>(nn.abase))[c];
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (uint32_t b = 0; b < 16; ++b) {
            const uint32_t x = 16u * c + b;  // byte of the next tile's aligned coordinates
            if (x >= nn.delta && x < nn.delta + halo) bb[rb(hi + x - nn.delta)] = (uint8_t)(w[b >> 2] >> (8u * (b & 3u)));
          }
        }
      } else {
        uint32_t k = t + 1;
        for (uint32_t i = lane; i < halo; i += 64) {
          const uint64_t o = after + i;  // span offset of the halo byte
          while (k + 1 < t1 && o >= tiles[k].span_off + tiles[k].len) ++k;
          const TileDesc nt = tiles[k];
          bb[rb(hi + i)] = gp(nt.abase)[nt.delta + (uint32_t)(o - nt.span_off)];
        }
      }
    }
    bb[rb(img_end + lane)] = 0;  // zero pad (64 bytes) so 16-byte reads near the end are defined
  }
  __syncthreads();
}


template <uint32_t kHaloMax = kZHalo, uint32_t kRows = kZRows>
__device__ __forceinline__ void stage_image(const TileDesc& td, const SpanDesc& sd, const uint32_t t,
                                            const TileDesc* __restrict__ tiles, uint32_t* s_img, const uint32_t lane,
                                            const uint32_t hi, const TileDesc* n1 = nullptr) {
  StagePre P;
  stage_issue<kHaloMax>(td, sd, t, lane, hi, n1, P);
  stage_finish<kHaloMax, kRows>(td, sd, t, tiles, s_img, lane, hi, n1, P);
}

// ---------------------------------------------------------------------------------
// One 64-lane workgroup decodes one tile at a time (persistent grid, below).
// ---------------------------------------------------------------------------------
// Tile geometry shared by the passes.
struct ZTile {
  TileDesc td;
  SpanDesc sd;
  uint32_t lo, hi, end_a, rs, re;
  bool first, last;  // first / last tile of its span
};
__device__ __forceinline__ ZTile ztile_of(const TileDesc& td, const SpanDesc& sd, uint32_t t, uint32_t lane) {
  ZTile z;
  z.td = td;
  z.sd = sd;
  z.first = t == z.sd.first_tile;
  z.last = t + 1 == z.sd.first_tile + z.sd.n_tiles;
  z.lo = z.td.delta;
  z.hi = z.td.delta + z.td.len;
  const uint64_t ea = z.sd.len - z.td.span_off + z.td.delta;
  z.end_a = ea > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)ea;
  const uint32_t r0 = lane * kZRegion;
  z.rs = r0 < z.lo ? z.lo : (r0 > z.hi ? z.hi : r0);
  z.re = r0 + kZRegion > z.hi ? z.hi : r0 + kZRegion;
  return z;
}
__device__ __forceinline__ ZTile ztile(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans, uint32_t t,
                                       uint32_t lane) {
  const TileDesc td = tiles[t];
  return ztile_of(td, spans[td.span], t, lane);
}

// Build the map in place over the tile's rows of the image (every lane of the wave calls it:
// it holds barriers).  The codes stay in registers until every lane has read the fields it
// needs (a record's fields reach into the next row).  The span's end is applied last.
// The tile's TimerTrigger / SourceCheckpoint bytes are compacted into `list` (the table's
// LDS, free until load_jl_map) and measured 64 at a time, every lane busy: measured per
// lane, a wave ran as many field decodes as its busiest lane's count, at about half lane use.
// A tile with more than kZLmList such bytes leaves the rest at code 0 (a deterministic
// function of the tile, like the rest of the map).
constexpr uint32_t kZLmList = 2 * kZJBitsDw + kZJCap;
__device__ __forceinline__ void build_lm(const ZTile& z, uint32_t* T, uint32_t* list, const uint32_t lane) {
  const bool on = z.rs < z.re;
  const uint32_t r0 = lane * kZRegion;
  uint32_t c[kZRowDw];
  // TimerTrigger / SourceCheckpoint bytes: word h, bit 32 s + 8 b + k <-> dword 16 h + 8 s + k of
  // the lane's set, byte b
  uint64_t cw0 = 0, cw1 = 0;
  // The lane's dwords: its row (dword j of row `lane`), or without row pads (pitch 32, where a
  // row-per-lane read puts all 32 lanes of a group on one bank) dword 64 j + lane of the tile,
  // so the lanes of a read touch 64 consecutive dwords.
  constexpr bool kCols = true;  // (the unpadded image)
  // (kCols) bit j: the row of dword 64 j + lane, 2 j + (lane >> 5), meets the tile (rows from 0,
  // since lo < 16, to (hi - 1) >> 7)
  const int32_t jmax = z.hi > z.lo ? ((int32_t)((z.hi - 1u) >> 7) - (int32_t)(lane >> 5)) >> 1 : -1;
  const uint32_t onm = jmax < 0 ? 0u : (jmax >= 31 ? 0xFFFFFFFFu : (2u << jmax) - 1u);
#pragma unroll
  for (uint32_t j = 0; j < kZRowDw; ++j) {
    const uint32_t x = kCols ? T[64u * j + lane] : T[lane * kZPitch + j];
    // 0xFF in every byte holding a tag (< 8): bytes with none of bits 3-7 set
    const uint32_t h = x & 0xF8F8F8F8u;
    const uint32_t zz = (h - 0x01010101u) & ~h & 0x80808080u;
    const uint32_t vm = __builtin_amdgcn_perm(zz << 8, zz, 0x090B080Au);  // sign of each byte
    c[j] = __builtin_amdgcn_perm(kLmHi, kLmLo, x) & vm;
    const uint64_t f = (uint64_t)((__builtin_amdgcn_perm(kLmCand, 0u, x) & vm) >> (7u - (j & 7u))) << (32u * ((j >> 3) & 1u));
    if (j < 16u) cw0 |= f; else cw1 |= f;
  }
  if (!kCols && !on) cw0 = cw1 = 0;
  // the lanes' candidates into the list, in lane order
  const uint32_t nc = (uint32_t)(__popcll(cw0) + __popcll(cw1));
  const uint32_t incl = wave_scan_u32(nc, lane);
  const uint32_t n = min(lane63(incl), kZLmList);
  uint32_t idx = incl - nc;
#pragma unroll 1
  for (uint32_t hh = 0; hh < 2; ++hh) {
    uint64_t m = hh ? cw1 : cw0;
    while (m) {
      const uint32_t i = (uint32_t)__builtin_ctzll(m);
      m &= m - 1u;
      const uint32_t jj = 16u * hh + 8u * (i >> 5) + (i & 7u), b = (i >> 3) & 3u;  // the lane's dword, byte
      const uint32_t a = kCols ? 4u * (64u * jj + lane) + b : r0 + 4u * jj + b;
      // (a row may run past the tile: those bytes are no candidates)
      if (idx < kZLmList) list[idx] = (kCols ? a >= z.lo && a < z.hi : a >= z.rs && a < z.re) ? a : 0xFFFFu;
      ++idx;
    }
  }
  __syncthreads();
  // their codes, 64 at a time: the length from the fields (the rules of decodeNext)
  for (uint32_t k = lane; k < n; k += 64) {
    const uint32_t a = list[k];
    const uint32_t code = a != 0xFFFFu ? lm_code(zlen_var(T, a, z.end_a, zb(T, a), 0u), true) : 0u;
    list[k] = a | code << 16;
  }
  __syncthreads();  // every lane has read the image
#pragma unroll
  for (uint32_t j = 0; j < kZRowDw; ++j)
    if ((onm >> j) & 1u) T[64u * j + lane] = c[j];
  __syncthreads();  // the rows hold codes: the candidates' go over them
  for (uint32_t k = lane; k < n; k += 64) {
    const uint32_t e = list[k];
    if (e >> 16) lm8_set(T, e & 0xFFFFu, e >> 16);
  }
  // the span's end: a fixed-length record must end by end_a (the wide ones were checked)
  if (on && z.end_a < r0 + kZRegion + 13u) {
    for (uint32_t a = z.end_a > r0 + 13u ? z.end_a - 13u : r0; a < r0 + kZRegion; ++a) {
      const uint32_t cc = lm8(T, a);
      if (a + (cc & 0x7Fu) > z.end_a) lm8_set(T, a, 0u);
    }
  }
}

// Span bytes from HBM by aligned coordinate (the map's true walk, for a code of 0: an
// invalid record, or one the map does not hold).
struct GSpan {
  const TileDesc* tiles;
  uint32_t t, t1, lo;
  uint64_t so;  // span offset of aligned coordinate lo
  __device__ uint32_t at(uint32_t a) const {
    const uint64_t o = so + (a - lo);
    uint32_t k = t;
    while (k + 1 < t1 && o >= tiles[k].span_off + tiles[k].len) ++k;
    const TileDesc d = tiles[k];
    return gp(d.abase)[d.delta + (uint32_t)(o - d.span_off)];
  }
};
struct GRec {
  GSpan g;  // by value: no address taken, the span stays in registers
  uint32_t base;
  __device__ int operator()(uint64_t k) const { return (int)g.at(base + (uint32_t)k); }
};
__device__ __forceinline__ uint32_t fld_be32(const GRec& b, uint32_t k) {
  return (uint32_t)b(k) << 24 | (uint32_t)b(k + 1) << 16 | (uint32_t)b(k + 2) << 8 | (uint32_t)b(k + 3);
}
// True length of the record at p by the full rules (-1: decodeNext rejects it); *wide.
__device__ __forceinline__ int lm_true_slow(const GSpan& g, uint32_t p, uint32_t end_a, const JL& jl, uint32_t* wide) {
  const uint32_t tg = g.at(p);
  *wide = is_wide((int)tg);
  if (tg == CLG_TAG_SERIALIZABLE) {
    const uint32_t v = jl_len(jl, p);
    return v ? (int)v : -1;
  }
  const int64_t L = len_fields(GRec{g, p}, (int)tg, (uint64_t)(end_a - p));
  return (L > 0 && L <= 0x7FFFFFF0ll) ? (int)L : -1;
}

// merge_walk_r over the map: the true chain takes a code's length (the full rules made it)
// and asks HBM only where the code is 0.
__device__ __forceinline__ Res merge_walk_lm(const uint32_t* M, uint32_t re, uint32_t end_a, uint32_t e, const SpecR& s,
                                             const JL& jl, const GSpan& g) {
  return merge_walk_h(re, end_a, e, s, [&](uint32_t p, uint32_t* Lp, bool* w, uint32_t* why) -> bool {
    const uint32_t cc = lm8(M, p);
    uint32_t L = cc & 0x7Fu, wu = cc >> 7;
    if (!L) {
      const int v = lm_true_slow(g, p, end_a, jl, &wu);
      if (v <= 0) {
        *why = 1;
        return false;
      }
      L = (uint32_t)v;
    }
    *Lp = L;
    *w = wu != 0;
    return true;
  });
}

// Canonical chain through the region from entry e: the speculative rule, except at a byte
// it skips that holds a valid Serializable / TimerTrigger / SourceCheckpoint record too long
// for it (map code 0x80; without the map: a zero speculative length) -- that record is
// measured by the full rules (up to a tile), so a long record across the tile end leaves
// the canonical exit at its end, where the true chain exits, not inside it.  The chain
// meets the region's speculative chain at a start at or past its last skip (from there on
// the two rules agree, so its exit is the region's).
template <bool J>
__device__ __forceinline__ uint32_t canon_walk_r(const uint32_t* T, uint32_t re, uint32_t end_a, uint32_t e,
                                                 const SpecR& s, const JL& jl, const GSpan& g) {
  if (e >= re) return e;
  const uint32_t r0 = (re - 1u) & ~(kZRegion - 1u);
  uint32_t p = e;
  while (p < re) {
    const uint32_t i = p - r0;
    if ((((i < 64u ? s.sb.lo : s.sb.hi) >> (i & 63u)) & 1ull) && p >= s.bad) return s.exit;
    uint32_t L;
    int v = 0;
    if (J && jl.lm) {
      const uint32_t c = lm8(jl.lm, p);
      L = c & 0x7Fu;
      if (c == 0x80u) {
        uint32_t w;
        v = lm_true_slow(g, p, end_a, jl, &w);
      }
    } else {
      bool w;
      L = spec_len_fast<J>(T, p, end_a, false, jl, &w);
      if (!L) {
        const uint32_t tg = zb8(T, p);
        if (tg == CLG_TAG_TIMER_TRIGGER || tg == CLG_TAG_SOURCE_CHECKPOINT) v = zlen_var(T, p, end_a, tg, 0u);
        else if (J && tg == CLG_TAG_SERIALIZABLE) v = (int)min(jl_len(jl, p), 0x7FFFFFFFu);
      }
    }
    if (!L) L = (v > 0 && v <= (int)kZTile) ? (uint32_t)v : 1u;
    p += L;
  }
  return p;
}

// Canonical exit of the tile from the lanes' speculative walks: lanes >= c0 (the last
// kZCanonLanes regions) chain their speculative exits, lane c0 starting from its own
// speculative chain; lanes whose entry changed merge again.
template <bool J>
__device__ __forceinline__ uint32_t canon_exit_r(const ZTile& z, const uint32_t* s_img, const SpecR& sp, uint32_t lane,
                                                 const JL& jl, const TileDesc* __restrict__ tiles, uint32_t t) {
  const GSpan g{tiles, t, z.sd.first_tile + z.sd.n_tiles, z.lo, z.td.span_off};
  const uint32_t last_l = z.hi > z.lo ? (z.hi - 1) >> 7 : 0;
  const uint32_t c0 = last_l >= kZCanonLanes - 1 ? last_l - (kZCanonLanes - 1) : 0;
  const bool on = lane >= c0 && z.rs < z.re;
  uint32_t cx = on ? sp.exit : z.rs, entry = kZCanon;
  for (int it = 0; it <= 64; ++it) {
    const uint32_t prev = wave_prev_u32(cx);
    const uint32_t want = lane <= c0 ? kZCanon : prev;
    const bool ch = want != entry;
    if (!__any(ch)) break;
    if (ch) {
      entry = want;
      cx = on ? canon_walk_r<J>(s_img, z.re, z.end_a, want, sp, jl, g) : want;
    }
  }
  return lane63(cx);
}

// Where lane `lane`'s speculative warm-up starts, warm bytes before its region start rs.
// Without row pads every region starts on bank 0, so the lanes' first reads would all hit
// one bank: the warm-up grows by 4 ((lane >> 1) & 15) bytes (the walk is a function of the
// tile's bytes either way).
constexpr uint32_t kZWarmFlat = 1u << 31;  // FusedCtl::warm flag: no stagger (a lone wave: latency first)
__device__ __forceinline__ uint32_t warm_start(uint32_t rs, uint32_t lo, uint32_t warm, uint32_t lane) {
  // Regions start 32 dwords apart, so the lanes' first reads hit banks 0 and 32 only (by lane
  // parity) and, walking at similar speeds, keep colliding.  The stagger's dword offsets
  // spread them: (lane >> 1) & 15 with the parity gives 32 banks (config-2 count 0.165 ->
  // 0.153 ms against lane & 7's 8 banks; tools/ab.sh), at 30 B more warm-up on average.
  // ((lane >> 1) & 31, every lane's first read on its own bank, costs 30 B more warm-up again)
  const uint32_t st = (lane >> 1) & 15u;
  const uint32_t w = (warm & kZWarmFlat) ? (warm & ~kZWarmFlat) : warm + 4u * st;
  return rs >= lo + w ? rs - w : lo;
}

// Pass 1 for one tile, given its true entry e_true (aligned coordinate): spec walks,
// true chain, exit checks, then the tile's record / wide-record counts and its
// record-start bitmap (1 KiB) for the emit pass.  *x_true = the tile's exit.  must_exit:
// the exit the successor already uses (kZCanon: none).  Returns 0, or the reason the chain
// went wrong (the caller decides what it means): 1 an invalid record, 2 the last record
// does not end at the span end, 5 a Serializable record without tables -- no counts
// written -- or 3: the exit is not must_exit (counts written: the tile itself is right,
// the successor entered at the wrong place).
template <bool J>
__device__ __forceinline__ uint32_t count_tile(const uint32_t t, const ZTile& z, const uint32_t e_true,
                                           const uint32_t must_exit, const FusedCtl& ctl, const uint32_t* s_img,
                                           const uint32_t lane, uint32_t* x_out, const JL& jl,
                                           const TileDesc* __restrict__ tiles = nullptr,
                                           const SpecR* walked = nullptr, uint64_t* cnt_out = nullptr,
                                           uint64_t* bm_out = nullptr, uint32_t* fail_out = nullptr) {
#define ZPHASE(i) \
  if (ctl.prof && lane == 0) ctl.prof[(uint64_t)t * 8 + (i)] = __builtin_amdgcn_s_memtime()
  ZPHASE(1);
  const uint32_t lo = z.lo, rs = z.rs, re = z.re, end_a = z.end_a;
  // ---- speculative walk of the lane's region (with warm-up), starts in registers (walked:
  // the chunk prologue's walk of this same tile, a function of the tile's bytes only)
  const uint32_t ws = warm_start(rs, lo, ctl.warm, lane), wsb = warm_start(lane * kZRegion + 64u, lo, ctl.warm, lane);
  const SpecR sp = walked ? *walked
                          : rs < re ? spec_walk_fast<J>(s_img, ws, wsb, rs, re, end_a, lane * kZRegion, jl, ctl.lean != 0u)
                                    : SpecR{{0, 0}, {0, 0}, rs, rs, 0};

  ZPHASE(2);
  // ---- true chain: lanes merge from guessed entries (the previous lane's speculative
  // exit; lane 0 the true entry), then lanes whose entry changed re-merge until the chain
  // is consistent (each pass fixes at least the lowest changed lane)
  const uint32_t guess = wave_prev_u32(sp.exit);
  uint32_t entry = lane == 0 ? e_true : guess;
  const GSpan g{tiles, t, z.sd.first_tile + z.sd.n_tiles, lo, z.td.span_off};
  auto merge = [&](uint32_t from) -> Res {
    if (rs >= re) return Res{{0, 0}, {0, 0}, from, 0, 0, 0};
    if (J && jl.lm) return merge_walk_lm(s_img, re, end_a, from, sp, jl, g);
    if (!J && ctl.lean) return merge_walk_lean(s_img, re, end_a, from, sp);
    return merge_walk_r<J>(s_img, re, end_a, from, sp, jl);
  };
  Res r = merge(entry);
  uint32_t steps0 = r.steps, steps_more = 0, iters = 0;
  // A chain that keeps its offset from the speculative one in every region (records at odd
  // offsets of a run of 2-byte Order records, where every speculative chain is even) changes
  // one lane per pass: 64 passes.  When two passes in a row each changed one lane by the same
  // shift, the lanes above it take that shift too (a guess: the next pass checks it, and
  // every pass still settles its lowest changed lane for good).
  uint32_t shift = 0;
  for (int it = 0; it <= 64; ++it) {
    const uint32_t prev = wave_prev_u32(r.exit);
    uint32_t want = lane == 0 ? e_true : prev;
    bool ch = want != entry;
    const uint64_t cm = __ballot(ch);
    if (!cm) break;
    ++iters;
    const uint32_t low = (uint32_t)__builtin_ctzll(cm);
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)(want - entry), (int)low);
    if ((cm & (cm - 1)) == 0 && d == shift && lane > low) {
      want = entry + d;
      ch = true;
    }
    shift = (cm & (cm - 1)) == 0 ? d : 0u;
    if (ch) {
      entry = want;
      r = merge(want);
      steps_more += r.steps;
    }
  }
  if (ctl.prof) {  // diagnostics: max first-merge steps, max re-merge steps, fix-up passes
    uint32_t m0 = steps0, m1 = steps_more;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      m0 = max(m0, (uint32_t)__shfl_xor(m0, off));
      m1 = max(m1, (uint32_t)__shfl_xor(m1, off));
    }
    if (lane == 0) ctl.prof[(uint64_t)t * 8 + 5] = (uint64_t)m0 | (uint64_t)m1 << 20 | (uint64_t)iters << 40;
  }
  const uint32_t x_true = lane63(r.exit);
  *x_out = x_true;
  // the true chain meets an invalid record (1) or a Serializable one without tables (5):
  // the lowest such lane decides (lanes above it may have run from guessed entries)
  const uint64_t badm = __ballot(r.bad != 0u);
  uint32_t reason = badm ? (__shfl(r.bad, (int)__builtin_ctzll(badm)) == 2u ? 5u : 1u) : 0u;
  if (z.last) {
    if (x_true != end_a) reason = reason ? reason : 2u;  // the last record must end at the span end
  } else if (must_exit != kZCanon && x_true != must_exit) {
    reason = reason ? reason : 3u;  // the successor already entered at the published exit
  }
  if (reason && ctl.dbg) {  // developer diagnostics: the first aborting tile's lane state
    uint32_t claim = 0;
    if (lane == 0) claim = atomicCAS(ctl.dbg, 0u, 1u) == 0u ? 1u : 0u;
    if (__shfl(claim, 0)) {
      if (lane == 0) {
        ctl.dbg[1] = t; ctl.dbg[2] = reason; ctl.dbg[3] = must_exit; ctl.dbg[4] = x_true; ctl.dbg[5] = e_true;
        ctl.dbg[6] = lo; ctl.dbg[7] = z.hi; ctl.dbg[8] = end_a;
      }
      uint32_t* d = ctl.dbg + 24 + 8 * lane;
      d[0] = rs; d[1] = re; d[2] = sp.exit; d[3] = sp.bad; d[4] = sp.first; d[5] = 0; d[6] = entry;
      d[7] = r.exit | r.bad << 31;
    }
  }
  // an invalid record on the true chain with errors kept (ctl.span_err): the tile's counts and
  // bits cover the records before it -- the lanes below the failing one, and its starts before
  // the failing record -- so that a confirmed error costs its span no second decode
  uint32_t fail_a = 0xFFFFFFFFu;
  if (reason == 1u && badm && ctl.span_err) {
    const uint32_t bl = (uint32_t)__builtin_ctzll(badm);
    fail_a = (uint32_t)__shfl((int)r.fail, (int)bl);
    if (lane > bl) {
      r.bm = Bits{0, 0};
      r.wb = Bits{0, 0};
    }
  }
  if (fail_out) *fail_out = fail_a;
  if (reason && reason != 3u && fail_a == 0xFFFFFFFFu) return reason;

  ZPHASE(3);
  // ---- counts and the record-start bitmap for the emit pass
  // one packed sum: a tile holds at most 4096 records, its lanes at most 64 each
  const uint32_t pk = wave_sum_u32(bcount(r.bm) | bcount(r.wb) << 16);
  const uint32_t rec = pk & 0xFFFFu, wide = pk >> 16;
  if (lane == 0) gp(ctl.cnt)[t] = pack_cnt(rec, wide);
  if (cnt_out) *cnt_out = pack_cnt(rec, wide);
  if (bm_out) {
    bm_out[0] = r.bm.lo;
    bm_out[1] = r.bm.hi;
  }
  if (!bm_out) {  // (bm_out: the caller emits from registers -- the small and one-pass decodes)
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    u64x2 out_bits;
    out_bits.x = r.bm.lo;
    out_bits.y = r.bm.hi;
    gp(reinterpret_cast<u64x2*>(ctl.bits))[(uint64_t)t * 64 + lane] = out_bits;
  }
  ZPHASE(4);
#undef ZPHASE
  return reason;
}

// ---------------------------------------------------------------------------------
// Pass 2: exclusive scan of the per-tile counts.  scan1: one 256-thread workgroup per
// 1024 tiles (block-relative bases + the block's total); scan2: one workgroup scans the
// block totals into block offsets.  The emit pass adds the two.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, uint32_t lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(v, off);
    if ((int)lane >= off) v += y;
  }
  return v;
}

__global__ __launch_bounds__(256) void k_decode_scan1(FusedCtl ctl) {
  __shared__ uint64_t s_w[4];
  if (ld_agent32(ctl.abort)) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t nt = ctl.n_tiles, blk = blockIdx.x, i0 = blk * kZScanBlock + tid * 4u;
  uint64_t v[4], sum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = i0 + j < nt ? gp(ctl.cnt)[i0 + j] : 0ull;
    sum += v[j];
  }
  const uint64_t incl = wave_incl_scan(sum, lane);
  if (lane == 63u) s_w[wv] = incl;
  __syncthreads();
  uint64_t run = incl - sum;
  for (uint32_t k = 0; k < wv; ++k) run += s_w[k];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (i0 + j < nt) gp(ctl.base)[i0 + j] = run;
    run += v[j];
  }
  if (tid == 255u) gp(ctl.boff)[blk] = run;  // block total (scan2 turns it into an offset)
}

// 256 threads, 4 block totals each: a 1024-thread workgroup waited up to 60 us for a CU with
// 16 free wave slots while the slice gather (beside the decode) held them.
__global__ __launch_bounds__(256) void k_decode_scan2(FusedCtl ctl, uint32_t n_blocks) {
  __shared__ uint64_t s_w[4];
  if (ld_agent32(ctl.abort)) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6, i0 = 4u * tid;
  uint64_t v[4], sum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = i0 + j < n_blocks ? gp(ctl.boff)[i0 + j] : 0ull;
    sum += v[j];
  }
  const uint64_t incl = wave_incl_scan(sum, lane);
  if (lane == 63u) s_w[wv] = incl;
  __syncthreads();
  uint64_t run = incl - sum;
  for (uint32_t k = 0; k < wv; ++k) run += s_w[k];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (i0 + j < n_blocks) gp(ctl.boff)[i0 + j] = run;
    run += v[j];
  }
}

// Each span's record / wide-record range from the scan (the host reads them before the
// emit pass, so an asynchronous caller knows its record counts while emit still runs).
__global__ __launch_bounds__(256) void k_decode_spans(const SpanDesc* __restrict__ spans, uint32_t n_spans,
                                                      FusedCtl ctl) {
  const uint32_t s = blockIdx.x * 256 + threadIdx.x;
  if (s >= n_spans || ld_agent32(ctl.abort)) return;
  const SpanDesc sd = spans[s];
  if (!sd.n_tiles) return;
  const uint32_t t0 = sd.first_tile, t1 = sd.first_tile + sd.n_tiles - 1;
  gp(ctl.span_lo)[s] = gp(ctl.base)[t0] + gp(ctl.boff)[t0 / kZScanBlock];
  gp(ctl.span_hi)[s] = gp(ctl.base)[t1] + gp(ctl.boff)[t1 / kZScanBlock] + gp(ctl.cnt)[t1];
}

// Pass 2 in one launch (phase 5): scan1's per-block bases, the block offsets by a decoupled
// look-back (a ticket gives each workgroup its block, so it only ever waits for blocks that
// started before it), and the span ranges -- span_hi of every span whose last tile is in the
// block, and, for batches of few spans (ctl.h_res set), also into the host's read-back buffer
// with the abort words, so the host needs no copy after the decode.  Three launches were ~25 us
// between count and emit beside the slice gather, and the read-back copy another ~45 us (its
// blit kernel waits for CU slots too).  Each host write is its own bus transaction, though: for
// config 4's 66 k spans they took 2.5 ms, so many-span batches copy the words back instead.
constexpr uint32_t kLbAgg = 1u, kLbPre = 2u;  // pk_word states: block aggregate, inclusive prefix
__global__ __launch_bounds__(256) void k_decode_scan(const TileDesc* __restrict__ tiles,
                                                     const SpanDesc* __restrict__ spans, uint32_t n_spans,
                                                     FusedCtl ctl) {
  __shared__ uint64_t s_w[4];
  __shared__ uint64_t s_pre;
  __shared__ uint32_t s_blk;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t nt = ctl.n_tiles;
  if (tid == 0) s_blk = atomicAdd(reinterpret_cast<unsigned int*>(ctl.lb), 1u);
  __syncthreads();
  const uint32_t blk = s_blk;
  volatile uint32_t* hab = ctl.h_res ? reinterpret_cast<volatile uint32_t*>(ctl.h_res + 2ull * n_spans) : nullptr;
  if (blk == 0 && hab && tid < kZAbortWords) hab[tid] = ld_agent32(ctl.abort + tid);  // final: count and repair ran
  if (blk == 0 && hab && ctl.jwork && tid < 2u) hab[kZAbortWords + tid] = ld_agent32(ctl.jwork + tid);  // table work used
  if (ld_agent32(ctl.abort)) return;  // (every block: nothing writes it during this kernel)
  const uint32_t i0 = blk * kZScanBlock + tid * 4u;
  uint64_t v[4], sum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = i0 + j < nt ? gp(ctl.cnt)[i0 + j] : 0ull;
    sum += v[j];
  }
  const uint64_t incl = wave_incl_scan(sum, lane);
  if (lane == 63u) s_w[wv] = incl;
  __syncthreads();
  uint64_t run = incl - sum;
  for (uint32_t k = 0; k < wv; ++k) run += s_w[k];
  uint64_t lb_[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lb_[j] = run;
    if (i0 + j < nt) gp(ctl.base)[i0 + j] = run;
    run += v[j];
  }
  if (tid == 0) {
    const uint64_t total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    uint64_t* W = ctl.lb + 1;
    uint64_t pre = 0;
    if (blk == 0) {
      st_agent(&W[0], pk_word(kLbPre, total));
    } else {
      st_agent(&W[blk], pk_word(kLbAgg, total));
      const uint64_t t0 = __builtin_amdgcn_s_memtime();
      for (uint32_t j = blk - 1;;) {
        const uint64_t x = ld_agent(&W[j]);
        const uint32_t st = pk_state(x);
        if (!st) {
          if (__builtin_amdgcn_s_memtime() - t0 > kZSpinLimit) {  // (cannot happen: earlier tickets run)
            raise_abort(ctl, 4, 0u);  // a wait timed out: the batch goes robust
            if (hab) {
              hab[4] = ~0u;
              hab[0] = 1u;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        pre += pk_val(x);
        if (st == kLbPre) break;
        --j;
      }
      if ((ctl.perturb >> 16) && blk == 1) ++pre;  // (test switch: a wrong look-back result; 0 in production)
      st_agent(&W[blk], pk_word(kLbPre, pre + total));
    }
    gp(ctl.boff)[blk] = pre;
    s_pre = pre;
  }
  __syncthreads();
  const uint64_t pre = s_pre;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t t = i0 + j;
    if (t >= nt) break;
    const uint32_t sp = tiles[t].span;
    const SpanDesc sd = spans[sp];
    if (t + 1 == sd.first_tile + sd.n_tiles) {  // the span's last tile
      const uint64_t hi = pre + lb_[j] + v[j];
      gp(ctl.span_hi)[sp] = hi;
      if (ctl.h_res) reinterpret_cast<volatile uint64_t*>(ctl.h_res)[n_spans + sp] = hi;
    }
  }
}

// The look-back above, checked after it (emit, a kernel boundary later: every word final):
// block k's offset must equal block k - 1's final inclusive prefix.  Block 0's offset is 0 and
// each block's total is summed from the counts locally, so when every block k >= 1 passes,
// by induction every offset is the sum of the totals before it -- whatever value a look-back
// poll read.  A mismatch aborts the batch, which the host decodes again (rep[2] counts it;
// emit's stores so far are overwritten then).  One lane of emit's block for tile 1024 k.
__device__ __forceinline__ void lookback_check(const FusedCtl& ctl, uint32_t k) {
  const uint64_t w = ld_agent(ctl.lb + k);  // W[k - 1] (W = lb + 1)
  if (pk_state(w) == kLbPre && pk_val(w) == ld_agent(&ctl.boff[k])) return;
  atomicAdd(ctl.rep + 2, 1u);
  __hip_atomic_store(ctl.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ctl.h_res) {  // (the scan copied the abort words into the host's read-back already)
    volatile uint32_t* hab = reinterpret_cast<volatile uint32_t*>(ctl.h_res + 2ull * ctl.n_spans);
    hab[10] = 1u;
    hab[0] = 1u;
  }
}

// ---------------------------------------------------------------------------------
// Pass 3 for one tile: record starts dropped into LDS by output index (from the bitmap),
// then consecutive lanes decode consecutive records, so each SoA store of the wave is one
// contiguous run.
// ---------------------------------------------------------------------------------
// The count pass's table (step-code map built): the Serializable codes go into the map, and
// the entries stay in LDS as sorted positions and lengths for the true walk's rare lookups
// (a code of 0: a stream longer than the map holds, or an invalid one) -- no bitmap or
// ranks to build.
struct JLPre;
__device__ __forceinline__ JL load_jl_map(const FusedCtl& ctl, uint32_t t, uint32_t* s_j, uint32_t lane, uint32_t* lm,
                                         const JLPre& pre);

// Tile t's entry count and the first 64 entries of its table (one per lane), loaded before
// the tile is staged so that their latency overlaps the staging's (config 3 holds ~50
// entries per tile; load_jl loads any past 64 itself).
struct JLPre {
  uint32_t n, a, L;
};
__device__ __forceinline__ JLPre jl_prefetch(const FusedCtl& ctl, uint32_t t, uint32_t lane) {
  const uint64_t b = (uint64_t)t * kZJCap + lane;  // inside the table even past its entries
  return JLPre{gp(ctl.jn)[t], gp(ctl.jpos)[b], gp(ctl.jlen)[b]};
}
// Entry i of tile t's table: its slot in jpos / jlen (past kZJCap: the overflow arena).
__device__ __forceinline__ uint64_t jslot(const FusedCtl& ctl, uint32_t t, uint32_t i) {
  return i < kZJCap ? (uint64_t)t * kZJCap + i
                    : (uint64_t)ctl.n_tiles * kZJCap + gp(ctl.jbase)[t] + (i - kZJCap);
}
// The overflow entries of tile t (n entries in all) into j.
__device__ __forceinline__ void jl_overflow(const FusedCtl& ctl, uint32_t t, uint32_t n, JL& j) {
  n = __builtin_amdgcn_readfirstlane(n);  // (the same in every lane: the scalar unit branches on it)
  if (n <= kZJCap) return;
  const uint64_t s = jslot(ctl, t, kZJCap);
  j.opos = ctl.jpos + s;
  j.olen = ctl.jlen + s;
  j.on = n - kZJCap;
}
// The count pass walks the map, and looks a Serializable record up only where its code is 0
// (an invalid stream) or 0x80 (longer than kZLmMax): so the LDS list holds just the entries
// longer than kZLmMax -- at most a tile / kZLmMax of them, whatever the tile's entry count --
// in position order (a ballot per 64), and a position not in it reads as invalid.  More than
// kZJCap such entries (overlapping false candidates): abort reason 6, the batch goes robust.
__device__ __forceinline__ JL load_jl_map(const FusedCtl& ctl, uint32_t t, uint32_t* s_j, uint32_t lane, uint32_t* lm,
                                         const JLPre& pre) {
  uint32_t* pos = s_j;
  uint32_t* len = s_j + kZJCap;
  __syncthreads();  // every row of the map is written (build_lm) before codes go over them
  uint32_t kept = 0;
  for (uint32_t i0 = 0; i0 < pre.n; i0 += 64) {
    const uint32_t i = i0 + lane;
    uint32_t a = 0, L = 0;
    if (i < pre.n) {
      const bool p0 = i0 == 0;
      const uint64_t sl = p0 ? 0 : jslot(ctl, t, i);
      a = p0 ? pre.a : gp(ctl.jpos)[sl];
      L = p0 ? pre.L : gp(ctl.jlen)[sl];
      lm8_set(lm, a, lm_code(L <= 0x7FFFFFFFu ? (int)L : 0, true));
    }
    const bool keep = i < pre.n && L <= 0x7FFFFFFFu && L > kZLmMax;
    const uint64_t m = __ballot(keep);
    const uint32_t at = kept + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (keep && at < kZJCap) {
      pos[at] = a;
      len[at] = L;
    }
    kept += (uint32_t)__popcll(m);
  }
  if (kept > kZJCap && lane == 0) raise_abort(ctl, 6, t);
  __syncthreads();  // the map's rows (written before the call) and the codes above
  JL j{nullptr, nullptr, len, lm};
  j.pos = pos;
  j.n = min(kept, kZJCap);
  return j;
}

// Stage tile t's Serializable table into LDS (J passes): bitmap, per-dword ranks, lengths
// (the first kZJCap; the bitmap and ranks cover every entry).
// lm: the count pass's step-code map (built, barrier passed): Serializable codes go into it.
__device__ __forceinline__ JL load_jl(const FusedCtl& ctl, uint32_t t, uint32_t* s_j, uint32_t lane,
                                     uint32_t* lm = nullptr, const JLPre* pre = nullptr) {
  uint32_t* bits = s_j;
  uint32_t* rank = s_j + kZJBitsDw;
  uint32_t* len = s_j + 2 * kZJBitsDw;
  for (uint32_t i = lane; i < kZJBitsDw; i += 64) bits[i] = 0;
  __syncthreads();
  const uint32_t n = pre ? pre->n : gp(ctl.jn)[t];
  for (uint32_t i = lane; i < n; i += 64) {
    const bool p0 = pre && i == lane;
    const uint64_t sl = p0 ? 0 : jslot(ctl, t, i);
    const uint32_t a = p0 ? pre->a : gp(ctl.jpos)[sl];
    const uint32_t L = p0 ? pre->L : gp(ctl.jlen)[sl];
    if (i < kZJCap) len[i] = L;
    atomicOr(&bits[a >> 5], 1u << (a & 31u));
    if (lm) lm8_set(lm, a, lm_code(L <= 0x7FFFFFFFu ? (int)L : 0, true));
  }
  __syncthreads();
  // ranks: lane l takes dwords [5 l, 5 l + 5) (64 x 5 >= 260)
  uint32_t c[5], sum = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t i = 5 * lane + (uint32_t)k;
    c[k] = i < kZJBitsDw ? (uint32_t)__popc(bits[i]) : 0u;
    sum += c[k];
  }
  uint32_t incl = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off);
    if ((int)lane >= off) incl += y;
  }
  uint32_t run = incl - sum;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t i = 5 * lane + (uint32_t)k;
    if (i < kZJBitsDw) rank[i] = run;
    run += c[k];
  }
  __syncthreads();
  JL j{bits, rank, len, lm};
  jl_overflow(ctl, t, n, j);
  return j;
}

// Emit's LDS: the image, record starts of the window by output position and the
// Serializable table.  With Serializable tables (J: the batches with many wide records) the
// entries are 32-bit and, reused in place, also hold the window's wide records (position |
// window index << 16) for a compacted wide pass; without, 16-bit entries and wide records
// decoded inline (same 2 KiB of LDS either way).
// CW: the window's wide records compacted and decoded in a pass of their own (32-bit
// entries); else decoded inline (16-bit entries).  Batches with tables always compact; the
// single-launch small decode compacts too (config 1's window logs hold a TimerTrigger every
// ten records or so, and inline each one took the whole wave through the wide decode).
template <bool J, bool CW = J>
struct EmitLds {
  using PosT = typename std::conditional<CW, uint32_t, uint16_t>::type;
  static constexpr uint32_t kWin = CW ? kZEmitWin : kZWin;
  uint32_t img[kZImgDw];
  PosT pos[kWin];
  uint32_t j[J ? 2 * kZJBitsDw + kZJCap : 1];
};

// Pass 3 for tile t whose first record is record `base` of the batch (wide<<31 | records).
template <bool J, bool CW = J>
__device__ __forceinline__ void emit_tile(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                          const FusedCtl& ctl, const DecodeOut& out, const uint32_t t,
                                          const uint32_t lane, const uint64_t base, EmitLds<J, CW>& L,
                                          const uint64_t* bm_in = nullptr) {
  using PosT = typename EmitLds<J, CW>::PosT;
  constexpr uint32_t kWin = EmitLds<J, CW>::kWin;
  uint32_t* const s_img = L.img;
  PosT* const s_pos = L.pos;
  uint32_t* const s_j = L.j;
  const TileDesc td = tiles[t];
  const TileDesc n1 = tiles[t + 1 < ctl.n_tiles ? t + 1 : t];  // halo source, loaded beside td
  const SpanDesc sd = spans[td.span];
  const uint32_t lo = td.delta, hi = td.delta + td.len;
  const uint64_t ea = sd.len - td.span_off + td.delta;
  const uint32_t end_a = ea > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)ea;
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  // bm_in: the lane's bitmap words straight from the count, the image still staged in L.img
  // (the single-launch small decode and the one pass); else both from memory
  u64x2 bits = bm_in ? u64x2{bm_in[0], bm_in[1]} : gp(reinterpret_cast<const u64x2*>(ctl.bits))[(uint64_t)t * 64 + lane];
  if (lane * kZRegion >= hi) bits = u64x2{0, 0};  // past the tile (the lane path of small spans skips them)
  JLPre pre{};
  if (J) pre = jl_prefetch(ctl, t, lane);
  if (!bm_in) stage_image(td, sd, t, tiles, s_img, lane, hi, &n1);
  JL jl{nullptr, nullptr, nullptr};
  if (J) jl = load_jl(ctl, t, s_j, lane, nullptr, &pre);
  const uint32_t r0 = lane * kZRegion;
  const uint32_t cnt = (uint32_t)(__popcll(bits.x) + __popcll(bits.y));
  const uint32_t incl = wave_scan_u32(cnt, lane);
  const uint32_t total = lane63(incl);
  const uint64_t rec0 = base & ((1ull << 31) - 1), wide0 = base >> 31;
  // wave-uniform output bases (scalar registers; per-lane 32-bit offsets) and one capacity
  // test per tile instead of one per record
  const uint64_t rec0u = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)rec0) |
                         (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(rec0 >> 32)) << 32;
  auto* const o_off = gp(out.off) + rec0u;
  auto* const o_tag = gp(out.tag) + rec0u;
  auto* const o_v0 = gp(out.v0) + rec0u;
  const bool fits = rec0u + total <= out.cap;
  Bits cur{bits.x, bits.y};
  uint32_t idx = incl - cnt;
  uint64_t wide = wide0;
  for (uint32_t w0 = 0; w0 < total; w0 += kWin) {
    const uint32_t wend = w0 + kWin;
    // the lane's record starts into s_pos in order: the low 64 region bytes, then the high
    // 64 (one 64-bit word per loop: no per-start choice between the halves)
    while (cur.lo && idx < wend) {
      s_pos[idx - w0] = (PosT)(r0 + (uint32_t)__builtin_ctzll(cur.lo));
      cur.lo &= cur.lo - 1;
      ++idx;
    }
    while (!cur.lo && cur.hi && idx < wend) {
      s_pos[idx - w0] = (PosT)(r0 + 64u + (uint32_t)__builtin_ctzll(cur.hi));
      cur.hi &= cur.hi - 1;
      ++idx;
    }
    __syncthreads();
    const uint32_t nw = total - w0 < kWin ? total - w0 : kWin;
    uint32_t nwide = 0;  // wide records of the window so far (wave-uniform)
    // two records per lane per pass, both loaded before either is decoded: the positions' and
    // image reads of the second overlap the first's (a wave alone on its SIMD -- the
    // single-launch small decode -- waits on every read otherwise)
    for (uint32_t i0 = 0; i0 < nw; i0 += 64u * kZEmitPair) {
      uint32_t a2[kZEmitPair], dd[kZEmitPair][4];
#pragma unroll
      for (int h = 0; h < kZEmitPair; ++h) {
        const uint32_t i = i0 + 64u * h + lane;
        a2[h] = i < nw ? s_pos[i] : lo;
      }
#pragma unroll
      for (int h = 0; h < kZEmitPair; ++h) {
        const uint32_t kk = rk(a2[h] >> 2);
#pragma unroll
        for (int q = 0; q < 4; ++q) dd[h][q] = s_img[kk + q];
      }
#pragma unroll
      for (int h = 0; h < kZEmitPair; ++h) {
        const uint32_t i = i0 + 64u * h + lane;
        const bool act = i < nw;
        const uint32_t a = a2[h], sh = 8u * (a & 3u);
        const uint32_t d0 = dd[h][0], d1 = dd[h][1], d2 = dd[h][2], d3 = dd[h][3];
        const uint32_t x0 = __builtin_amdgcn_alignbit(d1, d0, sh);
        const uint32_t x1 = __builtin_amdgcn_alignbit(d2, d1, sh);
        const uint32_t x2 = __builtin_amdgcn_alignbit(d3, d2, sh);
        uint32_t tg = x0 & 0xFFu;
        const uint32_t blo = (x0 >> 8) | (x1 << 24), bhi = (x1 >> 8) | (x2 << 24);  // bytes a+1..a+8 (LE)
        // v0 without branches: Order's channel byte, Timestamp's big-endian i64, else (RNG,
        // BufferBuilt) a big-endian i32; wide records get theirs in the wide pass
        const bool is_ts = tg == CLG_TAG_TIMESTAMP;
        const uint32_t be32 = __builtin_bswap32(blo);
        const uint32_t v_lo = is_ts ? __builtin_bswap32(bhi)
                                    : (tg == CLG_TAG_ORDER ? (uint32_t)(int32_t)(int8_t)(blo & 0xFFu) : be32);
        const uint32_t v_hi = is_ts ? be32 : (uint32_t)((int32_t)v_lo >> 31);
        const int64_t v0 = (int64_t)((uint64_t)v_hi << 32 | v_lo);
        const bool wide_rec = act && is_wide((int)tg);
        const uint64_t wm = __ballot(wide_rec);
        if constexpr (CW) {
          if (act) {
            const uint32_t so = (uint32_t)(td.span_off + (a - lo));
            if (fits || rec0 + w0 + i < out.cap) {
              const uint32_t j = w0 + i;
              o_off[j] = so;
              o_tag[j] = (uint8_t)tg;
              if (!wide_rec) o_v0[j] = v0;
            }
            // compaction in place: every entry below i0 + 64 kZEmitPair has been read already
            if (wide_rec) s_pos[nwide + (uint32_t)__popcll(wm & ((1ull << lane) - 1ull))] = a | i << 16;
          }
          nwide += (uint32_t)__popcll(wm);
        } else {
          Rec rr{};
          int64_t v = v0;
          if (wide_rec) {
            uint32_t tgu;
            const int L = zlen(s_img, a, end_a, &tgu);
            decode_fields(ZBytes{s_img, a}, (int)tg, (int64_t)L, rr);
            v = rr.v0;
          }
          if (act) {
            const uint32_t so = (uint32_t)(td.span_off + (a - lo));
            const uint64_t g = rec0 + w0 + i;
            if (fits || g < out.cap) {
              const uint32_t j = w0 + i;
              o_off[j] = so;
              o_tag[j] = (uint8_t)tg;
              o_v0[j] = v;
            }
            if (wide_rec) {
              const uint64_t wi = wide + (uint64_t)__popcll(wm & ((1ull << lane) - 1ull));
              if (wi < out.wcap) {
                gp(out.w_idx)[wi] = (uint32_t)g;
                gp(out.w_rc)[wi] = rr.rc;
                gp(out.w_v1)[wi] = rr.v1;
                gp(out.w_var_off)[wi] = rr.var_off ? so + rr.var_off : 0u;
                gp(out.w_var_len)[wi] = rr.var_len;
                gp(out.w_sub)[wi] = rr.sub;
              }
            }
          }
          wide += (uint64_t)__popcll(wm);
        }
      }
    }
    __syncthreads();
    // the window's wide records, 64 at a time: field decoding and side-table rows run with
    // every lane busy instead of inside the record loop's divergent branch
    for (uint32_t k0 = 0; CW && k0 < nwide; k0 += 64) {
      const uint32_t k = k0 + lane;
      if (k < nwide) {
        const uint32_t e = s_pos[k], a = e & 0xFFFFu, i = e >> 16;
        const uint64_t g = rec0 + w0 + i;
        // Branch-free over the four wide tags (the count pass validated every record, so
        // the lengths need no checks): the record's bytes a .. a+31 as eight little-endian
        // dwords x[j] = bytes a+4j .. a+4j+3 from nine LDS reads, every field taken from
        // them, the values selected by tag -- decode_fields' rules (dev_common.h;
        // SimpleDeterminantEncoder.java:202-341).
        const uint32_t k0 = a >> 2, sh = 8u * (a & 3u);
        uint32_t d[9], x[8];
#pragma unroll
        for (uint32_t j = 0; j < 9; ++j) d[j] = s_img[rk(k0 + j)];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) x[j] = __builtin_amdgcn_alignbit(d[j + 1], d[j], sh);
        auto be32 = [&](uint32_t off) {  // bytes a+off .. a+off+3, big-endian (off constant)
          return __builtin_bswap32(__builtin_amdgcn_alignbyte(x[(off >> 2) + 1], x[off >> 2], off & 3u));
        };
        const uint32_t tg = x[0] & 0xFFu;
        const bool ser = tg == CLG_TAG_SERIALIZABLE, tt = tg == CLG_TAG_TIMER_TRIGGER, sc = tg == CLG_TAG_SOURCE_CHECKPOINT;
        const uint32_t b13 = (x[3] >> 8) & 0xFFu, b21 = (x[5] >> 8) & 0xFFu, b22 = (x[5] >> 16) & 0xFFu;
        const bool tt_name = tt && b13 == 6u, sc_ref = sc && b22 != 0u;
        const uint32_t jlen = J && ser ? jl_len_bits(jl, a) : 0u;  // (without tables no Serializable record gets here)
        const uint32_t L = ser ? jlen : tt_name ? 18u + be32(14) : tt ? 14u : sc_ref ? 27u + be32(23) : sc ? 23u : 13u;
        const uint32_t var_off = ser ? 1u : tt_name ? 18u : sc_ref ? 27u : 0u;
        const int64_t v0 = ser ? (int64_t)L - 1 : (int64_t)((uint64_t)be32(5) << 32 | be32(9));
        if (fits || g < out.cap) o_v0[w0 + i] = v0;
        const uint64_t wi = wide + k;
        if (wi < out.wcap) {
          const uint32_t so = (uint32_t)(td.span_off + (a - lo));
          gp(out.w_idx)[wi] = (uint32_t)g;
          gp(out.w_rc)[wi] = ser ? 0 : (int32_t)be32(1);
          gp(out.w_v1)[wi] = sc ? (int64_t)((uint64_t)be32(13) << 32 | be32(17)) : 0;
          gp(out.w_var_off)[wi] = var_off ? so + var_off : 0u;
          gp(out.w_var_len)[wi] = var_off ? L - var_off : 0u;
          gp(out.w_sub)[wi] = (uint8_t)(tt ? b13 : sc ? (b21 | (sc_ref ? 0x80u : 0u)) : 0u);
        }
      }
    }
    wide += nwide;
    __syncthreads();
  }
}

template <bool J>
__global__ __launch_bounds__(64) void k_decode_emit(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                    FusedCtl ctl, DecodeOut out) {
  __shared__ EmitLds<J> L;
  const uint32_t t = blockIdx.x, lane = threadIdx.x;
  if (ld_agent32(ctl.abort)) return;  // (then the scan returned before its look-back too)
  if (ctl.lb_check && t && t % kZScanBlock == 0 && lane == 0) lookback_check(ctl, t / kZScanBlock);
  if (ctl.skip_bad && gp(ctl.span_bad)[tiles[t].span]) return;  // the robust output fills this span
  if (ctl.span_err && tiles[t].span_off > gp(ctl.span_err)[tiles[t].span]) return;  // past a kept error
  emit_tile<J>(tiles, spans, ctl, out, t, lane, gp(ctl.base)[t] + gp(ctl.boff)[t / kZScanBlock], L);
}

// Pass 0 (batches holding them): small whole spans, a lane each.  A batch of many small logs
// (config 4: 65 536 subpartition logs of 320 bytes) gives one tile per span, and a wave spent
// on a 320-byte tile costs as much as one on 8 KiB.  Lane i of block b takes tile 64 b + i
// when it is a whole span of at most kZTiny bytes and walks the span alone from HBM through a
// 16-byte window: fixed-length records only (Order, Timestamp, RNG, BufferBuilt,
// IgnoreCheckpoint -- lengths need no field), with the reference's bounds.  It writes the
// tile's count and record-start bitmap words (emit reads the words of the regions the tile
// reaches) and marks the tile done in st_x (unused for a whole-span tile: no successor
// enters at its exit), so the count pass skips it.  A TimerTrigger / SourceCheckpoint /
// Serializable record leaves the tile to the count pass; an invalid record marks the span
// bad (abort reason 1), as count_tile does.  A separate kernel: inside the count kernel the
// walk's registers cost the wave path 16 VGPRs and an occupancy step.
constexpr uint64_t kZTinyDone = 1ull << 62;  // st_x word of a tile pass 0 counted
__device__ __forceinline__ bool tiny_tile(const TileDesc& td, const SpanDesc& sd) {
  return sd.n_tiles == 1 && td.span_off == 0 && td.len > 0 && td.len <= kZTiny && td.len == sd.len;
}
__global__ __launch_bounds__(64) void k_decode_count_tiny(const TileDesc* __restrict__ tiles,
                                                          const SpanDesc* __restrict__ spans, FusedCtl ctl) {
  const uint32_t ti = blockIdx.x * 64 + threadIdx.x;
  if (ti >= ctl.n_tiles) return;
  const TileDesc td = tiles[ti];
  if (!tiny_tile(td, spans[td.span]) || (ctl.skip_bad && gp(ctl.span_bad)[td.span])) return;
  // 0 ok, 1 invalid record (a bad tag or a record past the span end), 3 a tag this path leaves
  uint32_t why = 0, rec = 0, wide = 0;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  const CLG_GLOBAL u32x4* src = gp(reinterpret_cast<const u32x4*>(td.abase));
  auto* bits = gp(reinterpret_cast<u64x2*>(ctl.bits)) + (uint64_t)ti * 64;
  const uint32_t end = td.delta + td.len;
  uint32_t a = td.delta, wb = 0xFFFFFFFFu, cur = 0;
  u32x4 w{};
  uint64_t blo = 0, bhi = 0;
  constexpr uint32_t kLut = 2u | 9u << 4 | 5u << 8 | 13u << 24 | 5u << 28;  // fixed lengths (0: fields)
  while (a < end) {
    if ((a >> 4) != wb) {  // the 16-byte window holding the tag
      wb = a >> 4;
      w = src[wb];
    }
    const uint32_t q = a & 15u;
    const uint32_t dw = q < 8u ? (q < 4u ? w.x : w.y) : (q < 12u ? w.z : w.w);
    const uint32_t tg = (dw >> (8u * (q & 3u))) & 0xFFu;
    const uint32_t L = tg < 8u ? (kLut >> (4u * tg)) & 0xFu : 0u;
    if (!L) {
      why = (tg == CLG_TAG_SERIALIZABLE || tg == CLG_TAG_TIMER_TRIGGER || tg == CLG_TAG_SOURCE_CHECKPOINT) ? 3u : 1u;
      break;
    }
    if (a + L > end) {  // (the true chain's bound: an invalid record, count_tile's reason 1)
      why = 1u;
      break;
    }
    for (const uint32_t r = a >> 7; cur < r; ++cur) {  // the regions before this start are complete
      u64x2 v;
      v.x = blo;
      v.y = bhi;
      bits[cur] = v;
      blo = bhi = 0;
    }
    const uint32_t i = a & 127u;
    if (i < 64u) blo |= 1ull << i; else bhi |= 1ull << (i - 64u);
    ++rec;
    wide += tg == CLG_TAG_IGNORE_CHECKPOINT ? 1u : 0u;
    a += L;
  }
  if (why == 3u) return;  // the count pass takes this tile (its words are rewritten there)
  if (why == 0u || ctl.span_err) {  // (an invalid record with errors kept: the records before it)
    for (const uint32_t r = (end - 1) >> 7; cur <= r; ++cur) {
      u64x2 v;
      v.x = blo;
      v.y = bhi;
      bits[cur] = v;
      blo = bhi = 0;
    }
    gp(ctl.cnt)[ti] = pack_cnt(rec, wide);
  }
  if (why) {
    raise_abort(ctl, why, ti);
    if (ctl.span_bad) __hip_atomic_store(ctl.span_bad + td.span, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    note_error(ctl, td.span, (uint64_t)(a - td.delta));  // (a whole span: span offset = a - delta)
  }
  gp(ctl.st_x)[ti] = kZTinyDone;
}

// Chunk-boundary repair.  A chunk enters at its predecessor's published canonical exit.
// Where the predecessor's true exit differs (a record the canonical walk cannot measure --
// longer than a tile, or a chunk's last tile lying wholly inside one -- crosses the chunk
// end), or where a chain from a published entry goes wrong, the block records a request
// instead of failing the span.  k_decode_repair then serves the requests in chunk order:
// from the true exit of the tile before the chunk it counts tiles again until the new
// chain's exit equals the old chain's (from there on the two agree), the span ends, or the
// chain fails (then the span is bad, for real).  Then any tile of that chunk's first span
// still without an exit failed on the true chain: its span is bad.
constexpr uint64_t kZExValid = 1ull << 63;  // ex[t]: the tile's exit (span offset) is known
constexpr uint64_t kZExFail = 1ull << 62;   // ex[t] (not valid): its chain met an invalid record at span offset ex & ~flag

// A request: chunk c's flag (idempotent, so a chunk asked for twice is served once) and the
// request count, which lets k_decode_repair return at once in the usual batch.
__device__ __forceinline__ void push_repair(const FusedCtl& ctl, uint32_t c) {
  gp(ctl.rep_flag)[c] = 1u;
  atomicAdd(ctl.rep + 1, 1u);
}
__device__ __forceinline__ void mark_bad(const FusedCtl& ctl, uint32_t reason, uint32_t t, uint32_t span) {
  raise_abort(ctl, reason, t);
  if (ctl.span_bad) __hip_atomic_store(ctl.span_bad + span, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// First tile of chunk c of the count pass's G chunks (c = G: n_tiles).
__device__ __forceinline__ uint32_t chunk_first(const FusedCtl& ctl, uint32_t c, uint32_t K, uint32_t G) {
  if (c >= G) return ctl.n_tiles;
  return ctl.chunk ? ctl.chunk[c] : min(ctl.n_tiles, c * K);
}
// After chunk c's request: a tile of its first span without an exit failed for real.
__device__ __forceinline__ void check_chunk(const FusedCtl& ctl, const TileDesc* __restrict__ tiles, uint32_t f,
                                            uint32_t ce, uint32_t lane) {
  const uint32_t span = tiles[f].span;
  uint32_t bad = 0xFFFFFFFFu;
  for (uint32_t i = f + lane; i < ce; i += 64) {
    if (tiles[i].span != span) break;
    if (!(ld_agent(&ctl.ex[i]) & kZExValid)) {
      bad = i;
      break;
    }
  }
  const uint64_t m = __ballot(bad != 0xFFFFFFFFu);
  if (m && lane == (uint32_t)__builtin_ctzll(m)) {
    mark_bad(ctl, 1, bad, span);
    // the chain that failed there is the true one (the repair walk met it before): its position
    const uint64_t e = ld_agent(&ctl.ex[bad]);
    if (e & kZExFail) note_error(ctl, span, e & ~kZExFail);
  }
}

// Tile t staged (image, and with tables the map and table) and counted from entry xs (span
// offset); *x = its exit (span offset).  count_tile's reason.
template <bool J>
__device__ __forceinline__ uint32_t count_staged(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                 const FusedCtl& ctl, uint32_t* s_img, uint32_t* s_j, uint32_t lane,
                                                 uint32_t t, const ZTile& z, uint64_t xs, uint32_t must_exit,
                                                 const SpecR* walked, uint64_t* x, uint64_t* cnt_out = nullptr,
                                                 uint64_t* bm_out = nullptr, uint64_t* fail_so = nullptr) {
  const uint32_t nt = ctl.n_tiles;
  const TileDesc n1 = tiles[t + 1 < nt ? t + 1 : t];
  const uint64_t ee = xs - z.td.span_off + z.lo;
  const uint32_t e_true = ee > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)ee;
  JL jl{nullptr, nullptr, nullptr};
  JLPre pre{};
  if (J) pre = jl_prefetch(ctl, t, lane);
  // (the next tile's loads issued during this walk were slower: config-2 count 0.185 against
  // 0.175 ms, 127 VGPRs; round 4)
  stage_image(z.td, z.sd, t, tiles, s_img, lane, z.hi, &n1);
  if (J) build_lm(z, s_img, s_j, lane);  // the image becomes the step-code map
  if (J) jl = load_jl_map(ctl, t, s_j, lane, s_img, pre);
  uint32_t x_true, fa = 0xFFFFFFFFu;
  const uint32_t why = count_tile<J>(t, z, e_true, must_exit, ctl, s_img, lane, &x_true, jl, tiles, walked, cnt_out,
                                     bm_out, fail_so ? &fa : nullptr);
  *x = z.td.span_off + (x_true - z.lo);
  if (fail_so) *fail_so = fa != 0xFFFFFFFFu ? z.td.span_off + (fa - z.lo) : ~0ull;
  return why;
}

// Tiles a repair walk may find where the old chain had an exit too, a different one.  Past
// that the two are taken to be chains that never meet -- a run of channel-0 Order records
// ("00 00") at odd offsets, where every chunk entered on the even chain -- and the span goes
// to the robust pipeline instead of a walk to its end (one wave counts about a tile per 50 us
// with nothing to hide its latencies).  Tiles where the old chain had failed (entered inside
// a long record) do not count: a run of long records a short gap apart needs a long walk.
constexpr uint32_t kZWalkDisagree = 4;

// A tile (not its span's last) whose bytes are all zero, entered at span offset xs: a run of
// Order records of channel 0 ("00 00", SimpleDeterminantEncoder.java:120-121, any channel byte
// is valid), the reference's output while one input channel carries every buffer
// (CausalBufferOrderService.java:112).  Its records start at xs, xs + 2, ... below the tile end,
// so its counts, start bitmap and exit follow without a walk -- the repair walk crosses long
// runs, where the published chain has the other parity in every tile, at one load per tile.
// Returns false (nothing written) unless every loaded byte is zero.
__device__ __forceinline__ bool zero_tile_walk(const ZTile& z, uint64_t xs, const FusedCtl& ctl, uint32_t t,
                                               uint32_t lane, uint64_t* x) {
  const uint32_t words = (z.hi + 15) >> 4;
  const CLG_GLOBAL u32x4* src = gp(reinterpret_cast<const u32x4*>(z.td.abase));
  uint32_t any = 0;
#pragma unroll
  for (int i = 0; i < kZLoads; ++i) {
    const uint32_t w = lane + 64u * (uint32_t)i;
    const u32x4 v = src[w < words ? w : words - 1u];
    any |= v.x | v.y | v.z | v.w;
  }
  if (__any(any != 0u)) return false;
  const uint32_t e = (uint32_t)(xs - z.td.span_off) + z.lo;  // aligned coordinate of the entry, < hi
  const uint32_t n = (z.hi - e + 1u) >> 1;                  // starts e, e + 2, ... < hi
  const uint32_t r0 = lane * kZRegion;
  const uint64_t pat = (e & 1u) ? 0xAAAAAAAAAAAAAAAAull : 0x5555555555555555ull;
  auto word = [&](uint32_t b0) -> uint64_t {  // starts among positions b0 .. b0 + 63
    uint64_t m = pat;
    if (e > b0) m = e - b0 >= 64u ? 0ull : m & (~0ull << (e - b0));
    if (z.hi < b0 + 64u) m = z.hi <= b0 ? 0ull : m & ((1ull << (z.hi - b0)) - 1ull);
    return m;
  };
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  u64x2 bits;
  bits.x = word(r0);
  bits.y = word(r0 + 64u);
  gp(reinterpret_cast<u64x2*>(ctl.bits))[(uint64_t)t * 64 + lane] = bits;
  if (lane == 0) gp(ctl.cnt)[t] = pack_cnt(n, 0);
  *x = z.td.span_off + (e + 2u * n - z.lo);
  return true;
}

// Whether chunk c (first tile f) entered at a published exit other than the true exit of the
// tile before it.  Read after the count pass (a kernel boundary), from the words the count
// pass stored: the entry the chunk actually took (ent[c]) and the tile before's exit (ex[f-1];
// not valid: that tile failed, and its span is the chunk's first).  Independent of how the
// count pass's poll of st_x went.
__device__ __forceinline__ bool wrong_entry(const FusedCtl& ctl, uint32_t c, uint32_t f) {
  const uint64_t e = ld_agent(&ctl.ent[c]);
  if (!pk_state(e) || f == 0) return false;  // (the chunk started its span, or never counted)
  const uint64_t xe = ld_agent(&ctl.ex[f - 1]);
  return !(xe & kZExValid) || (xe & ~kZExValid) != pk_val(e);
}

// Chunk c's request (k_decode_repair).  *walk_end: past the last tile a walk reached.
template <bool J>
__device__ __forceinline__ void serve_chunk(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                            const FusedCtl& ctl, uint32_t* s_img, uint32_t* s_j, uint32_t lane,
                                            uint32_t c, uint32_t f, uint32_t ce, uint32_t* walk_end) {
  if (f == 0 || f >= ce || tiles[f].span_off == 0) return;  // the chunk starts its span
  if (f >= *walk_end) {  // (else a walk has rewritten this chunk's entry already)
    const uint64_t xe = ld_agent(&ctl.ex[f - 1]);
    if (!(xe & kZExValid)) {  // the tile before failed: its span (this chunk's first) is bad
      if (lane == 0) mark_bad(ctl, 1, f - 1, tiles[f].span);
      return;
    }
    uint64_t xs = xe & ~kZExValid;
    // the entry the chunk took (or, never stored, the published exit it would have taken)
    const uint64_t e = ld_agent(&ctl.ent[c]);
    const uint64_t taken = pk_state(e) ? pk_val(e) : pk_val(ld_agent(&ctl.st_x[f - 1]));
    if (xs != taken) {  // entered elsewhere: walk from the true exit
      uint32_t disagree = 0;
      for (uint32_t t = f; t < ctl.n_tiles; ++t) {
        const ZTile z = ztile(tiles, spans, t, lane);
        *walk_end = t + 1;
        uint64_t x = xs, fso = ~0ull;
        uint32_t why = 0;
        bool zero = false;
        if (!z.last && xs >= z.td.span_off + z.td.len) {  // wholly inside a record: no starts
          typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
          gp(reinterpret_cast<u64x2*>(ctl.bits))[(uint64_t)t * 64 + lane] = u64x2{0, 0};
          if (lane == 0) gp(ctl.cnt)[t] = 0;
        } else if (!z.last && zero_tile_walk(z, xs, ctl, t, lane, &x)) {
          zero = true;  // a run of Order(channel 0) records: settled without a walk
        } else {
          why = count_staged<J>(tiles, spans, ctl, s_img, s_j, lane, t, z, xs, kZCanon, nullptr, &x, nullptr, nullptr,
                                &fso);
          __syncthreads();  // the image is reused
          if (why == 1u && lane == 0) note_error(ctl, z.td.span, fso);  // (the walk's entry is the true one)
        }
        if (why) {
          if (lane == 0) {
            mark_bad(ctl, why, t, z.td.span);
            // the tile's word: this chain's failure, not the count pass's from another entry
            // (a later chunk check of this tile must not take that one for real)
            st_agent(&ctl.ex[t], why == 1u && fso != ~0ull ? kZExFail | fso : 0ull);
          }
          break;
        }
        const uint64_t xv = kZExValid | x;
        uint32_t old = 0;
        if (lane == 0) {
          const uint64_t o = ld_agent(&ctl.ex[t]);
          old = o == xv ? 1u : (o & kZExValid) ? 2u : 0u;  // 1 the same, 2 another exit, 0 none
          st_agent(&ctl.ex[t], xv);
          if (ctl.dbg) {  // developer diagnostics (CLONOS_FUSED_DEBUG): who wrote ex[t], from which entry
            uint64_t* w = reinterpret_cast<uint64_t*>(ctl.dbg + kZDbgTiles) + 2 * (uint64_t)t;
            w[0] = xs;
            w[1] = 2ull << 60 | (uint64_t)blockIdx.x << 32 | (uint64_t)(f & 0xFFFFFF) << 4 | old;
          }
        }
        old = __shfl(old, 0);
        if (old == 1u || z.last) break;  // resynchronised, or the span ends
        if (old == 2u && !zero && ++disagree > kZWalkDisagree) {  // chains that do not meet: the span goes robust
          if (lane == 0) {
            mark_bad(ctl, 3, t, z.td.span);
            if (ctl.dbg) {  // developer diagnostics (CLONOS_FUSED_DEBUG): the walk that gave up
              ctl.dbg[9] = 0xD15A; ctl.dbg[10] = f; ctl.dbg[11] = t; ctl.dbg[12] = (uint32_t)(xs - z.td.span_off);
              ctl.dbg[13] = (uint32_t)(x - z.td.span_off); ctl.dbg[14] = z.td.span; ctl.dbg[15] = disagree;
            }
          }
          break;
        }
        xs = x;
      }
    }
  }
  check_chunk(ctl, tiles, f, ce, lane);  // its failures past the walk are real
}

// Pass 1 kernel.  Persistent grid (at most what the device keeps resident, see
// launch_decode_fused); block b decodes the chunk of tiles [chunk[b], chunk[b + 1]).
// Inside a chunk a tile's entry is its predecessor's true exit.  Across chunks: each block
// first publishes the canonical exit of its chunk's last tile (no waiting before that),
// and a chunk's first tile enters at the previous chunk's published exit, which that
// chunk's last tile then checks (a mismatch: a repair request, above).  Blocks are all
// resident and publish first, so the one wait always ends; a wait past kZSpinLimit cycles
// aborts the batch instead.
// 128 VGPRs (4 waves per SIMD by registers, 3.25 by LDS with tables): count<J> 0.396 to
// 0.376 ms on the config-3 subset, count<false> (88 VGPRs) unaffected.  The same bound on
// k_decode_jser made it slower (0.26 to 0.28 ms), so that kernel keeps its 150.
// Waves per SIMD the count kernel is compiled for (its VGPR bound): 4 (128 VGPRs), except with
// tables, where 128 VGPRs spilled into the walks (config-3 count +60 %) -- 3.
template <bool J>
constexpr int kZCountWaves = J ? 3 : 4;
template <bool J>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kZCountWaves<J>))) void k_decode_count(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                     FusedCtl ctl) {
  __shared__ uint32_t s_img[kZImgDw];
  __shared__ uint32_t s_j[J ? 2 * kZJBitsDw + kZJCap : 1];
  const uint32_t lane = threadIdx.x, nt = ctl.n_tiles;
  JL jl{nullptr, nullptr, nullptr};
  const uint32_t K = (nt + gridDim.x - 1) / gridDim.x;
  const uint32_t t0 = chunk_first(ctl, blockIdx.x, K, gridDim.x), t1 = chunk_first(ctl, blockIdx.x + 1, K, gridDim.x);
  // the chunk's last tile: publish its canonical exit (span offset) for the next chunk
  uint32_t x_pub = kZCanon;
  SpecR sp_last{{0, 0}, {0, 0}, 0, 0, 0};  // its speculative walk, reused when the loop reaches it
  if (t0 < t1) {
    const ZTile z = ztile(tiles, spans, t1 - 1, lane);
    if (!z.last && t1 < nt) {
      stage_image(z.td, z.sd, t1 - 1, tiles, s_img, lane, z.hi);
      if (J) build_lm(z, s_img, s_j, lane);  // the image becomes the step-code map
      if (J) jl = load_jl_map(ctl, t1 - 1, s_j, lane, s_img, jl_prefetch(ctl, t1 - 1, lane));
      const uint32_t ws = warm_start(z.rs, z.lo, ctl.warm, lane);
      const uint32_t wsb = warm_start(lane * kZRegion + 64u, z.lo, ctl.warm, lane);
      sp_last = z.rs < z.re ? spec_walk_fast<J>(s_img, ws, wsb, z.rs, z.re, z.end_a, lane * kZRegion, jl, ctl.lean != 0u)
                            : SpecR{{0, 0}, {0, 0}, z.rs, z.rs, 0};
      x_pub = canon_exit_r<J>(z, s_img, sp_last, lane, jl, tiles, t1 - 1);
      // An exit is the first record start at or past the tile end.  One before it is a fault
      // of the canonical walk: publish the tile end instead (a guess; this chunk's last tile
      // checks it against its true exit and files a repair when they differ), and count it.
      if (x_pub < z.hi) {
        if (lane == 0) atomicAdd(ctl.rep + 3, 1u);
        x_pub = z.hi;
      }
      // (64-bit: the exit's span offset, never wrapped)
      if (lane == 0) st_agent(&ctl.st_x[t1 - 1], pk_word(2u, (uint64_t)z.td.span_off + (x_pub - z.lo)));
      __syncthreads();
    }
  }
  uint64_t x_prev = 0;  // previous tile's exit, span offset
  uint32_t bad_span = 0xFFFFFFFFu;  // a span whose chain went wrong: its later tiles are skipped
  uint32_t sus_span = 0xFFFFFFFFu;  // the chunk's first span, entered at a published exit
  for (uint32_t t = t0; t < t1; ++t) {
    const ZTile z = ztile(tiles, spans, t, lane);
    if (z.td.span == bad_span) continue;  // (wave-uniform) the host decodes that span robustly
    if (!J && ctl.tiny && z.first && z.last && z.td.len <= kZTiny && gp(ctl.st_x)[t] == kZTinyDone)
      continue;  // (wave-uniform) pass 0 counted this small whole span
    if (ctl.prof && lane == 0) ctl.prof[(uint64_t)t * 8] = __builtin_amdgcn_s_memtime();
    uint64_t xs;
    if (z.first) {
      xs = z.td.span_off;  // a span starts on a record boundary
    } else if (t > t0) {
      xs = x_prev;
    } else {  // chunk start: the previous chunk's published exit
      uint64_t v;
      uint32_t nb = 1;
      const uint64_t w0 = __builtin_amdgcn_s_memtime();
      for (;;) {
        v = ld_agent(&ctl.st_x[t - 1]);
        // published, and not before this tile: an exit of the tile before lies in this one or
        // later.  A chunk once entered at span offset 0 from a word read as published (about 1
        // batch in 30 on config 2; the word held the right exit afterwards): such a read is
        // not taken, the poll goes on
        if (pk_state(v) && pk_val(v) >= z.td.span_off) break;
        if (pk_state(v) && ctl.dbg && lane == 0) {  // developer diagnostics: the reads not taken
          if (atomicAdd(ctl.dbg + 16, 1u) == 0u) {
            ctl.dbg[17] = t; ctl.dbg[18] = (uint32_t)v; ctl.dbg[19] = (uint32_t)(v >> 32);
            ctl.dbg[20] = (uint32_t)z.td.span_off; ctl.dbg[21] = nb;
          }
        }
        if (ld_agent32(ctl.abort + 4)) return;  // another wait timed out: the batch goes robust
        if (!backoff(nb, w0)) {
          if (lane == 0) raise_abort(ctl, 4, t);
          return;
        }
      }
      xs = pk_val(v) + (ctl.perturb & 0xFFFFu);  // (perturb: a test switch, 0 in production)
      sus_span = z.td.span;
      // the entry taken, for k_decode_repair's check against the true exit before it
      if (lane == 0) st_agent(&ctl.ent[blockIdx.x], pk_word(2u, xs));
    }
    const bool reuse = t + 1 == t1 && x_pub != kZCanon;
    uint64_t x;
    uint64_t fso = ~0ull;
    const uint32_t why = count_staged<J>(tiles, spans, ctl, s_img, s_j, lane, t, z, xs, t + 1 == t1 ? x_pub : kZCanon,
                                         reuse ? &sp_last : nullptr, &x, nullptr, nullptr, &fso);
    if (why == 0u || why == 3u) {
      x_prev = x;
      if (lane == 0) {
        st_agent(&ctl.ex[t], kZExValid | x);
        if (ctl.dbg) {  // developer diagnostics (CLONOS_FUSED_DEBUG): who wrote ex[t], from which entry
          uint64_t* w = reinterpret_cast<uint64_t*>(ctl.dbg + kZDbgTiles) + 2 * (uint64_t)t;
          w[0] = xs;
          w[1] = 1ull << 60 | (uint64_t)blockIdx.x << 32 | (uint64_t)(t0 & 0xFFFFFF) << 4 | why;
        }
        if (why == 3u) {  // the chunk holding the next tile entered elsewhere (empty chunks skipped)
          uint32_t c = blockIdx.x + 1;
          while (chunk_first(ctl, c + 1, K, gridDim.x) == t1) ++c;
          push_repair(ctl, c);
        }
      }
    } else {
      const bool soft = why != 5u && z.td.span == sus_span;  // the published entry may be wrong
      if (lane == 0) {
        if (soft) {
          push_repair(ctl, blockIdx.x);
          if (why == 1u && fso != ~0ull) st_agent(&ctl.ex[t], kZExFail | fso);  // for check_chunk, if real
        } else {
          mark_bad(ctl, why, t, z.td.span);
          if (why == 1u) note_error(ctl, z.td.span, fso);  // the entry is the true chain's
        }
      }
      if (!soft && !ctl.span_bad) return;
      if (soft)  // go on from the next tile's first byte (a guess; the repair checks it), so that
        x_prev = z.td.span_off + z.td.len;  // the chunk's later tiles have exits to resync with
      else
        bad_span = z.td.span;  // the next span starts on a record boundary: go on there
    }
    __syncthreads();  // the image is reused by the next tile
  }
}

// The repair requests, right after the count pass: one block per chunk (the count pass's
// grid).  Block b serves the flagged chunks of the span holding chunk b's first tile, in
// order, when b is that span's first flagged chunk; spans are independent, so their walks run
// side by side.  In the usual batch (no requests) every block reads one word and returns.  A
// loop of its own in the count kernel, the repairs took it from 93 to 121 VGPRs (128 to 179
// with tables), and as a second loop after the chunk's, with tables, to 158.
template <bool J>
__global__ __launch_bounds__(64) void k_decode_repair(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                      FusedCtl ctl) {
  __shared__ uint32_t s_img[kZImgDw];
  __shared__ uint32_t s_j[J ? 2 * kZJBitsDw + kZJCap : 1];
  // the batch goes again anyway (4 a wait timed out, 5 Serializable records without tables:
  // again with them, 6 a table overflowed)
  if (ld_agent32(ctl.abort + 4) || ld_agent32(ctl.abort + 5) || ld_agent32(ctl.abort + 6)) return;
  const uint32_t G = gridDim.x, b = blockIdx.x, lane = threadIdx.x, K = (ctl.n_tiles + G - 1) / G;
  const uint32_t fb = chunk_first(ctl, b, K, G);
  if (fb >= chunk_first(ctl, b + 1, K, G)) return;  // (an empty chunk is never asked for)
  // chunk c needs serving: a request filed by the count pass, or an entry other than the true
  // exit before it (every block checks its own chunk: two words; the usual batch stops here)
  auto need = [&](uint32_t c, uint32_t f) -> bool { return gp(ctl.rep_flag)[c] || wrong_entry(ctl, c, f); };
  if (!need(b, fb)) return;
  const uint32_t span = tiles[fb].span;
  // an earlier chunk of the same span needing service: that chunk's block serves this one
  for (uint32_t hi = b; hi > 0;) {
    const uint32_t lo = hi > 64u ? hi - 64u : 0u, k = lo + lane;
    const bool in = k < hi;
    const uint32_t ft = in ? chunk_first(ctl, k, K, G) : 0u;
    const uint32_t kt = in ? chunk_first(ctl, k + 1, K, G) : 0u;
    // a chunk's need is for its first tile's span: chunk k counts when that is this span (an
    // empty chunk: no tiles, the scan goes on past it)
    const bool empty = in && kt == ft, same = in && !empty && tiles[ft].span == span;
    if (__any(same && need(k, ft))) return;
    if (!__all(!in || empty || same)) break;  // the span starts inside [lo, hi)
    hi = lo;
  }
  uint32_t walk_end = 0;
  for (uint32_t c = b; c < G; ++c) {
    const uint32_t f = chunk_first(ctl, c, K, G), ce = chunk_first(ctl, c + 1, K, G);
    if (f >= ce) continue;
    if (tiles[f].span != span) break;
    if (!gp(ctl.rep_flag)[c]) {
      if (!wrong_entry(ctl, c, f)) continue;
      // counted (the bench line and the tests read it) where the tile before has an exit: else
      // it failed, and its span is bad already
      if (lane == 0 && (ld_agent(&ctl.ex[f - 1]) & kZExValid)) atomicAdd(ctl.rep, 1u);
    }
    serve_chunk<J>(tiles, spans, ctl, s_img, s_j, lane, c, f, ce, &walk_end);
  }
}

// ---------------------------------------------------------------------------------
// Small batches in one launch (config 1: an epoch of 44 logs, 73 KB, where the three-pass
// sequence's ~15 queue operations cost more than the decode; config 5's replay-prep decode:
// 16 main logs of ~45 KB, 6 tiles each).  A block per tile: every block stages its tile and
// walks it speculatively at once; then it takes its entry from the tile before's published
// exit (the span start for a span's first tile) -- only the merge of the true chain is serial
// along a span -- publishes its exit and counts, sums every earlier tile's counts (look-back:
// blocks wait only on lower ones, dispatched first, so the waits end) and emits its tile from
// the image it holds.  A tile whose chain goes wrong -- an invalid record, a Serializable
// record (no tables here) -- flags the batch and the host decodes it the usual way, which
// classifies the error; a wait past kZSpinLimit flags it too.  agg: counts at [t], exits at
// [nt + t]; res: see launch_decode_small (kernels.h), res[3 + s] for the spans with tiles (the
// host fills the empty ones).
// ---------------------------------------------------------------------------------
constexpr uint32_t kZAggSet = 2u, kZAggBad = 3u;  // pk_word states: published, published and bad

__device__ __forceinline__ void decode_small_tiles(const TileDesc* __restrict__ tiles,
                                                   const SpanDesc* __restrict__ spans, uint32_t nt, const FusedCtl& ctl,
                                                   const DecodeOut& out, uint64_t* agg, uint64_t* agg_next,
                                                   uint64_t* res) {
  __shared__ EmitLds<false, true> L;
  const uint32_t t = blockIdx.x, lane = threadIdx.x;
  for (uint32_t j = t + nt * lane; j < kZSmallAggWords; j += 64u * nt) agg_next[j] = 0;
  const ZTile z = ztile(tiles, spans, t, lane);
  const TileDesc n1 = tiles[t + 1 < nt ? t + 1 : t];
  stage_image(z.td, z.sd, t, tiles, L.img, lane, z.hi, &n1);
  const JL jl{nullptr, nullptr, nullptr};
  const uint32_t ws = warm_start(z.rs, z.lo, ctl.warm, lane), wsb = warm_start(lane * kZRegion + 64u, z.lo, ctl.warm, lane);
  const SpecR sp = z.rs < z.re ? spec_walk_fast<false>(L.img, ws, wsb, z.rs, z.re, z.end_a, lane * kZRegion, jl,
                                                       ctl.lean != 0u)
                               : SpecR{{0, 0}, {0, 0}, z.rs, z.rs, 0};
  // the entry: the span start, or the tile before's exit (one lane polls)
  uint64_t xs = z.td.span_off;
  bool bad = false;
  if (!z.first) {
    uint64_t v = 0;
    if (lane == 0) {
      const uint64_t w0 = __builtin_amdgcn_s_memtime();
      while (!pk_state(v = ld_agent(&agg[nt + t - 1]))) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memtime() - w0 >= kZSpinLimit) {
          v = pk_word(kZAggBad, 0);
          break;
        }
      }
    }
    v = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    bad = pk_state(v) == kZAggBad;
    xs = pk_val(v) + (ctl.perturb & 0xFFFFu);  // (perturb: a test switch, 0 in production)
  }
  uint64_t c = 0, x = 0, bm[2] = {0, 0};
  if (!bad) {
    const uint64_t ee = xs - z.td.span_off + z.lo;
    const uint32_t e_true = ee > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)ee;
    uint32_t x_true;
    const uint32_t why = count_tile<false>(t, z, e_true, kZCanon, ctl, L.img, lane, &x_true, jl, tiles, &sp, &c, bm);
    x = z.td.span_off + (x_true - z.lo);
    bad = why != 0u;
  }
  if (lane == 0) {
    st_agent(&agg[nt + t], pk_word(bad ? kZAggBad : kZAggSet, x));
    st_agent(&agg[t], pk_word(bad ? kZAggBad : kZAggSet, c));
  }
  // look-back: every earlier tile's counts
  uint64_t pre = 0;
  bool any_bad = bad;
  for (uint32_t j0 = 0; j0 < t && !any_bad; j0 += 64) {
    const uint32_t j = j0 + lane;
    uint64_t v = 0;
    if (j < t) {
      const uint64_t w0 = __builtin_amdgcn_s_memtime();
      while (!pk_state(v = ld_agent(&agg[j]))) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memtime() - w0 >= kZSpinLimit) {
          v = pk_word(kZAggBad, 0);
          break;
        }
      }
    }
    any_bad = __any(pk_state(v) == kZAggBad);
    uint64_t cj = pk_val(v);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cj += __shfl_xor(cj, off);
    pre += cj;
  }
  if (any_bad) {
    if (lane == 0) __hip_atomic_store(res + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  emit_tile<false, true>(tiles, spans, ctl, out, t, lane, pre, L, bm);
  if (lane == 0) {
    // the hand-offs this tile took, for the host to check once the kernel is done (every tile
    // but a span's first entered at the exit of the tile before; every base is the one before
    // it plus that tile's counts): entry | exit << 32 (span offsets, a small span < 4 GiB),
    // base, counts
    uint64_t* ck = res + 3 + ctl.n_spans + 3ull * t;
    ck[0] = (uint64_t)(uint32_t)xs | (uint64_t)(uint32_t)x << 32;
    ck[1] = pre;
    ck[2] = c;
    if (z.first) res[3 + z.td.span] = pre;
    if (t + 1 == nt) {
      res[0] = (pre + c) & ((1ull << 31) - 1);
      res[1] = (pre + c) >> 31;
    }
  }
}

__global__ __launch_bounds__(64) void k_decode_small_tiles(const TileDesc* __restrict__ tiles,
                                                           const SpanDesc* __restrict__ spans, uint32_t n_tiles,
                                                           FusedCtl ctl, DecodeOut out, uint64_t* agg,
                                                           uint64_t* agg_next, uint64_t* res) {
  decode_small_tiles(tiles, spans, n_tiles, ctl, out, agg, agg_next, res);
}
__global__ __launch_bounds__(64) void k_decode_small_tiles_arg(const SmallPlanArg plan, uint32_t n_tiles, FusedCtl ctl,
                                                               DecodeOut out, uint64_t* agg, uint64_t* agg_next,
                                                               uint64_t* res) {
  decode_small_tiles(plan.tiles, plan.spans, n_tiles, ctl, out, agg, agg_next, res);
}

// ---------------------------------------------------------------------------------
// One pass for large batches without Serializable tables (config 2: 64 logs of 5.5 MB).  A
// block per tile, dispatched in tile order, counts its tile, takes its record base by a
// decoupled look-back and emits from the image and start bitmap it still holds: the log is
// read once and no bitmap goes through HBM (the three passes read the log twice and write and
// read 1 KiB of bitmap per tile), and a wave's chain walk can run beside another's emit stores.
// The true chain's entry is the canonical exit the tile before publishes right after its
// speculative walk (canon_exit_r: the speculative chain over that tile's last 2 KiB, which
// does not depend on its entry), so no tile waits for another's true chain.  Every tile then
// checks that its own true exit equals the canonical exit it published (count_tile's
// must_exit).  Whatever the fast rules do not settle in one tile -- a mismatch there (a record
// longer than the canonical walk's reach crossing a tile end), an invalid record, a record past
// the span end, a Serializable record -- aborts the batch, and the host decodes it with the
// three passes, which repair chunk entries and keep errors.  Blocks wait only on lower blocks,
// dispatched before them, so every wait ends; a wait past kZSpinLimit aborts.
// Words (zeroed by the prep kernel): st_x[t] = pk_word(2, tile t's canonical exit), ex[t] =
// its look-back word (kLbAgg: its packed counts, kLbPre: its inclusive prefix, kZOneBad: it
// aborted), ent[] the counts of finished blocks.  After its emit each tile reads again the two
// words it took -- the tile before's exit and final prefix, which must equal its entry and its
// base -- and aborts the batch on a difference; the last block to finish copies the abort
// words into the host's read-back.
// ---------------------------------------------------------------------------------
constexpr uint32_t kZOneBad = 3u;
// A wait here is short (the tile before is a block dispatched just before this one, at the same
// phase): a fixed short sleep between polls, not the count pass's doubling backoff -- which,
// escalating to ~15 us per poll, made every tile's three waits cost more than its work.
__device__ __forceinline__ bool one_wait(uint64_t w0) {
  __builtin_amdgcn_s_sleep(2);
  return __builtin_amdgcn_s_memtime() - w0 < kZSpinLimit;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ uint64_t first_lane_u64(uint64_t v) {
  return (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32 | (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}
__global__ __launch_bounds__(64) void k_decode_one(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                   FusedCtl ctl, DecodeOut out) {
  __shared__ EmitLds<false, false> L;
  const uint32_t lane = threadIdx.x, nt = ctl.n_tiles;
  // (tiles in block order: an XCD-aware order -- chunks of 64 consecutive tiles per XCD, so that a
  // tile's predecessor ran on its own XCD -- measured slower, 0.61 against 0.58 ms)
  const uint32_t t = blockIdx.x;
  uint32_t why = ld_agent32(ctl.abort) ? 4u : 0u;  // (another tile aborted the batch: nothing to do)
  // developer diagnostics (CLONOS_SCAN_PHASES): per tile, s_memrealtime (100 MHz) at the phase
  // boundaries, in the second half of ctl.prof (the first holds count_tile's stamps);
  // tools/one_pass_phases.py reads them
#define OSTAMP(k) \
  if (ctl.prof && lane == 0) ctl.prof[(uint64_t)(nt + t) * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
  OSTAMP(0);
  if (ctl.prof && lane == 0)
    ctl.prof[(uint64_t)(nt + t) * 8 + 7] = (uint64_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) << 32;
  if (!why) {
    const ZTile z = ztile(tiles, spans, t, lane);
    const TileDesc n1 = tiles[t + 1 < nt ? t + 1 : t];
    stage_image(z.td, z.sd, t, tiles, L.img, lane, z.hi, &n1);
    const JL jl{nullptr, nullptr, nullptr};
    const uint32_t ws = warm_start(z.rs, z.lo, ctl.warm, lane);
    const uint32_t wsb = warm_start(lane * kZRegion + 64u, z.lo, ctl.warm, lane);
    const SpecR sp = z.rs < z.re ? spec_walk_fast<false>(L.img, ws, wsb, z.rs, z.re, z.end_a, lane * kZRegion, jl,
                                                         ctl.lean != 0u)
                                 : SpecR{{0, 0}, {0, 0}, z.rs, z.rs, 0};
    // the successor's entry, published before this tile's own wait
    uint32_t x_pub = kZCanon;
    if (!z.last) {
      x_pub = canon_exit_r<false>(z, L.img, sp, lane, jl, tiles, t);
      if (x_pub < z.hi) {  // (an exit lies at or past the tile end; see k_decode_count)
        if (lane == 0) atomicAdd(ctl.rep + 3, 1u);
        x_pub = z.hi;
      }
      if (lane == 0) st_agent(&ctl.st_x[t], pk_word(2u, (uint64_t)z.td.span_off + (x_pub - z.lo)));
    }
    OSTAMP(1);
    // this tile's entry: the span start, or the tile before's canonical exit (one lane polls)
    uint64_t xs = z.td.span_off;
    if (!z.first) {
      uint64_t v = 0;
      if (lane == 0) {
        const uint64_t w0 = __builtin_amdgcn_s_memtime();
        for (;;) {
          v = ld_agent(&ctl.st_x[t - 1]);
          if (pk_state(v) && pk_val(v) >= z.td.span_off) break;
          if (ld_agent32(ctl.abort) || !one_wait(w0)) {
            v = 0;
            break;
          }
        }
      }
      v = first_lane_u64(v);
      if (!pk_state(v)) why = 4u;
      xs = pk_val(v) + (ctl.perturb & 0xFFFFu);  // (perturb: a test switch, 0 in production)
    }
    OSTAMP(2);
    uint64_t c = 0, bm[2] = {0, 0};
    if (!why) {
      const uint64_t ee = xs - z.td.span_off + z.lo;
      const uint32_t e_true = ee > 0xFFFFFF00ull ? 0xFFFFFF00u : (uint32_t)ee;
      uint32_t x_true;
      why = count_tile<false>(t, z, e_true, x_pub, ctl, L.img, lane, &x_true, jl, tiles, &sp, &c, bm);
    }
    OSTAMP(3);
    // counts published, then the base: look back over the tiles before, 64 at a time
    uint64_t pre = 0;
    if (!why) {
      if (lane == 0) st_agent(&ctl.ex[t], pk_word(t == 0 ? kLbPre : kLbAgg, c));
      const uint64_t w0 = __builtin_amdgcn_s_memtime();
      for (uint32_t hi = t; hi > 0;) {  // window: tiles hi - 1, hi - 2, ... (lane 0 the nearest)
        const bool in = lane < hi;
        const uint64_t v = in ? ld_agent(&ctl.ex[hi - 1 - lane]) : pk_word(kLbPre, 0);
        const uint32_t st = pk_state(v);
        const uint64_t m_pre = __ballot(st == kLbPre), m_bad = __ballot(st == kZOneBad), m_none = __ballot(st == 0u);
        const uint32_t f = m_pre ? (uint32_t)__builtin_ctzll(m_pre) : 64u;  // the nearest prefix
        const uint64_t upto = f >= 63u ? ~0ull : (2ull << f) - 1ull;   // lanes 0 .. f
        if (m_bad & upto) {
          why = 4u;
          break;
        }
        if (m_none & upto) {  // not all published yet: the same window again
          if (ld_agent32(ctl.abort) || !one_wait(w0)) {
            why = 4u;
            break;
          }
          continue;
        }
        pre += wave_sum_u64(lane <= f ? pk_val(v) : 0ull);
        if (f < 64u) break;
        hi = hi > 64u ? hi - 64u : 0u;
      }
      if (!why) {
        if ((ctl.perturb >> 16) && t == 1) ++pre;  // (test switch: a wrong look-back result)
        if (lane == 0 && t) st_agent(&ctl.ex[t], pk_word(kLbPre, pre + c));
        if (z.last && lane == 0) {  // the span's record range ends here
          gp(ctl.span_hi)[z.td.span] = pre + c;
          if (ctl.h_res) reinterpret_cast<volatile uint64_t*>(ctl.h_res)[ctl.n_spans + z.td.span] = pre + c;
        }
        OSTAMP(4);
        emit_tile<false, false>(tiles, spans, ctl, out, t, lane, pre, L, bm);
        OSTAMP(5);
        // the words taken, read again: the tile before's exit and its final prefix
        if (lane == 0 && t) {
          if (!z.first && pk_val(ld_agent(&ctl.st_x[t - 1])) != xs) why = 7u;
          uint64_t w;
          const uint64_t w2 = __builtin_amdgcn_s_memtime();
          while (pk_state(w = ld_agent(&ctl.ex[t - 1])) != kLbPre) {
            if (pk_state(w) == kZOneBad || ld_agent32(ctl.abort) || !one_wait(w2)) break;
          }
          if (pk_state(w) == kLbPre && pk_val(w) != pre) why = 7u;
        }
        why = __shfl(why, 0);
      }
    }
    if (why && lane == 0) {  // (7: a word taken differed from its final value; rep[2] counts it)
      if (why == 7u) atomicAdd(ctl.rep + 2, 1u);
      st_agent(&ctl.ex[t], pk_word(kZOneBad, 0));
      raise_abort(ctl, why == 7u ? 4u : why, t);
      __threadfence();  // (the abort words before this block's count below)
    }
  }
  OSTAMP(6);
#undef OSTAMP
  // the last block to finish copies the abort words into the host's read-back.  Finished
  // blocks are counted in 64 shards (tile t in shard t & 63, each on its own 128-byte line of
  // the zeroed ent words), and a shard's last block counts the shard: one counter taking every
  // block's returning atomic held the blocks ~70 ns each, serialised (3.6 ms for 43 k tiles)
  if (lane == 0 && ctl.h_res) {
    uint32_t* shard = reinterpret_cast<uint32_t*>(ctl.ent) + 32u * (t & 63u);
    const uint32_t in_shard = (nt - (t & 63u) + 63u) >> 6;
    if (atomicAdd(shard, 1u) + 1u == in_shard) {
      const uint32_t shards = nt < 64u ? nt : 64u;
      if (atomicAdd(reinterpret_cast<uint32_t*>(ctl.ent) + 32u * 64u, 1u) + 1u == shards) {
        __threadfence();
        volatile uint32_t* hab = reinterpret_cast<volatile uint32_t*>(ctl.h_res + 2ull * ctl.n_spans);
        for (uint32_t k = 0; k < kZAbortWords; ++k) hab[k] = ld_agent32(ctl.abort + k);
      }
    }
  }
}

int launch_decode_small(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, uint32_t n_spans,
                        FusedCtl ctl, DecodeOut out, uint64_t* agg, uint64_t* agg_next, uint64_t* res, void* stream,
                        const SmallPlanArg* plan) {
  if (!n_spans) return CLG_OK;
  if (!n_tiles || n_tiles > kZSmallTilesMax) return CLG_E_INVALID_ARG;
  ctl.n_tiles = n_tiles;
  if (plan) {
    if (n_tiles > kZSmallArgTiles || n_spans > kZSmallArgSpans) return CLG_E_INVALID_ARG;
    hipLaunchKernelGGL(k_decode_small_tiles_arg, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, *plan, n_tiles, ctl,
                       out, agg, agg_next, res);
  } else {
    hipLaunchKernelGGL(k_decode_small_tiles, dim3(n_tiles), dim3(64), 0, (hipStream_t)stream, d_tiles, d_spans, n_tiles,
                       ctl, out, agg, agg_next, res);
  }
  return launch_status(hipGetLastError());
}

// ---------------------------------------------------------------------------------
// Phase 3 (only for batches holding Serializable records): per tile, the positions of
// "03 AC ED 00 05" (tag + stream magic) and the record length there -- the length of one
// Java serialization stream (jser_device.h walker; TC_STRING streams inline), 0 for an
// invalid stream.  Streams may run past the tile: bytes beyond the LDS image are read
// from the span's next tiles in HBM.
// ---------------------------------------------------------------------------------
struct ZStreamBytes {  // stream byte k = span byte at aligned coordinate base + k
  const uint32_t* T;
  uint32_t base, img_end, lo;
  uint64_t so;  // span offset of aligned coordinate lo
  const TileDesc* tiles;
  uint32_t k, t1;  // tile searched last, end of the span's tiles
  __device__ int operator()(uint64_t i) {
    const uint64_t a = base + i;
    if (a < img_end) return (int)zb(T, (uint32_t)a);
    const uint64_t o = so + (a - lo);
    while (k + 1 < t1 && o >= tiles[k].span_off + tiles[k].len) ++k;
    const TileDesc d = tiles[k];
    return (int)gp(d.abase)[d.delta + (uint32_t)(o - d.span_off)];
  }
};

// Bytes q .. q+3 of the image, little-endian: two independent LDS reads, so a parser step
// that needs a tag and a big-endian u16 after it waits for one LDS latency, not three.
__device__ __forceinline__ uint32_t z4(const uint32_t* T, uint32_t q) {
  const uint32_t k = q >> 2;
  return __builtin_amdgcn_alignbit(T[rk(k + 1)], T[rk(k)], (q & 3u) << 3);
}
__device__ __forceinline__ uint32_t be16_12(uint32_t v) { return ((v >> 8) & 0xFFu) << 8 | ((v >> 16) & 0xFFu); }

// Record length of the common stream shape (jser_flat.h), from the LDS image: 0 = some
// other shape (the general walker decides), or the stream leaves the image.
__device__ __forceinline__ uint32_t jser_flat_len(const uint32_t* T, uint32_t a, uint32_t img_end) {
  return jser_flat_len_t([T](uint32_t q) { return z4(T, q); }, a, img_end);
}

__device__ __forceinline__ bool zmagic(const uint32_t* T, uint32_t a) {
  return zb(T, a) == CLG_TAG_SERIALIZABLE && zbe32(T, a + 1) == 0xACED0005u;
}

// Record length of the candidate at a: inline for TC_STRING and flat objects, 0 = needs
// the general walker (*general set), or an invalid stream (0, *general clear).
__device__ __forceinline__ uint32_t jser_inline_len(const uint32_t* T, uint32_t a, uint32_t img_end, uint64_t avail,
                                                    bool* general) {
  const uint32_t v = z4(T, a + 5);
  const uint32_t tc = v & 0xFFu;
  *general = false;
  if (tc == jser::TC_STRING) {  // [03][AC ED 00 05][74][len u16][modified UTF-8]
    const uint64_t L = 8ull + be16_12(v);
    if (L > avail) return 0u;
    if ((uint64_t)a + L > img_end) {  // its bytes past the image: the walker checks them
      *general = true;
      return 0u;
    }
    return jf_mutf([T](uint32_t q) { return z4(T, q); }, a + 8u, (uint32_t)L - 8u) ? (uint32_t)L : 0u;
  }
  const uint32_t fl = tc == jser::TC_OBJECT ? jser_flat_len(T, a, img_end) : 0u;
  if (fl) return fl <= avail ? fl : 0u;
  *general = true;
  return 0u;
}

constexpr int kZJReg = 4;  // candidates a lane keeps in registers (more: second scan)
constexpr uint32_t kZJGeneral = 0xFFFFFFFFu;  // jlen placeholder: k_decode_jser_general fills it
constexpr uint32_t kZJHalo = 1024;  // phase 3 halo: streams starting near the tile end stay in LDS
constexpr uint32_t kZJRows = (kZTile + 15 + kZJHalo + 64 + 127) / 128 + 1;
__device__ __forceinline__ void jser_tile(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                          const FusedCtl& ctl, uint32_t* s_img, uint32_t* s_cand, const uint32_t t,
                                          const uint32_t lane, bool* flagged) {
  const uint64_t c0 = ctl.prof ? __builtin_amdgcn_s_memtime() : 0;
  const ZTile z = ztile(tiles, spans, t, lane);
  const TileDesc n1 = tiles[t + 1 < ctl.n_tiles ? t + 1 : t];  // halo source, loaded beside t's
  stage_image<kZJHalo, kZJRows>(z.td, z.sd, t, tiles, s_img, lane, z.hi, &n1);
  const uint64_t c1 = ctl.prof ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t after = z.td.span_off + z.td.len;
  const uint64_t rem = z.sd.len > after ? z.sd.len - after : 0;
  const uint32_t img_end = z.hi + (rem < (uint64_t)kZJHalo ? (uint32_t)rem : kZJHalo);
  // candidates in the lane's region (row `lane` of the image, dwords 32 lane + j; j = 32..33
  // are the next row's head).  First a mask of the row's dwords holding an
  // ED byte (rare outside the magic), branch-free; then only the dwords where a magic could
  // start (its ED byte, at +2, lies in that dword or the next) are tested at their four
  // byte offsets for "03 AC ED 00 05" -- a loop over a few set bits per lane, where testing
  // every dword under a per-dword branch ran the test for nearly every dword of the wave
  uint32_t nm = 0, cand[kZJReg];
  const uint32_t r0 = lane * kZRegion;
  const uint32_t* row = s_img + lane * kZPitch;
  uint64_t edm = 0;  // bit j: dword j (0..33) holds an ED byte
  // The rows start 32 dwords apart, so reading dword j of every row at once
  // hits two banks (a 32-way conflict: 7.4 cycles per LDS instruction).  Each lane starts its
  // pass at its own dword and wraps: lane l reads bank 32 (l & 1) + (j + (l >> 1)) mod 34, so
  // the 64 reads of one instruction fall on distinct banks but for wrapped dwords 32-33
  const uint32_t rot = (lane >> 1) & 31u;
  for (uint32_t j0 = 0; j0 < kZRowDw + 2u; j0 += 17u) {  // two slices of 17 dwords (registers)
    uint32_t D[17], J[17];
#pragma unroll
    for (uint32_t j = 0; j < 17; ++j) {
      const uint32_t k = j0 + j + rot;
      J[j] = k >= kZRowDw + 2u ? k - (kZRowDw + 2u) : k;
      D[j] = row[J[j]];
    }
#pragma unroll
    for (uint32_t j = 0; j < 17; ++j) {
      const uint32_t e = D[j] ^ 0xEDEDEDEDu;
      edm |= (((e - 0x01010101u) & ~e & 0x80808080u) ? 1ull : 0ull) << J[j];
    }
  }
  uint64_t sm = (edm | (edm >> 1)) & 0xFFFFFFFFull;  // dwords where a magic may start
  while (sm) {
    const uint32_t j = (uint32_t)__builtin_ctzll(sm);
    sm &= sm - 1u;
    const uint32_t x = row[j], y = row[j + 1], z2 = row[j + 2];
#pragma unroll
    for (uint32_t sh = 0; sh < 4; ++sh) {
      const uint32_t w0 = __builtin_amdgcn_alignbyte(y, x, sh);   // bytes a .. a+3 (LE)
      const uint32_t w1 = __builtin_amdgcn_alignbyte(z2, y, sh);  // bytes a+4 .. a+7
      const uint32_t a = r0 + 4u * j + sh;
      if (w0 == 0x00EDAC03u && (w1 & 0xFFu) == 0x05u && a >= z.rs && a < z.re) {
#pragma unroll
        for (int r = 0; r < kZJReg; ++r)
          if ((uint32_t)r == nm) cand[r] = a;
        ++nm;
      }
    }
  }
  const uint64_t c2 = ctl.prof ? __builtin_amdgcn_s_memtime() : 0;
  uint32_t ex = nm;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(ex, off);
    if ((int)lane >= off) ex += y;
  }
  const uint32_t total = __shfl(ex, 63);
  // past kZJCap candidates the rest go to the overflow arena (a tile of short Serializable
  // strings holds up to ~300); arena exhausted: abort reason 6, the host grows it and retries
  uint32_t ob = 0;
  if (lane == 0) {
    uint32_t n = total;
    if (total && !*flagged) __hip_atomic_store(ctl.abort + 7, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (total > kZJCap) {
      ob = atomicAdd(ctl.jwork + 1, total - kZJCap);
      if (ob + (total - kZJCap) > ctl.jovf_cap) {
        raise_abort(ctl, 6, t);
        n = kZJCap;  // (the batch runs again: no pass reads past the arena meanwhile)
      } else {
        gp(ctl.jbase)[t] = ob;
      }
    }
    gp(ctl.jn)[t] = n;
  }
  ob = __shfl(ob, 0);
  const bool ovf_ok = total <= kZJCap || ob + (total - kZJCap) <= ctl.jovf_cap;
  *flagged = *flagged || total;  // one flag store per block
  uint32_t idx = ex - nm;
  // A candidate's stream length (inline shapes; else the general walker's work list) into
  // table slot sl.
  auto measure = [&](uint32_t a, uint64_t sl) {
    const uint64_t avail = (uint64_t)(z.end_a - a);  // record start to span end
    bool general;
    const uint64_t L = jser_inline_len(s_img, a, img_end, avail, &general);
    gp(ctl.jpos)[sl] = a;
    gp(ctl.jlen)[sl] = general ? kZJGeneral : (L <= 0x7FFFFFF0ull ? (uint32_t)L : 0u);
    if (general) {  // nested objects, arrays, ...: k_decode_jser_general walks the grammar
      const uint32_t w = atomicAdd(ctl.jwork, 1u);
      if (w < ctl.jwork_cap) {
        ctl.jwork[2 + w] = (uint32_t)sl;
        ctl.jwork[2 + ctl.jwork_cap + w] = t;
      } else {
        raise_abort(ctl, 6, t);
      }
    }
  };
  // the tile's first kZJCap candidates in order into LDS, then their lengths 64 at a time (a
  // lane holds ~1 candidate on average: computed in place, the inline parser ran once per
  // register slot with few lanes active); any past them measured in place, into the arena
  auto put = [&](uint32_t a) {
    if (idx < kZJCap) s_cand[idx] = a;
    else if (ovf_ok) measure(a, (uint64_t)ctl.n_tiles * kZJCap + ob + (idx - kZJCap));
    ++idx;
  };
  if (!nm) {
  } else if (nm <= (uint32_t)kZJReg) {
#pragma unroll
    for (int r = 0; r < kZJReg; ++r)
      if ((uint32_t)r < nm) put(cand[r]);
  } else {  // rare: rescan the region
    for (uint32_t k = z.rs >> 2; 4 * k < z.re; ++k) {
      const uint32_t w = s_img[rk(k)] ^ 0x03030303u;
      if (!((w - 0x01010101u) & ~w & 0x80808080u)) continue;
      for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t a = 4 * k + i;
        if (a >= z.rs && a < z.re && zmagic(s_img, a)) put(a);
      }
    }
  }
  __syncthreads();
  const uint32_t nc = total < kZJCap ? total : kZJCap;
  for (uint32_t k = lane; k < nc; k += 64) measure(s_cand[k], (uint64_t)t * kZJCap + k);
  if (ctl.prof && lane == 0) {  // developer diagnostics: stage / scan+lengths cycles
    ctl.prof[(uint64_t)t * 8 + 6] = c1 - c0;
    ctl.prof[(uint64_t)t * 8 + 7] = (c2 - c1) | (__builtin_amdgcn_s_memtime() - c2) << 32;
  }
}

// The same table from the write path's candidates (kernels.h SideCar), without reading the
// tile: its segment's entries inside the tile, those of unknown length kept only where the
// magic is there (read from HBM: a prefix at a chunk's end, or a stream running past it),
// ranked by position; lengths the writer measured are used when the stream ends inside the
// span, every other candidate goes to the general walker (which then decides as it would for
// the scan's candidates).  false: the tile is not in the pool, its segment's list overflowed
// or it holds more than kZSideKept candidates -- the caller scans it (nothing written but
// the scratch).  Wave-uniform; `scr`: the wave's own 2 kZSideKept words of LDS.
constexpr uint32_t kZSideKept = 256;  // candidates of one tile a wave ranks in LDS
// td: tile t's descriptor (the caller loads it a tile ahead).
__device__ __forceinline__ bool side_tile(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                          const FusedCtl& ctl, uint32_t* scr, const uint32_t t, const TileDesc& td,
                                          const uint32_t lane, bool* flagged) {
  const SideCar& S = ctl.side;
  const uint64_t c0 = ctl.prof ? __builtin_amdgcn_s_memtime() : 0;
  const uintptr_t ab = (uintptr_t)td.abase, pb = (uintptr_t)S.pool;
  if (ab < pb || ab - pb >= S.pool_bytes) return false;
  const uint64_t off = ab - pb;
  const uint32_t seg = (uint32_t)(off / S.seg_bytes), so0 = (uint32_t)(off % S.seg_bytes);
  const uint32_t n = (uint32_t)gp(S.hdr)[seg];
  const SpanDesc sd = spans[td.span];  // (issued with the header's load)
  if (n > S.cap) return false;
  const ZTile z = ztile_of(td, sd, t, lane);
  const uint64_t c1 = ctl.prof ? __builtin_amdgcn_s_memtime() : 0;
  const uint32_t lo = so0 + z.lo, hi = so0 + z.hi;  // the tile's bytes, as segment positions
  const CLG_GLOBAL uint32_t* ent = gp(S.ent) + (size_t)seg * S.cap;
  uint32_t* s_a = scr;               // kept candidates: image coordinate
  uint32_t* s_c = scr + kZSideKept;  // and length code
  uint32_t kept = 0;
  for (uint32_t k0 = 0; k0 < n; k0 += 64u) {  // wave-uniform: kept entries compacted in list order
    const uint32_t k = k0 + lane;
    bool keep = false;
    uint32_t a = 0, code = 0;
    if (k < n) {
      const uint32_t e = ent[k];
      const uint32_t pos = e & 0xFFFFu;
      code = e >> 16;
      a = pos - so0;
      keep = pos >= lo && pos < hi && a + 5u <= z.end_a;
      if (keep && code == kSideUnknown) {
        ZStreamBytes acc{nullptr, a, 0u, z.lo, z.td.span_off, tiles, t, z.sd.first_tile + z.sd.n_tiles};
        keep = acc(0) == CLG_TAG_SERIALIZABLE && acc(1) == 0xAC && acc(2) == 0xED && acc(3) == 0x00 && acc(4) == 0x05;
      }
    }
    const uint64_t m = __ballot(keep);
    if (keep) {
      const uint32_t i = kept + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      if (i < kZSideKept) {
        s_a[i] = a;
        s_c[i] = code;
      }
    }
    kept += (uint32_t)__popcll(m);
  }
  if (kept > kZSideKept) return false;
  const uint64_t c2 = ctl.prof ? __builtin_amdgcn_s_memtime() : 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the wave's LDS stores before its reads
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t total = kept;
  uint32_t ob = 0;
  if (lane == 0) {  // as jser_tile: the batch flag, the overflow arena, the tile's count
    uint32_t nn = total;
    if (total > kZJCap) {  // (the batch flag: set once per block by the caller, k_decode_jser_side)
      ob = atomicAdd(ctl.jwork + 1, total - kZJCap);
      if (ob + (total - kZJCap) > ctl.jovf_cap) {
        raise_abort(ctl, 6, t);
        nn = kZJCap;
      } else {
        gp(ctl.jbase)[t] = ob;
      }
    }
    gp(ctl.jn)[t] = nn;
  }
  ob = __shfl(ob, 0);
  const bool ovf_ok = total <= kZJCap || ob + (total - kZJCap) <= ctl.jovf_cap;
  *flagged = *flagged || total;
  // in position order already (the usual case: a list is out of order only where chunks of one
  // launch wrote one segment), else ranked
  bool sorted = true;
  for (uint32_t i = lane; i < total; i += 64u)
    if (i && s_a[i - 1] >= s_a[i]) sorted = false;
  sorted = __ballot(!sorted) == 0;
  uint32_t ngen = 0;  // (diagnostics)
  for (uint32_t i0 = 0; i0 < total; i0 += 64u) {  // wave-uniform: one work-list reservation per pass
    const uint32_t i = i0 + lane;
    const bool on = i < total;
    const uint32_t a = on ? s_a[i] : 0u, code = on ? s_c[i] : 0u;
    uint32_t r = i;  // rank by position
    if (on && !sorted) {
      r = 0;
      for (uint32_t j = 0; j < total; ++j) {
        const uint32_t b = s_a[j];
        r += b < a || (b == a && j < i) ? 1u : 0u;
      }
    }
    uint64_t sl = ~0ull;
    if (on && r < kZJCap) sl = (uint64_t)t * kZJCap + r;
    else if (on && ovf_ok) sl = (uint64_t)ctl.n_tiles * kZJCap + ob + (r - kZJCap);
    const bool known = code != kSideUnknown && a + code <= z.end_a;
    const bool gen = sl != ~0ull && !known;  // the general walker measures it (jser_tile's measure)
    const uint64_t gm = __ballot(gen);
    uint32_t wb = 0;
    if (gm && lane == 0) wb = atomicAdd(ctl.jwork, (uint32_t)__popcll(gm));
    wb = __shfl(wb, 0);
    ngen += (uint32_t)__popcll(gm);
    if (sl == ~0ull) continue;
    gp(ctl.jpos)[sl] = a;
    if (!gen) {
      gp(ctl.jlen)[sl] = code;
    } else {
      gp(ctl.jlen)[sl] = kZJGeneral;
      const uint32_t w = wb + (uint32_t)__popcll(gm & ((1ull << lane) - 1ull));
      if (w < ctl.jwork_cap) {
        ctl.jwork[2 + w] = (uint32_t)sl;
        ctl.jwork[2 + ctl.jwork_cap + w] = t;
      } else {
        raise_abort(ctl, 6, t);
      }
    }
  }
  if (ctl.prof && lane == 0) {  // developer diagnostics: start; descriptor+header, entries, rank+tables
    const uint64_t c3 = __builtin_amdgcn_s_memtime();
    ctl.prof[(uint64_t)t * 8 + 6] = c0;
    ctl.prof[(uint64_t)t * 8 + 7] = (c1 - c0) | (c2 - c1) << 21 | (c3 - c2) << 42 | (uint64_t)(ngen < 31 ? ngen : 31) << 59;
  }
  return true;
}

// The tiles the sidecar does not serve (side_tile false), for k_decode_jser: [0] their
// count, then the tiles (after the general walker's work list; [0] zeroed per batch).
__device__ __forceinline__ uint32_t* side_scan_list(const FusedCtl& ctl) { return ctl.jwork + 2 + 2 * ctl.jwork_cap; }

// Phase 3 from the sidecars: a wave per tile, four to a block, persistent over the tiles;
// tiles it cannot serve are listed for the scan.  Per tile the work is a few dependent
// loads (descriptor, list header, entries), so many waves are resident to overlap them.
__global__ __launch_bounds__(256) void k_decode_jser_side(const TileDesc* __restrict__ tiles,
                                                          const SpanDesc* __restrict__ spans, FusedCtl ctl) {
  __shared__ uint32_t s_scr[4][2 * kZSideKept];
  __shared__ uint32_t s_flag;
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint32_t* list = side_scan_list(ctl);
  if (threadIdx.x == 0) s_flag = 0;
  __syncthreads();
  bool flagged = false;
  const uint32_t stride = gridDim.x * 4u;
  uint32_t t = blockIdx.x * 4u + wv;
  TileDesc td = tiles[t < ctl.n_tiles ? t : 0];
  for (; t < ctl.n_tiles; t += stride) {
    const TileDesc tdn = tiles[t + stride < ctl.n_tiles ? t + stride : t];  // the next tile's, a tile ahead
    if (!side_tile(tiles, spans, ctl, s_scr[wv], t, td, lane, &flagged) && lane == 0) {
      const uint32_t i = atomicAdd(list, 1u);
      list[1 + i] = t;
    }
    td = tdn;
  }
  if (flagged && lane == 0) s_flag = 1;
  __syncthreads();
  // "the batch holds Serializable records" (the host's table hint): one store per block at most,
  // and none once another block's is visible -- a store per wave to this one word queued
  // behind each other and stalled the waves' next loads (the kernel 0.37 against 0.17 ms)
  if (threadIdx.x == 0 && s_flag && !ld_agent32(ctl.abort + 7))
    __hip_atomic_store(ctl.abort + 7, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Persistent grid: block b takes tiles b, b + G, ... (with the sidecar: the listed tiles)
__global__ __launch_bounds__(64) void k_decode_jser(const TileDesc* __restrict__ tiles, const SpanDesc* __restrict__ spans,
                                                    FusedCtl ctl) {
  __shared__ uint32_t s_img[kZJRows * kZPitch];
  __shared__ uint32_t s_cand[kZJCap];
  bool flagged = false;
  const uint32_t* list = ctl.side.hdr ? side_scan_list(ctl) : nullptr;
  const uint32_t n = list ? min(ld_agent32(list), ctl.n_tiles) : ctl.n_tiles;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    jser_tile(tiles, spans, ctl, s_img, s_cand, list ? list[1 + i] : i, threadIdx.x, &flagged);
    __syncthreads();  // the image is reused by the next tile
  }
}

// Phase 3b: the candidates the inline shapes do not cover (nested objects, arrays,
// block data, streams longer than the staged halo), one lane each, through the grammar
// walker (jser_device.h) reading the span from HBM.  Persistent grid over the work list.
__global__ __launch_bounds__(64) void k_decode_jser_general(const TileDesc* __restrict__ tiles,
                                                            const SpanDesc* __restrict__ spans, FusedCtl ctl) {
  const uint32_t n = min(ld_agent32(ctl.jwork), ctl.jwork_cap);
  for (uint32_t i = blockIdx.x * 64 + threadIdx.x; i < n; i += gridDim.x * 64) {
    const uint32_t item = ctl.jwork[2 + i], t = ctl.jwork[2 + ctl.jwork_cap + i];
    const TileDesc td = tiles[t];
    const SpanDesc sd = spans[td.span];
    const uint32_t a = ctl.jpos[item];
    const uint64_t so = td.span_off + (a - td.delta);  // span offset of the record
    ZStreamBytes acc{nullptr, a + 1, 0u, td.delta, td.span_off, tiles, t, sd.first_tile + sd.n_tiles};
    const jser::DevArena ar{ctl.jar};
    const int64_t sl = jser::stream_len(acc, sd.len - so - 1, ar);  // kJsSpill: 0, the robust pipeline retries
    const uint64_t L = sl > 0 ? 1ull + (uint64_t)sl : 0ull;
    ctl.jlen[item] = L <= 0x7FFFFFF0ull ? (uint32_t)L : 0u;
  }
}

// Per-span fallback: one block per bad span sets its tiles' counts.
__global__ __launch_bounds__(256) void k_decode_inject(const SpanDesc* __restrict__ spans, const uint32_t* __restrict__ bad,
                                                       const uint64_t* __restrict__ packed, FusedCtl ctl) {
  const SpanDesc sd = spans[bad[blockIdx.x]];
  const uint64_t v = packed[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < sd.n_tiles; i += 256) gp(ctl.cnt)[sd.first_tile + i] = i == 0 ? v : 0ull;
}
int launch_decode_inject(const SpanDesc* d_spans, const uint32_t* d_bad, const uint64_t* d_packed, uint32_t n_bad,
                         FusedCtl ctl, void* stream) {
  if (!n_bad) return CLG_OK;
  hipLaunchKernelGGL(k_decode_inject, dim3(n_bad), dim3(256), 0, (hipStream_t)stream, d_spans, d_bad, d_packed, ctl);
  return launch_status(hipGetLastError());
}
__global__ __launch_bounds__(256) void k_add_u32(uint32_t* __restrict__ x, uint64_t n, uint32_t delta) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) gp(x)[i] += delta;
}
int launch_add_u32(uint32_t* d_x, uint64_t n, uint32_t delta, void* stream) {
  if (!n) return CLG_OK;
  const uint64_t nb = (n + 255) / 256;
  hipLaunchKernelGGL(k_add_u32, dim3(nb < 1024 ? (uint32_t)nb : 1024u), dim3(256), 0, (hipStream_t)stream, d_x, n, delta);
  return launch_status(hipGetLastError());
}

// grid (bad spans, 16): block (i, y) takes rows y, y + 16, ... of 256 each of span i
__global__ __launch_bounds__(256) void k_sf_place(const SfPlace* __restrict__ place, DecodeOut sc, DecodeOut out,
                                                  FusedCtl ctl) {
  const SfPlace p = place[blockIdx.x];
  const uint64_t base = gp(ctl.span_lo)[p.span];
  const uint64_t R = base & ((1ull << 31) - 1), W = base >> 31;
  const uint64_t step = 256ull * gridDim.y, first = 256ull * blockIdx.y + threadIdx.x;
  if (R + p.nrec <= out.cap)
    for (uint64_t k = first; k < p.nrec; k += step) {
      gp(out.off)[R + k] = gp(sc.off)[p.rbase + k];
      gp(out.tag)[R + k] = gp(sc.tag)[p.rbase + k];
      gp(out.v0)[R + k] = gp(sc.v0)[p.rbase + k];
    }
  if (W + p.nwide <= out.wcap)
    for (uint64_t k = first; k < p.nwide; k += step) {
      const uint64_t j = p.wbase + k;
      gp(out.w_idx)[W + k] = gp(sc.w_idx)[j] + (uint32_t)(R - p.rbase);
      gp(out.w_rc)[W + k] = gp(sc.w_rc)[j];
      gp(out.w_v1)[W + k] = gp(sc.w_v1)[j];
      gp(out.w_var_off)[W + k] = gp(sc.w_var_off)[j];
      gp(out.w_var_len)[W + k] = gp(sc.w_var_len)[j];
      gp(out.w_sub)[W + k] = gp(sc.w_sub)[j];
    }
}
int launch_sf_place(const SfPlace* d_place, uint32_t n_bad, DecodeOut scratch, DecodeOut out, FusedCtl ctl, void* stream) {
  if (!n_bad) return CLG_OK;
  hipLaunchKernelGGL(k_sf_place, dim3(n_bad, 16), dim3(256), 0, (hipStream_t)stream, d_place, scratch, out, ctl);
  return launch_status(hipGetLastError());
}

uint32_t decode_count_grid(bool jser, uint32_t n_tiles) {
  constexpr int kMaxDev = 64;
  static int resident[kMaxDev][2] = {};  // per device: blocks the device keeps resident for the count kernel
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
  const int j = jser ? 1 : 0;
  if (!resident[dev][j]) {
    int per_cu = 0, cus = 0;
    const hipError_t oe = j ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_decode_count<true>, 64, 0)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_decode_count<false>, 64, 0);
    if (oe != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        per_cu < 1 || cus < 1)
      return 0;
    // developer switch: blocks per CU left free (default 1), clamped to [0, per_cu - 1] -- a
    // grid larger than the device keeps resident would leave waiting blocks unscheduled
    const char* m = getenv("CLONOS_COUNT_MARGIN");
    int margin = m ? atoi(m) : 1;
    margin = margin < 0 ? 0 : (margin > per_cu - 1 ? per_cu - 1 : margin);
    resident[dev][j] = (per_cu - margin) * cus;
  }
  return n_tiles < (uint32_t)resident[dev][j] ? n_tiles : (uint32_t)resident[dev][j];
}

// Checked launch: a configuration error names its kernel and grid (stderr) and is returned.
#define ZLAUNCH(k, grid, block, ...)                                                                     \
  do {                                                                                                  \
    hipLaunchKernelGGL(k, grid, block, __VA_ARGS__);                                                    \
    const hipError_t le_ = hipGetLastError();                                                           \
    if (le_ != hipSuccess) {                                                                            \
      fprintf(stderr, "[clonos] launch of %s (grid %u, block %u) failed: %s\n", #k, (unsigned)dim3(grid).x, \
              (unsigned)dim3(block).x, hipGetErrorString(le_));                                        \
      return launch_status(le_);                                                                        \
    }                                                                                                   \
  } while (0)
int launch_decode_fused(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, uint32_t n_spans,
                        FusedCtl ctl, DecodeOut out, void* stream, uint32_t phase) {
  if (!n_tiles) return CLG_OK;
  if (const hipError_t pre = hipGetLastError(); pre != hipSuccess)  // a stale error is not this launch's
    fprintf(stderr, "[clonos] HIP error pending before the decode launch: %s\n", hipGetErrorString(pre));
  ctl.n_tiles = n_tiles;
  const uint32_t nt = n_tiles;
  hipStream_t st = (hipStream_t)stream;
  if (phase == 0) {
    const uint32_t grid = decode_count_grid(ctl.jser != 0, nt);
    if (!grid) return CLG_E_DEVICE;
    const int j = ctl.jser ? 1 : 0;
    if (j) {
      ZLAUNCH(k_decode_count<true>, dim3(grid), dim3(64), 0, st, d_tiles, d_spans, ctl);
      ZLAUNCH(k_decode_repair<true>, dim3(grid), dim3(64), 0, st, d_tiles, d_spans, ctl);
    } else {
      ZLAUNCH(k_decode_count<false>, dim3(grid), dim3(64), 0, st, d_tiles, d_spans, ctl);
      ZLAUNCH(k_decode_repair<false>, dim3(grid), dim3(64), 0, st, d_tiles, d_spans, ctl);
    }
  } else if (phase == 4) {
    ZLAUNCH(k_decode_count_tiny, dim3((nt + 63) / 64), dim3(64), 0, st, d_tiles, d_spans, ctl);
  } else if (phase == 6) {  // the one-pass decode (no tables; ctl.lb, st_x and ex zeroed)
    if (ctl.jser) return CLG_E_INVALID_ARG;
    ZLAUNCH(k_decode_one, dim3(nt), dim3(64), 0, st, d_tiles, d_spans, ctl, out);

  } else if (phase == 5) {  // scan, block offsets and span ranges in one launch (ctl.lb zeroed)
    const uint32_t nb = (n_tiles + kZScanBlock - 1) / kZScanBlock;
    ZLAUNCH(k_decode_scan, dim3(nb), dim3(256), 0, st, d_tiles, d_spans, n_spans, ctl);
  } else if (phase == 1) {
    const uint32_t nb = (n_tiles + kZScanBlock - 1) / kZScanBlock;
    if (nb > 1024u) return CLG_E_INVALID_ARG;  // > 1M tiles (8 GiB) per batch: the host splits
    ZLAUNCH(k_decode_scan1, dim3(nb), dim3(256), 0, st, ctl);
    ZLAUNCH(k_decode_scan2, dim3(1), dim3(256), 0, st, ctl, nb);
    ZLAUNCH(k_decode_spans, dim3((n_spans + 255) / 256), dim3(256), 0, st, d_spans, n_spans, ctl);
  } else if (phase == 2) {
    if (ctl.jser)
      ZLAUNCH(k_decode_emit<true>, dim3(nt), dim3(64), 0, st, d_tiles, d_spans, ctl, out);
    else
      ZLAUNCH(k_decode_emit<false>, dim3(nt), dim3(64), 0, st, d_tiles, d_spans, ctl, out);
  } else {
    static int jres = 0;  // blocks the device keeps resident for the table kernel
    if (!jres) {
      int dev = 0, per_cu = 0, cus = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_decode_jser, 64, 0) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1 || cus < 1)
        return CLG_E_DEVICE;
      jres = per_cu * cus;
    }
    if (ctl.side.hdr) {
      static int sres = 0;  // blocks the device keeps resident for the sidecar kernel
      if (!sres) {
        int dev = 0, per_cu = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_decode_jser_side, 256, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1 || cus < 1)
          return CLG_E_DEVICE;
        sres = per_cu * cus;
      }
      const uint32_t nb = (nt + 3u) / 4u;
      ZLAUNCH(k_decode_jser_side, dim3(nb < (uint32_t)sres ? nb : (uint32_t)sres), dim3(256), 0, st, d_tiles, d_spans,
              ctl);
    }
    ZLAUNCH(k_decode_jser, dim3(nt < (uint32_t)jres ? nt : (uint32_t)jres), dim3(64), 0, st,
                       d_tiles, d_spans, ctl);
    ZLAUNCH(k_decode_jser_general, dim3(256), dim3(64), 0, st, d_tiles, d_spans, ctl);
  }
  return launch_status(hipGetLastError());
}

}  // namespace clg
