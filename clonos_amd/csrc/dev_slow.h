// dev_slow.h -- exact out-of-line record parsing through a span reader, including the
// Java serialization walker.  Kernels that call these functions pay for a call ABI
// (registers, scratch), so the hot fast-path kernels do not include this header.
#pragma once
#include "dev_common.h"
#include "jser_device.h"

namespace clg {

// Exact record length at a record start (decodeNext read order and error precedence).
// `avail` = bytes from the record start to the span end (>= 1).  Returns L > 0 or a
// negative CLG_E_* status; CLG_E_NOSPACE: the stream walker's spill arena (b.arena())
// is full -- not a decode result, the engine grows the arena and decodes again.
template <class F>
__device__ __noinline__ int64_t rec_len_slow(F& b, uint64_t avail) {
  const int tag = (int8_t)b(0);
  int64_t L;
  switch (tag) {
    case CLG_TAG_ORDER: L = 2; break;
    case CLG_TAG_TIMESTAMP: L = 9; break;
    case CLG_TAG_RNG:
    case CLG_TAG_BUFFER_BUILT: L = 5; break;
    case CLG_TAG_IGNORE_CHECKPOINT: L = 13; break;
    case CLG_TAG_TIMER_TRIGGER: {
      if (avail < 14) return CLG_E_TRUNCATED;
      const int ord = (int8_t)b(13);
      if (ord < 0 || ord > 6) return CLG_E_BAD_ENUM;
      if (ord == 6) {
        if (avail < 18) return CLG_E_TRUNCATED;
        const int32_t nl = (int32_t)rd_be32(b, 14);
        if (nl < 0) return CLG_E_NEG_LEN;
        L = 18 + (int64_t)nl;
      } else {
        L = 14;
      }
      break;
    }
    case CLG_TAG_SOURCE_CHECKPOINT: {
      if (avail < 23) return CLG_E_TRUNCATED;
      if (b(22) != 0) {
        if (avail < 27) return CLG_E_TRUNCATED;
        const int32_t rl = (int32_t)rd_be32(b, 23);
        if (rl < 0) return CLG_E_NEG_LEN;
        L = 27 + (int64_t)rl;
      } else {
        L = 23;
      }
      if ((uint64_t)L > avail) return CLG_E_TRUNCATED;
      const int ord = (int8_t)b(21);
      if (ord < 0 || ord > 1) return CLG_E_BAD_ENUM;
      return L;
    }
    case CLG_TAG_SERIALIZABLE: {
      struct Shift {
        F* f;
        __device__ int operator()(uint64_t k) { return (*f)(k + 1); }
      } sh{&b};
      const jser::DevArena ar{b.arena()};
      const int64_t j = jser::stream_len(sh, avail - 1, ar);
      if (j == jser::kJsSpill) return CLG_E_NOSPACE;
      if (j < 0) return CLG_E_BAD_SERIAL;
      L = 1 + j;
      break;
    }
    default:
      return CLG_E_CORRUPT_TAG;
  }
  if ((uint64_t)L > avail) return CLG_E_TRUNCATED;
  return L;
}

template <class F>
__device__ int decode_rec(F& b, uint64_t avail, Rec& r) {
  const int64_t L = rec_len_slow(b, avail);
  if (L < 0) return (int)L;
  const int tag = b(0);
  r.tag = (uint8_t)tag;
  r.L = (uint32_t)L;
  r.wide = (uint8_t)is_wide(tag);
  r.v1 = 0;
  r.rc = 0;
  r.var_off = 0;
  r.var_len = 0;
  r.sub = 0;
  switch (tag) {
    case CLG_TAG_ORDER: r.v0 = (int8_t)b(1); break;
    case CLG_TAG_TIMESTAMP: r.v0 = (int64_t)rd_be64(b, 1); break;
    case CLG_TAG_RNG:
    case CLG_TAG_BUFFER_BUILT: r.v0 = (int32_t)rd_be32(b, 1); break;
    case CLG_TAG_IGNORE_CHECKPOINT:
      r.rc = (int32_t)rd_be32(b, 1);
      r.v0 = (int64_t)rd_be64(b, 5);
      break;
    case CLG_TAG_TIMER_TRIGGER:
      r.rc = (int32_t)rd_be32(b, 1);
      r.v0 = (int64_t)rd_be64(b, 5);
      r.sub = (uint8_t)b(13);
      if (r.sub == 6) {
        r.var_off = 18;
        r.var_len = (uint32_t)(L - 18);
      }
      break;
    case CLG_TAG_SOURCE_CHECKPOINT:
      r.rc = (int32_t)rd_be32(b, 1);
      r.v0 = (int64_t)rd_be64(b, 5);
      r.v1 = (int64_t)rd_be64(b, 13);
      r.sub = (uint8_t)b(21);
      if (b(22) != 0) {
        r.sub |= 0x80;
        r.var_off = 27;
        r.var_len = (uint32_t)(L - 27);
      }
      break;
    case CLG_TAG_SERIALIZABLE:
      r.v0 = L - 1;
      r.var_off = 1;
      r.var_len = (uint32_t)(L - 1);
      break;
  }
  return CLG_OK;
}

// Exact length through the span reader (Serializable streams; error classification).
__device__ __noinline__ int64_t len_slow_span(SpanReader* sr, uint64_t so) {
  AtSpan b{sr, so};
  return rec_len_slow(b, sr->len - so);
}

// Length of the record at aligned coordinate a (< hi), fast path + slow fallback.
__device__ __forceinline__ int64_t rec_len_at(const uint32_t* T, SpanReader* sr, uint32_t a, uint32_t lo,
                                              uint64_t tile_so, uint64_t end_a, int* tag_out) {
  const int tag = t_u8(T, a);
  *tag_out = tag;
  int64_t L = len_inline(T, tag, a, end_a);
  if (L == kLenSlow) {
    L = len_slow_span(sr, tile_so + (a - lo));
    if (L <= 0) L = kLenErr;
  }
  return L;
}

// Forward parse of one region from an entry (aligned coordinate `a`) to `stop`.
// Returns the exit (first record start >= stop) and counts, or kLenErr.
__device__ int region_forward(const uint32_t* T, SpanReader* sr, uint32_t lo, uint64_t tile_so, uint64_t end_a,
                              uint32_t a, uint32_t stop, uint32_t* exit, uint32_t* cnt, uint32_t* wcnt) {
  uint32_t c = 0, w = 0;
  while (a < stop) {
    int tag;
    const int64_t L = rec_len_at(T, sr, a, lo, tile_so, end_a, &tag);
    if (L < 0) return CLG_E_STATE;
    w += is_wide(tag);
    ++c;
    if ((uint64_t)a + (uint64_t)L > 0xFFFFFFF0ull) return CLG_E_STATE;
    a += (uint32_t)L;
  }
  *exit = a;
  *cnt = c;
  *wcnt = w;
  return CLG_OK;
}

}  // namespace clg
