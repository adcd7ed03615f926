// handoff.h -- the encoding of a 64-bit word one block publishes and another polls.
//
// Used by the fused decode for a chunk's published exit (FusedCtl.st_x), the small path's
// look-back words and the one-launch scan's look-back words (decode_fused.hip).  A 2-bit state
// (0: not published) sits in bits 63:62 and again in 31:30; the 60-bit value is split, high 30
// bits in 61:32, low 30 bits in 29:0.  Store and load are single dwordx2 accesses, yet a poll
// in the count pass once took a wrong chunk entry ("A rare chunk-repair abort"), so
// a word whose two states differ -- half of one write beside half of another, or of the zeroed
// word -- is taken as not (yet) published and polled again.  Host-compiled by
// tests/handoff_host.cpp, where tests/test_handoff_words.py checks every such mix.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clg {

__host__ __device__ __forceinline__ uint64_t pk_word(uint32_t state, uint64_t v) {
  const uint32_t h = state << 30 | ((uint32_t)(v >> 30) & 0x3FFFFFFFu), l = state << 30 | ((uint32_t)v & 0x3FFFFFFFu);
  return (uint64_t)h << 32 | l;
}
__host__ __device__ __forceinline__ uint32_t pk_state(uint64_t w) {
  const uint32_t h = (uint32_t)(w >> 62), l = ((uint32_t)w >> 30) & 3u;
  return h == l ? h : 0u;
}
__host__ __device__ __forceinline__ uint64_t pk_val(uint64_t w) {
  return ((w >> 32) & 0x3FFFFFFFull) << 30 | (w & 0x3FFFFFFFull);
}

}  // namespace clg
