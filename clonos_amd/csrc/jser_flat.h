// jser_flat.h -- record length of the common Serializable stream shape, call-free.
//
// One TC_OBJECT whose class and superclasses are fresh TC_CLASSDESCs with flags
// SC_SERIALIZABLE only, primitive fields only and an empty annotation (java.lang.Boolean,
// Integer, Long, ...); its class data is then the fields' primitive values.  Grammar: Java
// Object Serialization Specification 6.4 (newObject, newClassDesc, classDescInfo, fieldDesc,
// nowrclass); the records are SimpleDeterminantEncoder.java:316-341's.  Shared by the decode
// (bytes from the LDS image) and the write path's sidecar (bytes from the staged chunk), so
// both give the same length for the same bytes; compiled for the host by
// tests/jser_walker_host.cpp, where tests/test_jser_reference.py holds it to the oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jser_device.h"

namespace clg {

__host__ __device__ __forceinline__ uint32_t jf_be16_12(uint32_t v) { return ((v >> 8) & 0xFFu) << 8 | ((v >> 16) & 0xFFu); }

// Bytes [q, q + len) as readUTF takes them (all present): modified UTF-8, JDK 8
// ObjectInputStream.BlockDataInputStream.readUTFBody -- units 0xxxxxxx, 110xxxxx 10xxxxxx,
// 1110xxxx 10xxxxxx 10xxxxxx, none cut by the length (else UTFDataFormatException).  Four
// ASCII bytes at a time.
template <class Rd4>
__host__ __device__ __forceinline__ bool jf_mutf(Rd4&& rd4, uint32_t q, uint32_t len) {
  for (uint32_t i = 0; i < len;) {
    const uint32_t w = rd4(q + i);
    if (len - i >= 4u && !(w & 0x80808080u)) {
      i += 4u;
      continue;
    }
    const uint32_t b1 = w & 0xFFu;
    if (b1 < 0x80u) {
      ++i;
      continue;
    }
    const uint32_t k = (b1 >> 5) == 6u ? 2u : (b1 >> 4) == 14u ? 3u : 0u;
    if (!k || len - i < k || ((w >> 8) & 0xC0u) != 0x80u || (k == 3u && ((w >> 16) & 0xC0u) != 0x80u)) return false;
    i += k;
  }
  return true;
}

// rd4(q): bytes q .. q+3 little-endian (bytes at or past `end` may be anything).  a: the
// record's tag byte ("03", then AC ED 00 05).  Returns the record length, or 0: some other
// shape (the general walker decides), or the stream does not end before `end`.
template <class Rd4>
__host__ __device__ __forceinline__ uint32_t jser_flat_len_t(Rd4&& rd4, uint32_t a, uint32_t end) {
  uint32_t p = a + 5;  // after the tag and AC ED 00 05
  if (p + 1 > end || (rd4(p) & 0xFFu) != jser::TC_OBJECT) return 0u;
  ++p;
  uint32_t data = 0;
  for (int depth = 0;; ++depth) {
    if (p + 1 > end || depth > 8) return 0u;
    const uint32_t v = rd4(p);  // [TC_CLASSDESC][className length u16] or [TC_NULL]
    const uint32_t b = v & 0xFFu;
    if (b == jser::TC_NULL && depth > 0) {  // no (further) superclass (the object's own class
      ++p;                                   // null: not a stream the JDK reads -- the walker says so)
      break;
    }
    if (b != jser::TC_CLASSDESC || p + 3 > end) return 0u;
    const uint32_t nq = p + 3, nl = jf_be16_12(v);
    p += 3 + nl + 8;  // className, serialVersionUID
    if (p + 3 > end || !jf_mutf(rd4, nq, nl)) return 0u;
    const uint32_t f = rd4(p);  // [flags][field count u16]
    if ((f & 0xFFu) != jser::SC_SERIALIZABLE) return 0u;
    const uint32_t nf = jf_be16_12(f);
    if (nf & 0x8000u) return 0u;
    p += 3;
    for (uint32_t i = 0; i < nf; ++i) {
      if (p + 3 > end) return 0u;
      const uint32_t fv = rd4(p);  // [typecode][fieldName length u16]
      const uint32_t tc = fv & 0xFFu;
      // primitive sizes: B 1, C 2, D 8, F 4, I 4, J 8, S 2, Z 1
      const uint32_t sz = tc == 'B' || tc == 'Z' ? 1u : tc == 'C' || tc == 'S' ? 2u : tc == 'I' || tc == 'F' ? 4u
                          : tc == 'J' || tc == 'D' ? 8u : 0u;
      if (!sz) return 0u;
      data += sz;
      const uint32_t fq = p + 3, fl = jf_be16_12(fv);
      p += 3 + fl;
      if (p > end || !jf_mutf(rd4, fq, fl)) return 0u;  // the field name
    }
    if (p + 1 > end || (rd4(p) & 0xFFu) != jser::TC_ENDBLOCKDATA) return 0u;
    ++p;
  }
  p += data;
  return p <= end ? p - a : 0u;
}

}  // namespace clg
