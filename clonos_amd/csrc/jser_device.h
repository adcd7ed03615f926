// jser_device.h -- the length of one Java Object Serialization stream, on the device.
//
// SERIALIZABLE determinants carry `ObjectOutputStream(...).writeObject(o)` bytes with no
// length prefix (reference: causal/determinant/SimpleDeterminantEncoder.java:316-341);
// decodeNext relies on ObjectInputStream consuming exactly one object.  To find the
// record end on the GPU we walk the stream grammar (Java Object Serialization
// Specification section 6.4) with an explicit frame stack, one lane per stream.
//
// Tables.  The walk keeps a handle table, class descriptors, their field typecodes and
// the frame stack.  A first tier lives in the lane's private memory (enough for every
// stream the reference's own test resources hold but a few); past it each table doubles
// into the spill arena (kernels.h JArena: bump-allocated HBM scratch).  A walk that finds
// the arena full returns kJsSpill -- never "invalid" -- and the engine grows the arena and
// decodes again, so no table bound rejects a valid stream.
//
// Limits that are semantics, not capacity (identical in both CPU restatements under
// oracle/): object nesting deeper than kMaxDepth stands for the JVM's
// StackOverflowError (an Error the reference's `catch (Exception e)` does not catch), a
// class hierarchy longer than kMaxChain for a cyclic superclass chain.  A class
// descriptor is usable only once complete (its superclass read): JDK 8's
// ObjectStreamClass is initialised at the end of readNonProxyDesc.
//
// The walk is __host__ __device__ so that tests compile this very code for the CPU and
// compare it with the oracle (tests/jser_walker_host.cpp).  Independent of the oracle's
// recursive walker.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace clg {
namespace jser {

constexpr uint8_t TC_NULL = 0x70, TC_REFERENCE = 0x71, TC_CLASSDESC = 0x72, TC_OBJECT = 0x73,
                  TC_STRING = 0x74, TC_ARRAY = 0x75, TC_CLASS = 0x76, TC_BLOCKDATA = 0x77,
                  TC_ENDBLOCKDATA = 0x78, TC_RESET = 0x79, TC_BLOCKDATALONG = 0x7A,
                  TC_LONGSTRING = 0x7C, TC_PROXYCLASSDESC = 0x7D, TC_ENUM = 0x7E;
constexpr uint8_t SC_WRITE_METHOD = 0x01, SC_SERIALIZABLE = 0x02, SC_EXTERNALIZABLE = 0x04,
                  SC_BLOCK_DATA = 0x08;

constexpr int kMaxDepth = 512;  // open object() activations (oracle JWalker::object)
constexpr int kMaxChain = 256;  // classes in one object's hierarchy
// private first tier (entries)
constexpr uint32_t kPrivHandles = 64, kPrivDescs = 16, kPrivFields = 128, kPrivFrames = 32;

constexpr int64_t kJsInvalid = -1;  // not a stream (the record is CLG_E_BAD_SERIAL)
constexpr int64_t kJsSpill = -2;    // the spill arena is full: grow it and decode again

enum : uint8_t { K_OBJ, K_STROBJ, K_DESC, K_NEWHANDLE, K_ANNOT, K_ODATA, K_ARR };

struct Desc {
  uint32_t f0, nf;  // the class's field typecodes: ftab[f0, f0 + nf)
  int32_t super;    // superclass descriptor, -1 none
  uint8_t flags;    // 0 until the descriptor is complete (unusable before)
  uint8_t arr;      // component typecode of an array class ("[I" -> 'I'), 0 otherwise
  uint8_t pad[2];
};
struct Frame {
  uint8_t kind, st;
  uint16_t act;  // object() activations that end when this frame pops
  int32_t d, i, n, j;
};

// Spill allocator over the device arena (one atomic per table growth; rare).
struct DevArena {
  JArena a;
  __device__ void* take(uint64_t bytes) const {
    if (!a.base) return nullptr;
    bytes = (bytes + 15) & ~15ull;
    const uint64_t o = atomicAdd(a.used, (unsigned long long)bytes);
    return o + bytes <= a.cap ? a.base + o : nullptr;
  }
};

// Doubles table p (n == cap entries in use) into the arena.
template <class T, class A>
__host__ __device__ inline bool grow(const A& ar, T*& p, uint32_t& cap, uint32_t n) {
  const uint64_t nc = 2ull * cap;
  if (nc > (1ull << 30)) return false;
  T* q = static_cast<T*>(ar.take(nc * sizeof(T)));
  if (!q) return false;
  for (uint32_t k = 0; k < n; ++k) q[k] = p[k];
  p = q;
  cap = uint32_t(nc);
  return true;
}

// F: callable returning the byte at stream offset k (k < avail), as int; the walk asks for
// offsets in non-decreasing order (the device readers keep a forward-only cursor over the
// span's tiles: an offset before it would be read out of bounds).  A: spill
// allocator (take(bytes) -> pointer or null).  Returns the stream length (magic through
// the end of the first object), kJsInvalid or kJsSpill.
template <class F, class A>
__host__ __device__ __noinline__ int64_t stream_len(F& at, uint64_t avail, const A& ar) {
  if (avail < 5) return kJsInvalid;
  if (at(0) != 0xAC || at(1) != 0xED || at(2) != 0x00 || at(3) != 0x05) return kJsInvalid;
  uint64_t pos = 4;
  int32_t h_priv[kPrivHandles];  // handle -> descriptor index; -1 other object, -2 string
  Desc d_priv[kPrivDescs];
  uint8_t f_priv[kPrivFields];
  Frame s_priv[kPrivFrames];
  int32_t* handles = h_priv;
  Desc* descs = d_priv;
  uint8_t* ftab = f_priv;
  Frame* st = s_priv;
  uint32_t ch = kPrivHandles, cd = kPrivDescs, cf = kPrivFields, cs = kPrivFrames;
  uint32_t nh = 0, nd = 0, nf = 0, sp = 0;
  int od = 0;       // open object() activations
  int32_t ret = -1;  // descriptor the last completed classDesc resolved to (-1: null)

#define JS_FAIL return kJsInvalid
#define JS_NEED(k) \
  if ((uint64_t)(k) > avail - pos) JS_FAIL
#define JS_PUSH(kd)                                           \
  do {                                                        \
    if (sp == cs && !grow(ar, st, cs, sp)) return kJsSpill;   \
    st[sp] = Frame{(uint8_t)(kd), 0, 0, 0, 0, 0, 0};          \
    ++sp;                                                     \
  } while (0)
#define JS_POP()           \
  do {                     \
    od -= st[sp - 1].act;  \
    --sp;                  \
  } while (0)
#define JS_NEWHANDLE(v)                                            \
  do {                                                             \
    if (nh == ch && !grow(ar, handles, ch, nh)) return kJsSpill;   \
    handles[nh++] = (int32_t)(v);                                  \
  } while (0)
#define JS_NEWDESC(di)                                         \
  do {                                                         \
    if (nd == cd && !grow(ar, descs, cd, nd)) return kJsSpill; \
    di = (int32_t)nd++;                                        \
    descs[di] = Desc{nf, 0, -1, 0, 0, {0, 0}};                 \
  } while (0)

  auto u8 = [&]() -> int { return at(pos++); };
  auto u16 = [&]() -> uint32_t { uint32_t v = (uint32_t)at(pos) << 8 | (uint32_t)at(pos + 1); pos += 2; return v; };
  auto s32 = [&]() -> int32_t {
    uint32_t v = (uint32_t)at(pos) << 24 | (uint32_t)at(pos + 1) << 16 | (uint32_t)at(pos + 2) << 8 | (uint32_t)at(pos + 3);
    pos += 4;
    return (int32_t)v;
  };
  // bytes [pos, pos + l) (present) as readUTF takes them: modified UTF-8, JDK 8
  // BlockDataInputStream.readUTFBody -- units 0xxxxxxx, 110xxxxx 10xxxxxx, 1110xxxx 10xxxxxx
  // 10xxxxxx, none cut by the length; anything else is UTFDataFormatException.  Every byte read
  // once, in order; *c01 (optional): the first two (0 past the end)
  auto mutf = [&](uint64_t l, uint32_t* c01 = nullptr) -> bool {
    uint32_t first = 0;
    for (uint64_t i = 0; i < l;) {
      const uint32_t b1 = (uint32_t)at(pos + i);
      if (i == 0) first = b1;
      if (b1 < 0x80u) {
        if (i == 1) first |= b1 << 8;
        ++i;
        continue;
      }
      const uint64_t k = (b1 >> 5) == 6u ? 2u : (b1 >> 4) == 14u ? 3u : 0u;
      if (!k || l - i < k) return false;
      if (i == 1) first |= b1 << 8;
      for (uint64_t j = 1; j < k; ++j) {
        const uint32_t bj = (uint32_t)at(pos + i + j);
        if (i + j == 1) first |= bj << 8;
        if ((bj & 0xC0u) != 0x80u) return false;
      }
      i += k;
    }
    if (c01) *c01 = first;
    return true;
  };

  // Termination: every step consumes bytes, pushes a frame that will, pops, or advances a
  // frame's bounded state (class index < chain length <= kMaxChain); no step bound needed.
  JS_PUSH(K_OBJ);
  while (sp > 0) {
    Frame& f = st[sp - 1];  // not used after a push (the stack may move)
    switch (f.kind) {
      case K_OBJ: {
        const uint32_t inh = f.act;  // activations (an enum's) that end with this object
        --sp;                        // replaced by whatever the object needs
        const uint32_t base = sp;
        if (++od > kMaxDepth) JS_FAIL;
        int tc;
        for (;;) {  // readObject0 consumes leading TC_RESETs
          JS_NEED(1);
          tc = u8();
          if (tc != TC_RESET) break;
          nh = 0;
        }
        switch (tc) {
          case TC_NULL: break;
          case TC_REFERENCE: {
            JS_NEED(4);
            const int64_t k = (int64_t)s32() - 0x7E0000;
            if (k < 0 || k >= (int64_t)nh) JS_FAIL;
            break;
          }
          case TC_STRING: {
            JS_NEWHANDLE(-2);
            JS_NEED(2);
            const uint32_t l = u16();
            JS_NEED(l);
            if (!mutf(l)) JS_FAIL;
            pos += l;
            break;
          }
          case TC_LONGSTRING: {
            JS_NEWHANDLE(-2);
            JS_NEED(8);
            const uint64_t hi = (uint32_t)s32(), lo = (uint32_t)s32();
            const uint64_t l = hi << 32 | lo;
            if (l > avail - pos || !mutf(l)) JS_FAIL;  // readLongUTF
            pos += l;
            break;
          }
          case TC_CLASSDESC:
          case TC_PROXYCLASSDESC:
            --pos;
            JS_PUSH(K_DESC);
            break;
          case TC_CLASS:
            JS_PUSH(K_NEWHANDLE);
            JS_PUSH(K_DESC);
            break;
          case TC_ENUM:
            JS_PUSH(K_STROBJ);
            JS_PUSH(K_NEWHANDLE);
            JS_PUSH(K_DESC);
            break;
          case TC_ARRAY:
            JS_PUSH(K_ARR);
            JS_PUSH(K_DESC);
            break;
          case TC_OBJECT:
            JS_PUSH(K_ODATA);
            JS_PUSH(K_DESC);
            break;
          default:
            JS_FAIL;
        }
        if (sp > base) st[base].act = (uint16_t)(inh + 1);  // the object ends when its bottom frame pops
        else od -= (int)(inh + 1);
        break;
      }
      case K_STROBJ: {  // className1 / enum constant name: must be a String object
        JS_NEED(1);
        const int tc = at(pos);
        if (tc != TC_STRING && tc != TC_LONGSTRING && tc != TC_REFERENCE) JS_FAIL;
        f.kind = K_OBJ;
        break;
      }
      case K_NEWHANDLE:
        JS_NEWHANDLE(-1);
        JS_POP();
        break;
      case K_ANNOT: {  // contents up to TC_ENDBLOCKDATA
        JS_NEED(1);
        const int tc = at(pos);
        if (tc == TC_ENDBLOCKDATA) {
          ++pos;
          JS_POP();
        } else if (tc == TC_BLOCKDATA) {
          ++pos;
          JS_NEED(1);
          const uint32_t l = (uint32_t)u8();
          JS_NEED(l);
          pos += l;
        } else if (tc == TC_BLOCKDATALONG) {
          ++pos;
          JS_NEED(4);
          const int32_t l = s32();
          if (l < 0) JS_FAIL;
          JS_NEED(l);
          pos += (uint32_t)l;
        } else {
          JS_PUSH(K_OBJ);
        }
        break;
      }
      case K_DESC: {  // d: descriptor, i/n: fields read/declared, j: flags | arr << 8
        if (f.st == 0) {
          JS_NEED(1);
          const int tc = u8();
          if (tc == TC_NULL) {
            ret = -1;
            JS_POP();
          } else if (tc == TC_REFERENCE) {
            JS_NEED(4);
            const int64_t k = (int64_t)s32() - 0x7E0000;
            if (k < 0 || k >= (int64_t)nh || handles[k] < 0) JS_FAIL;
            ret = handles[k];
            JS_POP();
          } else if (tc == TC_CLASSDESC) {
            JS_NEED(2);
            const uint32_t l = u16();
            JS_NEED(l);
            uint32_t c01 = 0;  // (its first two bytes, read by the check: readers only go forwards)
            if (!mutf(l, &c01)) JS_FAIL;  // the class name
            const uint8_t c0 = (uint8_t)c01, c1 = (uint8_t)(c01 >> 8);
            pos += l;
            JS_NEED(8);
            pos += 8;  // serialVersionUID
            int32_t di;
            JS_NEWDESC(di);
            JS_NEWHANDLE(di);  // assigned before classDescInfo (ObjectInputStream.readNonProxyDesc)
            JS_NEED(1);
            const uint32_t flags = (uint32_t)u8();
            JS_NEED(2);
            const uint32_t cnt = u16();
            f.d = di;
            f.i = 0;
            f.n = (int32_t)cnt;
            f.j = (int32_t)(flags | (c0 == '[' ? (uint32_t)c1 : 0u) << 8);
            f.st = 1;
          } else if (tc == TC_PROXYCLASSDESC) {
            int32_t di;
            JS_NEWDESC(di);
            JS_NEWHANDLE(di);
            JS_NEED(4);
            const int32_t cnt = s32();
            if (cnt < 0) JS_FAIL;
            for (int32_t k = 0; k < cnt; ++k) {
              JS_NEED(2);
              const uint32_t l = u16();
              JS_NEED(l);
              if (!mutf(l)) JS_FAIL;  // an interface name
              pos += l;
            }
            f.d = di;
            f.n = 0;
            f.j = SC_SERIALIZABLE;
            f.st = 2;
            JS_PUSH(K_ANNOT);
          } else {
            JS_FAIL;
          }
        } else if (f.st == 1) {  // field descriptors
          if (f.i < f.n) {
            JS_NEED(1);
            const int t = u8();
            JS_NEED(2);
            const uint32_t l = u16();
            JS_NEED(l);
            if (!mutf(l)) JS_FAIL;
            pos += l;  // field name
            const bool obj = t == 'L' || t == '[';
            if (!obj && !(t == 'B' || t == 'C' || t == 'D' || t == 'F' || t == 'I' || t == 'J' || t == 'S' || t == 'Z'))
              JS_FAIL;
            if (nf == cf && !grow(ar, ftab, cf, nf)) return kJsSpill;
            ftab[nf++] = (uint8_t)t;
            f.i++;
            if (obj) JS_PUSH(K_STROBJ);
          } else {
            descs[f.d].f0 = nf - (uint32_t)f.n;  // className1 strings add no fields: contiguous
            descs[f.d].nf = (uint32_t)f.n;
            f.st = 2;
            JS_PUSH(K_ANNOT);  // classAnnotation
          }
        } else if (f.st == 2) {
          f.st = 3;
          JS_PUSH(K_DESC);  // superClassDesc
        } else {  // complete: usable from now on
          Desc& dd = descs[f.d];
          dd.super = ret;
          dd.flags = (uint8_t)(f.j & 0xFF);
          dd.arr = (uint8_t)((uint32_t)f.j >> 8);
          ret = f.d;
          JS_POP();
        }
        break;
      }
      case K_ODATA: {  // d: class, n: hierarchy length, i: class (top-most first), j: field
        if (f.st == 0) {
          if (ret < 0) JS_FAIL;
          JS_NEWHANDLE(-1);
          f.d = ret;
          int n = 0;
          for (int32_t c = ret; c >= 0; c = descs[c].super)
            if (++n > kMaxChain) JS_FAIL;
          f.n = n;
          f.i = 0;
          f.j = 0;
          const uint8_t fl = descs[f.d].flags;
          if (fl & SC_EXTERNALIZABLE) {
            if (!(fl & SC_BLOCK_DATA)) JS_FAIL;  // protocol-1 externalizable: length unknowable
            f.st = 2;
            JS_PUSH(K_ANNOT);
          } else {
            f.st = 1;
          }
        } else if (f.st == 1) {
          if (f.i >= f.n) {
            JS_POP();
            break;
          }
          int32_t c = f.d;
          for (int k = 0; k < f.n - 1 - f.i; ++k) c = descs[c].super;
          const Desc dc = descs[c];
          if (!(dc.flags & SC_SERIALIZABLE)) JS_FAIL;
          if ((uint32_t)f.j < dc.nf) {
            const int t = ftab[dc.f0 + (uint32_t)f.j];
            f.j++;
            const int sz = (t == 'B' || t == 'Z') ? 1 : (t == 'C' || t == 'S') ? 2 : (t == 'I' || t == 'F') ? 4
                           : (t == 'J' || t == 'D') ? 8 : 0;
            if (sz) {
              JS_NEED(sz);
              pos += (uint64_t)sz;
            } else {
              JS_PUSH(K_OBJ);
            }
          } else {
            f.j = 0;
            f.i++;
            if (dc.flags & SC_WRITE_METHOD) JS_PUSH(K_ANNOT);  // custom data up to TC_ENDBLOCKDATA
          }
        } else {
          JS_POP();
        }
        break;
      }
      case K_ARR: {
        if (f.st == 0) {
          if (ret < 0) JS_FAIL;
          JS_NEWHANDLE(-1);
          JS_NEED(4);
          const int32_t size = s32();
          if (size < 0) JS_FAIL;
          int es;
          switch (descs[ret].arr) {
            case 'B': case 'Z': es = 1; break;
            case 'C': case 'S': es = 2; break;
            case 'I': case 'F': es = 4; break;
            case 'J': case 'D': es = 8; break;
            case 'L': case '[': es = 0; break;
            default: JS_FAIL;
          }
          if (es) {
            const uint64_t b = (uint64_t)(uint32_t)size * (uint64_t)es;
            if (b > avail - pos) JS_FAIL;
            pos += b;
            JS_POP();
          } else {
            f.i = 0;
            f.n = size;
            f.st = 1;
          }
        } else {
          if (f.i < f.n) {
            f.i++;
            JS_PUSH(K_OBJ);
          } else {
            JS_POP();
          }
        }
        break;
      }
      default:
        JS_FAIL;
    }
  }
#undef JS_FAIL
#undef JS_NEED
#undef JS_PUSH
#undef JS_POP
#undef JS_NEWHANDLE
#undef JS_NEWDESC
  return (int64_t)pos;
}

}  // namespace jser
}  // namespace clg
