// jser_device.h -- device-side length of one Java Object Serialization stream.
//
// SERIALIZABLE determinants carry `ObjectOutputStream(...).writeObject(o)` bytes with no
// length prefix (reference: causal/determinant/SimpleDeterminantEncoder.java:316-341);
// decodeNext relies on ObjectInputStream consuming exactly one object.  To find the
// record end on the GPU we walk the stream grammar (Java Object Serialization
// Specification section 6.4) with an explicit stack -- one lane per record, bounded
// tables.  Streams that exceed the bounds are reported as malformed (CLG_E_BAD_SERIAL).
// Independent of the CPU oracle's recursive walker (oracle/clonos_oracle.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clg {
namespace jser {

constexpr uint8_t TC_NULL = 0x70, TC_REFERENCE = 0x71, TC_CLASSDESC = 0x72, TC_OBJECT = 0x73,
                  TC_STRING = 0x74, TC_ARRAY = 0x75, TC_CLASS = 0x76, TC_BLOCKDATA = 0x77,
                  TC_ENDBLOCKDATA = 0x78, TC_RESET = 0x79, TC_BLOCKDATALONG = 0x7A,
                  TC_LONGSTRING = 0x7C, TC_PROXYCLASSDESC = 0x7D, TC_ENUM = 0x7E;
constexpr uint8_t SC_WRITE_METHOD = 0x01, SC_SERIALIZABLE = 0x02, SC_EXTERNALIZABLE = 0x04,
                  SC_BLOCK_DATA = 0x08;

constexpr int kMaxHandles = 64, kMaxDescs = 16, kMaxFields = 128, kMaxStack = 32;
constexpr int kMaxSteps = 1 << 16;

enum : uint8_t { K_OBJ, K_STROBJ, K_DESC, K_NEWHANDLE, K_ANNOT, K_ODATA, K_ARR };

struct Desc {
  uint8_t flags;
  uint8_t arr;  // component typecode for array classes ("[I" -> 'I'), 0 otherwise
  uint8_t f0;   // first field in the field table
  uint8_t nf;
  int8_t super;
  uint8_t pad[3];
};
struct Frame {
  uint8_t kind, st;
  int16_t d;
  int32_t i, n, j;
};

// F: callable returning the byte at stream offset k (k < avail), as int.
// Returns the stream length (magic through the end of the first object) or -1.
template <class F>
__device__ __noinline__ int64_t stream_len(F& at, uint64_t avail) {
  if (avail < 5) return -1;
  if (at(0) != 0xAC || at(1) != 0xED || at(2) != 0x00 || at(3) != 0x05) return -1;
  uint64_t pos = 4;
  int16_t handles[kMaxHandles];
  Desc descs[kMaxDescs];
  uint8_t ftab[kMaxFields];
  Frame st[kMaxStack];
  int nh = 0, nd = 0, nf = 0, sp = 0, ret = -1;

#define JS_FAIL return -1
#define JS_NEED(k) if ((uint64_t)(k) > avail - pos) JS_FAIL
#define JS_PUSH(kd)                      \
  do {                                   \
    if (sp >= kMaxStack) JS_FAIL;        \
    st[sp].kind = (kd); st[sp].st = 0;   \
    st[sp].d = 0; st[sp].i = st[sp].n = st[sp].j = 0; \
    ++sp;                                \
  } while (0)
#define JS_NEWHANDLE(v)                  \
  do {                                   \
    if (nh >= kMaxHandles) JS_FAIL;      \
    handles[nh++] = (int16_t)(v);        \
  } while (0)

  auto u8 = [&]() -> int { return at(pos++); };
  auto u16 = [&]() -> uint32_t { uint32_t v = (uint32_t)at(pos) << 8 | (uint32_t)at(pos + 1); pos += 2; return v; };
  auto s32 = [&]() -> int32_t {
    uint32_t v = (uint32_t)at(pos) << 24 | (uint32_t)at(pos + 1) << 16 | (uint32_t)at(pos + 2) << 8 | (uint32_t)at(pos + 3);
    pos += 4;
    return (int32_t)v;
  };

  JS_PUSH(K_OBJ);
  for (int steps = 0; sp > 0; ++steps) {
    if (steps > kMaxSteps) JS_FAIL;
    Frame& f = st[sp - 1];
    switch (f.kind) {
      case K_OBJ: {
        int tc;
        for (;;) {  // readObject0 consumes leading TC_RESETs
          JS_NEED(1);
          tc = u8();
          if (tc != TC_RESET) break;
          nh = 0;
        }
        --sp;  // this frame is replaced by whatever the object needs
        switch (tc) {
          case TC_NULL: break;
          case TC_REFERENCE: {
            JS_NEED(4);
            int64_t k = (int64_t)s32() - 0x7E0000;
            if (k < 0 || k >= nh) JS_FAIL;
            break;
          }
          case TC_STRING: {
            JS_NEWHANDLE(-2);
            JS_NEED(2);
            uint32_t l = u16();
            JS_NEED(l);
            pos += l;
            break;
          }
          case TC_LONGSTRING: {
            JS_NEWHANDLE(-2);
            JS_NEED(8);
            uint64_t hi = (uint32_t)s32(), lo = (uint32_t)s32();
            uint64_t l = hi << 32 | lo;
            if (l > avail - pos) JS_FAIL;
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
        break;
      }
      case K_STROBJ: {  // className1 / enum constant: must be a String object
        JS_NEED(1);
        int tc = at(pos);
        if (tc != TC_STRING && tc != TC_LONGSTRING && tc != TC_REFERENCE) JS_FAIL;
        f.kind = K_OBJ;
        break;
      }
      case K_NEWHANDLE:
        JS_NEWHANDLE(-1);
        --sp;
        break;
      case K_ANNOT: {  // contents up to TC_ENDBLOCKDATA
        JS_NEED(1);
        int tc = at(pos);
        if (tc == TC_ENDBLOCKDATA) {
          ++pos;
          --sp;
        } else if (tc == TC_BLOCKDATA) {
          ++pos;
          JS_NEED(1);
          uint32_t l = (uint32_t)u8();
          JS_NEED(l);
          pos += l;
        } else if (tc == TC_BLOCKDATALONG) {
          ++pos;
          JS_NEED(4);
          int32_t l = s32();
          if (l < 0) JS_FAIL;
          JS_NEED(l);
          pos += (uint32_t)l;
        } else {
          JS_PUSH(K_OBJ);
        }
        break;
      }
      case K_DESC: {
        if (f.st == 0) {
          JS_NEED(1);
          int tc = u8();
          if (tc == TC_NULL) {
            ret = -1;
            --sp;
          } else if (tc == TC_REFERENCE) {
            JS_NEED(4);
            int64_t k = (int64_t)s32() - 0x7E0000;
            if (k < 0 || k >= nh || handles[k] < 0) JS_FAIL;
            ret = handles[k];
            --sp;
          } else if (tc == TC_CLASSDESC) {
            JS_NEED(2);
            uint32_t l = u16();
            JS_NEED(l);
            uint8_t c0 = l > 0 ? (uint8_t)at(pos) : 0, c1 = l > 1 ? (uint8_t)at(pos + 1) : 0;
            pos += l;
            JS_NEED(8 + 1 + 2);
            pos += 8;  // serialVersionUID
            if (nd >= kMaxDescs) JS_FAIL;
            int di = nd++;
            JS_NEWHANDLE(di);
            descs[di].flags = (uint8_t)u8();
            descs[di].arr = (c0 == '[') ? c1 : 0;
            uint32_t cnt = u16();
            if (nf + cnt > (uint32_t)kMaxFields) JS_FAIL;
            descs[di].f0 = (uint8_t)nf;
            descs[di].nf = (uint8_t)cnt;
            descs[di].super = -1;
            f.d = (int16_t)di;
            f.i = 0;
            f.n = (int32_t)cnt;
            f.st = 1;
          } else if (tc == TC_PROXYCLASSDESC) {
            if (nd >= kMaxDescs) JS_FAIL;
            int di = nd++;
            JS_NEWHANDLE(di);
            descs[di].flags = SC_SERIALIZABLE;
            descs[di].arr = 0;
            descs[di].f0 = (uint8_t)nf;
            descs[di].nf = 0;
            descs[di].super = -1;
            JS_NEED(4);
            int32_t cnt = s32();
            if (cnt < 0) JS_FAIL;
            for (int32_t k = 0; k < cnt; ++k) {
              JS_NEED(2);
              uint32_t l = u16();
              JS_NEED(l);
              pos += l;
            }
            f.d = (int16_t)di;
            f.st = 2;
            JS_PUSH(K_ANNOT);
          } else {
            JS_FAIL;
          }
        } else if (f.st == 1) {  // field descriptors
          if (f.i < f.n) {
            JS_NEED(3);
            int t = u8();
            uint32_t l = u16();
            JS_NEED(l);
            pos += l;  // field name
            ftab[nf++] = (uint8_t)t;
            f.i++;
            if (t == 'L' || t == '[') {
              JS_PUSH(K_STROBJ);
            } else if (!(t == 'B' || t == 'C' || t == 'D' || t == 'F' || t == 'I' || t == 'J' || t == 'S' || t == 'Z')) {
              JS_FAIL;
            }
          } else {
            f.st = 2;
            JS_PUSH(K_ANNOT);  // classAnnotation
          }
        } else if (f.st == 2) {
          f.st = 3;
          JS_PUSH(K_DESC);  // superClassDesc
        } else {
          descs[f.d].super = (int8_t)ret;
          ret = f.d;
          --sp;
        }
        break;
      }
      case K_ODATA: {
        if (f.st == 0) {
          if (ret < 0) JS_FAIL;
          JS_NEWHANDLE(-1);
          f.d = (int16_t)ret;
          int n = 0;
          for (int c = ret; c >= 0; c = descs[c].super)
            if (++n > kMaxDescs) JS_FAIL;
          f.n = n;  // chain length
          f.i = 0;  // class index counted from the top-most superclass
          f.j = 0;  // field index within the class
          if (descs[f.d].flags & SC_EXTERNALIZABLE) {
            if (!(descs[f.d].flags & SC_BLOCK_DATA)) JS_FAIL;  // protocol-1 externalizable
            f.st = 2;
            JS_PUSH(K_ANNOT);
          } else {
            f.st = 1;
          }
        } else if (f.st == 1) {
          if (f.i >= f.n) {
            --sp;
            break;
          }
          int c = f.d;
          for (int k = 0; k < f.n - 1 - f.i; ++k) c = descs[c].super;
          const Desc& dc = descs[c];
          if (!(dc.flags & SC_SERIALIZABLE)) JS_FAIL;
          if (f.j < dc.nf) {
            int t = ftab[dc.f0 + f.j];
            f.j++;
            int sz = 0;
            switch (t) {
              case 'B': case 'Z': sz = 1; break;
              case 'C': case 'S': sz = 2; break;
              case 'I': case 'F': sz = 4; break;
              case 'J': case 'D': sz = 8; break;
              default: sz = -1; break;
            }
            if (sz > 0) {
              JS_NEED(sz);
              pos += sz;
            } else {
              JS_PUSH(K_OBJ);
            }
          } else {
            f.j = 0;
            f.i++;
            if (dc.flags & SC_WRITE_METHOD) JS_PUSH(K_ANNOT);  // custom data up to TC_ENDBLOCKDATA
          }
        } else {
          --sp;
        }
        break;
      }
      case K_ARR: {
        if (f.st == 0) {
          if (ret < 0) JS_FAIL;
          JS_NEWHANDLE(-1);
          JS_NEED(4);
          int32_t size = s32();
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
            uint64_t b = (uint64_t)(uint32_t)size * (uint64_t)es;
            if (b > avail - pos) JS_FAIL;
            pos += b;
            --sp;
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
            --sp;
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
#undef JS_NEWHANDLE
  return (int64_t)pos;
}

}  // namespace jser
}  // namespace clg
