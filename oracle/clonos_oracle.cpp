// clonos_oracle.cpp -- CPU ORACLE (test infrastructure only; see clonos_oracle.h).
//
// Sequential restatement of the reference Java on the causal-log hot path.  Every
// function cites the reference lines it follows.  R/ = /root/reference/flink-runtime/
// src/main/java/org/apache/flink/runtime/causal/.
#include "clonos_oracle.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// Big-endian ByteBuf accessors (Netty default byte order).
// ---------------------------------------------------------------------------
inline uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline uint64_t be64(const uint8_t* p) { return (uint64_t(be32(p)) << 32) | be32(p + 4); }
inline void put32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v >> 24); p[1] = uint8_t(v >> 16); p[2] = uint8_t(v >> 8); p[3] = uint8_t(v);
}
inline void put64(uint8_t* p, uint64_t v) { put32(p, uint32_t(v >> 32)); put32(p + 4, uint32_t(v)); }

// ---------------------------------------------------------------------------
// Java Object Serialization grammar walker (JDK 8 ObjectInputStream semantics,
// spec section 6.4).  Used for SERIALIZABLE determinants, whose payload is one
// ObjectOutputStream stream with no length prefix
// (R/determinant/SimpleDeterminantEncoder.java:316-341).  Recursive, unbounded
// containers: an independent implementation from the device walker.
// ---------------------------------------------------------------------------
enum : uint8_t {
  TC_NULL = 0x70, TC_REFERENCE = 0x71, TC_CLASSDESC = 0x72, TC_OBJECT = 0x73,
  TC_STRING = 0x74, TC_ARRAY = 0x75, TC_CLASS = 0x76, TC_BLOCKDATA = 0x77,
  TC_ENDBLOCKDATA = 0x78, TC_RESET = 0x79, TC_BLOCKDATALONG = 0x7A,
  TC_EXCEPTION = 0x7B, TC_LONGSTRING = 0x7C, TC_PROXYCLASSDESC = 0x7D, TC_ENUM = 0x7E
};
enum : uint8_t { SC_WRITE_METHOD = 0x01, SC_SERIALIZABLE = 0x02, SC_EXTERNALIZABLE = 0x04, SC_BLOCK_DATA = 0x08 };

struct JWalker {
  const uint8_t* b;
  size_t n;
  size_t pos = 0;
  int depth = 0;
  struct Field { char type; };
  struct Desc { std::string name; uint8_t flags = 0; std::vector<Field> fields; int super = -1; };
  std::vector<Desc> descs;
  // handle table: -2 = string, -1 = other object, >=0 = desc index
  std::vector<int> handles;

  bool need(size_t k) const { return pos + k <= n; }
  bool u8(uint8_t& v) { if (!need(1)) return false; v = b[pos++]; return true; }
  bool peek(uint8_t& v) const { if (!need(1)) return false; v = b[pos]; return true; }
  bool u16(uint32_t& v) { if (!need(2)) return false; v = (uint32_t(b[pos]) << 8) | b[pos + 1]; pos += 2; return true; }
  bool s32(int32_t& v) { if (!need(4)) return false; v = int32_t(be32(b + pos)); pos += 4; return true; }
  bool skip(uint64_t k) { if (k > n - pos) return false; pos += size_t(k); return true; }
  // Modified UTF-8 as JDK 8 reads it (ObjectInputStream.BlockDataInputStream.readUTFBody /
  // readUTFSpan): every unit 0xxxxxxx, 110xxxxx 10xxxxxx or 1110xxxx 10xxxxxx 10xxxxxx, none
  // cut by the length; anything else throws UTFDataFormatException.
  static bool mutf(const uint8_t* s, uint64_t len) {
    for (uint64_t i = 0; i < len;) {
      const uint8_t b1 = s[i];
      if (b1 < 0x80) { ++i; continue; }
      const uint64_t k = (b1 >> 5) == 6 ? 2 : (b1 >> 4) == 14 ? 3 : 0;
      if (!k || len - i < k) return false;
      for (uint64_t j = 1; j < k; ++j)
        if ((s[i + j] & 0xC0) != 0x80) return false;
      i += k;
    }
    return true;
  }
  bool utf(std::string* out) {  // readUTF
    uint32_t len;
    if (!u16(len) || !need(len) || !mutf(b + pos, len)) return false;
    if (out) out->assign(reinterpret_cast<const char*>(b + pos), len);
    pos += len;
    return true;
  }

  // classDesc: newClassDesc | nullReference | prevObject(desc).  *idx = -1 for null.
  bool classDesc(int* idx) {
    uint8_t tc;
    if (!u8(tc)) return false;
    if (tc == TC_NULL) { *idx = -1; return true; }
    if (tc == TC_REFERENCE) {
      int32_t h;
      if (!s32(h)) return false;
      int64_t k = int64_t(h) - 0x7E0000;
      if (k < 0 || k >= int64_t(handles.size()) || handles[size_t(k)] < 0) return false;
      *idx = handles[size_t(k)];
      return true;
    }
    if (tc == TC_CLASSDESC) {
      Desc d;
      if (!utf(&d.name)) return false;
      if (!skip(8)) return false;  // serialVersionUID
      int di = int(descs.size());
      descs.push_back(Desc());
      handles.push_back(di);  // newHandle assigned before classDescInfo (ObjectInputStream.readNonProxyDesc)
      if (!u8(d.flags)) return false;
      uint32_t nf;
      if (!u16(nf)) return false;
      for (uint32_t i = 0; i < nf; ++i) {
        uint8_t t;
        if (!u8(t)) return false;
        if (!utf(nullptr)) return false;  // field name
        switch (t) {
          case 'B': case 'C': case 'D': case 'F': case 'I': case 'J': case 'S': case 'Z': break;
          case 'L': case '[': {
            if (!stringObject()) return false;  // className1
            break;
          }
          default: return false;
        }
        d.fields.push_back(Field{char(t)});
      }
      if (!annotation()) return false;  // classAnnotation
      int sup;
      if (!classDesc(&sup)) return false;  // superClassDesc
      d.super = sup;
      descs[size_t(di)] = d;
      *idx = di;
      return true;
    }
    if (tc == TC_PROXYCLASSDESC) {
      Desc d;
      d.name = "<proxy>";
      d.flags = SC_SERIALIZABLE;
      int di = int(descs.size());
      descs.push_back(Desc());
      handles.push_back(di);
      int32_t cnt;
      if (!s32(cnt) || cnt < 0) return false;
      for (int32_t i = 0; i < cnt; ++i) if (!utf(nullptr)) return false;
      if (!annotation()) return false;
      int sup;
      if (!classDesc(&sup)) return false;
      d.super = sup;
      descs[size_t(di)] = d;
      *idx = di;
      return true;
    }
    return false;
  }

  // className1: (String)object -> TC_STRING / TC_LONGSTRING / TC_REFERENCE
  bool stringObject() {
    uint8_t tc;
    if (!peek(tc)) return false;
    if (tc == TC_STRING || tc == TC_LONGSTRING || tc == TC_REFERENCE) return object();
    return false;
  }

  // contents until TC_ENDBLOCKDATA (classAnnotation / objectAnnotation / skipCustomData)
  bool annotation() {
    for (;;) {
      uint8_t tc;
      if (!peek(tc)) return false;
      if (tc == TC_ENDBLOCKDATA) { pos++; return true; }
      if (tc == TC_BLOCKDATA) {
        uint8_t len; pos++;
        if (!u8(len) || !skip(len)) return false;
        continue;
      }
      if (tc == TC_BLOCKDATALONG) {
        int32_t len; pos++;
        if (!s32(len) || len < 0 || !skip(uint32_t(len))) return false;
        continue;
      }
      if (!object()) return false;
    }
  }

  bool fieldValues(const Desc& d) {
    for (const Field& f : d.fields) {
      switch (f.type) {
        case 'B': case 'Z': if (!skip(1)) return false; break;
        case 'C': case 'S': if (!skip(2)) return false; break;
        case 'I': case 'F': if (!skip(4)) return false; break;
        case 'J': case 'D': if (!skip(8)) return false; break;
        default: if (!object()) return false; break;
      }
    }
    return true;
  }

  bool object() {
    if (++depth > 512) return false;
    bool ok = objectInner();
    --depth;
    return ok;
  }

  bool objectInner() {
    uint8_t tc;
    for (;;) {  // readObject0 consumes leading TC_RESETs
      if (!u8(tc)) return false;
      if (tc != TC_RESET) break;
      handles.clear();
    }
    switch (tc) {
      case TC_NULL: return true;
      case TC_REFERENCE: {
        int32_t h;
        if (!s32(h)) return false;
        int64_t k = int64_t(h) - 0x7E0000;
        return k >= 0 && k < int64_t(handles.size());
      }
      case TC_STRING: {
        handles.push_back(-2);
        return utf(nullptr);
      }
      case TC_LONGSTRING: {
        handles.push_back(-2);
        if (!need(8)) return false;
        uint64_t len = be64(b + pos);
        pos += 8;
        return len <= n - pos && mutf(b + pos, len) && skip(len);  // readLongUTF
      }
      case TC_CLASSDESC: case TC_PROXYCLASSDESC: {
        pos--;
        int idx;
        return classDesc(&idx);
      }
      case TC_CLASS: {
        int idx;
        if (!classDesc(&idx)) return false;
        handles.push_back(-1);
        return true;
      }
      case TC_ENUM: {
        int idx;
        if (!classDesc(&idx)) return false;
        handles.push_back(-1);
        return stringObject();  // enumConstantName
      }
      case TC_ARRAY: {
        int idx;
        if (!classDesc(&idx) || idx < 0) return false;
        handles.push_back(-1);
        int32_t size;
        if (!s32(size) || size < 0) return false;
        const std::string nm = descs[size_t(idx)].name;
        if (nm.size() < 2 || nm[0] != '[') return false;
        uint64_t es;
        switch (nm[1]) {
          case 'B': case 'Z': es = 1; break;
          case 'C': case 'S': es = 2; break;
          case 'I': case 'F': es = 4; break;
          case 'J': case 'D': es = 8; break;
          case 'L': case '[': es = 0; break;
          default: return false;
        }
        if (es) return skip(es * uint64_t(uint32_t(size)));
        for (int32_t i = 0; i < size; ++i) if (!object()) return false;
        return true;
      }
      case TC_OBJECT: {
        int idx;
        if (!classDesc(&idx) || idx < 0) return false;
        handles.push_back(-1);
        // class hierarchy, top-most superclass first (ObjectStreamClass.getClassDataLayout)
        std::vector<int> chain;
        for (int c = idx; c >= 0; c = descs[size_t(c)].super) {
          chain.push_back(c);
          if (chain.size() > 256) return false;
        }
        const Desc top = descs[size_t(idx)];  // copies: nested parsing may grow `descs`
        if (top.flags & SC_EXTERNALIZABLE) {
          if (!(top.flags & SC_BLOCK_DATA)) return false;  // protocol-1 externalizable: length unknowable
          return annotation();
        }
        for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
          const Desc d = descs[size_t(*it)];
          if (!(d.flags & SC_SERIALIZABLE)) return false;
          if (!fieldValues(d)) return false;
          if (d.flags & SC_WRITE_METHOD)
            if (!annotation()) return false;  // custom data up to TC_ENDBLOCKDATA (skipCustomData)
        }
        return true;
      }
      default:
        return false;  // TC_EXCEPTION, block data at object position, garbage
    }
  }
};

int64_t jser_len(const uint8_t* p, size_t avail) {
  if (avail < 4 || p[0] != 0xAC || p[1] != 0xED || p[2] != 0x00 || p[3] != 0x05) return ORC_E_BAD_SERIAL;
  JWalker w;
  w.b = p;
  w.n = avail;
  w.pos = 4;
  if (!w.object()) return ORC_E_BAD_SERIAL;
  return int64_t(w.pos);
}

// ---------------------------------------------------------------------------
// decodeNext (R/determinant/SimpleDeterminantEncoder.java:78-93 and readers
// :116-341).  Error precedence follows the Java read order: a short read throws
// IndexOutOfBounds before any enum lookup; TimerTrigger looks up the enum before
// reading the name (:231); SourceCheckpoint reads the reference first and looks
// up CheckpointType last (:285).
// ---------------------------------------------------------------------------
struct Rec { uint32_t off; uint8_t tag; int64_t v0; bool wide; int32_t rc; int64_t v1; uint32_t var_off; uint32_t var_len; uint8_t sub; };

int decode_one(const uint8_t* b, size_t len, size_t pos, Rec* r, size_t* next) {
  const size_t avail = len - pos;
  const int8_t tag = int8_t(b[pos]);
  r->off = uint32_t(pos);
  r->tag = uint8_t(tag);
  r->wide = false;
  r->rc = 0; r->v1 = 0; r->var_off = 0; r->var_len = 0; r->sub = 0;
  switch (tag) {
    case 0:  // ORDER :120-121
      if (avail < 2) return ORC_E_TRUNCATED;
      r->v0 = int8_t(b[pos + 1]);
      *next = pos + 2;
      return ORC_OK;
    case 1:  // TIMESTAMP :142-143
      if (avail < 9) return ORC_E_TRUNCATED;
      r->v0 = int64_t(be64(b + pos + 1));
      *next = pos + 9;
      return ORC_OK;
    case 2:  // RNG :163-164
    case 7:  // BUFFER_BUILT :185-186
      if (avail < 5) return ORC_E_TRUNCATED;
      r->v0 = int32_t(be32(b + pos + 1));
      *next = pos + 5;
      return ORC_OK;
    case 4: {  // TIMER_TRIGGER :228-242
      if (avail < 14) return ORC_E_TRUNCATED;
      r->wide = true;
      r->rc = int32_t(be32(b + pos + 1));
      r->v0 = int64_t(be64(b + pos + 5));
      int8_t ord = int8_t(b[pos + 13]);
      if (ord < 0 || ord > 6) return ORC_E_BAD_ENUM;  // ProcessingTimeCallbackID.Type.values()[ord]
      r->sub = uint8_t(ord);
      if (ord == 6) {  // INTERNAL
        if (avail < 18) return ORC_E_TRUNCATED;
        int32_t nl = int32_t(be32(b + pos + 14));
        if (nl < 0) return ORC_E_NEG_LEN;
        if (avail - 18 < uint64_t(nl)) return ORC_E_TRUNCATED;
        r->var_off = uint32_t(pos + 18);
        r->var_len = uint32_t(nl);
        *next = pos + 18 + size_t(nl);
      } else {
        *next = pos + 14;
      }
      return ORC_OK;
    }
    case 5: {  // SOURCE_CHECKPOINT :273-287
      if (avail < 23) return ORC_E_TRUNCATED;
      r->wide = true;
      r->rc = int32_t(be32(b + pos + 1));
      r->v0 = int64_t(be64(b + pos + 5));
      r->v1 = int64_t(be64(b + pos + 13));
      int8_t ord = int8_t(b[pos + 21]);
      bool has_ref = b[pos + 22] != 0;  // readBoolean
      size_t end = pos + 23;
      if (has_ref) {
        if (avail < 27) return ORC_E_TRUNCATED;
        int32_t rl = int32_t(be32(b + pos + 23));
        if (rl < 0) return ORC_E_NEG_LEN;
        if (avail - 27 < uint64_t(rl)) return ORC_E_TRUNCATED;
        r->var_off = uint32_t(pos + 27);
        r->var_len = uint32_t(rl);
        end = pos + 27 + size_t(rl);
      }
      if (ord < 0 || ord > 1) return ORC_E_BAD_ENUM;  // CheckpointType.values()[typeOrd]
      r->sub = uint8_t(ord) | (has_ref ? 0x80 : 0);
      *next = end;
      return ORC_OK;
    }
    case 6:  // IGNORE_CHECKPOINT :309-313
      if (avail < 13) return ORC_E_TRUNCATED;
      r->wide = true;
      r->rc = int32_t(be32(b + pos + 1));
      r->v0 = int64_t(be64(b + pos + 5));
      *next = pos + 13;
      return ORC_OK;
    case 3: {  // SERIALIZABLE :333-341
      int64_t jl = jser_len(b + pos + 1, avail - 1);
      if (jl < 0) return ORC_E_BAD_SERIAL;
      r->wide = true;
      r->v0 = jl;
      r->var_off = uint32_t(pos + 1);
      r->var_len = uint32_t(jl);
      *next = pos + 1 + size_t(jl);
      return ORC_OK;
    }
    default:
      return ORC_E_CORRUPT_TAG;  // CorruptDeterminantArrayException(tag) :92
  }
}

// ---------------------------------------------------------------------------
// ThreadCausalLogImpl model (R/log/thread/ThreadCausalLogImpl.java:51-527) over a
// Netty CompositeByteBuf of fixed-size components.
// ---------------------------------------------------------------------------
struct EpochStart { int64_t id; int32_t offset; };
struct Consumer { std::shared_ptr<EpochStart> epoch_start; int32_t offset; };
struct ChKey {
  uint64_t lo, hi;
  bool operator<(const ChKey& o) const { return lo != o.lo ? lo < o.lo : hi < o.hi; }
};

}  // namespace

struct orc_log {
  uint32_t C;
  int32_t depth;
  std::vector<std::vector<uint8_t>> comps;  // composite components, each C bytes
  int32_t writer = 0;                        // visibleWriterIndex == composite writerIndex
  std::map<int64_t, std::shared_ptr<EpochStart>> epochs;
  std::map<ChKey, Consumer> consumers;

  int32_t capacity() const { return int32_t(comps.size()) * int32_t(C); }
  void add_component() { comps.emplace_back(C, uint8_t(0)); }  // addComponent :438-452
  void ensure(int32_t n) { while (capacity() - writer < n) add_component(); }  // notEnoughSpaceFor :351-353
  void write(const uint8_t* src, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) {
      int32_t p = writer + int32_t(i);
      comps[size_t(p) / C][size_t(p) % C] = src[i];
    }
    writer += int32_t(n);
  }
  void read(int32_t phys, uint32_t n, uint8_t* out) const {  // makeDeltaUnsafe :364-382
    for (uint32_t i = 0; i < n; ++i) {
      int32_t p = phys + int32_t(i);
      out[i] = comps[size_t(p) / C][size_t(p) % C];
    }
  }
  std::shared_ptr<EpochStart> compute_if_absent(int64_t e) {
    auto it = epochs.find(e);
    if (it != epochs.end()) return it->second;
    auto es = std::make_shared<EpochStart>(EpochStart{e, writer});
    epochs[e] = es;
    return es;
  }
  int32_t bytes_to_send(int64_t epoch, int32_t phys) const {  // computeNumberOfBytesToSend :384-395
    auto it = epochs.find(epoch + 1);
    return (it != epochs.end() ? it->second->offset : writer) - phys;
  }
};

extern "C" {

int64_t orc_encode(const orc_det* d, uint8_t* out, size_t cap) {
  // SimpleDeterminantEncoder.encodeTo :56-75 with per-type writers.
  size_t need;
  switch (d->tag) {
    case 0: need = 2; break;
    case 1: need = 9; break;
    case 2: case 7: need = 5; break;
    case 3: need = 1 + d->var_len; break;
    case 4: need = (d->sub == 6) ? 18 + d->var_len : 14; break;
    case 5: need = (d->sub & 0x80) ? 27 + d->var_len : 23; break;
    case 6: need = 13; break;
    default: return ORC_E_INVALID_ARG;
  }
  if (need > cap) return ORC_E_CAPACITY;
  out[0] = d->tag;
  switch (d->tag) {
    case 0: out[1] = uint8_t(d->v0); break;                        // :124-127
    case 1: put64(out + 1, uint64_t(d->v0)); break;                 // :145-148
    case 2: case 7: put32(out + 1, uint32_t(d->v0)); break;         // :167-170, :189-192
    case 3: if (d->var_len) memcpy(out + 1, d->var, d->var_len); break;  // :316-323
    case 4:                                                          // :202-213
      put32(out + 1, uint32_t(d->record_count));
      put64(out + 5, uint64_t(d->v0));
      out[13] = d->sub;
      if (d->sub == 6) { put32(out + 14, d->var_len); if (d->var_len) memcpy(out + 18, d->var, d->var_len); }
      break;
    case 5:                                                          // :244-257
      put32(out + 1, uint32_t(d->record_count));
      put64(out + 5, uint64_t(d->v0));
      put64(out + 13, uint64_t(d->v1));
      out[21] = d->sub & 0x7F;
      out[22] = (d->sub & 0x80) ? 1 : 0;
      if (d->sub & 0x80) { put32(out + 23, d->var_len); if (d->var_len) memcpy(out + 27, d->var, d->var_len); }
      break;
    case 6:                                                          // :289-293
      put32(out + 1, uint32_t(d->record_count));
      put64(out + 5, uint64_t(d->v0));
      break;
  }
  return int64_t(need);
}

int64_t orc_jser_len(const uint8_t* p, size_t avail) { return jser_len(p, avail); }

int orc_decode_span(const uint8_t* buf, size_t len, uint32_t* off, uint8_t* tag, int64_t* v0,
                    uint32_t* w_idx, int32_t* w_rc, int64_t* w_v1, uint32_t* w_var_off,
                    uint32_t* w_var_len, uint8_t* w_sub, size_t cap, size_t wcap,
                    size_t* n_rec, size_t* n_wide, int64_t* err_off, int32_t* err_tag) {
  size_t pos = 0, nr = 0, nw = 0;
  *err_off = -1;
  *err_tag = 0;
  while (pos < len) {  // decodeNext returns null when !isReadable (:81-82)
    Rec r;
    size_t next;
    int st = decode_one(buf, len, pos, &r, &next);
    if (st != ORC_OK) {
      *n_rec = nr; *n_wide = nw; *err_off = int64_t(pos); *err_tag = int8_t(buf[pos]);
      return st;
    }
    if (nr >= cap || (r.wide && nw >= wcap)) { *n_rec = nr; *n_wide = nw; return ORC_E_CAPACITY; }
    off[nr] = r.off; tag[nr] = r.tag; v0[nr] = r.v0;
    if (r.wide) {
      w_idx[nw] = uint32_t(nr); w_rc[nw] = r.rc; w_v1[nw] = r.v1;
      w_var_off[nw] = r.var_off; w_var_len[nw] = r.var_len; w_sub[nw] = r.sub;
      nw++;
    }
    nr++;
    pos = next;
  }
  *n_rec = nr; *n_wide = nw;
  return ORC_OK;
}

int orc_decode_count(const uint8_t* buf, size_t len, size_t* n_rec, size_t* n_wide) {
  size_t pos = 0, nr = 0, nw = 0;
  while (pos < len) {
    Rec r;
    size_t next;
    int st = decode_one(buf, len, pos, &r, &next);
    if (st != ORC_OK) { *n_rec = nr; *n_wide = nw; return st; }
    nr++;
    nw += r.wide;
    pos = next;
  }
  *n_rec = nr; *n_wide = nw;
  return ORC_OK;
}

// ------------------------------- log model ---------------------------------
orc_log* orc_log_new(uint32_t component_bytes, int32_t sharing_depth) {
  if (component_bytes == 0) return nullptr;
  orc_log* l = new orc_log();
  l->C = component_bytes;
  l->depth = sharing_depth;
  l->add_component();  // ctor :101-102
  return l;
}

void orc_log_free(orc_log* l) { delete l; }

int orc_log_append(orc_log* l, int64_t epoch, const uint8_t* bytes, uint32_t n) {
  if (l->depth == 0) return ORC_OK;  // :159-160
  l->compute_if_absent(epoch);       // :168
  l->ensure(int32_t(n));             // :169-170
  l->write(bytes, n);                // :171-172
  return ORC_OK;
}

int orc_log_upstream(orc_log* l, const uint8_t* delta, uint32_t n, int32_t off_from_epoch, int64_t epoch) {
  if (n == 0) return ORC_OK;  // :124
  auto es = l->compute_if_absent(epoch);                         // :127-128
  int32_t cur = l->writer - es->offset;                          // :130
  int32_t num_new = (off_from_epoch + int32_t(n)) - cur;         // :132
  if (num_new > 0) {
    l->ensure(num_new);  // :136-137 -- components are added before the reader index is set
    if (num_new > int32_t(n)) return ORC_E_GAP;  // delta.readerIndex(negative) -> IndexOutOfBounds (:143)
    l->write(delta + (n - uint32_t(num_new)), uint32_t(num_new));  // :143-146
  }
  return ORC_OK;
}

int orc_log_has_delta(orc_log* l, uint64_t lo, uint64_t hi, int64_t epoch, int* out) {
  *out = 0;
  if (l->depth == 0) return ORC_OK;  // :197-198
  auto it = l->epochs.find(epoch);
  if (it == l->epochs.end()) return ORC_OK;  // :202-208
  ChKey k{lo, hi};
  auto ci = l->consumers.find(k);
  if (ci == l->consumers.end())
    ci = l->consumers.emplace(k, Consumer{it->second, 0}).first;  // :210-211
  Consumer& c = ci->second;
  if (c.epoch_start->id != epoch) {                                // :213-226
    if (c.epoch_start->id > epoch) return ORC_E_CONSUMER_BACKWARDS;
    c.epoch_start = it->second;
    c.offset = 0;
  }
  int32_t phys = c.epoch_start->offset + c.offset;
  *out = l->bytes_to_send(epoch, phys) != 0;  // :228-236
  return ORC_OK;
}

int orc_log_offset(orc_log* l, uint64_t lo, uint64_t hi, int32_t* out) {
  auto ci = l->consumers.find(ChKey{lo, hi});
  if (ci == l->consumers.end()) return ORC_E_NO_CONSUMER;
  *out = ci->second.offset;
  return ORC_OK;
}

int orc_log_get_delta(orc_log* l, uint64_t lo, uint64_t hi, int64_t epoch, uint8_t* out, uint32_t cap, uint32_t* n) {
  *n = 0;
  auto ci = l->consumers.find(ChKey{lo, hi});
  if (ci == l->consumers.end()) return ORC_E_NO_CONSUMER;
  Consumer& c = ci->second;
  int32_t phys = c.epoch_start->offset + c.offset;       // :256
  int32_t nb = l->bytes_to_send(epoch, phys);            // :258
  if (nb < 0 || phys < 0 || phys + nb > l->capacity()) return ORC_E_STATE;
  if (uint32_t(nb) > cap) return ORC_E_CAPACITY;
  if (nb) l->read(phys, uint32_t(nb), out);              // :264-269
  c.offset += nb;                                        // :272
  *n = uint32_t(nb);
  return ORC_OK;
}

int orc_log_get_determinants(orc_log* l, int64_t start_epoch, uint8_t* out, uint32_t cap, uint32_t* n) {
  *n = 0;
  if (l->depth == 0) return ORC_OK;  // :286-287
  int32_t start = 0;
  auto it = l->epochs.find(start_epoch);
  if (it != l->epochs.end()) start = it->second->offset;                 // :294-296
  else if (!l->epochs.empty()) start = l->epochs.begin()->second->offset; // :297-301 (min key)
  int32_t nb = l->writer - start;
  if (nb < 0 || start < 0 || start + nb > l->capacity()) return ORC_E_STATE;  // makeDeltaUnsafe IOOBE
  if (uint32_t(nb) > cap) return ORC_E_CAPACITY;
  if (nb) l->read(start, uint32_t(nb), out);
  *n = uint32_t(nb);
  return ORC_OK;
}

int orc_log_length(orc_log* l, int32_t* out) {  // :180-192
  *out = l->epochs.empty() ? l->writer : l->writer - l->epochs.begin()->second->offset;
  return ORC_OK;
}

int orc_log_checkpoint_complete(orc_log* l, int64_t cp) {  // :398-435
  auto following = l->compute_if_absent(cp);
  for (auto it = l->epochs.begin(); it != l->epochs.end();) {
    if (it->first < cp) it = l->epochs.erase(it); else ++it;
  }
  int32_t R = following->offset;
  if (R < 0 || R > l->writer) return ORC_E_STATE;  // buf.readerIndex(R) bounds check
  // Netty 4.1.24 CompositeByteBuf.discardReadComponents (pinned by NettyTests.java:173-175):
  //  * readerIndex == 0                      -> nothing removed
  //  * readerIndex == writerIndex == capacity -> every component removed, indexes reset to 0
  //  * otherwise                              -> components wholly before readerIndex removed
  int32_t move = 0;
  if (R != 0) {
    if (R == l->writer && l->writer == l->capacity()) {
      move = R;
      l->comps.clear();
    } else {
      int32_t first = R / int32_t(l->C);  // toComponentIndex(readerIndex)
      l->comps.erase(l->comps.begin(), l->comps.begin() + first);
      move = first * int32_t(l->C);
    }
  }
  for (auto& e : l->epochs) e.second->offset -= move;  // :422-430 (stale consumer refs untouched)
  l->writer -= move;                                   // :431
  return ORC_OK;
}

int orc_log_unregister(orc_log* l, uint64_t lo, uint64_t hi) {
  l->consumers.erase(ChKey{lo, hi});
  return ORC_OK;
}

int orc_log_state(orc_log* l, int32_t* writer, int32_t* capacity, int32_t* n_components,
                  int64_t* epoch_ids, int32_t* epoch_offs, int32_t cap_epochs, int32_t* n_epochs) {
  *writer = l->writer;
  *capacity = l->capacity();
  *n_components = int32_t(l->comps.size());
  int32_t i = 0;
  for (auto& e : l->epochs) {
    if (i < cap_epochs) { epoch_ids[i] = e.first; epoch_offs[i] = e.second->offset; }
    i++;
  }
  *n_epochs = i;
  return i > cap_epochs ? ORC_E_CAPACITY : ORC_OK;
}

int orc_log_consumer(orc_log* l, uint64_t lo, uint64_t hi, int* exists, int64_t* epoch, int32_t* offset) {
  auto ci = l->consumers.find(ChKey{lo, hi});
  *exists = ci != l->consumers.end();
  if (*exists) { *epoch = ci->second.epoch_start->id; *offset = ci->second.offset; }
  return ORC_OK;
}

int orc_log_read_phys(orc_log* l, int32_t phys, uint32_t n, uint8_t* out) {
  if (phys < 0 || int64_t(phys) + n > l->capacity()) return ORC_E_STATE;
  l->read(phys, n, out);
  return ORC_OK;
}

// ----------------------------- CPU baseline ---------------------------------
int64_t orc_bench_decode(const uint8_t* buf, const uint64_t* span_off, const uint64_t* span_len,
                         uint32_t n_spans, uint32_t threads) {
  if (threads == 0) threads = 1;
  std::vector<int64_t> counts(threads, 0);
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < threads; ++t) {
    pool.emplace_back([&, t]() {
      // SoA outputs sized for the largest span this thread owns, allocated once per thread
      // and not zero-filled (the decode writes every row it reports): the timed work is the
      // decodeNext loop, not page-faulting output buffers in.
      size_t maxlen = 0;
      for (uint32_t s = t; s < n_spans; s += threads) maxlen = std::max<size_t>(maxlen, span_len[s]);
      size_t cap = maxlen / 2 + 1;
      std::unique_ptr<uint32_t[]> off(new uint32_t[cap]), w_idx(new uint32_t[cap]), w_var_off(new uint32_t[cap]),
          w_var_len(new uint32_t[cap]);
      std::unique_ptr<uint8_t[]> tag(new uint8_t[cap]), w_sub(new uint8_t[cap]);
      std::unique_ptr<int64_t[]> v0(new int64_t[cap]), w_v1(new int64_t[cap]);
      std::unique_ptr<int32_t[]> w_rc(new int32_t[cap]);
      for (uint32_t s = t; s < n_spans; s += threads) {
        size_t nr = 0, nw = 0;
        int64_t eo;
        int32_t et;
        orc_decode_span(buf + span_off[s], span_len[s], off.get(), tag.get(), v0.get(), w_idx.get(), w_rc.get(),
                        w_v1.get(), w_var_off.get(), w_var_len.get(), w_sub.get(), cap, cap, &nr, &nw, &eo, &et);
        counts[t] += int64_t(nr);
      }
    });
  }
  for (auto& th : pool) th.join();
  int64_t total = 0;
  for (auto c : counts) total += c;
  return total;
}

int64_t orc_bench_slice(const uint8_t* buf, const uint64_t* src_off, const uint64_t* len,
                        const uint64_t* dst_off, uint32_t n_req, uint8_t* out, uint32_t threads) {
  if (threads == 0) threads = 1;
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < threads; ++t) {
    pool.emplace_back([&, t]() {
      for (uint32_t r = t; r < n_req; r += threads) memcpy(out + dst_off[r], buf + src_off[r], len[r]);
    });
  }
  for (auto& th : pool) th.join();
  int64_t total = 0;
  for (uint32_t r = 0; r < n_req; ++r) total += int64_t(len[r]);
  return total;
}

}  // extern "C"
