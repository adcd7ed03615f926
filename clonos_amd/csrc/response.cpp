// response.cpp -- DeterminantResponseEvent wire format and merge (host side of replay-prep).
//
// Reference (R/ = flink-runtime/src/main/java/org/apache/flink/runtime/causal/):
//   R/DeterminantResponseEvent.java:93-107   write    :109-125 read    :128-148 merge
//   R/log/job/CausalLogID.java:128-186       equals / hashCode / write / read
// The event's map is a java.util.HashMap (JDK 8); its iteration order decides the wire
// order of write().  We keep the entries in that order: buckets ascending, each bucket in
// insertion order (bins append at the tail; resize splits a bin keeping relative order),
// so iteration order under a larger table is a stable sort by the new bucket index.
// Tree bins (9+ colliding ids in a table >= 64) order by identity hash codes in the JVM and
// cannot be reproduced; such maps keep the same content in bucket order here.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/clonos_engine.h"

namespace clg_internal {
int set_error(int code, const char* msg);
}

namespace {

using clg_internal::set_error;

bool id_equal(const clg_causal_log_id& a, const clg_causal_log_id& b) {  // CausalLogID.equals :128-149
  if (a.vertex_id != b.vertex_id) return false;
  if ((a.is_main != 0) != (b.is_main != 0)) return false;
  if (a.is_main) return true;
  return a.irp_upper == b.irp_upper && a.irp_lower == b.irp_lower && a.subpartition == b.subpartition;
}

int32_t id_hash(const clg_causal_log_id& id) {  // CausalLogID.hashCode :151-163 (Java int wrap-around)
  uint32_t h = 17;
  h = 31u * h + uint32_t(int32_t(id.vertex_id));
  h = 31u * h + (id.is_main ? 1u : 0u);
  if (id.is_main) return int32_t(h);
  const uint64_t lo = uint64_t(id.irp_lower), up = uint64_t(id.irp_upper);
  h = 31u * h + uint32_t(lo ^ (lo >> 32));
  h = 31u * h + uint32_t(up ^ (up >> 32));
  h = 31u * h + uint32_t(int32_t(id.subpartition));
  return int32_t(h);
}

uint32_t bucket(const clg_causal_log_id& id, uint32_t cap) {  // HashMap.hash + (n - 1) & hash
  const uint32_t h = uint32_t(id_hash(id));
  return (h ^ (h >> 16)) & (cap - 1);
}

void rehash(clg_response* r) {  // HashMap.resize, expressed on the iteration-ordered array
  std::vector<clg_response_entry> tmp(r->entries, r->entries + r->n);
  std::vector<uint32_t> b(r->n);
  for (uint32_t i = 0; i < r->n; ++i) b[i] = bucket(tmp[i].id, r->table_cap);
  std::vector<uint32_t> idx(r->n);
  for (uint32_t i = 0; i < r->n; ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return b[x] < b[y]; });
  for (uint32_t i = 0; i < r->n; ++i) r->entries[i] = tmp[idx[i]];
}

int find(const clg_response* r, const clg_causal_log_id& id) {
  for (uint32_t i = 0; i < r->n; ++i)
    if (id_equal(r->entries[i].id, id)) return int(i);
  return -1;
}

// HashMap.putVal for a key known to be absent: append at its bin's tail, then the two
// resize triggers (treeifyBin on a table < 64 when the bin reaches 9 nodes; size > 0.75 cap).
void insert_new(clg_response* r, const clg_response_entry& e) {
  if (r->table_cap == 0) r->table_cap = 16;
  const uint32_t b = bucket(e.id, r->table_cap);
  uint32_t pos = r->n, in_bin = 0;
  for (uint32_t i = 0; i < r->n; ++i) {
    const uint32_t bi = bucket(r->entries[i].id, r->table_cap);
    if (bi == b) ++in_bin;
    if (bi > b) {
      pos = i;
      break;
    }
  }
  std::memmove(r->entries + pos + 1, r->entries + pos, sizeof(clg_response_entry) * (r->n - pos));
  r->entries[pos] = e;
  r->n += 1;
  if (in_bin + 1 >= 9 && r->table_cap < 64) {  // TREEIFY_THRESHOLD, MIN_TREEIFY_CAPACITY
    r->table_cap *= 2;
    rehash(r);
  }
  if (uint64_t(r->n) * 4 > uint64_t(r->table_cap) * 3) {  // ++size > threshold (0.75)
    r->table_cap *= 2;
    rehash(r);
  }
}

clg_causal_log_id norm(const clg_causal_log_id& id) {
  clg_causal_log_id k{};
  k.vertex_id = id.vertex_id;
  k.is_main = id.is_main ? 1 : 0;
  if (!id.is_main) {
    k.irp_lower = id.irp_lower;
    k.irp_upper = id.irp_upper;
    k.subpartition = id.subpartition;
  }
  return k;
}

inline void put16(uint8_t* p, uint16_t v) { p[0] = uint8_t(v >> 8); p[1] = uint8_t(v); }
inline void put32(uint8_t* p, uint32_t v) { put16(p, uint16_t(v >> 16)); put16(p + 2, uint16_t(v)); }
inline void put64(uint8_t* p, uint64_t v) { put32(p, uint32_t(v >> 32)); put32(p + 4, uint32_t(v)); }
inline uint32_t be32(const uint8_t* p) { return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | p[3]; }
inline uint64_t be64(const uint8_t* p) { return uint64_t(be32(p)) << 32 | be32(p + 4); }

uint32_t id_wire_size(const clg_causal_log_id& id) { return id.is_main ? 3u : 20u; }

}  // namespace

extern "C" {

int32_t clg_causal_log_id_hash(const clg_causal_log_id* id) { return id ? id_hash(*id) : 0; }

int clg_response_put(clg_response* r, const clg_causal_log_id* id, const uint8_t* bytes, uint64_t len) {
  if (!r || !id || (len && !bytes)) return set_error(CLG_E_INVALID_ARG, "null argument");
  const clg_causal_log_id k = norm(*id);
  const int i = find(r, k);
  if (i >= 0) {  // HashMap.put on an existing key replaces the value in place
    r->entries[i].bytes = bytes;
    r->entries[i].len = len;
    return CLG_OK;
  }
  if (r->n >= r->cap || !r->entries) return set_error(CLG_E_CAPACITY, "response entry capacity exceeded");
  insert_new(r, clg_response_entry{k, bytes, len});
  return CLG_OK;
}

// n puts in order, in O((size + n) log) instead of one linear find and bin scan per put (a
// failed task's response holds 129 logs at p = 128; one by one they cost ~0.6 us each).
// The result is the sequential puts' exactly: keys already present (or put twice) have their
// value replaced in place; the table capacity follows HashMap's two resize triggers put by
// put (bin counts kept per bucket); and since a resize splits every bin keeping its order and
// a new key goes to its bin's tail, the final iteration order is the stable sort, by bucket
// under the final capacity, of the old order followed by the new keys in put order.  A batch
// that would pass the entry capacity runs the puts one by one (same partial result, same error).
int clg_response_put_batch(clg_response* r, const clg_causal_log_id* ids, const uint8_t* const* bytes,
                           const uint64_t* lens, uint32_t n) {
  if (n && (!ids || !bytes || !lens)) return set_error(CLG_E_INVALID_ARG, "null argument");
  if (!r) return set_error(CLG_E_INVALID_ARG, "null argument");
  if (n < 8) {
    for (uint32_t i = 0; i < n; ++i) {
      const int st = clg_response_put(r, &ids[i], bytes[i], lens[i]);
      if (st != CLG_OK) return st;
    }
    return CLG_OK;
  }
  // the distinct keys: old entries, then new keys in first-put order; a later put of a key
  // replaces its value (found by sorting (hash, position) -- no per-key allocations)
  const uint32_t n0 = r->n;
  std::vector<clg_response_entry> all(r->entries, r->entries + n0);
  all.reserve(size_t(n0) + n);
  for (uint32_t i = 0; i < n; ++i) {
    if (lens[i] && !bytes[i]) return set_error(CLG_E_INVALID_ARG, "null argument");
    all.push_back(clg_response_entry{norm(ids[i]), bytes[i], lens[i]});
  }
  std::vector<uint64_t> key(all.size());  // hash << 32 | position
  for (size_t j = 0; j < all.size(); ++j) key[j] = uint64_t(uint32_t(id_hash(all[j].id))) << 32 | uint32_t(j);
  std::sort(key.begin(), key.end());
  std::vector<uint32_t> owner(all.size());  // position -> the first position holding its key
  for (size_t j = 0; j < all.size(); ++j) owner[j] = uint32_t(j);
  for (size_t j = 0; j < key.size();) {  // runs of equal hashes: first-occurrence per key
    size_t e = j + 1;
    while (e < key.size() && (key[e] >> 32) == (key[j] >> 32)) ++e;
    for (size_t x = j + 1; x < e; ++x)
      for (size_t y = j; y < x; ++y) {
        const uint32_t px = uint32_t(key[x]), py = uint32_t(key[y]);
        if (owner[py] == py && id_equal(all[px].id, all[py].id)) {
          owner[px] = py;
          break;
        }
      }
    j = e;
  }
  std::vector<clg_response_entry> uniq;
  uniq.reserve(all.size());
  std::vector<uint32_t> slot(all.size());
  for (size_t j = 0; j < all.size(); ++j) {
    if (owner[j] == j) {
      slot[j] = uint32_t(uniq.size());
      uniq.push_back(all[j]);
    } else {  // put again: the value replaced in place
      uniq[slot[owner[j]]].bytes = all[j].bytes;
      uniq[slot[owner[j]]].len = all[j].len;
    }
  }
  all.swap(uniq);
  if (all.size() == n0) {  // replacements only: values in place, order and capacity unchanged
    for (uint32_t j = 0; j < n0; ++j) r->entries[j] = all[j];
    return CLG_OK;
  }
  if (all.size() > r->cap || !r->entries) {  // the capacity error, at the same put as one by one
    for (uint32_t i = 0; i < n; ++i) {
      const int st = clg_response_put(r, &ids[i], bytes[i], lens[i]);
      if (st != CLG_OK) return st;
    }
    return CLG_OK;
  }
  // the capacity, insertion by insertion (insert_new's triggers)
  uint32_t cap = r->table_cap ? r->table_cap : 16;
  std::vector<uint32_t> cnt(cap, 0);
  auto recount = [&](size_t upto) {
    cnt.assign(cap, 0);
    for (size_t j = 0; j < upto; ++j) ++cnt[bucket(all[j].id, cap)];
  };
  recount(n0);
  for (size_t j = n0; j < all.size(); ++j) {
    const uint32_t in_bin = cnt[bucket(all[j].id, cap)]++;
    const uint64_t size = j + 1;
    if (in_bin + 1 >= 9 && cap < 64) {  // TREEIFY_THRESHOLD, MIN_TREEIFY_CAPACITY
      cap *= 2;
      recount(j + 1);
    }
    if (size * 4 > uint64_t(cap) * 3) {  // ++size > threshold (0.75)
      cap *= 2;
      recount(j + 1);
    }
  }
  r->table_cap = cap;
  std::vector<uint32_t> b(all.size()), idx(all.size());
  for (size_t j = 0; j < all.size(); ++j) {
    b[j] = bucket(all[j].id, cap);
    idx[j] = uint32_t(j);
  }
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return b[x] < b[y]; });
  for (size_t j = 0; j < all.size(); ++j) r->entries[j] = all[idx[j]];
  r->n = uint32_t(all.size());
  return CLG_OK;
}

int clg_response_write(const clg_response* r, uint8_t* out, uint64_t cap, uint64_t* n_out) {
  if (!r || !n_out || (r->n && !r->entries)) return set_error(CLG_E_INVALID_ARG, "null argument");
  uint64_t need = 12;  // found (1) | vertexID (2) | correlationID (8) | size (1)
  for (uint32_t i = 0; i < r->n; ++i) need += id_wire_size(r->entries[i].id) + 4 + r->entries[i].len;
  *n_out = need;
  if (need > cap || !out) return set_error(CLG_E_CAPACITY, "output too small for the response (required size in *n_out)");
  for (uint32_t i = 0; i < r->n; ++i)
    if (r->entries[i].len > 0x7FFFFFFFull) return set_error(CLG_E_INVALID_ARG, "buffer over 2^31-1 bytes");
  uint8_t* p = out;
  *p++ = r->found ? 1 : 0;
  put16(p, uint16_t(r->vertex_id));
  p += 2;
  put64(p, uint64_t(r->correlation_id));
  p += 8;
  *p++ = uint8_t(r->n);  // writeByte(size): the low 8 bits
  for (uint32_t i = 0; i < r->n; ++i) {
    const clg_response_entry& e = r->entries[i];
    put16(p, uint16_t(e.id.vertex_id));  // CausalLogID.write :165-174
    p[2] = e.id.is_main ? 1 : 0;
    p += 3;
    if (!e.id.is_main) {
      put64(p, uint64_t(e.id.irp_lower));
      put64(p + 8, uint64_t(e.id.irp_upper));
      p[16] = uint8_t(e.id.subpartition);
      p += 17;
    }
    put32(p, uint32_t(e.len));
    p += 4;
    if (e.len) std::memcpy(p, e.bytes, e.len);
    p += e.len;
  }
  return CLG_OK;
}

int clg_response_read(const uint8_t* in, uint64_t n, clg_response* r, uint64_t* consumed) {
  if (!r || (n && !in)) return set_error(CLG_E_INVALID_ARG, "null argument");
  if (n < 12) return set_error(CLG_E_TRUNCATED, "response header truncated");
  r->found = in[0] != 0 ? 1 : 0;
  r->vertex_id = int16_t(uint16_t(in[1]) << 8 | in[2]);
  r->correlation_id = int64_t(be64(in + 3));
  const int count = int(int8_t(in[11]));  // readByte is signed: 128..255 entries read as none
  r->n = 0;
  r->table_cap = 16;
  uint64_t p = 12;
  for (int i = 0; i < count; ++i) {
    clg_causal_log_id id{};
    if (p + 3 > n) return set_error(CLG_E_TRUNCATED, "CausalLogID truncated");
    id.vertex_id = int16_t(uint16_t(in[p]) << 8 | in[p + 1]);
    id.is_main = in[p + 2] != 0 ? 1 : 0;
    p += 3;
    if (!id.is_main) {
      if (p + 17 > n) return set_error(CLG_E_TRUNCATED, "CausalLogID truncated");
      id.irp_lower = int64_t(be64(in + p));
      id.irp_upper = int64_t(be64(in + p + 8));
      id.subpartition = int8_t(in[p + 16]);
      p += 17;
    }
    if (p + 4 > n) return set_error(CLG_E_TRUNCATED, "buffer length truncated");
    const int32_t len = int32_t(be32(in + p));
    p += 4;
    if (len < 0) return set_error(CLG_E_NEG_LEN, "negative buffer length");  // new byte[len]
    if (p + uint64_t(len) > n) return set_error(CLG_E_TRUNCATED, "buffer truncated");
    const int st = clg_response_put(r, &id, in + p, uint64_t(len));
    if (st != CLG_OK) return st;
    p += uint64_t(len);
  }
  if (consumed) *consumed = p;
  return CLG_OK;
}

int clg_response_merge(clg_response* acc, const clg_response* other) {
  if (!acc || !other || (other->n && !other->entries)) return set_error(CLG_E_INVALID_ARG, "null argument");
  if (!acc->found && !other->found) return CLG_OK;  // :130-131
  uint32_t fresh = 0;
  for (uint32_t i = 0; i < other->n; ++i) fresh += find(acc, other->entries[i].id) < 0 ? 1u : 0u;
  if (acc->n + fresh > acc->cap || (fresh && !acc->entries))
    return set_error(CLG_E_CAPACITY, "response entry capacity exceeded");
  acc->found = 1;  // :133-134
  for (uint32_t i = 0; i < other->n; ++i) {  // Map.merge over other's entrySet, iteration order
    const clg_response_entry& v2 = other->entries[i];
    const int j = find(acc, v2.id);
    if (j < 0) {
      insert_new(acc, v2);
    } else if (!(acc->entries[j].len > v2.len)) {  // v1 kept only if strictly longer
      acc->entries[j].bytes = v2.bytes;
      acc->entries[j].len = v2.len;
    }
  }
  return CLG_OK;
}

}  // extern "C"
