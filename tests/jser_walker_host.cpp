// jser_walker_host.cpp -- the device Serializable stream walker (clonos_amd/csrc/
// jser_device.h), compiled for the host so CPU tests can hold it against the oracle and
// the reference-held JDK streams (tests/test_jser_reference.py).  Test infrastructure:
// the same source the GPU kernels instantiate, with a host spill allocator.
#include <stdint.h>
#include <stdlib.h>

#include <vector>

#include "../clonos_amd/csrc/jser_device.h"
#include "../clonos_amd/csrc/jser_flat.h"

namespace {
uint64_t g_backwards = 0;  // reads before an earlier one: the device readers' cursors only go forwards
struct HostBytes {
  const uint8_t* p;
  uint64_t hi = 0;
  int operator()(uint64_t k) {
    if (k < hi) ++g_backwards;
    hi = k > hi ? k : hi;
    return p[k];
  }
};
struct HostArena {  // bump allocator over a fixed buffer, like the device arena
  uint8_t* base;
  uint64_t cap;
  uint64_t* used;
  void* take(uint64_t bytes) const {
    bytes = (bytes + 15) & ~uint64_t(15);
    const uint64_t o = *used;
    *used += bytes;
    return o + bytes <= cap ? base + o : nullptr;
  }
};
}  // namespace

// Stream length of p[0, n) (magic first), -1 invalid, -2 spill arena of `arena_bytes`
// full; *spilled = arena bytes the walk took.
extern "C" int64_t walker_stream_len(const uint8_t* p, uint64_t n, uint64_t arena_bytes, uint64_t* spilled) {
  std::vector<uint8_t> buf(arena_bytes + 16);
  uint64_t used = 0;
  HostArena ar{reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(buf.data()) + 15) & ~uintptr_t(15)),
               arena_bytes, &used};
  HostBytes at{p};
  const int64_t r = clg::jser::stream_len(at, n, ar);
  if (spilled) *spilled = used;
  return r;
}

// The inline flat-object length (clonos_amd/csrc/jser_flat.h) of the record rec[0, n) (tag
// byte first): the record length, or 0 (another shape, or the stream does not end in n).
extern "C" uint32_t flat_record_len(const uint8_t* rec, uint32_t n) {
  auto rd4 = [rec, n](uint32_t q) -> uint32_t {
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; ++k)
      if (q + k < n) v |= uint32_t(rec[q + k]) << (8 * k);
    return v;
  };
  return clg::jser_flat_len_t(rd4, 0u, n);
}

// Reads the walker made at an offset before an earlier read's, since the library loaded (the
// device readers step through the span's tiles forwards only: such a read is out of bounds).
extern "C" uint64_t walker_backward_reads() { return g_backwards; }
