// replay.hip -- gfx950 kernels of replay preparation (ReplayingState.java:108-214).
//
//  * k_bufsizes           BufferBuilt sizes of the subpartition recovery buffers
//                         (SubpartitionRecoveryThread.run :161-188: decodeNext in a loop,
//                         anything but a BufferBuilt determinant is an error)
//  * k_bufsizes_classify  the status that loop hits first, per buffer
//
// A well-formed recovery buffer is a run of 5-byte records [07][bytes i32 BE], so record
// k starts at 5k and every record is independent: one thread per record, coalesced byte
// loads, one i32 store.  HBM-bound: 5 B read + 4 B written per record.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/clonos_engine.h"
#include "dev_slow.h"
#include "kernels.h"

namespace clg {

constexpr uint32_t kBufThreads = 256;

__global__ __launch_bounds__(kBufThreads) void k_bufsizes(const BufChunk* __restrict__ chunks,
                                                          const BufSpan* __restrict__ spans,
                                                          int32_t* __restrict__ sizes,
                                                          unsigned long long* __restrict__ first_bad) {
  const BufChunk c = chunks[blockIdx.x];
  const BufSpan s = spans[c.span];
  const uint64_t k = c.k0 + threadIdx.x;
  if (k >= c.k1) return;
  const uint64_t p = 5 * k;
  const uint8_t* b = s.src + p;
  bool ok = p + 5 <= s.len && b[0] == CLG_TAG_BUFFER_BUILT;
  if (ok) {
    const uint32_t v = (uint32_t)b[1] << 24 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 8 | (uint32_t)b[4];
    sizes[s.out_base + k] = (int32_t)v;
  } else {
    atomicMin(first_bad + c.span, (unsigned long long)k);
  }
}

struct GBytes {  // bytes of a record start through the span end
  const uint8_t* p;
  uint64_t n;
  JArena ar;
  __device__ __forceinline__ int operator()(uint64_t k) const { return k < n ? (int)p[k] : 0; }
  __device__ __forceinline__ JArena arena() const { return ar; }
};

__global__ void k_bufsizes_classify(const BufSpan* __restrict__ spans, uint32_t n_spans,
                                    const uint64_t* __restrict__ first_bad, uint64_t* __restrict__ count,
                                    int32_t* __restrict__ status, int64_t* __restrict__ err_off,
                                    int32_t* __restrict__ err_tag, JArena ar) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_spans) return;
  const BufSpan s = spans[i];
  const uint64_t k = first_bad[i];
  const uint64_t n_full = s.len / 5;
  if (k == ~0ull || 5 * k >= s.len) {  // every record is a BufferBuilt, none left over
    count[i] = k == ~0ull ? n_full : k;
    status[i] = CLG_OK;
    err_off[i] = -1;
    err_tag[i] = -1;
    return;
  }
  const uint64_t p = 5 * k;
  count[i] = k;
  GBytes b{s.src + p, s.len - p, ar};
  const int tag = (int8_t)s.src[p];
  err_off[i] = (int64_t)p;
  err_tag[i] = tag;
  // decodeNext first (its exceptions win), then the instanceof check (:172)
  const int64_t L = rec_len_slow(b, s.len - p);
  status[i] = L < 0 ? (int32_t)L : (tag == CLG_TAG_BUFFER_BUILT ? CLG_E_STATE : CLG_E_NOT_BUFFER_BUILT);
}

int launch_bufsizes(const BufChunk* d_chunks, uint32_t n_chunks, const BufSpan* d_spans, int32_t* d_sizes,
                    uint64_t* d_first_bad, void* stream) {
  if (!n_chunks) return CLG_OK;
  hipLaunchKernelGGL(k_bufsizes, dim3(n_chunks), dim3(kBufThreads), 0, (hipStream_t)stream, d_chunks, d_spans,
                     d_sizes, reinterpret_cast<unsigned long long*>(d_first_bad));
  return launch_status(hipGetLastError());
}

int launch_bufsizes_classify(const BufSpan* d_spans, uint32_t n_spans, const uint64_t* d_first_bad,
                             uint64_t* d_count, int32_t* d_status, int64_t* d_err_off, int32_t* d_err_tag,
                             JArena ar, void* stream) {
  if (!n_spans) return CLG_OK;
  hipLaunchKernelGGL(k_bufsizes_classify, dim3((n_spans + 63) / 64), dim3(64), 0, (hipStream_t)stream, d_spans,
                     n_spans, d_first_bad, d_count, d_status, d_err_off, d_err_tag, ar);
  return launch_status(hipGetLastError());
}

}  // namespace clg
