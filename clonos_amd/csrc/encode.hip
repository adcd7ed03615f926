// encode.hip -- batched determinant encode on gfx950 (the inverse of the decode).
//
// SimpleDeterminantEncoder.encodeTo (reference flink-runtime causal/determinant/
// SimpleDeterminantEncoder.java:56-75) with the per-type writers :124-323, applied to a
// whole batch given in the decode's SoA layout (clg_decoded): tag / v0 per record, a
// side-table row per wide record (tags 3-6) and a byte pool for the variable payloads
// (TimerTrigger names, SourceCheckpoint storage references, Serializable streams).
//
//  * k_enc_sums   per block of kEncBlock records: wide records (side rows are in order)
//  * k_enc_scan   one workgroup: exclusive prefix of the wide counts
//  * k_enc_bytes  per block: record lengths (validating tags and side rows) -> bytes
//  * k_enc_scan64 one workgroup: exclusive prefix of the block bytes
//  * k_enc_write  per block: record lengths -> LDS scan -> records assembled in LDS
//                 (big-endian fields) -> coalesced byte stores; blocks whose bytes do not
//                 fit the LDS buffer (long payloads) store directly
// Memory-bound: reads 9 B per record (+ 25 B per wide record and the payloads), writes
// the encoded bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/clonos_engine.h"
#include "kernels.h"

namespace clg {

constexpr uint32_t kEncThreads = 256;
constexpr uint32_t kEncPer = 4;                       // records per thread
constexpr uint32_t kEncBlock = kEncThreads * kEncPer;  // 1024
constexpr uint32_t kEncLds = 28 * 1024;               // staged output bytes per block

__device__ __forceinline__ bool enc_wide(uint32_t tg) { return tg - 3u < 4u; }

// Encoded length of record i (w: its side-table row, valid for wide records).
__device__ __forceinline__ uint64_t enc_len(const EncodeIn& in, uint32_t tg, uint64_t w) {
  switch (tg) {
    case CLG_TAG_ORDER: return 2;
    case CLG_TAG_TIMESTAMP: return 9;
    case CLG_TAG_RNG:
    case CLG_TAG_BUFFER_BUILT: return 5;
    case CLG_TAG_IGNORE_CHECKPOINT: return 13;
    case CLG_TAG_TIMER_TRIGGER: return in.w_sub[w] == 6 ? 18ull + in.w_var_len[w] : 14ull;
    case CLG_TAG_SOURCE_CHECKPOINT: return (in.w_sub[w] & 0x80u) ? 27ull + in.w_var_len[w] : 23ull;
    case CLG_TAG_SERIALIZABLE: return 1ull + in.w_var_len[w];
    default: return 0;  // invalid tag: flagged by k_enc_sums
  }
}

// Wide records per block (their side-table rows are consecutive, in record order).
__global__ __launch_bounds__(kEncThreads) void k_enc_sums(EncodeIn in, uint32_t* __restrict__ wsum) {
  __shared__ uint32_t s_w[kEncThreads];
  const uint32_t tid = threadIdx.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * kEncBlock + tid * kEncPer;
  uint32_t wc = 0;
  uint8_t tg[kEncPer];
#pragma unroll
  for (uint32_t k = 0; k < kEncPer; ++k) {
    tg[k] = i0 + k < in.n ? in.tag[i0 + k] : (uint8_t)0;
    wc += (i0 + k < in.n && enc_wide(tg[k])) ? 1u : 0u;
  }
  s_w[tid] = wc;
  __syncthreads();
  // wide records before this thread inside the block (inclusive scan, Hillis-Steele)
  for (uint32_t off = 1; off < kEncThreads; off <<= 1) {
    const uint32_t v = tid >= off ? s_w[tid - off] : 0u;
    __syncthreads();
    s_w[tid] += v;
    __syncthreads();
  }
  if (tid == kEncThreads - 1) wsum[blockIdx.x] = s_w[tid];
}

__global__ __launch_bounds__(1024) void k_enc_scan(uint32_t* __restrict__ wsum, uint32_t n_blocks,
                                                 uint64_t* __restrict__ wbase) {
  __shared__ uint64_t s[1024];
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < n_blocks; b0 += 1024) {
    const uint32_t b = b0 + threadIdx.x;
    const uint64_t v = b < n_blocks ? wsum[b] : 0ull;
    s[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
      const uint64_t y = threadIdx.x >= off ? s[threadIdx.x - off] : 0ull;
      __syncthreads();
      s[threadIdx.x] += y;
      __syncthreads();
    }
    if (b < n_blocks) wbase[b] = carry + s[threadIdx.x] - v;
    carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) wbase[n_blocks] = carry;
}

// Per block: record lengths (side rows from the wide prefix) and their block total;
// *bad = lowest invalid record (tag > 7, or a wide record whose side row names another
// record), ~0 if none.
__global__ __launch_bounds__(kEncThreads) void k_enc_bytes(EncodeIn in, const uint64_t* __restrict__ wbase,
                                                         uint64_t* __restrict__ bsum, uint32_t* __restrict__ bad) {
  __shared__ uint32_t s_w[kEncThreads];
  __shared__ uint64_t s_b[kEncThreads];
  const uint32_t tid = threadIdx.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * kEncBlock + tid * kEncPer;
  uint32_t wc = 0;
  uint8_t tg[kEncPer];
#pragma unroll
  for (uint32_t k = 0; k < kEncPer; ++k) {
    tg[k] = i0 + k < in.n ? in.tag[i0 + k] : (uint8_t)0;
    wc += (i0 + k < in.n && enc_wide(tg[k])) ? 1u : 0u;
  }
  s_w[tid] = wc;
  __syncthreads();
  for (uint32_t off = 1; off < kEncThreads; off <<= 1) {
    const uint32_t v = tid >= off ? s_w[tid - off] : 0u;
    __syncthreads();
    s_w[tid] += v;
    __syncthreads();
  }
  uint64_t w = wbase[blockIdx.x] + s_w[tid] - wc, bytes = 0;
#pragma unroll
  for (uint32_t k = 0; k < kEncPer; ++k) {
    if (i0 + k >= in.n) break;
    const bool wd = enc_wide(tg[k]);
    if (tg[k] > 7u || (wd && (w >= in.n_wide || in.w_idx[w] != i0 + k))) {
      atomicMin(bad, (uint32_t)min(i0 + k, (uint64_t)0xFFFFFFFEu));
      break;
    }
    bytes += enc_len(in, tg[k], w);
    w += wd ? 1u : 0u;
  }
  s_b[tid] = bytes;
  __syncthreads();
  for (uint32_t off = kEncThreads / 2; off > 0; off >>= 1) {
    if (tid < off) s_b[tid] += s_b[tid + off];
    __syncthreads();
  }
  if (tid == 0) bsum[blockIdx.x] = s_b[0];
}

__global__ __launch_bounds__(1024) void k_enc_scan64(uint64_t* __restrict__ v, uint32_t n_blocks,
                                                   uint64_t* __restrict__ base) {
  __shared__ uint64_t s[1024];
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < n_blocks; b0 += 1024) {
    const uint32_t b = b0 + threadIdx.x;
    const uint64_t x = b < n_blocks ? v[b] : 0ull;
    s[threadIdx.x] = x;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
      const uint64_t y = threadIdx.x >= off ? s[threadIdx.x - off] : 0ull;
      __syncthreads();
      s[threadIdx.x] += y;
      __syncthreads();
    }
    if (b < n_blocks) base[b] = carry + s[threadIdx.x] - x;
    carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) base[n_blocks] = carry;
}

// Big-endian field writers into a byte sink (LDS buffer or global output).
template <class P>
__device__ __forceinline__ void put_be(P p, uint64_t at, uint64_t v, uint32_t width) {
  for (uint32_t k = 0; k < width; ++k) p[at + k] = (uint8_t)(v >> (8u * (width - 1u - k)));
}
template <class P>
__device__ __forceinline__ void enc_record(P p, uint64_t at, const EncodeIn& in, uint32_t tg, int64_t v0, uint64_t w) {
  p[at] = (uint8_t)tg;
  switch (tg) {
    case CLG_TAG_ORDER: p[at + 1] = (uint8_t)v0; break;                       // :124-127
    case CLG_TAG_TIMESTAMP: put_be(p, at + 1, (uint64_t)v0, 8); break;        // :145-148
    case CLG_TAG_RNG:                                                         // :167-170
    case CLG_TAG_BUFFER_BUILT: put_be(p, at + 1, (uint64_t)v0, 4); break;     // :189-192
    case CLG_TAG_IGNORE_CHECKPOINT:                                           // :289-293
      put_be(p, at + 1, (uint32_t)in.w_rc[w], 4);
      put_be(p, at + 5, (uint64_t)v0, 8);
      break;
    case CLG_TAG_TIMER_TRIGGER: {                                             // :202-213
      put_be(p, at + 1, (uint32_t)in.w_rc[w], 4);
      put_be(p, at + 5, (uint64_t)v0, 8);
      const uint32_t sub = in.w_sub[w];
      p[at + 13] = (uint8_t)sub;
      if (sub == 6) {
        const uint32_t nl = in.w_var_len[w];
        put_be(p, at + 14, nl, 4);
        const uint8_t* src = in.var + in.w_var_off[w];
        for (uint32_t k = 0; k < nl; ++k) p[at + 18 + k] = src[k];
      }
      break;
    }
    case CLG_TAG_SOURCE_CHECKPOINT: {                                         // :244-257
      put_be(p, at + 1, (uint32_t)in.w_rc[w], 4);
      put_be(p, at + 5, (uint64_t)v0, 8);
      put_be(p, at + 13, (uint64_t)in.w_v1[w], 8);
      const uint32_t sub = in.w_sub[w];
      p[at + 21] = (uint8_t)(sub & 0x7Fu);
      p[at + 22] = (uint8_t)(sub >> 7);
      if (sub & 0x80u) {
        const uint32_t rl = in.w_var_len[w];
        put_be(p, at + 23, rl, 4);
        const uint8_t* src = in.var + in.w_var_off[w];
        for (uint32_t k = 0; k < rl; ++k) p[at + 27 + k] = src[k];
      }
      break;
    }
    default: {                                                                // SERIALIZABLE :316-323
      const uint32_t sl = in.w_var_len[w];
      const uint8_t* src = in.var + in.w_var_off[w];
      for (uint32_t k = 0; k < sl; ++k) p[at + 1 + k] = src[k];
      break;
    }
  }
}

__global__ __launch_bounds__(kEncThreads) void k_enc_write(EncodeIn in, const uint64_t* __restrict__ wbase,
                                                         const uint64_t* __restrict__ bbase, uint8_t* __restrict__ out) {
  __shared__ uint8_t s_out[kEncLds];
  __shared__ uint32_t s_w[kEncThreads];
  __shared__ uint64_t s_b[kEncThreads];
  const uint32_t tid = threadIdx.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * kEncBlock + tid * kEncPer;
  uint32_t wc = 0;
  uint8_t tg[kEncPer];
#pragma unroll
  for (uint32_t k = 0; k < kEncPer; ++k) {
    tg[k] = i0 + k < in.n ? in.tag[i0 + k] : (uint8_t)0;
    wc += (i0 + k < in.n && enc_wide(tg[k])) ? 1u : 0u;
  }
  s_w[tid] = wc;
  __syncthreads();
  for (uint32_t off = 1; off < kEncThreads; off <<= 1) {
    const uint32_t v = tid >= off ? s_w[tid - off] : 0u;
    __syncthreads();
    s_w[tid] += v;
    __syncthreads();
  }
  const uint64_t w0 = wbase[blockIdx.x] + s_w[tid] - wc;
  uint64_t w = w0, bytes = 0;
#pragma unroll
  for (uint32_t k = 0; k < kEncPer; ++k) {
    if (i0 + k < in.n) {
      bytes += enc_len(in, tg[k], w);
      w += enc_wide(tg[k]) ? 1u : 0u;
    }
  }
  s_b[tid] = bytes;
  __syncthreads();
  for (uint32_t off = 1; off < kEncThreads; off <<= 1) {
    const uint64_t v = tid >= off ? s_b[tid - off] : 0ull;
    __syncthreads();
    s_b[tid] += v;
    __syncthreads();
  }
  const uint64_t blk = s_b[kEncThreads - 1], base = bbase[blockIdx.x];
  const bool staged = blk <= kEncLds;
  uint64_t at = s_b[tid] - bytes;  // block-relative
  w = w0;
#pragma unroll
  for (uint32_t k = 0; k < kEncPer; ++k) {
    if (i0 + k < in.n) {
      if (staged)
        enc_record(s_out, at, in, tg[k], in.v0[i0 + k], w);
      else
        enc_record(out + base, at, in, tg[k], in.v0[i0 + k], w);
      at += enc_len(in, tg[k], w);
      w += enc_wide(tg[k]) ? 1u : 0u;
    }
  }
  if (!staged) return;
  __syncthreads();
  for (uint32_t b = tid; b < blk; b += kEncThreads) out[base + b] = s_out[b];
}

int launch_encode(const EncodeIn& in, uint32_t* d_wsum, uint64_t* d_wbase, uint64_t* d_bsum, uint64_t* d_bbase,
                  uint32_t* d_bad, uint8_t* d_out, uint32_t phase, void* stream) {
  const uint32_t nb = (uint32_t)((in.n + kEncBlock - 1) / kEncBlock);
  hipStream_t st = (hipStream_t)stream;
  if (!nb) return CLG_OK;
  if (phase == 0) {  // sizes: wide prefix, byte prefix, validity
    hipLaunchKernelGGL(k_enc_sums, dim3(nb), dim3(kEncThreads), 0, st, in, d_wsum);
    hipLaunchKernelGGL(k_enc_scan, dim3(1), dim3(1024), 0, st, d_wsum, nb, d_wbase);
    hipLaunchKernelGGL(k_enc_bytes, dim3(nb), dim3(kEncThreads), 0, st, in, d_wbase, d_bsum, d_bad);
    hipLaunchKernelGGL(k_enc_scan64, dim3(1), dim3(1024), 0, st, d_bsum, nb, d_bbase);
  } else {
    hipLaunchKernelGGL(k_enc_write, dim3(nb), dim3(kEncThreads), 0, st, in, d_wbase, d_bbase, d_out);
  }
  return launch_status(hipGetLastError());
}

}  // namespace clg
